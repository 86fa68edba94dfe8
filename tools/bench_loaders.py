"""Cohort-scale IBS / IBD loader timing: host C++ parser vs
the Python restatement on synthetic computeIBSpbwt / iLASH files.

    python tools/bench_loaders.py [--samples 50000] [--nbr 20] [--out f.json]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from grid_amd import _abi  # noqa: E402
from grid_amd.utils import hi_inference as hi  # noqa: E402


def make_files(d, n, k, seed=0):
    rng = np.random.default_rng(seed)
    ids = [f"NWD{i:07d}" for i in range(n)]
    ibs = os.path.join(d, "ibs.tsv")
    with open(ibs, "w") as f:
        f.write("ID\thap\tnbrInd\tcMlen\tcMedge\tIDnbr\thapNbr\n")
        for i in range(n):
            js = rng.integers(0, n, 2 * k)
            for h in (1, 2):
                f.write("".join(f"{ids[i]}\t{h}\t{t}\t{rng.random() * 5:.3f}\t{rng.random():.3f}\t"
                                f"{ids[js[(h - 1) * k + t]]}\t{1 + (t & 1)}\n" for t in range(k)))
    ibd = os.path.join(d, "ibd.txt")
    with open(ibd, "w") as f:
        for i in range(n):
            js = rng.integers(0, n, k)
            bp = rng.integers(1_000_000, 2_000_000, k)
            f.write("".join(f"{ids[i]}\t{ids[i]}_{t & 1}\t{ids[j]}\t{ids[j]}_{(t >> 1) & 1}\tchr1\t{b}\t{b + 250000}"
                            f"\trs1\trs2\t{rng.uniform(0.5, 8):.2f}\t{rng.uniform(0.7, 1):.3f}\n"
                            for t, (j, b) in enumerate(zip(js, bp))))
    return ids, ibs, ibd


def timed(fn, reps=1):
    best = float("inf")
    for _ in range(reps):
        t = time.perf_counter()
        r = fn()
        best = min(best, time.perf_counter() - t)
    return best, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=50000)
    ap.add_argument("--nbr", type=int, default=20)
    ap.add_argument("--out")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        ids, ibs, ibd = make_files(d, a.samples, a.nbr)
        idx = {k: i for i, k in enumerate(ids)}
        res = {"samples": a.samples, "nbr_per_hap": a.nbr}
        for name, path, nat, py in (
                ("ibs", ibs, lambda: _abi.load_ibs(ibs, ids, 10),
                 lambda: hi._load_ibs_neighbors_py(ibs, idx, 10)),
                ("ibd_weighted", ibd, lambda: _abi.load_ibd(ibd, ids, 10, 1_300_000, 1_500_000, 0.5, 0.7, True, 1e6),
                 lambda: hi._load_ibd_neighbors_py(ibd, idx, 10, 1_300_000, 1_500_000, 0.5, 0.7, True, 1e6))):
            tn, (off, nbr, w) = timed(nat, 3)
            tp, lists = timed(py)
            po, pn, pw = hi.engine.csr_from_lists(lists)
            same = np.array_equal(off, po) and np.array_equal(nbr, pn) and np.array_equal(w, pw)
            mb = os.path.getsize(path) / 1e6
            res[name] = {"file_MB": round(mb, 1), "native_s": round(tn, 3), "python_s": round(tp, 3),
                         "speedup": round(tp / tn, 1), "native_MBps": round(mb / tn, 1), "identical": bool(same)}
            print(name, res[name], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
