"""Step-4 ingest from files: the host C++ parser (ingest_native, --threads)
against the device ingest (ingest_device: GPU + CPU inflate split by the cost
model, parse in HBM), and the device ingest forced all-GPU / all-CPU, on a
synthetic cohort (tools/gen_cohort: the bench cohort as mosdepth
regions.bed.gz, BGZF unless --plain).  Every variant's ids, regions and
matrix must equal the host parser's.

    python tools/bench_dev_ingest.py [--samples 256] [--bins 3000000] [--plain] [--json out.json]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from grid_amd import _abi  # noqa: E402
from grid_amd.utils import ingest_device  # noqa: E402
from grid_amd.utils import normalize_mosdepth as nm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--samples", type=int, default=256)
ap.add_argument("--bins", type=int, default=3_000_000)
ap.add_argument("--plain", action="store_true", help="one gzip member per file instead of BGZF")
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--dir", default="/dev/shm/grid_dev_ingest")
ap.add_argument("--modes", default="host,model,gpu,cpu")
ap.add_argument("--json", default="")
a = ap.parse_args()

mos = os.path.join(a.dir, "plain" if a.plain else "bgzf")
os.makedirs(mos, exist_ok=True)
gen = os.path.join(ROOT, "tools", "gen_cohort")
if not os.path.exists(gen):
    subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", "-o", gen, gen + ".cpp", "-lz"], check=True)
t0 = time.perf_counter()
if len([f for f in os.listdir(mos) if f.endswith(".regions.bed.gz")]) != a.samples:
    for i0 in range(0, a.samples, 64):
        n = min(64, a.samples - i0)
        subprocess.run([gen, mos, str(n), str(a.bins), "20260821", str(a.threads), str(i0)]
                       + ([] if a.plain else ["bgzf"]), check=True)
        print(f"generated {i0 + n} files", flush=True)
gen_s = time.perf_counter() - t0
ids = [f"S{i:05d}" for i in range(a.samples)]
inds = nm.map_mosdepth_files_to_samples(mos, ids)
inds = {k: inds[k] for k in ids}
dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())


def digest(r):
    q = r[2].numpy() if isinstance(r[2], _abi.DevBuf) else r[2]
    h = hashlib.sha256(q.tobytes())
    h.update(repr((r[0], r[1][:5], r[1][-5:], len(r[1]))).encode())
    return h.hexdigest()[:16], q.shape


res = {"samples": a.samples, "bins": a.bins, "bgzf": not a.plain, "threads": a.threads, "generate_s": gen_s,
       "cohort_gb": sum(os.path.getsize(os.path.join(mos, f)) for f in os.listdir(mos)) / 1e9, "modes": {}}
ref = None
for mode in a.modes.split(","):
    orig = ingest_device._Split.plan
    if mode == "gpu":
        ingest_device._Split.plan = lambda self, f, t, b: (sorted(f), [])
    elif mode == "cpu":
        ingest_device._Split.plan = lambda self, f, t, b: ([], sorted(f))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if mode == "host":
        r = nm.ingest_native(inds, mos, "chr1", None, None, {}, 20, 100, a.threads)
    else:
        r = nm._ingest_dev(dev, inds, mos, "chr1", None, None, {}, 20, 100, a.threads)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t1
    ingest_device._Split.plan = orig
    dg = digest(r)
    ref = ref or dg
    res["modes"][mode] = {"seconds": dt, "digest": dg[0], "shape": list(dg[1]), "same_as_first": dg == ref}
    print(json.dumps({mode: res["modes"][mode]}), flush=True)
    del r
assert all(v["same_as_first"] for v in res["modes"].values())
print(json.dumps(res), flush=True)
if a.json:
    open(a.json, "w").write(json.dumps(res) + "\n")
