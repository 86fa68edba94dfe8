#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
implementation (caterer-z-t/GRiD, read-only at /root/reference).

Run in the build container only (the GPU box has no /root/reference):

    python tests/golden/make_golden.py

What it writes (all small):
  g1/  file-level cohort, genome-scale mode (no window), chrom filter chr1 with
       chr10/chr2 decoy lines, a repeat mask, read counts, IBS + IBD neighbour
       files; expected outputs of reference steps 4,5,6,7 (IBS) and 7 (IBD,
       weighted) run through the reference's own step functions.
  g1b/ file-level cohort crossing the 8192-element NumPy reduction block
       (M > 8192 bins), LPA-style window off.
  g1c/ LPA-style window (chrom/start_bp/end_bp set), kd-tree k-NN path.
  g2.npz   normalize_matrix on widths 8191/8192/8193/16385/... with NaN holes,
           a zero row, an all-NaN column and a zero column.
  g3.json  find_neighbors_sklearn on tie-free hundredth matrices (brute and
           kd-tree paths).
  g4.json  _run_phasing/_compute_imp on IBS-style and IBD-weighted lists.
  g5.json  %.2f / %.3f formatting edge cases.
  meta.json  library versions of the oracle run.

pysam is stubbed exactly as the reference's own test/conftest.py:9-11 does.
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import sys
import tempfile
from pathlib import Path
from unittest.mock import MagicMock

import numpy as np
import yaml

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent

sys.modules.setdefault("pysam", MagicMock())
sys.path.insert(0, str(REF))

from rich.console import Console  # noqa: E402

import grid.cli  # noqa: E402
from grid.utils import normalize_mosdepth as ref_norm  # noqa: E402
from grid.utils import find_neighbors as ref_fn  # noqa: E402
from grid.utils import compute_dipcn as ref_dip  # noqa: E402
from grid.utils import hi_inference as ref_hi  # noqa: E402

CONSOLE = Console(theme=grid.cli.grid_theme, quiet=True)


from cohort_files import inputs_digest, make_file_cohort  # noqa: E402


def run_reference(cfg, root: Path):
    """Run the reference's step functions (not the CLI: it would also try the
    OOS steps)."""
    out = Path(cfg["output_dir"])
    out.mkdir(parents=True, exist_ok=True)
    (out / "counts.tsv").write_text((root / "counts.tsv").read_text())
    ref_norm.normalize_mosdepth(cfg, CONSOLE)
    ref_fn.find_neighbors(cfg, CONSOLE)
    ref_dip.compute_diploid_genotypes(cfg, CONSOLE)
    ref_hi.hi_inference(cfg, CONSOLE)
    # IBD, weighted, as a second step-7 run
    cfg2 = json.loads(json.dumps(cfg))
    hc = cfg2["compute_haploid_genotypes"]
    hc.update({"method": "ibd", "ibd_output": str(root / "ibd.txt"), "weighted": True,
               "weight_scale": 1_000_000, "min_length": 0.5, "min_match": 0.7,
               "output_file_prefix": "haploid_ibd", "min_neighbors": 2, "max_neighbors": 6,
               "n_iters": 37})
    cfg2.setdefault("start_bp", 1_500_000)
    cfg2.setdefault("end_bp", 1_600_000)
    ref_hi.hi_inference(cfg2, CONSOLE)
    return cfg2


def check_tie_free(norm_gz: Path, k: int, zmax: float, sigma2_max: float):
    """Exact-integer check that no row of the reference's k-NN input has a
    distance tie inside its first k+2 neighbours (sklearn's tie order is
    unspecified)."""
    ids, ratios, z, _ = ref_fn.read_normalized_data(norm_gz)
    z = np.nan_to_num(np.clip(z, -zmax, zmax), nan=0.0)
    idx, _ = ref_fn.filter_regions_by_variance(ratios, 1.0, sigma2_max)
    q = np.rint(z[:, idx] * 100).astype(np.int64)
    g = q @ q.T
    n = np.diag(g)
    d2 = n[:, None] + n[None, :] - 2 * g
    for i in range(len(ids)):
        row = np.sort(d2[i])[: k + 3]
        if len(set(row.tolist())) != len(row):
            return False
    return True


def finalize_cohort(name, root: Path, cfg, cfg_ibd):
    dst = HERE / name
    if dst.exists():
        shutil.rmtree(dst)
    (dst / "expected").mkdir(parents=True)
    (dst / "inputs").mkdir()
    shutil.copytree(root / "mosdepth", dst / "inputs" / "mosdepth")
    for f in ("samples.txt", "mask.bed", "counts.tsv", "ibs.tsv.gz", "ibd.txt"):
        shutil.copy(root / f, dst / "inputs" / f)
    out = Path(cfg["output_dir"])
    # store expected outputs decompressed-content-identical (re-gzip small)
    for f in out.iterdir():
        shutil.copy(f, dst / "expected" / f.name)

    def rel(c):
        c = json.loads(json.dumps(c))
        c["samples_file"] = "inputs/samples.txt"
        c["output_dir"] = "out"
        c["mosdepth"]["work_dir"] = "inputs/mosdepth"
        c["mosdepth"]["normalize"]["repeat_mask_file"] = "inputs/mask.bed"
        hc = c["compute_haploid_genotypes"]
        if "ibs_output" in hc:
            hc["ibs_output"] = "inputs/ibs.tsv.gz"
        if "ibd_output" in hc:
            hc["ibd_output"] = "inputs/ibd.txt"
        return c

    (dst / "config.yaml").write_text(yaml.safe_dump(rel(cfg), sort_keys=False))
    (dst / "config_ibd.yaml").write_text(yaml.safe_dump(rel(cfg_ibd), sort_keys=False))


def file_cohort(name, seed, n, m, chrom, window=None, decoys=True, start0=0, bin_size=1000,
                k=None, n_clusters=4):
    for attempt in range(20):
        rng = np.random.default_rng(seed + 1000 * attempt)
        tmp = Path(tempfile.mkdtemp(prefix=f"golden_{name}_"))
        cfg = make_file_cohort(tmp, rng, n, m, chrom, window, decoys, bin_size, start0, n_clusters)
        if k is not None:
            cfg["mosdepth"]["neighbors"]["num_neighbors"] = k
        cfg_ibd = run_reference(cfg, tmp)
        norm = Path(cfg["output_dir"]) / "normalized.tsv.gz"
        if check_tie_free(norm, cfg["mosdepth"]["neighbors"]["num_neighbors"], 2.0, 1000):
            finalize_cohort(name, tmp, cfg, cfg_ibd)
            shutil.rmtree(tmp)
            print(f"{name}: ok (seed attempt {attempt})")
            return
        shutil.rmtree(tmp)
    raise RuntimeError(f"{name}: could not make a tie-free cohort")


def config1_cohort():
    """BASELINE config 1: 100 samples x 30k bins (1 kb), k = 10, the reference's
    CPU path.  The inputs (100 mosdepth files, ~3M lines) are regenerated by
    the test from the recorded seed (tests/golden/cohort_files.py) and checked
    against the recorded input digest; the small outputs are stored whole, the
    normalised matrix as the sha256 + length of its decompressed text."""
    import hashlib
    name = "g_cfg1"
    for attempt in range(20):
        seed = 101 + 1000 * attempt
        rng = np.random.default_rng(seed)
        tmp = Path(tempfile.mkdtemp(prefix=f"golden_{name}_"))
        cfg = make_file_cohort(tmp, rng, 100, 30_000, "chr1", decoys=True)
        cfg["mosdepth"]["neighbors"]["num_neighbors"] = 10
        cfg["compute_diploid_genotypes"]["n_nbr"] = 10
        cfg_ibd = run_reference(cfg, tmp)
        out = Path(cfg["output_dir"])
        if not check_tie_free(out / "normalized.tsv.gz", 10, 2.0, 1000):
            shutil.rmtree(tmp)
            continue
        dst = HERE / name
        if dst.exists():
            shutil.rmtree(dst)
        (dst / "expected").mkdir(parents=True)
        for f in out.iterdir():
            if f.name != "normalized.tsv.gz":
                shutil.copy(f, dst / "expected" / f.name)
        text = gzip.decompress((out / "normalized.tsv.gz").read_bytes())
        meta = {"seed": seed, "n": 100, "m": 30_000, "chrom": "chr1", "decoys": True, "k": 10,
                "inputs_sha256": inputs_digest(tmp),
                "normalized_sha256": hashlib.sha256(text).hexdigest(), "normalized_bytes": len(text),
                "normalized_head": text[:2000].decode()}
        (dst / "cohort.json").write_text(json.dumps(meta, indent=1))
        # configs with paths relative to the regenerated cohort root
        for fname, c in (("config.yaml", cfg), ("config_ibd.yaml", cfg_ibd)):
            c = json.loads(json.dumps(c).replace(str(tmp) + "/", ""))
            (dst / fname).write_text(yaml.safe_dump(c, sort_keys=False))
        shutil.rmtree(tmp)
        print(f"{name}: ok (seed {seed})")
        return
    raise RuntimeError(f"{name}: could not make a tie-free cohort")


# ---------------------------------------------------------------- vectors --
def g2():
    rng = np.random.default_rng(2)
    out = {}
    cases = [(4, 5), (3, 130), (2, 8191), (2, 8192), (2, 8193), (2, 16385), (6, 300)]
    for ci, (n, m) in enumerate(cases):
        q = rng.integers(1, 9000, size=(n, m)).astype(np.float64)
        mat = q / 100.0
        mat[rng.random((n, m)) < 0.05] = np.nan
        if ci == 6:
            mat[:, 3] = np.nan          # all-NaN column
            mat[:, 4] = 0.0             # zero column (mu = 0 -> not transformed)
            mat[2, :] = 0.0             # zero row (row mean 0 -> NaN row)
        with np.errstate(all="ignore"):
            raw = np.nanmean(mat, axis=1)
            z, ratios, mu, var = ref_norm.normalize_matrix(mat)
        keys = sorted(ratios)
        out[f"c{ci}_in"] = mat
        out[f"c{ci}_raw"] = raw
        out[f"c{ci}_z"] = z
        out[f"c{ci}_mu"] = mu
        out[f"c{ci}_var"] = var
        out[f"c{ci}_rkeys"] = np.array(keys, dtype=np.int64)
        out[f"c{ci}_rvals"] = np.array([ratios[k] for k in keys])
        for tf in (0.0, 0.1, 0.5, 0.9):
            out[f"c{ci}_sel_{tf}"] = np.array(ref_norm.select_high_variance_regions(ratios, tf), dtype=np.int64)
    np.savez_compressed(HERE / "g2.npz", **out)
    print("g2: ok")


def g3():
    rng = np.random.default_rng(3)
    cases = []
    for (n, r, k) in [(50, 40, 10), (50, 8, 6), (12, 20, 30), (3, 1, 5), (40, 16, 39)]:
        for attempt in range(200):
            q = rng.integers(-200, 201, size=(n, r))
            g = q @ q.T
            nn = np.diag(g)
            d2 = nn[:, None] + nn[None, :] - 2 * g
            ok = all(len(set(np.sort(d2[i]).tolist())) == n for i in range(n))
            if ok or n > 40:
                break
        data = q / 100.0
        ids = [f"X{i:03d}" for i in range(n)]
        res = ref_fn.find_neighbors_sklearn(data, ids, n_neighbors=k)
        cases.append({"q": q.tolist(), "k": k,
                      "res": {sid: [[nb, float(d).hex()] for nb, d in lst] for sid, lst in res.items()}})
    (HERE / "g3.json").write_text(json.dumps(cases))
    print("g3: ok")


def g4():
    rng = np.random.default_rng(4)
    cases = []
    for (n, min_nbr, iters, weighted) in [(30, 1, 100, False), (25, 0, 7, False), (40, 3, 50, False),
                                          (30, 2, 20, True), (1, 1, 5, False)]:
        irr = [float(x) for x in rng.uniform(0.2, 4.0, size=n)]
        if n > 3:
            irr[2] = 0.0
        hap_nbrs = []
        for h in range(2 * n):
            k = int(rng.integers(0, 8))
            lst = []
            for _ in range(k):
                nb = int(rng.integers(0, 2 * n))
                w = float(rng.uniform(0.05, 1.0)) if weighted else 1.0
                lst.append((nb, w))
            if h % 11 == 0:
                lst.append((h, 1.0))                    # self neighbour
            if h % 13 == 0 and lst:
                lst.append(lst[0])                      # duplicate
            hap_nbrs.append(lst)
        hap, mean = ref_hi._run_phasing(irr, hap_nbrs, min_nbr, iters, CONSOLE)
        imp = [ref_hi._compute_imp(i, hap, hap_nbrs, mean) for i in range(n)]
        cases.append({"irr": [x.hex() for x in irr], "nbrs": [[[a, b.hex()] for a, b in l] for l in hap_nbrs],
                      "min_nbr": min_nbr, "iters": iters,
                      "hap": [x.hex() for x in hap], "mean": mean.hex(),
                      "imp": [[a.hex(), b.hex()] for a, b in imp]})
    (HERE / "g4.json").write_text(json.dumps(cases))
    print("g4: ok")


def g5():
    vals = [0.125, 0.135, 2.675, -0.001, -0.0, 0.0, -0.005, 0.005, 1e-9, -1e-9, 123456.785,
            0.045, 1.005, 2.5e-3, -2.5e-3, 99.995, -99.995, float("inf")]
    rng = np.random.default_rng(5)
    vals += [float(x) for x in rng.uniform(-5, 5, 200)]
    vals += [float(k) / 200.0 for k in range(-400, 401)]     # exact-ish halves of hundredths
    vals += [float(k) / 2000.0 for k in range(-60, 61)]      # halves of thousandths
    (HERE / "g5.json").write_text(json.dumps([[v.hex(), f"{v:.2f}", f"{v:.3f}"] for v in vals]))
    print("g5: ok")


def main():
    import sklearn
    import pandas
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    if sys.argv[1:] == ["cfg1"]:
        config1_cohort()
        return
    file_cohort("g1", 11, 40, 2400, "chr1", decoys=True)
    file_cohort("g1b", 21, 10, 8600, "chr1", decoys=False)
    file_cohort("g1c", 31, 30, 60, "chr6", window=(160_605_062, 160_647_661), decoys=False,
                start0=160_590_000, k=7)
    g2()
    g3()
    g4()
    g5()
    meta = {"numpy": np.__version__, "sklearn": sklearn.__version__, "pandas": pandas.__version__,
            "python": sys.version.split()[0], "reference": str(REF)}
    (HERE / "meta.json").write_text(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
