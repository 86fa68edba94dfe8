"""Host ingest throughput (R1-R4): native C++ parser vs the line-by-line
Python restatement, on a synthetic mosdepth cohort written to --dir.

    python tools/bench_ingest.py [--samples 32] [--bins 300000] [--threads 8]
"""
import argparse
import gzip
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grid_amd.utils import normalize_mosdepth as nm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--samples", type=int, default=32)
ap.add_argument("--bins", type=int, default=300_000)
ap.add_argument("--threads", type=int, default=8)
ap.add_argument("--dir", default="/tmp/grid_ingest_bench")
ap.add_argument("--py-samples", type=int, default=4, help="samples timed on the Python parser")
a = ap.parse_args()

os.makedirs(a.dir, exist_ok=True)
rng = np.random.default_rng(0)
base = rng.gamma(20.0, 1.5, a.bins)
starts = np.arange(a.bins, dtype=np.int64) * 1000
names = [f"S{i:06d}" for i in range(a.samples)]
t0 = time.perf_counter()
for nmx in names:
    p = os.path.join(a.dir, f"{nmx}.regions.bed.gz")
    if os.path.exists(p):
        continue
    d = np.round(base * rng.uniform(0.6, 1.4) * rng.normal(1, 0.05, a.bins), 2)
    txt = "".join(f"chr1\t{s}\t{s + 1000}\t{v:.2f}\n" for s, v in zip(starts.tolist(), d.tolist()))
    with gzip.open(p, "wt", compresslevel=1) as f:
        f.write(txt)
gen = time.perf_counter() - t0
raw = a.samples * a.bins
inds = nm.map_mosdepth_files_to_samples(a.dir, names)
t0 = time.perf_counter()
ids, regions, q = nm.ingest_native(inds, a.dir, "chr1", None, None, {}, 20, 100, a.threads)
tn = time.perf_counter() - t0
sub = {k: inds[k] for k in list(inds)[: a.py_samples]}
t0 = time.perf_counter()
nm.ingest_py(sub, a.dir, "chr1", None, None, {}, 20, 100, a.threads)
tp = (time.perf_counter() - t0) * a.samples / len(sub)
print(f"cohort {a.samples} x {a.bins} (generated in {gen:.1f}s): matrix {q.shape}")
print(f"native C++ ingest ({a.threads} threads): {tn:.2f} s = {raw / tn / 1e6:.1f} M lines/s, "
      f"{a.samples / tn:.1f} samples/s")
print(f"python line-by-line (one parse, {a.threads} threads, scaled from {len(sub)} samples): {tp:.1f} s "
      f"-> native {tp / tn:.1f}x")
