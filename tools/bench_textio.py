"""Throughput of the normalised-matrix text writer / reader (host C++,
threaded) vs Python's gzip on the same text.

    python tools/bench_textio.py [--n 3202] [--r 270000] [--threads 16]
"""
import argparse
import gzip
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grid_amd import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=3202)
ap.add_argument("--r", type=int, default=270_000)
ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
ap.add_argument("--level", type=int, default=6)
ap.add_argument("--python-rows", type=int, default=64, help="rows for the Python gzip baseline")
a = ap.parse_args()

rng = np.random.default_rng(0)
zq = np.clip(np.rint(rng.normal(0, 120, (a.n, a.r))), -3000, 3000).astype(np.int32)
raw = rng.uniform(20, 40, a.n)
means = rng.uniform(0.8, 1.2, a.r)
ratios = rng.uniform(0.5, 20, a.r)
ids = [f"S{i:06d}" for i in range(a.n)]
d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
path = os.path.join(d, "norm.tsv.gz")
t0 = time.perf_counter()
_abi.write_normalized_gz(path, ids, raw, means, ratios, zq, level=a.level, threads=a.threads)
tw = time.perf_counter() - t0
gz_bytes = os.path.getsize(path)
t1 = time.perf_counter()
rid, rsc, rmu, rrat, rzq = _abi.read_normalized_gz(path, threads=a.threads)
tr = time.perf_counter() - t1
assert np.array_equal(rzq, zq)
with gzip.open(path, "rb") as f:
    text_bytes = sum(len(b) for b in iter(lambda: f.read(1 << 24), b""))
# Python baseline on a row sample: the reference's per-cell f-string + gzip.open("wt")
k = min(a.python_rows, a.n)
z = zq[:k] / 100.0
t2 = time.perf_counter()
with gzip.open(os.path.join(d, "py.tsv.gz"), "wt") as f:
    for i in range(k):
        f.write(f"{ids[i]}\t{raw[i]:.2f}\t" + "\t".join(f"{v:.2f}" for v in z[i]) + "\n")
tp = (time.perf_counter() - t2) * a.n / k
os.remove(path)
print(json.dumps({"n": a.n, "r": a.r, "threads": a.threads, "level": a.level, "text_GB": text_bytes / 1e9,
                  "gz_GB": gz_bytes / 1e9, "write_s": tw, "write_text_GBps": text_bytes / tw / 1e9,
                  "read_s": tr, "read_text_GBps": text_bytes / tr / 1e9,
                  "python_writer_s_scaled": tp, "python_rows_sampled": k}))
