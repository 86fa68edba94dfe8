"""Device writer of the step-4 file (grid_write_normalized_gz_dev) on a
config-2-like matrix: wall time, output size, and the host writer's
(libdeflate) size on the same text; the file is read back and compared.

    python tools/bench_gzwrite_dev.py [--n 200] [--r 2700000] [--host-level 1]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grid_amd import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=200)
ap.add_argument("--r", type=int, default=2_700_000)
ap.add_argument("--host-level", type=int, default=1)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--threads", type=int, default=16)
a = ap.parse_args()

rng = np.random.default_rng(0)
zq = np.rint(rng.normal(0, 100, (a.n, a.r))).astype(np.int32)   # z in hundredths, as step 4 leaves it
raw = rng.uniform(20, 40, a.n)
means = rng.uniform(0.8, 1.2, a.r)
ratios = rng.uniform(0.5, 20, a.r)
ids = [f"S{i:06d}" for i in range(a.n)]
dev = _abi.Device(0)
dz = dev.upload(zq)
d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
dpath, hpath = os.path.join(d, "dev.tsv.gz"), os.path.join(d, "host.tsv.gz")
times = []
for _ in range(a.reps):
    t0 = time.perf_counter()
    _abi.write_normalized_gz_dev(dev, dpath, ids, raw, means, ratios, dz, a.n, a.r, a.r, level=1, threads=a.threads)
    times.append(time.perf_counter() - t0)
dev_bytes = os.path.getsize(dpath)
t0 = time.perf_counter()
_abi.write_normalized_gz(hpath, ids, raw, means, ratios, zq, level=a.host_level, threads=a.threads)
th = time.perf_counter() - t0
host_bytes = os.path.getsize(hpath)
rid, rsc, rmu, rrat, rzq = _abi.read_normalized_gz(dpath, threads=a.threads)
same = rid == ids and np.array_equal(rzq, zq)
text_bytes = sum(len(x) for x in ids) + a.n * 8 + int(np.sum([len(f"{v / 100:.2f}") for v in zq[0]])) * a.n + a.n * a.r
os.remove(dpath)
os.remove(hpath)
print(json.dumps({"n": a.n, "r": a.r, "dev_write_s": times, "dev_bytes": dev_bytes, "host_level": a.host_level,
                  "host_bytes": host_bytes, "host_write_s": th, "dev_over_host": dev_bytes / host_bytes,
                  "text_bytes_est": text_bytes, "dev_ratio_est": dev_bytes / text_bytes,
                  "dev_text_GBps_est": text_bytes / min(times) / 1e9, "read_back_equal": bool(same)}))
