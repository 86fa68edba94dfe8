"""Host read rate of a mosdepth cohort into staging buffers (the device
ingest's read_batch): files of DIR read by T threads into one pinned or
pageable buffer, per method.  Prints one JSON line per (method, threads).

    python tools/bench_read.py DIR [--gb 8]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grid_amd import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--gb", type=float, default=8.0)
a = ap.parse_args()
names = sorted(f for f in os.listdir(a.dir) if f.endswith(".regions.bed.gz"))
paths = [os.path.join(a.dir, f) for f in names]
sizes = [os.path.getsize(p) for p in paths]
take, tot = [], 0
for p, s in zip(paths, sizes):
    if tot + s > a.gb * 1e9:
        break
    take.append((p, s))
    tot += s
off = np.zeros(len(take) + 1, np.int64)
off[1:] = np.cumsum([-(-s // 256) * 256 for _, s in take])
t = time.perf_counter()
pin = _abi.PinnedBuf(int(off[-1]) + 256)
t_pin = time.perf_counter() - t
page = np.empty(int(off[-1]) + 256, np.uint8)
page[::4096] = 0


def run(buf, threads, how):
    def one(k):
        p, s = take[k]
        if how == "readinto":
            with open(p, "rb", buffering=0) as fh:
                fh.readinto(memoryview(buf)[off[k]:off[k] + s])
        else:                                      # os.preadv in 8 MiB pieces
            fd = os.open(p, os.O_RDONLY)
            try:
                pos = 0
                while pos < s:
                    n = os.preadv(fd, [memoryview(buf)[off[k] + pos:off[k] + min(s, pos + (8 << 20))]], pos)
                    if n <= 0:
                        break
                    pos += n
            finally:
                os.close(fd)
    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(one, range(len(take))))
        return time.perf_counter() - t0


print(json.dumps({"files": len(take), "bytes": tot, "pin_alloc_s": t_pin}), flush=True)
for threads in (8, 16, 32):
    for how in ("readinto", "preadv"):
        for name, buf in (("pinned", pin.array), ("pageable", page)):
            dt = run(buf, threads, how)
            print(json.dumps({"method": how, "buffer": name, "threads": threads, "s": dt, "GBps": tot / dt / 1e9}),
                  flush=True)

# host -> HBM copy rate from each buffer (grid_h2d: hipMemcpyAsync + sync)
dev = _abi.Device(0)
d = dev.alloc(int(off[-1]) + 256, np.uint8)
for name, buf in (("pinned", pin.array), ("pageable", page)):
    for rep in range(2):
        t = time.perf_counter()
        _abi.call("grid_h2d", dev.ctx, d.ptr, buf.ctypes.data, int(off[-1]))
        dt = time.perf_counter() - t
        print(json.dumps({"h2d": name, "rep": rep, "s": dt, "GBps": off[-1] / dt / 1e9}), flush=True)
