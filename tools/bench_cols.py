"""Column-statistics passes in isolation at the bench shape (VERDICT r4 item
5): k_col_means / k_col_vars on the bench's compact depth matrix (3,202 x
3,000,000), each timed alone with HIP events, back to back (no Gram or zquant
around them), against the same passes inside the chain (bench.py stages).

    python tools/bench_cols.py [--reps 10] [--n 3202] [--m 3000000]
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from grid_amd import _abi  # noqa: E402
from grid_amd._abi import call, ptr  # noqa: E402
from grid_amd.fused import Depth16, HipOps, Steps47, TorchAlloc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=3202)
ap.add_argument("--m", type=int, default=3_000_000)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()

dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
ta = TorchAlloc(0)
d16 = Depth16.synth(ta, dev.ctx, bench.SEED, a.n, a.m, 0, bench.NCL)
reads, off, nbr, w = bench.synth_reads_and_ibs(a.n)
st = Steps47(HipOps(dev), ta, a.n, a.m, 0, a.m, k=10, n_nbr=300, n_iters=1)
st.set_reads(reads)
st.set_phasing_graph(off, nbr, w)
st.run(d16, d16.ld)                       # row means, mu, var of the real chain
torch.cuda.synchronize()
mu = torch.empty(a.m, dtype=torch.float64, device="cuda")
var = torch.empty(a.m, dtype=torch.float64, device="cuda")
ratio = torch.empty(a.m, dtype=torch.float64, device="cuda")


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


res = {"means": [], "vars": []}
for _ in range(a.reps):
    res["means"].append(timed(lambda: call("grid_norm_col_means_q16", dev.ctx, C.byref(d16.desc), a.n, a.m, d16.ld,
                                            ptr(st.rm), ptr(mu))))
    res["vars"].append(timed(lambda: call("grid_norm_col_vars_q16", dev.ctx, C.byref(d16.desc), a.n, a.m, d16.ld,
                                           ptr(st.rm), ptr(mu), ptr(var), ptr(ratio))))
assert torch.equal(mu, st.mu[: a.m]) and torch.equal(var, st.var[: a.m])
out = {k: {"min_ms": min(v), "median_ms": sorted(v)[len(v) // 2], "all": [round(x, 3) for x in v]} for k, v in res.items()}
out["shape"] = [a.n, a.m]
out["bytes_per_pass"] = a.n * d16.ld * 2
print(json.dumps(out))
