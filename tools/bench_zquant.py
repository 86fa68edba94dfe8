"""Microbenchmark of the step-4 quantisation kernel at the bench shape:
full output vs without the int32 z matrix (zq) vs without the bf16 panel (zb),
to split its time between the q reads and the two writes.

    python tools/bench_zquant.py [--reps 3]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "--env" in sys.argv:   # the probes live in the tools build (make -C grid_amd/csrc probes)
    os.environ.setdefault("GRID_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                        "grid_amd", "_lib", "libgridhip_probes.so"))
import bench  # noqa: E402
from grid_amd import _abi  # noqa: E402
from grid_amd._abi import call, ptr  # noqa: E402
from grid_amd.fused import Depth16, HipOps, Steps47, TorchAlloc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=3202)
ap.add_argument("--m", type=int, default=3_000_000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--q16", action="store_true", help="compact depth matrix (grid_depth16) as the source")
ap.add_argument("--groups", default="1", help="comma list of GRID_ZQUANT_GROUPS values to time")
ap.add_argument("--ldz-align", type=int, default=8, help="step-4 output row stride rounded up to this many columns")
ap.add_argument("--env", default="", help="semicolon list of K=V[,K=V] settings to time full16 under "
                "(the tools build's probes, e.g. GRID_Z7_PROBE=3)")
a = ap.parse_args()


dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
q = torch.empty((a.n, a.m), dtype=torch.int32, device="cuda")
call("grid_synth_depth", dev.ctx, bench.SEED, a.n, a.m, a.m, 0, bench.NCL, q.data_ptr())
reads, off, nbr, w = bench.synth_reads_and_ibs(a.n)
st = Steps47(HipOps(dev), TorchAlloc(0), a.n, a.m, 0, a.m, k=10, n_nbr=300, n_iters=1)
st.set_reads(reads)
st.set_phasing_graph(off, nbr, w)
st.run(q, a.m)
torch.cuda.synchronize()
of = C.c_int32()
zq32 = torch.empty((a.n, st.r_loc), dtype=torch.int32, device="cuda")
LDZ = -(-st.r_loc // a.ldz_align) * a.ldz_align          # the chain's step-4 output row stride is a multiple of 4 (m)
zq16 = torch.empty((a.n, LDZ), dtype=torch.int16, device="cuda")
if a.q16:
    d16 = Depth16.synth(TorchAlloc(0), dev.ctx, bench.SEED, a.n, a.m, 0, bench.NCL)
    del q
    torch.cuda.empty_cache()
cases = {"full16": (zq16, st.zb), "full": (zq32, st.zb), "no_zq": (None, st.zb), "no_zb": (zq32, None),
         "read_only": (None, None)}
res = {}
nesc = 0
for rep in range(a.reps):
    for g in a.groups.split(","):
        os.environ["GRID_ZQUANT_GROUPS"] = g
        for name, (zq, zb) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if name == "full16":
                ne = C.c_int64()
                if a.q16:
                    call("grid_norm_zquant_kb16_q16", dev.ctx, C.byref(d16.desc), a.n, d16.ld, ptr(st.sel), st.r_loc,
                         ptr(st.rm), ptr(st.mu), st.scale, ptr(zq), LDZ, ptr(st.colmap), st.qmax, ptr(zb),
                         st.np_, ptr(st.esc_idx), ptr(st.esc_val), st.esc_idx.numel(), C.byref(ne), C.byref(of))
                else:
                    call("grid_norm_zquant_kb16", dev.ctx, q.data_ptr(), a.n, a.m, ptr(st.sel), st.r_loc, ptr(st.rm),
                         ptr(st.mu), st.scale, ptr(zq), LDZ, ptr(st.colmap), st.qmax, ptr(zb), st.np_,
                         ptr(st.esc_idx), ptr(st.esc_val), st.esc_idx.numel(), C.byref(ne), C.byref(of))
                nesc = ne.value
            elif a.q16:
                call("grid_norm_zquant_kb_q16", dev.ctx, C.byref(d16.desc), a.n, d16.ld, ptr(st.sel), st.r_loc,
                     ptr(st.rm), ptr(st.mu), st.scale, ptr(zq), st.r_loc, ptr(st.colmap), st.qmax, ptr(zb), st.np_,
                     C.byref(of))
            else:
                call("grid_norm_zquant_kb", dev.ctx, q.data_ptr(), a.n, a.m, ptr(st.sel), st.r_loc, ptr(st.rm),
                     ptr(st.mu), st.scale, ptr(zq), st.r_loc, ptr(st.colmap), st.qmax, ptr(zb), st.np_, C.byref(of))
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(f"{name} groups={g}", []).append(e0.elapsed_time(e1))
for setting in [x for x in a.env.split(";") if x]:
    kv = dict(p.split("=") for p in setting.split(","))
    old_env = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    ts = []
    for rep in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ne = C.c_int64()
        e0.record()
        if a.q16:
            call("grid_norm_zquant_kb16_q16", dev.ctx, C.byref(d16.desc), a.n, d16.ld, ptr(st.sel), st.r_loc,
                 ptr(st.rm), ptr(st.mu), st.scale, ptr(zq16), LDZ, ptr(st.colmap), st.qmax, ptr(st.zb),
                 st.np_, ptr(st.esc_idx), ptr(st.esc_val), st.esc_idx.numel(), C.byref(ne), C.byref(of))
        else:
            call("grid_norm_zquant_kb16", dev.ctx, q.data_ptr(), a.n, a.m, ptr(st.sel), st.r_loc, ptr(st.rm),
                 ptr(st.mu), st.scale, ptr(zq16), LDZ, ptr(st.colmap), st.qmax, ptr(st.zb), st.np_,
                 ptr(st.esc_idx), ptr(st.esc_val), st.esc_idx.numel(), C.byref(ne), C.byref(of))
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    res[f"full16 {setting}"] = ts
    for k, v in old_env.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
R = st.r_loc
for name, t in res.items():
    print(f"{name}: min {min(t):.2f} ms  median {np.median(t):.2f} ms", flush=True)
print(f"escapes (int16 form): {nesc}")
print(f"bytes: q {a.n * a.m * (2 if a.q16 else 4) / 1e9:.1f} GB, zq {a.n * R * 4 / 1e9:.1f} GB, zb {st.np_ * st.kpad * 2 / 1e9:.1f} GB")
