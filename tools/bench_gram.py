"""A/B microbenchmark of the exact Gram kernel variants at the bench shape
(interleaved in one process, random integer data in [-qmax, qmax]).

    python tools/bench_gram.py [--n 3202] [--k 2700000] [--reps 3]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# timing probes and A/B kernels live in the tools build only (make -C grid_amd/csrc probes)
os.environ.setdefault("GRID_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "grid_amd", "_lib", "libgridhip_probes.so"))
from grid_amd import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=3202)
ap.add_argument("--k", type=int, default=2_700_000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--variants", default="21,kb21")
ap.add_argument("--qmax", type=int, default=200)
ap.add_argument("--ld-extra", type=int, default=0, help="extra bf16 columns of row padding (row stride)")
a = ap.parse_args()

np_ = -(-a.n // 256) * 256
kpad = -(-a.k // 64) * 64
dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
g = torch.Generator(device="cuda").manual_seed(1)
ld = kpad + a.ld_extra
zb = torch.zeros((np_, ld), dtype=torch.int16, device="cuda")
for r0 in range(0, a.n, 256):
    r1 = min(a.n, r0 + 256)
    zi = torch.randint(-a.qmax, a.qmax + 1, (r1 - r0, kpad), device="cuda", dtype=torch.int32, generator=g)
    zb[r0:r1, :kpad] = zi.to(torch.bfloat16).view(torch.int16)
    del zi
gram = torch.zeros((np_, np_), dtype=torch.int64, device="cuda")
# "kbNN": variant NN through grid_knn_gram_kb on the K-blocked panel [kpad/KBW][row][KBW]
zbb = None
if any(v.startswith("kb") for v in a.variants.split(",")):   # K-blocked [kpad/KBW][np][KBW]
    zbb = zb[:, :kpad].reshape(np_, kpad // _abi.KBW, _abi.KBW).permute(1, 0, 2).contiguous()
res = {}
first = None
flops = 2.0 * a.n * a.n * a.k
for rep in range(a.reps):
    for vv in a.variants.split(","):
        # "kb21:LAG=2:KC=9" -> variant kb21 with GRID_GRAM_LAG=2, GRID_GRAM_KC=9 (performance knobs)
        v, *knobs = vv.split(":")
        for kv in ("LAG", "SPIN", "KC", "KX", "QL", "UF", "DYN", "PART_MB", "Q16", "PER", "GS"):
            os.environ.pop("GRID_GRAM_" + kv, None)
        for kv in knobs:
            key, val = kv.split("=")
            os.environ["GRID_GRAM_" + key] = val
        os.environ["GRID_GRAM_VARIANT"] = v[2:] if v.startswith("kb") else v
        gram.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if v.startswith("kb"):
            _abi.call("grid_knn_gram_kb", dev.ctx, zbb.data_ptr(), np_, kpad, a.qmax, gram.data_ptr())
        else:
            _abi.call("grid_knn_gram", dev.ctx, zb.data_ptr(), np_, kpad, ld, a.qmax, gram.data_ptr())
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        res.setdefault(vv, []).append(ms)
        if rep == 0:
            # check a few upper-triangle tiles against a float64 product on the GPU
            zz = zb[:256, :kpad].view(torch.bfloat16).double()
            ref = (zz @ zz.T).long()
            ok = torch.equal(gram[:128, :256], ref[:128, :256])
            # every variant's whole Gram (upper tiles) against the first variant's
            if first is None:
                first = gram.clone()
                same = True
            else:
                same = torch.equal(gram, first)
            print(f"variant {vv}: tile check {'OK' if ok else 'MISMATCH'}, "
                  f"whole Gram {'equal to' if same else 'DIFFERENT from'} the first variant", flush=True)
for v, t in res.items():
    ms = min(t)
    print(f"variant {v}: min {ms:.2f} ms  median {np.median(t):.2f} ms  "
          f"-> {flops / ms / 1e9:.0f} TFLOP/s (2N^2K), {flops / ms / 1e9 / 2516.6 * 100:.1f}% of bf16 peak",
          flush=True)
