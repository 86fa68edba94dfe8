"""Reference point for the Gram kernel: the vendor bf16 GEMM (hipBLASLt via
torch.matmul, fp32 accumulation, bf16 output -- NOT exact, timing only) on
integer data in [-200, 200].  Reports executed TFLOP/s per shape, to compare
with k_gram8's executed-MFMA rate (bench.py roofline.executed_mfma_tflops).

    python tools/bench_blaslt.py
"""
import json

import torch

SHAPES = [(3328, 3328, 2_700_032), (16384, 16384, 65536), (8192, 8192, 262144), (50176, 12544, 65536)]
res = []
for m, n, k in SHAPES:
    a = torch.randint(-200, 201, (m, k), device="cuda", dtype=torch.int16).to(torch.bfloat16)
    b = a[:n] if n <= m else torch.randint(-200, 201, (n, k), device="cuda", dtype=torch.int16).to(torch.bfloat16)
    out = torch.matmul(a, b.t())
    torch.cuda.synchronize()
    ms = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = torch.matmul(a, b.t())
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    t = min(ms)
    res.append({"m": m, "n": n, "k": k, "ms": t, "tflops": 2.0 * m * n * k / t / 1e9})
    print(json.dumps(res[-1]), flush=True)
    del a, b, out
    torch.cuda.empty_cache()
