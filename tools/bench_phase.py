"""Time the phasing kernel alone at the bench shape for several n_iters."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from grid_amd import _abi  # noqa: E402
from grid_amd.fused import TorchAlloc  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3202
dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
reads, off, nbr, w = bench.synth_reads_and_ibs(n)
order, loff, nl, pk_nbr, pk_w, pk_cnt = _abi.hi_schedule(off, nbr, w)
A = TorchAlloc(0)
irr = A.upload(np.random.default_rng(0).uniform(0.5, 3, n))
d = [A.upload(x) for x in (off.astype(np.int64), nbr.astype(np.int32), w.astype(np.float64),
                           order.astype(np.int32), loff.astype(np.int32), pk_nbr, pk_w, pk_cnt)]
hap, imp, mean = A.empty(2 * n, np.float64), A.empty(2 * n, np.float64), A.empty(1, np.float64)
print("levels", nl, "sizes min/max", np.diff(loff).min(), np.diff(loff).max())
for it in (0, 1, 10, 100):
    ts = []
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _abi.call("grid_hi_phase", dev.ctx, n, irr.data_ptr(), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                  1, it, d[3].data_ptr(), d[4].data_ptr(), nl, d[5].data_ptr(), d[6].data_ptr(), d[7].data_ptr(),
                  hap.data_ptr(), imp.data_ptr(), mean.data_ptr())
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"iters {it}: {min(ts):.3f} ms  -> per level {(min(ts)) / max(it * nl, 1) * 1000:.2f} us", flush=True)
