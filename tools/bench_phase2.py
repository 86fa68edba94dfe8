"""Phasing kernel cost vs neighbour-list length (same level structure): the
default k_phase4 (256 lanes) against round 5's split-lane kernel
(GRID_HI_PH2), the paired-lane one (GRID_HI_PAIRED) and the per-neighbour one
(GRID_HI_LEGACY).  ``--probes``: the timing probes of the paired kernel
(libgridhip_probes.so).  ``--json PATH``: the timings as JSON."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PROBES = "--probes" in sys.argv
JSON = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
if PROBES:
    # the timing probes live in the tools build only (make -C grid_amd/csrc probes)
    os.environ.setdefault("GRID_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                        "grid_amd", "_lib", "libgridhip_probes.so"))
import bench  # noqa: E402
from grid_amd import _abi  # noqa: E402
from grid_amd.fused import TorchAlloc  # noqa: E402

n = 3202
dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
A = TorchAlloc(0)
reads, off0, nbr0, w0 = bench.synth_reads_and_ibs(n)
order, loff, nl = _abi.hi_levels(off0, nbr0)        # keep the real schedule
irr = A.upload(np.random.default_rng(0).uniform(0.5, 3, n))
res = {"n": n, "levels": int(nl), "sweeps": 100, "ms": {}}
outs = {}
for keep in (10, 0):
    # truncate every list to `keep` entries, same schedule
    off = np.zeros_like(off0)
    nb, ww = [], []
    for h in range(2 * n):
        seg = nbr0[off0[h]:off0[h + 1]][:keep]
        nb += seg.tolist()
        ww += [1.0] * len(seg)
        off[h + 1] = off[h] + len(seg)
    nb = np.array(nb, np.int32)
    ww = np.array(ww)
    pk_nbr = np.zeros((n, 2, 16), np.int32)
    pk_w = np.zeros((n, 2, 16))
    pk_cnt = np.zeros((n, 2), np.int32)
    _abi.call("grid_hi_pack", n, off.ctypes.data, (nb if nb.size else np.zeros(1, np.int32)).ctypes.data,
              (ww if ww.size else np.zeros(1)).ctypes.data, order.ctypes.data, 16, pk_nbr.ctypes.data,
              pk_w.ctypes.data, pk_cnt.ctypes.data)
    d = [A.upload(x) for x in (off, nb if nb.size else np.zeros(1, np.int32), ww if ww.size else np.zeros(1),
                               order, loff, pk_nbr, pk_w, pk_cnt)]
    hap, imp, mean = A.empty(2 * n, np.float64), A.empty(2 * n, np.float64), A.empty(1, np.float64)
    runs = [(1, "k_phase4", "0"), (1 | 8, "k_phase2_split_r5", "0"), (1 | 4, "paired", "0"),
            (1 | 2, "legacy", "0")]
    if PROBES:
        runs += [(1 | 4 | 8, "paired-probe-noprefetch", "1"), (1 | 4 | 8, "paired-probe-noarith", "2"),
                 (1 | 4 | 8, "paired-probe-barriers-only", "3"),
                 (1, "k_phase4-probe-nobarriers", "4"), (1, "k_phase4-probe-nowork", "5"),
                 (1, "k_phase4-probe-noprefetch", "6"), (1, "k_phase4-probe-barriers-only", "7")]
    for flags, name, probe in runs:
        os.environ["GRID_PHASE_PROBE"] = probe
        ts = []
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _abi.call("grid_hi_phase", dev.ctx, n, irr.data_ptr(), d[0].data_ptr(), d[1].data_ptr(),
                      d[2].data_ptr(), 0, 100, d[3].data_ptr(), d[4].data_ptr(), nl, d[5].data_ptr(),
                      d[6].data_ptr(), d[7].data_ptr(), hap.data_ptr(), imp.data_ptr(), mean.data_ptr(), flags, keep)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"{name} list len {keep}: {min(ts):.3f} ms -> {min(ts) / (100 * nl) * 1000:.2f} us/level", flush=True)
        res["ms"][f"{name}/len{keep}"] = round(min(ts), 4)
        if probe == "0":
            got = (hap.cpu().numpy().tobytes(), imp.cpu().numpy().tobytes(), float(mean.item()))
            ref = outs.setdefault(keep, got)
            assert got == ref, f"{name} differs from k_phase4 at list length {keep}"
if JSON:
    with open(JSON, "w") as f:
        json.dump(res, f, indent=1)
