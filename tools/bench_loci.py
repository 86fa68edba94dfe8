"""BASELINE config 5: batched haplotype phasing of many loci (VNTR regions)
in one launch, one workgroup per locus (grid_hi_phase_batch).

Synthetic cohort: per locus, IRRs ~ CN x U(0.9, 1.1) and an IBS-like graph of
``--per-hap`` same-cluster haplotype neighbours per haplotype (26 clusters),
as bench.py builds for one locus.  Prints one JSON line: loci/s,
sample-iterations/s, and the oracle (NumPy/Python restatement of the
reference _run_phasing) timed on one small locus of the same kind on this
host, scaled per sample-iteration.

    python tools/bench_loci.py [--loci 734] [--samples 10000] [--iters 100]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from grid_amd import _abi, engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--loci", type=int, default=734)
ap.add_argument("--samples", type=int, default=10000)
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--per-hap", type=int, default=10)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cpu-samples", type=int, default=1000)
ap.add_argument("--paired", action="store_true", help="A/B: the two-haplotypes-per-lane kernel")
ap.add_argument("--inflight", type=int, default=3, help="groups of loci running at once (engine.phase_batch)")
ap.add_argument("--group", type=int, default=0, help="loci per group (0: the CU count)")
a = ap.parse_args()


def locus(rng, n, per_hap):
    clus = rng.integers(0, 26, n)
    irr = rng.choice([1.0, 1.5, 2.0, 2.5, 3.0], size=n) * rng.uniform(0.9, 1.1, n)
    order = np.argsort(clus, kind="stable")
    start = np.searchsorted(clus[order], np.arange(26))
    size = np.bincount(clus, minlength=26)
    hc = np.repeat(clus, 2)                                   # cluster of each haplotype
    pick = (rng.random((2 * n, per_hap)) * size[hc][:, None]).astype(np.int64)
    js = order[start[hc][:, None] + pick]
    nbr = (2 * js + rng.integers(0, 2, js.shape)).astype(np.int32).reshape(-1)
    off = np.arange(0, 2 * n * per_hap + 1, per_hap, dtype=np.int64)
    return irr, off, nbr, np.ones(len(nbr))


rng = np.random.default_rng(20260821)
t0 = time.perf_counter()
loci = [locus(rng, a.samples, a.per_hap) for _ in range(a.loci)]
gen_s = time.perf_counter() - t0
dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
res, times = None, []
for rep in range(a.reps + 1):          # first call: schedules, uploads and warm-up
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = engine.phase_batch(dev, loci, 1, a.iters, paired=a.paired, group=a.group or None, inflight=a.inflight)
    torch.cuda.synchronize()
    times.append(time.perf_counter() - t1)


# the phasing launch alone (device time) on the prepared batch: rerun with events
def device_ms():
    import ctypes as C
    sched = [_abi.hi_schedule(off, nbr, w, packed_w=False) for _, off, nbr, w in loci]
    keep, descs = [], []
    for (irr, off, nbr, w), (order, loff, nl, pk_nbr, pk_w, pk_cnt, flags, ml) in zip(loci, sched):
        b = [None if x is None else dev.upload(np.ascontiguousarray(x))
             for x in (irr, off, nbr.astype(np.int32), w, order.astype(np.int32), loff.astype(np.int32), pk_nbr,
                       pk_w, pk_cnt)]
        outs = [dev.alloc(2 * len(irr), np.float64), dev.alloc(2 * len(irr), np.float64), dev.alloc(1, np.float64)]
        keep += b + outs
        pk = [None if x is None else x.ptr for x in b[6:]]     # pk_w None: unit weights, not packed
        descs.append(_abi.HiLocus(len(irr), *[x.ptr for x in b[:6]], nl, 0, *pk, *[x.ptr for x in outs]))
    arr = (_abi.HiLocus * len(descs))(*descs)
    d = dev.alloc(C.sizeof(arr), np.uint8)
    _abi.call("grid_h2d", dev.ctx, d.ptr, C.addressof(arr), C.sizeof(arr))
    max_nl = max(s[2] for s in sched)
    max_list = max(s[7] for s in sched)
    ms = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _abi.call("grid_hi_phase_batch", dev.ctx, len(descs), d.ptr, a.samples, max_nl, 1, a.iters,
                  1 | (_abi.HI_PAIRED if a.paired else 0), max_list)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return min(ms), max_nl


gpu_ms, max_nl = device_ms()
# oracle on one small locus of the same kind (host cores; pure Python loops)
from oracle import steps  # noqa: E402
irr, off, nbr, w = locus(np.random.default_rng(1), a.cpu_samples, a.per_hap)
hn = [[(int(nbr[t]), 1.0) for t in range(off[h], off[h + 1])] for h in range(2 * a.cpu_samples)]
c_iters = 5
t2 = time.perf_counter()
steps.run_phasing(list(irr), hn, 1, c_iters)
cpu_per_si = (time.perf_counter() - t2) / (a.cpu_samples * c_iters)
si = a.loci * a.samples * a.iters
print(json.dumps({
    "metric": "loci/s batched haplotype phasing (config 5)", "value": a.loci / (gpu_ms * 1e-3), "unit": "loci/s",
    "config": {"loci": a.loci, "samples": a.samples, "n_iters": a.iters, "per_hap": a.per_hap,
               "max_levels": max_nl, "inflight": a.inflight, "group": a.group},
    "device_ms": gpu_ms, "sample_iters_per_s": si / (gpu_ms * 1e-3),
    "end_to_end_s": min(times[1:]), "first_call_s": times[0], "synthetic_generation_s": gen_s,
    "cpu_baseline": {"sample_iters_per_s": 1.0 / cpu_per_si, "cores": 1, "kind": "port",
                     "sample": f"oracle run_phasing on one {a.cpu_samples}-sample locus x {c_iters} iterations",
                     "loci_per_s_scaled": 1.0 / (cpu_per_si * a.samples * a.iters)},
}), flush=True)
