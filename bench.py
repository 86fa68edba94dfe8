#!/usr/bin/env python3
"""Benchmark: GRiD steps 4-7 end to end on MI355X (BASELINE.json metric).

One "step" = one pass of the device-resident steps 4-7 chain
(grid_amd/fused.py) over the BASELINE config-2 cohort: 3,202 samples x
3,000,000 bins (hg38 @ 1 kb), k = 10 neighbours, n_iters = 100, synthetic
data generated in HBM before timing.  value = samples / s (whole job).

Multi-GPU (torch.distributed.run, one rank per GPU, RCCL): the same cohort is
bin-sharded in 8192-aligned ranges (strong scaling); the Gram all-reduce is
the only data-path collective.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

METRIC = "samples/sec end-to-end steps 4–7 (50k×3M bins); k-NN distance HBM GB/s vs peak"
PEAK_BF16_TFLOPS = 2516.6     # 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (dense), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
# HBM bytes per Gram launch from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes
# of this same command (tools/gpu_round.sh -> tools/pmc_traffic.py)
TRAFFIC_JSON = "profiles/r01h_pmc_traffic.json"
GRAM_KERNEL = "k_gram8<0, true"
SEED = 20260821
NCL = 26
M64 = (1 << 64) - 1


def mix(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def sample_meta(n, seed=SEED):
    """Cluster and depth scale of each synthetic sample (same hash as
    grid_amd/csrc/synth.hip)."""
    clus = np.empty(n, dtype=np.int64)
    scale = np.empty(n)
    for i in range(n):
        hs = mix(seed ^ (0xA5A5 << 48) ^ i)
        clus[i] = mix(hs) % NCL
        scale[i] = 0.6 + 0.8 * ((hs >> 40) / 16777216.0)
    return clus, scale


def synth_reads_and_ibs(n, seed=SEED, per_hap=10):
    """Read counts (~CN x depth) and a computeIBSpbwt-like hap-neighbour CSR:
    ``per_hap`` same-cluster haplotype neighbours per haplotype."""
    clus, scale = sample_meta(n, seed)
    rng = np.random.default_rng(seed)
    cn = rng.choice([1.0, 1.5, 2.0, 2.5], size=n)
    reads = np.rint(400.0 * scale * cn * rng.uniform(0.9, 1.1, n))
    members = [np.where(clus == c)[0] for c in range(NCL)]
    off = np.zeros(2 * n + 1, dtype=np.int64)
    nbr = []
    for h in range(2 * n):
        pool = members[clus[h // 2]]
        js = pool[rng.integers(0, len(pool), per_hap)] if len(pool) else np.zeros(0, np.int64)
        hs = rng.integers(0, 2, len(js))
        nbr.extend((2 * js + hs).tolist())
        off[h + 1] = off[h] + len(js)
    nbr = np.array(nbr, dtype=np.int32)
    return reads, off, nbr, np.ones(len(nbr))


def cpu_baseline(q_host, n, m_total, reads, off, nbr, w, k, n_iters):
    """The oracle (NumPy restatement of the reference, oracle/) timed on this
    host on a bounded column sample of the same cohort; normalisation and
    k-NN (linear in bins) are scaled to the full bin count."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import steps
    from oracle.npsum import nanmean_rows
    ms = q_host.shape[1]
    mat = q_host / 100.0
    t0 = time.perf_counter()
    raw = nanmean_rows(mat)
    z, ratios, mu, var, scale = steps.normalize_matrix(mat)
    sel = steps.select_high_variance_regions(ratios, 0.1)
    zs = np.round(z[:, sel], 2)        # stands in for the %.2f write/read round trip
    t1 = time.perf_counter()
    r3 = np.round(np.array([ratios[j] for j in sel]), 3)
    idx, ruse = steps.filter_regions_by_variance(r3, 1.0, 1000.0)
    qz = np.clip(np.rint(zs[:, idx] * 100), -200, 200).astype(np.int64)
    nb = steps.knn_exact(qz, k)
    t2 = time.perf_counter()
    ids = [f"S{i:06d}" for i in range(n)]
    sc = {ids[i]: float(f"{raw[i]:.2f}") for i in range(n)}
    nbrs = {ids[i]: [(ids[j], sc[ids[j]]) for j, _ in nb[i]] for i in range(n)}
    rd = {ids[i]: float(reads[i]) for i in range(n)}
    dip = steps.dipcn(nbrs, sc, rd, 300)
    t3 = time.perf_counter()
    irr = [v for _, v in dip]
    hn = [[(int(nbr[t]), float(w[t])) for t in range(off[h], off[h + 1])] for h in range(2 * n)]
    hap, mean = steps.run_phasing(irr, hn, 1, n_iters)
    _ = [steps.compute_imp(i, hap, hn, mean) for i in range(n)]
    t4 = time.perf_counter()
    f = m_total / ms
    total = (t1 - t0) * f + (t2 - t1) * f + (t3 - t2) + (t4 - t3)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": n / total, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": (f"oracle steps 4-7 on {n} samples x {ms} bins of the same cohort "
                       f"(normalise {t1 - t0:.2f}s + kNN {t2 - t1:.2f}s scaled x{f:.1f} to {m_total} bins; "
                       f"dipCN {t3 - t2:.2f}s, phasing {t4 - t3:.2f}s unscaled)")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--samples", type=int, default=3202)
    ap.add_argument("--bins", type=int, default=3_000_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-iters", type=int, default=100)
    ap.add_argument("--cpu-bins", type=int, default=16384)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap", action="store_true", help="run step 7 inline on the main stream")
    ap.add_argument("--depth-format", choices=["int32", "q16"], default="int32",
                    help="depth matrix in HBM: int32 hundredths (default) or the compact uint16 + escapes form "
                         "(half the bytes; measured slower: the step-4 passes are not byte-bound)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GRID_BENCH_SHARE_GPU=1 (rehearsal only): ranks share the visible GPUs
    # round-robin, with GRID_DIST_BACKEND=gloo since RCCL needs one GPU per rank
    if os.environ.get("GRID_BENCH_SHARE_GPU") == "1":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist = None
    comm = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("GRID_DIST_BACKEND", "nccl")     # "nccl" = RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        from grid_amd.fused import TorchComm
        comm = TorchComm(dist)

    from grid_amd import _abi
    from grid_amd.fused import Depth16, HipOps, Steps47, TorchAlloc, shard_range

    dev = _abi.Device(local)
    dev.set_stream(torch.cuda.current_stream())
    n, m = args.samples, args.bins
    c0, c1 = shard_range(m, rank, world)
    ml = c1 - c0
    talloc = TorchAlloc(local)
    if args.depth_format == "q16":
        # compact depth matrix: uint16 hundredths + escape table (half the HBM
        # bytes of the four step-4 passes; same int32 values after decoding)
        q = Depth16.synth(talloc, dev.ctx, SEED, n, ml, c0, NCL)
        ldq = q.ld
    else:
        q = torch.empty((n, max(ml, 1)), dtype=torch.int32, device="cuda")
        _abi.call("grid_synth_depth", dev.ctx, SEED, n, ml, ml, c0, NCL, q.data_ptr())
        ldq = ml
    reads, off, nbr, w = synth_reads_and_ibs(n)
    # step 7 on its own stream: it overlaps the next pass's steps 4-5 (every
    # pass is still complete inside the timed region: the final synchronize
    # waits for both streams)
    lane = None
    if not args.no_overlap:
        pdev = _abi.Device(local)
        pstream = torch.cuda.Stream()
        pdev.set_stream(pstream)
        lane = (HipOps(pdev), pstream)
    st = Steps47(HipOps(dev), talloc, n, m, c0, ml, k=args.k, n_nbr=300, top_frac=0.1, zmax=2.0,
                 sigma2_max=1000.0, frac_r=1.0, min_nbr=1, n_iters=args.n_iters, comm=comm, phase_lane=lane)
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)

    for _ in range(args.warmup):
        st.run(q, ldq)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.steps):
        st.run(q, ldq, gram_events=ev[s])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    gram_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    st.run(q, ldq, profile=True)              # untimed pass: per-stage device times
    torch.cuda.synchronize()
    stages = {k: round(v, 3) for k, v in st.stage_ms().items()}

    valid = int(st.valid[:n].sum().item())
    traffic, tsrc = None, None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), TRAFFIC_JSON)
    if os.path.exists(tpath):
        tk = json.load(open(tpath))["kernels"]
        hits = [v for k, v in tk.items() if k.startswith(GRAM_KERNEL)]
        if hits and n == 3202 and m == 3_000_000 and world == 1:
            traffic, tsrc = hits[0]["traffic_bytes"], TRAFFIC_JSON
    flops = 2.0 * n * n * st.ruse_loc                       # 2 N^2 R_use per launch
    nt, ni = st.np_ // 128, st.np_ // 256            # k_gram8: 256x128 tiles (I, j >= 2I)
    executed = 2.0 * sum(nt - 2 * i for i in range(ni)) * 256 * 128 * (-(-st.ruse_loc // 64) * 64)
    out = {
        "metric": METRIC,
        "value": n * args.steps / elapsed,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64 (statistics) + bf16-MFMA exact-integer (k-NN)",
        "data": "synthetic (counter-based cohort generated in HBM; 26 ancestry clusters)",
        "config": {"workload": f"BASELINE config 2: {n} samples x {m} bins (hg38 @ 1 kb), k={args.k}, "
                               f"n_iters={args.n_iters}", "samples": n, "bins": m, "k": args.k,
                   "n_iters": args.n_iters, "parallelism": f"bin-sharded x{world}",
                   "depth_format": args.depth_format,
                   "selected_regions": None, "R_use_rank0": st.ruse_loc, "dipcn_valid": valid,
                   "phasing_levels": st.nlev},
        "stages_ms": stages,
        "roofline": {"kernel": "k_gram (exact bf16-MFMA Gram)", "bound": "mfma",
                     "achieved": flops / (gram_ms * 1e-3) / 1e12, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": flops / (gram_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS,
                     "traffic": traffic, "traffic_source": tsrc,
                     "hbm_gbs": traffic / (gram_ms * 1e-3) / 1e9 if traffic else None,
                     "hbm_frac": traffic / (gram_ms * 1e-3) / 1e9 / PEAK_HBM_GBS if traffic else None,
                     "gram_ms": gram_ms,
                     "executed_mfma_tflops": executed / (gram_ms * 1e-3) / 1e12,
                     "flops_def": "2*N^2*R_use per launch (SURVEY 8d); executed = the 256x128 upper-triangle "
                                  "tiles k_gram8 computes"},
    }
    out["config"]["selected_regions"] = st.r_loc if world == 1 else None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ms = min(args.cpu_bins, ml)
        qs = torch.empty((n, ms), dtype=torch.int32, device="cuda")   # same cells, int32 form
        _abi.call("grid_synth_depth", dev.ctx, SEED, n, ms, ms, c0, NCL, qs.data_ptr())
        qh = qs.cpu().numpy()
        del qs
        out["cpu_baseline"] = cpu_baseline(qh, n, m, reads, off, nbr, w, args.k, args.n_iters)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
