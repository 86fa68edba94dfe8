#!/usr/bin/env python3
"""Benchmark: GRiD steps 4-7 end to end on MI355X (BASELINE.json metric).

The headline: ONE step = one whole
`grid wgs` run FROM FILES -- run_wgs_pipeline over BASELINE config 2 (3,202
mosdepth BGZF regions.bed.gz files x 3,000,000 bins, k = 10, n_iters = 100):
ingest, normalisation, the normalised gz file written, neighbours, dipCN,
haploid calls, every output file written.  value = samples / s of those runs
(whole job).  The cohort is generated before the clock (tools/gen_cohort, the
bench's depth model as mosdepth text) in --files-dir.  With --gpus N the N
ranks run the distributed drop-in (grid_amd/utils/dist_step4.py: files
sliced over the ranks, all-to-all to column shards, RCCL collectives,
offset-placed writer); steps 6-7 on rank 0.

Beside it, in the same line:
  * device_chain: the device-resident chain of steps 4-7 (grid_amd/fused.py)
    on the same shape, the depth matrix generated in HBM before timing --
    its Gram is the line's roofline (the metric's "k-NN distance vs peak");
  * config3_1gpu (N = 1): the metric's own 50k x 3M shape, bin-streamed;
  * cpu_baseline: the oracle on a bounded slice, and the committed sweep.

Multi-GPU: one rank per GPU over RCCL.  ``--gpus N`` without an external
launcher starts ``torch.distributed.run`` with N ranks as a child process
before anything touches the GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--headline files|chain]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

METRIC = "samples/sec end-to-end steps 4–7 (50k×3M bins); k-NN distance HBM GB/s vs peak"
PEAK_BF16_TFLOPS = 2516.6     # 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (dense), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
# HBM bytes per Gram launch from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes
# of this same command (tools/gpu_round.sh -> tools/pmc_traffic.py)
TRAFFIC_JSON = "profiles/r05az_pmc_traffic.json"
# the oracle from files over N x M, per-stage fits (tools/cpu_sweep.py,
# run on a GPU box's host cores); reported beside the live bounded sample
CPU_SWEEP_JSON = "profiles/r04k_cpu_sweep.json"
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


def cpu_baseline(q_host, n_total, m_total, k, n_iters, seed=SEED):
    """The oracle (NumPy restatement of the reference, oracle/) timed on this
    host on a bounded sample of the same cohort: the first ns samples x ms
    bins (q_host).  Each stage is scaled by its complexity to the full
    workload: normalisation by (n m) / (ns ms), k-NN by (n^2 m) / (ns^2 ms),
    dipCN and phasing by n / ns."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import steps
    from oracle.npsum import nanmean_rows
    ns, ms = q_host.shape
    reads, off, nbr, w = synth_reads_and_ibs(ns, seed)
    mat = np.where(q_host == -(2 ** 31), np.nan, q_host / 100.0)
    t0 = time.perf_counter()
    raw = nanmean_rows(mat)
    z, ratios, mu, var, scale = steps.normalize_matrix(mat)
    sel = steps.select_high_variance_regions(ratios, 0.1)
    zs = np.round(z[:, sel], 2)        # stands in for the %.2f write/read round trip
    t1 = time.perf_counter()
    r3 = np.round(np.array([ratios[j] for j in sel]), 3)
    idx, ruse = steps.filter_regions_by_variance(r3, 1.0, 1000.0)
    qz = np.clip(np.rint(np.nan_to_num(zs[:, idx], nan=0.0) * 100), -200, 200).astype(np.int64)
    nb = steps.knn_exact(qz, k)
    t2 = time.perf_counter()
    ids = [f"S{i:06d}" for i in range(ns)]
    sc = {ids[i]: float(f"{raw[i]:.2f}") for i in range(ns)}
    nbrs = {ids[i]: [(ids[j], sc[ids[j]]) for j, _ in nb[i]] for i in range(ns)}
    rd = {ids[i]: float(reads[i]) for i in range(ns)}
    dip = steps.dipcn(nbrs, sc, rd, 300)
    t3 = time.perf_counter()
    irr = [v for _, v in dip]
    hn = [[(int(nbr[t]), float(w[t])) for t in range(off[h], off[h + 1])] for h in range(2 * ns)]
    hap, mean = steps.run_phasing(irr, hn, 1, n_iters)
    _ = [steps.compute_imp(i, hap, hn, mean) for i in range(ns)]
    t4 = time.perf_counter()
    return scale_cpu_baseline((ns, ms, t1 - t0, t2 - t1, t3 - t2, t4 - t3), n_total, m_total)


def scale_cpu_baseline(meas, n_total, m_total):
    """The oracle sample's stage times scaled by complexity to n_total x
    m_total: normalisation n m, k-NN n^2 m, dipCN and phasing n."""
    ns, ms, tn, tk, td, tp = meas
    fn, fm = n_total / ns, m_total / ms
    total = tn * fn * fm + tk * fn * fn * fm + td * fn + tp * fn
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": n_total / total, "unit": "samples/s", "cores": threads, "kind": "port", "measured": meas,
            "sample": (f"oracle steps 4-7 on the first {ns} samples x {ms} bins of the same cohort, scaled to "
                       f"{n_total} x {m_total}: normalise {tn:.2f}s x{fn * fm:.1f}, kNN {tk:.2f}s "
                       f"x{fn * fn * fm:.1f}, dipCN {td:.2f}s x{fn:.1f}, phasing {tp:.2f}s x{fn:.1f} "
                       f"(extrapolated; host memory bounds the reference well below this shape)")}


def cpu_baseline_from_files(n_target, m_target, k, n_iters):
    """The reference's whole step cost, file to file: the oracle's steps 4-7
    (oracle/pipeline.py: mosdepth gzip parse, normalize_matrix, "%.2f"/"%.3f"
    text into gzip level 9, re-read and parse in step 5, exact k-NN, dipCN,
    phasing), measured on BASELINE config 1 (100 samples x 30k bins, k=10;
    the cohort regenerated from tests/golden/g_cfg1's seed) on this host's
    cores, then each stage scaled by its complexity to n_target x m_target:
    parse / normalise / text write / text read by cells (n m, selected
    columns ~ m), k-NN by n^2 m, dipCN and the neighbour file by n, phasing by
    n x n_iters / 100."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import pipeline
    from tests.golden import cohort_files
    tmp = tempfile.mkdtemp(prefix="grid_cfg1_")
    try:
        t0 = time.perf_counter()
        cfg, _, meta = cohort_files.regenerate("g_cfg1", tmp)
        gen = time.perf_counter() - t0
        t = pipeline.run(cfg)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    shape = t.pop("shape")
    n1, m1 = meta["n"], meta["m"]
    cells = (n_target * m_target) / (n1 * m1)
    knn = (n_target / n1) ** 2 * (m_target / m1)
    lin = n_target / n1
    scale = {"ingest": cells, "normalize": cells, "write_normalized": cells, "read_normalized": cells,
             "knn": knn, "write_neighbors": lin, "dipcn": lin, "load_hap_neighbors": lin,
             "phasing": lin * n_iters / 100.0, "write_haploid": lin}
    total1 = sum(t.values())
    est = {kk: v * scale[kk] for kk, v in t.items()}
    total = sum(est.values())
    return {"config1_measured": {"samples": n1, "bins": m1, "k": meta["k"], "stages_s": {kk: round(v, 3) for kk, v
            in t.items()}, "total_s": total1, "samples_per_s": n1 / total1, "shape": shape,
            "cohort_generation_s": gen},
            "extrapolated": {"samples": n_target, "bins": m_target, "total_s": total,
                             "samples_per_s": n_target / total,
                             "stages_s": {kk: round(v, 1) for kk, v in est.items()},
                             "note": "config-1 stage times scaled by complexity; the reference's fp64 matrix "
                                     "(8 B/cell) exceeds host memory well before this shape"},
            "cores": 1, "kind": "port",
            "sample": "oracle/pipeline.py steps 4-7 from mosdepth files to output files at BASELINE config 1 "
                      "(single-threaded Python/NumPy, as the reference runs with threads=1)"}


FILES_DIRNAME = "grid_bench_cfg2"


def prepare_files_cohort(data, out, n, m, gen_threads=16, threads=16, bgzf=True, note=print):
    """The from-files cohort in ``data``: ``n`` mosdepth regions.bed.gz files
    of ``m`` 1 kb bins (tools/gen_cohort: the bench's depth model as "%.2f"
    text, BGZF like mosdepth, libdeflate level 1), samples.txt, an empty
    repeat mask, the IBS hap-neighbour file (synth_reads_and_ibs), counts.tsv
    in ``out`` and config.yaml (`grid wgs` steps 4-7, k = 10, n_iters = 100).
    Runs before anything touches the GPU (a child process).  Returns
    (config path, generation seconds, cohort bytes)."""
    import gzip
    import yaml
    t0 = time.perf_counter()
    root = os.path.dirname(os.path.abspath(__file__))
    mos = os.path.join(data, "mosdepth")
    os.makedirs(mos, exist_ok=True)
    os.makedirs(out, exist_ok=True)
    gen = os.path.join(root, "tools", "gen_cohort")
    if not os.path.exists(gen) or os.path.getmtime(gen) < os.path.getmtime(gen + ".cpp"):
        subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", "-o", gen, gen + ".cpp", "-lz", "-ldl"], check=True)
    have = len([f for f in os.listdir(mos) if f.endswith(".regions.bed.gz")])
    if have != n:
        note(f"generating {n} x {m} mosdepth files in {mos}")
        subprocess.run([gen, mos, str(n), str(m), "20260821", str(gen_threads), "0"] + (["bgzf"] if bgzf else []),
                       check=True, stdout=sys.stderr)
    ids = [f"S{i:05d}" for i in range(n)]
    reads, off, nbr, w = synth_reads_and_ibs(n)
    with open(os.path.join(data, "samples.txt"), "w") as f:
        f.write("\n".join(ids) + "\n")
    with open(os.path.join(out, "counts.tsv"), "w") as f:
        f.write("Sample\tchr1:1-3000000000\n")
        f.writelines(f"{ids[i]}\t{int(reads[i])}\n" for i in range(n))
    with gzip.open(os.path.join(data, "ibs.tsv.gz"), "wt", compresslevel=1) as f:
        f.write("ID\thap\tnbrInd\tcMlen\tcMedge\tIDnbr\thapNbr\n")
        for h in range(2 * n):
            for t in range(off[h], off[h + 1]):
                j = int(nbr[t])
                f.write(f"{ids[h // 2]}\t{h % 2 + 1}\t{t - off[h]}\t5.0\t0\t{ids[j // 2]}\t{j % 2 + 1}\n")
    open(os.path.join(data, "mask.bed"), "w").close()
    cfg = {
        "samples_file": os.path.join(data, "samples.txt"), "output_dir": out, "threads": threads,
        "chrom": "chr1", "output_file_type": "tsv", "index": {"run": False},
        "count_reads": {"run": False, "output_file_prefix": "counts"},
        "mosdepth": {"run": False, "work_dir": mos, "remove_intermediate": False,
                     "normalize": {"run": True, "min_depth": 20, "max_depth": 100, "top_frac": 0.1,
                                   "device_ingest": True, "output_file_prefix": "normalized",
                                   "repeat_mask_file": os.path.join(data, "mask.bed")},
                     "neighbors": {"run": True, "output_file_prefix": "neighbors", "num_neighbors": 10, "zmax": 2.0,
                                   "sigma2_max": 1000}},
        "compute_diploid_genotypes": {"run": True, "output_file_prefix": "dipcn", "n_nbr": 10},
        "compute_haploid_genotypes": {"run": True, "output_file_prefix": "haploid", "method": "ibs",
                                      "min_neighbors": 1, "max_neighbors": 10, "n_iters": 100,
                                      "ibs_output": os.path.join(data, "ibs.tsv.gz")},
    }
    path = os.path.join(data, "config.yaml")
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)
    nbytes = sum(os.path.getsize(os.path.join(mos, f)) for f in os.listdir(mos))
    return path, time.perf_counter() - t0, nbytes


def files_paths(args):
    import tempfile
    data = os.path.join(args.files_dir, FILES_DIRNAME)
    out = os.path.join(tempfile.gettempdir(), FILES_DIRNAME + "_out")
    return data, out


def files_prepare(args, rank, local, world, note):
    """Rank 0 writes the cohort (before the GPU is touched); the other ranks
    of this job wait for its marker (the job's master port in it, so a
    marker left by another job is not taken).  Returns (config path,
    generation s, bytes) or a dict {"skipped": why}."""
    import shutil
    data, out = files_paths(args)
    marker = os.path.join(data, "READY")
    token = f"{os.environ.get('MASTER_PORT', 'solo')}:{args.samples}x{args.bins}"
    if rank == 0:
        try:
            free = shutil.disk_usage(args.files_dir).free
        except OSError as e:
            why = f"{args.files_dir}: {e}"
            free = 0
        else:
            why = f"{args.files_dir} has {free / 1e9:.0f} GB free; the BGZF cohort needs ~{args.samples * args.bins * 8e-9:.0f} GB"
        if os.path.exists(marker):
            os.remove(marker)
        need = args.samples * args.bins * 8 + (20 << 30)
        if free < need and not os.path.isdir(os.path.join(data, "mosdepth")):
            res = {"skipped": why}
        else:
            note("from files: generating the BGZF cohort (outside the clock)")
            try:
                res = prepare_files_cohort(data, out, args.samples, args.bins, gen_threads=16,
                                           threads=args.files_threads, note=note)
            except (OSError, subprocess.CalledProcessError) as e:
                res = {"skipped": f"cohort generation: {e}"}
        if world > 1:
            os.makedirs(data, exist_ok=True)
            with open(marker + ".tmp", "w") as f:
                f.write(token + "\n" + json.dumps(res if isinstance(res, dict) else list(res)))
            os.replace(marker + ".tmp", marker)
        return res
    t0 = time.time()
    while time.time() - t0 < args.files_timeout:
        try:
            with open(marker) as f:
                head, body = f.read().split("\n", 1)
            if head == token:
                res = json.loads(body)
                return res if isinstance(res, dict) else tuple(res)
        except (OSError, ValueError):
            pass
        time.sleep(0.5)
    return {"skipped": "timed out waiting for rank 0's cohort"}


def inflate_roofline(data, dev, note, max_bytes=4 << 30, reps=3):
    """The from-files headline's dominant kernel against HBM: k_inflate is
    ~2/3 of that step's GPU time (profiles/r06zp_bench_files_headline_kernel_stats.csv,
    the ingest ~70 % of its wall).  One pipelined ingest batch's worth of the
    cohort's BGZF files (<= 4 GB compressed, what a batch holds) is inflated
    in HBM by the ingest's own launch, grid_gunzip_batch (k_inflate, one wave
    per member, + k_member_check, each member's CRC and ISIZE; k_inflate ~96 %
    of it), timed with HIP events on the context's stream.  Algorithmic HBM
    bytes per launch = compressed bytes read + text written + text re-read by
    the check.  The kernel is issue-bound (one serial Huffman stream per wave,
    DESIGN round-6 item 5), so the HBM fraction is small by construction."""
    import glob
    import numpy as np
    from grid_amd import _abi
    names = sorted(glob.glob(os.path.join(data, "mosdepth", "*.regions.bed.gz")))
    blobs, tot = [], 0
    for f in names:
        sz = os.path.getsize(f)
        if blobs and tot + sz > max_bytes:
            break
        with open(f, "rb") as fh:
            blobs.append(fh.read())
        tot += sz
    io, il, oo, oc = [], [], [], []
    pos = opos = 0
    for b in blobs:
        ms, ml, mi = _abi.gz_members(b)
        cum = np.zeros(len(mi), np.int64)
        np.cumsum(mi[:-1], out=cum[1:])
        io.append(pos + ms)
        il.append(ml)
        oo.append(opos + cum)
        oc.append(mi.astype(np.int64))
        pos += -(-len(b) // 256) * 256
        opos += -(-int(mi.sum()) // 256) * 256
    io, il, oo, oc = (np.concatenate(x).astype(np.int64) for x in (io, il, oo, oc))
    src = np.zeros(pos + 256, np.uint8)
    p = 0
    for b in blobs:
        src[p:p + len(b)] = np.frombuffer(b, np.uint8)
        p += -(-len(b) // 256) * 256
    del blobs
    d_src = dev.upload(src)
    del src
    d = [dev.upload(x) for x in (io, il, oo, oc)]
    nu = len(io)
    out = dev.alloc(opos + 256, np.uint8)
    mem = dev.alloc(nu * _abi.GZ_MEMBER_BYTES, np.uint8)
    st_d, ln_d, nm_d = dev.alloc(nu, np.int32), dev.alloc(nu, np.int64), dev.alloc(nu, np.int32)
    ms_l = []
    for rep in range(reps + 1):                   # the first launch untimed
        dev.record(0)
        _abi.call("grid_gunzip_batch", dev.ctx, d_src.ptr, d[0].ptr, d[1].ptr, nu, out.ptr, d[2].ptr, d[3].ptr,
                  mem.ptr, 1, st_d.ptr, ln_d.ptr, nm_d.ptr)
        dev.record(1)
        t = dev.elapsed_ms(0, 1)
        if rep:
            ms_l.append(t)
    ust, uln = st_d.numpy(), ln_d.numpy()
    if not (ust == 0).all():
        raise RuntimeError(f"inflate leg: member statuses {np.unique(ust, return_counts=True)}")
    text = int(uln.sum())
    if text != int(oc.sum()):
        raise RuntimeError("inflate leg: text length differs from the members' ISIZEs")
    comp = int(il.sum())
    ms = float(np.mean(ms_l))
    alg = comp + 2 * text
    peak = 8000.0
    ach = alg / (ms * 1e-3) / 1e9
    note(f"inflate leg: {len(io)} members, {comp / 1e9:.2f} GB -> {text / 1e9:.2f} GB text in {ms:.1f} ms")
    return {"kernel": "grid_gunzip_batch (k_inflate + k_member_check, the ingest's launch)", "bound": "hbm",
            "achieved": ach, "peak": peak, "unit": "GB/s", "frac": ach / peak, "traffic": None,
            "algorithmic_bytes_per_launch": alg, "bytes_def": "compressed read + text written + text re-read (CRC)",
            "compressed_bytes": comp, "text_bytes": text, "members": int(nu), "launch_ms": ms,
            "launch_ms_each": ms_l, "text_gbs": text / (ms * 1e-3) / 1e9,
            "note": "issue-bound (one serial Huffman stream per wave, 8 waves per SIMD): the HBM fraction is small "
                    "by construction; the line's `roofline` is the device chain's Gram"}


def files_leg(args, prep, steps, warmup, world, rank, dist, note):
    """The headline: ``steps`` timed runs of run_wgs_pipeline (the drop-in
    `grid wgs`, steps 4-7 from the mosdepth files to every output file) after
    ``warmup`` untimed ones, every rank (the distributed drop-in at N > 1),
    bracketed by a barrier and a device synchronisation on both sides; the
    max over ranks.  The ingest buffers stay cached from run to run
    (keep_buffers: a service's steady state), so no run pays their release.
    Per-step wall times of the four step functions (and, at one rank, the
    ingest / text write inside step 4) are averaged over the timed runs."""
    import functools
    import torch
    from grid_amd import pipeline
    from grid_amd.utils import compute_dipcn as cd
    from grid_amd.utils import find_neighbors as fn
    from grid_amd.utils import hi_inference as hi
    from grid_amd.utils import normalize_mosdepth as nm
    cfg_path, gen_s, nbytes = prep
    phases = {}
    wrapped = []

    def timed(mod, name, key):
        fun = getattr(mod, name)

        @functools.wraps(fun)
        def wrap(*a, **kw):
            t = time.perf_counter()
            try:
                return fun(*a, **kw)
            finally:
                phases[key] = phases.get(key, 0.0) + time.perf_counter() - t
        setattr(mod, name, wrap)
        wrapped.append((mod, name, fun))

    timed(nm, "normalize_mosdepth", "step4_total")
    timed(fn, "find_neighbors", "step5_total")
    timed(cd, "compute_diploid_genotypes", "step6_total")
    timed(hi, "hi_inference", "step7_total")
    if world == 1:
        timed(nm, "ingest", "step4_ingest")
        timed(nm, "_write_normalized_q", "step4_write_text")
    else:
        from grid_amd.utils import dist_step4
    try:
        for w_ in range(warmup):
            pipeline.run_wgs_pipeline(console=None, config=cfg_path, keep_buffers=True)
            note(f"from files: warmup {w_} done")
        phases.clear()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s_ in range(steps):
            pipeline.run_wgs_pipeline(console=None, config=cfg_path, keep_buffers=True)
            if world > 1:                  # this rank's phases of the distributed step 4 (dist_step4.py)
                for k, v in dist_step4.LAST_PHASES.items():
                    phases["step4_rank_" + k] = phases.get("step4_rank_" + k, 0.0) + v
            note(f"from files: step {s_} done")
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
    finally:
        for mod, name, fun in wrapped:
            setattr(mod, name, fun)
    el = torch.tensor([t1 - t0], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    data, out = files_paths(args)
    outputs = {f: os.path.getsize(os.path.join(out, f)) for f in sorted(os.listdir(out))} if rank == 0 else None
    digests = None
    if rank == 0:
        try:
            import xxhash
            import gzip
            digests = {}
            for f in sorted(os.listdir(out)):
                pth = os.path.join(out, f)
                if f.startswith("normalized"):
                    continue                 # 16 GB: its size above (its bytes differ with N: per-rank codes)
                h = xxhash.xxh3_64()
                with (gzip.open(pth, "rb") if f.endswith(".gz") else open(pth, "rb")) as fh:
                    h.update(fh.read())
                digests[f] = h.hexdigest()
        except ImportError:
            pass
    stages = {k: round(v / steps, 4) for k, v in sorted(phases.items())}
    stage_sum = sum(v for k, v in stages.items() if k.endswith("_total"))
    return {
        "value": args.samples * steps / elapsed, "ms_per_step": 1000.0 * elapsed / steps, "elapsed": elapsed,
        "stages_s": stages, "stages_total_s": round(stage_sum, 4),
        "stages_vs_step": round(stage_sum / (elapsed / steps), 4),
        "cohort_generation_s": round(gen_s, 1), "cohort_bytes": nbytes, "outputs_bytes": outputs,
        "outputs_xxh3_64_text": digests, "threads": args.files_threads,
    }


def cpu_sweep_fit():
    """The committed CPU-baseline sweep (tools/cpu_sweep.py: the oracle from
    files at N in {100, 400, 1600} x M in {30k, 100k}, one single-threaded
    process per point) and its per-stage fits extrapolated to configs 2 and 3
    -- measured offline on a GPU box's host cores, not in this run."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), CPU_SWEEP_JSON)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    return {"source": CPU_SWEEP_JSON, "cores_per_point": d["cores_per_point"], "host_cpus": d.get("host_cpus"),
            "points": [{"samples": p["n"], "bins": p["m"], "total_s": round(p["total_s"], 2),
                        "stages_s": {k: round(v, 3) for k, v in p["stages_s"].items()}} for p in d["points"]],
            "fit_seconds_per_unit": d["fit_seconds_per_unit"], "fit_units": d["fit_units"],
            "fit_check": d["fit_check"],
            "config2_samples_per_s": d["extrapolated"]["config2_3202x3M"]["samples_per_s"],
            "config3_samples_per_s": d["extrapolated"]["config3_50kx3M"]["samples_per_s"],
            "config2_total_s": d["extrapolated"]["config2_3202x3M"]["total_s"],
            "kind": "port", "note": "oracle/pipeline.py from mosdepth files to output files (the reference's step "
                                    "functions restated), fitted per stage and extrapolated: the reference's fp64 "
                                    "matrix does not fit host memory at configs 2-3"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(gpus):
    """One rank per GPU: torch.distributed.run as a CHILD process (this
    process has not touched the GPU), exit with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def plan_memory(n, ml, world, budget, shard="bin", piece_bytes=0):
    """Resident (one chunk) when the whole shard fits the HBM budget, else the
    widest 8192-multiple chunk that does.  Returns (chunk or None, bytes)."""
    np_ = -(-max(n, 1) // 256) * 256
    if shard == "cohort" and world > 1:
        # no whole Gram: the two row segments (B (2W+1) B int64, B a multiple
        # of 256) and two panel-piece buffers (fused.Steps47, split="cohort")
        B = -(-(-(-np_ // (2 * world))) // 256) * 256
        fixed = B * (2 * world + 1) * B * 8 + 2 * piece_bytes
    else:
        # Gram + (multi-GPU) the segment send / receive buffers: (2W+1)/(4W) and
        # 1/W of that of np^2 int64 (fused.Steps47._step5_segments)
        seg = (2 * world + 1) / (4.0 * world) * (1 + 1.0 / world) if world > 1 else 0.0
        fixed = np_ * np_ * 8 * (1 + seg)
    fixed += n * (-(-ml // 8192)) * 24 + ml * 64
    per_col_resident = n * 4 + n * 2 + np_ * 2            # q int32 + z int16 + bf16 panel
    if fixed + per_col_resident * ml <= budget:
        return None, fixed + per_col_resident * ml
    per_col = n * 4 + n * 2 + np_ * 2                     # chunk buffers: q, z, panel
    chunk = int((budget - fixed) // per_col) // 8192 * 8192
    if chunk < 8192:
        raise SystemExit(f"bench: {n} samples do not fit the HBM budget ({budget / 1e9:.0f} GB)")
    return min(chunk, -(-ml // 8192) * 8192), fixed + per_col * chunk


def run_workload(args, n, m, steps, warmup, world, rank, local, dist, comm, dev, note, profile_pass=True):
    """One workload's timed steps (steps 4-7 of an n x m cohort over `world`
    ranks): the bench line's fields for it.  With --sim-world W the process
    is rank --sim-rank of a simulated W-rank run on one GPU (fused.SimComm):
    `world` / `rank` are then the simulated ones, the clock this process's."""
    import torch

    from grid_amd import _abi
    from grid_amd.fused import Depth16, HipOps, Steps47, SynthSource, TorchAlloc, shard_range

    c0, c1 = shard_range(m, rank, world)
    ml = c1 - c0
    talloc = TorchAlloc(local)
    ops = HipOps(dev)
    piece_bytes = int(args.piece_mb * 2 ** 20)
    if args.chunk and (n, m) == (args.samples, args.bins):
        chunk, _ = args.chunk, None
    else:
        chunk, _ = plan_memory(n, ml, world, args.hbm_budget_gb * 1e9, args.shard, piece_bytes)
    streamed = chunk is not None and chunk < ml
    depth_format = args.depth_format
    if depth_format == "auto":
        depth_format = "int32" if streamed else "q16"
    if streamed:
        if depth_format != "int32":
            raise SystemExit("bench: the compact depth form is resident-only")
        q, ldq = SynthSource(ops, SEED, n, c0, NCL), None
    elif depth_format == "q16":
        # compact depth matrix: uint16 hundredths + escape table (half the HBM
        # bytes of the four step-4 passes; same int32 values after decoding)
        q = Depth16.synth(talloc, dev.ctx, SEED, n, ml, c0, NCL)
        ldq = q.ld
    else:
        q = torch.empty((n, max(ml, 1)), dtype=torch.int32, device="cuda")
        _abi.call("grid_synth_depth", dev.ctx, SEED, n, ml, ml, c0, NCL, q.data_ptr())
        ldq = ml
    reads, off, nbr, w = synth_reads_and_ibs(n)
    # step 7 on its own stream, deferred behind the next pass's Gram (fused.py
    # Steps47): it overlaps that pass's top-k/dipCN and the next statistics;
    # every pass's phasing still completes inside the timed region (finish()
    # before the final synchronize)
    # two lanes, one per dipCN buffer: the last two passes' phasings (the
    # deferred one and finish()'s) overlap instead of queueing at the end
    lane = None
    col_lane = None
    if not args.no_overlap:
        # --cu-mask (A/B only): the phasing workgroup on a stream masked to ONE
        # CU and the column passes on a stream masked to all the others, so they
        # never share a CU.  Measured slower (r06e: 13.98 against 8.67 ms per
        # rank; every pass on the masked streams ran 1.5-1.6x longer), so the
        # lanes are ordinary streams by default
        ncu = _abi.device_cu_count(dev)
        cu_mask = args.cu_mask and ncu > 8
        lane = []
        for li in range(2):
            pdev = _abi.Device(local)
            if cu_mask:
                pdev.own_stream_cumask([ncu - 1 - li], ncu)
                pstream = torch.cuda.ExternalStream(pdev.stream_handle())
            else:
                pstream = torch.cuda.Stream()
                pdev.set_stream(pstream)
            lane.append((HipOps(pdev), pstream))
        if cu_mask:
            cdev = _abi.Device(local)
            cdev.own_stream_cumask(range(ncu - 2), ncu)
            col_lane = (HipOps(cdev), torch.cuda.ExternalStream(cdev.stream_handle()))
    st = Steps47(ops, talloc, n, m, c0, ml, k=args.k, n_nbr=300, top_frac=0.1, zmax=2.0, sigma2_max=1000.0,
                 frac_r=1.0, min_nbr=1, n_iters=args.n_iters, comm=comm, phase_lane=lane,
                 chunk=chunk if streamed else None, keep_z=not streamed, split=args.shard, piece_bytes=piece_bytes,
                 col_lane=col_lane)
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)

    note(f"{n} x {m}, shard {ml} bins, {st.nch} chunk(s); warmup {warmup}, steps {steps}")
    for w_ in range(warmup):
        st.run(q, ldq)
        st.finish()
        torch.cuda.synchronize()
        note(f"warmup {w_} done")
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gms, glaunch = 0.0, 0
    gram_pairs = []
    if hasattr(comm, "bytes_in"):
        comm.bytes_in.clear()
    for s in range(steps):
        st.run(q, ldq, time_gram=True)
        gram_pairs += st.gram_evs
        if st.nch > 1:                          # long streamed steps: progress for the watchdog
            note(f"step {s} queued")
    st.finish()                                 # the last step's (deferred) phasing, inside the clock
    torch.cuda.synchronize()
    note("timed steps done")
    sim_bytes = dict(comm.bytes_in) if hasattr(comm, "bytes_in") else None     # the timed steps' only
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    gms = sum(a.elapsed_time(b) for a, b in gram_pairs) / max(steps, 1)      # Gram ms per step
    glaunch = len(gram_pairs) // max(steps, 1)
    stages = None
    if profile_pass:
        st.run(q, ldq, profile=True)          # untimed pass: per-stage device times
        torch.cuda.synchronize()
        stages = {k: round(v, 3) for k, v in st.stage_ms().items()}

    valid = int(st.valid[:n].sum().item())
    traffic, tsrc = None, None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), args.traffic_json)
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        shape_ok = tj.get("bench", {}).get("samples", 3202) == n and tj.get("bench", {}).get("bins", 3_000_000) == m
        hits = [v for kk, v in tj["kernels"].items() if kk.startswith(GRAM_KERNEL)]
        if hits and shape_ok and world == 1 and not streamed:
            traffic, tsrc = hits[0]["traffic_bytes"], args.traffic_json
    ruse = st.ruse_loc
    cohort = st.split == "cohort"
    if cohort:
        # this rank's share of 2 N^2 R_use over all ranks' columns, and the
        # MFMA work its segment launches executed (fused.Steps47._gram_piece)
        flops = 2.0 * n * n * st.ruse_tot / world
        executed = st.exec_flops
    else:
        flops = 2.0 * n * n * ruse                      # 2 N^2 R_use per step (this rank)
        nt, ni = st.np_ // 128, st.np_ // 256           # k_gram8: 256x128 tiles (I, j >= 2I)
        ntiles = sum(nt - 2 * i for i in range(ni))
        executed = 2.0 * ntiles * 256 * 128 * sum(-(-u // 64) * 64 for u in st.chunk_used)
    gsec = gms * 1e-3
    streamed_note = (f", bin-streamed in {st.nch} chunks of {chunk} bins regenerated on the device every pass "
                     f"(inside the timed region), step-4 output written per chunk") if streamed else ""
    cfgname = {(3202, 3_000_000): "BASELINE config 2", (50_000, 3_000_000): "BASELINE config 3 shape",
               (50_000, 30_000_000): "BASELINE config 4 shape"}.get((n, m), "custom")
    out = {
        "metric": METRIC,
        "value": n * steps / elapsed,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": 1000.0 * elapsed / steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64 (statistics) + bf16-MFMA exact-integer (k-NN)",
        "data": "synthetic (counter-based cohort generated in HBM; 26 ancestry clusters)",
        "config": {"workload": f"{cfgname}: {n} samples x {m} bins, k={args.k}, n_iters={args.n_iters}, "
                               f"{world} GPU(s){streamed_note}",
                   "samples": n, "bins": m, "k": args.k, "n_iters": args.n_iters,
                   "parallelism": (f"{args.shard}-sharded x{world}" + (f" (rank {rank} of a simulated {world}-rank run "
                                   f"on one GPU)" if args.sim_world else "")), "shard": args.shard,
                   "depth_format": depth_format,
                   "streamed": streamed, "chunk_bins": chunk if streamed else None, "chunks": st.nch,
                   "selected_regions": st.r_loc if world == 1 else None, "R_use_rank0": ruse,
                   "dipcn_valid": valid, "phasing_levels": st.nlev},
        "stages_ms": stages,
        "roofline": {"kernel": "k_gram8 (exact bf16-MFMA Gram)", "bound": "mfma",
                     "achieved": flops / gsec / 1e12, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": flops / gsec / 1e12 / PEAK_BF16_TFLOPS,
                     "traffic": traffic, "traffic_source": tsrc,
                     "hbm_gbs": traffic * glaunch / gsec / 1e9 if traffic else None,
                     "hbm_frac": traffic * glaunch / gsec / 1e9 / PEAK_HBM_GBS if traffic else None,
                     "gram_ms": gms, "gram_launches_per_step": glaunch,
                     "executed_mfma_tflops": executed / gsec / 1e12,
                     "executed_frac": executed / gsec / 1e12 / PEAK_BF16_TFLOPS,
                     "flops_def": ("2*N^2*R_use per step on this rank (SURVEY 8d), over the summed HIP-event time "
                                   "of its Gram launches; executed = the 256x128 upper-triangle tiles k_gram8 "
                                   "computes (the symmetric half is not executed)") if not cohort else
                                  ("cohort split: this rank's 1/W share of 2*N^2*R_use (all ranks' columns) over the "
                                   "summed HIP-event time of its segment Gram launches (grid_knn_gram_kb_rows, one "
                                   "pair per gathered panel piece); executed = the segment tiles it computes")},
    }
    if sim_bytes is not None:
        # simulated rank: what the real collectives would bring into this rank per step
        out["sim_collective_bytes_in_per_step"] = {k: v / steps for k, v in sim_bytes.items()}
    timing = {"stages": stages, "elapsed": elapsed}
    # release the workload's device memory before another one
    del st, q
    if lane is not None:
        del lane
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out, timing


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--samples", type=int, default=3202)
    ap.add_argument("--bins", type=int, default=3_000_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-iters", type=int, default=100)
    ap.add_argument("--chunk", type=int, default=0, help="bins per streamed chunk (multiple of 8192); "
                    "0 = resident when the shard fits, else the widest chunk that fits")
    ap.add_argument("--hbm-budget-gb", type=float, default=200.0)
    ap.add_argument("--cpu-samples", type=int, default=4096)
    ap.add_argument("--cpu-bins", type=int, default=16384)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--files-baseline", action="store_true",
                    help="also time the oracle from files at config 1 (~30 s of host time; the committed sweep is "
                         "reported either way)")
    ap.add_argument("--no-files-baseline", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-overlap", action="store_true", help="run step 7 inline on the main stream")
    ap.add_argument("--cu-mask", action="store_true",
                    help="A/B: phase lanes on streams masked to one CU each, the column passes on a stream masked to "
                         "the others (hipExtStreamCreateWithCUMask; measured SLOWER, r06e: 13.98 vs 8.67 ms per rank)")
    ap.add_argument("--no-cu-mask", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--headline", choices=["auto", "files", "chain"], default="auto",
                    help="the line's value: files = K whole `grid wgs` runs from the mosdepth files (the default at "
                         "BASELINE config 2), chain = K passes of the device chain over a cohort generated in HBM")
    ap.add_argument("--no-files-config2", action="store_true", help="= --headline chain")
    ap.add_argument("--keep-files", action="store_true", help="keep the generated cohort and outputs afterwards")
    ap.add_argument("--files-dir", default="/dev/shm")
    ap.add_argument("--files-threads", type=int, default=16)
    ap.add_argument("--files-timeout", type=float, default=360.0)
    ap.add_argument("--config3-steps", type=int, default=1,
                    help="N=1: timed steps of the BASELINE config-3 shape (50k x 3M, streamed) reported beside the "
                         "line as config3_1gpu (0 = skip)")
    ap.add_argument("--config3-warmup", type=int, default=1)
    ap.add_argument("--traffic-json", default=TRAFFIC_JSON,
                    help="rocprofv3 PMC summary (tools/pmc_traffic.py) of this same command, for roofline.traffic")
    ap.add_argument("--shard", choices=["bin", "cohort"], default="bin",
                    help="multi-rank split of step 5's all-pairs Gram: bin = every rank sums the whole upper triangle "
                         "over its bins, one reduce-scatter of int64 segments; cohort = the Gram's rows sharded, the "
                         "quantised panel all-gathered in pieces overlapped with the segment Gram (step 4 stays "
                         "bin-sharded either way)")
    ap.add_argument("--piece-mb", type=float, default=2048.0,
                    help="cohort split: bytes of one gathered panel piece (all ranks), two buffers")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="per-rank timing on ONE GPU: run rank --sim-rank of a simulated W-rank job (fused.SimComm: "
                         "collectives do their local copies only; xGMI time not included)")
    ap.add_argument("--sim-rank", type=int, default=0)
    ap.add_argument("--depth-format", choices=["auto", "int32", "q16"], default="auto",
                    help="depth matrix in HBM: the compact uint16 hundredths + escape table (q16: half the bytes of "
                         "the step-4 passes, same int32 values after decoding) or int32 hundredths; auto = q16 when "
                         "the shard is resident, int32 chunks when it is streamed")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    # ONE JSON line on stdout: whatever libraries write to fd 1 (RCCL prints
    # its version banner there at communicator init, once per rank) goes to
    # stderr; the result line is written to a saved copy of the real stdout
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    def note(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    n, m = args.samples, args.bins
    headline = args.headline
    if args.no_files_config2 or args.sim_world:
        headline = "chain"
    if headline == "auto":
        headline = "files" if (n, m) == (3202, 3_000_000) else "chain"
    # the from-files cohort is written before anything touches the GPU (a child process)
    prep = files_prepare(args, rank, local, world, note) if headline == "files" else None

    import torch
    # GRID_BENCH_SHARE_GPU=1 (rehearsal only): ranks share the visible GPUs
    # round-robin, with GRID_DIST_BACKEND=gloo since RCCL needs one GPU per rank
    if os.environ.get("GRID_BENCH_SHARE_GPU") == "1":
        local = local % torch.cuda.device_count()
        os.environ["GRID_SHARE_GPU"] = "1"          # the drop-in's get_device likewise
    torch.cuda.set_device(local)
    dist = None
    comm = None
    # GRID_BENCH_FORCE_DIST=1: the torch.distributed path (RCCL collectives,
    # TorchComm) even at world 1 -- a one-GPU check of the multi-GPU code path
    if world > 1 or os.environ.get("GRID_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist
        backend = os.environ.get("GRID_DIST_BACKEND", "nccl")     # "nccl" = RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        from grid_amd.fused import TorchComm
        comm = TorchComm(dist)

    from grid_amd import _abi

    if args.sim_world:
        dev = _abi.Device(local)
        dev.set_stream(torch.cuda.current_stream())
        if world != 1 or not 0 <= args.sim_rank < args.sim_world:
            raise SystemExit("bench: --sim-world runs one process (no --gpus) with 0 <= --sim-rank < --sim-world")
        from grid_amd.fused import SimComm
        comm = SimComm(args.sim_world, args.sim_rank)
        out, timing = run_workload(args, n, m, args.steps, args.warmup, args.sim_world, args.sim_rank, local, None,
                                   comm, dev, note)
        out["n_gpus"] = 1
        out["value"] = None          # not a job throughput: one rank's work of a W-rank step
        out["rank_ms_per_step"] = out["ms_per_step"]
        out["build"] = _abi.build_info()
        print(json.dumps(out), file=result_out, flush=True)
        return

    # ---- the headline: `grid wgs` from files, K whole runs ----
    files = None
    if headline == "files":
        if isinstance(prep, dict):
            files = prep                                   # {"skipped": why}
            note(f"from files skipped: {prep['skipped']}")
        else:
            note(f"from files: {n} x {m}, {world} rank(s); warmup {args.warmup}, steps {args.steps}")
            files = files_leg(args, prep, args.steps, args.warmup, world, rank, dist, note)
        # the pipeline's device context holds its ingest buffers: free them for the chain below
        from grid_amd.device import release_ingest_buffers
        release_ingest_buffers()
        torch.cuda.empty_cache()

    # ---- the device chain (inputs generated in HBM): the Gram's roofline ----
    dev = _abi.Device(local)
    dev.set_stream(torch.cuda.current_stream())
    chain, timing = run_workload(args, n, m, args.steps, args.warmup, world, rank, local, dist, comm, dev, note)
    if files is not None and "value" in files:
        out = dict(chain)
        out["value"] = files["value"]
        out["ms_per_step"] = files["ms_per_step"]
        out["data"] = ("synthetic mosdepth BGZF cohort on disk (tools/gen_cohort: the bench's 26-cluster depth model "
                       "as '%.2f' text, 1 kb bins), generated before the clock")
        out["config"] = {
            "workload": (f"BASELINE config 2 FROM FILES: {n} mosdepth regions.bed.gz x {m} bins -> `grid wgs` steps "
                         f"4-7 (run_wgs_pipeline: device ingest, normalised gz file, neighbours, dipCN, haploid calls, "
                         f"every output written), k={args.k}, n_iters={args.n_iters}, {world} GPU(s)"
                         + (" (distributed drop-in: files sliced over the ranks, all-to-all to 8192-aligned column "
                            "shards, RCCL segment reduce-scatter, row-sharded writer)" if world > 1 else "")),
            "samples": n, "bins": m, "k": args.k, "n_iters": args.n_iters,
            "parallelism": f"files x{world} -> bins x{world} -> rows x{world}" if world > 1 else "1 GPU",
            "threads": args.files_threads, "step": "one whole run_wgs_pipeline call (ingest buffers kept cached between "
                                                  "runs; outputs rewritten every run)"}
        out["from_files"] = files
        dc = {k: chain[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup", "config", "stages_ms")}
        dc["data"] = chain["data"]
        dc["roofline"] = chain["roofline"]
        out["device_chain"] = dc
        out["roofline"] = dict(chain["roofline"], measured_in="device_chain (the same config-2 shape, inputs in HBM; "
                                                              "the metric's k-NN distance kernel)")
    else:
        out = chain
        if files is not None:
            out["from_files"] = files
    # the metric's own shape (BASELINE config 3: 50k x 3M, streamed on one
    # GPU): one more timed measurement in the same run, beside the line's
    # workload (N = 1 only: the scaling runs keep one workload per N)
    c3 = None
    if world == 1 and args.config3_steps > 0 and (n, m) != (50_000, 3_000_000):
        note("config 3 shape (50,000 x 3,000,000, streamed) as a second measurement")
        o3, _ = run_workload(args, 50_000, 3_000_000, args.config3_steps, args.config3_warmup, world, rank, local, dist,
                             comm, dev, note, profile_pass=False)
        c3 = {k: o3[k] for k in ("value", "unit", "steps", "warmup", "ms_per_step")}
        c3["config"] = o3["config"]
        c3["gram_ms"] = o3["roofline"]["gram_ms"]
        c3["gram_frac_2N2R"] = o3["roofline"]["frac"]
        c3["executed_frac"] = o3["roofline"]["executed_frac"]
        out["config3_1gpu"] = c3
    if rank == 0 and world == 1 and headline == "files" and files is not None and "value" in files:
        try:
            out["ingest_roofline"] = inflate_roofline(files_paths(args)[0], dev, note)
        except Exception as e:                     # the line still prints; the reason is on it
            out["ingest_roofline"] = {"error": repr(e)[:300]}
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        c0 = 0
        ns, ms = min(args.cpu_samples, n), min(args.cpu_bins, m)
        qs = torch.empty((ns, ms), dtype=torch.int32, device="cuda")   # same cells, int32 form
        _abi.call("grid_synth_depth", dev.ctx, SEED, ns, ms, ms, c0, NCL, qs.data_ptr())
        qh = qs.cpu().numpy()
        del qs
        math = cpu_baseline(qh, n, m, args.k, args.n_iters)
        if c3 is not None:
            cb3 = scale_cpu_baseline(math["measured"], 50_000, 3_000_000)
            c3["cpu_baseline"] = {k: cb3[k] for k in ("value", "unit", "cores", "kind", "sample")}
            c3["speedup_vs_cpu_baseline"] = c3["value"] / cb3["value"]
        if headline == "files" or args.files_baseline:
            # the headline's own basis: the oracle file to
            # file, timed here on one core as the reference runs (threads=1),
            # scaled by stage complexity; the math slice is kept for the chain
            note("cpu baseline: the oracle from files at config 1")
            ffb = cpu_baseline_from_files(n, m, args.k, args.n_iters)
            ex = ffb["extrapolated"]
            out["cpu_baseline"] = {"value": ex["samples_per_s"], "unit": "samples/s", "cores": ffb["cores"],
                                   "kind": ffb["kind"],
                                   "sample": ffb["sample"] + f"; measured {ffb['config1_measured']['total_s']:.1f} s "
                                             f"at 100 x 30,000, scaled to {n} x {m}",
                                   "from_files": ffb, "device_chain_math_slice": math}
        else:
            out["cpu_baseline"] = math
        sweep = cpu_sweep_fit()
        if sweep is not None:
            out["cpu_baseline"]["sweep"] = sweep
    if rank == 0 and "cpu_baseline" in out:
        # which CPU number each ratio divides by (say it on the line)
        cb = out["cpu_baseline"]
        mcb = cb.get("device_chain_math_slice", cb)
        sp = {"device_chain_vs_math_slice": chain["value"] / mcb["value"],
              "basis_device_chain_vs_math_slice": "device_chain.value (inputs in HBM) / cpu_baseline.value (the "
                                                  "oracle's math on a bounded slice of the same cohort, scaled)"}
        sw, ff = cb.get("sweep"), out.get("from_files", {})
        if "from_files" in cb and ff.get("value"):
            sp["from_files_vs_cpu_baseline"] = ff["value"] / cb["value"]
            sp["basis_from_files_vs_cpu_baseline"] = (
                "value (grid wgs steps 4-7 from mosdepth files) / cpu_baseline.value (the oracle from files, measured "
                "at config 1 on this host, one core, scaled to config 2)")
        if sw and ff.get("value"):
            sp["from_files_vs_reference_from_files"] = ff["value"] / sw["config2_samples_per_s"]
            sp["basis_from_files_vs_reference_from_files"] = (
                "value (grid wgs steps 4-7 from mosdepth files, every output written) / "
                "cpu_baseline.sweep.config2_samples_per_s (the oracle from files, per-stage fits of the measured sweep "
                "extrapolated to config 2)")
        out["speedup_vs_cpu_baseline"] = sp
    if rank == 0:
        out["build"] = _abi.build_info()          # the library's source sha256 = this tree's (checked at load)
        print(json.dumps(out), file=result_out, flush=True)
    if dist:
        dist.barrier()
    if headline == "files" and rank == 0 and not args.keep_files:
        import shutil
        for d in files_paths(args):
            shutil.rmtree(d, ignore_errors=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
