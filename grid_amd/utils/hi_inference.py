"""Step 7 -- haplotype inference (IBS / IBD-constrained phasing), MI355X path.

Drop-in for grid/utils/hi_inference.py.  The file readers keep the
reference's parsing rules; the Gauss-Seidel proportional phasing
(_run_phasing :175-226) and the imputation (_compute_imp :229-250) run on the
GPU (grid_amd/csrc/dipcn_phase.hip).  The in-place sweep is executed as a
level schedule computed from the neighbour graph (grid_hi_levels): samples
in one level read, then write, and the result is bit-identical to the
sequential in-place order.
"""
from __future__ import annotations

import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

from .. import _abi, engine
from ..device import get_device
from .utils import log, open_maybe_gz


def _read_dip_cn_file(dip_cn_file):
    """:10-31"""
    ids, irrs, idx = [], [], {}
    with open_maybe_gz(dip_cn_file) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            parts = line.split()
            if len(parts) < 2:
                continue
            try:
                v = float(parts[1])
            except ValueError:
                continue
            idx[parts[0]] = len(irrs)
            ids.append(parts[0])
            irrs.append(v)
    return ids, irrs, idx


def _ids_in_order(IDtoInd):
    """The sample IDs by index, or None when the mapping is not 0..N-1 (the
    native loaders need it to be; duplicates in the dipCN file break it)."""
    ids = [None] * len(IDtoInd)
    for k, v in IDtoInd.items():
        if not (isinstance(v, int) and 0 <= v < len(ids)) or ids[v] is not None:
            return None
        ids[v] = k
    return ids


def _native_csr(loader, *args):
    """Run a native loader; None when it declines (GRID_EUNSUPPORTED)."""
    try:
        return loader(*args)
    except _abi.GridNativeError as e:
        if e.code != _abi.GRID_EUNSUPPORTED:
            raise
        return None


def _csr_to_lists(off, nbr, w):
    return [[(int(nbr[t]), float(w[t])) for t in range(off[h], off[h + 1])] for h in range(len(off) - 1)]


def _load_ibs_csr(neighbors_file, IDtoInd, MAX_NBR):
    """(off, nbr, w) of _load_ibs_neighbors: host C++ parser, Python restatement
    for inputs it declines."""
    ids = _ids_in_order(IDtoInd)
    if ids is not None and isinstance(MAX_NBR, int) and -(1 << 62) < MAX_NBR < (1 << 62):
        r = _native_csr(_abi.load_ibs, neighbors_file, ids, MAX_NBR)
        if r is not None:
            return r
    return engine.csr_from_lists(_load_ibs_neighbors_py(neighbors_file, IDtoInd, MAX_NBR))


def _load_ibd_csr(ilash_file, IDtoInd, MAX_NBR, region_start, region_end, min_length=0.5, min_match=0.70,
                  weighted=False, weight_scale=1_000_000):
    """(off, nbr, w) of _load_ibd_neighbors (see _load_ibs_csr)."""
    ids = _ids_in_order(IDtoInd)
    num = (int, float)
    lim = 1 << 62   # region bounds the native int64 arithmetic takes exactly
    ok = (ids is not None and isinstance(MAX_NBR, int) and MAX_NBR >= 0 and isinstance(min_length, num)
          and isinstance(min_match, num) and isinstance(weight_scale, num)
          and (not weighted or (isinstance(region_start, int) and isinstance(region_end, int)
                                and abs(region_start) < lim and abs(region_end) < lim)))
    if ok:
        r = _native_csr(_abi.load_ibd, ilash_file, ids, MAX_NBR, region_start, region_end, min_length, min_match,
                        weighted, weight_scale)
        if r is not None:
            return r
    return engine.csr_from_lists(_load_ibd_neighbors_py(ilash_file, IDtoInd, MAX_NBR, region_start, region_end,
                                                        min_length, min_match, weighted, weight_scale))


def _load_ibs_neighbors(neighbors_file, IDtoInd, MAX_NBR):
    """:34-74 -> hap_nbrs lists (reference API; the step itself uses the CSR)."""
    return _csr_to_lists(*_load_ibs_csr(neighbors_file, IDtoInd, MAX_NBR))


def _load_ibd_neighbors(ilash_file, IDtoInd, MAX_NBR, region_start, region_end, min_length=0.5,
                        min_match=0.70, weighted=False, weight_scale=1_000_000):
    """:86-172 -> hap_nbrs lists (reference API; the step itself uses the CSR)."""
    return _csr_to_lists(*_load_ibd_csr(ilash_file, IDtoInd, MAX_NBR, region_start, region_end, min_length,
                                        min_match, weighted, weight_scale))


def _load_ibs_neighbors_py(neighbors_file, IDtoInd, MAX_NBR):
    """:34-74 (computeIBSpbwt: header + ID hap nbrInd cMlen cMedge IDnbr hapNbr)."""
    hap_nbrs = [[] for _ in range(2 * len(IDtoInd))]
    with open_maybe_gz(neighbors_file) as f:
        next(f)
        for line in f:
            line = line.strip()
            if not line:
                continue
            p = line.split()
            if len(p) < 7:
                continue
            try:
                hap, hap_nbr = int(p[1]), int(p[6])
            except ValueError:
                continue
            if hap not in (1, 2) or hap_nbr not in (1, 2):
                continue
            i, j = IDtoInd.get(p[0]), IDtoInd.get(p[5])
            if i is not None and j is not None:
                h = 2 * i + hap - 1
                if len(hap_nbrs[h]) < MAX_NBR:
                    hap_nbrs[h].append((2 * j + hap_nbr - 1, 1.0))
    return hap_nbrs


def _segment_distance(bp1, bp2, region_start, region_end):
    """:77-83"""
    if bp2 < region_start:
        return float(region_start - bp2)
    if bp1 > region_end:
        return float(bp1 - region_end)
    return 0.0


def _load_ibd_neighbors_py(ilash_file, IDtoInd, MAX_NBR, region_start, region_end, min_length=0.5,
                           min_match=0.70, weighted=False, weight_scale=1_000_000):
    """:86-172 (iLASH, 11 columns; symmetric; sorted by cM desc; optional
    Lorentzian distance x match weight)."""
    raw = defaultdict(list)
    with open_maybe_gz(ilash_file) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            p = line.split("\t")
            if len(p) < 11:
                p = line.split()
            if len(p) < 11:
                continue
            try:
                bp1, bp2 = int(p[5]), int(p[6])
                length, match = float(p[9]), float(p[10])
            except (ValueError, IndexError):
                continue
            if length < min_length or match < min_match:
                continue
            try:
                h1 = int(p[1].rsplit("_", 1)[-1])
                h2 = int(p[3].rsplit("_", 1)[-1])
            except ValueError:
                continue
            if h1 not in (0, 1) or h2 not in (0, 1):
                continue
            i, j = IDtoInd.get(p[0]), IDtoInd.get(p[2])
            if i is None or j is None:
                continue
            if weighted:
                w = (weight_scale / (_segment_distance(bp1, bp2, region_start, region_end) + weight_scale)) * match
            else:
                w = 1.0
            a, b = 2 * i + h1, 2 * j + h2
            raw[a].append((b, w, length))
            raw[b].append((a, w, length))
    hap_nbrs = [[] for _ in range(2 * len(IDtoInd))]
    for h, segs in raw.items():
        segs.sort(key=lambda x: -x[2])
        hap_nbrs[h] = [(nb, w) for nb, w, _ in segs[:MAX_NBR]]
    return hap_nbrs


def _run_phasing(IRRs, hap_nbrs, MIN_NBR, N_ITERS, console=None):
    """:175-226 on the GPU.  Returns (hap_IRRs list, mean_IRRs)."""
    hap, _, mean = _phase_device(IRRs, hap_nbrs, MIN_NBR, N_ITERS, console)
    return [float(x) for x in hap], mean


def _phase_device(IRRs, hap_nbrs, MIN_NBR, N_ITERS, console=None, dev=None):
    return _phase_device_csr(IRRs, *engine.csr_from_lists(hap_nbrs), MIN_NBR, N_ITERS, console, dev)


def _phase_device_csr(IRRs, off, nbr, w, MIN_NBR, N_ITERS, console=None, dev=None):
    n = len(IRRs)
    n_ph = sum(1 for i in range(n) if off[2 * i + 1] - off[2 * i] >= MIN_NBR
               and off[2 * i + 2] - off[2 * i + 1] >= MIN_NBR)
    log(console, f"Phasing {n_ph} samples with >={MIN_NBR} neighbors for both haps")
    if n_ph > 0:
        tot = sum(int(off[2 * i + 2] - off[2 * i]) for i in range(n)
                  if off[2 * i + 1] - off[2 * i] >= MIN_NBR and off[2 * i + 2] - off[2 * i + 1] >= MIN_NBR)
        log(console, f"Avg neighbors per hap: {tot / (2.0 * n_ph):.2f}")
    return engine.phase(dev or get_device(), np.asarray(IRRs, dtype=np.float64), off, nbr, w, MIN_NBR, N_ITERS)


def run_phasing_batch(IRRs_per_locus, hap_nbrs_per_locus, MIN_NBR, N_ITERS, dev=None, paired=False):
    """_run_phasing + _compute_imp (:175-250) for many loci (VNTR regions) in
    one GPU launch, one workgroup per locus (BASELINE config 5).  Equal, locus
    by locus, to calling the reference per region.  Returns a list of
    (hap_IRRs [2n], imp [2n], mean_IRRs)."""
    loci = []
    for irrs, hap_nbrs in zip(IRRs_per_locus, hap_nbrs_per_locus):
        off, nbr, w = engine.csr_from_lists(hap_nbrs)
        loci.append((np.asarray(irrs, dtype=np.float64), off, nbr, w))
    return engine.phase_batch(dev or get_device(), loci, MIN_NBR, N_ITERS, paired=paired)


def _compute_imp(i, hap_IRRs, hap_nbrs, mean_IRRs):
    """:229-250 (single-sample API; the step computes all samples on the GPU)."""
    import math
    ws, wv = [1e-9, 1e-9], [0.0, 0.0]
    for h in range(2):
        for nb, w in hap_nbrs[2 * i + h]:
            v = hap_IRRs[nb]
            if not math.isnan(v):
                ws[h] += w
                wv[h] += w * v
    i0, i1 = wv[0] / ws[0], wv[1] / ws[1]
    if ws[0] <= 1e-9:
        i0 = mean_IRRs / 2
    if ws[1] <= 1e-9:
        i1 = mean_IRRs / 2
    return i0, i1


def _write_haploid(output_file, IDs, IRRs, hap, imp):
    """The step-7 output table (:329-337)."""
    with open_maybe_gz(output_file, "wt") as fout:
        fout.write("ID\tIRRs\thap1phased\thap2phased\thap1imp\thap2imp\n")
        for i in range(len(IRRs)):
            fout.write(f"{IDs[i]}\t{IRRs[i]:.2f}\t{hap[2*i]:.2f}\t{hap[2*i+1]:.2f}\t"
                       f"{imp[2*i]:.2f}\t{imp[2*i+1]:.2f}\n")


# ---------------------------------------------------------------------------
# Multi-locus step (BASELINE config 5): the reference runs step 7 once per
# region config (chrom/start_bp/end_bp, :300-301).  A loci table such as
# files/734_possible_coding_vntr_regions.IBD2R_gt_0.25.uniq.txt lists the
# regions; every locus is the reference's single-locus step with that
# region's inputs, and all of a rank's loci are phased in ONE batched launch
# (grid_hi_phase_batch, one workgroup per locus).  Loci are dealt round-robin
# over the ranks of a torch.distributed job (no data-path collective: loci
# are independent); every rank writes its own loci's files.

LOCI_COLS = {"chrom": ("CHR", "CHROM", "#CHROM", "CHROMOSOME"),
             "start": ("BP_START_HG38", "BP_START", "START", "START_BP"),
             "end": ("BP_END_HG38", "BP_END", "END", "END_BP"),
             "gene": ("GENE", "NAME", "ID")}


def read_loci_file(path):
    """Loci table: a tab/space-separated header naming the chromosome, start,
    end and (optional) name columns (the 734-region file's CHR,
    BP_START_HG38, BP_END_HG38, GENE), one region per line.  Returns a list of
    dicts {chrom, start, end, gene, index}."""
    loci = []
    with open_maybe_gz(path) as f:
        header = None
        for line in f:
            line = line.rstrip("\r\n")
            if not line.strip():
                continue
            p = line.split("\t") if "\t" in line else line.split()
            if header is None:
                up = [c.strip().upper() for c in p]
                header = {}
                for key, names in LOCI_COLS.items():
                    for nm in names:
                        if nm in up:
                            header[key] = up.index(nm)
                            break
                missing = [k for k in ("chrom", "start", "end") if k not in header]
                if missing:
                    raise ValueError(f"loci file {path}: no column for {', '.join(missing)} in the header")
                continue
            try:
                rec = {"chrom": p[header["chrom"]].strip(), "start": int(p[header["start"]]),
                       "end": int(p[header["end"]])}
            except (IndexError, ValueError) as e:
                raise ValueError(f"loci file {path}: bad line {line!r}") from e
            rec["gene"] = p[header["gene"]].strip() if "gene" in header and header["gene"] < len(p) else \
                f"{rec['chrom']}_{rec['start']}_{rec['end']}"
            rec["index"] = len(loci)
            loci.append(rec)
    return loci


def _locus_path(template, locus, **kw):
    """A per-locus path: ``template`` with {chrom} {start} {end} {gene}
    {index} {locus} (and the step's own keys) substituted."""
    return Path(str(template).format(chrom=locus["chrom"], start=locus["start"], end=locus["end"],
                                     gene=locus["gene"], index=locus["index"],
                                     locus=f"{locus['chrom']}_{locus['start']}_{locus['end']}_{locus['gene']}", **kw))


def _rank_world(comm=None):
    if comm is not None:
        return comm.get_rank(), comm.get_world_size()
    # an initialised default process group means torch.distributed is already
    # imported; never import torch just to ask (seconds on a fresh host)
    dist = sys.modules.get("torch.distributed")
    if dist is not None and dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def hi_inference_loci(config, console, comm=None):
    """Step 7 over every region of ``compute_haploid_genotypes.loci_file``.

    Per-locus inputs and outputs are path templates ({chrom} {start} {end}
    {gene} {index} {locus}; {output_dir} {prefix} {dip_prefix} {type} too):
      * ``dip_cn_file`` (default ``{output_dir}/{dip_prefix}.{locus}.{type}``,
        {locus} = ``{chrom}_{start}_{end}_{gene}``: gene names repeat in the
        734-region table, regions do not),
      * ``ibs_output`` / ``ibd_output`` (a template, or one shared file).  The
        reference's IBD loader (hi_inference.py:86-172) does not filter
        segments by region or chromosome: every locus reads every segment of
        its file, and only ``weighted`` uses the locus' start/end (the
        Lorentzian weight of the segment's distance to the region).  One
        shared IBD file across loci on several chromosomes is therefore read
        genome-wide for each locus, as the reference would; a warning says so
        (use a {chrom} template for per-chromosome files),
      * ``loci_output`` (default ``{output_dir}/{prefix}.{locus}.{type}``).
    Each output file is what the reference's hi_inference writes for a
    config with that locus' chrom/start_bp/end_bp.  ``comm``: a
    torch.distributed-like object (get_rank/get_world_size); by default the
    initialised default process group, if any.  Returns the loci this rank
    phased (dicts with their output paths)."""
    try:
        hc = config.get("compute_haploid_genotypes", {})
        prefix = hc.get("output_file_prefix", "haploid_genotypes")
        ftype = config.get("output_file_type", "tsv")
        output_dir = config.get("output_dir", ".")
        dip_prefix = config["compute_diploid_genotypes"].get("output_file_prefix")
        method = hc.get("method", "ibs").lower()
        MIN_NBR = hc.get("min_neighbors", 1)
        MAX_NBR = hc.get("max_neighbors", 10)
        N_ITERS = hc.get("n_iters", 100)
        loci_file = hc["loci_file"]
        keys = dict(output_dir=output_dir, prefix=prefix, dip_prefix=dip_prefix, type=ftype)
        dip_t = hc.get("dip_cn_file", "{output_dir}/{dip_prefix}.{locus}.{type}")
        out_t = hc.get("loci_output", "{output_dir}/{prefix}.{locus}.{type}")
        if method not in ("ibs", "ibd"):
            raise ValueError(f"unknown method '{method}', must be 'ibs' or 'ibd'")
        nbr_t = hc.get("ibs_output" if method == "ibs" else "ibd_output")
        if not nbr_t:
            raise ValueError(f"{method}_output required for method='{method}'")
    except Exception as e:
        log(console, f"Config error: {e}", style="danger")
        return None

    loci = read_loci_file(loci_file)
    outs = [_locus_path(out_t, lc, **keys) for lc in loci]
    if len(set(outs)) != len(outs):
        log(console, "Config error: loci_output names collide (add {index} or {start} to the template)",
            style="danger")
        return None
    if method == "ibd" and "{" not in str(nbr_t) and len({lc["chrom"] for lc in loci}) > 1:
        log(console, f"ibd_output {nbr_t} is one file for loci on {len({lc['chrom'] for lc in loci})} "
            "chromosomes: every locus reads all of its segments (no region filter, as the reference)",
            style="warning")
    rank, world = _rank_world(comm)
    mine = [lc for lc in loci if lc["index"] % world == rank]
    log(console, f"Phasing {len(mine)} of {len(loci)} loci on rank {rank}/{world} ({method})")

    def load(lc):
        IDs, IRRs, IDtoInd = _read_dip_cn_file(_locus_path(dip_t, lc, **keys))
        src = _locus_path(nbr_t, lc, **keys)
        if method == "ibs":
            csr = _load_ibs_csr(src, IDtoInd, MAX_NBR)
        else:
            csr = _load_ibd_csr(src, IDtoInd, MAX_NBR, lc["start"], lc["end"],
                                min_length=hc.get("min_length", 0.5), min_match=hc.get("min_match", 0.70),
                                weighted=hc.get("weighted", False), weight_scale=hc.get("weight_scale", 1_000_000))
        return IDs, IRRs, csr

    # the loaders are host C++ that release the GIL: parse loci in parallel
    import os
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 1))) as ex:
        inputs = list(ex.map(load, mine))
    res = engine.phase_batch(get_device(config), [(np.asarray(irr, dtype=np.float64), *csr)
                                                   for _, irr, csr in inputs], MIN_NBR, N_ITERS)
    done = []
    for lc, (IDs, IRRs, _), (hap, imp, _mean) in zip(mine, inputs, res):
        out = outs[lc["index"]]
        out.parent.mkdir(parents=True, exist_ok=True)
        _write_haploid(out, IDs, IRRs, hap, imp)
        done.append(dict(lc, output=str(out), samples=len(IRRs)))
    log(console, f"Haploid genotypes of {len(done)} loci written (rank {rank})", style="success")
    return done


def hi_inference(config, console):
    """Step entry point (:253-339)."""
    try:
        hc = config.get("compute_haploid_genotypes", {})
        prefix = hc.get("output_file_prefix", "haploid_genotypes")
        ftype = config.get("output_file_type", "tsv")
        output_dir = config.get("output_dir", ".")
        output_file = Path(f"{output_dir}/{prefix}.{ftype}")
        dip_prefix = config["compute_diploid_genotypes"].get("output_file_prefix")
        dip_file = Path(f"{output_dir}/{dip_prefix}.{ftype}")
        method = hc.get("method", "ibs").lower()
        MIN_NBR = hc.get("min_neighbors", 1)
        MAX_NBR = hc.get("max_neighbors", 10)
        N_ITERS = hc.get("n_iters", 100)
    except Exception as e:
        log(console, f"Config error: {e}", style="danger")
        return

    from .dist_step4 import dist_comm, rank0_step
    comm = dist_comm()
    if comm is not None:                    # torch.distributed: rank 0 phases the locus, the others wait
        rank0_step(comm, lambda: _hi_inference_one(config, console, hc, output_file, dip_file, method, MIN_NBR,
                                                   MAX_NBR, N_ITERS))
        return
    _hi_inference_one(config, console, hc, output_file, dip_file, method, MIN_NBR, MAX_NBR, N_ITERS)


def _hi_inference_one(config, console, hc, output_file, dip_file, method, MIN_NBR, MAX_NBR, N_ITERS):
    IDs, IRRs, IDtoInd = _read_dip_cn_file(dip_file)
    N = len(IRRs)
    log(console, f"Read diploid IRR data for {N} samples", style="success")
    if method == "ibs":
        ibs = hc.get("ibs_output")
        if not ibs:
            log(console, "Config error: ibs_output required for method='ibs'", style="danger")
            return
        log(console, f"Loading IBS neighbors from {ibs}")
        csr = _load_ibs_csr(ibs, IDtoInd, MAX_NBR)
    elif method == "ibd":
        ibd = hc.get("ibd_output")
        if not ibd:
            log(console, "Config error: ibd_output required for method='ibd'", style="danger")
            return
        weighted = hc.get("weighted", False)
        log(console, f"Loading IBD neighbors from {ibd} (weighted={weighted})")
        csr = _load_ibd_csr(ibd, IDtoInd, MAX_NBR, config.get("start_bp"), config.get("end_bp"),
                            min_length=hc.get("min_length", 0.5), min_match=hc.get("min_match", 0.70),
                            weighted=weighted, weight_scale=hc.get("weight_scale", 1_000_000))
    else:
        log(console, f"Config error: unknown method '{method}', must be 'ibs' or 'ibd'", style="danger")
        return

    hap, imp, _ = _phase_device_csr(IRRs, *csr, MIN_NBR, N_ITERS, console, get_device(config))
    _write_haploid(output_file, IDs, IRRs, hap, imp)
    log(console, f"Haploid genotypes written to {output_file}", style="success")
