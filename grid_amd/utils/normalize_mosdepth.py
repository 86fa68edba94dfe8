"""Step 4 -- mosdepth depth normalisation, MI355X path.

Drop-in for grid/utils/normalize_mosdepth.py (same public names and
behaviour; file:line references are to that file).  Host code parses the
mosdepth ``*.regions.bed.gz`` files into an int32-hundredths matrix; the
statistics (row means, column mean/variance, variance ratios, median,
selection, z-scores and their exact ``%.2f`` quantisation) run as HIP kernels
in HBM (grid_amd/csrc/normalize.hip), bit-identical to the reference's NumPy.
"""
from __future__ import annotations

import gzip
import os
import sys
from collections import defaultdict
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

from .. import _abi, engine
from ..device import get_device, release_ingest_buffers, step4_done
from . import handoff, ingest_device
from .mosdepth import remove_intermediate_files
from .utils import get_samples, log, progress_bar, setup_output_file

GZ_LEVEL = 1   # the decompressed text is the contract; level 1 writes 8x faster than 6 for +24 % bytes


class UnsupportedDepth(ValueError):
    """A depth that is not an exact 2-decimal value (the int32 path needs it)."""


# ------------------------------------------------------------ file helpers --
def norm_chrom(chrom: str) -> str:
    """:210-215"""
    return chrom if chrom.startswith("chr") else f"chr{chrom}"


def map_mosdepth_files_to_samples(mosdepth_dir, samples) -> dict:
    """:148-174 -- sample id -> *.regions.bed.gz by underscore-prefix match."""
    wanted = set(samples)
    out = {}
    for f in Path(mosdepth_dir).glob("*.regions.bed.gz"):
        parts = f.name.split(".")[0].split("_")
        for i in range(len(parts), 0, -1):
            cand = "_".join(parts[:i])
            if cand in wanted:
                out[cand] = f
                break
    return out


def find_bed_gz_for_individual(individual_id: str, mosdepth_dir) -> Path:
    """:557-573 -- first glob match of *{id}*regions.bed.gz."""
    d = Path(mosdepth_dir)
    hits = list(d.glob(f"*{individual_id}*regions.bed.gz"))
    return hits[0] if hits else d / f"{individual_id}.regions.bed.gz"


def find_bed_gz_paths(individual_ids, mosdepth_dir) -> dict:
    """``find_bed_gz_for_individual`` for many IDs from ONE directory listing.

    The reference globs the directory once per sample (:569), which is
    quadratic: ~15 s of fnmatch for 3,202 files.  Path.glob of the
    single-component pattern "*{id}*regions.bed.gz" yields the scandir entries
    whose name matches, in scandir order; for an ID without glob
    metacharacters a name matches iff it ends with "regions.bed.gz" and the
    part before that contains the ID.  So each ID gets the first such name in
    the same scandir order (or the same non-existent default); an ID with
    "*", "?" or "[" takes the reference's own glob."""
    d = Path(mosdepth_dir)
    tail = "regions.bed.gz"
    ids = list(individual_ids)
    plain = {i for i in ids if i and not any(ch in i for ch in "*?[")}      # "" makes "**..." (glob raises)
    lens = sorted({len(i) for i in plain})
    first = {}
    try:
        with os.scandir(d) as it:
            names = [e.name for e in it]
    except OSError:
        names = []
    for name in names:
        if not name.endswith(tail):
            continue
        stem = name[: len(name) - len(tail)]
        for ln in lens:
            if ln > len(stem):
                break
            for a in range(len(stem) - ln + 1):
                sub = stem[a:a + ln]
                if sub in plain and sub not in first:
                    first[sub] = d / name
    return {i: first.get(i, d / f"{i}.regions.bed.gz") if i in plain else find_bed_gz_for_individual(i, d)
            for i in ids}


def load_repeat_mask(repeat_bed) -> dict:
    """:177-207 -- {chrN: set(kb)} with inclusive end kb."""
    excluded = defaultdict(set)
    with open(repeat_bed) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            parts = line.strip().split()
            if len(parts) < 3:
                continue
            try:
                s, e = int(parts[1]), int(parts[2])
            except ValueError:
                continue
            excluded[norm_chrom(parts[0])].update(range(s // 1000, e // 1000 + 1))
    return excluded


def _read_regions(path, chromosome, start, end, excluded) -> dict:
    """One pass over a regions.bed.gz with the reference's filters
    (:262-285 == :321-352): chrom by ``startswith`` (quirk Q2), window
    overlap, depth > 0, repeat-mask kb overlap.  Duplicate (start, end) keys
    keep the last value (quirk Q1).  Raises on malformed numbers (the
    reference then drops the whole sample)."""
    cm = norm_chrom(chromosome) if chromosome else None
    windowed = start is not None and end is not None
    rec = {}
    with gzip.open(path, "rt") as f:
        for line in f:
            if cm and not line.startswith(cm):
                continue
            fields = line.strip().split("\t")
            if len(fields) < 4:
                continue
            c = norm_chrom(fields[0])
            s, e, d = int(fields[1]), int(fields[2]), float(fields[3])
            if windowed:
                if not (d > 0 and e >= start and s <= end):
                    continue
            elif d <= 0:
                continue
            ex = excluded.get(c)
            if ex and not ex.isdisjoint(range(s // 1000, e // 1000 + 1)):
                continue
            rec[(s, e)] = d
    return rec


def compute_population_mean_depths(individuals, mosdepth_dir, chromosome, start, end, excluded,
                                   threads=1, console=None) -> dict:
    """:218-301.  Sums are accumulated in ``individuals`` order (the
    reference's order with threads=1; with threads>1 its order depends on
    thread timing, quirk Q4)."""
    per = _read_all(individuals, mosdepth_dir, chromosome, start, end, excluded, threads)
    sums, cnts = defaultdict(float), defaultdict(int)
    for ind in individuals:
        for r, d in per.get(ind, {}).items():
            sums[r] += d
            cnts[r] += 1
    return {r: sums[r] / cnts[r] for r in sums if cnts[r] > 0}


def process_one_individual(individual_id, mosdepth_dir, chromosome, start, end, valid_regions, excluded):
    """:304-357 -> (id, [(start, end, depth), ...])."""
    p = find_bed_gz_for_individual(individual_id, mosdepth_dir)
    if not p.exists():
        return individual_id, []
    try:
        rec = _read_regions(p, chromosome, start, end, excluded)
    except Exception:
        return individual_id, []
    return individual_id, [(s, e, d) for (s, e), d in rec.items() if (s, e) in valid_regions]


def filter_empty_samples(regions_to_extract, console=None):
    """:576-600"""
    out = {k: v for k, v in regions_to_extract.items() if len(v) > 0}
    removed = len(regions_to_extract) - len(out)
    if removed > 0:
        msg = f"Removed {removed} samples with 0 regions"
        log(console, msg, style="warning") if console else print(msg)
    return out


def build_matrix_from_regions(regions_to_extract, individuals_order=None):
    """:379-416 -> (individuals_order, float64 matrix with NaN)."""
    if individuals_order is None:
        individuals_order = sorted(regions_to_extract.keys())
    regions = sorted({(s, e) for ind in individuals_order for s, e, _ in regions_to_extract.get(ind, [])})
    col = {r: j for j, r in enumerate(regions)}
    row = {ind: i for i, ind in enumerate(individuals_order)}
    mat = np.full((len(individuals_order), len(regions)), np.nan)
    for ind, lst in regions_to_extract.items():
        i = row[ind]
        for s, e, d in lst:
            j = col.get((s, e))
            if j is not None:
                mat[i, j] = d
    return individuals_order, mat


# ------------------------------------------------------------- compute ----
def to_hundredths(mat: np.ndarray) -> np.ndarray:
    """float64 depths (NaN = missing) -> int32 hundredths, exactly or raise."""
    mat = np.asarray(mat, dtype=np.float64)
    nan = np.isnan(mat)
    safe = np.where(nan, 0.0, mat)
    if np.any(np.abs(safe) >= 2 ** 31 / 100 - 1):
        raise UnsupportedDepth("depth outside the int32 hundredths range")
    q = np.rint(safe * 100.0)
    if not np.array_equal(q / 100.0, safe):
        raise UnsupportedDepth("depths must be exact 2-decimal values (mosdepth %.2f output)")
    q = q.astype(np.int32)
    q[nan] = _abi.MISSING
    return q


def normalize_matrix(mat):
    """:419-476 on the GPU.  Returns (normalized_mat, variance_ratios,
    col_means, col_vars) exactly as the reference does."""
    q = to_hundredths(mat)
    n, m = q.shape
    dev = get_device()
    qd = dev.upload(q)
    st = engine.normalize_stats(dev, qd, n, m, m)
    z = dev.alloc((max(n, 1), max(m, 1)), np.float64)
    _abi.call("grid_norm_zfull", dev.ctx, qd.ptr, n, m, m, st.rowmean.ptr, st.mu.ptr, st.scale, z.ptr)
    zz = z.numpy()[:n, :m]
    ratio = st.ratio.numpy()[:m]
    ratios = {i: float(ratio[i]) for i in range(m) if not np.isnan(ratio[i])}
    return zz, ratios, st.mu.numpy()[:m], st.var.numpy()[:m]


def select_high_variance_regions(variance_ratios: dict, top_frac: float = 0.9) -> list:
    """:479-499 (keeps ratio > sorted[int(top_frac*n)])."""
    if not variance_ratios:
        return []
    srt = sorted(variance_ratios.values())
    thr = srt[int(top_frac * len(srt))]
    return [i for i, r in variance_ratios.items() if r > thr]


def _fmt3(v) -> str:
    return "NA" if np.isnan(v) else f"{v:.3f}"


def _header_lines(n, sel_means, sel_vars, ratio_mult=100.0):
    with np.errstate(invalid="ignore", divide="ignore"):
        sel_ratios = np.where(sel_means > 0, ratio_mult * sel_vars / sel_means, np.nan)
    r = len(sel_means)
    return (f"{n}\t{r}\t" + "\t".join(_fmt3(v) for v in sel_means) + "\n",
            f"{n}\t{r}\t" + "\t".join(_fmt3(v) for v in sel_ratios) + "\n")


def write_normalized_output(mat, individuals_order, selected_indices, output_file, col_means, col_vars,
                            individual_raw_means, ratio_mult: float = 100.0):
    """:502-554 (float z matrix API)."""
    sel = list(selected_indices)
    h0, h1 = _header_lines(len(individuals_order), np.asarray(col_means)[sel], np.asarray(col_vars)[sel],
                           ratio_mult)
    with gzip.open(output_file, "wt", compresslevel=GZ_LEVEL) as out:
        out.write(h0)
        out.write(h1)
        for i, ind in enumerate(individuals_order):
            vals = ["NA" if np.isnan(mat[i, j]) else f"{mat[i, j]:.2f}" for j in sel]
            out.write(f"{ind}\t{individual_raw_means[i]:.2f}\t" + "\t".join(vals) + "\n")


def _write_normalized_q(path, ids, raw, sel_means, sel_vars, zq, ratio_mult=100.0, dev=None):
    """Fast writer: z rows are exact integer hundredths.  ``zq`` on the device
    (a DevBuf [n][>= r], with ``dev``): the rows are formatted and Huffman-coded
    in HBM (grid_write_normalized_gz_dev) and only compressed bytes come back;
    a host array: threaded host C++ formatting + libdeflate
    (grid_write_normalized_gz).  Either way a multi-member gzip whose text is
    the reference's after gunzip."""
    sel_means = np.asarray(sel_means, dtype=np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        sel_ratios = np.where(sel_means > 0, ratio_mult * np.asarray(sel_vars, dtype=np.float64) / sel_means, np.nan)
    if isinstance(zq, _abi.DevBuf):
        n, r = len(ids), len(sel_means)
        _abi.write_normalized_gz_dev(dev, path, list(ids), np.asarray(raw, dtype=np.float64), sel_means, sel_ratios,
                                     zq, n, r, zq.shape[1] if len(zq.shape) == 2 else r, level=GZ_LEVEL)
        return
    _abi.write_normalized_gz(path, list(ids), np.asarray(raw, dtype=np.float64), sel_means, sel_ratios,
                             np.asarray(zq).reshape(len(ids), len(sel_means)), level=GZ_LEVEL)


# ---------------------------------------------------------------- ingest --
def _read_all(individuals, mosdepth_dir, chromosome, start, end, excluded, threads):
    where = find_bed_gz_paths(individuals, mosdepth_dir)

    def one(ind):
        p = where[ind]
        if not p.exists():
            return ind, None
        try:
            return ind, _read_regions(p, chromosome, start, end, excluded)
        except Exception:
            return ind, None

    with ThreadPoolExecutor(max_workers=max(1, int(threads or 1))) as ex:
        res = dict(ex.map(one, list(individuals)))
    return {k: v for k, v in res.items() if v is not None}


def ingest(individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth, max_depth, threads,
           console=None, dev=None):
    """R1-R4 (:218-416): mosdepth files -> (ids, regions, int32 hundredths).
    With a device (``dev``): inflated and parsed in HBM (ingest_device.py;
    the matrix is returned as a device buffer); the host C++ parser
    (``grid_ingest_*``, grid_amd/csrc/ingest.cpp) takes any cohort outside
    that path's common case, with one multithreaded parse per file; text that
    leaves the strict mosdepth grammar (or a non-integer window) goes through
    the line-by-line restatement ``ingest_py``."""
    ints = all(v is None or (isinstance(v, int) and not isinstance(v, bool)) for v in (start, end))
    if ints and dev is not None:
        try:
            return _ingest_dev(dev, individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth,
                               max_depth, threads, console)
        except ingest_device.DeviceIngestUnsupported as e:
            msg = f"device mosdepth parser: {e}; using the host parser"
            log(console, msg, style="warning") if console else print(msg)
            release_ingest_buffers(dev)        # the host parser and step 4 get the HBM back
        except _abi.GridNativeError as e:
            # e.g. the device buffers do not fit (a smaller GPU, ranks sharing
            # one): what the device path allocated and cached goes now
            msg = f"device mosdepth ingest failed ({e}); using the host parser"
            log(console, msg, style="warning") if console else print(msg)
            release_ingest_buffers(dev)
    if ints:
        try:
            return ingest_native(individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth,
                                 max_depth, threads, console)
        except _abi.IngestUnsupported as e:
            msg = f"native mosdepth parser: {e}; using the line-by-line parser"
            log(console, msg, style="warning") if console else print(msg)
    return ingest_py(individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth, max_depth,
                     threads, console)


def _ingest_dev(dev, individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth, max_depth, threads,
                console=None):
    """R1-R4 on the device (ingest_device.py); same (ids, regions, matrix) as
    ``ingest_native``, the matrix a device buffer."""
    import time
    t0 = time.perf_counter()
    inds = list(individuals)
    where = find_bed_gz_paths(inds, mosdepth_dir)
    paths = [str(where[ind]) if where[ind].exists() else None for ind in inds]
    window = (start, end) if start is not None and end is not None else None
    if ingest_device.TRACE:
        print(f"[ingest] paths in {time.perf_counter() - t0:.3f} s", file=sys.stderr, flush=True)
    rows, state, nval, status = ingest_device.ingest_device(
        dev, paths, norm_chrom(chromosome) if chromosome else None, window, excluded or {}, min_depth, max_depth,
        threads=max(1, int(threads or 1)))
    if ingest_device.TRACE:
        print(f"[ingest] device ingest returned at {time.perf_counter() - t0:.3f} s", file=sys.stderr, flush=True)
    keep = {ind: i for i, ind in enumerate(inds) if status[i] == 0 and state is not None and nval[i] > 0}
    removed = len(inds) - len(keep)
    if removed > 0:                           # filter_empty_samples (:576-600)
        msg = f"Removed {removed} samples with 0 regions"
        log(console, msg, style="warning") if console else print(msg)
    ids = sorted(keep)
    if not ids:
        return [], [], np.zeros((0, 0), dtype=np.int32)
    q, regions = ingest_device.gather(dev, state, [keep[i] for i in ids], len(inds))
    if ingest_device.TRACE:
        print(f"[ingest] gathered at {time.perf_counter() - t0:.3f} s", file=sys.stderr, flush=True)
    return ids, regions, q


def ingest_native(individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth, max_depth, threads,
                  console=None):
    """R1-R4 on the host C++ parser (see ``ingest``)."""
    inds = list(individuals)
    where = find_bed_gz_paths(inds, mosdepth_dir)
    paths = [str(where[ind]) if where[ind].exists() else None for ind in inds]
    window = (start, end) if start is not None and end is not None else None
    ing = _abi.Ingest(paths, norm_chrom(chromosome) if chromosome else None, window, excluded or {},
                      min_depth, max_depth, threads=max(1, int(threads or 1)))
    try:
        keep = {ind: i for i, ind in enumerate(inds) if ing.status[i] == 0 and ing.nvalid[i] > 0}
        removed = len(inds) - len(keep)
        if removed > 0:                       # filter_empty_samples (:576-600)
            msg = f"Removed {removed} samples with 0 regions"
            log(console, msg, style="warning") if console else print(msg)
        ids = sorted(keep)
        rof = np.full(len(inds), -1, dtype=np.int32)
        for r, ind in enumerate(ids):
            rof[keep[ind]] = r
        q = ing.fill(rof) if ids else np.zeros((0, ing.m), dtype=np.int32)
        regions = list(zip(ing.starts.tolist(), ing.ends.tolist())) if ids else []
        if not ids:
            q = np.zeros((0, 0), dtype=np.int32)
        return ids, regions, q
    finally:
        ing.close()


def ingest_py(individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth, max_depth, threads,
              console=None):
    """R1-R4 in one parse per file: population means (:218-301) -> valid
    regions (:81-83) -> per-sample extraction (:304-357) -> empty-sample
    filter (:576) -> sorted rows x sorted (start, end) columns (:379-416).
    Returns (ids, regions, int32 hundredths matrix)."""
    per = _read_all(individuals, mosdepth_dir, chromosome, start, end, excluded, threads)
    # population mean per (start, end), accumulated in `individuals` order
    keys = sorted({r for rec in per.values() for r in rec})
    kidx = {r: j for j, r in enumerate(keys)}
    sums = np.zeros(len(keys))
    cnts = np.zeros(len(keys), dtype=np.int64)
    for ind in individuals:
        rec = per.get(ind)
        if not rec:
            continue
        idx = np.fromiter((kidx[r] for r in rec), dtype=np.int64, count=len(rec))
        sums[idx] = sums[idx] + np.fromiter(rec.values(), dtype=np.float64, count=len(rec))
        cnts[idx] += 1
    with np.errstate(invalid="ignore", divide="ignore"):
        means = sums / cnts
    valid = (means >= min_depth) & (means <= max_depth) & (cnts > 0)
    rows = {}
    for ind in individuals:
        rec = per.get(ind)
        if rec is None:
            rows[ind] = []
            continue
        rows[ind] = [r for r in rec if valid[kidx[r]]]
    rows = filter_empty_samples(rows, console)
    ids = sorted(rows)
    regions = sorted({r for ind in ids for r in rows[ind]})
    col = {r: j for j, r in enumerate(regions)}
    q = np.full((len(ids), len(regions)), _abi.MISSING, dtype=np.int32)
    for i, ind in enumerate(ids):
        rec = per[ind]
        js = np.fromiter((col[r] for r in rows[ind]), dtype=np.int64, count=len(rows[ind]))
        d = np.fromiter((rec[r] for r in rows[ind]), dtype=np.float64, count=len(rows[ind]))
        try:
            q[i, js] = to_hundredths(d)
        except UnsupportedDepth as e:
            # mosdepth prints "%.2f"; other depth text takes the fp64 route
            # (the reference reads any decimal with float(), :272,334)
            where = find_bed_gz_for_individual(ind, mosdepth_dir)
            msg = f"{where}: {e}; normalising the cohort from fp64 depths"
            log(console, msg, style="warning") if console else print(msg)
            return ids, regions, _depth_matrix_f64(per, ids, rows, col, len(regions))
    return ids, regions, q


def _depth_matrix_f64(per, ids, rows, col, m):
    """The sorted rows x sorted (start, end) float64 matrix, NaN missing (:379-416)."""
    x = np.full((len(ids), m), np.nan, dtype=np.float64)
    for i, ind in enumerate(ids):
        rec = per[ind]
        js = np.fromiter((col[r] for r in rows[ind]), dtype=np.int64, count=len(rows[ind]))
        x[i, js] = np.fromiter((rec[r] for r in rows[ind]), dtype=np.float64, count=len(rows[ind]))
    return x


# ------------------------------------------------------------------ step --
def normalize_mosdepth(config, console):
    """Step entry point (:23-145)."""
    try:
        samples_file = config["samples_file"]
        samples = get_samples(samples_file)
        chrom = config.get("chrom", None)
        start = config.get("start_bp", None)
        end = config.get("end_bp", None)
        threads = config.get("threads", 1)
        prefix = config.get("mosdepth", {}).get("normalize", {}).get("output_file_prefix", None)
        ftype = config.get("output_file_type", "tsv")
        output_dir = config.get("output_dir", ".")
        output_file = Path(f"{output_dir}/{prefix}.{ftype}.gz")
        remove_intermediate = config.get("mosdepth", {}).get("remove_intermediate", False)
        mosdepth_dir = config.get("mosdepth", {}).get("work_dir", None)
        min_depth = config["mosdepth"]["normalize"].get("min_depth", 20)
        max_depth = config["mosdepth"]["normalize"].get("max_depth", 100)
        top_frac = config["mosdepth"]["normalize"].get("top_frac", 0.1)
        repeat_mask = config["mosdepth"]["normalize"].get("repeat_mask_file", None)
    except Exception as e:
        log(console, f"[red]Config error: {e}[/red]")
        return

    from .dist_step4 import dist_comm
    comm = dist_comm()                   # torch.distributed with > 1 rank: every GPU of the job
    output_path = Path(output_file).expanduser()
    output_path.parent.mkdir(parents=True, exist_ok=True)
    if comm is None or comm.rank == 0:
        output_path = setup_output_file(output_path, chrom, start, end)

    individuals = map_mosdepth_files_to_samples(mosdepth_dir, samples)
    if not individuals:
        log(console, f"✗ No mosdepth files found in {mosdepth_dir}", style="danger")
        sys.exit(1)
    excluded = load_repeat_mask(repeat_mask)
    args = (config, console, individuals, mosdepth_dir, chrom, start, end, excluded, min_depth, max_depth, top_frac,
            threads, output_path, remove_intermediate)
    if comm is not None:
        from . import dist_step4
        if _normalize_distributed(comm, *args):
            return
        # a case outside the distributed path (agreed by every rank): rank 0
        # runs the one-GPU step, the others wait for it
        dist_step4.rank0_step(comm, lambda: _normalize_one(*args))
        return
    _normalize_one(*args)


def _normalize_distributed(comm, config, console, individuals, mosdepth_dir, chrom, start, end, excluded, min_depth,
                           max_depth, top_frac, threads, output_path, remove_intermediate):
    """Steps 4 (+ 5's neighbour search when it is enabled) over every rank of
    the job (dist_step4.py).  False when the ranks agreed to fall back."""
    from . import dist_step4
    nbr = config["mosdepth"].get("neighbors", {})
    nbr_params = None
    if nbr.get("run") == True:  # noqa: E712  (the pipeline's own gate)
        nbr_params = {"zmax": nbr.get("zmax", 2.0), "sigma2_max": nbr.get("sigma2_max", 1000.0),
                      "frac_r": nbr.get("frac_r", 1.0), "n_neighbors": nbr.get("num_neighbors", 500)}
    if not bool(config["mosdepth"]["normalize"].get("device_ingest", True)):
        return False
    backend = dist_step4.make_backend(config)
    try:
        with backend.stream_ctx():
            rec = dist_step4.normalize_dist(comm, backend, individuals=individuals, mosdepth_dir=mosdepth_dir,
                                            chromosome=chrom, start=start, end=end, excluded=excluded,
                                            min_depth=min_depth, max_depth=max_depth, top_frac=top_frac,
                                            threads=max(1, int(threads or 1)), output_path=output_path,
                                            nbr_params=nbr_params, console=console)
            backend.sync()
    except dist_step4.DistFallback:
        release_ingest_buffers(*([backend.dev] if hasattr(backend, "dev") else []))
        return False
    if rec is None:
        log(console, "No valid samples with regions found.", style="danger")
        sys.exit(1)
    handoff.publish_neighbors(output_path, rec)
    if hasattr(backend, "dev"):
        step4_done(backend.dev)
    if comm.rank == 0:
        log(console, f"Mosdepth normalization complete. Results written to {output_path}", style="success")
        if remove_intermediate:
            remove_intermediate_files(mosdepth_dir, console, include_region_bed_gz=True)
    comm.barrier()
    return True


def _normalize_one(config, console, individuals, mosdepth_dir, chrom, start, end, excluded, min_depth, max_depth,
                   top_frac, threads, output_path, remove_intermediate):
    """Step 4 on one GPU (:23-145)."""
    dev = get_device(config)
    # mosdepth.normalize.device_ingest (default on): inflate on the GPU and the
    # host threads side by side, parse in HBM (ingest_device.py); anything
    # outside its grammar goes to the host parser.  Config 2 from files: 35 s
    # (BGZF) / 33 s (one gzip member per file) against 56 / 52 s for the host
    # parser (profiles/r03h_*, r03k_*)
    dev_ingest = bool(config["mosdepth"]["normalize"].get("device_ingest", True))
    with progress_bar(console, total=len(individuals), description="Extracting per-sample regions...") as (p, t):
        ids, regions, q = ingest(individuals, mosdepth_dir, chrom, start, end, excluded, min_depth, max_depth,
                                 threads, console, dev=dev if dev_ingest else None)
        p.update(t, completed=len(individuals))
    if not ids:
        log(console, "No valid samples with regions found.", style="danger")
        sys.exit(1)

    n, m = q.shape
    qd = q if isinstance(q, _abi.DevBuf) else dev.upload(q)     # the device ingest leaves it in HBM
    f64 = q.dtype == np.float64                      # depth text that is not exact hundredths
    st = (engine.normalize_stats_f64 if f64 else engine.normalize_stats)(dev, qd, n, m, m)
    sel, r = engine.select_regions(dev, st, top_frac)
    zq = dev.alloc((n, max(r, 1)), np.int32)
    if r:
        if f64:
            engine.zquant_f64(dev, qd, n, m, sel, r, st, zq)
        else:
            engine.zquant(dev, qd, n, m, sel, r, st, zq=zq)
    sel_h = sel.numpy()[:r]
    raw = st.rowmean.numpy()[:n]
    sel_means, sel_vars = st.mu.numpy()[:m][sel_h], st.var.numpy()[:m][sel_h]
    _write_normalized_q(output_path, ids, raw, sel_means, sel_vars, zq, dev=dev)     # from HBM (gzwrite.hip)
    # step 5 in this process takes the matrix from here instead of re-parsing
    # the file (values exactly as the text prints them; handoff.py)
    with np.errstate(invalid="ignore", divide="ignore"):
        ratios = np.where(sel_means > 0, 100.0 * sel_vars / sel_means, np.nan)
    handoff.publish(output_path, ids, engine.round_decimals(dev, raw, 2), engine.round_decimals(dev, ratios, 3),
                    zq, (n, r))
    step4_done(dev)         # the ingest's cached buffers (kept to the end of a pipeline run)
    log(console, f"Mosdepth normalization complete. Results written to {output_path}", style="success")
    if remove_intermediate:
        remove_intermediate_files(mosdepth_dir, console, include_region_bed_gz=True)
