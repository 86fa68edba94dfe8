"""Array-level driver of the MI355X hot path (steps 4-7).

Each function stages inputs in HBM, launches the HIP kernels of
libgridhip.so through ``grid_amd._abi`` and returns results.  The scalar
decision logic the reference performs in Python between its NumPy calls
(median -> scale, ``sorted(...)[int(top_frac*n)]`` threshold, sigma2 bounds)
stays here, on a handful of values read back from the device.

Reference correspondence (paths under /root/reference):
  normalize_stats / select   grid/utils/normalize_mosdepth.py:120, 419-499
  knn_*                      grid/utils/find_neighbors.py:57-65, 128-227
  dipcn                      grid/utils/compute_dipcn.py:62-88
  phase                      grid/utils/hi_inference.py:175-250
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import BLOCK, KBW, Device, DevBuf, GridNativeError, call, ptr

F8, I4, I8, U2, U1 = np.float64, np.int32, np.int64, np.uint16, np.uint8


def _read(buf: DevBuf, index: int):
    out = np.empty(1, dtype=buf.dtype)
    call("grid_d2h", buf.dev.ctx, out.ctypes.data, buf.ptr + index * buf.dtype.itemsize, buf.dtype.itemsize)
    return out[0]


def py_index(n: int, idx: int) -> int:
    """Python list indexing semantics (negative wraps, else IndexError)."""
    if idx < 0:
        idx += n
    if idx < 0 or idx >= n:
        raise IndexError("list index out of range")
    return idx


# ------------------------------------------------------------------ step 4 --
@dataclass
class NormStats:
    n: int
    m: int
    rowmean: DevBuf       # [n] f64 (== individual_raw_means)
    mu: DevBuf            # [m] f64
    var: DevBuf           # [m] f64
    ratio: DevBuf         # [m] f64 (NaN where mu <= 0)
    nvalid: int
    scale: float
    sorted_ratio: DevBuf  # [m] f64, first nvalid ascending


def row_means(dev: Device, q: DevBuf, n: int, m: int, ld: int) -> DevBuf:
    nblk = -(-m // BLOCK)
    bsum = dev.alloc((max(n, 1), max(nblk, 1)), F8)
    bcnt = dev.alloc((max(n, 1), max(nblk, 1)), I4)
    call("grid_norm_row_blocks", dev.ctx, ptr(q), n, m, ld, bsum.ptr, bcnt.ptr)
    rm = dev.alloc(max(n, 1), F8)
    call("grid_norm_row_means", dev.ctx, bsum.ptr, bcnt.ptr, n, nblk, rm.ptr)
    return rm


def median_scale(sorted_ratio: DevBuf, nvalid: int) -> float:
    """normalize_mosdepth.py:460-468 from the device-sorted valid ratios."""
    if nvalid == 0:
        return 1.0
    if nvalid % 2:
        med = float(_read(sorted_ratio, nvalid // 2))
    else:
        med = (float(_read(sorted_ratio, nvalid // 2 - 1)) + float(_read(sorted_ratio, nvalid // 2))) / 2.0
    if med > 0:
        return 1.0 / math.sqrt(med / 100.0)
    return 1.0


def normalize_stats(dev: Device, q: DevBuf, n: int, m: int, ld: int) -> NormStats:
    rm = row_means(dev, q, n, m, ld)
    mu, var, ratio = dev.alloc(max(m, 1), F8), dev.alloc(max(m, 1), F8), dev.alloc(max(m, 1), F8)
    call("grid_norm_col_means", dev.ctx, ptr(q), n, m, ld, rm.ptr, mu.ptr)
    call("grid_norm_col_vars", dev.ctx, ptr(q), n, m, ld, rm.ptr, mu.ptr, var.ptr, ratio.ptr)
    srt = dev.alloc(max(m, 1), F8)
    nv = C.c_int64()
    call("grid_sort_valid", dev.ctx, ratio.ptr, m, srt.ptr, C.byref(nv))
    scale = median_scale(srt, nv.value)
    return NormStats(n, m, rm, mu, var, ratio, nv.value, scale, srt)


def normalize_stats_f64(dev: Device, x: DevBuf, n: int, m: int, ld: int) -> NormStats:
    """normalize_stats on fp64 depths (NaN = missing): the route for depth text
    that is not exact hundredths (the reference parses any decimal, :272,334)."""
    nblk = -(-m // BLOCK)
    bsum = dev.alloc((max(n, 1), max(nblk, 1)), F8)
    bcnt = dev.alloc((max(n, 1), max(nblk, 1)), I4)
    call("grid_norm_row_blocks_f64", dev.ctx, ptr(x), n, m, ld, bsum.ptr, bcnt.ptr)
    rm = dev.alloc(max(n, 1), F8)
    call("grid_norm_row_means", dev.ctx, bsum.ptr, bcnt.ptr, n, nblk, rm.ptr)
    mu, var, ratio = dev.alloc(max(m, 1), F8), dev.alloc(max(m, 1), F8), dev.alloc(max(m, 1), F8)
    call("grid_norm_col_stats_f64", dev.ctx, ptr(x), n, m, ld, rm.ptr, mu.ptr, var.ptr, ratio.ptr)
    srt = dev.alloc(max(m, 1), F8)
    nv = C.c_int64()
    call("grid_sort_valid", dev.ctx, ratio.ptr, m, srt.ptr, C.byref(nv))
    scale = median_scale(srt, nv.value)
    return NormStats(n, m, rm, mu, var, ratio, nv.value, scale, srt)


def select_regions(dev: Device, st: NormStats, top_frac: float):
    """select_high_variance_regions (normalize_mosdepth.py:492-499)."""
    if st.nvalid == 0:
        return dev.alloc(1, I4), 0
    k = py_index(st.nvalid, int(top_frac * st.nvalid))
    thr = float(_read(st.sorted_ratio, k))
    sel = dev.alloc(max(st.m, 1), I4)
    cnt = C.c_int64()
    call("grid_select_gt", dev.ctx, st.ratio.ptr, st.m, thr, sel.ptr, C.byref(cnt))
    return sel, cnt.value


def zquant(dev: Device, q, n, ld, sel: DevBuf, r: int, st: NormStats, zq: DevBuf | None = None,
           colmap: DevBuf | None = None, qmax: int = 0, zb: DevBuf | None = None, ld_zb: int = 0):
    of = C.c_int32()
    call("grid_norm_zquant", dev.ctx, ptr(q), n, ld, sel.ptr, r, st.rowmean.ptr, st.mu.ptr, st.scale,
         ptr(zq), r, ptr(colmap), qmax, ptr(zb), ld_zb, C.byref(of))
    if of.value:
        raise GridNativeError("normalised z-score exceeds the int32 hundredths range")


def zquant_f64(dev: Device, x, n, ld, sel: DevBuf, r: int, st: NormStats, zq: DevBuf):
    """zquant on fp64 depths (int32 z hundredths of the selected columns)."""
    of = C.c_int32()
    call("grid_norm_zquant_f64", dev.ctx, ptr(x), n, ld, sel.ptr, r, st.rowmean.ptr, st.mu.ptr, st.scale,
         ptr(zq), r, C.byref(of))
    if of.value:
        raise GridNativeError("normalised z-score exceeds the int32 hundredths range")


# ------------------------------------------------------------------ step 5 --
def qmax_for_zmax(zmax: float) -> int:
    """Clip bound in hundredths for the exact integer path, or raise."""
    q = int(round(zmax * 100))
    if q / 100.0 != zmax or not (0 <= q <= 256):
        raise GridNativeError(f"zmax={zmax!r}: the exact bf16 k-NN path needs zmax = k/100 with 0 <= k <= 256")
    return q


def pad_to(x: int, a: int) -> int:
    return -(-x // a) * a


def sigma2_min(dev: Device, r3: DevBuf, r: int, frac_r: float):
    """find_neighbors.py:148-161 on device-resident ratios; None if no finite."""
    srt = dev.alloc(max(r, 1), F8)
    nv = C.c_int64()
    call("grid_sort_valid", dev.ctx, r3.ptr, r, srt.ptr, C.byref(nv))
    if nv.value == 0:
        return None
    lo = min(int(r * (1.0 - frac_r)), nv.value - 1)
    return float(_read(srt, lo))


def knn(dev: Device, zb: DevBuf, n: int, np_: int, kpad: int, ld: int, qmax: int, k: int,
        r_use: int, kblocked: bool = False):
    """Exact k-NN on a bf16 hundredths panel (row-major [np][ld], or
    K-blocked [kpad/32][np][32]): returns (idx, d2 hundredths^2, cnt) numpy."""
    if 4 * qmax * qmax * max(r_use, 1) >= 2 ** 44:
        raise GridNativeError("R_use too large for the packed distance key")
    gram = dev.zeros((np_, np_), I8)
    if kblocked:
        call("grid_knn_gram_kb", dev.ctx, zb.ptr, np_, kpad, qmax, gram.ptr)
    else:
        call("grid_knn_gram", dev.ctx, zb.ptr, np_, kpad, ld, qmax, gram.ptr)
    kk = max(k, 1)
    idx, d2, cnt = dev.alloc((n, kk), I4), dev.alloc((n, kk), I8), dev.alloc(n, I4)
    call("grid_knn_topk", dev.ctx, gram.ptr, n, np_, k, 0, n, idx.ptr, d2.ptr, cnt.ptr)
    return idx.numpy(), d2.numpy(), cnt.numpy()


def knn_from_hundredths(dev: Device, zq: np.ndarray, k: int, qmax: int):
    """Host (n x R_use) int hundredths, already clipped to +-qmax, NaN -> 0:
    (idx, exact d2 in hundredths^2, cnt)."""
    zq = np.ascontiguousarray(zq, dtype=np.int32)
    return _knn_zq(dev, zq, np.arange(zq.shape[1], dtype=np.int32), k, qmax / 100.0, False)


def _dist_key_scale(bound: float, integer: bool) -> float:
    """Power-of-two key scale with floor(d2 * scale) < 2^44 for d2 <= bound:
    1 for exact integer distances that fit (they then stay exact), else the
    finest scale (fp64 distances keep 44 significant bits of the largest)."""
    if integer and bound < 2.0 ** 44:
        return 1.0
    return math.ldexp(1.0, 43 - math.frexp(bound)[1])


def _knn_zq(dev: Device, zq: np.ndarray, cols: np.ndarray, k: int, zmax: float, values: bool):
    """Step 5 on integer hundredths zq [n][ld] (GRID_MISSING = NaN; GRID_ZQ_NEG0,
    the step-4 "-0.00" code in a hand-off, = 0) restricted
    to columns ``cols``, clipped to +-zmax (find_neighbors.py:57-58).  Path:
      * zmax = q/100, q <= 256: bf16-exact MFMA Gram (k_gram8) + row top-k;
      * zmax = q/100, q > 256: exact int64 direct-difference distances;
      * otherwise (clips are not hundredths): fixed-order fp64 distances.
    Returns (idx, d2, cnt); d2 is float64 in value^2 units when ``values``,
    else int64 hundredths^2 (integer paths only)."""
    if isinstance(zq, list):                    # a holder: this call takes the only reference
        zq = zq.pop()
    if isinstance(zq, DevBuf):                  # already on the device (step-4 hand-off)
        assert zq.dtype == np.int32 and len(zq.shape) == 2
    else:
        zq = np.ascontiguousarray(zq, dtype=np.int32)
    n, ld = zq.shape
    r = len(cols)
    kk = max(k, 1)
    if n == 0:
        return np.zeros((0, kk), I4), np.zeros((0, kk), F8 if values else I8), np.zeros(0, I4)
    q = int(round(zmax * 100))
    hundredths = q / 100.0 == zmax and 0 <= q < 2 ** 30
    dz = zq if isinstance(zq, DevBuf) else dev.upload(zq)
    dcols = dev.upload(np.ascontiguousarray(cols if r else np.zeros(1), dtype=I4))
    np_ = pad_to(n, 256)
    if hundredths and q <= 256:
        kpad = pad_to(max(r, 1), 64)
        zb = dev.alloc((kpad // KBW, np_, KBW), U2)
        call("grid_knn_panel_i32", dev.ctx, dz.ptr, n, ld, dcols.ptr, r, q, zb.ptr, np_, kpad)
        del dz, zq                              # step 4's matrix is freed before the Gram is allocated
        idx, d2, cnt = knn(dev, zb, n, np_, kpad, kpad, q, k, r, kblocked=True)
        return idx, (d2 / 10000.0 if values else d2), cnt
    d2m = dev.alloc((np_, np_), F8)
    if hundredths:
        if 4.0 * q * q * max(r, 1) >= 2.0 ** 53:
            raise GridNativeError("zmax too large for exact int64 distances stored as fp64")
        g = dev.alloc((n, max(r, 1)), I4)
        call("grid_knn_gather_i32", dev.ctx, dz.ptr, n, ld, dcols.ptr, r, q, g.ptr)
        del dz, zq
        call("grid_knn_dist_i32", dev.ctx, g.ptr, n, r, max(r, 1), d2m.ptr, np_)
        scale = _dist_key_scale(4.0 * q * q * max(r, 1), True)
        unit = 10000.0
    else:
        g = dev.alloc((n, max(r, 1)), F8)
        call("grid_knn_gather_f64", dev.ctx, dz.ptr, n, ld, dcols.ptr, r, float(zmax), g.ptr)
        del dz, zq
        call("grid_knn_dist_f64", dev.ctx, g.ptr, n, r, max(r, 1), d2m.ptr, np_)
        scale = _dist_key_scale(4.0 * zmax * zmax * max(r, 1) + 1.0, False)
        unit = 1.0
    del g
    idx, d2, cnt = dev.alloc((n, kk), I4), dev.alloc((n, kk), F8), dev.alloc(n, I4)
    call("grid_knn_topk_d2", dev.ctx, d2m.ptr, np_, scale, n, k, 0, n, idx.ptr, d2.ptr, cnt.ptr)
    d2h = d2.numpy()
    if values:
        return idx.numpy(), d2h / unit, cnt.numpy()
    if unit != 10000.0:
        raise GridNativeError("integer distances requested from the fp64 path")
    return idx.numpy(), d2h.astype(I8), cnt.numpy()


def knn_from_zq(dev: Device, zq: np.ndarray, cols: np.ndarray, k: int, zmax: float):
    """find_neighbors.py:57-65 + find_neighbors_sklearn on the step-4
    hundredths: (idx, squared distances in value^2 units, cnt).  ``zq`` may be
    a one-element list holding the matrix: the call then owns it and frees it
    once the k-NN panel is built (step 5's peak HBM is max(zq + panel,
    panel + Gram), not their sum)."""
    return _knn_zq(dev, zq, cols, k, zmax, True)


def knn_values(dev: Device, data: np.ndarray, k: int):
    """find_neighbors_sklearn (:179-227) on an arbitrary float64 matrix (already
    clipped / NaN-free): exact integer paths when every value is a hundredth,
    the fp64 direct-difference path otherwise.  (idx, d2 values, cnt)."""
    data = np.ascontiguousarray(data, dtype=F8)
    n, r = data.shape
    kk = max(k, 1)
    if n == 0:
        return np.zeros((0, kk), I4), np.zeros((0, kk), F8), np.zeros(0, I4)
    if not np.all(np.isfinite(data)):
        raise GridNativeError("find_neighbors_sklearn: NaN/inf in the data matrix (sklearn rejects it too)")
    qv = np.rint(data * 100.0)
    if np.array_equal(qv / 100.0, data) and (qv.size == 0 or np.abs(qv).max() < 2 ** 30):
        qmax = int(np.abs(qv).max()) if qv.size else 0
        return _knn_zq(dev, qv.astype(np.int32), np.arange(r, dtype=np.int32), k, qmax / 100.0, True)
    np_ = pad_to(n, 256)
    dz = dev.upload(data)
    d2m = dev.alloc((np_, np_), F8)
    call("grid_knn_dist_f64", dev.ctx, dz.ptr, n, r, r, d2m.ptr, np_)
    m = float(np.abs(data).max()) if data.size else 0.0
    scale = _dist_key_scale(4.0 * m * m * max(r, 1) + 1.0, False)
    idx, d2, cnt = dev.alloc((n, kk), I4), dev.alloc((n, kk), F8), dev.alloc(n, I4)
    call("grid_knn_topk_d2", dev.ctx, d2m.ptr, np_, scale, n, k, 0, n, idx.ptr, d2.ptr, cnt.ptr)
    return idx.numpy(), d2.numpy(), cnt.numpy()


def round_decimals(dev: Device, v: np.ndarray, decimals: int) -> np.ndarray:
    """float("%.{decimals}f" % x) for every x (grid_round_decimals; NaN stays NaN)."""
    v = np.ascontiguousarray(v, dtype=F8)
    if v.size == 0:
        return v.copy()
    d = dev.upload(v)
    call("grid_round_decimals", dev.ctx, d.ptr, v.size, decimals, d.ptr)
    return d.numpy()


# ------------------------------------------------------------------ step 6 --
def dipcn(dev: Device, reads: np.ndarray, has: np.ndarray, scale: np.ndarray, nbr: np.ndarray,
          nscale: np.ndarray, ncnt: np.ndarray, n_nbr: int, n_rows: int | None = None):
    """reads/has/scale are indexed by sample id over a universe that starts
    with the ``n_rows`` neighbour-file rows; nbr holds universe indices."""
    n = len(ncnt) if n_rows is None else n_rows
    ld = nbr.shape[1] if nbr.ndim == 2 else 0
    d = [dev.upload(np.ascontiguousarray(a)) for a in
         (reads.astype(F8), has.astype(U1), scale.astype(F8), nbr.astype(I4), nscale.astype(F8), ncnt.astype(I4))]
    out, valid = dev.alloc(max(n, 1), F8), dev.alloc(max(n, 1), U1)
    zd = C.c_int32()
    call("grid_dipcn", dev.ctx, n, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, d[4].ptr, d[5].ptr, ld, n_nbr,
         out.ptr, valid.ptr, C.byref(zd))
    if zd.value:
        raise ZeroDivisionError("float division by zero")
    return out.numpy()[:n], valid.numpy()[:n].astype(bool)


# ------------------------------------------------------------------ step 7 --
def csr_from_lists(hap_nbrs):
    off = np.zeros(len(hap_nbrs) + 1, dtype=I8)
    for h, lst in enumerate(hap_nbrs):
        off[h + 1] = off[h] + len(lst)
    nbr = np.fromiter((a for lst in hap_nbrs for a, _ in lst), dtype=I4, count=int(off[-1]))
    w = np.fromiter((b for lst in hap_nbrs for _, b in lst), dtype=F8, count=int(off[-1]))
    return off, nbr, w


def phase(dev: Device, irr: np.ndarray, off: np.ndarray, nbr: np.ndarray, w: np.ndarray, min_nbr: int,
          n_iters: int, legacy: bool = False, paired: bool = False):
    """``legacy`` selects the per-neighbour LDS kernel (k_phase) that larger
    loci run anyway; ``paired`` the register-pipelined kernel with both
    haplotypes of a sample on one lane (A/B tests; same results)."""
    n = len(irr)
    if n == 0:
        return np.zeros(0), np.zeros(0), 0.0
    order, loff, nl, pk_nbr, pk_w, pk_cnt, flags, max_list = _abi.hi_schedule(off, nbr, w)
    bufs = [dev.upload(np.ascontiguousarray(a)) for a in
            (np.asarray(irr, F8), off.astype(I8), (nbr if nbr.size else np.zeros(1, I4)).astype(I4),
             (w if w.size else np.zeros(1, F8)).astype(F8), order.astype(I4), loff.astype(I4), pk_nbr, pk_w,
             pk_cnt)]
    hap, imp, mean = dev.alloc(2 * n, F8), dev.alloc(2 * n, F8), dev.alloc(1, F8)
    call("grid_hi_phase", dev.ctx, n, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, bufs[3].ptr, min_nbr, n_iters,
         bufs[4].ptr, bufs[5].ptr, nl, bufs[6].ptr, bufs[7].ptr, bufs[8].ptr, hap.ptr, imp.ptr, mean.ptr,
         flags | (_abi.HI_LEGACY if legacy else 0) | (_abi.HI_PAIRED if paired else 0), max_list)
    return hap.numpy(), imp.numpy(), float(mean.numpy()[0])


def phase_batch(dev: Device, loci, min_nbr: int, n_iters: int, legacy: bool = False, paired: bool = False,
                group: int | None = None, inflight: int = 3):
    """Batched phasing + imputation of L independent loci (one workgroup per
    locus; BASELINE config 5).  ``loci``: sequence of (irr [n], off [2n+1],
    nbr, w) per locus (CSR as csr_from_lists).  Returns a list of (hap [2n],
    imp [2n], mean) equal to phase() per locus.

    The loci run in GROUPS of ``group`` (default: the device's CU count, one
    workgroup per CU, so a group is one round of the launch the whole batch
    would make).  Host work per group is the level schedules (grid_hi_levels,
    host C++ on a thread pool: the calls release the GIL) and one arena of the
    group's inputs, copied to HBM in ONE transfer on a copy stream -- done by a
    background thread for group g+1 while group g phases on the device.  The
    packed neighbour lists are built on the device (grid_hi_pack_batch);
    every group writes into one output arena, copied back once.  Unit-weight
    loci share one device vector of ones as their weights.

    Up to ``inflight`` groups run at once, each on a stream of its own: a
    50k-sample locus keeps its haplotypes in global memory and its workgroup
    waits on gathers, and a CU holds up to three of these workgroups (75
    VGPRs, 512 threads), so groups launched one after another on one stream
    left two thirds of every CU idle."""
    import os
    from concurrent.futures import ThreadPoolExecutor
    if not len(loci):
        return []
    legacy_f = _abi.HI_LEGACY if legacy else 0
    if group is None:
        group = max(1, _abi.device_cu_count(dev))
    pool = ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 1)))
    bg = ThreadPoolExecutor(1)
    cdev = Device(dev.index)                  # its own non-blocking stream: uploads beside the phasing
    lanes = [dev] + [Device(dev.index) for _ in range(max(1, int(inflight)) - 1)]   # launch streams

    def al(x):
        return -(-int(x) // 256) * 256

    def prep(l):
        irr, off, nbr, w = l
        off = np.ascontiguousarray(off, dtype=I8)
        nbr = np.ascontiguousarray(nbr if len(nbr) else np.zeros(1), dtype=I4)
        order, loff, nl = _abi.hi_levels(off, nbr)
        unit = len(w) == 0 or bool(np.all(np.asarray(w) == 1.0))
        lens = np.diff(off) if len(off) > 1 else np.zeros(1, I8)
        return off, nbr, order, loff, nl, unit, int(lens.max()) if lens.size else 0

    sizes = [len(l[0]) for l in loci]
    o_hap = np.zeros(len(sizes) + 1, dtype=np.int64)
    np.cumsum([2 * max(n, 1) for n in sizes], out=o_hap[1:])
    tot = int(o_hap[-1])
    d_out = dev.alloc(2 * tot + len(sizes), F8)

    def stage(g0, g1):
        """Host prep + upload of loci [g0, g1); returns what the launches need."""
        sub = loci[g0:g1]
        pre = list(pool.map(prep, sub))
        flags = _abi.HI_UNIT_WEIGHTS if all(p[5] for p in pre) else 0
        need_pkw = bool(legacy_f) or not flags
        max_nnz = max(len(p[1]) for p in pre)
        arrs, offs, pos = [], [], 0
        for (irr, _, _, w), (off, nbr, order, loff, nl, unit, _) in zip(sub, pre):
            n = len(irr)
            la = [np.ascontiguousarray(irr if n else np.zeros(1), dtype=F8), off, nbr,
                  None if unit else np.ascontiguousarray(w if len(w) else np.zeros(1), dtype=F8),
                  np.ascontiguousarray(order if n else np.zeros(1), dtype=I4), np.ascontiguousarray(loff, dtype=I4)]
            lo = []
            for x in la:
                lo.append(None if x is None else pos)
                pos += 0 if x is None else al(x.nbytes)
            arrs.append(la)
            offs.append(lo)
        host = np.empty(max(pos, 1), dtype=U1)

        def fill(k):
            for x, o in zip(arrs[k], offs[k]):
                if x is not None:
                    host[o:o + x.nbytes] = x.view(U1).reshape(-1)
        list(pool.map(fill, range(len(sub))))
        d_in = cdev.upload(host)
        ones = cdev.upload(np.ones(max(max_nnz, 1), dtype=F8)) if any(p[5] for p in pre) else None
        pk_pos, ppos = [], 0
        for l in sub:
            n1 = max(len(l[0]), 1)
            a1 = ppos + al(n1 * 2 * _abi.PACK_CAP * 4)
            pk_pos.append((ppos, a1, a1 + al(n1 * 8)))
            ppos = a1 + al(n1 * 8) + (al(n1 * 2 * _abi.PACK_CAP * 8) if need_pkw else 0)
        d_pk = cdev.alloc(max(ppos, 1), U1)
        descs = []
        for k, l in enumerate(sub):
            n, gk = len(l[0]), g0 + k
            io = [None if o is None else d_in.ptr + o for o in offs[k]]
            p0, p1, p2 = (d_pk.ptr + x for x in pk_pos[k])
            hap = d_out.ptr + 8 * int(o_hap[gk])
            imp = d_out.ptr + 8 * (tot + int(o_hap[gk]))
            mean = d_out.ptr + 8 * (2 * tot + gk)
            w_ptr = io[3] if io[3] is not None else ones.ptr
            descs.append(_abi.HiLocus(n, io[0], io[1], io[2], w_ptr, io[4], io[5], pre[k][4], 0, p0,
                                      p2 if need_pkw else None, p1, hap, imp, mean))
        arr = (_abi.HiLocus * len(descs))(*descs)
        d_arr = cdev.alloc(C.sizeof(arr), U1)
        call("grid_h2d", cdev.ctx, d_arr.ptr, C.addressof(arr), C.sizeof(arr))
        meta = (len(descs), max(len(l[0]) for l in sub), max(p[4] for p in pre), max(p[6] for p in pre), flags)
        return (d_in, ones, d_pk, d_arr), meta

    bounds = [(g0, min(len(loci), g0 + group)) for g0 in range(0, len(loci), group)]
    keep = [None] * len(lanes)                # per launch stream: the inputs of its group in flight
    try:
        fut = bg.submit(stage, *bounds[0])
        for gi in range(len(bounds)):
            bufs, (nd, max_n, max_nlev, max_list, flags) = fut.result()
            if gi + 1 < len(bounds):
                fut = bg.submit(stage, *bounds[gi + 1])
            ln = lanes[gi % len(lanes)]
            if keep[gi % len(lanes)] is not None:
                # that stream's previous group's inputs are dead once its phasing ends:
                # device memory follows the groups in flight, not the number of loci
                ln.sync()
                for b_ in keep[gi % len(lanes)]:
                    if b_ is not None:
                        b_.free()
            keep[gi % len(lanes)] = bufs
            d_arr = bufs[3]
            # the group's inputs were copied on cdev's stream: order the launches
            # behind them through the runtime, not only through the host's wait
            call("grid_stream_after", ln.ctx, cdev.ctx)
            for l0 in range(0, nd, 65535):            # grid.y of the pack launch
                call("grid_hi_pack_batch", ln.ctx, min(65535, nd - l0), d_arr.ptr + l0 * C.sizeof(_abi.HiLocus),
                     max_n)
            call("grid_hi_phase_batch", ln.ctx, nd, d_arr.ptr, max_n, max_nlev, min_nbr, n_iters,
                 flags | legacy_f | (_abi.HI_PAIRED if paired else 0), max_list)
        for ln in lanes:
            ln.sync()
        out = d_out.numpy()
    finally:
        bg.shutdown(wait=True)
        pool.shutdown(wait=True)
        for ln in lanes:
            ln.sync()
        for bufs_ in keep:                    # cdev's buffers, freed before its context closes
            for b_ in bufs_ or ():
                if b_ is not None:
                    b_.free()
        cdev.close()
        for ln in lanes[1:]:
            ln.close()
    res = []
    for k, n in enumerate(sizes):
        h0 = int(o_hap[k])
        res.append((out[h0:h0 + 2 * n].copy(), out[tot + h0:tot + h0 + 2 * n].copy(),
                    float(out[2 * tot + k]) if n else 0.0))
    return res
