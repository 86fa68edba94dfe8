"""Array-level restatement of GRiD steps 4-7 (TEST INFRASTRUCTURE ONLY).

Each function below re-expresses, with the same fp64 operation order, one
piece of the reference (paths relative to /root/reference):

  step 4  grid/utils/normalize_mosdepth.py  normalize_matrix :419-476,
          select_high_variance_regions :479-499, write_normalized_output :502-554
  step 5  grid/utils/find_neighbors.py  read/clip :57-58, filter :128-175,
          find_neighbors_sklearn :179-227, save_neighbors :231-267
  step 6  grid/utils/compute_dipcn.py   :62-88
  step 7  grid/utils/hi_inference.py    _run_phasing :175-226, _compute_imp :229-250

The k-NN restatement computes exact squared distances on the integer
hundredths (an fp64 BLAS product of integers < 2**53 is exact) and orders by
(distance, index).  scikit-learn's brute ArgKmin (third-party, sklearn 1.7.2,
un-vendored) returns the same order wherever exact distances differ; its
order among exact ties is unspecified (sklearn utils/_sorting.pyx), so the
golden fixtures are generated tie-free at the k boundary.
"""
from __future__ import annotations

import math

import numpy as np

from .npsum import nanmean_cols, nanmean_rows, nansum_cols


# ----------------------------------------------------------------- step 4 --
def normalize_matrix(mat: np.ndarray):
    """normalize_mosdepth.py:419-476."""
    mat = np.array(mat, dtype=np.float64, copy=True)
    row_means = nanmean_rows(mat)                                   # :440
    row_means_safe = np.where(row_means == 0, np.nan, row_means)    # :441
    with np.errstate(invalid="ignore", divide="ignore"):
        mat = mat / row_means_safe[:, None]                         # :442
    n = mat.shape[0]
    with np.errstate(invalid="ignore", divide="ignore"):
        col_means = nanmean_cols(mat)                               # :445
        d = mat - col_means[None, :]
        col_vars = nansum_cols(d * d) / (n - 1)                     # :446
        var_ratio = np.where(col_means > 0, (100.0 * col_vars) / col_means, np.nan)  # :451
    mu_pos = col_means > 0
    sqrt_mu = np.sqrt(np.where(mu_pos, col_means, np.nan))
    with np.errstate(invalid="ignore"):
        mat[:, mu_pos] = (mat[:, mu_pos] - col_means[mu_pos]) / sqrt_mu[mu_pos]   # :458
    valid = var_ratio[~np.isnan(var_ratio)]
    scale = 1.0
    if valid.size > 0:
        med = median(valid)
        if med > 0:
            scale = 1.0 / math.sqrt(med / 100.0)                    # :464
    mat = mat * scale                                               # :470
    ratios = {i: float(var_ratio[i]) for i in range(len(col_means)) if not np.isnan(var_ratio[i])}
    return mat, ratios, col_means, col_vars, scale


def median(v: np.ndarray) -> float:
    """np.median of a NaN-free vector: middle element, or (a+b)/2."""
    s = sorted(float(x) for x in v)
    n = len(s)
    if n % 2:
        return s[n // 2]
    return (s[n // 2 - 1] + s[n // 2]) / 2.0


def select_high_variance_regions(ratios: dict, top_frac: float):
    """normalize_mosdepth.py:479-499 (keeps ratio > sorted[int(top_frac*n)])."""
    if not ratios:
        return []
    srt = sorted(ratios.values())
    thr = srt[int(top_frac * len(srt))]
    return [i for i, r in ratios.items() if r > thr]


def raw_means(mat: np.ndarray) -> np.ndarray:
    """individual_raw_means, normalize_mosdepth.py:120."""
    return nanmean_rows(np.asarray(mat, dtype=np.float64))


def normalized_lines(z, ids, sel, col_means, col_vars, raw):
    """Text lines of write_normalized_output (normalize_mosdepth.py:535-554)."""
    n, r = len(ids), len(sel)
    sm = col_means[sel]
    sv = col_vars[sel]
    with np.errstate(invalid="ignore", divide="ignore"):
        sr = np.where(sm > 0, 100.0 * sv / sm, np.nan)
    out = [f"{n}\t{r}\t" + "\t".join("NA" if np.isnan(v) else f"{v:.3f}" for v in sm) + "\n",
           f"{n}\t{r}\t" + "\t".join("NA" if np.isnan(v) else f"{v:.3f}" for v in sr) + "\n"]
    for i, sid in enumerate(ids):
        vals = ["NA" if np.isnan(z[i, j]) else f"{z[i, j]:.2f}" for j in sel]
        out.append(f"{sid}\t{raw[i]:.2f}\t" + "\t".join(vals) + "\n")
    return out


# ----------------------------------------------------------------- step 5 --
def parse_normalized(lines):
    """read_normalized_data, find_neighbors.py:99-124 (from decompressed lines)."""
    parts = lines[1].strip().split("\t")
    ratios = np.array([np.nan if v in ("NA", "nan") else float(v) for v in parts[2:]])
    ids, scales, rows = [], {}, []
    for line in lines[2:]:
        p = line.strip().split("\t")
        ids.append(p[0])
        scales[p[0]] = float(p[1])
        rows.append([np.nan if v in ("NA", "nan") else float(v) for v in p[2:]])
    return ids, ratios, np.array(rows, dtype=float), scales


def filter_regions_by_variance(r: np.ndarray, frac_r=1.0, sigma2_max=1000.0):
    """find_neighbors.py:148-175."""
    R = len(r)
    finite = np.isfinite(r)
    fv = np.sort(r[finite])
    if len(fv) == 0:
        return np.arange(R), R
    lo = min(int(R * (1.0 - frac_r)), len(fv) - 1)
    smin = float(fv[lo])
    keep = finite & (r >= smin) & (r <= sigma2_max)
    idx = np.where(keep)[0]
    return idx, len(idx)


def knn_exact(zq: np.ndarray, n_neighbors: int):
    """Exact restatement of find_neighbors_sklearn (find_neighbors.py:179-227)
    on integer hundredths ``zq`` (N x R_use, int).  Returns per-row lists of
    (index, S) where S = sum((zq_i - zq_j)**2) in 1e-4 units (exact int)."""
    N = zq.shape[0]
    k = min(n_neighbors + 1, N)
    q = zq.astype(np.float64)
    g = q @ q.T                               # exact: integers < 2**53
    nrm = np.diag(g).copy()
    d2 = (nrm[:, None] + nrm[None, :] - 2.0 * g).astype(np.int64)
    res = []
    for i in range(N):
        order = np.lexsort((np.arange(N), d2[i]))[:k]
        lst = []
        for j in order:
            if j == i:
                continue
            lst.append((int(j), int(d2[i, j])))
            if len(lst) == n_neighbors:
                break
        res.append(lst)
    return res


def knn_direct_f64(data: np.ndarray, n_neighbors: int):
    """find_neighbors_sklearn semantics on general fp64 values, restated as the
    direct-difference distance d2_ij = sum_k (x_ik - x_jk)^2 accumulated
    sequentially in k (np.cumsum is sequential), ordered by (d2, j).  This is
    the arithmetic grid_knn_dist_f64 performs, so d2 values compare bit for
    bit; sklearn (find_neighbors.py:207-213) computes the same distances up to
    its fp64 rounding (GEMM trick).  Returns per-row lists of (index, d2)."""
    x = np.asarray(data, dtype=np.float64)
    N = x.shape[0]
    k = min(n_neighbors + 1, N)
    res = []
    for i in range(N):
        d = (x[i][None, :] - x) ** 2
        d2 = np.cumsum(d, axis=1)[:, -1] if x.shape[1] else np.zeros(N)
        order = np.lexsort((np.arange(N), d2))[:k]
        lst = [(int(j), float(d2[j])) for j in order if j != i][:n_neighbors]
        res.append(lst)
    return res


def neighbor_lines(ids, scales, nbrs, R_use):
    """save_neighbors text (find_neighbors.py:258-267); d2 in 1e-4 units."""
    if R_use == 0:
        R_use = 1
    out = []
    for i, sid in enumerate(ids):
        line = f"{sid}\t{scales.get(sid, 1.0):.2f}"
        for j, s in nbrs[i]:
            sq = s / 10000.0
            nd = sq / (2 * R_use)
            line += f"\t{ids[j]}\t{scales.get(ids[j], 1.0):.2f}\t{nd:.2f}"
        out.append(line + "\n")
    return out


# ----------------------------------------------------------------- step 6 --
def dipcn(neighbors: dict, sample_scales: dict, reads: dict, n_nbr: int):
    """compute_dipcn.py:62-88.  Returns [(sample_id, norm_reads)]."""
    out = []
    for sid, lst in neighbors.items():
        s = sample_scales.get(sid)
        if s is None or sid not in reads:
            continue
        total, count = 0.0, 0
        for nid, ns in lst:
            if count >= n_nbr:
                break
            if nid not in reads:
                continue
            total += reads[nid] / ns
            count += 1
        if count == 0:
            continue
        out.append((sid, (reads[sid] / s) / (total / count)))
    return out


# ----------------------------------------------------------------- step 7 --
def run_phasing(irr, hap_nbrs, min_nbr, n_iters):
    """hi_inference.py:175-226 (in-place Gauss-Seidel)."""
    N = len(irr)
    hap = [float("nan")] * (2 * N)
    n_ph, mean = 0, 0.0
    for i in range(N):
        if len(hap_nbrs[2 * i]) >= min_nbr and len(hap_nbrs[2 * i + 1]) >= min_nbr:
            hap[2 * i] = irr[i] / 2
            hap[2 * i + 1] = irr[i] / 2
            n_ph += 1
            mean += irr[i]
    if n_ph > 0:
        mean /= n_ph
    for _ in range(n_iters):
        for i in range(N):
            if math.isnan(hap[2 * i]):
                continue
            ws = [1e-9, 1e-9]
            wv = [0.0, 0.0]
            for h in range(2):
                for nb, w in hap_nbrs[2 * i + h]:
                    v = hap[nb]
                    if not math.isnan(v):
                        ws[h] += w
                        wv[h] += w * v
            m0 = wv[0] / ws[0]
            m1 = wv[1] / ws[1]
            den = m0 + m1
            if den > 0:
                hap[2 * i] = irr[i] * m0 / den
                hap[2 * i + 1] = irr[i] * m1 / den
    return hap, mean


def compute_imp(i, hap, hap_nbrs, mean):
    """hi_inference.py:229-250."""
    ws = [1e-9, 1e-9]
    wv = [0.0, 0.0]
    for h in range(2):
        for nb, w in hap_nbrs[2 * i + h]:
            v = hap[nb]
            if not math.isnan(v):
                ws[h] += w
                wv[h] += w * v
    i0 = wv[0] / ws[0]
    i1 = wv[1] / ws[1]
    if ws[0] <= 1e-9:
        i0 = mean / 2
    if ws[1] <= 1e-9:
        i1 = mean / 2
    return i0, i1


def haploid_lines(ids, irr, hap, imp):
    """hi_inference.py:329-337."""
    out = ["ID\tIRRs\thap1phased\thap2phased\thap1imp\thap2imp\n"]
    for i, sid in enumerate(ids):
        out.append(f"{sid}\t{irr[i]:.2f}\t{hap[2*i]:.2f}\t{hap[2*i+1]:.2f}\t"
                   f"{imp[i][0]:.2f}\t{imp[i][1]:.2f}\n")
    return out
