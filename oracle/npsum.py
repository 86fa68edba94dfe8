"""Exact restatement of NumPy 2.2's float64 add-reductions used by the
reference's ``np.nanmean`` / ``np.nansum`` calls (TEST INFRASTRUCTURE ONLY).

Row reductions (``axis=1`` on a C-contiguous matrix,
normalize_mosdepth.py:120, :440) go through the buffered reduce loop: the row
is cut into chunks of the 8192-element iterator buffer and the running
output is updated ``acc = acc + pairwise(chunk)`` (numpy
``loops_utils.h.src`` pairwise_sum, PW_BLOCKSIZE = 128, 8 partial sums).

Column reductions (``axis=0``, normalize_mosdepth.py:445-446) are a plain
sequential ``out += row`` over the rows in order.

All functions are vectorised over the *other* axis so the per-element IEEE
operation sequence is exactly the scalar one.
"""
import numpy as np

BUFSIZE = 8192      # numpy NPY_BUFSIZE
PW_BLOCK = 128      # numpy PW_BLOCKSIZE


def pairwise_cols(a: np.ndarray, lo: int, n: int) -> np.ndarray:
    """pairwise_sum of a[:, lo:lo+n] for every row at once (returns shape (rows,))."""
    if n < 8:
        res = np.zeros(a.shape[0], dtype=np.float64)
        for i in range(n):
            res = res + a[:, lo + i]
        return res
    if n <= PW_BLOCK:
        r = [a[:, lo + j].copy() for j in range(8)]
        i = 8
        stop = n - (n % 8)
        while i < stop:
            for j in range(8):
                r[j] = r[j] + a[:, lo + i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res = res + a[:, lo + i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return pairwise_cols(a, lo, n2) + pairwise_cols(a, lo + n2, n - n2)


def row_sum(a: np.ndarray) -> np.ndarray:
    """np.add.reduce(a, axis=1) for a C-contiguous float64 matrix."""
    a = np.asarray(a, dtype=np.float64)
    acc = np.zeros(a.shape[0], dtype=np.float64)
    m = a.shape[1]
    for lo in range(0, m, BUFSIZE):
        acc = acc + pairwise_cols(a, lo, min(BUFSIZE, m - lo))
    return acc


def row_block_sums(a: np.ndarray):
    """Per-row list of 8192-block pairwise sums (the device's first stage)."""
    a = np.asarray(a, dtype=np.float64)
    m = a.shape[1]
    return [pairwise_cols(a, lo, min(BUFSIZE, m - lo)) for lo in range(0, m, BUFSIZE)]


def col_sum(a: np.ndarray) -> np.ndarray:
    """np.add.reduce(a, axis=0): sequential over rows."""
    a = np.asarray(a, dtype=np.float64)
    acc = np.zeros(a.shape[1], dtype=np.float64)
    for i in range(a.shape[0]):
        acc = acc + a[i]
    return acc


def nanmean_rows(a: np.ndarray) -> np.ndarray:
    """np.nanmean(a, axis=1) (numpy nanfunctions: NaN->0, sum, / count)."""
    mask = np.isnan(a)
    b = np.where(mask, 0.0, a)
    cnt = (~mask).sum(axis=1)
    with np.errstate(invalid="ignore", divide="ignore"):
        return row_sum(b) / cnt.astype(np.float64)


def nanmean_cols(a: np.ndarray) -> np.ndarray:
    mask = np.isnan(a)
    b = np.where(mask, 0.0, a)
    cnt = (~mask).sum(axis=0)
    with np.errstate(invalid="ignore", divide="ignore"):
        return col_sum(b) / cnt.astype(np.float64)


def nansum_cols(a: np.ndarray) -> np.ndarray:
    return col_sum(np.where(np.isnan(a), 0.0, a))
