"""Property checks of the streamed steps 4-7 chain at the BASELINE shapes
(configs 3-4: 50,000 samples x 3M / 30M bins), where the oracle cannot run
the whole cohort.  Used by tests/test_gpu_configs.py (MI355X only).

What is checked, and against what (reference arithmetic in brackets):

* every chunk's step-4 output and bf16 panel, cell by cell, against an
  independent IEEE fp64 recomputation on the device (``grid_verify_zquant``),
  plus a sample of the int16 escapes (|z| > 327.65) against Python's "%.2f"
  [normalize_mosdepth.py:456-476, :553];
* the 8192-block row partial sums of sampled blocks, for EVERY row, against
  the oracle's restatement of NumPy's pairwise sum (oracle/npsum.py), and
  every row mean as the oracle's sequential chain over those blocks
  [normalize_mosdepth.py:440];
* column means / variances / ratios of sampled column windows against the
  oracle's sequential axis-0 sums [:445-451];
* the median scale, the top-frac selection, the "%.3f" sigma^2 filter and the
  panel column map against NumPy on the device's ratio vector [:462-499;
  find_neighbors.py:128-175];
* the neighbours and d^2 of sampled query rows against an fp64 product of
  the panel accumulated chunk by chunk (exact: integer sums < 2^53), ordered
  by (d^2, index) [find_neighbors.py:207-213];
* dipCN of every sample and phasing (a few sweeps) against the oracle given
  the chain's neighbours [compute_dipcn.py:62-88, hi_inference.py:175-226].
"""
from __future__ import annotations

import ctypes as C
import math
import os
import sys
import time

import numpy as np
import torch

from grid_amd import _abi
from oracle import npsum, steps

NUM_ESC_SAMPLE = 2000


def log(msg):
    """Progress lines for long GPU runs (stderr is not captured with -s)."""
    print(f"[bigcheck {time.strftime('%H:%M:%S')}] {msg}", file=sys.__stderr__, flush=True)


def fmt_code(z):
    t = f"{z:.2f}"
    k = int(t.replace(".", ""))
    return _abi.ZQ_NEG0 if (k == 0 and t.startswith("-")) else k


class ChunkChecker:
    """on_z_chunk consumer: verifies each chunk while its buffers are live and
    accumulates the fp64 Gram rows of the sampled queries."""

    def __init__(self, dev, st, n, rows, slice_cols=8192):
        self.dev, self.st, self.n = dev, st, n
        self.rows = torch.as_tensor(rows, dtype=torch.int64, device="cuda")
        self.G = torch.zeros((len(rows), n), dtype=torch.float64, device="cuda")
        self.nrm = torch.zeros(n, dtype=torch.float64, device="cuda")
        self.slice = slice_cols
        self.bad = [0, 0]
        self.cells = 0
        self.esc_checked = 0
        self.chunks = 0

    def __call__(self, zq16, ld, s0, s1, esc_idx, esc_val):
        st, n, c = self.st, self.n, self.st.cur
        r = s1 - s0
        counts = (C.c_int64 * 3)()
        mu_c = st.mu[c["a"]:c["b"]]
        _abi.call("grid_verify_zquant", self.dev.ctx, c["q"].data_ptr(), n, c["ld"], c["sel"].data_ptr(), r,
                  st.rm.data_ptr(), mu_c.data_ptr(), st.scale, zq16.data_ptr(), ld, c["colmap"].data_ptr(),
                  st.qmax, st.zb.data_ptr(), st.np_, counts)
        self.bad[0] += counts[0]
        self.bad[1] += counts[1]
        self.cells += n * r
        self._escapes(zq16, ld, esc_idx, esc_val, mu_c)
        self._gram(c["used"])
        self.chunks += 1
        if self.chunks % 8 == 1:
            log(f"chunk {c['ci']}: {r} selected columns, {esc_idx.numel()} escapes, mismatches {self.bad}")

    def _escapes(self, zq16, ld, esc_idx, esc_val, mu_c):
        ne = esc_idx.numel()
        if ne == 0:
            return
        st, c = self.st, self.st.cur
        pick = torch.linspace(0, ne - 1, min(ne, NUM_ESC_SAMPLE), device="cuda").round().long().unique()
        ei, ev = esc_idx[pick], esc_val[pick]
        row, s = ei // ld, ei % ld
        j = c["sel"].long()[s]
        qv = c["q"].view(-1)[row * c["ld"] + j]
        code = zq16.view(-1)[ei]
        rm, mu = st.rm[row], mu_c[j]
        qv, code, rm, mu, ev, row, s = (t.cpu().numpy() for t in (qv, code, rm, mu, ev, row, s))
        for t in range(len(qv)):
            x = int(qv[t]) / 100.0
            m = float(mu[t])
            z = ((x / float(rm[t]) - m) / math.sqrt(m)) * st.scale
            assert int(code[t]) == _abi.ZQ16_ESC, ("escape slot", int(row[t]), int(s[t]))
            assert int(ev[t]) == fmt_code(z), ("escape value", int(row[t]), int(s[t]), z)
        self.esc_checked += len(pick)

    def _gram(self, used):
        st, n, kbw = self.st, self.n, _abi.KBW
        for k0 in range(0, used, self.slice):
            k1 = min(used, k0 + self.slice)
            blk = st.zb[k0 // kbw: -(-k1 // kbw)]                       # [s][np][32]
            p = blk.permute(1, 0, 2)[:n].reshape(n, -1)[:, : k1 - k0]
            pf = p.view(torch.bfloat16).to(torch.float64)
            del p
            self.G += pf[self.rows] @ pf.T
            self.nrm += pf.square().sum(1)
            del pf


def check_knn(ck, st, n, k):
    """Sampled queries: neighbours and d^2 from the fp64 product."""
    rows = ck.rows
    d2 = (ck.nrm[rows][:, None] + ck.nrm[None, :] - 2.0 * ck.G).round().to(torch.int64)
    assert bool((d2 >= 0).all())
    key = d2 * (1 << 17) + torch.arange(n, device="cuda")[None, :]
    key[torch.arange(len(rows), device="cuda"), rows] = torch.iinfo(torch.int64).max     # self dropped
    top = torch.topk(key, k, dim=1, largest=False).values
    got_idx = st.idx_out[rows].to(torch.int64)
    got_d2 = st.d2[rows]
    assert torch.equal(got_idx, top % (1 << 17)), "neighbour indices"
    assert torch.equal(got_d2, top // (1 << 17)), "neighbour d2"


def synth_slab(dev, seed, n, c0, w, ncl):
    q = torch.empty((n, w), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, seed, n, w, w, c0, ncl, q.data_ptr())
    return q.cpu().numpy()


def as_float(q):
    return np.where(q == _abi.MISSING, np.nan, q / 100.0)


def check_row_means(dev, st, seed, n, m, ncl, blocks):
    """Sampled blocks' partial sums for every row vs the oracle's pairwise sum;
    every row mean as the sequential chain over the device's block sums."""
    bsum = st.bsum[:n].cpu().numpy()
    bcnt = st.bcnt[:n].cpu().numpy()
    for b in blocks:
        c0 = b * _abi.BLOCK
        w = min(_abi.BLOCK, m - c0)
        q = torch.empty((n, w), dtype=torch.int32, device="cuda")
        _abi.call("grid_synth_depth", dev.ctx, seed, n, w, w, c0, ncl, q.data_ptr())
        # nanmean's operand np.where(isnan(a), 0, a) with a = q / 100.0, built
        # column-major: the int32 transpose is made on the device (so the
        # oracle's column walks read contiguous memory), the division by NumPy
        # (torch divides by a scalar as a multiply by its reciprocal: not IEEE /)
        qt = q.t().contiguous().cpu().numpy()
        del q
        miss = qt == _abi.MISSING
        z0 = np.where(miss, 0.0, qt / 100.0).T
        cnt = (~miss).sum(axis=0)
        del qt, miss
        exp = npsum.pairwise_cols(z0, 0, w)
        assert np.array_equal(bsum[:, b], exp), f"row block sums, block {b}"
        assert np.array_equal(bcnt[:, b], cnt), f"row block counts, block {b}"
    acc = np.zeros(n)
    for b in range(bsum.shape[1]):
        acc = acc + bsum[:, b]
    with np.errstate(invalid="ignore", divide="ignore"):
        rm = acc / bcnt.sum(axis=1).astype(np.float64)
    assert np.array_equal(st.rm[:n].cpu().numpy(), rm, equal_nan=True), "row means"
    return rm


def check_col_stats(dev, st, seed, n, ncl, rm, windows, w=2048):
    mu_d, var_d, ratio_d = st.mu.cpu().numpy(), st.var.cpu().numpy(), st.ratio.cpu().numpy()
    rms = np.where(rm == 0, np.nan, rm)
    for c0 in windows:
        mat = as_float(synth_slab(dev, seed, n, c0, w, ncl)) / rms[:, None]
        with np.errstate(invalid="ignore", divide="ignore"):
            mu = npsum.nanmean_cols(mat)
            d = mat - mu[None, :]
            var = npsum.nansum_cols(d * d) / (n - 1)
            ratio = np.where(mu > 0, (100.0 * var) / mu, np.nan)
        sl = slice(c0, c0 + w)
        assert np.array_equal(mu_d[sl], mu, equal_nan=True), f"column means at {c0}"
        assert np.array_equal(var_d[sl], var, equal_nan=True), f"column variances at {c0}"
        assert np.array_equal(ratio_d[sl], ratio, equal_nan=True), f"ratios at {c0}"


def check_selection(st, m, top_frac=0.1, sigma2_max=1000.0, fmt_all=True):
    ratio = st.ratio[:m].cpu().numpy()
    valid = np.sort(ratio[~np.isnan(ratio)])
    nv = len(valid)
    med = valid[nv // 2] if nv % 2 else (valid[nv // 2 - 1] + valid[nv // 2]) / 2.0
    scale = 1.0 / math.sqrt(med / 100.0) if med > 0 else 1.0
    assert st.scale == scale, "median scale"
    thr = valid[int(top_frac * nv)]
    with np.errstate(invalid="ignore"):
        sel = np.nonzero(ratio > thr)[0]
    assert st.r_loc == len(sel), "selected count"
    assert np.array_equal(st.sel[: st.r_loc].cpu().numpy(), sel), "selection"
    # step 5 reads the ratios as printed with "%.3f"
    r3 = st.r3[: st.r_loc].cpu().numpy()
    rs = ratio[sel]
    pick = np.arange(len(sel)) if fmt_all else np.unique(np.linspace(0, len(sel) - 1, 200_000).astype(np.int64))
    exp3 = np.array([float(f"{v:.3f}") for v in rs[pick]])
    assert np.array_equal(r3[pick], exp3), "%.3f ratios"
    idx, ruse = steps.filter_regions_by_variance(r3, 1.0, sigma2_max)
    assert st.ruse_loc == ruse, "R_use"
    cm = np.full(len(sel), -1, dtype=np.int64)
    cm[idx] = np.arange(ruse)
    assert np.array_equal(st.colmap[: st.r_loc].cpu().numpy(), cm), "panel column map"


def check_dipcn_phasing(st, n, k, n_nbr, reads, off, nbr, iters):
    ids = [f"S{i:06d}" for i in range(n)]
    sc = {ids[i]: float(v) for i, v in enumerate(st.scale2[:n].cpu().numpy())}
    rmv = st.rm[:n].cpu().numpy()
    assert all(sc[ids[i]] == float(f"{rmv[i]:.2f}") for i in range(0, n, 97)), "printed scales"
    idx = st.idx_out[:n].cpu().numpy()
    cnt = st.cnt_out[:n].cpu().numpy()
    nbrs = {ids[i]: [(ids[j], sc[ids[j]]) for j in idx[i, : cnt[i]]] for i in range(n)}
    dip = steps.dipcn(nbrs, sc, {ids[i]: float(reads[i]) for i in range(n)}, n_nbr)
    assert len(dip) == n
    assert np.array_equal(st.dip[:n].cpu().numpy(), np.array([v for _, v in dip])), "dipCN"
    hn = [[(int(nbr[t]), 1.0) for t in range(off[h], off[h + 1])] for h in range(2 * n)]
    hap, _ = steps.run_phasing([v for _, v in dip], hn, 1, iters)
    assert np.array_equal(st.hap[: 2 * n].cpu().numpy(), np.array(hap), equal_nan=True), "phasing"


def run(n, m, *, k=10, n_iters=3, n_rows=128, n_blocks=4, n_windows=4, budget_gb=200.0, full_rows=0,
        fmt_all=True):
    """The streamed chain at n x m (bench.py's cohort, its chunk plan), every
    check above.  Returns a summary dict."""
    from grid_amd.fused import HipOps, Steps47, SynthSource
    from grid_amd.fused import TorchAlloc
    import bench
    t0 = time.perf_counter()
    dev = _abi.Device(0)
    dev.set_stream(torch.cuda.current_stream())
    ops = HipOps(dev)
    chunk, _ = bench.plan_memory(n, m, 1, budget_gb * 1e9)
    assert chunk is not None and chunk < m, "the shape must stream"
    reads, off, nbr, w = bench.synth_reads_and_ibs(n)
    st = Steps47(ops, TorchAlloc(0), n, m, 0, m, k=k, n_nbr=300, top_frac=0.1, zmax=2.0, sigma2_max=1000.0,
                 frac_r=1.0, min_nbr=1, n_iters=n_iters, chunk=chunk, keep_z=False)
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)
    rng = np.random.default_rng(n ^ m)
    rows = np.sort(rng.choice(n, n_rows, replace=False))
    rows[0], rows[-1] = 0, n - 1
    ck = ChunkChecker(dev, st, n, rows)
    st.on_z_chunk = ck
    log(f"{n} x {m}: {st.nch} chunks of {chunk} bins; setup {time.perf_counter() - t0:.1f}s")
    t1 = time.perf_counter()
    st.run(SynthSource(ops, bench.SEED, n, 0, bench.NCL), None)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    log(f"chain + per-chunk checks {t2 - t1:.1f}s; cells {ck.cells}, mismatches {ck.bad}, "
        f"escapes checked {ck.esc_checked}")
    assert ck.chunks == st.nch
    assert ck.bad == [0, 0], ck.bad
    assert ck.cells == n * st.r_loc
    check_knn(ck, st, n, k)
    log("k-NN rows ok")
    nblk = -(-m // _abi.BLOCK)
    blocks = sorted({0, nblk - 1, *rng.choice(nblk, n_blocks - 2, replace=False).tolist()})
    rm = check_row_means(dev, st, bench.SEED, n, m, bench.NCL, blocks)
    log(f"row means ok (blocks {blocks})")
    if full_rows:
        q = torch.empty((full_rows, m), dtype=torch.int32, device="cuda")
        _abi.call("grid_synth_depth", dev.ctx, bench.SEED, full_rows, m, m, 0, bench.NCL, q.data_ptr())
        assert np.array_equal(npsum.nanmean_rows(as_float(q.cpu().numpy())), rm[:full_rows]), "whole rows"
        del q
    windows = sorted({0, m - 2048, *(rng.choice((m - 2048) // 64, n_windows) * 64).tolist()})
    check_col_stats(dev, st, bench.SEED, n, bench.NCL, rm, windows)
    log("column statistics ok")
    check_selection(st, m, fmt_all=fmt_all)
    log(f"selection ok: R={st.r_loc}, R_use={st.ruse_loc}")
    check_dipcn_phasing(st, n, k, 300, reads, off, nbr, n_iters)
    log(f"dipCN + phasing ok; total {time.perf_counter() - t0:.1f}s")
    res = {"n": n, "m": m, "chunks": st.nch, "chunk": chunk, "R": st.r_loc, "R_use": st.ruse_loc,
           "cells_verified": ck.cells, "escapes_checked": ck.esc_checked, "query_rows": len(rows),
           "chain_s": t2 - t1, "total_s": time.perf_counter() - t0}
    st.on_z_chunk = None                 # st <-> ck cycle: free the ~200 GB of chunk buffers now
    del ck, st
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    import json
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    n, m = int(sys.argv[1]), int(sys.argv[2])
    print(json.dumps(run(n, m, full_rows=2 if m <= 3_000_000 else 0, fmt_all=m <= 3_000_000)), flush=True)
