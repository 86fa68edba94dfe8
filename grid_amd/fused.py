"""Device-resident chain of steps 4-7 with preallocated HBM buffers.

This is the same arithmetic as the drop-in step modules, without the text
files in between: the normalised matrix stays in HBM as exact hundredths
(int32, the step-4 output) plus the clipped bf16 panel that step 5 reads,
the neighbour lists feed the dipCN kernel directly, and the dipCN values
feed phasing.  ``bench.py`` and ``__graft_entry__.smoke()`` drive it.

Multi-GPU: the bin (column) axis is sharded in 8192-aligned ranges
(``shard_range``).  Exactness across shards rests on three facts:
  * row means: every rank computes 8192-block pairwise sums of its columns;
    the blocks are all-gathered and every rank runs the same sequential chain
    (padding blocks are exact zeros);
  * column statistics need no communication (sequential over all rows
    locally); medians/thresholds come from all-gathered ratio vectors;
  * the Gram matrix is an integer sum over bins: per-rank partials are
    combined with one all-reduce (int64 sum, order-free, exact).
``comm`` is None for one GPU, else a torch.distributed wrapper
(``TorchComm``).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _abi
from ._abi import BLOCK, call, ptr
from .engine import pad_to, py_index, qmax_for_zmax

F8, I4, I8, U2, U1 = np.float64, np.int32, np.int64, np.uint16, np.uint8


def shard_range(m: int, rank: int, world: int):
    """Column range [c0, c1) of ``rank``: whole 8192-blocks, balanced."""
    nblk = -(-m // BLOCK)
    b0 = (nblk * rank) // world
    b1 = (nblk * (rank + 1)) // world
    return min(b0 * BLOCK, m), min(b1 * BLOCK, m)


class TorchAlloc:
    """Device buffers as torch tensors (so torch.distributed can use them)."""

    def __init__(self, device_index: int):
        import torch
        self.torch = torch
        self.device = torch.device("cuda", device_index)
        self._dt = {np.dtype(F8): torch.float64, np.dtype(I4): torch.int32, np.dtype(I8): torch.int64,
                    np.dtype(U2): torch.int16, np.dtype(U1): torch.uint8}

    def empty(self, shape, dtype):
        return self.torch.empty(shape, dtype=self._dt[np.dtype(dtype)], device=self.device)

    def zero_(self, t):
        t.zero_()

    @staticmethod
    def numpy(t):
        a = t.cpu().numpy()
        return a.view(np.uint16) if a.dtype == np.int16 else a

    @staticmethod
    def read(t, i):
        return t.view(-1)[i].item()


class AbiAlloc:
    """Device buffers from libgridhip (no torch)."""

    def __init__(self, dev):
        self.dev = dev

    def empty(self, shape, dtype):
        return self.dev.alloc(shape, dtype)

    @staticmethod
    def zero_(b):
        b.zero()

    @staticmethod
    def numpy(b):
        return b.numpy()

    @staticmethod
    def read(b, i):
        out = np.empty(1, dtype=b.dtype)
        call("grid_d2h", b.dev.ctx, out.ctypes.data, b.ptr + i * b.dtype.itemsize, b.dtype.itemsize)
        return out[0].item()


class TorchComm:
    """The three collectives the sharded chain needs, over torch.distributed
    (backend "nccl" = RCCL over xGMI on MI355X, "gloo" on CPU)."""

    def __init__(self, dist):
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()

    def all_gather(self, t):
        import torch
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.dist.all_gather_into_tensor(out, t.contiguous())
        return out

    def all_reduce_sum(self, t):
        self.dist.all_reduce(t)
        return t

    def all_reduce_min(self, t):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return t


class Steps47:
    """One GPU's share of the steps 4-7 chain for an n x m cohort.

    Inputs (device): q [n][ld] int32 hundredths of this rank's columns,
    reads [n] f64 (read counts of every sample), the IBS hap-neighbour CSR of
    the cohort and its GS level schedule.
    """

    def __init__(self, dev, alloc, n, m_total, col0, m_local, *, k=10, n_nbr=300, top_frac=0.1, zmax=2.0,
                 sigma2_max=1000.0, frac_r=1.0, min_nbr=1, n_iters=100, comm=None):
        self.dev, self.A, self.comm = dev, alloc, comm
        self.rank = comm.rank if comm else 0
        self.world = comm.world if comm else 1
        self.n, self.m, self.col0, self.ml = n, m_total, col0, m_local
        assert col0 % BLOCK == 0
        self.k, self.n_nbr, self.top_frac = k, n_nbr, top_frac
        self.zmax, self.sigma2_max, self.frac_r = zmax, sigma2_max, frac_r
        self.min_nbr, self.n_iters = min_nbr, n_iters
        self.qmax = qmax_for_zmax(zmax)
        a = alloc
        n1 = max(n, 1)
        self.nblk_l = -(-m_local // BLOCK)
        self.nblk_max = max(-(-(shard_range(m_total, r, self.world)[1] - shard_range(m_total, r, self.world)[0])
                              // BLOCK) for r in range(self.world))
        self.bsum = a.empty((n1, max(self.nblk_l, 1)), F8)
        self.bcnt = a.empty((n1, max(self.nblk_l, 1)), I4)
        if self.world > 1:
            self.bsum_pad = a.empty((n1, max(self.nblk_max, 1)), F8)
            self.bcnt_pad = a.empty((n1, max(self.nblk_max, 1)), I4)
        self.rm = a.empty(n1, F8)
        ml1 = max(m_local, 1)
        self.mlmax = max(shard_range(m_total, r, self.world)[1] - shard_range(m_total, r, self.world)[0]
                         for r in range(self.world))
        self.mu, self.var = a.empty(ml1, F8), a.empty(ml1, F8)
        self.ratio = a.empty(max(self.mlmax, 1), F8)
        self.ratio_all = a.empty(max(self.mlmax * self.world, 1), F8)
        self.sorted = a.empty(max(self.mlmax * self.world, 1), F8)
        self.sel = a.empty(ml1, I4)
        self.r3 = a.empty(max(self.mlmax, 1), F8)
        self.colmap = a.empty(ml1, I4)
        self.zq = a.empty((n1, ml1), I4)                       # step-4 output: exact hundredths
        self.np_ = pad_to(n1, 128)
        self.kpad = pad_to(ml1, 64)
        self.zb = a.empty((self.np_, self.kpad), U2)          # step-5 input panel (bf16)
        a.zero_(self.zb)                                       # pad rows/cols stay zero
        self.gram = a.empty((self.np_, self.np_), I8)
        kk = max(k, 1)
        self.rows_per = -(-n // self.world)
        self.idx_l = a.empty((self.rows_per, kk), I4)
        self.d2_l = a.empty((self.rows_per, kk), I8)
        self.cnt_l = a.empty(self.rows_per, I4)
        self.idx = a.empty((n1, kk), I4)
        self.d2 = a.empty((n1, kk), I8)
        self.cnt = a.empty(n1, I4)
        self.scale2 = a.empty(n1, F8)
        self.nscale = a.empty((n1, kk), F8)
        self.dip = a.empty(n1, F8)
        self.valid = a.empty(n1, U1)
        self.hap = a.empty(2 * n1, F8)
        self.imp = a.empty(2 * n1, F8)
        self.mean = a.empty(1, F8)
        self.zerodiv = C.c_int32()
        self.events = None

    # ------------------------------------------------------------------
    def set_phasing_graph(self, off, nbr, w):
        order, loff, nl = _abi.hi_levels(off, nbr)
        up = lambda x, dt: self._upload(np.ascontiguousarray(x, dtype=dt))  # noqa: E731
        self.off, self.nbr, self.w = up(off, I8), up(nbr if nbr.size else np.zeros(1), I4), \
            up(w if w.size else np.zeros(1), F8)
        self.order, self.loff, self.nlev = up(order, I4), up(loff, I4), nl

    def set_reads(self, reads):
        self.reads = self._upload(np.ascontiguousarray(reads, dtype=F8))
        self.has = self._upload(np.ones(max(self.n, 1), dtype=U1))

    def _upload(self, arr):
        b = self.A.empty(arr.shape, arr.dtype)
        if hasattr(b, "copy_"):
            import torch
            src = torch.from_numpy(arr.view(np.int16) if arr.dtype == np.uint16 else arr)
            b.copy_(src)
        else:
            b.copy_from(arr)
        return b

    def _read(self, b, i):
        return self.A.read(b, i)

    def _gather_padded(self, b, count, maxcount, fill):
        """All-gather the first ``count`` entries of a 1-D f64 buffer from
        every rank (padded with ``fill``); returns (buffer, total length)."""
        if self.comm is None:
            return b, count
        import torch
        if count < maxcount:
            b.view(-1)[count:maxcount].fill_(fill)
        g = self.comm.all_gather(b.view(-1)[:maxcount])
        return g.view(-1), self.world * maxcount

    # ------------------------------------------------------------------
    def _mark(self, name):
        if self.marks is not None:
            import torch
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append((name, e))

    def stage_ms(self):
        """Per-stage device time of the last run(profile=True) (ms)."""
        out = {}
        for (_, a), (name, b) in zip(self.marks, self.marks[1:]):
            out[name] = out.get(name, 0.0) + a.elapsed_time(b)
        return out

    def run(self, q, ld, gram_events=None, profile=False):
        """One pass of steps 4-7.  ``q``: device pointer/buffer [n][ld] int32.
        ``gram_events``: optional (start, end) torch.cuda.Event pair recorded
        around the Gram kernel (same stream as every kernel here)."""
        d, ctx, n, ml = self.dev, self.dev.ctx, self.n, self.ml
        ev = gram_events
        self.marks = [] if profile else None
        self._mark("start")
        # ---- step 4: row means (8192-block pairwise partials, gathered) ----
        call("grid_norm_row_blocks", ctx, ptr(q), n, ml, ld, ptr(self.bsum), ptr(self.bcnt))
        nblk_tot = self.nblk_l
        bsum, bcnt = self.bsum, self.bcnt
        if self.comm is not None:
            import torch
            self.bsum_pad.zero_()
            self.bcnt_pad.zero_()
            self.bsum_pad[:, : self.nblk_l].copy_(self.bsum)
            self.bcnt_pad[:, : self.nblk_l].copy_(self.bcnt)
            gs = self.comm.all_gather(self.bsum_pad)        # [world][n][nblk_max]
            gc = self.comm.all_gather(self.bcnt_pad)
            bsum = gs.permute(1, 0, 2).contiguous()
            bcnt = gc.permute(1, 0, 2).contiguous()
            nblk_tot = self.world * self.nblk_max
        call("grid_norm_row_means", ctx, ptr(bsum), ptr(bcnt), n, nblk_tot, ptr(self.rm))
        self._mark("row_means")
        # ---- column statistics (local, exact) ----
        call("grid_norm_col_means", ctx, ptr(q), n, ml, ld, ptr(self.rm), ptr(self.mu))
        call("grid_norm_col_vars", ctx, ptr(q), n, ml, ld, ptr(self.rm), ptr(self.mu), ptr(self.var),
             ptr(self.ratio))
        self._mark("col_stats")
        rall, rlen = self._gather_padded(self.ratio, ml, self.mlmax, float("nan"))
        nv = C.c_int64()
        call("grid_sort_valid", ctx, ptr(rall), rlen, ptr(self.sorted), C.byref(nv))
        nvalid = nv.value
        scale = 1.0
        if nvalid:
            if nvalid % 2:
                med = self._read(self.sorted, nvalid // 2)
            else:
                med = (self._read(self.sorted, nvalid // 2 - 1) + self._read(self.sorted, nvalid // 2)) / 2.0
            if med > 0:
                scale = 1.0 / math.sqrt(med / 100.0)
            thr = self._read(self.sorted, py_index(nvalid, int(self.top_frac * nvalid)))
            cnt = C.c_int64()
            call("grid_select_gt", ctx, ptr(self.ratio), ml, thr, ptr(self.sel), C.byref(cnt))
            r_loc = cnt.value
        else:
            r_loc = 0
        self.scale, self.r_loc = scale, r_loc
        # ---- step 5 region filter on the "%.3f" ratios (find_neighbors.py:148-171) ----
        call("grid_gather_f64", ctx, ptr(self.ratio), ptr(self.sel), r_loc, ptr(self.r3))
        call("grid_round_decimals", ctx, ptr(self.r3), r_loc, 3, ptr(self.r3))
        r3all, r3len = self._gather_padded(self.r3, r_loc, self.mlmax, float("nan"))
        r_tot = r_loc if self.comm is None else self._sum_int(r_loc)
        call("grid_sort_valid", ctx, ptr(r3all), r3len, ptr(self.sorted), C.byref(nv))
        if nv.value:
            smin = self._read(self.sorted, min(int(r_tot * (1.0 - self.frac_r)), nv.value - 1))
            smax = float(self.sigma2_max)
        else:
            smin, smax = -math.inf, math.inf
        ruse = C.c_int64()
        call("grid_colmap_range", ctx, ptr(self.r3), r_loc, smin, smax, ptr(self.colmap), C.byref(ruse))
        self.ruse_loc = ruse.value
        self._mark("select_sort")
        # ---- z-scores: exact hundredths (step-4 output) + clipped bf16 panel ----
        of = C.c_int32()
        call("grid_norm_zquant", ctx, ptr(q), n, ld, ptr(self.sel), r_loc, ptr(self.rm), ptr(self.mu), scale,
             ptr(self.zq), max(ml, 1), ptr(self.colmap), self.qmax, ptr(self.zb), self.kpad, C.byref(of))
        if of.value:
            raise _abi.GridNativeError("z-score outside the int32 hundredths range")
        self._mark("zquant")
        # ---- step 5: exact Gram (MFMA) -> all-reduce -> top-k ----
        self.A.zero_(self.gram)
        kpad_used = pad_to(max(self.ruse_loc, 1), 64)
        if kpad_used > self.ruse_loc and n > 0:
            self.zb[:n, self.ruse_loc:kpad_used].zero_()      # columns colmap did not write this pass
        if ev:
            ev[0].record()
        call("grid_knn_gram", ctx, ptr(self.zb), self.np_, kpad_used, self.kpad, self.qmax, ptr(self.gram))
        if ev:
            ev[1].record()
        self._mark("gram")
        if self.comm is not None:
            self.comm.all_reduce_sum(self.gram)
            self._mark("allreduce")
        r0 = min(self.rank * self.rows_per, n)
        nr = max(min(n - r0, self.rows_per), 0)
        call("grid_knn_topk", ctx, ptr(self.gram), n, self.np_, self.k, r0, nr, ptr(self.idx_l), ptr(self.d2_l),
             ptr(self.cnt_l))
        if self.comm is not None:
            gi = self.comm.all_gather(self.idx_l).view(-1, max(self.k, 1))[:n]
            gd = self.comm.all_gather(self.d2_l).view(-1, max(self.k, 1))[:n]
            gc = self.comm.all_gather(self.cnt_l).view(-1)[:n]
            self.idx[:n].copy_(gi)
            self.d2[:n].copy_(gd)
            self.cnt[:n].copy_(gc)
            idx, cntb = self.idx, self.cnt
        else:
            idx, cntb = self.idx_l, self.cnt_l
        self._mark("topk")
        # ---- step 6: dipCN (scales as printed "%.2f", neighbour gather) ----
        call("grid_round_decimals", ctx, ptr(self.rm), n, 2, ptr(self.scale2))
        call("grid_gather_f64", ctx, ptr(self.scale2), ptr(idx), n * max(self.k, 1), ptr(self.nscale))
        call("grid_dipcn", ctx, n, ptr(self.reads), ptr(self.has), ptr(self.scale2), ptr(idx), ptr(self.nscale),
             ptr(cntb), max(self.k, 1), self.n_nbr, ptr(self.dip), ptr(self.valid), C.byref(self.zerodiv))
        if self.zerodiv.value:
            raise ZeroDivisionError("float division by zero")
        self._mark("dipcn")
        # ---- step 7: level-scheduled Gauss-Seidel phasing + imputation ----
        call("grid_hi_phase", ctx, n, ptr(self.dip), ptr(self.off), ptr(self.nbr), ptr(self.w), self.min_nbr,
             self.n_iters, ptr(self.order), ptr(self.loff), self.nlev, ptr(self.hap), ptr(self.imp), ptr(self.mean))
        self._mark("phase")
        self.idx_out, self.cnt_out = idx, cntb

    def _sum_int(self, v):
        import torch
        t = torch.tensor([v], dtype=torch.int64, device=self.gram.device)
        self.comm.all_reduce_sum(t)
        return int(t.item())
