"""CPU restatement of ``grid_amd.fused.HipOps`` for tests (uses the oracle's
arithmetic on CPU torch tensors).  Lets the sharded chain (fused.Steps47)
run under torch.distributed/gloo without a GPU, so the sharding logic --
8192-aligned shards, padded all-gathers, global thresholds, the Gram
all-reduce -- is checked on CPU.  TEST INFRASTRUCTURE ONLY."""
import math

import numpy as np

from oracle import steps
from oracle.npsum import col_sum, row_block_sums

KBW = 32   # K-block width of the k-NN panel (grid_amd._abi.KBW; this module runs without the library)

MISSING = -(2 ** 31)
NEG0 = -(2 ** 31) + 1


def _np(t):
    return t.numpy()


def _hundredths(z):
    """f"{v:.2f}" of every cell as int64 hundredths (NaN -> MISSING, a
    negative value printing as "-0.00" -> NEG0).  rint(v * 100) is the
    correctly rounded decimal unless the exact product lies within an ulp of a
    half (|v * 100| < 2^31 here, an ulp < 2^-21): those cells -- and only
    those -- are printed by Python's formatter."""
    with np.errstate(invalid="ignore"):
        t = z * 100.0
        k = np.rint(t)
        near = np.abs(np.abs(t - np.trunc(t)) - 0.5) < 1e-6
    out = np.where(np.isnan(z), MISSING, k).astype(np.int64)
    for i, s in zip(*np.nonzero(near & ~np.isnan(z))):
        out[i, s] = int(f"{z[i, s]:.2f}".replace(".", ""))
    out[(out == 0) & np.signbit(z) & ~np.isnan(z)] = NEG0
    return out


class NumpyOps:
    @staticmethod
    def _mat(q, n, m, ld):
        """[n][m] view of a matrix buffer with row stride ld (2-D or flat)."""
        a = _np(q).reshape(-1)
        return a[: (n - 1) * ld + m].reshape(-1)[np.arange(n)[:, None] * ld + np.arange(m)[None, :]] if n else \
            np.zeros((0, m), a.dtype)

    def row_blocks(self, q, n, m, ld, bsum, bcnt):
        qa = self._mat(q, n, m, ld)
        x = np.where(qa == MISSING, 0.0, qa / 100.0)
        nblk = -(-m // 8192)
        bs = _np(bsum).reshape(-1)[: n * nblk].reshape(n, nblk)     # kernel layout: [n][ceil(m/8192)]
        bc = _np(bcnt).reshape(-1)[: n * nblk].reshape(n, nblk)
        for b, s in enumerate(row_block_sums(x)):
            bs[:, b] = s
            bc[:, b] = (qa[:, b * 8192:(b + 1) * 8192] != MISSING).sum(axis=1)

    def row_means(self, bsum, bcnt, n, nblk, rm):
        bs, bc = _np(bsum)[:n, :nblk], _np(bcnt)[:n, :nblk]
        acc = np.zeros(n)
        for b in range(nblk):
            acc = acc + bs[:, b]
        with np.errstate(all="ignore"):
            _np(rm)[:n] = acc / bc.sum(axis=1).astype(np.float64)

    def _y(self, q, n, m, ld, rm):
        qa = self._mat(q, n, m, ld)
        r = _np(rm)[:n]
        rs = np.where(r == 0, np.nan, r)
        with np.errstate(all="ignore"):
            return np.where(qa == MISSING, np.nan, (qa / 100.0) / rs[:, None])

    def col_means(self, q, n, m, ld, rm, mu):
        y = self._y(q, n, m, ld, rm)
        with np.errstate(all="ignore"):
            _np(mu)[:m] = col_sum(np.nan_to_num(y, nan=0.0)) / (~np.isnan(y)).sum(axis=0)

    def col_vars(self, q, n, m, ld, rm, mu, var, ratio):
        y = self._y(q, n, m, ld, rm)
        mj = _np(mu)[:m]
        with np.errstate(all="ignore"):
            d = y - mj[None, :]
            v = col_sum(np.nan_to_num(d * d, nan=0.0)) / (n - 1)
            _np(var)[:m] = v
            _np(ratio)[:m] = np.where(mj > 0, (100.0 * v) / mj, np.nan)

    def count_valid(self, v, n):
        a = _np(v).reshape(-1)[:n]
        return int((~np.isnan(a)).sum())

    def select_kth(self, v, n, ks):
        # grid_select_kth's order: keys with every bit flipped for negatives, the sign bit otherwise
        a = _np(v).reshape(-1)[:n]
        u = a[~np.isnan(a)].view(np.uint64)
        neg = (u >> np.uint64(63)).astype(bool)
        key = np.sort(np.where(neg, ~u, u | np.uint64(1 << 63)))
        out = []
        for k in ks:
            kk = key[k]
            uu = kk & np.uint64((1 << 63) - 1) if kk >> np.uint64(63) else ~kk
            out.append(float(np.array([uu], dtype=np.uint64).view(np.float64)[0]))
        return out

    def sort_valid(self, v, n, out):
        a = _np(v).reshape(-1)[:n]
        s = np.sort(a[~np.isnan(a)])
        _np(out).reshape(-1)[: len(s)] = s
        return len(s)

    def select_gt(self, v, n, thr, idx):
        a = _np(v).reshape(-1)[:n]
        with np.errstate(invalid="ignore"):
            sel = np.where(a > thr)[0]
        _np(idx)[: len(sel)] = sel
        return len(sel)

    def gather(self, v, idx, n, out):
        src = _np(v).reshape(-1)
        ix = _np(idx).reshape(-1)[:n]
        _np(out).reshape(-1)[:n] = np.where(ix >= 0, src[np.clip(ix, 0, None)], np.nan)

    def round_decimals(self, v, n, dec, out):
        a = _np(v).reshape(-1)[:n].copy()
        _np(out).reshape(-1)[:n] = [x if (math.isnan(x) or math.isinf(x)) else float(f"{x:.{dec}f}") for x in a]

    def colmap_range(self, r, n, smin, smax, colmap):
        a = _np(r).reshape(-1)[:n]
        keep = np.isfinite(a) & (a >= smin) & (a <= smax)
        cm = np.cumsum(keep) - 1
        _np(colmap)[:n] = np.where(keep, cm, -1)
        return int(keep.sum())

    # grid_sel_stage1 / _stage2 / _read: the device-resident pass C on a state
    # tensor of GRID_SEL_STATE int64 slots (doubles as bits)
    @staticmethod
    def _setf(st, k, x):
        _np(st)[k] = np.array([x], np.float64).view(np.int64)[0]

    def sel_stage1(self, rall, rlen, ratio, ml, len_pad, top_frac, sel, r3, st):
        a = _np(st)
        a[:] = 0
        nvalid = self.count_valid(rall, rlen) if rlen else 0
        a[0] = nvalid
        if nvalid:
            ks = [nvalid // 2, nvalid // 2] if nvalid % 2 else [nvalid // 2 - 1, nvalid // 2]
            t = int(top_frac * nvalid)
            t = t + nvalid if t < 0 else t
            if not 0 <= t < nvalid:
                a[5], t = 1, 0
            vals = self.select_kth(rall, rlen, ks + [t])
            for j in range(3):
                self._setf(st, 9 + j, vals[j])
            self._setf(st, 8, vals[2])
        else:
            self._setf(st, 8, float("nan"))
        r_loc = self.select_gt(ratio, ml, float(np.array([a[8]]).view(np.float64)[0]), sel) if ml else 0
        a[1] = a[2] = r_loc
        if len_pad:
            self.gather(ratio, sel, r_loc, r3)
            self.round_decimals(r3, r_loc, 3, r3)
            _np(r3).reshape(-1)[r_loc:len_pad] = np.nan

    def sel_stage2(self, r3all, r3len, r3, ml, frac_r, sigma2_max, colmap, st):
        a = _np(st)
        nv = self.count_valid(r3all, r3len) if r3len else 0
        a[3] = nv
        if nv:
            k = min(int(int(a[2]) * (1.0 - frac_r)), nv - 1)
            if k < 0:
                a[5], k = 2, 0
            smin, smax = self.select_kth(r3all, r3len, [k])[0], float(sigma2_max)
        else:
            smin, smax = -math.inf, math.inf
        self._setf(st, 12, smin)
        self._setf(st, 13, smax)
        r_loc = int(a[1])
        ruse = self.colmap_range(r3, r_loc, smin, smax, colmap) if r_loc else 0
        _np(colmap).reshape(-1)[r_loc:ml] = -1
        a[4] = ruse

    def sel_read(self, st):
        return _np(st).copy()

    def zquant(self, q, n, ld, sel, r, rm, mu, scale, zq, ld_zq, colmap, qmax, zb, np_zb):
        if r == 0:
            return 0
        js = _np(sel)[:r]
        qa = self._mat(q, n, int(js.max()) + 1, ld)[:, js]
        rr = _np(rm)[:n]
        mj = _np(mu)[js]
        with np.errstate(all="ignore"):
            y = np.where(qa == MISSING, np.nan, (qa / 100.0) / np.where(rr == 0, np.nan, rr)[:, None])
            z = ((y - mj[None, :]) / np.sqrt(mj)[None, :]) * scale
        out = _hundredths(z)
        zqa = _np(zq).reshape(-1)                # row stride ld_zq (flat views allowed)
        zqa[(np.arange(n)[:, None] * ld_zq + np.arange(r)[None, :]).reshape(-1)] = out.reshape(-1)
        cm = _np(colmap)[:r]
        clip = np.where((out == MISSING) | (out == NEG0), 0, np.clip(out, -qmax, qmax)).astype(np.float32)
        bits = (clip.view(np.uint32) >> 16).astype(np.uint16).view(np.int16)
        zba = _np(zb)                      # K-blocked [kpad/32][np_zb][32]
        for s in range(r):
            if cm[s] >= 0:
                zba[cm[s] // KBW, :n, cm[s] % KBW] = bits[:, s]
        return 0

    def gram(self, zb, np_, kpad, qmax, gram):
        """Upper 128-tiles only, like the HIP kernels (the lower triangle is
        the mirror's job)."""
        zr = _np(zb)[: kpad // KBW, :np_].transpose(1, 0, 2).reshape(np_, kpad)
        bits = zr.view(np.uint16).astype(np.uint32) << 16
        z = bits.view(np.float32).astype(np.float64)
        g = (z @ z.T).astype(np.int64)
        t = np.arange(np_) // 128
        _np(gram)[:np_, :np_] += np.where(t[:, None] <= t[None, :], g, 0)

    def gram_rows(self, zb, np_, kpad, qmax, row0, nrows, out, ld):
        """Cohort split (grid_knn_gram_kb_rows): the upper-triangle 256x128
        tiles of rows [row0, row0+nrows), added at out[(i-row0)*ld + j-row0]."""
        assert row0 % 256 == 0 and nrows % 256 == 0 and row0 + nrows <= np_ and ld >= np_ - row0
        zr = _np(zb).reshape(-1)[: (kpad // KBW) * np_ * KBW].reshape(kpad // KBW, np_, KBW)
        zr = zr.transpose(1, 0, 2).reshape(np_, kpad)
        z = (zr.view(np.uint16).astype(np.uint32) << 16).view(np.float32).astype(np.float64)
        g = (z[row0:row0 + nrows] @ z[row0:].T).astype(np.int64)
        ti = (np.arange(row0, row0 + nrows) // 256)[:, None]
        tj = (np.arange(row0, np_) // 128)[None, :]
        o = _np(out).reshape(-1)[: nrows * ld].reshape(nrows, ld)
        o[:, : np_ - row0] += np.where(tj >= 2 * ti, g, 0)

    def mirror(self, gram, np_):
        g = _np(gram)[:np_, :np_]
        b = np.arange(np_) // 64
        low = b[:, None] > b[None, :]
        g[low] = g.T[low]

    def mirror_ld(self, buf, n, ld):
        g = _np(buf).reshape(-1)[: n * ld].reshape(n, ld)[:, :n]
        b = np.arange(n) // 64
        low = b[:, None] > b[None, :]
        g[low] = g.T[low]

    def diag(self, gram, np_, n, norms):
        """norms[j] = gram[j * np_ + j] (np_ = the row stride)."""
        _np(norms).reshape(-1)[:n] = _np(gram).reshape(-1)[np.arange(n) * (np_ + 1)]

    # multi-GPU step 5 (grid_knn_seg_topk / grid_knn_seg_merge): packed keys
    # (d2 << 20 | index) as uint64 bits in int64 buffers, K1 = 16 per list
    K1 = 16

    def seg_topk(self, seg, ld, nrows, ncols, norms, n, k, r0, c0, rowc, colc):
        s = _np(seg).reshape(-1)[: nrows * ld].reshape(nrows, ld)[:, :ncols]
        dg = _np(norms)[:n].astype(np.int64)
        rc = _np(rowc).reshape(nrows, self.K1).view(np.uint64)
        cc = _np(colc).reshape(-1, self.K1)[:ncols].view(np.uint64)
        rc[:] = np.uint64(2 ** 64 - 1)
        cc[:] = np.uint64(2 ** 64 - 1)
        ktake = min(k + 1, n)
        for u in range(nrows):
            i = r0 + u
            if i >= n:
                break
            js = np.arange(c0, n)
            d = dg[i] + dg[js] - 2 * s[u, : n - c0]
            keys = np.sort((d.astype(np.uint64) << np.uint64(20)) | js.astype(np.uint64))[:ktake]
            rc[u, : len(keys)] = keys
        for t in range(ncols):
            j = c0 + t
            if j >= n:
                break
            iu = np.arange(min(nrows, max(n - r0, 0)))
            d = dg[r0 + iu] + dg[j] - 2 * s[iu, t]
            keys = np.sort((d.astype(np.uint64) << np.uint64(20)) | (r0 + iu).astype(np.uint64))[: self.K1]
            cc[t, : len(keys)] = keys

    def seg_merge(self, rowc, colc, ldc, B, n, k, idx, d2, cnt):
        rc = _np(rowc).reshape(-1, self.K1).view(np.uint64)
        cc = _np(colc).reshape(-1, ldc, self.K1).view(np.uint64)
        ktake = min(k + 1, n)
        for i in range(n):
            bi = i // B
            cand = set(rc[i].tolist())
            for b in range(bi + 1):
                cand.update(cc[b, i - b * B].tolist())
            keys = sorted(c for c in cand if c != 2 ** 64 - 1)[:ktake]
            lst = [(key & 0xFFFFF, key >> 20) for key in keys]
            lst = [(j, dd) for j, dd in lst if j != i][:k] if any(j == i for j, _ in lst) else lst[:k]
            _np(idx)[i, :] = -1
            _np(d2)[i, :] = 0
            for t, (j, dd) in enumerate(lst):
                _np(idx)[i, t] = j
                _np(d2)[i, t] = dd
            _np(cnt)[i] = len(lst)

    def topk_rows(self, rows, ld, norms, n, k, row0, nrows, idx, d2, cnt):
        g = _np(rows).reshape(-1)
        dg = _np(norms)[:n]
        for r in range(nrows):
            i = row0 + r
            d = dg[i] + dg - 2 * g[r * ld: r * ld + n]
            order = np.lexsort((np.arange(n), d))[: min(k + 1, n)]
            lst = [(int(j), int(d[j])) for j in order if j != i][:k]
            _np(idx)[r, :] = -1
            _np(d2)[r, :] = 0
            for t, (j, dd) in enumerate(lst):
                _np(idx)[r, t] = j
                _np(d2)[r, t] = dd
            _np(cnt)[r] = len(lst)

    def dipcn(self, n, reads, has, scale, nbr, nscale, ncnt, ld, n_nbr, out, valid, defer=None):
        if defer is not None:                  # HipOps' deferred flag (never set here)
            _np(defer)[0] = self.dipcn(n, reads, has, scale, nbr, nscale, ncnt, ld, n_nbr, out, valid)
            return None
        rd, hs, sc = _np(reads), _np(has), _np(scale)
        nb, ns, nc = _np(nbr), _np(nscale), _np(ncnt)
        for i in range(n):
            _np(valid)[i] = 0
            if not hs[i]:
                continue
            tot, c = 0.0, 0
            for t in range(nc[i]):
                if c >= n_nbr:
                    break
                j = nb[i, t]
                if j < 0 or not hs[j]:
                    continue
                tot += rd[j] / ns[i, t]
                c += 1
            if c:
                _np(out)[i] = (rd[i] / sc[i]) / (tot / c)
                _np(valid)[i] = 1
        return 0

    def phase(self, n, irr, off, nbr, w, min_nbr, iters, sched, hap, imp, mean):
        o, nb, ww = _np(off), _np(nbr), _np(w)
        hn = [[(int(nb[t]), float(ww[t])) for t in range(o[h], o[h + 1])] for h in range(2 * n)]
        hp, mn = steps.run_phasing([float(x) for x in _np(irr)[:n]], hn, min_nbr, iters)
        _np(hap)[: 2 * n] = hp
        for i in range(n):
            _np(imp)[2 * i: 2 * i + 2] = steps.compute_imp(i, hp, hn, mn)
        _np(mean)[0] = mn

    def schedule(self, off, nbr, w):
        from grid_amd import _abi
        return _abi.hi_schedule(off, nbr, w)
