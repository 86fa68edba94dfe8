"""Step-4 ingest on the device: mosdepth regions.bed.gz files -> the int32
hundredths depth matrix in HBM (R1-R4, normalize_mosdepth.py:96-112 and
:218-416), for the cohorts the host parser would read the common way.

Per batch of files (bounded compressed and text bytes): host threads read the
compressed bytes into pinned memory, one copy to the device, the files are
inflated there (grid_gunzip_batch: one wave per file, CRC-checked), cut in
64 KiB chunks and parsed (grid_md_count / grid_md_parse_map: the reference's
line filters, each record placed by its (start, end) in the key list K of the
reference file).  Then the population means in file order, the valid
columns, the empty-sample filter and the rows in sorted-ID order
(grid_md_finish / grid_md_gather) -- the matrix never exists on the host.

Anything outside the common shape -- a line outside the canonical mosdepth
grammar or a non-ASCII byte, reference keys that are not strictly
increasing, a key outside K, a repeated key, a file of plain gzip members
whose total size its trailer does not give -- raises DeviceIngestUnsupported
and the caller reads the cohort with the host parser (ingest.cpp), which
covers every case the reference reads.  A file that does not inflate (corrupt,
truncated, not gzip) is dropped as the reference drops it.
"""
from __future__ import annotations

import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .. import _abi
from .._abi import MdOpts, call

CH = 65536                      # parse chunk (mosdepth_dev.hip CH)
BATCH_IN = 4 << 30              # compressed bytes per batch
BATCH_TEXT = 24 << 30           # inflated bytes per batch


class DeviceIngestUnsupported(Exception):
    """The cohort leaves the device parser's common case (see the module doc)."""


def _align(x, a=256):
    return -(-int(x) // a) * a


class _Pinned:
    """Reusable pinned host staging (torch allocates the page-locked memory)."""

    def __init__(self):
        self.t = None

    def get(self, n):
        import torch
        if self.t is None or self.t.numel() < n:
            self.t = torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=True)
        return self.t.numpy()


def _opts(dev, prefix, window, excluded, keep):
    pre = (prefix or "").encode()
    d_pre = dev.upload(np.frombuffer(pre or b"\0", np.uint8))
    names = sorted(excluded or {})
    nb = [n.encode() for n in names]
    noff = np.zeros(len(nb) + 1, np.int32)
    noff[1:] = np.cumsum([len(b) for b in nb]) if nb else []
    kb = [np.unique(np.fromiter(excluded[n], dtype=np.int64, count=len(excluded[n]))) for n in names]
    koff = np.zeros(len(kb) + 1, np.int64)
    koff[1:] = np.cumsum([len(k) for k in kb]) if kb else []
    d_names = dev.upload(np.frombuffer(b"".join(nb) or b"\0", np.uint8))
    d_noff, d_koff = dev.upload(noff), dev.upload(koff)
    d_kb = dev.upload(np.concatenate(kb) if kb and koff[-1] else np.zeros(1, np.int64))
    keep += [d_pre, d_names, d_noff, d_koff, d_kb]
    s, e = window if window else (0, 0)
    return MdOpts(d_pre.ptr, len(pre), 1 if window else 0, int(s), int(e), len(names), 0, d_names.ptr, d_noff.ptr,
                  d_koff.ptr, d_kb.ptr)


def _chunks(files, tlen):
    """Chunk table of the files (batch-local indices) with text."""
    cfile, cstart, cfirst = [], [], [0]
    for f in files:
        n = -(-int(tlen[f]) // CH)
        cfile += [f] * n
        cstart += list(range(0, n * CH, CH))
        cfirst.append(len(cfile))
    return (np.asarray(cfile or [0], np.int32), np.asarray(cstart or [0], np.int64), np.asarray(cfirst, np.int32),
            len(cfile))


def ingest_device(dev, paths, prefix, window, excluded, min_depth, max_depth, threads=16):
    """paths: one per individual in file order (None = no file).  Returns
    (ok files in file order, the device state for ``gather``, records in valid
    columns per file, status per file: 0 ok, 1 failed, 3 missing); raises
    DeviceIngestUnsupported."""
    nfiles = len(paths)
    keep = []
    opts = _opts(dev, prefix, window, excluded, keep)
    sizes = np.array([os.path.getsize(p) if p else -1 for p in paths], np.int64)
    status = np.where(sizes < 0, 3, 0).astype(np.int32)       # 3: missing (ingest.cpp FS_MISSING)
    kept = dev.zeros(max(nfiles, 1), np.uint64)
    order = [f for f in range(nfiles) if sizes[f] >= 0]
    # batches in file order
    batches, cur, cin = [], [], 0
    for f in order:
        if cur and cin + _align(sizes[f]) > BATCH_IN:
            batches.append(cur)
            cur, cin = [], 0
        cur.append(f)
        cin += _align(sizes[f])
    if cur:
        batches.append(cur)
    pins = [_Pinned(), _Pinned()]
    pool = ThreadPoolExecutor(max(1, min(int(threads or 1), 32)))

    def read_batch(bi):
        fs = batches[bi]
        off = np.zeros(len(fs) + 1, np.int64)
        off[1:] = np.cumsum([_align(max(sizes[f], 1)) for f in fs])
        buf = pins[bi % 2].get(int(off[-1]) + 256)

        def one(k):
            f = fs[k]
            with open(paths[f], "rb") as fh:
                n = fh.readinto(memoryview(buf)[off[k]:off[k] + sizes[f]])
            if n != sizes[f]:
                raise DeviceIngestUnsupported(f"{paths[f]} changed while reading")
            return _abi.gz_text_size(buf[off[k]:off[k] + sizes[f]]) if sizes[f] else (0, 0)
        caps = list(pool.map(one, range(len(fs))))
        return buf, off, caps

    K = kidx = Q = None
    nK = ref_nlines = 0
    d_in = d_text = None
    pending = pool.submit(read_batch, 0) if batches else None
    try:
        for bi, fs in enumerate(batches):
            buf, off, caps = pending.result()
            pending = pool.submit(read_batch, bi + 1) if bi + 1 < len(batches) else None
            nb = len(fs)
            caps_ = np.array([c[0] if c else 0 for c in caps], np.int64)
            gz = np.array([c is not None for c in caps])
            tcap = np.array([_align(max(c, 1), 256) for c in caps_], np.int64)
            toff = np.zeros(nb + 1, np.int64)
            toff[1:] = np.cumsum(tcap)
            if toff[-1] > BATCH_TEXT * 2:
                raise DeviceIngestUnsupported("a batch of files inflates beyond the device text buffer")
            if d_in is None or d_in.nbytes < off[-1] + 256:
                d_in = dev.alloc(int(max(off[-1] + 256, BATCH_IN + 256)), np.uint8)
            if d_text is None or d_text.nbytes < toff[-1] + 256:
                d_text = dev.alloc(int(max(toff[-1] + 256, min(BATCH_TEXT, 1 << 34))), np.uint8)
            call("grid_h2d", dev.ctx, d_in.ptr, buf.ctypes.data, int(off[-1]))
            lens = np.array([sizes[f] if gz[k] else 0 for k, f in enumerate(fs)], np.int64)
            mcap = max(1, int(max((s // 4096 + 16 for s in lens), default=1)))
            d_off, d_len = dev.upload(off[:nb]), dev.upload(lens)
            d_toff, d_tcap = dev.upload(toff[:nb]), dev.upload(caps_)
            mem = dev.alloc(nb * mcap * _abi.GZ_MEMBER_BYTES, np.uint8)
            st, ln, nm = dev.alloc(nb, np.int32), dev.alloc(nb, np.int64), dev.alloc(nb, np.int32)
            call("grid_gunzip_batch", dev.ctx, d_in.ptr, d_off.ptr, d_len.ptr, nb, d_text.ptr, d_toff.ptr,
                 d_tcap.ptr, mem.ptr, mcap, st.ptr, ln.ptr, nm.ptr)
            gst, tlen = st.numpy(), ln.numpy()
            for k, f in enumerate(fs):
                if sizes[f] == 0:
                    gst[k], tlen[k] = 0, 0                 # an empty file: no lines (gzip.open reads nothing)
                elif not gz[k]:
                    gst[k] = _abi.GZ_EHEADER
                if gst[k] == _abi.GZ_ESPACE:
                    raise DeviceIngestUnsupported(f"{paths[f]}: several gzip members (text size unknown)")
                status[f] = 0 if gst[k] == 0 else 1        # 1: failed (the reference drops the sample)
            okb = [k for k in range(nb) if gst[k] == 0 and tlen[k] > 0]
            cfile, cstart, cfirst, nch = _chunks(okb, tlen)
            if nch == 0:
                continue
            d_tl = dev.upload(tlen)
            d_cfile, d_cstart, d_cfirst = dev.upload(cfile), dev.upload(cstart), dev.upload(cfirst)
            cnl, cline0 = dev.alloc(nch, np.int32), dev.alloc(nch, np.int64)
            # flags per batch file, folded into the cohort's afterwards
            bflags = dev.zeros(nb, np.int32)
            call("grid_md_count", dev.ctx, d_text.ptr, d_toff.ptr, d_tl.ptr, nch, d_cfile.ptr, d_cstart.ptr,
                 d_cfirst.ptr, len(okb), cnl.ptr, cline0.ptr, bflags.ptr)
            if K is None:
                # the reference key list: the first file that inflated with text
                r = okb[0]
                c0, c1 = int(cfirst[0]), int(cfirst[1])
                rc_file = np.zeros(c1 - c0, np.int32) + r
                cl = cline0.numpy()[c0:c1]
                nl = cnl.numpy()[c0:c1]
                tail = np.zeros(1, np.uint8)
                call("grid_d2h", dev.ctx, tail.ctypes.data, d_text.ptr + int(toff[r] + tlen[r] - 1), 1)
                ref_nlines = int(cl[-1] + nl[-1]) + (0 if tail[0] == 10 else 1)
                kline = dev.alloc(max(ref_nlines, 1), np.uint8)
                keys_line = dev.alloc((max(ref_nlines, 1), 2), np.int64)
                K = dev.alloc((max(ref_nlines, 1), 2), np.int64)
                kidx = dev.alloc(max(ref_nlines, 1), np.int32)
                h_nK, h_uns = C.c_int64(), C.c_int32()
                d_rcf, d_rcs, d_rcl = dev.upload(rc_file), dev.upload(cstart[c0:c1]), dev.upload(cl)
                call("grid_md_parse_ref", dev.ctx, d_text.ptr, d_toff.ptr, d_tl.ptr, c1 - c0, d_rcf.ptr,
                     d_rcs.ptr, d_rcl.ptr, C.byref(opts), bflags.ptr, ref_nlines,
                     kline.ptr, keys_line.ptr, K.ptr, kidx.ptr, C.byref(h_nK), C.byref(h_uns))
                del kline, keys_line
                if h_uns.value:
                    raise DeviceIngestUnsupported("the reference file's keys are not strictly increasing")
                nK = h_nK.value
                if nK == 0:
                    raise DeviceIngestUnsupported("the reference file keeps no record")
                Q = dev.alloc((nfiles, nK), np.int32)
                call("grid_fill_i32", dev.ctx, Q.ptr, nfiles * nK, _abi.MISSING)
            qrow = dev.upload(np.asarray(fs, np.int32))
            bk = dev.zeros(nb, np.uint64)
            call("grid_md_parse_map", dev.ctx, d_text.ptr, d_toff.ptr, d_tl.ptr, nch, d_cfile.ptr, d_cstart.ptr,
                 cline0.ptr, C.byref(opts), bflags.ptr, K.ptr, nK, kidx.ptr, ref_nlines, Q.ptr, nK, qrow.ptr, bk.ptr)
            bf, bkv = bflags.numpy(), bk.numpy()
            for k in okb:
                if bf[k]:
                    why = "a line outside the mosdepth grammar" if bf[k] & _abi.MD_EXOTIC else "a key outside K"
                    raise DeviceIngestUnsupported(f"{paths[fs[k]]}: {why}")
            kept_h = kept.numpy()
            kept_h[np.asarray(fs)] += bkv
            kept.copy_from(kept_h)
    finally:
        if pending is not None:
            try:
                pending.result()
            except Exception:
                pass
        pool.shutdown(wait=True)
    if K is None:
        return [], [], None, status
    rows = np.array([f for f in range(nfiles) if status[f] == 0], np.int32)
    mean = dev.alloc(nK, np.float64)
    valid, cpos = dev.alloc(nK, np.int32), dev.alloc(nK, np.int64)
    present, nvalid = dev.alloc(max(nfiles, 1), np.uint64), dev.alloc(max(nfiles, 1), np.uint64)
    m = C.c_int64()
    d_rows = dev.upload(rows if rows.size else np.zeros(1, np.int32))
    call("grid_md_finish", dev.ctx, Q.ptr, nK, nK, nfiles, d_rows.ptr, len(rows), float(min_depth),
         float(max_depth), mean.ptr, valid.ptr, cpos.ptr, present.ptr, nvalid.ptr, C.byref(m))
    pres, nval, kh = present.numpy()[:nfiles], nvalid.numpy()[:nfiles], kept.numpy()[:nfiles]
    if np.any(pres[rows] != kh[rows]):
        raise DeviceIngestUnsupported("a repeated (start, end) key in a file")
    m = m.value
    return rows, (Q, nK, valid, cpos, K, m), nval, status


def gather(dev, state, row_files, nfiles):
    """The matrix rows of ``row_files`` (file indices, in output order) and
    the valid columns' (start, end)."""
    Q, nK, valid, cpos, K, m = state
    dst = np.full(max(nfiles, 1), -1, np.int32)
    dst[np.asarray(row_files, np.int64)] = np.arange(len(row_files), dtype=np.int32)
    out = dev.alloc((max(len(row_files), 1), max(m, 1)), np.int32)
    st, en = dev.alloc(max(m, 1), np.int64), dev.alloc(max(m, 1), np.int64)
    d_dst = dev.upload(dst)
    call("grid_md_gather", dev.ctx, Q.ptr, nK, nK, nfiles, valid.ptr, cpos.ptr, d_dst.ptr, out.ptr,
         max(m, 1), K.ptr, st.ptr, en.ptr)
    regions = list(zip(st.numpy()[:m].tolist(), en.numpy()[:m].tolist()))
    out.shape = (len(row_files), m)            # the allocation keeps >= 1 element
    return out, regions
