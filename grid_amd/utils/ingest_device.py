"""Step-4 ingest on the device: mosdepth regions.bed.gz files -> the int32
hundredths depth matrix in HBM (R1-R4, normalize_mosdepth.py:96-112 and
:218-416), for the cohorts the host parser would read the common way.

Per batch of files (bounded compressed and text bytes): host threads read the
compressed bytes into pinned memory and find each file's BGZF members (what
mosdepth writes: independent gzip members of <= 64 KiB text).  The batch's
files are then inflated by the GPU and the host CPUs AT ONCE, split by a cost
model whose rates are re-measured every batch (``_Split``):
  * GPU (grid_gunzip_batch, CRC-checked): one wave per BGZF member -- a
    member-granular work list that fills every CU -- or one wave per file for
    a single-member gzip file (serial by nature: the model gives the GPU such
    a file only when a wave's rate makes it worth it);
  * CPU (grid_gunzip_host: libdeflate, zlib without it): threads inflate
    whole files into pinned staging, copied to HBM on a second stream while
    the GPU works.
The text then is cut in 64 KiB chunks and parsed on the GPU (grid_md_count /
grid_md_parse_map: the reference's line filters, each record placed by its
(start, end) in the key list K of the reference file).  Then the population
means in file order, the valid columns, the empty-sample filter and the rows
in sorted-ID order (grid_md_finish / grid_md_gather) -- the matrix never
exists on the host.

Text the host threads inflated is checked where it sits in HBM before it is
parsed: the CRC-32 of each such file's text in d_text (grid_text_crc32) must
equal the CRC its gzip trailers give (the GPU-inflated members are checked the
same way by grid_gunzip_batch's k_gz_crc); a mismatch hands the cohort to the
host parser.

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
import time
from collections.abc import Sequence
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .. import _abi
from .._abi import MdOpts, call

CH = 16384                      # parse chunk (mosdepth_dev.hip CH)
BATCH_IN = 4 << 30              # compressed bytes per batch
BATCH_TEXT = 24 << 30           # inflated bytes per batch
FIRST_BATCH_IN = 256 << 20      # the first batch (read and inflated synchronously: the reference key list)
PIPELINE = True                 # BGZF batches after the first: enqueued without host round trips (_Async)
STAGE = 1 << 30                 # pinned staging per CPU sub-batch (two of them)
TRACE = bool(os.environ.get("GRID_INGEST_TRACE"))   # per-batch phase times on stderr
XSTREAM_WAIT = True             # dev's stream waits for the copy stream (False only in a GPU test's control arm)
AFTER_HOST_TEXT = None          # test seam: called (dev, d_text, toff, files) once host text is in HBM
# pipelined BGZF batches: the fraction of each batch's files the host threads
# inflate beside the GPU (every k-th file; 0 = the GPU inflates all).  With 16
# host threads beside the MI355X's 37 GB/s, config-2 ingest (r04y, kept
# staging): 0.15 9.9 s, 0.2 9.5 s, 0.25 9.1-9.25 s, 0.33 9.3-9.6 s
HOST_FRAC = float(os.environ.get("GRID_INGEST_HOST_FRAC", "0.25"))
# the host share is sized from the config's `threads` (the
# reference defaults to 1 thread, its example config uses 4): the host files
# take as long as the GPU's when f / (t H) = (1 - f) / G, so f = t H / (G + t H)
# with H one thread's inflate rate beside the GPU and G the GPU's; 0.25 at 16
# threads (the r04ae optimum) gives H ~ 0.77 GB/s at G ~ 37 GB/s.  Round 5's
# inflate runs at G ~ 63 GB/s (r05ag), where the model's 16 % at 16 threads
# measured slower than none (config 2 ingest 6.34 vs 6.04 s, r05ah: the host
# reads, copies and checks its files beside the batch and they no longer hide
# under the GPU's part); below one file in 5 the share is not used
HOST_RATE_PER_THREAD = 0.77e9
GPU_INFLATE_RATE = 63e9          # r05ag: BGZF members (tools/bench_inflate.py --bgzf --units)
HOST_FRAC_MIN = 0.2
# file reads and member tables: a pool of their own, independent of `threads`
READ_THREADS = int(os.environ.get("GRID_INGEST_READ_THREADS", "8"))


def host_frac(threads):
    """Fraction of a pipelined batch's BGZF files the host threads inflate."""
    t = max(1, int(threads))
    f = t * HOST_RATE_PER_THREAD / (GPU_INFLATE_RATE + t * HOST_RATE_PER_THREAD)
    f = min(f, HOST_FRAC)
    return f if f >= HOST_FRAC_MIN else 0.0


class DeviceIngestUnsupported(Exception):
    """The cohort leaves the device parser's common case (see the module doc)."""


def _align(x, a=256):
    return -(-int(x) // a) * a


class _Pinned:
    """Reusable host staging.  Page-locked (grid_host_alloc: no torch in the
    step path -- a first ``import torch`` costs seconds on a fresh host) for
    the asynchronous copies of host-inflated text; PAGEABLE (``pinned=False``)
    for the compressed input: the runtime copies pageable memory to HBM as fast
    as page-locked here (56 vs 52-58 GB/s, profiles/r04i_host_read_h2d.jsonl),
    while page-locking 4 GB costs ~0.65 s that stalls every other HIP call."""

    def __init__(self, bound, pinned=True):
        self.b = None
        self.bound = int(bound)        # the size a request normally stays within
        self.pinned = pinned

    def get(self, n):
        if self.b is None or self.b.nbytes < n:
            if self.b is not None:
                self.b.free()
            # room to grow at once: a buffer re-pinned a few MB larger each
            # batch stalled that batch's copy to HBM by ~1 s (profiles/r03q)
            nb = max(int(n), min(2 * int(n), self.bound), 1)
            self.b = _abi.PinnedBuf(nb) if self.pinned else _Pageable(nb)
        return self.b.array


_libc = C.CDLL(None, use_errno=True)
_libc.mmap.restype = C.c_void_p
_libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
_libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
_libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]


class _Pageable:
    """Pageable staging mapped through libc (anonymous, transparent huge pages
    advised, as NumPy does for large arrays) and unmapped through a foreign
    call, so the multi-GB munmap runs without the GIL (a NumPy array's free
    holds it: the staging released on a background thread stalled the step's
    own thread for ~0.5 s at the end of the config-2 ingest)."""

    def __init__(self, nbytes):
        self.nbytes = max(int(nbytes), 1)
        p = _libc.mmap(None, self.nbytes, 3, 0x22, -1, 0)      # PROT_READ|WRITE, MAP_PRIVATE|ANONYMOUS
        if p is None or p == C.c_void_p(-1).value:
            raise MemoryError(f"staging of {self.nbytes} bytes")
        _libc.madvise(p, self.nbytes, 14)                      # MADV_HUGEPAGE (advice only)
        self.ptr = p
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))
        # its own reference: at interpreter exit the module's globals may be
        # gone before this object's __del__ runs
        self._munmap = _libc.munmap

    def free(self):
        if self.ptr:
            self.array = None
            self._munmap(self.ptr, self.nbytes)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


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


class _Split:
    """Which files of a batch the GPU inflates and which the CPU threads do,
    from rates measured on the previous batches (initial values: MI355X with
    16 host threads, tools/bench_inflate.py): the GPU's aggregate text rate
    over BGZF members, one wave's rate on a whole single-member file, and one
    CPU thread's rate.  Greedy, largest file first, to the side that would
    finish sooner."""

    def __init__(self, threads):
        self.threads = max(1, int(threads))
        self.gpu = 18.0e9         # B/s, member-parallel, as seen by a batch (beside its disk reads; learned)
        self.wave = 9.0e6         # B/s, one wave on one whole file
        self.cpu = 0.4e9          # B/s per thread while the GPU inflates too (0.6-0.7 alone)

    def plan(self, files, text, bgzf):
        """BGZF files all go to the GPU: with the member-parallel inflate at
        ~18 GB/s of text the host threads (~10 GB/s alone) only slow both sides
        down when they run beside it -- host memory traffic of their text and
        stage copies (1,024 files: GPU alone 7.1 s, split 8.3 s; config 2:
        split 30.0 s, profiles/r03o_*, r03p_*).  Single-member files (a serial
        stream each) go to whichever side the rates say."""
        if all(bgzf[k] for k in files):
            return sorted(files), []
        g_mem = g_whole = c = 0.0
        gpu, cpu = [], []
        for k in sorted(files, key=lambda k: -int(text[k])):
            s = float(text[k])
            tg = max((g_mem + s) / self.gpu, g_whole) if bgzf[k] else max(g_mem / self.gpu, g_whole, s / self.wave)
            tc = (c + s) / (self.cpu * self.threads)
            cur_g = max(g_mem / self.gpu, g_whole)
            cur_c = c / (self.cpu * self.threads)
            if max(tg, cur_c) <= max(cur_g, tc):
                gpu.append(k)
                if bgzf[k]:
                    g_mem += s
                else:
                    g_whole = max(g_whole, s / self.wave)
            else:
                cpu.append(k)
                c += s
        return sorted(gpu), sorted(cpu)

    def learn(self, g_mem_bytes, g_whole_max, t_gpu, c_bytes, t_cpu):
        a = 0.5                   # moving average over batches
        if t_gpu > 0.05:
            if g_mem_bytes and not g_whole_max:
                self.gpu = (1 - a) * self.gpu + a * g_mem_bytes / t_gpu
            elif g_whole_max and not g_mem_bytes:
                self.wave = (1 - a) * self.wave + a * g_whole_max / t_gpu
        if t_cpu > 0.05 and c_bytes:
            self.cpu = (1 - a) * self.cpu + a * c_bytes / (t_cpu * self.threads)


def _gpu_inflate(dev, d_in, d_text, units, mcap):
    """Launch grid_gunzip_batch over units (in_off, in_len, out_off, cap);
    returns the device buffers to read after the stream syncs."""
    n = len(units[0])
    d = [dev.upload(np.asarray(u, np.int64)) for u in units]
    mem = dev.alloc(n * mcap * _abi.GZ_MEMBER_BYTES, np.uint8)
    st, ln, nm = dev.alloc(n, np.int32), dev.alloc(n, np.int64), dev.alloc(n, np.int32)
    call("grid_gunzip_batch", dev.ctx, d_in.ptr, d[0].ptr, d[1].ptr, n, d_text.ptr, d[2].ptr, d[3].ptr, mem.ptr,
         mcap, st.ptr, ln.ptr, nm.ptr)
    return d, mem, st, ln, nm


def _chunks(files, tlen):
    """Chunk table of the files (batch-local indices) with text: per chunk its
    file and start; per file its first chunk (cfirst[k], k in file order)."""
    files = np.asarray(files, np.int64)
    n = -(-np.asarray(tlen, np.int64)[files] // CH) if len(files) else np.zeros(0, np.int64)
    cfirst = np.zeros(len(files) + 1, np.int32)
    np.cumsum(n, out=cfirst[1:])
    tot = int(cfirst[-1])
    if tot == 0:
        return np.zeros(1, np.int32), np.zeros(1, np.int64), cfirst, 0
    cfile = np.repeat(files, n).astype(np.int32)
    cstart = (np.arange(tot, dtype=np.int64) - np.repeat(cfirst[:-1].astype(np.int64), n)) * CH
    return cfile, cstart, cfirst, tot


# The host staging of the device ingest, kept between the batches and the
# ingests of one run: releasing tens of GB of staging the HIP runtime has
# copied from (page-locked, or pageable pages it has seen) holds the runtime for
# 0.4-0.8 s, and every HIP call of the step after the ingest waited for it (r04y,
# r04ac).  release_staging() frees it: at the end of a pipeline run or of a
# standalone step 4, and when the ingest hands over to the host parser
# (grid_amd/device.py release_ingest_buffers).
_STAGING = {}


def _staging(name, bound, pinned=False):
    b = _STAGING.get(name)
    if b is None:
        b = _STAGING[name] = _Pinned(bound, pinned=pinned)
    return b


def staging_bytes():
    return sum(p.b.nbytes for p in _STAGING.values() if p.b is not None)


def release_staging():
    """Free the kept host staging; returns the bytes released."""
    freed = 0
    for p in list(_STAGING.values()):
        if p.b is not None:
            freed += p.b.nbytes
            p.b.free()
            p.b = None
    _STAGING.clear()
    return freed


class _Async:
    """The device ingest's pipelined batches (every file BGZF, all inflated by
    the GPU; after the first batch, which builds the key list K synchronously).
    Per batch, with no host round trip:
      copy stream:  [wait: batch b-2's parse done] compressed input + the batch's
                    tables (member units, files, 64 KiB chunks: one pinned arena)
                    -> HBM (d_in / tables of parity b % 2); event h2d[b % 2];
      main stream:  [wait h2d] grid_gunzip_batch (inflate + CRC) -> grid_file_status
                    (files with a failed member are skipped by the parse, as the
                    reference drops them) -> grid_md_count -> grid_md_parse_map;
                    event done[b % 2].
    So batch b+1's 4 GB copy runs under batch b's inflate, and the host only
    builds tables.  A file's text length is the sum of its members' ISIZEs
    (the inflater checks every member against its ISIZE and CRC).  Statuses,
    lengths, flags and kept counts stay on the device per batch and are read
    once at the end (results)."""

    def __init__(self, dev, cdev, opts, K, nK, kidx, ref_nlines, Q):
        self.dev, self.cdev, self.opts = dev, cdev, opts
        self.K, self.nK, self.kidx, self.ref_nlines, self.Q = K, nK, kidx, ref_nlines, Q
        self.h2d = [_abi.Event(), _abi.Event()]
        self.done = [_abi.Event(), _abi.Event()]
        self.issued = [False, False]
        self.arena_h = [_staging("arena0", 64 << 20), _staging("arena1", 64 << 20)]
        self.arena_d = [None, None]
        self.scr = [None, None]                 # per parity: member table, chunk counts/lines, file status
        self.out = []                           # per batch: (fs, owner, unit status, unit length, flags, kept, okb)
        self.htext = [_abi.Event(), _abi.Event()]   # host-inflated text of parity p is in HBM
        self.hbad = []                          # host-share files whose text failed its CRC in HBM
        self.one = None                         # page-locked int32 1: a failed host-share file's device status

    @staticmethod
    def _pack(parts):
        offs, pos = [], 0
        for a in parts:
            offs.append(pos)
            pos += _align(a.nbytes)
        return offs, pos

    def batch(self, bi, fs, buf, off, caps_, gz, members, toff, d_in, d_text, fsizes, hshare=None):
        """hshare: (files, future) -- files of the batch the host threads inflate
        (the future returns per file (status, length, crc, staging, offset));
        their text is copied into d_text once the previous batch's parse is done
        and checked there against its gzip CRC on the copy stream, while the
        GPU inflates the rest; the parse waits for the copy (event htext)."""
        dev, cdev, p = self.dev, self.cdev, bi % 2
        nb = len(fs)
        mu = [k for k in range(nb) if gz[k] and fsizes[k] > 0 and members[k] is not None]
        hset = set(hshare[0]) if hshare else set()
        uo, ul, to, tc, owner = [], [], [], [], []
        for k in mu:
            if k in hset:
                continue
            ms, ml, mi = members[k]
            uo.append(off[k] + ms)
            ul.append(ml)
            cum = np.zeros(len(mi), np.int64)
            np.cumsum(mi[:-1], out=cum[1:])
            to.append(toff[k] + cum)
            tc.append(mi.astype(np.int64))
            owner.append(np.full(len(mi), k, np.int64))
        cat = (lambda x: np.concatenate(x) if x else np.zeros(0, np.int64))
        units = [cat(x) for x in (uo, ul, to, tc, owner)]
        nu = len(units[0])
        tlen = np.zeros(nb, np.int64)               # text of a file that inflates: its members' ISIZEs
        for k in mu:
            tlen[k] = int(members[k][2].astype(np.int64).sum())
        okb = [k for k in mu if tlen[k] > 0]
        cfile, cstart, cfirst, nch = _chunks(okb, tlen)
        parts = units + [tlen, np.ascontiguousarray(toff[:nb]), np.asarray(fs, np.int32), cfile, cstart, cfirst]
        offs, nbytes = self._pack(parts)
        # the arena of parity p: its previous copy (batch bi-2) must be done
        if self.issued[p]:
            self.h2d[p].host_wait()
        host = self.arena_h[p].get(nbytes + 256)
        for a, o in zip(parts, offs):
            host[o:o + a.nbytes] = a.view(np.uint8).reshape(-1)
        if self.arena_d[p] is None or self.arena_d[p].nbytes < nbytes + 256:
            self.drain()
            self.arena_d[p] = None
            self.arena_d[p] = dev.alloc(max(nbytes + 256, 16 << 20) * 5 // 4, np.uint8)
        need = (nu * _abi.GZ_MEMBER_BYTES, nu * 4, nch * 4, nch * 8, nb * 4)
        sc = self.scr[p]
        if sc is None or any(b.nbytes < n + 256 for b, n in zip(sc, need)):
            self.drain()
            self.scr[p] = None
            self.scr[p] = sc = [dev.alloc(max(n + 256, 4096) * 5 // 4, np.uint8) for n in need]
        mem, unm, cnl, cline0, fst = sc
        # per-batch outputs read at the end (small)
        ust, uln = dev.alloc(max(nu, 1), np.int32), dev.alloc(max(nu, 1), np.int64)
        bflags, bk = dev.zeros(nb, np.int32), dev.zeros(nb, np.uint64)
        # copy context: after batch bi-2's parse (same parity buffers), the input
        # and the tables, from pageable staging (the call returns once they are in
        # HBM; it runs while the device inflates batch bi-1)
        if self.issued[p]:
            self.done[p].host_wait()
        call("grid_h2d", cdev.ctx, d_in.ptr, buf.ctypes.data, int(off[-1]))
        call("grid_h2d", cdev.ctx, self.arena_d[p].ptr, host.ctypes.data, nbytes)
        self.h2d[p].put(cdev)
        # main stream
        self.h2d[p].wait(dev)
        A = self.arena_d[p].ptr
        d_uo, d_ul, d_to, d_tc, d_own, d_tl, d_toff, d_qrow, d_cf, d_cs, d_c1 = (A + o for o in offs)
        if nu:
            call("grid_gunzip_batch", dev.ctx, d_in.ptr, d_uo, d_ul, nu, d_text.ptr, d_to, d_tc, mem.ptr, 1,
                 ust.ptr, uln.ptr, unm.ptr)
        hfail = []
        if hset:
            res = hshare[1].result()
            # the previous batch's parse reads d_text: its regions are free once it is done
            q = 1 - p
            if self.issued[q]:
                self.done[q].host_wait()
            hk = []
            for k in sorted(hset):
                st_, ln_, crc_, stage, so = res[k]
                if st_ != 0 or ln_ != tlen[k]:
                    hfail.append(k)              # dropped, as a file with a failed member on the GPU
                    continue
                if ln_:
                    call("grid_h2d", cdev.ctx, d_text.ptr + int(toff[k]), stage.ctypes.data + int(so), int(ln_))
                    hk.append(k)
            self.htext[p].put(cdev)
            self.htext[p].wait(dev)
            if hk and AFTER_HOST_TEXT is not None:
                AFTER_HOST_TEXT(cdev, d_text, toff, hk)
            if hk:
                # the guard, on the copy stream (it wrote the text): a mismatch hands
                # the cohort to the host parser once the batches are done
                got = _abi.text_crc32(cdev, d_text.ptr, toff[hk], tlen[hk])
                for k, c in zip(hk, got):
                    if int(c) != int(res[k][2]):
                        self.hbad.append((fs[k], "its text in HBM does not match its gzip CRC"))
        call("grid_file_status", dev.ctx, ust.ptr, d_own, nu, fst.ptr, nb)
        if hfail:
            # the parse skips them: their device status set after grid_file_status (stream order)
            if self.one is None:
                self.one = _abi.PinnedBuf(64)
                self.one.array[:4] = np.array([1], np.int32).view(np.uint8)
            for k in hfail:
                call("grid_h2d_async", dev.ctx, fst.ptr + 4 * k, self.one.ptr, 4)
        if nch:
            call("grid_md_count", dev.ctx, d_text.ptr, d_toff, d_tl, nch, d_cf, d_cs, d_c1, len(okb), cnl.ptr,
                 cline0.ptr, bflags.ptr, fst.ptr)
            call("grid_md_parse_map", dev.ctx, d_text.ptr, d_toff, d_tl, nch, d_cf, d_cs, cline0.ptr,
                 C.byref(self.opts), bflags.ptr, self.K.ptr, self.nK, self.kidx.ptr, self.ref_nlines, self.Q.ptr,
                 self.nK, d_qrow, bk.ptr, fst.ptr)
        self.done[p].put(dev)
        self.issued[p] = True
        # not gzip at all: dropped (GZ_EHEADER in the synchronous path)
        hdr_bad = [k for k in range(nb) if not gz[k] and fsizes[k] > 0]
        self.out.append((list(fs), units[4], ust, uln, bflags, bk, okb, nu, hdr_bad, hfail))
        return self.h2d[p]

    def drain(self):
        self.dev.sync()
        self.cdev.sync()

    def results(self, paths):
        """(file, status 0/1, kept) per file of the pipelined batches; raises
        DeviceIngestUnsupported for a parse flag, as the synchronous path."""
        if self.hbad:
            f, why = self.hbad[0]
            raise DeviceIngestUnsupported(f"{paths[f]}: {why} ({len(self.hbad)} host-inflated file(s))")
        res = []
        self.kept = []
        for fs, owner, ust, uln, bflags, bk, okb, nu, hdr_bad, hfail in self.out:
            nb = len(fs)
            bad = np.zeros(nb, np.int32)
            bad[hdr_bad] = _abi.GZ_EHEADER
            bad[hfail] = _abi.GZ_EDATA
            if nu:
                st = ust.numpy()[:nu]
                # a member past its BGZF size is corrupt (dropped), not several members
                np.maximum.at(bad, owner, np.where(st == _abi.GZ_ESPACE, _abi.GZ_EDATA, st))
            bf, bkv = bflags.numpy(), bk.numpy()
            for k in okb:
                if bad[k] == 0 and bf[k]:
                    why = "a line outside the mosdepth grammar" if bf[k] & _abi.MD_EXOTIC else "a key outside K"
                    raise DeviceIngestUnsupported(f"{paths[fs[k]]}: {why}")
            for k, f in enumerate(fs):
                res.append((f, 0 if bad[k] == 0 else 1, int(bkv[k])))
            self.kept.append((np.asarray(fs), bkv))
        return res

    def kept_total(self, nfiles):
        tot = np.zeros(max(nfiles, 1), np.uint64)
        for fs, bkv in self.kept:
            tot[fs] += bkv
        return tot

    def close(self):
        try:
            self.drain()
        finally:
            if self.one is not None:
                self.one.free()
                self.one = None
            self.out = []
            self.arena_d = [None, None]
            self.scr = [None, None]


def ingest_device(dev, paths, prefix, window, excluded, min_depth, max_depth, threads=16, ref=None,
                  keys_only=False, finish=True):
    """paths: one per individual in file order (None = no file).  Returns
    (ok files in file order, the device state for ``gather``, records in valid
    columns per file, status per file: 0 ok, 1 failed, 3 missing); raises
    DeviceIngestUnsupported.

    The distributed step 4 (dist_step4.py) splits this in two: rank 0 runs
    ``keys_only`` (the first batch only: the reference key list K as host
    arrays (K [nK][2] int64, kidx int32, ref_nlines), or None when no file
    inflates), every rank then parses its slice of the files over that K
    (``ref``) with ``finish=False``: (Q [nfiles][nK] int32 on the device, nK,
    status, records kept per file) -- the population means are a chain over
    the ranks there."""
    nfiles = len(paths)
    t_start = time.perf_counter()
    keep = []
    opts = _opts(dev, prefix, window, excluded, keep)
    sizes = np.array([os.path.getsize(p) if p else -1 for p in paths], np.int64)
    status = np.where(sizes < 0, 3, 0).astype(np.int32)       # 3: missing (ingest.cpp FS_MISSING)
    kept = dev.zeros(max(nfiles, 1), np.uint64)
    order = [f for f in range(nfiles) if sizes[f] >= 0]
    # batches in file order
    batches, cur, cin = [], [], 0
    for f in order:
        lim = min(FIRST_BATCH_IN, BATCH_IN) if not batches and ref is None else BATCH_IN
        if cur and cin + _align(sizes[f]) > lim:
            batches.append(cur)
            cur, cin = [], 0
        cur.append(f)
        cin += _align(sizes[f])
    if cur:
        batches.append(cur)
    in_need = 256 + max((sum(_align(max(sizes[f], 1)) for f in b) for b in batches), default=0)
    pins = [_staging("in0", BATCH_IN + 512), _staging("in1", BATCH_IN + 512)]
    first = _staging("first", FIRST_BATCH_IN + 512)        # the (small) first batch: K, quickly
    stages = [_staging("text0", STAGE + 512, pinned=True), _staging("text1", STAGE + 512, pinned=True)]
    nthreads = max(1, min(int(threads or 1), 32))
    pool = ThreadPoolExecutor(nthreads)   # host inflate (the host share, non-BGZF files)
    iopool = ThreadPoolExecutor(max(1, READ_THREADS))   # file reads + member tables
    rpool = ThreadPoolExecutor(1)         # the next batch's read (its files on `iopool`)
    hfrac = host_frac(nthreads)
    copier = ThreadPoolExecutor(1)        # H2D of CPU-inflated text, on its own stream
    waiter = ThreadPoolExecutor(1)        # notes when the GPU's inflate ends
    hctl = ThreadPoolExecutor(1)          # pipelined batches: the host share's inflate (its files on `pool`)
    hstages = [_staging("host0", 8 << 30), _staging("host1", 8 << 30)]
    cdev = _abi.Device(dev.index)          # its own non-blocking stream
    split = _Split(nthreads)

    h2d_done = [None] * len(batches)       # per pipelined batch: the event after its copies to HBM

    def read_batch(bi):
        fs = batches[bi]
        off = np.zeros(len(fs) + 1, np.int64)
        off[1:] = np.cumsum([_align(max(sizes[f], 1)) for f in fs])
        if bi >= 2 and h2d_done[bi - 2] is not None:
            h2d_done[bi - 2].host_wait()        # pins[bi % 2] still feeds batch bi-2's copy
        buf = (first if bi == 0 else pins[bi % 2]).get(int(off[-1]) + 256)

        def one(k):
            f = fs[k]
            with open(paths[f], "rb") as fh:
                n = fh.readinto(memoryview(buf)[off[k]:off[k] + sizes[f]])
            if n != sizes[f]:
                raise DeviceIngestUnsupported(f"{paths[f]} changed while reading")
            if not sizes[f]:
                return (0, 0), None
            v = buf[off[k]:off[k] + sizes[f]]
            return _abi.gz_text_size(v), _abi.gz_members(v)
        info = list(iopool.map(one, range(len(fs))))
        return buf, off, [i[0] for i in info], [i[1] for i in info]

    def inflate(buf, off, fs, caps_, gz, members, toff, d_in, d_text, plan):
        """Inflate the batch's files into d_text + toff[k]; (status, length) per file."""
        nb = len(fs)
        gst = np.zeros(nb, np.int32)
        tlen = np.zeros(nb, np.int64)
        hcrc = np.zeros(nb, np.uint32)
        todo = [k for k in range(nb) if gz[k] and sizes[fs[k]] > 0]
        for k in range(nb):
            if not sizes[fs[k]]:
                gst[k] = 0                             # an empty file: no lines (gzip.open reads nothing)
            elif not gz[k]:
                gst[k] = _abi.GZ_EHEADER
        bgzf = {k: members[k] is not None for k in todo}
        on_gpu, on_cpu = plan
        t0 = time.perf_counter()
        launched = []
        if on_gpu:
            call("grid_h2d", dev.ctx, d_in.ptr, buf.ctypes.data, int(off[-1]))
            mu = [k for k in on_gpu if bgzf[k]]
            wu = [k for k in on_gpu if not bgzf[k]]
            if wu:                                     # whole files: one wave each, started first
                mcap = max(1, int(max(sizes[fs[k]] // 4096 + 16 for k in wu)))
                units = ([off[k] for k in wu], [sizes[fs[k]] for k in wu], [toff[k] for k in wu],
                         [caps_[k] for k in wu])
                launched.append(("whole", wu, None, _gpu_inflate(dev, d_in, d_text, units, mcap)))
            if mu:                                     # BGZF: one wave per member
                uo, ul, to, tc, owner = [], [], [], [], []
                for k in mu:
                    ms, ml, mi = members[k]
                    uo.append(off[k] + ms)
                    ul.append(ml)
                    cum = np.zeros(len(mi), np.int64)
                    np.cumsum(mi[:-1], out=cum[1:])
                    to.append(toff[k] + cum)
                    tc.append(mi.astype(np.int64))
                    owner.append(np.full(len(mi), k, np.int64))
                units = [np.concatenate(x) for x in (uo, ul, to, tc)]
                launched.append(("members", mu, np.concatenate(owner), _gpu_inflate(dev, d_in, d_text, units, 1)))
            gpu_done = waiter.submit(lambda: (dev.sync(), time.perf_counter())[1])
        # CPU files meanwhile: sub-batches through two pinned stages, each
        # copied to HBM on the copy stream while the next one inflates
        c_bytes = 0
        pend = [None, None]
        i = sb = 0
        while i < len(on_cpu):
            grp, room = [], 0
            while i < len(on_cpu) and (not grp or room + _align(caps_[on_cpu[i]]) <= STAGE):
                grp.append(on_cpu[i])
                room += _align(caps_[on_cpu[i]])
                i += 1
            j = sb % 2
            sb += 1
            if pend[j] is not None:
                pend[j].result()
            stage = stages[j].get(room + 256)
            soff = np.zeros(len(grp) + 1, np.int64)
            soff[1:] = np.cumsum([_align(caps_[k]) for k in grp])

            def one(t, grp=grp, stage=stage, soff=soff):
                k = grp[t]
                v = buf[off[k]:off[k] + sizes[fs[k]]]
                return _abi.gunzip_host(v, stage[soff[t]:soff[t] + caps_[k]], with_crc=True)
            res = list(pool.map(one, range(len(grp))))
            for t, k in enumerate(grp):
                gst[k], tlen[k], hcrc[k] = res[t]
                c_bytes += int(tlen[k])

            def h2d(grp=grp, stage=stage, soff=soff, res=res):
                for t, k in enumerate(grp):
                    if res[t][0] == 0 and res[t][1]:
                        call("grid_h2d", cdev.ctx, d_text.ptr + int(toff[k]), stage.ctypes.data + int(soff[t]),
                             int(res[t][1]))
            pend[j] = copier.submit(h2d)
        t_cpu = time.perf_counter() - t0
        for p_ in pend:
            if p_ is not None:
                p_.result()
        if on_cpu and XSTREAM_WAIT:
            # the parse kernels on dev's stream read text the copy stream wrote
            # over d_text -- lines the previous batch's kernels had cached: order
            # the stream behind the copies through the runtime (event + wait), not
            # through the host's view of their completion alone
            call("grid_stream_after", dev.ctx, cdev.ctx)
        hk = [k for k in on_cpu if gst[k] == 0 and tlen[k] > 0]
        if hk:
            # the guard: the host-inflated text as it sits in HBM against the CRC
            # of its gzip trailers, read on dev's stream (where the parse runs)
            if AFTER_HOST_TEXT is not None:
                AFTER_HOST_TEXT(dev, d_text, toff, hk)
            got = _abi.text_crc32(dev, d_text.ptr, toff[hk], tlen[hk])
            bad = [fs[k] for k, c in zip(hk, got) if int(c) != int(hcrc[k])]
            if bad:
                raise DeviceIngestUnsupported(f"{paths[bad[0]]}: its text in HBM does not match its gzip CRC "
                                              f"({len(bad)} host-inflated file(s))")
        g_mem = g_whole = 0
        t_gpu = 0.0
        if launched:
            t_gpu = gpu_done.result() - t0
            for kind, ks, owner, (_d, _mem, st, ln, _nm) in launched:
                ust, uln = st.numpy(), ln.numpy()
                if kind == "whole":
                    gst[ks], tlen[ks] = ust, uln
                    g_whole = max(g_whole, int(uln.max()))
                else:
                    bad = np.zeros(nb, np.int32)
                    # a member past its BGZF size is corrupt (dropped), not several members
                    np.maximum.at(bad, owner, np.where(ust == _abi.GZ_ESPACE, _abi.GZ_EDATA, ust))
                    tot = np.zeros(nb, np.int64)
                    np.add.at(tot, owner, uln)
                    gst[ks], tlen[ks] = bad[ks], tot[ks]
                    g_mem += int(uln.sum())
        split.learn(g_mem, g_whole, t_gpu, c_bytes, t_cpu)
        if TRACE:
            import sys
            print(f"[ingest] batch files gpu {len(on_gpu)} cpu {len(on_cpu)} text gpu {g_mem + g_whole:.3e} "
                  f"cpu {c_bytes:.3e} B  t_gpu {t_gpu:.3f} t_cpu {t_cpu:.3f} s  rates gpu {split.gpu:.3e} "
                  f"cpu/thread {split.cpu:.3e} B/s", file=sys.stderr, flush=True)
        return gst, tlen

    K = kidx = Q = None
    nK = ref_nlines = 0
    if ref is not None:                    # the key list of another rank's reference file
        K_h, kidx_h, ref_nlines = ref
        nK = len(K_h)
        K = dev.upload(np.ascontiguousarray(K_h, np.int64).reshape(max(nK, 1), 2) if nK else np.zeros((1, 2), np.int64))
        kidx = dev.upload(np.ascontiguousarray(kidx_h, np.int32) if len(kidx_h) else np.zeros(1, np.int32))
        ref_nlines = int(ref_nlines)
        Q = dev.alloc((max(nfiles, 1), max(nK, 1)), np.int32)
        call("grid_fill_i32", dev.ctx, Q.ptr, max(nfiles, 1) * max(nK, 1), _abi.MISSING)
    d_text = None
    d_ins = [None, None]
    pipe = None
    pending = rpool.submit(read_batch, 0) if batches else None
    try:
        for bi, fs in enumerate(batches):
            t_w = time.perf_counter()
            buf, off, caps, members = pending.result()
            pending = rpool.submit(read_batch, bi + 1) if bi + 1 < len(batches) else None
            nb = len(fs)
            caps_ = np.array([c[0] if c else 0 for c in caps], np.int64)
            gz = np.array([c is not None for c in caps])
            tcap = np.array([_align(max(c, 1), 256) for c in caps_], np.int64)
            toff = np.zeros(nb + 1, np.int64)
            toff[1:] = np.cumsum(tcap)
            if toff[-1] > BATCH_TEXT * 2:
                raise DeviceIngestUnsupported("a batch of files inflates beyond the device text buffer")
            # device buffers sized from the cohort, not from the batch bounds: the
            # compressed bytes of the largest batch (known from the file sizes), the
            # text grown with 1/8 headroom as batches need it
            if d_ins[bi % 2] is None or d_ins[bi % 2].nbytes < off[-1] + 256:
                if pipe is not None:
                    pipe.drain()
                d_ins[bi % 2] = None
                d_ins[bi % 2] = dev.cached(f"ingest_in{bi % 2}", in_need if bi else int(off[-1]) + 256)
            if d_text is None or d_text.nbytes < toff[-1] + 256:
                if pipe is not None:
                    pipe.drain()
                d_text = None
                d_text = dev.cached("ingest_text", int(min(toff[-1] + 256 + toff[-1] // 8, 2 * BATCH_TEXT + 256)))
            d_in = d_ins[bi % 2]
            todo = [k for k in range(nb) if gz[k] and sizes[fs[k]] > 0]
            bgzf = {k: members[k] is not None for k in todo}
            plan = split.plan(todo, caps_, bgzf)
            if PIPELINE and K is not None and all(bgzf.values()) and not plan[1]:
                # every file BGZF (what mosdepth writes): the GPU inflates all of
                # them, and the batch is enqueued behind the previous one
                if pipe is None:
                    pipe = _Async(dev, cdev, opts, K, nK, kidx, ref_nlines, Q)
                hshare = None
                if hfrac > 0 and len(todo) > 1:
                    # every step-th file to the host threads (they start now, beside the
                    # GPU's work on the previous batch and this batch's copies)
                    step = max(2, int(round(1.0 / hfrac)))
                    hfiles = todo[step - 1::step]
                    so, pos = {}, 0
                    for k in hfiles:
                        so[k] = pos
                        pos += _align(int(caps_[k]))
                    harr = hstages[bi % 2].get(pos + 256)

                    def run_host(hfiles=hfiles, harr=harr, so=so, buf=buf, off=off, fs=fs, caps_=caps_):
                        def one(k):
                            v = buf[off[k]:off[k] + sizes[fs[k]]]
                            st_, ln_, crc_ = _abi.gunzip_host(v, harr[so[k]:so[k] + int(caps_[k])], with_crc=True)
                            return k, (int(st_), int(ln_), int(crc_), harr, so[k])
                        return dict(pool.map(one, hfiles))
                    hshare = (hfiles, hctl.submit(run_host))
                h2d_done[bi] = pipe.batch(bi, fs, buf, off, caps_, gz, members, toff, d_in, d_text,
                                          [sizes[f] for f in fs], hshare=hshare)
                if TRACE:
                    import sys
                    print(f"[ingest] batch {bi}: {nb} files enqueued, wait read {time.perf_counter() - t_w:.3f} s "
                          f"(at {time.perf_counter() - t_start:.3f})", file=sys.stderr, flush=True)
                continue
            if pipe is not None:
                pipe.drain()
            t_b = time.perf_counter()
            gst, tlen = inflate(buf, off, fs, caps_, gz, members, toff, d_in, d_text, plan)
            t_i = time.perf_counter()
            for k, f in enumerate(fs):
                if gst[k] == _abi.GZ_ESPACE:
                    raise DeviceIngestUnsupported(f"{paths[f]}: several gzip members (text size unknown)")
                status[f] = 0 if gst[k] == 0 else 1        # 1: failed (the reference drops the sample)
            okb = [k for k in range(nb) if gst[k] == 0 and tlen[k] > 0]
            cfile, cstart, cfirst, nch = _chunks(okb, tlen)
            if nch == 0:
                continue
            d_tl, d_toff = dev.upload(tlen), dev.upload(toff[:nb])
            d_cfile, d_cstart, d_cfirst = dev.upload(cfile), dev.upload(cstart), dev.upload(cfirst)
            cnl, cline0 = dev.alloc(nch, np.int32), dev.alloc(nch, np.int64)
            # flags per batch file, folded into the cohort's afterwards
            bflags = dev.zeros(nb, np.int32)
            call("grid_md_count", dev.ctx, d_text.ptr, d_toff.ptr, d_tl.ptr, nch, d_cfile.ptr, d_cstart.ptr,
                 d_cfirst.ptr, len(okb), cnl.ptr, cline0.ptr, bflags.ptr, None)
            if K is None:
                # the reference key list: the first batch's file with the most
                # text (a short or truncated file sorted first
                # no longer sends the cohort to the host parser; K must hold
                # every later file's keys, which the largest file does)
                ri = int(np.argmax(tlen[okb]))
                r = okb[ri]
                c0, c1 = int(cfirst[ri]), int(cfirst[ri + 1])
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
                if keys_only:
                    break
                Q = dev.alloc((nfiles, nK), np.int32)
                call("grid_fill_i32", dev.ctx, Q.ptr, nfiles * nK, _abi.MISSING)
            qrow = dev.upload(np.asarray(fs, np.int32))
            bk = dev.zeros(nb, np.uint64)
            call("grid_md_parse_map", dev.ctx, d_text.ptr, d_toff.ptr, d_tl.ptr, nch, d_cfile.ptr, d_cstart.ptr,
                 cline0.ptr, C.byref(opts), bflags.ptr, K.ptr, nK, kidx.ptr, ref_nlines, Q.ptr, nK, qrow.ptr, bk.ptr,
                 None)
            bf, bkv = bflags.numpy(), bk.numpy()
            for k in okb:
                if bf[k]:
                    why = "a line outside the mosdepth grammar" if bf[k] & _abi.MD_EXOTIC else "a key outside K"
                    raise DeviceIngestUnsupported(f"{paths[fs[k]]}: {why}")
            kept_h = kept.numpy()
            kept_h[np.asarray(fs)] += bkv
            kept.copy_from(kept_h)
            if TRACE:
                import sys
                print(f"[ingest] batch {bi}: {nb} files, wait read {t_b - t_w:.3f} inflate {t_i - t_b:.3f} "
                      f"parse {time.perf_counter() - t_i:.3f} s (at {time.perf_counter() - t_start:.3f})",
                      file=sys.stderr, flush=True)
        if pipe is not None:
            t_d = time.perf_counter()
            pipe.drain()
            for f, st_, kp in pipe.results(paths):
                status[f] = st_
            kept_h = kept.numpy()
            kept_h += pipe.kept_total(nfiles)
            kept.copy_from(kept_h)
            if TRACE:
                import sys
                print(f"[ingest] pipeline drained in {time.perf_counter() - t_d:.3f} s", file=sys.stderr, flush=True)
    finally:
        if pending is not None:
            try:
                pending.result()
            except Exception:
                pass
        if pipe is not None:
            pipe.close()
        rpool.shutdown(wait=True)
        iopool.shutdown(wait=True)
        pool.shutdown(wait=True)
        copier.shutdown(wait=True)
        waiter.shutdown(wait=True)
        hctl.shutdown(wait=True)
        cdev.close()
    if TRACE:
        import sys
        print(f"[ingest] batches done (threads joined, copy context closed) at {time.perf_counter() - t_start:.3f} s",
              file=sys.stderr, flush=True)
    # the batches' device buffers stay cached on the context (Device.cached,
    # names "ingest_*") and the host staging in _STAGING until
    # device.release_ingest_buffers() -- the end of the run or of a standalone
    # step 4 -- since their release holds the HIP runtime for a fraction of a
    # second; here only this function's references go
    d_ins = d_text = d_in = pipe = None
    if TRACE:
        import sys
        print(f"[ingest] input/text buffers freed at {time.perf_counter() - t_start:.3f} s", file=sys.stderr,
              flush=True)
    if keys_only:
        if K is None:
            return None
        return K.numpy()[:nK].copy(), kidx.numpy()[:max(ref_nlines, 0)].copy(), ref_nlines
    if not finish:
        return Q, nK, status, kept.numpy()[:nfiles].copy()
    if K is None:
        return [], [], None, status
    rows = np.array([f for f in range(nfiles) if status[f] == 0], np.int32)
    mean = dev.alloc(nK, np.float64)
    valid, cpos = dev.alloc(nK, np.int32), dev.alloc(nK, np.int64)
    present, nvalid = dev.alloc(max(nfiles, 1), np.uint64), dev.alloc(max(nfiles, 1), np.uint64)
    m = C.c_int64()
    if TRACE:
        import sys
        print(f"[ingest] finish buffers at {time.perf_counter() - t_start:.3f} s", file=sys.stderr, flush=True)
    d_rows = dev.upload(rows if rows.size else np.zeros(1, np.int32))
    call("grid_md_finish", dev.ctx, Q.ptr, nK, nK, nfiles, d_rows.ptr, len(rows), float(min_depth),
         float(max_depth), mean.ptr, valid.ptr, cpos.ptr, present.ptr, nvalid.ptr, C.byref(m))
    pres, nval, kh = present.numpy()[:nfiles], nvalid.numpy()[:nfiles], kept.numpy()[:nfiles]
    if np.any(pres[rows] != kh[rows]):
        raise DeviceIngestUnsupported("a repeated (start, end) key in a file")
    m = m.value
    if TRACE:
        import sys
        print(f"[ingest] finish done at {time.perf_counter() - t_start:.3f} s", file=sys.stderr, flush=True)
    return rows, (Q, nK, valid, cpos, K, m), nval, status


class Regions(Sequence):
    """The valid columns' (start, end) pairs as a read-only sequence built on
    demand from two int64 arrays (a list of 3 M tuples costs ~1 s, and the
    step itself never needs it)."""

    def __init__(self, starts, ends):
        self.s, self.e = starts, ends

    def __len__(self):
        return len(self.s)

    def __getitem__(self, k):
        if isinstance(k, slice):
            return list(zip(self.s[k].tolist(), self.e[k].tolist()))
        return int(self.s[k]), int(self.e[k])

    def __iter__(self):
        return zip(self.s.tolist(), self.e.tolist())

    def __eq__(self, other):
        try:
            return len(self) == len(other) and list(self) == list(other)
        except TypeError:
            return NotImplemented

    __hash__ = None


def gather(dev, state, row_files, nfiles):
    """The matrix rows of ``row_files`` (file indices, in output order) and
    the valid columns' (start, end)."""
    Q, nK, valid, cpos, K, m = state
    if m == nK and m > 0 and len(row_files) == nfiles and np.array_equal(np.asarray(row_files), np.arange(nfiles)):
        # every key valid and every file a row, already in output order: the
        # placed matrix IS the result (no 38 GB copy at config 2)
        kh = K.numpy()[:m]
        Q.shape = (nfiles, m)
        return Q, Regions(np.ascontiguousarray(kh[:, 0]), np.ascontiguousarray(kh[:, 1]))
    t0 = time.perf_counter()
    dst = np.full(max(nfiles, 1), -1, np.int32)
    dst[np.asarray(row_files, np.int64)] = np.arange(len(row_files), dtype=np.int32)
    out = dev.alloc((max(len(row_files), 1), max(m, 1)), np.int32)
    st, en = dev.alloc(max(m, 1), np.int64), dev.alloc(max(m, 1), np.int64)
    t1 = time.perf_counter()
    d_dst = dev.upload(dst)
    call("grid_md_gather", dev.ctx, Q.ptr, nK, nK, nfiles, valid.ptr, cpos.ptr, d_dst.ptr, out.ptr,
         max(m, 1), K.ptr, st.ptr, en.ptr)
    regions = Regions(st.numpy()[:m], en.numpy()[:m])
    if TRACE:
        import sys
        print(f"[ingest] gather: {len(row_files)} of {nfiles} rows, {m} of {nK} columns; alloc "
              f"{t1 - t0:.3f} s, gather {time.perf_counter() - t1:.3f} s", file=sys.stderr, flush=True)
    out.shape = (len(row_files), m)            # the allocation keeps >= 1 element
    return out, regions
