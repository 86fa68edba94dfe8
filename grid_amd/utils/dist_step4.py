"""Steps 4-5 of `grid wgs` across the GPUs of a node (one process per GPU,
launched by torch.distributed.run; the default process group carries RCCL
over xGMI).

Reference: grid/pipeline.py:66-103 runs normalize_mosdepth and
find_neighbors in one process; grid/utils/normalize_mosdepth.py:96-123 reads
every sample's regions.bed.gz, :419-476 normalises the matrix, :502-554
writes it; grid/utils/find_neighbors.py:204-213 runs the all-pairs search.
Here the cohort is split twice:

  * by FILES for the ingest -- rank r inflates and parses a contiguous slice
    of the files (in file order, balanced by compressed bytes) into its own
    [files][K] int32 hundredths matrix over the reference key list K (rank 0
    reads K from the first batch and broadcasts it);
  * the population means (:218-301, fp64 sums in file order) are a chain
    over the ranks: rank r continues rank r-1's (sum, count) over its rows
    and passes them on (grid_md_popsum, point-to-point), the last rank's
    totals give the valid columns (grid_md_popvalid), broadcast;
  * by BINS for the statistics: ONE all-to-all moves every rank's rows of
    the valid columns to the owners of 8192-aligned column shards
    (grid_md_pack_shards; fused.shard_range), where the rows are put in
    sorted-ID order; the chain fused.Steps47 then runs steps 4-5 exactly as
    the bench's multi-GPU chain does (row-block partials all-gathered, column
    statistics local, the selection from all-gathered ratios, the Gram's
    upper-triangle segments reduce-scattered, candidate lists all-gathered
    and merged: the same neighbours on every rank);
  * by ROWS for the writer: a second all-to-all brings each rank the z rows
    [n t / W, n (t+1) / W) of every column; each rank codes its rows as gzip
    members in host memory (grid_gz_parts_rows_dev), the ranks exchange their
    byte counts and write at the exclusive prefix sum (rank 0 first writes
    member 0, the header lines).

Every integer sum is order-free and every fp64 sum keeps the reference's
order, so the files equal the one-GPU run's after gunzip (and the
reference's).  Anything outside this path's common case -- the device
ingest handing over, a float window, zmax that is not hundredths, a
repeated key -- is agreed on by all ranks and rank 0 then runs the one-GPU
step (the others wait): slower, never different.

The chain is written against a ``backend`` (HipBackend: libgridhip.so
kernels on this rank's GPU; the tests substitute a CPU restatement to run it
under gloo without a GPU).
"""
from __future__ import annotations

import os
import sys

import numpy as np

from .. import _abi

I4, I8, F8 = np.int32, np.int64, np.float64

# wall seconds per phase of the last normalize_dist on this rank (bench.py reports rank 0's)
LAST_PHASES: dict = {}


class DistFallback(Exception):
    """Every rank agreed to leave the distributed path (rank 0 runs the one-GPU step)."""


# ------------------------------------------------------------ process group --
def dist_comm():
    """The TorchComm of an initialised default process group with more than
    one rank, else None.  Never imports torch just to ask."""
    dist = sys.modules.get("torch.distributed")
    if dist is None or not dist.is_available() or not dist.is_initialized() or dist.get_world_size() < 2:
        return None
    from ..fused import TorchComm
    return TorchComm(dist)


def init_from_env():
    """Under torch.distributed.run (WORLD_SIZE > 1 in the environment) start
    the default process group once: RCCL ("nccl") with this rank's GPU
    (LOCAL_RANK), or GRID_DIST_BACKEND (gloo: ranks sharing one GPU in a
    rehearsal).  Returns the TorchComm or None at one rank."""
    if int(os.environ.get("WORLD_SIZE", "1")) < 2:
        return None
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        backend = os.environ.get("GRID_DIST_BACKEND", "nccl")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return dist_comm()


def _ctl_dev(comm):
    """Where the control tensors of a collective live: this rank's GPU for
    RCCL, the host for gloo."""
    import torch
    if comm.dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _ctl(comm, vals, dtype=I8):
    """A small control tensor on the collective's device."""
    import torch
    return torch.tensor(np.asarray(vals, dtype=dtype), device=_ctl_dev(comm))


def agree(comm, ok):
    """True iff every rank passes ok=True."""
    t = _ctl(comm, [0 if ok else 1])
    comm.all_reduce_sum(t)
    return int(t.cpu()[0]) == 0


def gather_rows(comm, arr, maxlen, fill=-1):
    """All ranks' 1-D int64 arrays (each <= maxlen long) -> list of arrays."""
    import torch
    a = np.asarray(arr, dtype=I8)
    buf = np.full(max(maxlen, 1) + 1, fill, dtype=I8)
    buf[0] = len(a)
    buf[1:1 + len(a)] = a
    g = comm.all_gather(torch.from_numpy(buf).to(_ctl_dev(comm))).cpu().numpy()
    return [g[q, 1:1 + int(g[q, 0])].copy() for q in range(comm.world)]


def gather_f64(comm, arr, maxlen):
    """All ranks' 1-D float64 arrays (each <= maxlen long), concatenated in rank order."""
    import torch
    a = np.asarray(arr, dtype=F8)
    lens = gather_rows(comm, [len(a)], 1)
    buf = np.zeros(max(maxlen, 1), dtype=F8)
    buf[:len(a)] = a
    g = comm.all_gather(torch.from_numpy(buf).to(_ctl_dev(comm))).cpu().numpy()
    return np.concatenate([g[q, :int(lens[q][0])] for q in range(comm.world)])


def rank0_step(comm, fn):
    """Run ``fn`` on rank 0 only; every rank leaves together (a SystemExit on
    rank 0 -- the reference's sys.exit(1) -- ends every rank the same way;
    an exception propagates on rank 0 after the others are released)."""
    code, err = 0, None
    if comm.rank == 0:
        try:
            fn()
        except SystemExit as e:
            code = int(e.code) if isinstance(e.code, int) else 1
            code = code or 0
            err = e
        except BaseException as e:          # noqa: BLE001 -- re-raised below, after the others are released
            err = e
    t = _ctl(comm, [code])
    comm.all_reduce_sum(t)
    code = int(t.cpu()[0])
    if err is not None and not isinstance(err, SystemExit):
        raise err
    if code:
        sys.exit(code)


# ------------------------------------------------------------------ backend --
# test seam: the CPU tests set this to build their restatement of the backend
# (tests/dist_cpu_backend.py); the product always builds HipBackend
BACKEND_FACTORY = None


def make_backend(config):
    if BACKEND_FACTORY is not None:
        return BACKEND_FACTORY(config)
    from ..device import get_device
    return HipBackend(get_device(config))


class HipBackend:
    """The distributed step's compute on this rank's GPU: the device ingest,
    the grid_md_* chain kernels, fused.HipOps for steps 4-5, the device
    writer.  Torch tensors and the library's kernels share one stream."""

    def __init__(self, dev):
        import torch
        from ..fused import HipOps, TorchAlloc
        self.torch = torch
        self.dev = dev
        self.stream = torch.cuda.Stream(device=dev.index)
        dev.set_stream(self.stream)
        self.alloc = TorchAlloc(dev.index)
        self.ops = HipOps(dev)

    def stream_ctx(self):
        return self.torch.cuda.stream(self.stream)

    def ref_keys(self, paths, prefix, window, excluded, min_depth, max_depth, threads):
        from . import ingest_device
        return ingest_device.ingest_device(self.dev, paths, prefix, window, excluded, min_depth, max_depth,
                                           threads=threads, keys_only=True)

    def ingest(self, paths, ref, prefix, window, excluded, min_depth, max_depth, threads):
        from . import ingest_device
        Q, nK, status, kept = ingest_device.ingest_device(self.dev, paths, prefix, window, excluded, min_depth,
                                                          max_depth, threads=threads, ref=ref, finish=False)
        return Q, status, kept

    def free(self, Q):
        if isinstance(Q, _abi.DevBuf):
            Q.free()

    def popsum(self, Q, nK, rows, s, c):
        if len(rows) and nK:
            d_rows = self.alloc.upload(np.asarray(rows, I4))
            _abi.call("grid_md_popsum", self.dev.ctx, _abi.ptr(Q), nK, nK, _abi.ptr(d_rows), len(rows),
                      _abi.ptr(s), _abi.ptr(c))

    def popvalid(self, s, c, nK, min_depth, max_depth, valid):
        _abi.call("grid_md_popvalid", self.dev.ctx, _abi.ptr(s), _abi.ptr(c), nK, float(min_depth),
                  float(max_depth), _abi.ptr(valid))

    def rowstats(self, Q, nK, nfiles, valid):
        """-> (cpos tensor, present, nvalid host arrays, m)."""
        import ctypes as C
        cpos = self.alloc.empty(max(nK, 1), I8)
        present = self.alloc.empty(max(nfiles, 1), I8)
        nvalid = self.alloc.empty(max(nfiles, 1), I8)
        m = C.c_int64()
        _abi.call("grid_md_rowstats", self.dev.ctx, _abi.ptr(Q), nK, nK, nfiles, _abi.ptr(valid), _abi.ptr(cpos),
                  _abi.ptr(present), _abi.ptr(nvalid), C.byref(m))
        return cpos, present.cpu().numpy()[:nfiles], nvalid.cpu().numpy()[:nfiles], m.value

    def pack(self, Q, nK, valid, cpos, src_rows, bounds):
        """[rows][width_s] blocks of every shard s, one int32 tensor."""
        nrows, m = len(src_rows), int(bounds[-1])
        out = self.alloc.empty(max(nrows * m, 1), I4)
        if nrows and m:
            d_src = self.alloc.upload(np.asarray(src_rows, I4))
            d_b = self.alloc.upload(np.asarray(bounds, I8))
            _abi.call("grid_md_pack_shards", self.dev.ctx, _abi.ptr(Q), nK, nK, _abi.ptr(valid), _abi.ptr(cpos),
                      _abi.ptr(d_src), nrows, _abi.ptr(d_b), len(bounds) - 1, _abi.ptr(out))
        return out

    def parts_rows(self, parts, ids, raw, z32, row0):
        n, r = z32.shape
        parts.rows_dev(self.dev, ids, raw, z32, n, r, r, row0)

    def sync(self):
        self.torch.cuda.synchronize(self.dev.index)


# ---------------------------------------------------------------- the step --
def file_slices(sizes, world):
    """Contiguous file ranges [b[r], b[r+1]) balanced by compressed bytes."""
    nf = len(sizes)
    sz = np.maximum(np.asarray(sizes, dtype=F8), 0.0) + 1.0        # +1: empty files still count
    start = np.concatenate([[0.0], np.cumsum(sz)[:-1]]) if nf else np.zeros(0)
    tot = float(sz.sum()) if nf else 0.0
    b = [0] + [int(np.searchsorted(start, tot * r / world, side="left")) for r in range(1, world)] + [nf]
    for r in range(1, world + 1):
        b[r] = max(b[r], b[r - 1])
    return b


def row_blocks(n, world):
    return [n * t // world for t in range(world + 1)]


def _codes_to_i32(torch, blk):
    """int16 step-4 codes -> int32 hundredths (sentinels; escapes stay as the code)."""
    z = blk.to(torch.int32)
    z[blk == _abi.ZQ16_NAN] = _abi.ZQ_NAN
    z[blk == _abi.ZQ16_NEG0] = _abi.ZQ_NEG0
    return z


def _write_parts(comm, parts, output_path):
    """Every rank's coded bytes at the exclusive prefix sum of the ranks'
    byte counts (rank 0 sizes the file first); returns once the file is
    complete on every rank."""
    sizes_b = [int(x[0]) for x in gather_rows(comm, [parts.size()], 1)]
    if comm.rank == 0:
        fd = os.open(str(output_path), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        os.ftruncate(fd, sum(sizes_b))
        os.close(fd)
    comm.barrier()
    parts.write(output_path, sum(sizes_b[:comm.rank]))
    comm.barrier()


def normalize_dist(comm, backend, *, individuals, mosdepth_dir, chromosome, start, end, excluded, min_depth,
                   max_depth, top_frac, threads, output_path, nbr_params, console=None):
    """Steps 4 (and 5, when ``nbr_params`` is given: dict zmax, sigma2_max,
    frac_r, n_neighbors) of the cohort over every rank.  Returns the
    hand-off record for step 5 (``handoff.publish_neighbors``) or raises
    DistFallback (agreed by all ranks)."""
    import time
    from ..fused import Steps47, shard_range
    from .normalize_mosdepth import find_bed_gz_paths, norm_chrom
    from .utils import log
    torch = backend.torch
    LAST_PHASES.clear()
    clock = [time.perf_counter()]

    def mark(name):
        backend.sync()
        t = time.perf_counter()
        LAST_PHASES[name] = LAST_PHASES.get(name, 0.0) + t - clock[0]
        clock[0] = t
    W, rank = comm.world, comm.rank
    inds = list(individuals)
    where = find_bed_gz_paths(inds, mosdepth_dir)
    paths = [str(where[i]) if where[i].exists() else None for i in inds]
    sizes = [os.path.getsize(p) if p else 0 for p in paths]
    fb = file_slices(sizes, W)
    f0, f1 = fb[rank], fb[rank + 1]
    prefix = norm_chrom(chromosome) if chromosome else None
    window = (start, end) if start is not None and end is not None else None
    ints = all(v is None or (isinstance(v, int) and not isinstance(v, bool)) for v in (start, end))
    if not agree(comm, ints):
        raise DistFallback("the window is not integer base pairs")
    from .ingest_device import DeviceIngestUnsupported

    # ---- the reference key list K: rank 0's first batch, broadcast ----
    ok, ref = True, None
    if rank == 0:
        try:
            ref = backend.ref_keys(paths, prefix, window, excluded, min_depth, max_depth, threads)
        except (DeviceIngestUnsupported, _abi.GridNativeError) as e:
            log(console, f"distributed ingest: {e}; rank 0 reads the cohort", style="warning")
            ok = False
    if not agree(comm, ok):
        raise DistFallback("reference keys")
    hdr = _ctl(comm, [-1, 0] if ref is None else [len(ref[0]), int(ref[2])])
    comm.broadcast(hdr, 0)
    nK, ref_nlines = (int(x) for x in hdr.cpu().numpy())
    if nK < 0:
        return None                                  # no file inflates: no samples (every rank)
    Kt = backend.alloc.empty((max(nK, 1), 2), I8)
    kt = backend.alloc.empty(max(ref_nlines, 1), I4)
    if rank == 0:
        Kt[:nK].copy_(torch.from_numpy(np.ascontiguousarray(ref[0], I8)))
        kt[:ref_nlines].copy_(torch.from_numpy(np.ascontiguousarray(ref[1], I4)))
    comm.broadcast(Kt, 0)
    comm.broadcast(kt, 0)
    ref = (Kt[:nK].cpu().numpy(), kt[:ref_nlines].cpu().numpy(), ref_nlines)
    del Kt, kt
    mark("keys")

    # ---- this rank's files over K ----
    ok, Q = True, None
    try:
        Q, status, kept = backend.ingest(paths[f0:f1], ref, prefix, window, excluded, min_depth, max_depth, threads)
    except (DeviceIngestUnsupported, _abi.GridNativeError) as e:
        log(console, f"distributed ingest on rank {rank}: {e}; rank 0 reads the cohort", style="warning")
        ok = False
    if not agree(comm, ok):
        if Q is not None:
            backend.free(Q)
        raise DistFallback("ingest")
    nf = f1 - f0
    rows_local = [f for f in range(nf) if status[f] == 0]
    mark("ingest")

    # ---- population sums: a chain over the ranks in file order ----
    s = backend.alloc.empty(max(nK, 1), F8)
    c = backend.alloc.empty(max(nK, 1), I8)
    if rank == 0:
        s.zero_()
        c.zero_()
    else:
        comm.recv(s, rank - 1)
        comm.recv(c, rank - 1)
    backend.popsum(Q, nK, rows_local, s, c)
    if rank < W - 1:
        comm.send(s, rank + 1)
        comm.send(c, rank + 1)
    valid = backend.alloc.empty(max(nK, 1), I4)
    if rank == W - 1:
        backend.popvalid(s, c, nK, min_depth, max_depth, valid)
    comm.broadcast(valid, W - 1)
    del s, c
    mark("popsum_chain")
    cpos, present, nval, m = backend.rowstats(Q, nK, nf, valid)
    dup = any(int(present[f]) != int(kept[f]) for f in rows_local)
    if not agree(comm, not dup):
        backend.free(Q)
        raise DistFallback("a repeated (start, end) key in a file")

    # ---- the cohort's rows: sorted IDs of the files that read and keep a record ----
    maxnf = max(fb[q + 1] - fb[q] for q in range(W))
    keep_local = [f for f in range(nf) if status[f] == 0 and nval[f] > 0]
    kl = gather_rows(comm, [f0 + f for f in keep_local], maxnf)
    keep_files = sorted(int(x) for a in kl for x in a)
    removed = len(inds) - len(keep_files)
    if removed > 0 and rank == 0:                   # filter_empty_samples (:576-600)
        msg = f"Removed {removed} samples with 0 regions"
        log(console, msg, style="warning") if console else print(msg)
    ids = sorted(inds[f] for f in keep_files)
    n = len(ids)
    if n == 0:
        backend.free(Q)
        return None
    row_of = {inds[f]: i for i, f in enumerate(sorted(keep_files, key=lambda f: inds[f]))}
    grow = {f: row_of[inds[f]] for f in keep_files}
    # sender order: every rank's kept files by global row; the receiver's rows
    # come in rank order, each rank's ascending
    send_files = [[f for f in sorted((int(x) for x in kl[q]), key=lambda f: grow[f])] for q in range(W)]
    recv_rows = np.array([grow[f] for q in range(W) for f in send_files[q]], dtype=I8)
    bounds = [shard_range(m, q, W)[0] for q in range(W)] + [m]
    c0, c1 = bounds[rank], bounds[rank + 1]
    ml = c1 - c0
    src_local = [f - f0 for f in send_files[rank]]
    mark("rows")
    send = backend.pack(Q, nK, valid, cpos, src_local, bounds)
    backend.free(Q)
    del Q, valid, cpos
    nr_send = len(src_local)
    in_splits = [nr_send * (bounds[s_ + 1] - bounds[s_]) for s_ in range(W)]
    out_splits = [len(send_files[q]) * ml for q in range(W)]
    recv = backend.alloc.empty(max(n * ml, 1), I4)
    comm.all_to_all(recv, send, out_splits, in_splits)
    del send
    q = backend.alloc.empty((n, max(ml, 1)), I4)
    if ml:
        idx = torch.from_numpy(recv_rows).to(q.device)
        q.index_copy_(0, idx, recv[: n * ml].view(n, ml))
    del recv
    mark("to_column_shards")

    # ---- steps 4-5 on this rank's column shard (fused.Steps47, bin split) ----
    upto = "step4"
    zmax = 2.0
    kk = 10
    if nbr_params is not None:
        from ..engine import qmax_for_zmax
        try:
            qmax_for_zmax(nbr_params["zmax"])
            upto, zmax, kk = "step5", nbr_params["zmax"], int(nbr_params["n_neighbors"])
        except _abi.GridNativeError:
            upto = "step4"                           # step 5 reads the file on rank 0 (the general k-NN paths)
    st = Steps47(backend.ops, backend.alloc, n, m, c0, ml, k=kk, top_frac=top_frac, zmax=zmax,
                 sigma2_max=float(nbr_params["sigma2_max"]) if nbr_params else 1000.0,
                 frac_r=float(nbr_params["frac_r"]) if nbr_params else 1.0, comm=comm, keep_z=True, split="bin")
    st.run(q, max(ml, 1), upto=upto)
    del q
    mark("steps4_5")

    # ---- header values: the selected columns' means and "%.3f" ratios, in column order ----
    r_loc = st.r_loc
    sel = st.sel[:r_loc].cpu().numpy()
    mu, var = st.mu[:max(ml, 1)].cpu().numpy(), st.var[:max(ml, 1)].cpu().numpy()
    r_locs = [int(x[0]) for x in gather_rows(comm, [r_loc], 1)]
    rmax = max(r_locs)
    sel_means = gather_f64(comm, mu[sel] if r_loc else np.zeros(0), rmax)
    sel_vars = gather_f64(comm, var[sel] if r_loc else np.zeros(0), rmax)
    r_tot = sum(r_locs)
    with np.errstate(invalid="ignore", divide="ignore"):
        sel_ratios = np.where(sel_means > 0, 100.0 * sel_vars / sel_means, np.nan)
    raw = st.rm[:n].cpu().numpy()

    # ---- z rows of this rank: [n t / W, n (t+1) / W) of every column ----
    rb = row_blocks(n, W)
    a, b = rb[rank], rb[rank + 1]
    nr = b - a
    z16 = agree(comm, st.zq_is16)
    ld = max(ml, 1)
    if z16:
        zl = st.zq16.view(-1)[: n * ld].view(n, ld)[:, :r_loc]
    else:
        zl = st.zq_int32().view(-1)[: n * ld].view(n, ld)[:, :r_loc]
    send = torch.cat([zl[rb[t]:rb[t + 1]].reshape(-1) for t in range(W)]) if r_loc else zl.new_zeros(1)
    recv = zl.new_empty(max(nr * r_tot, 1))
    comm.all_to_all(recv, send, [nr * r_locs[qq] for qq in range(W)],
                    [(rb[t + 1] - rb[t]) * r_loc for t in range(W)])
    del send, zl
    z32 = backend.alloc.empty((max(nr, 1), max(r_tot, 1)), I4)
    off, col = 0, 0
    for qq in range(W):
        w = r_locs[qq]
        if w and nr:
            blk = recv[off: off + nr * w].view(nr, w)
            z32[:nr, col:col + w].copy_(_codes_to_i32(torch, blk) if z16 else blk)
        off += nr * w
        col += w
    del recv
    if z16:
        # int16 escapes (|z| > 327.65: exact in the escape list): every rank's
        # list as (row, global column, value), this rank applies its rows'
        ne = st.nesc
        e_idx = st.esc_idx[:ne].cpu().numpy() if ne else np.zeros(0, I8)
        e_val = st.esc_val[:ne].cpu().numpy().astype(I8) if ne else np.zeros(0, I8)
        cum0 = sum(r_locs[:rank])
        loc = np.stack([e_idx // ld, e_idx % ld + cum0, e_val], axis=1).reshape(-1) if ne else np.zeros(0, I8)
        nes = gather_rows(comm, [ne], 1)
        allv = gather_rows(comm, loc, 3 * max(int(x[0]) for x in nes))
        for arr in allv:
            if len(arr):
                e = arr.reshape(-1, 3)
                e = e[(e[:, 0] >= a) & (e[:, 0] < b)]
                if len(e):
                    ri = torch.from_numpy(e[:, 0] - a).to(z32.device)
                    ci = torch.from_numpy(e[:, 1]).to(z32.device)
                    z32[ri, ci] = torch.from_numpy(e[:, 2].astype(I4)).to(z32.device)

    # ---- the file: member 0 on rank 0, then every rank's rows at its offset ----
    mark("to_row_blocks")
    parts = _abi.GzParts()
    try:
        if rank == 0:
            parts.header(n, sel_means, sel_ratios, level=1)
        if nr:
            backend.parts_rows(parts, ids[a:b], raw[a:b], z32[:nr, :r_tot] if r_tot else z32[:nr, :0], a)
        del z32
        mark("code_rows")
        _write_parts(comm, parts, output_path)
        mark("write")
    finally:
        parts.free()

    # ---- step 5's result, the same on every rank ----
    nb = None
    if upto == "step5":
        ruse = _ctl(comm, [st.ruse_loc])
        comm.all_reduce_sum(ruse)
        idx = st.idx_out[:n].cpu().numpy()
        d2 = st.d2[:n].cpu().numpy()
        cnt = st.cnt_out[:n].cpu().numpy()
        nb = {"idx": idx, "d2": d2, "cnt": cnt, "R_use": int(ruse.cpu()[0]), "params": dict(nbr_params)}
    scales = np.array([float(f"{x:.2f}") for x in raw])
    return {"ids": ids, "scales": scales, "n": n, "r": r_tot, "neighbors": nb}
