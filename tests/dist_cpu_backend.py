"""CPU restatement of grid_amd.utils.dist_step4.HipBackend for tests: the
distributed `grid wgs` steps 4-5 (ingest slice, population-sum chain, the
all-to-all to column shards, fused.Steps47, the row-sharded writer) run under
torch.distributed/gloo without a GPU.  The ingest is the drop-in's
line-by-line parser (normalize_mosdepth._read_regions: the reference's
filters) over a key list of every kept key; steps 4-5 are tests/cpu_ops.py;
the writer is the host C++ member coder (grid_gz_parts_rows).  TEST
INFRASTRUCTURE ONLY -- the product always builds HipBackend."""
import contextlib

import numpy as np
import torch

from grid_amd import _abi
from grid_amd.fused import TorchAlloc
from tests.cpu_ops import NumpyOps

MISSING = -(2 ** 31)


class CpuBackend:
    def __init__(self, config=None):
        self.torch = torch
        self.alloc = TorchAlloc("cpu")
        self.ops = NumpyOps()

    def stream_ctx(self):
        return contextlib.nullcontext()

    def _records(self, path, prefix, window, excluded):
        from grid_amd.utils.normalize_mosdepth import _read_regions
        start, end = window if window else (None, None)
        return _read_regions(path, prefix, start, end, excluded)

    def ref_keys(self, paths, prefix, window, excluded, min_depth, max_depth, threads):
        keys = set()
        for p in paths:
            if p is None:
                continue
            try:
                keys.update(self._records(p, prefix, window, excluded))
            except Exception:
                pass
        if not keys:
            return None
        K = np.array(sorted(keys), dtype=np.int64).reshape(-1, 2)
        return K, np.zeros(0, np.int32), 0

    def ingest(self, paths, ref, prefix, window, excluded, min_depth, max_depth, threads):
        from grid_amd.utils.ingest_device import DeviceIngestUnsupported
        K = ref[0]
        kpos = {(int(s), int(e)): j for j, (s, e) in enumerate(K)}
        nf, nK = len(paths), len(K)
        Q = np.full((max(nf, 1), max(nK, 1)), MISSING, dtype=np.int32)
        status = np.zeros(nf, np.int32)
        kept = np.zeros(nf, np.uint64)
        for f, p in enumerate(paths):
            if p is None:
                status[f] = 3
                continue
            try:
                rec = self._records(p, prefix, window, excluded)
            except Exception:
                status[f] = 1
                continue
            for key, d in rec.items():
                j = kpos.get(key)
                if j is None:
                    raise DeviceIngestUnsupported(f"{p}: a key outside K")
                q = round(d * 100)
                if q / 100.0 != d:
                    raise DeviceIngestUnsupported(f"{p}: a depth that is not hundredths")
                Q[f, j] = q
            kept[f] = len(rec)
        return torch.from_numpy(Q), status, kept

    def free(self, Q):
        pass

    def popsum(self, Q, nK, rows, s, c):
        q = Q.numpy()
        sa, ca = s.numpy(), c.numpy()
        for r in rows:
            v = q[r, :nK]
            m = v != MISSING
            sa[:nK][m] = sa[:nK][m] + v[m] / 100.0
            ca[:nK][m] += 1

    def popvalid(self, s, c, nK, min_depth, max_depth, valid):
        sa, ca = s.numpy()[:nK], c.numpy()[:nK]
        with np.errstate(invalid="ignore", divide="ignore"):
            mean = np.where(ca > 0, sa / np.maximum(ca, 1), 0.0)
        valid.numpy()[:nK] = (ca > 0) & (min_depth <= mean) & (mean <= max_depth)

    def rowstats(self, Q, nK, nfiles, valid):
        q = Q.numpy()[:nfiles, :nK]
        v = valid.numpy()[:nK].astype(bool)
        cpos = np.zeros(max(nK, 1), np.int64)
        cpos[:nK] = np.cumsum(v) - v
        present = (q != MISSING).sum(axis=1).astype(np.int64)
        nvalid = ((q != MISSING) & v[None, :]).sum(axis=1).astype(np.int64)
        return torch.from_numpy(cpos), present, nvalid, int(v.sum())

    def pack(self, Q, nK, valid, cpos, src_rows, bounds):
        q = Q.numpy()
        v = valid.numpy()[:nK].astype(bool)
        cols = q[:, :nK][:, v]                          # valid columns in order
        nrows, m = len(src_rows), int(bounds[-1])
        out = np.zeros(max(nrows * m, 1), np.int32)
        for s in range(len(bounds) - 1):
            a, b = bounds[s], bounds[s + 1]
            blk = cols[np.asarray(src_rows, np.int64)][:, a:b] if nrows else np.zeros((0, b - a), np.int32)
            out[nrows * a: nrows * a + nrows * (b - a)] = blk.reshape(-1)
        return torch.from_numpy(out)

    def parts_rows(self, parts, ids, raw, z32, row0):
        parts.rows(ids, raw, z32.numpy(), row0, level=1)

    def sync(self):
        pass
