"""Correctness at the timed size (MI355X only; VERDICT r1 "parity at the
timed scale"):

(a) k_gram8 at n = 3202 (np = 3328, 26 x 13 tiles) with K long enough for
    several int32 chunks per XCD K-range, and with one K-range per XCD group
    (GRID_GRAM_KX=1): the whole int64 Gram against an fp64 product (exact:
    integers < 2^53) and the row top-k against torch on the same distances;
(b) the device mismatch count of the step-4 output and the bf16 panel against
    an independent IEEE fp64 recomputation (grid_verify_zquant) over the full
    3202 x 3M synthetic bench cohort: 0 expected;
(c) adversarial rounding boundaries: z within a few ulps of (k + 0.5)/100
    and tiny negative z ("-0.00"), through the fp32 fast path and its exact
    fallback, against Python's "%.2f" (normalize_mosdepth.py:553).
"""
import math

import numpy as np
import pytest

from grid_amd import _abi
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from grid_amd._abi import Device
    d = Device(0)
    d.set_stream(torch.cuda.current_stream())
    return d


@pytest.mark.parametrize("kx", [None, "1"])
def test_gram_3202_multi_chunk(dev, kx, monkeypatch):
    from grid_amd._abi import call
    if kx:
        monkeypatch.setenv("GRID_GRAM_KX", kx)
    n, np_, qmax = 3202, 3328, 200
    steps_ = 8 * 838 * 2 + 37                       # > 2 int32-exact chunks per XCD K-range
    kpad = 64 * steps_
    g = torch.Generator(device="cuda").manual_seed(5)
    z = torch.zeros((np_, kpad), dtype=torch.int16, device="cuda")
    for r0 in range(0, n, 512):
        r1 = min(n, r0 + 512)
        zi = torch.randint(-qmax, qmax + 1, (r1 - r0, kpad), device="cuda", dtype=torch.int32, generator=g)
        zi[:, : 64 * 50] = qmax                     # worst-case magnitudes in the first chunk
        z[r0:r1] = zi.to(torch.bfloat16).view(torch.int16)
        del zi
    zkb = z.view(np_, steps_ * 64 // _abi.KBW, _abi.KBW).permute(1, 0, 2).contiguous()
    gram = torch.zeros((np_, np_), dtype=torch.int64, device="cuda")
    call("grid_knn_gram_kb", dev.ctx, zkb.data_ptr(), np_, kpad, qmax, gram.data_ptr())
    call("grid_knn_mirror", dev.ctx, gram.data_ptr(), np_)
    del zkb
    zf = z.view(torch.bfloat16).to(torch.float64)
    del z
    ref = zf @ zf.T                                  # exact: |sums| < 2^53
    del zf
    assert torch.equal(gram, ref.round().to(torch.int64))
    # row top-k on the full rows vs torch on the same exact distances
    k = 10
    norms = torch.diagonal(gram).contiguous()
    idx = torch.empty((n, k), dtype=torch.int32, device="cuda")
    d2 = torch.empty((n, k), dtype=torch.int64, device="cuda")
    cnt = torch.empty(n, dtype=torch.int32, device="cuda")
    call("grid_knn_topk_rows", dev.ctx, gram.data_ptr(), np_, norms.data_ptr(), n, k, 0, n, idx.data_ptr(),
         d2.data_ptr(), cnt.data_ptr())
    dd = norms[:n, None] + norms[None, :n] - 2 * gram[:n, :n]
    key = dd * 4096 + torch.arange(n, device="cuda")[None, :]        # (d2, j) order, j < 4096
    key.fill_diagonal_(torch.iinfo(torch.int64).max)                 # self dropped
    top = torch.topk(key, k, dim=1, largest=False).values
    assert torch.equal(idx.to(torch.int64), top % 4096)
    assert torch.equal(d2, top // 4096)
    assert bool((cnt == k).all())


def test_zquant_full_bench_cohort_exact(dev):
    """(b): the bench chain at 3202 x 3M, every selected cell checked."""
    from grid_amd import _abi
    from grid_amd.fused import HipOps, Steps47, TorchAlloc
    import bench
    n, m = 3202, 3_000_000
    q = torch.empty((n, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, bench.SEED, n, m, m, 0, bench.NCL, q.data_ptr())
    reads, off, nbr, w = bench.synth_reads_and_ibs(n)
    st = Steps47(HipOps(dev), TorchAlloc(0), n, m, 0, m, k=10, n_iters=5)
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)
    st.run(q, m)
    torch.cuda.synchronize()
    assert st.zq_is16
    import ctypes as C
    counts = (C.c_int64 * 3)()
    _abi.call("grid_verify_zquant", dev.ctx, q.data_ptr(), n, m, st.sel.data_ptr(), st.r_loc, st.rm.data_ptr(),
              st.mu.data_ptr(), st.scale, st.zq16.data_ptr(), m, st.colmap.data_ptr(), st.qmax, st.zb.data_ptr(),
              st.np_, counts)
    assert st.r_loc > 2_500_000
    assert list(counts) == [0, 0, 0], list(counts)


def test_zquant7_full_bench_cohort_exact(dev):
    """(b) for the compact depth form (k_zquant7, the bench default): the chain
    on the Depth16 cohort, every selected cell checked against the int32
    matrix it encodes."""
    from grid_amd import _abi
    from grid_amd.fused import Depth16, HipOps, Steps47, TorchAlloc
    import bench
    import ctypes as C
    n, m = 3202, 3_000_000
    d16 = Depth16.synth(TorchAlloc(0), dev.ctx, bench.SEED, n, m, 0, bench.NCL)
    reads, off, nbr, w = bench.synth_reads_and_ibs(n)
    st = Steps47(HipOps(dev), TorchAlloc(0), n, m, 0, m, k=10, n_iters=5)
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)
    st.run(d16, d16.ld)
    torch.cuda.synchronize()
    assert st.zq_is16
    q = torch.empty((n, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, bench.SEED, n, m, m, 0, bench.NCL, q.data_ptr())
    counts = (C.c_int64 * 3)()
    _abi.call("grid_verify_zquant", dev.ctx, q.data_ptr(), n, m, st.sel.data_ptr(), st.r_loc, st.rm.data_ptr(),
              st.mu.data_ptr(), st.scale, st.zq16.data_ptr(), m, st.colmap.data_ptr(), st.qmax, st.zb.data_ptr(),
              st.np_, counts)
    assert st.r_loc > 2_500_000
    assert list(counts) == [0, 0, 0], list(counts)


def _fmt_code(z):
    t = f"{z:.2f}"
    k = int(t.replace(".", ""))
    return -(2 ** 31) + 1 if (k == 0 and t.startswith("-")) else k


def test_zquant_rounding_boundaries(dev):
    """(c): per row a mean chosen so that column 0's z lands within a few ulps
    of a rounding boundary (k + 0.5)/100, or at a tiny negative value."""
    from grid_amd import _abi
    rng = np.random.default_rng(3)
    rows = []
    mus = np.array([1.0, 0.37, 2.9, 17.25])
    scale = 1.0 / math.sqrt(1.234)
    for t in range(4096):
        mu = float(mus[t % 4])
        kk = int(rng.integers(-400, 400))
        target = (kk + 0.5) / 100.0 if t % 7 else -1e-9 * (1 + t % 5)
        qv = int(rng.integers(1000, 9000))
        rm0 = (qv / 100.0) / (mu + target * math.sqrt(mu) / scale)
        for ulp in range(-3, 4):
            rm = rm0
            for _ in range(abs(ulp)):
                rm = float(np.nextafter(rm, np.inf if ulp > 0 else -np.inf))
            rows.append((qv, rm, mu))
    n = len(rows)
    ld = 4
    q = np.zeros((n, ld), dtype=np.int32)
    rmv = np.zeros(n)
    for i, (qv, rm, mu) in enumerate(rows):
        q[i, :] = [qv, qv + 1, qv + 2, qv + 3]
        rmv[i] = rm
    # one column per distinct mu: row i's cells all use column mu; build 4 column sets
    out_all = {}
    for c, mu in enumerate(mus):
        sel_rows = np.array([i for i, r in enumerate(rows) if r[2] == mu])
        qq = np.ascontiguousarray(q[sel_rows])
        rr = np.ascontiguousarray(rmv[sel_rows])
        nn = len(sel_rows)
        mu_arr = np.full(ld, mu)
        sel = np.arange(ld, dtype=np.int32)
        d = {k: dev.upload(v) for k, v in (("q", qq), ("rm", rr), ("mu", mu_arr), ("sel", sel))}
        np_zb = -(-nn // 64) * 64
        for mode in ("int32", "int16", "q16"):
            zb = dev.zeros((1, np_zb, _abi.KBW), np.uint16)
            if mode == "q16":              # compact source (k_zquant7): the same codes, 8-wide rows
                import ctypes as C
                q16 = dev.zeros((nn, 8), np.uint16)
                eoff = dev.zeros(nn + 1, np.int64)
                ecol, evl = dev.zeros(1, np.int32), dev.zeros(1, np.int32)
                need = C.c_int64()
                _abi.call("grid_q16_encode", dev.ctx, d["q"].ptr, nn, ld, ld, q16.ptr, 8, eoff.ptr, ecol.ptr,
                          evl.ptr, 1, C.byref(need))
                desc = _abi.Depth16Desc(q16.ptr, eoff.ptr, ecol.ptr, evl.ptr)
                zq = dev.alloc((nn, ld), np.int16)
                ei, ev = dev.alloc(1 << 16, np.int64), dev.alloc(1 << 16, np.int32)
                of, ne = C.c_int32(), C.c_int64()
                _abi.call("grid_norm_zquant_kb16_q16", dev.ctx, C.byref(desc), nn, 8, d["sel"].ptr, ld, d["rm"].ptr,
                          d["mu"].ptr, scale, zq.ptr, ld, None, 200, zb.ptr, np_zb, ei.ptr, ev.ptr, 1 << 16,
                          C.byref(ne), C.byref(of))
                assert of.value == 0
                got = zq.numpy().astype(np.int64)
                got[got == -32767] = -(2 ** 31) + 1
            elif mode == "int32":
                zq = dev.alloc((nn, ld), np.int32)
                import ctypes as C
                of = C.c_int32()
                _abi.call("grid_norm_zquant_kb", dev.ctx, d["q"].ptr, nn, ld, d["sel"].ptr, ld, d["rm"].ptr,
                          d["mu"].ptr, scale, zq.ptr, ld, None, 200, zb.ptr, np_zb, C.byref(of))
                got = zq.numpy()
            else:
                zq = dev.alloc((nn, ld), np.int16)
                ei, ev = dev.alloc(1 << 16, np.int64), dev.alloc(1 << 16, np.int32)
                import ctypes as C
                of, ne = C.c_int32(), C.c_int64()
                _abi.call("grid_norm_zquant_kb16", dev.ctx, d["q"].ptr, nn, ld, d["sel"].ptr, ld, d["rm"].ptr,
                          d["mu"].ptr, scale, zq.ptr, ld, None, 200, zb.ptr, np_zb, ei.ptr, ev.ptr, 1 << 16,
                          C.byref(ne), C.byref(of))
                assert of.value == 0
                got = zq.numpy().astype(np.int64)
                got[got == -32767] = -(2 ** 31) + 1
            for a, i in enumerate(sel_rows):
                for j in range(ld):
                    x = q[i, j] / 100.0
                    z = ((x / rmv[i] - mu) / math.sqrt(mu)) * scale
                    assert got[a, j] == _fmt_code(z), (mode, i, j, z)
            panel = zb.numpy()[0, :nn, :ld]
            for a, i in enumerate(sel_rows):
                for j in range(ld):
                    x = q[i, j] / 100.0
                    z = ((x / rmv[i] - mu) / math.sqrt(mu)) * scale
                    code = _fmt_code(z)
                    w = 0 if code == -(2 ** 31) + 1 else max(-200, min(200, code))
                    assert panel[a, j] == (np.float32(w).view(np.uint32) >> 16), (mode, i, j)
        out_all[mu] = True
    assert len(out_all) == 4
