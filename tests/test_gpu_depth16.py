"""Compact depth matrix (grid_depth16: uint16 hundredths + row-sorted escape
table): the encoder round-trips exactly, the synthetic generator's compact
form equals the encoded int32 cohort, and every step-4 kernel gives the same
bits from either form (so the whole chain does)."""
import ctypes as C

import numpy as np
import pytest
import torch

from grid_amd import _abi

pytestmark = pytest.mark.gpu

MISSING = -(2 ** 31)
MAXV, ESC, MISS = 0xFFFD, 0xFFFE, 0xFFFF


@pytest.fixture(scope="module")
def dev():
    from grid_amd import _abi
    d = _abi.Device(0)
    d.set_stream(torch.cuda.current_stream())
    return d


def encode(dev, q):
    """int32 device tensor [n][m] -> (q16, eoff, ecol, eval) torch tensors."""
    from grid_amd import _abi
    n, m = q.shape
    ld16 = -(-m // 8) * 8
    q16 = torch.zeros((n, ld16), dtype=torch.int16, device="cuda")
    eoff = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    cap = int((q.cpu() > MAXV).sum() + 1)
    ecol = torch.zeros(cap, dtype=torch.int32, device="cuda")
    ev = torch.zeros(cap, dtype=torch.int32, device="cuda")
    need = C.c_int64()
    _abi.call("grid_q16_encode", dev.ctx, q.data_ptr(), n, m, m, q16.data_ptr(), ld16, eoff.data_ptr(),
              ecol.data_ptr(), ev.data_ptr(), cap, C.byref(need))
    return q16, eoff, ecol[: need.value], ev[: need.value], ld16


def decode_host(q16, eoff, ecol, ev, m):
    c = q16.cpu().numpy().view(np.uint16)[:, :m].astype(np.int64)
    out = np.where(c == MISS, MISSING, c)
    eo, ec, evv = eoff.cpu().numpy(), ecol.cpu().numpy(), ev.cpu().numpy()
    for i in range(c.shape[0]):
        cols = ec[eo[i]: eo[i + 1]]
        assert np.all(np.diff(cols) > 0)
        assert np.all(c[i, cols] == ESC)
        out[i, cols] = evv[eo[i]: eo[i + 1]]
    assert int((c == ESC).sum()) == len(ec)
    return out.astype(np.int64)


def random_depths(n, m, seed):
    rng = np.random.default_rng(seed)
    q = rng.integers(0, 9000, (n, m)).astype(np.int64)
    q[rng.random((n, m)) < 0.01] = MISSING
    big = rng.random((n, m)) < 0.002
    q[big] = rng.integers(MAXV - 2, 400000, int(big.sum()))
    q[0, :5] = [MAXV, MAXV + 1, 0, MISSING, 2 ** 31 - 1]
    return q.astype(np.int32)


def test_encode_roundtrip(dev):
    q = random_depths(37, 20003, 1)
    qd = torch.from_numpy(q).cuda()
    q16, eoff, ecol, ev, _ = encode(dev, qd)
    assert np.array_equal(decode_host(q16, eoff, ecol, ev, q.shape[1]), q.astype(np.int64))


def test_synth_q16_equals_encoded_synth(dev):
    from grid_amd import _abi
    from grid_amd.fused import Depth16, TorchAlloc
    n, m, col0 = 50, 70001, 8192 * 3
    q = torch.empty((n, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, 77, n, m, m, col0, 26, q.data_ptr())
    q16, eoff, ecol, ev, _ = encode(dev, q)
    assert len(ecol) > 10                      # the model's x40 spikes reach the escape table
    d = Depth16.synth(TorchAlloc(0), dev.ctx, 77, n, m, col0, 26, exc_cap=4)   # exercises the regrow
    assert torch.equal(d.q16[:, :m], q16[:, :m])
    assert torch.equal(d.eoff, eoff)
    k = int(eoff[-1])
    assert torch.equal(d.ecol[:k], ecol) and torch.equal(d.evals[:k], ev)


# raw-code software-pipelined column kernels (GRID_COL_PF; 1 or 2 columns per
# thread, 8 or 16 rows per group) and the streamed row-block kernel
# (GRID_ROWBLK16_PB=0; GRID_ROWBLK16_WPC=1: one workgroup per CU, many units
# each); the knobs take effect in the tools build
# (GRID_AMD_LIB=.../libgridhip_probes.so), the product library runs its defaults
PF_KNOBS = [{"GRID_COL_PF": "0", "GRID_ROWBLK16_PB": "0"}, {"GRID_ROWBLK16_PB": "0", "GRID_ROWBLK16_WPC": "1"},
            {"GRID_ROWBLK16_XOR": "0"}, {"GRID_COL_PF": "1"}, {"GRID_COL_PF": "1", "GRID_COL16_VW": "1"},
            {"GRID_COL_PF": "1", "GRID_COL16_VW": "1", "GRID_COL16_CU": "16"},
            {"GRID_COL_PF": "1", "GRID_COL16_CU": "16"}]


@pytest.mark.parametrize("knobs", [{}, {"GRID_COL16_VW": "1", "GRID_ROWBLK16_PB": "1"},
                                   {"GRID_COL16_VW": "4", "GRID_ROWBLK16_PB": "4", "GRID_ROWBLK_NT": "0",
                                    "GRID_COL_NT": "0", "GRID_ZQUANT_NT": "0", "GRID_ZQUANT_GROUPS": "3"},
                                   {"GRID_COL16_CU": "16", "GRID_ROWBLK16_PB": "2", "GRID_ZQUANT_GROUPS": "5"},
                                   {"GRID_ZQUANT7": "0"}] + PF_KNOBS)
@pytest.mark.parametrize("pattern", ["every3", "dense"])
def test_step4_kernels_q16_equal_int32(dev, knobs, pattern, monkeypatch):
    """Every q16 kernel variant (columns per thread, blocks per workgroup,
    streaming loads: timing knobs) gives the int32 kernels' bits, including
    the int16 step-4 codes and their escape list."""
    from grid_amd.fused import Depth16, HipOps
    for k_, v_ in knobs.items():
        monkeypatch.setenv(k_, v_)
    n, m = 300, 5 * 8192 + 516          # ld % 4 == 0: the int32 layout of the int16 output
    q = random_depths(n, m, 2)
    q[:, 100] = MISSING
    qd = torch.from_numpy(q).cuda()
    q16, eoff, ecol, ev, ld16 = encode(dev, qd)
    d16 = Depth16(q16, eoff, ecol, ev, ld16)
    ops = HipOps(dev)
    nblk = -(-m // 8192)
    out = {}
    for name, src, ld in (("i32", qd, m), ("q16", d16, ld16)):
        bsum = torch.zeros((n, nblk), dtype=torch.float64, device="cuda")
        bcnt = torch.zeros((n, nblk), dtype=torch.int32, device="cuda")
        ops.row_blocks(src, n, m, ld, bsum, bcnt)
        rm = torch.zeros(n, dtype=torch.float64, device="cuda")
        ops.row_means(bsum, bcnt, n, nblk, rm)
        mu, var, ratio = (torch.zeros(m, dtype=torch.float64, device="cuda") for _ in range(3))
        ops.col_means(src, n, m, ld, rm, mu)
        ops.col_vars(src, n, m, ld, rm, mu, var, ratio)
        if pattern == "every3":     # 4 selected columns never share an 8-code window: per-cell gathers
            sel = torch.arange(0, m, 3, dtype=torch.int32, device="cuda")
            colmap = torch.arange(len(sel), dtype=torch.int32, device="cuda")
        else:                       # ~90 % selected, r % 4 != 0, panel holes (colmap -1) and runs
            keep = np.random.default_rng(5).random(m) < 0.9
            keep[-3:] = [True, False, True]
            sel_np = np.flatnonzero(keep).astype(np.int32)
            if len(sel_np) % 4 == 0:
                sel_np = sel_np[:-1]
            hole = np.random.default_rng(6).random(len(sel_np)) < 0.05
            cm_np = np.where(hole, -1, np.cumsum(~hole) - 1).astype(np.int32)
            sel = torch.from_numpy(sel_np).cuda()
            colmap = torch.from_numpy(cm_np).cuda()
        r = len(sel)
        zq = torch.zeros((n, r), dtype=torch.int32, device="cuda")
        kp = -(-r // 64) * 64
        zb = torch.zeros((kp // _abi.KBW, 512, _abi.KBW), dtype=torch.int16, device="cuda")
        ops.zquant(src, n, ld, sel, r, rm, mu, 1.7, zq, r, colmap, 200, zb, 512)
        zq16 = torch.zeros((n, r), dtype=torch.int16, device="cuda")
        zb16 = torch.zeros_like(zb)
        eidx = torch.zeros(1 << 16, dtype=torch.int64, device="cuda")
        eval_ = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
        of, ne = ops.zquant16(src, n, ld, sel, r, rm, mu, 1.7, zq16, r, colmap, 200, zb16, 512, eidx, eval_)
        assert of == 0
        order = torch.argsort(eidx[:ne])
        esc = (eidx[:ne][order], eval_[:ne][order])
        out[name] = [t.cpu().numpy() for t in (bsum, bcnt, rm, mu, var, ratio, zq, zb, zq16, zb16) + esc]
    for a, b in zip(out["i32"], out["q16"]):
        assert np.array_equal(a, b, equal_nan=True)


def test_chain_q16_equals_int32(dev):
    from grid_amd import _abi
    from grid_amd.fused import Depth16, HipOps, Steps47, TorchAlloc
    import bench
    n, m, k, iters = 260, 3 * 8192 + 100, 6, 10
    reads, off, nbr, w = bench.synth_reads_and_ibs(n, seed=3, per_hap=4)
    q = torch.empty((n, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, 3, n, m, m, 0, 26, q.data_ptr())
    d16 = Depth16.synth(TorchAlloc(0), dev.ctx, 3, n, m, 0, 26)
    res = {}
    for name, src, ld in (("i32", q, m), ("q16", d16, d16.ld)):
        st = Steps47(HipOps(dev), TorchAlloc(0), n, m, 0, m, k=k, n_nbr=3, n_iters=iters)
        st.set_reads(reads)
        st.set_phasing_graph(off, nbr, w)
        st.run(src, ld)
        torch.cuda.synchronize()
        res[name] = [t.cpu().numpy() for t in (st.rm[:n], st.mu[:m], st.var[:m], st.zq_int32()[:n, : st.r_loc],
                                               st.idx_out[:n], st.d2[:n], st.dip[:n], st.hap[: 2 * n])]
    for a, b in zip(res["i32"], res["q16"]):
        assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("tail", [1, 7, 8, 9, 127, 128, 129, 136, 255, 257, 1000, 1728, 4095, 4096, 6360, 8191])
def test_row_means_every_tail_length(dev, tail):
    """The partial last block's pairwise tree (planned on the host per tail
    length): row means of both depth forms equal NumPy's nanmean bit for bit,
    with escapes and missing cells inside the tail."""
    from grid_amd.fused import Depth16, HipOps
    from oracle.npsum import nanmean_rows
    n, m = 70, 8192 + tail
    q = random_depths(n, m, 100 + tail)
    q[3, 8192:] = MISSING                       # a row whose tail is all missing
    q[4, -1] = 300000                           # an escape in the tail's last leaf
    qd = torch.from_numpy(q).cuda()
    q16, eoff, ecol, ev, ld16 = encode(dev, qd)
    d16 = Depth16(q16, eoff, ecol, ev, ld16)
    ops = HipOps(dev)
    mat = np.where(q == MISSING, np.nan, q / 100.0)
    exp = nanmean_rows(mat)
    for src, ld in ((qd, m), (d16, ld16)):
        bsum = torch.zeros((n, 2), dtype=torch.float64, device="cuda")
        bcnt = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
        ops.row_blocks(src, n, m, ld, bsum, bcnt)
        rm = torch.zeros(n, dtype=torch.float64, device="cuda")
        ops.row_means(bsum, bcnt, n, 2, rm)
        assert np.array_equal(rm.cpu().numpy(), exp, equal_nan=True)
        assert np.array_equal(bcnt.cpu().numpy()[:, 1], (q[:, 8192:] != MISSING).sum(1))


@pytest.mark.parametrize("knobs", [{}] + PF_KNOBS)
@pytest.mark.parametrize("n,m", [(1, 9), (7, 1001), (8, 64), (33, 777), (257, 4099), (300, 5 * 8192 + 517),
                                 (520, 2 * 8192 + 1)])
def test_col_stats_pipelined_equal_int32(dev, n, m, knobs, monkeypatch):
    """The pipelined compact column kernel (k_col16_pipe: LDS row windows,
    groups of 8 rows in flight, ragged last column) gives the int32 column
    kernels' bits: rows not a multiple of 8 or 32, windows of 256 rows, odd m,
    missing cells, escapes and a zero-mean row."""
    from grid_amd.fused import Depth16, HipOps
    for k_, v_ in knobs.items():
        monkeypatch.setenv(k_, v_)
    q = random_depths(n, m, 7 * n + m)
    if n > 3:
        q[3, :] = 0                                  # row mean 0: a bad row (skipped)
    qd = torch.from_numpy(q).cuda()
    q16, eoff, ecol, ev, ld16 = encode(dev, qd)
    d16 = Depth16(q16, eoff, ecol, ev, ld16)
    ops = HipOps(dev)
    nblk = -(-m // 8192)
    out = {}
    for name, src, ld in (("i32", qd, m), ("q16", d16, ld16)):
        bsum = torch.zeros((n, nblk), dtype=torch.float64, device="cuda")
        bcnt = torch.zeros((n, nblk), dtype=torch.int32, device="cuda")
        ops.row_blocks(src, n, m, ld, bsum, bcnt)
        rm = torch.zeros(n, dtype=torch.float64, device="cuda")
        ops.row_means(bsum, bcnt, n, nblk, rm)
        mu, var, ratio = (torch.full((m + 1,), -7.0, dtype=torch.float64, device="cuda") for _ in range(3))
        ops.col_means(src, n, m, ld, rm, mu)
        ops.col_vars(src, n, m, ld, rm, mu, var, ratio)
        out[name] = [t.cpu().numpy() for t in (rm, mu, var, ratio)]
    for a, b in zip(out["i32"], out["q16"]):
        assert np.array_equal(a, b, equal_nan=True)
    assert out["q16"][1][m] == -7.0                  # nothing stored past the last column
