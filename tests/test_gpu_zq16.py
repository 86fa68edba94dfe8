"""Compact step-4 output (grid_norm_zquant_kb16): the int16 codes plus the
escape list decode to exactly the int32 hundredths grid_norm_zquant_kb writes
(sentinels included), the bf16 panel is unchanged (also with a colmap that
leaves holes), and a pass whose escapes overflow the list falls back to the
int32 form with identical results downstream."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from grid_amd import _abi
    d = _abi.Device(0)
    d.set_stream(torch.cuda.current_stream())
    return d


def stats(dev, q, n, m):
    from grid_amd.fused import HipOps
    ops = HipOps(dev)
    nblk = -(-m // 8192)
    bsum = torch.zeros((n, nblk), dtype=torch.float64, device="cuda")
    bcnt = torch.zeros((n, nblk), dtype=torch.int32, device="cuda")
    ops.row_blocks(q, n, m, m, bsum, bcnt)
    rm = torch.zeros(n, dtype=torch.float64, device="cuda")
    ops.row_means(bsum, bcnt, n, nblk, rm)
    mu, var, ratio = (torch.zeros(m, dtype=torch.float64, device="cuda") for _ in range(3))
    ops.col_means(q, n, m, m, rm, mu)
    ops.col_vars(q, n, m, m, rm, mu, var, ratio)
    return ops, rm, mu


def decode(z16, idx=None, val=None):
    from grid_amd import _abi
    z = z16.astype(np.int64)
    z[z16 == _abi.ZQ16_NAN] = _abi.ZQ_NAN
    z[z16 == _abi.ZQ16_NEG0] = _abi.ZQ_NEG0
    z = z.astype(np.int32)
    if idx is not None and len(idx):
        assert (z.reshape(-1)[idx] == _abi.ZQ16_ESC).all()
        z.reshape(-1)[idx] = val
    return z


@pytest.mark.parametrize("scale", [1.7, 0.05])
def test_kb16_codes_equal_int32(dev, scale):
    from grid_amd import _abi
    n, m = 300, 3 * 8192 + 104
    q = torch.empty((n, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, 11, n, m, m, 0, 26, q.data_ptr())
    q[5, 7:40] = _abi.MISSING                      # missing cells -> "NA"
    q[9, :] = 0                                    # an all-zero row
    q[11, 301:321] = 50_000_000                    # |z| > 327.65 -> escapes
    ops, rm, mu = stats(dev, q, n, m)
    sel = torch.arange(1, m, 2, dtype=torch.int32, device="cuda")
    r = len(sel)
    colmap = torch.arange(r, dtype=torch.int32, device="cuda")
    colmap[::7] = -1                               # dropped by the step-5 filter
    kp = -(-r // 64) * 64
    out = {}
    for form in ("i32", "i16"):
        zb = torch.zeros((kp // _abi.KBW, 512, _abi.KBW), dtype=torch.int16, device="cuda")
        if form == "i32":
            zq = torch.zeros((n, r), dtype=torch.int32, device="cuda")
            of = ops.zquant(q, n, m, sel, r, rm, mu, scale, zq, r, colmap, 200, zb, 512)
            assert of == 0
            out[form] = (zq.cpu().numpy(), zb.cpu().numpy())
        else:
            zq = torch.zeros((n, r), dtype=torch.int16, device="cuda")
            ei = torch.zeros(4096, dtype=torch.int64, device="cuda")
            ev = torch.zeros(4096, dtype=torch.int32, device="cuda")
            of, ne = ops.zquant16(q, n, m, sel, r, rm, mu, scale, zq, r, colmap, 200, zb, 512, ei, ev)
            assert of == 0 and (ne > 0 or scale < 1)
            out[form] = (decode(zq.cpu().numpy(), ei[:ne].cpu().numpy(), ev[:ne].cpu().numpy()), zb.cpu().numpy())
    assert np.array_equal(out["i32"][0], out["i16"][0])
    assert np.array_equal(out["i32"][1], out["i16"][1])
    z = out["i32"][0]
    assert (z == _abi.ZQ_NAN).any() and (z == _abi.ZQ_NEG0).any()


def test_kb16_escape_overflow_flag(dev):
    from grid_amd import _abi
    n, m = 64, 8192
    q = torch.empty((n, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, 5, n, m, m, 0, 4, q.data_ptr())
    for i in range(40):                           # 40 single-cell spikes: |z| far beyond 327.65
        q[i, 100 + 3 * i] = 2_000_000_000
    ops, rm, mu = stats(dev, q, n, m)
    sel = torch.arange(m, dtype=torch.int32, device="cuda")
    zq = torch.zeros((n, m), dtype=torch.int16, device="cuda")
    zb = torch.zeros((m // _abi.KBW, 64, _abi.KBW), dtype=torch.int16, device="cuda")
    ei = torch.zeros(8, dtype=torch.int64, device="cuda")
    ev = torch.zeros(8, dtype=torch.int32, device="cuda")
    of, ne = ops.zquant16(q, n, m, sel, m, rm, mu, 1.0, zq, m, None, 200, zb, 64, ei, ev)
    assert of & 2 and not of & 1 and ne >= 40


def test_chain_zq16_equals_int32(dev):
    """Steps 4-7 with the int16 output vs the int32 one, and the fallback."""
    from grid_amd import _abi
    from grid_amd.fused import HipOps, Steps47, TorchAlloc
    import bench
    n, m, k, iters = 260, 3 * 8192 + 100, 6, 10
    reads, off, nbr, w = bench.synth_reads_and_ibs(n, seed=3, per_hap=4)
    q = torch.empty((n, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, 3, n, m, m, 0, 26, q.data_ptr())
    qs = q.clone()
    qs[7, 1234] = 2_000_000_000                   # a few escapes
    qx = q.clone()
    for i in range(n):                            # 2 spikes per row: 520 escapes, list of 300
        qx[i, (1000 + 37 * i) % m] = 2_000_000_000
        qx[i, (20000 + 41 * i) % m] = 2_000_000_000
    res = {}
    for name, src, z16 in (("i32", q, False), ("i16", q, True), ("i32s", qs, False), ("i16s", qs, True),
                           ("i32x", qx, False), ("fallback", qx, True)):
        st = Steps47(HipOps(dev), TorchAlloc(0), n, m, 0, m, k=k, n_nbr=3, n_iters=iters, zq16=z16)
        if name == "fallback":
            st.esc_idx, st.esc_val = st.esc_idx[:300], st.esc_val[:300]
        st.set_reads(reads)
        st.set_phasing_graph(off, nbr, w)
        st.run(src, m)
        torch.cuda.synchronize()
        assert st.zq_is16 == (name in ("i16", "i16s"))
        if name == "i16s":
            assert st.nesc > 0
        res[name] = [t.cpu().numpy() for t in (st.zq_int32()[:n, : st.r_loc], st.zb, st.idx_out[:n], st.d2[:n],
                                               st.dip[:n], st.hap[: 2 * n])]
    for a, b in zip(res["i32"], res["i16"]):
        assert np.array_equal(a, b, equal_nan=True)
    for a, b in zip(res["i32s"], res["i16s"]):
        assert np.array_equal(a, b, equal_nan=True)
    for a, b in zip(res["i32x"], res["fallback"]):
        assert np.array_equal(a, b, equal_nan=True)
