"""Bin-axis streaming with the real HIP kernels (MI355X only): the chain run
in 8192-aligned chunks -- from a resident matrix read chunk by chunk, from the
on-device generator (SynthSource, regenerated every pass, the bench's configs
3-4 mode) and from a host array -- gives the one-chunk (resident) chain's
statistics, step-4 output, neighbours, dipCN and phasing bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, M, K, ITERS, SEED = 300, 5 * 8192 + 517, 6, 12, 99


def _chain(q, ld, chunk, keep_z=True, on_z=None, m=None, esc_cap=None):
    from grid_amd import _abi
    from grid_amd.fused import HipOps, Steps47, TorchAlloc
    import bench
    M_ = m or M
    dev = _abi.Device(0)
    dev.set_stream(torch.cuda.current_stream())
    ops = HipOps(dev)
    if callable(q):
        q = q(ops)
    reads, off, nbr, w = bench.synth_reads_and_ibs(N, seed=SEED, per_hap=5)
    st = Steps47(ops, TorchAlloc(0), N, M_, 0, M_, k=K, n_nbr=4, n_iters=ITERS, chunk=chunk, keep_z=keep_z,
                 on_z_chunk=on_z)
    if esc_cap is not None:                     # a small int16 escape list (tests its per-chunk reuse)
        st.esc_idx, st.esc_val = st.esc_idx[:esc_cap], st.esc_val[:esc_cap]
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)
    st.run(q, ld)
    torch.cuda.synchronize()
    out = {"rm": st.rm[:N].cpu().numpy(), "mu": st.mu[:M_].cpu().numpy(), "var": st.var[:M_].cpu().numpy(),
           "sel": st.sel[: st.r_loc].cpu().numpy(), "idx": st.idx_out[:N].cpu().numpy(),
           "d2": st.d2[:N].cpu().numpy(), "dip": st.dip[:N].cpu().numpy(), "hap": st.hap[: 2 * N].cpu().numpy(),
           "imp": st.imp[: 2 * N].cpu().numpy(), "ruse": st.ruse_loc, "scale": st.scale, "nch": st.nch,
           "nesc": st.nesc}
    if keep_z:
        out["zq"] = st.zq_int32()[:N, : st.r_loc].cpu().numpy()
    return out


@pytest.fixture(scope="module")
def resident():
    from grid_amd import _abi
    q = torch.empty((N, M), dtype=torch.int32, device="cuda")
    dev = _abi.Device(0)
    _abi.call("grid_synth_depth", dev.ctx, SEED, N, M, M, 0, 7, q.data_ptr())
    torch.cuda.synchronize()
    return q, _chain(q, M, None)


KEYS = ("rm", "mu", "var", "sel", "idx", "d2", "dip", "hap", "imp", "ruse", "scale")


def _same(a, b, keys=KEYS):
    for key in keys:
        assert np.array_equal(np.asarray(a[key]), np.asarray(b[key]), equal_nan=True), key


def test_resident_in_chunks(resident):
    q, ref = resident
    got = _chain(q, M, 16384)
    assert got["nch"] == 3
    _same(got, ref, KEYS + ("zq",))


def test_synth_source_streamed(resident):
    from grid_amd.fused import SynthSource
    _, ref = resident
    got = _chain(lambda ops: SynthSource(ops, SEED, N, 0, 7), None, 8192)
    assert got["nch"] == 6
    _same(got, ref, KEYS + ("zq",))


def test_host_source_fused_z(resident):
    """keep_z=False (fused mode): each chunk's step-4 output is handed to the
    consumer before the buffer is reused; concatenated, it is the resident
    output."""
    from grid_amd import _abi
    from grid_amd.fused import HostSource, zq16_to_int32
    q, ref = resident
    parts = {}

    def on_z(zq16, ld, s0, s1, ei, ev):
        z = zq16_to_int32(torch, zq16.view(-1)[: N * ld].view(N, ld)[:, : s1 - s0].contiguous(),
                          torch.zeros(0, dtype=torch.int64, device=zq16.device), ev[:0])
        if ei.numel():                               # escapes: flat index in the chunk buffer
            r, c = ei // ld, ei % ld
            z[r, c] = ev
        parts[s0] = z.cpu().numpy()

    got = _chain(HostSource(q.cpu().numpy()), M, 16384, keep_z=False, on_z=on_z)
    _same(got, ref)
    z = np.concatenate([parts[s] for s in sorted(parts)], axis=1)
    assert np.array_equal(z, ref["zq"])


def _on_z_collect(parts):
    from grid_amd.fused import zq16_to_int32

    def on_z(zq16, ld, s0, s1, ei, ev):
        z = zq16_to_int32(torch, zq16.view(-1)[: N * ld].view(N, ld)[:, : s1 - s0].contiguous(),
                          torch.zeros(0, dtype=torch.int64, device=zq16.device), ev[:0])
        if ei.numel():                               # escapes: flat index in the chunk buffer
            r, c = ei // ld, ei % ld
            z[r, c] = ev
        parts[s0] = (z.cpu().numpy(), ei.numel())
    return on_z


def test_streamed_escapes_reuse_the_list_per_chunk():
    """in fused mode every chunk's int16 escapes (|z| > 327.65) are
    consumed before the next chunk, so each chunk's list starts at 0 and the
    capacity applies per chunk.  A cohort whose hot columns each hold one
    30000x outlier (one escape per selected column), 8 chunks, a 3000-entry
    list: more escapes in total than the list holds, fewer per chunk; the
    concatenated step-4 output equals the resident chain's."""
    from grid_amd import _abi
    m = 8 * 8192
    dev = _abi.Device(0)
    qd = torch.empty((N, m), dtype=torch.int32, device="cuda")
    _abi.call("grid_synth_depth", dev.ctx, SEED, N, m, m, 0, 7, qd.data_ptr())
    qh = qd.cpu().numpy()
    hot = np.arange(3, m, 8)                          # 12.5 % of the columns
    qh[(hot * 7) % N, hot] = 3_000_000
    ref = _chain(torch.from_numpy(qh).cuda(), m, None, m=m)
    parts = {}
    got = _chain(HostSource_(qh), m, 8192, keep_z=False, on_z=_on_z_collect(parts), m=m, esc_cap=3000)
    _same(got, ref)
    per_chunk = [parts[s][1] for s in sorted(parts)]
    assert len(per_chunk) == 8 and sum(per_chunk) > 3000 and max(per_chunk) <= 3000, per_chunk
    z = np.concatenate([parts[s][0] for s in sorted(parts)], axis=1)
    assert np.array_equal(z, ref["zq"])


def HostSource_(q):
    from grid_amd.fused import HostSource
    return HostSource(q)


@pytest.mark.parametrize("knobs", [{"GRID_ROWBLK_NT": "0"}, {"GRID_COL_NT": "0"}, {"GRID_ZQUANT_NT": "0"},
                                   {"GRID_ZQUANT_GROUPS": "3"},
                                   {"GRID_GRAM_KX": "1", "GRID_GRAM_LAG": "0", "GRID_GRAM_SPIN": "0"},
                                   {"GRID_GRAM_KC": "5", "GRID_GRAM_LAG": "3"}])
def test_performance_knobs_do_not_change_results(resident, knobs, monkeypatch):
    """The product library's getenv knobs are performance-only: every
    alternative they select gives the default chain's results bit for bit."""
    q, ref = resident
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    _same(_chain(q, M, None), ref, KEYS + ("zq",))
