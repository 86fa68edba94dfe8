"""The cohort split of step 5 on the GPU: the Gram's row
segments computed directly from panel pieces (grid_knn_gram_kb_rows) and
their diagonal blocks completed (grid_knn_mirror_ld), against a float64
product (exact: |sums| < 2^53); then the whole chain at world 2/4/8 with the
ranks sharing the one GPU (gloo standing in for RCCL) against one rank.
Reference all-pairs search: /root/reference/grid/utils/find_neighbors.py:204-213."""
import numpy as np
import pytest

from grid_amd import _abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = _abi.Device(0)
    yield d
    d.close()


def _kblocked(q):
    np_, r = q.shape
    zf = (q.astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
    return np.ascontiguousarray(zf.reshape(np_, r // _abi.KBW, _abi.KBW).transpose(1, 0, 2))


@pytest.mark.parametrize("qmax", [200, 256])
def test_gram_rows_pieces_equal_the_product(dev, qmax):
    """Every 256-row range of np = 1024, accumulated over two K pieces of
    different lengths (several int32-exact units each), the ranges taken in
    an order that cycles more keys than the tile-list slots (eviction and
    re-upload); the diagonal block mirrored; columns past np - row0 in the
    padded stride untouched."""
    from grid_amd._abi import call
    n, np_ = 900, 1024
    r1, r2 = 64 * (2 * 838 + 7), 64 * 301
    rng = np.random.default_rng(qmax)
    q = np.zeros((np_, r1 + r2), dtype=np.int64)
    q[:n] = rng.integers(-qmax, qmax + 1, size=(n, r1 + r2))
    q[:3] = np.where(rng.random((3, r1 + r2)) < 0.5, -qmax, qmax)
    p1, p2 = dev.upload(_kblocked(q[:, :r1])), dev.upload(_kblocked(q[:, r1:]))
    qf = q.astype(np.float64)
    ref = (qf @ qf.T).astype(np.int64)
    ranges = [(0, 256), (256, 512), (512, 256), (768, 256), (0, 1024), (256, 768), (0, 256)]
    for row0, nr in ranges:
        ld = np_ - row0 + 64
        out = dev.zeros((nr, ld), np.int64)
        call("grid_knn_gram_kb_rows", dev.ctx, p1.ptr, np_, r1, qmax, row0, nr, out.ptr, ld)
        call("grid_knn_gram_kb_rows", dev.ctx, p2.ptr, np_, r2, qmax, row0, nr, out.ptr, ld)
        call("grid_knn_mirror_ld", dev.ctx, out.ptr, nr, ld)
        got = out.numpy()
        assert np.array_equal(got[:, : np_ - row0], ref[row0:row0 + nr, row0:]), (row0, nr)
        assert not got[:, np_ - row0:].any(), (row0, nr)


def test_gram_rows_rejects_unaligned_rows(dev):
    from grid_amd._abi import GridNativeError, call
    z = dev.zeros((2, 512, _abi.KBW), np.uint16)
    out = dev.zeros((256, 512), np.int64)
    with pytest.raises(GridNativeError):
        call("grid_knn_gram_kb_rows", dev.ctx, z.ptr, 512, 64, 200, 128, 256, out.ptr, 512)
    with pytest.raises(GridNativeError):
        call("grid_knn_gram_kb_rows", dev.ctx, z.ptr, 512, 64, 200, 256, 256, out.ptr, 128)
