"""Device writer of the step-4 file (grid_write_normalized_gz_dev): the
decompressed text must equal the host writer's (which tests/test_textio_cpu.py
and the e2e goldens pin to the reference) byte for byte, across batch and
member boundaries, sentinels and wide values; the 'GR' index must let the
library's reader parse it back."""
import gzip
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev():
    from grid_amd import _abi
    return _abi.Device(0)


def _case(n, r, seed, wide=False):
    rng = np.random.default_rng(seed)
    zq = np.clip(np.rint(rng.normal(0, 120, (n, r))), -2 ** 31 + 2, 2 ** 31 - 1).astype(np.int32)
    if wide and n and r:
        zq.flat[rng.integers(0, n * r, 50)] = rng.integers(-2 ** 31 + 2, 2 ** 31 - 1, 50)
        zq.flat[0] = 2 ** 31 - 1
        zq.flat[-1] = -2 ** 31 + 2
    if n and r:
        zq.flat[rng.integers(0, n * r, 30)] = -(2 ** 31)        # NA
        zq.flat[rng.integers(0, n * r, 30)] = -(2 ** 31) + 1    # -0.00
    ids = [f"SAMPLE_{i:05d}" for i in range(n)]
    raw = rng.uniform(5, 90, n)
    raw[:1] = [1e300] if n else raw[:1]
    mu = rng.uniform(10, 60, r)
    ra = rng.uniform(0, 9, r)
    if r:
        mu[0] = np.nan
    return ids, raw, mu, ra, zq


def _members(path):
    """(first row, member size) of every member from the 'GR' subfields."""
    data = open(path, "rb").read()
    out, p = [], 0
    while p < len(data):
        assert data[p:p + 4] == b"\x1f\x8b\x08\x04"
        size, row = struct.unpack_from("<Qq", data, p + 16)
        out.append((row, size))
        p += size
    assert p == len(data)
    return out


@pytest.mark.parametrize("n,r,batch,wide", [(7, 5000, 0, False), (33, 3001, 40000, True), (1, 1, 0, False),
                                            (4, 0, 0, False), (300, 17, 9000, False), (2, 70000, 300000, True),
                                            (5, 1_500_000, 30_000_000, False)])   # 5 batches of one row
def test_device_writer_equals_host_writer(tmp_path, n, r, batch, wide):
    from grid_amd import _abi
    dev = _dev()
    ids, raw, mu, ra, zq = _case(n, r, seed=n * 1000 + r, wide=wide)
    ld = max(r, 1) + 3                      # a row stride wider than r
    zpad = np.zeros((n, ld), np.int32)
    zpad[:, :r] = zq
    dz = dev.upload(zpad)
    host, devf = tmp_path / "host.tsv.gz", tmp_path / "dev.tsv.gz"
    _abi.write_normalized_gz(str(host), ids, raw, mu, ra, zq, level=1)
    _abi.write_normalized_gz_dev(dev, str(devf), ids, raw, mu, ra, dz, n, r, ld, level=1, batch_bytes=batch)
    a, b = gzip.open(host, "rb").read(), gzip.open(devf, "rb").read()
    assert a == b
    mem = _members(devf)
    assert mem[0][0] == -1 and [m[0] for m in mem[1:]] == sorted(m[0] for m in mem[1:])
    if r:
        got = _abi.read_normalized_gz(str(devf))
        assert got[0] == ids and np.array_equal(got[4], np.where(zq == -(2 ** 31) + 1, 0, zq))


def test_device_writer_large_rows_size(tmp_path):
    """A config-2-like row (2.7 M cells): the device writer's LZ77 output
    within 6 % of the host writer's (libdeflate level 1) size, same text
    (literal-only Huffman was ~28 % larger)."""
    from grid_amd import _abi
    dev = _dev()
    n, r = 3, 2_700_000
    rng = np.random.default_rng(5)
    zq = np.clip(np.rint(rng.normal(0, 100, (n, r))), -200, 200).astype(np.int32)
    ids, raw = ["A", "B", "C"], np.array([30.0, 31.5, 29.25])
    mu, ra = rng.uniform(10, 60, r), rng.uniform(0, 9, r)
    host, devf = tmp_path / "h.gz", tmp_path / "d.gz"
    _abi.write_normalized_gz(str(host), ids, raw, mu, ra, zq, level=1)
    _abi.write_normalized_gz_dev(dev, str(devf), ids, raw, mu, ra, dev.upload(zq), n, r, r, level=1)
    assert gzip.open(host, "rb").read() == gzip.open(devf, "rb").read()
    assert devf.stat().st_size < 1.06 * host.stat().st_size


@pytest.mark.parametrize("kind", ["zeros", "period3", "period700", "runs", "short_rows"])
def test_device_writer_lz77_edge_cases(tmp_path, kind):
    """Text the LZ77 parse handles at its limits: 258-byte matches back to
    back (a constant row), overlapping copies at short periods, periods
    longer than any cell, long runs broken at random, rows shorter than a
    4-byte match -- each decompressed by Python's zlib (CRC-checked) equal to
    the host writer's text; matches never reach before their member."""
    from grid_amd import _abi
    dev = _dev()
    rng = np.random.default_rng(11)
    # "runs" rows are longer than a member's 8 MB of text: one member per row
    n, r = {"short_rows": (700, 1), "runs": (3, 1_500_001)}.get(kind, (6, 90_001))
    if kind == "zeros":
        zq = np.zeros((n, r), np.int32)
    elif kind == "period3":
        zq = np.tile(np.array([5, -5, 123], np.int32), (n, r // 3 + 1))[:, :r]
    elif kind == "period700":
        zq = np.tile(rng.integers(-300, 300, 700).astype(np.int32), (n, r // 700 + 1))[:, :r]
    elif kind == "runs":
        zq = np.repeat(rng.integers(-3, 3, (n, r // 997 + 1)).astype(np.int32), 997, axis=1)[:, :r]
        zq.flat[rng.integers(0, zq.size, 500)] = rng.integers(-10 ** 6, 10 ** 6, 500)
    else:
        zq = rng.integers(-5, 5, (n, r)).astype(np.int32)
    ids = [f"S{i}" for i in range(n)]
    raw = rng.uniform(5, 90, n)
    mu, ra = rng.uniform(10, 60, r), rng.uniform(0, 9, r)
    host, devf = tmp_path / "h.gz", tmp_path / "d.gz"
    _abi.write_normalized_gz(str(host), ids, raw, mu, ra, zq, level=1)
    for batch in (0, 300_000):                    # one batch; batches of a few rows
        _abi.write_normalized_gz_dev(dev, str(devf), ids, raw, mu, ra, dev.upload(zq), n, r, r, level=1,
                                     batch_bytes=batch)
        assert gzip.decompress(devf.read_bytes()) == gzip.open(host, "rb").read()
        data, p = devf.read_bytes(), 0
        for _, size in _members(devf):            # every member decodes on its own
            assert gzip.decompress(data[p:p + size])
            p += size
        if kind in ("zeros", "period3"):              # the row members (member 0 holds the header lines)
            rows_gz = sum(size for row, size in _members(devf) if row >= 0)
            rows_text = len(gzip.open(host, "rb").read().split(b"\n", 2)[2])
            assert rows_gz < 0.02 * rows_text


@pytest.mark.parametrize("where", ["tmp", "shm"])
def test_device_writer_direct_and_buffered(tmp_path, where):
    """The writer's two ways to the file -- O_DIRECT for 4 KiB-aligned ranges
    with the unaligned carry through the ordinary descriptor (a disk file
    system), or the ordinary descriptor only (where O_DIRECT is refused) -- give
    the same bytes, over many batches whose sizes are not multiples of 4 KiB."""
    import os
    import tempfile
    from grid_amd import _abi
    dev = _dev()
    n, r = 40, 20011
    ids, raw, mu, ra, zq = _case(n, r, seed=77)
    dz = dev.upload(zq)
    d = tmp_path if where == "tmp" else tempfile.mkdtemp(dir="/dev/shm") if os.path.isdir("/dev/shm") else tmp_path
    outs = []
    for batch in (0, 123457):                     # one batch; ~20 batches of odd sizes
        f = os.path.join(str(d), f"o{batch}.gz")
        _abi.write_normalized_gz_dev(dev, f, ids, raw, mu, ra, dz, n, r, r, level=1, batch_bytes=batch)
        outs.append(open(f, "rb").read())
        _members(f)
        os.remove(f)
    if str(d) != str(tmp_path):
        os.rmdir(d)
    host = tmp_path / "host.gz"
    _abi.write_normalized_gz(str(host), ids, raw, mu, ra, zq, level=1)
    assert gzip.decompress(outs[0]) == gzip.decompress(outs[1]) == gzip.open(host, "rb").read()
