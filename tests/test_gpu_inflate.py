"""gzip inflate on the device (grid_gunzip_batch; grid_amd/csrc/inflate.hip)
against zlib: every DEFLATE block type and strategy, levels 0-9, multi-member
and BGZF files, the golden cohorts' mosdepth files, empty text; corrupt and
truncated files must be rejected exactly when zlib rejects them."""
import gzip
import os
import random
import struct
import zlib

import numpy as np
import pytest

from grid_amd import _abi

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _variants():
    rng = random.Random(1)
    texts = [b"", b"a", b"hello hello hello hello", bytes(rng.getrandbits(8) for _ in range(70000)),
             b"".join(b"chr1\t%d\t%d\t%.2f\n" % (i * 1000, i * 1000 + 1000, rng.uniform(0, 100)) for i in range(20000)),
             b"A" * 100000, bytes(range(256)) * 300]
    # matches beyond the LDS ring (inflate.hip: dist > 8192 - 258 reads the
    # flushed output in HBM), up to DEFLATE's 32768, and both sides of the edge
    rb = lambda k: bytes(rng.getrandbits(8) for _ in range(k))    # noqa: E731
    x, y, a, b = rb(12000), rb(5000), rb(16384), rb(16384)
    texts += [x + y + x, a + b + a]
    for e in (7933, 7934, 7935, 7936, 8192, 8193):
        z = rb(e)
        texts.append(z + z + z[:300])
    out = []
    for t in texts:
        for lvl in (0, 1, 6, 9):
            out.append((gzip.compress(t, compresslevel=lvl), t))
        out.append((gzip.compress(t[: len(t) // 2], 1) + gzip.compress(t[len(t) // 2:], 9), t))
        for strat in (zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE):
            c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, strat)
            out.append((c.compress(t) + c.flush(), t))
    return out


def _bgzf(data, block=65280):
    o = bytearray()
    for a in range(0, len(data), block):
        ch = data[a:a + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        body = c.compress(ch) + c.flush()
        o += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<H", 6) + b"BC"
        o += struct.pack("<HH", 2, 12 + 6 + len(body) + 8 - 1) + body + struct.pack("<II", zlib.crc32(ch), len(ch))
    return bytes(o) + bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _run(dev, blobs, caps):
    st, ln, nm, out, off = _abi.gunzip_batch(dev, blobs, caps)
    host = out.numpy()
    return st, [bytes(host[off[f]:off[f] + ln[f]]) for f in range(len(blobs))], nm


def _zlib(b):
    """zlib's verdict on every member back to back (gzip.decompress semantics)."""
    try:
        return gzip.decompress(b) if b else None
    except Exception:
        return None


@pytest.fixture(scope="module")
def dev():
    import torch
    d = _abi.Device(0)
    d.set_stream(torch.cuda.current_stream())
    return d


def test_inflate_variants_equal_zlib(dev):
    cases = _variants()
    mos = sorted(os.listdir(os.path.join(G, "g1", "inputs", "mosdepth")))
    for name in mos:
        b = open(os.path.join(G, "g1", "inputs", "mosdepth", name), "rb").read()
        cases.append((b, gzip.decompress(b)))
    big = b"".join(b"chr1\t%d\t%d\t%.2f\n" % (i * 1000, i * 1000 + 1000, (i * 7919 % 10007) / 100.0)
                   for i in range(300000))
    ib = len(cases)
    cases.append((_bgzf(big), big))                          # BGZF: ~140 members + the EOF member
    cases.append((gzip.compress(big, 1), big))
    cases.append((gzip.compress(big[:5000]) + b"\x00" * 5 + gzip.compress(big[5000:9000]) + b"\x00", big[:9000]))
    blobs = [c for c, _ in cases]
    st, got, nm = _run(dev, blobs, [max(len(t), 1) for _, t in cases])
    for f, (b, t) in enumerate(cases):
        if not t and not b:
            continue
        assert st[f] == 0, (f, st[f])
        assert got[f] == t, f
    assert nm[ib] > 100


def test_inflate_capacity_and_empty(dev):
    t = b"x" * 5000 + b"yz" * 3000
    b = gzip.compress(t, 6)
    st, got, _ = _run(dev, [b, b, b""], [len(t), len(t) - 1, 16])
    assert st[0] == 0 and got[0] == t
    assert st[1] == _abi.GZ_ESPACE
    assert st[2] == _abi.GZ_EHEADER


def test_inflate_rejects_exactly_what_zlib_rejects(dev):
    rng = random.Random(7)
    base = [c for c, t in _variants() if t][::3]
    blobs, refs = [], []
    for b in base:
        for k in range(6):
            x = bytearray(b)
            if k % 2 == 0:
                x = x[: rng.randrange(len(x) + 1)]
            else:
                for _ in range(1 + k // 2):
                    i = rng.randrange(len(x))
                    x[i] ^= 1 << rng.randrange(8)
            blobs.append(bytes(x))
            refs.append(_zlib(bytes(x)))
    st, got, _ = _run(dev, blobs, [1 << 20] * len(blobs))
    for f, r in enumerate(refs):
        if r is None:
            assert st[f] != 0, f
        else:
            assert st[f] == 0 and got[f] == r, (f, st[f])


@pytest.mark.parametrize("mcap", [4, 1])
def test_streams_at_any_offset(dev, mcap):
    """The ingest's member-granular launch: every BGZF member is its own
    stream, packed at any byte offset, its text at any byte offset (the
    members of a file back to back) -- and the reject cases with them.
    mcap = 1 is the ingest's launch (k_member_check: a wave per member); a
    member whose trailer CRC is changed must be rejected (GZ_ECRC)."""
    rng = random.Random(11)
    texts = [b"".join(b"chr1\t%d\t%d\t%.2f\n" % (i * 1000, i * 1000 + 1000, rng.uniform(0, 90))
                      for i in range(n)) for n in (1, 700, 9000)]
    streams, refs = [], []
    for t in texts:
        bg = _bgzf(t, block=rng.choice([4093, 65280]))
        ms, ml, mi = _abi.gz_members(bg)
        for s_, l_, i_ in zip(ms, ml, mi):
            streams.append(bg[s_:s_ + l_])
            refs.append(zlib.decompress(bg[s_:s_ + l_], 31))
            assert len(refs[-1]) == i_
    # one member far past 64 KiB (several 1 KiB chunks per lane in the check),
    # first, so the corrupt copies below stay within the 64 KiB cap
    streams.insert(0, gzip.compress(texts[2], 6))
    refs.insert(0, texts[2])
    streams.append(gzip.compress(texts[1], 1)[:-9])        # truncated
    refs.append(None)
    for k in (1, len(streams) // 2, len(streams) - 2):    # a wrong trailer CRC: every byte decodes
        x = bytearray(streams[k])
        x[-8 + rng.randrange(4)] ^= 1 << rng.randrange(8)
        streams.append(bytes(x))
        refs.append(None)
    src = bytearray(b"\x00" * 3)
    in_off, out_off, caps = [], [], []
    opos = 5
    for b, r in zip(streams, refs):
        src += b"\x00" * rng.randrange(0, 4)
        in_off.append(len(src))
        src += b
        out_off.append(opos)
        caps.append(len(r) if r is not None else 1 << 16)
        opos += caps[-1] + rng.randrange(0, 3)
    n = len(streams)
    d_src = dev.upload(np.frombuffer(bytes(src) + b"\x00" * 256, np.uint8))
    d_io, d_il = dev.upload(np.array(in_off, np.int64)), dev.upload(np.array([len(b) for b in streams], np.int64))
    d_oo, d_cap = dev.upload(np.array(out_off, np.int64)), dev.upload(np.array(caps, np.int64))
    out = dev.alloc(opos + 256, np.uint8)
    mem = dev.alloc(n * mcap * _abi.GZ_MEMBER_BYTES, np.uint8)
    st, ln, nm = dev.alloc(n, np.int32), dev.alloc(n, np.int64), dev.alloc(n, np.int32)
    _abi.call("grid_gunzip_batch", dev.ctx, d_src.ptr, d_io.ptr, d_il.ptr, n, out.ptr, d_oo.ptr, d_cap.ptr, mem.ptr,
              mcap, st.ptr, ln.ptr, nm.ptr)
    st, ln, host = st.numpy(), ln.numpy(), out.numpy()
    assert all(st[f] == _abi.GZ_ECRC for f in range(n - 3, n))
    for f, r in enumerate(refs):
        if r is None:
            assert st[f] != 0
        else:
            assert st[f] == 0 and bytes(host[out_off[f]:out_off[f] + ln[f]]) == r, f
