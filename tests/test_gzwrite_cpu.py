"""Host checks of the device writer's member coding (grid_gz_huffman_member:
the host restatement of k_lz_parse's LZ77 tokens -- same segments, windows,
hash rounds, lazy rule and token chain -- and the same package-merge codes,
canonical codes, block header, symbol tables and CRC-32 as gzwrite.hip's
device kernels): every member must inflate, with zlib and with the library's
own reader, to exactly its text."""
import ctypes as C
import gzip
import os
import zlib

import numpy as np
import pytest

from grid_amd import _abi


def _member(text: bytes) -> bytes:
    lib = _abi.load()
    need = C.c_int64()
    buf = np.zeros(len(text) * 2 + 4096, dtype=np.uint8)
    src = np.frombuffer(text, dtype=np.uint8) if text else np.zeros(1, np.uint8)
    rc = lib.grid_gz_huffman_member(src.ctypes.data, len(text), buf.ctypes.data, buf.size, C.byref(need))
    assert rc == 0, _abi.load().grid_last_error()
    return buf[: need.value].tobytes()


def _z_text(rng, n):
    z = np.clip(rng.normal(0, 1.2, n), -30, 30)
    cells = [f"{v:.2f}" for v in z]
    cells[:: 97] = ["NA"] * len(cells[:: 97])
    cells[1:: 89] = ["-0.00"] * len(cells[1:: 89])
    return ("S0001\t23.45\t" + "\t".join(cells) + "\n").encode()


@pytest.mark.parametrize("case", ["empty", "one", "zrow", "allbytes", "skewed", "long"])
def test_huffman_member_roundtrip(case):
    rng = np.random.default_rng(7)
    text = {
        "empty": b"",
        "one": b"7",
        "zrow": _z_text(rng, 5000),
        "allbytes": bytes(range(256)) * 3,
        "skewed": b"0" * 100000 + b"1",              # length limits: one symbol dominates
        "long": rng.integers(0, 256, 300000, dtype=np.uint8).tobytes(),
    }[case]
    m = _member(text)
    assert gzip.decompress(m) == text
    d = zlib.decompressobj(31)
    assert d.decompress(m) + d.flush() == text and d.eof


def test_huffman_member_is_smallish_on_z_text():
    """LZ77 + Huffman on "%.2f" text: smaller than zlib level 1 (order-0
    Huffman alone, the round-4 writer, was ~1.2x it)."""
    text = _z_text(np.random.default_rng(3), 200000)
    assert len(_member(text)) < 0.95 * len(zlib.compress(text, 1))


@pytest.mark.parametrize("case", ["runs", "period", "window_edge"])
def test_lz77_member_matches(case):
    """Matches at the parse's limits: 258-byte matches back to back,
    overlapping copies (distance < length), repeats exactly at the 2 KiB
    window and 4 KiB segment edges; zlib must inflate each to its text."""
    rng = np.random.default_rng(5)
    if case == "runs":
        text = b"0.00\t" * 50000 + b"x" + b"\t-1.25" * 30000
    elif case == "period":
        text = (b"ab" * 3 + b"c") * 20000
    else:
        blk = rng.integers(48, 58, 2048, dtype=np.uint8).tobytes()
        text = blk + blk + rng.integers(48, 58, 6000, dtype=np.uint8).tobytes() + blk * 5
    m = _member(text)
    assert zlib.decompress(m, 31) == text
    if case != "window_edge":
        assert len(m) < len(text) // 50


def test_reader_takes_huffman_members(tmp_path):
    """A normalised file whose row members are single LZ77 + dynamic-Huffman
    blocks (what the device writer emits) reads back through
    grid_read_normalized_gz."""
    rng = np.random.default_rng(11)
    n, r = 5, 300
    zq = rng.integers(-500, 500, (n, r)).astype(np.int32)
    zq[0, 3] = _abi.ZQ_NAN
    zq[2, 7] = _abi.ZQ_NEG0
    ids = [f"S{i}" for i in range(n)]
    raw = rng.uniform(20, 40, n)
    mu = rng.uniform(20, 40, r)
    ra = rng.uniform(0, 5, r)
    ref = tmp_path / "ref.tsv.gz"
    _abi.write_normalized_gz(str(ref), ids, raw, mu, ra, zq, level=1)
    with gzip.open(ref, "rb") as f:
        lines = f.read().split(b"\n")
    hdr = b"\n".join(lines[:2]) + b"\n"
    rows = [ln + b"\n" for ln in lines[2:-1]]
    out = tmp_path / "huff.tsv.gz"
    with open(out, "wb") as f:
        f.write(gzip.compress(hdr, 1))
        for row in rows:
            f.write(_member(row))
    assert gzip.open(out, "rb").read() == gzip.open(ref, "rb").read()
    got = _abi.read_normalized_gz(str(out))
    want = _abi.read_normalized_gz(str(ref))
    for a, b in zip(got, want):
        if isinstance(a, np.ndarray):
            assert np.array_equal(a, b, equal_nan=True)
        else:
            assert a == b
