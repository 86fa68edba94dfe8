"""The device inflater's decoding core (grid_amd/csrc/inflate_core.hpp) on the
host, against zlib: the same Inflater template compiled with g++ over a plain
host policy (tests/native/inflate_core_host.cpp), at the device's fast-table
width (2^8 literal/length entries, round 3) and at the earlier 2^10 -- stored,
fixed and dynamic blocks, codes up to 15 bits (the canonical walk), matches up
to 32 KiB back, multi-member (BGZF) streams, and truncated / corrupt input.
The device's own fast loop is covered against zlib on the GPU
(tests/test_gpu_inflate.py)."""
import ctypes as C
import gzip
import os
import shutil
import struct
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", params=[8, 10])
def core(request, tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not present")
    d = tmp_path_factory.mktemp(f"icore{request.param}")
    so = d / "libicore.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", f"-DGRID_INFLATE_LFAST={request.param}",
                    "-I" + os.path.join(ROOT, "grid_amd", "csrc"), os.path.join(ROOT, "tests", "native",
                                                                                "inflate_core_host.cpp"),
                    "-o", str(so), "-lz"], check=True)
    lib = C.CDLL(str(so))
    lib.host_gunzip.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(C.c_int64),
                                C.POINTER(C.c_int32)]
    assert lib.host_lfast() == request.param
    return lib


def run(lib, blob, cap):
    src = np.frombuffer(blob, np.uint8) if blob else np.zeros(1, np.uint8)
    out = np.zeros(max(cap, 1), np.uint8)
    n, m = C.c_int64(), C.c_int32()
    rc = lib.host_gunzip(src.ctypes.data, len(blob), out.ctypes.data, cap, C.byref(n), C.byref(m))
    return rc, out[: n.value].tobytes(), m.value


def bgzf(data, block=65280, level=6):
    o = b""
    for i in range(0, len(data), block):
        ch = data[i:i + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(ch) + c.flush()
        o += b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC"
        o += struct.pack("<HH", 2, 12 + 6 + len(body) + 8 - 1) + body + struct.pack("<II", zlib.crc32(ch), len(ch))
    return o


def mosdepth_text(rng, n):
    pos = np.cumsum(rng.integers(1, 3, n)) * 1000
    dep = rng.gamma(2.0, 15.0, n)
    return "".join(f"chr{1 + (i * 7) // n}\t{p}\t{p + 1000}\t{d:.2f}\n" for i, (p, d) in enumerate(zip(pos, dep))).encode()


def skewed(rng, n):
    # a steep symbol distribution: dynamic blocks with literal codes of 12-15 bits
    p = 0.5 ** np.arange(1, 40)
    p = p / p.sum()
    return bytes(rng.choice(np.arange(39) * 5 + 17, size=n, p=p).astype(np.uint8))


CASES = {
    "text_l1": lambda r: gzip.compress(mosdepth_text(r, 4000), 1),
    "text_l6": lambda r: gzip.compress(mosdepth_text(r, 4000), 6),
    "text_l9": lambda r: gzip.compress(mosdepth_text(r, 4000), 9),
    "random_stored": lambda r: gzip.compress(bytes(r.integers(0, 256, 70000, dtype=np.uint8)), 6),
    "level0": lambda r: gzip.compress(mosdepth_text(r, 500), 0),
    "tiny_fixed": lambda r: gzip.compress(b"chr1\t0\t1000\t12.34\n", 9),
    "empty": lambda r: gzip.compress(b"", 6),
    "skewed_long_codes": lambda r: gzip.compress(skewed(r, 200000), 9),
    "far_matches": lambda r: gzip.compress((bytes(r.integers(0, 256, 30000, dtype=np.uint8)) * 3), 9),
    "bgzf_members": lambda r: bgzf(mosdepth_text(r, 6000)),
    "two_members": lambda r: gzip.compress(b"a" * 1000, 6) + gzip.compress(mosdepth_text(r, 300), 1),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_core_equals_zlib(core, name):
    rng = np.random.default_rng(sum(map(ord, name)))
    blob = CASES[name](rng)
    exp = gzip.decompress(blob)
    rc, got, m = run(core, blob, len(exp) + 64)
    assert rc == 0, rc
    assert got == exp
    assert m >= 1


def test_long_codes_really_occur(core):
    # the skewed case must reach codes longer than the fast table (else it tests nothing)
    rng = np.random.default_rng(5)
    data = skewed(rng, 200000)
    counts = np.bincount(np.frombuffer(data, np.uint8), minlength=256)
    assert (counts[counts > 0].min() / len(data)) < 2.0 ** -12


def test_corrupt_and_truncated_are_rejected(core):
    rng = np.random.default_rng(9)
    data = mosdepth_text(rng, 3000)
    blob = bytearray(gzip.compress(data, 6))
    rc, _, _ = run(core, bytes(blob[: len(blob) // 2]), len(data) + 64)
    assert rc != 0                                    # truncated
    blob[len(blob) // 2] ^= 0x40
    rc, _, _ = run(core, bytes(blob), len(data) + 64)
    assert rc != 0                                    # corrupt: a data or CRC error, never a silent decode
    rc, _, _ = run(core, b"not a gzip stream", 100)
    assert rc == 4                                    # E_HEADER
    rc, _, _ = run(core, gzip.compress(data, 6), len(data) - 1)
    assert rc == 3                                    # E_SPACE: never writes past the capacity
