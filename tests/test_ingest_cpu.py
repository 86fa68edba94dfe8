"""Host C++ mosdepth ingest (grid_ingest_*, grid_amd/csrc/ingest.cpp) against
the line-by-line restatement of normalize_mosdepth.py:218-416 (ingest_py,
itself pinned to the oracle and the reference's golden cohorts in
test_host_cpu.py).  CPU only: the ingest is host code."""
import gzip
import os

import numpy as np
import pytest

from grid_amd import _abi
from grid_amd.utils import normalize_mosdepth as nm
from oracle import ingest as oracle_ingest

G = os.path.join(os.path.dirname(__file__), "golden")


def _write(path, lines, gz=True, members=1):
    data = "".join(lines).encode()
    if not gz:
        path.write_bytes(data)
        return
    # several gzip members back to back (BGZF-like)
    cut = [len(data) * i // members for i in range(members + 1)]
    with open(path, "wb") as f:
        for a, b in zip(cut, cut[1:]):
            f.write(gzip.compress(data[a:b]))


def _cohort(tmp_path, files, gz=True, members=1):
    d = tmp_path / "md"
    d.mkdir()
    for name, lines in files.items():
        _write(d / f"{name}.regions.bed.gz", lines, gz=gz, members=members)
    return d


def _both(d, samples, chrom=None, start=None, end=None, excluded=None, lo=20, hi=100, threads=3, **kw):
    inds = nm.map_mosdepth_files_to_samples(d, samples)
    ex = excluded or {}
    a = nm.ingest_native(inds, d, chrom, start, end, ex, lo, hi, threads, **kw)
    b = nm.ingest_py(inds, d, chrom, start, end, ex, lo, hi, threads)
    return a, b


def _same(a, b):
    assert a[0] == b[0]
    assert a[1] == b[1]
    assert a[2].shape == b[2].shape and np.array_equal(a[2], b[2])


def _rand_lines(rng, n, chrom="chr1", step=1000, lo=5.0, hi=120.0):
    out = []
    for i in range(n):
        d = rng.uniform(lo, hi)
        out.append(f"{chrom}\t{i * step}\t{(i + 1) * step}\t{d:.2f}\n")
    return out


def test_random_cohort_matches(tmp_path):
    rng = np.random.default_rng(1)
    files = {f"S{i:03d}": _rand_lines(rng, 3000) for i in range(12)}
    d = _cohort(tmp_path, files, members=3)
    a, b = _both(d, sorted(files))
    _same(a, b)
    assert a[2].shape[0] == 12 and a[2].shape[1] > 100


def test_streaming_mode_matches(tmp_path, monkeypatch):
    rng = np.random.default_rng(2)
    files = {f"S{i:03d}": _rand_lines(rng, 2000) for i in range(6)}
    d = _cohort(tmp_path, files)
    inds = nm.map_mosdepth_files_to_samples(d, sorted(files))
    paths = [str(nm.find_bed_gz_for_individual(i, d)) for i in inds]
    full = _abi.Ingest(paths, None, None, {}, 20, 100, threads=2)
    stream = _abi.Ingest(paths, None, None, {}, 20, 100, threads=2, cache_bytes=0)
    rof = np.arange(len(paths), dtype=np.int32)
    assert np.array_equal(full.fill(rof), stream.fill(rof))
    assert full.population_means() == stream.population_means()


def test_population_means_are_the_reference_chain(tmp_path):
    """Sums in sample order, fp64, float(text) each (normalize_mosdepth.py:218-301)."""
    rng = np.random.default_rng(3)
    files = {f"S{i:03d}": _rand_lines(rng, 500, lo=0.01, hi=3.0) for i in range(25)}
    d = _cohort(tmp_path, files)
    inds = nm.map_mosdepth_files_to_samples(d, sorted(files))
    paths = [str(nm.find_bed_gz_for_individual(i, d)) for i in inds]
    ing = _abi.Ingest(paths, None, None, {}, 0, 1e9, threads=4)
    got = ing.population_means()
    exp = nm.compute_population_mean_depths(inds, d, None, None, None, {}, threads=1)
    assert got.keys() == exp.keys()
    assert all(got[k] == exp[k] for k in exp)     # bit-exact


def test_quirks_chrom_prefix_window_mask_duplicates(tmp_path):
    lines_a = [
        "chr1\t0\t1000\t30.00\n",
        "chr10\t0\t1000\t55.50\n",          # startswith("chr1") quirk: same (s, e) key, last wins
        "chr1\t1000\t2000\t40.1\n",
        "chr1\t2000\t3000\t0.00\n",          # depth 0 dropped
        "chr1\t3000\t4000\t-5\n",            # negative depth dropped
        "chr2\t4000\t5000\t44.00\n",         # other chromosome
        "chr1\t6000\t7000\t35\n",
        "chr1\t5000\t6000\t33.33\n",         # unsorted
        "chr1\t7000\t9000\t36.00\n",         # masked (kb 7..9)
        "chr1\t9500\t9600\t37.00\t\textra\n",
        "chr1\t12000\t13000\t38.00\t\n",     # trailing tab stripped
        "short\tline\n",
        "\n",
    ]
    lines_b = [l.replace("30.00", "31.00") for l in lines_a]
    d = _cohort(tmp_path, {"A": lines_a, "B": lines_b})
    for chrom in (None, "1", "chr1"):
        for win in ((None, None), (1500, 9550), (0, 100000)):
            a, b = _both(d, ["A", "B"], chrom=chrom, start=win[0], end=win[1], excluded={"chr1": {8}})
            _same(a, b)
    # with no chromosome filter the "short\tline" text is still < 4 fields -> skipped


def test_invalid_number_drops_sample(tmp_path):
    good = ["chr1\t0\t1000\t30.00\n", "chr1\t1000\t2000\t40.00\n"]
    bad = ["chr1\t0\t1000\t30.00\n", "chr1\tx\t2000\t40.00\n"]
    bad2 = ["chr1\t0\t1000\t30.00\n", "chr1\t1000\t2000\t4o.00\n"]
    d = _cohort(tmp_path, {"A": good, "B": bad, "C": bad2, "D": good})
    a, b = _both(d, ["A", "B", "C", "D", "E"])       # E: no file
    _same(a, b)
    assert a[0] == ["A", "D"]


def test_exotic_text_falls_back_identically(tmp_path, capsys):
    rng = np.random.default_rng(4)
    base = _rand_lines(rng, 50, lo=20.0, hi=90.0)
    variants = {
        "exp": base + ["chr1\t50000\t51000\t3e1\n"],
        "ws": base + ["chr1\t50000\t51000\t 30.00\n"],
        "crlf": [l.replace("\n", "\r\n") for l in base],
        "under": base + ["chr1\t50_000\t51000\t30.00\n"],
        "decimals": base + ["chr1\t50000\t51000\t30.125\n"],
        "nan": base + ["chr1\t50000\t51000\tnan\n"],
    }
    for k, extra in variants.items():
        sub = tmp_path / k
        sub.mkdir()
        d = _cohort(sub, {"A": base, "B": extra})
        inds = nm.map_mosdepth_files_to_samples(d, ["A", "B"])
        with pytest.raises(_abi.IngestUnsupported):
            nm.ingest_native(inds, d, None, None, None, {}, 20, 100, 2)
        if k == "decimals":
            # the reference keeps 30.125 in the matrix: the cohort takes the fp64
            # route (NaN missing), equal to the oracle's float matrix
            ids, regs, x = nm.ingest(inds, d, None, None, None, {}, 20, 100, 2)
            o_ids, o_regs, o_mat = oracle_ingest.ingest(d, ["A", "B"], None, None, None, None, 20, 100)
            assert x.dtype == np.float64 and ids == o_ids and regs == o_regs
            assert np.array_equal(x, o_mat, equal_nan=True) and (x == 30.125).sum() == 1
            assert "fp64" in capsys.readouterr().out
            continue
        got = nm.ingest(inds, d, None, None, None, {}, 20, 100, 2)
        _same(got, nm.ingest_py(inds, d, None, None, None, {}, 20, 100, 2))


def test_plain_text_and_empty_files(tmp_path):
    rng = np.random.default_rng(5)
    d = tmp_path / "md"
    d.mkdir()
    _write(d / "A.regions.bed.gz", _rand_lines(rng, 300), gz=False)   # not gzip: Python drops the sample
    _write(d / "B.regions.bed.gz", _rand_lines(rng, 300))
    _write(d / "C.regions.bed.gz", [])
    a, b = _both(d, ["A", "B", "C"])
    _same(a, b)


def test_depth_boundaries_of_the_valid_filter(tmp_path):
    """Population means landing exactly on min/max depth (inclusive)."""
    lines = lambda v: [f"chr1\t{i * 1000}\t{(i + 1) * 1000}\t{v[i]}\n" for i in range(len(v))]  # noqa: E731
    d = _cohort(tmp_path, {"A": lines(["20.00", "100.00", "19.99", "100.01", "20.10"]),
                           "B": lines(["20.00", "100.00", "20.01", "99.99", "19.90"])})
    a, b = _both(d, ["A", "B"])
    _same(a, b)
    assert len(a[1]) == 5      # every mean lands on 20.0 or 100.0 (inclusive bounds)


@pytest.mark.parametrize("name", ["g1", "g1b", "g1c"])
def test_golden_cohorts_streaming(name, monkeypatch):
    import yaml
    with open(os.path.join(G, name, "config.yaml")) as f:
        c = yaml.safe_load(f)
    p = lambda r: os.path.join(G, name, r)  # noqa: E731
    ncfg = c["mosdepth"]["normalize"]
    samples = [s.strip() for s in open(p(c["samples_file"])) if s.strip()]
    wd = p(c["mosdepth"]["work_dir"])
    inds = nm.map_mosdepth_files_to_samples(wd, samples)
    ex = nm.load_repeat_mask(p(ncfg["repeat_mask_file"]))
    args = (inds, wd, c.get("chrom"), c.get("start_bp"), c.get("end_bp"), ex, ncfg["min_depth"],
            ncfg["max_depth"], 4)
    real = _abi.Ingest.__init__
    monkeypatch.setattr(_abi.Ingest, "__init__",
                        lambda self, *a, **k: real(self, *a, **{**k, "cache_bytes": 0}))
    _same(nm.ingest_native(*args), nm.ingest_py(*args))


def test_truncated_and_garbage_gzip_drop_sample(tmp_path):
    rng = np.random.default_rng(6)
    d = tmp_path / "md"
    d.mkdir()
    _write(d / "A.regions.bed.gz", _rand_lines(rng, 400))
    _write(d / "B.regions.bed.gz", _rand_lines(rng, 400))
    blob = (d / "B.regions.bed.gz").read_bytes()
    (d / "B.regions.bed.gz").write_bytes(blob[: len(blob) // 2])          # truncated
    _write(d / "C.regions.bed.gz", _rand_lines(rng, 400))
    a, b = _both(d, ["A", "B", "C"])
    _same(a, b)
    assert a[0] == ["A", "C"]


_ZLIB_ONLY = r'''
import sys, numpy as np
from grid_amd import _abi
paths = sys.argv[2:]
ing = _abi.Ingest(paths, None, None, {}, 20, 100, threads=2)
rof = np.where(ing.status == ing.status[0], np.arange(len(paths)), -1).astype(np.int32)
np.save(sys.argv[1], np.concatenate([ing.status.astype(np.int32), ing.fill(rof).ravel()]))
'''


def test_libdeflate_and_zlib_paths_agree(tmp_path):
    """The whole-file libdeflate inflate (fastgz.hpp) and the streaming zlib
    reader (GRID_NO_LIBDEFLATE=1, a fresh process) give identical matrices,
    for single- and multi-member files and a truncated one."""
    import subprocess
    import sys
    rng = np.random.default_rng(7)
    d = tmp_path / "md"
    d.mkdir()
    _write(d / "A.regions.bed.gz", _rand_lines(rng, 1500))
    _write(d / "B.regions.bed.gz", _rand_lines(rng, 1500), members=4)
    _write(d / "C.regions.bed.gz", _rand_lines(rng, 1500))
    blob = (d / "C.regions.bed.gz").read_bytes()
    (d / "C.regions.bed.gz").write_bytes(blob[: len(blob) - 9])            # truncated trailer
    paths = [str(d / f"{s}.regions.bed.gz") for s in "ABC"]
    ing = _abi.Ingest(paths, None, None, {}, 20, 100, threads=2)
    assert ing.status[0] == ing.status[1] != ing.status[2]       # C dropped on both paths
    rof = np.array([0, 1, -1], dtype=np.int32)
    fast = np.concatenate([ing.status.astype(np.int32), ing.fill(rof).ravel()])
    out = tmp_path / "zlib.npy"
    env = dict(os.environ, GRID_NO_LIBDEFLATE="1")
    subprocess.run([sys.executable, "-c", _ZLIB_ONLY, str(out), *paths], check=True, env=env,
                   cwd=os.path.dirname(os.path.dirname(__file__)))
    assert np.array_equal(fast, np.load(out))


def _bgzf(data: bytes, block=65280):
    """BGZF (what mosdepth writes, via htslib): gzip members of <= 64 KiB of
    text, each with the "BC" extra subfield holding its length - 1, then the
    28-byte empty EOF member."""
    import struct
    import zlib
    out = bytearray()
    for a in range(0, len(data), block):
        chunk = data[a:a + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        bsize = 12 + 6 + len(body) + 8
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<H", 6)
        out += b"BC" + struct.pack("<HH", 2, bsize - 1) + body
        out += struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


def test_bgzf_many_members_linear_time(tmp_path):
    """A real mosdepth file is BGZF: thousands of 64 KiB members and an empty
    EOF member last (ISIZE 0).  The whole-file inflate sizes each member from
    its own BSIZE/ISIZE (fastgz.hpp member_isize), so the cost stays linear in
    the text (the old sizing zero-filled 4x the rest of the file per
    member, quadratic).  Same matrix as the line-by-line restatement."""
    import time
    rng = np.random.default_rng(11)
    d = tmp_path / "md"
    d.mkdir()
    names = ["P1", "P2", "P3"]
    for s in names:
        (d / f"{s}.regions.bed.gz").write_bytes(_bgzf("".join(_rand_lines(rng, 120_000)).encode()))
    assert (d / "P1.regions.bed.gz").stat().st_size > 600_000        # ~50 members per file
    t0 = time.perf_counter()
    a, b = _both(d, names, threads=3)
    _same(a, b)
    paths = [str(d / f"{s}.regions.bed.gz") for s in names]
    t1 = time.perf_counter()
    ing = _abi.Ingest(paths, None, None, {}, 20, 100, threads=1)
    assert list(ing.status) == [0, 0, 0] and ing.m > 50_000
    assert time.perf_counter() - t1 < 5.0, "BGZF inflate is not linear"
    assert t1 - t0 < 120


def test_zero_padding_after_members(tmp_path):
    """CPython's gzip reader (the reference's gzip.open) skips zero bytes after
    a member; the native ingest does too."""
    rng = np.random.default_rng(3)
    d = tmp_path / "md"
    d.mkdir()
    lines = "".join(_rand_lines(rng, 3000)).encode()
    blob = gzip.compress(lines[:40000]) + b"\x00" * 9 + gzip.compress(lines[40000:]) + b"\x00" * 3
    (d / "Z1.regions.bed.gz").write_bytes(blob)
    assert gzip.decompress(blob) == lines
    a, b = _both(d, ["Z1"], threads=1)
    _same(a, b)
    assert a[2].shape[1] > 1000


def test_host_gunzip_and_bgzf_members():
    """grid_gunzip_host (the CPU side of the device ingest) and
    grid_gz_members against zlib / CPython gzip: BGZF, multi-member, zero
    padding, too little room, corrupt and truncated input, not gzip."""
    import gzip
    rng = np.random.default_rng(5)
    t = "".join(_rand_lines(rng, 20000)).encode()
    bg = _bgzf(t)
    ms, ml, mi = _abi.gz_members(bg)
    assert len(ms) == -(-len(t) // 65280) + 1 and int(mi.sum()) == len(t) and mi[-1] == 0
    assert ms[0] == 0 and int(ms[-1] + ml[-1]) == len(bg)
    assert _abi.gz_members(gzip.compress(t)) is None
    cases = [bg, gzip.compress(t, 1), gzip.compress(t[:999]) + b"\0\0" + gzip.compress(t[999:]),
             bg + b"\0" * 7]
    import zlib
    for b in cases:
        out = np.empty(len(t) + 3, np.uint8)
        st, n = _abi.gunzip_host(b, out)
        assert st == 0 and out[:n].tobytes() == t
        # the CRC the device ingest's guard checks HBM against: the members'
        # trailer CRCs combined = the CRC of the whole text
        st, n, crc = _abi.gunzip_host(b, out, with_crc=True)
        assert st == 0 and crc == zlib.crc32(t)
    one = gzip.compress(b"") + gzip.compress(t[:5])            # an empty first member
    assert _abi.gunzip_host(one, np.empty(16, np.uint8), with_crc=True) == (0, 5, zlib.crc32(t[:5]))
    small = np.empty(100, np.uint8)
    assert _abi.gunzip_host(bg, small)[0] == _abi.GZ_ESPACE
    assert _abi.gunzip_host(b"plain text, not gzip", small)[0] == _abi.GZ_EHEADER
    big = np.empty(len(t), np.uint8)
    assert _abi.gunzip_host(bg[: len(bg) // 2], big)[0] == _abi.GZ_EDATA
    x = bytearray(gzip.compress(t, 6))
    x[len(x) // 2] ^= 0x10
    assert _abi.gunzip_host(bytes(x), big)[0] == _abi.GZ_EDATA
    assert _abi.gunzip_host(bg + b"junk after the members", big)[0] == _abi.GZ_EDATA


def test_find_bed_gz_paths_equals_per_sample_glob(tmp_path):
    """One directory listing gives every sample the file the reference's
    per-sample glob (normalize_mosdepth.py:569) finds first, scandir order
    included (S1 also matches S10...; names with the ID inside; no match)."""
    from grid_amd.utils import normalize_mosdepth as nm
    names = ["S10.regions.bed.gz", "S1.regions.bed.gz", "xS3y.regions.bed.gz", "S4.regions.bed.gz.csi",
             "S5regions.bed.gz", "S6_a.regions.bed.gz", "S6.regions.bed.gz", "a[1].regions.bed.gz",
             ".S7.regions.bed.gz", "S8.mosdepth.global.dist.txt"]
    for nmx in names:
        (tmp_path / nmx).write_bytes(b"")
    ids = ["S1", "S10", "S3", "S4", "S5", "S6", "S6_a", "a[1]", "S7", "S8", "S9", "regions"]
    got = nm.find_bed_gz_paths(ids, tmp_path)
    for i in ids:
        assert got[i] == nm.find_bed_gz_for_individual(i, tmp_path), i
    with pytest.raises(ValueError):                  # "**regions.bed.gz": pathlib rejects it, as for the reference
        nm.find_bed_gz_paths([""], tmp_path)


def test_device_ingest_chunk_table():
    """ingest_device._chunks (the parse kernels' chunk table, built with numpy
    per pipelined batch): every file with text cut in CH-byte chunks, in file
    order, its first chunk in cfirst."""
    from grid_amd.utils import ingest_device as d
    rng = np.random.default_rng(3)
    for _ in range(100):
        nb = int(rng.integers(1, 12))
        tlen = rng.integers(0, 5 * d.CH, nb)
        tlen[rng.random(nb) < 0.2] = 0
        files = [f for f in range(nb) if tlen[f] > 0 and rng.random() < 0.8]
        cfile, cstart, cfirst, tot = d._chunks(files, tlen)
        exp = [(f, s) for f in files for s in range(0, int(tlen[f]), d.CH)]
        assert tot == len(exp)
        assert [(int(a), int(b)) for a, b in zip(cfile[:tot], cstart[:tot])] == exp
        assert cfirst.tolist() == [0] + list(np.cumsum([-(-int(tlen[f]) // d.CH) for f in files]))


def test_staging_is_kept_and_grows():
    """The device ingest's host staging (ingest_device._staging): one buffer
    per name for the process, reused while large enough, replaced by a larger
    one when a request outgrows it; the pageable form is an anonymous mapping
    released through a foreign call (no GIL held while it unmaps)."""
    from grid_amd.utils import ingest_device as idv
    name = "test_staging_cpu"
    idv._STAGING.pop(name, None)
    s = idv._staging(name, 1 << 20)
    a = s.get(4096)
    a[:4] = [1, 2, 3, 4]
    assert idv._staging(name, 1 << 20) is s
    b = s.get(1000)                       # fits: the same memory
    assert b.ctypes.data == a.ctypes.data and list(b[:4]) == [1, 2, 3, 4]
    c = s.get(3 << 20)                    # larger than the buffer: a new one
    assert c.nbytes >= 3 << 20
    c[-1] = 7
    s.b.free()
    s.b = None
    idv._STAGING.pop(name, None)


def test_staging_release_and_host_share_from_threads():
    """release_staging() frees every kept staging
    buffer; the pipelined batches' host share is sized from the config's
    `threads` -- none at the reference's default of 1, at its example
    config's 4 and at 16 since round 5's 63 GB/s inflate (a 16 % share
    measured slower than none, r05ah), a share only where the host threads
    would take a fifth of the files or more -- and never above
    GRID_INGEST_HOST_FRAC."""
    from grid_amd.utils import ingest_device as idv
    s = idv._staging("test_release_cpu", 1 << 20)
    s.get(1 << 16)
    assert idv.staging_bytes() >= 1 << 16
    assert idv.release_staging() >= 1 << 16
    assert idv.staging_bytes() == 0 and not idv._STAGING
    assert idv.host_frac(1) == 0.0 and idv.host_frac(4) == 0.0 and idv.host_frac(16) == 0.0
    assert idv.HOST_FRAC_MIN <= idv.host_frac(24) < idv.HOST_FRAC
    assert idv.host_frac(64) == idv.HOST_FRAC
