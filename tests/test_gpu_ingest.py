"""Step-4 ingest on the device (grid_amd/utils/ingest_device.py: gzip inflate,
mosdepth parse, population means, valid columns, row order -- all in HBM)
against the host parser ingest_native (itself pinned to the reference's
golden cohorts and the line-by-line restatement in test_ingest_cpu.py and
test_host_cpu.py): the same ids, regions and matrix, bit for bit, or the
documented hand-over to the host parser for cohorts outside the device path's
common case."""
import gzip
import os
import shutil

import numpy as np
import pytest
import yaml

from grid_amd import _abi
from grid_amd.utils import ingest_device
from grid_amd.utils import normalize_mosdepth as nm
from tests.test_ingest_cpu import _bgzf, _cohort, _rand_lines

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    import torch
    d = _abi.Device(0)
    d.set_stream(torch.cuda.current_stream())
    return d


SPLITS = {
    "gpu": lambda self, files, text, bgzf: (sorted(files), []),
    "cpu": lambda self, files, text, bgzf: ([], sorted(files)),
    "alternate": lambda self, files, text, bgzf: (sorted(files)[0::2], sorted(files)[1::2]),
}


def _batch_alternate(self, files, text, bgzf):
    # whole batches alternate between the sides: the text of a GPU-inflated
    # batch is then overwritten in d_text by the next batch's copy stream
    self.calls = getattr(self, "calls", 0) + 1
    return (sorted(files), []) if self.calls % 2 else ([], sorted(files))


SPLITS["batches"] = _batch_alternate


@pytest.fixture(params=["model", "gpu", "cpu", "alternate", "batches"])
def split(request, monkeypatch):
    """Which side inflates: the cost model, or forced GPU / CPU / every other
    file / every other batch."""
    if request.param != "model":
        monkeypatch.setattr(ingest_device._Split, "plan", SPLITS[request.param])
    return request.param


def _dev_vs_host(dev, d, samples, chrom=None, start=None, end=None, excluded=None, lo=20, hi=100):
    # the file order is the caller's sample order, not the directory's glob
    # order: the device path takes the first batch's largest file as its key
    # list, and a later file with a key outside it hands the cohort to the host
    # parser (test_short_file_first_stays_on_the_device) -- the r03af failure was
    # a shorter file first in one box's directory order, when the first file
    # that inflated was the key list
    m = nm.map_mosdepth_files_to_samples(d, samples)
    inds = {s: m[s] for s in samples if s in m}
    ex = excluded or {}
    a = nm._ingest_dev(dev, inds, d, chrom, start, end, ex, lo, hi, 4)
    b = nm.ingest_native(inds, d, chrom, start, end, ex, lo, hi, 4)
    assert a[0] == b[0], (a[0], b[0])
    assert a[1] == b[1]
    qa = a[2].numpy() if isinstance(a[2], _abi.DevBuf) else a[2]
    assert qa.shape == b[2].shape and np.array_equal(qa, b[2])
    return a


def test_random_cohorts(dev, tmp_path, split):
    rng = np.random.default_rng(1)
    files = {f"S{i:03d}": _rand_lines(rng, 3000) for i in range(12)}
    d = _cohort(tmp_path, files, members=1)
    a = _dev_vs_host(dev, d, sorted(files) + ["MISSING1"])
    assert len(a[0]) == 12 and a[2].shape[1] > 100
    # window, mask, chromosome prefix
    _dev_vs_host(dev, d, sorted(files), chrom="1", start=500_000, end=2_000_000, excluded={"chr1": {7, 8, 900}})


def test_files_of_many_parse_chunks(dev, tmp_path):
    """Files of ~4.5 MB of text: ~275 16 KiB parse chunks each, so the
    per-file newline scan (k_md_scan, a workgroup per file, 256 chunks a
    round) carries its running base across rounds; the device matrix must equal
    the host parser's."""
    rng = np.random.default_rng(5)
    files = {f"L{i}": _rand_lines(rng, 200_000 - 7919 * i) for i in range(3)}
    d = _cohort(tmp_path, files, members=1)
    a = _dev_vs_host(dev, d, sorted(files))
    assert len(a[0]) == 3


def test_golden_cohorts(dev, tmp_path):
    """g1b / g1c on the device path; g1's chr10 decoy lines repeat chr1's
    (start, end) keys (reference quirk Q1, last line wins) -- outside the
    device path, handed over to the host parser, same result."""
    for name in ("g1", "g1b", "g1c"):
        c = yaml.safe_load(open(os.path.join(G, name, "config.yaml")))
        src = os.path.join(G, name, "inputs")
        samples = [s.strip() for s in open(os.path.join(src, "samples.txt")) if s.strip()]
        ex = nm.load_repeat_mask(os.path.join(src, "mask.bed"))
        kw = dict(chrom=c.get("chrom"), start=c.get("start_bp"), end=c.get("end_bp"), excluded=ex,
                  lo=c["mosdepth"]["normalize"]["min_depth"], hi=c["mosdepth"]["normalize"]["max_depth"])
        d = os.path.join(src, "mosdepth")
        if name == "g1":
            inds = nm.map_mosdepth_files_to_samples(d, samples)
            with pytest.raises(ingest_device.DeviceIngestUnsupported):
                nm._ingest_dev(dev, inds, d, kw["chrom"], kw["start"], kw["end"], ex, kw["lo"], kw["hi"], 2)
            continue
        _dev_vs_host(dev, d, samples, **kw)


def test_subsets_bgzf_empty_corrupt_and_zero_depth(dev, tmp_path, split, monkeypatch):
    # small batches and staging: several batches, both staging buffers reused
    monkeypatch.setattr(ingest_device, "BATCH_IN", 48 << 10)
    monkeypatch.setattr(ingest_device, "STAGE", 64 << 10)
    rng = np.random.default_rng(2)
    base = _rand_lines(rng, 5000)
    files = {}
    for i in range(8):
        lines = list(base)
        for j in rng.choice(len(lines), 40, replace=False):            # zero-depth bins: keys missing per file
            lines[j] = lines[j].rsplit("\t", 1)[0] + "\t0.00\n"
        if i == 3:
            lines = lines[:4000]                                        # a shorter file (a subset of the keys)
        files[f"S{i:03d}"] = lines
    d = tmp_path / "md"
    d.mkdir()
    for k, (name, lines) in enumerate(files.items()):
        data = "".join(lines).encode()
        blob = _bgzf(data) if k % 2 else gzip.compress(data, 6)
        (d / f"{name}.regions.bed.gz").write_bytes(blob)
    (d / "E000.regions.bed.gz").write_bytes(b"")                       # empty file: no lines
    good = (d / "S001.regions.bed.gz").read_bytes()
    (d / "C000.regions.bed.gz").write_bytes(good[: len(good) // 2])    # truncated: dropped
    (d / "N000.regions.bed.gz").write_bytes(b"not a gzip file at all")  # dropped
    bg = bytearray(_bgzf("".join(files["S001"]).encode()))
    bg[len(bg) // 2] ^= 0x55                                            # a corrupt BGZF member: dropped
    (d / "B000.regions.bed.gz").write_bytes(bytes(bg))
    samples = sorted(files) + ["E000", "C000", "N000", "B000"]
    a = _dev_vs_host(dev, d, samples)
    assert len(a[0]) == 8


def test_short_file_first_stays_on_the_device(dev, tmp_path):
    """The r03af case: a file holding only a subset of the
    bins, or a truncated file, sorted first.  The device path's key list K is
    the first batch's LARGEST file, so the cohort stays on the device and
    equals the host parser's matrix (the earlier rule -- the first file that
    inflated -- handed the whole cohort to the ~5x slower host parser).  Which
    file is first follows the directory's glob order
    (map_mosdepth_files_to_samples, reference normalize_mosdepth.py:162)."""
    rng = np.random.default_rng(2)
    base = _rand_lines(rng, 3000)
    files = {"A_short": base[:2500], "B_full": base, "C_full": list(base)}
    d = _cohort(tmp_path, files, members=1)
    good = (d / "B_full.regions.bed.gz").read_bytes()
    (d / "A_trunc.regions.bed.gz").write_bytes(good[: len(good) // 3])      # truncated: dropped
    for order in (["A_short", "B_full", "C_full"], ["A_trunc", "A_short", "B_full", "C_full"],
                  ["B_full", "A_short", "C_full"]):
        a = _dev_vs_host(dev, d, order)
        assert "A_short" in a[0] and "A_trunc" not in a[0]


def test_no_file_of_the_first_batch_holds_every_key_hands_over(dev, tmp_path):
    """When even the first batch's largest file lacks a key another file has,
    that file's record falls outside K and the device path hands the cohort
    over (DeviceIngestUnsupported); ingest() then returns the host parser's
    result, and the device ingest's cached buffers and staging are released."""
    from grid_amd.device import release_ingest_buffers
    rng = np.random.default_rng(4)
    base = _rand_lines(rng, 3000)
    files = {"A_head": base[:2500], "B_tail": base[400:]}       # B larger; A holds keys B lacks
    d = _cohort(tmp_path, files, members=1)
    m = nm.map_mosdepth_files_to_samples(d, list(files))
    inds = {k: m[k] for k in files}
    with pytest.raises(ingest_device.DeviceIngestUnsupported, match="a key outside K"):
        nm._ingest_dev(dev, inds, d, None, None, None, {}, 20, 100, 2)
    release_ingest_buffers(dev)
    got = nm.ingest(inds, d, None, None, None, {}, 20, 100, 2, dev=dev)
    exp = nm.ingest_native(inds, d, None, None, None, {}, 20, 100, 2)
    assert got[0] == exp[0] and got[1] == exp[1]
    assert np.array_equal(np.asarray(got[2]), np.asarray(exp[2]))
    assert dev.cached_bytes() == 0 and ingest_device.staging_bytes() == 0


def test_outside_the_common_case_hands_over(dev, tmp_path):
    """Unsorted reference keys, duplicate keys, keys outside the reference,
    non-canonical text: DeviceIngestUnsupported, and ingest() gives the host
    parser's result."""
    rng = np.random.default_rng(3)
    base = _rand_lines(rng, 800)
    cases = {
        "unsorted": ([base[5]] + base[:5] + base[6:], base),
        "dup": (base, base[:100] + [base[50]] + base[100:]),
        # each file holds a key the other lacks: outside K whichever is larger
        "extra_key": (base[:-2] + [base[-1]], base[:-1]),
        "exotic": (base, base[:10] + ["chr1\t9999000\t9999100\t3e1\n"] + base[10:]),
    }
    for name, (la, lb) in cases.items():
        root = tmp_path / name
        root.mkdir()
        d = _cohort(root, {"A": la, "B": lb})
        m = nm.map_mosdepth_files_to_samples(d, ["A", "B"])
        inds = {k: m[k] for k in ("A", "B")}
        with pytest.raises(ingest_device.DeviceIngestUnsupported):
            nm._ingest_dev(dev, inds, d, None, None, None, {}, 20, 100, 2)
        got = nm.ingest(inds, d, None, None, None, {}, 20, 100, 2, dev=dev)
        exp = nm.ingest_native(inds, d, None, None, None, {}, 20, 100, 2) if name != "exotic" else \
            nm.ingest_py(inds, d, None, None, None, {}, 20, 100, 2)
        assert got[0] == exp[0] and got[1] == exp[1]
        assert np.array_equal(np.asarray(got[2]), np.asarray(exp[2]))


def test_host_text_guard_catches_a_corrupt_byte(dev, tmp_path, monkeypatch):
    """The guard over host-inflated text: a byte of
    d_text overwritten after the copy to HBM is caught by the CRC check before
    the parse (DeviceIngestUnsupported), and ingest() then returns the host
    parser's result.  Without the corruption the guard passes and the device
    path gives the host parser's result itself."""
    monkeypatch.setattr(ingest_device._Split, "plan", SPLITS["cpu"])
    rng = np.random.default_rng(11)
    files = {f"S{i:03d}": _rand_lines(rng, 2000) for i in range(5)}
    d = _cohort(tmp_path, files, members=1)
    samples = sorted(files)
    _dev_vs_host(dev, d, samples)                      # clean: the guard passes
    hits = []

    def corrupt(dev_, d_text, toff, ks):
        k = ks[len(ks) // 2]
        pos = int(toff[k]) + 700
        b = np.zeros(1, np.uint8)
        _abi.call("grid_d2h", dev_.ctx, b.ctypes.data, d_text.ptr + pos, 1)
        b[0] = ord("7") if b[0] != ord("7") else ord("3")      # a digit for a digit: still parses
        _abi.call("grid_h2d", dev_.ctx, d_text.ptr + pos, b.ctypes.data, 1)
        hits.append(k)

    monkeypatch.setattr(ingest_device, "AFTER_HOST_TEXT", corrupt)
    inds = nm.map_mosdepth_files_to_samples(d, samples)
    with pytest.raises(ingest_device.DeviceIngestUnsupported, match="gzip CRC"):
        nm._ingest_dev(dev, inds, d, None, None, None, {}, 20, 100, 2)
    assert hits
    got = nm.ingest(inds, d, None, None, None, {}, 20, 100, 2, dev=dev)
    exp = nm.ingest_native(inds, d, None, None, None, {}, 20, 100, 2)
    assert got[0] == exp[0] and got[1] == exp[1]
    assert np.array_equal(np.asarray(got[2]), np.asarray(exp[2]))


def test_device_error_hands_over_to_the_host_parser(dev, tmp_path, monkeypatch):
    """a native error in the device path (here: the device buffers
    cannot be allocated) is logged and the host parser reads the cohort."""
    rng = np.random.default_rng(12)
    files = {f"S{i:03d}": _rand_lines(rng, 1500) for i in range(3)}
    d = _cohort(tmp_path, files, members=1)
    inds = nm.map_mosdepth_files_to_samples(d, sorted(files))

    def no_room(*a, **k):
        raise _abi.GridNativeError("hipMalloc: out of memory (test)")

    monkeypatch.setattr(dev, "alloc", no_room)
    got = nm.ingest(inds, d, None, None, None, {}, 20, 100, 2, dev=dev)
    exp = nm.ingest_native(inds, d, None, None, None, {}, 20, 100, 2)
    assert got[0] == exp[0] and got[1] == exp[1]
    assert np.array_equal(np.asarray(got[2]), np.asarray(exp[2]))


def test_text_crc32_matches_zlib(dev):
    """grid_text_crc32 (the guard's device CRC) against zlib over ranges that
    cross its 1 MiB pieces, empty ones and unaligned starts."""
    import zlib
    rng = np.random.default_rng(13)
    data = rng.integers(0, 256, 5 << 20, dtype=np.uint8)
    buf = dev.upload(data)
    offs = [0, 1, 3, 4096, (1 << 20) - 1, 12345, 0, 77]
    lens = [0, 1, 17, 1 << 20, (1 << 20) + 2, (3 << 20) + 5, 5 << 20, 100]
    got = _abi.text_crc32(dev, buf.ptr, offs, lens)
    assert [int(c) for c in got] == [zlib.crc32(data[o:o + n].tobytes()) for o, n in zip(offs, lens)]


@pytest.mark.parametrize("host_frac", [0.0, 0.5])
def test_pipelined_batches_equal_the_host_parser(dev, tmp_path, monkeypatch, host_frac):
    """The pipelined BGZF batches (ingest_device._Async: copies on their own
    stream, no host round trip per batch, failed files skipped on the device)
    against the host parser, and against the synchronous path, over several
    batches with a corrupt member, a truncated file, an empty file and a file
    that is not gzip in later batches.  host_frac 0.5: every second file of a
    batch inflated by the host threads beside the GPU (its text copied into
    HBM behind the previous batch's parse and CRC-checked there; a host file
    that fails to inflate is dropped like a GPU one)."""
    # batches of a few files (one file each when host_frac is 0: many batches)
    monkeypatch.setattr(ingest_device, "BATCH_IN", (120 if host_frac else 40) << 10)
    monkeypatch.setattr(ingest_device, "host_frac", lambda threads: host_frac)
    rng = np.random.default_rng(21)
    base = _rand_lines(rng, 3000)
    files = {}
    for i in range(10):
        lines = list(base)
        for j in rng.choice(len(lines), 30, replace=False):
            lines[j] = lines[j].rsplit("\t", 1)[0] + "\t0.00\n"
        files[f"S{i:03d}"] = lines
    d = tmp_path / "md"
    d.mkdir()
    for name, lines in files.items():
        (d / f"{name}.regions.bed.gz").write_bytes(_bgzf("".join(lines).encode()))
    bg = bytearray(_bgzf("".join(files["S004"]).encode()))
    bg[len(bg) // 2] ^= 0x55
    (d / "X001.regions.bed.gz").write_bytes(bytes(bg))                  # corrupt member: dropped
    good = (d / "S002.regions.bed.gz").read_bytes()
    (d / "X002.regions.bed.gz").write_bytes(good[: len(good) // 2])     # truncated: dropped
    (d / "X003.regions.bed.gz").write_bytes(b"")                        # empty: no lines
    (d / "X004.regions.bed.gz").write_bytes(b"not gzip")                # dropped
    # a BGZF member whose ISIZE understates its text (it inflates past it,
    # GZ_ESPACE): a corrupt member, dropped on every path, as the
    # host parser drops it (the reference's gzip raises on the length check)
    bz = bytearray(_bgzf("".join(files["S005"]).encode()))
    end = int.from_bytes(bz[16:18], "little") + 1                       # BSIZE + 1: the first member's end
    isz = int.from_bytes(bz[end - 4:end], "little")
    bz[end - 4:end] = (isz - 1).to_bytes(4, "little")
    (d / "X005.regions.bed.gz").write_bytes(bytes(bz))
    samples = sorted(files)[:3] + ["X001", "X002"] + sorted(files)[3:] + ["X003", "X004", "X005"]
    calls = []
    orig = ingest_device._Async.batch

    def counted(self, *a, **k):
        calls.append(len(k["hshare"][0]) if k.get("hshare") else 0)
        return orig(self, *a, **k)

    monkeypatch.setattr(ingest_device._Async, "batch", counted)
    a = _dev_vs_host(dev, d, samples)
    assert len(calls) >= 2, "the pipelined path did not run"
    assert (sum(calls) > 0) == (host_frac > 0), calls
    monkeypatch.setattr(ingest_device, "PIPELINE", False)
    b = _dev_vs_host(dev, d, samples)
    assert a[0] == b[0] and a[1] == b[1]
    assert np.array_equal(a[2].numpy(), b[2].numpy())


def test_pipelined_host_share_guard(dev, tmp_path, monkeypatch):
    """The pipelined batches' host share: a byte of host-inflated text changed
    in HBM after its copy is caught by the CRC check on the copy stream, and
    the device path hands the cohort over (DeviceIngestUnsupported); clean, the
    same cohort gives the host parser's result on the device path."""
    monkeypatch.setattr(ingest_device, "BATCH_IN", 120 << 10)
    monkeypatch.setattr(ingest_device, "host_frac", lambda threads: 0.5)
    rng = np.random.default_rng(23)
    base = _rand_lines(rng, 3000)
    d = tmp_path / "md"
    d.mkdir()
    for i in range(8):
        (d / f"S{i:03d}.regions.bed.gz").write_bytes(_bgzf("".join(base).encode()))
    samples = [f"S{i:03d}" for i in range(8)]
    _dev_vs_host(dev, d, samples)
    hits = []

    def corrupt(dev_, d_text, toff, ks):
        k = ks[0]
        pos = int(toff[k]) + 900
        b = np.zeros(1, np.uint8)
        _abi.call("grid_d2h", dev_.ctx, b.ctypes.data, d_text.ptr + pos, 1)
        b[0] = ord("7") if b[0] != ord("7") else ord("3")
        _abi.call("grid_h2d", dev_.ctx, d_text.ptr + pos, b.ctypes.data, 1)
        hits.append(k)

    monkeypatch.setattr(ingest_device, "AFTER_HOST_TEXT", corrupt)
    inds = nm.map_mosdepth_files_to_samples(d, samples)
    with pytest.raises(ingest_device.DeviceIngestUnsupported, match="gzip CRC"):
        nm._ingest_dev(dev, inds, d, None, None, None, {}, 20, 100, 2)
    assert hits
