"""Haplotype-neighbour loaders in host C++ (grid_load_ibs / grid_load_ibd,
SURVEY 8f #3) against the oracle's restatement of hi_inference.py:34-74 and
:86-172 (oracle/loaders.py) on files built to hit Python's text semantics:
universal newlines, str.strip()/split() whitespace, int()/float() grammars,
header handling, MAX_NBR truncation and the stable longest-first sort.
Inputs the native parser declines (GRID_EUNSUPPORTED) go to the Python
restatement, and the step's loaders return the oracle's lists either way."""
import gzip

import numpy as np
import pytest

from grid_amd import _abi
from grid_amd.utils import hi_inference as hi
from oracle import loaders

IDS = [f"S{i}" for i in range(12)] + ["x_y", "7"]
IDX = {k: i for i, k in enumerate(IDS)}


def lists_of(csr):
    off, nbr, w = csr
    return canon([[(int(nbr[t]), float(w[t])) for t in range(off[h], off[h + 1])] for h in range(len(off) - 1)])


def canon(hap_nbrs):
    """NaN weights (match = nan) compared by value, and -0.0 kept apart from 0.0."""
    return [[(nb, repr(w)) for nb, w in lst] for lst in hap_nbrs]


def write(path, text, gz=False):
    if gz:
        with gzip.open(path, "wb") as f:
            f.write(text.encode())
    else:
        with open(path, "wb") as f:
            f.write(text.encode())
    return str(path)


IBS_HAP_TOKENS = ["1", "2", "+1", " 2", "01", "1_0", "0", "3", "-1", "1.0", "x", "2_", "1"]
IBS_ID_TOKENS = IDS + ["nobody", "S1x"]


def ibs_text(rng, n_lines, eol="\n"):
    out = ["ID\thap\tnbrInd\tcMlen\tcMedge\tIDnbr\thapNbr"]
    for _ in range(n_lines):
        r = rng.random()
        if r < 0.05:
            out.append("")
            continue
        if r < 0.08:
            out.append("   \t ")
            continue
        if r < 0.11:
            out.append("S1 1 2 3")      # short line
            continue
        toks = [rng.choice(IBS_ID_TOKENS), rng.choice(IBS_HAP_TOKENS), str(rng.integers(0, 99)),
                f"{rng.random():.3f}", f"{rng.random():.3f}", rng.choice(IBS_ID_TOKENS),
                rng.choice(IBS_HAP_TOKENS)]
        if rng.random() < 0.1:
            toks.append("extra")
        sep = rng.choice(["\t", " ", "  ", "\t \x1f"])
        lead = rng.choice(["", " ", "\t", "\x0b"])
        out.append(lead + sep.join(toks) + rng.choice(["", " ", "\t", "\x0c"]))
    return eol.join(out) + rng.choice(["", eol])


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("eol", ["\n", "\r\n", "\r"])
def test_ibs_native_equals_oracle(tmp_path, seed, eol):
    rng = np.random.default_rng(seed)
    text = ibs_text(rng, 400, eol)
    for gz in (False, True):
        p = write(tmp_path / ("ibs.tsv.gz" if gz else "ibs.tsv"), text, gz)
        for max_nbr in (0, 1, 3, 50):
            want = canon(loaders.load_ibs(p, IDX, max_nbr))
            assert lists_of(_abi.load_ibs(p, IDS, max_nbr)) == want
            assert canon(hi._load_ibs_neighbors(p, IDX, max_nbr)) == want


def ibd_text(rng, n_lines, eol="\n"):
    out = []
    for _ in range(n_lines):
        r = rng.random()
        if r < 0.05:
            out.append("")
            continue
        if r < 0.08:
            out.append("a\tb\tc")
            continue
        a, b = rng.choice(IBS_ID_TOKENS), rng.choice(IBS_ID_TOKENS)
        ha = f"{a}_{rng.choice(['0', '1', '1', '0', '2', 'x', '+1', '0_0', ''])}"
        hb = f"{b}_{rng.choice(['0', '1', '1', '0', '-0', ' 1'])}"
        bp1 = int(rng.integers(1_000_000, 2_000_000))
        bp2 = bp1 + int(rng.integers(0, 400_000))
        length = rng.choice([f"{rng.uniform(0.2, 9):.2f}", "1.5", "1.5", "2", "1e0", "inf", "1_0.5", ".5", "5.",
                             "x", "-inf"])
        match = rng.choice([f"{rng.uniform(0.5, 1):.3f}", "0.9", "1", "0.7", "0.69", "nan", "INF"])
        toks = [a, ha, b, hb, "chr1", str(bp1) if rng.random() > 0.05 else f"{bp1:_}", str(bp2),
                "rs1", "rs2", length, match]
        if rng.random() < 0.3:
            line = " ".join(toks) if rng.random() < 0.5 else "  ".join(toks)
        else:
            line = "\t".join(toks)
            if rng.random() < 0.1:
                line = line.replace("\t", " \t", 1)
        out.append(rng.choice(["", " "]) + line + rng.choice(["", "\t", " "]))
    return eol.join(out) + rng.choice(["", eol])


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("eol", ["\n", "\r\n"])
def test_ibd_native_equals_oracle(tmp_path, seed, eol):
    rng = np.random.default_rng(100 + seed)
    text = ibd_text(rng, 500, eol)
    for gz in (False, True):
        p = write(tmp_path / ("ibd.txt.gz" if gz else "ibd.txt"), text, gz)
        for max_nbr in (0, 2, 7, 100):
            for weighted in (False, True):
                for ml, mm, ws in ((0.5, 0.7, 1_000_000), (0.0, 0.0, 250_000.5), (2.0, 0.9, 1)):
                    args = (p, IDX, max_nbr, 1_300_000, 1_500_000, ml, mm, weighted, ws)
                    want = canon(loaders.load_ibd(*args))
                    got = lists_of(_abi.load_ibd(p, IDS, max_nbr, 1_300_000, 1_500_000, ml, mm, weighted, ws))
                    assert got == want
                    assert canon(hi._load_ibd_neighbors(*args)) == want


def test_ibd_equal_lengths_keep_file_order(tmp_path):
    rows = [f"S0\tS0_0\tS{j}\tS{j}_1\tc\t10\t20\ta\tb\t{1.0 if j % 2 else 2.0}\t0.9" for j in range(1, 10)]
    p = write(tmp_path / "ibd.txt", "\n".join(rows))
    want = canon(loaders.load_ibd(p, IDX, 6, 0, 100, 0.5, 0.7, False, 1_000_000))
    assert lists_of(_abi.load_ibd(p, IDS, 6, 0, 100, 0.5, 0.7, False, 1_000_000)) == want
    assert [nb for nb, _ in want[0]] == [2 * j + 1 for j in (2, 4, 6, 8, 1, 3)]


def test_ibs_header_only_and_blank_first_line(tmp_path):
    for text in ("header only", "\nS1 1 0 0 0 S2 2\n", "S1 1 0 0 0 S2 2\nS1 1 0 0 0 S3 2\n"):
        p = write(tmp_path / "ibs.tsv", text)
        assert lists_of(_abi.load_ibs(p, IDS, 5)) == canon(loaders.load_ibs(p, IDX, 5))


@pytest.mark.parametrize("case", ["nonascii", "dup_ids", "nan_len", "empty_ibs", "zero_div"])
def test_declined_inputs_fall_back(tmp_path, case):
    ids, idx = IDS, IDX
    if case == "nonascii":
        p = write(tmp_path / "ibs.tsv", "h\nS1 1 0 0 0 S2 2\nSé 1 0 0 0 S2 2\n")
        with pytest.raises(_abi.GridNativeError) as e:
            _abi.load_ibs(p, ids, 5)
        assert e.value.code == _abi.GRID_EUNSUPPORTED
        assert hi._load_ibs_neighbors(p, idx, 5) == loaders.load_ibs(p, idx, 5)
    elif case == "dup_ids":
        p = write(tmp_path / "ibs.tsv", "h\nS1 1 0 0 0 S2 2\n")
        with pytest.raises(_abi.GridNativeError) as e:
            _abi.load_ibs(p, ids + ["S1"], 5)
        assert e.value.code == _abi.GRID_EUNSUPPORTED
        assert hi._ids_in_order({"S1": 1, "S2": 1}) is None
    elif case == "nan_len":
        p = write(tmp_path / "ibd.txt", "S1\tS1_0\tS2\tS2_1\tc\t1\t2\ta\tb\tnan\t0.9\n"
                                        "S1\tS1_0\tS3\tS3_1\tc\t1\t2\ta\tb\t3\t0.9\n")
        with pytest.raises(_abi.GridNativeError) as e:
            _abi.load_ibd(p, ids, 5, 0, 10, 0.5, 0.7, False, 1e6)
        assert e.value.code == _abi.GRID_EUNSUPPORTED
        assert hi._load_ibd_neighbors(p, idx, 5, 0, 10, 0.5, 0.7, False, 1e6) == \
            loaders.load_ibd(p, idx, 5, 0, 10, 0.5, 0.7, False, 1e6)
    elif case == "empty_ibs":
        p = write(tmp_path / "ibs.tsv", "")
        with pytest.raises(_abi.GridNativeError):
            _abi.load_ibs(p, ids, 5)
        with pytest.raises((StopIteration, RuntimeError)):
            hi._load_ibs_neighbors(p, idx, 5)
    else:
        p = write(tmp_path / "ibd.txt", "S1\tS1_0\tS2\tS2_1\tc\t100\t200\ta\tb\t3\t0.9\n")
        with pytest.raises(_abi.GridNativeError):
            _abi.load_ibd(p, ids, 5, 100, 200, 0.5, 0.7, True, 0)
        with pytest.raises(ZeroDivisionError):
            hi._load_ibd_neighbors(p, idx, 5, 100, 200, 0.5, 0.7, True, 0)


def test_golden_inputs(tmp_path):
    import os
    g = os.path.join(os.path.dirname(__file__), "golden", "g1")
    _, _, idx = loaders.read_dipcn(os.path.join(g, "expected", "dipcn.tsv"))
    ids = hi._ids_in_order(idx)
    ibs = os.path.join(g, "inputs", "ibs.tsv.gz")
    assert lists_of(_abi.load_ibs(ibs, ids, 10)) == canon(loaders.load_ibs(ibs, idx, 10))
    ibd = os.path.join(g, "inputs", "ibd.txt")
    for w in (False, True):
        assert lists_of(_abi.load_ibd(ibd, ids, 6, 1_500_000, 1_600_000, 0.5, 0.7, w, 1_000_000)) == \
            canon(loaders.load_ibd(ibd, idx, 6, 1_500_000, 1_600_000, 0.5, 0.7, w, 1_000_000))


@pytest.mark.parametrize("eol", ["\n", "\r\n", "\r"])
def test_multi_chunk_parse(tmp_path, monkeypatch, eol):
    """Files of several MiB are cut into line-aligned chunks parsed by threads;
    records merge back in file order (MAX_NBR cap, stable sort)."""
    monkeypatch.setenv("GRID_LOADER_THREADS", "5")
    rng = np.random.default_rng(7)
    ibs = write(tmp_path / "ibs.tsv", ibs_text(rng, 60000, eol))
    for max_nbr in (2, 40):
        assert lists_of(_abi.load_ibs(ibs, IDS, max_nbr)) == canon(loaders.load_ibs(ibs, IDX, max_nbr))
    ibd = write(tmp_path / "ibd.txt", ibd_text(rng, 40000, eol))
    for w in (False, True):
        assert lists_of(_abi.load_ibd(ibd, IDS, 9, 1_300_000, 1_500_000, 0.5, 0.7, w, 1e6)) == \
            canon(loaders.load_ibd(ibd, IDX, 9, 1_300_000, 1_500_000, 0.5, 0.7, w, 1e6))
