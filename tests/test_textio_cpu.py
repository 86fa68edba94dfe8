"""Normalised-matrix text I/O in host C++ (grid_write_normalized_gz /
grid_read_normalized_gz): the threaded multi-member gzip decompresses to
exactly the reference's text (normalize_mosdepth.py:535-554, restated in
oracle.steps.normalized_lines), and the reader returns what the reference's
parser (find_neighbors.py:99-124, oracle.steps.parse_normalized) does."""
import gzip

import numpy as np
import pytest

from grid_amd import _abi
from oracle import steps

ZQ_NAN, ZQ_NEG0 = -(2 ** 31), -(2 ** 31) + 1


def cohort(n, r, seed):
    rng = np.random.default_rng(seed)
    zq = rng.integers(-60000, 60000, (n, r)).astype(np.int32)
    zq[rng.random((n, r)) < 0.02] = ZQ_NAN
    zq[rng.random((n, r)) < 0.01] = ZQ_NEG0
    if n and r >= 4:
        zq[0, :4] = [5, -5, 100, 0]
    raw = rng.uniform(0, 80, n)
    raw[: min(n, 4)] = [np.nan, 0.125, 2.675, -0.0][: min(n, 4)]
    means = rng.uniform(0.5, 2.0, r)
    vars_ = rng.uniform(0.0, 0.3, r)
    means[: min(r, 4)] = [np.nan, -0.0001, 0.0005, 123456.7895][: min(r, 4)]
    ids = [f"S{i:05d}" for i in range(n)]
    return ids, raw, means, vars_, zq


def expected_lines(ids, raw, means, vars_, zq):
    z = np.where(zq == ZQ_NAN, np.nan, zq / 100.0)
    z[zq == ZQ_NEG0] = -0.0
    return steps.normalized_lines(z, ids, list(range(zq.shape[1])), means, vars_, raw)


def ratios_of(means, vars_):
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(means > 0, 100.0 * vars_ / means, np.nan)


@pytest.mark.parametrize("n,r,threads", [(37, 513, 4), (12, 300_000, 3), (0, 5, 2), (3, 0, 2)])
def test_writer_text_equals_reference(tmp_path, n, r, threads):
    ids, raw, means, vars_, zq = cohort(n, r, n + r)
    path = tmp_path / "norm.tsv.gz"
    _abi.write_normalized_gz(path, ids, raw, means, ratios_of(means, vars_), zq, level=1, threads=threads)
    with gzip.open(path, "rt") as f:
        got = f.read()
    assert got == "".join(expected_lines(ids, raw, means, vars_, zq))


@pytest.mark.parametrize("single_member", [False, True])
def test_reader_equals_reference_parser(tmp_path, single_member):
    ids, raw, means, vars_, zq = cohort(41, 2049, 3)
    path = tmp_path / "norm.tsv.gz"
    lines = expected_lines(ids, raw, means, vars_, zq)
    if single_member:                       # as the reference writes it (one gzip stream)
        with gzip.open(path, "wt") as f:
            f.write("".join(lines))
    else:
        _abi.write_normalized_gz(path, ids, raw, means, ratios_of(means, vars_), zq, threads=4)
    rid, rsc, rmu, rrat, rzq = _abi.read_normalized_gz(path, threads=3)
    eid, erat, edata, esc = steps.parse_normalized(lines)
    assert rid == eid
    assert np.array_equal(rsc, np.array([esc[i] for i in eid]), equal_nan=True)
    assert np.array_equal(rrat, erat, equal_nan=True)
    assert np.array_equal(np.where(rzq == _abi.MISSING, np.nan, rzq / 100.0), edata, equal_nan=True)


def test_reader_rejects_other_grammar_and_step_falls_back(tmp_path):
    from grid_amd.utils import find_neighbors
    ids, raw, means, vars_, zq = cohort(5, 7, 9)
    lines = expected_lines(ids, raw, means, vars_, zq)
    parts = lines[3].rstrip("\n").split("\t")
    parts[4] = "1.250"                      # three decimals: a valid float, not "%.2f" text
    lines[3] = "\t".join(parts) + "\n"
    path = tmp_path / "odd.tsv.gz"
    with gzip.open(path, "wt") as f:
        f.write("".join(lines))
    with pytest.raises(_abi.GridNativeError) as ei:
        _abi.read_normalized_gz(path)
    assert ei.value.code == _abi.GRID_EUNSUPPORTED
    got_ids, got_sc, got_zq, got_rat = find_neighbors._read_normalized_q(path)
    eid, erat, edata, esc = steps.parse_normalized(lines)
    assert got_ids == eid and list(got_sc) == list(esc)
    assert np.array_equal([got_sc[i] for i in eid], [esc[i] for i in eid], equal_nan=True)
    assert np.array_equal(np.where(got_zq == _abi.MISSING, np.nan, got_zq / 100.0), edata, equal_nan=True)
