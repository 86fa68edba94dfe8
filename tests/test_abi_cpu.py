"""CPU-side checks of the native library: it loads, exports every symbol of
include/grid_abi.h, and its host-only functions (formatting, GS level
schedule) are correct.  No GPU needed."""
import json
import os
import re

import numpy as np
import pytest

from oracle import steps

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "grid_abi.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(grid_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from grid_amd import _abi
    lib = _abi.load()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_abi.EXPORTS)


def test_format_hundredths_matches_python():
    from grid_amd import _abi
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.integers(-10 ** 7, 10 ** 7, 5000), np.arange(-250, 251)]).astype(np.int32)
    assert _abi.format_hundredths(v) == "\t".join(f"{x / 100:.2f}" for x in v.tolist())
    assert _abi.format_hundredths(np.array([_abi.ZQ_NAN, _abi.ZQ_NEG0], np.int32)) == "NA\t-0.00"
    assert _abi.format_hundredths(np.zeros(0, np.int32)) == ""


def _run_levels(irr, hn, min_nbr, iters):
    """Execute the level schedule in Python (read-all-then-write per level)."""
    import math
    from grid_amd import _abi, engine
    off, nbr, w = engine.csr_from_lists(hn)
    order, loff, nl = _abi.hi_levels(off, nbr)
    n = len(irr)
    assert sorted(order.tolist()) == list(range(n))
    hap = [float("nan")] * (2 * n)
    for i in range(n):
        if len(hn[2 * i]) >= min_nbr and len(hn[2 * i + 1]) >= min_nbr:
            hap[2 * i] = hap[2 * i + 1] = irr[i] / 2
    for _ in range(iters):
        for l in range(nl):
            upd = []
            for e in range(loff[l], loff[l + 1]):
                i = int(order[e])
                if math.isnan(hap[2 * i]):
                    continue
                ws, wv = [1e-9, 1e-9], [0.0, 0.0]
                for h in range(2):
                    for nb, wt in hn[2 * i + h]:
                        v = hap[nb]
                        if not math.isnan(v):
                            ws[h] += wt
                            wv[h] += wt * v
                m0, m1 = wv[0] / ws[0], wv[1] / ws[1]
                if m0 + m1 > 0:
                    upd.append((i, irr[i] * m0 / (m0 + m1), irr[i] * m1 / (m0 + m1)))
            for i, a, b in upd:
                hap[2 * i], hap[2 * i + 1] = a, b
    return hap


def test_level_schedule_reproduces_gauss_seidel():
    for case in json.load(open(os.path.join(G, "g4.json"))):
        irr = [float.fromhex(x) for x in case["irr"]]
        hn = [[(a, float.fromhex(b)) for a, b in l] for l in case["nbrs"]]
        hap = _run_levels(irr, hn, case["min_nbr"], case["iters"])
        assert [x.hex() for x in hap] == case["hap"]
    rng = np.random.default_rng(1)
    n = 300
    irr = list(rng.uniform(0.1, 3, n))
    hn = [[(int(rng.integers(0, 2 * n)), 1.0) for _ in range(int(rng.integers(0, 9)))] for _ in range(2 * n)]
    exp, _ = steps.run_phasing(irr, hn, 1, 9)
    got = _run_levels(irr, hn, 1, 9)
    assert np.array_equal(np.array(got), np.array(exp), equal_nan=True)


PROBE_SELECTORS = (b"GRID_GRAM_VARIANT", b"GRID_PHASE_PROBE", b"GRID_ZQUANT_VARIANT", b"GRID_COL_VW",
                   b"GRID_COL_CU", b"GRID_PHASE_LEGACY")


def test_product_library_has_no_probe_selectors():
    """The timing probes (wrong results by design) and A/B kernels are built
    only into libgridhip_probes.so (make probes, -DGRID_PROBES): the product
    library contains none of the environment variables that select them, so
    no environment can change its results.  The remaining getenv knobs are
    performance-only (tests/test_gpu_kernels.py checks results under them)."""
    from grid_amd import _abi
    blob = open(_abi.LIB_PATH, "rb").read()
    for s in PROBE_SELECTORS:
        assert s not in blob, s
    knobs = set(re.findall(rb"GRID_[A-Z0-9_]+", blob))
    allowed = {b"GRID_GRAM_LAG", b"GRID_GRAM_SPIN", b"GRID_GRAM_KC", b"GRID_GRAM_KX", b"GRID_ROWBLK_NT",
               b"GRID_COL_NT", b"GRID_ZQUANT_NT", b"GRID_ZQUANT_GROUPS", b"GRID_LOADER_THREADS"}
    env_like = {k for k in knobs if k not in (b"GRID_OK",)}
    # every GRID_* string in the binary is either an allowed knob or a message token, never a probe selector
    assert not (env_like & set(PROBE_SELECTORS))
    assert allowed & env_like                     # the knobs are present (sanity of the scan)
    # the getenv names themselves (NUL-terminated strings): exactly the tested,
    # result-neutral knobs (tests/test_gpu_streamed.py::test_performance_knobs_do_not_change_results,
    # GRID_NO_LIBDEFLATE: tests/test_ingest_cpu.py); every A/B selector reads
    # through GRID_AB_KNOB, which the product build compiles to "unset"
    names = set(re.findall(rb"\x00(GRID_[A-Z0-9_]+)\x00", blob))
    assert names <= allowed | {b"GRID_NO_LIBDEFLATE"}, sorted(names - allowed)


def test_library_provenance_matches_the_tree(monkeypatch):
    """The loaded library was compiled from the sources in this tree (the
    Makefile's sha256 of them is compiled in), and a library built from other
    sources is refused at load instead of running."""
    from grid_amd import _abi
    info = _abi.build_info()
    assert info["src_sha256"] == _abi.source_sha256()
    # the library names the files it hashed: the loader hashes those
    names = info["src_files"].split()
    assert info["src_sha256"] == _abi.source_sha256(names)
    assert sorted(n for n in names if not n.startswith("..")) == _abi._HASHED
    assert info["arch"] == "gfx950" and info["built_utc"]
    monkeypatch.setattr(_abi, "_lib", None)
    # a source the tree hashes that the library did not: refused
    monkeypatch.setattr(_abi, "_HASHED", sorted(_abi._HASHED + ["added_later.hip"]))
    with pytest.raises(_abi.GridNativeError, match="other source files"):
        _abi.load()
    monkeypatch.undo()
    monkeypatch.setattr(_abi, "_lib", None)
    monkeypatch.setattr(_abi, "source_sha256", lambda names=None: "0" * 64)
    with pytest.raises(_abi.GridNativeError, match="other sources"):
        _abi.load()
