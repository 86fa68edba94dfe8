"""Kernel-level parity of the HIP path against the CPU oracle (MI355X only).

Bar: bit-exact for every fp64 statistic, index and integer; printed text
identical.  Sizes are small enough for the oracle to finish in seconds.
"""
import json
import math
import os

import numpy as np
import pytest

from grid_amd import _abi

from oracle import steps
from oracle.npsum import nanmean_rows

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    from grid_amd._abi import Device
    d = Device(0)
    yield d
    d.close()


def to_q(mat):
    from grid_amd._abi import MISSING
    q = np.where(np.isnan(mat), 0, np.rint(mat * 100)).astype(np.int64)
    assert np.array_equal(np.where(np.isnan(mat), 0, q / 100.0), np.where(np.isnan(mat), 0, mat))
    q = np.where(np.isnan(mat), MISSING, q).astype(np.int32)
    return np.ascontiguousarray(q)


def run_normalize(dev, mat, top_frac=0.1, f64=False):
    from grid_amd import engine
    q = np.ascontiguousarray(mat, dtype=np.float64) if f64 else to_q(mat)
    n, m = q.shape
    qd = dev.upload(q)
    st = (engine.normalize_stats_f64 if f64 else engine.normalize_stats)(dev, qd, n, m, m)
    sel, r = engine.select_regions(dev, st, top_frac)
    zq = dev.alloc((n, max(r, 1)), np.int32)
    if r:
        if f64:
            engine.zquant_f64(dev, qd, n, m, sel, r, st, zq)
        else:
            engine.zquant(dev, qd, n, m, sel, r, st, zq=zq)
    return st, sel.numpy()[:r], zq.numpy()[:, :r]


def check_normalize(dev, mat, top_frac=0.1, f64=False):
    from grid_amd import _abi
    st, sel, zq = run_normalize(dev, mat, top_frac, f64)
    with np.errstate(all="ignore"):
        z, ratios, mu, var, scale = steps.normalize_matrix(mat)
        raw = nanmean_rows(mat)
    assert np.array_equal(st.rowmean.numpy()[: len(raw)], raw, equal_nan=True)
    assert np.array_equal(st.mu.numpy()[: len(mu)], mu, equal_nan=True)
    assert np.array_equal(st.var.numpy()[: len(var)], var, equal_nan=True)
    r_ref = np.full(len(mu), np.nan)
    for k, v in ratios.items():
        r_ref[k] = v
    assert np.array_equal(st.ratio.numpy()[: len(mu)], r_ref, equal_nan=True)
    assert st.scale == scale
    exp_sel = steps.select_high_variance_regions(ratios, top_frac)
    assert sel.tolist() == exp_sel
    for i in range(mat.shape[0]):
        exp = "\t".join("NA" if np.isnan(z[i, j]) else f"{z[i, j]:.2f}" for j in exp_sel)
        assert _abi.format_hundredths(zq[i]) == exp, f"row {i}"


def test_normalize_golden_g2(dev):
    d = np.load(os.path.join(G, "g2.npz"))
    n_cases = len([k for k in d.files if k.endswith("_in")])
    for ci in range(n_cases):
        check_normalize(dev, d[f"c{ci}_in"])


@pytest.mark.parametrize("n,m,seed", [(37, 20000, 1), (5, 8192 * 3, 2), (130, 1000, 3), (2, 7, 4)])
def test_normalize_random(dev, n, m, seed):
    rng = np.random.default_rng(seed)
    q = rng.integers(1, 20000, size=(n, m))
    mat = q / 100.0
    mat[rng.random((n, m)) < 0.03] = np.nan
    check_normalize(dev, mat, top_frac=[0.1, 0.0, 0.5, 0.9][seed % 4])


def test_round_decimals_g5(dev):
    cases = json.load(open(os.path.join(G, "g5.json")))
    v = np.array([float.fromhex(c[0]) for c in cases])
    vd = dev.upload(v)
    for dec, col in ((2, 1), (3, 2)):
        out = dev.alloc(len(v), np.float64)
        from grid_amd._abi import call
        call("grid_round_decimals", dev.ctx, vd.ptr, len(v), dec, out.ptr)
        got = out.numpy()
        exp = np.array([float(c[col]) for c in cases])
        assert np.array_equal(got, exp), [(c, g) for c, g, e in zip(cases, got, exp) if g != e][:5]
        # sign of zero as printed
        assert [math.copysign(1, g) for g in got] == [math.copysign(1, e) for e in exp]


def test_knn_golden_g3(dev):
    from grid_amd import engine
    for case in json.load(open(os.path.join(G, "g3.json"))):
        q = np.array(case["q"], dtype=np.int64)
        k = case["k"]
        idx, d2, cnt = engine.knn_from_hundredths(dev, q, k, 200)
        exp = steps.knn_exact(q, k)
        for i in range(q.shape[0]):
            assert cnt[i] == len(exp[i])
            assert idx[i, : cnt[i]].tolist() == [j for j, _ in exp[i]]
            assert d2[i, : cnt[i]].tolist() == [s for _, s in exp[i]]


@pytest.mark.parametrize("n,r,k,qmax,seed", [(300, 5000, 10, 200, 1), (129, 64, 5, 256, 2),
                                             (700, 3000, 40, 200, 3), (1, 10, 3, 200, 4)])
def test_knn_random(dev, n, r, k, qmax, seed):
    from grid_amd import engine
    rng = np.random.default_rng(seed)
    q = rng.integers(-qmax, qmax + 1, size=(n, r))
    idx, d2, cnt = engine.knn_from_hundredths(dev, q, k, qmax)
    exp = steps.knn_exact(q, k)
    for i in range(n):
        assert idx[i, : cnt[i]].tolist() == [j for j, _ in exp[i]]
        assert d2[i, : cnt[i]].tolist() == [s for _, s in exp[i]]


def test_gram_exact_worst_case(dev):
    """bf16 MFMA + fp32 partials are exact at the integer bounds (all |q| = qmax):
    6-step fp32 chunks up to qmax 209 (k_gram8), 4-step chunks above (k_gram7)."""
    from grid_amd._abi import call
    for qmax in (200, 209, 210, 256):
        rng = np.random.default_rng(qmax)
        n, r = 256, 64 * 700
        q = np.where(rng.random((n, r)) < 0.5, -qmax, qmax).astype(np.int64)
        q[:3] = qmax                     # rows with maximal positive sums
        zf = (q.astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
        zb = dev.upload(zf)
        g = dev.zeros((n, n), np.int64)
        call("grid_knn_gram", dev.ctx, zb.ptr, n, r, r, qmax, g.ptr)
        got = g.numpy()
        ref = q @ q.T
        for ti in range(2):
            for tj in range(ti, 2):
                assert np.array_equal(got[ti*128:(ti+1)*128, tj*128:(tj+1)*128],
                                      ref[ti*128:(ti+1)*128, tj*128:(tj+1)*128])


@pytest.mark.parametrize("wide", ["0", "1"])
@pytest.mark.parametrize("qmax", [200, 256])
def test_gram_kblocked_multi_slice(dev, qmax, wide, monkeypatch):
    """grid_knn_gram_kb (k_gram8 on the K-blocked panel zquant_kb writes) on
    several int32 K-slices with a partial last 6-step group, both fp32 chunk
    lengths (qmax 200: 384 products, 256: 192), all-|qmax| worst-case rows;
    wide: the 16x16 layout's flush in 512-B row segments (GRID_GRAM_WIDE, live
    in the tools build)."""
    from grid_amd._abi import call
    monkeypatch.setenv("GRID_GRAM_WIDE", wide)
    n, np_ = 600, 768
    r = 64 * (2 * (((1 << 31) - 1) // (qmax * qmax * 64)) + 7)
    rng = np.random.default_rng(qmax)
    q = np.zeros((np_, r), dtype=np.int64)
    q[:n] = rng.integers(-qmax, qmax + 1, size=(n, r))
    q[:4] = np.where(rng.random((4, r)) < 0.5, -qmax, qmax)
    q[4] = qmax
    zf = (q.astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
    zkb = np.ascontiguousarray(zf.reshape(np_, r // _abi.KBW, _abi.KBW).transpose(1, 0, 2))
    zb = dev.upload(zkb)
    g = dev.zeros((np_, np_), np.int64)
    call("grid_knn_gram_kb", dev.ctx, zb.ptr, np_, r, qmax, g.ptr)
    got = g.numpy()
    qf = q.astype(np.float64)
    ref = (qf @ qf.T).astype(np.int64)
    for ti in range(np_ // 128):
        for tj in range(ti, np_ // 128):
            blk = (slice(ti * 128, (ti + 1) * 128), slice(tj * 128, (tj + 1) * 128))
            assert np.array_equal(got[blk], ref[blk]), (ti, tj)


@pytest.mark.parametrize("np_,knobs", [(768, {}), (640, {}), (768, {"GRID_GRAM_KX": "1"}),
                                       (768, {"GRID_GRAM_KX": "2", "GRID_GRAM_KC": "5"}),
                                       (768, {"GRID_GRAM_KX": "4", "GRID_GRAM_LAG": "3"}),
                                       (768, {"GRID_GRAM_KX": "8", "GRID_GRAM_SPIN": "0"})])
def test_gram_variants_multi_slice(dev, np_, knobs, monkeypatch):
    """The product Gram paths on a shape with several int32 K-slices, a
    partial last slice (remainder steps not a multiple of 4) and a partial
    256-row block, against a float64 product (exact: |sums| < 2^53): k_gram8
    (np % 256 == 0) under every K-split / chunk / pacing knob (performance
    knobs: results must not change), and k_gram_dma (np % 256 != 0)."""
    from grid_amd._abi import call
    for key, val in knobs.items():
        monkeypatch.setenv(key, val)
    qmax, n = 200, 600
    r = 64 * (2 * 838 + 7)
    rng = np.random.default_rng(np_ + len(knobs))
    q = np.zeros((np_, r), dtype=np.int64)
    q[:n] = rng.integers(-qmax, qmax + 1, size=(n, r))
    zf = (q.astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
    zb = dev.upload(zf)
    g = dev.zeros((np_, np_), np.int64)
    call("grid_knn_gram", dev.ctx, zb.ptr, np_, r, r, qmax, g.ptr)
    got = g.numpy()
    qf = q.astype(np.float64)
    ref = (qf @ qf.T).astype(np.int64)
    for ti in range(np_ // 128):
        for tj in range(ti, np_ // 128):
            blk = (slice(ti * 128, (ti + 1) * 128), slice(tj * 128, (tj + 1) * 128))
            assert np.array_equal(got[blk], ref[blk]), (ti, tj)
    call("grid_knn_mirror", dev.ctx, g.ptr, np_)
    assert np.array_equal(g.numpy(), ref)


def test_dipcn_random(dev):
    from grid_amd import engine
    rng = np.random.default_rng(7)
    n, k = 200, 12
    ids = [f"S{i:04d}" for i in range(n)]
    reads = {ids[i]: float(rng.integers(0, 5000)) for i in range(n) if i % 17}
    reads[ids[5]] = 0.0
    scale = np.round(rng.uniform(5, 60, n), 2)
    nbr = np.array([rng.choice(n, k, replace=False) for _ in range(n)], dtype=np.int32)
    nbrs = {ids[i]: [(ids[j], float(scale[j])) for j in nbr[i]] for i in range(n)}
    sc = {ids[i]: float(scale[i]) for i in range(n)}
    exp = dict(steps.dipcn(nbrs, sc, reads, 7))
    has = np.array([ids[i] in reads for i in range(n)])
    rd = np.array([reads.get(ids[i], 0.0) for i in range(n)])
    out, valid = engine.dipcn(dev, rd, has, scale, nbr, scale[nbr], np.full(n, k, np.int32), 7)
    assert {ids[i] for i in range(n) if valid[i]} == set(exp)
    for i in range(n):
        if valid[i]:
            assert out[i] == exp[ids[i]]


def test_phasing_golden_g4(dev):
    from grid_amd import engine
    for case in json.load(open(os.path.join(G, "g4.json"))):
        irr = np.array([float.fromhex(x) for x in case["irr"]])
        hn = [[(a, float.fromhex(b)) for a, b in l] for l in case["nbrs"]]
        off, nbr, w = engine.csr_from_lists(hn)
        hap, imp, mean = engine.phase(dev, irr, off, nbr, w, case["min_nbr"], case["iters"])
        assert [float(x).hex() for x in hap] == case["hap"]
        assert float(mean).hex() == case["mean"]
        assert [[float(imp[2*i]).hex(), float(imp[2*i+1]).hex()] for i in range(len(irr))] == case["imp"]


@pytest.mark.parametrize("n,seed", [(500, 1), (3000, 2), (9000, 3)])
def test_phasing_random(dev, n, seed):
    from grid_amd import engine
    rng = np.random.default_rng(seed)
    irr = rng.uniform(0.1, 4.0, n)
    hn = []
    for h in range(2 * n):
        c = (h // 2) % 26
        lst = []
        for _ in range(int(rng.integers(0, 11))):
            j = int(rng.integers(0, n // 26)) * 26 + c
            lst.append((min(2 * j + int(rng.integers(0, 2)), 2 * n - 1), 1.0))
        hn.append(lst)
    off, nbr, w = engine.csr_from_lists(hn)
    iters = 20
    hap, imp, mean = engine.phase(dev, irr, off, nbr, w, 1, iters)
    eh, em = steps.run_phasing(list(irr), hn, 1, iters)
    assert np.array_equal(hap, np.array(eh), equal_nan=True)
    assert mean == em
    ei = [steps.compute_imp(i, eh, hn, em) for i in range(n)]
    assert np.array_equal(imp, np.array(ei).reshape(-1))


@pytest.mark.parametrize("weighted,maxlen,legacy,paired,n", [
    (False, 6, False, False, 700), (True, 6, False, False, 700), (True, 14, False, False, 700),
    (False, 40, False, False, 700), (True, 40, False, False, 700), (True, 14, True, False, 700),
    (False, 6, False, True, 700), (True, 14, False, True, 700), (True, 40, False, True, 700),
    (False, 6, False, False, 6000), (True, 40, False, False, 6000), (True, 14, False, True, 6000)])
def test_phasing_kernel_variants(dev, weighted, maxlen, legacy, paired, n):
    """Register capacities 8/16, unit and general weights, lists longer than
    the packed capacity (CSR loop), the legacy kernel and the paired-lane
    register kernel (the default splits a sample's haplotypes over two
    lanes), vs the oracle.  n = 6000 does not fit LDS: the default runs the
    split kernel with hap in global memory, paired the global k_phase."""
    from grid_amd import engine
    rng = np.random.default_rng(maxlen * 2 + weighted + n)
    irr = rng.uniform(0.1, 4.0, n)
    irr[3] = np.nan
    hn = []
    for h in range(2 * n):
        c = (h // 2) % 13
        lst = []
        for _ in range(int(rng.integers(0, maxlen + 1))):
            j = int(rng.integers(0, n // 13)) * 13 + c
            wt = float(rng.uniform(0.05, 3.0)) if weighted else 1.0
            lst.append((min(2 * j + int(rng.integers(0, 2)), 2 * n - 1), wt))
        hn.append(lst)
    off, nbr, w = engine.csr_from_lists(hn)
    hap, imp, mean = engine.phase(dev, irr, off, nbr, w, 1, 15, legacy=legacy, paired=paired)
    eh, em = steps.run_phasing(list(irr), hn, 1, 15)
    assert np.array_equal(hap, np.array(eh), equal_nan=True)
    assert mean == em or (np.isnan(mean) and np.isnan(em))
    ei = [steps.compute_imp(i, eh, hn, em) for i in range(n)]
    assert np.array_equal(imp, np.array(ei).reshape(-1), equal_nan=True)


def _random_locus(rng, n, weighted, maxlen):
    irr = rng.uniform(0.1, 4.0, n)
    irr[rng.random(n) < 0.02] = 0.0
    hn = []
    for h in range(2 * n):
        lst = []
        for _ in range(int(rng.integers(0, maxlen + 1))):
            j = int(rng.integers(0, 2 * n))
            lst.append((j, float(rng.uniform(0.05, 3.0)) if weighted else 1.0))
        hn.append(lst)
    return list(irr), hn


@pytest.mark.parametrize("big,weighted,min_nbr,paired", [(False, False, 1, False), (False, True, 2, False),
                                                         (True, False, 1, False), (True, True, 0, False),
                                                         (False, True, 2, True)])
def test_phasing_batch_equals_per_locus_oracle(dev, big, weighted, min_nbr, paired):
    """grid_hi_phase_batch (one workgroup per locus, config 5) on loci of
    different sizes against the reference arithmetic run per locus; big=True
    puts a 5,000-sample locus in the batch, which moves every locus to the
    global-memory kernel (LDS too small)."""
    from grid_amd.utils.hi_inference import run_phasing_batch
    rng = np.random.default_rng(7 + big * 2 + weighted)
    sizes = [1, 37, 256, 300, 1201] + ([5000] if big else [])
    loci = [_random_locus(rng, n, weighted and i % 2 == 0, 12 if i != 2 else 20) for i, n in enumerate(sizes)]
    iters = 9
    got = run_phasing_batch([a for a, _ in loci], [b for _, b in loci], min_nbr, iters, dev=dev, paired=paired)
    for (irr, hn), (hap, imp, mean) in zip(loci, got):
        eh, em = steps.run_phasing(irr, hn, min_nbr, iters)
        assert np.array_equal(hap, np.array(eh), equal_nan=True)
        assert mean == em
        ei = [steps.compute_imp(i, eh, hn, em) for i in range(len(irr))]
        assert np.array_equal(imp, np.array(ei).reshape(-1), equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 7, 4096, 3_000_001])
def test_select_kth_equals_sorted(dev, n):
    """grid_select_kth / grid_count_valid (radix select) give grid_sort_valid's
    values: NaNs skipped, duplicates, negatives.  The sort keeps -0.0 and +0.0
    as equal keys in input order (as Python's sorted() does) while the select
    ranks -0.0 first, so a zero may differ in sign only; every use of these
    values (median > 0, ratio > thr, range tests) compares, so ranks are
    checked by value with the sign of zero ignored, and exactly otherwise."""
    import ctypes as C
    from grid_amd._abi import call
    rng = np.random.default_rng(n)
    v = rng.standard_normal(n) * 10.0 ** rng.integers(-3, 4, n)
    v[rng.random(n) < 0.1] = np.nan
    v[rng.random(n) < 0.05] = 0.0
    v[rng.random(n) < 0.05] = -0.0
    v[rng.random(n) < 0.05] = 3.25                  # duplicates
    d = dev.upload(v)
    out = dev.zeros(n, np.float64)
    nv = C.c_int64()
    call("grid_sort_valid", dev.ctx, d.ptr, n, out.ptr, C.byref(nv))
    nc = C.c_int64()
    call("grid_count_valid", dev.ctx, d.ptr, n, C.byref(nc))
    assert nc.value == nv.value == int((~np.isnan(v)).sum())
    if nv.value == 0:
        return
    srt = out.numpy()[: nv.value]
    ks = sorted({0, nv.value - 1, nv.value // 2, max(nv.value // 2 - 1, 0), int(0.9 * nv.value) % nv.value})
    for i in range(0, len(ks), 4):
        kk = ks[i:i + 4]
        karr = (C.c_int64 * len(kk))(*kk)
        vals = (C.c_double * len(kk))()
        call("grid_select_kth", dev.ctx, d.ptr, n, karr, len(kk), vals)
        for k, got in zip(kk, vals):
            if srt[k] == 0.0:
                assert got == 0.0, (k, got, srt[k])
            else:
                assert np.float64(got).view(np.uint64) == srt[k].view(np.uint64), (k, got, srt[k])


@pytest.mark.gpu
def test_normalize_f64_golden_g2(dev):
    """The fp64-depth route reproduces the golden normalize_matrix outputs."""
    d = np.load(os.path.join(G, "g2.npz"))
    n_cases = len([k for k in d.files if k.endswith("_in")])
    for ci in range(n_cases):
        check_normalize(dev, d[f"c{ci}_in"], f64=True)


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,seed", [(37, 20000, 11), (5, 8192 * 2 + 3, 12), (130, 1000, 13), (2, 7, 14)])
def test_normalize_f64_random(dev, n, m, seed):
    """Depths that are not hundredths (3+ decimals, as float() parses them), NaN
    holes, a zero row: every statistic and z code equal to the oracle's."""
    rng = np.random.default_rng(seed)
    mat = rng.uniform(5.0, 80.0, size=(n, m)).round(rng.integers(3, 7))
    mat[rng.random((n, m)) < 0.05] = np.nan
    if n > 3:
        mat[1] = 0.0
    check_normalize(dev, mat, f64=True)
