"""Every BASELINE configuration at its own shape on the GPU (MI355X only).

* configs 3 and 4 -- 50,000 samples x 3M / 30M bins, bin-streamed through
  HBM (the bench's chunk plan, the on-device cohort generator): the property
  checks of tests/bigcheck.py over every chunk, sampled rows/columns/blocks
  against the oracle, sampled k-NN queries against an fp64 product;
* config 5 -- 734 loci x 50,000 samples batched phasing: the batch launch
  equals per-locus launches bit for bit, and two loci equal the oracle's
  restatement of _run_phasing/_compute_imp (hi_inference.py:175-250) at a
  reduced n_iters;
* config 1 (100 x 30k, k=10) is the reference-generated golden cohort g_cfg1
  in tests/test_gpu_e2e.py.

The small case runs the same machinery at a size the box finishes in
seconds, so a failure there is cheap to read.
"""
import numpy as np
import pytest
import torch

from tests import bigcheck

pytestmark = pytest.mark.gpu


def test_streamed_property_checks_small():
    """bigcheck's machinery on a 600-sample cohort forced into 3 chunks."""
    res = bigcheck.run(600, 5 * 8192 + 517, k=6, n_rows=64, n_blocks=2, n_windows=2, budget_gb=0.09,
                       full_rows=3, n_iters=4)
    assert res["chunks"] >= 3


@pytest.mark.timeout(900)
def test_config3_50k_x_3M_streamed():
    res = bigcheck.run(50_000, 3_000_000, full_rows=2)
    assert res["chunks"] >= 7 and res["R"] > 2_500_000


@pytest.mark.timeout(1200)
def test_config4_50k_x_30M_streamed():
    res = bigcheck.run(50_000, 30_000_000, n_rows=64, fmt_all=False)
    assert res["chunks"] >= 60 and res["R"] > 25_000_000


def _locus(rng, n, per_hap=10):
    """tools/bench_loci.py's synthetic locus: IRRs ~ CN x U(0.9, 1.1), per_hap
    same-cluster haplotype neighbours per haplotype (26 clusters)."""
    clus = rng.integers(0, 26, n)
    irr = rng.choice([1.0, 1.5, 2.0, 2.5, 3.0], size=n) * rng.uniform(0.9, 1.1, n)
    order = np.argsort(clus, kind="stable")
    start = np.searchsorted(clus[order], np.arange(26))
    size = np.bincount(clus, minlength=26)
    hc = np.repeat(clus, 2)
    pick = (rng.random((2 * n, per_hap)) * size[hc][:, None]).astype(np.int64)
    js = order[start[hc][:, None] + pick]
    nbr = (2 * js + rng.integers(0, 2, js.shape)).astype(np.int32).reshape(-1)
    off = np.arange(0, 2 * n * per_hap + 1, per_hap, dtype=np.int64)
    return irr, off, nbr, np.ones(len(nbr))


@pytest.mark.timeout(900)
def test_config5_734_loci_x_50k():
    from grid_amd import _abi, engine
    from oracle import steps
    n, L = 50_000, 734
    rng = np.random.default_rng(734)
    loci = [_locus(rng, n) for _ in range(L)]
    dev = _abi.Device(0)
    dev.set_stream(torch.cuda.current_stream())
    bigcheck.log("config 5: batch of 734 loci x 50k, 100 iterations")
    res = engine.phase_batch(dev, loci, 1, 100)
    assert len(res) == L
    for li in sorted({0, L - 1, *range(17, L, 61)}):
        irr, off, nbr, w = loci[li]
        hap, imp, mean = engine.phase(dev, irr, off, nbr, w, 1, 100)
        assert np.array_equal(res[li][0], hap, equal_nan=True), f"locus {li}: hap"
        assert np.array_equal(res[li][1], imp, equal_nan=True), f"locus {li}: imp"
        assert res[li][2] == mean, f"locus {li}: mean"
    bigcheck.log("config 5: batch == per-locus launches")
    # the oracle on two 50k loci at a reduced n_iters (pure-Python sweeps)
    two = [loci[3], loci[L - 2]]
    got = engine.phase_batch(dev, two, 1, 3)
    for (irr, off, nbr, w), (hap, imp, mean) in zip(two, got):
        hn = [[(int(nbr[t]), 1.0) for t in range(off[h], off[h + 1])] for h in range(2 * n)]
        eh, em = steps.run_phasing(list(irr), hn, 1, 3)
        assert np.array_equal(hap, np.array(eh), equal_nan=True)
        assert mean == em
        ei = [steps.compute_imp(i, eh, hn, em) for i in range(n)]
        assert np.array_equal(imp, np.array(ei).reshape(-1), equal_nan=True)
    bigcheck.log("config 5: 2 loci == oracle (3 sweeps)")


@pytest.mark.timeout(600)
def test_config5_batch_loci_100_sweeps_vs_oracle():
    """the batched launch at the full n_iters = 100 against
    the oracle's _run_phasing/_compute_imp (hi_inference.py:175-250) on
    1000G-sized loci (3,202 samples: hap vectors in LDS) and a small one, in a
    batch that also holds a 50k-sample locus (hap vectors in global memory),
    which must equal its own single-locus launch."""
    from grid_amd import _abi, engine
    from oracle import steps
    rng = np.random.default_rng(3202)
    sizes = [3202, 50_000, 3202, 777]
    loci = [_locus(rng, n) for n in sizes]
    dev = _abi.Device(0)
    dev.set_stream(torch.cuda.current_stream())
    res = engine.phase_batch(dev, loci, 1, 100)
    hap, imp, mean = engine.phase(dev, *loci[1], 1, 100)
    assert np.array_equal(res[1][0], hap, equal_nan=True) and np.array_equal(res[1][1], imp, equal_nan=True)
    assert res[1][2] == mean
    for li in (0, 2, 3):
        irr, off, nbr, w = loci[li]
        n = len(irr)
        hn = [[(int(nbr[t]), 1.0) for t in range(off[h], off[h + 1])] for h in range(2 * n)]
        eh, em = steps.run_phasing(list(irr), hn, 1, 100)
        assert np.array_equal(res[li][0], np.array(eh), equal_nan=True), f"locus {li}: hap"
        assert res[li][2] == em
        ei = [steps.compute_imp(i, eh, hn, em) for i in range(n)]
        assert np.array_equal(res[li][1], np.array(ei).reshape(-1), equal_nan=True), f"locus {li}: imp"
