"""Static checks of the shipped gfx950 ISA (CPU only; tools/isa_barriers.py
disassembles the code objects inside libgridhip.so).

* barrier frontier: at every EXEC-dependent branch of every kernel that has a
  workgroup barrier, both directions reach the same next barriers, so no wave
  can skip a barrier its neighbours wait at (the hang class the round-2 note
  on the half-split Gram asked to rule out);
* the exact Gram's K loops (k_gram8, every shipped instantiation): the
  steady-state loop runs a fixed number of barriers per trip (6 K-steps: one
  barrier per step for the quad-row ring, two for the half-split ring), and
  no innermost loop that streams the LDS-DMA ring holds a scratch (spill)
  access, whose vmcnt wait would drain the ring (the unit prologue outside
  the K loops does spill a few address registers)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_barriers  # noqa: E402

LIB = os.path.join(ROOT, "grid_amd", "_lib", "libgridhip.so")


@pytest.fixture(scope="module")
def report():
    if not os.path.exists(LIB):
        pytest.skip("libgridhip.so not built")
    funcs = {}
    for co in isa_barriers.code_objects(LIB):
        funcs.update(isa_barriers.parse_functions(isa_barriers.disassemble(co)))
    return isa_barriers.check(funcs, "")


def test_every_barrier_kernel_reconverges_before_its_barriers(report):
    assert len(report) >= 60
    bad = {k: v["errors"] for k, v in report.items() if v["errors"]}
    assert not bad, bad


def test_gram_k_loops_fixed_barriers_and_no_spills(report):
    """The steady-state K loop (every step's DMA lead exists: one vmcnt wait
    per barrier) of every shipped k_gram8: a fixed barrier count per trip
    and, for the fp32-chunk-of-384 kernels (FL = 1: qmax <= 209, the default
    zmax = 2.0), no scratch access at all and one vmcnt wait per barrier.
    The FL = 2 kernels (qmax in (209, 256]) reload up to 11 spilled dwords
    per 6-step trip; the last group and
    the tail of each unit (<= 8 K-steps) reload more -- both recorded here so
    a code-generation change shows up as a test failure."""
    grams = {k: v for k, v in report.items() if k.startswith("k_gram8<0,")}
    assert len(grams) == 9, sorted(grams)                  # LAY 4 (16x16x32 MFMAs) ships for FL = 1 only
    for name, v in grams.items():
        fl, lay = (int(x) for x in name.rstrip(">").split(",")[-2:])
        assert fl == 1 or lay != 4, name
        per_step = 2 if lay >= 2 else 1                      # half-split ring: two barriers per K-step
        mfma = 192 if lay == 4 else 96                       # 6 K-steps of 16x16x32 (4x4 per wave) or 32x32x16 (2x2)
        ring = [l for l in v["loops"] if l["lds_dma"] == 36 and l["mfma"] == mfma and l["innermost"]]
        assert ring and all(l["barriers_per_iter"] == [6 * per_step] * 2 for l in ring), (name, ring)
        steady = min(ring, key=lambda l: l["vmcnt"])       # the loop with no tail conditions
        if fl == 1:
            assert steady["scratch"] == 0 and steady["vmcnt"] == 6 * per_step, (name, steady)
        else:
            assert steady["scratch"] <= 11, (name, steady)


def test_round2_no_flush_probe_has_the_production_skeleton():
    """the no-flush Gram probe that hung in round 2, rebuilt
    (knn.hip -DGRID_ISA_PROBE, compile only) -- its MFMAs are dead code, but its
    barriers, vmcnt waits and LDS-DMA per steady K-loop trip equal production
    k_gram8<0, true, 1, 3>'s and no EXEC-divergent branch separates a barrier."""
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not present")
    assert isa_barriers.probe_compare() == 0
