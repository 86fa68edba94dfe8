"""The device-resident region selection (grid_sel_stage1 / _stage2 / _read,
the fused chain's pass C) against the host-synchronising entry points it
replaces (grid_count_valid, grid_select_kth, grid_select_gt, gather + "%.3f",
grid_colmap_range) on edge cases: no valid ratio, odd and even counts,
thresholds at the ends, ties, -0.0, nothing selected, padding for the
all-gather."""
import math

import numpy as np
import pytest
import torch

from grid_amd import _abi
from grid_amd.engine import py_index
from grid_amd.fused import HipOps

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    d = _abi.Device(0)
    d.set_stream(torch.cuda.current_stream())
    return HipOps(d)


def host_path(o, ratio, ml, top_frac, frac_r, s2max):
    """fused.Steps47.run's pass C before round 3 (world 1)."""
    sel = torch.zeros(max(ml, 1), dtype=torch.int32, device="cuda")
    r3 = torch.full((max(ml, 1),), float("nan"), dtype=torch.float64, device="cuda")
    cm = torch.full((max(ml, 1),), -5, dtype=torch.int32, device="cuda")
    nvalid = o.count_valid(ratio, ml)
    scale, r_loc, vals = 1.0, 0, None
    if nvalid:
        ks = [nvalid // 2] if nvalid % 2 else [nvalid // 2 - 1, nvalid // 2]
        ks.append(py_index(nvalid, int(top_frac * nvalid)))
        vals = o.select_kth(ratio, ml, ks)
        med = vals[0] if nvalid % 2 else (vals[0] + vals[1]) / 2.0
        if med > 0:
            scale = 1.0 / math.sqrt(med / 100.0)
        r_loc = o.select_gt(ratio, ml, vals[-1], sel)
    o.gather(ratio, sel, r_loc, r3)
    o.round_decimals(r3, r_loc, 3, r3)
    nv = o.count_valid(r3, r_loc)
    if nv:
        smin = o.select_kth(r3, r_loc, [min(int(r_loc * (1.0 - frac_r)), nv - 1)])[0]
        smax = s2max
    else:
        smin, smax = -math.inf, math.inf
    ruse = o.colmap_range(r3, r_loc, smin, smax, cm)
    return dict(scale=scale, r_loc=r_loc, ruse=ruse, sel=sel[:r_loc].cpu(), r3=r3[:r_loc].cpu(),
                cm=cm[:r_loc].cpu(), smin=smin, smax=smax)


def device_path(o, ratio, ml, top_frac, frac_r, s2max, pad):
    sel = torch.zeros(max(ml, 1), dtype=torch.int32, device="cuda")
    r3 = torch.full((max(pad, 1),), 7.0, dtype=torch.float64, device="cuda")
    cm = torch.full((max(ml, 1),), -5, dtype=torch.int32, device="cuda")
    st = torch.zeros(_abi.SEL_STATE, dtype=torch.int64, device="cuda")
    o.sel_stage1(ratio, ml, ratio, ml, pad, top_frac, sel, r3, st)
    o.sel_stage2(r3, pad, r3, ml, frac_r, s2max, cm, st)
    h = o.sel_read(st)
    f = h.view(np.float64)
    nvalid, r_loc = int(h[_abi.SEL_NVALID]), int(h[_abi.SEL_RLOC])
    scale = 1.0
    if nvalid:
        med = f[_abi.SEL_V0] if nvalid % 2 else (f[_abi.SEL_V0] + f[_abi.SEL_V0 + 1]) / 2.0
        if med > 0:
            scale = 1.0 / math.sqrt(med / 100.0)
    return dict(scale=scale, r_loc=r_loc, ruse=int(h[_abi.SEL_RUSE]), sel=sel[:r_loc].cpu(), r3=r3[:r_loc].cpu(),
                cm=cm[:r_loc].cpu(), smin=float(f[_abi.SEL_SMIN]), smax=float(f[_abi.SEL_SMAX]),
                pad=r3[r_loc:pad].cpu(), cm_rest=cm[r_loc:ml].cpu(), err=int(h[_abi.SEL_ERR]))


def cases():
    rng = np.random.default_rng(11)
    v = rng.gamma(2.0, 3.0, 5000)
    yield "random", v, 0.1
    w = v.copy()
    w[rng.random(5000) < 0.3] = np.nan
    yield "nans_odd", w[:4999], 0.25
    yield "all_nan", np.full(300, np.nan), 0.1
    yield "ties", np.round(v, 1), 0.5
    z = v.copy()
    z[:50] = 0.0
    z[50:60] = -0.0
    z[60:70] = -1.5
    yield "zeros_neg", z, 0.0
    yield "top_end", v[:1001], 0.999
    yield "one", np.array([3.25]), 0.0
    yield "inf", np.concatenate([v[:100], [np.inf, -np.inf]]), 0.2
    # many compaction blocks (4096 values each) and many equal leading digits
    big = rng.gamma(2.0, 3.0, 200_003)
    big[rng.random(big.size) < 0.05] = np.nan
    big[::7] = 4.0
    yield "large", big, 0.1


@pytest.mark.parametrize("name,vals,top_frac", list(cases()), ids=[c[0] for c in cases()])
@pytest.mark.parametrize("frac_r,s2max", [(0.2, 50.0), (0.0, 1e9), (1.0, 5.0)])
def test_device_selection_equals_host_path(ops, name, vals, top_frac, frac_r, s2max):
    ml = len(vals)
    ratio = torch.from_numpy(np.ascontiguousarray(vals, np.float64)).cuda()
    exp = host_path(ops, ratio, ml, top_frac, frac_r, s2max)
    for pad in (ml, ml + 37):
        got = device_path(ops, ratio, ml, top_frac, frac_r, s2max, pad)
        assert got["err"] == 0
        for k in ("scale", "r_loc", "ruse"):
            assert got[k] == exp[k], k
        assert np.array_equal(np.array([got["smin"], got["smax"]]), np.array([exp["smin"], exp["smax"]]))
        assert torch.equal(got["sel"], exp["sel"])
        assert np.array_equal(got["r3"].numpy(), exp["r3"].numpy(), equal_nan=True)
        assert np.array_equal(np.signbit(got["r3"].numpy()), np.signbit(exp["r3"].numpy()))
        assert torch.equal(got["cm"], exp["cm"])
        assert torch.isnan(got["pad"]).all()
        assert (got["cm_rest"] == -1).all()


def test_device_selection_index_error(ops):
    """top_frac = 1.0 indexes past the end: the reference raises IndexError;
    the device path flags it for the caller."""
    ratio = torch.arange(1, 11, dtype=torch.float64, device="cuda")
    r = device_path(ops, ratio, 10, 1.0, 0.2, 50.0, 10)
    assert r["err"] == 1
