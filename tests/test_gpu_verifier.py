"""The 50k-scale step-4 verifier (grid_verify_zquant, used by tests/bigcheck.py
on every cell of configs 3-4) pinned by reference fixtures (VERDICT r3 item
7): fed the reference's own printed z values as int16 codes it must report
zero mismatches, and exactly one after one code is changed.

  * g2 (tests/golden/make_golden.py: the reference's normalize_matrix on
    matrices of widths 8191/8192/8193/16385 with NaN holes, a zero row, all-NaN
    and zero columns): the codes are "%.2f" of the reference's z;
  * g_cfg1 (BASELINE config 1, 100 x 30k from mosdepth files): the codes are
    the rows of step 4's normalised text, whose sha256 equals the reference
    run's (tests/golden/g_cfg1/cohort.json), with the q, row means, column
    means and scale step 4 computed."""
import gzip
import hashlib
import os

import numpy as np
import pytest

from oracle import steps

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
NAN16, NEG0, ESC, LO, HI = -32768, -32767, -32766, -32765, 32767


@pytest.fixture(scope="module")
def dev():
    from grid_amd._abi import Device
    d = Device(0)
    yield d
    d.close()


def _code(t: str) -> int:
    """int16 step-4 code of one printed z ("%.2f" text or "NA")."""
    if t == "NA":
        return NAN16
    if t == "-0.00":
        return NEG0
    v = int(t.replace(".", ""))
    return v if LO <= v <= HI else ESC


def _verify(dev, q, sel, rm, mu, scale, codes):
    import ctypes as C

    from grid_amd import _abi
    n, ld = q.shape
    r = len(sel)
    dq, dsel = dev.upload(np.ascontiguousarray(q, np.int32)), dev.upload(np.asarray(sel, np.int32))
    drm, dmu = dev.upload(np.asarray(rm, np.float64)), dev.upload(np.asarray(mu, np.float64))
    dz = dev.upload(np.ascontiguousarray(codes, np.int16))
    cnt = (C.c_int64 * 3)()
    _abi.call("grid_verify_zquant", dev.ctx, dq.ptr, n, ld, dsel.ptr, r, drm.ptr, dmu.ptr, float(scale), dz.ptr, r,
              None, 0, None, 0, cnt)
    return list(cnt)


def _checked(dev, q, sel, rm, mu, scale, codes, skipped):
    got = _verify(dev, q, sel, rm, mu, scale, codes)
    assert got[0] == 0 and got[2] == skipped, got
    # one changed code: exactly one mismatch (the verifier is not blind)
    live = np.argwhere((codes != NAN16) & (codes != ESC))
    if len(live):
        i, s = live[len(live) // 2]
        bad = codes.copy()
        bad[i, s] = bad[i, s] + 1 if bad[i, s] < HI else bad[i, s] - 1
        assert _verify(dev, q, sel, rm, mu, scale, bad)[0] == 1


def test_verifier_on_g2_reference_z(dev):
    from tests.test_gpu_kernels import to_q
    d = np.load(os.path.join(G, "g2.npz"))
    for ci in range(len([k for k in d.files if k.endswith("_in")])):
        mat = d[f"c{ci}_in"]
        z, _, mu, _, scale = steps.normalize_matrix(mat)
        assert np.array_equal(z, d[f"c{ci}_z"], equal_nan=True)          # the oracle's scale is the reference's
        sel = d[f"c{ci}_sel_0.1"]
        if not len(sel):
            continue
        q, rm, mu = to_q(mat), d[f"c{ci}_raw"], d[f"c{ci}_mu"]
        zr = d[f"c{ci}_z"][:, sel]
        codes = np.array([[_code("NA" if np.isnan(v) else f"{v:.2f}") for v in row] for row in zr], np.int16)
        # the verifier skips missing cells and rows / columns whose z is not the transformed one
        skipped = int(np.sum((np.isnan(mat[:, sel])) | ~((rm != 0) & ~np.isnan(rm))[:, None] | ~(mu[sel] > 0)[None, :]))
        _checked(dev, q, sel, rm, mu, scale, codes, skipped)


def test_verifier_on_config1_reference_text(dev, tmp_path, monkeypatch):
    from grid_amd import engine
    from grid_amd.utils.normalize_mosdepth import normalize_mosdepth
    from tests.golden import cohort_files
    cfg, _, meta = cohort_files.regenerate("g_cfg1", tmp_path)
    seen = {}
    orig = engine.zquant

    def capture(dev_, qd, n, m, sel, r, st, **kw):
        seen.update(q=qd.numpy()[:n, :m].copy(), sel=sel.numpy()[:r].copy(), rm=st.rowmean.numpy()[:n].copy(),
                    mu=st.mu.numpy()[:m].copy(), scale=st.scale)
        return orig(dev_, qd, n, m, sel, r, st, **kw)
    monkeypatch.setattr(engine, "zquant", capture)
    normalize_mosdepth(cfg, None)
    text = gzip.decompress((tmp_path / "out" / "normalized.tsv.gz").read_bytes())
    assert hashlib.sha256(text).hexdigest() == meta["normalized_sha256"], "step 4's text is not the reference's"
    rows = text.decode().split("\n")[2:]
    rows = [r.split("\t")[2:] for r in rows if r]
    codes = np.array([[_code(t) for t in r] for r in rows], np.int16)
    q, sel, rm, mu = seen["q"], seen["sel"], seen["rm"], seen["mu"]
    assert codes.shape == (q.shape[0], len(sel))
    from grid_amd._abi import MISSING
    skipped = int(np.sum((q[:, sel] == MISSING) | ~((rm != 0) & ~np.isnan(rm))[:, None] | ~(mu[sel] > 0)[None, :]))
    _checked(dev, q, sel, rm, mu, seen["scale"], codes, skipped)

