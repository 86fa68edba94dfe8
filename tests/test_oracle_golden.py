"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import gzip
import json
import os

import numpy as np
import pandas as pd
import pytest
import yaml

from oracle import ingest, loaders, steps
from oracle.npsum import nanmean_rows

G = os.path.join(os.path.dirname(__file__), "golden")


def _gz_lines(p):
    with gzip.open(p, "rt") as f:
        return f.readlines()


def _cfg(name, fname="config.yaml"):
    with open(os.path.join(G, name, fname)) as f:
        return yaml.safe_load(f)


def _p(name, rel):
    return os.path.join(G, name, rel)


@pytest.mark.parametrize("name", ["g1", "g1b", "g1c"])
def test_oracle_pipeline_matches_reference_files(name):
    c = _cfg(name)
    nc = c["mosdepth"]["normalize"]
    samples = [l.strip() for l in open(_p(name, c["samples_file"])) if l.strip()]
    ids, regions, mat = ingest.ingest(_p(name, c["mosdepth"]["work_dir"]), samples, c.get("chrom"),
                                      c.get("start_bp"), c.get("end_bp"),
                                      _p(name, nc["repeat_mask_file"]), nc["min_depth"], nc["max_depth"])
    raw = nanmean_rows(mat)
    z, ratios, mu, var, _ = steps.normalize_matrix(mat)
    sel = steps.select_high_variance_regions(ratios, nc["top_frac"])
    lines = steps.normalized_lines(z, ids, sel, mu, var, raw)
    exp = _gz_lines(_p(name, "expected/normalized.tsv.gz"))
    assert lines == exp

    # step 5 from the expected normalised file
    nb = c["mosdepth"]["neighbors"]
    ids5, r5, z5, sc5 = steps.parse_normalized(exp)
    zmax = nb["zmax"]
    zc = np.nan_to_num(np.clip(z5, -zmax, zmax), nan=0.0)
    idx, ruse = steps.filter_regions_by_variance(r5, 1.0, nb["sigma2_max"])
    q = np.rint(zc[:, idx] * 100).astype(np.int64)
    assert np.array_equal(q / 100.0, zc[:, idx])
    nbrs = steps.knn_exact(q, nb["num_neighbors"])
    lines5 = steps.neighbor_lines(ids5, sc5, nbrs, ruse)
    assert lines5 == _gz_lines(_p(name, "expected/neighbors.zMax2.0.tsv.gz"))

    # step 6
    nbd, scd = loaders.load_neighbors(_p(name, "expected/neighbors.zMax2.0.tsv.gz"))
    reads = loaders.read_counts(_p(name, "expected/counts.tsv"))
    dip = steps.dipcn(nbd, scd, reads, c["compute_diploid_genotypes"]["n_nbr"])
    df = pd.DataFrame(dip, columns=["Sample", "Norm_Reads"])
    assert df.to_csv(sep="\t", index=False) == open(_p(name, "expected/dipcn.tsv")).read()

    # step 7, IBS and IBD-weighted
    for cfgname, outname in (("config.yaml", "haploid.tsv"), ("config_ibd.yaml", "haploid_ibd.tsv")):
        cc = _cfg(name, cfgname)
        hc = cc["compute_haploid_genotypes"]
        hid, irr, hidx = loaders.read_dipcn(_p(name, "expected/dipcn.tsv"))
        if hc["method"] == "ibs":
            hn = loaders.load_ibs(_p(name, hc["ibs_output"]), hidx, hc["max_neighbors"])
        else:
            hn = loaders.load_ibd(_p(name, hc["ibd_output"]), hidx, hc["max_neighbors"], cc.get("start_bp"),
                                  cc.get("end_bp"), hc["min_length"], hc["min_match"], hc["weighted"],
                                  hc["weight_scale"])
        hap, mean = steps.run_phasing(irr, hn, hc["min_neighbors"], hc["n_iters"])
        imp = [steps.compute_imp(i, hap, hn, mean) for i in range(len(irr))]
        assert "".join(steps.haploid_lines(hid, irr, hap, imp)) == open(_p(name, "expected/" + outname)).read()


def test_oracle_normalize_matrix_bitexact():
    d = np.load(os.path.join(G, "g2.npz"))
    n_cases = len([k for k in d.files if k.endswith("_in")])
    for ci in range(n_cases):
        mat = d[f"c{ci}_in"]
        with np.errstate(all="ignore"):
            z, ratios, mu, var, _ = steps.normalize_matrix(mat)
            raw = nanmean_rows(mat)
        assert np.array_equal(raw, d[f"c{ci}_raw"], equal_nan=True)
        assert np.array_equal(z.view(np.int64), d[f"c{ci}_z"].view(np.int64)) or \
            np.array_equal(z, d[f"c{ci}_z"], equal_nan=True)
        assert np.array_equal(mu, d[f"c{ci}_mu"], equal_nan=True)
        assert np.array_equal(var, d[f"c{ci}_var"], equal_nan=True)
        keys = sorted(ratios)
        assert keys == d[f"c{ci}_rkeys"].tolist()
        assert np.array_equal(np.array([ratios[k] for k in keys]), d[f"c{ci}_rvals"])
        for tf in (0.0, 0.1, 0.5, 0.9):
            assert steps.select_high_variance_regions(ratios, tf) == d[f"c{ci}_sel_{tf}"].tolist()


def test_oracle_knn_matches_sklearn_vectors():
    for case in json.load(open(os.path.join(G, "g3.json"))):
        q = np.array(case["q"], dtype=np.int64)
        ids = [f"X{i:03d}" for i in range(q.shape[0])]
        got = steps.knn_exact(q, case["k"])
        for i, sid in enumerate(ids):
            exp = case["res"][sid]
            assert [ids[j] for j, _ in got[i]] == [e[0] for e in exp]
            for (j, s), (_, dh) in zip(got[i], exp):
                # sklearn's fp64 distance agrees with the exact one to rounding
                assert abs(s / 1e4 - float.fromhex(dh)) <= 1e-9 * max(1.0, s / 1e4)


def test_oracle_phasing_bitexact():
    for case in json.load(open(os.path.join(G, "g4.json"))):
        irr = [float.fromhex(x) for x in case["irr"]]
        hn = [[(a, float.fromhex(b)) for a, b in l] for l in case["nbrs"]]
        hap, mean = steps.run_phasing(irr, hn, case["min_nbr"], case["iters"])
        assert [x.hex() for x in hap] == case["hap"]
        assert mean.hex() == case["mean"]
        imp = [steps.compute_imp(i, hap, hn, mean) for i in range(len(irr))]
        assert [[a.hex(), b.hex()] for a, b in imp] == case["imp"]
