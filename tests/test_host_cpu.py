"""Host-side logic of the drop-in (CPU only): file ingest vs the oracle,
pipeline gating and CLI, loaders, and the no-fallback rule."""
import gzip
import os
import shutil
from unittest.mock import patch

import numpy as np
import pytest
import yaml
from click.testing import CliRunner

from oracle import ingest as oingest
from oracle import loaders

G = os.path.join(os.path.dirname(__file__), "golden")


def _cfg(name, fname="config.yaml"):
    with open(os.path.join(G, name, fname)) as f:
        return yaml.safe_load(f)


@pytest.mark.parametrize("name", ["g1", "g1b", "g1c"])
def test_ingest_matches_oracle(name):
    from grid_amd import _abi
    from grid_amd.utils import normalize_mosdepth as nm
    c = _cfg(name)
    p = lambda r: os.path.join(G, name, r)  # noqa: E731
    ncfg = c["mosdepth"]["normalize"]
    samples = [s.strip() for s in open(p(c["samples_file"])) if s.strip()]
    inds = nm.map_mosdepth_files_to_samples(p(c["mosdepth"]["work_dir"]), samples)
    ex = nm.load_repeat_mask(p(ncfg["repeat_mask_file"]))
    ids, regions, q = nm.ingest(inds, p(c["mosdepth"]["work_dir"]), c.get("chrom"), c.get("start_bp"),
                                c.get("end_bp"), ex, ncfg["min_depth"], ncfg["max_depth"], 2)
    oids, oreg, omat = oingest.ingest(p(c["mosdepth"]["work_dir"]), samples, c.get("chrom"), c.get("start_bp"),
                                      c.get("end_bp"), p(ncfg["repeat_mask_file"]), ncfg["min_depth"],
                                      ncfg["max_depth"])
    assert ids == oids and regions == oreg
    back = np.where(q == _abi.MISSING, np.nan, q / 100.0)
    assert np.array_equal(back, omat, equal_nan=True)


def test_mask_and_chrom_helpers(tmp_path):
    from grid_amd.utils import normalize_mosdepth as nm
    assert nm.norm_chrom("6") == "chr6" and nm.norm_chrom("chrX") == "chrX"
    b = tmp_path / "m.bed"
    b.write_text("# c\n\n6\t1000\t3000\nchr1\t0\nchr2\tx\t5\n")
    ex = nm.load_repeat_mask(str(b))
    assert ex == {"chr6": {1, 2, 3}}
    assert nm.select_high_variance_regions({0: 1.0, 1: 5.0, 2: 10.0, 3: 2.0}, 0.5) == [2]
    assert nm.select_high_variance_regions({}, 0.5) == []
    with pytest.raises(IndexError):
        nm.select_high_variance_regions({0: 1.0}, 1.0)


def test_to_hundredths_rejects_non_two_decimal():
    from grid_amd.utils import normalize_mosdepth as nm
    assert nm.to_hundredths(np.array([[1.25, np.nan]]))[0, 0] == 125
    with pytest.raises(nm.UnsupportedDepth):
        nm.to_hundredths(np.array([[1.255]]))


def test_loaders_match_oracle():
    from grid_amd.utils import compute_dipcn as cd
    from grid_amd.utils import hi_inference as hi
    nb = os.path.join(G, "g1", "expected", "neighbors.zMax2.0.tsv.gz")
    assert cd.load_neighbors(nb) == loaders.load_neighbors(nb)
    assert cd._read_counts(os.path.join(G, "g1", "expected", "counts.tsv")) == \
        loaders.read_counts(os.path.join(G, "g1", "expected", "counts.tsv"))
    dip = os.path.join(G, "g1", "expected", "dipcn.tsv")
    ids, irr, idx = hi._read_dip_cn_file(dip)
    assert (ids, irr, idx) == loaders.read_dipcn(dip)
    assert hi._load_ibs_neighbors(os.path.join(G, "g1", "inputs", "ibs.tsv.gz"), idx, 10) == \
        loaders.load_ibs(os.path.join(G, "g1", "inputs", "ibs.tsv.gz"), idx, 10)
    for w in (False, True):
        a = hi._load_ibd_neighbors(os.path.join(G, "g1", "inputs", "ibd.txt"), idx, 6, 1_500_000, 1_600_000,
                                   0.5, 0.7, w, 1_000_000)
        b = loaders.load_ibd(os.path.join(G, "g1", "inputs", "ibd.txt"), idx, 6, 1_500_000, 1_600_000,
                             0.5, 0.7, w, 1_000_000)
        assert a == b


def test_hundredths_token_parser():
    from grid_amd.utils.find_neighbors import _hundredths
    from grid_amd import _abi
    for s in ["0.00", "-0.00", "1.25", "-12.50", "123456.78", "-0.01"]:
        assert _hundredths(s) == round(float(s) * 100)
    assert _hundredths("NA") == _abi.MISSING


def test_no_cpu_fallback():
    """Without a GPU the compute path must fail loudly, never fall back."""
    from grid_amd import _abi
    from grid_amd.utils import normalize_mosdepth as nm
    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU present")
    with pytest.raises(_abi.GridNativeError):
        nm.normalize_matrix(np.array([[1.0, 2.0], [3.0, 4.0]]))


# ---------------------------------------------------------------- pipeline --
def write_config(tmp_path, extra=None):
    cfg = {"index": {"run": False}, "count_reads": {"run": False},
           "mosdepth": {"run": False, "normalize": {"run": False}, "neighbors": {"run": False}},
           "compute_diploid_genotypes": {"run": False}, "compute_haploid_genotypes": {"run": False}}
    if extra:
        cfg.update(extra)
    p = tmp_path / "config.yaml"
    p.write_text(yaml.dump(cfg))
    return str(p)


def test_pipeline_requires_config():
    from grid_amd.pipeline import run_wgs_pipeline
    with pytest.raises(Exception):
        run_wgs_pipeline(console=None, config=None)


def test_pipeline_all_disabled(tmp_path):
    from grid_amd.pipeline import run_wgs_pipeline
    run_wgs_pipeline(console=None, config=write_config(tmp_path))


@pytest.mark.parametrize("section,target", [
    ({"mosdepth": {"run": False, "normalize": {"run": True}, "neighbors": {"run": False}}},
     "grid_amd.utils.normalize_mosdepth.normalize_mosdepth"),
    ({"mosdepth": {"run": False, "normalize": {"run": False}, "neighbors": {"run": True}}},
     "grid_amd.utils.find_neighbors.find_neighbors"),
    ({"compute_diploid_genotypes": {"run": True}}, "grid_amd.utils.compute_dipcn.compute_diploid_genotypes"),
    ({"compute_haploid_genotypes": {"run": True}}, "grid_amd.utils.hi_inference.hi_inference"),
])
def test_pipeline_gates(tmp_path, section, target):
    from grid_amd.pipeline import run_wgs_pipeline
    with patch(target) as m:
        run_wgs_pipeline(console=None, config=write_config(tmp_path, section))
        m.assert_called_once()


def test_pipeline_step_exception_is_logged(tmp_path, capsys):
    from grid_amd.pipeline import run_wgs_pipeline
    cfg = write_config(tmp_path, {"compute_haploid_genotypes": {"run": True}})
    with patch("grid_amd.utils.hi_inference.hi_inference", side_effect=RuntimeError("boom")):
        run_wgs_pipeline(console=None, config=cfg)
    assert "boom" in capsys.readouterr().out


def test_pipeline_missing_section_is_keyerror(tmp_path):
    from grid_amd.pipeline import run_wgs_pipeline
    p = tmp_path / "c.yaml"
    p.write_text(yaml.dump({"index": {"run": False}}))
    with pytest.raises(KeyError):
        run_wgs_pipeline(console=None, config=str(p))


def test_cli(tmp_path):
    from grid_amd.cli import cli
    r = CliRunner()
    res = r.invoke(cli, ["--help"])
    assert res.exit_code == 0 and "GRiD" in res.output
    assert r.invoke(cli, ["wgs", "--help"]).exit_code == 0
    assert r.invoke(cli, ["wgs", "/nonexistent.yaml"]).exit_code != 0
    with patch("grid_amd.pipeline.run_wgs_pipeline") as m:
        res = r.invoke(cli, ["wgs", write_config(tmp_path)])
    assert res.exit_code == 0, res.output
    m.assert_called_once()


def test_handoff_only_for_the_unchanged_file(tmp_path):
    """grid_amd/utils/handoff.py: an entry is taken once, and only while the
    file is byte-for-byte the one published (size and mtime)."""
    import os
    from grid_amd.utils import handoff
    p = tmp_path / "normalized.tsv.gz"
    p.write_bytes(b"x" * 10)
    handoff.publish(p, ["A"], [1.0], [2.0], "dev", (1, 1))
    got = handoff.take(str(p))
    assert got is not None and got[0] == ["A"] and got[3] == "dev"
    assert handoff.take(p) is None                          # consumed
    handoff.publish(p, ["A"], [1.0], [2.0], "dev", (1, 1))
    p.write_bytes(b"y" * 11)                                 # replaced
    assert handoff.take(p) is None
    handoff.publish(p, ["A"], [1.0], [2.0], "dev", (1, 1))
    st = os.stat(p)
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns + 10**9))
    assert handoff.take(p) is None
    handoff.publish(p, ["A"], [1.0], [2.0], "dev", (1, 1))
    handoff.clear()
    assert handoff.take(p) is None
