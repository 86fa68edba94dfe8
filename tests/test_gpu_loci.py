"""Multi-locus step 7 (BASELINE config 5) through the HIP batch kernel: every
locus' output file equals the reference's single-locus step restated by the
oracle (loaders, in-place Gauss-Seidel, imputation, formatting), for one rank
and for loci sharded over world 2 (gloo; ranks share the visible GPU)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.loci_cohort import expected_outputs, write_cohort

pytestmark = pytest.mark.gpu


def _check(cfg):
    exp = expected_outputs(cfg)
    assert len(exp) == 7
    for path, text in exp.items():
        assert open(path).read() == text, path


@pytest.mark.parametrize("method", ["ibs", "ibd"])
def test_loci_single_rank(tmp_path, method):
    from grid_amd.utils.hi_inference import hi_inference_loci
    cfg, _ = write_cohort(str(tmp_path))
    if method == "ibd":
        hc = cfg["compute_haploid_genotypes"]
        hc.update(method="ibd", ibd_output=str(tmp_path / "ibd.txt"), weighted=True, weight_scale=50_000)
    done = hi_inference_loci(cfg, None)
    assert len(done) == 7
    _check(cfg)


def test_loci_pipeline_route(tmp_path):
    """`grid wgs` reaches the multi-locus step when loci_file is set."""
    import yaml
    from grid_amd.pipeline import run_wgs_pipeline
    cfg, _ = write_cohort(str(tmp_path))
    cfg.update({"index": {"run": False}, "count_reads": {"run": False},
                "mosdepth": {"run": False, "normalize": {"run": False}, "neighbors": {"run": False}}})
    cfg["compute_diploid_genotypes"]["run"] = False
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    run_wgs_pipeline(console=None, config=str(p))
    _check(cfg)


def _worker(rank, world, port, cfg):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.pop("LOCAL_RANK", None)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from grid_amd.utils.hi_inference import hi_inference_loci
    done = hi_inference_loci(cfg, None)
    assert sorted(d["index"] for d in done) == [i for i in range(7) if i % world == rank]
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_loci_sharded_world2(tmp_path):
    cfg, _ = write_cohort(str(tmp_path))
    mp.start_processes(_worker, args=(2, _free_port(), cfg), nprocs=2, join=True, start_method="spawn")
    _check(cfg)


def test_phase_batch_groups_equal_one_group():
    """engine.phase_batch in groups of 3 loci (host prep of group g+1 beside
    group g's phasing, several launches) = one group, bit for bit, with unit
    and general weights and loci of different sizes."""
    import numpy as np
    from grid_amd import engine
    from grid_amd.device import get_device
    rng = np.random.default_rng(5)
    loci = []
    for k in range(8):
        n = int(rng.integers(20, 300))
        irr = rng.choice([1.0, 1.5, 2.0, 2.5, 3.0], size=n) * rng.uniform(0.9, 1.1, n)
        per = int(rng.integers(1, 12))
        nbr = rng.integers(0, 2 * n, 2 * n * per).astype(np.int32)
        off = np.arange(0, 2 * n * per + 1, per, dtype=np.int64)
        w = np.ones(len(nbr)) if k % 3 else rng.uniform(0.1, 2.0, len(nbr))
        loci.append((irr, off, nbr, w))
    dev = get_device()
    one = engine.phase_batch(dev, loci, 1, 20)
    grouped = engine.phase_batch(dev, loci, 1, 20, group=3)
    for (h1, i1, m1), (h2, i2, m2) in zip(one, grouped):
        assert np.array_equal(h1, h2, equal_nan=True) and np.array_equal(i1, i2, equal_nan=True) and m1 == m2
