"""The distributed drop-in on the GPU's kernels: `grid wgs` (run_wgs_pipeline)
under torch.distributed with 2 and 4 ranks SHARING the box's one GPU (gloo
carries the collectives through host memory; RCCL refuses two ranks on one
GPU -- the driver's 8-GPU run takes RCCL).  Steps 4-5 run over every rank
(grid_amd/utils/dist_step4.py: the device ingest of each rank's file slice,
the population-sum chain, the all-to-all to column shards, fused.Steps47 on
HipOps, the z all-to-all and the device member coder placing each rank's
rows at its offset); steps 6-7 on rank 0.  Every output file must equal the
reference's (golden cohorts; BASELINE config 1 by its sha256)."""
import gzip
import os
import shutil
import socket

import pytest
import yaml

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
FILES = ("normalized.tsv.gz", "neighbors.zMax2.0.tsv.gz", "dipcn.tsv", "haploid.tsv")


def _content(p):
    if str(p).endswith(".gz"):
        with gzip.open(p, "rt") as f:
            return f.read()
    return open(p).read()


def _stage(name, tmp_path):
    src = os.path.join(G, name)
    shutil.copytree(os.path.join(src, "inputs"), tmp_path / "inputs")
    c = yaml.safe_load(open(os.path.join(src, "config.yaml")))
    c["samples_file"] = str(tmp_path / c["samples_file"])
    c["output_dir"] = str(tmp_path / "out")
    c["mosdepth"]["work_dir"] = str(tmp_path / c["mosdepth"]["work_dir"])
    c["mosdepth"]["normalize"]["repeat_mask_file"] = str(tmp_path / c["mosdepth"]["normalize"]["repeat_mask_file"])
    hc = c["compute_haploid_genotypes"]
    for k in ("ibs_output", "ibd_output"):
        if k in hc:
            hc[k] = str(tmp_path / hc[k])
    os.makedirs(c["output_dir"], exist_ok=True)
    shutil.copy(os.path.join(src, "expected", "counts.tsv"), os.path.join(c["output_dir"], "counts.tsv"))
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(c))
    return c, str(p)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, log):
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), GRID_DIST_BACKEND="gloo", GRID_SHARE_GPU="1")
    sys.stdout = open(f"{log}.{rank}", "w")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from grid_amd.pipeline import run_wgs_pipeline
    run_wgs_pipeline(console=None, config=cfg)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def _run(world, cfg, tmp_path):
    import torch.multiprocessing as mp
    log = str(tmp_path / "log")
    mp.start_processes(_worker, args=(world, _free_port(), cfg, log), nprocs=world, join=True, start_method="spawn")
    return "".join(open(f"{log}.{r}").read() for r in range(world))


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("name", ["g1", "g1b", "g1c"])
def test_dist_wgs_shared_gpu_matches_reference(name, world, tmp_path):
    """The golden cohorts' files at 2 and 4 ranks.  Their decoy lines make the
    reference file's keys non-monotone, which the device ingest hands to the
    host parser at one rank too: under torch.distributed every rank agrees
    and rank 0 runs the one-GPU step -- the fallback path, checked here."""
    c, p = _stage(name, tmp_path)
    logs = _run(world, p, tmp_path)
    assert "Failed" not in logs, logs
    exp = os.path.join(G, name, "expected")
    for f in FILES:
        assert _content(os.path.join(c["output_dir"], f)) == _content(os.path.join(exp, f)), (f, logs)


def test_dist_wgs_shared_gpu_config1(tmp_path):
    """BASELINE config 1 at world 2 (both ranks own bins): every file of the
    reference, the normalised matrix by its sha256."""
    from tests.golden import cohort_files
    cfg, _, _ = cohort_files.regenerate("g_cfg1", tmp_path)
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(cfg))
    logs = _run(2, str(p), tmp_path)
    assert "Failed" not in logs, logs
    cohort_files.check_outputs("g_cfg1", tmp_path / "out", ibd=False)


@pytest.fixture(scope="module")
def bgzf_cohort(tmp_path_factory):
    """A mosdepth-like BGZF cohort the device ingest takes whole (tools/gen_cohort,
    the bench's depth model: 203 samples x 70,000 bins, 9 column blocks of 8192),
    and the one-GPU `grid wgs` outputs on it."""
    import bench
    root = tmp_path_factory.mktemp("bgzf")
    data, out1 = root / "data", root / "out1"
    cfg_path, _, _ = bench.prepare_files_cohort(str(data), str(out1), 203, 70_000, gen_threads=8, threads=4)
    from grid_amd.pipeline import run_wgs_pipeline
    run_wgs_pipeline(console=None, config=cfg_path)
    return root, cfg_path, out1


@pytest.mark.parametrize("world", [2, 4])
def test_dist_wgs_shared_gpu_equals_one_gpu(bgzf_cohort, world, tmp_path):
    """The distributed path proper (no fallback): every rank's device ingest of
    its file slice, the chain, the all-to-alls, HipOps' steps 4-5 on column
    shards and the offset-placed device writer -- every output file's text equal
    to the one-GPU run's (whose equality with the reference the e2e goldens
    show)."""
    import yaml
    root, cfg_path, out1 = bgzf_cohort
    c = yaml.safe_load(open(cfg_path))
    outw = tmp_path / "out"
    os.makedirs(outw)
    shutil.copy(out1 / "counts.tsv", outw / "counts.tsv")
    c["output_dir"] = str(outw)
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(c))
    logs = _run(world, str(p), tmp_path)
    assert "Failed" not in logs and "rank 0 reads the cohort" not in logs, logs
    for f in FILES:
        assert _content(outw / f) == _content(out1 / f), f
    from grid_amd import _abi
    ids, sc, mu, rt, zq = _abi.read_normalized_gz(str(outw / "normalized.tsv.gz"))   # the 'GR' index, global rows
    assert len(ids) == 203 and zq.shape[0] == 203
