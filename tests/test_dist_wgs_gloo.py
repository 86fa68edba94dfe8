"""The distributed drop-in on CPU: `grid wgs` (run_wgs_pipeline) under
torch.distributed with gloo at world sizes 2, 3 and 4, steps 4-5 over every
rank (grid_amd/utils/dist_step4.py: files sliced over the ranks, the
population-sum chain, the all-to-all to 8192-aligned column shards,
fused.Steps47's bin split, the z all-to-all to row blocks and the
offset-placed writer) must give the reference's files -- the golden cohorts'
normalised matrix and neighbour lists, byte for byte after gunzip.

The compute is the CPU restatement (tests/dist_cpu_backend.py: the
line-by-line ingest, tests/cpu_ops.py, the host member coder); what is under
test is the distribution itself.  The same path on the GPU's kernels, with
ranks sharing the GPU: tests/test_gpu_dist_wgs.py."""
import gzip
import os
import shutil
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import yaml

G = os.path.join(os.path.dirname(__file__), "golden")
FILES = ("normalized.tsv.gz", "neighbors.zMax2.0.tsv.gz")


def _content(p):
    with gzip.open(p, "rt") as f:
        return f.read()


def _stage(name, tmp_path):
    src = os.path.join(G, name)
    shutil.copytree(os.path.join(src, "inputs"), tmp_path / "inputs")
    c = yaml.safe_load(open(os.path.join(src, "config.yaml")))
    c["samples_file"] = str(tmp_path / c["samples_file"])
    c["output_dir"] = str(tmp_path / "out")
    c["mosdepth"]["work_dir"] = str(tmp_path / c["mosdepth"]["work_dir"])
    c["mosdepth"]["normalize"]["repeat_mask_file"] = str(tmp_path / c["mosdepth"]["normalize"]["repeat_mask_file"])
    c["compute_diploid_genotypes"]["run"] = False        # steps 6-7 run on rank 0 (GPU kernels)
    c["compute_haploid_genotypes"]["run"] = False
    os.makedirs(c["output_dir"], exist_ok=True)
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
                      LOCAL_RANK=str(rank), GRID_DIST_BACKEND="gloo")
    sys.stdout = open(f"{log}.{rank}", "w")
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from grid_amd.utils import dist_step4
    from tests.dist_cpu_backend import CpuBackend
    dist_step4.BACKEND_FACTORY = lambda c: CpuBackend(c)
    from grid_amd.pipeline import run_wgs_pipeline
    run_wgs_pipeline(console=None, config=cfg)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def run_world(name, world, tmp_path):
    c, p = _stage(name, tmp_path)
    log = str(tmp_path / "log")
    mp.start_processes(_worker, args=(world, _free_port(), p, log), nprocs=world, join=True, start_method="spawn")
    logs = "".join(open(f"{log}.{r}").read() for r in range(world))
    return c["output_dir"], logs


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("name", ["g1", "g1b", "g1c"])
def test_dist_wgs_matches_reference(name, world, tmp_path):
    out, logs = run_world(name, world, tmp_path)
    assert "Failed" not in logs, logs
    assert "rank 0 reads the cohort" not in logs, logs          # the distributed path ran, no fallback
    exp = os.path.join(G, name, "expected")
    for f in FILES:
        assert _content(os.path.join(out, f)) == _content(os.path.join(exp, f)), (f, logs)


def test_dist_wgs_config1_world2(tmp_path):
    """BASELINE config 1 (100 samples x 30k bins, the golden's seed): every rank
    of 8192-aligned shards owns bins; the 13.7 MB normalised matrix and the
    neighbour file equal the reference's (make_golden.py cfg1)."""
    from tests.golden import cohort_files
    cfg, _, _ = cohort_files.regenerate("g_cfg1", tmp_path)
    cfg["compute_diploid_genotypes"]["run"] = False
    cfg["compute_haploid_genotypes"]["run"] = False
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(cfg))
    log = str(tmp_path / "log")
    mp.start_processes(_worker, args=(2, _free_port(), str(p), log), nprocs=2, join=True, start_method="spawn")
    logs = "".join(open(f"{log}.{r}").read() for r in range(2))
    assert "Failed" not in logs and "rank 0 reads the cohort" not in logs, logs
    cohort_files.check_outputs("g_cfg1", tmp_path / "out", only=FILES)


def test_file_slices_and_row_blocks_cover_everything():
    """The ingest's file slices (contiguous, balanced by compressed bytes, empty
    and missing files counted) and the writer's row blocks partition their
    ranges for every world size, including more ranks than files."""
    from grid_amd.utils.dist_step4 import file_slices, row_blocks
    import numpy as np
    rng = np.random.default_rng(3)
    for nf in (0, 1, 3, 40, 3202):
        sizes = rng.integers(0, 5 << 20, nf).tolist()
        for world in (1, 2, 3, 8, 64):
            b = file_slices(sizes, world)
            assert b[0] == 0 and b[-1] == nf and len(b) == world + 1
            assert all(b[r] <= b[r + 1] for r in range(world))
            if nf >= 8 * world and world > 1:
                per = [sum(sizes[b[r]:b[r + 1]]) for r in range(world)]
                assert max(per) <= sum(sizes) / world + max(sizes) + nf     # balanced to one file
        for world in (1, 2, 5, 8):
            rb = row_blocks(nf, world)
            assert rb[0] == 0 and rb[-1] == nf and all(rb[t] <= rb[t + 1] for t in range(world))
