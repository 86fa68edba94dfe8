"""Multi-GPU path with the real HIP kernels: the bin-sharded steps 4-7 chain
at world sizes 2, 3, 4 and 8 (ranks sharing the one visible GPU, gloo standing in
for RCCL, which needs a GPU per rank) must give bit-identical neighbours,
dipCN and phasing to one rank, with step 7 on its own stream (the bench's
overlapped configuration) on every rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, M, K, ITERS = 300, 8 * 8192 + 517, 6, 12     # 9 bin blocks: every rank of 8 owns bins


def cohort():
    rng = np.random.default_rng(5)
    base = rng.uniform(25, 55, M)
    clus = rng.integers(0, 4, N)
    off = rng.uniform(-0.08, 0.08, (4, M))
    scale = rng.uniform(0.6, 1.4, N)
    q = np.rint(base[None, :] * (1 + off[clus]) * scale[:, None] * rng.uniform(0.8, 1.2, (N, M)) * 100)
    q = q.astype(np.int32)
    q[rng.random((N, M)) < 0.01] = -(2 ** 31)
    reads = np.rint(rng.uniform(200, 900, N))
    offs = np.zeros(2 * N + 1, dtype=np.int64)
    nbr = []
    for h in range(2 * N):
        js = rng.integers(0, 2 * N, int(rng.integers(0, 8)))
        nbr += js.tolist()
        offs[h + 1] = offs[h] + len(js)
    return q, reads, offs, np.array(nbr, dtype=np.int32), np.ones(len(nbr))


def run_chain(rank, world, comm, lane, split="bin", piece_bytes=1 << 31):
    from grid_amd import _abi
    from grid_amd.fused import HipOps, Steps47, TorchAlloc, shard_range
    q, reads, off, nbr, w = cohort()
    c0, c1 = shard_range(M, rank, world)
    dev = _abi.Device(0)
    dev.set_stream(torch.cuda.current_stream())
    qs = torch.from_numpy(np.ascontiguousarray(q[:, c0:c1])).cuda()
    pl = None
    if lane:                             # lane = 1 or 2 phasing lanes (two: one per dipCN buffer)
        pl = []
        for _ in range(lane):
            pdev = _abi.Device(0)
            ps = torch.cuda.Stream()
            pdev.set_stream(ps)
            pl.append((HipOps(pdev), ps))
        pl = pl[0] if lane == 1 else pl
    st = Steps47(HipOps(dev), TorchAlloc(0), N, M, c0, c1 - c0, k=K, n_nbr=4, n_iters=ITERS, comm=comm,
                 phase_lane=pl, split=split, piece_bytes=piece_bytes)
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)
    st.run(qs, c1 - c0)
    st.run(qs, c1 - c0)                  # second pass: the lane's cross-pass ordering
    st.finish()                          # the second pass's deferred phasing
    torch.cuda.synchronize()
    ml = c1 - c0
    return {
        "rm": st.rm[:N].cpu().numpy(), "mu": st.mu[:ml].cpu().numpy(), "var": st.var[:ml].cpu().numpy(),
        "zq": st.zq_int32()[:N, : st.r_loc].cpu().numpy(), "idx": st.idx_out[:N].cpu().numpy(),
        "d2": st.d2[:N].cpu().numpy(), "dip": st.dip[:N].cpu().numpy(), "hap": st.hap[: 2 * N].cpu().numpy(),
        "imp": st.imp[: 2 * N].cpu().numpy(), "scale": st.scale, "ruse": st.ruse_loc,
    }


def _worker(rank, world, port, out_path, split="bin", piece_bytes=1 << 31):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from grid_amd.fused import TorchComm
    res = run_chain(rank, world, TorchComm(dist), lane=2 if world % 2 == 0 else 1, split=split,
                    piece_bytes=piece_bytes)
    np.savez(f"{out_path}.{rank}.npz", **{k: np.asarray(v) for k, v in res.items()})
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def single():
    return run_chain(0, 1, None, lane=False)


def _run(world, tmp_path, split="bin", piece_bytes=1 << 31):
    port = _free_port()
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, port, out, split, piece_bytes), nprocs=world, join=True,
                       start_method="spawn")
    return [dict(np.load(f"{out}.{r}.npz")) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_gpu_sharded_equals_single(single, world, tmp_path):
    _check(_run(world, tmp_path), single)


# the cohort split: np = 512 in 256-row blocks, so at
# world 2 ranks hold blocks (0, 3), (1, 2), at 4 and 8 ranks >= 1 have padding
# blocks; small pieces: several all-gathers per pass, a short last piece
@pytest.mark.parametrize("world,piece", [(2, 1 << 31), (2, 2 * 512 * 64 * 22), (4, 4 * 512 * 64 * 10),
                                         (8, 1 << 31)])
def test_gpu_cohort_split_equals_single(single, world, piece, tmp_path):
    _check(_run(world, tmp_path, split="cohort", piece_bytes=piece), single)


def _check(parts, single):
    for key in ("rm", "idx", "d2", "dip", "hap", "imp"):
        for p in parts:
            assert np.array_equal(p[key], single[key], equal_nan=True), key
    assert np.array_equal(np.concatenate([p["mu"] for p in parts]), single["mu"], equal_nan=True)
    assert np.array_equal(np.concatenate([p["var"] for p in parts]), single["var"], equal_nan=True)
    assert np.array_equal(np.concatenate([p["zq"] for p in parts], axis=1), single["zq"])
    assert sum(int(p["ruse"]) for p in parts) == int(single["ruse"])
    assert all(float(p["scale"]) == single["scale"] for p in parts)
