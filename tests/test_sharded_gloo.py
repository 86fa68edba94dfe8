"""Multi-GPU path on CPU: the bin-sharded steps 4-7 chain (grid_amd/fused.py)
run under torch.distributed with the gloo backend at world sizes 2, 3, 4, 5
and 8 must give bit-identical results to one rank, and to the oracle.

The compute ops are the CPU restatement in tests/cpu_ops.py (the product
always uses HipOps); what is under test is the sharding: 8192-aligned
ranges, padded all-gathers of row-block partials and ratios, the global
selection threshold and sigma2 bound, the int64 Gram all-reduce, the
row-block top-k and its all-gather."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, M, K, ITERS = 20, 3 * 8192 + 517, 4, 6
# the world-4/5/8 cohort: every rank of 8 owns bins (9 blocks of 8192, the last
# partial), np = 512 rows in 2W segment blocks -- at W = 8 blocks 10-15 hold
# only padding rows (n = 300), at W = 5 2W*B = 520 > np (padded blocks)
WIDE = (300, 8 * 8192 + 517)


def cohort(n=N, m=M):
    N, M = n, m
    rng = np.random.default_rng(11)
    base = rng.uniform(25, 55, M)
    clus = rng.integers(0, 3, N)
    off = rng.uniform(-0.08, 0.08, (3, M))
    scale = rng.uniform(0.6, 1.4, N)
    q = np.rint(base[None, :] * (1 + off[clus]) * scale[:, None] * rng.uniform(0.8, 1.2, (N, M)) * 100)
    q = q.astype(np.int32)
    q[rng.random((N, M)) < 0.01] = -(2 ** 31)          # a few missing cells
    reads = np.rint(rng.uniform(200, 900, N))
    offs = np.zeros(2 * N + 1, dtype=np.int64)
    nbr = []
    for h in range(2 * N):
        js = rng.integers(0, 2 * N, int(rng.integers(0, 5)))
        nbr += js.tolist()
        offs[h + 1] = offs[h] + len(js)
    return q, reads, offs, np.array(nbr, dtype=np.int32), np.ones(len(nbr))


def run_chain(rank, world, comm, chunk=None, source="resident", shape=(N, M), split="bin", piece_bytes=1 << 31):
    from grid_amd.fused import HostSource, Steps47, TorchAlloc, shard_range
    from tests.cpu_ops import NumpyOps
    N, M = shape
    q, reads, off, nbr, w = cohort(N, M)
    c0, c1 = shard_range(M, rank, world)
    qs = torch.from_numpy(np.ascontiguousarray(q[:, c0:c1]))
    st = Steps47(NumpyOps(), TorchAlloc("cpu"), N, M, c0, c1 - c0, k=K, n_nbr=3, n_iters=ITERS, comm=comm,
                 chunk=chunk, split=split, piece_bytes=piece_bytes)
    st.set_reads(reads)
    st.set_phasing_graph(off, nbr, w)
    st.run(HostSource(qs.numpy()) if source == "host" else qs, c1 - c0)
    ml = c1 - c0
    return {
        "rm": st.rm.numpy()[:N].copy(), "mu": st.mu.numpy()[:ml].copy(), "var": st.var.numpy()[:ml].copy(),
        "sel": (st.sel.numpy()[: st.r_loc] + c0).copy(), "zq": st.zq_int32().numpy()[:N, : st.r_loc].copy(),
        "idx": st.idx_out.numpy()[:N].copy(), "d2": st.d2.numpy()[:N].copy(), "dip": st.dip.numpy()[:N].copy(),
        "hap": st.hap.numpy()[: 2 * N].copy(), "imp": st.imp.numpy()[: 2 * N].copy(), "scale": st.scale,
        "ruse": st.ruse_loc,
    }


def _worker(rank, world, port, out_path, chunk, shape=(N, M), split="bin", piece_bytes=1 << 31):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from grid_amd.fused import TorchComm
    res = run_chain(rank, world, TorchComm(dist), chunk=chunk, shape=shape, split=split, piece_bytes=piece_bytes)
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
    return run_chain(0, 1, None)


def test_single_rank_matches_oracle(single):
    from oracle import steps
    from oracle.npsum import nanmean_rows
    q = cohort()[0]
    mat = np.where(q == -(2 ** 31), np.nan, q / 100.0)
    z, ratios, mu, var, scale = steps.normalize_matrix(mat)
    assert np.array_equal(single["rm"], nanmean_rows(mat))
    assert np.array_equal(single["mu"], mu, equal_nan=True)
    assert single["scale"] == scale
    assert single["sel"].tolist() == steps.select_high_variance_regions(ratios, 0.1)


@pytest.mark.parametrize("chunk,source", [(8192, "resident"), (16384, "host"), (8192, "host")])
def test_streamed_equals_single(single, chunk, source):
    """Bin-axis streaming (3-4 chunks, the last one partial) gives the
    one-chunk chain's results bit for bit, from a resident matrix read in
    chunks and from a host source copied slab by slab."""
    res = run_chain(0, 1, None, chunk=chunk, source=source)
    for key in ("rm", "mu", "var", "sel", "zq", "idx", "d2", "dip", "hap", "imp", "ruse", "scale"):
        assert np.array_equal(np.asarray(res[key]), np.asarray(single[key]), equal_nan=True), key


@pytest.fixture(scope="module")
def single_wide():
    return run_chain(0, 1, None, shape=WIDE)


def _run_world(world, chunk, shape, tmp_path, split="bin", piece_bytes=1 << 31):
    port = _free_port()
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, port, out, chunk, shape, split, piece_bytes), nprocs=world, join=True,
                       start_method="spawn")
    return [dict(np.load(f"{out}.{r}.npz")) for r in range(world)]


@pytest.mark.parametrize("world,chunk", [(2, None), (3, None), (2, 8192)])
def test_sharded_equals_single(single, world, chunk, tmp_path):
    _check_parts(_run_world(world, chunk, (N, M), tmp_path), single)


@pytest.mark.parametrize("world,chunk", [(4, None), (5, None), (8, None), (8, 8192)])
def test_sharded_world_4_5_8_equals_single(single_wide, world, chunk, tmp_path):
    """the driver's 8-GPU layout (blocks r and 2W-1-r of
    B = np/2W rows, the all-padding blocks of ranks 5-7 at n = 300, one or
    two 8192-blocks of bins per rank) and a world (5) whose 2W*B exceeds np."""
    from grid_amd.fused import shard_range
    assert all(shard_range(WIDE[1], r, world)[1] > shard_range(WIDE[1], r, world)[0] for r in range(world))
    _check_parts(_run_world(world, chunk, WIDE, tmp_path), single_wide)


# cohort split: the Gram's rows sharded, the panel
# all-gathered in pieces.  piece_bytes small enough for several pieces per
# chunk (odd piece counts, a short last piece) at N = 20 (np 256, 1 block of
# 256 rows: ranks > 0 hold only padding blocks) and at N = 300 (np 512)
@pytest.mark.parametrize("world,chunk,piece", [(2, None, 1 << 31), (2, 8192, 40 * 256 * 64), (3, None, 6 * 256 * 64)])
def test_cohort_split_equals_single(single, world, chunk, piece, tmp_path):
    _check_parts(_run_world(world, chunk, (N, M), tmp_path, split="cohort", piece_bytes=piece), single)


@pytest.mark.parametrize("world,chunk,piece", [(4, None, 4 * 512 * 64 * 30), (8, None, 1 << 31),
                                               (8, 8192, 8 * 512 * 64 * 50)])
def test_cohort_split_world_2_4_8_equals_single(single_wide, world, chunk, piece, tmp_path):
    _check_parts(_run_world(world, chunk, WIDE, tmp_path, split="cohort", piece_bytes=piece), single_wide)


def test_wide_single_rank_matches_oracle_neighbours(single_wide):
    """The world-1 reference of the wide cases against the oracle's exact
    k-NN on the printed step-4 values (so the bit-identity above is anchored)."""
    from oracle import steps
    q = cohort(*WIDE)[0]
    mat = np.where(q == -(2 ** 31), np.nan, q / 100.0)
    z, ratios, mu, var, scale = steps.normalize_matrix(mat)
    assert single_wide["scale"] == scale
    sel = steps.select_high_variance_regions(ratios, 0.1)
    assert single_wide["sel"].tolist() == sel
    # step 5 on the printed values, as smoke() does
    raw = np.nanmean(mat, axis=1)
    lines = steps.normalized_lines(z, [f"S{i}" for i in range(WIDE[0])], sel, mu, var, raw)
    ids, r5, z5, sc5 = steps.parse_normalized(lines)
    idx5, _ = steps.filter_regions_by_variance(r5, 1.0, 1000.0)
    qz = np.rint(np.nan_to_num(np.clip(z5, -2.0, 2.0), nan=0.0)[:, idx5] * 100).astype(np.int64)
    nb = steps.knn_exact(qz, K)
    for i in range(WIDE[0]):
        assert single_wide["idx"][i, : len(nb[i])].tolist() == [j for j, _ in nb[i]], i


def _check_parts(parts, single):
    for key in ("rm", "idx", "d2", "dip", "hap", "imp"):
        for p in parts:
            assert np.array_equal(p[key], single[key], equal_nan=True), key
    assert np.array_equal(np.concatenate([p["mu"] for p in parts]), single["mu"], equal_nan=True)
    assert np.array_equal(np.concatenate([p["var"] for p in parts]), single["var"], equal_nan=True)
    assert np.concatenate([p["sel"] for p in parts]).tolist() == single["sel"].tolist()
    assert np.array_equal(np.concatenate([p["zq"] for p in parts], axis=1), single["zq"])
    assert sum(int(p["ruse"]) for p in parts) == int(single["ruse"])
    assert all(float(p["scale"]) == single["scale"] for p in parts)


@pytest.mark.parametrize("split", ["bin", "cohort"])
def test_simulated_rank_runs(split):
    """bench.py --sim-world W --sim-rank r (per-rank timing on one GPU): rank
    r's share of a W-rank step runs through fused.SimComm, whose collectives
    do only their local copies, and counts the bytes the real ones would
    bring in (the results are meaningless by design: other ranks' parts are
    this rank's)."""
    from grid_amd.fused import SimComm
    comm = SimComm(4, 1)
    res = run_chain(1, 4, comm, shape=WIDE, split=split, piece_bytes=4 * 512 * 64 * 8)
    assert res["idx"].shape == (WIDE[0], K)
    kinds = set(comm.bytes_in)
    assert {"all_gather", "all_reduce"} <= kinds
    assert ("all_gather_panel" in kinds) == (split == "cohort")
    assert ("reduce_scatter" in kinds) == (split == "bin")
