"""Step 6 -- neighbour-normalised diploid copy number, MI355X path.

Drop-in for grid/utils/compute_dipcn.py.  Counts and neighbour files are
read exactly as the reference reads them (pandas for the counts, :46-49);
the per-sample gather-ratio (:62-88) runs as a HIP kernel
(grid_amd/csrc/dipcn_phase.hip) in fp64 with the reference's operation
order, including its ZeroDivisionError cases.
"""
from __future__ import annotations

import gzip
from pathlib import Path

import numpy as np
import pandas as pd

from .. import engine
from ..device import get_device
from .utils import log, progress_bar


def load_neighbors(neighbors_file):
    """:105-152 -> ({id: [(nbr_id, nbr_scale), ...]}, {id: scale})."""
    neighbors, scales = {}, {}
    with gzip.open(neighbors_file, "rt") as f:
        for line in f:
            parts = line.strip().split("\t")
            if len(parts) < 2:
                continue
            try:
                s = float(parts[1])
            except ValueError:
                continue
            scales[parts[0]] = s
            lst = []
            i = 2
            while i + 2 <= len(parts):
                try:
                    lst.append((parts[i], float(parts[i + 1])))
                except ValueError:
                    pass
                i += 3
            neighbors[parts[0]] = lst
    return neighbors, scales


def _read_counts(path) -> dict:
    """:46-49, verbatim semantics (pandas parses all-numeric IDs as ints)."""
    raw = pd.read_csv(path, sep="\t", header=0, names=["Sample", "Reads"])
    raw["Reads"] = pd.to_numeric(raw["Reads"], errors="coerce")
    raw.dropna(subset=["Reads"], inplace=True)
    return raw.set_index("Sample")["Reads"].to_dict()


def dipcn_arrays(neighbors: dict, sample_scales: dict, reads: dict, n_nbr: int, dev=None):
    """Run the device kernel on dict inputs; returns ([(id, value)], missing_ids)."""
    ids = list(neighbors)
    n = len(ids)
    universe = {sid: i for i, sid in enumerate(ids)}
    for lst in neighbors.values():
        for nid, _ in lst:
            if nid not in universe:
                universe[nid] = len(universe)
    u = len(universe)
    names = list(universe)
    has = np.array([x in reads for x in names], dtype=np.uint8)
    rd = np.array([float(reads[x]) if h else 0.0 for x, h in zip(names, has)], dtype=np.float64)
    k = max((len(l) for l in neighbors.values()), default=0)
    nbr = np.full((max(n, 1), max(k, 1)), -1, dtype=np.int32)
    nsc = np.zeros((max(n, 1), max(k, 1)), dtype=np.float64)
    cnt = np.zeros(max(n, 1), dtype=np.int32)
    scale = np.zeros(max(u, 1), dtype=np.float64)
    missing = set()
    for i, sid in enumerate(ids):
        lst = neighbors[sid]
        cnt[i] = len(lst)
        scale[i] = sample_scales[sid]
        c = 0
        for t, (nid, ns) in enumerate(lst):
            nbr[i, t] = universe[nid]
            nsc[i, t] = ns
            if c < n_nbr and sid in reads:
                if nid in reads:
                    c += 1
                else:
                    missing.add(nid)
    if n == 0:
        return [], missing
    out, valid = engine.dipcn(dev or get_device(), rd, has, scale, nbr, nsc, cnt, int(n_nbr), n_rows=n)
    return [(ids[i], float(out[i])) for i in range(n) if valid[i]], missing


def compute_diploid_genotypes(config, console) -> None:
    """Step entry point (:10-101)."""
    try:
        prefix = config.get("compute_diploid_genotypes", {}).get("output_file_prefix", None)
        ftype = config.get("output_file_type", "tsv")
        output_dir = config.get("output_dir", ".")
        output_file = Path(f"{output_dir}/{prefix}.{ftype}")
        n_nbr = config.get("compute_diploid_genotypes", {}).get("n_nbr", 300)
        counts_prefix = config["count_reads"].get("output_file_prefix", None)
        counts_file = Path(f"{output_dir}/{counts_prefix}.{ftype}")
        zmax = config["mosdepth"]["neighbors"].get("zmax", 2.0)
        nb_prefix = config["mosdepth"]["neighbors"].get("output_file_prefix", None)
        neighbors_file = Path(f"{output_dir}/{nb_prefix}.zMax{zmax:.1f}.{ftype}.gz")
    except Exception as e:
        log(console, f"Config error: {e}", style="danger")
        return

    from .dist_step4 import dist_comm, rank0_step
    comm = dist_comm()
    if comm is not None:                    # torch.distributed: rank 0 computes, the others wait
        rank0_step(comm, lambda: _compute_one(console, counts_file, neighbors_file, n_nbr, output_file, config))
        return
    _compute_one(console, counts_file, neighbors_file, n_nbr, output_file, config)


def _compute_one(console, counts_file, neighbors_file, n_nbr, output_file, config):
    reads = _read_counts(counts_file)
    neighbors, scales = load_neighbors(neighbors_file)
    with progress_bar(console, total=len(neighbors), description="Computing dipCN...") as (progress, task):
        rows, missing = dipcn_arrays(neighbors, scales, reads, n_nbr, get_device(config))
        progress.advance(task, len(neighbors))
    if missing:
        log(console, f"Warning: {len(missing)} neighbor IDs not found in read counts "
                     f"(showing up to 5: {list(missing)[:5]})", style="warning")
    df = pd.DataFrame(rows, columns=["Sample", "Norm_Reads"])
    df.to_csv(output_file, sep="\t", index=False)
    log(console, f"Saved {len(df)} samples → {output_file}", style="success")
