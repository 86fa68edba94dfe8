"""Step 5 -- nearest neighbours on normalised coverage, MI355X path.

Drop-in for grid/utils/find_neighbors.py.  The reference calls scikit-learn's
brute-force Euclidean ArgKmin (:207-213).  Here the clipped z-scores, which
the normalised file holds as exact hundredths, are uploaded once as int32 and
turned on the device into (grid_amd/engine.py _knn_zq):
  * zmax = q/100 with q <= 256 (the default 2.0): an integer bf16 panel whose
    Gram matrix is computed exactly on the MFMA pipe;
  * zmax = q/100 with q > 256: exact int64 direct-difference distances;
  * any other zmax (clipped values are not hundredths): fixed-order fp64
    direct-difference distances;
and the k+1 nearest are selected per row on the GPU (grid_amd/csrc/knn.hip).
On the integer paths the neighbour order equals sklearn's wherever exact
distances differ (sklearn's own tie order is undefined).
"""
from __future__ import annotations

import gzip
from pathlib import Path

import numpy as np

from .. import _abi, engine
from ..device import get_device
from . import handoff
from .utils import log, progress_bar


def _hundredths(tok: str) -> int:
    """"%.2f" text -> integer hundredths (NA -> missing)."""
    if tok in ("NA", "nan"):
        return _abi.MISSING
    neg = tok.startswith("-")
    t = tok[1:] if neg else tok
    ip, _, fp = t.partition(".")
    if len(fp) != 2 or not ip.isdigit() or not fp.isdigit():
        v = float(tok)
        k = round(v * 100)
        if k / 100.0 != v:
            raise ValueError(f"z value {tok!r} is not a 2-decimal number")
        return k
    k = int(ip) * 100 + int(fp)
    return -k if neg else k


def read_normalized_data(input_file):
    """:81-124 -> (individuals, sigma2ratios, data_matrix float64, scales)."""
    ids, scales, zq, ratios = _read_normalized_q(input_file)
    data = np.where(zq == _abi.MISSING, np.nan, zq / 100.0)
    return ids, ratios, data, scales


def _read_normalized_q(input_file):
    """-> (ids, {id: scale}, zq [n][r] int hundredths, ratios).  Threaded host
    C++ parser (grid_read_normalized_gz); text outside its strict "%.2f"
    grammar goes through the general line parser below."""
    try:
        ids, sc, _means, ratios, zq = _abi.read_normalized_gz(input_file)
        return ids, {i: float(v) for i, v in zip(ids, sc)}, zq, ratios
    except _abi.GridNativeError as e:
        if e.code != _abi.GRID_EUNSUPPORTED:
            raise
    return _read_normalized_q_py(input_file)


def _read_normalized_q_py(input_file):
    ids, scales, rows = [], {}, []
    with gzip.open(input_file, "rt") as f:
        f.readline()
        parts = f.readline().strip().split("\t")
        ratios = np.array([np.nan if v in ("NA", "nan") else float(v) for v in parts[2:]])
        for line in f:
            p = line.strip().split("\t")
            ids.append(p[0])
            scales[p[0]] = float(p[1])
            rows.append([_hundredths(v) for v in p[2:]])
    r = len(rows[0]) if rows else 0
    zq = np.array(rows, dtype=np.int64).reshape(len(rows), r) if rows else np.zeros((0, 0), np.int64)
    if zq.size and (zq[zq != _abi.MISSING].max(initial=0) >= 2 ** 31 or zq.min() < _abi.MISSING):
        raise ValueError("normalised z value outside the int32 hundredths range")
    return ids, scales, zq.astype(np.int32), ratios


def filter_regions_by_variance(sigma2ratios, frac_r: float = 1.0, sigma2_max: float = 1000.0, console=None):
    """:128-175 (host; R values)."""
    sigma2ratios = np.asarray(sigma2ratios, dtype=np.float64)
    R = len(sigma2ratios)
    finite = np.isfinite(sigma2ratios)
    fv = np.sort(sigma2ratios[finite])
    if len(fv) == 0:
        log(console, "Warning: no finite variance ratios — keeping all regions", style="warning")
        return np.arange(R), R
    lo = min(int(R * (1.0 - frac_r)), len(fv) - 1)
    smin = float(fv[lo])
    extreme = int(np.sum(sigma2ratios > sigma2_max))
    if extreme and console:
        log(console, f"Removed {extreme} / {R} regions with sigma2ratio > {sigma2_max}", style="warning")
    keep = finite & (sigma2ratios >= smin) & (sigma2ratios <= sigma2_max)
    idx = np.where(keep)[0]
    return idx, len(idx)


def find_neighbors_sklearn(data_matrix, individuals, n_neighbors: int = 500):
    """:179-227 API: {id: [(neighbour_id, squared distance), ...]} computed on
    the GPU for any finite float64 matrix (engine.knn_values: exact integer
    paths when every value is a hundredth, fixed-order fp64 otherwise)."""
    data = np.asarray(data_matrix, dtype=np.float64)
    if data.ndim != 2:
        raise ValueError("data_matrix must be 2-D")
    idx, d2, cnt = engine.knn_values(get_device(), data, int(n_neighbors))
    return {ind: [(individuals[int(idx[i, t])], float(d2[i, t])) for t in range(cnt[i])]
            for i, ind in enumerate(individuals)}


def save_neighbors(neighbors_dict, scales, output_file, zmax, R_use) -> None:
    """:231-267"""
    if R_use == 0:
        R_use = 1
    with gzip.open(output_file, "wt", compresslevel=6) as out:
        for ind, nbrs in neighbors_dict.items():
            line = f"{ind}\t{scales.get(ind, 1.0):.2f}"
            for nid, sq in nbrs:
                line += f"\t{nid}\t{scales.get(nid, 1.0):.2f}\t{sq / (2 * R_use):.2f}"
            out.write(line + "\n")


def find_neighbors(config, console):
    """Step entry point (:11-77)."""
    try:
        zmax = config["mosdepth"]["neighbors"].get("zmax", 2.0)
        sigma2_max = config["mosdepth"]["neighbors"].get("sigma2_max", 1000.0)
        n_neighbors = config["mosdepth"]["neighbors"].get("num_neighbors", 500)
        frac_r = config["mosdepth"]["neighbors"].get("frac_r", 1.0)
        in_prefix = config["mosdepth"]["normalize"].get("output_file_prefix")
        ftype = config.get("output_file_type", "tsv")
        output_dir = config.get("output_dir", ".")
        input_file = Path(f"{output_dir}/{in_prefix}.{ftype}.gz")
        out_prefix = config["mosdepth"]["neighbors"].get("output_file_prefix", "neighbor_coverage")
        output_file = Path(output_dir) / f"{out_prefix}.zMax{zmax:.1f}.{ftype}.gz"
    except Exception as e:
        log(console, f"Config error: {e}", style="danger")
        return
    output_file.parent.mkdir(parents=True, exist_ok=True)

    from .dist_step4 import agree, dist_comm, rank0_step
    comm = dist_comm()
    if comm is not None:
        # torch.distributed: step 4 ran the search across the ranks (every rank
        # holds the lists); rank 0 writes them.  Otherwise rank 0 runs the
        # one-GPU step from the file while the others wait.
        params = {"zmax": zmax, "sigma2_max": sigma2_max, "frac_r": frac_r, "n_neighbors": n_neighbors}
        rec = handoff.take_neighbors(input_file, params)
        if agree(comm, rec is not None):
            def write():
                ids, nb = rec["ids"], rec["neighbors"]
                scales = {i: float(v) for i, v in zip(ids, rec["scales"])}
                idx, d2, cnt = nb["idx"], nb["d2"], nb["cnt"]
                nbrs = {ind: [(ids[int(idx[i, t])], float(d2[i, t]) / 10000.0) for t in range(cnt[i])]
                        for i, ind in enumerate(ids)}
                save_neighbors(nbrs, scales, output_file, zmax, nb["R_use"])
                log(console, f"Saved neighbors to {output_file}", style="success")
            rank0_step(comm, write)
        else:
            rank0_step(comm, lambda: _find_neighbors_one(config, console, input_file, output_file, zmax, sigma2_max,
                                                         n_neighbors, frac_r))
        return
    _find_neighbors_one(config, console, input_file, output_file, zmax, sigma2_max, n_neighbors, frac_r)


def _find_neighbors_one(config, console, input_file, output_file, zmax, sigma2_max, n_neighbors, frac_r):
    """Step 5 in one process (:11-77)."""
    got = handoff.take(input_file)              # step 4 ran in this process: its matrix, no re-parse
    if got is not None:
        ids, sc, ratios, zq, _shape = got
        scales = {i: float(v) for i, v in zip(ids, sc)}
    else:
        ids, scales, zq, ratios = _read_normalized_q(input_file)
    N = len(ids)
    valid, R_use = filter_regions_by_variance(ratios, frac_r=frac_r, sigma2_max=sigma2_max, console=console)

    # clip (:57), NaN -> 0 (:58) and the column filter (:171) run on the device
    # over the int32 hundredths (no host copies of the matrix)
    # the matrix goes to the k-NN in a holder: the call owns it and frees it
    # once the panel is built (a device hand-off is GBs of HBM)
    holder = [zq.reshape(N, -1) if N and got is None else zq]
    del zq, got
    with progress_bar(console, total=N, description="Finding neighbors...") as (progress, task):
        idx, d2, cnt = engine.knn_from_zq(get_device(config), holder, np.asarray(valid, dtype=np.int32),
                                          int(n_neighbors), float(zmax))
        progress.advance(task, N)

    nbrs = {ind: [(ids[int(idx[i, t])], float(d2[i, t])) for t in range(cnt[i])]
            for i, ind in enumerate(ids)}
    save_neighbors(nbrs, scales, output_file, zmax, R_use)
    log(console, f"Saved neighbors to {output_file}", style="success")
