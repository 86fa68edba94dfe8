"""Steps 4-7 from files to files, as the reference runs them (TEST
INFRASTRUCTURE ONLY: the checker and bench.py's CPU baseline).

Follows the reference's step functions end to end on one cohort config:
normalize_mosdepth (normalize_mosdepth.py:23-145: ingest, normalize_matrix,
select_high_variance_regions, write_normalized_output with "%.2f"/"%.3f" text
into gzip at its default level 9), find_neighbors (find_neighbors.py:11-77:
gzip read and parse, clip, sigma^2 filter, exact k-NN, save_neighbors),
compute_diploid_genotypes (compute_dipcn.py:10-100) and hi_inference
(hi_inference.py:253-339), composed from the restatements in this package.
Each step reads the previous step's file, as the reference does.  Returns
the wall time of every stage, so the bench can report the reference's whole
step cost (parse and text I/O included), not only its arithmetic.
"""
from __future__ import annotations

import gzip
import os
import time

import numpy as np

from . import ingest, loaders, steps
from .npsum import nanmean_rows


def _path(root, p):
    return p if os.path.isabs(p) else os.path.join(root, p)


def run(cfg: dict, root: str = "", only_step7: bool = False) -> dict:
    """Run steps 4-7 of ``cfg`` (paths relative to ``root``); writes the four
    output files into cfg["output_dir"] and returns {stage: seconds}.
    ``only_step7``: hi_inference alone, on the dipCN file already there."""
    t = {}
    if only_step7:
        return _step7(cfg, root, t)
    out = _path(root, cfg["output_dir"])
    os.makedirs(out, exist_ok=True)
    typ = cfg["output_file_type"]
    nc = cfg["mosdepth"]["normalize"]
    nbc = cfg["mosdepth"]["neighbors"]
    # ---- step 4 ----
    t0 = time.perf_counter()
    samples = [s.strip() for s in open(_path(root, cfg["samples_file"])) if s.strip()]
    ids, regions, mat = ingest.ingest(_path(root, cfg["mosdepth"]["work_dir"]), samples, cfg.get("chrom"),
                                      cfg.get("start_bp"), cfg.get("end_bp"),
                                      _path(root, nc["repeat_mask_file"]) if nc.get("repeat_mask_file") else None,
                                      nc["min_depth"], nc["max_depth"])
    t1 = time.perf_counter()
    raw = nanmean_rows(mat)
    z, ratios, mu, var, _ = steps.normalize_matrix(mat)
    sel = steps.select_high_variance_regions(ratios, nc["top_frac"])
    t2 = time.perf_counter()
    norm = os.path.join(out, f"{nc['output_file_prefix']}.{typ}.gz")
    with gzip.open(norm, "wt") as f:
        f.writelines(steps.normalized_lines(z, ids, sel, mu, var, raw))
    t3 = time.perf_counter()
    t.update(ingest=t1 - t0, normalize=t2 - t1, write_normalized=t3 - t2)
    # ---- step 5 ----
    with gzip.open(norm, "rt") as f:
        lines = f.readlines()
    ids5, r5, z5, sc5 = steps.parse_normalized(lines)
    t4 = time.perf_counter()
    zmax = nbc["zmax"]
    zc = np.nan_to_num(np.clip(z5, -zmax, zmax), nan=0.0)
    idx, ruse = steps.filter_regions_by_variance(r5, 1.0, nbc["sigma2_max"])
    q = np.rint(zc[:, idx] * 100).astype(np.int64)
    nbrs = steps.knn_exact(q, nbc["num_neighbors"])
    t5 = time.perf_counter()
    nfile = os.path.join(out, f"{nbc['output_file_prefix']}.zMax{zmax:.1f}.{typ}.gz")
    with gzip.open(nfile, "wt") as f:
        f.writelines(steps.neighbor_lines(ids5, sc5, nbrs, ruse))
    t6 = time.perf_counter()
    t.update(read_normalized=t4 - t3, knn=t5 - t4, write_neighbors=t6 - t5)
    # ---- step 6 ----
    import pandas as pd
    dc = cfg["compute_diploid_genotypes"]
    nbd, scd = loaders.load_neighbors(nfile)
    reads = loaders.read_counts(os.path.join(out, f"{cfg['count_reads']['output_file_prefix']}.{typ}"))
    dip = steps.dipcn(nbd, scd, reads, dc["n_nbr"])
    dfile = os.path.join(out, f"{dc['output_file_prefix']}.{typ}")
    pd.DataFrame(dip, columns=["Sample", "Norm_Reads"]).to_csv(dfile, sep="\t", index=False)
    t7 = time.perf_counter()
    t["dipcn"] = t7 - t6
    t["shape"] = {"n": len(ids), "m": mat.shape[1], "R": len(sel), "R_use": int(ruse)}
    return _step7(cfg, root, t)


def _step7(cfg, root, t):
    out = _path(root, cfg["output_dir"])
    typ = cfg["output_file_type"]
    dfile = os.path.join(out, f"{cfg['compute_diploid_genotypes']['output_file_prefix']}.{typ}")
    t7 = time.perf_counter()
    hc = cfg["compute_haploid_genotypes"]
    hid, irr, hidx = loaders.read_dipcn(dfile)
    if hc["method"] == "ibs":
        hn = loaders.load_ibs(_path(root, hc["ibs_output"]), hidx, hc["max_neighbors"])
    else:
        hn = loaders.load_ibd(_path(root, hc["ibd_output"]), hidx, hc["max_neighbors"], cfg.get("start_bp"),
                              cfg.get("end_bp"), hc["min_length"], hc["min_match"], hc["weighted"],
                              hc["weight_scale"])
    t8 = time.perf_counter()
    hap, mean = steps.run_phasing(irr, hn, hc["min_neighbors"], hc["n_iters"])
    imp = [steps.compute_imp(i, hap, hn, mean) for i in range(len(irr))]
    t9 = time.perf_counter()
    with open(os.path.join(out, f"{hc['output_file_prefix']}.{typ}"), "w") as f:
        f.write("".join(steps.haploid_lines(hid, irr, hap, imp)))
    t10 = time.perf_counter()
    t.update(load_hap_neighbors=t8 - t7, phasing=t9 - t8, write_haploid=t10 - t9)
    return t
