"""Multi-locus (BASELINE config 5) test cohort: a few regions of the
734-VNTR table, per-locus dipCN and computeIBSpbwt-style files, one shared
iLASH file, and the oracle's expected step-7 output per locus
(hi_inference.py:253-339 restated in oracle/: loaders, run_phasing,
compute_imp, haploid_lines)."""
import os

import numpy as np

from oracle import loaders, steps

LOCI_TABLE = os.path.join(os.path.dirname(__file__), "golden", "loci",
                          "734_possible_coding_vntr_regions.IBD2R_gt_0.25.uniq.txt")


def write_cohort(root, n_loci=7, n=60, seed=11):
    """Writes the cohort under ``root``; returns (config, loci table path)."""
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "out"), exist_ok=True)
    rows = open(LOCI_TABLE).read().splitlines()
    table = os.path.join(root, "loci.txt")
    with open(table, "w") as f:
        f.write("\n".join([rows[0]] + rows[1: 1 + n_loci]) + "\n")
    ids = [f"HG{i:05d}" for i in range(n)]
    from grid_amd.utils.hi_inference import read_loci_file, _locus_path
    for lc in read_loci_file(table):
        name = f"{lc['chrom']}_{lc['start']}_{lc['end']}_{lc['gene']}"
        irr = rng.choice([1.0, 1.5, 2.0, 2.5, 3.0], n) * rng.uniform(0.9, 1.1, n)
        with open(os.path.join(root, "out", f"dipcn.{name}.tsv"), "w") as f:
            f.write("ID\tIRRs\n")
            for i in range(n):
                if rng.random() < 0.03:          # a sample missing at this locus
                    continue
                f.write(f"{ids[i]}\t{irr[i]:.6f}\n")
        with open(os.path.join(root, f"ibs.{lc['chrom']}_{lc['start']}.txt"), "w") as f:
            f.write("ID\thap\tnbrInd\tcMlen\tcMedge\tIDnbr\thapNbr\n")
            for i in range(n):
                for h in (1, 2):
                    for t in range(int(rng.integers(0, 12))):
                        j = int(rng.integers(0, n))
                        f.write(f"{ids[i]}\t{h}\t{t}\t{rng.uniform(0.5, 9):.3f}\t0\t{ids[j]}\t{int(rng.integers(1, 3))}\n")
    # one genome-wide iLASH file shared by every locus (weights depend on the region)
    with open(os.path.join(root, "ibd.txt"), "w") as f:
        for _ in range(40 * n):
            i, j = rng.integers(0, n, 2)
            bp1 = int(rng.integers(500_000, 2_500_000))
            bp2 = bp1 + int(rng.integers(1000, 400_000))
            f.write(f"{ids[i]}\t{ids[i]}_{int(rng.integers(0, 2))}\t{ids[j]}\t{ids[j]}_{int(rng.integers(0, 2))}\t1\t"
                    f"{bp1}\t{bp2}\trs1\trs2\t{rng.uniform(0.2, 8):.3f}\t{rng.uniform(0.6, 1.0):.4f}\n")
    cfg = {
        "output_dir": os.path.join(root, "out"), "output_file_type": "tsv",
        "compute_diploid_genotypes": {"run": True, "output_file_prefix": "dipcn"},
        "compute_haploid_genotypes": {"run": True, "method": "ibs", "output_file_prefix": "haploid",
                                      "loci_file": table, "n_iters": 25, "max_neighbors": 10, "min_neighbors": 1,
                                      "ibs_output": os.path.join(root, "ibs.{chrom}_{start}.txt")},
        "gpu": {"device": 0},
    }
    return cfg, table


def expected_outputs(cfg):
    """{output path: expected text} of the reference's step 7 run once per
    locus (the oracle restatement, loaders included)."""
    from grid_amd.utils.hi_inference import read_loci_file, _locus_path
    hc = cfg["compute_haploid_genotypes"]
    keys = dict(output_dir=cfg["output_dir"], prefix=hc["output_file_prefix"],
                dip_prefix=cfg["compute_diploid_genotypes"]["output_file_prefix"], type=cfg["output_file_type"])
    out = {}
    for lc in read_loci_file(hc["loci_file"]):
        ids, irr, idx = loaders.read_dipcn(_locus_path("{output_dir}/{dip_prefix}.{locus}.{type}", lc, **keys))
        if hc["method"] == "ibs":
            hn = loaders.load_ibs(_locus_path(hc["ibs_output"], lc, **keys), idx, hc["max_neighbors"])
        else:
            hn = loaders.load_ibd(_locus_path(hc["ibd_output"], lc, **keys), idx, hc["max_neighbors"], lc["start"],
                                  lc["end"], weighted=hc.get("weighted", False),
                                  weight_scale=hc.get("weight_scale", 1_000_000))
        hap, mean = steps.run_phasing(irr, hn, hc["min_neighbors"], hc["n_iters"])
        imp = [steps.compute_imp(i, hap, hn, mean) for i in range(len(irr))]
        path = str(_locus_path("{output_dir}/{prefix}.{locus}.{type}", lc, **keys))
        out[path] = "".join(steps.haploid_lines(ids, irr, hap, imp))
    return out
