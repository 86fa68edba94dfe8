"""Synthetic file cohorts in the reference's on-disk formats (mosdepth
regions.bed.gz, samples list, repeat mask, read counts, computeIBSpbwt IBS,
iLASH IBD) and the step config that points at them.

Shared by tests/golden/make_golden.py (which runs the REFERENCE on them to
produce the expected outputs) and by the GPU tests that regenerate a cohort
too large to commit (config 1: 100 x 30k) from its seed; the regenerated
inputs are checked against the content hash stored with the fixture.
"""
from __future__ import annotations

import gzip
import hashlib
from pathlib import Path

import numpy as np


# ------------------------------------------------------------ synthesis ----
def synth_cohort(rng, n, m, n_clusters, bin_size=1000, start0=0):
    """Depth hundredths (n x m) with per-bin base depth, cluster offsets,
    per-sample scale, CNVs and gamma noise."""
    base = rng.gamma(20.0, 1.5, size=m)
    clus = rng.integers(0, n_clusters, size=n)
    offs = 1.0 + rng.uniform(-0.08, 0.08, size=(n_clusters, m))
    scale = rng.uniform(0.6, 1.4, size=n)
    cnv = np.ones((n, m))
    hit = rng.random((n, m)) < 0.02
    cnv[hit] = rng.choice([0.5, 1.5], size=hit.sum())
    lam = base[None, :] * offs[clus] * scale[:, None] * cnv
    noise = rng.gamma(40.0, 1.0 / 40.0, size=(n, m))
    q = np.maximum(0, np.rint(lam * noise * 100)).astype(np.int64)
    starts = start0 + np.arange(m) * bin_size
    return q, starts, clus


def write_bed(path, chrom_rows):
    with gzip.open(path, "wt") as f:
        for chrom, s, e, q in chrom_rows:
            f.write(f"{chrom}\t{s}\t{e}\t{q // 100}.{q % 100:02d}\n")


def make_file_cohort(root: Path, rng, n, m, chrom, window=None, decoys=True,
                     bin_size=1000, start0=0, n_clusters=4):
    root.mkdir(parents=True, exist_ok=True)
    md = root / "mosdepth"
    md.mkdir(exist_ok=True)
    q, starts, clus = synth_cohort(rng, n, m, n_clusters, bin_size, start0)
    ids = [f"S{i:04d}" for i in range(n)]
    for i, sid in enumerate(ids):
        rows = []
        if decoys:
            # chr10 lines: start with "chr1" -> kept by the startswith filter
            # (reference quirk Q2); first 30 collide with chr1 coordinates
            # (last-wins, Q1), the rest are new coordinates.
            for b in range(30):
                rows.append(("chr10", int(starts[b]), int(starts[b] + bin_size), int(q[i, b] // 2 + 150)))
            for b in range(3):
                s = int(starts[-1] + (b + 5) * bin_size)
                rows.append(("chr10", s, s + bin_size, int(3000 + 7 * i + b)))
            rows.append(("chr2", 0, bin_size, 5000))
        for b in range(m):
            rows.append((chrom, int(starts[b]), int(starts[b] + bin_size), int(q[i, b])))
        # a malformed line (skipped by the reference: < 4 fields)
        rows_txt = rows
        name = f"{sid}_LPA.regions.bed.gz" if i % 3 else f"{sid}.regions.bed.gz"
        write_bed(md / name, rows_txt)
    # a stray file for a sample not in the list
    write_bed(md / "ZZ9999_LPA.regions.bed.gz", [(chrom, int(starts[0]), int(starts[0] + bin_size), 4000)])
    # sample list: all + one with no file
    (root / "samples.txt").write_text("\n".join(ids + ["S9998"]) + "\n")
    # repeat mask: a handful of intervals, chrom without 'chr' prefix for one
    lines = ["# repeat mask", ""]
    for b in rng.choice(m, size=max(1, m // 40), replace=False):
        s = int(starts[b]) + 200
        lines.append(f"{chrom}\t{s}\t{s + 300}\tAluY")
    lines.append(f"{chrom.replace('chr', '')}\t{int(starts[min(7, m-1)])}\t{int(starts[min(7, m-1)]) + 10}")
    lines.append("chrX\t1")
    (root / "mask.bed").write_text("\n".join(lines) + "\n")
    # read counts (count_reads format, header replaced by pandas names=)
    cnt = ["Sample\tchr6:1-2"]
    for i, sid in enumerate(ids):
        if i == 3:
            cnt.append(f"{sid}\tError")
            continue
        if i == 5:
            continue
        cn = rng.choice([1.0, 1.5, 2.0, 2.5])
        cnt.append(f"{sid}\t{int(rng.poisson(cn * 400 * (0.6 + (i % 7) * 0.1)))}")
    (root / "counts.tsv").write_text("\n".join(cnt) + "\n")
    # IBS (computeIBSpbwt) neighbours: header + ID hap nbrInd cMlen cMedge IDnbr hapNbr
    ibs = ["ID\thap\tnbrInd\tcMlen\tcMedge\tIDnbr\thapNbr"]
    for i, sid in enumerate(ids):
        same = [j for j in range(n) if clus[j] == clus[i]]
        for hap in (1, 2):
            k = int(rng.integers(0, 14))
            for t in range(k):
                j = int(rng.choice(same))
                ibs.append(f"{sid}\t{hap}\t{j}\t{rng.uniform(0.5, 9):.3f}\t0.1\t{ids[j]}\t{int(rng.integers(1, 3))}")
        if i % 9 == 0:
            ibs.append(f"{sid}\t3\t0\t1.0\t0.1\t{ids[0]}\t1")       # invalid hap
            ibs.append(f"{sid}\t1\t0\t1.0\t0.1\tNOPE\t1")           # unknown id
            ibs.append(f"{sid}\t1\t0\t1.0")                          # short line
    with gzip.open(root / "ibs.tsv.gz", "wt") as f:
        f.write("\n".join(ibs) + "\n")
    # IBD (iLASH): FID1 HAP_ID1 FID2 HAP_ID2 CHR BP1 BP2 SNP_BP1 SNP_BP2 LENGTH MATCH
    ibd = []
    for t in range(n * 8):
        i, j = int(rng.integers(0, n)), int(rng.integers(0, n))
        h1, h2 = int(rng.integers(0, 2)), int(rng.integers(0, 2))
        bp1 = int(rng.integers(0, 4_000_000))
        bp2 = bp1 + int(rng.integers(1000, 3_000_000))
        ibd.append(f"{ids[i]}\t{ids[i]}_{h1}\t{ids[j]}\t{ids[j]}_{h2}\t6\t{bp1}\t{bp2}\t{bp1}\t{bp2}"
                   f"\t{rng.uniform(0.2, 12):.4f}\t{rng.uniform(0.5, 1.0):.3f}")
    (root / "ibd.txt").write_text("\n".join(ibd) + "\n")
    cfg = {
        "samples_file": str(root / "samples.txt"),
        "output_dir": str(root / "out"),
        "threads": 1,
        "chrom": chrom,
        "output_file_type": "tsv",
        "index": {"run": False},
        "count_reads": {"run": False, "output_file_prefix": "counts"},
        "mosdepth": {
            "run": False,
            "work_dir": str(md),
            "remove_intermediate": False,
            "normalize": {"run": True, "min_depth": 20, "max_depth": 100, "top_frac": 0.1,
                          "output_file_prefix": "normalized", "repeat_mask_file": str(root / "mask.bed")},
            "neighbors": {"run": True, "output_file_prefix": "neighbors", "num_neighbors": 5,
                          "zmax": 2.0, "sigma2_max": 1000},
        },
        "compute_diploid_genotypes": {"run": True, "output_file_prefix": "dipcn", "n_nbr": 4},
        "compute_haploid_genotypes": {"run": True, "output_file_prefix": "haploid", "method": "ibs",
                                      "min_neighbors": 1, "max_neighbors": 10, "n_iters": 100,
                                      "ibs_output": str(root / "ibs.tsv.gz")},
    }
    if window:
        cfg["start_bp"], cfg["end_bp"] = window
    return cfg


def inputs_digest(root: Path) -> str:
    """sha256 over the decompressed content of every input file of a cohort
    (gzip headers carry mtimes, so the compressed bytes differ run to run)."""
    h = hashlib.sha256()
    for p in sorted(Path(root).rglob("*")):
        if not p.is_file() or "out" in p.relative_to(root).parts:
            continue
        h.update(str(p.relative_to(root)).encode())
        data = p.read_bytes()
        h.update(gzip.decompress(data) if p.suffix == ".gz" else data)
    return h.hexdigest()


def regenerate(name: str, root: Path, golden: Path | None = None):
    """Rebuild a hashed golden cohort (g_cfg1) under ``root`` from its
    recorded seed; returns (config with absolute paths, cohort.json).  Fails
    if the regenerated inputs differ from the ones the reference was run on."""
    import json
    import shutil

    import yaml
    golden = Path(golden or Path(__file__).resolve().parent) / name
    meta = json.loads((golden / "cohort.json").read_text())
    root = Path(root)
    make_file_cohort(root, np.random.default_rng(meta["seed"]), meta["n"], meta["m"], meta["chrom"],
                     decoys=meta["decoys"])
    assert inputs_digest(root) == meta["inputs_sha256"], "regenerated cohort differs from the golden inputs"
    out = root / "out"
    out.mkdir(exist_ok=True)
    shutil.copy(golden / "expected" / "counts.tsv", out / "counts.tsv")

    def absolute(c):
        c["samples_file"] = str(root / c["samples_file"])
        c["output_dir"] = str(out)
        c["mosdepth"]["work_dir"] = str(root / c["mosdepth"]["work_dir"])
        c["mosdepth"]["normalize"]["repeat_mask_file"] = str(root / c["mosdepth"]["normalize"]["repeat_mask_file"])
        hc = c["compute_haploid_genotypes"]
        for k in ("ibs_output", "ibd_output"):
            if k in hc:
                hc[k] = str(root / hc[k])
        return c
    cfg = absolute(yaml.safe_load((golden / "config.yaml").read_text()))
    cfg_ibd = absolute(yaml.safe_load((golden / "config_ibd.yaml").read_text()))
    return cfg, cfg_ibd, meta


def check_outputs(name: str, out: Path, golden: Path | None = None, ibd: bool = True, only=None):
    """The step outputs in ``out`` against the golden: small files byte for
    byte (after gunzip), the normalised matrix by its sha256."""
    import json
    golden = Path(golden or Path(__file__).resolve().parent) / name
    meta = json.loads((golden / "cohort.json").read_text())

    def content(p):
        data = Path(p).read_bytes()
        return gzip.decompress(data) if str(p).endswith(".gz") else data
    text = content(Path(out) / "normalized.tsv.gz")
    assert len(text) == meta["normalized_bytes"] and text[:2000].decode() == meta["normalized_head"]
    assert hashlib.sha256(text).hexdigest() == meta["normalized_sha256"], "normalized.tsv.gz"
    files = ["neighbors.zMax2.0.tsv.gz", "dipcn.tsv", "haploid.tsv"] + (["haploid_ibd.tsv"] if ibd else [])
    if only is not None:
        files = [f for f in files if f in only]
    for f in files:
        assert content(Path(out) / f) == content(golden / "expected" / f), f
