"""Restatement of the step-4 file ingest (TEST INFRASTRUCTURE ONLY).

Follows grid/utils/normalize_mosdepth.py: map_mosdepth_files_to_samples
:148-174, load_repeat_mask :177-207, norm_chrom :210-215,
compute_population_mean_depths :218-301 (threads=1 order), process_one_individual
:304-357, build_matrix_from_regions :379-416, find_bed_gz_for_individual
:557-573, filter_empty_samples :576-600.
"""
from __future__ import annotations

import gzip
from collections import defaultdict
from pathlib import Path

import numpy as np


def norm_chrom(c):
    return c if c.startswith("chr") else f"chr{c}"


def map_files(work_dir, samples):
    d = Path(work_dir)
    ss = set(samples)
    res = {}
    for f in d.glob("*.regions.bed.gz"):
        parts = f.name.split(".")[0].split("_")
        for i in range(len(parts), 0, -1):
            c = "_".join(parts[:i])
            if c in ss:
                res[c] = f
                break
    return res


def find_bed(ind, work_dir):
    d = Path(work_dir)
    m = list(d.glob(f"*{ind}*regions.bed.gz"))
    return m[0] if m else d / f"{ind}.regions.bed.gz"


def load_mask(path):
    ex = defaultdict(set)
    with open(path) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            p = line.strip().split()
            if len(p) < 3:
                continue
            try:
                s, e = int(p[1]), int(p[2])
            except ValueError:
                continue
            for kb in range(s // 1000, e // 1000 + 1):
                ex[norm_chrom(p[0])].add(kb)
    return ex


def _records(path, chrom, start, end, excluded):
    cm = norm_chrom(chrom) if chrom else None
    with gzip.open(path, "rt") as f:
        for line in f:
            if cm and not line.startswith(cm):
                continue
            fl = line.strip().split("\t")
            if len(fl) < 4:
                continue
            c = norm_chrom(fl[0])
            s, e, d = int(fl[1]), int(fl[2]), float(fl[3])
            if start is not None and end is not None:
                if not (d > 0 and e >= start and s <= end):
                    continue
            elif d <= 0:
                continue
            if set(range(s // 1000, e // 1000 + 1)) & excluded.get(c, set()):
                continue
            yield s, e, d


def ingest(work_dir, samples, chrom, start, end, mask_path, min_depth, max_depth):
    inds = map_files(work_dir, samples)
    ex = load_mask(mask_path) if mask_path else {}
    sums, cnts = defaultdict(float), defaultdict(int)
    for ind in inds:
        p = find_bed(ind, work_dir)
        if not p.exists():
            continue
        local = {}
        for s, e, d in _records(p, chrom, start, end, ex):
            local[(s, e)] = d
        for r, d in local.items():
            sums[r] += d
            cnts[r] += 1
    pop = {r: sums[r] / cnts[r] for r in sums if cnts[r] > 0}
    valid = {r for r, m in pop.items() if min_depth <= m <= max_depth}
    per = {}
    for ind in inds:
        p = find_bed(ind, work_dir)
        res = []
        if p.exists():
            for s, e, d in _records(p, chrom, start, end, ex):
                if (s, e) in valid:
                    res.append((s, e, d))
        per[ind] = res
    per = {k: v for k, v in per.items() if v}
    order = sorted(per)
    regions = sorted({(s, e) for k in order for s, e, _ in per[k]})
    ri = {r: j for j, r in enumerate(regions)}
    mat = np.full((len(order), len(regions)), np.nan)
    for i, k in enumerate(order):
        for s, e, d in per[k]:
            mat[i, ri[(s, e)]] = d
    return order, regions, mat
