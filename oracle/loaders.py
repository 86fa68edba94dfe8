"""Restatement of the step 6/7 text loaders (TEST INFRASTRUCTURE ONLY).

grid/utils/compute_dipcn.py load_neighbors :105-152 and counts read :46-49;
grid/utils/hi_inference.py _read_dip_cn_file :10-31, _load_ibs_neighbors
:34-74, _segment_distance :77-83, _load_ibd_neighbors :86-172.
"""
from __future__ import annotations

import gzip
from collections import defaultdict


def _open(path, mode="rt"):
    return gzip.open(path, mode) if str(path).endswith(".gz") else open(path, mode)


def load_neighbors(path):
    nb, sc = {}, {}
    with gzip.open(path, "rt") as f:
        for line in f:
            p = line.strip().split("\t")
            if len(p) < 2:
                continue
            try:
                s = float(p[1])
            except ValueError:
                continue
            sc[p[0]] = s
            lst, i = [], 2
            while i + 2 <= len(p):
                try:
                    lst.append((p[i], float(p[i + 1])))
                except ValueError:
                    pass
                i += 3
            nb[p[0]] = lst
    return nb, sc


def read_counts(path):
    import pandas as pd
    r = pd.read_csv(path, sep="\t", header=0, names=["Sample", "Reads"])
    r["Reads"] = pd.to_numeric(r["Reads"], errors="coerce")
    r.dropna(subset=["Reads"], inplace=True)
    return r.set_index("Sample")["Reads"].to_dict()


def read_dipcn(path):
    ids, irr, idx = [], [], {}
    with _open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            p = line.split()
            if len(p) < 2:
                continue
            try:
                v = float(p[1])
            except ValueError:
                continue
            idx[p[0]] = len(irr)
            ids.append(p[0])
            irr.append(v)
    return ids, irr, idx


def load_ibs(path, idx, max_nbr):
    hn = [[] for _ in range(2 * len(idx))]
    with _open(path) as f:
        next(f)
        for line in f:
            line = line.strip()
            if not line:
                continue
            p = line.split()
            if len(p) < 7:
                continue
            try:
                hap, hn2 = int(p[1]), int(p[6])
            except ValueError:
                continue
            if hap not in (1, 2) or hn2 not in (1, 2):
                continue
            i, j = idx.get(p[0]), idx.get(p[5])
            if i is not None and j is not None:
                h = 2 * i + hap - 1
                if len(hn[h]) < max_nbr:
                    hn[h].append((2 * j + hn2 - 1, 1.0))
    return hn


def seg_dist(bp1, bp2, rs, re_):
    if bp2 < rs:
        return float(rs - bp2)
    if bp1 > re_:
        return float(bp1 - re_)
    return 0.0


def load_ibd(path, idx, max_nbr, rs, re_, min_length=0.5, min_match=0.70, weighted=False,
             weight_scale=1_000_000):
    raw = defaultdict(list)
    with _open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            p = line.split("\t")
            if len(p) < 11:
                p = line.split()
            if len(p) < 11:
                continue
            try:
                bp1, bp2, ln, mt = int(p[5]), int(p[6]), float(p[9]), float(p[10])
            except (ValueError, IndexError):
                continue
            if ln < min_length or mt < min_match:
                continue
            try:
                h1 = int(p[1].rsplit("_", 1)[-1])
                h2 = int(p[3].rsplit("_", 1)[-1])
            except ValueError:
                continue
            if h1 not in (0, 1) or h2 not in (0, 1):
                continue
            i, j = idx.get(p[0]), idx.get(p[2])
            if i is None or j is None:
                continue
            w = (weight_scale / (seg_dist(bp1, bp2, rs, re_) + weight_scale)) * mt if weighted else 1.0
            raw[2 * i + h1].append((2 * j + h2, w, ln))
            raw[2 * j + h2].append((2 * i + h1, w, ln))
    hn = [[] for _ in range(2 * len(idx))]
    for h, segs in raw.items():
        segs.sort(key=lambda x: -x[2])
        hn[h] = [(nb, w) for nb, w, _ in segs[:max_nbr]]
    return hn
