"""Step 4 -> step 5 hand-off inside one `grid wgs` process.

The reference's find_neighbors re-reads the normalised matrix that
normalize_mosdepth wrote moments earlier (find_neighbors.py:81-124: gunzip
and parse of every "%.2f" cell; 15.6 GB of gzip at BASELINE config 2).  When
both steps run in the same process, step 4 publishes what step 5 would parse
from that file -- the sample ids, the row scales and the "%.3f" ratios as the
text prints them, and the int32 z hundredths still on the device -- keyed by
the file's resolved path, size and mtime.  Step 5 takes the entry only while
the file on disk is still exactly the one step 4 wrote; any other file (a
separate run, a file edited or replaced in between) is read and parsed as
before.  The file itself is always written: it is the step contract.
"""
from __future__ import annotations

import os

_entries: dict = {}


def _stamp(path):
    st = os.stat(path)
    return st.st_size, st.st_mtime_ns


def publish(path, ids, scales, ratios, zq_dev, shape):
    """Record step 4's output for ``path`` (call after the file is closed).
    scales / ratios: the values the text holds ("%.2f" / "%.3f" read back),
    zq_dev: device int32 hundredths [n][r] (GRID_ZQ_NAN = "NA", GRID_ZQ_NEG0 =
    "-0.00": the k-NN gathers read both as zero, find_neighbors.py:57-58)."""
    _entries.clear()                       # one matrix at a time: it holds device memory
    _entries[os.path.realpath(path)] = (_stamp(path), list(ids), scales, ratios, zq_dev, shape)


def take(path):
    """(ids, scales array, ratios array, zq device buffer, (n, r)) when ``path``
    is still the file step 4 published, else None.  The entry is consumed."""
    key = os.path.realpath(path)
    ent = _entries.pop(key, None)
    if ent is None:
        return None
    try:
        if _stamp(path) != ent[0]:
            return None
    except OSError:
        return None
    return ent[1:]


def publish_neighbors(path, rec):
    """The distributed step 4 (dist_step4.py) ran step 5's search as well:
    record the sample ids, the "%.2f" scales and the neighbour lists (every
    rank holds them) for ``path`` -- call on every rank once the file is
    complete.  rec["neighbors"] is None when step 5 was not run there."""
    _entries.pop(("nbr", os.path.realpath(path)), None)
    _entries[("nbr", os.path.realpath(path))] = (_stamp(path), rec)


def take_neighbors(path, params):
    """The record published for ``path`` when the file is unchanged and its
    search used ``params`` (zmax, sigma2_max, frac_r, n_neighbors), else None.
    The entry is consumed."""
    ent = _entries.pop(("nbr", os.path.realpath(path)), None)
    if ent is None:
        return None
    try:
        if _stamp(path) != ent[0]:
            return None
    except OSError:
        return None
    rec = ent[1]
    nb = rec.get("neighbors")
    if nb is None or nb["params"] != params:
        return None
    return rec


def clear():
    _entries.clear()
