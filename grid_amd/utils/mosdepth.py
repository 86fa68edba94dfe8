"""Only the cleanup helper step 4 calls (reference grid/utils/mosdepth.py
remove_intermediate_files :300-326).  Running mosdepth itself (step 3) is
out of scope."""
from __future__ import annotations

from pathlib import Path

from .utils import log


def remove_intermediate_files(work_dir, console=None, include_region_bed_gz: bool = False) -> None:
    suffixes = ["mosdepth.global.dist.txt", "mosdepth.region.dist.txt", "regions.bed.gz.csi"]
    if include_region_bed_gz:
        suffixes.append("regions.bed.gz")
    for f in Path(work_dir).glob("*"):
        if any(f.name.endswith(s) for s in suffixes):
            try:
                f.unlink()
            except Exception as e:
                log(console, f"Failed to remove intermediate file {f}: {e}", style="warning")
