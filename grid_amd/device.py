"""Per-process device selection for the step modules.

The YAML may carry an optional ``gpu: {device: N}`` section (ignored by the
reference, which does not read unknown keys); LOCAL_RANK wins under a
multi-process launcher.  There is no CPU fallback.
"""
from __future__ import annotations

import contextlib
import os

from ._abi import Device

_dev = {}
_defer = 0


def release_ingest_buffers(*devs):
    """Free what the device ingest keeps between its batches and ingests: the
    device input / text buffers cached on the step contexts (get_device) and
    on ``devs`` (Device.cached, names "ingest_*"), and the host staging
    (ingest_device._STAGING).  Returns (device bytes, host bytes) released."""
    from .utils import ingest_device
    ds = {id(d): d for d in list(_dev.values()) + list(devs) if getattr(d, "ctx", None)}
    dbytes = sum(d.release_cached("ingest_") for d in ds.values())
    return dbytes, ingest_device.release_staging()


def step4_done(dev=None):
    """End of step 4: its ingest buffers go now, unless a pipeline run (or a
    benchmark) holds them to the end (``deferred_release``) -- their release
    holds the HIP runtime for a fraction of a second -- and even
    then when less than a quarter of the device's HBM is free (a smaller GPU:
    step 5's Gram needs it more than the next run needs the buffers)."""
    if not _defer:
        release_ingest_buffers(*([dev] if dev is not None else []))
        return
    if dev is not None:
        free, total = dev.mem_info()
        if free < total // 4:
            release_ingest_buffers(dev)


@contextlib.contextmanager
def deferred_release(release=True):
    """Keep the ingest buffers until the outermost such block ends (the end of
    ``run_wgs_pipeline``), then release them -- or, with release=False, keep
    them cached for the process's next run (a service running the pipeline
    again on a cohort of the same shape; bench.py's timed runs): HBM is then
    held until the next release or the process's end."""
    global _defer
    _defer += 1
    try:
        yield
    finally:
        _defer -= 1
        if not _defer and release:
            release_ingest_buffers()


def get_device(config=None) -> Device:
    idx = int(os.environ.get("LOCAL_RANK", (config or {}).get("gpu", {}).get("device", 0) if config else 0))
    if os.environ.get("GRID_SHARE_GPU") == "1":
        # rehearsal only: the ranks of a gloo job share the visible GPUs round-robin
        from ._abi import device_count
        idx %= max(device_count(), 1)
    d = _dev.get(idx)
    if d is None:
        d = Device(idx)
        _dev[idx] = d
    return d
