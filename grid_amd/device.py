"""Per-process device selection for the step modules.

The YAML may carry an optional ``gpu: {device: N}`` section (ignored by the
reference, which does not read unknown keys); LOCAL_RANK wins under a
multi-process launcher.  There is no CPU fallback.
"""
from __future__ import annotations

import os

from ._abi import Device

_dev = {}


def get_device(config=None) -> Device:
    idx = int(os.environ.get("LOCAL_RANK", (config or {}).get("gpu", {}).get("device", 0) if config else 0))
    d = _dev.get(idx)
    if d is None:
        d = Device(idx)
        _dev[idx] = d
    return d
