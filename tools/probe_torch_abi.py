"""Probe: libgridhip.so shares torch's HIP runtime (pointers + streams)."""
import numpy as np
import torch
from grid_amd import _abi, engine

print("torch", torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))
dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
q = torch.randint(1, 9000, (64, 20000), dtype=torch.int32, device="cuda")
st = engine.normalize_stats(dev, q, 64, 20000, 20000)
dev.sync()
rm = st.rowmean.numpy()
ref = (q.double().cpu().numpy() / 100.0)
from oracle.npsum import nanmean_rows
print("rowmean exact via torch pointer:", np.array_equal(rm, nanmean_rows(ref)))
import os
maps = open("/proc/self/maps").read()
print("hip runtimes loaded:", sorted({l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}))
