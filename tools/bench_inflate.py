"""Device gzip inflate throughput (grid_gunzip_batch) on synthetic mosdepth
files (tools/gen_cohort: the bench cohort as regions.bed.gz, 1 kb bins, zlib
level 1; or --bgzf: each file re-packed as BGZF, what mosdepth writes).

    python tools/bench_inflate.py [--files 256] [--bins 3000000] [--bgzf] [--json out.json]
"""
import argparse
import gzip
import json
import os
import struct
import subprocess
import sys
import time
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from grid_amd import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--files", type=int, default=256)
ap.add_argument("--bins", type=int, default=3_000_000)
ap.add_argument("--distinct", type=int, default=16, help="distinct files generated (the rest repeat them)")
ap.add_argument("--bgzf", action="store_true")
ap.add_argument("--units", action="store_true", help="BGZF: one wave per member (the ingest's launch)")
ap.add_argument("--dir", default="/tmp/grid_inflate_bench")
ap.add_argument("--json", default="")
a = ap.parse_args()


def bgzf(data, block=65280):
    o = bytearray()
    for s in range(0, len(data), block):
        ch = data[s:s + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        body = c.compress(ch) + c.flush()
        o += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<H", 6) + b"BC"
        o += struct.pack("<HH", 2, 12 + 6 + len(body) + 8 - 1) + body + struct.pack("<II", zlib.crc32(ch), len(ch))
    return bytes(o) + bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


os.makedirs(a.dir, exist_ok=True)
gen = os.path.join(ROOT, "tools", "gen_cohort")
if not os.path.exists(gen):
    subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", "-o", gen, gen + ".cpp", "-lz"], check=True)
t0 = time.perf_counter()
subprocess.run([gen, a.dir, str(a.distinct), str(a.bins), "20260821", "16", "0"], check=True)
names = sorted(f for f in os.listdir(a.dir) if f.endswith(".regions.bed.gz"))[: a.distinct]
blobs = [open(os.path.join(a.dir, f), "rb").read() for f in names]
texts = [gzip.decompress(b) for b in blobs[:2]]
if a.bgzf:
    blobs = [bgzf(gzip.decompress(b)) for b in blobs]
gen_s = time.perf_counter() - t0
files = [blobs[i % len(blobs)] for i in range(a.files)]
caps = [struct.unpack("<I", b[-4:])[0] if not a.bgzf else len(gzip.decompress(b)) for b in blobs]
caps = [caps[i % len(blobs)] for i in range(a.files)]
dev = _abi.Device(0)
dev.set_stream(torch.cuda.current_stream())
res = []
if a.units:
    # every member its own stream, text back to back per file (ingest_device.inflate)
    assert a.bgzf
    io, il, oo, oc, fo = [], [], [], [], []
    pos = opos = 0
    for b in files:
        ms, ml, mi = _abi.gz_members(b)
        cum = np.zeros(len(mi), np.int64)
        np.cumsum(mi[:-1], out=cum[1:])
        io.append(pos + ms)
        il.append(ml)
        oo.append(opos + cum)
        oc.append(mi.astype(np.int64))
        fo.append(opos)
        pos += -(-len(b) // 256) * 256
        opos += -(-int(mi.sum()) // 256) * 256
    io, il, oo, oc = (np.concatenate(x) for x in (io, il, oo, oc))
    src = np.zeros(pos + 256, np.uint8)
    p = 0
    for b in files:
        src[p:p + len(b)] = np.frombuffer(b, np.uint8)
        p += -(-len(b) // 256) * 256
    d_src = dev.upload(src)
    d = [dev.upload(x) for x in (io, il, oo, oc)]
    nu = len(io)
    out = dev.alloc(opos + 256, np.uint8)
    mem = dev.alloc(nu * _abi.GZ_MEMBER_BYTES, np.uint8)
    st_d, ln_d, nm_d = dev.alloc(nu, np.int32), dev.alloc(nu, np.int64), dev.alloc(nu, np.int32)
    for rep in range(3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        _abi.call("grid_gunzip_batch", dev.ctx, d_src.ptr, d[0].ptr, d[1].ptr, nu, out.ptr, d[2].ptr, d[3].ptr,
                  mem.ptr, 1, st_d.ptr, ln_d.ptr, nm_d.ptr)
        torch.cuda.synchronize()
        res.append(time.perf_counter() - t1)
    ust, uln = st_d.numpy(), ln_d.numpy()
    assert (ust == 0).all(), np.unique(ust, return_counts=True)
    owner = np.concatenate([np.full(len(_abi.gz_members(b)[0]), f) for f, b in enumerate(files)])
    ln = np.bincount(owner, weights=uln, minlength=len(files)).astype(np.int64)
    st = np.zeros(len(files), np.int32)
    nm = np.bincount(owner, minlength=len(files))
    off = np.array(fo, np.int64)
else:
    for rep in range(3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        st, ln, nm, out, off = _abi.gunzip_batch(dev, files, caps)
        torch.cuda.synchronize()
        res.append(time.perf_counter() - t1)
for f in range(min(2, a.files)):
    assert st[f] == 0, st[f]
    host = np.empty(int(ln[f]), dtype=np.uint8)
    _abi.call("grid_d2h", dev.ctx, host.ctypes.data, out.ptr + int(off[f]), host.nbytes)
    assert host.tobytes() == texts[f]
assert (st == 0).all(), np.unique(st, return_counts=True)
tot_in, tot_out = sum(len(b) for b in files), int(ln.sum())
r = {"files": a.files, "bins": a.bins, "bgzf": a.bgzf, "units": a.units, "compressed_gb": tot_in / 1e9, "text_gb": tot_out / 1e9,
     "members_per_file": int(nm[0]), "seconds": min(res), "text_gbs": tot_out / min(res) / 1e9,
     "files_per_s": a.files / min(res),
     "note": "the CRC check included; the H2D copy of the compressed bytes too, except with --units"}
print(json.dumps(r), flush=True)
if a.json:
    open(a.json, "w").write(json.dumps(r) + "\n")
