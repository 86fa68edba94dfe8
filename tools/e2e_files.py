"""`grid wgs` from files at BASELINE config 2 (3,202 samples x 3 M bins):
steps 4-7 through the drop-in step API on a synthetic mosdepth cohort written
to disk, with per-phase wall times and the process's peak host RSS.

    python tools/e2e_files.py [--samples 3202] [--bins 3000000] [--data /dev/shm/grid_e2e]
                              [--out /tmp/grid_e2e_out] [--json gpurun_out/e2e.json]

The cohort (tools/gen_cohort, built here: g++ ... -lz) is the bench's depth
model as mosdepth text ("%.2f", 1 kb bins, gzip level 1); counts and the IBS
hap-neighbour file come from bench.synth_reads_and_ibs.  Phases are timed by
wrapping the step modules' own functions (no change to the product code).
"""
import argparse
import functools
import gzip
import json
import os
import resource
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--samples", type=int, default=3202)
ap.add_argument("--bins", type=int, default=3_000_000)
ap.add_argument("--data", default="/dev/shm/grid_e2e")
ap.add_argument("--out", default="/tmp/grid_e2e_out")
ap.add_argument("--threads", type=int, default=16, help="the config's `threads` (the reference defaults to 1, "
                "its example config uses 4)")
ap.add_argument("--gen-threads", type=int, default=16, help="threads of the cohort generator (outside the clock)")
ap.add_argument("--json", default=os.path.join(ROOT, "gpurun_out", "e2e_files.json"))
ap.add_argument("--keep", action="store_true", help="keep the generated cohort")
ap.add_argument("--bgzf", action="store_true", help="BGZF files (what mosdepth writes) instead of one gzip member")
ap.add_argument("--ingest", choices=["device", "host"], default="device",
                help="mosdepth.normalize.device_ingest true (the default: inflate + parse in HBM) or false")
ap.add_argument("--device-ingest", action="store_true", help=argparse.SUPPRESS)   # older spelling of --ingest device
ap.add_argument("--reuse", action="store_true", help="keep the cohort in --data for a later run (implies --keep)")
ap.add_argument("--generate-only", action="store_true", help="write the cohort and inputs into --data, then exit")
ap.add_argument("--verify-normalized", action="store_true",
                help="after the timed steps, read the step-4 file back and digest the parsed matrix")
a = ap.parse_args()


def note(msg):
    print(f"[e2e] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


res = {"config": {"samples": a.samples, "bins": a.bins, "data": a.data, "out": a.out, "bgzf": a.bgzf,
                  "device_ingest": a.ingest == "device", "threads": a.threads}, "phases_s": {},
       "peak_rss_gb_after": {}}
mos = os.path.join(a.data, "mosdepth")
os.makedirs(mos, exist_ok=True)
os.makedirs(a.out, exist_ok=True)
ids = [f"S{i:05d}" for i in range(a.samples)]

# ---- inputs --------------------------------------------------------------
t0 = time.perf_counter()
gen = os.path.join(ROOT, "tools", "gen_cohort")
if not os.path.exists(gen) or os.path.getmtime(gen) < os.path.getmtime(gen + ".cpp"):
    subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", "-o", gen, gen + ".cpp", "-lz", "-ldl"], check=True)
have = len([f for f in os.listdir(mos) if f.endswith(".regions.bed.gz")])
if have != a.samples:
    note(f"generating {a.samples} x {a.bins} mosdepth files in {mos}")
    # one call (the per-bin tables once); it prints a progress line per 200 files
    subprocess.run([gen, mos, str(a.samples), str(a.bins), "20260821", str(a.gen_threads), "0"]
                   + (["bgzf"] if a.bgzf else []), check=True)
res["phases_s"]["generate_cohort"] = time.perf_counter() - t0
res["cohort_bytes"] = sum(os.path.getsize(os.path.join(mos, f)) for f in os.listdir(mos))

import bench  # noqa: E402  (reads + IBS graph of the bench cohort)
reads, off, nbr, w = bench.synth_reads_and_ibs(a.samples)
with open(os.path.join(a.data, "samples.txt"), "w") as f:
    f.write("\n".join(ids) + "\n")
with open(os.path.join(a.out, "counts.tsv"), "w") as f:
    f.write("Sample\tchr1:1-3000000000\n")
    f.writelines(f"{ids[i]}\t{int(reads[i])}\n" for i in range(a.samples))
with gzip.open(os.path.join(a.data, "ibs.tsv.gz"), "wt", compresslevel=1) as f:
    f.write("ID\thap\tnbrInd\tcMlen\tcMedge\tIDnbr\thapNbr\n")
    for h in range(2 * a.samples):
        for t in range(off[h], off[h + 1]):
            j = int(nbr[t])
            f.write(f"{ids[h // 2]}\t{h % 2 + 1}\t{t - off[h]}\t5.0\t0\t{ids[j // 2]}\t{j % 2 + 1}\n")
open(os.path.join(a.data, "mask.bed"), "w").close()
cfg = {
    "samples_file": os.path.join(a.data, "samples.txt"), "output_dir": a.out, "threads": a.threads,
    "chrom": "chr1", "output_file_type": "tsv", "index": {"run": False},
    "count_reads": {"run": False, "output_file_prefix": "counts"},
    "mosdepth": {"run": False, "work_dir": mos, "remove_intermediate": False,
                 "normalize": {"run": True, "min_depth": 20, "max_depth": 100, "top_frac": 0.1,
                               "device_ingest": a.ingest == "device",
                               "output_file_prefix": "normalized",
                               "repeat_mask_file": os.path.join(a.data, "mask.bed")},
                 "neighbors": {"run": True, "output_file_prefix": "neighbors", "num_neighbors": 10, "zmax": 2.0,
                               "sigma2_max": 1000}},
    "compute_diploid_genotypes": {"run": True, "output_file_prefix": "dipcn", "n_nbr": 10},
    "compute_haploid_genotypes": {"run": True, "output_file_prefix": "haploid", "method": "ibs",
                                  "min_neighbors": 1, "max_neighbors": 10, "n_iters": 100,
                                  "ibs_output": os.path.join(a.data, "ibs.tsv.gz")},
}
res["phases_s"]["write_inputs"] = time.perf_counter() - t0 - res["phases_s"]["generate_cohort"]
if a.generate_only:
    note("cohort written")
    sys.exit(0)

# ---- timed steps ---------------------------------------------------------
from grid_amd import engine  # noqa: E402
from grid_amd.utils import compute_dipcn as cd  # noqa: E402
from grid_amd.utils import find_neighbors as fn  # noqa: E402
from grid_amd.utils import hi_inference as hi  # noqa: E402
from grid_amd.utils import normalize_mosdepth as nm  # noqa: E402


def timed(mod, name, key):
    fun = getattr(mod, name)

    @functools.wraps(fun)
    def wrap(*args, **kw):
        t = time.perf_counter()
        try:
            return fun(*args, **kw)
        finally:
            res["phases_s"][key] = res["phases_s"].get(key, 0.0) + time.perf_counter() - t
            note(f"  {key}: {res['phases_s'][key]:.1f} s, peak RSS {rss_gb():.1f} GB")
    setattr(mod, name, wrap)


timed(nm, "ingest", "step4_ingest")
timed(nm, "_write_normalized_q", "step4_write_text")
timed(engine, "normalize_stats", "step4_device_stats")
timed(engine, "zquant", "step4_device_zquant")
timed(fn, "_read_normalized_q", "step5_read_text")
timed(engine, "knn_from_zq", "step5_knn")
timed(fn, "save_neighbors", "step5_write")

from grid_amd.device import deferred_release  # noqa: E402

# as run_wgs_pipeline does: step 4's ingest buffers are kept to the end of the
# run, then released -- that release is timed on its own, after steps 4-7
with deferred_release():
    for step, fun in (("step4", lambda: nm.normalize_mosdepth(cfg, None)),
                      ("step5", lambda: fn.find_neighbors(cfg, None)),
                      ("step6", lambda: cd.compute_diploid_genotypes(cfg, None)),
                      ("step7", lambda: hi.hi_inference(cfg, None))):
        note(f"{step} ...")
        t = time.perf_counter()
        fun()
        res["phases_s"][step + "_total"] = time.perf_counter() - t
        res["peak_rss_gb_after"][step] = rss_gb()
        note(f"{step} done in {res['phases_s'][step + '_total']:.1f} s, peak RSS {rss_gb():.1f} GB")
    t_rel = time.perf_counter()
res["phases_s"]["release_ingest_buffers_after_step7"] = time.perf_counter() - t_rel

res["outputs"] = {f: os.path.getsize(os.path.join(a.out, f)) for f in sorted(os.listdir(a.out))}
if a.verify_normalized:
    # outside the timed steps: the step-4 file read back by the library's reader
    # (every member inflated and its CRC-32 -- computed on the device from the
    # text before compression -- checked), and a digest of the parsed matrix
    # that runs with other writers can be compared on
    from grid_amd import _abi  # noqa: E402
    import numpy as np  # noqa: E402
    t = time.perf_counter()
    nf = [f for f in os.listdir(a.out) if f.startswith("normalized")][0]
    rid, rsc, rmu, rrat, rzq = _abi.read_normalized_gz(os.path.join(a.out, nf), threads=16)
    t_read = time.perf_counter() - t
    import xxhash  # noqa: E402
    res["normalized_readback"] = {"file": nf, "seconds": t_read, "rows": int(rzq.shape[0]), "cols": int(rzq.shape[1]),
                                  "ids_ok": rid == ids, "zq_xxh3_64": xxhash.xxh3_64(np.ascontiguousarray(rzq)).hexdigest()}
    del rzq
    note(f"normalized file read back in {t_read:.1f} s")
try:                                    # content digests (outside the timed steps): runs compare byte for byte
    import xxhash

    def digest(path):
        # a small .gz (Python's gzip.open, as the reference's writers) carries
        # its write time in the header: digest its text; the device writer's
        # large file has MTIME 0: its bytes
        h = xxhash.xxh3_64()
        small_gz = path.endswith(".gz") and os.path.getsize(path) < (64 << 20)
        with (gzip.open(path, "rb") if small_gz else open(path, "rb")) as fh:
            for blk in iter(lambda: fh.read(1 << 26), b""):
                h.update(blk)
        return h.hexdigest()
    t = time.perf_counter()
    res["outputs_xxh3_64"] = {f: digest(os.path.join(a.out, f)) for f in sorted(os.listdir(a.out))}
    res["phases_s"]["digest_outputs"] = time.perf_counter() - t
except ImportError:
    pass
res["steps_4_7_s"] = sum(res["phases_s"][s + "_total"] for s in ("step4", "step5", "step6", "step7"))
res["samples_per_s_from_files"] = a.samples / res["steps_4_7_s"]
os.makedirs(os.path.dirname(a.json), exist_ok=True)
json.dump(res, open(a.json, "w"), indent=1)
print(json.dumps(res), flush=True)
import shutil  # noqa: E402  (no child process once the GPU is in use)
if not (a.keep or a.reuse):
    shutil.rmtree(a.data, ignore_errors=True)
    shutil.rmtree(a.out, ignore_errors=True)
elif a.reuse:
    shutil.rmtree(a.out, ignore_errors=True)
