"""the CPU baseline as a sweep and per-stage fits.

The oracle's steps 4-7 from files (oracle/pipeline.py: the reference's
step functions restated -- mosdepth gzip parse, normalize_matrix, "%.2f" text
into gzip level 9, re-read, exact k-NN, dipCN, phasing) on synthetic mosdepth
cohorts of N samples x M bins, N in {100, 400, 1600} x M in {30k, 100k}, each
point in its own single-threaded process (OMP/BLAS threads = 1: the reference
runs its parse pool GIL-bound, threads = 1 by default), several points at a
time.  Then per-stage models fitted through the origin:

    ingest, normalize, write_normalized, read_normalized  ~ a * N * M
    knn                                                   ~ a * N^2 * R_use
    write_neighbors, dipcn, load_hap_neighbors, phasing, write_haploid ~ a * N

and the fitted total extrapolated to BASELINE configs 2 (3,202 x 3 M) and 3
(50 k x 3 M).  ONE JSON document on stdout (and --json).

    python tools/cpu_sweep.py [--points 100x30000,...] [--workers 6] [--data /dev/shm/grid_sweep]
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIN_CELLS = ("ingest", "normalize", "write_normalized", "read_normalized")
LIN_N = ("write_neighbors", "dipcn", "load_hap_neighbors", "phasing", "write_haploid")


def one_point(n, m, data, seed=20260821):
    """Generate the cohort, run the oracle from files, return its stage times."""
    import gzip
    import shutil
    sys.path.insert(0, ROOT)
    import bench
    from oracle import pipeline
    root = os.path.join(data, f"p{n}x{m}")
    mos, out = os.path.join(root, "mosdepth"), os.path.join(root, "out")
    os.makedirs(mos, exist_ok=True)
    os.makedirs(out, exist_ok=True)
    gen = os.path.join(ROOT, "tools", "gen_cohort")
    t0 = time.perf_counter()
    subprocess.run([gen, mos, str(n), str(m), str(seed), "2", "0", "bgzf"], check=True, stderr=subprocess.DEVNULL)
    ids = [f"S{i:05d}" for i in range(n)]
    reads, off, nbr, _ = bench.synth_reads_and_ibs(n, seed)
    with open(os.path.join(root, "samples.txt"), "w") as f:
        f.write("\n".join(ids) + "\n")
    with open(os.path.join(out, "counts.tsv"), "w") as f:
        f.write("Sample\tchr1:1-3000000000\n")
        f.writelines(f"{ids[i]}\t{int(reads[i])}\n" for i in range(n))
    with gzip.open(os.path.join(root, "ibs.tsv.gz"), "wt", compresslevel=1) as f:
        f.write("ID\thap\tnbrInd\tcMlen\tcMedge\tIDnbr\thapNbr\n")
        for h in range(2 * n):
            for t in range(off[h], off[h + 1]):
                j = int(nbr[t])
                f.write(f"{ids[h // 2]}\t{h % 2 + 1}\t{t - off[h]}\t5.0\t0\t{ids[j // 2]}\t{j % 2 + 1}\n")
    open(os.path.join(root, "mask.bed"), "w").close()
    gen_s = time.perf_counter() - t0
    cfg = {"samples_file": os.path.join(root, "samples.txt"), "output_dir": out, "chrom": "chr1",
           "output_file_type": "tsv", "count_reads": {"output_file_prefix": "counts"},
           "mosdepth": {"work_dir": mos,
                        "normalize": {"min_depth": 20, "max_depth": 100, "top_frac": 0.1,
                                      "output_file_prefix": "normalized",
                                      "repeat_mask_file": os.path.join(root, "mask.bed")},
                        "neighbors": {"output_file_prefix": "neighbors", "num_neighbors": 10, "zmax": 2.0,
                                      "sigma2_max": 1000}},
           "compute_diploid_genotypes": {"output_file_prefix": "dipcn", "n_nbr": 10},
           "compute_haploid_genotypes": {"output_file_prefix": "haploid", "method": "ibs", "min_neighbors": 1,
                                         "max_neighbors": 10, "n_iters": 100,
                                         "ibs_output": os.path.join(root, "ibs.tsv.gz")}}
    try:
        t = pipeline.run(cfg)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    shape = t.pop("shape")
    return {"n": n, "m": m, "shape": shape, "stages_s": t, "total_s": sum(t.values()), "generate_s": gen_s}


def _child(n, m, data):
    print(json.dumps(one_point(n, m, data)), flush=True)


def fit(points):
    """Least squares through the origin per stage: seconds per unit."""
    units = {}
    for st in LIN_CELLS:
        units[st] = [(p["shape"]["n"] * p["m"], p["stages_s"][st]) for p in points]
    units["knn"] = [(p["shape"]["n"] ** 2 * p["shape"]["R_use"], p["stages_s"]["knn"]) for p in points]
    for st in LIN_N:
        units[st] = [(p["shape"]["n"], p["stages_s"][st]) for p in points]
    coef = {}
    for st, xy in units.items():
        sxx = sum(x * x for x, _ in xy)
        coef[st] = sum(x * y for x, y in xy) / sxx if sxx else 0.0
    # relative residual of the fitted total per point
    res = []
    for p in points:
        pred = predict(coef, p["shape"]["n"], p["m"], p["shape"]["R_use"])
        res.append({"n": p["n"], "m": p["m"], "measured_s": p["total_s"], "fitted_s": pred["total_s"]})
    return coef, res


def predict(coef, n, m, r_use):
    st = {s: coef[s] * n * m for s in LIN_CELLS}
    st["knn"] = coef["knn"] * n * n * r_use
    st.update({s: coef[s] * n for s in LIN_N})
    return {"stages_s": {k: round(v, 3) for k, v in st.items()}, "total_s": sum(st.values()),
            "samples_per_s": n / sum(st.values())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", default="100x30000,400x30000,1600x30000,100x100000,400x100000,1600x100000")
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--data", default="/dev/shm/grid_sweep")
    ap.add_argument("--json", default=None)
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:
        n, m = (int(x) for x in a.child.split("x"))
        _child(n, m, a.data)
        return
    gen = os.path.join(ROOT, "tools", "gen_cohort")
    if not os.path.exists(gen) or os.path.getmtime(gen) < os.path.getmtime(gen + ".cpp"):
        subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", "-o", gen, gen + ".cpp", "-lz", "-ldl"], check=True)
    pts = [tuple(int(x) for x in p.split("x")) for p in a.points.split(",")]
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    todo = sorted(pts, key=lambda p: -p[0] * p[1])           # largest first
    running, results, t0 = [], [], time.perf_counter()
    stop = threading.Event()

    def beat():                                              # progress for a watchdog
        while not stop.wait(60):
            print(f"[cpu_sweep] {time.perf_counter() - t0:.0f} s: {len(results)} of {len(pts)} points done",
                  file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    while todo or running:
        while todo and len(running) < a.workers:
            n, m = todo.pop(0)
            p = subprocess.Popen([sys.executable, __file__, "--child", f"{n}x{m}", "--data", a.data], env=env,
                                 stdout=subprocess.PIPE, text=True)
            running.append(p)
        time.sleep(1)
        for p in list(running):
            if p.poll() is not None:
                running.remove(p)
                out = p.stdout.read().strip().splitlines()
                if p.returncode != 0 or not out:
                    raise SystemExit(f"cpu_sweep: a point failed ({p.args})")
                results.append(json.loads(out[-1]))
                r = results[-1]
                print(f"[cpu_sweep] {r['n']} x {r['m']}: {r['total_s']:.1f} s", file=sys.stderr, flush=True)
    stop.set()
    results.sort(key=lambda r: (r["m"], r["n"]))
    coef, resid = fit(results)
    doc = {"what": "oracle/pipeline.py steps 4-7 from mosdepth BGZF files to output files, one single-threaded "
                   "process per point (OMP/BLAS threads 1)",
           "cores_per_point": 1, "host_cpus": os.cpu_count(), "workers": a.workers, "points": results,
           "fit_seconds_per_unit": coef,
           "fit_units": {**{s: "N*M" for s in LIN_CELLS}, "knn": "N^2*R_use", **{s: "N" for s in LIN_N}},
           "fit_check": resid,
           "extrapolated": {"config2_3202x3M": predict(coef, 3202, 3_000_000, 2_700_000),
                            "config3_50kx3M": predict(coef, 50_000, 3_000_000, 2_700_000)},
           "wall_s": time.perf_counter() - t0}
    s = json.dumps(doc, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            f.write(s)
    print(s, flush=True)


if __name__ == "__main__":
    main()
