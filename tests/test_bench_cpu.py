"""The committed records bench.py reads at run time (CPU only): the PMC traffic
summary behind roofline.traffic and the CPU-baseline sweep must be in the tree
and hold what the line takes from them, or the driver's bench line silently
reports traffic / the sweep as null."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_const(name):
    src = open(os.path.join(ROOT, "bench.py")).read()
    m = re.search(rf'^{name} = "([^"]+)"', src, re.M)
    assert m, name
    return m.group(1)


def test_traffic_record_has_the_gram_kernel():
    path = os.path.join(ROOT, _bench_const("TRAFFIC_JSON"))
    tj = json.load(open(path))
    gram = _bench_const("GRAM_KERNEL")
    hits = [v for k, v in tj["kernels"].items() if k.startswith(gram)]
    assert len(hits) == 1
    # per-launch HBM bytes of the dominant kernel: fetch + write, both positive
    h = hits[0]
    assert h["fetch_bytes"] > 0 and h["write_bytes"] > 0
    assert abs(h["traffic_bytes"] - (h["fetch_bytes"] + h["write_bytes"])) <= 1e-6 * h["traffic_bytes"]


def test_cpu_sweep_record_has_the_config2_fit():
    sw = json.load(open(os.path.join(ROOT, _bench_const("CPU_SWEEP_JSON"))))
    assert sw["points"] and sw["fit_seconds_per_unit"]
    assert set(sw["fit_seconds_per_unit"]) == set(sw["fit_units"])
