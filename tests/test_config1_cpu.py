"""BASELINE config 1 (100 samples x 30k bins, k = 10: the reference's CPU
path) pins the oracle at its own shape: the cohort is regenerated from the
seed recorded in tests/golden/g_cfg1 (input digest checked), the oracle runs
steps 4-7 from files to files (oracle/pipeline.py) and every output equals
the reference's (make_golden.py cfg1).  CPU only; the GPU run of the same
cohort is tests/test_gpu_e2e.py::test_config1_100x30k_matches_reference."""
import json

from oracle import pipeline
from tests.golden import cohort_files


def test_oracle_config1_matches_reference(tmp_path):
    cfg, cfg_ibd, meta = cohort_files.regenerate("g_cfg1", tmp_path)
    t = pipeline.run(cfg)
    assert t["shape"]["n"] == 100 and t["shape"]["m"] > 25_000
    pipeline.run(cfg_ibd, only_step7=True)          # the golden's second step-7 run: IBD, weighted
    cohort_files.check_outputs("g_cfg1", tmp_path / "out")
    print(json.dumps({k: v for k, v in t.items()}))
