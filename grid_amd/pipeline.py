"""WGS pipeline orchestrator (reference: grid/pipeline.py:9-103).

Same YAML, same step gates, same catch-and-log-and-continue behaviour per
step.  Steps 4-7 run on the MI355X path; steps 1-3 (CRAM indexing, read
counting, mosdepth) are producers outside this build's scope: when enabled
they are reported, and their output files must already exist.
"""
from __future__ import annotations

import yaml

from .utils.utils import log


def _oos(console, what):
    log(console, f"{what} is not part of grid_amd (steps 4-7 only); using existing outputs", style="warning")


def run_wgs_pipeline(console=False, config=None, keep_buffers=False, **args):
    """Steps 4-7 as the reference's run_wgs_pipeline (:9-103).  Under
    torch.distributed.run (WORLD_SIZE > 1) every rank runs this and steps 4-5
    use every GPU of the job (utils/dist_step4.py); steps 6-7 run on rank 0
    (a loci table's loci are dealt over the ranks).  ``keep_buffers``: keep
    the device ingest's buffers cached for the process's next run instead of
    releasing them at the end (their release holds the HIP runtime ~0.5 s)."""
    from .device import deferred_release
    from .utils.dist_step4 import init_from_env
    init_from_env()
    # step 4's ingest buffers are kept to the end of the run, then released
    # (their release holds the HIP runtime for a fraction of a second)
    with deferred_release(release=not keep_buffers):
        _run(console, config)


def _run(console, config):
    if not config:
        raise log(console, "Config file is required for running the WGS pipeline.", style="danger")
    try:
        with open(config, "r") as f:
            cfg = yaml.safe_load(f)
    except Exception as e:
        raise log(console, f"Failed to read the config file: {e}", style="danger")

    # gates read exactly like the reference (a missing section is a KeyError)
    if cfg["index"].get("run") is False or cfg["index"].get("run") is True:
        _oos(console, "Index check/creation (step 1)")
    if cfg["count_reads"].get("run") == True:  # noqa: E712
        _oos(console, "Read counting (step 2)")
    if cfg["mosdepth"].get("run") == True:  # noqa: E712
        _oos(console, "mosdepth (step 3)")

    if cfg["mosdepth"]["normalize"].get("run") == True:  # noqa: E712
        try:
            from .utils.normalize_mosdepth import normalize_mosdepth
            normalize_mosdepth(cfg, console)
        except Exception as e:
            log(console, f"Failed to normalize coverage: {e}", style="danger")

    if cfg["mosdepth"]["neighbors"].get("run") == True:  # noqa: E712
        try:
            from .utils.find_neighbors import find_neighbors
            find_neighbors(cfg, console)
        except Exception as e:
            log(console, f"Failed to find neighbors: {e}", style="danger")
    from .utils import handoff
    handoff.clear()                 # step 4's device matrix, if step 5 did not run

    if cfg["compute_diploid_genotypes"].get("run") == True:  # noqa: E712
        try:
            from .utils.compute_dipcn import compute_diploid_genotypes
            compute_diploid_genotypes(cfg, console)
        except Exception as e:
            log(console, f"Failed to compute diploid CNV calls: {e}", style="danger")

    if cfg["compute_haploid_genotypes"].get("run") == True:  # noqa: E712
        try:
            from .utils.hi_inference import hi_inference, hi_inference_loci
            if cfg["compute_haploid_genotypes"].get("loci_file"):
                hi_inference_loci(cfg, console)      # many regions (BASELINE config 5)
            else:
                hi_inference(cfg, console)
        except Exception as e:
            log(console, f"Failed to compute haploid CNV calls: {e}", style="danger")
