"""grid_amd -- MI355X-native (gfx950) implementation of the GRiD pipeline's
steps 4-7 hot path, a drop-in behind the reference's step API:

  grid_amd.cli            `grid wgs CONFIG`            (grid/cli.py)
  grid_amd.pipeline       run_wgs_pipeline             (grid/pipeline.py)
  grid_amd.utils.*        step modules, same names      (grid/utils/*.py)
  grid_amd._abi           ctypes binding of libgridhip.so (include/grid_abi.h)
  grid_amd.engine         array-level driver of the HIP kernels
"""
__version__ = "0.1.0"
