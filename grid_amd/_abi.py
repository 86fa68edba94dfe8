"""ctypes binding of libgridhip.so (include/grid_abi.h).

This is the only module that talks to the native library.  There is no CPU
fallback: if the library is missing, was not built, or no gfx950 device is
visible, every compute entry point raises ``GridNativeError``.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("GRID_AMD_LIB", _HERE / "_lib" / "libgridhip.so"))

GRID_OK, GRID_EINVAL, GRID_EHIP, GRID_EZERODIV, GRID_EUNSUPPORTED, GRID_ERANGE = range(6)
MISSING = -(2 ** 31)          # GRID_MISSING / GRID_ZQ_NAN
ZQ_NAN = -(2 ** 31)
ZQ_NEG0 = -(2 ** 31) + 1
ZQ16_NAN, ZQ16_NEG0, ZQ16_ESC = -32768, -32767, -32766   # GRID_ZQ16_* (grid_norm_zquant_kb16)
BLOCK = 8192
KBW = 32                       # K-block width of the k-NN panel (common.hpp KBW)
SEG_K1 = 16                    # GRID_SEG_K1: candidate keys per row / column (multi-GPU step 5)
SEL_STATE = 16                 # GRID_SEL_STATE: int64 slots of the device selection state
SEL_NVALID, SEL_RLOC, SEL_RTOT, SEL_NV, SEL_RUSE, SEL_ERR = 0, 1, 2, 3, 4, 5   # GRID_SEL_* slots
SEL_THR, SEL_V0, SEL_SMIN, SEL_SMAX = 8, 9, 12, 13

_i64, _i32, _f64, _vp = C.c_int64, C.c_int32, C.c_double, C.c_void_p

# name -> argtypes (all return int)
_SIGS = {
    "grid_abi_version": [],
    "grid_device_count": [C.POINTER(C.c_int)],
    "grid_ctx_create": [C.c_int, C.POINTER(_vp)],
    "grid_ctx_destroy": [_vp],
    "grid_ctx_set_stream": [_vp, _vp],
    "grid_ctx_own_stream": [_vp],
    "grid_sync": [_vp],
    "grid_ctx_cu_count": [_vp, C.POINTER(_i32)],
    "grid_mem_info": [_vp, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)],
    "grid_dev_alloc": [_vp, C.c_size_t, C.POINTER(_vp)],
    "grid_dev_free": [_vp, _vp],
    "grid_host_alloc": [C.c_size_t, C.POINTER(_vp)],
    "grid_host_free": [_vp],
    "grid_h2d": [_vp, _vp, _vp, C.c_size_t],
    "grid_d2h": [_vp, _vp, _vp, C.c_size_t],
    "grid_d2d": [_vp, _vp, _vp, C.c_size_t],
    "grid_memset": [_vp, _vp, C.c_int, C.c_size_t],
    "grid_event_record": [_vp, C.c_int],
    "grid_stream_after": [_vp, _vp],
    "grid_event_elapsed": [_vp, C.c_int, C.c_int, C.POINTER(C.c_float)],
    "grid_norm_row_blocks": [_vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "grid_norm_row_means": [_vp, _vp, _vp, _i64, _i64, _vp],
    "grid_norm_col_means": [_vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "grid_norm_col_vars": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "grid_sort_valid": [_vp, _vp, _i64, _vp, C.POINTER(_i64)],
    "grid_count_valid": [_vp, _vp, _i64, C.POINTER(_i64)],
    "grid_norm_row_blocks_f64": [_vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "grid_norm_col_stats_f64": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "grid_norm_zquant_f64": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _f64, _vp, _i64, C.POINTER(_i32)],
    "grid_select_kth": [_vp, _vp, _i64, _vp, _i32, _vp],
    "grid_select_gt": [_vp, _vp, _i64, _f64, _vp, C.POINTER(_i64)],
    "grid_sel_stage1": [_vp, _vp, _i64, _vp, _i64, _i64, _f64, _vp, _vp, _vp],
    "grid_sel_stage2": [_vp, _vp, _i64, _vp, _i64, _f64, _f64, _vp, _vp],
    "grid_sel_read": [_vp, _vp, _vp],
    "grid_status_copy": [_vp, _vp],
    "grid_round_decimals": [_vp, _vp, _i64, C.c_int, _vp],
    "grid_gather_f64": [_vp, _vp, _vp, _i64, _vp],
    "grid_colmap_range": [_vp, _vp, _i64, _f64, _f64, _vp, C.POINTER(_i64)],
    "grid_norm_zquant": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _f64, _vp, _i64, _vp, _i32,
                         _vp, _i64, C.POINTER(_i32)],
    "grid_norm_zquant_kb": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _f64, _vp, _i64, _vp, _i32,
                            _vp, _i64, C.POINTER(_i32)],
    "grid_norm_zquant_kb16": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _f64, _vp, _i64, _vp, _i32,
                              _vp, _i64, _vp, _vp, _i64, C.POINTER(_i64), C.POINTER(_i32)],
    "grid_norm_zfull": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _f64, _vp],
    "grid_verify_zquant": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _f64, _vp, _i64, _vp, _i32, _vp, _i64, _vp],
    "grid_knn_gram": [_vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "grid_knn_gram_kb": [_vp, _vp, _i64, _i64, _i32, _vp],
    "grid_knn_topk": [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _vp],
    "grid_knn_mirror": [_vp, _vp, _i64],
    "grid_knn_gram_kb_rows": [_vp, _vp, _i64, _i64, _i32, _i64, _i64, _vp, _i64],
    "grid_knn_mirror_ld": [_vp, _vp, _i64, _i64],
    "grid_knn_diag": [_vp, _vp, _i64, _i64, _vp],
    "grid_knn_topk_rows": [_vp, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp],
    "grid_knn_topk_d2": [_vp, _vp, _i64, _f64, _i64, _i64, _i64, _i64, _vp, _vp, _vp],
    "grid_knn_seg_topk": [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _vp, _vp],
    "grid_knn_seg_merge": [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp],
    "grid_knn_dist_i32": [_vp, _vp, _i64, _i64, _i64, _vp, _i64],
    "grid_knn_dist_f64": [_vp, _vp, _i64, _i64, _i64, _vp, _i64],
    "grid_knn_panel_i32": [_vp, _vp, _i64, _i64, _vp, _i64, _i32, _vp, _i64, _i64],
    "grid_knn_gather_i32": [_vp, _vp, _i64, _i64, _vp, _i64, _i32, _vp],
    "grid_knn_gather_f64": [_vp, _vp, _i64, _i64, _vp, _i64, _f64, _vp],
    "grid_dipcn": [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, C.POINTER(_i32)],
    "grid_hi_levels": [_i64, _vp, _vp, _vp, _vp, C.POINTER(_i32)],
    "grid_hi_pack": [_i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp],
    "grid_hi_phase": [_vp, _i64, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                      _i32, _i32],
    "grid_hi_phase_batch": [_vp, _i64, _vp, _i64, _i32, _i64, _i64, _i32, _i32],
    "grid_hi_pack_batch": [_vp, _i64, _vp, _i64],
    "grid_write_normalized_gz": [C.c_char_p, _i64, _i64, C.c_char_p, _vp, _vp, _vp, _vp, _i64, _i32, _i32],
    "grid_read_normalized_gz": [C.c_char_p, _i32, C.POINTER(_vp), C.POINTER(_i64), C.POINTER(_i64)],
    "grid_write_normalized_gz_dev": [_vp, C.c_char_p, _i64, _i64, C.c_char_p, _vp, _vp, _vp, _vp, _i64, _i32, _i32,
                                     _i64],
    "grid_gz_huffman_member": [_vp, _i64, _vp, _i64, C.POINTER(_i64)],
    "grid_ntext_ids_len": [_vp, C.POINTER(_i64)],
    "grid_ntext_fetch": [_vp, _vp, _i64, _vp, _vp, _vp, _vp],
    "grid_ntext_free": [_vp],
    "grid_load_ibs": [C.c_char_p, C.c_char_p, _i64, _i64, C.POINTER(_vp), C.POINTER(_i64)],
    "grid_load_ibd": [C.c_char_p, C.c_char_p, _i64, _i64, _i32, _i64, _i64, _f64, _f64, _f64, C.POINTER(_vp),
                      C.POINTER(_i64)],
    "grid_hapnbr_fetch": [_vp, _vp, _vp, _vp],
    "grid_hapnbr_free": [_vp],
    "grid_q16_encode": [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _i64, C.POINTER(_i64)],
    "grid_synth_depth_q16": [_vp, C.c_uint64, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _i64,
                             C.POINTER(_i64)],
    "grid_norm_row_blocks_q16": [_vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "grid_norm_col_means_q16": [_vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "grid_norm_col_vars_q16": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "grid_norm_zquant_kb_q16": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _f64, _vp, _i64, _vp, _i32,
                                _vp, _i64, C.POINTER(_i32)],
    "grid_norm_zquant_kb16_q16": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _f64, _vp, _i64, _vp, _i32,
                                  _vp, _i64, _vp, _vp, _i64, C.POINTER(_i64), C.POINTER(_i32)],
    "grid_synth_depth": [_vp, C.c_uint64, _i64, _i64, _i64, _i64, _i32, _vp],
    "grid_format_hundredths": [_vp, _i64, _vp, _i64, C.POINTER(_i64)],
    "grid_ingest_mosdepth": [_vp, _i64, C.c_char_p, C.c_int, _i64, _i64, _i64, _vp, _vp, _vp, _f64, _f64,
                             C.c_int, _i64, C.POINTER(_vp)],
    "grid_ingest_summary": [_vp, C.POINTER(_i64), _vp, _vp],
    "grid_ingest_columns": [_vp, _vp, _vp],
    "grid_ingest_population_means": [_vp, _vp, _vp, _vp, _i64, C.POINTER(_i64)],
    "grid_ingest_fill": [_vp, _vp, _vp, _i64, _i64],
    "grid_ingest_free": [_vp],
    "grid_gunzip_batch": [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp],
    "grid_gz_text_size": [_vp, _i64, C.POINTER(_i64), C.POINTER(_i32)],
    "grid_gz_members": [_vp, _i64, _vp, _vp, _vp, _i32, C.POINTER(_i32)],
    "grid_gunzip_host": [_vp, _i64, _vp, _i64, C.POINTER(_i64), C.POINTER(_i32), C.POINTER(C.c_uint32)],
    "grid_text_crc32": [_vp, _vp, _vp, _vp, _i64, _vp],
    "grid_md_count": [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp],
    "grid_file_status": [_vp, _vp, _vp, _i64, _vp, _i64],
    "grid_h2d_async": [_vp, _vp, _vp, C.c_size_t],
    "grid_d2h_async": [_vp, _vp, _vp, C.c_size_t],
    "grid_event_new": [C.POINTER(_vp)],
    "grid_event_free": [_vp],
    "grid_event_put": [_vp, _vp],
    "grid_event_wait": [_vp, _vp],
    "grid_event_host_wait": [_vp],
    "grid_md_parse_ref": [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                          C.POINTER(_i64), C.POINTER(_i32)],
    "grid_md_parse_map": [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                          _vp, _vp],
    "grid_fill_i32": [_vp, _vp, _i64, _i32],
    "grid_md_finish": [_vp, _vp, _i64, _i64, _i64, _vp, _i32, _f64, _f64, _vp, _vp, _vp, _vp, _vp, C.POINTER(_i64)],
    "grid_md_gather": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp],
    "grid_ctx_own_stream_cumask": [_vp, _vp, _i32],
    "grid_ctx_stream": [_vp, C.POINTER(_vp)],
    "grid_knn_seg_pack": [_vp, _vp, _i64, _i64, _i64, _vp],
    # distributed `grid wgs` (grid_amd/utils/dist_step4.py)
    "grid_md_popsum": [_vp, _vp, _i64, _i64, _vp, _i32, _vp, _vp],
    "grid_md_popvalid": [_vp, _vp, _vp, _i64, _f64, _f64, _vp],
    "grid_md_rowstats": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, C.POINTER(_i64)],
    "grid_md_pack_shards": [_vp, _vp, _i64, _i64, _vp, _vp, _vp, _i32, _vp, _i32, _vp],
    "grid_gz_parts_new": [C.POINTER(_vp)],
    "grid_gz_parts_header": [_vp, _i64, _i64, _vp, _vp, _i32, _i32],
    "grid_gz_parts_rows": [_vp, _i64, _i64, _i64, C.c_char_p, _vp, _vp, _i64, _i32, _i32],
    "grid_gz_parts_rows_dev": [_vp, _vp, _i64, _i64, _i64, C.c_char_p, _vp, _vp, _i64, _i32, _i64],
    "grid_gz_parts_size": [_vp, C.POINTER(_i64)],
    "grid_gz_parts_write": [_vp, C.c_char_p, _i64, _i32],
    "grid_gz_parts_free": [_vp],
}
EXPORTS = tuple(_SIGS) + ("grid_last_error", "grid_build_info")


class GridNativeError(RuntimeError):
    """The HIP native path failed or is unavailable (no silent fallback).
    ``code``: the GRID_E* return code (None when not from a library call)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


_lib = None


def load():
    """Load libgridhip.so once.  If torch is already imported, the library
    binds to torch's HIP runtime (same soname), so torch device pointers and
    streams can be passed straight through."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise GridNativeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                              "or `make -C grid_amd/csrc`")
    lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    try:
        for name, args in _SIGS.items():
            f = getattr(lib, name)
            f.argtypes = args
            f.restype = C.c_int
        lib.grid_last_error.argtypes = []
        lib.grid_last_error.restype = C.c_char_p
        info = _build_info(lib)
    except AttributeError as e:
        raise GridNativeError(f"{LIB_PATH} lacks an entry point this package binds ({e}): rebuild with "
                              "`make -C grid_amd/csrc`") from None
    # the file list the library hashed (its build info), so the two sides
    # cannot drift apart when a source is added to the Makefile
    files = info.get("src_files")
    if files and (_CSRC / "Makefile").exists():          # a source tree, not an installed copy
        # a source added to the Makefile after the library was built: the
        # library's own list no longer names every hashed file
        named = sorted(n for n in files.split() if not n.startswith(".."))
        if named != _HASHED:
            raise GridNativeError(f"{LIB_PATH} hashed other source files ({' '.join(named)}) than this tree "
                                  f"lists: rebuild with `make -C grid_amd/csrc`")
    want = source_sha256(files.split() if files else None)
    if want is not None and info.get("src_sha256") != want:
        raise GridNativeError(f"{LIB_PATH} was built from other sources (library {info.get('src_sha256')}, "
                              f"tree {want}): rebuild with `make -C grid_amd/csrc`")
    _lib = lib
    return lib


# the files grid_amd/csrc/Makefile hashes into the library (HASHED), in its sorted order
_CSRC = _HERE / "csrc"
_HASHED = sorted(["core.hip", "normalize.hip", "knn.hip", "dipcn_phase.hip", "synth.hip", "depth16.hip",
                  "inflate.hip", "mosdepth_dev.hip", "gzwrite.hip", "ingest.cpp", "textio.cpp", "hapnbr.cpp",
                  "common.hpp", "synth_model.hpp", "inflate_core.hpp", "fastgz.hpp"])


def source_sha256(names=None):
    """sha256 of the native sources as the Makefile hashes them: ``names``
    relative to grid_amd/csrc in the Makefile's order (the library's build
    info carries them), else the list below (None when the tree holds no
    sources, e.g. an installed copy)."""
    import hashlib
    if names is not None:
        files = [_CSRC / f for f in names]
    else:
        files = [_CSRC / f for f in _HASHED] + [_HERE.parent / "include" / "grid_abi.h"]
    if not all(f.exists() for f in files):
        return None
    h = hashlib.sha256()
    for f in files:
        h.update(f.read_bytes())
    return h.hexdigest()


def _build_info(lib):
    import json
    lib.grid_build_info.argtypes = [C.c_char_p, C.c_int64]
    lib.grid_build_info.restype = C.c_int
    buf = C.create_string_buffer(512)
    lib.grid_build_info(buf, 512)
    return json.loads(buf.value.decode())


def build_info():
    """The loaded library's provenance: source sha256, compiler, arch, build time."""
    return _build_info(load())


def check(rc: int, what: str = ""):
    if rc == GRID_OK:
        return
    msg = load().grid_last_error().decode(errors="replace")
    if rc == GRID_EZERODIV:
        raise ZeroDivisionError(msg or "float division by zero")
    raise GridNativeError(f"{what}: {msg} (code {rc})", rc)


def call(name: str, *args):
    check(getattr(load(), name)(*args), name)


def ptr(a) -> int:
    """Address of a numpy array, DevBuf or torch tensor."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags.c_contiguous:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    if isinstance(a, DevBuf):
        return a.ptr
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return int(a)


class PinnedBuf:
    """Page-locked host memory (grid_host_alloc) viewed as a uint8 array."""

    def __init__(self, nbytes: int):
        h = _vp()
        call("grid_host_alloc", int(nbytes), C.byref(h))
        self.ptr, self.nbytes = h.value, int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            self.array = None
            load().grid_host_free(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Device:
    """One HIP context (one GPU, one stream).  Not shared across threads."""

    def __init__(self, device: int = 0, stream=None):
        lib = load()
        self.index = device
        h = _vp()
        check(lib.grid_ctx_create(device, C.byref(h)), "grid_ctx_create")
        self.ctx = h.value
        if stream is not None:
            self.set_stream(stream)

    def set_stream(self, stream):
        """Enqueue on ``stream`` (a torch.cuda.Stream, a raw handle, or
        None/0 for the default stream)."""
        s = stream if isinstance(stream, int) or stream is None else stream.cuda_stream
        call("grid_ctx_set_stream", self.ctx, s or None)

    def sync(self):
        call("grid_sync", self.ctx)

    def own_stream_cumask(self, cus, ncu):
        """Enqueue on a stream of this context's own restricted to the CUs
        ``cus`` (indices < ncu; hipExtStreamCreateWithCUMask)."""
        words = np.zeros((ncu + 31) // 32, dtype=np.uint32)
        for c in cus:
            words[c // 32] |= np.uint32(1 << (c % 32))
        call("grid_ctx_own_stream_cumask", self.ctx, words.ctypes.data, len(words))

    def stream_handle(self):
        h = _vp()
        call("grid_ctx_stream", self.ctx, C.byref(h))
        return h.value or 0

    def cached(self, name, nbytes) -> "DevBuf":
        """A uint8 device buffer of at least ``nbytes`` kept on this context
        under ``name`` for reuse by later calls (the device ingest's input and
        text buffers, tens of GB: releasing them took ~0.4 s of the step's
        time, hipFree holding the device); freed by close() or when a larger
        one replaces it."""
        cache = self.__dict__.setdefault("_cache", {})
        b = cache.get(name)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                b.free()
                cache[name] = b = None
            b = cache[name] = self.alloc(int(nbytes), np.uint8)
        return b

    def release_cached(self, prefix=""):
        """Free the buffers cached under names starting with ``prefix``;
        returns the bytes freed."""
        cache = self.__dict__.get("_cache", {})
        freed = 0
        for name in [k for k in cache if k.startswith(prefix)]:
            b = cache.pop(name)
            if b is not None:
                freed += b.nbytes
                b.free()
        return freed

    def cached_bytes(self):
        return sum(b.nbytes for b in self.__dict__.get("_cache", {}).values() if b is not None)

    def mem_info(self):
        """(free, total) HBM bytes of this device (hipMemGetInfo)."""
        f, t = C.c_size_t(), C.c_size_t()
        call("grid_mem_info", self.ctx, C.byref(f), C.byref(t))
        return f.value, t.value

    def close(self):
        if getattr(self, "ctx", None):
            for b in self.__dict__.pop("_cache", {}).values():
                if b is not None:
                    b.free()
            load().grid_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- memory -----------------------------------------------------------
    def alloc(self, shape, dtype) -> "DevBuf":
        return DevBuf(self, shape, dtype)

    def upload(self, a: np.ndarray) -> "DevBuf":
        a = np.ascontiguousarray(a)
        b = DevBuf(self, a.shape, a.dtype)
        call("grid_h2d", self.ctx, b.ptr, a.ctypes.data, a.nbytes)
        return b

    def zeros(self, shape, dtype) -> "DevBuf":
        b = DevBuf(self, shape, dtype)
        b.zero()
        return b

    def record(self, slot: int):
        call("grid_event_record", self.ctx, slot)

    def elapsed_ms(self, a: int, b: int) -> float:
        f = C.c_float()
        call("grid_event_elapsed", self.ctx, a, b, C.byref(f))
        return float(f.value)


class Event:
    """A HIP event (timing disabled) for ordering streams and the host
    (grid_event_*)."""

    def __init__(self):
        h = _vp()
        call("grid_event_new", C.byref(h))
        self.h = h.value

    def put(self, dev: "Device"):
        call("grid_event_put", dev.ctx, self.h)

    def wait(self, dev: "Device"):
        call("grid_event_wait", dev.ctx, self.h)

    def host_wait(self):
        call("grid_event_host_wait", self.h)

    def __del__(self):
        try:
            if self.h:
                load().grid_event_free(self.h)
                self.h = None
        except Exception:
            pass


class DevBuf:
    """Device allocation with a numpy-style shape/dtype."""

    def __init__(self, dev: Device, shape, dtype):
        self.dev = dev
        self.shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        h = _vp()
        call("grid_dev_alloc", dev.ctx, self.nbytes, C.byref(h))
        self.ptr = h.value

    def zero(self):
        call("grid_memset", self.dev.ctx, self.ptr, 0, self.nbytes)
        return self

    def fill_bytes(self, v: int):
        call("grid_memset", self.dev.ctx, self.ptr, v, self.nbytes)
        return self

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, dtype=self.dtype)
        call("grid_d2h", self.dev.ctx, out.ctypes.data, self.ptr, self.nbytes)
        return out

    def copy_from(self, a: np.ndarray):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes <= self.nbytes
        call("grid_h2d", self.dev.ctx, self.ptr, a.ctypes.data, a.nbytes)

    def free(self):
        if self.ptr:
            load().grid_dev_free(self.dev.ctx, self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            if self.ptr and self.dev.ctx:
                self.free()
        except Exception:
            pass


def device_cu_count(dev) -> int:
    """Compute units of ``dev``'s GPU (256 on MI355X)."""
    n = _i32()
    call("grid_ctx_cu_count", dev.ctx, C.byref(n))
    return n.value


def device_count() -> int:
    n = C.c_int()
    call("grid_device_count", C.byref(n))
    return n.value


def format_hundredths(v: np.ndarray) -> str:
    """Exact "%.2f" text of integer hundredths, tab-joined (host C++)."""
    v = np.ascontiguousarray(v, dtype=np.int32)
    cap = 16 * v.size + 16
    buf = C.create_string_buffer(cap)
    n = _i64()
    call("grid_format_hundredths", v.ctypes.data if v.size else None, v.size, buf, cap, C.byref(n))
    return buf.raw[: n.value].decode("ascii")


def write_normalized_gz(path, ids, raw, sel_means, sel_ratios, zq, level=6, threads=None):
    """Step-4 output file (normalize_mosdepth.py:502-554 text), threaded host
    C++ formatting + multi-member gzip.  zq: [n][r] int32 hundredths."""
    zq = np.ascontiguousarray(zq, dtype=np.int32)
    n, r = (zq.shape if zq.ndim == 2 else (len(ids), 0))
    raw = np.ascontiguousarray(raw, dtype=np.float64)
    mu = np.ascontiguousarray(sel_means, dtype=np.float64)
    rt = np.ascontiguousarray(sel_ratios, dtype=np.float64)
    ids_b = "\n".join(ids).encode()
    thr = threads or min(16, os.cpu_count() or 1)
    call("grid_write_normalized_gz", str(path).encode(), n, r, ids_b, raw.ctypes.data, mu.ctypes.data,
         rt.ctypes.data, zq.ctypes.data if zq.size else None, max(r, 0), level, thr)


def write_normalized_gz_dev(dev, path, ids, raw, sel_means, sel_ratios, d_zq, n, r, ld, level=1, threads=None,
                           batch_bytes=0):
    """Step-4 output file from the int32 hundredths in HBM (d_zq: DevBuf or
    device pointer, [n][ld]): row members formatted and Huffman-coded on the
    device (grid_write_normalized_gz_dev), same decompressed text as
    write_normalized_gz."""
    raw = np.ascontiguousarray(raw, dtype=np.float64)
    mu = np.ascontiguousarray(sel_means, dtype=np.float64)
    rt = np.ascontiguousarray(sel_ratios, dtype=np.float64)
    ids_b = "\n".join(ids).encode()
    thr = threads or min(16, os.cpu_count() or 1)
    call("grid_write_normalized_gz_dev", dev.ctx, str(path).encode(), n, r, ids_b, raw.ctypes.data if n else None,
         mu.ctypes.data if r else None, rt.ctypes.data if r else None, ptr(d_zq) if (n and r) else None, max(ld, r),
         level, thr, int(batch_bytes))


class GzParts:
    """One rank's share of a normalised file written by several ranks
    (grid_gz_parts_*): gzip members coded into host memory, then written at
    the rank's byte offset once the ranks have exchanged their sizes."""

    def __init__(self):
        h = _vp()
        call("grid_gz_parts_new", C.byref(h))
        self.h = h.value

    def header(self, n_total, sel_means, sel_ratios, level=1, threads=None):
        """Member 0: the two header lines (N = n_total)."""
        mu = np.ascontiguousarray(sel_means, dtype=np.float64)
        rt = np.ascontiguousarray(sel_ratios, dtype=np.float64)
        call("grid_gz_parts_header", self.h, int(n_total), len(mu), mu.ctypes.data if len(mu) else None,
             rt.ctypes.data if len(rt) else None, level, threads or min(16, os.cpu_count() or 1))

    def rows(self, ids, raw, zq, row0, level=1, threads=None):
        """Row members of host int32 hundredths zq [n][r] (rows row0 + i)."""
        zq = np.ascontiguousarray(zq, dtype=np.int32)
        n, r = zq.shape
        raw = np.ascontiguousarray(raw, dtype=np.float64)
        call("grid_gz_parts_rows", self.h, n, int(row0), r, "\n".join(ids).encode(), raw.ctypes.data if n else None,
             zq.ctypes.data if zq.size else None, max(r, 0), level, threads or min(16, os.cpu_count() or 1))

    def rows_dev(self, dev, ids, raw, d_zq, n, r, ld, row0, batch_bytes=0):
        """Row members of int32 hundredths in HBM (d_zq [n][ld]), coded on the
        device as write_normalized_gz_dev codes them."""
        raw = np.ascontiguousarray(raw, dtype=np.float64)
        call("grid_gz_parts_rows_dev", dev.ctx, self.h, n, int(row0), r, "\n".join(ids).encode(),
             raw.ctypes.data if n else None, ptr(d_zq) if (n and r) else None, max(ld, r), 1, int(batch_bytes))

    def size(self):
        s = _i64()
        call("grid_gz_parts_size", self.h, C.byref(s))
        return s.value

    def write(self, path, offset, threads=4):
        call("grid_gz_parts_write", self.h, str(path).encode(), int(offset), threads)

    def free(self):
        if self.h:
            load().grid_gz_parts_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def read_normalized_gz(path, threads=None):
    """Parse the step-4 file: (ids, scales [n], means [r], ratios [r], zq [n][r]
    int32 hundredths).  Raises GridNativeError(code GRID_EUNSUPPORTED) when
    the text leaves the "%.2f" grammar."""
    lib = load()
    h, n, r = _vp(), _i64(), _i64()
    thr = threads or min(16, os.cpu_count() or 1)
    check(lib.grid_read_normalized_gz(str(path).encode(), thr, C.byref(h), C.byref(n), C.byref(r)),
          "grid_read_normalized_gz")
    try:
        n, r = n.value, r.value
        ln = _i64()
        call("grid_ntext_ids_len", h, C.byref(ln))
        ids_buf = C.create_string_buffer(max(ln.value, 1))
        scales, means, ratios = np.empty(n), np.empty(r), np.empty(r)
        zq = np.empty((n, r), dtype=np.int32)
        call("grid_ntext_fetch", h, ids_buf, ln.value, scales.ctypes.data, means.ctypes.data, ratios.ctypes.data,
             zq.ctypes.data)
        ids = ids_buf.raw[: ln.value].decode().split("\n")[:n]
        return ids, scales, means, ratios, zq
    finally:
        lib.grid_ntext_free(h)


def _hapnbr_result(rc, h, nnz, n, what):
    check(rc, what)
    try:
        off = np.empty(2 * n + 1, dtype=np.int64)
        nbr = np.empty(max(nnz.value, 1), dtype=np.int32)
        w = np.empty(max(nnz.value, 1), dtype=np.float64)
        call("grid_hapnbr_fetch", h, off.ctypes.data, nbr.ctypes.data, w.ctypes.data)
        return off, nbr[: nnz.value], w[: nnz.value]
    finally:
        load().grid_hapnbr_free(h)


def load_ibs(path, ids, max_nbr):
    """computeIBSpbwt file -> CSR (off [2n+1], nbr, w); hi_inference.py:34-74."""
    h, nnz = _vp(), _i64()
    rc = load().grid_load_ibs(str(path).encode(), "\n".join(ids).encode(), len(ids), int(max_nbr), C.byref(h),
                              C.byref(nnz))
    return _hapnbr_result(rc, h, nnz, len(ids), "grid_load_ibs")


def load_ibd(path, ids, max_nbr, region_start, region_end, min_length, min_match, weighted, weight_scale):
    """iLASH file -> CSR (off [2n+1], nbr, w); hi_inference.py:86-172."""
    h, nnz = _vp(), _i64()
    rc = load().grid_load_ibd(str(path).encode(), "\n".join(ids).encode(), len(ids), int(max_nbr),
                              1 if weighted else 0, int(region_start or 0), int(region_end or 0),
                              float(min_length), float(min_match), float(weight_scale), C.byref(h), C.byref(nnz))
    return _hapnbr_result(rc, h, nnz, len(ids), "grid_load_ibd")


def hi_levels(off: np.ndarray, nbr: np.ndarray):
    """Level schedule of the in-place Gauss-Seidel sweep (host C++)."""
    off = np.ascontiguousarray(off, dtype=np.int64)
    nbr = np.ascontiguousarray(nbr, dtype=np.int32)
    n = (len(off) - 1) // 2
    order = np.empty(max(n, 1), dtype=np.int32)
    loff = np.empty(n + 2, dtype=np.int32)
    nl = _i32()
    call("grid_hi_levels", n, off.ctypes.data, nbr.ctypes.data if nbr.size else None, order.ctypes.data,
         loff.ctypes.data, C.byref(nl))
    return order[:n], loff[: nl.value + 1], nl.value


PACK_CAP = 16
HI_UNIT_WEIGHTS, HI_LEGACY, HI_PAIRED = 1, 2, 4     # grid_hi_phase flags


def hi_schedule(off: np.ndarray, nbr: np.ndarray, w: np.ndarray, packed_w: bool = True):
    """Level schedule + schedule-ordered packed neighbour lists (host C++).
    ``packed_w=False``: with unit weights the packed weights (2/3 of the packed
    bytes) are not built and pk_w is None (pass NULL: the kernels read 1.0)."""
    order, loff, nl = hi_levels(off, nbr)
    n = len(order)
    off = np.ascontiguousarray(off, dtype=np.int64)
    unit = len(w) == 0 or bool(np.all(np.asarray(w) == 1.0))
    flags = HI_UNIT_WEIGHTS if unit else 0
    nbr = np.ascontiguousarray(nbr if len(nbr) else np.zeros(1), dtype=np.int32)
    w = np.ascontiguousarray(w if len(w) else np.zeros(1), dtype=np.float64)
    pk_nbr = np.empty((max(n, 1), 2, PACK_CAP), dtype=np.int32)
    skip_w = unit and not packed_w
    pk_w = None if skip_w else np.empty((max(n, 1), 2, PACK_CAP), dtype=np.float64)
    pk_cnt = np.zeros((max(n, 1), 2), dtype=np.int32)
    call("grid_hi_pack", n, off.ctypes.data, nbr.ctypes.data, w.ctypes.data, order.ctypes.data if n else None,
         PACK_CAP, pk_nbr.ctypes.data, None if skip_w else pk_w.ctypes.data, pk_cnt.ctypes.data)
    if n == 0:
        pk_nbr[:] = 0
        if pk_w is not None:
            pk_w[:] = 0
    lens = np.diff(off) if len(off) > 1 else np.zeros(1, np.int64)
    return order, loff, nl, pk_nbr, pk_w, pk_cnt, flags, int(lens.max()) if lens.size else 0


GZ_MEMBER_BYTES = 24                 # include/grid_abi.h grid_gz_member
GZ_OK, GZ_EDATA, GZ_ETRUNC, GZ_ESPACE, GZ_EHEADER, GZ_ECRC = range(6)


def gunzip_batch(dev, blobs, caps, mcap=None):
    """Inflate gzip files on the device (grid_gunzip_batch, one wave per file).
    blobs: compressed bytes per file; caps: output capacity per file.  Returns
    (status [n], lengths [n], members [n], out DevBuf, out offsets [n]) -- the
    text of file f is out[off[f] : off[f] + lengths[f]] when status[f] == 0."""
    n = len(blobs)
    in_off = np.zeros(max(n, 1), np.int64)
    out_off = np.zeros(max(n, 1), np.int64)
    pos = opos = 0
    for f, b in enumerate(blobs):
        in_off[f], out_off[f] = pos, opos
        pos += -(-max(len(b), 1) // 256) * 256
        opos += -(-max(int(caps[f]), 1) // 256) * 256
    src = np.zeros(pos + 256, np.uint8)
    for f, b in enumerate(blobs):
        src[in_off[f]:in_off[f] + len(b)] = np.frombuffer(b, np.uint8)
    mcap = mcap or max(1, max((len(b) // 4096 + 16 for b in blobs), default=1))
    d_src = dev.upload(src)
    d_in_off, d_out_off = dev.upload(in_off), dev.upload(out_off)
    d_in_len = dev.upload(np.array([len(b) for b in blobs] or [0], np.int64))
    d_cap = dev.upload(np.asarray(list(caps) or [0], np.int64))
    out = dev.alloc(opos + 256, np.uint8)
    mem = dev.alloc(max(n, 1) * mcap * GZ_MEMBER_BYTES, np.uint8)
    st, ln, nm = dev.alloc(max(n, 1), np.int32), dev.alloc(max(n, 1), np.int64), dev.alloc(max(n, 1), np.int32)
    call("grid_gunzip_batch", dev.ctx, d_src.ptr, d_in_off.ptr, d_in_len.ptr, n, out.ptr, d_out_off.ptr, d_cap.ptr,
         mem.ptr, mcap, st.ptr, ln.ptr, nm.ptr)
    return st.numpy()[:n], ln.numpy()[:n], nm.numpy()[:n], out, out_off[:n]


class MdOpts(C.Structure):
    """include/grid_abi.h grid_md_opts (device pointers)."""
    _fields_ = [("d_prefix", C.c_void_p), ("npre", C.c_int32), ("has_window", C.c_int32), ("start", C.c_int64),
                ("end", C.c_int64), ("nmask", C.c_int32), ("reserved", C.c_int32), ("d_mask_names", C.c_void_p),
                ("d_mask_name_off", C.c_void_p), ("d_mask_kb_off", C.c_void_p), ("d_mask_kb", C.c_void_p)]


MD_EXOTIC, MD_NOTINK = 1, 2


def gz_text_size(buf) -> tuple[int, int] | None:
    """(inflated size, members) of a gzip file held in ``buf`` (bytes/ndarray),
    None if it is not gzip (host C++)."""
    a = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    size, m = _i64(), _i32()
    rc = load().grid_gz_text_size(a.ctypes.data if a.size else None, a.size, C.byref(size), C.byref(m))
    if rc == GRID_EUNSUPPORTED:
        return None
    check(rc, "grid_gz_text_size")
    return size.value, m.value


def gz_members(buf):
    """BGZF members of a gzip file held in ``buf``: (offsets, lengths, isizes)
    int64/int64/uint32 arrays, or None if the file is not BGZF throughout."""
    a = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    cap = max(16, a.size // 8192 + 16)
    for _ in range(2):
        st, ln, isz = np.empty(cap, np.int64), np.empty(cap, np.int64), np.empty(cap, np.uint32)
        cnt = _i32()
        rc = load().grid_gz_members(a.ctypes.data if a.size else None, a.size, st.ctypes.data, ln.ctypes.data,
                                    isz.ctypes.data, cap, C.byref(cnt))
        if rc == GRID_EUNSUPPORTED:
            return None
        check(rc, "grid_gz_members")
        if cnt.value <= cap:
            k = cnt.value
            return st[:k], ln[:k], isz[:k]
        cap = cnt.value
    raise GridNativeError("grid_gz_members: member count changed")


def gunzip_host(src, out, with_crc=False):
    """Inflate the gzip file in ``src`` into the uint8 array ``out`` (host,
    libdeflate or zlib; releases the GIL).  Returns (status GZ_*, bytes), and
    with ``with_crc`` the text's CRC-32 from the members' trailers as well."""
    a = np.frombuffer(src, np.uint8) if not isinstance(src, np.ndarray) else src
    n, st, crc = _i64(), _i32(), C.c_uint32()
    call("grid_gunzip_host", a.ctypes.data if a.size else None, a.size, out.ctypes.data if out.size else None,
         out.size, C.byref(n), C.byref(st), C.byref(crc))
    return (st.value, n.value, crc.value) if with_crc else (st.value, n.value)


def text_crc32(dev, base_ptr, offs, lens) -> np.ndarray:
    """CRC-32 of the device byte ranges base_ptr + offs[i], lens[i] bytes
    (grid_text_crc32; synchronises dev's stream)."""
    o = np.ascontiguousarray(offs, np.int64)
    ln = np.ascontiguousarray(lens, np.int64)
    out = np.zeros(max(len(o), 1), np.uint32)
    if len(o):
        call("grid_text_crc32", dev.ctx, base_ptr, o.ctypes.data, ln.ctypes.data, len(o), out.ctypes.data)
    return out[:len(o)]


class Depth16Desc(C.Structure):
    """include/grid_abi.h grid_depth16 (device pointers)."""
    _fields_ = [("q", C.c_void_p), ("eoff", C.c_void_p), ("ecol", C.c_void_p), ("eval", C.c_void_p)]


class HiLocus(C.Structure):
    """include/grid_abi.h grid_hi_locus (device pointers of one locus)."""
    _fields_ = [("n", C.c_int64), ("irr", C.c_void_p), ("off", C.c_void_p), ("nbr", C.c_void_p),
                ("w", C.c_void_p), ("order", C.c_void_p), ("loff", C.c_void_p), ("nlev", C.c_int32),
                ("reserved", C.c_int32), ("pk_nbr", C.c_void_p), ("pk_w", C.c_void_p), ("pk_cnt", C.c_void_p),
                ("hap", C.c_void_p), ("imp", C.c_void_p), ("mean", C.c_void_p)]


class IngestUnsupported(GridNativeError):
    """A mosdepth file left the strict grammar the native parser covers."""


class Ingest:
    """Host C++ ingest of mosdepth regions files (grid_ingest_* in
    include/grid_abi.h): one parse per file, ordered population means,
    valid columns, then ``fill`` of the int32 hundredths matrix."""

    def __init__(self, paths, chrom_prefix, window, mask, min_depth, max_depth, threads=1,
                 cache_bytes=None):
        lib = load()
        self.n = len(paths)
        enc = [(str(p).encode() if p is not None else b"") for p in paths]
        arr = (C.c_char_p * max(self.n, 1))(*enc)
        names = sorted(mask)
        carr = (C.c_char_p * max(len(names), 1))(*[c.encode() for c in names])
        moff = np.zeros(len(names) + 1, dtype=np.int64)
        kb = []
        for i, c in enumerate(names):
            v = np.fromiter(mask[c], dtype=np.int64, count=len(mask[c]))
            kb.append(v)
            moff[i + 1] = moff[i] + len(v)
        kbv = np.ascontiguousarray(np.concatenate(kb) if kb else np.zeros(1, np.int64))
        if cache_bytes is None:
            try:
                cache_bytes = int(os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES") * 0.5)
            except (ValueError, OSError):
                cache_bytes = 1 << 33
        has_w = window is not None
        s, e = window if has_w else (0, 0)
        h = _vp()
        rc = lib.grid_ingest_mosdepth(arr, self.n, chrom_prefix.encode() if chrom_prefix else None, int(has_w),
                                      int(s), int(e), len(names), carr, moff.ctypes.data, kbv.ctypes.data,
                                      float(min_depth), float(max_depth), int(max(1, threads)), int(cache_bytes),
                                      C.byref(h))
        if rc == GRID_EUNSUPPORTED:
            raise IngestUnsupported(lib.grid_last_error().decode(errors="replace"))
        check(rc, "grid_ingest_mosdepth")
        self.h = h.value
        m = _i64()
        self.status = np.zeros(max(self.n, 1), dtype=np.int32)
        self.nvalid = np.zeros(max(self.n, 1), dtype=np.int64)
        call("grid_ingest_summary", self.h, C.byref(m), self.status.ctypes.data, self.nvalid.ctypes.data)
        self.status, self.nvalid = self.status[: self.n], self.nvalid[: self.n]
        self.m = m.value
        st = np.zeros(max(self.m, 1), dtype=np.int64)
        en = np.zeros(max(self.m, 1), dtype=np.int64)
        call("grid_ingest_columns", self.h, st.ctypes.data, en.ctypes.data)
        self.starts, self.ends = st[: self.m], en[: self.m]

    def population_means(self):
        nk = _i64()
        call("grid_ingest_population_means", self.h, None, None, None, 0, C.byref(nk))
        k = max(nk.value, 1)
        st, en, mu = np.zeros(k, np.int64), np.zeros(k, np.int64), np.zeros(k)
        call("grid_ingest_population_means", self.h, st.ctypes.data, en.ctypes.data, mu.ctypes.data, k,
             C.byref(nk))
        n = nk.value
        return {(int(a), int(b)): float(v) for a, b, v in zip(st[:n], en[:n], mu[:n])}

    def fill(self, row_of_file, out=None):
        rof = np.ascontiguousarray(row_of_file, dtype=np.int32)
        nrows = int(rof.max()) + 1 if rof.size and rof.max() >= 0 else 0
        if out is None:
            out = np.empty((nrows, self.m), dtype=np.int32)
        call("grid_ingest_fill", self.h, rof.ctypes.data, out.ctypes.data if out.size else None, nrows,
             out.shape[1] if out.ndim == 2 else self.m)
        return out

    def close(self):
        if getattr(self, "h", None):
            load().grid_ingest_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
