"""ctypes binding of libtmhip.so (the C-ABI declared in include/tmhip.h).

This is the ``tmlib/hip`` module the north star names: the product path of
every class in ``tmlibrary_amd`` goes through it.  There is no CPU fallback:
if the library (or a GPU) is missing, ``lib()`` raises ``HipUnavailableError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TMH_LIB", os.path.join(_HERE, "libtmhip.so"))

TMH_OK = 0
TMH_EINVAL = -22
TMH_ENOMEM = -12
TMH_EDEVICE = -5
TMH_ESTATE = -71
TMH_STATS_DEFERRED_PCT = 1
TMH_STATS_KEEP_SITE_HIST = 2
TMH_STATS_SERIAL = 4
TMH_OPT_FUSED_CONFIG = 1
TMH_OPT_WELFORD_PARTS = 2
TMH_OPT_COPY_THREADS = 4
TMH_OPT_HOST_STAGING = 5
TMH_OPT_FUSED_CUS = 8
TMH_OPT_FUSED_BANDS = 9
TMH_FUSED_NO_HIST = 100
TMH_SYNTH_STANDARD = 0
TMH_SYNTH_BRIGHT = 1
TMH_SYNTH_UNIFORM = 2
ABI_VERSION = 4

_P = C.c_void_p
_I64 = C.c_int64
_I = C.c_int
_D = C.c_double

# name -> (restype, argtypes); must match include/tmhip.h exactly
SIGNATURES = {
    "tmh_abi_version": (_I, []),
    "tmh_last_error": (C.c_char_p, []),
    "tmh_device_count": (_I, [C.POINTER(_I)]),
    "tmh_set_device": (_I, [_I]),
    "tmh_synchronize": (_I, [_P]),
    "tmh_stats_create": (_I, [_I, _I, _I, _P, _P, _P, _P, _I, C.c_uint, C.POINTER(_P)]),
    "tmh_stats_destroy": (None, [_P]),
    "tmh_stats_set_stream": (_I, [_P, _P]),
    "tmh_stats_reset": (_I, [_P]),
    "tmh_stats_set_option": (_I, [_P, _I, _I]),
    "tmh_stats_variance": (_I, [_P, _P]),
    "tmh_stats_wide_groups": (_I, [_P, _P, _P]),
    "tmh_stats_job_choice": (_I, [_P, _P, _P, _P]),
    "tmh_stats_get_hist_device": (_I, [_P, _P, _P]),
    "tmh_stats_set_hist_device": (_I, [_P, _P, _P]),
    "tmh_stats_update": (_I, [_P, _P, _I64, _I, _P]),
    "tmh_stats_update_device": (_I, [_P, _P, _I64, _I, _P]),
    "tmh_stats_zero_counts": (_I, [_P, _P, _I64, _P]),
    "tmh_stats_update_welford_device": (_I, [_P, _P, _I64, _I, _P]),
    "tmh_stats_probe_device": (_I, [_P, _P, _I64, _P]),
    "tmh_stats_probe_blocks_device": (_I, [_P, _P, _I, _I64, _P]),
    "tmh_corrector_update_multi_device": (_I, [_P, _I, _P, _P, _P]),
    "tmh_job_planes_multi_device": (_I, [_P, _P, _I, _P, _P, _P, _P, _D, _P]),
    "tmh_stats_update_welford_blocks_device": (_I, [_P, _P, _I, _I64, _I, _P]),
    "tmh_stats_finalize": (_I, [_P, _P, _P, _P, _P, _P]),
    "tmh_stats_finalize_device": (_I, [_P, _P, _P, _P]),
    "tmh_stats_site_histogram": (_I, [_P, _I64, _P]),
    "tmh_stats_site_order_stats": (_I, [_P, _I64, _P, _P]),
    "tmh_stats_get_n": (_I, [_P, C.POINTER(_I64)]),
    "tmh_stats_set_n": (_I, [_P, _I64]),
    "tmh_stats_merge_stage1": (_I, [_P, _P, _P]),
    "tmh_stats_merge_stage2": (_I, [_P, _P, _I64, _P, _P]),
    "tmh_stats_merge_stage3": (_I, [_P, _I64, _P, _P]),
    "tmh_stats_pct_accumulate": (_I, [_P, _P, _P]),
    "tmh_stats_pct_accumulate_range": (_I, [_P, _P, _I, _I, _P]),
    "tmh_stats_set_pct_sum": (_I, [_P, _P, _P]),
    "tmh_stats_get_pct_sum_device": (_I, [_P, _P, _P]),
    "tmh_smooth_f64": (_I, [_P, _P, _I, _I, _D]),
    "tmh_smooth_f64_device": (_I, [_P, _P, _P, _I, _I, _D, _P]),
    "tmh_smooth2_f64_device": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _D, _P]),
    "tmh_corrector_create": (_I, [_P, _P, _I, _I, _I, _D, C.POINTER(_P)]),
    "tmh_corrector_create_device": (_I, [_P, _P, _I, _I, _I, _D, _P, C.POINTER(_P)]),
    "tmh_corrector_destroy": (None, [_P]),
    "tmh_corrector_update_device": (_I, [_P, _P, _P, _P]),
    "tmh_corrector_set_option": (_I, [_P, _I, _I]),
    "tmh_corrector_means": (_I, [_P, C.POINTER(_D), C.POINTER(_D)]),
    "tmh_correct_u16": (_I, [_P, _P, _P, _I64, _I, _I]),
    "tmh_correct_u16_device": (_I, [_P, _P, _P, _I64, _I, _I, _P]),
    "tmh_correct_u16_hist_device": (_I, [_P, _P, _P, _P, _I64, _I, _I, _P]),
    "tmh_correct_u16_hist_blocks_device": (_I, [_P, _P, _P, _P, _I, _I64, _I, _I, _P]),
    "tmh_correct_u16_hist_multi_device": (_I, [_P, _P, _I, _P, _P, _P, _I, _I, _P]),
    "tmh_correct_u16_hist_multi_blocks_device": (_I, [_P, _P, _I, _P, _P, _I, _P, _I, _I, _P]),
    "tmh_correct_u8": (_I, [_P, _P, _P, _I64, _I, _I]),
    "tmh_clip_u16": (_I, [_P, _P, _I64, _I, _I]),
    "tmh_align": (_I, [_P, _P, _I, _I64, _I, _I, _P, _I, _I]),
    "tmh_map_u16_to_u8": (_I, [_P, _P, _I64, _I, _I]),
    "tmh_correct_chain_u8_device": (_I, [_P, _P, _P, _I64, _P, _I, _I, _P]),
    "tmh_correct_chain_u8": (_I, [_P, _P, _P, _I64, _P, _I, _I]),
    "tmh_synth_sites_device": (_I, [_P, _I64, _I, _I, C.c_uint64, _I, _I64, _I, _P]),
    "tmh_synth_tables": (_I, [_I, _I, _I, _P, _P, _P, _P]),
    "tmh_box_probe_device": (_I, [_P, _P, _I, _I64, _I, _I, _I, _I, _P, C.POINTER(_D),
                                  C.POINTER(_D)]),
    "tmh_inflate_scratch_bytes": (_I64, [_I64, _I64]),
    "tmh_inflate_device": (_I, [_P, _I64, _P, _I64, _I64, _P, _I64, _P, _I64, _P, _P]),
    "tmh_place_chunks_device": (_I, [_P, _P, _I64, _I, _I, _I, _I, _I, _P, _P]),
    "tmh_malloc_device": (_I, [C.POINTER(_P), C.c_size_t]),
    "tmh_free_device": (_I, [_P]),
    "tmh_memcpy": (_I, [_P, _P, C.c_size_t, _I, _P]),
    "tmh_profile_enable": (_I, [_I]),
    "tmh_profile_read": (_I, [C.c_char_p, C.POINTER(_D), C.POINTER(_I64)]),
    "tmh_profile_reset": (_I, []),
}


#: struct tmh_window (include/tmhip.h) as a numpy record: one alignment window per site
WINDOW_DTYPE = np.dtype([("src_r0", np.int32), ("src_c0", np.int32), ("dst_r0", np.int32),
                         ("dst_c0", np.int32), ("rows", np.int32), ("cols", np.int32)])


#: struct tmh_zchunk (include/tmhip.h): one HDF5 gzip chunk of the input path
ZCHUNK_DTYPE = np.dtype([("src_off", np.int64), ("src_len", np.int64), ("raw_off", np.int64),
                         ("raw_len", np.int64), ("image", np.int64), ("row0", np.int32),
                         ("col0", np.int32), ("flags", np.int32), ("reserved", np.int32)])
assert ZCHUNK_DTYPE.itemsize == 56
TMH_ZCHUNK_STORED = 1
#: tmh_inflate_device per-chunk status codes (TMH_Z_*)
Z_STATUS = {0: "ok", 1: "not a zlib stream", 2: "invalid deflate block type",
            3: "invalid Huffman code", 4: "back-reference before the chunk start",
            5: "more output than the chunk holds", 6: "ran past the chunk's bytes",
            7: "Adler-32 mismatch", 8: "less output than the chunk holds",
            9: "stored block length mismatch", 10: "invalid code lengths"}


class HipUnavailableError(RuntimeError):
    """libtmhip.so is missing or no HIP device is usable (no CPU fallback)."""


class HipError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("%s (code %d)" % (message, code))
        self.code = code


_lib = None
_lock = threading.Lock()


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load the shared library and declare every exported signature (no GPU needed)."""
    if not os.path.exists(path):
        raise HipUnavailableError(
            "libtmhip.so not found at %s — build it with `python -c "
            "'import __graft_entry__ as g; g.build()'` or `make -C tmlibrary_amd/csrc`" % path)
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7
    # (same soname as /opt/rocm's).  Whichever loads first serves both; if
    # ours came first, a later torch.cuda initialisation found no GPU
    # (seen running a GPU test module on its own), so let torch's load first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    # an A/B build of an earlier tree (TMH_LIB elsewhere, tools/gpu.sh ab) may
    # lack entry points added since; the in-tree library must export them all
    own = os.path.abspath(path) == os.path.join(_HERE, "libtmhip.so")
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if own:
                raise
            continue
        fn.restype = res
        fn.argtypes = args
    return lib


def lib() -> C.CDLL:
    """The loaded library, checked for a usable device (raises otherwise)."""
    global _lib
    with _lock:
        if _lib is None:
            L = load_library()
            if L.tmh_abi_version() != ABI_VERSION:
                raise HipUnavailableError("libtmhip ABI version mismatch")
            n = C.c_int(0)
            rc = L.tmh_device_count(C.byref(n))
            if rc != TMH_OK or n.value < 1:
                raise HipUnavailableError("no HIP device available for libtmhip (%s)" %
                                          L.tmh_last_error().decode())
            _lib = L
        return _lib


def check(rc: int):
    """Map a C-ABI return code to the reference's exception types."""
    if rc == TMH_OK:
        return
    msg = _lib.tmh_last_error().decode() if _lib is not None else "libtmhip error"
    if rc == TMH_EINVAL:
        raise ValueError(msg)
    if rc == TMH_ENOMEM:
        raise MemoryError(msg)
    raise HipError(rc, msg)


def ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def ptr_or_null(a):
    return None if a is None else ptr(a)


def available() -> bool:
    try:
        lib()
        return True
    except HipUnavailableError:
        return False
