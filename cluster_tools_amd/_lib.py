"""ctypes binding of libctg.so (the C ABI declared in include/ctg.h).

The product path has no CPU fallback: if the HIP library cannot be loaded, or
no GPU is visible, every compute call raises.  ``load()`` works without a GPU
(symbol/ABI checks in the CPU test-suite only need the shared object).
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('CTG_LIB') or os.path.join(_HERE, 'libctg.so')  # CTG_LIB: A/B builds (tools/)

CTG_OK = 0
CTG_MEM_HOST = 0
CTG_MEM_DEVICE = 1
CTG_DATA_NONE = 0
CTG_DATA_F32 = 1
CTG_DATA_U8 = 2
CTG_KEEP_STATS = 1
CTG_NO_ADJ_FILTER = 2
CTG_NO_NODES = 4
CTG_DEFER_STATS = 8
CTG_ERR_STALE = -5
CTG_MAX_CHANNELS = 24
CTG_N_FEATURES = 10
CTG_NBINS = 40
CTG_WIDE_RECORD_WORDS = 48
CTG_MGPU_SAMPLES = 1024
CTG_MGPU_ROW_WORDS = 28
CTG_MGPU_MAX_WORLD = 32
CTG_IO_N5 = 0
CTG_IO_ZARR_DOT = 1
CTG_IO_ZARR_SLASH = 2
CTG_IO_RAW = 0
CTG_IO_GZIP = 1
CTG_IO_ZLIB = 2

_lock = threading.Lock()
_lib = None

c_i64p = ctypes.POINTER(ctypes.c_int64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_dblp = ctypes.POINTER(ctypes.c_double)
c_vp = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/ctg.h one to one
PROTOTYPES = {
    'ctg_version': (ctypes.c_int, []),
    'ctg_init': (ctypes.c_int, [ctypes.c_int]),
    'ctg_last_error': (ctypes.c_char_p, []),
    'ctg_device_count': (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    'ctg_rag_features': (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_int, ctypes.c_int, c_vp,
                                        c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                        ctypes.c_int, ctypes.c_int, c_vp, ctypes.POINTER(c_vp)]),
    'ctg_rag_blocks': (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp,
                                      ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_int, ctypes.c_int, c_vp, ctypes.POINTER(c_vp)]),
    'ctg_result_num_blocks': (ctypes.c_int, [c_vp]),
    'ctg_result_block_offsets': (ctypes.c_int, [c_vp, c_vp, c_vp]),
    'ctg_host_alloc': (c_vp, [ctypes.c_int64]),
    'ctg_host_free': (None, [c_vp]),
    'ctg_unique_labels': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_int, c_vp, ctypes.POINTER(c_vp)]),
    'ctg_merge_stats': (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_int, ctypes.c_int, c_vp, ctypes.POINTER(c_vp)]),
    'ctg_mgpu_slab': (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, c_vp, ctypes.c_int, c_vp]),
    'ctg_mgpu_sample': (ctypes.c_int, [c_vp, c_vp, c_vp]),
    'ctg_mgpu_split': (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, c_vp, c_vp]),
    'ctg_mgpu_pack': (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp]),
    'ctg_mgpu_merge': (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                      ctypes.c_double, c_vp, ctypes.POINTER(c_vp)]),
    'ctg_merge_feature_rows': (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, c_vp,
                                              ctypes.c_int, c_vp]),
    'ctg_unique_pairs': (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int, c_vp, ctypes.POINTER(c_vp)]),
    'ctg_unique_values': (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int, c_vp, ctypes.POINTER(c_vp)]),
    'ctg_map_edge_ids': (ctypes.c_int, [c_vp, ctypes.c_int64, c_vp, ctypes.c_int64, c_vp, ctypes.c_int, c_vp]),
    'ctg_result_num_edges': (ctypes.c_int64, [c_vp]),
    'ctg_result_num_nodes': (ctypes.c_int64, [c_vp]),
    'ctg_result_copy_edges': (ctypes.c_int, [c_vp, c_vp, ctypes.c_int]),
    'ctg_result_copy_nodes': (ctypes.c_int, [c_vp, c_vp, ctypes.c_int]),
    'ctg_result_copy_features': (ctypes.c_int, [c_vp, c_vp, ctypes.c_int]),
    'ctg_result_copy_stats': (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int]),
    'ctg_result_device_edges': (c_vp, [c_vp]),
    'ctg_result_device_features': (c_vp, [c_vp]),
    'ctg_result_info': (ctypes.c_int, [c_vp, c_i64p, c_i64p]),
    'ctg_free': (None, [c_vp]),
    'ctg_synth_volume': (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int64, c_vp, ctypes.c_int, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_double, c_vp]),
    'ctg_synth_affinities': (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int, c_vp, c_vp]),
    'ctg_filter_conv_axis': (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int, c_vp, ctypes.c_int, c_vp]),
    'ctg_filter_combine': (ctypes.c_int, [ctypes.c_int, c_vp, c_vp, c_vp, c_vp, ctypes.c_int64, c_vp]),
    'ctg_sym_eigenvalues': (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int64, c_vp, c_vp]),
    'ctg_trim': (ctypes.c_int, []),
    'ctg_io_read_box': (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       c_vp, c_vp, ctypes.c_int, c_vp, c_vp, c_vp, ctypes.c_int, c_vp]),
    'ctg_io_read_varlen': (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, c_vp,
                                          ctypes.c_int, c_vp, c_vp, ctypes.c_int]),
    'ctg_io_free': (None, [c_vp]),
    'ctg_io_cache_clear': (None, []),
    'ctg_io_cache_stats': (None, [ctypes.c_void_p]),
    'ctg_io_cache_drop': (None, [ctypes.c_char_p]),
    'ctg_io_write_chunks': (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int64, c_vp, c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int]),
    'ctg_set_profiling': (ctypes.c_int, [ctypes.c_int]),
    'ctg_last_timings': (ctypes.c_int, [c_dblp, ctypes.c_int]),
}


class BlockDesc(ctypes.Structure):
    """ctg_block_desc (include/ctg.h)."""
    _fields_ = [('label_offset', ctypes.c_int64), ('data_offset', ctypes.c_int64),
                ('shape', ctypes.c_int64 * 3), ('own_begin', ctypes.c_int64 * 3), ('own_end', ctypes.c_int64 * 3),
                ('graph_begin', ctypes.c_int64 * 3), ('graph_end', ctypes.c_int64 * 3)]


class CtgError(RuntimeError):
    """Raised for every non-zero ctg status (pybind11 raises RuntimeError for
    nifty's C++ exceptions; cluster_tasks.py:114-159 treats both as a failed
    job)."""


def load():
    """Load libctg.so and bind every prototype.  Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise CtgError(
                "libctg.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C cluster_tools_amd/csrc` (the HIP path has no CPU fallback)" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            if os.environ.get('CTG_LIB') and not hasattr(lib, name):
                continue   # an older A/B build (tools/ab_variants.py) without a newer entry point
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc, what=''):
    if rc != CTG_OK:
        msg = load().ctg_last_error()
        msg = msg.decode() if msg else 'unknown error'
        raise CtgError('%s failed (status %d): %s' % (what or 'ctg call', rc, msg))


_inited = set()


def init_device(device=None):
    """Bind the calling thread to ``device`` (default: torch's current device
    or 0) and create the per-device workspace."""
    lib = load()
    if device is None:
        # torch's current device when the caller already uses torch on the GPU;
        # otherwise CTG_DEVICE (default 0) -- a job process of the drop-in path
        # never imports torch (its import and runtime start cost seconds)
        torch = sys.modules.get('torch')
        if torch is not None and torch.cuda.is_initialized():
            device = torch.cuda.current_device()
        else:
            device = int(os.environ.get('CTG_DEVICE', '0'))
    check(lib.ctg_init(int(device)), 'ctg_init(%d)' % device)
    _inited.add(int(device))
    return int(device)
