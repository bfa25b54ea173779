"""ctypes binding of ``libflame_amd.so`` (the C ABI in ``include/flame_amd.h``).

The library is REQUIRED: importing the compute entry points without it raises
immediately -- there is no CPU or eager-PyTorch fallback for the hot path.
"""
from __future__ import annotations

import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLAME_AMD_LIB", os.path.join(PKG, "libflame_amd.so"))

# constants mirrored from include/flame_amd.h
FLAME_OK, FLAME_EINVAL, FLAME_EHIP, FLAME_ENOTSUP = 0, 1, 2, 3
FLAME_F32, FLAME_BF16, FLAME_F16, FLAME_F64, FLAME_I64, FLAME_I32 = range(6)
FLAME_U8, FLAME_I8, FLAME_I16, FLAME_BOOL = range(6, 10)       # flame_elementwise only
FLAME_AGG_INIT_FIRST = 1
FLAME_AGG_SEG_RATES = 2
FLAME_AGG_XCD_MAP = 4
FLAME_FEDADAM, FLAME_FEDYOGI, FLAME_FEDADAGRAD = 0, 1, 2
FLAME_OPT_STATE_ZERO = 1
FLAME_OPT_XCD_MAP = 2
FLAME_SEG_UNALIGNED = 1
FLAME_SEG_CUR_IS_AVG = 2
FLAME_HIER_TOP_ACCUM = 1
FLAME_HIER_TOP_APPLY = 2
FLAME_HIER_MID_READONLY = 4
FLAME_HIER_SYNC = 8
FLAME_DYN_W, FLAME_DYN_AVG, FLAME_DYN_HIN, FLAME_DYN_HOUT, FLAME_DYN_MEAN = 1, 2, 4, 8, 16
HIER_SEGMENT_INT64S = 8  # sizeof(flame_hier_segment) / 8
DYN_SEGMENT_INT64S = 8  # sizeof(flame_dyn_segment) / 8
SEGMENT_INT64S = 10  # sizeof(flame_segment) / 8
TILE_COPY_INT64S = 4  # sizeof(flame_tile_copy) / 8
FLAME_TILE_BYTES = 4096

# every symbol include/flame_amd.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "flame_abi_version", "flame_last_error", "flame_chunk_elems", "flame_scale_add_chunk_elems",
    "flame_agg_reduce", "flame_agg_reduce_argmeta", "flame_agg_argmeta_max_bytes", "flame_fedopt_reduce_adapt", "flame_fedopt_reduce_adapt_argmeta", "flame_fedopt_chain", "flame_fedbuff_scale_add", "flame_hier_fedbuff", "flame_hier_fedbuff_argmeta",
    "flame_hier_resident_per_cu", "flame_feddyn_round", "flame_elementwise", "flame_elementwise_segments", "flame_synth_fill",
    "flame_host_register", "flame_host_unregister", "flame_host_device_pointer",
    "flame_slab_write", "flame_slab_write_2d",
    "flame_launch_branches", "flame_launch_branch_name", "flame_launch_branch_count",
)


class FlameError(RuntimeError):
    """A nonzero FLAME_E* status returned by the native library."""


_lib = None


def lib() -> ctypes.CDLL:
    """Load the native library (raises ImportError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"flame_amd native library not found at {LIB_PATH}; build it with "
            "`python -m flame_amd.build` (hipcc --offload-arch=gfx950). There is no fallback.")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32, u64, f32 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint,
                                   ctypes.c_uint64, ctypes.c_float)
    L.flame_abi_version.restype = ctypes.c_int
    L.flame_abi_version.argtypes = []
    L.flame_last_error.restype = ctypes.c_char_p
    L.flame_last_error.argtypes = []
    L.flame_chunk_elems.restype = i64
    L.flame_chunk_elems.argtypes = [ctypes.c_int]
    L.flame_scale_add_chunk_elems.restype = i64
    L.flame_scale_add_chunk_elems.argtypes = [ctypes.c_int]
    L.flame_agg_reduce.restype = ctypes.c_int
    L.flame_agg_reduce.argtypes = [ctypes.c_int, u32, vp, i32, i64, vp, i32, vp, vp, vp]
    L.flame_agg_reduce_argmeta.restype = ctypes.c_int
    L.flame_agg_reduce_argmeta.argtypes = [ctypes.c_int, u32, vp, i64, i32, i64, i32, i64, i64, i64, vp]
    L.flame_agg_argmeta_max_bytes.restype = i64
    L.flame_agg_argmeta_max_bytes.argtypes = []
    L.flame_fedopt_reduce_adapt.restype = ctypes.c_int
    L.flame_fedopt_reduce_adapt.argtypes = [ctypes.c_int, ctypes.c_int, u32, vp, i32, i64, vp, i32, vp] + [f32] * 6 + [vp]
    L.flame_fedopt_chain.restype = ctypes.c_int
    L.flame_fedopt_chain.argtypes = [ctypes.c_int, ctypes.c_int, u32, vp, i32, i64, vp, i32, vp, vp] + [f32] * 6 + [vp]
    L.flame_fedopt_reduce_adapt_argmeta.restype = ctypes.c_int
    L.flame_fedopt_reduce_adapt_argmeta.argtypes = [ctypes.c_int, ctypes.c_int, u32, vp, i64, i32, i64, i32, i64,
                                                    i64] + [f32] * 6 + [vp]
    L.flame_fedbuff_scale_add.restype = ctypes.c_int
    L.flame_fedbuff_scale_add.argtypes = [ctypes.c_int, vp, i32, i64, i64, vp]
    L.flame_hier_fedbuff.restype = ctypes.c_int
    L.flame_hier_fedbuff.argtypes = [ctypes.c_int, u32, vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, vp, f32, vp]
    L.flame_hier_fedbuff_argmeta.restype = ctypes.c_int
    L.flame_hier_fedbuff_argmeta.argtypes = [ctypes.c_int, u32, vp, i64, i32, i64, i32, i32] + [i64] * 6 + [f32, vp]
    L.flame_hier_resident_per_cu.restype = ctypes.c_int
    L.flame_hier_resident_per_cu.argtypes = [ctypes.c_int, u32, i32]
    L.flame_feddyn_round.restype = ctypes.c_int
    L.flame_feddyn_round.argtypes = [ctypes.c_int, vp, i32, i64, vp, vp, i32, i32, ctypes.c_double,
                                     ctypes.c_double, vp]
    L.flame_elementwise.restype = ctypes.c_int
    L.flame_elementwise.argtypes = [vp, i32, vp, i32, i64, vp]
    L.flame_elementwise_segments.restype = ctypes.c_int
    L.flame_elementwise_segments.argtypes = [vp, i32, vp, i32, vp, i32, i64, vp]
    L.flame_synth_fill.restype = ctypes.c_int
    L.flame_synth_fill.argtypes = [ctypes.c_int, vp, i64, u64, u64, i64, f32, vp]
    L.flame_host_register.restype = ctypes.c_int
    L.flame_host_register.argtypes = [vp, u64]
    L.flame_host_unregister.restype = ctypes.c_int
    L.flame_host_unregister.argtypes = [vp]
    L.flame_host_device_pointer.restype = ctypes.c_int
    L.flame_host_device_pointer.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p)]
    L.flame_slab_write.restype = ctypes.c_int
    L.flame_slab_write.argtypes = [vp, i32, vp]
    L.flame_slab_write_2d.restype = ctypes.c_int
    L.flame_slab_write_2d.argtypes = [vp, i32, vp]
    L.flame_launch_branches.restype = i32
    L.flame_launch_branches.argtypes = []
    L.flame_launch_branch_name.restype = ctypes.c_char_p
    L.flame_launch_branch_name.argtypes = [i32]
    L.flame_launch_branch_count.restype = i64
    L.flame_launch_branch_count.argtypes = [i32]
    if L.flame_abi_version() != 1:
        raise ImportError(f"flame_amd ABI mismatch: library {L.flame_abi_version()} != 1")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != FLAME_OK:
        msg = lib().flame_last_error().decode(errors="replace")
        raise FlameError(f"flame_amd status {rc}: {msg}")


def launch_branch_counts() -> dict:
    """{branch name: successful launches so far} for every launch branch of the C ABI
    (flame_launch_branches); which kernel instantiation each call took."""
    L = lib()
    return {L.flame_launch_branch_name(i).decode(): int(L.flame_launch_branch_count(i))
            for i in range(L.flame_launch_branches())}
