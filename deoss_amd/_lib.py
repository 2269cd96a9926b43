"""Loader for ``libdeoss_merkle.so`` (the HIP/gfx950 Merkle path behind include/deoss_merkle.h).

There is no CPU fallback anywhere in this package: if the shared library is missing, or no GPU
is visible, calls raise :class:`DeossMerkleError`.  The library is built in-tree by
``__graft_entry__.build()`` (or ``python -m deoss_amd.build``).
"""
from __future__ import annotations

import ctypes
import os
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libdeoss_merkle.so"
# DEOSS_MERKLE_LIB: load another build of the same library (a tuning variant, a sanitizer build)
LIB_PATH = os.environ.get("DEOSS_MERKLE_LIB") or os.path.join(PKG_DIR, LIB_NAME)

DM_OK = 0
DM_ERR_EMPTY = -1
DM_ERR_INVALID = -2
DM_ERR_HIP = -3
DM_ERR_RCCL = -4
DM_ERR_NOMEM = -5
DM_ERR_IO = -6
DM_ERR_NODEV = -7

# Every symbol include/deoss_merkle.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = (
    "dm_create", "dm_create_lanes", "dm_destroy", "dm_strerror", "dm_last_error", "dm_device_count",
    "dm_lane_count", "dm_gpu_count", "dm_keep_claimed", "dm_can_shard",
    "dm_new_hash_tree", "dm_root_chunks", "dm_root_buffer", "dm_root_batch",
    "dm_root_device", "dm_root_device_async", "dm_subtree_device_async", "dm_finish_device_async",
    "dm_root_batch_device_async", "dm_fill_synthetic_async", "dm_read_probe_async", "dm_host_alloc",
    "dm_host_free", "dm_set_leaf_kernel", "dm_leaf_kernel_for",
    "dm_set_timing", "dm_stream_open", "dm_stream_write", "dm_stream_close", "dm_stream_abort",
    "dm_stream_error",
    "dm_timing_summary",
    "dm_rs_create", "dm_rs_destroy", "dm_rs_matrix", "dm_rs_encode", "dm_rs_encode_buffer", "dm_rs_reconstruct",
    "dm_rs_verify", "dm_rs_encode_device_async", "dm_rs_reconstruct_device_async",
    "dm_process_device_async", "dm_process_buffer", "dm_process_batch", "dm_full_processing", "dm_fragment_lookup",
    "dm_pstream_open", "dm_pstream_write", "dm_pstream_close", "dm_pstream_abort",
    "dm_tree_node_count", "dm_tree_depth", "dm_tree_levels_device_async", "dm_tree_levels",
    "dm_merkle_paths_device_async", "dm_merkle_paths", "dm_verify_paths_device_async", "dm_verify_paths",
    "dm_verify_object_device_async",
    "dm_batcher_create", "dm_batcher_destroy", "dm_batcher_root", "dm_batcher_process", "dm_batcher_stats",
    "dm_batcher_last_error",
    "dm_plan_shards", "dm_plan_route", "dm_route_constants", "dm_pstream_stats", "dm_exchange_timing", "dm_last_call_devices",
)


class DeossMerkleError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


_lock = threading.Lock()
_lib = None


def _declare(L: ctypes.CDLL) -> None:
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    pvp, pu64 = ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)
    sigs = {
        "dm_create": ([ctypes.POINTER(vp), ctypes.POINTER(i32), i32], i32),
        "dm_create_lanes": ([ctypes.POINTER(vp), ctypes.POINTER(i32), i32, i32], i32),
        "dm_lane_count": ([vp], i32),
        "dm_destroy": ([vp], None),
        "dm_strerror": ([i32], ctypes.c_char_p),
        "dm_last_error": ([vp], ctypes.c_char_p),
        "dm_device_count": ([vp], i32),
        "dm_gpu_count": ([], i32),
        "dm_keep_claimed": ([i32, pu64], i32),
        "dm_can_shard": ([vp], i32),
        "dm_new_hash_tree": ([vp, ctypes.POINTER(ctypes.c_char_p), u64, vp, vp], i32),
        "dm_root_chunks": ([vp, pvp, pu64, u64, vp, vp], i32),
        "dm_root_buffer": ([vp, vp, u64, u64, vp, vp], i32),
        "dm_root_batch": ([vp, pvp, pu64, u64, u64, vp], i32),
        "dm_root_device": ([vp, vp, u64, u64, vp], i32),
        "dm_root_device_async": ([vp, vp, u64, u64, vp, vp, vp], i32),
        "dm_subtree_device_async": ([vp, vp, u64, u64, u32, vp, pu64, vp], i32),
        "dm_finish_device_async": ([vp, vp, u64, i32, vp, vp], i32),
        "dm_root_batch_device_async": ([vp, pvp, pu64, u64, u64, vp, vp], i32),
        "dm_fill_synthetic_async": ([vp, vp, u64, u64, u64, vp], i32),
        "dm_read_probe_async": ([vp, vp, u64, vp, vp], i32),
        "dm_host_alloc": ([u64, ctypes.POINTER(vp)], i32),
        "dm_host_free": ([vp], None),
        "dm_stream_open": ([vp, u64, ctypes.POINTER(vp)], i32),
        "dm_stream_write": ([vp, vp, u64], i32),
        "dm_stream_close": ([vp, vp, u64, pu64, vp], i32),
        "dm_stream_abort": ([vp], None),
        "dm_stream_error": ([vp], ctypes.c_char_p),
        "dm_set_leaf_kernel": ([vp, i32], i32),
        "dm_leaf_kernel_for": ([vp, u64], i32),
        "dm_set_timing": ([vp, i32], i32),
        "dm_timing_summary": ([vp, pu64, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double)], i32),
        "dm_rs_create": ([vp, i32, i32, ctypes.POINTER(vp)], i32),
        "dm_rs_destroy": ([vp], None),
        "dm_rs_matrix": ([vp, vp], i32),
        "dm_rs_encode": ([vp, pvp, pvp, u64], i32),
        "dm_rs_encode_buffer": ([vp, vp, u64, vp, pu64], i32),
        "dm_rs_reconstruct": ([vp, pvp, vp, u64], i32),
        "dm_rs_verify": ([vp, pvp, u64, ctypes.POINTER(i32)], i32),
        "dm_rs_encode_device_async": ([vp, vp, u64, vp, u64, u64, u64, vp], i32),
        "dm_rs_reconstruct_device_async": ([vp, pvp, vp, u64, vp], i32),
        "dm_process_device_async": ([vp, vp, u64, u64, vp, vp, vp, vp, vp], i32),
        "dm_process_buffer": ([vp, vp, u64, u64, vp, vp, vp, vp], i32),
        "dm_process_batch": ([vp, pvp, pu64, u64, u64, pvp, pvp, pvp, vp], i32),
        "dm_full_processing": ([vp, ctypes.c_char_p, ctypes.c_char_p, u64, i32, vp, vp, u64, pu64, vp], i32),
        "dm_fragment_lookup": ([vp, ctypes.c_char_p, u64, vp, vp, u64, ctypes.POINTER(i32), pu64,
                                ctypes.POINTER(i32)], i32),
        "dm_pstream_open": ([vp, u64, ctypes.c_char_p, i32, ctypes.POINTER(vp)], i32),
        "dm_pstream_write": ([vp, vp, u64], i32),
        "dm_pstream_close": ([vp, vp, vp, u64, pu64, vp], i32),
        "dm_pstream_abort": ([vp], None),
        "dm_tree_node_count": ([u64], u64),
        "dm_tree_depth": ([u64], u32),
        "dm_tree_levels_device_async": ([vp, vp, u64, vp, vp], i32),
        "dm_tree_levels": ([vp, vp, u64, vp], i32),
        "dm_merkle_paths_device_async": ([vp, vp, vp, u64, vp, u64, vp, vp, vp], i32),
        "dm_merkle_paths": ([vp, vp, u64, vp, u64, vp, vp], i32),
        "dm_verify_paths_device_async": ([vp, pvp, pu64, u64, vp, vp, u32, vp, u64, vp, vp], i32),
        "dm_verify_paths": ([vp, pvp, pu64, u64, vp, vp, u32, vp, u64, vp], i32),
        "dm_verify_object_device_async": ([vp, vp, u64, u64, vp, vp, u32, vp, u64, vp, vp], i32),
        "dm_batcher_create": ([ctypes.POINTER(i32), i32, i32, u64, i32, i32, i32, u64, u64, u32, ctypes.POINTER(vp)],
                              i32),
        "dm_batcher_destroy": ([vp], None),
        "dm_batcher_root": ([vp, vp, u64, vp, vp], i32),
        "dm_batcher_process": ([vp, vp, u64, vp, vp, vp, vp], i32),
        "dm_batcher_stats": ([vp, pu64, pu64, pu64], i32),
        "dm_batcher_last_error": ([], ctypes.c_char_p),
        "dm_pstream_stats": ([vp, pu64, pu64], i32),
        "dm_exchange_timing": ([vp, pu64, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(i32)], i32),
        "dm_last_call_devices": ([vp, ctypes.POINTER(i32), ctypes.POINTER(i32), i32, ctypes.POINTER(i32)], i32),
        "dm_plan_shards": ([u64, i32, ctypes.POINTER(u32), pu64, pu64, pu64], i32),
        "dm_plan_route": ([u64, u64, u64, i32, i32, i32, i32, i32, i32, ctypes.POINTER(ctypes.c_double)], i32),
        "dm_route_constants": ([vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)], i32),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res


def _share_torch_runtime() -> None:
    """Let PyTorch's HIP runtime load first when PyTorch is installed.

    torch ships its own libamdhip64 with the same soname (libamdhip64.so.7) as /opt/rocm's, so
    one process gets ONE runtime: whichever is loaded first.  The library then uses torch's
    (device pointers and hipStream_t handles from torch stay valid in dm_* calls); loaded the
    other way round, torch.cuda finds a runtime it was not built against and reports no GPU.
    Outside Python (Go, C++) the library uses /opt/rocm's runtime as linked."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the HIP library; raises (never falls back) when it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise DeossMerkleError(
                DM_ERR_NODEV,
                f"{path} not built: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
        _share_torch_runtime()
        L = ctypes.CDLL(path)
        _declare(L)
        _lib = L
        return L


def strerror(code: int) -> str:
    return load_library().dm_strerror(code).decode()
