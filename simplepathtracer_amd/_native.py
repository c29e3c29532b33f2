"""ctypes binding of libspt_hip.so (include/spt_hip.h).

The product path is native: every render goes through the HIP kernels in this
library.  There is no CPU fallback -- if the library cannot be loaded, import
of the renderer fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", os.environ.get("SPT_LIB", "libspt_hip.so"))
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "spt_hip.h")

ABI_VERSION = 11  # SPT_ABI_VERSION of include/spt_hip.h
SPT_OK = 0
STATUS_NAMES = {0: "SPT_OK", 1: "SPT_ERR_ARG", 2: "SPT_ERR_STATE", 3: "SPT_ERR_HIP", 4: "SPT_ERR_NOMEM",
                5: "SPT_ERR_NODEVICE", 6: "SPT_ERR_TIMEOUT"}
MODE_SEGMENT, MODE_TASK = 0, 1
TREE_AUTO = 0xFFFFFFFF  # spt_set_cluster_tree default
CLUSTER_AUTO = 0xFFFFFFFF  # spt_set_cluster_size default
ENGINE_MEGAKERNEL, ENGINE_WAVEFRONT = 0, 1
SELFTEST_COLS = 16


class SptError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [
        ("samples", ctypes.c_uint64),
        ("casts", ctypes.c_uint64),
        ("dropped", ctypes.c_uint64),
        ("launches", ctypes.c_uint64),
        ("render_ms", ctypes.c_double),
        ("fold_ms", ctypes.c_double),
        ("last_render_ms", ctypes.c_double),
        ("grid_blocks", ctypes.c_uint32),
        ("block_threads", ctypes.c_uint32),
        ("render_busy_ms", ctypes.c_double),
        ("diag", ctypes.c_uint64 * 26),  # SPT_DIAG_WORDS
        ("batches", ctypes.c_uint64),
        ("batched_calls", ctypes.c_uint64),
        ("svc_sessions", ctypes.c_uint64),
        ("svc_jobs", ctypes.c_uint64),
        ("svc_watchdog_exits", ctypes.c_uint64),
        ("svc_kernel_ms", ctypes.c_double),
        ("svc_running", ctypes.c_uint32),
        ("svc_grid_blocks", ctypes.c_uint32),
        ("svc_flow_restarts", ctypes.c_uint64),
        ("svc_closing_restarts", ctypes.c_uint64),
        ("prim_list_blocks", ctypes.c_uint32),
        ("prim_list_entries", ctypes.c_uint32),
        ("prim_list_build_ms", ctypes.c_double),
        ("prim_list_builds", ctypes.c_uint64),
        ("accel_build_ms", ctypes.c_double),
    ]


def build(force: bool = False) -> str:
    """Compile the gfx950 library in-tree (hipcc via the csrc Makefile)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-j4", "-C", os.path.join(PKG_DIR, "csrc")], check=True)
    return LIB_PATH


def declared_symbols() -> list[str]:
    """Function names declared in include/spt_hip.h."""
    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"^\s*(?:SPT_API\s+)?(?:int|void|const char \*)\s*\*?\s*(spt_[a-z0-9_]+)\s*\(", text,
                                 re.M)))


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    P, I = ctypes.c_void_p, ctypes.c_int
    u32, u64 = ctypes.c_uint32, ctypes.c_uint64
    sig = {
        "spt_abi_version": ([], I),
        "spt_device_count": ([P], I),
        "spt_ctx_create": ([I, P], I),
        "spt_ctx_create_multi": ([P, u32, P], I),
        "spt_ctx_devices": ([P, P, P], I),
        "spt_render_frame": ([P, I, P, P], I),
        "spt_ctx_destroy": ([P], None),
        "spt_last_error": ([P], ctypes.c_char_p),
        "spt_set_scene": ([P, P, P, P, P, P, u32], I),
        "spt_set_camera": ([P, P, P, P], I),
        "spt_set_params": ([P, u32, u32, u32, u32, u64], I),
        "spt_set_workspace": ([P, u64], I),
        "spt_set_cluster_size": ([P, u32], I),
        "spt_set_cluster_tree": ([P, u32], I),
        "spt_set_reserved_cus": ([P, u32], I),
        "spt_prepare_dropin": ([P], I),
        "spt_set_engine": ([P, I], I),
        "spt_accel_check": ([P, P, u32, u32, u32, P], I),
        "spt_prim_lists_check": ([P, P, u32, P, P, u32, u32, u32, P, P, P, P, u32, P], I),
        "spt_render_segment": ([P, u32, u32, u32, u32, P, P], I),
        "spt_render_segment_task": ([P, u32, u32, u32, u32, P, P], I),
        "spt_render_rows_async": ([P, I, u32, u32, u32, u32, u32, u32, u32, P, P, P], I),
        "spt_rows_count": ([u32, u32, u32, u32, u32, P], I),
        "spt_assemble_rows_async": ([P, P, u32, u32, u32, u32, u32, u32, u32, P, P, P], I),
        "spt_synchronize": ([P], I),
        "spt_render_samples": ([P, I, u32, u32, u32, u32, P], I),
        "spt_get_stats": ([P, P], I),
        "spt_reset_stats": ([P], I),
        "spt_scene_generate_random": ([u32, u32, P, P, P, P, P, P], I),
        "spt_scene_generate_random_rows": ([u32, ctypes.c_float, u32, P, P, P, P, P, P], I),
        "spt_scene_init_reference": ([u32, P, P, P, P, P, P], I),
        "spt_scene_generate_stress": ([u32, u32, P, P, P, P, P], I),
        "spt_camera_basis": ([P, P, P, P], I),
        "spt_save_bmp": ([ctypes.c_char_p, u32, u32, u32, P], I),
        "spt_render_progressive": ([P, I, u32, u32, u32, u32, u32, P, P, P, P], I),
        "spt_pin_host": ([P, P, ctypes.c_size_t], I),
        "spt_unpin_host": ([P, P], I),
        "spt_selftest_numerics": ([P, P, P, P, u32, P], I),
        "spt_service_start": ([P], I),
        "spt_service_stop": ([P], I),
        "spt_tiles_create": ([P, ctypes.c_char_p, u32, u32, u64, u32, P], I),
        "spt_tiles_handle": ([P, P], I),
        "spt_tiles_attach": ([P, P], I),
        "spt_tiles_unlink": ([P], I),
        "spt_tiles_buffer": ([P, u64, P], I),
        "spt_tiles_send_async": ([P, u64, P, P], I),
        "spt_tiles_send_range_async": ([P, u64, P, u64, u64, P], I),
        "spt_task_range": ([u32, u32, u32, u32, P, P], I),
        "spt_render_task_range_async": ([P, u32, u32, P, P], I),
        "spt_tiles_recv_async": ([P, u64, P], I),
        "spt_tiles_release_async": ([P, u64, P], I),
        "spt_tiles_destroy": ([P], None),
        "spt_tiles_abort": ([P], I),
        "spt_service_set_full_grid": ([P, u32], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.spt_abi_version() != ABI_VERSION:
        raise ImportError("libspt_hip.so ABI version mismatch")
    _lib = L
    return L


def check(code: int, ctx=None) -> None:
    if code != SPT_OK:
        msg = lib().spt_last_error(ctx)
        raise SptError(code, msg.decode() if msg else "")
