"""ctypes binding of the C ABI in ``include/gsr.h`` and ``include/gsr_io.h``
(``gsviewer_amd/libgsr.so``).

The shared library is the product: there is no Python or CPU fallback.  If it
is missing or fails to load, every entry point raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
# GSR_LIB_PATH selects an alternative build (A/B experiments); default: in-tree.
_DEFAULT_LIB = os.path.join(_PKG, "libgsr.so")
LIB_PATH = os.environ.get("GSR_LIB_PATH") or _DEFAULT_LIB


def check_fresh(lib):
    """The in-tree library must be built from the sources beside it
    (_srcid.py): a stale .so raises instead of standing in for the tree.
    Skipped when the sources are absent (an installed package)."""
    from gsviewer_amd import _srcid
    if not os.path.isdir(_srcid.CSRC):
        return
    want = _srcid.source_digest()
    got = lib.gsr_source_digest()
    got = got.decode() if got else ""
    if got != want:
        raise RuntimeError(f"gsviewer_amd: {_DEFAULT_LIB} was built from other sources (digest {got}, tree {want}); "
                           "rebuild it with `python -m gsviewer_amd.build`")


class GsrCamera(ctypes.Structure):
    _fields_ = [
        ("view", ctypes.c_float * 16),
        ("proj", ctypes.c_float * 16),
        ("campos", ctypes.c_float * 3),
        ("hfovxy_focal", ctypes.c_float * 3),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
    ]


class GsrSettings(ctypes.Structure):
    _fields_ = [
        ("scale_modifier", ctypes.c_float),
        ("screen_scale", ctypes.c_float),
        ("render_mod", ctypes.c_int32),
        ("dc_factor", ctypes.c_float),
        ("extra_factor", ctypes.c_float),
        ("color_scale", ctypes.c_float * 3),
        ("rot_modifier", ctypes.c_float * 4),
        ("light_rotation", ctypes.c_float * 3),
        ("enable_aabb", ctypes.c_int32),
        ("enable_obb", ctypes.c_int32),
        ("cube_rotation", ctypes.c_float * 9),
        ("cube_min", ctypes.c_float * 3),
        ("cube_max", ctypes.c_float * 3),
        ("points_center", ctypes.c_float * 3),
        ("bg", ctypes.c_float * 3),
        ("t_min", ctypes.c_float),
        ("out_layout", ctypes.c_int32),
        ("blend", ctypes.c_int32),
    ]


class GsrFrameStats(ctypes.Structure):
    _fields_ = [
        ("n_gaussians", ctypes.c_int64),
        ("n_visible", ctypes.c_int64),
        ("n_instances", ctypes.c_int64),
        ("tiles_x", ctypes.c_int32),
        ("tiles_y", ctypes.c_int32),
    ]


class GsrPlySceneInfo(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("sh_dim", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("points_center", ctypes.c_float * 3),
        ("scale_factor", ctypes.c_float),
        ("bbox_center", ctypes.c_float * 3),
    ]


class GsrPlyInfo(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("sh_dim", ctypes.c_int32),
        ("format", ctypes.c_int32),
        ("n_properties", ctypes.c_int32),
        ("row_bytes", ctypes.c_int32),
        ("body_offset", ctypes.c_int64),
    ]


class GsrBox(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("cube_min", ctypes.c_double * 3),
        ("cube_max", ctypes.c_double * 3),
        ("rot_inv", ctypes.c_double * 9),
    ]


GSR_OK, GSR_ERR_INVALID, GSR_ERR_HIP, GSR_ERR_NOMEM, GSR_ERR_OVERFLOW = 0, -1, -2, -3, -4  # gsr_status
GSR_PLY_BINARY_LE, GSR_PLY_BINARY_BE, GSR_PLY_ASCII = 0, 1, 2
GSR_BOX_NONE, GSR_BOX_AABB, GSR_BOX_OBB = 0, 1, 2

# name -> (restype, argtypes); every symbol declared in include/gsr.h and include/gsr_io.h
_P = ctypes.c_void_p
SIGNATURES = {
    "gsr_abi_version": (ctypes.c_int, []),
    "gsr_last_error": (ctypes.c_char_p, []),
    "gsr_source_digest": (ctypes.c_char_p, []),
    "gsr_settings_default": (None, [ctypes.POINTER(GsrSettings)]),
    "gsr_scene_create": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_int64, ctypes.c_int32, _P,
                                        ctypes.POINTER(_P)]),
    "gsr_scene_create_flat": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int32, _P, ctypes.POINTER(_P)]),
    "gsr_scene_destroy": (ctypes.c_int, [_P]),
    "gsr_scene_count": (ctypes.c_int64, [_P]),
    "gsr_scene_sh_dim": (ctypes.c_int32, [_P]),
    "gsr_context_create": (ctypes.c_int, [ctypes.POINTER(_P)]),
    "gsr_context_destroy": (ctypes.c_int, [_P]),
    "gsr_context_reserve": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _P]),
    "gsr_context_workspace": (ctypes.c_int64, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "gsr_workspace_size": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64]),
    "gsr_context_attach_workspace": (ctypes.c_int, [_P, _P, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int32,
                                                    ctypes.c_int32, ctypes.c_int64, _P]),
    "gsr_render": (ctypes.c_int, [_P, _P, ctypes.POINTER(GsrCamera), ctypes.POINTER(GsrSettings), _P, _P, _P]),
    "gsr_render_begin": (ctypes.c_int, [_P, _P, ctypes.POINTER(GsrCamera), ctypes.POINTER(GsrSettings), _P, _P, _P]),
    "gsr_render_finish": (ctypes.c_int, [_P, _P]),
    "gsr_render_begin_views": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int32, _P, ctypes.POINTER(GsrCamera),
                                              ctypes.POINTER(GsrSettings), ctypes.POINTER(_P), ctypes.POINTER(_P),
                                              _P]),
    "gsr_render_begin_sort": (ctypes.c_int, [_P, _P]),
    "gsr_render_begin_sorts": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int32, _P]),
    "gsr_render_finish_views": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int32, _P]),
    "gsr_render_wait_counts": (ctypes.c_int, [_P]),
    "gsr_context_stats": (ctypes.c_int, [_P, ctypes.POINTER(GsrFrameStats)]),
    "gsr_sort_depth": (ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.c_float * 16), _P, _P]),
    "gsr_debug_host_times": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "gsr_debug_sort_pairs": (ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _P, _P, _P]),
    "gsr_debug_copy": (ctypes.c_int64, [_P, ctypes.c_int32, _P, ctypes.c_int64, _P]),
    "gsr_debug_stall": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "gsr_context_knob": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "gsr_context_set_profiling": (ctypes.c_int, [_P, ctypes.c_int32]),
    "gsr_context_stage_times": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "gsr_context_group_spans": (ctypes.c_int64, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]),
    "gsr_context_group_times": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                               ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    # gsr_io.h
    "gsr_ply_probe": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(GsrPlyInfo)]),
    "gsr_ply_read": (ctypes.c_int, [ctypes.c_char_p, _P, _P, _P, _P, _P, ctypes.c_int32]),
    "gsr_scene_load_ply": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_float, ctypes.c_int32, _P, ctypes.POINTER(_P),
                                          ctypes.POINTER(GsrPlySceneInfo)]),
    "gsr_scene_read_flat": (ctypes.c_int, [_P, _P, _P]),
    "gsr_ply_write_3dgs": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, _P, ctypes.c_int64, ctypes.c_int32]),
    "gsr_points_center": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.POINTER(ctypes.c_float * 3), _P]),
    "gsr_export_select": (ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_float * 3),
                                         ctypes.POINTER(GsrBox), _P, ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_float * 6), ctypes.POINTER(ctypes.c_int32), _P]),
}

STAGES = ["cull", "preprocess", "depth_sort", "binning", "tile_sort", "tile_ranges", "composite", "sync", "merge"]

GSR_DEBUG_RECORDS, GSR_DEBUG_DEPTH_ORDER, GSR_DEBUG_TILE_RANGES, GSR_DEBUG_TILE_LIST = 0, 1, 2, 3

ABI_VERSION = 7
MAX_VIEWS = 8  # GSR_MAX_VIEWS (include/gsr.h)

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load (once) and return the library handle.  Raises RuntimeError."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"gsviewer_amd: HIP library {path} is missing; build it with "
                "`python -m gsviewer_amd.build` (there is no CPU fallback)")
        # Share the HIP runtime torch already loaded (same soname libamdhip64.so.7).
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is part of the image
            pass
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise RuntimeError(f"gsviewer_amd: failed to load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.gsr_abi_version() != ABI_VERSION:
            raise RuntimeError("gsviewer_amd: ABI version mismatch between libgsr.so and bindings")
        if path == _DEFAULT_LIB:
            check_fresh(lib)
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().gsr_last_error()
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def default_settings() -> GsrSettings:
    s = GsrSettings()
    load().gsr_settings_default(ctypes.byref(s))
    return s
