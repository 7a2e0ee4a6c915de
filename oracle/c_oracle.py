"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/gl_oracle.c.

Takes the same uniform dict as oracle/gl_oracle.py (default_uniforms) and
returns the same image (mode 'float' or 'gl8'), computed multithreaded.
"""
import ctypes
import os

import numpy as np

from . import gl_oracle as O
from .build_oracle import OUT, build

F = np.float32


class _U(ctypes.Structure):
    _fields_ = [("view", ctypes.c_float * 16), ("proj", ctypes.c_float * 16), ("hfov", ctypes.c_float * 3),
                ("campos", ctypes.c_float * 3), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("gsf", ctypes.c_float), ("sdsf", ctypes.c_float), ("dc_factor", ctypes.c_float),
                ("extra_factor", ctypes.c_float), ("cscale", ctypes.c_float * 3), ("render_mod", ctypes.c_int32),
                ("rotmod", ctypes.c_float * 4), ("lcos", ctypes.c_float * 3), ("lsin", ctypes.c_float * 3),
                ("pcenter", ctypes.c_float * 3), ("enable_aabb", ctypes.c_int32), ("enable_obb", ctypes.c_int32),
                ("obb_inv", ctypes.c_float * 9), ("cmin", ctypes.c_float * 3), ("cmax", ctypes.c_float * 3),
                ("bg", ctypes.c_float * 3)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(OUT):
            build()
        _lib = ctypes.CDLL(OUT)
        _lib.oracle_render.restype = ctypes.c_int64
        _lib.oracle_render.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(_U),
                                       ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        _lib.oracle_sort_depth.restype = ctypes.c_int64
        _lib.oracle_sort_depth.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int32]
    return _lib


def _arr(dst, v):
    dst[:] = [float(x) for x in np.asarray(v, F).reshape(-1)]


def to_struct(U):
    u = _U()
    _arr(u.view, U["view"]); _arr(u.proj, U["proj"]); _arr(u.hfov, U["hfovxy_focal"]); _arr(u.campos, U["cam_pos"])
    u.width, u.height = U["width"], U["height"]
    u.gsf, u.sdsf = float(U["gaussian_scale_factor"]), float(U["screen_display_scale_factor"])
    u.dc_factor, u.extra_factor = float(U["dc_factor"]), float(U["extra_factor"])
    _arr(u.cscale, U["color_scale_factors"])
    u.render_mod = int(U["render_mod"])
    _arr(u.rotmod, U["rot_modifier"])
    c, s = O.light_rotation_cs(U["light_rotation"])
    _arr(u.lcos, c); _arr(u.lsin, s)
    _arr(u.pcenter, U["points_center"])
    u.enable_aabb, u.enable_obb = int(U["enable_aabb"]), int(U["enable_obb"])
    _arr(u.obb_inv, O.obb_inverse(U["cube_rotation"]))
    _arr(u.cmin, U["cubeMin"]); _arr(u.cmax, U["cubeMax"]); _arr(u.bg, U["bg"])
    return u


def render(flat, sh_dim, U, mode="float", threads=0, return_order=False):
    flat = np.ascontiguousarray(flat, F)
    n = flat.shape[0]
    img = np.empty((U["height"], U["width"], 3), F)
    order = np.empty(max(n, 1), np.int32) if return_order else None
    u = to_struct(U)
    m = lib().oracle_render(flat.ctypes.data, n, sh_dim, ctypes.byref(u), 1 if mode == "gl8" else 0,
                            img.ctypes.data, order.ctypes.data if order is not None else None, int(threads))
    if m < 0:
        raise MemoryError("oracle_render")
    if return_order:
        return img, order[:m]
    return img


def sort_depth(xyz, view, threads=0):
    """renderer_ogl.py:16-26 _sort_gaussian_cpu: ascending view z, ties by id."""
    xyz = np.ascontiguousarray(xyz, F)
    v = np.ascontiguousarray(view, F).reshape(16)
    out = np.empty(len(xyz), np.int32)
    if lib().oracle_sort_depth(xyz.ctypes.data, len(xyz), v.ctypes.data, out.ctypes.data, int(threads)) < 0:
        raise MemoryError("oracle_sort_depth")
    return out
