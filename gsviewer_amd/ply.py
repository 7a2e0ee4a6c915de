"""Scene ingestion and export with the reference's interface
(SURVEY.md §8(f) rows 2-3), over the C ABI in include/gsr_io.h.

``load_ply(path)`` mirrors ``util_gau.load_ply`` (util_gau.py:236-305).  The
vertex columns are parsed by libgsr's multithreaded memory-mapped reader (no
plyfile/pandas).  The activations use the reference's own NumPy expressions,
so a float32 PLY loads bit-identically.

``export_ply(...)`` mirrors ``util_gau.export_ply`` (util_gau.py:388-430) for
3DGS sources:
  * points_center, the AABB/OBB mask, the bbox of the as-loaded positions and
    the row compaction run on the GPU;
  * gsconverter's crop-and-write becomes libgsr's row writer.
It returns True/False as the reference does.  Other gsconverter formats are
out of scope.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from .camera import euler_to_rotation_matrix
from .gaussian_data import GaussianData


def probe(path: str) -> _lib.GsrPlyInfo:
    info = _lib.GsrPlyInfo()
    _lib.check(_lib.load().gsr_ply_probe(os.fsencode(path), ctypes.byref(info)), f"gsr_ply_probe({path})")
    return info


def read_raw(path: str, n_threads: int = 0):
    """Pre-activation columns (float32): xyz [N,3], rot [N,4], scale [N,3],
    opacity [N,1], sh [N,3|48] in load_ply's coefficient-major RGB layout."""
    info = probe(path)
    n = int(info.n)
    xyz = np.empty((n, 3), np.float32)
    rot = np.empty((n, 4), np.float32)
    scale = np.empty((n, 3), np.float32)
    opacity = np.empty((n, 1), np.float32)
    sh = np.empty((n, int(info.sh_dim)), np.float32)
    ptr = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    _lib.check(_lib.load().gsr_ply_read(os.fsencode(path), ptr(xyz), ptr(rot), ptr(scale), ptr(opacity), ptr(sh),
                                        int(n_threads)), f"gsr_ply_read({path})")
    return xyz, rot, scale, opacity, sh


def load_ply(path: str, n_threads: int = 0) -> GaussianData:
    """util_gau.load_ply: native parse + the reference's activations (util_gau.py:297-303)."""
    xyz, rots, scales, opacities, shs = read_raw(path, n_threads)
    rots = rots / np.linalg.norm(rots, axis=-1, keepdims=True)
    rots = rots.astype(np.float32)
    scales = np.exp(scales).astype(np.float32)
    opacities = (1 / (1 + np.exp(-opacities))).astype(np.float32)  # sigmoid
    return GaussianData(xyz, rots, scales, opacities, shs, path=path)


def _is_3dgs(path: str) -> bool:
    """gsconverter's format detection (utility.py:16-32), 3dgs branch."""
    with open(path, "rb") as f:
        return "property float f_dc_0" in f.read(2048).decode("utf-8", errors="ignore")


def export_select(xyz_cur, xyz_orig, enable_aabb, enable_obb, cube_min, cube_max, cube_rotation, stream=None):
    """GPU part of export_ply: (rows kept, bbox or None, points_center).

    xyz_cur / xyz_orig: float32 [N,3] torch CUDA tensors (current, as-loaded).
    The thresholds are formed with NumPy from the caller's values.  That keeps
    the reference's dtype promotion for `points_center + cubeMin` (util_gau.py:402).
    """
    import torch

    lib = _lib.load()
    n = int(xyz_cur.shape[0])
    if xyz_orig.shape[0] != n:
        raise ValueError("export_select: current and original point counts differ")
    for t in (xyz_cur, xyz_orig):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.shape[-1] == 3):
            raise ValueError("export_select: expected contiguous float32 CUDA tensors [N,3]")
    s = ctypes.c_void_p(stream if stream is not None else torch.cuda.current_stream().cuda_stream)
    c = (ctypes.c_float * 3)()
    _lib.check(lib.gsr_points_center(ctypes.c_void_p(xyz_cur.data_ptr()), n, ctypes.byref(c), s),
               "gsr_points_center")
    center = np.array(list(c), np.float32)
    box = _lib.GsrBox()
    if enable_aabb == 0 and enable_obb == 0:
        box.mode = _lib.GSR_BOX_NONE
    elif enable_obb == 1:
        box.mode = _lib.GSR_BOX_OBB
        lo, hi = np.asarray(cube_min), np.asarray(cube_max)
        box.rot_inv[:] = np.linalg.inv(euler_to_rotation_matrix(cube_rotation)).reshape(-1).tolist()
    elif enable_aabb == 1:
        box.mode = _lib.GSR_BOX_AABB
        lo, hi = center + cube_min, center + cube_max  # the reference's double offset, NumPy dtypes
    else:
        raise ValueError("export_ply: enable_aabb / enable_obb must be 0 or 1")
    if box.mode != _lib.GSR_BOX_NONE:
        box.cube_min[:] = [float(v) for v in np.broadcast_to(lo, (3,))]
        box.cube_max[:] = [float(v) for v in np.broadcast_to(hi, (3,))]
    rows = torch.empty(max(n, 1), dtype=torch.int64, device=xyz_cur.device)
    n_rows = ctypes.c_int64()
    bbox = (ctypes.c_float * 6)()
    has_bbox = ctypes.c_int32()
    _lib.check(lib.gsr_export_select(ctypes.c_void_p(xyz_cur.data_ptr()), ctypes.c_void_p(xyz_orig.data_ptr()), n,
                                     ctypes.byref(c), ctypes.byref(box), ctypes.c_void_p(rows.data_ptr()),
                                     ctypes.byref(n_rows), ctypes.byref(bbox), ctypes.byref(has_bbox), s),
               "gsr_export_select")
    return rows[: n_rows.value], (tuple(float(v) for v in bbox) if has_bbox.value else None), center


def export_ply(gaussian_data: GaussianData, output_path: str, enable_aabb, enable_obb, cube_min, cube_max,
               cube_rotation, overwrite: bool = False) -> bool:
    """util_gau.export_ply for a 3DGS source file: writes the rows of
    ``gaussian_data.path`` that gsconverter would keep, in its 3dgs layout.
    The reference asks before overwriting; here an existing output fails
    (returns False) unless ``overwrite``."""
    import torch

    if not output_path.lower().endswith(".ply"):  # gsconverter main.py:35-36
        output_path += ".ply"
    src = gaussian_data.path
    if src is None or not os.path.exists(src) or not _is_3dgs(src):
        return False
    if os.path.exists(output_path) and not overwrite:
        return False
    cur = torch.from_numpy(np.ascontiguousarray(gaussian_data.xyz, dtype=np.float32)).cuda()
    orig = torch.from_numpy(np.ascontiguousarray(gaussian_data.original_xyz, dtype=np.float32)).cuda()
    rows, _, _ = export_select(cur, orig, enable_aabb, enable_obb, cube_min, cube_max, cube_rotation)
    return write_3dgs(src, output_path, rows.cpu().numpy())


def write_3dgs(in_path: str, out_path: str, rows=None, n_threads: int = 0) -> bool:
    """Rows of a PLY in gsconverter's 3dgs layout (libgsr row writer)."""
    lib = _lib.load()
    if rows is None:
        rc = lib.gsr_ply_write_3dgs(os.fsencode(in_path), os.fsencode(out_path), None, 0, int(n_threads))
    else:
        r = np.ascontiguousarray(rows, dtype=np.int64)
        rc = lib.gsr_ply_write_3dgs(os.fsencode(in_path), os.fsencode(out_path), ctypes.c_void_p(r.ctypes.data),
                                    len(r), int(n_threads))
    _lib.check(rc, "gsr_ply_write_3dgs")
    return True
