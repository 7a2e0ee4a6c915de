"""CPU oracle for scene ingestion and export.

TEST INFRASTRUCTURE ONLY.  Only tests/ may import this module.  The product
path (gsviewer_amd/ply.py over libgsr.so) never calls it.

It restates, in NumPy:
  * PlyData.read's vertex element for binary_little_endian, binary_big_endian
    and ascii bodies (plyfile itself is not installed in this image, so parity
    is pinned on the reference's own expressions below and on files this
    module writes);
  * util_gau.load_ply (util_gau.py:236-305): the column gathers, the
    f_rest reshape (N,3,15) -> transpose -> flatten, and the activations, in
    the same NumPy expressions and dtypes;
  * util_gau.export_ply's filter (util_gau.py:388-413): points_center,
    AABB/OBB masks with the reference's dtype promotions, the bbox of the
    as-loaded xyz;
  * gsconverter's crop_by_bbox (base_converter.py:175-184) and its 3dgs output
    (define_dtype :148-170, copy_data_with_prefix_check utility.py:35-65,
    PlyData.write with native byte order, main.py:108-110).
"""
from __future__ import annotations

import numpy as np

_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
          "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
          "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}
_TYPE_NAME = {"i1": "char", "u1": "uchar", "i2": "short", "u2": "ushort", "i4": "int", "u4": "uint",
              "f4": "float", "f8": "double"}


def read_vertex(path):
    """Structured array of the 'vertex' element (fixed-size properties only)."""
    raw = open(path, "rb").read()
    end = raw.index(b"end_header") + len(b"end_header")
    end = raw.index(b"\n", end) + 1
    lines = raw[:end].decode("ascii").splitlines()
    assert lines[0] == "ply"
    fmt, elements = None, []
    for ln in lines[1:]:
        t = ln.split()
        if not t or t[0] in ("comment", "obj_info", "end_header"):
            continue
        if t[0] == "format":
            fmt = t[1]
        elif t[0] == "element":
            elements.append([t[1], int(t[2]), []])
        elif t[0] == "property":
            assert t[1] != "list", "list properties are not restated"
            elements[-1][2].append((t[2], _TYPES[t[1]]))
    order = "<" if fmt == "binary_little_endian" else ">"
    body = raw[end:]
    if fmt == "ascii":
        rows = body.decode("ascii").split("\n")
        skip = 0
        for name, count, props in elements:
            if name == "vertex":
                dt = np.dtype([(p, t) for p, t in props])
                vals = np.array([r.split() for r in rows[skip:skip + count]], dtype=np.float64)
                out = np.zeros(count, dt)
                for j, (p, _) in enumerate(props):
                    out[p] = vals[:, j]
                return out
            skip += count
        raise ValueError("no vertex element")
    off = 0
    for name, count, props in elements:
        dt = np.dtype([(p, order + t) for p, t in props])
        if name == "vertex":
            return np.frombuffer(body, dtype=dt, count=count, offset=off)
        off += dt.itemsize * count
    raise ValueError("no vertex element")


def load_ply_raw(path):
    """load_ply's column gathers (util_gau.py:241-293): pre-activation arrays,
    the way plyfile -> NumPy/pandas hands them over (columns keep the file's
    dtype; the casts to float32 happen at the activations)."""
    v = read_vertex(path)
    names = v.dtype.names
    xyz = np.stack([np.asarray(v["x"]), np.asarray(v["y"]), np.asarray(v["z"])], 1)
    opacities = np.asarray(v["opacity"])[..., np.newaxis]
    features_dc = np.stack([np.asarray(v["f_dc_0"]), np.asarray(v["f_dc_1"]), np.asarray(v["f_dc_2"])], 1)
    extra = sorted((n for n in names if n.startswith("f_rest_")), key=lambda x: int(x.split("_")[-1]))
    scale_names = sorted((n for n in names if n.startswith("scale_")), key=lambda x: int(x.split("_")[-1]))
    rot_names = sorted((n for n in names if n.startswith("rot")), key=lambda x: int(x.split("_")[-1]))
    max_sh_degree = 3
    features_extra = np.stack([np.asarray(v[n]) for n in extra], 1) if extra else np.zeros((len(v), 0))
    if features_extra.shape[1] == 0:
        max_sh_degree = 0
    features_extra = features_extra.reshape((features_extra.shape[0], 3, (max_sh_degree + 1) ** 2 - 1))
    features_extra = np.transpose(features_extra, [0, 2, 1])
    scales = np.stack([np.asarray(v[n]) for n in scale_names], 1)
    rots = np.stack([np.asarray(v[n]) for n in rot_names], 1)
    return dict(xyz=xyz, rots=rots, scales=scales, opacities=opacities,
                features_dc=features_dc, features_extra=features_extra)


def activate(raw):
    """util_gau.py:295-303, the same expressions on the same dtypes."""
    xyz = raw["xyz"].astype(np.float32)
    rots = raw["rots"] / np.linalg.norm(raw["rots"], axis=-1, keepdims=True)
    rots = rots.astype(np.float32)
    scales = np.exp(raw["scales"]).astype(np.float32)
    opacities = (1 / (1 + np.exp(-raw["opacities"]))).astype(np.float32)
    shs = np.concatenate([raw["features_dc"].reshape(-1, 3),
                          raw["features_extra"].reshape(len(raw["features_dc"]), -1)], axis=-1).astype(np.float32)
    return xyz, rots, scales, opacities, shs


def load_ply(path):
    return activate(load_ply_raw(path))


def points_center(xyz):
    """util_gau.py:391 (np.mean over axis 0 of the float32 scene)."""
    return np.mean(xyz, axis=0)


def export_mask(xyz_cur, enable_aabb, enable_obb, cube_min, cube_max, rotation_matrix, center=None):
    """util_gau.py:389-405 with the reference's dtype promotions.
    Returns (mask, the thresholds the comparisons use)."""
    if center is None:
        center = points_center(xyz_cur)
    transformed = xyz_cur - center
    if enable_aabb == 0 and enable_obb == 0:
        return np.ones(len(xyz_cur), bool), None
    if enable_obb == 1:
        t = np.dot(np.linalg.inv(rotation_matrix), transformed.T).T
        mask = (t >= np.asarray(cube_min)).all(axis=1) & (t <= np.asarray(cube_max)).all(axis=1)
        return mask, (np.asarray(cube_min), np.asarray(cube_max))
    if enable_aabb == 1:
        lo = center + cube_min
        hi = center + cube_max
        mask = (transformed >= lo).all(axis=1) & (transformed <= hi).all(axis=1)
        return mask, (lo, hi)
    raise ValueError("export_ply: enable_aabb / enable_obb must be 0 or 1")


def export_rows(xyz_cur, xyz_orig, enable_aabb, enable_obb, cube_min, cube_max, rotation_matrix, center=None):
    """Rows gsconverter writes for export_ply: the bbox of xyz_orig[mask]
    (util_gau.py:411-413), then crop_by_bbox on the file rows
    (base_converter.py:177-184); no bbox (empty mask) -> every row."""
    mask, _ = export_mask(xyz_cur, enable_aabb, enable_obb, cube_min, cube_max, rotation_matrix, center)
    filtered = xyz_orig[mask]
    if filtered.size == 0:
        return np.arange(len(xyz_orig)), None
    bbox = tuple(np.concatenate([np.min(filtered, axis=0), np.max(filtered, axis=0)]).tolist())
    min_x, min_y, min_z, max_x, max_y, max_z = bbox
    x, y, z = xyz_orig[:, 0], xyz_orig[:, 1], xyz_orig[:, 2]
    keep = (x >= min_x) & (x <= max_x) & (y >= min_y) & (y <= max_y) & (z >= min_z) & (z <= max_z)
    return np.nonzero(keep)[0], bbox


THREEDGS_FIELDS = (["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
                   + [f"f_rest_{i}" for i in range(45)] + ["opacity", "scale_0", "scale_1", "scale_2",
                                                           "rot_0", "rot_1", "rot_2", "rot_3"])


def to_3dgs(vertex):
    """Format3dgs.to_3dgs (format_3dgs.py:66-87): copy by name into the 3dgs dtype."""
    out = np.zeros(len(vertex), dtype=[(n, "f4") for n in THREEDGS_FIELDS])
    for name in vertex.dtype.names:
        if name in out.dtype.names:
            out[name] = vertex[name]
            continue
        for prefix in ("", "scal_", "scalar_", "scalar_scal_"):
            if name.startswith(prefix) and name[len(prefix):] in out.dtype.names:
                out[name[len(prefix):]] = vertex[name]
                break
    return out


def ply_bytes(struct_array, fmt="binary_little_endian"):
    """PLY file bytes of a structured array as the 'vertex' element."""
    hdr = ["ply", f"format {fmt} 1.0", f"element vertex {len(struct_array)}"]
    for name in struct_array.dtype.names:
        hdr.append(f"property {_TYPE_NAME[struct_array.dtype[name].str[1:]]} {name}")
    hdr.append("end_header")
    head = ("\n".join(hdr) + "\n").encode("ascii")
    if fmt == "ascii":
        rows = [" ".join(repr(float(v)) if isinstance(v, (float, np.floating)) else str(v) for v in r)
                for r in struct_array.tolist()]
        return head + ("\n".join(rows) + "\n").encode("ascii")
    order = "<" if fmt == "binary_little_endian" else ">"
    dt = np.dtype([(n, order + struct_array.dtype[n].str[1:]) for n in struct_array.dtype.names])
    return head + struct_array.astype(dt).tobytes()
