"""Native PLY ingestion and the 3dgs row writer,
checked bit-exactly against the NumPy restatement of util_gau.load_ply and
gsconverter in oracle/ply_oracle.py.  Host code only (no GPU)."""
import numpy as np
import pytest

from gsviewer_amd import _lib
from gsviewer_amd.ply import load_ply, probe, read_raw, write_3dgs
from oracle import ply_oracle as P


def vertex_array(n, deg=3, seed=0, extra=(), order=None, xyz_type="f4"):
    """A 3DGS-style vertex element (the layout 3DGS training writes)."""
    rng = np.random.default_rng(seed)
    fields = [("x", xyz_type), ("y", xyz_type), ("z", xyz_type), ("nx", "f4"), ("ny", "f4"), ("nz", "f4"),
              ("f_dc_0", "f4"), ("f_dc_1", "f4"), ("f_dc_2", "f4")]
    if deg == 3:
        fields += [(f"f_rest_{i}", "f4") for i in range(45)]
    fields += [("opacity", "f4"), ("scale_0", "f4"), ("scale_1", "f4"), ("scale_2", "f4"),
               ("rot_0", "f4"), ("rot_1", "f4"), ("rot_2", "f4"), ("rot_3", "f4")]
    fields += list(extra)
    if order is not None:
        fields = [fields[i] for i in order(len(fields))]
    a = np.zeros(n, dtype=fields)
    for name, t in fields:
        if t in ("f4", "f8"):
            a[name] = rng.normal(0, 1.5, n)
        else:
            a[name] = rng.integers(0, 200, n)
    a["opacity"] = rng.normal(0, 2, n)
    for k in range(3):
        a[f"scale_{k}"] = rng.normal(-4.6, 0.6, n)
    return a


def write(tmp_path, arr, fmt="binary_little_endian", name="s.ply"):
    p = tmp_path / name
    p.write_bytes(P.ply_bytes(arr, fmt))
    return str(p)


def assert_same_scene(path):
    g = load_ply(path)
    xyz, rot, scale, op, sh = P.load_ply(path)
    for got, want in ((g.xyz, xyz), (g.rot, rot), (g.scale, scale), (g.opacity, op), (g.sh, sh)):
        assert got.dtype == np.float32 and got.shape == want.shape
        np.testing.assert_array_equal(got, want)
    return g


@pytest.mark.parametrize("deg", [0, 3])
def test_load_ply_bit_exact(tmp_path, deg):
    g = assert_same_scene(write(tmp_path, vertex_array(3001, deg=deg, seed=deg)))
    assert g.sh.shape[1] == (48 if deg == 3 else 3)
    info = probe(g.path)
    assert info.n == 3001 and info.sh_dim == g.sh.shape[1] and info.format == _lib.GSR_PLY_BINARY_LE


def test_sh_layout_is_coefficient_major(tmp_path):
    # load_ply: f_rest reshaped (3, 15) and transposed -> sh[3 + 3j + c] = f_rest[c*15 + j]
    a = vertex_array(5, deg=3, seed=7)
    g = load_ply(write(tmp_path, a))
    for c in range(3):
        for j in range(15):
            np.testing.assert_array_equal(g.sh[:, 3 + 3 * j + c], a[f"f_rest_{c * 15 + j}"].astype(np.float32))


def test_property_order_and_extra_properties(tmp_path):
    extra = [("red", "u1"), ("custom", "f8"), ("flags", "i2")]
    rng = np.random.default_rng(3)
    a = vertex_array(2000, deg=3, seed=3, extra=extra, order=lambda n: rng.permutation(n))
    assert_same_scene(write(tmp_path, a))


def test_big_endian_and_ascii(tmp_path):
    assert_same_scene(write(tmp_path, vertex_array(1500, deg=3, seed=4), "binary_big_endian", "be.ply"))
    assert_same_scene(write(tmp_path, vertex_array(60, deg=3, seed=5), "ascii", "a.ply"))
    assert probe(str(tmp_path / "be.ply")).format == _lib.GSR_PLY_BINARY_BE
    assert probe(str(tmp_path / "a.ply")).format == _lib.GSR_PLY_ASCII


def test_double_positions(tmp_path):
    # x/y/z stored as float64: load_ply casts them with astype(float32); so does the reader
    g = load_ply(write(tmp_path, vertex_array(1000, deg=0, seed=6, xyz_type="f8")))
    np.testing.assert_array_equal(g.xyz, P.load_ply(g.path)[0])


def test_threads_do_not_change_the_result(tmp_path):
    path = write(tmp_path, vertex_array(70000, deg=3, seed=8))
    one = read_raw(path, n_threads=1)
    many = read_raw(path, n_threads=8)
    for a, b in zip(one, many):
        np.testing.assert_array_equal(a, b)


def test_element_before_vertex(tmp_path):
    a = vertex_array(100, deg=0, seed=9)
    cam = np.zeros(2, dtype=[("fx", "f4"), ("fy", "f4"), ("id", "i4")])
    head = b"ply\nformat binary_little_endian 1.0\nelement camera 2\nproperty float fx\nproperty float fy\n" \
           b"property int id\n"
    body = P.ply_bytes(a)
    vh = body[body.index(b"element vertex"):]
    p = tmp_path / "cam.ply"
    p.write_bytes(head + vh[:vh.index(b"end_header\n") + 11] + cam.tobytes() + vh[vh.index(b"end_header\n") + 11:])
    g = load_ply(str(p))
    np.testing.assert_array_equal(g.xyz, np.stack([a["x"], a["y"], a["z"]], 1))


@pytest.mark.parametrize("case", ["f_rest_24", "no_opacity", "not_ply", "truncated", "list_prop"])
def test_malformed_files_fail_loudly(tmp_path, case):
    p = tmp_path / "bad.ply"
    if case == "f_rest_24":      # load_ply reshapes f_rest to (N, 3, 15): 24 values cannot
        a = vertex_array(10, deg=0)
        extra = np.zeros(10, dtype=a.dtype.descr + [(f"f_rest_{i}", "f4") for i in range(24)])
        for n in a.dtype.names:
            extra[n] = a[n]
        p.write_bytes(P.ply_bytes(extra))
    elif case == "no_opacity":
        a = vertex_array(10, deg=0)
        keep = [n for n in a.dtype.names if n != "opacity"]
        p.write_bytes(P.ply_bytes(np.ascontiguousarray(a[keep]).astype([(n, "f4") for n in keep])))
    elif case == "not_ply":
        p.write_bytes(b"hello\n")
    elif case == "truncated":
        p.write_bytes(P.ply_bytes(vertex_array(100, deg=3))[:-1000])
    else:
        p.write_bytes(b"ply\nformat binary_little_endian 1.0\nelement vertex 1\nproperty float x\n"
                      b"property list uchar int vertex_indices\nend_header\n" + b"\0" * 16)
    with pytest.raises(RuntimeError):
        load_ply(str(p))


def test_write_3dgs_rows_match_gsconverter(tmp_path):
    a = vertex_array(5000, deg=3, seed=11, extra=[("red", "u1")])
    src = write(tmp_path, a)
    rows = np.sort(np.random.default_rng(1).choice(5000, 1234, replace=False))
    out = str(tmp_path / "out.ply")
    assert write_3dgs(src, out, rows)
    want = P.ply_bytes(P.to_3dgs(a[rows]))
    assert open(out, "rb").read() == want


def test_write_3dgs_prefix_names_and_missing_fields(tmp_path):
    # gsconverter copies scal_/scalar_ prefixed fields by stripped name; absent fields stay 0
    a = vertex_array(300, deg=0, seed=12)
    renamed = a.astype([(("scal_" + n) if n.startswith("f_dc") else n, t) for n, t in a.dtype.descr])
    renamed = np.rec.fromarrays([a[n] for n in a.dtype.names], dtype=renamed.dtype)
    src = write(tmp_path, np.asarray(renamed))
    out = str(tmp_path / "o.ply")
    assert write_3dgs(src, out)
    got = P.read_vertex(out)
    want = P.to_3dgs(np.asarray(renamed))
    assert got.dtype.names == want.dtype.names
    for n in want.dtype.names:
        np.testing.assert_array_equal(got[n], want[n])
    assert (got["f_rest_0"] == 0).all() and (got["f_dc_1"] == a["f_dc_1"]).all()


def test_write_3dgs_rejects_bad_rows(tmp_path):
    src = write(tmp_path, vertex_array(10, deg=0))
    with pytest.raises(RuntimeError):
        write_3dgs(src, str(tmp_path / "o.ply"), np.array([3, 2]))
    with pytest.raises(RuntimeError):
        write_3dgs(src, str(tmp_path / "o.ply"), np.array([11]))
