"""GPU box mask + compaction for export, through the
C ABI, against the NumPy restatement of util_gau.export_ply + gsconverter's
crop in oracle/ply_oracle.py."""
import numpy as np
import pytest

from gsviewer_amd.camera import euler_to_rotation_matrix
from oracle import ply_oracle as P

pytestmark = pytest.mark.gpu


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


@pytest.mark.parametrize("n", [1, 2, 255, 100_003])
def test_points_center_is_numpy_mean(gpu, n):
    import ctypes

    from gsviewer_amd import _lib
    xyz = (np.random.default_rng(n).normal(1.0, 3.0, (n, 3))).astype(np.float32)
    t = _t(xyz)
    c = (ctypes.c_float * 3)()
    _lib.check(_lib.load().gsr_points_center(ctypes.c_void_p(t.data_ptr()), n, ctypes.byref(c), None), "center")
    np.testing.assert_array_equal(np.array(list(c), np.float32), np.mean(xyz, axis=0))


def _scene(n, seed):
    rng = np.random.default_rng(seed)
    orig = rng.normal(0, 2.0, (n, 3)).astype(np.float32)
    # the viewer rescales the scene (scale_data) before export; the box acts on the current positions
    cur = (orig * np.float32(0.5) + np.float32(0.05)).astype(np.float32)
    return cur, orig


CASES = [
    ("none", 0, 0, [-1, -1, -1], [1, 1, 1], [0, 0, 0]),
    ("aabb", 1, 0, [-0.8, -0.5, -0.6], [0.7, 0.9, 0.4], [0, 0, 0]),
    ("aabb_f32", 1, 0, np.array([-0.8, -0.5, -0.6], np.float32), np.array([0.7, 0.9, 0.4], np.float32), [0, 0, 0]),
    ("obb", 0, 1, [-0.9, -0.4, -0.7], [0.6, 0.8, 0.5], [30.0, 15.0, 0.0]),
    ("obb_wins", 1, 1, [-0.9, -0.4, -0.7], [0.6, 0.8, 0.5], [10.0, -20.0, 45.0]),
    ("empty", 1, 0, [50, 50, 50], [60, 60, 60], [0, 0, 0]),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_export_select_matches_oracle(gpu, case):
    from gsviewer_amd.ply import export_select
    _, aabb, obb, cmin, cmax, rot = case
    cur, orig = _scene(20_000, 3)
    rows, bbox, center = export_select(_t(cur), _t(orig), aabb, obb, cmin, cmax, rot)
    np.testing.assert_array_equal(center, np.mean(cur, axis=0))
    want_rows, want_bbox = P.export_rows(cur, orig, aabb, obb, cmin, cmax, euler_to_rotation_matrix(rot))
    np.testing.assert_array_equal(rows.cpu().numpy(), want_rows)
    assert bbox == want_bbox
    if case[0] == "empty":
        assert bbox is None and len(want_rows) == len(cur)   # bbox=None: gsconverter keeps every row
    elif case[0] != "none":
        assert 0 < len(want_rows) < len(cur)


def test_export_select_matches_reference_run(gpu, golden):
    """gsr_box_select against the reference itself: export_ply's bbox and
    gsconverter's crop rows recorded by tests/golden/make_golden.py (the
    reference's export_ply run with its gsconverter call captured, and
    BaseConverter.crop_by_bbox on the original positions)."""
    from gsviewer_amd.ply import export_select
    from test_oracle_golden import export_cases
    cur, orig = golden["export_cur"], golden["export_orig"]
    cases = export_cases(golden)
    assert len(cases) == 6
    for aabb, obb, cmin, cmax, rot, bbox, rows in cases:
        got_rows, got_bbox, _ = export_select(_t(cur), _t(orig), aabb, obb, cmin, cmax, rot)
        assert got_bbox == bbox
        np.testing.assert_array_equal(got_rows.cpu().numpy(), rows)


def test_export_ply_end_to_end(gpu, tmp_path):
    from gsviewer_amd.ply import export_ply, load_ply
    from test_ply import vertex_array
    a = vertex_array(30_000, deg=3, seed=21)
    src = tmp_path / "scene.ply"
    src.write_bytes(P.ply_bytes(a))
    g = load_ply(str(src))
    g.scale_data(5.0)                      # what the viewer does after loading (gs_elements_control.py:41-42)
    cmin, cmax, rot = [-1.0, -0.8, -1.2], [1.1, 0.9, 0.7], [25.0, 0.0, -10.0]
    out = str(tmp_path / "crop")           # '.ply' is appended, as gsconverter does
    assert export_ply(g, out, 0, 1, cmin, cmax, rot)
    rows, _ = P.export_rows(g.xyz, g.original_xyz, 0, 1, cmin, cmax, euler_to_rotation_matrix(rot))
    assert 0 < len(rows) < len(a)
    assert open(out + ".ply", "rb").read() == P.ply_bytes(P.to_3dgs(P.read_vertex(str(src))[rows]))
    # an existing output is not overwritten (the reference asks; non-interactively it fails)
    assert not export_ply(g, out, 0, 1, cmin, cmax, rot)
    assert export_ply(g, out, 0, 1, cmin, cmax, rot, overwrite=True)
