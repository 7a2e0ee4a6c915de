"""Pin the CPU oracle and the host-side data model against golden vectors
generated from the reference itself (tests/golden/make_golden.py)."""
import numpy as np

from gsviewer_amd.camera import Camera, euler_to_rotation_matrix, rotation_matrix_to_euler
from gsviewer_amd.gaussian_data import GaussianData, naive_gaussian
from oracle import gl_oracle as O
from oracle import ply_oracle as P


def test_naive_gaussian_layout(golden):
    g = naive_gaussian()
    for k in ("xyz", "rot", "scale", "opacity", "sh"):
        np.testing.assert_array_equal(getattr(g, k), golden[f"naive_{k}"])
    np.testing.assert_array_equal(g.flat(), golden["naive_flat"])
    assert g.sh_dim == int(golden["naive_sh_dim"])


def test_flat_layout_and_bbox(golden):
    g = GaussianData(golden["rand_xyz"], golden["rand_rot"], golden["rand_scale"], golden["rand_opacity"],
                     golden["rand_sh"])
    np.testing.assert_array_equal(g.flat(), golden["rand_flat"])
    np.testing.assert_array_equal(g.points_center, golden["rand_points_center"])
    mn, mx, corners = g.compute_aabb
    np.testing.assert_array_equal(mn, golden["rand_aabb_min"])
    np.testing.assert_array_equal(mx, golden["rand_aabb_max"])
    np.testing.assert_array_equal(corners, golden["rand_aabb_corners"])


def test_scale_data_bit_exact(golden):
    g = GaussianData(golden["scale_in_xyz"].copy(), golden["scale_in_rot"].copy(), golden["rand_scale"].copy(),
                     golden["rand_opacity"].copy(), golden["rand_sh"].copy())
    g.scale_data(5.0)
    np.testing.assert_array_equal(g.xyz, golden["scale_out_xyz"])
    np.testing.assert_array_equal(g.rot, golden["scale_out_rot"])
    np.testing.assert_array_equal(g.scale, golden["scale_out_scale"])


def test_oracle_sort_matches_reference(golden):
    """oracle.sort_back_to_front(view z) == renderer_ogl._sort_gaussian_cpu."""
    flat = golden["rand_flat"]
    for V, ref in zip(golden["sort_views"], golden["sort_index"]):
        U = O.default_uniforms(V, np.eye(4), [1, 1, 100], [0, 0, 0], 64, 64)
        vs = O.vertex_stage(flat, 48, U)
        order = O.sort_back_to_front(vs["view_z"])
        np.testing.assert_array_equal(order, ref)


def test_euler_rotation_matrix(golden):
    for a, R in zip(golden["euler_angles"], golden["euler_R"]):
        np.testing.assert_allclose(euler_to_rotation_matrix(a), R, rtol=0, atol=1e-15)


def test_default_camera_matrices():
    cam = Camera(720, 1280)
    V = cam.get_view_matrix()
    np.testing.assert_array_equal(V, np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, -5], [0, 0, 0, 1]], np.float32))
    np.testing.assert_array_equal(cam.position, np.array([0, 0, 5], np.float32))
    P = cam.get_project_matrix()
    t = np.float32(np.tan(np.float32(np.pi / 2) / 2))
    assert P[1, 1] == np.float32(1) / t and P[3, 2] == -1 and P[3, 3] == 0
    htx, hty, f = cam.get_htanfovxy_focal()
    assert abs(hty - 1) < 1e-12 and abs(htx - 1280 / 720) < 1e-12 and abs(f - 360) < 1e-9


def test_camera_yaw_views_orbit_target():
    for k in range(8):
        cam = Camera(1080, 1920).yaw(45.0 * k)
        V = cam.get_view_matrix()
        # target (origin) stays on the optical axis at distance 5
        p = V @ np.array([0, 0, 0, 1], np.float32)
        np.testing.assert_allclose(p[:3], [0, 0, -5], atol=2e-6)
        np.testing.assert_allclose(np.linalg.norm(cam.position), 5, rtol=1e-6)


def test_rotation_matrix_to_euler_bit_exact(golden):
    """util.convert_rotation_matrix_to_euler_angles (util.py:494-501, scipy
    as_euler('xyz')) on the OBB test rotations, a gimbal-lock case and random
    rotations: bit-exact, and the inverse of euler_to_rotation_matrix."""
    for R, e in zip(golden["r2e_R"], golden["r2e_euler"]):
        np.testing.assert_array_equal(rotation_matrix_to_euler(R), e)
    for a in golden["euler_angles"][:3]:
        np.testing.assert_allclose(euler_to_rotation_matrix(rotation_matrix_to_euler(euler_to_rotation_matrix(a))),
                                   euler_to_rotation_matrix(a), atol=1e-12)


def test_compute_obb_bit_exact(golden):
    """GaussianData.compute_obb (util_gau.py:114-138): min, max, axes and
    corners bit-exact on three point sets (uniform, rescaled, anisotropic)."""
    for k in range(3):
        p = golden[f"obb{k}_xyz"]
        n = len(p)
        g = GaussianData(p, np.tile(np.float32([1, 0, 0, 0]), (n, 1)), np.ones((n, 3), np.float32),
                         np.ones((n, 1), np.float32), np.zeros((n, 3), np.float32))
        mn, mx, U, corners = g.compute_obb
        np.testing.assert_array_equal(mn, golden[f"obb{k}_min"])
        np.testing.assert_array_equal(mx, golden[f"obb{k}_max"])
        np.testing.assert_array_equal(U, golden[f"obb{k}_U"])
        np.testing.assert_array_equal(corners, golden[f"obb{k}_corners"])


def export_cases(golden):
    """(aabb, obb, cube_min, cube_max, euler, bbox or None, rows) of the
    reference-run export_ply + crop_by_bbox fixtures (make_golden.py)."""
    rows = np.split(golden["export_rows"], np.cumsum(golden["export_nrows"])[:-1])
    out = []
    for prm, bbox, r in zip(golden["export_params"], golden["export_bbox"], rows):
        bb = None if np.isnan(bbox).all() else tuple(bbox.tolist())
        out.append((int(prm[0]), int(prm[1]), list(prm[2:5]), list(prm[5:8]), list(prm[8:11]), bb, r))
    return out


def test_export_oracle_matches_reference(golden):
    """oracle/ply_oracle.export_rows == util_gau.export_ply's bbox (util_gau.py:
    388-413) + gsconverter's crop_by_bbox rows (base_converter.py:175-191),
    run on the reference itself: the export oracle is pinned."""
    cur, orig = golden["export_cur"], golden["export_orig"]
    for aabb, obb, cmin, cmax, rot, bbox, rows in export_cases(golden):
        got_rows, got_bbox = P.export_rows(cur, orig, aabb, obb, cmin, cmax, euler_to_rotation_matrix(rot))
        assert got_bbox == bbox
        np.testing.assert_array_equal(got_rows, rows)
