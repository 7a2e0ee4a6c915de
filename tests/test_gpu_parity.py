"""GPU parity: the HIP rasterizer (through the C ABI) against the CPU oracle of
the reference's OpenGL path, on the same seeded inputs."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera, euler_to_rotation_matrix
from gsviewer_amd.gaussian_data import garden_standin, naive_gaussian, random_scene
from oracle import gl_oracle as O
from helpers import (TOL_TMIN, alpha_box_rects, compare_images, decode_records, frame_depth_order, kept_fragments,
                     narrowed_rects,
                     tile_lists_for, expected_interval_form, expected_quadratic, gpu_frame,
                     uniforms_for)

pytestmark = pytest.mark.gpu


def _settings(**kw):
    from gsviewer_amd.rasterizer import RenderSettings
    return RenderSettings(**kw)


def _check(g, cam, st, mode="float", **cmp):
    res = gpu_frame(g, cam, st, with_debug=True, radii=True)
    U = uniforms_for(cam, st)
    vs = O.vertex_stage(g.flat().astype(np.float32), g.sh_dim, U)
    ref = O.composite(vs, U, mode=mode)
    info = compare_images(res["image"], ref, **cmp)
    return res, vs, U, ref, info


def test_naive_scene_default_camera(gpu):
    g = naive_gaussian()
    for (w, h) in [(1280, 720), (640, 480)]:
        res, vs, U, ref, info = _check(g, Camera(h, w), _settings(t_min=0.0))
        assert res["stats"]["n_visible"] == 4
        # the four splats are clearly drawn: centre pixel of Gaussian 0 is magenta-ish
        assert res["image"][h // 2, w // 2].max() > 0.5


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_random_scene_exact_mode(gpu, deg):
    g = random_scene(2500, sh_degree=deg, seed=10 + deg)
    res, vs, U, ref, info = _check(g, Camera(120, 160), _settings(t_min=0.0))
    assert res["stats"]["n_visible"] == int(vs["visible"].sum())


def test_preprocess_records_bit_exact(gpu):
    g = random_scene(3000, sh_degree=3, seed=3)
    cam = Camera(96, 128).yaw(20)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), 48, U)
    vis_desc = np.nonzero(vs["visible"])[0][::-1]          # slot s -> Gaussian id
    rec = decode_records(res["records"])
    assert len(vis_desc) == len(rec["opacity"])
    np.testing.assert_array_equal(rec["center"], vs["center"][vis_desc])
    qa, qb, qc = expected_quadratic(vs)
    np.testing.assert_array_equal(rec["qa"], qa[vis_desc])
    np.testing.assert_array_equal(rec["qb"], qb[vis_desc])
    np.testing.assert_array_equal(rec["qc"], qc[vis_desc])
    s, col, mid = expected_interval_form(vs["opacity"][vis_desc], np.clip(vs["color"][vis_desc], 0, 1))
    np.testing.assert_array_equal(rec["opacity"], s)
    np.testing.assert_array_equal(rec["color"], col)
    np.testing.assert_allclose(rec["mid"], mid, rtol=1e-6, atol=1e-6)
    # covered rectangle = the oracle's quad narrowed by the alpha box (bit-exact mirror)
    rx0, rx1, rr0, rr1 = (a[vis_desc] for a in O.splat_rects(vs, U))
    x0, x1, r0, r1 = alpha_box_rects(rec, (rx0, rx1, rr0, rr1), U["height"])
    ne = (x0 <= x1) & (r0 <= r1)
    for a, b in [(rec["x0"], x0), (rec["x1"], x1), (rec["r0"], r0), (rec["r1"], r1)]:
        np.testing.assert_array_equal(a[ne], b[ne])
    assert np.all(rec["x0"][~ne] > rec["x1"][~ne])
    # it only narrows, and it does narrow a sizeable share of this scene
    assert np.all((x0[ne] >= rx0[ne]) & (x1[ne] <= rx1[ne]) & (r0[ne] >= rr0[ne]) & (r1[ne] <= rr1[ne]))
    area = lambda a0, a1, b0, b1: ((a1 - a0 + 1) * (b1 - b0 + 1))[ne]
    assert (area(x0, x1, r0, r1) < area(rx0, rx1, rr0, rr1)).mean() > 0.1

@pytest.mark.parametrize("mode", [-6, -5, -4])
def test_preprocess_records_plain_for_other_fragment_classes(gpu, mode):
    """Ball / billboard classes keep the plain opacity and colour (mid = 0)."""
    g = random_scene(1500, sh_degree=1, seed=4)
    cam = Camera(64, 96).yaw(10)
    st = _settings(render_mod=mode, t_min=0.0)
    res = gpu_frame(g, cam, st, with_debug=True)
    U = uniforms_for(cam, st)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    vis_desc = np.nonzero(vs["visible"])[0][::-1]
    rec = decode_records(res["records"])
    np.testing.assert_array_equal(rec["opacity"], vs["opacity"][vis_desc])
    col = vs["color"][vis_desc] if mode == -6 else np.clip(vs["color"][vis_desc], 0, 1)
    np.testing.assert_array_equal(rec["color"], col)
    assert np.all(rec["mid"] == 0)


def test_depth_order_and_tile_lists_exact(gpu):
    g = random_scene(4000, sh_degree=0, seed=5)
    cam = Camera(80, 112).yaw(-35)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), 3, U)
    vis_desc = np.nonzero(vs["visible"])[0][::-1]
    # the frame's global order: the coarse depth order (helpers.frame_depth_order),
    # or, with GSR_DEPTH_COARSE=0, the reverse of the GL draw order
    np.testing.assert_array_equal(vis_desc[res["depth_order"]], frame_depth_order(vs, res["depth_coarse"]))
    # per-tile instance lists == GL order restricted to the tile, reversed, over
    # the quads narrowed by the alpha box
    rects = narrowed_rects(res, vs, U)
    lists = tile_lists_for(vs, U, rects)
    ranges, tl = res["ranges"], res["tile_list"]
    for t, want in enumerate(lists):
        b, e = ranges[t]
        got = vis_desc[tl[b:e]] if e > b else np.zeros(0, np.int64)
        np.testing.assert_array_equal(got, np.asarray(want, np.int64), err_msg=f"tile {t}")
    assert res["stats"]["n_instances"] == sum(len(x) for x in lists)
    # the narrowing drops only instances without a single kept fragment in the tile
    full = O.tile_lists(vs, U)
    qx0, qx1, qr0, qr1 = O.splat_rects(vs, U)
    tx_n = (U["width"] + 15) // 16
    dropped = 0
    for t, (f, ours) in enumerate(zip(full, lists)):
        keep = set(ours)
        assert [x for x in f if x in keep] == ours, f"tile {t}: order"
        ty, tx = divmod(t, tx_n)
        for gid in set(f) - keep:
            xs = np.arange(max(qx0[gid], 16 * tx), min(qx1[gid], 16 * tx + 15) + 1)
            rows = np.arange(max(qr0[gid], 16 * ty), min(qr1[gid], 16 * ty + 15) + 1)
            assert not kept_fragments(vs, U, gid, xs, rows).any(), f"tile {t}: Gaussian {gid} dropped"
            dropped += 1
    assert dropped > 0


def test_alpha_box_keeps_every_fragment(gpu):
    """The narrowed rectangle holds every fragment of the quad that the alpha
    test keeps (opacities over the whole range, anisotropic splats)."""
    rng = np.random.default_rng(12)
    g = random_scene(3000, sh_degree=0, seed=12, scale_range=(0.01, 0.12))
    g.opacity[:] = rng.uniform(0.0, 1.0, g.opacity.shape).astype(np.float32)
    cam = Camera(96, 128).yaw(25)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), 3, U)
    x0, x1, r0, r1 = narrowed_rects(res, vs, U)
    qx0, qx1, qr0, qr1 = O.splat_rects(vs, U)
    ids = np.nonzero(vs["visible"] & (qx0 <= qx1) & (qr0 <= qr1))[0]
    narrowed = 0
    for gid in ids:
        xs = np.arange(qx0[gid], qx1[gid] + 1)
        rows = np.arange(qr0[gid], qr1[gid] + 1)
        keep = kept_fragments(vs, U, gid, xs, rows)
        inside = ((xs >= x0[gid]) & (xs <= x1[gid]))[None, :] & ((rows >= r0[gid]) & (rows <= r1[gid]))[:, None]
        assert not (keep & ~inside).any(), f"Gaussian {gid}"
        narrowed += int(not inside.all())
    assert narrowed > len(ids) // 10
    compare_images(res["image"], O.composite(vs, U))


def test_alpha_box_4k_large_anisotropic(gpu):
    """The same at 3840x2160 with large, strongly anisotropic splats (needles
    and flat discs at every orientation, hundreds of pixels long) and the
    whole opacity range: the margin of the alpha box (x 1.002 + 0.01 px) and
    its degeneracy cut (|rho| > 0.995 keeps the quad) hold every kept
    fragment inside the narrowed rectangle."""
    rng = np.random.default_rng(21)
    g = random_scene(1200, sh_degree=0, seed=21, scale_range=(0.02, 0.35))
    squash = rng.uniform(0.02, 1.0, g.scale.shape).astype(np.float32)
    squash[np.arange(len(g)), rng.integers(0, 3, len(g))] = 1.0  # one long axis each
    g.scale[:] = (g.scale * squash).astype(np.float32)
    g.opacity[:] = rng.uniform(1.0 / 255, 1.0, g.opacity.shape).astype(np.float32)
    cam = Camera(2160, 3840).yaw(10)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), 3, U)
    x0, x1, r0, r1 = narrowed_rects(res, vs, U)
    qx0, qx1, qr0, qr1 = O.splat_rects(vs, U)
    ids = np.nonzero(vs["visible"] & (qx0 <= qx1) & (qr0 <= qr1))[0]
    narrowed, big = 0, 0
    for gid in ids:
        xs = np.arange(qx0[gid], qx1[gid] + 1)
        rows = np.arange(qr0[gid], qr1[gid] + 1)
        keep = kept_fragments(vs, U, gid, xs, rows)
        inside = ((xs >= x0[gid]) & (xs <= x1[gid]))[None, :] & ((rows >= r0[gid]) & (rows <= r1[gid]))[:, None]
        assert not (keep & ~inside).any(), f"Gaussian {gid}"
        narrowed += int(not inside.all())
        big += int(max(len(xs), len(rows)) > 200)
    assert narrowed > len(ids) // 10 and big > 20, (narrowed, big, len(ids))


def test_radii(gpu):
    g = random_scene(2000, sh_degree=0, seed=8)
    cam = Camera(120, 160)
    res = gpu_frame(g, cam, _settings(), radii=True)
    vs = O.vertex_stage(g.flat(), 3, uniforms_for(cam))
    np.testing.assert_array_equal(res["radii"], O.radii(vs))


def test_default_t_min_error_bound(gpu):
    g = random_scene(3000, sh_degree=3, seed=11, scale_range=(0.02, 0.1))
    cam = Camera(96, 128)
    res, vs, U, ref, info = _check(g, cam, _settings(t_min=1e-4), tol=TOL_TMIN + 2e-5, frac=0.999)


@pytest.mark.parametrize("mode", [-6, -5, -4, -3, -2, -1, 0, 1, 2, 3, 6])
def test_render_modes(gpu, mode):
    g = random_scene(1500, sh_degree=3, seed=20, scale_range=(0.01, 0.06))
    _check(g, Camera(96, 128), _settings(render_mod=mode, t_min=0.0))


def test_appearance_uniforms(gpu):
    g = random_scene(1500, sh_degree=3, seed=21)
    st = _settings(t_min=0.0, dc_factor=0.7, extra_factor=1.6, color_scale=[0.9, 1.1, 0.5],
                   scale_modifier=1.7, screen_scale=1.3, light_rotation=[10.0, -25.0, 40.0], bg=[0.1, 0.2, 0.3])
    st.set_rot_modifier_euler([15.0, -30.0, 5.0])
    # light rotation cos/sin are computed by libm on the host vs numpy in the
    # oracle: allow their last-ulp difference
    _check(g, Camera(96, 128).yaw(30), st, tol=1e-4)


def test_aabb_and_obb_cull(gpu):
    g = random_scene(3000, sh_degree=1, seed=30)
    cam = Camera(120, 160)
    c = g.points_center
    st = _settings(t_min=0.0, enable_aabb=1, points_center=c, cube_min=[-1.0, -0.5, -2.0], cube_max=[0.5, 1.0, 1.0])
    res, vs, *_ = _check(g, cam, st)
    assert 0 < vs["visible"].sum() < len(g)
    st = _settings(t_min=0.0, enable_obb=1, points_center=c, cube_min=[-1.5] * 3, cube_max=[1.5] * 3,
                   cube_rotation=euler_to_rotation_matrix([30, 15, 0]))
    _check(g, cam, st)


def test_gl8_framebuffer_closeness(gpu):
    """The float output against the RGBA8 framebuffer.
    The framebuffer's fixed-point blend (llvmpipe's, pinned by
    tests/golden/llvmpipe_golden.npz) rounds each of its two products to 8 bits,
    so it drifts from the float blend by a few steps over a deep pixel: on this
    scene the oracle's own float and gl8 frames are 99.99 % within 3/255, at
    most 4.07/255 apart, 57.9 dB.  Bounds: 99.9 % within 3/255, none over
    6/255, PSNR >= 50 dB."""
    g = random_scene(2500, sh_degree=3, seed=12)
    cam = Camera(120, 160)
    res = gpu_frame(g, cam, _settings())
    U = uniforms_for(cam)
    ref8 = O.composite(O.vertex_stage(g.flat(), 48, U), U, mode="gl8")
    d = np.abs(res["image"] - ref8)
    assert (d <= 3.0 / 255 + 1e-6).mean() >= 0.999, d.max()
    assert d.max() <= 6.0 / 255, d.max()
    mse = float((d ** 2).mean())
    assert 10 * np.log10(1.0 / max(mse, 1e-20)) >= 50.0


def test_empty_and_culled_scenes(gpu):
    g = random_scene(100, sh_degree=0, seed=1)
    g.xyz[:] = np.array([0, 0, 100.0], np.float32)  # behind the camera at z=5 looking -z
    res = gpu_frame(g, Camera(48, 64), _settings(bg=[0.25, 0.5, 0.75]))
    assert res["stats"]["n_visible"] == 0
    assert np.all(res["image"] == np.array([0.25, 0.5, 0.75], np.float32))


def test_ragged_image_sizes(gpu):
    g = random_scene(1200, sh_degree=0, seed=2, scale_range=(0.02, 0.08))
    for (w, h) in [(17, 9), (33, 47), (100, 1)]:
        _check(g, Camera(h, w), _settings(t_min=0.0))


def test_garden_standin_small(gpu):
    g = garden_standin(6000, seed=1)
    _check(g, Camera(90, 160), _settings(t_min=0.0))


@pytest.mark.parametrize("chunk", ["16", "64"])
def test_multi_chunk_merge(gpu, monkeypatch, chunk):
    """Small compositing chunks force every busy tile through the partial
    (C, T) + in-order merge path."""
    monkeypatch.setenv("GSR_CHUNK", chunk)
    g = random_scene(5000, sh_degree=3, seed=70, scale_range=(0.02, 0.09))
    _check(g, Camera(96, 128), _settings(t_min=0.0))
    _check(g, Camera(96, 128), _settings(t_min=1e-4), tol=TOL_TMIN + 2e-5)


@pytest.mark.parametrize("target,mode", [("64", 0), ("256", 0), ("64", -4), ("64", -5), ("64", -6)])
def test_deep_frame_chunks(gpu, monkeypatch, target, mode):
    """A frame alone with many instances per chunk target (GSR_CHUNK_TARGET:
    chunks of at least n_dup / target instances, here forced on a small
    scene) takes the deep-frame form: longer chunks, first chunks dispatched
    first, later chunks stopped by the earlier ones' transmittance bound
    (api.hip frame_chunk).  Against the oracle at the stated tolerances, for
    every fragment class (the bound form is compiled per class)."""
    monkeypatch.setenv("GSR_CHUNK", "64")
    monkeypatch.setenv("GSR_CHUNK_TARGET", target)
    g = random_scene(20_000, sh_degree=3, seed=71, scale_range=(0.02, 0.09))
    _check(g, Camera(96, 128), _settings(t_min=0.0, render_mod=mode))
    _check(g, Camera(96, 128), _settings(t_min=1e-4, render_mod=mode), tol=TOL_TMIN + 2e-5)
