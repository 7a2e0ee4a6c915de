"""GPU parity at scale: the sorts and the tile binning over many radix tiles.

The small-scene parity tests fit in one 4096-item radix tile; these cover
hundreds of tiles, exact depth ties and narrow/wide depth ranges (the depth
sort chooses its digit width on the device from the frame's key range).
Checks are exact (integer order and index work) against the oracle's
vertex stage and NumPy's stable argsort (pinned to the reference's
_sort_gaussian_cpu by tests/test_oracle_golden.py)."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import GaussianData, garden_standin, random_scene
from oracle import gl_oracle as O
from helpers import frame_depth_order, gpu_frame, narrowed_rects, uniforms_for

pytestmark = pytest.mark.gpu

TILE = 16


def _settings(**kw):
    from gsviewer_amd.rasterizer import RenderSettings
    return RenderSettings(**kw)


def expected_instances(vs, U, rects):
    """(tile, gid) of every tile instance of the visible splats, vectorized."""
    W, H = U["width"], U["height"]
    tiles_x = (W + TILE - 1) // TILE
    x0, x1, r0, r1 = rects[:4]
    ok = vs["visible"] & (x0 <= x1) & (r0 <= r1)
    gid = np.nonzero(ok)[0]
    tx0, tx1, ty0, ty1 = x0[gid] // TILE, x1[gid] // TILE, r0[gid] // TILE, r1[gid] // TILE
    ntx = tx1 - tx0 + 1
    cnt = ntx * (ty1 - ty0 + 1)
    rep = np.repeat(np.arange(len(gid)), cnt)
    k = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    tile = (ty0[rep] + k // ntx[rep]) * tiles_x + tx0[rep] + k % ntx[rep]
    return tile.astype(np.int64), gid[rep]


def check_frame_order(res, vs, U):
    vis = vs["visible"]
    vis_desc = np.nonzero(vis)[0][::-1]          # compact slot -> Gaussian id
    nv = len(vis_desc)
    assert res["stats"]["n_visible"] == nv
    # global front-to-back order == reverse of the GL draw order (ties: descending id)
    f2b = O.sort_back_to_front(vs["view_z"], vis)[::-1]
    np.testing.assert_array_equal(vis_desc[res["depth_order"]], frame_depth_order(vs, res["depth_coarse"]))
    # every tile list == the global order restricted to the tile
    rank = np.empty(len(vis), np.int64)
    rank[f2b] = np.arange(nv)
    # the quads narrowed by the alpha box (tests/helpers.py mirrors preprocess.hip)
    tile_e, gid_e = expected_instances(vs, U, narrowed_rects(res, vs, U))
    o = np.lexsort((rank[gid_e], tile_e))
    tile_e, gid_e = tile_e[o], gid_e[o]
    ranges = res["ranges"].astype(np.int64)
    lens = ranges[:, 1] - ranges[:, 0]
    assert res["stats"]["n_instances"] == len(gid_e) == int(lens.sum())
    np.testing.assert_array_equal(lens, np.bincount(tile_e, minlength=len(ranges)))
    nz = lens > 0
    np.testing.assert_array_equal(ranges[nz, 0], np.concatenate([[0], np.cumsum(lens[nz])[:-1]]))
    np.testing.assert_array_equal(vis_desc[res["tile_list"]], gid_e)


@pytest.mark.parametrize("n,seed", [(300_000, 3), (70_001, 4)])
def test_depth_order_and_tile_lists_many_radix_tiles(gpu, n, seed):
    g = random_scene(n, sh_degree=0, seed=seed, scale_range=(0.003, 0.03))
    cam = Camera(270, 480).yaw(10)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    U = uniforms_for(cam)
    check_frame_order(res, O.vertex_stage(g.flat(), g.sh_dim, U), U)


def test_garden_standin_order_1080p(gpu):
    g = garden_standin(400_000, seed=1, sh_degree=0)
    cam = Camera(1080, 1920).yaw(45)
    res = gpu_frame(g, cam, _settings(), with_debug=True)
    U = uniforms_for(cam)
    check_frame_order(res, O.vertex_stage(g.flat(), g.sh_dim, U), U)


def _plane_scene(n, zvals, seed):
    """Gaussians on a few exact depth planes: massive exact ties and a tiny key range."""
    rng = np.random.default_rng(seed)
    xyz = np.empty((n, 3), np.float32)
    xyz[:, :2] = rng.uniform(-2, 2, (n, 2))
    xyz[:, 2] = rng.choice(np.asarray(zvals, np.float32), n)
    rot = np.tile(np.array([1, 0, 0, 0], np.float32), (n, 1))
    scale = np.full((n, 3), 0.01, np.float32)
    opacity = np.full((n, 1), 0.5, np.float32)
    sh = rng.normal(0, 0.5, (n, 3)).astype(np.float32)
    return GaussianData(xyz, rot, scale, opacity, sh)


@pytest.mark.parametrize("zvals", [[0.0], [0.0, 0.25, -0.75], [0.0, 1e-6]])
def test_exact_depth_ties_and_narrow_key_range(gpu, zvals):
    g = _plane_scene(50_000, zvals, seed=len(zvals))
    cam = Camera(240, 320)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    U = uniforms_for(cam)
    check_frame_order(res, O.vertex_stage(g.flat(), g.sh_dim, U), U)


def test_sort_depth_service_matches_reference_golden(gpu, golden):
    """gsr_sort_depth == renderer_ogl._sort_gaussian_cpu on the reference's own outputs."""
    from gsviewer_amd.rasterizer import HipScene, depth_order
    g = GaussianData(golden["rand_xyz"], golden["rand_rot"], golden["rand_scale"], golden["rand_opacity"],
                     golden["rand_sh"])
    scene = HipScene.from_gaussian_data(g)
    for V, ref in zip(golden["sort_views"], golden["sort_index"]):
        got = depth_order(scene, V).cpu().numpy().reshape(-1)
        np.testing.assert_array_equal(got, ref)
    scene.close()


def test_sort_depth_service_1m_with_ties(gpu):
    from gsviewer_amd.rasterizer import HipScene, depth_order
    g = random_scene(1_000_000, sh_degree=0, seed=9)
    V = Camera(1080, 1920).yaw(30).get_view_matrix()
    F = np.float32
    x, y, z = g.xyz[:, 0], g.xyz[:, 1], g.xyz[:, 2]
    vz = ((F(V[2, 0]) * x + F(V[2, 1]) * y) + F(V[2, 2]) * z) + F(V[2, 3])
    want = np.argsort(vz, kind="stable")
    assert len(np.unique(vz)) < len(vz), "the case must contain exact ties"
    scene = HipScene.from_gaussian_data(g)
    got = depth_order(scene, V).cpu().numpy().reshape(-1)
    scene.close()
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("limit", ["0", "1700", "1900"])
def test_binning_mixes_staged_and_direct_blocks(gpu, monkeypatch, limit):
    """k_bin_write stages a block's instances in LDS only when the block holds
    at most GSR_BIN_STAGE_LIMIT (default 2048) of them; larger blocks write
    directly.  The garden stand-in averages ~1.8 instances per splat, so the
    limits 1700 / 1900 split one frame's 1024-splat blocks between the two
    paths (0: every block direct).  Single view (k_bin_write) and a group of
    views (k_bin_write_views): the tile lists must be the oracle's exactly.
    That is the separate binning (GSR_BIN_FUSED=0); both knobs are read at
    context creation."""
    from gsviewer_amd.rasterizer import HipScene
    from helpers import batched_frames
    monkeypatch.setenv("GSR_BIN_STAGE_LIMIT", limit)
    monkeypatch.setenv("GSR_BIN_FUSED", "0")
    g = garden_standin(200_000, seed=1, sh_degree=0)
    cam = Camera(540, 960).yaw(45)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    res = gpu_frame(g, cam, _settings(), with_debug=True)
    check_frame_order(res, vs, U)
    scene = HipScene.from_gaussian_data(g)
    cams = [cam, Camera(540, 960).yaw(135)]
    got = batched_frames(scene, cams, _settings(), group=2, debug_views=(0,))
    scene.close()
    check_frame_order(got[0], vs, U)


def test_frame_wider_than_packed_rects(gpu):
    """A frame of more than 256 tiles across: the depth sort carries no packed
    rect payload and the binning gathers the rects by record slot.  Only a
    band of the scene is visible, so (fused cull, uncompacted slots) the
    gathered slots reach past V: tile lists exactly the oracle's."""
    g = garden_standin(100_000, seed=4, sh_degree=0)
    cam = Camera(96, 4128).yaw(20)  # 258 x 6 tiles
    cam.target_dist = 1.0  # inside the scene: ~74 % visible
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    nv = int(vs["visible"].sum())
    assert 0 < nv < len(g) * 0.9, nv
    res = gpu_frame(g, cam, _settings(), with_debug=True)
    assert res["stats"]["tiles_x"] > 256
    check_frame_order(res, vs, U)
