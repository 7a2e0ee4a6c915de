"""GPU tests of the reference-facing boundary, driven the way the reference
drives it (not only through the C ABI):

* ``GaussianRasterizer`` built exactly as ``CUDARenderer`` builds its settings
  (``renderer_cuda.py:104-120`` init, ``:147-150`` update_gaussian_data,
  ``:196-213`` update_camera_pose / update_camera_intrin) and called as in
  ``CUDARenderer.draw`` (``:226-243``): a NEW rasterizer per frame, shs as
  [N, K, 3], planar color[3,H,W] and radii[N] out;
* ``HIPRenderer`` through the OpenGLRenderer setter sequence of
  ``main.py:128-137`` (update_activated_renderer_state) and the appearance
  setters (``renderer_ogl.py:246-318``);
* ``HipScene.from_flat`` (the flat() SSBO-0 layout, ``renderer_ogl.py:238``,
  ``util_gau.py:40-42``) and the planar output layout.
The oracle is the C restatement of the OGL path (oracle/gl_oracle.c)."""
import ctypes

import numpy as np
import pytest
import torch

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import garden_standin, random_scene
from oracle import c_oracle as C
from oracle import gl_oracle as O
from helpers import TOL_TMIN, compare_images, uniforms_for

pytestmark = pytest.mark.gpu


def _cuda_renderer_settings(camera, sh_dim, w, h):
    """CUDARenderer.raster_settings after __init__ (:106-119),
    update_gaussian_data (:150), update_camera_pose (:196-203) and
    update_camera_intrin (:205-213), restated line by line."""
    rs = {"image_height": int(h), "image_width": int(w), "tanfovx": 1, "tanfovy": 1,
          "bg": torch.Tensor([0., 0., 0]).float().cuda(), "scale_modifier": 1., "viewmatrix": None,
          "projmatrix": None, "sh_degree": 3, "campos": None, "prefiltered": False, "debug": False}
    rs["sh_degree"] = int(np.round(np.sqrt(sh_dim))) - 1
    view_matrix = camera.get_view_matrix()
    view_matrix[[0, 2], :] = -view_matrix[[0, 2], :]
    proj = camera.get_project_matrix() @ view_matrix
    rs["viewmatrix"] = torch.tensor(view_matrix.T).float().cuda()
    rs["campos"] = torch.tensor(camera.position).float().cuda()
    rs["projmatrix"] = torch.tensor(proj.T).float().cuda()
    view_matrix = camera.get_view_matrix()
    view_matrix[[0, 2], :] = -view_matrix[[0, 2], :]
    proj = camera.get_project_matrix() @ view_matrix
    rs["projmatrix"] = torch.tensor(proj.T).float().cuda()
    hfovx, hfovy, focal = camera.get_htanfovxy_focal()
    rs["tanfovx"] = hfovx
    rs["tanfovy"] = hfovy
    return rs


def _gaus_cuda(g):
    """gaus_cuda_from_cpu (renderer_cuda.py:92-101): sh reshaped to [N, K, 3]."""
    t = {f: torch.tensor(getattr(g, f)).float().cuda() for f in ("xyz", "rot", "scale", "opacity", "sh")}
    t["sh"] = t["sh"].reshape(len(g), -1, 3).contiguous()
    return t


def _draw(rs, gc):
    """CUDARenderer.draw's rasterizer call (renderer_cuda.py:226-243)."""
    from gsviewer_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
    raster_settings = GaussianRasterizationSettings(**rs)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    with torch.no_grad():
        img, radii = rasterizer(means3D=gc["xyz"], means2D=None, shs=gc["sh"], colors_precomp=None,
                                opacities=gc["opacity"], scales=gc["scale"], rotations=gc["rot"],
                                cov3D_precomp=None)
    return img, radii


def _oracle(g, U, threads=8):
    return C.render(g.flat(), g.sh_dim, U, threads=threads)


def test_rasterizer_called_like_cuda_renderer(gpu):
    from gsviewer_amd.rasterizer import gl_matrices_from_settings, scene_cache
    g = random_scene(20_000, sh_degree=3, seed=21)
    W, H = 320, 240
    gc = _gaus_cuda(g)
    scene_cache.clear()
    creates0 = scene_cache.creates
    for yaw in (0.0, 35.0, -70.0):
        cam = Camera(H, W).yaw(yaw)
        rs = _cuda_renderer_settings(cam, g.sh.shape[1] // 3, W, H)
        for _ in range(2):   # a new rasterizer per frame, like draw()
            img, radii = _draw(rs, gc)
        torch.cuda.synchronize()
        assert tuple(img.shape) == (3, H, W) and img.dtype == torch.float32
        assert tuple(radii.shape) == (len(g),) and radii.dtype == torch.int32
        # V comes back exactly; P to within the float32 rounding of the product
        # P V' the reference hands over (its [2,3] entry, -0.002, is recovered from
        # -5.002 and keeps ~2.4e-7 absolute error: it only moves the z_ndc clip)
        from gsviewer_amd.rasterizer import GaussianRasterizationSettings
        V, P = gl_matrices_from_settings(GaussianRasterizationSettings(**rs))
        np.testing.assert_array_equal(V, cam.get_view_matrix())
        np.testing.assert_allclose(P, cam.get_project_matrix(), rtol=0, atol=1e-6)
        P0 = cam.get_project_matrix()
        np.testing.assert_array_equal(P[:2], P0[:2])          # x/y rows: exact
        np.testing.assert_array_equal(P[3], P0[3])
        # image and radii against the oracle given the matrices the GPU received
        U = O.default_uniforms(V, P, np.asarray([rs["tanfovx"], rs["tanfovy"], H / (2.0 * rs["tanfovy"])],
                                                np.float32), cam.position, W, H)
        ref = _oracle(g, U)
        compare_images(img.permute(1, 2, 0).cpu().numpy(), ref, tol=TOL_TMIN + 2e-5)
        vs = O.vertex_stage(g.flat(), g.sh_dim, U)
        np.testing.assert_array_equal(radii.cpu().numpy(), O.radii(vs))
        # and against the oracle on the camera's own matrices (the OGL uniforms)
        compare_images(img.permute(1, 2, 0).cpu().numpy(), _oracle(g, uniforms_for(cam)), tol=TOL_TMIN + 2e-5)
    # one scene repack for all frames and cameras (renderer_cuda.py:147-150 happens once)
    assert scene_cache.creates - creates0 == 1
    # update_gaussian_data with new tensors -> a new scene
    gc2 = _gaus_cuda(g)
    _draw(rs, gc2)
    assert scene_cache.creates - creates0 == 2
    # in-place edit of a tensor (version bump) -> a new scene, and the image follows it
    gc2["opacity"].mul_(0.0)
    img, _ = _draw(rs, gc2)
    assert scene_cache.creates - creates0 == 3
    assert float(img.abs().max()) == 0.0
    scene_cache.clear()


def test_rasterizer_sh_degree_caps_like_render_mod(gpu):
    g = random_scene(5000, sh_degree=3, seed=22)
    W, H = 200, 150
    gc = _gaus_cuda(g)
    cam = Camera(H, W).yaw(15)
    rs = _cuda_renderer_settings(cam, 16, W, H)
    for deg in (0, 1, 2):
        rs["sh_degree"] = deg
        img, _ = _draw(rs, gc)
        ref = _oracle(g, uniforms_for(cam, render_mod=deg))
        compare_images(img.permute(1, 2, 0).cpu().numpy(), ref, tol=TOL_TMIN + 2e-5)


def test_hip_renderer_setter_sequence(gpu):
    """main.py:128-137 then appearance/box setters, each draw vs the oracle."""
    from gsviewer_amd.renderer import HIPRenderer
    from gsviewer_amd.rasterizer import RenderSettings
    g = garden_standin(30_000, seed=4, sh_degree=3)
    W, H = 256, 192
    cam = Camera(H, W)
    r = HIPRenderer(W, H, cam)
    # update_activated_renderer_state (main.py:128-137), start-up values (main.py:66-75)
    r.update_gaussian_data(g)
    r.sort_and_update()
    r.set_scale_modifier(1.0)
    r.set_screen_scale_factor(1.0)
    r.set_rot_modifier([0.0, 0.0, 0.0])
    r.set_render_mod(9 - 3)
    r.update_camera_pose()
    r.update_camera_intrin()
    r.set_render_reso(cam.w, cam.h)
    st = RenderSettings()

    def check():
        img = r.draw()
        torch.cuda.synchronize()
        assert tuple(img.shape) == (H, W, 3)
        ref = _oracle(g, uniforms_for(cam, st))
        return compare_images(img.cpu().numpy(), ref, tol=TOL_TMIN + 2e-5)

    check()
    # reduce_updates: an unchanged state returns the same frame object
    assert r.draw() is r.draw()
    r.set_render_mod(1); st.render_mod = 1
    check()
    r.adjust_dc_features(0.7); st.dc_factor = 0.7
    r.adjust_extra_features(1.6); st.extra_factor = 1.6
    r.update_color_factor([1.0, 0.5, 0.8]); st.color_scale = [1.0, 0.5, 0.8]
    r.set_render_mod(3); st.render_mod = 3
    check()
    r.set_scale_modifier(1.7); st.scale_modifier = 1.7
    r.set_light_rotation([10.0, 40.0, 0.0]); st.light_rotation = [10.0, 40.0, 0.0]
    r.set_rot_modifier([20.0, 0.0, 5.0]); st.set_rot_modifier_euler([20.0, 0.0, 5.0])
    check()
    pc = [float(v) for v in g.points_center]
    r.set_points_center(pc); st.points_center = pc
    r.set_enable_obb(1); st.enable_obb = 1
    r.set_cube_rotation([30.0, 15.0, 0.0]); st.set_cube_rotation_euler([30.0, 15.0, 0.0])
    r.set_point_cubeMin([-1.0, -1.0, -1.0]); st.cube_min = [-1.0, -1.0, -1.0]
    r.set_point_cubeMax([1.0, 1.0, 1.0]); st.cube_max = [1.0, 1.0, 1.0]
    check()
    # camera move -> rerender
    cam.yaw(30.0)
    r.update_camera_pose()
    check()
    # the depth-order service matches the reference sort
    order = r.depth_order().cpu().numpy().reshape(-1)
    V = cam.get_view_matrix()
    F = np.float32
    vz = ((F(V[2, 0]) * g.xyz[:, 0] + F(V[2, 1]) * g.xyz[:, 1]) + F(V[2, 2]) * g.xyz[:, 2]) + F(V[2, 3])
    np.testing.assert_array_equal(order, np.argsort(vz, kind="stable"))


def test_scene_from_flat_matches_fields(gpu):
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    g = random_scene(8000, sh_degree=2, seed=23)
    cam = Camera(144, 176).yaw(-20)
    st = RenderSettings(t_min=0.0, out_layout=1)
    outs = []
    for scene in (HipScene.from_gaussian_data(g), HipScene.from_flat(torch.from_numpy(g.flat()).cuda(), g.sh_dim)):
        ctx = HipContext()
        out = torch.empty((cam.h, cam.w, 3), dtype=torch.float32, device="cuda")
        render_into(ctx, scene, camera_from(cam), st, out)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
        ctx.close()
        scene.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    compare_images(outs[1], _oracle(g, uniforms_for(cam, st)))


@pytest.mark.parametrize("chunk", [None, "16"])
def test_planar_layout_equals_interleaved(gpu, monkeypatch, chunk):
    """out_layout 0 ([3,H,W], the rasterizer's) vs 1 ([H,W,3]): the single-chunk
    write path and, with GSR_CHUNK=16, the multi-chunk merge path."""
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    if chunk:
        monkeypatch.setenv("GSR_CHUNK", chunk)
    g = garden_standin(40_000, seed=5, sh_degree=1)
    cam = Camera(180, 320).yaw(10)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    imgs = {}
    for layout in (0, 1):
        st = RenderSettings(t_min=1e-4, out_layout=layout)
        shape = (3, cam.h, cam.w) if layout == 0 else (cam.h, cam.w, 3)
        out = torch.full(shape, -1.0, dtype=torch.float32, device="cuda")
        render_into(ctx, scene, camera_from(cam), st, out)
        torch.cuda.synchronize()
        imgs[layout] = out.cpu().numpy()
    np.testing.assert_array_equal(imgs[0].transpose(1, 2, 0), imgs[1])
    compare_images(imgs[1], _oracle(g, uniforms_for(cam)), tol=TOL_TMIN + 2e-5)
    scene.close()
    ctx.close()


def test_bad_arguments_raise(gpu):
    from gsviewer_amd import _lib
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    g = random_scene(100, sh_degree=0, seed=1)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    cam = Camera(32, 32)
    out = torch.empty((3, 32, 32), dtype=torch.float32, device="cuda")
    with pytest.raises(RuntimeError, match="out_layout"):
        render_into(ctx, scene, camera_from(cam), RenderSettings(out_layout=2), out)
    lib = _lib.load()
    st = RenderSettings().to_c()
    st.out_layout = 7
    rc = lib.gsr_render(ctx.handle, scene.handle, ctypes.byref(camera_from(cam)), ctypes.byref(st),
                        ctypes.c_void_p(out.data_ptr()), None, None)
    assert rc == _lib.GSR_ERR_INVALID and b"out_layout" in lib.gsr_last_error()
    st = RenderSettings().to_c()
    st.t_min = 1.5
    rc = lib.gsr_render(ctx.handle, scene.handle, ctypes.byref(camera_from(cam)), ctypes.byref(st),
                        ctypes.c_void_p(out.data_ptr()), None, None)
    assert rc == _lib.GSR_ERR_INVALID
    # the context still renders after rejected calls
    render_into(ctx, scene, camera_from(cam), RenderSettings(out_layout=0), out)
    torch.cuda.synchronize()
    scene.close()
    ctx.close()


def test_context_regrowth_sequence(gpu):
    """One context through empty -> small -> large -> small -> larger scenes and
    frame sizes (buffers grow without freeing in-flight memory): every frame
    equals a fresh context's frame."""
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    cases = [(0, 64, 48), (500, 64, 48), (200_000, 640, 360), (300, 32, 32), (400_000, 1280, 720)]
    shared = HipContext()
    for n, w, h in cases:
        g = random_scene(max(n, 1), sh_degree=1, seed=n % 97)[:n] if n else random_scene(1, sh_degree=1)[:0]
        scene = HipScene.from_gaussian_data(g)
        cam = Camera(h, w).yaw(7.0)
        st = RenderSettings(out_layout=1)
        imgs = []
        for ctx in (shared, HipContext()):
            out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
            render_into(ctx, scene, camera_from(cam), st, out)
            torch.cuda.synchronize()
            imgs.append(out.cpu().numpy())
            assert ctx.stats()["n_gaussians"] == n
        np.testing.assert_array_equal(imgs[0], imgs[1])
        if n == 0:
            assert float(np.abs(imgs[0]).max()) == 0.0
        scene.close()
    shared.close()


def test_context_reserve_means_no_allocation_in_frames(gpu):
    """gsr_context_reserve sizes the workspace up front: frames within the
    reserved bounds (scene size, frame size, instances) make no device
    allocation, across views in flight on other streams; a frame beyond them
    still grows (and stays correct)."""
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    g = random_scene(50_000, sh_degree=1, seed=11)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    ctx.reserve(50_000, 640, 480, max_instances=400_000)
    b0, a0 = ctx.workspace()
    assert b0 > 50_000 * 48 and a0 > 0
    st = RenderSettings(out_layout=0)
    ref_ctx = HipContext()
    s = torch.cuda.Stream()
    for yaw in (0.0, 40.0, 80.0):
        for w, h in ((640, 480), (320, 200)):
            cam = camera_from(Camera(h, w).yaw(yaw))
            out = torch.empty((3, h, w), dtype=torch.float32, device="cuda")
            ref = torch.empty_like(out)
            render_into(ctx, scene, cam, st, out, stream=s)
            render_into(ref_ctx, scene, cam, st, ref)
            s.synchronize()
            torch.cuda.synchronize()
            assert ctx.stats()["n_instances"] <= 400_000
            assert torch.equal(out, ref)
    assert ctx.workspace() == (b0, a0)
    # beyond the reservation: grows, still the same image
    big = HipScene.from_gaussian_data(random_scene(120_000, sh_degree=1, seed=12))
    cam = camera_from(Camera(720, 1280))
    out = torch.empty((3, 720, 1280), dtype=torch.float32, device="cuda")
    ref = torch.empty_like(out)
    render_into(ctx, big, cam, st, out)
    render_into(HipContext(), big, cam, st, ref)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert ctx.workspace()[1] > a0
    with pytest.raises(RuntimeError, match="context_reserve"):
        ctx.reserve(-1, 64, 64)
    ctx.close()
    ref_ctx.close()
    scene.close()
    big.close()


def test_caller_provided_workspace(gpu):
    """gsr_workspace_size + gsr_context_attach_workspace (the
    rasterizer writes into caller-provided output and workspace): a context
    carved out of a caller's device tensor (unaligned base) renders the same
    images as a self-allocating one, makes no allocation of its own, and a
    frame beyond its bounds or a too-small workspace fails loudly."""
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into, workspace_size
    n, w, h, d = 50_000, 640, 480, 400_000
    need = workspace_size(n, w, h, d)
    probe = HipContext()
    probe.reserve(n, w, h, max_instances=d)
    held, _ = probe.workspace()
    probe.close()
    assert held <= need <= held + 256 * 32
    g = random_scene(n, sh_degree=1, seed=11)
    scene = HipScene.from_gaussian_data(g)
    base = torch.empty(need + 7, dtype=torch.uint8, device="cuda")
    ws = base[7:]
    ws.fill_(0xAB)  # the context must not rely on zeroed memory
    torch.cuda.synchronize()
    ctx = HipContext()
    ctx.attach_workspace(ws, n, w, h, max_instances=d)  # enqueues nothing: no sync before the side stream
    b0, a0 = ctx.workspace()
    assert b0 == held
    st = RenderSettings(out_layout=0)
    ref_ctx = HipContext()
    s = torch.cuda.Stream()
    for yaw in (0.0, 40.0, 80.0):
        for ww, hh in ((640, 480), (320, 200)):
            cam = camera_from(Camera(hh, ww).yaw(yaw))
            out = torch.empty((3, hh, ww), dtype=torch.float32, device="cuda")
            ref = torch.empty_like(out)
            render_into(ctx, scene, cam, st, out, stream=s)
            render_into(ref_ctx, scene, cam, st, ref)
            s.synchronize()
            torch.cuda.synchronize()
            assert torch.equal(out, ref)
    assert ctx.workspace() == (b0, a0)
    # the frames wrote into the caller's tensor (it was filled with 0xAB before the attach)
    assert int((ws != 0xAB).sum()) > 50_000
    big = HipScene.from_gaussian_data(random_scene(120_000, sh_degree=1, seed=12))
    out = torch.empty((3, h, w), dtype=torch.float32, device="cuda")
    with pytest.raises(RuntimeError, match="exceeds the bounds"):
        render_into(ctx, big, camera_from(Camera(h, w)), st, out)
    torch.cuda.synchronize()
    # nothing was carved past the reservation, and a frame within the bounds still renders
    assert ctx.workspace() == (b0, a0)
    cam = camera_from(Camera(h, w).yaw(40.0))
    render_into(ctx, scene, cam, st, out, stream=s)
    ref = torch.empty_like(out)
    render_into(ref_ctx, scene, cam, st, ref)
    s.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    ctx.close()
    small = HipContext()
    with pytest.raises(RuntimeError, match="too small"):
        small.attach_workspace(ws[: need // 2], n, w, h, max_instances=d)
    small.close()
    used = HipContext()
    render_into(used, scene, camera_from(Camera(h, w)), st, out)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="already holds"):
        used.attach_workspace(ws, n, w, h, max_instances=d)
    used.close()
    ref_ctx.close()
    scene.close()
    big.close()


def test_wait_for_counts_has_a_deadline(gpu, monkeypatch):
    """A stream that makes no progress fails gsr_render_finish with
    GSR_ERR_HIP after GSR_WAIT_TIMEOUT_MS instead of hanging the host; the
    context then refuses new frames."""
    import time
    from gsviewer_amd import _lib
    from gsviewer_amd.rasterizer import (HipContext, HipScene, RenderSettings, _stream_handle, camera_from,
                                         render_begin, render_finish, render_into)
    monkeypatch.setenv("GSR_WAIT_TIMEOUT_MS", "300")
    g = random_scene(1000, sh_degree=0, seed=3)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    cam = Camera(48, 64)
    out = torch.empty((3, 48, 64), dtype=torch.float32, device="cuda")
    st = RenderSettings(out_layout=0)
    s = torch.cuda.Stream()
    lib = _lib.load()
    _lib.check(lib.gsr_debug_stall(_stream_handle(s), 1_500_000), "debug_stall")  # 1.5 s of a busy stream
    render_begin(ctx, scene, camera_from(cam), st, out, stream=s)
    t0 = time.perf_counter()
    with pytest.raises(RuntimeError, match="timed out"):
        render_finish(ctx, s)
    assert 0.25 < time.perf_counter() - t0 < 1.4
    s.synchronize()
    with pytest.raises(RuntimeError, match="failed earlier"):
        render_begin(ctx, scene, camera_from(cam), st, out, stream=s)
    ctx.close()
    # a new context works
    ctx2 = HipContext()
    render_into(ctx2, scene, camera_from(cam), st, out)
    torch.cuda.synchronize()
    ctx2.close()
    scene.close()


@pytest.mark.parametrize("how", ["reserve", "attach"])
def test_first_frame_on_side_stream_after_sizing(gpu, how):
    """gsr_context_reserve / gsr_context_attach_workspace on torch's default
    stream, then the context's first frame at once on a fresh non-blocking
    stream with no synchronisation (bench.py's order): the sizing calls
    enqueue nothing, and the first frame zeroes its completion counter on its
    own stream, so the frame publishes its counts and matches the oracle."""
    import numpy as np
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into, workspace_size
    from oracle import gl_oracle as O
    n, w, h = 3000, 160, 120
    g = random_scene(n, sh_degree=1, seed=21)
    scene = HipScene.from_gaussian_data(g)
    torch.cuda.synchronize()
    ws = None
    for yaw in (0.0, 30.0):
        ctx = HipContext()
        if how == "reserve":
            ctx.reserve(n, w, h)
        else:
            ws = torch.empty(workspace_size(n, w, h), dtype=torch.uint8, device="cuda")
            ws.fill_(0xFF)  # a stale all-ones counter would never publish (V, D, seq)
            ctx.attach_workspace(ws, n, w, h)
        s = torch.cuda.Stream()
        if ws is not None:
            # the all-ones fill is really there when the frame starts: the stale-counter case is exercised
            # every time, not only when the fill happens to land first (the sizing call itself syncs nothing)
            s.wait_stream(torch.cuda.current_stream())
        cam = Camera(h, w).yaw(yaw)
        out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        st = RenderSettings(out_layout=1, t_min=0.0)
        with torch.cuda.stream(s):
            render_into(ctx, scene, camera_from(cam), st, out, stream=s)
            render_into(ctx, scene, camera_from(cam), st, out, stream=s)  # the re-armed counter
        s.synchronize()
        img = out.cpu().numpy()
        U = O.default_uniforms(cam.get_view_matrix(), cam.get_project_matrix(),
                               np.asarray(cam.get_htanfovxy_focal(), np.float32), cam.position, w, h)
        ref = O.composite(O.vertex_stage(g.flat(), g.sh_dim, U), U)
        d = np.abs(img - ref)
        assert (d <= 2e-5).mean() >= 0.999 and d.max() <= 2e-3, (d.max(), (d > 2e-5).sum())
        ctx.close()
    scene.close()


def test_finish_views_nomem_ends_every_view(gpu):
    """A group finish that fails with GSR_ERR_NOMEM (a view's instances beyond
    its caller workspace) ends every view's frame: each context then begins
    and finishes a frame within its bounds (later contexts of the
    group used to stay 'active' and refuse their next frame)."""
    from gsviewer_amd.rasterizer import (HipContext, HipScene, RenderSettings, camera_from, render_begin_sorts,
                                         render_begin_views, render_finish_views, render_into, workspace_size)
    n, w, h = 20_000, 320, 240
    g = random_scene(n, sh_degree=0, seed=5)
    scene = HipScene.from_gaussian_data(g)
    st = RenderSettings(out_layout=0)
    cams = [camera_from(Camera(h, w).yaw(30.0 * v)) for v in range(3)]
    outs = [torch.empty((3, h, w), dtype=torch.float32, device="cuda") for _ in range(3)]
    probe = HipContext()
    render_into(probe, scene, cams[0], st, outs[0])
    torch.cuda.synchronize()
    d0 = probe.stats()["n_instances"]
    probe.close()
    assert d0 > 1000
    wss, ctxs = [], []
    for v in range(3):
        d = d0 // 4 if v == 0 else 8 * d0  # view 0's workspace holds a quarter of a frame's instances
        wss.append(torch.empty(workspace_size(n, w, h, d), dtype=torch.uint8, device="cuda"))
        c = HipContext()
        c.attach_workspace(wss[-1], n, w, h, max_instances=d)
        ctxs.append(c)
    s = torch.cuda.Stream()
    render_begin_views(ctxs, scene, cams, st, outs, stream=s)
    render_begin_sorts(ctxs, stream=s)
    with pytest.raises(RuntimeError, match="exceeds the bounds|too small"):
        render_finish_views(ctxs, stream=s)
    s.synchronize()
    # every context takes a new frame; views 1 and 2 render correctly
    for v in (1, 2):
        ref_ctx = HipContext()
        ref = torch.empty_like(outs[v])
        render_into(ref_ctx, scene, cams[v], st, ref)
        render_into(ctxs[v], scene, cams[v], st, outs[v], stream=s)
        s.synchronize()
        torch.cuda.synchronize()
        assert torch.equal(outs[v], ref)
        ref_ctx.close()
    # view 0 within its bounds: a scene of 500 Gaussians
    few = HipScene.from_gaussian_data(random_scene(500, sh_degree=0, seed=6))
    ref_ctx = HipContext()
    ref = torch.empty_like(outs[0])
    render_into(ref_ctx, few, cams[0], st, ref)
    render_into(ctxs[0], few, cams[0], st, outs[0], stream=s)
    s.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(outs[0], ref)
    ref_ctx.close()
    few.close()
    for c in ctxs:
        c.close()
    scene.close()


def test_instance_count_beyond_32_bits_fails_the_frame(gpu):
    """600K splats that each cover every tile of a 1080p frame make 4.9e9 tile
    instances: the frame fails with GSR_ERR_OVERFLOW (the count's high word is
    published beside it) instead of overrunning the instance buffers, and the
    context renders its next frame normally."""
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    g = random_scene(600_000, sh_degree=0, seed=31, extent=0.5)
    g.scale[:] = 30.0
    g.opacity[:] = 0.99
    huge = HipScene.from_gaussian_data(g)
    cam = Camera(1080, 1920)
    st = RenderSettings(t_min=1e-4, out_layout=1)
    ctx = HipContext()
    out = torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda")
    with pytest.raises(RuntimeError, match="tile instances"):
        render_into(ctx, huge, camera_from(cam), st, out)
    torch.cuda.synchronize()
    huge.close()
    small = garden_standin(20_000, seed=32, sh_degree=1)
    scene = HipScene.from_gaussian_data(small)
    cam2 = Camera(180, 320).yaw(30)
    o1 = torch.empty((180, 320, 3), dtype=torch.float32, device="cuda")
    o2 = torch.empty_like(o1)
    render_into(ctx, scene, camera_from(cam2), st, o1)
    fresh = HipContext()
    render_into(fresh, scene, camera_from(cam2), st, o2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(o1.cpu().numpy(), o2.cpu().numpy())
    for c in (ctx, fresh):
        c.close()
    scene.close()
