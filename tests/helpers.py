"""Shared test helpers: run the same frame through the HIP path and the oracle."""
from __future__ import annotations

import numpy as np

from gsviewer_amd.camera import Camera
from oracle import gl_oracle as O

# Stated float tolerances (north star: "pixel-for-pixel within a stated float
# tolerance").  Exact mode (t_min = 0): per-splat records are bit-identical,
# so image differences come only from blend order (front-to-back with T vs
# back-to-front over) and exp() ulps.
TOL_EXACT = 2e-5           # |GPU - oracle(float)| per channel, exact mode
TOL_EXACT_FRAC = 0.999     # fraction of pixel-channels within TOL_EXACT
TOL_MAX = 8e-3             # any pixel-channel: a fragment whose alpha sits on the 1/255 discard
                           # threshold can be kept on one side and dropped on the other (exp ulps);
                           # one such flip moves a channel by < alpha * |colour| <= 1/255 * 0.99,
                           # and two flips in one pixel stay below 2/255 = 7.8e-3
TOL_TMIN = 1e-4            # extra error allowed by early termination at t_min = 1e-4


def depth_coarse_bits(path="alone") -> int:
    """A frame depth sort's coarse bits: api.hip kDepthCoarseAlone for a frame
    alone (gsr_render; GSR_DEPTH_COARSE=0 exact, 8..16 otherwise), 0 for a
    group's frames (always exact)."""
    import os
    if path != "alone" or os.environ.get("GSR_BIN_FUSED") == "0":  # (the repair needs the fused binning's keys)
        return 0
    bits = 16
    v = os.environ.get("GSR_DEPTH_COARSE")
    if v is not None and (int(v) == 0 or 8 <= int(v) <= 16):
        bits = int(v)
    return bits


def frame_depth_order(vs, coarse=None):
    """The order a frame's depth sort leaves (GSR_DEBUG_DEPTH_ORDER), as Gaussian
    ids front to back.  Exact: the reverse of the GL draw order (ties: descending
    id).  Coarse (the default, api.hip kDepthCoarse): only the top `coarse` bits
    of the frame's key range (key = order-preserving bits of -z, minus the
    smallest visible key) are ordered, equal coarse keys by descending id; the
    tile lists are still exact (k_tile_ranges restores each run)."""
    vis = vs["visible"]
    f2b = O.sort_back_to_front(vs["view_z"], vis)[::-1]
    coarse = depth_coarse_bits("alone") if coarse is None else coarse
    if coarse == 0:
        return f2b
    gid = np.nonzero(vis)[0]
    if gid.size == 0:
        return f2b
    b = (-vs["view_z"][gid].astype(np.float32)).view(np.uint32).astype(np.uint64)
    key = np.where(b & 0x80000000, ~b & 0xFFFFFFFF, b | 0x80000000)
    kmin, kmax = int(key.min()), int(key.max())
    B = (kmax - kmin).bit_length()
    s0 = max(0, B - coarse)
    ck = (key - kmin) >> np.uint64(s0)
    return gid[np.lexsort((-gid, ck))]


def check_depth_order(res, vs):
    """A frame's GSR_DEBUG_DEPTH_ORDER against frame_depth_order with the
    frame's coarse bits (res["depth_coarse"], 0 when absent)."""
    vis_desc = np.nonzero(vs["visible"])[0][::-1]
    np.testing.assert_array_equal(vis_desc[res["depth_order"]], frame_depth_order(vs, res.get("depth_coarse", 0)))
    return True


def uniforms_for(cam: Camera, settings=None, **over):
    """Oracle uniform dict from a Camera + RenderSettings (same inputs the GPU gets)."""
    V = cam.get_view_matrix()
    P = cam.get_project_matrix()
    kw = {}
    if settings is not None:
        kw = dict(gaussian_scale_factor=np.float32(settings.scale_modifier),
                  screen_display_scale_factor=np.float32(settings.screen_scale),
                  dc_factor=np.float32(settings.dc_factor), extra_factor=np.float32(settings.extra_factor),
                  color_scale_factors=np.asarray(settings.color_scale, np.float32),
                  render_mod=int(settings.render_mod),
                  rot_modifier=np.asarray(settings.rot_modifier, np.float32),
                  light_rotation=np.asarray(settings.light_rotation, np.float32),
                  points_center=np.asarray(settings.points_center, np.float32),
                  enable_aabb=int(settings.enable_aabb), enable_obb=int(settings.enable_obb),
                  cube_rotation=np.asarray(settings.cube_rotation, np.float32),
                  cubeMin=np.asarray(settings.cube_min, np.float32),
                  cubeMax=np.asarray(settings.cube_max, np.float32),
                  bg=np.asarray(settings.bg, np.float32))
    kw.update(over)
    return O.default_uniforms(V, P, np.asarray(cam.get_htanfovxy_focal(), np.float32), cam.position, cam.w, cam.h,
                              **kw)


def gpu_frame(g, cam, settings, with_debug=False, radii=False):
    """Render on the GPU through the C ABI; returns numpy image [H,W,3] (+extras)."""
    import ctypes

    import torch

    from gsviewer_amd import _lib
    from gsviewer_amd.rasterizer import HipContext, HipScene, camera_from, render_into

    scene = HipScene.from_gaussian_data(g.astype32())
    ctx = HipContext()
    out = torch.empty((cam.h, cam.w, 3), dtype=torch.float32, device="cuda")
    rad = torch.empty((len(g),), dtype=torch.int32, device="cuda") if radii else None
    settings.out_layout = 1
    render_into(ctx, scene, camera_from(cam), settings, out, rad)
    torch.cuda.synchronize()
    # the coarse bits this frame's depth sort took (0: exact; scenes over 2M Gaussians sort exactly, api.hip
    # kCoarseMaxN)
    res = {"image": out.cpu().numpy(), "stats": ctx.stats(), "depth_coarse": ctx.knob("frame_coarse")}
    if radii:
        res["radii"] = rad.cpu().numpy()
    if with_debug:
        res.update(grab_debug(ctx, res["stats"]))
    scene.close()
    ctx.close()
    return res


def grab_debug(ctx, st):
    """The last frame's internal arrays of a context (gsr_debug_copy)."""
    import ctypes

    import torch

    from gsviewer_amd import _lib
    lib = _lib.load()
    nv, nd, nt = st["n_visible"], st["n_instances"], st["tiles_x"] * st["tiles_y"]

    def grab(what, nbytes, dtype):
        buf = torch.empty(max(nbytes, 4) // 4 + 1, dtype=torch.int32, device="cuda")
        got = lib.gsr_debug_copy(ctx.handle, what, ctypes.c_void_p(buf.data_ptr()), nbytes, None)
        assert got >= 0, lib.gsr_last_error()
        torch.cuda.synchronize()
        return buf.cpu().numpy().view(np.uint8)[:got].view(dtype)

    n_all = max(int(st.get("n_gaussians", nv)), nv)
    records = grab(_lib.GSR_DEBUG_RECORDS, n_all * 48, np.uint8)
    depth_order = grab(_lib.GSR_DEBUG_DEPTH_ORDER, nv * 4, np.uint32)
    tile_list = grab(_lib.GSR_DEBUG_TILE_LIST, nd * 4, np.uint32)
    if records.size == n_all * 48 and n_all != nv:
        # culling fused into the preprocess (GSR_FUSED_CULL, the default):
        # Gaussian i owns slot n-1-i.  The compacted slots of the separate
        # cull keep the same order, so the visible slots map to them by rank.
        vis_slots = np.sort(depth_order)
        records = records.reshape(n_all, 48)[vis_slots]
        depth_order = np.searchsorted(vis_slots, depth_order).astype(np.uint32)
        tile_list = np.searchsorted(vis_slots, tile_list).astype(np.uint32)
    return dict(records=records.reshape(nv, 48), depth_order=depth_order,
                ranges=grab(_lib.GSR_DEBUG_TILE_RANGES, nt * 8, np.uint32).reshape(nt, 2),
                tile_list=tile_list)


def batched_frames(scene, cams, settings, group=4, debug_views=()):
    """Render len(cams) views through the path bench.py times:
    ViewBatchPipeline (shared cull + preprocess per group, batched depth
    sorts, batched finish), one stream per group, planar [3,H,W] outputs.
    Returns per view: image [H,W,3] (numpy), stats, and the debug arrays for
    the views listed in debug_views."""
    import torch

    from gsviewer_amd.multiview import ViewBatchPipeline
    from gsviewer_amd.rasterizer import HipContext, camera_from
    assert len(cams) % group == 0
    settings.out_layout = 0
    ctxs = [HipContext() for _ in cams]
    outs = [torch.full((3, c.h, c.w), -1.0, dtype=torch.float32, device="cuda") for c in cams]
    streams = [torch.cuda.Stream() for _ in range(len(cams) // group)]
    camcs = [camera_from(c) for c in cams]
    groups = [(ctxs[i:i + group], camcs[i:i + group], outs[i:i + group], streams[i // group])
              for i in range(0, len(cams), group)]
    pipe = ViewBatchPipeline(groups, scene, settings)
    for _ in groups:
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()
    res = []
    for v, (ctx, out) in enumerate(zip(ctxs, outs)):
        r = {"image": out.permute(1, 2, 0).contiguous().cpu().numpy(), "stats": ctx.stats(),
             "depth_coarse": depth_coarse_bits("views")}
        if v in debug_views:
            r.update(grab_debug(ctx, r["stats"]))
        res.append(r)
    for c in ctxs:
        c.close()
    return res


def error_census(gpu, ref, tol):
    """Count and locate the channels whose |GPU - oracle| exceeds `tol`."""
    d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    bad = d > tol
    ys, xs, _ = np.nonzero(bad)
    return dict(max=float(d.max()), mean=float(d.mean()), n_over=int(bad.sum()), channels=int(d.size),
                frac_over=float(bad.mean()), pixels_over=int(bad.any(axis=2).sum()),
                over_gt_1e3=int((d > 1e-3).sum()), over_gt_4e3=int((d > 4e-3).sum()),
                rows=(int(ys.min()), int(ys.max())) if len(ys) else None)


def decode_records(raw):
    """48-B SplatRec (gsviewer_amd/csrc/gsr_internal.h)."""
    f = raw.view(np.float32).reshape(-1, 12)
    u = raw.view(np.uint32).reshape(-1, 12)
    return dict(center=f[:, 0:2], opacity=f[:, 2], x0=(u[:, 3] & 0xFFFF).astype(np.int64),
                x1=(u[:, 3] >> 16).astype(np.int64), qa=f[:, 4], qb=f[:, 5], qc=f[:, 6],
                r0=(u[:, 7] & 0xFFFF).astype(np.int64), r1=(u[:, 7] >> 16).astype(np.int64), color=f[:, 8:11],
                mid=f[:, 11])


def expected_interval_form(opacity, color):
    """kFragGauss record fields in interval form (gsr_internal.h, SplatRec):
    s = sqrt(opacity/255)/0.99 and 0.99*colour, both correctly rounded float32
    (exact), and mid = -log2(255*opacity)/2 (device log2f: compare with a
    tolerance)."""
    F = np.float32
    op = np.asarray(opacity, F)
    s = (np.sqrt(op / F(255.0)) / F(0.99)).astype(F)
    col = (F(0.99) * np.asarray(color, F)).astype(F)
    with np.errstate(divide="ignore"):
        mid = -0.5 * np.log2(255.0 * op.astype(np.float64))
    return s, col, mid


def expected_quadratic(vs):
    """qa, qb, qc of the record from the oracle's conic and coordxy scale, in
    the kernel's float32 evaluation order (preprocess.hip)."""
    F = np.float32
    L = F(1.4426950408889634)
    A, B, C = vs["conic"][:, 0], vs["conic"][:, 1], vs["conic"][:, 2]
    sx, sy = vs["coord_scale"][:, 0], vs["coord_scale"][:, 1]
    qa = (((F(-0.5) * L) * A) * sx) * sx
    qb = (((-L) * B) * sx) * sy
    qc = (((F(-0.5) * L) * C) * sy) * sy
    return qa.astype(F), qb.astype(F), qc.astype(F)


def compare_images(gpu, ref, tol=TOL_EXACT, frac=TOL_EXACT_FRAC, tol_max=TOL_MAX):
    d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    ok_frac = float((d <= tol).mean())
    info = dict(max=float(d.max()), ok_frac=ok_frac, mean=float(d.mean()))
    assert np.isfinite(gpu).all(), "non-finite pixels"
    assert ok_frac >= frac, info
    assert d.max() <= tol_max, info
    return info


def alpha_box_rects(rec, rects, height):
    """The preprocess's alpha-box narrowing of the covered rectangles
    (preprocess.hip alpha_box), mirrored op for op in float32 from the
    record's own quadratic form, centre and mid (kFragGauss records).
    `rects` = (x0, x1, r0, r1) of the same splats from the oracle."""
    F = np.float32
    qa, qb, qc = rec["qa"].astype(F), rec["qb"].astype(F), rec["qc"].astype(F)
    cx, cy = rec["center"][:, 0].astype(F), rec["center"][:, 1].astype(F)
    thr = (F(2.0) * rec["mid"].astype(F)).astype(F)
    x0, x1, r0, r1 = (np.asarray(a, np.int64).copy() for a in rects)
    with np.errstate(all="ignore"):
        empty = ~(thr <= F(0.0))
        d4 = (F(4.0) * qa) * qc
        disc = d4 - qb * qb
        ok = ~empty & (qa < F(0.0)) & (qc < F(0.0)) & (disc > F(1e-2) * d4)
        s4 = (F(4.0) * thr) / disc
        hx = np.sqrt(qc * s4) * F(1.002) + F(0.01)
        hy = np.sqrt(qa * s4) * F(1.002) + F(0.01)
        ok &= (hx < F(65536.0)) & (hy < F(65536.0))
        bx0 = np.ceil((cx - hx) - F(0.5)); bx1 = np.floor((cx + hx) - F(0.5))
        bj0 = np.ceil((cy - hy) - F(0.5)); bj1 = np.floor((cy + hy) - F(0.5))
    bx0 = np.where(ok, bx0, 0).astype(np.int64); bx1 = np.where(ok, bx1, 0).astype(np.int64)
    bj0 = np.where(ok, bj0, 0).astype(np.int64); bj1 = np.where(ok, bj1, 0).astype(np.int64)
    x0 = np.where(ok, np.maximum(x0, bx0), x0); x1 = np.where(ok, np.minimum(x1, bx1), x1)
    r0 = np.where(ok, np.maximum(r0, (height - 1) - bj1), r0); r1 = np.where(ok, np.minimum(r1, (height - 1) - bj0), r1)
    x0 = np.where(empty, 1, x0); x1 = np.where(empty, 0, x1)
    return x0, x1, r0, r1


def narrowed_rects(res, vs, U):
    """Per-Gaussian covered rectangles as the GPU bins them (kFragGauss):
    the oracle's quad narrowed by the alpha box, indexed by Gaussian id.
    Needs res from gpu_frame(..., with_debug=True)."""
    vis_desc = np.nonzero(vs["visible"])[0][::-1]
    rec = decode_records(res["records"])
    rects = O.splat_rects(vs, U)
    x0, x1, r0, r1 = alpha_box_rects(rec, tuple(a[vis_desc] for a in rects), U["height"])
    out = [a.astype(np.int64).copy() for a in rects]
    for dst, v in zip(out, (x0, x1, r0, r1)):
        dst[vis_desc] = v
    return tuple(out)


def tile_lists_for(vs, U, rects, tile=16):
    """O.tile_lists with the given per-Gaussian rectangles (front-to-back)."""
    W, H = U["width"], U["height"]
    tx_n, ty_n = (W + tile - 1) // tile, (H + tile - 1) // tile
    x0, x1, r0, r1 = rects[:4]
    order = O.sort_back_to_front(vs["view_z"], vs["visible"])[::-1]
    lists = [[] for _ in range(tx_n * ty_n)]
    for g in order:
        if x0[g] > x1[g] or r0[g] > r1[g]:
            continue
        for ty in range(r0[g] // tile, r1[g] // tile + 1):
            for tx in range(x0[g] // tile, x1[g] // tile + 1):
                lists[ty * tx_n + tx].append(int(g))
    return lists


def kept_fragments(vs, U, g, xs, rows):
    """Oracle fragment keep mask (gau_frag.glsl discards) of Gaussian g over
    pixel columns xs x image rows `rows`, ignoring the quad's coverage."""
    F = np.float32
    H = U["height"]
    px = np.asarray(xs).astype(F) + F(0.5)
    pyw = (F(H - 1) - np.asarray(rows).astype(F)) + F(0.5)
    dx = (px - vs["center"][g, 0]) * vs["coord_scale"][g, 0]
    dy = (pyw - vs["center"][g, 1]) * vs["coord_scale"][g, 1]
    DX, DY = np.meshgrid(dx.astype(F), dy.astype(F))
    _, _, keep = O.fragment(vs, g, DX, DY, U["render_mod"])
    return keep
