"""TEST INFRASTRUCTURE ONLY -- not part of the product.

CPU (NumPy, float32) restatement of the reference's OpenGL splat path, used as
the parity oracle for the HIP rasterizer in ``gsviewer_amd``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker.  The product path never calls it.

What it restates (all citations into the read-only reference snapshot):

* vertex stage  -- ``shaders/gau_vert.glsl:75-331`` (computeCov3D :75-95,
  computeCov2D :97-122, quatMultiply :134-141, rotateLightDirection :146-170,
  isInsideRotatedCube :172-191, main :193-331);
* fragment stage -- ``shaders/gau_frag.glsl:14-53``;
* GL fixed function -- instanced quads drawn in ``gi`` order
  (``render/renderer_ogl.py:406-412``), blend ``SRC_ALPHA,
  ONE_MINUS_SRC_ALPHA`` (``renderer_ogl.py:178-180``) into an RGBA8 target
  cleared to (0,0,0,1) (``main.py:197-198``);
* depth sort -- ``render/renderer_ogl.py:16-26`` (ascending view z).

Parity pinning: the reference has no tests and no golden images.  Its GLSL is
run on Mesa's llvmpipe in the build container (``oracle/gl_ref/llvmpipe_gl.c``,
``tests/golden/make_gl_golden.py``): the framebuffers it produces pin both
blend modes of this restatement (``tests/test_oracle_gl_golden.py``).  The parts
of the path that are plain NumPy in the reference (``GaussianData.flat``,
``_sort_gaussian_cpu``, ``scale_data``, ``naive_gaussian``,
``convert_euler_angles_to_rotation_matrix``) are pinned by golden vectors made
by importing the reference (``tests/golden/make_golden.py``).  The shader
arithmetic is restated line by line and checked against the llvmpipe frames
-- see DESIGN.md section "(c) Oracle and parity".

Implementation-defined GL details are fixed here (and mirrored exactly by the
HIP kernels) as follows:

* float32 everywhere, left-to-right evaluation, no fused multiply-add;
* a pixel (window column i, window row j, origin bottom-left) is covered by a
  splat's quad iff ``L_x <= 256 i < H_x`` and ``L_y <= 256 j < H_y`` where
  ``L = rint((lo - 0.5) * 256)``, ``H = rint((hi - 0.5) * 256)`` (float32
  subtraction, round half to even) and lo/hi are the quad's window-space
  corners: vertices snapped to 8 sub-pixel bits, then the top-left fill rule
  of an axis-aligned rectangle.  This is llvmpipe's rasteriser (Mesa's
  FIXED_ORDER 8, pixel centres at +0.5); 8 sub-pixel bits is also what
  desktop GPUs use;
* ``gl8`` blending is the RGBA8 framebuffer's fixed-point arithmetic as Mesa
  llvmpipe performs it: the fragment colour and alpha are converted to unorm8
  (``rint(fl32(v * 255/256) * 256)``), then
  ``dst = min(255, mul8(src, a) + mul8(dst, 255 - a))`` with llvmpipe's
  approximation of x y / 255, ``mul8(x, y) = (t + (t >> 8) + 128) >> 8``,
  ``t = x y`` (not exactly rounded: 24 of the 65536 pairs differ);
* ``coordxy`` at a pixel centre is the affine interpolation of the
  per-vertex values ``position*quadwh_scr`` (all four vertices have w = 1);
* primitives with ``|ndc.z| > 1`` are clipped away entirely (all four
  vertices share z); NaN positions are culled.
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32

# gau_vert.glsl:3-18
SH_C0 = F(0.28209479177387814)
SH_C1 = F(0.4886025119029199)
SH_C2 = [F(1.0925484305920792), F(-1.0925484305920792), F(0.31539156525252005),
         F(-1.0925484305920792), F(0.5462742152960396)]
SH_C3 = [F(-0.5900435899266435), F(2.890611442640554), F(-0.4570457994644658),
         F(0.3731763325901154), F(-0.4570457994644658), F(1.445305721320277),
         F(-0.5900435899266435)]

POS_IDX, ROT_IDX, SCALE_IDX, OPACITY_IDX, SH_IDX = 0, 3, 7, 10, 11  # gau_vert.glsl:28-32

TILE = 16


# ----------------------------------------------------------------------------
# uniforms
# ----------------------------------------------------------------------------
def default_uniforms(view, proj, hfovxy_focal, cam_pos, width, height, **kw):
    """Uniform state after the reference's start-up sequence.

    ``main.py:128-137`` + ``renderer_ogl.py:183-187`` + GL zero-init
    (SURVEY.md Appendix A.2).  ``view``/``proj`` are the math (row-major)
    matrices, i.e. what GLSL sees after ``util.set_uniform_mat4``'s transpose
    and column-major upload (``util.py:364-375``).
    """
    u = dict(
        view=np.asarray(view, F).reshape(4, 4),
        proj=np.asarray(proj, F).reshape(4, 4),
        hfovxy_focal=np.asarray(hfovxy_focal, F).reshape(3),
        cam_pos=np.asarray(cam_pos, F).reshape(3),
        width=int(width), height=int(height),
        gaussian_scale_factor=F(1.0),
        screen_display_scale_factor=F(1.0),
        dc_factor=F(1.0), extra_factor=F(1.0),
        color_scale_factors=np.ones(3, F),
        render_mod=6,
        rot_modifier=np.array([0, 0, 0, 1], F),      # (x, y, z, w) uniform order
        light_rotation=np.zeros(3, F),               # degrees
        points_center=np.zeros(3, F),
        enable_aabb=0, enable_obb=0,
        cube_rotation=np.eye(3, dtype=F),
        cubeMin=np.zeros(3, F), cubeMax=np.zeros(3, F),
        bg=np.zeros(3, F),
    )
    for k, v in kw.items():
        if k not in u:
            raise KeyError(k)
        u[k] = v
    return u


def _mv4(M, x, y, z, w):
    """M @ (x,y,z,w) row by row, left-to-right, no FMA."""
    return [((M[i, 0] * x + M[i, 1] * y) + M[i, 2] * z) + M[i, 3] * w for i in range(4)]


def _mv3(M, x, y, z):
    return [(M[i, 0] * x + M[i, 1] * y) + M[i, 2] * z for i in range(3)]


def light_rotation_cs(light_rotation_deg):
    """radians() + cos/sin of ``rotateLightDirection`` (gau_vert.glsl:148-166),
    evaluated once per frame in float32 (the values are uniform)."""
    rad = np.asarray(light_rotation_deg, F) * F(math.pi / 180.0)
    return np.cos(rad).astype(F), np.sin(rad).astype(F)


def obb_inverse(cube_rotation):
    """``inverse(rotation)`` of isInsideRotatedCube (gau_vert.glsl:180),
    evaluated once per frame (the matrix is uniform)."""
    return np.linalg.inv(np.asarray(cube_rotation, np.float64)).astype(F)


# ----------------------------------------------------------------------------
# vertex stage (gau_vert.glsl)
# ----------------------------------------------------------------------------
def vertex_stage(flat, sh_dim, U):
    """Per-Gaussian vertex-shader outputs for a ``GaussianData.flat()`` buffer.

    Returns a dict of float32/bool arrays indexed by Gaussian id.
    """
    flat = np.asarray(flat, F)
    n = flat.shape[0]
    assert flat.shape[1] == 11 + sh_dim
    with np.errstate(all="ignore"):
        x, y, z = flat[:, 0], flat[:, 1], flat[:, 2]
        V, P = U["view"], U["proj"]

        # isInsideRotatedCube (gau_vert.glsl:172-191, called at :201)
        c = U["points_center"]
        inside = np.ones(n, bool)
        if U["enable_obb"] == 1:
            Minv = obb_inverse(U["cube_rotation"])
            t = _mv3(Minv, x - c[0], y - c[1], z - c[2])
            inside = np.ones(n, bool)
            for k in range(3):
                inside &= (t[k] >= U["cubeMin"][k]) & (t[k] <= U["cubeMax"][k])
        elif U["enable_aabb"] == 1:
            t = [x - c[0], y - c[1], z - c[2]]
            for k in range(3):
                inside &= (t[k] >= c[k] + U["cubeMin"][k]) & (t[k] <= c[k] + U["cubeMax"][k])

        # view / projection / NDC (gau_vert.glsl:209-218)
        pv = _mv4(V, x, y, z, F(1.0))
        pc = _mv4(P, pv[0], pv[1], pv[2], pv[3])
        ndc = [pc[k] / pc[3] for k in range(3)]
        lim = F(1.3)
        vis = inside & (np.abs(ndc[0]) <= lim) & (np.abs(ndc[1]) <= lim) & (np.abs(ndc[2]) <= lim)
        # GL clip volume -w <= z <= w with w == 1 (whole quad shares z)
        vis &= (ndc[2] >= F(-1.0)) & (ndc[2] <= F(1.0))

        # computeCov3D(g_scale * gaussian_scale_factor, quatMultiply(g_rot, rot_modifier))
        q1 = flat[:, 3:7]
        q2 = U["rot_modifier"]
        q1x, q1y, q1z, q1w = q1[:, 0], q1[:, 1], q1[:, 2], q1[:, 3]
        q2x, q2y, q2z, q2w = q2[0], q2[1], q2[2], q2[3]
        # quatMultiply (gau_vert.glsl:134-141), (x,y,z,w) convention
        qx = ((q1w * q2x + q1x * q2w) + q1y * q2z) - q1z * q2y
        qy = ((q1w * q2y - q1x * q2z) + q1y * q2w) + q1z * q2x
        qz = ((q1w * q2z + q1x * q2y) - q1y * q2x) + q1z * q2w
        qw = ((q1w * q2w - q1x * q2x) - q1y * q2y) - q1z * q2z
        gsf = U["gaussian_scale_factor"]
        s = [flat[:, 7] * gsf, flat[:, 8] * gsf, flat[:, 9] * gsf]
        Sig = cov3d(s, qx, qy, qz, qw)

        # computeCov2D (gau_vert.glsl:97-122)
        hf = U["hfovxy_focal"]
        a, b, cc = cov2d(pv, hf[2], hf[2], hf[0], hf[1], Sig, V)
        det = a * cc - b * b
        det_inv = F(1.0) / det
        conic = np.stack([cc * det_inv, -b * det_inv, a * det_inv], 1)

        # quad (gau_vert.glsl:225, 242-245)
        wh = [(F(2.0) * hf[0]) * hf[2], (F(2.0) * hf[1]) * hf[2]]
        qs = [F(3.0) * np.sqrt(a), F(3.0) * np.sqrt(cc)]
        qn = [qs[0] / wh[0] * F(2.0), qs[1] / wh[1] * F(2.0)]
        sdsf = U["screen_display_scale_factor"]
        Wf, Hf = F(U["width"]), F(U["height"])
        half = [Wf * F(0.5), Hf * F(0.5)]
        lo, hi, cw, sc = [], [], [], []
        for k in range(2):
            off = qn[k] * sdsf
            # vertex NDC ndc +/- off, then viewport transform x_w = x_ndc*W/2 + W/2
            lo_k = (ndc[k] + (-off)) * half[k] + half[k]
            hi_k = (ndc[k] + off) * half[k] + half[k]
            c_k = ndc[k] * half[k] + half[k]
            lo.append(lo_k); hi.append(hi_k); cw.append(c_k)
            # coordxy = affine interpolation of -qs .. +qs over [lo, hi]
            sc.append(qs[k] / ((hi_k - lo_k) * F(0.5)))

        color = vertex_color(flat, sh_dim, U, x, y, z, pv)

    return dict(
        visible=vis, view_z=pv[2].astype(F), ndc=np.stack(ndc, 1).astype(F),
        cov2d=np.stack([a, b, cc], 1).astype(F), conic=conic.astype(F),
        quadwh_scr=np.stack(qs, 1).astype(F), lo=np.stack(lo, 1).astype(F),
        hi=np.stack(hi, 1).astype(F), center=np.stack(cw, 1).astype(F),
        coord_scale=np.stack(sc, 1).astype(F), color=color.astype(F),
        opacity=flat[:, OPACITY_IDX].astype(F),
        normal_color=normal_color(flat, U),
    )


def cov3d(s, qx, qy, qz, qw):
    """computeCov3D (gau_vert.glsl:75-95).  The quaternion is read as
    (r,x,y,z) = (q.x,q.y,q.z,q.w); ``R`` is built column-major, M = S*R,
    Sigma = M^T M.  Returns the 6 unique entries (00,01,02,11,12,22)."""
    r, x, y, z = qx, qy, qz, qw
    two, one = F(2.0), F(1.0)
    # Rg[row][col] as the GLSL mat3 constructor fills columns
    R = [[one - two * (y * y + z * z), two * (x * y + r * z), two * (x * z - r * y)],
         [two * (x * y - r * z), one - two * (x * x + z * z), two * (y * z + r * x)],
         [two * (x * z + r * y), two * (y * z - r * x), one - two * (x * x + y * y)]]
    M = [[s[i] * R[i][j] for j in range(3)] for i in range(3)]
    Sg = {}
    for i in range(3):
        for j in range(i, 3):
            Sg[(i, j)] = (M[0][i] * M[0][j] + M[1][i] * M[1][j]) + M[2][i] * M[2][j]
    return Sg


def cov2d(pv, fx, fy, tanx, tany, Sg, V):
    """computeCov2D (gau_vert.glsl:97-122): EWA with clamped t, T = W*J,
    cov = T^T Sigma T (top-left 2x2) + 0.3 I."""
    tx, ty, tz = pv[0], pv[1], pv[2]
    limx = F(1.3) * tanx
    limy = F(1.3) * tany
    txtz = tx / tz
    tytz = ty / tz
    tx = np.minimum(limx, np.maximum(-limx, txtz)) * tz
    ty = np.minimum(limy, np.maximum(-limy, tytz)) * tz
    tz2 = tz * tz
    # columns of Jg (GLSL mat3 constructor fills columns): j0, j1; column 2 is 0
    j0 = [fx / tz, np.zeros_like(tz), -(fx * tx) / tz2]
    j1 = [np.zeros_like(tz), fy / tz, -(fy * ty) / tz2]
    # T = W * Jg, W = transpose(mat3(V))  ->  T[:,c] = V3^T jc
    u = [(V[0, i] * j0[0] + V[1, i] * j0[1]) + V[2, i] * j0[2] for i in range(3)]
    v = [(V[0, i] * j1[0] + V[1, i] * j1[1]) + V[2, i] * j1[2] for i in range(3)]

    def S(i, j):
        return Sg[(min(i, j), max(i, j))]

    Su = [(S(i, 0) * u[0] + S(i, 1) * u[1]) + S(i, 2) * u[2] for i in range(3)]
    a = (u[0] * Su[0] + u[1] * Su[1]) + u[2] * Su[2]
    b = (v[0] * Su[0] + v[1] * Su[1]) + v[2] * Su[2]
    Sv = [(S(i, 0) * v[0] + S(i, 1) * v[1]) + S(i, 2) * v[2] for i in range(3)]
    c = (v[0] * Sv[0] + v[1] * Sv[1]) + v[2] * Sv[2]
    return a + F(0.3), b, c + F(0.3)


def _normalize(vx, vy, vz):
    n = np.sqrt((vx * vx + vy * vy) + vz * vz)
    return vx / n, vy / n, vz / n


def normal_color(flat, U):
    """0.5*(normalize(cam_pos - pos)+1) -- gau_vert.glsl:262-271 and the
    billboard-normal fragment path gau_frag.glsl:23-27 (which normalises the
    already-normalised varying once more)."""
    cp = U["cam_pos"]
    with np.errstate(all="ignore"):
        nx, ny, nz = _normalize(cp[0] - flat[:, 0], cp[1] - flat[:, 1], cp[2] - flat[:, 2])
        n2 = _normalize(nx, ny, nz)
        h = F(0.5)
        out_v = np.stack([h * (nx + F(1.0)), h * (ny + F(1.0)), h * (nz + F(1.0))], 1)
        out_f = np.stack([h * (n2[0] + F(1.0)), h * (n2[1] + F(1.0)), h * (n2[2] + F(1.0))], 1)
    return dict(vertex=out_v.astype(F), fragment=out_f.astype(F))


def vertex_color(flat, sh_dim, U, x, y, z, pv):
    """Colour varying (gau_vert.glsl:251-330)."""
    n = flat.shape[0]
    mode = U["render_mod"]
    if mode == -3:  # depth (gau_vert.glsl:252-259)
        d = -pv[2]
        d = np.where(d < F(0.05), F(1.0), d)
        d = F(1.0) / d
        return np.stack([d, d, d], 1)
    if mode == -2:  # normal (gau_vert.glsl:265-272)
        return normal_color(flat, U)["vertex"]
    cp = U["cam_pos"]
    dx, dy, dz = _normalize(x - cp[0], y - cp[1], z - cp[2])
    # rotateLightDirection (gau_vert.glsl:146-170)
    cs, sn = light_rotation_cs(U["light_rotation"])
    ry = dy * cs[0] - dz * sn[0]
    rz = dy * sn[0] + dz * cs[0]
    dy, dz = ry, rz
    rx = dx * cs[1] + dz * sn[1]
    rz = -dx * sn[1] + dz * cs[1]
    dx, dz = rx, rz
    rx = dx * cs[2] - dy * sn[2]
    ry = dx * sn[2] + dy * cs[2]
    dx, dy = rx, ry

    sh = flat[:, SH_IDX:SH_IDX + sh_dim]

    def g(k):
        return sh[:, 3 * k:3 * k + 3]

    col = SH_C0 * g(0)
    if sh_dim > 3 and mode >= 1:
        X, Y, Z = dx[:, None], dy[:, None], dz[:, None]
        col = ((col - SH_C1 * Y * g(1)) + SH_C1 * Z * g(2)) - SH_C1 * X * g(3)
        col = col * U["dc_factor"]
        if sh_dim > 12 and mode >= 2:
            xx, yy, zz = X * X, Y * Y, Z * Z
            xy, yz, xz = X * Y, Y * Z, X * Z
            col = ((((col + SH_C2[0] * xy * g(4)) + SH_C2[1] * yz * g(5))
                    + SH_C2[2] * (F(2.0) * zz - xx - yy) * g(6))
                   + SH_C2[3] * xz * g(7)) + SH_C2[4] * (xx - yy) * g(8)
            if sh_dim > 27 and mode >= 3:
                col = ((((((col + SH_C3[0] * Y * (F(3.0) * xx - yy) * g(9))
                           + SH_C3[1] * xy * Z * g(10))
                          + SH_C3[2] * Y * (F(4.0) * zz - xx - yy) * g(11))
                         + SH_C3[3] * Z * (F(2.0) * zz - F(3.0) * xx - F(3.0) * yy) * g(12))
                        + SH_C3[4] * X * (F(4.0) * zz - xx - yy) * g(13))
                       + SH_C3[5] * Z * (xx - yy) * g(14)) + SH_C3[6] * X * (xx - F(3.0) * yy) * g(15)
            col = col * U["extra_factor"]
    col = col + F(0.5)
    col = col * U["color_scale_factors"]
    return col.astype(F).reshape(n, 3)


# ----------------------------------------------------------------------------
# sort (renderer_ogl.py:16-26)
# ----------------------------------------------------------------------------
def sort_back_to_front(view_z, visible=None):
    """Ascending view z == back-to-front (``_sort_gaussian_cpu``).  Stable, so
    exact ties keep ascending Gaussian index (the reference's default argsort
    leaves ties unordered; fixtures avoid them)."""
    order = np.argsort(view_z, kind="stable")
    if visible is not None:
        order = order[visible[order]]
    return order


# ----------------------------------------------------------------------------
# coverage
# ----------------------------------------------------------------------------
def snap8(v):
    """Window coordinate -> fixed point with 8 sub-pixel bits in the frame whose
    pixel centres are integers (llvmpipe ``subpixel_snap(v - 0.5)``): float32
    subtraction, exact scaling, round half to even.  float64 result (exact)."""
    v = np.clip(np.asarray(v, F), F(-1048576.0), F(1048576.0))
    return np.rint((v - F(0.5)) * F(256.0)).astype(np.float64)


def pixel_span(lo, hi, limit):
    """Integer pixel index range [p0, p1] covered by the quad edges lo, hi:
    ``snap8(lo) <= 256 p < snap8(hi)``, clamped to [-1, limit]."""
    lo = np.asarray(lo, F)
    hi = np.asarray(hi, F)
    with np.errstate(invalid="ignore"):
        p0 = np.ceil(snap8(lo) / 256.0)
        p1 = np.ceil(snap8(hi) / 256.0) - 1.0
    p0 = np.where(np.isnan(lo) | np.isnan(hi), limit, p0)
    p1 = np.where(np.isnan(lo) | np.isnan(hi), -1, p1)
    return np.clip(p0, -1, limit).astype(np.int64), np.clip(p1, -1, limit).astype(np.int64)


def splat_rects(vs, U):
    """Per-Gaussian covered pixel rectangle in IMAGE coordinates (row 0 = top):
    (x0, x1, r0, r1), inclusive; empty if x0 > x1 or r0 > r1."""
    W, H = U["width"], U["height"]
    x0, x1 = pixel_span(vs["lo"][:, 0], vs["hi"][:, 0], W)
    j0, j1 = pixel_span(vs["lo"][:, 1], vs["hi"][:, 1], H)   # window rows
    x0, x1 = np.maximum(x0, 0), np.minimum(x1, W - 1)
    j0, j1 = np.maximum(j0, 0), np.minimum(j1, H - 1)
    r0, r1 = (H - 1) - j1, (H - 1) - j0
    return x0, x1, r0, r1


def tile_lists(vs, U, tile=TILE):
    """Per 16x16 tile: visible Gaussian ids covering >=1 pixel of the tile, in
    FRONT-TO-BACK order (the reverse of the GL draw order restricted to the
    tile)."""
    W, H = U["width"], U["height"]
    tx_n, ty_n = (W + tile - 1) // tile, (H + tile - 1) // tile
    x0, x1, r0, r1 = splat_rects(vs, U)
    order = sort_back_to_front(vs["view_z"], vs["visible"])[::-1]
    lists = [[] for _ in range(tx_n * ty_n)]
    for g in order:
        if x0[g] > x1[g] or r0[g] > r1[g]:
            continue
        for ty in range(r0[g] // tile, r1[g] // tile + 1):
            for tx in range(x0[g] // tile, x1[g] // tile + 1):
                lists[ty * tx_n + tx].append(int(g))
    return lists


# ----------------------------------------------------------------------------
# fragment stage + blend (gau_frag.glsl, GL blend)
# ----------------------------------------------------------------------------
def fragment(vs, g, dx, dy, mode):
    """gau_frag.glsl:14-53 for Gaussian ``g`` at pixel offsets dx, dy (arrays).
    Returns (rgb [..,3], alpha [..], keep mask)."""
    col = vs["color"][g]
    if mode == -4:  # billboard
        a = np.ones(dx.shape, F)
        return np.broadcast_to(col, dx.shape + (3,)), a, np.ones(dx.shape, bool)
    if mode == -1:  # billboard normal
        a = np.ones(dx.shape, F)
        return np.broadcast_to(vs["normal_color"]["fragment"][g], dx.shape + (3,)), a, np.ones(dx.shape, bool)
    A, B, C = vs["conic"][g]
    with np.errstate(all="ignore"):
        power = F(-0.5) * (A * dx * dx + C * dy * dy) - B * dx * dy
        e = np.exp(power.astype(F)).astype(F)
        a = np.minimum(F(0.99), vs["opacity"][g] * e)
    keep = ~(power > F(0.0)) & ~(a < F(1.0) / F(255.0))
    rgb = np.broadcast_to(col, dx.shape + (3,))
    if mode == -5:
        a = np.where(a > F(0.22), F(1.0), F(0.0)).astype(F)
    elif mode == -6:
        a = np.where(a > F(0.22), F(1.0), F(0.0)).astype(F)
        rgb = rgb * e[..., None]
    return rgb, a.astype(F), keep


def to_unorm8(v):
    """float -> unorm8 as llvmpipe converts a fragment output for an RGBA8
    target (lp_build_clamped_float_to_unsigned_norm: x * 255/256 in float32,
    then the 1/256 grid, round half to even)."""
    t = (np.clip(np.asarray(v, F), F(0.0), F(1.0)) * F(255.0 / 256.0)).astype(F)
    return np.rint(t.astype(np.float64) * 256.0).astype(np.int32)


def mul8(x, y):
    """llvmpipe's approximation of x*y/255 for two unorm8 values (Blinn's
    form, lp_build_mul_norm): not exactly rounded, it differs from
    round(x*y/255) on 24 of the 65536 pairs; the llvmpipe goldens pin it."""
    t = x * y
    return (t + (t >> 8) + 128) >> 8


def blend8(src8, a8, dst8):
    """SRC_ALPHA, ONE_MINUS_SRC_ALPHA on an RGBA8 target, integer form."""
    return np.minimum(255, mul8(src8, a8) + mul8(dst8, 255 - a8))


def composite(vs, U, mode="float", order=None):
    """Instanced-draw + blend restatement.  ``mode='float'`` blends in float32
    (SURVEY Appendix A.5 mode (a)); ``mode='gl8'`` is the RGBA8 framebuffer
    (mode (b)), every blend in unorm8 fixed point (``blend8``).  Returns the RGB
    image [H, W, 3] float32 with row 0 = TOP (as ``Save Image`` writes it,
    gs_elements_control.py:192-196, and as the CUDA boundary returns it); in
    gl8 mode the values are k / 255."""
    W, H = U["width"], U["height"]
    rm = U["render_mod"]
    if mode == "gl8":
        img = np.broadcast_to(to_unorm8(U["bg"]), (H, W, 3)).astype(np.int32).copy()
    else:
        img = np.broadcast_to(U["bg"].astype(F), (H, W, 3)).copy()
    if order is None:
        order = sort_back_to_front(vs["view_z"], vs["visible"])
    x0, x1, r0, r1 = splat_rects(vs, U)
    for g in order:
        if x0[g] > x1[g] or r0[g] > r1[g]:
            continue
        xs = np.arange(x0[g], x1[g] + 1)
        rs = np.arange(r0[g], r1[g] + 1)
        px = xs.astype(F) + F(0.5)
        pyw = (F(H - 1) - rs.astype(F)) + F(0.5)
        dx = (px - vs["center"][g, 0]) * vs["coord_scale"][g, 0]
        dy = (pyw - vs["center"][g, 1]) * vs["coord_scale"][g, 1]
        DX, DY = np.meshgrid(dx.astype(F), dy.astype(F))
        rgb, a, keep = fragment(vs, g, DX, DY, rm)
        rgb = np.clip(rgb, F(0.0), F(1.0)).astype(F)   # unorm colour target
        a = np.clip(a, F(0.0), F(1.0)).astype(F)
        dst = img[r0[g]:r1[g] + 1, x0[g]:x1[g] + 1]
        if mode == "gl8":
            new = blend8(to_unorm8(rgb), to_unorm8(a)[..., None], dst)
        else:
            new = (rgb * a[..., None] + dst * (F(1.0) - a)[..., None]).astype(F)
        img[r0[g]:r1[g] + 1, x0[g]:x1[g] + 1] = np.where(keep[..., None], new, dst)
    if mode == "gl8":
        return (img.astype(F) / F(255.0)).astype(F)
    return img.astype(F)


def radii(vs):
    """Per-Gaussian integer radius returned next to the image: 0 if culled,
    else ceil(max(3*sqrt(cov.x), 3*sqrt(cov.z))) (the quad half-extents of
    gau_vert.glsl:242)."""
    q = vs["quadwh_scr"].astype(np.float64)
    r = np.ceil(np.maximum(q[:, 0], q[:, 1]))
    r = np.where(vs["visible"] & np.isfinite(r), r, 0)
    return r.astype(np.int32)


def render(flat, sh_dim, U, mode="float"):
    vs = vertex_stage(flat, sh_dim, U)
    return composite(vs, U, mode=mode), vs
