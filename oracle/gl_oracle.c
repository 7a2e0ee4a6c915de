/*
 * TEST INFRASTRUCTURE ONLY -- not part of the product.
 *
 * C restatement of the reference's OpenGL splat path, identical in arithmetic
 * to oracle/gl_oracle.py (float32, left-to-right, compiled with
 * -ffp-contract=off), used (a) as the parity oracle at sizes where the NumPy
 * restatement is too slow and (b) as bench.py's timed CPU baseline
 * ("kind": "port").  It follows, step by step:
 *   depth sort            render/renderer_ogl.py:16-26 (ascending view z; parallel radix)
 *   vertex stage          shaders/gau_vert.glsl:75-331
 *   rasterisation         GL quad coverage at pixel centres, 8 sub-pixel bits (oracle/gl_oracle.py header)
 *   fragment stage        shaders/gau_frag.glsl:14-53
 *   blending              SRC_ALPHA, ONE_MINUS_SRC_ALPHA in draw order (renderer_ogl.py:178-180);
 *                         gl8: the RGBA8 target's unorm8 arithmetic as Mesa llvmpipe does it
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    float view[16], proj[16], hfov[3], campos[3];
    int32_t width, height;
    float gsf, sdsf, dc_factor, extra_factor, cscale[3];
    int32_t render_mod;
    float rotmod[4], lcos[3], lsin[3], pcenter[3];
    int32_t enable_aabb, enable_obb;
    float obb_inv[9], cmin[3], cmax[3], bg[3];
} oracle_uniforms;

typedef struct {
    float view_z, cx, cy, sx, sy, A, B, C, opacity, r, g, b, nr, ng, nb;
    int32_t visible, x0, x1, r0, r1;
} vtx_out;

static const float SH_C0 = 0.28209479177387814f, SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* GL coverage with 8 sub-pixel bits (oracle/gl_oracle.py pixel_span/snap8):
 * snap(v) = rint((v - 0.5) * 256) in float32, pixel p covered iff
 * snap(lo) <= 256 p < snap(hi). */
static double snap8(float v) {
    if (v < -1048576.0f) v = -1048576.0f;
    if (v > 1048576.0f) v = 1048576.0f;
    return (double)rintf((v - 0.5f) * 256.0f);
}

static void span(float lo, float hi, int limit, int* p0, int* p1) {
    if (!(lo == lo) || !(hi == hi)) { *p0 = limit; *p1 = -1; return; }
    double a = ceil(snap8(lo) / 256.0), b = ceil(snap8(hi) / 256.0) - 1.0;
    if (a < -1) a = -1;
    if (a > limit) a = limit;
    if (b < -1) b = -1;
    if (b > limit) b = limit;
    *p0 = (int)a; *p1 = (int)b;
}

static void normalize3(float* v) {
    float n = sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    v[0] = v[0] / n; v[1] = v[1] / n; v[2] = v[2] / n;
}

static void vertex(const float* f, int sh_dim, const oracle_uniforms* u, vtx_out* o) {
    const float x = f[0], y = f[1], z = f[2];
    const float* V = u->view;
    const float* P = u->proj;
    float pv[4], pc[4], ndc[3];
    for (int i = 0; i < 4; ++i) pv[i] = ((V[4 * i] * x + V[4 * i + 1] * y) + V[4 * i + 2] * z) + V[4 * i + 3] * 1.0f;
    for (int i = 0; i < 4; ++i)
        pc[i] = ((P[4 * i] * pv[0] + P[4 * i + 1] * pv[1]) + P[4 * i + 2] * pv[2]) + P[4 * i + 3] * pv[3];
    for (int k = 0; k < 3; ++k) ndc[k] = pc[k] / pc[3];
    o->view_z = pv[2];
    int inside = 1;
    if (u->enable_obb == 1) {
        const float dx = x - u->pcenter[0], dy = y - u->pcenter[1], dz = z - u->pcenter[2];
        const float* M = u->obb_inv;
        float t[3];
        for (int k = 0; k < 3; ++k) t[k] = (M[3 * k] * dx + M[3 * k + 1] * dy) + M[3 * k + 2] * dz;
        for (int k = 0; k < 3; ++k) inside &= (t[k] >= u->cmin[k]) & (t[k] <= u->cmax[k]);
    } else if (u->enable_aabb == 1) {
        const float t[3] = {x - u->pcenter[0], y - u->pcenter[1], z - u->pcenter[2]};
        for (int k = 0; k < 3; ++k)
            inside &= (t[k] >= u->pcenter[k] + u->cmin[k]) & (t[k] <= u->pcenter[k] + u->cmax[k]);
    }
    const float lim = 1.3f;
    o->visible = inside && fabsf(ndc[0]) <= lim && fabsf(ndc[1]) <= lim && fabsf(ndc[2]) <= lim &&
                 ndc[2] >= -1.0f && ndc[2] <= 1.0f;
    if (!o->visible) return;

    /* quatMultiply + computeCov3D */
    const float q1x = f[3], q1y = f[4], q1z = f[5], q1w = f[6];
    const float q2x = u->rotmod[0], q2y = u->rotmod[1], q2z = u->rotmod[2], q2w = u->rotmod[3];
    const float r = ((q1w * q2x + q1x * q2w) + q1y * q2z) - q1z * q2y;
    const float qx = ((q1w * q2y - q1x * q2z) + q1y * q2w) + q1z * q2x;
    const float qy = ((q1w * q2z + q1x * q2y) - q1y * q2x) + q1z * q2w;
    const float qz = ((q1w * q2w - q1x * q2x) - q1y * q2y) - q1z * q2z;
    const float s[3] = {f[7] * u->gsf, f[8] * u->gsf, f[9] * u->gsf};
    const float R[3][3] = {
        {1.0f - 2.0f * (qy * qy + qz * qz), 2.0f * (qx * qy + r * qz), 2.0f * (qx * qz - r * qy)},
        {2.0f * (qx * qy - r * qz), 1.0f - 2.0f * (qx * qx + qz * qz), 2.0f * (qy * qz + r * qx)},
        {2.0f * (qx * qz + r * qy), 2.0f * (qy * qz - r * qx), 1.0f - 2.0f * (qx * qx + qy * qy)}};
    float M[3][3], S[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) M[a][b] = s[a] * R[a][b];
    for (int a = 0; a < 3; ++a)
        for (int b = a; b < 3; ++b) {
            S[a][b] = (M[0][a] * M[0][b] + M[1][a] * M[1][b]) + M[2][a] * M[2][b];
            S[b][a] = S[a][b];
        }
    /* computeCov2D */
    const float fx = u->hfov[2], fy = u->hfov[2];
    float tx = pv[0], ty = pv[1];
    const float tz = pv[2];
    const float limx = 1.3f * u->hfov[0], limy = 1.3f * u->hfov[1];
    const float txtz = tx / tz, tytz = ty / tz;
    tx = fminf(limx, fmaxf(-limx, txtz)) * tz;
    ty = fminf(limy, fmaxf(-limy, tytz)) * tz;
    const float tz2 = tz * tz;
    const float j0[3] = {fx / tz, 0.0f, -(fx * tx) / tz2};
    const float j1[3] = {0.0f, fy / tz, -(fy * ty) / tz2};
    float uu[3], vv[3], Su[3], Sv[3];
    for (int k = 0; k < 3; ++k) {
        uu[k] = (V[k] * j0[0] + V[4 + k] * j0[1]) + V[8 + k] * j0[2];
        vv[k] = (V[k] * j1[0] + V[4 + k] * j1[1]) + V[8 + k] * j1[2];
    }
    for (int k = 0; k < 3; ++k) {
        Su[k] = (S[k][0] * uu[0] + S[k][1] * uu[1]) + S[k][2] * uu[2];
        Sv[k] = (S[k][0] * vv[0] + S[k][1] * vv[1]) + S[k][2] * vv[2];
    }
    const float ca = ((uu[0] * Su[0] + uu[1] * Su[1]) + uu[2] * Su[2]) + 0.3f;
    const float cb = (vv[0] * Su[0] + vv[1] * Su[1]) + vv[2] * Su[2];
    const float cc = ((vv[0] * Sv[0] + vv[1] * Sv[1]) + vv[2] * Sv[2]) + 0.3f;
    const float det = ca * cc - cb * cb;
    const float det_inv = 1.0f / det;
    o->A = cc * det_inv; o->B = -cb * det_inv; o->C = ca * det_inv;
    o->opacity = f[10];
    const float wh[2] = {(2.0f * u->hfov[0]) * u->hfov[2], (2.0f * u->hfov[1]) * u->hfov[2]};
    const float qs[2] = {3.0f * sqrtf(ca), 3.0f * sqrtf(cc)};
    const float half[2] = {(float)u->width * 0.5f, (float)u->height * 0.5f};
    float lo[2], hi[2], cw[2], sc[2];
    for (int k = 0; k < 2; ++k) {
        const float qn = qs[k] / wh[k] * 2.0f;
        const float off = qn * u->sdsf;
        lo[k] = (ndc[k] + (-off)) * half[k] + half[k];
        hi[k] = (ndc[k] + off) * half[k] + half[k];
        cw[k] = ndc[k] * half[k] + half[k];
        sc[k] = qs[k] / ((hi[k] - lo[k]) * 0.5f);
    }
    o->cx = cw[0]; o->cy = cw[1]; o->sx = sc[0]; o->sy = sc[1];
    int x0, x1, j0i, j1i;
    span(lo[0], hi[0], u->width, &x0, &x1);
    span(lo[1], hi[1], u->height, &j0i, &j1i);
    if (x0 < 0) x0 = 0;
    if (x1 > u->width - 1) x1 = u->width - 1;
    if (j0i < 0) j0i = 0;
    if (j1i > u->height - 1) j1i = u->height - 1;
    o->x0 = x0; o->x1 = x1;
    o->r0 = (u->height - 1) - j1i; o->r1 = (u->height - 1) - j0i;

    /* normal colours (vertex -2 and fragment -1 variants) */
    float nv[3] = {u->campos[0] - x, u->campos[1] - y, u->campos[2] - z};
    normalize3(nv);
    float nf[3] = {nv[0], nv[1], nv[2]};
    normalize3(nf);
    const int mode = u->render_mod;
    if (mode == -3) {
        float d = -pv[2];
        d = d < 0.05f ? 1.0f : d;
        d = 1.0f / d;
        o->r = o->g = o->b = d;
        return;
    }
    if (mode == -2) {
        o->r = 0.5f * (nv[0] + 1.0f); o->g = 0.5f * (nv[1] + 1.0f); o->b = 0.5f * (nv[2] + 1.0f);
        return;
    }
    o->nr = 0.5f * (nf[0] + 1.0f); o->ng = 0.5f * (nf[1] + 1.0f); o->nb = 0.5f * (nf[2] + 1.0f);
    float d[3] = {x - u->campos[0], y - u->campos[1], z - u->campos[2]};
    normalize3(d);
    float dx = d[0], dy = d[1], dz = d[2], t1, t2;
    t1 = dy * u->lcos[0] - dz * u->lsin[0]; t2 = dy * u->lsin[0] + dz * u->lcos[0]; dy = t1; dz = t2;
    t1 = dx * u->lcos[1] + dz * u->lsin[1]; t2 = -dx * u->lsin[1] + dz * u->lcos[1]; dx = t1; dz = t2;
    t1 = dx * u->lcos[2] - dy * u->lsin[2]; t2 = dx * u->lsin[2] + dy * u->lcos[2]; dx = t1; dy = t2;
    const float* g = f + 11;
#define G(k, c) g[3 * (k) + (c)]
    float col[3];
    for (int c = 0; c < 3; ++c) col[c] = SH_C0 * G(0, c);
    if (sh_dim > 3 && mode >= 1) {
        const float X = dx, Y = dy, Z = dz;
        for (int c = 0; c < 3; ++c) {
            col[c] = ((col[c] - (SH_C1 * Y) * G(1, c)) + (SH_C1 * Z) * G(2, c)) - (SH_C1 * X) * G(3, c);
            col[c] = col[c] * u->dc_factor;
        }
        if (sh_dim > 12 && mode >= 2) {
            const float xx = X * X, yy = Y * Y, zz = Z * Z, xy = X * Y, yz = Y * Z, xz = X * Z;
            const float k4 = SH_C2[0] * xy, k5 = SH_C2[1] * yz, k6 = SH_C2[2] * ((2.0f * zz - xx) - yy);
            const float k7 = SH_C2[3] * xz, k8 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; ++c)
                col[c] = ((((col[c] + k4 * G(4, c)) + k5 * G(5, c)) + k6 * G(6, c)) + k7 * G(7, c)) + k8 * G(8, c);
            if (sh_dim > 27 && mode >= 3) {
                const float k9 = (SH_C3[0] * Y) * (3.0f * xx - yy);
                const float k10 = (SH_C3[1] * xy) * Z;
                const float k11 = (SH_C3[2] * Y) * ((4.0f * zz - xx) - yy);
                const float k12 = (SH_C3[3] * Z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
                const float k13 = (SH_C3[4] * X) * ((4.0f * zz - xx) - yy);
                const float k14 = (SH_C3[5] * Z) * (xx - yy);
                const float k15 = (SH_C3[6] * X) * (xx - 3.0f * yy);
                for (int c = 0; c < 3; ++c)
                    col[c] = ((((((col[c] + k9 * G(9, c)) + k10 * G(10, c)) + k11 * G(11, c)) + k12 * G(12, c)) +
                               k13 * G(13, c)) + k14 * G(14, c)) + k15 * G(15, c);
            }
            for (int c = 0; c < 3; ++c) col[c] = col[c] * u->extra_factor;
        }
    }
#undef G
    o->r = (col[0] + 0.5f) * u->cscale[0];
    o->g = (col[1] + 0.5f) * u->cscale[1];
    o->b = (col[2] + 0.5f) * u->cscale[2];
}

/* ------------------------------------------------------------------ sort */
typedef struct { float z; int32_t id; } zkey;

/* Ascending (z, id) as a parallel LSD radix sort of the 64-bit words
 * (order-preserving bits of z) << 32 | id: equal z keep ascending id, the
 * order the reference's argsort gives its equal keys (tests/golden:
 * _sort_gaussian_cpu orders).  -0.0 sorts as +0.0 (the two compare equal).
 * 3 passes of 11 bits over the z bits; every thread histograms and scatters
 * its own contiguous range (OpenMP).  It replaces a qsort that ran 94 ms at
 * 1M on one thread against the reference's NumPy argsort (26 ms). */
static inline uint64_t zword(float z, int32_t id) {
    uint32_t b;
    if (z == 0.0f) z = 0.0f;
    memcpy(&b, &z, 4);
    b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    return ((uint64_t)b << 32) | (uint32_t)id;
}

#define ZR_BITS 11
#define ZR_BUCKETS (1 << ZR_BITS)

static int radix_sort_zkeys(zkey* k, int64_t m) {
    if (m <= 1) return 0;
    uint64_t* a = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m);
    uint64_t* t = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m);
    int nt = 1;
#ifdef _OPENMP
    nt = m < 262144 ? 1 : omp_get_max_threads();
#endif
    int64_t* hist = (int64_t*)malloc(sizeof(int64_t) * (size_t)nt * ZR_BUCKETS);
    if (!a || !t || !hist) { free(a); free(t); free(hist); return -1; }
    uint64_t *src = a, *dst = t;
#pragma omp parallel num_threads(nt)
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        const int64_t b = m * tid / nt, e = m * (tid + 1) / nt;
        int64_t* h = hist + (size_t)ZR_BUCKETS * tid;
        for (int64_t i = b; i < e; ++i) a[i] = zword(k[i].z, k[i].id);
        for (int pass = 0; pass < 3; ++pass) {
            const int sh = 32 + ZR_BITS * pass;
            memset(h, 0, sizeof(int64_t) * ZR_BUCKETS);
            for (int64_t i = b; i < e; ++i) h[(src[i] >> sh) & (ZR_BUCKETS - 1)]++;
#pragma omp barrier
#pragma omp single
            {
                int64_t run = 0;
                for (int d = 0; d < ZR_BUCKETS; ++d)
                    for (int u = 0; u < nt; ++u) {
                        const int64_t c = hist[(size_t)ZR_BUCKETS * u + d];
                        hist[(size_t)ZR_BUCKETS * u + d] = run;
                        run += c;
                    }
            }
            for (int64_t i = b; i < e; ++i) dst[h[(src[i] >> sh) & (ZR_BUCKETS - 1)]++] = src[i];
#pragma omp barrier
#pragma omp single
            {
                uint64_t* x = src; src = dst; dst = x;
            }
        }
        for (int64_t i = b; i < e; ++i) k[i].id = (int32_t)(uint32_t)src[i];  /* (only ids are read back) */
    }
    free(a); free(t); free(hist);
    return 0;
}

/* Back-to-front order of visible Gaussians (ascending view z, ties by id). */
static int64_t sort_visible(const vtx_out* vo, int64_t n, int32_t* order) {
    zkey* k = (zkey*)malloc(sizeof(zkey) * (size_t)(n > 0 ? n : 1));
    if (!k) return -1;
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i)
        if (vo[i].visible) { k[m].z = vo[i].view_z; k[m].id = (int32_t)i; ++m; }
    if (radix_sort_zkeys(k, m)) { free(k); return -1; }
    for (int64_t i = 0; i < m; ++i) order[i] = k[i].id;
    free(k);
    return m;
}

static inline float clamp01(float v) { return v < 0.f ? 0.f : (v > 1.f ? 1.f : v); }
/* RGBA8 target arithmetic as Mesa llvmpipe performs it (oracle/gl_oracle.py
 * to_unorm8 / mul8 / blend8). */
static inline int to_unorm8(float v) { return (int)rintf((clamp01(v) * (255.0f / 256.0f)) * 256.0f); }
static inline int mul8(int x, int y) { const int t = x * y; return (t + (t >> 8) + 128) >> 8; }
static inline int blend8(int s, int a, int d) { const int n = mul8(s, a) + mul8(d, 255 - a); return n < 255 ? n : 255; }
static inline int from_img8(float v) { return (int)(v * 255.0f + 0.5f); }

/* ------------------------------------------------------------------ entry */
/* Renders into img (H*W*3, row 0 = top).  Returns the number of visible
 * Gaussians, or -1 on allocation failure.  order_out (optional, n int32)
 * receives the back-to-front draw order; n_vis_out the count. */
int64_t oracle_render(const float* flat, int64_t n, int32_t sh_dim, const oracle_uniforms* u, int32_t gl8,
                      float* img, int32_t* order_out, int32_t threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    const int W = u->width, H = u->height;
    vtx_out* vo = (vtx_out*)malloc(sizeof(vtx_out) * (size_t)(n > 0 ? n : 1));
    int32_t* order = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    if (!vo || !order) { free(vo); free(order); return -1; }
    const int64_t rec = 11 + sh_dim;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) vertex(flat + rec * i, sh_dim, u, &vo[i]);
    const int64_t m = sort_visible(vo, n, order);
    if (m < 0) { free(vo); free(order); return -1; }
    const int mode = u->render_mod;
    const float bg[3] = {gl8 ? (float)to_unorm8(u->bg[0]) / 255.0f : u->bg[0],
                         gl8 ? (float)to_unorm8(u->bg[1]) / 255.0f : u->bg[1],
                         gl8 ? (float)to_unorm8(u->bg[2]) / 255.0f : u->bg[2]};
#pragma omp parallel
    {
        int nt = 1, t = 0;
#ifdef _OPENMP
        nt = omp_get_num_threads();
        t = omp_get_thread_num();
#endif
        const int rb = (int)((int64_t)H * t / nt), re = (int)((int64_t)H * (t + 1) / nt);
        for (int r = rb; r < re; ++r)
            for (int x = 0; x < W; ++x) {
                float* p = img + 3 * ((size_t)r * W + x);
                p[0] = bg[0]; p[1] = bg[1]; p[2] = bg[2];
            }
        for (int64_t k = 0; k < m; ++k) {
            const vtx_out* s = &vo[order[k]];
            if (s->x0 > s->x1 || s->r0 > s->r1) continue;
            const int ra = s->r0 > rb ? s->r0 : rb, rz = s->r1 < re - 1 ? s->r1 : re - 1;
            for (int r = ra; r <= rz; ++r) {
                const float pyw = ((float)(H - 1) - (float)r) + 0.5f;
                const float dy = (pyw - s->cy) * s->sy;
                for (int x = s->x0; x <= s->x1; ++x) {
                    const float dx = (((float)x + 0.5f) - s->cx) * s->sx;
                    float a, cr = s->r, cg = s->g, cb = s->b;
                    if (mode == -4 || mode == -1) {
                        a = 1.0f;
                        if (mode == -1) { cr = s->nr; cg = s->ng; cb = s->nb; }
                    } else {
                        const float power = -0.5f * (s->A * dx * dx + s->C * dy * dy) - s->B * dx * dy;
                        const float e = expf(power);
                        a = fminf(0.99f, s->opacity * e);
                        if (power > 0.0f || a < 1.0f / 255.0f) continue;
                        if (mode == -5 || mode == -6) a = a > 0.22f ? 1.0f : 0.0f;
                        if (mode == -6) { cr *= e; cg *= e; cb *= e; }
                    }
                    cr = clamp01(cr); cg = clamp01(cg); cb = clamp01(cb); a = clamp01(a);
                    float* p = img + 3 * ((size_t)r * W + x);
                    if (gl8) {  /* the framebuffer holds k / 255 */
                        const int a8 = to_unorm8(a);
                        p[0] = (float)blend8(to_unorm8(cr), a8, from_img8(p[0])) / 255.0f;
                        p[1] = (float)blend8(to_unorm8(cg), a8, from_img8(p[1])) / 255.0f;
                        p[2] = (float)blend8(to_unorm8(cb), a8, from_img8(p[2])) / 255.0f;
                    } else {
                        p[0] = cr * a + p[0] * (1.0f - a);
                        p[1] = cg * a + p[1] * (1.0f - a);
                        p[2] = cb * a + p[2] * (1.0f - a);
                    }
                }
            }
        }
    }
    if (order_out) memcpy(order_out, order, sizeof(int32_t) * (size_t)m);
    free(vo);
    free(order);
    return m;
}

/* Sort-only baseline: the reference's _sort_gaussian_cpu (dot + argsort). */
int64_t oracle_sort_depth(const float* xyz, int64_t n, const float* view, int32_t* order_out, int32_t threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    zkey* k = (zkey*)malloc(sizeof(zkey) * (size_t)(n > 0 ? n : 1));
    if (!k) return -1;
    for (int64_t i = 0; i < n; ++i) {
        const float* p = xyz + 3 * i;
        k[i].z = ((view[8] * p[0] + view[9] * p[1]) + view[10] * p[2]) + view[11];
        k[i].id = (int32_t)i;
    }
    if (radix_sort_zkeys(k, n)) { free(k); return -1; }
    for (int64_t i = 0; i < n; ++i) order_out[i] = k[i].id;
    free(k);
    return n;
}
