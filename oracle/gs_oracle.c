/*
 * gs_oracle.c -- CPU restatement of the differentiable Gaussian rasterizer (TEST INFRASTRUCTURE).
 *
 * THIS FILE IS A CHECKER, NOT PRODUCT CODE.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path (gaussian-splatting-skysphere_amd/)
 * never links, loads or calls anything under oracle/.
 *
 * What it restates
 * ----------------
 * The rasterizer behind `diff_gaussian_rasterization.GaussianRasterizer`, as called from the
 * reference's render adapter (/root/reference/gaussian_renderer/__init__.py:36-93).  The native
 * rasterizer itself is an un-vendored git submodule (/root/reference/.gitmodules:4-6,
 * graphdeco-inria/diff-gaussian-rasterization, 2023 two-output / 12-field-settings API; pinned
 * SHA unrecoverable).  Its published algorithm is restated here from the
 * spec in SURVEY.md §8a rows a4-a8.  Pieces that ARE pinned by reference code in this container:
 *   - SH -> RGB (+0.5, clamp >= 0): /root/reference/utils/sh_utils.py:57-100 and
 *     /root/reference/gaussian_renderer/__init__.py:73-78  (golden vectors in tests/golden/).
 *   - cov3D = R S S^T R^T, 6-vector (xx,xy,xz,yy,yz,zz): /root/reference/scene/gaussian_model.py:27-31,
 *     /root/reference/utils/general_utils.py:78-110                       (golden vectors).
 *   - camera conventions: /root/reference/utils/graphics_utils.py:38-71, scene/cameras.py:54-57.
 * The compositing core (render fwd/bwd) is "parity unpinned" by the reference; it is cross-checked
 * by tests against an independent dense PyTorch restatement + autograd (tests/test_oracle_*.py).
 *
 * Numerics contract (shared with the HIP kernels):
 *   - fp32 everywhere, IEEE round-to-nearest, NO contraction (build with -ffp-contract=off);
 *     every FMA is an explicit fmaf().  ndc->pixel is evaluated in double as upstream.
 *   - the Gaussian falloff is 2^t with t = log2(e) * power from a conic pre-scaled by log2(e)
 *     (falloff_log2, two FMAs) and exp2 by a degree-6 polynomial + ldexp (oracle_exp2), built
 *     only from correctly-rounded IEEE ops, so CPU and GPU agree bit-for-bit on every threshold
 *     decision (alpha < 1/255, T < 1e-4).
 *   - Operation order for every expression is fixed (left-to-right as written here).
 *   - Gradient sums over pixels / tiles are accumulated in double here (order-independent
 *     reference); the GPU sums in fp32 in its own order -> tolerance documented in tests.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define TILE 16
#define NCH 3

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* ------------------------------------------------------------------------------------------ */
/* scalar helpers                                                                              */
/* ------------------------------------------------------------------------------------------ */

static inline float f_as(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t u_as(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* 2^t for the splat falloff, t <= 0 in practice: t is clamped to [-125, 0] (below, the result
 * <= 2.4e-38 only ever meets `alpha < 1/255` or a zero weight; above 0 the caller skips; the clamp
 * keeps every result a normal float); n = rint(t), 2^(t - n) by a degree-6 minimax polynomial on
 * [-0.5, 0.5], scaled by ldexp.  Identical op sequence in csrc/gs_common.h:gs_exp2. */
float oracle_exp2(float t) {
    t = fminf(fmaxf(t, -125.0f), 0.0f);
    float n = rintf(t);
    float f = t - n;
    float p = 1.5345810970757157e-4f;
    p = fmaf(p, f, 1.3399930903688073e-3f);
    p = fmaf(p, f, 9.618489071726799e-3f);
    p = fmaf(p, f, 5.550328642129898e-2f);
    p = fmaf(p, f, 2.4022646248340607e-1f);
    p = fmaf(p, f, 6.931471824645996e-1f);
    p = fmaf(p, f, 1.0f);
    return ldexpf(p, (int)n);
}

/* exp(x) = 2^(x log2 e), t rounded to float: relative error <= 5.1e-7 on [-8, 0] */
float oracle_exp(float x) { return oracle_exp2(x * 1.44269504088896341f); }

/* log2(e) * power of a splat at pixel offset (dx, dy) = mean - pixel, with the conic scaled once
 * per splat: A = cxx (-log2e / 2), B = cxy (-log2e), C = cyy (-log2e / 2);
 * t = (A dx) dx + dy (B dx + C dy): three multiplies, two FMAs.  Identical op sequence in the HIP
 * render kernels (csrc/gs_common.h:falloff_log2); upstream's power = -0.5 (cxx dx^2 + cyy dy^2)
 * - cxy dx dy times log2(e), up to rounding. */
#define K_HALF_LOG2E (-0.72134752044448170f)
#define K_LOG2E (-1.44269504088896341f)
static inline float falloff_log2(const float* conic, float dx, float dy) {
    float A = conic[0] * K_HALF_LOG2E, B = conic[1] * K_LOG2E, C = conic[2] * K_HALF_LOG2E;
    float a2 = (A * dx) * dx;
    float b = B * dx;
    float t = fmaf(C, dy, b);
    return fmaf(dy, t, a2);
}

/* world point -> view (transformPoint4x3).  m is the 4x4 `world_view_transform`
 * (W2C^T, row-vector convention, /root/reference/scene/cameras.py:54) flattened row-major. */
static inline void xf43(const float* m, const float* p, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
static inline void xf44(const float* m, const float* p, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}

static inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

/* tile rectangle touched by a splat of integer radius r at pixel position (x,y) */
static inline void get_rect(float x, float y, int r, int gx, int gy, int* rmin, int* rmax) {
    float fr = (float)r;
    rmin[0] = imin(gx, imax(0, (int)((x - fr) / 16.0f)));
    rmin[1] = imin(gy, imax(0, (int)((y - fr) / 16.0f)));
    rmax[0] = imin(gx, imax(0, (int)((((x + fr) + 16.0f) - 1.0f) / 16.0f)));
    rmax[1] = imin(gy, imax(0, (int)((((y + fr) + 16.0f) - 1.0f) / 16.0f)));
}

/* ln(x) for x >= 1 from correctly-rounded IEEE ops only (frexp by bit fields, atanh series):
 * |error| < 2e-7 relative.  Identical op sequence in csrc/gs_common.h:gs_log. */
float oracle_log(float x) {
    uint32_t u = u_as(x);
    int e = (int)((u >> 23) & 255u) - 127;
    float m = f_as((u & 0x7FFFFFu) | 0x3F800000u);
    if (m > 1.41421356f) { m = m * 0.5f; e = e + 1; }
    float f = m - 1.0f;
    float t = f / (2.0f + f);
    float t2 = t * t;
    float p = 0.11111111f;
    p = fmaf(p, t2, 0.14285715f);
    p = fmaf(p, t2, 0.2f);
    p = fmaf(p, t2, 0.33333334f);
    p = fmaf(p, t2, 1.0f);
    return fmaf((float)e, 0.69314718f, (2.0f * t) * p);
}

/* culling limit of the alpha >= 1/255 ellipse, q(d) <= lim (negative: never reaches 1/255) */
static inline float cull_lim(float op) {
    return op >= 1.0f / 255.0f ? 2.0f * fmaxf(oracle_log(255.0f * op), 0.0f) * 1.001f + 1e-3f : -1.0f;
}

/* Tile-exact binning: tiles [ta, tb) of tile row ty whose pixel square can hold a pixel with
 * q(d) <= lim.  Conservative (a dropped tile has alpha < 1/255 at all of its pixels), so images and
 * gradients equal those of the full upstream rectangle (tested: oracle_set_exact_tiles(0) vs 1).
 * Identical op sequence in csrc/gs_common.h:span_ctx / row_span. */
static int g_exact_tiles = 1;
void oracle_set_exact_tiles(int on) { g_exact_tiles = on; }

/* Backward accumulation precision.  Default: fp64 sums (the reference answer).  With
 * oracle_set_acc_f32(1) every per-instance and per-Gaussian sum is rounded to fp32 after each add,
 * in this file's order (pixels row-major within a tile, then instances in list order): another
 * valid fp32 summation order, whose distance from the fp64 answer measures how much an fp32
 * implementation (upstream's atomics, the device's wave trees) can move an ill-conditioned
 * gradient.  Tests only; it never changes the forward. */
static int g_acc_f32 = 0;
void oracle_set_acc_f32(int on) { g_acc_f32 = on; }
static inline double acc_add(double a, double x) { return g_acc_f32 ? (double)((float)a + (float)x) : a + x; }

typedef struct { float mx, my, A, B, det, R, dyr, AL; int x0, x1, mode; } SpanCtx;
static SpanCtx span_ctx(float mx, float my, float A, float B, float C, float L, int x0, int x1) {
    SpanCtx s;
    s.mx = mx; s.my = my; s.A = A; s.B = B; s.x0 = x0; s.x1 = x1;
    s.det = A * C - B * B;
    s.mode = !(L >= 0.0f) ? 2 : ((A > 0.0f && C > 0.0f && s.det > 0.0f) ? 0 : 1);
    if (!g_exact_tiles) s.mode = 1;
    s.R = 0.0f; s.dyr = 0.0f; s.AL = 0.0f;
    if (s.mode == 0) {
        s.AL = A * L;
        s.R = sqrtf(s.AL / s.det) * 1.0001f + 0.01f;
        s.dyr = -B * sqrtf(L / (C * s.det));
    }
    return s;
}
static void row_span(const SpanCtx* s, int ty, int* ta, int* tb) {
    *ta = *tb = s->x0;
    if (s->mode == 2) return;
    if (s->mode == 1) { *tb = s->x1; return; }
    float lo = fmaxf((float)(TILE * ty) - s->my, -s->R);
    float hi = fminf((float)(TILE * ty + TILE - 1) - s->my, s->R);
    if (!(lo <= hi)) return;
    float d1 = fminf(fmaxf(s->dyr, lo), hi), d2 = fminf(fmaxf(-s->dyr, lo), hi);
    float xr = (-s->B * d1 + sqrtf(fmaxf(s->AL - s->det * d1 * d1, 0.0f))) / s->A;
    float xl = (-s->B * d2 - sqrtf(fmaxf(s->AL - s->det * d2 * d2, 0.0f))) / s->A;
    float X0 = fmaxf((s->mx + xl) - (0.05f + 0.001f * fabsf(xl)), -1.0e6f);
    float X1 = fminf((s->mx + xr) + (0.05f + 0.001f * fabsf(xr)), 1.0e6f);
    int a = imax(s->x0, (int)ceilf((X0 - 15.0f) / 16.0f));
    int b = imin(s->x1, (int)floorf(X1 / 16.0f) + 1);
    *ta = a;
    *tb = b > a ? b : a;
}

/* ------------------------------------------------------------------------------------------ */
/* cov3D  (ref: gaussian_model.py:27-31 + general_utils.py:78-110;  SURVEY §8a a4 step 4)        */
/* ------------------------------------------------------------------------------------------ */

/* rotation matrix of the (w,x,y,z) quaternion q, as used un-normalised by the rasterizer */
static inline void quat_rot(const float* q, float R[3][3]) {
    float r = q[0], x = q[1], y = q[2], z = q[3];
    R[0][0] = 1.f - 2.f * (y * y + z * z);
    R[0][1] = 2.f * (x * y - r * z);
    R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z);
    R[1][1] = 1.f - 2.f * (x * x + z * z);
    R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y);
    R[2][1] = 2.f * (y * z + r * x);
    R[2][2] = 1.f - 2.f * (x * x + y * y);
}

/* Sigma = L L^T, L = R diag(s); m[i][a] = s_i * R[a][i] (row i of M = S R^T) */
static void cov3d_one(const float* s, float mod, const float* q, float* cov) {
    float R[3][3];
    quat_rot(q, R);
    float sv[3] = {mod * s[0], mod * s[1], mod * s[2]};
    float m[3][3];
    for (int i = 0; i < 3; i++)
        for (int a = 0; a < 3; a++) m[i][a] = sv[i] * R[a][i];
#define SIG(a, b) (m[0][a] * m[0][b] + m[1][a] * m[1][b] + m[2][a] * m[2][b])
    cov[0] = SIG(0, 0);
    cov[1] = SIG(0, 1);
    cov[2] = SIG(0, 2);
    cov[3] = SIG(1, 1);
    cov[4] = SIG(1, 2);
    cov[5] = SIG(2, 2);
#undef SIG
}

void oracle_cov3d(int P, const float* scales, float mod, const float* rots, float* cov) {
    for (int i = 0; i < P; i++) cov3d_one(scales + 3 * i, mod, rots + 4 * i, cov + 6 * i);
}

/* d cov / d (scale, quaternion); gradient w.r.t. the raw (un-normalised) quaternion. */
static void cov3d_bwd_one(const float* s, float mod, const float* q, const float* dcov, float* dscale,
                          float* drot) {
    float R[3][3];
    quat_rot(q, R);
    float sv[3] = {mod * s[0], mod * s[1], mod * s[2]};
    float m[3][3];
    for (int i = 0; i < 3; i++)
        for (int a = 0; a < 3; a++) m[i][a] = sv[i] * R[a][i];
    /* symmetric dL/dSigma with halved off-diagonals */
    float g[3][3];
    g[0][0] = dcov[0];
    g[1][1] = dcov[3];
    g[2][2] = dcov[5];
    g[0][1] = g[1][0] = 0.5f * dcov[1];
    g[0][2] = g[2][0] = 0.5f * dcov[2];
    g[1][2] = g[2][1] = 0.5f * dcov[4];
    /* dL/dm[i][a] = 2 * sum_b m[i][b] g[b][a] */
    float dm[3][3];
    for (int i = 0; i < 3; i++)
        for (int a = 0; a < 3; a++) dm[i][a] = 2.0f * (m[i][0] * g[0][a] + m[i][1] * g[1][a] + m[i][2] * g[2][a]);
    /* m[i][a] = sv_i * R[a][i]  ->  dL/dsv_i = sum_a R[a][i] dm[i][a] */
    for (int i = 0; i < 3; i++) {
        float ds = R[0][i] * dm[i][0] + R[1][i] * dm[i][1] + R[2][i] * dm[i][2];
        dscale[i] = ds * mod;
    }
    /* dL/dR[a][i] = sv_i * dm[i][a] */
    float dR[3][3];
    for (int a = 0; a < 3; a++)
        for (int i = 0; i < 3; i++) dR[a][i] = sv[i] * dm[i][a];
    float r = q[0], x = q[1], y = q[2], z = q[3];
    /* R entries as functions of (r,x,y,z):  see quat_rot */
    drot[0] = 2.f * z * (dR[1][0] - dR[0][1]) + 2.f * y * (dR[0][2] - dR[2][0]) + 2.f * x * (dR[2][1] - dR[1][2]);
    drot[1] = 2.f * y * (dR[0][1] + dR[1][0]) + 2.f * z * (dR[0][2] + dR[2][0]) + 2.f * r * (dR[2][1] - dR[1][2]) -
              4.f * x * (dR[1][1] + dR[2][2]);
    drot[2] = 2.f * x * (dR[0][1] + dR[1][0]) + 2.f * r * (dR[0][2] - dR[2][0]) + 2.f * z * (dR[1][2] + dR[2][1]) -
              4.f * y * (dR[0][0] + dR[2][2]);
    drot[3] = 2.f * r * (dR[1][0] - dR[0][1]) + 2.f * x * (dR[0][2] + dR[2][0]) + 2.f * y * (dR[1][2] + dR[2][1]) -
              4.f * z * (dR[0][0] + dR[1][1]);
}

void oracle_cov3d_backward(int P, const float* scales, float mod, const float* rots, const float* dcov,
                           float* dscale, float* drot) {
    for (int i = 0; i < P; i++) cov3d_bwd_one(scales + 3 * i, mod, rots + 4 * i, dcov + 6 * i, dscale + 3 * i, drot + 4 * i);
}

/* ------------------------------------------------------------------------------------------ */
/* SH -> RGB  (ref: sh_utils.py:57-100, gaussian_renderer/__init__.py:73-78)                    */
/* ------------------------------------------------------------------------------------------ */

static void sh_dir(const float* p, const float* campos, float* dir, float* dir_raw) {
    float dx = p[0] - campos[0], dy = p[1] - campos[1], dz = p[2] - campos[2];
    dir_raw[0] = dx; dir_raw[1] = dy; dir_raw[2] = dz;
    float len = sqrtf(dx * dx + dy * dy + dz * dz);
    dir[0] = dx / len; dir[1] = dy / len; dir[2] = dz / len;
}

/* rgb for one Gaussian: sh points at M*3 floats ([k][c]) */
static void sh_eval_one(int deg, const float* sh, const float* dir, float* rgb, unsigned char* clamped) {
    float x = dir[0], y = dir[1], z = dir[2];
    for (int c = 0; c < 3; c++) {
#define S(k) sh[3 * (k) + c]
        float res = SH_C0 * S(0);
        if (deg > 0) {
            res = res - (SH_C1 * y) * S(1) + (SH_C1 * z) * S(2) - (SH_C1 * x) * S(3);
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z;
                float xy = x * y, yz = y * z, xz = x * z;
                res = res + (SH_C2[0] * xy) * S(4) + (SH_C2[1] * yz) * S(5) + (SH_C2[2] * (2.0f * zz - xx - yy)) * S(6) +
                      (SH_C2[3] * xz) * S(7) + (SH_C2[4] * (xx - yy)) * S(8);
                if (deg > 2) {
                    res = res + ((SH_C3[0] * y) * (3.0f * xx - yy)) * S(9) + ((SH_C3[1] * xy) * z) * S(10) +
                          ((SH_C3[2] * y) * (4.0f * zz - xx - yy)) * S(11) +
                          ((SH_C3[3] * z) * (2.0f * zz - 3.0f * xx - 3.0f * yy)) * S(12) +
                          ((SH_C3[4] * x) * (4.0f * zz - xx - yy)) * S(13) + ((SH_C3[5] * z) * (xx - yy)) * S(14) +
                          ((SH_C3[6] * x) * (xx - 3.0f * yy)) * S(15);
                }
            }
        }
#undef S
        res = res + 0.5f;
        clamped[c] = res < 0.0f;
        rgb[c] = res < 0.0f ? 0.0f : res;
    }
}

void oracle_sh_forward(int P, int deg, int M, const float* means, const float* campos, const float* shs,
                       float* rgb, unsigned char* clamped) {
    for (int i = 0; i < P; i++) {
        float dir[3], raw[3];
        sh_dir(means + 3 * i, campos, dir, raw);
        sh_eval_one(deg, shs + (size_t)i * M * 3, dir, rgb + 3 * i, clamped + 3 * i);
    }
}

/* d rgb -> d sh (written, M*3) and d mean (returned in dmean, overwritten) */
static void sh_bwd_one(int deg, int M, const float* p, const float* campos, const float* sh,
                       const unsigned char* clamped, const float* drgb_in, float* dsh, float* dmean) {
    float dir[3], raw[3];
    sh_dir(p, campos, dir, raw);
    float x = dir[0], y = dir[1], z = dir[2];
    float g[3];
    for (int c = 0; c < 3; c++) g[c] = clamped[c] ? 0.0f : drgb_in[c];
    for (int k = 0; k < M * 3; k++) dsh[k] = 0.0f;
    float ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    float b[16];
    b[0] = SH_C0;
    if (deg > 0) { b[1] = -SH_C1 * y; b[2] = SH_C1 * z; b[3] = -SH_C1 * x; }
    if (deg > 1) {
        b[4] = SH_C2[0] * xy; b[5] = SH_C2[1] * yz; b[6] = SH_C2[2] * (2.0f * zz - xx - yy);
        b[7] = SH_C2[3] * xz; b[8] = SH_C2[4] * (xx - yy);
    }
    if (deg > 2) {
        b[9] = (SH_C3[0] * y) * (3.0f * xx - yy);
        b[10] = (SH_C3[1] * xy) * z;
        b[11] = (SH_C3[2] * y) * (4.0f * zz - xx - yy);
        b[12] = (SH_C3[3] * z) * (2.0f * zz - 3.0f * xx - 3.0f * yy);
        b[13] = (SH_C3[4] * x) * (4.0f * zz - xx - yy);
        b[14] = (SH_C3[5] * z) * (xx - yy);
        b[15] = (SH_C3[6] * x) * (xx - 3.0f * yy);
    }
    int K = (deg + 1) * (deg + 1);
    for (int k = 0; k < K; k++)
        for (int c = 0; c < 3; c++) dsh[3 * k + c] = b[k] * g[c];
    for (int c = 0; c < 3; c++) {
#define S(k) sh[3 * (k) + c]
        if (deg > 0) {
            ddx[c] = -SH_C1 * S(3);
            ddy[c] = -SH_C1 * S(1);
            ddz[c] = SH_C1 * S(2);
            if (deg > 1) {
                ddx[c] = ddx[c] + (SH_C2[0] * y) * S(4) + (SH_C2[2] * (-2.f * x)) * S(6) + (SH_C2[3] * z) * S(7) +
                         (SH_C2[4] * (2.f * x)) * S(8);
                ddy[c] = ddy[c] + (SH_C2[0] * x) * S(4) + (SH_C2[1] * z) * S(5) + (SH_C2[2] * (-2.f * y)) * S(6) +
                         (SH_C2[4] * (-2.f * y)) * S(8);
                ddz[c] = ddz[c] + (SH_C2[1] * y) * S(5) + (SH_C2[2] * (4.f * z)) * S(6) + (SH_C2[3] * x) * S(7);
                if (deg > 2) {
                    ddx[c] = ddx[c] + (SH_C3[0] * (6.f * xy)) * S(9) + (SH_C3[1] * yz) * S(10) +
                             (SH_C3[2] * (-2.f * xy)) * S(11) + (SH_C3[3] * (-6.f * xz)) * S(12) +
                             (SH_C3[4] * (-3.f * xx + 4.f * zz - yy)) * S(13) + (SH_C3[5] * (2.f * xz)) * S(14) +
                             (SH_C3[6] * (3.f * (xx - yy))) * S(15);
                    ddy[c] = ddy[c] + (SH_C3[0] * (3.f * (xx - yy))) * S(9) + (SH_C3[1] * xz) * S(10) +
                             (SH_C3[2] * (-3.f * yy + 4.f * zz - xx)) * S(11) + (SH_C3[3] * (-6.f * yz)) * S(12) +
                             (SH_C3[4] * (-2.f * xy)) * S(13) + (SH_C3[5] * (-2.f * yz)) * S(14) +
                             (SH_C3[6] * (-6.f * xy)) * S(15);
                    ddz[c] = ddz[c] + (SH_C3[1] * xy) * S(10) + (SH_C3[2] * (8.f * yz)) * S(11) +
                             (SH_C3[3] * (3.f * (2.f * zz - xx - yy))) * S(12) + (SH_C3[4] * (8.f * xz)) * S(13) +
                             (SH_C3[5] * (xx - yy)) * S(14);
                }
            }
        }
#undef S
    }
    float dldir[3];
    dldir[0] = ddx[0] * g[0] + ddx[1] * g[1] + ddx[2] * g[2];
    dldir[1] = ddy[0] * g[0] + ddy[1] * g[1] + ddy[2] * g[2];
    dldir[2] = ddz[0] * g[0] + ddz[1] * g[1] + ddz[2] * g[2];
    /* d normalize(v) / dv */
    float vx = raw[0], vy = raw[1], vz = raw[2];
    float sum2 = vx * vx + vy * vy + vz * vz;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    dmean[0] = ((sum2 - vx * vx) * dldir[0] - vy * vx * dldir[1] - vz * vx * dldir[2]) * invsum32;
    dmean[1] = (-vx * vy * dldir[0] + (sum2 - vy * vy) * dldir[1] - vz * vy * dldir[2]) * invsum32;
    dmean[2] = (-vx * vz * dldir[0] - vy * vz * dldir[1] + (sum2 - vz * vz) * dldir[2]) * invsum32;
}

void oracle_sh_backward(int P, int deg, int M, const float* means, const float* campos, const float* shs,
                        const unsigned char* clamped, const float* drgb, float* dsh, float* dmean) {
    for (int i = 0; i < P; i++)
        sh_bwd_one(deg, M, means + 3 * i, campos, shs + (size_t)i * M * 3, clamped + 3 * i, drgb + 3 * i,
                   dsh + (size_t)i * M * 3, dmean + 3 * i);
}

/* ------------------------------------------------------------------------------------------ */
/* preprocess forward                                                           */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    float xy[2];
    float conic[3];
    float opacity;
    float rgb[3];
    float depth;
    int radius;
    int rmin[2], rmax[2];
    float lim;
    uint32_t count; /* tile-exact instance count (row spans) */
    unsigned char clamped[3];
} Splat;

typedef struct {
    int P, D, M, W, H, gx, gy;
    const float *bg, *means, *shs, *colors, *opac, *scales, *rots, *cov3d, *view, *proj, *campos;
    float mod, tanfovx, tanfovy, fx, fy;
} Scene;

/* 2D covariance (a, b, c) of one Gaussian; also returns T (2x3) and the clamp flags */
static void cov2d_one(const Scene* s, const float* p, const float* cov3, float* abc, float Tm[2][3], float* tview,
                      float* gradmul) {
    float t[3];
    xf43(s->view, p, t);
    float limx = 1.3f * s->tanfovx, limy = 1.3f * s->tanfovy;
    float txtz = t[0] / t[2], tytz = t[1] / t[2];
    float cx = fminf(limx, fmaxf(-limx, txtz)), cy = fminf(limy, fmaxf(-limy, tytz));
    t[0] = cx * t[2];
    t[1] = cy * t[2];
    if (gradmul) {
        gradmul[0] = (txtz < -limx || txtz > limx) ? 0.0f : 1.0f;
        gradmul[1] = (tytz < -limy || tytz > limy) ? 0.0f : 1.0f;
    }
    float tz2 = t[2] * t[2];
    float J00 = s->fx / t[2], J02 = -(s->fx * t[0]) / tz2;
    float J11 = s->fy / t[2], J12 = -(s->fy * t[1]) / tz2;
    const float* v = s->view; /* Rw[i][j] = v[4*j + i] */
    for (int r = 0; r < 3; r++) {
        Tm[0][r] = v[4 * r + 0] * J00 + v[4 * r + 2] * J02;
        Tm[1][r] = v[4 * r + 1] * J11 + v[4 * r + 2] * J12;
    }
    float V[3][3] = {{cov3[0], cov3[1], cov3[2]}, {cov3[1], cov3[3], cov3[4]}, {cov3[2], cov3[4], cov3[5]}};
    float U[2][3];
    for (int i = 0; i < 2; i++)
        for (int b = 0; b < 3; b++) U[i][b] = Tm[i][0] * V[0][b] + Tm[i][1] * V[1][b] + Tm[i][2] * V[2][b];
    float c00 = U[0][0] * Tm[0][0] + U[0][1] * Tm[0][1] + U[0][2] * Tm[0][2];
    float c01 = U[0][0] * Tm[1][0] + U[0][1] * Tm[1][1] + U[0][2] * Tm[1][2];
    float c11 = U[1][0] * Tm[1][0] + U[1][1] * Tm[1][1] + U[1][2] * Tm[1][2];
    abc[0] = c00 + 0.3f;
    abc[1] = c01;
    abc[2] = c11 + 0.3f;
    if (tview) { tview[0] = t[0]; tview[1] = t[1]; tview[2] = t[2]; }
}

/* returns 1 if visible (radius > 0 and touches >= 1 tile) */
static int preprocess_one(const Scene* s, int i, Splat* o) {
    memset(o, 0, sizeof(*o));
    const float* p = s->means + 3 * i;
    float pv[3];
    xf43(s->view, p, pv);
    if (pv[2] <= 0.2f) return 0;
    float ph[4];
    xf44(s->proj, p, ph);
    float pw = 1.0f / (ph[3] + 0.0000001f);
    float pproj[2] = {ph[0] * pw, ph[1] * pw};
    float cov3[6];
    if (s->cov3d) memcpy(cov3, s->cov3d + 6 * i, sizeof(cov3));
    else cov3d_one(s->scales + 3 * i, s->mod, s->rots + 4 * i, cov3);
    float abc[3], Tm[2][3];
    cov2d_one(s, p, cov3, abc, Tm, NULL, NULL);
    float det = abc[0] * abc[2] - abc[1] * abc[1];
    if (det == 0.0f) return 0;
    float det_inv = 1.f / det;
    float conic[3] = {abc[2] * det_inv, -abc[1] * det_inv, abc[0] * det_inv};
    float mid = 0.5f * (abc[0] + abc[2]);
    float disc = fmaxf(0.1f, mid * mid - det);
    float l1 = mid + sqrtf(disc), l2 = mid - sqrtf(disc);
    int radius = (int)ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    float px = ndc2pix(pproj[0], s->W), py = ndc2pix(pproj[1], s->H);
    int rmin[2], rmax[2];
    get_rect(px, py, radius, s->gx, s->gy, rmin, rmax);
    if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) return 0;
    if (s->colors) {
        memcpy(o->rgb, s->colors + 3 * i, 3 * sizeof(float));
    } else {
        float dir[3], raw[3];
        sh_dir(p, s->campos, dir, raw);
        sh_eval_one(s->D, s->shs + (size_t)i * s->M * 3, dir, o->rgb, o->clamped);
    }
    o->xy[0] = px; o->xy[1] = py;
    o->conic[0] = conic[0]; o->conic[1] = conic[1]; o->conic[2] = conic[2];
    o->opacity = s->opac[i];
    o->depth = pv[2];
    o->radius = radius;
    o->rmin[0] = rmin[0]; o->rmin[1] = rmin[1]; o->rmax[0] = rmax[0]; o->rmax[1] = rmax[1];
    o->lim = cull_lim(o->opacity);
    SpanCtx sp = span_ctx(px, py, conic[0], conic[1], conic[2], o->lim, rmin[0], rmax[0]);
    uint32_t count = 0;
    for (int ty = rmin[1]; ty < rmax[1]; ty++) {
        int ta, tb;
        row_span(&sp, ty, &ta, &tb);
        count += (uint32_t)(tb - ta);
    }
    o->count = count;
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* binning: (tile, depth) ordering with Gaussian-index tie-break                 */
/* ------------------------------------------------------------------------------------------ */

typedef struct { uint32_t tile, dkey, gid; } Inst;

static int inst_cmp(const void* a, const void* b) {
    const Inst *x = (const Inst*)a, *y = (const Inst*)b;
    if (x->tile != y->tile) return x->tile < y->tile ? -1 : 1;
    if (x->dkey != y->dkey) return x->dkey < y->dkey ? -1 : 1;
    if (x->gid != y->gid) return x->gid < y->gid ? -1 : 1;
    return 0;
}

typedef struct {
    Splat* sp;
    Inst* inst;
    long long I;
    uint32_t* rng; /* tiles*2 */
} Binned;

static int bin_scene(const Scene* s, Binned* b) {
    b->sp = (Splat*)calloc((size_t)(s->P ? s->P : 1), sizeof(Splat));
    long long I = 0;
#pragma omp parallel for schedule(static) reduction(+ : I)
    for (int i = 0; i < s->P; i++)
        if (preprocess_one(s, i, &b->sp[i])) I += (long long)b->sp[i].count;
    b->I = I;
    b->inst = (Inst*)malloc((size_t)(I ? I : 1) * sizeof(Inst));
    long long k = 0;
    for (int i = 0; i < s->P; i++) {
        Splat* o = &b->sp[i];
        if (o->radius == 0) continue;
        SpanCtx sp = span_ctx(o->xy[0], o->xy[1], o->conic[0], o->conic[1], o->conic[2], o->lim, o->rmin[0],
                              o->rmax[0]);
        for (int y = o->rmin[1]; y < o->rmax[1]; y++) {
            int ta, tb;
            row_span(&sp, y, &ta, &tb);
            for (int x = ta; x < tb; x++) {
                b->inst[k].tile = (uint32_t)(y * s->gx + x);
                b->inst[k].dkey = u_as(o->depth);
                b->inst[k].gid = (uint32_t)i;
                k++;
            }
        }
    }
    qsort(b->inst, (size_t)I, sizeof(Inst), inst_cmp);
    int tiles = s->gx * s->gy;
    b->rng = (uint32_t*)calloc((size_t)tiles * 2, sizeof(uint32_t));
    for (long long j = 0; j < I; j++) {
        uint32_t t = b->inst[j].tile;
        if (j == 0 || b->inst[j - 1].tile != t) b->rng[2 * t] = (uint32_t)j;
        if (j == I - 1 || b->inst[j + 1].tile != t) b->rng[2 * t + 1] = (uint32_t)(j + 1);
    }
    return 0;
}

static void free_bins(Binned* b) { free(b->sp); free(b->inst); free(b->rng); }

static void init_scene(Scene* s, int P, int D, int M, const float* bg, int W, int H, const float* means,
                       const float* shs, const float* colors, const float* opac, const float* scales, float mod,
                       const float* rots, const float* cov3d, const float* view, const float* proj,
                       const float* campos, float tanfovx, float tanfovy) {
    s->P = P; s->D = D; s->M = M; s->W = W; s->H = H;
    s->gx = (W + TILE - 1) / TILE; s->gy = (H + TILE - 1) / TILE;
    s->bg = bg; s->means = means; s->shs = shs; s->colors = colors; s->opac = opac;
    s->scales = scales; s->rots = rots; s->cov3d = cov3d; s->view = view; s->proj = proj; s->campos = campos;
    s->mod = mod; s->tanfovx = tanfovx; s->tanfovy = tanfovy;
    s->fy = (float)H / (2.0f * tanfovy);
    s->fx = (float)W / (2.0f * tanfovx);
}

/* ------------------------------------------------------------------------------------------ */
/* render forward                                                              */
/* ------------------------------------------------------------------------------------------ */

/* Optional per-pixel flags for the device's fast numerics mode (hardware exp2, <= 1 ulp): a pixel
 * is marked when one of its discrete decisions sits so close to its threshold that a 1-ulp exp2
 * or the drift of T it causes could flip it -- alpha within 1e-6 (relative) of 1/255, or a tested
 * T(1 - alpha) within 2e-5 (relative) of 1e-4.  Side output only: the oracle's arithmetic is the
 * same with or without it. */
static unsigned char* g_near = NULL;
void oracle_set_near_flags(unsigned char* flags) { g_near = flags; }

static void render_fwd(const Scene* s, const Binned* b, float* out, float* finalT, uint32_t* ncontrib) {
    int W = s->W, H = s->H;
    int ntiles = s->gx * s->gy;
#pragma omp parallel for schedule(dynamic, 4)
    for (int t_ = 0; t_ < ntiles; t_++) {
        {
            int ty = t_ / s->gx, tx = t_ % s->gx;
            uint32_t t = (uint32_t)t_;
            uint32_t r0 = b->rng[2 * t], r1 = b->rng[2 * t + 1];
            for (int ly = 0; ly < TILE; ly++)
                for (int lx = 0; lx < TILE; lx++) {
                    int px = tx * TILE + lx, py = ty * TILE + ly;
                    if (px >= W || py >= H) continue;
                    float pfx = (float)px, pfy = (float)py;
                    float T = 1.0f, C[3] = {0, 0, 0};
                    uint32_t contributor = 0, last = 0;
                    int near = 0;
                    for (uint32_t k = r0; k < r1; k++) {
                        contributor++;
                        const Splat* o = &b->sp[b->inst[k].gid];
                        float dx = o->xy[0] - pfx, dy = o->xy[1] - pfy;
                        float power2 = falloff_log2(o->conic, dx, dy);
                        if (power2 > 0.0f) continue;
                        float a_raw = o->opacity * oracle_exp2(power2);
                        if (g_near && fabs((double)a_raw * 255.0 - 1.0) < 1e-6) near = 1;
                        float alpha = fminf(0.99f, a_raw);
                        if (alpha < 1.0f / 255.0f) continue;
                        float test_T = T * (1.0f - alpha);
                        if (g_near && fabs((double)test_T * 1e4 - 1.0) < 2e-5) near = 1;
                        if (test_T < 0.0001f) break;
                        for (int c = 0; c < 3; c++) C[c] += o->rgb[c] * alpha * T;
                        T = test_T;
                        last = contributor;
                    }
                    size_t pix = (size_t)py * W + px;
                    if (g_near) g_near[pix] = (unsigned char)near;
                    if (finalT) finalT[pix] = T;
                    if (ncontrib) ncontrib[pix] = last;
                    for (int c = 0; c < 3; c++) out[(size_t)c * H * W + pix] = C[c] + T * s->bg[c];
                }
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* public forward                                                                              */
/* ------------------------------------------------------------------------------------------ */

/* Returns num_rendered.  Optional outputs may be NULL.  out_list receives the Gaussian ids of
 * the sorted instance list (num_rendered entries; call once with out_list = NULL to size it). */
long long oracle_forward(int P, int D, int M, const float* bg, int W, int H, const float* means,
                         const float* shs, const float* colors, const float* opac, const float* scales,
                         float mod, const float* rots, const float* cov3d, const float* view, const float* proj,
                         const float* campos, float tanfovx, float tanfovy, float* out_color, int* radii,
                         float* out_xy, float* out_conic_o, float* out_rgb, float* out_depth, uint32_t* out_tiles,
                         unsigned char* out_clamped, float* out_finalT, uint32_t* out_ncontrib,
                         uint32_t* out_list, uint32_t* out_ranges) {
    Scene s;
    init_scene(&s, P, D, M, bg, W, H, means, shs, colors, opac, scales, mod, rots, cov3d, view, proj, campos,
               tanfovx, tanfovy);
    memset(out_color, 0, sizeof(float) * 3 * (size_t)W * H);
    if (P == 0) {
        if (out_finalT) for (size_t i = 0; i < (size_t)W * H; i++) out_finalT[i] = 1.0f;
        if (out_ncontrib) memset(out_ncontrib, 0, sizeof(uint32_t) * (size_t)W * H);
        if (out_ranges) memset(out_ranges, 0, sizeof(uint32_t) * 2 * (size_t)s.gx * s.gy);
        return 0;
    }
    Binned b;
    bin_scene(&s, &b);
    for (int i = 0; i < P; i++) {
        const Splat* o = &b.sp[i];
        radii[i] = o->radius;
        int area = (o->rmax[0] - o->rmin[0]) * (o->rmax[1] - o->rmin[1]);
        if (out_xy) { out_xy[2 * i] = o->xy[0]; out_xy[2 * i + 1] = o->xy[1]; }
        if (out_conic_o) {
            out_conic_o[4 * i] = o->conic[0]; out_conic_o[4 * i + 1] = o->conic[1];
            out_conic_o[4 * i + 2] = o->conic[2]; out_conic_o[4 * i + 3] = o->opacity;
        }
        if (out_rgb) for (int c = 0; c < 3; c++) out_rgb[3 * i + c] = o->rgb[c];
        if (out_depth) out_depth[i] = o->depth;
        if (out_tiles) out_tiles[i] = o->radius > 0 ? o->count : 0u;
        (void)area;
        if (out_clamped) for (int c = 0; c < 3; c++) out_clamped[3 * i + c] = o->clamped[c];
    }
    render_fwd(&s, &b, out_color, out_finalT, out_ncontrib);
    if (out_list) for (long long k = 0; k < b.I; k++) out_list[k] = b.inst[k].gid;
    if (out_ranges) memcpy(out_ranges, b.rng, sizeof(uint32_t) * 2 * (size_t)s.gx * s.gy);
    long long I = b.I;
    free_bins(&b);
    return I;
}

/* ------------------------------------------------------------------------------------------ */
/* backward                                                                  */
/* ------------------------------------------------------------------------------------------ */

/* Recomputes the forward, then runs render bwd and preprocess bwd.  Every output has P rows;
 * dL_dcov3D / dL_dsh / dL_dscale / dL_drot / dL_dconic may be NULL. */
long long oracle_backward(int P, int D, int M, const float* bg, int W, int H, const float* means,
                          const float* shs, const float* colors, const float* opac, const float* scales,
                          float mod, const float* rots, const float* cov3d, const float* view, const float* proj,
                          const float* campos, float tanfovx, float tanfovy, const float* dL_dpix,
                          float* dL_dmean2D, float* dL_dcolor, float* dL_dopacity, float* dL_dmeans3D,
                          float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot, float* dL_dconic) {
    Scene s;
    init_scene(&s, P, D, M, bg, W, H, means, shs, colors, opac, scales, mod, rots, cov3d, view, proj, campos,
               tanfovx, tanfovy);
    memset(dL_dmean2D, 0, sizeof(float) * 3 * (size_t)P);
    memset(dL_dcolor, 0, sizeof(float) * 3 * (size_t)P);
    memset(dL_dopacity, 0, sizeof(float) * (size_t)P);
    memset(dL_dmeans3D, 0, sizeof(float) * 3 * (size_t)P);
    if (dL_dcov3D) memset(dL_dcov3D, 0, sizeof(float) * 6 * (size_t)P);
    if (dL_dsh) memset(dL_dsh, 0, sizeof(float) * 3 * (size_t)P * (M > 0 ? M : 1));
    if (dL_dscale) memset(dL_dscale, 0, sizeof(float) * 3 * (size_t)P);
    if (dL_drot) memset(dL_drot, 0, sizeof(float) * 4 * (size_t)P);
    if (dL_dconic) memset(dL_dconic, 0, sizeof(float) * 4 * (size_t)P);
    if (P == 0) return 0;
    Binned b;
    bin_scene(&s, &b);
    size_t npix = (size_t)W * H;
    float* fout = (float*)malloc(sizeof(float) * 3 * npix);
    float* finalT = (float*)malloc(sizeof(float) * npix);
    uint32_t* ncon = (uint32_t*)malloc(sizeof(uint32_t) * npix);
    render_fwd(&s, &b, fout, finalT, ncon);
    /* per-instance double accumulators (each instance belongs to one tile -> one thread):
     * color(3), mean2D(2), conic(3: xx, xy, yy), opacity(1); summed per Gaussian afterwards */
    double* iacc = (double*)calloc((size_t)(b.I ? b.I : 1) * 9, sizeof(double));
    float ddelx_dx = (float)(0.5 * W), ddely_dy = (float)(0.5 * H);
    int ntiles = s.gx * s.gy;
#pragma omp parallel for schedule(dynamic, 4)
    for (int t_ = 0; t_ < ntiles; t_++) {
        {
            int ty = t_ / s.gx, tx = t_ % s.gx;
            uint32_t t = (uint32_t)t_;
            uint32_t r0 = b.rng[2 * t], r1 = b.rng[2 * t + 1];
            for (int ly = 0; ly < TILE; ly++)
                for (int lx = 0; lx < TILE; lx++) {
                    int px = tx * TILE + lx, py = ty * TILE + ly;
                    if (px >= W || py >= H) continue;
                    size_t pix = (size_t)py * W + px;
                    float pfx = (float)px, pfy = (float)py;
                    float T_final = finalT[pix], T = T_final;
                    uint32_t last_contributor = ncon[pix];
                    float dpix[3];
                    for (int c = 0; c < 3; c++) dpix[c] = dL_dpix[(size_t)c * npix + pix];
                    float accum_rec[3] = {0, 0, 0}, last_color[3] = {0, 0, 0}, last_alpha = 0.0f;
                    float bg_dot = bg[0] * dpix[0] + bg[1] * dpix[1] + bg[2] * dpix[2];
                    uint32_t contributor = r1 - r0;
                    for (uint32_t kk = r1; kk > r0; kk--) {
                        uint32_t k = kk - 1;
                        contributor--;
                        if (contributor >= last_contributor) continue;
                        uint32_t gid = b.inst[k].gid;
                        const Splat* o = &b.sp[gid];
                        float dx = o->xy[0] - pfx, dy = o->xy[1] - pfy;
                        float power2 = falloff_log2(o->conic, dx, dy);
                        if (power2 > 0.0f) continue;
                        float G = oracle_exp2(power2);
                        float alpha = fminf(0.99f, o->opacity * G);
                        if (alpha < 1.0f / 255.0f) continue;
                        /* T recovered with one correctly rounded reciprocal, reused for the background
                         * term (upstream divides twice; identical up to one rounding) */
                        float inv = 1.f / (1.f - alpha);
                        T = T * inv;
                        float dchannel_dcolor = alpha * T;
                        float dL_dalpha = 0.0f;
                        double* a = iacc + (size_t)k * 9;
                        for (int c = 0; c < 3; c++) {
                            float col = o->rgb[c];
                            accum_rec[c] = last_alpha * last_color[c] + (1.f - last_alpha) * accum_rec[c];
                            last_color[c] = col;
                            dL_dalpha += (col - accum_rec[c]) * dpix[c];
                            a[c] = acc_add(a[c], (double)(dchannel_dcolor * dpix[c]));
                        }
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final * inv) * bg_dot;
                        float dL_dG = o->opacity * dL_dalpha;
                        float gdx = G * dx, gdy = G * dy;
                        float dG_ddelx = -gdx * o->conic[0] - gdy * o->conic[1];
                        float dG_ddely = -gdy * o->conic[2] - gdx * o->conic[1];
                        a[3] = acc_add(a[3], (double)(dL_dG * dG_ddelx * ddelx_dx));
                        a[4] = acc_add(a[4], (double)(dL_dG * dG_ddely * ddely_dy));
                        a[5] = acc_add(a[5], (double)(-0.5f * gdx * dx * dL_dG));
                        a[6] = acc_add(a[6], (double)(-0.5f * gdx * dy * dL_dG));
                        a[7] = acc_add(a[7], (double)(-0.5f * gdy * dy * dL_dG));
                        a[8] = acc_add(a[8], (double)(G * dL_dalpha));
                    }
                }
        }
    }
    double* acc = (double*)calloc((size_t)P * 9, sizeof(double));
    for (long long k = 0; k < b.I; k++)
        for (int c = 0; c < 9; c++) {
            double* d = &acc[(size_t)b.inst[k].gid * 9 + c];
            *d = acc_add(*d, iacc[(size_t)k * 9 + c]);
        }
    free(iacc);
    /* preprocess backward for every visible Gaussian */
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; i++) {
        const Splat* o = &b.sp[i];
        if (o->radius <= 0) continue;
        double* a = acc + (size_t)i * 9;
        float dcol[3] = {(float)a[0], (float)a[1], (float)a[2]};
        float dm2[2] = {(float)a[3], (float)a[4]};
        float dcon[3] = {(float)a[5], (float)a[6], (float)a[7]};
        dL_dcolor[3 * i] = dcol[0]; dL_dcolor[3 * i + 1] = dcol[1]; dL_dcolor[3 * i + 2] = dcol[2];
        dL_dmean2D[3 * i] = dm2[0]; dL_dmean2D[3 * i + 1] = dm2[1]; dL_dmean2D[3 * i + 2] = 0.0f;
        dL_dopacity[i] = (float)a[8];
        if (dL_dconic) {
            dL_dconic[4 * i] = dcon[0]; dL_dconic[4 * i + 1] = dcon[1];
            dL_dconic[4 * i + 2] = 0.0f; dL_dconic[4 * i + 3] = dcon[2];
        }
        const float* p = means + 3 * i;
        float cov3[6];
        if (cov3d) memcpy(cov3, cov3d + 6 * i, sizeof(cov3));
        else cov3d_one(scales + 3 * i, mod, rots + 4 * i, cov3);
        /* --- conic -> cov2D -> cov3D / mean (computeCov2D backward) --- */
        float abc[3], Tm[2][3], t[3], gm[2];
        cov2d_one(&s, p, cov3, abc, Tm, t, gm);
        float A = abc[0], Bv = abc[1], Cv = abc[2];
        float denom = A * Cv - Bv * Bv;
        float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float dcv[6] = {0, 0, 0, 0, 0, 0};
        if (denom2inv != 0.0f) {
            dL_da = denom2inv * (-Cv * Cv * dcon[0] + 2.f * Bv * Cv * dcon[1] + (denom - A * Cv) * dcon[2]);
            dL_dc = denom2inv * (-A * A * dcon[2] + 2.f * A * Bv * dcon[1] + (denom - A * Cv) * dcon[0]);
            dL_db = denom2inv * 2.f * (Bv * Cv * dcon[0] - (denom + 2.f * Bv * Bv) * dcon[1] + A * Bv * dcon[2]);
            dcv[0] = Tm[0][0] * Tm[0][0] * dL_da + Tm[0][0] * Tm[1][0] * dL_db + Tm[1][0] * Tm[1][0] * dL_dc;
            dcv[3] = Tm[0][1] * Tm[0][1] * dL_da + Tm[0][1] * Tm[1][1] * dL_db + Tm[1][1] * Tm[1][1] * dL_dc;
            dcv[5] = Tm[0][2] * Tm[0][2] * dL_da + Tm[0][2] * Tm[1][2] * dL_db + Tm[1][2] * Tm[1][2] * dL_dc;
            dcv[1] = 2.f * Tm[0][0] * Tm[0][1] * dL_da + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_db +
                     2.f * Tm[1][0] * Tm[1][1] * dL_dc;
            dcv[2] = 2.f * Tm[0][0] * Tm[0][2] * dL_da + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_db +
                     2.f * Tm[1][0] * Tm[1][2] * dL_dc;
            dcv[4] = 2.f * Tm[0][2] * Tm[0][1] * dL_da + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_db +
                     2.f * Tm[1][1] * Tm[1][2] * dL_dc;
        }
        float V[3][3] = {{cov3[0], cov3[1], cov3[2]}, {cov3[1], cov3[3], cov3[4]}, {cov3[2], cov3[4], cov3[5]}};
        float dT0[3], dT1[3];
        for (int r = 0; r < 3; r++) {
            float tv0 = Tm[0][0] * V[r][0] + Tm[0][1] * V[r][1] + Tm[0][2] * V[r][2];
            float tv1 = Tm[1][0] * V[r][0] + Tm[1][1] * V[r][1] + Tm[1][2] * V[r][2];
            dT0[r] = 2.f * tv0 * dL_da + tv1 * dL_db;
            dT1[r] = 2.f * tv1 * dL_dc + tv0 * dL_db;
        }
        const float* v = view; /* Rw[i][j] = v[4*j+i] */
        float dJ00 = v[0] * dT0[0] + v[4] * dT0[1] + v[8] * dT0[2];
        float dJ02 = v[2] * dT0[0] + v[6] * dT0[1] + v[10] * dT0[2];
        float dJ11 = v[1] * dT1[0] + v[5] * dT1[1] + v[9] * dT1[2];
        float dJ12 = v[2] * dT1[0] + v[6] * dT1[1] + v[10] * dT1[2];
        float tz = 1.f / t[2], tz2 = tz * tz, tz3 = tz2 * tz;
        float dL_dtx = gm[0] * -s.fx * tz2 * dJ02;
        float dL_dty = gm[1] * -s.fy * tz2 * dJ12;
        float dL_dtz = -s.fx * tz2 * dJ00 - s.fy * tz2 * dJ11 + (2.f * s.fx * t[0]) * tz3 * dJ02 +
                       (2.f * s.fy * t[1]) * tz3 * dJ12;
        float dmean[3];
        dmean[0] = v[0] * dL_dtx + v[1] * dL_dty + v[2] * dL_dtz;
        dmean[1] = v[4] * dL_dtx + v[5] * dL_dty + v[6] * dL_dtz;
        dmean[2] = v[8] * dL_dtx + v[9] * dL_dty + v[10] * dL_dtz;
        if (dL_dcov3D) for (int k = 0; k < 6; k++) dL_dcov3D[6 * i + k] = dcv[k];
        /* --- projection: mean2D (NDC) -> mean3D --- */
        float ph[4];
        xf44(proj, p, ph);
        float m_w = 1.0f / (ph[3] + 0.0000001f);
        float mul1 = (proj[0] * p[0] + proj[4] * p[1] + proj[8] * p[2] + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * p[0] + proj[5] * p[1] + proj[9] * p[2] + proj[13]) * m_w * m_w;
        float pm[3];
        pm[0] = (proj[0] * m_w - proj[3] * mul1) * dm2[0] + (proj[1] * m_w - proj[3] * mul2) * dm2[1];
        pm[1] = (proj[4] * m_w - proj[7] * mul1) * dm2[0] + (proj[5] * m_w - proj[7] * mul2) * dm2[1];
        pm[2] = (proj[8] * m_w - proj[11] * mul1) * dm2[0] + (proj[9] * m_w - proj[11] * mul2) * dm2[1];
        for (int k = 0; k < 3; k++) dmean[k] = dmean[k] + pm[k];
        /* --- SH --- */
        if (shs && !colors && M > 0) {
            float shm[3], tmp[48 * 3];
            float* dsh_i = dL_dsh ? dL_dsh + (size_t)i * M * 3 : tmp;
            sh_bwd_one(D, M, p, campos, shs + (size_t)i * M * 3, o->clamped, dcol, dsh_i, shm);
            for (int k = 0; k < 3; k++) dmean[k] = dmean[k] + shm[k];
        }
        for (int k = 0; k < 3; k++) dL_dmeans3D[3 * i + k] = dmean[k];
        /* --- cov3D -> scale, rotation --- */
        if (!cov3d && scales && rots && dL_dscale && dL_drot)
            cov3d_bwd_one(scales + 3 * i, mod, rots + 4 * i, dcv, dL_dscale + 3 * i, dL_drot + 4 * i);
    }
    long long I = b.I;
    free(acc); free(fout); free(finalT); free(ncon);
    free_bins(&b);
    return I;
}

/* mark_visible: near-plane test only (upstream in_frustum with prefiltered = false) */
void oracle_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

void oracle_mark_visible(int P, const float* means, const float* view, const float* proj, unsigned char* out) {
    (void)proj;
    for (int i = 0; i < P; i++) {
        float pv[3];
        xf43(view, means + 3 * i, pv);
        out[i] = !(pv[2] <= 0.2f);
    }
}

/* simple-knn distCUDA2 restatement: mean of the squared distances to the 3 nearest other points
 * (brute force O(P^2); test sizes only).  Ref call site: scene/gaussian_model.py:134-135. */
void oracle_knn_mean_dist2(int P, const float* pts, float* out) {
    for (int i = 0; i < P; i++) {
        float best[3] = {INFINITY, INFINITY, INFINITY};
        for (int j = 0; j < P; j++) {
            if (j == i) continue;
            float dx = pts[3 * j] - pts[3 * i], dy = pts[3 * j + 1] - pts[3 * i + 1], dz = pts[3 * j + 2] - pts[3 * i + 2];
            float d = dx * dx + dy * dy + dz * dz;
            if (d < best[2]) {
                if (d < best[1]) {
                    best[2] = best[1];
                    if (d < best[0]) { best[1] = best[0]; best[0] = d; }
                    else best[1] = d;
                } else best[2] = d;
            }
        }
        out[i] = (best[0] + best[1] + best[2]) / 3.0f;
    }
}
