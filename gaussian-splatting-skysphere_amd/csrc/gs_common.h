// gs_common.h -- shared device helpers for the MI355X (gfx950, CDNA4) Gaussian rasterizer.
//
// Numerics contract: fp32, no implicit contraction (-ffp-contract=off),
// every FMA explicit, fixed left-to-right operation order.  The CPU oracle (oracle/gs_oracle.c)
// is an independent restatement of the same spec; the two agree bit-for-bit on every
// per-Gaussian and per-pixel value of the forward pass, so every threshold decision of the
// compositing loop (alpha < 1/255, T < 1e-4, power > 0) is identical on both sides.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GS_TILE 16
#define GS_BLOCK 256  // pixels per tile = threads per render workgroup = 4 wave64
#define GS_WAVE 64

namespace gs {

// Workgroup barrier that first drains this wave's LDS operations (s_waitcnt lgkmcnt(0)).
// __syncthreads() is a workgroup-scope release fence + s_barrier, and the gfx950 compiler may
// leave the release's lgkmcnt(0) wait out (its memory model takes LDS operations of all waves as
// totally ordered).  Measured on MI355X: the backward's flush, reading the partner wave's LDS
// accumulators right after the barrier, missed that wave's last ds_write about once per few
// thousand tiles when two processes shared the GPU (C4 ring views: dcolor / dmean2D of 1-5
// Gaussians differed run to run), and in single-process runs more rarely.  Every barrier that
// orders LDS writes of one wave before reads of another goes through here.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// launch tracing (gs_api.cpp): error capture after every launch, optional per-launch sync
// (settings.debug) and optional HIP-event timing per kernel name (bench / profiling).
// ------------------------------------------------------------------------------------------
void trace_begin(const char* name, hipStream_t st);
void trace_end(const char* name, hipStream_t st);
// the set of kernels launched since load (GSRAST_LAUNCH_LOG=1 / gs_debug_launch_log; tests list it
// against the code object's kernels)
void launch_record(const void* kernel_handle);
// a host-side error of the current call (the message lands in gs_last_error; the call fails)
void host_error(const char* msg);

#define GS_LAUNCH(name, kern, grid, block, shm, st, ...)              \
  do {                                                                \
    ::gs::trace_begin(name, st);                                      \
    ::gs::launch_record(reinterpret_cast<const void*>(kern));         \
    hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__);      \
    ::gs::trace_end(name, st);                                        \
  } while (0)

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C20 = 1.0925484305920792f, SH_C21 = -1.0925484305920792f, SH_C22 = 0.31539156525252005f,
                SH_C23 = -1.0925484305920792f, SH_C24 = 0.5462742152960396f;
constexpr float SH_C30 = -0.5900435899266435f, SH_C31 = 2.890611442640554f, SH_C32 = -0.4570457994644658f,
                SH_C33 = 0.3731763325901154f, SH_C34 = -0.4570457994644658f, SH_C35 = 1.445305721320277f,
                SH_C36 = -0.5900435899266435f;

// exp(x) of the splat falloff (x = power <= 0) as 2^t, t = x log2(e) rounded: rndne, one sub,
// a degree-6 minimax polynomial for 2^(t - n) on [-0.5, 0.5] and v_ldexp_f32 -- correctly rounded
// IEEE ops only, so the CPU oracle reproduces it bit-for-bit (oracle/gs_oracle.c:oracle_exp).
// Relative error <= 5.1e-7 on [-8, 0].  Branch-free: x is clamped to [-80, 0] (below -80 the
// result, <= 2e-35, only meets `alpha < 1/255` or a zero weight; results stay normal floats).
// The hardware v_exp_f32 is not used: it is not correctly rounded (measured: 2.2 % of the floats
// in [-126, 0] differ by 1 ulp from round(2^x); tools/probes/exp2_probe.hip), so no CPU
// restatement could reproduce the threshold decisions that depend on it.
__device__ __forceinline__ float gs_exp2(float t) {
  t = fminf(fmaxf(t, -125.0f), 0.0f);
  const float n = __builtin_rintf(t);
  const float f = t - n;
  float p = 1.5345810970757157e-4f;
  p = __builtin_fmaf(p, f, 1.3399930903688073e-3f);
  p = __builtin_fmaf(p, f, 9.618489071726799e-3f);
  p = __builtin_fmaf(p, f, 5.550328642129898e-2f);
  p = __builtin_fmaf(p, f, 2.4022646248340607e-1f);
  p = __builtin_fmaf(p, f, 6.931471824645996e-1f);
  p = __builtin_fmaf(p, f, 1.0f);
  return __builtin_ldexpf(p, (int)n);
}
__device__ __forceinline__ float gs_exp(float x) { return gs_exp2(x * 1.44269504088896341f); }

// Packed (two-pixel) form of gs_exp2: identical op sequence per element, so each element is
// bit-identical to gs_exp2; mul/fma/add issue as v_pk_*_f32.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 gs_exp2_pk(f2 t) {
  t.x = fminf(fmaxf(t.x, -125.0f), 0.0f);
  t.y = fminf(fmaxf(t.y, -125.0f), 0.0f);
  f2 n;
  n.x = __builtin_rintf(t.x);
  n.y = __builtin_rintf(t.y);
  const f2 f = t - n;
  f2 p = (f2)(1.5345810970757157e-4f);
  p = pk_fma(p, f, (f2)(1.3399930903688073e-3f));
  p = pk_fma(p, f, (f2)(9.618489071726799e-3f));
  p = pk_fma(p, f, (f2)(5.550328642129898e-2f));
  p = pk_fma(p, f, (f2)(2.4022646248340607e-1f));
  p = pk_fma(p, f, (f2)(6.931471824645996e-1f));
  p = pk_fma(p, f, (f2)(1.0f));
  f2 r;
  r.x = __builtin_ldexpf(p.x, (int)n.x);
  r.y = __builtin_ldexpf(p.y, (int)n.y);
  return r;
}

// Render-loop exp2 by numerics mode (gs_set_exact_exp): EXACT = the deterministic polynomial above,
// mirrored by the CPU oracle (bit-exact forward); otherwise the hardware v_exp_f32 (<= 1 ulp, not
// reproducible on the CPU), 11 -> 1 VALU ops per evaluation.  Same clamp to [-125, 0] in both.
template <bool EXACT>
__device__ __forceinline__ float exp2_m(float t) {
  if constexpr (EXACT) return gs_exp2(t);
  // fast mode: the hardware exp2 without the exact mode's clamp to [-125, 0] (t > 0 only occurs
  // by rounding next to a splat centre and such an entry is skipped (power > 0); below -125 the
  // result only ever meets alpha < 1/255)
  else return __builtin_amdgcn_exp2f(t);
}
template <bool EXACT>
__device__ __forceinline__ f2 exp2_pk_m(f2 t) {
  if constexpr (EXACT) return gs_exp2_pk(t);
  else {
    f2 r;
    r.x = exp2_m<false>(t.x);
    r.y = exp2_m<false>(t.y);
    return r;
  }
}

// log2(e) * power of a splat at pixel offset (dx, dy) = mean - pixel.  The conic is scaled once
// per staged splat (fall_coefs): A = cxx (-log2e / 2), B = cxy (-log2e), C = cyy (-log2e / 2), and
// t = (A dx) dx + dy (B dx + C dy): three multiplies + two FMAs per pixel, and for the backward's
// two pixels of one column (same dx) the three multiplies are shared, so the pair costs two
// packed FMAs.  Bit-identical to oracle/gs_oracle.c:falloff_log2.
constexpr float K_HALF_LOG2E = -0.72134752044448170f, K_LOG2E = -1.44269504088896341f;
__device__ __forceinline__ float4 fall_coefs(float cxx, float cxy, float cyy, float opacity) {
  return make_float4(cxx * K_HALF_LOG2E, cxy * K_LOG2E, cyy * K_HALF_LOG2E, opacity);
}
__device__ __forceinline__ float falloff_log2(float4 k, float dx, float dy) {
  const float a2 = (k.x * dx) * dx;
  const float b = k.y * dx;
  const float t = __builtin_fmaf(k.z, dy, b);
  return __builtin_fmaf(dy, t, a2);
}
// By numerics mode (gs_set_exact_exp).  EXACT: as above, alpha = min(0.99, o 2^t) with the oracle's
// operation order.  Fast: the opacity enters the exponent -- the staged fourth coefficient is
// log2(o) (v_log_f32; -inf for o = 0) and the first product becomes an FMA with it, so
// alpha = min(0.99, 2^(t + log2 o)) costs no multiply per pixel (the forward's walk and the
// backward's slots evaluate the same expression, so their per-entry decisions agree; the fast
// mode's deviation from o 2^t stays below the oracle's near-threshold margins, relative < 1e-6 of
// alpha where it can decide).
template <bool EXACT>
__device__ __forceinline__ float4 fall_coefs_m(float cxx, float cxy, float cyy, float opacity) {
  return make_float4(cxx * K_HALF_LOG2E, cxy * K_LOG2E, cyy * K_HALF_LOG2E,
                     EXACT ? opacity : __builtin_amdgcn_logf(opacity));
}
template <bool EXACT>
__device__ __forceinline__ float falloff_log2_m(float4 k, float dx, float dy) {
  if constexpr (EXACT) return falloff_log2(k, dx, dy);
  const float a2 = __builtin_fmaf(k.x * dx, dx, k.w);
  const float b = k.y * dx;
  const float t = __builtin_fmaf(k.z, dy, b);
  return __builtin_fmaf(dy, t, a2);
}
// o G = o 2^t from the exponent falloff_log2_m returned (fast: the opacity is already in it)
template <bool EXACT>
__device__ __forceinline__ float opac_gauss(float4 k, float t) {
  if constexpr (EXACT) return k.w * exp2_m<true>(t);
  else return exp2_m<false>(t);
}

// m = 4x4 world_view_transform / full_proj_transform, row-major flattening of the torch tensor
// (row-vector convention: translation in row 3; /root/reference/scene/cameras.py:54-56).
struct float3v { float x, y, z; };

__device__ __forceinline__ float3v xf43(const float* m, float px, float py, float pz) {
  float3v o;
  o.x = m[0] * px + m[4] * py + m[8] * pz + m[12];
  o.y = m[1] * px + m[5] * py + m[9] * pz + m[13];
  o.z = m[2] * px + m[6] * py + m[10] * pz + m[14];
  return o;
}
__device__ __forceinline__ float xf44w(const float* m, float px, float py, float pz) {
  return m[3] * px + m[7] * py + m[11] * pz + m[15];
}

__device__ __forceinline__ float ndc2pix(float v, int S) {
  return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

// tile rectangle [rmin, rmax) touched by a splat of integer radius r centred at (x, y) (pixels)
__device__ __forceinline__ void get_rect(float x, float y, int r, int gx, int gy, int& x0, int& y0, int& x1,
                                         int& y1) {
  float fr = (float)r;
  x0 = min(gx, max(0, (int)((x - fr) / 16.0f)));
  y0 = min(gy, max(0, (int)((y - fr) / 16.0f)));
  x1 = min(gx, max(0, (int)((((x + fr) + 16.0f) - 1.0f) / 16.0f)));
  y1 = min(gy, max(0, (int)((((y + fr) + 16.0f) - 1.0f) / 16.0f)));
}

// ln(x) for x >= 1 from correctly rounded IEEE ops only (frexp by bit fields, atanh series),
// |error| < 2e-7 relative; the CPU oracle reproduces it bit-for-bit (oracle_log).  Used for the
// culling limit, which must agree exactly between the binning here and in the oracle.
__device__ __forceinline__ float gs_log(float x) {
  const uint32_t u = __float_as_uint(x);
  int e = (int)((u >> 23) & 255u) - 127;
  float m = __uint_as_float((u & 0x7FFFFFu) | 0x3F800000u);
  if (m > 1.41421356f) {
    m = m * 0.5f;
    e = e + 1;
  }
  const float f = m - 1.0f;
  const float t = f / (2.0f + f);
  const float t2 = t * t;
  float p = 0.11111111f;
  p = __builtin_fmaf(p, t2, 0.14285715f);
  p = __builtin_fmaf(p, t2, 0.2f);
  p = __builtin_fmaf(p, t2, 0.33333334f);
  p = __builtin_fmaf(p, t2, 1.0f);
  return __builtin_fmaf((float)e, 0.69314718f, (2.0f * t) * p);
}
// culling limit of the alpha >= 1/255 ellipse: q(d) <= lim (negative: never reaches 1/255)
__device__ __forceinline__ float cull_lim(float op) {
  return op >= 1.0f / 255.0f ? 2.0f * fmaxf(gs_log(255.0f * op), 0.0f) * 1.001f + 1e-3f : -1.0f;
}

// Block-wide copy of 256 consecutive SH rows (3M floats each) between global memory and an LDS
// array with an odd row stride (3M + 1: conflict-free per-thread row access); dwordx4 global
// accesses when rows are 16-B multiples and the base is aligned.
__device__ __forceinline__ void rows_to_lds(const float* __restrict__ src, float* lds, int n, int rowf, int stride) {
  const int total = n * rowf;
  if ((rowf & 3) == 0 && (((uintptr_t)src) & 15) == 0) {
    for (int q = threadIdx.x; q < (total >> 2); q += 256) {
      const float4 v = reinterpret_cast<const float4*>(src)[q];
      const int e = q << 2, t = e / rowf;
      float* d = lds + t * stride + (e - t * rowf);
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
  } else {
    for (int e = threadIdx.x; e < total; e += 256) {
      const int t = e / rowf;
      lds[t * stride + (e - t * rowf)] = src[e];
    }
  }
}
__device__ __forceinline__ void lds_to_rows(const float* lds, float* __restrict__ dst, int n, int rowf, int stride) {
  const int total = n * rowf;
  if ((rowf & 3) == 0 && (((uintptr_t)dst) & 15) == 0) {
    for (int q = threadIdx.x; q < (total >> 2); q += 256) {
      const int e = q << 2, t = e / rowf;
      const float* d = lds + t * stride + (e - t * rowf);
      reinterpret_cast<float4*>(dst)[q] = make_float4(d[0], d[1], d[2], d[3]);
    }
  } else {
    for (int e = threadIdx.x; e < total; e += 256) {
      const int t = e / rowf;
      dst[e] = lds[t * stride + (e - t * rowf)];
    }
  }
}

// Tile-exact binning.  A splat is binned only into the tiles of its upstream rectangle whose
// 16x16 pixel square can hold a pixel with alpha >= 1/255, i.e. q(d) <= lim for the conic q and the
// culling limit lim (splat record).  Per tile row the x-extent of the ellipse over the row's pixel
// band is closed-form (x_r(dy) is concave, x_l(dy) convex: their extrema over the band sit at the
// clamp of the ellipse's extreme-x points), widened by margins, so the test is conservative: a
// dropped (splat, tile) pair contributes alpha < 1/255 to every pixel of the tile and is skipped
// by the compositing anyway.  Images and gradients are unchanged; the instance count drops
// (C3: 6.58M -> 4.3M).  The op sequence is mirrored bit-for-bit by oracle/gs_oracle.c:row_span.
struct SpanCtx {
  float mx, my, A, B, det, R, dyr, AL;
  int x0, x1, mode;  // mode 0: ellipse, 1: whole rectangle row (degenerate conic), 2: nothing
};
__device__ __forceinline__ SpanCtx span_ctx(float mx, float my, float A, float B, float C, float L, int x0, int x1) {
  SpanCtx s;
  s.mx = mx;
  s.my = my;
  s.A = A;
  s.B = B;
  s.x0 = x0;
  s.x1 = x1;
  s.det = A * C - B * B;
  s.mode = !(L >= 0.0f) ? 2 : ((A > 0.0f && C > 0.0f && s.det > 0.0f) ? 0 : 1);
  s.R = 0.0f;
  s.dyr = 0.0f;
  s.AL = 0.0f;
  if (s.mode == 0) {
    s.AL = A * L;
    s.R = sqrtf(s.AL / s.det) * 1.0001f + 0.01f;
    s.dyr = -B * sqrtf(L / (C * s.det));
  }
  return s;
}
// tiles [ta, tb) of tile row ty (empty: ta == tb)
__device__ __forceinline__ void row_span(const SpanCtx& s, int ty, int& ta, int& tb) {
  ta = tb = s.x0;
  if (s.mode == 2) return;
  if (s.mode == 1) {
    tb = s.x1;
    return;
  }
  const float lo = fmaxf((float)(GS_TILE * ty) - s.my, -s.R);
  const float hi = fminf((float)(GS_TILE * ty + GS_TILE - 1) - s.my, s.R);
  if (!(lo <= hi)) return;
  const float d1 = fminf(fmaxf(s.dyr, lo), hi), d2 = fminf(fmaxf(-s.dyr, lo), hi);
  const float xr = (-s.B * d1 + sqrtf(fmaxf(s.AL - s.det * d1 * d1, 0.0f))) / s.A;
  const float xl = (-s.B * d2 - sqrtf(fmaxf(s.AL - s.det * d2 * d2, 0.0f))) / s.A;
  const float X0 = fmaxf((s.mx + xl) - (0.05f + 0.001f * fabsf(xl)), -1.0e6f);
  const float X1 = fminf((s.mx + xr) + (0.05f + 0.001f * fabsf(xr)), 1.0e6f);
  const int a = max(s.x0, (int)ceilf((X0 - 15.0f) / 16.0f));
  const int b = min(s.x1, (int)floorf(X1 / 16.0f) + 1);
  ta = a;
  tb = b > a ? b : a;
}

// rotation of the (w, x, y, z) quaternion, un-normalised (the caller normalises:
// /root/reference/scene/gaussian_model.py:41,100-101)
struct mat3 { float m[3][3]; };
__device__ __forceinline__ mat3 quat_rot(float r, float x, float y, float z) {
  mat3 R;
  R.m[0][0] = 1.f - 2.f * (y * y + z * z);
  R.m[0][1] = 2.f * (x * y - r * z);
  R.m[0][2] = 2.f * (x * z + r * y);
  R.m[1][0] = 2.f * (x * y + r * z);
  R.m[1][1] = 1.f - 2.f * (x * x + z * z);
  R.m[1][2] = 2.f * (y * z - r * x);
  R.m[2][0] = 2.f * (x * z - r * y);
  R.m[2][1] = 2.f * (y * z + r * x);
  R.m[2][2] = 1.f - 2.f * (x * x + y * y);
  return R;
}

// cov3D 6-vector (xx, xy, xz, yy, yz, zz) of R diag(mod*s)^2 R^T
__device__ __forceinline__ void cov3d(float sx, float sy, float sz, float mod, float qr, float qx, float qy,
                                      float qz, float* cov) {
  mat3 R = quat_rot(qr, qx, qy, qz);
  float sv[3] = {mod * sx, mod * sy, mod * sz};
  float m[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int a = 0; a < 3; a++) m[i][a] = sv[i] * R.m[a][i];
#define GS_SIG(a, b) (m[0][a] * m[0][b] + m[1][a] * m[1][b] + m[2][a] * m[2][b])
  cov[0] = GS_SIG(0, 0);
  cov[1] = GS_SIG(0, 1);
  cov[2] = GS_SIG(0, 2);
  cov[3] = GS_SIG(1, 1);
  cov[4] = GS_SIG(1, 2);
  cov[5] = GS_SIG(2, 2);
#undef GS_SIG
}

// EWA 2D covariance: returns (a, b, c) with the 0.3 low-pass dilation, plus the 2x3 Jacobian
// product T = J Rw and the view-space point (clamped x, y).
struct Cov2D {
  float a, b, c;
  float T[2][3];
  float tx, ty, tz;
  float gmx, gmy;  // 0 where the tx/tz (ty/tz) frustum clamp was active
};

__device__ __forceinline__ Cov2D cov2d(const float* view, float px, float py, float pz, const float* cov3,
                                       float fx, float fy, float tanfovx, float tanfovy) {
  Cov2D o;
  float3v t = xf43(view, px, py, pz);
  float limx = 1.3f * tanfovx, limy = 1.3f * tanfovy;
  float txtz = t.x / t.z, tytz = t.y / t.z;
  float cx = fminf(limx, fmaxf(-limx, txtz)), cy = fminf(limy, fmaxf(-limy, tytz));
  o.gmx = (txtz < -limx || txtz > limx) ? 0.0f : 1.0f;
  o.gmy = (tytz < -limy || tytz > limy) ? 0.0f : 1.0f;
  t.x = cx * t.z;
  t.y = cy * t.z;
  float tz2 = t.z * t.z;
  float J00 = fx / t.z, J02 = -(fx * t.x) / tz2;
  float J11 = fy / t.z, J12 = -(fy * t.y) / tz2;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    o.T[0][r] = view[4 * r + 0] * J00 + view[4 * r + 2] * J02;
    o.T[1][r] = view[4 * r + 1] * J11 + view[4 * r + 2] * J12;
  }
  float V[3][3] = {{cov3[0], cov3[1], cov3[2]}, {cov3[1], cov3[3], cov3[4]}, {cov3[2], cov3[4], cov3[5]}};
  float U[2][3];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int b = 0; b < 3; b++) U[i][b] = o.T[i][0] * V[0][b] + o.T[i][1] * V[1][b] + o.T[i][2] * V[2][b];
  float c00 = U[0][0] * o.T[0][0] + U[0][1] * o.T[0][1] + U[0][2] * o.T[0][2];
  float c01 = U[0][0] * o.T[1][0] + U[0][1] * o.T[1][1] + U[0][2] * o.T[1][2];
  float c11 = U[1][0] * o.T[1][0] + U[1][1] * o.T[1][1] + U[1][2] * o.T[1][2];
  o.a = c00 + 0.3f;
  o.b = c01;
  o.c = c11 + 0.3f;
  o.tx = t.x;
  o.ty = t.y;
  o.tz = t.z;
  return o;
}

// ------------------------------------------------------------------------------------------
// wave64 helpers (CDNA: 64-lane wavefront, 64-bit ballots)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  uint32_t l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// DPP move helpers (gfx9 encodings: quad_perm, row_half_mirror, row_mirror, row_bcast15/31)
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF, bool BOUND_CTRL = false>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, BANK_MASK, BOUND_CTRL));
}

// Sum over the 64 lanes; the full sum lands in lane 63 (other lanes hold partials).
// Inactive lanes must hold 0 (callers keep EXEC full and zero non-contributors).
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
  v = v + dpp_f<0xB1>(v);        // quad_perm [1,0,3,2]
  v = v + dpp_f<0x4E>(v);        // quad_perm [2,3,0,1]
  v = v + dpp_f<0x141>(v);       // row_half_mirror
  v = v + dpp_f<0x140>(v);       // row_mirror: every lane holds its row-of-16 sum
  v = v + dpp_f<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v = v + dpp_f<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Nine independent 64-lane sums, interleaved step by step so consecutive DPP ops never read a
// VGPR written by the instruction just before (no s_nop wait states); totals land in lane 63.
template <int N>
__device__ __forceinline__ void wave_sumN_to_lane63(float* v) {
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0xB1>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x4E>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x141>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x140>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x142, 0xA>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x143, 0xC>(v[k]);
}
__device__ __forceinline__ void wave_sum9_to_lane63(float* v) { wave_sumN_to_lane63<9>(v); }

// Row (16-lane) sums of N values: after this every lane of a row holds its row's sum.
template <int N>
__device__ __forceinline__ void row_sumN(float* v) {
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0xB1>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x4E>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x141>(v[k]);
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = v[k] + dpp_f<0x140>(v[k]);
}

// Wave sums of nine values with half-wave / row transposes: v_permlane32_swap and
// v_permlane16_swap exchange halves of two registers so that one add halves the lane count of
// two values at once.  On return row r (lanes 16r..16r+15) of d0 holds the 64-lane sum of s[r],
// of d1 that of s[4 + r], and of d8 the sum of s[8] over row r only (the four row values add up
// to the total of s[8]).  Every lane of a row holds its row's value.
__device__ __forceinline__ float swap32_add(float a, float b) {
  // lanes 0-31: a[l] + a[l + 32]; lanes 32-63: b[l - 32] + b[l]
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_add(float a, float b) {
  // row pairs (0,1) and (2,3): rows 0 / 2 get a's, rows 1 / 3 get b's two-row sums
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ void wave_sum9_rows(const float* s, float& d0, float& d1, float& d8) {
  const float c0 = swap32_add(s[0], s[2]), c1 = swap32_add(s[1], s[3]);
  const float c2 = swap32_add(s[4], s[6]), c3 = swap32_add(s[5], s[7]);
  float v[3] = {swap16_add(c0, c1), swap16_add(c2, c3), s[8]};
  row_sumN<3>(v);
  d0 = v[0];
  d1 = v[1];
  d8 = v[2];
}

// Nine wave sums down to 8-lane groups, with a half-row transpose after the swaps: on return
// lanes 16 r + 8 h .. + 7 (r < 4, h < 2) hold in d the 64-lane sum of s[r + 4 h] and in d8 the sum
// of s[8] over that 8-lane group of the swapped layout (the eight group values add up to the
// total).  The transpose (two selects and one row_ror:8 add) halves two values at once, so d needs
// three more DPP steps instead of 2 x 4, and d8 stops at 8-lane sums.  hi: lane bit 3.
__device__ __forceinline__ void wave_sum9_halfrows(const float* s, bool hi, float& d, float& d8) {
  const float c0 = swap32_add(s[0], s[2]), c1 = swap32_add(s[1], s[3]);
  const float c2 = swap32_add(s[4], s[6]), c3 = swap32_add(s[5], s[7]);
  const float a = swap16_add(c0, c1), b = swap16_add(c2, c3);
  // lanes 0-7 of a row keep a (plus lane + 8's a), lanes 8-15 keep b (plus lane - 8's b)
  const float keep = hi ? b : a, send = hi ? a : b;
  float v[2] = {keep + dpp_f<0x128>(send), s[8]};  // row_ror:8
#pragma unroll
  for (int k = 0; k < 2; k++) v[k] = v[k] + dpp_f<0xB1>(v[k]);
#pragma unroll
  for (int k = 0; k < 2; k++) v[k] = v[k] + dpp_f<0x4E>(v[k]);
#pragma unroll
  for (int k = 0; k < 2; k++) v[k] = v[k] + dpp_f<0x141>(v[k]);
  d = v[0];
  d8 = v[1];
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ float readlane63(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// ------------------------------------------------------------------------------------------
// render tiling: a 16x16 tile is split into per-wave pixel rectangles (8x8 quadrants in the
// forward, 8x16 halves in the backward).  Each staged batch entry carries a mask of the
// rectangles its alpha >= 1/255 ellipse can reach; a wave walks only its entries (scalar loop).
// ------------------------------------------------------------------------------------------
struct QuadPix {
  int px, py;
};
__device__ __forceinline__ QuadPix quad_pixel(int tx, int ty, int wid, int lane) {
  QuadPix q;
  q.px = tx * GS_TILE + 8 * (wid & 1) + (lane & 7);
  q.py = ty * GS_TILE + 8 * (wid >> 1) + (lane >> 3);
  return q;
}

// Conservative culling of (splat, pixel-rectangle) pairs.  A pixel p can only contribute if
// alpha >= 1/255, i.e. q(p - m) <= 2 ln(255 o) with q(d) = cxx dx^2 + 2 cxy dx dy + cyy dy^2
// (power = -q/2).  preprocess stores lim = 2 ln(255 o) (1 + 1e-3) + 1e-3 (or -1 when o < 1/255);
// the minimum of q over the rectangle of pixel centres is compared with lim.  The margins absorb
// rounding, so a culled pair never contributes: results are unchanged, only work is skipped.
//
// The minimum (convex quadratic, minimum at d = 0): 0 when the centre lies in the rectangle, else
// on an edge that faces the centre (at a constrained minimum d* on edge x = e the KKT multiplier
// mu >= 0 with grad q(d*) = (mu, 0) and convexity give mu (0 - e) < 0, so e > 0 for the low edge
// -- the centre lies beyond it).  So per axis ONE edge is evaluated: the facing one when the centre
// lies outside that axis's range, and otherwise an arbitrary one, harmless since any point of the
// rectangle is >= the minimum.  On the edge x = e the 1-D minimiser dy = -cxy e / cyy is clamped to
// the edge; rcp for 1 / cyy (the minimiser only needs to be close: q is flat there, second order).
__device__ __forceinline__ float q_form(float cx, float cy2, float cz, float dx, float dy) {
  return __builtin_fmaf(dx, __builtin_fmaf(cx, dx, cy2 * dy), (cz * dy) * dy);
}

struct EllipseCull {
  float cx, cy2, cz, kx, ky;  // conic (cxy doubled), edge minimiser slopes -cxy / cxx, -cxy / cyy
  bool degenerate;            // not positive definite on the axes: never culled
};
__device__ __forceinline__ EllipseCull ellipse_cull(float cx, float cy, float cz) {
  EllipseCull e;
  e.cx = cx, e.cy2 = 2.0f * cy, e.cz = cz;
  e.degenerate = !(cx > 0.0f && cz > 0.0f);
  e.kx = -cy * __builtin_amdgcn_rcpf(cx);
  e.ky = -cy * __builtin_amdgcn_rcpf(cz);
  return e;
}
// min of q over [dxl, dxh] x [dyl, dyh] (offsets from the centre) <= lim; the centre-inside case
// is the caller's (q = 0 there)
__device__ __forceinline__ bool rect_min_within(const EllipseCull& e, float dxl, float dxh, float dyl, float dyh,
                                                float lim) {
  const float dxe = dxl > 0.0f ? dxl : dxh, dye = dyl > 0.0f ? dyl : dyh;
  const float a = q_form(e.cx, e.cy2, e.cz, dxe, fminf(fmaxf(dxe * e.ky, dyl), dyh));
  const float b = q_form(e.cx, e.cy2, e.cz, fminf(fmaxf(dye * e.kx, dxl), dxh), dye);
  return fminf(a, b) <= lim;
}
__device__ __forceinline__ bool ellipse_meets_rect(float mx, float my, float cx, float cy, float cz, float lim,
                                                   float x0, float x1, float y0, float y1) {
  if (!(lim >= 0.0f)) return false;
  const float dxl = x0 - mx, dxh = x1 - mx, dyl = y0 - my, dyh = y1 - my;
  const bool inside = dxl <= 0.0f && dxh >= 0.0f && dyl <= 0.0f && dyh >= 0.0f;
  const EllipseCull e = ellipse_cull(cx, cy, cz);
  return inside || e.degenerate || rect_min_within(e, dxl, dxh, dyl, dyh, lim);
}

// bit w set if the splat can contribute to a pixel of 8x8 quadrant w of tile (tx, ty); the
// column / row offsets and the edge slopes are shared by the four rectangles
__device__ __forceinline__ uint32_t quadrant_mask(float mx, float my, float cx, float cy, float cz, float lim, int tx,
                                                  int ty) {
  if (!(lim >= 0.0f)) return 0u;
  const float x0 = (float)(tx * GS_TILE), y0 = (float)(ty * GS_TILE);
  const EllipseCull e = ellipse_cull(cx, cy, cz);
  if (e.degenerate) return 0xFu;
  float xl[2], xh[2], yl[2], yh[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    xl[h] = (x0 + 8.0f * h) - mx, xh[h] = (x0 + 8.0f * h + 7.0f) - mx;
    yl[h] = (y0 + 8.0f * h) - my, yh[h] = (y0 + 8.0f * h + 7.0f) - my;
  }
  uint32_t m = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const int c = w & 1, r = w >> 1;
    const bool inside = xl[c] <= 0.0f && xh[c] >= 0.0f && yl[r] <= 0.0f && yh[r] >= 0.0f;
    m |= (inside || rect_min_within(e, xl[c], xh[c], yl[r], yh[r], lim)) ? (1u << w) : 0u;
  }
  return m;
}

}  // namespace gs
