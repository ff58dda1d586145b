// gs_loss.hip -- fused SSIM (forward + backward) for the photometric loss of train.py.
//
// Restates /root/reference/utils/loss_utils.py:ssim/_ssim (11x11 Gaussian window, sigma 1.5,
// zero padding 5, C1 = 0.01^2, C2 = 0.03^2, mean of the SSIM map), which the reference evaluates
// as five depthwise conv2d calls plus their autograd backward every iteration
// (train.py:91-92).  Here one kernel produces, per plane (image x channel) and 32x32 tile, the
// five windowed moments by a separable 11-tap filter through LDS, the SSIM map sum (and, for the
// fused photometric loss, the |x - y| sum) and the three per-pixel partials dS/dmu1, dS/dE[x^2],
// dS/dE[xy]; a second kernel filters those partials with the same window (the adjoint of a
// symmetric, zero-padded correlation) and forms dL/dimg1 (fused loss: plus the L1 term).
// 1080p x 3 planes: fwd 64 us, bwd 52 us (round 1's 16x16 tiles without register reuse: 103 / 79).
//
//   S = (2 m1 m2 + C1)(2 s12 + C2) / ((m1^2 + m2^2 + C1)(s11 + s22 + C2)),
//   s11 = E[x^2] - m1^2, s22 = E[y^2] - m2^2, s12 = E[xy] - m1 m2
//   dS/dm1 = 2 m2 (A2 - A1) / (B1 B2) - 2 m1 S (1/B1 - 1/B2),  dS/dE[x^2] = -S / B2,
//   dS/dE[xy] = 2 A1 / (B1 B2)
//   dL/dx(q) = scale * [ (w * dS/dm1)(q) + 2 x(q) (w * dS/dE[x^2])(q) + y(q) (w * dS/dE[xy])(q) ]
//
// The sums are reduced per workgroup and then per plane (or over all planes, k_loss_finish) in a
// fixed order (deterministic).
#include "gs_internal.h"

namespace gs {

// 32x32 output tiles, 256 (forward) / 384 (backward) threads.  The window is applied as two 1-D passes through LDS with
// register reuse: the horizontal pass gives each thread 4 adjacent outputs of one row (16 inputs
// read as four 16-B LDS loads, products formed once per input), the vertical pass 4 adjacent
// outputs of one column (14 row values per moment).  Row strides are chosen for conflict-free
// 16-B accesses over 16 consecutive rows (44, 36 = 4 x odd) and for the two half-waves of the
// vertical pass to read disjoint bank halves (rows 8 apart: 8 x 36 = 288 = 32 mod 64).
constexpr int SS_T = 32;                 // output tile
constexpr int SS_R = 5;                  // window radius
constexpr int SS_IN = SS_T + 2 * SS_R;   // 42: input rows / columns with halo
constexpr int SS_LI = 44;                // input row stride (floats)
constexpr int SS_LH = 36;                // horizontal-result row stride (floats)
constexpr int SS_HG = SS_IN * (SS_T / 4);  // 336 horizontal groups of 4 outputs
static_assert(SS_LI >= 4 * (SS_T / 4 - 1) + 16, "the last group's 16-B loads stay in the row");
constexpr int SS_FWD_LDS = 2 * SS_IN * SS_LI > 5 * SS_IN * SS_LH ? 2 * SS_IN * SS_LI : 5 * SS_IN * SS_LH;
constexpr int SS_BWD_LDS = 3 * SS_IN * SS_LI > 3 * SS_IN * SS_LH ? 3 * SS_IN * SS_LI : 3 * SS_IN * SS_LH;

struct SsimWin {
  float w[2 * SS_R + 1];
};

// stage a 42x42 halo tile of NP planes (zero outside the image: conv2d's padding).  Every load of
// the thread is issued before the first LDS store, so the 7 x NP global loads are in flight
// together (a load -> store loop waits out one memory latency per element).
// The backward runs SS_BWD_NT = 384 threads (6 waves): one horizontal group per thread (336), the
// first four waves take the vertical pass (53.1 -> 51.8 us at 1080p x 3, with the image loads
// issued at the start).  The forward keeps 256 (two groups for the first two waves): its vertical
// pass and epilogue are the long phase, and at 6 waves per workgroup (88 VGPRs) only 3 workgroups
// share a CU in it against 4 -- measured 63.8 -> 73.4 us; nor did its moments 0-1 stored early
// (102 VGPRs: 62.5-65.8 -> 65.0-66.1 us) or that at 5 waves per SIMD by attribute (36 B of
// spills: 68.9-73.9 us) pay.
constexpr int SS_BWD_NT = 384;
static_assert(SS_HG <= SS_BWD_NT && SS_BWD_NT % 64 == 0, "one horizontal group per thread");
template <int NP, int NT>
__device__ __forceinline__ void stage_tiles(float (*dst)[SS_IN][SS_LI], const float* const* src, int H, int W, int y0,
                                            int x0) {
  constexpr int NS = (SS_IN * SS_IN + NT - 1) / NT;  // elements per thread and plane: 7 (256), 5 (384)
  float v[NP][NS];
  int rr[NS], cc[NS];
#pragma unroll
  for (int q = 0; q < NS; q++) {
    const int i = threadIdx.x + NT * q;
    rr[q] = i / SS_IN;
    cc[q] = i - rr[q] * SS_IN;
    const int y = y0 - SS_R + rr[q], x = x0 - SS_R + cc[q];
    const bool ok = i < SS_IN * SS_IN && y >= 0 && y < H && x >= 0 && x < W;
#pragma unroll
    for (int p = 0; p < NP; p++) v[p][q] = ok ? src[p][(size_t)y * W + x] : 0.0f;
  }
#pragma unroll
  for (int q = 0; q < NS; q++)
    if (threadIdx.x + NT * q < SS_IN * SS_IN)
#pragma unroll
      for (int p = 0; p < NP; p++) dst[p][rr[q]][cc[q]] = v[p][q];
}

__device__ __forceinline__ void ld16(const float* row, float* v) {
  // 16-B aligned (row strides and c0 are multiples of 4 floats): one ds_read_b128 per quarter.
  // The empty asm keeps each 16-B load whole: otherwise the loads shrink to the used elements and
  // are re-paired as ds_read2_b64 across the 16-B slots, which banks on (a/4) mod 32 and conflicts
  // 2-way over the 16 rows a lane group reads.
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f* r4 = reinterpret_cast<const v4f*>(row);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    v4f t = r4[q];
    asm volatile("" : "+v"(t));
    v[4 * q] = t.x, v[4 * q + 1] = t.y, v[4 * q + 2] = t.z, v[4 * q + 3] = t.w;
  }
}

// vertical-pass thread mapping: column c, output rows 4 j .. 4 j + 3; the two half-waves of
// wave w take row groups 8 rows apart (w = 0: 0 / 2, 1: 1 / 3, 2: 4 / 6, 3: 5 / 7)
__device__ __forceinline__ void vmap(int tid, int& c, int& j) {
  const int w = tid >> 6, half = (tid >> 5) & 1;
  c = tid & 31;
  j = (w & 1) + 4 * (w >> 1) + 2 * half;
}

__global__ __launch_bounds__(256) void k_ssim_fwd(int H, int W, SsimWin win, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, float* __restrict__ dmaps,
                                                  float* __restrict__ partial, float* __restrict__ partial_l1) {
  // one LDS block: the staged image pair, then (after the horizontal pass has read it into
  // registers) the five horizontally filtered moments -- 30 KB, 5 workgroups per CU
  __shared__ __attribute__((aligned(16))) float s_lds[SS_FWD_LDS];
  __shared__ float s_red[2][4];
  float(*sxy)[SS_IN][SS_LI] = reinterpret_cast<float(*)[SS_IN][SS_LI]>(s_lds);
  float(*sh)[SS_IN][SS_LH] = reinterpret_cast<float(*)[SS_IN][SS_LH]>(s_lds);
  const int plane = blockIdx.z;
  const int x0 = blockIdx.x * SS_T, y0 = blockIdx.y * SS_T;
  const size_t HW = (size_t)H * W;
  const int tid = threadIdx.x;
  {
    const float* src[2] = {img1 + plane * HW, img2 + plane * HW};
    stage_tiles<2, 256>(sxy, src, H, W, y0, x0);
  }
  lds_barrier();
  // horizontal pass: group g -> row g % 42, outputs 4 (g / 42) .. + 3 (consecutive lanes, consecutive
  // rows); a thread's groups are tid and tid + 256.  The L1 term |x - y| of the tile's pixels is
  // summed here too, from the groups' centre values.
  float o[2][5][4];
  float l = 0.f;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int g = tid + 256 * h;
    if (g >= SS_HG) break;
    const int r = g % SS_IN, c0 = 4 * (g / SS_IN);
    float x[16], y[16];
    ld16(&sxy[0][r][c0], x);
    ld16(&sxy[1][r][c0], y);
#pragma unroll
    for (int m = 0; m < 5; m++)
#pragma unroll
      for (int i = 0; i < 4; i++) o[h][m][i] = 0.f;
#pragma unroll
    for (int q = 0; q < 14; q++) {
      const float xx = x[q] * x[q], yy = y[q] * y[q], xy = x[q] * y[q];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int k = q - i;
        if (k < 0 || k > 2 * SS_R) continue;
        const float wk = win.w[k];
        o[h][0][i] = __builtin_fmaf(wk, x[q], o[h][0][i]);
        o[h][1][i] = __builtin_fmaf(wk, y[q], o[h][1][i]);
        o[h][2][i] = __builtin_fmaf(wk, xx, o[h][2][i]);
        o[h][3][i] = __builtin_fmaf(wk, yy, o[h][3][i]);
        o[h][4][i] = __builtin_fmaf(wk, xy, o[h][4][i]);
      }
    }
    const int py = y0 + r - SS_R;
    if (r >= SS_R && r < SS_R + SS_T && py < H) {
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (x0 + c0 + i < W) l += fabsf(x[i + SS_R] - y[i + SS_R]);
    }
  }
  lds_barrier();  // every thread has read the staged pair: the moments go over it
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int g = tid + 256 * h;
    if (g >= SS_HG) break;
    const int r = g % SS_IN, c0 = 4 * (g / SS_IN);
#pragma unroll
    for (int m = 0; m < 5; m++)
      *reinterpret_cast<float4*>(&sh[m][r][c0]) = make_float4(o[h][m][0], o[h][m][1], o[h][m][2], o[h][m][3]);
  }
  lds_barrier();
  int c, j;
  vmap(tid, c, j);
  float mo[5][4];
#pragma unroll
  for (int m = 0; m < 5; m++) {
    float v[14];
#pragma unroll
    for (int q = 0; q < 14; q++) v[q] = sh[m][4 * j + q][c];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 2 * SS_R + 1; k++) a = __builtin_fmaf(win.w[k], v[i + k], a);
      mo[m][i] = a;
    }
  }
  const float C1 = 1e-4f, C2 = 9e-4f;  // 0.01 ** 2, 0.03 ** 2 as the float32 tensor ops see them
  const size_t PHW = (size_t)gridDim.z * HW;
  const int px = x0 + c;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const float m1 = mo[0][i], m2 = mo[1][i], e11 = mo[2][i], e22 = mo[3][i], e12 = mo[4][i];
    const float mu12 = m1 * m2;
    const float A1 = 2.f * mu12 + C1, A2 = 2.f * (e12 - mu12) + C2;
    const float B1 = m1 * m1 + m2 * m2 + C1, B2 = (e11 - m1 * m1) + (e22 - m2 * m2) + C2;
    const float iB1 = 1.f / B1, iB2 = 1.f / B2, iB = iB1 * iB2;
    const float S = A1 * A2 * iB;
    const int py = y0 + 4 * j + i;
    if (px < W && py < H) {
      const size_t o = plane * HW + (size_t)py * W + px;
      dmaps[o] = 2.f * m2 * (A2 - A1) * iB - 2.f * m1 * S * (iB1 - iB2);  // dS/dm1
      dmaps[PHW + o] = -S * iB2;                                          // dS/dE[x^2]
      dmaps[2 * PHW + o] = 2.f * A1 * iB;                                 // dS/dE[xy]
      v += S;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    v += __shfl_xor(v, d, 64);
    l += __shfl_xor(l, d, 64);
  }
  if ((tid & 63) == 0) {
    s_red[0][tid >> 6] = v;
    s_red[1][tid >> 6] = l;
  }
  lds_barrier();
  const size_t t = ((size_t)plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  if (tid == 0) partial[t] = (s_red[0][0] + s_red[0][1]) + (s_red[0][2] + s_red[0][3]);
  if (tid == 1 && partial_l1) partial_l1[t] = (s_red[1][0] + s_red[1][1]) + (s_red[1][2] + s_red[1][3]);
}

// The fused photometric loss of train.py:91-92 from the per-tile partials, in a fixed order (fp64):
// out = [(1 - lambda) L1 + lambda (1 - SSIM), L1, SSIM], means over all n pixels of all planes
// (loss_utils.py:17-18 and size_average=True of :40, which average over the same elements)
__global__ __launch_bounds__(1024) void k_loss_finish(int count, double inv_n, float lambda,
                                                      const float* __restrict__ partial,
                                                      const float* __restrict__ partial_l1, float* __restrict__ out) {
  __shared__ double s[2][16];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < count; i += 1024) {
    a += (double)partial[i];
    b += (double)partial_l1[i];
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    a += __shfl_xor(a, d, 64);
    b += __shfl_xor(b, d, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    s[0][w] = a;
    s[1][w] = b;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    double sa = 0.0, sb = 0.0;
    for (int k = 0; k < 16; k++) {
      sa += s[0][k];
      sb += s[1][k];
    }
    // the value as the reference's float32 expression forms it from the two float32 means
    const float ssim = (float)(sa * inv_n), l1 = (float)(sb * inv_n);
    out[0] = (1.0f - lambda) * l1 + lambda * (1.0f - ssim);
    out[1] = l1;
    out[2] = ssim;
  }
}

// per-plane SSIM-map sums in a fixed order (one workgroup per plane)
__global__ __launch_bounds__(256) void k_ssim_plane_sum(int tiles, const float* __restrict__ partial,
                                                        float* __restrict__ plane_sum) {
  __shared__ double s[256];
  const float* p = partial + (size_t)blockIdx.x * tiles;
  double a = 0.0;
  for (int i = threadIdx.x; i < tiles; i += 256) a += (double)p[i];
  s[threadIdx.x] = a;
  lds_barrier();
  for (int d = 128; d >= 1; d >>= 1) {
    if ((int)threadIdx.x < d) s[threadIdx.x] += s[threadIdx.x + d];
    lds_barrier();
  }
  if (threadIdx.x == 0) plane_sum[blockIdx.x] = (float)s[0];
}

// FUSED: the photometric loss's gradient, dimg1 = g (kS dSSIM-sum/dimg1 + kL sign(img1 - img2)) with
// g = scale[0] (the loss's incoming gradient, on the device), kS = -lambda / n, kL = (1 - lambda) / n;
// otherwise dimg1 = scale[plane / C] dSSIM-sum/dimg1.  Same tiling and passes as k_ssim_fwd, over
// the three partial maps.
template <bool FUSED>
__global__ __launch_bounds__(SS_BWD_NT) void k_ssim_bwd(int H, int W, int C, SsimWin win, const float* __restrict__ img1,
                                                    const float* __restrict__ img2, const float* __restrict__ dmaps,
                                                    const float* __restrict__ scale, float kS, float kL,
                                                    float* __restrict__ dimg1) {
  // the staged maps, then (after the horizontal pass) the filtered maps over them: 22 KB
  __shared__ __attribute__((aligned(16))) float s_lds[SS_BWD_LDS];
  float(*sd)[SS_IN][SS_LI] = reinterpret_cast<float(*)[SS_IN][SS_LI]>(s_lds);
  float(*sh)[SS_IN][SS_LH] = reinterpret_cast<float(*)[SS_IN][SS_LH]>(s_lds);
  const int plane = blockIdx.z;
  const int x0 = blockIdx.x * SS_T, y0 = blockIdx.y * SS_T;
  const size_t HW = (size_t)H * W, PHW = (size_t)gridDim.z * HW;
  const int tid = threadIdx.x;
  {
    const float* src[3] = {dmaps + plane * HW, dmaps + PHW + plane * HW, dmaps + 2 * PHW + plane * HW};
    stage_tiles<3, SS_BWD_NT>(sd, src, H, W, y0, x0);
  }
  // the vertical pass's threads (the first four waves): column c, rows 4 j .. 4 j + 3; their 8
  // image loads are issued now and land during the horizontal pass
  const bool vt = tid < 256;
  int c, j;
  vmap(tid, c, j);
  const int px = x0 + c;
  float xs[4], ys[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int py = y0 + 4 * j + i;
    const bool ok = vt && px < W && py < H;
    const size_t o = ok ? plane * HW + (size_t)py * W + px : 0;
    xs[i] = ok ? img1[o] : 0.f;
    ys[i] = ok ? img2[o] : 0.f;
  }
  lds_barrier();
  const bool hg = tid < SS_HG;
  const int r = tid % SS_IN, c0 = 4 * (tid / SS_IN);
  float o[3][4];
  if (hg) {
#pragma unroll
    for (int m = 0; m < 3; m++) {
      float x[16];
      ld16(&sd[m][r][c0], x);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < 2 * SS_R + 1; k++) a = __builtin_fmaf(win.w[k], x[i + k], a);
        o[m][i] = a;
      }
    }
  }
  lds_barrier();
  if (hg) {
#pragma unroll
    for (int m = 0; m < 3; m++)
      *reinterpret_cast<float4*>(&sh[m][r][c0]) = make_float4(o[m][0], o[m][1], o[m][2], o[m][3]);
  }
  lds_barrier();
  if (!vt || px >= W) return;
  float gm[3][4];
#pragma unroll
  for (int m = 0; m < 3; m++) {
    float v[14];
#pragma unroll
    for (int q = 0; q < 14; q++) v[q] = sh[m][4 * j + q][c];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 2 * SS_R + 1; k++) a = __builtin_fmaf(win.w[k], v[i + k], a);
      gm[m][i] = a;
    }
  }
  const float sc = FUSED ? scale[0] : scale[plane / C];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int py = y0 + 4 * j + i;
    if (py >= H) break;
    const size_t o = plane * HW + (size_t)py * W + px;
    const float x = xs[i], y = ys[i];
    const float dS = gm[0][i] + 2.f * x * gm[1][i] + y * gm[2][i];
    if constexpr (FUSED) {
      // d|u|/du = sign(u), 0 at u = 0 (torch's abs backward)
      const float u = x - y, sg = u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
      dimg1[o] = sc * __builtin_fmaf(kS, dS, kL * sg);
    } else {
      dimg1[o] = sc * dS;
    }
  }
}

void ssim_forward(int planes, int H, int W, const float* win11, const float* img1, const float* img2, float* dmaps,
                  float* partial, float* plane_sum, hipStream_t st) {
  SsimWin w;
  for (int k = 0; k < 2 * SS_R + 1; k++) w.w[k] = win11[k];
  const dim3 grid((W + SS_T - 1) / SS_T, (H + SS_T - 1) / SS_T, planes);
  GS_LAUNCH("ssim_fwd", k_ssim_fwd, grid, dim3(256), 0, st, H, W, w, img1, img2, dmaps, partial, nullptr);
  GS_LAUNCH("ssim_sum", k_ssim_plane_sum, dim3(planes), dim3(256), 0, st, (int)(grid.x * grid.y), partial, plane_sum);
}

void photometric_forward(int planes, int H, int W, const float* win11, const float* img, const float* gt,
                         float lambda, float* dmaps, float* partial, float* out3, hipStream_t st) {
  SsimWin w;
  for (int k = 0; k < 2 * SS_R + 1; k++) w.w[k] = win11[k];
  const dim3 grid((W + SS_T - 1) / SS_T, (H + SS_T - 1) / SS_T, planes);
  const int count = (int)ssim_partial_count(planes, H, W);
  GS_LAUNCH("ssim_fwd", k_ssim_fwd, grid, dim3(256), 0, st, H, W, w, img, gt, dmaps, partial, partial + count);
  GS_LAUNCH("loss_finish", k_loss_finish, dim3(1), dim3(1024), 0, st, count,
            1.0 / ((double)planes * (double)H * (double)W), lambda, partial, partial + count, out3);
}

void photometric_backward(int planes, int H, int W, const float* win11, const float* img, const float* gt,
                          const float* dmaps, float lambda, const float* grad, float* dimg, hipStream_t st) {
  SsimWin w;
  for (int k = 0; k < 2 * SS_R + 1; k++) w.w[k] = win11[k];
  const dim3 grid((W + SS_T - 1) / SS_T, (H + SS_T - 1) / SS_T, planes);
  const double n = (double)planes * (double)H * (double)W;
  GS_LAUNCH("ssim_bwd", k_ssim_bwd<true>, grid, dim3(SS_BWD_NT), 0, st, H, W, 1, w, img, gt, dmaps, grad,
            (float)(-(double)lambda / n), (float)((1.0 - (double)lambda) / n), dimg);
}

void ssim_backward(int planes, int C, int H, int W, const float* win11, const float* img1, const float* img2,
                   const float* dmaps, const float* scale, float* dimg1, hipStream_t st) {
  SsimWin w;
  for (int k = 0; k < 2 * SS_R + 1; k++) w.w[k] = win11[k];
  const dim3 grid((W + SS_T - 1) / SS_T, (H + SS_T - 1) / SS_T, planes);
  GS_LAUNCH("ssim_bwd", k_ssim_bwd<false>, grid, dim3(SS_BWD_NT), 0, st, H, W, C, w, img1, img2, dmaps, scale, 0.0f, 0.0f,
            dimg1);
}

size_t ssim_partial_count(int planes, int H, int W) {
  return (size_t)planes * ((W + SS_T - 1) / SS_T) * ((H + SS_T - 1) / SS_T);
}

}  // namespace gs
