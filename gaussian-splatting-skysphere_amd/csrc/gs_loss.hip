// gs_loss.hip -- fused SSIM (forward + backward) for the photometric loss of train.py.
//
// Restates /root/reference/utils/loss_utils.py:ssim/_ssim (11x11 Gaussian window, sigma 1.5,
// zero padding 5, C1 = 0.01^2, C2 = 0.03^2, mean of the SSIM map), which the reference evaluates
// as five depthwise conv2d calls plus their autograd backward every iteration
// (train.py:91-92).  Here one kernel produces, per plane (image x channel) and 16x16 tile, the
// five windowed moments by a separable 11-tap filter through LDS, the SSIM map sum and the three
// per-pixel partials dS/dmu1, dS/dE[x^2], dS/dE[xy]; a second kernel filters those partials with
// the same window (the adjoint of a symmetric, zero-padded correlation) and forms dL/dimg1.
//
//   S = (2 m1 m2 + C1)(2 s12 + C2) / ((m1^2 + m2^2 + C1)(s11 + s22 + C2)),
//   s11 = E[x^2] - m1^2, s22 = E[y^2] - m2^2, s12 = E[xy] - m1 m2
//   dS/dm1 = 2 m2 (A2 - A1) / (B1 B2) - 2 m1 S (1/B1 - 1/B2),  dS/dE[x^2] = -S / B2,
//   dS/dE[xy] = 2 A1 / (B1 B2)
//   dL/dx(q) = scale * [ (w * dS/dm1)(q) + 2 x(q) (w * dS/dE[x^2])(q) + y(q) (w * dS/dE[xy])(q) ]
//
// The map sum is reduced per workgroup and then per plane in a fixed order (deterministic).
#include "gs_internal.h"

namespace gs {

constexpr int SS_T = 16;                 // output tile
constexpr int SS_R = 5;                  // window radius
constexpr int SS_IN = SS_T + 2 * SS_R;   // 26: input tile with halo
constexpr int SS_LD = SS_IN + 1;         // padded LDS row

struct SsimWin {
  float w[2 * SS_R + 1];
};

__device__ __forceinline__ float ld_plane(const float* p, int H, int W, int y, int x) {
  return (y >= 0 && y < H && x >= 0 && x < W) ? p[(size_t)y * W + x] : 0.0f;
}

__global__ __launch_bounds__(256) void k_ssim_fwd(int H, int W, SsimWin win, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, float* __restrict__ dmaps,
                                                  float* __restrict__ partial, float* __restrict__ partial_l1) {
  __shared__ float sx[SS_IN][SS_LD], sy[SS_IN][SS_LD];
  __shared__ float sh[5][SS_IN][SS_T + 1];
  __shared__ float s_red[2][4];
  const int plane = blockIdx.z;
  const int x0 = blockIdx.x * SS_T, y0 = blockIdx.y * SS_T;
  const size_t HW = (size_t)H * W;
  const float* p1 = img1 + plane * HW;
  const float* p2 = img2 + plane * HW;
  const int tid = threadIdx.x;
  for (int i = tid; i < SS_IN * SS_IN; i += 256) {
    const int r = i / SS_IN, c = i - r * SS_IN;
    sx[r][c] = ld_plane(p1, H, W, y0 - SS_R + r, x0 - SS_R + c);
    sy[r][c] = ld_plane(p2, H, W, y0 - SS_R + r, x0 - SS_R + c);
  }
  lds_barrier();
  // horizontal pass: 26 rows x 16 columns, five moments
  for (int i = tid; i < SS_IN * SS_T; i += 256) {
    const int r = i / SS_T, c = i - r * SS_T;
    float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
    for (int k = 0; k < 2 * SS_R + 1; k++) {
      const float x = sx[r][c + k], y = sy[r][c + k], wk = win.w[k];
      a = __builtin_fmaf(wk, x, a);
      b = __builtin_fmaf(wk, y, b);
      aa = __builtin_fmaf(wk, x * x, aa);
      bb = __builtin_fmaf(wk, y * y, bb);
      ab = __builtin_fmaf(wk, x * y, ab);
    }
    sh[0][r][c] = a;
    sh[1][r][c] = b;
    sh[2][r][c] = aa;
    sh[3][r][c] = bb;
    sh[4][r][c] = ab;
  }
  lds_barrier();
  const int tx = tid & (SS_T - 1), ty = tid / SS_T;
  float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
  for (int k = 0; k < 2 * SS_R + 1; k++) {
    const float wk = win.w[k];
    m1 = __builtin_fmaf(wk, sh[0][ty + k][tx], m1);
    m2 = __builtin_fmaf(wk, sh[1][ty + k][tx], m2);
    e11 = __builtin_fmaf(wk, sh[2][ty + k][tx], e11);
    e22 = __builtin_fmaf(wk, sh[3][ty + k][tx], e22);
    e12 = __builtin_fmaf(wk, sh[4][ty + k][tx], e12);
  }
  const float C1 = 1e-4f, C2 = 9e-4f;  // 0.01 ** 2, 0.03 ** 2 as the float32 tensor ops see them
  const float mu12 = m1 * m2;
  const float A1 = 2.f * mu12 + C1, A2 = 2.f * (e12 - mu12) + C2;
  const float B1 = m1 * m1 + m2 * m2 + C1, B2 = (e11 - m1 * m1) + (e22 - m2 * m2) + C2;
  const float iB1 = 1.f / B1, iB2 = 1.f / B2, iB = iB1 * iB2;
  const float S = A1 * A2 * iB;
  const int px = x0 + tx, py = y0 + ty;
  const bool inside = px < W && py < H;
  if (inside) {
    const size_t o = plane * HW + (size_t)py * W + px;
    const size_t PHW = (size_t)gridDim.z * HW;
    dmaps[o] = 2.f * m2 * (A2 - A1) * iB - 2.f * m1 * S * (iB1 - iB2);  // dS/dm1
    dmaps[PHW + o] = -S * iB2;                                          // dS/dE[x^2]
    dmaps[2 * PHW + o] = 2.f * A1 * iB;                                 // dS/dE[xy]
  }
  float v = inside ? S : 0.f;
  // |x - y| of the pixel (the L1 term of the fused photometric loss), from the staged tile
  float l = inside ? fabsf(sx[ty + SS_R][tx + SS_R] - sy[ty + SS_R][tx + SS_R]) : 0.f;
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
// otherwise dimg1 = scale[plane / C] dSSIM-sum/dimg1.
template <bool FUSED>
__global__ __launch_bounds__(256) void k_ssim_bwd(int H, int W, int C, SsimWin win, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, const float* __restrict__ dmaps,
                                                  const float* __restrict__ scale, float kS, float kL,
                                                  float* __restrict__ dimg1) {
  __shared__ float sd[3][SS_IN][SS_LD];
  __shared__ float sh[3][SS_IN][SS_T + 1];
  const int plane = blockIdx.z;
  const int x0 = blockIdx.x * SS_T, y0 = blockIdx.y * SS_T;
  const size_t HW = (size_t)H * W, PHW = (size_t)gridDim.z * HW;
  const int tid = threadIdx.x;
  for (int i = tid; i < SS_IN * SS_IN; i += 256) {
    const int r = i / SS_IN, c = i - r * SS_IN;
    const int y = y0 - SS_R + r, x = x0 - SS_R + c;
#pragma unroll
    for (int q = 0; q < 3; q++) sd[q][r][c] = ld_plane(dmaps + q * PHW + plane * HW, H, W, y, x);
  }
  lds_barrier();
  for (int i = tid; i < SS_IN * SS_T; i += 256) {
    const int r = i / SS_T, c = i - r * SS_T;
    float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < 2 * SS_R + 1; k++) {
      const float wk = win.w[k];
      a = __builtin_fmaf(wk, sd[0][r][c + k], a);
      b = __builtin_fmaf(wk, sd[1][r][c + k], b);
      d = __builtin_fmaf(wk, sd[2][r][c + k], d);
    }
    sh[0][r][c] = a;
    sh[1][r][c] = b;
    sh[2][r][c] = d;
  }
  lds_barrier();
  const int tx = tid & (SS_T - 1), ty = tid / SS_T;
  const int px = x0 + tx, py = y0 + ty;
  if (px >= W || py >= H) return;
  float g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
  for (int k = 0; k < 2 * SS_R + 1; k++) {
    const float wk = win.w[k];
    g0 = __builtin_fmaf(wk, sh[0][ty + k][tx], g0);
    g1 = __builtin_fmaf(wk, sh[1][ty + k][tx], g1);
    g2 = __builtin_fmaf(wk, sh[2][ty + k][tx], g2);
  }
  const size_t o = plane * HW + (size_t)py * W + px;
  const float x = img1[o], y = img2[o];
  const float dS = g0 + 2.f * x * g1 + y * g2;
  if constexpr (FUSED) {
    // d|u|/du = sign(u), 0 at u = 0 (torch's abs backward)
    const float u = x - y, sg = u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
    dimg1[o] = scale[0] * __builtin_fmaf(kS, dS, kL * sg);
  } else {
    dimg1[o] = scale[plane / C] * dS;
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
  GS_LAUNCH("ssim_bwd", k_ssim_bwd<true>, grid, dim3(256), 0, st, H, W, 1, w, img, gt, dmaps, grad,
            (float)(-(double)lambda / n), (float)((1.0 - (double)lambda) / n), dimg);
}

void ssim_backward(int planes, int C, int H, int W, const float* win11, const float* img1, const float* img2,
                   const float* dmaps, const float* scale, float* dimg1, hipStream_t st) {
  SsimWin w;
  for (int k = 0; k < 2 * SS_R + 1; k++) w.w[k] = win11[k];
  const dim3 grid((W + SS_T - 1) / SS_T, (H + SS_T - 1) / SS_T, planes);
  GS_LAUNCH("ssim_bwd", k_ssim_bwd<false>, grid, dim3(256), 0, st, H, W, C, w, img1, img2, dmaps, scale, 0.0f, 0.0f,
            dimg1);
}

size_t ssim_partial_count(int planes, int H, int W) {
  return (size_t)planes * ((W + SS_T - 1) / SS_T) * ((H + SS_T - 1) / SS_T);
}

}  // namespace gs
