// gs_train.hip -- fused per-iteration training updates around the rasterizer.
//
//   k_adam              one launch for all parameter groups of GaussianModel's optimizer
//                       (/root/reference/scene/gaussian_model.py:154-163: torch.optim.Adam, six
//                       groups, eps 1e-15): m, v, p updated in one pass, 16-B accesses.  Same update
//                       as torch's Adam (amsgrad off, no weight decay):
//                         m = m + (1 - b1) (g - m);  v = b2 v + (1 - b2) g^2
//                         p = p - (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
//                       in torch's operation order (see adam_update, gs_internal.h).
//   k_densify_stats     train.py:114-115 + gaussian_model.py:405-407 in one pass:
//                         vis = radii > 0; max_r[vis] = max(max_r, radii)
//                         accum[vis] += |grad2D[vis, :2]|;  denom[vis] += 1
//   k_activate_fwd/bwd  the render() inputs of GaussianModel's properties (gaussian_model.py:95-115,
//                       read at gaussian_renderer/__init__.py:53-80) in one launch each way:
//                         shs = cat(f_dc, f_rest, 1)   opacity = sigmoid(o)   scales = exp(s)
//                         rotations = q / max(|q|, 1e-12)      (F.normalize, p = 2, dim = 1)
//                       and their adjoints.  Blocks [0, feat_blocks) move the SH rows, 4 floats per
//                       thread (a Gaussian's 16x3 row is 12 float4); the rest do the per-Gaussian
//                       activations.
#include <cmath>

#include "gs_internal.h"

namespace gs {

// k_adam uses non-temporal 16-B loads / stores.  C3 train step: k_adam 310 -> 264 us, and the next
// iteration's k_activate_fwd 100 -> 72 us (no dirty lines of the update left to write back).
// Non-temporal accesses in the activation kernels measured slower or neutral (their lane-strided
// scalar stores lose the cache's line merging: k_activate_bwd 101 -> 354 us).
// One launch updates up to ADAM_MAX_TENSORS parameter tensors; a thread owns 4 consecutive
// elements of one tensor (16-B loads/stores of p, g, m, v when aligned, scalar tail otherwise).
struct AdamLaunch {
  float* p[ADAM_MAX_TENSORS];
  const float* g[ADAM_MAX_TENSORS];
  float* m[ADAM_MAX_TENSORS];
  float* v[ADAM_MAX_TENSORS];
  uint64_t end[ADAM_MAX_TENSORS];  // inclusive-scan end of each tensor, in 4-element chunks
  uint64_t n[ADAM_MAX_TENSORS];    // elements
  float neg_step_size[ADAM_MAX_TENSORS];  // -lr / (1 - b1^t)
  float bc2_sqrt[ADAM_MAX_TENSORS];       // sqrt(1 - b2^t)
  float wd[ADAM_MAX_TENSORS];
  int mode[ADAM_MAX_TENSORS];  // AdamGrad: how the tensor's gradient is formed from g
  int count;
  int sh_row, sh_rest;    // AG_SH_*: floats per row of the SH gradient source (3M) and of f_rest (3(M - 1))
  AdamConsts k;
};

// The element's gradient, from a gradient source g (base pointer) and the raw parameter values
// (before this update).  AG_SH_* / AG_SIGMOID / AG_EXP / AG_NORMALIZE apply the adjoint of the
// activation that render() puts between the parameter and the rasterizer (k_activate_bwd's
// expressions, operation for operation: the same floats as activate's backward followed by Adam)
// so the raw-parameter gradients never go through memory.
__device__ __forceinline__ float act_grad1(const AdamLaunch& a, int k, const float* g, uint64_t e, float praw) {
  switch (a.mode[k]) {
    case AG_SH_DC: {
      const uint64_t gi = e / 3;
      return g[gi * a.sh_row + (e - 3 * gi)];
    }
    case AG_SH_REST: {
      const uint64_t gi = e / (uint64_t)a.sh_rest;
      return g[gi * a.sh_row + 3 + (e - gi * a.sh_rest)];
    }
    case AG_SIGMOID:
      return sigmoid_adjoint(g[e], praw);
    case AG_EXP:
      return exp_adjoint(g[e], praw);
    default:
      return g[e];
  }
}

__global__ __launch_bounds__(256) void k_adam(AdamLaunch a, uint64_t total_chunks) {
  const uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= total_chunks) return;
  int k = 0;
  while (k + 1 < a.count && c >= a.end[k]) k++;
  const uint64_t i = (c - (k ? a.end[k - 1] : 0)) * 4;
  const uint64_t n = a.n[k];
  const int mode = a.mode[k];
  float *p = a.p[k] + i, *m = a.m[k] + i, *v = a.v[k] + i;
  const float* g = a.g[k] + i;  // AG_PLAIN
  const float ss = a.neg_step_size[k], ib = a.bc2_sqrt[k], wd = a.wd[k];
  const bool vec = i + 4 <= n && (((uintptr_t)p | (uintptr_t)m | (uintptr_t)v) & 15) == 0 &&
                   (mode == AG_SH_DC || mode == AG_SH_REST || (((uintptr_t)g) & 15) == 0);
  if (vec) {
    // streaming: every byte is touched once per step and the step's 1.65 GB (C3) exceeds the caches
    typedef float v4f __attribute__((ext_vector_type(4)));
    v4f P = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    v4f M = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(m));
    v4f V = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(v));
    float G[4];
    if (mode == AG_PLAIN) {
      const v4f Gv = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(g));
      G[0] = Gv.x, G[1] = Gv.y, G[2] = Gv.z, G[3] = Gv.w;
    } else if (mode == AG_NORMALIZE) {
      const float4 gq = *reinterpret_cast<const float4*>(g);
      const float gv[4] = {gq.x, gq.y, gq.z, gq.w}, q[4] = {P.x, P.y, P.z, P.w};
      normalize_adjoint(gv, q, G);
    } else if (mode == AG_SH_DC || mode == AG_SH_REST) {
      // four consecutive elements of f_dc / f_rest: one (row, column) division for the chunk
      // (32-bit: the tensors hold < 2^32 floats), then column steps with row carries
      const uint32_t w = mode == AG_SH_DC ? 3u : (uint32_t)a.sh_rest, off = mode == AG_SH_DC ? 0u : 3u;
      uint32_t r = (uint32_t)i / w, col = (uint32_t)i - r * w;
      const float* src = a.g[k];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        G[e] = src[(uint64_t)r * a.sh_row + off + col];
        if (++col == w) col = 0, r++;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; e++) G[e] = act_grad1(a, k, a.g[k], i + e, P[e]);
    }
#pragma unroll
    for (int e = 0; e < 4; e++) {
      float pe = P[e], me = M[e], ve = V[e];
      adam_update(pe, G[e], me, ve, a.k, ss, ib, wd);
      P[e] = pe, M[e] = me, V[e] = ve;
    }
    __builtin_nontemporal_store(P, reinterpret_cast<v4f*>(p));
    __builtin_nontemporal_store(M, reinterpret_cast<v4f*>(m));
    __builtin_nontemporal_store(V, reinterpret_cast<v4f*>(v));
  } else {
    const int cnt = (int)(n - i < 4 ? n - i : 4);
    float G[4];
    if (mode == AG_NORMALIZE) {  // rows of 4 (validated): the chunk is one whole quaternion
      const float gv[4] = {g[0], g[1], g[2], g[3]}, q[4] = {p[0], p[1], p[2], p[3]};
      normalize_adjoint(gv, q, G);
    } else {
      for (int j = 0; j < cnt; j++) G[j] = mode == AG_PLAIN ? g[j] : act_grad1(a, k, a.g[k], i + j, p[j]);
    }
    for (int j = 0; j < cnt; j++) adam_update(p[j], G[j], m[j], v[j], a.k, ss, ib, wd);
  }
}

__global__ __launch_bounds__(256) void k_densify_stats(int P, const int* __restrict__ radii,
                                                       const float* __restrict__ grad2d, int gstride, float* __restrict__ max_r,
                                                       float* __restrict__ accum, float* __restrict__ denom) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  densify_stat_one(i, radii, grad2d, gstride, max_r, accum, denom);
}

void adam_step(int count, float* const* params, const float* const* grads, float* const* exp_avg,
               float* const* exp_avg_sq, const long long* numel, const double* lr, const long long* step,
               const double* weight_decay, double beta1, double beta2, double eps, bool maximize, hipStream_t st,
               const int* modes, int sh_coeffs) {
  for (int base = 0; base < count; base += ADAM_MAX_TENSORS) {
    AdamLaunch a{};
    uint64_t chunks = 0;
    for (int k = base; k < count && k < base + ADAM_MAX_TENSORS; k++) {
      if (numel[k] <= 0) continue;
      const int j = a.count++;
      a.p[j] = params[k];
      a.g[j] = grads[k];
      a.m[j] = exp_avg[k];
      a.v[j] = exp_avg_sq[k];
      a.n[j] = (uint64_t)numel[k];
      chunks += (a.n[j] + 3) / 4;
      a.end[j] = chunks;
      adam_scalars(lr[k], step[k], beta1, beta2, &a.neg_step_size[j], &a.bc2_sqrt[j]);
      a.wd[j] = weight_decay ? (float)weight_decay[k] : 0.0f;
      a.mode[j] = modes ? modes[k] : AG_PLAIN;
    }
    if (!a.count) continue;
    a.sh_row = 3 * sh_coeffs;
    a.sh_rest = 3 * (sh_coeffs - 1);
    a.k = adam_consts(beta1, beta2, eps, maximize);
    GS_LAUNCH("adam", k_adam, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, st, a, chunks);
  }
}

void densify_stats(int P, const int* radii, const float* grad2d, int grad_stride, float* max_radii2D,
                   float* grad_accum, float* denom, hipStream_t st) {
  GS_LAUNCH("densify_stats", k_densify_stats, dim3((P + 255) / 256), dim3(256), 0, st, P, radii, grad2d,
            grad_stride, max_radii2D, grad_accum, denom);
}


__global__ __launch_bounds__(256) void k_activate_fwd(int P, int feat_blocks, int rest_w,
                                                      const float* __restrict__ f_dc, const float* __restrict__ f_rest,
                                                      const float* __restrict__ o_raw, const float* __restrict__ s_raw,
                                                      const float* __restrict__ q_raw, float* __restrict__ shs,
                                                      float* __restrict__ opac, float* __restrict__ scales,
                                                      float* __restrict__ rots) {
  const int row = 3 + rest_w;
  if ((int)blockIdx.x < feat_blocks) {
    const uint64_t e = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (e >= (uint64_t)P * row) return;
    const uint64_t gi = e / row;
    const int k = (int)(e - gi * row);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int kk = k + j;
      // rows of 3 + rest_w floats: a float4 may straddle two Gaussians when row % 4 != 0
      const uint64_t g2 = kk < row ? gi : gi + 1;
      const int k2 = kk < row ? kk : kk - row;
      v[j] = (g2 >= (uint64_t)P) ? 0.f : (k2 < 3 ? f_dc[g2 * 3 + k2] : f_rest[g2 * rest_w + (k2 - 3)]);
    }
    if (row % 4 == 0) {
      *reinterpret_cast<float4*>(shs + e) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int j = 0; j < 4 && e + j < (uint64_t)P * row; j++) shs[e + j] = v[j];
    }
    return;
  }
  const int i = (blockIdx.x - feat_blocks) * 256 + threadIdx.x;
  if (i >= P) return;
  opac[i] = 1.0f / (1.0f + expf(-o_raw[i]));
#pragma unroll
  for (int j = 0; j < 3; j++) scales[3 * i + j] = expf(s_raw[3 * i + j]);
  const float4 q = *reinterpret_cast<const float4*>(q_raw + 4 * i);
  const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
  *reinterpret_cast<float4*>(rots + 4 * i) = make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}

// Adjoint.  opacity: dL/do = g * (1 - y) * y (y = sigmoid(o), saved); scales: dL/ds = g * exp(s)
// (saved output); rotation: y = q / n, n = max(|q|, 1e-12):
//   dL/dq = g / n - q * <g, q> / (n^2 |q|) * [|q| > 1e-12]  (div, clamp_min and norm adjoints)
__global__ __launch_bounds__(256) void k_activate_bwd(int P, int feat_blocks, int rest_w,
                                                      const float* __restrict__ dshs, const float* __restrict__ dopac,
                                                      const float* __restrict__ dscales, const float* __restrict__ drots,
                                                      const float* __restrict__ opac, const float* __restrict__ scales,
                                                      const float* __restrict__ q_raw, float* __restrict__ d_dc,
                                                      float* __restrict__ d_rest, float* __restrict__ d_o,
                                                      float* __restrict__ d_s, float* __restrict__ d_q) {
  const int row = 3 + rest_w;
  if ((int)blockIdx.x < feat_blocks) {
    const uint64_t e = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    const uint64_t tot = (uint64_t)P * row;
    if (e >= tot) return;
    float v[4];
    if (row % 4 == 0) {
      const float4 t = *reinterpret_cast<const float4*>(dshs + e);
      v[0] = t.x, v[1] = t.y, v[2] = t.z, v[3] = t.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = e + j < tot ? dshs[e + j] : 0.f;
    }
    const uint64_t gi = e / row;
    const int k = (int)(e - gi * row);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (e + j >= tot) break;
      const int kk = k + j;
      const uint64_t g2 = kk < row ? gi : gi + 1;
      const int k2 = kk < row ? kk : kk - row;
      if (k2 < 3)
        d_dc[g2 * 3 + k2] = v[j];
      else
        d_rest[g2 * rest_w + (k2 - 3)] = v[j];
    }
    return;
  }
  const int i = (blockIdx.x - feat_blocks) * 256 + threadIdx.x;
  if (i >= P) return;
  if (dopac) {
    const float y = opac[i];
    d_o[i] = dopac[i] * (1.0f - y) * y;
  }
  if (dscales) {
#pragma unroll
    for (int j = 0; j < 3; j++) d_s[3 * i + j] = dscales[3 * i + j] * scales[3 * i + j];
  }
  if (drots) {
    const float4 q = *reinterpret_cast<const float4*>(q_raw + 4 * i);
    const float4 g = *reinterpret_cast<const float4*>(drots + 4 * i);
    const float len = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    const float n = fmaxf(len, 1e-12f);
    const float dot = g.x * q.x + g.y * q.y + g.z * q.z + g.w * q.w;
    const float c = len > 1e-12f ? dot / (n * n) / len : 0.0f;
    *reinterpret_cast<float4*>(d_q + 4 * i) =
        make_float4(g.x / n - c * q.x, g.y / n - c * q.y, g.z / n - c * q.z, g.w / n - c * q.w);
  }
}

void activate_forward(int P, int rest_w, const float* f_dc, const float* f_rest, const float* o_raw,
                      const float* s_raw, const float* q_raw, float* shs, float* opac, float* scales, float* rots,
                      hipStream_t st) {
  // shs == null: the SH rows are not concatenated (a split-SH rasterizer call reads f_dc / f_rest)
  const uint64_t fe = shs ? ((uint64_t)P * (3 + rest_w) + 3) / 4 : 0;
  const int fb = (int)((fe + 255) / 256), gb = (P + 255) / 256;
  GS_LAUNCH("activate_fwd", k_activate_fwd, dim3(fb + gb), dim3(256), 0, st, P, fb, rest_w, f_dc, f_rest, o_raw,
            s_raw, q_raw, shs, opac, scales, rots);
}

void activate_backward(int P, int rest_w, const float* dshs, const float* dopac, const float* dscales,
                       const float* drots, const float* opac, const float* scales, const float* q_raw, float* d_dc,
                       float* d_rest, float* d_o, float* d_s, float* d_q, hipStream_t st) {
  const uint64_t fe = dshs ? ((uint64_t)P * (3 + rest_w) + 3) / 4 : 0;
  const int fb = (int)((fe + 255) / 256), gb = (P + 255) / 256;
  GS_LAUNCH("activate_bwd", k_activate_bwd, dim3(fb + gb), dim3(256), 0, st, P, fb, rest_w, dshs, dopac, dscales,
            drots, opac, scales, q_raw, d_dc, d_rest, d_o, d_s, d_q);
}

}  // namespace gs
