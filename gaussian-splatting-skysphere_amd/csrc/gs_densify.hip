// gs_densify.hip -- GaussianModel.densify_and_prune in three passes over the Gaussians.
//
// The reference (/root/reference/scene/gaussian_model.py:258-403, called at train.py:118-120)
// rewrites all six parameter tensors and their Adam state four times per call: cat of the clones
// (densify_and_clone :375-389 -> densification_postfix :328-344), cat of the split children
// (densify_and_split :348-373), a prune of the split parents (:372-373, prune_points :289-305) and
// the final prune (:391-403).  Every intermediate layout is a stable order, so the final layout
// is known from the original one:
//
//   [ kept originals | kept clones | split children, k-major: child k of the r-th kept parent ]
//
// with, per original Gaussian j (g = accum/denom, NaN -> 0; s = exp(scaling); o = sigmoid(opacity)):
//   clone_j    = |g| >= thr and max(s) <= pd_ext                       (:377-378)
//   split_j    = g >= thr and max(s) > pd_ext                          (:353-356; clones have g = 0
//                                                                       and max(s) <= pd_ext: never split)
//   prune(o,s) = o < min_op or (screen and (0 > max_screen or max(s) > big_ext))
//                (:394-398; max_radii2D was reset to 0 by densification_postfix :342-344, so the
//                 screen-size test only fires for a negative max_screen_size)
//   keepA_j = !split_j and !prune(o, s);  keepB_j = clone_j and !prune(o, s)
//   child scaling = log(s * (1 / (0.8 N))) (:364), keepC_j = split_j and !prune(o, exp(child scaling))
//   child xyz     = R(q_j) sample + xyz_j, sample = torch.normal(0, s_j) drawn by the caller in
//                   the reference's order (:358-363: row k * n_split + rank of j among split)
// Clone and child rows get zero Adam moments (:315-316); the stats are re-zeroed by the caller.
//
// Passes: k_dens_classify (flags + per-block counts) -> k_dens_scan (exclusive block bases,
// totals) -> [host reads the totals, allocates, draws the samples] -> k_dens_stds (the std rows of
// the split draws) -> k_dens_emit (every output row; wave-cooperative row copies so that reads
// of the wide f_rest rows stay coalesced).
#include <cmath>

#include "gs_internal.h"

namespace gs {

constexpr uint8_t DF_CLONE = 1, DF_SPLIT = 2, DF_KEEP_A = 4, DF_KEEP_B = 8, DF_KEEP_C = 16;
constexpr int DENS_T = 256;

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ __launch_bounds__(DENS_T) void k_dens_classify(int P, DensifyParams dp, const float* __restrict__ accum,
                                                          const float* __restrict__ denom,
                                                          const float* __restrict__ opacity,
                                                          const float* __restrict__ scaling,
                                                          uint8_t* __restrict__ flags, uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_cnt[DENS_T / 64][4];
  const int j = blockIdx.x * DENS_T + threadIdx.x;
  uint8_t f = 0;
  if (j < P) {
    float g = accum[j] / denom[j];
    if (g != g) g = 0.0f;  // grads[grads.isnan()] = 0.0
    const float s0 = expf(scaling[3 * j]), s1 = expf(scaling[3 * j + 1]), s2 = expf(scaling[3 * j + 2]);
    const float ms = fmaxf(fmaxf(s0, s1), s2);
    const bool clone = fabsf(g) >= dp.thr && ms <= dp.pd_ext;
    const bool split = g >= dp.thr && ms > dp.pd_ext;
    const float o = sigmoid_f(opacity[j]);
    const bool prune = o < dp.min_op || (dp.screen && (0.0f > dp.max_screen || ms > dp.big_ext));
    f |= clone ? DF_CLONE : 0;
    f |= split ? DF_SPLIT : 0;
    f |= (!split && !prune) ? DF_KEEP_A : 0;
    f |= (clone && !prune) ? DF_KEEP_B : 0;
    if (split) {
      const float c0 = expf(logf(s0 * dp.inv_split)), c1 = expf(logf(s1 * dp.inv_split)),
                  c2 = expf(logf(s2 * dp.inv_split));
      const float mc = fmaxf(fmaxf(c0, c1), c2);
      const bool cprune = o < dp.min_op || (dp.screen && (0.0f > dp.max_screen || mc > dp.big_ext));
      f |= !cprune ? DF_KEEP_C : 0;
    }
    flags[j] = f;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t nA = __popcll(ballot64(f & DF_KEEP_A)), nB = __popcll(ballot64(f & DF_KEEP_B)),
                 nS = __popcll(ballot64(f & DF_SPLIT)), nC = __popcll(ballot64(f & DF_KEEP_C));
  if (lane == 0) s_cnt[w][0] = nA, s_cnt[w][1] = nB, s_cnt[w][2] = nS, s_cnt[w][3] = nC;
  lds_barrier();
  if (threadIdx.x < 4) {
    uint32_t t = 0;
    for (int q = 0; q < DENS_T / 64; q++) t += s_cnt[q][threadIdx.x];
    counts[(size_t)blockIdx.x * 4 + threadIdx.x] = t;
  }
}

// Exclusive scan of the per-block counts (in place, 4 independent counters), totals[4].
__global__ __launch_bounds__(1024) void k_dens_scan(int blocks, uint32_t* __restrict__ counts,
                                                    uint32_t* __restrict__ totals) {
  __shared__ uint32_t s_part[1024][4];
  const int t = threadIdx.x;
  const int per = (blocks + 1023) / 1024;
  const int b0 = t * per, b1 = min(blocks, b0 + per);
  uint32_t sum[4] = {0, 0, 0, 0};
  for (int b = b0; b < b1; b++)
    for (int q = 0; q < 4; q++) sum[q] += counts[(size_t)b * 4 + q];
  for (int q = 0; q < 4; q++) s_part[t][q] = sum[q];
  lds_barrier();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan over the 1024 partials
    uint32_t v[4];
    for (int q = 0; q < 4; q++) v[q] = t >= d ? s_part[t - d][q] : 0u;
    lds_barrier();
    for (int q = 0; q < 4; q++) s_part[t][q] += v[q];
    lds_barrier();
  }
  uint32_t run[4];
  for (int q = 0; q < 4; q++) run[q] = s_part[t][q] - sum[q];
  for (int b = b0; b < b1; b++)
    for (int q = 0; q < 4; q++) {
      const uint32_t c = counts[(size_t)b * 4 + q];
      counts[(size_t)b * 4 + q] = run[q];
      run[q] += c;
    }
  if (t == 1023)
    for (int q = 0; q < 4; q++) totals[q] = s_part[1023][q];
}

// Ranks of this lane's Gaussian among the block's flagged ones, plus the block base.
struct DensRanks {
  uint32_t a, b, s, c;
};
__device__ __forceinline__ DensRanks dens_ranks(uint8_t f, const uint32_t* __restrict__ bases) {
  __shared__ uint32_t s_cnt[DENS_T / 64][4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  const uint64_t bA = ballot64(f & DF_KEEP_A), bB = ballot64(f & DF_KEEP_B), bS = ballot64(f & DF_SPLIT),
                 bC = ballot64(f & DF_KEEP_C);
  if (lane == 0) s_cnt[w][0] = __popcll(bA), s_cnt[w][1] = __popcll(bB), s_cnt[w][2] = __popcll(bS),
                 s_cnt[w][3] = __popcll(bC);
  lds_barrier();
  DensRanks r;
  r.a = bases[(size_t)blockIdx.x * 4 + 0] + __popcll(bA & lt);
  r.b = bases[(size_t)blockIdx.x * 4 + 1] + __popcll(bB & lt);
  r.s = bases[(size_t)blockIdx.x * 4 + 2] + __popcll(bS & lt);
  r.c = bases[(size_t)blockIdx.x * 4 + 3] + __popcll(bC & lt);
  for (int q = 0; q < w; q++) r.a += s_cnt[q][0], r.b += s_cnt[q][1], r.s += s_cnt[q][2], r.c += s_cnt[q][3];
  return r;
}

// stds[k * n_split + rank_split(j)] = exp(scaling_j) for k < N (get_scaling[mask].repeat(N, 1), :358)
__global__ __launch_bounds__(DENS_T) void k_dens_stds(int P, int N, uint32_t n_split, const uint8_t* __restrict__ flags,
                                                      const uint32_t* __restrict__ bases,
                                                      const float* __restrict__ scaling, float* __restrict__ stds) {
  const int j = blockIdx.x * DENS_T + threadIdx.x;
  const uint8_t f = j < P ? flags[j] : 0;
  const DensRanks r = dens_ranks(f, bases);
  if (!(f & DF_SPLIT)) return;
  const float s0 = expf(scaling[3 * j]), s1 = expf(scaling[3 * j + 1]), s2 = expf(scaling[3 * j + 2]);
  for (int k = 0; k < N; k++) {
    float* o = stds + ((size_t)k * n_split + r.s) * 3;
    o[0] = s0, o[1] = s1, o[2] = s2;
  }
}

// Copy (or zero) rows of width w for the wave's 64 consecutive sources j0.. into the destination
// slot each lane holds (-1: none).  Flat element loop: coalesced reads of the source block.
__device__ __forceinline__ void wave_rows(const float* __restrict__ src, float* __restrict__ dst, int w, int j0,
                                          int nrows, int slot, bool zero) {
  if (!ballot64(slot >= 0)) return;  // wave-uniform: nothing to write
  const int lane = threadIdx.x & 63;
  const int tot = nrows * w;
  for (int base = 0; base < tot; base += 64) {
    const int e = base + lane;
    const int r = e < tot ? e / w : 0;
    const int s = __shfl(slot, r, 64);
    if (e < tot && s >= 0) dst[(size_t)s * w + (e - r * w)] = zero ? 0.0f : src[(size_t)(j0 + r) * w + (e - r * w)];
  }
}

__global__ __launch_bounds__(DENS_T) void k_dens_emit(int P, int N, DensifyParams dp, DensCounts n,
                                                      const uint8_t* __restrict__ flags,
                                                      const uint32_t* __restrict__ bases,
                                                      const float* __restrict__ samples, DensTensors t) {
  const int j = blockIdx.x * DENS_T + threadIdx.x;
  const uint8_t f = j < P ? flags[j] : 0;
  const DensRanks r = dens_ranks(f, bases);
  const int j0 = blockIdx.x * DENS_T + (threadIdx.x & ~63);
  const int nrows = max(0, min(64, P - j0));
  if (nrows == 0) return;  // wave-uniform
  const int slotA = (f & DF_KEEP_A) ? (int)r.a : -1;
  const int slotB = (f & DF_KEEP_B) ? (int)(n.keep_a + r.b) : -1;
  // kept originals: params and moments copied; clones: params copied, moments zero (:315-316)
  for (int q = 0; q < DENS_TENSORS; q++) {
    const int w = t.width[q];
    wave_rows(t.src[q], t.dst[q], w, j0, nrows, slotA, false);
    wave_rows(t.src[q], t.dst[q], w, j0, nrows, slotB, false);
    if (t.m_src[q]) {
      wave_rows(t.m_src[q], t.m_dst[q], w, j0, nrows, slotA, false);
      wave_rows(t.v_src[q], t.v_dst[q], w, j0, nrows, slotA, false);
      wave_rows(nullptr, t.m_dst[q], w, j0, nrows, slotB, true);
      wave_rows(nullptr, t.v_dst[q], w, j0, nrows, slotB, true);
    }
  }
  // split children: f_dc / f_rest / opacity / rotation repeated (:366-369), xyz and scaling new
  const uint32_t cbase = n.keep_a + n.keep_b;
  const bool child = (f & DF_KEEP_C) != 0;
  float R[9], x0 = 0.f, x1 = 0.f, x2 = 0.f, cs[3] = {0.f, 0.f, 0.f};
  if (child) {
    // build_rotation (general_utils.py:78-100): q / |q|, |q| summed left to right
    const float* qr = t.src[DT_ROT] + 4 * (size_t)j;
    const float nq = sqrtf(qr[0] * qr[0] + qr[1] * qr[1] + qr[2] * qr[2] + qr[3] * qr[3]);
    const float w = qr[0] / nq, x = qr[1] / nq, y = qr[2] / nq, z = qr[3] / nq;
    R[0] = 1.f - 2.f * (y * y + z * z), R[1] = 2.f * (x * y - w * z), R[2] = 2.f * (x * z + w * y);
    R[3] = 2.f * (x * y + w * z), R[4] = 1.f - 2.f * (x * x + z * z), R[5] = 2.f * (y * z - w * x);
    R[6] = 2.f * (x * z - w * y), R[7] = 2.f * (y * z + w * x), R[8] = 1.f - 2.f * (x * x + y * y);
    const float* xs = t.src[DT_XYZ] + 3 * (size_t)j;
    x0 = xs[0], x1 = xs[1], x2 = xs[2];
    const float* ss = t.src[DT_SCALING] + 3 * (size_t)j;
    for (int c = 0; c < 3; c++) cs[c] = logf(expf(ss[c]) * dp.inv_split);  // (:364), see DensifyParams
  }
  for (int k = 0; k < N; k++) {
    const int slotC = child ? (int)(cbase + (uint32_t)k * n.keep_c + r.c) : -1;
    for (int q = 0; q < DENS_TENSORS; q++) {
      if (q != DT_XYZ && q != DT_SCALING) wave_rows(t.src[q], t.dst[q], t.width[q], j0, nrows, slotC, false);
      if (t.m_src[q]) {
        wave_rows(nullptr, t.m_dst[q], t.width[q], j0, nrows, slotC, true);
        wave_rows(nullptr, t.v_dst[q], t.width[q], j0, nrows, slotC, true);
      }
    }
    if (child) {
      const float* sm = samples + ((size_t)k * n.split + r.s) * 3;
      float* xo = t.dst[DT_XYZ] + 3 * (size_t)slotC;
      // torch.bmm(rots, samples[..., None]) + xyz (:362)
      xo[0] = fmaf(R[2], sm[2], fmaf(R[1], sm[1], R[0] * sm[0])) + x0;
      xo[1] = fmaf(R[5], sm[2], fmaf(R[4], sm[1], R[3] * sm[0])) + x1;
      xo[2] = fmaf(R[8], sm[2], fmaf(R[7], sm[1], R[6] * sm[0])) + x2;
      float* so = t.dst[DT_SCALING] + 3 * (size_t)slotC;
      so[0] = cs[0], so[1] = cs[1], so[2] = cs[2];
    }
  }
}

void densify_classify(int P, const DensifyParams& dp, const float* accum, const float* denom, const float* opacity,
                      const float* scaling, uint8_t* flags, uint32_t* counts, uint32_t* totals, hipStream_t st) {
  const int blocks = (P + DENS_T - 1) / DENS_T;
  GS_LAUNCH("dens_classify", k_dens_classify, dim3(blocks), dim3(DENS_T), 0, st, P, dp, accum, denom, opacity,
            scaling, flags, counts);
  GS_LAUNCH("dens_scan", k_dens_scan, dim3(1), dim3(1024), 0, st, blocks, counts, totals);
}

void densify_stds(int P, int N, uint32_t n_split, const uint8_t* flags, const uint32_t* bases, const float* scaling,
                  float* stds, hipStream_t st) {
  const int blocks = (P + DENS_T - 1) / DENS_T;
  GS_LAUNCH("dens_stds", k_dens_stds, dim3(blocks), dim3(DENS_T), 0, st, P, N, n_split, flags, bases, scaling, stds);
}

void densify_emit(int P, int N, const DensifyParams& dp, const DensCounts& n, const uint8_t* flags,
                  const uint32_t* bases, const float* samples, const DensTensors& t, hipStream_t st) {
  const int blocks = (P + DENS_T - 1) / DENS_T;
  GS_LAUNCH("dens_emit", k_dens_emit, dim3(blocks), dim3(DENS_T), 0, st, P, N, dp, n, flags, bases, samples, t);
}

}  // namespace gs
