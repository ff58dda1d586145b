// gs_backward.hip -- backward pass of the MI355X Gaussian rasterizer (gfx950).
//
// Restates the un-vendored upstream backward (spec SURVEY.md §8a a7-a8) without global atomics:
//   k_render_bwd      one 128-lane workgroup per tile walks the tile's list back to front
//                     (starting at the tile's max n_contrib -- later entries never contribute);
//                     each wave64 owns an 8x16 half (two pixels per lane) and visits only the
//                     entries whose exact alpha ellipse meets it (scalar walk over ballot masks),
//                     recovers T with one reciprocal, forms the 9 per-entry sums of its lane's two
//                     pixels, reduces them over the wave with permlane32/16 swaps (two values per
//                     add) + DPP row sums, and stores them in an LDS record per wave; the flush adds
//                     the two waves' records and STORES one 9-float record per (Gaussian, tile)
//                     instance at the instance's depth-ordered slot.
//   k_preprocess_bwd  one lane per Gaussian sums its contiguous instance records (fixed order:
//                     deterministic, no float atomics) and runs conic -> cov2D -> cov3D / mean,
//                     projection, SH and scale/rotation gradients in one pass.
// Upstream instead issues 9 float atomics per contributing (pixel, Gaussian) pair; on MI355X
// per-lane scattered float atomics run at ~0.08 TB/s (MI355X_MICROARCH.md §Global float atomics),
// while the record store + contiguous re-read moves the same information at HBM stream rates.
#include "gs_internal.h"

namespace gs {

#ifdef GS_TIMING
// diagnostic build only (-DGS_TIMING, tools/bwd_timing.py): per backward wave b (blockIdx.x): start /
// end stamps, tile << 32 | n_eff, hw ids, entries walked << 32 | slots evaluated
GS_TIMING_BUFFER(g_bwd_timing, gs_debug_bwd_timing)
#define GS_BWD_T0() const unsigned long long t_start = timing_stamp()
#define GS_BWD_TREC(tile, n_eff, walked, slots) timing_record(g_bwd_timing, t_start, tile, n_eff, walked, slots)
#else
#define GS_BWD_T0() (void)0
#define GS_BWD_TREC(tile, n_eff, walked, slots) (void)0
#endif

// a 36-B gradient record as three 12-B stores (global_store_dwordx3; 4-B alignment is enough)
struct __attribute__((aligned(4))) Rec3 {
  float a, b, c;
};

// the 36-B record read as three 12-B pieces (merged into 16-B loads; 4-B alignment is enough)
__device__ __forceinline__ void load_rec(const float* p, float* v) {
  const Rec3* r = reinterpret_cast<const Rec3*>(p);
  const Rec3 a = r[0], b = r[1], c = r[2];
  v[0] = a.a, v[1] = a.b, v[2] = a.c, v[3] = b.a, v[4] = b.b, v[5] = b.c, v[6] = c.a, v[7] = c.b, v[8] = c.c;
}

// ------------------------------------------------------------------------------------------
// Tile-wave backward: ONE wave64 per tile, four pixel slots per lane.
//
// Lane l owns pixel (l & 7, l >> 3) of each 8x8 quadrant k of the tile (slot k).  A staged entry
// carries the set of quadrants its alpha >= 1/255 ellipse meets (the forward's per-quadrant cull)
// and the walk evaluates and commits only those slots: the C3 oracle study
// (tools/bwd_layout_stats.py, profiles/r04_bwd_layout_stats_c3.txt) puts the pixel slots
// evaluated per walked entry at 143 (quadrant slots) against 193 for the two 8x16 half waves of
// k_render_bwd, and the nine per-entry sums are reduced over the wave ONCE per tile entry (0.86
// reductions per walked entry instead of 1.36).  The lane's slots are pre-summed in registers
// (one FMA per term and slot).  One wave per workgroup: staging, walk and flush need no workgroup
// barrier, and every lane stages (and later flushes) one entry of a 64-entry batch, keeping that
// entry's raw conic, opacity and slot in its registers.
// Same per-pixel recurrence and decisions as k_render_bwd (and as the forward); only the order in
// which a tile entry's per-pixel terms are summed differs.
// ------------------------------------------------------------------------------------------

struct BwdSlot {
  float T, U, d0, d1, d2;
  uint32_t last;
};

// one slot's evaluation + commit for one entry; s[] accumulates the lane's slot terms
template <bool EXACT>
__device__ __forceinline__ uint64_t bwd_slot(BwdSlot& q, float pfx, float pfy, const float4 xr, const float4 co,
                                         const float4 br, uint32_t e, float* s) {
  const float bl = br.x;
  const float dx = xr.x - pfx, dy = xr.y - pfy;
  const float pw = falloff_log2_m<EXACT>(co, dx, dy);  // log2(e) * power (fast: + log2 o)
  const float oG = opac_gauss<EXACT>(co, pw);
  // same decision as the forward (k_render_fwd_q): alpha = min(0.99, o G) >= 1/255 <=> o G >= 1/255
  const bool c_walk = e < q.last, c_alpha = oG >= 1.0f / 255.0f, c_pw = !EXACT || pw <= 0.0f;
  const bool con = c_walk && c_pw && c_alpha;
  // a non-contributing pixel runs as an o G = 0 entry: T and U pass through unchanged bit for bit
  const float oGm = con ? oG : 0.0f;
  const float ae = __builtin_amdgcn_fmed3f(oGm, 0.0f, 0.99f);
  const float omA = 1.0f - ae;
  float inv = __builtin_amdgcn_rcpf(omA);
  if constexpr (EXACT) inv = __builtin_fmaf(inv, __builtin_fmaf(-omA, inv, 1.0f), inv);
  const float Tn = q.T * inv;
  const float dch = ae * Tn;
  const float Cd = __builtin_fmaf(bl, q.d2, __builtin_fmaf(xr.w, q.d1, xr.z * q.d0));
  const float dLa = __builtin_fmaf(Tn, Cd, -(q.U * inv));
  const float qq = oGm * dLa;  // dL/dG G = o G dL/dalpha (not gated by the 0.99 clamp)
  // moments of q about the entry's reference point r = the splat mean clamped to the tile's pixel
  // box (u = dx - (mean - r) = r - pixel): for a splat centred in the tile u is dx itself, for one
  // centred outside it |u| <= 15 instead of the distance to the mean -- the terms stay small, so
  // the fp32 sums keep the precision the covariance chain needs.  The flush shifts them to the
  // mean in fp64 (k_render_bwd_tw).
  const float mx = dx - br.y, my = dy - br.z;
  const float qx = qq * mx, qy = qq * my;
  s[0] = __builtin_fmaf(dch, q.d0, s[0]);
  s[1] = __builtin_fmaf(dch, q.d1, s[1]);
  s[2] = __builtin_fmaf(dch, q.d2, s[2]);
  s[3] = s[3] + qx;
  s[4] = s[4] + qy;
  s[5] = __builtin_fmaf(qx, mx, s[5]);
  s[6] = __builtin_fmaf(qx, my, s[6]);
  s[7] = __builtin_fmaf(qy, my, s[7]);
  s[8] = s[8] + qq;
  q.T = Tn;
  q.U = __builtin_fmaf(Cd, dch, q.U);
  // the lanes where this slot contributes, from the compares' own lane masks (a ballot of their
  // conjunction would be re-materialised through a VGPR: two VALU per slot)
  uint64_t m = __builtin_amdgcn_ballot_w64(c_walk) & __builtin_amdgcn_ballot_w64(c_alpha);
  if constexpr (EXACT) m &= __builtin_amdgcn_ballot_w64(c_pw);
  return m;
}

template <bool EXACT>
__global__ __launch_bounds__(64) void k_render_bwd_tw(CameraArgs c, const uint2* __restrict__ ranges,
                                                                    const uint32_t* __restrict__ point_list,
                                                                    const uint32_t* __restrict__ point_gid,
                                                                    const float4* __restrict__ splat,
                                                                    const float* __restrict__ final_T,
                                                                    const uint32_t* __restrict__ n_contrib,
                                                                    const uint32_t* __restrict__ tile_max,
                                                                    const uint32_t* __restrict__ tile_order,
                                                                    const float* __restrict__ dL_dpix,
                                                                    float* __restrict__ gradrec) {
  __shared__ float4 s_xy[64];  // (x, y, r, g)
  __shared__ float4 s_co[64];  // falloff coefficients + opacity (fall_coefs)
  __shared__ float4 s_br[64];  // (b, mean - r: x, y, -), r the moments' reference point (bwd_slot)
  // entry rows of 16 floats (a stride of 20, which puts the flush's 16-B row reads on distinct
  // banks, measured 343 -> 361 us at C3)
  constexpr int ROW = 16;
  __shared__ __attribute__((aligned(16))) float s_acc[64][ROW];
  GS_BWD_T0();
  const uint32_t tile = __builtin_amdgcn_readfirstlane(tile_order ? tile_order[blockIdx.x] : blockIdx.x);
  if (tile == ~0u) return;  // a hole of the XCD-group launch order
  const int tx = (int)(tile % (uint32_t)c.gx), ty = (int)(tile / (uint32_t)c.gx);
  const int lane = threadIdx.x;
  const uint2 range = ranges[tile];
  const uint32_t n = range.y - range.x;
  // per-quadrant largest n_contrib (the forward's quadrant waves): slot k's walk ends there
  const uint4 qm = reinterpret_cast<const uint4*>(tile_max)[tile];
  const uint32_t qlast[4] = {min(qm.x, n), min(qm.y, n), min(qm.z, n), min(qm.w, n)};
  const uint32_t n_eff = max(max(qlast[0], qlast[1]), max(qlast[2], qlast[3]));
  if (n_eff == 0) {
    GS_BWD_TREC(tile, 0u, 0u, 0u);
    return;  // no instance walked: no records (k_sum_records reads none below a cut of 0)
  }
#ifdef GS_TIMING
  uint32_t t_walked = 0, t_slots = 0;
#endif

  const size_t HW = (size_t)c.W * c.H;
  const int qx0 = tx * GS_TILE + (lane & 7), qy0 = ty * GS_TILE + (lane >> 3);
  BwdSlot p[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int px = qx0 + 8 * (k & 1), py = qy0 + 8 * (k >> 1);
    const bool in = px < c.W && py < c.H;
    const size_t pix = in ? (size_t)py * c.W + px : 0;
    const float Tf = in ? final_T[pix] : 0.0f;
    p[k].T = Tf;
    p[k].last = in ? n_contrib[pix] : 0u;
    p[k].d0 = in ? dL_dpix[pix] : 0.0f;
    p[k].d1 = in ? dL_dpix[HW + pix] : 0.0f;
    p[k].d2 = in ? dL_dpix[2 * HW + pix] : 0.0f;
    // U = S + T_final bg . dL/dpix (see k_render_bwd)
    p[k].U = Tf * (c.bg[0] * p[k].d0 + c.bg[1] * p[k].d1 + c.bg[2] * p[k].d2);
  }
  const float ddelx_dx = (float)(0.5 * c.W), ddely_dy = (float)(0.5 * c.H);
  const float pfx0 = (float)qx0, pfy0 = (float)qy0;
  using lds_float = __attribute__((address_space(3))) float;
  // writer lanes 16 r + 8 h: s[r + 4 h] at slot r + 4 h, their s8 partial at slot 8 + r + 4 h
  lds_float* const acc_lane = (lds_float*)(&s_acc[0][(lane >> 4) + 4 * ((lane >> 3) & 1)]);
  const bool hi8 = (lane & 8) != 0;

  // staging pipeline (one entry per lane): while batch k is walked, the splat records of batch
  // k + 1, the ids of batch k + 2 and (ids by slot) the slots of batch k + 3 are in flight.
  // Batch k's entry of lane t sits at list position range.x + e0 - 64 k, e0 = n_eff - 1 - t.
  // The loads are unconditional, with list positions below 0 clamped to 0 (a valid entry: the
  // lane stages nothing then): a load under a condition has to keep the register's old value on
  // the other path, and the copy that merges the two makes the compiler wait for the load right
  // where it is issued instead of at the next batch.
  const int32_t e0 = (int32_t)n_eff - 1 - lane;
  const uint32_t* const plist = point_list + range.x;
  auto pos = [&](int32_t e) { return (uint32_t)max(e, 0); };
  uint32_t slot_c = plist[pos(e0)];
  uint32_t G1 = point_gid[slot_c];
  float4 pa = splat[3 * G1], pb = splat[3 * G1 + 1], pd = splat[3 * G1 + 2];
  uint32_t S1 = plist[pos(e0 - 64)];
  G1 = point_gid[S1];
  uint32_t S2 = plist[pos(e0 - 128)];

  uint32_t rec_lanes = 0;  // lanes holding a mapped record in their LDS row (the last flushed batch)
  auto store_records = [&]() {
    if ((uint32_t)lane < rec_lanes) {
      const float4* row = reinterpret_cast<const float4*>(&s_acc[lane][0]);
      const float4 a = row[0], b = row[1], d = row[2];
      Rec3* r = reinterpret_cast<Rec3*>(gradrec + (size_t)__float_as_uint(d.y) * GRAD_REC);
      r[0] = Rec3{a.x, a.y, a.z};
      r[1] = Rec3{a.w, b.x, b.y};
      r[2] = Rec3{b.z, b.w, d.x};
    }
  };
  for (uint32_t base = 0; base < n_eff; base += 64) {
    const uint32_t cnt = min(64u, n_eff - base);
    // stage: lane t holds entry t of the batch (walk order: back to front)
    const bool mine = (uint32_t)lane < cnt;
    const uint32_t slot = slot_c;
    const float ccx = pa.z, ccy = pa.w, ccz = pb.x, cop = pb.y;  // raw conic + opacity (flush)
    uint32_t qmask = 0;
    if (mine) {
      s_xy[lane] = make_float4(pa.x, pa.y, pb.z, pb.w);
      s_co[lane] = fall_coefs_m<EXACT>(pa.z, pa.w, pb.x, pb.y);
      const float x0 = (float)(tx * GS_TILE), y0 = (float)(ty * GS_TILE);
      s_br[lane] = make_float4(pd.x, pa.x - fminf(fmaxf(pa.x, x0), x0 + 15.0f),
                               pa.y - fminf(fmaxf(pa.y, y0), y0 + 15.0f), 0.0f);
      qmask = quadrant_mask(pa.x, pa.y, pa.z, pa.w, pb.x, pd.z, tx, ty);
    }
    // issue the next batch's splat loads, the ids after it and (ids by slot) the slots after those
    const int32_t e1 = e0 - (int32_t)(base + 64);
    slot_c = S1;
    pa = splat[3 * G1], pb = splat[3 * G1 + 1], pd = splat[3 * G1 + 2];
    S1 = S2;
    G1 = point_gid[S2];
    S2 = plist[pos(e1 - 128)];
    // the previous batch's records (mapped by its flush into the lanes' LDS rows, slot in word 9):
    // stored now, behind this batch's loads, so that the wait for those loads at the next staging
    // does not also wait for just-issued stores (loads and stores share one counter)
    if (base > 0) store_records();
    // per-slot entry sets; entries no pixel of quadrant k reaches (e >= qlast[k]) sit at the low bits
    uint64_t M[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint64_t mk = __ballot((qmask >> k) & 1u);
      const int jmin = (int)n_eff - (int)qlast[k] - (int)base;  // entry j reaches quadrant k iff j >= jmin
      if (jmin > 0) mk &= jmin >= 64 ? 0ull : ~((1ull << jmin) - 1ull);
      M[k] = mk;
    }
    __builtin_amdgcn_wave_barrier();
    uint64_t m = (M[0] | M[1]) | (M[2] | M[3]);
    uint64_t wrote = 0;
#pragma unroll 1
    while (m) {
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      const float4 xr = s_xy[j], co = s_co[j], br = s_br[j];
      const uint32_t e = n_eff - 1 - (base + j);
      // -0 (the additive identity of IEEE addition): the first contributing slot's FMAs / adds into
      // it fold to plain products / moves (with +0 they cannot: x + 0 differs from x for x = -0)
      float s[GRAD_REC];
#pragma unroll
      for (int t = 0; t < GRAD_REC; t++) s[t] = -0.0f;
#ifdef GS_TIMING
      t_walked++;
      t_slots += ((M[0] >> j) & 1ull) + ((M[1] >> j) & 1ull) + ((M[2] >> j) & 1ull) + ((M[3] >> j) & 1ull);
#endif
      uint64_t con = 0;  // lanes with a contributing slot
#pragma unroll
      for (int k = 0; k < 4; k++)
        if ((M[k] >> j) & 1ull)
          con |= bwd_slot<EXACT>(p[k], pfx0 + (float)(8 * (k & 1)), pfy0 + (float)(8 * (k >> 1)), xr, co, br, e, s);
      if (con != 0) {
        wrote |= 1ull << j;
        float d, d8;
        wave_sum9_halfrows(s, hi8, d, d8);
        asm volatile("" ::"v"(d), "v"(d8));
        if ((lane & 7) == 0) {
          uint32_t eo = j * ROW;
          asm volatile("" : "+s"(eo));
          lds_float* acc = acc_lane + eo;
          acc[0] = d;
          acc[8] = d8;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    // flush: lane t maps the sums of its entry into the record (zeros for an entry no pixel took),
    // written back into its LDS row with the slot; stored by the next batch (or after the loop)
    if (mine) {
      float S[GRAD_REC];
      if ((wrote >> lane) & 1ull) {
        const float4 a0 = *reinterpret_cast<const float4*>(&s_acc[lane][0]);
        const float4 a1 = *reinterpret_cast<const float4*>(&s_acc[lane][4]);
        const float4 a2 = *reinterpret_cast<const float4*>(&s_acc[lane][8]);
        const float4 a3 = *reinterpret_cast<const float4*>(&s_acc[lane][12]);
        S[0] = a0.x, S[1] = a0.y, S[2] = a0.z, S[3] = a0.w, S[4] = a1.x, S[5] = a1.y, S[6] = a1.z, S[7] = a1.w;
        S[8] = ((a2.x + a2.y) + (a2.z + a2.w)) + ((a3.x + a3.y) + (a3.z + a3.w));
      } else {
#pragma unroll
        for (int t = 0; t < GRAD_REC; t++) S[t] = 0.0f;
      }
      // S3..S7 are the moments of q about the reference point r; with R = mean - r (dx = u + R):
      // sum q dx = S3 + R.x S8, sum q dx^2 = S5 + 2 R.x S3 + R.x^2 S8, ... in fp64, one rounding to
      // the record (R = 0, nothing to shift, for a splat centred in the tile)
      const float2 R = *reinterpret_cast<const float2*>(&s_br[lane].y);
      const double Rx = R.x, Ry = R.y, q0 = S[8];
      const float m1x = (float)__builtin_fma(Rx, q0, (double)S[3]), m1y = (float)__builtin_fma(Ry, q0, (double)S[4]);
      __builtin_amdgcn_sched_barrier(0);
      const float m2xx = (float)__builtin_fma(Rx, __builtin_fma(Rx, q0, 2.0 * (double)S[3]), (double)S[5]);
      __builtin_amdgcn_sched_barrier(0);
      const float m2xy = (float)__builtin_fma(Rx, __builtin_fma(Ry, q0, (double)S[4]),
                                              __builtin_fma(Ry, (double)S[3], (double)S[6]));
      __builtin_amdgcn_sched_barrier(0);
      const float m2yy = (float)__builtin_fma(Ry, __builtin_fma(Ry, q0, 2.0 * (double)S[4]), (double)S[7]);
      __builtin_amdgcn_sched_barrier(0);
      float4* row = reinterpret_cast<float4*>(&s_acc[lane][0]);
      row[0] = make_float4(S[0], S[1], S[2], -ddelx_dx * (ccx * m1x + ccy * m1y));
      row[1] = make_float4(-ddely_dy * (ccz * m1y + ccy * m1x), -0.5f * m2xx, -0.5f * m2xy, -0.5f * m2yy);
      // S8 = o sum G dL/dalpha (a contributor has o >= 1/255)
      row[2] = make_float4(S[8] != 0.0f ? S[8] / cop : 0.0f, __uint_as_float(slot), 0.0f, 0.0f);
    }
    rec_lanes = cnt;
    __builtin_amdgcn_wave_barrier();  // the next batch overwrites the staged entries
  }
  store_records();
  GS_BWD_TREC(tile, n_eff, t_walked, t_slots);
}

// Longest-first launch order for the backward.  A tile's walk is as long as its largest
// n_contrib (the forward's per-quadrant maxima), which varies ~10x across an image, and dense
// tiles sit together: in index order the last workgroups to start include heavy ones and the
// grid ends on a long tail.  The forward buckets every tile by that length and ranks it in its
// bucket of its XCD group (tile_finish); here each thread places one tile at (bucket base + rank)
// within the group's launch positions, so the heavy tiles start first and the tail is made of
// light ones (list scheduling, LPT).  The order inside a bucket is arbitrary: a tile's outputs do
// not depend on when it runs.
constexpr int ORDER_THREADS = 256;
// Also (always) each tile's record cut: records exist only for a tile's first n_eff instances
// (those its walk reaches, n_eff = its largest n_contrib); tile_cut = 1 + the slot of the last
// of them.  A tile's list is in slot order, so k_sum_records keeps a record of slot s in tile T
// iff s < tile_cut[T] and the backward writes no zero records for the rest.
__global__ __launch_bounds__(ORDER_THREADS) void k_tile_order(const uint32_t* __restrict__ len_hist,
                                                              const uint32_t* __restrict__ tile_brank, uint32_t gx,
                                                              uint32_t gy, uint32_t* __restrict__ order,
                                                              const uint32_t* __restrict__ tile_max,
                                                              const uint2* __restrict__ ranges,
                                                              const uint32_t* __restrict__ point_list,
                                                              uint32_t* __restrict__ tile_cut,
                                                              uint32_t* __restrict__ cut_max) {
  __shared__ uint32_t s_base[ORDER_GROUPS][ORDER_BUCKETS];
  const uint32_t tid = threadIdx.x, t = blockIdx.x * ORDER_THREADS + tid, lane = tid & 63, wid = tid >> 6;
  const uint32_t tiles = gx * gy;
  uint32_t cut = 0;
  if (t < tiles) {
    const uint4 q = reinterpret_cast<const uint4*>(tile_max)[t];
    const uint2 r = ranges[t];
    const uint32_t n_eff = min(max(max(q.x, q.y), max(q.z, q.w)), r.y - r.x);
    cut = n_eff ? point_list[r.x + n_eff - 1] + 1u : 0u;
    tile_cut[t] = cut;
  }
  {
    // the largest cut (all lanes take part in the wave max): k_sum_records stops there -- slots
    // are in depth order, so past it no tile walked an instance
    const uint32_t wm = wave_max_u32(cut);
    if (lane == 0 && wm) atomicMax(cut_max, wm);
  }
  if (!order) return;  // (uniform)
  const uint32_t br = t < tiles ? tile_brank[t] : 0u;
  static_assert(ORDER_BUCKETS == 64 && ORDER_GROUPS == 2 * (ORDER_THREADS / 64), "two groups per wave");
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t g = wid + h * (ORDER_THREADS / 64);
    const uint32_t v = len_hist[g * ORDER_BUCKETS + lane];
    s_base[g][lane] = wave_incl_scan(v) - v;
  }
  lds_barrier();
  // the j-th tile of group g (longest first) takes launch position 8 j + g
  if (t < tiles) {
    const uint32_t g = t % ORDER_GROUPS;
    order[ORDER_GROUPS * (s_base[g][br >> 22] + (br & 0x3FFFFFu)) + g] = t;
  }
}

void bwd_render(int P, const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin, const ImgPtrs& img,
                const float* dL_dpix, float* gradrec, hipStream_t st) {
  const int tiles = c.gx * c.gy;
  uint32_t* order = img.tile_order;
  const uint32_t slots = (uint32_t)tiles;
  GS_LAUNCH("tile_order", k_tile_order, dim3((slots + ORDER_THREADS - 1) / ORDER_THREADS), dim3(ORDER_THREADS), 0, st,
            img.len_hist, img.tile_brank, (uint32_t)c.gx, (uint32_t)c.gy, order, img.tile_max, img.ranges,
            bin.point_list, img.tile_cut, img.cut_max);
  if (exact_exp())
    GS_LAUNCH("render_bwd", k_render_bwd_tw<true>, dim3(slots), dim3(64), 0, st, c, img.ranges, bin.point_list,
              bin.presort_gid, geo.splat, img.final_T, img.n_contrib, img.tile_max, order, dL_dpix, gradrec);
  else
    GS_LAUNCH("render_bwd", k_render_bwd_tw<false>, dim3(slots), dim3(64), 0, st, c, img.ranges, bin.point_list,
              bin.presort_gid, geo.splat, img.final_T, img.n_contrib, img.tile_max, order, dL_dpix, gradrec);
}

// ------------------------------------------------------------------------------------------
// per-Gaussian record sums
//
// Each visible Gaussian owns the contiguous records [offsets[r], offsets[r + 1]) (r = its depth
// rank).  A wave takes 64 consecutive ranks and sweeps their records 64 at a time (coalesced
// loads, no per-Gaussian loop divergence): every lane finds its record's owner by a binary search
// over the 64 offsets held in the lanes, a segmented inclusive wave scan sums the records of one
// owner, and the segment's last lane adds the partial into the owner's fp64 LDS accumulator (a
// large splat's tile partials cancel, so the cross-tile sum is kept in fp64).  The total goes
// back into the owner's first record.  Fixed order throughout: deterministic.
// ------------------------------------------------------------------------------------------
constexpr int SUMREC_WAVES = 4;  // (2 or 8 measured within 2 us at C3)
// one step of the segmented wave scan: v += (shifted v) when the shifted lane has the same owner
// (owners are carried +1 so a lane without a source (0) never matches)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void seg_scan_step(float* v, uint32_t own1) {
  const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)own1, CTRL, ROW_MASK, 0xF, false);
  const float f = o == own1 ? 1.0f : 0.0f;
#pragma unroll
  for (int c = 0; c < GRAD_REC; c++) v[c] = __builtin_fmaf(dpp_f<CTRL, ROW_MASK>(v[c]), f, v[c]);
}

__global__ __launch_bounds__(64 * SUMREC_WAVES) void k_sum_records(const uint32_t* __restrict__ counters,
                                                                   const uint32_t* __restrict__ offsets,
                                                                   const uint32_t* __restrict__ sorted_gid,
                                                                   const uint32_t* __restrict__ slot_tile,
                                                                   const uint32_t* __restrict__ tile_cut,
                                                                   const uint32_t* __restrict__ cut_max,
                                                                   const float* __restrict__ gradrec,
                                                                   float* __restrict__ gsum, uint32_t P) {
  __shared__ double s_acc[SUMREC_WAVES][64][GRAD_REC];
  __shared__ unsigned long long s_mark[SUMREC_WAVES];
  const uint32_t V = counters[CNT_V], I = counters[CNT_I];
  const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t r0 = (blockIdx.x * SUMREC_WAVES + wid) * 64;
  if (counters[CNT_ERR] & ERR_INVALID) {
    // the forward's instance list is invalid (reported by the host): no valid records, zero sums
    if (r0 + lane < P)
      for (int c = 0; c < GRAD_REC; c++) gsum[(size_t)(r0 + lane) * GRAD_REC + c] = 0.0f;
    return;
  }
  if (r0 >= V) return;  // wave-uniform; the kernel has no workgroup barrier
  const uint32_t nr = min(64u, V - r0);
  const uint32_t my_off = lane < nr ? offsets[r0 + lane] : 0xFFFFFFFFu;
  const uint32_t S0 = (uint32_t)__shfl((int)my_off, 0, 64);
  // the wave's records end at its last owner's end or at the largest tile cut, whichever is first
  const uint32_t S1 = min((r0 + 64 < V) ? offsets[r0 + 64] : I, *cut_max);
#pragma unroll
  for (int c = 0; c < GRAD_REC; c++) s_acc[wid][lane][c] = 0.0;
  const unsigned long long le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  uint32_t jbase = 0xFFFFFFFFu;  // (number of owners starting before `base`) - 1
  // records of the next chunk are loaded one chunk ahead (their HBM latency overlaps this chunk)
  float vn[GRAD_REC];
  unsigned long long hn;  // lanes of the next chunk that hold a record
  {
    const uint32_t kk = S0 + lane;
#pragma unroll
    for (int c = 0; c < GRAD_REC; c++) vn[c] = 0.0f;
    const bool h = kk < S1 && kk < tile_cut[slot_tile[kk]];
    if (h) load_rec(gradrec + (size_t)kk * GRAD_REC, vn);
    hn = __ballot(h);
  }
  for (uint32_t base = S0; base < S1; base += 64) {
    float v[GRAD_REC];
#pragma unroll
    for (int c = 0; c < GRAD_REC; c++) v[c] = vn[c];
    const unsigned long long hc = hn;
    if (base + 64 < S1) {
      // records past their tile's cut were never written: zeros (no load)
      const uint32_t kn = base + 64 + lane;
#pragma unroll
      for (int c = 0; c < GRAD_REC; c++) vn[c] = 0.0f;
      const bool h = kn < S1 && kn < tile_cut[slot_tile[kn]];
      if (h) load_rec(gradrec + (size_t)kn * GRAD_REC, vn);
      hn = __ballot(h);
    }
    if (hc == 0) {
      // no record in the chunk (every slot behind its tile's walk, as for most of a dense
      // scene's instances): only count the owners that start in it
      jbase += (uint32_t)__popcll(__ballot(my_off >= base && my_off < base + 64));
      continue;
    }
    // slots of the chunk that start an owner -> bit mask -> owner of my slot by popcount
    if (lane == 0) s_mark[wid] = 0ull;
    __builtin_amdgcn_wave_barrier();
    if (my_off >= base && my_off < base + 64) atomicOr(&s_mark[wid], 1ull << (my_off - base));
    __builtin_amdgcn_wave_barrier();
    const unsigned long long B = s_mark[wid];
    const uint32_t own = jbase + (uint32_t)__popcll(B & le);
    jbase += (uint32_t)__popcll(B);
    const uint32_t k = base + lane;
    const bool valid = k < S1;
#pragma unroll
    for (int c = 0; c < GRAD_REC; c++) v[c] = valid ? v[c] : 0.0f;
    const uint32_t own1 = valid ? own + 1 : 0;
    seg_scan_step<0x111, 0xF>(v, own1);  // row_shr:1
    seg_scan_step<0x112, 0xF>(v, own1);  // row_shr:2
    seg_scan_step<0x114, 0xF>(v, own1);  // row_shr:4
    seg_scan_step<0x118, 0xF>(v, own1);  // row_shr:8
    seg_scan_step<0x142, 0xA>(v, own1);  // row_bcast:15 -> rows 1, 3
    seg_scan_step<0x143, 0xC>(v, own1);  // row_bcast:31 -> rows 2, 3
    const uint32_t next1 = (uint32_t)__shfl_down((int)own1, 1, 64);
    if (valid && (lane == 63 || next1 != own1)) {
#pragma unroll
      for (int c = 0; c < GRAD_REC; c++) atomicAdd(&s_acc[wid][own][c], (double)v[c]);  // ds_add_f64: one lane per owner, fixed order
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane < nr) {
    const size_t gid = sorted_gid[r0 + lane];
#pragma unroll
    for (int c = 0; c < GRAD_REC; c++) gsum[gid * GRAD_REC + c] = (float)s_acc[wid][lane][c];
  }
}

static void launch_sum_records(const GaussianArgs& g, const GeomPtrs& geo, const BinPtrs& bin, const ImgPtrs& img,
                               float* gradrec, uint32_t R, hipStream_t st) {
  GS_LAUNCH("sum_records", k_sum_records, dim3((g.P + 64 * SUMREC_WAVES - 1) / (64 * SUMREC_WAVES)),
            dim3(64 * SUMREC_WAVES), 0, st, geo.counters, geo.offsets, geo.sorted_gid, bin.slot_tile, img.tile_cut,
            img.cut_max, gradrec, geo.gsum, (uint32_t)g.P);
}

// ------------------------------------------------------------------------------------------
// preprocess backward
// ------------------------------------------------------------------------------------------

// SH backward for one Gaussian (order identical to oracle/gs_oracle.c sh_bwd_one).
// `row` is the Gaussian's SH row (3M floats) staged in LDS, or (REG) its first 3K floats in
// registers; on return it holds dL/dsh (REG: the caller zero-fills [3K, 3M)).
// ACC (multi-view pass): `row` is left alone and dL/dsh goes to acc[0, 3K): written when `first`,
// else added (fp32 acc + new, the arithmetic of a bucket's `grad += g`).
template <int DEG, bool REG = false, bool ACC = false>
__device__ __forceinline__ void sh_backward(float* row, int M, float vx, float vy, float vz,
                                            uint32_t clamped, const float* dcol, float* dmean,
                                            float* acc = nullptr, bool first = true) {
  constexpr int K = (DEG + 1) * (DEG + 1);
  const float len = sqrtf(vx * vx + vy * vy + vz * vz);
  const float x = vx / len, y = vy / len, z = vz / len;
  float g[3];
#pragma unroll
  for (int ch = 0; ch < 3; ch++) g[ch] = ((clamped >> ch) & 1) ? 0.0f : dcol[ch];
  const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
  float b[16];
  b[0] = SH_C0;
  if (DEG > 0) {
    b[1] = -SH_C1 * y;
    b[2] = SH_C1 * z;
    b[3] = -SH_C1 * x;
  }
  if (DEG > 1) {
    b[4] = SH_C20 * xy;
    b[5] = SH_C21 * yz;
    b[6] = SH_C22 * (2.0f * zz - xx - yy);
    b[7] = SH_C23 * xz;
    b[8] = SH_C24 * (xx - yy);
  }
  if (DEG > 2) {
    b[9] = (SH_C30 * y) * (3.0f * xx - yy);
    b[10] = (SH_C31 * xy) * z;
    b[11] = (SH_C32 * y) * (4.0f * zz - xx - yy);
    b[12] = (SH_C33 * z) * (2.0f * zz - 3.0f * xx - 3.0f * yy);
    b[13] = (SH_C34 * x) * (4.0f * zz - xx - yy);
    b[14] = (SH_C35 * z) * (xx - yy);
    b[15] = (SH_C36 * x) * (xx - 3.0f * yy);
  }
  float ddx[3] = {0.f, 0.f, 0.f}, ddy[3] = {0.f, 0.f, 0.f}, ddz[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < 3; ch++) {
#define S(k) row[3 * (k) + ch]
    if (DEG > 0) {
      ddx[ch] = -SH_C1 * S(3);
      ddy[ch] = -SH_C1 * S(1);
      ddz[ch] = SH_C1 * S(2);
      if (DEG > 1) {
        ddx[ch] = ddx[ch] + (SH_C20 * y) * S(4) + (SH_C22 * (-2.f * x)) * S(6) + (SH_C23 * z) * S(7) +
                  (SH_C24 * (2.f * x)) * S(8);
        ddy[ch] = ddy[ch] + (SH_C20 * x) * S(4) + (SH_C21 * z) * S(5) + (SH_C22 * (-2.f * y)) * S(6) +
                  (SH_C24 * (-2.f * y)) * S(8);
        ddz[ch] = ddz[ch] + (SH_C21 * y) * S(5) + (SH_C22 * (4.f * z)) * S(6) + (SH_C23 * x) * S(7);
        if (DEG > 2) {
          ddx[ch] = ddx[ch] + (SH_C30 * (6.f * xy)) * S(9) + (SH_C31 * yz) * S(10) + (SH_C32 * (-2.f * xy)) * S(11) +
                    (SH_C33 * (-6.f * xz)) * S(12) + (SH_C34 * (-3.f * xx + 4.f * zz - yy)) * S(13) +
                    (SH_C35 * (2.f * xz)) * S(14) + (SH_C36 * (3.f * (xx - yy))) * S(15);
          ddy[ch] = ddy[ch] + (SH_C30 * (3.f * (xx - yy))) * S(9) + (SH_C31 * xz) * S(10) +
                    (SH_C32 * (-3.f * yy + 4.f * zz - xx)) * S(11) + (SH_C33 * (-6.f * yz)) * S(12) +
                    (SH_C34 * (-2.f * xy)) * S(13) + (SH_C35 * (-2.f * yz)) * S(14) + (SH_C36 * (-6.f * xy)) * S(15);
          ddz[ch] = ddz[ch] + (SH_C31 * xy) * S(10) + (SH_C32 * (8.f * yz)) * S(11) +
                    (SH_C33 * (3.f * (2.f * zz - xx - yy))) * S(12) + (SH_C34 * (8.f * xz)) * S(13) +
                    (SH_C35 * (xx - yy)) * S(14);
        }
      }
    }
#undef S
  }
#pragma unroll
  for (int k = 0; k < K; k++)
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
      if constexpr (ACC)
        acc[3 * k + ch] = first ? b[k] * g[ch] : acc[3 * k + ch] + b[k] * g[ch];
      else
        row[3 * k + ch] = b[k] * g[ch];
    }
  if (!REG && !ACC)
    for (int k = 3 * K; k < 3 * M; k++) row[k] = 0.0f;
  const float d0 = ddx[0] * g[0] + ddx[1] * g[1] + ddx[2] * g[2];
  const float d1 = ddy[0] * g[0] + ddy[1] * g[1] + ddy[2] * g[2];
  const float d2 = ddz[0] * g[0] + ddz[1] * g[1] + ddz[2] * g[2];
  const float sum2 = vx * vx + vy * vy + vz * vz;
  const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
  dmean[0] = ((sum2 - vx * vx) * d0 - vy * vx * d1 - vz * vx * d2) * invsum32;
  dmean[1] = (-vx * vy * d0 + (sum2 - vy * vy) * d1 - vz * vy * d2) * invsum32;
  dmean[2] = (-vx * vz * d0 - vy * vz * d1 + (sum2 - vz * vz) * d2) * invsum32;
}

// cov3D backward (order identical to oracle/gs_oracle.c cov3d_bwd_one)
__device__ __forceinline__ void cov3d_backward(float sx, float sy, float sz, float mod, float qr, float qx, float qy,
                                               float qz, const float* dcov, float* dscale, float* drot) {
  mat3 R = quat_rot(qr, qx, qy, qz);
  float sv[3] = {mod * sx, mod * sy, mod * sz};
  float m[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int a = 0; a < 3; a++) m[i][a] = sv[i] * R.m[a][i];
  float g[3][3];
  g[0][0] = dcov[0];
  g[1][1] = dcov[3];
  g[2][2] = dcov[5];
  g[0][1] = g[1][0] = 0.5f * dcov[1];
  g[0][2] = g[2][0] = 0.5f * dcov[2];
  g[1][2] = g[2][1] = 0.5f * dcov[4];
  float dm[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int a = 0; a < 3; a++) dm[i][a] = 2.0f * (m[i][0] * g[0][a] + m[i][1] * g[1][a] + m[i][2] * g[2][a]);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    float ds = R.m[0][i] * dm[i][0] + R.m[1][i] * dm[i][1] + R.m[2][i] * dm[i][2];
    dscale[i] = ds * mod;
  }
  float dR[3][3];
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int i = 0; i < 3; i++) dR[a][i] = sv[i] * dm[i][a];
  const float r = qr, x = qx, y = qy, z = qz;
  drot[0] = 2.f * z * (dR[1][0] - dR[0][1]) + 2.f * y * (dR[0][2] - dR[2][0]) + 2.f * x * (dR[2][1] - dR[1][2]);
  drot[1] = 2.f * y * (dR[0][1] + dR[1][0]) + 2.f * z * (dR[0][2] + dR[2][0]) + 2.f * r * (dR[2][1] - dR[1][2]) -
            4.f * x * (dR[1][1] + dR[2][2]);
  drot[2] = 2.f * x * (dR[0][1] + dR[1][0]) + 2.f * r * (dR[0][2] - dR[2][0]) + 2.f * z * (dR[1][2] + dR[2][1]) -
            4.f * y * (dR[0][0] + dR[2][2]);
  drot[3] = 2.f * r * (dR[1][0] - dR[0][1]) + 2.f * x * (dR[0][2] + dR[2][0]) + 2.f * y * (dR[1][2] + dR[2][1]) -
            4.f * z * (dR[0][0] + dR[1][1]);
}

// Camera-dependent part of the per-Gaussian backward (upstream computeCov2DCUDA + the projection
// term of preprocessCUDA's backward, order identical to oracle/gs_oracle.c): conic gradient ->
// cov2D -> cov3D gradient (dcv) and the view-space mean gradient incl. the NDC-mean term (dmean).
__device__ __forceinline__ void camera_grads(const CameraArgs& c, float px, float py, float pz, const float* cov3,
                                             float dcon0, float dcon1, float dcon2, float dm2x, float dm2y,
                                             float* dcv, float* dmean) {
#pragma unroll
  for (int k = 0; k < 6; k++) dcv[k] = 0.f;
  // conic -> cov2D -> cov3D and view-space mean
  const Cov2D cv = cov2d(c.view, px, py, pz, cov3, c.fx, c.fy, c.tanfovx, c.tanfovy);
  const float A = cv.a, Bv = cv.b, Cc = cv.c;
  const float denom = A * Cc - Bv * Bv;
  float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
  const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
  const float(*Tm)[3] = cv.T;
  if (denom2inv != 0.0f) {
    dL_da = denom2inv * (-Cc * Cc * dcon0 + 2.f * Bv * Cc * dcon1 + (denom - A * Cc) * dcon2);
    dL_dc = denom2inv * (-A * A * dcon2 + 2.f * A * Bv * dcon1 + (denom - A * Cc) * dcon0);
    dL_db = denom2inv * 2.f * (Bv * Cc * dcon0 - (denom + 2.f * Bv * Bv) * dcon1 + A * Bv * dcon2);
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
  const float V[3][3] = {{cov3[0], cov3[1], cov3[2]}, {cov3[1], cov3[3], cov3[4]}, {cov3[2], cov3[4], cov3[5]}};
  float dT0[3], dT1[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const float tv0 = Tm[0][0] * V[r][0] + Tm[0][1] * V[r][1] + Tm[0][2] * V[r][2];
    const float tv1 = Tm[1][0] * V[r][0] + Tm[1][1] * V[r][1] + Tm[1][2] * V[r][2];
    dT0[r] = 2.f * tv0 * dL_da + tv1 * dL_db;
    dT1[r] = 2.f * tv1 * dL_dc + tv0 * dL_db;
  }
  const float* v = c.view;
  const float dJ00 = v[0] * dT0[0] + v[4] * dT0[1] + v[8] * dT0[2];
  const float dJ02 = v[2] * dT0[0] + v[6] * dT0[1] + v[10] * dT0[2];
  const float dJ11 = v[1] * dT1[0] + v[5] * dT1[1] + v[9] * dT1[2];
  const float dJ12 = v[2] * dT1[0] + v[6] * dT1[1] + v[10] * dT1[2];
  const float tz = 1.f / cv.tz, tz2 = tz * tz, tz3 = tz2 * tz;
  const float dL_dtx = cv.gmx * -c.fx * tz2 * dJ02;
  const float dL_dty = cv.gmy * -c.fy * tz2 * dJ12;
  const float dL_dtz =
      -c.fx * tz2 * dJ00 - c.fy * tz2 * dJ11 + (2.f * c.fx * cv.tx) * tz3 * dJ02 + (2.f * c.fy * cv.ty) * tz3 * dJ12;
  dmean[0] = v[0] * dL_dtx + v[1] * dL_dty + v[2] * dL_dtz;
  dmean[1] = v[4] * dL_dtx + v[5] * dL_dty + v[6] * dL_dtz;
  dmean[2] = v[8] * dL_dtx + v[9] * dL_dty + v[10] * dL_dtz;
  // projection: NDC mean2D -> mean3D
  const float* P = c.proj;
  const float hw = xf44w(P, px, py, pz);
  const float m_w = 1.0f / (hw + 0.0000001f);
  const float mul1 = (P[0] * px + P[4] * py + P[8] * pz + P[12]) * m_w * m_w;
  const float mul2 = (P[1] * px + P[5] * py + P[9] * pz + P[13]) * m_w * m_w;
  const float pm0 = (P[0] * m_w - P[3] * mul1) * dm2x + (P[1] * m_w - P[3] * mul2) * dm2y;
  const float pm1 = (P[4] * m_w - P[7] * mul1) * dm2x + (P[5] * m_w - P[7] * mul2) * dm2y;
  const float pm2 = (P[8] * m_w - P[11] * mul1) * dm2x + (P[9] * m_w - P[11] * mul2) * dm2y;
  dmean[0] = dmean[0] + pm0;
  dmean[1] = dmean[1] + pm1;
  dmean[2] = dmean[2] + pm2;
}

// one gradient output element: written, or (GS_ACC bit set for the output) added to the caller's
// buffer as autograd's `grad += g` does (fp32 old + new)
__device__ __forceinline__ void gput(float* p, size_t k, float v, uint32_t acc, uint32_t bit) {
  p[k] = (acc & bit) ? p[k] + v : v;
}

// One visible Gaussian's gradients from its record sum (upstream's preprocess backward, order
// identical to oracle/gs_oracle.c): the screen-space terms, conic -> cov2D -> cov3D / mean, the
// projection, SH (DEG >= 0: dL/dsh into `row`, see sh_backward) and scale / rotation.  Each result
// goes to `sink` as soon as it is formed (the stores of the plain path stay where they were, which
// keeps the values' live ranges -- and the kernels' register counts -- short).
template <int DEG, bool REG, class Sink>
__device__ __forceinline__ void preprocess_bwd_visible(int i, const GaussianArgs& g, const CameraArgs& c,
                                                       const uint8_t* __restrict__ clamped,
                                                       const float* __restrict__ gsum, float* row, bool want_sr,
                                                       Sink& sink) {
  // the Gaussian's per-tile records, summed by k_sum_records (index order: coalesced here)
  const float* rec = gsum + (size_t)i * GRAD_REC;
  float a[GRAD_REC];
#pragma unroll
  for (int k = 0; k < GRAD_REC; k++) a[k] = rec[k];
  const float dcol[3] = {a[0], a[1], a[2]};
  const float dm2x = a[3], dm2y = a[4];
  const float dcon0 = a[5], dcon1 = a[6], dcon2 = a[7];
  sink.color(dcol);
  sink.mean2d(dm2x, dm2y);
  sink.opacity(a[8]);
  const float px = g.means3D[3 * i], py = g.means3D[3 * i + 1], pz = g.means3D[3 * i + 2];
  float cov3[6];
  if (g.cov3D) {
#pragma unroll
    for (int k = 0; k < 6; k++) cov3[k] = g.cov3D[6 * i + k];
  } else {
    cov3d(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2], g.scale_modifier, g.rotations[4 * i],
          g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3], cov3);
  }
  float dcv[6], dmean[3];
  camera_grads(c, px, py, pz, cov3, dcon0, dcon1, dcon2, dm2x, dm2y, dcv, dmean);
  sink.cov3d(dcv);
  if (DEG >= 0) {
    float shm[3];
    const float vx = px - c.campos[0], vy = py - c.campos[1], vz = pz - c.campos[2];
    sh_backward<(DEG < 0 ? 0 : DEG), REG>(row, g.M, vx, vy, vz, clamped[i], dcol, shm);
    dmean[0] = dmean[0] + shm[0];
    dmean[1] = dmean[1] + shm[1];
    dmean[2] = dmean[2] + shm[2];
  }
  sink.mean3d(dmean);
  if (!g.cov3D && want_sr) {
    float ds[3], dr[4];
    cov3d_backward(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2], g.scale_modifier, g.rotations[4 * i],
                   g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3], dcv, ds, dr);
    sink.scale_rot(ds, dr);
  }
}

// the plain path's sink: the caller's gradient outputs, written or (GS_ACC_* bits) added
struct StoreSink {
  const GradOut& out;
  const int i;
  __device__ void color(const float* d) {
    if (out.dcolor)
      for (int k = 0; k < 3; k++) gput(out.dcolor, 3 * i + k, d[k], out.acc, GS_ACC_COLORS);
  }
  __device__ void mean2d(float x, float y) {
    gput(out.dmean2D, 3 * i, x, out.acc, GS_ACC_MEANS2D);
    gput(out.dmean2D, 3 * i + 1, y, out.acc, GS_ACC_MEANS2D);
    gput(out.dmean2D, 3 * i + 2, 0.0f, out.acc, GS_ACC_MEANS2D);
  }
  __device__ void opacity(float d) { gput(out.dopacity, i, d, out.acc, GS_ACC_OPACITY); }
  __device__ void cov3d(const float* d) {
    if (out.dcov3D)
#pragma unroll
      for (int k = 0; k < 6; k++) gput(out.dcov3D, 6 * i + k, d[k], out.acc, GS_ACC_COV3D);
  }
  __device__ void mean3d(const float* d) {
#pragma unroll
    for (int k = 0; k < 3; k++) gput(out.dmean3D, 3 * i + k, d[k], out.acc, GS_ACC_MEANS3D);
  }
  __device__ void scale_rot(const float* ds, const float* dr) {
#pragma unroll
    for (int k = 0; k < 3; k++) gput(out.dscale, 3 * i + k, ds[k], out.acc, GS_ACC_SCALES);
#pragma unroll
    for (int k = 0; k < 4; k++) gput(out.drot, 4 * i + k, dr[k], out.acc, GS_ACC_ROTATIONS);
  }
};

template <int DEG, bool REG = false>
__device__ __forceinline__ void preprocess_bwd_one(int i, const GaussianArgs& g, const CameraArgs& c,
                                                   const uint32_t* __restrict__ tiles,
                                                   const uint8_t* __restrict__ clamped,
                                                   const float* __restrict__ gsum, const GradOut& out,
                                                   float* row) {
  const uint32_t cnt = tiles[i];
  const uint32_t acc = out.acc;
  if (cnt == 0) {
    // invisible: every gradient is zero (upstream: zero-initialised outputs, radii == 0 skipped);
    // an accumulated output keeps what it holds (+ 0)
    if (!(acc & GS_ACC_MEANS2D)) {
      out.dmean2D[3 * i] = 0.f;
      out.dmean2D[3 * i + 1] = 0.f;
      out.dmean2D[3 * i + 2] = 0.f;
    }
    if (out.dcolor && !(acc & GS_ACC_COLORS)) {
      out.dcolor[3 * i] = 0.f;
      out.dcolor[3 * i + 1] = 0.f;
      out.dcolor[3 * i + 2] = 0.f;
    }
    if (!(acc & GS_ACC_OPACITY)) out.dopacity[i] = 0.f;
    if (!(acc & GS_ACC_MEANS3D)) {
      out.dmean3D[3 * i] = 0.f;
      out.dmean3D[3 * i + 1] = 0.f;
      out.dmean3D[3 * i + 2] = 0.f;
    }
    if (out.dcov3D && !(acc & GS_ACC_COV3D))
      for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = 0.f;
    if (DEG >= 0 && !REG)
      for (int k = 0; k < 3 * g.M; k++) row[k] = 0.f;
    if (DEG >= 0 && REG && !(acc & GS_ACC_SH))
      for (int k = 0; k < 3 * g.M; k++) out.dsh[(size_t)i * 3 * g.M + k] = 0.f;
    if (out.dscale && !(acc & GS_ACC_SCALES))
      for (int k = 0; k < 3; k++) out.dscale[3 * i + k] = 0.f;
    if (out.drot && !(acc & GS_ACC_ROTATIONS))
      for (int k = 0; k < 4; k++) out.drot[4 * i + k] = 0.f;
    return;
  }
  StoreSink sink{out, i};
  preprocess_bwd_visible<DEG, REG>(i, g, c, clamped, gsum, row, out.dscale && out.drot, sink);
}

// colours precomputed (no SH gradient)
__global__ __launch_bounds__(256) void k_preprocess_bwd_colors(GaussianArgs g, CameraArgs c,
                                                               const uint32_t* __restrict__ tiles,
                                                               const uint8_t* __restrict__ clamped,
                                                               const float* __restrict__ gsum, GradOut out) {
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  if (i < g.P) preprocess_bwd_one<-1>(i, g, c, tiles, clamped, gsum, out, nullptr);
}

// Register variant: the lane loads its own SH row (first 3K floats, 16-B loads when
// the rows allow) and stores dL/dsh the same way; no LDS, so occupancy is set by registers alone.
template <int DEG, bool SPLIT = false>  // SPLIT: SH rows from g.shs (features_dc) + g.shs_rest
__global__ __launch_bounds__(256) void k_preprocess_bwd_reg(GaussianArgs g, CameraArgs c,
                                                            const uint32_t* __restrict__ tiles,
                                                            const uint8_t* __restrict__ clamped,
                                                            const float* __restrict__ gsum, GradOut out) {
  constexpr int KF = 3 * (DEG + 1) * (DEG + 1);
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  if (i >= g.P) return;
  const int rowf = 3 * g.M;
  const float* src = g.shs + (size_t)i * rowf;
  float* dst = out.dsh + (size_t)i * rowf;
  const bool vec = (KF & 3) == 0 && (rowf & 3) == 0 && ((((uintptr_t)g.shs) | ((uintptr_t)out.dsh)) & 15) == 0;
  // dL/dsh rows stay [P, M, 3] whether or not the inputs are split
  const bool vec_out = SPLIT ? (KF & 3) == 0 && (rowf & 3) == 0 && (((uintptr_t)out.dsh) & 15) == 0 : vec;
  float row[KF];
  if constexpr (SPLIT) {  // split rows: features_dc [P, 1, 3] + features_rest [P, M - 1, 3], 12-B pieces
    const F3 d = reinterpret_cast<const F3*>(g.shs)[i];
    row[0] = d.a, row[1] = d.b, row[2] = d.c;
    const F3* r3 = reinterpret_cast<const F3*>(g.shs_rest + (size_t)i * (rowf - 3));
#pragma unroll
    for (int j = 0; j < KF / 3 - 1; j++) {
      const F3 t = r3[j];
      row[3 + 3 * j] = t.a, row[4 + 3 * j] = t.b, row[5 + 3 * j] = t.c;
    }
  } else if (vec) {
#pragma unroll
    for (int q = 0; q < KF / 4; q++) {
      const float4 v = reinterpret_cast<const float4*>(src)[q];
      row[4 * q] = v.x, row[4 * q + 1] = v.y, row[4 * q + 2] = v.z, row[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < KF; k++) row[k] = src[k];
  }
  // invisible: every gradient (dL/dsh too) is written as zero by this call; split from the
  // visible call so each inlined copy is specialised (measured 113 -> 109.5 us at C3)
  if (tiles[i] == 0) {
    preprocess_bwd_one<DEG, true>(i, g, c, tiles, clamped, gsum, out, row);
    return;
  }
  preprocess_bwd_one<DEG, true>(i, g, c, tiles, clamped, gsum, out, row);
  if (out.acc & GS_ACC_SH) {  // (uniform) multi-view accumulation: dL/dsh += this view's
    if (vec_out) {
#pragma unroll
      for (int q = 0; q < KF / 4; q++) {
        const float4 o = reinterpret_cast<const float4*>(dst)[q];
        reinterpret_cast<float4*>(dst)[q] =
            make_float4(o.x + row[4 * q], o.y + row[4 * q + 1], o.z + row[4 * q + 2], o.w + row[4 * q + 3]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < KF; k++) dst[k] = dst[k] + row[k];
    }
    return;  // coefficients past (D + 1)^2 get + 0
  }
  if (vec_out) {
#pragma unroll
    for (int q = 0; q < KF / 4; q++)
      reinterpret_cast<float4*>(dst)[q] = make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < KF; k++) dst[k] = row[k];
  }
  for (int k = KF; k < rowf; k++) dst[k] = 0.0f;
}

// Staged variant (degree 3 with whole 48-float rows, dL/dsh written not added):
// the workgroup's 256 SH rows come in (stage_sh_rows48) and its 256 dL/dsh rows go out as
// contiguous blocks of coalesced 16-B accesses through LDS, instead of 12-16 lane-strided loads /
// stores per lane each touching 64 cache lines; the lane's row moves between LDS and registers
// with 16-B reads / writes.  53 KB of LDS per workgroup (3 waves per SIMD, the register variant
// ran at 4): 124 -> 100 us at C3.  (Keeping the row in LDS for the SH backward instead of
// registers: 101 us; the same staging in the forward preprocess: 80 -> 85 us, not used.)
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_preprocess_bwd_stage(GaussianArgs g, CameraArgs c,
                                                              const uint32_t* __restrict__ tiles,
                                                              const uint8_t* __restrict__ clamped,
                                                              const float* __restrict__ gsum, GradOut out) {
  constexpr int KF = 48, Q = KF / 4;  // launched for degree 3 with M == 16 only
  __shared__ __attribute__((aligned(16))) float s_rows[256 * SH_STAGE_ROW];
  const int i0 = blockIdx.x * 256, t = (int)threadIdx.x, i = i0 + t;
  const int nG = g.P - i0 < 256 ? g.P - i0 : 256;
  stage_sh_rows48<SPLIT>(g, i0, nG, s_rows);
  lds_barrier();
  const bool live = i < g.P;
  if (live) {
    float row[KF];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const float4 r4 = lds_ld16(&s_rows[t * SH_STAGE_ROW + 4 * q]);
      row[4 * q] = r4.x, row[4 * q + 1] = r4.y, row[4 * q + 2] = r4.z, row[4 * q + 3] = r4.w;
    }
    // dL/dsh leaves through LDS: the per-Gaussian call must not store it (GS_ACC_SH set on its
    // copy of the outputs; that bit only gates the SH rows)
    GradOut o = out;
    o.acc |= GS_ACC_SH;
    if (tiles[i] == 0) {
      preprocess_bwd_one<3, true>(i, g, c, tiles, clamped, gsum, o, row);
#pragma unroll
      for (int k = 0; k < KF; k++) row[k] = 0.0f;
    } else {
      preprocess_bwd_one<3, true>(i, g, c, tiles, clamped, gsum, o, row);
    }
#pragma unroll
    for (int q = 0; q < Q; q++)
      *reinterpret_cast<float4*>(&s_rows[t * SH_STAGE_ROW + 4 * q]) =
          make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
  }
  lds_barrier();
  float4* dst4 = reinterpret_cast<float4*>(out.dsh + (size_t)i0 * KF);
  const int n4 = nG * Q;
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const int f = t + 256 * q;
    if (f < n4) {
      const int r = f / Q;
      dst4[f] = *reinterpret_cast<const float4*>(&s_rows[r * SH_STAGE_ROW + 4 * (f - r * Q)]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// The per-Gaussian half of one view's backward fused with the optimizer step of GaussianModel's six
// parameter groups (gs_backward_gaussians_adam, the opt-in train step of gs_train_step).
//
// The unfused train step writes every Gaussian's 59-float gradient row (k_preprocess_bwd_stage,
// 236 MB at 1M Gaussians) and reads it back in k_adam.  Here the workgroup's 256 Gaussians get
// their gradients in registers (xyz, opacity, scaling, rotation) and in LDS (the SH rows, staged as
// in k_preprocess_bwd_stage), apply the adjoint of render()'s activations to the raw parameters
// and run Adam on them directly: the gradient rows never touch HBM.  Same floats as the stage
// kernel followed by k_adam in its activated modes (the same device functions, operation for
// operation): parameters and moments are bit-identical to the unfused step (test_train_step.py).
// M = 16 split SH rows, 16-B aligned, any active degree; scales / rotations activated.
// ------------------------------------------------------------------------------------------
struct RegSink {
  float dop, dmean[3] = {0.f, 0.f, 0.f}, ds[3] = {0.f, 0.f, 0.f}, dr[4] = {0.f, 0.f, 0.f, 0.f};
  __device__ void color(const float*) {}
  __device__ void mean2d(float, float) {}  // written by the view's k_mean2d_grad (gs_backward_render)
  __device__ void opacity(float d) { dop = d; }
  __device__ void cov3d(const float*) {}
  __device__ void mean3d(const float* d) {
#pragma unroll
    for (int k = 0; k < 3; k++) dmean[k] = d[k];
  }
  __device__ void scale_rot(const float* s, const float* r) {
#pragma unroll
    for (int k = 0; k < 3; k++) ds[k] = s[k];
#pragma unroll
    for (int k = 0; k < 4; k++) dr[k] = r[k];
  }
};

typedef float v4f __attribute__((ext_vector_type(4)));

// The Adam step of one float4 of a workgroup's features_dc / features_rest block: the gradients
// come from the staged dL/dsh rows (column `off` + col of row r, the identity adjoint of the SH
// concatenation).  Loads of p, m, v for the whole batch are issued before any update so that
// the batch's HBM latency overlaps (the stores could alias the loads as far as the compiler knows).
template <int NB, int W>  // NB float4s per thread per batch, W floats per Gaussian row of the tensor
__device__ __forceinline__ void adam_sh_block(const FusedAdamArgs& a, int tk, int i0, int nG, int t,
                                              const float* s_rows) {
  constexpr int OFF = W == 3 ? 0 : 3;
  const int n = nG * W, n4 = n >> 2;
  float* p = a.p[tk] + (size_t)i0 * W;
  float* m = a.m[tk] + (size_t)i0 * W;
  float* v = a.v[tk] + (size_t)i0 * W;
  const float nss = a.nss[tk], bc2s = a.bc2s[tk], wd = a.wd[tk];
  for (int f0 = t; f0 < n4; f0 += 256 * NB) {
    v4f P[NB], M[NB], V[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int f = f0 + 256 * b;
      if (f < n4) {
        P[b] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p) + f);
        M[b] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(m) + f);
        V[b] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(v) + f);
      }
    }
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int f = f0 + 256 * b;
      if (f < n4) {
        int e = 4 * f, r = e / W, col = e - r * W;
        float pp[4] = {P[b].x, P[b].y, P[b].z, P[b].w}, mm[4] = {M[b].x, M[b].y, M[b].z, M[b].w},
              vv[4] = {V[b].x, V[b].y, V[b].z, V[b].w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          adam_update(pp[j], s_rows[r * SH_STAGE_ROW + OFF + col], mm[j], vv[j], a.k, nss, bc2s, wd);
          if (++col == W) col = 0, r++;
        }
        __builtin_nontemporal_store((v4f){pp[0], pp[1], pp[2], pp[3]}, reinterpret_cast<v4f*>(p) + f);
        __builtin_nontemporal_store((v4f){mm[0], mm[1], mm[2], mm[3]}, reinterpret_cast<v4f*>(m) + f);
        __builtin_nontemporal_store((v4f){vv[0], vv[1], vv[2], vv[3]}, reinterpret_cast<v4f*>(v) + f);
      }
    }
  }
  // tail of a partial last block (n not a multiple of 4)
  for (int e = 4 * n4 + t; e < n; e += 256) {
    const int r = e / W;
    float pe = p[e], me = m[e], ve = v[e];
    adam_update(pe, s_rows[r * SH_STAGE_ROW + OFF + (e - r * W)], me, ve, a.k, nss, bc2s, wd);
    p[e] = pe, m[e] = me, v[e] = ve;
  }
}

template <int DEG>
__global__ __launch_bounds__(256) void k_preprocess_bwd_adam(GaussianArgs g, CameraArgs c,
                                                             const uint32_t* __restrict__ tiles,
                                                             const uint8_t* __restrict__ clamped,
                                                             const float* __restrict__ gsum, FusedAdamArgs a) {
  constexpr int KF = 48, Q = KF / 4;  // M == 16 rows; the active degree DEG uses the first 3 (DEG + 1)^2
  constexpr int K3 = 3 * (DEG + 1) * (DEG + 1);
  __shared__ __attribute__((aligned(16))) float s_rows[256 * SH_STAGE_ROW];
  // an invalid forward (capacity overflow, look-back timeout, culled prefiltered point): no update
  // (the host raises when it reads the flags; the step counts are committed only after that)
  if (*a.err != 0u) return;  // (uniform)
  const int i0 = blockIdx.x * 256, t = (int)threadIdx.x, i = i0 + t;
  const int nG = g.P - i0 < 256 ? g.P - i0 : 256;
  stage_sh_rows48<true>(g, i0, nG, s_rows);
  // the lane's own rows of xyz (plain), opacity (sigmoid), scaling (exp), rotation (normalize):
  // p / m / v loaded up front, in flight with the SH rows' staging loads
  const bool live = i < g.P;
  const size_t i3 = 3 * (size_t)(live ? i : 0), i4 = 4 * (size_t)(live ? i : 0), io = live ? i : 0;
  float px[3], mx[3], vx[3], ps[3], ms[3], vs[3], po, mo, vo;
  v4f pq, mq, vq;
  if (live) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      px[k] = __builtin_nontemporal_load(a.p[DT_XYZ] + i3 + k);
      mx[k] = __builtin_nontemporal_load(a.m[DT_XYZ] + i3 + k);
      vx[k] = __builtin_nontemporal_load(a.v[DT_XYZ] + i3 + k);
      ps[k] = __builtin_nontemporal_load(a.p[DT_SCALING] + i3 + k);
      ms[k] = __builtin_nontemporal_load(a.m[DT_SCALING] + i3 + k);
      vs[k] = __builtin_nontemporal_load(a.v[DT_SCALING] + i3 + k);
    }
    po = __builtin_nontemporal_load(a.p[DT_OPACITY] + io);
    mo = __builtin_nontemporal_load(a.m[DT_OPACITY] + io);
    vo = __builtin_nontemporal_load(a.v[DT_OPACITY] + io);
    pq = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(a.p[DT_ROT] + i4));
    mq = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(a.m[DT_ROT] + i4));
    vq = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(a.v[DT_ROT] + i4));
  }
  lds_barrier();
  if (live) {
    float row[KF];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const float4 r4 = lds_ld16(&s_rows[t * SH_STAGE_ROW + 4 * q]);
      row[4 * q] = r4.x, row[4 * q + 1] = r4.y, row[4 * q + 2] = r4.z, row[4 * q + 3] = r4.w;
    }
    RegSink gr;
    gr.dop = 0.0f;
    if (tiles[i] == 0) {  // invisible: every gradient is zero (the Adam step still runs on them)
#pragma unroll
      for (int k = 0; k < KF; k++) row[k] = 0.0f;
    } else {
      preprocess_bwd_visible<DEG, true>(i, g, c, clamped, gsum, row, true, gr);
#pragma unroll
      for (int k = K3; k < KF; k++) row[k] = 0.0f;  // coefficients past the active degree: zero gradient
    }
#pragma unroll
    for (int q = 0; q < Q; q++)
      *reinterpret_cast<float4*>(&s_rows[t * SH_STAGE_ROW + 4 * q]) =
          make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
    const float gq_in[4] = {gr.dr[0], gr.dr[1], gr.dr[2], gr.dr[3]}, q[4] = {pq.x, pq.y, pq.z, pq.w};
    float gq[4];
    normalize_adjoint(gq_in, q, gq);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      adam_update(px[k], gr.dmean[k], mx[k], vx[k], a.k, a.nss[DT_XYZ], a.bc2s[DT_XYZ], a.wd[DT_XYZ]);
      adam_update(ps[k], exp_adjoint(gr.ds[k], ps[k]), ms[k], vs[k], a.k, a.nss[DT_SCALING], a.bc2s[DT_SCALING],
                  a.wd[DT_SCALING]);
    }
    adam_update(po, sigmoid_adjoint(gr.dop, po), mo, vo, a.k, a.nss[DT_OPACITY], a.bc2s[DT_OPACITY],
                a.wd[DT_OPACITY]);
    float rq[4] = {pq.x, pq.y, pq.z, pq.w}, rm[4] = {mq.x, mq.y, mq.z, mq.w}, rv[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
    for (int k = 0; k < 4; k++)
      adam_update(rq[k], gq[k], rm[k], rv[k], a.k, a.nss[DT_ROT], a.bc2s[DT_ROT], a.wd[DT_ROT]);
    pq = (v4f){rq[0], rq[1], rq[2], rq[3]};
    mq = (v4f){rm[0], rm[1], rm[2], rm[3]};
    vq = (v4f){rv[0], rv[1], rv[2], rv[3]};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      __builtin_nontemporal_store(px[k], a.p[DT_XYZ] + i3 + k);
      __builtin_nontemporal_store(mx[k], a.m[DT_XYZ] + i3 + k);
      __builtin_nontemporal_store(vx[k], a.v[DT_XYZ] + i3 + k);
      __builtin_nontemporal_store(ps[k], a.p[DT_SCALING] + i3 + k);
      __builtin_nontemporal_store(ms[k], a.m[DT_SCALING] + i3 + k);
      __builtin_nontemporal_store(vs[k], a.v[DT_SCALING] + i3 + k);
    }
    __builtin_nontemporal_store(po, a.p[DT_OPACITY] + io);
    __builtin_nontemporal_store(mo, a.m[DT_OPACITY] + io);
    __builtin_nontemporal_store(vo, a.v[DT_OPACITY] + io);
    __builtin_nontemporal_store(pq, reinterpret_cast<v4f*>(a.p[DT_ROT] + i4));
    __builtin_nontemporal_store(mq, reinterpret_cast<v4f*>(a.m[DT_ROT] + i4));
    __builtin_nontemporal_store(vq, reinterpret_cast<v4f*>(a.v[DT_ROT] + i4));
    // train.py:115-116 in the same pass (k_densify_stats's arithmetic; skipped with the update)
    if (a.max_r) densify_stat_one(i, a.radii, a.grad2d, a.gstride, a.max_r, a.accum, a.denom);
  }
  lds_barrier();
  // features_dc / features_rest: the workgroup's contiguous blocks (16-B aligned: 256 rows of 12 /
  // 180 B), coalesced float4s, dL/dsh from the staged rows
  adam_sh_block<1, 3>(a, DT_FDC, i0, nG, t, s_rows);
  adam_sh_block<6, 45>(a, DT_FREST, i0, nG, t, s_rows);
}

void bwd_gaussians_adam(const GaussianArgs& g, const CameraArgs& c, const GeomPtrs& geo, const FusedAdamArgs& a,
                        hipStream_t st) {
  if (g.P <= 0) return;
  const dim3 grid((g.P + 255) / 256), block(256);
#define GS_PBWD_ADAM(D) \
  GS_LAUNCH("preprocess_bwd_adam", k_preprocess_bwd_adam<D>, grid, block, 0, st, g, c, geo.tiles, geo.clamped, geo.gsum, a)
  switch (g.D) {
    case 0: GS_PBWD_ADAM(0); break;
    case 1: GS_PBWD_ADAM(1); break;
    case 2: GS_PBWD_ADAM(2); break;
    default: GS_PBWD_ADAM(3); break;
  }
#undef GS_PBWD_ADAM
}

// ------------------------------------------------------------------------------------------
// Per-Gaussian backward of K views at once (view-parallel step, gs_backward_gaussians).
//
// A step that renders K views of one set of Gaussians into one gradient bucket would run the
// per-Gaussian backward K times, each reading the 192-B SH row and read-modify-writing the 236-B
// gradient row of every Gaussian (C3: ~0.7 GB per view, HBM-bound).  Here one lane per Gaussian
// reads its inputs once, walks the K views' record sums (36 B per view, summed by each view's
// k_sum_records) and cameras, forms every view's gradient with the single-view arithmetic, and
// writes (or adds once into) the bucket: the per-view outputs are combined in view order as
// `g = g0; g = g + g1; ...`, exactly the fp32 sums the sequential accumulate path produces.
// ------------------------------------------------------------------------------------------
// r = (first ? v : r + v): the bucket arithmetic of one view's write / `grad += g`
__device__ __forceinline__ void vput(float& r, float v, bool first) { r = first ? v : r + v; }

// The workgroup's 256 SH rows come in (and their gradient rows go out) as one
// contiguous block through LDS -- coalesced 16-B accesses -- instead of one lane-strided 192-B
// row per lane (every load instruction touching 64 cache lines).  The kernel runs at 2 waves per
// SIMD for its registers anyway, so the 53 KB of LDS per workgroup costs no occupancy.
constexpr int BG_ROW = 52;  // staged row stride (floats): 16-B aligned, conflict-free 16-B reads

template <int DEG>  // -1: colours precomputed (no SH gradient)
__global__ __launch_bounds__(256) void k_backward_gaussians(GaussianArgs g, FusedViews fv, GradOut out) {
  constexpr int D = DEG < 0 ? 0 : DEG;
  constexpr int KF = DEG < 0 ? 1 : 3 * (D + 1) * (D + 1);
  constexpr bool LDS = DEG >= 0 && KF % 4 == 0;
  __shared__ __attribute__((aligned(16))) float s_rows[LDS ? 256 * BG_ROW : 1];
  const int i0 = blockIdx.x * 256;
  const int i = i0 + (int)threadIdx.x;
  const bool live = i < g.P;
  const uint32_t acc = out.acc;
  const int rowf = 3 * g.M;
  // the SH row (its first 3K floats) and the accumulators; an output with its GS_ACC bit starts
  // from the caller's value and every view adds
  float row[KF], dsh[KF];
  const bool vec = DEG >= 0 && (KF & 3) == 0 && (rowf & 3) == 0 &&
                   ((((uintptr_t)g.shs) | ((uintptr_t)out.dsh)) & 15) == 0;
  // staged: whole rows of exactly 3K floats (the active degree is the stored one), 16-B aligned
  const bool stage = LDS && vec && rowf == KF && out.dsh;  // (uniform)
  const int nG = g.P - i0 < 256 ? g.P - i0 : 256;
  if (stage) {
    // all of the block's row loads in flight, then the LDS stores
    constexpr int PER = LDS ? KF / 4 : 1;  // float4 per row = per thread
    const float4* src4 = reinterpret_cast<const float4*>(g.shs + (size_t)i0 * KF);
    const int n4 = nG * PER;
    float4 v[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int f = (int)threadIdx.x + 256 * q;
      v[q] = f < n4 ? src4[f] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int f = (int)threadIdx.x + 256 * q;
      if (f < n4) {
        const int r = f / PER, c = f - r * PER;
        *reinterpret_cast<float4*>(&s_rows[r * BG_ROW + 4 * c]) = v[q];
      }
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const float4 t = lds_ld16(&s_rows[threadIdx.x * BG_ROW + 4 * q]);
      row[4 * q] = t.x, row[4 * q + 1] = t.y, row[4 * q + 2] = t.z, row[4 * q + 3] = t.w;
    }
  }
  if (live) {
    if (DEG >= 0 && !stage) {
      const float* src = g.shs + (size_t)i * rowf;
      if (vec) {
#pragma unroll
        for (int q = 0; q < KF / 4; q++) {
          const float4 v = reinterpret_cast<const float4*>(src)[q];
          row[4 * q] = v.x, row[4 * q + 1] = v.y, row[4 * q + 2] = v.z, row[4 * q + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < KF; k++) row[k] = src[k];
      }
    }
    const float px = g.means3D[3 * i], py = g.means3D[3 * i + 1], pz = g.means3D[3 * i + 2];
    float cov3[6];
    if (g.cov3D) {
#pragma unroll
      for (int k = 0; k < 6; k++) cov3[k] = g.cov3D[6 * i + k];
    } else {
      cov3d(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2], g.scale_modifier, g.rotations[4 * i],
            g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3], cov3);
    }
    const bool sr = !g.cov3D && out.dscale && out.drot;
    float a_col[3], a_op, a_mean[3], a_cov[6], a_s[3], a_r[4];
    bool f_col = !(acc & GS_ACC_COLORS), f_op = !(acc & GS_ACC_OPACITY), f_mean = !(acc & GS_ACC_MEANS3D),
         f_cov = !(acc & GS_ACC_COV3D), f_sh = !(acc & GS_ACC_SH), f_s = !(acc & GS_ACC_SCALES),
         f_r = !(acc & GS_ACC_ROTATIONS);
    if (out.dcolor && !f_col)
      for (int k = 0; k < 3; k++) a_col[k] = out.dcolor[3 * i + k];
    if (!f_op) a_op = out.dopacity[i];
    if (!f_mean)
      for (int k = 0; k < 3; k++) a_mean[k] = out.dmean3D[3 * i + k];
    if (out.dcov3D && !f_cov)
      for (int k = 0; k < 6; k++) a_cov[k] = out.dcov3D[6 * i + k];
    if (DEG >= 0 && !f_sh) {
      const float* d = out.dsh + (size_t)i * rowf;
#pragma unroll
      for (int k = 0; k < KF; k++) dsh[k] = d[k];
    }
    if (sr && !f_s)
      for (int k = 0; k < 3; k++) a_s[k] = out.dscale[3 * i + k];
    if (sr && !f_r)
      for (int k = 0; k < 4; k++) a_r[k] = out.drot[4 * i + k];

    // a view's per-Gaussian inputs (visibility, record sum, clamp bits) are loaded one view ahead:
    // the loop over the K views is not unrolled (K is a launch argument), so without it every view
    // waited out its loads at 2 waves per SIMD
    float an[GRAD_REC];
    uint32_t tn = fv.v[0].tiles[i];
    uint8_t cn = fv.v[0].clamped ? fv.v[0].clamped[i] : 0;
    {
      const float* rec = fv.v[0].gsum + (size_t)i * GRAD_REC;
#pragma unroll
      for (int k = 0; k < GRAD_REC; k++) an[k] = rec[k];
    }
    for (int v = 0; v < fv.K; v++) {
      const ViewGrad& w = fv.v[v];
      float dcol[3] = {0.f, 0.f, 0.f}, dop = 0.f, dmean[3] = {0.f, 0.f, 0.f}, dcv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      float ds[3] = {0.f, 0.f, 0.f}, dr[4] = {0.f, 0.f, 0.f, 0.f};
      float a[GRAD_REC];
#pragma unroll
      for (int k = 0; k < GRAD_REC; k++) a[k] = an[k];
      const bool vis = tn != 0;
      const uint8_t clamp_bits = cn;
      if (v + 1 < fv.K) {  // (uniform)
        const ViewGrad& wn = fv.v[v + 1];
        tn = wn.tiles[i];
        cn = wn.clamped ? wn.clamped[i] : 0;
        const float* rec = wn.gsum + (size_t)i * GRAD_REC;
#pragma unroll
        for (int k = 0; k < GRAD_REC; k++) an[k] = rec[k];
      }
      if (vis) {
        dcol[0] = a[0], dcol[1] = a[1], dcol[2] = a[2];
        dop = a[8];
        camera_grads(w.c, px, py, pz, cov3, a[5], a[6], a[7], a[3], a[4], dcv, dmean);
        if (DEG >= 0) {
          float shm[3];
          const float vx = px - w.c.campos[0], vy = py - w.c.campos[1], vz = pz - w.c.campos[2];
          sh_backward<D, true, true>(row, g.M, vx, vy, vz, clamp_bits, dcol, shm, dsh, f_sh);
          dmean[0] = dmean[0] + shm[0];
          dmean[1] = dmean[1] + shm[1];
          dmean[2] = dmean[2] + shm[2];
        }
        if (sr)
          cov3d_backward(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2], g.scale_modifier,
                         g.rotations[4 * i], g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3],
                         dcv, ds, dr);
      } else if (DEG >= 0) {
#pragma unroll
        for (int k = 0; k < KF; k++) vput(dsh[k], 0.0f, f_sh);
      }
      if (DEG >= 0) f_sh = false;
      for (int k = 0; k < 3; k++) vput(a_col[k], dcol[k], f_col);
      f_col = false;
      vput(a_op, dop, f_op);
      f_op = false;
      for (int k = 0; k < 3; k++) vput(a_mean[k], dmean[k], f_mean);
      f_mean = false;
      for (int k = 0; k < 6; k++) vput(a_cov[k], dcv[k], f_cov);
      f_cov = false;
      for (int k = 0; k < 3; k++) vput(a_s[k], ds[k], f_s);
      f_s = false;
      for (int k = 0; k < 4; k++) vput(a_r[k], dr[k], f_r);
      f_r = false;
    }
    if (out.dcolor)
      for (int k = 0; k < 3; k++) out.dcolor[3 * i + k] = a_col[k];
    out.dopacity[i] = a_op;
    for (int k = 0; k < 3; k++) out.dmean3D[3 * i + k] = a_mean[k];
    if (out.dcov3D)
      for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = a_cov[k];
    if (sr) {
      for (int k = 0; k < 3; k++) out.dscale[3 * i + k] = a_s[k];
      for (int k = 0; k < 4; k++) out.drot[4 * i + k] = a_r[k];
    }
    if (DEG >= 0 && out.dsh && !stage) {
      float* dst = out.dsh + (size_t)i * rowf;
      if (vec) {
#pragma unroll
        for (int q = 0; q < KF / 4; q++)
          reinterpret_cast<float4*>(dst)[q] = make_float4(dsh[4 * q], dsh[4 * q + 1], dsh[4 * q + 2], dsh[4 * q + 3]);
      } else {
#pragma unroll
        for (int k = 0; k < KF; k++) dst[k] = dsh[k];
      }
      if (!(acc & GS_ACC_SH))  // coefficients past (D + 1)^2: zero (accumulated: + 0)
        for (int k = KF; k < rowf; k++) dst[k] = 0.0f;
    }
  }
  if (stage) {
    // the gradient rows out the same way (rows of exactly 3K floats: nothing past (D + 1)^2)
    constexpr int PER = LDS ? KF / 4 : 1;
    lds_barrier();  // every lane has read its staged SH row
    if (live) {
#pragma unroll
      for (int q = 0; q < PER; q++)
        *reinterpret_cast<float4*>(&s_rows[threadIdx.x * BG_ROW + 4 * q]) =
            make_float4(dsh[4 * q], dsh[4 * q + 1], dsh[4 * q + 2], dsh[4 * q + 3]);
    }
    lds_barrier();
    float4* dst4 = reinterpret_cast<float4*>(out.dsh + (size_t)i0 * KF);
    const int n4 = nG * PER;
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int f = (int)threadIdx.x + 256 * q;
      if (f < n4) {
        const int r = f / PER, c = f - r * PER;
        dst4[f] = *reinterpret_cast<const float4*>(&s_rows[r * BG_ROW + 4 * c]);
      }
    }
  }
}

void bwd_gaussians(const GaussianArgs& g, const FusedViews& fv, const GradOut& out, hipStream_t st) {
  if (g.P <= 0 || fv.K <= 0) return;
  dim3 grid((g.P + 255) / 256), block(256);
  const bool sh = g.colors == nullptr && g.shs != nullptr && out.dsh != nullptr;
  if (!sh) {
    GS_LAUNCH("backward_gaussians", k_backward_gaussians<-1>, grid, block, 0, st, g, fv, out);
    return;
  }
  switch (g.D) {
    case 0: GS_LAUNCH("backward_gaussians", k_backward_gaussians<0>, grid, block, 0, st, g, fv, out); break;
    case 1: GS_LAUNCH("backward_gaussians", k_backward_gaussians<1>, grid, block, 0, st, g, fv, out); break;
    case 2: GS_LAUNCH("backward_gaussians", k_backward_gaussians<2>, grid, block, 0, st, g, fv, out); break;
    default: GS_LAUNCH("backward_gaussians", k_backward_gaussians<3>, grid, block, 0, st, g, fv, out); break;
  }
}

// dL/dmeans2D of one view straight from its record sums (the per-view output of the split
// backward; the per-Gaussian half runs later, over all of the step's views at once)
__global__ __launch_bounds__(256) void k_mean2d_grad(int P, const uint32_t* __restrict__ tiles,
                                                     const float* __restrict__ gsum, float* __restrict__ dmean2D,
                                                     uint32_t acc) {
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  if (i >= P) return;
  const bool vis = tiles[i] != 0;
  const float x = vis ? gsum[(size_t)i * GRAD_REC + 3] : 0.0f, y = vis ? gsum[(size_t)i * GRAD_REC + 4] : 0.0f;
  gput(dmean2D, 3 * i, x, acc, GS_ACC_MEANS2D);
  gput(dmean2D, 3 * i + 1, y, acc, GS_ACC_MEANS2D);
  gput(dmean2D, 3 * i + 2, 0.0f, acc, GS_ACC_MEANS2D);
}

void bwd_records(const GaussianArgs& g, const GeomPtrs& geo, const BinPtrs& bin, const ImgPtrs& img, float* gradrec,
                 uint32_t R, bool have_records, float* dmean2D, uint32_t acc, hipStream_t st) {
  if (g.P <= 0) return;
  if (have_records) launch_sum_records(g, geo, bin, img, gradrec, R, st);
  if (dmean2D)
    GS_LAUNCH("mean2d_grad", k_mean2d_grad, dim3((g.P + 255) / 256), dim3(256), 0, st, g.P, geo.tiles, geo.gsum,
              dmean2D, acc);
}

void bwd_preprocess(const GaussianArgs& g, const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin,
                    const ImgPtrs& img, float* gradrec, uint32_t R,
                    bool have_records, const GradOut& out, hipStream_t st) {
  if (g.P <= 0) return;
  if (have_records) launch_sum_records(g, geo, bin, img, gradrec, R, st);
  dim3 grid((g.P + 255) / 256), block(256);
  const bool sh = g.colors == nullptr && g.shs != nullptr && out.dsh != nullptr;
  if (!sh) {
    GS_LAUNCH("preprocess_bwd", k_preprocess_bwd_colors, grid, block, 0, st, g, c, geo.tiles, geo.clamped, geo.gsum,
              out);
    return;
  }
  if (sh_stage_ok(g) && (((uintptr_t)out.dsh) & 15) == 0 && !(out.acc & GS_ACC_SH)) {
    if (g.shs_rest)
      GS_LAUNCH("preprocess_bwd", k_preprocess_bwd_stage<true>, grid, block, 0, st, g, c, geo.tiles, geo.clamped,
                geo.gsum, out);
    else
      GS_LAUNCH("preprocess_bwd", k_preprocess_bwd_stage<false>, grid, block, 0, st, g, c, geo.tiles, geo.clamped,
                geo.gsum, out);
    return;
  }
  // split SH rows are otherwise read by the register variant only
  if (g.shs_rest) {
#define GS_PBWD_SPLIT(D)                                                                                        \
  GS_LAUNCH("preprocess_bwd", (k_preprocess_bwd_reg<D, true>), grid, block, 0, st, g, c, geo.tiles, geo.clamped, \
            geo.gsum, out)
    switch (g.D) {
      case 0: GS_PBWD_SPLIT(0); break;
      case 1: GS_PBWD_SPLIT(1); break;
      case 2: GS_PBWD_SPLIT(2); break;
      default: GS_PBWD_SPLIT(3); break;
    }
#undef GS_PBWD_SPLIT
    return;
  }
  switch (g.D) {
    case 0:
      GS_LAUNCH("preprocess_bwd", k_preprocess_bwd_reg<0>, grid, block, 0, st, g, c, geo.tiles, geo.clamped, geo.gsum, out);
      break;
    case 1:
      GS_LAUNCH("preprocess_bwd", k_preprocess_bwd_reg<1>, grid, block, 0, st, g, c, geo.tiles, geo.clamped, geo.gsum, out);
      break;
    case 2:
      GS_LAUNCH("preprocess_bwd", k_preprocess_bwd_reg<2>, grid, block, 0, st, g, c, geo.tiles, geo.clamped, geo.gsum, out);
      break;
    default:
      GS_LAUNCH("preprocess_bwd", k_preprocess_bwd_reg<3>, grid, block, 0, st, g, c, geo.tiles, geo.clamped, geo.gsum, out);
      break;
  }
}

}  // namespace gs
