// gs_internal.h -- host/device shared structures of the rasterizer: argument packs and the HBM
// layout of the three opaque state buffers that travel from forward to backward (the same role as
// upstream's geomBuffer / binningBuffer / imgBuffer).
//
// Layout (all arrays 256-B aligned, structure-of-arrays except the 48-B splat record):
//   geometry  (per Gaussian, P)      splat float4x3 | binrec float4x2 | tiles u32 |
//                                    clamped u8 | depth-sort keys/vals x2 u32 (keys_a: depth keys
//                                    written by preprocess) | offsets u32 |
//                                    scan partials | sort scratch | counters
//   binning   (per instance, I)      tile keys/vals x2 u32 | presort_gid u32 | sort scratch
//   image     (per pixel / tile)     ranges uint2 | final_T f32 | n_contrib u32 | tile_max u32 x4
//                                    (largest n_contrib of each 8x8 quadrant) | tile_order u32 |
//                                    tile_cut u32 | tile_done u64 + length buckets | bucket rank u32
//   gradient  (per instance, I)      9 f32 per (Gaussian, tile) instance (backward scratch)
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <cmath>

#include "../../include/gsrast.h"  // GS_ACC_* bits
#include "gs_common.h"
#include "gs_sortscan.h"

namespace gs {

// Numerics mode of the render loops (gs_set_exact_exp): true = deterministic exp2 (bit-exact with
// the CPU oracle), false = hardware v_exp_f32 (default).  Process-wide, read at launch time.
bool exact_exp();

// The renders look a sorted instance's Gaussian id up by its presort slot (presort_gid[slot]).
// (Carrying the ids through the tile sort as an aux stream instead, read by list position, cost
// +16 us over the two tile-sort scatters and saved 8 us in render_fwd at C3: not kept.)

constexpr int GRAD_REC = 9;    // dcolor(3), dmean2D(2), dconic(xx, xy, yy), dopacity

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Duplicate blocks: DUP_SLOTS consecutive instance slots per workgroup.  The owner table
// dup_first has P + 1 entries, so the load-balanced duplicate runs while I <= DUP_SLOTS * P
// (more than 2048 tiles per Gaussian on average falls back to the per-Gaussian kernel).
constexpr uint32_t DUP_SLOTS = 2048;
__host__ __device__ inline bool dup_balanced(uint32_t I, uint32_t P) {
  return (uint64_t)I <= (uint64_t)DUP_SLOTS * (uint64_t)P;
}

struct GaussianArgs {
  int P, D, M;
  const float* means3D;
  const float* shs;        // [P, M, 3] or null
  const float* colors;     // [P, 3] or null
  const float* opacities;  // [P]
  const float* scales;     // [P, 3] or null
  const float* rotations;  // [P, 4] or null
  const float* cov3D;      // [P, 6] or null
  float scale_modifier;
  // split SH rows (gs_forward_preprocess_split / gs_backward_accumulate_split): when set, `shs` is
  // features_dc [P, 1, 3] and this is features_rest [P, M - 1, 3] (GaussianModel's own tensors,
  // no concatenated copy); only the single-view preprocess and preprocess backward read it
  const float* shs_rest = nullptr;
  // first workgroup of a launch that covers only part of the rows (the forward preprocess launched
  // in row chunks behind row waits, gs_set_row_waits): workgroup blockIdx.x + blk0 owns rows
  // [256 (blockIdx.x + blk0), +256); 0 for every whole-grid launch
  int blk0 = 0;
};

// a 12-B row piece loaded with one global_load_dwordx3 (4-B alignment is enough)
struct __attribute__((aligned(4))) F3 {
  float a, b, c;
};

// Coalesced staging of a workgroup's 256 degree-3 SH rows (48 floats each) into LDS, row stride
// SH_STAGE_ROW floats (16-B aligned rows, conflict-free 16-B lane reads), for the preprocess
// backward (k_preprocess_bwd_stage): the block of rows is contiguous in HBM, so it is read with 16-B loads, every load in
// flight before the LDS stores -- instead of one lane-strided 192-B row per lane, each load
// instruction touching 64 cache lines.  SPLIT: features_dc's block (12 B per Gaussian, g.shs) and
// features_rest's (180 B, g.shs_rest) are each contiguous; their 16-B pieces straddle rows and are
// stored as dwords.  Needs 16-B aligned bases.  The caller puts a barrier after it.
// A 16-B LDS read kept whole (one ds_read_b128): the compiler otherwise shrinks a float4 LDS load
// to the elements it sees used and re-pairs the pieces as ds_read2_b32 / ds_read2_b64, which bank on
// (a/4) mod 32 per 32-lane half and turn a row stride that is conflict-free for 16-B reads (52
// floats here) into a 4-way conflict.
__device__ __forceinline__ float4 lds_ld16(const float* p) {
  typedef float v4f_t __attribute__((ext_vector_type(4)));
  v4f_t t = *reinterpret_cast<const v4f_t*>(p);
  asm volatile("" : "+v"(t));
  return make_float4(t.x, t.y, t.z, t.w);
}
constexpr int SH_STAGE_ROW = 52;
template <bool SPLIT>
__device__ __forceinline__ void stage_sh_rows48(const GaussianArgs& g, int i0, int nG, float* s_rows) {
  constexpr int KF = 48, Q = KF / 4;
  const int t = (int)threadIdx.x;
  if constexpr (SPLIT) {
    constexpr int RF = KF - 3, RQ = (256 * RF + 1023) / 1024;  // features_rest float4 per thread (12)
    const float* rest = g.shs_rest + (size_t)i0 * RF;
    const int nf = nG * RF, n4 = nf >> 2;
    float4 v[RQ];
#pragma unroll
    for (int q = 0; q < RQ; q++) {
      const int f = t + 256 * q;
      v[q] = f < n4 ? reinterpret_cast<const float4*>(rest)[f] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float* dc = g.shs + (size_t)i0 * 3;
    float4 d4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const int nd4 = (nG * 3) >> 2;
    if (t < nd4) d4 = reinterpret_cast<const float4*>(dc)[t];
#pragma unroll
    for (int q = 0; q < RQ; q++) {
      const int f = t + 256 * q;
      if (f < n4) {
        const float e4[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int e = 4 * f + j, r = e / RF;
          s_rows[r * SH_STAGE_ROW + 3 + (e - r * RF)] = e4[j];
        }
      }
    }
    if (t < nd4) {
      const float e4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int e = 4 * t + j, r = e / 3;
        s_rows[r * SH_STAGE_ROW + (e - 3 * r)] = e4[j];
      }
    }
    // tails of a partial last block (float counts that are not multiples of 4)
    if (t < nf - 4 * n4) {
      const int e = 4 * n4 + t, r = e / RF;
      s_rows[r * SH_STAGE_ROW + 3 + (e - r * RF)] = rest[e];
    }
    if (t < nG * 3 - 4 * nd4) {
      const int e = 4 * nd4 + t, r = e / 3;
      s_rows[r * SH_STAGE_ROW + (e - 3 * r)] = dc[e];
    }
  } else {
    const float4* src4 = reinterpret_cast<const float4*>(g.shs + (size_t)i0 * KF);
    const int n4 = nG * Q;
    float4 v[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int f = t + 256 * q;
      v[q] = f < n4 ? src4[f] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int f = t + 256 * q;
      if (f < n4) {
        const int r = f / Q;
        *reinterpret_cast<float4*>(&s_rows[r * SH_STAGE_ROW + 4 * (f - r * Q)]) = v[q];
      }
    }
  }
}
// launch condition of the staged kernels: degree 3, M == 16, 16-B aligned row bases
inline bool sh_stage_ok(const GaussianArgs& g) {
  return g.D == 3 && g.M == 16 && g.shs && !g.colors &&
         ((((uintptr_t)g.shs) | ((uintptr_t)g.shs_rest)) & 15) == 0;
}

struct CameraArgs {
  const float* view;    // 16, device
  const float* proj;    // 16, device
  const float* campos;  // 3, device
  const float* bg;      // 3, device
  float tanfovx, tanfovy, fx, fy;
  int W, H, gx, gy;
  int prefiltered;
};

constexpr int CNT_I = 1, CNT_ERR = 2, CNT_NREND = 4, CNT_V = 5, CNT_LB_TILE = 9;
// advanced by every forward's counter finalize: the look-back scans' epochs (k_scan_lb) differ
// between HIP-graph replays
constexpr int CNT_SEQ = 13;
// error flags in counters[CNT_ERR]: 1 prefiltered cull, 4 look-back timeout, 8 instance count overflow,
// 16 more instances than the binning buffer's capacity (gs_forward_bounded)
constexpr uint32_t ERR_PREFILTERED = 1u, ERR_LOOKBACK = 4u, ERR_INSTANCES = 8u, ERR_CAPACITY = 16u;
// flags under which the instance list is not valid: the binning kernels write placeholders that
// keep every later kernel in bounds, the renders composite nothing, the record sums are zero
constexpr uint32_t ERR_INVALID = ERR_LOOKBACK | ERR_CAPACITY;
// Largest instance count of one view: the sorts and scans index instances with 32-bit positions
// (a position plus one sort chunk must stay below 2^32).
constexpr long long GS_MAX_INSTANCES = (1ll << 31) - 1;

// A preprocess workgroup's totals: its instance count and its count of Gaussians with instances
// (bit 31: a Gaussian was culled although `prefiltered` is set), stored per workgroup (no atomics,
// no zeroing).  The first depth-sort histogram launch sums them in 64-bit (k_radix_hist<true>),
// writes the view's counters and copies them to the host's readback words.
struct WgTotals {
  uint32_t inst;  // tiles touched by the workgroup's Gaussians (<= 256 x tiles of the image)
  uint32_t vis;   // Gaussians with instances | ERR_PREFILTERED << 31
};
__device__ __forceinline__ void store_wg_totals(WgTotals* wg, uint32_t b, uint32_t nv, uint32_t tot,
                                                bool culled_prefiltered) {
  wg[b] = WgTotals{tot, nv | (culled_prefiltered ? 0x80000000u : 0u)};
}

struct GeomPtrs {
  float4* splat;  // 3 per Gaussian: (x, y, cxx, cxy) (cyy, opacity, r, g) (b, depth, cull_lim, -)
  float4* binrec;  // 2 per Gaussian: (x, y, cxx, cxy) (cyy, cull_lim, x0 | x1 << 16, y0 | y1 << 16) for binning
  uint32_t* tiles;
  uint8_t* clamped;
  uint32_t *keys_a, *vals_a, *keys_b, *vals_b;
  uint32_t* offsets;  // per depth rank
  uint32_t *rtiles_a, *rtiles_b;  // tile counts carried through the depth sort (aux stream)
  uint32_t* tiles_by_rank;        // = rtiles_a or rtiles_b after the depth sort
  uint32_t* dup_first;  // [P + 1] depth rank owning the first instance slot of each duplicate block
  float* gsum;  // [P][9] per-Gaussian sums of the backward records (k_sum_records -> k_preprocess_bwd)
  uint32_t* scan_partial;
  uint64_t* lb_status;  // look-back scan status words (lb_tiles(P))
  uint32_t* sort_scratch;
  // [1] instances I (offsets scan), [2] error flags (ERR_*), [4] / [5] num_rendered / V
  // (Gaussians with instances) from the preprocess workgroups' WgTotals (CounterFinalize, the first
  // depth-sort histogram launch), [9] look-back tile counter (offsets scan)
  uint32_t* counters;
  uint32_t* sorted_gid;  // = vals_a or vals_b after the depth sort
  WgTotals* wg_tot;      // per preprocess workgroup (ceil(P / 256))
};

inline size_t geom_layout(size_t P, GeomPtrs* out, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes);
    return o;
  };
  size_t Pn = P ? P : 1;
  size_t o_splat = take(Pn * 48);
  size_t o_bin = take(Pn * 32);
  size_t o_tiles = take(Pn * 4), o_cl = take(Pn);
  size_t o_ka = take(Pn * 4), o_va = take(Pn * 4), o_kb = take(Pn * 4), o_vb = take(Pn * 4);
  size_t o_offs = take(Pn * 4);
  size_t o_rta = take(Pn * 4), o_rtb = take(Pn * 4);
  size_t o_df = take((Pn + 1) * 4);
  size_t o_gs = take(Pn * 4 * GRAD_REC);
  size_t o_sp = take((size_t)scan_plan(Pn).nb * 4 + 64);
  size_t o_lb = take((size_t)lb_tiles(Pn) * 8);
  size_t o_ss = take(sort_scratch_words(Pn) * 4);
  size_t o_cnt = take(64);
  size_t o_wg = take(((Pn + 255) / 256) * sizeof(WgTotals));
  if (out && base) {
    out->splat = (float4*)(base + o_splat);
    out->binrec = (float4*)(base + o_bin);
    out->tiles = (uint32_t*)(base + o_tiles);
    out->clamped = (uint8_t*)(base + o_cl);
    out->keys_a = (uint32_t*)(base + o_ka);
    out->vals_a = (uint32_t*)(base + o_va);
    out->keys_b = (uint32_t*)(base + o_kb);
    out->vals_b = (uint32_t*)(base + o_vb);
    out->offsets = (uint32_t*)(base + o_offs);
    out->rtiles_a = (uint32_t*)(base + o_rta);
    out->rtiles_b = (uint32_t*)(base + o_rtb);
    out->tiles_by_rank = (radix_passes(32) % 2 == 0) ? out->rtiles_b : out->rtiles_a;
    out->dup_first = (uint32_t*)(base + o_df);
    out->gsum = (float*)(base + o_gs);
    out->scan_partial = (uint32_t*)(base + o_sp);
    out->lb_status = (uint64_t*)(base + o_lb);
    out->sort_scratch = (uint32_t*)(base + o_ss);
    out->counters = (uint32_t*)(base + o_cnt);
    out->wg_tot = (WgTotals*)(base + o_wg);
    out->sorted_gid = (radix_passes(32) % 2 == 0) ? out->vals_a : out->vals_b;
  }
  return off;
}

struct BinPtrs {
  uint32_t *keys_a, *vals_a, *keys_b, *vals_b;
  uint32_t* presort_gid;
  uint32_t* sort_scratch;
  uint32_t* point_list;  // sorted presort slots (= vals_a or vals_b after the tile sort)
  uint32_t* sorted_tile;
  uint32_t* slot_tile;   // tile of every instance slot (duplicate output, kept: the tile sort's
                         // first pass reads it and writes keys_b)
  uint32_t* count;       // [0]: the view's instance count bounded by the buffer's capacity (the duplicate
                         // writes it; the tile sort and k_ranges read it from this buffer)
};


// (Tried in round 2 and not kept: the forward's quadrant waves storing each staged entry's 48-B splat
// record at its list position for the backward to stream instead of gathering slot -> id -> splat.
// render_bwd PMC traffic 664 -> 324 MB but 401 -> 396 us only -- not fetch bound -- while the
// forward's redundant stores cost 175 -> 232 us.)

inline int tile_bits(int tiles) {
  int b = 1;
  while (b < 32 && ((uint64_t)1 << b) < (uint64_t)tiles) b++;
  return b;
}

inline size_t bin_layout(size_t I, int tiles, BinPtrs* out, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes);
    return o;
  };
  size_t In = I ? I : 1;
  size_t o_ka = take(In * 4), o_va = take(In * 4), o_kb = take(In * 4), o_vb = take(In * 4);
  size_t o_pg = take(In * 4), o_st = take(In * 4);
  size_t o_ss = take(sort_scratch_words(In) * 4);
  size_t o_cn = take(64);
  if (out && base) {
    out->count = (uint32_t*)(base + o_cn);
    out->keys_a = (uint32_t*)(base + o_ka);
    out->vals_a = (uint32_t*)(base + o_va);
    out->keys_b = (uint32_t*)(base + o_kb);
    out->vals_b = (uint32_t*)(base + o_vb);
    out->presort_gid = (uint32_t*)(base + o_pg);
    out->slot_tile = (uint32_t*)(base + o_st);
    out->sort_scratch = (uint32_t*)(base + o_ss);
    bool in_b = radix_passes(tile_bits(tiles)) % 2 == 1;
    out->point_list = in_b ? out->vals_b : out->vals_a;
    out->sorted_tile = in_b ? out->keys_b : out->keys_a;
  }
  return off;
}

struct ImgPtrs {
  uint2* ranges;
  float* final_T;
  uint32_t* n_contrib;
  uint32_t* tile_max;
  uint32_t* tile_order;  // backward launch order (k_tile_order)
  uint32_t* tile_cut;    // per tile: 1 + the slot of its last walked instance (0: none), k_tile_order
  uint64_t* tile_done;   // per tile: finished quadrant waves + their length bits (zeroed by k_ranges),
  uint32_t* len_hist;    //   then ORDER_GROUPS x ORDER_BUCKETS walk-length bucket counts
  uint32_t* tile_brank;  // bucket << 22 | rank within the bucket, per tile
  uint32_t* cut_max;     // the largest tile_cut (after len_hist; zeroed with it): no instance slot at
                         // or past it has a gradient record
};

// Backward launch order: tiles bucketed by walk length (largest n_contrib), longest first.
constexpr int ORDER_BUCKETS = 64;
// (The forward's completion counters -- 16 tiles' tile_done words per 128-B line, the 512 len_hist
// counts in 16 lines -- padded to one line each measured the same: render_fwd 171.5 / 171.9 us.)
// scheduling words zeroed per binning (k_ranges): tile_done, len_hist, cut_max
inline uint32_t sched_words(uint32_t tiles);

// The forward's quadrant waves are laid out in ORDER_GROUPS groups: group g = tile % 8 fills
// workgroups g, g + 8, g + 16, ..., which the dispatcher sends to one XCD (workgroup b runs on XCD
// b % 8), so the four quadrant waves of a tile share that XCD's L2 (XCD g owns every 8th tile
// column); the backward's units of group g are taken first by the waves running on XCD g.
// (Measured in round 2: each XCD rendering a vertical strip of the image instead, so that a splat's
// neighbouring tiles in both directions share one L2, made both renders slower: render_fwd 174 ->
// 184 us, render_bwd 404 -> 417 us.)
constexpr int ORDER_GROUPS = 8;
inline uint32_t sched_words(uint32_t tiles) { return 2u * tiles + ORDER_GROUPS * ORDER_BUCKETS + 1u; }
// tiles per group (the last groups may hold one fewer)
__host__ __device__ inline uint32_t xcd_span(uint32_t tiles) { return (tiles + ORDER_GROUPS - 1) / ORDER_GROUPS; }
// the k-th tile of group g (~0u past its end)
__host__ __device__ inline uint32_t xcd_tile(uint32_t g, uint32_t k, uint32_t gx, uint32_t gy) {
  const uint32_t t = ORDER_GROUPS * k + g;
  return t < gx * gy ? t : ~0u;
}

inline size_t img_layout(int W, int H, ImgPtrs* out, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes);
    return o;
  };
  size_t tiles = (size_t)((W + GS_TILE - 1) / GS_TILE) * ((H + GS_TILE - 1) / GS_TILE);
  size_t npix = (size_t)W * H;
  if (tiles == 0) tiles = 1;
  if (npix == 0) npix = 1;
  size_t o_r = take(tiles * 8), o_t = take(npix * 4), o_n = take(npix * 4), o_m = take(tiles * 16),
         o_o = take(tiles * 4), o_c = take(tiles * 4), o_d = take((size_t)sched_words((uint32_t)tiles) * 4),
         o_b = take(tiles * 4);
  if (out && base) {
    out->ranges = (uint2*)(base + o_r);
    out->final_T = (float*)(base + o_t);
    out->n_contrib = (uint32_t*)(base + o_n);
    out->tile_max = (uint32_t*)(base + o_m);
    out->tile_order = (uint32_t*)(base + o_o);
    out->tile_cut = (uint32_t*)(base + o_c);
    out->tile_done = (uint64_t*)(base + o_d);
    out->len_hist = (uint32_t*)(out->tile_done + tiles);
    out->cut_max = out->len_hist + ORDER_GROUPS * ORDER_BUCKETS;
    out->tile_brank = (uint32_t*)(base + o_b);
  }
  return off;
}

#ifdef GS_TIMING
// Diagnostic builds only (-DGS_TIMING; tools/bwd_timing.py, tools/fwd_timing.py): per-wave
// s_memrealtime stamps (100 MHz) of the render kernels, one buffer per kernel (per code object):
// [b][0] start, [1] end, [2] a << 32 | b, [3] xcc_id << 32 | hw_id, [4] c << 32 | d (the kernel's
// own counts).  Nothing in the kernels reads them.
constexpr int TIMING_MAX = 1 << 16;
#define GS_TIMING_BUFFER(buf, fn)                                                                   \
  __device__ unsigned long long buf[TIMING_MAX][5];                                                 \
  extern "C" int fn(unsigned long long* host_out, int n, int reset) {                               \
    if (n > TIMING_MAX) n = TIMING_MAX;                                                             \
    if (host_out && hipMemcpyFromSymbol(host_out, HIP_SYMBOL(buf), (size_t)n * 5 * 8) != hipSuccess) \
      return 1;                                                                                     \
    if (reset) {                                                                                    \
      void* p = nullptr;                                                                            \
      if (hipGetSymbolAddress(&p, HIP_SYMBOL(buf)) != hipSuccess) return 1;                          \
      if (hipMemset(p, 0, sizeof(buf)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1; \
    }                                                                                               \
    return 0;                                                                                       \
  }
__device__ __forceinline__ unsigned long long timing_stamp() {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ void timing_record(unsigned long long (*buf)[5], unsigned long long t0, uint32_t a,
                                              uint32_t b, uint32_t c, uint32_t d) {
  const unsigned long long t1 = timing_stamp();
  if (threadIdx.x == 0 && blockIdx.x < TIMING_MAX) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    unsigned long long* o = buf[blockIdx.x];
    o[0] = t0;
    o[1] = t1;
    o[2] = ((unsigned long long)a << 32) | b;
    o[3] = ((unsigned long long)xcc << 32) | hw;
    o[4] = ((unsigned long long)c << 32) | d;
  }
}
#endif

// ---- stages (gs_forward.hip / gs_backward.hip) ----
void fwd_preprocess(const GaussianArgs& g, const CameraArgs& c, int* radii, const GeomPtrs& geo, hipStream_t st);
void fwd_preprocess_grid(const GaussianArgs& g, const CameraArgs& c, int* radii, const GeomPtrs& geo, hipStream_t st,
                         dim3 grid);
// Row waits of this thread (gs_set_row_waits): chunk k covers the rows below `hi` not covered by an
// earlier chunk and must wait for `ev` (null: nothing to wait for).  take_row_waits() moves them out
// (the next forward preprocess consumes them); stream_wait() is hipStreamWaitEvent with the error
// captured (gs_last_error).
constexpr int GS_MAX_ROW_WAITS = 64;
struct RowWait {
  int hi;
  hipEvent_t ev;
};
int take_row_waits(RowWait* out, int max);
bool stream_wait(hipStream_t st, hipEvent_t ev);
// compaction, depth sort, instance offsets; the view's totals are finalised by the first histogram
// launch (written to host_counts when given: [I lo, I hi, V, err]), after which counts_ready is recorded.
// cap: the binning buffer's instance capacity (more instances: ERR_CAPACITY); sticky (pinned host
// words, or null): a view with error flags stores them into sticky[0] and its count into [1], [2].
// views > 1: the orderings of `views` views at once, view v's geometry buffer lying v * vstride
// bytes after geo's (slices of one allocation); cap[v] per view (null: unbounded), host_counts + 8 v
void fwd_order(int P, const GeomPtrs& geo, hipStream_t st, uint32_t* host_counts = nullptr,
               hipEvent_t counts_ready = nullptr, const uint32_t* cap = nullptr, uint32_t* sticky = nullptr,
               int views = 1, uint64_t vstride = 0);
// clear error flag bits in the geometry buffer's counters[CNT_ERR] (stream-ordered)
void fwd_clear_flags(const GeomPtrs& geo, uint32_t bits, hipStream_t st);
void fwd_bin(int P, uint32_t I, const CameraArgs& c, const int* radii, const GeomPtrs& geo, const BinPtrs& bin,
             const ImgPtrs& img, hipStream_t st);
// the binning of `views` views of one image size at once: view v's geometry / binning / image
// buffers lie v * {geo,bin,img}_stride bytes after geo's / bin's / img's (I: the largest capacity)
void fwd_bin_views(int views, int P, uint32_t I, const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin,
                   const ImgPtrs& img, uint64_t geo_stride, uint64_t bin_stride, uint64_t img_stride, hipStream_t st);
// err_host (device-visible pinned host word, or null): the ordering's error flags, stored by the render
// when nonzero (the host clears the word before it hands it out)
void fwd_render(const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin, const ImgPtrs& img, float* out_color,
                hipStream_t st, uint32_t* err_host = nullptr);
void mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present,
                  hipStream_t st);
void bwd_render(int P, const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin, const ImgPtrs& img,
                const float* dL_dpix, float* gradrec, hipStream_t st);
struct GradOut {
  float* dmean2D;   // [P, 3]
  float* dcolor;    // [P, 3] or null
  float* dopacity;  // [P]
  float* dmean3D;   // [P, 3]
  float* dcov3D;    // [P, 6] or null
  float* dsh;       // [P, M, 3] or null
  float* dscale;    // [P, 3] or null
  float* drot;      // [P, 4] or null
  // GS_ACC_* bits: the output is ADDED to what the buffer holds (multi-view gradient
  // accumulation into a caller-owned bucket, gsrast.h gs_backward_accumulate) instead of written
  uint32_t acc;
};
// multi-view per-Gaussian backward (gs_backward_gaussians): K views of one set of Gaussians
constexpr int FUSED_MAX_VIEWS = 8;
struct ViewGrad {
  CameraArgs c;
  const uint32_t* tiles;   // that view's geom buffer: tile counts (0 = invisible), SH clamp bits and
  const uint8_t* clamped;  //   per-Gaussian record sums (k_sum_records)
  const float* gsum;
};
struct FusedViews {
  int K;
  ViewGrad v[FUSED_MAX_VIEWS];
};
void bwd_gaussians(const GaussianArgs& g, const FusedViews& fv, const GradOut& out, hipStream_t st);
// preprocess of K views of one set of Gaussians in one launch (gs_forward_preprocess_views): each
// view's outputs exactly as fwd_preprocess writes them into that view's geometry buffer
struct PreViews {
  int K;
  CameraArgs c[FUSED_MAX_VIEWS];
  int* radii[FUSED_MAX_VIEWS];
  GeomPtrs geo[FUSED_MAX_VIEWS];
};
void fwd_preprocess_views(const GaussianArgs& g, const PreViews& pv, hipStream_t st);
// the per-tile half of a split backward: record sums into the geom buffer (+ dL/dmeans2D)
// R: the binning buffer's instance count / capacity (gradrec holds R records + the record-sum scratch)
void bwd_records(const GaussianArgs& g, const GeomPtrs& geo, const BinPtrs& bin, const ImgPtrs& img, float* gradrec,
                 uint32_t R, bool have_records, float* dmean2D, uint32_t acc, hipStream_t st);
void bwd_preprocess(const GaussianArgs& g, const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin,
                    const ImgPtrs& img, float* gradrec, uint32_t R,
                    bool have_records, const GradOut& out, hipStream_t st);
void knn_mean_dist2(int P, const float* pts, float* out, char* scratch, hipStream_t st);
void ssim_forward(int planes, int H, int W, const float* win11, const float* img1, const float* img2, float* dmaps,
                  float* partial, float* plane_sum, hipStream_t st);
void ssim_backward(int planes, int C, int H, int W, const float* win11, const float* img1, const float* img2,
                   const float* dmaps, const float* scale, float* dimg1, hipStream_t st);
size_t ssim_partial_count(int planes, int H, int W);
void photometric_forward(int planes, int H, int W, const float* win11, const float* img, const float* gt,
                         float lambda, float* dmaps, float* partial, float* out3, hipStream_t st);
void photometric_backward(int planes, int H, int W, const float* win11, const float* img, const float* gt,
                          const float* dmaps, float lambda, const float* grad, float* dimg, hipStream_t st);
constexpr int ADAM_MAX_TENSORS = 16;  // parameter tensors per Adam launch
// ---- Adam (torch.optim.Adam semantics), shared by k_adam and the fused per-Gaussian backward ----
struct AdamConsts {
  float w1, w2, b2, eps;  // 1 - b1, 1 - b2, b2, eps (rounded to float from the Python doubles)
  int maximize;
};
inline AdamConsts adam_consts(double beta1, double beta2, double eps, bool maximize) {
  return AdamConsts{(float)(1.0 - beta1), (float)(1.0 - beta2), (float)beta2, (float)eps, maximize ? 1 : 0};
}
// per tensor: -lr / (1 - b1^t) and sqrt(1 - b2^t), in double on the host as torch's Adam forms them
// from the Python step, then rounded to float
inline void adam_scalars(double lr, long long step, double beta1, double beta2, float* neg_step_size,
                         float* bc2_sqrt) {
  const double t = (double)step;
  const double bc1 = 1.0 - std::pow(beta1, t), bc2 = 1.0 - std::pow(beta2, t);
  *neg_step_size = (float)(-(lr / bc1));
  *bc2_sqrt = (float)std::sqrt(bc2);
}
// Operation order of torch's foreach Adam on the device (torch/optim/adam.py _multi_tensor_adam,
// ATen lerp / addcmul / addcdiv functors, compiled with FMA contraction): scalars rounded to float
// from the Python doubles, each tensor op rounded to float.
__device__ __forceinline__ void adam_update(float& p, float g, float& m, float& v, const AdamConsts& a, float nss,
                                            float bc2s, float wd) {
  if (a.maximize) g = -g;
  if (wd != 0.0f) g = __builtin_fmaf(wd, p, g);  // grad.add(param, alpha=weight_decay)
  m = __builtin_fmaf(a.w1, g - m, m);             // exp_avg.lerp_(grad, 1 - beta1), weight < 0.5 branch
  v = __builtin_fmaf(a.w2 * g, g, v * a.b2);      // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(v) / bc2s + a.eps;    // (sqrt(v) / sqrt(bc2)) + eps
  p = __builtin_fmaf(nss, m / denom, p);          // param.addcdiv_(m, denom, -lr / bc1)
}
// Adjoints of GaussianModel's activations (gaussian_model.py:95-115; k_activate_bwd's expressions,
// operation for operation), from the raw parameter values
__device__ __forceinline__ float sigmoid_adjoint(float g, float praw) {
  const float y = 1.0f / (1.0f + expf(-praw));
  return g * (1.0f - y) * y;
}
__device__ __forceinline__ float exp_adjoint(float g, float praw) { return g * expf(praw); }
// q / max(|q|, 1e-12) (F.normalize): the quaternion's adjoint
__device__ __forceinline__ void normalize_adjoint(const float* gq, const float* q, float* out) {
  const float len = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const float n = fmaxf(len, 1e-12f);
  const float dot = gq[0] * q[0] + gq[1] * q[1] + gq[2] * q[2] + gq[3] * q[3];
  const float c = len > 1e-12f ? dot / (n * n) / len : 0.0f;
#pragma unroll
  for (int j = 0; j < 4; j++) out[j] = gq[j] / n - c * q[j];
}
// train.py:115-116 (gaussian_model.py:405-407) for Gaussian i: k_densify_stats's body, shared with
// the fused backward + Adam step so both write the same floats
__device__ __forceinline__ void densify_stat_one(int i, const int* __restrict__ radii, const float* __restrict__ grad2d,
                                                 int gstride, float* __restrict__ max_r, float* __restrict__ accum,
                                                 float* __restrict__ denom) {
  const int r = radii[i];
  if (r <= 0) return;
  max_r[i] = fmaxf(max_r[i], (float)r);
  const float gx = grad2d[(size_t)gstride * i], gy = grad2d[(size_t)gstride * i + 1];
  accum[i] += sqrtf(gx * gx + gy * gy);
  denom[i] += 1.0f;
}
// the six parameter groups of GaussianModel (xyz, f_dc, f_rest, opacity, scaling, rotation) for the
// fused per-Gaussian backward + Adam step (gs_backward_gaussians_adam)
struct FusedAdamArgs {
  float* p[6];
  float* m[6];
  float* v[6];
  float nss[6], bc2s[6], wd[6];
  AdamConsts k;
  // the view's forward error flags (counters[CNT_ERR]): non-zero -> the update is skipped, so a
  // step launched before the host has read them leaves an invalid view's parameters untouched
  const uint32_t* err;
  // optional densification statistics of the view (max_r == nullptr: none), densify_stat_one
  const int* radii;
  const float* grad2d;
  int gstride;
  float *max_r, *accum, *denom;
};
// one view's per-Gaussian half fused with the Adam step (g: M == 16 split SH rows, 16-B aligned)
void bwd_gaussians_adam(const GaussianArgs& g, const CameraArgs& c, const GeomPtrs& geo, const FusedAdamArgs& a,
                        hipStream_t st);
// how k_adam forms a tensor's gradient from its source g (gs_adam_step_activated)
enum AdamGrad { AG_PLAIN = 0, AG_SH_DC = 1, AG_SH_REST = 2, AG_SIGMOID = 3, AG_EXP = 4, AG_NORMALIZE = 5 };
void adam_step(int count, float* const* params, const float* const* grads, float* const* exp_avg,
               float* const* exp_avg_sq, const long long* numel, const double* lr, const long long* step,
               const double* weight_decay, double beta1, double beta2, double eps, bool maximize, hipStream_t st,
               const int* modes = nullptr, int sh_coeffs = 1);
void activate_forward(int P, int rest_w, const float* f_dc, const float* f_rest, const float* o_raw,
                      const float* s_raw, const float* q_raw, float* shs, float* opac, float* scales, float* rots,
                      hipStream_t st);
void activate_backward(int P, int rest_w, const float* dshs, const float* dopac, const float* dscales,
                       const float* drots, const float* opac, const float* scales, const float* q_raw, float* d_dc,
                       float* d_rest, float* d_o, float* d_s, float* d_q, hipStream_t st);
// densify_and_prune (csrc/gs_densify.hip)
struct DensifyParams {
  // scalars rounded to float as torch compares them; a tensor divided by a Python scalar is
  // multiplied by the float reciprocal on the device (ATen div_true with a CPU scalar), hence inv_split
  float thr, pd_ext, min_op, big_ext, max_screen, inv_split;
  int screen;                                                  // `if max_screen_size:`
};
struct DensCounts {
  uint32_t keep_a, keep_b, split, keep_c;
};
constexpr int DENS_TENSORS = 6;
enum { DT_XYZ = 0, DT_FDC = 1, DT_FREST = 2, DT_OPACITY = 3, DT_SCALING = 4, DT_ROT = 5 };
struct DensTensors {
  const float* src[DENS_TENSORS];
  const float* m_src[DENS_TENSORS];  // Adam exp_avg (NULL: the group has no state yet)
  const float* v_src[DENS_TENSORS];
  float* dst[DENS_TENSORS];
  float* m_dst[DENS_TENSORS];
  float* v_dst[DENS_TENSORS];
  int width[DENS_TENSORS];
};
void densify_classify(int P, const DensifyParams& dp, const float* accum, const float* denom, const float* opacity,
                      const float* scaling, uint8_t* flags, uint32_t* counts, uint32_t* totals, hipStream_t st);
void densify_stds(int P, int N, uint32_t n_split, const uint8_t* flags, const uint32_t* bases, const float* scaling,
                  float* stds, hipStream_t st);
void densify_emit(int P, int N, const DensifyParams& dp, const DensCounts& n, const uint8_t* flags,
                  const uint32_t* bases, const float* samples, const DensTensors& t, hipStream_t st);
void densify_stats(int P, const int* radii, const float* grad2d, int grad_stride, float* max_radii2D,
                   float* grad_accum, float* denom, hipStream_t st);
size_t knn_scratch_bytes(int P);

}  // namespace gs
