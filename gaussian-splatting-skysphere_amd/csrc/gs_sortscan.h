// gs_sortscan.h -- hand-written device-wide exclusive scan and stable LSD radix sort (u32 keys,
// u32 values) for gfx950.  Used for: visibility compaction, per-Gaussian instance offsets, the
// depth sort of visible Gaussians and the stable tile sort of (tile, presort-slot) instances.
//
// Scan: reduce -> single-workgroup partial scan -> down-sweep (3 launches).  Workgroup count is
// capped at 1024 so the partial scan is one 1024-lane workgroup.
// Radix sort: per pass (8-bit digit) upsweep histogram [digit][block] -> per-digit row scan ->
// stable scatter (3 launches per pass; the scatter adds the digit bases itself).
// The scatter ranks keys inside a 256-key tile with wave64 ballots (per-bit peer masks, the
// CDNA analogue of match_any), combines the 4 waves through LDS and keeps a running per-digit
// base per workgroup, so equal digits keep input order (LSD stability).
//
// Element counts may live on the device (`n_dev`, e.g. the number of visible Gaussians) with a
// host-side upper bound `n_max` that sizes the grids; surplus workgroups see an empty range.
#pragma once
#include "gs_common.h"

namespace gs {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 4;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;  // 1024 elements per tile
constexpr int SCAN_MAX_BLOCKS = 1024;

struct ScanPlan {
  uint32_t nb;     // workgroups
  uint32_t chunk;  // elements per workgroup (multiple of SCAN_TILE)
};

inline ScanPlan scan_plan(uint64_t n_max) {
  uint64_t tiles = (n_max + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles == 0) tiles = 1;
  uint64_t per = (tiles + SCAN_MAX_BLOCKS - 1) / SCAN_MAX_BLOCKS;
  ScanPlan p;
  p.nb = (uint32_t)((tiles + per - 1) / per);
  p.chunk = (uint32_t)(per * SCAN_TILE);
  return p;
}

__device__ __forceinline__ uint32_t resolve_n(const uint32_t* n_dev, uint32_t n_max) {
  if (n_dev == nullptr) return n_max;
  uint32_t n = *n_dev;
  return n < n_max ? n : n_max;
}

// inclusive wave64 scan (u32)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

// exclusive scan of one value per thread over a 256-thread workgroup; returns the exclusive
// prefix and writes the workgroup total to *total.  `sh` needs 4 u32 of LDS.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) sh[wid] = inc;
  lds_barrier();
  uint32_t w0 = sh[0], w1 = sh[1], w2 = sh[2], w3 = sh[3];
  uint32_t before = (wid > 0 ? w0 : 0) + (wid > 1 ? w1 : 0) + (wid > 2 ? w2 : 0);
  *total = w0 + w1 + w2 + w3;
  lds_barrier();
  return before + inc - v;
}

template <class Src>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_reduce(Src src, const uint32_t* n_dev, uint32_t n_max,
                                                              uint32_t chunk, uint32_t* partial) {
  __shared__ uint32_t sh[4];
  const uint32_t n = resolve_n(n_dev, n_max);
  const uint64_t start = (uint64_t)blockIdx.x * chunk;
  const uint64_t end = start + chunk < n ? start + chunk : n;
  uint32_t s = 0;
  for (uint64_t i = start + threadIdx.x; i < end; i += SCAN_THREADS) s += src((uint32_t)i);
  uint32_t tot;
  block_excl_scan(s, sh, &tot);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

// single workgroup (1024 lanes): exclusive scan of partial[0..nb) in place; total -> *total_out
// (a template, like every kernel of this header: vague linkage, so the TUs that include it share one
// exported kernel handle -- the launch log resolves it by name)
template <int = 0>
__global__ __launch_bounds__(1024) void k_scan_partials(uint32_t* partial, uint32_t nb, uint32_t* total_out) {
  __shared__ uint32_t sh[16];
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nb; base += 1024) {
    uint32_t i = base + threadIdx.x;
    uint32_t v = i < nb ? partial[i] : 0u;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) sh[wid] = inc;
    lds_barrier();
    uint32_t before = 0, tot = 0;
    for (uint32_t w = 0; w < 16; w++) {
      uint32_t x = sh[w];
      if (w < wid) before += x;
      tot += x;
    }
    if (i < nb) partial[i] = carry + before + inc - v;
    carry += tot;
    lds_barrier();
  }
  if (threadIdx.x == 0 && total_out) *total_out = carry;
}

template <class Src, class Dst>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_down(Src src, Dst dst, const uint32_t* n_dev,
                                                            uint32_t n_max, uint32_t chunk,
                                                            const uint32_t* partial) {
  __shared__ uint32_t sh[4];
  const uint32_t n = resolve_n(n_dev, n_max);
  const uint64_t start = (uint64_t)blockIdx.x * chunk;
  const uint64_t end = start + chunk < n ? start + chunk : n;
  uint32_t carry = partial[blockIdx.x];
  for (uint64_t base = start; base < end; base += SCAN_TILE) {
    uint64_t i0 = base + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS], loc = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
      v[k] = (i0 + k < end) ? src((uint32_t)(i0 + k)) : 0u;
      loc += v[k];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan(loc, sh, &tot) + carry;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
      if (i0 + k < end) dst((uint32_t)(i0 + k), ex, v[k]);
      ex += v[k];
    }
    carry += tot;
  }
}

// host: run the 3-launch scan.  partial must hold >= plan.nb u32.
template <class Src, class Dst>
inline void scan_exclusive(Src src, Dst dst, const uint32_t* n_dev, uint32_t n_max, uint32_t* partial,
                           uint32_t* total_out, hipStream_t st) {
  ScanPlan p = scan_plan(n_max);
  GS_LAUNCH("scan_reduce", (k_scan_reduce<Src>), dim3(p.nb), dim3(SCAN_THREADS), 0, st, src, n_dev, n_max,
            p.chunk, partial);
  GS_LAUNCH("scan_partials", k_scan_partials<>, dim3(1), dim3(1024), 0, st, partial, p.nb, total_out);
  GS_LAUNCH("scan_down", (k_scan_down<Src, Dst>), dim3(p.nb), dim3(SCAN_THREADS), 0, st, src, dst, n_dev, n_max,
            p.chunk, partial);
}

// ------------------------------------------------------------------------------------------
// Single-pass exclusive scan with decoupled look-back (1 launch instead of reduce / partials /
// down-sweep).  Each workgroup takes the next tile id from a counter (ids follow start order, so
// a workgroup only ever waits for workgroups that are already running), scans its 2048-element
// tile, publishes its aggregate, then one wave looks back 64 predecessors at a time until it
// finds an inclusive prefix, and publishes its own.  A status word is one 64-bit atomic:
// [63:34] epoch (per call, so stale words from earlier calls never match), [33:32] state
// (1 aggregate, 2 inclusive prefix), [31:0] value.  The counter must be 0 at launch (the forward
// zeroes its counters before preprocessing).  Waits are bounded: a word that never arrives sets
// err_flag bit 2 and the scan finishes (with a wrong result) instead of hanging the device.
// ------------------------------------------------------------------------------------------
constexpr int LB_THREADS = 256;
constexpr int LB_ITEMS = 8;
constexpr int LB_TILE = LB_THREADS * LB_ITEMS;  // 2048 elements
constexpr uint64_t LB_AGG = 1, LB_PREFIX = 2;
constexpr uint32_t LB_SPIN_LIMIT = 1u << 22;
constexpr uint32_t LB_STATIC_MAX = 512;

inline uint32_t lb_tiles(uint64_t n_max) { return (uint32_t)((n_max + LB_TILE - 1) / LB_TILE) + (n_max == 0); }

__device__ __forceinline__ uint64_t lb_word(uint32_t epoch, uint64_t state, uint32_t v) {
  return ((uint64_t)epoch << 34) | (state << 32) | v;
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t w) {
  __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class Src, class Dst>
__global__ __launch_bounds__(LB_THREADS) void k_scan_lb(Src src, Dst dst, const uint32_t* n_dev, uint32_t n_max,
                                                        uint64_t* __restrict__ status, uint32_t* tile_counter,
                                                        uint32_t epoch, const uint32_t* epoch_seq,
                                                        uint32_t* total_out, uint32_t* err_flag,
                                                        uint32_t spin_limit) {
  // epoch_seq: a device word advanced once per forward before this launch -- a HIP graph replays
  // the host epoch unchanged, and the previous replay's status words must not match this one's
  if (epoch_seq) epoch = ((epoch + *epoch_seq) % ((1u << 30) - 1u)) + 1u;
  __shared__ uint32_t sh[4];
  __shared__ uint32_t s_tile, s_excl;
  // Tile ids: with a grid every CU can hold at once (LB_STATIC_MAX workgroups, a quarter of the
  // residency of this small kernel) all workgroups run concurrently and blockIdx is safe;
  // larger grids take ids in start order from the counter (one same-address atomic per workgroup).
  uint32_t tile = blockIdx.x;
  if (gridDim.x > LB_STATIC_MAX) {
    if (threadIdx.x == 0) s_tile = atomicAdd(tile_counter, 1u);
    lds_barrier();
    tile = s_tile;
  }
  const uint32_t n = resolve_n(n_dev, n_max);
  const uint64_t i0 = (uint64_t)tile * LB_TILE + (uint64_t)threadIdx.x * LB_ITEMS;
  uint32_t v[LB_ITEMS], loc = 0;
#pragma unroll
  for (int k = 0; k < LB_ITEMS; k++) {
    v[k] = (i0 + k < n) ? src((uint32_t)(i0 + k)) : 0u;
    loc += v[k];
  }
  uint32_t agg;
  uint32_t ex = block_excl_scan(loc, sh, &agg);
  if (threadIdx.x < 64) {
    const uint32_t lane = threadIdx.x;
    if (lane == 0) lb_store(&status[tile], lb_word(epoch, tile == 0 ? LB_PREFIX : LB_AGG, agg));
    // look back LB_WIN predecessors per round: lane l holds tiles t - 4l .. t - 4l - 3
    uint32_t excl = 0;
    int64_t t = (int64_t)tile - 1;
    while (t >= 0) {
      uint64_t w[4];
      bool ready = true;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int64_t idx = t - 4 * (int64_t)lane - k;
        w[k] = idx >= 0 ? lb_load(&status[idx]) : lb_word(epoch, LB_PREFIX, 0);
        ready = ready && (uint32_t)(w[k] >> 34) == epoch;
      }
      uint32_t spins = 0;
      bool forced = spin_limit == 0;  // test hook (gs_debug_set_scan_spin_limit(0)): time out at once
      while (forced || __ballot(!ready) != 0) {  // wait until every word of the window has been published
        __builtin_amdgcn_s_sleep(1);
        ready = true;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int64_t idx = t - 4 * (int64_t)lane - k;
          if ((uint32_t)(w[k] >> 34) != epoch) w[k] = lb_load(&status[idx]);
          ready = ready && (uint32_t)(w[k] >> 34) == epoch;
        }
        if (forced || ++spins > spin_limit) {
          if (lane == 0) atomicOr(err_flag, 4u);
#pragma unroll
          for (int k = 0; k < 4; k++) w[k] = lb_word(epoch, LB_PREFIX, 0);
          ready = true;
          forced = false;
        }
      }
      // nearest inclusive prefix: first (lane, k) in window order
      int kf = 4;
#pragma unroll
      for (int k = 3; k >= 0; k--)
        if (((w[k] >> 32) & 3u) == LB_PREFIX) kf = k;
      const uint64_t pm = __ballot(kf < 4);
      const uint32_t stop = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (lane < stop || (lane == stop && k <= kf)) c += (uint32_t)w[k];
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) c += (uint32_t)__shfl_xor((int)c, d, 64);
      excl += c;
      if (pm) break;
      t -= 256;
    }
    if (lane == 0) {
      if (tile > 0) lb_store(&status[tile], lb_word(epoch, LB_PREFIX, excl + agg));
      s_excl = excl;
      if (tile == gridDim.x - 1 && total_out) *total_out = excl + agg;
    }
  }
  lds_barrier();
  ex += s_excl;
#pragma unroll
  for (int k = 0; k < LB_ITEMS; k++) {
    if (i0 + k < n) dst((uint32_t)(i0 + k), ex, v[k]);
    ex += v[k];
  }
}

uint32_t next_scan_epoch();  // host: a fresh non-zero epoch per call (gs_api.hip)
uint32_t scan_spin_limit();  // host: LB_SPIN_LIMIT unless a test lowered it (gs_api.hip)

// host: one-launch scan.  status needs lb_tiles(n_max) u64; *tile_counter must be 0; epoch_seq (or
// null) is a device word that changes between calls a HIP graph may replay.
template <class Src, class Dst>
inline void scan_exclusive_lb(Src src, Dst dst, const uint32_t* n_dev, uint32_t n_max, uint64_t* status,
                              uint32_t* tile_counter, uint32_t* total_out, uint32_t* err_flag, hipStream_t st,
                              const uint32_t* epoch_seq, const char* name = "scan_lb") {
  const uint32_t tiles = lb_tiles(n_max);
  GS_LAUNCH(name, (k_scan_lb<Src, Dst>), dim3(tiles), dim3(LB_THREADS), 0, st, src, dst, n_dev, n_max, status,
            tile_counter, next_scan_epoch(), epoch_seq, total_out, err_flag, scan_spin_limit());
}

// simple functors
struct SrcArray {
  const uint32_t* a;
  __device__ uint32_t operator()(uint32_t i) const { return a[i]; }
};
struct DstArray {
  uint32_t* a;
  __device__ void operator()(uint32_t i, uint32_t ex, uint32_t) const { a[i] = ex; }
};

// ------------------------------------------------------------------------------------------
// radix sort
//
// Stable LSD radix sort, 8-bit digits.  Per pass: k_radix_hist (per-block digit counts) ->
// k_radix_rowscan (exclusive scan of each digit's row of the [digit][block] matrix + row totals)
// -> k_radix_scatter (digit base = exclusive scan of the row totals, done per workgroup).  A block walks its chunk in
// tiles of 2048 keys (8 per lane): each wave ranks its 512 consecutive keys round by round with
// ballot peer masks (stable), the 4 waves are combined per digit in LDS, the tile is reordered by
// digit in LDS, and runs of equal digits are written out contiguously (coalesced stores).
// ------------------------------------------------------------------------------------------
constexpr uint32_t DEPTH_DROP = 0xFFFFFFFFu;  // key of a Gaussian without instances (dropped)
constexpr int RADIX_BITS = 8;
constexpr int RADIX = 1 << RADIX_BITS;
constexpr int SORT_THREADS = 256;
constexpr int SORT_ITEMS = 8;
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;  // 2048 keys
constexpr int SORT_MAX_BLOCKS = 4096;  // one 2048-key tile per workgroup up to 8M keys

struct SortPlan {
  uint32_t nb, chunk;
};

inline int radix_passes(int end_bit) { return (end_bit + RADIX_BITS - 1) / RADIX_BITS; }
// digit width of every pass (the last may be narrower): equal widths, 13 bits -> 7 + 6
inline int radix_width(int end_bit) {
  const int np = radix_passes(end_bit);
  return (end_bit + np - 1) / np;
}
// width of the first pass: the remainder (13 -> 6 + 7; the narrower digit first saved 3.6 us over
// the C3 tile sort's six scatters)
inline int radix_first_bits(int end_bit) {
  const int w = radix_width(end_bit);
  if (end_bit <= w) return end_bit;
  return end_bit - (radix_passes(end_bit) - 1) * w;
}

// max_blocks: workgroups per pass (each takes whole 2048-key tiles); fewer, longer workgroups
// make the [digit][block] histogram and its row scan smaller
inline SortPlan sort_plan(uint64_t n_max, uint32_t max_blocks = SORT_MAX_BLOCKS) {
  uint64_t tiles = (n_max + SORT_TILE - 1) / SORT_TILE;
  if (tiles == 0) tiles = 1;
  if (max_blocks == 0 || max_blocks > SORT_MAX_BLOCKS) max_blocks = SORT_MAX_BLOCKS;
  uint64_t per = (tiles + max_blocks - 1) / max_blocks;
  SortPlan p;
  p.nb = (uint32_t)((tiles + per - 1) / per);
  p.chunk = (uint32_t)(per * SORT_TILE);
  return p;
}

// scratch words needed by radix_sort_pairs: [digit][block] histogram + per-digit row totals.  Sized
// for min(tiles, SORT_MAX_BLOCKS) blocks, an upper bound of sort_plan's nb (which drops when n passes
// a multiple of SORT_MAX_BLOCKS tiles) that never decreases with n: every buffer size built from it
// grows monotonically with its count, which gs_binning_layout_count's search relies on.
inline size_t sort_scratch_words(uint64_t n_max) {
  uint64_t tiles = (n_max + SORT_TILE - 1) / SORT_TILE;
  if (tiles == 0) tiles = 1;
  const size_t nb = (size_t)(tiles < SORT_MAX_BLOCKS ? tiles : SORT_MAX_BLOCKS);
  return (size_t)RADIX * nb + RADIX + 16;
}

// View batching: one launch sorts the same-shaped arrays of several views (blockIdx.y = view) whose
// buffers lie `vstride` bytes apart (the views' geometry buffers are slices of one allocation).
// vptr(p): this workgroup's view's copy of p (null stays null).
template <class T>
__device__ __forceinline__ T* vptr(T* p, uint64_t vstride) {
  return p ? (T*)((char*)p + (uint64_t)blockIdx.y * vstride) : p;
}
template <class T>
__device__ __forceinline__ const T* vptr(const T* p, uint64_t vstride) {
  return p ? (const T*)((const char*)p + (uint64_t)blockIdx.y * vstride) : p;
}

// lanes of this wave whose `bits`-bit digit equals mine (valid lanes only)
__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid, int bits) {
  uint64_t peers = __ballot(valid);
#pragma unroll
  for (int b = 0; b < bits; b++) {
    const uint64_t bb = __ballot((d >> b) & 1);
    peers &= ((d >> b) & 1) ? bb : ~bb;
  }
  return peers;
}

// Fin: work of one extra workgroup (blockIdx nb, all 256 threads; the launch then has nb + 1
// workgroups) beside the counting ones, e.g. the forward's counter finalisation in the first
// depth-sort pass (gs_forward.hip CounterFinalize); NoFin: none.
// Fin::operator()(view) runs for each view of a batched launch (blockIdx.y).
struct NoFin {
  static constexpr bool active = false;
  __device__ void operator()(uint32_t) const {}
};
// Row scan of one digit's row of the [digit][block] histogram in place (exclusive per-block
// offsets within the digit) and its total; every thread of the workgroup calls it.
__device__ __forceinline__ void radix_row_scan(uint32_t* row, uint32_t nb, uint32_t* row_total, uint32_t* sh) {
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nb; base += SORT_THREADS * 4) {
    const uint32_t i0 = base + threadIdx.x * 4;
    uint32_t v[4], loc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      v[k] = i0 + k < nb ? row[i0 + k] : 0u;
      loc += v[k];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan(loc, sh, &tot) + carry;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (i0 + k < nb) row[i0 + k] = ex;
      ex += v[k];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) *row_total = carry;
}

template <class Fin = NoFin>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_hist(const uint32_t* __restrict__ keys, const uint32_t* n_dev,
                                                             uint32_t n_max, int shift, int bits, uint32_t chunk,
                                                             uint32_t nb, uint32_t* __restrict__ hist, bool drop,
                                                             uint64_t vstride, Fin fin = Fin()) {
  __shared__ uint32_t h[RADIX];
  if constexpr (Fin::active) {
    if (blockIdx.x == nb) {  // (uniform) the extra workgroup runs beside the counting ones
      fin(blockIdx.y);
      return;
    }
  }
  keys = vptr(keys, vstride), n_dev = vptr(n_dev, vstride), hist = vptr(hist, vstride);
  const uint32_t n = resolve_n(n_dev, n_max);
  h[threadIdx.x] = 0;
  lds_barrier();
  const uint64_t start = (uint64_t)blockIdx.x * chunk;
  const uint64_t end = start + chunk < n ? start + chunk : n;
  const uint32_t mask = (1u << bits) - 1u;
  for (uint64_t t0 = start; t0 < end; t0 += SORT_TILE) {
    uint32_t d[SORT_ITEMS];
    bool v[SORT_ITEMS];
#pragma unroll
    for (int k = 0; k < SORT_ITEMS; k++) {
      const uint64_t i = t0 + (uint64_t)k * SORT_THREADS + threadIdx.x;
      const uint32_t key = i < end ? keys[i] : DEPTH_DROP;
      v[k] = i < end && !(drop && key == DEPTH_DROP);
      d[k] = (key >> shift) & mask;
    }
#pragma unroll
    for (int k = 0; k < SORT_ITEMS; k++)
      if (v[k]) atomicAdd(&h[d[k]], 1u);  // counts only: order-free, deterministic
  }
  lds_barrier();
  hist[(size_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// Row scan of the [digit][block] histogram: workgroup d turns row d into exclusive per-block
// offsets (within digit d) and writes the row total; the scatter adds the digit base itself.
template <int = 0>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_rowscan(uint32_t* __restrict__ hist, uint32_t nb,
                                                                        uint32_t* __restrict__ row_total,
                                                                        uint64_t vstride) {
  __shared__ uint32_t sh[4];
  hist = vptr(hist, vstride), row_total = vptr(row_total, vstride);
  radix_row_scan(hist + (size_t)blockIdx.x * nb, nb, row_total + blockIdx.x, sh);
}

// AUX: a second value stream travels with the keys (aux_in[i] -> aux_out[pos]).  BITS: the digit
// width, a template parameter so the ballot ranking unrolls.
// 32-bit positions: the scatter takes 86 VGPRs (5 waves / SIMD; 64-bit: 108, 4 waves): C3 1026 ->
// 1037 it/s, scatter 19.4 -> 18.1 us.  6 waves requested (80 VGPRs, one spill): no further change.
template <bool AUX, int BITS>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, const uint32_t* n_dev, uint32_t n_max, int shift, uint32_t chunk,
    uint32_t nb, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ row_total, bool drop,
    const uint32_t* __restrict__ aux_in, uint32_t* __restrict__ aux_out, uint64_t vstride) {
  __shared__ uint32_t s_base[RADIX];      // global position of the next key of each digit
  __shared__ uint32_t s_wcnt[4][RADIX];   // per-wave running counts -> per-wave exclusive prefix
  __shared__ uint32_t s_loc[RADIX];       // digit offsets inside the tile (for the LDS reorder)
  __shared__ uint32_t s_tot[RADIX];
  __shared__ uint32_t s_scan[4];
  __shared__ uint32_t s_key[SORT_TILE];
  __shared__ uint32_t s_val[SORT_TILE];
  __shared__ uint32_t s_aux[AUX ? SORT_TILE : 1];
  keys_in = vptr(keys_in, vstride), vals_in = vptr(vals_in, vstride), keys_out = vptr(keys_out, vstride);
  vals_out = vptr(vals_out, vstride), n_dev = vptr(n_dev, vstride), hist = vptr(hist, vstride);
  row_total = vptr(row_total, vstride), aux_in = vptr(aux_in, vstride), aux_out = vptr(aux_out, vstride);
  const uint32_t n = resolve_n(n_dev, n_max);
  const uint32_t tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  {
    uint32_t all;
    const uint32_t digit_base = block_excl_scan(row_total[tid], s_scan, &all);
    s_base[tid] = digit_base + hist[(size_t)tid * nb + blockIdx.x];
  }
  // 32-bit positions (n < 2^32): fewer registers than 64-bit index math for the 8 items
  const uint32_t start = blockIdx.x * chunk;
  const uint32_t end = start + chunk < n ? start + chunk : n;
  constexpr uint32_t mask = (1u << BITS) - 1u;
  for (uint32_t t0 = start; t0 < end; t0 += SORT_TILE) {
    s_wcnt[0][tid] = 0;
    s_wcnt[1][tid] = 0;
    s_wcnt[2][tid] = 0;
    s_wcnt[3][tid] = 0;
    lds_barrier();
    // wave wid ranks positions t0 + wid*512 + r*64 + lane, r = 0..7 (in order -> stable)
    uint32_t key[SORT_ITEMS], val[SORT_ITEMS], rank[SORT_ITEMS], aux[AUX ? SORT_ITEMS : 1];
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
      const uint32_t i = t0 + wid * (SORT_ITEMS * 64) + (uint32_t)r * 64 + lane;
      const bool v = i < end;
      key[r] = v ? keys_in[i] : 0xFFFFFFFFu;
      val[r] = v ? (vals_in ? vals_in[i] : (uint32_t)i) : 0u;
      if constexpr (AUX) aux[r] = v ? aux_in[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
      const uint32_t i = t0 + wid * (SORT_ITEMS * 64) + (uint32_t)r * 64 + lane;
      const bool v = i < end && !(drop && key[r] == DEPTH_DROP);
      const uint32_t d = (key[r] >> shift) & mask;
      const uint64_t peers = digit_peers(d, v, BITS);
      const uint32_t before = (uint32_t)__popcll(peers & lanemask_lt());
      const uint32_t run = v ? s_wcnt[wid][d] : 0u;
      rank[r] = run + before;
      // make sure every lane read the running count before the leader bumps it
      __builtin_amdgcn_wave_barrier();
      if (v && before == 0) s_wcnt[wid][d] = run + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    lds_barrier();
    // digit tid: prefix over waves, tile total, then exclusive scan of totals over digits
    const uint32_t c0 = s_wcnt[0][tid], c1 = s_wcnt[1][tid], c2 = s_wcnt[2][tid], c3 = s_wcnt[3][tid];
    const uint32_t tot = c0 + c1 + c2 + c3;
    uint32_t tot_all;
    const uint32_t loc = block_excl_scan(tot, s_scan, &tot_all);
    s_wcnt[0][tid] = 0;
    s_wcnt[1][tid] = c0;
    s_wcnt[2][tid] = c0 + c1;
    s_wcnt[3][tid] = c0 + c1 + c2;
    s_loc[tid] = loc;
    s_tot[tid] = tot;
    lds_barrier();
    // reorder the tile by digit in LDS
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
      const uint32_t i = t0 + wid * (SORT_ITEMS * 64) + (uint32_t)r * 64 + lane;
      if (i < end && !(drop && key[r] == DEPTH_DROP)) {
        const uint32_t d = (key[r] >> shift) & mask;
        const uint32_t slot = s_loc[d] + s_wcnt[wid][d] + rank[r];
        s_key[slot] = key[r];
        s_val[slot] = val[r];
        if constexpr (AUX) s_aux[slot] = aux[r];
      }
    }
    lds_barrier();
    // write runs of equal digits contiguously
    const uint32_t ntile = tot_all;  // keys kept in this tile
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
      const uint32_t slot = (uint32_t)r * SORT_THREADS + tid;
      if (slot < ntile) {
        const uint32_t k = s_key[slot];
        const uint32_t d = (k >> shift) & mask;
        const uint32_t pos = s_base[d] + (slot - s_loc[d]);
        keys_out[pos] = k;
        vals_out[pos] = s_val[slot];
        if constexpr (AUX) aux_out[pos] = s_aux[slot];
      }
    }
    lds_barrier();
    s_base[tid] += s_tot[tid];
  }
}

template <bool AUX>
static inline void launch_scatter(int bits, uint32_t nb, hipStream_t st, const uint32_t* kin, const uint32_t* vin,
                                  uint32_t* kout, uint32_t* vout, const uint32_t* nd, uint32_t n_max, int shift,
                                  uint32_t chunk, const uint32_t* hist, const uint32_t* row_total, bool drop,
                                  const uint32_t* ain, uint32_t* aout, int views, uint64_t vstride) {
#define GS_SCATTER(B)                                                                                       \
  GS_LAUNCH("radix_scatter", (k_radix_scatter<AUX, B>), dim3(nb, views), dim3(SORT_THREADS), 0, st, kin, vin, \
            kout, vout, nd, n_max, shift, chunk, nb, hist, row_total, drop, ain, aout, vstride)
  if constexpr (AUX) {
    // a second value stream travels only with the 32-bit depth keys (four 8-bit passes): no other
    // width is instantiated
    GS_SCATTER(8);
  } else {
    switch (bits) {
      case 8: GS_SCATTER(8); break;
      case 7: GS_SCATTER(7); break;
      case 6: GS_SCATTER(6); break;
      case 5: GS_SCATTER(5); break;
      case 4: GS_SCATTER(4); break;
      case 3: GS_SCATTER(3); break;
      case 2: GS_SCATTER(2); break;
      default: GS_SCATTER(1); break;
    }
  }
#undef GS_SCATTER
}

// aux0 / aux_a / aux_b (optional): a second value stream in input order (aux0) that travels with
// the keys (32-bit keys only: every pass then has 8-bit digits, the only aux scatter built); pass p writes aux_a (p even) or aux_b (p odd), so the result is in aux_b after an even
// number of passes and in aux_a after an odd one.
// hist0_ready: the caller already wrote the first pass's [digit][block] counts into scratch.
// drop_first: the first pass reads n_max keys (host count) and drops those equal to DEPTH_DROP;
// the later passes then sort the *n_dev survivors.  Otherwise every pass sorts n (n_dev / n_max).
// views / vstride: `views` such sorts at once, view v's arrays (every pointer argument) lying
// v * vstride bytes after view 0's.
static inline bool radix_sort_pairs(uint32_t* keys_a, uint32_t* vals_a, uint32_t* keys_b, uint32_t* vals_b,
                                    bool vals_identity, const uint32_t* n_dev, uint32_t n_max, int end_bit,
                                    uint32_t* scratch, hipStream_t st, bool drop_first = false,
                                    bool hist0_ready = false, const uint32_t* aux0 = nullptr,
                                    uint32_t* aux_a = nullptr, uint32_t* aux_b = nullptr,
                                    const uint32_t* keys_in0 = nullptr, uint32_t max_blocks = SORT_MAX_BLOCKS,
                                    int views = 1, uint64_t vstride = 0) {
  if (aux0 && end_bit != 32) {
    // only the 8-bit aux scatter is built (launch_scatter<true>): a second value stream needs 32-bit keys
    host_error("radix_sort_pairs: a second value stream travels only with 32-bit keys (four 8-bit passes)");
    return false;
  }
  SortPlan p = sort_plan(n_max, max_blocks);
  uint32_t* hist = scratch;
  const size_t hist_n = (size_t)RADIX * p.nb;
  uint32_t* row_total = scratch + hist_n;
  uint32_t *kin = keys_a, *vin = vals_a, *kout = keys_b, *vout = vals_b;
  bool in_b = false;
  const uint32_t* ain = aux0;
  uint32_t* aout = aux_a;
  // digits of (nearly) equal width, the narrower first: 13 bits -> 6 + 7 (C3: -3.6 us over the six scatters)
  const int width = radix_width(end_bit);
  for (int shift = 0; shift < end_bit;) {
    int bits = shift == 0 ? radix_first_bits(end_bit) : (end_bit - shift < width ? end_bit - shift : width);
    const bool drop = drop_first && shift == 0;
    const uint32_t* nd = drop ? nullptr : n_dev;
    // keys_in0: the first pass reads its keys from there (kept), not from keys_a
    const uint32_t* kin_p = (shift == 0 && keys_in0) ? keys_in0 : kin;
    if (!(hist0_ready && shift == 0))
      GS_LAUNCH("radix_hist", k_radix_hist<NoFin>, dim3(p.nb, views), dim3(SORT_THREADS), 0, st, kin_p, nd, n_max,
                shift, bits, p.chunk, p.nb, hist, drop, vstride, NoFin());
    GS_LAUNCH("radix_rowscan", k_radix_rowscan<>, dim3(RADIX, views), dim3(SORT_THREADS), 0, st, hist, p.nb,
              row_total, vstride);
    const uint32_t* vsrc = (shift == 0 && vals_identity) ? nullptr : vin;
    if (aux0) {
      launch_scatter<true>(bits, p.nb, st, kin_p, vsrc, kout, vout, nd, n_max, shift, p.chunk, hist, row_total, drop, ain,
                           aout, views, vstride);
      ain = aout;
      aout = aout == aux_a ? aux_b : aux_a;
    } else {
      launch_scatter<false>(bits, p.nb, st, kin_p, vsrc, kout, vout, nd, n_max, shift, p.chunk, hist, row_total, drop,
                            nullptr, nullptr, views, vstride);
    }
    uint32_t* t;
    t = kin; kin = kout; kout = t;
    t = vin; vin = vout; vout = t;
    in_b = !in_b;
    shift += bits;
  }
  return in_b;
}


}  // namespace gs
