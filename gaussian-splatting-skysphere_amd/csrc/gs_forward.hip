// gs_forward.hip -- forward pass of the MI355X Gaussian rasterizer (gfx950).
//
// Restates the un-vendored upstream forward (graphdeco-inria/diff-gaussian-rasterization,
// /root/reference/.gitmodules:4-6; spec SURVEY.md §8a a4-a6) as:
//   k_preprocess   one lane per Gaussian: cull, project, cov3D -> EWA cov2D -> conic, radius,
//                  tile rectangle, SH -> RGB; writes the 48-B splat record used by render.
//   fwd_order      stable 32-bit depth radix sort of the Gaussians with instances (the first
//                  pass drops the others: compaction), exclusive scan of their tile counts in
//                  depth order.
//   k_duplicate    one lane per depth-ranked Gaussian writes its (tile, slot) instances; slots of
//                  a Gaussian are contiguous and in depth order.
//   tile sort      stable radix sort of the instances by tile id only: because the input is
//                  already depth-ordered (ties by Gaussian index) this equals upstream's sort by
//                  the 64-bit key (tile << 32 | depth bits) with a ~3x smaller sort.
//   k_ranges       per-tile [start, end) of the sorted list.
//   k_render_fwd   one 256-lane workgroup (4 wave64) per 16x16 tile; Gaussians staged through LDS
//                  256 at a time; front-to-back compositing with the block-wide early exit.
#include "gs_internal.h"

namespace gs {

// ------------------------------------------------------------------------------------------
// preprocess
// ------------------------------------------------------------------------------------------

// SH -> RGB for one Gaussian, channel-major evaluation order identical to oracle/gs_oracle.c
// sh_eval_one (reference: /root/reference/utils/sh_utils.py:57-100, +0.5 and clamp_min(0) as
// /root/reference/gaussian_renderer/__init__.py:77-78).
// rest != null: split rows (sh = the Gaussian's features_dc row, rest = its features_rest row),
// read as 12-B pieces; the evaluation is the same.
template <int DEG>
__device__ __forceinline__ void sh_to_rgb(const float* __restrict__ sh, const float* __restrict__ rest, int M, float x,
                                          float y, float z, float* rgb, uint32_t& clamped) {
  constexpr int K = (DEG + 1) * (DEG + 1);
  float s[K * 3];
  if (rest) {
    const F3 d = *reinterpret_cast<const F3*>(sh);
    s[0] = d.a, s[1] = d.b, s[2] = d.c;
    const F3* r3 = reinterpret_cast<const F3*>(rest);
#pragma unroll
    for (int j = 0; j < K - 1; j++) {
      const F3 t = r3[j];
      s[3 + 3 * j] = t.a, s[4 + 3 * j] = t.b, s[5 + 3 * j] = t.c;
    }
  } else if (((M * 3) & 3) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(sh);
#pragma unroll
    for (int v = 0; v < (K * 3 + 3) / 4; v++) {
      float4 q = s4[v];
      if (4 * v + 0 < K * 3) s[4 * v + 0] = q.x;
      if (4 * v + 1 < K * 3) s[4 * v + 1] = q.y;
      if (4 * v + 2 < K * 3) s[4 * v + 2] = q.z;
      if (4 * v + 3 < K * 3) s[4 * v + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < K * 3; k++) s[k] = sh[k];
  }
  clamped = 0;
#pragma unroll
  for (int c = 0; c < 3; c++) {
#define S(k) s[3 * (k) + c]
    float res = SH_C0 * S(0);
    if (DEG > 0) {
      res = res - (SH_C1 * y) * S(1) + (SH_C1 * z) * S(2) - (SH_C1 * x) * S(3);
      if (DEG > 1) {
        float xx = x * x, yy = y * y, zz = z * z;
        float xy = x * y, yz = y * z, xz = x * z;
        res = res + (SH_C20 * xy) * S(4) + (SH_C21 * yz) * S(5) + (SH_C22 * (2.0f * zz - xx - yy)) * S(6) +
              (SH_C23 * xz) * S(7) + (SH_C24 * (xx - yy)) * S(8);
        if (DEG > 2) {
          res = res + ((SH_C30 * y) * (3.0f * xx - yy)) * S(9) + ((SH_C31 * xy) * z) * S(10) +
                ((SH_C32 * y) * (4.0f * zz - xx - yy)) * S(11) +
                ((SH_C33 * z) * (2.0f * zz - 3.0f * xx - 3.0f * yy)) * S(12) +
                ((SH_C34 * x) * (4.0f * zz - xx - yy)) * S(13) + ((SH_C35 * z) * (xx - yy)) * S(14) +
                ((SH_C36 * x) * (xx - 3.0f * yy)) * S(15);
        }
      }
    }
#undef S
    res = res + 0.5f;
    if (res < 0.0f) clamped |= 1u << c;
    rgb[c] = res < 0.0f ? 0.0f : res;
  }
}

// DEG = -1: colours precomputed by the caller
// One Gaussian; returns the number of tiles it touches (0 when culled).
// SPLIT: SH rows from g.shs (features_dc) + g.shs_rest when g.shs_rest is set (a uniform branch:
// with both row loaders in the kernel the scheduler keeps the split loads where they are used, 91
// VGPRs; a split-only instantiation hoists them, 130 VGPRs, 75 -> 97 us at C3)
template <int DEG, bool SPLIT = false>
__device__ __forceinline__ uint32_t preprocess_one(int i, const GaussianArgs& g, const CameraArgs& c,
                                                   int* __restrict__ radii, float4* __restrict__ splat,
                                                   float4* __restrict__ binrec, uint32_t& dbits,
                                                   uint32_t* __restrict__ tiles, uint8_t* __restrict__ clamped,
                                                   bool& culled_prefiltered) {
  radii[i] = 0;
  tiles[i] = 0;
  const float px = g.means3D[3 * i + 0], py = g.means3D[3 * i + 1], pz = g.means3D[3 * i + 2];
  const float3v pv = xf43(c.view, px, py, pz);
  if (pv.z <= 0.2f) {
    culled_prefiltered = c.prefiltered != 0;  // upstream raises "Point is filtered although prefiltered is set"
    return 0;
  }
  const float* P = c.proj;
  const float hx = P[0] * px + P[4] * py + P[8] * pz + P[12];
  const float hy = P[1] * px + P[5] * py + P[9] * pz + P[13];
  const float hw = xf44w(P, px, py, pz);
  const float pw = 1.0f / (hw + 0.0000001f);
  const float projx = hx * pw, projy = hy * pw;

  float cov3[6];
  if (g.cov3D) {
#pragma unroll
    for (int k = 0; k < 6; k++) cov3[k] = g.cov3D[6 * i + k];
  } else {
    cov3d(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2], g.scale_modifier, g.rotations[4 * i],
          g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3], cov3);
  }
  const Cov2D cv = cov2d(c.view, px, py, pz, cov3, c.fx, c.fy, c.tanfovx, c.tanfovy);
  const float det = cv.a * cv.c - cv.b * cv.b;
  if (det == 0.0f) return 0;
  const float det_inv = 1.f / det;
  const float cxx = cv.c * det_inv, cxy = -cv.b * det_inv, cyy = cv.a * det_inv;
  const float mid = 0.5f * (cv.a + cv.c);
  const float disc = fmaxf(0.1f, mid * mid - det);
  const float l1 = mid + sqrtf(disc), l2 = mid - sqrtf(disc);
  const int radius = (int)ceilf(3.f * sqrtf(fmaxf(l1, l2)));
  const float sx = ndc2pix(projx, c.W), sy = ndc2pix(projy, c.H);
  int x0, y0, x1, y1;
  get_rect(sx, sy, radius, c.gx, c.gy, x0, y0, x1, y1);
  const int area = (x1 - x0) * (y1 - y0);
  if (area == 0) return 0;

  float rgb[3];
  uint32_t cl = 0;
  if (DEG < 0) {
    rgb[0] = g.colors[3 * i];
    rgb[1] = g.colors[3 * i + 1];
    rgb[2] = g.colors[3 * i + 2];
  } else {
    float dx = px - c.campos[0], dy = py - c.campos[1], dz = pz - c.campos[2];
    float len = sqrtf(dx * dx + dy * dy + dz * dz);
    if (SPLIT && g.shs_rest)
      sh_to_rgb<(DEG < 0 ? 0 : DEG)>(g.shs + (size_t)i * 3, g.shs_rest + (size_t)i * (g.M - 1) * 3, g.M, dx / len,
                                     dy / len, dz / len, rgb, cl);
    else
      sh_to_rgb<(DEG < 0 ? 0 : DEG)>(g.shs + (size_t)i * g.M * 3, nullptr, g.M, dx / len, dy / len, dz / len, rgb, cl);
  }
  // culling limit of the {alpha >= 1/255} ellipse (render-side work skipping only; never
  // changes a result, see ellipse_meets_rect): q(d) <= 2 ln(255 o), with safety margins
  const float op = g.opacities[i];
  const float lim = cull_lim(op);
  splat[3 * i + 0] = make_float4(sx, sy, cxx, cxy);
  splat[3 * i + 1] = make_float4(cyy, op, rgb[0], rgb[1]);
  splat[3 * i + 2] = make_float4(rgb[2], pv.z, lim, 0.0f);
  dbits = __float_as_uint(pv.z);
  radii[i] = radius;  // upstream visibility: the rectangle is non-empty
  // tile-exact instance count (may be 0 for a visible splat whose alpha never reaches 1/255)
  const SpanCtx sp = span_ctx(sx, sy, cxx, cxy, cyy, lim, x0, x1);
  uint32_t count = 0;
  for (int ty = y0; ty < y1; ty++) {
    int ta, tb;
    row_span(sp, ty, ta, tb);
    count += (uint32_t)(tb - ta);
  }
  binrec[2 * i + 0] = make_float4(sx, sy, cxx, cxy);
  binrec[2 * i + 1] = make_float4(cyy, lim, __uint_as_float((uint32_t)x0 | ((uint32_t)x1 << 16)),
                                  __uint_as_float((uint32_t)y0 | ((uint32_t)y1 << 16)));
  tiles[i] = count;
  clamped[i] = (uint8_t)cl;
  return count;
}


// The workgroup's tile total and count of Gaussians with instances (+ a prefiltered cull) -> its
// WgTotals slot; the first depth-sort histogram launch sums the slots (CounterFinalize).
__device__ __forceinline__ void workgroup_totals(uint32_t area, bool culled, WgTotals* wg, uint32_t b) {
  __shared__ uint32_t s_sum[4], s_vis[4];
  uint32_t vis = area ? 1u : 0u;
  const uint64_t cm = __ballot(culled);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    area += (uint32_t)__shfl_xor((int)area, d, 64);
    vis += (uint32_t)__shfl_xor((int)vis, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_sum[threadIdx.x >> 6] = area;
    s_vis[threadIdx.x >> 6] = vis | (cm ? 0x80000000u : 0u);
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    const uint32_t tot = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
    const uint32_t v4 = s_vis[0] | s_vis[1] | s_vis[2] | s_vis[3];
    const uint32_t nv = (s_vis[0] & 0x7FFFFFFFu) + (s_vis[1] & 0x7FFFFFFFu) + (s_vis[2] & 0x7FFFFFFFu) +
                        (s_vis[3] & 0x7FFFFFFFu);
    store_wg_totals(wg, b, nv, tot, (v4 >> 31) != 0);
  }
}

// The workgroup's tile total (num_rendered, read back by the host right after the first depth-sort
// histogram launch while the ordering kernels run) and its count of Gaussians with instances (V)
// go to its WgTotals slot (workgroup_totals).  depth_key[i] is the depth's bits for those and
// DEPTH_DROP for every other Gaussian: the first depth-sort pass drops them, which is the
// visibility compaction.
template <int DEG>
__global__ __launch_bounds__(256) void k_preprocess(GaussianArgs g, CameraArgs c, int* __restrict__ radii,
                                                    float4* __restrict__ splat, float4* __restrict__ binrec,
                                                    uint32_t* __restrict__ depth_key,
                                                    uint32_t* __restrict__ tiles, uint8_t* __restrict__ clamped,
                                                    WgTotals* __restrict__ wg) {
  const int b = (int)blockIdx.x + g.blk0, i = b * 256 + (int)threadIdx.x;
  uint32_t area = 0, dbits = 0;
  bool culled = false;
  if (i < g.P) {
    area = preprocess_one<DEG>(i, g, c, radii, splat, binrec, dbits, tiles, clamped, culled);
    depth_key[i] = area ? dbits : DEPTH_DROP;
  }
  workgroup_totals(area, culled, wg, (uint32_t)b);
}

// The split-SH preprocess: k_preprocess's body with the split row loader (preprocess_one SPLIT).
template <int DEG>
__global__ __launch_bounds__(256) void k_preprocess_split(
    GaussianArgs g, CameraArgs c, int* __restrict__ radii, float4* __restrict__ splat, float4* __restrict__ binrec,
    uint32_t* __restrict__ depth_key, uint32_t* __restrict__ tiles, uint8_t* __restrict__ clamped,
    WgTotals* __restrict__ wg) {
  const int b = (int)blockIdx.x + g.blk0, i = b * 256 + (int)threadIdx.x;
  uint32_t area = 0, dbits = 0;
  bool culled = false;
  if (i < g.P) {
    area = preprocess_one<DEG, true>(i, g, c, radii, splat, binrec, dbits, tiles, clamped, culled);
    depth_key[i] = area ? dbits : DEPTH_DROP;
  }
  workgroup_totals(area, culled, wg, (uint32_t)b);
}

// The preprocess grid, launched whole or -- with row waits installed on this thread
// (gs_set_row_waits) -- in row chunks: before chunk k the stream waits for event k, and chunk k
// launches the workgroups whose last row lies below its end, so every row a workgroup reads is
// behind all the waits of the chunks it spans (e.g. the all-gather of a sharded optimizer step's
// row chunk, gs_view_parallel.ShardedAdam).  Same workgroups, same outputs as one launch.
template <class Launch>
static void launch_row_chunks(const GaussianArgs& g, hipStream_t st, Launch&& launch) {
  const int nb = (g.P + 255) / 256;
  RowWait w[GS_MAX_ROW_WAITS];
  const int n = take_row_waits(w, GS_MAX_ROW_WAITS);
  int b0 = 0;
  for (int k = 0; k < n && b0 < nb; k++) {
    if (w[k].ev && !stream_wait(st, w[k].ev)) return;
    const int b1 = w[k].hi >= g.P ? nb : w[k].hi / 256;
    if (b1 > b0) {
      GaussianArgs gc = g;
      gc.blk0 = b0;
      launch(gc, dim3(b1 - b0));
      b0 = b1;
    }
  }
  if (b0 < nb) {
    GaussianArgs gc = g;
    gc.blk0 = b0;
    launch(gc, dim3(nb - b0));
  }
}

void fwd_preprocess(const GaussianArgs& g0, const CameraArgs& c, int* radii, const GeomPtrs& geo, hipStream_t st) {
  launch_row_chunks(g0, st, [&](const GaussianArgs& g, dim3 grid) { fwd_preprocess_grid(g, c, radii, geo, st, grid); });
}

void fwd_preprocess_grid(const GaussianArgs& g, const CameraArgs& c, int* radii, const GeomPtrs& geo, hipStream_t st,
                         dim3 grid) {
  const dim3 block(256);
  if (g.colors) {
    GS_LAUNCH("preprocess", k_preprocess<-1>, grid, block, 0, st, g, c, radii, geo.splat, geo.binrec, geo.keys_a, geo.tiles,
              geo.clamped, geo.wg_tot);
    return;
  }
  if (g.shs_rest) {  // split SH rows (M >= 2, so D >= 0 applies)
#define GS_PRE_SPLIT(D)                                                                                        \
  GS_LAUNCH("preprocess", (k_preprocess_split<D>), grid, block, 0, st, g, c, radii, geo.splat, geo.binrec, \
            geo.keys_a, geo.tiles, geo.clamped, geo.wg_tot)
    switch (g.D) {
      case 0: GS_PRE_SPLIT(0); break;
      case 1: GS_PRE_SPLIT(1); break;
      case 2: GS_PRE_SPLIT(2); break;
      default: GS_PRE_SPLIT(3); break;
    }
#undef GS_PRE_SPLIT
    return;
  }
  switch (g.D) {
    case 0:
      GS_LAUNCH("preprocess", k_preprocess<0>, grid, block, 0, st, g, c, radii, geo.splat, geo.binrec, geo.keys_a, geo.tiles,
                geo.clamped, geo.wg_tot);
      break;
    case 1:
      GS_LAUNCH("preprocess", k_preprocess<1>, grid, block, 0, st, g, c, radii, geo.splat, geo.binrec, geo.keys_a, geo.tiles,
                geo.clamped, geo.wg_tot);
      break;
    case 2:
      GS_LAUNCH("preprocess", k_preprocess<2>, grid, block, 0, st, g, c, radii, geo.splat, geo.binrec, geo.keys_a, geo.tiles,
                geo.clamped, geo.wg_tot);
      break;
    default:
      GS_LAUNCH("preprocess", k_preprocess<3>, grid, block, 0, st, g, c, radii, geo.splat, geo.binrec, geo.keys_a, geo.tiles,
                geo.clamped, geo.wg_tot);
      break;
  }
}

// K views in one launch: every lane runs the single-view preprocess of its Gaussian for each
// camera in turn (preprocess_one, so each view's outputs are bit-identical to its own launch);
// the Gaussian's inputs come from HBM once, the later views read them from the caches.  The
// per-view workgroup totals go to each view's WgTotals slots as in k_preprocess.
template <int DEG>
__global__ __launch_bounds__(256) void k_preprocess_views(GaussianArgs g, PreViews pv) {
  const int b = (int)blockIdx.x + g.blk0, i = b * 256 + (int)threadIdx.x;
  for (int v = 0; v < pv.K; v++) {
    const GeomPtrs& geo = pv.geo[v];
    uint32_t area = 0, dbits = 0;
    bool culled = false;
    if (i < g.P) {
      area = preprocess_one<DEG>(i, g, pv.c[v], pv.radii[v], geo.splat, geo.binrec, dbits, geo.tiles, geo.clamped,
                                 culled);
      geo.keys_a[i] = area ? dbits : DEPTH_DROP;
    }
    workgroup_totals(area, culled, geo.wg_tot, (uint32_t)b);
    lds_barrier();  // workgroup_totals' LDS is reused by the next view
  }
}

void fwd_preprocess_views(const GaussianArgs& g0, const PreViews& pv, hipStream_t st) {
  launch_row_chunks(g0, st, [&](const GaussianArgs& g, dim3 grid) {
    const dim3 block(256);
    if (g.colors) {
      GS_LAUNCH("preprocess_views", k_preprocess_views<-1>, grid, block, 0, st, g, pv);
      return;
    }
    switch (g.D) {
      case 0: GS_LAUNCH("preprocess_views", k_preprocess_views<0>, grid, block, 0, st, g, pv); break;
      case 1: GS_LAUNCH("preprocess_views", k_preprocess_views<1>, grid, block, 0, st, g, pv); break;
      case 2: GS_LAUNCH("preprocess_views", k_preprocess_views<2>, grid, block, 0, st, g, pv); break;
      default: GS_LAUNCH("preprocess_views", k_preprocess_views<3>, grid, block, 0, st, g, pv); break;
    }
  });
}

// ------------------------------------------------------------------------------------------
// ordering: compaction -> depth sort -> instance offsets
// ------------------------------------------------------------------------------------------

struct SrcTilesByRank {
  const uint32_t *tiles, *sorted_gid;
  uint32_t P;
  // (a depth sort whose look-back timed out leaves stale ids: stay in bounds, the forward raises)
  __device__ uint32_t operator()(uint32_t s) const {
    const uint32_t g = sorted_gid[s];
    return g < P ? tiles[g] : 0u;
  }
};

// instance offsets in depth order; also records, for every DUP_SLOTS-aligned slot, the depth rank
// that owns it (the start of each load-balanced duplicate block)
struct DstOffsets {
  uint32_t* offsets;
  uint32_t* first;
  const uint32_t* counters;  // [CNT_NREND] I (summed by preprocess, complete before this scan runs)
  uint32_t P;
  __device__ void operator()(uint32_t s, uint32_t ex, uint32_t v) const {
    offsets[s] = ex;
    const uint32_t I = counters[CNT_NREND];
    if (!dup_balanced(I, P)) return;
    for (uint32_t m = (ex + DUP_SLOTS - 1) / DUP_SLOTS; m * DUP_SLOTS < ex + v && m * DUP_SLOTS < I; m++) first[m] = s;
  }
};

// workgroups per tile-sort / depth-sort pass (sort_plan): one per 2048-key tile up to 8M keys
// (128 or 256 depth-sort workgroups, smaller histograms but longer scatters: 961 -> 953 / 924 it/s)
constexpr uint32_t GS_TILE_SORT_BLOCKS = 4096, GS_DEPTH_SORT_BLOCKS = 4096;
// The extra workgroup of the first depth-sort histogram launch: the view's totals from the preprocess
// workgroups' WgTotals (64-bit instance sum: an overflow of the 32-bit instance positions is seen
// exactly), written to the view's counters (which need no zeroing beforehand: every counter the
// later kernels read is set here) and to the host's readback words (host: a device-visible pointer
// into pinned host memory, or null): [0] instances low, [1] high, [2] V, [3] error flags.
struct CounterFinalize {
  static constexpr bool active = true;
  const WgTotals* wg;
  uint32_t nwg;
  uint32_t* counters;
  uint32_t* host;    // view v's words at host + 8 v
  uint32_t* sticky;  // pinned host words for a view with error flags (gs_forward_bounded), or null
  uint64_t vstride;  // bytes between the views' geometry buffers (batched launch)
  uint32_t cap[FUSED_MAX_VIEWS];  // the views' binning capacities
  __device__ void operator()(uint32_t v) const {
    const WgTotals* wg = vptr(this->wg, vstride);
    uint32_t* counters = vptr(this->counters, vstride);
    uint32_t* host = this->host ? this->host + 8 * v : nullptr;
    const uint32_t cap = this->cap[v];
    __shared__ uint32_t s_lo[4], s_hi[4], s_v[4], s_e[4];
    unsigned long long si = 0;
    uint32_t sv = 0, se = 0;
    for (uint32_t k = threadIdx.x; k < nwg; k += SORT_THREADS) {
      const WgTotals t = wg[k];
      si += t.inst;
      sv += t.vis & 0x7FFFFFFFu;
      se |= t.vis >> 31;
    }
    uint32_t lo = (uint32_t)si, hi = (uint32_t)(si >> 32);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const uint32_t olo = (uint32_t)__shfl_xor((int)lo, d, 64), ohi = (uint32_t)__shfl_xor((int)hi, d, 64);
      const unsigned long long a = ((unsigned long long)hi << 32 | lo) + ((unsigned long long)ohi << 32 | olo);
      lo = (uint32_t)a;
      hi = (uint32_t)(a >> 32);
      sv += (uint32_t)__shfl_xor((int)sv, d, 64);
      se |= (uint32_t)__shfl_xor((int)se, d, 64);
    }
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s_lo[w] = lo, s_hi[w] = hi, s_v[w] = sv, s_e[w] = se;
    lds_barrier();
    if (threadIdx.x == 0) {
      unsigned long long I = 0;
      uint32_t V = 0, e = 0;
      for (int k = 0; k < SORT_THREADS / 64; k++) {
        I += (unsigned long long)s_hi[k] << 32 | s_lo[k];
        V += s_v[k];
        e |= s_e[k];
      }
      const uint32_t err = (e ? ERR_PREFILTERED : 0u) | (I > (unsigned long long)GS_MAX_INSTANCES ? ERR_INSTANCES : 0u) |
                           (I > (unsigned long long)cap ? ERR_CAPACITY : 0u);
      counters[CNT_NREND] = (uint32_t)I;
      counters[CNT_V] = V;
      counters[CNT_ERR] = err;
      counters[CNT_I] = 0u;
      counters[CNT_LB_TILE] = 0u;
      counters[CNT_SEQ] = counters[CNT_SEQ] + 1u;
      if (host) {
        host[0] = (uint32_t)I;
        host[1] = (uint32_t)(I >> 32);
        host[2] = V;
        host[3] = err;
      }
      if (sticky && err) {
        sticky[0] = err;
        sticky[1] = (uint32_t)I;
        sticky[2] = (uint32_t)(I >> 32);
      }
    }
  }
};

void fwd_scan(int P, const GeomPtrs& geo, hipStream_t st);

void fwd_order(int P, const GeomPtrs& geo, hipStream_t st, uint32_t* host_counts, hipEvent_t counts_ready,
               const uint32_t* cap, uint32_t* sticky, int views, uint64_t vstride) {
  const uint32_t n = (uint32_t)P;
  // the first depth-sort pass's counts, with each view's totals finalised by an extra workgroup
  // (the host waits for this launch only: the rest of the ordering overlaps its readback)
  const SortPlan sp = sort_plan(n, GS_DEPTH_SORT_BLOCKS);
  CounterFinalize fin{geo.wg_tot, (n + 255) / 256, geo.counters, host_counts, sticky, vstride, {}};
  for (int v = 0; v < FUSED_MAX_VIEWS; v++) fin.cap[v] = cap && v < views ? cap[v] : 0xFFFFFFFFu;
  GS_LAUNCH("radix_hist", k_radix_hist<CounterFinalize>, dim3(sp.nb + 1, views), dim3(SORT_THREADS), 0, st,
            geo.keys_a, nullptr, n, 0, radix_first_bits(32), sp.chunk, sp.nb, geo.sort_scratch, true, vstride, fin);
  if (counts_ready) (void)hipEventRecord(counts_ready, st);
  // depth sort of the Gaussians with instances: the first pass reads all P keys in index order
  // and drops the DEPTH_DROP ones (compaction), the later passes sort the V survivors; every
  // view's passes in one set of launches (blockIdx.y = view)
  if (lb_tiles(n) <= LB_STATIC_MAX) {
    radix_sort_pairs(geo.keys_a, geo.vals_a, geo.keys_b, geo.vals_b, true, &geo.counters[CNT_V], n, 32,
                     geo.sort_scratch, st, /*drop_first=*/true, /*hist0_ready=*/true, nullptr, nullptr, nullptr,
                     nullptr, GS_DEPTH_SORT_BLOCKS, views, vstride);
  } else {
    // larger scenes: the tile counts travel with the keys through the sort (read in index order by
    // the first pass), and the 3-launch scan reads them in depth order, coalesced (C5, 5M: the
    // per-rank gather and the ticketed look-back took 197 us)
    radix_sort_pairs(geo.keys_a, geo.vals_a, geo.keys_b, geo.vals_b, true, &geo.counters[CNT_V], n, 32,
                     geo.sort_scratch, st, /*drop_first=*/true, /*hist0_ready=*/true, geo.tiles, geo.rtiles_a,
                     geo.rtiles_b, nullptr, GS_DEPTH_SORT_BLOCKS, views, vstride);
  }
  for (int v = 0; v < views; v++) {
    GeomPtrs g = geo;
    if (v) geom_layout((size_t)P, &g, (char*)geo.splat + (uint64_t)v * vstride);
    fwd_scan(P, g, st);
  }
}

__global__ __launch_bounds__(64) void k_clear_flags(uint32_t* __restrict__ err, uint32_t bits) {
  if (threadIdx.x == 0) err[0] = err[0] & ~bits;
}
void fwd_clear_flags(const GeomPtrs& geo, uint32_t bits, hipStream_t st) {
  GS_LAUNCH("clear_flags", k_clear_flags, dim3(1), dim3(64), 0, st, &geo.counters[CNT_ERR], bits);
}

// instance offsets in depth order (+ the duplicate's block owner table), after the depth sort
void fwd_scan(int P, const GeomPtrs& geo, hipStream_t st) {
  const uint32_t n = (uint32_t)P;
  if (lb_tiles(n) <= LB_STATIC_MAX) {
    // up to 1M Gaussians: one look-back launch whose grid is resident (static tile ids); it
    // gathers each rank's tile count (cheaper here than carrying the counts through the four sort
    // passes)
    scan_exclusive_lb(SrcTilesByRank{geo.tiles, geo.sorted_gid, n}, DstOffsets{geo.offsets, geo.dup_first, geo.counters, n},
                      &geo.counters[CNT_V], n, geo.lb_status, &geo.counters[CNT_LB_TILE], &geo.counters[CNT_I],
                      &geo.counters[CNT_ERR], st, &geo.counters[CNT_SEQ]);
  } else {
    scan_exclusive(SrcArray{geo.tiles_by_rank}, DstOffsets{geo.offsets, geo.dup_first, geo.counters, n},
                   &geo.counters[CNT_V], n, geo.scan_partial, &geo.counters[CNT_I], st);
  }
}

// ------------------------------------------------------------------------------------------
// binning
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ SpanCtx span_of(const float4* __restrict__ binrec, uint32_t gid, int& y0, int& y1) {
  const float4 a = binrec[2 * gid], b = binrec[2 * gid + 1];
  const uint32_t xr = __float_as_uint(b.z), yr = __float_as_uint(b.w);
  y0 = (int)(yr & 0xFFFFu);
  y1 = (int)(yr >> 16);
  return span_ctx(a.x, a.y, a.z, a.w, b.x, b.y, (int)(xr & 0xFFFFu), (int)(xr >> 16));
}

__global__ __launch_bounds__(256) void k_duplicate(uint32_t P, const uint32_t* __restrict__ counters,
                                                   const uint32_t* __restrict__ sorted_gid,
                                                   const uint32_t* __restrict__ offsets,
                                                   const float4* __restrict__ binrec, int gx,
                                                   uint32_t* __restrict__ tile_keys,
                                                   uint32_t* __restrict__ presort_gid) {
  const uint32_t s = blockIdx.x * 256 + threadIdx.x;
  if (s >= P || s >= counters[CNT_V] || (counters[CNT_ERR] & ERR_INVALID)) return;  // (invalid list: write nothing)
  const uint32_t gid = sorted_gid[s];
  uint32_t off = offsets[s];
  // (a timed-out offsets scan only under-estimates offsets: every write stays below I)
  int y0, y1;
  const SpanCtx sp = span_of(binrec, gid, y0, y1);
  for (int ty = y0; ty < y1; ty++) {
    int ta, tb;
    row_span(sp, ty, ta, tb);
    for (int x = ta; x < tb; x++) {
      tile_keys[off] = (uint32_t)(ty * gx + x);
      presort_gid[off] = gid;
      off++;
    }
  }
}

// Load-balanced duplicate: workgroup b writes instance slots [b S, (b + 1) S), S = DUP_SLOTS.
// The depth ranks owning those slots are [dup_first[b], dup_first[b + 1]] (at most S + 1 of
// them).  Each splat's instances are its tile-exact row spans (row_span), laid out row by row;
// the row segments meeting the block are numbered with a workgroup scan, every slot finds its
// segment by an inclusive max-scan over segment start marks, and keys / presort ids are written
// fully coalesced.  The workgroups also clear the tile ranges (k_ranges fills the non-empty ones).
constexpr int DUP_THREADS = 256;
constexpr int DUP_ITEMS = DUP_SLOTS / DUP_THREADS;
// LDS index of slot i in the owner array: one pad word per 8 slots keeps the per-thread runs of
// 8 consecutive slots on distinct banks
__device__ __forceinline__ uint32_t own_idx(uint32_t i) { return i + (i >> 3); }

// Views (blockIdx.y): view v's geometry / binning / image arrays lie v * gs / bs / is bytes further.
__global__ __launch_bounds__(DUP_THREADS) void k_duplicate_lb(
    uint32_t I, const uint32_t* __restrict__ counters, const uint32_t* __restrict__ dup_first,
    const uint32_t* __restrict__ sorted_gid, const uint32_t* __restrict__ offsets,
    const float4* __restrict__ binrec, int gx, int gy, uint32_t* __restrict__ tile_keys,
    uint32_t* __restrict__ presort_gid, uint2* __restrict__ ranges, uint32_t* __restrict__ hist0, uint32_t mask0,
    uint32_t* __restrict__ n_copy, uint64_t gs, uint64_t bs, uint64_t is) {
  counters = vptr(counters, gs), dup_first = vptr(dup_first, gs), sorted_gid = vptr(sorted_gid, gs);
  offsets = vptr(offsets, gs), binrec = vptr(binrec, gs);
  tile_keys = vptr(tile_keys, bs), presort_gid = vptr(presort_gid, bs), hist0 = vptr(hist0, bs);
  n_copy = vptr(n_copy, bs), ranges = vptr(ranges, is);
  __shared__ uint32_t s_own[DUP_SLOTS + DUP_SLOTS / 8];  // (slot + 1) << 16 | segment at segment starts
  // per row segment: (tile id of its first slot) - (that slot), mod 2^32 (the slot may precede the
  // block), so slot k of the segment has key base + k; one table instead of two keeps the LDS at
  // 26 KB: 6 workgroups per CU
  __shared__ uint32_t s_seg_base[DUP_SLOTS];
  __shared__ uint32_t s_seg_gid[DUP_SLOTS];
  __shared__ uint32_t s_wmax[DUP_THREADS / 64];
  __shared__ uint32_t s_nseg;
  __shared__ uint32_t s_hist[RADIX];
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  s_hist[tid] = 0;
  const uint32_t tiles = (uint32_t)(gx * gy);
  for (uint32_t t = b * DUP_THREADS + tid; t < tiles; t += gridDim.x * DUP_THREADS) ranges[t] = make_uint2(0u, 0u);
  const uint32_t V = counters[CNT_V];
  // I: the binning buffer's capacity (= the count, unless the buffer was sized ahead of it)
  I = min(I, counters[CNT_NREND]);
  if (b == 0 && tid == 0) n_copy[0] = I;  // for the tile sort and k_ranges (kernels after this one)
  const uint32_t k0 = b * DUP_SLOTS;
  const uint32_t k1 = k0 < I ? min(k0 + DUP_SLOTS, I) : k0;
  if (counters[CNT_ERR] & ERR_INVALID) {
    // a look-back wait of the depth sort or the offsets scan timed out, or the instances exceed the
    // buffer (the host raises at its next call): the owner table is not valid, so fill the block's
    // slots with a safe placeholder -- tile 0, Gaussian 0 -- that keeps every later kernel in bounds
    const uint32_t g0 = 0u;
    for (uint32_t k = k0 + tid; k < k1; k += DUP_THREADS) {
      tile_keys[k] = 0u;
      presort_gid[k] = g0;
    }
    if (hist0) {
      hist0[(size_t)tid * gridDim.x + b] = tid == 0 ? k1 - k0 : 0u;
    }
    return;
  }
  if (k1 == k0) {  // past the count (a buffer sized ahead of it): no slots
    if (hist0) hist0[(size_t)tid * gridDim.x + b] = 0u;
    return;
  }
  const uint32_t s_lo = dup_first[b];
  const uint32_t s_hi = (k1 < I) ? dup_first[b + 1] : V - 1;
  const uint32_t nG = s_hi - s_lo + 1;
  for (uint32_t i = tid; i < DUP_SLOTS + DUP_SLOTS / 8; i += DUP_THREADS) s_own[i] = 0;
  if (tid == 0) s_nseg = 0;
  lds_barrier();
  // row segments of the block's splats that meet [k0, k1): any segment numbering works, the
  // marks carry their slot so the scan below picks the segment that starts last at or before
  // each slot (deterministic output)
  for (uint32_t r = tid; r < nG; r += DUP_THREADS) {
    const uint32_t gid = sorted_gid[s_lo + r];
    uint32_t pos = offsets[s_lo + r];
    if (pos >= k1) continue;
    int y0, y1;
    const SpanCtx sp = span_of(binrec, gid, y0, y1);
    for (int ty = y0; ty < y1 && pos < k1; ty++) {
      int ta, tb;
      row_span(sp, ty, ta, tb);
      const uint32_t w = (uint32_t)(tb - ta);
      if (w && pos + w > k0) {
        const uint32_t seg = atomicAdd(&s_nseg, 1u);
        s_seg_base[seg] = (uint32_t)(ty * gx + ta) - pos;
        s_seg_gid[seg] = gid;
        const uint32_t at = (pos > k0 ? pos : k0) - k0;
        s_own[own_idx(at)] = ((at + 1) << 16) | seg;
      }
      pos += w;
    }
  }
  lds_barrier();
  // inclusive max-scan of the marks over the block's slots (consecutive DUP_ITEMS per thread)
  uint32_t v[DUP_ITEMS];
  uint32_t run = 0;
#pragma unroll
  for (int r = 0; r < DUP_ITEMS; r++) {
    run = max(run, s_own[own_idx(tid * DUP_ITEMS + r)]);
    v[r] = run;
  }
  uint32_t incl = run;
  const uint32_t lane = tid & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)incl, d, 64);
    if (lane >= (uint32_t)d) incl = max(incl, o);
  }
  if (lane == 63) s_wmax[tid >> 6] = incl;
  uint32_t excl = (uint32_t)__shfl_up((int)incl, 1, 64);
  if (lane == 0) excl = 0;
  lds_barrier();
  for (uint32_t w = 0; w < (tid >> 6); w++) excl = max(excl, s_wmax[w]);
#pragma unroll
  for (int r = 0; r < DUP_ITEMS; r++) s_own[own_idx(tid * DUP_ITEMS + r)] = max(v[r], excl);
  lds_barrier();
#pragma unroll
  for (int r = 0; r < DUP_ITEMS; r++) {
    const uint32_t i = (uint32_t)r * DUP_THREADS + tid;
    const uint32_t k = k0 + i;
    if (k < k1) {
      const uint32_t o = s_own[own_idx(i)] & 0xFFFFu;
      const uint32_t key = s_seg_base[o] + k;
      tile_keys[k] = key;
      presort_gid[k] = s_seg_gid[o];
      if (hist0) atomicAdd(&s_hist[key & mask0], 1u);  // counts only: order-free
    }
  }
  // the tile sort's first-pass digit counts of this block's slots (its sort tile is the same 2048
  // slots): the sort skips that pass's counting launch
  if (hist0) {
    lds_barrier();
    hist0[(size_t)tid * gridDim.x + b] = s_hist[tid];
  }
}

// tile ranges over the sorted instance list, 4 instances per lane
__global__ __launch_bounds__(256) void k_ranges(uint32_t I, const uint32_t* __restrict__ n_dev,
                                                const uint32_t* __restrict__ tile, uint2* __restrict__ ranges,
                                                uint32_t* __restrict__ sched, uint32_t n_sched, uint32_t tiles,
                                                uint64_t bs, uint64_t is) {
  n_dev = vptr(n_dev, bs), tile = vptr(tile, bs), ranges = vptr(ranges, is), sched = vptr(sched, is);
  // clear the render's per-tile completion words and the backward queue (k_render_fwd_q epilogue)
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n_sched; i += gridDim.x * 256) sched[i] = 0u;
  I = min(I, *n_dev);  // the capacity I, or the count when below it
  const uint32_t k0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (k0 >= I) return;
  uint32_t t[6];
  t[0] = k0 > 0 ? tile[k0 - 1] : 0xFFFFFFFFu;
  if (k0 + 4 <= I && (k0 & 3) == 0) {
    const uint4 q = *reinterpret_cast<const uint4*>(tile + k0);
    t[1] = q.x;
    t[2] = q.y;
    t[3] = q.z;
    t[4] = q.w;
  } else {
#pragma unroll
    for (int r = 0; r < 4; r++) t[1 + r] = k0 + r < I ? tile[k0 + r] : 0xFFFFFFFFu;
  }
  t[5] = k0 + 4 < I ? tile[k0 + 4] : 0xFFFFFFFFu;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t k = k0 + r;
    if (k >= I) break;
    if (t[r + 1] >= tiles) continue;  // only after a timed-out sort (reported): stay in bounds
    if (t[r + 1] != t[r]) ranges[t[r + 1]].x = k;
    if (t[r + 2] != t[r + 1]) ranges[t[r + 1]].y = k + 1;
  }
}

void fwd_bin(int P, uint32_t I, const CameraArgs& c, const int* radii, const GeomPtrs& geo, const BinPtrs& bin,
             const ImgPtrs& img, hipStream_t st) {
  (void)radii;
  fwd_bin_views(1, P, I, c, geo, bin, img, 0, 0, 0, st);
}

void fwd_bin_views(int views, int P, uint32_t I, const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin,
                   const ImgPtrs& img, uint64_t gs, uint64_t bs, uint64_t is, hipStream_t st) {
  const int tiles = c.gx * c.gy;
  const uint32_t sched_n = sched_words((uint32_t)tiles);
  if (I == 0 || !dup_balanced(I, (uint32_t)P)) {
    // no instances (capacity 0), or more than DUP_SLOTS per Gaussian on average: view by view
    for (int v = 0; v < views; v++) {
      GeomPtrs g;
      BinPtrs bb;
      ImgPtrs im;
      geom_layout((size_t)P, &g, (char*)geo.splat + (uint64_t)v * gs);
      bin_layout((size_t)I, tiles, &bb, (char*)bin.keys_a + (uint64_t)v * bs);
      img_layout(c.W, c.H, &im, (char*)img.ranges + (uint64_t)v * is);
      if (I == 0) {
        (void)hipMemsetAsync(im.ranges, 0, sizeof(uint2) * (size_t)tiles, st);
        (void)hipMemsetAsync(im.tile_done, 0, sizeof(uint32_t) * sched_n, st);
        continue;
      }
      (void)hipMemsetAsync(im.ranges, 0, sizeof(uint2) * (size_t)tiles, st);
      GS_LAUNCH("duplicate", k_duplicate, dim3((P + 255) / 256), dim3(256), 0, st, (uint32_t)P, g.counters,
                g.sorted_gid, g.offsets, g.binrec, c.gx, bb.slot_tile, bb.presort_gid);
      radix_sort_pairs(bb.keys_a, bb.vals_a, bb.keys_b, bb.vals_b, true, &g.counters[CNT_NREND], I, tile_bits(tiles),
                       bb.sort_scratch, st, false, false, nullptr, nullptr, nullptr, bb.slot_tile,
                       GS_TILE_SORT_BLOCKS);
      GS_LAUNCH("ranges", k_ranges, dim3((I + 1023) / 1024), dim3(256), 0, st, I, &g.counters[CNT_NREND],
                bb.sorted_tile, im.ranges, (uint32_t*)im.tile_done, sched_n, (uint32_t)tiles, 0ull, 0ull);
    }
    return;
  }
  const int tbits = tile_bits(tiles);
  // one duplicate block per sort tile: the duplicate also counts the first sort pass's digits; it
  // copies each view's bounded count into its binning buffer (bin.count) for the sort and ranges
  const bool hist0 = sort_plan(I, GS_TILE_SORT_BLOCKS).chunk == DUP_SLOTS;
  GS_LAUNCH("duplicate", k_duplicate_lb, dim3((I + DUP_SLOTS - 1) / DUP_SLOTS, views), dim3(DUP_THREADS), 0, st, I,
            geo.counters, geo.dup_first, geo.sorted_gid, geo.offsets, geo.binrec, c.gx, c.gy, bin.slot_tile,
            bin.presort_gid, img.ranges, hist0 ? bin.sort_scratch : nullptr, (1u << radix_first_bits(tbits)) - 1u,
            bin.count, gs, bs, is);
  // the device count bounds the sort (I is the buffers' capacity, which may exceed it)
  radix_sort_pairs(bin.keys_a, bin.vals_a, bin.keys_b, bin.vals_b, true, bin.count, I, tbits, bin.sort_scratch, st,
                   false, hist0, nullptr, nullptr, nullptr, bin.slot_tile,
                   GS_TILE_SORT_BLOCKS, views, bs);
  GS_LAUNCH("ranges", k_ranges, dim3((I + 1023) / 1024, views), dim3(256), 0, st, I, bin.count, bin.sorted_tile,
            img.ranges, (uint32_t*)img.tile_done, sched_n, (uint32_t)tiles, bs, is);
}

// ------------------------------------------------------------------------------------------
// render forward
// ------------------------------------------------------------------------------------------
// Entries are staged as three 16-B LDS records at one byte offset o (o, o + 16 NB, o + 32 NB for
// a batch of NB entries):
//   (x, y, r, g) | falloff coefficients + opacity | (b, bits(entry index + 1), -, -)
// and each quadrant wave's dense list holds the offsets (u32), read FWD_ILP = 4 at a time with one
// 16-B LDS read: a list entry costs no address arithmetic, no unpacking and no dependent list read.
// (8 entries per trip: 60 -> 74 VGPRs, 8 -> 6 waves per SIMD, render_fwd 174 -> 189 us)
constexpr int FWD_ILP = 4;  // a multiple of 4 (whole 16-B list reads)
static_assert(FWD_ILP % 4 == 0, "list groups are read 16 B at a time");

struct FwdPix {
  float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
  uint32_t last = 0;
  uint64_t done;  // lane mask (wave-uniform): pixels that stopped or lie outside the image
};

// Walk one quadrant wave's list of qcnt staged entries for the lane's pixel.  The list is padded
// with 2 FWD_ILP offsets of a staged dummy entry of opacity 0 (alpha 0 at every pixel), so the walk
// needs no per-entry end-of-list test (175.8 -> 172.6 us at C3).
template <bool EXACT, int NB>
__device__ __forceinline__ void fwd_walk(const char* ent, const uint32_t* qlist, uint32_t qcnt, float pfx, float pfy,
                                         FwdPix& px) {
  // FWD_ILP entries per trip: their power / exp / alpha chains are independent (ILP); the
  // compositing is then applied entry by entry in list order, exactly as one at a time.  The
  // next group's offsets are read one trip ahead (one dependent LDS round trip per trip).
  constexpr int NQ = FWD_ILP / 4;
  uint4 wn[NQ];
#pragma unroll
  for (int r = 0; r < NQ; r++) wn[r] = *reinterpret_cast<const uint4*>(&qlist[4 * r]);
  for (uint32_t k = 0; k < qcnt; k += FWD_ILP) {
    uint32_t o[FWD_ILP];
#pragma unroll
    for (int r = 0; r < NQ; r++) {
      o[4 * r] = wn[r].x, o[4 * r + 1] = wn[r].y, o[4 * r + 2] = wn[r].z, o[4 * r + 3] = wn[r].w;
      wn[r] = *reinterpret_cast<const uint4*>(&qlist[k + FWD_ILP + 4 * r]);
    }
    float pw[FWD_ILP], al[FWD_ILP];
#pragma unroll
    for (int u = 0; u < FWD_ILP; u++) {
      const float4 xr = *reinterpret_cast<const float4*>(ent + o[u]);
      const float4 co = *reinterpret_cast<const float4*>(ent + o[u] + 16 * NB);
      pw[u] = falloff_log2_m<EXACT>(co, xr.x - pfx, xr.y - pfy);  // log2(e) * power (fast: + log2 o)
      al[u] = fminf(0.99f, opac_gauss<EXACT>(co, pw[u]));
    }
#pragma unroll
    for (int u = 0; u < FWD_ILP; u++) {
      const float4 xr = *reinterpret_cast<const float4*>(ent + o[u]);
      const float2 bl = *reinterpret_cast<const float2*>(ent + o[u] + 32 * NB);
      const float rr = xr.z, rg = xr.w, rb = bl.x;
      // branch-free compositing (selects instead of divergent ifs); the per-entry decisions are
      // lane masks combined on the scalar unit (ballot / inverse ballot), so the VALU does the
      // two threshold compares and the selects only.
      // upstream skips power > 0; with a positive-definite conic that only happens by rounding
      // within ~1e-3 px of a splat centre, so the fast mode leaves the test out (the backward
      // matches it entry for entry)
      const uint64_t m_a = __builtin_amdgcn_ballot_w64((!EXACT || pw[u] <= 0.0f) && al[u] >= 1.0f / 255.0f);
      uint64_t m_cu = m_a & ~px.done;
      if constexpr (EXACT) {  // upstream's order, T (1 - alpha) and (rgb alpha) T, mirrored by the oracle
        const float tT = px.T * (1.0f - al[u]);
        // T would drop below 1e-4: stop before this entry
        const uint64_t m_stop = m_cu & __builtin_amdgcn_ballot_w64(tT < 0.0001f);
        px.done |= m_stop;
        m_cu &= ~m_stop;
        const bool cu = __builtin_amdgcn_inverse_ballot_w64(m_cu);
        px.C0 = cu ? px.C0 + rr * al[u] * px.T : px.C0;
        px.C1 = cu ? px.C1 + rg * al[u] * px.T : px.C1;
        px.C2 = cu ? px.C2 + rb * al[u] * px.T : px.C2;
        px.T = cu ? tT : px.T;
        px.last = cu ? __float_as_uint(bl.y) : px.last;
      } else {
        // T - alpha T as one FMA (one rounding of T (1 - alpha)); one weight, three FMAs (a
        // skipped entry adds rgb * 0)
        const float tT = __builtin_fmaf(-al[u], px.T, px.T);
        const uint64_t m_keep = __builtin_amdgcn_ballot_w64(tT >= 0.0001f);
        px.done |= m_cu & ~m_keep;
        m_cu &= m_keep;
        const bool cu = __builtin_amdgcn_inverse_ballot_w64(m_cu);
        const float wgt = cu ? al[u] * px.T : 0.0f;
        px.C0 = __builtin_fmaf(rr, wgt, px.C0);
        px.C1 = __builtin_fmaf(rg, wgt, px.C1);
        px.C2 = __builtin_fmaf(rb, wgt, px.C2);
        px.T = cu ? tT : px.T;
        px.last = cu ? __float_as_uint(bl.y) : px.last;
      }
    }
    if (px.done == ~0ull) break;
  }
}

#ifdef GS_TIMING
// diagnostic build only: per quadrant wave b (blockIdx.x): tile << 32 | quadrant, batches staged <<
// 32 | entries walked (tools/fwd_timing.py)
GS_TIMING_BUFFER(g_fwd_timing, gs_debug_fwd_timing)
#endif

// Epilogue of one quadrant wave (one lane): one 64-bit atomic per wave adds 1 (finished waves, low
// 3 bits) plus a one-hot bit of the quadrant's walk-length class (bit 8 + class).  The tile's
// fourth finisher gets the other three from the returned value, with no fence: the highest set
// bit of the sum is the tile's longest class (or one above it, when classes coincide and carry),
// which is all the longest-first order needs.  It takes a rank in that bucket; k_tile_order turns
// (bucket, rank) into the backward's launch order.
__device__ __forceinline__ void tile_finish(uint32_t tile, uint32_t grp, uint32_t wave_last,
                                            uint64_t* __restrict__ tile_done, uint32_t* __restrict__ len_hist,
                                            uint32_t* __restrict__ tile_brank) {
  // length classes on a log scale, four per octave
  const uint32_t cls = min((uint32_t)(4.0f * __log2f((float)wave_last + 1.0f)), 47u);
  const uint64_t mine = (1ull << (8 + cls)) + 1ull;
  const uint64_t old = atomicAdd((unsigned long long*)&tile_done[tile], (unsigned long long)mine);
  if ((old & 7ull) != 3ull) return;
  const uint32_t top = 63u - (uint32_t)__builtin_clzll((old + mine) >> 8);  // 0 .. 49
  const uint32_t b = (uint32_t)ORDER_BUCKETS - 1u - top;                    // descending length
  tile_brank[tile] = b << 22 | atomicAdd(&len_hist[grp * ORDER_BUCKETS + b], 1u);
}

__device__ __forceinline__ void fwd_store(const CameraArgs& c, const QuadPix& q, bool inside, const FwdPix& px,
                                          float* __restrict__ out, float* __restrict__ final_T,
                                          uint32_t* __restrict__ n_contrib) {
  if (inside) {
    const size_t pix = (size_t)q.py * c.W + q.px, HW = (size_t)c.W * c.H;
    final_T[pix] = px.T;
    n_contrib[pix] = px.last;
    out[pix] = px.C0 + px.T * c.bg[0];
    out[HW + pix] = px.C1 + px.T * c.bg[1];
    out[2 * HW + pix] = px.C2 + px.T * c.bg[2];
  }
}

// One wave per (tile, quadrant), no workgroup barriers: each wave stages the tile's entries 64 at
// a time, culls them to its own quadrant and walks them, and finishes as soon as its 64 pixels
// are done (a workgroup per tile would wait for its slowest quadrant: 203 -> 188 us at C3 when this
// went in).  Workgroup b takes the (b / 32)-th tile of XCD group b % 8 (xcd_tile), quadrant
// (b / 8) % 4, so the four quadrant waves of a tile share the workgroup-to-XCD round robin (b % 8)
// and their repeated entry loads hit one L2.
// (Tried and not kept: the next batch's ids / records prefetched one batch ahead, 168 -> 179 us --
// the loads past the stop are wasted; 32-entry batches, 174 -> 195 us.)
constexpr int FWDQ_NB = 64;  // entries staged per round (one per lane)
// record stride of the staged batch: one more than the batch for the padding's dummy entry
constexpr int FWDQ_NBS = FWDQ_NB + 1;
template <bool EXACT>
__global__ __launch_bounds__(64) void k_render_fwd_q(CameraArgs c, const uint2* __restrict__ ranges,
                                                     const uint32_t* __restrict__ point_list,
                                                     const uint32_t* __restrict__ point_gid,
                                                     const float4* __restrict__ splat, float* __restrict__ out,
                                                     ImgPtrs img, const uint32_t* __restrict__ err,
                                                     uint32_t* __restrict__ err_host) {
  __shared__ float4 s_ent[3 * FWDQ_NBS];
  __shared__ __attribute__((aligned(16))) uint32_t s_qlist[FWDQ_NB + 2 * FWD_ILP];
  if (threadIdx.x < 3)  // the dummy entry: position 0, opacity 0 (never contributes; fast: log2 0 = -inf)
    s_ent[threadIdx.x * FWDQ_NBS + FWDQ_NB] =
        make_float4(0.0f, 0.0f, 0.0f, (EXACT || threadIdx.x != 1) ? 0.0f : -__builtin_inff());
  const uint32_t b = blockIdx.x;
  const uint32_t tile = xcd_tile(b & 7, b >> 5, c.gx, c.gy);
  if (tile == ~0u) return;  // (grid padded to whole groups of 8 tiles)
#ifdef GS_TIMING
  const unsigned long long t_start = timing_stamp();
  uint32_t t_batches = 0, t_walked = 0;
#endif
  const int wid = (int)((b >> 3) & 3);
  const int tx = (int)(tile % (uint32_t)c.gx), ty = (int)(tile / (uint32_t)c.gx);
  const int lane = threadIdx.x;
  // the ordering's error flags (final once the binning kernels are done) -> the host's readback word
  if (b == 0 && lane == 0 && err_host && *err) err_host[0] = *err;
  const QuadPix q = quad_pixel(tx, ty, wid, lane);
  const bool inside = q.px < c.W && q.py < c.H;
  const uint2 range = ranges[tile];
  // a sort / scan look-back that timed out (reported by the host) leaves no valid list: render none
  const uint32_t n = (*err & ERR_INVALID) ? 0u : range.y - range.x;
  const char* ent = reinterpret_cast<const char*>(s_ent);
  const float qx = (float)(tx * GS_TILE + 8 * (wid & 1)), qy = (float)(ty * GS_TILE + 8 * (wid >> 1));
  FwdPix px;
  px.done = __builtin_amdgcn_ballot_w64(!inside);
  for (uint32_t base = 0; base < n; base += FWDQ_NB) {
    if (px.done == ~0ull) break;
    bool meets = false;
    if (lane < (uint32_t)FWDQ_NB && base + lane < n) {
      const uint32_t gid = point_gid[point_list[range.x + base + lane]];
      const float4 a = splat[3 * gid], bb = splat[3 * gid + 1], d = splat[3 * gid + 2];
      s_ent[lane] = make_float4(a.x, a.y, bb.z, bb.w);
      s_ent[FWDQ_NBS + lane] = fall_coefs_m<EXACT>(a.z, a.w, bb.x, bb.y);
      s_ent[2 * FWDQ_NBS + lane] = make_float4(d.x, __uint_as_float(base + lane + 1), 0.0f, 0.0f);
      meets = d.z >= 0.0f && ellipse_meets_rect(a.x, a.y, a.z, a.w, bb.x, d.z, qx, qx + 7.0f, qy, qy + 7.0f);
    }
    const uint64_t m = __ballot(meets);
    if (meets)
      s_qlist[__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
          16u * lane;
    const uint32_t qcnt = (uint32_t)__popcll(m);
    if (lane < 2 * FWD_ILP) s_qlist[qcnt + lane] = 16u * FWDQ_NB;
    __builtin_amdgcn_wave_barrier();
#ifdef GS_TIMING
    t_batches++;
    t_walked += qcnt;
#endif
    fwd_walk<EXACT, FWDQ_NBS>(ent, s_qlist, qcnt, (float)q.px, (float)q.py, px);
    __builtin_amdgcn_wave_barrier();  // the next round overwrites the staged entries
  }
  fwd_store(c, q, inside, px, out, img.final_T, img.n_contrib);
  const uint32_t wmax = wave_max_u32(px.last);
  if (lane == 0) {
    img.tile_max[4 * tile + wid] = wmax;
    tile_finish(tile, tile % ORDER_GROUPS, wmax, img.tile_done, img.len_hist, img.tile_brank);
  }
#ifdef GS_TIMING
  timing_record(g_fwd_timing, t_start, tile, (uint32_t)wid | n << 2, t_batches, t_walked);
#endif
}

void fwd_render(const CameraArgs& c, const GeomPtrs& geo, const BinPtrs& bin, const ImgPtrs& img, float* out_color,
                hipStream_t st, uint32_t* err_host) {
  const int tiles = c.gx * c.gy;
  const int blocks = (int)xcd_span((uint32_t)tiles) * 32;
  if (exact_exp())
    GS_LAUNCH("render_fwd", k_render_fwd_q<true>, dim3(blocks), dim3(64), 0, st, c, img.ranges, bin.point_list,
              bin.presort_gid, geo.splat, out_color, img, &geo.counters[CNT_ERR], err_host);
  else
    GS_LAUNCH("render_fwd", k_render_fwd_q<false>, dim3(blocks), dim3(64), 0, st, c, img.ranges, bin.point_list,
              bin.presort_gid, geo.splat, out_color, img, &geo.counters[CNT_ERR], err_host);
}

// ------------------------------------------------------------------------------------------
// mark_visible (upstream checkFrustum: near-plane test, prefiltered = false)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means,
                                                      const float* __restrict__ view, uint8_t* __restrict__ present) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const float3v pv = xf43(view, means[3 * i], means[3 * i + 1], means[3 * i + 2]);
  present[i] = !(pv.z <= 0.2f);
}

void mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present,
                  hipStream_t st) {
  (void)proj;
  if (P <= 0) return;
  GS_LAUNCH("mark_visible", k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, st, P, means3D, view, present);
}

}  // namespace gs
