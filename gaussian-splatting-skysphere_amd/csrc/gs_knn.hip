// gs_knn.hip -- simple-knn distCUDA2 for gfx950: mean squared distance of every point to its
// 3 nearest other points (/root/reference/scene/gaussian_model.py:134-135 uses it once to
// initialise scales; upstream: gitlab.inria.fr/bkerbl/simple-knn, un-vendored, .gitmodules:1-3).
//
// Exact search: points are Morton-sorted (hand-written radix sort), grouped into boxes of 32
// consecutive points and super-boxes of 1024, each with an AABB.  A lane per point seeds its
// 3-best from its Morton neighbours, then visits super-boxes / boxes / points whose AABB distance
// is below the current 3rd-best distance.
#include <float.h>

#include "gs_internal.h"

namespace gs {

constexpr int KNN_BOX = 32;
constexpr int KNN_SUPER = 1024;

__device__ __forceinline__ int f2ord(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

__global__ void k_knn_init(int* bb) {
  if (threadIdx.x < 3) bb[threadIdx.x] = INT_MAX;
  else if (threadIdx.x < 6) bb[threadIdx.x] = INT_MIN;
}

__global__ __launch_bounds__(256) void k_knn_bbox(int P, const float* __restrict__ pts, int* __restrict__ bb) {
  __shared__ int smin[3][256], smax[3][256];
  int mn[3] = {INT_MAX, INT_MAX, INT_MAX}, mx[3] = {INT_MIN, INT_MIN, INT_MIN};
  for (int i = blockIdx.x * 256 + threadIdx.x; i < P; i += gridDim.x * 256)
    for (int k = 0; k < 3; k++) {
      int v = f2ord(pts[3 * i + k]);
      mn[k] = min(mn[k], v);
      mx[k] = max(mx[k], v);
    }
  for (int k = 0; k < 3; k++) {
    smin[k][threadIdx.x] = mn[k];
    smax[k][threadIdx.x] = mx[k];
  }
  lds_barrier();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int k = 0; k < 3; k++) {
        smin[k][threadIdx.x] = min(smin[k][threadIdx.x], smin[k][threadIdx.x + s]);
        smax[k][threadIdx.x] = max(smax[k][threadIdx.x], smax[k][threadIdx.x + s]);
      }
    lds_barrier();
  }
  if (threadIdx.x == 0)
    for (int k = 0; k < 3; k++) {
      atomicMin(&bb[k], smin[k][0]);
      atomicMax(&bb[3 + k], smax[k][0]);
    }
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__global__ __launch_bounds__(256) void k_knn_morton(int P, const float* __restrict__ pts, const int* __restrict__ bb,
                                                    uint32_t* __restrict__ code) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  uint32_t q[3];
  for (int k = 0; k < 3; k++) {
    float lo = ord2f(bb[k]), hi = ord2f(bb[3 + k]);
    float ext = hi - lo;
    float t = ext > 0.f ? (pts[3 * i + k] - lo) / ext : 0.f;
    int v = (int)(t * 1023.0f);
    q[k] = (uint32_t)min(1023, max(0, v));
  }
  code[i] = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
}

// AABB of each group of `group` consecutive sorted points: 6 floats (min xyz, max xyz)
__global__ __launch_bounds__(256) void k_knn_boxes(int P, int group, const float* __restrict__ pts,
                                                   const uint32_t* __restrict__ order, float* __restrict__ boxes) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  const int nb = (P + group - 1) / group;
  if (b >= nb) return;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  const int e = min(P, (b + 1) * group);
  for (int s = b * group; s < e; s++) {
    const uint32_t i = order[s];
    for (int k = 0; k < 3; k++) {
      mn[k] = fminf(mn[k], pts[3 * i + k]);
      mx[k] = fmaxf(mx[k], pts[3 * i + k]);
    }
  }
  for (int k = 0; k < 3; k++) {
    boxes[6 * b + k] = mn[k];
    boxes[6 * b + 3 + k] = mx[k];
  }
}

__device__ __forceinline__ float box_dist2(const float* bx, float x, float y, float z) {
  float dx = fmaxf(fmaxf(bx[0] - x, x - bx[3]), 0.f);
  float dy = fmaxf(fmaxf(bx[1] - y, y - bx[4]), 0.f);
  float dz = fmaxf(fmaxf(bx[2] - z, z - bx[5]), 0.f);
  return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ void upd3(float d, float* b) {
  if (d < b[2]) {
    if (d < b[1]) {
      b[2] = b[1];
      if (d < b[0]) {
        b[1] = b[0];
        b[0] = d;
      } else
        b[1] = d;
    } else
      b[2] = d;
  }
}

__global__ __launch_bounds__(256) void k_knn_search(int P, const float* __restrict__ pts,
                                                    const uint32_t* __restrict__ order,
                                                    const float* __restrict__ boxes, const float* __restrict__ sboxes,
                                                    float* __restrict__ out) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= P) return;
  const uint32_t i = order[s];
  const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
  float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
  auto visit = [&](int t) {
    const uint32_t j = order[t];
    const float dx = pts[3 * j] - x, dy = pts[3 * j + 1] - y, dz = pts[3 * j + 2] - z;
    upd3(dx * dx + dy * dy + dz * dz, best);
  };
  for (int t = max(0, s - 4); t < min(P, s + 5); t++)
    if (t != s) visit(t);
  const int nsb = (P + KNN_SUPER - 1) / KNN_SUPER;
  for (int sb = 0; sb < nsb; sb++) {
    if (box_dist2(sboxes + 6 * sb, x, y, z) >= best[2]) continue;
    const int b0 = sb * (KNN_SUPER / KNN_BOX), b1 = min((P + KNN_BOX - 1) / KNN_BOX, b0 + KNN_SUPER / KNN_BOX);
    for (int b = b0; b < b1; b++) {
      if (box_dist2(boxes + 6 * b, x, y, z) >= best[2]) continue;
      const int e = min(P, (b + 1) * KNN_BOX);
      for (int t = b * KNN_BOX; t < e; t++) {
        if (t == s || (t >= s - 4 && t <= s + 4)) continue;
        visit(t);
      }
    }
  }
  out[i] = (best[0] + best[1] + best[2]) / 3.0f;
}

struct KnnPtrs {
  uint32_t *keys_a, *vals_a, *keys_b, *vals_b, *sort_scratch;
  int* bb;
  float *boxes, *sboxes;
};

static size_t knn_layout(size_t P, KnnPtrs* o, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t x = off;
    off += align_up(bytes);
    return x;
  };
  size_t Pn = P ? P : 1;
  size_t a = take(Pn * 4), b = take(Pn * 4), c = take(Pn * 4), d = take(Pn * 4);
  size_t e = take(sort_scratch_words(Pn) * 4);
  size_t f = take(64);
  size_t g = take(((Pn + KNN_BOX - 1) / KNN_BOX) * 24);
  size_t h = take(((Pn + KNN_SUPER - 1) / KNN_SUPER) * 24);
  if (o && base) {
    o->keys_a = (uint32_t*)(base + a);
    o->vals_a = (uint32_t*)(base + b);
    o->keys_b = (uint32_t*)(base + c);
    o->vals_b = (uint32_t*)(base + d);
    o->sort_scratch = (uint32_t*)(base + e);
    o->bb = (int*)(base + f);
    o->boxes = (float*)(base + g);
    o->sboxes = (float*)(base + h);
  }
  return off;
}

size_t knn_scratch_bytes(int P) { return knn_layout((size_t)(P > 0 ? P : 1), nullptr, nullptr); }

void knn_mean_dist2(int P, const float* pts, float* out, char* scratch, hipStream_t st) {
  KnnPtrs k;
  knn_layout((size_t)P, &k, scratch);
  GS_LAUNCH("knn_init", k_knn_init, dim3(1), dim3(64), 0, st, k.bb);
  const int blocks = min(1024, (P + 255) / 256);
  GS_LAUNCH("knn_bbox", k_knn_bbox, dim3(blocks), dim3(256), 0, st, P, pts, k.bb);
  GS_LAUNCH("knn_morton", k_knn_morton, dim3((P + 255) / 256), dim3(256), 0, st, P, pts, k.bb, k.keys_a);
  const bool in_b = radix_sort_pairs(k.keys_a, k.vals_a, k.keys_b, k.vals_b, true, nullptr, (uint32_t)P, 30,
                                     k.sort_scratch, st);
  const uint32_t* order = in_b ? k.vals_b : k.vals_a;
  const int nbox = (P + KNN_BOX - 1) / KNN_BOX, nsb = (P + KNN_SUPER - 1) / KNN_SUPER;
  GS_LAUNCH("knn_boxes", k_knn_boxes, dim3((nbox + 255) / 256), dim3(256), 0, st, P, KNN_BOX, pts, order, k.boxes);
  GS_LAUNCH("knn_boxes", k_knn_boxes, dim3((nsb + 255) / 256), dim3(256), 0, st, P, KNN_SUPER, pts, order, k.sboxes);
  GS_LAUNCH("knn_search", k_knn_search, dim3((P + 255) / 256), dim3(256), 0, st, P, pts, order, k.boxes, k.sboxes,
            out);
}

}  // namespace gs
