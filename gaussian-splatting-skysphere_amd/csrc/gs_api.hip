#include <dlfcn.h>

#include <atomic>
#include <cstdlib>
// gs_api.hip -- C ABI (include/gsrast.h): argument validation, buffer layout, stage orchestration,
// error capture, debug synchronisation and per-kernel HIP-event timing.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/gsrast.h"
#include "gs_internal.h"

namespace gs {

// ------------------------------------------------------------------------------------------
// error / debug / timing state
// ------------------------------------------------------------------------------------------
static thread_local std::string t_err;
static thread_local bool t_failed = false;
static thread_local bool t_debug = false;

static void set_error(const char* fmt, ...) {
  if (t_failed) return;  // keep the first error
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  t_failed = true;
}
static void clear_error(int debug) {
  t_err.clear();
  t_failed = false;
  t_debug = debug != 0;
}

struct ProfEntry {
  std::string name;
  double ms;
  long long n;
};
struct Pending {
  const char* name;
  hipEvent_t a, b;
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::vector<Pending> g_pending;
static std::vector<hipEvent_t> g_pool;
static std::vector<ProfEntry> g_stats;

static hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void trace_begin(const char* name, hipStream_t st) {
  if (!g_prof_on) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  hipEvent_t a = get_event();
  (void)hipEventRecord(a, st);
  g_pending.push_back(Pending{name, a, nullptr});
}

void trace_end(const char* name, hipStream_t st) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) set_error("kernel %s launch failed: %s", name, hipGetErrorString(e));
  if (g_prof_on) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    hipEvent_t b = get_event();
    (void)hipEventRecord(b, st);
    if (!g_pending.empty() && g_pending.back().b == nullptr) g_pending.back().b = b;
  }
  if (t_debug) {
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) set_error("kernel %s failed: %s", name, hipGetErrorString(e));
  }
}

static std::atomic<int> g_launch_log{-1};  // -1: not yet read from GSRAST_LAUNCH_LOG
static std::mutex g_launch_mu;
static std::vector<const void*> g_launched;

static int launch_log_on() {
  int v = g_launch_log.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("GSRAST_LAUNCH_LOG");
    v = (e && atoi(e) != 0) ? 1 : 0;
    g_launch_log.store(v, std::memory_order_relaxed);
  }
  return v;
}

void launch_record(const void* k) {
  if (!launch_log_on()) return;
  std::lock_guard<std::mutex> lk(g_launch_mu);
  for (const void* x : g_launched)
    if (x == k) return;
  g_launched.push_back(k);
}

void host_error(const char* msg) { set_error("%s", msg); }

static bool check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) set_error("%s failed: %s", what, hipGetErrorString(e));
  return e == hipSuccess;
}

static CameraArgs make_camera(const float* bg, int W, int H, const float* view, const float* proj, const float* campos,
                              float tanfovx, float tanfovy, int prefiltered) {
  CameraArgs c;
  c.view = view;
  c.proj = proj;
  c.campos = campos;
  c.bg = bg;
  c.tanfovx = tanfovx;
  c.tanfovy = tanfovy;
  c.fy = (float)H / (2.0f * tanfovy);
  c.fx = (float)W / (2.0f * tanfovx);
  c.W = W;
  c.H = H;
  c.gx = (W + GS_TILE - 1) / GS_TILE;
  c.gy = (H + GS_TILE - 1) / GS_TILE;
  c.prefiltered = prefiltered;
  return c;
}

static bool validate(int P, int D, int M, int W, int H, const float* means3D, const float* shs, const float* colors,
                     const float* opac, const float* scales, const float* rots, const float* cov3D, const float* view,
                     const float* proj, const float* campos, const float* bg, bool need_opac = true) {
  if (P < 0) return set_error("P must be >= 0"), false;
  if (W <= 0 || H <= 0) return set_error("image size must be positive (got %d x %d)", W, H), false;
  if (P == 0) return true;
  if (!means3D || (need_opac && !opac) || !view || !proj || !bg)
    return set_error("missing required input pointer"), false;
  if ((shs == nullptr) == (colors == nullptr))
    return set_error("Please provide excatly one of either SHs or precomputed colors!"), false;
  if (((scales == nullptr || rots == nullptr) && cov3D == nullptr) || ((scales || rots) && cov3D))
    return set_error("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!"), false;
  if (shs) {
    if (D < 0 || D > 3) return set_error("SH degree must be in [0, 3] (got %d)", D), false;
    if (M < (D + 1) * (D + 1)) return set_error("shs has %d coefficients, degree %d needs %d", M, D, (D + 1) * (D + 1)), false;
    if (!campos) return set_error("campos is required with SHs"), false;
  }
  if ((size_t)P * 48 > ((size_t)1 << 40)) return set_error("P too large"), false;
  return true;
}

// ------------------------------------------------------------------------------------------
// debug export kernel
// ------------------------------------------------------------------------------------------
// entries past the list's device count (past a bounded buffer's capacity) are not written by the
// forward: exported as ~0 (no gather through them)
__global__ void k_export_list(uint32_t I, const uint32_t* counters, const uint32_t* point_list, const uint32_t* ids,
                              uint32_t* out) {
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  if (k >= I) return;
  const uint32_t n = min(I, counters[CNT_I]);
  if (k >= n) {
    out[k] = 0xFFFFFFFFu;
    return;
  }
  const uint32_t s = point_list[k];
  out[k] = s < I ? ids[s] : 0xFFFFFFFFu;
}
__global__ void k_export_splat(int P, const float4* splat, float* xy, float* co, float* rgb, float* depth) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const float4 a = splat[3 * i], b = splat[3 * i + 1], d = splat[3 * i + 2];
  if (xy) {
    xy[2 * i] = a.x;
    xy[2 * i + 1] = a.y;
  }
  if (co) {
    co[4 * i] = a.z;
    co[4 * i + 1] = a.w;
    co[4 * i + 2] = b.x;
    co[4 * i + 3] = b.y;
  }
  if (rgb) {
    rgb[3 * i] = b.z;
    rgb[3 * i + 1] = b.w;
    rgb[3 * i + 2] = d.x;
  }
  if (depth) depth[i] = d.y;
}

}  // namespace gs

using namespace gs;

namespace gs {
static std::atomic<int> g_exact_exp{-1};  // -1: not yet read from GSRAST_EXACT_EXP
bool exact_exp() {
  int v = g_exact_exp.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("GSRAST_EXACT_EXP");
    v = (e && e[0] && e[0] != '0') ? 1 : 0;
    g_exact_exp.store(v, std::memory_order_relaxed);
  }
  return v != 0;
}
}  // namespace gs

namespace gs {
static std::atomic<uint32_t> g_spin_limit{LB_SPIN_LIMIT};
uint32_t scan_spin_limit() { return g_spin_limit.load(std::memory_order_relaxed); }

// row waits installed by gs_set_row_waits, per host thread, until the next forward preprocess
static thread_local RowWait t_row_waits[GS_MAX_ROW_WAITS];
static thread_local int t_row_wait_count = 0;
int take_row_waits(RowWait* out, int max) {
  const int n = t_row_wait_count < max ? t_row_wait_count : max;
  for (int k = 0; k < n; k++) out[k] = t_row_waits[k];
  t_row_wait_count = 0;
  return n;
}
bool stream_wait(hipStream_t st, hipEvent_t ev) {
  const hipError_t e = hipStreamWaitEvent(st, ev, 0);
  if (e != hipSuccess) set_error("row wait: hipStreamWaitEvent failed: %s", hipGetErrorString(e));
  return e == hipSuccess;
}
uint32_t next_scan_epoch() {
  static std::atomic<uint32_t> e{0};
  return (e.fetch_add(1, std::memory_order_relaxed) % ((1u << 30) - 1u)) + 1u;
}
}  // namespace gs

extern "C" {

int gs_abi_version(void) { return GSRAST_ABI_VERSION; }
const char* gs_last_error(void) { return t_err.c_str(); }

size_t gs_geom_buffer_bytes(int P) { return geom_layout((size_t)(P > 0 ? P : 1), nullptr, nullptr); }
size_t gs_binning_buffer_bytes(long long num_rendered, int W, int H) {
  int tiles = ((W + GS_TILE - 1) / GS_TILE) * ((H + GS_TILE - 1) / GS_TILE);
  return bin_layout((size_t)(num_rendered > 0 ? num_rendered : 1), tiles, nullptr, nullptr);
}
size_t gs_image_buffer_bytes(int W, int H) { return img_layout(W, H, nullptr, nullptr); }
long long gs_binning_layout_count(size_t bytes, int W, int H) {
  // every array of bin_layout has a size that never decreases with the count (sort_scratch_words
  // is a monotone bound, not sort_plan's nb), so gs_binning_buffer_bytes is non-decreasing, and two
  // counts with the same byte size have the same aligned array sizes, hence the same layout: the
  // largest count that fits `bytes` lays the buffer out exactly as the count it was sized for
  // (tests/test_abi.py checks this around the sort's block-count steps at k * 2^23 instances)
  if (gs_binning_buffer_bytes(1, W, H) > bytes) return 0;
  long long lo = 1, hi = GS_MAX_INSTANCES;
  while (lo < hi) {
    const long long mid = lo + (hi - lo + 1) / 2;
    if (gs_binning_buffer_bytes(mid, W, H) <= bytes)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}
size_t gs_grad_buffer_bytes(long long num_rendered) {
  const size_t R = (size_t)(num_rendered > 0 ? num_rendered : 1);
  return align_up(R * GRAD_REC * sizeof(float));
}

// Pinned, device-mapped host words: kernels store into them directly (vector stores through the
// device pointer), so a readback costs no copy launch.
static bool mapped_words(size_t bytes, uint32_t** host, uint32_t** dev) {
  void* p = nullptr;
  void* d = nullptr;
  if (!check_hip(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc")) return false;
  if (!check_hip(hipHostGetDevicePointer(&d, p, 0), "hipHostGetDevicePointer")) return false;
  memset(p, 0, bytes);
  *host = (uint32_t*)p;
  *dev = (uint32_t*)d;
  return true;
}

// Per-thread, per-device readback words + events (reused call after call: a call waits on its
// events before returning, so the slot is free again when the next call starts).  View v's
// totals land in words [8 v, 8 v + 4): instances low / high, V, error flags (CounterFinalize).
struct ReadbackSlot {
  uint32_t* host = nullptr;
  uint32_t* dev = nullptr;
  hipEvent_t ev[FUSED_MAX_VIEWS] = {};  // view v's totals written (the first depth-sort histogram launch)
};
static ReadbackSlot* readback_slot() {
  static thread_local ReadbackSlot slots[64];
  int dev = 0;
  if (!check_hip(hipGetDevice(&dev), "hipGetDevice")) return nullptr;
  if (dev < 0 || dev >= 64) return set_error("device ordinal out of range"), nullptr;
  ReadbackSlot& s = slots[dev];
  if (!s.host) {
    if (!mapped_words(32 * FUSED_MAX_VIEWS, &s.host, &s.dev)) return nullptr;
    for (int v = 0; v < FUSED_MAX_VIEWS; v++)
      if (!check_hip(hipEventCreateWithFlags(&s.ev[v], hipEventDisableTiming), "hipEventCreate")) return nullptr;
  }
  return &s;
}

// view v's instance count from its readback words; false (error set) for an invalid view
static bool read_view_totals(const uint32_t* w, int v, int views, long long* num_rendered) {
  const uint32_t err = w[3];
  const unsigned long long I = (unsigned long long)w[1] << 32 | w[0];
  if (err & ERR_PREFILTERED) return set_error("Point is filtered although prefiltered is set. This shouldn't happen!"), false;
  if ((err & ERR_INSTANCES) || I > (unsigned long long)GS_MAX_INSTANCES) {
    if (views > 1) return set_error("view %d has %llu (Gaussian, tile) instances, more than %lld", v, I, GS_MAX_INSTANCES), false;
    return set_error("the view has %llu (Gaussian, tile) instances, more than %lld", I, GS_MAX_INSTANCES), false;
  }
  *num_rendered = (long long)I;
  return true;
}

// Error flags of the last forwards' sorts / scans, per device (not per thread: the backward of a
// forward runs on the autograd engine's device thread).  Each gs_forward_render's render kernel
// stores them into a pinned word of a small ring, behind an event; once its own launches are
// queued, a forward checks the forwards queued before it, and the next backward or forward call
// checks this one (ERR_LOOKBACK: a look-back wait ran out), so no host wait idles the GPU.
// A forward reserves its word and its sequence number in one critical section; reusing a word
// first checks the forward that last held it, so concurrent host threads never share or drop one.
constexpr int ORDER_RING = 8;
struct OrderFlags {
  std::mutex mu;
  uint32_t* host = nullptr;  // words 16 k (k < ORDER_RING): the ordering error flags of forward seq % ORDER_RING
  uint32_t* dev = nullptr;   // device pointer of `host`
  hipEvent_t ev[ORDER_RING] = {};
  int state[ORDER_RING] = {};  // 0 free, 1 reserved (render not queued yet), 2 queued, not checked
  unsigned long long seq = 0;  // forwards that reserved a word so far
};
static OrderFlags g_order[64];

static OrderFlags* order_flags() {
  int dev = 0;
  if (!check_hip(hipGetDevice(&dev), "hipGetDevice")) return nullptr;
  if (dev < 0 || dev >= 64) return set_error("device ordinal out of range"), nullptr;
  return &g_order[dev];
}

// check ring slot k's queued forward (waits for its render kernel; with wait=false a forward whose
// render has not finished yet stays queued for a later check); true: failed (error set)
static bool check_order_slot_locked(OrderFlags& o, int k, bool wait = true) {
  if (o.state[k] != 2) return false;
  if (!wait) {
    const hipError_t q = hipEventQuery(o.ev[k]);
    if (q == hipErrorNotReady) return false;
    if (!check_hip(q, "hipEventQuery")) return true;
  }
  o.state[k] = 0;
  if (!check_hip(hipEventSynchronize(o.ev[k]), "hipEventSynchronize")) return true;
  if (o.host[16 * k] & ERR_LOOKBACK) {
    set_error("forward ordering: a look-back wait of the offsets scan or a one-sweep sort timed out "
              "(the instance list of that forward is invalid)");
    return true;
  }
  return false;
}
// every queued forward's flags.  wait=false (the backward entry points): only the forwards whose
// render kernel has finished -- a backward is queued right behind its forward's render, and waiting
// for that render here would stall the host while the device has work; a forward whose render
// has not finished is checked by the next call (at the latest the next forward, whose instance-count
// readback comes after it on the stream)
// skip: a forward (sequence number) left out, e.g. the caller's own, whose render was just queued
static bool check_order_flags(bool wait = true, long long skip = -1) {
  OrderFlags* o = order_flags();
  if (!o) return true;
  std::lock_guard<std::mutex> lk(o->mu);
  bool failed = false;
  for (int k = 0; k < ORDER_RING; k++)
    if (skip < 0 || k != (int)(skip % ORDER_RING)) failed |= check_order_slot_locked(*o, k, wait);
  return failed;
}

// forward q's flags now (waits for its render kernel), if its word still holds them; true: failed
static bool check_order_seq(unsigned long long q) {
  OrderFlags* o = order_flags();
  if (!o) return true;
  std::lock_guard<std::mutex> lk(o->mu);
  const int k = (int)(q % ORDER_RING);
  return o->seq - q <= (unsigned long long)ORDER_RING && check_order_slot_locked(*o, k);
}

// The device word this forward's render kernel stores its ordering flags into, and (*seq_out) the
// forward's sequence number; null on error.
static uint32_t* order_flags_word(unsigned long long* seq_out) {
  OrderFlags* o = order_flags();
  if (!o) return nullptr;
  std::lock_guard<std::mutex> lk(o->mu);
  if (!o->host) {
    if (!mapped_words(16 * ORDER_RING, &o->host, &o->dev)) return nullptr;
    for (int k = 0; k < ORDER_RING; k++)
      if (!check_hip(hipEventCreateWithFlags(&o->ev[k], hipEventDisableTiming), "hipEventCreate")) return nullptr;
  }
  const unsigned long long q = o->seq;
  const int k = (int)(q % ORDER_RING);
  if (o->state[k] == 1) return set_error("more than %d forwards queueing at once on one device", ORDER_RING), nullptr;
  if (check_order_slot_locked(*o, k)) return nullptr;  // the word's previous forward
  o->seq++;
  o->state[k] = 1;
  *seq_out = q;
  // the render stores nonzero flags only: clear the word
  o->host[16 * k] = 0u;
  return o->dev + 16 * k;
}
// the render kernel that stores forward `q`'s flags is queued on `st`: record its event, then
// check the forwards queued before it whose renders have finished (no wait: the views of a step
// render on two streams, and waiting here for the previous view's render stalled the host for that
// render's length in every step; the unfinished ones are checked after the next count readback)
static bool queue_order_flags(hipStream_t st, unsigned long long q) {
  OrderFlags* o = order_flags();
  if (!o) return true;
  std::lock_guard<std::mutex> lk(o->mu);
  const int k = (int)(q % ORDER_RING);
  if (!check_hip(hipEventRecord(o->ev[k], st), "hipEventRecord")) {
    o->state[k] = 0;
    return true;
  }
  o->state[k] = 2;
  bool failed = false;
  for (int j = 0; j < ORDER_RING; j++)
    if (j != k) failed |= check_order_slot_locked(*o, j, false);
  return failed;
}
// a forward that reserved a word and failed before queueing its render gives the word back
static void release_order_word(unsigned long long q) {
  OrderFlags* o = order_flags();
  if (!o) return;
  std::lock_guard<std::mutex> lk(o->mu);
  const int k = (int)(q % ORDER_RING);
  if (o->state[k] == 1) o->state[k] = 0;
}

// Status of bounded forwards (gs_forward_bounded), per device: pinned words the kernels store into
// only when a view has error flags -- [0] the preprocess totals' flags (CounterFinalize) with [1], [2]
// that view's instance count, [4] the ordering flags (render kernel) -- so no event, no host wait
// and nothing per call (HIP-graph capturable).  gs_bounded_status reads and clears them.
struct BoundedStatus {
  std::mutex mu;
  uint32_t* host = nullptr;
  uint32_t* dev = nullptr;
};
static BoundedStatus g_bounded[64];
static BoundedStatus* bounded_status() {
  int dev = 0;
  if (!check_hip(hipGetDevice(&dev), "hipGetDevice")) return nullptr;
  if (dev < 0 || dev >= 64) return set_error("device ordinal out of range"), nullptr;
  BoundedStatus& b = g_bounded[dev];
  std::lock_guard<std::mutex> lk(b.mu);
  if (!b.host && !mapped_words(64, &b.host, &b.dev)) return nullptr;
  return &b;
}
// flags of the bounded forwards since the last read (0: none), and the instance count of a view that
// raised them; clears them
static uint32_t take_bounded_status(BoundedStatus* b, long long* instances) {
  std::lock_guard<std::mutex> lk(b->mu);
  uint32_t* w = b->host;
  // take and clear each flag word in one atomic exchange: a bounded kernel still in flight that
  // stores its flags between a read and a clear would otherwise lose them (the count words are
  // only meaningful beside a flag, so they are taken after the flags)
  const uint32_t f = __atomic_exchange_n(&w[0], 0u, __ATOMIC_ACQ_REL) | __atomic_exchange_n(&w[4], 0u, __ATOMIC_ACQ_REL);
  const uint32_t lo = __atomic_exchange_n(&w[1], 0u, __ATOMIC_ACQ_REL), hi = __atomic_exchange_n(&w[2], 0u, __ATOMIC_ACQ_REL);
  if (instances) *instances = f ? (long long)((unsigned long long)hi << 32 | lo) : 0;
  return f;
}
static bool bounded_status_error(uint32_t f, long long inst) {
  if (f & ERR_PREFILTERED) return set_error("Point is filtered although prefiltered is set. This shouldn't happen!"), true;
  if (f & (ERR_CAPACITY | ERR_INSTANCES))
    return set_error("bounded forward: a view had %lld (Gaussian, tile) instances, more than its binning capacity "
                     "(its image and gradients are invalid; rerun with a larger capacity)", inst), true;
  if (f & ERR_LOOKBACK)
    return set_error("bounded forward: a look-back wait of the offsets scan or a one-sweep sort timed out "
                     "(the instance list of that forward is invalid)"), true;
  return false;
}

// split SH inputs (features_dc + features_rest rows): shs_rest needs SH colours with M >= 2
static bool validate_split(int M, const float* shs, const float* shs_rest, const float* colors_precomp) {
  if (!shs_rest) return true;
  if (!shs || colors_precomp) return set_error("split SH: features_dc and features_rest replace shs (no colours)"), false;
  if (M < 2) return set_error("split SH: M must be >= 2 (got %d)", M), false;
  return true;
}

static int forward_preprocess_impl(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                                   const float* shs, const float* shs_rest, const float* colors_precomp,
                                   const float* opacities, const float* scales, float scale_modifier,
                                   const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                                   const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                                   int prefiltered, int* radii_out, void* geom_buffer, long long* num_rendered_host,
                                   int debug, void* stream) {
  clear_error(debug);
  if (num_rendered_host) *num_rendered_host = 0;
  if (!validate(P, D, M, W, H, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, viewmatrix,
                projmatrix, campos, background))
    return 1;
  if (!validate_split(M, shs, shs_rest, colors_precomp)) return 1;
  if (P == 0) return 0;
  if (!radii_out || !geom_buffer || !num_rendered_host) return set_error("missing output pointer"), 1;
  hipStream_t st = (hipStream_t)stream;
  GeomPtrs geo;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  GaussianArgs g{P, D, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, scale_modifier,
                 shs_rest};
  CameraArgs c = make_camera(background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, prefiltered);
  // num_rendered is the sum of the per-Gaussian tile counts, known when the first depth-sort
  // histogram launch has summed the preprocess workgroups' totals: that launch stores it straight
  // into pinned memory, and the host waits for it while the GPU goes on with the depth sort and
  // the instance offsets, so the host round trip overlaps device work.
  ReadbackSlot* rb = readback_slot();
  if (!rb) return 1;
  // earlier forwards' look-back waits: the finished ones now (no wait before the launches), then,
  // after this forward's own readback (behind them on the stream), the rest
  if (check_order_flags(false)) return 1;
  fwd_preprocess(g, c, radii_out, geo, st);
  fwd_order(P, geo, st, rb->dev, rb->ev[0]);
  check_hip(hipEventSynchronize(rb->ev[0]), "hipEventSynchronize");
  if (t_failed) return 1;
  if (check_order_flags()) return 1;
  return read_view_totals(rb->host, 0, 1, num_rendered_host) ? 0 : 1;
}

int gs_forward_preprocess(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                          const float* shs, const float* colors_precomp, const float* opacities, const float* scales,
                          float scale_modifier, const float* rotations, const float* cov3D_precomp,
                          const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                          float tan_fovy, int prefiltered, int* radii_out, void* geom_buffer,
                          long long* num_rendered_host, int debug, void* stream) {
  return forward_preprocess_impl(P, D, M, background, W, H, means3D, shs, nullptr, colors_precomp, opacities, scales,
                                 scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx,
                                 tan_fovy, prefiltered, radii_out, geom_buffer, num_rendered_host, debug, stream);
}

int gs_forward_preprocess_split(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                                const float* shs_dc, const float* shs_rest, const float* opacities,
                                const float* scales, float scale_modifier, const float* rotations,
                                const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                                const float* campos, float tan_fovx, float tan_fovy, int prefiltered, int* radii_out,
                                void* geom_buffer, long long* num_rendered_host, int debug, void* stream) {
  if (!shs_rest) {
    clear_error(debug);
    if (num_rendered_host) *num_rendered_host = 0;
    return set_error("split SH: features_rest is NULL"), 1;
  }
  return forward_preprocess_impl(P, D, M, background, W, H, means3D, shs_dc, shs_rest, nullptr, opacities, scales,
                                 scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx,
                                 tan_fovy, prefiltered, radii_out, geom_buffer, num_rendered_host, debug, stream);
}

// The K views' depth sorts as one set of launches (contiguous geometry buffers); GSRAST_BATCH_VIEWS=0
// in the environment runs them view by view on the views' streams (A/B runs; the Python layer then
// also bins the views one by one)
constexpr int GS_BATCH_ORDER_MAX = 2 << 20;      // Gaussians up to which the views' depth sorts batch
constexpr uint32_t GS_BATCH_BIN_MAX = 8u << 20;  // instances per view up to which gs_forward_bin_views batches
static bool batch_views() {
  static const bool on = [] {
    const char* e = getenv("GSRAST_BATCH_VIEWS");
    return !(e && e[0] == '0');
  }();
  return on;
}
// capacity (bounded, gs_forward_preprocess_views_bounded): per-view binning capacities; the counts
// are not read back (num_rendered_host unused), a view over its capacity leaves the sticky flag
static int preprocess_views_impl(int K, int P, int D, int M, const float* const* background, const int* image_width,
                                 const int* image_height, const float* means3D, const float* shs,
                                 const float* colors_precomp, const float* opacities, const float* scales,
                                 float scale_modifier, const float* rotations, const float* cov3D_precomp,
                                 const float* const* viewmatrix, const float* const* projmatrix,
                                 const float* const* campos, const float* tan_fovx, const float* tan_fovy,
                                 int prefiltered, int* const* radii_out, void* const* geom_buffer,
                                 long long* num_rendered_host, const long long* capacity, int debug, void* stream,
                                 void* const* view_streams) {
  clear_error(debug);
  if (K <= 0 || K > FUSED_MAX_VIEWS) return set_error("views: 1 to 8 per call"), 1;
  if (!background || !image_width || !image_height || !viewmatrix || !projmatrix || !campos || !tan_fovx ||
      !tan_fovy || !radii_out || !geom_buffer || (!num_rendered_host && !capacity))
    return set_error("missing per-view argument array"), 1;
  for (int v = 0; v < K; v++) {
    if (num_rendered_host) num_rendered_host[v] = 0;
    if (capacity && (capacity[v] < 0 || capacity[v] > GS_MAX_INSTANCES)) return set_error("capacity out of range"), 1;
    if (!validate(P, D, M, image_width[v], image_height[v], means3D, shs, colors_precomp, opacities, scales, rotations,
                  cov3D_precomp, viewmatrix[v], projmatrix[v], campos[v], background[v]))
      return 1;
    if (P > 0 && (!radii_out[v] || !geom_buffer[v])) return set_error("missing output pointer"), 1;
  }
  if (P == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  GaussianArgs g{P, D, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, scale_modifier};
  PreViews pv;
  pv.K = K;
  for (int v = 0; v < K; v++) {
    pv.c[v] = make_camera(background[v], image_width[v], image_height[v], viewmatrix[v], projmatrix[v], campos[v],
                          tan_fovx[v], tan_fovy[v], prefiltered);
    pv.radii[v] = radii_out[v];
    geom_layout((size_t)P, &pv.geo[v], (char*)geom_buffer[v]);
  }
  // (bounded: no readback slot, the views' flags go to the sticky words)
  ReadbackSlot* rb = capacity ? nullptr : readback_slot();
  if (!capacity && !rb) return 1;
  BoundedStatus* bs = capacity ? bounded_status() : nullptr;
  if (capacity && !bs) return 1;
  if (bs) {
    long long inst = 0;
    if (bounded_status_error(take_bounded_status(bs, &inst), inst)) return 1;  // an earlier bounded forward
  }
  // one fork event per thread and slot of a ring: a captured step may hold several forks
  static thread_local hipEvent_t ev_pre[4] = {};
  static thread_local unsigned ev_next = 0;
  hipEvent_t& fork = ev_pre[ev_next++ & 3];
  if (!fork && !check_hip(hipEventCreateWithFlags(&fork, hipEventDisableTiming), "hipEventCreate")) return 1;
  if (!capacity && check_order_flags(false)) return 1;  // earlier forwards' look-back waits (finished ones)
  uint32_t cap32[FUSED_MAX_VIEWS];
  for (int v = 0; v < K; v++) cap32[v] = capacity ? (uint32_t)capacity[v] : 0xFFFFFFFFu;
  // geometry buffers at one stride (slices of one allocation, as prepare_views makes them): the K
  // orderings run as one set of launches on `stream` (blockIdx.y = view), every view's totals
  // stored by the first histogram launch into readback words [8 v, 8 v + 4)
  const ptrdiff_t vstride = K > 1 ? (char*)geom_buffer[1] - (char*)geom_buffer[0] : 0;
  // (up to GS_BATCH_ORDER_MAX Gaussians: larger sorts fill the GPU on their own, and view by view
  // on the views' streams they overlap the other views' render kernels)
  bool batched = batch_views() && K > 1 && P <= GS_BATCH_ORDER_MAX && vstride >= (ptrdiff_t)gs_geom_buffer_bytes(P) &&
                 vstride % 256 == 0;
  for (int v = 2; v < K && batched; v++) batched = (char*)geom_buffer[v] == (char*)geom_buffer[0] + v * vstride;
  fwd_preprocess_views(g, pv, st);
  if (batched) {
    fwd_order(P, pv.geo[0], st, capacity ? nullptr : rb->dev, capacity ? nullptr : rb->ev[0], cap32,
              capacity ? bs->dev : nullptr, K, (uint64_t)vstride);
    // the views' later kernels run on their streams, after the orderings
    check_hip(hipEventRecord(fork, st), "hipEventRecord");
    for (int v = 0; v < K; v++) {
      hipStream_t vs = view_streams && view_streams[v] ? (hipStream_t)view_streams[v] : st;
      if (vs != st) check_hip(hipStreamWaitEvent(vs, fork, 0), "hipStreamWaitEvent");
    }
  } else {
    // each view's ordering on its own stream (view_streams[v], or `stream`), after the preprocess
    check_hip(hipEventRecord(fork, st), "hipEventRecord");
    for (int v = 0; v < K; v++) {
      hipStream_t vs = view_streams && view_streams[v] ? (hipStream_t)view_streams[v] : st;
      if (vs != st) check_hip(hipStreamWaitEvent(vs, fork, 0), "hipStreamWaitEvent");
      if (capacity)
        fwd_order(P, pv.geo[v], vs, nullptr, nullptr, &cap32[v], bs->dev);
      else
        fwd_order(P, pv.geo[v], vs, rb->dev + 8 * v, rb->ev[v]);
    }
  }
  if (capacity) return t_failed ? 1 : 0;
  for (int v = 0; v < (batched ? 1 : K); v++) check_hip(hipEventSynchronize(rb->ev[v]), "hipEventSynchronize");
  if (t_failed) return 1;
  if (check_order_flags()) return 1;  // the rest of the earlier forwards (behind their renders, as a rule)
  for (int v = 0; v < K; v++)
    if (!read_view_totals(rb->host + 8 * v, v, K, &num_rendered_host[v])) return 1;
  return 0;
}

int gs_forward_preprocess_views(int K, int P, int D, int M, const float* const* background, const int* image_width,
                                const int* image_height, const float* means3D, const float* shs,
                                const float* colors_precomp, const float* opacities, const float* scales,
                                float scale_modifier, const float* rotations, const float* cov3D_precomp,
                                const float* const* viewmatrix, const float* const* projmatrix,
                                const float* const* campos, const float* tan_fovx, const float* tan_fovy,
                                int prefiltered, int* const* radii_out, void* const* geom_buffer,
                                long long* num_rendered_host, int debug, void* stream, void* const* view_streams) {
  if (!num_rendered_host) {
    clear_error(debug);
    return set_error("missing per-view argument array"), 1;
  }
  return preprocess_views_impl(K, P, D, M, background, image_width, image_height, means3D, shs, colors_precomp,
                               opacities, scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix,
                               campos, tan_fovx, tan_fovy, prefiltered, radii_out, geom_buffer, num_rendered_host,
                               nullptr, debug, stream, view_streams);
}

int gs_forward_preprocess_views_bounded(int K, int P, int D, int M, const float* const* background,
                                        const int* image_width, const int* image_height, const float* means3D,
                                        const float* shs, const float* colors_precomp, const float* opacities,
                                        const float* scales, float scale_modifier, const float* rotations,
                                        const float* cov3D_precomp, const float* const* viewmatrix,
                                        const float* const* projmatrix, const float* const* campos,
                                        const float* tan_fovx, const float* tan_fovy, int prefiltered,
                                        int* const* radii_out, void* const* geom_buffer, const long long* capacity,
                                        int debug, void* stream, void* const* view_streams) {
  if (!capacity) {
    clear_error(debug);
    return set_error("missing capacity array"), 1;
  }
  return preprocess_views_impl(K, P, D, M, background, image_width, image_height, means3D, shs, colors_precomp,
                               opacities, scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix,
                               campos, tan_fovx, tan_fovy, prefiltered, radii_out, geom_buffer, nullptr, capacity,
                               debug, stream, view_streams);
}

static int forward_render_impl(int P, const float* background, int W, int H, const float* viewmatrix,
                               const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                               const int* radii, void* geom_buffer, long long num_rendered, void* binning_buffer,
                               void* image_buffer, float* out_color, bool bounded, int debug, void* stream,
                               unsigned long long* oseq_out = nullptr) {
  clear_error(debug);
  if (P <= 0) return 0;
  if (W <= 0 || H <= 0) return set_error("image size must be positive"), 1;
  if (num_rendered < 0 || num_rendered > GS_MAX_INSTANCES) return set_error("num_rendered out of range"), 1;
  if (!geom_buffer || !binning_buffer || !image_buffer || !out_color || !radii)
    return set_error("missing buffer pointer"), 1;
  hipStream_t st = (hipStream_t)stream;
  CameraArgs c = make_camera(background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, 0);
  GeomPtrs geo;
  BinPtrs bin;
  ImgPtrs img;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  bin_layout((size_t)num_rendered, c.gx * c.gy, &bin, (char*)binning_buffer);
  img_layout(W, H, &img, (char*)image_buffer);
  // the look-back waits of the offsets scan and of the one-sweep sorts (never expected to run out:
  // the waited-for workgroups are running) leave ERR_LOOKBACK; the render kernel stores the flags
  // into pinned memory, behind an event that the next backward or forward call checks, so no host
  // wait idles the device
  // (bounded: the sticky word, nothing recorded or checked here)
  BoundedStatus* bs = bounded ? bounded_status() : nullptr;
  unsigned long long oseq = 0;
  uint32_t* flags_word = bounded ? (bs ? bs->dev + 4 : nullptr) : order_flags_word(&oseq);
  if (!flags_word) return 1;
  fwd_bin(P, (uint32_t)num_rendered, c, radii, geo, bin, img, st);
  fwd_render(c, geo, bin, img, out_color, st, flags_word);
  if (!bounded) {
    if (oseq_out) *oseq_out = oseq;
    if (t_failed) release_order_word(oseq);
    else if (queue_order_flags(st, oseq)) return 1;
  }
  return t_failed ? 1 : 0;
}

int gs_forward_bin_views(int K, int P, int W, int H, void* const* geom_buffer, const long long* num_rendered,
                         void* const* binning_buffer, void* const* image_buffer, int debug, void* stream,
                         void* const* view_streams) {
  clear_error(debug);
  if (K <= 0 || K > FUSED_MAX_VIEWS) return set_error("views: 1 to 8 per call"), 1;
  if (P < 0) return set_error("P must be >= 0"), 1;
  if (W <= 0 || H <= 0) return set_error("image size must be positive"), 1;
  if (!geom_buffer || !num_rendered || !binning_buffer || !image_buffer) return set_error("missing per-view array"), 1;
  if (P == 0) return 0;
  long long I = 0;
  for (int v = 0; v < K; v++) {
    if (!geom_buffer[v] || !binning_buffer[v] || !image_buffer[v]) return set_error("view %d: missing buffer", v), 1;
    if (num_rendered[v] < 0 || num_rendered[v] > GS_MAX_INSTANCES) return set_error("num_rendered out of range"), 1;
    I = num_rendered[v] > I ? num_rendered[v] : I;
  }
  hipStream_t st = (hipStream_t)stream;
  CameraArgs c = make_camera(nullptr, W, H, nullptr, nullptr, nullptr, 1.0f, 1.0f, 0);
  // every view's buffers at one stride per kind (slices of one allocation each)
  auto stride_of = [&](void* const* b, size_t min_bytes, uint64_t* out) {
    const ptrdiff_t d = K > 1 ? (char*)b[1] - (char*)b[0] : 0;
    if (K > 1 && (d < (ptrdiff_t)min_bytes || d % 256 != 0)) return false;
    for (int v = 2; v < K; v++)
      if ((char*)b[v] != (char*)b[0] + v * d) return false;
    *out = (uint64_t)d;
    return true;
  };
  uint64_t gs = 0, bs = 0, is = 0;
  if (!stride_of(geom_buffer, gs_geom_buffer_bytes(P), &gs) ||
      !stride_of(binning_buffer, gs_binning_buffer_bytes(I, W, H), &bs) ||
      !stride_of(image_buffer, gs_image_buffer_bytes(W, H), &is))
    return set_error("bin_views: each kind of buffer must be K slices of one allocation, one stride apart, each "
                     "sized for the largest num_rendered"), 1;
  GeomPtrs geo;
  BinPtrs bin;
  ImgPtrs img;
  if (!batch_views() || I > (long long)GS_BATCH_BIN_MAX) {
    // large views: each view's binning on its own stream, where it overlaps the other views'
    // render kernels (a batched sort of K large views would serialise in front of them)
    for (int v = 0; v < K; v++) {
      hipStream_t vs = view_streams && view_streams[v] ? (hipStream_t)view_streams[v] : st;
      geom_layout((size_t)P, &geo, (char*)geom_buffer[v]);
      bin_layout((size_t)I, c.gx * c.gy, &bin, (char*)binning_buffer[v]);
      img_layout(W, H, &img, (char*)image_buffer[v]);
      fwd_bin_views(1, P, (uint32_t)I, c, geo, bin, img, 0, 0, 0, vs);
    }
    return t_failed ? 1 : 0;
  }
  geom_layout((size_t)P, &geo, (char*)geom_buffer[0]);
  bin_layout((size_t)I, c.gx * c.gy, &bin, (char*)binning_buffer[0]);
  img_layout(W, H, &img, (char*)image_buffer[0]);
  fwd_bin_views(K, P, (uint32_t)I, c, geo, bin, img, gs, bs, is, st);
  // the views' renders run on their streams, after the binning
  static thread_local hipEvent_t ev_bin[4] = {};
  static thread_local unsigned ev_next = 0;
  hipEvent_t& done = ev_bin[ev_next++ & 3];
  if (!done && !check_hip(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate")) return 1;
  check_hip(hipEventRecord(done, st), "hipEventRecord");
  for (int v = 0; v < K; v++) {
    hipStream_t vs = view_streams && view_streams[v] ? (hipStream_t)view_streams[v] : st;
    if (vs != st) check_hip(hipStreamWaitEvent(vs, done, 0), "hipStreamWaitEvent");
  }
  return t_failed ? 1 : 0;
}

int gs_forward_render_binned(int P, const float* background, int W, int H, const float* viewmatrix,
                             const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                             void* geom_buffer, long long num_rendered, void* binning_buffer, void* image_buffer,
                             float* out_color, int bounded, int debug, void* stream) {
  clear_error(debug);
  if (P <= 0) return 0;
  if (W <= 0 || H <= 0) return set_error("image size must be positive"), 1;
  if (num_rendered < 0 || num_rendered > GS_MAX_INSTANCES) return set_error("num_rendered out of range"), 1;
  if (!geom_buffer || !binning_buffer || !image_buffer || !out_color) return set_error("missing buffer pointer"), 1;
  hipStream_t st = (hipStream_t)stream;
  CameraArgs c = make_camera(background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, 0);
  GeomPtrs geo;
  BinPtrs bin;
  ImgPtrs img;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  bin_layout((size_t)num_rendered, c.gx * c.gy, &bin, (char*)binning_buffer);
  img_layout(W, H, &img, (char*)image_buffer);
  BoundedStatus* bst = bounded ? bounded_status() : nullptr;
  unsigned long long oseq = 0;
  uint32_t* flags_word = bounded ? (bst ? bst->dev + 4 : nullptr) : order_flags_word(&oseq);
  if (!flags_word) return 1;
  fwd_render(c, geo, bin, img, out_color, st, flags_word);
  if (!bounded) {
    if (t_failed) release_order_word(oseq);
    else if (queue_order_flags(st, oseq)) return 1;
  }
  return t_failed ? 1 : 0;
}

int gs_forward_render(int P, const float* background, int W, int H, const float* viewmatrix, const float* projmatrix,
                      const float* campos, float tan_fovx, float tan_fovy, const int* radii, void* geom_buffer,
                      long long num_rendered, void* binning_buffer, void* image_buffer, float* out_color, int debug,
                      void* stream) {
  return forward_render_impl(P, background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii,
                             geom_buffer, num_rendered, binning_buffer, image_buffer, out_color, false, debug, stream);
}

int gs_forward_render_bounded(int P, const float* background, int W, int H, const float* viewmatrix,
                              const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                              const int* radii, void* geom_buffer, long long capacity, void* binning_buffer,
                              void* image_buffer, float* out_color, int debug, void* stream) {
  return forward_render_impl(P, background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii,
                             geom_buffer, capacity, binning_buffer, image_buffer, out_color, true, debug, stream);
}

int gs_forward_bounded(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                       const float* shs, const float* shs_rest, const float* colors_precomp, const float* opacities,
                       const float* scales, float scale_modifier, const float* rotations, const float* cov3D_precomp,
                       const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                       float tan_fovy, int prefiltered, int* radii_out, void* geom_buffer, long long capacity,
                       void* binning_buffer, void* image_buffer, float* out_color, int debug, void* stream) {
  clear_error(debug);
  if (!validate(P, D, M, W, H, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, viewmatrix,
                projmatrix, campos, background))
    return 1;
  if (!validate_split(M, shs, shs_rest, colors_precomp)) return 1;
  if (P == 0) return 0;
  if (capacity < 0 || capacity > GS_MAX_INSTANCES) return set_error("capacity out of range"), 1;
  if (!radii_out || !geom_buffer || !binning_buffer || !image_buffer || !out_color)
    return set_error("missing buffer pointer"), 1;
  BoundedStatus* bs = bounded_status();
  if (!bs) return 1;
  long long inst = 0;
  if (bounded_status_error(take_bounded_status(bs, &inst), inst)) return 1;  // an earlier bounded forward
  hipStream_t st = (hipStream_t)stream;
  GeomPtrs geo;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  GaussianArgs g{P, D, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, scale_modifier,
                 shs_rest};
  CameraArgs c = make_camera(background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, prefiltered);
  fwd_preprocess(g, c, radii_out, geo, st);
  const uint32_t cap32 = (uint32_t)capacity;
  fwd_order(P, geo, st, nullptr, nullptr, &cap32, bs->dev);
  if (t_failed) return 1;
  return forward_render_impl(P, background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii_out,
                             geom_buffer, capacity, binning_buffer, image_buffer, out_color, true, debug, stream);
}

// The eager forward with its count read back at the end (gsrast.h): the ordering stores the totals
// into the readback slot and flags ERR_CAPACITY against `capacity`; the binning and the render are
// queued behind it on the stream at once, so the device never waits for the host's round trip.
int gs_forward_counted(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                       const float* shs, const float* shs_rest, const float* colors_precomp, const float* opacities,
                       const float* scales, float scale_modifier, const float* rotations, const float* cov3D_precomp,
                       const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                       float tan_fovy, int prefiltered, int* radii_out, void* geom_buffer, long long capacity,
                       void* binning_buffer, void* image_buffer, float* out_color, long long* num_rendered_host,
                       int debug, void* stream) {
  clear_error(debug);
  if (num_rendered_host) *num_rendered_host = 0;
  if (!validate(P, D, M, W, H, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, viewmatrix,
                projmatrix, campos, background))
    return 1;
  if (!validate_split(M, shs, shs_rest, colors_precomp)) return 1;
  if (P == 0) return 0;
  if (capacity < 0 || capacity > GS_MAX_INSTANCES) return set_error("capacity out of range"), 1;
  if (!radii_out || !geom_buffer || !binning_buffer || !image_buffer || !out_color || !num_rendered_host)
    return set_error("missing buffer pointer"), 1;
  ReadbackSlot* rb = readback_slot();
  if (!rb) return 1;
  if (check_order_flags(false)) return 1;  // earlier forwards' look-back waits (the finished ones)
  hipStream_t st = (hipStream_t)stream;
  GeomPtrs geo;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  GaussianArgs g{P, D, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, scale_modifier,
                 shs_rest};
  CameraArgs c = make_camera(background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, prefiltered);
  fwd_preprocess(g, c, radii_out, geo, st);
  const uint32_t cap32 = (uint32_t)capacity;
  fwd_order(P, geo, st, rb->dev, rb->ev[0], &cap32, nullptr);
  // the count readback is queued into this thread's slot: every return from here on waits for it,
  // so no kernel of this call can still write the slot's words when the thread's next call reads them
  auto drain = [&]() { (void)hipEventSynchronize(rb->ev[0]); };
  if (t_failed) return drain(), 1;
  unsigned long long oseq = 0;
  if (forward_render_impl(P, background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii_out,
                          geom_buffer, capacity, binning_buffer, image_buffer, out_color, false, debug, stream,
                          &oseq))
    return drain(), 1;
  check_hip(hipEventSynchronize(rb->ev[0]), "hipEventSynchronize");
  if (t_failed) return 1;
  // (this forward's render is queued: check the others, without waiting for it)
  if (check_order_flags(true, (long long)oseq)) return 1;
  long long I = 0;
  if (!read_view_totals(rb->host, 0, 1, &I)) return 1;
  *num_rendered_host = I;
  if (I > capacity) {
    // the queued binning and render skipped their work (ERR_CAPACITY): clear the flag so that
    // gs_forward_render can bin the same geometry into a buffer of the exact size
    fwd_clear_flags(geo, ERR_CAPACITY, st);
    // the skipped render carries this ordering's look-back flags: read them now (it finishes
    // quickly, having skipped its work), so a timed-out ordering fails here, once, instead of
    // again at the next call through the re-binned forward's flags
    if (t_failed || check_order_seq(oseq)) return 1;
    return GS_COUNT_SHORT;
  }
  return 0;
}

int gs_bounded_status(unsigned* flags, long long* instances) {
  clear_error(0);
  BoundedStatus* bs = bounded_status();
  if (!bs) return 1;
  long long inst = 0;
  const uint32_t f = take_bounded_status(bs, &inst);
  if (flags) *flags = f;
  if (instances) *instances = inst;
  return bounded_status_error(f, inst) ? 1 : 0;
}

size_t gs_geom_flags_offset(int P) {
  // the layout's offsets from a dummy base address (nothing is dereferenced)
  alignas(256) static char base[256];
  GeomPtrs geo;
  geom_layout((size_t)(P > 0 ? P : 1), &geo, base);
  return (size_t)((uintptr_t)geo.counters - (uintptr_t)base) + CNT_ERR * sizeof(uint32_t);
}

int gs_forward_order_status(void) {
  clear_error(0);
  return check_order_flags(true) ? 1 : 0;
}

int gs_set_row_waits(int n, const int* bounds, void* const* events) {
  clear_error(0);
  t_row_wait_count = 0;
  if (n == 0) return 0;
  if (n < 0 || n > GS_MAX_ROW_WAITS) return set_error("row waits: 0..%d chunks (got %d)", GS_MAX_ROW_WAITS, n), 1;
  if (!bounds || !events) return set_error("row waits: missing bounds / events"), 1;
  if (bounds[0] != 0) return set_error("row waits: the first chunk must start at row 0"), 1;
  for (int k = 0; k < n; k++)
    if (bounds[k + 1] <= bounds[k]) return set_error("row waits: chunk bounds must increase"), 1;
  for (int k = 0; k < n; k++) t_row_waits[k] = RowWait{bounds[k + 1], (hipEvent_t)events[k]};
  t_row_wait_count = n;
  return 0;
}

long long gs_rasterize_forward(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                               const float* shs, const float* colors_precomp, const float* opacities,
                               const float* scales, float scale_modifier, const float* rotations,
                               const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                               const float* campos, float tan_fovx, float tan_fovy, int prefiltered, float* out_color,
                               int* radii_out, gs_alloc_fn alloc, void* alloc_ctx, void** geom_out,
                               void** binning_out, void** image_out, int debug, void* stream) {
  if (!alloc) {
    clear_error(debug);
    set_error("alloc callback is NULL");
    return -1;
  }
  void* geom = alloc(alloc_ctx, 0, gs_geom_buffer_bytes(P));
  long long I = 0;
  if (gs_forward_preprocess(P, D, M, background, W, H, means3D, shs, colors_precomp, opacities, scales,
                            scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx,
                            tan_fovy, prefiltered, radii_out, geom, &I, debug, stream))
    return -1;
  void* bin = alloc(alloc_ctx, 1, gs_binning_buffer_bytes(I, W, H));
  void* img = alloc(alloc_ctx, 2, gs_image_buffer_bytes(W, H));
  if (geom_out) *geom_out = geom;
  if (binning_out) *binning_out = bin;
  if (image_out) *image_out = img;
  if (gs_forward_render(P, background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii_out, geom, I,
                        bin, img, out_color, debug, stream))
    return -1;
  return I;
}

static int backward_impl(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                         const float* shs, const float* shs_rest, const float* colors_precomp, const float* opacities, const float* scales,
                         float scale_modifier, const float* rotations, const float* cov3D_precomp,
                         const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                         float tan_fovy, const void* geom_buffer, long long num_rendered, const void* binning_buffer,
                         const void* image_buffer, const float* dL_dout_color, void* grad_buffer, float* dL_dmeans2D,
                         float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                         float* dL_dscales, float* dL_drotations, unsigned accumulate, void* wait_event, int debug,
                         void* stream) {
  clear_error(debug);
  (void)opacities;  // the opacity is carried by the forward's splat records
  if (!validate(P, D, M, W, H, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, viewmatrix,
                projmatrix, campos, background, false))
    return 1;
  if (!validate_split(M, shs, shs_rest, colors_precomp)) return 1;
  if (P == 0) return 0;
  if (!geom_buffer || !binning_buffer || !image_buffer || !dL_dout_color || !grad_buffer)
    return set_error("missing buffer pointer"), 1;
  if (!dL_dmeans2D || !dL_dopacity || !dL_dmeans3D) return set_error("missing gradient output pointer"), 1;
  if (num_rendered < 0 || num_rendered > GS_MAX_INSTANCES) return set_error("num_rendered out of range"), 1;
  if (accumulate & ~0xFFu) return set_error("accumulate: unknown GS_ACC bits 0x%x", accumulate), 1;
  hipStream_t st = (hipStream_t)stream;
  CameraArgs c = make_camera(background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, 0);
  GeomPtrs geo;
  BinPtrs bin;
  ImgPtrs img;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  bin_layout((size_t)num_rendered, c.gx * c.gy, &bin, (char*)binning_buffer);
  img_layout(W, H, &img, (char*)image_buffer);
  GaussianArgs g{P, D, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp, scale_modifier,
                 shs_rest};
  float* gradrec = (float*)grad_buffer;
  if (num_rendered > 0) bwd_render(P, c, geo, bin, img, dL_dout_color, gradrec, st);
  // dL_dcov3D is filled whenever the caller passes it: upstream writes it for scale/rotation
  // inputs too (the covariance gradient the scale / rotation chain starts from)
  GradOut out{dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
              shs ? dL_dsh : nullptr, cov3D_precomp ? nullptr : dL_dscales, cov3D_precomp ? nullptr : dL_drotations,
              accumulate};
  // the gradient outputs may be shared with views on other streams: order only this last kernel
  if (wait_event && !check_hip(hipStreamWaitEvent(st, (hipEvent_t)wait_event, 0), "hipStreamWaitEvent")) return 1;
  bwd_preprocess(g, c, geo, bin, img, gradrec, (uint32_t)num_rendered, num_rendered > 0, out, st);
  // the ordering flags of the forwards that have finished, now that this backward's kernels are queued
  if (!t_failed && check_order_flags(false)) return 1;
  return t_failed ? 1 : 0;
}

int gs_backward(int P, int D, int M, const float* background, int W, int H, const float* means3D, const float* shs,
                const float* colors_precomp, const float* opacities, const float* scales, float scale_modifier,
                const float* rotations, const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                const float* campos, float tan_fovx, float tan_fovy, const int* radii, const void* geom_buffer,
                long long num_rendered, const void* binning_buffer, const void* image_buffer,
                const float* dL_dout_color, void* grad_buffer, float* dL_dmeans2D, float* dL_dcolors,
                float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                float* dL_drotations, int debug, void* stream) {
  (void)radii;
  return backward_impl(P, D, M, background, W, H, means3D, shs, nullptr, colors_precomp, opacities, scales, scale_modifier,
                       rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, geom_buffer,
                       num_rendered, binning_buffer, image_buffer, dL_dout_color, grad_buffer, dL_dmeans2D,
                       dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations, 0u, nullptr,
                       debug, stream);
}

int gs_backward_accumulate(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                           const float* shs, const float* colors_precomp, const float* opacities,
                           const float* scales, float scale_modifier, const float* rotations,
                           const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                           const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                           const void* geom_buffer, long long num_rendered, const void* binning_buffer,
                           const void* image_buffer, const float* dL_dout_color, void* grad_buffer,
                           float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                           float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                           unsigned accumulate, void* wait_event, int debug, void* stream) {
  (void)radii;
  return backward_impl(P, D, M, background, W, H, means3D, shs, nullptr, colors_precomp, opacities, scales, scale_modifier,
                       rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, geom_buffer,
                       num_rendered, binning_buffer, image_buffer, dL_dout_color, grad_buffer, dL_dmeans2D,
                       dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations, accumulate,
                       wait_event, debug, stream);
}

int gs_backward_accumulate_split(int P, int D, int M, const float* background, int W, int H, const float* means3D,
                                 const float* shs_dc, const float* shs_rest, const float* opacities,
                                 const float* scales, float scale_modifier, const float* rotations,
                                 const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                                 const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                                 const void* geom_buffer, long long num_rendered, const void* binning_buffer,
                                 const void* image_buffer, const float* dL_dout_color, void* grad_buffer,
                                 float* dL_dmeans2D, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D,
                                 float* dL_dsh, float* dL_dscales, float* dL_drotations, unsigned accumulate,
                                 void* wait_event, int debug, void* stream) {
  (void)radii;
  if (!shs_rest) {
    clear_error(debug);
    return set_error("split SH: features_rest is NULL"), 1;
  }
  return backward_impl(P, D, M, background, W, H, means3D, shs_dc, shs_rest, nullptr, opacities, scales,
                       scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy,
                       geom_buffer, num_rendered, binning_buffer, image_buffer, dL_dout_color, grad_buffer,
                       dL_dmeans2D, nullptr, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations,
                       accumulate, wait_event, debug, stream);
}

int gs_backward_render(int P, int D, int M, const float* background, int W, int H, const float* viewmatrix,
                       const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                       const void* geom_buffer, long long num_rendered, const void* binning_buffer,
                       const void* image_buffer, const float* dL_dout_color, void* grad_buffer, float* dL_dmeans2D,
                       unsigned accumulate, int debug, void* stream) {
  clear_error(debug);
  if (P < 0) return set_error("P must be >= 0"), 1;
  if (W <= 0 || H <= 0) return set_error("image size must be positive (got %d x %d)", W, H), 1;
  if (P == 0) return 0;
  if (!viewmatrix || !projmatrix || !background) return set_error("missing required input pointer"), 1;
  if (!geom_buffer || !binning_buffer || !image_buffer || !dL_dout_color || !grad_buffer)
    return set_error("missing buffer pointer"), 1;
  if (num_rendered < 0 || num_rendered > GS_MAX_INSTANCES) return set_error("num_rendered out of range"), 1;
  if (accumulate & ~GS_ACC_MEANS2D) return set_error("accumulate: only GS_ACC_MEANS2D applies here"), 1;
  hipStream_t st = (hipStream_t)stream;
  CameraArgs c = make_camera(background, W, H, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, 0);
  GeomPtrs geo;
  BinPtrs bin;
  ImgPtrs img;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  bin_layout((size_t)num_rendered, c.gx * c.gy, &bin, (char*)binning_buffer);
  img_layout(W, H, &img, (char*)image_buffer);
  GaussianArgs g{P, D, M, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1.0f};
  float* gradrec = (float*)grad_buffer;
  if (num_rendered > 0) bwd_render(P, c, geo, bin, img, dL_dout_color, gradrec, st);
  bwd_records(g, geo, bin, img, gradrec, (uint32_t)num_rendered, num_rendered > 0, dL_dmeans2D, accumulate, st);
  if (!t_failed && check_order_flags(false)) return 1;
  return t_failed ? 1 : 0;
}

static int backward_gaussians_impl(int P, int first, int count, int D, int M, const float* means3D, const float* shs,
                                   const float* colors_precomp, const float* scales, float scale_modifier,
                                   const float* rotations, const float* cov3D_precomp, int num_views,
                                   const gs_view_grad* views, float* dL_dcolors, float* dL_dopacity,
                                   float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                                   float* dL_drotations, unsigned accumulate, void* wait_event, int debug,
                                   void* stream) {
  clear_error(debug);
  if (P < 0) return set_error("P must be >= 0"), 1;
  if (first < 0 || count < 0 || (long long)first + count > P) return set_error("Gaussian range out of bounds"), 1;
  if (num_views < 0 || (num_views > 0 && !views)) return set_error("bad view list"), 1;
  if (P == 0 || count == 0 || num_views == 0) return 0;
  if (!means3D) return set_error("missing required input pointer"), 1;
  if ((shs == nullptr) == (colors_precomp == nullptr))
    return set_error("Please provide excatly one of either SHs or precomputed colors!"), 1;
  if (((scales == nullptr || rotations == nullptr) && cov3D_precomp == nullptr) ||
      ((scales || rotations) && cov3D_precomp))
    return set_error("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!"), 1;
  if (shs && (D < 0 || D > 3 || M < (D + 1) * (D + 1))) return set_error("bad SH degree / coefficient count"), 1;
  if (!dL_dopacity || !dL_dmeans3D) return set_error("missing gradient output pointer"), 1;
  if (accumulate & ~0xFFu) return set_error("accumulate: unknown GS_ACC bits 0x%x", accumulate), 1;
  for (int v = 0; v < num_views; v++) {
    const gs_view_grad& w = views[v];
    if (!w.viewmatrix || !w.projmatrix || !w.geom_buffer || (shs && !w.campos))
      return set_error("view %d: missing pointer", v), 1;
    if (w.image_width <= 0 || w.image_height <= 0) return set_error("view %d: bad image size", v), 1;
  }
  hipStream_t st = (hipStream_t)stream;
  if (wait_event && !check_hip(hipStreamWaitEvent(st, (hipEvent_t)wait_event, 0), "hipStreamWaitEvent")) return 1;
  // the range [first, first + count) as a P = count problem: every per-Gaussian array is row-indexed,
  // so the rows' pointers are offset by `first` (the geom buffers keep their P-row layout)
  const size_t f = (size_t)first;
  auto off = [f](const float* p, size_t w) { return p ? p + f * w : nullptr; };
  auto offw = [f](float* p, size_t w) { return p ? p + f * w : nullptr; };
  GaussianArgs g{count, D, M, off(means3D, 3), off(shs, 3 * (size_t)M), off(colors_precomp, 3), nullptr,
                 off(scales, 3), off(rotations, 4), off(cov3D_precomp, 6), scale_modifier};
  // passes of up to FUSED_MAX_VIEWS views; the later passes add to what the earlier wrote
  for (int v0 = 0; v0 < num_views; v0 += FUSED_MAX_VIEWS) {
    FusedViews fv;
    fv.K = num_views - v0 < FUSED_MAX_VIEWS ? num_views - v0 : FUSED_MAX_VIEWS;
    for (int k = 0; k < fv.K; k++) {
      const gs_view_grad& w = views[v0 + k];
      GeomPtrs geo;
      geom_layout((size_t)P, &geo, (char*)w.geom_buffer);
      fv.v[k].c = make_camera(nullptr, w.image_width, w.image_height, w.viewmatrix, w.projmatrix, w.campos,
                              w.tan_fovx, w.tan_fovy, 0);
      fv.v[k].tiles = geo.tiles + f;
      fv.v[k].clamped = geo.clamped + f;
      fv.v[k].gsum = geo.gsum + f * GRAD_REC;
    }
    GradOut out{nullptr, offw(dL_dcolors, 3), offw(dL_dopacity, 1), offw(dL_dmeans3D, 3), offw(dL_dcov3D, 6),
                shs ? offw(dL_dsh, 3 * (size_t)M) : nullptr, cov3D_precomp ? nullptr : offw(dL_dscales, 3),
                cov3D_precomp ? nullptr : offw(dL_drotations, 4), v0 == 0 ? accumulate : 0xFFu};
    bwd_gaussians(g, fv, out, st);
  }
  return t_failed ? 1 : 0;
}

int gs_backward_gaussians(int P, int D, int M, const float* means3D, const float* shs, const float* colors_precomp,
                          const float* scales, float scale_modifier, const float* rotations,
                          const float* cov3D_precomp, int num_views, const gs_view_grad* views, float* dL_dcolors,
                          float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                          float* dL_dscales, float* dL_drotations, unsigned accumulate, void* wait_event, int debug,
                          void* stream) {
  return backward_gaussians_impl(P, 0, P, D, M, means3D, shs, colors_precomp, scales, scale_modifier, rotations,
                                 cov3D_precomp, num_views, views, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
                                 dL_dsh, dL_dscales, dL_drotations, accumulate, wait_event, debug, stream);
}

int gs_backward_gaussians_range(int P, int first, int count, int D, int M, const float* means3D, const float* shs,
                                const float* colors_precomp, const float* scales, float scale_modifier,
                                const float* rotations, const float* cov3D_precomp, int num_views,
                                const gs_view_grad* views, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                                float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                                unsigned accumulate, void* wait_event, int debug, void* stream) {
  return backward_gaussians_impl(P, first, count, D, M, means3D, shs, colors_precomp, scales, scale_modifier,
                                 rotations, cov3D_precomp, num_views, views, dL_dcolors, dL_dopacity, dL_dmeans3D,
                                 dL_dcov3D, dL_dsh, dL_dscales, dL_drotations, accumulate, wait_event, debug, stream);
}

int gs_backward_gaussians_adam(int P, int D, int M, const float* means3D, const float* shs_dc, const float* shs_rest,
                               const float* scales, float scale_modifier, const float* rotations,
                               const gs_view_grad* view, float* const* params_host, float* const* exp_avg_host,
                               float* const* exp_avg_sq_host, const double* lr_host, const long long* step_host,
                               const double* weight_decay_host, double beta1, double beta2, double eps, int maximize,
                               int debug, void* stream) {
  return gs_backward_gaussians_adam_stats(P, D, M, means3D, shs_dc, shs_rest, scales, scale_modifier, rotations, view,
                                          params_host, exp_avg_host, exp_avg_sq_host, lr_host, step_host,
                                          weight_decay_host, beta1, beta2, eps, maximize, nullptr, nullptr, 0, nullptr,
                                          nullptr, nullptr, debug, stream);
}

int gs_backward_gaussians_adam_stats(int P, int D, int M, const float* means3D, const float* shs_dc,
                                     const float* shs_rest, const float* scales, float scale_modifier,
                                     const float* rotations, const gs_view_grad* view, float* const* params_host,
                                     float* const* exp_avg_host, float* const* exp_avg_sq_host, const double* lr_host,
                                     const long long* step_host, const double* weight_decay_host, double beta1,
                                     double beta2, double eps, int maximize, const int* radii, const float* grad2d,
                                     int grad_stride, float* max_radii2D, float* grad_accum, float* denom, int debug,
                                     void* stream) {
  clear_error(debug);
  if (P < 0) return set_error("P must be >= 0"), 1;
  if (P == 0) return 0;
  if (D < 0 || D > 3 || M != 16) return set_error("fused Adam backward: 16 SH coefficients, degree 0..3 only"), 1;
  if (!means3D || !shs_dc || !shs_rest || !scales || !rotations || !view || !params_host || !exp_avg_host ||
      !exp_avg_sq_host || !lr_host || !step_host)
    return set_error("missing required input pointer"), 1;
  if (!view->viewmatrix || !view->projmatrix || !view->campos || !view->geom_buffer)
    return set_error("view: missing pointer"), 1;
  if (view->image_width <= 0 || view->image_height <= 0) return set_error("view: bad image size"), 1;
  for (int k = 0; k < 6; k++) {
    if (!params_host[k] || !exp_avg_host[k] || !exp_avg_sq_host[k]) return set_error("missing tensor pointer"), 1;
    if (step_host[k] < 1) return set_error("adam: step must be >= 1"), 1;
  }
  if (means3D != params_host[DT_XYZ]) return set_error("means3D must be the xyz parameter (params_host[0])"), 1;
  if (((uintptr_t)params_host[DT_ROT]) & 15) return set_error("rotation parameter must be 16-byte aligned"), 1;
  GaussianArgs g{P, D, M, means3D, shs_dc, nullptr, nullptr, scales, rotations, nullptr, scale_modifier};
  g.shs_rest = shs_rest;
  if ((((uintptr_t)shs_dc) | ((uintptr_t)shs_rest)) & 15) return set_error("split SH rows must be 16-byte aligned"), 1;
  FusedAdamArgs a{};
  for (int k = 0; k < 6; k++) {
    a.p[k] = params_host[k];
    a.m[k] = exp_avg_host[k];
    a.v[k] = exp_avg_sq_host[k];
    adam_scalars(lr_host[k], step_host[k], beta1, beta2, &a.nss[k], &a.bc2s[k]);
    a.wd[k] = weight_decay_host ? (float)weight_decay_host[k] : 0.0f;
  }
  a.k = adam_consts(beta1, beta2, eps, maximize != 0);
  const bool any_stat = radii || grad2d || max_radii2D || grad_accum || denom;
  if (any_stat) {
    if (!radii || !grad2d || !max_radii2D || !grad_accum || !denom)
      return set_error("densify stats: all five pointers or none"), 1;
    if (grad_stride < 2) return set_error("densify stats: grad_stride must be >= 2"), 1;
    a.radii = radii, a.grad2d = grad2d, a.gstride = grad_stride;
    a.max_r = max_radii2D, a.accum = grad_accum, a.denom = denom;
  }
  GeomPtrs geo;
  geom_layout((size_t)P, &geo, (char*)view->geom_buffer);
  a.err = &geo.counters[CNT_ERR];
  CameraArgs c = make_camera(nullptr, view->image_width, view->image_height, view->viewmatrix, view->projmatrix,
                             view->campos, view->tan_fovx, view->tan_fovy, 0);
  bwd_gaussians_adam(g, c, geo, a, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, uint8_t* present,
                    void* stream) {
  clear_error(0);
  if (P < 0) return set_error("P must be >= 0"), 1;
  if (P > 0 && (!means3D || !viewmatrix || !present)) return set_error("missing pointer"), 1;
  mark_visible(P, means3D, viewmatrix, projmatrix, present, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

size_t gs_knn_scratch_bytes(int P) { return knn_scratch_bytes(P); }

int gs_knn_mean_dist2(int P, const float* points, float* out, void* scratch, void* stream) {
  clear_error(0);
  if (P < 0) return set_error("P must be >= 0"), 1;
  if (P == 0) return 0;
  if (!points || !out || !scratch) return set_error("missing pointer"), 1;
  knn_mean_dist2(P, points, out, (char*)scratch, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

unsigned gs_debug_set_scan_spin_limit(unsigned limit) {
  return gs::g_spin_limit.exchange(limit, std::memory_order_relaxed);
}

/* ---- launched-kernel log (tests: every kernel in the code object is launched by some test) ---- */
int gs_debug_launch_log(int enable) {
  const int prev = gs::launch_log_on();
  gs::g_launch_log.store(enable ? 1 : 0, std::memory_order_relaxed);
  return prev;
}

long long gs_debug_launched_kernels(char* buf, long long cap) {
  std::string out;
  {
    std::lock_guard<std::mutex> lk(gs::g_launch_mu);
    for (const void* k : gs::g_launched) {
      Dl_info info;
      if (dladdr(k, &info) && info.dli_sname && info.dli_saddr == k)
        out += info.dli_sname;
      else
        out += "?";
      out += '\n';
    }
  }
  if (buf && cap > (long long)out.size()) memcpy(buf, out.c_str(), out.size() + 1);
  return (long long)out.size();
}

/* ---- numerics mode of the render loops ---- */
int gs_set_exact_exp(int exact) {
  const int prev = exact_exp() ? 1 : 0;
  gs::g_exact_exp.store(exact ? 1 : 0, std::memory_order_relaxed);
  return prev;
}

/* ---- fused SSIM (utils/loss_utils.py:ssim) ---- */
size_t gs_ssim_partial_count(int planes, int H, int W) { return ssim_partial_count(planes, H, W); }

int gs_ssim_forward(int planes, int H, int W, const float* window11_host, const float* img1, const float* img2,
                    float* dmaps, float* partial, float* plane_sum, void* stream) {
  clear_error(0);
  if (planes <= 0 || H <= 0 || W <= 0) return set_error("ssim: empty image"), 1;
  if (!window11_host || !img1 || !img2 || !dmaps || !partial || !plane_sum) return set_error("ssim: missing pointer"), 1;
  ssim_forward(planes, H, W, window11_host, img1, img2, dmaps, partial, plane_sum, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_ssim_backward(int planes, int channels, int H, int W, const float* window11_host, const float* img1,
                     const float* img2, const float* dmaps, const float* scale, float* dimg1, void* stream) {
  clear_error(0);
  if (planes <= 0 || H <= 0 || W <= 0 || channels <= 0 || planes % channels) return set_error("ssim: bad shape"), 1;
  if (!window11_host || !img1 || !img2 || !dmaps || !scale || !dimg1) return set_error("ssim: missing pointer"), 1;
  ssim_backward(planes, channels, H, W, window11_host, img1, img2, dmaps, scale, dimg1, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

/* ---- fused photometric loss (train.py:91-92) ---- */
int gs_photometric_loss_forward(int planes, int H, int W, const float* window11_host, const float* img,
                                const float* gt, float lambda_dssim, float* dmaps, float* partial, float* out3,
                                void* stream) {
  clear_error(0);
  if (planes <= 0 || H <= 0 || W <= 0) return set_error("photometric loss: empty image"), 1;
  if (!window11_host || !img || !gt || !dmaps || !partial || !out3)
    return set_error("photometric loss: missing pointer"), 1;
  photometric_forward(planes, H, W, window11_host, img, gt, lambda_dssim, dmaps, partial, out3, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_photometric_loss_backward(int planes, int H, int W, const float* window11_host, const float* img,
                                 const float* gt, const float* dmaps, float lambda_dssim, const float* grad,
                                 float* dimg, void* stream) {
  clear_error(0);
  if (planes <= 0 || H <= 0 || W <= 0) return set_error("photometric loss: empty image"), 1;
  if (!window11_host || !img || !gt || !dmaps || !grad || !dimg)
    return set_error("photometric loss: missing pointer"), 1;
  photometric_backward(planes, H, W, window11_host, img, gt, dmaps, lambda_dssim, grad, dimg, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

/* ---- fused optimizer step and densification statistics (train.py:114-124) ---- */
int gs_adam_step(int count, float* const* params_host, const float* const* grads_host, float* const* exp_avg_host,
                 float* const* exp_avg_sq_host, const long long* numel_host, const double* lr_host,
                 const long long* step_host, const double* weight_decay_host, double beta1, double beta2, double eps,
                 int maximize, void* stream) {
  clear_error(0);
  if (count < 0) return set_error("adam: count must be >= 0"), 1;
  if (count == 0) return 0;
  if (!params_host || !grads_host || !exp_avg_host || !exp_avg_sq_host || !numel_host || !lr_host || !step_host)
    return set_error("adam: missing pointer"), 1;
  for (int k = 0; k < count; k++) {
    if (numel_host[k] > 0 && (!params_host[k] || !grads_host[k] || !exp_avg_host[k] || !exp_avg_sq_host[k]))
      return set_error("adam: missing tensor pointer"), 1;
    if (step_host[k] < 1) return set_error("adam: step must be >= 1"), 1;
  }
  adam_step(count, params_host, grads_host, exp_avg_host, exp_avg_sq_host, numel_host, lr_host, step_host,
            weight_decay_host, beta1, beta2, eps, maximize != 0, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_adam_step_activated(int count, float* const* params_host, const float* const* grad_src_host,
                           const int* grad_mode_host, int sh_coeffs, float* const* exp_avg_host,
                           float* const* exp_avg_sq_host, const long long* numel_host, const double* lr_host,
                           const long long* step_host, const double* weight_decay_host, double beta1, double beta2,
                           double eps, int maximize, void* stream) {
  clear_error(0);
  if (count < 0) return set_error("adam: count must be >= 0"), 1;
  if (count == 0) return 0;
  if (!params_host || !grad_src_host || !grad_mode_host || !exp_avg_host || !exp_avg_sq_host || !numel_host ||
      !lr_host || !step_host)
    return set_error("adam: missing pointer"), 1;
  for (int k = 0; k < count; k++) {
    const long long n = numel_host[k];
    const int md = grad_mode_host[k];
    if (md < AG_PLAIN || md > AG_NORMALIZE) return set_error("adam: unknown gradient mode %d", md), 1;
    if (n > 0 && (!params_host[k] || !grad_src_host[k] || !exp_avg_host[k] || !exp_avg_sq_host[k]))
      return set_error("adam: missing tensor pointer"), 1;
    if (step_host[k] < 1) return set_error("adam: step must be >= 1"), 1;
    if ((md == AG_SH_DC || md == AG_SH_REST) && sh_coeffs < 1) return set_error("adam: sh_coeffs must be >= 1"), 1;
    if (md == AG_SH_DC && n % 3) return set_error("adam: features_dc must have 3 floats per Gaussian"), 1;
    if (md == AG_SH_REST && (sh_coeffs < 2 ? n != 0 : n % (3LL * (sh_coeffs - 1))))
      return set_error("adam: features_rest must have 3 (sh_coeffs - 1) floats per Gaussian"), 1;
    if ((md == AG_SH_DC || md == AG_SH_REST) && n >= (1LL << 32)) return set_error("adam: SH tensor too large"), 1;
    if (md == AG_NORMALIZE && (n % 4 || ((uintptr_t)grad_src_host[k] & 15)))
      return set_error("adam: rotation rows of 4 floats with a 16-byte aligned gradient source required"), 1;
  }
  adam_step(count, params_host, grad_src_host, exp_avg_host, exp_avg_sq_host, numel_host, lr_host, step_host,
            weight_decay_host, beta1, beta2, eps, maximize != 0, (hipStream_t)stream, grad_mode_host, sh_coeffs);
  return t_failed ? 1 : 0;
}

int gs_activate_forward(int P, int sh_rest, const float* features_dc, const float* features_rest,
                        const float* opacity_raw, const float* scaling_raw, const float* rotation_raw, float* shs,
                        float* opacity, float* scales, float* rotations, void* stream) {
  clear_error(0);
  if (P < 0 || sh_rest < 0) return set_error("activate: P and sh_rest must be >= 0"), 1;
  if (P == 0) return 0;
  // shs may be null: only opacity / scales / rotations are activated (split-SH rasterizer inputs)
  if ((shs && (!features_dc || (sh_rest && !features_rest))) || !opacity_raw || !scaling_raw || !rotation_raw ||
      !opacity || !scales || !rotations)
    return set_error("activate: missing pointer"), 1;
  if (((uintptr_t)rotation_raw | (uintptr_t)rotations | (uintptr_t)shs) & 15)
    return set_error("activate: rotation / shs buffers must be 16-byte aligned"), 1;
  activate_forward(P, sh_rest, features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw, shs, opacity,
                   scales, rotations, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_activate_backward(int P, int sh_rest, const float* dL_dshs, const float* dL_dopacity, const float* dL_dscales,
                         const float* dL_drotations, const float* opacity, const float* scales,
                         const float* rotation_raw, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
                         float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw, void* stream) {
  clear_error(0);
  if (P < 0 || sh_rest < 0) return set_error("activate: P and sh_rest must be >= 0"), 1;
  if (P == 0) return 0;
  if ((dL_dshs && (!dL_dfeatures_dc || (sh_rest && !dL_dfeatures_rest))) ||
      (dL_dopacity && (!opacity || !dL_dopacity_raw)) || (dL_dscales && (!scales || !dL_dscaling_raw)) ||
      (dL_drotations && (!rotation_raw || !dL_drotation_raw)))
    return set_error("activate: missing pointer"), 1;
  if (((uintptr_t)dL_dshs | (uintptr_t)dL_drotations | (uintptr_t)rotation_raw | (uintptr_t)dL_drotation_raw) & 15)
    return set_error("activate: rotation / shs buffers must be 16-byte aligned"), 1;
  activate_backward(P, sh_rest, dL_dshs, dL_dopacity, dL_dscales, dL_drotations, opacity, scales, rotation_raw,
                    dL_dfeatures_dc, dL_dfeatures_rest, dL_dopacity_raw, dL_dscaling_raw, dL_drotation_raw,
                    (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

/* ---- densify_and_prune (gaussian_model.py:391-403) ---- */
static DensifyParams make_dens_params(double grad_threshold, double pd_extent, double min_opacity, double big_extent,
                                      int has_screen, double max_screen, int N) {
  DensifyParams dp;
  dp.thr = (float)grad_threshold;
  dp.pd_ext = (float)pd_extent;
  dp.min_op = (float)min_opacity;
  dp.big_ext = (float)big_extent;
  dp.max_screen = (float)max_screen;
  dp.inv_split = 1.0f / (float)(0.8 * N);
  dp.screen = has_screen ? 1 : 0;
  return dp;
}

size_t gs_densify_block_count(int P) { return P > 0 ? (size_t)((P + 255) / 256) : 0; }

int gs_densify_classify(int P, const float* grad_accum, const float* denom, const float* opacity_raw,
                        const float* scaling_raw, double grad_threshold, double pd_extent, double min_opacity,
                        double big_extent, int has_screen, double max_screen, int N, uint8_t* flags,
                        uint32_t* block_counts, uint32_t* totals, void* stream) {
  clear_error(0);
  if (P <= 0 || N < 1) return set_error("densify: P must be > 0 and N >= 1"), 1;
  if (!grad_accum || !denom || !opacity_raw || !scaling_raw || !flags || !block_counts || !totals)
    return set_error("densify: missing pointer"), 1;
  const DensifyParams dp = make_dens_params(grad_threshold, pd_extent, min_opacity, big_extent, has_screen,
                                            max_screen, N);
  densify_classify(P, dp, grad_accum, denom, opacity_raw, scaling_raw, flags, block_counts, totals,
                   (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_densify_split_stds(int P, int N, const uint32_t* totals_host, const uint8_t* flags,
                          const uint32_t* block_counts, const float* scaling_raw, float* stds, void* stream) {
  clear_error(0);
  if (P <= 0 || N < 1 || !totals_host) return set_error("densify: bad arguments"), 1;
  if (totals_host[2] == 0) return 0;
  if (!flags || !block_counts || !scaling_raw || !stds) return set_error("densify: missing pointer"), 1;
  densify_stds(P, N, totals_host[2], flags, block_counts, scaling_raw, stds, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_densify_emit(int P, int N, const uint32_t* totals_host, const uint8_t* flags, const uint32_t* block_counts,
                    const float* samples, const float* const* params_host, const float* const* exp_avg_host,
                    const float* const* exp_avg_sq_host, float* const* out_params_host,
                    float* const* out_exp_avg_host, float* const* out_exp_avg_sq_host, const int* widths_host,
                    void* stream) {
  clear_error(0);
  if (P <= 0 || N < 1 || !totals_host || !flags || !block_counts || !params_host || !out_params_host || !widths_host)
    return set_error("densify: missing argument"), 1;
  if (totals_host[2] && !samples) return set_error("densify: split samples missing"), 1;
  if (widths_host[DT_XYZ] != 3 || widths_host[DT_FDC] != 3 || widths_host[DT_OPACITY] != 1 ||
      widths_host[DT_SCALING] != 3 || widths_host[DT_ROT] != 4 || widths_host[DT_FREST] < 0)
    return set_error("densify: row widths must be xyz 3, f_dc 3, f_rest 3K, opacity 1, scaling 3, rotation 4"), 1;
  DensTensors t;
  for (int q = 0; q < DENS_TENSORS; q++) {
    t.src[q] = params_host[q];
    t.dst[q] = out_params_host[q];
    t.width[q] = widths_host[q];
    const bool has_m = exp_avg_host && exp_avg_host[q];
    if (has_m && (!exp_avg_sq_host || !exp_avg_sq_host[q] || !out_exp_avg_host || !out_exp_avg_host[q] ||
                  !out_exp_avg_sq_host || !out_exp_avg_sq_host[q]))
      return set_error("densify: incomplete optimizer state pointers"), 1;
    t.m_src[q] = has_m ? exp_avg_host[q] : nullptr;
    t.v_src[q] = has_m ? exp_avg_sq_host[q] : nullptr;
    t.m_dst[q] = has_m ? out_exp_avg_host[q] : nullptr;
    t.v_dst[q] = has_m ? out_exp_avg_sq_host[q] : nullptr;
    if ((!t.src[q] || !t.dst[q]) && t.width[q] > 0) return set_error("densify: missing parameter pointer"), 1;
  }
  DensCounts n{totals_host[0], totals_host[1], totals_host[2], totals_host[3]};
  const DensifyParams dp = make_dens_params(0, 0, 0, 0, 0, 0, N);
  densify_emit(P, N, dp, n, flags, block_counts, samples, t, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_densify_stats(int P, const int* radii, const float* grad2d, int grad_stride, float* max_radii2D,
                     float* grad_accum, float* denom, void* stream) {
  clear_error(0);
  if (P < 0) return set_error("densify_stats: P must be >= 0"), 1;
  if (P == 0) return 0;
  if (grad_stride < 2) return set_error("densify_stats: grad_stride must be >= 2"), 1;
  if (!radii || !grad2d || !max_radii2D || !grad_accum || !denom) return set_error("densify_stats: missing pointer"), 1;
  densify_stats(P, radii, grad2d, grad_stride, max_radii2D, grad_accum, denom, (hipStream_t)stream);
  return t_failed ? 1 : 0;
}

int gs_debug_export(int P, int W, int H, long long num_rendered, const void* geom_buffer, const void* binning_buffer,
                    const void* image_buffer, uint32_t* point_list, uint32_t* ranges, float* xy, float* conic_opacity,
                    float* rgb, float* depth, uint32_t* tiles_touched, float* final_T, uint32_t* n_contrib,
                    void* stream) {
  clear_error(0);
  hipStream_t st = (hipStream_t)stream;
  const int gx = (W + GS_TILE - 1) / GS_TILE, gy = (H + GS_TILE - 1) / GS_TILE;
  if (P <= 0) return 0;
  GeomPtrs geo;
  BinPtrs bin;
  ImgPtrs img;
  geom_layout((size_t)P, &geo, (char*)geom_buffer);
  bin_layout((size_t)num_rendered, gx * gy, &bin, (char*)binning_buffer);
  img_layout(W, H, &img, (char*)image_buffer);
  if (point_list && num_rendered > 0)
    GS_LAUNCH("export_list", k_export_list, dim3((unsigned)((num_rendered + 255) / 256)), dim3(256), 0, st,
              (uint32_t)num_rendered, geo.counters, bin.point_list, bin.presort_gid,
              point_list);
  if (ranges) check_hip(hipMemcpyAsync(ranges, img.ranges, sizeof(uint2) * gx * gy, hipMemcpyDeviceToDevice, st), "copy");
  if (xy || conic_opacity || rgb || depth)
    GS_LAUNCH("export_splat", k_export_splat, dim3((P + 255) / 256), dim3(256), 0, st, P, geo.splat, xy, conic_opacity,
              rgb, depth);
  if (tiles_touched)
    check_hip(hipMemcpyAsync(tiles_touched, geo.tiles, sizeof(uint32_t) * P, hipMemcpyDeviceToDevice, st), "copy");
  if (final_T)
    check_hip(hipMemcpyAsync(final_T, img.final_T, sizeof(float) * W * H, hipMemcpyDeviceToDevice, st), "copy");
  if (n_contrib)
    check_hip(hipMemcpyAsync(n_contrib, img.n_contrib, sizeof(uint32_t) * W * H, hipMemcpyDeviceToDevice, st), "copy");
  return t_failed ? 1 : 0;
}

int gs_debug_export_slots(int W, int H, long long num_rendered, const void* binning_buffer, const void* image_buffer,
                          uint32_t* slots, uint32_t* tile_cut, void* stream) {
  clear_error(0);
  hipStream_t st = (hipStream_t)stream;
  if (W <= 0 || H <= 0 || num_rendered < 0) return set_error("debug_export_slots: bad arguments"), 1;
  const int gx = (W + GS_TILE - 1) / GS_TILE, gy = (H + GS_TILE - 1) / GS_TILE;
  BinPtrs bin;
  ImgPtrs img;
  bin_layout((size_t)num_rendered, gx * gy, &bin, (char*)binning_buffer);
  img_layout(W, H, &img, (char*)image_buffer);
  if (slots && num_rendered > 0)
    check_hip(hipMemcpyAsync(slots, bin.point_list, sizeof(uint32_t) * (size_t)num_rendered, hipMemcpyDeviceToDevice,
                             st), "copy");
  if (tile_cut)
    check_hip(hipMemcpyAsync(tile_cut, img.tile_cut, sizeof(uint32_t) * (size_t)gx * gy, hipMemcpyDeviceToDevice, st),
              "copy");
  return t_failed ? 1 : 0;
}

void gs_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_on = on != 0;
}

int gs_profile_collect(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  int n = 0;
  for (Pending& p : g_pending) {
    if (!p.b) continue;
    (void)hipEventSynchronize(p.b);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      bool found = false;
      for (ProfEntry& e : g_stats)
        if (e.name == p.name) {
          e.ms += ms;
          e.n += 1;
          found = true;
          break;
        }
      if (!found) g_stats.push_back(ProfEntry{p.name, (double)ms, 1});
      n++;
    }
    g_pool.push_back(p.a);
    g_pool.push_back(p.b);
  }
  g_pending.clear();
  return n;
}

void gs_profile_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_stats.clear();
}

int gs_profile_stat(int i, char* name, int name_len, double* total_ms, long long* launches) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (i < 0 || i >= (int)g_stats.size()) return 0;
  if (name && name_len > 0) {
    strncpy(name, g_stats[i].name.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (total_ms) *total_ms = g_stats[i].ms;
  if (launches) *launches = g_stats[i].n;
  return 1;
}

}  // extern "C"
