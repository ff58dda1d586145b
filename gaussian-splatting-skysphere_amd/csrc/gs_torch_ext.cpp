// gs_torch_ext.cpp -- host-side fast path of diff_gaussian_rasterization._C (torch C++ extension).
//
// The upstream package binds its rasterizer through a torch C++ extension (`_C`, un-vendored
// submodule /root/reference/.gitmodules:4-6; entry points restated in SURVEY.md §8b).  This module
// is the same layer for the eager per-call path: argument validation, output / scratch allocation
// from torch's caching allocator and the C-ABI calls of include/gsrast.h, without the Python
// per-argument work of the ctypes bridge (_C.py), which measured 0.41 ms of host time per eager
// fwd+bwd against ~0.17 ms of kernels at C2 (profiles/r03_host_profile_c2.txt).
//
// It does not link libgsrast.so: _native.load() has already loaded it RTLD_GLOBAL, and init()
// resolves the entry points from that one copy (its per-device state -- bounded status, ordering
// flags, numerics mode -- stays shared with the ctypes path).  Same exception texts as _C.py.
// Every call of the training paths goes through here: the eager forward, the bounded forward
// (binning capacity), prepared views, the backward with gradient sinks / a wait event, and the
// split backward halves; the ctypes bridge keeps the debug exports and the want_all backward of the
// upstream-named entry.  The forward reads its instance count back after queueing every launch
// (gs_forward_counted, binning buffer sized from the last count), so neither the device nor the
// host idles across the host round trip that upstream's resize callbacks need between the halves.
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <dlfcn.h>
#include <torch/extension.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "gsrast.h"

namespace {

// the entry points' types come from include/gsrast.h itself, so a signature change there fails this
// build instead of calling the library with the wrong arguments (and init() checks the loaded
// library's ABI version against the header's)
struct Fns {
  decltype(&gs_forward_preprocess) preprocess = nullptr;
  decltype(&gs_forward_preprocess_split) preprocess_split = nullptr;
  decltype(&gs_forward_render) render = nullptr;
  decltype(&gs_forward_counted) counted = nullptr;
  decltype(&gs_forward_render_bounded) render_bounded = nullptr;
  decltype(&gs_forward_bounded) fwd_bounded = nullptr;
  decltype(&gs_forward_preprocess_views) pre_views = nullptr;
  decltype(&gs_forward_preprocess_views_bounded) pre_views_bounded = nullptr;
  decltype(&gs_forward_bin_views) bin_views = nullptr;
  decltype(&gs_forward_render_binned) render_binned = nullptr;
  decltype(&gs_backward_render) bwd_render = nullptr;
  decltype(&gs_backward_accumulate) backward = nullptr;
  decltype(&gs_backward_accumulate_split) backward_split = nullptr;
  decltype(&gs_backward_gaussians_range) bwd_gaussians = nullptr;
  decltype(&gs_geom_buffer_bytes) geom_bytes = nullptr;
  decltype(&gs_binning_buffer_bytes) binning_bytes = nullptr;
  decltype(&gs_image_buffer_bytes) image_bytes = nullptr;
  decltype(&gs_grad_buffer_bytes) grad_bytes = nullptr;
  decltype(&gs_binning_layout_count) layout_count = nullptr;
  decltype(&gs_last_error) last_error = nullptr;
} F;

template <typename T>
void resolve(T& fn, const char* name) {
  fn = reinterpret_cast<T>(dlsym(RTLD_DEFAULT, name));
  TORCH_CHECK(fn, "gs_torch_ext: libgsrast.so symbol ", name, " not found (load the library first)");
}

void init() {
  decltype(&gs_abi_version) abi = nullptr;
  resolve(abi, "gs_abi_version");
  TORCH_CHECK(abi() == GSRAST_ABI_VERSION, "gs_torch_ext: the loaded libgsrast.so has ABI ", abi(),
              ", this extension was built against include/gsrast.h ABI ", GSRAST_ABI_VERSION,
              ": rebuild the extension (setup_ext.py) or the library");
  resolve(F.preprocess, "gs_forward_preprocess");
  resolve(F.preprocess_split, "gs_forward_preprocess_split");
  resolve(F.render, "gs_forward_render");
  resolve(F.counted, "gs_forward_counted");
  resolve(F.render_bounded, "gs_forward_render_bounded");
  resolve(F.fwd_bounded, "gs_forward_bounded");
  resolve(F.pre_views, "gs_forward_preprocess_views");
  resolve(F.pre_views_bounded, "gs_forward_preprocess_views_bounded");
  resolve(F.bin_views, "gs_forward_bin_views");
  resolve(F.render_binned, "gs_forward_render_binned");
  resolve(F.bwd_render, "gs_backward_render");
  resolve(F.backward, "gs_backward_accumulate");
  resolve(F.backward_split, "gs_backward_accumulate_split");
  resolve(F.bwd_gaussians, "gs_backward_gaussians_range");
  resolve(F.geom_bytes, "gs_geom_buffer_bytes");
  resolve(F.binning_bytes, "gs_binning_buffer_bytes");
  resolve(F.image_bytes, "gs_image_buffer_bytes");
  resolve(F.grad_bytes, "gs_grad_buffer_bytes");
  resolve(F.layout_count, "gs_binning_layout_count");
  resolve(F.last_error, "gs_last_error");
}

void check(int rc, const char* what) {
  if (rc != 0) {
    const char* m = F.last_error();
    TORCH_CHECK(false, what, ": ", (m && *m) ? m : "unknown error");
  }
}

void dev_check(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "diff_gaussian_rasterization (MI355X/HIP) needs device tensors; ", name, " is on ",
              t.device().str(), ". There is no CPU rasterizer in the product path.");
}

// _C._f32: contiguous fp32 device tensor, or undefined for an absent / empty input; host_ok: a
// camera-side input of <= 16 floats may come from the host and is copied over
at::Tensor f32(const c10::optional<at::Tensor>& o, const char* name, const c10::Device& dev, bool host_ok = false) {
  if (!o.has_value() || !o->defined() || o->numel() == 0) return at::Tensor();
  at::Tensor t = *o;
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32 (got ", t.scalar_type(), ")");
  if (t.device() != dev) {
    if (host_ok && t.numel() <= 16) {
      t = t.to(dev);
    } else {
      dev_check(t, name);
      TORCH_CHECK(false, name, " is on ", t.device().str(), ", expected ", dev.str());
    }
  }
  return t.contiguous();
}

inline const float* fp(const at::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }
inline void* vp(const at::Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }

// _C._Inputs: validated, contiguous views of one call's tensors
struct Inputs {
  c10::Device dev = c10::Device(c10::kCPU);
  int64_t P = 0, M = 0;
  at::Tensor means3D, bg, colors, opacity, scales, rotations, cov3D, view, proj, sh, campos, sh_rest;

  Inputs(const at::Tensor& background, const at::Tensor& m3, const c10::optional<at::Tensor>& colors_,
         const c10::optional<at::Tensor>& opacity_, const c10::optional<at::Tensor>& scales_,
         const c10::optional<at::Tensor>& rotations_, const c10::optional<at::Tensor>& cov3D_,
         const at::Tensor& viewmatrix, const at::Tensor& projmatrix, const c10::optional<at::Tensor>& sh_,
         const at::Tensor& campos_, bool need_opacity, const c10::optional<at::Tensor>& sh_rest_) {
    TORCH_CHECK(m3.dim() == 2 && m3.size(1) == 3, "means3D must have dimensions (num_points, 3)");
    dev_check(m3, "means3D");
    dev = m3.device();
    P = m3.size(0);
    means3D = f32(m3, "means3D", dev);
    bg = f32(background, "background", dev, true);
    colors = f32(colors_, "colors_precomp", dev);
    opacity = f32(opacity_, "opacities", dev);
    scales = f32(scales_, "scales", dev);
    rotations = f32(rotations_, "rotations", dev);
    cov3D = f32(cov3D_, "cov3D_precomp", dev);
    view = f32(viewmatrix, "viewmatrix", dev, true);
    proj = f32(projmatrix, "projmatrix", dev, true);
    sh = f32(sh_, "sh", dev);
    campos = f32(campos_, "campos", dev, true);
    M = !sh.defined() ? 0 : (sh.dim() == 3 ? sh.size(1) : sh.numel() / std::max<int64_t>(1, 3 * P));
    sh_rest = f32(sh_rest_, "features_rest", dev);
    if (sh_rest.defined()) {
      TORCH_CHECK(sh.defined() && !colors.defined(),
                  "split SH: features_dc and features_rest replace shs (no colors_precomp)");
      TORCH_CHECK(sh.dim() == 3 && sh.size(0) == P && sh.size(1) == 1 && sh.size(2) == 3 && sh_rest.dim() == 3 &&
                      sh_rest.size(0) == P && sh_rest.size(2) == 3,
                  "split SH: expected features_dc [P, 1, 3] and features_rest [P, M - 1, 3]");
      M = 1 + sh_rest.size(1);
    }
    if (P > 0) {
      TORCH_CHECK(!colors.defined() || colors.numel() == 3 * P, "colors_precomp must have shape (P, 3)");
      TORCH_CHECK(!need_opacity || (opacity.defined() && opacity.numel() == P), "opacities must have shape (P, 1)");
    }
  }
};

inline void* stream_of(const c10::Device& dev) { return at::hip::getCurrentHIPStream(dev.index()).stream(); }

// Instance-count estimates per (device, P, W, H): the next forward of that shape sizes its binning
// buffer ahead of its count (gs_forward_counted), so the count is read back once every launch is
// queued instead of between the two halves.  The estimate follows the recent maximum (the counts of
// a training loop's cameras differ view to view): max(count, 0.98 x the previous estimate).  A
// forward whose count outgrew its buffer bins again into one of the exact size (the geometry is
// kept); a shape's first forward, a debug forward and that fallback run the two-call path.  Keyed
// by shape, so a small scene rendered after a large one is not given the large one's buffer.
constexpr int GS_EST_SLOTS = 128;
struct CountEst {
  int64_t P = -1;
  int W = 0, H = 0, dev = -1;
  long long est = 0;
};
std::mutex g_est_mu;
CountEst g_est[GS_EST_SLOTS];
constexpr long long GS_CAP_ROUND = 1 << 16;

int est_slot(int dev, int64_t P, int W, int H) {
  const uint64_t h = (uint64_t)P * 0x9E3779B97F4A7C15ull ^ ((uint64_t)W << 20 | (uint64_t)H << 4 | (uint64_t)dev);
  return (int)((h ^ (h >> 29)) % GS_EST_SLOTS);
}
long long est_get(int dev, int64_t P, int W, int H) {
  std::lock_guard<std::mutex> lk(g_est_mu);
  const CountEst& e = g_est[est_slot(dev, P, W, H)];
  return (e.P == P && e.W == W && e.H == H && e.dev == dev) ? e.est : 0;
}
void est_put(int dev, int64_t P, int W, int H, long long n, bool reset = false) {
  std::lock_guard<std::mutex> lk(g_est_mu);
  CountEst& e = g_est[est_slot(dev, P, W, H)];
  const bool same = e.P == P && e.W == W && e.H == H && e.dev == dev;
  const long long decayed = same && !reset ? e.est - e.est / 50 : 0;
  e.P = P, e.W = W, e.H = H, e.dev = dev;
  e.est = std::max<long long>(n, decayed);
}

long long capacity_for(long long est) {
  const long long want = est + est / 8 + GS_CAP_ROUND;  // +12.5 % and one rounding step of headroom
  const long long cap = (want + GS_CAP_ROUND - 1) / GS_CAP_ROUND * GS_CAP_ROUND;
  return std::min<long long>(cap, (1ll << 31) - 1);
}

// _C.rasterize_gaussians (no prepared view, no capacity): both halves of the forward
py::tuple forward(const at::Tensor& background, const at::Tensor& means3D, const c10::optional<at::Tensor>& colors,
                  const c10::optional<at::Tensor>& opacity, const c10::optional<at::Tensor>& scales,
                  const c10::optional<at::Tensor>& rotations, double scale_modifier,
                  const c10::optional<at::Tensor>& cov3D, const at::Tensor& viewmatrix, const at::Tensor& projmatrix,
                  double tan_fovx, double tan_fovy, int64_t H, int64_t W, const c10::optional<at::Tensor>& sh,
                  int64_t degree, const at::Tensor& campos, bool prefiltered, bool debug,
                  const c10::optional<at::Tensor>& sh_rest) {
  Inputs x(background, means3D, colors, opacity, scales, rotations, cov3D, viewmatrix, projmatrix, sh, campos, true,
           sh_rest);
  const auto u8 = at::TensorOptions().dtype(at::kByte).device(x.dev);
  const auto f32o = at::TensorOptions().dtype(at::kFloat).device(x.dev);
  if (x.P == 0) {
    // upstream: nothing is launched for an empty scene; the image stays all-zero (no background)
    return py::make_tuple(0, at::zeros({3, H, W}, f32o), at::zeros({0}, f32o.dtype(at::kInt)), at::empty({0}, u8),
                          at::empty({0}, u8), at::empty({0}, u8));
  }
  c10::DeviceGuard guard(x.dev);
  void* st = stream_of(x.dev);
  at::Tensor out_color = at::empty({3, H, W}, f32o);
  at::Tensor radii = at::empty({x.P}, f32o.dtype(at::kInt));
  at::Tensor geom = at::empty({(int64_t)F.geom_bytes((int)x.P)}, u8);
  at::Tensor img = at::empty({(int64_t)F.image_bytes((int)W, (int)H)}, u8);
  long long nr = 0;
  const bool split = x.sh_rest.defined();
  const int di = x.dev.index();
  const long long e = est_get(di, x.P, (int)W, (int)H);
  if (e > 0 && !debug) {
    const long long cap = capacity_for(e);
    at::Tensor binning = at::empty({(int64_t)F.binning_bytes(cap, (int)W, (int)H)}, u8);
    const int rc = F.counted((int)x.P, (int)degree, (int)x.M, fp(x.bg), (int)W, (int)H, fp(x.means3D), fp(x.sh),
                             fp(x.sh_rest), fp(x.colors), fp(x.opacity), fp(x.scales), (float)scale_modifier,
                             fp(x.rotations), fp(x.cov3D), fp(x.view), fp(x.proj), fp(x.campos), (float)tan_fovx,
                             (float)tan_fovy, (int)prefiltered, radii.data_ptr<int>(), geom.data_ptr(), cap,
                             binning.data_ptr(), img.data_ptr(), out_color.data_ptr<float>(), &nr, (int)debug, st);
    if (rc != 2) check(rc, "rasterize_gaussians");
    est_put(di, x.P, (int)W, (int)H, nr);
    if (rc == 0) return py::make_tuple((int64_t)nr, out_color, radii, geom, binning, img);
    // (2: more instances than the estimate; radii and geometry are complete, nr exact)
  } else {
    check((split ? F.preprocess_split : F.preprocess)(
              (int)x.P, (int)degree, (int)x.M, fp(x.bg), (int)W, (int)H, fp(x.means3D), fp(x.sh),
              split ? fp(x.sh_rest) : fp(x.colors), fp(x.opacity), fp(x.scales), (float)scale_modifier,
              fp(x.rotations), fp(x.cov3D), fp(x.view), fp(x.proj), fp(x.campos), (float)tan_fovx, (float)tan_fovy,
              (int)prefiltered, radii.data_ptr<int>(), geom.data_ptr(), &nr, (int)debug, st),
          "rasterize_gaussians (preprocess)");
    est_put(di, x.P, (int)W, (int)H, nr);
  }
  at::Tensor binning = at::empty({(int64_t)F.binning_bytes(nr, (int)W, (int)H)}, u8);
  check(F.render((int)x.P, fp(x.bg), (int)W, (int)H, fp(x.view), fp(x.proj), fp(x.campos), (float)tan_fovx,
                 (float)tan_fovy, radii.data_ptr<int>(), geom.data_ptr(), nr, binning.data_ptr(), img.data_ptr(),
                 out_color.data_ptr<float>(), (int)debug, st),
        "rasterize_gaussians (render)");
  return py::make_tuple((int64_t)nr, out_color, radii, geom, binning, img);
}

// _C.rasterize_gaussians with a binning capacity: the whole forward enqueued without a host wait
// (gs_forward_bounded); num_rendered is returned as the capacity
py::tuple forward_bounded(const at::Tensor& background, const at::Tensor& means3D,
                          const c10::optional<at::Tensor>& colors, const c10::optional<at::Tensor>& opacity,
                          const c10::optional<at::Tensor>& scales, const c10::optional<at::Tensor>& rotations,
                          double scale_modifier, const c10::optional<at::Tensor>& cov3D, const at::Tensor& viewmatrix,
                          const at::Tensor& projmatrix, double tan_fovx, double tan_fovy, int64_t H, int64_t W,
                          const c10::optional<at::Tensor>& sh, int64_t degree, const at::Tensor& campos,
                          bool prefiltered, bool debug, const c10::optional<at::Tensor>& sh_rest, int64_t capacity) {
  Inputs x(background, means3D, colors, opacity, scales, rotations, cov3D, viewmatrix, projmatrix, sh, campos, true,
           sh_rest);
  const auto u8 = at::TensorOptions().dtype(at::kByte).device(x.dev);
  const auto f32o = at::TensorOptions().dtype(at::kFloat).device(x.dev);
  if (x.P == 0) {
    return py::make_tuple(0, at::zeros({3, H, W}, f32o), at::zeros({0}, f32o.dtype(at::kInt)), at::empty({0}, u8),
                          at::empty({0}, u8), at::empty({0}, u8));
  }
  c10::DeviceGuard guard(x.dev);
  at::Tensor out_color = at::empty({3, H, W}, f32o);
  at::Tensor radii = at::empty({x.P}, f32o.dtype(at::kInt));
  at::Tensor geom = at::empty({(int64_t)F.geom_bytes((int)x.P)}, u8);
  at::Tensor binning = at::empty({(int64_t)F.binning_bytes((long long)capacity, (int)W, (int)H)}, u8);
  at::Tensor img = at::empty({(int64_t)F.image_bytes((int)W, (int)H)}, u8);
  check(F.fwd_bounded((int)x.P, (int)degree, (int)x.M, fp(x.bg), (int)W, (int)H, fp(x.means3D), fp(x.sh),
                      fp(x.sh_rest), fp(x.colors), fp(x.opacity), fp(x.scales), (float)scale_modifier,
                      fp(x.rotations), fp(x.cov3D), fp(x.view), fp(x.proj), fp(x.campos), (float)tan_fovx,
                      (float)tan_fovy, (int)prefiltered, radii.data_ptr<int>(), geom.data_ptr(), (long long)capacity,
                      binning.data_ptr(), img.data_ptr(), out_color.data_ptr<float>(), (int)debug, stream_of(x.dev)),
        "rasterize_gaussians (bounded)");
  return py::make_tuple(capacity, out_color, radii, geom, binning, img);
}

// _C.binning_layout_count: the instance count the binning buffer is laid out for (R, or the capacity
// of a gs_forward_counted buffer)
long long layout_count(long long R, const at::Tensor& binning, int64_t W, int64_t H) {
  const size_t n = (size_t)binning.numel();
  if (n == F.binning_bytes(R, (int)W, (int)H)) return R;
  const long long L = F.layout_count(n, (int)W, (int)H);
  TORCH_CHECK(L >= R, "binningBuffer (", n, " bytes) is too small for num_rendered = ", R);
  return L;
}

// _C.backward_impl with want_all=False.  sinks: {name: (buffer, accumulate)} -- that gradient is
// written into (accumulate: added to) the caller's buffer, returned in its place (gradient buckets);
// wait_event: a hipEvent_t the stream waits for before the gradient-writing kernel (0: none)
py::tuple backward(const at::Tensor& background, const at::Tensor& means3D, const at::Tensor& radii,
                   const c10::optional<at::Tensor>& colors, const c10::optional<at::Tensor>& scales,
                   const c10::optional<at::Tensor>& rotations, double scale_modifier,
                   const c10::optional<at::Tensor>& cov3D, const at::Tensor& viewmatrix, const at::Tensor& projmatrix,
                   double tan_fovx, double tan_fovy, const at::Tensor& dL_dout_color,
                   const c10::optional<at::Tensor>& sh, int64_t degree, const at::Tensor& campos,
                   const at::Tensor& geom, int64_t R, const at::Tensor& binning, const at::Tensor& img, bool debug,
                   const c10::optional<at::Tensor>& sh_rest, const py::dict& sinks, int64_t wait_event) {
  Inputs x(background, means3D, colors, c10::nullopt, scales, rotations, cov3D, viewmatrix, projmatrix, sh, campos,
           false, sh_rest);
  const int64_t P = x.P, M = x.M;
  const auto f32o = at::TensorOptions().dtype(at::kFloat).device(x.dev);
  const int64_t H = dL_dout_color.size(1), W = dL_dout_color.size(2);
  const bool has_sr = x.scales.defined() && x.rotations.defined() && !x.cov3D.defined();
  const bool need_sr = x.scales.defined() && x.rotations.defined();
  unsigned acc = 0;
  // a computed gradient with a sink goes to the sink's buffer (GS_ACC bit `bit` when accumulating)
  auto sunk = [&](const char* name, int bit, int64_t numel, at::Tensor& out) -> bool {
    if (sinks.empty() || !sinks.contains(name)) return false;
    py::tuple t = sinks[name].cast<py::tuple>();
    at::Tensor buf = t[0].cast<at::Tensor>();
    TORCH_CHECK(buf.scalar_type() == at::kFloat && buf.device() == x.dev && buf.is_contiguous() &&
                    buf.numel() == numel,
                "gradient sink for ", name, ": expected a contiguous float32 buffer of ", numel, " elements on ",
                x.dev.str());
    out = buf;
    if (t[1].cast<bool>()) acc |= 1u << bit;
    return true;
  };
  // upstream order: means2D, colors, opacity, means3D, cov3D, sh, scales, rotations
  at::Tensor g_m2, g_op, g_m3, g_col, g_cov, g_sh, g_sc, g_rot;
  if (!sunk("means2D", 0, 3 * P, g_m2)) g_m2 = at::empty({P, 3}, f32o);
  if (x.colors.defined() && !sunk("colors", 1, 3 * P, g_col)) g_col = at::empty({P, 3}, f32o);
  if (!sunk("opacity", 2, P, g_op)) g_op = at::empty({P, 1}, f32o);
  if (!sunk("means3D", 3, 3 * P, g_m3)) g_m3 = at::empty({P, 3}, f32o);
  if (x.cov3D.defined() && !sunk("cov3D", 4, 6 * P, g_cov)) g_cov = at::empty({P, 6}, f32o);
  if (x.sh.defined() && !sunk("sh", 5, 3 * M * P, g_sh)) g_sh = at::empty({P, M, 3}, f32o);
  if (need_sr) {
    if (!(has_sr && sunk("scales", 6, 3 * P, g_sc))) g_sc = has_sr ? at::empty({P, 3}, f32o) : at::zeros({P, 3}, f32o);
    if (!(has_sr && sunk("rotations", 7, 4 * P, g_rot)))
      g_rot = has_sr ? at::empty({P, 4}, f32o) : at::zeros({P, 4}, f32o);
  }
  auto opt = [](const at::Tensor& t) -> py::object { return t.defined() ? py::cast(t) : py::none(); };
  auto result = [&]() {
    return py::make_tuple(opt(g_m2), opt(g_col), opt(g_op), opt(g_m3), opt(g_cov), opt(g_sh), opt(g_sc), opt(g_rot));
  };
  if (P == 0) return result();
  at::Tensor dpix = f32(dL_dout_color, "dL_dout_color", x.dev);
  c10::DeviceGuard guard(x.dev);
  void* st = stream_of(x.dev);
  R = layout_count((long long)R, binning, W, H);
  at::Tensor scratch = at::empty({(int64_t)F.grad_bytes((long long)R)}, f32o.dtype(at::kByte));
  const at::Tensor sc_out = has_sr ? g_sc : at::Tensor(), rot_out = has_sr ? g_rot : at::Tensor();
  if (x.sh_rest.defined()) {  // split SH rows: SH colours, so no dL/dcolors output
    check(F.backward_split((int)P, (int)degree, (int)M, fp(x.bg), (int)W, (int)H, fp(x.means3D), fp(x.sh),
                           fp(x.sh_rest), fp(x.opacity), fp(x.scales), (float)scale_modifier, fp(x.rotations),
                           fp(x.cov3D), fp(x.view), fp(x.proj), fp(x.campos), (float)tan_fovx, (float)tan_fovy,
                           radii.data_ptr<int>(), geom.data_ptr(), (long long)R, binning.data_ptr(), img.data_ptr(),
                           fp(dpix), scratch.data_ptr(), g_m2.data_ptr<float>(), g_op.data_ptr<float>(),
                           g_m3.data_ptr<float>(), (float*)vp(g_cov), (float*)vp(g_sh), (float*)vp(sc_out),
                           (float*)vp(rot_out), acc, reinterpret_cast<void*>(wait_event), (int)debug, st),
          "rasterize_gaussians_backward");
    return result();
  }
  check(F.backward((int)P, (int)degree, (int)M, fp(x.bg), (int)W, (int)H, fp(x.means3D), fp(x.sh), fp(x.colors),
                   fp(x.opacity), fp(x.scales), (float)scale_modifier, fp(x.rotations), fp(x.cov3D), fp(x.view),
                   fp(x.proj), fp(x.campos), (float)tan_fovx, (float)tan_fovy, radii.data_ptr<int>(), geom.data_ptr(),
                   (long long)R, binning.data_ptr(), img.data_ptr(), fp(dpix), scratch.data_ptr(),
                   g_m2.data_ptr<float>(), (float*)vp(g_col), g_op.data_ptr<float>(), g_m3.data_ptr<float>(),
                   (float*)vp(g_cov), (float*)vp(g_sh), (float*)vp(sc_out), (float*)vp(rot_out), acc,
                   reinterpret_cast<void*>(wait_event), (int)debug, st),
        "rasterize_gaussians_backward");
  return result();
}

// ---- the multi-view path (prepare_views, prepared renders, deferred backwards) ----

// _C.preprocess_views: the first half of K views' forwards in one set of launches, then (same
// image size, GSRAST_BATCH_VIEWS unset or not 0) their binning in one set; per view the tuple
// (num_rendered, radii, geom, bounded[, binning, img]) that _C.rasterize_gaussians(prepared=) takes.
// streams: the views' HIP stream handles (or empty: the current stream); the view's buffers are
// recorded on its stream, as _C.py does.
py::list preprocess_views(const std::vector<at::Tensor>& backgrounds, const at::Tensor& means3D,
                          const c10::optional<at::Tensor>& colors, const c10::optional<at::Tensor>& opacity,
                          const c10::optional<at::Tensor>& scales, const c10::optional<at::Tensor>& rotations,
                          double scale_modifier, const c10::optional<at::Tensor>& cov3D,
                          const std::vector<at::Tensor>& viewmatrices, const std::vector<at::Tensor>& projmatrices,
                          const std::vector<double>& tan_fovx, const std::vector<double>& tan_fovy,
                          const std::vector<int64_t>& heights, const std::vector<int64_t>& widths,
                          const c10::optional<at::Tensor>& sh, int64_t degree, const std::vector<at::Tensor>& campos,
                          bool prefiltered, bool debug, const std::vector<int64_t>& streams,
                          const c10::optional<std::vector<int64_t>>& capacities) {
  const int K = (int)viewmatrices.size();
  TORCH_CHECK(K >= 1 && K <= 8, "preprocess_views: 1 to 8 views per call");
  TORCH_CHECK(backgrounds.size() == (size_t)K && projmatrices.size() == (size_t)K && tan_fovx.size() == (size_t)K &&
                  tan_fovy.size() == (size_t)K && heights.size() == (size_t)K && widths.size() == (size_t)K &&
                  campos.size() == (size_t)K && (streams.empty() || streams.size() == (size_t)K),
              "preprocess_views: one entry per view in every per-view argument");
  Inputs x(backgrounds[0], means3D, colors, opacity, scales, rotations, cov3D, viewmatrices[0], projmatrices[0], sh,
           campos[0], true, c10::nullopt);
  const auto u8 = at::TensorOptions().dtype(at::kByte).device(x.dev);
  const auto i32 = at::TensorOptions().dtype(at::kInt).device(x.dev);
  std::vector<at::Tensor> radii(K), geoms(K), bgs(K), views(K), projs(K), cams(K);
  for (int k = 0; k < K; k++) radii[k] = at::empty({x.P}, i32);
  const int64_t gb = x.P ? (int64_t)F.geom_bytes((int)x.P) : 0;
  at::Tensor geom_all = at::empty({K * gb}, u8);
  for (int k = 0; k < K; k++) geoms[k] = geom_all.narrow(0, k * gb, gb);
  py::list out;
  if (x.P == 0) {
    for (int k = 0; k < K; k++) out.append(py::make_tuple(0, radii[k], geoms[k], false));
    return out;
  }
  TORCH_CHECK(!capacities.has_value() || capacities->size() == (size_t)K, "preprocess_views: one capacity per view");
  for (int k = 0; k < K; k++) {
    bgs[k] = k ? f32(backgrounds[k], "background", x.dev, true) : x.bg;
    views[k] = k ? f32(viewmatrices[k], "viewmatrix", x.dev, true) : x.view;
    projs[k] = k ? f32(projmatrices[k], "projmatrix", x.dev, true) : x.proj;
    cams[k] = k ? f32(campos[k], "campos", x.dev, true) : x.campos;
  }
  c10::DeviceGuard guard(x.dev);
  void* st = stream_of(x.dev);
  const float *bgp[8], *vp_[8], *pp[8], *cp[8];
  int wv[8], hv[8];
  float tx[8], ty[8];
  int* rp[8];
  void *gp[8], *vst[8];
  long long nr[8] = {};
  for (int k = 0; k < K; k++) {
    bgp[k] = fp(bgs[k]), vp_[k] = fp(views[k]), pp[k] = fp(projs[k]), cp[k] = fp(cams[k]);
    wv[k] = (int)widths[k], hv[k] = (int)heights[k], tx[k] = (float)tan_fovx[k], ty[k] = (float)tan_fovy[k];
    rp[k] = radii[k].data_ptr<int>(), gp[k] = geoms[k].data_ptr();
    vst[k] = streams.empty() ? nullptr : reinterpret_cast<void*>(streams[k]);
  }
  const bool bounded = capacities.has_value();
  if (bounded) {
    for (int k = 0; k < K; k++) nr[k] = (*capacities)[k];
    check(F.pre_views_bounded(K, (int)x.P, (int)degree, (int)x.M, bgp, wv, hv, fp(x.means3D), fp(x.sh), fp(x.colors),
                              fp(x.opacity), fp(x.scales), (float)scale_modifier, fp(x.rotations), fp(x.cov3D), vp_, pp,
                              cp, tx, ty, (int)prefiltered, rp, gp, nr, (int)debug, st,
                              streams.empty() ? nullptr : vst),
          "preprocess_views");
  } else {
    check(F.pre_views(K, (int)x.P, (int)degree, (int)x.M, bgp, wv, hv, fp(x.means3D), fp(x.sh), fp(x.colors),
                      fp(x.opacity), fp(x.scales), (float)scale_modifier, fp(x.rotations), fp(x.cov3D), vp_, pp, cp, tx,
                      ty, (int)prefiltered, rp, gp, nr, (int)debug, st, streams.empty() ? nullptr : vst),
          "preprocess_views");
  }
  bool same_size = true;
  for (int k = 1; k < K; k++) same_size = same_size && wv[k] == wv[0] && hv[k] == hv[0];
  static const bool batch = [] {
    const char* e = getenv("GSRAST_BATCH_VIEWS");
    return !(e && e[0] == '0' && e[1] == 0);
  }();
  std::vector<py::tuple> tuples;
  if (batch && same_size) {
    // the K views' binning as one set of launches: every binning buffer a slice of one allocation,
    // sized for the largest count, which then stands for every view's num_rendered
    long long I = 0;
    for (int k = 0; k < K; k++) I = std::max(I, nr[k]);
    const int64_t bb = (int64_t)F.binning_bytes(I, wv[0], hv[0]), ib = (int64_t)F.image_bytes(wv[0], hv[0]);
    at::Tensor bin_all = at::empty({K * bb}, u8), img_all = at::empty({K * ib}, u8);
    void *bp[8], *ip[8];
    std::vector<at::Tensor> bins(K), imgs(K);
    for (int k = 0; k < K; k++) {
      bins[k] = bin_all.narrow(0, k * bb, bb), imgs[k] = img_all.narrow(0, k * ib, ib);
      bp[k] = bins[k].data_ptr(), ip[k] = imgs[k].data_ptr();
    }
    check(F.bin_views(K, (int)x.P, wv[0], hv[0], gp, nr, bp, ip, (int)debug, st, streams.empty() ? nullptr : vst),
          "preprocess_views (binning)");
    for (int k = 0; k < K; k++) tuples.push_back(py::make_tuple((int64_t)I, radii[k], geoms[k], bounded, bins[k], imgs[k]));
    if (!streams.empty())
      for (int k = 0; k < K; k++) {
        // (torch on ROCm keys its HIP streams as CUDA streams)
        const c10::Stream sk =
            at::hip::getStreamFromExternalMasqueradingAsCUDA((hipStream_t)vst[k], x.dev.index()).unwrap();
        radii[k].record_stream(sk), geoms[k].record_stream(sk), bins[k].record_stream(sk), imgs[k].record_stream(sk);
      }
  } else {
    for (int k = 0; k < K; k++) tuples.push_back(py::make_tuple((int64_t)nr[k], radii[k], geoms[k], bounded));
    if (!streams.empty())
      for (int k = 0; k < K; k++) {
        // (torch on ROCm keys its HIP streams as CUDA streams)
        const c10::Stream sk =
            at::hip::getStreamFromExternalMasqueradingAsCUDA((hipStream_t)vst[k], x.dev.index()).unwrap();
        radii[k].record_stream(sk), geoms[k].record_stream(sk);
      }
  }
  for (auto& t : tuples) out.append(t);
  return out;
}

// _C.rasterize_gaussians(prepared=): the rest of a view's forward after preprocess_views
py::tuple forward_prepared(const at::Tensor& background, const at::Tensor& means3D, const at::Tensor& viewmatrix,
                           const at::Tensor& projmatrix, double tan_fovx, double tan_fovy, int64_t H, int64_t W,
                           const at::Tensor& campos, bool debug, const py::tuple& prepared) {
  TORCH_CHECK(means3D.dim() == 2 && means3D.size(1) == 3, "means3D must have dimensions (num_points, 3)");
  dev_check(means3D, "means3D");
  const c10::Device dev = means3D.device();
  const int64_t P = means3D.size(0);
  const auto f32o = at::TensorOptions().dtype(at::kFloat).device(dev);
  const auto u8 = at::TensorOptions().dtype(at::kByte).device(dev);
  const long long nr = prepared[0].cast<long long>();
  at::Tensor radii = prepared[1].cast<at::Tensor>(), geom = prepared[2].cast<at::Tensor>();
  const bool bounded = prepared.size() > 3 && prepared[3].cast<bool>();
  if (P == 0)
    return py::make_tuple(0, at::zeros({3, H, W}, f32o), at::zeros({0}, f32o.dtype(at::kInt)), at::empty({0}, u8),
                          at::empty({0}, u8), at::empty({0}, u8));
  TORCH_CHECK(radii.numel() == P && geom.numel() == (int64_t)F.geom_bytes((int)P),
              "rasterize_gaussians: the prepared view does not match these inputs");
  at::Tensor bg = f32(background, "background", dev, true), view = f32(viewmatrix, "viewmatrix", dev, true);
  at::Tensor proj = f32(projmatrix, "projmatrix", dev, true), cam = f32(campos, "campos", dev, true);
  c10::DeviceGuard guard(dev);
  void* st = stream_of(dev);
  at::Tensor out_color = at::empty({3, H, W}, f32o);
  if (prepared.size() > 4) {  // binned with the other prepared views: the compositing only
    at::Tensor binning = prepared[4].cast<at::Tensor>(), img = prepared[5].cast<at::Tensor>();
    TORCH_CHECK(img.numel() == (int64_t)F.image_bytes((int)W, (int)H),
                "rasterize_gaussians: the prepared view was binned for another image size");
    check(F.render_binned((int)P, fp(bg), (int)W, (int)H, fp(view), fp(proj), fp(cam), (float)tan_fovx,
                          (float)tan_fovy, geom.data_ptr(), nr, binning.data_ptr(), img.data_ptr(),
                          out_color.data_ptr<float>(), (int)bounded, (int)debug, st),
          "rasterize_gaussians (render)");
    return py::make_tuple((int64_t)nr, out_color, radii, geom, binning, img);
  }
  at::Tensor binning = at::empty({(int64_t)F.binning_bytes(nr, (int)W, (int)H)}, u8);
  at::Tensor img = at::empty({(int64_t)F.image_bytes((int)W, (int)H)}, u8);
  check((bounded ? F.render_bounded : F.render)((int)P, fp(bg), (int)W, (int)H, fp(view), fp(proj), fp(cam),
                                                (float)tan_fovx, (float)tan_fovy, radii.data_ptr<int>(),
                                                geom.data_ptr(), nr, binning.data_ptr(), img.data_ptr(),
                                                out_color.data_ptr<float>(), (int)debug, st),
        "rasterize_gaussians (render)");
  return py::make_tuple((int64_t)nr, out_color, radii, geom, binning, img);
}

// _C.backward_render: the per-tile half of one view's backward (its record sums stay in the
// geometry buffer) and its dL_dmeans2D [P, 3] (or None)
py::object backward_render(const at::Tensor& background, const at::Tensor& viewmatrix, const at::Tensor& projmatrix,
                           const at::Tensor& campos, double tan_fovx, double tan_fovy, const at::Tensor& dL_dout_color,
                           int64_t P, int64_t degree, int64_t M, const at::Tensor& geom, int64_t R,
                           const at::Tensor& binning, const at::Tensor& img, bool want_means2D, bool debug) {
  const c10::Device dev = geom.device();
  const int64_t H = dL_dout_color.size(1), W = dL_dout_color.size(2);
  const auto f32o = at::TensorOptions().dtype(at::kFloat).device(dev);
  at::Tensor dm2 = want_means2D ? at::empty({P, 3}, f32o) : at::Tensor();
  auto ret = [&]() -> py::object { return dm2.defined() ? py::cast(dm2) : py::none(); };
  if (P == 0) return ret();
  at::Tensor bg = f32(background, "background", dev, true), view = f32(viewmatrix, "viewmatrix", dev, true);
  at::Tensor proj = f32(projmatrix, "projmatrix", dev, true), cam = f32(campos, "campos", dev, true);
  at::Tensor dpix = f32(dL_dout_color, "dL_dout_color", dev);
  R = layout_count((long long)R, binning, W, H);
  c10::DeviceGuard guard(dev);
  void* st = stream_of(dev);
  at::Tensor scratch = at::empty({(int64_t)F.grad_bytes((long long)R)}, f32o.dtype(at::kByte));
  check(F.bwd_render((int)P, (int)degree, (int)M, fp(bg), (int)W, (int)H, fp(view), fp(proj), fp(cam),
                     (float)tan_fovx, (float)tan_fovy, geom.data_ptr(), (long long)R, binning.data_ptr(),
                     img.data_ptr(), fp(dpix), scratch.data_ptr(), dm2.defined() ? dm2.data_ptr<float>() : nullptr, 0u,
                     (int)debug, st),
        "rasterize_gaussians_backward (render half)");
  return ret();
}

// the estimate the next forward of this shape sizes its binning buffer from (tests; 0: none yet,
// the two-call path); set_count_estimate replaces it (0: forget it)
long long count_estimate(int64_t device, int64_t P, int64_t W, int64_t H) {
  return est_get((int)device, P, (int)W, (int)H);
}
// _C.backward_gaussians: the per-Gaussian half of the backward for several views at once.
// views: [(viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, W, H, geomBuffer)]; outs: {name:
// buffer}; wait_event: a hipEvent_t handle (0: none); count < 0: the Gaussians [first, P)
void backward_gaussians(const at::Tensor& means3D, const c10::optional<at::Tensor>& sh,
                        const c10::optional<at::Tensor>& colors, const c10::optional<at::Tensor>& scales,
                        const c10::optional<at::Tensor>& rotations, const c10::optional<at::Tensor>& cov3D,
                        double scale_modifier, int64_t degree, const py::list& views, const py::dict& outs,
                        int64_t accumulate, int64_t wait_event, bool debug, int64_t first, int64_t count) {
  Inputs x(at::Tensor(), means3D, colors, c10::nullopt, scales, rotations, cov3D, at::Tensor(), at::Tensor(), sh,
           at::Tensor(), false, c10::nullopt);
  const int K = (int)views.size();
  if (x.P == 0 || K == 0) return;
  std::vector<at::Tensor> keep;
  keep.reserve(3 * K);
  std::vector<gs_view_grad> arr(K);
  for (int k = 0; k < K; k++) {
    const py::tuple v = views[k].cast<py::tuple>();
    TORCH_CHECK(v.size() == 8, "backward_gaussians: a view is (viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, "
                               "W, H, geomBuffer)");
    at::Tensor vm = f32(v[0].cast<at::Tensor>(), "viewmatrix", x.dev, true);
    at::Tensor pm = f32(v[1].cast<at::Tensor>(), "projmatrix", x.dev, true);
    at::Tensor cp = v[2].is_none() ? at::Tensor() : f32(v[2].cast<at::Tensor>(), "campos", x.dev, true);
    keep.push_back(vm), keep.push_back(pm), keep.push_back(cp);
    arr[k] = gs_view_grad{fp(vm), fp(pm), fp(cp), (float)v[3].cast<double>(), (float)v[4].cast<double>(),
                          v[5].cast<int>(), v[6].cast<int>(), v[7].cast<at::Tensor>().data_ptr()};
  }
  auto out = [&](const char* n) -> float* {
    if (!outs.contains(n)) return nullptr;
    const py::object o = outs[n];
    if (o.is_none()) return nullptr;
    const at::Tensor t = o.cast<at::Tensor>();
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.device() == x.dev, "backward_gaussians: ", n,
                " output must be a contiguous float32 tensor on ", x.dev.str());
    return t.data_ptr<float>();
  };
  float *o_col = out("colors"), *o_op = out("opacity"), *o_m3 = out("means3D"), *o_cov = out("cov3D");
  float *o_sh = out("sh"), *o_sc = out("scales"), *o_rot = out("rotations");
  const int64_t n = count < 0 ? x.P - first : count;
  c10::DeviceGuard guard(x.dev);
  check(F.bwd_gaussians((int)x.P, (int)first, (int)n, (int)degree, (int)x.M, fp(x.means3D), fp(x.sh), fp(x.colors),
                        fp(x.scales), (float)scale_modifier, fp(x.rotations), fp(x.cov3D), K, arr.data(), o_col, o_op,
                        o_m3, o_cov, o_sh, o_sc, o_rot, (unsigned)accumulate, reinterpret_cast<void*>(wait_event),
                        (int)debug, stream_of(x.dev)),
        "rasterize_gaussians_backward (per-Gaussian half)");
}

void set_count_estimate(int64_t device, int64_t P, int64_t W, int64_t H, long long n) {
  est_put((int)device, P, (int)W, (int)H, std::max<long long>(n, 0), true);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "host fast path of diff_gaussian_rasterization._C over libgsrast.so (see gs_torch_ext.cpp)";
  m.def("init", &init);
  m.def("forward", &forward);
  m.def("forward_bounded", &forward_bounded);
  m.def("backward", &backward);
  m.def("preprocess_views", &preprocess_views);
  m.def("forward_prepared", &forward_prepared);
  m.def("backward_render", &backward_render);
  m.def("backward_gaussians", &backward_gaussians);
  m.def("count_estimate", &count_estimate);
  m.def("set_count_estimate", &set_count_estimate);
}
