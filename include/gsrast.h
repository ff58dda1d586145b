/*
 * gsrast.h -- C ABI of the MI355X-native differentiable Gaussian rasterizer (libgsrast.so).
 *
 * Drop-in boundary for the reference's native rasterizer.  The reference binds an un-vendored
 * CUDA/C++ torch extension `diff_gaussian_rasterization._C` (/root/reference/.gitmodules:4-6)
 * through `GaussianRasterizer(...)(...)` at /root/reference/gaussian_renderer/__init__.py:51,85-93
 * (import at :14).  Each entry point below names the upstream native function it replaces
 * (upstream signatures restated in SURVEY.md §8b):
 *
 *   gs_forward_preprocess + gs_forward_render  <-  _C.rasterize_gaussians(...)
 *       (upstream runs both halves in one call with resize callbacks for its three scratch
 *        buffers; here the caller sizes the binning buffer from the returned num_rendered, so no
 *        callback into the host language is needed.  gs_rasterize_forward() is the one-call
 *        variant with the upstream-style allocator callback.)
 *   gs_backward                                <-  _C.rasterize_gaussians_backward(...)
 *   gs_backward_accumulate                     <-  same, adding into caller gradient buffers
 *                                                  (multi-view gradient accumulation; the
 *                                                  reference's `param.grad += g` of autograd,
 *                                                  train.py:93, fused into the last kernel)
 *   gs_mark_visible                            <-  _C.mark_visible(...)
 *   gs_forward_preprocess_views                <-  (extension) the first half of K views' forwards
 *   gs_forward_bounded / gs_bounded_status     <-  (extension) _C.rasterize_gaussians with the
 *                                                  binning buffer sized ahead (no host wait,
 *                                                  HIP-graph capturable)
 *   gs_knn_mean_dist2                          <-  simple_knn._C.distCUDA2(points)
 *                                                  (/root/reference/scene/gaussian_model.py:20,134)
 *   gs_ssim_forward / gs_ssim_backward         <-  utils.loss_utils.ssim(img1, img2)
 *                                                  (/root/reference/utils/loss_utils.py:33-60,
 *                                                   called at train.py:92)
 *   gs_photometric_loss_forward / _backward    <-  train.py:91-92 (l1_loss + ssim, lambda_dssim)
 *   gs_adam_step(_activated)                   <-  torch.optim.Adam.step() of GaussianModel
 *                                                  (/root/reference/scene/gaussian_model.py:163)
 *   gs_densify_stats                           <-  train.py:115-116 / gaussian_model.py:405-407
 *   gs_densify_classify / _split_stds / _emit  <-  GaussianModel.densify_and_prune
 *                                                  (gaussian_model.py:391-403)
 *   gs_activate_forward / gs_activate_backward <-  GaussianModel.get_features / get_opacity /
 *                                                  get_scaling / get_rotation (gaussian_model.py:95-115)
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer (HBM of the current HIP device) unless its name
 *     ends in `_host`.  Arrays are dense row-major fp32 unless stated.  Optional inputs are NULL.
 *   - viewmatrix / projmatrix are the 4x4 `world_view_transform` / `full_proj_transform` tensors
 *     of /root/reference/scene/cameras.py:54-56 (row-vector convention), flattened row-major.
 *   - The caller owns every buffer (the host framework's allocator); the library never allocates
 *     or frees device memory.  Buffers returned by forward must stay alive until backward.
 *   - stream: a hipStream_t; all work is enqueued on it.  gs_forward_preprocess synchronises the
 *     stream once to read num_rendered (as upstream does).
 *   - Return value: 0 on success, non-zero on error; gs_last_error() describes the last error of
 *     the calling thread.  With debug != 0 every kernel is followed by a stream synchronisation
 *     and an error check (upstream `debug` semantics).
 */
#ifndef GSRAST_H
#define GSRAST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSRAST_ABI_VERSION 17  /* v17: gs_geom_flags_offset, gs_forward_order_status, gs_set_row_waits; v16: gs_backward_gaussians_adam_stats (v15: gs_backward_gaussians_adam; v14: gs_forward_counted + gs_binning_layout_count) */

int gs_abi_version(void);
const char* gs_last_error(void);

/* ---- scratch sizing (bytes) ---- */
size_t gs_geom_buffer_bytes(int P);
size_t gs_binning_buffer_bytes(long long num_rendered, int image_width, int image_height);
size_t gs_image_buffer_bytes(int image_width, int image_height);
size_t gs_grad_buffer_bytes(long long num_rendered);
/* The instance count a binning buffer of `bytes` bytes is laid out for: the largest n with
 * gs_binning_buffer_bytes(n, W, H) <= bytes (every such n gives the same layout).  A buffer that
 * gs_forward_counted filled for `capacity` instances goes to the backward with this count in place
 * of num_rendered. */
long long gs_binning_layout_count(size_t bytes, int image_width, int image_height);

/* ---- forward, part 1: preprocess, cull, depth order, instance offsets ----
 * P Gaussians; D = active SH degree; M = SH coefficients per colour (stride of shs, 0 if none).
 * Exactly one of {shs, colors_precomp} and one of {(scales, rotations), cov3D_precomp} is non-NULL.
 * Writes radii_out[P] (int32) and the geometry buffer; returns num_rendered in *num_rendered_host.
 * Ref: upstream rasterize_gaussians (first half: preprocess, InclusiveSum, D2H of num_rendered). */
int gs_forward_preprocess(int P, int D, int M, const float* background, int image_width, int image_height,
                          const float* means3D, const float* shs, const float* colors_precomp,
                          const float* opacities, const float* scales, float scale_modifier,
                          const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                          const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                          int prefiltered, int* radii_out, void* geom_buffer, long long* num_rendered_host,
                          int debug, void* stream);

/* ---- forward, part 1 for K views of one set of Gaussians (1 <= K <= 8, view-parallel steps) ----
 * One preprocess launch projects every Gaussian into the K cameras (its inputs are read from HBM
 * once); view v's radii_out[v] and geom_buffer[v] hold exactly what gs_forward_preprocess writes
 * for that camera.  Then view v's depth order is enqueued on view_streams[v] (NULL: on `stream`)
 * after the preprocess, and one host wait reads the K num_rendered.  Per-view arguments are host
 * arrays of K entries.  Then gs_forward_render per view, on its stream. */
int gs_forward_preprocess_views(int K, int P, int D, int M, const float* const* background, const int* image_width,
                                const int* image_height, const float* means3D, const float* shs,
                                const float* colors_precomp, const float* opacities, const float* scales,
                                float scale_modifier, const float* rotations, const float* cov3D_precomp,
                                const float* const* viewmatrix, const float* const* projmatrix,
                                const float* const* campos, const float* tan_fovx, const float* tan_fovy,
                                int prefiltered, int* const* radii_out, void* const* geom_buffer,
                                long long* num_rendered_host, int debug, void* stream, void* const* view_streams);

/* ---- forward, part 2: duplicate, tile sort, ranges, compositing ----
 * out_color[3, H, W] fp32 (CHW).  binning_buffer >= gs_binning_buffer_bytes(num_rendered, W, H),
 * image_buffer >= gs_image_buffer_bytes(W, H). */
int gs_forward_render(int P, const float* background, int image_width, int image_height,
                      const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                      float tan_fovy, const int* radii, void* geom_buffer, long long num_rendered,
                      void* binning_buffer, void* image_buffer, float* out_color, int debug, void* stream);

/* ---- forward in one call without a host wait (bounded binning buffer) ----
 * Both halves of gs_forward_preprocess + gs_forward_render, enqueued without reading num_rendered
 * back: the caller sizes binning_buffer for `capacity` instances (gs_binning_buffer_bytes(capacity,
 * W, H)) and passes capacity wherever num_rendered goes afterwards (gs_backward*: num_rendered and
 * gs_grad_buffer_bytes).  The instance count on the device drives every kernel, so outputs are
 * bit-identical to the two-call forward whenever the count fits.  A view with more instances than
 * `capacity` (or a prefiltered cull, or a timed-out look-back) leaves a sticky per-device flag, its
 * image and gradients invalid (zero records, nothing composited, every access in bounds): the next
 * gs_forward_bounded fails with the message, and gs_bounded_status reads / clears it.  Nothing
 * here synchronises, records events or allocates, so a step of bounded forwards and their backwards
 * can be captured into a HIP graph.  shs_rest: split SH rows as gs_forward_preprocess_split
 * (shs = features_dc), or NULL. */
int gs_forward_bounded(int P, int D, int M, const float* background, int image_width, int image_height,
                       const float* means3D, const float* shs, const float* shs_rest, const float* colors_precomp,
                       const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                       const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                       const float* campos, float tan_fovx, float tan_fovy, int prefiltered, int* radii_out,
                       void* geom_buffer, long long capacity, void* binning_buffer, void* image_buffer,
                       float* out_color, int debug, void* stream);
/* ---- forward in one call, count read back at the end (ABI 14) ----
 * _C.rasterize_gaussians' eager path without the mid-call host wait of gs_forward_preprocess: the
 * caller sizes binning_buffer for an estimate `capacity` (gs_binning_buffer_bytes(capacity, W, H)),
 * every launch is queued, then the call waits for the instance count -- stored into pinned memory by
 * the first depth-sort launch, so by then normally long written -- and returns it in
 * *num_rendered_host (exact, as upstream's num_rendered).
 *   0: the count fitted.  The binning buffer is laid out for `capacity` instances: the backward takes
 *      gs_binning_layout_count(its bytes, W, H) (= capacity) where it takes num_rendered.
 *   2 (GS_COUNT_SHORT): the count exceeds `capacity`; nothing was composited.  radii_out and
 *      geom_buffer are complete: gs_forward_render with a binning buffer for *num_rendered_host
 *      finishes the forward exactly as the two-call path does.
 *   1: error (gs_last_error()), as gs_forward_preprocess.
 * shs_rest: split SH rows as gs_forward_preprocess_split (shs = features_dc), or NULL. */
#define GS_COUNT_SHORT 2
int gs_forward_counted(int P, int D, int M, const float* background, int image_width, int image_height,
                       const float* means3D, const float* shs, const float* shs_rest, const float* colors_precomp,
                       const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                       const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                       const float* campos, float tan_fovx, float tan_fovy, int prefiltered, int* radii_out,
                       void* geom_buffer, long long capacity, void* binning_buffer, void* image_buffer,
                       float* out_color, long long* num_rendered_host, int debug, void* stream);
/* The bounded forms of the two-call forward: gs_forward_preprocess_views without the readback
 * (capacity: K binning capacities; nothing waits), then gs_forward_render_bounded per view with
 * that view's capacity in place of num_rendered.  Same sticky status as gs_forward_bounded. */
int gs_forward_preprocess_views_bounded(int K, int P, int D, int M, const float* const* background,
                                        const int* image_width, const int* image_height, const float* means3D,
                                        const float* shs, const float* colors_precomp, const float* opacities,
                                        const float* scales, float scale_modifier, const float* rotations,
                                        const float* cov3D_precomp, const float* const* viewmatrix,
                                        const float* const* projmatrix, const float* const* campos,
                                        const float* tan_fovx, const float* tan_fovy, int prefiltered,
                                        int* const* radii_out, void* const* geom_buffer, const long long* capacity,
                                        int debug, void* stream, void* const* view_streams);
int gs_forward_render_bounded(int P, const float* background, int image_width, int image_height,
                              const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                              float tan_fovy, const int* radii, void* geom_buffer, long long capacity,
                              void* binning_buffer, void* image_buffer, float* out_color, int debug, void* stream);
/* Flags (*flags: 1 prefiltered cull, 4 look-back timeout, 8 / 16 more instances than 2^31 - 1 /
 * than the capacity) that bounded forwards left on the current device since the last call, with the
 * instance count of a view that raised them (*instances); clears them.  Returns non-zero (message in
 * gs_last_error) when a flag is set.  Only forwards whose kernels have run are seen: call it after
 * a synchronisation point to cover every forward before it. */
int gs_bounded_status(unsigned* flags, long long* instances);
/* (ABI v17) Byte offset, inside a geometry buffer laid out for P Gaussians, of the 32-bit word
 * holding that view's forward error flags (the bits above; 0 for a valid view).  Every kernel of
 * the forward that records an error stores it there, and the backward's record sums and the fused
 * backward + Adam read it (an invalid view adds nothing / is skipped).  A caller copies the word
 * out stream-ordered behind the forward to decide, at its next sync, whether that view's update
 * happened (gs_train_step: the fused step's step counts). */
size_t gs_geom_flags_offset(int P);
/* (ABI v17) The ordering flags of every forward queued on the current device whose render has been
 * queued (read-back forwards: a look-back wait of their sorts that timed out): waits for their
 * render kernels, takes the flags (each forward is reported once) and returns non-zero with the
 * message in gs_last_error when one timed out.  Without this call the next forward or backward
 * reports them; a caller that has already seen a view's flags word name ERR_LOOKBACK consumes the
 * report here, in its own call. */
int gs_forward_order_status(void);
/* (ABI v17) Row waits for the next forward preprocess of the calling thread (any forward entry
 * point: counted, two-call, bounded, split, or the K-view gs_forward_preprocess_views): chunk k
 * covers the Gaussian rows [bounds[k], bounds[k + 1]) (bounds[0] == 0, increasing) and `events[k]`
 * is a hipEvent_t recorded when those rows' inputs are ready (null: none).  The preprocess then
 * launches in row chunks, each behind hipStreamWaitEvent on its chunk's event, so it starts on the
 * first rows while later rows are still being written on another stream -- the all-gather of a
 * sharded optimizer step (gs_view_parallel.ShardedAdam: parameters updated by row chunk).  Outputs
 * are those of the whole-grid launch.  The waits are consumed by that preprocess; n = 0 clears
 * them.  This mirrors no upstream entry point (upstream has no optimizer sharding). */
int gs_set_row_waits(int n, const int* bounds, void* const* events);

/* ---- the binning of K prepared views at once (ABI v11) ----
 * After gs_forward_preprocess_views(_bounded): duplicate + tile sort + tile ranges of all K views as
 * one set of launches on `stream` (each view's count on the device bounds its part), then each view
 * stream waits for them.  Each kind of buffer (geometry, binning, image) must be K slices of one
 * allocation, one stride apart; every binning slice sized for the largest num_rendered[v]
 * (gs_binning_buffer_bytes(max, W, H)), which is then the num_rendered of every view afterwards
 * (gs_forward_render_binned, backward, gs_grad_buffer_bytes).  All views share W x H. */
int gs_forward_bin_views(int K, int P, int image_width, int image_height, void* const* geom_buffer,
                         const long long* num_rendered, void* const* binning_buffer, void* const* image_buffer,
                         int debug, void* stream, void* const* view_streams);
/* The compositing of one binned view (gs_forward_render without its binning); bounded: the view
 * came from gs_forward_preprocess_views_bounded (flags to the sticky status). */
int gs_forward_render_binned(int P, const float* background, int image_width, int image_height,
                             const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                             float tan_fovy, void* geom_buffer, long long num_rendered, void* binning_buffer,
                             void* image_buffer, float* out_color, int bounded, int debug, void* stream);

/* ---- one-call forward with an upstream-style allocator callback ----
 * alloc(ctx, which, bytes) returns a device pointer of >= bytes (which: 0 geometry, 1 binning,
 * 2 image) that stays valid until backward.  Returns num_rendered (>= 0) or -1 on error. */
typedef void* (*gs_alloc_fn)(void* ctx, int which, size_t bytes);
long long gs_rasterize_forward(int P, int D, int M, const float* background, int image_width, int image_height,
                               const float* means3D, const float* shs, const float* colors_precomp,
                               const float* opacities, const float* scales, float scale_modifier,
                               const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                               const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                               int prefiltered, float* out_color, int* radii_out, gs_alloc_fn alloc,
                               void* alloc_ctx, void** geom_out, void** binning_out, void** image_out, int debug,
                               void* stream);

/* ---- backward ----
 * dL_dout_color[3, H, W].  grad_buffer >= gs_grad_buffer_bytes(num_rendered) (scratch).
 * Outputs (P rows each): dL_dmeans2D[P,3] (gradient w.r.t. the NDC projected mean; column 2 = 0),
 * dL_dcolors[P,3], dL_dopacity[P,1], dL_dmeans3D[P,3], dL_dcov3D[P,6], dL_dsh[P,M,3],
 * dL_dscales[P,3], dL_drotations[P,4].  dL_dcolors, dL_dcov3D, dL_dsh, dL_dscales and
 * dL_drotations may be NULL when the matching input was not given (they are then not computed).
 * Ref: upstream rasterize_gaussians_backward. */
int gs_backward(int P, int D, int M, const float* background, int image_width, int image_height,
                const float* means3D, const float* shs, const float* colors_precomp, const float* opacities,
                const float* scales, float scale_modifier, const float* rotations, const float* cov3D_precomp,
                const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                float tan_fovy, const int* radii, const void* geom_buffer, long long num_rendered,
                const void* binning_buffer, const void* image_buffer, const float* dL_dout_color,
                void* grad_buffer, float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                int debug, void* stream);

/* ---- backward, accumulating ----
 * Same arguments and outputs as gs_backward; bit k of `accumulate` (GS_ACC_*) makes output k
 * ADDED to the buffer's current contents (fp32 `old + new`, as autograd's in-place `grad += g`)
 * instead of overwriting it.  Used to sum several views' gradients into one flat gradient
 * bucket with no extra pass over it (view-parallel training).
 * wait_event (hipEvent_t or NULL): the stream waits for it after the per-tile work and before the
 * kernel that writes / adds the gradient outputs, so views rendered on two streams can share one
 * bucket: their forward, sort and tile backward overlap, only the bucket updates are ordered. */
#define GS_ACC_MEANS2D 1u
#define GS_ACC_COLORS 2u
#define GS_ACC_OPACITY 4u
#define GS_ACC_MEANS3D 8u
#define GS_ACC_COV3D 16u
#define GS_ACC_SH 32u
#define GS_ACC_SCALES 64u
#define GS_ACC_ROTATIONS 128u
int gs_backward_accumulate(int P, int D, int M, const float* background, int image_width, int image_height,
                           const float* means3D, const float* shs, const float* colors_precomp,
                           const float* opacities, const float* scales, float scale_modifier,
                           const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                           const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                           const int* radii, const void* geom_buffer, long long num_rendered,
                           const void* binning_buffer, const void* image_buffer, const float* dL_dout_color,
                           void* grad_buffer, float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                           float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                           float* dL_drotations, unsigned accumulate, void* wait_event, int debug, void* stream);

/* ---- split SH rows (ABI v8, an extension beyond upstream) ----
 * render() concatenates GaussianModel's features_dc [P,1,3] and features_rest [P,M-1,3] into shs
 * (gaussian_model.py:99-103) once per iteration.  These variants read the two tensors in place:
 * shs_dc / shs_rest replace shs (SH colours only; M >= 2 is the coefficient count of the
 * concatenation); dL_dsh is still the [P,M,3] gradient of the concatenation (what
 * gs_adam_step_activated's features_dc / features_rest modes read).  Results are bit-identical to
 * gs_forward_preprocess / gs_backward_accumulate on the concatenated rows.  Every other argument as
 * there (no dL_dcolors: SH colours). */
int gs_forward_preprocess_split(int P, int D, int M, const float* background, int image_width, int image_height,
                                const float* means3D, const float* shs_dc, const float* shs_rest,
                                const float* opacities, const float* scales, float scale_modifier,
                                const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                                const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                                int prefiltered, int* radii_out, void* geom_buffer, long long* num_rendered,
                                int debug, void* stream);
int gs_backward_accumulate_split(int P, int D, int M, const float* background, int image_width, int image_height,
                                 const float* means3D, const float* shs_dc, const float* shs_rest,
                                 const float* opacities, const float* scales, float scale_modifier,
                                 const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                                 const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                                 const int* radii, const void* geom_buffer, long long num_rendered,
                                 const void* binning_buffer, const void* image_buffer, const float* dL_dout_color,
                                 void* grad_buffer, float* dL_dmeans2D, float* dL_dopacity, float* dL_dmeans3D,
                                 float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                                 unsigned accumulate, void* wait_event, int debug, void* stream);

/* ---- backward, split for multi-view steps (an extension beyond upstream) ----
 * A view-parallel step renders K views of ONE set of Gaussians into one gradient bucket
 * (DESIGN.md §7).  gs_backward splits into its per-tile half and its per-Gaussian half, and the
 * per-Gaussian half runs once for all K views: every Gaussian's inputs are read and its gradient
 * row written (or added) once instead of K times.  The bucket receives exactly the fp32 sums that
 * K gs_backward_accumulate calls in view order produce.
 *
 * gs_backward_render: the tile pass and the per-Gaussian record sums of one view, kept in that
 *   view's geom_buffer (which must stay alive until gs_backward_gaussians has run), plus that
 *   view's dL_dmeans2D [P,3] (written, or added with GS_ACC_MEANS2D; NULL: not produced).
 *   Arguments as gs_backward.
 * gs_backward_gaussians: views[0 .. num_views) in order (any count: more than 8 run as several
 *   passes); outputs and `accumulate` bits as gs_backward_accumulate (dL_dmeans2D excluded);
 *   wait_event as gs_backward_accumulate. */
typedef struct gs_view_grad {
  const float* viewmatrix; /* 16, device (as the forward's) */
  const float* projmatrix; /* 16, device */
  const float* campos;     /* 3, device (NULL only without SHs) */
  float tan_fovx, tan_fovy;
  int image_width, image_height;
  const void* geom_buffer; /* that view's forward state, after its gs_backward_render */
} gs_view_grad;
int gs_backward_render(int P, int D, int M, const float* background, int image_width, int image_height,
                       const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                       float tan_fovy, const void* geom_buffer, long long num_rendered, const void* binning_buffer,
                       const void* image_buffer, const float* dL_dout_color, void* grad_buffer, float* dL_dmeans2D,
                       unsigned accumulate, int debug, void* stream);
int gs_backward_gaussians(int P, int D, int M, const float* means3D, const float* shs, const float* colors_precomp,
                          const float* scales, float scale_modifier, const float* rotations,
                          const float* cov3D_precomp, int num_views, const gs_view_grad* views, float* dL_dcolors,
                          float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                          float* dL_dscales, float* dL_drotations, unsigned accumulate, void* wait_event, int debug,
                          void* stream);

/* gs_backward_gaussians_range (ABI v9): gs_backward_gaussians for the Gaussians [first, first +
 *   count) of the P only (every pointer is the whole-array one; the views' geom buffers are laid
 *   out for P).  A view-parallel step runs the per-Gaussian half in Gaussian-range chunks and
 *   starts each chunk's gradient all-reduce as soon as that chunk is written (gs_view_parallel
 *   GradBucket chunks); the union of the chunks equals one whole-range call, bit for
 *   bit (every Gaussian's arithmetic is independent of the others). */
int gs_backward_gaussians_range(int P, int first, int count, int D, int M, const float* means3D, const float* shs,
                                const float* colors_precomp, const float* scales, float scale_modifier,
                                const float* rotations, const float* cov3D_precomp, int num_views,
                                const gs_view_grad* views, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                                float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                                unsigned accumulate, void* wait_event, int debug, void* stream);

/* ---- mark_visible: present[P] (uint8 0/1), near-plane test ---- */
int gs_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                    uint8_t* present, void* stream);

/* ---- simple-knn: mean squared distance to the 3 nearest other points ---- */
size_t gs_knn_scratch_bytes(int P);
int gs_knn_mean_dist2(int P, const float* points, float* out, void* scratch, void* stream);

/* ---- launched-kernel log (ABI v15, test support) ----
 * gs_debug_launch_log(enable): record the distinct kernels this library launches from now on (the
 *   initial state comes from GSRAST_LAUNCH_LOG=1); returns the previous state.
 * gs_debug_launched_kernels: the recorded kernels' mangled symbol names (the names of the code
 *   object's kernel descriptors without ".kd"), one per line; returns the text's length and copies it,
 *   NUL-terminated, when buf holds more than that.  tests/test_zz_kernel_coverage.py checks that every
 *   kernel of the code object is launched by some GPU test. */
int gs_debug_launch_log(int enable);
long long gs_debug_launched_kernels(char* buf, long long cap);

/* ---- numerics mode of the render loops (process-wide) ----
 * exact != 0: the render kernels evaluate exp2 with a deterministic polynomial that the CPU oracle
 * mirrors, so the whole forward is bit-identical to the oracle.  exact == 0 (default): the
 * hardware v_exp_f32 (<= 1 ulp); forward images / final_T then match the oracle within float
 * tolerance, with identical integer outputs except near the alpha / T thresholds (tests/
 * test_gpu_parity.py, fast-mode cases).  The initial mode comes from GSRAST_EXACT_EXP=1.
 * Returns the previous mode.  Set it between steps, not while a step is in flight. */
int gs_set_exact_exp(int exact);

/* ---- fused SSIM of the photometric loss  <-  utils/loss_utils.py:ssim (train.py:91-92) ----
 * img1, img2: [planes, H, W] fp32 (planes = images x channels), window11_host: the 11 float32
 * weights of loss_utils.gaussian(11, 1.5) (host memory).  Forward writes per-plane sums of the
 * SSIM map to plane_sum[planes] and the three per-pixel partials to dmaps[3, planes, H, W]
 * (kept for backward); partial has gs_ssim_partial_count(planes, H, W) floats.  Backward writes
 * dimg1 = scale[plane / channels] * dSSIM-sum/dimg1 (scale: device, one per image). */
size_t gs_ssim_partial_count(int planes, int H, int W);
int gs_ssim_forward(int planes, int H, int W, const float* window11_host, const float* img1, const float* img2,
                    float* dmaps, float* partial, float* plane_sum, void* stream);
int gs_ssim_backward(int planes, int channels, int H, int W, const float* window11_host, const float* img1,
                     const float* img2, const float* dmaps, const float* scale, float* dimg1, void* stream);

/* ---- fused photometric loss  <-  train.py:91-92
 *      loss = (1 - lambda) l1_loss(img, gt) + lambda (1 - ssim(img, gt))  (utils/loss_utils.py) ----
 * img, gt: [planes, H, W] fp32.  Forward: one SSIM pass that also sums |img - gt| per tile, then
 * one fixed-order fp64 reduction writing out3 = [loss, l1, ssim] (device floats, means over all
 * planes x H x W elements); dmaps[3, planes, H, W] as gs_ssim_forward; partial holds
 * 2 x gs_ssim_partial_count(planes, H, W) floats.  Backward: dimg = grad[0] x dloss/dimg (grad: the
 * loss's incoming gradient, one device float), the SSIM and L1 terms in one kernel. */
int gs_photometric_loss_forward(int planes, int H, int W, const float* window11_host, const float* img,
                                const float* gt, float lambda_dssim, float* dmaps, float* partial, float* out3,
                                void* stream);
int gs_photometric_loss_backward(int planes, int H, int W, const float* window11_host, const float* img,
                                 const float* gt, const float* dmaps, float lambda_dssim, const float* grad,
                                 float* dimg, void* stream);

/* ---- fused Adam step  <-  torch.optim.Adam.step() of GaussianModel's optimizer
 *      (/root/reference/scene/gaussian_model.py:154-163, stepped at train.py:123-124) ----
 * count parameter tensors, each with its own lr / step (the reference has one tensor per param
 * group, per-group lr from the schedulers).  The pointer/size arrays are HOST arrays of DEVICE
 * pointers; each tensor is dense fp32 with numel elements and p, grad, exp_avg, exp_avg_sq of equal
 * size.  step[k] >= 1 is the step count AFTER this update (torch increments before updating).
 * lr / weight_decay / betas / eps are the Python doubles of the param groups (rounded to float on the
 * way to the device exactly where torch rounds them).  weight_decay_host may be NULL (all zero).
 * amsgrad is not supported (the reference never sets it). */
int gs_adam_step(int count, float* const* params_host, const float* const* grads_host, float* const* exp_avg_host,
                 float* const* exp_avg_sq_host, const long long* numel_host, const double* lr_host,
                 const long long* step_host, const double* weight_decay_host, double beta1, double beta2, double eps,
                 int maximize, void* stream);

/* gs_adam_step whose gradients are formed from the render() inputs' gradients (the adjoint of
 * gs_activate_forward, applied inside the update: the raw-parameter gradients are never stored).
 * grad_mode_host[k] per tensor, with grad_src_host[k] its source:
 *   0 plain: the tensor's own gradient;
 *   1 features_dc, 2 features_rest: rows of dL/dshs [P, sh_coeffs, 3] (coefficient 0 / 1..M-1);
 *   3 sigmoid (opacity): dL/dopacity * (1 - y) * y, y = sigmoid(p) of the raw value before the update;
 *   4 exp (scaling): dL/dscales * exp(p);
 *   5 normalize (rotation, rows of 4): the F.normalize adjoint of dL/drotations at q = p.
 * Same floats as gs_activate_backward followed by gs_adam_step. */
int gs_adam_step_activated(int count, float* const* params_host, const float* const* grad_src_host,
                           const int* grad_mode_host, int sh_coeffs, float* const* exp_avg_host,
                           float* const* exp_avg_sq_host, const long long* numel_host, const double* lr_host,
                           const long long* step_host, const double* weight_decay_host, double beta1, double beta2,
                           double eps, int maximize, void* stream);

/* gs_backward_gaussians_adam (ABI v15): one view's per-Gaussian backward half fused with the Adam
 * step of GaussianModel's six parameter groups (train.py:93 loss.backward() + train.py:123-124
 * optimizer.step() of one iteration, gaussian_model.py:154-163 groups; the opt-in fused train step
 * of gs_train_step).  Call after the view's gs_backward_render (its dL_dmeans2D, which the
 * densification statistics read, comes from there).  Same floats as gs_backward_accumulate_split
 * (accumulate 0) followed by gs_adam_step_activated in the modes plain / features_dc /
 * features_rest / sigmoid / exp / normalize: every Gaussian's parameters and moments are
 * bit-identical to that pair, and no gradient is stored.
 * M == 16 split SH rows (shs_dc / shs_rest 16-byte aligned), active degree D 0..3 (coefficients
 * past it get zero gradients, as in gs_backward_accumulate_split); scales /
 * rotations are the activated render() inputs the forward read, means3D is params_host[0].
 * params / exp_avg / exp_avg_sq: HOST arrays of 6 DEVICE pointers in group order xyz [P,3],
 * f_dc [P,1,3], f_rest [P,15,3], opacity [P,1], scaling [P,3], rotation [P,4] (raw parameters,
 * rotation 16-byte aligned); lr / step / weight_decay per group as gs_adam_step (weight_decay_host
 * may be NULL).  The Adam update runs in place while the kernel reads the parameters: nothing else
 * may read or write them on another stream until the call's work completes.  A view whose forward
 * recorded an error (its geometry buffer's flags: capacity overflow, look-back timeout, culled
 * prefiltered point) is not updated, so a caller may launch this before reading the forward's status
 * and keep its step counts unchanged when that raises. */
int gs_backward_gaussians_adam(int P, int D, int M, const float* means3D, const float* shs_dc, const float* shs_rest,
                               const float* scales, float scale_modifier, const float* rotations,
                               const gs_view_grad* view, float* const* params_host, float* const* exp_avg_host,
                               float* const* exp_avg_sq_host, const double* lr_host, const long long* step_host,
                               const double* weight_decay_host, double beta1, double beta2, double eps, int maximize,
                               int debug, void* stream);

/* gs_backward_gaussians_adam_stats (ABI v16): gs_backward_gaussians_adam plus the view's
 * densification statistics (train.py:115-116, gaussian_model.py:405-407, i.e. gs_densify_stats) in
 * the same pass: for every i with radii[i] > 0, max_radii2D[i] = max(max_radii2D[i], radii[i]),
 * grad_accum[i] += |grad2d[i * grad_stride + 0..1]|, denom[i] += 1 -- the same floats as
 * gs_densify_stats.  grad2d is the view's dL/dmeans2D (its gs_backward_render output, grad_stride
 * >= 2 floats per row), radii the forward's.  The five stats pointers are all given or all NULL (NULL:
 * exactly gs_backward_gaussians_adam).  A view whose forward recorded an error updates neither its
 * parameters nor its statistics. */
int gs_backward_gaussians_adam_stats(int P, int D, int M, const float* means3D, const float* shs_dc,
                                     const float* shs_rest, const float* scales, float scale_modifier,
                                     const float* rotations, const gs_view_grad* view, float* const* params_host,
                                     float* const* exp_avg_host, float* const* exp_avg_sq_host, const double* lr_host,
                                     const long long* step_host, const double* weight_decay_host, double beta1,
                                     double beta2, double eps, int maximize, const int* radii, const float* grad2d,
                                     int grad_stride, float* max_radii2D, float* grad_accum, float* denom, int debug,
                                     void* stream);

/* ---- render() inputs from GaussianModel's raw parameters  <-  get_features / get_opacity /
 *      get_scaling / get_rotation (/root/reference/scene/gaussian_model.py:95-115, read at
 *      gaussian_renderer/__init__.py:53-80) ----
 * Forward: shs[P, 1 + sh_rest/3, 3] = cat(features_dc[P,1,3], features_rest[P,sh_rest/3,3]);
 * opacity[P] = sigmoid(opacity_raw); scales[P,3] = exp(scaling_raw);
 * rotations[P,4] = rotation_raw / max(|rotation_raw|, 1e-12).
 * Backward: the adjoints (any of the four dL_d* inputs may be NULL: its outputs are not written);
 * opacity / scales are the forward OUTPUTS, rotation_raw the forward input.  Rotation and shs
 * buffers must be 16-byte aligned.  shs == NULL (ABI v8): the SH rows are not concatenated (for the
 * split-SH rasterizer entries); features_dc / features_rest are then not read. */
int gs_activate_forward(int P, int sh_rest, const float* features_dc, const float* features_rest,
                        const float* opacity_raw, const float* scaling_raw, const float* rotation_raw, float* shs,
                        float* opacity, float* scales, float* rotations, void* stream);
int gs_activate_backward(int P, int sh_rest, const float* dL_dshs, const float* dL_dopacity, const float* dL_dscales,
                         const float* dL_drotations, const float* opacity, const float* scales,
                         const float* rotation_raw, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
                         float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw, void* stream);

/* ---- densify_and_prune  <-  GaussianModel.densify_and_prune (/root/reference/scene/
 *      gaussian_model.py:391-403 with densify_and_clone :375-389, densify_and_split :348-373,
 *      prune_points :289-305, cat_tensors_to_optimizer :307-326), called at train.py:118-120 ----
 * Three steps with one host read in between (the caller allocates the new tensors):
 *  1. gs_densify_classify: per Gaussian flags[P] (u8) and per-block counts
 *     (block_counts: 4 * gs_densify_block_count(P) u32, scanned in place to block bases);
 *     totals[4] (device) = {kept originals, kept clones, split parents, kept split parents}.
 *     Scalars are the Python values of the reference call (grad_threshold = max_grad,
 *     pd_extent = percent_dense * extent, big_extent = 0.1 * extent, has_screen = bool(max_screen_size)).
 *  2. gs_densify_split_stds (totals copied to the host): stds[N * totals[2], 3] = exp(scaling) of the
 *     split parents in the reference's repeat order; the caller draws
 *     samples = torch.normal(mean=zeros, std=stds) exactly as gaussian_model.py:358-360 does.
 *  3. gs_densify_emit: writes the final rows (P' = totals[0] + totals[1] + N * totals[3]) of the six
 *     parameter tensors in order xyz, f_dc, f_rest, opacity, scaling, rotation (row widths
 *     3, 3, 3K, 1, 3, 4) and of their Adam moments (NULL entries: group without state). */
size_t gs_densify_block_count(int P);
int gs_densify_classify(int P, const float* grad_accum, const float* denom, const float* opacity_raw,
                        const float* scaling_raw, double grad_threshold, double pd_extent, double min_opacity,
                        double big_extent, int has_screen, double max_screen, int N, uint8_t* flags,
                        uint32_t* block_counts, uint32_t* totals, void* stream);
int gs_densify_split_stds(int P, int N, const uint32_t* totals_host, const uint8_t* flags,
                          const uint32_t* block_counts, const float* scaling_raw, float* stds, void* stream);
int gs_densify_emit(int P, int N, const uint32_t* totals_host, const uint8_t* flags, const uint32_t* block_counts,
                    const float* samples, const float* const* params_host, const float* const* exp_avg_host,
                    const float* const* exp_avg_sq_host, float* const* out_params_host,
                    float* const* out_exp_avg_host, float* const* out_exp_avg_sq_host, const int* widths_host,
                    void* stream);

/* ---- densification statistics  <-  train.py:115-116 + GaussianModel.add_densification_stats
 *      (/root/reference/scene/gaussian_model.py:405-407) ----
 * For every i with radii[i] > 0:  max_radii2D[i] = max(max_radii2D[i], radii[i]);
 * grad_accum[i] += |grad2d[i * grad_stride + 0..1]|_2;  denom[i] += 1.  (grad_accum, denom: [P, 1]) */
int gs_densify_stats(int P, const int* radii, const float* grad2d, int grad_stride, float* max_radii2D,
                     float* grad_accum, float* denom, void* stream);

/* ---- debug export of forward intermediates (tests) ----
 * Copies (device -> device) whichever outputs are non-NULL: point_list[num_rendered] (Gaussian ids
 * of the tile-sorted instance list), ranges[tiles*2] (u32), xy[P*2], conic_opacity[P*4],
 * rgb[P*3], depth[P], tiles_touched[P] (u32), final_T[H*W], n_contrib[H*W] (u32). */
int gs_debug_export(int P, int image_width, int image_height, long long num_rendered, const void* geom_buffer,
                    const void* binning_buffer, const void* image_buffer, uint32_t* point_list,
                    uint32_t* ranges, float* xy, float* conic_opacity, float* rgb, float* depth,
                    uint32_t* tiles_touched, float* final_T, uint32_t* n_contrib, void* stream);

/* ---- test hook: spin limit of the offsets scan's look-back waits (process-wide) ----
 * 0 makes every waiting workgroup time out at once: the forward must then fail with
 * "look-back wait timed out" (gs_forward_render).  Returns the previous limit (default 1 << 22). */
unsigned gs_debug_set_scan_spin_limit(unsigned limit);

/* ---- debug export of the raw tile-sorted instance slots (tests) ----
 * slots[num_rendered]: the depth-ordered instance slot of every entry of the tile-sorted list
 * (the backward writes entry k's gradient record at slots[k]); tile_cut[tiles]: 1 + the slot
 * of the last instance each tile's backward walk reaches (valid after a backward).  Within a
 * tile the slots must be strictly increasing (the record cut relies on it). */
int gs_debug_export_slots(int image_width, int image_height, long long num_rendered, const void* binning_buffer,
                          const void* image_buffer, uint32_t* slots, uint32_t* tile_cut, void* stream);

/* ---- per-kernel timing with HIP events on the launch stream (bench / profiling) ----
 * While enabled every launch is bracketed by a hipEvent pair.  gs_profile_collect() waits for the
 * recorded events and folds them into per-kernel totals; gs_profile_stat(i, ...) reads entry i
 * (returns 0 past the end). */
void gs_profile_enable(int on);
int gs_profile_collect(void);
void gs_profile_reset(void);
int gs_profile_stat(int i, char* name, int name_len, double* total_ms, long long* launches);

#ifdef __cplusplus
}
#endif
#endif /* GSRAST_H */
