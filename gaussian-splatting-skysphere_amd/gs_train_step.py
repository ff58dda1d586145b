"""One train.py iteration on MI355X, end to end (SURVEY.md §8d metric (2)).

`train_step` runs the per-iteration sequence of /root/reference/train.py:86-128 for one view:
  render()                      gaussian_renderer/__init__.py:18-100 (activations, screen-space
                                carrier, GaussianRasterizer forward)
  loss = (1 - l) L1 + l (1 - SSIM)                     train.py:91-92 (lambda_dssim 0.2)
  loss.backward()                                      train.py:93
  max_radii2D / add_densification_stats               train.py:115-116
  densify_and_prune (`densify`; the caller runs it every 100 iterations)  train.py:118-120
  optimizer.step(); zero_grad(set_to_none=True)        train.py:127-128
with this package's HIP paths for every part: gs_train.render_inputs (one activation launch each
way; by default the backward's activation adjoint runs inside the Adam update,
FusedAdam.step_activated), the rasterizer, gs_loss.photometric_loss (L1 + SSIM in one forward and
one backward kernel), gs_train.add_densification_stats, FusedAdam, gs_train.densify_and_prune.  `fused=False`
keeps the rasterizer and the SSIM kernels but runs the reference's own torch glue for
activations, the L1 term and the loss expression, densification statistics and Adam (the
comparison point for the fused glue).

`TrainModel` holds the GaussianModel fields one iteration touches (scene/gaussian_model.py:44-61,
149-163): the six raw parameters, their Adam groups with training_setup's learning rates, the
densification statistics, percent_dense and active_sh_degree.  The learning-rate schedule
(update_learning_rate, only xyz) and reset_opacity stay in the caller, as in the reference.
"""
from __future__ import annotations

import threading

import torch

import gs_loss
import gs_train
from diff_gaussian_rasterization import GaussianRasterizer, _C, bounded_status, register_gradient_sink, \
    unregister_gradient_sink

# OptimizationParams defaults (/root/reference/arguments/__init__.py:74-83)
POSITION_LR_INIT = 0.00016
FEATURE_LR = 0.0025
OPACITY_LR = 0.05
SCALING_LR = 0.005
ROTATION_LR = 0.001
PERCENT_DENSE = 0.01
LAMBDA_DSSIM = 0.2
DENSIFY_GRAD_THRESHOLD = 0.0002


class TrainModel:
    """The GaussianModel state one training iteration reads and writes, built from an activated
    scene (gs_scenes.GaussianScene): raw parameters are the inverse activations (log scale,
    inverse-sigmoid opacity; f_dc / f_rest split of the SH rows, gaussian_model.py:133-147)."""

    def __init__(self, scene, device, spatial_lr_scale: float = 1.0, fused: bool = True):
        d = scene.to(device)
        P = d.means3D.shape[0]
        op = d.opacities.clamp(1e-6, 1 - 1e-6)
        raw = {
            "_xyz": d.means3D.clone(),
            "_features_dc": d.shs[:, :1].clone().contiguous(),
            "_features_rest": d.shs[:, 1:].clone().contiguous(),
            "_opacity": torch.log(op / (1 - op)),  # inverse_sigmoid (general_utils.py:17)
            "_scaling": torch.log(d.scales),
            "_rotation": d.rotations.clone(),
        }
        for k, v in raw.items():
            setattr(self, k, torch.nn.Parameter(v.contiguous().requires_grad_(True)))
        self.active_sh_degree = self.max_sh_degree = scene.sh_degree
        self.percent_dense = PERCENT_DENSE
        self.spatial_lr_scale = spatial_lr_scale
        groups = [
            {"params": [self._xyz], "lr": POSITION_LR_INIT * spatial_lr_scale, "name": "xyz"},
            {"params": [self._features_dc], "lr": FEATURE_LR, "name": "f_dc"},
            {"params": [self._features_rest], "lr": FEATURE_LR / 20.0, "name": "f_rest"},
            {"params": [self._opacity], "lr": OPACITY_LR, "name": "opacity"},
            {"params": [self._scaling], "lr": SCALING_LR, "name": "scaling"},
            {"params": [self._rotation], "lr": ROTATION_LR, "name": "rotation"},
        ]
        opt = gs_train.FusedAdam if fused else torch.optim.Adam
        self.optimizer = opt(groups, lr=0.0, eps=1e-15)
        self.max_radii2D = torch.zeros((P,), device=device)
        self.xyz_gradient_accum = torch.zeros((P, 1), device=device)
        self.denom = torch.zeros((P, 1), device=device)

    @property
    def P(self) -> int:
        return self._xyz.shape[0]

    # the reference getters in torch (gaussian_model.py:95-115), for fused=False
    def torch_render_inputs(self):
        return (self._xyz, torch.cat((self._features_dc, self._features_rest), dim=1), torch.sigmoid(self._opacity),
                torch.exp(self._scaling), torch.nn.functional.normalize(self._rotation))


class _AdamBackward:
    """Gradient-sink owner of the fused-Adam train step (train_step(fuse_adam=True)).  Armed on
    the step's rasterizer inputs (xyz and the activated leaves), it receives the view's
    per-Gaussian backward through diff_gaussian_rasterization's deferral protocol (`defers`,
    `defer_view`: only the per-tile half and dL/dmeans2D run inside loss.backward()); train_step
    then runs that half fused with the optimizer step (FusedAdam.step_fused_backward) where
    train.py steps the optimizer, after loss.item() and the densification statistics."""

    defers = True
    accepts_sh_split = True

    def __init__(self):
        self.tensors, self.pending, self.geom = [], None, None

    def arm(self, tensors):
        for t in tensors:
            register_gradient_sink(t, self)
        self.tensors = list(tensors)

    def disarm(self):
        for t in self.tensors:
            unregister_gradient_sink(t)
        self.tensors, self.pending, self.geom = [], None, None

    def forwarded(self, geom, P):
        """The step's forward (diff_gaussian_rasterization calls this after it): its geometry buffer,
        whose error-flags word train_step copies out behind the loss."""
        if self.geom is not None:
            raise RuntimeError("train_step(fuse_adam=True): more than one rasterizer forward in one step")
        self.geom = (geom, P)

    def claim(self, t):
        return None  # not deferred (a backward that needs another input's gradient): plain autograd

    def defer_view(self, ctx, inputs, view):
        if self.pending is not None:
            raise RuntimeError("train_step(fuse_adam=True): more than one rasterizer backward in one step")
        self.pending = (inputs, view)


def render(model: TrainModel, settings, fused: bool = True, act_leaves: list | None = None, split_sh: bool = True,
           binning_capacity: int | None = None, sink_owner=None, row_waits=None):
    """gaussian_renderer.render() for the default pipe (SH and covariance in the rasterizer).
    act_leaves (a list): the activated inputs are made autograd leaves (their adjoint then runs in
    FusedAdam.step_activated) and appended to it as (shs, opacity, scales, rotations).
    binning_capacity: a bounded forward (no host wait; HIP-graph capturable), see train_step.
    sink_owner: armed on xyz and the activated leaves before the rasterizer call (_AdamBackward).
    row_waits (fused=True, the autograd activation; [(lo, hi, event)] from row 0): the parameters'
    rows become ready chunk by chunk on other streams (ShardedAdam's all-gathers of the previous
    step); the activation and the rasterizer's preprocess run chunk by chunk behind them."""
    if row_waits and (act_leaves is not None or not fused):
        raise ValueError("render: row_waits apply to the fused autograd activation only")
    sh_split = None
    act_waits = []
    if act_leaves is not None and not split_sh:
        acts = gs_train.activate_values(model._features_dc, model._features_rest, model._opacity, model._scaling,
                                        model._rotation)
        for t in acts:
            t.requires_grad_(True)
        act_leaves.extend(acts)
        means3D, (shs, opacity, scales, rotations) = model._xyz, acts
    elif act_leaves is not None:
        # the SH rows are read in place by the rasterizer (sh_split): no per-iteration concatenation;
        # `shs` is the [P, M, 3] carrier of dL/dshs that FusedAdam.step_activated maps back to
        # features_dc / features_rest
        _, opacity, scales, rotations = gs_train.activate_values(
            model._features_dc, model._features_rest, model._opacity, model._scaling, model._rotation, with_sh=False)
        P, M = model._features_dc.shape[0], 1 + model._features_rest.shape[1]
        shs = torch.empty((P, M, 3), dtype=torch.float32, device=model._xyz.device)
        sh_split = (model._features_dc, model._features_rest)
        acts = (shs, opacity, scales, rotations)
        for t in acts:
            t.requires_grad_(True)
        act_leaves.extend(acts)
        means3D = model._xyz
    elif fused:
        means3D, shs, opacity, scales, rotations = gs_train.render_inputs(model, row_waits, act_waits)
    else:
        means3D, shs, opacity, scales, rotations = model.torch_render_inputs()
    if sink_owner is not None:
        sink_owner.arm([means3D, shs, opacity, scales, rotations])
    # __init__.py:26 (zeros_like(...) + 0, then retain_grad): the screen-space gradient carrier as a
    # leaf; the rasterizer never reads its values (only its .grad is written), so no fill launch
    screenspace_points = torch.empty_like(means3D, requires_grad=True)
    with _C.row_waits(act_waits):
        image, radii = GaussianRasterizer(raster_settings=settings)(
            means3D=means3D, means2D=screenspace_points, shs=shs, colors_precomp=None, opacities=opacity,
            scales=scales, rotations=rotations, cov3D_precomp=None, sh_split=sh_split,
            binning_capacity=binning_capacity)
    if act_waits:  # (the preprocess waited for every chunk; anything after it on this stream sees all rows)
        torch.cuda.current_stream(means3D.device).wait_event(act_waits[-1][2])
    return image, screenspace_points, radii


def _torch_densification_stats(model: TrainModel, viewspace, radii):
    vis = radii > 0  # train.py:115-116, gaussian_model.py:405-407
    model.max_radii2D[vis] = torch.max(model.max_radii2D[vis], radii[vis].to(model.max_radii2D.dtype))
    model.xyz_gradient_accum[vis] += torch.norm(viewspace.grad[vis, :2], dim=-1, keepdim=True)
    model.denom[vis] += 1


_PINNED = threading.local()


def _pinned_words(device):
    """Two pinned host words per thread and device: the fused step's early read-back of the loss
    (float32, word 0) and of the view's forward error flags (int32, word 1); per thread: two
    threads' steps must not share the copy target."""
    cache = getattr(_PINNED, "bufs", None)
    if cache is None:
        cache = _PINNED.bufs = {}
    b = cache.get(device)
    if b is None:
        b = cache[device] = torch.zeros((2,), dtype=torch.int32, pin_memory=True)
    return b


def train_step(model: TrainModel, settings, gt_image: torch.Tensor, fused: bool = True, densify_stats: bool = True,
               lambda_dssim: float = LAMBDA_DSSIM, fused_adjoint: bool = True, split_sh: bool = True,
               loss_item: bool = False, binning_capacity: int | None = None, fuse_adam: bool = False):
    """One iteration (module docstring).  Returns the loss tensor, or with loss_item=True the
    reference's per-iteration `loss.item()` (train.py:99, its progress-bar EMA): a host read-back
    that waits for the forward and backward, taken where train.py takes it (before the statistics
    and the optimizer step).
    fused_adjoint (with fused): the activation's backward runs inside the Adam update
    (FusedAdam.step_activated), so the raw parameters' gradients are never stored; same floats as
    activate's backward followed by FusedAdam.step, .grad of the activated parameters stays None.
    binning_capacity: the forward runs bounded (its binning buffer sized ahead, no host wait, so the
    iteration can be captured in a HIP graph).  A view with more instances than the capacity is
    invalid: the flags land in the device's bounded status, which train_step reads at the
    loss.item() sync point (loss_item=True) and raises there -- the iteration that overflowed, not
    a later one, and before its optimizer step.  Without loss_item the caller polls
    bounded_status() after its own sync.
    fuse_adam (with fused, fused_adjoint, split_sh and 16 SH coefficients): the per-Gaussian half of
    the backward runs fused with the Adam step, in one pass over the Gaussians where train.py runs
    optimizer.step() (_AdamBackward, FusedAdam.step_fused_backward): no gradient of the six
    parameters is ever stored; parameters and moments bit-identical to the unfused step, the
    screen-space carrier's .grad (the densification statistics' input) as there."""
    acts = [] if (fused and fused_adjoint) else None
    owner = None
    if fuse_adam and acts is not None and split_sh and model._features_rest.shape[1] == 15:
        owner = _AdamBackward()
    try:
        image, viewspace, radii = render(model, settings, fused, acts, split_sh, binning_capacity, owner)
        if fused:  # the whole loss expression in one fused forward / backward (gs_loss.photometric_loss)
            loss, Ll1 = gs_loss.photometric_loss(image, gt_image, lambda_dssim)
        else:
            Ll1 = gs_loss.l1_loss(image, gt_image)
            loss = (1.0 - lambda_dssim) * Ll1 + lambda_dssim * (1.0 - gs_loss.ssim(image, gt_image))
        early = None
        if loss_item and owner is not None and owner.geom is not None:
            # fused Adam: the loss value and the view's forward error flags are copied out right after
            # the loss kernel and read through an event, so the host's sync does not wait for the
            # backward and the optimizer step queued behind it (below)
            buf = _pinned_words(loss.device)
            buf[0:1].view(torch.float32).copy_(loss.detach().reshape(1), non_blocking=True)
            buf[1:2].copy_(_C.view_flags_word(*owner.geom), non_blocking=True)
            early = (buf, torch.cuda.Event())
            early[1].record()
        loss.backward()
        fused_launch = None
        if owner is not None and owner.pending is not None:
            inputs, view = owner.pending
            owner.pending = None
            stats = None
            if densify_stats:  # train.py:115-116 in the fused pass (gs_backward_gaussians_adam_stats)
                if viewspace.grad is None:
                    raise RuntimeError("train_step: the screen-space carrier has no gradient after backward")
                stats = (model.max_radii2D, model.xyz_gradient_accum, model.denom, radii, viewspace.grad)
            fused_launch = model.optimizer.prepare_fused_backward(
                [model._xyz, model._features_dc, model._features_rest, model._opacity, model._scaling,
                 model._rotation], inputs, view, stats)
        value = None
        if early is not None and fused_launch is not None:
            # train.py:99 (loss.item()) before :127 (optimizer.step()): the fused backward + Adam is
            # launched BEFORE the host reads the loss and the forward's status, with its step counts
            # committed only after that check -- the kernel skips the update of a view whose forward
            # recorded an error (a nonzero flags word), and the host decides from the same
            # word, copied out behind the loss: an invalid view (an overflowing bounded forward, or a
            # look-back timeout in any forward's sorts) raises here with parameters, moments, step
            # counts and statistics untouched, as the reference order guarantees
            with torch.no_grad():
                commit = fused_launch(defer_commit=True)
            early[1].synchronize()
            value = float(early[0][0:1].view(torch.float32).item())
            vflags = int(early[0][1])
            if vflags != 0:
                # the kernel skips on any flag, so no step count moves.  The device-wide reports name the
                # cause (and are consumed, so the next call does not raise them again)
                if binning_capacity is not None:
                    bounded_status()
                _C.forward_order_status()
                raise RuntimeError(f"train_step: the view's forward recorded error flags {vflags:#x} (its instance "
                                   "list is invalid); the optimizer step was skipped")
            commit()
            fused_launch = None
            if binning_capacity is not None:
                bounded_status()  # earlier bounded forwards' flags (this view's update stands)
            with torch.no_grad():
                model.optimizer.zero_grad(set_to_none=True)
            return value
        if loss_item:
            # train.py:99 reads loss.item() here, after the backward and before the statistics and
            # the optimizer step (train.py:115-128): an iteration whose bounded forward overflowed
            # raises now, before any parameter, moment or statistic is updated from its invalid
            # gradients
            value = loss.item()
            try:
                if binning_capacity is not None:
                    bounded_status()
                # a look-back timeout in this forward's sorts (read-back forwards report it at the next
                # rasterizer call): taken now, past the sync, before the optimizer uses the gradients
                _C.forward_order_status()
            except RuntimeError:
                with torch.no_grad():  # the invalid gradients must not reach the next iteration either
                    model.optimizer.zero_grad(set_to_none=True)
                raise
        with torch.no_grad():
            if fused_launch is not None:
                # the fused backward + Adam, with the statistics (train.py:115-116) in its pass: they
                # read only the screen-space gradient and the radii, which the update does not touch
                fused_launch()
            elif densify_stats:
                if fused:
                    gs_train.add_densification_stats(model, viewspace, radii)
                else:
                    _torch_densification_stats(model, viewspace, radii)
            if fused_launch is not None:
                pass  # (the optimizer step ran above, fused with the per-Gaussian backward)
            elif acts:
                shs, opac, scales, rots = acts
                model.optimizer.step_activated(
                    {model._features_dc: ("features_dc", shs.grad), model._features_rest: ("features_rest", shs.grad),
                     model._opacity: ("sigmoid", opac.grad), model._scaling: ("exp", scales.grad),
                     model._rotation: ("normalize", rots.grad)}, sh_coeffs=shs.shape[1])
            else:
                model.optimizer.step()
            model.optimizer.zero_grad(set_to_none=True)
    finally:
        if owner is not None:
            owner.disarm()
    return value if loss_item else loss


def train_step_views(model: TrainModel, bucket, views, lambda_dssim: float = LAMBDA_DSSIM, densify_stats: bool = True,
                     average: bool = False, sharded=None, exchange: bool = True):
    """One view-parallel optimizer step (gs_view_parallel): this rank's views
    `views` = [(settings, gt_image)] each run render -> L1 + SSIM -> backward with the fused glue,
    their raw-parameter gradients accumulate in `bucket` (a gs_view_parallel.GradBucket over the six
    parameters, lazy_zero=False: the activation backward accumulates too), ONE all-reduce sums the
    bucket over the ranks (every rank holds the same sum), then every rank runs the same Adam step,
    so the replicas stay bit-identical.  Densification statistics stay per rank until
    gs_view_parallel.reduce_densify_stats at densify time.  sharded (a gs_view_parallel.ShardedAdam
    over the bucket and model.optimizer): reduce-scatter -> sharded Adam -> all-gather in place of the
    all-reduce and the replicated step (call its gather_state() before densify).  With
    ShardedAdam(overlap=True) the previous step's all-gathers are still in flight when this step
    starts: the first view's activation and preprocess wait for them row chunk by row chunk
    (take_row_waits, render(row_waits=...)), and every backward waits for the collective stream's
    zero-fill of the bucket (GradBucket.before_backward).  exchange=False (a measurement baseline,
    bench.py `view_parallel_train`): no collective, every rank steps on its own gradients -- the
    step's cost with a free exchange; the replicas diverge.  Returns the rank's losses."""
    waits = sharded.take_row_waits() if sharded is not None else []
    bucket.zero_grad()
    losses = []
    for settings, gt in views:
        image, viewspace, radii = render(model, settings, fused=True, row_waits=waits)
        waits = []  # (the first view's preprocess waited for every chunk)
        loss, _ = gs_loss.photometric_loss(image, gt, lambda_dssim)
        bucket.before_backward()
        loss.backward()
        if densify_stats:
            with torch.no_grad():
                gs_train.add_densification_stats(model, viewspace, radii)
        losses.append(loss)
    if sharded is not None:
        sharded.step(average=average)
        return losses
    if exchange:
        bucket.allreduce(average=average)
    else:
        bucket.finalize()
    with torch.no_grad():
        model.optimizer.step()
    return losses


def synthetic_densify_stats(model: TrainModel, frac: float = 0.05, seed: int = 0,
                            threshold: float = DENSIFY_GRAD_THRESHOLD) -> None:
    """Densification statistics for a densify step on synthetic gradients:
    denom ~ U{1..4}, mean view-space gradient ~ U(0, threshold / (1 - frac)), so a fraction `frac`
    of the Gaussians crosses densify_grad_threshold (clone or split by their scale)."""
    g = torch.Generator(device=model._xyz.device).manual_seed(seed)
    P = model.P
    dev = model._xyz.device
    model.denom = torch.randint(1, 5, (P, 1), generator=g, device=dev).float()
    mean_grad = torch.rand((P, 1), generator=g, device=dev) * (threshold / (1.0 - frac))
    model.xyz_gradient_accum = mean_grad * model.denom


def densify(model: TrainModel, extent: float, max_screen_size=20,
            threshold: float = DENSIFY_GRAD_THRESHOLD, group=None) -> None:
    """train.py:118-120: densify_and_prune(densify_grad_threshold, 0.005, cameras_extent, 20).
    `extent` is scene.cameras_extent (getNerfppNorm's radius, scene/dataset_readers.py:45-66); a
    single synthetic camera has none, so callers pass one.  View-parallel replicas: call
    gs_view_parallel.reduce_densify_stats first; the split draws are synchronised across `group`."""
    gs_train.densify_and_prune(model, threshold, 0.005, extent, max_screen_size, group=group)

