"""diff_gaussian_rasterization -- MI355X-native drop-in for the 3DGS differentiable rasterizer.

Public surface used by the reference's render adapter
(/root/reference/gaussian_renderer/__init__.py:14 import, :36-49 settings, :51 rasterizer,
:85-93 call):

    GaussianRasterizationSettings(image_height, image_width, tanfovx, tanfovy, bg, scale_modifier,
                                  viewmatrix, projmatrix, sh_degree, campos, prefiltered, debug)
    GaussianRasterizer(raster_settings)(means3D, means2D, opacities, shs=None, colors_precomp=None,
                                        scales=None, rotations=None, cov3D_precomp=None)
        -> (color [3, H, W] fp32, radii [P] int32)
    GaussianRasterizer.markVisible(positions) -> bool [P]
    rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings)

This is the 2023 two-output API of graphdeco-inria/diff-gaussian-rasterization (the reference's
un-vendored submodule, /root/reference/.gitmodules:4-6), implemented over libgsrast.so (hand-written
HIP for gfx950, C ABI in include/gsrast.h).  Gradients flow to every tensor input that requires
them, including `means2D`, whose .grad holds the NDC-space screen gradient read by densification
(/root/reference/scene/gaussian_model.py:405-407).
"""
from __future__ import annotations

import weakref
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "cpu_deep_copy_tuple",
           "register_gradient_sink", "unregister_gradient_sink", "prepare_views", "last_num_rendered",
           "bounded_status"]

# ------------------------------------------------------------------------------------------
# Gradient sinks (an extension beyond the upstream API, used by gs_view_parallel.GradBucket).
# A leaf tensor registered here gets its rasterizer gradient written -- or, once the step already
# holds one, ADDED (gs_backward_accumulate) -- straight into the buffer its owner hands out
# (normally the tensor's own .grad, a view into a flat all-reduce bucket), and the autograd
# Function returns None for it.  The result equals autograd's `grad += g` with no extra pass over
# the gradients and no pack/unpack copy.  owner.claim(tensor) -> (buffer, accumulate) or None
# (None: the normal autograd path).  Optional: owner.write_order(stream) -> torch.cuda.Event or None
# (the stream waits for it before the gradient-writing kernel) and owner.written(stream), called
# once the backward is enqueued -- an owner shared by views on several streams orders its writes.
# ------------------------------------------------------------------------------------------
_SINKS: dict = {}  # id(tensor) -> (weakref to the tensor, owner)


def register_gradient_sink(tensor: torch.Tensor, owner) -> None:
    if not tensor.is_leaf:
        raise ValueError("register_gradient_sink: only leaf tensors can own a gradient sink")
    _SINKS[id(tensor)] = (weakref.ref(tensor), owner)


def unregister_gradient_sink(tensor: torch.Tensor) -> None:
    e = _SINKS.get(id(tensor))
    if e is not None and e[0]() is tensor:
        del _SINKS[id(tensor)]


def _sink_owner(t):
    if t is None or not isinstance(t, torch.Tensor) or not t.requires_grad:
        return None
    e = _SINKS.get(id(t))
    return e[1] if e is not None and e[0]() is t else None


# autograd input index -> gradient name (_C.GRAD_NAMES)
_SINK_INPUTS = ((0, "means3D"), (1, "means2D"), (2, "sh"), (3, "colors"), (4, "opacity"), (5, "scales"),
                (6, "rotations"), (7, "cov3D"))


def cpu_deep_copy_tuple(input_tuple):
    """CPU copies of every tensor in the tuple (used for the debug snapshot on failure)."""
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings, prepared=None, sh_split=None, binning_capacity=None):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings, prepared, sh_split, binning_capacity)


# ------------------------------------------------------------------------------------------
# Bounded forwards (an extension beyond the upstream API, ABI v10).  Upstream reads num_rendered
# back to size its binning buffer, one host wait per forward.  With `binning_capacity=N` the
# buffer is sized for N instances ahead of time and the forward is enqueued without any host
# wait, event or allocation inside the library, so a training step can be captured into a
# HIP graph (torch.cuda.CUDAGraph).  Outputs are bit-identical while the view's instance count
# fits; a view that exceeds N leaves a sticky flag (its outputs invalid, all accesses in bounds)
# that the next bounded forward raises, or bounded_status() reports.  last_num_rendered() is the
# count of the last forward that read it back, a base for N.
# ------------------------------------------------------------------------------------------
def last_num_rendered() -> int:
    return _C._LAST_NUM_RENDERED[0]


def bounded_status():
    """(flags, instances) left by bounded forwards on the current device since the last call
    (cleared); raises RuntimeError if one exceeded its capacity, culled a prefiltered point or
    timed out.  Covers the forwards whose kernels ran: call it after a synchronisation."""
    return _C.bounded_status()


class PreparedView:
    """The first half of one view's forward, computed by prepare_views for several views at once
    (an extension beyond the upstream API).  Hand it to that view's GaussianRasterizer call as
    `prepared=`; it is checked against the call's settings and inputs and used once."""

    def __init__(self, triple, settings, inputs):
        self.triple, self.settings, self.inputs = triple, settings, inputs
        # autograd version counters: an in-place update between prepare_views and the call (an
        # optimizer step) would leave the prepared geometry stale
        self.versions = tuple(None if t is None else t._version for t in inputs)

    def take(self, settings, inputs):
        if self.triple is None:
            raise RuntimeError("prepare_views: a prepared view is used once")
        if settings is not self.settings or any(
                (a is None) != (b is None) or (a is not None and (a.data_ptr(), a.shape) != (b.data_ptr(), b.shape))
                for a, b in zip(inputs, self.inputs)):
            raise RuntimeError("prepare_views: the rasterizer call does not match the prepared view")
        if any(v is not None and b._version != v for b, v in zip(self.inputs, self.versions)):
            raise RuntimeError("prepare_views: an input was modified in place after prepare_views (stale prepared "
                               "view); prepare the views again")
        t, self.triple = self.triple, None
        return t


def prepare_views(rasterizers, means3D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                  cov3D_precomp=None, streams=None, binning_capacity=None):
    """Run the first half of the forward (preprocess, depth order, instance offsets) of several
    views of the same Gaussians at once: one preprocess launch reads every Gaussian's inputs once
    for all cameras (gs_forward_preprocess_views) and one host wait returns every view's instance
    count.  Returns one PreparedView per rasterizer, to pass as `prepared=` to that rasterizer's
    call with the same tensors; view k's ordering runs on streams[k] (its call must run there).
    The rasterizers must share sh_degree, scale_modifier, prefiltered and debug.
    binning_capacity (one int, or one per view): bounded views -- no instance count is read back,
    each view's binning buffer is sized for its capacity (see bounded_status())."""
    ss = [r.raster_settings for r in rasterizers]
    s0 = ss[0]
    for s in ss[1:]:
        if (s.sh_degree, s.scale_modifier, s.prefiltered, s.debug) != (s0.sh_degree, s0.scale_modifier,
                                                                          s0.prefiltered, s0.debug):
            raise ValueError("prepare_views: the views must share sh_degree, scale_modifier, prefiltered, debug")
    empty = torch.Tensor([])
    e = lambda t: empty if t is None else t  # noqa: E731
    caps = None
    if binning_capacity is not None:
        caps = ([int(binning_capacity)] * len(ss) if isinstance(binning_capacity, int)
                else [int(c) for c in binning_capacity])
    # view k's matrices are read on the current stream (the preprocess) and on streams[k]
    own = [None] * len(ss) if not streams else [[streams[k]] for k in range(len(ss))]
    views = [_contiguous_matrix(s.viewmatrix, o) for s, o in zip(ss, own)]
    projs = [_contiguous_matrix(s.projmatrix, o) for s, o in zip(ss, own)]
    with torch.no_grad():
        tri = _C.preprocess_views([s.bg for s in ss], means3D.detach(), e(colors_precomp).detach(), opacities.detach(),
                                  e(scales).detach(), e(rotations).detach(), s0.scale_modifier,
                                  e(cov3D_precomp).detach(), views, projs, [s.tanfovx for s in ss],
                                  [s.tanfovy for s in ss], [s.image_height for s in ss], [s.image_width for s in ss],
                                  e(shs).detach(), s0.sh_degree, [s.campos for s in ss], s0.prefiltered, s0.debug,
                                  streams, caps)
    inputs = (means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp)
    return [PreparedView(t, s, inputs) for t, s in zip(tri, ss)]


_CONTIG: dict = {}  # id(camera tensor) -> (weakref, _version, contiguous copy)


def _contiguous_matrix(t: torch.Tensor, streams=None) -> torch.Tensor:
    """t.contiguous() for the camera matrices, memoised per source tensor and version.  The
    reference's Camera keeps world_view_transform / full_proj_transform as transposed views
    (scene/cameras.py:54-56), so every render() would otherwise copy both (one copy launch each).
    The copy is made on the current stream; `streams` (views rendered on other streams) are
    recorded on it, so that the allocator does not reuse it while their kernels may still read
    it after the memo drops it."""
    if t.is_contiguous():
        c = t
    else:
        e = _CONTIG.get(id(t))
        if e is not None and e[0]() is t and e[1] == t._version:
            c = e[2]
        else:
            c = t.contiguous()
            if len(_CONTIG) > 256:
                _CONTIG.clear()
            _CONTIG[id(t)] = (weakref.ref(t), t._version, c)
    if streams and c.is_cuda:
        for st in streams:
            if st is not None:
                c.record_stream(st)
    return c


def _run_with_snapshot(fn, args, debug, dump_name, phase):
    """settings.debug: keep CPU copies of the arguments and dump them if the native call fails."""
    if not debug:
        return fn(*args)
    cpu_args = cpu_deep_copy_tuple(args)
    try:
        return fn(*args)
    except Exception:
        torch.save(cpu_args, dump_name)
        print(f"\nAn error occured in {phase}. Please forward {dump_name} for debugging.")
        raise


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, prepared=None, sh_split=None, binning_capacity=None):
        s = raster_settings
        # the camera matrices arrive transposed (cameras.py:54-56 world_view_transform is a
        # .transpose(0, 1) view); make them contiguous once and reuse them in backward
        view, proj = _contiguous_matrix(s.viewmatrix), _contiguous_matrix(s.projmatrix)
        sh_rest = None
        sh_input = sh  # the autograd input (with sh_split: the gradient carrier; its sink owner receives dL/dshs)
        if sh_split is not None:
            # split SH rows: the kernels read features_dc / features_rest in place; `sh` is only the
            # [P, M, 3] carrier of the concatenation's gradient (its values are never read)
            dc, sh_rest = (t.detach() for t in sh_split)
            if prepared is not None:
                raise RuntimeError("sh_split: not supported with prepared views")
            if tuple(sh.shape) != (dc.shape[0], 1 + sh_rest.shape[1], 3):
                raise RuntimeError("sh_split: shs must be the [P, M, 3] gradient carrier of cat(features_dc, "
                                   "features_rest)")
            sh = dc
        args = (s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                view, proj, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
                s.campos, s.prefiltered, s.debug)
        if prepared is not None and binning_capacity is not None:
            raise RuntimeError("binning_capacity: not supported with prepared views")
        if sh_rest is not None or binning_capacity is not None:
            num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _run_with_snapshot(
                lambda *a: _C.rasterize_gaussians(*a, sh_rest=sh_rest, capacity=binning_capacity), args, s.debug,
                "snapshot_fw.dump", "forward")
        elif prepared is not None:
            nz = lambda t: None if t is None or t.numel() == 0 else t  # noqa: E731
            tri = prepared.take(s, (means3D, nz(sh), nz(colors_precomp), opacities, nz(scales), nz(rotations),
                                    nz(cov3Ds_precomp)))
            num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _C.rasterize_gaussians(*args,
                                                                                                     prepared=tri)
        else:
            num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _run_with_snapshot(
                _C.rasterize_gaussians, args, s.debug, "snapshot_fw.dump", "forward")
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.matrices = (view, proj)
        ctx.sh_rest = sh_rest
        # the split rows are kept outside save_for_backward (they are not inputs of the Function):
        # their version counters stand in for autograd's in-place check
        ctx.sh_split_versions = None if sh_rest is None else (sh._version, sh_rest._version)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the (int) radii output
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer,
                              binningBuffer, imgBuffer)
        ctx.mark_non_differentiable(radii)
        sinks = []
        if _SINKS:
            inputs = (means3D, means2D, sh_input, colors_precomp, opacities, scales, rotations, cov3Ds_precomp)
            for k, name in _SINK_INPUTS:
                owner = _sink_owner(inputs[k])
                if owner is not None:
                    sinks.append((k, name, inputs[k], owner))
            # an owner that follows its views' forward status (gs_train_step._AdamBackward) gets the
            # view's geometry buffer now, while its error-flags word can still be copied out
            # stream-ordered behind this forward
            for owner in {id(o): o for _k, _n, _t, o in sinks}.values():
                if hasattr(owner, "forwarded"):
                    owner.forwarded(geomBuffer, means3D.shape[0])
        ctx.sinks = sinks
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii):
        s = ctx.raster_settings
        if grad_out_color is None:  # the colour output did not reach the loss
            return (None,) * 12
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer, imgBuffer = (
            ctx.saved_tensors)
        if ctx.sh_rest is not None and (sh._version, ctx.sh_rest._version) != ctx.sh_split_versions:
            raise RuntimeError("sh_split: features_dc or features_rest was modified by an inplace operation between "
                               "the forward and the backward")
        view, proj = ctx.matrices
        args = (s.bg, means3D, radii, colors_precomp, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                view, proj, s.tanfovx, s.tanfovy, grad_out_color.contiguous(), sh, s.sh_degree,
                s.campos, geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, s.debug)

        # a sink owner that defers the per-Gaussian half (GradBucket(defer=True)) takes this view
        # when every parameter gradient the call needs goes to it: only the per-tile half and
        # dL_dmeans2D run now, the per-Gaussian half later for all of its views in one pass
        deferrer = _deferring_owner(ctx)
        if deferrer is not None and ctx.sh_rest is not None and not getattr(deferrer, "accepts_sh_split", False):
            raise RuntimeError("sh_split: not supported with a deferring gradient bucket")
        if deferrer is not None:
            M = (1 + ctx.sh_rest.size(1)) if ctx.sh_rest is not None else (sh.size(1) if sh.ndimension() == 3 else 0)
            dm2 = _C.backward_render(s.bg, view, proj, s.campos, s.tanfovx, s.tanfovy, grad_out_color.contiguous(),
                                     means3D.size(0), s.sh_degree, M,
                                     geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, ctx.needs_input_grad[1],
                                     s.debug)
            deferrer.defer_view(ctx, dict(means3D=means3D, sh=sh, colors=colors_precomp, scales=scales,
                                          rotations=rotations, cov3D=cov3Ds_precomp, scale_modifier=s.scale_modifier,
                                          degree=s.sh_degree, debug=s.debug, sh_rest=ctx.sh_rest),
                                (view, proj, s.campos, s.tanfovx, s.tanfovy, s.image_width, s.image_height,
                                 geomBuffer))
            return (None, dm2) + (None,) * 10

        sinks, sunk, owners = {}, set(), []
        for k, name, t, owner in ctx.sinks:
            if ctx.needs_input_grad[k]:
                claim = owner.claim(t)
                if claim is not None:
                    sinks[name] = claim
                    sunk.add(k)
                    if all(o is not owner for o in owners):
                        owners.append(owner)
        # sink owners may order their buffer's writes across streams (views rendered on several
        # streams, GradBucket): the last kernel waits for the owner's previous write
        wait = None
        if owners:
            st = torch.cuda.current_stream(grad_out_color.device)
            evs = [e for e in (o.write_order(st) for o in owners if hasattr(o, "write_order")) if e is not None]
            for e in evs[1:]:
                st.wait_event(e)
            wait = evs[0] if evs else None

        def _bwd(*a):
            return _C.backward_impl(*a, want_all=False, sinks=sinks, wait_event=wait, sh_rest=ctx.sh_rest)

        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh, grad_scales,
         grad_rotations) = _run_with_snapshot(_bwd, args, s.debug, "snapshot_bw.dump", "backward")
        for o in owners:
            if hasattr(o, "written"):
                o.written(st)
        grads = [grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                 grad_rotations, grad_cov3Ds_precomp, None, None, None, None]
        for k in sunk:  # already in the sink's buffer (the tensor's .grad)
            grads[k] = None
        return tuple(grads)


def _deferring_owner(ctx):
    """The one sink owner with `defer_view` that receives every input gradient this backward must
    produce (means2D aside), or None."""
    if not ctx.sinks:
        return None
    owner = ctx.sinks[0][3]
    if not getattr(owner, "defers", False):
        return None
    sunk = {k for k, _name, _t, o in ctx.sinks if o is owner}
    for k in range(8):
        if k != 1 and ctx.needs_input_grad[k] and k not in sunk:
            return None
    return owner


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, prepared=None, sh_split=None, binning_capacity=None):
        """prepared: this call's PreparedView from prepare_views (extension; default: none).
        binning_capacity: size the binning buffer for that many instances and run the forward
        without a host wait (extension, ABI v10; see bounded_status()).
        sh_split: (features_dc [P,1,3], features_rest [P,M-1,3]) read in place instead of the
        concatenated shs (extension, ABI v8: no per-iteration cat); `shs` is then a [P,M,3] tensor
        whose values are never read and whose .grad receives dL/d cat(features_dc, features_rest)
        (what FusedAdam.step_activated consumes).  Bit-identical to passing the concatenation."""
        s = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        empty = torch.Tensor([])
        shs = empty if shs is None else shs
        colors_precomp = empty if colors_precomp is None else colors_precomp
        scales = empty if scales is None else scales
        rotations = empty if rotations is None else rotations
        cov3D_precomp = empty if cov3D_precomp is None else cov3D_precomp
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                   s, prepared, sh_split, binning_capacity)
