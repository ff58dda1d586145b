"""Per-iteration training updates of train.py on MI355X, around the rasterizer.

`FusedAdam` is a drop-in for the `torch.optim.Adam` that GaussianModel.training_setup builds
(/root/reference/scene/gaussian_model.py:154-163: six param groups, one tensor each, per-group lr
from the schedulers, eps 1e-15) and that train.py steps every iteration (train.py:123-124).  All
parameter tensors are updated by ONE HIP launch (csrc/gs_train.hip k_adam: p, grad, exp_avg,
exp_avg_sq in one pass, 16-B accesses) instead of torch's foreach chain of eight kernels per
tensor list.  It keeps torch's optimizer state exactly: `state[p]` holds 'step' (CPU float32
tensor), 'exp_avg', 'exp_avg_sq', so GaussianModel's densification code that concatenates / masks
/ replaces those entries (gaussian_model.py:286-300, 317-340) and `state_dict()` /
`load_state_dict()` checkpoints work unchanged, in both directions with torch.optim.Adam.

`activate` / `render_inputs` produce the rasterizer inputs from GaussianModel's raw parameters
(get_features / get_opacity / get_scaling / get_rotation, gaussian_model.py:95-115, read by
gaussian_renderer/__init__.py:53-80) with one HIP launch forward and one backward, in place of
torch's cat + sigmoid + exp + normalize chains and their autograd graph.

`add_densification_stats` folds train.py:115-116 (max_radii2D update + GaussianModel.
add_densification_stats, gaussian_model.py:405-407) into one HIP pass over the Gaussians.

Use:  in GaussianModel.training_setup, `self.optimizer = FusedAdam(l, lr=0.0, eps=1e-15)`;
in render(), `means3D, shs, opacity, scales, rotations = render_inputs(pc)`;
in train.py, `add_densification_stats(gaussians, viewspace_point_tensor, radii)`.
"""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _native

_lib = _native.load()

_MAX_TENSORS = 64  # per C call (the library splits into launches of 16 tensors)


def _check_f32_dense(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: MI355X/HIP path needs device tensors; there is no CPU path")
    if t.dtype != torch.float32:
        raise TypeError(f"{what}: expected float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: must be contiguous")


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False) with one fused HIP launch per step.

    Update per element, as torch's Adam:  g <- -g if maximize; g <- g + weight_decay * p;
    m <- m + (1 - b1)(g - m);  v <- b2 v + (1 - b2) g^2;
    p <- p - lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                 decoupled_weight_decay=False):
        if not 0.0 <= float(lr):
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if amsgrad:
            raise NotImplementedError("FusedAdam: amsgrad is not supported (the reference never sets it)")
        if decoupled_weight_decay:
            raise NotImplementedError("FusedAdam: decoupled weight decay (AdamW) is not supported")
        if capturable or differentiable:
            raise NotImplementedError("FusedAdam: capturable / differentiable modes are not supported")
        # same defaults keys as torch.optim.Adam so state_dicts move between the two
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused,
                        decoupled_weight_decay=decoupled_weight_decay)
        super().__init__(params, defaults)

    def _peek_step(self, p):
        """The step count p's next update uses (state unchanged; the state exists: _checked_state)."""
        step_t = self.state[p]["step"]
        return (int(step_t.item()) if torch.is_tensor(step_t) else int(step_t)) + 1

    def _advance(self, p):
        """The parameter's Adam state (created as torch creates it), its step count incremented:
        (exp_avg, exp_avg_sq, step after this update)."""
        state = self.state[p]
        if len(state) == 0:
            state["step"] = torch.tensor(0.0, dtype=torch.float32)
            state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        step_t = state["step"]
        if torch.is_tensor(step_t):
            if step_t.device.type == "cpu" and step_t.dim() == 0 and not step_t.requires_grad:
                # the CPU step counter in place through numpy (shares the storage): 0.4 us instead of
                # 7 us for a torch add + item() -- an optimizer step that follows the iteration's
                # loss.item() sync runs these on the device's critical path
                a = step_t.numpy()
                a[()] += 1
                t = int(a)
            else:
                step_t += 1
                t = int(step_t.item())
        else:
            t = int(step_t) + 1
            state["step"] = torch.tensor(float(t), dtype=torch.float32)
        return state["exp_avg"], state["exp_avg_sq"], t

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches: dict = {}
        for group in self.param_groups:
            if group.get("amsgrad", False) or group.get("decoupled_weight_decay", False):
                raise NotImplementedError("FusedAdam: amsgrad / decoupled weight decay are not supported")
            b1, b2 = group["betas"]
            key_h = (float(b1), float(b2), float(group["eps"]), bool(group.get("maximize", False)))
            lr = float(group["lr"])
            wd = float(group.get("weight_decay", 0.0))
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad
                if grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                _check_f32_dense(p, "FusedAdam param")
                if grad.shape != p.shape:
                    raise ValueError(f"FusedAdam: grad shape {tuple(grad.shape)} != param {tuple(p.shape)}")
                if grad.dtype != torch.float32 or grad.device != p.device:
                    raise TypeError("FusedAdam: grad must be float32 on the parameter's device")
                if not grad.is_contiguous():
                    grad = grad.contiguous()
                m, v = self._checked_state(p)
                t = self._advance(p)[2]
                batches.setdefault((p.device, key_h), []).append((p, grad, m, v, lr, t, wd))
        for (dev, (b1, b2, eps, maximize)), items in batches.items():
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for s in range(0, len(items), _MAX_TENSORS):
                self._launch(items[s:s + _MAX_TENSORS], b1, b2, eps, maximize, dev, st)
        return loss

    _MODES = {"plain": 0, "features_dc": 1, "features_rest": 2, "sigmoid": 3, "exp": 4, "normalize": 5}

    @torch.no_grad()
    def step_activated(self, sources: dict, sh_coeffs: int):
        """step() whose gradients come from the render() inputs' gradients, through the activation
        adjoint inside the update kernel (gs_adam_step_activated): `sources` maps a parameter to
        (mode, gradient source), mode in "features_dc" / "features_rest" (source: dL/dshs
        [P, sh_coeffs, 3]), "sigmoid" (dL/dopacity), "exp" (dL/dscales), "normalize"
        (dL/drotations); parameters not in `sources` use their own .grad ("plain").  The floats
        are those of activate()'s backward followed by step(); the parameters' .grad stay untouched
        (None for the activated ones)."""
        batches: dict = {}
        for group in self.param_groups:
            b1, b2 = group["betas"]
            key_h = (float(b1), float(b2), float(group["eps"]), bool(group.get("maximize", False)))
            lr = float(group["lr"])
            wd = float(group.get("weight_decay", 0.0))
            for p in group["params"]:
                mode, src = sources.get(p, ("plain", p.grad))
                if src is None:
                    continue
                _check_f32_dense(p, "FusedAdam param")
                _check_f32_dense(src, "FusedAdam gradient source")
                if mode not in self._MODES:
                    raise ValueError(f"FusedAdam.step_activated: unknown mode {mode!r}")
                # the kernel reads the source by the parameter's row count: its shape must match
                # exactly (a stale carrier from before a densify step would read out of bounds)
                if mode in ("features_dc", "features_rest"):
                    want = (p.shape[0], int(sh_coeffs), 3)
                    if tuple(src.shape) != want:
                        raise ValueError(f"FusedAdam: {mode} gradient source must be dL/dshs of shape {want}, got "
                                         f"{tuple(src.shape)}")
                elif src.shape != p.shape:
                    raise ValueError(f"FusedAdam: {mode} gradient source shape {tuple(src.shape)} != param "
                                     f"{tuple(p.shape)}")
                m, v = self._checked_state(p)
                t = self._advance(p)[2]
                batches.setdefault((p.device, key_h), []).append((p, src, m, v, lr, t, wd, self._MODES[mode]))
        for (dev, (b1, b2, eps, maximize)), items in batches.items():
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for s0 in range(0, len(items), _MAX_TENSORS):
                it = items[s0:s0 + _MAX_TENSORS]
                n = len(it)
                ptrs = ctypes.c_void_p * n
                P, G, M, V = (ptrs(*[ctypes.c_void_p(x[j].data_ptr()) for x in it]) for j in range(4))
                numel = (ctypes.c_longlong * n)(*[x[0].numel() for x in it])
                lr = (ctypes.c_double * n)(*[x[4] for x in it])
                steps = (ctypes.c_longlong * n)(*[x[5] for x in it])
                wd = (ctypes.c_double * n)(*[x[6] for x in it])
                modes = (ctypes.c_int * n)(*[x[7] for x in it])
                cast = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
                with torch.cuda.device(dev):
                    _native.check(_lib.gs_adam_step_activated(
                        n, cast(P), cast(G), cast(modes), int(sh_coeffs), cast(M), cast(V), cast(numel), cast(lr),
                        cast(steps), cast(wd), b1, b2, eps, int(maximize), st), "adam step (activated)")

    def _checked_state(self, p):
        """(exp_avg, exp_avg_sq) of p, created if absent, checked dense fp32 of p's size (a state
        loaded from a checkpoint may not be)."""
        state = self.state[p]
        if len(state) == 0:
            state["step"] = torch.tensor(0.0, dtype=torch.float32)
            state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        m, v = state["exp_avg"], state["exp_avg_sq"]
        _check_f32_dense(m, "FusedAdam exp_avg")
        _check_f32_dense(v, "FusedAdam exp_avg_sq")
        if m.numel() != p.numel() or v.numel() != p.numel():
            raise ValueError("FusedAdam: optimizer state does not match the parameter size")
        return m, v

    @torch.no_grad()
    def step_fused_backward(self, params, inputs: dict, view, stats=None) -> None:
        """prepare_fused_backward(...)() (below)."""
        self.prepare_fused_backward(params, inputs, view, stats)()

    @torch.no_grad()
    def prepare_fused_backward(self, params, inputs: dict, view, stats=None):
        """The per-Gaussian half of one view's backward fused with step_activated (one HIP launch,
        gs_backward_gaussians_adam): `params` are GaussianModel's six raw parameters in group
        order (xyz, features_dc, features_rest, opacity, scaling, rotation), `inputs` / `view` the
        deferred rasterizer backward of that view (diff_gaussian_rasterization's deferral
        protocol: the call's Gaussian inputs and (viewmatrix, projmatrix, campos, tan_fovx,
        tan_fovy, W, H, geomBuffer), after its per-tile half).  Same floats as the unfused backward
        followed by step_activated in the modes plain / features_dc / features_rest / sigmoid / exp /
        normalize, and no gradient is stored (.grad of the six stays as it is).
        stats: (max_radii2D, xyz_gradient_accum, denom, radii, viewspace_grad) -- the view's
        densification statistics (densify_stats, train.py:115-116) in the same pass
        (gs_backward_gaussians_adam_stats), the same floats as densify_stats after the step.
        Returns the launch: every check and argument is done here, so a caller that must read the
        loss first (train.py:99 before :127) prepares before that host sync and launches after it;
        the step counts advance at the launch."""
        from diff_gaussian_rasterization import _C

        if len(params) != 6:
            raise ValueError("step_fused_backward: the six GaussianModel parameters in group order")
        where = {id(p): g for g in self.param_groups for p in g["params"]}
        xyz, dc, rest, op, sc, rot = params
        P = xyz.shape[0]
        shapes = ((P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4))
        hyper = set()
        ms, vs, lrs, steps, wds = [], [], [], [], []
        for p, want in zip(params, shapes):
            g = where.get(id(p))
            if g is None:
                raise ValueError("step_fused_backward: a parameter is not in this optimizer")
            _check_f32_dense(p, "FusedAdam param")
            if tuple(p.shape) != want:
                raise ValueError(f"step_fused_backward: parameter of shape {tuple(p.shape)}, expected {want} "
                                 "(16 SH coefficients)")
            b1, b2 = g["betas"]
            hyper.add((float(b1), float(b2), float(g["eps"]), bool(g.get("maximize", False))))
            m, v = self._checked_state(p)
            ms.append(m)
            vs.append(v)
            lrs.append(float(g["lr"]))
            wds.append(float(g.get("weight_decay", 0.0)))
        if len(hyper) != 1:
            raise ValueError("step_fused_backward: the six groups must share betas, eps and maximize")
        if rot.data_ptr() % 16:
            raise ValueError("step_fused_backward: the rotation parameter must be 16-byte aligned")
        mean3, sh, sh_rest = inputs["means3D"], inputs["sh"], inputs.get("sh_rest")
        if mean3.data_ptr() != xyz.data_ptr() or sh_rest is None or sh.data_ptr() != dc.data_ptr() or \
                sh_rest.data_ptr() != rest.data_ptr():
            raise ValueError("step_fused_backward: the deferred view must have read xyz and the split SH rows "
                             "(features_dc / features_rest) of these parameters")
        scales, rots = inputs["scales"], inputs["rotations"]
        dev = xyz.device
        vm, pm, cp, tx, ty, W, H, geom = view
        vm, pm = _C._f32(vm, "viewmatrix", dev, host_ok=True), _C._f32(pm, "projmatrix", dev, host_ok=True)
        cp = _C._f32(cp, "campos", dev, host_ok=True)
        vg = _native.ViewGrad(vm.data_ptr(), pm.data_ptr(), cp.data_ptr(), float(tx), float(ty), int(W), int(H),
                              geom.data_ptr())
        (b1, b2, eps, maximize), = hyper
        if stats is not None:
            max_r, accum, denom, radii, vgrad = stats
            _check_densify_stats(max_r, accum, denom, radii, vgrad)
            if radii.shape[0] != P:
                raise ValueError(f"step_fused_backward: statistics of {radii.shape[0]} Gaussians, expected {P}")
            stat_args = [_ptr(radii), _ptr(vgrad), vgrad.shape[1], _ptr(max_r), _ptr(accum), _ptr(denom)]
        else:
            stat_args = [None, None, 0, None, None, None]
        arr = lambda ts: ctypes.cast((ctypes.c_void_p * 6)(*[t.data_ptr() for t in ts]), ctypes.c_void_p)  # noqa: E731
        steps_c = (ctypes.c_longlong * 6)()
        args = [P, int(inputs["degree"]), 16, _ptr(xyz), _ptr(dc), _ptr(rest), _ptr(scales),
                float(inputs["scale_modifier"]), _ptr(rots), ctypes.byref(vg), arr(params), arr(ms), arr(vs),
                ctypes.cast((ctypes.c_double * 6)(*lrs), ctypes.c_void_p), ctypes.cast(steps_c, ctypes.c_void_p),
                ctypes.cast((ctypes.c_double * 6)(*wds), ctypes.c_void_p), b1, b2, eps, int(maximize), *stat_args,
                int(bool(inputs.get("debug", False))), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)]
        keep = (vm, pm, cp, geom, vg, inputs, stats)  # alive until the launch

        def launch(defer_commit: bool = False):
            """Advances the step counts and launches.  defer_commit: launches with the next step
            counts but returns a commit() that advances them, for a caller that reads the view's
            forward status after the launch -- the kernel skips the update of a view whose forward
            recorded an error, so a caller that raises then leaves parameters, moments and step
            counts as they were (and commits after its check otherwise)."""
            for k, p in enumerate(params):
                steps_c[k] = self._peek_step(p) if defer_commit else self._advance(p)[2]
            with torch.cuda.device(dev):
                _native.check(_lib.gs_backward_gaussians_adam_stats(*args), "backward + adam step (fused)")
            assert keep  # (the closure holds the arguments' tensors until the launch)
            if defer_commit:
                def commit():
                    for k, p in enumerate(params):
                        if self._advance(p)[2] != steps_c[k]:
                            raise RuntimeError("step_fused_backward: a step count moved between launch and commit")
                return commit
            return None

        return launch

    @staticmethod
    def _launch(items, b1, b2, eps, maximize, dev, st):
        n = len(items)
        ptrs = ctypes.c_void_p * n
        P, G, M, V = (ptrs(*[ctypes.c_void_p(it[j].data_ptr()) for it in items]) for j in range(4))
        numel = (ctypes.c_longlong * n)(*[it[0].numel() for it in items])
        lr = (ctypes.c_double * n)(*[it[4] for it in items])
        steps = (ctypes.c_longlong * n)(*[it[5] for it in items])
        wd = (ctypes.c_double * n)(*[it[6] for it in items])
        cast = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
        with torch.cuda.device(dev):
            _native.check(_lib.gs_adam_step(n, cast(P), cast(G), cast(M), cast(V), cast(numel), cast(lr),
                                            cast(steps), cast(wd), b1, b2, eps, int(maximize), st), "adam step")


def densify_stats(max_radii2D: torch.Tensor, grad_accum: torch.Tensor, denom: torch.Tensor, radii: torch.Tensor,
                  viewspace_grad: torch.Tensor) -> None:
    """In place, for every i with radii[i] > 0 (train.py:115, gaussian_model.py:405-407):
    max_radii2D[i] = max(max_radii2D[i], radii[i]); grad_accum[i] += ||viewspace_grad[i, :2]||;
    denom[i] += 1."""
    _check_densify_stats(max_radii2D, grad_accum, denom, radii, viewspace_grad)
    P = radii.shape[0]
    if P == 0:
        return
    dev = radii.device
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    with torch.cuda.device(dev):
        _native.check(_lib.gs_densify_stats(P, ctypes.c_void_p(radii.data_ptr()),
                                            ctypes.c_void_p(viewspace_grad.data_ptr()), viewspace_grad.shape[1],
                                            ctypes.c_void_p(max_radii2D.data_ptr()),
                                            ctypes.c_void_p(grad_accum.data_ptr()),
                                            ctypes.c_void_p(denom.data_ptr()), st), "densify stats")


def _check_densify_stats(max_radii2D, grad_accum, denom, radii, viewspace_grad) -> None:
    P = radii.shape[0]
    for t, name in ((max_radii2D, "max_radii2D"), (grad_accum, "xyz_gradient_accum"), (denom, "denom")):
        _check_f32_dense(t, name)
        if t.numel() != P:
            raise ValueError(f"{name}: expected {P} entries, got {t.numel()}")
    _check_f32_dense(viewspace_grad, "viewspace grad")
    if viewspace_grad.dim() != 2 or viewspace_grad.shape[0] != P or viewspace_grad.shape[1] < 2:
        raise ValueError(f"viewspace grad: expected [{P}, >=2], got {tuple(viewspace_grad.shape)}")
    if radii.dtype != torch.int32 or not radii.is_cuda or not radii.is_contiguous():
        raise TypeError("radii: expected a contiguous int32 device tensor (the rasterizer's output)")


def add_densification_stats(gaussians, viewspace_point_tensor: torch.Tensor, radii: torch.Tensor) -> None:
    """train.py:115-116 in one launch: updates gaussians.max_radii2D, .xyz_gradient_accum, .denom
    for the visible Gaussians (radii > 0, the reference's visibility_filter)."""
    if viewspace_point_tensor.grad is None:
        raise RuntimeError("add_densification_stats: viewspace_point_tensor has no gradient (call backward first)")
    densify_stats(gaussians.max_radii2D, gaussians.xyz_gradient_accum, gaussians.denom, radii,
                  viewspace_point_tensor.grad)


def _aligned(t: torch.Tensor) -> torch.Tensor:
    """contiguous with a 16-byte aligned base (the float4 paths of the activation kernels)"""
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


_SIDE = {}


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(dev)
    return s


def row_chunks(P: int, waits):
    """The row chunks of `waits` ([(lo, hi, event)] contiguous from row 0) at 256-row granularity,
    as the rasterizer's chunked preprocess launches them (csrc/gs_forward.hip launch_row_chunks):
    [(lo, hi, event)] where chunk k holds the rows of the 256-row blocks whose last row lies below
    its end, and must wait for its event and every earlier one."""
    nb = (P + 255) // 256
    out, b0 = [], 0
    for _lo, hi, ev in waits:
        if b0 >= nb:
            break
        b1 = nb if hi >= P else hi // 256
        if b1 > b0:
            out.append((256 * b0, min(P, 256 * b1), ev))
            b0 = b1
        elif ev is not None:
            out.append((256 * b0, 256 * b0, ev))  # nothing to launch, but later chunks wait for it too
    if b0 < nb:
        out.append((256 * b0, P, None))
    return out


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f_dc, f_rest, opacity_raw, scaling_raw, rotation_raw, with_sh=True, row_waits=None,
                waits_out=None):
        P = f_dc.shape[0]
        if f_dc.shape[1:] != (1, 3) or f_rest.dim() != 3 or f_rest.shape[0] != P or f_rest.shape[2] != 3:
            raise ValueError(f"activate: expected features_dc [P,1,3] and features_rest [P,K,3], got "
                             f"{tuple(f_dc.shape)} / {tuple(f_rest.shape)}")
        if opacity_raw.numel() != P or scaling_raw.shape != (P, 3) or rotation_raw.shape != (P, 4):
            raise ValueError("activate: expected opacity [P,1], scaling [P,3], rotation [P,4]")
        ins = [_aligned(t.detach()) for t in (f_dc, f_rest, opacity_raw, scaling_raw, rotation_raw)]
        for t, name in zip(ins, ("features_dc", "features_rest", "opacity", "scaling", "rotation")):
            _check_f32_dense(t, name)
        dc, rest, o, s, q = ins
        K = rest.shape[1]
        dev = dc.device
        # with_sh=False: no concatenated rows (a split-SH rasterizer call reads f_dc / f_rest in place)
        shs = torch.empty((P, 1 + K, 3), dtype=torch.float32, device=dev) if with_sh else None
        opac = torch.empty(tuple(opacity_raw.shape), dtype=torch.float32, device=dev)
        scales = torch.empty((P, 3), dtype=torch.float32, device=dev)
        rots = torch.empty((P, 4), dtype=torch.float32, device=dev)
        if row_waits:
            # rows become ready chunk by chunk on other streams (a sharded optimizer step's all-gathers):
            # each chunk is activated on a side stream as soon as its rows are in, and waits_out gets
            # [(lo, hi, event)] for the rasterizer's chunked preprocess (gs_set_row_waits)
            cur = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(cur)  # the outputs were allocated on the current stream
            outs = (shs, opac, scales, rots)
            ins5 = (dc, rest, o, s, q)
            widths_in = (3, 3 * K, 1, 3, 4)
            widths_out = (3 * (1 + K), 1, 3, 4)
            with torch.cuda.device(dev):
                st = ctypes.c_void_p(side.cuda_stream)
                for lo, hi, ev in row_chunks(P, row_waits):
                    if ev is not None:
                        side.wait_event(ev)
                    if hi > lo:
                        pi = [ctypes.c_void_p(t.data_ptr() + 4 * lo * w) for t, w in zip(ins5, widths_in)]
                        po = [None if t is None else ctypes.c_void_p(t.data_ptr() + 4 * lo * w)
                              for t, w in zip(outs, widths_out)]
                        _native.check(_lib.gs_activate_forward(hi - lo, 3 * K, *pi, *po, st), "activate (row chunk)")
                    done = torch.cuda.Event()
                    done.record(side)
                    if waits_out is not None:
                        waits_out.append((lo, hi, done))
            for t in outs + ins5:
                if t is not None:
                    t.record_stream(side)
            if waits_out is not None:  # the rasterizer's chunks must be contiguous: merge empty ones
                merged = []
                for lo, hi, e in waits_out:
                    if merged and merged[-1][1] == merged[-1][0]:
                        merged[-1] = (merged[-1][0], hi, e)
                    else:
                        merged.append((lo, hi, e))
                waits_out[:] = merged
        else:
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            with torch.cuda.device(dev):
                _native.check(_lib.gs_activate_forward(P, 3 * K, _ptr(dc), _ptr(rest), _ptr(o), _ptr(s), _ptr(q),
                                                       _ptr(shs), _ptr(opac), _ptr(scales), _ptr(rots), st),
                              "activate")
        ctx.P, ctx.K = P, K
        ctx.shapes = (tuple(f_dc.shape), tuple(f_rest.shape), tuple(opacity_raw.shape))
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(opac, scales, q)
        return shs, opac, scales, rots

    @staticmethod
    def backward(ctx, dshs, dopac, dscales, drots):
        opac, scales, q = ctx.saved_tensors
        P, K = ctx.P, ctx.K
        dev = q.device
        need = ctx.needs_input_grad
        dshs = _aligned(dshs) if dshs is not None and (need[0] or need[1]) else None
        dopac = dopac.contiguous() if dopac is not None and need[2] else None
        dscales = dscales.contiguous() if dscales is not None and need[3] else None
        drots = _aligned(drots) if drots is not None and need[4] else None
        g_dc = torch.empty(ctx.shapes[0], dtype=torch.float32, device=dev) if dshs is not None else None
        g_rest = torch.empty(ctx.shapes[1], dtype=torch.float32, device=dev) if dshs is not None else None
        g_o = torch.empty(ctx.shapes[2], dtype=torch.float32, device=dev) if dopac is not None else None
        g_s = torch.empty((P, 3), dtype=torch.float32, device=dev) if dscales is not None else None
        g_q = torch.empty((P, 4), dtype=torch.float32, device=dev) if drots is not None else None
        if any(t is not None for t in (dshs, dopac, dscales, drots)):
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            with torch.cuda.device(dev):
                _native.check(_lib.gs_activate_backward(P, 3 * K, _ptr(dshs), _ptr(dopac), _ptr(dscales),
                                                        _ptr(drots), _ptr(opac), _ptr(scales), _ptr(q), _ptr(g_dc),
                                                        _ptr(g_rest), _ptr(g_o), _ptr(g_s), _ptr(g_q), st),
                              "activate backward")
        return g_dc, g_rest, g_o, g_s, g_q, None, None, None


def activate_values(features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw, with_sh=True):
    """activate()'s forward only (one launch, no autograd graph): fresh (shs, opacity, scales,
    rotations) tensors, for a step whose adjoint runs inside FusedAdam.step_activated.
    with_sh=False: shs is None (the SH rows go to the rasterizer split, GaussianRasterizer sh_split)."""
    with torch.no_grad():
        return _Activate.forward(_NoCtx(), features_dc, features_rest, opacity_raw, scaling_raw,
                                 rotation_raw, with_sh)


class _NoCtx:
    """stand-in autograd context for calling _Activate.forward outside autograd"""

    def save_for_backward(self, *a):
        pass

    def set_materialize_grads(self, v):
        pass


def activate(features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw, row_waits=None, waits_out=None):
    """(shs, opacity, scales, rotations) = (cat(dc, rest, 1), sigmoid(o), exp(s), normalize(q)),
    differentiable; one HIP launch each way (csrc/gs_train.hip k_activate_fwd / k_activate_bwd).
    row_waits ([(lo, hi, event)] contiguous from row 0): the raw rows become ready chunk by chunk
    on other streams; each chunk is activated on a side stream once its event fires, and waits_out
    (a list) receives the chunks' completion events for the rasterizer (row_chunks, _C.row_waits)."""
    return _Activate.apply(features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw, True, row_waits,
                           waits_out)


def render_inputs(pc, row_waits=None, waits_out=None):
    """The tensors gaussian_renderer.render() reads from a GaussianModel (__init__.py:53-80):
    (means3D, shs, opacity, scales, rotations).  row_waits / waits_out: as activate()."""
    shs, opac, scales, rots = activate(pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation,
                                       row_waits, waits_out)
    return pc._xyz, shs, opac, scales, rots


_DENS_NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
_DENS_ATTRS = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")


def densify_and_prune(gaussians, max_grad, min_opacity, extent, max_screen_size, N: int = 2, group=None) -> None:
    """GaussianModel.densify_and_prune (gaussian_model.py:391-403) in three HIP passes.

    Same effect on `gaussians` as the reference: the six parameters become new nn.Parameters of
    the final size in the reference's order (kept originals, kept clones, kept split children), the
    Adam moments follow them (zeros for new rows, 'step' kept), the densification stats are re-zeroed,
    and the split draws come from torch.normal with the reference's shapes and order (same RNG
    stream).  Every parameter and moment is rewritten once instead of four times
    (csrc/gs_densify.hip).

    View-parallel replicas (a torch.distributed process group of more than one rank, `group` or the
    default one; gs_view_parallel): every rank draws, then rank 0's split samples are broadcast, so
    the replicas stay bit-identical (their parameters, moments and reduced statistics already are).
    A gs_view_parallel.GradBucket that holds the replaced parameters' gradients is rebound to the new
    parameters."""
    sharded = getattr(gaussians.optimizer, "_gs_sharded_moments", None)
    if sharded is not None and sharded.moments_sharded():
        raise RuntimeError("densify_and_prune: the Adam moments are sharded over the ranks (gs_view_parallel."
                           "ShardedAdam); call its gather_state() first")
    if sharded is not None:
        sharded.sync()  # an overlapped step's all-gathers, before the parameters are read here
    params = [getattr(gaussians, a) for a in _DENS_ATTRS]
    xyz = params[0]
    P = xyz.shape[0]
    if P == 0:
        return
    dev = xyz.device
    src = [p.detach() for p in params]
    for t, n in zip(src, _DENS_NAMES):
        _check_f32_dense(t, n)
        if t.shape[0] != P:
            raise ValueError(f"densify: {n} has {t.shape[0]} rows, xyz has {P}")
    accum = gaussians.xyz_gradient_accum.contiguous()
    denom = gaussians.denom.contiguous()
    for t, n in ((accum, "xyz_gradient_accum"), (denom, "denom")):
        _check_f32_dense(t, n)
        if t.numel() != P:
            raise ValueError(f"densify: {n} must have {P} entries")
    widths = [int(t[0].numel()) for t in src]
    flags = torch.empty((P,), dtype=torch.uint8, device=dev)
    counts = torch.empty((4 * _lib.gs_densify_block_count(P),), dtype=torch.int32, device=dev)
    totals = torch.empty((4,), dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    with torch.cuda.device(dev):
        _native.check(_lib.gs_densify_classify(
            P, _ptr(accum), _ptr(denom), _ptr(src[3]), _ptr(src[4]), float(max_grad),
            float(gaussians.percent_dense * extent), float(min_opacity), float(0.1 * extent),
            1 if max_screen_size else 0, float(max_screen_size) if max_screen_size else 0.0, int(N),
            _ptr(flags), _ptr(counts), _ptr(totals), st), "densify classify")
        tot = [int(v) for v in totals.cpu()]  # the one host read: sizes of the new tensors
        tot_h = (ctypes.c_uint32 * 4)(*tot)
        n_split = tot[2]
        stds = torch.empty((N * n_split, 3), dtype=torch.float32, device=dev)
        _native.check(_lib.gs_densify_split_stds(P, N, tot_h, _ptr(flags), _ptr(counts), _ptr(src[4]),
                                                 _ptr(stds) if n_split else None, st), "densify stds")
        # the reference's draw (gaussian_model.py:359-360): same shapes, same generator stream
        samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=dev), std=stds).contiguous()
        if n_split:
            import gs_view_parallel

            gs_view_parallel.sync_from_rank0(samples, group)  # replicas: rank 0's draw (no-op alone)
        Pn = tot[0] + tot[1] + N * tot[3]
        groups = {g["name"]: g for g in gaussians.optimizer.param_groups}
        states, outs, m_in, v_in, m_out, v_out = [], [], [], [], [], []
        for n, t in zip(_DENS_NAMES, src):
            grp = groups[n]
            if len(grp["params"]) != 1 or grp["params"][0] is not params[_DENS_NAMES.index(n)]:
                raise ValueError(f"densify: optimizer group '{n}' must hold exactly the model's tensor")
            stt = gaussians.optimizer.state.get(grp["params"][0], None)
            states.append(stt)
            outs.append(torch.empty((Pn,) + tuple(t.shape[1:]), dtype=torch.float32, device=dev))
            if stt is not None:
                m, v = stt["exp_avg"].contiguous(), stt["exp_avg_sq"].contiguous()
                _check_f32_dense(m, f"{n} exp_avg")
                if m.shape != t.shape or v.shape != t.shape:
                    raise ValueError(f"densify: optimizer state of '{n}' does not match the parameter")
                m_in.append(m)
                v_in.append(v)
                m_out.append(torch.empty_like(outs[-1]))
                v_out.append(torch.empty_like(outs[-1]))
            else:
                m_in.append(None)
                v_in.append(None)
                m_out.append(None)
                v_out.append(None)
        arr = lambda ts: (ctypes.c_void_p * 6)(*[_ptr(x) for x in ts])  # noqa: E731
        _native.check(_lib.gs_densify_emit(
            P, N, tot_h, _ptr(flags), _ptr(counts), _ptr(samples) if n_split else None,
            ctypes.cast(arr(src), ctypes.c_void_p), ctypes.cast(arr(m_in), ctypes.c_void_p),
            ctypes.cast(arr(v_in), ctypes.c_void_p), ctypes.cast(arr(outs), ctypes.c_void_p),
            ctypes.cast(arr(m_out), ctypes.c_void_p), ctypes.cast(arr(v_out), ctypes.c_void_p),
            ctypes.cast((ctypes.c_int * 6)(*widths), ctypes.c_void_p), st), "densify emit")
    # gradient buckets (gs_view_parallel.GradBucket) that own the old parameters' gradients
    from diff_gaussian_rasterization import _sink_owner

    owners = []
    for p in params:
        o = _sink_owner(p)
        if o is not None and hasattr(o, "rebind") and all(o is not x for x in owners):
            owners.append(o)
    replaced = {}
    # optimizer surgery as cat_tensors_to_optimizer / _prune_optimizer do it
    for i, n in enumerate(_DENS_NAMES):
        grp = groups[n]
        old = grp["params"][0]
        newp = torch.nn.Parameter(outs[i].requires_grad_(True))
        stt = states[i]
        if stt is not None:
            stt["exp_avg"], stt["exp_avg_sq"] = m_out[i], v_out[i]
            del gaussians.optimizer.state[old]
            gaussians.optimizer.state[newp] = stt
        grp["params"][0] = newp
        setattr(gaussians, _DENS_ATTRS[i], newp)
        replaced[id(old)] = newp
    for o in owners:
        o.rebind([replaced.get(id(p), p) for p in o.params])
    gaussians.xyz_gradient_accum = torch.zeros((Pn, 1), device=dev)
    gaussians.denom = torch.zeros((Pn, 1), device=dev)
    gaussians.max_radii2D = torch.zeros((Pn,), device=dev)
    torch.cuda.empty_cache()
