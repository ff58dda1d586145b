"""Fused training updates (gs_train, csrc/gs_train.hip) against the reference's own formulation.

FusedAdam is checked against torch.optim.Adam -- the optimizer GaussianModel.training_setup
builds (/root/reference/scene/gaussian_model.py:163, torch 2.10 here, foreach implementation on
the device) -- over several steps with per-group learning rates that change every step (the
reference's xyz scheduler), odd tensor sizes (vector body + scalar tail), a misaligned tensor
(scalar path only), densification-style state replacement between steps
(gaussian_model.py:286-340) and state_dict hand-over in both directions.
The kernel follows torch's operation order (fma where ATen's contracted lerp / addcmul / addcdiv
functors fuse), so most elements agree bitwise; tolerances cover a float32 ulp of the operands:
params rtol 2e-6 + 1e-7 absolute, exp_avg / exp_avg_sq rtol 1e-5 + 2e-6 absolute (gradients here
reach |g| ~ 12, whose float32 ulp is ~1e-6; m near 0 comes from cancellation of such terms).

activate is checked against GaussianModel's property formulation (gaussian_model.py:95-115:
torch.cat, torch.sigmoid, torch.exp, F.normalize) forward and backward, for SH widths 0..15 rest
rows, a zero quaternion, and partial output gradients: shs bit-exact (a copy), activations rtol
2e-6 (expf / division ulps), gradients rtol 1e-5.

densify_stats is checked against train.py:115 + gaussian_model.py:405-407 written in torch:
max_radii2D and denom bit-exact, xyz_gradient_accum rtol 1e-6 (one sqrt of a 2-term sum)."""
import pytest
import torch

P_TOL = dict(rtol=2e-6, atol=1e-7)
S_TOL = dict(rtol=1e-5, atol=2e-6)
LRS = [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3]


def test_fused_adam_rejects_cpu_and_unsupported_modes():
    from gs_train import FusedAdam

    p = torch.zeros(4, requires_grad=True)
    with pytest.raises(NotImplementedError):
        FusedAdam([p], amsgrad=True)
    opt = FusedAdam([p], lr=0.1, eps=1e-15)
    p.grad = torch.ones(4)
    with pytest.raises(RuntimeError, match="no CPU path"):
        opt.step()
    assert opt.defaults.keys() == torch.optim.Adam([p]).defaults.keys()


def test_adam_abi_validation_without_gpu():
    import ctypes

    from diff_gaussian_rasterization import _native

    lib = _native.load()
    assert lib.gs_adam_step(0, None, None, None, None, None, None, None, None, 0.9, 0.999, 1e-15, 0, None) == 0
    rc = lib.gs_adam_step(1, None, None, None, None, None, None, None, None, 0.9, 0.999, 1e-15, 0, None)
    assert rc != 0 and "missing" in _native.last_error()
    rc = lib.gs_densify_stats(5, None, None, 1, None, None, None, None)
    assert rc != 0 and "grad_stride" in _native.last_error()
    assert lib.gs_densify_stats(0, None, None, 3, None, None, None, None) == 0
    # the fused step's statistics (ABI 16): all five pointers or none, checked before any launch
    # (the other arguments are placeholders that are only range-checked on the host here)
    fake = [ctypes.c_void_p(0x10000 * (k + 1)) for k in range(6)]
    arr = lambda: ctypes.cast((ctypes.c_void_p * 6)(*fake), ctypes.c_void_p)  # noqa: E731
    steps = ctypes.cast((ctypes.c_longlong * 6)(*[1] * 6), ctypes.c_void_p)
    lrs = ctypes.cast((ctypes.c_double * 6)(*[1e-3] * 6), ctypes.c_void_p)
    vg = _native.ViewGrad(0x1000, 0x2000, 0x3000, 0.5, 0.5, 8, 8, 0x4000)
    base = [5, 3, 16, fake[0], fake[1], fake[2], ctypes.c_void_p(0x9000), 1.0, ctypes.c_void_p(0xA000),
            ctypes.byref(vg), arr(), arr(), arr(), lrs, steps, None, 0.9, 0.999, 1e-15, 0]
    some = [ctypes.c_void_p(0xB000), None, 2, None, None, None]
    assert lib.gs_backward_gaussians_adam_stats(*base, *some, 0, None) != 0
    assert "all five pointers or none" in _native.last_error()
    every = [ctypes.c_void_p(0xB000 + 0x100 * k) for k in range(6)]
    every[2] = 1
    assert lib.gs_backward_gaussians_adam_stats(*base, *every, 0, None) != 0
    assert "grad_stride" in _native.last_error()
    assert lib.gs_backward_gaussians_adam_stats(0, *base[1:], *some, 0, None) == 0  # P == 0: nothing to do


def _make_params(device, sizes, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=g).to(device) for s in sizes]


def _groups(params):
    return [{"params": [p], "lr": lr, "name": str(i)} for i, (p, lr) in enumerate(zip(params, LRS))]


def _run_pair(device, sizes, steps, *, kw=None, mutate=None, seed=0):
    from gs_train import FusedAdam

    kw = kw or {}
    base = _make_params(device, sizes, seed)
    ours = [t.clone().requires_grad_(True) for t in base]
    ref = [t.clone().requires_grad_(True) for t in base]
    o1 = FusedAdam(_groups(ours), lr=0.0, eps=1e-15, **kw)
    o2 = torch.optim.Adam(_groups(ref), lr=0.0, eps=1e-15, **kw)
    g = torch.Generator().manual_seed(seed + 1)
    for it in range(steps):
        for a, b in zip(ours, ref):
            gr = (torch.randn(a.shape, generator=g) * (0.1 + it)).to(device)
            a.grad = gr.clone()
            b.grad = gr.clone()
        for o in (o1, o2):  # the xyz scheduler changes group 0's lr every iteration
            o.param_groups[0]["lr"] = LRS[0] * (0.97 ** it)
        o1.step()
        o2.step()
        if mutate is not None:
            ours, ref = mutate(it, o1, ours), mutate(it, o2, ref)
    return o1, o2, ours, ref


def _compare(o1, o2, ours, ref, exact_frac=None):
    same = total = 0
    for a, b in zip(ours, ref):
        same += int((a.detach() == b.detach()).sum())
        total += a.numel()
        torch.testing.assert_close(a.detach(), b.detach(), **P_TOL)
        s1, s2 = o1.state[a], o2.state[b]
        torch.testing.assert_close(s1["exp_avg"], s2["exp_avg"], **S_TOL)
        torch.testing.assert_close(s1["exp_avg_sq"], s2["exp_avg_sq"], **S_TOL)
        assert float(s1["step"]) == float(s2["step"])
        assert s1["step"].device.type == "cpu" and s1["step"].dtype == torch.float32
    if exact_frac is not None:
        assert same >= exact_frac * total, f"only {same}/{total} parameters bit-identical to torch.optim.Adam"


@pytest.mark.gpu
def test_fused_adam_matches_torch_adam_gaussian_groups(device):
    P = 4099  # odd: every tensor has a scalar tail
    sizes = [(P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4)]
    _compare(*_run_pair(device, sizes, 12), exact_frac=0.9)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{"weight_decay": 0.01}, {"maximize": True}, {"betas": (0.8, 0.99)}])
def test_fused_adam_options(device, kw):
    _compare(*_run_pair(device, [(1,), (3,), (5,), (1000,), (7, 3), (64,)], 6, kw=kw))


@pytest.mark.gpu
def test_fused_adam_many_tensors_and_misaligned(device):
    """More tensors than one launch carries (16), and a parameter view at a 4-byte offset."""
    from gs_train import FusedAdam

    storage = torch.randn(1 + 4 * 257, device=device)
    odd = storage[1:].view(257, 4)  # data_ptr % 16 == 4: scalar path only
    base = [odd] + _make_params(device, [(i * 13 + 1,) for i in range(20)])
    ours = [t.detach().clone() if i else t.detach() for i, t in enumerate(base)]
    ours = [t.requires_grad_(True) for t in ours]
    ref = [t.detach().clone().requires_grad_(True) for t in base]
    o1 = FusedAdam(ours, lr=1e-2, eps=1e-15)
    o2 = torch.optim.Adam(ref, lr=1e-2, eps=1e-15)
    g = torch.Generator().manual_seed(5)
    for _ in range(4):
        for a, b in zip(ours, ref):
            gr = torch.randn(a.shape, generator=g).to(device)
            a.grad, b.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
    _compare(o1, o2, ours, ref)


def _densify_like(it, opt, params):
    """GaussianModel.cat_tensors_to_optimizer / _prune_optimizer on every group (gaussian_model.py:286-340):
    step 3 appends 17 new Gaussians with zero state, step 6 drops every third one."""
    if it not in (3, 6):
        return params
    out = []
    for group in opt.param_groups:
        p = group["params"][0]
        st = opt.state.get(p, None)
        if it == 3:
            gen = torch.Generator().manual_seed(p.numel())  # same rows for both optimizers
            ext = torch.randn((17,) + tuple(p.shape[1:]), generator=gen).to(p.device)
            new = torch.nn.Parameter(torch.cat((p.detach(), ext), 0).requires_grad_(True))
            if st is not None:
                st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(ext)), 0)
                st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(ext)), 0)
        else:
            keep = torch.arange(p.shape[0], device=p.device) % 3 != 0
            new = torch.nn.Parameter(p.detach()[keep].requires_grad_(True))
            if st is not None:
                st["exp_avg"] = st["exp_avg"][keep]
                st["exp_avg_sq"] = st["exp_avg_sq"][keep]
        if st is not None:
            del opt.state[p]
            opt.state[new] = st
        group["params"][0] = new
        out.append(new)
    return out


@pytest.mark.gpu
def test_fused_adam_survives_densification_state_surgery(device):
    P = 1001
    sizes = [(P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4)]
    _compare(*_run_pair(device, sizes, 9, mutate=_densify_like))


@pytest.mark.gpu
def test_fused_adam_state_dict_roundtrip_with_torch_adam(device):
    from gs_train import FusedAdam

    sizes = [(300, 3), (300, 1, 3), (300, 15, 3), (300, 1), (300, 3), (300, 4)]
    o1, o2, ours, ref = _run_pair(device, sizes, 3)
    # torch Adam -> FusedAdam and FusedAdam -> torch Adam, then continue both
    a = [t.detach().clone().requires_grad_(True) for t in ref]
    b = [t.detach().clone().requires_grad_(True) for t in ours]
    fa = FusedAdam(_groups(a), lr=0.0, eps=1e-15)
    fa.load_state_dict(o2.state_dict())
    ta = torch.optim.Adam(_groups(b), lr=0.0, eps=1e-15)
    ta.load_state_dict(o1.state_dict())
    g = torch.Generator().manual_seed(9)
    for _ in range(3):
        for x, y in zip(a, b):
            gr = torch.randn(x.shape, generator=g).to(device)
            x.grad, y.grad = gr.clone(), gr.clone()
        fa.step()
        ta.step()
    _compare(fa, ta, a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 255, 100_003])
def test_densify_stats_matches_train_py(device, P):
    from gs_train import add_densification_stats

    g = torch.Generator().manual_seed(P)
    radii = torch.randint(-2, 9, (P,), generator=g, dtype=torch.int32).clamp_min(0).to(device)

    class Model:
        pass

    ours, ref = Model(), Model()
    for m in (ours, ref):
        m.max_radii2D = (torch.rand(P, generator=torch.Generator().manual_seed(1)) * 6).floor().to(device)
        m.xyz_gradient_accum = torch.rand((P, 1), generator=torch.Generator().manual_seed(2)).to(device)
        m.denom = torch.randint(0, 5, (P, 1), generator=torch.Generator().manual_seed(3)).float().to(device)
    vs = torch.zeros((P, 3), device=device, requires_grad=True)
    vs.grad = torch.randn((P, 3), generator=g).to(device)
    for _ in range(2):
        add_densification_stats(ours, vs, radii)
        vis = radii > 0  # train.py:115-116 as written in the reference
        ref.max_radii2D[vis] = torch.max(ref.max_radii2D[vis], radii[vis])
        ref.xyz_gradient_accum[vis] += torch.norm(vs.grad[vis, :2], dim=-1, keepdim=True)
        ref.denom[vis] += 1
    assert torch.equal(ours.max_radii2D, ref.max_radii2D)
    assert torch.equal(ours.denom, ref.denom)
    torch.testing.assert_close(ours.xyz_gradient_accum, ref.xyz_gradient_accum, rtol=1e-6, atol=0)


def _raw_params(P, K, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = [torch.randn((P, 1, 3), generator=g), torch.randn((P, K, 3), generator=g), torch.randn((P, 1), generator=g) * 3,
         torch.randn((P, 3), generator=g) - 3, torch.randn((P, 4), generator=g)]
    if P > 2:
        t[4][1] = 0.0  # zero quaternion: F.normalize clamps the norm at 1e-12
        t[4][2] *= 1e-8
    return [x.to(device) for x in t]


@pytest.mark.gpu
@pytest.mark.parametrize("P,K", [(1, 15), (5, 0), (1001, 3), (4097, 8), (30011, 15)])
def test_activate_matches_gaussian_model_properties(device, P, K):
    from gs_train import activate

    raw = _raw_params(P, K, device, seed=P + K)
    a = [t.clone().requires_grad_(True) for t in raw]
    b = [t.clone().requires_grad_(True) for t in raw]
    ours = activate(*a)
    ref = (torch.cat((b[0], b[1]), dim=1), torch.sigmoid(b[2]), torch.exp(b[3]), torch.nn.functional.normalize(b[4]))
    assert torch.equal(ours[0], ref[0])
    for x, y in zip(ours[1:], ref[1:]):
        assert x.shape == y.shape
        torch.testing.assert_close(x, y, rtol=2e-6, atol=1e-30)
    g = torch.Generator().manual_seed(7)
    grads = [torch.randn(t.shape, generator=g).to(device) for t in ref]
    torch.autograd.backward(ours, grads)
    torch.autograd.backward(ref, grads)
    assert torch.equal(a[0].grad, b[0].grad) and torch.equal(a[1].grad, b[1].grad)
    for x, y in zip(a[2:], b[2:]):
        torch.testing.assert_close(x.grad, y.grad, rtol=1e-5, atol=1e-6 * float(y.grad.abs().max()))


@pytest.mark.gpu
def test_activate_partial_gradients(device):
    """Only shs and opacity reach the loss (e.g. cov3D precomputed): scale / rotation get no gradient."""
    from gs_train import activate

    raw = [t.requires_grad_(True) for t in _raw_params(300, 15, device)]
    shs, opac, scales, rots = activate(*raw)
    (shs.square().sum() + opac.sum()).backward()
    assert raw[3].grad is None and raw[4].grad is None
    torch.testing.assert_close(raw[1].grad, 2 * raw[1].detach(), rtol=0, atol=0)
    s = torch.sigmoid(raw[2].detach())
    torch.testing.assert_close(raw[2].grad, s * (1 - s), rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("P,K", [(1, 15), (5, 0), (1001, 3), (4097, 8), (30011, 15)])
def test_adam_step_activated_equals_activate_backward_then_step(device, P, K):
    """FusedAdam.step_activated (the activation adjoint inside the update, csrc/gs_train.hip
    AG_* modes) against activate()'s autograd backward followed by FusedAdam.step, over 3 steps
    with per-step learning rates: parameters and both moments bit-identical (the same float
    operations), the activated parameters' .grad left unset; xyz (plain mode) included."""
    from gs_train import FusedAdam, activate, activate_values

    raw = _raw_params(P, K, device, seed=3 * P + K)
    xyz0 = torch.randn((P, 3), generator=torch.Generator().manual_seed(5)).to(device)
    runs = []
    for fused_adjoint in (False, True):
        ps = [torch.nn.Parameter(t.clone()) for t in [xyz0] + raw]
        opt = FusedAdam([{"params": [p], "lr": lr} for p, lr in zip(ps, LRS)], lr=0.0, eps=1e-15)
        g = torch.Generator().manual_seed(11)
        for it in range(3):
            for grp, lr in zip(opt.param_groups, LRS):
                grp["lr"] = lr * (1.0 + 0.1 * it)
            outs_g = [torch.randn(s, generator=g).to(device) for s in ((P, 1 + K, 3), (P, 1), (P, 3), (P, 4))]
            gxyz = torch.randn((P, 3), generator=g).to(device)
            if fused_adjoint:
                acts = activate_values(*ps[1:])
                assert torch.equal(acts[0], torch.cat((ps[1], ps[2]), 1).detach())
                ps[0].grad = gxyz.clone()
                opt.step_activated({ps[1]: ("features_dc", outs_g[0]), ps[2]: ("features_rest", outs_g[0]),
                                    ps[3]: ("sigmoid", outs_g[1]), ps[4]: ("exp", outs_g[2]),
                                    ps[5]: ("normalize", outs_g[3])}, sh_coeffs=1 + K)
                assert all(p.grad is None for p in ps[1:])
            else:
                acts = activate(*ps[1:])
                torch.autograd.backward(acts, outs_g)
                ps[0].grad = gxyz.clone()
                opt.step()
            opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        runs.append((ps, opt))
    (pa, oa), (pb, ob) = runs
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
        sa, sb = oa.state[a], ob.state[b]
        assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])
        assert float(sa["step"]) == float(sb["step"]) == 3.0


def test_adam_step_activated_validation():
    """Argument checks of the C entry point run before any device work."""
    import ctypes

    from diff_gaussian_rasterization import _native

    lib = _native.load()
    one = (ctypes.c_void_p * 1)(ctypes.c_void_p(16))
    n = (ctypes.c_longlong * 1)(10)
    lr = (ctypes.c_double * 1)(1e-3)
    st = (ctypes.c_longlong * 1)(1)
    cast = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    for mode, coeffs, msg in ((9, 16, "unknown gradient mode"), (5, 16, "rows of 4"), (1, 16, "3 floats"),
                              (2, 16, "features_rest")):
        modes = (ctypes.c_int * 1)(mode)
        rc = lib.gs_adam_step_activated(1, cast(one), cast(one), cast(modes), coeffs, cast(one), cast(one), cast(n),
                                        cast(lr), cast(st), None, 0.9, 0.999, 1e-15, 0, None)
        assert rc != 0 and msg in _native.last_error(), _native.last_error()
