"""densify_and_prune (gs_train.densify_and_prune, csrc/gs_densify.hip) against the reference.

Chain of pins:
  * oracle/densify_oracle.py (a restatement of scene/gaussian_model.py:258-403) reproduces the
    reference's own GaussianModel.densify_and_prune bit for bit on CPU
    (tests/golden/densify_golden.npz, made by tests/golden/make_golden.py: same inputs, same
    torch.manual_seed before the call so torch.normal draws the same split samples);
  * on the GPU the HIP path is compared with the oracle on the same inputs and the same CUDA
    generator state.  Every output row is a copy, a zero or computed with the reference's float32
    operation order, so all tensors are compared bit-exactly except the split children's xyz
    (R(q) @ sample + xyz: torch.bmm's reduction order is the library's), which is held to
    rtol 1e-6 / atol 1e-6.  (The child scaling divides by 0.8 N the way torch does on the device:
    a tensor divided by a Python scalar is multiplied by the float reciprocal there.)
"""
import numpy as np
import pytest
import torch

from oracle import densify_oracle as DO

G = np.load(__file__.rsplit("/", 1)[0] + "/golden/densify_golden.npz")
LRS = [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3]


class Model:
    pass


def _model_from(arrays: dict, device, with_state=True, step=2.0):
    m = Model()
    m.percent_dense = 0.01
    groups = []
    for n, a, lr in zip(DO.NAMES, DO.ATTRS, LRS):
        p = torch.nn.Parameter(torch.tensor(arrays[n]).to(device).requires_grad_(True))
        setattr(m, a, p)
        groups.append({"params": [p], "lr": lr, "name": n})
    m.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
    if with_state:
        for grp in m.optimizer.param_groups:
            n = grp["name"]
            m.optimizer.state[grp["params"][0]] = {
                "step": torch.tensor(step),
                "exp_avg": torch.tensor(arrays[f"{n}_exp_avg"]).to(device),
                "exp_avg_sq": torch.tensor(arrays[f"{n}_exp_avg_sq"]).to(device)}
    m.xyz_gradient_accum = torch.tensor(arrays["accum"]).to(device)
    m.denom = torch.tensor(arrays["denom"]).to(device)
    m.max_radii2D = torch.tensor(arrays["max_radii2D"]).to(device)
    return m


def _golden_inputs(case):
    pre = f"{case}_in_"
    return {k[len(pre):]: G[k] for k in G.files if k.startswith(pre)}


def _args(case):
    thr, min_op, extent, screen, seed = G[f"{case}_args"]
    return float(thr), float(min_op), float(extent), (None if screen < 0 else float(screen)), int(seed)


def _check_model_structure(m):
    for grp in m.optimizer.param_groups:
        p = grp["params"][0]
        assert getattr(m, DO.ATTRS[DO.NAMES.index(grp["name"])]) is p
        assert isinstance(p, torch.nn.Parameter) and p.requires_grad
    n = m._xyz.shape[0]
    assert m.xyz_gradient_accum.shape == (n, 1) and m.denom.shape == (n, 1) and m.max_radii2D.shape == (n,)
    assert not m.xyz_gradient_accum.any() and not m.denom.any() and not m.max_radii2D.any()


@pytest.mark.parametrize("case", ["a", "b"])
def test_oracle_matches_reference_golden(case):
    thr, min_op, extent, screen, seed = _args(case)
    m = _model_from(_golden_inputs(case), "cpu")
    torch.manual_seed(seed)
    DO.densify_and_prune(m, thr, min_op, extent, screen)
    _check_model_structure(m)
    assert m._xyz.shape[0] == int(G[f"{case}_out_sizes"][0])
    for grp in m.optimizer.param_groups:
        n = grp["name"]
        np.testing.assert_array_equal(grp["params"][0].detach().numpy(), G[f"{case}_out_{n}"], err_msg=n)
        st = m.optimizer.state[grp["params"][0]]
        np.testing.assert_array_equal(st["exp_avg"].numpy(), G[f"{case}_out_{n}_exp_avg"], err_msg=n)
        np.testing.assert_array_equal(st["exp_avg_sq"].numpy(), G[f"{case}_out_{n}_exp_avg_sq"], err_msg=n)
        assert float(st["step"]) == float(G[f"{case}_out_{n}_step"])


def test_densify_abi_validation_without_gpu():
    from diff_gaussian_rasterization import _native

    lib = _native.load()
    assert lib.gs_densify_block_count(0) == 0 and lib.gs_densify_block_count(257) == 2
    rc = lib.gs_densify_classify(10, None, None, None, None, 2e-4, 0.02, 0.005, 0.2, 0, 0.0, 2, None, None, None, None)
    assert rc != 0 and "missing" in _native.last_error()


def _compare_models(ours, ref, xyz_tol=True):
    assert ours._xyz.shape == ref._xyz.shape, (ours._xyz.shape, ref._xyz.shape)
    _check_model_structure(ours)
    for g1, g2 in zip(ours.optimizer.param_groups, ref.optimizer.param_groups):
        n = g1["name"]
        a, b = g1["params"][0].detach(), g2["params"][0].detach()
        if n == "xyz" and xyz_tol:
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6, msg=n)
        else:
            assert torch.equal(a, b), f"{n}: max |d| {(a - b).abs().max().item():.3e}"
        s1, s2 = ours.optimizer.state.get(g1["params"][0]), ref.optimizer.state.get(g2["params"][0])
        assert (s1 is None) == (s2 is None)
        if s1 is not None:
            assert torch.equal(s1["exp_avg"], s2["exp_avg"]), n
            assert torch.equal(s1["exp_avg_sq"], s2["exp_avg_sq"]), n
            assert float(s1["step"]) == float(s2["step"])


def _run_both(arrays, device, thr, min_op, extent, screen, seed, N=2, with_state=True):
    from gs_train import densify_and_prune

    ours = _model_from(arrays, device, with_state)
    ref = _model_from(arrays, device, with_state)
    torch.cuda.manual_seed(seed)
    DO.densify_and_prune(ref, thr, min_op, extent, screen, N)
    torch.cuda.manual_seed(seed)
    densify_and_prune(ours, thr, min_op, extent, screen, N)
    return ours, ref


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["a", "b"])
def test_densify_matches_oracle_on_golden_inputs(device, case):
    thr, min_op, extent, screen, seed = _args(case)
    _compare_models(*_run_both(_golden_inputs(case), device, thr, min_op, extent, screen, seed))


def _random_arrays(P, seed):
    import math

    g = torch.Generator().manual_seed(seed)
    d = {
        "xyz": torch.randn((P, 3), generator=g),
        "f_dc": torch.randn((P, 1, 3), generator=g),
        "f_rest": torch.randn((P, 15, 3), generator=g),
        "opacity": torch.randn((P, 1), generator=g) * 3,
        # log-uniform in [0.002, 0.05] per axis: clone / split / big all present at extent 0.5
        "scaling": math.log(0.002) + torch.rand((P, 3), generator=g) * math.log(25.0),
        "rotation": torch.randn((P, 4), generator=g),
    }
    for n in DO.NAMES:
        d[f"{n}_exp_avg"] = torch.randn(d[n].shape, generator=g) * 1e-3
        d[f"{n}_exp_avg_sq"] = torch.rand(d[n].shape, generator=g) * 1e-6
    d["denom"] = torch.randint(0, 4, (P, 1), generator=g).float()
    d["accum"] = torch.rand((P, 1), generator=g) * 4e-4 * d["denom"]
    d["max_radii2D"] = torch.randint(0, 40, (P,), generator=g).float()
    return {k: v.numpy() for k, v in d.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("P,N,screen,with_state", [(1, 2, 20.0, True), (255, 3, None, True),
                                                   (200_003, 2, 20.0, True), (5000, 2, 20.0, False)])
def test_densify_matches_oracle_random(device, P, N, screen, with_state):
    arrays = _random_arrays(P, seed=P)
    ours, ref = _run_both(arrays, device, 2e-4, 0.005, 0.5, screen, seed=7, N=N, with_state=with_state)
    _compare_models(ours, ref)
