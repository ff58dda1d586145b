"""The settings and inputs the reference's render() adapter hands to the rasterizer, pinned by a
fixture the reference itself produced (tests/golden/render_golden.npz, tests/golden/make_golden.py
render_vectors: /root/reference/gaussian_renderer/__init__.py:18-100 driven with the reference's
own Camera, scene/cameras.py:17-57, and GaussianModel getters, scene/gaussian_model.py:95-118,
with a recording stand-in for the rasterizer).

CPU: gs_scenes' camera builder + raster_settings_for reproduce every GaussianRasterizationSettings
field bit for bit (tanfov, the W2C^T matrix, full_proj_transform = W2C^T (x) P^T via bmm,
campos = inverse()[3, :3]).
GPU: gs_train.render_inputs (the HIP activations) against the getters' tensors, and the recorded
settings + inputs (including the Python colour / covariance paths, scale_modifier 0.7, a
non-black background) through GaussianRasterizer against the oracle."""
import math
import os

import numpy as np
import pytest
import torch

import gs_scenes

GOLD = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "render_golden.npz"))
CASES = sorted({k.split("_case")[0] for k in GOLD.files if k.endswith("_case")})
RING = {  # case -> how the synthetic workloads build that camera
    "c4v3": lambda W, H, fy: gs_scenes.circle_cameras(8, 6.0, W, H, fovy_deg=fy)[3],
    "ring_py": lambda W, H, fy: gs_scenes.look_at_camera((1.5, -0.4, -3.0), (0.1, 0.2, 0.3), W, H, fy),
}


def _case(name):
    W, H, fovy_deg, deg_act, deg_max, mod, cov_py, sh_py = GOLD[f"{name}_case"]
    return int(W), int(H), float(fovy_deg), int(deg_act), int(deg_max), float(mod), bool(cov_py), bool(sh_py)


def _camera(name):
    W, H, fy = _case(name)[:3]
    return RING[name](W, H, fy) if name in RING else gs_scenes.identity_camera(W, H, fy)


def _settings(name, device):
    W, H, fy, deg_act, _, mod, _, _ = _case(name)
    return gs_scenes.raster_settings_for(_camera(name), deg_act, bg=torch.tensor(GOLD[f"{name}_bg"], device=device),
                                         scale_modifier=mod, device=device)


def test_fixture_covers_the_workload_cameras():
    assert {"c1", "c2", "c3", "c4v3", "ring_py"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_raster_settings_bitwise_equal_reference_render(name):
    cam = _camera(name)
    np.testing.assert_array_equal(np.array([cam.FoVx, cam.FoVy]), GOLD[f"{name}_fov"])
    s = _settings(name, "cpu")
    assert (s.image_height, s.image_width) == tuple(int(v) for v in GOLD[f"{name}_hw"])
    assert (s.tanfovx, s.tanfovy) == tuple(float(v) for v in GOLD[f"{name}_tanfov"])
    for k in ("bg", "viewmatrix", "projmatrix", "campos"):
        got = getattr(s, k)
        assert got.dtype == torch.float32, k
        np.testing.assert_array_equal(got.numpy(), GOLD[f"{name}_{k}"], err_msg=k)
    mod, deg, pref, dbg = GOLD[f"{name}_scalars"]
    assert (s.scale_modifier, s.sh_degree, s.prefiltered, s.debug) == (mod, int(deg), bool(pref), bool(dbg))


def test_reference_inputs_follow_the_render_paths():
    """Which optional inputs render() passes: shs + scales/rotations by default, colors_precomp /
    cov3D_precomp with convert_SHs_python / compute_cov3D_python (gaussian_renderer/__init__.py:59-82)."""
    for name in CASES:
        cov_py, sh_py = _case(name)[6:8]
        has = lambda k: f"{name}_in_{k}" in GOLD.files  # noqa: E731
        assert has("means3D") and has("means2D") and has("opacities")
        assert has("cov3D_precomp") == cov_py and has("scales") == (not cov_py) and has("rotations") == (not cov_py)
        assert has("colors_precomp") == sh_py and has("shs") == (not sh_py)
        assert not GOLD[f"{name}_in_means2D"].any()


# ---------------------------------------------------------------- GPU


def _params(name, device):
    return [torch.tensor(GOLD[f"{name}_param{p}"], device=device) for p in
            ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")]


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_render_inputs_match_reference_getters(device, name):
    """gs_train.render_inputs (k_activate_fwd) vs GaussianModel.get_xyz / get_features / get_opacity
    / get_scaling / get_rotation as render() read them (tolerances as tests/test_train_updates.py)."""
    import gs_train

    xyz, dc, rest, o, s, q = _params(name, device)

    class PC:
        _xyz, _features_dc, _features_rest, _opacity, _scaling, _rotation = xyz, dc, rest, o, s, q

    m3, shs, opac, scales, rots = gs_train.render_inputs(PC)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m3.cpu().numpy(), GOLD[f"{name}_in_means3D"])
    np.testing.assert_allclose(opac.cpu().numpy(), GOLD[f"{name}_in_opacities"], rtol=2e-6, atol=0)
    if f"{name}_in_shs" in GOLD.files:
        np.testing.assert_array_equal(shs.cpu().numpy(), GOLD[f"{name}_in_shs"])
    if f"{name}_in_scales" in GOLD.files:
        np.testing.assert_allclose(scales.cpu().numpy(), GOLD[f"{name}_in_scales"], rtol=2e-6, atol=0)
        np.testing.assert_allclose(rots.cpu().numpy(), GOLD[f"{name}_in_rotations"], rtol=2e-6, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_reference_render_call_through_rasterizer_vs_oracle(oracle, device, name):
    """The exact settings and inputs render() produced, through the drop-in GaussianRasterizer
    (exact numerics mode): image bit-exact vs the oracle, gradients at the backward tolerance
    1e-5*|ref| + 1e-5*max|ref|; the conic -> covariance chain (means3D, scales, rotations, cov3D) at
    1e-5*|ref| + 1e-4*max|ref|, as test_large_and_elongated_splats: the fixture's log-normal
    scales include splats far larger than the image (conditioning)."""
    from diff_gaussian_rasterization import GaussianRasterizer, _native

    lib = _native.load()
    prev = lib.gs_set_exact_exp(1)
    try:
        W, H, _, deg_act, _, mod, _, _ = _case(name)
        s = _settings(name, device)
        ins = {k[len(name) + 4:]: GOLD[k] for k in GOLD.files if k.startswith(f"{name}_in_")}
        leaves = {k: torch.tensor(v, device=device).requires_grad_(True) for k, v in ins.items()}
        img, radii = GaussianRasterizer(s)(**leaves)
        dpix = gs_scenes.dl_dimage(H, W, seed=5, scale=1.0).numpy()
        (img * torch.tensor(dpix, device=device)).sum().backward()
        torch.cuda.synchronize()
        cam = _camera(name)
        osc = oracle.Scene(bg=GOLD[f"{name}_bg"], means3D=ins["means3D"], opacities=ins["opacities"], W=W, H=H,
                           viewmatrix=cam.world_view_transform.numpy(), projmatrix=cam.full_proj_transform.numpy(),
                           campos=cam.camera_center.numpy(), tanfovx=math.tan(cam.FoVx / 2),
                           tanfovy=math.tan(cam.FoVy / 2), shs=ins.get("shs"), sh_degree=deg_act,
                           colors_precomp=ins.get("colors_precomp"), scales=ins.get("scales"),
                           rotations=ins.get("rotations"), cov3D_precomp=ins.get("cov3D_precomp"), scale_modifier=mod)
        ofw = oracle.forward(osc)
        assert int((radii > 0).sum()) > 0
        np.testing.assert_array_equal(radii.cpu().numpy(), ofw["radii"])
        np.testing.assert_array_equal(img.detach().cpu().numpy(), ofw["color"])
        gr = oracle.backward(osc, dpix)
        pairs = [("means2D", "dmeans2D"), ("opacities", "dopacity"), ("means3D", "dmeans3D"), ("shs", "dsh"),
                 ("colors_precomp", "dcolors"), ("scales", "dscales"), ("rotations", "drotations"),
                 ("cov3D_precomp", "dcov3D")]
        for k, o in pairs:
            if k not in leaves:
                continue
            g = leaves[k].grad.detach().cpu().numpy().astype(np.float64)
            r = np.asarray(gr[o], np.float64).reshape(g.shape)
            frac = 1e-4 if k in ("means3D", "scales", "rotations", "cov3D_precomp") else 1e-5
            tol = 1e-5 * np.abs(r) + frac * max(np.abs(r).max(), 1e-30)
            assert (np.abs(g - r) <= tol).all(), f"{k}: max|d| {np.abs(g - r).max():.3e} max|ref| {np.abs(r).max():.3e}"
    finally:
        lib.gs_set_exact_exp(prev)
