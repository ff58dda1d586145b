"""Cross-check the CPU oracle's compositing core and analytic backward against an independent dense
PyTorch restatement differentiated by autograd (tests/dense_ref.py).  This is what pins the
render fwd/bwd + preprocess bwd of the oracle, since the reference has no test or fixture for them
("parity unpinned" by the reference itself)."""
import math

import numpy as np
import pytest
import torch

import dense_ref
import gs_scenes


def _scene(P, W, H, deg, seed, scale_range=(0.02, 0.15), z_range=(2.0, 6.0)):
    cam = gs_scenes.identity_camera(W, H, fovy_deg=60.0)
    sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=seed, scale_range=scale_range, z_range=z_range)
    # keep centres well inside the frustum (the tx/tz clamp changes the gradient semantics)
    sc.means3D[:, 0] *= 0.85
    sc.means3D[:, 1] *= 0.85
    sc.opacities.clamp_(max=0.95)
    return cam, sc


def _oracle_scene(oracle, cam, sc, bg, colors=None, cov3D=None, mod=1.0, deg=None):
    deg = sc.sh_degree if deg is None else deg
    return oracle.Scene(bg=bg, means3D=sc.means3D.numpy(), opacities=sc.opacities.numpy(), W=cam.image_width,
                        H=cam.image_height, viewmatrix=cam.world_view_transform.numpy(),
                        projmatrix=cam.full_proj_transform.numpy(), campos=cam.camera_center.numpy(),
                        tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
                        shs=None if colors is not None else sc.shs.numpy(), sh_degree=deg,
                        colors_precomp=colors, scales=None if cov3D is not None else sc.scales.numpy(),
                        rotations=None if cov3D is not None else sc.rotations.numpy(), cov3D_precomp=cov3D,
                        scale_modifier=mod)


def _close(a, b, rtol=1e-5, frac=1e-5, name=""):
    """|a-b| <= rtol*|b| + frac*max|b| elementwise (fp32 oracle vs fp64 dense); default 1e-5 / 1e-5."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    tol = rtol * np.abs(b) + frac * max(np.abs(b).max(), 1e-30)
    bad = np.abs(a - b) > tol
    assert not bad.any(), f"{name}: {bad.sum()} / {bad.size} off, max |d| {np.abs(a - b).max():.3e}, max|ref| {np.abs(b).max():.3e}"


@pytest.mark.parametrize("deg,W,H,bgv", [(3, 70, 48, 0.0), (1, 64, 40, 0.3), (0, 33, 17, 1.0)])
def test_oracle_forward_backward_vs_dense_autograd(oracle, deg, W, H, bgv):
    cam, sc = _scene(40, W, H, deg, seed=deg + 11)
    bg = np.full(3, bgv, np.float32)
    osc = _oracle_scene(oracle, cam, sc, bg)
    fw = oracle.forward(osc)
    dpix = gs_scenes.dl_dimage(H, W, seed=3, scale=1.0).numpy()
    gr = oracle.backward(osc, dpix)

    d = torch.float64
    m3 = sc.means3D.to(d).requires_grad_(True)
    m2 = torch.zeros((40, 3), dtype=d, requires_grad=True)
    op = sc.opacities.to(d).requires_grad_(True)
    shs = sc.shs.to(d).requires_grad_(True)
    scl = sc.scales.to(d).requires_grad_(True)
    rot = sc.rotations.to(d).requires_grad_(True)
    img, radii = dense_ref.render(m3, m2, op[:, 0], cam.world_view_transform.to(d), cam.full_proj_transform.to(d),
                                  cam.camera_center.to(d), math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), W, H,
                                  torch.tensor(bg, dtype=d), shs=shs, deg=deg, scales=scl, rots=rot)
    assert fw["num_rendered"] > 0
    np.testing.assert_array_equal(fw["radii"], radii.numpy())
    _close(fw["color"], img.detach().numpy(), rtol=1e-5, frac=1e-5, name="image")
    (img * torch.tensor(dpix, dtype=d)).sum().backward()
    _close(gr["dmeans2D"][:, :2], m2.grad[:, :2].numpy(), name="dmeans2D")
    assert np.all(gr["dmeans2D"][:, 2] == 0)
    _close(gr["dopacity"], op.grad.numpy(), name="dopacity")
    _close(gr["dsh"], shs.grad.numpy(), name="dsh")
    _close(gr["dscales"], scl.grad.numpy(), name="dscales")
    _close(gr["drotations"], rot.grad.numpy(), name="drotations")
    _close(gr["dmeans3D"], m3.grad.numpy(), name="dmeans3D")


def test_oracle_precomputed_colors_and_cov3d_vs_dense(oracle):
    W, H = 48, 48
    cam, sc = _scene(30, W, H, 0, seed=5)
    g = torch.Generator().manual_seed(2)
    colors = torch.rand((30, 3), generator=g)
    cov = torch.tensor(oracle.cov3d(sc.scales.numpy(), 1.0, sc.rotations.numpy()))
    bg = np.array([0.1, 0.2, 0.3], np.float32)
    osc = _oracle_scene(oracle, cam, sc, bg, colors=colors.numpy(), cov3D=cov.numpy())
    fw = oracle.forward(osc)
    dpix = gs_scenes.dl_dimage(H, W, seed=4, scale=1.0).numpy()
    gr = oracle.backward(osc, dpix)
    d = torch.float64
    m3 = sc.means3D.to(d).requires_grad_(True)
    m2 = torch.zeros((30, 3), dtype=d, requires_grad=True)
    op = sc.opacities.to(d).requires_grad_(True)
    col = colors.to(d).requires_grad_(True)
    cv = cov.to(d).requires_grad_(True)
    img, radii = dense_ref.render(m3, m2, op[:, 0], cam.world_view_transform.to(d), cam.full_proj_transform.to(d),
                                  cam.camera_center.to(d), math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), W, H,
                                  torch.tensor(bg, dtype=d), colors=col, cov3D=cv)
    np.testing.assert_array_equal(fw["radii"], radii.numpy())
    _close(fw["color"], img.detach().numpy(), rtol=1e-5, frac=1e-5, name="image")
    (img * torch.tensor(dpix, dtype=d)).sum().backward()
    _close(gr["dcolors"], col.grad.numpy(), name="dcolors")
    _close(gr["dcov3D"], cv.grad.numpy(), name="dcov3D")
    _close(gr["dmeans3D"], m3.grad.numpy(), name="dmeans3D")
    _close(gr["dopacity"], op.grad.numpy(), name="dopacity")


def test_oracle_empty_scene_is_all_zero(oracle):
    cam = gs_scenes.identity_camera(32, 32)
    osc = oracle.Scene(bg=np.ones(3, np.float32), means3D=np.zeros((0, 3), np.float32),
                       opacities=np.zeros((0, 1), np.float32), W=32, H=32,
                       viewmatrix=cam.world_view_transform.numpy(), projmatrix=cam.full_proj_transform.numpy(),
                       campos=cam.camera_center.numpy(), tanfovx=0.5, tanfovy=0.5,
                       colors_precomp=np.zeros((0, 3), np.float32), cov3D_precomp=np.zeros((0, 6), np.float32))
    fw = oracle.forward(osc)
    assert fw["num_rendered"] == 0 and np.all(fw["color"] == 0)


def test_oracle_sorted_list_is_tile_depth_index_ordered(oracle):
    cam, sc = _scene(200, 96, 64, 0, seed=8)
    osc = _oracle_scene(oracle, cam, sc, np.zeros(3, np.float32))
    fw = oracle.forward(osc, intermediates=True)
    lst, rng, depth = fw["point_list"], fw["ranges"], fw["depth"]
    assert lst.shape[0] == fw["num_rendered"] == int(fw["tiles_touched"].sum())
    for t in range(rng.shape[0]):
        a, b = rng[t]
        ids = lst[a:b]
        keys = list(zip(depth[ids].view(np.uint32), ids))
        assert keys == sorted(keys)


def _wide_scene(P, W, H, deg, seed):
    """P Gaussians filling a W x H view: centres up to 1.6x the half-FoV (so a share of them sits past
    the 1.3x tx/tz clamp of the EWA Jacobian while their splats still reach the image), depths 1.5-6,
    scales 0.04-0.4 (log-uniform; x3 past the clamp), opacities uniform up to 0.999 (the 0.99 alpha clamp fires)."""
    cam = gs_scenes.identity_camera(W, H, fovy_deg=60.0)
    g = torch.Generator().manual_seed(seed)
    tx, ty = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
    z = 1.5 + 4.5 * torch.rand((P,), generator=g)
    x = (2 * torch.rand((P,), generator=g) - 1) * 1.6 * tx * z
    y = (2 * torch.rand((P,), generator=g) - 1) * 1.6 * ty * z
    sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=seed + 1, scale_range=(0.04, 0.4))
    sc.means3D = torch.stack([x, y, z], 1).contiguous()  # identity camera: world = camera space
    outside = (x.abs() > 1.3 * tx * z) | (y.abs() > 1.3 * ty * z)
    sc.scales[outside] *= 3.0  # big enough to reach into the image from past the clamp
    sc.opacities = (0.05 + 0.949 * torch.rand((P, 1), generator=g)).contiguous()
    return cam, sc


@pytest.mark.parametrize("deg,W,H,bgv,mod", [(3, 128, 128, 0.0, 1.0), (1, 128, 96, 0.4, 0.8)])
def test_oracle_vs_dense_500_gaussians_clamp_region(oracle, deg, W, H, bgv, mod):
    """The oracle's compositing core + analytic backward against the fp64 autograd restatement on 500
    Gaussians: the tx/tz clamp region, the 0.99 alpha clamp and saturated pixels (T < 1e-4 stop) are
    all exercised (asserted).  Tolerance 1e-5*|ref| + 1e-5*max|ref| (the north-star bound) on the
    image and every gradient, the covariance chain (dmeans3D, dscales, drotations) included."""
    P = 500
    cam, sc = _wide_scene(P, W, H, deg, seed=100 + deg)
    bg = np.full(3, bgv, np.float32)
    osc = _oracle_scene(oracle, cam, sc, bg, mod=mod)
    fw = oracle.forward(osc, intermediates=True)
    dpix = gs_scenes.dl_dimage(H, W, seed=7, scale=1.0).numpy()
    gr = oracle.backward(osc, dpix)

    d = torch.float64
    m3 = sc.means3D.to(d).requires_grad_(True)
    m2 = torch.zeros((P, 3), dtype=d, requires_grad=True)
    op = sc.opacities.to(d).requires_grad_(True)
    shs = sc.shs.to(d).requires_grad_(True)
    scl = sc.scales.to(d).requires_grad_(True)
    rot = sc.rotations.to(d).requires_grad_(True)
    img, radii = dense_ref.render(m3, m2, op[:, 0], cam.world_view_transform.to(d), cam.full_proj_transform.to(d),
                                  cam.camera_center.to(d), math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), W, H,
                                  torch.tensor(bg, dtype=d), shs=shs, deg=deg, scales=scl, rots=rot, mod=mod)
    np.testing.assert_array_equal(fw["radii"], radii.numpy())
    vis = fw["radii"] > 0
    # coverage of the regimes this test is for
    z = sc.means3D[:, 2].numpy()
    clamped = (np.abs(sc.means3D[:, 0].numpy() / z) > 1.3 * math.tan(cam.FoVx / 2)) | \
              (np.abs(sc.means3D[:, 1].numpy() / z) > 1.3 * math.tan(cam.FoVy / 2))
    assert (clamped & vis).sum() >= 10, f"only {(clamped & vis).sum()} visible Gaussians in the clamp region"
    assert (sc.opacities.numpy()[vis, 0] > 0.99).sum() >= 3
    assert (fw["final_T"] < 1e-4).sum() == 0 and (fw["final_T"] < 1e-2).mean() > 0.01  # near-saturated pixels
    _close(fw["color"], img.detach().numpy(), rtol=1e-5, frac=1e-5, name="image")
    (img * torch.tensor(dpix, dtype=d)).sum().backward()
    t = dict(rtol=1e-5, frac=1e-5)
    _close(gr["dmeans2D"][:, :2], m2.grad[:, :2].numpy(), name="dmeans2D", **t)
    _close(gr["dopacity"], op.grad.numpy(), name="dopacity", **t)
    _close(gr["dsh"], shs.grad.numpy(), name="dsh", **t)
    chain = dict(rtol=1e-5, frac=1e-5)
    _close(gr["dscales"], scl.grad.numpy(), name="dscales", **chain)
    _close(gr["drotations"], rot.grad.numpy(), name="drotations", **chain)
    _close(gr["dmeans3D"], m3.grad.numpy(), name="dmeans3D", **chain)
    # the clamp region's Gaussians carry gradient through the clamped Jacobian too
    assert np.abs(gr["dmeans3D"][clamped & vis]).max() > 0


def test_oracle_f32_accumulation_probe(oracle):
    """oracle.backward_f32_acc (the fp32-order noise probe of the GPU chain checks) changes only the
    summation precision: the forward is untouched, the fp64 default comes back afterwards, and the
    two backward answers differ by fp32 rounding only on a well-conditioned scene."""
    cam, sc = _scene(400, 96, 80, 2, seed=5)
    osc = _oracle_scene(oracle, cam, sc, np.zeros(3, np.float32))
    dpix = gs_scenes.dl_dimage(80, 96, seed=6).numpy()
    g64 = oracle.backward(osc, dpix)
    g32 = oracle.backward_f32_acc(osc, dpix)
    again = oracle.backward(osc, dpix)
    for k in ("dmeans2D", "dopacity", "dmeans3D", "dsh", "dscales", "drotations"):
        np.testing.assert_array_equal(again[k], g64[k])  # default restored
        _close(g32[k], g64[k], rtol=1e-4, frac=1e-5, name=k)
    assert any(not np.array_equal(g32[k], g64[k]) for k in ("dmeans2D", "dsh", "dscales"))


def test_dense_local_compositor_equals_dense():
    """dense_ref.render_local (the rect-local compositor the GPU test runs at thousands of Gaussians)
    is the same function as dense_ref.render: image and every autograd gradient agree to fp64
    round-off on a small scene."""
    cam, sc = _scene(60, 70, 45, 3, seed=5)
    d = torch.float64
    outs = []
    for fn in (dense_ref.render, dense_ref.render_local):
        m3 = sc.means3D.to(d).requires_grad_(True)
        op = sc.opacities.to(d).requires_grad_(True)
        shs = sc.shs.to(d).requires_grad_(True)
        scl = sc.scales.to(d).requires_grad_(True)
        rot = sc.rotations.to(d).requires_grad_(True)
        m2 = torch.zeros((60, 3), dtype=d, requires_grad=True)
        res = fn(m3, m2, op, cam.world_view_transform.to(d), cam.full_proj_transform.to(d), cam.camera_center.to(d),
                 math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 70, 45, torch.full((3,), 0.2, dtype=d), shs=shs,
                 deg=3, scales=scl, rots=rot)
        img = res[0]
        dpix = gs_scenes.dl_dimage(45, 70, seed=9, scale=1.0).to(d)
        (img * dpix).sum().backward()
        outs.append([img.detach(), m3.grad, m2.grad, op.grad, shs.grad, scl.grad, rot.grad])
    for a, b in zip(*outs):
        assert torch.allclose(a, b, rtol=1e-10, atol=1e-13)
