"""GPU tests of the depth-slab forward (ABI v12, gs_set_slabs; gs_forward.hip fwd_bin_render_slabs).

A view with many instances per tile bins and renders its nearest depth ranks first (about a quarter
of the instances), then bins the remaining ranks only into tiles that still have a running pixel and
resumes those from the saved pixel state.  Per pixel the entries and their order are those of the
full list up to where the pixel stops, so every output must be bit-identical to the one-list
forward: image, radii, final_T, n_contrib and every gradient.  The slabs are forced on here
(gs_set_slabs(2)) for scenes of every depth complexity: deep (most tiles saturate in the near slab),
shallow (few do), mixed with large splats, plus the split SH rows and the bounded forward.  The
full C5 run against the oracle (test_gpu_parity.py) uses them by size."""
import pytest
import torch

import gs_scenes

pytestmark = pytest.mark.gpu


def _lib():
    from diff_gaussian_rasterization import _native

    return _native.load()


def _run(cam, sc, device, dpix, slabs, cap=None, split=False):
    from diff_gaussian_rasterization import GaussianRasterizer, _C, last_num_rendered

    prev = _lib().gs_set_slabs(slabs)
    try:
        s = gs_scenes.raster_settings_for(cam, sc.sh_degree, device=device)
        d = sc.to(device)
        p = [t.clone().requires_grad_(True) for t in (d.means3D, d.shs, d.opacities, d.scales, d.rotations)]
        m2 = torch.zeros_like(p[0], requires_grad=True)
        kw = {}
        if split:
            kw["sh_split"] = (p[1].detach()[:, :1].contiguous(), p[1].detach()[:, 1:].contiguous())
        img, radii = GaussianRasterizer(s)(means3D=p[0], means2D=m2, opacities=p[2], shs=p[1], scales=p[3],
                                           rotations=p[4], binning_capacity=cap, **kw)
        img.backward(dpix)
        # the image buffer's per-pixel outputs (the list itself differs by design)
        e = torch.Tensor([])
        num, _, _, geom, binb, imgb = _C.rasterize_gaussians(
            s.bg, d.means3D, e, d.opacities, d.scales, d.rotations, s.scale_modifier, e, s.viewmatrix, s.projmatrix,
            s.tanfovx, s.tanfovy, s.image_height, s.image_width, d.shs, sc.sh_degree, s.campos, False, False,
            capacity=cap)
        ex = _C.debug_export(sc.P, cam.image_width, cam.image_height, num, geom, binb, imgb, device)
        torch.cuda.synchronize()
        n = last_num_rendered()
        return [img.detach(), radii, ex["final_T"], ex["n_contrib"], m2.grad] + [t.grad for t in p], n
    finally:
        _lib().gs_set_slabs(prev)


def _scene(kind, device):
    if kind == "deep":  # C5's depth complexity at 1/6 of its resolution (scales x 6, 1/34 of the
        # Gaussians): most tiles saturate within the near slab
        cam = gs_scenes.identity_camera(320, 192)
        sc = gs_scenes.random_gaussians(150_000, 3, cam=cam, seed=31, scale_range=(0.03, 0.18))
    elif kind == "shallow":  # few layers: most tiles keep running pixels into the far slab
        cam = gs_scenes.identity_camera(640, 360)
        sc = gs_scenes.random_gaussians(20_000, 3, cam=cam, seed=32)
    else:  # many small splats plus large ones spanning dozens of tiles
        cam = gs_scenes.identity_camera(640, 360)
        small = gs_scenes.random_gaussians(150_000, 2, cam=cam, seed=33)
        big = gs_scenes.random_gaussians(80, 2, cam=cam, seed=34, scale_range=(0.3, 1.5), z_range=(2.0, 6.0))
        sc = gs_scenes.concat_scenes(small, big)
    return cam, sc


@pytest.mark.parametrize("kind", ["deep", "shallow", "mixed"])
def test_slabs_equal_one_list_forward(device, kind):
    cam, sc = _scene(kind, device)
    dpix = gs_scenes.dl_dimage(cam.image_height, cam.image_width, seed=35).to(device)
    ref, n = _run(cam, sc, device, dpix, slabs=0)
    got, n2 = _run(cam, sc, device, dpix, slabs=2)
    assert n == n2 and n > 0
    names = ["image", "radii", "final_T", "n_contrib", "means2D", "means3D", "shs", "opacities", "scales",
             "rotations"]
    for name, a, b in zip(names, ref, got):
        assert torch.equal(a, b), (kind, name, float((a.double() - b.double()).abs().max()))


def test_slabs_with_split_sh_and_bounded_forward(device):
    cam, sc = _scene("deep", device)
    dpix = gs_scenes.dl_dimage(cam.image_height, cam.image_width, seed=36).to(device)
    ref, n = _run(cam, sc, device, dpix, slabs=0)
    got, _ = _run(cam, sc, device, dpix, slabs=2, split=True)
    for k, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), ("split", k)
    got, _ = _run(cam, sc, device, dpix, slabs=2, cap=int(n * 1.2))
    for k, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), ("bounded", k)
    from diff_gaussian_rasterization import bounded_status

    assert bounded_status() == (0, 0)


def test_slab_binning_keeps_only_walkable_instances(device):
    """The deep scene's combined list is much shorter than num_rendered (the skipped instances lie in
    tiles whose every pixel stopped in the near slab), and every tile's walk stays within it."""
    from diff_gaussian_rasterization import _C

    cam, sc = _scene("deep", device)
    prev = _lib().gs_set_slabs(2)
    try:
        s = gs_scenes.raster_settings_for(cam, sc.sh_degree, device=device)
        d = sc.to(device)
        e = torch.Tensor([])
        num, _, _, geom, binb, imgb = _C.rasterize_gaussians(
            s.bg, d.means3D, e, d.opacities, d.scales, d.rotations, s.scale_modifier, e, s.viewmatrix, s.projmatrix,
            s.tanfovx, s.tanfovy, s.image_height, s.image_width, d.shs, sc.sh_degree, s.campos, False, False)
        ex = _C.debug_export(sc.P, cam.image_width, cam.image_height, num, geom, binb, imgb, device)
        torch.cuda.synchronize()
    finally:
        _lib().gs_set_slabs(prev)
    rg = ex["ranges"].to(torch.int64)
    kept = int(rg[:, 1].max())
    assert kept < 0.75 * num, (kept, num)
    W, H = cam.image_width, cam.image_height
    gx, gy = (W + 15) // 16, (H + 15) // 16
    nc = torch.zeros((gy * 16, gx * 16), dtype=torch.int64, device=device)
    nc[:H, :W] = ex["n_contrib"].to(torch.int64)
    tmax = nc.view(gy, 16, gx, 16).amax(dim=(1, 3)).reshape(-1)
    assert bool((tmax <= rg[:, 1] - rg[:, 0]).all())
    print(f"\n[slabs] kept {kept} of {num} instances ({kept / num:.1%})")
