"""GPU tests of the torch C++ host path (diff_gaussian_rasterization._gs_ext, csrc/gs_torch_ext.cpp)
and of the forward it runs, gs_forward_counted (ABI 14: every launch queued, the instance count read
back at the end, the binning buffer sized ahead from the last count).

  - the extension is the path a plain GaussianRasterizer call takes on a GPU box;
  - its outputs and gradients are bit-identical to the ctypes two-call path (gs_forward_preprocess
    + gs_forward_render), for the concatenated and the split SH rows, and num_rendered is the exact
    instance count (upstream semantics), not the capacity;
  - a forward whose count outgrows the estimate (the fallback: the same geometry binned again into
    an exact buffer) and one far below it (a larger layout than its count) give the same bits;
  - debug_export reads a counted forward's buffers (layout count vs num_rendered);
  - a timed-out look-back in a forward that outgrew its estimate fails in that forward, once (the
    skipped render's flags are read before re-binning), and the next call is clean;
  - a deferred GradBucket's per-Gaussian pass runs through the ext, bit-identical to ctypes.
"""
import pytest
import torch

import gs_scenes

pytestmark = pytest.mark.gpu

W, H = 320, 240


def _leaves(d):
    return [d.means3D.clone().requires_grad_(True), d.shs.clone().requires_grad_(True),
            d.opacities.clone().requires_grad_(True), d.scales.clone().requires_grad_(True),
            d.rotations.clone().requires_grad_(True)]


def _fwd_bwd(rast, d, dpix, split=False):
    p = _leaves(d)
    m2 = torch.zeros_like(p[0], requires_grad=True)
    kw = {}
    if split:
        kw["sh_split"] = (p[1].detach()[:, :1].contiguous(), p[1].detach()[:, 1:].contiguous())
    img, radii = rast(means3D=p[0], means2D=m2, opacities=p[2], shs=p[1], scales=p[3], rotations=p[4], **kw)
    img.backward(dpix)
    torch.cuda.synchronize()
    return [img.detach(), radii, m2.grad] + [t.grad for t in p]


def _assert_same(ref, got, what):
    for k, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), (what, k, float((a.float() - b.float()).abs().max()))


def _ext():
    from diff_gaussian_rasterization import _C

    assert _C._EXT is not None, "the torch C++ host path (_gs_ext) is not loaded on this GPU box"
    return _C


def test_ext_is_the_eager_path(device):
    _C = _ext()
    import diff_gaussian_rasterization as dgr

    d = gs_scenes.random_gaussians(5_000, 3, seed=1, ball_radius=2.0).to(device)
    cam = gs_scenes.circle_cameras(1, 6.0, W, H)[0]
    rast = dgr.GaussianRasterizer(gs_scenes.raster_settings_for(cam, 3, device=device))
    calls = []
    real = _C._EXT

    class Spy:
        def __getattr__(self, name):
            calls.append(name)
            return getattr(real, name)

    _C._EXT = Spy()
    try:
        _fwd_bwd(rast, d, gs_scenes.dl_dimage(H, W, seed=2).to(device))
    finally:
        _C._EXT = real
    assert calls == ["forward", "backward"]


@pytest.mark.parametrize("split", [False, True], ids=["concat_sh", "split_sh"])
def test_counted_forward_equals_two_call_forward(device, split, monkeypatch):
    _C = _ext()
    import diff_gaussian_rasterization as dgr

    d = gs_scenes.random_gaussians(20_000, 3, seed=5, ball_radius=2.0).to(device)
    dpix = gs_scenes.dl_dimage(H, W, seed=3).to(device)
    dev = torch.device(device).index or 0
    for cam in gs_scenes.circle_cameras(3, 6.0, W, H):
        rast = dgr.GaussianRasterizer(gs_scenes.raster_settings_for(cam, 3, device=device))
        with monkeypatch.context() as m:
            m.setattr(_C, "_EXT", None)
            ref = _fwd_bwd(rast, d, dpix, split)
            n = dgr.last_num_rendered()
        # estimates: none (two-call path), about right, far above, below the count (fallback)
        P = d.means3D.shape[0]
        for est in (0, n, 4 * n + 100_000, n // 3):
            _C._EXT.set_count_estimate(dev, P, W, H, est)
            got = _fwd_bwd(rast, d, dpix, split)
            _assert_same(ref, got, ("estimate", est))
            assert dgr.last_num_rendered() == n  # exact, not the capacity
            e = _C._EXT.count_estimate(dev, P, W, H)
            assert e >= n and (est > n or e == n), (est, e, n)  # the recent maximum


def test_counted_forward_buffers_and_debug_export(device):
    _C = _ext()
    d = gs_scenes.random_gaussians(8_000, 3, seed=7, ball_radius=2.0).to(device)
    cam = gs_scenes.circle_cameras(1, 6.0, W, H)[0]
    s = gs_scenes.raster_settings_for(cam, 3, device=device)
    args = (s.bg, d.means3D, torch.empty(0, device=device), d.opacities, d.scales, d.rotations, s.scale_modifier,
            torch.empty(0, device=device), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, d.shs,
            s.sh_degree, s.campos, s.prefiltered, False)
    dev = torch.device(device).index or 0
    P = d.means3D.shape[0]
    _C._EXT.set_count_estimate(dev, P, W, H, 0)
    n0, img0, radii0, geom0, bin0, imgbuf0 = _C.rasterize_gaussians(*args)
    _C._EXT.set_count_estimate(dev, P, W, H, 5 * n0)
    n1, img1, radii1, geom1, bin1, imgbuf1 = _C.rasterize_gaussians(*args)
    assert n1 == n0 and torch.equal(img0, img1) and torch.equal(radii0, radii1)
    assert bin1.numel() > bin0.numel()  # laid out for the capacity
    L = _C.binning_layout_count(n1, bin1, W, H)
    assert L > n1 and _C._lib.gs_binning_buffer_bytes(L, W, H) == bin1.numel()
    assert _C.binning_layout_count(n0, bin0, W, H) == n0
    e0 = _C.debug_export(d.means3D.shape[0], W, H, n0, geom0, bin0, imgbuf0, d.means3D.device)
    e1 = _C.debug_export(d.means3D.shape[0], W, H, n1, geom1, bin1, imgbuf1, d.means3D.device)
    torch.cuda.synchronize()
    for k in e0:
        assert torch.equal(e0[k], e1[k]), k
    with pytest.raises(RuntimeError, match="too small"):
        _C.binning_layout_count(n0 + 1_000_000, bin0, W, H)


def test_short_forward_with_timed_out_lookback_fails_once(device):
    _C = _ext()
    import diff_gaussian_rasterization as dgr

    lib = _C._lib
    cam = gs_scenes.identity_camera(320, 240)
    d = gs_scenes.random_gaussians(200_000, 0, cam=cam, seed=60).to(device)
    rast = dgr.GaussianRasterizer(gs_scenes.raster_settings_for(cam, 0, device=device))

    def fwd():
        return rast(means3D=d.means3D, means2D=torch.zeros_like(d.means3D), opacities=d.opacities, shs=d.shs,
                    scales=d.scales, rotations=d.rotations)

    ref, _ = fwd()
    torch.cuda.synchronize()
    dev = torch.device(device).index or 0
    _C._EXT.set_count_estimate(dev, 200_000, 320, 240, 1)  # the next forward outgrows its buffer
    prev = lib.gs_debug_set_scan_spin_limit(0)
    try:
        with pytest.raises(RuntimeError, match="look-back wait"):
            fwd()
        torch.cuda.synchronize()
    finally:
        lib.gs_debug_set_scan_spin_limit(prev)
    img, _ = fwd()  # clean: nothing left over from the failed forward
    torch.cuda.synchronize()
    assert torch.equal(img, ref)


def test_count_estimates_are_kept_per_shape(device):
    """A small scene rendered after a large one is not sized from the large one's count: the
    estimates are keyed by (device, P, W, H) and follow each shape's recent maximum."""
    _C = _ext()
    import diff_gaussian_rasterization as dgr

    dev = torch.device(device).index or 0
    cam = gs_scenes.circle_cameras(1, 6.0, W, H)[0]
    rast = dgr.GaussianRasterizer(gs_scenes.raster_settings_for(cam, 3, device=device))
    big = gs_scenes.random_gaussians(40_000, 3, seed=8, ball_radius=2.0).to(device)
    small = gs_scenes.random_gaussians(3_000, 3, seed=9, ball_radius=2.0).to(device)
    dpix = gs_scenes.dl_dimage(H, W, seed=3).to(device)
    for sc in (big, small):
        _C._EXT.set_count_estimate(dev, sc.means3D.shape[0], W, H, 0)
    _fwd_bwd(rast, big, dpix)
    nb = dgr.last_num_rendered()
    _fwd_bwd(rast, small, dpix)
    ns = dgr.last_num_rendered()
    assert _C._EXT.count_estimate(dev, 40_000, W, H) == nb
    assert _C._EXT.count_estimate(dev, 3_000, W, H) == ns < nb


class _Spy:
    """Forwards every attribute of the ext module; counts backward_gaussians calls."""

    def __init__(self, ext):
        self.ext, self.calls = ext, 0

    def __getattr__(self, name):
        if name == "backward_gaussians":
            self.calls += 1
        return getattr(self.ext, name)


def test_deferred_pass_goes_through_ext_and_equals_ctypes(device, monkeypatch):
    """A deferred GradBucket's per-Gaussian pass (finalize -> _C.backward_gaussians) runs through
    the ext (round 4), and its gradients are bit-identical to the ctypes bridge's."""
    _C = _ext()
    import gs_view_parallel as vp
    from diff_gaussian_rasterization import GaussianRasterizer

    cams = gs_scenes.circle_cameras(2, 6.0, W, H)
    d = gs_scenes.random_gaussians(8_000, 3, seed=9, ball_radius=2.0).to(device)
    rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, 3, device=device)) for c in cams]
    dpix = [gs_scenes.dl_dimage(H, W, seed=70 + v).to(device) for v in range(2)]

    def step():
        p = _leaves(d)
        b = vp.GradBucket(p, lazy_zero=True, defer=True)
        b.zero_grad()
        for r, dp in zip(rasts, dpix):
            m2 = torch.zeros_like(p[0], requires_grad=True)
            img, _ = r(means3D=p[0], means2D=m2, opacities=p[2], shs=p[1], scales=p[3], rotations=p[4])
            img.backward(dp)
        b.finalize()
        torch.cuda.synchronize()
        out = [t.grad.clone() for t in p]
        b.close()
        return out

    spy = _Spy(_C._EXT)
    monkeypatch.setattr(_C, "_EXT", spy)
    got = step()
    assert spy.calls >= 1, "the deferred per-Gaussian pass did not go through the ext"
    ref_fn = _C.backward_gaussians

    def ctypes_pass(*a, **kw):
        e, _C._EXT = _C._EXT, None
        try:
            return ref_fn(*a, **kw)
        finally:
            _C._EXT = e

    monkeypatch.setattr(_C, "backward_gaussians", ctypes_pass)
    ref = step()
    _assert_same(ref, got, "deferred pass ext vs ctypes")
