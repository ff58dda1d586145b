"""GPU tests of the bounded forward (ABI v10, gs_forward_bounded / gs_bounded_status): the whole
forward enqueued without reading num_rendered back, the binning buffer sized ahead for a capacity.

  - outputs and every gradient are bit-identical to the two-call forward (gs_forward_preprocess +
    gs_forward_render) whenever the instance count fits, for the concatenated and the split SH rows
    and for capacities at and above the count;
  - a view with more instances than the capacity stays in bounds (nothing composited, zero record
    sums), and its sticky flag is reported by bounded_status() and by the next bounded forward;
  - a view-parallel step of bounded forwards and their backwards into a GradBucket is captured into
    a HIP graph (torch.cuda.CUDAGraph) and its replays equal the eager step bit for bit.
"""
import pytest
import torch

import gs_scenes

pytestmark = pytest.mark.gpu

W, H = 320, 240


def _scene(device, P=20_000, seed=5):
    return gs_scenes.random_gaussians(P, 3, seed=seed, ball_radius=2.0).to(device)


def _leaves(d):
    return [d.means3D.clone().requires_grad_(True), d.shs.clone().requires_grad_(True),
            d.opacities.clone().requires_grad_(True), d.scales.clone().requires_grad_(True),
            d.rotations.clone().requires_grad_(True)]


def _fwd_bwd(rast, p, dpix, cap=None, split=False):
    m2 = torch.zeros_like(p[0], requires_grad=True)
    kw = {}
    if split:
        dc, rest = p[1].detach()[:, :1].contiguous(), p[1].detach()[:, 1:].contiguous()
        kw["sh_split"] = (dc, rest)
    img, radii = rast(means3D=p[0], means2D=m2, opacities=p[2], shs=p[1], scales=p[3], rotations=p[4],
                      binning_capacity=cap, **kw)
    img.backward(dpix)
    torch.cuda.synchronize()
    return [img.detach(), radii, m2.grad] + [t.grad for t in p]


@pytest.mark.parametrize("split", [False, True], ids=["concat_sh", "split_sh"])
def test_bounded_forward_equals_two_call_forward(device, split):
    from diff_gaussian_rasterization import GaussianRasterizer, bounded_status, last_num_rendered

    d = _scene(device)
    cams = gs_scenes.circle_cameras(2, 6.0, W, H)
    dpix = gs_scenes.dl_dimage(H, W, seed=3).to(device)
    for cam in cams:
        rast = GaussianRasterizer(gs_scenes.raster_settings_for(cam, 3, device=device))
        ref = _fwd_bwd(rast, _leaves(d), dpix, split=split)
        n = last_num_rendered()
        assert n > 0
        for cap in (n, int(n * 1.37) + 5):
            got = _fwd_bwd(rast, _leaves(d), dpix, cap=cap, split=split)
            for k, (a, b) in enumerate(zip(ref, got)):
                assert torch.equal(a, b), (cap, k, float((a.float() - b.float()).abs().max()))
        assert bounded_status() == (0, 0)


def test_bounded_capacity_overflow_is_reported_and_stays_in_bounds(device):
    from diff_gaussian_rasterization import GaussianRasterizer, bounded_status, last_num_rendered

    d = _scene(device)
    rast = GaussianRasterizer(gs_scenes.raster_settings_for(gs_scenes.circle_cameras(1, 6.0, W, H)[0], 3,
                                                            device=device))
    dpix = gs_scenes.dl_dimage(H, W, seed=4).to(device)
    ref = _fwd_bwd(rast, _leaves(d), dpix)
    n = last_num_rendered()
    # a third of the instances: the forward and backward run, every access in bounds
    got = _fwd_bwd(rast, _leaves(d), dpix, cap=n // 3)
    bg = rast.raster_settings.bg.view(3, 1, 1).expand(3, H, W)
    assert torch.equal(got[0], bg)  # nothing composited: the background
    assert torch.equal(got[1], ref[1])  # radii come from the preprocess, before the binning
    for g in got[2:]:
        assert torch.isfinite(g).all() and float(g.abs().max()) == 0.0  # zero record sums
    with pytest.raises(RuntimeError, match="binning capacity"):
        bounded_status()
    assert bounded_status() == (0, 0)  # cleared
    # the next bounded forward raises an earlier overflow too (and clears it)
    _fwd_bwd(rast, _leaves(d), dpix, cap=n // 3)
    p = _leaves(d)
    with pytest.raises(RuntimeError, match="binning capacity"):
        rast(means3D=p[0], means2D=torch.zeros_like(p[0]), opacities=p[2], shs=p[1], scales=p[3], rotations=p[4],
             binning_capacity=n)
    again = _fwd_bwd(rast, _leaves(d), dpix, cap=n)
    for a, b in zip(ref, again):
        assert torch.equal(a, b)
    assert bounded_status() == (0, 0)


@pytest.mark.parametrize("front", ["per_view", "fused_front"])
def test_bounded_view_parallel_step_replays_in_a_hip_graph(device, front):
    """per_view: each view's bounded forward on one stream, backwards into a lazy bucket.
    fused_front: the bench's step -- prepare_views (one preprocess launch, bounded) with the views'
    orderings and renders on two streams, the bucket deferring the per-Gaussian half to finalize."""
    import gs_view_parallel as vp
    from diff_gaussian_rasterization import GaussianRasterizer, bounded_status, last_num_rendered, prepare_views

    d = _scene(device, seed=9)
    cams = gs_scenes.circle_cameras(3, 6.0, W, H)
    rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, 3, device=device)) for c in cams]
    dpix = [gs_scenes.dl_dimage(H, W, seed=60 + v).to(device) for v in range(3)]
    cap = 0
    with torch.no_grad():
        p0 = _leaves(d)
        for r in rasts:
            r(means3D=p0[0], means2D=torch.zeros_like(p0[0]), opacities=p0[2], shs=p0[1], scales=p0[3],
              rotations=p0[4])
            cap = max(cap, last_num_rendered())
    cap = int(cap * 1.25)
    p = _leaves(d)
    fused = front == "fused_front"
    bucket = vp.GradBucket(p, lazy_zero=True, defer=fused)
    streams = [torch.cuda.Stream(device) for _ in range(2 if fused else 1)]
    imgs = [None] * len(rasts)

    def view(k, r, dp, pre, c):
        def run():
            m2 = torch.empty_like(p[0], requires_grad=True)
            img, _ = r(means3D=p[0], means2D=m2, opacities=p[2], shs=p[1], scales=p[3], rotations=p[4],
                       prepared=pre, binning_capacity=None if pre is not None else c)
            img.backward(dp)
            imgs[k] = img.detach()
        return run

    def step(c):  # c: binning capacity (None: the read-back forwards)
        bucket.zero_grad()
        pres = [None] * len(rasts)
        if fused:
            pres = prepare_views(rasts, p[0], p[2], shs=p[1], scales=p[3], rotations=p[4],
                                 streams=[streams[k % 2] for k in range(len(rasts))], binning_capacity=c)
        vp.run_views([view(k, r, dp, pre, c) for k, (r, dp, pre) in enumerate(zip(rasts, dpix, pres))], streams)
        bucket.finalize()

    step(None)  # the eager read-back step is the reference
    torch.cuda.synchronize()
    ref_flat = bucket.flat.clone()
    ref_imgs = [t.clone() for t in imgs]
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        for _ in range(2):
            step(cap)
    torch.cuda.current_stream(device).wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(bucket.flat, ref_flat)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step(cap)
    bucket.flat.fill_(float("nan"))
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(bucket.flat, ref_flat)
        for a, b in zip(imgs, ref_imgs):
            assert torch.equal(a, b)
        bucket.flat.fill_(float("nan"))
    # new parameter values between replays: the look-back scans' epochs advance on the device (the
    # counter finalize's sequence word), so no status word of the previous replay is taken as this one's
    gen = torch.Generator(device=device).manual_seed(77)
    for _ in range(2):
        with torch.no_grad():
            for t, amp in zip(p[:3], (0.01, 0.05, 0.05)):  # means, SH, opacities (the counts stay below cap)
                t.add_(amp * torch.randn(t.shape, device=device, generator=gen))
        step(None)
        torch.cuda.synchronize()
        ref_flat = bucket.flat.clone()
        ref_imgs = [t.clone() for t in imgs]
        bucket.flat.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(bucket.flat, ref_flat)
        for a, b in zip(imgs, ref_imgs):
            assert torch.equal(a, b)
    assert bounded_status() == (0, 0)
    del graph
    bucket.close()
