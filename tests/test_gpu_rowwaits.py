"""GPU tests of the forward's row waits (ABI v17 gs_set_row_waits, _C.row_waits): the preprocess
launched in Gaussian-row chunks, each behind a stream wait on its chunk's event -- what lets a
sharded optimizer step's all-gathers (gs_view_parallel.ShardedAdam(overlap=True)) run into the next
step's forward.

Each test writes the inputs chunk by chunk on a side stream that first runs a long busy kernel, so
a preprocess that did not wait for a chunk's event would read the zeros the inputs were cleared to:
outputs must equal the plain forward bit for bit."""
import pytest
import torch

import gs_scenes

pytestmark = pytest.mark.gpu

W, H = 320, 240


def _delayed_fill(dsts, srcs, bounds, dev):
    """Clear dsts on the current stream; on a side stream, after ~ms of busy work, copy srcs' rows
    chunk by chunk into them, recording an event per chunk: [(lo, hi, event)]."""
    cur = torch.cuda.current_stream(dev)
    for t in dsts:
        t.zero_()
    side = torch.cuda.Stream(dev)
    side.wait_stream(cur)
    waits = []
    with torch.cuda.stream(side):
        a = torch.randn((2048, 2048), device=dev)
        for _ in range(8):  # busy: the chunks land well after the forward was queued
            a = a @ a
            a = a / a.norm()
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            for d, s in zip(dsts, srcs):
                d[lo:hi].copy_(s[lo:hi])
            ev = torch.cuda.Event()
            ev.record(side)
            waits.append((lo, hi, ev))
    for t in dsts:
        t.record_stream(side)
    return waits, side


@pytest.mark.parametrize("bounds", [[0, 700, 1999, 5000], [0, 256, 512, 5000], [0, 5000]],
                         ids=["ragged", "aligned", "one"])
def test_row_waited_forward_equals_plain(device, bounds):
    from diff_gaussian_rasterization import GaussianRasterizer, _C

    cam = gs_scenes.identity_camera(W, H)
    d = gs_scenes.random_gaussians(5000, 3, cam=cam, seed=21).to(device)
    rast = GaussianRasterizer(gs_scenes.raster_settings_for(cam, 3, device=device))
    srcs = [d.means3D, d.shs, d.opacities, d.scales, d.rotations]

    def fwd(ins):
        return rast(means3D=ins[0], means2D=torch.zeros_like(ins[0]), shs=ins[1], opacities=ins[2], scales=ins[3],
                    rotations=ins[4])

    with torch.no_grad():
        ref_img, ref_radii = fwd(srcs)
        torch.cuda.synchronize()
        dsts = [torch.empty_like(t) for t in srcs]
        waits, side = _delayed_fill(dsts, srcs, bounds, device)
        with _C.row_waits(waits):
            img, radii = fwd(dsts)
        torch.cuda.synchronize()
    assert torch.equal(img, ref_img) and torch.equal(radii, ref_radii)


def test_row_waited_prepared_views_equal_plain(device):
    """The K-view preprocess (prepare_views -> gs_forward_preprocess_views) honours the waits too."""
    from diff_gaussian_rasterization import GaussianRasterizer, _C, prepare_views

    cams = gs_scenes.jittered_cameras(3, W, H, seed=5)
    d = gs_scenes.random_gaussians(6000, 3, cam=cams[0], seed=22).to(device)
    rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, 3, device=device)) for c in cams]
    srcs = [d.means3D, d.shs, d.opacities, d.scales, d.rotations]

    def run(ins, waits=None):
        with _C.row_waits(waits or []):
            pre = prepare_views(rasts, ins[0], ins[2], shs=ins[1], scales=ins[3], rotations=ins[4])
        return [r(means3D=ins[0], means2D=torch.zeros_like(ins[0]), shs=ins[1], opacities=ins[2], scales=ins[3],
                  rotations=ins[4], prepared=p)[0] for r, p in zip(rasts, pre)]

    with torch.no_grad():
        ref = run(srcs)
        torch.cuda.synchronize()
        dsts = [torch.empty_like(t) for t in srcs]
        waits, _ = _delayed_fill(dsts, srcs, [0, 1000, 3000, 6000], device)
        got = run(dsts, waits)
        torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_row_waited_train_render_equals_plain(device):
    """gs_train_step.render(row_waits=...): the activation runs chunk by chunk on a side stream behind
    the waits and hands the rasterizer its own chunk events; image, radii and the raw-parameter
    gradients of loss.backward() equal the plain render's."""
    import gs_loss
    import gs_train_step as ts

    cam = gs_scenes.identity_camera(W, H)
    sc = gs_scenes.random_gaussians(5000, 3, cam=cam, seed=23)
    settings = gs_scenes.raster_settings_for(cam, 3, device=device)
    gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(3)).to(device)
    names = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")
    out = []
    for delayed in (False, True):
        m = ts.TrainModel(sc, device)
        waits = []
        if delayed:
            params = [getattr(m, n) for n in names]
            with torch.no_grad():
                vals = [p.detach().clone() for p in params]
                waits, _ = _delayed_fill([p.data for p in params], vals, [0, 1300, 2600, 5000], device)
        img, _, radii = ts.render(m, settings, fused=True, row_waits=waits)
        loss, _ = gs_loss.photometric_loss(img, gt)
        loss.backward()
        torch.cuda.synchronize()
        out.append([img.detach(), radii] + [getattr(m, n).grad.clone() for n in names])
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_row_waits_are_validated_and_cleared(device):
    from diff_gaussian_rasterization import _C, _native

    lib = _native.load()
    ev = torch.cuda.Event()
    ev.record()
    with pytest.raises(ValueError, match="contiguous"):
        with _C.row_waits([(0, 10, ev), (11, 20, ev)]):
            pass
    with pytest.raises(ValueError, match="row 0"):
        with _C.row_waits([(5, 10, ev)]):
            pass
    import ctypes

    evs = (ctypes.c_void_p * 2)(ev.cuda_event, ev.cuda_event)
    for bad in ([5, 10, 20], [0, 10, 10]):  # not from row 0; not increasing
        b = (ctypes.c_int * 3)(*bad)
        assert lib.gs_set_row_waits(2, ctypes.cast(b, ctypes.c_void_p), ctypes.cast(evs, ctypes.c_void_p)) != 0
    assert lib.gs_set_row_waits(2, None, None) != 0
    assert lib.gs_set_row_waits(0, None, None) == 0
