"""The debug=True failure path of the drop-in API (settings.debug, /root/reference/arguments/__init__.py:68;
README :143-146 of the reference: "If your training is failing, set debug ... and send us the
snapshot_fw.dump / snapshot_bw.dump"): a native failure in the rasterizer's forward or backward
prints the upstream notice, writes a CPU copy of the call's arguments to snapshot_fw.dump /
snapshot_bw.dump in the working directory, and re-raises.  The dumps load with
torch.load(weights_only=True) and hold the call's arguments."""
import pytest
import torch

import gs_scenes

pytestmark = pytest.mark.gpu


def _scene(device, P=400, W=96, H=80):
    cam = gs_scenes.identity_camera(W, H)
    sc = gs_scenes.random_gaussians(P, 0, cam=cam, seed=31).to(device)
    return cam, sc


def test_forward_failure_dumps_snapshot_fw(device, tmp_path, monkeypatch, capsys):
    """prefiltered=True with a culled point (the upstream 'Point is filtered ...' failure)."""
    from diff_gaussian_rasterization import GaussianRasterizer

    monkeypatch.chdir(tmp_path)
    cam, sc = _scene(device)
    sc.means3D[0, 2] = 0.1  # in front of the near plane: culled although prefiltered
    s = gs_scenes.raster_settings_for(cam, 0, device=device)._replace(prefiltered=True, debug=True)
    with pytest.raises(RuntimeError, match="Point is filtered although prefiltered is set"):
        GaussianRasterizer(s)(means3D=sc.means3D, means2D=torch.zeros_like(sc.means3D), opacities=sc.opacities,
                              shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    assert "An error occured in forward. Please forward snapshot_fw.dump for debugging." in capsys.readouterr().out
    snap = torch.load(tmp_path / "snapshot_fw.dump", weights_only=True)
    # (bg, means3D, colors, opacities, scales, rotations, scale_modifier, cov3D, view, proj, tanfovx, tanfovy,
    #  H, W, sh, sh_degree, campos, prefiltered, debug): upstream's argument tuple, on the CPU
    assert isinstance(snap, tuple) and len(snap) == 19
    assert all(not (isinstance(t, torch.Tensor) and t.is_cuda) for t in snap)
    assert torch.equal(snap[1], sc.means3D.cpu()) and torch.equal(snap[3], sc.opacities.cpu())
    assert torch.equal(snap[14], sc.shs.cpu()) and torch.equal(snap[0], s.bg.cpu())
    assert (snap[12], snap[13], snap[15], snap[17], snap[18]) == (s.image_height, s.image_width, 0, True, True)
    assert not (tmp_path / "snapshot_bw.dump").exists()


def test_backward_failure_dumps_snapshot_bw(device, tmp_path, monkeypatch, capsys):
    """A look-back wait of the forward's offsets scan that timed out (forced: spin limit 0) is reported
    by the next call -- the backward -- which then fails in debug mode with its snapshot."""
    from diff_gaussian_rasterization import GaussianRasterizer, _native

    monkeypatch.chdir(tmp_path)
    lib = _native.load()
    cam, sc = _scene(device, P=6000)  # three look-back tiles
    s = gs_scenes.raster_settings_for(cam, 0, device=device)._replace(debug=True)
    rast = GaussianRasterizer(s)
    leaves = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.opacities, sc.shs, sc.scales, sc.rotations)]

    def fwd():
        return rast(means3D=leaves[0], means2D=torch.zeros_like(sc.means3D), opacities=leaves[1], shs=leaves[2],
                    scales=leaves[3], rotations=leaves[4])[0]

    fwd().sum().backward()  # warm: the instance-count estimate of this shape is set, so the next forward
    torch.cuda.synchronize()  # binds into its estimated buffer and does not check its own ordering flags
    prev = lib.gs_debug_set_scan_spin_limit(0)
    try:
        img = fwd()
    finally:
        lib.gs_debug_set_scan_spin_limit(prev)
    torch.cuda.synchronize()
    dpix = torch.ones_like(img)
    with pytest.raises(RuntimeError, match="look-back wait"):
        img.backward(dpix)
    assert "An error occured in backward. Please forward snapshot_bw.dump for debugging." in capsys.readouterr().out
    snap = torch.load(tmp_path / "snapshot_bw.dump", weights_only=True)
    # (bg, means3D, radii, colors, scales, rotations, scale_modifier, cov3D, view, proj, tanfovx, tanfovy,
    #  dL_dout_color, sh, sh_degree, campos, geomBuffer, num_rendered, binningBuffer, imageBuffer, debug)
    assert isinstance(snap, tuple) and len(snap) == 21
    assert torch.equal(snap[1], sc.means3D.cpu()) and torch.equal(snap[12], dpix.cpu())
    assert snap[2].dtype == torch.int32 and snap[2].shape == (6000,)
    assert snap[16].dtype == torch.uint8 and snap[20] is True
    # the failure was reported once: the next call runs clean
    fwd().sum().backward()
    torch.cuda.synchronize()
