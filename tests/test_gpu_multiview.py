"""GPU tests of the multi-view / view-parallel path (BASELINE config C4) and of the
boundary details the per-view parity tests do not reach:

  - gradient buckets: the rasterizer writing / adding into the .grad views of a flat bucket
    (gs_backward_accumulate) equals autograd's per-view gradients summed with `+=`, bit for bit;
  - C4 at full size: 1M Gaussians in a ball seen from the 8 ring cameras, every view through
    GaussianRasterizer, one view against the oracle;
  - two ranks (gloo, both on cuda:0) each rendering its share of the 8 C4 views, one all-reduce of
    the bucket, against the single-process sum of all 8 views (test_two_rank_* runs first: its
    children start before this process touches the GPU);
  - the raw upstream backward tuple (dL_dcov3D for scale / rotation inputs), the record-cut
    invariant of the backward (slots strictly increasing within a tile), and the reporting of a
    timed-out look-back wait in the offsets scan.
"""
import math
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import gs_scenes
from test_gpu_parity import RTOL, _check_backward, _check_forward_exact, _gpu_run, _oracle_scene, _tol_check

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    from diff_gaussian_rasterization import _native

    return _native.load()


@pytest.fixture
def exact_mode():
    prev = _lib().gs_set_exact_exp(1)
    yield
    _lib().gs_set_exact_exp(prev)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.spawn_first
def test_two_rank_view_parallel_matches_single_process_sum(tmp_path):
    """C4 view parallelism end to end on one GPU: torchrun starts 2 ranks (gloo; RCCL needs one GPU
    per rank), each renders views v = rank (mod 2) of the 8 ring cameras through the HIP
    rasterizer into its GradBucket, one all-reduce sums the buckets, and rank 0 compares the
    result with the 8 views rendered and summed in one process (tolerance 1e-5 |ref| + 1e-5 max:
    the two sums associate differently)."""
    out = tmp_path / "vp_result.txt"
    env = dict(os.environ, GS_VP_OUT=str(out), HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "vp_gpu_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"workers failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = out.read_text()
    print(res)
    assert res.startswith("OK"), res


@pytest.mark.spawn_first
def test_two_rank_training_with_densify_keeps_replicas_identical(tmp_path):
    """View-parallel training across a densify step (2 ranks, gloo, one GPU): train steps through
    the bucket all-reduce, reduce_densify_stats, densify_and_prune with differently seeded rank
    generators (rank 0's split draws are broadcast), the bucket rebound to the new parameters, two
    more steps; every parameter and Adam moment bit-identical across the ranks (replica digest)."""
    out = tmp_path / "vp_train.txt"
    env = dict(os.environ, GS_VP_OUT=str(out), HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "vp_train_worker.py"),
           "gloo2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"workers failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = out.read_text()
    print(res)
    assert res.startswith("OK"), res


@pytest.mark.spawn_first
def test_two_rank_sharded_adam_equals_allreduce_across_densify(tmp_path):
    """The reduce-scatter -> sharded FusedAdam -> all-gather step (gs_view_parallel.ShardedAdam, 3
    Gaussian-row chunks) against the bucket all-reduce + replicated FusedAdam (2 ranks, gloo, one
    GPU): three view-parallel train steps, densify_and_prune, two more steps; parameters, moments and
    step counts bit-identical, and identical across the ranks."""
    out = tmp_path / "vp_sharded.txt"
    env = dict(os.environ, GS_VP_OUT=str(out), HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "vp_train_worker.py"),
           "gloo2_sharded"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"workers failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = out.read_text()
    print(res)
    assert res.startswith("OK"), res


@pytest.mark.spawn_first
def test_two_rank_deferred_sharded_adam_equals_allreduce(tmp_path):
    """bench.py's step shape (activated leaves, GradBucket(lazy_zero=True, defer=True): the
    per-Gaussian half runs once per optimizer step) through ShardedAdam, whose deferred pass runs in
    row chunks on the compute stream while the previous chunk's reduce-scatter / update /
    all-gather run on the side stream -- and with overlap=True, the all-gathers left in flight into
    the next step's chunked preprocess (2 ranks, gloo, one GPU): four steps bit-identical to the
    bucket all-reduce + replicated FusedAdam, and identical across the ranks."""
    out = tmp_path / "vp_deferred.txt"
    env = dict(os.environ, GS_VP_OUT=str(out), HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "vp_train_worker.py"),
           "gloo2_deferred"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"workers failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = out.read_text()
    print(res)
    assert res.startswith("OK"), res


@pytest.mark.spawn_first
def test_rccl_world1_bucket_allreduce_equals_single_process(tmp_path):
    """The RCCL path (torch.distributed backend "nccl" = RCCL on ROCm) at world size 1: the view-
    parallel train step with its bucket all-reduce issued through RCCL equals the same steps without
    a process group, bit for bit."""
    out = tmp_path / "vp_nccl.txt"
    env = dict(os.environ, GS_VP_OUT=str(out), HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "vp_train_worker.py"), "nccl1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"worker failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = out.read_text()
    print(res)
    assert res.startswith("OK"), res


@pytest.mark.spawn_first
def test_concurrent_processes_are_deterministic():
    """Two processes render the 8 C4 views forward + backward on the same GPU at once, four passes
    each; every image and gradient must be bitwise identical across passes.  Sharing the GPU
    shifts the waves' relative timing: this caught a barrier that did not drain the LDS writes of
    the partner wave (render_bwd flush; gs_common.h lds_barrier), which flipped the dcolor /
    dmean2D sums of a few Gaussians in ~1 of 5 C4 views."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(ROOT, "tests", "det_gpu_worker.py"), "3"]
    procs = [subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for _ in range(2)]
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0 and o.startswith("OK"), f"rc {p.returncode}: {o[-2000:]}\n{e[-2000:]}"


def _leaves(d):
    return [d.means3D.clone().requires_grad_(True), d.shs.clone().requires_grad_(True),
            d.opacities.clone().requires_grad_(True), d.scales.clone().requires_grad_(True),
            d.rotations.clone().requires_grad_(True)]


def _render(rast, p, means2D):
    img, radii = rast(means3D=p[0], means2D=means2D, opacities=p[2], shs=p[1], scales=p[3], rotations=p[4])
    return img, radii


@pytest.mark.parametrize("lazy", [True, False], ids=["lazy_zero", "zero_filled"])
@pytest.mark.parametrize("nstreams", [1, 2, 3], ids=["1stream", "2streams", "3streams"])
@pytest.mark.parametrize("defer", [False, True], ids=["per_view", "deferred"])
def test_bucket_accumulation_equals_autograd_sum(device, lazy, nstreams, defer):
    """The bucket equals autograd's per-view gradients summed with += in view order, bit for bit,
    also when the views run round-robin on several streams (vp.run_views: the forward passes and
    tile backward passes overlap; the bucket orders its writes by events), and when the
    per-Gaussian half of the backward runs once for all views (defer: gs_backward_gaussians)."""
    import gs_view_parallel as vp
    from diff_gaussian_rasterization import GaussianRasterizer

    W, H = 320, 240
    cams = gs_scenes.circle_cameras(3, 6.0, W, H)
    d = gs_scenes.random_gaussians(20_000, 3, seed=5, ball_radius=2.0).to(device)
    rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, 3, device=device)) for c in cams]
    dpix = [gs_scenes.dl_dimage(H, W, seed=40 + v).to(device) for v in range(3)]
    # reference: plain autograd, one fresh gradient per view, summed with += in view order
    ref, m2_ref = None, []
    for r, dp in zip(rasts, dpix):
        p = _leaves(d)
        m2 = torch.zeros_like(p[0], requires_grad=True)
        img, _ = _render(r, p, m2)
        img.backward(dp)
        m2_ref.append(m2.grad.clone())
        g = [t.grad for t in p]
        if ref is None:
            ref = [x.clone() for x in g]
        else:
            for a, b in zip(ref, g):
                a += b
    p = _leaves(d)
    b = vp.GradBucket(p, lazy_zero=lazy, defer=defer)
    calls = []
    orig = b.claim
    b.claim = lambda t: calls.append(1) or orig(t)  # noqa: E731
    streams = [torch.cuda.Stream(device) for _ in range(nstreams)]

    m2s = []

    def view(r, dp):
        def run():
            m2 = torch.zeros_like(p[0], requires_grad=True)
            img, _ = _render(r, p, m2)
            img.backward(dp)
            m2s.append(m2)
        return run

    for step in range(2):  # the second step reuses the bucket (stale values must not leak)
        b.zero_grad()
        vp.run_views([view(r, dp) for r, dp in zip(rasts, dpix)], streams)
        b.finalize()
        torch.cuda.synchronize()
        for k, (t, x) in enumerate(zip(p, ref)):
            assert t.grad.data_ptr() == b.views[id(t)].data_ptr()
            assert torch.equal(t.grad, x), (step, k, float((t.grad - x).abs().max()))
        for v, (m2, x) in enumerate(zip(m2s, m2_ref)):  # each view's screen-space gradient
            assert torch.equal(m2.grad, x), (step, v)
        m2s.clear()
    # every view's backward wrote through the sink (deferred: one claim per tensor and step)
    assert len(calls) == (2 * 5 if defer else 2 * 3 * 5)
    b.close()


def test_raw_backward_returns_every_upstream_gradient(oracle, device, exact_mode):
    """_C.rasterize_gaussians_backward returns upstream's 8-tuple: dL_dcov3D is filled for
    scale / rotation inputs too (the covariance gradient the scale / rotation chain starts from),
    dL_dcolors for SH inputs (the per-Gaussian colour gradient); all against the oracle."""
    from diff_gaussian_rasterization import _C

    W, H = 160, 120
    cam = gs_scenes.identity_camera(W, H)
    sc = gs_scenes.random_gaussians(3000, 2, cam=cam, seed=17)
    bg = np.array([0.1, 0.0, 0.2], np.float32)
    s = gs_scenes.raster_settings_for(cam, 2, bg=torch.tensor(bg, device=device), device=device)
    dsc = sc.to(device)
    e = torch.Tensor([])
    num, color, radii, geom, binb, imgb = _C.rasterize_gaussians(
        s.bg, dsc.means3D, e, dsc.opacities, dsc.scales, dsc.rotations, 1.0, e, s.viewmatrix, s.projmatrix,
        s.tanfovx, s.tanfovy, H, W, dsc.shs, 2, s.campos, False, False)
    dpix = gs_scenes.dl_dimage(H, W, seed=18)
    out = _C.rasterize_gaussians_backward(s.bg, dsc.means3D, radii, e, dsc.scales, dsc.rotations, 1.0, e,
                                          s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix.to(device),
                                          dsc.shs, 2, s.campos, geom, num, binb, imgb, False)
    assert len(out) == 8
    gr = oracle.backward(_oracle_scene(oracle, cam, sc, bg), dpix.numpy())
    for t, k in zip(out, ("dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales",
                          "drotations")):
        ref = gr[k].reshape(t.shape)
        assert np.abs(ref).max() > 0, k
        _tol_check(t.cpu().numpy(), ref, k)


def _occluded_scene():
    """Two layers of small opaque splats tile the left half of the image (every pixel there
    saturates, T < 1e-4, before depth 2) and one large splat at depth 6 spans the whole width: its
    instances in the left tiles lie past every pixel's last contributor (no backward record:
    cut), in the right tiles they are walked (kept).  Plus 2000 random splats."""
    W, H = 256, 128
    cam = gs_scenes.identity_camera(W, H)
    rnd = gs_scenes.random_gaussians(2000, 1, cam=cam, seed=50)
    fx = W / (2.0 * math.tan(cam.FoVx / 2))
    fy = H / (2.0 * math.tan(cam.FoVy / 2))
    layers = []
    for z in (1.5, 1.7):
        px, py = np.meshgrid(np.arange(0.0, 128.0, 2.0), np.arange(-2.0, 130.0, 2.0))
        n = px.size
        m = torch.tensor(np.stack([(px.ravel() - W / 2) / fx * z, (py.ravel() - H / 2) / fy * z,
                                   np.full(n, z)], 1), dtype=torch.float32)
        lay = gs_scenes.random_gaussians(n, 1, cam=cam, seed=int(z * 10))
        lay.means3D = m
        lay.scales = torch.full((n, 3), 3.0 * z / fx)
        lay.rotations = torch.tensor([[1.0, 0.0, 0.0, 0.0]]).repeat(n, 1)
        lay.opacities = torch.full((n, 1), 0.999)
        layers.append(lay)
    back = gs_scenes.random_gaussians(1, 1, cam=cam, seed=52)
    back.means3D[0] = torch.tensor([0.0, 0.0, 6.0])
    back.scales[0] = torch.tensor([60.0 * 6.0 / fx, 30.0 * 6.0 / fy, 0.05])
    back.rotations[0] = torch.tensor([1.0, 0.0, 0.0, 0.0])
    back.opacities[0] = 0.6
    return cam, gs_scenes.concat_scenes(rnd, *layers, back)


def test_record_cut_invariant_and_partly_cut_gaussian(oracle, device, exact_mode):
    """k_sum_records keeps a tile's record of slot s iff s < tile_cut (1 + the slot of the last
    instance the tile's walk reaches): that needs the slots strictly increasing within every
    tile's list.  Checked directly on the exported slots, plus a Gaussian that is cut in some
    tiles and kept in others, against the oracle."""
    from diff_gaussian_rasterization import _C

    cam, sc = _occluded_scene()
    W, H = cam.image_width, cam.image_height
    bg = np.zeros(3, np.float32)
    osc = _oracle_scene(oracle, cam, sc, bg)
    ofw = oracle.forward(osc, intermediates=True)
    ofw["bg"] = bg
    _check_forward_exact(ofw, cam, sc, device)
    dpix = gs_scenes.dl_dimage(H, W, seed=53).numpy()
    img, _, leaves = _gpu_run(cam, sc, device, bg, dpix)
    _check_backward(oracle.backward(osc, dpix), leaves)
    # slots / cuts of a forward + backward through the raw entry points
    s = gs_scenes.raster_settings_for(cam, 1, device=device)
    d = sc.to(device)
    e = torch.Tensor([])
    num, color, radii, geom, binb, imgb = _C.rasterize_gaussians(
        s.bg, d.means3D, e, d.opacities, d.scales, d.rotations, 1.0, e, s.viewmatrix, s.projmatrix, s.tanfovx,
        s.tanfovy, H, W, d.shs, 1, s.campos, False, False)
    _C.rasterize_gaussians_backward(s.bg, d.means3D, radii, e, d.scales, d.rotations, 1.0, e, s.viewmatrix,
                                    s.projmatrix, s.tanfovx, s.tanfovy, torch.tensor(dpix, device=device), d.shs, 1,
                                    s.campos, geom, num, binb, imgb, False)
    slots, cuts = _C.debug_export_slots(W, H, num, binb, imgb, device)
    ex = _C.debug_export(sc.P, W, H, num, geom, binb, imgb, device)
    rng = ex["ranges"].long().cpu().numpy()
    sl = slots.long().cpu().numpy()
    cuts = cuts.long().cpu().numpy()
    lst = ex["point_list"].long().cpu().numpy()
    back = sc.P - 1
    cut_tiles = kept_tiles = 0
    for t, (a, b) in enumerate(rng):
        if b <= a:
            continue
        assert (np.diff(sl[a:b]) > 0).all(), f"tile {t}: slots not strictly increasing"
        hit = np.nonzero(lst[a:b] == back)[0]
        if hit.size:
            if sl[a + hit[0]] < cuts[t]:
                kept_tiles += 1
            else:
                cut_tiles += 1
    assert cut_tiles > 0 and kept_tiles > 0, (cut_tiles, kept_tiles)


def test_lookback_timeout_is_reported(device):
    """A look-back wait that runs out (offsets scan or a one-sweep sort pass) leaves an invalid
    instance list: every later kernel of that forward stays in bounds (the render draws no list,
    the record sums are zero) and the NEXT call of the thread -- its backward or another forward --
    fails loudly, in every mode (not only debug).  The test hook makes every waiting workgroup time
    out at once."""
    from diff_gaussian_rasterization import GaussianRasterizer

    lib = _lib()
    cam = gs_scenes.identity_camera(320, 240)
    d = gs_scenes.random_gaussians(200_000, 0, cam=cam, seed=60).to(device)
    rast = GaussianRasterizer(gs_scenes.raster_settings_for(cam, 0, device=device))

    def fwd(means3D):
        return rast(means3D=means3D, means2D=torch.zeros_like(d.means3D), opacities=d.opacities, shs=d.shs,
                    scales=d.scales, rotations=d.rotations)

    # one clean forward first: the torch host path then sizes the next binning buffer from this
    # scene's count, so the timed-out forward below fits it (the case where the count outgrows the
    # estimate fails in the forward itself: test_gpu_ext.py)
    fwd(d.means3D)
    torch.cuda.synchronize()
    # forward only: the next forward reports it
    prev = lib.gs_debug_set_scan_spin_limit(0)
    try:
        img, _ = fwd(d.means3D)
        torch.cuda.synchronize()
    finally:
        lib.gs_debug_set_scan_spin_limit(prev)
    assert torch.isfinite(img).all()
    with pytest.raises(RuntimeError, match="look-back wait"):
        fwd(d.means3D)
    img, _ = fwd(d.means3D)
    assert torch.isfinite(img).all() and float(img.abs().max()) > 0
    # forward + backward: the backward reports it (after queuing its own, in-bounds, kernels)
    m = d.means3D.clone().requires_grad_(True)
    prev = lib.gs_debug_set_scan_spin_limit(0)
    try:
        img, _ = fwd(m)
    finally:
        lib.gs_debug_set_scan_spin_limit(prev)
    with pytest.raises(RuntimeError, match="look-back wait"):
        img.sum().backward()
    torch.cuda.synchronize()
    img, _ = fwd(d.means3D)
    torch.cuda.synchronize()
    assert torch.isfinite(img).all()


def _c4_properties(ex, num, color, W, H):
    lst = ex["point_list"].long()
    rng = ex["ranges"].long()
    assert num == int(ex["tiles_touched"].sum())
    nonempty = rng[:, 1] > rng[:, 0]
    starts, ends = rng[nonempty, 0], rng[nonempty, 1]
    assert starts[0] == 0 and ends[-1] == num and torch.all(starts[1:] == ends[:-1])
    depth_bits = ex["depth"].view(torch.int32).long()
    tile_of = torch.repeat_interleave(torch.arange(rng.shape[0], device=lst.device)[nonempty], ends - starts)
    same = tile_of[1:] == tile_of[:-1]
    d0, d1 = depth_bits[lst[:-1]], depth_bits[lst[1:]]
    assert torch.all(((d1 > d0) | ((d1 == d0) & (lst[1:] > lst[:-1])))[same])
    assert int(ex["n_contrib"].long().max()) <= int((ends - starts).max())
    assert torch.isfinite(color).all() and (color >= 0).all()


def test_c4_ring_views_full_size(oracle, device):
    """BASELINE C4: 1M Gaussians SH3 in a ball of radius 2, the 8 ring cameras at radius 6,
    1920x1080.  Every view goes through GaussianRasterizer forward + backward (size-independent
    properties: list ordered by (tile, depth, index), ranges partition the list, finite image and
    gradients, bit-identical rerun of the forward); view 3 is compared with the oracle at full
    size in the bit-exact mode (forward bit-exact, gradients at 1e-5)."""
    from diff_gaussian_rasterization import GaussianRasterizer, _C

    W, H = 1920, 1080
    cams = gs_scenes.circle_cameras(8, 6.0, W, H)
    sc = gs_scenes.random_gaussians(1_000_000, 3, seed=0, ball_radius=2.0)
    d = sc.to(device)
    e = torch.Tensor([])
    dpix = gs_scenes.dl_dimage(H, W, seed=1).to(device)
    for v, cam in enumerate(cams):
        s = gs_scenes.raster_settings_for(cam, 3, device=device)
        args = (s.bg, d.means3D, e, d.opacities, d.scales, d.rotations, 1.0, e, s.viewmatrix, s.projmatrix,
                s.tanfovx, s.tanfovy, H, W, d.shs, 3, s.campos, False, False)
        num, color, radii, geom, binb, imgb = _C.rasterize_gaussians(*args)
        num2, color2, radii2, *_ = _C.rasterize_gaussians(*args)
        assert num == num2 and torch.equal(color, color2) and torch.equal(radii, radii2)
        assert int((radii > 0).sum()) > 500_000, f"view {v}: only {int((radii > 0).sum())} visible"
        _c4_properties(_C.debug_export(sc.P, W, H, num, geom, binb, imgb, device), num, color, W, H)
        p = _leaves(d)
        m2 = torch.zeros_like(p[0], requires_grad=True)
        img, _ = _render(GaussianRasterizer(s), p, m2)
        assert torch.equal(img, color)
        img.backward(dpix)
        for t in p + [m2]:
            assert torch.isfinite(t.grad).all()
        assert float(p[1].grad.abs().max()) > 0
        del geom, binb, imgb, p, m2, img
    prev = _lib().gs_set_exact_exp(1)
    try:
        cam = cams[3]
        bg = np.zeros(3, np.float32)
        osc = _oracle_scene(oracle, cam, sc, bg)
        ofw = oracle.forward(osc, intermediates=True)
        ofw["bg"] = bg
        _check_forward_exact(ofw, cam, sc, device)
        dp = dpix.cpu().numpy()
        _, _, leaves = _gpu_run(cam, sc, device, bg, dp)
        _check_backward(oracle.backward(osc, dp), leaves)
    finally:
        _lib().gs_set_exact_exp(prev)


def test_prepared_views_equal_single_view_calls(device):
    """prepare_views (one preprocess launch for several cameras, gs_forward_preprocess_views) then
    each view's call with prepared=: images, radii and every gradient bit-identical to plain
    per-view calls, with the views' orderings on two streams."""
    from diff_gaussian_rasterization import GaussianRasterizer, prepare_views

    W, H = 320, 200
    cams = gs_scenes.circle_cameras(5, 6.0, W, H)
    sc = gs_scenes.random_gaussians(20000, 3, seed=21, ball_radius=2.0).to(device)
    rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, 3, device=device)) for c in cams]
    dpix = gs_scenes.dl_dimage(H, W, seed=4, scale=1.0).to(device)

    import gs_view_parallel as vp

    def run(prepared):
        leaves = [t.clone().requires_grad_(True) for t in (sc.means3D, sc.shs, sc.opacities, sc.scales, sc.rotations)]
        # views on two streams write the leaves' gradients through a GradBucket (the rasterizer's
        # gradient sink, ordered across the streams by the bucket), not through autograd's
        # per-leaf accumulation, whose node would be shared between the streams
        bucket = vp.GradBucket(leaves)
        bucket.zero_grad()
        sts = [torch.cuda.Stream(device) for _ in range(2)]
        pre = (prepare_views(rasts, leaves[0], leaves[2], shs=leaves[1], scales=leaves[3], rotations=leaves[4],
                             streams=[sts[k % 2] for k in range(len(rasts))]) if prepared else [None] * len(rasts))
        outs = []
        main = torch.cuda.current_stream()
        for st in sts:
            st.wait_stream(main)
        for k, (r, p) in enumerate(zip(rasts, pre)):
            with torch.cuda.stream(sts[k % 2]):
                m2 = torch.zeros_like(leaves[0], requires_grad=True)
                img, radii = r(means3D=leaves[0], means2D=m2, opacities=leaves[2], shs=leaves[1], scales=leaves[3],
                               rotations=leaves[4], prepared=p)
                (img * dpix).sum().backward()
                outs.append((img.detach().clone(), radii.clone(), m2.grad.clone()))
        for st in sts:
            main.wait_stream(st)
        bucket.finalize()
        torch.cuda.synchronize()
        grads = [t.grad.clone() for t in leaves]
        bucket.close()
        return outs, grads

    a_out, a_grad = run(False)
    b_out, b_grad = run(True)
    for (ia, ra, ma), (ib, rb, mb) in zip(a_out, b_out):
        assert torch.equal(ia, ib) and torch.equal(ra, rb) and torch.equal(ma, mb)
        assert (ra > 0).any()
    for ga, gb in zip(a_grad, b_grad):
        assert torch.equal(ga, gb)
    # a prepared view is checked against the call and used once
    pre = prepare_views(rasts[:2], sc.means3D, sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    m2 = torch.zeros_like(sc.means3D)
    with pytest.raises(RuntimeError, match="does not match"):
        rasts[1](means3D=sc.means3D, means2D=m2, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                 rotations=sc.rotations, prepared=pre[0])
    rasts[0](means3D=sc.means3D, means2D=m2, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
             rotations=sc.rotations, prepared=pre[0])
    with pytest.raises(RuntimeError, match="used once"):
        rasts[0](means3D=sc.means3D, means2D=m2, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                 rotations=sc.rotations, prepared=pre[0])


@pytest.mark.parametrize("deg", [-1, 0, 1, 2], ids=["colors", "sh0", "sh1", "sh2"])
def test_prepared_deferred_views_every_degree(device, deg):
    """prepare_views (gs_forward_preprocess_views) and the deferred per-Gaussian half
    (gs_backward_gaussians) for precomputed colours and SH degrees 0-2 (degree 3: the tests above):
    three views' images, radii and gradient sums bit-identical to plain per-view calls whose
    gradients autograd sums with += in view order."""
    import gs_view_parallel as vp
    from diff_gaussian_rasterization import GaussianRasterizer, prepare_views

    W, H = 160, 120
    cams = gs_scenes.circle_cameras(3, 6.0, W, H)
    sc = gs_scenes.random_gaussians(5000, max(deg, 0), seed=31, ball_radius=2.0).to(device)
    rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(c, max(deg, 0), device=device)) for c in cams]
    dpix = [gs_scenes.dl_dimage(H, W, seed=60 + v).to(device) for v in range(3)]
    colors = torch.rand((sc.P, 3), generator=torch.Generator().manual_seed(3)).to(device)
    feat = colors if deg < 0 else sc.shs

    def leaves():
        return [t.clone().requires_grad_(True) for t in (sc.means3D, feat, sc.opacities, sc.scales, sc.rotations)]

    def call(r, p, m2, prepared=None):
        kw = dict(colors_precomp=p[1]) if deg < 0 else dict(shs=p[1])
        return r(means3D=p[0], means2D=m2, opacities=p[2], scales=p[3], rotations=p[4], prepared=prepared, **kw)

    ref, outs_ref = None, []
    for r, dp in zip(rasts, dpix):
        p = leaves()
        m2 = torch.zeros_like(p[0], requires_grad=True)
        img, radii = call(r, p, m2)
        img.backward(dp)
        outs_ref.append((img.detach().clone(), radii.clone(), m2.grad.clone()))
        g = [t.grad for t in p]
        ref = [x.clone() for x in g] if ref is None else [a + b for a, b in zip(ref, g)]
    p = leaves()
    b = vp.GradBucket(p, lazy_zero=True, defer=True)
    b.zero_grad()
    kw = dict(colors_precomp=p[1]) if deg < 0 else dict(shs=p[1])
    pre = prepare_views(rasts, p[0], p[2], scales=p[3], rotations=p[4], **kw)
    outs = []
    for r, pv, dp in zip(rasts, pre, dpix):
        m2 = torch.zeros_like(p[0], requires_grad=True)
        img, radii = call(r, p, m2, pv)
        img.backward(dp)
        outs.append((img.detach().clone(), radii.clone(), m2))
    b.finalize()
    torch.cuda.synchronize()
    for (ia, ra, ma), (ib, rb, m2) in zip(outs_ref, outs):
        assert torch.equal(ia, ib) and torch.equal(ra, rb) and torch.equal(ma, m2.grad)
        assert (ra > 0).any()
    for k, (t, x) in enumerate(zip(p, ref)):
        assert torch.equal(t.grad, x), k
    b.close()
