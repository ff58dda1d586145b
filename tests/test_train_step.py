"""One train.py iteration through gs_train_step (render -> L1 + SSIM -> backward -> densification
statistics -> Adam), with the fused HIP glue against the reference's torch glue
(/root/reference/train.py:86-128, scene/gaussian_model.py:95-115, 405-407) on the same scene, and
a densify step on the trained model (gaussian_model.py:391-403)."""
import numpy as np
import pytest
import torch

import gs_scenes

pytestmark = pytest.mark.gpu


def _setup(device, P=3000, W=160, H=120, deg=3):
    cam = gs_scenes.identity_camera(W, H)
    sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=4)
    settings = gs_scenes.raster_settings_for(cam, deg, device=device)
    gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(9)).to(device)
    return sc, settings, gt


def test_fused_train_step_matches_torch_glue(device):
    """Loss per iteration within 1e-5 relative, densification statistics equal (max_radii2D, denom
    exactly; the gradient-norm sums at rtol 1e-5), parameters after 3 iterations within 2 Adam
    steps of the largest learning rate (Adam's first steps are sign(g) lr, so a gradient component
    near zero may take either sign when the activations differ by an ulp) and equal for >= 99 % of
    the entries at 1e-6 relative + 1e-7."""
    import gs_train_step as ts

    sc, settings, gt = _setup(device)
    runs = {}
    for fused in (True, False):
        m = ts.TrainModel(sc, device, fused=fused)
        losses = [ts.train_step(m, settings, gt, fused=fused).item() for _ in range(3)]
        torch.cuda.synchronize()
        runs[fused] = (m, losses)
    (mf, lf), (mt, lt) = runs[True], runs[False]
    np.testing.assert_allclose(lf, lt, rtol=1e-5)
    assert lf[2] < lf[0]  # the loss goes down
    np.testing.assert_array_equal(mf.max_radii2D.cpu().numpy(), mt.max_radii2D.cpu().numpy())
    np.testing.assert_array_equal(mf.denom.cpu().numpy(), mt.denom.cpu().numpy())
    np.testing.assert_allclose(mf.xyz_gradient_accum.cpu().numpy(), mt.xyz_gradient_accum.cpu().numpy(),
                               rtol=1e-5, atol=1e-9)
    for name, lr in (("_xyz", ts.POSITION_LR_INIT), ("_features_dc", ts.FEATURE_LR),
                     ("_features_rest", ts.FEATURE_LR / 20), ("_opacity", ts.OPACITY_LR),
                     ("_scaling", ts.SCALING_LR), ("_rotation", ts.ROTATION_LR)):
        a = getattr(mf, name).detach().cpu().numpy()
        b = getattr(mt, name).detach().cpu().numpy()
        d = np.abs(a - b)
        assert d.max() <= 2 * 3 * lr + 1e-6, f"{name}: max |d| {d.max():.3e}"
        close = d <= 1e-6 * np.abs(b) + 1e-7
        assert close.mean() >= 0.99, f"{name}: only {close.mean():.4f} of the entries agree"


def test_densify_after_train_steps(device):
    """densify_and_prune on the trained model (synthetic statistics: 5 % over the threshold):
    clones + split children appended, parents pruned, optimizer state resized with the parameters,
    and the next iteration runs at the new size."""
    import gs_train_step as ts

    sc, settings, gt = _setup(device)
    m = ts.TrainModel(sc, device, fused=True)
    ts.train_step(m, settings, gt)
    P0 = m.P
    ts.synthetic_densify_stats(m, frac=0.05, seed=1)
    grads = (m.xyz_gradient_accum / m.denom).squeeze(1)
    over = grads >= ts.DENSIFY_GRAD_THRESHOLD
    big = torch.exp(m._scaling).max(1).values > m.percent_dense * 2.0
    n_clone, n_split = int((over & ~big).sum()), int((over & big).sum())
    assert n_clone > 0 and n_split > 0
    ts.densify(m, extent=2.0)
    torch.cuda.synchronize()
    assert m.P == P0 + n_clone + n_split  # + 2 children - 1 parent per split (no pruning here)
    for grp in m.optimizer.param_groups:
        p = grp["params"][0]
        assert p.shape[0] == m.P
        st = m.optimizer.state[p]
        assert st["exp_avg"].shape == p.shape and st["exp_avg_sq"].shape == p.shape
    assert m.max_radii2D.shape[0] == m.P and not m.denom.any()
    loss = ts.train_step(m, settings, gt).item()
    assert np.isfinite(loss)


def _state(m):
    out = []
    for grp in m.optimizer.param_groups:
        p = grp["params"][0]
        st = m.optimizer.state[p]
        out += [p.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone()]
    return out


def test_split_sh_train_steps_bitwise_equal_concatenated(device):
    """Three fused train steps with the SH rows read in place (split_sh=True: shs is only the
    gradient carrier) and with the concatenated rows (split_sh=False): parameters and both Adam
    moments bit-identical."""
    import gs_train_step as ts

    sc, settings, gt = _setup(device)
    res = []
    for split in (True, False):
        m = ts.TrainModel(sc, device, fused=True)
        for _ in range(3):
            ts.train_step(m, settings, gt, split_sh=split)
        torch.cuda.synchronize()
        res.append(_state(m))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_split_sh_with_gradient_bucket_equals_autograd(device):
    """sh_split with a non-deferring GradBucket over the rasterizer's inputs (the lazy_zero claim
    path: the kernels write dL/dshs of the carrier straight into the bucket view) equals the plain
    autograd gradients bit for bit, for two accumulated views."""
    import gs_train
    import gs_view_parallel as vp
    from diff_gaussian_rasterization import GaussianRasterizer

    import gs_train_step as ts

    sc, settings, gt = _setup(device)
    m = ts.TrainModel(sc, device, fused=True)
    _, opac, scales, rots = gs_train.activate_values(m._features_dc, m._features_rest, m._opacity, m._scaling,
                                                     m._rotation, with_sh=False)
    P, M = m.P, 1 + m._features_rest.shape[1]
    dpix = [gs_scenes.dl_dimage(settings.image_height, settings.image_width, seed=s).to(device) for s in (3, 4)]

    def leaves():
        return [m._xyz.detach().clone().requires_grad_(True),
                torch.empty((P, M, 3), device=device).requires_grad_(True),
                opac.clone().requires_grad_(True), scales.clone().requires_grad_(True),
                rots.clone().requires_grad_(True)]

    def views(p):
        for dp in dpix:
            m2 = torch.zeros_like(p[0], requires_grad=True)
            img, _ = GaussianRasterizer(settings)(means3D=p[0], means2D=m2, shs=p[1], opacities=p[2], scales=p[3],
                                                  rotations=p[4], sh_split=(m._features_dc, m._features_rest))
            img.backward(dp)

    ref = leaves()
    views(ref)
    got = leaves()
    b = vp.GradBucket(got, lazy_zero=True)
    b.zero_grad()
    views(got)
    b.finalize()
    torch.cuda.synchronize()
    for a, r in zip(got, ref):
        assert torch.equal(a.grad, r.grad)
    b.close()


def test_bounded_train_step_raises_at_its_own_loss_item(device):
    """A train step with a bounded forward (binning_capacity) that fits equals the plain step bit
    for bit; one whose view overflows its capacity raises at that iteration's loss.item() sync
    (train.py:99), not one call later, and the status is cleared after it."""
    import gs_train_step as ts
    from diff_gaussian_rasterization import bounded_status, last_num_rendered

    sc, settings, gt = _setup(device)
    a, b = ts.TrainModel(sc, device), ts.TrainModel(sc, device)
    la = ts.train_step(a, settings, gt, loss_item=True)
    n = last_num_rendered()
    lb = ts.train_step(b, settings, gt, loss_item=True, binning_capacity=n + 64)
    assert la == lb
    for name in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    names = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")

    def snapshot(m):
        st = m.optimizer.state_dict()["state"]
        moments = {(i, k): v.clone() for i, s in st.items() for k, v in s.items() if torch.is_tensor(v)}
        steps = {(i, k): v for i, s in st.items() for k, v in s.items() if not torch.is_tensor(v)}
        return ({n: getattr(m, n).detach().clone() for n in names}, moments, steps,
                [t.clone() for t in (m.max_radii2D, m.xyz_gradient_accum, m.denom)])

    before = snapshot(b)
    with pytest.raises(RuntimeError, match="binning capacity"):
        ts.train_step(b, settings, gt, loss_item=True, binning_capacity=n // 4)
    assert bounded_status() == (0, 0)
    # the overflowing iteration raised at its loss.item() (train.py:99), before the statistics and
    # the optimizer step: no parameter, moment, step count or statistic took its gradients
    after = snapshot(b)
    for n_ in names:
        assert torch.equal(before[0][n_], after[0][n_]), n_
    assert before[1].keys() == after[1].keys() and before[2] == after[2]
    for k in before[1]:
        assert torch.equal(before[1][k], after[1][k]), k
    for x, y in zip(before[3], after[3]):
        assert torch.equal(x, y)


def test_fused_adam_bounded_overflow_raises_with_state_untouched(device):
    """The fused-Adam step launches its backward + Adam before the host reads the loss and the
    forward's status (train_step's early read-back); an overflowing bounded iteration must still
    raise at its own loss.item() with parameters, moments, step counts and statistics untouched:
    the kernel skips the update of a view whose forward recorded an error and the step counts are
    committed only after the check.  The next (fitting) iteration then equals the plain step's."""
    import gs_train_step as ts
    from diff_gaussian_rasterization import bounded_status, last_num_rendered

    sc, settings, gt = _setup(device)
    a, b = ts.TrainModel(sc, device), ts.TrainModel(sc, device)
    ts.train_step(a, settings, gt, loss_item=True, fuse_adam=True)
    n = last_num_rendered()
    ts.train_step(b, settings, gt, loss_item=True, fuse_adam=True, binning_capacity=n + 64)
    names = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")

    def snapshot(m):
        torch.cuda.synchronize()
        st = m.optimizer.state_dict()["state"]
        moments = {(i, k): v.clone() for i, s in st.items() for k, v in s.items() if torch.is_tensor(v) and v.dim()}
        steps = {(i, k): float(v) for i, s in st.items() for k, v in s.items() if not torch.is_tensor(v) or not v.dim()}
        return ({n_: getattr(m, n_).detach().clone() for n_ in names}, moments, steps,
                [t.clone() for t in (m.max_radii2D, m.xyz_gradient_accum, m.denom)])

    before = snapshot(b)
    with pytest.raises(RuntimeError, match="binning capacity"):
        ts.train_step(b, settings, gt, loss_item=True, fuse_adam=True, binning_capacity=n // 4)
    assert bounded_status() == (0, 0)
    after = snapshot(b)
    for n_ in names:
        assert torch.equal(before[0][n_], after[0][n_]), n_
    assert before[1].keys() == after[1].keys() and before[2] == after[2]
    for k in before[1]:
        assert torch.equal(before[1][k], after[1][k]), k
    for x, y in zip(before[3], after[3]):
        assert torch.equal(x, y)
    # the model continues as if the failed iteration had not happened
    la = ts.train_step(a, settings, gt, loss_item=True, fuse_adam=True)
    lb = ts.train_step(b, settings, gt, loss_item=True, fuse_adam=True, binning_capacity=n + 64)
    assert la == lb
    for n_ in names:
        assert torch.equal(getattr(a, n_), getattr(b, n_)), n_


def _full_snapshot(m):
    names = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")
    torch.cuda.synchronize()
    st = m.optimizer.state_dict()["state"]
    moments = {(i, k): v.clone() for i, s in st.items() for k, v in s.items() if torch.is_tensor(v) and v.dim()}
    steps = {(i, k): float(v) for i, s in st.items() for k, v in s.items() if not torch.is_tensor(v) or not v.dim()}
    return ({n_: getattr(m, n_).detach().clone() for n_ in names}, moments, steps,
            [t.clone() for t in (m.max_radii2D, m.xyz_gradient_accum, m.denom)])


def _assert_same_snapshot(before, after):
    for n_ in before[0]:
        assert torch.equal(before[0][n_], after[0][n_]), n_
    assert before[1].keys() == after[1].keys() and before[2] == after[2]
    for k in before[1]:
        assert torch.equal(before[1][k], after[1][k]), k
    for x, y in zip(before[3], after[3]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("fuse_adam", [True, False])
def test_lookback_timeout_raises_in_its_own_step_with_state_untouched(device, fuse_adam):
    """A read-back forward whose offsets scan's look-back wait times out (forced with
    gs_debug_set_scan_spin_limit(0)) does not raise in its own rasterizer call; train_step(loss_item=
    True) must raise in that iteration (train.py:99, before :127) with parameters, moments, step
    counts and statistics untouched -- with the fused backward + Adam launched before the loss
    read-back, the view's flags word (copied out behind the loss) is what tells the host that the
    kernel skipped the update.  The report is consumed: the next iterations run clean and equal a
    model that never saw the failed one."""
    import gs_train_step as ts
    from diff_gaussian_rasterization import _native

    lib = _native.load()
    sc, settings, gt = _setup(device)  # 3000 Gaussians: two look-back tiles in the offsets scan
    a, b = ts.TrainModel(sc, device), ts.TrainModel(sc, device)
    ts.train_step(a, settings, gt, loss_item=True, fuse_adam=fuse_adam)
    ts.train_step(b, settings, gt, loss_item=True, fuse_adam=fuse_adam)
    before = _full_snapshot(b)
    prev = lib.gs_debug_set_scan_spin_limit(0)
    try:
        with pytest.raises(RuntimeError, match="look-back wait"):
            ts.train_step(b, settings, gt, loss_item=True, fuse_adam=fuse_adam)
    finally:
        lib.gs_debug_set_scan_spin_limit(prev)
    _assert_same_snapshot(before, _full_snapshot(b))
    for _ in range(2):
        la = ts.train_step(a, settings, gt, loss_item=True, fuse_adam=fuse_adam)
        lb = ts.train_step(b, settings, gt, loss_item=True, fuse_adam=fuse_adam)
        assert la == lb
    _assert_same_snapshot(_full_snapshot(a), _full_snapshot(b))


def test_fused_adam_commit_follows_its_own_view_not_earlier_flags(device, monkeypatch):
    """Another bounded forward that overflows while this step is in flight (queued after this step's
    forward checked the device's bounded status, here: from inside the step's loss call) leaves its
    flags in the device-wide status.  The fused-Adam step's own view is valid, so its update must be
    committed -- its flags word is clean -- and the foreign flags reported after the commit:
    parameters, moments and step counts stay consistent (equal to a model stepped as often)."""
    import gs_loss
    import gs_train_step as ts
    from diff_gaussian_rasterization import bounded_status, last_num_rendered

    sc, settings, gt = _setup(device)
    a, b = ts.TrainModel(sc, device), ts.TrainModel(sc, device)
    ts.train_step(a, settings, gt, loss_item=True, fuse_adam=True)
    n = last_num_rendered()
    ts.train_step(b, settings, gt, loss_item=True, fuse_adam=True, binning_capacity=n + 64)
    c = ts.TrainModel(sc, device)
    orig = gs_loss.photometric_loss

    def loss_with_foreign_overflow(*args, **kw):
        monkeypatch.setattr(gs_loss, "photometric_loss", orig)
        with torch.no_grad():  # an overflowing bounded render of another model, never polled by its caller
            ts.render(c, settings, fused=True, binning_capacity=n // 4)
        return orig(*args, **kw)

    monkeypatch.setattr(gs_loss, "photometric_loss", loss_with_foreign_overflow)
    with pytest.raises(RuntimeError, match="binning capacity"):
        ts.train_step(b, settings, gt, loss_item=True, fuse_adam=True, binning_capacity=n + 64)
    assert bounded_status() == (0, 0)
    ts.train_step(a, settings, gt, loss_item=True, fuse_adam=True)
    _assert_same_snapshot(_full_snapshot(a), _full_snapshot(b))


def test_bounded_overflow_in_a_captured_step_raises_in_the_loop(device):
    """render -> L1 + SSIM -> backward with a bounded forward, captured once into a HIP graph
    (torch.cuda.CUDAGraph) and replayed in a training loop that polls bounded_status() at its
    per-iteration sync: replays that fit report nothing; after the capacity is exceeded (the scene
    grown in place past it) the loop's poll raises at that iteration."""
    import gs_loss
    import gs_train_step as ts
    from diff_gaussian_rasterization import bounded_status, last_num_rendered

    sc, settings, gt = _setup(device)
    m = ts.TrainModel(sc, device)
    ts.train_step(m, settings, gt, loss_item=True)
    n = last_num_rendered()
    static = {}

    def step():
        img, _, _ = ts.render(m, settings, fused=True, binning_capacity=n + 256)
        loss, _ = gs_loss.photometric_loss(img, gt)
        loss.backward()
        static["loss"] = loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):  # warm-up on the capture stream
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    bounded_status()
    # the warm-up's loss would keep its autograd graph (and the leaves' AccumulateGrad nodes, made on
    # the warm-up stream) alive into the capture, which runs on the capture stream
    static.clear()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
        static["loss"].item()
        assert bounded_status() == (0, 0)
    # every Gaussian four times as large (in place: the graph reads the same parameter storage)
    with torch.no_grad():
        m._scaling.add_(float(np.log(4.0)))
    g.replay()
    static["loss"].item()
    with pytest.raises(RuntimeError, match="binning capacity"):
        bounded_status()


@pytest.mark.parametrize("active_degree,P", [(3, 3000), (2, 3000), (1, 3000), (0, 3000), (3, 2999)])
def test_fused_adam_train_step_bitwise_equal_unfused(device, active_degree, P, monkeypatch):
    """train_step(fuse_adam=True): the per-Gaussian backward fused with the Adam step
    (gs_backward_gaussians_adam) against the default step (backward, then FusedAdam.step_activated)
    over three iterations: every parameter, both Adam moments, the step counts and the densification
    statistics bit-identical, the same loss.item() values -- at the full SH degree and at an active
    degree below the 16 stored coefficients (train.py's oneupSHdegree schedule).  P = 2999 leaves a
    last workgroup of 183 rows: 549 / 8235 floats of features_dc / features_rest, not multiples of 4,
    so the SH update's scalar tail runs too (3000: 184 rows, float4s only)."""
    import gs_train
    import gs_train_step as ts

    sc, settings, gt = _setup(device, P=P)
    settings = settings._replace(sh_degree=active_degree)
    runs = []
    for fuse in (False, True):
        m = ts.TrainModel(sc, device, fused=True)
        if fuse:  # the fused step must not fall back to the unfused optimizer update
            def refuse(*a, **k):
                raise AssertionError("fused step fell back to step_activated")
            monkeypatch.setattr(gs_train.FusedAdam, "step_activated", refuse)
            # ... nor run the statistics as their own launch (they are in the fused pass, ABI 16)
            monkeypatch.setattr(gs_train, "densify_stats", refuse)
        losses = [ts.train_step(m, settings, gt, loss_item=True, fuse_adam=fuse) for _ in range(3)]
        torch.cuda.synchronize()
        monkeypatch.undo()
        steps = [float(m.optimizer.state[g["params"][0]]["step"]) for g in m.optimizer.param_groups]
        runs.append((losses, _state(m), steps, [t.clone() for t in (m.max_radii2D, m.xyz_gradient_accum, m.denom)],
                     m))
    (la, sa, ta, da, ma), (lb, sb, tb, db, mb) = runs
    assert la == lb and ta == tb == [3.0] * 6
    for k, (a, b) in enumerate(zip(sa, sb)):
        assert torch.equal(a, b), k
    for a, b in zip(da, db):
        assert torch.equal(a, b)
    assert mb.denom.sum() > 0
    for name in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"):
        assert getattr(mb, name).grad is None, name


@pytest.mark.parametrize("loss_item", [True, False])
def test_fused_adam_train_step_without_stats_leaves_them(device, loss_item):
    """train_step(fuse_adam=True, densify_stats=False) (past densify_until_iter): the fused pass
    updates the parameters as with statistics and leaves max_radii2D / xyz_gradient_accum / denom
    untouched; with statistics, denom counts the visible Gaussians (radii > 0) of each step."""
    import gs_train_step as ts

    sc, settings, gt = _setup(device)
    ma, mb = ts.TrainModel(sc, device, fused=True), ts.TrainModel(sc, device, fused=True)
    for _ in range(2):
        ts.train_step(ma, settings, gt, loss_item=loss_item, fuse_adam=True, densify_stats=False)
        ts.train_step(mb, settings, gt, loss_item=loss_item, fuse_adam=True, densify_stats=True)
    torch.cuda.synchronize()
    for t in (ma.max_radii2D, ma.xyz_gradient_accum, ma.denom):
        assert int(torch.count_nonzero(t)) == 0
    for a, b in zip(_state(ma), _state(mb)):
        assert torch.equal(a, b)
    assert mb.denom.sum() > 0 and float(mb.denom.max()) <= 2.0
    assert torch.equal(mb.denom.reshape(-1) > 0, mb.max_radii2D.reshape(-1) > 0)


def test_fused_adam_train_step_releases_its_sinks(device):
    """After a fused-Adam step the rasterizer inputs are no longer gradient sinks: a plain autograd
    backward through the model's xyz afterwards gets its own .grad."""
    import gs_train_step as ts
    from diff_gaussian_rasterization import _sink_owner

    sc, settings, gt = _setup(device, P=500)
    m = ts.TrainModel(sc, device, fused=True)
    ts.train_step(m, settings, gt, fuse_adam=True)
    assert _sink_owner(m._xyz) is None
    img, _, _ = ts.render(m, settings, fused=True)
    img.sum().backward()
    assert m._xyz.grad is not None and m._xyz.grad.abs().sum() > 0
