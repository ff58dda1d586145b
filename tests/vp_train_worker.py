"""Worker of the view-parallel training tests in tests/test_gpu_multiview.py (GPU; launched before the
test process touches the GPU).

mode "gloo2" (torchrun, 2 ranks, gloo, both on cuda:0): each rank holds a replica of one model
(gs_train_step.TrainModel, FusedAdam) with a GradBucket over its six parameters and trains on its
own views (gs_train_step.train_step_views: render -> L1 + SSIM -> backward into the bucket -> ONE
all-reduce -> Adam).  Then the densification statistics are reduced (gs_view_parallel.
reduce_densify_stats), a densify_and_prune step runs (split draws: every rank's generator is seeded
differently, rank 0's draw is broadcast), the bucket is rebound to the new parameters, and two more
steps run.  Every parameter and Adam moment must be bit-identical across the ranks at the end
(gs_view_parallel.check_replicas), and the step must have split and cloned something.

mode "nccl1" (one process, RCCL, world size 1): the same step through the RCCL all-reduce equals the
step without a process group, bit for bit; the collective runs (world 1: in place).

Writes "OK ..." or "FAIL ..." to $GS_VP_OUT (rank 0).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

P, W, H, DEG = 20_000, 320, 240, 3


def setup(dev, rank):
    import gs_scenes

    cams = gs_scenes.jittered_cameras(4, W, H, seed=11)
    sc = gs_scenes.random_gaussians(P, DEG, cam=cams[0], seed=3)
    settings = [gs_scenes.raster_settings_for(c, DEG, device=dev) for c in cams]
    gts = [torch.rand((3, H, W), generator=torch.Generator().manual_seed(50 + v)).to(dev) for v in range(4)]
    return sc, settings, gts


def model_tensors(m):
    out = []
    for grp in m.optimizer.param_groups:
        p = grp["params"][0]
        st = m.optimizer.state[p]
        out += [p.detach(), st["exp_avg"], st["exp_avg_sq"]]
    return out


def gloo2():
    import gs_train_step as ts
    import gs_view_parallel as vp

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(1000 + rank)  # different generators: only the broadcast keeps the split draws equal
    sc, settings, gts = setup(dev, rank)
    m = ts.TrainModel(sc, dev, fused=True)
    bucket = vp.GradBucket([m._xyz, m._features_dc, m._features_rest, m._opacity, m._scaling, m._rotation])
    mine = [(settings[v], gts[v]) for v in vp.shard_views(4, rank, world)]
    for _ in range(3):
        ts.train_step_views(m, bucket, mine)
    ok_before = vp.check_replicas(model_tensors(m))
    vp.reduce_densify_stats(m.xyz_gradient_accum, m.denom, m.max_radii2D)
    # push a share of the Gaussians over the threshold (the real statistics of 3 small steps rarely
    # cross it), identically on both ranks
    g = torch.Generator(device=dev).manual_seed(7)
    boost = (torch.rand((m.P, 1), generator=g, device=dev) < 0.05).float() * 1e-2
    m.xyz_gradient_accum += boost * m.denom
    P0 = m.P
    old_flat = bucket.flat
    ts.densify(m, extent=0.5)
    rebound = bucket.flat is not old_flat and bucket.numel == 59 * m.P and m._xyz.grad is not None
    for _ in range(2):
        ts.train_step_views(m, bucket, mine)
    torch.cuda.synchronize()
    ok_after = vp.check_replicas(model_tensors(m))
    # the broadcast matters: the ranks' own draws differ
    n = torch.randn((8,), device=dev)
    lo, hi = n.clone(), n.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    draws_differ = not torch.equal(lo, hi)
    if rank == 0:
        ok = ok_before and ok_after and rebound and m.P != P0 and draws_differ
        msg = ("OK " if ok else "FAIL ") + (f"replicas equal before densify {ok_before}, after {ok_after}; bucket "
                                            f"rebound {rebound}; P {P0} -> {m.P}; rank draws differ {draws_differ}")
        with open(os.environ["GS_VP_OUT"], "w") as f:
            f.write(msg + "\n")
    dist.barrier()
    bucket.close()
    dist.destroy_process_group()


def gloo2_sharded():
    """Three replicas per rank from the same scene: A steps through the bucket all-reduce + FusedAdam,
    B through gs_view_parallel.ShardedAdam (reduce-scatter -> FusedAdam on the rank's row slices ->
    all-gather, 3 row chunks), C through ShardedAdam(overlap=True) (the all-gathers left in flight:
    the next step's activation and preprocess wait for them chunk by chunk, the bucket is zero-filled
    on the collective stream); three steps, reduce_densify_stats, gather_state, densify_and_prune (same
    seeded draws, rank 0's broadcast), two more steps.  A, B and C bit-identical on every rank and B,
    C identical across the ranks."""
    import gs_train_step as ts
    import gs_view_parallel as vp

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sc, settings, gts = setup(dev, rank)
    mine = [(settings[v], gts[v]) for v in vp.shard_views(4, rank, world)]
    runs = []
    for mode in ("allreduce", "sharded", "overlap"):
        m = ts.TrainModel(sc, dev, fused=True)
        bucket = vp.GradBucket([m._xyz, m._features_dc, m._features_rest, m._opacity, m._scaling, m._rotation])
        sh = vp.ShardedAdam(m.optimizer, bucket, chunks=3, overlap=mode == "overlap") if mode != "allreduce" else None
        for _ in range(3):
            ts.train_step_views(m, bucket, mine, sharded=sh)
        vp.reduce_densify_stats(m.xyz_gradient_accum, m.denom, m.max_radii2D)
        g = torch.Generator(device=dev).manual_seed(7)
        boost = (torch.rand((m.P, 1), generator=g, device=dev) < 0.05).float() * 1e-2
        m.xyz_gradient_accum += boost * m.denom
        if sh is not None:
            sh.gather_state()
        torch.manual_seed(1000 + rank)
        P0 = m.P
        ts.densify(m, extent=0.5)
        for _ in range(2):
            ts.train_step_views(m, bucket, mine, sharded=sh)
        if sh is not None:
            sh.gather_state()
        torch.cuda.synchronize()
        runs.append(([t.clone() for t in model_tensors(m)], P0, m.P,
                     [float(m.optimizer.state[g_["params"][0]]["step"]) for g_ in m.optimizer.param_groups]))
        bucket.close()
    (ta, p0a, pa, sa), (tb, p0b, pb, sb), (tc, p0c, pc, sc_) = runs
    same = len(ta) == len(tb) and all(torch.equal(x, y) for x, y in zip(ta, tb))
    same_o = len(ta) == len(tc) and all(torch.equal(x, y) for x, y in zip(ta, tc))
    replicas = vp.check_replicas(tb) and vp.check_replicas(tc)
    if rank == 0:
        ok = same and same_o and replicas and pa == pb == pc and pa != p0a and sa == sb == sc_ == [5.0] * 6
        msg = ("OK " if ok else "FAIL ") + (f"sharded == all-reduce {same}; overlapped sharded == all-reduce {same_o}; "
                                            f"sharded replicas equal {replicas}; P {p0a} -> {pa} / {pb} / {pc}; "
                                            f"steps {sa} / {sb} / {sc_}")
        with open(os.environ["GS_VP_OUT"], "w") as f:
            f.write(msg + "\n")
    dist.barrier()
    dist.destroy_process_group()


def gloo2_deferred():
    """bench.py's step shape on two gloo ranks (one GPU): the activated inputs are the leaves, a
    GradBucket(lazy_zero=True, defer=True) takes every view's per-Gaussian half for one pass at the
    optimizer step.  A: bucket.allreduce() + FusedAdam.step(); B: ShardedAdam (the deferred pass in
    row chunks, each chunk's reduce-scatter / update / all-gather on the side stream); C: the same
    with overlap=True (the next step's first forward waits for the all-gathers chunk by chunk through
    _C.row_waits).  Four steps; A, B, C bit-identical, B and C identical across the ranks."""
    import gs_scenes
    import gs_train
    import gs_view_parallel as vp
    from diff_gaussian_rasterization import GaussianRasterizer, _C

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sc, settings, _ = setup(dev, rank)
    d = sc.to(dev)
    mine = [settings[v] for v in vp.shard_views(4, rank, world)]
    dpix = [gs_scenes.dl_dimage(H, W, seed=90 + v).to(dev) for v in range(4)]
    mine_d = [dpix[v] for v in vp.shard_views(4, rank, world)]
    lrs = [1.6e-4, 2.5e-3, 5e-2, 5e-3, 1e-3]
    runs = []
    for mode in ("allreduce", "sharded", "overlap"):
        params = [t.clone().requires_grad_(True) for t in (d.means3D, d.shs, d.opacities, d.scales, d.rotations)]
        opt = gs_train.FusedAdam([{"params": [p], "lr": lr} for p, lr in zip(params, lrs)], lr=0.0, eps=1e-15)
        bucket = vp.GradBucket(params, lazy_zero=True, defer=True)
        sh = vp.ShardedAdam(opt, bucket, chunks=3, overlap=mode == "overlap") if mode != "allreduce" else None
        for _ in range(4):
            waits = sh.take_row_waits() if sh is not None else []
            bucket.zero_grad()
            for s_, dp in zip(mine, mine_d):
                m2 = torch.empty_like(params[0], requires_grad=True)
                with _C.row_waits(waits):
                    img, _ = GaussianRasterizer(s_)(means3D=params[0], means2D=m2, opacities=params[2],
                                                    shs=params[1], scales=params[3], rotations=params[4])
                waits = []
                img.backward(dp)
            if sh is None:
                bucket.allreduce()
                opt.step()
            else:
                sh.step()
        if sh is not None:
            sh.gather_state()
        torch.cuda.synchronize()
        runs.append([t.detach().clone() for p in params for t in (p, opt.state[p]["exp_avg"], opt.state[p]["exp_avg_sq"])])
        bucket.close()
    same_b = all(torch.equal(x, y) for x, y in zip(runs[0], runs[1]))
    same_c = all(torch.equal(x, y) for x, y in zip(runs[0], runs[2]))
    replicas = vp.check_replicas(runs[1]) and vp.check_replicas(runs[2])
    if rank == 0:
        ok = same_b and same_c and replicas
        msg = ("OK " if ok else "FAIL ") + (f"deferred sharded == all-reduce {same_b}; overlapped {same_c}; "
                                            f"replicas equal {replicas}")
        with open(os.environ["GS_VP_OUT"], "w") as f:
            f.write(msg + "\n")
    dist.barrier()
    dist.destroy_process_group()


def nccl1():
    import gs_train_step as ts
    import gs_view_parallel as vp

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sc, settings, gts = setup(dev, 0)
    views = [(settings[v], gts[v]) for v in range(2)]

    def run(sharded=False):
        m = ts.TrainModel(sc, dev, fused=True)
        b = vp.GradBucket([m._xyz, m._features_dc, m._features_rest, m._opacity, m._scaling, m._rotation])
        sh = vp.ShardedAdam(m.optimizer, b, chunks=3, overlap=sharded == "overlap") if sharded else None
        for _ in range(2):
            ts.train_step_views(m, b, views, sharded=sh)
        if sh is not None:
            sh.sync()
        torch.cuda.synchronize()
        b.close()
        return [t.clone() for t in model_tensors(m)]

    ref = run()  # no process group: the bucket is only finalized
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
    dist.init_process_group("nccl", device_id=dev)
    calls = []
    orig = dist.all_reduce
    dist.all_reduce = lambda *a, **k: calls.append(1) or orig(*a, **k)  # noqa: E731
    got = run()
    dist.all_reduce = orig
    same = all(torch.equal(a, b) for a, b in zip(ref, got))
    # the sharded step through RCCL (reduce-scatter / all-gather at world 1, coalesced per chunk),
    # and with the all-gathers overlapped into the next step
    sharded_same = all(torch.equal(a, b) for a, b in zip(ref, run(sharded=True)))
    sharded_same = sharded_same and all(torch.equal(a, b) for a, b in zip(ref, run(sharded="overlap")))
    # the chunked all-reduce (RCCL coalesced groups per Gaussian-row range, on a side stream,
    # overlapping the deferred per-Gaussian pass) against the bucket's one-shot finalize
    chunk_same = chunked_vs_finalize(sc, settings, dev)
    backend = dist.get_backend()
    dist.destroy_process_group()
    ok = same and len(calls) == 2 and backend == "nccl" and chunk_same and sharded_same
    msg = ("OK " if ok else "FAIL ") + (f"backend {backend}; all-reduces {len(calls)}; bitwise equal to no-group "
                                        f"{same}; chunked all-reduce equal to finalize {chunk_same}; sharded step "
                                        f"equal {sharded_same}")
    with open(os.environ["GS_VP_OUT"], "w") as f:
        f.write(msg + "\n")


def chunked_vs_finalize(sc, settings, dev):
    import gs_scenes
    import gs_view_parallel as vp
    from diff_gaussian_rasterization import GaussianRasterizer

    d = sc.to(dev)

    def run(chunks, reduce):
        params = [t.clone().requires_grad_(True) for t in (d.means3D, d.shs, d.opacities, d.scales, d.rotations)]
        b = vp.GradBucket(params, lazy_zero=True, defer=True, chunks=chunks)
        b.zero_grad()
        for v, s in enumerate(settings[:3]):
            m2 = torch.empty_like(params[0], requires_grad=True)
            img, _ = GaussianRasterizer(s)(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1],
                                           scales=params[3], rotations=params[4])
            img.backward(gs_scenes.dl_dimage(H, W, seed=70 + v).to(dev))
        b.allreduce() if reduce else b.finalize()
        torch.cuda.synchronize()
        out = b.flat.clone()
        b.close()
        return out

    return bool(torch.equal(run(4, True), run(1, False)))


if __name__ == "__main__":
    {"gloo2": gloo2, "gloo2_sharded": gloo2_sharded, "gloo2_deferred": gloo2_deferred, "nccl1": nccl1}[sys.argv[1]]()
