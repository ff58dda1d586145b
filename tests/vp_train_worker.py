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
    """Two replicas per rank from the same scene: A steps through the bucket all-reduce + FusedAdam,
    B through gs_view_parallel.ShardedAdam (reduce-scatter -> FusedAdam on the rank's row slices ->
    all-gather, 3 row chunks); three steps, reduce_densify_stats, gather_state, densify_and_prune (same
    seeded draws for A and B, rank 0's broadcast), two more steps.  A and B bit-identical on every rank
    and B identical across the ranks."""
    import gs_train_step as ts
    import gs_view_parallel as vp

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sc, settings, gts = setup(dev, rank)
    mine = [(settings[v], gts[v]) for v in vp.shard_views(4, rank, world)]
    runs = []
    for sharded in (False, True):
        m = ts.TrainModel(sc, dev, fused=True)
        bucket = vp.GradBucket([m._xyz, m._features_dc, m._features_rest, m._opacity, m._scaling, m._rotation])
        sh = vp.ShardedAdam(m.optimizer, bucket, chunks=3) if sharded else None
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
    (ta, p0a, pa, sa), (tb, p0b, pb, sb) = runs
    same = len(ta) == len(tb) and all(torch.equal(x, y) for x, y in zip(ta, tb))
    replicas = vp.check_replicas(tb)
    if rank == 0:
        ok = same and replicas and pa == pb and pa != p0a and sa == sb == [5.0] * 6
        msg = ("OK " if ok else "FAIL ") + (f"sharded == all-reduce {same}; sharded replicas equal {replicas}; "
                                            f"P {p0a} -> {pa} / {pb}; steps {sa} / {sb}")
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
        sh = vp.ShardedAdam(m.optimizer, b, chunks=3) if sharded else None
        for _ in range(2):
            ts.train_step_views(m, b, views, sharded=sh)
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
    # the sharded step through RCCL (reduce-scatter / all-gather at world 1, coalesced per chunk)
    sharded_same = all(torch.equal(a, b) for a, b in zip(ref, run(sharded=True)))
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
    {"gloo2": gloo2, "gloo2_sharded": gloo2_sharded, "nccl1": nccl1}[sys.argv[1]]()
