"""bench.py -- rasterizer forward+backward throughput on MI355X (BASELINE.json metric).

Other BASELINE configs: --workload c1 / c2 (smaller), c4 (8 ring views of a 1M ball scene, one
step = the 8 views sharded over the ranks + one all-reduce: strong scaling), c5 (5M Gaussians: HBM
footprint in "hbm").

Workload (N=1): BASELINE.json configs[2] "C3" -- 1M Gaussians, SH degree 3, 1920x1080, 16x16
tiles (synthetic scene per SURVEY.md §8d: frustum-uniform means, seed 0).  One iteration = one
view's GaussianRasterizer forward + backward (dL/dimage fixed, seed 1) through the drop-in
package, i.e. exactly what train.py:86-93 runs on the rasterizer; `value` counts iterations
(views) per second over the whole job.  A step = --views-per-rank views per rank (default 4 at
every N, so the 1/2/4/8-GPU lines divide the same step) whose gradients accumulate in one flat
59-float/Gaussian bucket (the .grad tensors are views into it; the rasterizer's backward writes
/ adds straight into them), followed with --gpus N>1 (torchrun, one rank per GPU, RCCL) by ONE
all-reduce of that bucket (view-parallel data parallelism, weak scaling).

Output: one JSON line (rank 0) with the metric, a per-kernel HIP-event breakdown, the roofline of
the dominant kernel and the CPU oracle baseline timed on this host.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

# Only torch here: nothing that loads libgsrast.so or touches the GPU may run before the launcher
# below has decided whether this process is a rank or the parent of N ranks.
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

gs_scenes = vp = GaussianRasterizer = _C = _native = prepare_views = None


def _import_product():
    """The drop-in packages (loads libgsrast.so): imported by the ranks only."""
    global gs_scenes, vp, GaussianRasterizer, _C, _native, prepare_views
    import gs_scenes as _s
    import gs_view_parallel as _vp
    from diff_gaussian_rasterization import GaussianRasterizer as _R, _C as _c, _native as _n, prepare_views as _p

    gs_scenes, vp, GaussianRasterizer, _C, _native, prepare_views = _s, _vp, _R, _c, _n, _p


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) started without torchrun: start the N ranks as torchrun children
    (one process per GPU, RCCL) and exit with their status.  The parent has not touched the GPU
    (only torch is imported); rank 0 prints the JSON line to the inherited stdout."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC on this host driver
    return subprocess.call(cmd, env=env)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s HBM3E
# wave64 VALU issue peak: 256 CUs x 4 SIMD32 x 2.4 GHz / 2 cycles per wave64 instruction
VALU_PEAK_IPS = 256 * 4 * 2.4e9 / 2

WORKLOADS = {
    "c3": dict(P=1_000_000, deg=3, W=1920, H=1080, desc="C3: 1M Gaussians SH3 1920x1080, 16x16 tiles"),
    "c2": dict(P=100_000, deg=3, W=800, H=800, desc="C2: 100k Gaussians SH3 800x800"),
    "c1": dict(P=10_000, deg=0, W=256, H=256, desc="C1: 10k Gaussians SH0 256x256"),
    # C4: one step = the 8 ring views (sharded over the ranks) + one gradient all-reduce
    "c4": dict(P=1_000_000, deg=3, W=1920, H=1080, views=8,
               desc="C4: 1M Gaussians SH3 1920x1080 in a ball, 8 ring views sharded over ranks"),
    "c5": dict(P=5_000_000, deg=3, W=1920, H=1080, desc="C5: 5M Gaussians SH3 1920x1080 (HBM footprint)"),
}


def kernel_bytes(name, P, V, I, M, W, H, tiles, E=None, acc_frac=0.0, K=1):
    """Algorithmic (minimum) HBM bytes of ONE launch of each kernel.
    E: instances the render walks reach (sum over tiles of min(largest n_contrib, list length));
    only those are staged, and only those have backward records.  acc_frac: fraction of the
    preprocess_bwd launches that add into the gradient bucket (views after a step's first), which
    also read the old gradients (means3D 12 + sh 12M + opacity 4 + scales 12 + rotations 16 B).
    K: views per backward_gaussians launch (its inputs and outputs once, the K views' record sums,
    tile counts and clamp bits each)."""
    npix = W * H
    sh = 12 * M
    E = I if E is None else E
    # sorts, averaged over one view's launches: depth passes (4) -- the first reads the P keys in
    # index order and writes the V kept (key, id) pairs, the others move V pairs; above 1M
    # Gaussians the tile counts travel with them (aux); tile passes (2) over I pairs, the first
    # with identity ids (keys read only).  Histograms read one key per element.
    aux = P > 1_048_576
    depth_scatter = P * 4 + V * 8 + 3 * V * 16 + (P * 4 + V * 4 + 3 * V * 8 if aux else 0)
    tile_scatter = I * (4 + 8) + I * 16
    tile_hists = 2 if I > 4096 * 2048 else 1  # the duplicate counts the first tile pass up to 8M
    return {
        "radix_scatter": (depth_scatter + tile_scatter) // 6,
        "radix_hist": (P * 4 + 3 * V * 4 + tile_hists * I * 4) // (4 + tile_hists),
        "preprocess": P * (44 + sh + 4 + 4) + V * (48 + 32 + 4 + 1),
        "preprocess_views": P * (44 + sh + 4 + 4) + K * V * (48 + 32 + 4 + 1),
        "render_fwd": E * (4 + 4 + 48) + npix * 20 + tiles * 12,
        "render_bwd": E * (4 + 4 + 48 + 36) + npix * 20 + tiles * 12,
        "sum_records": E * 36 + I * 4 + V * (4 + 36),
        "preprocess_bwd": P * (8 + 44 + sh + 1 + 32 + 24 + sh) + V * 36 + int(acc_frac * P * (44 + sh)),
        "backward_gaussians": P * (40 + sh + 44 + sh) + K * (P * 5 + V * 36),
        "mean2d_grad": P * (4 + 12) + V * 8,
        "duplicate": V * (4 + 4 + 32 + 4) + I * 8,
        "ranges": I * 4 + tiles * 8,
    }.get(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100,
                    help="timed steps (4 views each by default: ~0.4 s at C3, long enough for an external utilisation sampler)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads (0 = the CPUs this job may use: affinity, cgroup quota, OMP_NUM_THREADS)")
    ap.add_argument("--cpu-runs", type=int, default=3, help="timed CPU-oracle runs after one warm-up (median)")
    ap.add_argument("--views-per-rank", type=int, default=4,
                    help="C1-C3/C5: views each rank renders (fwd+bwd, gradients accumulated in the bucket) per "
                         "step, i.e. per gradient all-reduce (DESIGN.md §7); value counts views")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams the views of a step are spread over (view k on stream k mod n): one "
                         "view's sorts and scans overlap another's tile passes; 1 = strictly serial")
    ap.add_argument("--no-fused-front", action="store_true",
                    help="run each view's preprocess in its own launch instead of one launch for the step's views "
                         "(prepare_views / gs_forward_preprocess_views)")
    ap.add_argument("--no-defer", action="store_true",
                    help="run the per-Gaussian backward per view (gs_backward_accumulate) instead of once per "
                         "step for all views (gs_backward_gaussians)")
    ap.add_argument("--no-train-step", action="store_true",
                    help="skip the secondary train.py-step measurement (SURVEY §8d metric (2); N=1 only)")
    ap.add_argument("--train-steps", type=int, default=20, help="timed iterations of the train-step measurement")
    ap.add_argument("--step-events", action="store_true",
                    help="diagnostic: record a HIP event after every timed step (no host syncs) and report the "
                         "per-step times of the timed region in deciles")
    ap.add_argument("--regions", type=int, default=5,
                    help="timed regions of --steps steps each; `value` is the median region's rate, every "
                         "region's rate is reported (`regions_iters_s`)")
    ap.add_argument("--sustain-s", type=float, default=2.0,
                    help="after the timed steps, keep stepping for this long (untimed for `value`) and report "
                         "the sustained rate too")
    ap.add_argument("--single-view-steps", type=int, default=100,
                    help="timed iterations of the batch-1 measurement (`single_view`: one view per step, per-view "
                         "backward, one stream: the shape of train.py's loop); 0 = skip")
    ap.add_argument("--c4-views-per-rank", type=int, default=0,
                    help="C4 weak scaling: every rank renders this many views of a ring of N x K cameras per step "
                         "(default 0: the 8 ring views of BASELINE config 4 sharded over the ranks, strong scaling)")
    ap.add_argument("--allreduce-chunks", type=int, default=4,
                    help="N > 1: the deferred per-Gaussian pass runs in this many Gaussian-row ranges and each "
                         "range's gradient rows are all-reduced (RCCL, side stream) as soon as they are written")
    ap.add_argument("--vp-train-steps", type=int, default=10,
                    help="timed optimizer steps of the view-parallel training measurement (`view_parallel_train`: "
                         "gs_train_step.train_step_views with the fused glue through ShardedAdam(overlap=True), the "
                         "bucket all-reduce + replicated Adam, and the exchange-free step, at every N); 0 = skip")
    ap.add_argument("--no-graph", action="store_true",
                    help="skip the HIP-graph measurement (the same step with bounded binning buffers, captured "
                         "once into a torch.cuda.CUDAGraph and replayed; N = 1)")
    ap.add_argument("--profile-pass-only", action="store_true",
                    help="run only the per-kernel event pass (W warm-up + K steps, one stream, as the default run's "
                         "second pass), print its per-kernel averages as one JSON line and exit: the command "
                         "`rocprofv3 --kernel-trace --stats` profiles to reproduce roofline.frac")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, check the process group against --gpus, print one JSON line and exit "
                         "before any GPU work (tests of the launcher; GS_BENCH_BACKEND=gloo runs it on CPU)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a mislabelled scaling point",
              file=sys.stderr)
        sys.exit(2)
    # GS_BENCH_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU (the
    # driver's multi-GPU runs use RCCL, one rank per GPU)
    backend = os.environ.get("GS_BENCH_BACKEND", "nccl")
    if args.launch_check:
        if world > 1:
            dist.init_process_group(backend)
            got = dist.get_world_size()
            dist.barrier()
        else:
            got = 1
        if got != args.gpus:
            sys.exit(2)
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": got, "backend": backend if world > 1 else None,
                              "ranks_from": "torchrun env"}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    _import_product()
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    if world > 1:
        if backend == "nccl":
            vp.init_from_env("nccl")
        else:
            torch.cuda.set_device(dev)
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, "process group size != --gpus"
    wl = WORKLOADS[args.workload]
    P, deg, W, H = wl["P"], wl["deg"], wl["W"], wl["H"]
    n_views = wl.get("views", 0)
    if n_views and args.c4_views_per_rank > 0:
        n_views = world * args.c4_views_per_rank  # weak C4: K views per rank on a ring of N x K cameras
    if n_views:  # C4: ball scene seen from a ring of cameras; this rank's share of the views
        cams = gs_scenes.circle_cameras(n_views, 6.0, W, H)
        my_views = vp.shard_views(n_views, rank, world)
        sc = gs_scenes.random_gaussians(P, deg, seed=0, ball_radius=2.0)
        cam = cams[my_views[0]]
    else:
        # the rank's K views of a step are K distinct nearby poses of the frustum-filled scene (view
        # 0 is the C3 identity camera the scene is drawn in; the others are turned by <= 2 degrees and
        # moved by <= 0.05); ranks draw different poses
        cam = gs_scenes.identity_camera(W, H)
        k_views = max(1, args.views_per_rank)
        cams = gs_scenes.jittered_cameras(k_views, W, H, seed=7 + rank) if k_views > 1 else [cam]
        cams[0] = cam
        my_views = list(range(k_views))
        sc = gs_scenes.random_gaussians(P, deg, cam=cam, seed=0)
    settings = gs_scenes.raster_settings_for(cam, deg, device=dev)
    d = sc.to(dev)
    M = d.shs.shape[1]
    params = [t.clone().requires_grad_(True) for t in (d.means3D, d.shs, d.opacities, d.scales, d.rotations)]
    means2D = torch.zeros_like(params[0], requires_grad=True)
    dpix = gs_scenes.dl_dimage(H, W, seed=1).to(dev)
    rasts = [GaussianRasterizer(gs_scenes.raster_settings_for(cams[v], deg, device=dev)) for v in my_views]
    rast = rasts[0]
    # the parameters' .grad are views of ONE flat bucket; the rasterizer is the only gradient
    # producer here, so the step's first backward overwrites and the others add (lazy zeroing)
    # defer: the per-Gaussian half of the backward runs once for all of the step's views (at
    # finalize / allreduce) instead of once per view (--no-defer: per view)
    bucket = vp.GradBucket(params, lazy_zero=True, defer=not args.no_defer,
                           chunks=args.allreduce_chunks if world > 1 else 1)

    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]

    def view_fn(r, pre=None):
        def run():
            # a fresh screen-space carrier per render, as the reference's render() makes
            # (gaussian_renderer/__init__.py:24); the rasterizer never reads its values (only its
            # .grad is written), so it is not zero-filled; its gradient is not kept here
            m2 = torch.empty_like(params[0], requires_grad=True)
            img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
                       rotations=params[4], prepared=pre)
            img.backward(dpix)
        return run

    view_fns = [view_fn(r) for r in rasts]
    fused_front = not args.no_fused_front and len(rasts) > 1

    def step(sts=streams):
        bucket.zero_grad()
        fns = view_fns
        if fused_front:
            # the step's views' preprocess in one launch (each Gaussian's inputs read once), each
            # view's depth order on its stream; then every view's binning, render and backward
            pre = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4],
                                streams=[sts[k % len(sts)] for k in range(len(rasts))])
            fns = [view_fn(r, p) for r, p in zip(rasts, pre)]
        # this rank's views, round-robin over the streams: gradients accumulate in the bucket
        vp.run_views(fns, sts)
        if world > 1:
            bucket.allreduce()  # one RCCL all-reduce of the 59-f32/Gaussian bucket, in place
        else:
            bucket.finalize()

    # workload counters (one extra forward, untimed)
    e = torch.Tensor([])
    num_rendered, _, radii, geom_b, bin_b, img_b = _C.rasterize_gaussians(
        settings.bg, d.means3D, e, d.opacities, d.scales, d.rotations, 1.0, e, settings.viewmatrix,
        settings.projmatrix, settings.tanfovx, settings.tanfovy, H, W, d.shs, deg, settings.campos, False, False)
    visible = int((radii > 0).sum())
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    # instances the render walks reach: per tile min(largest n_contrib, list length)
    ex = _C.debug_export(P, W, H, num_rendered, geom_b, bin_b, img_b, dev)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ncp = torch.zeros((gy * 16, gx * 16), dtype=torch.int64, device=dev)
    ncp[:H, :W] = ex["n_contrib"].to(torch.int64)
    tmax = ncp.view(gy, 16, gx, 16).amax(dim=(1, 3)).reshape(-1)
    rg = ex["ranges"].to(torch.int64)
    walked = int(torch.minimum(tmax, rg[:, 1] - rg[:, 0]).sum())
    del ex, geom_b, bin_b, img_b

    if args.profile_pass_only:
        # only the kernel-duration pass below (its one-stream step), nothing else on the device
        for _ in range(args.warmup):
            step(streams[:1])
        torch.cuda.synchronize()
        lib = _native.load()
        lib.gs_profile_reset()
        lib.gs_profile_enable(1)
        for _ in range(args.steps):
            step(streams[:1])
        torch.cuda.synchronize()
        lib.gs_profile_enable(0)
        prof = _native.profile_stats()
        if rank == 0:
            print(json.dumps({"profile_pass": {"workload": args.workload, "steps": args.steps, "warmup": args.warmup,
                                               "views_per_step": len(my_views),
                                               "kernels_avg_us": {k: round(1e3 * ms / max(n, 1), 2)
                                                                  for k, (ms, n) in sorted(prof.items())},
                                               "launches": {k: n for k, (ms, n) in sorted(prof.items())}}}))
        return

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    # `regions` timed regions of exactly K steps each, every one bracketed by a barrier and a device
    # sync (max over ranks); `value` is the median region (host-bound configurations such as C2 vary
    # from region to region with the box's host load; every region is reported)
    region_s = []
    for reg in range(max(1, args.regions)):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if args.step_events and reg == 0:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
            evs[0].record()
            for k in range(args.steps):
                step()
                evs[k + 1].record()
        else:
            for _ in range(args.steps):
                step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        region_s.append(el)
    elapsed = sorted(region_s)[len(region_s) // 2]
    peak_hbm = torch.cuda.max_memory_allocated(dev)

    # sustained rate: keep stepping for ~--sustain-s (a longer region than the K timed steps,
    # which last only tens of ms; the same step, reported beside `value`, not instead of it)
    sustained = None
    if args.sustain_s > 0:
        n_s = max(1, int(args.sustain_s / max(elapsed / args.steps, 1e-4)))
        if world > 1:
            nt = torch.tensor([n_s], dtype=torch.int64, device=dev)
            dist.all_reduce(nt, op=dist.ReduceOp.MIN)
            n_s = int(nt.item())
            dist.barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(n_s):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el_s = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([el_s], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_s = float(t.item())
        sustained = dict(steps=n_s, seconds=round(el_s, 3),
                         iters_s=round((n_views or world * len(my_views)) * n_s / el_s, 2))

    # the same step with the views strictly in sequence on one stream (no overlap between views)
    serial = None
    if len(streams) > 1:
        for _ in range(2):
            step(streams[:1])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tq = time.perf_counter()
        for _ in range(args.steps):
            step(streams[:1])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el_q = time.perf_counter() - tq
        if world > 1:
            t = torch.tensor([el_q], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_q = float(t.item())
        serial = dict(iters_s=round((n_views or world * len(my_views)) * args.steps / el_q, 2),
                      ms_per_step=round(1e3 * el_q / args.steps, 4))

    # per-kernel durations: a second pass of the same K steps with HIP events around every launch
    # (on the launch stream); kept out of the timed pass above because the event records add
    # host work and small gaps between kernels.  Views run on one stream here, so a kernel's time
    # is its own (with two streams, kernels of two views share the CUs and each looks slower)
    lib = _native.load()
    lib.gs_profile_reset()
    lib.gs_profile_enable(1)
    for _ in range(args.steps):
        step(streams[:1])
    torch.cuda.synchronize()
    lib.gs_profile_enable(0)
    prof = _native.profile_stats()

    # render-only (no_grad forward) throughput
    with torch.no_grad():
        for _ in range(2):
            rast(means3D=params[0], means2D=means2D, opacities=params[2], shs=params[1], scales=params[3],
                 rotations=params[4])
        torch.cuda.synchronize()
        tr = time.perf_counter()
        nr = max(5, args.steps // 2)
        for _ in range(nr):
            rast(means3D=params[0], means2D=means2D, opacities=params[2], shs=params[1], scales=params[3],
                 rotations=params[4])
        torch.cuda.synchronize()
        t_render = (time.perf_counter() - tr) / nr

        # the same forward in the step's batching: the rank's views per step with the fused front
        # on the step's streams (render throughput as the fwd+bwd metric batches its views)
        render_batched = None
        if len(rasts) > 1 and not args.no_fused_front:
            def render_step():
                pre = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3],
                                    rotations=params[4], streams=[streams[k % len(streams)] for k in range(len(rasts))])
                fns = [(lambda r=r, p=p: r(means3D=params[0], means2D=means2D, opacities=params[2], shs=params[1],
                                           scales=params[3], rotations=params[4], prepared=p))
                       for r, p in zip(rasts, pre)]
                vp.run_views(fns, streams)

            for _ in range(2):
                render_step()
            torch.cuda.synchronize()
            tb = time.perf_counter()
            for _ in range(nr):
                render_step()
            torch.cuda.synchronize()
            t_rb = (time.perf_counter() - tb) / nr / len(rasts)
            render_batched = {"views_per_step": len(rasts), "streams": len(streams),
                              "mpix_s": round(W * H / t_rb / 1e6, 1), "ms_per_view": round(1e3 * t_rb, 4)}

    # batch 1 (train.py's shape, train.py:76-93): one view per step, its whole backward (per-Gaussian
    # half included, written straight into the .grad bucket) before the next view starts, one stream
    single = None
    if args.single_view_steps > 0 and world == 1:
        single = single_view_bench(bucket, rast, params, dpix, args.single_view_steps, lib)

    # the same steps captured into HIP graphs (bounded binning buffers: no host wait in the forward)
    graphs = None
    if world == 1 and not args.no_graph:
        graphs = graph_bench(bucket, rasts, params, dpix, streams, fused_front, step, args.steps,
                             args.single_view_steps, len(my_views))

    ms_per_step = 1e3 * elapsed / args.steps
    # whole-job views (= reference train iterations) per second: weak scaling (C1-C3, C5) counts
    # every rank's views; a C4 step is the 8-view batch
    views_per_step = n_views or world * len(my_views)
    value = views_per_step * args.steps / elapsed

    # per-kernel breakdown + roofline of the dominant kernel
    k_local = len(my_views)
    acc_frac = (k_local - 1) / k_local  # preprocess_bwd launches that add into the bucket
    # views per launch of the sort / binning kernels: with the fused front the library runs the K
    # views' depth sorts (P <= 2M) and binnings (<= 8M instances per view) as one set of launches
    batched = (fused_front and os.environ.get("GSRAST_BATCH_VIEWS", "1") != "0" and P <= (2 << 20)
               and num_rendered <= (8 << 20))
    per_launch_views = {k: (k_local if batched else 1)
                        for k in ("radix_scatter", "radix_hist", "radix_rowscan", "duplicate", "ranges")}

    def kb(name):  # algorithmic bytes of one launch of `name`
        b = kernel_bytes(name, P, visible, num_rendered, M, W, H, tiles, walked, acc_frac, k_local)
        return b * per_launch_views.get(name, 1) if b else b

    kernels = {}
    for name, (ms, n) in prof.items():
        per_launch_ms = ms / max(n, 1)
        b = kb(name)
        kernels[name] = dict(total_ms_per_step=round(ms / args.steps, 4), launches_per_step=round(n / args.steps, 2),
                             avg_us=round(1e3 * per_launch_ms, 2),
                             algo_GBs=(round(b / (per_launch_ms * 1e-3) / 1e9, 1) if b else None))
    dom = max(kernels, key=lambda k: kernels[k]["total_ms_per_step"])
    dom_avg_ms = kernels[dom]["avg_us"] / 1e3
    dom_bytes = kb(dom)
    achieved = dom_bytes / (dom_avg_ms * 1e-3) / 1e9 if dom_bytes else None
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            traffic = json.load(open(pmc_path)).get(args.workload, {}).get(dom)
        except Exception:
            traffic = None
    roofline = dict(bound="hbm", kernel=dom, achieved=round(achieved, 1) if achieved else None, peak=HBM_PEAK_GBS,
                    unit="GB/s", frac=round(achieved / HBM_PEAK_GBS, 4) if achieved else None, traffic=traffic,
                    algo_bytes_per_launch=dom_bytes)
    # the render kernels are VALU-issue bound, not HBM bound: report the issue-rate fraction too,
    # from the committed PMC pass (SQ_INSTS_VALU per launch, device total) and the live duration
    valu_path = os.path.join(ROOT, "profiles", "pmc_valu.json")
    if os.path.exists(valu_path):
        try:
            vi = json.load(open(valu_path)).get(args.workload, {}).get(dom)
        except Exception:
            vi = None
        if vi:
            roofline["valu"] = dict(insts_per_launch=vi, peak_insts_per_s=VALU_PEAK_IPS,
                                    frac=round(vi / (dom_avg_ms * 1e-3) / VALU_PEAK_IPS, 4))
    # whole-step algorithmic bytes (P*a_G + I*a_I + Npix*a_px), per view: every kernel's
    # bytes per launch times its launches per step, over the step's views
    step_bytes = sum((kb(k) or 0)
                     * v["launches_per_step"] for k, v in kernels.items()) / k_local
    ms_per_view = ms_per_step / k_local
    step_roofline = dict(algo_bytes_per_view=int(step_bytes), ms_per_view=round(ms_per_view, 4),
                         achieved=round(step_bytes / (ms_per_view * 1e-3) / 1e9, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                         frac=round(step_bytes / (ms_per_view * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))

    # initialisation kNN (simple_knn distCUDA2 over the scene's P means, as create_from_pcd calls it,
    # scene/gaussian_model.py:134): one timed call after a warm-up
    from simple_knn._C import distCUDA2

    distCUDA2(params[0].detach())
    torch.cuda.synchronize()
    tk = time.perf_counter()
    distCUDA2(params[0].detach())
    torch.cuda.synchronize()
    knn = {"points": P, "ms": round(1e3 * (time.perf_counter() - tk), 3)}

    train = None
    if world == 1 and not args.no_train_step and not n_views:
        train = train_step_bench(sc, cam, deg, dev, args.train_steps, args.workload == "c5")

    vp_train = None
    if args.vp_train_steps > 0:
        try:
            vp_train = vp_train_bench(sc, cams, my_views, deg, dev, args.vp_train_steps, max(2, args.warmup // 3),
                                      world, args.allreduce_chunks)
        except Exception as e:  # a secondary measurement: report its failure in the line, keep the line
            vp_train = {"error": f"{type(e).__name__}: {e}"[:400]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(sc, cam, deg, W, H, dpix.cpu(), args.cpu_threads, args.cpu_runs)

    step_deciles = None
    if args.step_events:
        st_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
        nd = max(1, args.steps // 10)
        step_deciles = [round(sum(st_ms[j:j + nd]) / len(st_ms[j:j + nd]), 4) for j in range(0, args.steps, nd)]
    out = {
        "metric": "train iters/sec (fwd+bwd) + render Mpix/s @1080p, 1M Gaussians SH=3",
        "value": round(value, 2),
        "unit": "iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if (n_views and args.c4_views_per_rank <= 0) else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded; SURVEY.md §8d distribution)",
        "config": {"workload": wl["desc"], "gaussians": P, "sh_degree": deg, "width": W, "height": H,
                   "views_per_rank_per_step": len(my_views), "views_per_step": views_per_step,
                   "render_exp2": "exact-polynomial" if os.environ.get("GSRAST_EXACT_EXP", "0") not in ("", "0")
                   else "hardware v_exp_f32",
                   "parallelism": f"view-parallel dp{world}" +
                   (f" + {'RCCL' if backend == 'nccl' else backend} all-reduce of 59 f32/Gaussian in "
                    f"{bucket.chunks} row chunks overlapped with the per-Gaussian pass" if world > 1 else ""),
                   "backend": backend if world > 1 else None},
        "render_mpix_s": round(W * H / t_render / 1e6, 1),
        "render_ms": round(1e3 * t_render, 4),
        "render_batched": render_batched,
        "single_view": single,
        "graph": graphs,
        "num_rendered": int(num_rendered),
        "walked_instances": walked,
        "visible": visible,
        "hbm": {"peak_allocated_GB": round(peak_hbm / 1e9, 3),
                "scene_params_GB": round(sum(p.numel() for p in params) * 4 / 1e9, 3),
                "geom_buffer_GB": round(lib.gs_geom_buffer_bytes(P) / 1e9, 3),
                "binning_buffer_GB": round(lib.gs_binning_buffer_bytes(int(num_rendered), W, H) / 1e9, 3),
                "image_buffer_GB": round(lib.gs_image_buffer_bytes(W, H) / 1e9, 3),
                "grad_scratch_GB": round(lib.gs_grad_buffer_bytes(int(num_rendered)) / 1e9, 3)},
        "roofline": roofline,
        "ms_per_view": round(ms_per_view, 4),
        "step_roofline": step_roofline,
        "sustained": sustained,
        "regions_iters_s": [round((n_views or world * len(my_views)) * args.steps / r_, 2) for r_ in region_s],
        "streams": len(streams),
        "fused_front": fused_front,
        "serial_one_stream": serial,
        "kernels": kernels,
        # how `kernels` (and single_view's kernel_us_per_iter) are timed: HIP events around each
        # launch on its stream, so a short kernel's figure includes its dispatch gap; the
        # kernel-only durations are rocprofv3's (profiles/*rocprof*.csv, bench.py --profile-pass-only)
        "kernels_timing": "hip events per launch (dispatch gap included)",
        "train_step": train,
        "view_parallel_train": vp_train,
        "init_knn": knn,
        **({"step_ms_deciles": step_deciles} if step_deciles else {}),
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def vp_train_bench(sc, cams, my_views, deg, dev, steps, warmup, world, chunks):
    """View-parallel TRAINING steps: gs_train_step.train_step_views --
    every view of the rank through render -> L1 + SSIM -> backward into the rank's GradBucket
    (fused glue), then the optimizer step over the ranks -- timed per optimizer step, barrier +
    sync on both sides, max over ranks, in three modes:
      sharded:   ShardedAdam(overlap=True): reduce-scatter -> Adam on the rank's rows -> all-gather,
                 in row chunks on a side stream, the all-gathers running into the next step's
                 chunked activation / preprocess (the last step's are waited for inside the region);
      allreduce: one bucket all-reduce (RCCL) + the replicated FusedAdam step;
      local:     the same step without any collective (each rank on its own gradients: the cost of
                 the step with a free exchange).
    exposed_exchange_us = (mode - local) per step.  At N = 1 there is no process group: the three
    modes run the same kernels (sharded = one shard of every row)."""
    import gs_train_step as ts

    settings = [gs_scenes.raster_settings_for(cams[v], deg, device=dev) for v in my_views]
    H, W = settings[0].image_height, settings[0].image_width
    gts = [torch.rand((3, H, W), generator=torch.Generator().manual_seed(100 + v)).to(dev) for v in my_views]
    views = list(zip(settings, gts))
    names = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")

    def timed(mode):
        m = ts.TrainModel(sc, dev)
        bucket = vp.GradBucket([getattr(m, n) for n in names])
        sh = vp.ShardedAdam(m.optimizer, bucket, chunks=chunks, overlap=True) if mode == "sharded" else None

        def one():
            ts.train_step_views(m, bucket, views, sharded=sh, exchange=mode != "local")

        for _ in range(warmup):
            one()
        if sh is not None:
            sh.sync()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            one()
        if sh is not None:
            sh.sync()  # the last step's all-gathers belong to it
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        bucket.close()
        del m, bucket, sh
        torch.cuda.empty_cache()
        return el

    els = {mode: timed(mode) for mode in ("local", "allreduce", "sharded")}
    nv = world * len(views)
    out = {"views_per_rank_per_step": len(views), "steps": steps, "chunks": chunks,
           "glue": "fused (render_inputs activation, photometric_loss, densify stats, FusedAdam)"}
    for mode, el in els.items():
        out[mode] = {"iters_s": round(nv * steps / el, 2), "ms_per_step": round(1e3 * el / steps, 4)}
        if mode != "local":
            out[mode]["exposed_exchange_us"] = round(1e6 * (el - els["local"]) / steps, 1)
    return out


def single_view_bench(bucket, rast, params, dpix, steps, lib):
    """Batch-1 rasterizer iterations: zero_grad, one view's forward, its full backward into the
    gradient bucket (no deferral: the per-Gaussian half runs inside the view's backward), finalize;
    everything on the current stream.  Returns the rate and a per-kernel breakdown (HIP events on the
    launch stream, a second pass)."""
    defers = bucket.defers
    bucket.defers = False

    def sv_step():
        bucket.zero_grad()
        m2 = torch.empty_like(params[0], requires_grad=True)  # values never read (gradient carrier)
        img, _ = rast(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
                      rotations=params[4])
        img.backward(dpix)
        bucket.finalize()

    try:
        for _ in range(5):
            sv_step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            sv_step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / steps
        lib.gs_profile_reset()
        lib.gs_profile_enable(1)
        for _ in range(steps):
            sv_step()
        torch.cuda.synchronize()
        lib.gs_profile_enable(0)
        prof = _native.profile_stats()
    finally:
        bucket.defers = defers
    kern = {k: round(1e3 * ms / steps, 2) for k, (ms, n) in sorted(prof.items(), key=lambda kv: -kv[1][0])}
    return {"what": "one view per step (train.py's batch 1): forward, full backward into the .grad bucket, one "
                    "stream, no deferral, no overlap between views",
            "iters_s": round(1.0 / dt, 2), "ms_per_iter": round(1e3 * dt, 4), "steps": steps,
            "kernel_us_per_iter": kern, "kernel_us_sum": round(sum(kern.values()), 1)}


def graph_bench(bucket, rasts, params, dpix, streams, fused_front, eager_step, steps, sv_steps, k_views,
                headroom=1.10):
    """The timed step and the batch-1 step, each captured once into a HIP graph
    (torch.cuda.CUDAGraph) and replayed.  Their forwards are bounded (binning_capacity = each
    view's measured instance count x `headroom`): nothing in the step waits on the host, so the
    whole step -- fused front, both streams, backwards, deferred per-Gaussian pass -- is one graph
    launch.  The replays are checked bit for bit against the eager step, and the bounded status
    (no view over its capacity) after the timed replays."""
    from diff_gaussian_rasterization import bounded_status

    # instance counts of the step's views (eager, read back) -> capacities
    pre = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4])
    caps = [int(p.triple[0] * headroom) + 4096 for p in pre]
    del pre
    bounded_status()

    def run_graph(fn, n_rep, ref_fn):
        ref_fn()  # the eager (read-back) step: the reference bucket
        torch.cuda.synchronize()
        ref = bucket.flat.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        bucket.flat.zero_()
        g.replay()
        torch.cuda.synchronize()
        same = bool(torch.equal(bucket.flat, ref))
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n_rep):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / n_rep
        del g
        return dt, same

    def step_bounded():
        bucket.zero_grad()
        if fused_front:
            pv = prepare_views(rasts, params[0], params[2], shs=params[1], scales=params[3], rotations=params[4],
                               streams=[streams[k % len(streams)] for k in range(len(rasts))], binning_capacity=caps)
            fns = [(lambda r=r, p=p: _view_bwd(r, params, dpix, prepared=p)) for r, p in zip(rasts, pv)]
        else:
            fns = [(lambda r=r, c=c: _view_bwd(r, params, dpix, cap=c)) for r, c in zip(rasts, caps)]
        vp.run_views(fns, streams)
        bucket.finalize()

    out = {"what": "the timed step and the batch-1 step as HIP graphs: bounded binning buffers (measured "
                   f"instances x {headroom} + 4096), captured once, replayed",
           "capacities": caps}
    dt, same = run_graph(step_bounded, steps, eager_step)
    out["step"] = {"iters_s": round(k_views / dt, 2), "ms_per_step": round(1e3 * dt, 4), "bitwise_equal_eager": same}
    if sv_steps > 0:
        defers = bucket.defers
        bucket.defers = False

        def sv(cap):
            bucket.zero_grad()
            _view_bwd(rasts[0], params, dpix, cap=cap)
            bucket.finalize()

        try:
            dt1, same1 = run_graph(lambda: sv(caps[0]), sv_steps, lambda: sv(None))
        finally:
            bucket.defers = defers
        out["single_view"] = {"iters_s": round(1.0 / dt1, 2), "ms_per_iter": round(1e3 * dt1, 4),
                              "bitwise_equal_eager": same1}
    try:
        bounded_status()
        out["capacity_exceeded"] = False
    except RuntimeError as e:  # a view outgrew its capacity: the replays' results are invalid
        out["capacity_exceeded"] = str(e)
    return out


def _view_bwd(r, params, dpix, prepared=None, cap=None):
    m2 = torch.empty_like(params[0], requires_grad=True)
    img, _ = r(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
               rotations=params[4], prepared=prepared, binning_capacity=cap)
    img.backward(dpix)


def train_step_bench(sc, cam, deg, dev, steps, densify):
    """SURVEY §8d metric (2): one full train.py iteration per step (gs_train_step.train_step:
    render -> L1 + SSIM -> backward -> densification statistics -> Adam -> zero_grad) on the same
    scene and view against a seeded synthetic target image, with the fused glue and with the
    reference's torch glue (activations, statistics, Adam); the rasterizer and the loss are the
    HIP ones in both.  With `densify` (C5): then one densify_and_prune on synthetic statistics
    (5 % over the threshold, extent 2: clones and splits), and the peak HBM over the train steps
    and the densify step."""
    import gs_train_step as ts

    W, H = cam.image_width, cam.image_height
    settings = gs_scenes.raster_settings_for(cam, deg, device=dev)
    gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(2)).to(dev)
    out = {"what": "train.py:86-128 per iteration (one view): render, L1+SSIM (lambda 0.2), backward, "
                   "densification stats, Adam step, zero_grad; `fused` / `torch_glue` without the per-iteration "
                   "loss.item() readback of train.py:99, `fused_item` with it (as unmodified train.py runs)"}
    # train.py's own loop shape: the loss read back every iteration (host waits for the iteration)
    model = ts.TrainModel(sc, dev, fused=True)
    for _ in range(3):
        ts.train_step(model, settings, gt, fused=True, loss_item=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        ts.train_step(model, settings, gt, fused=True, loss_item=True)
    dt = (time.perf_counter() - t) / steps
    out["fused_item"] = {"iters_s": round(1.0 / dt, 2), "ms_per_iter": round(1e3 * dt, 4)}
    del model
    # the same loop with the per-Gaussian backward fused into the Adam step (train_step(fuse_adam=True),
    # gs_backward_gaussians_adam): bit-identical parameters and moments, no stored gradients
    model = ts.TrainModel(sc, dev, fused=True)
    for _ in range(3):
        ts.train_step(model, settings, gt, fused=True, loss_item=True, fuse_adam=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        ts.train_step(model, settings, gt, fused=True, loss_item=True, fuse_adam=True)
    dt = (time.perf_counter() - t) / steps
    out["fused_adam_item"] = {"iters_s": round(1.0 / dt, 2), "ms_per_iter": round(1e3 * dt, 4)}
    del model
    for fused in (True, False):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(dev)
        base = torch.cuda.memory_allocated(dev)
        model = ts.TrainModel(sc, dev, fused=fused)
        for _ in range(3):
            ts.train_step(model, settings, gt, fused=fused)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            ts.train_step(model, settings, gt, fused=fused)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / steps
        key = "fused" if fused else "torch_glue"
        out[key] = {"iters_s": round(1.0 / dt, 2), "ms_per_iter": round(1e3 * dt, 4),
                    "peak_GB": round((torch.cuda.max_memory_allocated(dev) - base) / 1e9, 3)}
        if densify and fused:
            P0 = model.P
            ts.synthetic_densify_stats(model, frac=0.05, seed=3)
            torch.cuda.synchronize()
            t = time.perf_counter()
            ts.densify(model, extent=2.0)
            torch.cuda.synchronize()
            out["densify"] = {"ms": round(1e3 * (time.perf_counter() - t), 3), "P_before": P0, "P_after": model.P,
                              "peak_GB_over_train_steps_and_densify":
                                  round((torch.cuda.max_memory_allocated(dev) - base) / 1e9, 3),
                              "extent": 2.0, "grad_threshold": ts.DENSIFY_GRAD_THRESHOLD}
            # one more iteration at the new size (the densified model trains on)
            ts.train_step(model, settings, gt, fused=True)
            torch.cuda.synchronize()
            out["densify"]["peak_GB_incl_next_iteration"] = round(
                (torch.cuda.max_memory_allocated(dev) - base) / 1e9, 3)
        del model
    return out


def job_cpus():
    """CPUs this job may use: the affinity mask, capped by a cgroup v2 CPU quota and by
    OMP_NUM_THREADS when the launcher sets it (the GPU box allots each job a share of the host:
    os.cpu_count() there shows the whole machine).  Returns (n, how)."""
    n = len(os.sched_getaffinity(0))
    how = [f"affinity {n}"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n_q = max(1, int(int(q) / int(per)))
            how.append(f"cgroup quota {n_q}")
            n = min(n, n_q)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        how.append(f"OMP_NUM_THREADS {omp}")
        n = min(n, int(omp))
    return n, ", ".join(how)


def cpu_model():
    try:
        import subprocess

        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline(sc, cam, deg, W, H, dpix, threads, runs):
    """CPU oracle (oracle/gs_oracle.c: this repo's C restatement of the algorithm; the reference has
    no CPU rasterizer) timed on the host for full fwd+bwd steps of the same workload: one warm-up,
    then the median of `runs` (BASELINE.md §2 protocol), on every CPU the job may use."""
    import numpy as np

    from oracle import gs_oracle

    gs_oracle.build()
    n, how = (threads, "--cpu-threads") if threads else job_cpus()
    gs_oracle.set_threads(n)
    osc = gs_oracle.Scene(bg=np.zeros(3, np.float32), means3D=sc.means3D.numpy(), opacities=sc.opacities.numpy(),
                          W=W, H=H, viewmatrix=cam.world_view_transform.numpy(),
                          projmatrix=cam.full_proj_transform.numpy(), campos=cam.camera_center.numpy(),
                          tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2), shs=sc.shs.numpy(),
                          sh_degree=deg, scales=sc.scales.numpy(), rotations=sc.rotations.numpy())
    times = []
    for r in range(1 + max(1, runs)):
        t = time.perf_counter()
        gs_oracle.forward(osc)
        gs_oracle.backward(osc, dpix.numpy())
        if r > 0:  # run 0 is the warm-up
            times.append(time.perf_counter() - t)
    dt = sorted(times)[len(times) // 2]
    return {"value": round(1.0 / dt, 5), "unit": "iters/s", "cores": n, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "cores_from": how,
            "runs_s": [round(x, 3) for x in times],
            "sample": f"full fwd+bwd steps of the same workload ({sc.P} Gaussians, {W}x{H}): one warm-up, median "
                      f"of {len(times)} runs = {dt:.2f} s on {n} threads"}


if __name__ == "__main__":
    main()
