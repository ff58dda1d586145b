"""Worker of tests/test_gpu_multiview.py::test_two_rank_view_parallel_matches_single_process_sum
(launched by torchrun, 2 ranks; gloo, both ranks on cuda:0).

Each rank renders its share of the 8 C4 ring views (v = rank mod 2) through the
HIP rasterizer into a GradBucket, the bucket is all-reduced once, and rank 0 compares it with all 8
views rendered into one bucket by a single process.  Writes "OK ..." or "FAIL ..." to $GS_VP_OUT.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-skysphere_amd"), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import gs_scenes  # noqa: E402
import gs_view_parallel as vp  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402

N_VIEWS, P, W, H = 8, 1_000_000, 1920, 1080
NAMES = ("means3D", "shs", "opacities", "scales", "rotations")


def render_views(d, cams, views, dev, chunks=1):
    params = [d.means3D.clone().requires_grad_(True), d.shs.clone().requires_grad_(True),
              d.opacities.clone().requires_grad_(True), d.scales.clone().requires_grad_(True),
              d.rotations.clone().requires_grad_(True)]
    bucket = vp.GradBucket(params, lazy_zero=True, defer=True, chunks=chunks)
    bucket.zero_grad()
    for v in views:
        rast = GaussianRasterizer(gs_scenes.raster_settings_for(cams[v], 3, device=dev))
        m2 = torch.zeros_like(params[0], requires_grad=True)
        img, _ = rast(means3D=params[0], means2D=m2, opacities=params[2], shs=params[1], scales=params[3],
                      rotations=params[4])
        img.backward(gs_scenes.dl_dimage(H, W, seed=100 + v).to(dev))
    return params, bucket


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cams = gs_scenes.circle_cameras(N_VIEWS, 6.0, W, H)
    d = gs_scenes.random_gaussians(P, 3, seed=0, ball_radius=2.0).to(dev)
    mine = vp.shard_views(N_VIEWS, rank, world)
    # the chunked all-reduce (per-Gaussian pass in 3 row ranges, each range's rows all-reduced as
    # soon as they are written) must give the one-shot bucket's sums bit for bit
    c_params, c_bucket = render_views(d, cams, mine, dev, chunks=3)
    c_bucket.allreduce()
    torch.cuda.synchronize()
    chunk_flat = c_bucket.flat.clone()
    c_bucket.close()
    del c_params, c_bucket
    params, bucket = render_views(d, cams, mine, dev)
    ptrs = [p.grad.data_ptr() for p in params]
    bucket.allreduce()
    torch.cuda.synchronize()
    chunked_equal = bool(torch.equal(chunk_flat, bucket.flat))
    msg = None
    if rank == 0:
        assert ptrs == [p.grad.data_ptr() for p in params]
        ref_params, ref_bucket = render_views(d, cams, range(N_VIEWS), dev)
        ref_bucket.finalize()
        torch.cuda.synchronize()
        lines = []
        ok = True
        for name, p, q in zip(NAMES, params, ref_params):
            got, ref = p.grad.double(), q.grad.double()
            scale = float(ref.abs().max())
            bad = (got - ref).abs() > 1e-5 * ref.abs() + 1e-5 * scale
            nbad = int(bad.sum())
            ok = ok and nbad == 0 and scale > 0 and chunked_equal
            lines.append(f"{name}: max|ref| {scale:.3e} max|d| {float((got - ref).abs().max()):.3e} beyond tol {nbad}")
        msg = ("OK " if ok else "FAIL ") + f"views/rank {len(mine)}; chunked all-reduce equal {chunked_equal}; " + \
            "; ".join(lines)
        with open(os.environ["GS_VP_OUT"], "w") as f:
            f.write(msg + "\n")
    dist.barrier()
    bucket.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
