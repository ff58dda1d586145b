"""View-parallel data parallelism for 3DGS training on one node.

The reference trains single-view SGD on one GPU (/root/reference/train.py:76-78, no
torch.distributed anywhere).  Views are independent given replicated Gaussians, so the
north-star scaling axis is: rank r renders views {v : v mod N == r}, every rank keeps a full
replica of the parameters and optimizer state, and the only exchange is ONE all-reduce of the
parameter gradients per optimizer step (RCCL over xGMI: torch.distributed backend "nccl").

Gradients of the six parameter groups of GaussianModel (/root/reference/scene/gaussian_model.py:
154-161: xyz 3, f_dc 3, f_rest 45, opacity 1, scaling 3, rotation 4 = 59 fp32 per Gaussian) go
through one flat bucket so the collective is a single large message (ring all-reduce is per-link
bandwidth bound on point-to-point xGMI; one 236 MB message at 1M Gaussians, not six).
Densification statistics are reduced only when densification runs (every 100 iterations,
train.py:118-121): gradient accumulators and denominators are summed, max_radii2D max-reduced.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist


def shard_views(num_views: int, rank: int, world: int) -> List[int]:
    """Views owned by `rank`: round-robin (v mod world == rank)."""
    return [v for v in range(num_views) if v % world == rank]


class GradBucket:
    """One flat fp32 buffer holding the gradients of `params` for a single all-reduce."""

    def __init__(self, params: Sequence[torch.Tensor]):
        self.params = list(params)
        self.numel = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.empty((self.numel,), dtype=torch.float32, device=dev)

    def _resize_if_needed(self):
        n = sum(p.numel() for p in self.params)
        if n != self.numel:  # densification changed P
            self.numel = n
            self.flat = torch.empty((n,), dtype=torch.float32, device=self.flat.device)

    def pack(self) -> torch.Tensor:
        self._resize_if_needed()
        grads = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in self.params]
        torch.cat(grads, out=self.flat)
        return self.flat

    def unpack(self):
        off = 0
        for p in self.params:
            n = p.numel()
            g = self.flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += n

    def allreduce(self, group=None, average: bool = False, unpack: bool = True):
        """Sum (or mean) the gradients across the process group in one collective.  With
        unpack=False the reduced gradients stay in `self.flat` (for an optimizer that steps on the
        flat buffer) and the per-parameter .grad tensors are left as they were."""
        flat = self.pack()
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
            if average:
                flat.div_(dist.get_world_size(group))
        if unpack:
            self.unpack()
        return flat


def allreduce_grads(params: Iterable[torch.Tensor], group=None, average: bool = False):
    GradBucket(list(params)).allreduce(group=group, average=average)


def reduce_densify_stats(xyz_gradient_accum: torch.Tensor, denom: torch.Tensor, max_radii2D: torch.Tensor,
                         group=None):
    """Combine the per-rank densification statistics (gaussian_model.py:405-407, train.py:115)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    dist.all_reduce(xyz_gradient_accum, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(denom, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX, group=group)


def init_from_env(backend: Optional[str] = None):
    """torchrun-style init (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or dist.is_initialized():
        return
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
