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

import ctypes
from typing import Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist


def shard_views(num_views: int, rank: int, world: int) -> List[int]:
    """Views owned by `rank`: round-robin (v mod world == rank)."""
    return [v for v in range(num_views) if v % world == rank]


class GradBucket:
    """One flat fp32 buffer that IS the gradient storage of `params`: every `p.grad` is a view
    into it, so the all-reduce runs over the .grad tensors themselves (no pack / unpack copy).

    The rasterizer writes its gradients straight into those views through the gradient sink of
    diff_gaussian_rasterization (gs_backward_accumulate): the first view of a step overwrites,
    later views add in the same kernel, exactly as autograd's `grad += g` would, with no extra
    pass.  Other autograd producers accumulate into the views as usual.

    lazy_zero=True (the rasterizer is the only gradient producer, as in the reference loop where
    the loss reaches the parameters only through render(); bench.py): zero_grad() writes nothing,
    the step's first rasterizer write overwrites, and views no backward wrote are zeroed before
    the all-reduce.  An in-place write by any other op into a not-yet-written view raises (it
    would have added to the previous step's values).  lazy_zero=False: zero_grad() zero-fills
    the bucket (one memset) and every write accumulates.
    """

    def __init__(self, params: Sequence[torch.Tensor], lazy_zero: bool = False, defer: bool = False,
                 chunks: int = 1):
        self.lazy_zero = lazy_zero
        # chunks > 1 (with defer): allreduce() runs the deferred per-Gaussian pass in `chunks`
        # Gaussian-row ranges and starts each range's all-reduce (its rows of every parameter) on a
        # side stream as soon as that range is written, so the collective overlaps the pass
        self.chunks = max(1, int(chunks))
        self._comm = None
        # defer=True: a rasterizer backward whose parameter gradients all come here runs only its
        # per-tile half; the per-Gaussian half of all such views runs in ONE pass at finalize() /
        # allreduce() (gs_backward_gaussians): every Gaussian's inputs are read and its gradient
        # row written once per step instead of once per view.  Same fp32 sums as without.
        self.defers = defer
        self._deferred = []
        self._ev_pool = []  # recorded-and-waited events of retired deferred views, reused by defer_view
        # stream ordering of the writes into the bucket: the last writer's event and stream (views
        # rendered on several streams add into one bucket one after another; their forward passes,
        # sorts and tile backward passes overlap)
        self._events = {}
        self._last = None
        # (event, stream, zeroed): the previous step's gradient reads on another stream (ShardedAdam
        # with overlap: its reduce-scatters, and with zeroed the zero-fill of the rows it consumed)
        self._foreign = None
        self._zero_wait = None
        self.params = []
        self._bind(list(params))

    def _bind(self, params):
        from diff_gaussian_rasterization import register_gradient_sink

        self._hooks = []
        for p in params:
            if p.dtype != torch.float32:
                raise TypeError("GradBucket: float32 parameters only")
        self.params = params
        self.numel = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros((self.numel,), dtype=torch.float32, device=dev)
        self.views = {}
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
            p.grad = v
            self.views[id(p)] = v
            register_gradient_sink(p, self)
            self._hooks.append(p.register_hook(self._grad_hook))
        self._fresh = {}  # id(p) -> _version of the view at zero_grad (lazy mode: not written yet)
        self.zero_grad()

    def rebind(self, params: Sequence[torch.Tensor]) -> None:
        """Make the bucket the gradient storage of `params` instead (e.g. the new nn.Parameters that
        densify_and_prune swaps in, with a new Gaussian count): a new flat buffer of the new size,
        every new .grad a view of it, the old parameters' sinks closed.  gs_train.densify_and_prune
        calls this for the bucket that owns the replaced parameters."""
        if self._deferred:
            raise RuntimeError("GradBucket.rebind: deferred views are pending (finalize / allreduce the step first)")
        old = self.params
        self.close()
        for p in old:
            if p.grad is self.views.get(id(p)):
                p.grad = None  # the old tensors keep no view of the old buffer
        self._events, self._last = {}, None
        self._bind(list(params))

    def close(self):
        from diff_gaussian_rasterization import unregister_gradient_sink

        for p in self.params:
            unregister_gradient_sink(p)
        for h in getattr(self, "_hooks", []):
            h.remove()
        self._hooks = []

    def _grad_hook(self, grad):
        """A gradient about to be accumulated into a bucket view by autograd (outside the sink
        protocol): its stream waits for a foreign zero-fill of the bucket first (after_foreign_read),
        so no backward can race it even without before_backward()."""
        ev = self._zero_wait
        if ev is not None and grad is not None and grad.is_cuda:
            torch.cuda.current_stream(grad.device).wait_event(ev)
        return None

    def _check_bound(self):
        """Every parameter's .grad must be its bucket view.  optimizer.zero_grad(set_to_none=True)
        (train.py:128) drops it: it is re-attached here.  Any other tensor in .grad means the
        gradients would bypass the all-reduce: raise."""
        for p in self.params:
            v = self.views[id(p)]
            if p.grad is None:
                p.grad = v
            elif p.grad is not v:
                raise RuntimeError("GradBucket: a parameter's .grad was replaced by another tensor; its gradient "
                                   "would bypass the bucket (call rebind() after replacing parameters)")

    def after_foreign_read(self, event, stream, zeroed: bool) -> None:
        """The step's gradients were read on `stream` (up to `event`), and with `zeroed` the bucket
        was zero-filled there afterwards (ShardedAdam(overlap=True)): the next zero_grad() then
        writes nothing and makes no stream wait, and the next step's writers wait for `event` --
        the rasterizer's sink writes through write_order, any other producer through
        before_backward() (gs_train_step.train_step_views calls it before each loss.backward())."""
        self._foreign = (event, stream, bool(zeroed))

    def before_backward(self) -> None:
        """Before a backward whose gradients reach the bucket outside the sink protocol (autograd's
        accumulation into the .grad views): the current stream waits for a foreign zero-fill now
        (the parameters' gradient hooks also wait for it, on the accumulating stream)."""
        ev = self._zero_wait
        if ev is not None and self.flat.is_cuda:
            torch.cuda.current_stream(self.flat.device).wait_event(ev)

    def zero_grad(self):
        self._check_bound()
        self._zero_wait = None
        foreign, self._foreign = self._foreign, None
        if foreign is not None:
            ev, st, zeroed = foreign
            if self.lazy_zero:
                self._fresh = {id(p): self.views[id(p)]._version for p in self.params}
            elif zeroed:
                self._fresh = {}
                self._zero_wait = ev
            else:
                torch.cuda.current_stream(self.flat.device).wait_event(ev)
                self.flat.zero_()
                self._fresh = {}
                self.written(torch.cuda.current_stream(self.flat.device))
                return
            self._last = (ev, st)  # the step's first sink write (on any stream) waits for the reads
            return
        if self.lazy_zero:
            self._fresh = {id(p): self.views[id(p)]._version for p in self.params}
        else:
            self.flat.zero_()
            self._fresh = {}
        # the step's first write, on whichever stream, follows everything queued on this one
        # (the previous step's all-reduce / optimizer reads, or the zero fill)
        if self.flat.is_cuda:
            self.written(torch.cuda.current_stream(self.flat.device))

    def write_order(self, stream):
        """Event a write on `stream` must wait for (the previous write was on another stream)."""
        if self._last is None or self._last[1] == stream:
            return None
        return self._last[0]

    def written(self, stream):
        """A write into the bucket was enqueued on `stream`: later writers on other streams wait for it."""
        ev = self._events.get(stream)
        if ev is None:
            ev = self._events[stream] = torch.cuda.Event()
        ev.record(stream)
        self._last = (ev, stream)

    def _join(self):
        # reads of the bucket on the current stream follow the last write on any stream
        if self.flat.is_cuda and self._last is not None:
            cur = torch.cuda.current_stream(self.flat.device)
            if self._last[1] != cur:
                cur.wait_event(self._last[0])

    def claim(self, p):
        """Gradient sink protocol: (buffer, accumulate) for the rasterizer backward."""
        v = self.views.get(id(p))
        if v is None or p.grad is not v:
            return None  # .grad was replaced by the user: plain autograd
        ver = self._fresh.pop(id(p), None)
        if ver is None:
            return v, True
        if v._version != ver:
            raise RuntimeError("GradBucket(lazy_zero=True): another op accumulated into a gradient view before the "
                               "rasterizer's first write of the step; use lazy_zero=False")
        return v, False

    # ---- deferred per-Gaussian backward (defer=True) ----
    def defer_view(self, ctx, inputs, view):
        """Rasterizer protocol: take one view's per-Gaussian backward (its per-tile half and record
        sums are enqueued on the current stream).  inputs: the Gaussian tensors of the call;
        view: (viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, W, H, geomBuffer)."""
        if self._deferred and not _same_inputs(self._deferred[0][0], inputs):
            self.flush()  # another set of Gaussians: finish the pending views first
        st = torch.cuda.current_stream(view[7].device)
        ev = self._ev_pool.pop() if self._ev_pool else torch.cuda.Event()
        ev.record(st)
        sunk = [(name, t) for k, name, t, o in ctx.sinks if o is self and ctx.needs_input_grad[k] and k != 1]
        self._deferred.append((inputs, view, ev, sunk))

    def _claim_deferred(self):
        """Join the pending views' streams and claim the outputs of their per-Gaussian pass:
        (inputs, views, outs, accumulate bits)."""
        from diff_gaussian_rasterization import _C

        inputs = self._deferred[0][0]
        cur = torch.cuda.current_stream(self.flat.device)
        for _, _, ev, _ in self._deferred:
            cur.wait_event(ev)
        self._join()
        outs, acc = {}, 0
        for name, t in self._deferred[0][3]:
            claim = self.claim(t)
            if claim is None:
                raise RuntimeError(f"GradBucket(defer=True): the .grad of the {name} input was replaced before "
                                   "the deferred backward ran")
            outs[name], accumulate = claim
            acc |= _C.GS_ACC[name] if accumulate else 0
        return inputs, [d[1] for d in self._deferred], outs, acc

    def _deferred_pass(self, inputs, views, outs, acc, first=0, count=None):
        from diff_gaussian_rasterization import _C

        _C.backward_gaussians(inputs["means3D"], inputs["sh"], inputs["colors"], inputs["scales"],
                              inputs["rotations"], inputs["cov3D"], inputs["scale_modifier"], inputs["degree"],
                              views, outs, acc, debug=inputs["debug"], first=first, count=count)

    def _retire_deferred(self, inputs, views):
        # the views' buffers were allocated on their own streams: keep them out of reuse there until
        # this stream's pass is done
        cur = torch.cuda.current_stream(self.flat.device)
        for v in views:
            for t in (v[0], v[1], v[2], v[7]):
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(cur)
        for t in inputs.values():
            if isinstance(t, torch.Tensor) and t.is_cuda and t.numel():
                t.record_stream(cur)
        self.written(cur)
        # the views' events are waited on (enqueued) already: free to record again
        self._ev_pool += [d[2] for d in self._deferred]
        self._deferred = []

    def flush(self):
        """Run the pending views' per-Gaussian backward in one pass on the current stream."""
        if not self._deferred:
            return
        inputs, views, outs, acc = self._claim_deferred()
        self._deferred_pass(inputs, views, outs, acc)
        self._retire_deferred(inputs, views)

    def _zero_unwritten(self):
        for p in self.params:
            ver = self._fresh.pop(id(p), None)
            if ver is not None:
                v = self.views[id(p)]
                if v._version != ver:
                    raise RuntimeError("GradBucket(lazy_zero=True): a gradient view was accumulated into without "
                                       "a rasterizer write in the step")
                v.zero_()

    def finalize(self):
        """Run any deferred per-Gaussian backward, zero the views no backward wrote this step (lazy
        mode); then the bucket holds the step's gradient sums (on the current stream: it waits for
        the last write on any stream)."""
        self._check_bound()
        self.flush()
        self._join()
        self._zero_unwritten()
        return self.flat

    def _chunk_rows(self):
        """Gaussian-row count of the chunked all-reduce, or None (every parameter must have the
        deferred inputs' row count)."""
        if self.chunks <= 1 or not self._deferred or not (dist.is_available() and dist.is_initialized()):
            return None
        P = self._deferred[0][0]["means3D"].shape[0]
        if P < self.chunks or any(p.dim() == 0 or p.shape[0] != P for p in self.params):
            return None
        return P

    def _allreduce_chunked(self, P, group):
        """The deferred per-Gaussian pass in self.chunks row ranges on the current stream; after each
        range, its rows of every parameter gradient are all-reduced on a side stream (one coalesced
        group with RCCL), so the collectives overlap the remaining ranges' pass.  The current stream
        then waits for every collective."""
        self._check_bound()
        inputs, views, outs, acc = self._claim_deferred()
        self._zero_unwritten()  # views no backward writes this step, before any collective reads them
        cur = torch.cuda.current_stream(self.flat.device)
        if self._comm is None:
            self._comm = torch.cuda.Stream(self.flat.device)
        comm = self._comm
        coalesce = dist.get_backend(group) == "nccl"
        bounds = [P * c // self.chunks for c in range(self.chunks + 1)]
        works = []
        for c in range(self.chunks):
            b, e = bounds[c], bounds[c + 1]
            self._deferred_pass(inputs, views, outs, acc, first=b, count=e - b)
            ev = torch.cuda.Event()
            ev.record(cur)
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                rows = [p.grad[b:e] for p in self.params]
                if coalesce:
                    with dist._coalescing_manager(group, device=self.flat.device, async_ops=True) as cm:
                        for t in rows:
                            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
                    works.append(cm)
                else:
                    works += [dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True) for t in rows]
        self._retire_deferred(inputs, views)
        for w in works:
            w.wait()  # the current stream waits for the collective
        cur.wait_stream(comm)
        self.written(cur)

    def allreduce(self, group=None, average: bool = False, async_op: bool = False):
        """Sum (or mean) the gradients across the process group in ONE collective over the flat
        bucket; the .grad views hold the result afterwards.  With a process group the collective is
        issued at every world size (world 1: RCCL's in-place copy), so one code path runs at N = 1..8.
        With chunks > 1 and a deferred pass pending, the all-reduce runs in row chunks overlapped with
        that pass (same sums: every element is reduced once, in the same rank order)."""
        P = self._chunk_rows()
        if P is not None:
            self._allreduce_chunked(P, group)
            if average:
                self.flat.div_(dist.get_world_size(group))
            return None if async_op else self.flat
        flat = self.finalize()
        work = None
        if dist.is_available() and dist.is_initialized():
            work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
            if average:
                if async_op:
                    work.wait()
                    work = None
                flat.div_(dist.get_world_size(group))
        return work if async_op else flat


class ShardedAdam:
    """The optimizer step of view-parallel training as reduce-scatter -> sharded Adam -> all-gather
    (ZeRO-1 style) instead of all-reduce -> replicated Adam, in Gaussian-row chunks.

    Rows [0, Pm) (Pm = P rounded down to a multiple of the world size N) are cut into `chunks` row
    ranges whose sizes are multiples of N; in chunk c every rank owns an equal slice of S_c rows.  Per
    chunk, for every parameter of the bucket: the gradient rows are reduce-scattered (each rank gets
    the summed rows of its slice), the rank runs the Adam update on its slice only (FusedAdam's
    kernel, the parameter's own lr / step / moments), and the updated rows are all-gathered in place
    into every replica.  The < N tail rows [Pm, P) are all-reduced and updated by every rank.  With a
    deferred per-Gaussian backward pending (GradBucket(defer=True)), chunk c's pass runs on the
    current stream while chunk c-1's collectives and update run on a side stream.

    Same values as GradBucket.allreduce + FusedAdam.step: every element is the same sum of the ranks'
    gradients (bit-identical at N = 2, where a sum of two is one rounding in any order; at N > 2 the
    ring's association may differ from the all-reduce's) and the same Adam arithmetic.  The moment
    tensors in optimizer.state stay full-size, but only the rows a rank owns are current:
    gather_state() all-gathers them, and must run before anything reads whole moments (densify_and_prune,
    state_dict); the row plan follows P afterwards.  Bytes on the wire per step equal the all-reduce's
    (an all-reduce IS a reduce-scatter + an all-gather); the Adam work per rank is 1/N of it."""

    def __init__(self, optimizer, bucket: GradBucket, group=None, chunks: int = 4, update=None,
                 overlap: bool = False):
        self.opt, self.bucket, self.group = optimizer, bucket, group
        self.chunks = max(1, int(chunks))
        self._update = update  # (items, b1, b2, eps, maximize) -> None; default: FusedAdam's HIP kernel
        self._comm = None
        self._bufs = {}
        # overlap: step() returns with its all-gathers in flight; their per-chunk events wait for
        # the next step's consumers (take_row_waits -> the forward's chunked activation and
        # preprocess), and the bucket is zero-filled on the collective stream
        self.overlap = bool(overlap)
        self._pending = []
        # the Gaussian count of the step that left every rank's moments current only on its own rows
        # (None: whole on every rank).  gather_state() clears it; a step at another count, a densify
        # or a state_dict() in between raise instead of reading stale moment rows.
        self._sharded_P = None
        self.opt._gs_sharded_moments = self
        if hasattr(self.opt, "register_state_dict_pre_hook"):
            self.opt.register_state_dict_pre_hook(lambda opt: self._check_whole("state_dict()"))

    def moments_sharded(self) -> bool:
        """True when the moments are current only on each rank's own rows (call gather_state())."""
        return self._sharded_P is not None

    def _check_whole(self, what: str) -> None:
        if self._sharded_P is not None:
            raise RuntimeError(f"ShardedAdam: {what} needs whole Adam moments, but each rank holds only its own rows "
                               "since the last step: call gather_state() first")

    def take_row_waits(self):
        """[(lo, hi, event)] of the last overlapped step's all-gathers (rows [lo, hi) of every
        parameter are whole once `event` has fired), handed to the next forward (gs_train_step.
        render(row_waits=...)), which then waits for them chunk by chunk; cleared here, so the caller
        owns the waits.  Empty when nothing is pending."""
        out, self._pending = self._pending, []
        return out

    def sync(self) -> None:
        """The current stream waits for every pending all-gather (before anything reads the
        parameters outside a row-waited forward)."""
        pend, self._pending = self._pending, []
        if pend and self.bucket.flat.is_cuda:
            cur = torch.cuda.current_stream(self.bucket.flat.device)
            for _lo, _hi, ev in pend:
                cur.wait_event(ev)

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    def plan(self, P: int):
        """[(b, e, S)]: the chunks' row ranges over [0, Pm) (e - b == N S) and Pm."""
        N, _ = self._world()
        Pm = (P // N) * N
        units = Pm // N
        C = max(1, min(self.chunks, units))
        cuts = [N * (units * c // C) for c in range(C + 1)]
        return [(cuts[c], cuts[c + 1], (cuts[c + 1] - cuts[c]) // N) for c in range(C) if cuts[c + 1] > cuts[c]], Pm

    def _groups(self):
        out = []
        where = {id(p): g for g in self.opt.param_groups for p in g["params"]}
        for p in self.bucket.params:
            g = where.get(id(p))
            if g is None:
                raise ValueError("ShardedAdam: a bucket parameter is not in the optimizer")
            out.append(g)
        return out

    def _run_update(self, items, hyper, dev):
        b1, b2, eps, maximize = hyper
        if self._update is not None:
            return self._update(items, b1, b2, eps, maximize)
        import gs_train

        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        gs_train.FusedAdam._launch(items, b1, b2, eps, maximize, dev, st)

    def _collective_ctx(self, dev):
        if dist.get_backend(self.group) == "nccl":
            return dist._coalescing_manager(self.group, device=dev, async_ops=True)
        return None

    @torch.no_grad()
    def step(self, average: bool = False) -> None:
        """One optimizer step from the bucket's gradients (replaces bucket.allreduce() +
        optimizer.step()).  The current stream waits for the step's collectives at the end."""
        b = self.bucket
        if self._pending:
            raise RuntimeError("ShardedAdam: the previous step's all-gathers were never waited for (pass "
                               "take_row_waits() to the next forward, or call sync())")
        b._check_bound()
        params = b.params
        P = params[0].shape[0]
        if any(p.dim() == 0 or p.shape[0] != P for p in params):
            raise ValueError("ShardedAdam: every bucket parameter must have the same row count")
        if self._sharded_P is not None and self._sharded_P != P:
            raise RuntimeError(f"ShardedAdam: the Gaussian count changed ({self._sharded_P} -> {P}) while the moments "
                               "were sharded: call gather_state() before densify_and_prune")
        N, r = self._world()
        groups = self._groups()
        hyper = {(float(g["betas"][0]), float(g["betas"][1]), float(g["eps"]), bool(g.get("maximize", False)))
                 for g in groups}
        if len(hyper) != 1:
            raise ValueError("ShardedAdam: the parameter groups must share betas, eps and maximize")
        hyper = hyper.pop()
        for g in groups:
            if g.get("amsgrad", False) or g.get("decoupled_weight_decay", False):
                raise NotImplementedError("ShardedAdam: amsgrad / decoupled weight decay are not supported")
        moments = [self._state(p) for p in params]
        steps = [self.opt._advance(p)[2] for p in params]
        lrs = [float(g["lr"]) for g in groups]
        wds = [float(g.get("weight_decay", 0.0)) for g in groups]
        local = not (dist.is_available() and dist.is_initialized())
        # no process group (one replica): nothing to exchange, so nothing to chunk or overlap -- one
        # update of every row, as FusedAdam.step
        chunks, Pm = ([(0, P, P)], P) if local else self.plan(P)
        dev = b.flat.device
        on_dev = b.flat.is_cuda
        deferred = bool(b._deferred)
        if deferred:
            inputs, views, outs, acc = b._claim_deferred()
            b._zero_unwritten()
        else:
            b.finalize()
        cur = torch.cuda.current_stream(dev) if on_dev else None
        if on_dev and self._comm is None:
            self._comm = torch.cuda.Stream(dev)
        comm = self._comm
        rows = [p.grad.view(P, -1) for p in params]  # gradient rows (bucket views)
        data = [p.detach().view(P, -1) for p in params]
        mv = [(m.view(P, -1), v.view(P, -1)) for m, v in moments]
        works = []
        overlap = self.overlap and on_dev and not local
        pending = []
        zero_ev = None
        last = len(chunks) - 1
        for c, (lo, hi, S) in enumerate(chunks + ([(Pm, Pm, 0)] if not chunks else [])):
            end = P if c == max(last, 0) else hi  # the last chunk's pass also covers the tail rows
            if deferred:
                b._deferred_pass(inputs, views, outs, acc, first=lo, count=end - lo)
            if on_dev:
                ev = torch.cuda.Event()
                ev.record(cur)
                comm.wait_event(ev)
            with (torch.cuda.stream(comm) if on_dev else _nullctx()):
                items = []
                if S > 0 and local:  # no process group (one replica): the rows are the rank's shard
                    shard = [g[lo:hi] for g in rows]
                    a, z = lo, hi
                elif S > 0:
                    shard = self._buf(c, rows, S, dev)
                    ctx = self._collective_ctx(dev) if on_dev else None
                    with (ctx if ctx is not None else _nullctx()) as cm:
                        for k, g in enumerate(rows):
                            dist.reduce_scatter_tensor(shard[k].view(-1), g[lo:hi].reshape(-1), group=self.group)
                    if cm is not None:
                        cm.wait()  # (the side stream waits for the coalesced group)
                    a, z = lo + r * S, lo + (r + 1) * S
                if S > 0:
                    for k in range(len(params)):
                        if average:
                            shard[k].div_(N)
                        items.append((data[k][a:z], shard[k], mv[k][0][a:z], mv[k][1][a:z], lrs[k], steps[k], wds[k]))
                if c == max(last, 0) and Pm < P:  # the tail: all-reduced, updated by every rank
                    for k, g in enumerate(rows):
                        t = g[Pm:P]
                        if not local:
                            dist.all_reduce(t, group=self.group)
                        if average:
                            t.div_(N)
                        items.append((data[k][Pm:P], t, mv[k][0][Pm:P], mv[k][1][Pm:P], lrs[k], steps[k], wds[k]))
                if items:
                    self._run_update(items, hyper, dev)
                if overlap:
                    # the chunk's gradient rows are consumed (reduce-scattered / all-reduced and
                    # updated): zero them here, so the next step's zero_grad needs no fill on its stream
                    for g in rows:
                        g[lo:end].zero_()
                    if c == max(last, 0):
                        zero_ev = torch.cuda.Event()
                        zero_ev.record(comm)
                if S > 0 and not local:
                    ctx = self._collective_ctx(dev) if on_dev else None
                    with (ctx if ctx is not None else _nullctx()) as cm:
                        for k in range(len(params)):
                            dist.all_gather_into_tensor(data[k][lo:hi].reshape(-1), data[k][a:z].reshape(-1),
                                                        group=self.group)
                    if cm is not None:
                        if overlap:
                            cm.wait()  # (the side stream waits for the coalesced group)
                        else:
                            works.append(cm)
                if overlap:
                    ev = torch.cuda.Event()
                    ev.record(comm)
                    pending.append((0 if not pending else pending[-1][1], end, ev))
        if deferred:
            b._retire_deferred(inputs, views)
        if N > 1:
            self._sharded_P = P
        if overlap:
            # no wait: the next forward waits for each chunk's all-gather (take_row_waits), the next
            # step's gradient writers for the zero-fill (the bucket's foreign read)
            self._pending = pending
            b.after_foreign_read(zero_ev, comm, zeroed=True)
            return
        for w in works:
            w.wait()
        if on_dev:
            cur.wait_stream(comm)
            b.written(cur)

    def _state(self, p):
        """(exp_avg, exp_avg_sq) of p, created as torch's Adam creates them, checked full-size"""
        st = self.opt.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0, dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        m, v = st["exp_avg"], st["exp_avg_sq"]
        for t in (m, v):
            if t.shape != p.shape or t.dtype != torch.float32 or not t.is_contiguous() or t.device != p.device:
                raise ValueError("ShardedAdam: optimizer state must be contiguous float32 of the parameter's shape")
        return m, v

    def _buf(self, c, rows, S, dev):
        key = (c, S, tuple(g.shape[1] for g in rows), str(dev))
        buf = self._bufs.get(key)
        if buf is None:
            if len(self._bufs) > 64:
                self._bufs.clear()
            buf = self._bufs[key] = [torch.empty((S, g.shape[1]), dtype=torch.float32, device=dev) for g in rows]
        return buf

    @torch.no_grad()
    def gather_state(self) -> None:
        """Make every rank's Adam moments whole (all-gather of the owned rows of exp_avg /
        exp_avg_sq, chunk by chunk): call before densify_and_prune or state_dict()."""
        self.sync()
        N, r = self._world()
        self._sharded_P = None
        if N == 1:
            return
        params = self.bucket.params
        P = params[0].shape[0]
        chunks, _ = self.plan(P)
        for p in params:
            st = self.opt.state.get(p)
            if not st:
                continue
            for t in (st["exp_avg"], st["exp_avg_sq"]):
                rows = t.view(P, -1)
                for lo, hi, S in chunks:
                    a, z = lo + r * S, lo + (r + 1) * S
                    dist.all_gather_into_tensor(rows[lo:hi].reshape(-1), rows[a:z].reshape(-1), group=self.group)


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


def _same_inputs(a, b) -> bool:
    for k in ("means3D", "sh", "colors", "scales", "rotations", "cov3D"):
        x, y = a[k], b[k]
        if (x is None) != (y is None):
            return False
        if x is not None and (x.data_ptr() != y.data_ptr() or x.shape != y.shape):
            return False
    return a["scale_modifier"] == b["scale_modifier"] and a["degree"] == b["degree"]


def run_views(view_fns: Sequence, streams: Sequence) -> None:
    """Run the views of one step round-robin on `streams` (view k on streams[k % n]): each view's
    forward (host-synchronous only up to its preprocess) and backward are enqueued on its stream,
    so one view's depth / tile sorts and scans overlap another view's tile passes.  Writes into a
    shared GradBucket are ordered by the bucket (write_order / written); the current stream then
    waits for every view stream.  Tensors a view allocates belong to its stream's allocator pool."""
    main = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(main)
    for k, fn in enumerate(view_fns):
        with _on_stream(streams[k % len(streams)], main):
            fn()
    for s in streams:
        main.wait_stream(s)


class _on_stream:
    """torch.cuda.stream(s) for a stream of the current device whose current stream is `main`:
    the same two stream switches without the context manager's device lookups (≈ 20 µs of host
    time per view, measured in tools/host_phases.py).  Another device's stream takes torch's path."""

    __slots__ = ("s", "main", "ctx")

    def __init__(self, s, main):
        self.s, self.main, self.ctx = s, main, None

    def __enter__(self):
        s = self.s
        if s.device_index != self.main.device_index:
            self.ctx = torch.cuda.stream(s)
            return self.ctx.__enter__()
        torch._C._cuda_setStream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)

    def __exit__(self, *exc):
        if self.ctx is not None:
            return self.ctx.__exit__(*exc)
        m = self.main
        torch._C._cuda_setStream(stream_id=m.stream_id, device_index=m.device_index, device_type=m.device_type)


def allreduce_grads(params: Iterable[torch.Tensor], group=None, average: bool = False):
    """One-off all-reduce of the .grad of `params` through a flat bucket (copies in and out; a
    training loop keeps a GradBucket instead, whose views ARE the gradients)."""
    params = [p for p in params]
    grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
    flat = torch.cat([g.reshape(-1) for g in grads])
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        if average:
            flat.div_(dist.get_world_size(group))
    off = 0
    for p in params:
        n = p.numel()
        p.grad = flat[off:off + n].view_as(p).clone()
        off += n


def replicated_group(group=None):
    """The process group whose ranks hold replicas of one model (view-parallel training), or None
    when there is none (no process group, or a world of one)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        return group if group is not None else dist.group.WORLD
    return None


def sync_from_rank0(t: torch.Tensor, group=None) -> torch.Tensor:
    """Every replica takes rank 0's values of `t` (in place).  Used for random draws that must be
    the same on every replica, e.g. densify_and_split's split samples
    (/root/reference/scene/gaussian_model.py:359-360): each rank draws (its generator advances as
    the reference's does), then rank 0's draw wins."""
    g = replicated_group(group)
    if g is not None:
        dist.broadcast(t, src=dist.get_global_rank(g, 0) if g is not dist.group.WORLD else 0, group=g)
    return t


_DIGEST_MOD = 2147483647  # 2^31 - 1


def replica_digest(tensors: Iterable[torch.Tensor]) -> torch.Tensor:
    """A bitwise digest of `tensors` (int64 [3]: two position-weighted sums of the 32-bit patterns
    modulo 2^31 - 1, and the element count): two ranks whose tensors differ in any bit get different
    digests with overwhelming probability.  Exact integer arithmetic on the tensors' device."""
    s1 = s2 = 0
    n = 0
    for t in tensors:
        b = t.detach().contiguous().view(-1).view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        b = b % _DIGEST_MOD
        i = torch.arange(b.numel(), dtype=torch.int64, device=b.device) + n
        w1 = i % 65521 + 1
        w2 = (i * 40503 + 7) % 65519 + 1
        s1 = (s1 + int(((b * w1) % _DIGEST_MOD).sum())) % _DIGEST_MOD
        s2 = (s2 + int(((b * w2) % _DIGEST_MOD).sum())) % _DIGEST_MOD
        n += b.numel()
    return torch.tensor([s1, s2, n], dtype=torch.int64)


def check_replicas(tensors: Sequence[torch.Tensor], group=None) -> bool:
    """True when every rank of the group holds bit-identical `tensors` (digest compared with a MIN
    and a MAX all-reduce).  Always True without a replicated group."""
    g = replicated_group(group)
    if g is None:
        return True
    d = replica_digest(tensors)
    dev = tensors[0].device if tensors and tensors[0].is_cuda else torch.device("cpu")
    lo, hi = d.to(dev).clone(), d.to(dev).clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=g)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=g)
    return bool(torch.equal(lo, hi))


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
