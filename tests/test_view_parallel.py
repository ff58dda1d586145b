"""View-parallel exchange (gs_view_parallel) on CPU with gloo, world_size 2: one flat bucket
all-reduce of the 59-float/Gaussian gradient set, densify-statistics reduction, view sharding."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import gs_view_parallel as vp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, P, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(rank)
        shapes = [(P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4)]  # xyz f_dc f_rest opacity scaling rotation
        params = [torch.zeros(s, requires_grad=True) for s in shapes]
        b = vp.GradBucket(params)
        assert b.numel == 59 * P
        for p in params:  # the .grad tensors ARE views of the bucket
            assert p.grad.data_ptr() >= b.flat.data_ptr()
            p.grad.copy_(torch.randn(p.shape, generator=g))
        local = [p.grad.clone() for p in params]
        ptrs = [p.grad.data_ptr() for p in params]
        b.allreduce()
        assert ptrs == [p.grad.data_ptr() for p in params]  # reduced in place, no unpack
        acc = torch.zeros(P, 1) + rank
        den = torch.ones(P, 1)
        mr = torch.full((P,), float(rank + 1))
        vp.reduce_densify_stats(acc, den, mr)
        out_q.put((rank, [t.numpy() for t in local], [p.grad.numpy() for p in params], acc.numpy(), den.numpy(),
                   mr.numpy()))
    finally:
        dist.destroy_process_group()


def test_bucket_allreduce_and_densify_stats_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    P = 37
    procs = [ctx.Process(target=_worker, args=(r, 2, port, P, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, local, red, acc, den, mr = q.get(timeout=120)
        res[r] = (local, red, acc, den, mr)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in range(6):
        expect = res[0][0][k] + res[1][0][k]
        for r in range(2):
            torch.testing.assert_close(torch.tensor(res[r][1][k]), torch.tensor(expect))
    for r in range(2):
        assert (res[r][2] == 1).all() and (res[r][3] == 2).all() and (res[r][4] == 2).all()


def test_shard_views_round_robin():
    assert vp.shard_views(8, 0, 8) == [0]
    assert vp.shard_views(8, 1, 2) == [1, 3, 5, 7]
    views = sorted(v for r in range(3) for v in vp.shard_views(10, r, 3))
    assert views == list(range(10))


def test_single_process_allreduce_is_identity():
    p = torch.zeros(5, 3, requires_grad=True)
    p.grad = torch.arange(15.0).reshape(5, 3)
    vp.allreduce_grads([p])
    assert torch.equal(p.grad, torch.arange(15.0).reshape(5, 3))


def test_bucket_views_are_the_gradients_and_autograd_accumulates_into_them():
    a = torch.zeros(4, 3, requires_grad=True)
    c = torch.zeros(4, 1, requires_grad=True)
    b = vp.GradBucket([a, c])
    assert a.grad.data_ptr() == b.flat.data_ptr() and c.grad.data_ptr() == b.flat.data_ptr() + 12 * 4
    ((a * 2).sum() + (c * 3).sum()).backward()
    ((a * 1).sum()).backward()
    assert torch.all(a.grad == 3) and torch.all(c.grad == 3)
    assert torch.equal(b.flat[:12], torch.full((12,), 3.0))
    b.zero_grad()
    assert torch.all(b.flat == 0)


def test_lazy_bucket_claim_protocol():
    """lazy_zero: the first rasterizer claim of a step overwrites, later ones accumulate; views
    nobody wrote are zeroed before the all-reduce; a foreign write into an unwritten view raises."""
    a = torch.zeros(6, requires_grad=True)
    c = torch.zeros(2, requires_grad=True)
    b = vp.GradBucket([a, c], lazy_zero=True)
    b.flat.fill_(7.0)  # stale values from an earlier step
    b.zero_grad()
    buf, acc = b.claim(a)
    assert buf is a.grad and acc is False
    assert b.claim(a)[1] is True
    b.finalize()
    assert torch.all(c.grad == 0) and torch.all(a.grad == 7.0)  # a: left to the (simulated) kernel
    b.zero_grad()
    c.grad.add_(1.0)  # someone else accumulates into a view the rasterizer has not written yet
    with pytest.raises(RuntimeError, match="lazy_zero"):
        b.claim(c)
    a.grad = torch.zeros(6)  # replaced by the user: the sink steps aside
    assert b.claim(a) is None
    b.close()


def test_bucket_rebind_and_set_to_none():
    """rebind(): the bucket becomes the gradient storage of new parameters (densify_and_prune swaps
    in nn.Parameters of a new size); the old ones keep no view.  optimizer.zero_grad(set_to_none=True)
    drops the views: zero_grad() re-attaches them; a foreign .grad tensor raises."""
    a = torch.zeros(4, 3, requires_grad=True)
    c = torch.zeros(4, 1, requires_grad=True)
    b = vp.GradBucket([a, c])
    opt = torch.optim.SGD([a, c], lr=0.1)
    opt.zero_grad(set_to_none=True)
    assert a.grad is None
    b.zero_grad()
    assert a.grad.data_ptr() == b.flat.data_ptr()
    (a.sum() * 2).backward()
    assert torch.all(b.flat[:12] == 2)
    a2 = torch.zeros(7, 3, requires_grad=True)
    b.rebind([a2, c])
    assert b.numel == 7 * 3 + 4 and a.grad is None
    assert a2.grad.data_ptr() == b.flat.data_ptr() and c.grad.data_ptr() == b.flat.data_ptr() + 21 * 4
    (a2.sum() + 3 * c.sum()).backward()
    assert torch.all(a2.grad == 1) and torch.all(c.grad == 3)
    c.grad = torch.ones(4, 1)
    with pytest.raises(RuntimeError, match="replaced"):
        b.zero_grad()
    b.close()


def test_replica_digest_sees_one_bit():
    x = torch.randn(1000)
    y = x.clone()
    assert torch.equal(vp.replica_digest([x]), vp.replica_digest([y]))
    y.view(torch.int32)[517] ^= 1  # one ulp
    assert not torch.equal(vp.replica_digest([x]), vp.replica_digest([y]))
    z = x.clone()
    z[3], z[4] = x[4], x[3]  # same values, other positions
    assert not torch.equal(vp.replica_digest([x]), vp.replica_digest([z]))


def _sync_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = torch.full((5, 3), float(rank + 1))
        vp.sync_from_rank0(t)
        same = vp.check_replicas([t])
        u = torch.full((4,), float(rank))
        differ = vp.check_replicas([u])
        out_q.put((rank, t.numpy(), same, differ))
    finally:
        dist.destroy_process_group()


def test_sync_from_rank0_and_check_replicas_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sync_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, same, differ in res:
        assert (t == 1.0).all() and same and not differ


def _np_adam(items, b1, b2, eps, maximize):
    """Adam on CPU rows for the sharding test (numpy float32 ufuncs: one rounding per op, so every
    element's result is independent of how the rows are sliced); the GPU path is FusedAdam's kernel."""
    import numpy as np

    f = np.float32
    for p, g, m, v, lr, t, wd in items:
        pn, gn, mn, vn = (x.numpy() for x in (p, g, m, v))
        gg = -gn if maximize else gn.copy()
        if wd:
            gg += f(wd) * pn
        mn += f(1 - b1) * (gg - mn)
        vn *= f(b2)
        vn += f(1 - b2) * gg * gg
        denom = np.sqrt(vn) / f(math.sqrt(1 - b2 ** t)) + f(eps)
        pn += f(-lr / (1 - b1 ** t)) * (mn / denom)


def _sharded_worker(rank, world, port, P, chunks, out_q, average=False):
    """Two replicas per rank from the same init: one steps through GradBucket.allreduce + Adam on all
    rows, the other through ShardedAdam (reduce-scatter, Adam on the rank's rows, all-gather); three
    steps, a densify-like resize (prune + append rows of params and moments, new P with a tail), two
    more steps."""
    import gs_train

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        widths = [(3,), (1, 3), (15, 3), (1,), (3,), (4,)]
        lrs = [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3]

        def make(P):
            g = torch.Generator().manual_seed(5)
            ps = [torch.nn.Parameter(torch.randn((P,) + w, generator=g)) for w in widths]
            opt = gs_train.FusedAdam([{"params": [p], "lr": lr} for p, lr in zip(ps, lrs)], lr=0.0, eps=1e-15)
            return ps, opt, vp.GradBucket(ps)

        pa, oa, ba = make(P)
        pb, ob, bb = make(P)
        sh = vp.ShardedAdam(ob, bb, chunks=chunks, update=_np_adam)

        def grads(step, ps, bucket):
            g = torch.Generator().manual_seed(100 * step + rank)
            bucket.zero_grad()
            for p in ps:
                p.grad.copy_(torch.randn(p.shape, generator=g))

        def step_a(step):
            grads(step, pa, ba)
            ba.allreduce(average=average)
            items = []
            for p, grp in zip(pa, oa.param_groups):
                st = oa.state[p]
                if not st:
                    st.update(step=torch.tensor(0.0), exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p))
                t = oa._advance(p)[2]
                items.append((p.detach(), p.grad, st["exp_avg"], st["exp_avg_sq"], grp["lr"], t, 0.0))
            _np_adam(items, 0.9, 0.999, 1e-15, False)

        def step_b(step):
            grads(step, pb, bb)
            sh.step(average=average)

        for s_ in range(3):
            step_a(s_)
            step_b(s_)
        sh.gather_state()

        def resize(ps, opt, bucket):  # keep 3 of every 4 rows, append 6 copies of the first rows
            keep = torch.arange(ps[0].shape[0]) % 4 != 1
            new = []
            for i, p in enumerate(ps):
                st = opt.state.pop(p)
                f = lambda t: torch.cat([t[keep], t[:6]]).contiguous()  # noqa: E731
                q = torch.nn.Parameter(f(p.detach()))
                st["exp_avg"], st["exp_avg_sq"] = f(st["exp_avg"]), f(st["exp_avg_sq"])
                opt.state[q] = st
                opt.param_groups[i]["params"][0] = q
                new.append(q)
            bucket.rebind(new)
            return new

        pa[:] = resize(pa, oa, ba)
        pb[:] = resize(pb, ob, bb)
        for s_ in range(3, 5):
            step_a(s_)
            step_b(s_)
        sh.gather_state()

        def dump(ps, opt):
            return [t.detach().numpy().copy() for p in ps for t in (p, opt.state[p]["exp_avg"], opt.state[p]["exp_avg_sq"])]

        out_q.put((rank, dump(pa, oa), dump(pb, ob), [float(ob.state[p]["step"]) for p in pb], pb[0].shape[0],
                   sh.plan(pb[0].shape[0])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,chunks,average", [(37, 3, False), (64, 4, False), (1, 2, False), (50, 2, True)])
def test_sharded_adam_equals_allreduce_gloo_world2(P, chunks, average):
    """ShardedAdam (reduce-scatter -> Adam on the rank's row slices -> all-gather, in row chunks, with
    the odd tail all-reduced) against GradBucket.allreduce + Adam on every row, world 2 (gloo, CPU):
    parameters and both moments bit-identical on both ranks after 3 steps, a resize of every
    parameter and moment (rows pruned and appended, as densify_and_prune does; gather_state first) and
    2 more steps."""
    import numpy as np

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, P, chunks, q, average)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, a, b, steps, Pn, plan = q.get(timeout=120)
        res[r] = (a, b, steps, Pn, plan)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        a, b, steps, Pn, plan = res[r]
        assert steps == [5.0] * 6
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(b, res[0][1]):
            np.testing.assert_array_equal(x, y)
    if P >= 4:
        assert len(res[0][4][0]) > 1  # the step ran in several chunks


def _guard_worker(rank, world, port, out_q):
    """ShardedAdam's sharded-moments guard: after a step every rank's moments are current only on its
    own rows, so state_dict(), densify_and_prune and a step at another Gaussian count must raise
    until gather_state() makes them whole again."""
    import types

    import gs_train

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        g = torch.Generator().manual_seed(5)
        ps = [torch.nn.Parameter(torch.randn((37,) + w, generator=g)) for w in [(3,), (4,)]]
        opt = gs_train.FusedAdam([{"params": [p], "lr": 1e-3} for p in ps], lr=0.0, eps=1e-15)
        bucket = vp.GradBucket(ps)
        sh = vp.ShardedAdam(opt, bucket, chunks=2, update=_np_adam, overlap=True)
        bucket.zero_grad()
        for p in ps:
            p.grad.fill_(1.0)
        sh.step()
        res["sharded_after_step"] = sh.moments_sharded()
        res["no_waits_on_cpu"] = sh.take_row_waits() == []  # (overlap needs device streams)

        def raises(fn, text):
            try:
                fn()
            except RuntimeError as e:
                return text in str(e)
            return False

        res["state_dict_raises"] = raises(opt.state_dict, "gather_state")
        model = types.SimpleNamespace(optimizer=opt)
        res["densify_raises"] = raises(lambda: gs_train.densify_and_prune(model, 2e-4, 0.005, 1.0, 20), "gather_state")
        # a Gaussian count change while sharded (a densify without gather_state) is refused at the next step
        new = [torch.nn.Parameter(p.detach()[:30].clone()) for p in ps]
        for i, (p, q) in enumerate(zip(ps, new)):
            st = opt.state.pop(p)
            st["exp_avg"], st["exp_avg_sq"] = st["exp_avg"][:30].clone(), st["exp_avg_sq"][:30].clone()
            opt.state[q] = st
            opt.param_groups[i]["params"][0] = q
        bucket.rebind(new)
        bucket.zero_grad()
        res["step_raises"] = raises(sh.step, "Gaussian count changed")
        sh.gather_state()
        res["whole_after_gather"] = not sh.moments_sharded() and isinstance(opt.state_dict(), dict)
        bucket.zero_grad()
        sh.step()  # at the new count, after gather_state
        res["steps"] = [float(opt.state[p]["step"]) for p in new]
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_sharded_adam_refuses_stale_moments_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        got = res[r]
        assert got.pop("steps") == [2.0, 2.0]
        assert all(got.values()), got
