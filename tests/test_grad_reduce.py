"""GradReducer (pointnerf_amd.parallel): the data-parallel finetune step's
gradient mean -- one flat all_reduce for the MLP, touched point rows gathered
and index-added -- equals DDP's dense mean all-reduce (base_model.py:61-71),
on gloo with world size 2 (and 3, uneven touched-row counts)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N = 500


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    dense = [torch.randn(7, 5, generator=g), torch.randn(11, generator=g)]
    touched = torch.randint(0, N, (40 + 17 * rank,), generator=g)   # duplicates allowed
    emb = torch.zeros(1, N, 32)
    col = torch.zeros(N, 3)
    conf = torch.zeros(N, 1)
    u = torch.unique(touched)
    emb[0, u] = torch.randn(u.numel(), 32, generator=g)
    col[u] = torch.randn(u.numel(), 3, generator=g)
    conf[u] = torch.randn(u.numel(), 1, generator=g)
    return dense, [emb, col, conf], touched


def _worker(rank, world, port, q, mode="dup"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pointnerf_amd.parallel import GradReducer
        dense_g, point_g, touched = _data(rank)
        dense = [torch.nn.Parameter(torch.zeros_like(t)) for t in dense_g]
        points = [torch.nn.Parameter(torch.zeros_like(t)) for t in point_g]
        for p, g in zip(dense + points, dense_g + point_g):
            p.grad = g.clone()
        if mode == "count":
            # render_rays_train's form: unique rows, -1 placeholders, the count on the host
            rows = torch.cat([torch.unique(touched), torch.tensor([-1, -1])])
            GradReducer(dense, points).reduce(rows, rows.numel())
        else:
            GradReducer(dense, points).reduce(touched)
        # DDP's reference: the dense mean over ranks
        ref = [sum(_data(r)[0][i] for r in range(world)) / world for i in range(2)]
        refp = [sum(_data(r)[1][i] for r in range(world)) / world for i in range(3)]
        for p, r in zip(dense + points, ref + refp):
            torch.testing.assert_close(p.grad, r, rtol=1e-6, atol=1e-6)
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _worker_inf(rank, world, port, q):
    """Row 0 of a rank's point gradient is inf but untouched; the -1 placeholders
    gather it and must add exact zeros (not 0 * inf = NaN) on every rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pointnerf_amd.parallel import GradReducer
        p = torch.nn.Parameter(torch.zeros(N, 4))
        g = torch.zeros(N, 4)
        g[0] = float("inf")
        rows = torch.tensor([5 + rank, 9, -1])
        g[rows[:2]] = torch.tensor([[1.0, 2.0, 3.0, 4.0]]) * (rank + 1)
        p.grad = g
        GradReducer([], [p]).reduce(rows, rows.numel())
        assert torch.isfinite(p.grad).all(), "NaN / inf spread by the padding"
        assert torch.equal(p.grad[0], torch.zeros(4))
        assert torch.allclose(p.grad[9], torch.tensor([1.0, 2.0, 3.0, 4.0]) * sum(r + 1 for r in range(world)) / world)
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_grad_reducer_padding_does_not_spread_inf():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_inf, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,mode", [(2, "dup"), (3, "dup"), (2, "count"), (3, "count")])
def test_grad_reducer_equals_dense_mean(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


def test_grad_reducer_single_process_is_identity():
    from pointnerf_amd.parallel import GradReducer
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(_free_port())
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        p = torch.nn.Parameter(torch.zeros(3))
        p.grad = torch.tensor([1.0, 2.0, 3.0])
        GradReducer([p], []).reduce()
        assert torch.equal(p.grad, torch.tensor([1.0, 2.0, 3.0]))
    finally:
        dist.destroy_process_group()
