"""Ray-tile sharding + all-gather assembly on world_size 2 (gloo, CPU).
Each rank renders its tiles with the CPU oracle (the renderer itself needs a
GPU); the assembled frame must equal the single-process render."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from formula import formula_params
from oracle import oracle as O
from scenes import oracle_points, scene

H = W = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    from pointnerf_amd.parallel import TileShard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scene(8000, H=H, W=W, theta=60.0)
    params = formula_params(salt=0.4)
    outs = []
    for frame in range(4):
        sh = TileShard(H, W, rank, world, frame, layout="bands" if frame < 2 else "tiles16")
        rd = sh.select(torch.from_numpy(sc["raydir"])).numpy()
        r = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], rd, sc["bg"])
        local = torch.from_numpy(np.concatenate([r["coarse_raycolor"], r["coarse_is_background"]], 1))
        outs.append(sh.assemble(local).numpy())
    if rank == 0:
        q.put(outs)
    dist.barrier()
    dist.destroy_process_group()


def test_tile_split_covers_every_pixel_once():
    from pointnerf_amd.parallel import tile_owner
    for world in (1, 2, 3, 8):
        for frame in range(3):
            own = tile_owner(800, 800, world, frame, "tiles16")
            c = np.bincount(own, minlength=world)
            assert c.sum() == 640000 and c.max() - c.min() <= 256   # at most one 16x16 tile apart


def test_band_shards_800_8_ranks_bookkeeping():
    """bench --shard tiles at 800x800 on 8 ranks (the driver's N = 8 run): per
    frame every pixel has exactly one owner, each rank's share is whole pixel
    rows (contiguous, row-major), the gathered-row map is a permutation, and
    over the 8 frames of a step every rank renders every band exactly once."""
    from pointnerf_amd.parallel import TileShard, tile_owner
    H = W = 800
    world = 8
    seen = np.zeros((world, world), dtype=np.int64)   # [rank, band] pixels over a step
    for frame in range(world):
        own = tile_owner(H, W, world, frame)
        assert np.bincount(own, minlength=world).tolist() == [H * W // world] * world
        shards = [TileShard(H, W, r, world, frame) for r in range(world)]
        for r, sh in enumerate(shards):
            px = sh.pixels[r]
            assert px.size % W == 0 and np.array_equal(px, np.arange(px[0], px[0] + px.size))
            band = (px[0] // W) * world // H
            seen[r, band] += px.size
        src = shards[0].src.numpy()
        assert np.array_equal(np.sort(src), np.arange(H * W)) and shards[0].max_count == H * W // world
    assert (seen == H * W // world).all()


def test_two_rank_render_assembles_full_frame():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sc = scene(8000, H=H, W=W, theta=60.0)
    full = O.render(sc["opt"], oracle_points(sc), formula_params(salt=0.4), sc["campos"], sc["camrot"],
                    sc["raydir"], sc["bg"])
    want = np.concatenate([full["coarse_raycolor"], full["coarse_is_background"]], 1)
    for got in outs:
        np.testing.assert_allclose(got, want, atol=1e-5, rtol=1e-5)


def _frame_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    from pointnerf_amd.parallel import FrameShard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fs = FrameShard(rank, world)
    params = formula_params(salt=0.4)
    outs = []
    for step in range(2):
        frame = fs.frame_of(step)   # whole frame step * world + rank, one camera per frame
        sc = scene(8000, H=24, W=24, theta=60.0 + 45.0 * frame)
        r = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
        local = torch.from_numpy(np.concatenate([r["coarse_raycolor"], r["coarse_is_background"]], 1))
        outs.append(fs.assemble_async(local).wait().numpy())
    if rank == 0:
        q.put(outs)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_frame_shards_gather_every_frame():
    """FrameShard (bench --shard frames): rank r renders frames r, r + 2, ...;
    after each step's all-gather every rank holds both frames, in frame order,
    equal to single-process renders."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_frame_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    params = formula_params(salt=0.4)
    for step, got in enumerate(outs):
        assert got.shape[0] == 2
        for r in range(2):
            sc = scene(8000, H=24, W=24, theta=60.0 + 45.0 * (step * 2 + r))
            full = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
            want = np.concatenate([full["coarse_raycolor"], full["coarse_is_background"]], 1)
            np.testing.assert_allclose(got[r], want, atol=1e-5, rtol=1e-5)


def _step_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    from pointnerf_amd.parallel import StepShard, TileShard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    params = formula_params(salt=0.4)
    scs = [scene(8000, H=24, W=24, theta=60.0 + 90.0 * f) for f in range(world)]
    st = StepShard([TileShard(24, 24, rank, world, f) for f in range(world)])
    rd = st.select([torch.from_numpy(sc["raydir"]) for sc in scs]).numpy()
    cam = st.ray_cam.numpy()
    rows = []
    for f, sc in enumerate(scs):   # the oracle renders each camera's rows of the one batch
        r = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], rd[cam == f], sc["bg"])
        rows.append(np.concatenate([r["coarse_raycolor"], r["coarse_is_background"]], 1))
    local = torch.from_numpy(np.concatenate(rows))
    q.put((rank, [t.numpy() for t in st.assemble_async(local).wait()]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_step_shard_one_gather_assembles_every_frame():
    """StepShard (bench --shard tiles): each rank's band shares of the step's
    frames form ONE batch (frame order, ray_cam = frame) and ONE all-gather
    assembles every frame on every rank, equal to single-process renders."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_step_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    params = formula_params(salt=0.4)
    for f in range(2):
        sc = scene(8000, H=24, W=24, theta=60.0 + 90.0 * f)
        full = O.render(sc["opt"], oracle_points(sc), params, sc["campos"], sc["camrot"], sc["raydir"], sc["bg"])
        want = np.concatenate([full["coarse_raycolor"], full["coarse_is_background"]], 1)
        for r in range(2):
            np.testing.assert_allclose(got[r][f], want, atol=1e-5, rtol=1e-5)
