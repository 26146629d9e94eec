"""Multi-rank rendering through libpnr: 2 ranks share the box's GPU and
exchange over gloo (the 8-GPU RCCL run is the driver's).  Each rank renders
its band / tile share of every frame with the sync-free HIP path
(render_rays(sync=False) + finish()), TileShard.assemble_async gathers the
frame, and every rank's assembled frame must equal the single-process render
of the whole frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from formula import formula_params
from scenes import scene

pytestmark = pytest.mark.gpu

H = W = 48
THETAS = (30.0, 120.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(cuda, precision):
    from test_gpu_render import _renderer
    sc = scene(20000, H=H, W=W, theta=THETAS[0])
    m = _renderer(sc, cuda, formula_params(salt=0.8))
    m.precision = precision
    return sc, m


def _worker(rank, world, port, precision, layout, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    from pointnerf_amd.parallel import TileShard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cuda = torch.device("cuda:0")
    torch.cuda.set_device(cuda)
    sc, m = _model(cuda, precision)
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    outs = []
    handles = []
    if layout == "batch":   # bench --shard tiles: the step's band shares as ONE multi-camera batch
        from pointnerf_amd.parallel import StepShard
        scs = [scene(20000, H=H, W=W, theta=th) for th in THETAS]
        st = StepShard([TileShard(H, W, rank, world, f, cuda) for f in range(len(THETAS))], cuda)
        rd = st.select([torch.from_numpy(x["raydir"]).to(cuda) for x in scs]).contiguous()
        cp = torch.stack([torch.from_numpy(x["campos"]).to(cuda) for x in scs])
        cr = torch.stack([torch.from_numpy(x["camrot"]).to(cuda) for x in scs])
        m.render_rays(cp, cr, rd, 2.0, 6.0, bg, ray_cam=st.ray_cam)
        color = m.render_rays(cp, cr, rd, 2.0, 6.0, bg, sync=False, ray_cam=st.ray_cam)[0]
        m.finish()
        q.put((rank, [t.numpy() for t in st.assemble_async(color.cpu()).wait()]))
        dist.barrier()
        dist.destroy_process_group()
        return
    for f, th in enumerate(THETAS):
        s2 = scene(20000, H=H, W=W, theta=th)
        cp, cr, rd = (torch.from_numpy(s2[k]).to(cuda) for k in ("campos", "camrot", "raydir"))
        sh = TileShard(H, W, rank, world, f, cuda, layout=layout)
        if f == 0:
            m.render_rays(cp, cr, sh.select(rd), 2.0, 6.0, bg)   # sync call: sizes the sync-free ones
        color = m.render_rays(cp, cr, sh.select(rd), 2.0, 6.0, bg, sync=False)[0]
        handles.append((sh, color))
    m.finish()
    for sh, color in handles:
        outs.append(sh.assemble_async(color.cpu()).wait().numpy())
    q.put((rank, outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("layout", ["bands", "tiles16", "batch"])
def test_two_rank_libpnr_render_assembles_frames(cuda, layout):
    precision = "fp32h2"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, precision, layout, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sc, m = _model(cuda, precision)
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    for f, th in enumerate(THETAS):
        s2 = scene(20000, H=H, W=W, theta=th)
        cp, cr, rd = (torch.from_numpy(s2[k]).to(cuda) for k in ("campos", "camrot", "raydir"))
        want = m.render_rays(cp, cr, rd, 2.0, 6.0, bg)[0].cpu().numpy()
        for r in range(2):
            np.testing.assert_allclose(got[r][f], want, atol=1e-6, rtol=0)


def _train_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    from pointnerf_amd.parallel import GradReducer
    from test_gpu_backward import _train_model
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cuda = torch.device("cuda:0")
        torch.cuda.set_device(cuda)
        sc = scene(20000, H=32, W=32, theta=60.0, default_conf=None)
        params = formula_params(salt=0.3)
        cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
        rd = torch.from_numpy(sc["raydir"]).to(cuda)
        bg = torch.from_numpy(sc["bg"]).to(cuda)
        G = torch.randn((rd.shape[0], 128), generator=torch.Generator().manual_seed(5)).to(cuda)

        def grads(m, idx, scale):
            for p in m.parameters():
                p.grad = None
            color = m.render_rays_train(cp, cr, rd[idx].contiguous(), 2.0, 6.0, bg)[0]
            ((color * G[idx]).sum() * scale).backward()
            npt = m.neural_points
            return m, {**{k: getattr(npt, k) for k in ("points_embeding", "points_color", "points_dir",
                                                          "points_conf")},
                       **{"mlp " + k: p for k, p in m.aggregator.named_parameters()}}

        # this rank's rays: every world-th ray; per-rank loss, DDP-mean gradients
        m, ps = grads(_train_model(sc, cuda, params), torch.arange(rank, rd.shape[0], world, device=cuda), 1.0)
        npt = m.neural_points
        red = GradReducer(list(m.aggregator.parameters()),
                          [npt.points_embeding, npt.points_color, npt.points_dir, npt.points_conf])
        red.reduce(m.last_train_aux["touched_rows"], m.last_train_aux["touched_count"])
        if rank == 0:
            # one process, all rays: the mean of the ranks' losses
            _, ref = grads(_train_model(sc, cuda, params), torch.arange(rd.shape[0], device=cuda), 1.0 / world)
            for k in ps:
                a, b = ps[k].grad, ref[k].grad
                big = float(b.abs().max())
                d = float((a.reshape(b.shape) - b).abs().max())
                assert big > 0 and d <= 2e-5 * big, (k, d, big)
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()[-1500:]))
    finally:
        dist.destroy_process_group()


def test_dp_finetune_step_equals_single_process():
    """SURVEY 8(e) training: 2 ranks each backpropagate half the rays, GradReducer
    averages (one flat MLP all_reduce + the touched point rows), and the result
    equals one process backpropagating all the rays with the same total loss
    (float-atomic point sums: up to 2e-5 of the largest entry)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


def _rccl_worker(port, q):
    """One rank on the box's GPU over the "nccl" backend (= RCCL): every RCCL
    branch of parallel.py runs (all_gather_into_tensor of tiles, step batches,
    frames and GradReducer's row gathers, a flat all_reduce)."""
    try:
        import torch.distributed as dist
        from pointnerf_amd.parallel import FrameShard, GradReducer, StepShard, TileShard
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        cuda = torch.device("cuda:0")
        torch.cuda.set_device(cuda)
        dist.init_process_group("nccl", rank=0, world_size=1)
        assert dist.get_backend() == "nccl"
        g = torch.Generator(device="cpu").manual_seed(3)
        frames = [torch.randn((H * W, 5), generator=g).to(cuda) for _ in THETAS]
        errs = []
        for layout in ("bands", "tiles16"):
            sh = TileShard(H, W, 0, 1, 0, cuda, layout=layout)
            if not torch.equal(sh.assemble(sh.select(frames[0])), frames[0]):
                errs.append("TileShard " + layout)
        st = StepShard([TileShard(H, W, 0, 1, f, cuda) for f in range(len(THETAS))], cuda)
        got = st.assemble_async(st.select(frames)).wait()
        if not all(torch.equal(a, b) for a, b in zip(got, frames)):
            errs.append("StepShard")
        fr = FrameShard(0, 1).assemble_async(frames[1]).wait()
        if not (fr.shape == (1, H * W, 5) and torch.equal(fr[0], frames[1])):
            errs.append("FrameShard")
        t = torch.arange(12, dtype=torch.float32, device=cuda).reshape(3, 4)
        gr = GradReducer([], [])
        if not torch.equal(gr._all_gather(t)[0], t):
            errs.append("GradReducer._all_gather")
        x = torch.ones(7, device=cuda)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        if not torch.equal(x, torch.ones(7, device=cuda)):
            errs.append("all_reduce")
        dist.destroy_process_group()
        q.put(errs)
    except Exception as e:   # noqa: BLE001 -- reported to the parent
        q.put([repr(e)])


def test_rccl_branches_single_rank():
    """The RCCL (backend "nccl") branches of TileShard / StepShard / FrameShard /
    GradReducer execute on the GPU box and assemble exactly (one rank: the
    8-GPU run is the driver's; RCCL does not allow two ranks on one GPU)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    errs = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0, p.exitcode
    assert errs == [], errs
