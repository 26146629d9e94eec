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
