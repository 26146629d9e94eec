"""Sync-free rendering (render_rays(sync=False) + finish()) and the HIP-graph
captured frame (RenderGraph): bitwise equal to the eager synchronous render
(the reference syncs at qpiw.py:656, 716 and
neural_points.py:786)."""
import gc

import pytest
import torch

from formula import formula_params
from scenes import scene
from test_gpu_render import _renderer

pytestmark = pytest.mark.gpu

PRECISIONS = ["fp32", "fp32h2", "bf16"]


def _cams(cuda, thetas=(30.0, 200.0), n=20000, H=40):
    out = []
    for th in thetas:
        sc = scene(n, H=H, W=H, theta=th)
        out.append(tuple(torch.from_numpy(sc[k]).to(cuda) for k in ("campos", "camrot", "raydir")))
    return sc, out


def _eq(a, b):
    return all(torch.equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize("precision", PRECISIONS)
def test_async_render_equals_sync(cuda, precision):
    sc, cams = _cams(cuda)
    m = _renderer(sc, cuda, formula_params(salt=0.4))
    m.precision = precision
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    want, counts = [], []
    for cp, cr, rd in cams:
        want.append([t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)])
        counts.append(dict(m.last_counts))
    got = [m.render_rays(cp, cr, rd, 2.0, 6.0, bg, sync=False) for cp, cr, rd in cams]
    assert len(m._pending) == 2
    assert m.finish() == counts
    assert m.overflow_rerenders == 0
    for w, g in zip(want, got):
        assert _eq(w, g)


@pytest.mark.parametrize("precision", ["fp32", "fp32h2"])
def test_partial_finish_keeps_later_calls_queued(cuda, precision):
    """finish(upto=k) completes the oldest k sync-free calls only (bench.py
    issues step s + 1 before completing step s); the rest complete at the next
    finish() -- counts in issue order, outputs equal to the synchronous renders;
    an overflowing call among them is re-rendered in place."""
    sc, cams = _cams(cuda, thetas=(30.0, 200.0, 120.0))
    m = _renderer(sc, cuda, formula_params(salt=0.4))
    m.precision = precision
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    want, counts = [], []
    for cp, cr, rd in cams:
        want.append([t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)])
        counts.append(dict(m.last_counts))
    got = [m.render_rays(cp, cr, rd, 2.0, 6.0, bg, sync=False) for cp, cr, rd in cams[:2]]
    assert m.finish(upto=1) == counts[:1]
    assert len(m._pending) == 1
    got.append(m.render_rays(*cams[2], 2.0, 6.0, bg, sync=False))
    assert m.finish(upto=1) == counts[1:2]
    m._sv_per_ray = 0.01            # the next call overflows its estimated feature buffer
    got.append(m.render_rays(*cams[0], 2.0, 6.0, bg, sync=False))
    assert m.finish() == [counts[2], counts[0]]
    assert m.overflow_rerenders == 1
    for w, g in zip(want + [want[0]], got):
        assert _eq(w, g)


@pytest.mark.parametrize("precision", ["fp32h2", "bf16"])
def test_query_stream_equals_sync(cuda, precision):
    """render_rays(sync=False, query_stream=s): each call's query on a second
    stream (two buffer sets in turn, each reused after the launch-stream work
    that read it) -- five queued calls over three cameras give the synchronous
    renders bitwise, and an overflowing call is still re-rendered in place."""
    sc, cams = _cams(cuda, thetas=(30.0, 200.0, 120.0))
    m = _renderer(sc, cuda, formula_params(salt=0.4))
    m.precision = precision
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    want = [[t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)] for cp, cr, rd in cams]
    qs = torch.cuda.Stream(cuda)
    torch.cuda.synchronize()
    order = [0, 1, 2, 0, 1]
    got = [m.render_rays(*cams[i], 2.0, 6.0, bg, sync=False, query_stream=qs) for i in order]
    m.finish()
    for i, g in zip(order, got):
        assert _eq(want[i], g)
    m._sv_per_ray = 0.01   # the next call overflows its feature buffer
    r0 = m.overflow_rerenders
    g = m.render_rays(*cams[2], 2.0, 6.0, bg, sync=False, query_stream=qs)
    m.finish()
    assert m.overflow_rerenders == r0 + 1 and _eq(want[2], g)
    # a non-contiguous raydir (its contiguous copy is the call's own, made on the
    # query stream) and an in-place point update on the launch stream between
    # queued calls (the query stream then waits for the launch stream)
    cp, cr, rd = cams[1]
    rd_nc = torch.cat([rd, rd], 1)[:, :3]
    assert not rd_nc.is_contiguous()
    g = m.render_rays(cp, cr, rd_nc, 2.0, 6.0, bg, sync=False, query_stream=qs)
    m.finish()
    assert _eq(want[1], g)
    xyz = m.neural_points.xyz
    with torch.no_grad():
        g0 = m.render_rays(*cams[0], 2.0, 6.0, bg, sync=False, query_stream=qs)
        xyz.add_(0.0625)                 # launch stream, after the queued call (bumps xyz._version)
        g1 = m.render_rays(*cams[0], 2.0, 6.0, bg, sync=False, query_stream=qs)
        m.finish()
        moved = [t.clone() for t in m.render_rays(*cams[0], 2.0, 6.0, bg)]
        xyz.sub_(0.0625)
    assert _eq(want[0], g0) and _eq(moved, g1)


def test_side_stream_p1_equals_sync(cuda):
    """fp32h2 sync-free calls run P1 (pnr_point_pre_h2) on a side stream beside
    the query and the aggregate waits on it: renders bitwise equal to the
    synchronous path (P1 inline), over two cameras and a re-use of the scratch."""
    sc, cams = _cams(cuda)
    m = _renderer(sc, cuda, formula_params(salt=0.4))
    m.precision = "fp32h2"
    m.p1_side_max_points_per_ray = 1e9   # the test scene has more points than rays
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    want = [[t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)] for cp, cr, rd in cams]
    for _ in range(2):
        ev = []
        got = [m.render_rays(cp, cr, rd, 2.0, 6.0, bg, sync=False, events=ev) for cp, cr, rd in cams]
        m.finish()
        assert sum(1 for name, _, _ in ev if name == "p1") == len(cams)
        for w, g in zip(want, got):
            assert _eq(w, g)


def test_async_overflow_rerenders_in_place(cuda):
    """A sync-free call whose valid samples outgrow the estimated feature
    buffer is composited memory-safely (rows past the buffer never read) and
    re-rendered by finish() into the same output tensors."""
    sc, cams = _cams(cuda, thetas=(30.0,))
    m = _renderer(sc, cuda, formula_params(salt=0.5))
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    cp, cr, rd = cams[0]
    want = [t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)]
    m._sv_per_ray = 0.01   # far below the scene's valid samples per ray
    got = m.render_rays(cp, cr, rd, 2.0, 6.0, bg, sync=False)
    m.finish()
    assert m.overflow_rerenders == 1
    assert _eq(want, got)
    assert m._sv_per_ray > 0.01   # the estimate learned the real count


@pytest.mark.parametrize("precision", PRECISIONS)
def test_render_graph_replay_bitwise(cuda, precision):
    """A frame captured in a HIP graph and replayed matches the eager render
    bitwise, and replaying with another camera copied into the static inputs
    matches that camera's eager render."""
    from pointnerf_amd.renderer import RenderGraph
    sc, cams = _cams(cuda, thetas=(30.0, 60.0))
    m = _renderer(sc, cuda, formula_params(salt=0.6))
    m.precision = precision
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    (cp, cr, rd), (cp2, cr2, rd2) = cams
    want = [t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)]
    want2 = [t.clone() for t in m.render_rays(cp2, cr2, rd2, 2.0, 6.0, bg)]
    g = RenderGraph(m, cp, cr, rd, 2.0, 6.0, bg, margin=1.5)
    out = g.replay()
    assert g.check()
    assert _eq(want, out)
    for _ in range(2):
        out = g.replay(cp2, cr2, rd2)
        assert g.check()
        assert _eq(want2, out)
    out = g.replay(cp, cr, rd)
    assert g.check() and _eq(want, out)


def _grid_in_cycle(cuda, sc):
    """A built GridHandle (device tables, pinned stats, an event) in a reference
    cycle, held by the returned list: once the list is cleared, the garbage
    collector, not the refcount, frees it."""
    from pointnerf_amd.querier import GridHandle
    h = GridHandle(cuda)
    h.build(sc["opt"], torch.from_numpy(sc["xyz"]).to(cuda).contiguous())
    torch.cuda.synchronize()
    h.cycle = h
    return [h]


def test_finaliser_inside_user_capture_keeps_graph_valid(cuda):
    """GPUTEST_r04's failure mode, forced: a dead GridHandle is collected inside
    a global-mode capture (torch's default).  Its finaliser must not call HIP
    (pnr_destroy's hipFree would invalidate the capture); the handle is freed
    at the next safe point instead."""
    from pointnerf_amd import querier as Q
    sc, _ = _cams(cuda, thetas=(30.0,))
    gc.collect()
    Q.release_deferred()
    gc_on = gc.isenabled()
    gc.disable()
    try:
        _grid_in_cycle(cuda, sc).clear()
        x = torch.zeros(16, device=cuda)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            assert gc.collect() > 0          # the finaliser runs here, mid-capture
            x.add_(1.0)
        assert len(Q._DEFERRED) == 1
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(x, torch.full_like(x, 2.0))
    finally:
        if gc_on:
            gc.enable()
    assert Q.release_deferred() == 1 and not Q._DEFERRED


@pytest.mark.parametrize("precision", ["fp32", "fp32h2"])
def test_render_graph_capture_survives_finaliser(cuda, precision):
    """RenderGraph with a GridHandle finaliser forced inside its capture window
    (an explicit collection at the captured call): the capture stays valid and
    the replay equals the eager render bitwise."""
    from pointnerf_amd import querier as Q
    from pointnerf_amd.renderer import RenderGraph
    sc, cams = _cams(cuda, thetas=(30.0,))
    m = _renderer(sc, cuda, formula_params(salt=0.6))
    m.precision = precision
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    cp, cr, rd = cams[0]
    want = [t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)]
    orig = m._render_rays
    seen = []
    holder = _grid_in_cycle(cuda, sc)

    def render_with_finaliser(*a, **kw):
        if kw.get("keep") is not None:        # the captured call
            holder.clear()                    # the handle becomes cyclic garbage mid-capture
            seen.append(gc.collect())
            seen.append(len(Q._DEFERRED))
        return orig(*a, **kw)

    m._render_rays = render_with_finaliser
    g = RenderGraph(m, cp, cr, rd, 2.0, 6.0, bg, margin=1.5)
    del m._render_rays
    assert seen and seen[0] > 0 and seen[1] >= 1
    assert not Q._DEFERRED                   # released right after the capture
    out = g.replay()
    assert g.check()
    assert _eq(want, out)


def test_render_graph_flags_overflow(cuda):
    """check() reports a replay whose valid samples outgrew the captured buffer."""
    from pointnerf_amd.renderer import RenderGraph
    sc, cams = _cams(cuda, thetas=(30.0,))
    m = _renderer(sc, cuda, formula_params(salt=0.7))
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    cp, cr, rd = cams[0]
    g = RenderGraph(m, cp, cr, rd, 2.0, 6.0, bg, margin=0.5)
    g.replay()
    assert not g.check()


@pytest.mark.parametrize("precision", ["fp32", "fp32x3", "fp32h2", "bf16"])
def test_render_views_one_batch_equals_per_view(cuda, precision):
    """render_views: several cameras' ray batches (the band shares of one
    multi-GPU step) in ONE query / aggregate / composite launch (per-ray
    camera index) give the per-camera renders: bitwise on the split paths
    (fp32x3 / fp32h2, the headline); the native-fp32 and bf16 pair kernels sum
    a tile's colour features in a tile-position-dependent order (measured
    <= 6e-8 / 4e-7), so there within 1e-6, with identical ray masks."""
    sc, cams = _cams(cuda, thetas=(30.0, 150.0, 260.0))
    m = _renderer(sc, cuda, formula_params(salt=0.9))
    m.precision = precision
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    views = [(cp, cr, rd[i::3].contiguous()) for i, (cp, cr, rd) in enumerate(cams)]
    want = [[t.clone() for t in m.render_rays(cp, cr, rd, 2.0, 6.0, bg)] for cp, cr, rd in views]
    got = m.render_views(views, 2.0, 6.0, bg)
    got2 = m.render_views(views, 2.0, 6.0, bg, sync=False)
    m.finish()
    for res in (got, got2):
        for w, g in zip(want, res):
            if precision in ("fp32x3", "fp32h2"):
                assert _eq(w, g)
            else:
                assert torch.equal(w[3], g[3])
                for x, y in zip(w[:3], g[:3]):
                    assert float((x - y).abs().max()) <= 1e-6


def test_partial_finish_does_not_wait_for_later_calls(cuda):
    """finish(upto=1) on fp32h2 reads call 1's range flag from the pinned copy
    taken behind call 1's event, not with a stream sync: it returns while a
    later call (queued behind a ~0.3 s spin kernel) is still running."""
    from pointnerf_amd import _lib as L
    sc, cams = _cams(cuda)
    m = _renderer(sc, cuda, formula_params(salt=0.4))
    m.precision = "fp32h2"
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    m.render_rays(*cams[0], 2.0, 6.0, bg)          # sizes the sync-free feature buffer
    m.render_rays(*cams[0], 2.0, 6.0, bg, sync=False)
    probe = torch.zeros(1, device=cuda)
    L.check(L.lib().pnr_clock_probe(L.ptr(probe), 1200000, L.stream_ptr(cuda)), "pnr_clock_probe")
    m.render_rays(*cams[1], 2.0, 6.0, bg, sync=False)
    ev = torch.cuda.Event()
    ev.record()
    assert len(m.finish(upto=1)) == 1
    assert not ev.query(), "finish(upto=1) waited for the later call"
    assert len(m.finish()) == 1
    assert ev.query()


def test_sync_call_keeps_pending_counts(cuda):
    """A synchronous render_rays drains the pending sync-free calls; their counts
    stay queued, so the next finish() still returns one entry per issued call."""
    sc, cams = _cams(cuda)
    m = _renderer(sc, cuda, formula_params(salt=0.4))
    bg = torch.from_numpy(sc["bg"]).to(cuda)
    m.render_rays(*cams[0], 2.0, 6.0, bg)
    want = dict(m.last_counts)
    m.render_rays(*cams[0], 2.0, 6.0, bg, sync=False)
    m.render_rays(*cams[1], 2.0, 6.0, bg, sync=False)
    m.render_rays(*cams[0], 2.0, 6.0, bg)           # synchronous: completes the two pending calls
    got = m.finish()
    assert len(got) == 2 and got[0] == want
