"""libpnr query kernels vs the CPU oracle (bit-exact integer/index results)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from scenes import scene

pytestmark = pytest.mark.gpu


def _engine(sc, cuda):
    from pointnerf_amd.querier import lighting_fast_querier
    return lighting_fast_querier(cuda, sc["opt"])


def _run(sc, cuda, q=None):
    q = q or _engine(sc, cuda)
    xyz = torch.from_numpy(sc["xyz"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda)
    cp = torch.from_numpy(sc["campos"]).to(cuda)
    cr = torch.from_numpy(sc["camrot"]).to(cuda)
    out = q.query_points(None, None, xyz[None], None, 800, 800, None, 2.0, 6.0, rd[None], cp[None], cr[None])
    return q, out


@pytest.mark.parametrize("slot0_drop", [1, 0])
def test_grid_tables_bit_exact(cuda, slot0_drop):
    sc = scene(20000, slot0_drop=slot0_drop)
    q = _engine(sc, cuda)
    xyz = torch.from_numpy(sc["xyz"]).to(cuda)
    hp = q.grid.build(sc["opt"], xyz)
    g = O.grid_build(sc["opt"], sc["xyz"])
    assert np.array_equal(hp["shift"], g["hp"]["shift"]) and np.array_equal(hp["dims"], g["hp"]["dims"])
    assert np.array_equal(hp["vsize_s"], g["hp"]["vsize_s"])
    t = q.grid.export()
    assert np.array_equal(t["coor_2_occ"].cpu().numpy(), g["coor_2_occ"])
    bits = t["occ_bits"].cpu().numpy().view(np.uint32)
    occ = ((bits[:, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(-1)[: g["coor_occ"].size]
    assert np.array_equal(occ.astype(np.uint8), g["coor_occ"])
    assert np.array_equal(t["occ_numpnts"].cpu().numpy(), g["occ_numpnts"])
    assert np.array_equal(t["occ_2_pnts"].cpu().numpy(), g["occ_2_pnts"])
    st = q.grid.stats()
    assert st["n_voxels"] == g["n_occ"] and st["n_points_dropped"] == 0
    if slot0_drop:
        assert g["occ_numpnts"][0] == 0  # the fill_occ2pnts `voxel_idx > 0` quirk (qpiw.py:372)


@pytest.mark.parametrize("n,max_o,P", [(20000, 1500, 1), (3, 8, 2), (70000, 400000, 9)])
def test_grid_tables_bit_exact_sizes_and_overflow(cuda, n, max_o, P):
    """The radix-sorted build across tile counts (1, 10 and 35 ragged tiles of
    2048 keys) and with both reservoirs active (max_o and P overflow)."""
    sc = scene(max(n, 20000), max_o=max_o, P=P)
    xyz = sc["xyz"][:n].copy()
    q = _engine(sc, cuda)
    q.grid.build(sc["opt"], torch.from_numpy(xyz).to(cuda))
    g = O.grid_build(sc["opt"], xyz)
    t = q.grid.export()
    assert np.array_equal(t["coor_2_occ"].cpu().numpy(), g["coor_2_occ"])
    assert np.array_equal(t["occ_numpnts"].cpu().numpy(), g["occ_numpnts"])
    assert np.array_equal(t["occ_2_pnts"].cpu().numpy(), g["occ_2_pnts"])
    bits = t["occ_bits"].cpu().numpy().view(np.uint32)
    occ = ((bits[:, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(-1)[: g["coor_occ"].size]
    assert np.array_equal(occ.astype(np.uint8), g["coor_occ"])
    st = q.grid.stats()
    assert st["n_voxels"] == g["n_occ"]
    kept = g["occ_numpnts"][: min(max_o, g["n_occ"])]
    assert st["n_points_dropped"] == int(np.maximum(kept - P, 0).sum())
    if n == 20000:
        assert g["n_occ"] > max_o and st["n_points_dropped"] > 0   # both reservoirs ran


# K 16 / 24 / 32 run the KMAX = 16 / 32 instantiations of k_knn (their
# LDS neighbour columns and replace-phase rescans are otherwise untested); their
# denser clouds and larger P fill all K slots of some samples, so candidates
# beyond K replace farther ones
@pytest.mark.parametrize("K,theta,n,P", [(8, 30.0, 20000, 9), (4, 130.0, 20000, 9), (16, 70.0, 200000, 26),
                                         (24, 200.0, 300000, 32), (32, 300.0, 300000, 40)])
def test_query_points_bit_exact(cuda, K, theta, n, P):
    sc = scene(n, H=48, W=40, theta=theta, K=K, P=P)
    _, out = _run(sc, cuda)
    ref = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    pidx, loc, loc_w, dirs, ray_mask = [t.cpu().numpy() for t in out[:5]]
    assert np.array_equal(ray_mask[0], ref["ray_mask"])
    assert ref["ray_mask"].sum() > 100, "scene must exercise the query"
    assert pidx.shape == (1,) + ref["sample_pidx"].shape
    assert np.array_equal(pidx[0], ref["sample_pidx"])          # same neighbours, same order
    if K >= 16:
        assert (ref["sample_pidx"][..., K - 1] >= 0).sum() > 0, "some samples must fill all K slots"
    assert np.array_equal(loc_w[0], ref["sample_loc_w"])
    assert np.array_equal(loc[0], ref["sample_loc"])
    assert np.array_equal(dirs[0], ref["sample_ray_dirs"])
    np.testing.assert_array_equal(out[6], ref["ranges"])


def test_query_internal_buffers(cuda):
    sc = scene(20000, H=32, W=32)
    q = _engine(sc, cuda)
    xyz = torch.from_numpy(sc["xyz"]).to(cuda)
    bufs, hp, rays, qp = q.run(xyz, torch.from_numpy(sc["raydir"]).to(cuda), torch.from_numpy(sc["campos"]).to(cuda),
                               torch.from_numpy(sc["camrot"]).to(cuda), 2.0, 6.0)
    c = bufs.read_counts()
    ref = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    R, SR = sc["raydir"].shape[0], sc["opt"].SR
    nf = bufs.n_filled[:R].cpu().numpy()
    assert np.array_equal(nf, ref["n_filled"])
    sd = bufs.slot_d[: R * SR].cpu().numpy().astype(np.int32).reshape(R, SR)
    for r in range(R):
        assert np.array_equal(sd[r, : nf[r]], ref["slot_d"][r, : nf[r]])
    assert c["S_filled"] == nf.sum() and c["R_hit"] == (nf > 0).sum()
    assert c["R_valid"] == ref["ray_mask"].sum()
    assert c["n_pairs"] == (ref["pidx_dense"] >= 0).sum()
    assert c["S_valid"] == (ref["pidx_dense"] >= 0).any(-1).sum()


def test_jittered_rays_per_ray_table(cuda):
    # training mode: per-ray jittered depths (diff_ray_marching.py:373-375)
    sc = scene(20000, H=24, W=24, is_train=1)
    q = _engine(sc, cuda)
    torch.manual_seed(3)
    _, out = _run(sc, cuda, q)
    torch.manual_seed(3)
    from pointnerf_amd.querier import ray_mid_t
    tv = ray_mid_t(2.0, 6.0, 400, R=sc["raydir"].shape[0], jitter=0.3, device=cuda).cpu().numpy()
    ref = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], mid_t=tv)
    assert np.array_equal(out[4].cpu().numpy()[0], ref["ray_mask"])
    assert np.array_equal(out[0].cpu().numpy()[0], ref["sample_pidx"])


def test_rays_missing_everything(cuda):
    # rays pointing away from the scene: R'' = 0, empty outputs, ray_mask all 0
    sc = scene(5000, H=8, W=8)
    sc["raydir"] = -sc["raydir"]
    _, out = _run(sc, cuda)
    assert out[0].shape == (1, 0, sc["opt"].SR, sc["opt"].K)
    assert int(out[4].sum()) == 0


def test_deterministic_and_repeatable(cuda):
    sc = scene(20000, H=32, W=32)
    q, a = _run(sc, cuda)
    q.grid.key = None  # force a rebuild
    _, b = _run(sc, cuda, q)
    for x, y in zip(a[:5], b[:5]):
        assert torch.equal(x, y)


def test_scan_matches_cumsum(cuda):
    from pointnerf_amd import _lib as L
    rng = np.random.default_rng(0)
    for n in (1, 7, 2048, 2049, 100000, 1 << 20, 5_000_000, 9_000_000):   # <= 4096 tiles: two launches; beyond: three
        x = torch.from_numpy(rng.integers(0, 5, size=n).astype(np.int32)).to(cuda)
        out = torch.empty(n + 1, dtype=torch.int32, device=cuda)
        tot = torch.empty(1, dtype=torch.int32, device=cuda)
        nb = L.c_size_t(0)
        L.lib().pnr_scan_scratch_bytes(n, L.ctypes.byref(nb))
        scratch = torch.empty(nb.value, dtype=torch.uint8, device=cuda)
        L.check(L.lib().pnr_exclusive_scan_i32(L.ptr(x), n, None, L.ptr(out), n + 1, L.ptr(tot), L.ptr(scratch),
                                               nb.value, L.stream_ptr()), "scan")
        ref = np.concatenate([[0], np.cumsum(x.cpu().numpy())])
        assert np.array_equal(out.cpu().numpy(), ref)
        assert int(tot.item()) == ref[-1]


def test_coop_march_equals_serial_march(cuda):
    """k_march_coop<16> (batches of <= 32768 rays: 16 lanes per ray) and
    k_march_coop<8> (larger batches) give the same slots, those of a serial walk
    along the ray (the oracle tests): the first 3000 rays of a 160x240 frame
    queried alone vs inside the frame."""
    sc = scene(20000, H=160, W=240, theta=75.0)
    q = _engine(sc, cuda)
    xyz = torch.from_numpy(sc["xyz"]).to(cuda)
    rd = torch.from_numpy(sc["raydir"]).to(cuda)
    cp, cr = torch.from_numpy(sc["campos"]).to(cuda), torch.from_numpy(sc["camrot"]).to(cuda)
    R, SR = rd.shape[0], sc["opt"].SR
    assert R > 32768
    big, _, _, _ = q.run(xyz, rd, cp, cr, 2.0, 6.0)
    nf_big = big.n_filled[:3000].clone()
    sd_big = big.slot_d[: R * SR].view(R, SR)[:3000].clone()
    small, _, _, _ = q.run(xyz, rd[:3000].contiguous(), cp, cr, 2.0, 6.0)
    nf = small.n_filled[:3000]
    assert torch.equal(nf, nf_big) and int(nf.sum()) > 1000
    sd = small.slot_d[: 3000 * SR].view(3000, SR)
    keep = torch.arange(SR, device=cuda)[None, :] < nf[:, None]
    assert torch.equal(sd[keep], sd_big[keep])


def test_march_box_clipping_edge_rays(cuda):
    """The shared-table march tests only the depths inside the grid box padded by
    one voxel (query.hip k_march_coop): rays from a camera inside the box in every
    direction, axis-parallel rays (zero direction components, +-x, +-y, +-z), and
    rays from outside that run along the box's faces -- the same filled slots and
    neighbours as the oracle's serial walk."""
    sc = scene(20000, H=16, W=16)
    xyz = sc["xyz"]
    lo, hi = xyz.min(0), xyz.max(0)
    ctr = ((lo + hi) / 2).astype(np.float32)
    rng = np.random.default_rng(7)
    d = rng.normal(size=(250, 3))
    d = np.concatenate([d, np.eye(3), -np.eye(3), [[1, 1, 0], [0, 1, -1], [1, 0, 1]]])
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    q = _engine(sc, cuda)
    xt = torch.from_numpy(xyz).to(cuda)
    cr = torch.from_numpy(sc["camrot"]).to(cuda)
    cams = [ctr,                                                          # inside the box
            np.array([lo[0] - 1.0, ctr[1], hi[2]], dtype=np.float32),     # on the top face's plane
            np.array([ctr[0], lo[1] - 0.5, lo[2]], dtype=np.float32)]     # on the bottom face's plane
    R, SR = d.shape[0], sc["opt"].SR
    filled = 0
    for cam in cams:
        bufs, _, _, _ = q.run(xt, torch.from_numpy(d).to(cuda), torch.from_numpy(cam).to(cuda), cr, 0.05, 3.0)
        ref = O.query_points(sc["opt"], xyz, cam, sc["camrot"], d, near=0.05, far=3.0)
        nf = bufs.n_filled[:R].cpu().numpy()
        assert np.array_equal(nf, ref["n_filled"])
        sd = bufs.slot_d[: R * SR].cpu().numpy().astype(np.int32).reshape(R, SR)
        for r in range(R):
            assert np.array_equal(sd[r, : nf[r]], ref["slot_d"][r, : nf[r]]), r
        filled += int(nf.sum())
    assert filled > 1000


def test_used_points_device_equals_torch(cuda):
    """pnr_used_points (device list + map, count in counts[5]) == the torch
    restatement train.used_points on the query's filled rows."""
    from pointnerf_amd.train import used_points, used_points_device
    sc = scene(20000, H=40, W=40, theta=50.0)
    q = _engine(sc, cuda)
    xyz = torch.from_numpy(sc["xyz"]).to(cuda)
    bufs, _, _, _ = q.run(xyz, torch.from_numpy(sc["raydir"]).to(cuda), torch.from_numpy(sc["campos"]).to(cuda),
                          torch.from_numpy(sc["camrot"]).to(cuda), 2.0, 6.0)
    K, N = sc["opt"].K, xyz.shape[0]
    used_buf, used_map = used_points_device(bufs, K, N)
    c = bufs.read_counts()
    u_ref, m_ref = used_points(bufs.pidx[: c["S_filled"] * K], N)
    assert c["n_used"] == u_ref.numel() > 100
    assert torch.equal(used_buf[: c["n_used"]], u_ref)
    assert torch.equal(used_map, m_ref)


@pytest.mark.parametrize("n_points", [1, 33, 100_003])
def test_used_points_ragged(cuda, n_points):
    """pnr_used_points (byte marks packed to one bit per point, word popcount ranks) on synthetic rows:
    point counts that are not a multiple of 32, empty (-1) slots, a device row
    count below the capacity and none (cap rows), vs train.used_points."""
    from pointnerf_amd import _lib as L
    from pointnerf_amd.train import used_points
    g = torch.Generator().manual_seed(n_points)
    K, cap = 8, 4000
    pidx = torch.randint(-1, n_points, (cap * K,), generator=g, dtype=torch.int32)
    pidx[torch.rand(cap * K, generator=g) < 0.5] = -1
    pidx = pidx.to(cuda)
    i32 = dict(dtype=torch.int32, device=cuda)
    nb = L.c_size_t(0)
    L.check(L.lib().pnr_used_points_scratch_bytes(n_points, L.ctypes.byref(nb)), "scratch")
    for n_rows in (None, 1234):
        flags, used_map, used = (torch.full((n_points,), 7, **i32) for _ in range(3))
        scratch = torch.empty(int(nb.value), dtype=torch.uint8, device=cuda)
        cnt = torch.zeros(2, **i32)
        if n_rows is not None:
            cnt[0] = n_rows
        L.check(L.lib().pnr_used_points(L.ptr(pidx), L.ptr(cnt) if n_rows is not None else None, K, cap, n_points,
                                        L.ptr(flags), L.ptr(used_map), L.ptr(used),
                                        L.c_void_p(cnt.data_ptr() + 4), L.ptr(scratch), scratch.numel(),
                                        L.stream_ptr(cuda)), "pnr_used_points")
        torch.cuda.synchronize()
        u_ref, m_ref = used_points(pidx[: (n_rows or cap) * K], n_points)
        assert int(cnt[1]) == u_ref.numel()
        assert torch.equal(used[: u_ref.numel()], u_ref)
        assert torch.equal(used_map, m_ref)


@pytest.mark.parametrize("case", ["inside", "crossing", "shifted"])
def test_device_geometry_equals_host(cuda, case):
    """pnr_grid_build_dev (get_hyperparameters on the device, no host read of the
    bbox) gives the host formula's shift / dims bits and the same tables and query
    as the host-geometry build -- for a cloud inside the ranges, one crossing
    them (clipped) and one in a corner (dims well below the allocation bound)."""
    from types import SimpleNamespace
    sc = scene(20000, H=24, W=24, theta=70.0)
    xyz = sc["xyz"].copy()
    if case == "crossing":
        xyz[::7] *= 1.6
    elif case == "shifted":
        xyz = (xyz * 0.4 + np.array([0.35, 0.6, 0.6], np.float32)).astype(np.float32)
    sc["xyz"] = xyz
    q_dev = _engine(sc, cuda)
    opt_host = SimpleNamespace(**{**vars(sc["opt"]), "grid_host_bbox": True})
    from pointnerf_amd.querier import lighting_fast_querier
    q_host = lighting_fast_querier(cuda, opt_host)
    t = torch.from_numpy(xyz).to(cuda)
    hp_d = q_dev.grid.build(sc["opt"], t)
    assert type(hp_d).__name__ == "GridHP"
    hp_h = q_host.grid.build(opt_host, t)
    g = O.grid_build(sc["opt"], xyz)
    for k in ("shift", "dims", "ranges"):
        assert np.array_equal(np.asarray(hp_d[k]), np.asarray(hp_h[k])), k
        assert np.array_equal(np.asarray(hp_d[k]), np.asarray(g["hp"][k])), k
    td, th = q_dev.grid.export(), q_host.grid.export()
    for k in td:
        assert torch.equal(td[k], th[k]), k
    _, od = _run(sc, cuda, q_dev)
    _, oh = _run(sc, cuda, q_host)
    for a, b in zip(od[:5], oh[:5]):
        assert torch.equal(a, b)


def test_grid_hp_tied_to_its_build_not_to_point_edits(cuda):
    """GridHP's lazy geometry read after an in-place point edit
    (no rebuild) returns the geometry of the grid that exists; after a rebuild
    an unread entry of the old dict raises."""
    from pointnerf_amd._lib import PnrError
    sc = scene(20000, H=24, W=24, theta=70.0)
    t = torch.from_numpy(sc["xyz"]).to(cuda)
    q = _engine(sc, cuda)
    hp = q.grid.build(sc["opt"], t)
    want = O.grid_build(sc["opt"], sc["xyz"])["hp"]
    with torch.no_grad():
        t.mul_(1.01)                     # in place, no rebuild
    for k in ("shift", "dims"):
        assert np.array_equal(np.asarray(hp[k]), np.asarray(want[k])), k
    hp2 = q.grid.build(sc["opt"], t)     # the version changed: a rebuild, hp2 unread
    assert type(hp2).__name__ == "GridHP"
    q.grid.build(sc["opt"], t, force=True)
    with pytest.raises(PnrError):
        hp2["shift"]


def test_device_grid_cell_budget_takes_host_path(cuda):
    """the sync-free device build sizes its tables for the whole
    opt.ranges box; a box over opt.grid_dev_max_cells builds on the host-read
    bbox instead (tables of the cloud's extent) with the same tables and
    query, and stats() reports the table size of each build."""
    from types import SimpleNamespace
    from pointnerf_amd.querier import lighting_fast_querier
    sc = scene(20000, H=24, W=24, theta=70.0)
    t = torch.from_numpy(sc["xyz"]).to(cuda)
    q_dev = _engine(sc, cuda)
    hp_d = q_dev.grid.build(sc["opt"], t)
    st_d = q_dev.grid.stats()
    assert type(hp_d).__name__ == "GridHP" and st_d["device_geometry"]
    small = SimpleNamespace(**{**vars(sc["opt"]), "grid_dev_max_cells": 1000})
    q_b = lighting_fast_querier(cuda, small)
    hp_b = q_b.grid.build(small, t)
    st_b = q_b.grid.stats()
    assert isinstance(hp_b, dict) and type(hp_b).__name__ == "dict" and not st_b["device_geometry"]
    assert st_b["table_cells"] == int(np.prod(hp_b["dims"].astype(np.int64))) <= st_d["table_cells"]
    assert st_b["table_bytes_est"] > 0
    for k in ("shift", "dims", "ranges"):
        assert np.array_equal(np.asarray(hp_d[k]), np.asarray(hp_b[k])), k
    td, tb = q_dev.grid.export(), q_b.grid.export()
    for k in td:
        assert torch.equal(td[k], tb[k]), k
