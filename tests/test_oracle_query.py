"""The query oracle (oracle/query_ref.c) against an independent brute-force
statement of the reference semantics (qpiw.py:243-528).  The reference query
cannot run here (pycuda CUDA text), so these properties pin the restatement."""
import numpy as np

from oracle import oracle as O
from scenes import scene


def _q(sc, **kw):
    return O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0, **kw)


def test_knn_equals_bruteforce_sets():
    sc = scene(6000, H=24, W=24, theta=75.0)
    q = _q(sc)
    g = q["grid"]
    filled = q["n_filled"] > 0
    loc, pid = [], []
    rp = O.raypos(sc["campos"], sc["raydir"], q["mid_t"])
    for r in np.nonzero(filled)[0][:150]:
        for s in range(q["n_filled"][r]):
            loc.append(rp[r, q["slot_d"][r, s]])
            pid.append(q["pidx_dense"][r, s])
    bf = O.knn_bruteforce(sc["xyz"], np.array(loc), g["hp"], sc["opt"], g)
    checked = 0
    for want, got in zip(bf, pid):
        got = got[got >= 0]
        k = min(len(want), sc["opt"].K)
        assert len(got) == k
        wd = sorted(d for d, _ in want)[:k]
        gd = sorted(float(np.sum((sc["xyz"][i] - loc[checked]) ** 2, dtype=np.float64)) for i in got)
        np.testing.assert_allclose(gd, wd, rtol=1e-5, atol=1e-12)
        checked += 1
    assert checked > 100


def test_neighbours_within_radius():
    sc = scene(8000, H=20, W=20)
    q = _q(sc)
    r2 = float(q["grid"]["hp"]["radius_limit2"])
    p = q["sample_pidx"]
    m = p >= 0
    d = sc["xyz"][p[m]] - np.repeat(q["sample_loc_w"][..., None, :], sc["opt"].K, -2)[m]
    assert np.all((d.astype(np.float32) ** 2).sum(-1) <= r2 * (1 + 1e-5))


def test_march_picks_first_sr_occupied_candidates():
    sc = scene(8000, H=16, W=16, SR=6)
    q = _q(sc)
    g = q["grid"]
    hp = g["hp"]
    rp = O.raypos(sc["campos"], sc["raydir"], q["mid_t"])
    c = np.floor((rp - hp["shift"]) / hp["vsize_s"]).astype(np.int64)
    dims = hp["dims"]
    inside = np.all((c >= 0) & (c < dims), -1)
    flat = (c[..., 0] * dims[1] + c[..., 1]) * dims[2] + c[..., 2]
    occ = np.zeros(inside.shape, bool)
    occ[inside] = g["coor_occ"][flat[inside]] > 0
    for r in range(rp.shape[0]):
        want = np.nonzero(occ[r])[0][:6]
        assert q["n_filled"][r] == len(want)
        assert np.array_equal(q["slot_d"][r, :len(want)], want)


def test_grid_slots_follow_first_point_order_and_slot0_quirk():
    sc = scene(3000)
    for drop in (1, 0):
        sc["opt"].slot0_drop = drop
        g = O.grid_build(sc["opt"], sc["xyz"])
        hp = g["hp"]
        c = np.floor((sc["xyz"] - hp["shift"]) / hp["vsize_s"]).astype(np.int64)
        dims = hp["dims"]
        flat = (c[:, 0] * dims[1] + c[:, 1]) * dims[2] + c[:, 2]
        flat[~np.all((c >= 0) & (c < dims), 1)] = -1          # out-of-grid points are ignored
        _, first = np.unique(flat, return_index=True)
        first = first[flat[first] >= 0]
        order = flat[np.sort(first)]                    # voxels in first-point order
        assert np.array_equal(g["coor_2_occ"][order], np.arange(len(order)))
        members = [np.nonzero(flat == v)[0] for v in order[:50]]
        for s, mem in enumerate(members):
            got = g["occ_2_pnts"][s][: g["occ_numpnts"][s]]
            if drop and s == 0:
                assert len(got) == 0                     # fill_occ2pnts `voxel_idx > 0` (qpiw.py:372)
            else:
                assert np.array_equal(got, mem[: sc["opt"].P])


def test_dilation_marks_query_neighbourhood():
    sc = scene(500)
    g = O.grid_build(sc["opt"], sc["xyz"])
    dims = g["hp"]["dims"]
    occ = g["coor_occ"].reshape(tuple(dims))
    for v in np.nonzero(g["coor_2_occ"] >= 0)[0][:40]:
        x, y, z = np.unravel_index(v, tuple(dims))
        blk = occ[max(0, x - 1):x + 2, max(0, y - 1):y + 2, max(0, z - 1):z + 2]
        assert blk.all()


def test_single_point_and_no_hits():
    sc = scene(500, H=6, W=6)
    one = sc["xyz"][:1].copy()
    q = O.query_points(sc["opt"], one, sc["campos"], sc["camrot"], sc["raydir"], near=2.0, far=6.0)
    assert q["sample_pidx"].shape[1:] == (80, 8)
    q2 = O.query_points(sc["opt"], sc["xyz"], sc["campos"], sc["camrot"], -sc["raydir"], near=2.0, far=6.0)
    assert q2["sample_pidx"].shape[0] == 0 and q2["ray_mask"].sum() == 0


def _hash32(seed, i):
    """res_hash32 (pnr_common.h / query_ref.c) in Python integers."""
    m = (1 << 64) - 1
    z = (seed ^ (i * 0x9E3779B97F4A7C15)) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    z ^= z >> 31
    return z >> 32


def test_overflow_reservoir_keeps_seeded_subsets():
    """max_o and P overflow (qpiw.py:289-298, 377-384): the reference keeps
    uniform random subsets by reservoir replacement with a time seed; the
    oracle (and libpnr) keep the subsets of smallest seeded key -- the max_o
    voxels of smallest hash32(seed, first point), numbered in first-point
    order, and per voxel the P points of smallest hash32(seed + salt, id),
    ascending -- restated here independently."""
    sc = scene(4000)
    x = sc["xyz"]
    sc["xyz"] = np.concatenate([x, x + np.float32(2e-4), x - np.float32(2e-4)]).astype(np.float32)
    opt = sc["opt"]
    opt.slot0_drop = 0
    opt.P = 2
    base = O.grid_build(opt, sc["xyz"])
    n_vox = base["n_occ"]
    opt.max_o = int(n_vox * 0.6)
    salt = 0x632BE59BD9B4E019
    kept_sets = []
    for seed in (0, 7):
        opt.grid_seed = seed
        g = O.grid_build(opt, sc["xyz"])
        assert g["n_occ"] == n_vox
        hp = g["hp"]
        c = np.floor((sc["xyz"] - hp["shift"]) / hp["vsize_s"]).astype(np.int64)
        dims = hp["dims"]
        flat = (c[:, 0] * dims[1] + c[:, 1]) * dims[2] + c[:, 2]
        flat[~np.all((c >= 0) & (c < dims), 1)] = -1
        _, first = np.unique(flat, return_index=True)
        first = np.sort(first[flat[first] >= 0])
        assert len(first) == n_vox
        vkeys = [(_hash32(seed, int(i)) << 32) | int(i) for i in first]
        thr = sorted(vkeys)[opt.max_o - 1]
        kept = [int(i) for i, k in zip(first, vkeys) if k <= thr]       # first-point order
        assert len(kept) == opt.max_o
        assert np.array_equal(g["coor_2_occ"][flat[kept]], np.arange(opt.max_o))
        assert int((g["coor_2_occ"] >= 0).sum()) == opt.max_o
        over = 0
        for s, f in enumerate(kept[:300]):
            mem = np.nonzero(flat == flat[f])[0]
            assert g["occ_numpnts"][s] == len(mem)                 # the reference's counter: all arrivals
            want = mem if len(mem) <= opt.P else np.sort(
                sorted(mem, key=lambda i: (_hash32(seed + salt, int(i)) << 32) | int(i))[:opt.P])
            over += len(mem) > opt.P
            assert np.array_equal(g["occ_2_pnts"][s][:min(len(mem), opt.P)], want)
        assert over > 10
        kept_sets.append(set(kept))
    assert kept_sets[0] != kept_sets[1]                             # the seed draws the subset
