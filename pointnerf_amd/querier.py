"""Drop-in world-coordinate querier backed by libpnr.so.

Mirrors ``lighting_fast_querier`` of
models/neural_points/query_point_indices_worldcoords.py:31-110 (same class
name, constructor, ``query_points`` signature, argument meaning and outputs)
so ``NeuralPoints.__init__`` (neural_points.py:330-331) can select it with
``--wcoord_query 1``.  Differences, all documented in DESIGN.md:
  * the voxel grid is persistent: rebuilt only when the point tensor changes
    (the reference rebuilds it for every ray chunk, qpiw.py:626);
  * slot assignment is deterministic (serial order of claim_occ); max_o / P
    overflow keeps the same uniform random subsets as the reference's
    reservoir replacement, drawn from a seeded hash (opt.grid_seed) instead of
    curand(time()) (qpiw.py:289-298, 377-384); opt.max_o_policy = "grow"
    raises max_o to the occupied-voxel count instead;
  * no pycuda context: everything runs on torch's current HIP stream.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def ray_mid_t(near: float, far: float, D: int, R: int = 1, jitter: float = 0.0,
              device=None, generator=None) -> torch.Tensor:
    """middle_point_ts of near_far_linear_ray_generation
    (models/rendering/diff_ray_marching.py:369-385), [R, D] fp32.  The same
    torch expressions as the reference, so linspace/cumsum round identically;
    evaluated on the CPU for the shared eval table (jitter 0), on the device
    for per-ray jittered tables."""
    dev = torch.device("cpu") if jitter == 0 else device
    tvals = torch.linspace(0, 1, D + 1, device=dev).view(1, -1)
    tvals = near * (1 - tvals) + far * tvals
    rand = torch.rand((1, R, D), device=dev, generator=generator)
    seg = (tvals[..., 1:] - tvals[..., :-1]) * (1 + jitter * (rand - 0.5))
    end = torch.cumsum(seg, dim=2)
    end = torch.cat([torch.zeros((1, R, 1), device=dev), end], dim=2)
    end = near + end
    mid = (end[:, :, :-1] + end[:, :, 1:]) / 2
    return mid[0].to(device) if device is not None else mid[0]


def hyperparameters_from_bbox(opt, min_xyz: np.ndarray, max_xyz: np.ndarray):
    """get_hyperparameters (qpiw.py:48-81) given the exact point bbox; the
    same numpy/torch dtype promotions as the reference."""
    vsize_np = opt.vsize
    vscale_np = np.array(opt.vscale, dtype=np.int32)
    scaled_vsize_np = (vsize_np * vscale_np).astype(np.float32)
    ranges = opt.ranges
    if ranges is not None and ranges[0] >= ranges[3]:
        ranges = None
    min_xyz = np.asarray(min_xyz, np.float32)
    max_xyz = np.asarray(max_xyz, np.float32)
    if ranges is not None:
        min_xyz = np.maximum(min_xyz, np.asarray(ranges[:3], dtype=np.float32))
        max_xyz = np.minimum(max_xyz, np.asarray(ranges[3:], dtype=np.float32))
    pad = (scaled_vsize_np * opt.kernel_size / 2).astype(np.float32)
    min_xyz = (min_xyz - pad).astype(np.float32)
    max_xyz = (max_xyz + pad).astype(np.float32)
    ranges_np = np.concatenate([min_xyz, max_xyz]).astype(np.float32)
    vdim_np = (max_xyz - min_xyz) / vsize_np
    scaled_vdim_np = np.ceil(vdim_np / vscale_np).astype(np.int32)
    radius_limit_np = np.asarray(opt.radius_limit_scale * max(vsize_np[0], vsize_np[1])).astype(np.float32)
    depth_limit_np = np.asarray(opt.depth_limit_scale * vsize_np[2]).astype(np.float32)
    return dict(ranges=ranges_np, shift=ranges_np[:3].copy(), vsize_s=scaled_vsize_np,
                dims=scaled_vdim_np, radius_limit=radius_limit_np, depth_limit=depth_limit_np,
                radius_limit2=np.float32(radius_limit_np ** 2), vsize=vsize_np, vscale=vscale_np)


class GridHP(dict):
    """get_hyperparameters' dict for a grid built on the device
    (pnr_grid_build_dev): the point-independent entries are host values, the
    bbox-derived ones (shift, dims, ranges) are read back from the device
    geometry on first access (one wait for the build).  The read is tied to the
    build that made this dict (its generation): after a rebuild of the handle an
    unread entry raises instead of returning the newer geometry.  An in-place
    edit of the points without a rebuild leaves the device geometry the one of
    this build, so the read still returns it.  It is refused while the stream
    is being captured (the wait is a host synchronisation)."""

    def __init__(self, handle, base, gen):
        super().__init__(base)
        self._handle = handle
        self._gen = gen

    def __missing__(self, key):
        if key not in ("shift", "dims", "ranges"):
            raise KeyError(key)
        h = self._handle
        if h.gen != self._gen:
            raise L.PnrError(f"grid hyperparameter {key!r} read after the grid was rebuilt: read it before "
                             "the next build (or use the handle's current hp)")
        if _capturing():
            raise L.PnrError(f"grid hyperparameter {key!r} first read during stream capture: it waits for the "
                             "build (read it once before capturing)")
        sh, vs, dm = (L.c_float * 3)(), (L.c_float * 3)(), (L.c_int32 * 3)()
        L.check(L.lib().pnr_grid_geometry(h.h, sh, vs, dm), "pnr_grid_geometry")
        shift = np.array(list(sh), np.float32)
        dims = np.array(list(dm), np.int32)
        # ranges_np = [min - pad, max + pad]: the min half is the shift; the max half is
        # the clipped bbox max + pad (bbox read once here, off the hot path)
        mx = np.asarray(h.bbox_max(), np.float32)
        ranges = np.asarray(self["opt_ranges"], np.float32)
        mx = (np.minimum(mx, ranges[3:]) + self["pad"]).astype(np.float32)
        self.update(shift=shift, dims=dims, ranges=np.concatenate([shift, mx]).astype(np.float32))
        return dict.__getitem__(self, key)


GRID_BYTES_PER_CELL = 13.5   # cell tables of one build: coor_2_occ, cell_start / cell_end, dilated bytes, bitmaps


def grid_dev_max_cells(opt) -> int:
    """Largest ranges-box grid (cells) the sync-free device build sizes its tables
    for (opt.grid_dev_max_cells, default 2^28 ~ 3.6 GB of tables); bigger boxes
    build on the host-read bbox."""
    return int(getattr(opt, "grid_dev_max_cells", 1 << 28))


def grid_spec(opt):
    """The point-independent half of get_hyperparameters (qpiw.py:48-81) as
    pnr_grid_spec, plus the host dict entries; None when opt.ranges is unset
    (the bbox then decides the extent: host path)."""
    ranges = opt.ranges
    if ranges is None or ranges[0] >= ranges[3]:
        return None, None
    vsize_np = opt.vsize
    vscale_np = np.array(opt.vscale, dtype=np.int32)
    scaled_vsize_np = (vsize_np * vscale_np).astype(np.float32)
    pad = (scaled_vsize_np * opt.kernel_size / 2).astype(np.float32)
    hp_max = hyperparameters_from_bbox(opt, np.asarray(ranges[:3], np.float32), np.asarray(ranges[3:], np.float32))
    sp = L.GridSpec()
    sp.ranges[:] = [float(x) for x in np.asarray(ranges, np.float32)]
    sp.pad[:] = [float(x) for x in pad]
    sp.vsize[:] = [float(x) for x in vsize_np]
    sp.vscale[:] = [int(x) for x in vscale_np]
    sp.vsize_s[:] = [float(x) for x in scaled_vsize_np]
    sp.dims_max[:] = [int(x) for x in hp_max["dims"]]
    sp.query_size[:] = [int(x) for x in opt.query_size]
    sp.max_o, sp.P = int(opt.max_o), int(opt.P)
    sp.slot0_drop = int(getattr(opt, "slot0_drop", 1))
    sp.seed = int(getattr(opt, "grid_seed", 0))
    base = {k: v for k, v in hp_max.items() if k not in ("shift", "dims", "ranges")}
    base.update(pad=pad, opt_ranges=np.asarray(ranges, np.float32))
    return sp, base


class QueryBuffers:
    """Caller-owned device buffers of pnr_query (torch allocations)."""

    def __init__(self, R: int, SR: int, K: int, device):
        i32 = dict(dtype=torch.int32, device=device)
        RS = R * SR
        self.R, self.SR, self.K = R, SR, K
        self.n_filled = torch.empty(max(R, 1), **i32)
        self.slot_d = torch.empty(max(RS, 1), dtype=torch.int16, device=device)
        self.ray_off = torch.empty(R + 1, **i32)
        self.fill_rs = torch.empty(max(RS, 1), **i32)
        self.pidx = torch.empty(max(RS * K, 1), **i32)
        self.valid_off = torch.empty(RS + 1, **i32)
        self.valid_list = torch.empty(max(RS, 1), **i32)
        self.vflag = torch.empty(max(RS, 1), **i32)
        self.ray_vcnt = torch.empty(max(R, 1), **i32)
        self.ray_row = torch.empty(R + 1, **i32)
        self.sample_w = torch.empty(max(RS, 1) * 3, dtype=torch.float32, device=device)
        self.sample_p = torch.empty(max(RS, 1) * 3, dtype=torch.float32, device=device)
        self.counts = torch.zeros(8, **i32)
        nbytes = L.c_size_t(0)
        L.check(L.lib().pnr_query_scratch_bytes(R, SR, L.ctypes.byref(nbytes)), "pnr_query_scratch_bytes")
        self.scratch = torch.empty(max(int(nbytes.value), 16), dtype=torch.uint8, device=device)
        self.c = L.QueryBufs(
            L.ptr(self.n_filled), L.ptr(self.slot_d), L.ptr(self.ray_off), L.ptr(self.fill_rs),
            L.ptr(self.pidx), L.ptr(self.valid_off), L.ptr(self.valid_list), L.ptr(self.vflag),
            L.ptr(self.ray_vcnt), L.ptr(self.ray_row), L.ptr(self.sample_w), L.ptr(self.sample_p),
            L.ptr(self.counts), L.ptr(self.scratch), self.scratch.numel())

    def fits(self, R, SR, K):
        return self.R == R and self.SR == SR and self.K == K

    def read_counts(self):
        """{S_filled, S_valid, R_hit, R_valid, n_pairs, n_cand} (one D2H copy, syncs)."""
        return counts_dict(self.counts.cpu())

    def read_counts_async(self) -> "CountsHandle":
        """The counts as they stand at this point of the stream, copied to pinned
        memory behind an event: .get() waits for that event only, not for the
        work enqueued after it (the training forward never drains the GPU)."""
        return CountsHandle(self.counts)


def counts_dict(c: torch.Tensor) -> dict:
    n_cand = int(c[6:8].view(torch.int64).item())
    c = c.tolist()
    return dict(S_filled=c[0], S_valid=c[1], R_hit=c[2], R_valid=c[3], n_pairs=c[4], n_cand=n_cand,
                n_used=c[5])   # n_used: pnr_used_points' count when the caller put it in counts[5]


class CountsHandle:
    """Pinned copy of a query's counts + the event after it (read_counts_async)."""

    def __init__(self, counts: torch.Tensor):
        self.host = torch.empty(counts.numel(), dtype=counts.dtype, pin_memory=True)
        self.host.copy_(counts, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record()
        self._d = None

    def get(self) -> dict:
        if self._d is None:
            self.event.synchronize()
            self._d = counts_dict(self.host)
        return self._d


# Handles whose owner was garbage-collected.  A finaliser can run at any
# allocation -- inside someone's HIP-graph capture too -- and pnr_destroy's
# hipFree / hipHostFree / hipEventDestroy are illegal there (they invalidate a
# global-mode capture: GPUTEST_r04's RenderGraph failure).  So __del__ never
# calls HIP; the handles are destroyed at the next safe point
# (release_deferred: a handle creation or build, finish(), RenderGraph after
# its capture).
_DEFERRED: list = []
_CAPTURES = [0]   # RenderGraph captures in progress (any stream of this process)


def _capturing() -> bool:
    if _CAPTURES[0]:
        return True
    try:
        return bool(torch.cuda.is_available() and torch.cuda.is_current_stream_capturing())
    except Exception:
        return False


def release_deferred() -> int:
    """Destroy the handles dropped by the garbage collector; a no-op while this
    thread's stream (or a RenderGraph) is capturing.  Returns the number freed."""
    if not _DEFERRED or _capturing():
        return 0
    n = 0
    while _DEFERRED:
        L.lib().pnr_destroy(_DEFERRED.pop())
        n += 1
    return n


class GridHandle:
    """pnr_handle + persistent grid for one point cloud version."""

    def __init__(self, device: torch.device):
        L.require_gpu()
        release_deferred()
        self.device = device
        h = L.c_void_p()
        L.check(L.lib().pnr_create(device.index or 0, L.ctypes.byref(h)), "pnr_create")
        self.h = h
        self.key = None
        self.hp = None
        self.gen = 0

    def close(self):
        """Free the grid now (explicit; refused during stream capture)."""
        if self.h:
            if _capturing():
                raise L.PnrError("GridHandle.close() during stream capture: pnr_destroy frees device memory")
            L.lib().pnr_destroy(self.h)
            self.h = None
        release_deferred()

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            _DEFERRED.append(h)   # no HIP call from a finaliser (see _DEFERRED)
            self.h = None

    def bbox(self, xyz: torch.Tensor):
        out = torch.empty(6, dtype=torch.float32, device=xyz.device)
        L.check(L.lib().pnr_points_bbox(L.ptr(xyz), xyz.shape[0], L.ptr(out), L.stream_ptr(xyz.device)),
                "pnr_points_bbox")
        b = out.cpu().numpy()
        return b[:3], b[3:]

    def bbox_max(self):
        """Max corner of the bbox the last device build derived its geometry from
        (pnr_grid_bbox: waits for the build; GridHP's ranges)."""
        out = (L.c_float * 6)()
        L.check(L.lib().pnr_grid_bbox(self.h, out), "pnr_grid_bbox")
        return np.array(list(out)[3:], np.float32)

    def build(self, opt, xyz: torch.Tensor, force: bool = False):
        """get_hyperparameters + build_occ_vox; skipped when the point tensor is
        unchanged (same storage, same version counter)."""
        xyz = xyz.reshape(-1, 3)
        L.require_gpu(xyz)
        assert xyz.dtype == torch.float32 and xyz.is_contiguous()
        policy = getattr(opt, "max_o_policy", "reservoir")
        if policy not in ("reservoir", "grow"):
            raise L.PnrError(f"max_o_policy {policy!r}: 'reservoir' (the reference's semantics) or 'grow'")
        key = (xyz.data_ptr(), xyz._version, xyz.shape[0], tuple(opt.vsize), tuple(opt.vscale),
               tuple(opt.kernel_size), tuple(opt.query_size), tuple(opt.ranges), opt.max_o, opt.P,
               int(getattr(opt, "slot0_drop", 1)), int(getattr(opt, "grid_seed", 0)), policy)
        if not force and key == self.key:
            return self.hp
        release_deferred()
        self.gen += 1
        sp, base = grid_spec(opt) if policy == "reservoir" else (None, None)
        if sp is not None and int(np.prod(np.asarray(list(sp.dims_max), np.int64))) > grid_dev_max_cells(opt):
            # the device path sizes its tables for the whole ranges box (it does not know the
            # bbox before the build): a room-scale box at a fine voxel size (ScanNet: +-10 m,
            # 0.016 m cells ~ 2G cells ~ 27 GB) takes the host bbox path instead
            sp = None
        if sp is not None and not getattr(opt, "grid_host_bbox", False):
            # no host sync: bbox -> get_hyperparameters -> build, all on the device
            L.check(L.lib().pnr_grid_build_dev(self.h, L.ptr(xyz), xyz.shape[0], L.ctypes.byref(sp),
                                               L.stream_ptr(xyz.device)), "pnr_grid_build_dev")
            self._xyz = xyz
            hp = GridHP(self, base, self.gen)
            self.key, self.hp = key, hp
            self._max_o, self._P = int(sp.max_o), int(opt.P)
            return hp
        mn, mx = self.bbox(xyz)
        hp = hyperparameters_from_bbox(opt, mn, mx)
        gp = L.GridParams()
        gp.shift[:] = [float(x) for x in hp["shift"]]
        gp.vsize[:] = [float(x) for x in hp["vsize_s"]]
        gp.dims[:] = [int(x) for x in hp["dims"]]
        gp.query_size[:] = [int(x) for x in opt.query_size]
        gp.max_o, gp.P = int(opt.max_o), int(opt.P)
        gp.slot0_drop = int(getattr(opt, "slot0_drop", 1))
        gp.seed = int(getattr(opt, "grid_seed", 0))
        L.check(L.lib().pnr_grid_build(self.h, L.ptr(xyz), xyz.shape[0], L.ctypes.byref(gp),
                                       L.stream_ptr(xyz.device)), "pnr_grid_build")
        if policy == "grow" and xyz.shape[0] > gp.max_o:
            # max_o raised to the occupied voxels (one host read of the count, once per
            # point-cloud version): no voxel is dropped, the reservoir only acts on P
            nv = self._stats_raw().n_voxels
            if nv > gp.max_o:
                gp.max_o = int(nv)
                L.check(L.lib().pnr_grid_build(self.h, L.ptr(xyz), xyz.shape[0], L.ctypes.byref(gp),
                                               L.stream_ptr(xyz.device)), "pnr_grid_build")
        self.key, self.hp = key, hp
        self._max_o, self._P = int(gp.max_o), int(opt.P)
        return hp

    def _stats_raw(self):
        s = L.GridStats()
        L.check(L.lib().pnr_grid_stats_get(self.h, L.ctypes.byref(s)), "pnr_grid_stats_get")
        return s

    def stats(self):
        s = self._stats_raw()
        cells = int(np.prod(np.asarray(list(s.dims), np.int64)))
        return dict(n_points_in_grid=s.n_points_in_grid, n_voxels=s.n_voxels,
                    n_voxels_kept=s.n_voxels_kept, n_points_dropped=s.n_points_dropped,
                    max_points_per_voxel=s.max_points_per_voxel, dims=list(s.dims),
                    table_cells=cells, table_bytes_est=int(cells * GRID_BYTES_PER_CELL),
                    device_geometry=isinstance(self.hp, GridHP))

    def export(self):
        """Grid tables as torch tensors (parity tests / inspection)."""
        hp, dev = self.hp, self.device
        gvol = int(np.prod(hp["dims"].astype(np.int64)))
        max_o, P = self._max_o, self._P
        i32 = dict(dtype=torch.int32, device=dev)
        c2o = torch.empty(gvol, **i32)
        bits = torch.empty((gvol + 31) // 32, **i32)
        npts = torch.empty(max_o, **i32)
        o2p = torch.empty(max_o * P, **i32)
        L.check(L.lib().pnr_grid_export(self.h, L.ptr(c2o), L.ptr(bits), L.ptr(npts), L.ptr(o2p),
                                        L.stream_ptr(dev)), "pnr_grid_export")
        return dict(coor_2_occ=c2o, occ_bits=bits, occ_numpnts=npts, occ_2_pnts=o2p.view(max_o, P))

    def query(self, opt, hp, rays: L.Rays, bufs: QueryBuffers):
        qp = query_params(opt, hp)
        L.check(L.lib().pnr_query(self.h, L.ctypes.byref(rays), L.ctypes.byref(qp),
                                  L.ctypes.byref(bufs.c), L.stream_ptr(self.device)), "pnr_query")
        return qp


def query_params(opt, hp) -> L.QueryParams:
    qp = L.QueryParams()
    qp.SR, qp.K = int(opt.SR), int(opt.K)
    qp.kernel_size[:] = [int(x) for x in opt.kernel_size]
    qp.radius_limit2 = float(hp["radius_limit2"])
    return qp


def make_rays(campos, camrot, raydir, tvals, per_ray: bool, ray_cam=None) -> L.Rays:
    r = L.Rays()
    r.campos_dev, r.camrot_dev = campos.data_ptr(), camrot.data_ptr()
    r.raydir_dev, r.tvals_dev = raydir.data_ptr(), tvals.data_ptr()
    r.R = raydir.shape[0]
    r.D = tvals.shape[-1]
    r.tvals_per_ray = 1 if per_ray else 0
    r.ray_cam = None if ray_cam is None else ray_cam.data_ptr()
    return r


def camera_tables(campos, camrot, ray_cam=None):
    """(campos, camrot) as the kernels read them: [3] / [3,3] for one camera,
    [n_cams,3] / [n_cams,3,3] tables when ray_cam (int32 [R]) picks a camera
    per ray (pnr_rays.ray_cam)."""
    if ray_cam is None:
        return campos.reshape(3).contiguous().float(), camrot.reshape(3, 3).contiguous().float()
    return campos.reshape(-1, 3).contiguous().float(), camrot.reshape(-1, 3, 3).contiguous().float()


class lighting_fast_querier:  # noqa: N801  (reference class name)
    """query_point_indices_worldcoords.lighting_fast_querier on libpnr.so."""

    def __init__(self, device, opt):
        self.device = torch.device(device) if not isinstance(device, torch.device) else device
        if self.device.type != "cuda":
            raise L.PnrError("lighting_fast_querier needs a cuda (ROCm) device")
        self.gpu = self.device.index or 0
        self.opt = opt
        self.inverse = getattr(opt, "inverse", 0)
        if self.inverse:
            raise L.PnrError("--inverse 1 (disparity ray generation) is not supported")
        if getattr(opt, "NN", 2) <= 0:
            raise L.PnrError("NN == 0 needs query_rand_along_ray, which the reference "
                             "module does not define either (qpiw.py:536)")
        self.grid = GridHandle(self.device)
        self._tv_cache = {}
        self.count = 0

    def clean_up(self):
        self.grid.close()

    def get_hyperparameters(self, vsize_np, point_xyz_w_tensor, ranges=None):
        mn, mx = self.grid.bbox(point_xyz_w_tensor.reshape(-1, 3).contiguous())
        o = self.opt
        from types import SimpleNamespace
        o2 = SimpleNamespace(**{**vars(o), "vsize": vsize_np, "ranges": ranges})
        return hyperparameters_from_bbox(o2, mn, mx)

    def tvals(self, near, far, R, device):
        jitter = 0.3 if getattr(self.opt, "is_train", 0) > 0 else 0.0
        D = self.opt.z_depth_dim
        if jitter == 0:
            key = (float(near), float(far), D)
            if key not in self._tv_cache:
                self._tv_cache[key] = ray_mid_t(near, far, D)[0].to(device).contiguous()
            return self._tv_cache[key], False
        return ray_mid_t(near, far, D, R=R, jitter=jitter, device=device).contiguous(), True

    def run(self, point_xyz_w, ray_dirs, cam_pos, cam_rot, near_depth, far_depth, bufs=None, ray_cam=None):
        """Device-side query of one ray batch; returns (bufs, hp, rays, qp).
        ray_cam (int32 [R], optional): camera of each ray, cam_pos / cam_rot
        then being [n_cams,3] / [n_cams,3,3] tables (a multi-frame batch)."""
        xyz = point_xyz_w.reshape(-1, 3).contiguous()
        hp = self.grid.build(self.opt, xyz)
        raydir = ray_dirs.reshape(-1, 3).contiguous().float()
        campos, camrot = camera_tables(cam_pos, cam_rot, ray_cam)
        R = raydir.shape[0]
        tv, per_ray = self.tvals(near_depth, far_depth, R, raydir.device)
        if ray_cam is not None:
            ray_cam = ray_cam.to(torch.int32).contiguous()
            assert ray_cam.shape[0] == R
        rays = make_rays(campos, camrot, raydir, tv, per_ray, ray_cam)
        if bufs is None or not bufs.fits(R, self.opt.SR, self.opt.K):
            bufs = QueryBuffers(R, self.opt.SR, self.opt.K, raydir.device)
        qp = self.grid.query(self.opt, hp, rays, bufs)
        bufs._keep = (raydir, campos, camrot, tv, ray_cam)  # keep alive for the async kernels
        return bufs, hp, rays, qp

    def query_points(self, pixel_idx_tensor, point_xyz_pers_tensor, point_xyz_w_tensor,
                     actual_numpoints_tensor, h, w, intrinsic, near_depth, far_depth,
                     ray_dirs_tensor, cam_pos_tensor, cam_rot_tensor):
        """qpiw.py:84-99.  Returns (sample_pidx [B,R'',SR,K] int32, sample_loc
        [B,R'',SR,3], sample_loc_w [B,R'',SR,3], sample_ray_dirs [B,R'',SR,3],
        ray_mask [B,R] int8, vsize_np, ranges_np).  B must be 1 (as in every
        reference driver)."""
        L.require_gpu(point_xyz_w_tensor)
        if point_xyz_w_tensor.dim() == 3 and point_xyz_w_tensor.shape[0] != 1:
            raise L.PnrError("batch size B > 1 is not supported (the reference uses B = 1)")
        near_depth, far_depth = np.asarray(near_depth).item(), np.asarray(far_depth).item()
        bufs, hp, rays, qp = self.run(point_xyz_w_tensor, ray_dirs_tensor, cam_pos_tensor,
                                      cam_rot_tensor, near_depth, far_depth)
        R, SR, K = bufs.R, self.opt.SR, self.opt.K
        Rv = bufs.read_counts()["R_valid"]
        dev = ray_dirs_tensor.device
        sample_pidx = torch.empty((1, Rv, SR, K), dtype=torch.int32, device=dev)
        sample_loc = torch.empty((1, Rv, SR, 3), dtype=torch.float32, device=dev)
        sample_loc_w = torch.empty((1, Rv, SR, 3), dtype=torch.float32, device=dev)
        sample_ray_dirs = torch.empty((1, Rv, SR, 3), dtype=torch.float32, device=dev)
        ray_mask = torch.empty((1, R), dtype=torch.int8, device=dev)
        L.check(L.lib().pnr_query_compact(L.ctypes.byref(rays), L.ctypes.byref(qp),
                                          L.ctypes.byref(bufs.c), Rv, L.ptr(sample_pidx),
                                          L.ptr(sample_loc), L.ptr(sample_loc_w),
                                          L.ptr(sample_ray_dirs), L.ptr(ray_mask),
                                          L.stream_ptr(dev)), "pnr_query_compact")
        self.count += 1
        return (sample_pidx, sample_loc, sample_loc_w, sample_ray_dirs, ray_mask,
                np.asarray(self.opt.vsize), hp["ranges"])

    def w2pers(self, point_xyz_w, camrotc2w, campos):
        """qpiw.py:102-109 (torch; not on the hot path)."""
        xyz_w_shift = point_xyz_w - campos[:, None, :]
        xyz_c = torch.sum(xyz_w_shift[..., None, :] * torch.transpose(camrotc2w, 1, 2)[:, None, None, ...], dim=-1)
        return torch.stack([xyz_c[..., 0] / xyz_c[..., 2], xyz_c[..., 1] / xyz_c[..., 2], xyz_c[..., 2]], dim=-1)
