"""Point-NeRF hot-path benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric "Mray-samples/sec at 800x800, K=8, 2M neural
points"): lego flag set (dev_scripts/w_n360/lego.sh), a seeded synthetic
2,000,000-point lego-like cloud, 800x800 NeRF-synthetic cameras, forward
render.  One step = every GPU renders one full frame's worth of rays through
the whole hot path: voxel-grid build, query, fused gather+MLP aggregation,
composite+fill_invalid; with N > 1 every one of the step's N frames is split
across the ranks in N row bands (band b of frame f on rank (b + f) mod N, so
each rank renders every band once per step), a rank renders its N bands as one
multi-camera ray batch, and one RCCL all-gather of the rendered tiles gives
every rank the step's N frames (weak scaling: per-GPU work is fixed).  A ray-sample is one (ray,
shading-slot) entry of the dense H*W*SR grid the reference materialises
(SURVEY 8(d)); value = all ranks' ray-samples / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FLOP_PER_PAIR = 542_720     # GEMM FLOPs per valid (sample, neighbour) pair
FLOP_PER_SAMPLE = 137_216   # colour-branch GEMM FLOPs per valid sample
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: F32 MFMA dense = vector peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)
HBM_PEAK_GBS = 8000.0
# committed PMC passes (tools/prof_bench.sh -> tools/profile_summary.py) per (config, dtype)
PMC_FILES = {("headline", "fp32"): "r01_fp32_pmc_aggregate.json",
             ("headline", "fp32x3"): "r01_pmc_aggregate_x3.json",
             ("headline", "fp32h2"): "r06_final_pmc_aggregate_h2.json",
             ("c5", "bf16"): "r06_c5_pmc_aggregate_bf16.json",
             ("c4", "fp32h2"): "r06_c4_pmc_aggregate_h2.json"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)   # the driver's own K / W (BENCH_rNN.json)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=tuple(CONFIGS), default="headline",
                    help="workload: headline = BASELINE's metric (lego flags, 2M points, 800x800); c4 = scene101 "
                         "flags, 10M points, 1296x968; c5 = truck flags, 20M points (overflowing max_o and P: "
                         "seeded reservoir), 1920x1080, bf16 table + bf16 MFMA")
    ap.add_argument("--points", type=int, default=None, help="override the config's point count")
    ap.add_argument("--hw", type=int, default=None, help="override H = W (headline config only)")
    ap.add_argument("--grid-rebuild", action="store_true",
                    help="rebuild the voxel grid inside every timed step (default: the grid persists across "
                         "frames, as the points do not change; its build is timed on its own line)")
    ap.add_argument("--no-gather", action="store_true", help="skip the all-gather of rendered rays (N > 1)")
    ap.add_argument("--shard", choices=("frames", "tiles"), default="tiles",
                    help="N > 1 ray batches: tiles (default) = every frame split over the ranks (--tile-layout), "
                         "a rank's N partial frames of the step rendered as ONE multi-camera batch, ONE RCCL "
                         "all-gather assembles the step's N frames on every rank; frames = each rank renders "
                         "whole frames (frame f on rank f mod N, one all-gather of the step's N frames)")
    ap.add_argument("--tile-layout", choices=("bands", "tiles16"), default="bands",
                    help="--shard tiles: bands = N row bands per frame, band b of frame f on rank (b+f) mod N "
                         "(every rank renders every band once per step); tiles16 = interleaved 16x16 tiles")
    ap.add_argument("--per-frame-calls", action="store_true",
                    help="--shard tiles: one render call per partial frame (N calls per step) instead of one "
                         "multi-camera batch (A/B of the per-call cost)")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="diagnostic (single process): do rank 0's share of an N-rank step (N partial frames of "
                         "1/N of the rays, no collective) to project per-rank overheads of the N-GPU run")
    ap.add_argument("--cpu-rays", type=int, default=None,
                    help="rays in the CPU-baseline sample (also the rays of the PSNR-vs-oracle check); "
                         "default 12000 (headline), 3000 (c4, c5)")
    ap.add_argument("--query-stream", choices=("auto", "on", "off"), default="auto",
                    help="on: every frame's query on a second stream, where it overlaps the previous frame's "
                         "aggregate; off: on the launch stream; auto (default): on for the headline, off for c4/c5, "
                         "where the 15-ms KNN beside the bucketed aggregate holds CU slots its small kernels wait "
                         "for (DESIGN.md section 14: c5 879 vs 960 Mray-samples/s)")
    ap.add_argument("--no-query-stream", action="store_true", help="same as --query-stream off")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only, no libpnr: the N-rank launcher, sharding, all-gather and timing with a "
                         "stand-in render (tests/test_bench_launch.py; PNR_DIST_BACKEND defaults to gloo)")
    ap.add_argument("--no-train-line", action="store_true",
                    help="headline run: skip the finetune-step measurement appended to the line ('train')")
    ap.add_argument("--profile-steps", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--train-precision", choices=("fp32h2", "fp32x3", "fp32"), default="fp32h2",
                    help="--mode train: the training forward's per-pair chain (fp32h2 split-f16 MFMA, fp32x3 "
                         "split-bf16 MFMA or native fp32)")
    ap.add_argument("--optimizer", choices=("hip", "torch"), default="hip",
                    help="--mode train: Adam on pnr_adam_step (pointnerf_amd.optim.Adam) or torch's fused Adam")
    ap.add_argument("--mode", choices=("render", "train"), default="render",
                    help="render: the headline forward frame render; train: the per-scene finetune "
                         "step (SURVEY config c3: fwd + bwd + Adam on random ray batches)")
    ap.add_argument("--train-rays", type=int, default=3600, help="rays per train step (random_sample_size 60^2)")
    ap.add_argument("--dtype", choices=("fp32", "fp32x3", "fp32h2", "bf16"), default=None,
                    help="MLP arithmetic: fp32h2 (headline, see below); fp32x3 = the reference's fp32 GEMMs as exact 3-way bf16 splits "
                         "(6 cross products) on v_mfma_f32_32x32x16_bf16, fp32-accurate (error vs an fp64 oracle "
                         "equal to native fp32's); fp32h2 = the same GEMMs as 2-way f16 splits (3 products) on "
                         "v_mfma_f32_32x32x16_f16, fp32-accurate; fp32 = native v_mfma_f32_32x32x2_f32; "
                         "bf16 = bf16 operands "
                         "(SURVEY config c5); default: the config's")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    args.points = args.points or cfg["points"]
    args.H, args.W = (args.hw, args.hw) if (args.hw and args.config == "headline") else (cfg["H"], cfg["W"])
    args.hw = args.H
    args.dtype = args.dtype or cfg["dtype"]
    args.cpu_rays = args.cpu_rays or (12000 if args.config == "headline" else 3000)
    return args


# BASELINE.json configs measured by this script (SURVEY 8(d) "Configs as concrete inputs")
CONFIGS = {
    "headline": dict(flags="lego", points=2_000_000, H=800, W=800, dtype="fp32h2",
                     metric="Mray-samples/sec at 800x800, K=8, 2M neural points; PSNR delta vs ref"),
    "c4": dict(flags="scene101", points=10_000_000, H=968, W=1296, dtype="fp32h2",
               metric="Mray-samples/sec at 1296x968, K=8, 10M neural points (config c4, scene101 flags)"),
    "c5": dict(flags="truck", points=20_000_000, H=1080, W=1920, dtype="bf16", cap=-1, scatter=0.1,
               metric="Mray-samples/sec at 1920x1080, K=8, 20M neural points (config c5, truck flags, bf16)"),
}


def build_scene(args, device):
    from pointnerf_amd import synthetic as S
    from pointnerf_amd.aggregator import PointAggregator
    from pointnerf_amd.options import flagset_opt
    from pointnerf_amd.renderer import NeuralPoints, NeuralPointsRayMarching
    cfg = CONFIGS[args.config]
    opt = flagset_opt(cfg["flags"])
    if cfg["flags"] == "lego":
        pts = S.lego_like_points(args.points, seed=0)
    else:
        pts = S.scene_points(cfg["flags"], args.points, opt, seed=0, cap=cfg.get("cap"),
                             scatter=cfg.get("scatter", 0.0))
    emb, color, dirs, conf = S.point_features(args.points, seed=0, default_conf=opt.default_conf)
    torch.manual_seed(0)
    agg = PointAggregator(opt).to(device).eval()   # random-init weights (xavier, networks.py:163-172)
    # bf16 (config c5): the embedding table itself in bf16 (104 B per point)
    emb_dtype = torch.bfloat16 if getattr(args, "dtype", "fp32h2") == "bf16" else torch.float32
    np_ = NeuralPoints(opt, device, torch.from_numpy(pts), emb, color, dirs, conf, emb_dtype=emb_dtype)
    model = NeuralPointsRayMarching(opt, np_, agg)
    return opt, pts, (emb, color, dirs, conf), agg, model


def cameras(n_frames, H, W, flags="lego"):
    """n_frames views of the config's camera path: the NeRF-synthetic orbit for
    lego, the scene's own views otherwise (synthetic.scene_camera)."""
    from pointnerf_amd import synthetic as S
    cams = []
    for i in range(n_frames):
        if flags == "lego":
            theta = -180.0 + 360.0 * i / max(n_frames, 1)
            campos, camrot = S.camera(theta, -30.0, 4.0)
            f = S.lego_focal(H)
        else:
            campos, camrot = S.scene_camera(flags, i, n_frames)
            W0, _, f0 = S.SCENE_INTRINSICS[flags]
            f = f0 * W / W0
        cams.append((campos, camrot, S.pixel_rays(H, W, f, camrot)))
    return cams


def cgroup_cpu_quota():
    """CPUs the process's cgroup may use (cpu.max quota / period), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except Exception:
        return None


def cpu_threads():
    """Host threads of the CPU baseline: every core the process is allowed --
    its affinity mask (len(os.sched_getaffinity(0))), bounded by the cgroup's
    CPU quota when one is set (threads beyond it are only throttled).
    OMP_NUM_THREADS is not a bound (the box sets it for builds)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    return max(1, min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(args, opt, pts, feats, agg, cam, H, W):
    """The oracle (CPU port of the reference path) on a bounded sample of the
    same workload: grid build once + query/aggregate/composite of a random
    subset of one frame's rays, extrapolated to the frame.  Returns (baseline
    dict, sampled ray indices, the oracle's render of them)."""
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    from oracle import oracle as O
    threads, aff, quota = cpu_threads()
    ctx = threadpool_limits(limits=threads) if threadpool_limits else None
    torch.set_num_threads(threads)
    O.set_threads(threads)
    emb, color, dirs, conf = feats
    points = dict(xyz=pts, emb=emb.numpy(), color=color.numpy(), dir=dirs.numpy(), conf=conf.numpy())
    params = {k: v.detach().cpu().numpy() for k, v in agg.state_dict().items()}
    campos, camrot, rd = cam
    rng = np.random.default_rng(0)
    sel = np.sort(rng.choice(rd.shape[0], size=min(args.cpu_rays, rd.shape[0]), replace=False))
    bg = np.random.default_rng(1).uniform(size=128).astype(np.float32)
    t0 = time.perf_counter()
    grid = O.grid_build(opt, pts)
    t1 = time.perf_counter()
    q = O.query_points(opt, pts, campos, camrot, rd[sel], near=opt.near_plane, far=opt.far_plane, grid=grid)
    ref = O.render(opt, points, params, campos, camrot, rd[sel], bg, q=q)
    t2 = time.perf_counter()
    if ctx is not None:
        ctx.__exit__(None, None, None)
    R = H * W
    t_frame = (t1 - t0) + (t2 - t1) * R / len(sel)
    out = {"value": round(R * opt.SR / t_frame / 1e6, 4), "unit": "Mray-samples/s", "cores": threads,
           "kind": "port",
           "sample": (f"oracle/ (C query: serial grid build + OpenMP ray/sample loops; NumPy fp32 "
                      f"aggregate/composite, BLAS) with {threads} threads (affinity mask {aff} CPUs, cgroup "
                      f"quota {quota if quota else 'none'}, os.cpu_count() = {os.cpu_count()}) on "
                      f"{len(sel)} random rays of one {H}x{W} frame, {args.points} points: grid build "
                      f"{t1 - t0:.2f}s + sample {t2 - t1:.2f}s, extrapolated to the frame "
                      f"({t_frame:.1f}s/frame)")}
    return out, sel, ref


def psnr_db(a, b):
    """10 log10(peak^2 / MSE) with peak = max|b| (the reference values)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    mse = float(np.mean((a - b) ** 2))
    return round(10 * np.log10(float(np.abs(b).max()) ** 2 / max(mse, 1e-300)), 2)


HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s


def executed_roofline(args, stage, launches, avg_agg_s):
    """The aggregate's EXECUTED matrix work against the dense peak of the MFMA
    it runs on: per pair 428 032 fp32 FLOP (block1.0's 224 point columns are
    evaluated once per point, not per pair: 114 688 FLOP x N points), per valid
    sample 137 216; fp32h2 issues 3 f16 products per fp32 MAC (2.5 PF dense
    f16), bf16 one bf16 product, fp32 / fp32x3 reported on their own peak."""
    n = max(launches, 1)
    ex = (stage["pairs"] * 428_032 + stage["valid"] * FLOP_PER_SAMPLE) / n + args.points * 114_688
    mult, peak = {"fp32h2": (3, BF16_MFMA_PEAK_TFLOPS), "bf16": (1, BF16_MFMA_PEAK_TFLOPS),
                  "fp32x3": (6, BF16_MFMA_PEAK_TFLOPS), "fp32": (1, FP32_MFMA_PEAK_TFLOPS)}[args.dtype]
    tf = mult * ex / avg_agg_s / 1e12 if avg_agg_s > 0 else 0.0
    return {"fp32_flops_per_launch": ex, "mfma_products_per_fp32_mac": mult, "achieved": round(tf, 2),
            "peak": peak, "unit": "TFLOP/s", "frac": round(tf / peak, 4)}


@torch.no_grad()
def accuracy_vs_oracle(model, opt, cam, bg, sel, ref):
    """The metric's PSNR half: the GPU render of the CPU-baseline rays against
    the oracle's render of the same rays (same points, weights, cameras)."""
    campos, camrot, rd = cam
    idx = torch.from_numpy(sel).to(rd.device)
    color, _, _, mask = model.render_rays(campos, camrot, rd[idx].contiguous(), opt.near_plane, opt.far_plane, bg)
    got = color.cpu().numpy()
    want = ref["coarse_raycolor"]
    hit = ref["ray_mask"] > 0
    return {"oracle_rays": int(len(sel)), "oracle_rays_hit": int(hit.sum()),
            "ray_mask_equal": bool(np.array_equal(mask.cpu().numpy(), ref["ray_mask"])),
            "psnr_vs_oracle_db": psnr_db(got[hit], want[hit]),
            "max_abs_err_vs_oracle": float(np.abs(got - want).max())}


@torch.no_grad()
def accuracy_vs_x3(model, opt, cam, bg, dtype):
    """Full frame: the headline arithmetic against fp32x3 (exact fp32 products,
    test_gpu_x3.py) on the same frame, outside the timed region."""
    campos, camrot, rd = cam
    ev_a, ev_b = [], []
    a = model.render_rays(campos, camrot, rd, opt.near_plane, opt.far_plane, bg, events=ev_a)
    prec = model.precision
    model.precision = "fp32x3"
    try:
        b = model.render_rays(campos, camrot, rd, opt.near_plane, opt.far_plane, bg, events=ev_b)
    finally:
        model.precision = prec
    torch.cuda.synchronize()
    hit = (b[3] > 0).cpu().numpy()
    x, y = a[0].cpu().numpy(), b[0].cpu().numpy()

    def agg_ms(ev):
        return round(sum(e0.elapsed_time(e1) for name, e0, e1 in ev if name == "aggregate"), 3)
    return {f"psnr_{dtype}_vs_fp32x3_full_frame_db": psnr_db(x[hit], y[hit]),
            f"max_abs_err_{dtype}_vs_fp32x3_full_frame": float(np.abs(x - y).max()),
            "full_frame_rays_hit": int(hit.sum()),
            # the strict-fp32 arithmetic's cost on the same frame (one synchronous render each,
            # P1 inline: not the timed steps' side-stream overlap)
            f"aggregate_ms_{dtype}_same_frame": agg_ms(ev_a), "aggregate_ms_fp32x3_same_frame": agg_ms(ev_b)}


def time_grid_build(model, opt, reps=5):
    """Forced rebuilds of the persistent voxel grid: pnr_grid_build_dev (bbox ->
    get_hyperparameters -> build, all on the device, no host read) timed with
    HIP events on the launch stream ("ms") and as wall time between two
    synchronisations ("wall_ms"), and the build's overflow statistics (seeded
    reservoir)."""
    q = model.neural_points.querier
    xyz = model.neural_points.xyz.detach().contiguous()
    ts, ws = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        q.grid.build(opt, xyz, force=True)
        e1.record()
        torch.cuda.synchronize()
        ws.append((time.perf_counter() - t0) * 1e3)
        ts.append(e0.elapsed_time(e1))
    st = q.grid.stats()
    return {"ms": round(float(np.median(ts)), 3), "wall_ms": round(float(np.median(ws)), 3),
            "host_sync": not isinstance(q.grid.hp, dict) or type(q.grid.hp).__name__ != "GridHP",
            "n_voxels": int(st["n_voxels"]),
            "n_voxels_kept": int(st["n_voxels_kept"]), "n_points_dropped": int(st["n_points_dropped"]),
            "max_o": int(opt.max_o), "P": int(opt.P), "dims": [int(d) for d in st["dims"]],
            "overflow_policy": getattr(opt, "max_o_policy", "reservoir") + " (seeded, grid_seed "
                               f"{int(getattr(opt, 'grid_seed', 0))})"}


def isolated_stage_times(model, opt, frames, bg):
    """Per-stage HIP-event times of the timed steps' frames rendered again with
    every stage on the launch stream (P1 not beside the query), outside the
    timed region: the stage rooflines describe each stage alone (same frames,
    so the same counts), while the headline value includes the side stream's
    overlap."""
    side = model.p1_side_stream
    model.p1_side_stream = False
    per = {}
    try:
        for cam in frames:
            ev = []
            model.render_rays(*cam, opt.near_plane, opt.far_plane, bg, events=ev, sync=False)
            model.finish()
            torch.cuda.synchronize()
            for name, a, b in ev:
                per.setdefault(name, []).append(a.elapsed_time(b))
    finally:
        model.p1_side_stream = side
    return per


def stage_rooflines(args, opt, model, stage, per, launches, grid=None):
    """SURVEY 8(d) compulsory-byte formulas for the memory/latency-bound stages,
    per frame, against HBM peak (informational; the headline roofline is the
    aggregate's).  query = march + KNN + compactions (+ the grid build when
    --grid-rebuild puts it in every step); grid_build = the persistent grid's
    build on its own."""
    n = max(launches, 1)
    dims = model.neural_points.querier.grid.hp["dims"]
    cells = int(np.prod(np.asarray(dims, dtype=np.int64)))
    R = stage["rays"] / n
    S = stage["filled"] / n
    V = stage["valid"] / n
    cand = stage["cand"] / n
    D, C, SR = int(opt.z_depth_dim), 128, int(opt.SR)
    grid_b = args.points * 12 + cells * 4 * 2 + int(opt.max_o) * (int(opt.P) + 4) * 4
    march_b = R * D * 4 + R * 16
    knn_b = S * 27 * 8 + cand * 16
    comp_b = V * (C + 1) * 4 + R * (C + 1 + SR) * 4
    q_b = march_b + knn_b + (grid_b if args.grid_rebuild else 0)
    res = {}
    for name, b in (("query", q_b), ("composite", comp_b)):
        ms = float(np.mean(per.get(name, [0.0])))
        gbs = b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        res[name] = {"bytes": int(b), "ms": round(ms, 3), "achieved_GBs": round(gbs, 1),
                     "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)}
    res["query"]["parts_bytes"] = {"march": int(march_b), "knn": int(knn_b)}
    if args.grid_rebuild:
        res["query"]["parts_bytes"]["grid_build"] = int(grid_b)
    res["query"]["knn_candidates"] = int(cand)
    if grid is not None:
        gbs = grid_b / (grid["ms"] * 1e-3) / 1e9 if grid["ms"] > 0 else 0.0
        res["grid_build"] = {"bytes": int(grid_b), "ms": grid["ms"], "achieved_GBs": round(gbs, 1),
                             "frac_hbm": round(gbs / HBM_PEAK_GBS, 4),
                             "note": "device time of the sync-free build (pnr_grid_build_dev); not inside the "
                                     "timed steps (the points do not move)"}
    return res


# fp32-equivalent MFMA ceilings of the training arithmetic (3 f16 / 6 bf16 products per fp32 MAC)
TRAIN_PEAK_TFLOPS = {"fp32h2": round(2500.0 / 3, 1), "fp32x3": round(2500.0 / 6, 1), "fp32": 157.3}
TRAIN_ARITH = {
    "fp32h2": "forward per-pair chain, colour branch, weight gradients and dX1 on the 2-way f16 split "
              "(v_mfma_f32_32x32x16_f16, 3 products); the per-pair dX chain (k_pairs_bwd) on the exact 3-way bf16 "
              "split (6 products); fp32 accumulation everywhere",
    "fp32x3": "every GEMM on the exact 3-way bf16 split (v_mfma_f32_32x32x16_bf16, 6 products), fp32 accumulation",
    "fp32": "native fp32 MFMA (v_mfma_f32_32x32x2_f32)"}


def run_train(args, device):
    """Finetune step: random batch of pixels of one of
    8 cameras -> query -> aggregate (training forward) -> composite -> MSE on
    the first 3 colour channels vs a synthetic target + 1e-4 x the zero_one loss
    on conf_coefficient (ship.sh) -> backward through the HIP kernels -> Adam on
    points_embeding/color/dir/conf and the aggregator."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    reducer = None
    if world > 1:
        # data-parallel finetune: each rank its own random rays, the
        # DDP-mean gradients (parallel.GradReducer: one flat MLP all_reduce + the
        # touched point rows), the same Adam step on every rank
        import torch.distributed as dist
        backend = os.environ.get("PNR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    opt, pts, feats, agg, model = build_scene(args, device)
    agg.train()
    model.train_precision = args.train_precision
    if world > 1:
        from pointnerf_amd.parallel import GradReducer
        npt = model.neural_points
        reducer = GradReducer(list(agg.parameters()),
                              [npt.points_embeding, npt.points_color, npt.points_dir, npt.points_conf, npt.xyz])
    H = W = args.hw
    cams = cameras(8, H, W)
    dev_cams = [tuple(torch.from_numpy(x).to(device) for x in c) for c in cams]
    bg = torch.from_numpy(np.random.default_rng(1).uniform(size=128).astype(np.float32)).to(device)
    target = torch.rand((H * W, 3), generator=torch.Generator().manual_seed(2)).to(device)
    params = [p for p in model.parameters() if p.requires_grad]
    if args.optimizer == "hip":
        from pointnerf_amd.optim import Adam
        optim = Adam(params, lr=5e-4)
    else:
        optim = torch.optim.Adam(params, lr=5e-4, fused=True)
    gen = torch.Generator(device=device).manual_seed(rank)
    stats = {"pairs": 0, "valid": 0, "filled": 0}
    host_ms = {"forward": 0.0, "loss": 0.0, "backward": 0.0, "optimizer": 0.0}   # host time per phase (timed steps)

    def step(i, timed):
        campos, camrot, rd = dev_cams[i % len(dev_cams)]
        t0 = time.perf_counter()
        sel = torch.randint(0, H * W, (args.train_rays,), generator=gen, device=device)
        optim.zero_grad(set_to_none=True)
        color, _, _, _ = model.render_rays_train(campos, camrot, rd[sel], opt.near_plane, opt.far_plane, bg)
        t1 = time.perf_counter()
        loss = torch.mean((color[:, :3] - target[sel]) ** 2)
        if "conf_coefficient" in model.last_train_aux:   # ship.sh: zero_one_loss_weights 1e-4
            loss = loss + 1e-4 * model.zero_one_conf_loss()
        t2 = time.perf_counter()
        loss.backward()
        if reducer is not None:
            reducer.reduce(model.last_train_aux["touched_rows"], model.last_train_aux["touched_count"])
        t3 = time.perf_counter()
        optim.step()
        if timed:
            t4 = time.perf_counter()
            for k, d in zip(host_ms, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                host_ms[k] += d * 1e3
            c = model.last_counts
            stats["pairs"] += c["n_pairs"]
            stats["valid"] += c["S_valid"]
            stats["filled"] += c["S_filled"]

    for i in range(args.warmup):
        step(i, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, True)
    t_issue = time.perf_counter() - t0   # host time to issue the steps (the GPU may still be working)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt)
        st = torch.tensor([stats["pairs"], stats["valid"], stats["filled"]], dtype=torch.float64, device=device)
        dist.all_reduce(st)
        stats = {"pairs": int(st[0]), "valid": int(st[1]), "filled": int(st[2])}
        if rank != 0:
            dist.destroy_process_group()
            return
    k = max(args.steps, 1)
    flops = 3.0 * (stats["pairs"] * FLOP_PER_PAIR + stats["valid"] * FLOP_PER_SAMPLE) / k  # fwd + 2x bwd GEMMs
    ms = t / k * 1e3
    tf = flops / (ms * 1e-3) / 1e12
    peak = TRAIN_PEAK_TFLOPS[args.train_precision]
    line = {
        "metric": "train steps/s (fwd+bwd+Adam, 3600-ray batches), 2M neural points",
        "value": round(1e3 / ms, 3), "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.train_precision, "arith": TRAIN_ARITH[args.train_precision],
        "train_forward": args.train_precision, "h2_fallbacks": int(model.h2_fallbacks),
        "optimizer": "pnr_adam_step" if args.optimizer == "hip" else "torch.optim.Adam(fused=True)",
        "data": "synthetic (seeded lego-like point cloud, random target colours)",
        "config": {"workload": f"finetune step, {args.train_rays} random rays of {H}x{W} frames, {args.points} points",
                   "K": opt.K, "SR": opt.SR},
        "ray_samples_per_s_M": round(world * args.train_rays * opt.SR / (ms * 1e-3) / 1e6, 3),
        "parallelism": (f"dp{world}: {args.train_rays} rays per rank per step, DDP-mean gradients "
                        f"(one flat MLP all_reduce + touched point rows all_gather)" if world > 1 else "single GPU"),
        "gemm_tflops_per_s": round(tf, 3),
        "roofline": {"bound": "mfma", "achieved": round(tf, 3), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(tf / peak, 4),
                     "note": "whole step (fwd + bwd + Adam + query) against the MLP GEMM work only: 3 x (542 720 "
                             "FLOP per valid pair + 137 216 per valid sample) per step (forward, data and weight "
                             "gradients); peak = the fp32-equivalent ceiling of the split arithmetic"},
        "counts_per_step": {k2: v // k for k2, v in stats.items()},
        # host time per step spent issuing (no device sync inside a step but the query-count
        # read): close to ms_per_step means the step is bound by its launches, not the GPU
        "host_issue_ms_per_step": round(t_issue / k * 1e3, 3),
        "host_phase_ms_per_step": {k2: round(v / k, 3) for k2, v in host_ms.items()}}
    if world > 1:
        dist.destroy_process_group()
    return line


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` without torchrun: start N rank processes with
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) BEFORE any GPU
    call in this process (it only parsed its arguments), wait for them, and print
    the ONE JSON line rank 0 wrote, with the launcher recorded in it.  A failing
    rank makes this process exit non-zero with the ranks' output tail."""
    import subprocess
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    env["PNR_BENCH_LAUNCHER"] = "self"
    # the ranks' stderr passes through live (progress); their stdout is captured for the line
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env, cwd=ROOT)
    out, _ = p.communicate()
    lines = []
    for ln in out.splitlines():
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                rec = json.loads(ln)
            except ValueError:
                continue
            if isinstance(rec, dict) and "metric" in rec:
                lines.append(rec)
    if p.returncode != 0 or len(lines) != 1:
        sys.stderr.write(out[-4000:])
        print(f"bench.py launcher: torch.distributed.run with {args.gpus} ranks exited {p.returncode} "
              f"with {len(lines)} result lines", file=sys.stderr)
        return p.returncode or 1
    rec = lines[0]
    rec["launcher"] = (f"bench.py --gpus {args.gpus}: {args.gpus} rank processes via torch.distributed.run "
                       f"(--nnodes=1 --nproc-per-node={args.gpus}, 127.0.0.1), started before any GPU call")
    print(json.dumps(rec), flush=True)
    return 0


def run_dry(args):
    """--dry-run (CPU, no libpnr, no GPU): the N-rank step machinery alone -- the
    launcher, init_process_group, the step's band shares as one batch
    (StepShard), a stand-in 'render' of every ray (a closed-form function of its
    direction), the all-gather that assembles the step's frames, the barrier +
    max-over-ranks timing and rank 0's one line.  Every assembled frame is
    checked against the stand-in render of the whole frame."""
    import torch.distributed as dist
    from pointnerf_amd.parallel import StepShard, TileShard
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(os.environ.get("PNR_DIST_BACKEND", "gloo"))
    if os.environ.get("PNR_BENCH_FAIL_RANK") == str(rank):   # launcher test: a rank that dies
        raise SystemExit(f"rank {rank}: failure injected by PNR_BENCH_FAIL_RANK")
    H = W = min(args.H, 64)
    cams = [torch.from_numpy(c[2]) for c in cameras(8, H, W)]

    def shade(rd):   # [n, 3] -> [n, 4]
        return torch.cat([rd, rd.square().sum(1, keepdim=True)], 1)

    def one_step(s):
        cis = [(s * world + i) % len(cams) for i in range(world)]
        if world == 1:
            return [shade(cams[cis[0]])], cis
        st = StepShard([TileShard(H, W, rank, world, i, None) for i in range(world)], None)
        return st.assemble_async(shade(st.select([cams[c] for c in cis]))).wait(), cis

    ok = True
    for s in range(args.warmup):
        one_step(s)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.steps):
        frames, cis = one_step(args.warmup + s)
        ok &= all(torch.equal(f, shade(cams[c])) for f, c in zip(frames, cis))
    if world > 1:
        dist.barrier()
    t_local = time.perf_counter() - t0
    per_rank = [t_local]
    if world > 1:
        tl = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(tl, torch.tensor([t_local, float(ok)], dtype=torch.float64))
        per_rank = [float(t[0]) for t in tl]
        ok = all(float(t[1]) == 1.0 for t in tl)
    t_max = max(per_rank)
    if rank == 0:
        print(json.dumps({
            "metric": "dry run (no GPU): assembled stand-in frames per second", "value": round(world * args.steps / t_max, 3),
            "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t_max / max(args.steps, 1) * 1e3, 3),
            "ms_per_step_per_rank": [round(t / max(args.steps, 1) * 1e3, 3) for t in per_rank],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "dry_run": True, "frames_equal": bool(ok),
            "rccl_world": dist.get_world_size() if world > 1 else 1,
            "dist_backend": dist.get_backend() if world > 1 else None,
            "config": {"workload": f"stand-in shading of {H}x{W} frames, band shards, one all-gather per step"}}),
            flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's `python bench.py --gpus N`: this process only launches the ranks
        sys.exit(launch_ranks(args))
    if args.dry_run:
        run_dry(args)
        return
    if args.mode == "train":
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        line = run_train(args, torch.device("cuda", local))
        if line is not None:
            print(json.dumps(line), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; the line reports n_gpus={world}",
              file=sys.stderr)
    ndev = torch.cuda.device_count()
    local_dev = local % max(ndev, 1)          # == local on a node with one GPU per rank
    torch.cuda.set_device(local_dev)
    device = torch.device("cuda", local_dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("PNR_DIST_BACKEND", "nccl")   # nccl = RCCL; gloo only for 1-GPU rehearsals
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    from pointnerf_amd import _lib as L

    H, W = args.H, args.W
    cfg = CONFIGS[args.config]
    opt, pts, feats, agg, model = build_scene(args, device)
    model.precision = args.dtype
    cams = cameras(8, H, W, cfg["flags"])
    SR = opt.SR
    # per-(frame, rank) pixel lists: step s renders frames s*world .. s*world+world-1
    shard_world = world if args.shard == "tiles" else 1   # partial frames per rank per step
    if world == 1 and args.emulate_world > 1:
        shard_world = args.emulate_world
    dev_cams = []
    for campos, camrot, rd in cams:
        dev_cams.append((torch.from_numpy(campos).to(device), torch.from_numpy(camrot).to(device),
                         torch.from_numpy(rd).to(device)))
    bg = torch.from_numpy(np.random.default_rng(1).uniform(size=128).astype(np.float32)).to(device)

    from pointnerf_amd.parallel import FrameShard, StepShard, TileShard
    shards = {}
    fshard = FrameShard(rank, world) if (world > 1 and args.shard == "frames") else None

    def my_rays(frame):
        ci = frame % len(cams)
        if shard_world == 1:
            return ci, dev_cams[ci][2], None
        key = (frame % shard_world, ci)
        if key not in shards:
            sh = TileShard(H, W, rank, shard_world, frame % shard_world, device, layout=args.tile_layout)
            shards[key] = (sh, sh.select(dev_cams[ci][2]))
        sh, rd = shards[key]
        return ci, rd, sh

    stage = {"flops": 0.0, "pairs": 0, "valid": 0, "filled": 0, "cand": 0, "rays": 0}
    # frame s + 1's query on its own stream, beside frame s's aggregate (render_rays(query_stream=));
    # --grid-rebuild keeps everything on the launch stream
    use_qs = {"on": True, "off": False, "auto": args.config == "headline"}[args.query_stream]
    qstream = None if (args.no_query_stream or args.grid_rebuild or not use_qs) else torch.cuda.Stream(device)

    steps = {}
    # shader clock under load: one probe wave per timed step on a side stream,
    # beside the step's kernels (pnr_clock_probe, ~10 ms of s_sleep)
    probe = {"stream": torch.cuda.Stream(device), "out": torch.zeros(max(args.steps, 1), device=device), "n": 0}

    def clock_probe():
        if probe["n"] >= probe["out"].numel():
            return
        with torch.cuda.stream(probe["stream"]):
            L.check(L.lib().pnr_clock_probe(L.ptr(probe["out"][probe["n"]:]), 20000, L.stream_ptr(device)),
                    "pnr_clock_probe")
        probe["n"] += 1

    def step_batch(s):
        """tiles mode: this rank's shares of the step's N frames as ONE ray batch
        (per-ray camera index) + the StepShard that assembles them."""
        cis = tuple((s * shard_world + i) % len(cams) for i in range(shard_world))
        if cis not in steps:
            st = StepShard([TileShard(H, W, rank, shard_world, i, device, layout=args.tile_layout)
                            for i in range(shard_world)], device)
            rd = st.select([dev_cams[ci][2] for ci in cis]).contiguous()
            cp = torch.stack([dev_cams[ci][0] for ci in cis])
            cr = torch.stack([dev_cams[ci][1] for ci in cis])
            steps[cis] = (st, rd, cp, cr)
        return steps[cis]

    def issue(s, timed):
        # every render call of the step is issued without a host sync
        # (render_rays(sync=False)); complete() holds the step's one sync; the
        # queries run on qstream (inputs were made before the timed region)
        parts = []
        ev_step = [] if timed else None
        if shard_world > 1 and not args.per_frame_calls:
            st, rd, cp, cr = step_batch(s)
            color = model.render_rays(cp, cr, rd, opt.near_plane, opt.far_plane, bg,
                                      force_grid=args.grid_rebuild, events=ev_step, sync=False,
                                      ray_cam=st.ray_cam, query_stream=qstream)[0]
            parts.append((st, color, rd.shape[0]))
        else:
            for f in range(shard_world):
                frame = s * shard_world + f
                if fshard is not None:
                    frame = fshard.frame_of(s)   # whole frame s*N + rank
                ci, rd, sh = my_rays(frame)
                campos, camrot, _ = dev_cams[ci]
                color = model.render_rays(campos, camrot, rd, opt.near_plane, opt.far_plane, bg,
                                          force_grid=(f == 0 and args.grid_rebuild),
                                          events=ev_step, reuse_p1=f > 0, sync=False, query_stream=qstream)[0]
                parts.append((sh, color, rd.shape[0]))
        if timed:
            clock_probe()
        return parts, ev_step, timed

    def complete(st):
        # model.finish(upto) waits for this step's calls only (the next step's are
        # already queued behind them, so the GPU does not idle while the host
        # checks the deferred feature-buffer sizes / f16 range) and returns the counts
        parts, ev_step, timed = st
        counts = model.finish(upto=len(parts))
        if timed:
            for c, (_, _, nr) in zip(counts, parts):
                stage["pairs"] += c["n_pairs"]
                stage["valid"] += c["S_valid"]
                stage["filled"] += c["S_filled"]
                stage["cand"] += c["n_cand"]
                stage["rays"] += nr
                stage["flops"] += c["n_pairs"] * FLOP_PER_PAIR + c["S_valid"] * FLOP_PER_SAMPLE
            stage["_ev"] = stage.get("_ev", []) + ev_step
            stage["_step_pairs"] = stage.get("_step_pairs", []) + [sum(c["n_pairs"] for c in counts)]
        frames = []
        for sh, color, _ in parts:
            if world > 1 and not args.no_gather:
                # RCCL all-gather of the rendered rays (async: they travel over xGMI while
                # the next step renders): tiles -> one all-gather assembles the step's N
                # frames on every rank; frames -> every rank holds the step's N frames
                frames.append((fshard or sh).assemble_async(color))
            else:
                frames.append(color)
        return frames

    def finish(handles):
        # the step's gathered frames; on RCCL wait() only orders the current
        # stream after the collective, so the host is not blocked
        return [f.wait() if hasattr(f, "wait") else f for f in handles]

    if shard_world > 1 and not args.per_frame_calls:
        for s in range(args.warmup + args.steps):   # ray batches + gather maps built outside the timed region
            step_batch(s)
    def step(s, timed):
        return complete(issue(s, timed))

    for s in range(args.warmup):
        finish(step(s, False))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    rerenders0 = model.overflow_rerenders
    t0 = time.perf_counter()
    prev = []
    pend = issue(args.warmup, True)
    for s in range(1, args.steps + 1):
        nxt = issue(args.warmup + s, True) if s < args.steps else None   # queued before step s-1's sync
        cur = complete(pend)
        finish(prev)   # step s-2's all-gather travelled over xGMI while steps s-1 and s rendered
        prev, pend = cur, nxt
    finish(prev)       # the last step's frames are gathered inside the timed region
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0
    per_rank_s = [t_local]
    if dist:
        dist.barrier()
        tdev = device if dist.get_backend() == "nccl" else "cpu"
        tt = [torch.zeros(1, device=tdev, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(tt, torch.tensor([t_local], device=tdev, dtype=torch.float64))
        per_rank_s = [float(x.item()) for x in tt]
    t_max = max(per_rank_s)
    torch.cuda.synchronize()
    # per-stage times from HIP events recorded on the launch stream
    per = {}
    for name, a, b in stage.get("_ev", []):
        per.setdefault(name, []).append(a.elapsed_time(b))
    agg_ms = per.get("aggregate", [0.0])
    p1_ms = per.get("p1")   # fp32h2: k_point_pre_h2 on the side stream, beside the query
    if p1_ms and len(p1_ms) == len(agg_ms):
        # the roofline keeps timing all three kernels of the aggregate: the side
        # stream's P1 duration is added back to the pairs + colour span
        agg_ms = [a + b for a, b in zip(agg_ms, p1_ms)]
    avg_agg_s = float(np.mean(agg_ms)) / 1e3
    launches = len(agg_ms)
    flops_per_launch = stage["flops"] / max(launches, 1)

    total_samples = H * W * SR * world * args.steps      # every rank renders one frame's worth
    value = total_samples / t_max / 1e6
    if rank == 0:
        # HBM bytes per aggregate launch from the committed PMC passes of this same command
        # (tools/prof_bench.sh -> tools/profile_summary.py; FETCH_SIZE x2 gfx950 correction + WRITE_SIZE)
        traffic = None
        pmc_name = PMC_FILES.get((args.config, args.dtype))
        pmc = os.path.join(ROOT, "profiles", pmc_name or "")
        if pmc_name and os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        achieved = flops_per_launch / avg_agg_s / 1e12 if avg_agg_s > 0 else 0.0
        # fp32x3: every fp32 MAC costs 6 bf16 MFMA products -> fp32-equivalent ceiling = bf16 dense / 6
        # fp32h2: 3 f16 MFMA products per fp32 MAC -> f16 dense (= bf16 dense) / 3
        peak = {"fp32": FP32_MFMA_PEAK_TFLOPS, "fp32x3": round(BF16_MFMA_PEAK_TFLOPS / 6, 1),
                "fp32h2": round(BF16_MFMA_PEAK_TFLOPS / 3, 1), "bf16": BF16_MFMA_PEAK_TFLOPS}[args.dtype]
        out = {
            "metric": cfg["metric"],
            "value": round(value, 3), "unit": "Mray-samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "ms_per_step_per_rank": [round(t / args.steps * 1e3, 3) for t in per_rank_s],
            "rccl_world": dist.get_world_size() if dist else 1,
            "dist_backend": dist.get_backend() if dist else None,
            "dtype": args.dtype,
            "arith": {"fp32": "fp32 MFMA (v_mfma_f32_32x32x2_f32)",
                      "fp32x3": "fp32-accurate: exact 3-way bf16 split of each fp32 operand, 6 cross products on "
                                "v_mfma_f32_32x32x16_bf16, fp32 accumulation (error vs an fp64 oracle = native "
                                "fp32's, tests/test_gpu_x3.py)",
                      "fp32h2": "fp32-accurate: 2-way f16 split of each fp32 operand (x = xh + 2^-11 xl), 3 "
                                "products on v_mfma_f32_32x32x16_f16, fp32 accumulation (error vs an fp64 oracle "
                                "~ native fp32's, tests/test_gpu_x3.py)",
                      "bf16": "bf16 operands, fp32 accumulation"}[args.dtype],
            "data": (f"synthetic (seeded {cfg['flags']}-like {args.points / 1e6:g}M-point cloud, random-init "
                     f"{cfg['flags']} viewmlp weights)"),
            "config": {"workload": f"{cfg['flags']} {W}x{H} forward render, K={opt.K}, SR={SR}, {args.points} points"
                                   + ("" if args.config == "headline" else f" (BASELINE config {args.config})"),
                       "points": args.points, "H": H, "W": W, "K": opt.K, "SR": SR, "P": opt.P,
                       "max_o": int(opt.max_o), "grid_rebuild_per_step": bool(args.grid_rebuild),
                       "query_stream": qstream is not None,
                       "point_table_bytes_per_point": model.neural_points.bytes_per_point(),
                       "parallelism": (f"dp{world} (whole-frame ray batches, async RCCL all_gather of the "
                                       f"step's frames)" if args.shard == "frames" else
                                       f"dp{world} ({args.tile_layout} ray shards of every frame, one multi-camera "
                                       f"batch per rank per step, async RCCL all_gather of the tiles)")
                       if world > 1 else "single GPU"},
            "roofline": {"bound": "mfma", "kernel": {
                             "fp32": "pnr_aggregate_fwd = k_point_pre + k_pairs + k_color (v_mfma_f32_32x32x2_f32)",
                             "fp32x3": "pnr_aggregate_fwd_x3 = k_point_pre + k_pairs_x3 (bf16x3 split, "
                                       "v_mfma_f32_32x32x16_bf16) + k_color",
                             "fp32h2": "pnr_aggregate_fwd_h2 = k_point_pre_h2 + k_pairs_h2 + k_color_h2 (f16x2 split, "
                                       "v_mfma_f32_32x32x16_f16; k_point_pre_h2 runs on a side stream beside "
                                       "the query, its duration added to the span)",
                             "bf16": "pnr_used_points (k_mark_used, scan, k_used_list) + pnr_aggregate_fwd_bf16 = "
                                     "k_point_pre_b + sample buckets + k_pairs_b<1/2/4/8> with the colour branch "
                                     "fused (v_mfma_f32_32x32x16_bf16)"}[args.dtype],
                         "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                         "peak_note": {"fp32": "fp32 MFMA dense peak",
                                       "fp32x3": "fp32-equivalent: bf16 MFMA dense peak / 6 products per fp32 MAC",
                                       "fp32h2": "fp32-equivalent: f16 MFMA dense peak / 3 products per fp32 MAC",
                                       "bf16": "bf16 MFMA dense peak"}[args.dtype],
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "traffic_source": f"profiles/{pmc_name}" if traffic is not None else None,
                         "flops_per_launch": flops_per_launch, "avg_launch_ms": round(avg_agg_s * 1e3, 3),
                         "executed": executed_roofline(args, stage, launches, avg_agg_s)},
            "stages_ms": {k: round(float(np.mean(v)), 3) for k, v in per.items()},
            "frames_per_s": round(world * args.steps / t_max, 3),
            "rays_per_s_M": round(H * W * world * args.steps / t_max / 1e6, 3),
            "counts_per_frame": {"valid_pairs": stage["pairs"] // max(launches, 1),
                                 "valid_samples": stage["valid"] // max(launches, 1),
                                 "filled_samples": stage["filled"] // max(launches, 1)},
        }
        if args.dtype == "fp32h2":
            # frames re-rendered on fp32x3 because an activation left the f16 range
            # (renderer.render_rays; 0 for these weights)
            out["h2_fallbacks"] = int(model.h2_fallbacks)
        # sync-free render calls re-rendered because their valid samples outgrew the
        # feature buffer sized from earlier frames (renderer.finish; 0 after warm-up)
        out["overflow_rerenders"] = int(model.overflow_rerenders - rerenders0)
        if shard_world != world:
            out["config"]["emulated_world"] = shard_world   # diagnostic: rank 0's share of an N-rank step
        # the shader clock the step's kernels ran at (pnr_clock_probe beside them)
        clk = probe["out"][:probe["n"]].cpu().numpy()
        clk = clk[clk > 0]
        out["sclk_mhz_in_run"] = round(float(np.median(clk)), 1) if len(clk) else None
        # per timed step: its frame's camera, valid pairs, aggregate span and probed
        # clock -- the bench cycles 8 cameras whose views differ in pair count, so a
        # K-step mean depends on which cameras the K steps cover
        sp = stage.get("_step_pairs", [])
        if shard_world == 1 and len(sp) == len(agg_ms):
            out["per_step"] = {"camera": [(args.warmup + i) % len(cams) for i in range(len(sp))],
                               "valid_pairs": [int(x) for x in sp],
                               "aggregate_ms": [round(float(x), 3) for x in agg_ms],
                               "sclk_mhz": [round(float(x), 1) for x in probe["out"][:probe["n"]].cpu().numpy()],
                               "ns_per_kpair": [round(float(a) * 1e6 / max(int(p), 1) * 1e3, 4)
                                                for a, p in zip(agg_ms, sp)]}
            r = np.array(agg_ms)
            out["per_step"]["aggregate_spread"] = {"min": round(float(r.min()), 3), "max": round(float(r.max()), 3),
                                                   "cv": round(float(r.std() / r.mean()), 4)}
        # the voxel grid persists across frames (the points do not change); its
        # build (bbox read + 8 kernels + scans) on its own line
        out["grid_build"] = time_grid_build(model, opt)
        per_stage = per
        if "p1" in per and shard_world == 1:
            # the timed steps ran P1 beside the query: their frames again, stages alone, for the stage rooflines
            per_stage = isolated_stage_times(model, opt, [dev_cams[(args.warmup + i) % len(dev_cams)]
                                                          for i in range(args.steps)], bg)
            out["stages_ms_isolated"] = {k: [round(float(x), 3) for x in v] for k, v in per_stage.items()}
        out["stage_rooflines"] = stage_rooflines(args, opt, model, stage, per_stage, launches, out["grid_build"])
        acc = {}
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"], sel, ref = cpu_baseline(args, opt, pts, feats, agg, cams[0], H, W)
                acc.update(accuracy_vs_oracle(model, opt, dev_cams[0], bg, sel, ref))
            except Exception as e:  # the baseline must never hide the GPU number
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        if world == 1 and args.dtype in ("fp32h2", "bf16"):
            acc.update(accuracy_vs_x3(model, opt, dev_cams[0], bg, args.dtype))
        out["accuracy"] = acc
        if world == 1 and args.config == "headline" and not args.no_train_line:
            # SURVEY config c3's finetune step on the same box, outside the timed region
            # (the line `bench.py --mode train` prints, with its own roofline)
            del model, agg
            torch.cuda.empty_cache()
            try:
                out["train"] = train_summary(args, device)
            except Exception as e:  # the render line must never be lost to the training extra
                out["train"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def train_summary(args, device):
    """The finetune step (--mode train, default flags) measured after the render
    line: 20 timed steps after 5 warm-up steps, same points and box."""
    import copy
    targs = copy.copy(args)
    targs.mode, targs.steps, targs.warmup, targs.dtype = "train", 20, 5, "fp32"
    line = run_train(targs, device)
    keep = ("value", "unit", "ms_per_step", "dtype", "arith", "roofline", "h2_fallbacks", "optimizer", "config",
            "counts_per_step", "gemm_tflops_per_s", "host_issue_ms_per_step", "host_phase_ms_per_step")
    return {"train_ms_per_step": line["ms_per_step"], **{k: line[k] for k in keep}}


if __name__ == "__main__":
    main()
