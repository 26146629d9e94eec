/*
 * pnr.h — C ABI of the MI355X-native Point-NeRF hot path (libpnr.so).
 *
 * The hot path of yjcaimeow/pointnerf is: world-coordinate voxel-grid KNN
 * query of neural points -> K-neighbour gather + inverse-distance weights ->
 * per-(sample, neighbour) MLP, K-weighted sum, per-sample colour MLP ->
 * ray-march alpha composite (+ fill_invalid).  Every stage below is a
 * hand-written HIP kernel for gfx950; this header is the only boundary.
 *
 * Conventions
 *   - Plain C types only.  Every pointer named *_dev is device memory owned by
 *     the caller (PyTorch tensors in the Python host); the handle owns only the
 *     persistent voxel-grid tables built by pnr_grid_build().
 *   - `stream` is a hipStream_t passed as void* (0 = default stream).  No
 *     function synchronises the stream unless its comment says so.
 *   - Every function returns an int status (PNR_OK, PNR_E*) and never throws.
 *     pnr_last_error() returns a static, thread-local message for the last
 *     failing call.
 *   - Variable-size results are written at their maximum size; the actual
 *     counts stay in device memory (counts_dev) so no host sync is needed.
 *
 * Reference interfaces replaced (file:line in the reference tree):
 *   pnr_points_bbox      <- lighting_fast_querier.get_hyperparameters
 *                           models/neural_points/query_point_indices_worldcoords.py:48-81
 *   pnr_grid_build       <- build_occ_vox + claim_occ/map_coor2occ/fill_occ2pnts
 *                           query_point_indices_worldcoords.py:546-611, 243-387
 *   pnr_query            <- query_grid_point_index (mask_raypos, cumsum SR pick,
 *                           get_shadingloc, query_neigh_along_ray_layered)
 *                           query_point_indices_worldcoords.py:614-721, 390-528
 *   pnr_query_compact    <- the R''-compaction + w2pers tail of query_points
 *                           query_point_indices_worldcoords.py:97-109, 715-719
 *   pnr_aggregate_fwd    <- NeuralPoints.forward gather (neural_points.py:782-812)
 *                           + PointAggregator.forward/viewmlp (agg_intrp_order 2)
 *                           models/aggregators/point_aggregators.py:729-816, 488-646
 *   pnr_composite_fwd    <- ray_dist + ray_march + fill_invalid of
 *                           NeuralPointsRayMarching.forward
 *                           models/neural_points_volumetric_model.py:293-389,
 *                           models/rendering/diff_ray_marching.py:509-555
 *   pnr_ray_march_fwd    <- ray_march on dense [B,R,SR,C+1] features
 *                           models/rendering/diff_ray_marching.py:509-555
 *   pnr_vox_closest      <- construct_vox_points_closest (point-cloud init down-sampling)
 *                           models/mvs/mvs_utils.py:537-561
 *   pnr_rgb_head_fwd/bwd <- the upstream colour head the fork commented out:
 *                           color_branch Linear(128,3) + raw2out_color
 *                           models/aggregators/point_aggregators.py:343, 269-273, 637-638
 *                           (radiance_render [..., 1:4], diff_render_func.py:48-50)
 */
#ifndef PNR_H_
#define PNR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* libpnr.so is built with -fvisibility=hidden: only the declarations below are exported. */
#pragma GCC visibility push(default)

#define PNR_ABI_VERSION 23

enum {
  PNR_OK = 0,
  PNR_EINVAL = 1,     /* bad argument (null pointer, bad size, unsupported config) */
  PNR_EOVERFLOW = 2,  /* a fixed-capacity table overflowed (see pnr_grid_stats) */
  PNR_EHIP = 3,       /* a HIP runtime call failed */
  PNR_ENOMEM = 4      /* device allocation failed */
};

typedef struct pnr_handle pnr_handle;

/* ---------------------------------------------------------------- handle */
int pnr_abi_version(void);
const char* pnr_last_error(void);
/* One handle per (device, point cloud).  Selects `device` for its lifetime. */
int pnr_create(int device, pnr_handle** out);
int pnr_destroy(pnr_handle* h);

/* -------------------------------------------------------------- grid build
 * Exact per-axis min/max of xyz[N,3] into out6_dev = {min xyz, max xyz}.
 * (qpiw.py:58; the reference reads it back with .cpu(), so does the host.) */
int pnr_points_bbox(const float* xyz_dev, int64_t n, float* out6_dev, void* stream);

typedef struct {
  float shift[3];       /* ranges_np[:3]: grid origin (qpiw.py:71)               */
  float vsize[3];       /* scaled_vsize_np = vsize*vscale (qpiw.py:60)            */
  int32_t dims[3];      /* scaled_vdim_np (qpiw.py:75)                            */
  int32_t query_size[3];/* dilation of the occupancy mask (qpiw.py:626, 330-338) */
  int32_t max_o;        /* occupied-voxel capacity (flag --max_o)                 */
  int32_t P;            /* points kept per voxel (flag --P)                       */
  int32_t slot0_drop;   /* 1 = reproduce `voxel_idx > 0` (qpiw.py:372): the voxel
                           given slot 0 keeps no points; 0 = keep them          */
  uint64_t seed;        /* seed of the overflow reservoir (the reference: time()) */
} pnr_grid_params;

/* Build the persistent sparse voxel tables from xyz[N,3] (device, fp32).
 * Deterministic: voxel slots are assigned in ascending order of the first
 * point index that lands in each voxel (the serial order of claim_occ), points
 * inside a voxel are kept in ascending index order.  On overflow -- more
 * occupied voxels than max_o, more points than P in a voxel -- the reference's
 * reservoir replacement (qpiw.py:289-298, 377-384: uniform random subsets, time
 * seed) becomes a seeded one: the max_o voxels with the smallest key
 * hash32(seed, first point) << 32 | first point are kept (slots in first-point
 * order), and a voxel keeps the P points with the smallest key
 * hash32(seed + 0x632BE59BD9B4E019, id) << 32 | id (ascending id); hash32 =
 * splitmix64 finaliser of seed ^ id * 0x9E3779B97F4A7C15, high 32 bits.  Tables
 * are reallocated only when dims/max_o/P grow; grids up to 2^36 cells (int64
 * cell indices).  No host sync: the build counters travel to pinned host memory
 * behind an event that only pnr_grid_stats_get waits on.  Returns PNR_OK on
 * overflow; inspect pnr_grid_stats. */
int pnr_grid_build(pnr_handle* h, const float* xyz_dev, int64_t n,
                   const pnr_grid_params* p, void* stream);

/* pnr_grid_build without a host read of the point bbox (training steps that
 * move xyz, prune / grow: neural_points.py:350-402): get_hyperparameters
 * (qpiw.py:48-81) runs on the device from the bbox -- min/max clipped to
 * ranges and padded in fp32, dims = ceil((max - min) / vsize / vscale) in
 * float64 as numpy promotes it -- so shift and dims equal the host formula's.
 * The tables are allocated for dims_max (the dims of bbox = ranges, an upper
 * bound); ranges must be set (min < max).  pnr_grid_geometry reads the exact
 * shift / cell size / dims back (waits for the build). */
typedef struct {
  float ranges[6];      /* opt.ranges                                           */
  float pad[3];         /* (vsize * vscale * kernel_size / 2) as get_hyperparameters rounds it (fp32) */
  double vsize[3];      /* opt.vsize (Python floats)                            */
  int32_t vscale[3];
  float vsize_s[3];     /* fp32(vsize * vscale): the cell size                  */
  int32_t dims_max[3];  /* dims of the bbox = ranges case                       */
  int32_t query_size[3];
  int32_t max_o;
  int32_t P;
  int32_t slot0_drop;
  uint64_t seed;
} pnr_grid_spec;
int pnr_grid_build_dev(pnr_handle* h, const float* xyz_dev, int64_t n, const pnr_grid_spec* spec, void* stream);
int pnr_grid_geometry(pnr_handle* h, float shift[3], float vsize[3], int32_t dims[3]);
/* The point bbox {min xyz, max xyz} the last pnr_grid_build_dev derived its
 * geometry from (waits for the build; ABI 21): what get_hyperparameters'
 * ranges come from, unaffected by later in-place edits of the points. */
int pnr_grid_bbox(pnr_handle* h, float out6[6]);

typedef struct {
  int64_t n_points_in_grid;   /* points whose voxel is inside dims            */
  int64_t n_voxels;           /* occupied voxels (before max_o truncation)    */
  int64_t n_voxels_kept;      /* min(n_voxels, max_o) (the reservoir's voxels) */
  int64_t n_points_dropped;   /* points of kept voxels beyond P (not in the reservoir) */
  int32_t max_points_per_voxel;
  int32_t dims[3];
} pnr_grid_stats;
int pnr_grid_stats_get(pnr_handle* h, pnr_grid_stats* out); /* waits for the last build */

/* Copy the grid tables out (inspection / parity tests; any pointer may be NULL):
 * coor_2_occ[gvol] (-1 empty), occ_bits[ceil(gvol/32)] dilated occupancy
 * bitmap, occ_numpnts[max_o], occ_2_pnts[max_o*P] point ids (-1 empty). */
int pnr_grid_export(pnr_handle* h, int32_t* coor_2_occ, uint32_t* occ_bits, int32_t* occ_numpnts,
                    int32_t* occ_2_pnts, void* stream);

/* ------------------------------------------------------------------ query
 * Rays: raypos(r,d) = campos + raydir[r] * tvals[d]  (diff_ray_marching.py:387,
 * mul then add, fp32, no contraction).  tvals holds the D mid-point depths
 * middle_point_ts (diff_ray_marching.py:369-385), either one table shared by
 * every ray (tvals_per_ray = 0, jitter = 0) or one row per ray.  Depths ascend
 * along a ray (as middle_point_ts makes them): with a shared table the march
 * tests only the depths inside the grid box, found from the table's order. */
typedef struct {
  const float* campos_dev;    /* [3]  ([n_cams,3] with ray_cam)        */
  const float* camrot_dev;    /* [3,3] row-major camrotc2w ([n_cams,3,3] with ray_cam) */
  const float* raydir_dev;    /* [R,3]                                 */
  const float* tvals_dev;     /* [D] or [R,D]                          */
  int64_t R;
  int32_t D;
  int32_t tvals_per_ray;
  const int32_t* ray_cam;     /* NULL: every ray from the one camera; else [R] camera
                                 index of each ray into campos/camrot: several frames'
                                 (partial) ray batches rendered as ONE batch (one
                                 query / aggregate / composite launch each), e.g. the
                                 N band shares of a multi-GPU step                      */
} pnr_rays;

typedef struct {
  int32_t SR;                 /* shading samples per ray (flag --SR)    */
  int32_t K;                  /* neighbours per sample (flag --K), 1..16 */
  int32_t kernel_size[3];     /* Chebyshev search extent (flag --kernel_size) */
  float radius_limit2;        /* (radius_limit_scale*max(vsize_x,vsize_y))^2, 0 = none */
} pnr_query_params;

/* Caller-owned device buffers of pnr_query; sizes from pnr_query_sizes(). */
typedef struct {
  int32_t* n_filled;    /* [R]      occupied candidates kept per ray (<= SR)          */
  uint16_t* slot_d;     /* [R*SR]   candidate index d of shading slot s (s < n_filled)*/
  int32_t* ray_off;     /* [R+1]    exclusive scan of n_filled                        */
  int32_t* fill_rs;     /* [R*SR]   filled-sample list, entry = r*SR + s              */
  int32_t* pidx;        /* [R*SR*K] neighbour point ids per filled sample, -1 = none  */
  int32_t* valid_off;   /* [R*SR+1] exclusive scan of (sample has >=1 neighbour)      */
  int32_t* valid_list;  /* [R*SR]   filled-sample index of every valid sample         */
  int32_t* vflag;       /* [R*SR]   1 if filled sample has >=1 neighbour              */
  int32_t* ray_vcnt;    /* [R]      valid samples per ray (ray_mask = ray_vcnt > 0)   */
  int32_t* ray_row;     /* [R+1]    exclusive scan of ray_mask: compacted row of ray  */
  float* sample_w;      /* [R*SR*3] world position of each filled sample              */
  float* sample_p;      /* [R*SR*3] camera-perspective (x/z, y/z, z) of each sample   */
  int32_t* counts;      /* [8] {S_filled, S_valid, R_hit(R'), R_valid(R''), n_pairs, 0,
                           n_cand (int64 in [6..7]: KNN candidate records read)};
                           8-byte aligned */
  void* scratch;        /* scan scratch, scratch_bytes from pnr_query_sizes()         */
  size_t scratch_bytes;
} pnr_query_bufs;

int pnr_query_scratch_bytes(int64_t R, int32_t SR, size_t* out);

/* march -> first SR occupied candidates -> filled list -> layered KNN ->
 * valid-sample compaction.  No host sync. */
int pnr_query(pnr_handle* h, const pnr_rays* rays, const pnr_query_params* q,
              pnr_query_bufs* b, void* stream);

/* Reference-shaped outputs of query_points for the first R'' = counts[3] rays
 * with ray_vcnt > 0 (ray order preserved):
 *   sample_pidx[R'',SR,K] (-1), sample_loc[R'',SR,3] (w2pers, unfilled slots =
 *   w2pers(0,0,0)), sample_loc_w[R'',SR,3] (0), sample_ray_dirs[R'',SR,3],
 *   ray_mask[R] int8.  rows_max bounds the outputs' first dimension. */
int pnr_query_compact(const pnr_rays* rays, const pnr_query_params* q,
                      const pnr_query_bufs* b, int64_t rows_max,
                      int32_t* sample_pidx, float* sample_loc, float* sample_loc_w,
                      float* sample_ray_dirs, int8_t* ray_mask, void* stream);

/* -------------------------------------------------------------- aggregate
 * viewmlp with agg_intrp_order 2, agg_distance_kernel linear, agg_dist_pers 20,
 * point_features_dim 32, num_feat_freqs 3, dist_xyz_freq 5, num_viewdir_freqs 4,
 * shading_feature_num 256, block1 x2, block3 x2, alpha x1, colour x3 (C=128).
 * Weights are device fp32 arrays in the MFMA A-operand "fragment" layout
 * produced by pointnerf_amd.aggregator.frag_pack() from the reference
 * nn.Linear [out,in] weight W:  W_f[t][T][lane] = W[32T + (lane&31)][2t + (lane>>5)]
 * for t < ceil(in/2) + 8 (8 trailing zero k-steps: prefetch padding), T < out/32. */
typedef struct {
  const float* w1af;                   /* block1.0 columns 0..223 (embedding + its PE) + bias:
                                          evaluated once per point (pnr_aggregate_fwd step 1) */
  const float* w1bf;                   /* block1.0 columns 224..283 (PE of the 6-d distance)  */
  const float* w2f; const float* b2;   /* block1.2  [256,256]                  */
  const float* w3f; const float* b3;   /* block3.0  [256,263]                  */
  const float* w4f; const float* b4;   /* block3.2  [256,256]                  */
  const float* wa;  const float* ba;   /* alpha_branch.0 [1,256]               */
  const float* wc1f; const float* bc1; /* color_branch.0 [128,280]             */
  const float* wc2f; const float* bc2; /* color_branch.2 [128,128]             */
  const float* wc3f; const float* bc3; /* color_branch.4 [128,128]             */
  const float* rw2c;                   /* [3,3] uniform Rw2c (identity default) */
  float neg_slope;                     /* LeakyReLU slope (0 = ReLU)           */
  int32_t act_super;                   /* 1: softplus(x-1), 0: relu(x)         */
} pnr_mlp;

typedef struct {
  int64_t n;            /* N: rows of every point table                             */
  const float* xyz;     /* [N,3] world xyz (index space of pidx)                   */
  const float* pers;    /* [N,3] perspective xyz, or NULL = w2pers(xyz) on the fly */
  const float* emb;     /* [N,32]                                                   */
  const float* color;   /* [N,3]                                                    */
  const float* dir;     /* [N,3]                                                    */
  const float* conf;    /* [N] or NULL (conf = 1)                                   */
  const float* campos;  /* [3] needed when pers == NULL                             */
  const float* camrot;  /* [3,3] needed when pers == NULL                           */
  const int32_t* used;  /* optional [n_used] point rows the samples reference (NULL = all
                           n rows): block1.0's point half (scratch P1) is then computed
                           for these rows only -- the training-batch case            */
  int64_t n_used;
  const int32_t* used_map; /* [n] row -> index into used (-1 = unreferenced); required
                              with used, except by pnr_aggregate_fwd_bf16: there used
                              without used_map computes P1 for the used rows only but
                              keeps the table indexed by point row ([n,256])         */
  int32_t p1_ready;     /* aggregate forward only: 1 = the scratch's first n_p1*256
                           values already hold block1.0's point half for these same
                           rows and weights (an earlier call on the same scratch with
                           the same emb / used rows / block1.0, e.g. the other ray
                           batches of one step), so the per-point pass is skipped.
                           Camera-independent.  0 = compute it (always safe).     */
  const uint16_t* emb_bf16; /* [N,32] bf16 embedding table (SURVEY config c5: 104 B per
                           point instead of 168), read instead of emb by
                           pnr_aggregate_fwd_bf16 when set (emb may then be NULL);
                           the fp32 paths ignore it                                  */
  const float* rw2c;    /* [N,3,3] per-point Rw2c (neural_points.py:799 gathers it when
                           Rw2c.dim() > 2), or NULL = the uniform pnr_mlp.rw2c.  A pair's
                           world distance and point dir are rotated by its point's
                           matrix, a sample's view dir by the matrix of its slot-0
                           neighbour (point_aggregators.py:492-496, 506, 526, 566)     */
  const int32_t* n_used_dev; /* optional device count of `used` (pnr_used_points writes it):
                           the kernels then take min(n_used, *n_used_dev) rows, n_used
                           being the capacity -- a training forward that never reads
                           the count on the host (ABI 19)                               */
} pnr_points;

typedef struct {
  const int32_t* samp_list;  /* [n_max] sample rows to decode                     */
  const int32_t* n_dev;      /* device count of valid entries in samp_list         */
  int64_t n_max;
  const int32_t* pidx;       /* [rows,K] point index per (sample row, k), -1 = none */
  const float* sample_w;     /* [rows,3] sample world xyz                          */
  const float* sample_p;     /* [rows,3] sample perspective xyz                    */
  const float* dirs;         /* ray directions, row chosen by dir_map/dir_div      */
  const int32_t* dir_map;    /* NULL: dirs row = sample row / dir_div;
                                else  dirs row = dir_map[sample row] / dir_div     */
  int32_t dir_div;
  int32_t K;
  const int32_t* ray_cam;    /* NULL: pts->campos / camrot is the one camera; else the
                                camera of dirs row r is ray_cam[r] into the pts tables
                                campos[n_cams,3] / camrot[n_cams,3,3] (pnr_rays.ray_cam) */
} pnr_samples;

/* For every entry v < min(*n_dev, n_max) of samp_list (row = samp_list[v], or
 * row = v when samp_list is NULL) that has >= 1 valid neighbour:
 * out_feat[v, 0] = alpha, out_feat[v, 1..128] = colour features (rows of
 * samples without neighbours are left untouched).  Optional (may be NULL):
 * out_weight[row,K] normalised weights, out_conf[row,K] clamped confidence.
 * scratch: 16-B aligned device buffer of pnr_aggregate_scratch_bytes(n_max, N)
 * (N = pts->n_used when pts->used is set).
 * Block1.0 is split exactly: W1[:, :224].[emb, PE(emb)] + b1 depends only on
 * the point, so it is computed once per point (N x 256) and gathered per
 * pair; only the 60 distance-PE columns run per (sample, neighbour) pair. */
int pnr_aggregate_scratch_bytes(int64_t n_max, int64_t n_points, size_t* out);
int pnr_aggregate_fwd(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                      float* out_feat, float* out_weight, float* out_conf, void* scratch,
                      size_t scratch_bytes, void* stream);

/* bf16-MFMA variant (SURVEY config c5: bf16 MLP on v_mfma_f32_32x32x16_bf16,
 * fp32 accumulation; NOT the reference's precision).  Weights are bf16
 * fragment packs from pointnerf_amd.aggregator.frag_pack_bf16():
 * W_f[t][T][lane][j] = W'[32T + (lane&31)][16t + 8(lane>>5) + j], W' = [W | bias | 0]
 * for t < ceil((in+1)/16) + 2.  Same inputs / outputs as pnr_aggregate_fwd
 * (pidx required); scratch of pnr_aggregate_scratch_bytes_bf16(n_max, N). */
typedef struct {
  const uint16_t* w1af;  /* block1.0 columns 0..223 + bias (per point)   */
  const uint16_t* w1bf;  /* block1.0 columns 224..283 (no bias)         */
  const uint16_t* w2f;   /* block1.2 + bias                             */
  const uint16_t* w3f;   /* block3.0 + bias                             */
  const uint16_t* w4f;   /* block3.2 + bias                             */
  const float* wa; const float* ba;   /* alpha_branch.0 (fp32)          */
  const uint16_t* wc1f; const uint16_t* wc2f; const uint16_t* wc3f;  /* color_branch.{0,2,4} + bias */
  const float* rw2c;
  float neg_slope;
  int32_t act_super;
  int32_t pair_buckets;  /* 1: the pairs stage runs each sample in a bucket of KT = 1, 2, 4 or 8
                            neighbour slots (its last filled slot + 1; tiles of 128/KT samples x KT:
                            sparse scenes skip the empty slots, point_aggregators.py:608-628's
                            masked holders), same outputs; 0: every sample on 16 x 8 tiles */
} pnr_mlp_bf16;

int pnr_aggregate_scratch_bytes_bf16(int64_t n_max, int64_t n_points, size_t* out);
int pnr_aggregate_fwd_bf16(const pnr_points* pts, const pnr_samples* s, const pnr_mlp_bf16* w,
                           float* out_feat, float* out_weight, float* out_conf, void* scratch,
                           size_t scratch_bytes, void* stream);

/* Same (v20), with the aggregated features themselves in bf16 -- config c5's
 * bf16 path end to end, half the feature bytes written here and read by the
 * composite.  out_feat_h: rows of PNR_FEAT_H_PITCH uint16 (272 B, 16-B aligned)
 * = [alpha as one fp32 in slots 0-1 | slots 2-7 unused | 128 bf16 features in
 * slots 8..135, each the round-to-nearest-even of pnr_aggregate_fwd_bf16's
 * fp32 value].  Read by pnr_composite_fwd_hf. */
#define PNR_FEAT_H_PITCH 136
int pnr_aggregate_fwd_bf16_hf(const pnr_points* pts, const pnr_samples* s, const pnr_mlp_bf16* w,
                              uint16_t* out_feat_h, float* out_weight, float* out_conf, void* scratch,
                              size_t scratch_bytes, void* stream);

/* fp32-accurate aggregation on bf16 MFMA (same contract and scratch as
 * pnr_aggregate_fwd).  Each fp32 GEMM operand is split exactly into three bf16
 * terms (x = x0 + x1 + x2) and block1.0's distance half, block1.2, block3.0 and
 * block3.2 run as the six cross products of weight >= 2^-16 on
 * v_mfma_f32_32x32x16_bf16 with fp32 accumulation: the dropped terms are
 * below one fp32 rounding of each product.  The per-point block1.0 half and
 * the colour branch stay on the fp32 MFMA.  wx: split packs from
 * pointnerf_amd.aggregator.frag_pack_x3 (uint16 bf16 planes). */
typedef struct {
  const void* w1bx;   /* block1.0 columns 224..283 */
  const void* w2x;    /* block1.2 + bias           */
  const void* w3x;    /* block3.0 + bias           */
  const void* w4x;    /* block3.2 + bias           */
} pnr_mlp_x3;
int pnr_aggregate_fwd_x3(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w, const pnr_mlp_x3* wx,
                         float* out_feat, float* out_weight, float* out_conf, void* scratch,
                         size_t scratch_bytes, void* stream);

/* fp32-accurate aggregation on f16 MFMA (same contract and scratch as
 * pnr_aggregate_fwd; replaces the same reference call,
 * point_aggregators.py:729-816 / 488-646).  Each fp32 operand is split into
 * two f16 terms, x = xh + 2^-11 xl (xh = f16(x), xl = f16((x - xh) 2^11),
 * round to nearest even), and block1.0's distance half, block1.2, block3.0 and
 * block3.2 run as three products, 2^-11 (2^11 Wh.Xh + Wh.Xl + Wl.Xh), on
 * v_mfma_f32_32x32x16_f16 with fp32 accumulation: the split and the dropped
 * Wl.Xl term are each below one fp32 rounding of the product.  Packs from
 * pointnerf_amd.aggregator.frag_pack_h2: layer weights pre-scaled by 2^-s
 * (|W 2^-s| < 16 so 2^11 Wh stays in f16), planes [t][T][Wh, Wl][lane][8],
 * scale[l] = 2^(s_l - 11).  Activations must stay inside the f16 range
 * (|x| < 65504): one that does not has an infinite high half, which makes
 * every output it reaches inf or NaN; a launch with a non-finite output sets
 * *range_flag = 1 (device int, caller-owned, may be NULL) and its outputs are
 * not valid (the renderer then re-renders on pnr_aggregate_fwd_x3).
 * Colour branch (point_aggregators.py:630-638): with wc1a..wc3h set it runs on
 * the same f16-split MFMA (k_color_h2; color_branch.0 split into columns
 * 0..143 and 144..279 + bias, both packed with ONE layer scale cscale[0]);
 * with wc1a NULL on the fp32 MFMA (k_color) like pnr_aggregate_fwd. */
typedef struct {
  const void* w1bh;   /* block1.0 columns 224..283                              */
  const void* w2h;    /* block1.2, NO bias column (the kernel adds w->b2 in fp32) */
  const void* w3h;    /* block3.0 + bias                                         */
  const void* w4h;    /* block3.2, NO bias column (the kernel adds w->b4 in fp32) */
  float scale[4];
  int32_t* range_flag;
  const void* wc1a;   /* color_branch.0 columns 0..143          (NULL: fp32 colour branch) */
  const void* wc1b;   /* color_branch.0 columns 144..279 + bias */
  const void* wc2h;   /* color_branch.2 + bias                  */
  const void* wc3h;   /* color_branch.4 + bias                  */
  float cscale[3];
  const void* w1ah;   /* block1.0 columns 0..223 + bias: the per-point half P1 on
                         f16-split MFMA (k_point_pre_h2; NULL: fp32 k_point_pre) */
  float scale1a;
} pnr_mlp_h2;
int pnr_aggregate_fwd_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w, const pnr_mlp_h2* wh,
                         float* out_feat, float* out_weight, float* out_conf, void* scratch,
                         size_t scratch_bytes, void* stream);

/* PointAggregator.forward signature (pre-gathered tensors): pts tables are the
 * gathered [rows*K, C] tensors, s->pidx must be NULL (pair row = row*K + k),
 * pts->pers required, validity from pair_mask[rows*K] (sample_pnt_mask). */
/* block1.0's per-point half alone (k_point_pre_h2): P1 rows of every point (of
 * pts->used when set) into the head of an aggregate scratch -- the rows
 * pnr_aggregate_fwd_h2 reads with pts->p1_ready = 1.  P1 depends on the points
 * and weights only, so the renderer issues it on a side stream beside the
 * (latency-bound) query instead of in front of the pairs kernel; wh's w1ah /
 * scale1a / range_flag as pnr_aggregate_fwd_h2. */
int pnr_point_pre_h2(const pnr_points* pts, const pnr_mlp_h2* wh, void* scratch, size_t scratch_bytes,
                     void* stream);
int pnr_aggregate_fwd_masked(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                             const uint8_t* pair_mask, float* out_feat, float* out_weight,
                             float* out_conf, void* scratch, size_t scratch_bytes, void* stream);

/* ------------------------------------------------------- aggregate backward
 * Training path (autograd of point_aggregators.py:729-816 /
 * 488-646 and the gather neural_points.py:788-799).  pnr_aggregate_fwd_train
 * runs the forward and keeps the activations the backward needs; all saved
 * arrays are indexed by sample-list entry v (< n_max) and pair row v*8 + k. */
typedef struct {
  float* h1; float* h2; float* h3; float* h4;  /* [n_max*8,256] post-activation outputs of
                                                  block1.0, block1.2, block3.0, block3.2 */
  float* pe5;      /* [n_max*8,64] PE_5 of the rotated 6-d distance (block1.0 cols 224..283),
                      columns 60..63 zero (GEMM padding)                                        */
  float* x3e;      /* [n_max*8,32] block3.0 inputs 256..262 (colour, R.dir - R.v, <R.dir,R.v>),
                      1, then zeros (GEMM padding)                                              */
  float* pa;       /* [n_max*8]    alpha_branch.0 output (before softplus(x - 1))              */
  float* wt;       /* [n_max*8]    w_k * clamp(conf_k); 0 for empty pairs                      */
  float* wn;       /* [n_max*8]    normalised distance weight w_k                              */
  int32_t* prow;   /* [n_max*8]    point row of the pair, -1 = empty                           */
  float* hid;      /* [n_max,256]  K-summed features (colour-branch input 0..255)              */
  float* vpe;      /* [n_max,24]   view-direction PE (colour-branch input 256..279)            */
  float* hc1; float* hc2; float* hc3;  /* [n_max,128] colour-branch activations              */
  int32_t* vmask;  /* [n_max]      sample has >= 1 valid neighbour                             */
  uint16_t* mask;  /* [n_max*8,64] LeakyReLU derivative bits of the four 256-wide layers
                      (layer l, tile T, lane half h: word 16l + 2T + h; bit r = pre-activation
                      of MFMA accumulator register r > 0), read by the backward            */
  uint32_t* dz_absmax; /* optional [5]: pnr_aggregate_bwd_pairs(_x3) max-es |dz1..dz4| and
                      |dpa| into it (float bits, atomic; the caller zeroes it): the scales
                      of pnr_gemm_tn_h2 without a pnr_absmax pass (ABI 19)               */
  float* x1;       /* optional [>= n_used][224] (ABI 23): block1.0's point-half inputs
                      [emb, PE_3(emb)] of the used points, written by the fp32h2 training
                      forward's k_point_pre_h2 (its angle-doubled PE) and read by the
                      backward's block1.0 weight gradient instead of a recomputation   */
} pnr_agg_saved;

/* Transposed weights for the backward GEMMs, fragment-packed like pnr_mlp
 * (frag_pack(W.T)): w4t = block3.2^T, w3t = block3.0[:, :256]^T, w2t = block1.2^T,
 * w3e = block3.0[:, 256:263] row-major [256,7]. */
typedef struct {
  const float* w4t; const float* w3t; const float* w2t; const float* w3e;
} pnr_mlp_bwd;

int pnr_aggregate_fwd_train(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                            const pnr_agg_saved* saved, float* out_feat, float* out_weight,
                            float* out_conf, void* scratch, size_t scratch_bytes, void* stream);
/* pnr_aggregate_fwd_train with the per-pair chain (block1.0 pair half, block1.2,
 * block3.0, block3.2) on the fp32x3 split-bf16 MFMA kernel of pnr_aggregate_fwd_x3
 * (wx: packed_x3); same saved arrays and outputs, fp32-accurate (not bitwise
 * the native-fp32 forward).  P1 and the colour branch stay on the fp32 kernels. */
int pnr_aggregate_fwd_train_x3(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                               const pnr_mlp_x3* wx, const pnr_agg_saved* saved, float* out_feat,
                               float* out_weight, float* out_conf, void* scratch, size_t scratch_bytes,
                               void* stream);
/* Same, for the PointAggregator.forward mirror (pre-gathered tables, pair_mask). */
/* pnr_aggregate_fwd_train with the per-pair chain on the fp32h2 kernel of
 * pnr_aggregate_fwd_h2 (k_pairs_h2 + the same saves; wh's w1bh / w2h / w3h / w4h
 * packs and scales, and w1ah / scale1a when set: P1 on k_point_pre_h2, else on
 * fp32 MFMA; with wc1a..wc3h / cscale set (ABI 22) the colour branch runs on
 * f16-split MFMA too, k_color_h2 with k_color<train>'s saves (vpe, hc1..hc3),
 * else on the fp32 training kernel), the range flag as pnr_aggregate_fwd_h2: set when an
 * activation left the f16 range, the caller then re-runs the step on
 * pnr_aggregate_fwd_train_x3).  Saved layout and outputs as the fp32 call. */
int pnr_aggregate_fwd_train_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                               const pnr_mlp_h2* wh, const pnr_agg_saved* saved, float* out_feat,
                               float* out_weight, float* out_conf, void* scratch, size_t scratch_bytes,
                               void* stream);
/* pnr_aggregate_fwd_train_h2 with its fallback on the device (v17): after the h2
 * chain, k_point_pre (when P1 ran on fp32h2) and the native-fp32 k_pairs<train>
 * (and, with the colour packs, the fp32 colour branch) are launched over the
 * same outputs and saves, and each workgroup returns at
 * once unless *wh->range_flag != 0 -- so a raised flag never needs a host read
 * inside the step (the caller reads it later, asynchronously, to re-pick the
 * shifts).  wh->range_flag is required.  Outputs: those of the h2 call when the
 * flag stays down, those of pnr_aggregate_fwd_train when it is raised. */
int pnr_aggregate_fwd_train_h2_guarded(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                       const pnr_mlp_h2* wh, const pnr_agg_saved* saved, float* out_feat,
                                       float* out_weight, float* out_conf, void* scratch, size_t scratch_bytes,
                                       void* stream);
int pnr_aggregate_fwd_train_masked(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                   const uint8_t* pair_mask, const pnr_agg_saved* saved,
                                   float* out_feat, float* out_weight, float* out_conf,
                                   void* scratch, size_t scratch_bytes, void* stream);

/* Per-pair backward of block3.2 .. block1.0's pair half, alpha branch, K-sums,
 * weights and gather, given d_feat[n,129] (column 0: d alpha) and
 * d_hid[n,256] (gradient of the K-summed features from the colour branch).
 * Writes dz1..dz4[n_max*8,256] (gradients of the four pre-activations; rows
 * of empty pairs are 0) and dpa[n_max*8]; accumulates (atomically, so the
 * caller zeroes them) d_p1[N,256] += dz1 per point (block1.0 point half; rows
 * are used_map[point] when pts->used is set, i.e. d_p1 is [n_used,256]),
 * d_color[N,3], d_dir[N,3], d_conf[N] (straight-through clamp gradient).
 * Any of d_color / d_dir / d_conf may be NULL. */
int pnr_aggregate_bwd_pairs(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                            const pnr_mlp_bwd* wb, const pnr_agg_saved* saved,
                            const float* d_feat, const float* d_hid, float* dz1, float* dz2,
                            float* dz3, float* dz4, float* dpa, float* d_p1, float* d_color,
                            float* d_dir, float* d_conf, void* stream);
/* The points referenced by a query's neighbour rows (pnr_points.used /
 * used_map for a training batch): flags[n_points] (scratch, 16-B aligned,
 * as is scratch: a byte and a bit per point), used_map[p] = rank
 * of p among the referenced points or -1, used[0 .. *n_used_dev) = the referenced
 * points ascending; rows pidx[0 .. (*n_samples_dev) * K) (n_samples_dev NULL:
 * cap_samples).  No host synchronisation (the count stays on the device). */
int pnr_used_points_scratch_bytes(int64_t n_points, size_t* out);
int pnr_used_points(const int32_t* pidx, const int32_t* n_samples_dev, int32_t K, int64_t cap_samples,
                    int64_t n_points, int32_t* flags, int32_t* used_map, int32_t* used, int32_t* n_used_dev,
                    void* scratch, size_t scratch_bytes, void* stream);
/* d_p1[row(p)] = sum of dz1[pair] over the pairs of point p, given the pairs'
 * point rows sorted (stable: each point's pairs in pair order, a deterministic
 * sum) and the pair index of each sorted entry: the atomic-free alternative to
 * pnr_aggregate_bwd_pairs' d_p1 (pass d_p1 = NULL there).  row(p) = used_map[p]
 * (or p when used_map is NULL); rows of points without pairs are not written;
 * negative point rows (empty pairs) are skipped. */
int pnr_pairs_to_points(const int32_t* prow_sorted, const int32_t* pair_of, int64_t P, const float* dz1,
                        const int32_t* used_map, float* d_p1, uint32_t* d_p1_absmax, void* stream);
/* The block3.0 extras of pnr_aggregate_bwd_pairs_x3 without float atomics (ABI 19;
 * that call skips its own extras pass when pnr_mlp_bwd.w3e is NULL):
 * pnr_aggregate_bwd_extras_rows writes per pair g_pair[pair][0..7] = (g0, g1, g2,
 * g3 + vrot0 g6, g4 + vrot1 g6, g5 + vrot2 g6, 0, 0), g_e = dz3[pair] . w3e[:, e]
 * (w3e = block3.0[:, 256:263] row-major [256,7]), vrot the pair's view direction
 * rotated as in the forward; pnr_pairs_to_points_ex is pnr_pairs_to_points plus,
 * per referenced point p over its pairs in pair order, d_color[p] = sum g[0..2]
 * and d_dir[p] = Rw_p^T sum g[3..5] (rw_pp [N,9] per-point, else rw_uniform [9],
 * else identity) -- written, not added; deterministic. */
int pnr_aggregate_bwd_extras_rows(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                  const pnr_agg_saved* saved, const float* w3e, const float* dz3, float* g_pair,
                                  void* stream);
int pnr_pairs_to_points_ex(const int32_t* prow_sorted, const int32_t* pair_of, int64_t P, const float* dz1,
                           const int32_t* used_map, float* d_p1, uint32_t* d_p1_absmax, const float* g_pair,
                           const float* rw_uniform, const float* rw_pp, float* d_color, float* d_dir,
                           void* stream);
/* zero_one_loss(conf_coefficient) (base_rendering_model.py:634-639) from per-point
 * entry counts (pnr_point_counts): out[0] = mean over the E = (*r_valid) * srk
 * entries of log(v) + log(1 - v), v = clamp(clamp(conf, 1e-4, 1), eps, 1 - eps),
 * the E - sum(counts) empty entries gathered as point 0; out[1] = those empty
 * entries, out[2] = E.  partials: 1024 device floats.  The backward: d_conf[p] =
 * g[0] (counts[p] (+ out[1] at p = 0)) f'(v_p) / E where eps <= cc_p <= 1 - eps,
 * else 0 (gradiant_clamp passes straight through).  Deterministic (ABI 19). */
int pnr_zero_one_loss_fwd(const float* conf, const float* counts, int64_t N, const int32_t* r_valid, int64_t srk,
                          float eps, float* partials, float* out, void* stream);
int pnr_zero_one_loss_bwd(const float* conf, const float* counts, int64_t N, float eps, const float* fwd_out,
                          const float* g, float* d_conf, void* stream);
/* counts[p] += number of entries p >= 0 in pidx rows [0, min(*n_dev, cap)) (K per
 * row); float counts, exact below 2^24 (the zero-one conf loss, ABI 19). */
int pnr_point_counts(const int32_t* pidx, const int32_t* n_dev, int32_t K, int64_t cap, float* counts, void* stream);
/* d_p1_absmax (optional, ABI 19): max |d_p1| as float bits, atomically max-ed
 * (the caller zeroes it) -- pnr_gemm_tn_h2 / pnr_gemm_nn_h2's scale for d_p1. */
/* Device weight packing (aggregator.py frag_pack / frag_pack_x3, one launch per
 * matrix): kind 0 = fp32 fragments F[t][T][lane] = W'[32T + (lane & 31)][2t + (lane >> 5)],
 * ceil(cols / 2) + pad_steps k-steps; kind 1 = fp32x3 split-bf16 fragments
 * F[t][T][plane][h][r][j] = plane of W'[32T + r][16t + 8h + j], ceil(cols / 16) +
 * pad_steps k-steps; W' = [W | bias | 0] (cols = kin + 1 with a bias),
 * W[o][k] = W[o * ld_row + k * ld_col] (element strides), out_f % 32 == 0. */
int pnr_pack_weights(int32_t kind, const float* W, int64_t ld_row, int64_t ld_col, int32_t out_f,
                     int32_t kin, const float* bias, int32_t pad_steps, void* out, size_t out_bytes,
                     void* stream);
/* fp32h2 packs (aggregator.py frag_pack_h2 with a given shift s, one launch):
 * F[t][T][plane][h][r][j] = plane of (2^-s W')[32T + r][16t + 8h + j], planes
 * (Wh, Wl): Wh = f16(x), Wl = f16((x - Wh) 2^11) (round to nearest even),
 * ceil(cols / 16) + pad_steps k-steps; *range_flag |= 1 when some |2^-s W'| >= 16
 * or is not finite (the pack is then unusable: the caller re-picks s).  The
 * training step keeps s across steps and packs without a host sync. */
int pnr_pack_weights_h2(const float* W, int64_t ld_row, int64_t ld_col, int32_t out_f, int32_t kin,
                        const float* bias, int32_t pad_steps, int32_t shift, int32_t* range_flag, void* out,
                        size_t out_bytes, void* stream);
/* pnr_pack_weights_h2 with the shift picked on the device (no host read of the
 * weights): s such that max |2^-s W'| lies in [8, 16) (0 for an all-zero or
 * non-finite W', as aggregator.h2_shift), scale_dev[0] = 2^(s - 11) (the
 * consumer's accumulator factor), scale_dev[1] is scratch. */
int pnr_pack_weights_h2_dev(const float* W, int64_t ld_row, int64_t ld_col, int32_t out_f, int32_t kin,
                            const float* bias, int32_t pad_steps, float* scale_dev, void* out, size_t out_bytes,
                            void* stream);
/* Same, with the three dX GEMMs on fp32x3 split-bf16 MFMA: wbx = frag_pack_x3 of
 * block3.2.weight^T, block3.0.weight[:, :256]^T, block1.2.weight^T (aggregator.py;
 * 16-B aligned); wb supplies w3e (w4t / w3t / w2t unused, may be NULL). */
typedef struct {
  const void* w4tx; const void* w3tx; const void* w2tx;
} pnr_mlp_bwd_x3;
int pnr_aggregate_bwd_pairs_x3(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                               const pnr_mlp_bwd* wb, const pnr_mlp_bwd_x3* wbx, const pnr_agg_saved* saved,
                               const float* d_feat, const float* d_hid, float* dz1, float* dz2, float* dz3,
                               float* dz4, float* dpa, float* d_p1, float* d_color, float* d_dir,
                               float* d_conf, void* stream);
/* Several weight packs in one launch (a training step rebuilds every pack per
 * step): job q is pnr_pack_weights(kind, ...) for kind 0 / 1 and
 * pnr_pack_weights_h2(..., shift, range_flag, ...) for kind 2 (shift and
 * range_flag ignored otherwise), same layouts, bitwise the same outputs;
 * 1 <= n <= 24. */
typedef struct {
  int32_t kind;
  const float* W; int64_t ld_row; int64_t ld_col;
  int32_t out_f; int32_t kin;
  const float* bias;
  int32_t pad_steps; int32_t shift;
  int32_t* range_flag;
  void* out; size_t out_bytes;
} pnr_pack_job;
int pnr_pack_batch(const pnr_pack_job* jobs, int32_t n, void* stream);
/* Same, with the three dX GEMMs on fp32h2 split-f16 MFMA (the fp32h2 training
 * step): wbh = pnr_pack_bwd_h2's packs and scales; each 64-pair tile's layer
 * input is scaled by a power of two picked from its max |value| inside the
 * kernel (no range flag, no fallback).  wb supplies w3e as above. */
typedef struct {
  const void* w4th; const void* w3th; const void* w2th;
  const float* scale;   /* device [3]: 2^(s - 11) of each pack */
} pnr_mlp_bwd_h2;
int pnr_aggregate_bwd_pairs_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                               const pnr_mlp_bwd* wb, const pnr_mlp_bwd_h2* wbh, const pnr_agg_saved* saved,
                               const float* d_feat, const float* d_hid, float* dz1, float* dz2, float* dz3,
                               float* dz4, float* dpa, float* d_p1, float* d_color, float* d_dir,
                               float* d_conf, void* stream);
/* The packs of pnr_aggregate_bwd_pairs_h2 in one launch: block3.2.weight^T
 * (w4, [256,256] row-major), block3.0.weight[:, :256]^T (w3, row stride ld3 >=
 * 256) and block1.2.weight^T (w2) as frag_pack_h2 packs of 16 + pad_steps
 * k-steps each (pad steps zero; the kernel reads 3 ahead: pad_steps >= 3),
 * back to back in out (3 x (16 + pad) x 2048 x 8 B); scale_dev[m] = 2^(s_m - 11)
 * with s_m picked on the device as pnr_pack_weights_h2_dev's. */
int pnr_pack_bwd_h2(const float* w4, const float* w3, int64_t ld3, const float* w2, int32_t pad_steps,
                    float* scale_dev, void* out, size_t out_bytes, void* stream);
/* The pairs grouped by point: the (prow_sorted, pair_of) of torch.sort(prow[0..m),
 * stable=True) over the pairs with prow >= 0 -- each referenced point's pairs in
 * pair order -- followed by the empty pairs (prow_sorted = -1, pair_of = 0) at
 * the END (torch.sort puts them first; pnr_pairs_to_points(_ex) skip them either
 * way).  Key of a pair = key_map[prow] (the used-point map, keys < n_keys) or
 * prow itself (key_map NULL, n_keys > max prow).  A counting sort with a
 * per-key sort back into pair order: deterministic, no host sync. */
int pnr_group_pairs_scratch_bytes(int64_t m, int64_t n_keys, size_t* out);
int pnr_group_pairs(const int32_t* prow, int64_t m, const int32_t* key_map, int64_t n_keys, int32_t* prow_sorted,
                    int32_t* pair_of, void* scratch, size_t scratch_bytes, void* stream);
/* alpha_branch.0's gradient: out_w[c] = sum_r dpa[r] h4[r][c] (c < 256, h4 rows of
 * 256), out_b[0] = sum_r dpa[r], r < m; deterministic (fixed per-block partials
 * summed in block order); partials: pnr_alpha_colsum_scratch_floats() floats. */
int pnr_alpha_colsum_scratch_floats(int64_t* out);
int pnr_alpha_colsum(const float* dpa, const float* h4, int64_t m, float* out_w, float* out_b, float* partials,
                     void* stream);
/* The fp32h2 finetune step's backward through the aggregator in one call
 * (replaces train.py AggregateFn.backward's sequence, point_aggregators.py
 * autograd as listed there): colour branch (pnr_color_dz, pnr_gemm_tn_h2 /
 * pnr_gemm_nn_h2), pnr_pack_bwd_h2 + pnr_aggregate_bwd_pairs_h2,
 * pnr_group_pairs + pnr_aggregate_bwd_extras_rows + pnr_pairs_to_points_ex,
 * the weight gradients, pnr_alpha_colsum, block1.0's point half
 * (pnr_point_pe3_rows, pnr_gemm_tn_h2 / pnr_gemm_nn_h2, pnr_point_pe3_bwd_rows).
 * prm: the 16 aggregator parameters as nn.Linear stores them (row-major), in
 * train.py _PARAM_NAMES order; out->g: their gradients (same shapes, written);
 * d_emb [N,32] written (zero for unreferenced points); d_color / d_dir [N,3],
 * d_conf [N] written when not NULL.  n = valid samples (d_feat [>= n, 129]),
 * n_used = referenced points (pts->used / used_map required).  Scratch:
 * pnr_aggregate_bwd_step_h2_scratch_bytes (256-B aligned).  No host sync. */
typedef struct { const float* p[16]; } pnr_agg_params;
typedef struct {
  float* g[16];
  float* d_emb; float* d_color; float* d_dir; float* d_conf;
} pnr_agg_grads;
int pnr_aggregate_bwd_step_h2_scratch_bytes(int64_t n, int64_t n_used, size_t* out);
int pnr_aggregate_bwd_step_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                              const pnr_agg_params* prm, const pnr_agg_saved* saved, const float* d_feat, int64_t n,
                              int64_t n_used, const pnr_agg_grads* out, void* scratch, size_t scratch_bytes,
                              void* stream);
/* Point-position gradient (--xyz_grad 1, neural_points.py:270; replaces the
 * autograd of sampled_xyz / sampled_xyz_pers, neural_points.py:635, 788-799,
 * through point_aggregators.py:775-804 and the PE_5 input of block1.0):
 * d_xyz[N,3] += (atomically) the gradient through the world distance (PE_5
 * channels 0..2 and the normalised inverse-distance weight) and the perspective
 * deltas (PE_5 channels 3..5, w2pers of the pair's camera, qpiw.py:102-109).
 * d_pe[n_max*8,64] = dz1 . W1[:, 224:284] (block1.0's PE_5 columns; 60..63
 * unused, the pitch of pnr_agg_saved.pe5); saved,
 * d_feat, d_hid as for pnr_aggregate_bwd_pairs; pts needs xyz and the camera
 * tables (ray_cam-indexed for multi-camera batches). */
int pnr_aggregate_bwd_xyz(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                          const pnr_agg_saved* saved, const float* d_feat, const float* d_hid,
                          const float* d_pe, float* d_xyz, void* stream);

/* Weight-gradient GEMM (replaces the dW = dY^T X of torch's nn.Linear autograd
 * for block1.0/1.2/3.0/3.2, point_aggregators.py:276-348 trained by
 * mvs_points_volumetric_model.py:102-123 setup_optimizer):
 * C[M,N] = A^T B over K rows (A[K,M], B[K,N] row-major,
 * leading dimensions lda/ldb), colsum_a[M] = column sums of A (bias gradient,
 * may be NULL).  M, N multiples of 32; scratch, C and colsum_a 16-B aligned.
 * Split-K on MFMA with a deterministic ordered reduction (its last level writes
 * C and colsum_a directly); scratch of pnr_gemm_tn_scratch_bytes(K, M, N). */
int pnr_gemm_tn_scratch_bytes(int64_t K, int32_t M, int32_t N, size_t* out);
int pnr_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M, int32_t N,
                float* C, float* colsum_a, void* scratch, size_t scratch_bytes, void* stream);
/* Same contract and scratch, fp32-accurate on bf16 MFMA: A and B split exactly
 * into three bf16 terms each, the six cross products of weight >= 2^-16 with
 * fp32 accumulation (the fp32x3 arithmetic of pnr_aggregate_fwd_x3; error vs an
 * fp64 GEMM ~ native fp32's).  The training path's default. */
int pnr_gemm_tn_x3(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M, int32_t N,
                   float* C, float* colsum_a, void* scratch, size_t scratch_bytes, void* stream);

/* Data-gradient product of the backward (dX = dZ W of an nn.Linear, replacing
 * the autograd mm of color_branch / block1.0, point_aggregators.py:488-646):
 * C[M,N] = A[M,K] B[K,N], row-major with unit column strides, exact fp32
 * products on fp32 MFMA; with act != NULL each C[m,n] is multiplied by the
 * LeakyReLU derivative of the saved activation act[m,n] (1 if > 0, else slope).
 * N a multiple of 32 in [32, 256]; any M >= 0, K > 0. */
/* fp32-accurate C = A^T B on f16 MFMA (the fp32h2 arithmetic of the forward):
 * A scaled by 2^e with max|A| 2^e in [4, 8) -- e from *a_absmax, the float bits
 * of max |A| (pnr_absmax) -- both operands split x = xh + 2^-11 xl, three f16
 * products per k-step (pnr_gemm_tn_x3 takes six bf16 ones).  An operand outside
 * the split's range (|B| >= 2^15, a stale max, NaN / inf) sets *range_flag and
 * the call's x3 kernel, launched behind the h2 one, then recomputes it: the
 * result is always the fp32-accurate one.  The caller zeroes *range_flag (one
 * flag can serve every call of a step) and may read it later to count fallbacks.
 * Same M, N, scratch and colsum rules as pnr_gemm_tn. */
int pnr_gemm_tn_h2(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M, int32_t N,
                   float* C, float* colsum_a, const uint32_t* a_absmax, int32_t* range_flag, void* scratch,
                   size_t scratch_bytes, void* stream);
/* pnr_gemm_nn on f16-split MFMA (the fp32h2 arithmetic): A scaled by its device
 * max (*a_absmax), three f16 products per 16-k step; operands outside the split's
 * range set *range_flag and the fp32 kernel, launched behind, recomputes C. */
int pnr_gemm_nn_h2(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int32_t K, int32_t N,
                   const float* act, int64_t ld_act, float slope, float* C, int64_t ldc, const uint32_t* a_absmax,
                   int32_t* range_flag, void* stream);
/* The colour branch's backward input in one pass (train.py: replaces the torch
 * ops (d_feat[:, 1:] * (vmask != 0)) then where(hc > 0, x, x * slope)):
 * dz[r][c] = that, r < n, c < C (C % 4 == 0; dz [n, C] row-major; d_feat rows of
 * ld_feat >= C + 1 floats, column 0 the alpha; hc rows of ld_hc, a multiple of 4;
 * hc and dz 16-B aligned); absmax (optional,
 * pre-zeroed): max |dz| folded in as float bits (NaN above inf), the scale of
 * the h2 GEMMs that consume dz. */
int pnr_color_dz(const float* d_feat, int64_t ld_feat, const int32_t* vmask, const float* hc, int64_t ld_hc,
                 int64_t n, int32_t C, float slope, float* dz, uint32_t* absmax, void* stream);
/* *out_bits = float bits of max |x[0, n)| (NaN if any x is NaN); partials:
 * pnr_absmax_scratch_floats() device floats.  No host sync. */
int pnr_absmax_scratch_floats(int64_t* out);
int pnr_absmax(const float* x, int64_t n, float* partials, uint32_t* out_bits, void* stream);
int pnr_gemm_nn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int32_t K, int32_t N,
                const float* act, int64_t ld_act, float slope, float* C, int64_t ldc, void* stream);

/* X1[p] = [emb_p, PE_3(emb_p)] (block1.0 columns 0..223) for p < n, and the
 * matching backward d_emb[p] += dX1[p] . dX1/d emb (networks.py:175-190). */
int pnr_point_pe3(const float* emb, int64_t n, float* x1, void* stream);
int pnr_point_pe3_bwd(const float* emb, const float* d_x1, int64_t n, float* d_emb, void* stream);
/* The same over a row list (ABI 19): X1[i] = PE_3(emb[rows[i]]) and
 * d_emb[rows[i]] += the PE_3 backward of d_x1[i] (rows distinct: the used points) --
 * no gathered copy of the embedding, no index_copy of its gradient. */
int pnr_point_pe3_rows(const float* emb, const int32_t* rows, int64_t n, float* x1, void* stream);
int pnr_point_pe3_bwd_rows(const float* emb, const int32_t* rows, const float* d_x1, int64_t n, float* d_emb,
                           void* stream);

/* -------------------------------------------------------------- composite
 * Fused ray_dist (cummax), alpha composite and fill_invalid for the full ray
 * batch R, straight from the query buffers and the decoded features
 * (indexed by filled-sample row).  Outputs (all [R,...]):
 *   ray_color[R,C]  opacity[R,SR]  is_bg[R]  ray_mask[R] (int8) */
typedef struct {
  float vsize_z;        /* vsize[2] of the querier (unscaled)                   */
  int32_t raydist_mode_unit;
  int32_t C;            /* 128 */
  const float* bg_color;/* [C] device                                           */
  int64_t feat_rows;    /* rows of feat (0 = unbounded).  A valid sample whose row is
                           >= feat_rows (more valid samples than the caller sized feat
                           for, counts[1] > feat_rows) is composited as empty and never
                           read: the output is then wrong but the call is memory-safe,
                           and the caller re-renders with a larger feat (renderer.py). */
} pnr_composite_params;

int pnr_composite_fwd(const pnr_rays* rays, const pnr_query_params* q,
                      const pnr_query_bufs* b, const pnr_composite_params* c,
                      const float* feat, float* ray_color, float* opacity,
                      float* is_bg, int8_t* ray_mask, void* stream);

/* pnr_composite_fwd on pnr_aggregate_fwd_bf16_hf's rows (v20; c->C even, <= 128):
 * the same blend in fp32 from bf16 features and the fp32 alpha. */
int pnr_composite_fwd_hf(const pnr_rays* rays, const pnr_query_params* q,
                         const pnr_query_bufs* b, const pnr_composite_params* c,
                         const uint16_t* feat_h, float* ray_color, float* opacity,
                         float* is_bg, int8_t* ray_mask, void* stream);

/* ray_march on dense inputs (diff_ray_marching.py:509-555, radiance_render,
 * alpha_blend): ray_dist[NR,SR], ray_valid[NR,SR] (uint8), feat[NR,SR,C+1],
 * bg[C] or NULL.  Outputs ray_color[NR,C], opacity[NR,SR], acc_T[NR,SR]
 * (exclusive), blend_w[NR,SR], bg_T[NR]. */
int pnr_ray_march_fwd(const float* ray_dist, const uint8_t* ray_valid, const float* feat,
                      const float* bg, int64_t NR, int32_t SR, int32_t C,
                      float* ray_color, float* opacity, float* acc_T, float* blend_w,
                      float* bg_T, void* stream);

/* Backward of pnr_composite_fwd with respect to feat (diff_ray_marching.py:509-555
 * autograd): d_feat[S_valid, C+1] from d_ray_color[R,C] (every valid row is
 * written; opacity / is_bg gradients are not propagated). */
int pnr_composite_bwd(const pnr_rays* rays, const pnr_query_params* q,
                      const pnr_query_bufs* b, const pnr_composite_params* c,
                      const float* feat, const float* d_ray_color, float* d_feat, void* stream);

/* Backward of pnr_ray_march_fwd with respect to feat: d_feat[NR,SR,C+1]. */
int pnr_ray_march_bwd(const float* ray_dist, const uint8_t* ray_valid, const float* feat,
                      const float* bg, int64_t NR, int32_t SR, int32_t C,
                      const float* d_ray_color, float* d_feat, void* stream);

/* Full reverse mode of pnr_ray_march_fwd (ray_march is differentiable in every
 * output, diff_ray_marching.py:509-555, called in training at
 * neural_points_volumetric_model.py:314): d_feat[NR,SR,C+1] and, when
 * d_ray_dist != NULL, d ray_dist[NR,SR], from d_ray_color[NR,C] and the optional
 * (NULL = 0) d_opacity / d_acc_T / d_blend_w [NR,SR] and d_bg_T [NR].  The
 * bg_color gradient is pnr_weighted_colsum(bg_T, d_ray_color). */
int pnr_ray_march_bwd_ex(const float* ray_dist, const uint8_t* ray_valid, const float* feat,
                         const float* bg, int64_t NR, int32_t SR, int32_t C, const float* d_ray_color,
                         const float* d_opacity, const float* d_acc_T, const float* d_blend_w,
                         const float* d_bg_T, float* d_feat, float* d_ray_dist, void* stream);

/* out[c] = sum_r w[r] x[r,c] (R rows, C <= 128 columns), bitwise repeatable: the
 * learned background's gradient (mvs_points_volumetric_model.py:92-94 optimises
 * bg_color).  For pnr_composite_fwd's rays w = is_bg (bg_T of a hit ray, 1 for a
 * background ray filled by fill_invalid, neural_points_volumetric_model.py:373-375),
 * x = d ray_color; for pnr_ray_march_fwd w = bg_T.  partials: device floats of
 * pnr_weighted_colsum_scratch_floats(C). */
int pnr_weighted_colsum_scratch_floats(int32_t C, int64_t* out);
/* Zero rows [0, min(*n_dev, n_cap)) of a row-major buffer (row_bytes % 4 == 0):
 * the device-counted part of a capacity-sized buffer, no host read of the
 * count (the sync-free training forward's feature / hid rows). */
int pnr_zero_rows(void* p, int64_t row_bytes, const int32_t* n_dev, int64_t n_cap, void* stream);
int pnr_weighted_colsum(const float* w, const float* x, int64_t R, int32_t C, float* out, float* partials,
                        void* stream);

/* The training outputs NeuralPointsRayMarching.forward adds to its dict
 * (neural_points_volumetric_model.py:335-338) in pnr_query_compact's row order
 * (the first rows_max of the R'' rays with a neighbour): weight[R'',SR,K] = the
 * aggregator's normalised inverse-distance weight before the conf factor
 * (point_aggregators.py:421-429, 803-804; 0 for empty slots), blend_weight[R'',SR]
 * = opacity * acc_T of ray_march from pnr_composite_fwd's opacity[R,SR].  Either
 * output may be NULL. */
int pnr_march_aux(const pnr_rays* rays, const pnr_query_params* q, const pnr_query_bufs* b,
                  const float* xyz, const float* opacity, int64_t rows_max, float* weight,
                  float* blend_weight, void* stream);

/* -------------------------------------------------------- 2-D neural renderer
 * NeuralRenderer(input_dim=128) (models/neural_render/neural_renderer.py:24-104,
 * applied at neural_points_volumetric_model.py:343-344 when neural_render == "cnn")
 * on the composited feature image x[H,W,128] (row-major pixels = ray order):
 * out_rgb[H,W,3] = sigmoid(conv_rgb0(x) + conv_rgb1(net0) + conv_rgb2(net1)),
 * net0 = lrelu_0.2(conv_layers.0(x)), net1 = lrelu_0.2(conv_layers.1(net0)),
 * all 3x3 / stride 1 / pad 1.  Per stage s the trunk conv's [cout, cin, 3, 3]
 * weights as rows, columns k = (ky*3 + kx) * cin + ci, fragment-packed like
 * pnr_mlp (frag_pack, no bias column), b_s its bias; the rgb conv's weights
 * row-major [3, 9 * cin] (same k order, not packed: they run on VALU beside the
 * trunk's MFMAs) and its 3 biases. */
typedef struct {
  const float* wf0; const float* b0;       /* conv_layers.0 (128->64): 64 rows */
  const float* wf1; const float* b1;       /* conv_layers.1 (64->32):  32 rows */
  const float* wrgb0; const float* brgb0;  /* conv_rgb.0 (128->3) */
  const float* wrgb1; const float* brgb1;  /* conv_rgb.1 (64->3) */
  const float* wrgb2; const float* brgb2;  /* conv_rgb.2 (32->3) */
  float neg_slope;                         /* 0.2 */
} pnr_neural_render_w;

int pnr_neural_render_scratch_bytes(int32_t H, int32_t W, size_t* out);
int pnr_neural_render_fwd(const float* x, int32_t H, int32_t W, const pnr_neural_render_w* w,
                          float* out_rgb, void* scratch, size_t scratch_bytes, void* stream);

/* Backward of pnr_neural_render_fwd (the autograd of neural_renderer.py:81-104
 * that the reference's finetune step takes through torch convolutions).
 * fwd_scratch = the forward's scratch after that call (net0[H,W,64] then
 * net1[H,W,32]); out_rgb its output; d_out = dL/d out_rgb.  Per stage the
 * data-gradient weights are the stage's stacked [trunk; rgb; zero] rows flipped
 * and transposed: rows = the stage's input channels ci (128 / 64 / 32),
 * columns k = (ky'*3 + kx')*M + j with value Wstack[j][ci][2-ky'][2-kx'],
 * j < M = 96 / 64 / 32 stacked rows (trunk, rgb, zero), frag_pack-ed.
 * Writes d_x[H,W,128] and dw_s = [M, 9*cin] stacked weight gradients (layout of
 * the forward's stacked rows before packing) followed by db_s[M]:
 * dw0 [96*1152 + 96], dw1 [64*576 + 64], dw2 [32*288 + 32].  Fixed-order
 * reductions: bitwise repeatable. */
typedef struct {
  const float* wt0;   /* 128 rows x 9*96 */
  const float* wt1;   /* 64 rows x 9*64 */
  const float* wt2;   /* 32 rows x 9*32 */
  float neg_slope;
} pnr_neural_render_wt;

int pnr_neural_render_bwd_scratch_bytes(int32_t H, int32_t W, size_t* out);
int pnr_neural_render_bwd(const float* x, const float* fwd_scratch, const float* out_rgb, const float* d_out,
                          int32_t H, int32_t W, const pnr_neural_render_wt* wt, float* d_x, float* dw0,
                          float* dw1, float* dw2, void* scratch, size_t scratch_bytes, void* stream);

/* The same renderer, forward and backward, with fp32 accuracy on f16 MFMA
 * (fp32h2, the MLP's split: x = xh + 2^-11 xl per input value, W' = Wh +
 * 2^-11 Wl per weight, three f16 products per 16 k).  Per stage s the stacked
 * [trunk; rgb; 0] rows (96 / 64 / 32 rows, columns k = (ky*3 + kx)*cin + ci)
 * as frag_pack_h2 packs wp_s with their scales ws[s] = 2^(shift - 11) in device
 * memory (pnr_pack_weights_h2_dev: packs rebuilt without a host sync), and the
 * stacked biases b_s (96 / 64 / 32 floats: trunk, rgb, 0).  Each image is
 * staged times a power of two chosen on the device from its max |value|, so
 * any finite input magnitude keeps fp32-level relative accuracy (no range
 * fallback, no host sync).  Scratch: net0[H,W,64], net1[H,W,32], then 256 B of
 * absmax words (the backward reads them from fwd_scratch). */
typedef struct {
  const void* wp0; const void* wp1; const void* wp2;
  const float* ws;                          /* device [6]: stage s's scale at ws[2 s] (pnr_pack_weights_h2_dev's
                                               scale_dev = ws + 2 s; ws[2 s + 1] its scratch) */
  const float* b0; const float* b1; const float* b2;
  float neg_slope;
} pnr_neural_render_h2w;

/* Backward packs: the data-gradient weights of pnr_neural_render_wt (flipped,
 * transposed stacks [128, 9*96], [64, 9*64], [32, 9*32]) as frag_pack_h2 packs
 * with their scales.  Outputs as pnr_neural_render_bwd; data and weight
 * gradients both on fp32h2 (fwd_scratch: pnr_neural_render_fwd_h2's, with its
 * absmax words).  Fixed-order reductions: bitwise repeatable. */
typedef struct {
  const void* wt0; const void* wt1; const void* wt2;
  const float* ws;                          /* device [6], as pnr_neural_render_h2w */
  float neg_slope;
} pnr_neural_render_h2wt;

int pnr_neural_render_h2_scratch_bytes(int32_t H, int32_t W, size_t* out);
int pnr_neural_render_fwd_h2(const float* x, int32_t H, int32_t W, const pnr_neural_render_h2w* w,
                             float* out_rgb, void* scratch, size_t scratch_bytes, void* stream);
int pnr_neural_render_bwd_h2_scratch_bytes(int32_t H, int32_t W, size_t* out);
int pnr_neural_render_bwd_h2(const float* x, const float* fwd_scratch, const float* out_rgb, const float* d_out,
                             int32_t H, int32_t W, const pnr_neural_render_h2wt* wt, float* d_x, float* dw0,
                             float* dw1, float* dw2, void* scratch, size_t scratch_bytes, void* stream);

/* ------------------------------------------------------ upstream RGB head
 * C_out = 3 mode (shading_color_channel_num 3): for v < min(*n_dev, n_max)
 * (n_dev may be NULL), with feat rows of ld >= 129 floats [alpha, f_1..f_128]:
 *   out[v, 0] = feat[v, 0]
 *   out[v, 1 + j] = raw2out_color(sum_c w[j*128 + c] f_c + b[j]),  j < 3
 *   raw2out_color(x) = sigmoid(x) * (1 + 2e-3) - 1e-3 if act_super > 0, else sigmoid(x)
 * Backward: d_feat[v, 0] = d_out[v, 0], d_feat[v, 1 + c] = sum_j g_j w[j, c] for
 * the same rows (other rows untouched); d_wb[3, 129] = (d W | d b), written (not
 * accumulated): PNR_HEAD_BWD_BLOCKS workgroups write per-block partial sums into
 * the caller's partials[PNR_HEAD_BWD_BLOCKS * 3 * 129] floats, which a second
 * launch adds in block order (bitwise repeatable, no float atomics). */
#define PNR_HEAD_BWD_BLOCKS 512
int pnr_rgb_head_fwd(const float* feat, int64_t ld, const int32_t* n_dev, int64_t n_max, const float* w,
                     const float* b, int32_t act_super, float* out, void* stream);
int pnr_rgb_head_bwd(const float* d_out, const float* feat, int64_t ld, const int32_t* n_dev, int64_t n_max,
                     const float* w, const float* b, int32_t act_super, float* d_feat, float* d_wb,
                     float* partials, void* stream);

/* ------------------------------------------------- point-cloud initialisation
 * construct_vox_points_closest(xyz, vox_res) (models/mvs/mvs_utils.py:537-561,
 * space_min = None: the form every reference driver calls, train_ddp.py:135):
 * the cube of edge max(max - min) * 1.05 around the points' bbox centre cut in
 * vox_res^3 voxels (torch's fp32 op order), the occupied voxels in
 * lexicographic (x, y, z) order (torch.unique(dim=0)).  For voxel v < counts[0]:
 * grid_idx[v,3] its cell, centroid[v,3] = mean of its points (summed in ascending
 * point order, scatter_mean), min_idx[v] = its point closest to the centroid
 * (scatter_min; ties to the smallest index).  inv_idx[N] (may be NULL) = voxel
 * of every point.  Outputs sized for N voxels; counts[0] = voxels, counts[1] = 1
 * when a cell coordinate left +-2^20 (outputs invalid).  No host sync. */
int pnr_vox_closest_scratch_bytes(int64_t n, size_t* out);
int pnr_vox_closest(const float* xyz_dev, int64_t n, int32_t vox_res, float* centroid, int32_t* grid_idx,
                    int64_t* min_idx, int32_t* inv_idx, int32_t* counts, void* scratch, size_t scratch_bytes,
                    void* stream);

/* ------------------------------------------------------------- optimizer */
/* One Adam step (torch.optim.Adam, amsgrad = False: the optimizer of the
 * reference's training loop, train_ddp.py / mvs_points_volumetric_model.py:102-123)
 * over n_tensors contiguous fp32 tensors: params[i], grads[i], exp_avg[i],
 * exp_avg_sq[i] of numel[i] elements each (device pointers; the tables
 * themselves are host arrays).  `step` is the 1-based step count of all of them
 * (bias corrections 1 - beta^step and 1 - beta in double on the host, as torch's
 * python-float hyperparameters, then rounded to fp32).  Updates params, exp_avg,
 * exp_avg_sq in place; no host sync. */
int pnr_adam_step(int32_t n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, const int64_t* numel, double lr, double beta1, double beta2,
                  double eps, double weight_decay, int64_t step, void* stream);

/* ------------------------------------------------------------- utilities */
/* Diagnostics: out_dev[0] = the shader clock (MHz) one wave measured over
 * `spins` s_sleep slices (s_memtime cycles / s_memrealtime 100 MHz ticks);
 * launched beside running kernels it reports the clock under that load. */
int pnr_clock_probe(float* out_dev, int32_t spins, void* stream);

/* Exclusive scan of n int32 values (n_dev: optional device-side length <= n,
 * entries past it are treated as 0 and out[] is written up to n_dev+1);
 * total written to *total_dev (may be NULL).  out_len: int32 entries at out,
 * at least n + 1 (the total is also stored at out[n_eff]); PNR_EINVAL otherwise
 * (ABI 21). */
int pnr_scan_scratch_bytes(int64_t n, size_t* out);
int pnr_exclusive_scan_i32(const int32_t* in, int64_t n, const int32_t* n_dev, int32_t* out, int64_t out_len,
                           int32_t* total_dev, void* scratch, size_t scratch_bytes,
                           void* stream);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* PNR_H_ */
