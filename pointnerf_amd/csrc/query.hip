// World-coordinate neural-point query: candidate march, first-SR pick,
// layered K-nearest search, and the R -> R' -> R'' compactions.
//
// Replaces query_grid_point_index (query_point_indices_worldcoords.py:614-721):
//   mask_raypos (qpiw.py:390-414)          -> k_march (bitmap probe, early exit at SR)
//   cumsum slot pick + get_shadingloc       -> k_march writes slot s of the first SR
//     (qpiw.py:655-677, 417-439)               occupied candidates directly
//   query_neigh_along_ray_layered           -> k_knn (same traversal order, same
//     (qpiw.py:442-528)                        K-buffer replacement rule)
//   masked_select / masked_scatter_          -> device scans (scan.hip), no host sync
//     (qpiw.py:655-661, 715-719)
// Positions are recomputed from (ray, candidate index) with the reference's
// fp32 operation order, so every kernel sees bit-identical sample positions
// without materialising raypos[R,400,3] (3.1 GB for an 800^2 frame).
#include "pnr_common.h"

namespace pnr {

constexpr int kQBlock = 256;

struct QGrid {
  float shift[3], vs[3];
  int dims[3];
  int P;
};

struct QRays {
  const float* campos;
  const float* camrot;
  const float* raydir;
  const float* tvals;
  int64_t R;
  int D;
  int per_ray;
};

__device__ __forceinline__ float tval(const QRays& q, int64_t r, int d) {
  return q.tvals[(q.per_ray ? r * q.D : 0) + d];
}

__device__ __forceinline__ void ray_point(const float c[3], const float dir[3], float t, float p[3]) {
  p[0] = ray_at(c[0], dir[0], t);
  p[1] = ray_at(c[1], dir[1], t);
  p[2] = ray_at(c[2], dir[2], t);
}

// mask_raypos + SR pick: the first SR candidates whose cell is set in the
// dilated occupancy (qpiw.py:406-413, 664-665).
__global__ void __launch_bounds__(kQBlock) k_march(QRays q, QGrid g, int SR,
                                                   const uint32_t* __restrict__ occ_bits,
                                                   int32_t* __restrict__ n_filled,
                                                   uint16_t* __restrict__ slot_d) {
  const float c[3] = {q.campos[0], q.campos[1], q.campos[2]};
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < q.R;
       r += (int64_t)gridDim.x * blockDim.x) {
    const float dir[3] = {q.raydir[r * 3], q.raydir[r * 3 + 1], q.raydir[r * 3 + 2]};
    int n = 0;
    for (int d = 0; d < q.D && n < SR; ++d) {
      float p[3];
      ray_point(c, dir, tval(q, r, d), p);
      const int x = vox_coord(p[0], g.shift[0], g.vs[0]);
      const int y = vox_coord(p[1], g.shift[1], g.vs[1]);
      const int z = vox_coord(p[2], g.shift[2], g.vs[2]);
      if (x < 0 || x >= g.dims[0] || y < 0 || y >= g.dims[1] || z < 0 || z >= g.dims[2]) continue;
      const int64_t id = ((int64_t)x * g.dims[1] + y) * g.dims[2] + z;
      if ((occ_bits[id >> 5] >> (id & 31)) & 1u) {
        slot_d[r * SR + n] = (uint16_t)d;
        ++n;
      }
    }
    n_filled[r] = n;
  }
}

__global__ void __launch_bounds__(kQBlock) k_fill_list(int64_t R, int SR, const int32_t* __restrict__ n_filled,
                                                       const int32_t* __restrict__ ray_off,
                                                       int32_t* __restrict__ fill_rs, int32_t* counts) {
  int hit = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < R;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int n = n_filled[r], off = ray_off[r];
    for (int s = 0; s < n; ++s) fill_rs[off + s] = (int)(r * SR + s);
    hit += n > 0;
  }
  hit = wave_sum_i32(hit);
  if ((threadIdx.x & 63) == 0 && hit) atomicAdd(counts + 2, hit);
}

// One accepted-or-rejected candidate record of query_neigh_along_ray_layered
// (qpiw.py:494-518): radius test, fill phase, then strict-closer replacement of
// the first farthest entry.
template <int KMAX>
__device__ __forceinline__ void knn_visit(const float4 v, const float p[3], int K, float r2, float buf[KMAX],
                                          int32_t out[KMAX], int& kid, int& far_ind, float& far2) {
  const float xv = __fsub_rn(v.x, p[0]);
  const float yv = __fsub_rn(v.y, p[1]);
  const float zv = __fsub_rn(v.z, p[2]);
  const float d2 = __fadd_rn(__fadd_rn(__fmul_rn(xv, xv), __fmul_rn(yv, yv)), __fmul_rn(zv, zv));
  if (!(r2 == 0.f || d2 <= r2)) return;
  const int pid = __float_as_int(v.w);
  if (kid < K) {
    // fill phase (qpiw.py:500-506)
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      if (i == kid) {
        out[i] = pid;
        buf[i] = d2;
      }
    }
    if (d2 > far2) {
      far2 = d2;
      far_ind = kid;
    }
    ++kid;
  } else {
    ++kid;
    // replace phase (qpiw.py:507-518): strictly closer than the
    // current farthest, then rescan for the first maximum.
    if (d2 < far2) {
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        if (i == far_ind) {
          out[i] = pid;
          buf[i] = d2;
        }
      }
      far2 = d2;
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        if (i < K && buf[i] > far2) {
          far2 = buf[i];
          far_ind = i;
        }
      }
    }
  }
}

// All records of one occupied voxel, in slot order, fetched 4 at a time
// (memory-level parallelism) and visited in order.
template <int KMAX>
__device__ __forceinline__ void knn_cell(const float4* __restrict__ rec, int cnt, const float p[3], int K, float r2,
                                         float buf[KMAX], int32_t out[KMAX], int& kid, int& far_ind, float& far2) {
  for (int g0 = 0; g0 < cnt; g0 += 4) {
    float4 vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) vb[u] = g0 + u < cnt ? rec[g0 + u] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (g0 + u >= cnt) break;
      knn_visit<KMAX>(vb[u], p, K, r2, buf, out, kid, far_ind, far2);
    }
  }
}

// query_neigh_along_ray_layered (qpiw.py:442-528) for one sample.  KMAX is the
// compile-time buffer size, K <= KMAX the runtime neighbour count.
template <int KMAX>
__device__ __forceinline__ int knn_one(const float p[3], const QGrid& g, int K, int layers, float r2,
                                       const int32_t* __restrict__ coor_2_occ,
                                       const int32_t* __restrict__ occ_numpnts,
                                       const float4* __restrict__ occ_pts, int32_t out[KMAX],
                                       int& n_cand) {
  const int fx = vox_coord(p[0], g.shift[0], g.vs[0]);
  const int fy = vox_coord(p[1], g.shift[1], g.vs[1]);
  const int fz = vox_coord(p[2], g.shift[2], g.vs[2]);
  float buf[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    buf[i] = 0.f;
    out[i] = -1;
  }
  int kid = 0, far_ind = 0;
  float far2 = 0.f;
  if (layers == 2) {
    // query 3x3x3 (every shipped config): the 27 cells in the reference's
    // traversal order (layer 0 = the centre, then layer 1 = x -> y -> z minus the
    // centre).  The slot and count lookups of all 27 cells are issued together
    // instead of as 27 dependent chains; the visit order is unchanged.
    int slot[27], cnt[27];
#pragma unroll
    for (int j = 0; j < 27; ++j) {
      const int x = j == 0 ? 0 : ((j <= 13 ? j - 1 : j) / 9) - 1;
      const int y = j == 0 ? 0 : (((j <= 13 ? j - 1 : j) / 3) % 3) - 1;
      const int z = j == 0 ? 0 : ((j <= 13 ? j - 1 : j) % 3) - 1;
      const int cx = fx + x, cy = fy + y, cz = fz + z;
      const bool in = (unsigned)cx < (unsigned)g.dims[0] && (unsigned)cy < (unsigned)g.dims[1] &&
                      (unsigned)cz < (unsigned)g.dims[2];
      slot[j] = in ? coor_2_occ[((int64_t)cx * g.dims[1] + cy) * g.dims[2] + cz] : -1;
    }
#pragma unroll
    for (int j = 0; j < 27; ++j) cnt[j] = slot[j] >= 0 ? min(g.P, occ_numpnts[slot[j]]) : 0;
#pragma unroll
    for (int j = 0; j < 27; ++j) {
      if (j == 1 && kid >= K) break;   // layer 0 already saw >= K candidates (qpiw.py:526)
      n_cand += cnt[j];
      knn_cell<KMAX>(occ_pts + (int64_t)max(slot[j], 0) * g.P, cnt[j], p, K, r2, buf, out, kid, far_ind, far2);
    }
    return kid < K ? kid : K;
  }
  for (int layer = 0; layer < layers; ++layer) {
    const int x0 = max(-fx, -layer), x1 = min(g.dims[0] - fx, layer + 1);
    const int y0 = max(-fy, -layer), y1 = min(g.dims[1] - fy, layer + 1);
    const int z0 = max(-fz, -layer), z1 = min(g.dims[2] - fz, layer + 1);
    for (int x = x0; x < x1; ++x) {
      for (int y = y0; y < y1; ++y) {
        for (int z = z0; z < z1; ++z) {
          if (max(abs(z), max(abs(x), abs(y))) != layer) continue;
          const int64_t cell = ((int64_t)(fx + x) * g.dims[1] + (fy + y)) * g.dims[2] + (fz + z);
          const int slot = coor_2_occ[cell];
          if (slot < 0) continue;
          const int cnt = min(g.P, occ_numpnts[slot]);
          n_cand += cnt;
          knn_cell<KMAX>(occ_pts + (int64_t)slot * g.P, cnt, p, K, r2, buf, out, kid, far_ind, far2);
        }
      }
    }
    if (kid >= K) break;
  }
  return kid < K ? kid : K;
}

template <int KMAX>
__global__ void __launch_bounds__(kQBlock) k_knn(QRays q, QGrid g, int SR, int K, int layers, float r2,
                                                 const int32_t* __restrict__ coor_2_occ,
                                                 const int32_t* __restrict__ occ_numpnts,
                                                 const float4* __restrict__ occ_pts,
                                                 const uint16_t* __restrict__ slot_d,
                                                 const int32_t* __restrict__ fill_rs,
                                                 int32_t* __restrict__ pidx, int32_t* __restrict__ vflag,
                                                 int32_t* __restrict__ ray_vcnt,
                                                 float* __restrict__ sample_w,
                                                 float* __restrict__ sample_p, int32_t* counts) {
  const int64_t S = counts[0];
  const float c[3] = {q.campos[0], q.campos[1], q.campos[2]};
  float Rm[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rm[i] = q.camrot[i];
  int pairs = 0, n_cand = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < S;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int rs = fill_rs[i];
    const int64_t r = rs / SR;
    const int d = slot_d[rs];
    const float dir[3] = {q.raydir[r * 3], q.raydir[r * 3 + 1], q.raydir[r * 3 + 2]};
    float p[3], pp[3];
    ray_point(c, dir, tval(q, r, d), p);
    world_to_pers(p, c, Rm, pp);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      sample_w[i * 3 + a] = p[a];
      sample_p[i * 3 + a] = pp[a];
    }
    int32_t out[KMAX];
    const int nk = knn_one<KMAX>(p, g, K, layers, r2, coor_2_occ, occ_numpnts, occ_pts, out, n_cand);
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int j = 0; j < KMAX; ++j)
        if (j == k) pidx[i * K + k] = out[j];
    }
    vflag[i] = nk > 0;
    if (nk > 0) atomicAdd(ray_vcnt + r, 1);
    pairs += nk;
  }
  pairs = wave_sum_i32(pairs);
  n_cand = wave_sum_i32(n_cand);
  if ((threadIdx.x & 63) == 0 && pairs) atomicAdd(counts + 4, pairs);
  // candidate records read (measurement only): int64 in counts[6..7]
  if ((threadIdx.x & 63) == 0 && n_cand)
    atomicAdd(reinterpret_cast<unsigned long long*>(counts + 6), (unsigned long long)n_cand);
}

__global__ void __launch_bounds__(kQBlock) k_valid_list(const int32_t* __restrict__ vflag,
                                                        const int32_t* __restrict__ valid_off,
                                                        int32_t* __restrict__ valid_list,
                                                        const int32_t* counts) {
  const int64_t S = counts[0];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < S;
       i += (int64_t)gridDim.x * blockDim.x)
    if (vflag[i]) valid_list[valid_off[i]] = (int)i;
}

// Reference-shaped query_points outputs for the R'' rays (qpiw.py:97-99, 715-719).
__global__ void __launch_bounds__(kQBlock) k_compact(QRays q, int SR, int K, int64_t rows_max,
                                                     const int32_t* __restrict__ n_filled,
                                                     const int32_t* __restrict__ ray_off,
                                                     const int32_t* __restrict__ ray_vcnt,
                                                     const int32_t* __restrict__ ray_row,
                                                     const int32_t* __restrict__ pidx,
                                                     const float* __restrict__ sample_w,
                                                     const float* __restrict__ sample_p,
                                                     int32_t* __restrict__ o_pidx, float* __restrict__ o_loc,
                                                     float* __restrict__ o_loc_w,
                                                     float* __restrict__ o_dirs, int8_t* __restrict__ ray_mask) {
  const float c[3] = {q.campos[0], q.campos[1], q.campos[2]};
  float Rm[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rm[i] = q.camrot[i];
  const float zero[3] = {0.f, 0.f, 0.f};
  float origin_p[3];
  world_to_pers(zero, c, Rm, origin_p);
  const int64_t total = q.R * SR;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / SR;
    const int s = (int)(e - r * SR);
    const bool m = ray_vcnt[r] > 0;
    if (s == 0) ray_mask[r] = m ? 1 : 0;
    if (!m) continue;
    const int64_t j = ray_row[r];
    if (j >= rows_max) continue;
    const int64_t o = j * SR + s;
    if (s < n_filled[r]) {
      const int64_t i = ray_off[r] + s;
      for (int k = 0; k < K; ++k) o_pidx[o * K + k] = pidx[i * K + k];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        o_loc_w[o * 3 + a] = sample_w[i * 3 + a];
        o_loc[o * 3 + a] = sample_p[i * 3 + a];
      }
    } else {
      for (int k = 0; k < K; ++k) o_pidx[o * K + k] = -1;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        o_loc_w[o * 3 + a] = 0.f;
        o_loc[o * 3 + a] = origin_p[a];
      }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) o_dirs[o * 3 + a] = q.raydir[r * 3 + a];
  }
}

QRays to_qrays(const pnr_rays* r) {
  QRays q;
  q.campos = r->campos_dev;
  q.camrot = r->camrot_dev;
  q.raydir = r->raydir_dev;
  q.tvals = r->tvals_dev;
  q.R = r->R;
  q.D = r->D;
  q.per_ray = r->tvals_per_ray;
  return q;
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_query_scratch_bytes(int64_t R, int32_t SR, size_t* out) {
  PNR_CHECK_ARG(out && R >= 0 && SR > 0, "query_scratch_bytes: bad args");
  *out = scan_scratch_bytes(R * SR + 1);
  return PNR_OK;
}

static int check_rays(const pnr_rays* r) {
  PNR_CHECK_ARG(r && r->campos_dev && r->camrot_dev && r->raydir_dev && r->tvals_dev,
                "rays: null pointer");
  PNR_CHECK_ARG(r->R >= 0 && r->D > 0 && r->D <= 65535, "rays: R=%lld D=%d out of range",
                (long long)r->R, r->D);
  return PNR_OK;
}

extern "C" int pnr_query(pnr_handle* h, const pnr_rays* rays, const pnr_query_params* qp,
                         pnr_query_bufs* b, void* stream) {
  int rc;
  PNR_CHECK_ARG(h && qp && b, "query: null pointer");
  if ((rc = check_rays(rays))) return rc;
  PNR_CHECK_ARG(h->built, "query: grid not built (call pnr_grid_build first)");
  PNR_CHECK_ARG(qp->SR > 0 && qp->K >= 1 && qp->K <= 32, "query: SR=%d K=%d unsupported", qp->SR, qp->K);
  PNR_CHECK_ARG(rays->R * qp->SR < ((int64_t)1 << 31), "query: R*SR exceeds int32 sample ids");
  PNR_CHECK_ARG(b->n_filled && b->slot_d && b->ray_off && b->fill_rs && b->pidx && b->valid_off &&
                    b->valid_list && b->vflag && b->ray_vcnt && b->ray_row && b->sample_w &&
                    b->sample_p && b->counts && b->scratch,
                "query: null buffer");
  const int64_t R = rays->R, RS = R * qp->SR;
  PNR_CHECK_ARG(b->scratch_bytes >= scan_scratch_bytes(RS + 1), "query: scratch too small");
  hipStream_t st = as_stream(stream);
  QRays q = to_qrays(rays);
  QGrid g;
  for (int a = 0; a < 3; ++a) {
    g.shift[a] = h->gp.shift[a];
    g.vs[a] = h->gp.vsize[a];
    g.dims[a] = h->gp.dims[a];
  }
  g.P = h->gp.P;
  PNR_HIP(hipMemsetAsync(b->counts, 0, 8 * sizeof(int32_t), st));
  PNR_HIP(hipMemsetAsync(b->ray_vcnt, 0, (size_t)(R > 0 ? R : 1) * sizeof(int32_t), st));
  if (R == 0) {
    PNR_HIP(hipMemsetAsync(b->ray_off, 0, sizeof(int32_t), st));
    PNR_HIP(hipMemsetAsync(b->ray_row, 0, sizeof(int32_t), st));
    PNR_HIP(hipMemsetAsync(b->valid_off, 0, sizeof(int32_t), st));
    return PNR_OK;
  }
  hipLaunchKernelGGL(k_march, dim3(grid_for(R, kQBlock)), dim3(kQBlock), 0, st, q, g, qp->SR,
                     h->occ_bits.as<uint32_t>(), b->n_filled, b->slot_d);
  PNR_LAUNCH_CHECK();
  if ((rc = exclusive_scan(b->n_filled, R, nullptr, b->ray_off, b->counts + 0, b->scratch,
                           b->scratch_bytes, st)))
    return rc;
  hipLaunchKernelGGL(k_fill_list, dim3(grid_for(R, kQBlock)), dim3(kQBlock), 0, st, R, qp->SR,
                     b->n_filled, b->ray_off, b->fill_rs, b->counts);
  PNR_LAUNCH_CHECK();
  const int layers = (qp->kernel_size[0] + 1) / 2;
  const unsigned gk = grid_for(RS, kQBlock, 256 * 16);
#define PNR_KNN(KM)                                                                              \
  hipLaunchKernelGGL(k_knn<KM>, dim3(gk), dim3(kQBlock), 0, st, q, g, qp->SR, qp->K, layers,      \
                     qp->radius_limit2, h->coor_2_occ.as<int32_t>(), h->occ_numpnts.as<int32_t>(), \
                     h->occ_pts.as<float4>(), b->slot_d, b->fill_rs, b->pidx, b->vflag,           \
                     b->ray_vcnt, b->sample_w, b->sample_p, b->counts)
  if (qp->K <= 8) PNR_KNN(8);
  else if (qp->K <= 16) PNR_KNN(16);
  else PNR_KNN(32);
#undef PNR_KNN
  PNR_LAUNCH_CHECK();
  if ((rc = exclusive_scan(b->vflag, RS, b->counts + 0, b->valid_off, b->counts + 1, b->scratch,
                           b->scratch_bytes, st)))
    return rc;
  hipLaunchKernelGGL(k_valid_list, dim3(grid_for(RS, kQBlock)), dim3(kQBlock), 0, st, b->vflag,
                     b->valid_off, b->valid_list, b->counts);
  PNR_LAUNCH_CHECK();
  if ((rc = exclusive_scan(b->ray_vcnt, R, nullptr, b->ray_row, b->counts + 3, b->scratch,
                           b->scratch_bytes, st, /*as_flag=*/1)))
    return rc;
  return PNR_OK;
}

extern "C" int pnr_query_compact(const pnr_rays* rays, const pnr_query_params* qp,
                                 const pnr_query_bufs* b, int64_t rows_max, int32_t* sample_pidx,
                                 float* sample_loc, float* sample_loc_w, float* sample_ray_dirs,
                                 int8_t* ray_mask, void* stream) {
  int rc;
  if ((rc = check_rays(rays))) return rc;
  PNR_CHECK_ARG(qp && b && ray_mask, "query_compact: null pointer");
  PNR_CHECK_ARG(rows_max == 0 || (sample_pidx && sample_loc && sample_loc_w && sample_ray_dirs),
                "query_compact: null output");
  if (rays->R == 0) return PNR_OK;
  hipStream_t st = as_stream(stream);
  QRays q = to_qrays(rays);
  const int64_t total = rays->R * qp->SR;
  hipLaunchKernelGGL(k_compact, dim3(grid_for(total, kQBlock)), dim3(kQBlock), 0, st, q, qp->SR, qp->K,
                     rows_max, b->n_filled, b->ray_off, b->ray_vcnt, b->ray_row, b->pidx, b->sample_w,
                     b->sample_p, sample_pidx, sample_loc, sample_loc_w, sample_ray_dirs, ray_mask);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
