/*
 * TEST INFRASTRUCTURE ONLY -- the CPU oracle for the world-coordinate query.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline; the product
 * path (pointnerf_amd) never calls it.
 *
 * A plain-C, single-threaded restatement of the reference's query kernels,
 * executed in the serial order of their thread indices (one legal schedule of
 * the parallel kernels; the only schedule with a defined result):
 *   claim_occ            query_point_indices_worldcoords.py:243-303
 *   map_coor2occ         query_point_indices_worldcoords.py:305-340
 *   fill_occ2pnts        query_point_indices_worldcoords.py:342-387
 *   mask_raypos          query_point_indices_worldcoords.py:390-414
 *   cumsum SR pick + get_shadingloc  query_point_indices_worldcoords.py:655-677, 417-439
 *   query_neigh_along_ray_layered    query_point_indices_worldcoords.py:442-528
 * Overflow (qpiw.py:289-298, 377-384): the reference replaces slots with
 * reservoir sampling (Algorithm R, curand seeded with time()), whose result is
 * a uniform random subset -- max_o of the occupied voxels, P of a voxel's
 * points -- with no reproducible draw.  Oracle and library draw the same
 * uniform subsets from a seeded hash instead ("seeded reservoir"): the kept
 * voxels are the max_o with the smallest key (hash32(seed, first point) << 32
 * | first point), numbered in first-point order; a voxel keeps the P points
 * with the smallest key (hash32(seed + PNR_PT_SALT, id) << 32 | id), in
 * ascending index order.  Without overflow both reduce to the serial order.
 *
 * Parity status: the reference's query is CUDA C inside a Python string that
 * pycuda JIT-compiles; it needs cuda.h / curand_kernel.h / pycuda, none of
 * which exist in this image, so it cannot be executed here.  This restatement
 * is therefore pinned by (a) golden vectors of the reference's own ray
 * generation (tests/golden) that fix every candidate position bit for bit and
 * (b) property tests against an independent brute-force statement of the same
 * search (tests/test_oracle_query.py).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: IEEE fp32, no FMA).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <string.h>

static int vox(float p, float shift, float vs) { return (int)floorf((p - shift) / vs); }

/* the seeded reservoir's keys (same integer arithmetic as pnr_common.h) */
#define PNR_PT_SALT 0x632BE59BD9B4E019ull
static uint32_t hash32(uint64_t seed, uint32_t id) {
  uint64_t z = seed ^ ((uint64_t)id * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
static uint64_t vkey(uint64_t seed, uint32_t id) { return ((uint64_t)hash32(seed, id) << 32) | id; }
static uint64_t pkey(uint64_t seed, uint32_t id) { return ((uint64_t)hash32(seed + PNR_PT_SALT, id) << 32) | id; }
static int cmp_u64(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}
static int cmp_i32(const void* a, const void* b) {
  int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
  return x < y ? -1 : x > y;
}

/* Grid tables (serial claim_occ -> map_coor2occ -> fill_occ2pnts, seeded
 * reservoir on overflow).  coor_2_occ[gvol] (-1 empty), coor_occ[gvol] (0/1
 * dilated), occ_numpnts[max_o] (points that reached the voxel, as the
 * reference's counter: may exceed P), occ_2_pnts[max_o*P] (-1); returns the
 * number of occupied voxels (occ_idx, before the max_o cut). */
int64_t oracle_grid_build(const float* xyz, int64_t n, const float shift[3], const float vs[3],
                          const int dims[3], const int qs[3], int max_o, int P, int slot0_drop, uint64_t seed,
                          int32_t* coor_2_occ, uint8_t* coor_occ, int32_t* occ_numpnts,
                          int32_t* occ_2_pnts) {
  const int64_t gvol = (int64_t)dims[0] * dims[1] * dims[2];
  int64_t* pcell = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int32_t* first = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1)); /* first point of voxel v */
  for (int64_t i = 0; i < gvol; ++i) {
    coor_2_occ[i] = -1;
    coor_occ[i] = 0;
  }
  for (int64_t i = 0; i < max_o; ++i) occ_numpnts[i] = 0;
  for (int64_t i = 0; i < (int64_t)max_o * P; ++i) occ_2_pnts[i] = -1;
  int64_t occ_idx = 0;
  /* claim_occ: voxels in first-point order (coor_2_occ temporarily = voxel number) */
  for (int64_t i = 0; i < n; ++i) {
    int c[3];
    for (int a = 0; a < 3; ++a) c[a] = vox(xyz[i * 3 + a], shift[a], vs[a]);
    pcell[i] = -1;
    if (c[0] < 0 || c[0] >= dims[0] || c[1] < 0 || c[1] >= dims[1] || c[2] < 0 || c[2] >= dims[2])
      continue;
    int64_t cell = ((int64_t)c[0] * dims[1] + c[1]) * dims[2] + c[2];
    pcell[i] = cell;
    if (coor_2_occ[cell] == -1) {
      coor_2_occ[cell] = (int32_t)occ_idx;
      first[occ_idx++] = (int32_t)i;
    }
  }
  /* reservoir over the voxels: keep the max_o smallest keys */
  uint64_t thr = ~0ull;
  if (occ_idx > max_o) {
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)occ_idx);
    for (int64_t v = 0; v < occ_idx; ++v) keys[v] = vkey(seed, (uint32_t)first[v]);
    qsort(keys, (size_t)occ_idx, sizeof(uint64_t), cmp_u64);
    thr = keys[max_o - 1];
    free(keys);
  }
  for (int64_t i = 0; i < gvol; ++i) coor_2_occ[i] = -1; /* qpiw.py:575 */
  /* map_coor2occ: kept voxels numbered in first-point order, dilation by query_size */
  int64_t s = 0;
  for (int64_t v = 0; v < occ_idx; ++v) {
    if (vkey(seed, (uint32_t)first[v]) > thr) continue;
    const int64_t cell = pcell[first[v]];
    const int c0 = (int)(cell / ((int64_t)dims[1] * dims[2])), c1 = (int)((cell / dims[2]) % dims[1]),
              c2 = (int)(cell % dims[2]);
    coor_2_occ[cell] = (int32_t)s++;
    int x0 = c0 - qs[0] / 2 > 0 ? c0 - qs[0] / 2 : 0;
    int x1 = c0 + (qs[0] + 1) / 2 < dims[0] ? c0 + (qs[0] + 1) / 2 : dims[0];
    int y0 = c1 - qs[1] / 2 > 0 ? c1 - qs[1] / 2 : 0;
    int y1 = c1 + (qs[1] + 1) / 2 < dims[1] ? c1 + (qs[1] + 1) / 2 : dims[1];
    int z0 = c2 - qs[2] / 2 > 0 ? c2 - qs[2] / 2 : 0;
    int z1 = c2 + (qs[2] + 1) / 2 < dims[2] ? c2 + (qs[2] + 1) / 2 : dims[2];
    for (int x = x0; x < x1; ++x)
      for (int y = y0; y < y1; ++y)
        for (int z = z0; z < z1; ++z) coor_occ[((int64_t)x * dims[1] + y) * dims[2] + z] = 1;
  }
  /* fill_occ2pnts: every point of a kept voxel (ascending index) ... */
  const int64_t nk = s;
  int64_t* off = (int64_t*)calloc((size_t)nk + 1, sizeof(int64_t));
  for (int64_t i = 0; i < n; ++i) {
    if (pcell[i] < 0) continue;
    int32_t v = coor_2_occ[pcell[i]];
    if (slot0_drop ? (v > 0) : (v >= 0)) ++off[v + 1];
  }
  for (int64_t v = 0; v < nk; ++v) off[v + 1] += off[v];
  int32_t* ids = (int32_t*)malloc(sizeof(int32_t) * (size_t)(off[nk] > 0 ? off[nk] : 1));
  for (int64_t i = 0; i < n; ++i) {
    if (pcell[i] < 0) continue;
    int32_t v = coor_2_occ[pcell[i]];
    if (slot0_drop ? (v > 0) : (v >= 0)) ids[off[v] + occ_numpnts[v]++] = (int32_t)i;
  }
  /* ... of which a voxel keeps P: the P smallest point keys, ascending index */
  for (int64_t v = 0; v < nk; ++v) {
    const int64_t cnt = off[v + 1] - off[v];
    int32_t* vi = ids + off[v];
    if (cnt > P) {
      uint64_t* k = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)cnt);
      for (int64_t j = 0; j < cnt; ++j) k[j] = pkey(seed, (uint32_t)vi[j]);
      qsort(k, (size_t)cnt, sizeof(uint64_t), cmp_u64);
      for (int j = 0; j < P; ++j) vi[j] = (int32_t)(k[j] & 0xffffffffu);
      qsort(vi, (size_t)P, sizeof(int32_t), cmp_i32);
      free(k);
    }
    for (int j = 0; j < cnt && j < P; ++j) occ_2_pnts[v * P + j] = vi[j];
  }
  free(ids);
  free(off);
  free(first);
  free(pcell);
  return occ_idx;
}

/* mask_raypos + first-SR pick: n_filled[R], slot_d[R*SR] (candidate index). */
void oracle_ray_march(const float campos[3], const float* raydir, int64_t R, const float* tvals,
                      int tvals_per_ray, int D, int SR, const float shift[3], const float vs[3],
                      const int dims[3], const uint8_t* coor_occ, int32_t* n_filled,
                      int32_t* slot_d) {
  /* rays are independent (one thread per ray in the reference): parallel over rays */
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t r = 0; r < R; ++r) {
    int cnt = 0;
    const float* tv = tvals + (tvals_per_ray ? r * D : 0);
    for (int d = 0; d < D && cnt < SR; ++d) {
      int c[3];
      for (int a = 0; a < 3; ++a) {
        float p = campos[a] + raydir[r * 3 + a] * tv[d];
        c[a] = vox(p, shift[a], vs[a]);
      }
      if (c[0] < 0 || c[0] >= dims[0] || c[1] < 0 || c[1] >= dims[1] || c[2] < 0 || c[2] >= dims[2])
        continue;
      if (coor_occ[((int64_t)c[0] * dims[1] + c[1]) * dims[2] + c[2]]) slot_d[r * SR + cnt++] = d;
    }
    n_filled[r] = cnt;
  }
}

/* query_neigh_along_ray_layered for n_samples sample positions loc[n,3];
 * pidx[n*K] (-1 = empty).  Returns the number of (sample, neighbour) pairs. */
int64_t oracle_knn(const float* xyz, const float* loc, int64_t n_samples, const float shift[3],
                   const float vs[3], const int dims[3], const int ks[3], int K, int P,
                   float radius_limit2, const int32_t* coor_2_occ, const int32_t* occ_numpnts,
                   const int32_t* occ_2_pnts, int32_t* pidx) {
  int64_t pairs = 0;
  /* samples are independent (one thread per sample in the reference) */
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : pairs)
  for (int64_t s = 0; s < n_samples; ++s) {
    float buf[64];
    const float cx = loc[s * 3], cy = loc[s * 3 + 1], cz = loc[s * 3 + 2];
    const int fx = vox(cx, shift[0], vs[0]), fy = vox(cy, shift[1], vs[1]), fz = vox(cz, shift[2], vs[2]);
    int32_t* out = pidx + s * K;
    for (int i = 0; i < K; ++i) out[i] = -1;
    int kid = 0, far_ind = 0;
    float far2 = 0.f;
    for (int layer = 0; layer < (ks[0] + 1) / 2; ++layer) {
      int xa = -fx > -layer ? -fx : -layer, xb = dims[0] - fx < layer + 1 ? dims[0] - fx : layer + 1;
      int ya = -fy > -layer ? -fy : -layer, yb = dims[1] - fy < layer + 1 ? dims[1] - fy : layer + 1;
      int za = -fz > -layer ? -fz : -layer, zb = dims[2] - fz < layer + 1 ? dims[2] - fz : layer + 1;
      for (int x = xa; x < xb; ++x) {
        for (int y = ya; y < yb; ++y) {
          for (int z = za; z < zb; ++z) {
            int ax = abs(x), ay = abs(y), az = abs(z);
            int mx = ax > ay ? ax : ay;
            mx = mx > az ? mx : az;
            if (mx != layer) continue;
            int32_t occ = coor_2_occ[((int64_t)(fx + x) * dims[1] + (fy + y)) * dims[2] + (fz + z)];
            if (occ < 0) continue;
            int cnt = occ_numpnts[occ] < P ? occ_numpnts[occ] : P;
            for (int g = 0; g < cnt; ++g) {
              int32_t pi = occ_2_pnts[(int64_t)occ * P + g];
              float xv = xyz[(int64_t)pi * 3] - cx;
              float yv = xyz[(int64_t)pi * 3 + 1] - cy;
              float zv = xyz[(int64_t)pi * 3 + 2] - cz;
              float d2 = xv * xv + yv * yv + zv * zv;
              if (!(radius_limit2 == 0.f || d2 <= radius_limit2)) continue;
              if (kid++ < K) {
                out[kid - 1] = pi;
                buf[kid - 1] = d2;
                if (d2 > far2) {
                  far2 = d2;
                  far_ind = kid - 1;
                }
              } else if (d2 < far2) {
                out[far_ind] = pi;
                buf[far_ind] = d2;
                far2 = d2;
                for (int i = 0; i < K; ++i) {
                  if (buf[i] > far2) {
                    far2 = buf[i];
                    far_ind = i;
                  }
                }
              }
            }
          }
        }
      }
      if (kid >= K) break;
    }
    pairs += kid < K ? kid : K;
  }
  return pairs;
}

/* OpenMP thread count of the ray / sample loops (the grid build stays serial:
 * its slot order is the serial schedule). */
void oracle_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}
