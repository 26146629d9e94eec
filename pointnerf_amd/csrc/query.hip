// World-coordinate neural-point query: candidate march, first-SR pick,
// layered K-nearest search, and the R -> R' -> R'' compactions.
//
// Replaces query_grid_point_index (query_point_indices_worldcoords.py:614-721):
//   mask_raypos (qpiw.py:390-414)          -> k_march_coop (bitmap probe, early exit at SR)
//   cumsum slot pick + get_shadingloc       -> k_march_coop writes slot s of the first SR
//     (qpiw.py:655-677, 417-439)               occupied candidates directly
//   query_neigh_along_ray_layered           -> k_knn (same traversal order, same
//     (qpiw.py:442-528)                        K-buffer replacement rule)
//   masked_select / masked_scatter_          -> device scans (scan.hip), no host sync
//     (qpiw.py:655-661, 715-719)
// Positions are recomputed from (ray, candidate index) with the reference's
// fp32 operation order, so every kernel sees bit-identical sample positions
// without materialising raypos[R,400,3] (3.1 GB for an 800^2 frame).
#include <algorithm>

#include "pnr_common.h"

namespace pnr {

constexpr int kQBlock = 256;
// k_knn is load-latency bound: registers capped for 8 waves per SIMD (A/B: no cap
// 2.73 ms -> 8 waves 2.33 ms query); candidate records fetched one at a time
// (A/B with the up-front lookups: 1 -> 2.12, 2 -> 2.15 ms), two for small launches
// (a few waves per CU: latency, not occupancy, bound); one full-occupancy wave
// of the chip (8 blocks per CU) walks the chunks.
constexpr int kKnnBatch = 1, kKnnBatchSmall = 2;
constexpr unsigned kKnnGrid = 2048;

struct QRays {
  const float* campos;
  const float* camrot;
  const float* raydir;
  const float* tvals;
  int64_t R;
  int D;
  int per_ray;
  const int32_t* ray_cam;   // NULL: one camera; else camera index per ray
};

// Camera of ray r: the batch's one camera or its entry of the camera tables.
__device__ __forceinline__ int64_t cam_of(const QRays& q, int64_t r) { return q.ray_cam ? (int64_t)q.ray_cam[r] : 0; }
__device__ __forceinline__ void load_cam(const QRays& q, int64_t cam, float c[3], float R[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) c[i] = q.campos[cam * 3 + i];
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = q.camrot[cam * 9 + i];
}

__device__ __forceinline__ float tval(const QRays& q, int64_t r, int d) {
  return q.tvals[(q.per_ray ? r * q.D : 0) + d];
}

__device__ __forceinline__ void ray_point(const float c[3], const float dir[3], float t, float p[3]) {
  p[0] = ray_at(c[0], dir[0], t);
  p[1] = ray_at(c[1], dir[1], t);
  p[2] = ray_at(c[2], dir[2], t);
}

// mask_raypos + SR pick (qpiw.py:406-413, 664-665): the first SR candidates
// whose cell is set in the dilated occupancy.  G lanes per ray test G
// consecutive candidates at a time and a ballot orders the group's hits, so a
// ray's first SR hits get the slots of a serial walk along the ray (same
// positions, same bits) in ~D/G dependent steps instead of D; 16 lanes for
// small ray batches (a training batch: far fewer rays than the chip holds).
constexpr int64_t kMarchCoopRays = 32768;
// Whole frames too: 8 lanes per ray, one workgroup per 32 rays, no grid cap
// (A/B over 4 bench cameras, two rounds, bit-identical pidx: one lane per ray
// with the 2048-block cap 2.218 / 2.210 / 2.047 / 2.167 ms query, uncapped
// 2.238 / 2.242 / 2.055 / 2.176, 4 lanes 2.186 / 2.194 / 2.056 / 2.149, 8 lanes
// 2.175 / 2.187 / 2.054 / 2.140, 16 lanes 2.191 / 2.204 / 2.075 / 2.150): the
// per-ray tvals rows are read 32 B at a time instead of one lane per 1.6 KB row.
constexpr int kMarchLanes = 8, kMarchUnroll = 4;
constexpr unsigned kMarchGridCap = 1u << 20;
// U candidates per lane and step: the U bitmap loads of a lane are in flight
// together, and the U ballots are taken in candidate order afterwards.
template <int G, int U>
__global__ void __launch_bounds__(kQBlock) k_march_coop(QRays q, const QGrid* __restrict__ gq, int SR,
                                                        const uint32_t* __restrict__ occ_bits,
                                                        int32_t* __restrict__ n_filled,
                                                        uint16_t* __restrict__ slot_d) {
  const QGrid g = *gq;
  const float inv[3] = {__fdiv_rn(1.0f, g.vs[0]), __fdiv_rn(1.0f, g.vs[1]), __fdiv_rn(1.0f, g.vs[2])};
  const int lane = threadIdx.x & 63, gl = lane & (G - 1);
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G; r < q.R;
       r += ((int64_t)gridDim.x * blockDim.x) / G) {
    const int64_t cam = cam_of(q, r);
    const float c[3] = {q.campos[cam * 3], q.campos[cam * 3 + 1], q.campos[cam * 3 + 2]};
    const float dir[3] = {q.raydir[r * 3], q.raydir[r * 3 + 1], q.raydir[r * 3 + 2]};
    int n = 0;   // hits so far: the same in every lane of the group
    // Shared (ascending) tvals: candidates outside the grid box padded by one voxel
    // cannot land in a cell (their coordinates fail the bounds test below), so the
    // walk covers only [d_lo, d_hi): the slab-test t range of the padded box,
    // widened for rounding, mapped to indices conservatively (every skipped
    // candidate lies outside it).  The same hits in the same slots; rays that miss
    // the box (most background rays of an object scene) test no candidate.
    int d_lo = 0, d_hi = q.D;
    if (!q.per_ray && q.D > 1) {
      float tlo = -INFINITY, thi = INFINITY;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float lo = g.shift[a] - g.vs[a], hi = g.shift[a] + (float)(g.dims[a] + 1) * g.vs[a];
        if (fabsf(dir[a]) < 1e-30f) {
          if (!(c[a] >= lo && c[a] <= hi)) tlo = INFINITY;
        } else {
          const float t0 = (lo - c[a]) / dir[a], t1 = (hi - c[a]) / dir[a];
          tlo = fmaxf(tlo, fminf(t0, t1));
          thi = fminf(thi, fmaxf(t0, t1));
        }
      }
      tlo -= 1e-3f * fabsf(tlo) + 1e-3f * g.vs[0];
      thi += 1e-3f * fabsf(thi) + 1e-3f * g.vs[0];
      if (!(tlo <= thi)) {
        d_hi = 0;   // no candidate can be inside (also: a NaN bound -- then no skip below)
        if (tlo != tlo || thi != thi) d_hi = q.D;
      } else {
        const float ta = tval(q, r, 0), tb = tval(q, r, q.D - 1);
        if (tb > ta) {   // index guesses from the end points, then moved until provably outside
          int a0 = (int)fminf(fmaxf(floorf((tlo - ta) / (tb - ta) * (float)(q.D - 1)), 0.f), (float)q.D);
          while (a0 > 0 && !(tval(q, r, a0 - 1) < tlo)) --a0;   // every d < a0: t(d) < tlo
          int b0 = (int)fminf(fmaxf(ceilf((thi - ta) / (tb - ta) * (float)(q.D - 1)) + 1.f, 0.f), (float)q.D);
          while (b0 < q.D && !(tval(q, r, b0) > thi)) ++b0;     // every d >= b0: t(d) > thi
          d_lo = a0;
          d_hi = b0 > a0 ? b0 : a0;
        }
      }
    }
    for (int d0 = d_lo; d0 < d_hi && n < SR; d0 += G * U) {
      bool hit[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int d = d0 + u * G + gl;
        hit[u] = false;
        if (d < d_hi) {
          float p[3];
          ray_point(c, dir, tval(q, r, d), p);
          const int x = vox_coord_fast(p[0], g.shift[0], g.vs[0], inv[0]);
          const int y = vox_coord_fast(p[1], g.shift[1], g.vs[1], inv[1]);
          const int z = vox_coord_fast(p[2], g.shift[2], g.vs[2], inv[2]);
          if (!(x < 0 || x >= g.dims[0] || y < 0 || y >= g.dims[1] || z < 0 || z >= g.dims[2])) {
            const int64_t id = ((int64_t)x * g.dims[1] + y) * g.dims[2] + z;
            hit[u] = (occ_bits[id >> 5] >> (id & 31)) & 1u;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const unsigned m =
            (unsigned)(__ballot(hit[u]) >> (lane & (64 - G))) & (G == 32 ? 0xffffffffu : (1u << G) - 1u);
        if (hit[u]) {
          const int pos = n + __popc(m & ((1u << gl) - 1u));
          if (pos < SR) slot_d[r * SR + pos] = (uint16_t)(d0 + u * G + gl);
        }
        n += __popc(m);
      }
    }
    if (gl == 0) n_filled[r] = n < SR ? n : SR;
  }
}

// fill_rs (the filled slots as r * SR + s, ray after ray): a wave takes 64 rays,
// whose slots are one contiguous output range [off(r0), off(r0) + their counts);
// lane j writes positions off(r0) + j, + 64, ... (coalesced), finding its ray by
// a binary search over the 64 offsets (the last ray whose offset <= position:
// rays without slots share the next ray's offset and come before it).  One
// thread per ray writing its own slots touched 64 lines per store (headline:
// 70 us for 24 MB).
__global__ void __launch_bounds__(kQBlock) k_fill_list(int64_t R, int SR, const int32_t* __restrict__ n_filled,
                                                       const int32_t* __restrict__ ray_off,
                                                       int32_t* __restrict__ fill_rs, int32_t* counts) {
  const int lane = threadIdx.x & 63;
  int hit = 0;
  const int64_t nwav = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t r0 = ((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6) * 64; r0 < R; r0 += nwav * 64) {
    const int64_t r = r0 + lane;
    const int n = r < R ? n_filled[r] : 0;
    const int off = r < R ? ray_off[r] : 0;
    hit += n > 0;
    const int last = (int)(R - 1 - r0 < 63 ? R - 1 - r0 : 63);   // the wave's last ray
    const int base = __shfl(off, 0), end = __shfl(off + n, last);
    const int iters = (end - base + 63) >> 6;   // wave-uniform: every lane takes part in the shuffles
    for (int it = 0; it < iters; ++it) {
      const int p = base + 64 * it + lane;
      int lo = 0;
#pragma unroll
      for (int step = 32; step > 0; step >>= 1) {
        const int c = lo + step;
        const int oc = __shfl(off, c <= last ? c : last);
        if (c <= last && oc <= p) lo = c;
      }
      const int olo = __shfl(off, lo);
      if (p < end) fill_rs[p] = (int)((r0 + lo) * SR + (p - olo));
    }
  }
  // R_hit: one atomic per block (per wave, 10 k same-address atomics serialised at
  // the L2 took ~70 us of this kernel at the headline)
  __shared__ int red[kQBlock / 64];
  hit = wave_sum_i32(hit);
  if (lane == 0) red[threadIdx.x >> 6] = hit;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int w = 0; w < kQBlock / 64; ++w) t += red[w];
    if (t) atomicAdd(counts + 2, t);
  }
}

// The K neighbour ids and distances of a lane's sample, in LDS: one column of
// the block's [KMAX][kQBlock] arrays, so a dynamic index is one ds_write instead
// of a select chain over KMAX registers, and 2 KMAX VGPRs stay free in a kernel
// that spilled at 8 waves per SIMD (KMAX 8: 18 KB of LDS per block, 8 blocks per
// CU; A/B: headline query 2.04 -> 1.84 ms, c5 10.17 -> 8.94 ms).
template <int KMAX>
struct KnnIds {
  int32_t* p;   // this thread's id column
  float* q;     // this thread's distance column
  __device__ __forceinline__ void set(int i, int32_t v) { p[i * kQBlock] = v; }
  __device__ __forceinline__ int32_t get(int i) const { return p[i * kQBlock]; }
  __device__ __forceinline__ void setd(int i, float v) { q[i * kQBlock] = v; }
  __device__ __forceinline__ float getd(int i) const { return q[i * kQBlock]; }
};

// One accepted-or-rejected candidate record of query_neigh_along_ray_layered
// (qpiw.py:494-518): radius test, fill phase, then strict-closer replacement of
// the first farthest entry.
template <int KMAX>
__device__ __forceinline__ void knn_visit(const float4 v, const float p[3], int K, float r2,
                                          KnnIds<KMAX>& out, int& kid, int& far_ind, float& far2) {
  const float xv = __fsub_rn(v.x, p[0]);
  const float yv = __fsub_rn(v.y, p[1]);
  const float zv = __fsub_rn(v.z, p[2]);
  const float d2 = __fadd_rn(__fadd_rn(__fmul_rn(xv, xv), __fmul_rn(yv, yv)), __fmul_rn(zv, zv));
  if (!(r2 == 0.f || d2 <= r2)) return;
  const int pid = __float_as_int(v.w);
  if (kid < K) {
    // fill phase (qpiw.py:500-506)
    out.set(kid, pid);
    out.setd(kid, d2);
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
      out.set(far_ind, pid);
      out.setd(far_ind, d2);
      far2 = d2;
      float bv[KMAX];
#pragma unroll
      for (int i = 0; i < KMAX; ++i) bv[i] = out.getd(i);   // all reads issued, then the scan
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        if (i < K && bv[i] > far2) {
          far2 = bv[i];
          far_ind = i;
        }
      }
    }
  }
}

// All records of one record range, in order, KB loads in flight.
template <int KMAX, int KB>
__device__ __forceinline__ void knn_cell(const float4* __restrict__ rec, int cnt, const float p[3], int K, float r2,
                                         KnnIds<KMAX>& out, int& kid, int& far_ind, float& far2) {
  for (int g0 = 0; g0 < cnt; g0 += KB) {
    float4 vb[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) vb[u] = g0 + u < cnt ? rec[g0 + u] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      if (g0 + u >= cnt) break;
      knn_visit<KMAX>(vb[u], p, K, r2, out, kid, far_ind, far2);
    }
  }
}

// The query index of one cell (grid.hip "query index"): held = the voxel keeps
// >= 1 point; then its records are recs[off .. off + cnt).  Cells outside the
// grid are not held (the reference's loop bounds skip them).
struct QIndex {
  const uint2* words;      // {held bits, rank of the word's first cell}
  const int32_t* rec_off;  // [ranks + 1]
  const float4* recs;
  const uint32_t* coarse;  // column filter: [ceil(dz/8)][dx][ceil(dy/32)] (grid.hip k_coarse_held)
};

// Columns (x, y) within 2 of the sample's that hold a kept point somewhere in the
// z-blocks of 8 cells covering [fz - 2, fz + 2]: bit 5 (dx + 2) + (dy + 2).  A
// column outside it has no held cell in any of the walk's first three layers
// (its z-runs lie inside that range), so its fine lookups are skipped; ~7
// coarse loads per sample stand for the ~35 bitmap-word loads of layers 1 and 2
// (c5: 94 % of samples walk layer 2, ~10 % of its column lookups hold a point).
__device__ __forceinline__ uint32_t coarse_mask(const QIndex& qi, const QGrid& g, int fx, int fy, int fz) {
  const int nyw = (g.dims[1] + 31) >> 5;
  const int zlo = max(fz - 2, 0), zhi = min(fz + 2, g.dims[2] - 1);
  const int ylo = max(fy - 2, 0), yhi = min(fy + 2, g.dims[1] - 1);
  const int b0 = zlo >> 3, b1 = zhi >> 3, w0 = ylo >> 5, w1 = yhi >> 5;
  const int s = fy - 2 - 32 * w0;   // window bit of y = fy - 2 (may be < 0)
  uint32_t m = 0u;
#pragma unroll
  for (int dx = -2; dx <= 2; ++dx) {
    const int x = fx + dx;
    if ((unsigned)x >= (unsigned)g.dims[0]) continue;
    uint32_t a = 0u, b = 0u;
    for (int bz = b0; bz <= b1; ++bz) {
      const uint32_t* row = qi.coarse + ((int64_t)bz * g.dims[0] + x) * nyw;
      a |= row[w0];
      if (w1 != w0) b |= row[w1];
    }
    const uint64_t win = ((uint64_t)b << 32) | a;
    const uint32_t m5 = (uint32_t)((s >= 0 ? win >> s : win << -s) & 31u);
    m |= m5 << (5 * (dx + 2));
  }
  return m;
}

__device__ __forceinline__ int held_rank(const uint2 wd, int bit) {
  return ((wd.x >> bit) & 1u) ? (int)wd.y + __popc(wd.x & ((1u << bit) - 1u)) : -1;
}

// query_neigh_along_ray_layered (qpiw.py:442-528) for one sample.  KMAX is the
// compile-time buffer size, K <= KMAX the runtime neighbour count.  Cells are
// visited in the reference's order (Chebyshev layer, then x -> y -> z); a cell
// whose voxel holds no point contributes nothing there either, so only held
// cells are looked up (bitmap + rank: no per-cell table of the whole grid).
template <int KMAX, int LAYERS, int KB>
__device__ __forceinline__ int knn_one(const float p[3], const QGrid& g, int K, int layers, float r2,
                                       const QIndex& qi, KnnIds<KMAX>& out, int& n_cand) {
  const int fx = vox_coord(p[0], g.shift[0], g.vs[0]);
  const int fy = vox_coord(p[1], g.shift[1], g.vs[1]);
  const int fz = vox_coord(p[2], g.shift[2], g.vs[2]);
#pragma unroll
  for (int i = 0; i < KMAX; ++i) out.set(i, -1);   // (distances: read only once all K are filled)
  int kid = 0, far_ind = 0;
  float far2 = 0.f;
  if (LAYERS == 2) {
    // query 3x3x3 (every shipped config but truck).  The 9 (x, y) columns of
    // the neighbourhood are runs of 3 consecutive cells (z fastest), and held
    // voxels are ranked in cell order with their records stored in rank order
    // (grid.hip "query index"), so the records of a column's run are ONE
    // contiguous range, already in the reference's visit order (z ascending):
    //   pos(c) = held cells before cell c = word rank + popcount below c's bit,
    //   column records = [rec_off[pos(z_lo)], rec_off[pos(z_hi) + held(z_hi)]).
    // Traversal (qpiw.py:481-527): layer 0 = the centre cell, then layer 1 =
    // columns x -> y, each run z -> (the centre skipped in its column).
    if ((unsigned)fz >= (unsigned)g.dims[2]) return 0;   // never: filled samples lie in held-dilated cells
    const int zlo = fz > 0 ? fz - 1 : fz, zhi = fz + 1 < g.dims[2] ? fz + 1 : fz;
    auto range = [&](int o, int e) {
      n_cand += e - o;
      knn_cell<KMAX, KB>(qi.recs + o, e - o, p, K, r2, out, kid, far_ind, far2);
    };
    // Every index lookup of the 27 cells is issued up front: one round of 9-18
    // independent word loads (a column's 3-cell run spans <= 2 words; the
    // centre cell is in column 4's), one round of rec_off loads, then the 11
    // record ranges (centre, columns 0-3, column 4 below / above the centre,
    // columns 5-8) walked by ONE visit loop in the reference's order (A/B vs
    // 9 x 2 dependent lookup rounds: DESIGN.md 13).  32-bit cell indices (this
    // kernel is launched only for grids of < 2^32 cells) keep addresses 1 VGPR.
    int lo[9], hi[9];
    int pc = 0, hc = 0;
#pragma unroll
    for (int col = 0; col < 9; ++col) {
      const int cx = fx + col / 3 - 1, cy = fy + col % 3 - 1;
      const bool in = (unsigned)cx < (unsigned)g.dims[0] && (unsigned)cy < (unsigned)g.dims[1];
      const uint32_t base = ((uint32_t)cx * (uint32_t)g.dims[1] + (uint32_t)cy) * (uint32_t)g.dims[2];
      const uint32_t clo = base + zlo, chi = base + zhi;
      const uint2 a = in ? qi.words[clo >> 5] : make_uint2(0u, 0u);
      const uint2 b = in && (chi >> 5) != (clo >> 5) ? qi.words[chi >> 5] : a;
      lo[col] = (int)a.y + __popc(a.x & ((1u << (clo & 31)) - 1u));
      hi[col] = (int)b.y + __popc(b.x & ((1u << (chi & 31)) - 1u)) + (int)((b.x >> (chi & 31)) & 1u);
      if (col == 4) {
        const uint32_t cc = base + fz;
        const uint2 w = (cc >> 5) == (clo >> 5) ? a : b;
        hc = (w.x >> (cc & 31)) & 1u;
        pc = (int)w.y + __popc(w.x & ((1u << (cc & 31)) - 1u));
      }
    }
#pragma unroll
    for (int col = 0; col < 9; ++col) {
      if (hi[col] == lo[col]) continue;   // no held cell in the run
      lo[col] = qi.rec_off[lo[col]];
      hi[col] = qi.rec_off[hi[col]];
    }
    // centre records [pco, pce); empty when the centre voxel holds no point
    const int pco = lo[4] == hi[4] ? lo[4] : qi.rec_off[pc];
    const int pce = hc ? qi.rec_off[pc + 1] : pco;
    auto sel = [&](int rg, int& o, int& e) {
      o = pco;
      e = pce;
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int r = j < 5 ? j + 1 : j + 2;   // range slot of column j (column 4: slots 5, 6)
        if (rg == r) {
          o = lo[j];
          e = j == 4 ? pco : hi[j];
        }
      }
      if (rg == 6) {
        o = pce;
        e = hi[4];
      }
    };
#pragma unroll 1
    for (int rg = 0; rg < 11; ++rg) {
      if (rg == 1 && kid >= K) break;   // layer 0 already saw >= K candidates (qpiw.py:526)
      int o, e;
      sel(rg, o, e);
      if (o == e) continue;
      range(o, e);
    }
    return kid < K ? kid : K;
  }
  // Any layer count (truck: 3 layers, 125 cells).  Layer L visits x -> y -> z
  // (qpiw.py:481-527) the cells of Chebyshev radius L: in a ring column
  // (max(|x|, |y|) = L) the whole z-run [fz - L, fz + L], in an inner column its
  // two end cells.  A run of consecutive cells is one record range in rank order
  // (grid.hip "query index"), so a ring column costs one or two word loads and,
  // only when it holds a point, one rec_off pair -- not a word load per cell.
  // the column filter covers the first three layers (every shipped flag set)
  const uint32_t cm = qi.coarse && layers <= 3 ? coarse_mask(qi, g, fx, fy, fz) : ~0u;
  for (int layer = 0; layer < layers; ++layer) {
    const int L = layer;
    const int x0 = max(-fx, -L), x1 = min(g.dims[0] - fx, L + 1);
    const int y0 = max(-fy, -L), y1 = min(g.dims[1] - fy, L + 1);
    const int zr0 = max(fz - L, 0), zr1 = min(fz + L, g.dims[2] - 1);   // a ring column's run
    for (int x = x0; x < x1; ++x) {
      for (int y = y0; y < y1; ++y) {
        if (L <= 2 && !((cm >> (5 * (x + 2) + (y + 2))) & 1u)) continue;   // no held cell near this column
        const int64_t base = ((int64_t)(fx + x) * g.dims[1] + (fy + y)) * g.dims[2];
        if (x == -L || x == L || y == -L || y == L) {
          const int64_t ca = base + zr0, cb = base + zr1;
          const uint2 wa = qi.words[ca >> 5];
          const uint2 wb = (cb >> 5) == (ca >> 5) ? wa : qi.words[cb >> 5];
          const int lo = (int)wa.y + __popc(wa.x & ((1u << (ca & 31)) - 1u));
          const int hi = (int)wb.y + __popc(wb.x & ((1u << (cb & 31)) - 1u)) + (int)((wb.x >> (cb & 31)) & 1u);
          if (hi == lo) continue;   // no held cell in the run
          const int o = qi.rec_off[lo];
          const int cn = qi.rec_off[hi] - o;
          n_cand += cn;
          knn_cell<KMAX, KB>(qi.recs + o, cn, p, K, r2, out, kid, far_ind, far2);
        } else {
          // the two end cells z = fz - L, fz + L (inside the grid only): one word load
          // when they share a word (c5: 94 % of samples walk layer 2, whose nine inner
          // columns were 18 of its ~45 word loads)
          const bool in0 = fz - L >= 0, in1 = fz + L < g.dims[2];
          const int64_t c0 = base + fz - L, c1 = base + fz + L;
          const uint2 w0 = in0 ? qi.words[c0 >> 5] : make_uint2(0u, 0u);
          const uint2 w1 = in1 ? (in0 && (c1 >> 5) == (c0 >> 5) ? w0 : qi.words[c1 >> 5]) : make_uint2(0u, 0u);
          const int re[2] = {in0 ? held_rank(w0, (int)(c0 & 31)) : -1, in1 ? held_rank(w1, (int)(c1 & 31)) : -1};
#pragma unroll
          for (int e = 0; e < 2; ++e) {   // z = fz - L, then fz + L
            const int r = re[e];
            if (r < 0) continue;
            const int o = qi.rec_off[r];
            const int cn = qi.rec_off[r + 1] - o;
            n_cand += cn;
            knn_cell<KMAX, KB>(qi.recs + o, cn, p, K, r2, out, kid, far_ind, far2);
          }
        }
      }
    }
    if (kid >= K) break;
  }
  return kid < K ? kid : K;
}

// LAYERS = 2: the 3x3x3 query specialised (its own kernel: the generic
// layered loop inlined beside it costs registers); 0: any layer count.
// Waves per SIMD: 7 for the 3x3x3 walk (72 VGPRs, 21 spilled, against 64 and 29
// at 8: headline query -0.7 %), 8 for the generic one (c5: 7 waves +6 %), fewer
// for KMAX > 8 (the [KMAX][256] LDS columns bound the blocks per CU);
// profiles/r05_knn_occupancy_lds_ab.json.
template <int KMAX, int LAYERS, int KB>
__global__ void __launch_bounds__(kQBlock) __attribute__((amdgpu_waves_per_eu(KMAX <= 8 ? (LAYERS == 2 ? 7 : 8) : 64 / KMAX))) k_knn(QRays q, const QGrid* __restrict__ gq, int SR, int K, int layers, float r2,
                                                 QIndex qi, const uint16_t* __restrict__ slot_d,
                                                 const int32_t* __restrict__ fill_rs,
                                                 int32_t* __restrict__ pidx, int32_t* __restrict__ vflag,
                                                 int32_t* __restrict__ ray_vcnt,
                                                 float* __restrict__ sample_w,
                                                 float* __restrict__ sample_p, int32_t* counts, int vec_pidx,
                                                 int32_t* __restrict__ xcd_ctr) {
  const QGrid g = *gq;
  const int64_t S = counts[0];
  float c[3], Rm[9];
  load_cam(q, 0, c, Rm);
  int pairs = 0, n_cand = 0;
  // A block takes 256 consecutive filled samples (~a dozen neighbouring rays of
  // one pixel row) and hands them to its lanes ordered by shading slot: lanes
  // of a wave then hold the same slot of adjacent rays, whose neighbourhoods
  // overlap, so their record loads share cache lines (the sample -> outputs
  // mapping is unchanged; only which lane computes which sample).
  __shared__ int hist[kQBlock], perm[kQBlock];
  __shared__ int32_t ids_lds[KMAX * kQBlock];
  __shared__ float dist_lds[KMAX * kQBlock];
  const bool by_slot = SR <= kQBlock;   // (A/B: lanes in fill order 3.45 ms query, by slot 2.94)
  const int tid = threadIdx.x, lane = tid & 63;
  // XCD-aware chunking (grid a multiple of 8; blocks b, b + 8, ... share an
  // XCD): XCD x walks the contiguous chunk range [C x / 8, C (x + 1) / 8) of the
  // sample list, so at any moment its L2 holds the records of a few image rows
  // instead of every XCD touching the same wide window (A/B in DESIGN.md 13).
  // Chunks are handed out in order by a per-XCD counter, and an XCD
  // whose range is exhausted takes chunks from the next XCDs' ranges (the
  // bands' per-sample costs differ, so static ranges finish unevenly).  Small
  // launches (a training batch's few hundred chunks) walk the plain grid
  // stride: there the counters' contention costs more than the locality gains.
  const int64_t C = (S + kQBlock - 1) / kQBlock;
  const bool whole = (gridDim.x & 7) == 0;
  const bool dyn = whole && C >= 4 * (int64_t)gridDim.x;
  const bool xcd = dyn;
  const int xg = xcd ? (int)(blockIdx.x & 7) : 0;
  const int64_t c_lo = xcd ? C * xg / 8 : 0, c_hi = xcd ? C * (xg + 1) / 8 : C;
  const int64_t c_step = xcd ? gridDim.x / 8 : gridDim.x;
  __shared__ int64_t s_ch;
  unsigned done = 0;   // (thread 0) XCD ranges this block found exhausted: never polled again
  auto next_chunk = [&](int64_t prev) -> int64_t {
    if (!dyn) return prev < 0 ? c_lo + (xcd ? blockIdx.x >> 3 : blockIdx.x) : prev + c_step;
    __syncthreads();   // every thread has read s_ch of the previous chunk
    if (tid == 0) {
      int64_t got = C;
      for (int k = 0; k < 8 && got == C; ++k) {
        const int y = (xg + k) & 7;
        if ((done >> y) & 1u) continue;
        const int64_t t = C * y / 8 + atomicAdd(xcd_ctr + y, 1);
        if (t < C * (y + 1) / 8) got = t;
        else done |= 1u << y;
      }
      s_ch = got;
    }
    __syncthreads();
    return s_ch;
  };
  const int64_t c_end = dyn ? C : c_hi;
  for (int64_t ch = next_chunk(-1); ch < c_end; ch = next_chunk(ch)) {
    const int64_t base = ch * kQBlock;
    int64_t i = base + tid;
    if (by_slot) {
      const int n_in = (int)min((int64_t)kQBlock, S - base);
      hist[tid] = 0;
      __syncthreads();
      const int s0 = tid < n_in ? fill_rs[base + tid] % SR : 0;
      const int at = tid < n_in ? atomicAdd(&hist[s0], 1) : 0;
      __syncthreads();
      if (tid < 64) {   // exclusive scan of hist[0 .. 256) by wave 0, 4 entries per lane
        const int a0 = hist[4 * lane], a1 = hist[4 * lane + 1], a2 = hist[4 * lane + 2], a3 = hist[4 * lane + 3];
        int t = a0 + a1 + a2 + a3, incl = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_up(incl, o);
          if (lane >= o) incl += v;
        }
        const int ex = incl - t;
        hist[4 * lane] = ex;
        hist[4 * lane + 1] = ex + a0;
        hist[4 * lane + 2] = ex + a0 + a1;
        hist[4 * lane + 3] = ex + a0 + a1 + a2;
      }
      __syncthreads();
      if (tid < n_in) perm[hist[s0] + at] = tid;
      __syncthreads();
      i = tid < n_in ? base + perm[tid] : S;
    }
    if (i >= S) continue;
    const int rs = fill_rs[i];
    const int64_t r = rs / SR;
    const int d = slot_d[rs];
    const float dir[3] = {q.raydir[r * 3], q.raydir[r * 3 + 1], q.raydir[r * 3 + 2]};
    // the sample's camera: the launch's (uniform, loaded once) or its ray's entry
    // of a multi-camera batch -- read per sample into temporaries, so no camera
    // is carried in VGPRs across the walk
    float cs[3], Rs[9];
    if (q.ray_cam) {
      load_cam(q, q.ray_cam[r], cs, Rs);
    } else {
#pragma unroll
      for (int a = 0; a < 3; ++a) cs[a] = c[a];
#pragma unroll
      for (int a = 0; a < 9; ++a) Rs[a] = Rm[a];
    }
    float p[3], pp[3];
    ray_point(cs, dir, tval(q, r, d), p);
    world_to_pers(p, cs, Rs, pp);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      sample_w[i * 3 + a] = p[a];
      sample_p[i * 3 + a] = pp[a];
    }
    KnnIds<KMAX> out{ids_lds + tid, dist_lds + tid};
    const int nk = knn_one<KMAX, LAYERS, KB>(p, g, K, layers, r2, qi, out, n_cand);
    if (KMAX == 8 && K == 8 && vec_pidx) {   // two 16-B stores (pidx 16-B aligned)
      int4* o4 = reinterpret_cast<int4*>(pidx + i * 8);
      o4[0] = make_int4(out.get(0), out.get(1), out.get(2), out.get(3));
      o4[1] = make_int4(out.get(4 % KMAX), out.get(5 % KMAX), out.get(6 % KMAX), out.get(7 % KMAX));
    } else {
      for (int k = 0; k < K; ++k) pidx[i * K + k] = out.get(k);
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
  const float zero[3] = {0.f, 0.f, 0.f};
  const int64_t total = q.R * SR;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / SR;
    const int s = (int)(e - r * SR);
    float c[3], Rm[9], origin_p[3];
    load_cam(q, cam_of(q, r), c, Rm);
    world_to_pers(zero, c, Rm, origin_p);
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
  q.ray_cam = r->ray_cam;
  return q;
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_query_scratch_bytes(int64_t R, int32_t SR, size_t* out) {
  PNR_CHECK_ARG(out && R >= 0 && SR > 0, "query_scratch_bytes: bad args");
  *out = std::max<size_t>(scan_scratch_bytes(R * SR + 1), 64);   // >= k_knn's 8 chunk counters
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
  PNR_CHECK_ARG(b->scratch_bytes >= std::max<size_t>(scan_scratch_bytes(RS + 1), 64), "query: scratch too small");
  hipStream_t st = as_stream(stream);
  QRays q = to_qrays(rays);
  // the grid's exact geometry lives on the device (h->geom); h->gp.dims bounds it
  const QGrid* g_dev = h->geom.as<QGrid>();
  const int* gdims = h->gp.dims;
  PNR_HIP(hipMemsetAsync(b->counts, 0, 8 * sizeof(int32_t), st));
  PNR_HIP(hipMemsetAsync(b->ray_vcnt, 0, (size_t)(R > 0 ? R : 1) * sizeof(int32_t), st));
  if (R == 0) {
    PNR_HIP(hipMemsetAsync(b->ray_off, 0, sizeof(int32_t), st));
    PNR_HIP(hipMemsetAsync(b->ray_row, 0, sizeof(int32_t), st));
    PNR_HIP(hipMemsetAsync(b->valid_off, 0, sizeof(int32_t), st));
    return PNR_OK;
  }
  if (R <= kMarchCoopRays)   // few rays: 16 lanes per ray (latency)
    hipLaunchKernelGGL((k_march_coop<16, 2>), dim3(grid_for(R * 16, kQBlock)), dim3(kQBlock), 0, st, q, g_dev, qp->SR,
                       h->occ_bits.as<uint32_t>(), b->n_filled, b->slot_d);
  else
    hipLaunchKernelGGL((k_march_coop<kMarchLanes, kMarchUnroll>), dim3(grid_for(R * kMarchLanes, kQBlock, kMarchGridCap)),
                       dim3(kQBlock), 0, st, q, g_dev, qp->SR, h->occ_bits.as<uint32_t>(), b->n_filled, b->slot_d);
  PNR_LAUNCH_CHECK();
  if ((rc = exclusive_scan(b->n_filled, R, nullptr, b->ray_off, R + 1, b->counts + 0, b->scratch,
                           b->scratch_bytes, st)))
    return rc;
  hipLaunchKernelGGL(k_fill_list, dim3(grid_for(R, kQBlock)), dim3(kQBlock), 0, st, R, qp->SR,
                     b->n_filled, b->ray_off, b->fill_rs, b->counts);
  PNR_LAUNCH_CHECK();
  const int layers = (qp->kernel_size[0] + 1) / 2;
  // launches of < 4 M sample slots (training batches): fewer waves than the
  // chip holds, so more records in flight per lane
  const bool small = RS < (int64_t(4) << 20);
  // the 3x3x3 kernel indexes cells in 32 bits
  const bool q3 = layers == 2 && (int64_t)gdims[0] * gdims[1] * gdims[2] < (int64_t(1) << 32);
  unsigned gk = grid_for(RS, kQBlock, kKnnGrid);
  if (gk >= 8) gk &= ~7u;   // whole XCD groups (k_knn's chunk walk)
  // k_knn's per-XCD chunk counters: the head of the scan scratch, free between
  // the fill-list and valid-list scans (stream order)
  PNR_HIP(hipMemsetAsync(b->scratch, 0, 8 * sizeof(int32_t), st));
  const int vec = ((uintptr_t)b->pidx & 15) == 0;
  QIndex qi;
  qi.words = h->q_words.as<uint2>();
  qi.coarse = reinterpret_cast<const uint32_t*>(h->cell_bytes.as<uint8_t>() + h->coarse_off);
  qi.rec_off = h->q_rec_off.as<int32_t>();
  qi.recs = h->q_recs.as<float4>();
#define PNR_KNN(KM)                                                                              \
  hipLaunchKernelGGL((q3 ? (small ? k_knn<KM, 2, kKnnBatchSmall> : k_knn<KM, 2, kKnnBatch>)           \
                          : k_knn<KM, 0, kKnnBatchSmall>), dim3(gk), dim3(kQBlock), 0, st, q, g_dev, qp->SR, qp->K, layers,      \
                     qp->radius_limit2, qi, b->slot_d, b->fill_rs, b->pidx, b->vflag,             \
                     b->ray_vcnt, b->sample_w, b->sample_p, b->counts, vec,                       \
                     reinterpret_cast<int32_t*>(b->scratch))
  if (qp->K <= 8) PNR_KNN(8);
  else if (qp->K <= 16) PNR_KNN(16);
  else PNR_KNN(32);
#undef PNR_KNN
  PNR_LAUNCH_CHECK();
  // valid_off and, in the same pass, valid_list[valid_off[i]] = i for vflag[i] (the
  // separate compaction re-read both arrays: c5 117 us)
  if ((rc = exclusive_scan(b->vflag, RS, b->counts + 0, b->valid_off, RS + 1, b->counts + 1, b->scratch,
                           b->scratch_bytes, st, 0, nullptr, b->valid_list)))
    return rc;
  if ((rc = exclusive_scan(b->ray_vcnt, R, nullptr, b->ray_row, R + 1, b->counts + 3, b->scratch,
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
