// Persistent sparse voxel grid of the neural points.
//
// Replaces build_occ_vox (query_point_indices_worldcoords.py:546-611) and its
// three atomics-ordered kernels claim_occ / map_coor2occ / fill_occ2pnts
// (qpiw.py:243-387).  The reference rebuilds this for every 2304-ray chunk and
// its slot order depends on atomic arrival; here it is built once per point
// cloud version, deterministically, in the serial order of the reference
// kernels (slot = rank of the first point index that lands in the voxel,
// points inside a voxel in ascending index order), which is what the serial
// execution of claim_occ/fill_occ2pnts produces when nothing overflows.  The
// points are grouped by a stable LSD radix sort of their cell keys, so
// claimer, count and the ordered run of every voxel come without atomics.
//
// HBM layout (MI355X, 288 GB): one dense int32 cell->slot grid (lego 162x290x189
// = 35.5 MB), one dilated-occupancy BITMAP (1 bit per cell: 1.1 MB, stays in
// every XCD's L2 for the ray march), and a slot-major float4 table
// {x, y, z, point id} of P entries per slot so the KNN loop reads one 16-B
// record per candidate instead of an index plus a 12-B xyz gather.  Cell
// indices are int64 (a +-10 m scene101 range at 16 mm voxels is 1.95e9 cells).
//
// Overflow (more occupied voxels than max_o, more points than P in a voxel):
// the reference's reservoir replacement (qpiw.py:289-298, 377-384) keeps a
// uniform random subset with a time seed; here the same uniform subsets come
// from a seeded hash (pnr_common.h res_vkey / res_pkey): the max_o voxels of
// smallest key, found by an 8-pass radix select on the device (no host sync),
// and per voxel the P points of smallest key.  Without overflow the tables
// are exactly the serial order.
#include "pnr_common.h"

namespace pnr {

constexpr int kBlock = 256;

// ---------------------------------------------------------------- bbox
__device__ __forceinline__ unsigned f2ord(float f) {
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ void k_bbox_init(unsigned* acc) {
  if (threadIdx.x < 3) acc[threadIdx.x] = 0xffffffffu;
  else if (threadIdx.x < 6) acc[threadIdx.x] = 0u;
}

__global__ void __launch_bounds__(kBlock) k_bbox(const float* __restrict__ xyz, int64_t n, unsigned* acc) {
  unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
  // 4 points (3 x 16 B) per thread and step when xyz is 16-B aligned, the rest one by one
  const bool vec = (reinterpret_cast<uintptr_t>(xyz) & 15) == 0;
  const int64_t n4 = vec ? n / 4 : 0;
  const float4* x4 = reinterpret_cast<const float4*>(xyz);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 a = x4[i * 3], b = x4[i * 3 + 1], c = x4[i * 3 + 2];
    const float v[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      const unsigned o = f2ord(v[e]);
      mn[e % 3] = min(mn[e % 3], o);
      mx[e % 3] = max(mx[e % 3], o);
    }
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      unsigned o = f2ord(xyz[i * 3 + c]);
      mn[c] = min(mn[c], o);
      mx[c] = max(mx[c], o);
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn[c] = min(mn[c], (unsigned)__shfl_xor((int)mn[c], o));
      mx[c] = max(mx[c], (unsigned)__shfl_xor((int)mx[c], o));
    }
  }
  // one atomic per block and bound (the per-wave atomics on 6 shared words serialised)
  __shared__ unsigned red[kBlock / 64][6];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      red[w][c] = mn[c];
      red[w][3 + c] = mx[c];
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int c = threadIdx.x;
    unsigned v = red[0][c];
    for (int i = 1; i < kBlock / 64; ++i) v = c < 3 ? min(v, red[i][c]) : max(v, red[i][c]);
    if (c < 3) atomicMin(acc + c, v);
    else atomicMax(acc + c, v);
  }
}

__global__ void k_bbox_fin(unsigned* acc) {
  if (threadIdx.x < 6) {
    float f = ord2f(acc[threadIdx.x]);
    reinterpret_cast<float*>(acc)[threadIdx.x] = f;
  }
}

// ---------------------------------------------------------------- build
struct GridDev {
  float shift[3], vs[3];
  int dims[3], qs[3];
  int max_o, P, slot0_drop;
  uint64_t seed;
};

// the launch's by-value parameters with the geometry (shift, cell size, dims)
// read from device memory (pnr_handle.geom)
__device__ __forceinline__ GridDev with_geom(const GridDev& g0, const QGrid* __restrict__ geo) {
  GridDev g = g0;
  const QGrid G = *geo;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    g.shift[a] = G.shift[a];
    g.vs[a] = G.vs[a];
    g.dims[a] = G.dims[a];
  }
  return g;
}

// get_hyperparameters (qpiw.py:48-81) on the device from the point bbox, for a
// build with opt.ranges set (no host read of the bbox): numpy's dtypes --
// min/max clipped to ranges and padded in fp32, vdim = (max - min) / vsize in
// float64 (vsize is a Python float list), dims = ceil(vdim / vscale) -- so shift
// and dims are the host formula's bits.  dims are clamped to [1, the bound
// the host allocated for].
__device__ __forceinline__ void grid_geom_from(const float* bbox, const pnr_grid_spec& sp, QGrid* geo) {
  QGrid G;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float mn = fmaxf(bbox[a], sp.ranges[a]);
    float mx = fminf(bbox[3 + a], sp.ranges[3 + a]);
    mn = __fsub_rn(mn, sp.pad[a]);
    mx = __fadd_rn(mx, sp.pad[a]);
    const double vdim = __ddiv_rn((double)__fsub_rn(mx, mn), sp.vsize[a]);
    double sd = ceil(__ddiv_rn(vdim, (double)sp.vscale[a]));
    int d = sd >= 1.0 ? (int)sd : 1;
    d = d < sp.dims_max[a] ? d : sp.dims_max[a];
    G.shift[a] = mn;
    G.vs[a] = sp.vsize_s[a];
    G.dims[a] = d;
  }
  G.P = sp.P;
  *geo = G;
}

// The device build's bbox + geometry in TWO launches (was four: k_bbox_init,
// k_bbox, k_bbox_fin, k_grid_geom): k_bbox reduces into the order-key
// accumulators, k_geom_acc converts them to the float bbox (out6), derives the
// geometry and puts the accumulators back in their initial state for the next
// build (the state k_bbox_acc_init gives them at allocation).  (One launch with
// a last-block ticket needed a device-scope release fence per block: 111 us.)
__global__ void k_bbox_acc_init(unsigned* acc) {
  if (threadIdx.x < 3) acc[threadIdx.x] = 0xffffffffu;
  else if (threadIdx.x < 8) acc[threadIdx.x] = 0u;
}

__device__ __forceinline__ void grid_geom_from(const float* bb, const pnr_grid_spec& sp, QGrid* geo);

__global__ void k_geom_acc(unsigned* acc, float* __restrict__ out6, pnr_grid_spec sp, QGrid* __restrict__ geo) {
  if (threadIdx.x != 0) return;
  float bb[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    bb[c] = ord2f(acc[c]);
    out6[c] = bb[c];
  }
  grid_geom_from(bb, sp, geo);
  acc[0] = acc[1] = acc[2] = 0xffffffffu;
  acc[3] = acc[4] = acc[5] = 0u;
}

__global__ void k_set_geom(QGrid G, QGrid* __restrict__ geo) {
  if (threadIdx.x == 0) *geo = G;
}

__device__ __forceinline__ int64_t cell_of(const float* p, const GridDev& g, int c[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) c[a] = vox_coord(p[a], g.shift[a], g.vs[a]);
  if (c[0] < 0 || c[0] >= g.dims[0] || c[1] < 0 || c[1] >= g.dims[1] || c[2] < 0 ||
      c[2] >= g.dims[2])
    return -1;
  return ((int64_t)c[0] * g.dims[1] + c[1]) * g.dims[2] + c[2];
}

// ---- points grouped by voxel (claim_occ + fill_occ2pnts, qpiw.py:243-387),
// order-free and without atomics: a point's key is its cell index, and a
// stable LSD radix sort of (key, point id) lays the points of one voxel out as
// one run in ascending id order.  The run's first id is the voxel's claimer
// (the smallest point id: the serial claim_occ's winner), its length the
// voxel's point count, and its first P ids the serial fill_occ2pnts order.
// Points outside the grid carry the key `sentinel` (> every cell) and sort last.
// RB: radix bits per pass (the build uses 8), D = 2^RB digits
constexpr int kSelPasses = 8;
struct SelState {
  int32_t active;  // 1: more occupied voxels than max_o
  int32_t pad;
};

template <int RB, typename K>
__device__ __forceinline__ int rs_digit(K k, int shift) {
  return (int)((k >> shift) & (K)((1 << RB) - 1));
}

constexpr int kRsItems = 8;
constexpr int kRsTile = kBlock * kRsItems;  // 2048 keys: ~4 tiles per CU at 2 M points

// Block b: the keys of sort tile b (kRsTile points) and the radix sort's first
// digit histogram of that tile (k_rs_hist's pass 0, without a launch and a
// re-read of the keys), and the empty state of slots [b kRsTile, (b+1) kRsTile).
template <int RB, typename K>
__global__ void __launch_bounds__(kBlock) k_cell_keys(const float* __restrict__ xyz, int64_t n, GridDev g0,
                                                      const QGrid* __restrict__ geo, K sentinel,
                                                      K* __restrict__ keys, int64_t n_slots,
                                                      int32_t* __restrict__ pt_flag,
                                                      int32_t* __restrict__ occ_numpnts,
                                                      int32_t* __restrict__ occ_2_coor, int32_t* __restrict__ counters,
                                                      int tiles, int32_t* __restrict__ hist,
                                                      uint32_t* __restrict__ sel_hist) {
  constexpr int D = 1 << RB;
  __shared__ int32_t h[D];
  const GridDev g = with_geom(g0, geo);
  if (blockIdx.x == 0 && threadIdx.x < 8) counters[threadIdx.x] = 0;
  if (blockIdx.x == 0 && sel_hist)   // the voxel reservoir's histograms (was k_sel_init)
    for (int i = threadIdx.x; i < kSelPasses * 256; i += kBlock) sel_hist[i] = 0u;
  for (int d = threadIdx.x; d < D; d += kBlock) h[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
  if ((int)blockIdx.x < tiles) {
#pragma unroll 4
    for (int r = 0; r < kRsItems; ++r) {
      const int64_t i = base + r * kBlock + threadIdx.x;
      if (i < n) {
        float p[3] = {xyz[i * 3 + 0], xyz[i * 3 + 1], xyz[i * 3 + 2]};
        int c[3];
        const int64_t cell = cell_of(p, g, c);
        const K k = cell >= 0 ? (K)cell : sentinel;
        keys[i] = k;
        pt_flag[i] = 0;
        atomicAdd(&h[rs_digit<RB>(k, 0)], 1);
      }
    }
  }
  for (int r = 0; r < kRsItems; ++r) {   // the slot tables' empty state
    const int64_t i = base + r * kBlock + threadIdx.x;
    if (i < n_slots) {
      occ_numpnts[i] = 0;
      occ_2_coor[i * 3 + 0] = -1;
      occ_2_coor[i * 3 + 1] = -1;
      occ_2_coor[i * 3 + 2] = -1;
    }
  }
  __syncthreads();
  if ((int)blockIdx.x < tiles)
    for (int d = threadIdx.x; d < D; d += kBlock) hist[(int64_t)d * tiles + blockIdx.x] = h[d];
}

// LSD radix sort, 8 key bits per pass over tiles of kRsTile keys: per-tile
// digit counts (k_rs_hist), their exclusive scan in digit-major order (the
// device scan), then a stable scatter (k_rs_scatter) that ranks the tile in
// LDS and writes each digit's keys of the tile as one contiguous run.
template <int RB, typename K>
__global__ void __launch_bounds__(kBlock) k_rs_hist(const K* __restrict__ keys, int64_t n, int shift, int tiles,
                                                    int32_t* __restrict__ hist) {
  constexpr int D = 1 << RB;
  __shared__ int32_t h[D];
  for (int d = threadIdx.x; d < D; d += kBlock) h[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
#pragma unroll 4
  for (int r = 0; r < kRsItems; ++r) {
    const int64_t i = base + r * kBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[rs_digit<RB>(keys[i], shift)], 1);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += kBlock) hist[(int64_t)d * tiles + blockIdx.x] = h[d];
}

// vin == nullptr: the values are the keys' positions (the point ids, pass 0)
template <int RB, typename K>
__global__ void __launch_bounds__(kBlock) k_rs_scatter(const K* __restrict__ kin, const int32_t* __restrict__ vin,
                                                       int64_t n, int shift, int tiles,
                                                       const int32_t* __restrict__ offs, K* __restrict__ kout,
                                                       int32_t* __restrict__ vout) {
  constexpr int D = 1 << RB;
  constexpr int DPT = D / kBlock;             // digits per thread (1 or 2)
  __shared__ K sk[kRsTile];
  __shared__ int32_t sv[kRsTile];
  __shared__ int32_t wcnt[kBlock / 64][D];    // this round's digit counts per wave
  __shared__ int32_t run[D];                  // digit counts of the earlier rounds, then digit starts
  __shared__ int32_t gb[D];                   // output position of the tile's digit-d keys minus their LDS start
  __shared__ int32_t wsum[kBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
  const int in_tile = (int)(n - base < kRsTile ? n - base : kRsTile);
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    run[tid * DPT + i] = 0;
#pragma unroll
    for (int q = 0; q < kBlock / 64; ++q) wcnt[q][tid * DPT + i] = 0;
  }
  K key[kRsItems];
  int32_t val[kRsItems], loc[kRsItems];
#pragma unroll
  for (int r = 0; r < kRsItems; ++r) {
    const int e = r * kBlock + tid;
    const bool ok = e < in_tile;
    key[r] = ok ? kin[base + e] : (K)0;
    val[r] = ok ? (vin ? vin[base + e] : (int32_t)(base + e)) : 0;
  }
  __syncthreads();
  // stable rank inside the tile: item e = r * 256 + tid comes after every
  // item of an earlier round, of a lower wave, and of a lower lane
#pragma unroll
  for (int r = 0; r < kRsItems; ++r) {
    const bool ok = r * kBlock + tid < in_tile;
    const int d = rs_digit<RB>(key[r], shift);
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const uint64_t m = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? m : ~m;
    }
    const int rk = __popcll(peers & below);
    if (ok && rk == 0) wcnt[w][d] = __popcll(peers);
    __syncthreads();
    int pre = run[d];
    for (int q = 0; q < w; ++q) pre += wcnt[q][d];
    loc[r] = pre + rk;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int dd = tid * DPT + i;
      int add = 0;
#pragma unroll
      for (int q = 0; q < kBlock / 64; ++q) {
        add += wcnt[q][dd];
        wcnt[q][dd] = 0;
      }
      run[dd] += add;
    }
    __syncthreads();
  }
  // digit starts inside the tile (exclusive scan of the D counts; thread t owns
  // digits t DPT .. t DPT + DPT - 1)
  int my[DPT], mine = 0;
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    my[i] = run[tid * DPT + i];
    mine += my[i];
  }
  int inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  for (int q = 0; q < w; ++q) inc += wsum[q];
  int start = inc - mine;
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    const int dd = tid * DPT + i;
    gb[dd] = offs[(int64_t)dd * tiles + blockIdx.x] - start;
    run[dd] = start;
    start += my[i];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRsItems; ++r) {
    if (r * kBlock + tid < in_tile) {
      const int p = run[rs_digit<RB>(key[r], shift)] + loc[r];
      sk[p] = key[r];
      sv[p] = val[r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRsItems; ++r) {
    const int e = r * kBlock + tid;
    if (e < in_tile) {
      const K k = sk[e];
      const int64_t pos = (int64_t)gb[rs_digit<RB>(k, shift)] + e;
      kout[pos] = k;
      vout[pos] = sv[e];
    }
  }
}

// Runs of the sorted keys: the claimer of each occupied voxel flagged by point
// id (its rank is the slot), the run's first and one-past-last sorted
// positions by cell; counters[1] = points inside the grid.
template <typename K>
__global__ void __launch_bounds__(kBlock) k_runs(const K* __restrict__ skey, const int32_t* __restrict__ sid,
                                                 int64_t n, K sentinel, int32_t* __restrict__ pt_flag,
                                                 int32_t* __restrict__ cell_start, int32_t* __restrict__ cell_end,
                                                 int32_t* __restrict__ counters) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const K k = skey[j];
    if (k == sentinel) continue;
    if (j == 0 || skey[j - 1] != k) {
      pt_flag[sid[j]] = 1;
      cell_start[(int64_t)k] = (int)j;
    }
    const K nx = j + 1 < n ? skey[j + 1] : sentinel;
    if (nx != k) {
      cell_end[(int64_t)k] = (int)(j + 1);
      if (nx == sentinel) counters[1] = (int)(j + 1);
    }
  }
}

// ---- voxel reservoir (claim_occ overflow, qpiw.py:283-298): radix select of
// the key of rank max_o - 1 among the occupied voxels' keys, 8 bits per pass,
// most significant first.  Pass q counts into its own 256-bin histogram; every
// later kernel re-derives the digits fixed so far from those histograms, so
// no launch is spent on the pick.  Nothing runs when the voxels fit max_o.


// Block of 256: s[0] = the key bits fixed by passes 0..npass-1, s[1] = the
// rank still to find below them (the digit of pass q: the first whose running
// count exceeds the rank, else 255).
__device__ void sel_derive(const uint32_t* __restrict__ hist, int npass, int max_o, unsigned long long* s,
                           uint32_t* wtot) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) {
    s[0] = 0ull;
    s[1] = (unsigned long long)(max_o - 1);
  }
  __syncthreads();
  for (int q = 0; q < npass; ++q) {
    const unsigned long long k = s[1];
    const uint32_t v = hist[q * 256 + t];
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(inc, o);
      if (lane >= o) inc += x;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    for (int i = 0; i < w; ++i) inc += wtot[i];
    const unsigned long long ex = inc - v;
    if (ex <= k && (t == 255 || k < inc)) {
      s[0] |= (unsigned long long)t << (56 - 8 * q);
      s[1] = k - ex;
    }
    __syncthreads();
  }
}

// Pass 0 walks every point's claim flag and lists the claimers by slot
// (cids[pt_slot[i]] = i: the first scan's ranks); the later passes and
// k_sel_apply walk that list (the occupied voxels, 2.7 M of c5's 20 M points).
__global__ void __launch_bounds__(kBlock) k_sel_hist(int64_t n, const int32_t* __restrict__ flag,
                                                     const int32_t* __restrict__ pt_slot,
                                                     int32_t* __restrict__ cids, const int32_t* __restrict__ n_vox,
                                                     uint64_t seed, int pass, int max_o,
                                                     SelState* __restrict__ st, uint32_t* __restrict__ hist) {
  // pass 0 decides from the voxel count (the first scan's total) and publishes the
  // flag for the later passes, k_sel_apply and the rescan
  const bool active = pass == 0 ? *n_vox > max_o : st->active != 0;
  if (pass == 0 && blockIdx.x == 0 && threadIdx.x == 0) st->active = active ? 1 : 0;
  if (!active) return;
  __shared__ uint32_t h[256];
  __shared__ unsigned long long s[2];
  __shared__ uint32_t wtot[kBlock / 64];
  h[threadIdx.x] = 0;
  sel_derive(hist, pass, max_o, s, wtot);
  const unsigned long long prefix = s[0];
  const int shift = 56 - 8 * pass;
  const unsigned long long hi = shift >= 56 ? 0ull : (~0ull << (shift + 8));
  if (pass == 0) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
      if (!flag[i]) continue;
      cids[pt_slot[i]] = (int32_t)i;
      const unsigned long long key = res_vkey(seed, (uint32_t)i);
      atomicAdd(&h[(key >> shift) & 255u], 1u);
    }
  } else {
    const int64_t nv = *n_vox;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nv; r += (int64_t)gridDim.x * blockDim.x) {
      const unsigned long long key = res_vkey(seed, (uint32_t)cids[r]);
      if (((key ^ prefix) & hi) == 0) atomicAdd(&h[(key >> shift) & 255u], 1u);
    }
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(hist + pass * 256 + threadIdx.x, h[threadIdx.x]);
}

// keep the claimer of a voxel only when its voxel is among the max_o kept
__global__ void __launch_bounds__(kBlock) k_sel_apply(const int32_t* __restrict__ cids,
                                                      const int32_t* __restrict__ n_vox, uint64_t seed, int max_o,
                                                      const SelState* __restrict__ st,
                                                      const uint32_t* __restrict__ hist, int32_t* __restrict__ flag) {
  if (!st->active) return;
  __shared__ unsigned long long s[2];
  __shared__ uint32_t wtot[kBlock / 64];
  sel_derive(hist, kSelPasses, max_o, s, wtot);
  const unsigned long long thr = s[0];
  const int64_t nv = *n_vox;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nv; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t i = cids[r];
    if (res_vkey(seed, (uint32_t)i) > thr) flag[i] = 0;
  }
}

// map_coor2occ + fill_occ2pnts (qpiw.py:305-387), one thread per sorted
// point of a kept voxel.  The run's head (its claimer) writes slot ->
// coor_2_occ / occ_2_coor, the occupancy byte (dilated by query_size in
// k_dilate_zy / k_dilate_x), the voxel's point count (`voxel_idx > 0`,
// qpiw.py:372: under slot0_drop the voxel holding slot 0 gets no points) and,
// when the run exceeds P, the P records of smallest reservoir key (res_pkey;
// the reference: reservoir with a time seed).  Runs that fit P: every point
// writes its own record, number j - head (the run is in ascending id order).
template <typename K>
__global__ void __launch_bounds__(kBlock) k_claim(const float* __restrict__ xyz, int64_t n, GridDev g0,
                                                  const QGrid* __restrict__ geo, const K* __restrict__ skey,
                                                  const int32_t* __restrict__ sid, K sentinel,
                                                  const int32_t* __restrict__ flag, const int32_t* __restrict__ pt_slot,
                                                  const int32_t* __restrict__ cell_start,
                                                  const int32_t* __restrict__ cell_end,
                                                  int32_t* __restrict__ coor_2_occ, int32_t* __restrict__ occ_2_coor,
                                                  uint8_t* __restrict__ occ_bytes, uint8_t* __restrict__ held_bytes,
                                                  uint32_t* __restrict__ coarse, int32_t* __restrict__ occ_numpnts,
                                                  float4* __restrict__ occ_pts, int32_t* __restrict__ slot_run,
                                                  int32_t* counters) {
  const GridDev g = with_geom(g0, geo);
  int dropped = 0, mx = 0;
  const int lane = threadIdx.x & 63;
  const uint64_t upto = lane == 63 ? ~0ull : (2ull << lane) - 1ull;   // lanes 0 .. lane
  // A wave takes 64 consecutive sorted points: a run's head lane (the first
  // point of its voxel) loads the run's claim flag, slot and length, and the
  // run's other lanes in the wave take them by shuffle; only lanes whose head
  // lies in an earlier wave look the run up through cell_start (c5: ~5 random
  // loads per point -> ~3 per run).
  for (int64_t j0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~63ll; j0 < n;
       j0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = j0 + lane;
    const K key = j < n ? skey[j] : sentinel;
    const bool in = key != sentinel;
    const bool head = in && (j == 0 || skey[j - 1] != key);
    const int64_t cell = (int64_t)key;
    int hd = (int)j, ok = 0, slot = 0, cnt = 0;
    if (head) {
      const int id0 = sid[j];
      ok = flag[id0];
      slot = pt_slot[id0];
      cnt = cell_end[cell] - (int)j;
    }
    const uint64_t heads = __ballot(head) & upto;
    const int hl = heads ? 63 - __builtin_clzll(heads) : -1;   // this lane's head lane, if in the wave
    const int ok_s = __shfl(ok, hl < 0 ? 0 : hl), slot_s = __shfl(slot, hl < 0 ? 0 : hl),
              cnt_s = __shfl(cnt, hl < 0 ? 0 : hl);
    if (hl >= 0) {
      hd = (int)j0 + hl;
      ok = ok_s;
      slot = slot_s;
      cnt = cnt_s;
    } else if (in) {   // the run began in an earlier wave
      hd = cell_start[cell];
      const int id0 = sid[hd];
      ok = flag[id0];
      slot = pt_slot[id0];
      cnt = cell_end[cell] - hd;
    }
    // ok: the voxel survived the max_o reservoir (slot < max_o always then)
    const bool live = in && ok && slot < g.max_o;
    const int cnt_kept = (g.slot0_drop && slot == 0) ? 0 : cnt;
    const int v = in ? sid[j] : 0;
    // fill_occ2pnts' reservoir for a run that lies inside this wave: each lane
    // ranks its point's res_pkey among the run's (keys are distinct), the P
    // smallest are kept and numbered in run (= id) order by a ballot.  Runs that
    // cross the wave go to k_reservoir (slot_run = head position).
    const bool rw = live && cnt_kept > g.P && hd >= j0 && hd + cnt <= j0 + 64;
    bool keep_rec = live && cnt_kept > 0 && cnt_kept <= g.P;
    int rec = (int)j - hd;
    if (__ballot(rw)) {
      // res_pkey = (hash << 32) | id and the run's ids ascend with the lane, so
      // key order = (hash, run position): one 32-bit shuffle per step
      const uint32_t myh = res_pkey_hash(g.seed, (uint32_t)v);
      int span = rw ? cnt : 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) span = max(span, __shfl_xor(span, o));
      const int hl0 = rw ? hd - (int)j0 : 0;
      const int me = lane - hl0;   // this lane's position in its run
      int rank = 0;
      for (int t = 0; t < span; ++t) {   // wave-uniform trip count
        const int src = rw && t < cnt ? hl0 + t : lane;
        const uint32_t ht = (uint32_t)__shfl((int)myh, src);
        rank += (rw && t < cnt && (ht < myh || (ht == myh && t < me))) ? 1 : 0;
      }
      const bool sel = rw && rank < g.P;
      const uint64_t selm = __ballot(sel);
      const uint64_t run_lo = hl0 >= 64 ? 0ull : ~((1ull << hl0) - 1ull);   // lanes hd - j0 .. 63
      const int rr = __popcll(selm & run_lo & ((1ull << lane) - 1ull));
      if (sel) rec = rr;
      keep_rec = keep_rec || sel;
    }
    int c[3] = {0, 0, 0};
    if (live && head) {
      if (cell <= 0x7fffffff) {   // 32-bit division when the cell index fits
        const int r = (int)cell / g.dims[2];
        c[2] = (int)cell - r * g.dims[2];
        c[0] = r / g.dims[1];
        c[1] = r - c[0] * g.dims[1];
      } else {
        c[2] = (int)(cell % g.dims[2]);
        c[1] = (int)((cell / g.dims[2]) % g.dims[1]);
        c[0] = (int)(cell / ((int64_t)g.dims[2] * g.dims[1]));
      }
    }
    // the KNN's coarse column map: bit y of word (z / 8, x, y / 32) for every held
    // voxel.  A column's held cells of one z-block are consecutive heads of the
    // sorted keys with the same word and bit: only the first of such a run in the
    // wave sets it (one same-address atomic per run instead of per voxel; they
    // serialised at the L2: 27 us of this kernel at the headline and at c5)
    {
      const bool cset = live && head && cnt_kept > 0;
      const int64_t cw = cset ? ((int64_t)(c[2] >> 3) * g.dims[0] + c[0]) * ((g.dims[1] + 31) >> 5) + (c[1] >> 5) : -1;
      const int cb = c[1] & 31;
      const uint64_t cm = __ballot(cset) & ((1ull << lane) - 1ull);   // setting lanes below this one
      const int pl = cm ? 63 - __builtin_clzll(cm) : lane;
      const int pw_lo = __shfl((int)(uint32_t)cw, pl), pw_hi = __shfl((int)(cw >> 32), pl), pb = __shfl(cb, pl);
      const int64_t pw = (int64_t)(((uint64_t)(uint32_t)pw_hi << 32) | (uint32_t)pw_lo);
      if (cset && (!cm || pw != cw || pb != cb)) atomicOr(coarse + cw, 1u << cb);
    }
    if (!live) continue;
    if (head) {
      coor_2_occ[cell] = slot;
      occ_2_coor[slot * 3 + 0] = c[0];
      occ_2_coor[slot * 3 + 1] = c[1];
      occ_2_coor[slot * 3 + 2] = c[2];
      occ_bytes[cell] = 1;
      if (cnt_kept > 0) held_bytes[cell] = 1;   // the query index's held voxels (was k_mark_held)
      occ_numpnts[slot] = cnt_kept;
      const int keep = min(cnt_kept, g.P);
      if (cnt_kept > g.P) slot_run[slot] = rw ? -1 : hd;   // -1: records written here, else by k_reservoir
      dropped += cnt_kept - keep;
      mx = max(mx, cnt_kept);
    }
    if (keep_rec)
      occ_pts[(int64_t)slot * g.P + rec] =
          make_float4(xyz[(int64_t)v * 3], xyz[(int64_t)v * 3 + 1], xyz[(int64_t)v * 3 + 2], __int_as_float(v));
  }
  dropped = wave_sum_i32(dropped);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  __shared__ int red[2][kBlock / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = dropped;
    red[1][w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int d = 0, m = 0;
    for (int q = 0; q < kBlock / 64; ++q) {
      d += red[0][q];
      m = max(m, red[1][q]);
    }
    if (d) atomicAdd(counters + 2, d);
    if (m) atomicMax(counters + 3, m);
  }
}

// fill_occ2pnts' reservoir (qpiw.py:377-384) for the voxels whose run exceeds
// P: the P points of smallest res_pkey (keys are distinct: the id is their low
// half), written in ascending id order.  One wave per 64 slots; the wave takes
// its overflowing slots one at a time (ballot) and works through each run with
// all 64 lanes: P rounds of a wave-wide minimum above the previous round's key
// find the P-th smallest key, then one ballot-ranked pass writes the points at
// or below it in run (= id) order.  (One lane per voxel walking its run P
// times serialised the long runs: c5, 1.76 ms.)
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
    const uint64_t w = ((uint64_t)hi << 32) | lo;
    v = w < v ? w : v;
  }
  return v;
}

constexpr int kResChunks = 8;   // runs of <= 512 points: hashes held in registers (longer: recomputed)

__global__ void __launch_bounds__(kBlock) k_reservoir(int n_slots, GridDev g, const float* __restrict__ xyz,
                                                      const int32_t* __restrict__ sid,
                                                      const int32_t* __restrict__ occ_numpnts,
                                                      const int32_t* __restrict__ slot_run,
                                                      float4* __restrict__ occ_pts) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  for (int64_t s0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63ll; s0 < n_slots;
       s0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sl = s0 + lane;
    const int mine = sl < n_slots ? occ_numpnts[sl] : 0;
    // (slot_run -1: the run fitted one wave of k_claim, which wrote its records)
    uint64_t todo = __ballot(mine > g.P && slot_run[sl < n_slots ? sl : 0] >= 0);
    while (todo) {
      const int b = __builtin_ctzll(todo);
      todo &= todo - 1;
      const int s = (int)s0 + b;
      const int cnt = __shfl(mine, b);
      const int32_t* ids = sid + slot_run[s];
      float4* dst = occ_pts + (int64_t)s * g.P;
      if (cnt <= 64 * kResChunks) {
        // key order = (hash, run position) (res_pkey's low half is the id, ascending
        // along the run).  MSB-first radix select of the P-th smallest hash with
        // ballots: per bit, the candidates whose bit is 0 are counted; the selection
        // stops as soon as the remaining candidates are exactly the ones still needed.
        uint32_t hs[kResChunks];
        uint64_t cand[kResChunks], sel[kResChunks];
#pragma unroll
        for (int c = 0; c < kResChunks; ++c) {
          const int e = 64 * c + lane;
          hs[c] = e < cnt ? res_pkey_hash(g.seed, (uint32_t)ids[e]) : 0u;
          cand[c] = __ballot(e < cnt);
          sel[c] = 0ull;
        }
        int rem = g.P;
        for (int bit = 31; bit >= 0 && rem > 0; --bit) {
          uint64_t zero[kResChunks];
          int n0 = 0, nc = 0;
#pragma unroll
          for (int c = 0; c < kResChunks; ++c) {
            zero[c] = 0ull;
            if (64 * c < cnt) {   // wave-uniform: only the run's chunks
              zero[c] = cand[c] & __ballot(((hs[c] >> bit) & 1u) == 0u);
              n0 += __popcll(zero[c]);
            }
          }
          if (rem <= n0) {
#pragma unroll
            for (int c = 0; c < kResChunks; ++c) cand[c] = zero[c];
          } else {
            rem -= n0;
#pragma unroll
            for (int c = 0; c < kResChunks; ++c) {
              sel[c] |= zero[c];
              cand[c] &= ~zero[c];
            }
          }
#pragma unroll
          for (int c = 0; c < kResChunks; ++c) nc += __popcll(cand[c]);
          if (nc == rem) {   // every remaining candidate is in
#pragma unroll
            for (int c = 0; c < kResChunks; ++c) sel[c] |= cand[c];
            rem = 0;
          }
        }
        // equal hashes past bit 0: the first `rem` of them in run (= id) order
#pragma unroll
        for (int c = 0; c < kResChunks; ++c) {
          while (rem > 0 && cand[c]) {
            const uint64_t lo = cand[c] & (~cand[c] + 1ull);
            sel[c] |= lo;
            cand[c] &= ~lo;
            --rem;
          }
        }
        int base = 0;
#pragma unroll
        for (int c = 0; c < kResChunks; ++c) {
          if ((sel[c] >> lane) & 1ull) {
            const int v = ids[64 * c + lane];
            dst[base + __popcll(sel[c] & below)] =
                make_float4(xyz[(int64_t)v * 3], xyz[(int64_t)v * 3 + 1], xyz[(int64_t)v * 3 + 2], __int_as_float(v));
          }
          base += __popcll(sel[c]);
        }
        continue;
      }
      // long runs: P rounds of a wave-wide minimum above the previous round's key
      uint64_t thr = 0;
      for (int q = 0; q < g.P; ++q) {
        uint64_t best = ~0ull;
        for (int e = lane; e < cnt; e += 64) {
          const uint64_t k = res_pkey(g.seed, (uint32_t)ids[e]);
          if ((q == 0 || k > thr) && k < best) best = k;
        }
        thr = wave_min_u64(best);
      }
      int written = 0;
      for (int e0 = 0; e0 < cnt && written < g.P; e0 += 64) {
        const int e = e0 + lane;
        const int v = e < cnt ? ids[e] : 0;
        const bool take = e < cnt && res_pkey(g.seed, (uint32_t)v) <= thr;
        const uint64_t m = __ballot(take);
        const int pos = written + __popcll(m & below);
        if (take && pos < g.P)
          dst[pos] = make_float4(xyz[(int64_t)v * 3], xyz[(int64_t)v * 3 + 1], xyz[(int64_t)v * 3 + 2],
                                 __int_as_float(v));
        written += __popcll(m);
      }
    }
  }
}

// The dilation of map_coor2occ (qpiw.py:321-337: every kept voxel c marks the
// cells [c - qs/2, c + (qs+1)/2) of each axis, clipped to the grid) as a
// separable box filter over occupancy bytes: cell v is marked when an
// occupied voxel lies in [v - (qs+1)/2 + 1, v + qs/2] on every axis.  One wave
// per (x, y) row of cells, lanes along z; 32-bit row arithmetic only.
__device__ __forceinline__ void dil_range(int v, int qs, int dim, int& lo, int& hi) {
  lo = max(0, v - (qs + 1) / 2 + 1);
  hi = min(dim - 1, v + qs / 2);
}

// z and y: in = one byte per occupied cell, out = the zy-dilated bytes.  Up to
// 3 x 3 contributing cells (query_size <= 3, every flag set) as independent
// predicated loads, so a lane has them all in flight; larger boxes loop.
__global__ void __launch_bounds__(kBlock) k_dilate_zy(GridDev g0, const QGrid* __restrict__ geo,
                                                      const uint8_t* __restrict__ in, uint8_t* __restrict__ out) {
  const GridDev g = with_geom(g0, geo);
  const int rows = g.dims[0] * g.dims[1];
  const int lane = threadIdx.x & 63;
  const bool small = g.qs[1] <= 3 && g.qs[2] <= 3;
  for (int row = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); row < rows;
       row += (int)((gridDim.x * blockDim.x) >> 6)) {
    const int x = row / g.dims[1], y = row - x * g.dims[1];
    int y0, y1;
    dil_range(y, g.qs[1], g.dims[1], y0, y1);
    for (int z = lane; z < g.dims[2]; z += 64) {
      int z0, z1;
      dil_range(z, g.qs[2], g.dims[2], z0, z1);
      uint8_t m = 0;
      if (small) {
        uint8_t v[9];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) {
            const bool ok = y0 + a <= y1 && z0 + b <= z1;
            const int yy = ok ? y0 + a : y, zz = ok ? z0 + b : z;
            v[a * 3 + b] = ok ? in[((int64_t)x * g.dims[1] + yy) * g.dims[2] + zz] : 0;
          }
#pragma unroll
        for (int q = 0; q < 9; ++q) m |= v[q];
      } else {
        for (int yy = y0; yy <= y1; ++yy) {
          const uint8_t* r = in + ((int64_t)x * g.dims[1] + yy) * g.dims[2];
          for (int zz = z0; zz <= z1; ++zz) m |= r[zz];
        }
      }
      out[(int64_t)row * g.dims[2] + z] = m;
    }
  }
}

// x: in = the zy-dilated bytes, out = the dilated occupancy bytes
__global__ void __launch_bounds__(kBlock) k_dilate_x(GridDev g0, const QGrid* __restrict__ geo,
                                                     const uint8_t* __restrict__ in, uint8_t* __restrict__ out) {
  const GridDev g = with_geom(g0, geo);
  const int rows = g.dims[0] * g.dims[1];
  const int64_t plane = (int64_t)g.dims[1] * g.dims[2];
  const int lane = threadIdx.x & 63;
  for (int row = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); row < rows;
       row += (int)((gridDim.x * blockDim.x) >> 6)) {
    const int x = row / g.dims[1];
    int x0, x1;
    dil_range(x, g.qs[0], g.dims[0], x0, x1);
    const int64_t base = (int64_t)row * g.dims[2];
    for (int z = lane; z < g.dims[2]; z += 64) {
      uint8_t m = 0;
      if (g.qs[0] <= 3) {
        uint8_t v[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) v[a] = x0 + a <= x1 ? in[base + (int64_t)(x0 + a - x) * plane + z] : 0;
        m = v[0] | v[1] | v[2];
      } else {
        for (int xx = x0; xx <= x1; ++xx) m |= in[base + (int64_t)(xx - x) * plane + z];
      }
      out[base + z] = m;
    }
  }
}

// Dilated occupancy bytes -> bitmap word w (cells 32w .. 32w+31).
__global__ void __launch_bounds__(kBlock) k_pack_bits(const uint8_t* __restrict__ occ_bytes, int64_t words,
                                                      uint32_t* __restrict__ occ_bits) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < words;
       w += (int64_t)gridDim.x * blockDim.x) {
    const uint4* b = reinterpret_cast<const uint4*>(occ_bytes + 32 * w);
    const uint4 lo = b[0], hi = b[1];
    const unsigned v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) bits |= ((v[q] >> (8 * k)) & 0xffu ? 1u : 0u) << (4 * q + k);
    occ_bits[w] = bits;
  }
}

// ---------------------------------------------------------------- query index
// Held voxels (>= 1 kept point: the slot-0 voxel under slot0_drop and the
// truncated ones are skipped exactly as the reference's loop `g < min(P,
// occ_numpnts)` skips them) arrive as one byte per cell from k_claim; packed
// to the query bitmap words with their popcounts.
__global__ void __launch_bounds__(kBlock) k_pack_held(const uint8_t* __restrict__ bytes, int64_t words,
                                                      uint2* __restrict__ qw, int32_t* __restrict__ wcnt) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < words;
       w += (int64_t)gridDim.x * blockDim.x) {
    const uint4* b = reinterpret_cast<const uint4*>(bytes + 32 * w);
    const uint4 lo = b[0], hi = b[1];
    const unsigned v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) bits |= ((v[q] >> (8 * k)) & 0xffu ? 1u : 0u) << (4 * q + k);
    qw[w].x = bits;
    wcnt[w] = __popc(bits);
  }
}

__global__ void __launch_bounds__(kBlock) k_word_rank(int64_t words, const int32_t* __restrict__ wrank,
                                                      uint2* __restrict__ qw) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < words;
       w += (int64_t)gridDim.x * blockDim.x)
    qw[w].y = (uint32_t)wrank[w];
}

__global__ void __launch_bounds__(kBlock) k_rank_slots(int n_slots, GridDev g0, const QGrid* __restrict__ geo,
                                                       const int32_t* __restrict__ occ_numpnts,
                                                       const int32_t* __restrict__ occ_2_coor,
                                                       const uint2* __restrict__ qw, int32_t* __restrict__ rank_slot,
                                                       int32_t* __restrict__ rank_cnt) {
  const GridDev g = with_geom(g0, geo);
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < n_slots; s += gridDim.x * blockDim.x) {
    if (occ_numpnts[s] <= 0 || occ_2_coor[s * 3] < 0) continue;
    const int64_t cell =
        ((int64_t)occ_2_coor[s * 3] * g.dims[1] + occ_2_coor[s * 3 + 1]) * g.dims[2] + occ_2_coor[s * 3 + 2];
    const uint2 wd = qw[cell >> 5];
    const int r = (int)wd.y + __popc(wd.x & ((1u << (cell & 31)) - 1u));
    rank_slot[r] = s;
    rank_cnt[r] = min(g.P, occ_numpnts[s]);
  }
}

// 16 lanes per rank: a voxel's records are one contiguous read and write
// The build's statistics for the host (counters, the device geometry, the bbox
// it came from) written by block 0 of the build's last kernel straight into the
// handle's pinned host buffers (three hipMemcpyAsync before: ~15 us of the build).
struct HostStats {
  const int32_t* counters;
  const QGrid* geo;
  const float* bbox;   // NULL: not a device-geometry build
  int32_t* h_cnt;
  QGrid* h_geo;
  float* h_bbox;
};

__global__ void __launch_bounds__(kBlock) k_fill_recs(GridDev g, const int32_t* __restrict__ n_ranks,
                                                      const int32_t* __restrict__ rank_slot,
                                                      const int32_t* __restrict__ rec_off,
                                                      const float4* __restrict__ occ_pts, float4* __restrict__ recs,
                                                      HostStats hs) {
  if (blockIdx.x == 0) {   // every value is final: written by the build's earlier kernels
    const int t = threadIdx.x;
    if (t < 8) hs.h_cnt[t] = hs.counters[t];
    if (t >= 8 && t < 8 + (int)(sizeof(QGrid) / 4))
      reinterpret_cast<int32_t*>(hs.h_geo)[t - 8] = reinterpret_cast<const int32_t*>(hs.geo)[t - 8];
    if (hs.bbox && t >= 32 && t < 40) hs.h_bbox[t - 32] = hs.bbox[t - 32];
  }
  const int64_t nr = *n_ranks;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nr * 16;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t >> 4;
    const int s = rank_slot[r], o = rec_off[r], c = rec_off[r + 1] - o;
    for (int q = (int)(t & 15); q < c; q += 16) recs[o + q] = occ_pts[(int64_t)s * g.P + q];
  }
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_points_bbox(const float* xyz_dev, int64_t n, float* out6_dev, void* stream) {
  PNR_CHECK_ARG(xyz_dev && out6_dev, "bbox: null pointer");
  PNR_CHECK_ARG(n > 0, "bbox: empty point set");
  hipStream_t st = as_stream(stream);
  unsigned* acc = reinterpret_cast<unsigned*>(out6_dev);
  hipLaunchKernelGGL(k_bbox_init, dim3(1), dim3(64), 0, st, acc);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bbox, dim3(grid_for(cdiv(n, 4), kBlock, 512)), dim3(kBlock), 0, st, xyz_dev, n, acc);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bbox_fin, dim3(1), dim3(64), 0, st, acc);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// bytes of the KNN's coarse column map for allocation bounds dims (16-B padded)
static size_t coarse_bytes(const int dims[3]) {
  return (((size_t)cdiv(dims[2], 8) * dims[0] * cdiv(dims[1], 32) * 4) + 15) & ~(size_t)15;
}

// Sort, claim, count and fill (K: the cell key type, uint32 unless the grid
// has 2^32 - 1 cells or more).
template <typename K>
static int build_tables(pnr_handle* h, const float* xyz_dev, int64_t n, const GridDev& g, int64_t gvol,
                        int64_t words, int64_t cap_o, hipStream_t st) {
  int rc;
  const QGrid* geo = h->geom.as<QGrid>();
  int32_t* counters = h->counters.as<int32_t>();
  int32_t* pt_flag = h->pt_flag.as<int32_t>();
  int32_t* pt_slot = h->pt_slot.as<int32_t>();
  int32_t* cell_start = h->cell_start.as<int32_t>();
  int32_t* cell_end = h->cell_end.as<int32_t>();
  const K sentinel = (K)gvol;
  const int bits = 64 - __builtin_clzll((unsigned long long)gvol);
  // 8-bit digits (kRB): 9-bit ones save c5's fourth pass (26-bit keys) but each
  // scatter pass took 185 instead of 120 us (4 keys per digit run of a tile:
  // partial lines) and the build 3.04 vs 2.79 ms (round 6)
  constexpr int kRB = 8;
  const int rbits = kRB;
  const int passes = (bits + rbits - 1) / rbits;
  const int tiles = (int)cdiv(n, kRsTile);
  const unsigned gp = grid_for(n, kBlock);

  // (cell, point id) sorted by cell, ids ascending inside a cell
  K* keys[2] = {h->sort_k[0].as<K>(), h->sort_k[1].as<K>()};
  int32_t* vals[2] = {h->sort_v[0].as<int32_t>(), h->sort_v[1].as<int32_t>()};
  const int64_t kblocks = cdiv(n > cap_o ? n : cap_o, kRsTile);
  PNR_CHECK_ARG(kblocks < (int64_t)1 << 31, "grid_build: too many sort tiles");
  hipLaunchKernelGGL((k_cell_keys<kRB, K>), dim3((unsigned)kblocks), dim3(kBlock), 0, st,
                     xyz_dev, n, g, geo, sentinel, keys[0], cap_o, pt_flag, h->occ_numpnts.as<int32_t>(),
                     h->occ_2_coor.as<int32_t>(), counters, tiles, h->sort_hist.as<int32_t>(),
                     n > cap_o ? reinterpret_cast<uint32_t*>(h->sel.as<SelState>() + 1) : nullptr);
  PNR_LAUNCH_CHECK();
  int cur = 0;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = rbits * pass;
    if (pass > 0) {   // (pass 0's histogram: k_cell_keys)
      hipLaunchKernelGGL((k_rs_hist<kRB, K>), dim3(tiles), dim3(kBlock), 0, st, keys[cur], n,
                         shift, tiles, h->sort_hist.as<int32_t>());
      PNR_LAUNCH_CHECK();
    }
    if ((rc = exclusive_scan(h->sort_hist.as<int32_t>(), ((int64_t)1 << rbits) * tiles, nullptr,
                             h->sort_offs.as<int32_t>(), (int64_t)(h->sort_offs.bytes / 4), nullptr, h->scan_tmp.p,
                             h->scan_tmp.bytes, st)))
      return rc;
    hipLaunchKernelGGL((k_rs_scatter<kRB, K>), dim3(tiles), dim3(kBlock), 0, st, keys[cur],
                       pass ? vals[cur] : nullptr, n, shift, tiles, h->sort_offs.as<int32_t>(), keys[cur ^ 1],
                       vals[cur ^ 1]);
    PNR_LAUNCH_CHECK();
    cur ^= 1;
  }
  const K* skey = keys[cur];
  const int32_t* sid = vals[cur];
  hipLaunchKernelGGL(k_runs<K>, dim3(gp), dim3(kBlock), 0, st, skey, sid, n, sentinel, pt_flag, cell_start,
                     cell_end, counters);
  PNR_LAUNCH_CHECK();
  // slot = rank of the claimer's point id (the serial claim order)
  if ((rc = exclusive_scan(pt_flag, n, nullptr, pt_slot, (int64_t)(h->pt_slot.bytes / 4), counters + 0, h->scan_tmp.p, h->scan_tmp.bytes, st)))
    return rc;
  if (n > cap_o) {
    // more points than max_o: the occupied voxels may overflow it (counters[0]
    // holds their number on the device); keep the reservoir's max_o of them
    SelState* ss = h->sel.as<SelState>();
    uint32_t* hist = reinterpret_cast<uint32_t*>(ss + 1);
    const unsigned gs = grid_for(n, kBlock, 1024);
    // the claimers listed by slot (pass 0) in sort_v[cur ^ 1]: free after the sort
    int32_t* cids = vals[cur ^ 1];
    // passes 1.. and the apply walk the claimer list (<= the occupied voxels): fewer blocks
    const unsigned gl = grid_for(cap_o, kBlock, 256);
    for (int pass = 0; pass < kSelPasses; ++pass) {
      hipLaunchKernelGGL(k_sel_hist, dim3(pass ? gl : gs), dim3(kBlock), 0, st, n, pt_flag, pt_slot, cids,
                         counters + 0, g.seed, pass, (int)cap_o, ss, hist);
      PNR_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_sel_apply, dim3(gl), dim3(kBlock), 0, st, cids, counters + 0, g.seed, (int)cap_o, ss, hist,
                       pt_flag);
    PNR_LAUNCH_CHECK();
    if ((rc = exclusive_scan(pt_flag, n, nullptr, pt_slot, (int64_t)(h->pt_slot.bytes / 4), counters + 6, h->scan_tmp.p, h->scan_tmp.bytes, st, 0,
                             &ss->active)))
      return rc;
  }
  // cell_bytes = [occupancy bytes | held bytes | coarse column map | word ranks]: the
  // first three cleared by one memset
  uint8_t* occ_bytes = h->cell_bytes.as<uint8_t>();
  PNR_HIP(hipMemsetAsync(occ_bytes, 0, (size_t)words * 64 + coarse_bytes(g.dims), st));
  hipLaunchKernelGGL(k_claim<K>, dim3(gp), dim3(kBlock), 0, st, xyz_dev, n, g, geo, skey, sid, sentinel, pt_flag,
                     pt_slot, cell_start, cell_end, h->coor_2_occ.as<int32_t>(), h->occ_2_coor.as<int32_t>(),
                     occ_bytes, occ_bytes + words * 32, reinterpret_cast<uint32_t*>(occ_bytes + words * 64),
                     h->occ_numpnts.as<int32_t>(), h->occ_pts.as<float4>(), h->q_rank_slot.as<int32_t>(), counters);
  PNR_LAUNCH_CHECK();
  // q_rank_slot is scratch until the query index below: slot -> run start
  hipLaunchKernelGGL(k_reservoir, dim3(grid_for(cap_o, kBlock)), dim3(kBlock), 0, st, (int)cap_o, g, xyz_dev, sid,
                     h->occ_numpnts.as<int32_t>(), h->q_rank_slot.as<int32_t>(), h->occ_pts.as<float4>());
  PNR_LAUNCH_CHECK();
  {
    // cell_end is dead after k_claim: its storage holds the zy-dilated bytes
    uint8_t* zy = h->cell_end.as<uint8_t>();
    const unsigned gr = grid_for((int64_t)g.dims[0] * g.dims[1] * 64, kBlock, 1 << 16);   // one wave per row
    hipLaunchKernelGGL(k_dilate_zy, dim3(gr), dim3(kBlock), 0, st, g, geo, occ_bytes, zy);
    PNR_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_dilate_x, dim3(gr), dim3(kBlock), 0, st, g, geo, zy, occ_bytes);
    PNR_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_pack_bits, dim3(grid_for(words, kBlock)), dim3(kBlock), 0, st, occ_bytes, words,
                     h->occ_bits.as<uint32_t>());
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// The build proper (both entry points): p gives the allocation bounds (dims)
// and the by-value parameters; the exact geometry is already in h->geom.
static int grid_build_body(pnr_handle* h, const float* xyz_dev, int64_t n, const pnr_grid_params* p,
                           hipStream_t st) {
  PNR_CHECK_ARG(n > 0 && n < (int64_t)1 << 31, "grid_build: point count %lld out of range", (long long)n);
  PNR_CHECK_ARG(p->dims[0] > 0 && p->dims[1] > 0 && p->dims[2] > 0, "grid_build: empty grid dims");
  PNR_CHECK_ARG(p->max_o > 0 && p->P > 0, "grid_build: max_o and P must be > 0");
  PNR_CHECK_ARG(p->vsize[0] > 0 && p->vsize[1] > 0 && p->vsize[2] > 0, "grid_build: vsize <= 0");
  const int64_t gvol = (int64_t)p->dims[0] * p->dims[1] * p->dims[2];
  PNR_CHECK_ARG(gvol < (int64_t)1 << 36, "grid_build: grid of %lld cells", (long long)gvol);
  int rc;
  const int64_t words = cdiv(gvol, 32);
  const int64_t cap_o = p->max_o;
  const bool wide = gvol >= ((int64_t)1 << 32) - 1;   // the sentinel key gvol must fit the key type
  const size_t kbytes = wide ? 8 : 4;
  const int64_t hist_n = (int64_t)256 * cdiv(n, kRsTile) + 1;
  int64_t scan_n = n;
  for (int64_t m : {cap_o, words, hist_n}) scan_n = m > scan_n ? m : scan_n;
  if ((rc = h->coor_2_occ.ensure(gvol * 4)) || (rc = h->cell_end.ensure(gvol * 4)) ||
      (rc = h->cell_bytes.ensure(words * 68 + 16 + coarse_bytes(p->dims))) || (rc = h->occ_bits.ensure(words * 4)) ||
      (rc = h->occ_numpnts.ensure(cap_o * 4)) || (rc = h->occ_pts.ensure(cap_o * p->P * sizeof(float4))) ||
      (rc = h->occ_2_coor.ensure(cap_o * 12)) || (rc = h->sort_k[0].ensure(n * kbytes)) ||
      (rc = h->sort_k[1].ensure(n * kbytes)) || (rc = h->sort_v[0].ensure(n * 4)) ||
      (rc = h->sort_v[1].ensure(n * 4)) || (rc = h->sort_hist.ensure(hist_n * 4)) ||
      (rc = h->sort_offs.ensure(hist_n * 4)) || (rc = h->cell_start.ensure(gvol * 4)) ||
      (rc = h->pt_flag.ensure(n * 4)) || (rc = h->pt_slot.ensure((n + 1) * 4)) ||
      (rc = h->counters.ensure(8 * 4)) || (rc = h->sel.ensure(sizeof(SelState) + kSelPasses * 256 * 4)) ||
      (rc = h->scan_tmp.ensure(scan_scratch_bytes(scan_n))) ||
      (rc = h->q_words.ensure(words * 8)) || (rc = h->q_wcnt.ensure((words + 1) * 4)) ||
      (rc = h->q_rank_slot.ensure(cap_o * 4)) || (rc = h->q_rank_cnt.ensure(cap_o * 4)) ||
      (rc = h->q_rec_off.ensure((cap_o + 1) * 4)) || (rc = h->q_recs.ensure(n * sizeof(float4))))
    return rc;
  int32_t* occ_numpnts = h->occ_numpnts.as<int32_t>();
  int32_t* occ_2_coor = h->occ_2_coor.as<int32_t>();
  int32_t* counters = h->counters.as<int32_t>();
  const QGrid* geo = h->geom.as<QGrid>();

  GridDev g;
  for (int a = 0; a < 3; ++a) {
    g.shift[a] = p->shift[a];
    g.vs[a] = p->vsize[a];
    g.dims[a] = p->dims[a];
    g.qs[a] = p->query_size[a];
  }
  g.max_o = p->max_o;
  g.P = p->P;
  g.slot0_drop = p->slot0_drop;
  g.seed = p->seed;

  // (pt_flag, the slot tables and the counters are cleared by k_cell_keys)
  PNR_HIP(hipMemsetAsync(h->coor_2_occ.p, 0xff, (size_t)gvol * 4, st));
  if ((rc = wide ? build_tables<uint64_t>(h, xyz_dev, n, g, gvol, words, cap_o, st)
                 : build_tables<uint32_t>(h, xyz_dev, n, g, gvol, words, cap_o, st)))
    return rc;
  float4* occ_pts = h->occ_pts.as<float4>();
  uint8_t* occ_bytes = h->cell_bytes.as<uint8_t>();
  // query index: held voxels ranked in cell order (k_knn's tables)
  {
    uint2* qw = h->q_words.as<uint2>();
    int32_t* wcnt = h->q_wcnt.as<int32_t>();
    const uint8_t* held_bytes = occ_bytes + words * 32;                    // written by k_claim
    const size_t cb = coarse_bytes(p->dims);
    h->coarse_off = (size_t)words * 64;   // the KNN reads the coarse map there (query.hip)
    int32_t* wrank = reinterpret_cast<int32_t*>(occ_bytes + words * 64 + cb);   // after the maps
    hipLaunchKernelGGL(k_pack_held, dim3(grid_for(words, kBlock)), dim3(kBlock), 0, st, held_bytes, words, qw, wcnt);
    PNR_LAUNCH_CHECK();
    if ((rc = exclusive_scan(wcnt, words, nullptr, wrank, (int64_t)((h->cell_bytes.bytes - words * 64 - cb) / 4), counters + 4, h->scan_tmp.p, h->scan_tmp.bytes, st)))
      return rc;
    hipLaunchKernelGGL(k_word_rank, dim3(grid_for(words, kBlock)), dim3(kBlock), 0, st, words, wrank, qw);
    PNR_LAUNCH_CHECK();

    hipLaunchKernelGGL(k_rank_slots, dim3(grid_for(cap_o, kBlock)), dim3(kBlock), 0, st, (int)cap_o, g, geo,
                       occ_numpnts, occ_2_coor, qw, h->q_rank_slot.as<int32_t>(), h->q_rank_cnt.as<int32_t>());
    PNR_LAUNCH_CHECK();
    if ((rc = exclusive_scan(h->q_rank_cnt.as<int32_t>(), cap_o, counters + 4, h->q_rec_off.as<int32_t>(),
                             (int64_t)(h->q_rec_off.bytes / 4), counters + 5, h->scan_tmp.p, h->scan_tmp.bytes, st)))
      return rc;
    if (!h->host_cnt) PNR_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->host_cnt), 8 * sizeof(int32_t)));
    if (!h->host_geom) PNR_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->host_geom), sizeof(QGrid)));
    if (h->geom_on_device && !h->host_bbox)
      PNR_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->host_bbox), 8 * sizeof(float)));
    if (!h->stats_ev) PNR_HIP(hipEventCreateWithFlags(&h->stats_ev, hipEventDisableTiming));
    if (h->stats_pending) PNR_HIP(hipEventSynchronize(h->stats_ev));   // the previous build's stats are written
    // (the bbox: of a device-geometry build, the one its geometry came from -- pnr_grid_bbox)
    const HostStats hs = {counters, geo, h->geom_on_device ? h->bbox.as<float>() : nullptr, h->host_cnt, h->host_geom,
                          h->host_bbox};
    hipLaunchKernelGGL(k_fill_recs, dim3(grid_for(cap_o * 16, kBlock)), dim3(kBlock), 0, st, g, counters + 4,
                       h->q_rank_slot.as<int32_t>(), h->q_rec_off.as<int32_t>(), occ_pts, h->q_recs.as<float4>(), hs);
    PNR_LAUNCH_CHECK();
  }
  PNR_HIP(hipEventRecord(h->stats_ev, st));
  h->stats_pending = true;
  h->gp = *p;
  h->gvol = gvol;
  h->n_points = n;
  for (int a = 0; a < 3; ++a) h->stats.dims[a] = p->dims[a];
  h->built = true;
  return PNR_OK;
}

extern "C" int pnr_grid_build(pnr_handle* h, const float* xyz_dev, int64_t n,
                              const pnr_grid_params* p, void* stream) {
  PNR_CHECK_ARG(h && xyz_dev && p, "grid_build: null pointer");
  PNR_HIP(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  int rc;
  if ((rc = h->geom.ensure(sizeof(QGrid)))) return rc;
  QGrid G;
  for (int a = 0; a < 3; ++a) {
    G.shift[a] = p->shift[a];
    G.vs[a] = p->vsize[a];
    G.dims[a] = p->dims[a];
  }
  G.P = p->P;
  hipLaunchKernelGGL(k_set_geom, dim3(1), dim3(64), 0, st, G, h->geom.as<QGrid>());
  PNR_LAUNCH_CHECK();
  h->geom_on_device = false;
  return grid_build_body(h, xyz_dev, n, p, st);
}

extern "C" int pnr_grid_build_dev(pnr_handle* h, const float* xyz_dev, int64_t n, const pnr_grid_spec* sp,
                                  void* stream) {
  PNR_CHECK_ARG(h && xyz_dev && sp, "grid_build_dev: null pointer");
  PNR_CHECK_ARG(n > 0 && n < (int64_t)1 << 31, "grid_build_dev: point count %lld out of range", (long long)n);
  for (int a = 0; a < 3; ++a) {
    PNR_CHECK_ARG(sp->ranges[a] < sp->ranges[3 + a], "grid_build_dev: needs ranges (min < max)");
    PNR_CHECK_ARG(sp->dims_max[a] > 0 && sp->vsize[a] > 0 && sp->vscale[a] > 0 && sp->vsize_s[a] > 0,
                  "grid_build_dev: bad spec");
  }
  PNR_HIP(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  int rc;
  const bool fresh = h->bbox_acc.p == nullptr;
  if ((rc = h->geom.ensure(sizeof(QGrid))) || (rc = h->bbox.ensure(8 * sizeof(float))) ||
      (rc = h->bbox_acc.ensure(8 * sizeof(unsigned))))
    return rc;
  if (fresh) {   // the accumulators' initial state (each build's last block restores it)
    hipLaunchKernelGGL(k_bbox_acc_init, dim3(1), dim3(64), 0, st, h->bbox_acc.as<unsigned>());
    PNR_LAUNCH_CHECK();
  }
  // bbox -> geometry on the device (get_hyperparameters)
  hipLaunchKernelGGL(k_bbox, dim3(grid_for(cdiv(n, 4), kBlock, 512)), dim3(kBlock), 0, st, xyz_dev, n,
                     h->bbox_acc.as<unsigned>());
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_geom_acc, dim3(1), dim3(64), 0, st, h->bbox_acc.as<unsigned>(), h->bbox.as<float>(), *sp,
                     h->geom.as<QGrid>());
  PNR_LAUNCH_CHECK();
  pnr_grid_params p{};
  for (int a = 0; a < 3; ++a) {
    p.shift[a] = sp->ranges[a] - sp->pad[a];   // unused by the kernels (geometry from h->geom)
    p.vsize[a] = sp->vsize_s[a];
    p.dims[a] = sp->dims_max[a];
    p.query_size[a] = sp->query_size[a];
  }
  p.max_o = sp->max_o;
  p.P = sp->P;
  p.slot0_drop = sp->slot0_drop;
  p.seed = sp->seed;
  h->geom_on_device = true;
  return grid_build_body(h, xyz_dev, n, &p, st);
}

extern "C" int pnr_grid_bbox(pnr_handle* h, float out6[6]) {
  PNR_CHECK_ARG(h && out6, "grid_bbox: null pointer");
  PNR_CHECK_ARG(h->built && h->geom_on_device && h->host_bbox, "grid_bbox: no device-geometry build");
  PNR_HIP(hipEventSynchronize(h->stats_ev));
  for (int a = 0; a < 6; ++a) out6[a] = h->host_bbox[a];
  return PNR_OK;
}

extern "C" int pnr_grid_geometry(pnr_handle* h, float shift[3], float vsize[3], int32_t dims[3]) {
  PNR_CHECK_ARG(h && h->built && h->host_geom, "grid_geometry: grid not built");
  PNR_CHECK_ARG(shift && vsize && dims, "grid_geometry: null pointer");
  PNR_HIP(hipEventSynchronize(h->stats_ev));
  for (int a = 0; a < 3; ++a) {
    shift[a] = h->host_geom->shift[a];
    vsize[a] = h->host_geom->vs[a];
    dims[a] = h->host_geom->dims[a];
  }
  return PNR_OK;
}

__global__ void k_export_ids(int n_slots, int P, const int32_t* __restrict__ occ_numpnts,
                             const float4* __restrict__ occ_pts, int32_t* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)n_slots * P;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = e / P;
    const int g = (int)(e - s * P);
    out[e] = g < occ_numpnts[s] ? __float_as_int(occ_pts[e].w) : -1;
  }
}

extern "C" int pnr_grid_export(pnr_handle* h, int32_t* coor_2_occ, uint32_t* occ_bits,
                               int32_t* occ_numpnts, int32_t* occ_2_pnts, void* stream) {
  PNR_CHECK_ARG(h && h->built, "grid_export: grid not built");
  hipStream_t st = as_stream(stream);
  // the tables are laid out by the exact dims (pnr_grid_geometry: waits for the build)
  float sh[3], vs[3];
  int32_t dm[3];
  int rc;
  if ((rc = pnr_grid_geometry(h, sh, vs, dm))) return rc;
  const int64_t gvol = (int64_t)dm[0] * dm[1] * dm[2];
  const int64_t words = cdiv(gvol, 32);
  const int64_t cap_o = h->gp.max_o;
  if (coor_2_occ)
    PNR_HIP(hipMemcpyAsync(coor_2_occ, h->coor_2_occ.p, gvol * 4, hipMemcpyDeviceToDevice, st));
  if (occ_bits) PNR_HIP(hipMemcpyAsync(occ_bits, h->occ_bits.p, words * 4, hipMemcpyDeviceToDevice, st));
  if (occ_numpnts)
    PNR_HIP(hipMemcpyAsync(occ_numpnts, h->occ_numpnts.p, cap_o * 4, hipMemcpyDeviceToDevice, st));
  if (occ_2_pnts) {
    hipLaunchKernelGGL(k_export_ids, dim3(grid_for(cap_o * h->gp.P, kBlock)), dim3(kBlock), 0, st,
                       (int)cap_o, h->gp.P, h->occ_numpnts.as<int32_t>(), h->occ_pts.as<float4>(),
                       occ_2_pnts);
    PNR_LAUNCH_CHECK();
  }
  return PNR_OK;
}

extern "C" int pnr_grid_stats_get(pnr_handle* h, pnr_grid_stats* out) {
  PNR_CHECK_ARG(h && out, "grid_stats: null pointer");
  PNR_CHECK_ARG(h->built, "grid_stats: grid not built");
  if (h->stats_pending) {
    PNR_HIP(hipEventSynchronize(h->stats_ev));
    const int32_t* cnt = h->host_cnt;
    h->stats.n_voxels = cnt[0];
    h->stats.n_voxels_kept = cnt[0] < h->gp.max_o ? cnt[0] : h->gp.max_o;
    h->stats.n_points_in_grid = cnt[1];
    h->stats.n_points_dropped = cnt[2];
    h->stats.max_points_per_voxel = cnt[3];
    for (int a = 0; a < 3; ++a) h->stats.dims[a] = h->host_geom->dims[a];
    h->stats_pending = false;
  }
  *out = h->stats;
  return PNR_OK;
}
