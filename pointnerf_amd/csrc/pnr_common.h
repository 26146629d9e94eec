// Shared host/device helpers for libpnr.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/pnr.h"

namespace pnr {

// ------------------------------------------------------------ error plumbing
void set_error(const char* fmt, ...);

#define PNR_CHECK_ARG(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      ::pnr::set_error(__VA_ARGS__);      \
      return PNR_EINVAL;                  \
    }                                     \
  } while (0)

#define PNR_HIP(call)                                                         \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) {                                                   \
      ::pnr::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,           \
                       hipGetErrorString(e_));                                \
      return PNR_EHIP;                                                        \
    }                                                                         \
  } while (0)

#define PNR_LAUNCH_CHECK() PNR_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Persistent-grid launch size for grid-stride kernels: enough workgroups to
// fill 256 CUs several times over, never more than the work needs.
inline unsigned grid_for(int64_t items, int block, int max_blocks = 256 * 8) {
  int64_t g = cdiv(items, block);
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (unsigned)g;
}

// Device-wide exclusive scan (scan.hip).
int64_t scan_blocks(int64_t n);
size_t scan_scratch_bytes(int64_t n);
// out_cap: int32 entries the caller allocated at out; the scan writes out[0 .. n]
// (n + 1 entries: the grand total lands at out[n_eff]), checked here.
int exclusive_scan(const int32_t* in, int64_t n, const int32_t* n_dev, int32_t* out, int64_t out_cap,
                   int32_t* total_dev, void* scratch, size_t scratch_bytes, hipStream_t st,
                   int as_flag = 0,   // as_flag: scan (in[i] != 0) instead of in[i]
                   const int32_t* run_if = nullptr,   // device flag: 0 = leave out untouched
                   int32_t* list = nullptr);          // optional stream compaction: list[out[i]] = i for in[i] != 0

// --------------------------------------------------------- device helpers
// floor((p - shift) / vs) exactly as the reference kernels compute it in fp32
// (qpiw.py:265-267, 406-408, 471-473): one rounded subtraction, one correctly
// rounded division, floor, truncating cast.
__device__ __forceinline__ int vox_coord(float p, float shift, float vs) {
  return (int)floorf(__fdiv_rn(__fsub_rn(p, shift), vs));
}

// vox_coord's value without the IEEE division on almost every call: t = x * inv
// (inv = RN(1 / vs)) is within |e| 2^-22 of e = x / vs and RN(e) within |e| 2^-24,
// so when t is farther than |t| 2^-20 from every integer, floor(t) is
// floor(RN(e)); otherwise (an integer within reach, x = 0) the exact division.
__device__ __forceinline__ int vox_coord_fast(float p, float shift, float vs, float inv) {
  const float x = __fsub_rn(p, shift);
  const float t = __fmul_rn(x, inv);
  const float f = floorf(t);
  const float m = __fmaf_rn(fabsf(t), 0x1p-20f, 0x1p-100f);
  if (__fsub_rn(t, f) > m && __fsub_rn(__fadd_rn(f, 1.0f), t) > m) return (int)f;
  return (int)floorf(__fdiv_rn(x, vs));
}

// raypos = campos + raydir * t  (diff_ray_marching.py:387: mul, then add).
__device__ __forceinline__ float ray_at(float c, float d, float t) {
  return __fadd_rn(c, __fmul_rn(d, t));
}

// Camera-space coordinates, xyz_c_j = sum_i (p_i - c_i) * R[i][j] with the
// reference's summation order (qpiw.py:104-105, neural_points.py:687-693).
__device__ __forceinline__ void world_to_cam(const float p[3], const float c[3],
                                             const float R[9], float out[3]) {
  float s0 = __fsub_rn(p[0], c[0]);
  float s1 = __fsub_rn(p[1], c[1]);
  float s2 = __fsub_rn(p[2], c[2]);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float a = __fmul_rn(s0, R[0 * 3 + j]);
    float b = __fmul_rn(s1, R[1 * 3 + j]);
    float d = __fmul_rn(s2, R[2 * 3 + j]);
    out[j] = __fadd_rn(__fadd_rn(a, b), d);
  }
}

// (x/z, y/z, z)
__device__ __forceinline__ void world_to_pers(const float p[3], const float c[3],
                                              const float R[9], float out[3]) {
  float xc[3];
  world_to_cam(p, c, R, xc);
  out[0] = __fdiv_rn(xc[0], xc[2]);
  out[1] = __fdiv_rn(xc[1], xc[2]);
  out[2] = xc[2];
}

// Seeded reservoir of the grid build (max_o / P overflow, qpiw.py:289-298,
// 377-384): a uniform random subset chosen by the smallest keys
// hash32(seed, id) << 32 | id (oracle/query_ref.c states the same keys).
constexpr uint64_t kPtSalt = 0x632BE59BD9B4E019ull;
__host__ __device__ inline uint32_t res_hash32(uint64_t seed, uint32_t id) {
  uint64_t z = seed ^ ((uint64_t)id * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
__host__ __device__ inline uint64_t res_vkey(uint64_t seed, uint32_t id) {
  return ((uint64_t)res_hash32(seed, id) << 32) | id;
}
__host__ __device__ inline uint64_t res_pkey(uint64_t seed, uint32_t id) {
  return ((uint64_t)res_hash32(seed + kPtSalt, id) << 32) | id;
}
__host__ __device__ inline uint32_t res_pkey_hash(uint64_t seed, uint32_t id) {   // res_pkey's high half
  return res_hash32(seed + kPtSalt, id);
}

// Sum over the 64 lanes of a wave.
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

}  // namespace pnr

// A device allocation that only grows.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t want) {
    if (p && bytes >= want) return PNR_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, want ? want : 16) != hipSuccess) {
      ::pnr::set_error("hipMalloc of %zu bytes failed", want);
      return PNR_ENOMEM;
    }
    bytes = want;
    return PNR_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

// Grid geometry as the build and query kernels read it from device memory
// (pnr_handle.geom): written by the host (pnr_grid_build) or derived from the
// points' bbox on the device (pnr_grid_build_dev, no host sync).
struct QGrid {
  float shift[3], vs[3];
  int dims[3];
  int P;
};

// Persistent grid tables owned by a handle (built by pnr_grid_build).
struct pnr_handle {
  int device = 0;
  pnr_grid_params gp{};
  int64_t gvol = 0;       // dims[0]*dims[1]*dims[2]
  DevBuf coor_2_occ;      // int32 [gvol]   cell -> slot, -1 = empty
  DevBuf occ_bits;        // uint32 [gvol/32] dilated occupancy bitmap
  DevBuf cell_end;        // int32 [gvol]   one past the last sorted position of the cell's run (occupied cells only)
  DevBuf cell_bytes;      // uint8 [32*words] x 2, the coarse column map, int32 [words+1]: occupancy bytes
                          //   before packing, held bytes, the KNN's coarse map (uint32 [ceil(dz/8)][dx]
                          //   [ceil(dy/32)]: bit y = column (x, y) holds a kept point in z-block bz), word ranks
  size_t coarse_off = 0;  // byte offset of the coarse map in cell_bytes
  DevBuf occ_numpnts;     // int32 [max_o]  points that fell in the voxel
  DevBuf occ_pts;         // float4 [max_o*P] {x, y, z, bitcast(point id)}
  DevBuf occ_2_coor;      // int32 [max_o*3]
  DevBuf sort_k[2];       // uint32/uint64 [N] cell keys (ping-pong of the LSD radix sort)
  DevBuf sort_v[2];       // int32 [N]      point ids riding with the keys
  DevBuf sort_hist;       // int32 [256*tiles + 1] per-tile digit counts, then their exclusive scan
  DevBuf sort_offs;       // int32 [256*tiles + 1]
  DevBuf cell_start;      // int32 [gvol]   first sorted position of the cell's run (occupied cells only)
  DevBuf pt_flag;         // int32 [N]
  DevBuf pt_slot;         // int32 [N+1]
  DevBuf counters;        // int32 [8]
  DevBuf sel;             // voxel reservoir: radix-select state + 8 x 256-bin histograms
  DevBuf scan_tmp;
  // Query index (what k_knn reads; the slot tables above stay the reference's
  // view for export / parity): the voxels that hold points, ranked in x-major
  // cell order, so a sample's 3x3x3 neighbourhood is found from a bitmap that
  // stays in L2 and its records sit near each other in HBM.
  DevBuf q_words;         // uint2 [gvol/32] {bits: cell holds >= 1 kept point, rank of the word's first cell}
  DevBuf q_wcnt;          // int32 [gvol/32] scratch: popcount per word
  DevBuf q_rank_slot;     // int32 [max_o]   slot of rank r (scratch)
  DevBuf q_rank_cnt;      // int32 [max_o]   min(P, points) of rank r (scratch)
  DevBuf q_rec_off;       // int32 [max_o+1] first record of rank r (exclusive scan of q_rank_cnt)
  DevBuf q_recs;          // float4 [N]      {x, y, z, bitcast(id)} in rank order, per voxel ascending id
  DevBuf geom;            // QGrid of the built grid (device)
  DevBuf bbox;            // float [8] point bbox of the last pnr_grid_build_dev
  DevBuf bbox_acc;        // uint32 [8] k_bbox_geom's order-key accumulators + block ticket (kept reset)
  QGrid* host_geom = nullptr;   // pinned copy of geom behind stats_ev
  float* host_bbox = nullptr;   // pinned copy of bbox (device builds) behind stats_ev
  bool geom_on_device = false;  // gp.shift / dims are bounds, the exact geometry is geom (device)
  int64_t n_points = 0;
  pnr_grid_stats stats{};
  bool built = false;
  // build counters read back without blocking the build: pinned copy + event,
  // waited on by pnr_grid_stats_get only
  int32_t* host_cnt = nullptr;
  hipEvent_t stats_ev = nullptr;
  bool stats_pending = false;
  void release_all() {
    if (host_cnt) (void)hipHostFree(host_cnt);
    if (host_geom) (void)hipHostFree(host_geom);
    host_geom = nullptr;
    if (host_bbox) (void)hipHostFree(host_bbox);
    host_bbox = nullptr;
    if (stats_ev) (void)hipEventDestroy(stats_ev);
    host_cnt = nullptr;
    stats_ev = nullptr;
    stats_pending = false;
    DevBuf* all[] = {&coor_2_occ, &occ_bits, &cell_end, &cell_bytes, &occ_numpnts, &occ_pts, &occ_2_coor,
                     &sort_k[0], &sort_k[1], &sort_v[0], &sort_v[1], &sort_hist, &sort_offs,
                     &cell_start, &pt_flag, &pt_slot, &counters, &sel, &scan_tmp, &q_words, &q_wcnt, &q_rank_slot, &q_rank_cnt,
                     &q_rec_off, &q_recs, &geom, &bbox, &bbox_acc};
    for (DevBuf* b : all) b->release();
  }
};
