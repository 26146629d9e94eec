// Point-cloud initialisation: voxel down-sampling to the point closest to each
// voxel's centroid.  Replaces construct_vox_points_closest
// (models/mvs/mvs_utils.py:537-561; torch.unique + torch_scatter's scatter_mean /
// scatter_min), which turns the MVS / lidar point cloud into the initial
// neural points (train_ddp.py:135, train_waymo_v1.py:145, 615).
//
//   space:  edge = max(max xyz - min xyz) * 1.05, mid = (max + min) / 2,
//           space_min = mid - edge / 2, vox_sz = edge / vox_res      (:540-544)
//   cell:   floor((xyz - space_min) / vox_sz) as int32               (:551-552)
//   unique: cells sorted lexicographically (torch.unique(dim=0)), inverse index
//   mean:   per-voxel sum in ascending point order / count           (scatter_mean)
//   pick:   per voxel the point with the smallest |xyz - centroid|,  (scatter_min)
//           ties to the smallest point index
//
// One 64-bit key per point (x, y, z biased by 2^20, 21 bits each: numeric order
// = lexicographic order), a stable rocPRIM radix sort of (key, point index)
// pairs, flags + scan for the voxel ids, then one thread per voxel walks its
// sorted run twice (sum, then arg-min): deterministic, no float atomics.
// Built with -ffp-contract=off (Makefile), like query.hip: the residuals must
// round like the reference's separate fp32 mul / add.
#include <rocprim/device/device_radix_sort.hpp>

#include "pnr_common.h"

namespace pnr {
namespace {

constexpr int kVBlock = 256;
constexpr int kBias = 1 << 20;

struct VoxSpace {
  float smin[3];
  float vsz;
  float edge;
};

// bbox (pnr_points_bbox's {min, max}) -> space_min / voxel size, with torch's
// fp32 op order (mvs_utils.py:540-544, 550)
__global__ void k_vox_space(const float* __restrict__ box, int vox_res, VoxSpace* sp) {
  if (threadIdx.x != 0) return;
  float edge = 0.f;
#pragma unroll
  for (int a = 0; a < 3; ++a) edge = fmaxf(edge, __fsub_rn(box[3 + a], box[a]));
  edge = __fmul_rn(edge, 1.05f);
  VoxSpace s;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float mid = __fdiv_rn(__fadd_rn(box[3 + a], box[a]), 2.f);
    s.smin[a] = __fsub_rn(mid, __fdiv_rn(edge, 2.f));
  }
  s.edge = edge;
  s.vsz = __fdiv_rn(edge, (float)vox_res);
  *sp = s;
}

__device__ __forceinline__ uint64_t pack_key(int x, int y, int z) {
  return ((uint64_t)(uint32_t)(x + kBias) << 42) | ((uint64_t)(uint32_t)(y + kBias) << 21) | (uint64_t)(uint32_t)(z + kBias);
}
__device__ __forceinline__ int key_coord(uint64_t k, int a) {
  return (int)((k >> (42 - 21 * a)) & ((1u << 21) - 1)) - kBias;
}

__global__ void __launch_bounds__(kVBlock) k_vox_keys(const float* __restrict__ xyz, int64_t n, const VoxSpace* sp,
                                                     uint64_t* __restrict__ keys, int32_t* __restrict__ idx,
                                                     int32_t* bad) {
  const VoxSpace s = *sp;
  int out_of_range = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int c[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float q = __fdiv_rn(__fsub_rn(xyz[i * 3 + a], s.smin[a]), s.vsz);
      const float f = floorf(q);
      out_of_range |= !(f > -(float)kBias && f < (float)kBias);
      c[a] = out_of_range ? 0 : (int)f;
    }
    keys[i] = pack_key(c[0], c[1], c[2]);
    idx[i] = (int32_t)i;
  }
  if (out_of_range) atomicOr(bad, 1);
}

__global__ void __launch_bounds__(kVBlock) k_vox_flags(const uint64_t* __restrict__ keys, int64_t n,
                                                      int32_t* __restrict__ flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// voxel id of every sorted position, the first position of every voxel, the
// inverse index (point -> voxel) when asked for
__global__ void __launch_bounds__(kVBlock) k_vox_runs(int64_t n, const int32_t* __restrict__ flag,
                                                     const int32_t* __restrict__ off, const int32_t* __restrict__ idx,
                                                     const int32_t* __restrict__ n_vox, int32_t* __restrict__ start,
                                                     int32_t* __restrict__ inv) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int v = off[i] + flag[i] - 1;
    if (flag[i]) start[v] = (int32_t)i;
    if (inv) inv[idx[i]] = v;
    if (i == 0) start[*n_vox] = (int32_t)n;
  }
}

// one thread per voxel: centroid = (sequential sum in ascending point order) / count,
// then the arg-min of |xyz - centroid| (strict <: the smallest index wins a tie)
__global__ void __launch_bounds__(kVBlock) k_vox_reduce(const float* __restrict__ xyz, const uint64_t* __restrict__ keys,
                                                       const int32_t* __restrict__ idx,
                                                       const int32_t* __restrict__ start,
                                                       const int32_t* __restrict__ n_vox, float* __restrict__ centroid,
                                                       int32_t* __restrict__ grid_idx, int64_t* __restrict__ min_idx) {
  const int m = *n_vox;
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < m; v += gridDim.x * blockDim.x) {
    const int b = start[v], e = start[v + 1];
    float s[3] = {0.f, 0.f, 0.f};
    for (int i = b; i < e; ++i) {
      const int64_t p = idx[i];
#pragma unroll
      for (int a = 0; a < 3; ++a) s[a] = __fadd_rn(s[a], xyz[p * 3 + a]);
    }
    const float cnt = (float)(e - b);
    float c[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      c[a] = __fdiv_rn(s[a], cnt);
      centroid[(int64_t)v * 3 + a] = c[a];
      grid_idx[(int64_t)v * 3 + a] = key_coord(keys[b], a);
    }
    float best = INFINITY;
    int64_t arg = idx[b];
    for (int i = b; i < e; ++i) {
      const int64_t p = idx[i];
      const float dx = __fsub_rn(xyz[p * 3], c[0]), dy = __fsub_rn(xyz[p * 3 + 1], c[1]),
                  dz = __fsub_rn(xyz[p * 3 + 2], c[2]);
      // correctly rounded fp32 sqrt (the fp32 square root is exactly representable
      // in double and the double root rounds to the fp32 one)
      const float r2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
      const float r = (float)__dsqrt_rn((double)r2);
      if (r < best) {
        best = r;
        arg = p;
      }
    }
    min_idx[v] = arg;
  }
}

struct VoxScratch {
  uint64_t* keys_in;
  uint64_t* keys_out;
  int32_t* idx_in;
  int32_t* idx_out;
  int32_t* flag;
  int32_t* off;
  int64_t off_cap;   // entries at off (m + 1: the scan's total lands at off[n])
  int32_t* start;
  float* box;
  VoxSpace* space;
  int32_t* bad;
  void* scan;
  size_t scan_bytes;
  void* sort;
  size_t sort_bytes;
};

size_t align16(size_t b) { return (b + 15) & ~(size_t)15; }

size_t sort_bytes(int64_t n) {
  size_t b = 0;
  (void)rocprim::radix_sort_pairs(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                  (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n, 0, 63);
  return b;
}

size_t carve(void* base, int64_t n, VoxScratch* s) {
  const int64_t m = n > 0 ? n : 1;
  size_t o = 0;
  char* p = static_cast<char*>(base);
  auto take = [&](size_t bytes) -> char* {
    char* r = p ? p + o : nullptr;
    o += align16(bytes);
    return r;
  };
  VoxScratch t;
  t.keys_in = reinterpret_cast<uint64_t*>(take(m * 8));
  t.keys_out = reinterpret_cast<uint64_t*>(take(m * 8));
  t.idx_in = reinterpret_cast<int32_t*>(take(m * 4));
  t.idx_out = reinterpret_cast<int32_t*>(take(m * 4));
  t.flag = reinterpret_cast<int32_t*>(take(m * 4));
  t.off = reinterpret_cast<int32_t*>(take((m + 1) * 4));
  t.off_cap = m + 1;
  t.start = reinterpret_cast<int32_t*>(take((m + 1) * 4));
  t.box = reinterpret_cast<float*>(take(8 * 4));
  t.space = reinterpret_cast<VoxSpace*>(take(sizeof(VoxSpace)));
  t.bad = reinterpret_cast<int32_t*>(take(16));
  t.scan_bytes = scan_scratch_bytes(m + 1);
  t.scan = take(t.scan_bytes);
  t.sort_bytes = sort_bytes(m);
  t.sort = take(t.sort_bytes);
  if (s) *s = t;
  return o;
}

}  // namespace
}  // namespace pnr

using namespace pnr;

extern "C" int pnr_vox_closest_scratch_bytes(int64_t n, size_t* out) {
  PNR_CHECK_ARG(out && n >= 0, "vox_closest_scratch_bytes: bad args");
  *out = carve(nullptr, n, nullptr);
  return PNR_OK;
}

extern "C" int pnr_vox_closest(const float* xyz, int64_t n, int32_t vox_res, float* centroid, int32_t* grid_idx,
                               int64_t* min_idx, int32_t* inv_idx, int32_t* counts, void* scratch,
                               size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(xyz && centroid && grid_idx && min_idx && counts && scratch, "vox_closest: null pointer");
  PNR_CHECK_ARG(n > 0 && n < ((int64_t)1 << 31), "vox_closest: point count %lld out of range", (long long)n);
  PNR_CHECK_ARG(vox_res > 0 && vox_res < (1 << 20), "vox_closest: vox_res %d out of range", vox_res);
  PNR_CHECK_ARG(((uintptr_t)scratch & 15) == 0, "vox_closest: 16-B aligned scratch required");
  VoxScratch s;
  const size_t need = carve(scratch, n, &s);
  PNR_CHECK_ARG(scratch_bytes >= need, "vox_closest: scratch too small (%zu < %zu)", scratch_bytes, need);
  hipStream_t st = as_stream(stream);
  int rc;
  if ((rc = pnr_points_bbox(xyz, n, s.box, stream))) return rc;
  hipLaunchKernelGGL(k_vox_space, dim3(1), dim3(64), 0, st, s.box, vox_res, s.space);
  PNR_LAUNCH_CHECK();
  PNR_HIP(hipMemsetAsync(counts, 0, 2 * sizeof(int32_t), st));
  const unsigned g = grid_for(n, kVBlock);
  hipLaunchKernelGGL(k_vox_keys, dim3(g), dim3(kVBlock), 0, st, xyz, n, s.space, s.keys_in, s.idx_in, counts + 1);
  PNR_LAUNCH_CHECK();
  size_t sb = s.sort_bytes;
  PNR_HIP(rocprim::radix_sort_pairs(s.sort, sb, s.keys_in, s.keys_out, s.idx_in, s.idx_out, (size_t)n, 0, 63, st));
  hipLaunchKernelGGL(k_vox_flags, dim3(g), dim3(kVBlock), 0, st, s.keys_out, n, s.flag);
  PNR_LAUNCH_CHECK();
  if ((rc = exclusive_scan(s.flag, n, nullptr, s.off, s.off_cap, counts, s.scan, s.scan_bytes, st))) return rc;
  hipLaunchKernelGGL(k_vox_runs, dim3(g), dim3(kVBlock), 0, st, n, s.flag, s.off, s.idx_out, counts, s.start,
                     inv_idx);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_vox_reduce, dim3(g), dim3(kVBlock), 0, st, xyz, s.keys_out, s.idx_out, s.start, counts,
                     centroid, grid_idx, min_idx);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
