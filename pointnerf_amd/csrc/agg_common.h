// Device helpers shared by the fp32 (aggregate.hip) and bf16 (aggregate_bf16.hip)
// aggregation kernels.
#pragma once
#include "pnr_common.h"

namespace pnr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kAggBlock = 256;     // 4 waves, each independent
constexpr int kKN = 8;
constexpr int kHid = 256;
constexpr int kEmb = 32;
constexpr int kC = 128;
constexpr int kCin = 280;          // 256 + 24 view PE

__device__ __forceinline__ float lrelu(float x, float s) { return x > 0.f ? x : x * s; }

__device__ __forceinline__ float softplus(float x) {  // torch.nn.Softplus(beta=1, threshold=20)
  return x > 20.f ? x : log1pf(expf(x));
}

// Row of the accumulator register `r` for lane half `h` (32x32 C/D layout).
__device__ __forceinline__ constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float xor8_sum(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  return v;
}

__device__ __forceinline__ void mat3(const float* R, const float v[3], float o[3]) {
  // (v @ R^T)_j = sum_i v_i R[j][i]   (point_aggregators.py:492, 506, 526, 566)
#pragma unroll
  for (int j = 0; j < 3; ++j) o[j] = v[0] * R[j * 3 + 0] + v[1] * R[j * 3 + 1] + v[2] * R[j * 3 + 2];
}

__device__ __forceinline__ int64_t sample_row(const pnr_samples& s, int64_t v) {
  return s.samp_list ? (int64_t)s.samp_list[v] : v;
}

__device__ __forceinline__ int64_t dir_row(const pnr_samples& s, int64_t row) {
  return (s.dir_map ? (int64_t)s.dir_map[row] : row) / s.dir_div;
}

__device__ __forceinline__ int64_t eff_n(const pnr_samples& s) {
  int64_t n = s.n_max;
  if (s.n_dev) {
    int64_t nd = *s.n_dev;
    n = nd < n ? nd : n;
  }
  return n;
}

}  // namespace pnr
