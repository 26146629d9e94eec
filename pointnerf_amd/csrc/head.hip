// Upstream RGB colour head (C_out = 3) on the decoded 128-channel features.
//
// The fork cut the colour head of point_aggregators.py (the final
// `nn.Linear(in, 3)` at :343 and `raw2out_color` at :637-638, :269-273); the
// upstream model keeps both, and its radiance_render returns feature[..., 1:4]
// (diff_render_func.py:48-50).  This kernel restores them behind the fused
// aggregation:
//   out[v] = [feat[v,0],  raw2out_color(W . feat[v,1:129] + b)]
//   raw2out_color(x) = sigmoid(x) * (1 + 2e-3) - 1e-3   (act_super > 0; else sigmoid)
// and its backward (d feat[v,1:], d W, d b).  HBM-bound: 129 x 4 B read and
// 4 x 4 B written per valid sample.  One 32-lane half-wave per sample, each
// lane owning four channels, the three dot products reduced with xor shuffles.
#include "pnr_common.h"

namespace pnr {

constexpr int kHBlock = 256;

__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float raw2out(float x, int act_super) {
  const float s = 1.f / (1.f + expf(-x));
  return act_super > 0 ? s * (1.f + 2e-3f) - 1e-3f : s;
}

__global__ void __launch_bounds__(kHBlock) k_rgb_head(const float* __restrict__ feat, int64_t ld,
                                                      const int32_t* __restrict__ n_dev, int64_t n_max,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      int act_super, float* __restrict__ out) {
  const int64_t n = n_dev ? min((int64_t)*n_dev, n_max) : n_max;
  const int lane = threadIdx.x & 31;
  float wr[3][4];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) wr[j][c] = w[j * 128 + 4 * lane + c];
  const float b0 = b[0], b1 = b[1], b2 = b[2];
  const int64_t halves = (int64_t)gridDim.x * (blockDim.x / 32);
  for (int64_t v = blockIdx.x * (int64_t)(blockDim.x / 32) + (threadIdx.x >> 5); v < n; v += halves) {
    const float* f = feat + v * ld;
    float x[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = f[1 + 4 * lane + c];
    float d[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) s = fmaf(wr[j][c], x[c], s);
      d[j] = half_sum(s);
    }
    if (lane < 4) {
      float o = f[0];
      if (lane == 1) o = raw2out(d[0] + b0, act_super);
      if (lane == 2) o = raw2out(d[1] + b1, act_super);
      if (lane == 3) o = raw2out(d[2] + b2, act_super);
      out[v * 4 + lane] = o;
    }
  }
}

// d_feat[v, 1 + c] = sum_j g_j W[j, c] with g_j = d_out[v, 1 + j] * d raw2out / dx;
// d_feat[v, 0] = d_out[v, 0].  d_wb[j*129 + c] (c < 128: d W, c = 128: d b):
// each of the kHeadBwdBlocks blocks writes its partial sums to partials[block]
// and k_rgb_head_wsum adds them in block order (bitwise repeatable, no atomics).
__global__ void __launch_bounds__(kHBlock) k_rgb_head_bwd(const float* __restrict__ d_out,
                                                          const float* __restrict__ feat, int64_t ld,
                                                          const int32_t* __restrict__ n_dev, int64_t n_max,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ b, int act_super,
                                                          float* __restrict__ d_feat, float* __restrict__ partials) {
  __shared__ float acc[kHBlock / 32][3][129];
  const int64_t n = n_dev ? min((int64_t)*n_dev, n_max) : n_max;
  const int lane = threadIdx.x & 31, hw = threadIdx.x >> 5;
  for (int i = threadIdx.x; i < (kHBlock / 32) * 3 * 129; i += blockDim.x) (&acc[0][0][0])[i] = 0.f;
  __syncthreads();
  float wr[3][4];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) wr[j][c] = w[j * 128 + 4 * lane + c];
  float aw[3][4] = {}, ab[3] = {};
  const int64_t halves = (int64_t)gridDim.x * (blockDim.x / 32);
  for (int64_t v = blockIdx.x * (int64_t)(blockDim.x / 32) + hw; v < n; v += halves) {
    const float* f = feat + v * ld;
    float* df = d_feat + v * ld;
    float x[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = f[1 + 4 * lane + c];
    float g[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {   // recompute the logit, then d raw2out / dx
      float z = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) z = fmaf(wr[j][c], x[c], z);
      z = half_sum(z) + b[j];
      const float s = 1.f / (1.f + expf(-z));
      const float sc = act_super > 0 ? 1.f + 2e-3f : 1.f;
      g[j] = d_out[v * 4 + 1 + j] * sc * s * (1.f - s);
      ab[j] += g[j];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        s = fmaf(g[j], wr[j][c], s);
        aw[j][c] = fmaf(g[j], x[c], aw[j][c]);
      }
      df[1 + 4 * lane + c] = s;
    }
    if (lane == 0) df[0] = d_out[v * 4];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[hw][j][4 * lane + c] = aw[j][c];
    if (lane == 0) acc[hw][j][128] = ab[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * 129; i += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int h = 0; h < kHBlock / 32; ++h) s += (&acc[h][0][0])[i];
    partials[(int64_t)blockIdx.x * 3 * 129 + i] = s;
  }
}

// d_wb[i] = sum over blocks of partials[block][i], in block order.
__global__ void __launch_bounds__(kHBlock) k_rgb_head_wsum(const float* __restrict__ partials, int nblk,
                                                           float* __restrict__ d_wb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * 129) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += partials[(int64_t)b * 3 * 129 + i];
  d_wb[i] = s;
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_rgb_head_fwd(const float* feat, int64_t ld, const int32_t* n_dev, int64_t n_max,
                                const float* w, const float* b, int32_t act_super, float* out, void* stream) {
  PNR_CHECK_ARG(feat && w && b && out && n_max >= 0 && ld >= 129, "rgb_head_fwd: bad arguments");
  if (n_max == 0) return PNR_OK;
  hipLaunchKernelGGL(k_rgb_head, dim3(grid_for(n_max, kHBlock / 32, 256 * 8)), dim3(kHBlock), 0,
                     as_stream(stream), feat, ld, n_dev, n_max, w, b, act_super, out);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_rgb_head_bwd(const float* d_out, const float* feat, int64_t ld, const int32_t* n_dev,
                                int64_t n_max, const float* w, const float* b, int32_t act_super, float* d_feat,
                                float* d_wb, float* partials, void* stream) {
  PNR_CHECK_ARG(d_out && feat && w && b && d_feat && d_wb && partials && n_max >= 0 && ld >= 129,
                "rgb_head_bwd: bad arguments");
  hipStream_t st = as_stream(stream);
  if (n_max == 0) return hipMemsetAsync(d_wb, 0, 3 * 129 * sizeof(float), st) == hipSuccess ? PNR_OK : PNR_EHIP;
  hipLaunchKernelGGL(k_rgb_head_bwd, dim3(PNR_HEAD_BWD_BLOCKS), dim3(kHBlock), 0, st, d_out, feat, ld, n_dev, n_max,
                     w, b, act_super, d_feat, partials);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_rgb_head_wsum, dim3(cdiv(3 * 129, kHBlock)), dim3(kHBlock), 0, st, partials,
                     PNR_HEAD_BWD_BLOCKS, d_wb);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
