// Weight fragment packing on the device (aggregator.frag_pack / frag_pack_x3):
// one launch per matrix instead of a dozen small torch ops, so a training step
// (weights change every step, every pack is rebuilt) is not launch-bound.
//   kind 0 (fp32, v_mfma_f32_32x32x2_f32):  F[t][T][lane] = W'[32T + (lane & 31)][2t + (lane >> 5)]
//   kind 1 (fp32x3, v_mfma_f32_32x32x16_bf16): F[t][T][plane][h][r][j] = plane of W'[32T + r][16t + 8h + j]
//     (planes: exact 3-way bf16 split, round-to-nearest-even, = aggregator.split3_bf16)
//   pnr_pack_weights_h2 (fp32h2, v_mfma_f32_32x32x16_f16): F[t][T][plane][h][r][j] = plane of
//     (2^-s W')[32T + r][16t + 8h + j], planes (Wh, Wl) of splith (= aggregator.frag_pack_h2
//     with a given shift s); the flag is raised when some |2^-s W'| >= 16 or is not finite
// W' = [W | bias | 0] (bias = input column kin when given), W[o][k] at
// W + o * ld_row + k * ld_col (a transposed view packs without a copy).
#include "agg_common.h"

namespace pnr {

__device__ __forceinline__ float wprime(const float* W, int64_t lr, int64_t lc, int kin, const float* bias, int o,
                                        int k) {
  if (k < kin) return W[o * lr + k * lc];
  return (k == kin && bias) ? bias[o] : 0.f;
}

// one element of a kind-0 pack
__device__ __forceinline__ void pack_item_fp32(const float* W, int64_t lr, int64_t lc, int NT, int kin,
                                               const float* bias, int64_t i, float* out) {
  const int lane = (int)(i & 63);
  const int64_t tT = i >> 6;
  const int T = (int)(tT % NT), t = (int)(tT / NT);
  out[i] = wprime(W, lr, lc, kin, bias, 32 * T + (lane & 31), 2 * t + (lane >> 5));
}

// item (t, T, h, r) of a kind-1 pack: 8 inputs -> one uint4 per plane
__device__ __forceinline__ void pack_item_x3(const float* W, int64_t lr, int64_t lc, int NT, int kin,
                                             const float* bias, int64_t i, uint4* out) {
  const int r = (int)(i & 31), h = (int)((i >> 5) & 1);
  const int64_t tT = i >> 6;
  const int T = (int)(tT % NT), t = (int)(tT / NT);
  const int o = 32 * T + r, k0 = 16 * t + 8 * h;
  unsigned w[3][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    split2(wprime(W, lr, lc, kin, bias, o, k0 + 2 * q), wprime(W, lr, lc, kin, bias, o, k0 + 2 * q + 1), w[0][q],
           w[1][q], w[2][q]);
#pragma unroll
  for (int pl = 0; pl < 3; ++pl)
    out[((tT * 3 + pl) * 2 + h) * 32 + r] = make_uint4(w[pl][0], w[pl][1], w[pl][2], w[pl][3]);
}

// item (t, T, h, r) of an h2 pack scaled by sc; true when a value is out of range
__device__ __forceinline__ bool pack_item_h2(const float* W, int64_t lr, int64_t lc, int NT, int kin,
                                             const float* bias, int64_t i, float sc, uint4* out) {
  const int r = (int)(i & 31), h = (int)((i >> 5) & 1);
  const int64_t tT = i >> 6;
  const int T = (int)(tT % NT), t = (int)(tT / NT);
  const int o = 32 * T + r, k0 = 16 * t + 8 * h;
  bool bad = false;
  unsigned w[2][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = wprime(W, lr, lc, kin, bias, o, k0 + 2 * q) * sc;
    const float b = wprime(W, lr, lc, kin, bias, o, k0 + 2 * q + 1) * sc;
    bad |= !(fabsf(a) < 16.f) || !(fabsf(b) < 16.f);
    splith(a, b, w[0][q], w[1][q]);
  }
#pragma unroll
  for (int pl = 0; pl < 2; ++pl)
    out[((tT * 2 + pl) * 2 + h) * 32 + r] = make_uint4(w[pl][0], w[pl][1], w[pl][2], w[pl][3]);
  return bad;
}

__global__ void k_pack_fp32(const float* __restrict__ W, int64_t lr, int64_t lc, int NT, int kin,
                            const float* __restrict__ bias, int64_t total, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    pack_item_fp32(W, lr, lc, NT, kin, bias, i, out);
}

__global__ void k_pack_x3(const float* __restrict__ W, int64_t lr, int64_t lc, int NT, int kin,
                          const float* __restrict__ bias, int64_t total, uint4* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    pack_item_x3(W, lr, lc, NT, kin, bias, i, out);
}

__global__ void k_pack_h2(const float* __restrict__ W, int64_t lr, int64_t lc, int NT, int kin,
                          const float* __restrict__ bias, int64_t total, float sc, int32_t* __restrict__ flag,
                          uint4* __restrict__ out) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    bad |= pack_item_h2(W, lr, lc, NT, kin, bias, i, sc, out);
  if (bad && flag) atomicOr(flag, 1);
}

// Several packs in one launch (pnr_pack_batch): job q owns blocks [blk0_q,
// blk0_{q+1}), one item per thread.  The job is picked with constant indices
// only (uniform selects), so the argument block is never indexed dynamically.
constexpr int kMaxPackJobs = 24;
struct PackJob {
  const float* W;
  const float* bias;
  void* out;
  int32_t* flag;
  int64_t lr, lc, total;
  int32_t kind, NT, kin, blk0;
  float sc;
};
struct PackBatch {
  PackJob j[kMaxPackJobs];
  int32_t n;
};

__global__ void __launch_bounds__(256) k_pack_batch(PackBatch B) {
  PackJob J = B.j[0];
#pragma unroll
  for (int q = 1; q < kMaxPackJobs; ++q)
    if (q < B.n && (int)blockIdx.x >= B.j[q].blk0) J = B.j[q];
  const int64_t i = (int64_t)(blockIdx.x - J.blk0) * 256 + threadIdx.x;
  bool bad = false;
  if (i < J.total) {
    if (J.kind == 0)
      pack_item_fp32(J.W, J.lr, J.lc, J.NT, J.kin, J.bias, i, static_cast<float*>(J.out));
    else if (J.kind == 1)
      pack_item_x3(J.W, J.lr, J.lc, J.NT, J.kin, J.bias, i, static_cast<uint4*>(J.out));
    else
      bad = pack_item_h2(J.W, J.lr, J.lc, J.NT, J.kin, J.bias, i, J.sc, static_cast<uint4*>(J.out));
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0 && J.flag) atomicOr(J.flag, 1);
}

// The shift picked on the device (pnr_pack_weights_h2_dev): k_w_absmax folds
// max |W'| into sc[1] (as bits), k_pack_h2_dev picks s with max |2^-s W'| in
// [8, 16) -- frag_pack_h2's h2_shift -- writes sc[0] = 2^(s - 11) and packs.
__global__ void k_w_absmax(const float* __restrict__ W, int64_t lr, int64_t lc, int out_f, int kin,
                           const float* __restrict__ bias, unsigned* __restrict__ word) {
  __shared__ float red[4];
  float m = 0.f;
  const int64_t total = (int64_t)out_f * (kin + 1);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(i / (kin + 1)), k = (int)(i % (kin + 1));
    const float a = fabsf(wprime(W, lr, lc, kin, bias, o, k));
    m = a != a ? __builtin_inff() : fmaxf(m, a);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
    if (m > 0.f) atomicMax(word, __float_as_uint(m));
  }
}

// 2^-s with max 2^-s in [8, 16) (s = 0 for an all-zero or non-finite W: the
// non-finite weights then reach the outputs as in fp32)
__device__ __forceinline__ int pick_shift(float m) {
  if (!(m > 0.f) || !(m <= 3.0e38f)) return 0;
  int E;
  (void)frexpf(m, &E);   // m = f 2^E, f in [0.5, 1): m 2^-(E-4) in [8, 16)
  return E - 4;
}

__global__ void k_pack_h2_dev(const float* __restrict__ W, int64_t lr, int64_t lc, int NT, int kin,
                              const float* __restrict__ bias, int64_t total, float* __restrict__ sc,
                              uint4* __restrict__ out) {
  const int sft = pick_shift(__uint_as_float(reinterpret_cast<const unsigned*>(sc)[1]));
  const float f = ldexpf(1.f, -sft);
  if (blockIdx.x == 0 && threadIdx.x == 0) sc[0] = ldexpf(1.f, sft - 11);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i & 31), h = (int)((i >> 5) & 1);
    const int64_t tT = i >> 6;
    const int T = (int)(tT % NT), t = (int)(tT / NT);
    const int o = 32 * T + r, k0 = 16 * t + 8 * h;
    unsigned w[2][4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      splith(wprime(W, lr, lc, kin, bias, o, k0 + 2 * q) * f, wprime(W, lr, lc, kin, bias, o, k0 + 2 * q + 1) * f,
             w[0][q], w[1][q]);
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      out[((tT * 2 + pl) * 2 + h) * 32 + r] = make_uint4(w[pl][0], w[pl][1], w[pl][2], w[pl][3]);
  }
}

// The fp32h2 backward's three dX packs in one launch (pnr_pack_bwd_h2):
// workgroup (t, m) packs k-step t of W_m^T (512 items: 8 neuron tiles x 64
// lanes, k_pack_h2_dev's layout, the pad steps zero) after folding max |W_m|
// over the whole 256 x 256 block itself (every workgroup of m reads the same
// 256 KB, from L2 after the first) -- the shift as k_pack_h2_dev picks it, no
// second launch; workgroup (0, m) writes scale[m] = 2^(s - 11).
__global__ void __launch_bounds__(512) k_pack_bwd_h2(const float* __restrict__ w4, const float* __restrict__ w3,
                                                     int64_t ld3, const float* __restrict__ w2, int pad,
                                                     float* __restrict__ scale, uint4* __restrict__ out) {
  const int t = blockIdx.x, mi = blockIdx.y;
  const float* W = mi == 0 ? w4 : (mi == 1 ? w3 : w2);
  const int64_t ld = mi == 1 ? ld3 : 256;
  __shared__ float red[8];
  float mx = 0.f;
  if ((ld & 3) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0) {
#pragma unroll 8
    for (int i = threadIdx.x; i < 256 * 64; i += 512) {
      const float4 v = *reinterpret_cast<const float4*>(W + (int64_t)(i >> 6) * ld + 4 * (i & 63));
      const float a = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
      const bool nan = v.x != v.x || v.y != v.y || v.z != v.z || v.w != v.w;
      mx = nan ? __builtin_inff() : fmaxf(mx, a);
    }
  } else {
#pragma unroll 8
    for (int i = threadIdx.x; i < 256 * 256; i += 512) {
      const float a = fabsf(W[(int64_t)(i >> 8) * ld + (i & 255)]);
      mx = a != a ? __builtin_inff() : fmaxf(mx, a);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) mx = fmaxf(mx, red[i]);
  const int sft = pick_shift(mx);
  const float f = ldexpf(1.f, -sft);
  if (t == 0 && threadIdx.x == 0) scale[mi] = ldexpf(1.f, sft - 11);
  const int r = threadIdx.x & 31, h = (threadIdx.x >> 5) & 1, T = threadIdx.x >> 6;
  const int oc = 32 * T + r, k0 = 16 * t + 8 * h;   // W^T[oc][k] = W[k][oc]
  unsigned w[2][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = k0 + 2 * q;
    const float a = k < 256 ? W[(int64_t)k * ld + oc] * f : 0.f;
    const float b = k + 1 < 256 ? W[(int64_t)(k + 1) * ld + oc] * f : 0.f;
    splith(a, b, w[0][q], w[1][q]);
  }
  uint4* o = out + (int64_t)mi * (16 + pad) * 8 * 64 * 2;
  const int tT = t * 8 + T;
#pragma unroll
  for (int pl = 0; pl < 2; ++pl)
    o[((tT * 2 + pl) * 2 + h) * 32 + r] = make_uint4(w[pl][0], w[pl][1], w[pl][2], w[pl][3]);
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_pack_bwd_h2(const float* w4, const float* w3, int64_t ld3, const float* w2, int32_t pad_steps,
                               float* scale_dev, void* out, size_t out_bytes, void* stream) {
  PNR_CHECK_ARG(w4 && w3 && w2 && scale_dev && out && ld3 >= 256 && pad_steps >= 3 && pad_steps <= 16,
                "pack_bwd_h2: bad args (ld3 %lld, pad %d)", (long long)ld3, pad_steps);
  PNR_CHECK_ARG(((uintptr_t)out & 15) == 0 && ((uintptr_t)scale_dev & 3) == 0,
                "pack_bwd_h2: output must be 16-B and scale 4-B aligned");
  const size_t need = (size_t)3 * (16 + pad_steps) * 8 * 64 * 2 * 16;
  PNR_CHECK_ARG(out_bytes >= need, "pack_bwd_h2: output too small (%zu < %zu)", out_bytes, need);
  hipLaunchKernelGGL(k_pack_bwd_h2, dim3(16 + pad_steps, 3), dim3(512), 0, as_stream(stream), w4, w3, ld3, w2,
                     pad_steps, scale_dev, static_cast<uint4*>(out));
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_pack_weights_h2_dev(const float* W, int64_t ld_row, int64_t ld_col, int32_t out_f, int32_t kin,
                                       const float* bias, int32_t pad_steps, float* scale_dev, void* out,
                                       size_t out_bytes, void* stream) {
  PNR_CHECK_ARG(W && out && scale_dev && out_f > 0 && out_f % 32 == 0 && kin > 0 && pad_steps >= 0,
                "pack_weights_h2_dev: bad args (out_f %d, kin %d)", out_f, kin);
  PNR_CHECK_ARG(((uintptr_t)out & 15) == 0 && ((uintptr_t)scale_dev & 7) == 0,
                "pack_weights_h2_dev: output must be 16-B and scale 8-B aligned");
  const int cols = kin + (bias ? 1 : 0);
  const int NT = out_f / 32;
  const int64_t tot = (cols + 15) / 16 + pad_steps;
  const int64_t total = tot * NT * 64;
  PNR_CHECK_ARG(out_bytes >= (size_t)total * 2 * 16, "pack_weights_h2_dev: output too small (%zu < %lld)", out_bytes,
                (long long)total * 32);
  hipStream_t st = as_stream(stream);
  PNR_HIP(hipMemsetAsync(scale_dev + 1, 0, sizeof(float), st));
  hipLaunchKernelGGL(k_w_absmax, dim3(grid_for((int64_t)out_f * (kin + 1), 256, 64)), dim3(256), 0, st, W, ld_row,
                     ld_col, out_f, kin, bias, reinterpret_cast<unsigned*>(scale_dev + 1));
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_pack_h2_dev, dim3(grid_for(total, 256)), dim3(256), 0, st, W, ld_row, ld_col, NT, kin, bias,
                     total, scale_dev, static_cast<uint4*>(out));
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_pack_weights_h2(const float* W, int64_t ld_row, int64_t ld_col, int32_t out_f, int32_t kin,
                                   const float* bias, int32_t pad_steps, int32_t shift, int32_t* range_flag,
                                   void* out, size_t out_bytes, void* stream) {
  PNR_CHECK_ARG(W && out && out_f > 0 && out_f % 32 == 0 && kin > 0 && pad_steps >= 0 && shift > -120 && shift < 120,
                "pack_weights_h2: bad args (out_f %d, kin %d, shift %d)", out_f, kin, shift);
  PNR_CHECK_ARG(((uintptr_t)out & 15) == 0, "pack_weights_h2: output must be 16-B aligned");
  const int cols = kin + (bias ? 1 : 0);
  const int NT = out_f / 32;
  const int64_t tot = (cols + 15) / 16 + pad_steps;
  const int64_t total = tot * NT * 64;   // threads: (t, T, h, r)
  PNR_CHECK_ARG(out_bytes >= (size_t)total * 2 * 16, "pack_weights_h2: output too small (%zu < %lld)", out_bytes,
                (long long)total * 32);
  hipLaunchKernelGGL(k_pack_h2, dim3(grid_for(total, 256)), dim3(256), 0, as_stream(stream), W, ld_row, ld_col, NT,
                     kin, bias, total, ldexpf(1.f, -shift), range_flag, static_cast<uint4*>(out));
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_pack_batch(const pnr_pack_job* jobs, int32_t n, void* stream) {
  PNR_CHECK_ARG(jobs && n >= 1 && n <= kMaxPackJobs, "pack_batch: %d jobs (1..%d)", n, kMaxPackJobs);
  PackBatch B = {};
  B.n = n;
  int64_t blocks = 0;
  for (int q = 0; q < n; ++q) {
    const pnr_pack_job& g = jobs[q];
    PNR_CHECK_ARG(g.kind >= 0 && g.kind <= 2, "pack_batch: job %d kind %d (0: fp32, 1: fp32x3, 2: fp32h2)", q,
                  g.kind);
    PNR_CHECK_ARG(g.W && g.out && g.out_f > 0 && g.out_f % 32 == 0 && g.kin > 0 && g.pad_steps >= 0 &&
                      g.shift > -120 && g.shift < 120,
                  "pack_batch: job %d bad args (out_f %d, kin %d)", q, g.out_f, g.kin);
    PNR_CHECK_ARG(((uintptr_t)g.out & 15) == 0, "pack_batch: job %d output must be 16-B aligned", q);
    const int cols = g.kin + (g.bias ? 1 : 0);
    const int NT = g.out_f / 32;
    const int64_t tot = g.kind == 0 ? (cols + 1) / 2 + g.pad_steps : (cols + 15) / 16 + g.pad_steps;
    const int64_t total = tot * NT * 64;
    const size_t need = (size_t)total * (g.kind == 0 ? 4 : g.kind == 1 ? 48 : 32);
    PNR_CHECK_ARG(g.out_bytes >= need, "pack_batch: job %d output too small (%zu < %zu)", q, g.out_bytes, need);
    PackJob& J = B.j[q];
    J.W = g.W;
    J.bias = g.bias;
    J.out = g.out;
    J.flag = g.kind == 2 ? g.range_flag : nullptr;
    J.lr = g.ld_row;
    J.lc = g.ld_col;
    J.total = total;
    J.kind = g.kind;
    J.NT = NT;
    J.kin = g.kin;
    J.blk0 = (int32_t)blocks;
    J.sc = ldexpf(1.f, -g.shift);
    blocks += cdiv(total, 256);
  }
  PNR_CHECK_ARG(blocks < (1 << 30), "pack_batch: too many items");
  hipLaunchKernelGGL(k_pack_batch, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), B);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_pack_weights(int32_t kind, const float* W, int64_t ld_row, int64_t ld_col, int32_t out_f,
                                int32_t kin, const float* bias, int32_t pad_steps, void* out, size_t out_bytes,
                                void* stream) {
  PNR_CHECK_ARG(kind == 0 || kind == 1, "pack_weights: kind %d (0: fp32, 1: fp32x3)", kind);
  PNR_CHECK_ARG(W && out && out_f > 0 && out_f % 32 == 0 && kin > 0 && pad_steps >= 0,
                "pack_weights: bad args (out_f %d, kin %d)", out_f, kin);
  PNR_CHECK_ARG(((uintptr_t)out & 15) == 0, "pack_weights: output must be 16-B aligned");
  const int cols = kin + (bias ? 1 : 0);
  const int NT = out_f / 32;
  hipStream_t st = as_stream(stream);
  if (kind == 0) {
    const int64_t tot = (cols + 1) / 2 + pad_steps;
    const int64_t total = tot * NT * 64;
    PNR_CHECK_ARG(out_bytes >= (size_t)total * 4, "pack_weights: output too small (%zu < %lld)", out_bytes,
                  (long long)total * 4);
    hipLaunchKernelGGL(k_pack_fp32, dim3(grid_for(total, 256)), dim3(256), 0, st, W, ld_row, ld_col, NT, kin, bias,
                       total, static_cast<float*>(out));
  } else {
    const int64_t tot = (cols + 15) / 16 + pad_steps;
    const int64_t total = tot * NT * 64;   // threads: (t, T, h, r)
    PNR_CHECK_ARG(out_bytes >= (size_t)total * 3 * 16, "pack_weights: output too small (%zu < %lld)", out_bytes,
                  (long long)total * 48);
    hipLaunchKernelGGL(k_pack_x3, dim3(grid_for(total, 256)), dim3(256), 0, st, W, ld_row, ld_col, NT, kin, bias,
                       total, static_cast<uint4*>(out));
  }
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
