// Adam step over the training parameters (the "+ Adam" of the c3 finetune step,
// train_ddp.py's torch.optim.Adam over the point tables and the aggregator MLP;
// mvs_points_volumetric_model.py:102-123 builds its param groups).
//
// torch.optim.Adam (amsgrad = False, maximize = False) per element, with the
// step count and bias corrections on the host:
//   g' = g + wd * p
//   m  = b1 m + (1 - b1) g'            v = b2 v + (1 - b2) g'^2
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// HBM-bound: 16 B read (p, g, m, v) + 12 B written (p, m, v) per element --
// 2.2 GB per step for the 2 M-point lego tables (39 floats per point).  One
// launch covers up to kAdamMax tensors: the host cuts every tensor into 8 K
// element chunks, a workgroup takes one chunk (its tensor found from the chunk
// prefix table, read from the kernel arguments), and its 256 lanes move float4
// quads (scalar lanes only for an unaligned tensor / a ragged tail).  Four quads
// per lane in flight measured the same (389 vs 385 us per step): ~9.5 K
// workgroups already keep enough loads in flight.
#include <cmath>

#include "pnr_common.h"

namespace pnr {

constexpr int kAdamMax = 32;
constexpr int kAdamBlock = 256;
constexpr int64_t kAdamChunk = 8192;   // elements per workgroup (32 per lane)
constexpr int kAdamQ = 4;               // float4 quads per lane in flight (2: 0.394 ms, 4: 0.377, one: 0.385)

struct AdamArgs {
  float* p[kAdamMax];
  const float* g[kAdamMax];
  float* m[kAdamMax];
  float* v[kAdamMax];
  int64_t n[kAdamMax];
  int64_t chunk0[kAdamMax + 1];   // first chunk of tensor i (prefix of ceil(n / kAdamChunk))
  int nt;
  float b1, b2, omb1, omb2, eps, wd, step_size, bc2_sqrt;   // omb = 1 - beta, rounded from double
};

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, const AdamArgs& a) {
  const float gd = a.wd != 0.f ? fmaf(a.wd, p, g) : g;
  m = fmaf(a.b1, m, a.omb1 * gd);
  v = fmaf(a.b2, v, a.omb2 * gd * gd);
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = fmaf(-a.step_size, m / denom, p);   // addcdiv_(m, denom, -step_size)
}

__global__ void __launch_bounds__(kAdamBlock) k_adam(AdamArgs a) {
  const int64_t c = blockIdx.x;
  int t = 0;
  while (t + 1 < a.nt && a.chunk0[t + 1] <= c) ++t;
  const int64_t n = a.n[t];
  const int64_t e0 = (c - a.chunk0[t]) * kAdamChunk;
  const int64_t e1 = min(n, e0 + kAdamChunk);
  float* __restrict__ P = a.p[t];
  const float* __restrict__ G = a.g[t];
  float* __restrict__ M = a.m[t];
  float* __restrict__ V = a.v[t];
  const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) |
                     reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(V)) & 15) == 0;
  if (vec) {
    const int64_t q1 = e0 + ((e1 - e0) & ~int64_t(3));   // float4 quads [e0, q1), e0 % 4 == 0
    typedef float f4 __attribute__((ext_vector_type(4)));
    // kAdamQ quads per lane per round, all 4 kAdamQ loads issued before any math
    // (tools/adam_bench.py, the finetune set's 78 M elements: 0.385 -> 0.377 ms, 5.8 TB/s)
    for (int64_t e = e0 + 4 * (int64_t)threadIdx.x; e < q1; e += 4 * kAdamQ * kAdamBlock) {
      f4 pv[kAdamQ], gv[kAdamQ], mv[kAdamQ], vv[kAdamQ];
#pragma unroll
      for (int u = 0; u < kAdamQ; ++u) {
        const int64_t eu = e + (int64_t)u * 4 * kAdamBlock;
        const int64_t ec = eu < q1 ? eu : e;   // past the tensor: reload (never stored)
        pv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(P + ec));
        gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(G + ec));
        mv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(M + ec));
        vv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(V + ec));
      }
#pragma unroll
      for (int u = 0; u < kAdamQ; ++u) {
        const int64_t eu = e + (int64_t)u * 4 * kAdamBlock;
        float4 p = make_float4(pv[u].x, pv[u].y, pv[u].z, pv[u].w), m = make_float4(mv[u].x, mv[u].y, mv[u].z, mv[u].w);
        float4 v = make_float4(vv[u].x, vv[u].y, vv[u].z, vv[u].w);
        const float4 g = make_float4(gv[u].x, gv[u].y, gv[u].z, gv[u].w);
        adam1(p.x, g.x, m.x, v.x, a);
        adam1(p.y, g.y, m.y, v.y, a);
        adam1(p.z, g.z, m.z, v.z, a);
        adam1(p.w, g.w, m.w, v.w, a);
        if (eu < q1) {
          __builtin_nontemporal_store((f4){p.x, p.y, p.z, p.w}, reinterpret_cast<f4*>(P + eu));
          __builtin_nontemporal_store((f4){m.x, m.y, m.z, m.w}, reinterpret_cast<f4*>(M + eu));
          __builtin_nontemporal_store((f4){v.x, v.y, v.z, v.w}, reinterpret_cast<f4*>(V + eu));
        }
      }
    }
    for (int64_t e = q1 + threadIdx.x; e < e1; e += kAdamBlock) adam1(P[e], G[e], M[e], V[e], a);
  } else {
    for (int64_t e = e0 + threadIdx.x; e < e1; e += kAdamBlock) adam1(P[e], G[e], M[e], V[e], a);
  }
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_adam_step(int32_t n_tensors, float* const* params, const float* const* grads,
                             float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                             double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                             void* stream) {
  PNR_CHECK_ARG(n_tensors >= 0 && (n_tensors == 0 || (params && grads && exp_avg && exp_avg_sq && numel)),
                "adam: null tensor table");
  PNR_CHECK_ARG(step >= 1, "adam: step counts from 1");
  PNR_CHECK_ARG(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0 && lr >= 0.0,
                "adam: bad hyperparameters");
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  hipStream_t st = as_stream(stream);
  int i = 0;
  while (i < n_tensors) {
    AdamArgs a;
    a.nt = 0;
    a.chunk0[0] = 0;
    for (; i < n_tensors && a.nt < kAdamMax; ++i) {
      PNR_CHECK_ARG(numel[i] >= 0, "adam: tensor %d numel < 0", i);
      if (numel[i] == 0) continue;
      PNR_CHECK_ARG(params[i] && grads[i] && exp_avg[i] && exp_avg_sq[i], "adam: tensor %d null", i);
      const int k = a.nt++;
      a.p[k] = params[i];
      a.g[k] = grads[i];
      a.m[k] = exp_avg[i];
      a.v[k] = exp_avg_sq[i];
      a.n[k] = numel[i];
      a.chunk0[k + 1] = a.chunk0[k] + cdiv(numel[i], kAdamChunk);
    }
    if (a.nt == 0) continue;
    a.b1 = (float)beta1;
    a.b2 = (float)beta2;
    a.omb1 = (float)(1.0 - beta1);   // as torch: 1 - beta on python floats, then fp32
    a.omb2 = (float)(1.0 - beta2);
    a.eps = (float)eps;
    a.wd = (float)weight_decay;
    a.step_size = (float)(lr / bc1);
    a.bc2_sqrt = (float)std::sqrt(bc2);
    const int64_t chunks = a.chunk0[a.nt];
    PNR_CHECK_ARG(chunks < (int64_t)1 << 31, "adam: too many chunks");
    hipLaunchKernelGGL(k_adam, dim3((unsigned)chunks), dim3(kAdamBlock), 0, st, a);
    PNR_LAUNCH_CHECK();
  }
  return PNR_OK;
}
