// Fused K-neighbour gather + inverse-distance weights + positional encodings +
// per-(sample, neighbour) MLP + K-weighted sums + per-sample colour MLP.
//
// Replaces, for agg_intrp_order 2 / agg_distance_kernel "linear" /
// agg_dist_pers 20 (the lego configuration, dev_scripts/w_n360/lego.sh):
//   NeuralPoints.forward gather             neural_points.py:782-812
//   PointAggregator.forward                 point_aggregators.py:729-816
//     linear kernel + normalisation         point_aggregators.py:421-429, 803-804
//     gradiant_clamp(conf)                  point_aggregators.py:724-726, 810-813
//   viewmlp (order 2)                       point_aggregators.py:488-646
//   positional_encoding                     models/helpers/networks.py:175-190
//
// CDNA4 mapping.  One wave owns 32 (sample, neighbour) pairs = 4 samples x K=8
// and carries them through all four 256-wide layers:
//   Y^T[256 x 32] = W[256 x Kin] . X^T[Kin x 32]  with v_mfma_f32_32x32x2_f32
// (exact fp32 fmaf chains; gfx950 has no TF32).  The pair is the MFMA column
// (lane & 31): the 8 accumulator tiles (128 AGPRs) hold the layer output with
// the neuron on the register and the pair on the lane.  Each layer's input
// X^T lives in a per-wave k-major LDS slice [k][32] (36 KB; 4 waves = 144 KB
// of the CU's 160 KB), read with one conflict-free ds_read_b32 per k-step and
// shared by the 8 MFMAs of the step; the activated accumulator is written
// back in natural neuron order, so every weight matrix uses one "fragment"
// layout W_f[t][T][lane] = W[32T + (lane&31)][2t + (lane>>5)] and every
// A-operand load is a coalesced 256-B wave load from L2.  Layer-1 inputs
// (embedding, 3-band PE of the embedding, 5-band PE of the 6-d distance) are
// produced straight into the LDS slice by the lane that owns the pair.  No
// workgroup barriers: waves run independent persistent loops.  The
// 280->128->128->128 colour branch (3 % of the FLOPs) runs on the VALU from
// the same (then dead) LDS slice.
#include "pnr_common.h"

namespace pnr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kAggBlock = 256;     // 4 waves
constexpr int kSampPerWave = 4;    // 4 samples x 8 neighbours = 32 MFMA columns
constexpr int kKN = 8;
constexpr int kHid = 256;
constexpr int kEmb = 32;
constexpr int kC = 128;
constexpr int kCin = 280;          // 256 + 24 view PE
constexpr int kFPitch = 288;       // LDS row pitch of the colour-branch input

struct AggArgs {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp w;
  float* out_feat;
  float* out_weight;
  float* out_conf;
  const uint8_t* pair_mask;   // mirror path: validity per (row, k); pidx == NULL
};

__device__ __forceinline__ float lrelu(float x, float s) { return x > 0.f ? x : x * s; }

__device__ __forceinline__ float softplus(float x) {  // torch.nn.Softplus(beta=1, threshold=20)
  return x > 20.f ? x : log1pf(expf(x));
}

// Row of the accumulator register `r` for lane half `h` (32x32 C/D layout).
__device__ __forceinline__ constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ void bias_init(f32x16 (&acc)[8], const float* __restrict__ b, int h) {
#pragma unroll
  for (int T = 0; T < 8; ++T)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[T][r] = b[32 * T + acc_row(r, h)];
}

// Y^T += W . X^T over nsteps k-steps (2 k-values each); X^T from the wave's
// LDS slice, W in fragment layout.  8 MFMAs share each B operand.
__device__ __forceinline__ void mlp_layer(f32x16 (&acc)[8], const float* __restrict__ wf,
                                          const float* X, int nsteps, int lane) {
  const int m = lane & 31, h = lane >> 5;
  const float* p = wf + lane;
#pragma unroll 2
  for (int t = 0; t < nsteps; ++t) {
    const float x = X[(2 * t + h) * 32 + m];
    float a[8];
#pragma unroll
    for (int T = 0; T < 8; ++T) a[T] = p[(t * 8 + T) * 64];
#pragma unroll
    for (int T = 0; T < 8; ++T) acc[T] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[T], x, acc[T], 0, 0, 0);
  }
}

// Activated accumulator -> X^T rows in natural neuron order.
__device__ __forceinline__ void store_act(const f32x16 (&acc)[8], float* X, float s, int lane) {
  const int m = lane & 31, h = lane >> 5;
#pragma unroll
  for (int T = 0; T < 8; ++T)
#pragma unroll
    for (int r = 0; r < 16; ++r) X[(32 * T + acc_row(r, h)) * 32 + m] = lrelu(acc[T][r], s);
}

__device__ __forceinline__ void activate(f32x16 (&acc)[8], float s) {  // in place
#pragma unroll
  for (int T = 0; T < 8; ++T)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[T][r] = lrelu(acc[T][r], s);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

constexpr int kXRows = 288;                 // >= 284 (layer-1 inputs), multiple of 32
constexpr int kWaveLds = kXRows * 32;       // floats per wave slice (36 KB)

__global__ void __launch_bounds__(kAggBlock, 1) k_aggregate(AggArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* X = lds_dyn + wid * kWaveLds;          // [kXRows][32] layer input X^T
  float* F = X;                                 // [4][kFPitch] colour input (aliases X)
  float* G = X + kSampPerWave * kFPitch;        // [4][kC] colour hidden (aliases X)
  const int m = lane & 31, h = lane >> 5, j = m >> 3, k = m & 7;
  const int K = A.s.K;
  int64_t n = A.s.n_max;
  if (A.s.n_dev) {
    int64_t nd = *A.s.n_dev;
    n = nd < n ? nd : n;
  }
  const int64_t ntiles = cdiv(n, kSampPerWave);
  const float neg = A.w.neg_slope;
  float Rw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
  float cam_c[3] = {0.f, 0.f, 0.f}, cam_R[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f};
  if (!A.pts.pers) {
#pragma unroll
    for (int i = 0; i < 3; ++i) cam_c[i] = A.pts.campos[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) cam_R[i] = A.pts.camrot[i];
  }

  for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    // ------------------------------------------------------------ gather (neural_points.py:788-799)
    const int64_t v = tile * kSampPerWave + j;
    const bool active = v < n;
    const int64_t row = active ? (A.s.samp_list ? (int64_t)A.s.samp_list[v] : v) : 0;
    int64_t prow = -1;  // point row
    bool valid = false;
    if (active && k < K) {
      if (A.s.pidx) {
        const int pid = A.s.pidx[row * K + k];
        valid = pid >= 0;
        prow = valid ? pid : 0;  // torch.clamp(sample_pidx, min=0)
      } else {
        prow = row * K + k;
        valid = A.pair_mask[prow] != 0;
      }
    }
    float sw[3] = {0.f, 0.f, 0.f}, sp[3] = {0.f, 0.f, 0.f}, vd[3] = {0.f, 0.f, 0.f};
    if (active) {
      const int64_t drow = (A.s.dir_map ? (int64_t)A.s.dir_map[row] : row) / A.s.dir_div;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        sw[a] = A.s.sample_w[row * 3 + a];
        sp[a] = A.s.sample_p[row * 3 + a];
        vd[a] = A.s.dirs[drow * 3 + a];
      }
    }
    float pw[3] = {0.f, 0.f, 0.f}, pp[3] = {0.f, 0.f, 0.f}, col[3] = {0.f, 0.f, 0.f},
          pdir[3] = {0.f, 0.f, 0.f};
    float cf = 1.f;
    if (valid) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        pw[a] = A.pts.xyz[prow * 3 + a];
        col[a] = A.pts.color ? A.pts.color[prow * 3 + a] : 0.f;
        pdir[a] = A.pts.dir ? A.pts.dir[prow * 3 + a] : 0.f;
      }
      if (A.pts.pers) {
#pragma unroll
        for (int a = 0; a < 3; ++a) pp[a] = A.pts.pers[prow * 3 + a];
      } else {
        world_to_pers(pw, cam_c, cam_R, pp);
      }
    }
    if (A.pts.conf && prow >= 0) cf = A.pts.conf[prow];
    // embedding -> X rows 0..31 (lane half h writes the odd/even rows)
    {
      const float* e = A.pts.emb + (valid ? prow : 0) * kEmb;
#pragma unroll
      for (int q = 0; q < kEmb / 2; ++q) X[(2 * q + h) * 32 + m] = valid ? e[2 * q + h] : 0.f;
    }
    // dists, agg_dist_pers == 20 (point_aggregators.py:775-783)
    float d6[6];
    d6[0] = pw[0] - sw[0];
    d6[1] = pw[1] - sw[1];
    d6[2] = pw[2] - sw[2];
    d6[3] = pp[0] * pp[2] - sp[0] * sp[2];
    d6[4] = pp[1] * pp[2] - sp[1] * sp[2];
    d6[5] = pp[2] - sp[2];
    // linear kernel (point_aggregators.py:421-429) and normalisation (:803-804)
    const float nrm = sqrtf(d6[0] * d6[0] + d6[1] * d6[1] + d6[2] * d6[2]);
    const float wl = valid ? 1.f / fmaxf(nrm, 1e-6f) : 0.f;
    const float wsum = xor8_sum(wl);
    const float wn = wl / fmaxf(wsum, 1e-8f);
    const float confc = fminf(fmaxf(cf, 1e-4f), 1.f);
    const float wt = wn * confc;
    const bool samp_valid = xor8_sum(valid ? 1.f : 0.f) > 0.f;
    if (h == 0 && active && k < K) {
      if (A.out_weight) A.out_weight[row * K + k] = wn;
      if (A.out_conf) A.out_conf[row * K + k] = confc;
    }
    // rotated distance / direction inputs (point_aggregators.py:506, 526, 566-570)
    float dr6[6];
    mat3(Rw, d6, dr6);
    dr6[3] = d6[3];
    dr6[4] = d6[4];
    dr6[5] = d6[5];
    float vrot[3], drot[3];
    mat3(Rw, vd, vrot);
    mat3(Rw, pdir, drot);
    wave_sync();
    // PE_3(embedding) -> X rows 32..223: row 32 + 2(3c+f) + {sin, cos}
    for (int i = 16; i < 112; ++i) {
      const int p = i - 16, c = p / 3, f = p - 3 * c;
      const float arg = X[c * 32 + m] * (float)(1 << f);
      X[(2 * i + h) * 32 + m] = h ? cosf(arg) : sinf(arg);
    }
    // PE_5(rotated dists) -> X rows 224..283
    for (int i = 112; i < 142; ++i) {
      const int p = i - 112, c = p / 5, f = p - 5 * c;
      float dc = dr6[0];
      dc = c == 1 ? dr6[1] : dc;
      dc = c == 2 ? dr6[2] : dc;
      dc = c == 3 ? dr6[3] : dc;
      dc = c == 4 ? dr6[4] : dc;
      dc = c == 5 ? dr6[5] : dc;
      const float arg = dc * (float)(1 << f);
      X[(2 * i + h) * 32 + m] = h ? cosf(arg) : sinf(arg);
    }
    wave_sync();

    f32x16 acc[8];
    // ------------------------------------------------------------ block1: 284 -> 256 -> 256
    bias_init(acc, A.w.b1, h);
    mlp_layer(acc, A.w.w1f, X, 142, lane);
    wave_sync();
    store_act(acc, X, neg, lane);
    wave_sync();
    bias_init(acc, A.w.b2, h);
    mlp_layer(acc, A.w.w2f, X, 128, lane);
    wave_sync();
    store_act(acc, X, neg, lane);
    // block3 extra inputs, rows 256..263: colour(3), R.dir - R.v (3), <R.dir, R.v> (1), 0
    {
      const float dot = drot[0] * vrot[0] + drot[1] * vrot[1] + drot[2] * vrot[2];
      const float ex[8] = {col[0], col[1], col[2], drot[0] - vrot[0],
                           drot[1] - vrot[1], drot[2] - vrot[2], dot, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) X[(256 + 2 * e + h) * 32 + m] = h ? ex[2 * e + 1] : ex[2 * e];
    }
    wave_sync();
    // ------------------------------------------------------------ block3: 263 -> 256 -> 256
    bias_init(acc, A.w.b3, h);
    mlp_layer(acc, A.w.w3f, X, 132, lane);
    wave_sync();
    store_act(acc, X, neg, lane);
    wave_sync();
    bias_init(acc, A.w.b4, h);
    mlp_layer(acc, A.w.w4f, X, 128, lane);
    activate(acc, neg);
    wave_sync();  // X is dead from here on: F/G alias it
    // ------------------------------------------------------------ alpha branch + K sums
    float pa = 0.f;
#pragma unroll
    for (int T = 0; T < 8; ++T)
#pragma unroll
      for (int r = 0; r < 16; ++r) pa += acc[T][r] * A.w.wa[32 * T + acc_row(r, h)];
    pa += __shfl_xor(pa, 32);
    pa += A.w.ba[0];
    const float alpha_k = A.w.act_super ? softplus(pa - 1.f) : fmaxf(pa, 0.f);
    const float alpha_s = xor8_sum(wt * alpha_k);   // point_aggregators.py:608-614
    // feature K-sum (point_aggregators.py:622-628) -> F[j][n]
#pragma unroll
    for (int T = 0; T < 8; ++T)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float s = xor8_sum(acc[T][r] * wt);
        if (k == 0) F[j * kFPitch + 32 * T + acc_row(r, h)] = s;
      }
    // view-direction PE, ori dropped (point_aggregators.py:507-512): sin block then cos block
    {
      const int qd = k * 2 + h;  // 0..15 per sample
#pragma unroll
      for (int rep = 0; rep < 2; ++rep) {
        const int q = qd + 16 * rep;
        if (q < 24) {
          const int blk = q / 12, c = (q % 12) / 4, f = q % 4;
          const float vc = c == 0 ? vrot[0] : (c == 1 ? vrot[1] : vrot[2]);
          const float arg = vc * (float)(1 << f);
          F[j * kFPitch + kHid + q] = blk ? cosf(arg) : sinf(arg);
        }
      }
    }
    wave_sync();
    // ------------------------------------------------------------ colour branch 280->128->128->128
    float c0[kSampPerWave], c1[kSampPerWave];
#pragma unroll
    for (int s = 0; s < kSampPerWave; ++s) {
      c0[s] = A.w.bc1[lane];
      c1[s] = A.w.bc1[lane + 64];
    }
#pragma unroll 4
    for (int kk = 0; kk < kCin; ++kk) {
      const float w0 = A.w.wc1t[kk * kC + lane], w1 = A.w.wc1t[kk * kC + 64 + lane];
#pragma unroll
      for (int s = 0; s < kSampPerWave; ++s) {
        const float x = F[s * kFPitch + kk];
        c0[s] += w0 * x;
        c1[s] += w1 * x;
      }
    }
#pragma unroll
    for (int s = 0; s < kSampPerWave; ++s) {
      G[s * kC + lane] = lrelu(c0[s], neg);
      G[s * kC + 64 + lane] = lrelu(c1[s], neg);
    }
    wave_sync();
#pragma unroll
    for (int s = 0; s < kSampPerWave; ++s) {
      c0[s] = A.w.bc2[lane];
      c1[s] = A.w.bc2[lane + 64];
    }
#pragma unroll 4
    for (int kk = 0; kk < kC; ++kk) {
      const float w0 = A.w.wc2t[kk * kC + lane], w1 = A.w.wc2t[kk * kC + 64 + lane];
#pragma unroll
      for (int s = 0; s < kSampPerWave; ++s) {
        const float x = G[s * kC + kk];
        c0[s] += w0 * x;
        c1[s] += w1 * x;
      }
    }
    wave_sync();
#pragma unroll
    for (int s = 0; s < kSampPerWave; ++s) {
      F[s * kFPitch + lane] = lrelu(c0[s], neg);
      F[s * kFPitch + 64 + lane] = lrelu(c1[s], neg);
    }
    wave_sync();
#pragma unroll
    for (int s = 0; s < kSampPerWave; ++s) {
      c0[s] = A.w.bc3[lane];
      c1[s] = A.w.bc3[lane + 64];
    }
#pragma unroll 4
    for (int kk = 0; kk < kC; ++kk) {
      const float w0 = A.w.wc3t[kk * kC + lane], w1 = A.w.wc3t[kk * kC + 64 + lane];
#pragma unroll
      for (int s = 0; s < kSampPerWave; ++s) {
        const float x = F[s * kFPitch + kk];
        c0[s] += w0 * x;
        c1[s] += w1 * x;
      }
    }
    // ------------------------------------------------------------ write [alpha, c_1..c_128]
    // each sample's (row, valid, alpha) comes from the lane owning its neighbour 0
#pragma unroll
    for (int s = 0; s < kSampPerWave; ++s) {
      const int src = s * 8;
      const bool act_s = __shfl((int)(active && samp_valid), src) != 0;
      const float al_s = __shfl(alpha_s, src);
      if (act_s) {
        // output row = position in the sample list (compact valid-sample index)
        float* o = A.out_feat + (tile * kSampPerWave + s) * (kC + 1);
        if (lane == 0) o[0] = al_s;
        o[1 + lane] = lrelu(c0[s], neg);
        o[1 + 64 + lane] = lrelu(c1[s], neg);
      }
    }
    wave_sync();
  }
}

constexpr size_t kAggLdsBytes = (size_t)4 * kWaveLds * sizeof(float);

}  // namespace pnr

using namespace pnr;

static void set_lds_attr() {
  static bool done = false;
  if (!done) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_aggregate),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAggLdsBytes);
    done = true;
  }
}

extern "C" int pnr_aggregate_fwd(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                 float* out_feat, float* out_weight, float* out_conf, void* stream) {
  PNR_CHECK_ARG(pts && s && w && out_feat, "aggregate: null pointer");
  PNR_CHECK_ARG(pts->xyz && pts->emb, "aggregate: point xyz/emb required");
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate: need pers or camera");
  PNR_CHECK_ARG(s->sample_w && s->sample_p && s->dirs, "aggregate: sample arrays required");
  PNR_CHECK_ARG(s->K >= 1 && s->K <= kKN, "aggregate: K=%d unsupported (1..8)", s->K);
  PNR_CHECK_ARG(s->dir_div >= 1, "aggregate: dir_div must be >= 1");
  PNR_CHECK_ARG(w->w1f && w->b1 && w->w2f && w->b2 && w->w3f && w->b3 && w->w4f && w->b4 && w->wa &&
                    w->ba && w->wc1t && w->bc1 && w->wc2t && w->bc2 && w->wc3t && w->bc3,
                "aggregate: null weight");
  PNR_CHECK_ARG(((uintptr_t)pts->emb & 15) == 0, "aggregate: emb must be 16-B aligned");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  const int64_t tiles = cdiv(s->n_max, kSampPerWave);
  const unsigned grid = grid_for(tiles, 4, 256);
  set_lds_attr();
  hipLaunchKernelGGL(k_aggregate, dim3(grid), dim3(kAggBlock), kAggLdsBytes, as_stream(stream), a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// Mirror-path entry: pre-gathered [rows,K,C] tensors (PointAggregator.forward
// signature), validity from sample_pnt_mask.  Not in the public header's hot
// path; used by pointnerf_amd.aggregator.PointAggregator.
extern "C" int pnr_aggregate_fwd_masked(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                        const uint8_t* pair_mask, float* out_feat, float* out_weight,
                                        float* out_conf, void* stream) {
  PNR_CHECK_ARG(pts && s && w && out_feat && pair_mask, "aggregate_masked: null pointer");
  PNR_CHECK_ARG(pts->xyz && pts->emb && pts->pers, "aggregate_masked: xyz/emb/pers required");
  PNR_CHECK_ARG(s->pidx == nullptr, "aggregate_masked: pidx must be NULL (identity rows)");
  PNR_CHECK_ARG(s->K >= 1 && s->K <= kKN, "aggregate_masked: K=%d unsupported (1..8)", s->K);
  PNR_CHECK_ARG(s->dir_div >= 1, "aggregate_masked: dir_div must be >= 1");
  PNR_CHECK_ARG(((uintptr_t)pts->emb & 15) == 0, "aggregate_masked: emb must be 16-B aligned");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = pair_mask;
  const int64_t tiles = cdiv(s->n_max, kSampPerWave);
  const unsigned grid = grid_for(tiles, 4, 256);
  set_lds_attr();
  hipLaunchKernelGGL(k_aggregate, dim3(grid), dim3(kAggBlock), kAggLdsBytes, as_stream(stream), a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
