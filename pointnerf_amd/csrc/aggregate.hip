// Fused K-neighbour gather + inverse-distance weights + positional encodings +
// per-(sample, neighbour) MLP + K-weighted sums, then the per-sample colour MLP.
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
// CDNA4 mapping.
// k_pairs: one wave owns 32 (sample, neighbour) pairs = 4 samples x K=8 and
// carries them through the four 256-wide layers as
//   Y^T[256 x 32] = W[256 x Kin] . X^T[Kin x 32]  on v_mfma_f32_32x32x2_f32
// (exact fp32 fmaf chains; gfx950 has no TF32).  The pair is the MFMA column
// (lane & 31): 8 accumulator tiles (128 AGPRs) hold a layer's output with the
// neuron on the register and the pair on the lane.  Each layer's input X^T
// lives in a per-wave k-major LDS slice [k][33] (38 KB; 4 waves = 153 KB of
// the CU's 160 KB), one conflict-free ds_read_b32 per k-step shared by 8
// MFMAs; activations are written back in natural neuron order, so every
// weight matrix uses one "fragment" layout W_f[t][T][lane] =
// W[32T + (lane&31)][2t + (lane>>5)] and every A-operand load is a coalesced
// 256-B wave load from L2, software-pipelined kPD k-steps ahead.  Layer-1
// inputs (embedding, 3-band PE of the embedding via sincos + angle doubling,
// 5-band PE of the 6-d distance) are produced straight into the LDS slice by
// the lane that owns the pair.  The K-sums run as wave shuffles; per valid
// sample only alpha (-> out_feat[:,0]) and the 256-d feature leave the kernel.
// k_color: one wave owns 32 samples and runs 280->128->128->128 with the same
// machinery (4 accumulator tiles), so the colour branch (3 % of the FLOPs) also
// runs on full-width MFMA instead of 4-sample VALU loops.
#include "pnr_common.h"

namespace pnr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kAggBlock = 256;     // 4 waves, each independent
constexpr int kSampPerWave = 4;    // 4 samples x 8 neighbours = 32 MFMA columns
constexpr int kKN = 8;
constexpr int kHid = 256;
constexpr int kEmb = 32;
constexpr int kC = 128;
constexpr int kCin = 280;          // 256 + 24 view PE
constexpr int kPitch = 33;         // LDS row pitch (floats) of X^T[k][32 + 1]
constexpr int kXRows = 296;        // >= 286 layer-1 inputs + bias, + x prefetch overrun
constexpr int kWaveLds = kXRows * kPitch;  // floats per wave slice
constexpr size_t kAggLdsBytes = (size_t)4 * kWaveLds * sizeof(float);
constexpr int kWtRow = 286;        // X^T row holding the per-pair blend weight after layer 4
constexpr int kPD = 4;             // weight prefetch depth in k-steps (packed weights are
                                   // padded with kPD zero k-steps so prefetch never overruns)

struct AggArgs {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp w;
  float* p1;                  // [N, 256] per-point block1.0 partial (k_point_pre -> k_pairs)
  float* hid;                 // [n_max, 256] K-summed features (k_pairs -> k_color)
  int32_t* vmask;             // [n_max] sample has >= 1 valid neighbour (k_pairs -> k_color)
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

template <int NT>
__device__ __forceinline__ void zero_acc(f32x16 (&acc)[NT]) {
#pragma unroll
  for (int T = 0; T < NT; ++T) acc[T] = (f32x16){0.f};
}

// The bias rides in the MFMA: the packed weights carry it as input column
// `kin` (frag_pack), so X^T row kin holds 1 and row kin+1 (if the k-step is
// shared) holds 0.
__device__ __forceinline__ void bias_rows(float* X, int kin, int lane) {
  const int m = lane & 31, h = lane >> 5;
  if ((kin & 1) == 0) X[(kin + h) * kPitch + m] = h ? 0.f : 1.f;
  else if (h == 0) X[kin * kPitch + m] = 1.f;
}

template <int NT>
__device__ __forceinline__ void load_w(float (&a)[NT], const float* __restrict__ p, int t) {
#pragma unroll
  for (int T = 0; T < NT; ++T) a[T] = p[(t * NT + T) * 64];
}

template <int NT>
__device__ __forceinline__ void mfma_step(f32x16 (&acc)[NT], const float (&a)[NT], float x) {
#pragma unroll
  for (int T = 0; T < NT; ++T) acc[T] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[T], x, acc[T], 0, 0, 0);
}

// Y^T += W . X^T over nsteps k-steps (2 k-values each); X^T from the wave's
// LDS slice, W in fragment layout, weight loads issued kPD steps ahead.
template <int NT>
__device__ __forceinline__ void mlp_layer(f32x16 (&acc)[NT], const float* __restrict__ wf,
                                          const float* X, int nsteps, int lane) {
  const int m = lane & 31, h = lane >> 5;
  const float* p = wf + lane;
  const float* xr = X + h * kPitch + m;
  float a0[NT], a1[NT], a2[NT], a3[NT];
  load_w<NT>(a0, p, 0);
  load_w<NT>(a1, p, 1);
  load_w<NT>(a2, p, 2);
  load_w<NT>(a3, p, 3);
  // B operands of the current 4 k-steps; the next 4 are read from LDS one
  // iteration ahead (rows past the layer's inputs are read but never used)
  float x0 = xr[0], x1 = xr[2 * kPitch], x2 = xr[4 * kPitch], x3 = xr[6 * kPitch];
  int t = 0;
#pragma unroll 1
  for (; t + kPD <= nsteps; t += kPD) {
    const float* xn = xr + 2 * (t + kPD) * kPitch;
    // sched_barrier(0) pins the software pipeline: hipcc otherwise sinks the
    // next iteration's LDS reads next to their use (exposed LDS latency)
    mfma_step<NT>(acc, a0, x0);
    const float y0 = xn[0], y1 = xn[2 * kPitch], y2 = xn[4 * kPitch], y3 = xn[6 * kPitch];
    load_w<NT>(a0, p, t + 4);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step<NT>(acc, a1, x1);
    load_w<NT>(a1, p, t + 5);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step<NT>(acc, a2, x2);
    load_w<NT>(a2, p, t + 6);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step<NT>(acc, a3, x3);
    load_w<NT>(a3, p, t + 7);
    __builtin_amdgcn_sched_barrier(0);
    x0 = y0;
    x1 = y1;
    x2 = y2;
    x3 = y3;
  }
  const int rem = nsteps - t;  // 0..3
  if (rem > 0) mfma_step<NT>(acc, a0, x0);
  if (rem > 1) mfma_step<NT>(acc, a1, x1);
  if (rem > 2) mfma_step<NT>(acc, a2, x2);
}

// Activated accumulator -> X^T rows in natural neuron order.
template <int NT>
__device__ __forceinline__ void store_act(const f32x16 (&acc)[NT], float* X, float s, int lane) {
  const int m = lane & 31, h = lane >> 5;
#pragma unroll
  for (int T = 0; T < NT; ++T)
#pragma unroll
    for (int r = 0; r < 16; ++r) X[(32 * T + acc_row(r, h)) * kPitch + m] = lrelu(acc[T][r], s);
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

// Per-point half of block1.0 (exact split of the 284-input Linear): the
// embedding and its 3-band PE depend only on the point, so
// P1[p] = W1[:, :224] . [emb_p, PE_3(emb_p)] + b1 is evaluated once per point
// and gathered per pair instead of being recomputed for every (sample,
// neighbour) pair that references the point (~22x reuse at 2 M points).
__global__ void __launch_bounds__(kAggBlock, 1) k_point_pre(AggArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* X = lds_dyn + wid * kWaveLds;
  const int m = lane & 31, h = lane >> 5;
  const int64_t np = A.pts.n;
  const int64_t ntiles = cdiv(np, 32);
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t pt = tile * 32 + m;
    const bool act = pt < np;
    // lane half h owns embedding channels [16h, 16h+16): the channel itself (row c)
    // and its 3-band PE (rows 32 + 2(3c+f) + {0: sin, 1: cos}); angle doubling
    // from one sincos: sin 2x = 2 sin x cos x, cos 2x = (c - s)(c + s).
    const float* e = A.pts.emb + (act ? pt : 0) * kEmb + 16 * h;
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
      float4 e4 = act ? reinterpret_cast<const float4*>(e)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float ev[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = 16 * h + 4 * q + u;
        X[c * kPitch + m] = ev[u];
        float s0, c0;
        sincosf(ev[u], &s0, &c0);
        const float s1 = 2.f * s0 * c0, c1 = (c0 - s0) * (c0 + s0);
        const float s2 = 2.f * s1 * c1, c2 = (c1 - s1) * (c1 + s1);
        const int r0 = kEmb + 6 * c;
        X[(r0 + 0) * kPitch + m] = s0;
        X[(r0 + 1) * kPitch + m] = c0;
        X[(r0 + 2) * kPitch + m] = s1;
        X[(r0 + 3) * kPitch + m] = c1;
        X[(r0 + 4) * kPitch + m] = s2;
        X[(r0 + 5) * kPitch + m] = c2;
      }
    }
    bias_rows(X, kEmb * 7, lane);   // row 224 = 1 (bias column), 225 = 0
    wave_sync();
    f32x16 acc[8];
    zero_acc<8>(acc);
    mlp_layer<8>(acc, A.w.w1af, X, 113, lane);
    if (act) {
      float4* o = reinterpret_cast<float4*>(A.p1 + pt * kHid);
#pragma unroll
      for (int T = 0; T < 8; ++T)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[8 * T + 2 * q + h] = make_float4(acc[T][4 * q], acc[T][4 * q + 1], acc[T][4 * q + 2], acc[T][4 * q + 3]);
    }
    wave_sync();
  }
}

__global__ void __launch_bounds__(kAggBlock, 1) k_pairs(AggArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* X = lds_dyn + wid * kWaveLds;          // [kXRows][kPitch] layer input X^T
  const int m = lane & 31, h = lane >> 5, j = m >> 3, k = m & 7;
  const int K = A.s.K;
  const int64_t n = eff_n(A.s);
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
    const int64_t row = active ? sample_row(A.s, v) : 0;
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
      const int64_t drow = dir_row(A.s, row);
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

    // ---------------------------------------------------- layer-1 inputs -> X^T
    // 5-band PE of the 6-d rotated distance: rows 2(5c+f) + {sin, cos} (block1.0
    // columns 224..283); half h owns channels 3h..3h+2
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) {
      const int c = 3 * h + cc;
      const float dc = h ? dr6[3 + cc] : dr6[cc];
#pragma unroll 1
      for (int f = 0; f < 5; ++f) {
        float s, co;
        sincosf(dc * (float)(1 << f), &s, &co);
        const int r = 2 * (5 * c + f);
        X[r * kPitch + m] = s;
        X[(r + 1) * kPitch + m] = co;
      }
    }
    wave_sync();

    f32x16 acc[8];
    // ------------------------------------------------------------ block1: 284 -> 256 -> 256
    // accumulator starts at the gathered per-point partial P1[p] (bias included)
    if (valid) {
      const float4* pr = reinterpret_cast<const float4*>(A.p1 + prow * kHid);
#pragma unroll
      for (int T = 0; T < 8; ++T)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v4 = pr[8 * T + 2 * q + h];
          acc[T][4 * q] = v4.x;
          acc[T][4 * q + 1] = v4.y;
          acc[T][4 * q + 2] = v4.z;
          acc[T][4 * q + 3] = v4.w;
        }
    } else {
      zero_acc<8>(acc);
    }
    mlp_layer<8>(acc, A.w.w1bf, X, 30, lane);       // + W1[:, 224:284] . PE_5(dist)
    wave_sync();
    store_act<8>(acc, X, neg, lane);
    bias_rows(X, 256, lane);
    wave_sync();
    zero_acc<8>(acc);
    mlp_layer<8>(acc, A.w.w2f, X, 129, lane);
    wave_sync();
    store_act<8>(acc, X, neg, lane);
    // block3 inputs rows 256..263: colour(3), R.dir - R.v (3), <R.dir, R.v> (1), bias 1
    {
      const float dot = drot[0] * vrot[0] + drot[1] * vrot[1] + drot[2] * vrot[2];
      const float ex[8] = {col[0], col[1], col[2], drot[0] - vrot[0],
                           drot[1] - vrot[1], drot[2] - vrot[2], dot, 1.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) X[(256 + 2 * e + h) * kPitch + m] = h ? ex[2 * e + 1] : ex[2 * e];
    }
    wave_sync();
    // ------------------------------------------------------------ block3: 263 -> 256 -> 256
    zero_acc<8>(acc);
    mlp_layer<8>(acc, A.w.w3f, X, 132, lane);
    wave_sync();
    store_act<8>(acc, X, neg, lane);
    bias_rows(X, 256, lane);
    wave_sync();
    zero_acc<8>(acc);
    mlp_layer<8>(acc, A.w.w4f, X, 129, lane);
    wave_sync();
    store_act<8>(acc, X, neg, lane);                // h4 -> X^T rows 0..255
    if (h == 0) X[kWtRow * kPitch + m] = wt;        // per-pair blend weight
    wave_sync();
    // ------------------------------------------------------------ alpha branch + K sums
    // alpha_k = softplus(W_a . h4 + b_a - 1) per pair (both lane halves compute it;
    // W_a[n] is wave-uniform -> scalar loads)
    float pa = A.w.ba[0];
    const float* xc = X + m;
#pragma unroll 8
    for (int nn = 0; nn < kHid; ++nn) pa += A.w.wa[nn] * xc[nn * kPitch];
    const float alpha_k = A.w.act_super ? softplus(pa - 1.f) : fmaxf(pa, 0.f);
    const float alpha_s = xor8_sum(wt * alpha_k);   // point_aggregators.py:608-614
    // feature K-sum (point_aggregators.py:622-628): lane owns neurons lane + 64i,
    // written straight to hid[v] (256-B coalesced rows)
    float wk[kKN];
#pragma unroll
    for (int q = 0; q < kKN; ++q) wk[q] = 0.f;
#pragma unroll
    for (int s = 0; s < kSampPerWave; ++s) {
      const int src = s * 8;
      const bool act_s = __shfl((int)(active && samp_valid), src) != 0;
      const float al_s = __shfl(alpha_s, src);
      const int64_t vo = tile * kSampPerWave + s;   // sample-list index
      if (vo < n && lane == 0) A.vmask[vo] = act_s;
      if (!act_s) continue;
#pragma unroll
      for (int q = 0; q < kKN; ++q) wk[q] = X[kWtRow * kPitch + s * 8 + q];
      if (lane == 0) A.out_feat[vo * (kC + 1)] = al_s;
#pragma unroll
      for (int i = 0; i < kHid / 64; ++i) {
        const float* xr = X + (lane + 64 * i) * kPitch + s * 8;
        float f = 0.f;
#pragma unroll
        for (int q = 0; q < kKN; ++q) f += wk[q] * xr[q];
        A.hid[vo * kHid + lane + 64 * i] = f;
      }
    }
    wave_sync();
  }
}

// colour branch (point_aggregators.py:630-641): [f(256), PE_4(R.v)(24)] -> 128 x3.
__global__ void __launch_bounds__(kAggBlock, 1) k_color(AggArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* X = lds_dyn + wid * kWaveLds;   // [kXRows][kPitch]
  const int m = lane & 31, h = lane >> 5;
  const int64_t n = eff_n(A.s);
  const int64_t ntiles = cdiv(n, 32);
  const float neg = A.w.neg_slope;
  float Rw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t v0 = tile * 32;
    const int nv = (int)((n - v0) < 32 ? (n - v0) : 32);
    const int my_valid = (m < nv) ? A.vmask[v0 + m] : 0;
    const unsigned long long vbits = __ballot(my_valid != 0);   // bit q (and q+32): sample q valid
    // hid rows (one 1-KB row per wave instruction) -> X^T rows 0..255 (transpose)
#pragma unroll 4
    for (int q = 0; q < 32; ++q) {
      float4 f4 = ((vbits >> q) & 1ull) ? reinterpret_cast<const float4*>(A.hid + (v0 + q) * kHid)[lane]
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
      X[(4 * lane + 0) * kPitch + q] = f4.x;
      X[(4 * lane + 1) * kPitch + q] = f4.y;
      X[(4 * lane + 2) * kPitch + q] = f4.z;
      X[(4 * lane + 3) * kPitch + q] = f4.w;
    }
    // view-direction PE, ori dropped (point_aggregators.py:506-512): rows 256..279 =
    // sin block (c*4+f) then cos block; lane half h writes block h
    {
      float vrot[3] = {0.f, 0.f, 0.f};
      if (m < nv) {
        const int64_t row = sample_row(A.s, v0 + m);
        const int64_t drow = dir_row(A.s, row);
        const float vd[3] = {A.s.dirs[drow * 3], A.s.dirs[drow * 3 + 1], A.s.dirs[drow * 3 + 2]};
        mat3(Rw, vd, vrot);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          float s, co;
          sincosf(vrot[c] * (float)(1 << f), &s, &co);
          X[(kHid + 12 * h + 4 * c + f) * kPitch + m] = h ? co : s;
        }
    }
    bias_rows(X, kCin, lane);
    wave_sync();
    f32x16 acc[4];
    zero_acc<4>(acc);
    mlp_layer<4>(acc, A.w.wc1f, X, 141, lane);      // 280 inputs + bias column
    wave_sync();
    store_act<4>(acc, X, neg, lane);
    bias_rows(X, kC, lane);
    wave_sync();
    zero_acc<4>(acc);
    mlp_layer<4>(acc, A.w.wc2f, X, 65, lane);
    wave_sync();
    store_act<4>(acc, X, neg, lane);
    bias_rows(X, kC, lane);
    wave_sync();
    zero_acc<4>(acc);
    mlp_layer<4>(acc, A.w.wc3f, X, 65, lane);
    wave_sync();
    store_act<4>(acc, X, neg, lane);   // X^T rows 0..127 = colour features
    wave_sync();
    // write out_feat[v, 1..128]: lane = channel pair, loop over the 32 samples
    for (int q = 0; q < nv; ++q) {
      if (!((vbits >> q) & 1ull)) continue;   // samples without neighbours keep zeros
      float* o = A.out_feat + (v0 + q) * (kC + 1) + 1;
      o[lane] = X[lane * kPitch + q];
      o[64 + lane] = X[(64 + lane) * kPitch + q];
    }
    wave_sync();
  }
}

int launch(const AggArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAggLdsBytes));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_point_pre),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAggLdsBytes));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_color),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAggLdsBytes));
    attr = true;
  }
  hipLaunchKernelGGL(k_point_pre, dim3(grid_for(cdiv(a.pts.n, 32), 4, 256)), dim3(kAggBlock), kAggLdsBytes,
                     st, a);
  PNR_LAUNCH_CHECK();
  const int64_t tiles = cdiv(a.s.n_max, kSampPerWave);
  hipLaunchKernelGGL(k_pairs, dim3(grid_for(tiles, 4, 256)), dim3(kAggBlock), kAggLdsBytes, st, a);
  PNR_LAUNCH_CHECK();
  const int64_t ctiles = cdiv(a.s.n_max, 32);
  hipLaunchKernelGGL(k_color, dim3(grid_for(ctiles, 4, 256)), dim3(kAggBlock), kAggLdsBytes, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

static size_t scratch_need(int64_t n_max, int64_t n_points) {
  const int64_t nm = n_max > 0 ? n_max : 1;
  return ((size_t)nm * kHid + (size_t)cdiv(nm, 4) * 4 + (size_t)(n_points > 0 ? n_points : 1) * kHid) *
         sizeof(float);
}

static void carve(AggArgs& a, void* scratch, int64_t n_max) {
  const int64_t nm = n_max > 0 ? n_max : 1;
  a.hid = static_cast<float*>(scratch);
  a.vmask = reinterpret_cast<int32_t*>(a.hid + nm * kHid);
  a.p1 = reinterpret_cast<float*>(a.vmask) + cdiv(nm, 4) * 4;
}

int check_common(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w, float* out_feat,
                 float* scratch, size_t scratch_bytes) {
  PNR_CHECK_ARG(pts && s && w && out_feat, "aggregate: null pointer");
  PNR_CHECK_ARG(pts->xyz && pts->emb, "aggregate: point xyz/emb required");
  PNR_CHECK_ARG(s->sample_w && s->sample_p && s->dirs, "aggregate: sample arrays required");
  PNR_CHECK_ARG(s->K >= 1 && s->K <= kKN, "aggregate: K=%d unsupported (1..8)", s->K);
  PNR_CHECK_ARG(s->dir_div >= 1, "aggregate: dir_div must be >= 1");
  PNR_CHECK_ARG(w->w1af && w->w1bf && w->w2f && w->b2 && w->w3f && w->b3 && w->w4f && w->b4 && w->wa &&
                    w->ba && w->wc1f && w->bc1 && w->wc2f && w->bc2 && w->wc3f && w->bc3,
                "aggregate: null weight");
  PNR_CHECK_ARG(((uintptr_t)pts->emb & 15) == 0, "aggregate: emb must be 16-B aligned");
  PNR_CHECK_ARG(scratch && ((uintptr_t)scratch & 15) == 0, "aggregate: 16-B aligned scratch required");
  PNR_CHECK_ARG(pts->n > 0, "aggregate: empty point table");
  PNR_CHECK_ARG(scratch_bytes >= scratch_need(s->n_max, pts->n),
                "aggregate: scratch too small (%zu bytes for %lld samples, %lld points)", scratch_bytes,
                (long long)s->n_max, (long long)pts->n);
  return PNR_OK;
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_aggregate_scratch_bytes(int64_t n_max, int64_t n_points, size_t* out) {
  PNR_CHECK_ARG(out && n_max >= 0 && n_points >= 0, "aggregate_scratch_bytes: bad args");
  *out = scratch_need(n_max, n_points);
  return PNR_OK;
}

extern "C" int pnr_aggregate_fwd(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                 float* out_feat, float* out_weight, float* out_conf, void* scratch,
                                 size_t scratch_bytes, void* stream) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate: need pers or camera");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max);
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  return launch(a, as_stream(stream));
}

extern "C" int pnr_aggregate_fwd_masked(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                        const uint8_t* pair_mask, float* out_feat, float* out_weight,
                                        float* out_conf, void* scratch, size_t scratch_bytes,
                                        void* stream) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  PNR_CHECK_ARG(pair_mask, "aggregate_masked: null pair_mask");
  PNR_CHECK_ARG(pts->pers, "aggregate_masked: pers required");
  PNR_CHECK_ARG(s->pidx == nullptr, "aggregate_masked: pidx must be NULL (identity rows)");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max);
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = pair_mask;
  return launch(a, as_stream(stream));
}
