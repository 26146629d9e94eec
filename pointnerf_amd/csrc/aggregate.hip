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
// CDNA4 mapping (three launches):
// k_point_pre: P1[p] = W1[:, :224] . [emb_p, PE_3(emb_p)] + b1 once per point
//   (the point-only half of block1.0; 32 points per wave, 8 accumulator tiles).
// k_pairs: a 4-wave workgroup owns 64 (sample, neighbour) pairs = 8 samples x
//   K=8 and runs the rest of block1 and block3 as Y^T[256 x 64] = W . X^T on
//   v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chains; gfx950 has no TF32); wave w
//   owns neuron tiles {2w, 2w+1} for both 32-pair halves, the tile's X^T sits in
//   a quad-row LDS layout (b64 operand reads, b128 activation stores); gather,
//   weights, PE, alpha and the K-sums are fused around the GEMMs.
// k_color: one wave owns 32 valid samples and runs 280->128->128->128 on the
//   same MFMA machinery (4 accumulator tiles).
// Every weight matrix uses one A-operand "fragment" layout
// W_f[t][T][lane] = W[32T + (lane&31)][2t + (lane>>5)] (bias as an extra input
// column), so every weight load is a coalesced 256-B wave load from L2,
// software-pipelined a few k-steps ahead.
#include "agg_common.h"


namespace pnr {

constexpr int kPitch = 33;         // LDS row pitch (floats) of X^T[k][32 + 1]
constexpr int kXRows = 296;        // >= 286 layer-1 inputs + bias, + x prefetch overrun
constexpr int kWaveLds = kXRows * kPitch;  // floats per wave slice
constexpr size_t kAggLdsBytes = (size_t)4 * kWaveLds * sizeof(float);
constexpr int kPD = 4;             // weight prefetch depth in k-steps of mlp_layer
constexpr int kPackPad = 8;        // zero k-steps padded onto every packed weight matrix
                                   // (>= every prefetch depth, so prefetch never overruns)

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
  pnr_agg_saved sv;           // training forward: activations kept for the backward
  const int32_t* run_if = nullptr;   // set: the kernel runs only when *run_if != 0 (the guarded h2 forward's fallback)
};

// The guarded fallback: every workgroup leaves at once unless the h2 range flag is raised.
__device__ __forceinline__ bool skip_run(const AggArgs& A) { return A.run_if && *A.run_if == 0; }

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

// NT tiles of this wave out of NTOT tiles per k-step in the packed layout
// (p already points at this wave's first tile).
template <int NT, int NTOT = NT>
__device__ __forceinline__ void load_w(float (&a)[NT], const float* __restrict__ p, int t) {
#pragma unroll
  for (int T = 0; T < NT; ++T) a[T] = p[(t * NTOT + T) * 64];
}

template <int NT>
__device__ __forceinline__ void mfma_step(f32x16 (&acc)[NT], const float (&a)[NT], float x) {
#pragma unroll
  for (int T = 0; T < NT; ++T) acc[T] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[T], x, acc[T], 0, 0, 0);
}

// Y^T += W . X^T over nsteps k-steps (2 k-values each); X^T from the wave's
// LDS slice, W in fragment layout, weight loads issued kPD steps ahead.
template <int NT, int NTOT = NT>
__device__ __forceinline__ void mlp_layer(f32x16 (&acc)[NT], const float* __restrict__ wf,
                                          const float* X, int nsteps, int lane) {
  const int m = lane & 31, h = lane >> 5;
  const float* p = wf + lane;
  const float* xr = X + h * kPitch + m;
  float a0[NT], a1[NT], a2[NT], a3[NT];
  load_w<NT, NTOT>(a0, p, 0);
  load_w<NT, NTOT>(a1, p, 1);
  load_w<NT, NTOT>(a2, p, 2);
  load_w<NT, NTOT>(a3, p, 3);
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
    load_w<NT, NTOT>(a0, p, t + 4);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step<NT>(acc, a1, x1);
    load_w<NT, NTOT>(a1, p, t + 5);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step<NT>(acc, a2, x2);
    load_w<NT, NTOT>(a2, p, t + 6);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step<NT>(acc, a3, x3);
    load_w<NT, NTOT>(a3, p, t + 7);
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
__device__ __forceinline__ void store_act(const f32x16 (&acc)[NT], float* X, float s, int lane, int T0 = 0) {
  const int m = lane & 31, h = lane >> 5;
#pragma unroll
  for (int T = 0; T < NT; ++T)
#pragma unroll
    for (int r = 0; r < 16; ++r) X[(32 * (T0 + T) + acc_row(r, h)) * kPitch + m] = lrelu(acc[T][r], s);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-point half of block1.0 (exact split of the 284-input Linear): the
// embedding and its 3-band PE depend only on the point, so
// P1[p] = W1[:, :224] . [emb_p, PE_3(emb_p)] + b1 is evaluated once per point
// and gathered per pair instead of being recomputed for every (sample,
// neighbour) pair that references the point (~22x reuse at 2 M points).
__global__ void __launch_bounds__(kAggBlock, 1) k_point_pre(AggArgs A) {
  if (skip_run(A)) return;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* X = lds_dyn + wid * kWaveLds;
  const int m = lane & 31, h = lane >> 5;
  const int64_t np = p1_rows(A.pts);   // P1 rows
  const int64_t ntiles = cdiv(np, 32);
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t pt = tile * 32 + m;                         // P1 row
    const bool act = pt < np;
    const int64_t prow = act ? (A.pts.used ? (int64_t)A.pts.used[pt] : pt) : 0;   // point row
    // lane half h owns embedding channels [16h, 16h+16): the channel itself (row c)
    // and its 3-band PE (rows 32 + 2(3c+f) + {0: sin, 1: cos}); angle doubling
    // from one sincos: sin 2x = 2 sin x cos x, cos 2x = (c - s)(c + s).
    const float* e = A.pts.emb + prow * kEmb + 16 * h;
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

// Post-activation accumulator tiles -> [row][ld] global rows (training saves);
// lane column m = row offset, rows of tile T at columns 32T + 8q + 4h.
template <int NT>
__device__ __forceinline__ void save_rows(const f32x16 (&acc)[NT], float* dst, int64_t row, int ld, float s,
                                          int lane, int T0 = 0) {
  const int h = lane >> 5;
#pragma unroll
  for (int T = 0; T < NT; ++T)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(dst + row * ld + 32 * (T0 + T) + 8 * q + 4 * h) =
          make_float4(lrelu(acc[T][4 * q], s), lrelu(acc[T][4 * q + 1], s), lrelu(acc[T][4 * q + 2], s),
                      lrelu(acc[T][4 * q + 3], s));
}



// ---------------------------------------------------------------------------
// k_pairs: one workgroup (4 waves) owns a tile of 64 pairs = 8 samples x K=8.
// Wave w computes neuron tiles {2w, 2w+1} for both 32-pair halves of the tile
// (4 accumulator tiles, 64 VGPRs), so every 256-B weight fragment fetched
// from L2 feeds two MFMAs and every LDS B-operand read feeds two.  Two
// workgroups per CU (2 waves per SIMD) overlap one tile's gather / PE / tail
// with the other's MFMA stream.
//
// LDS layout of the tile's layer input X^T (quad rows): neuron / input row n
// of pair column c lives at (n >> 2) * kQP + 4c + perm(n & 3) with
// perm = {0, 2, 1, 3}.  Then
//   * the MFMA B operand of k-steps t, t+1 (rows 2t+h, 2t+2+h for lane half
//     h) is ONE ds_read_b64 at (t >> 1) * kQP + 4c + 2h (t even), and
//   * an accumulator quad (rows 8q + 4h + 0..3 of a tile) is ONE
//     ds_write_b128,
// both conflict-free; kQP = 260 keeps the tail's row-strided b128 reads
// conflict-free too.
constexpr int kTP = 64;                 // pairs per tile
constexpr int kTS = kTP / kKN;          // samples per tile
constexpr int kQP = 4 * kTP + 4;        // floats per quad row
constexpr int kQD = 4;                  // k_pairs weight prefetch depth (k-steps)
constexpr int kQRows = (264 + 2 * kQD + 3) / 4;  // layer-3 input rows + x prefetch overrun
constexpr int kPairsLdsFloats = kQRows * kQP + kTP /*wt*/ + 4 * kTP /*alpha parts*/ + kTS /*flags*/ +
                                8 * kTP /*block3 extras*/;
static_assert(kQD <= kPackPad && kPD <= kPackPad, "prefetch deeper than the packed padding");
constexpr size_t kPairsLdsBytes = (size_t)kPairsLdsFloats * sizeof(float);

__device__ __forceinline__ constexpr int qperm(int i) { return ((i & 1) << 1) | (i >> 1); }
__device__ __forceinline__ constexpr int qaddr(int n, int c) { return (n >> 2) * kQP + 4 * c + qperm(n & 3); }

// Issue the first kQD k-steps of a layer's weight fragments into the ring.
// Called as soon as the previous layer's last MFMA is issued (or before the
// gather for layer 1), so the L2 latency hides behind the layer boundary.
template <int NT, int NTOT = 8>
__device__ __forceinline__ void prime_q(float (&a)[kQD][NT], const float* __restrict__ wf, int lane) {
#pragma unroll
  for (int d = 0; d < kQD; ++d) load_w<NT, NTOT>(a[d], wf + lane, d);
}

// Y^T += W . X^T for NT neuron tiles x PT 32-pair halves over nsteps k-steps.
// Weight fragments kQD steps ahead in a register ring (primed by prime_q);
// the next kQD steps' B operands read from LDS one iteration ahead (kQD/2 b64
// per half).
template <int NT, int PT, int NTOT = 8>
__device__ __forceinline__ void mlp_layer_q(f32x16 (&acc)[PT * NT], float (&a)[kQD][NT],
                                            const float* __restrict__ wf, const float* X, int nsteps,
                                            int lane) {
  constexpr int D = kQD;
  const int c = lane & 31, h = lane >> 5;
  const float* p = wf + lane;
  const float* xr = X + 4 * c + 2 * h;
  float2 x[D / 2][PT];
#pragma unroll
  for (int i = 0; i < D / 2; ++i)
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) x[i][pt] = *reinterpret_cast<const float2*>(xr + 128 * pt + i * kQP);
  auto step = [&](const float (&w)[NT], const float2 (&xx)[PT], bool hi) {
#pragma unroll
    for (int pt = 0; pt < PT; ++pt)
#pragma unroll
      for (int T = 0; T < NT; ++T)
        acc[pt * NT + T] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[T], hi ? xx[pt].y : xx[pt].x,
                                                                acc[pt * NT + T], 0, 0, 0);
  };
  int t = 0;
#pragma unroll 1
  for (; t + D <= nsteps; t += D) {
    const float* xn = xr + ((t + D) >> 1) * kQP;
    float2 y[D / 2][PT];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      step(a[d], x[d >> 1], d & 1);
      if (d == 0) {
#pragma unroll
        for (int i = 0; i < D / 2; ++i)
#pragma unroll
          for (int pt = 0; pt < PT; ++pt) y[i][pt] = *reinterpret_cast<const float2*>(xn + 128 * pt + i * kQP);
      }
      load_w<NT, NTOT>(a[d], p, t + D + d);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < D / 2; ++i)
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) x[i][pt] = y[i][pt];
  }
  const int rem = nsteps - t;  // 0..D-1
#pragma unroll
  for (int d = 0; d < D - 1; ++d)
    if (rem > d) step(a[d], x[d >> 1], d & 1);
}

// Activated accumulators -> quad rows (one b128 per accumulator quad).
template <int NT, int PT>
__device__ __forceinline__ void store_act_q(const f32x16 (&acc)[PT * NT], float* X, float s, int lane,
                                            int T0) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt)
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x16& v = acc[pt * NT + T];
        *reinterpret_cast<float4*>(X + (8 * (T0 + T) + 2 * q + h) * kQP + 4 * (32 * pt + c)) =
            make_float4(lrelu(v[4 * q], s), lrelu(v[4 * q + 2], s), lrelu(v[4 * q + 1], s),
                        lrelu(v[4 * q + 3], s));
      }
}

// X^T row kin = 1 (bias column of the packed weights), row kin + 1 = 0 when
// the k-step is shared; one wave, lane = pair column.
__device__ __forceinline__ void bias_rows_q(float* X, int kin, int lane) {
  X[qaddr(kin, lane)] = 1.f;
  if ((kin & 1) == 0) X[qaddr(kin + 1, lane)] = 0.f;
}

constexpr int kPairWaves = 4;
constexpr int kNTW = 8 / kPairWaves;   // neuron tiles per wave
constexpr int kPTW = kTP / 32;         // 32-pair halves per tile

// Training save of a colour-branch tile (output tile T0, PT sample halves) -> dst[v][128].
template <int PT>
__device__ __forceinline__ void save_cols(const f32x16 (&acc)[PT], float* dst, int64_t v0, int64_t n, float s,
                                          int lane, int T0) {
  const int c = lane & 31;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    const int64_t v = v0 + 32 * pt + c;
    if (v >= n) continue;
    f32x16 one[1] = {acc[pt]};
    save_rows<1>(one, dst, v, kC, s, lane, T0);
  }
}

// Training save of a tile's post-activation quad (both halves) -> dst[pair][256].
// Also keeps the LeakyReLU derivative as bits: mask[pair][16 * layer + 2T + h]
// bit r = (pre-activation of accumulator register r of tile T, lane half h > 0).
template <int NT, int PT>
__device__ __forceinline__ void save_pairs_q(const f32x16 (&acc)[PT * NT], float* dst, uint16_t* mask,
                                             int layer, int64_t tile, int64_t n, float s, int lane, int T0) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    const int col = 32 * pt + c;
    if (tile * kTS + (col >> 3) >= n) continue;
    f32x16 one[NT];
#pragma unroll
    for (int T = 0; T < NT; ++T) one[T] = acc[pt * NT + T];
    save_rows<NT>(one, dst, tile * kTP + col, kHid, s, lane, T0);
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      unsigned bits = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) bits |= (one[T][r] > 0.f ? 1u : 0u) << r;
      mask[(tile * kTP + col) * 64 + 16 * layer + 2 * (T0 + T) + h] = (uint16_t)bits;
    }
  }
}

constexpr int kPairSub = 1;   // tiles per workgroup sharing barriers (and weight-fragment fetches)

template <bool TRAIN>
__global__ void __launch_bounds__(64 * kPairWaves * kPairSub, 2 / kPairSub) k_pairs(AggArgs A) {
  if (skip_run(A)) return;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  const int sub = (threadIdx.x >> 6) / kPairWaves;   // which of the workgroup's tiles
  float* X = lds_dyn + sub * kPairsLdsFloats;  // quad rows [kQRows][kQP]
  float* wtL = X + kQRows * kQP;               // [64] per-pair blend weight w_k * conf_k
  float* apart = wtL + kTP;                    // [4][64] alpha partial dots
  int* sflag = reinterpret_cast<int*>(apart + 4 * kTP);  // [8] sample has a valid neighbour
  float* exL = apart + 4 * kTP + kTS;          // [8][64] block3.0 extra inputs, parked from the gather
  const int lane = threadIdx.x & 63, wid = (threadIdx.x >> 6) % kPairWaves;
  const int c = lane & 31, h = lane >> 5;
  const int j = lane >> 3, k = lane & 7;       // gather layout: lane = pair column
  const int T0 = wid * kNTW;
  const int K = A.s.K;
  const int64_t n = eff_n(A.s);
  const int64_t ntiles = cdiv(n, kTS);
  const int64_t ngroups = cdiv(ntiles, kPairSub);
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
  const float* w1b = A.w.w1bf + T0 * 64;
  const float* w2 = A.w.w2f + T0 * 64;
  const float* w3 = A.w.w3f + T0 * 64;
  const float* w4 = A.w.w4f + T0 * 64;
  float ring[kQD][kNTW];
  prime_q<kNTW>(ring, w1b, lane);

  for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t tile = grp * kPairSub + sub;   // past ntiles: every pair inactive
    // ------------------------------------------------------------ gather (neural_points.py:788-799)
    const int64_t v = tile * kTS + j;
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
    // this wave's neuron tiles of the gathered per-point block1.0 partial P1
    // (bias included) for the pairs of both halves (MFMA layout: column c)
    f32x16 acc[kPTW * kNTW];
#pragma unroll
    for (int pt = 0; pt < kPTW; ++pt) {
      const int64_t pr_pt = __shfl(prow, 32 * pt + c);
      const bool v_pt = __shfl((int)valid, 32 * pt + c) != 0;
      if (v_pt) {
        const int64_t p1r = A.pts.used_map ? (int64_t)A.pts.used_map[pr_pt] : pr_pt;
        const float4* pr = reinterpret_cast<const float4*>(A.p1 + p1r * kHid);
#pragma unroll
        for (int T = 0; T < kNTW; ++T)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v4 = pr[8 * (T0 + T) + 2 * q + h];
            acc[pt * kNTW + T][4 * q] = v4.x;
            acc[pt * kNTW + T][4 * q + 1] = v4.y;
            acc[pt * kNTW + T][4 * q + 2] = v4.z;
            acc[pt * kNTW + T][4 * q + 3] = v4.w;
          }
      } else {
#pragma unroll
        for (int T = 0; T < kNTW; ++T) acc[pt * kNTW + T] = (f32x16){0.f};
      }
    }
    float sw[3] = {0.f, 0.f, 0.f}, sp[3] = {0.f, 0.f, 0.f}, vd[3] = {0.f, 0.f, 0.f};
    int64_t drow = 0;
    if (active) {
      drow = dir_row(A.s, row);
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
        pair_pers(A.pts, A.s, drow, pw, cam_c, cam_R, pp);
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
    // rotated distance / direction inputs (point_aggregators.py:506, 526, 566-570)
    float dr6[6];
    mat3(Rw, d6, dr6);
    dr6[3] = d6[3];
    dr6[4] = d6[4];
    dr6[5] = d6[5];
    float vrot[3], drot[3];
    mat3(Rw, vd, vrot);
    mat3(Rw, pdir, drot);
    if (A.pts.rw2c) {   // per-point Rw2c (agg_common.h rot_point)
      rot_point(A.pts.rw2c, prow, d6, dr6);
      rot_point(A.pts.rw2c, prow, pdir, drot);
      rot_point(A.pts.rw2c, active ? slot0_point(A.s, row) : 0, vd, vrot);
    }
    if (wid == 0) {
      // block3 inputs 256..263: colour(3), R.dir - R.v (3), <R.dir, R.v> (1), bias 1
      const float dot = drot[0] * vrot[0] + drot[1] * vrot[1] + drot[2] * vrot[2];
      const float ex[8] = {col[0], col[1], col[2], drot[0] - vrot[0],
                           drot[1] - vrot[1], drot[2] - vrot[2], dot, 1.f};
#pragma unroll
      for (int e = 0; e < 8; ++e) exL[e * kTP + lane] = ex[e];
      if (TRAIN && active) {
#pragma unroll
        for (int e = 0; e < 8; ++e) A.sv.x3e[(tile * kTP + lane) * 32 + e] = ex[e];
        float4* z = reinterpret_cast<float4*>(A.sv.x3e + (tile * kTP + lane) * 32 + 8);
#pragma unroll
        for (int e = 0; e < 6; ++e) z[e] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (active && k < K) {
        if (A.out_weight) A.out_weight[row * K + k] = wn;
        if (A.out_conf) A.out_conf[row * K + k] = confc;
      }
      wtL[lane] = wt;
      if (k == 0) sflag[j] = active && samp_valid;
      if (TRAIN && active) {
        const int64_t pr = tile * kTP + lane;
        A.sv.wt[pr] = wt;
        A.sv.wn[pr] = wn;
        A.sv.prow[pr] = valid ? (int32_t)prow : -1;
      }
    }
    // 5-band PE of the 6-d rotated distance -> rows 2e + {0: sin, 1: cos},
    // e = 5 ch + f (block1.0 columns 224..283); wave w owns e = w (mod 4)
    {
#pragma unroll 1
      for (int e = wid; e < 30; e += kPairWaves) {
        const int ch = e / 5, f = e - 5 * ch;
        float dc = dr6[0];
        dc = ch == 1 ? dr6[1] : dc;
        dc = ch == 2 ? dr6[2] : dc;
        dc = ch == 3 ? dr6[3] : dc;
        dc = ch == 4 ? dr6[4] : dc;
        dc = ch == 5 ? dr6[5] : dc;
        float sn, cs;
        sincosf(dc * (float)(1 << f), &sn, &cs);
        X[qaddr(2 * e, lane)] = sn;
        X[qaddr(2 * e + 1, lane)] = cs;
        if (TRAIN && active) {
          float* pe = A.sv.pe5 + (tile * kTP + lane) * 64 + 2 * e;
          pe[0] = sn;
          pe[1] = cs;
        }
      }
    }
    if (TRAIN && active && wid == kPairWaves - 1)   // pe5 rows are padded to 64 for the dW GEMM
      *reinterpret_cast<float4*>(A.sv.pe5 + (tile * kTP + lane) * 64 + 60) = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    // ------------------------------------------------------------ block1: 284 -> 256 -> 256
    mlp_layer_q<kNTW, kPTW>(acc, ring, w1b, X, 30, lane);   // + W1[:, 224:284] . PE_5(dist)
    prime_q<kNTW>(ring, w2, lane);
    __syncthreads();
    store_act_q<kNTW, kPTW>(acc, X, neg, lane, T0);
    if (TRAIN) save_pairs_q<kNTW, kPTW>(acc, A.sv.h1, A.sv.mask, 0, tile, n, neg, lane, T0);
    if (wid == 0) bias_rows_q(X, 256, lane);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPTW * kNTW; ++i) acc[i] = (f32x16){0.f};
    mlp_layer_q<kNTW, kPTW>(acc, ring, w2, X, 129, lane);
    prime_q<kNTW>(ring, w3, lane);
    __syncthreads();
    store_act_q<kNTW, kPTW>(acc, X, neg, lane, T0);
    if (TRAIN) save_pairs_q<kNTW, kPTW>(acc, A.sv.h2, A.sv.mask, 1, tile, n, neg, lane, T0);
    // block3 inputs rows 256..263 (parked in exL by the gather)
    if (wid == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) X[qaddr(256 + e, lane)] = exL[e * kTP + lane];
    }
    __syncthreads();
    // ------------------------------------------------------------ block3: 263 -> 256 -> 256
#pragma unroll
    for (int i = 0; i < kPTW * kNTW; ++i) acc[i] = (f32x16){0.f};
    mlp_layer_q<kNTW, kPTW>(acc, ring, w3, X, 132, lane);
    prime_q<kNTW>(ring, w4, lane);
    __syncthreads();
    store_act_q<kNTW, kPTW>(acc, X, neg, lane, T0);
    if (TRAIN) save_pairs_q<kNTW, kPTW>(acc, A.sv.h3, A.sv.mask, 2, tile, n, neg, lane, T0);
    if (wid == 0) bias_rows_q(X, 256, lane);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPTW * kNTW; ++i) acc[i] = (f32x16){0.f};
    mlp_layer_q<kNTW, kPTW>(acc, ring, w4, X, 129, lane);
    prime_q<kNTW>(ring, w1b, lane);                   // the next tile's layer 1
    if (TRAIN) save_pairs_q<kNTW, kPTW>(acc, A.sv.h4, A.sv.mask, 3, tile, n, neg, lane, T0);
    {
      // ---------------------------------------------------------- alpha + K sums from registers
      // h4 = lrelu(acc) never goes to LDS.  alpha: each lane dots its 32 rows of
      // the wave's 64 neurons with W_a, the two lane halves and the 4 waves are
      // summed through LDS.  K sums (point_aggregators.py:622-628): the 8 pairs
      // of a sample are 8 adjacent lanes; a 3-round DPP reduce-scatter (row
      // half-mirror, quad xor 2, quad xor 1) leaves lane i of the 8 with the
      // sums of accumulator registers 2i, 2i+1 = two adjacent neurons.
      float pa_part[kPTW] = {0.f, 0.f};
#pragma unroll
      for (int pt = 0; pt < kPTW; ++pt) {
        const float wtp = wtL[32 * pt + c];
        const int sj = (32 * pt + c) >> 3;
        const int64_t vo = tile * kTS + sj;
        const bool wr = vo < n && sflag[sj];
        const int i8 = c & 7;
#pragma unroll
        for (int T = 0; T < kNTW; ++T) {
          float v[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float hv = lrelu(acc[pt * kNTW + T][r], neg);
            pa_part[pt] += A.w.wa[32 * (T0 + T) + acc_row(r, h)] * hv;
            v[r] = wtp * hv;
          }
          float w8[8], w4[4], w2[2];
          const bool b2 = (i8 & 4) != 0, b1 = (i8 & 2) != 0, b0 = (i8 & 1) != 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float send = b2 ? v[q] : v[q + 8];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send),
                                                                                  0x141, 0xf, 0xf, false));
            w8[q] = (b2 ? v[q + 8] : v[q]) + recv;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float send = b1 ? w8[q] : w8[q + 4];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send),
                                                                                  0x4E, 0xf, 0xf, false));
            w4[q] = (b1 ? w8[q + 4] : w8[q]) + recv;
          }
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float send = b0 ? w4[q] : w4[q + 2];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send),
                                                                                  0xB1, 0xf, 0xf, false));
            w2[q] = (b0 ? w4[q + 2] : w4[q]) + recv;
          }
          // registers 2 i8, 2 i8 + 1 -> rows (2 i8 & 3) + 8 (i8 >> 1) + 4h (+1)
          if (wr)
            *reinterpret_cast<float2*>(A.hid + vo * kHid + 32 * (T0 + T) + ((2 * i8) & 3) + 8 * (i8 >> 1) + 4 * h) =
                make_float2(w2[0], w2[1]);
        }
        pa_part[pt] += __shfl_xor(pa_part[pt], 32);
      }
      if (h == 0) {
        apart[wid * kTP + c] = pa_part[0];
        apart[wid * kTP + 32 + c] = pa_part[1];
      }
      __syncthreads();
      if (wid == 0) {
        const float pa = apart[lane] + apart[kTP + lane] + apart[2 * kTP + lane] + apart[3 * kTP + lane] +
                         A.w.ba[0];
        const float alpha_k = A.w.act_super ? softplus(pa - 1.f) : fmaxf(pa, 0.f);
        const float alpha_s = xor8_sum(wtL[lane] * alpha_k);   // point_aggregators.py:608-614
        const int64_t vo = tile * kTS + j;
        if (TRAIN && vo < n) A.sv.pa[tile * kTP + lane] = pa;
        if (k == 0 && vo < n) {
          A.vmask[vo] = sflag[j];
          if (sflag[j]) A.out_feat[vo * (kC + 1)] = alpha_s;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_color: the colour branch 280 -> 128 -> 128 -> 128 (LeakyReLU each,
// point_aggregators.py:630-638) for 64 valid samples per 4-wave workgroup, on
// the same quad-row LDS pipeline as k_pairs: wave w owns output tile w for
// both 32-sample halves (2 MFMAs per weight fragment).  Input rows: the
// K-summed features hid (transposed from [sample][256] rows with one float4
// per lane), the 4-band view-direction PE (sin block, cos block, :506-512)
// and the bias row.
constexpr int kColWaves = 4;
constexpr int kColQRows = (282 + 2 * kQD + 3) / 4;
constexpr size_t kColLdsBytes = (size_t)kColQRows * kQP * sizeof(float);

template <bool TRAIN>
__global__ void __launch_bounds__(64 * kColWaves, 2) k_color(AggArgs A) {
  if (skip_run(A)) return;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  float* X = lds_dyn;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int64_t n = eff_n(A.s);
  const int64_t ntiles = cdiv(n, kTP);
  const float neg = A.w.neg_slope;
  float Rw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
  const float* w1 = A.w.wc1f + wid * 64;
  const float* w2 = A.w.wc2f + wid * 64;
  const float* w3 = A.w.wc3f + wid * 64;
  float ring[kQD][1];
  prime_q<1, 4>(ring, w1, lane);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t v0 = tile * kTP;
    // hid rows -> X^T rows 0..255 (wave w: samples 16w..16w+15, lane = neuron quad)
    for (int i = 0; i < kTP / kColWaves; ++i) {
      const int col = wid * (kTP / kColWaves) + i;
      const int64_t v = v0 + col;
      const bool ok = v < n && A.vmask[v] != 0;
      const float4 f4 = ok ? reinterpret_cast<const float4*>(A.hid + v * kHid)[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(X + lane * kQP + 4 * col) = make_float4(f4.x, f4.z, f4.y, f4.w);
    }
    // view-direction PE (ori dropped): rows 256 + 4ch + f = sin, 268 + 4ch + f = cos;
    // wave ch < 3 owns channel ch, wave 3 the bias rows 280 (1) / 281 (0); lane = sample
    {
      const int64_t v = v0 + lane;
      if (wid < 3) {
        float vrot[3] = {0.f, 0.f, 0.f};
        if (v < n) {
          const int64_t row = sample_row(A.s, v);
          const int64_t drow = dir_row(A.s, row);
          const float vd[3] = {A.s.dirs[drow * 3], A.s.dirs[drow * 3 + 1], A.s.dirs[drow * 3 + 2]};
          mat3(Rw, vd, vrot);
          if (A.pts.rw2c) rot_point(A.pts.rw2c, slot0_point(A.s, row), vd, vrot);
        }
        const float x = wid == 0 ? vrot[0] : (wid == 1 ? vrot[1] : vrot[2]);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          float sn, cs;
          sincosf(x * (float)(1 << f), &sn, &cs);
          X[qaddr(kHid + 4 * wid + f, lane)] = sn;
          X[qaddr(kHid + 12 + 4 * wid + f, lane)] = cs;
          if (TRAIN && v < n) {
            A.sv.vpe[v * 24 + 4 * wid + f] = sn;
            A.sv.vpe[v * 24 + 12 + 4 * wid + f] = cs;
          }
        }
      } else {
        X[qaddr(kCin, lane)] = 1.f;
        X[qaddr(kCin + 1, lane)] = 0.f;
      }
    }
    __syncthreads();
    f32x16 acc[2];
    acc[0] = acc[1] = (f32x16){0.f};
    mlp_layer_q<1, 2, 4>(acc, ring, w1, X, 141, lane);   // 280 inputs + bias column
    prime_q<1, 4>(ring, w2, lane);
    __syncthreads();
    store_act_q<1, 2>(acc, X, neg, lane, wid);
    if (wid == 0) bias_rows_q(X, kC, lane);
    if (TRAIN) save_cols<2>(acc, A.sv.hc1, v0, n, neg, lane, wid);
    __syncthreads();
    acc[0] = acc[1] = (f32x16){0.f};
    mlp_layer_q<1, 2, 4>(acc, ring, w2, X, 65, lane);
    prime_q<1, 4>(ring, w3, lane);
    __syncthreads();
    store_act_q<1, 2>(acc, X, neg, lane, wid);
    if (wid == 0) bias_rows_q(X, kC, lane);
    if (TRAIN) save_cols<2>(acc, A.sv.hc2, v0, n, neg, lane, wid);
    __syncthreads();
    acc[0] = acc[1] = (f32x16){0.f};
    mlp_layer_q<1, 2, 4>(acc, ring, w3, X, 65, lane);
    prime_q<1, 4>(ring, w1, lane);   // the next tile
    if (TRAIN) save_cols<2>(acc, A.sv.hc3, v0, n, neg, lane, wid);
    // out_feat[v, 1 + n] (valid samples only; the others keep their zeros)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const int64_t v = v0 + 32 * pt + c;
      if (v >= n || A.vmask[v] == 0) continue;
      float* o = A.out_feat + v * (kC + 1) + 1 + 32 * wid + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) o[8 * q + i] = lrelu(acc[pt][4 * q + i], neg);
    }
    __syncthreads();
  }
}

constexpr int kStagePre = 1, kStagePairs = 2, kStageColor = 4, kStageAll = 7;

template <bool TRAIN>
int launch_t(const AggArgs& a, hipStream_t st, int stages = kStageAll) {
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs<TRAIN>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kPairsLdsBytes * kPairSub)));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_point_pre),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAggLdsBytes));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_color<TRAIN>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kColLdsBytes));
    attr = true;
  }
  if ((stages & kStagePre) && !a.pts.p1_ready) {
    hipLaunchKernelGGL(k_point_pre, dim3(grid_for(cdiv(a.pts.used ? a.pts.n_used : a.pts.n, 32), 4, 256)),
                       dim3(kAggBlock), kAggLdsBytes, st, a);
    PNR_LAUNCH_CHECK();
  }
  if (stages & kStagePairs) {
    const int64_t tiles = cdiv(a.s.n_max, kTS);
    hipLaunchKernelGGL(k_pairs<TRAIN>, dim3(grid_for(cdiv(tiles, kPairSub), 1, 256 * 2 / kPairSub)),
                       dim3(64 * kPairWaves * kPairSub), kPairsLdsBytes * kPairSub, st, a);
    PNR_LAUNCH_CHECK();
  }
  if (stages & kStageColor) {
    const int64_t ctiles = cdiv(a.s.n_max, kTP);
    hipLaunchKernelGGL(k_color<TRAIN>, dim3(grid_for(ctiles, 1, 256 * 2)), dim3(64 * kColWaves), kColLdsBytes, st,
                       a);
    PNR_LAUNCH_CHECK();
  }
  return PNR_OK;
}

int launch(const AggArgs& a, hipStream_t st, bool train) {
  return train ? launch_t<true>(a, st) : launch_t<false>(a, st);
}

// ===========================================================================
// Backward.  k_pairs_bwd mirrors k_pairs: a 4-wave workgroup
// owns 64 pairs, wave w owns neuron tiles {2w, 2w+1} of both halves, and the
// three dX GEMMs (block3.2^T, block3.0[:, :256]^T, block1.2^T) run on the same
// quad-row LDS pipeline with transposed, fragment-packed weights.  The dW
// GEMMs (sum over pairs) are plain GEMMs and left to the caller (hipBLASLt).
struct BwdArgs {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp w;
  pnr_mlp_bwd wb;
  pnr_agg_saved sv;
  const float* d_feat;   // [n,129]
  const float* d_hid;    // [n,256]
  float* dz[4];          // dz1..dz4 [n*8,256]
  float* dpa;            // [n*8]
  float* d_p1;           // [N,256] (+=)
  float* d_color;        // [N,3] (+=) or null
  float* d_dir;          // [N,3] (+=) or null
  float* d_conf;         // [N]   (+=) or null
  const void* wx[3];     // k_pairs_bwd<1>: frag_pack_x3 of W4^T, W3[:, :256]^T, W2^T;
                         // k_pairs_bwd<2>: the three pnr_pack_bwd_h2 packs
  const float* wxs;      // k_pairs_bwd<2>: device [3], the packs' scales 2^(s - 11)
};

constexpr int kBwdLdsFloats = 66 * kQP + 4 * kTP /*dot parts*/ + 4 * 7 * kTP /*extras parts*/;
constexpr size_t kBwdLdsBytes = (size_t)kBwdLdsFloats * sizeof(float);

// max |v| over a wave's lanes into an LDS slot (float bits compared as unsigned:
// a NaN's bits exceed every finite and infinite value, so it propagates).
__device__ __forceinline__ void wave_absmax_to(unsigned* slot, unsigned mb) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
  if ((threadIdx.x & 63) == 0 && mb) atomicMax(slot, mb);
}

// acc-layout float4 of a [pair][256] array for (half pt, tile T, quad q)
__device__ __forceinline__ float4 ld_q(const float* base, int64_t pair, int T, int q, int h) {
  return *reinterpret_cast<const float4*>(base + pair * kHid + 32 * T + 8 * q + 4 * h);
}

// Raw (no activation) accumulator quads -> quad rows.
template <int NT, int PT>
__device__ __forceinline__ void store_q(const f32x16 (&acc)[PT * NT], float* X, int lane, int T0) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt)
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x16& v = acc[pt * NT + T];
        *reinterpret_cast<float4*>(X + (8 * (T0 + T) + 2 * q + h) * kQP + 4 * (32 * pt + c)) =
            make_float4(v[4 * q], v[4 * q + 2], v[4 * q + 1], v[4 * q + 3]);
      }
}

// dz = dh * lrelu'(h) with h the saved post-activation (h > 0 <=> z > 0 for
// slope >= 0); writes dz back into acc and to dst rows of active pairs.
template <int NT, int PT>
__device__ __forceinline__ void lrelu_bwd_q(f32x16 (&acc)[PT * NT], const float* h_saved, float* dst,
                                            int64_t tile, int64_t n, float slope, int lane, int T0,
                                            unsigned* amx = nullptr) {
  const int c = lane & 31, h = lane >> 5;
  unsigned mb = 0;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    const int col = 32 * pt + c;
    const bool act = tile * kTS + (col >> 3) < n;
    const int64_t pair = tile * kTP + col;
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x16& v = acc[pt * NT + T];
        float4 hv = act ? ld_q(h_saved, pair, T0 + T, q, h) : make_float4(0.f, 0.f, 0.f, 0.f);
        v[4 * q + 0] = hv.x > 0.f ? v[4 * q + 0] : v[4 * q + 0] * slope;
        v[4 * q + 1] = hv.y > 0.f ? v[4 * q + 1] : v[4 * q + 1] * slope;
        v[4 * q + 2] = hv.z > 0.f ? v[4 * q + 2] : v[4 * q + 2] * slope;
        v[4 * q + 3] = hv.w > 0.f ? v[4 * q + 3] : v[4 * q + 3] * slope;
        if (!act) v[4 * q] = v[4 * q + 1] = v[4 * q + 2] = v[4 * q + 3] = 0.f;
        if (act)
          *reinterpret_cast<float4*>(dst + pair * kHid + 32 * (T0 + T) + 8 * q + 4 * h) =
              make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        if (amx) {
#pragma unroll
          for (int i = 0; i < 4; ++i) mb = max(mb, __float_as_uint(fabsf(v[4 * q + i])));
        }
      }
  }
  if (amx) wave_absmax_to(amx, mb);
}

// dz = dh * lrelu'(z) from the saved derivative bits (words prefetched by
// load_masks before the layer's GEMM, so the mask latency hides behind it).
template <int NT, int PT>
__device__ __forceinline__ void load_masks(unsigned (&mk)[PT * NT], const uint16_t* mask, int layer, int64_t tile,
                                           int64_t n, int lane, int T0) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    const int col = 32 * pt + c;
    const bool act = tile * kTS + (col >> 3) < n;
#pragma unroll
    for (int T = 0; T < NT; ++T)
      mk[pt * NT + T] = act ? mask[(tile * kTP + col) * 64 + 16 * layer + 2 * (T0 + T) + h] : 0u;
  }
}

template <int NT, int PT>
__device__ __forceinline__ void lrelu_bwd_m(f32x16 (&acc)[PT * NT], const unsigned (&mk)[PT * NT], float* dst,
                                            int64_t tile, int64_t n, float slope, int lane, int T0,
                                            unsigned* amx = nullptr) {
  const int c = lane & 31, h = lane >> 5;
  unsigned mb = 0;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    const int col = 32 * pt + c;
    const bool act = tile * kTS + (col >> 3) < n;
    const int64_t pair = tile * kTP + col;
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      f32x16& v = acc[pt * NT + T];
      const unsigned b = mk[pt * NT + T];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = act ? (((b >> r) & 1u) ? v[r] : v[r] * slope) : 0.f;
      if (act) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<float4*>(dst + pair * kHid + 32 * (T0 + T) + 8 * q + 4 * h) =
              make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      }
      if (amx) {
#pragma unroll
        for (int r = 0; r < 16; ++r) mb = max(mb, __float_as_uint(fabsf(v[r])));
      }
    }
  }
  if (amx) wave_absmax_to(amx, mb);
}

// ---- fp32x3 dX GEMMs of k_pairs_bwd<true>: the transposed weights as exact
// 3-way bf16 splits (frag_pack_x3: F[t][T][plane][lane][8], X3_PAD zero steps),
// the B fragments read from the fp32 quad rows and split into three bf16
// planes in registers (split2, exact), six cross products per 16-k step on
// v_mfma_f32_32x32x16_bf16 (smallest first) -- the arithmetic of the fp32x3
// forward (aggregate_x3.hip) on k_pairs_bwd's LDS layout.
constexpr int kX3D = 3;   // weight ring depth (k-steps in flight) <= X3_PAD
struct X3QRing {
  uint4 a[kX3D][2][3];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t x3q_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// this wave's two neuron tiles of k-step t, three planes each; voff = (T0 * 3 * 64 + lane) * 16
__device__ __forceinline__ void x3q_load(uint4 (&a)[2][3], __amdgpu_buffer_rsrc_t rs, int voff, int t) {
#pragma unroll
  for (int T = 0; T < 2; ++T)
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      a[T][pl] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + pl * 1024,
                                                                                   (t * 8 + T) * 3 * 1024, 0));
}

__device__ __forceinline__ void x3q_prime(X3QRing& w, __amdgpu_buffer_rsrc_t rs, int voff) {
#pragma unroll
  for (int d = 0; d < kX3D; ++d) x3q_load(w.a[d], rs, voff, d);
}

// B fragment of k-step t, pair half pt: inputs 16t + 8h .. +7 of pair 32pt + c
// (quad rows 4t + 2h, 4t + 2h + 1; each float4 holds neurons (0, 2, 1, 3))
__device__ __forceinline__ void x3q_b(const float* X, int t, int pt, int lane, uint4 (&b)[3]) {
  const int c = lane & 31, h = lane >> 5;
  const float* xb = X + (4 * t + 2 * h) * kQP + 4 * (32 * pt + c);
  const float4 q0 = *reinterpret_cast<const float4*>(xb);
  const float4 q1 = *reinterpret_cast<const float4*>(xb + kQP);
  unsigned w0[4], w1[4], w2[4];
  split2(q0.x, q0.z, w0[0], w1[0], w2[0]);
  split2(q0.y, q0.w, w0[1], w1[1], w2[1]);
  split2(q1.x, q1.z, w0[2], w1[2], w2[2]);
  split2(q1.y, q1.w, w0[3], w1[3], w2[3]);
  b[0] = make_uint4(w0[0], w0[1], w0[2], w0[3]);
  b[1] = make_uint4(w1[0], w1[1], w1[2], w1[3]);
  b[2] = make_uint4(w2[0], w2[1], w2[2], w2[3]);
}

// acc[2 pt + T] += W^T . X over nsteps 16-k steps (weights kX3D steps ahead
// in the ring)
// (the ring is primed here, not ahead across the tile's other phases: 72 VGPRs
// live through the whole tile made the kernel spill)
__device__ __forceinline__ void mlp_layer_x3q(f32x16 (&acc)[4], __amdgpu_buffer_rsrc_t rs, int voff,
                                              const float* X, int nsteps, int lane) {
  X3QRing w;
  x3q_prime(w, rs, voff);
  uint4 b[2][3];
  x3q_b(X, 0, 0, lane, b[0]);
  x3q_b(X, 0, 1, lane, b[1]);
  auto step = [&](uint4 (&a)[2][3], int t) {
    if (t > 0) {
      x3q_b(X, t, 0, lane, b[0]);
      x3q_b(X, t, 1, lane, b[1]);
    }
    // products smallest first (W2.X0, W1.X1, W0.X2, W1.X0, W0.X1, W0.X0), each
    // over the four accumulators in turn: four independent MFMA chains
    constexpr int kPa[6] = {2, 1, 0, 1, 0, 0}, kPb[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int p = 0; p < 6; ++p)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int T = 0; T < 2; ++T) acc[2 * pt + T] = mfma_bf16(a[T][kPa[p]], b[pt][kPb[p]], acc[2 * pt + T]);
    x3q_load(a, rs, voff, t + kX3D);   // packs carry kX3D zero steps
  };
  int t = 0;
#pragma unroll 1
  for (; t + kX3D <= nsteps; t += kX3D) {
#pragma unroll
    for (int d = 0; d < kX3D; ++d) step(w.a[d], t + d);
  }
#pragma unroll
  for (int d = 0; d < kX3D - 1; ++d)
    if (t + d < nsteps) step(w.a[d], t + d);
}

// ---- fp32h2 dX GEMMs of k_pairs_bwd<2>: the transposed weights as f16 (hi,
// 2^11 lo) pairs of 2^-s W (pnr_pack_bwd_h2: F[t][T][plane][lane][8], kX3D zero
// steps), the B fragments split from the fp32 quad rows times the tile's power
// of two xs (max |X| xs in [2^13, 2^14): every value of the tile keeps 22
// significant bits down to 2^-14 of the maximum), three products per 16-k step
// on v_mfma_f32_32x32x16_f16 -- 2^11 (2^-s W X xs) in the accumulators, which
// the caller scales back.
struct H2QRing {
  uint4 a[kX3D][2][2];
};

__device__ __forceinline__ void h2q_load(uint4 (&a)[2][2], __amdgpu_buffer_rsrc_t rs, int voff, int t) {
#pragma unroll
  for (int T = 0; T < 2; ++T)
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      a[T][pl] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + pl * 1024,
                                                                                   (t * 8 + T) * 2 * 1024, 0));
}

__device__ __forceinline__ void h2q_b(const float* X, int t, int pt, int lane, float xs, uint4 (&b)[2]) {
  const int c = lane & 31, h = lane >> 5;
  const float* xb = X + (4 * t + 2 * h) * kQP + 4 * (32 * pt + c);
  const float4 q0 = *reinterpret_cast<const float4*>(xb);
  const float4 q1 = *reinterpret_cast<const float4*>(xb + kQP);
  unsigned w0[4], w1[4];
  splith(q0.x * xs, q0.z * xs, w0[0], w1[0]);
  splith(q0.y * xs, q0.w * xs, w0[1], w1[1]);
  splith(q1.x * xs, q1.z * xs, w0[2], w1[2]);
  splith(q1.y * xs, q1.w * xs, w0[3], w1[3]);
  b[0] = make_uint4(w0[0], w0[1], w0[2], w0[3]);
  b[1] = make_uint4(w1[0], w1[1], w1[2], w1[3]);
}

__device__ __forceinline__ void mlp_layer_h2q(f32x16 (&acc)[4], __amdgpu_buffer_rsrc_t rs, int voff,
                                              const float* X, int nsteps, int lane, float xs) {
  H2QRing w;
#pragma unroll
  for (int d = 0; d < kX3D; ++d) h2q_load(w.a[d], rs, voff, d);
  uint4 b[2][2];
  h2q_b(X, 0, 0, lane, xs, b[0]);
  h2q_b(X, 0, 1, lane, xs, b[1]);
  auto step = [&](uint4 (&a)[2][2], int t) {
    if (t > 0) {
      h2q_b(X, t, 0, lane, xs, b[0]);
      h2q_b(X, t, 1, lane, xs, b[1]);
    }
    // smallest terms first: Wl.Xh, Wh.Xl, then 2^11 Wh.Xh; four independent chains
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int T = 0; T < 2; ++T) acc[2 * pt + T] = mfma_f16(a[T][1], b[pt][0], acc[2 * pt + T]);
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int T = 0; T < 2; ++T) acc[2 * pt + T] = mfma_f16(a[T][0], b[pt][1], acc[2 * pt + T]);
    const uint4 as0 = f16x8_scale2048(a[0][0]), as1 = f16x8_scale2048(a[1][0]);
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      acc[2 * pt] = mfma_f16(as0, b[pt][0], acc[2 * pt]);
      acc[2 * pt + 1] = mfma_f16(as1, b[pt][0], acc[2 * pt + 1]);
    }
    h2q_load(a, rs, voff, t + kX3D);   // packs carry kX3D zero steps
  };
  int t = 0;
#pragma unroll 1
  for (; t + kX3D <= nsteps; t += kX3D) {
#pragma unroll
    for (int d = 0; d < kX3D; ++d) step(w.a[d], t + d);
  }
#pragma unroll
  for (int d = 0; d < kX3D - 1; ++d)
    if (t + d < nsteps) step(w.a[d], t + d);
}

// max |v| over this wave's accumulators into slot (one float per wave; NaN as +inf)
__device__ __forceinline__ void wave_tile_absmax(const f32x16 (&acc)[4], float* slot) {
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float a = fabsf(acc[i][r]);
      m = a != a ? __builtin_inff() : fmaxf(m, a);
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) *slot = m;
}

// the tile's X factor xs = 2^e (max |X| xs in [2^13, 2^14), e <= 126) from the
// four waves' maxima; 1 for an all-zero or non-finite tile
__device__ __forceinline__ float tile_xscale(const float* slots) {
  const float m = fmaxf(fmaxf(slots[0], slots[1]), fmaxf(slots[2], slots[3]));
  if (!(m > 0.f) || !(m <= 3.0e38f)) return 1.f;
  int E;
  (void)frexpf(m, &E);   // m = f 2^E, f in [0.5, 1)
  return ldexpf(1.f, min(14 - E, 126));
}

// acc = acc / xs * ws (two steps: each factor alone stays in the normal range)
__device__ __forceinline__ void h2q_unscale(f32x16 (&acc)[4], float xs, float ws) {
  const float xu = 1.f / xs;   // exact: xs is a power of two
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = (acc[i][r] * xu) * ws;
}


// V = 0: native fp32 dX GEMMs; 1: fp32x3 (split bf16); 2: fp32h2 (split f16,
// per-tile power-of-two scaling of X).  V >= 1 leaves the block3.0 extras to a
// separate pass.
template <int V>
__global__ void __launch_bounds__(64 * kPairWaves, 2) k_pairs_bwd(BwdArgs A) {
  constexpr bool X3 = V != 0;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  float* X = lds_dyn;                   // quad rows [66][kQP]
  float* dotp = X + 66 * kQP;           // [4][64] partial <d_hid, h4> per wave
  float* exP = dotp + 4 * kTP;          // [4][7][64] partial block3.0 extras gradients (V == 0)
  float* tmx = exP;                     // [4] per-wave max |X| of the layer input (V == 2)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int j = lane >> 3;
  const int T0 = wid * kNTW;
  const int64_t n = eff_n(A.s);
  const int64_t ntiles = cdiv(n, kTS);
  const float slope = A.w.neg_slope;
  const float* w4t = X3 ? nullptr : A.wb.w4t + T0 * 64;
  const float* w3t = X3 ? nullptr : A.wb.w3t + T0 * 64;
  const float* w2t = X3 ? nullptr : A.wb.w2t + T0 * 64;
  float ring[kQD][kNTW];
  const int xvoff = (T0 * (V == 2 ? 2 : 3) * 64 + lane) * 16;
  const __amdgpu_buffer_rsrc_t x4 = x3q_rsrc(A.wx[0]), x3 = x3q_rsrc(A.wx[1]), x2 = x3q_rsrc(A.wx[2]);
  const float ws4 = V == 2 ? A.wxs[0] : 1.f, ws3 = V == 2 ? A.wxs[1] : 1.f, ws2 = V == 2 ? A.wxs[2] : 1.f;
  if constexpr (!X3) prime_q<kNTW>(ring, w4t, lane);
  // max |dz1..dz4|, |dpa| of this workgroup (pnr_agg_saved.dz_absmax: pnr_gemm_tn_h2's scales)
  __shared__ unsigned amx[5];
  unsigned* const am = A.sv.dz_absmax ? amx : nullptr;
  if (threadIdx.x < 5) amx[threadIdx.x] = 0u;
  __syncthreads();

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // ---------------------------------------------------------- per-pair scalars (lane = pair)
    const int64_t v = tile * kTS + j;
    const bool active = v < n;
    const int64_t pair = tile * kTP + lane;
    const bool svalid = active && A.sv.vmask[v] != 0;
    const float wt = active ? A.sv.wt[pair] : 0.f;
    const float pa = active ? A.sv.pa[pair] : 0.f;
    const float dalpha = svalid ? A.d_feat[v * (kC + 1)] : 0.f;
    // alpha_k = softplus(pa - 1) (threshold 20) or relu(pa) (point_aggregators.py:262-267)
    float a_k, sig;
    if (A.w.act_super) {
      const float x = pa - 1.f;
      a_k = softplus(x);
      sig = x > 20.f ? 1.f : 1.f / (1.f + expf(-x));
    } else {
      a_k = fmaxf(pa, 0.f);
      sig = pa > 0.f ? 1.f : 0.f;
    }
    const float dpa = dalpha * wt * sig;   // d alpha_s / d pa_k
    if (wid == 0 && active) A.dpa[pair] = dpa;
    if (am && wid == 0) wave_absmax_to(am + 4, active ? __float_as_uint(fabsf(dpa)) : 0u);
    // ---------------------------------------------------------- d h4 -> dz4 (acc layout)
    f32x16 acc[kPTW * kNTW];
    float dot[kPTW];
#pragma unroll
    for (int pt = 0; pt < kPTW; ++pt) {
      const int col = 32 * pt + c;
      const int64_t pp = tile * kTP + col;
      const int64_t vv = tile * kTS + (col >> 3);
      const bool act = vv < n;
      const float wt_p = __shfl(wt, col), dpa_p = __shfl(dpa, col);
      const bool sv_p = __shfl((int)svalid, col) != 0;
      dot[pt] = 0.f;
#pragma unroll
      for (int T = 0; T < kNTW; ++T)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 h4 = act ? ld_q(A.sv.h4, pp, T0 + T, q, h) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 df = sv_p ? ld_q(A.d_hid, vv, T0 + T, q, h) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 wa = *reinterpret_cast<const float4*>(A.w.wa + 32 * (T0 + T) + 8 * q + 4 * h);
          dot[pt] += df.x * h4.x + df.y * h4.y + df.z * h4.z + df.w * h4.w;
          // f_s = sum_k wt_k h4_k ; alpha_s = sum_k wt_k softplus(wa.h4_k + ba - 1)
          acc[pt * kNTW + T][4 * q + 0] = wt_p * df.x + dpa_p * wa.x;
          acc[pt * kNTW + T][4 * q + 1] = wt_p * df.y + dpa_p * wa.y;
          acc[pt * kNTW + T][4 * q + 2] = wt_p * df.z + dpa_p * wa.z;
          acc[pt * kNTW + T][4 * q + 3] = wt_p * df.w + dpa_p * wa.w;
        }
      dot[pt] += __shfl_xor(dot[pt], 32);
    }
    if (h == 0) {
      dotp[wid * kTP + c] = dot[0];
      dotp[wid * kTP + 32 + c] = dot[1];
    }
    lrelu_bwd_q<kNTW, kPTW>(acc, A.sv.h4, A.dz[3], tile, n, slope, lane, T0, am ? am + 3 : nullptr);
    store_q<kNTW, kPTW>(acc, X, lane, T0);
    if constexpr (V == 2) wave_tile_absmax(acc, tmx + wid);
    __syncthreads();
    // d wt_k = d alpha_s a_k + <d f_s, h4_k>  ->  d conf_k (straight-through clamp, :724-726)
    if (wid == 0 && active && A.d_conf) {
      const int32_t pr = A.sv.prow[pair];
      if (pr >= 0) {
        const float dwt = dalpha * a_k + dotp[lane] + dotp[kTP + lane] + dotp[2 * kTP + lane] +
                          dotp[3 * kTP + lane];
        atomicAdd(A.d_conf + pr, dwt * A.sv.wn[pair]);
      }
    }
    // ---------------------------------------------------------- block3.2^T: dh3 = W4^T dz4
#pragma unroll
    for (int i = 0; i < kPTW * kNTW; ++i) acc[i] = (f32x16){0.f};
    unsigned mk[kPTW * kNTW];
    load_masks<kNTW, kPTW>(mk, A.sv.mask, 2, tile, n, lane, T0);
    if constexpr (V == 2) {
      const float xs = tile_xscale(tmx);
      mlp_layer_h2q(acc, x4, xvoff, X, 16, lane, xs);
      h2q_unscale(acc, xs, ws4);
    } else if constexpr (X3) {
      mlp_layer_x3q(acc, x4, xvoff, X, 16, lane);
    } else {
      mlp_layer_q<kNTW, kPTW>(acc, ring, w4t, X, 128, lane);
      prime_q<kNTW>(ring, w3t, lane);
    }
    __syncthreads();
    lrelu_bwd_m<kNTW, kPTW>(acc, mk, A.dz[2], tile, n, slope, lane, T0, am ? am + 2 : nullptr);
    store_q<kNTW, kPTW>(acc, X, lane, T0);
    if constexpr (V == 2) wave_tile_absmax(acc, tmx + wid);
    // block3.0 extras (inputs 256..262): d x3e_e = sum_n W3[n, 256 + e] dz3[n];
    // wave w reads back its own 64 dz3 rows (quad rows 16w..16w+15), lane = pair
    wave_sync();
    if constexpr (!X3) {
      float ex[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int u = 16 * wid; u < 16 * wid + 16; ++u) {
        const float4 x4 = *reinterpret_cast<const float4*>(X + u * kQP + 4 * lane);
        const float xv[4] = {x4.x, x4.z, x4.y, x4.w};   // neurons 4u + 0..3 (quad perm)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float* we = A.wb.w3e + (4 * u + i) * 7;
#pragma unroll
          for (int e = 0; e < 7; ++e) ex[e] += we[e] * xv[i];
        }
      }
#pragma unroll
      for (int e = 0; e < 7; ++e) exP[(wid * 7 + e) * kTP + lane] = ex[e];
    }
    __syncthreads();
    // colour / dir gradients of the pair (wave 0, lane = pair), before the
    // block3.0^T GEMM: its registers stay free for the GEMM.  The pair's
    // indices are recomputed here rather than kept live across the GEMMs.
    if (!X3 && wid == 0 && tile * kTS + (lane >> 3) < n) {
      const int64_t pair = tile * kTP + lane;
      const int64_t v = tile * kTS + (lane >> 3);
      const int32_t pr = A.sv.prow[pair];
      if (pr >= 0) {
        float g[7];
#pragma unroll
        for (int e = 0; e < 7; ++e)
          g[e] = exP[(0 * 7 + e) * kTP + lane] + exP[(1 * 7 + e) * kTP + lane] + exP[(2 * 7 + e) * kTP + lane] +
                 exP[(3 * 7 + e) * kTP + lane];
        if (A.d_color) {
#pragma unroll
          for (int a = 0; a < 3; ++a) atomicAdd(A.d_color + (int64_t)pr * 3 + a, g[a]);
        }
        if (A.d_dir) {
          // inputs: R.dir - R.v (3), <R.dir, R.v> (1) with R.dir = dir @ Rw^T
          const int64_t row = sample_row(A.s, v);
          const int64_t drow = dir_row(A.s, row);
          const float vd[3] = {A.s.dirs[drow * 3], A.s.dirs[drow * 3 + 1], A.s.dirs[drow * 3 + 2]};
          float Rw[9];   // loaded here, not kept live across the tile's GEMMs
#pragma unroll
          for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
          float vrot[3];
          mat3(Rw, vd, vrot);
          if (A.pts.rw2c) {   // per-point: view dir by the slot-0 matrix, d dir through the pair's
            rot_point(A.pts.rw2c, slot0_point(A.s, row), vd, vrot);
#pragma unroll
            for (int i = 0; i < 9; ++i) Rw[i] = A.pts.rw2c[(int64_t)pr * 9 + i];
          }
          const float gd[3] = {g[3] + vrot[0] * g[6], g[4] + vrot[1] * g[6], g[5] + vrot[2] * g[6]};
          // drot_j = sum_i Rw[j][i] dir_i  ->  d dir_i = sum_j Rw[j][i] d drot_j
#pragma unroll
          for (int i = 0; i < 3; ++i)
            atomicAdd(A.d_dir + (int64_t)pr * 3 + i, Rw[i] * gd[0] + Rw[3 + i] * gd[1] + Rw[6 + i] * gd[2]);
        }
      }
    }
    // ---------------------------------------------------------- block3.0^T: dh2 = W3[:, :256]^T dz3
#pragma unroll
    for (int i = 0; i < kPTW * kNTW; ++i) acc[i] = (f32x16){0.f};
    load_masks<kNTW, kPTW>(mk, A.sv.mask, 1, tile, n, lane, T0);
    if constexpr (V == 2) {
      const float xs = tile_xscale(tmx);
      mlp_layer_h2q(acc, x3, xvoff, X, 16, lane, xs);
      h2q_unscale(acc, xs, ws3);
    } else if constexpr (X3) {
      mlp_layer_x3q(acc, x3, xvoff, X, 16, lane);
    } else {
      mlp_layer_q<kNTW, kPTW>(acc, ring, w3t, X, 128, lane);
      prime_q<kNTW>(ring, w2t, lane);
    }
    __syncthreads();
    lrelu_bwd_m<kNTW, kPTW>(acc, mk, A.dz[1], tile, n, slope, lane, T0, am ? am + 1 : nullptr);
    store_q<kNTW, kPTW>(acc, X, lane, T0);
    if constexpr (V == 2) wave_tile_absmax(acc, tmx + wid);
    __syncthreads();
    // ---------------------------------------------------------- block1.2^T: dh1 = W2^T dz2
#pragma unroll
    for (int i = 0; i < kPTW * kNTW; ++i) acc[i] = (f32x16){0.f};
    load_masks<kNTW, kPTW>(mk, A.sv.mask, 0, tile, n, lane, T0);
    if constexpr (V == 2) {
      const float xs = tile_xscale(tmx);
      mlp_layer_h2q(acc, x2, xvoff, X, 16, lane, xs);
      h2q_unscale(acc, xs, ws2);
    } else if constexpr (X3) {
      mlp_layer_x3q(acc, x2, xvoff, X, 16, lane);
    } else {
      mlp_layer_q<kNTW, kPTW>(acc, ring, w2t, X, 128, lane);
      prime_q<kNTW>(ring, w4t, lane);   // the next tile
    }
    lrelu_bwd_m<kNTW, kPTW>(acc, mk, A.dz[0], tile, n, slope, lane, T0, am ? am + 0 : nullptr);
    // block1.0 point half: d P1[p] += dz1 (the P1 gather's backward).  dz1 goes
    // through LDS so each pair's 1-KB row is added with 4 coalesced 256-B
    // atomic wave instructions (wave w: pairs 16w..16w+15, lane = neuron).
    // d_p1 == NULL: the caller reduces dz1 per point instead (pnr_pairs_to_points).
    __syncthreads();                 // every wave is done reading X (W2^T GEMM)
    if (A.d_p1 == nullptr) continue;
    store_q<kNTW, kPTW>(acc, X, lane, T0);
    __syncthreads();
    for (int i = 0; i < kTP / kPairWaves; ++i) {
      const int col = wid * (kTP / kPairWaves) + i;
      if (tile * kTS + (col >> 3) >= n) break;
      const int32_t pr = A.sv.prow[tile * kTP + col];
      if (pr < 0) continue;
      float* dst = A.d_p1 + (A.pts.used_map ? (int64_t)A.pts.used_map[pr] : (int64_t)pr) * kHid;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int nn = lane + 64 * q;
        atomicAdd(dst + nn, X[qaddr(nn, col)]);
      }
    }
    __syncthreads();
  }
  if (am) {   // one global max per workgroup and array
    __syncthreads();
    if (threadIdx.x < 5 && amx[threadIdx.x]) atomicMax(A.sv.dz_absmax + threadIdx.x, amx[threadIdx.x]);
  }
}

// block3.0 extras backward of k_pairs_bwd<true> as its own pass over the pairs:
// g_e = sum_n W3[n, 256 + e] dz3[pair][n] -> d colour (e 0..2) and d dir (e 3..6,
// through R.dir - R.v and <R.dir, R.v>).  One wave per 64 pairs, lane = pair.
__global__ void __launch_bounds__(256) k_extras_bwd(BwdArgs A) {
  const int lane = threadIdx.x & 63;
  const int64_t n = eff_n(A.s);
  const int64_t P = n * kKN;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t w = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); w * 64 < P; w += waves) {
    const int64_t pair = w * 64 + lane;
    if (pair >= P) continue;
    const int32_t pr = A.sv.prow[pair];
    if (pr < 0) continue;
    float g[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float4* z4 = reinterpret_cast<const float4*>(A.dz[2] + pair * kHid);
#pragma unroll 4
    for (int u = 0; u < kHid / 4; ++u) {
      const float4 z = z4[u];
      const float zv[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 7; ++e) g[e] += A.wb.w3e[(4 * u + i) * 7 + e] * zv[i];
    }
    if (A.d_color) {
#pragma unroll
      for (int a = 0; a < 3; ++a) atomicAdd(A.d_color + (int64_t)pr * 3 + a, g[a]);
    }
    if (A.d_dir) {
      float Rw[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
      const int64_t row = sample_row(A.s, pair / kKN);
      const int64_t drow = dir_row(A.s, row);
      const float vd[3] = {A.s.dirs[drow * 3], A.s.dirs[drow * 3 + 1], A.s.dirs[drow * 3 + 2]};
      float vrot[3];
      mat3(Rw, vd, vrot);
      if (A.pts.rw2c) {   // per-point: view dir by the slot-0 matrix, d dir through the pair's
        rot_point(A.pts.rw2c, slot0_point(A.s, row), vd, vrot);
#pragma unroll
        for (int i = 0; i < 9; ++i) Rw[i] = A.pts.rw2c[(int64_t)pr * 9 + i];
      }
      const float gd[3] = {g[3] + vrot[0] * g[6], g[4] + vrot[1] * g[6], g[5] + vrot[2] * g[6]};
#pragma unroll
      for (int i = 0; i < 3; ++i)
        atomicAdd(A.d_dir + (int64_t)pr * 3 + i, Rw[i] * gd[0] + Rw[3 + i] * gd[1] + Rw[6 + i] * gd[2]);
    }
  }
}

// Per-point entry counts of a query's neighbour lists: counts[p] += 1 for every
// pidx entry p >= 0 of the first (*n_dev) samples (float atomics of integers:
// exact and order-free below 2^24).
__global__ void k_point_counts(const int32_t* __restrict__ pidx, const int32_t* __restrict__ n_dev, int K,
                               int64_t cap, float* __restrict__ counts) {
  int64_t ns = *n_dev;
  ns = ns < cap ? ns : cap;
  const int64_t n = ns * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = pidx[i];
    if (p >= 0) atomicAdd(counts + p, 1.f);
  }
}

// pnr_used_points: a byte per point marked by plain stores (20 MB at c5's 20 M
// points, where an int32 flag per point was 80 MB of randomly touched lines;
// bit atomics measured slower: each drops its line from the XCD's L2), packed
// to one bit per point with the words' popcounts, ranked by a scan of those.
// The read comes before the store: neighbouring samples share most points, so
// nearly every flag is already set and stays a cached read.
__global__ void k_mark_used(const int32_t* __restrict__ pidx, const int32_t* __restrict__ n_dev, int K, int64_t cap,
                            uint8_t* __restrict__ flags) {
  const int64_t n = (n_dev ? (int64_t)*n_dev : cap) * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = pidx[i];
    if (p >= 0 && flags[p] == 0) flags[p] = 1;
  }
}

// word w of the bitset from flags[32w .. 32w+32) (two 16-B loads; the byte array
// is padded to whole words), cnt[w] = its popcount
__global__ void k_pack_used(const uint8_t* __restrict__ flags, int64_t nw, uint32_t* __restrict__ bits,
                            int32_t* __restrict__ cnt) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    const uint4* f = reinterpret_cast<const uint4*>(flags + w * 32);
    const uint4 a = f[0], b = f[1];
    const uint32_t q[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= ((q[j] >> (8 * k)) & 1u) << (4 * j + k);
    bits[w] = m;
    cnt[w] = __popc(m);
  }
}

// used_map[p] = rank of p (word prefix + set bits below p in its word) or -1;
// used[rank] = p.
__global__ void k_used_list(const uint32_t* __restrict__ bits, const int32_t* __restrict__ wpre, int64_t n_points,
                            int32_t* __restrict__ used_map, int32_t* __restrict__ used) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n_points;
       p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t word = bits[p >> 5];
    const int b = (int)(p & 31);
    if ((word >> b) & 1u) {
      const int32_t r = wpre[p >> 5] + __popc(word & ((1u << b) - 1u));
      used_map[p] = r;
      used[r] = (int32_t)p;
    } else {
      used_map[p] = -1;
    }
  }
}

// Sum of a run of pairs sorted by point row, in pair order (deterministic):
// the run's positions are found 64 at a time with one ballot, the pair ids
// loaded one per lane and broadcast, and four dz1 rows read before they are
// added, so a wave keeps four row loads in flight instead of one.
template <bool EX>
__device__ __forceinline__ void run_sum(const int32_t* __restrict__ prow_sorted, const int32_t* __restrict__ pair_of,
                                        int64_t P, int64_t i, int32_t pr, const float* __restrict__ dz1,
                                        const float* __restrict__ g_pair, float4& s, float& ge) {
  const int lane = threadIdx.x & 63;
  bool first = true;
  for (int64_t j0 = i;; j0 += 64) {
    const int64_t jj = j0 + lane;
    const int32_t pl = jj < P ? prow_sorted[jj] : -2;
    const uint64_t same = __ballot(pl == pr);
    const int len = same == ~0ull ? 64 : __builtin_ctzll(~same);
    const int32_t mine = lane < len ? pair_of[jj] : 0;
    int t = 0;
    for (; t + 4 <= len; t += 4) {
      int64_t pq[4];
      float4 v[4];
      float gq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) pq[u] = __shfl(mine, t + u);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = reinterpret_cast<const float4*>(dz1 + pq[u] * kHid)[lane];
        gq[u] = (EX && lane < 6) ? g_pair[pq[u] * 8 + lane] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (first && !EX) {
          s = v[u];
          first = false;
        } else {
          s.x += v[u].x;
          s.y += v[u].y;
          s.z += v[u].z;
          s.w += v[u].w;
        }
        if (EX && lane < 6) ge += gq[u];
      }
    }
    for (; t < len; ++t) {
      const int64_t pq = __shfl(mine, t);
      const float4 v = reinterpret_cast<const float4*>(dz1 + pq * kHid)[lane];
      if (first && !EX) {
        s = v;
        first = false;
      } else {
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
      if (EX && lane < 6) ge += g_pair[pq * 8 + lane];
    }
    if (len < 64) break;
  }
}

// A run that ends inside the caller's 64-position chunk: its pair ids are the
// chunk's lanes l .. l + len - 1 (`mine`), so only the dz1 rows are loaded.
template <bool EX>
__device__ __forceinline__ void run_sum_chunk(int32_t mine, int l, int len, const float* __restrict__ dz1,
                                              const float* __restrict__ g_pair, float4& s, float& ge) {
  const int lane = threadIdx.x & 63;
  int t = 0;
  for (; t + 4 <= len; t += 4) {
    int64_t pq[4];
    float4 v[4];
    float gq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) pq[u] = __shfl(mine, l + t + u);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = reinterpret_cast<const float4*>(dz1 + pq[u] * kHid)[lane];
      gq[u] = (EX && lane < 6) ? g_pair[pq[u] * 8 + lane] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (t + u == 0 && !EX) {
        s = v[u];
      } else {
        s.x += v[u].x;
        s.y += v[u].y;
        s.z += v[u].z;
        s.w += v[u].w;
      }
      if (EX && lane < 6) ge += gq[u];
    }
  }
  for (; t < len; ++t) {
    const int64_t pq = __shfl(mine, l + t);
    const float4 v = reinterpret_cast<const float4*>(dz1 + pq * kHid)[lane];
    if (t == 0 && !EX) {
      s = v;
    } else {
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    if (EX && lane < 6) ge += g_pair[pq * 8 + lane];
  }
}

// d P1 rows from dz1 without atomics: pairs sorted by point row (stable, so
// each point's pairs in pair order -- a deterministic sum); one wave per run of
// equal rows, lane = 4 neurons (float4).
__global__ void k_pairs_to_points(const int32_t* __restrict__ prow_sorted, const int32_t* __restrict__ pair_of,
                                  int64_t P, const float* __restrict__ dz1, const int32_t* __restrict__ used_map,
                                  float* __restrict__ d_p1, uint32_t* __restrict__ absmax) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  __shared__ unsigned bmax;
  if (threadIdx.x == 0) bmax = 0u;
  __syncthreads();
  unsigned mb = 0u;   // max |d_p1| of this lane's rows (float bits: NaN propagates)
  // 64 sorted positions per wave and step: one ballot finds the runs that start there
  for (int64_t i0 = (blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; i0 < P; i0 += waves * 64) {
    const int64_t ii = i0 + lane;
    const int32_t pr_l = ii < P ? prow_sorted[ii] : -1;
    const int32_t pv_l = ii > 0 && ii < P ? prow_sorted[ii - 1] : -1;
    const int32_t mine = ii < P ? pair_of[ii] : 0;
    uint64_t starts = __ballot(pr_l >= 0 && (ii == 0 || pv_l != pr_l));
    const uint64_t bounds = __ballot(ii >= P || ii == 0 || pv_l != pr_l);   // a new value (or the end) begins
    while (starts) {
      const int l = __builtin_ctzll(starts);
      starts &= starts - 1;
      const int64_t i = i0 + l;
      const int32_t pr = __shfl(pr_l, l);
      const uint64_t after = l == 63 ? 0ull : bounds & (~0ull << (l + 1));
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      float ge = 0.f;
      if (after) run_sum_chunk<false>(mine, l, __builtin_ctzll(after) - l, dz1, nullptr, s, ge);
      else run_sum<false>(prow_sorted, pair_of, P, i, pr, dz1, nullptr, s, ge);   // runs past the chunk
      reinterpret_cast<float4*>(d_p1 + (used_map ? (int64_t)used_map[pr] : (int64_t)pr) * kHid)[lane] = s;
      mb = max(max(mb, max(__float_as_uint(fabsf(s.x)), __float_as_uint(fabsf(s.y)))),
               max(__float_as_uint(fabsf(s.z)), __float_as_uint(fabsf(s.w))));
    }
  }
  if (absmax) {
    wave_absmax_to(&bmax, mb);
    __syncthreads();
    if (threadIdx.x == 0 && bmax) atomicMax(absmax, bmax);
  }
}

// The block3.0 extras per pair without atomics (pnr_aggregate_bwd_extras_rows):
// g_pair[pair] = (g0, g1, g2, g3 + vrot0 g6, g4 + vrot1 g6, g5 + vrot2 g6, 0, 0)
// with g_e = dz3[pair] . W3[:, 256 + e] and vrot the pair's rotated view
// direction; the per-point sums (and the point's Rw^T) follow in
// pnr_pairs_to_points_ex.  Four lanes per pair: a load instruction reads 16 rows'
// 64-B pieces (k_extras_bwd's lane-per-pair loop read 64 rows' 16-B pieces), the
// weights from LDS ([256][8]), two xor steps reduce the four partials.
__global__ void __launch_bounds__(256) k_extras_rows(BwdArgs A, float* __restrict__ g_pair) {
  __shared__ float4 wl[kHid][2];
  for (int i = threadIdx.x; i < kHid; i += blockDim.x) {
    const float* w = A.wb.w3e + i * 7;
    wl[i][0] = make_float4(w[0], w[1], w[2], w[3]);
    wl[i][1] = make_float4(w[4], w[5], w[6], 0.f);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, q = lane & 3;
  const int64_t n = eff_n(A.s);
  const int64_t P = n * kKN;
  float Ru[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Ru[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
  const int64_t groups = (int64_t)gridDim.x * (blockDim.x >> 2);
  for (int64_t pair = blockIdx.x * (int64_t)(blockDim.x >> 2) + (threadIdx.x >> 2); pair < P; pair += groups) {
    const int32_t pr = A.sv.prow[pair];
    float g[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (pr >= 0) {
      const float4* z4 = reinterpret_cast<const float4*>(A.dz[2] + pair * kHid);
#pragma unroll   // all 16 row pieces in flight (4 at a time: 90 us for 242 MB of dz3)
      for (int j = 0; j < kHid / 16; ++j) {
        const int c4 = 4 * j + q;   // float4 column: neurons 4 c4 .. 4 c4 + 3
        const float4 z = z4[c4];
        const float zv[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 w0 = wl[4 * c4 + i][0], w1 = wl[4 * c4 + i][1];
          g[0] += w0.x * zv[i];
          g[1] += w0.y * zv[i];
          g[2] += w0.z * zv[i];
          g[3] += w0.w * zv[i];
          g[4] += w1.x * zv[i];
          g[5] += w1.y * zv[i];
          g[6] += w1.z * zv[i];
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 7; ++e) {
      g[e] += __shfl_xor(g[e], 1);
      g[e] += __shfl_xor(g[e], 2);
    }
    if (q == 0) {
      float vrot[3] = {0.f, 0.f, 0.f};
      if (pr >= 0) {
        const int64_t row = sample_row(A.s, pair / kKN);
        const int64_t drow = dir_row(A.s, row);
        const float vd[3] = {A.s.dirs[drow * 3], A.s.dirs[drow * 3 + 1], A.s.dirs[drow * 3 + 2]};
        mat3(Ru, vd, vrot);
        if (A.pts.rw2c) rot_point(A.pts.rw2c, slot0_point(A.s, row), vd, vrot);
      }
      float4* o = reinterpret_cast<float4*>(g_pair + pair * 8);
      o[0] = make_float4(g[0], g[1], g[2], g[3] + vrot[0] * g[6]);
      o[1] = make_float4(g[4] + vrot[1] * g[6], g[5] + vrot[2] * g[6], 0.f, 0.f);
    }
  }
}

// pnr_pairs_to_points_ex: k_pairs_to_points plus the per-point sums of g_pair
// (lanes 0..5 of the run's wave): d_color[p] = sum g[0..2], d_dir[p] =
// Rw_p^T sum g[3..5] (Rw_p: the point's per-point Rw2c or the uniform one).
// Written, not added: every referenced point's rows, deterministic.
__global__ void k_pairs_to_points_ex(const int32_t* __restrict__ prow_sorted, const int32_t* __restrict__ pair_of,
                                     int64_t P, const float* __restrict__ dz1, const int32_t* __restrict__ used_map,
                                     float* __restrict__ d_p1, uint32_t* __restrict__ absmax,
                                     const float* __restrict__ g_pair, const float* __restrict__ rw_uniform,
                                     const float* __restrict__ rw_pp, float* __restrict__ d_color,
                                     float* __restrict__ d_dir) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  __shared__ unsigned bmax;
  if (threadIdx.x == 0) bmax = 0u;
  __syncthreads();
  unsigned mb = 0u;
  // 64 sorted positions per wave and step: one ballot finds the runs that start there
  for (int64_t i0 = (blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; i0 < P; i0 += waves * 64) {
    const int64_t ii = i0 + lane;
    const int32_t pr_l = ii < P ? prow_sorted[ii] : -1;
    const int32_t pv_l = ii > 0 && ii < P ? prow_sorted[ii - 1] : -1;
    const int32_t mine = ii < P ? pair_of[ii] : 0;
    uint64_t starts = __ballot(pr_l >= 0 && (ii == 0 || pv_l != pr_l));
    const uint64_t bounds = __ballot(ii >= P || ii == 0 || pv_l != pr_l);   // a new value (or the end) begins
    while (starts) {
      const int l = __builtin_ctzll(starts);
      starts &= starts - 1;
      const int64_t i = i0 + l;
      const int32_t pr = __shfl(pr_l, l);
      const uint64_t after = l == 63 ? 0ull : bounds & (~0ull << (l + 1));
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      float ge = 0.f;   // lane e < 6: sum of g_pair[.][e]
      if (after) run_sum_chunk<true>(mine, l, __builtin_ctzll(after) - l, dz1, g_pair, s, ge);
      else run_sum<true>(prow_sorted, pair_of, P, i, pr, dz1, g_pair, s, ge);   // runs past the chunk
      reinterpret_cast<float4*>(d_p1 + (used_map ? (int64_t)used_map[pr] : (int64_t)pr) * kHid)[lane] = s;
      mb = max(max(mb, max(__float_as_uint(fabsf(s.x)), __float_as_uint(fabsf(s.y)))),
               max(__float_as_uint(fabsf(s.z)), __float_as_uint(fabsf(s.w))));
      const float g3 = __shfl(ge, 3), g4 = __shfl(ge, 4), g5 = __shfl(ge, 5);
      if (lane < 3) {
        if (d_color) d_color[(int64_t)pr * 3 + lane] = ge;
        if (d_dir) {   // d dir_a = sum_j Rw[j][a] gd_j
          const float* R = rw_pp ? rw_pp + (int64_t)pr * 9 : rw_uniform;
          const float r0 = R ? R[lane] : (lane == 0 ? 1.f : 0.f);
          const float r1 = R ? R[3 + lane] : (lane == 1 ? 1.f : 0.f);
          const float r2 = R ? R[6 + lane] : (lane == 2 ? 1.f : 0.f);
          d_dir[(int64_t)pr * 3 + lane] = r0 * g3 + r1 * g4 + r2 * g5;
        }
      }
    }
  }
  if (absmax) {
    wave_absmax_to(&bmax, mb);
    __syncthreads();
    if (threadIdx.x == 0 && bmax) atomicMax(absmax, bmax);
  }
}

// X1[p] = [emb, PE_3(emb)] (networks.py:175-190: channel d, band f -> 32 + 2(3d+f) + {sin, cos})
__global__ void k_point_pe3(const float* __restrict__ emb, const int32_t* __restrict__ rows, int64_t n,
                            float* __restrict__ x1) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * kEmb;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / kEmb;
    const int d = (int)(i - p * kEmb);
    const float e = emb[(rows ? (int64_t)rows[p] : p) * kEmb + d];   // rows: the used points (a gather)
    float* o = x1 + p * 224;
    o[d] = e;
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      float sn, cs;
      sincosf(e * (float)(1 << f), &sn, &cs);
      o[kEmb + 2 * (3 * d + f)] = sn;
      o[kEmb + 2 * (3 * d + f) + 1] = cs;
    }
  }
}

__global__ void k_point_pe3_bwd(const float* __restrict__ emb, const int32_t* __restrict__ rows,
                                const float* __restrict__ dx1, int64_t n, float* __restrict__ d_emb) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * kEmb;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / kEmb;
    const int d = (int)(i - p * kEmb);
    const int64_t t = (rows ? (int64_t)rows[p] : p) * kEmb + d;   // rows: scatter into the full table
    const float e = emb[t];
    const float* g = dx1 + p * 224;
    float acc = g[d];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const float b = (float)(1 << f);
      float sn, cs;
      sincosf(e * b, &sn, &cs);
      acc += b * (cs * g[kEmb + 2 * (3 * d + f)] - sn * g[kEmb + 2 * (3 * d + f) + 1]);
    }
    d_emb[t] += acc;
  }
}

// hid rows for n_max samples rounded up to whole 64-sample tiles (the h2
// planes layout, kHidTile in aggregate_x3.hip)
static int64_t hid_rows(int64_t n_max) { return cdiv(n_max > 0 ? n_max : 1, 64) * 64; }

static size_t scratch_need(int64_t n_max, int64_t n_points) {
  const int64_t nm = hid_rows(n_max);
  // + 8 ints: the split kernels' tile counters (k_pairs_x3 / k_pairs_h2, one per XCD group), padded to 16 B
  return ((size_t)nm * kHid + (size_t)cdiv(nm, 4) * 4 + 16 + (size_t)(n_points > 0 ? n_points : 1) * kHid) *
         sizeof(float);
}

// scratch = P1 [n_p1, 256] | hid [n_max, 256] | vmask | tile counter: P1 first,
// so its place does not depend on n_max and a later call may reuse it
// (pnr_points.p1_ready)
static void carve(AggArgs& a, void* scratch, int64_t n_max, int64_t n_p1) {
  const int64_t nm = hid_rows(n_max);
  a.p1 = static_cast<float*>(scratch);
  a.hid = a.p1 + (n_p1 > 0 ? n_p1 : 1) * kHid;
  a.vmask = reinterpret_cast<int32_t*>(a.hid + nm * kHid);
}
static int32_t* tile_counter(const AggArgs& a, int64_t n_max) {
  const int64_t nm = hid_rows(n_max);
  return a.vmask + cdiv(nm, 4) * 4;
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
  PNR_CHECK_ARG(!pts->used || (pts->used_map && pts->n_used >= 0 && pts->n_used <= pts->n),
                "aggregate: used list needs used_map and 0 <= n_used <= n");
  PNR_CHECK_ARG(scratch_bytes >= scratch_need(s->n_max, pts->used ? pts->n_used : pts->n),
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
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  return launch(a, as_stream(stream), false);
}

extern "C" int pnr_aggregate_fwd_x3(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                    const pnr_mlp_x3* wx, float* out_feat, float* out_weight, float* out_conf,
                                    void* scratch, size_t scratch_bytes, void* stream) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate_x3: need pers or camera");
  PNR_CHECK_ARG(s->pidx, "aggregate_x3: pidx required");
  PNR_CHECK_ARG(wx && wx->w1bx && wx->w2x && wx->w3x && wx->w4x, "aggregate_x3: null split weight pack");
  PNR_CHECK_ARG(w->neg_slope >= 0.f && w->neg_slope <= 1.f, "aggregate_x3: LeakyReLU slope must be in [0, 1]");
  PNR_CHECK_ARG((((uintptr_t)wx->w1bx | (uintptr_t)wx->w2x | (uintptr_t)wx->w3x | (uintptr_t)wx->w4x) & 15) == 0,
                "aggregate_x3: split packs must be 16-B aligned");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  hipStream_t st = as_stream(stream);
  // k_point_pre (fp32 P1) -> k_pairs_x3 (aggregate_x3.hip) -> k_color
  if ((rc = launch_t<false>(a, st, kStagePre))) return rc;
  SplitW sw = {{wx->w1bx, wx->w2x, wx->w3x, wx->w4x}, {1.f, 1.f, 1.f, 1.f}, nullptr};
  if ((rc = launch_pairs_split<false>(a.pts, a.s, a.w, sw, a.p1, a.hid, a.vmask, out_feat, out_weight, out_conf,
                                      tile_counter(a, s->n_max), st)))
    return rc;
  return launch_t<false>(a, st, kStageColor);
}

extern "C" int pnr_aggregate_fwd_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                    const pnr_mlp_h2* wh, float* out_feat, float* out_weight, float* out_conf,
                                    void* scratch, size_t scratch_bytes, void* stream) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate_h2: need pers or camera");
  PNR_CHECK_ARG(s->pidx, "aggregate_h2: pidx required");
  PNR_CHECK_ARG(wh && wh->w1bh && wh->w2h && wh->w3h && wh->w4h, "aggregate_h2: null split weight pack");
  PNR_CHECK_ARG(w->neg_slope >= 0.f && w->neg_slope <= 1.f, "aggregate_h2: LeakyReLU slope must be in [0, 1]");
  PNR_CHECK_ARG((((uintptr_t)wh->w1bh | (uintptr_t)wh->w2h | (uintptr_t)wh->w3h | (uintptr_t)wh->w4h) & 15) == 0,
                "aggregate_h2: split packs must be 16-B aligned");
  for (int i = 0; i < 4; ++i)
    PNR_CHECK_ARG(wh->scale[i] > 0.f && wh->scale[i] < 1e30f, "aggregate_h2: bad layer scale %d", i);
  if (wh->w1ah)
    PNR_CHECK_ARG(((uintptr_t)wh->w1ah & 15) == 0 && wh->scale1a > 0.f && wh->scale1a < 1e30f,
                  "aggregate_h2: bad block1.0 point-half pack");
  if (wh->wc1a) {
    PNR_CHECK_ARG(wh->wc1b && wh->wc2h && wh->wc3h, "aggregate_h2: partial colour-branch packs");
    PNR_CHECK_ARG((((uintptr_t)wh->wc1a | (uintptr_t)wh->wc1b | (uintptr_t)wh->wc2h | (uintptr_t)wh->wc3h) & 15) == 0,
                  "aggregate_h2: colour packs must be 16-B aligned");
    for (int i = 0; i < 3; ++i)
      PNR_CHECK_ARG(wh->cscale[i] > 0.f && wh->cscale[i] < 1e30f, "aggregate_h2: bad colour layer scale %d", i);
  }
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  hipStream_t st = as_stream(stream);
  SplitW sw = {{wh->w1bh, wh->w2h, wh->w3h, wh->w4h},
               {wh->scale[0], wh->scale[1], wh->scale[2], wh->scale[3]},
               wh->range_flag};
  // k_point_pre_h2 / k_point_pre (P1) -> k_pairs_h2 (aggregate_x3.hip) -> k_color_h2 / k_color
  if (wh->w1ah) {
    if (!a.pts.p1_ready && (rc = launch_point_pre_h2(a.pts, wh->w1ah, wh->scale1a, wh->range_flag, a.p1, st)))
      return rc;
  } else if ((rc = launch_t<false>(a, st, kStagePre))) {
    return rc;
  }
  if ((rc = launch_pairs_split<true>(a.pts, a.s, a.w, sw, a.p1, a.hid, a.vmask, out_feat, out_weight, out_conf,
                                     tile_counter(a, s->n_max), st)))
    return rc;
  if (wh->wc1a) {
    const void* cp[4] = {wh->wc1a, wh->wc1b, wh->wc2h, wh->wc3h};
    return launch_color_h2(a.s, a.w, cp, wh->cscale, wh->range_flag, a.hid, a.vmask, out_feat, st, a.pts.rw2c);
  }
  return launch_t<false>(a, st, kStageColor);
}

extern "C" int pnr_point_pre_h2(const pnr_points* pts, const pnr_mlp_h2* wh, void* scratch, size_t scratch_bytes,
                                void* stream) {
  PNR_CHECK_ARG(pts && wh && pts->emb && scratch, "point_pre_h2: null pointer");
  PNR_CHECK_ARG(wh->w1ah && ((uintptr_t)wh->w1ah & 15) == 0 && wh->scale1a > 0.f && wh->scale1a < 1e30f,
                "point_pre_h2: bad block1.0 point-half pack");
  PNR_CHECK_ARG(((uintptr_t)pts->emb & 15) == 0 && ((uintptr_t)scratch & 15) == 0,
                "point_pre_h2: emb and scratch must be 16-B aligned");
  const int64_t n_p1 = pts->used ? pts->n_used : pts->n;
  PNR_CHECK_ARG(n_p1 >= 0 && scratch_bytes >= (size_t)(n_p1 > 0 ? n_p1 : 1) * kHid * sizeof(float),
                "point_pre_h2: scratch too small for the P1 rows");
  if (n_p1 == 0) return PNR_OK;
  return launch_point_pre_h2(*pts, wh->w1ah, wh->scale1a, wh->range_flag, static_cast<float*>(scratch),
                             as_stream(stream));
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
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = pair_mask;
  return launch(a, as_stream(stream), false);
}

static int check_saved(const pnr_agg_saved* sv) {
  PNR_CHECK_ARG(sv, "aggregate train: null saved struct");
  PNR_CHECK_ARG(sv->h1 && sv->h2 && sv->h3 && sv->h4 && sv->pe5 && sv->x3e && sv->pa && sv->wt && sv->wn &&
                    sv->prow && sv->hid && sv->vpe && sv->hc1 && sv->hc2 && sv->hc3 && sv->vmask && sv->mask,
                "aggregate train: null saved array");
  PNR_CHECK_ARG((((uintptr_t)sv->h1 | (uintptr_t)sv->h2 | (uintptr_t)sv->h3 | (uintptr_t)sv->h4 |
                  (uintptr_t)sv->hid | (uintptr_t)sv->hc1 | (uintptr_t)sv->hc2 | (uintptr_t)sv->hc3) & 15) == 0,
                "aggregate train: saved activations must be 16-B aligned");
  return PNR_OK;
}

extern "C" int pnr_aggregate_fwd_train(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                       const pnr_agg_saved* saved, float* out_feat, float* out_weight,
                                       float* out_conf, void* scratch, size_t scratch_bytes, void* stream) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  if ((rc = check_saved(saved))) return rc;
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate: need pers or camera");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  a.sv = *saved;
  a.hid = saved->hid;
  a.vmask = saved->vmask;
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  return launch(a, as_stream(stream), true);
}

extern "C" int pnr_aggregate_fwd_train_x3(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                          const pnr_mlp_x3* wx, const pnr_agg_saved* saved, float* out_feat,
                                          float* out_weight, float* out_conf, void* scratch, size_t scratch_bytes,
                                          void* stream) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  if ((rc = check_saved(saved))) return rc;
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate_train_x3: need pers or camera");
  PNR_CHECK_ARG(s->pidx, "aggregate_train_x3: pidx required");
  PNR_CHECK_ARG(wx && wx->w1bx && wx->w2x && wx->w3x && wx->w4x, "aggregate_train_x3: null split weight pack");
  PNR_CHECK_ARG(w->neg_slope >= 0.f && w->neg_slope <= 1.f, "aggregate_train_x3: LeakyReLU slope must be in [0, 1]");
  PNR_CHECK_ARG((((uintptr_t)wx->w1bx | (uintptr_t)wx->w2x | (uintptr_t)wx->w3x | (uintptr_t)wx->w4x) & 15) == 0,
                "aggregate_train_x3: split packs must be 16-B aligned");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  int32_t* tile_ctr = tile_counter(a, s->n_max);   // in the scratch (before vmask is redirected to the saved one)
  a.sv = *saved;
  a.hid = saved->hid;
  a.vmask = saved->vmask;
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  hipStream_t st = as_stream(stream);
  // k_point_pre (fp32 P1) -> k_pairs_x3_train (aggregate_x3.hip) -> k_color<true>
  if ((rc = launch_t<false>(a, st, kStagePre))) return rc;
  SplitW sw = {{wx->w1bx, wx->w2x, wx->w3x, wx->w4x}, {1.f, 1.f, 1.f, 1.f}, nullptr};
  if ((rc = launch_pairs_split<false>(a.pts, a.s, a.w, sw, a.p1, a.hid, a.vmask, out_feat, out_weight, out_conf,
                                      tile_ctr, st, saved)))
    return rc;
  return launch_t<true>(a, st, kStageColor);
}

static int fwd_train_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w, const pnr_mlp_h2* wh,
                        const pnr_agg_saved* saved, float* out_feat, float* out_weight, float* out_conf,
                        void* scratch, size_t scratch_bytes, void* stream, bool guarded) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  if ((rc = check_saved(saved))) return rc;
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate_train_h2: need pers or camera");
  PNR_CHECK_ARG(s->pidx, "aggregate_train_h2: pidx required");
  PNR_CHECK_ARG(wh && wh->w1bh && wh->w2h && wh->w3h && wh->w4h, "aggregate_train_h2: null split weight pack");
  PNR_CHECK_ARG(w->neg_slope >= 0.f && w->neg_slope <= 1.f, "aggregate_train_h2: LeakyReLU slope must be in [0, 1]");
  PNR_CHECK_ARG((((uintptr_t)wh->w1bh | (uintptr_t)wh->w2h | (uintptr_t)wh->w3h | (uintptr_t)wh->w4h) & 15) == 0,
                "aggregate_train_h2: split packs must be 16-B aligned");
  for (int i = 0; i < 4; ++i)
    PNR_CHECK_ARG(wh->scale[i] > 0.f && wh->scale[i] < 1e30f, "aggregate_train_h2: bad layer scale %d", i);
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  int32_t* tile_ctr = tile_counter(a, s->n_max);   // in the scratch (before vmask is redirected to the saved one)
  a.sv = *saved;
  a.hid = saved->hid;
  a.vmask = saved->vmask;
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = nullptr;
  hipStream_t st = as_stream(stream);
  // k_point_pre_h2 (P1 on fp32h2 when wh->w1ah is given) / k_point_pre -> k_pairs_h2_train
  // (aggregate_x3.hip) -> k_color<true>
  if (wh->w1ah) {
    PNR_CHECK_ARG(((uintptr_t)wh->w1ah & 15) == 0 && wh->scale1a > 0.f && wh->scale1a < 1e30f,
                  "aggregate_train_h2: bad block1.0 point-half pack");
    PNR_CHECK_ARG(((uintptr_t)saved->x1 & 15) == 0, "aggregate_train_h2: saved x1 must be 16-B aligned");
    if ((rc = launch_point_pre_h2(a.pts, wh->w1ah, wh->scale1a, wh->range_flag, a.p1, st, saved->x1))) return rc;
  } else if ((rc = launch_t<false>(a, st, kStagePre))) {
    return rc;
  }
  SplitW sw = {{wh->w1bh, wh->w2h, wh->w3h, wh->w4h},
               {wh->scale[0], wh->scale[1], wh->scale[2], wh->scale[3]},
               wh->range_flag};
  if ((rc = launch_pairs_split<true>(a.pts, a.s, a.w, sw, a.p1, a.hid, a.vmask, out_feat, out_weight, out_conf,
                                     tile_ctr, st, saved)))
    return rc;
  if (guarded) {   // the native-fp32 chain over the same outputs, run on the device only if the flag is up
    AggArgs f = a;
    f.run_if = wh->range_flag;
    f.pts.p1_ready = wh->w1ah ? 0 : 1;   // P1 again on fp32 when k_point_pre_h2 made it
    if ((rc = launch_t<true>(f, st, kStagePre | kStagePairs))) return rc;
  }
  if (wh->wc1a && wh->wc1b && wh->wc2h && wh->wc3h) {
    // the colour branch on f16-split MFMA too (k_color_h2<true>: the same saves as
    // k_color<true>), its fp32 rerun behind it when the flag is up (guarded)
    PNR_CHECK_ARG((((uintptr_t)wh->wc1a | (uintptr_t)wh->wc1b | (uintptr_t)wh->wc2h | (uintptr_t)wh->wc3h) & 15) == 0,
                  "aggregate_train_h2: colour packs must be 16-B aligned");
    for (int i = 0; i < 3; ++i)
      PNR_CHECK_ARG(wh->cscale[i] > 0.f && wh->cscale[i] < 1e30f, "aggregate_train_h2: bad colour scale %d", i);
    const void* cp[4] = {wh->wc1a, wh->wc1b, wh->wc2h, wh->wc3h};
    if ((rc = launch_color_h2(a.s, a.w, cp, wh->cscale, wh->range_flag, saved->hid, a.vmask, out_feat, st,
                              a.pts.rw2c, saved)))
      return rc;
    if (!guarded) return PNR_OK;
    AggArgs f = a;
    f.run_if = wh->range_flag;
    return launch_t<true>(f, st, kStageColor);
  }
  return launch_t<true>(a, st, kStageColor);
}

extern "C" int pnr_aggregate_fwd_train_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                          const pnr_mlp_h2* wh, const pnr_agg_saved* saved, float* out_feat,
                                          float* out_weight, float* out_conf, void* scratch, size_t scratch_bytes,
                                          void* stream) {
  return fwd_train_h2(pts, s, w, wh, saved, out_feat, out_weight, out_conf, scratch, scratch_bytes, stream, false);
}

extern "C" int pnr_aggregate_fwd_train_h2_guarded(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                                  const pnr_mlp_h2* wh, const pnr_agg_saved* saved,
                                                  float* out_feat, float* out_weight, float* out_conf,
                                                  void* scratch, size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(wh && wh->range_flag, "aggregate_train_h2_guarded: range_flag required");
  return fwd_train_h2(pts, s, w, wh, saved, out_feat, out_weight, out_conf, scratch, scratch_bytes, stream, true);
}

extern "C" int pnr_aggregate_fwd_train_masked(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                              const uint8_t* pair_mask, const pnr_agg_saved* saved,
                                              float* out_feat, float* out_weight, float* out_conf,
                                              void* scratch, size_t scratch_bytes, void* stream) {
  int rc;
  if ((rc = check_common(pts, s, w, out_feat, static_cast<float*>(scratch), scratch_bytes))) return rc;
  if ((rc = check_saved(saved))) return rc;
  PNR_CHECK_ARG(pair_mask, "aggregate_masked: null pair_mask");
  PNR_CHECK_ARG(pts->pers, "aggregate_masked: pers required");
  PNR_CHECK_ARG(s->pidx == nullptr, "aggregate_masked: pidx must be NULL (identity rows)");
  if (s->n_max <= 0) return PNR_OK;
  AggArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  carve(a, scratch, s->n_max, pts->used ? pts->n_used : pts->n);
  a.sv = *saved;
  a.hid = saved->hid;
  a.vmask = saved->vmask;
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.pair_mask = pair_mask;
  return launch(a, as_stream(stream), true);
}

static int bwd_pairs(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w, const pnr_mlp_bwd* wb,
                     const pnr_mlp_bwd_x3* wbx, const pnr_mlp_bwd_h2* wbh, const pnr_agg_saved* saved,
                     const float* d_feat,
                     const float* d_hid, float* dz1, float* dz2, float* dz3, float* dz4, float* dpa, float* d_p1,
                     float* d_color, float* d_dir, float* d_conf, void* stream) {
  int rc;
  PNR_CHECK_ARG(pts && s && w && wb, "aggregate_bwd: null pointer");
  if ((rc = check_saved(saved))) return rc;
  PNR_CHECK_ARG((wb->w3e || wbx || wbh) && w->wa && (wbx || wbh || (wb->w4t && wb->w3t && wb->w2t)),
                "aggregate_bwd: null weight");
  PNR_CHECK_ARG(!wbh || (wbh->w4th && wbh->w3th && wbh->w2th && wbh->scale &&
                         (((uintptr_t)wbh->w4th | (uintptr_t)wbh->w3th | (uintptr_t)wbh->w2th) & 15) == 0),
                "aggregate_bwd_h2: null or unaligned split weight pack");
  PNR_CHECK_ARG(!wbx || (wbx->w4tx && wbx->w3tx && wbx->w2tx &&
                         (((uintptr_t)wbx->w4tx | (uintptr_t)wbx->w3tx | (uintptr_t)wbx->w2tx) & 15) == 0),
                "aggregate_bwd_x3: null or unaligned split weight pack");
  PNR_CHECK_ARG(d_feat && d_hid && dz1 && dz2 && dz3 && dz4 && dpa, "aggregate_bwd: null buffer");
  PNR_CHECK_ARG((((uintptr_t)d_hid | (uintptr_t)dz1 | (uintptr_t)dz2 | (uintptr_t)dz3 | (uintptr_t)dz4) & 15) == 0,
                "aggregate_bwd: gradient buffers must be 16-B aligned");
  PNR_CHECK_ARG(s->dirs && s->dir_div >= 1, "aggregate_bwd: sample dirs required");
  PNR_CHECK_ARG(s->K >= 1 && s->K <= kKN, "aggregate_bwd: K=%d unsupported (1..8)", s->K);
  if (s->n_max <= 0) return PNR_OK;
  hipStream_t st = as_stream(stream);
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_bwd<0>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBwdLdsBytes));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_bwd<1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBwdLdsBytes));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_bwd<2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBwdLdsBytes));
    attr = true;
  }
  BwdArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  a.wb = *wb;
  a.sv = *saved;
  a.d_feat = d_feat;
  a.d_hid = d_hid;
  a.dz[0] = dz1;
  a.dz[1] = dz2;
  a.dz[2] = dz3;
  a.dz[3] = dz4;
  a.dpa = dpa;
  a.d_p1 = d_p1;
  a.d_color = d_color;
  a.d_dir = d_dir;
  a.d_conf = d_conf;
  a.wx[0] = wbx ? wbx->w4tx : (wbh ? wbh->w4th : nullptr);
  a.wx[1] = wbx ? wbx->w3tx : (wbh ? wbh->w3th : nullptr);
  a.wx[2] = wbx ? wbx->w2tx : (wbh ? wbh->w2th : nullptr);
  a.wxs = wbh ? wbh->scale : nullptr;
  const int64_t tiles = cdiv(s->n_max, kTS);
  if (wbx || wbh) {
    if (wbh)
      hipLaunchKernelGGL(k_pairs_bwd<2>, dim3(grid_for(tiles, 1, 256 * 2)), dim3(64 * kPairWaves), kBwdLdsBytes,
                         st, a);
    else
      hipLaunchKernelGGL(k_pairs_bwd<1>, dim3(grid_for(tiles, 1, 256 * 2)), dim3(64 * kPairWaves), kBwdLdsBytes,
                         st, a);
    PNR_LAUNCH_CHECK();
    // wb->w3e == NULL: the caller runs the extras per point inside
    // pnr_pairs_to_points_ex (no float atomics, coalesced dz3 rows)
    if ((d_color || d_dir) && wb->w3e)
      hipLaunchKernelGGL(k_extras_bwd, dim3(grid_for(cdiv(s->n_max * kKN, 64), 4, 2048)), dim3(256), 0, st, a);
  } else
    hipLaunchKernelGGL(k_pairs_bwd<0>, dim3(grid_for(tiles, 1, 256 * 2)), dim3(64 * kPairWaves), kBwdLdsBytes,
                       st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_aggregate_bwd_pairs(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                       const pnr_mlp_bwd* wb, const pnr_agg_saved* saved,
                                       const float* d_feat, const float* d_hid, float* dz1, float* dz2,
                                       float* dz3, float* dz4, float* dpa, float* d_p1, float* d_color,
                                       float* d_dir, float* d_conf, void* stream) {
  return bwd_pairs(pts, s, w, wb, nullptr, nullptr, saved, d_feat, d_hid, dz1, dz2, dz3, dz4, dpa, d_p1, d_color,
                   d_dir, d_conf, stream);
}

extern "C" int pnr_aggregate_bwd_pairs_x3(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                          const pnr_mlp_bwd* wb, const pnr_mlp_bwd_x3* wbx,
                                          const pnr_agg_saved* saved, const float* d_feat, const float* d_hid,
                                          float* dz1, float* dz2, float* dz3, float* dz4, float* dpa, float* d_p1,
                                          float* d_color, float* d_dir, float* d_conf, void* stream) {
  PNR_CHECK_ARG(wbx, "aggregate_bwd_x3: null split weight packs");
  return bwd_pairs(pts, s, w, wb, wbx, nullptr, saved, d_feat, d_hid, dz1, dz2, dz3, dz4, dpa, d_p1, d_color, d_dir,
                   d_conf, stream);
}

extern "C" int pnr_aggregate_bwd_pairs_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                          const pnr_mlp_bwd* wb, const pnr_mlp_bwd_h2* wbh,
                                          const pnr_agg_saved* saved, const float* d_feat, const float* d_hid,
                                          float* dz1, float* dz2, float* dz3, float* dz4, float* dpa, float* d_p1,
                                          float* d_color, float* d_dir, float* d_conf, void* stream) {
  PNR_CHECK_ARG(wbh, "aggregate_bwd_h2: null split weight packs");
  return bwd_pairs(pts, s, w, wb, nullptr, wbh, saved, d_feat, d_hid, dz1, dz2, dz3, dz4, dpa, d_p1, d_color, d_dir,
                   d_conf, stream);
}

// ---------------------------------------------------------------------------
// d xyz (--xyz_grad 1, neural_points.py:270): the point position enters the
// pair through sampled_xyz (neural_points.py:788-799) -- the world distance
// d = p - s_w, rotated into PE_5's first three channels and giving the inverse-
// distance weight w = 1 / max(|d|, 1e-6), normalised over the K slots
// (point_aggregators.py:775-804) -- and through sampled_xyz_pers =
// w2pers(p) (neural_points.py:635, qpiw.py:102-109), whose deltas
// (x z - x_s z_s, y z - y_s z_s, z - z_s) are PE_5's last three channels.  One
// thread per pair (8 lanes = a sample's K slots, xor8 sums the weight
// normalisation), given d PE_5 = dz1 . W1[:, 224:284] (pnr_gemm_nn) and
// d wt = d alpha a_k + <d hid, h4_k>; atomics into d_xyz.
struct XyzBwdArgs {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp w;
  pnr_agg_saved sv;
  const float* d_feat;   // [n,129]
  const float* d_hid;    // [n,256]
  const float* d_pe;     // [n*8,64] (columns 60..63 unused)
  float* d_xyz;          // [N,3] (+=)
};

__global__ void __launch_bounds__(256) k_xyz_bwd(XyzBwdArgs A) {
  const int64_t n = eff_n(A.s);
  const int64_t pair = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t v = pair >> 3;
  if (v >= n) return;   // whole 8-lane groups
  const int32_t pr = A.sv.prow[pair];
  const bool valid = pr >= 0;
  const int64_t row = sample_row(A.s, v);
  float pw[3] = {0.f, 0.f, 0.f}, d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (valid) pw[a] = A.pts.xyz[(int64_t)pr * 3 + a];
    d[a] = pw[a] - A.s.sample_w[row * 3 + a];
  }
  const float nrm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  const float wl = valid ? 1.f / fmaxf(nrm, 1e-6f) : 0.f;
  const float S = xor8_sum(wl);
  // d wt_k: alpha_s = sum_k wt_k a_k, f_s = sum_k wt_k h4_k
  float dwt = 0.f;
  if (valid && A.sv.vmask[v] != 0) {
    const float pa = A.sv.pa[pair];
    const float a_k = A.w.act_super ? softplus(pa - 1.f) : fmaxf(pa, 0.f);
    const float4* h4 = reinterpret_cast<const float4*>(A.sv.h4 + pair * kHid);
    const float4* dh = reinterpret_cast<const float4*>(A.d_hid + v * kHid);
    float dot = 0.f;
#pragma unroll 8
    for (int q = 0; q < kHid / 4; ++q) {
      const float4 x = h4[q], y = dh[q];
      dot += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    dwt = A.d_feat[v * (kC + 1)] * a_k + dot;
  }
  // wt = wn clamp(conf), wn_k = wl_k / max(S, 1e-8)
  const float confc = (valid && A.pts.conf) ? fminf(fmaxf(A.pts.conf[pr], 1e-4f), 1.f) : 1.f;
  const float dwn = dwt * confc;
  const float dS = S >= 1e-8f ? -xor8_sum(dwn * wl) / (S * S) : 0.f;
  const float dwl = dwn / fmaxf(S, 1e-8f) + dS;
  if (!valid) return;
  float g[3] = {0.f, 0.f, 0.f};
  if (nrm > 1e-6f) {
    const float dn = -dwl / (nrm * nrm * nrm);   // d(1/|d|) / dd = -d / |d|^3
#pragma unroll
    for (int a = 0; a < 3; ++a) g[a] = dn * d[a];
  }
  // PE_5: value 2(5c + f) = sin(2^f x_c), + 1 = cos(2^f x_c)
  const float* pe = A.sv.pe5 + pair * 64;
  const float* gp = A.d_pe + pair * 64;
  float dd[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    float acc = 0.f;
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      const int j = 2 * (5 * c + f);
      acc += (float)(1 << f) * (pe[j + 1] * gp[j] - pe[j] * gp[j + 1]);
    }
    dd[c] = acc;
  }
  // channels 0..2: R.d (d_i gets sum_j R[j][i] dd_j)
  float Rw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
  if (A.pts.rw2c) {   // per-point Rw2c: the pair's own matrix
#pragma unroll
    for (int i = 0; i < 9; ++i) Rw[i] = A.pts.rw2c[(int64_t)pr * 9 + i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) g[i] += Rw[i] * dd[0] + Rw[3 + i] * dd[1] + Rw[6 + i] * dd[2];
  // channels 3..5 through the perspective coordinates of the pair's camera
  float c3[3], R[9];
  const int64_t cam = A.s.ray_cam ? (int64_t)A.s.ray_cam[dir_row(A.s, row)] : 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) c3[i] = A.pts.campos[cam * 3 + i];
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = A.pts.camrot[cam * 9 + i];
  float xc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j)
    xc[j] = (pw[0] - c3[0]) * R[j] + (pw[1] - c3[1]) * R[3 + j] + (pw[2] - c3[2]) * R[6 + j];
  const float pp[3] = {xc[0] / xc[2], xc[1] / xc[2], xc[2]};
  const float dp0 = dd[3] * pp[2], dp1 = dd[4] * pp[2], dp2 = dd[3] * pp[0] + dd[4] * pp[1] + dd[5];
  const float iz = 1.f / xc[2];
  const float dx0 = dp0 * iz, dx1 = dp1 * iz, dx2 = dp2 - (dp0 * pp[0] + dp1 * pp[1]) * iz;
#pragma unroll
  for (int i = 0; i < 3; ++i) g[i] += R[i * 3] * dx0 + R[i * 3 + 1] * dx1 + R[i * 3 + 2] * dx2;
#pragma unroll
  for (int i = 0; i < 3; ++i) atomicAdd(A.d_xyz + (int64_t)pr * 3 + i, g[i]);
}

extern "C" int pnr_aggregate_bwd_xyz(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                     const pnr_agg_saved* saved, const float* d_feat, const float* d_hid,
                                     const float* d_pe, float* d_xyz, void* stream) {
  PNR_CHECK_ARG(pts && s && w && saved && d_feat && d_hid && d_pe && d_xyz, "aggregate_bwd_xyz: null argument");
  PNR_CHECK_ARG(pts->xyz && pts->campos && pts->camrot, "aggregate_bwd_xyz: need xyz and the camera tables");
  PNR_CHECK_ARG(saved->prow && saved->pa && saved->h4 && saved->pe5 && saved->vmask,
                "aggregate_bwd_xyz: missing saved activations");
  PNR_CHECK_ARG(s->K <= kKN, "aggregate_bwd_xyz: K > %d", kKN);
  if (s->n_max <= 0) return PNR_OK;
  XyzBwdArgs a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  a.sv = *saved;
  a.d_feat = d_feat;
  a.d_hid = d_hid;
  a.d_pe = d_pe;
  a.d_xyz = d_xyz;
  hipLaunchKernelGGL(k_xyz_bwd, dim3((unsigned)cdiv(s->n_max * kKN, 256)), dim3(256), 0, as_stream(stream), a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// flags: the bytes [32 * nw] | the bitset [nw] (fits the caller's int32 [n_points]
// only from 64 points up: below, both live in scratch); scratch: the word prefix
// [nw + 1] | (small n: bytes + bits) | the scan's scratch, each 16-B padded
static size_t pad16(size_t b) { return (b + 15) & ~(size_t)15; }
static bool used_small(int64_t n_points) { return cdiv(n_points, 32) * 36 > n_points * 4; }
static size_t used_head_bytes(int64_t n_points) {
  const int64_t nw = cdiv(n_points, 32);
  return pad16((size_t)(nw + 1) * 4) + (used_small(n_points) ? pad16((size_t)nw * 36) : 0);
}

extern "C" int pnr_used_points_scratch_bytes(int64_t n_points, size_t* out) {
  PNR_CHECK_ARG(out && n_points >= 0, "used_points_scratch_bytes: bad args");
  *out = used_head_bytes(n_points) + scan_scratch_bytes(cdiv(n_points, 32));
  return PNR_OK;
}

extern "C" int pnr_used_points(const int32_t* pidx, const int32_t* n_samples_dev, int32_t K, int64_t cap_samples,
                               int64_t n_points, int32_t* flags, int32_t* used_map, int32_t* used, int32_t* n_used_dev,
                               void* scratch, size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(pidx && flags && used_map && used && n_used_dev && scratch && K > 0 && cap_samples >= 0 &&
                    n_points > 0, "used_points: bad args");
  const int64_t nw = cdiv(n_points, 32);
  const size_t hb = used_head_bytes(n_points);
  PNR_CHECK_ARG(scratch_bytes >= hb + scan_scratch_bytes(nw), "used_points: scratch too small (%zu < %zu)",
                scratch_bytes, hb + scan_scratch_bytes(nw));
  PNR_CHECK_ARG(((uintptr_t)flags & 15) == 0 && ((uintptr_t)scratch & 15) == 0,
                "used_points: flags / scratch must be 16-B aligned");
  hipStream_t st = as_stream(stream);
  int32_t* wpre = static_cast<int32_t*>(scratch);
  uint8_t* bytes = used_small(n_points) ? static_cast<uint8_t*>(scratch) + pad16((size_t)(nw + 1) * 4)
                                        : reinterpret_cast<uint8_t*>(flags);
  uint32_t* bits = reinterpret_cast<uint32_t*>(bytes + nw * 32);
  PNR_HIP(hipMemsetAsync(bytes, 0, (size_t)nw * 32, st));
  if (cap_samples > 0) {
    hipLaunchKernelGGL(k_mark_used, dim3(grid_for(cap_samples * K, 256)), dim3(256), 0, st, pidx, n_samples_dev, K,
                       cap_samples, bytes);
    PNR_LAUNCH_CHECK();
  }
  // the words' popcounts go through `used` (n_points >= nw entries, written after)
  hipLaunchKernelGGL(k_pack_used, dim3(grid_for(nw, 256)), dim3(256), 0, st, bytes, nw, bits, used);
  PNR_LAUNCH_CHECK();
  int rc;
  if ((rc = exclusive_scan(used, nw, nullptr, wpre, nw + 1, n_used_dev, static_cast<char*>(scratch) + hb,
                           scratch_bytes - hb, st, 0)))
    return rc;
  hipLaunchKernelGGL(k_used_list, dim3(grid_for(n_points, 256)), dim3(256), 0, st, bits, wpre, n_points, used_map,
                     used);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_aggregate_bwd_extras_rows(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                             const pnr_agg_saved* saved, const float* w3e, const float* dz3,
                                             float* g_pair, void* stream) {
  PNR_CHECK_ARG(pts && s && w && saved && saved->prow && w3e, "aggregate_bwd_extras_rows: null pointer");
  PNR_CHECK_ARG(s->n_max == 0 || (dz3 && g_pair && (((uintptr_t)dz3 | (uintptr_t)g_pair) & 15) == 0),
                "aggregate_bwd_extras_rows: dz3 / g_pair must be 16-B aligned");
  PNR_CHECK_ARG(s->dirs && s->dir_div >= 1, "aggregate_bwd_extras_rows: sample dirs required");
  if (s->n_max <= 0) return PNR_OK;
  BwdArgs a;
  memset(&a, 0, sizeof(a));
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  a.sv = *saved;
  a.wb.w3e = w3e;
  a.dz[2] = const_cast<float*>(dz3);
  hipLaunchKernelGGL(k_extras_rows, dim3(grid_for(s->n_max * kKN, 64, 4096)), dim3(256), 0, as_stream(stream), a,
                     g_pair);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_pairs_to_points_ex(const int32_t* prow_sorted, const int32_t* pair_of, int64_t P,
                                      const float* dz1, const int32_t* used_map, float* d_p1, uint32_t* d_p1_absmax,
                                      const float* g_pair, const float* rw_uniform, const float* rw_pp,
                                      float* d_color, float* d_dir, void* stream) {
  PNR_CHECK_ARG(P >= 0 && (P == 0 || (prow_sorted && pair_of && dz1 && d_p1 && g_pair)),
                "pairs_to_points_ex: bad args");
  PNR_CHECK_ARG((((uintptr_t)dz1 | (uintptr_t)d_p1) & 15) == 0, "pairs_to_points_ex: rows must be 16-B aligned");
  if (P == 0) return PNR_OK;
  hipLaunchKernelGGL(k_pairs_to_points_ex, dim3(grid_for(cdiv(P, 64), 4, 2048)), dim3(256), 0, as_stream(stream), prow_sorted,
                     pair_of, P, dz1, used_map, d_p1, d_p1_absmax, g_pair, rw_uniform, rw_pp, d_color, d_dir);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_point_counts(const int32_t* pidx, const int32_t* n_dev, int32_t K, int64_t cap, float* counts,
                                void* stream) {
  PNR_CHECK_ARG(n_dev && K > 0 && cap >= 0 && (cap == 0 || (pidx && counts)), "point_counts: bad args");
  if (cap == 0) return PNR_OK;
  hipLaunchKernelGGL(k_point_counts, dim3(grid_for(cap * K, 256, 2048)), dim3(256), 0, as_stream(stream), pidx,
                     n_dev, K, cap, counts);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_pairs_to_points(const int32_t* prow_sorted, const int32_t* pair_of, int64_t P, const float* dz1,
                                   const int32_t* used_map, float* d_p1, uint32_t* d_p1_absmax, void* stream) {
  PNR_CHECK_ARG(P >= 0 && (P == 0 || (prow_sorted && pair_of && dz1 && d_p1)), "pairs_to_points: bad args");
  PNR_CHECK_ARG((((uintptr_t)dz1 | (uintptr_t)d_p1) & 15) == 0, "pairs_to_points: rows must be 16-B aligned");
  if (P == 0) return PNR_OK;
  hipLaunchKernelGGL(k_pairs_to_points, dim3(grid_for(cdiv(P, 64), 4, 2048)), dim3(256), 0, as_stream(stream), prow_sorted,
                     pair_of, P, dz1, used_map, d_p1, d_p1_absmax);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_point_pe3(const float* emb, int64_t n, float* x1, void* stream) {
  PNR_CHECK_ARG(emb && x1 && n >= 0, "point_pe3: bad args");
  if (n == 0) return PNR_OK;
  hipLaunchKernelGGL(k_point_pe3, dim3(grid_for(n * kEmb, 256)), dim3(256), 0, as_stream(stream), emb, nullptr, n,
                     x1);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_point_pe3_bwd(const float* emb, const float* d_x1, int64_t n, float* d_emb, void* stream) {
  PNR_CHECK_ARG(emb && d_x1 && d_emb && n >= 0, "point_pe3_bwd: bad args");
  if (n == 0) return PNR_OK;
  hipLaunchKernelGGL(k_point_pe3_bwd, dim3(grid_for(n * kEmb, 256)), dim3(256), 0, as_stream(stream), emb, nullptr,
                     d_x1, n, d_emb);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_point_pe3_rows(const float* emb, const int32_t* rows, int64_t n, float* x1, void* stream) {
  PNR_CHECK_ARG(emb && rows && x1 && n >= 0, "point_pe3_rows: bad args");
  if (n == 0) return PNR_OK;
  hipLaunchKernelGGL(k_point_pe3, dim3(grid_for(n * kEmb, 256)), dim3(256), 0, as_stream(stream), emb, rows, n, x1);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_point_pe3_bwd_rows(const float* emb, const int32_t* rows, const float* d_x1, int64_t n,
                                      float* d_emb, void* stream) {
  PNR_CHECK_ARG(emb && rows && d_x1 && d_emb && n >= 0, "point_pe3_bwd_rows: bad args");
  if (n == 0) return PNR_OK;
  hipLaunchKernelGGL(k_point_pe3_bwd, dim3(grid_for(n * kEmb, 256)), dim3(256), 0, as_stream(stream), emb, rows,
                     d_x1, n, d_emb);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
