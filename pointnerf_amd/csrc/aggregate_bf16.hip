// bf16-MFMA variant of the fused aggregation (SURVEY config c5: "bf16 point
// features + MFMA MLP"): same algorithm and data flow as aggregate.hip, with
// every GEMM on v_mfma_f32_32x32x16_bf16 (bf16 operands, fp32 accumulation,
// 16x the fp32 MFMA rate).  Not the headline path (the reference computes in
// fp32); selected explicitly by the caller.
//
// Layout.  A layer input X is kept in LDS pair-major in bf16, Xb[pair][k]
// (pitch kPB, 16-B aligned rows): the B fragment of k-step t for lane
// (c, h) -- B[k = 16t + 8h + j][col c], j = 0..7 -- is ONE ds_read_b128 at
// Xb[pair c][16t + 8h] (row pitch 560 B spreads 16 lanes over all 64 banks),
// and an accumulator quad (4 consecutive neurons of one pair) is one 8-B
// store.  Weights are fragment-packed (aggregator.frag_pack_bf16):
// W_f[t][T][lane][j] = W'[32T + (lane&31)][16t + 8(lane>>5) + j], one 16-B
// load per lane per (k-step, tile).
//
// Tiles.  A 4-wave workgroup owns 128 (sample, neighbour) pairs = 16 samples
// x K 8 (k_pairs_b; its colour branch runs on the tile's samples) or 128
// points (k_point_pre_b);
// wave w owns output tiles {2w, 2w+1} (256-wide layers) or {w} (128-wide)
// for all four 32-column quarters, so each 1-KB weight fragment feeds 4
// MFMAs.  ~78 KB of LDS per workgroup -> 2 per CU (2 waves per SIMD).
#include "agg_common.h"


namespace pnr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));   // (HIP's uint4 arrays can land in scratch)

constexpr int kBT = 128;                 // columns (pairs / samples / points) per tile
constexpr int kBPT = kBT / 32;           // 32-column quarters per tile
constexpr int kBWaves = 4;
constexpr int kPB = 280;                 // Xb pitch (bf16) for <= 272 input rows (k_pairs_b, k_point_pre_b)
constexpr int kBPad = 6;                 // zero k-steps padded onto bf16 weight packs (the ring's lead)

struct AggArgsB {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp_bf16 w;
  uint16_t* p1;      // [n_p1, 256] bf16 per-point block1.0 partial, accumulator order
  float* out_feat;     // [n, C + 1] fp32 rows, or
  uint16_t* out_feat_h;   // [n, PNR_FEAT_H_PITCH]: alpha fp32 (slots 0-1), C bf16 from slot 8
  float* out_weight;
  float* out_conf;
};

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  bf16x2 p = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, p);
}
__device__ __forceinline__ float bf16_lo(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __builtin_bit_cast(float, u & 0xffff0000u); }
__device__ __forceinline__ uint16_t to_bf16(float a) { return __builtin_bit_cast(uint16_t, (__bf16)a); }

// Y^T += W . X^T on bf16 MFMA: NT output tiles x PT 32-column quarters over
// nsteps k-steps of 16.  Weight fragments WD steps ahead in a register ring
// (raw buffer loads; the packs carry kBPad >= WD zero steps), B fragments one
// step ahead from LDS.  sched_barrier(0) pins the order: without it hipcc sank
// each weight load next to its MFMAs and waited vmcnt(0) on it every k-step
// (the colour kernel of round 4 then ran at 0.14 MFMA busy).
// BROW: the B rows of the last k-step's upper half (16 (nsteps - 1) + 8 .. + 15)
// are the bias row (1) and zeros, whatever Xb holds there (the fused colour
// branch keeps its 280 input rows at pitch kPB: no room for the bias row).
template <int NT, int PT, int NTOT, int PITCH, int WD, bool BROW = false>
__device__ __forceinline__ void mlp_layer_ring(f32x16 (&acc)[PT * NT], const uint4* __restrict__ wf,
                                            const uint16_t* Xb, int nsteps, int lane) {
  static_assert(WD <= kBPad, "the packs' zero steps cover the ring's lead");
  const int c = lane & 31, h = lane >> 5;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(wf), 0, 0x7fffffff, 0x00020000);
  const int voff = lane * 16;
  uint4 w[WD][NT];
  auto ldw = [&](uint4 (&a)[NT], int t) {
#pragma unroll
    for (int T = 0; T < NT; ++T)
      a[T] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, (t * NTOT + T) * 1024, 0));
  };
#pragma unroll
  for (int d = 0; d < WD; ++d) ldw(w[d], d);
  const uint16_t* xr = Xb + c * PITCH + 8 * h;
  uint4 x[2][PT];
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) x[0][pt] = *reinterpret_cast<const uint4*>(xr + 32 * pt * PITCH);
  auto step = [&](int t, int d, int xs) {
    const int tn = t + 1 < nsteps ? t + 1 : t;
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) x[xs ^ 1][pt] = *reinterpret_cast<const uint4*>(xr + 32 * pt * PITCH + 16 * tn);
    if constexpr (BROW) {
      const bool bias = h && tn == nsteps - 1;
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) x[xs ^ 1][pt] = bias ? make_uint4(0x3f80u, 0u, 0u, 0u) : x[xs ^ 1][pt];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int pt = 0; pt < PT; ++pt)
#pragma unroll
      for (int T = 0; T < NT; ++T)
        acc[pt * NT + T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            __builtin_bit_cast(bf16x8, w[d][T]), __builtin_bit_cast(bf16x8, x[xs][pt]), acc[pt * NT + T], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    ldw(w[d], t + WD);   // zero padding past the last step
    __builtin_amdgcn_sched_barrier(0);
  };
  // unrolled by U = lcm(WD, 2): ring slot and B slot compile-time
  constexpr int U = WD % 2 ? 2 * WD : WD;
  int t = 0;
#pragma unroll 1
  for (; t + U <= nsteps; t += U) {
#pragma unroll
    for (int d = 0; d < U; ++d) step(t + d, d % WD, d & 1);
  }
#pragma unroll
  for (int d = 0; d < U - 1; ++d)
    if (t + d < nsteps) step(t + d, d % WD, d & 1);
}

// WD = 0: compiler-scheduled (it loads each step's weights where they are used):
// the k_pairs_b tiles whose registers have no room for a ring (measured faster)
template <int NT, int PT, int NTOT, int PITCH, int WD = 2, bool BROW = false>
__device__ __forceinline__ void mlp_layer_b(f32x16 (&acc)[PT * NT], const uint4* __restrict__ wf,
                                            const uint16_t* Xb, int nsteps, int lane) {
  if constexpr (WD > 0) {
    mlp_layer_ring<NT, PT, NTOT, PITCH, WD, BROW>(acc, wf, Xb, nsteps, lane);
  } else {
    static_assert(!BROW, "bias-row override: ring layers only");
    // the round-4 loop (a0 / a1 and x / y one step ahead as written; hipcc
    // schedules the loads itself)
    const int c = lane & 31, h = lane >> 5;
    const uint4* p = wf + lane;
    uint4 a0[NT], a1[NT];
#pragma unroll
    for (int T = 0; T < NT; ++T) {
      a0[T] = p[(0 * NTOT + T) * 64];
      a1[T] = p[(1 * NTOT + T) * 64];
    }
    const uint16_t* xr = Xb + c * PITCH + 8 * h;
    uint4 x[PT];
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) x[pt] = *reinterpret_cast<const uint4*>(xr + 32 * pt * PITCH);
#pragma unroll 1
    for (int t = 0; t < nsteps; ++t) {
      uint4 y[PT];
      const int tn = t + 1 < nsteps ? t + 1 : t;
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) y[pt] = *reinterpret_cast<const uint4*>(xr + 32 * pt * PITCH + 16 * tn);
#pragma unroll
      for (int pt = 0; pt < PT; ++pt)
#pragma unroll
        for (int T = 0; T < NT; ++T)
          acc[pt * NT + T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              __builtin_bit_cast(bf16x8, a0[T]), __builtin_bit_cast(bf16x8, x[pt]), acc[pt * NT + T], 0, 0, 0);
#pragma unroll
      for (int T = 0; T < NT; ++T) {
        a0[T] = a1[T];
        a1[T] = p[((t + 2) * NTOT + T) * 64];   // packs carry kBPad zero steps
      }
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) x[pt] = y[pt];
    }
  }
}

// Activated accumulators (rows 32(T0+T) + 8q + 4h + i) -> Xb[col][row] bf16.
template <int NT, int PT, int PITCH>
__device__ __forceinline__ void store_act_b(const f32x16 (&acc)[PT * NT], uint16_t* Xb, float s, int lane, int T0) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt)
#pragma unroll
    for (int T = 0; T < NT; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x16& v = acc[pt * NT + T];
        uint2 u;
        u.x = pack_bf16x2(lrelu(v[4 * q], s), lrelu(v[4 * q + 1], s));
        u.y = pack_bf16x2(lrelu(v[4 * q + 2], s), lrelu(v[4 * q + 3], s));
        *reinterpret_cast<uint2*>(Xb + (32 * pt + c) * PITCH + 32 * (T0 + T) + 8 * q + 4 * h) = u;
      }
}

// Accumulators of output rows 32(T0+T) + 8q + 4h + i start at the layer's bias
// (bf16, the value its pack holds in the bias column): the layer then runs
// without its bias k-step (bias rows of Xb neither written nor read).
template <int NT, int PT>
__device__ __forceinline__ void acc_bias_b(f32x16 (&acc)[PT * NT], const uint16_t* bias, int lane, int T0) {
  const int h = lane >> 5;
#pragma unroll
  for (int T = 0; T < NT; ++T)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint2 u = *reinterpret_cast<const uint2*>(bias + 32 * (T0 + T) + 8 * q + 4 * h);
      const float v0 = bf16_lo(u.x), v1 = bf16_hi(u.x), v2 = bf16_lo(u.y), v3 = bf16_hi(u.y);
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) {
        acc[pt * NT + T][4 * q] = v0;
        acc[pt * NT + T][4 * q + 1] = v1;
        acc[pt * NT + T][4 * q + 2] = v2;
        acc[pt * NT + T][4 * q + 3] = v3;
      }
    }
}

// Rows [r0, r0 + 16) of one column: first `nval` from vals, then 1 (bias) if
// bias, then zeros -- the inputs past a layer's last real row.
__device__ __forceinline__ void tail_rows_b(uint16_t* Xb, int pitch, int col, int r0, const float* vals, int nval) {
  unsigned w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float lo = 2 * i < nval ? vals[2 * i] : 0.f;
    const float hi = 2 * i + 1 < nval ? vals[2 * i + 1] : 0.f;
    w[i] = pack_bf16x2(lo, hi);
  }
  uint4* d = reinterpret_cast<uint4*>(Xb + col * pitch + r0);
  d[0] = make_uint4(w[0], w[1], w[2], w[3]);
  d[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// ---------------------------------------------------------------------------
// k_point_pre_b: P1[p] = W1[:, :224] . [emb, PE_3(emb)] + b1 (bf16 result).
__global__ void __launch_bounds__(64 * kBWaves, 2) k_point_pre_b(AggArgsB A) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xb_dyn[];
  uint16_t* Xb = xb_dyn;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int64_t np = p1_rows(A.pts);   // P1 rows
  const int64_t ntiles = cdiv(np, kBT);
  const uint4* wf = reinterpret_cast<const uint4*>(A.w.w1af) + 2 * wid * 64;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // inputs: thread = (point col = tid & 127, half = tid >> 7): channels [16 half, 16 half + 16)
    {
      const int col = threadIdx.x & (kBT - 1), half = threadIdx.x >> 7;
      const int64_t pt = tile * kBT + col;
      const bool act = pt < np;
      const int64_t prow = act ? (A.pts.used ? (int64_t)A.pts.used[pt] : pt) : 0;
      const float* e = A.pts.emb + prow * kEmb + 16 * half;
      const uint2* eb = reinterpret_cast<const uint2*>(A.pts.emb_bf16 + prow * kEmb + 16 * half);
      uint16_t* xc = Xb + col * kPB;
#pragma unroll 2
      for (int q = 0; q < 4; ++q) {
        float ev[4] = {0.f, 0.f, 0.f, 0.f};
        if (act && A.pts.emb_bf16) {   // bf16 table (config c5): 8 B per 4 channels
          const uint2 b = eb[q];
          ev[0] = __uint_as_float(b.x << 16);
          ev[1] = __uint_as_float(b.x & 0xffff0000u);
          ev[2] = __uint_as_float(b.y << 16);
          ev[3] = __uint_as_float(b.y & 0xffff0000u);
        } else if (act) {
          const float4 e4 = reinterpret_cast<const float4*>(e)[q];
          ev[0] = e4.x;
          ev[1] = e4.y;
          ev[2] = e4.z;
          ev[3] = e4.w;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ch = 16 * half + 4 * q + u;
          xc[ch] = to_bf16(ev[u]);
          float s0, c0;
          sincosf(ev[u], &s0, &c0);
          const float s1 = 2.f * s0 * c0, c1 = (c0 - s0) * (c0 + s0);
          const float s2 = 2.f * s1 * c1, c2 = (c1 - s1) * (c1 + s1);
          const int r0 = kEmb + 6 * ch;
          *reinterpret_cast<unsigned*>(xc + r0) = pack_bf16x2(s0, c0);
          *reinterpret_cast<unsigned*>(xc + r0 + 2) = pack_bf16x2(s1, c1);
          *reinterpret_cast<unsigned*>(xc + r0 + 4) = pack_bf16x2(s2, c2);
        }
      }
      if (half == 0) {
        const float one = 1.f;
        tail_rows_b(Xb, kPB, col, 224, &one, 1);   // bias row 224, zeros to 239
      }
    }
    __syncthreads();
    f32x16 acc[kBPT * 2];
#pragma unroll
    for (int i = 0; i < kBPT * 2; ++i) acc[i] = (f32x16){0.f};
    mlp_layer_b<2, kBPT, 8, kPB>(acc, wf, Xb, 15, lane);
#pragma unroll
    for (int pt = 0; pt < kBPT; ++pt) {
      const int64_t row = tile * kBT + 32 * pt + c;
      if (row >= np) continue;
      // used rows without used_map: the table stays indexed by point row (only the
      // rows the frame references are computed; k_pairs_b reads P1[pid] directly)
      const int64_t orow = A.pts.used && !A.pts.used_map ? (int64_t)A.pts.used[row] : row;
      // P1 rows in accumulator order: neuron tile T, lane half h -> 16 contiguous
      // bf16 (the tile's 16 registers), so k_pairs_b reloads them with 2 x 16-B loads
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        const f32x16& v = acc[pt * 2 + T];
        uint4* d = reinterpret_cast<uint4*>(A.p1 + orow * kHid + 32 * (2 * wid + T) + 16 * h);
        d[0] = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                          pack_bf16x2(v[6], v[7]));
        d[1] = make_uint4(pack_bf16x2(v[8], v[9]), pack_bf16x2(v[10], v[11]), pack_bf16x2(v[12], v[13]),
                          pack_bf16x2(v[14], v[15]));
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_pairs_b<KT>: gather + weights + PE_5 + the rest of block1, block3, alpha and
// K-sums for 128 pair columns per workgroup = 128 / KT samples x KT neighbour
// slots (column = j KT + k).  KT = 8 with list == NULL: the samples 0..n-1 in
// order, every slot (the unbucketed launch).  KT < 8: the samples of one bucket
// of buckets.hip (list[0 .. *n_list)), whose slots >= KT are all empty -- the
// outputs are the same numbers as the KT = 8 launch (the dropped slots carried
// zero weights; the xor-tree and DPP reduce-scatter sums below pair the
// remaining lanes exactly as the 8-lane trees do).
constexpr int kBTSmax = kBT;   // samples per tile at KT = 1
// Xb | wtL | apart | sflag | exB (bf16) | prowL | vL | vrL | waL | bL (bf16 biases)
constexpr int kBiasL = 2 * kHid + 2 * kC;   // block1.2, block3.2, color_branch.2, color_branch.4
constexpr size_t kPairsBLds =
    (size_t)kBT * kPB * 2 + (kBT + 4 * kBT + kBTSmax + 4 * kBT + kBT + kBTSmax + 3 * kBTSmax + kHid) * 4 + kBiasL * 2;
static_assert(2 * kPairsBLds <= 160 * 1024, "two k_pairs_b workgroups per CU");
constexpr int kOPitch = kC + 4;   // fp32 output staging pitch: 16-B rows, an accumulator quad is one b128 write
static_assert((size_t)kBT * kOPitch * 4 <= (size_t)kBT * kPB * 2, "output staging must fit the Xb tile");
static_assert(kHid + 24 <= kPB, "the colour branch's hid + view-PE rows must fit the Xb pitch");

// weight-ring depth of k_pairs_b's layers (measured at c5 with the colour branch
// fused and the render variant's branch-free gather: two steps ahead for every
// tile shape, 58.9 ms against 60.1 with one step for KT > 1, alternating on one box)
template <int KT>
constexpr int kPairsWD = 2;
// colour layers' ring depth: one fragment per k-step (4 VGPRs a slot), so the
// lead can be long (c5: 2 steps 55.0 ms, 4 steps 53.9, 6 steps 53.7)
constexpr int kColWD = 6;


// GEN = false: no per-point Rw2c, no used_map, no multi-camera batch, no
// out_weight / out_conf (the render path) -- the general-path branches are compiled out, so no branch
// merge makes the gather wait (vmcnt(0)) for the P1 rows in flight.
template <int KT, bool GEN>
__global__ void __launch_bounds__(64 * kBWaves, 2) k_pairs_b(AggArgsB A, const int32_t* bk_list, const int32_t* bk_info,
                                                              int bucket) {
  constexpr int SPT = kBT / KT;                            // samples per tile
  extern __shared__ __attribute__((aligned(16))) uint16_t xb_dyn[];
  uint16_t* Xb = xb_dyn;                                   // [128][kPB]
  float* wtL = reinterpret_cast<float*>(Xb + kBT * kPB);   // [128]
  float* apart = wtL + kBT;                                // [4][128]
  int* sflag = reinterpret_cast<int*>(apart + 4 * kBT);    // [SPT]
  // block3.0's extra inputs, bf16 as they enter the GEMM (tail_rows_b rounds them
  // the same way): half the LDS of fp32 rows, which leaves room for waL
  uint16_t* exB = reinterpret_cast<uint16_t*>(sflag + kBTSmax);   // [8][128]
  int* prowL = reinterpret_cast<int*>(exB + 8 * kBT);      // [128]
  int* vL = prowL + kBT;                                   // [SPT] sample index of each tile row
  float* vrL = reinterpret_cast<float*>(vL + kBTSmax);     // [3][SPT] rotated view dir of each sample
  float* waL = vrL + 3 * kBTSmax;                          // [256] alpha_branch weights (loaded once)
  uint16_t* bL = reinterpret_cast<uint16_t*>(waL + kHid);  // [kBiasL] layer biases (loaded once)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar addressing
  const int c = lane & 31, h = lane >> 5;
  const int K = A.s.K;
  // bucket samples list[0 .. n) (buckets.hip), or every sample in order
  const int32_t* list = bk_list ? bk_list + bk_info[bucket] : nullptr;
  const int64_t n = bk_list ? (int64_t)bk_info[4 + bucket] : eff_n(A.s);
  const int64_t ntiles = cdiv(n, SPT);
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
  const int T0 = 2 * wid;
  const uint4* w1b = reinterpret_cast<const uint4*>(A.w.w1bf) + T0 * 64;
  const uint4* w2 = reinterpret_cast<const uint4*>(A.w.w2f) + T0 * 64;
  const uint4* w3 = reinterpret_cast<const uint4*>(A.w.w3f) + T0 * 64;
  const uint4* w4 = reinterpret_cast<const uint4*>(A.w.w4f) + T0 * 64;

  // The gather's dependent index chain (bucket list -> sample list -> neighbour
  // id) for the NEXT tile runs one link per layer of this tile (pf_*), so a
  // tile's gather starts from the neighbour id: two HBM round trips fewer on
  // its critical path.
  const int pf_col = threadIdx.x & (kBT - 1);
  const int pf_j = pf_col / KT, pf_k = pf_col % KT;
  auto pf_v = [&](int64_t t) -> int {   // sample-list entry of this column's sample, -1 past the end
    const int64_t jv = t * SPT + pf_j;
    return (t < ntiles && jv < n) ? (list ? list[jv] : (int)jv) : -1;
  };
  auto pf_row = [&](int v) -> int { return v >= 0 ? (int)sample_row(A.s, v) : -1; };
  auto pf_pid = [&](int row) -> int { return (row >= 0 && pf_k < K) ? A.s.pidx[(int64_t)row * K + pf_k] : -1; };
  auto pf_drow = [&](int row) -> int { return row >= 0 ? (int)dir_row(A.s, row) : 0; };   // ray-dir row
  int nx_v = pf_v(blockIdx.x);
  int nx_row = pf_row(nx_v);
  int nx_pid = pf_pid(nx_row);
  int nx_drow = pf_drow(nx_row);
  waL[threadIdx.x] = A.w.wa[threadIdx.x];   // 256 threads, 256 weights (ordered by the tile's first barrier)
  {
    // bias of output n = 32 T + c: pack entry [last step][T][lane c][0] (frag_pack_bf16:
    // W' = [W | bias | 0], bias column 256 -> step 16 (block1.2 / 3.2, 8 tiles), 128 ->
    // step 8 (color_branch.2 / .4, 4 tiles))
    const int T = threadIdx.x >> 5, cc = threadIdx.x & 31;
    bL[threadIdx.x] = A.w.w2f[((size_t)(16 * 8 + T) * 64 + cc) * 8];
    bL[kHid + threadIdx.x] = A.w.w4f[((size_t)(16 * 8 + T) * 64 + cc) * 8];
    if (threadIdx.x < kC) {
      bL[2 * kHid + threadIdx.x] = A.w.wc2f[((size_t)(8 * 4 + T) * 64 + cc) * 8];
      bL[2 * kHid + kC + threadIdx.x] = A.w.wc3f[((size_t)(8 * 4 + T) * 64 + cc) * 8];
    }
  }
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // -------------------------------------------- gather (thread = pair col, role = tid >> 7)
    // Order: the gather's own loads, an LDS-only barrier that hands the pair ids
    // (prefetched chain) to the MFMA lanes, their raw P1 row loads, then the
    // gather's math -- so the math waits for its loads only (vmcnt counts in
    // issue order) and the P1 rows travel meanwhile.  Every load unconditional
    // (clamped rows, zeroed at the unpack).
    if (threadIdx.x < kBT) prowL[threadIdx.x] = nx_pid;
    u32x4v p1raw[kBPT][2][2];
    unsigned p1m = 0;
    {
      const int col = threadIdx.x & (kBT - 1), role = threadIdx.x >> 7;
      const int j = col / KT, k = col % KT;
      const int64_t jv = tile * SPT + j;
      const bool active = jv < n;
      const int64_t v = active ? (int64_t)nx_v : 0;
      const int64_t row = active ? (int64_t)nx_row : 0;
      const bool slot = active && k < K;
      const bool valid = slot && nx_pid >= 0;
      const int64_t prow = valid ? nx_pid : 0;
      const int64_t drow = active ? (int64_t)nx_drow : 0;
      // Every load unconditional -- clamped rows, absent arrays read through a
      // present one -- and masked afterwards: a load under a branch made hipcc
      // drain vmcnt(0) after it (one HBM round trip per load group: the gather was
      // 15.5 k of a 100 k-cycle tile at c5), and these now travel together.
      const float* colp = A.pts.color ? A.pts.color : A.pts.xyz;
      const float* dirp = A.pts.dir ? A.pts.dir : A.pts.xyz;
      const float* persp = A.pts.pers ? A.pts.pers : A.pts.xyz;
      const float* confp = A.pts.conf ? A.pts.conf : A.pts.xyz;
      float sw[3] = {0.f, 0.f, 0.f}, sp[3], vd[3] = {0.f, 0.f, 0.f}, pw[3], pp[3], colr[3] = {0.f, 0.f, 0.f},
            pdir[3] = {0.f, 0.f, 0.f};
      float cfl = 1.f;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        sp[a] = A.s.sample_p[row * 3 + a];
        pw[a] = A.pts.xyz[prow * 3 + a];
        pp[a] = persp[prow * 3 + a];
      }
      // role 1 (waves 2-3: PE channels 3-5 = the perspective half of the distance)
      // needs only sample_p and the point's xyz / pers; the wave-uniform branch
      // keeps the other 13 loads to role 0 (c5: aggregate -0.6 %)
      if (role == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          sw[a] = A.s.sample_w[row * 3 + a];
          vd[a] = A.s.dirs[drow * 3 + a];
          colr[a] = colp[prow * 3 + a];
          pdir[a] = dirp[prow * 3 + a];
        }
        cfl = confp[slot ? prow : 0];
      }
      __builtin_amdgcn_sched_barrier(0);
      lds_barrier();   // prowL: LDS only, the loads above stay in flight
#pragma unroll
      for (int pt = 0; pt < kBPT; ++pt) {
        const int pr = prowL[32 * pt + c];
        p1m |= (pr >= 0 ? 1u : 0u) << pt;
        const int prc = pr >= 0 ? pr : 0;
        // (the clamped row's used_map entry may be -1: clamp again)
        const int64_t p1r = GEN && A.pts.used_map ? (int64_t)max(A.pts.used_map[prc], 0) : (int64_t)prc;
#pragma unroll
        for (int T = 0; T < 2; ++T) {
          const u32x4v* src = reinterpret_cast<const u32x4v*>(A.p1 + p1r * kHid + 32 * (T0 + T) + 16 * h);
          // (plain loads: a non-temporal hint here cost 2.6 ms and 4.2 GB at c5 --
          // neighbouring tiles share P1 rows through L2 / MALL)
          p1raw[pt][T][0] = src[0];
          p1raw[pt][T][1] = src[1];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        sw[a] = active ? sw[a] : 0.f;
        sp[a] = active ? sp[a] : 0.f;
        vd[a] = active ? vd[a] : 0.f;
        pw[a] = valid ? pw[a] : 0.f;
        colr[a] = valid && A.pts.color ? colr[a] : 0.f;
        pdir[a] = valid && A.pts.dir ? pdir[a] : 0.f;
        pp[a] = valid && A.pts.pers ? pp[a] : 0.f;
      }
      if (!A.pts.pers) {
        // w2pers under the camera of the pair's ray: the launch's one camera
        // (registers) or, GEN only, the ray's entry of the camera tables (loads)
        float ppc[3];
        if (GEN)
          pair_pers(A.pts, A.s, drow, pw, cam_c, cam_R, ppc);
        else
          world_to_pers(pw, cam_c, cam_R, ppc);
#pragma unroll
        for (int a = 0; a < 3; ++a) pp[a] = valid ? ppc[a] : 0.f;
      }
      const float cf = A.pts.conf && slot ? cfl : 1.f;
      float d6[6];
      d6[0] = pw[0] - sw[0];
      d6[1] = pw[1] - sw[1];
      d6[2] = pw[2] - sw[2];
      d6[3] = pp[0] * pp[2] - sp[0] * sp[2];
      d6[4] = pp[1] * pp[2] - sp[1] * sp[2];
      d6[5] = pp[2] - sp[2];
      const float nrm = sqrtf(d6[0] * d6[0] + d6[1] * d6[1] + d6[2] * d6[2]);
      const float wl = valid ? 1.f / fmaxf(nrm, 1e-6f) : 0.f;
      const float wsum = xork_sum_nc<KT>(wl);
      const float wn = wl / fmaxf(wsum, 1e-8f);
      const float confc = fminf(fmaxf(cf, 1e-4f), 1.f);
      const bool samp_valid = xork_sum<KT>(valid ? 1.f : 0.f) > 0.f;
      float dr6[6];
      mat3(Rw, d6, dr6);
      dr6[3] = d6[3];
      dr6[4] = d6[4];
      dr6[5] = d6[5];
      if (GEN && A.pts.rw2c) rot_point(A.pts.rw2c, prow, d6, dr6);   // per-point Rw2c (agg_common.h)
      if (role == 0) {
        float vrot[3], drot[3];
        mat3(Rw, vd, vrot);
        mat3(Rw, pdir, drot);
        if (GEN && A.pts.rw2c) {
          rot_point(A.pts.rw2c, prow, pdir, drot);
          rot_point(A.pts.rw2c, active ? slot0_point(A.s, row) : 0, vd, vrot);
        }
        const float dot = drot[0] * vrot[0] + drot[1] * vrot[1] + drot[2] * vrot[2];
        const float ex[8] = {colr[0], colr[1], colr[2], drot[0] - vrot[0], drot[1] - vrot[1], drot[2] - vrot[2],
                             dot, 1.f};
#pragma unroll
        for (int e = 0; e < 8; ++e) exB[e * kBT + col] = to_bf16(ex[e]);
        wtL[col] = wn * confc;
        if (k == 0) {
          sflag[j] = active && samp_valid;
          vL[j] = (int)v;   // the list entry, read once here (not per store below)
          // the colour branch's view-PE input (kept from the gather: no second walk
          // sample row -> dir map -> ray dir)
#pragma unroll
          for (int a = 0; a < 3; ++a) vrL[a * kBTSmax + j] = vrot[a];
        }
        if (active && k < K) {
          // the bucket's dropped slots (KT..K-1) are empty: weight 0, their gathered conf
          if (GEN && A.out_weight) {
            A.out_weight[row * K + k] = wn;
            if (k == 0)
              for (int kk = KT; kk < K; ++kk) A.out_weight[row * K + kk] = 0.f;
          }
          if (GEN && A.out_conf) {
            A.out_conf[row * K + k] = confc;
            if (k == 0)
              for (int kk = KT; kk < K; ++kk) {
                const int pid = A.s.pidx[row * K + kk];
                const float c2 = A.pts.conf ? A.pts.conf[pid >= 0 ? pid : 0] : 1.f;
                A.out_conf[row * K + kk] = fminf(fmaxf(c2, 1e-4f), 1.f);
              }
          }
        }
        *reinterpret_cast<uint2*>(Xb + col * kPB + 60) = make_uint2(0u, 0u);   // rows 60..63: k padding
      }
      // 5-band PE of the rotated distance -> rows 2e, 2e+1 (e = 5 ch + f); role r:
      // channels 3r .. 3r + 2.  One sincosf per channel, the higher bands by angle
      // doubling (k_point_pre_b's PE_3): <= ~16 ulp at band 4, far below the bf16
      // rounding of the MFMA operands.
      uint16_t* xc = Xb + col * kPB;
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        const int ch = 3 * role + cc;
        const float dc = role == 0 ? dr6[cc] : dr6[3 + cc];
        float sn, cs;
        sincosf(dc, &sn, &cs);
#pragma unroll
        for (int f = 0; f < 5; ++f) {
          *reinterpret_cast<unsigned*>(xc + 2 * (5 * ch + f)) = pack_bf16x2(sn, cs);
          const float s2 = 2.f * sn * cs, c2 = (cs - sn) * (cs + sn);
          sn = s2;
          cs = c2;
        }
      }
    }
    __syncthreads();
    // -------------------------------------------- P1 rows into the accumulators
    f32x16 acc[kBPT * 2];
#pragma unroll
    for (int pt = 0; pt < kBPT; ++pt) {
      const bool has = (p1m >> pt) & 1;
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        const u32x4v u0 = p1raw[pt][T][0], u1 = p1raw[pt][T][1];
        const unsigned w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          acc[pt * 2 + T][2 * q] = has ? bf16_lo(w[q]) : 0.f;
          acc[pt * 2 + T][2 * q + 1] = has ? bf16_hi(w[q]) : 0.f;
        }
      }
    }
    nx_v = pf_v(tile + gridDim.x);   // the next tile's chain, link 1
    // -------------------------------------------- block1: + W1[:, 224:284] . PE_5 (4 steps), block1.2
    mlp_layer_b<2, kBPT, 8, kPB, kPairsWD<KT>>(acc, w1b, Xb, 4, lane);
    __syncthreads();
    store_act_b<2, kBPT, kPB>(acc, Xb, neg, lane, T0);
    __syncthreads();
    acc_bias_b<2, kBPT>(acc, bL, lane, T0);
    nx_row = pf_row(nx_v);   // link 2
    mlp_layer_b<2, kBPT, 8, kPB, kPairsWD<KT>>(acc, w2, Xb, 16, lane);
    __syncthreads();
    store_act_b<2, kBPT, kPB>(acc, Xb, neg, lane, T0);
    if (wid == 0) {   // block3.0 inputs 256..263 (+ zeros to 271)
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int col = lane + 64 * half;
        float ex[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) ex[e] = __uint_as_float((unsigned)exB[e * kBT + col] << 16);
        tail_rows_b(Xb, kPB, col, 256, ex, 8);
      }
    }
    __syncthreads();
    // -------------------------------------------- block3
#pragma unroll
    for (int i = 0; i < kBPT * 2; ++i) acc[i] = (f32x16){0.f};
    nx_pid = pf_pid(nx_row);   // link 3
    nx_drow = pf_drow(nx_row);
    mlp_layer_b<2, kBPT, 8, kPB, kPairsWD<KT>>(acc, w3, Xb, 17, lane);
    __syncthreads();
    store_act_b<2, kBPT, kPB>(acc, Xb, neg, lane, T0);
    __syncthreads();
    acc_bias_b<2, kBPT>(acc, bL + kHid, lane, T0);
    mlp_layer_b<2, kBPT, 8, kPB, kPairsWD<KT>>(acc, w4, Xb, 16, lane);
    __syncthreads();   // Xb is free: the K-sums are staged there (hid rows, kHP pitch)
    // -------------------------------------------- alpha + K sums from the fp32 accumulators
    {
    float pa_part[kBPT] = {0.f, 0.f, 0.f, 0.f};
    const int ik = c % KT;   // the lane's slot within its sample
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      float wa[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) wa[r] = waL[32 * (T0 + T) + acc_row(r, h)];
#pragma unroll
      for (int pt = 0; pt < kBPT; ++pt) {
        const int col = 32 * pt + c;
        const float wtp = wtL[col];
        const int sj = col / KT;
        float vv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float hv = lrelu(acc[pt * 2 + T][r], neg);
          pa_part[pt] += wa[r] * hv;
          vv[r] = wtp * hv;
        }
        // K-sum of the sample's KT lanes as a DPP reduce-scatter: each lane keeps
        // 16 / KT of the 16 accumulator rows (the 8-lane tree's pairing)
        uint16_t* hrow = Xb + sj * kPB + 32 * (T0 + T) + 4 * h;   // staged row of sample sj
        if constexpr (KT == 8) {
          const bool b2 = (ik & 4) != 0, b1 = (ik & 2) != 0, b0 = (ik & 1) != 0;
          float w8[8], w4v[4], w2[2];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float send = b2 ? vv[q] : vv[q + 8];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0x141,
                                                                                  0xf, 0xf, false));
            w8[q] = add_nc(b2 ? vv[q + 8] : vv[q], recv);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float send = b1 ? w8[q] : w8[q + 4];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0x4E,
                                                                                  0xf, 0xf, false));
            w4v[q] = add_nc(b1 ? w8[q + 4] : w8[q], recv);
          }
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float send = b0 ? w4v[q] : w4v[q + 2];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1,
                                                                                  0xf, 0xf, false));
            w2[q] = add_nc(b0 ? w4v[q + 2] : w4v[q], recv);
          }
          *reinterpret_cast<unsigned*>(hrow + ((2 * ik) & 3) + 8 * (ik >> 1)) = pack_bf16x2(w2[0], w2[1]);
        } else if constexpr (KT == 4) {
          // stages lane ^ 2, lane ^ 1: lane ik keeps registers 4 ik .. 4 ik + 3 = neurons 8 ik + q
          const bool b1 = (ik & 2) != 0, b0 = (ik & 1) != 0;
          float w8[8], w4v[4];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float send = b1 ? vv[q] : vv[q + 8];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0x4E,
                                                                                  0xf, 0xf, false));
            w8[q] = add_nc(b1 ? vv[q + 8] : vv[q], recv);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float send = b0 ? w8[q] : w8[q + 4];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1,
                                                                                  0xf, 0xf, false));
            w4v[q] = add_nc(b0 ? w8[q + 4] : w8[q], recv);
          }
          *reinterpret_cast<uint2*>(hrow + 8 * ik) = make_uint2(pack_bf16x2(w4v[0], w4v[1]),
                                                                pack_bf16x2(w4v[2], w4v[3]));
        } else if constexpr (KT == 2) {
          // stage lane ^ 1: lane ik keeps registers 8 ik .. 8 ik + 7 = neurons 16 ik + {0..3, 8..11}
          const bool b0 = (ik & 1) != 0;
          float w8[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float send = b0 ? vv[q] : vv[q + 8];
            const float recv = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1,
                                                                                  0xf, 0xf, false));
            w8[q] = add_nc(b0 ? vv[q + 8] : vv[q], recv);
          }
          *reinterpret_cast<uint2*>(hrow + 16 * ik) = make_uint2(pack_bf16x2(w8[0], w8[1]),
                                                                 pack_bf16x2(w8[2], w8[3]));
          *reinterpret_cast<uint2*>(hrow + 16 * ik + 8) = make_uint2(pack_bf16x2(w8[4], w8[5]),
                                                                     pack_bf16x2(w8[6], w8[7]));
        } else {
          // one slot: the lane's 16 registers are the sample's rows 8 g + 4 h + q
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<uint2*>(hrow + 8 * g) = make_uint2(pack_bf16x2(vv[4 * g], vv[4 * g + 1]),
                                                                 pack_bf16x2(vv[4 * g + 2], vv[4 * g + 3]));
        }
      }
    }
#pragma unroll
    for (int pt = 0; pt < kBPT; ++pt) pa_part[pt] += __shfl_xor(pa_part[pt], 32);
    if (h == 0) {
#pragma unroll
      for (int pt = 0; pt < kBPT; ++pt) apart[wid * kBT + 32 * pt + c] = pa_part[pt];
    }
    __syncthreads();
    if (wid < 2) {
      const int col = 64 * wid + lane;
      const int j = col / KT, k = col % KT;
      const float pa = apart[col] + apart[kBT + col] + apart[2 * kBT + col] + apart[3 * kBT + col] + A.w.ba[0];
      const float alpha_k = A.w.act_super ? softplus(pa - 1.f) : fmaxf(pa, 0.f);
      const float alpha_s = xork_sum_nc<KT>(wtL[col] * alpha_k);
      const int64_t jv = tile * SPT + j;
      if (k == 0 && jv < n && sflag[j]) {
        if (A.out_feat_h)
          *reinterpret_cast<float*>(A.out_feat_h + (int64_t)vL[j] * PNR_FEAT_H_PITCH) = alpha_s;
        else
          A.out_feat[(int64_t)vL[j] * (kC + 1)] = alpha_s;
      }
    } else if (threadIdx.x - 128 < SPT) {
      // colour-branch inputs 256 .. 279 of sample j: PE_4 of the rotated view dir
      // (ori dropped; masked samples: 0) -- rows 256 + 4 ch + f sin, 268 + 4 ch + f cos
      const int j = threadIdx.x - 128;
      const bool valid = sflag[j] != 0;
      uint16_t* xc = Xb + j * kPB;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float vr = valid ? vrL[ch * kBTSmax + j] : 0.f;
        float sn[4], cs[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) sincosf(vr * (float)(1 << f), &sn[f], &cs[f]);
        *reinterpret_cast<uint2*>(xc + 256 + 4 * ch) = make_uint2(pack_bf16x2(sn[0], sn[1]), pack_bf16x2(sn[2], sn[3]));
        *reinterpret_cast<uint2*>(xc + 268 + 4 * ch) = make_uint2(pack_bf16x2(cs[0], cs[1]), pack_bf16x2(cs[2], cs[3]));
      }
    }
    }
    __syncthreads();
    // -------------------------------------------- colour branch on the tile's samples
    // [hid (K-summed, staged above), PE_4(view)] -> 128 -> 128 -> 128 (the
    // reference's color_branch, point_aggregators.py:640-646), columns = samples:
    // the K-summed rows never leave the CU.  Bias of the first layer: the ring's
    // last-step override (row 280 = 1), the 280 real rows fill the pitch.
    {
      constexpr int PTc = SPT >= 32 ? SPT / 32 : 1;   // 32-column quarters holding the SPT samples
      const uint4* wc1 = reinterpret_cast<const uint4*>(A.w.wc1f) + wid * 64;
      const uint4* wc2 = reinterpret_cast<const uint4*>(A.w.wc2f) + wid * 64;
      const uint4* wc3 = reinterpret_cast<const uint4*>(A.w.wc3f) + wid * 64;
      f32x16 cacc[PTc];
#pragma unroll
      for (int i = 0; i < PTc; ++i) cacc[i] = (f32x16){0.f};
      mlp_layer_b<1, PTc, 4, kPB, kColWD, true>(cacc, wc1, Xb, 18, lane);
      __syncthreads();
      store_act_b<1, PTc, kPB>(cacc, Xb, neg, lane, wid);
      __syncthreads();
      acc_bias_b<1, PTc>(cacc, bL + 2 * kHid, lane, wid);
      mlp_layer_b<1, PTc, 4, kPB, kColWD>(cacc, wc2, Xb, 8, lane);
      __syncthreads();
      store_act_b<1, PTc, kPB>(cacc, Xb, neg, lane, wid);
      __syncthreads();
      acc_bias_b<1, PTc>(cacc, bL + 2 * kHid + kC, lane, wid);
      mlp_layer_b<1, PTc, 4, kPB, kColWD>(cacc, wc3, Xb, 8, lane);
      __syncthreads();   // every wave's layer-3 reads of Xb are done
      // out_feat rows (valid samples only) through LDS, two rows per store
      // instruction (lane half = row, 16 B per lane, rows 516 B apart: 4-B aligned)
      float* Ob = reinterpret_cast<float*>(Xb);   // [32 PTc][kOPitch] fp32
#pragma unroll
      for (int pt = 0; pt < PTc; ++pt)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<float4*>(Ob + (32 * pt + c) * kOPitch + 32 * wid + 4 * h + 8 * q) =
              make_float4(lrelu(cacc[pt][4 * q], neg), lrelu(cacc[pt][4 * q + 1], neg), lrelu(cacc[pt][4 * q + 2], neg),
                          lrelu(cacc[pt][4 * q + 3], neg));
      __syncthreads();
      typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
      for (int r2 = wid; r2 < SPT / 2; r2 += kBWaves) {
        const int r = 2 * r2 + (lane >> 5), l = lane & 31;
        if (tile * SPT + r >= n || !sflag[r]) continue;
        const float4 s4 = *reinterpret_cast<const float4*>(Ob + r * kOPitch + 4 * l);
        if (A.out_feat_h) {   // bf16 rows: 8 B per lane, a 272-B row per lane half
          typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
          const u32x2v hv = {pack_bf16x2(s4.x, s4.y), pack_bf16x2(s4.z, s4.w)};
          __builtin_nontemporal_store(hv, reinterpret_cast<u32x2v*>(A.out_feat_h + (int64_t)vL[r] * PNR_FEAT_H_PITCH +
                                                                    8 + 4 * l));
        } else {
          const f4u v = {s4.x, s4.y, s4.z, s4.w};
          __builtin_nontemporal_store(v, reinterpret_cast<f4u*>(A.out_feat + (int64_t)vL[r] * (kC + 1) + 1 + 4 * l));
        }
      }
    }
    __syncthreads();
  }
}


template <int KT>
static void launch_pairs_b(bool gen, unsigned grid, hipStream_t st, const AggArgsB& a, const int32_t* list,
                           const int32_t* info, int bucket) {
  if (gen)
    hipLaunchKernelGGL((k_pairs_b<KT, true>), dim3(grid), dim3(64 * kBWaves), kPairsBLds, st, a, list, info, bucket);
  else
    hipLaunchKernelGGL((k_pairs_b<KT, false>), dim3(grid), dim3(64 * kBWaves), kPairsBLds, st, a, list, info, bucket);
}

static size_t scratch_need_b(int64_t n_max, int64_t n_p1) {
  const int64_t nm = n_max > 0 ? n_max : 1;
  const int64_t np = n_p1 > 0 ? n_p1 : 1;
  // P1 | pair buckets (buckets.hip)
  return (size_t)np * kHid * 2 + (size_t)bucket_scratch_ints(nm) * 4;
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_aggregate_scratch_bytes_bf16(int64_t n_max, int64_t n_points, size_t* out) {
  PNR_CHECK_ARG(out && n_max >= 0 && n_points >= 0, "aggregate_scratch_bytes_bf16: bad args");
  *out = scratch_need_b(n_max, n_points);
  return PNR_OK;
}

static int aggregate_fwd_bf16(const pnr_points* pts, const pnr_samples* s, const pnr_mlp_bf16* w, float* out_feat,
                              uint16_t* out_feat_h, float* out_weight, float* out_conf, void* scratch,
                              size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(pts && s && w && (out_feat || out_feat_h), "aggregate_bf16: null pointer");
  PNR_CHECK_ARG(((uintptr_t)out_feat_h & 15) == 0, "aggregate_bf16_hf: out_feat_h must be 16-B aligned");
  PNR_CHECK_ARG(pts->xyz && (pts->emb || pts->emb_bf16) && s->pidx, "aggregate_bf16: point xyz/emb and pidx required");
  PNR_CHECK_ARG(s->sample_w && s->sample_p && s->dirs && s->dir_div >= 1, "aggregate_bf16: sample arrays required");
  PNR_CHECK_ARG(s->K >= 1 && s->K <= kKN, "aggregate_bf16: K=%d unsupported (1..8)", s->K);
  PNR_CHECK_ARG(w->w1af && w->w1bf && w->w2f && w->w3f && w->w4f && w->wa && w->ba && w->wc1f && w->wc2f && w->wc3f,
                "aggregate_bf16: null weight");
  PNR_CHECK_ARG(((uintptr_t)pts->emb & 15) == 0 && ((uintptr_t)pts->emb_bf16 & 7) == 0 &&
                    ((uintptr_t)scratch & 15) == 0,
                "aggregate_bf16: emb (16 B), emb_bf16 (8 B) and scratch (16 B) must be aligned");
  PNR_CHECK_ARG(pts->pers || (pts->campos && pts->camrot), "aggregate_bf16: need pers or camera");
  PNR_CHECK_ARG(!pts->used || (pts->n_used >= 0 && pts->n_used <= pts->n), "aggregate_bf16: bad n_used");
  // P1 table rows: the used rows (compact, indexed through used_map) or every point
  // row (also when used is given without used_map: only those rows are computed)
  const int64_t n_p1 = pts->used && pts->used_map ? pts->n_used : pts->n;
  const int64_t n_pre = pts->used ? pts->n_used : pts->n;   // rows k_point_pre_b computes (capacity)
  PNR_CHECK_ARG(scratch_bytes >= scratch_need_b(s->n_max, n_p1), "aggregate_bf16: scratch too small");
  if (s->n_max <= 0) return PNR_OK;
  hipStream_t st = as_stream(stream);
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_point_pre_b),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kBT * kPB * 2)));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<1, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<1, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<2, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<2, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<4, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<4, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<8, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_b<8, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairsBLds));
    attr = true;
  }
  const int64_t nm = s->n_max;
  AggArgsB a;
  a.pts = *pts;
  a.s = *s;
  a.w = *w;
  // P1 [n_p1, 256] first (fixed place, reusable via p1_ready) | pair buckets
  a.p1 = static_cast<uint16_t*>(scratch);
  int32_t* bk_scratch = reinterpret_cast<int32_t*>(a.p1 + (n_p1 > 0 ? n_p1 : 1) * kHid);
  a.out_feat = out_feat;
  a.out_feat_h = out_feat_h;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  if (!pts->p1_ready) {
    hipLaunchKernelGGL(k_point_pre_b, dim3(grid_for(cdiv(n_pre, kBT), 1, 256 * 2)), dim3(64 * kBWaves),
                       kBT * kPB * 2, st, a);
    PNR_LAUNCH_CHECK();
  }
  // the general path's branches only when a caller needs them
  const bool gen = pts->rw2c || pts->used_map || out_weight || out_conf || s->ray_cam;
  if (w->pair_buckets) {
    // samples partitioned by filled slots, one launch per bucket (the heaviest first)
    PairBuckets bk;
    int rc;
    if ((rc = launch_buckets(a.s, bk_scratch, &bk, st))) return rc;
    const unsigned g8 = grid_for(cdiv(nm, kBT / 8), 1, 256 * 2), g4 = grid_for(cdiv(nm, kBT / 4), 1, 256 * 2),
                   g2 = grid_for(cdiv(nm, kBT / 2), 1, 256 * 2), g1 = grid_for(cdiv(nm, kBT), 1, 256 * 2);
    launch_pairs_b<8>(gen, g8, st, a, bk.list, bk.info, 3);
    PNR_LAUNCH_CHECK();
    launch_pairs_b<4>(gen, g4, st, a, bk.list, bk.info, 2);
    PNR_LAUNCH_CHECK();
    launch_pairs_b<2>(gen, g2, st, a, bk.list, bk.info, 1);
    PNR_LAUNCH_CHECK();
    launch_pairs_b<1>(gen, g1, st, a, bk.list, bk.info, 0);
    PNR_LAUNCH_CHECK();
  } else {
    launch_pairs_b<8>(gen, grid_for(cdiv(nm, kBT / 8), 1, 256 * 2), st, a, nullptr, nullptr, 3);
    PNR_LAUNCH_CHECK();
  }
  return PNR_OK;
}

extern "C" int pnr_aggregate_fwd_bf16(const pnr_points* pts, const pnr_samples* s, const pnr_mlp_bf16* w,
                                      float* out_feat, float* out_weight, float* out_conf, void* scratch,
                                      size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(out_feat, "aggregate_bf16: null out_feat");
  return aggregate_fwd_bf16(pts, s, w, out_feat, nullptr, out_weight, out_conf, scratch, scratch_bytes, stream);
}

extern "C" int pnr_aggregate_fwd_bf16_hf(const pnr_points* pts, const pnr_samples* s, const pnr_mlp_bf16* w,
                                         uint16_t* out_feat_h, float* out_weight, float* out_conf, void* scratch,
                                         size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(out_feat_h, "aggregate_bf16_hf: null out_feat_h");
  return aggregate_fwd_bf16(pts, s, w, nullptr, out_feat_h, out_weight, out_conf, scratch, scratch_bytes, stream);
}
