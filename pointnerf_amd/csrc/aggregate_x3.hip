// fp32-accurate k_pairs on 16-bit MFMA: block1.0's distance half, block1.2,
// block3.0 and block3.2 for 64 (sample, neighbour) pairs per tile, as in
// aggregate.hip's k_pairs, with every fp32 GEMM done on split operands
// (agg_common.h):
//   * k_pairs_x3 (pnr_aggregate_fwd_x3): exact 3-way bf16 split, six cross
//     products per 16-k step on v_mfma_f32_32x32x16_bf16 (split2);
//   * k_pairs_h2 (pnr_aggregate_fwd_h2): 2-way f16 split with a 2^11-scaled low
//     half, three products on v_mfma_f32_32x32x16_f16 (splith) -- half the
//     MFMA work, two activation planes instead of three.
// Both are one kernel body templated on H (false: bf16 x3, true: f16 h2).
//
// Producer / consumer workgroup (one 8-wave workgroup per CU):
//   * consumers (waves 0..3) own neuron tiles {2w, 2w+1} x both 32-pair halves
//     and run the MFMA stream: 6 (x3) / 3 (h2) products per 16-k step, weights
//     from split packs three steps ahead (buffer loads), B fragments = one
//     ds_read_b128 per plane of the layer input.  Each activation is split ONCE, by the
//     wave that produced it, when it is stored (not once per consuming wave).
//   * producers (waves 4..7) prepare the NEXT tile while the consumers run
//     block1.2 of the current one: gather (pidx, xyz, w2pers, colour, dir,
//     conf), 6-d distance, normalised weights, the 5-band PE split into planes,
//     the block3.0 extras -- so the gather latency and the sincos never stall
//     the MFMA pipe.  The consumers prefetch the next tile's per-point
//     block1.0 half (P1) into registers during block3.2.
// LDS (135 KB x3, 100 KB h2): layer-input planes [NPL][34 row groups][64 pairs][8 x 16 bit]
// (rows 0..271; row group g, pair c at (g*64 + c)*16 B, so a B fragment is one
// conflict-free ds_read_b128 and an accumulator quad one ds_write_b64 per
// plane), next-tile PE planes [NPL][8][64][8], and double-buffered per-tile
// extras / weights / point rows / sample flags.
#include "agg_common.h"


namespace pnr {
namespace {

constexpr int kXT = 64;            // pairs per tile
constexpr int kXTS = kXT / kKN;    // samples per tile
// h2 K-summed features (k_pairs_h2 -> k_color_h2): f16-split planes, per tile of
// 64 samples [plane 2][row group 32][64 samples][8 f16] = the colour kernel's
// LDS image, so one global_load_lds wave-instruction copies one group (1 KB).
// Samples without a valid neighbour are never written (the colour kernel
// ignores their columns).
constexpr int kHidPlane = 32 * 64 * 16;
constexpr int kHidTile = 2 * kHidPlane;
constexpr int kXG = 34;            // 8-row groups of a layer input (272 rows)
constexpr int kPG = 8;             // 8-row groups of the distance PE (64 rows)
constexpr int kPlaneX = kXG * kXT * 16;
constexpr int kPlaneP = kPG * kXT * 16;
constexpr int kP1Pitch = kHid + 4;                 // floats per parked P1 row (conflict-free b128 reads)

// Per-variant layout: NPL activation planes (x3: 3 bf16, h2: 2 f16), NPW weight
// planes per (k-step, neuron tile) in the packs (x3: W0 W1 W2; h2: Wh Wl).
template <bool H>
struct XL {
  static constexpr int NPL = H ? 2 : 3;
  static constexpr int NPW = H ? 2 : 3;
  static constexpr unsigned kOne = H ? 0x3C00u : 0x3F80u;   // 1.0 (bias input row)
  static constexpr int OffPE = NPL * kPlaneX;
  static constexpr int OffEx = OffPE + NPL * kPlaneP;       // float [2][8][64]
  // blend-weight / sample-flag slots: h2 runs a tile's tail one tile later on
  // the producers (three slots in flight), x3 on the consumers (two)
  static constexpr int NWB = H ? 3 : 2;
  static constexpr int OffWt = OffEx + 2 * 8 * kXT * 4;    // float [NWB][64]
  static constexpr int OffPr = OffWt + NWB * kXT * 4;      // int   [2][64]
  static constexpr int OffSf = OffPr + 2 * kXT * 4;        // int   [NWB][8]
  static constexpr int OffAp = OffSf + NWB * kXTS * 4;     // float [4][64] (x3: alpha partials)
  static constexpr int OffWa = OffAp + 4 * kXT * 4;        // float [256] alpha_branch.0 weights
  static constexpr int OffH4 = OffWa + kHid * 4;           // h2: float [64][kP1Pitch] block3.2 accumulators
  static constexpr int OffTq = OffH4 + (H ? kXT * kP1Pitch * 4 : 0);   // int [4] tile of iteration i at i % 4
  static constexpr size_t Lds = (size_t)OffTq + 16;
  static_assert(OffSf % 16 == 0 && OffWa % 16 == 0 && OffH4 % 16 == 0, "16-B aligned LDS arrays");
  static_assert(kXT * kP1Pitch * 4 <= NPL * kPlaneX, "parked P1 fits the layer-input area");
  static_assert(Lds <= 160 * 1024, "LDS budget");
};

constexpr int kProducerPrio = 3;   // producer wave priority (s_setprio): measured 0: 110.6, 2: 110.1, 3: 109.6 ms

typedef float f32x2n __attribute__((ext_vector_type(2)));
typedef float f32x4n __attribute__((ext_vector_type(4)));

struct X3Args {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp w;
  SplitW wx;
  const float* p1;
  float* hid;
  int32_t* vmask;
  float* out_feat;
  float* out_weight;
  float* out_conf;
  int32_t* tile_ctr;   // zeroed per launch: tiles past the first gridDim.x are handed out in order
  pnr_agg_saved sv;    // k_pairs_x3_train: activations kept for the backward (aggregate.hip layout)
};

// Dynamic tile schedule: each workgroup starts on tile blockIdx.x and takes
// the next free tile from tile_ctr when it starts the one before (producer
// wave 0, lane 0, one tile ahead; the index travels through LDS ring TQ), so
// workgroups that start late or run slow (another kernel on the CU, an RCCL
// copy) take fewer tiles instead of finishing late.
//
// XCD-aware (large launches): blocks b and b + 8 share an XCD (round-robin
// dispatch, MI355X_MICROARCH "Workgroup dispatch"), so block group b % 8 works
// through its own contiguous eighth of the tiles with its own counter and then
// helps the other groups.  Neighbouring tiles (the same or adjacent rays) share
// most of their points, so their P1 rows are re-read from that XCD's L2.
__device__ __forceinline__ bool xcd_mode(int64_t nt) { return nt >= 2 * (int64_t)gridDim.x + 16; }
__device__ __forceinline__ int64_t xcd_lo(int64_t nt, int x) { return nt * x / 8; }
__device__ __forceinline__ int64_t xcd_nb(int x) { return ((int)gridDim.x - x + 7) / 8; }   // blocks of group x

__device__ __forceinline__ int64_t first_tile(int64_t nt) {
  if (!xcd_mode(nt)) return blockIdx.x;
  return xcd_lo(nt, blockIdx.x & 7) + (blockIdx.x >> 3);
}

__device__ __forceinline__ int64_t take_tile(const X3Args& A, int64_t nt) {
  if (!xcd_mode(nt)) return (int64_t)gridDim.x + atomicAdd(A.tile_ctr, 1);
  const int x0 = blockIdx.x & 7;
  for (int i = 0; i < 8; ++i) {
    const int x = (x0 + i) & 7;
    const int64_t t = xcd_lo(nt, x) + xcd_nb(x) + atomicAdd(A.tile_ctr + x, 1);
    if (t < xcd_lo(nt, x + 1)) return t;
  }
  return nt;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// this wave's 2 neuron tiles of k-step t, NPW planes each; voff = (T0 * NPW * 64 + lane) * 16
template <bool H, int NTK = 8>
__device__ __forceinline__ void load_w(uint4 (&a)[2][XL<H>::NPW], __amdgpu_buffer_rsrc_t rs, int voff, int t) {
  constexpr int NPW = XL<H>::NPW;
#pragma unroll
  for (int T = 0; T < 2; ++T)
#pragma unroll
    for (int pl = 0; pl < NPW; ++pl)
      a[T][pl] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(
                     rs, voff + pl * 1024, (t * NTK + T) * NPW * 1024, 0));
}

// weight ring depth (k-steps in flight); the packs carry >= kWD zero steps
// (X3_PAD / H2_PAD in aggregator.py)
template <bool H>
struct WRing {
  static constexpr int kWD = 3;
  uint4 a[kWD][2][XL<H>::NPW];
};

template <bool H, int NTK = 8>
__device__ __forceinline__ void prime(WRing<H>& w, __amdgpu_buffer_rsrc_t rs, int voff) {
#pragma unroll
  for (int d = 0; d < WRing<H>::kWD; ++d) load_w<H, NTK>(w.a[d], rs, voff, d);
}

// Y^T += W . X^T over nsteps 16-k steps; X^T = the bf16 planes at `planes`
// (plane stride pstride bytes, 64 pairs per 8-row group).  Weights kWD steps
// ahead in the ring (slot d: steps = d mod kWD), B one step ahead.  NTK: neuron
// tiles per k-step in the pack (256 outputs: 8, the colour branch: 4).
template <bool H, int NTK = 8>
__device__ __forceinline__ void layer(f32x16 (&acc)[4], WRing<H>& w, __amdgpu_buffer_rsrc_t rs, int voff,
                                      const char* planes, int pstride, int nsteps, int lane) {
  constexpr int NPL = XL<H>::NPL, NPW = XL<H>::NPW, kWD = WRing<H>::kWD;
  const int c = lane & 31, h = lane >> 5;
  const char* base = planes + (h * kXT + c) * 16;
  auto ldb = [&](int t, int pt, uint4 (&bb)[NPL]) {
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
      bb[pl] = *reinterpret_cast<const uint4*>(base + pl * pstride + (2 * t * kXT + 32 * pt) * 16);
  };
  // B fragments BD steps ahead (slot = step mod BD)
  constexpr int BD = H ? 2 : 1;   // h2: B fragments (LDS) read two k-steps ahead
  uint4 b[BD][2][NPL];
#pragma unroll
  for (int sl = 0; sl < BD; ++sl) {
    const int t0 = sl < nsteps ? sl : nsteps - 1;
    ldb(t0, 0, b[sl][0]);
    ldb(t0, 1, b[sl][1]);
  }
  // One step = 2 halves x 12 MFMAs.  Each B plane of a half is re-read for the
  // next step, and each weight plane re-loaded kWD steps ahead, right after
  // its last MFMA of this step, so the loads sit in MFMA gaps instead of in
  // bursts; sched_barrier(0) pins the order (hipcc would otherwise sink the
  // LDS reads next to their uses and merge the waits).
  auto mm = [&](int pt, const uint4& av0, const uint4& av1, const uint4& bv) {
    if constexpr (H) {
      acc[2 * pt] = mfma_f16(av0, bv, acc[2 * pt]);
      acc[2 * pt + 1] = mfma_f16(av1, bv, acc[2 * pt + 1]);
    } else {
      acc[2 * pt] = mfma_bf16(av0, bv, acc[2 * pt]);
      acc[2 * pt + 1] = mfma_bf16(av1, bv, acc[2 * pt + 1]);
    }
  };
  auto wl = [&](uint4 (&a)[2][NPW], int pl, int tw) {
#pragma unroll
    for (int T = 0; T < 2; ++T)
      a[T][pl] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(
                     rs, voff + pl * 1024, (tw * NTK + T) * NPW * 1024, 0));
  };
  auto bl = [&](int bs, int tn, int pt, int pl) {
    b[bs][pt][pl] = *reinterpret_cast<const uint4*>(base + pl * pstride + (2 * tn * kXT + 32 * pt) * 16);
  };
  // h2 step per half: Ws.Xh, Wl.Xh, Wh.Xl (Ws = 2^11 Wh, made in registers)
  // Ws = 2^11 Wh of the NEXT step is made in the middle of this one (scl), so
  // the v_pk_mul_f16 results are never waited on by the MFMA right after them.
  uint4 scl[2];
  auto scale_next = [&](const uint4 (&an)[2][NPW], int T) {   // one tile per MFMA gap (4 v_pk_mul_f16)
    scl[T] = f16x8_scale2048(an[T][0]);
  };
  if constexpr (H) {
    scale_next(w.a[0], 0);
    scale_next(w.a[0], 1);
  }
  auto step_h = [&](uint4 (&a)[2][NPW], const uint4 (&an)[2][NPW], int t, int bs) {
    const int tn = t + BD < nsteps ? t + BD : nsteps - 1;
    const uint4 s0 = scl[0], s1 = scl[1];
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      mm(pt, s0, s1, b[bs][pt][0]);                                // Ws.Xh
      __builtin_amdgcn_sched_barrier(0);
      mm(pt, a[0][1], a[1][1], b[bs][pt][0]);                      // Wl.Xh
      __builtin_amdgcn_sched_barrier(0);
      if (pt == 1) wl(a, 1, t + kWD);
      if (pt == 0) scale_next(an, 0);
      bl(bs, tn, pt, 0);
      __builtin_amdgcn_sched_barrier(0);
      mm(pt, a[0][0], a[1][0], b[bs][pt][1]);                      // Wh.Xl
      __builtin_amdgcn_sched_barrier(0);
      bl(bs, tn, pt, 1);
      if (pt == 0) scale_next(an, 1);
      if (pt == 1) wl(a, 0, t + kWD);   // packs carry kWD zero steps
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto step = [&](uint4 (&a)[2][NPW], const uint4 (&an)[2][NPW], int t, int bs) {
    if constexpr (H) {
      step_h(a, an, t, bs);
    } else {
      const int tn = t + BD < nsteps ? t + BD : nsteps - 1;
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        mm(pt, a[0][2], a[1][2], b[bs][pt][0]);                      // W2.X0
        __builtin_amdgcn_sched_barrier(0);
        if (pt == 1) wl(a, 2, t + kWD);
        __builtin_amdgcn_sched_barrier(0);
        mm(pt, a[0][1], a[1][1], b[bs][pt][1]);                      // W1.X1
        mm(pt, a[0][0], a[1][0], b[bs][pt][2]);                      // W0.X2
        __builtin_amdgcn_sched_barrier(0);
        bl(bs, tn, pt, 2);
        __builtin_amdgcn_sched_barrier(0);
        mm(pt, a[0][1], a[1][1], b[bs][pt][0]);                      // W1.X0
        __builtin_amdgcn_sched_barrier(0);
        if (pt == 1) wl(a, 1, t + kWD);
        __builtin_amdgcn_sched_barrier(0);
        mm(pt, a[0][0], a[1][0], b[bs][pt][1]);                      // W0.X1
        __builtin_amdgcn_sched_barrier(0);
        bl(bs, tn, pt, 1);
        __builtin_amdgcn_sched_barrier(0);
        mm(pt, a[0][0], a[1][0], b[bs][pt][0]);                      // W0.X0
        __builtin_amdgcn_sched_barrier(0);
        bl(bs, tn, pt, 0);
        if (pt == 1) wl(a, 0, t + kWD);   // packs carry kWD zero steps
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // unrolled by U = lcm(kWD, BD) so the weight and B slots are compile-time
  constexpr int U = (BD == 2 && kWD % 2) ? 2 * kWD : kWD;
  int t = 0;
#pragma unroll 1
  for (; t + U <= nsteps; t += U) {
#pragma unroll
    for (int d = 0; d < U; ++d) step(w.a[d % kWD], w.a[(d + 1) % kWD], t + d, d % BD);
  }
#pragma unroll
  for (int d = 0; d < U - 1; ++d)   // the ring then holds padding; prime() refills it
    if (t + d < nsteps) step(w.a[d % kWD], w.a[(d + 1) % kWD], t + d, d % BD);
}

// (x0, x1) -> f16 split of y = lrelu(x mul) (splith's planes: hi = f16(y),
// lo = f16((y - hi) 2^11), bit-identical), from Y = 2^11 y = max(x k, x ks)
// (k = 2^11 mul, ks = k s; mul is a power of two, so Y is exact) with four
// v_fma_mix ops: hi = f16(Y 2^-11), lo = f16(Y - 2^11 hi), one rounding each.
// 4 VALU per pair of values (+ the packed lrelu) instead of splith's 6.
__device__ __forceinline__ void lrelu_splith(float x0, float x1, float k, float ks, unsigned& hi, unsigned& lo) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 x = {x0, x1};
  const f2 Y = __builtin_elementwise_max(x * k, x * ks);
  asm volatile(
      "v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %0, %5, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, %0, %5, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(Y.x), "v"(Y.y), "s"(0x1p-11f), "s"(-2048.f));
}

// lrelu(mul * acc) -> layer-input planes, rows 32(T0+T) + 8q + 4h + i: one
// ds_write_b64 per plane and quad.  (h2: an activation beyond the f16 range
// becomes an infinite high half; the launch detects it from its non-finite
// outputs, see the range flag, instead of testing every activation.)
template <bool H>
__device__ __forceinline__ void store_act(const f32x16 (&acc)[4], char* planes, float s, float mul, int lane,
                                          int T0, int pstride = kPlaneX) {
  const int c = lane & 31, h = lane >> 5;
  if constexpr (H) {
    const float k = 2048.f * mul, ks = k * s;   // exact: mul is a power of two
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x16& v = acc[2 * pt + T];
          unsigned a0, a1, b0, b1;
          lrelu_splith(v[4 * q], v[4 * q + 1], k, ks, a0, a1);
          lrelu_splith(v[4 * q + 2], v[4 * q + 3], k, ks, b0, b1);
          char* d = planes + ((4 * (T0 + T) + q) * kXT + 32 * pt + c) * 16 + 8 * h;
          *reinterpret_cast<uint2*>(d) = make_uint2(a0, b0);
          *reinterpret_cast<uint2*>(d + pstride) = make_uint2(a1, b1);
        }
    return;
  }
#pragma unroll
  for (int pt = 0; pt < 2; ++pt)
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x16& v = acc[2 * pt + T];
        unsigned a0, a1, a2, b0, b1, b2;
        // lrelu(x) = max(x, s x) for 0 <= s <= 1 (same value and sign of zero)
        split2(fmaxf(v[4 * q], s * v[4 * q]), fmaxf(v[4 * q + 1], s * v[4 * q + 1]), a0, a1, a2);
        split2(fmaxf(v[4 * q + 2], s * v[4 * q + 2]), fmaxf(v[4 * q + 3], s * v[4 * q + 3]), b0, b1, b2);
        char* d = planes + ((4 * (T0 + T) + q) * kXT + 32 * pt + c) * 16 + 8 * h;
        *reinterpret_cast<uint2*>(d) = make_uint2(a0, b0);
        *reinterpret_cast<uint2*>(d + kPlaneX) = make_uint2(a1, b1);
        *reinterpret_cast<uint2*>(d + 2 * kPlaneX) = make_uint2(a2, b2);
      }
}

// h2: block1.2 / block3.2 biases start the accumulators (acc = b / scale,
// exact: the scale is a power of two) instead of riding in the GEMM as an
// extra input row, so those layers take 16 k-steps instead of 17.
template <bool H>
__device__ __forceinline__ void acc_init(f32x16 (&acc)[4], const float* bias, float inv_scale, int lane, int T0) {
  if constexpr (H) {
    const int h = lane >> 5;
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(bias + 32 * (T0 + T) + 8 * q + 4 * h);
        const float v[4] = {b.x * inv_scale, b.y * inv_scale, b.z * inv_scale, b.w * inv_scale};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[T][4 * q + i] = v[i];
          acc[2 + T][4 * q + i] = v[i];
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x16){0.f};
  }
}
constexpr int kBiasSteps(bool H) { return H ? 16 : 17; }   // block1.2 / block3.2 k-steps

// 8 fp32 rows of one pair -> row group g of the NPL planes (ds_write_b128 each)
template <bool H>
__device__ __forceinline__ void store_group(char* planes, int pstride, int g, int pair, const float (&v)[8]) {
  if constexpr (H) {
    uint4 p0, p1;
    splith(v[0], v[1], p0.x, p1.x);
    splith(v[2], v[3], p0.y, p1.y);
    splith(v[4], v[5], p0.z, p1.z);
    splith(v[6], v[7], p0.w, p1.w);
    char* d = planes + (g * kXT + pair) * 16;
    *reinterpret_cast<uint4*>(d) = p0;
    *reinterpret_cast<uint4*>(d + pstride) = p1;
    return;
  }
  uint4 p0, p1, p2;
  split2(v[0], v[1], p0.x, p1.x, p2.x);
  split2(v[2], v[3], p0.y, p1.y, p2.y);
  split2(v[4], v[5], p0.z, p1.z, p2.z);
  split2(v[6], v[7], p0.w, p1.w, p2.w);
  char* d = planes + (g * kXT + pair) * 16;
  *reinterpret_cast<uint4*>(d) = p0;
  *reinterpret_cast<uint4*>(d + pstride) = p1;
  *reinterpret_cast<uint4*>(d + 2 * pstride) = p2;
}

// producer wave pw (0..3), lane = pair column: gather + weights + PE planes of `tile`
// into buffer nb (neural_points.py:788-799, point_aggregators.py:421-429, 775-804).
// The gather is split in three stages so its dependent loads travel across
// barriers (the producers' barriers wait on LDS only): the sample row (stage
// 0, tile start), then pidx / sample positions / dir row (stage 1, S1b), then
// the point rows and everything computed from them (gather, during block1.2).
struct GatherState {
  int64_t tile;
  int64_t row;
  int pid;
  float sw[3], sp[3];
  int64_t dmap;
  bool active;
};

__device__ __forceinline__ void gather_row(const X3Args& A, int64_t tile, int lane, GatherState& g) {
  const int64_t v = tile * kXTS + (lane >> 3);
  g.tile = tile;
  g.active = v < eff_n(A.s);
  g.row = g.active ? sample_row(A.s, v) : 0;
}

__device__ __forceinline__ void gather_sample(const X3Args& A, int lane, GatherState& g) {
  const int k = lane & 7, K = A.s.K;
  g.pid = (g.active && k < K) ? A.s.pidx[g.row * K + k] : -1;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    g.sw[a] = g.active ? A.s.sample_w[g.row * 3 + a] : 0.f;
    g.sp[a] = g.active ? A.s.sample_p[g.row * 3 + a] : 0.f;
  }
  g.dmap = A.s.dir_map ? (int64_t)A.s.dir_map[g.row] : g.row;
}

template <bool H, bool TR = false>
__device__ __forceinline__ void gather(const X3Args& A, const GatherState& g, int nb, int nw, char* lds, int pw, int lane,
                                       float (&dr6)[6]) {
  using L = XL<H>;
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
  const int j = lane >> 3, k = lane & 7;
  const int K = A.s.K;
  const bool active = g.active;
  const int64_t row = g.row;
  const bool valid = g.pid >= 0;
  const int64_t prow = valid ? g.pid : (active && k < K ? 0 : -1);   // torch.clamp(sample_pidx, min=0)
  float sw[3], sp[3], vd[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    sw[a] = g.sw[a];
    sp[a] = g.sp[a];
  }
  const int64_t drow = active ? g.dmap / A.s.dir_div : 0;
  // the view / point directions, colour and confidence feed the extras and the
  // weights, which producer wave 0 alone writes: the others load only what their
  // PE channels need (wave-uniform branch)
  if (active && pw == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) vd[a] = A.s.dirs[drow * 3 + a];
  }
  float pw3[3] = {0.f, 0.f, 0.f}, pp[3] = {0.f, 0.f, 0.f}, col[3] = {0.f, 0.f, 0.f}, pdir[3] = {0.f, 0.f, 0.f};
  float cf = 1.f;
  if (valid) {
#pragma unroll
    for (int a = 0; a < 3; ++a) pw3[a] = A.pts.xyz[prow * 3 + a];
    if (pw == 0) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        col[a] = A.pts.color ? A.pts.color[prow * 3 + a] : 0.f;
        pdir[a] = A.pts.dir ? A.pts.dir[prow * 3 + a] : 0.f;
      }
    }
    if (A.pts.pers) {
#pragma unroll
      for (int a = 0; a < 3; ++a) pp[a] = A.pts.pers[prow * 3 + a];
    } else {
      pair_pers(A.pts, A.s, drow, pw3, cam_c, cam_R, pp);
    }
  }
  if (pw == 0 && A.pts.conf && prow >= 0) cf = A.pts.conf[prow];
  float d6[6];
  d6[0] = pw3[0] - sw[0];
  d6[1] = pw3[1] - sw[1];
  d6[2] = pw3[2] - sw[2];
  d6[3] = pp[0] * pp[2] - sp[0] * sp[2];
  d6[4] = pp[1] * pp[2] - sp[1] * sp[2];
  d6[5] = pp[2] - sp[2];
  mat3(Rw, d6, dr6);
  dr6[3] = d6[3];
  dr6[4] = d6[4];
  dr6[5] = d6[5];
  if (A.pts.rw2c) rot_point(A.pts.rw2c, prow, d6, dr6);   // per-point Rw2c (agg_common.h)
  if (pw == 0) {
    const float nrm = sqrtf(d6[0] * d6[0] + d6[1] * d6[1] + d6[2] * d6[2]);
    const float wl = valid ? 1.f / fmaxf(nrm, 1e-6f) : 0.f;
    const float wsum = xor8_sum(wl);
    const float wn = wl / fmaxf(wsum, 1e-8f);
    const float confc = fminf(fmaxf(cf, 1e-4f), 1.f);
    const bool samp_valid = xor8_sum(valid ? 1.f : 0.f) > 0.f;
    float vrot[3], drot[3];
    mat3(Rw, vd, vrot);
    mat3(Rw, pdir, drot);
    if (A.pts.rw2c) {
      rot_point(A.pts.rw2c, prow, pdir, drot);
      rot_point(A.pts.rw2c, active ? slot0_point(A.s, row) : 0, vd, vrot);
    }
    const float dot = drot[0] * vrot[0] + drot[1] * vrot[1] + drot[2] * vrot[2];
    const float ex[8] = {col[0], col[1], col[2], drot[0] - vrot[0], drot[1] - vrot[1], drot[2] - vrot[2], dot, 1.f};
    float* exL = reinterpret_cast<float*>(lds + L::OffEx) + nb * 8 * kXT;
#pragma unroll
    for (int e = 0; e < 8; ++e) exL[e * kXT + lane] = ex[e];
    reinterpret_cast<float*>(lds + L::OffWt)[nw * kXT + lane] = wn * confc;
    reinterpret_cast<int*>(lds + L::OffPr)[nb * kXT + lane] = valid ? (int)prow : -1;
    if (k == 0) reinterpret_cast<int*>(lds + L::OffSf)[nw * kXTS + j] = active && samp_valid;
    if (active && k < K) {
      if (A.out_weight) A.out_weight[row * K + k] = wn;
      if (A.out_conf) A.out_conf[row * K + k] = confc;
    }
    if (TR && active) {   // training saves, k_pairs<true>'s layout (aggregate.hip)
      const int64_t pr = g.tile * kXT + lane;
      float4* x = reinterpret_cast<float4*>(A.sv.x3e + pr * 32);
      x[0] = make_float4(ex[0], ex[1], ex[2], ex[3]);
      x[1] = make_float4(ex[4], ex[5], ex[6], ex[7]);
#pragma unroll
      for (int e = 2; e < 8; ++e) x[e] = make_float4(0.f, 0.f, 0.f, 0.f);
      A.sv.wt[pr] = wn * confc;
      A.sv.wn[pr] = wn;
      A.sv.prow[pr] = valid ? (int32_t)prow : -1;
    }
  }
}

// 5-band PE of the rotated 6-d distance of this lane's pair -> rows 2e (sin),
// 2e + 1 (cos), e = 5 ch + f, of the PE planes (networks.py:175-190).
// Producer wave pw owns channel ch = pw (PART 0) and ch = 4 + pw (PART 1, pw < 2),
// one sincosf per band, as the reference (angle doubling was measured 0.3 ms
// faster but rounded differently where the compiler inlined it in the prologue
// and in the loop, which made a sample's bits depend on its tile).
template <bool H>
__device__ __forceinline__ void pe_store(char* lds, int lane, int e, float sn, float cs) {
  using L = XL<H>;
  const int r = 2 * e;
  char* d = lds + L::OffPE + ((r >> 3) * kXT + lane) * 16 + 2 * (r & 7);
  if constexpr (H) {
    unsigned x0, x1;
    splith(sn, cs, x0, x1);
    *reinterpret_cast<unsigned*>(d) = x0;
    *reinterpret_cast<unsigned*>(d + kPlaneP) = x1;
  } else {
    unsigned x0, x1, x2;
    split2(sn, cs, x0, x1, x2);
    *reinterpret_cast<unsigned*>(d) = x0;
    *reinterpret_cast<unsigned*>(d + kPlaneP) = x1;
    *reinterpret_cast<unsigned*>(d + 2 * kPlaneP) = x2;
  }
}

template <bool H, int PART, bool TR = false>
__device__ __forceinline__ void pe_planes(char* lds, int pw, int lane, const float (&dr6)[6],
                                          const X3Args* A = nullptr, const GatherState* g = nullptr) {
  using L = XL<H>;
  float* pe5 = TR && g->active ? A->sv.pe5 + (g->tile * kXT + lane) * 64 : nullptr;   // training: [pair][64]
  if (pw == 0 && PART == 0) {   // rows 60..63: the 4th 16-k step reads them
    char* pz = lds + L::OffPE + (7 * kXT + lane) * 16 + 8;
#pragma unroll
    for (int pl = 0; pl < L::NPL; ++pl) *reinterpret_cast<uint2*>(pz + pl * kPlaneP) = make_uint2(0u, 0u);
    if (TR && pe5) *reinterpret_cast<float4*>(pe5 + 60) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int mine = __builtin_amdgcn_readfirstlane(PART == 0 ? pw : 4 + pw);
#pragma unroll
  for (int ch = 4 * PART; ch < (PART == 0 ? 4 : 6); ++ch) {
    if (ch != mine) continue;   // wave-uniform
    float s0, c0, s1, c1, s2, c2, s3, c3, s4, c4;
    sincosf(dr6[ch], &s0, &c0);
    sincosf(dr6[ch] * 2.f, &s1, &c1);
    sincosf(dr6[ch] * 4.f, &s2, &c2);
    sincosf(dr6[ch] * 8.f, &s3, &c3);
    sincosf(dr6[ch] * 16.f, &s4, &c4);
    pe_store<H>(lds, lane, 5 * ch + 0, s0, c0);
    pe_store<H>(lds, lane, 5 * ch + 1, s1, c1);
    pe_store<H>(lds, lane, 5 * ch + 2, s2, c2);
    pe_store<H>(lds, lane, 5 * ch + 3, s3, c3);
    pe_store<H>(lds, lane, 5 * ch + 4, s4, c4);
    if (TR && pe5) {
      const float sv[10] = {s0, c0, s1, c1, s2, c2, s3, c3, s4, c4};
#pragma unroll
      for (int i = 0; i < 10; i += 2) *reinterpret_cast<float2*>(pe5 + 10 * ch + i) = make_float2(sv[i], sv[i + 1]);
    }
  }
}

// Tile schedule (8 barriers per tile; consumers C = waves 0..3, producers P = 4..7):
//   C: acc = W1b . PE           | P: park P1(tile), finalize alpha of the previous tile
//   S1  C: acc += P1 (parked)   |
//   S1b C: store act1, bias     |
//   S2  C: block1.2             | P: gather(next)
//   S3  C: store act2, extras   | P: fetch P1(next) (registers), PE planes part 1
//   S4  C: block3.0             |
//   S5  C: store act3, bias     | P: PE planes part 2
//   S6  C: block3.2, K sums, alpha partials
//   S7
// The consumers never wait on a producer phase shorter than the layer it
// overlaps; the P1 rows travel during block3.0 / block3.2.
#define X3_SYNC() __syncthreads()

template <bool H, bool TR = false>
__device__ __forceinline__ void finalize_alpha(const X3Args& A, char* lds, int buf, int64_t tile, int lane) {
  using L = XL<H>;
  const int64_t n = eff_n(A.s);
  const int j = lane >> 3, k = lane & 7;
  const float* apart = reinterpret_cast<const float*>(lds + L::OffAp);
  const float* wtL = reinterpret_cast<const float*>(lds + L::OffWt) + buf * kXT;
  const int* sflag = reinterpret_cast<const int*>(lds + L::OffSf) + buf * kXTS;
  const float pa = apart[lane] + apart[kXT + lane] + apart[2 * kXT + lane] + apart[3 * kXT + lane] + A.w.ba[0];
  const float alpha_k = A.w.act_super ? softplus(pa - 1.f) : fmaxf(pa, 0.f);
  const float alpha_s = xor8_sum(wtL[lane] * alpha_k);   // point_aggregators.py:608-614
  const int64_t vo = tile * kXTS + j;
  if (TR && vo < n) A.sv.pa[tile * kXT + lane] = pa;
  if (k == 0 && vo < n) {
    A.vmask[vo] = sflag[j];
    if (sflag[j]) A.out_feat[vo * (kC + 1)] = alpha_s;
  }
}

// Training save of a layer's pre-activations acc * sc (sc: the h2 layer's output
// factor, 1 on x3 -- the same product store_act rounds): lrelu -> dst[pair][256]
// and the LeakyReLU derivative bits mask[pair][16 layer + 2T + h] (bit r: register
// r of neuron tile T, lane half h), the layout of aggregate.hip's save_pairs_q.
template <bool H>
__device__ __forceinline__ void save_act_train(const X3Args& A, const f32x16 (&acc)[4], float* dst, int layer,
                                               int64_t tile, int64_t n, float neg, int lane, int T0, float sc) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) {
    const int col = 32 * pt + c;
    if (tile * kXTS + (col >> 3) >= n) continue;
    const int64_t pr = tile * kXT + col;
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      f32x16 v = acc[2 * pt + T];
      if constexpr (H) v = v * sc;
      unsigned bits = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(dst + pr * kHid + 32 * (T0 + T) + 8 * q + 4 * h) =
            make_float4(lrelu(v[4 * q], neg), lrelu(v[4 * q + 1], neg), lrelu(v[4 * q + 2], neg),
                        lrelu(v[4 * q + 3], neg));
#pragma unroll
      for (int r = 0; r < 16; ++r) bits |= (v[r] > 0.f ? 1u : 0u) << r;
      A.sv.mask[pr * 64 + 16 * layer + 2 * (T0 + T) + h] = (uint16_t)bits;
    }
  }
}

template <bool H, bool TR = false>
__device__ __forceinline__ void consumer_loop(const X3Args& A, char* lds, int wid, int lane) {
  using L = XL<H>;
  const int c = lane & 31, h = lane >> 5;
  const int64_t n = eff_n(A.s);
  const int64_t ntiles = cdiv(n, kXTS);
  const float neg = A.w.neg_slope;
  char* XP = lds;
  const char* PE = lds + L::OffPE;
  const float* P1L = reinterpret_cast<const float*>(lds);   // P1 rows parked in the XP area between tiles
  float* apart = reinterpret_cast<float*>(lds + L::OffAp);
  const float* waL = reinterpret_cast<const float*>(lds + L::OffWa);
  const int T0 = 2 * wid;
  const int voff = (T0 * L::NPW * 64 + lane) * 16;
  const __amdgpu_buffer_rsrc_t r1 = rsrc(A.wx.pack[0]), r2 = rsrc(A.wx.pack[1]), r3 = rsrc(A.wx.pack[2]),
                               r4 = rsrc(A.wx.pack[3]);
  // layer output factors (h2: 2^(s-11) of the pre-scaled f16 packs; x3: 1, unused)
  const float sc1 = A.wx.scale[0], sc2 = A.wx.scale[1], sc3 = A.wx.scale[2], sc4 = A.wx.scale[3];
  WRing<H> wr;
  f32x16 acc[4];
  prime<H>(wr, r1, voff);
  X3_SYNC();   // S0: the first tile's PE planes, extras and weights are in LDS
  const int* TQ = reinterpret_cast<const int*>(lds + L::OffTq);
  int it = 0;
  for (int64_t tile = first_tile(ntiles); tile < ntiles; tile = TQ[(it + 1) & 3], ++it) {
    const int buf = it & 1;
    // ------------------------------------------------------------ block1.0 = P1 + W1[:, 224:] . PE_5
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x16){0.f};
    layer<H>(acc, wr, r1, voff, PE, kPlaneP, 4, lane);
    prime<H>(wr, r2, voff);
    X3_SYNC();   // S1: P1 parked, PE planes consumed
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v4 = *reinterpret_cast<const float4*>(P1L + (32 * pt + c) * kP1Pitch + 32 * (T0 + T) + 8 * q +
                                                             4 * h);
          if constexpr (H) {
            acc[2 * pt + T][4 * q] = fmaf(acc[2 * pt + T][4 * q], sc1, v4.x);
            acc[2 * pt + T][4 * q + 1] = fmaf(acc[2 * pt + T][4 * q + 1], sc1, v4.y);
            acc[2 * pt + T][4 * q + 2] = fmaf(acc[2 * pt + T][4 * q + 2], sc1, v4.z);
            acc[2 * pt + T][4 * q + 3] = fmaf(acc[2 * pt + T][4 * q + 3], sc1, v4.w);
          } else {
            acc[2 * pt + T][4 * q] += v4.x;
            acc[2 * pt + T][4 * q + 1] += v4.y;
            acc[2 * pt + T][4 * q + 2] += v4.z;
            acc[2 * pt + T][4 * q + 3] += v4.w;
          }
        }
    X3_SYNC();   // S1b: the parked P1 read by every consumer (the planes overwrite it)
    store_act<H>(acc, XP, neg, 1.f, lane, T0);
    if constexpr (TR) save_act_train<H>(A, acc, A.sv.h1, 0, tile, n, neg, lane, T0, 1.f);
    if (wid == 0) {
#pragma unroll
      for (int pl = 0; pl < L::NPL; ++pl) {   // row 256 = 1 (bias column), 257..271 = 0 (the parked P1 was here)
        *reinterpret_cast<uint4*>(XP + pl * kPlaneX + (32 * kXT + lane) * 16) =
            make_uint4(pl == 0 ? L::kOne : 0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(XP + pl * kPlaneX + (33 * kXT + lane) * 16) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    acc_init<H>(acc, A.w.b2, 1.f / sc2, lane, T0);
    X3_SYNC();   // S2
    // ------------------------------------------------------------ block1.2
    layer<H>(acc, wr, r2, voff, XP, kPlaneX, kBiasSteps(H), lane);
    prime<H>(wr, r3, voff);
    X3_SYNC();   // S3
    store_act<H>(acc, XP, neg, sc2, lane, T0);
    if constexpr (TR) save_act_train<H>(A, acc, A.sv.h2, 1, tile, n, neg, lane, T0, sc2);
    if (wid == 0) {   // block3.0 inputs 256..263: colour, R.dir - R.v, <R.dir, R.v>, bias
      const float* exL = reinterpret_cast<const float*>(lds + L::OffEx) + buf * 8 * kXT;
      float ex[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ex[e] = exL[e * kXT + lane];
      store_group<H>(XP, kPlaneX, 32, lane, ex);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x16){0.f};
    X3_SYNC();   // S4
    // ------------------------------------------------------------ block3.0
    layer<H>(acc, wr, r3, voff, XP, kPlaneX, 17, lane);
    prime<H>(wr, r4, voff);
    X3_SYNC();   // S5
    store_act<H>(acc, XP, neg, sc3, lane, T0);
    if constexpr (TR) save_act_train<H>(A, acc, A.sv.h3, 2, tile, n, neg, lane, T0, sc3);
    if (wid == 0 && !H) {
#pragma unroll
      for (int pl = 0; pl < L::NPL; ++pl)
        *reinterpret_cast<uint4*>(XP + pl * kPlaneX + (32 * kXT + lane) * 16) =
            make_uint4(pl == 0 ? L::kOne : 0u, 0u, 0u, 0u);
    }
    acc_init<H>(acc, A.w.b4, 1.f / sc4, lane, T0);
    X3_SYNC();   // S6
    // ------------------------------------------------------------ block3.2, alpha partials, K sums
    layer<H>(acc, wr, r4, voff, XP, kPlaneX, kBiasSteps(H), lane);
    prime<H>(wr, r1, voff);   // the next tile's block1.0
    if constexpr (H) {
      if constexpr (TR) save_act_train<H>(A, acc, A.sv.h4, 3, tile, n, neg, lane, T0, sc4);
      // block3.2 accumulators -> LDS [pair][row] for the producers' tail (next tile):
      // one ds_write_b128 per accumulator quad, conflict-free at kP1Pitch
      float* H4 = reinterpret_cast<float*>(lds + L::OffH4);
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int T = 0; T < 2; ++T)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x16& v = acc[2 * pt + T];
            *reinterpret_cast<float4*>(H4 + (32 * pt + c) * kP1Pitch + 32 * (T0 + T) + 8 * q + 4 * h) =
                make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
          }
    } else {
      if constexpr (TR) save_act_train<H>(A, acc, A.sv.h4, 3, tile, n, neg, lane, T0, 1.f);
      const float* wtL = reinterpret_cast<const float*>(lds + L::OffWt) + buf * kXT;
      const int* sflag = reinterpret_cast<const int*>(lds + L::OffSf) + buf * kXTS;
      float pa_part[2] = {0.f, 0.f};
      const int i8 = c & 7;
      const bool b2 = (i8 & 4) != 0, b1 = (i8 & 2) != 0, b0 = (i8 & 1) != 0;
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const float wtp = wtL[32 * pt + c];
        const int sj = (32 * pt + c) >> 3;
        const int64_t vo = tile * kXTS + sj;
        const bool wrt = vo < n && sflag[sj];
#pragma unroll
        for (int T = 0; T < 2; ++T) {
          float v[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float hv = lrelu(H ? acc[2 * pt + T][r] * sc4 : acc[2 * pt + T][r], neg);
            pa_part[pt] += waL[32 * (T0 + T) + acc_row(r, h)] * hv;
            v[r] = wtp * hv;
          }
          // K sums (point_aggregators.py:622-628): DPP reduce-scatter over the 8 lanes of a sample
          float w8[8], w4[4], w2[2];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float send = b2 ? v[q] : v[q + 8];
            const float recv = __builtin_bit_cast(
                float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0x141, 0xf, 0xf, false));
            w8[q] = (b2 ? v[q + 8] : v[q]) + recv;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float send = b1 ? w8[q] : w8[q + 4];
            const float recv = __builtin_bit_cast(
                float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0x4E, 0xf, 0xf, false));
            w4[q] = (b1 ? w8[q + 4] : w8[q]) + recv;
          }
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float send = b0 ? w4[q] : w4[q + 2];
            const float recv = __builtin_bit_cast(
                float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xf, 0xf, false));
            w2[q] = (b0 ? w4[q + 2] : w4[q]) + recv;
          }
          if (wrt)
            __builtin_nontemporal_store(
                (f32x2n){w2[0], w2[1]},
                reinterpret_cast<f32x2n*>(A.hid + vo * kHid + 32 * (T0 + T) + ((2 * i8) & 3) + 8 * (i8 >> 1) + 4 * h));
        }
        pa_part[pt] += __shfl_xor(pa_part[pt], 32);
      }
      if (h == 0) {
        apart[wid * kXT + c] = pa_part[0];
        apart[wid * kXT + 32 + c] = pa_part[1];
      }
    }
    X3_SYNC();   // S7: layer-input planes free (the producers park the next P1 there), alpha partials ready
  }
}

// Producer wave pw: P1 rows 16 pw .. 16 pw + 15 of a tile (1 KB each, one
// coalesced float4 per lane per row) into registers.
__device__ __forceinline__ unsigned fetch_p1(f32x4n (&r)[16], const X3Args& A, const int* prow, int pw, int lane) {
  // branch-free: every lane loads (row 0 for an empty slot) and zeroes afterwards,
  // so the 16 loads issue back to back; streamed once -> non-temporal (keeps the
  // weight packs in L2)
  int64_t rows[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int pr = prow[16 * pw + i];
    rows[i] = pr < 0 ? -1 : (A.pts.used_map ? (int64_t)A.pts.used_map[pr] : (int64_t)pr);
  }
  unsigned empty = 0;   // bit i: row i has no point (zeroed when parked, so the loads are not waited on here)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    r[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4n*>(A.p1 + (rows[i] < 0 ? 0 : rows[i]) * kHid) +
                                      lane);
    if (rows[i] < 0) empty |= 1u << i;
  }
  return empty;
}

__device__ __forceinline__ void park_p1(const f32x4n (&r)[16], unsigned empty, char* lds, int pw, int lane) {
  float* P1L = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const f32x4n z = {0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4n*>(P1L + (16 * pw + i) * kP1Pitch + 4 * lane) = ((empty >> i) & 1) ? z : r[i];
  }
}

// h2 tile tail on the producers (one tile late, during the consumers' block1.2):
// from the block3.2 accumulators the consumers parked in H4, per sample j of
// the tile (wave pw: samples 2pw, 2pw + 1; lane & 31 = neurons 8ng .. 8ng + 7)
//   h = lrelu(acc * scale)                    point_aggregators.py (block3)
//   hid[j] = sum_k wt_k h_k                   (K sums, :622-628)
//   alpha_k = act(wa . h_k + ba), alpha_j = sum_k wt_k alpha_k   (:608-614)
// the dot over 256 neurons is a reduce-scatter over the 32 lanes.  chk picks
// up every output as 0 * x: NaN once one is not finite (an f16-split
// activation beyond 65504 has an infinite high half, and every output it
// reaches is inf or NaN, 0 x inf on the empty pairs' zero weights included).
struct TailState {
  float hs[8], pa[8];
};

// PART 0: pairs k = 0..3 of every sample; PART 1: k = 4..7, the reductions and
// the stores (the halves run in two producer segments, see producer_loop)
template <int PART, bool TR = false>
__device__ __forceinline__ void producer_tail(const X3Args& A, char* lds, int slot, int64_t tile, int pw, int lane,
                                              TailState& ts, float& chk) {
  using L = XL<true>;
  const int64_t n = eff_n(A.s);
  const int j = 2 * pw + (lane >> 5), ng = lane & 31;
  const float* H4 = reinterpret_cast<const float*>(lds + L::OffH4);
  const float* wtL = reinterpret_cast<const float*>(lds + L::OffWt) + slot * kXT + 8 * j;
  const int sf = reinterpret_cast<const int*>(lds + L::OffSf)[slot * kXTS + j];
  const float* waL = reinterpret_cast<const float*>(lds + L::OffWa) + 8 * ng;
  const float sc = A.wx.scale[3], neg = A.w.neg_slope;
  const float4 wa0 = *reinterpret_cast<const float4*>(waL), wa1 = *reinterpret_cast<const float4*>(waL + 4);
  const float wa[8] = {wa0.x, wa0.y, wa0.z, wa0.w, wa1.x, wa1.y, wa1.z, wa1.w};
  const float4 wt0 = *reinterpret_cast<const float4*>(wtL), wt1 = *reinterpret_cast<const float4*>(wtL + 4);
  const float wt[8] = {wt0.x, wt0.y, wt0.z, wt0.w, wt1.x, wt1.y, wt1.z, wt1.w};
  float (&hs)[8] = ts.hs;
  float (&pa)[8] = ts.pa;
#pragma unroll
  for (int k = 4 * PART; k < 4 * PART + 4; ++k) {
    const float* row = H4 + (8 * j + k) * kP1Pitch + 8 * ng;
    const float4 a = *reinterpret_cast<const float4*>(row), b = *reinterpret_cast<const float4*>(row + 4);
    const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    float p = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float hv = lrelu(x[i] * sc, neg);
      p = fmaf(wa[i], hv, p);
      hs[i] = k == 0 ? wt[0] * hv : fmaf(wt[k], hv, hs[i]);
    }
    pa[k] = p;
  }
  if (PART == 0) return;
  // reduce-scatter of pa[0..7] over the 32 lanes: lane ng ends with pair k = ng >> 2
  const bool b4 = (ng & 16) != 0, b3 = (ng & 8) != 0, b2 = (ng & 4) != 0;
  float r4[4], r2[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) r4[q] = (b4 ? pa[q + 4] : pa[q]) + __shfl_xor(b4 ? pa[q] : pa[q + 4], 16);
#pragma unroll
  for (int q = 0; q < 2; ++q) r2[q] = (b3 ? r4[q + 2] : r4[q]) + __shfl_xor(b3 ? r4[q] : r4[q + 2], 8);
  float r1 = (b2 ? r2[1] : r2[0]) + __shfl_xor(b2 ? r2[0] : r2[1], 4);
  r1 += __shfl_xor(r1, 2);
  r1 += __shfl_xor(r1, 1);
  const float pk = r1 + A.w.ba[0];
  if (TR && (ng & 3) == 0 && tile * kXTS + j < n) A.sv.pa[tile * kXT + 8 * j + (ng >> 2)] = pk;
  const float alpha_k = A.w.act_super ? softplus(pk - 1.f) : fmaxf(pk, 0.f);
  float as = wtL[ng >> 2] * alpha_k;   // each k held by 4 lanes: sum over bits 2..4
  as += __shfl_xor(as, 4);
  as += __shfl_xor(as, 8);
  as += __shfl_xor(as, 16);
  chk = fmaf(0.f, (hs[0] + hs[1]) + (hs[2] + hs[3]) + (hs[4] + hs[5]) + (hs[6] + hs[7]) + as, chk);
  const int64_t vo = tile * kXTS + j;
  if (vo < n) {
    if (ng == 0) {
      A.vmask[vo] = sf;
      if (sf) A.out_feat[vo * (kC + 1)] = as;
    }
    if (TR) {   // training: fp32 hid rows [n][256] for the fp32 colour branch (k_color<true>)
      if (sf) {
        float4* dst = reinterpret_cast<float4*>(A.hid + vo * kHid + 8 * ng);
        dst[0] = make_float4(hs[0], hs[1], hs[2], hs[3]);
        dst[1] = make_float4(hs[4], hs[5], hs[6], hs[7]);
      }
    } else if (sf) {   // hid rows 8ng..8ng+7 as one 16-B piece per plane (kHidTile layout)
      typedef unsigned u32x4n __attribute__((ext_vector_type(4)));
      unsigned a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) splith(hs[2 * i], hs[2 * i + 1], a[i], b[i]);
      const u32x4n p0 = {a[0], a[1], a[2], a[3]}, p1 = {b[0], b[1], b[2], b[3]};
      u32x4n* dst = reinterpret_cast<u32x4n*>(reinterpret_cast<char*>(A.hid) + (vo / kXT) * kHidTile +
                                              (ng * kXT + vo % kXT) * 16);
      dst[0] = p0;   // plain stores: the tile's 4 producer waves fill each 128-B line in
      dst[kHidPlane / 16] = p1;   // 32-B pieces, merged in L2 (nontemporal: +1.4 ms)
    }
  }
}

template <bool H, bool TR = false>
__device__ __forceinline__ void producer_loop(const X3Args& A, char* lds, int pw, int lane) {
  using L = XL<H>;
  const int64_t n = eff_n(A.s);
  const int64_t ntiles = cdiv(n, kXTS);
  __builtin_amdgcn_s_setprio(kProducerPrio);   // producer issue priority over the MFMA stream
  f32x4n p1r[16];
  unsigned p1e = 0;
  float dr6[6];
  GatherState g;
  gather_row(A, first_tile(ntiles), lane, g);
  gather_sample(A, lane, g);
  gather<H, TR>(A, g, 0, 0, lds, pw, lane, dr6);
  pe_planes<H, 0, TR>(lds, pw, lane, dr6, &A, &g);
  pe_planes<H, 1, TR>(lds, pw, lane, dr6, &A, &g);
  int* TQ = reinterpret_cast<int*>(lds + L::OffTq);
  if (pw == 0 && lane == 0) TQ[1] = (int)take_tile(A, ntiles);
  X3_SYNC();   // P0: prow of the first tile visible to all producers, TQ[1] too
  p1e = fetch_p1(p1r, A, reinterpret_cast<const int*>(lds + L::OffPr), pw, lane);
  X3_SYNC();   // S0
  float chk = 0.f;   // h2 tails: 0 * outputs (producer_tail)
  TailState ts;
  int it = 0;
  int64_t prev = -1;   // the previous iteration's tile (its tail / alpha run one tile late)
  for (int64_t tile = first_tile(ntiles); tile < ntiles; prev = tile, tile = TQ[(it + 1) & 3], ++it) {
    const int nbuf = (it & 1) ^ 1;
    const int nw = H ? (it + 1) % 3 : nbuf;   // Wt / Sf slot of the next tile
    const int64_t next = TQ[(it + 1) & 3];
    // the tile after next, published before S1 (only while this workgroup goes on:
    // a tile taken by a workgroup that stops would be lost)
    if (pw == 0 && lane == 0) TQ[(it + 2) & 3] = next < ntiles ? (int)take_tile(A, ntiles) : (int)ntiles;
    park_p1(p1r, p1e, lds, pw, lane);   // the layer-input planes are free since the last S7
    gather_row(A, next, lane, g);
    X3_SYNC();   // S1
    // alpha of the previous tile (its partials stay until this tile's K sums, after S6)
    if (!H && pw == 0 && it > 0) finalize_alpha<H, TR>(A, lds, nbuf, prev, lane);
    X3_SYNC();   // S1b
    gather_sample(A, lane, g);
    X3_SYNC();   // S2
    // during block1.2: gather of the next tile (its slots are free: their last
    // readers were the previous finalize / tail)
    gather<H, TR>(A, g, nbuf, nw, lds, pw, lane, dr6);
    if constexpr (H)   // first half of the previous tile's tail
      if (it > 0) producer_tail<0, TR>(A, lds, (it + 2) % 3, prev, pw, lane, ts, chk);
    X3_SYNC();   // S3: the next tile's point rows are in LDS
    // the P1 rows travel during block3.0 / block3.2 (loads stay in flight across the barriers)
    p1e = fetch_p1(p1r, A, reinterpret_cast<const int*>(lds + L::OffPr) + nbuf * kXT, pw, lane);
    X3_SYNC();   // S4
    pe_planes<H, 0, TR>(lds, pw, lane, dr6, &A, &g);   // during block3.0 (PE planes free since S1)
    // (h2) during block3.0: the second half of the previous tile's tail (its
    // accumulators are overwritten after this tile's S6)
    if constexpr (H)
      if (it > 0) producer_tail<1, TR>(A, lds, (it + 2) % 3, prev, pw, lane, ts, chk);
    X3_SYNC();   // S5
    X3_SYNC();   // S6
    pe_planes<H, 1, TR>(lds, pw, lane, dr6, &A, &g);   // during block3.2
    X3_SYNC();   // S7
  }
  if constexpr (H) {
    // the last tile's tail (its accumulators were parked before the final S7)
    if (it > 0) {
      producer_tail<0, TR>(A, lds, (it - 1) % 3, prev, pw, lane, ts, chk);
      producer_tail<1, TR>(A, lds, (it - 1) % 3, prev, pw, lane, ts, chk);
    }
    if (A.wx.range_flag && chk != 0.f) atomicOr(A.wx.range_flag, 1);
  } else {
    if (pw == 0 && it > 0) finalize_alpha<H, TR>(A, lds, (it - 1) & 1, prev, lane);
  }
}

template <bool H, bool TR = false>
__device__ __forceinline__ void pairs_body(const X3Args& A) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // alpha_branch.0 weights for the consumers' tail
  if (threadIdx.x < kHid) reinterpret_cast<float*>(lds + XL<H>::OffWa)[threadIdx.x] = A.w.wa[threadIdx.x];
  if (wid < 4) {
    X3_SYNC();   // P0
    consumer_loop<H, TR>(A, lds, wid, lane);
  } else {
    producer_loop<H, TR>(A, lds, wid - 4, lane);
  }
}

__global__ void __launch_bounds__(512, 1) k_pairs_x3(X3Args A) { pairs_body<false>(A); }
__global__ void __launch_bounds__(512, 1) k_pairs_h2(X3Args A) { pairs_body<true>(A); }
// training forward (pnr_aggregate_fwd_train_x3): k_pairs_x3 + the saves of k_pairs<true>
__global__ void __launch_bounds__(512, 1) k_pairs_x3_train(X3Args A) { pairs_body<false, true>(A); }
// training forward on fp32h2 (pnr_aggregate_fwd_train_h2): k_pairs_h2 + the same saves, hid in fp32 rows
__global__ void __launch_bounds__(512, 1) k_pairs_h2_train(X3Args A) { pairs_body<true, true>(A); }

// ---------------------------------------------------------------------------
// k_color_h2: the colour branch 280 -> 128 -> 128 -> 128 (LeakyReLU each,
// point_aggregators.py:630-638) on the input [hid (K-summed features),
// PE_4(R.viewdir) sin block, cos block] (:506-512), as fp32-accurate f16-split
// GEMMs on the machinery of k_pairs_h2.  A 2-wave workgroup owns 64 valid
// samples; wave w owns output tiles {2w, 2w+1} for both 32-sample halves (the
// `layer` step: every weight fragment and every B fragment feeds two MFMAs).
// Layer inputs sit in split planes [2][18 row groups][64 samples][8 f16]
// (37 KB, four workgroups = two waves per SIMD per CU, so one workgroup's hid
// loads hide behind another's MFMAs): colour layer 1 runs as two 144-row halves
// (packs wc1a = columns 0..143, wc1b = columns 144..279 + bias), layers 2 and
// 3 as 128-row GEMMs from bias-initialised accumulators.
constexpr int kCG = 18;                       // 8-row groups per half (144 rows)
constexpr int kCPlane = kCG * kXT * 16;       // bytes per f16 plane
constexpr size_t kColH2Lds = 2 * (size_t)kCPlane;
constexpr int kOPitch = kC + 4;   // fp32 output staging pitch: 16-B rows, an accumulator quad is one b128 write
static_assert((size_t)kXT * kOPitch * 4 <= kColH2Lds, "output staging must fit the planes");

struct ColH2Args {
  pnr_samples s;
  pnr_mlp w;
  const void* pack[4];   // wc1a, wc1b, wc2, wc3 (frag_pack_h2, 4 neuron tiles per k-step)
  float scale[3];        // per-layer output factor 2^(s - 11)
  int32_t* range_flag;
  const float* hid;
  const int32_t* vmask;
  float* out_feat;
  const float* rw2c_pp;   // pnr_points.rw2c (per-point Rw2c) or NULL
  // training (k_color_h2<true>): hid as fp32 rows [n][256] (k_pairs_h2_train's),
  // and the saves of k_color<true>: vpe [n][24], hc1..hc3 [n][128] post-activation
  const float* hid_rows;
  float* vpe;
  float* hc[3];
};

// hid row groups [G0, G0 + NG) of the tile's 64 samples (both planes) ->
// plane groups 0..NG-1, by global_load_lds: no VGPR staging, no split work
// (k_pairs_h2 stored the planes).  Wave w copies plane w.
template <int G0, int NG>
__device__ __forceinline__ void color_load_hid(const ColH2Args& A, char* lds, int64_t tile) {
  const int lane = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const char* src = reinterpret_cast<const char*>(A.hid) + tile * kHidTile + lane * 16;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + pl * kHidPlane + (G0 + g) * kXT * 16),
        (__attribute__((address_space(3))) void*)(lds + pl * kCPlane + g * kXT * 16), 16, 0, 0);
  }
}

// training: hid row groups [G0, G0 + NG) of the tile's 64 samples from fp32 rows,
// split into the planes here (wave w: groups w, w + 2, ...; lane = sample;
// samples past n read as zeros)
template <int G0, int NG>
__device__ __forceinline__ void color_split_hid(const ColH2Args& A, char* lds, int64_t tile, int64_t n) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t v = tile * kXT + lane;
  const bool ok = v < n;
  const float4* src = reinterpret_cast<const float4*>(A.hid_rows + (ok ? v : 0) * kHid);
#pragma unroll
  for (int gg = 0; gg < (NG + 1) / 2; ++gg) {
    const int g = 2 * gg + wid;
    if (g >= NG) break;
    const float4 a = ok ? src[2 * (G0 + g)] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b = ok ? src[2 * (G0 + g) + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float g8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    store_group<true>(lds, kCPlane, g, lane, g8);
  }
}

// training saves: lrelu(scale acc) rows [v][128] of the tile's samples v < n
// (acc[2 pt + T]: sample 32 pt + c, neurons 32 (T0 + T) + 8 q + 4 h + i)
__device__ __forceinline__ void save_act_rows(const f32x16 (&acc)[4], float* dst, int64_t v0, int64_t n, float neg,
                                              float scale, int lane, int T0) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) {
    const int64_t v = v0 + 32 * pt + c;
    if (v >= n) continue;
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x16& a = acc[2 * pt + T];
        *reinterpret_cast<float4*>(dst + v * kC + 32 * (T0 + T) + 8 * q + 4 * h) =
            make_float4(lrelu(a[4 * q] * scale, neg), lrelu(a[4 * q + 1] * scale, neg),
                        lrelu(a[4 * q + 2] * scale, neg), lrelu(a[4 * q + 3] * scale, neg));
      }
  }
}

template <bool TR>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) k_color_h2(ColH2Args A) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int64_t n = eff_n(A.s);
  const int64_t ntiles = cdiv(n, kXT);
  const float neg = A.w.neg_slope;
  float Rw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
  const int T0 = 2 * wid;
  const int voff = (T0 * XL<true>::NPW * 64 + lane) * 16;
  const __amdgpu_buffer_rsrc_t r1a = rsrc(A.pack[0]), r1b = rsrc(A.pack[1]), r2 = rsrc(A.pack[2]),
                               r3 = rsrc(A.pack[3]);
  float chk = 0.f;   // 0 * (outputs): NaN once any output is not finite (see k_pairs_h2)
  WRing<true> wr;
  f32x16 acc[4];
  prime<true, 4>(wr, r1a, voff);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t v0 = tile * kXT;
    const uint64_t vm = __ballot(v0 + lane < n && A.vmask[v0 + lane] != 0);   // sample validity, one load
    // ---------------------------------------------------- layer 1, input rows 0..143 (hid)
    if constexpr (TR) color_split_hid<0, kCG>(A, lds, tile, n);
    else color_load_hid<0, kCG>(A, lds, tile);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x16){0.f};
    layer<true, 4>(acc, wr, r1a, voff, lds, kCPlane, 9, lane);
    prime<true, 4>(wr, r1b, voff);
    __syncthreads();
    // ---------------------------------------------------- rows 144..255 (hid), 256..279 (view PE), 280 (bias)
    if constexpr (TR) color_split_hid<kCG, 14>(A, lds, tile, n);
    else color_load_hid<kCG, 14>(A, lds, tile);
    if (wid == 0) {   // lane = sample: PE_4 of the rotated view direction (k_color's order)
      const int64_t v = v0 + lane;
      float vrot[3] = {0.f, 0.f, 0.f};
      if (v < n) {
        const int64_t row = sample_row(A.s, v);
        const int64_t drow = dir_row(A.s, row);
        const float vd[3] = {A.s.dirs[drow * 3], A.s.dirs[drow * 3 + 1], A.s.dirs[drow * 3 + 2]};
        mat3(Rw, vd, vrot);
        if (A.rw2c_pp) rot_point(A.rw2c_pp, slot0_point(A.s, row), vd, vrot);
      }
      float pe[32];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          float sn, cs;
          sincosf(vrot[ch] * (float)(1 << f), &sn, &cs);
          pe[4 * ch + f] = sn;
          pe[12 + 4 * ch + f] = cs;
        }
      if (TR && v < n) {   // vpe[v] = rows 256..279 (k_color<true>'s order)
#pragma unroll
        for (int i = 0; i < 24; ++i) A.vpe[v * 24 + i] = pe[i];
      }
      pe[24] = 1.f;
#pragma unroll
      for (int i = 25; i < 32; ++i) pe[i] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float g8[8] = {pe[8 * q], pe[8 * q + 1], pe[8 * q + 2], pe[8 * q + 3],
                             pe[8 * q + 4], pe[8 * q + 5], pe[8 * q + 6], pe[8 * q + 7]};
        store_group<true>(lds, kCPlane, 14 + q, lane, g8);
      }
    }
    __syncthreads();
    layer<true, 4>(acc, wr, r1b, voff, lds, kCPlane, 9, lane);
    prime<true, 4>(wr, r2, voff);
    __syncthreads();
    // ---------------------------------------------------- layer 2
    // (layers 2 and 3: accumulators start at bias / scale, as block1.2 / 3.2 in
    // k_pairs_h2: 8 k-steps, the packs' bias step and the bias input row unused)
    if (TR) save_act_rows(acc, A.hc[0], v0, n, neg, A.scale[0], lane, T0);
    store_act<true>(acc, lds, neg, A.scale[0], lane, T0, kCPlane);
    acc_init<true>(acc, A.w.bc2, 1.f / A.scale[1], lane, T0);
    __syncthreads();
    layer<true, 4>(acc, wr, r2, voff, lds, kCPlane, 8, lane);
    prime<true, 4>(wr, r3, voff);
    __syncthreads();
    // ---------------------------------------------------- layer 3
    if (TR) save_act_rows(acc, A.hc[1], v0, n, neg, A.scale[1], lane, T0);
    store_act<true>(acc, lds, neg, A.scale[1], lane, T0, kCPlane);
    acc_init<true>(acc, A.w.bc3, 1.f / A.scale[2], lane, T0);
    __syncthreads();
    layer<true, 4>(acc, wr, r3, voff, lds, kCPlane, 8, lane);
    prime<true, 4>(wr, r1a, voff);   // the next tile
    // out_feat[v, 1 + 32 (T0 + T) + row] (valid samples only; the others keep their zeros)
    const float sc3 = A.scale[2];
    if (TR) save_act_rows(acc, A.hc[2], v0, n, neg, sc3, lane, T0);
#pragma unroll
    for (int i = 0; i < 4; ++i)   // valid columns only: the others hold stale plane data
      if ((vm >> (32 * (i >> 1) + c)) & 1)
#pragma unroll
        for (int r = 0; r < 16; r += 2) chk = fmaf(0.f, acc[i][r] + acc[i][r + 1], chk);
    // staged through LDS (the planes are free once both waves' layer-3 reads are
    // done): one store then writes 64 consecutive channels of a row instead of
    // one float in each of 32 rows
    __syncthreads();
    float* Ob = reinterpret_cast<float*>(lds);   // [64][kOPitch] fp32
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // rows acc_row(4q .. 4q + 3, h): 4 consecutive neurons
          const f32x16& a = acc[2 * pt + T];
          *reinterpret_cast<float4*>(Ob + (32 * pt + c) * kOPitch + 32 * (T0 + T) + 8 * q + 4 * h) =
              make_float4(lrelu(a[4 * q] * sc3, neg), lrelu(a[4 * q + 1] * sc3, neg), lrelu(a[4 * q + 2] * sc3, neg),
                          lrelu(a[4 * q + 3] * sc3, neg));
        }
    __syncthreads();
    for (int r = wid; r < kXT; r += 2) {
      if (!((vm >> r) & 1)) continue;
      float* o = A.out_feat + (v0 + r) * (kC + 1) + 1;
      o[lane] = Ob[r * kOPitch + lane];
      o[64 + lane] = Ob[r * kOPitch + 64 + lane];
    }
    __syncthreads();   // the planes are rewritten by the next tile's loads
  }
  if (A.range_flag && chk != 0.f) atomicOr(A.range_flag, 1);   // non-finite output: see k_pairs_h2
}

// ---------------------------------------------------------------------------
// k_point_pre_h2: the per-point half of block1.0, P1[p] = W1[:, :224] .
// [emb_p, PE_3(emb_p)] + b1 (k_point_pre's split of the 284-input Linear,
// aggregate.hip), as an fp32-accurate f16-split GEMM on the `layer` machinery:
// a 4-wave workgroup owns 64 points (wave w: neuron tiles {2w, 2w+1} x both
// halves), inputs in split planes [2][30 row groups][64 points][8] (rows: emb
// 0..31, PE 32 + 6c + {sin, cos} x 3 bands (angle doubling as k_point_pre),
// bias row 224), 61 KB: two workgroups per CU.  P1 rows stay fp32.
constexpr int kPG1 = 30;                      // 8-row groups (240 rows = 15 k-steps)
constexpr int kP1Plane = kPG1 * kXT * 16;
constexpr size_t kP1H2Lds = 2 * (size_t)kP1Plane;

struct P1H2Args {
  pnr_points pts;
  const void* pack;     // W1[:, :224] + b1, frag_pack_h2
  float scale;
  int32_t* range_flag;
  float* p1;
  float* x1;            // training (optional): the input rows [emb, PE_3] [np][224] (pnr_agg_saved.x1)
};

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) k_point_pre_h2(P1H2Args A) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int64_t np = p1_rows(A.pts);   // P1 rows
  const int64_t ntiles = cdiv(np, kXT);
  const int T0 = 2 * wid;
  const int voff = (T0 * XL<true>::NPW * 64 + lane) * 16;
  const __amdgpu_buffer_rsrc_t rw = rsrc(A.pack);
  float chk = 0.f;   // 0 * outputs: NaN once one is not finite (an input beyond the f16 range)
  WRing<true> wr;
  f32x16 acc[4];
  prime<true>(wr, rw, voff);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // thread (point lane, channel block wid): emb channels 8 wid .. 8 wid + 7 and their PE
    {
      const int64_t pt = tile * kXT + lane;
      const bool act = pt < np;
      const int64_t prow = act ? (A.pts.used ? (int64_t)A.pts.used[pt] : pt) : 0;
      float e[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (act) {
        const float4 a = reinterpret_cast<const float4*>(A.pts.emb + prow * kEmb + 8 * wid)[0];
        const float4 b = reinterpret_cast<const float4*>(A.pts.emb + prow * kEmb + 8 * wid)[1];
        e[0] = a.x; e[1] = a.y; e[2] = a.z; e[3] = a.w; e[4] = b.x; e[5] = b.y; e[6] = b.z; e[7] = b.w;
      }
      store_group<true>(lds, kP1Plane, wid, lane, e);
      if (A.x1 && act) {   // training: this wave's emb channels of the input row
        float4* xr = reinterpret_cast<float4*>(A.x1 + pt * 224 + 8 * wid);
        xr[0] = make_float4(e[0], e[1], e[2], e[3]);
        xr[1] = make_float4(e[4], e[5], e[6], e[7]);
      }
      float pe[48];
#pragma unroll
      for (int u = 0; u < 8; ++u) {   // networks.py:175-190 order: rows 32 + 6c + {s0, c0, s1, c1, s2, c2}
        float s0, c0;
        sincosf(e[u], &s0, &c0);
        const float s1 = 2.f * s0 * c0, c1 = (c0 - s0) * (c0 + s0);
        const float s2 = 2.f * s1 * c1, c2 = (c1 - s1) * (c1 + s1);
        pe[6 * u] = s0; pe[6 * u + 1] = c0; pe[6 * u + 2] = s1;
        pe[6 * u + 3] = c1; pe[6 * u + 4] = s2; pe[6 * u + 5] = c2;
      }
#pragma unroll
      for (int g = 0; g < 6; ++g) {
        const float g8[8] = {pe[8 * g], pe[8 * g + 1], pe[8 * g + 2], pe[8 * g + 3],
                             pe[8 * g + 4], pe[8 * g + 5], pe[8 * g + 6], pe[8 * g + 7]};
        store_group<true>(lds, kP1Plane, 4 + 6 * wid + g, lane, g8);
      }
      if (A.x1 && act) {   // ... and their PE rows 32 + 48 wid .. + 47
        float4* xr = reinterpret_cast<float4*>(A.x1 + pt * 224 + 32 + 48 * wid);
#pragma unroll
        for (int q = 0; q < 12; ++q) xr[q] = make_float4(pe[4 * q], pe[4 * q + 1], pe[4 * q + 2], pe[4 * q + 3]);
      }
      if (wid == 0) {   // row 224 = 1 (bias column), 225..239 = 0
        const float one[8] = {1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const float zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        store_group<true>(lds, kP1Plane, 28, lane, one);
        store_group<true>(lds, kP1Plane, 29, lane, zero);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x16){0.f};
    layer<true>(acc, wr, rw, voff, lds, kP1Plane, 15, lane);
    prime<true>(wr, rw, voff);   // the next tile
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const int64_t prow = tile * kXT + 32 * pt + c;   // P1 row (index into used when set)
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x16& v = acc[2 * pt + T];
          const float4 o = make_float4(v[4 * q] * A.scale, v[4 * q + 1] * A.scale, v[4 * q + 2] * A.scale,
                                       v[4 * q + 3] * A.scale);
          chk = fmaf(0.f, (o.x + o.y) + (o.z + o.w), chk);
          if (prow < np)
            *reinterpret_cast<float4*>(A.p1 + prow * kHid + 32 * (T0 + T) + 8 * q + 4 * h) = o;
        }
    }
    __syncthreads();   // the planes are rewritten by the next tile
  }
  if (A.range_flag && chk != 0.f) atomicOr(A.range_flag, 1);
}

}  // namespace

int launch_point_pre_h2(const pnr_points& pts, const void* pack, float scale, int32_t* range_flag, float* p1,
                        hipStream_t st, float* x1) {
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_point_pre_h2),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kP1H2Lds));
    attr = true;
  }
  P1H2Args a;
  a.pts = pts;
  a.pack = pack;
  a.scale = scale;
  a.range_flag = range_flag;
  a.p1 = p1;
  a.x1 = x1;
  const int64_t np = pts.used ? pts.n_used : pts.n;
  hipLaunchKernelGGL(k_point_pre_h2, dim3(grid_for(cdiv(np, kXT), 1, 256 * 2)), dim3(256), kP1H2Lds, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

int launch_color_h2(const pnr_samples& s, const pnr_mlp& w, const void* const pack[4], const float scale[3],
                    int32_t* range_flag, const float* hid, const int32_t* vmask, float* out_feat, hipStream_t st,
                    const float* rw2c_pp, const pnr_agg_saved* train) {
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_color_h2<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kColH2Lds));
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_color_h2<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kColH2Lds));
    attr = true;
  }
  ColH2Args a;
  a.s = s;
  a.w = w;
  for (int i = 0; i < 4; ++i) a.pack[i] = pack[i];
  for (int i = 0; i < 3; ++i) a.scale[i] = scale[i];
  a.range_flag = range_flag;
  a.hid = hid;
  a.vmask = vmask;
  a.out_feat = out_feat;
  a.rw2c_pp = rw2c_pp;
  a.hid_rows = train ? train->hid : nullptr;
  a.vpe = train ? train->vpe : nullptr;
  a.hc[0] = train ? train->hc1 : nullptr;
  a.hc[1] = train ? train->hc2 : nullptr;
  a.hc[2] = train ? train->hc3 : nullptr;
  const dim3 grid(grid_for(cdiv(s.n_max, kXT), 1, 256 * 4));
  if (train) hipLaunchKernelGGL(k_color_h2<true>, grid, dim3(128), kColH2Lds, st, a);
  else hipLaunchKernelGGL(k_color_h2<false>, grid, dim3(128), kColH2Lds, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}


template <bool H>
int launch_pairs_split(const pnr_points& pts, const pnr_samples& s, const pnr_mlp& w, const SplitW& wx,
                       const float* p1, float* hid, int32_t* vmask, float* out_feat, float* out_weight,
                       float* out_conf, int32_t* tile_ctr, hipStream_t st, const pnr_agg_saved* sv) {
  const void* fn = H ? (sv ? reinterpret_cast<const void*>(&k_pairs_h2_train) : reinterpret_cast<const void*>(&k_pairs_h2))
                     : (sv ? reinterpret_cast<const void*>(&k_pairs_x3_train) : reinterpret_cast<const void*>(&k_pairs_x3));
  static bool attr[2] = {false, false};   // (per H instantiation)
  if (!attr[sv ? 1 : 0]) {
    PNR_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)XL<H>::Lds));
    attr[sv ? 1 : 0] = true;
  }
  X3Args a;
  a.pts = pts;
  a.s = s;
  a.w = w;
  a.wx = wx;
  a.p1 = p1;
  a.hid = hid;
  a.vmask = vmask;
  a.out_feat = out_feat;
  a.out_weight = out_weight;
  a.out_conf = out_conf;
  a.tile_ctr = tile_ctr;
  if (sv) a.sv = *sv;
  else memset(&a.sv, 0, sizeof(a.sv));
  PNR_HIP(hipMemsetAsync(tile_ctr, 0, 8 * sizeof(int32_t), st));
  const int64_t tiles = cdiv(s.n_max, kXTS);
  if (H && sv)
    hipLaunchKernelGGL(k_pairs_h2_train, dim3(grid_for(tiles, 1, 256)), dim3(512), XL<H>::Lds, st, a);
  else if (H)
    hipLaunchKernelGGL(k_pairs_h2, dim3(grid_for(tiles, 1, 256)), dim3(512), XL<H>::Lds, st, a);
  else if (sv)
    hipLaunchKernelGGL(k_pairs_x3_train, dim3(grid_for(tiles, 1, 256)), dim3(512), XL<H>::Lds, st, a);
  else
    hipLaunchKernelGGL(k_pairs_x3, dim3(grid_for(tiles, 1, 256)), dim3(512), XL<H>::Lds, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
template int launch_pairs_split<false>(const pnr_points&, const pnr_samples&, const pnr_mlp&, const SplitW&,
                                       const float*, float*, int32_t*, float*, float*, float*, int32_t*,
                                       hipStream_t, const pnr_agg_saved*);
template int launch_pairs_split<true>(const pnr_points&, const pnr_samples&, const pnr_mlp&, const SplitW&,
                                      const float*, float*, int32_t*, float*, float*, float*, int32_t*,
                                      hipStream_t, const pnr_agg_saved*);

}  // namespace pnr
