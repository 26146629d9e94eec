// k_pairs_as: the pairs stage of pnr_aggregate_fwd_h2 (block1.0's distance
// half, block1.2, block3.0, block3.2, the alpha branch and the K-weighted sum of
// point_aggregators.py:488-646 for every (sample, neighbour) pair), as fp32-
// accurate f16-split GEMMs on v_mfma_f32_32x32x16_f16 -- ACTIVATION-STATIONARY.
//
// One 4-wave workgroup per CU (one wave per SIMD, up to 512 registers).  Each
// wave owns a wave tile of 32 pairs (4 samples x K 8) and carries it through
// all four layers itself: every layer's 256 outputs of its 32 pairs stay in
// the wave's accumulators (8 neuron tiles x f32x16 = 128 registers), and the
// next layer's B operand is made from them in registers, one 16-row k-step at
// a time: with 32x32x16 MFMAs lane (c, h) holds rows 8q + 4h + i of every
// neuron tile, and the B fragment of a k-step wants 8 consecutive k-rows per
// lane half -- so the k-rows of each step are the accumulator's own rows
// (the weight packs permute their input columns to match), and no activation
// ever goes through LDS.  Two accumulator sets alternate between layers
// (L1 -> X, L2 -> Y, L3 -> X, L4 -> Y), so the conversion of one layer's
// output (lrelu + f16 split, 4 VALU per value) runs in the MFMA gaps of the
// next layer instead of in a serial phase.
//
// The weights stream through LDS, shared by the four waves (they run the
// same 53 k-steps per tile in lockstep): a ring of 3 k-step slots of 24 KB
// (planes Ws = 2^11 Wh, Wl, Wk = k Wh x 8 neuron tiles x 64 lanes x 16 B),
// each wave copying a quarter of the step after next (6 x 1 KB, loaded one
// step ahead into registers), one barrier per k-step.
//
// Split arithmetic (agg_common.h splith): an input x = xh + 2^-11 xl; for
// layer L >= 2 the input is lrelu(z) of the previous layer, whose accumulator
// holds z / sc (sc = 2^(s - 11), s >= 0 the pack shift), and the split is
// taken from L = lrelu(acc) directly: xh = f16(L sc), xl' = f16(L - xh / sc)
// = xl / k with k = 2^11 sc >= 1, which the Wk plane (k Wh) undoes -- one
// fma_mix each, no rescaling of L.  The products per k-step and neuron tile:
// Ws.Xh + Wl.Xh + Wk.Xl' (the dropped Wl.Xl term is <= 2^-22 |w x|).
//
// Per wave tile and layer (53 k-steps, 24 MFMAs each) the other work runs in
// the MFMA gaps of fixed steps:
//   L1 (4 steps, X = P1/sc1 + W1b.PE5)  the previous tile's tail on Y: lrelu,
//                                       alpha dot, K-weighted sums (DPP
//                                       reduce-scatter over a sample's 8
//                                       lanes), hid / alpha / vmask stores
//   L2 (16, Y = b2' + W2.X)             gather of the next tile (sample row,
//                                       neighbour ids, point rows, 6-d
//                                       distance, weights, block3.0 extras)
//   L3 (17, X = W3.[Y; extras])         PE5 of the next tile (15 sincosf)
//   L4 (16, Y = b4' + W4.X)             P1 rows of the next tile loaded
//                                       straight into X as its tiles free up
#include <utility>

#include "agg_common.h"

namespace pnr {
namespace {

constexpr int kWT = 32;                        // pairs per wave tile (4 samples x K 8)
constexpr int kWS = kWT / kKN;                 // samples per wave tile
constexpr int kBS = 4 * kWS;                   // samples per workgroup block
constexpr int kL1 = 4, kL2 = 16, kL3 = 17, kL4 = 16;
constexpr int kTileSteps = kL1 + kL2 + kL3 + kL4;   // 53
constexpr int kStepBytes = 3 * 8 * 64 * 16;         // 24 KB per k-step (3 planes x 8 tiles x 64 lanes x 16 B)
constexpr int kRing = 4;                        // k-step slots: read, next, landing, issued
constexpr int kHidPlane = 32 * 64 * 16;        // k_color_h2's input layout (aggregate_x3.hip)
constexpr int kHidTile = 2 * kHidPlane;
// LDS
// (the small, often-read tables first: ds_read/ds_write immediate offsets reach
// 64 KB, so their addresses fold into the instructions instead of VGPRs)
constexpr int OffTab = 0;                      // float [3][2 h][128]: b2', b4', wa' in accumulator order
constexpr int OffQ = OffTab + 3 * 2 * 128 * 4; // int [4] next block
constexpr int OffEx = OffQ + 16;               // per tile parity, wave [2 planes][64 lanes][16 B]: block3.0 extras
constexpr int OffPE = OffEx + 2 * 4 * 2 * 64 * 16;   // per wave [2 planes][4 steps][64 lanes][16 B]: the next tile's PE5
constexpr int OffRing = OffPE + 4 * 2 * 4 * 64 * 16; // kRing k-step slots of kStepBytes
constexpr size_t kAsLds = OffRing + kRing * kStepBytes;
static_assert(kAsLds <= 160 * 1024, "LDS budget");

struct AsArgs {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp w;
  const char* pack;    // [53 steps][3 planes][8 tiles][64 lanes][8 f16]
  const float* tabs;   // [3][2][128]: b2 / sc2, b4 / sc4, wa, each in accumulator order
  float sc1, sc2, sc3, sc4;   // layer output factors 2^(s - 11)
  float inv_k3;        // 1 / k3 = 1 / (2^11 sc2): low half of the block3.0 extras
  const float* p1;     // [N][256] block1.0 point half / sc1
  float* hid;
  int32_t* vmask;
  float* out_feat;
  int32_t* blk_ctr;    // [8] zeroed per launch (XCD groups)
  int32_t* range_flag;
  const uint4* rec;    // pair records [kRecPlanes][rec_stride] (k_pair_rec)
  int64_t rec_stride;
};

// Pair records, one 16-B entry per (sample, neighbour) pair in each of 4
// planes of as_rec_stride entries (agg_common.h), written by k_pair_rec and read once per wave tile by
// k_pairs_as (pair = sample * 8 + neighbour):
//   plane 0  {P1 row | sflag << 31, wt = normalised weight x clamped conf, d6[3], d6[4]}
//   plane 1  {(R.(p_w - s_w))[0..2], d6[5]}       the 6-d distance (lane half 0 | 1 channels)
//   plane 2  block3.0 extras, f16 high parts (8 x f16)
//   plane 3  block3.0 extras, f16 low parts / k3

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// ------------------------------------------------------------- block schedule
// XCD-aware dynamic blocks as k_pairs_h2's take_tile: block group b % 8 (the
// blocks sharing an XCD) walks its own contiguous eighth of the blocks, then
// helps the others; neighbouring blocks share most of their P1 rows (L2 reuse).
__device__ __forceinline__ bool xcd_mode(int64_t nb) { return nb >= 2 * (int64_t)gridDim.x + 16; }
__device__ __forceinline__ int64_t xcd_lo(int64_t nb, int x) { return nb * x / 8; }
__device__ __forceinline__ int64_t xcd_nb(int x) { return ((int)gridDim.x - x + 7) / 8; }
__device__ __forceinline__ int64_t first_block(int64_t nb) {
  if (!xcd_mode(nb)) return blockIdx.x;
  return xcd_lo(nb, blockIdx.x & 7) + (blockIdx.x >> 3);
}
__device__ __forceinline__ int64_t take_block(int32_t* ctr, int64_t nb) {
  if (!xcd_mode(nb)) return (int64_t)gridDim.x + atomicAdd(ctr, 1);
  const int x0 = blockIdx.x & 7;
  for (int i = 0; i < 8; ++i) {
    const int x = (x0 + i) & 7;
    const int64_t t = xcd_lo(nb, x) + xcd_nb(x) + atomicAdd(ctr + x, 1);
    if (t < xcd_lo(nb, x + 1)) return t;
  }
  return nb;
}

// ------------------------------------------------------------- split helpers
// (x0, x1) -> L = lrelu(x) = max(x, s x) (0 <= s <= 1), then the f16 pair
// hi = f16(L m), lo = f16(L - hi / m)  (m = sc, nim = -1 / sc): one v_fma_mix each
// (exact product, one rounding), written as fma + casts so the compiler sees (and
// interleaves) plain VALU instructions.
// 0 <= s <= 1: max(x, s x).  v_max_f32 by hand: fmaxf would first quiet x
// (IEEE mode), one more VALU op per value; x is never a signalling NaN here.
__device__ __forceinline__ float lrelu_s(float x, float s) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(x * s));
  return r;
}

__device__ __forceinline__ void lrelu_mixsplit(float x0, float x1, float s, float m, float nim, unsigned& hi,
                                               unsigned& lo) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const float l0 = lrelu_s(x0, s), l1 = lrelu_s(x1, s);
  const _Float16 h0 = (_Float16)__builtin_fmaf(l0, m, 0.f), h1 = (_Float16)__builtin_fmaf(l1, m, 0.f);
  const _Float16 q0 = (_Float16)__builtin_fmaf((float)h0, nim, l0);
  const _Float16 q1 = (_Float16)__builtin_fmaf((float)h1, nim, l1);
  const h2 H = {h0, h1}, Q = {q0, q1};
  hi = __builtin_bit_cast(unsigned, H);
  lo = __builtin_bit_cast(unsigned, Q);
}

// B fragment of a k-step from accumulator tile `a`, half u: the 8 values
// r = 8u .. 8u + 7 of this lane (k-rows 8h .. 8h + 7 of the step)
__device__ __forceinline__ void conv8(const f32x16& a, int u, float slope, float m, float nim, uint4& xh, uint4& xl) {
  unsigned hh[4], ll[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) lrelu_mixsplit(a[8 * u + 2 * p], a[8 * u + 2 * p + 1], slope, m, nim, hh[p], ll[p]);
  xh = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  xl = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// ------------------------------------------------------------- per-wave state
struct Next {         // gather results of the next wave tile (this lane's pair)
  int v;              // sample index
  int prow;           // P1 / point row (clamped neighbour id)
  bool act;           // sample exists
  float wt;           // normalised weight x clamped conf
  int sflag;          // the sample has a neighbour
  float d3[3];        // this lane half's 3 distance channels (h 0: R.(p_w - s_w), h 1: camera deltas)
};

struct Cur {          // the tile whose tail is pending
  int v;
  float wt;
  int sflag;
  bool act;
};

template <int CTRL>
__device__ __forceinline__ float dpp_c(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

// block3.0 extras -> B fragment of L3's last k-step (lane half 0 holds rows 256..263)
__device__ __forceinline__ void extras_b(const float (&ex)[8], float inv_k3, uint4& xh, uint4& xl) {
  unsigned hh[4], ll[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    unsigned a, b;
    splith(ex[2 * p], ex[2 * p + 1], a, b);   // lo = f16((x - xh) 2^11)
    hh[p] = a;
    // xl' = xl / k3 (the Wk plane carries k3 Wh): exact power-of-two rescale
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 x = {ex[2 * p], ex[2 * p + 1]};
    const f2 hf = __builtin_convertvector(__builtin_bit_cast(h2, a), f2);
    const f2 r = (x - hf) * (2048.f * inv_k3);
    ll[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, h2));
    (void)b;
  }
  xh = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  xl = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// gather of one (sample, neighbour) pair (neural_points.py:788-799,
// point_aggregators.py:421-429, 775-804), one thread per pair, 8 consecutive
// lanes = one sample's K slots -> its record (k_pair_rec).
struct RecArgs {
  pnr_points pts;
  pnr_samples s;
  pnr_mlp w;
  float inv_k3;
  uint4* rec;
  int64_t rec_stride;
  float* out_weight;
  float* out_conf;
};

__global__ void __launch_bounds__(256) k_pair_rec(RecArgs A) {
  const int64_t n = eff_n(A.s);
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t v = gid >> 3;
  const int k = (int)(gid & 7), K = A.s.K;
  if (v >= n) return;   // whole 8-lane groups (xor8_sum stays within a sample)
  const int64_t row = sample_row(A.s, v);
  const int pid = k < K ? A.s.pidx[row * K + k] : -1;
  float sw[3], sp[3], vd[3], pw3[3] = {0.f, 0.f, 0.f}, pp[3] = {0.f, 0.f, 0.f}, col[3] = {0.f, 0.f, 0.f},
        pdir[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    sw[a] = A.s.sample_w[row * 3 + a];
    sp[a] = A.s.sample_p[row * 3 + a];
  }
  const int64_t drow = dir_row(A.s, row);
#pragma unroll
  for (int a = 0; a < 3; ++a) vd[a] = A.s.dirs[drow * 3 + a];
  const bool valid = pid >= 0;
  const int64_t prow = valid ? pid : 0;   // torch.clamp(sample_pidx, min=0)
  if (valid) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      pw3[a] = A.pts.xyz[prow * 3 + a];
      col[a] = A.pts.color ? A.pts.color[prow * 3 + a] : 0.f;
      pdir[a] = A.pts.dir ? A.pts.dir[prow * 3 + a] : 0.f;
      if (A.pts.pers) pp[a] = A.pts.pers[prow * 3 + a];
    }
  }
  const float cf = (A.pts.conf && k < K) ? A.pts.conf[prow] : 1.f;
  // P1 row (the used-row index when P1 covers the referenced points only); an
  // empty slot takes row 0, finite and weighted 0
  const int p1row = (valid && A.pts.used_map) ? A.pts.used_map[prow] : (int)prow;
  float Rw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rw[i] = A.w.rw2c ? A.w.rw2c[i] : (i % 4 == 0 ? 1.f : 0.f);
  if (valid && !A.pts.pers) {
    float cam_c[3], cam_R[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) cam_c[i] = A.pts.campos[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) cam_R[i] = A.pts.camrot[i];
    pair_pers(A.pts, A.s, drow, pw3, cam_c, cam_R, pp);
  }
  float d6[6];
  d6[0] = pw3[0] - sw[0];
  d6[1] = pw3[1] - sw[1];
  d6[2] = pw3[2] - sw[2];
  d6[3] = pp[0] * pp[2] - sp[0] * sp[2];
  d6[4] = pp[1] * pp[2] - sp[1] * sp[2];
  d6[5] = pp[2] - sp[2];
  float dr[3];
  mat3(Rw, d6, dr);
  const float nrm = sqrtf(d6[0] * d6[0] + d6[1] * d6[1] + d6[2] * d6[2]);
  const float wl = valid ? 1.f / fmaxf(nrm, 1e-6f) : 0.f;
  const float wsum = xor8_sum(wl);
  const float wn = wl / fmaxf(wsum, 1e-8f);
  const float confc = fminf(fmaxf(cf, 1e-4f), 1.f);
  const float wt = wn * confc;
  const bool sflag = xor8_sum(valid ? 1.f : 0.f) > 0.f;
  float vrot[3], drot[3];
  mat3(Rw, vd, vrot);
  mat3(Rw, pdir, drot);
  const float dot = drot[0] * vrot[0] + drot[1] * vrot[1] + drot[2] * vrot[2];
  const float ex[8] = {col[0], col[1], col[2], drot[0] - vrot[0], drot[1] - vrot[1], drot[2] - vrot[2], dot, 1.f};
  uint4 xh, xl;
  extras_b(ex, A.inv_k3, xh, xl);
  const int64_t pr = v * 8 + k;
  uint4* R = A.rec;
  R[pr] = make_uint4((unsigned)p1row | (sflag ? 0x80000000u : 0u), __float_as_uint(wt), __float_as_uint(d6[3]),
                     __float_as_uint(d6[4]));
  R[A.rec_stride + pr] = make_uint4(__float_as_uint(dr[0]), __float_as_uint(dr[1]), __float_as_uint(dr[2]),
                                    __float_as_uint(d6[5]));
  R[2 * A.rec_stride + pr] = xh;
  R[3 * A.rec_stride + pr] = xl;
  if (k < K) {
    if (A.out_weight) A.out_weight[row * K + k] = wn;
    if (A.out_conf) A.out_conf[row * K + k] = confc;
  }
}

// a wave tile's records: lane (c, h) = pair c of the tile, lane half h
struct Rec {
  uint4 a, b, xh, xl;
};
// (a tile past the last block -- the drain tile, or a block index past nblk
// from take_block -- reads tile 0's records, which rec_take then ignores)
__device__ __forceinline__ void rec_load(const AsArgs& A, int64_t wtile, int64_t nblk, int lane, Rec& r) {
  const int64_t pr = (wtile < nblk * 4 ? wtile : 0) * kWT + (lane & 31);
  r.a = A.rec[pr];
  r.b = A.rec[A.rec_stride + pr];
  r.xh = A.rec[2 * A.rec_stride + pr];
  r.xl = A.rec[3 * A.rec_stride + pr];
}
// records -> the next tile's state; the extras' B fragment (lane half 0 holds
// rows 256..263 of block3.0's input) -> ex_lds.  Samples past n: every value
// zero (their lanes' results are never stored, and stay finite).
__device__ __forceinline__ void rec_take(const Rec& r, int64_t wtile, int64_t n, int lane, Next& g, char* ex_lds) {
  const int c = lane & 31, h = lane >> 5;
  const int64_t v = wtile * kWS + (c >> 3);
  g.v = (int)v;
  g.act = v < n;
  g.prow = g.act ? (int)(r.a.x & 0x7fffffffu) : 0;
  g.sflag = (g.act && (r.a.x >> 31)) ? 1 : 0;
  g.wt = g.act ? __uint_as_float(r.a.y) : 0.f;
  const unsigned d0 = h ? r.a.z : r.b.x, d1 = h ? r.a.w : r.b.y, d2 = h ? r.b.w : r.b.z;
  g.d3[0] = g.act ? __uint_as_float(d0) : 0.f;
  g.d3[1] = g.act ? __uint_as_float(d1) : 0.f;
  g.d3[2] = g.act ? __uint_as_float(d2) : 0.f;
  const bool ex_on = g.act && h == 0;
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  uint4* d = reinterpret_cast<uint4*>(ex_lds) + lane;
  d[0] = ex_on ? r.xh : z;
  d[64] = ex_on ? r.xl : z;
}

// 16 P1 values of neuron tile T (rows 32T + 8q + 4h + i) into accumulator a
__device__ __forceinline__ void load_p1(const AsArgs& A, int prow, int h, int T, f32x16& a) {
  const float4* src = reinterpret_cast<const float4*>(A.p1 + (int64_t)prow * kHid + 32 * T + 4 * h);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = src[2 * q];
    a[4 * q] = v.x;
    a[4 * q + 1] = v.y;
    a[4 * q + 2] = v.z;
    a[4 * q + 3] = v.w;
  }
}

// bias start of an accumulator set (b / sc in accumulator order, from LDS)
__device__ __forceinline__ void init_bias(f32x16 (&acc)[8], const char* lds, int tab, int h) {
  const float4* b = reinterpret_cast<const float4*>(lds + OffTab + (tab * 2 + h) * 128 * 4);
#pragma unroll
  for (int T = 0; T < 8; ++T)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = b[4 * T + q];
      acc[T][4 * q] = v.x;
      acc[T][4 * q + 1] = v.y;
      acc[T][4 * q + 2] = v.z;
      acc[T][4 * q + 3] = v.w;
    }
}

// ------------------------------------------------------------- weight stream
struct Stream {
  int g;              // global k-step
  const char* pack;   // the wave's 6 KB quarter of pack step 0 (wave-uniform)
  unsigned lane_off;  // this lane's 16 B in a 1 KB piece
  unsigned ring;      // LDS byte address of this wave's quarter of ring slot 0
};

// Ring fill by LDS-DMA: wave w copies 1 KB piece i of its quarter of pack step
// `step` straight into ring slot `slot` (global_load_lds_dwordx4: LDS address
// = M0 + 16 lane).  Inline asm, so hipcc's vmcnt bookkeeping never waits on it;
// step_barrier() counts these loads itself.
// 4 (G 0) or 2 (G 1) of the wave's 6 pieces under one M0: the instruction
// offset moves the global and the LDS address alike.
template <int G>
__device__ __forceinline__ void stream_dma_group(const Stream& S, int step, int slot) {
  // the step's base in SGPRs, opaque to hipcc: otherwise it hoists all the
  // per-step addresses of a tile out of the loop (and spills them)
  unsigned off = step * kStepBytes + G * 4096;
  asm volatile("" : "+s"(off));
  const char* base = S.pack + off;
  const unsigned dst = S.ring + slot * kStepBytes + G * 4096;
  unsigned keep;
  if constexpr (G == 0)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\tglobal_load_lds_dwordx4 %1, %2 offset:1024\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:2048\n\tglobal_load_lds_dwordx4 %1, %2 offset:3072\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(S.lane_off), "s"(base), "s"(dst)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\tglobal_load_lds_dwordx4 %1, %2 offset:1024\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(S.lane_off), "s"(base), "s"(dst)
        : "memory");
}

constexpr int kFragRegs = 6;    // A fragment registers (24 divides by it: the rotation restarts every step)
constexpr int kFragDist = 3;    // A fragments in flight ahead of the MFMA stream
struct Frag {
  uint4 w[kFragRegs];   // the next kFragRegs slots' A fragments
};
__device__ __forceinline__ uint4 read_plane(const char* lds, int slot, int T, int p, int lane) {
  return reinterpret_cast<const uint4*>(lds + OffRing + slot * kStepBytes)[(p * 8 + T) * 64 + lane];
}

// Barrier of a k-step: the ring DMA issued one step earlier has landed (the 6
// of this step stay in flight: vmcnt counts in order, so this also retires any
// older load), every LDS op but the youngest kFragDist (the next step's
// first fragment reads, which stay in flight across it) completed, s_barrier.
__device__ __forceinline__ void step_barrier() {
  asm volatile("s_waitcnt vmcnt(6) lgkmcnt(%0)" ::"n"(kFragDist) : "memory");
  __builtin_amdgcn_s_barrier();
}

// One k-step as 24 MFMA slots in a fixed order (sched_barrier fences): slot i
// issues MFMA i (neuron tile T = i / 3, product p = i % 3: Ws.Xh, Wl.Xh,
// Wk.Xl'), refills fragment register p with the next tile's plane p (for tile 7:
// the next step's tile 0, whose slot the previous barrier published), then that
// slot's share of the other work -- the ring copy (slots 0-5: LDS writes of the
// step after next, 6-11: buffer loads of the one after) and `work(i)` (the
// layer's conversion pieces and extra work) -- so every MFMA gap carries a few
// VALU / memory instructions.  work must issue no LDS write in slots 21-23.
template <typename W>
__device__ __forceinline__ void kstep(char* lds, Stream& S, int wid, int lane, f32x16 (&acc)[8], const uint4& xh,
                                      const uint4& xl, Frag& fr, W&& work) {
  const int slot = S.g % kRing, nslot = (S.g + 1) % kRing, dslot = (S.g + 3) % kRing;
  const int lstep = (S.g + 3) % kTileSteps;
  static_for<0, 24>([&](auto ii) {
    // product-major order: the 8 neuron tiles' MFMAs of one product stand
    // between two dependent MFMAs (same accumulator), so none waits on the
    // previous one's result
    constexpr int i = decltype(ii)::value, p = i / 8, T = i % 8;
    // slot j's fragment goes to register j % kFragRegs, kFragDist slots ahead:
    // that register last fed the MFMA kFragRegs - kFragDist slots back (no
    // load overwrites an operand of the MFMA just issued)
    constexpr int j = i + kFragDist, r = j % kFragRegs;
    acc[T] = mfma_f16(fr.w[i % kFragRegs], p == 2 ? xl : xh, acc[T]);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (i < 2) stream_dma_group<i>(S, lstep, dslot);
    work(ii);
    fr.w[r] = j < 24 ? read_plane(lds, slot, j % 8, j / 8, lane) : read_plane(lds, nslot, (j - 24) % 8, (j - 24) / 8, lane);
    __builtin_amdgcn_sched_barrier(0);
  });
  step_barrier();
  ++S.g;
}

// The next step's B fragment from accumulator tile `a`, half u, in pieces:
// slot 2j lrelu of value j (j < 8), slot 4q + 3 the f16 split of values 2q, 2q + 1.
struct Conv {
  float l[8];
  unsigned hh[4], ll[4];
};
template <int I>
__device__ __forceinline__ void conv_piece(const f32x16& a, int u, float slope, float m, float nim, Conv& cv) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  if constexpr (I < 16 && (I & 1) == 0) cv.l[I / 2] = lrelu_s(a[8 * u + I / 2], slope);
  if constexpr (I < 16 && (I & 3) == 3) {
    constexpr int q = I / 4;
    const float l0 = cv.l[2 * q], l1 = cv.l[2 * q + 1];
    const _Float16 h0 = (_Float16)__builtin_fmaf(l0, m, 0.f), h1 = (_Float16)__builtin_fmaf(l1, m, 0.f);
    const _Float16 q0 = (_Float16)__builtin_fmaf((float)h0, nim, l0);
    const _Float16 q1 = (_Float16)__builtin_fmaf((float)h1, nim, l1);
    const h2 H = {h0, h1}, Q = {q0, q1};
    cv.hh[q] = __builtin_bit_cast(unsigned, H);
    cv.ll[q] = __builtin_bit_cast(unsigned, Q);
  }
}

// ------------------------------------------------------------- the tail
// K-weighted sum (point_aggregators.py:622-628) and alpha (:608-614) of the tile
// whose block3.2 accumulators are in Y, spread over the 4 k-steps of the next
// tile's block1.0 (24 slots each): step 0 / 1 = neuron tiles 0..3 / 4..7:
// Y = wt lrelu(Y) in place and the alpha dot, one register quad per slot;
// step 2: reduce-scatter round 1 over lane bit 2; step 3: rounds 2 and 3, then
// the stores.  Lane (c, h) ends with the 16 sums of neuron tile T = c & 7 (rows
// 32T + 8q + 4h + i) of its sample.
template <int STEP, int I>
__device__ __forceinline__ void tail_piece(const AsArgs& A, const char* lds, f32x16 (&Y)[8], const Cur& cur, int lane,
                                           float slope, float& pa, float& chk) {
  const int c = lane & 31, h = lane >> 5, i8 = c & 7;
  if constexpr (STEP <= 1 && I < 16) {
    constexpr int T = 4 * STEP + I / 4, q = I % 4;
    if constexpr (STEP == 0 && I == 0) pa = 0.f;
    const float4 w4 = reinterpret_cast<const float4*>(lds + OffTab + (2 * 2 + h) * 128 * 4)[4 * T + q];
    const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float L = lrelu_s(Y[T][4 * q + i], slope);
      pa = fmaf(wv[i], L, pa);
      Y[T][4 * q + i] = cur.wt * L;
    }
  } else if constexpr (STEP == 2 && I < 16) {
    // round 1 (row_half_mirror: i8 <-> 7 - i8): keep tiles 4 b2 .. 4 b2 + 3; slot I: tile I / 4, registers 4 (I % 4) ..
    constexpr int T = I / 4, r0 = 4 * (I % 4);
    const bool b2 = (i8 & 4) != 0;
#pragma unroll
    for (int r = r0; r < r0 + 4; ++r) {
      const float keep = b2 ? Y[T + 4][r] : Y[T][r];
      const float send = b2 ? Y[T][r] : Y[T + 4][r];
      Y[T][r] = keep + dpp_c<0x141>(send);
    }
  } else if constexpr (STEP == 3 && I < 8) {
    // round 2 (quad_perm [2,3,0,1]: lane ^ 2): slot I: tile I / 4, registers 4 (I % 4) ..
    constexpr int T = I / 4, r0 = 4 * (I % 4);
    const bool b1 = (i8 & 2) != 0;
#pragma unroll
    for (int r = r0; r < r0 + 4; ++r) {
      const float keep = b1 ? Y[T + 2][r] : Y[T][r];
      const float send = b1 ? Y[T][r] : Y[T + 2][r];
      Y[T][r] = keep + dpp_c<0x4E>(send);
    }
  } else if constexpr (STEP == 3 && I >= 8 && I < 12) {
    // round 3 (quad_perm [1,0,3,2]: lane ^ 1)
    constexpr int r0 = 4 * (I - 8);
    const bool b0 = (i8 & 1) != 0;
#pragma unroll
    for (int r = r0; r < r0 + 4; ++r) {
      const float keep = b0 ? Y[1][r] : Y[0][r];
      const float send = b0 ? Y[0][r] : Y[1][r];
      Y[0][r] = keep + dpp_c<0xB1>(send);
    }
  } else if constexpr (STEP == 3 && I == 12) {
    // alpha: the two lane halves hold the two 128-row halves of the dot
    const float pk = (pa + __shfl_xor(pa, 32)) * A.sc4 + A.w.ba[0];
    const float alpha_k = A.w.act_super ? softplus(pk - 1.f) : fmaxf(pk, 0.f);
    pa = xor8_sum(cur.wt * alpha_k);   // pa now holds the sample's alpha
  } else if constexpr (STEP == 3 && I >= 13 && I < 17) {
    // hid rows 32 i8 + 8q + 4h .. +3 -> row group 4 i8 + q, bytes 8h .. 8h + 7 of its 16-B piece
    constexpr int q = I - 13;
    const float h0 = Y[0][4 * q] * A.sc4, h1 = Y[0][4 * q + 1] * A.sc4, h2v = Y[0][4 * q + 2] * A.sc4,
                h3 = Y[0][4 * q + 3] * A.sc4;
    chk = fmaf(0.f, (h0 + h1) + (h2v + h3), chk);   // NaN once an output is not finite (f16-range overflow)
    if (cur.act && cur.sflag) {
      unsigned a0, a1, b0, b1;
      splith(h0, h1, a0, a1);
      splith(h2v, h3, b0, b1);
      char* d = reinterpret_cast<char*>(A.hid) + (int64_t)(cur.v / 64) * kHidTile + (cur.v % 64) * 16 + 8 * h +
                (4 * i8 + q) * 64 * 16;
      *reinterpret_cast<uint2*>(d) = make_uint2(a0, b0);
      *reinterpret_cast<uint2*>(d + kHidPlane) = make_uint2(a1, b1);
    }
  } else if constexpr (STEP == 3 && I == 17) {
    chk = fmaf(0.f, pa, chk);
    if (cur.act && i8 == 0 && h == 0) {
      A.vmask[cur.v] = cur.sflag;
      if (cur.sflag) A.out_feat[(int64_t)cur.v * (kC + 1)] = pa;
    }
  }
}

template <int STEP>
__device__ __forceinline__ void tail_step(const AsArgs& A, const char* lds, f32x16 (&Y)[8], const Cur& cur, int lane,
                                          float slope, float& pa, float& chk) {
  static_for<0, 24>([&](auto ii) { tail_piece<STEP, decltype(ii)::value>(A, lds, Y, cur, lane, slope, pa, chk); });
}

// ------------------------------------------------------------- PE
// value e of this lane half (e < 30): channel 3h + e / 10, band (e % 10) / 2,
// sin (e even) / cos (e odd) -- W1 column 224 + 30h + e (networks.py:175-190 order)
// sin / cos of |x| <= 3000: Cody-Waite reduction by a 3-part pi/2 (12 + 12 +
// 24 bits: k C1 and k C2 exact for k < 2^12) and the cephes minimax polynomials
// on |r| <= pi/4 -- <= 1.6 ulp (9.3e-8 absolute) against the exact values,
// measured over 2M random arguments per decade up to 3000; larger arguments take
// sincosf.  A third of sincosf's VALU cost on the MFMA stream.
__device__ __forceinline__ void sincos_pe(float x, float& sn, float& cs) {
  if (__builtin_expect(fabsf(x) > 3000.f, 0)) {
    sincosf(x, &sn, &cs);
    return;
  }
  const float k = rintf(x * 0.636619772367581343f);
  float r = x - k * 1.5703125f;
  r = r - k * 4.837512969970703125e-4f;
  r = r - k * 7.549789954891837e-8f;
  const float z = r * r;
  const float s = r + r * z * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
  const float c = 1.f - 0.5f * z + z * z * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
  const int q = (int)k & 3;
  const float s1 = (q & 1) ? c : s, c1 = (q & 1) ? s : c;
  sn = (q & 2) ? -s1 : s1;
  cs = ((q + 1) & 2) ? -c1 : c1;
}

template <int E2>   // one (sin, cos) pair: values 2 E2, 2 E2 + 1 -> k-step E2 / 4, f16 pair E2 % 4
__device__ __forceinline__ void pe_pair(const float (&d3)[3], char* pe_lds, int lane) {
  constexpr int ch = (2 * E2) / 10, f = ((2 * E2) % 10) / 2;
  float sn, cs;
  sincos_pe(d3[ch] * (float)(1 << f), sn, cs);
  unsigned hi, lo;
  splith(sn, cs, hi, lo);
  unsigned* d = reinterpret_cast<unsigned*>(pe_lds + ((E2 / 4) * 64 + lane) * 16) + (E2 % 4);
  d[0] = hi;
  d[4 * 64 * 4] = lo;   // plane 1: + 4 steps x 64 lanes x 16 B
}

// the last pair (values 30, 31) of lane half h is zero padding (W1 columns none)
__device__ __forceinline__ void pe_pad(char* pe_lds, int lane) {
  unsigned* d = reinterpret_cast<unsigned*>(pe_lds + (3 * 64 + lane) * 16) + 3;
  d[0] = 0u;
  d[4 * 64 * 4] = 0u;
}

__device__ __forceinline__ void pe_read(const char* pe_lds, int t, int lane, uint4& xh, uint4& xl) {
  const uint4* src = reinterpret_cast<const uint4*>(pe_lds) + t * 64 + lane;
  xh = src[0];
  xl = src[4 * 64];
}

// block3.0 extras of this wave's tile: planes [2][64 lanes][16 B] (gather_s3)
__device__ __forceinline__ void ex_read(const char* ex_lds, int lane, uint4& xh, uint4& xl) {
  const uint4* src = reinterpret_cast<const uint4*>(ex_lds) + lane;
  xh = src[0];
  xl = src[64];
}

__device__ __forceinline__ void load_p1_q(const AsArgs& A, int prow, int h, int T, int q, f32x16& a) {
  const float4 v = reinterpret_cast<const float4*>(A.p1 + (int64_t)prow * kHid + 32 * T + 4 * h)[2 * q];
  a[4 * q] = v.x;
  a[4 * q + 1] = v.y;
  a[4 * q + 2] = v.z;
  a[4 * q + 3] = v.w;
}

__global__ void __launch_bounds__(256, 1) k_pairs_as(AsArgs A) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int64_t n = eff_n(A.s);
  const int64_t nblk = cdiv(n, kBS);
  const float slope = A.w.neg_slope;
  const float m1 = A.sc1, m2 = A.sc2, m3 = A.sc3;
  const float nim1 = -1.f / A.sc1, nim2 = -1.f / A.sc2, nim3 = -1.f / A.sc3;
  int* Q = reinterpret_cast<int*>(lds + OffQ);
  // tables (b2', b4', wa') -> LDS
  for (int i = threadIdx.x; i < 3 * 2 * 128; i += 256) reinterpret_cast<float*>(lds + OffTab)[i] = A.tabs[i];
  int64_t blk = first_block(nblk);
  if (blk >= nblk) return;   // uniform over the workgroup: no barrier reached yet
  // weight ring prologue: steps 0..2 into slots 0..2
  Stream S;
  S.pack = A.pack + __builtin_amdgcn_readfirstlane(wid) * 6 * 1024;
  S.lane_off = lane * 16;
  S.ring = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds + OffRing) + wid * 6 * 1024);
  S.g = 0;
#pragma unroll
  for (int st = 0; st < 3; ++st) {
    stream_dma_group<0>(S, st, st);
    stream_dma_group<1>(S, st, st);
  }
  // first tile: gather, PE, P1
  char* pe_lds = lds + OffPE + wid * (2 * 4 * 64 * 16);
  auto ex_lds = [&](int parity) { return lds + OffEx + (parity * 4 + wid) * (2 * 64 * 16); };
  Next nx;
  {
    Rec r0;
    rec_load(A, blk * 4 + wid, nblk, lane, r0);
    rec_take(r0, blk * 4 + wid, n, lane, nx, ex_lds(0));
  }
  static_for<0, 15>([&](auto e) { pe_pair<decltype(e)::value>(nx.d3, pe_lds, lane); });
  pe_pad(pe_lds, lane);
  f32x16 X[8], Y[8];
#pragma unroll
  for (int T = 0; T < 8; ++T) Y[T] = (f32x16){0.f};   // the first tile's "previous" tile: finite, never stored
#pragma unroll
  for (int T = 0; T < 8; ++T) load_p1(A, nx.prow, h, T, X[T]);
  Cur cur{nx.v, nx.wt, nx.sflag, nx.act}, prev{0, 0.f, 0, false};
  bool drain = false;
  float pa = 0.f, chk = 0.f;
  int par = 0;   // tile parity: the extras buffer of the current tile
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // ring slots 0..2 landed (hipcc does not count the DMA)
  __syncthreads();   // ring slots 0..2, the tables, PE and extras visible
  Frag fr;
#pragma unroll
  for (int r = 0; r < kFragDist; ++r) fr.w[r] = read_plane(lds, 0, r % 8, r / 8, lane);
  uint4 bh, bl;
  pe_read(pe_lds, 0, lane, bh, bl);
  while (true) {
    // ------------------------------------------------ L1: X = P1/sc1 + W1b.PE5 ; tail of the previous tile
    if (wid == 0 && lane == 0) Q[0] = drain ? (int)nblk : (int)take_block(A.blk_ctr, nblk);
    static_for<0, kL1>([&](auto tt) {
      constexpr int t = decltype(tt)::value;
      uint4 nh, nl;
      kstep(lds, S, wid, lane, X, bh, bl, fr, [&](auto ii) {
        constexpr int i = decltype(ii)::value;
        tail_piece<t, i>(A, lds, Y, prev, lane, slope, pa, chk);   // first tile: an empty prev (act false)
        if constexpr (i == 12 && t + 1 < kL1) pe_read(pe_lds, t + 1, lane, nh, nl);
      });
      if constexpr (t + 1 < kL1) {
        bh = nh;
        bl = nl;
      }
    });
    // ------------------------------------------------ L2: Y = b2' + W2.lrelu(X) ; gather of the next tile
    conv8(X[0], 0, slope, m1, nim1, bh, bl);
    init_bias(Y, lds, 0, h);
    const int64_t nblk_next = Q[0];   // published before the L1 barriers
    Rec rn;
    static_for<0, kL2>([&](auto tt) {
      constexpr int t = decltype(tt)::value;
      Conv cv;
      kstep(lds, S, wid, lane, Y, bh, bl, fr, [&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr (t + 1 < kL2) conv_piece<i>(X[(t + 1) >> 1], (t + 1) & 1, slope, m1, nim1, cv);
        if constexpr (i == 12 && t == 7) rec_load(A, nblk_next * 4 + wid, nblk, lane, rn);
        if constexpr (i == 18 && t == 11) rec_take(rn, nblk_next * 4 + wid, n, lane, nx, ex_lds(par ^ 1));
      });
      if constexpr (t + 1 < kL2) {
        bh = make_uint4(cv.hh[0], cv.hh[1], cv.hh[2], cv.hh[3]);
        bl = make_uint4(cv.ll[0], cv.ll[1], cv.ll[2], cv.ll[3]);
      }
    });
    // ------------------------------------------------ L3: X = W3.[lrelu(Y); extras] ; PE of the next tile
    conv8(Y[0], 0, slope, m2, nim2, bh, bl);
#pragma unroll
    for (int T = 0; T < 8; ++T) X[T] = (f32x16){0.f};
    static_for<0, kL3>([&](auto tt) {
      constexpr int t = decltype(tt)::value;
      Conv cv;
      uint4 eh, el;
      kstep(lds, S, wid, lane, X, bh, bl, fr, [&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr (t + 1 < 16) conv_piece<i>(Y[(t + 1) >> 1], (t + 1) & 1, slope, m2, nim2, cv);
        if constexpr (i == 18 && t < 15) pe_pair<t>(nx.d3, pe_lds, lane);
        if constexpr (i == 18 && t == 15) pe_pad(pe_lds, lane);
        if constexpr (i == 12 && t + 1 == 16) ex_read(ex_lds(par), lane, eh, el);
      });
      if constexpr (t + 1 < 16) {
        bh = make_uint4(cv.hh[0], cv.hh[1], cv.hh[2], cv.hh[3]);
        bl = make_uint4(cv.ll[0], cv.ll[1], cv.ll[2], cv.ll[3]);
      } else if constexpr (t + 1 == 16) {
        bh = eh;
        bl = el;
      }
    });
    // ------------------------------------------------ L4: Y = b4' + W4.lrelu(X) ; P1 of the next tile into X
    conv8(X[0], 0, slope, m3, nim3, bh, bl);
    init_bias(Y, lds, 1, h);
    static_for<0, kL4>([&](auto tt) {
      constexpr int t = decltype(tt)::value;
      Conv cv;
      uint4 ph, pl;
      kstep(lds, S, wid, lane, Y, bh, bl, fr, [&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr (t + 1 < kL4) conv_piece<i>(X[(t + 1) >> 1], (t + 1) & 1, slope, m3, nim3, cv);
        // all of X is free once step 14's conversion has read its last tile: the
        // next tile's P1 rows go in as one batch (one exposed gather latency per tile)
        if constexpr (t == kL4 - 1 && i >= 8) load_p1_q(A, nx.prow, h, (i - 8) >> 1, 2 * ((i - 8) & 1), X[(i - 8) >> 1]);
        if constexpr (t == kL4 - 1 && i >= 8) load_p1_q(A, nx.prow, h, (i - 8) >> 1, 2 * ((i - 8) & 1) + 1, X[(i - 8) >> 1]);
        if constexpr (i == 12 && t + 1 == kL4) pe_read(pe_lds, 0, lane, ph, pl);   // the next tile's first B
      });
      if constexpr (t + 1 < kL4) {
        bh = make_uint4(cv.hh[0], cv.hh[1], cv.hh[2], cv.hh[3]);
        bl = make_uint4(cv.ll[0], cv.ll[1], cv.ll[2], cv.ll[3]);
      } else {
        bh = ph;
        bl = pl;
      }
    });
    par ^= 1;
    prev = cur;
    cur = Cur{nx.v, nx.wt, nx.sflag, nx.act};
    if (drain) break;
    // uniform: every wave read the same Q[0].  Past the last block one more
    // (empty) tile runs, so that every real tile's tail is the in-loop one: a
    // sample's bits never depend on whether its tile was a workgroup's last.
    drain = nblk_next >= nblk;
  }
  if (A.range_flag && chk != 0.f) atomicOr(A.range_flag, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no ring DMA may land after the workgroup's LDS is freed
}

}  // namespace

int launch_pairs_as(const pnr_points& pts, const pnr_samples& s, const pnr_mlp& w, const AsPack& ap, const float* p1,
                    float* hid, int32_t* vmask, float* out_feat, float* out_weight, float* out_conf,
                    int32_t* blk_ctr, uint4* rec, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pairs_as), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kAsLds));
    attr = true;
  }
  AsArgs a;
  a.pts = pts;
  a.s = s;
  a.w = w;
  a.pack = static_cast<const char*>(ap.pack);
  a.tabs = ap.tabs;
  a.sc1 = ap.scale[0];
  a.sc2 = ap.scale[1];
  a.sc3 = ap.scale[2];
  a.sc4 = ap.scale[3];
  a.inv_k3 = 1.f / (2048.f * ap.scale[1]);
  a.p1 = p1;
  a.hid = hid;
  a.vmask = vmask;
  a.out_feat = out_feat;
  a.blk_ctr = blk_ctr;
  a.range_flag = ap.range_flag;
  a.rec = rec;
  a.rec_stride = as_rec_stride(s.n_max);
  RecArgs r;
  r.pts = pts;
  r.s = s;
  r.w = w;
  r.inv_k3 = a.inv_k3;
  r.rec = rec;
  r.rec_stride = a.rec_stride;
  r.out_weight = out_weight;
  r.out_conf = out_conf;
  const int64_t blocks = cdiv(s.n_max, kBS);
  hipLaunchKernelGGL(k_pair_rec, dim3((unsigned)cdiv(s.n_max * 8, 256)), dim3(256), 0, st, r);
  PNR_LAUNCH_CHECK();
  PNR_HIP(hipMemsetAsync(blk_ctr, 0, 8 * sizeof(int32_t), st));
  hipLaunchKernelGGL(k_pairs_as, dim3(grid_for(blocks, 1, 256)), dim3(256), kAsLds, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

}  // namespace pnr
