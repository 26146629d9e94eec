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

// Per-point Rw2c (pnr_points.rw2c, [N][9]; neural_points.py:799 gathers it per
// pair when Rw2c.dim() > 2): o = R_p v for the point of row prow.  A pair's world
// distance and point dir use its own point's matrix, a sample's view dir the
// matrix of its slot-0 neighbour (point_aggregators.py:492-496, 506, 526, 566).
// The kernels compute the uniform-Rw2c values first and overwrite them with
// these under a wave-uniform `pts.rw2c != NULL` test, so the uniform path's
// code is unchanged.
__device__ __forceinline__ void rot_point(const float* rw_pp, int64_t prow, const float v[3], float o[3]) {
  const float* R = rw_pp + (prow > 0 ? prow : 0) * 9;
  float m[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) m[i] = R[i];
  mat3(m, v, o);
}

// Point row whose Rw2c rotates the view dir of sample `row`: its slot-0
// neighbour (sampled_Rw2c[..., 0, :, :], clamp(pidx, 0)), or in pair-table mode
// (pnr_samples.pidx NULL) the sample's first pair row.
__device__ __forceinline__ int64_t slot0_point(const pnr_samples& s, int64_t row) {
  if (!s.pidx) return row * s.K;
  const int32_t p = s.pidx[row * s.K];
  return p > 0 ? p : 0;
}

__device__ __forceinline__ int64_t sample_row(const pnr_samples& s, int64_t v) {
  return s.samp_list ? (int64_t)s.samp_list[v] : v;
}

__device__ __forceinline__ int64_t dir_row(const pnr_samples& s, int64_t row) {
  return (s.dir_map ? (int64_t)s.dir_map[row] : row) / s.dir_div;
}

// Perspective coordinates of a gathered point (qpiw.py:102-109 w2pers) under the
// camera of the pair's ray: the launch's one camera (cam_c / cam_R, loaded once)
// or, for a multi-camera ray batch (pnr_samples.ray_cam), the ray's entry of the
// camera tables pts.campos[n_cams][3] / pts.camrot[n_cams][9].
__device__ __forceinline__ void pair_pers(const pnr_points& P, const pnr_samples& S, int64_t ray, const float pw[3],
                                          const float cam_c[3], const float cam_R[9], float pp[3]) {
  if (S.ray_cam) {
    const int64_t cam = S.ray_cam[ray];
    float c[3], R[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) c[i] = P.campos[cam * 3 + i];
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = P.camrot[cam * 9 + i];
    world_to_pers(pw, c, R, pp);
  } else {
    world_to_pers(pw, cam_c, cam_R, pp);
  }
}

// Rows of block1.0's point half (P1): the used points (device count when given,
// ABI 19) or every point.
__device__ __forceinline__ int64_t p1_rows(const pnr_points& p) {
  if (!p.used) return p.n;
  int64_t n = p.n_used;
  if (p.n_used_dev) {
    const int64_t d = *p.n_used_dev;
    n = d < n ? d : n;
  }
  return n;
}

__device__ __forceinline__ int64_t eff_n(const pnr_samples& s) {
  int64_t n = s.n_max;
  if (s.n_dev) {
    int64_t nd = *s.n_dev;
    n = nd < n ? nd : n;
  }
  return n;
}

// ---------------------------------------------------------------------------
// Exact 3-way bf16 split of fp32 values for the fp32-accurate bf16-MFMA GEMMs
// (aggregate_x3.hip): x = x0 + x1 + x2 with x0 = bf16(x), x1 = bf16(x - x0),
// x2 = bf16(x - x0 - x1), round-to-nearest-even, every residual exact in fp32.
// W . X then keeps the six cross products of weight >= 2^-16,
//   W2.X0 + W1.X1 + W0.X2 + W1.X0 + W0.X1 + W0.X0,
// on v_mfma_f32_32x32x16_bf16 (bf16 products are exact in fp32, fp32
// accumulation): the dropped terms are <= 2^-24 |w x|, one fp32 rounding.
__device__ __forceinline__ unsigned cvt_bf16x2(float a, float b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  bf2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}
// low bf16 of a pair as fp32 (v_perm_b32: `u << 16` gets rewritten into a second cvt)
__device__ __forceinline__ float bf16_lo_f(unsigned u) {
  return __builtin_bit_cast(float, __builtin_amdgcn_perm(u, 0u, 0x05040c0cu));
}
__device__ __forceinline__ float bf16_hi_f(unsigned u) { return __builtin_bit_cast(float, u & 0xffff0000u); }

// (a, b) -> three bf16 pairs (low half = a); 9 VALU
__device__ __forceinline__ void split2(float a, float b, unsigned& x0, unsigned& x1, unsigned& x2) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  x0 = cvt_bf16x2(a, b);
  const f2 r = v - (f2){bf16_lo_f(x0), bf16_hi_f(x0)};
  x1 = cvt_bf16x2(r.x, r.y);
  const f2 r2 = r - (f2){bf16_lo_f(x1), bf16_hi_f(x1)};
  x2 = cvt_bf16x2(r2.x, r2.y);
}

__device__ __forceinline__ f32x16 mfma_bf16(const uint4& a, const uint4& b, const f32x16& c) {
  typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Exact-enough 2-way fp16 split for the fp32-accurate f16-MFMA GEMMs
// (aggregate_x3.hip, pnr_aggregate_fwd_h2): x = xh + 2^-11 xl with
// xh = f16(x), xl = f16((x - xh) * 2^11), round-to-nearest-even; x - xh is exact
// in fp32 and |x - xh| <= 2^-12 |x| (normal range), so xl keeps the next 11
// bits and the split error is <= 2^-24 |x|.  W . X = 2^-11 (Ws.Xh + Wh.Xl + Wl.Xh)
// with Ws = 2^11 Wh (exact in f16: the weight pack is pre-scaled so |W| < 16):
// three products on v_mfma_f32_32x32x16_f16 instead of six; the dropped term
// 2^-22 Wl.Xl is <= 2^-24 |w x|.
__device__ __forceinline__ void splith(float a, float b, unsigned& x0, unsigned& x1) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  const h2 hi = __builtin_convertvector(v, h2);
  const f2 r = (v - __builtin_convertvector(hi, f2)) * 2048.f;
  const h2 lo = __builtin_convertvector(r, h2);
  x0 = __builtin_bit_cast(unsigned, hi);
  x1 = __builtin_bit_cast(unsigned, lo);
}

__device__ __forceinline__ f32x16 mfma_f16(const uint4& a, const uint4& b, const f32x16& c) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

// 8 f16 values x 2^11 (exact: the packs keep |Wh| < 16)
__device__ __forceinline__ uint4 f16x8_scale2048(const uint4& a) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  return __builtin_bit_cast(uint4, __builtin_bit_cast(h8, a) * (h8)((_Float16)2048.f));
}

// gemm.hip, for the native backward step (train_step.hip): C[:, :ncols] (rows of
// ldc floats) = A^T B on mode 0 fp32 / 1 fp32x3 / 2 fp32h2 (pnr_gemm_tn*), and
// the scratch that takes.
size_t gemm_scratch(int64_t K, int M, int N);
int gemm_tn_run(int mode, const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M, int32_t N,
                float* C, int64_t ldc, int32_t ncols, float* colsum_a, void* scratch, size_t scratch_bytes,
                void* stream, const uint32_t* a_absmax, int32_t* range_flag);
// C = A B (x LeakyReLU derivative) on fp32 / fp32h2 (pnr_gemm_nn*), max |C| folded
// into c_absmax when given (pre-zeroed): the next h2 product's scale, no pnr_absmax pass.
// b_split (h2, optional): B pre-split by nn_b_split (the same weights for every
// row block: split once per call instead of per workgroup and chunk).
int gemm_nn_run(bool h2, const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int32_t K, int32_t N,
                const float* act, int64_t ld_act, float slope, float* C, int64_t ldc, const uint32_t* a_absmax,
                int32_t* range_flag, uint32_t* c_absmax, void* stream, const void* b_split = nullptr);
size_t nn_b_split_bytes(int K, int N);
int nn_b_split(int n, const float* const* B, const int64_t* ldb, const int* K, const int* N, void* const* out,
               int32_t* flag, void* stream);

// aggregate_x3.hip: the pairs stage of pnr_aggregate_fwd_x3 (H = false: 3-way
// bf16 split, six products) and pnr_aggregate_fwd_h2 (H = true: 2-way f16
// split, three products).  packs: block1.0[:, 224:], block1.2, block3.0,
// block3.2; scale: per-layer output factor (1 for the bf16 packs);
// range_flag: set to 1 when an f16-split activation leaves the f16 range.
struct SplitW {
  const void* pack[4];
  float scale[4];
  int32_t* range_flag;
};
template <bool H>
int launch_pairs_split(const pnr_points& pts, const pnr_samples& s, const pnr_mlp& w, const SplitW& wx,
                       const float* p1, float* hid, int32_t* vmask, float* out_feat, float* out_weight,
                       float* out_conf, int32_t* tile_ctr, hipStream_t st, const pnr_agg_saved* sv = nullptr);
// k_point_pre_h2 (aggregate_x3.hip): P1 = W1[:, :224].[emb, PE_3(emb)] + b1 on
// f16-split MFMA (pack: frag_pack_h2 of W1[:, :224] with b1).
// x1 (training, optional): the input rows [emb, PE_3(emb)] are written there too
int launch_point_pre_h2(const pnr_points& pts, const void* pack, float scale, int32_t* range_flag, float* p1,
                        hipStream_t st, float* x1 = nullptr);
// Workgroup barrier for an LDS hand-off only: lgkmcnt(0) + s_barrier between
// LDS-scoped fences, so the compiler keeps LDS accesses on their side while
// global loads stay in flight across it (__syncthreads' fence drains them with
// vmcnt(0)).  Only where no global-memory hand-off between waves crosses.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Sample buckets by filled neighbour slots (buckets.hip): list = the sample
// indices partitioned by bucket b (KT = 1 << b slots), bucket b at
// [info[b], info[b] + info[4 + b]), in sample order within a bucket.
struct PairBuckets {
  int32_t* list;
  int32_t* info;
};
int64_t bucket_scratch_ints(int64_t n_max);
int launch_buckets(const pnr_samples& s, int32_t* scratch, PairBuckets* out, hipStream_t st);

// An add the compiler may not fuse with the multiply that produced an operand
// (hipcc contracts a * b + c into one FMA by default).  The bucketed K-sums of
// k_pairs_b rely on it: the KT = 8 tree adds rounded products to exact zeros
// where a KT < 8 tree adds them to each other, so a fused first stage would
// round differently between the two launches.
__device__ __forceinline__ float add_nc(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}

// xor-tree sum over the KT lanes of one sample (KT = 8: xor8_sum)
template <int KT>
__device__ __forceinline__ float xork_sum(float v) {
  if constexpr (KT >= 2) v += __shfl_xor(v, 1);
  if constexpr (KT >= 4) v += __shfl_xor(v, 2);
  if constexpr (KT >= 8) v += __shfl_xor(v, 4);
  return v;
}

// xork_sum whose adds never fuse with the multiply producing v (k_pairs_b's
// bucketed launches: every KT rounds a sample's sum like the 8-lane tree)
template <int KT>
__device__ __forceinline__ float xork_sum_nc(float v) {
  if constexpr (KT >= 2) v = add_nc(v, __shfl_xor(v, 1));
  if constexpr (KT >= 4) v = add_nc(v, __shfl_xor(v, 2));
  if constexpr (KT >= 8) v = add_nc(v, __shfl_xor(v, 4));
  return v;
}

// k_color_h2 (aggregate_x3.hip): the colour branch on f16-split MFMA; pack =
// color_branch.0 columns 0..143 / 144..279 + bias, color_branch.2, .4 (+ bias).
// train: the training forward (hid from its fp32 rows, saves vpe / hc1..hc3 as
// k_color<true> does); NULL: inference (hid planes from k_pairs_h2).
int launch_color_h2(const pnr_samples& s, const pnr_mlp& w, const void* const pack[4], const float scale[3],
                    int32_t* range_flag, const float* hid, const int32_t* vmask, float* out_feat, hipStream_t st,
                    const float* rw2c_pp, const pnr_agg_saved* train = nullptr);

}  // namespace pnr
