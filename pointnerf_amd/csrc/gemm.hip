// Weight-gradient GEMM of the backward pass: C[M,N] = A^T B summed over a long
// K (every (sample, neighbour) pair of the batch), A[K,M] / B[K,N] row-major
// -- dW = dZ^T X for block3.2, block3.0, block1.2 and block1.0's point half
// (the reference gets these from autograd of nn.Linear).
//
// CDNA4 mapping: v_mfma_f32_32x32x2_f32 consumes two K rows per step and both
// operands come straight from global memory in MFMA lane order (lane l reads
// A[k0 + (l>>5)][m0 + (l&31)] and B[k0 + (l>>5)][n0 + (l&31)]: two 128-B
// row segments per half-wave, no LDS and no transpose).  A workgroup of 8
// waves owns the whole C (M <= 256 rows, N <= 256 columns; wave w: rows
// 32w..32w+31 x every column tile, up to 128 accumulator VGPRs) for one K
// split, so A and B are read from HBM exactly once; the 8 waves read the same
// B rows (L1 hits).  K is split over ~256 workgroups (one per CU, 2 waves per
// SIMD); every split writes its own partial C, summed in a fixed order by a
// two-level reduction: deterministic, no float atomics.  Column sums of A
// (the bias gradients) ride along as an extra partial row.
#include "agg_common.h"

namespace pnr {

typedef float f32x16g __attribute__((ext_vector_type(16)));

constexpr int kGWaves = 8;   // waves per workgroup = 32-row tiles of C (M <= 256)
constexpr int kGMaxNT = 8;   // 32-column tiles of C (N <= 256)
constexpr int kGUnroll = 4;  // k-steps per software-pipeline stage
constexpr int kGGroup = 16;  // splits summed per first-level reduction thread

struct GemmArgs {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  int64_t K;
  int M, N;
  int64_t kchunk;      // rows of K per split (multiple of 2 * kGUnroll)
  float* part;         // [nsplit][M*N + M]  (C partial, then colsum partial)
  int colsum;
  const uint32_t* a_absmax;   // h2: bits of max |A| (pnr_absmax), picks A's power-of-two scale
  int32_t* range_flag;        // h2: set when a scaled operand leaves the f16 split's range
};

template <int NT>
__device__ __forceinline__ void gemm_body(const GemmArgs& g, int m0, int64_t k_begin, int64_t k_end, float* out,
                                          float* cs_out) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 31, h = lane >> 5;
  f32x16g acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = (f32x16g){0.f};
  float csum = 0.f;
  const float* pa = g.A + m0 + c;
  const float* pb = g.B + c;
  int64_t k = k_begin;
  // software pipeline: the next stage's operands are loaded while this
  // stage's MFMAs run (double-buffered registers)
  if (k + 2 * kGUnroll <= k_end) {
    float a[kGUnroll], b[kGUnroll][NT];
#pragma unroll
    for (int u = 0; u < kGUnroll; ++u) {
      const int64_t r = k + 2 * u + h;
      a[u] = pa[r * g.lda];
#pragma unroll
      for (int t = 0; t < NT; ++t) b[u][t] = pb[r * g.ldb + 32 * t];
    }
    for (;;) {
      const int64_t kn = k + 2 * kGUnroll;
      const bool more = kn + 2 * kGUnroll <= k_end;
      float an[kGUnroll], bn[kGUnroll][NT];
      if (more) {
#pragma unroll
        for (int u = 0; u < kGUnroll; ++u) {
          const int64_t r = kn + 2 * u + h;
          an[u] = pa[r * g.lda];
#pragma unroll
          for (int t = 0; t < NT; ++t) bn[u][t] = pb[r * g.ldb + 32 * t];
        }
      }
#pragma unroll
      for (int u = 0; u < kGUnroll; ++u) {
        csum += a[u];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u][t], acc[t], 0, 0, 0);
      }
      k = kn;
      if (!more) break;
      for (int u = 0; u < kGUnroll; ++u) {
        a[u] = an[u];
        for (int t = 0; t < NT; ++t) b[u][t] = bn[u][t];
      }
    }
  }
  for (; k < k_end; k += 2) {
    const int64_t r = k + h;
    const bool ok = r < k_end;
    const float a = ok ? pa[r * g.lda] : 0.f;
    csum += a;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float b = ok ? pb[r * g.ldb + 32 * t] : 0.f;
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
    }
  }
  // C/D layout: row = (r&3) + 8(r>>2) + 4h, col = c
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) out[(int64_t)(m0 + (r & 3) + 8 * (r >> 2) + 4 * h) * g.N + 32 * t + c] = acc[t][r];
  if (cs_out) {
    csum += __shfl_xor(csum, 32);
    if (h == 0) cs_out[m0 + c] = csum;
  }
}

__global__ void __launch_bounds__(64 * kGWaves, 1) k_gemm_tn_part(GemmArgs g) {
  const int wid = threadIdx.x >> 6;
  const int m0 = 32 * wid;
  if (m0 >= g.M) return;
  const int split = blockIdx.x;
  const int64_t k_begin = (int64_t)split * g.kchunk;
  int64_t k_end = k_begin + g.kchunk;
  if (k_end > g.K) k_end = g.K;
  const int64_t stride = (int64_t)g.M * g.N + g.M;
  float* out = g.part + (int64_t)split * stride;
  float* cs = g.colsum ? out + (int64_t)g.M * g.N : nullptr;
  switch (g.N / 32) {   // column tiles (N % 32 == 0, N <= 256)
    case 1: gemm_body<1>(g, m0, k_begin, k_end, out, cs); break;
    case 2: gemm_body<2>(g, m0, k_begin, k_end, out, cs); break;
    case 3: gemm_body<3>(g, m0, k_begin, k_end, out, cs); break;
    case 4: gemm_body<4>(g, m0, k_begin, k_end, out, cs); break;
    case 5: gemm_body<5>(g, m0, k_begin, k_end, out, cs); break;
    case 6: gemm_body<6>(g, m0, k_begin, k_end, out, cs); break;
    case 7: gemm_body<7>(g, m0, k_begin, k_end, out, cs); break;
    default: gemm_body<8>(g, m0, k_begin, k_end, out, cs); break;
  }
}

// ---------------------------------------------------------------- x3 variant
// fp32-accurate C = A^T B on bf16 MFMA (pnr_gemm_tn_x3): every operand split
// exactly into three bf16 terms (agg_common.h split2) and the six cross
// products of weight >= 2^-16 summed with fp32 accumulation (the forward's
// fp32x3 arithmetic): 6 v_mfma_f32_32x32x16_bf16 per 16 k-rows instead of 8
// v_mfma_f32_32x32x2_f32 per 2.  Per K split one 8-wave workgroup owns all of C
// as before; 16-row chunks of A and B are staged in LDS as split planes
// ([plane][row][k], 48-B lines), double-buffered: the next chunk's global loads
// are in flight during this chunk's MFMAs, split and written after them.  Wave w
// owns M tiles 2(w % 4) .. +1 x N tiles 4(w / 4) .. +3 (8 accumulators).
constexpr int kXK = 16;                 // k rows per chunk (one bf16 MFMA k-step)
constexpr int kXPitch = 24;             // bf16 per LDS line (16 k + 8 pad)
constexpr int kXPlane = 256 * kXPitch;  // bf16 per plane (256 rows)
constexpr size_t kXLds = 2 * 2 * 3 * (size_t)kXPlane * 2;   // [buf][A|B][plane] = 144 KB

// One K split of the x3 product; plane(buf, p) is the LDS address of split
// plane p (0..2: A, 3..5: B) of staging buffer buf, red a 1-KB LDS scratch for
// the column sums.  Shared by k_gemm_tn_x3_part and k_gemm_tn_h2_part's
// in-place fallback (which lays the twelve planes over its own LDS).
template <class Plane>
__device__ __forceinline__ void tn_x3_split(const GemmArgs& g, Plane plane, float* red) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int64_t k_begin = (int64_t)blockIdx.x * g.kchunk;
  const int64_t k_end = k_begin + g.kchunk < g.K ? k_begin + g.kchunk : g.K;
  const int64_t stride = (int64_t)g.M * g.N + g.M;
  float* out = g.part + (int64_t)blockIdx.x * stride;
  // staging role: column col of A and of B, k rows 8 kh .. 8 kh + 7 of a chunk
  const int col = tid & 255, kh = tid >> 8;
  const bool stA = col < g.M, stB = col < g.N;
  float csum = 0.f;
  auto load = [&](int64_t k0, float (&va)[8], float (&vb)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t r = k0 + 8 * kh + j;
      const bool ok = r < k_end;
      va[j] = ok && stA ? g.A[r * g.lda + col] : 0.f;
      vb[j] = ok && stB ? g.B[r * g.ldb + col] : 0.f;
    }
  };
  auto put = [&](int buf, const float (&va)[8], const float (&vb)[8]) {
    const int off = col * kXPitch + 8 * kh;
    uint4 pa[3], pb[3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      csum += va[2 * q] + va[2 * q + 1];
      unsigned x0, x1, x2;
      split2(va[2 * q], va[2 * q + 1], x0, x1, x2);
      reinterpret_cast<unsigned*>(&pa[0])[q] = x0;
      reinterpret_cast<unsigned*>(&pa[1])[q] = x1;
      reinterpret_cast<unsigned*>(&pa[2])[q] = x2;
      split2(vb[2 * q], vb[2 * q + 1], x0, x1, x2);
      reinterpret_cast<unsigned*>(&pb[0])[q] = x0;
      reinterpret_cast<unsigned*>(&pb[1])[q] = x1;
      reinterpret_cast<unsigned*>(&pb[2])[q] = x2;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      *reinterpret_cast<uint4*>(plane(buf, p) + off) = pa[p];
      *reinterpret_cast<uint4*>(plane(buf, 3 + p) + off) = pb[p];
    }
  };
  f32x16 acc[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (f32x16){0.f};
  const int mt0 = 2 * (wid & 3), nt0 = 4 * (wid >> 2);
  auto compute = [&](int buf) {
    const int off = c * kXPitch + 8 * h;
    uint4 a[2][3];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        a[mi][p] = *reinterpret_cast<const uint4*>(plane(buf, p) + off + 32 * (mt0 + mi) * kXPitch);
    // per N tile: its B planes, then the six products of both M tiles, smallest
    // terms first (A2B0, A1B1, A0B2, A1B0, A0B1, A0B0)
    constexpr int kPa[6] = {2, 1, 0, 1, 0, 0}, kPb[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      if (32 * (nt0 + ni) >= g.N) continue;
      uint4 b[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        b[p] = *reinterpret_cast<const uint4*>(plane(buf, 3 + p) + off + 32 * (nt0 + ni) * kXPitch);
#pragma unroll
      for (int e = 0; e < 6; ++e)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          if (32 * (mt0 + mi) < g.M) acc[mi][ni] = mfma_bf16(a[mi][kPa[e]], b[kPb[e]], acc[mi][ni]);
    }
  };
  // Two register sets of staged rows rotate statically (loop unrolled by two):
  // chunk i + 3's global loads are issued while chunk i is multiplied and are
  // consumed (split + LDS store) two chunks later, so two chunks of loads are
  // always in flight.  Chunks past k_end load as zeros (never multiplied).
  // the next chunk's global loads are in flight during this chunk's MFMAs, split
  // and written to the other LDS buffer after them.  (Two chunks in flight from
  // two rotating register sets measured 1.7x slower: 16 more VGPRs spill; 16
  // waves of 4 accumulators each, 4 waves per SIMD, 1.2x slower.)
  float va[8], vb[8];
  load(k_begin, va, vb);
  put(0, va, vb);
  __syncthreads();
  int it1 = 0;
  for (int64_t k0 = k_begin; k0 < k_end; k0 += kXK, ++it1) {
    const int buf = it1 & 1;
    const bool more = k0 + kXK < k_end;
    if (more) load(k0 + kXK, va, vb);
    compute(buf);
    if (more) put(buf ^ 1, va, vb);
    __syncthreads();
  }
  // C/D layout: row = (r&3) + 8(r>>2) + 4h, col = c
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int m0 = 32 * (mt0 + mi), n0 = 32 * (nt0 + ni);
      if (m0 >= g.M || n0 >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) out[(int64_t)(m0 + (r & 3) + 8 * (r >> 2) + 4 * h) * g.N + n0 + c] = acc[mi][ni][r];
    }
  if (g.colsum) {   // column sums of A: the two k-halves of every column
    __syncthreads();
    if (kh == 1) red[col] = csum;
    __syncthreads();
    if (kh == 0 && stA) out[(int64_t)g.M * g.N + col] = csum + red[col];
  }
}

__global__ void __launch_bounds__(512, 1) k_gemm_tn_x3_part(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t glds[];
  tn_x3_split(g, [&](int buf, int p) { return glds + (size_t)(buf * 6 + p) * kXPlane; },
              reinterpret_cast<float*>(glds));
}

// ---------------------------------------------------------------- h2 variant
// fp32-accurate C = A^T B on f16 MFMA (pnr_gemm_tn_h2), the forward's fp32h2
// arithmetic (aggregate_x3.hip) for the weight gradients: A is scaled by 2^e so
// that max |A| 2^e lies in [4, 8) (e from the device max the producer wrote:
// gradients of any magnitude use the f16 exponent range), both operands split
// x = xh + 2^-11 xl (splith, exact residuals), and
//   2^11 (A 2^e)^T B ~= (2^11 Ah)^T Bh + Ah^T Bl + Al^T Bh
// -- three v_mfma_f32_32x32x16_f16 per 16 k-rows instead of x3's six bf16
// products.  2^11 Ah is exact in f16 (|Ah| < 8).  The dropped 2^-22 Al^T Bl and
// the split residuals are <= ~2^-21 |a b| per product.  Operands outside the
// split's range (|B| >= 2^15, a stale max, non-finite) raise range_flag, and
// the workgroups that saw them redo their split on the x3 path in place
// (tn_x3_split over this kernel's LDS): no second launch.
//
// Staging: the raw fp32 rows of a 16-row chunk (A and B, one <= 1-KB row per
// wave instruction) go global -> LDS by buffer_load ... lds (no VGPRs), three
// chunks in flight in three LDS slots (the chunk loop is latency-bound with one
// chunk of register-staged loads per CU: ~3.4 TB/s on a 256 x 256 x 240 k
// product); rows past the split and columns past M / N read as zeros (out of
// the buffer's range).  Per chunk: counted vmcnt for the oldest slot, barrier,
// split into two f16 planes per operand (one LDS image), barrier, refill the
// slot, MFMAs.  Raw s_barrier with explicit waits (a __syncthreads() would
// drain the in-flight DMAs with vmcnt(0)).
constexpr int kHRawRow = 1024;                        // bytes per staged row (256 fp32)
constexpr int kHRawSlot = 2 * kXK * kHRawRow;         // A rows then B rows: 32 KB
constexpr int kHSlots = 3;
constexpr size_t kHPlanes = 4 * (size_t)kXPlane * 2;  // Ah, Al, Bh, Bl: 48 KB
// the in-place x3 fallback's twelve planes: four over the h2 planes, eight over raw
static_assert(kHSlots * kHRawSlot == 8 * kXPlane * 2 && kHPlanes == 4 * (size_t)kXPlane * 2, "x3 fallback LDS map");

__device__ __forceinline__ void hw_barrier_lds() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) only (vmcnt / expcnt left at their maxima)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 16 B per lane global -> LDS (buffer_load_dwordx4 ... lds): LDS address = m0 +
// lane * 16.  Issued as inline asm so that the compiler, which cannot tell the
// three slots apart, does not drain every DMA with vmcnt(0) before each LDS
// access; the kernel orders them itself (wait_vm before the barrier that
// precedes a slot's reads, a barrier before a slot is refilled).
typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i buf_desc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  return (v4i){(int)(uint32_t)a, (int)(uint32_t)((a >> 32) & 0xffffu), (int)bytes, 0x00020000};
}
__device__ __forceinline__ void dma16(v4i desc, uint32_t voff, uint32_t lds_addr) {
  // m0 is not named as a clobber (a reserved register): nothing else in the
  // kernel's loop reads it (checked in the ISA: the only m0 writes are these)
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(desc), "s"(lds_addr)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {   // vmcnt(N), other counters unconstrained
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

__global__ void __launch_bounds__(512, 1) k_gemm_tn_h2_part(GemmArgs g) {
  // two distinct LDS objects: the DMA destinations provably never alias the
  // planes, so the compiler's waits for the DMAs stay out of the plane accesses
  __shared__ __attribute__((aligned(16))) uint16_t glds[kHPlanes / 2];
  __shared__ __attribute__((aligned(16))) char raw[kHSlots * kHRawSlot];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int64_t k_begin = (int64_t)blockIdx.x * g.kchunk;
  const int64_t k_end = k_begin + g.kchunk < g.K ? k_begin + g.kchunk : g.K;
  const int nchunk = (int)cdiv(k_end - k_begin, (int64_t)kXK);
  const int64_t stride = (int64_t)g.M * g.N + g.M;
  float* out = g.part + (int64_t)blockIdx.x * stride;
  // A's scale 2^e: max |A| 2^e in [4, 8)
  int e = 0;
  {
    const float amax = __uint_as_float(*g.a_absmax);
    if (amax > 0.f && amax <= 3.0e38f) {
      int x;
      frexpf(amax, &x);   // amax = f 2^x, f in [0.5, 1)
      e = 3 - x;
    }
  }
  const float sa = ldexpf(1.f, e);
  // the split's rows as buffers: rows >= k_end and bytes past a row's M / N columns read 0
  const uint32_t rowsA = (uint32_t)(k_end - k_begin);
  const v4i rA = buf_desc(g.A + k_begin * g.lda, rowsA * (uint32_t)g.lda * 4u);
  const v4i rB = buf_desc(g.B + k_begin * g.ldb, rowsA * (uint32_t)g.ldb * 4u);
  const uint32_t raw0 = (uint32_t)reinterpret_cast<uintptr_t>(raw);   // LDS byte address
  const bool inA = lane * 16 < g.M * 4, inB = lane * 16 < g.N * 4;
  // wave w stages rows 2w, 2w + 1 of A and of B of every chunk
  auto issue = [&](int chunk) {
    const uint32_t slot = raw0 + (uint32_t)((chunk % kHSlots) * kHRawSlot);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = 2 * wid + j;
      const uint32_t row = (uint32_t)(chunk * kXK + r);
      const uint32_t oa = inA ? row * (uint32_t)g.lda * 4u + lane * 16 : 0x7ffffff0u;
      const uint32_t ob = inB ? row * (uint32_t)g.ldb * 4u + lane * 16 : 0x7ffffff0u;
      dma16(rA, oa, __builtin_amdgcn_readfirstlane(slot + r * kHRawRow));
      dma16(rB, ob, __builtin_amdgcn_readfirstlane(slot + (kXK + r) * kHRawRow));
    }
  };
  const int col = tid & 255, kh = tid >> 8;
  const bool stA = col < g.M;
  float csum = 0.f;
  bool bad = false;   // a scaled A with |a| >= 8, a B with |b| >= 2^15, or a NaN / inf
  f32x16 acc[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (f32x16){0.f};
  const int mt0 = 2 * (wid & 3), nt0 = 4 * (wid >> 2);
  for (int q = 0; q < kHSlots && q < nchunk; ++q) issue(q);
  for (int it = 0; it < nchunk; ++it) {
    // this wave's DMAs of chunk `it` are done when at most those of the chunks after it remain
    const int ahead = nchunk - 1 - it < kHSlots - 1 ? nchunk - 1 - it : kHSlots - 1;
    if (ahead >= 2) wait_vm<8>();
    else if (ahead == 1) wait_vm<4>();
    else wait_vm<0>();
    hw_barrier_lds();
    {   // split: column col of A and B, k rows 8 kh .. 8 kh + 7 of the chunk
      const float* ra = reinterpret_cast<const float*>(raw + (it % kHSlots) * kHRawSlot) + col;
      const float* rb = ra + kXK * (kHRawRow / 4);
      uint4 pa[2], pb[2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r0 = 8 * kh + 2 * q;
        const float v0 = ra[r0 * (kHRawRow / 4)], v1 = ra[(r0 + 1) * (kHRawRow / 4)];
        const float b0 = rb[r0 * (kHRawRow / 4)], b1 = rb[(r0 + 1) * (kHRawRow / 4)];
        const float a0 = v0 * sa, a1 = v1 * sa;
        csum += v0 + v1;
        const bool ok = (fabsf(a0) < 8.f) && (fabsf(a1) < 8.f) && (fabsf(b0) < 32768.f) && (fabsf(b1) < 32768.f);
        bad = bad || !ok;
        unsigned x0, x1;
        splith(a0, a1, x0, x1);
        reinterpret_cast<unsigned*>(&pa[0])[q] = x0;
        reinterpret_cast<unsigned*>(&pa[1])[q] = x1;
        splith(b0, b1, x0, x1);
        reinterpret_cast<unsigned*>(&pb[0])[q] = x0;
        reinterpret_cast<unsigned*>(&pb[1])[q] = x1;
      }
      uint16_t* base = glds + col * kXPitch + 8 * kh;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        *reinterpret_cast<uint4*>(base + p * kXPlane) = pa[p];
        *reinterpret_cast<uint4*>(base + (2 + p) * kXPlane) = pb[p];
      }
    }
    hw_barrier_lds();   // planes written; the raw slot fully read
    if (it + kHSlots < nchunk) issue(it + kHSlots);
    {   // MFMAs on the planes
      const uint16_t* lb = glds + c * kXPitch + 8 * h;
      uint4 ah[2], al[2], as[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        ah[mi] = *reinterpret_cast<const uint4*>(lb + 32 * (mt0 + mi) * kXPitch);
        al[mi] = *reinterpret_cast<const uint4*>(lb + kXPlane + 32 * (mt0 + mi) * kXPitch);
        as[mi] = f16x8_scale2048(ah[mi]);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        if (32 * (nt0 + ni) >= g.N) continue;
        const uint4 bh = *reinterpret_cast<const uint4*>(lb + 2 * kXPlane + 32 * (nt0 + ni) * kXPitch);
        const uint4 bl = *reinterpret_cast<const uint4*>(lb + 3 * kXPlane + 32 * (nt0 + ni) * kXPitch);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          if (32 * (mt0 + mi) >= g.M) continue;
          acc[mi][ni] = mfma_f16(al[mi], bh, acc[mi][ni]);   // smallest terms first
          acc[mi][ni] = mfma_f16(ah[mi], bl, acc[mi][ni]);
          acc[mi][ni] = mfma_f16(as[mi], bh, acc[mi][ni]);
        }
      }
    }
    hw_barrier_lds();   // every wave is done reading the planes
  }
  wait_vm<0>();
  const float unscale = ldexpf(1.f, -(e + 11));   // exact: a power of two
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int m0 = 32 * (mt0 + mi), n0 = 32 * (nt0 + ni);
      if (m0 >= g.M || n0 >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(int64_t)(m0 + (r & 3) + 8 * (r >> 2) + 4 * h) * g.N + n0 + c] = acc[mi][ni][r] * unscale;
    }
  if (g.colsum) {   // column sums of A (unscaled fp32): the two k-halves of every column
    float* red = reinterpret_cast<float*>(glds);
    __syncthreads();
    if (kh == 1) red[col] = csum;
    __syncthreads();
    if (kh == 0 && stA) out[(int64_t)g.M * g.N + col] = csum + red[col];
  }
  // written first so that no accumulator is live below
  if (__syncthreads_or(bad)) {
    // an operand of this split outside the f16 split's range (or NaN / inf): the
    // split again on the exact x3 path, in place -- its twelve planes laid over
    // this kernel's LDS (buffer 0 in raw[0 .. 6 planes), buffer 1 in glds' four
    // planes + raw's last two) -- overwriting this split's partial; the other
    // splits keep their h2 partials
    if (tid == 0) atomicOr(g.range_flag, 1);
    uint16_t* r16 = reinterpret_cast<uint16_t*>(raw);
    tn_x3_split(g,
                [&](int buf, int p) {
                  return buf == 0 ? r16 + p * kXPlane : (p < 4 ? glds + p * kXPlane : r16 + (p + 2) * kXPlane);
                },
                reinterpret_cast<float*>(glds));
  }
}

// max |x| over x[0, n) as float bits (pnr_absmax): per-block maxima, then one
// block (no atomics, no pre-zeroed output).  NaN propagates (the h2 GEMM then
// raises its range flag and runs the x3 fallback).
constexpr int kAbsBlocks = 1024;
__global__ void __launch_bounds__(256) k_absmax_part(const float* __restrict__ x, int64_t n, float* __restrict__ part) {
  __shared__ float red[4];
  float m = 0.f;
  const int64_t n4 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 ? n / 4 : 0;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = x4[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    if (v.x != v.x || v.y != v.y || v.z != v.z || v.w != v.w) m = __int_as_float(0x7fc00000);
  }
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = x[i];
    m = fmaxf(m, fabsf(v));
    if (v != v) m = __int_as_float(0x7fc00000);
  }
  const bool nan = m != m;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const bool anynan = __any(nan);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = anynan ? __int_as_float(0x7fc00000) : m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    bool bn = false;
    for (int w = 0; w < 4; ++w) {
      bn |= red[w] != red[w];
      r = fmaxf(r, red[w]);
    }
    part[blockIdx.x] = bn ? __int_as_float(0x7fc00000) : r;
  }
}

__global__ void __launch_bounds__(256) k_absmax_final(const float* __restrict__ part, int nb, uint32_t* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  bool nan = false;
  for (int i = threadIdx.x; i < nb; i += 256) {
    const float v = part[i];
    nan |= v != v;
    m = fmaxf(m, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const bool anynan = __any(nan);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = anynan ? __int_as_float(0x7fc00000) : m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    bool bn = false;
    for (int w = 0; w < 4; ++w) {
      bn |= red[w] != red[w];
      r = fmaxf(r, red[w]);
    }
    out[0] = __float_as_uint(bn ? __int_as_float(0x7fc00000) : r);
  }
}

// out[grp][i] = sum_{s in group grp} part[s][i] in split order (float4 lanes).
__global__ void k_reduce_splits(const float* __restrict__ part, int64_t n4, int nsplit, int group,
                                float* __restrict__ out) {
  const int grp = blockIdx.y;
  const int s0 = grp * group, s1 = min(nsplit, s0 + group);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = s0; q < s1; ++q) {
      const float4 v = reinterpret_cast<const float4*>(part)[(int64_t)q * n4 + i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    reinterpret_cast<float4*>(out)[(int64_t)grp * n4 + i] = acc;
  }
}

// Last level: c[i] = sum_g part[g][i] (float4 lanes) straight into the caller's
// C (first nc4 lanes) and column sums (the rest; skipped when cs == NULL).
// C [M, N] as rows of ldc floats of which the first ncols are written (a slice
// of a wider gradient: ldc != N or ncols < N -> scalar stores).
__global__ void k_reduce_final(const float* __restrict__ part, int64_t n4, int nsplit, int64_t nc4,
                               float* __restrict__ c, float* __restrict__ cs, int nq, int64_t ldc, int ncols) {
  const bool dense = ldc == 4 * nq && ncols == 4 * nq;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    if (i >= nc4 && cs == nullptr) break;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < nsplit; ++q) {
      const float4 v = reinterpret_cast<const float4*>(part)[(int64_t)q * n4 + i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    if (i >= nc4) {
      reinterpret_cast<float4*>(cs)[i - nc4] = acc;
    } else if (dense) {
      reinterpret_cast<float4*>(c)[i] = acc;
    } else {
      const int64_t row = i / nq;
      const int c0 = 4 * (int)(i - row * nq);
      float* o = c + row * ldc + c0;
      if (c0 < ncols) o[0] = acc.x;
      if (c0 + 1 < ncols) o[1] = acc.y;
      if (c0 + 2 < ncols) o[2] = acc.z;
      if (c0 + 3 < ncols) o[3] = acc.w;
    }
  }
}

static void gemm_plan(int64_t K, int* nsplit, int64_t* kchunk) {
  int64_t s = 256;                                   // one 8-wave workgroup per CU
  const int64_t maxs = K / 128 > 0 ? K / 128 : 1;    // >= 128 k-rows per split
  if (s > maxs) s = maxs;
  int64_t kc = cdiv(K > 0 ? K : 1, s);
  kc = cdiv(kc, 16) * 16;   // whole 16-row chunks (x3) and 2 * kGUnroll pipeline stages (fp32)
  *kchunk = kc;
  *nsplit = (int)(K > 0 ? cdiv(K, kc) : 1);
}

size_t gemm_scratch(int64_t K, int M, int N) {
  int ns;
  int64_t kc;
  gemm_plan(K, &ns, &kc);
  const size_t stride = (size_t)M * N + M;
  return (stride * ns + stride * cdiv(ns, kGGroup)) * sizeof(float);
}

// ---------------------------------------------------------------- NN variant
// Data-gradient products of the backward: C[M,N] = A[M,K] B[K,N] (dX = dZ W of
// an nn.Linear, W row-major as stored), optionally times the LeakyReLU
// derivative of a saved activation: C[m,n] *= act[m,n] > 0 ? 1 : slope
// (torch.where(h > 0, dy, dy * slope) fused into the epilogue).  Exact fp32
// products on v_mfma_f32_32x32x2_f32 (64 cycles each: the kernel is
// MFMA-bound once its operands are in LDS).  An 8-wave workgroup owns 32 WM
// rows of C and all N <= 256 columns: WM waves along M x (8 / WM) along N
// (WM = 4 for long M, 2 for the ~30 k-row colour-branch batches so that the
// grid still covers the CUs).  32-deep k chunks of its A rows (pitch 33:
// conflict-free A-operand reads) and of B (pitch N, + 32 floats when
// N % 64 == 0: the two half-waves' rows 32 banks apart) are staged in LDS; the
// next chunk's global loads are issued before this chunk's MFMAs and written to
// LDS after them.
constexpr int kNK = 32, kNPitch = kNK + 1, kNBMax = kNK * (256 + 32);

struct GemmNNArgs {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  const float* act;
  int64_t ld_act;
  int64_t M;
  int K, N;
  float slope;
  const uint32_t* a_absmax;   // h2: bits of max |A|
  int32_t* range_flag;        // h2: operand outside the f16 split's range
  uint32_t* c_absmax;         // optional: max |C| folded in (float bits, atomic; pre-zeroed)
  const int32_t* run_if;      // fp32: run only when *run_if != 0 (the h2 call's fallback)
  const uint4* b_split;       // h2, optional: B already split (nn_b_split: [K/8][N][hi, lo]), range checked
};

// max |v| of this thread's values into *word, one atomic per workgroup (NaN above inf)
__device__ __forceinline__ void block_absmax_to(uint32_t* word, unsigned mb, unsigned* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mb;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) mb = max(mb, red[w]);
    if (mb) atomicMax(word, mb);
  }
}

__device__ __forceinline__ unsigned abs_bits(float v) {
  const float a = fabsf(v);
  return a != a ? 0x7fc00000u : __float_as_uint(a);
}

// The fp32 product of rows row0 .. row0 + 32 WM (k_gemm_nn's body): as / bs the
// LDS staging (32 WM x kNPitch and kNBMax floats).
template <int NT, int WM>
__device__ __forceinline__ void nn_fp32_rows(const GemmNNArgs& g, int64_t row0, float* as, float* bs) {
  constexpr int WN = 8 / WM;               // waves along N
  constexpr int NW = (NT + WN - 1) / WN;   // column tiles per wave (at most)
  constexpr int ROWS = 32 * WM;
  constexpr int AV = ROWS * kNK / 512;     // staged A floats per thread
  constexpr int BV = kNK * 32 * NT / 512;  // staged B floats per thread
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wm = wid % WM, wn = wid / WM;
  const int N = 32 * NT;
  const int bp = N % 64 == 0 ? N + 32 : N;   // B pitch in LDS
  float ra[AV], rb[BV];
  // A: thread -> rows (tid >> 5) + 16 j, k = tid & 31 (128-B row segments);
  // B: thread -> k rows (tid >> 5) + 16 (j / NT), columns 32 (j % NT) + (tid & 31)
  auto load = [&](int k0) {
    const int kk = k0 + (tid & 31);
#pragma unroll
    for (int j = 0; j < AV; ++j) {
      const int64_t gr = row0 + (tid >> 5) + 16 * j;
      ra[j] = gr < g.M && kk < g.K ? g.A[gr * g.lda + kk] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < BV; ++j) {
      const int r = k0 + (tid >> 5) + 16 * (j / NT);
      rb[j] = r < g.K ? g.B[(int64_t)r * g.ldb + 32 * (j % NT) + (tid & 31)] : 0.f;
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int j = 0; j < AV; ++j) as[((tid >> 5) + 16 * j) * kNPitch + (tid & 31)] = ra[j];
#pragma unroll
    for (int j = 0; j < BV; ++j) bs[((tid >> 5) + 16 * (j / NT)) * bp + 32 * (j % NT) + (tid & 31)] = rb[j];
  };
  f32x16g acc[NW];
#pragma unroll
  for (int t = 0; t < NW; ++t) acc[t] = (f32x16g){0.f};
  load(0);
  put();
  __syncthreads();
  const float* arow = as + (32 * wm + c) * kNPitch + h;
  const float* brow = bs + h * bp + c;
  for (int k0 = 0; k0 < g.K; k0 += kNK) {
    const bool more = k0 + kNK < g.K;
    if (more) load(k0 + kNK);   // in flight during the MFMAs
#pragma unroll
    for (int s = 0; s < kNK / 2; ++s) {
      const float a = arow[2 * s];
#pragma unroll
      for (int u = 0; u < NW; ++u) {
        const int t = wn + WN * u;
        if (t < NT) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, brow[2 * s * bp + 32 * t], acc[u], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
      put();
      __syncthreads();
    }
  }
  // C/D layout: row = (r&3) + 8(r>>2) + 4h, col = c
  unsigned mb = 0u;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (m >= g.M) continue;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int t = wn + WN * u;
      if (t >= NT) continue;
      const int n = 32 * t + c;
      float v = acc[u][r];
      if (g.act != nullptr && !(g.act[m * g.ld_act + n] > 0.f)) v *= g.slope;
      g.C[m * g.ldc + n] = v;
      mb = max(mb, abs_bits(v));
    }
  }
  if (g.c_absmax) block_absmax_to(g.c_absmax, mb, reinterpret_cast<unsigned*>(as));
}

template <int NT, int WM>
__global__ void __launch_bounds__(512, 1) k_gemm_nn(GemmNNArgs g) {
  if (g.run_if && *g.run_if == 0) return;   // guarded fallback of an h2 call whose operands fit
  __shared__ float as[32 * WM * kNPitch];
  __shared__ float bs[kNBMax];
  nn_fp32_rows<NT, WM>(g, (int64_t)blockIdx.x * 32 * WM, as, bs);
}

// h2 variant (pnr_gemm_nn_h2): the same C = A B (x LeakyReLU derivative) on
// f16-split MFMA -- A scaled by 2^e (max |A| 2^e in [4, 8), from *a_absmax),
// both operands split x = xh + 2^-11 xl, C = 2^-(e+11) ((2^11 Ah) Bh + Ah Bl +
// Al Bh): three v_mfma_f32_32x32x16_f16 per 16-k step where the fp32 kernel
// issues eight v_mfma_f32_32x32x2_f32 of 64 cycles.  A workgroup owns 128 rows
// (wave w: row tile w % 4, column tiles w / 4 + 2u); per 16-k chunk its A rows
// ([row][k]) and B's columns ([n][k], the transpose staged on the fly) are split
// into two f16 planes each, double-buffered in LDS (2 x 37 KB).  Out-of-range
// operands (|B| >= 2^15, a stale max, NaN / inf) raise range_flag; the caller
// launches the fp32 kernel behind it with run_if = range_flag.  (Redoing the
// flagged rows in place, as k_gemm_tn_h2_part does, made these kernels ~10 %
// slower: the fp32 body's registers and 4 spills at 128 VGPRs.)
constexpr int kNHRows = 128;
constexpr int kNHPlaneA = kNHRows * kXPitch;   // f16 per A plane
constexpr int kNHPlaneB = 256 * kXPitch;       // f16 per B plane
constexpr size_t kNHLds = 2 * (2 * (size_t)kNHPlaneA + 2 * (size_t)kNHPlaneB) * 2;

template <int NT, bool BS>   // BS: B pre-split (g.b_split)
__global__ void __launch_bounds__(512, 1) k_gemm_nn_h2(GemmNNArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t nlds[];
  constexpr int NW = (NT + 1) / 2;   // column tiles per wave (waves 0-3: even tiles, 4-7: odd)
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * kNHRows;
  const int wm = wid & 3, wn = wid >> 2;
  int e = 0;
  {
    const float amax = __uint_as_float(*g.a_absmax);
    if (amax > 0.f && amax <= 3.0e38f) {
      int x;
      frexpf(amax, &x);
      e = 3 - x;
    }
  }
  const float sa = ldexpf(1.f, e);
  bool bad = false;
  // staging roles -- A: row tid >> 2, k (tid & 3) * 4 .. +3; B: column tid & 255, k 8 (tid >> 8) .. +7
  const int ar = tid >> 2, ak = (tid & 3) * 4;
  const int bn = tid & 255, bk = 8 * (tid >> 8);
  const bool stB = bn < g.N;
  float4 va;
  float vb[BS ? 1 : 8];
  uint4 bsh = make_uint4(0u, 0u, 0u, 0u), bsl = bsh;
  auto load = [&](int k0) {
    const int64_t gr = row0 + ar;
    const int kk = k0 + ak;
    if (gr < g.M && kk + 3 < g.K) {
      const float* src = g.A + gr * g.lda + kk;
      va = (((uintptr_t)src & 15) == 0) ? *reinterpret_cast<const float4*>(src)
                                         : make_float4(src[0], src[1], src[2], src[3]);
    } else {
      const float* src = g.A + (gr < g.M ? gr : 0) * g.lda;
      va.x = gr < g.M && kk < g.K ? src[kk] : 0.f;
      va.y = gr < g.M && kk + 1 < g.K ? src[kk + 1] : 0.f;
      va.z = gr < g.M && kk + 2 < g.K ? src[kk + 2] : 0.f;
      va.w = gr < g.M && kk + 3 < g.K ? src[kk + 3] : 0.f;
    }
    if constexpr (BS) {   // the f16 planes straight from the pre-split B (L2-resident)
      // columns >= N (their LDS rows are never multiplied) read column N - 1
      const uint4* q = g.b_split + ((int64_t)((k0 + bk) >> 3) * g.N + (stB ? bn : g.N - 1)) * 2;
      bsh = q[0];
      bsl = q[1];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = k0 + bk + j;
        vb[j] = stB && r < g.K ? g.B[(int64_t)r * g.ldb + bn] : 0.f;
      }
    }
  };
  auto put = [&](int buf) {
    uint16_t* pa = nlds + (size_t)buf * (2 * kNHPlaneA + 2 * kNHPlaneB);
    uint16_t* pb = pa + 2 * kNHPlaneA;
    const float a0 = va.x * sa, a1 = va.y * sa, a2 = va.z * sa, a3 = va.w * sa;
    bool ok = fabsf(a0) < 8.f && fabsf(a1) < 8.f && fabsf(a2) < 8.f && fabsf(a3) < 8.f;
    unsigned h0, l0, h1, l1;
    splith(a0, a1, h0, l0);
    splith(a2, a3, h1, l1);
    *reinterpret_cast<uint2*>(pa + ar * kXPitch + ak) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(pa + kNHPlaneA + ar * kXPitch + ak) = make_uint2(l0, l1);
    uint4 bh, bl;
    if constexpr (BS) {
      bh = bsh;
      bl = bsl;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ok = ok && fabsf(vb[2 * q]) < 32768.f && fabsf(vb[2 * q + 1]) < 32768.f;
        unsigned x0, x1;
        splith(vb[2 * q], vb[2 * q + 1], x0, x1);
        reinterpret_cast<unsigned*>(&bh)[q] = x0;
        reinterpret_cast<unsigned*>(&bl)[q] = x1;
      }
    }
    *reinterpret_cast<uint4*>(pb + bn * kXPitch + bk) = bh;
    *reinterpret_cast<uint4*>(pb + kNHPlaneB + bn * kXPitch + bk) = bl;
    bad = bad || !ok;
  };
  f32x16 acc[NW];
#pragma unroll
  for (int u = 0; u < NW; ++u) acc[u] = (f32x16){0.f};
  load(0);
  put(0);
  __syncthreads();
  int it = 0;
  for (int k0 = 0; k0 < g.K; k0 += 16, ++it) {
    const int buf = it & 1;
    const bool more = k0 + 16 < g.K;
    if (more) load(k0 + 16);
    const uint16_t* pa = nlds + (size_t)buf * (2 * kNHPlaneA + 2 * kNHPlaneB);
    const uint16_t* pb = pa + 2 * kNHPlaneA;
    const uint4 ah = *reinterpret_cast<const uint4*>(pa + (32 * wm + c) * kXPitch + 8 * h);
    const uint4 al = *reinterpret_cast<const uint4*>(pa + kNHPlaneA + (32 * wm + c) * kXPitch + 8 * h);
    const uint4 as = f16x8_scale2048(ah);
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int t = wn + 2 * u;
      if (t >= NT) continue;
      const uint4 bh = *reinterpret_cast<const uint4*>(pb + (32 * t + c) * kXPitch + 8 * h);
      const uint4 bl = *reinterpret_cast<const uint4*>(pb + kNHPlaneB + (32 * t + c) * kXPitch + 8 * h);
      acc[u] = mfma_f16(al, bh, acc[u]);   // smallest terms first
      acc[u] = mfma_f16(ah, bl, acc[u]);
      acc[u] = mfma_f16(as, bh, acc[u]);
    }
    if (more) put(buf ^ 1);
    __syncthreads();
  }
  const float unscale = ldexpf(1.f, -(e + 11));
  unsigned mb = 0u;
  // C/D layout: row = (r&3) + 8(r>>2) + 4h (the A rows), col = c
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (m >= g.M) continue;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int t = wn + 2 * u;
      if (t >= NT) continue;
      const int n = 32 * t + c;
      float v = acc[u][r] * unscale;
      if (g.act != nullptr && !(g.act[m * g.ld_act + n] > 0.f)) v *= g.slope;
      g.C[m * g.ldc + n] = v;
      mb = max(mb, abs_bits(v));
    }
  }
  if (bad) atomicOr(g.range_flag, 1);
  // (on a raised flag the fp32 kernel behind this one rewrites C and folds its
  // own max in: the word may then hold the discarded values' max too -- only
  // ever larger, a valid scale for its consumer)
  if (g.c_absmax) block_absmax_to(g.c_absmax, mb, reinterpret_cast<unsigned*>(nlds));
}

template <int NT>
static void launch_gemm_nn(const GemmNNArgs& g, hipStream_t st) {
  // long M: 128-row workgroups, two per CU (<= 128 VGPRs, 54 KB LDS; measured
  // 1.32x faster than one 256-row workgroup per CU at 200 k x 256 x 224); short M
  // (the ~30 k-row colour-branch batches): 64-row workgroups, so the grid still
  // spans the CUs
  // (and NT 5..7 at any M: their 4-way column split over WM = 2's waves is uneven)
  if (g.M >= 256 * 512 || (NT >= 5 && NT <= 7)) {
    hipLaunchKernelGGL((k_gemm_nn<NT, 4>), dim3((unsigned)cdiv(g.M, (int64_t)128)), dim3(512), 0, st, g);
  } else {
    hipLaunchKernelGGL((k_gemm_nn<NT, 2>), dim3((unsigned)cdiv(g.M, (int64_t)64)), dim3(512), 0, st, g);
  }
}

// B of a gemm_nn_h2 pre-split once (nn_b_split): out[k8][n] = (hi, lo) uint4 pairs
// of rows 8 k8 .. 8 k8 + 7 of column n (rows >= K zero) -- the planes every
// workgroup of k_gemm_nn_h2 would otherwise split from the same weights per
// 16-k chunk; an out-of-range entry (|b| >= 2^15, NaN / inf) raises the flag
// (the fp32 kernel behind the h2 call then recomputes C).  Up to 4 matrices.
struct NNSplitJob {
  const float* B;
  int64_t ldb;
  uint4* out;
  int K, N, blk0;
};
struct NNSplitBatch {
  NNSplitJob j[4];
  int n;
  int32_t* flag;
};
__global__ void __launch_bounds__(256) k_nn_b_split(NNSplitBatch B) {
  NNSplitJob J = B.j[0];
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (q < B.n && (int)blockIdx.x >= B.j[q].blk0) J = B.j[q];
  const int i = (blockIdx.x - J.blk0) * 256 + threadIdx.x;
  const int k8n = ((J.K + 15) / 16) * 2;   // 8-row groups (K padded to whole 16-k chunks)
  if (i >= k8n * J.N) return;
  const int k8 = i / J.N, n = i - k8 * J.N;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = 8 * k8 + j;
    v[j] = r < J.K ? J.B[(int64_t)r * J.ldb + n] : 0.f;
  }
  bool ok = true;
  uint4 bh, bl;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ok = ok && fabsf(v[2 * q]) < 32768.f && fabsf(v[2 * q + 1]) < 32768.f;
    unsigned x0, x1;
    splith(v[2 * q], v[2 * q + 1], x0, x1);
    reinterpret_cast<unsigned*>(&bh)[q] = x0;
    reinterpret_cast<unsigned*>(&bl)[q] = x1;
  }
  J.out[(int64_t)i * 2] = bh;
  J.out[(int64_t)i * 2 + 1] = bl;
  if (!ok) atomicOr(B.flag, 1);
}

// The colour branch's first backward product input in one pass
// (pnr_color_dz): dz[r][c] = lrelu'(hc[r][c]) (d_feat[r][1 + c] * (vmask[r] != 0)),
// the torch ops' arithmetic (where(h > 0, x, x * slope) of x = d_feat * vm),
// and max |dz| folded into *absmax (float bits, NaN as 0x7fc00000 > inf).
__global__ void __launch_bounds__(256) k_color_dz(const float* __restrict__ d_feat, int64_t ldf,
                                                  const int32_t* __restrict__ vmask, const float* __restrict__ hc,
                                                  int64_t ldh, int64_t n, int C, float slope, float* __restrict__ dz,
                                                  uint32_t* __restrict__ absmax) {
  __shared__ unsigned red[4];
  unsigned mb = 0u;
  const int c4n = C >> 2;   // float4 columns per row (C % 4 == 0, hc / dz rows 16-B aligned)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * c4n; i += stride) {
    const int64_t r = i / c4n;
    const int c = 4 * (int)(i - r * c4n);
    const float vm = vmask[r] != 0 ? 1.f : 0.f;
    const float* f = d_feat + r * ldf + 1 + c;
    const float4 h = *reinterpret_cast<const float4*>(hc + r * ldh + c);
    const float x0 = f[0] * vm, x1 = f[1] * vm, x2 = f[2] * vm, x3 = f[3] * vm;
    const float4 d = make_float4(h.x > 0.f ? x0 : x0 * slope, h.y > 0.f ? x1 : x1 * slope,
                                 h.z > 0.f ? x2 : x2 * slope, h.w > 0.f ? x3 : x3 * slope);
    *reinterpret_cast<float4*>(dz + r * C + c) = d;
    const float a[4] = {fabsf(d.x), fabsf(d.y), fabsf(d.z), fabsf(d.w)};
#pragma unroll
    for (int q = 0; q < 4; ++q) mb = max(mb, a[q] != a[q] ? 0x7fc00000u : __float_as_uint(a[q]));
  }
  if (absmax) {   // one atomic per workgroup
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mb;
    __syncthreads();
    if (threadIdx.x == 0) {
      mb = max(max(red[0], red[1]), max(red[2], red[3]));
      if (mb) atomicMax(absmax, mb);
    }
  }
}

}  // namespace pnr

using namespace pnr;

int pnr::gemm_nn_run(bool h2, const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int32_t K,
                     int32_t N, const float* act, int64_t ld_act, float slope, float* C, int64_t ldc,
                     const uint32_t* a_absmax, int32_t* range_flag, uint32_t* c_absmax, void* stream,
                     const void* b_split) {
  PNR_CHECK_ARG(!b_split || (h2 && ((uintptr_t)b_split & 15) == 0), "gemm_nn: b_split needs h2 and 16-B alignment");
  PNR_CHECK_ARG(M == 0 || (A && B && C), "gemm_nn: null pointer");
  PNR_CHECK_ARG(M >= 0 && K > 0 && N > 0 && N % 32 == 0 && N <= 32 * kGMaxNT, "gemm_nn: N must be a multiple of 32 "
                "in [32, 256], K > 0");
  PNR_CHECK_ARG(lda >= K && ldb >= N && ldc >= N && (act == nullptr || ld_act >= N), "gemm_nn: bad leading dimensions");
  if (M == 0) return PNR_OK;
  GemmNNArgs g;
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.act = act;
  g.ld_act = ld_act;
  g.M = M;
  g.K = K;
  g.N = N;
  g.slope = slope;
  g.a_absmax = a_absmax;
  g.range_flag = range_flag;
  g.c_absmax = c_absmax;
  g.run_if = nullptr;
  g.b_split = static_cast<const uint4*>(b_split);
  hipStream_t st = as_stream(stream);
  if (h2) {
    static bool attr = false;
    if (!attr) {
#define PNR_NNH2_ATTR(T)                                                                                  \
  PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_nn_h2<T, false>),                   \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kNHLds));             \
  PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_nn_h2<T, true>),                    \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kNHLds));
      PNR_NNH2_ATTR(1) PNR_NNH2_ATTR(2) PNR_NNH2_ATTR(3) PNR_NNH2_ATTR(4)
      PNR_NNH2_ATTR(5) PNR_NNH2_ATTR(6) PNR_NNH2_ATTR(7) PNR_NNH2_ATTR(8)
#undef PNR_NNH2_ATTR
      attr = true;
    }
    const dim3 grid((unsigned)cdiv(M, (int64_t)kNHRows));
#define PNR_NNH2_GO(T)                                                                        \
  if (g.b_split) hipLaunchKernelGGL((k_gemm_nn_h2<T, true>), grid, dim3(512), kNHLds, st, g); \
  else hipLaunchKernelGGL((k_gemm_nn_h2<T, false>), grid, dim3(512), kNHLds, st, g);
    switch (N / 32) {
      case 1: PNR_NNH2_GO(1) break;
      case 2: PNR_NNH2_GO(2) break;
      case 3: PNR_NNH2_GO(3) break;
      case 4: PNR_NNH2_GO(4) break;
      case 5: PNR_NNH2_GO(5) break;
      case 6: PNR_NNH2_GO(6) break;
      case 7: PNR_NNH2_GO(7) break;
      default: PNR_NNH2_GO(8) break;
    }
#undef PNR_NNH2_GO
    PNR_LAUNCH_CHECK();
    g.run_if = range_flag;   // the fp32 kernel below recomputes C only when the flag is up
  }
  switch (N / 32) {
    case 1: launch_gemm_nn<1>(g, st); break;
    case 2: launch_gemm_nn<2>(g, st); break;
    case 3: launch_gemm_nn<3>(g, st); break;
    case 4: launch_gemm_nn<4>(g, st); break;
    case 5: launch_gemm_nn<5>(g, st); break;
    case 6: launch_gemm_nn<6>(g, st); break;
    case 7: launch_gemm_nn<7>(g, st); break;
    default: launch_gemm_nn<8>(g, st); break;
  }
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_gemm_nn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int32_t K,
                           int32_t N, const float* act, int64_t ld_act, float slope, float* C, int64_t ldc,
                           void* stream) {
  return gemm_nn_run(false, A, lda, B, ldb, M, K, N, act, ld_act, slope, C, ldc, nullptr, nullptr, nullptr, stream,
                     nullptr);
}

extern "C" int pnr_gemm_nn_h2(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int32_t K,
                              int32_t N, const float* act, int64_t ld_act, float slope, float* C, int64_t ldc,
                              const uint32_t* a_absmax, int32_t* range_flag, void* stream) {
  PNR_CHECK_ARG(a_absmax && range_flag, "gemm_nn_h2: a_absmax and range_flag required");
  return gemm_nn_run(true, A, lda, B, ldb, M, K, N, act, ld_act, slope, C, ldc, a_absmax, range_flag, nullptr,
                     stream, nullptr);
}


extern "C" int pnr_gemm_tn_scratch_bytes(int64_t K, int32_t M, int32_t N, size_t* out) {
  PNR_CHECK_ARG(out && K >= 0 && M > 0 && N > 0, "gemm_tn_scratch_bytes: bad args");
  *out = gemm_scratch(K, M, N);
  return PNR_OK;
}

size_t pnr::nn_b_split_bytes(int K, int N) { return (size_t)((K + 15) / 16) * 2 * N * 32; }

int pnr::nn_b_split(int n, const float* const* B, const int64_t* ldb, const int* K, const int* N, void* const* out,
                    int32_t* flag, void* stream) {
  PNR_CHECK_ARG(n >= 1 && n <= 4 && flag, "nn_b_split: 1..4 matrices and a flag");
  NNSplitBatch b = {};
  b.n = n;
  b.flag = flag;
  int blocks = 0;
  for (int q = 0; q < n; ++q) {
    PNR_CHECK_ARG(B[q] && out[q] && K[q] > 0 && N[q] > 0 && ldb[q] >= N[q] && ((uintptr_t)out[q] & 15) == 0,
                  "nn_b_split: bad matrix %d", q);
    b.j[q] = {B[q], ldb[q], static_cast<uint4*>(out[q]), K[q], N[q], blocks};
    blocks += (int)cdiv((int64_t)((K[q] + 15) / 16) * 2 * N[q], 256);
  }
  hipLaunchKernelGGL(k_nn_b_split, dim3(blocks), dim3(256), 0, as_stream(stream), b);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

int pnr::gemm_tn_run(int mode, const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M, int32_t N,
                float* C, int64_t ldc, int32_t ncols, float* colsum_a, void* scratch, size_t scratch_bytes,
                void* stream, const uint32_t* a_absmax, int32_t* range_flag) {
  const bool x3 = mode == 1, h2 = mode == 2;
  PNR_CHECK_ARG(C && scratch && (K == 0 || (A && B)), "gemm_tn: null pointer");
  PNR_CHECK_ARG(ncols >= 1 && ncols <= N && ldc >= ncols, "gemm_tn: bad output slice (ldc %lld, ncols %d)",
                (long long)ldc, ncols);
  PNR_CHECK_ARG(M > 0 && N > 0 && M % 32 == 0 && N % 32 == 0 && M <= 32 * kGWaves && N <= 32 * kGMaxNT,
                "gemm_tn: M, N must be multiples of 32 in [32, 256]");
  PNR_CHECK_ARG(lda >= M && ldb >= N && K >= 0, "gemm_tn: bad leading dimensions");
  PNR_CHECK_ARG(((uintptr_t)scratch & 15) == 0 && ((ldc == N && ncols == N) ? ((uintptr_t)C & 15) == 0 : true) &&
                    ((uintptr_t)colsum_a & 15) == 0,
                "gemm_tn: 16-B aligned scratch, C and colsum_a required");
  PNR_CHECK_ARG(scratch_bytes >= gemm_scratch(K, M, N), "gemm_tn: scratch too small");
  hipStream_t st = as_stream(stream);
  if (K == 0) {
    PNR_HIP(hipMemset2DAsync(C, (size_t)ldc * sizeof(float), 0, (size_t)ncols * sizeof(float), (size_t)M, st));
    if (colsum_a) PNR_HIP(hipMemsetAsync(colsum_a, 0, (size_t)M * sizeof(float), st));
    return PNR_OK;
  }
  int ns;
  int64_t kc;
  gemm_plan(K, &ns, &kc);
  GemmArgs g;
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.K = K;
  g.M = M;
  g.N = N;
  g.kchunk = kc;
  g.part = static_cast<float*>(scratch);
  g.colsum = colsum_a != nullptr;
  g.a_absmax = a_absmax;
  g.range_flag = range_flag;
  static bool attr = false;
  if (!attr && (x3 || h2)) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_tn_x3_part),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kXLds));
    attr = true;
  }
  if (h2) {
    hipLaunchKernelGGL(k_gemm_tn_h2_part, dim3(ns), dim3(512), 0, st, g);
  } else if (x3) {
    hipLaunchKernelGGL(k_gemm_tn_x3_part, dim3(ns), dim3(512), kXLds, st, g);
  } else {
    hipLaunchKernelGGL(k_gemm_tn_part, dim3(ns), dim3(64 * kGWaves), 0, st, g);
  }
  PNR_LAUNCH_CHECK();
  // two-level ordered reduction: groups of kGGroup splits, then the groups
  const int64_t stride = (int64_t)M * N + M;   // multiple of 4 (M % 32 == 0)
  const int64_t n4 = stride / 4;
  const int ngrp = (int)cdiv(ns, kGGroup);
  float* lvl1 = g.part + (size_t)ns * stride;
  hipLaunchKernelGGL(k_reduce_splits, dim3(grid_for(n4, 256, 256), ngrp), dim3(256), 0, st, g.part, n4, ns, kGGroup,
                     lvl1);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_reduce_final, dim3(grid_for(n4, 256, 256)), dim3(256), 0, st, lvl1, n4, ngrp,
                     (int64_t)M * N / 4, C, colsum_a, N / 4, ldc, ncols);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M,
                           int32_t N, float* C, float* colsum_a, void* scratch, size_t scratch_bytes,
                           void* stream) {
  return gemm_tn_run(0, A, lda, B, ldb, K, M, N, C, N, N, colsum_a, scratch, scratch_bytes, stream, nullptr, nullptr);
}

extern "C" int pnr_gemm_tn_x3(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M,
                              int32_t N, float* C, float* colsum_a, void* scratch, size_t scratch_bytes,
                              void* stream) {
  return gemm_tn_run(1, A, lda, B, ldb, K, M, N, C, N, N, colsum_a, scratch, scratch_bytes, stream, nullptr, nullptr);
}

extern "C" int pnr_gemm_tn_h2(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K, int32_t M,
                              int32_t N, float* C, float* colsum_a, const uint32_t* a_absmax, int32_t* range_flag,
                              void* scratch, size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(a_absmax && range_flag, "gemm_tn_h2: a_absmax and range_flag required");
  return gemm_tn_run(2, A, lda, B, ldb, K, M, N, C, N, N, colsum_a, scratch, scratch_bytes, stream, a_absmax,
                     range_flag);
}

extern "C" int pnr_color_dz(const float* d_feat, int64_t ld_feat, const int32_t* vmask, const float* hc, int64_t ld_hc,
                            int64_t n, int32_t C, float slope, float* dz, uint32_t* absmax, void* stream) {
  PNR_CHECK_ARG(n >= 0 && C >= 4 && C % 4 == 0 && ld_feat >= C + 1 && ld_hc >= C && ld_hc % 4 == 0 &&
                    (n == 0 || (d_feat && vmask && hc && dz)),
                "color_dz: bad args (n %lld, C %d, ld_hc %lld)", (long long)n, C, (long long)ld_hc);
  PNR_CHECK_ARG((((uintptr_t)hc | (uintptr_t)dz) & 15) == 0, "color_dz: hc and dz must be 16-B aligned");
  if (n == 0) return PNR_OK;
  hipLaunchKernelGGL(k_color_dz, dim3(grid_for(n * (C / 4), 256, 256)), dim3(256), 0, as_stream(stream), d_feat,
                     ld_feat, vmask, hc, ld_hc, n, C, slope, dz, absmax);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_absmax_scratch_floats(int64_t* out) {
  PNR_CHECK_ARG(out, "absmax_scratch_floats: null");
  *out = kAbsBlocks;
  return PNR_OK;
}

extern "C" int pnr_absmax(const float* x, int64_t n, float* partials, uint32_t* out_bits, void* stream) {
  PNR_CHECK_ARG(partials && out_bits && n >= 0 && (x || n == 0), "absmax: bad args");
  hipStream_t st = as_stream(stream);
  const int nb = (int)(n > 0 ? (cdiv(n, 4 * 256) < kAbsBlocks ? cdiv(n, 4 * 256) : kAbsBlocks) : 1);
  hipLaunchKernelGGL(k_absmax_part, dim3(nb), dim3(256), 0, st, x, n, partials);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_absmax_final, dim3(1), dim3(256), 0, st, partials, nb, out_bits);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
