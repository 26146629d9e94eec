// The finetune step's backward through the aggregator as ONE host call
// (pnr_aggregate_bwd_step_h2): train.py's AggregateFn.backward for the fp32h2
// training precision -- the colour branch, the per-pair dX chain, the per-point
// sums, every weight gradient and block1.0's point half -- enqueued from C++
// instead of ~60 Python-level torch / ctypes calls (the
// step was bound by its host issue, 2.4 ms of Python per backward).  Same
// kernels and arithmetic as the Python sequence it replaces, except two
// helpers it needs in native form:
//   * pnr_group_pairs: the pairs grouped by point row in pair order -- the
//     (prow_sorted, pair_of) of torch.sort(prow, stable=True) over the pairs
//     that reference a point (the empty ones, -1, go to the END here instead of
//     the front; pnr_pairs_to_points(_ex) skips them either way).  A counting
//     sort: per-key counts, an exclusive scan, an atomic fill, then each key's
//     few entries sorted back into pair order (one thread per key; keys with
//     more than 32 entries by a workgroup, rank by comparison) -- deterministic.
//   * the alpha_branch.0 gradient as a deterministic weighted column sum
//     (d wa[c] = sum_pairs dpa h4[:, c], d ba = sum dpa) instead of an M = 1 GEMM
//     padded to 32 rows.
#include "agg_common.h"

namespace pnr {

// ---------------------------------------------------------------- pair grouping
__global__ void __launch_bounds__(256) k_grp_count(const int32_t* __restrict__ prow, int64_t m,
                                                   const int32_t* __restrict__ map, int32_t* __restrict__ cnt) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < m; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t pr = prow[p];
    if (pr >= 0) atomicAdd(cnt + (map ? map[pr] : pr), 1);
  }
}

__global__ void __launch_bounds__(256) k_grp_fill(const int32_t* __restrict__ prow, int64_t m,
                                                  const int32_t* __restrict__ map, const int32_t* __restrict__ off,
                                                  int32_t* __restrict__ cnt, int32_t* __restrict__ prow_sorted,
                                                  int32_t* __restrict__ pair_of) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < m; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t pr = prow[p];
    if (pr < 0) continue;
    const int32_t u = map ? map[pr] : pr;
    const int32_t pos = off[u] + atomicSub(cnt + u, 1) - 1;
    prow_sorted[pos] = pr;
    pair_of[pos] = (int32_t)p;
  }
}

constexpr int kGrpSmall = 32;   // entries a single thread sorts (insertion sort)

// each key's entries back into pair order; keys with more entries are listed
// for k_grp_sort_big; the tail past the referenced pairs gets key -1
__global__ void __launch_bounds__(256) k_grp_sort(const int32_t* __restrict__ off, int64_t nk, int64_t m,
                                                  int32_t* __restrict__ pair_of, int32_t* __restrict__ prow_sorted,
                                                  int32_t* __restrict__ big, int32_t* __restrict__ n_big) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t first = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t u = first; u < nk; u += stride) {
    const int32_t b = off[u], e = off[u + 1];
    const int L = e - b;
    if (L <= 1) continue;
    if (L > kGrpSmall) {
      big[atomicAdd(n_big, 1)] = (int32_t)u;
      continue;
    }
    int32_t* v = pair_of + b;
    for (int i = 1; i < L; ++i) {
      const int32_t x = v[i];
      int j = i - 1;
      while (j >= 0 && v[j] > x) {
        v[j + 1] = v[j];
        --j;
      }
      v[j + 1] = x;
    }
  }
  for (int64_t i = off[nk] + first; i < m; i += stride) {
    prow_sorted[i] = -1;
    pair_of[i] = 0;
  }
}

// one workgroup per listed key: rank of each entry = entries below it (unique
// pair indices), scattered through tmp
__global__ void __launch_bounds__(256) k_grp_sort_big(const int32_t* __restrict__ off, const int32_t* __restrict__ big,
                                                      const int32_t* __restrict__ n_big, int32_t* __restrict__ pair_of,
                                                      int32_t* __restrict__ tmp) {
  const int nb = *n_big;
  for (int q = blockIdx.x; q < nb; q += gridDim.x) {
    const int32_t u = big[q];
    const int32_t b = off[u], L = off[u + 1] - b;
    const int32_t* v = pair_of + b;
    for (int i = threadIdx.x; i < L; i += blockDim.x) {
      const int32_t x = v[i];
      int32_t r = 0;
      for (int j = 0; j < L; ++j) r += v[j] < x ? 1 : 0;
      tmp[b + r] = x;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < L; i += blockDim.x) pair_of[b + i] = tmp[b + i];
    __syncthreads();
  }
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t group_scratch(int64_t m, int64_t nk) {
  return a256((size_t)(nk + 1) * 4) /*cnt + n_big*/ + a256((size_t)(nk + 1) * 4) /*off*/ +
         a256(scan_scratch_bytes(nk)) + a256((size_t)(nk > 0 ? nk : 1) * 4) /*big*/ +
         a256((size_t)(m > 0 ? m : 1) * 4) /*tmp*/;
}

// cnt_zeroed: the caller already zeroed the scratch's first nk + 1 words (the counts)
int group_pairs(const int32_t* prow, int64_t m, const int32_t* map, int64_t nk, int32_t* prow_sorted,
                int32_t* pair_of, void* scratch, size_t bytes, hipStream_t st, const int32_t** off_out = nullptr,
                bool cnt_zeroed = false) {
  PNR_CHECK_ARG(prow_sorted && pair_of && scratch && (m == 0 || prow) && m >= 0 && nk >= 1 && m < (1ll << 31) &&
                    nk < (1ll << 31),
                "group_pairs: bad args (m %lld, keys %lld)", (long long)m, (long long)nk);
  PNR_CHECK_ARG(bytes >= group_scratch(m, nk), "group_pairs: scratch too small (%zu < %zu)", bytes,
                group_scratch(m, nk));
  char* sp = static_cast<char*>(scratch);
  if (m == 0) {   // no pairs: every key empty
    int32_t* off0 = reinterpret_cast<int32_t*>(sp + a256((size_t)(nk + 1) * 4));
    PNR_HIP(hipMemsetAsync(off0, 0, (size_t)(nk + 1) * 4, st));
    if (off_out) *off_out = off0;
    return PNR_OK;
  }
  int32_t* cnt = reinterpret_cast<int32_t*>(sp);   // [nk] counts, then n_big
  int32_t* n_big = cnt + nk;
  sp += a256((size_t)(nk + 1) * 4);
  int32_t* off = reinterpret_cast<int32_t*>(sp);
  sp += a256((size_t)(nk + 1) * 4);
  void* scan_s = sp;
  sp += a256(scan_scratch_bytes(nk));
  int32_t* big = reinterpret_cast<int32_t*>(sp);
  sp += a256((size_t)nk * 4);
  int32_t* tmp = reinterpret_cast<int32_t*>(sp);
  if (off_out) *off_out = off;
  if (!cnt_zeroed) PNR_HIP(hipMemsetAsync(cnt, 0, (size_t)(nk + 1) * 4, st));
  const unsigned gm = grid_for(m, 256, 2048), gk = grid_for(nk, 256, 2048);
  hipLaunchKernelGGL(k_grp_count, dim3(gm), dim3(256), 0, st, prow, m, map, cnt);
  PNR_LAUNCH_CHECK();
  int rc = exclusive_scan(cnt, nk, nullptr, off, nk + 1, nullptr, scan_s, scan_scratch_bytes(nk), st);
  if (rc) return rc;
  hipLaunchKernelGGL(k_grp_fill, dim3(gm), dim3(256), 0, st, prow, m, map, off, cnt, prow_sorted, pair_of);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_grp_sort, dim3(gk > gm ? gk : gm), dim3(256), 0, st, off, nk, m, pair_of, prow_sorted, big,
                     n_big);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_grp_sort_big, dim3(256), dim3(256), 0, st, off, big, n_big, pair_of, tmp);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// The per-point sums over the groups (the step's pnr_pairs_to_points_ex): 16
// lanes per used point u (4 points per wave), lane l the floats 16 l .. 16 l + 15
// of the 256-wide rows (four float4 loads in flight per pair): d_p1[u] = sum of
// dz1 over u's pairs in pair order (zero for a point without pairs), lanes 0..5
// the g_pair sums -> d_color / d_dir of point used[u] (Rw_p^T for d dir), max
// |d_p1| folded into *absmax.  Same sums in the same order as
// k_pairs_to_points_ex: the same bits.
__global__ void __launch_bounds__(256) k_points_from_groups(const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ pair_of, int64_t nk,
                                                            const int32_t* __restrict__ used,
                                                            const float* __restrict__ dz1, float* __restrict__ d_p1,
                                                            uint32_t* __restrict__ absmax,
                                                            const float* __restrict__ g_pair,
                                                            const float* __restrict__ rw_uniform,
                                                            const float* __restrict__ rw_pp,
                                                            float* __restrict__ d_color, float* __restrict__ d_dir) {
  __shared__ unsigned red[4];
  constexpr int kLp = 16, kQ = 64 / kLp;   // lanes per point, float4 per lane (8: 133 us, 16: 115 us)
  const int lane = threadIdx.x & 63, l = lane & (kLp - 1), grp = lane / kLp;
  unsigned mb = 0u;
  const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / kLp);
  for (int64_t u = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kLp; u < nk; u += gstride) {
    const int32_t b = off[u], e = off[u + 1];
    float4 s[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) s[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    float ge = 0.f;
    for (int32_t j = b; j < e; ++j) {
      const int64_t pq = pair_of[j];
      const float4* row = reinterpret_cast<const float4*>(dz1 + pq * 256) + kQ * l;
      float4 v[kQ];
#pragma unroll
      for (int q = 0; q < kQ; ++q) v[q] = row[q];
      if (l < 6) ge += g_pair[pq * 8 + l];
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        if (j == b) {
          s[q] = v[q];
        } else {
          s[q].x += v[q].x;
          s[q].y += v[q].y;
          s[q].z += v[q].z;
          s[q].w += v[q].w;
        }
      }
    }
    float4* o = reinterpret_cast<float4*>(d_p1 + u * 256) + kQ * l;
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      o[q] = s[q];
      mb = max(max(mb, max(__float_as_uint(fabsf(s[q].x)), __float_as_uint(fabsf(s[q].y)))),
               max(__float_as_uint(fabsf(s[q].z)), __float_as_uint(fabsf(s[q].w))));
    }
    const int src = grp * kLp;
    const float g3 = __shfl(ge, src + 3), g4 = __shfl(ge, src + 4), g5 = __shfl(ge, src + 5);
    if (e > b) {
      const int32_t pr = used[u];
      if (l < 3) {
        if (d_color) d_color[(int64_t)pr * 3 + l] = ge;
        if (d_dir) {   // d dir_a = sum_j Rw[j][a] gd_j
          const float* R = rw_pp ? rw_pp + (int64_t)pr * 9 : rw_uniform;
          const float r0 = R ? R[l] : (l == 0 ? 1.f : 0.f);
          const float r1 = R ? R[3 + l] : (l == 1 ? 1.f : 0.f);
          const float r2 = R ? R[6 + l] : (l == 2 ? 1.f : 0.f);
          d_dir[(int64_t)pr * 3 + l] = r0 * g3 + r1 * g4 + r2 * g5;
        }
      }
    }
  }
  if (absmax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
    if (lane == 0) red[threadIdx.x >> 6] = mb;
    __syncthreads();
    if (threadIdx.x == 0) {
      mb = max(max(red[0], red[1]), max(red[2], red[3]));
      if (mb) atomicMax(absmax, mb);
    }
  }
}

// ---------------------------------------------------------------- alpha gradient
// part[b][c] = sum over block b's rows r of dpa[r] h4[r][c] (c < 256), part[b][256]
// = sum dpa[r]; then out_w[c] / out_b = the blocks' partials in block order.
constexpr int kAcBlocks = 1024;
__global__ void __launch_bounds__(256) k_alpha_colsum_part(const float* __restrict__ dpa, const float* __restrict__ h4,
                                                           int64_t m, float* __restrict__ part) {
  const int c = threadIdx.x;
  const int64_t rows = cdiv(m, (int64_t)gridDim.x);
  const int64_t r0 = blockIdx.x * rows, r1 = r0 + rows < m ? r0 + rows : m;
  float acc = 0.f, sb = 0.f;
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {
    const float d0 = dpa[r], d1 = dpa[r + 1], d2 = dpa[r + 2], d3 = dpa[r + 3];
    const float x0 = h4[r * 256 + c], x1 = h4[(r + 1) * 256 + c], x2 = h4[(r + 2) * 256 + c],
                x3 = h4[(r + 3) * 256 + c];
    acc += d0 * x0;
    acc += d1 * x1;
    acc += d2 * x2;
    acc += d3 * x3;
    sb += d0;
    sb += d1;
    sb += d2;
    sb += d3;
  }
  for (; r < r1; ++r) {
    acc += dpa[r] * h4[r * 256 + c];
    sb += dpa[r];
  }
  part[blockIdx.x * 257 + c] = acc;
  if (c == 0) part[blockIdx.x * 257 + 256] = sb;
}

// one workgroup per column c (257: the 256 weights, then the bias): thread t sums
// partials t, t + 256, ... in order, then a fixed-shape LDS tree (deterministic)
__global__ void __launch_bounds__(256) k_alpha_colsum_final(const float* __restrict__ part, int nb,
                                                            float* __restrict__ out_w, float* __restrict__ out_b) {
  __shared__ float red[256];
  const int c = blockIdx.x, t = threadIdx.x;
  float s = 0.f;
  for (int b = t; b < nb; b += 256) s += part[b * 257 + c];
  red[t] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) {
    if (c < 256) out_w[c] = red[0];
    else out_b[0] = red[0];
  }
}

// The step's preparation in one launch: zero up to six buffers (the point-table
// gradients d emb, d colour, d dir, d conf -- rows the backward does not write
// stay zero -- the step's absmax / flag words and the grouping's counts) and
// gather block3.0's extras columns W3[:, 256:263] into a [256][7] table.
constexpr int kPrepBufs = 6;
struct StepPrep {
  float* p[kPrepBufs];
  int64_t n4[kPrepBufs];    // float4 count (16-B aligned buffers)
  int64_t tail[kPrepBufs];  // 4-byte words past the last whole float4
  float* w3e;
  const float* w3;          // [256][263]
};
__global__ void __launch_bounds__(256) k_step_prep(StepPrep z) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t first = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
#pragma unroll
  for (int q = 0; q < kPrepBufs; ++q) {
    if (!z.p[q]) continue;
    float4* d = reinterpret_cast<float4*>(z.p[q]);
    for (int64_t i = first; i < z.n4[q]; i += stride) d[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = first; i < z.tail[q]; i += stride) z.p[q][4 * z.n4[q] + i] = 0.f;
  }
  for (int64_t i = first; i < 256 * 7; i += stride) z.w3e[i] = z.w3[(i / 7) * 263 + 256 + i % 7];
}

// [n, 24] -> [n, 32] rows (zero padding: pnr_gemm_tn's N multiple of 32)
__global__ void __launch_bounds__(256) k_pad_rows32(const float* __restrict__ src, int64_t n, int cols,
                                                    float* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * 32; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i >> 5;
    const int c = (int)(i & 31);
    dst[i] = c < cols ? src[r * cols + c] : 0.f;
  }
}

// ---------------------------------------------------------------- the step's scratch
struct StepPlan {
  size_t words, dzc3, dzc2, dzc1, d_hid, vpe32, dz[4], dpa, d_p1, g_pair, prow_sorted, pair_of, grp, x1, dx1, packs,
      pscale, w3e, gemm, absp, acp, bsplit[4], total;
  size_t gemm_bytes, grp_bytes;
};

static StepPlan plan_step(int64_t n, int64_t n_used) {
  StepPlan p{};
  const int64_t m = n * kKN, nu = n_used > 0 ? n_used : 1, nn = n > 0 ? n : 1, mm = m > 0 ? m : 1;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += a256(bytes);
    return at;
  };
  p.words = take(64);
  p.dzc3 = take((size_t)nn * 128 * 4);
  p.dzc2 = take((size_t)nn * 128 * 4);
  p.dzc1 = take((size_t)nn * 128 * 4);
  p.d_hid = take((size_t)nn * 256 * 4);
  p.vpe32 = take((size_t)nn * 32 * 4);
  for (int i = 0; i < 4; ++i) p.dz[i] = take((size_t)mm * 256 * 4);
  p.dpa = take((size_t)mm * 4);
  p.d_p1 = take((size_t)nu * 256 * 4);
  p.g_pair = take((size_t)mm * 8 * 4);
  p.prow_sorted = take((size_t)mm * 4);
  p.pair_of = take((size_t)mm * 4);
  p.grp_bytes = group_scratch(m, nu);
  p.grp = take(p.grp_bytes);
  p.x1 = take((size_t)nu * 224 * 4);
  p.dx1 = take((size_t)nu * 224 * 4);
  p.packs = take((size_t)3 * (16 + 3) * 2048 * 8);
  p.pscale = take(16);
  p.w3e = take(256 * 7 * 4);
  size_t g = 0;
  const int64_t shapes[][3] = {{n, 128, 128}, {n, 128, 256}, {n, 128, 32}, {m, 256, 256}, {m, 256, 32},
                               {m, 256, 64},  {n_used, 256, 224}};
  for (const auto& sh : shapes) {
    const size_t b = gemm_scratch(sh[0] > 0 ? sh[0] : 1, (int)sh[1], (int)sh[2]);
    g = b > g ? b : g;
  }
  p.gemm_bytes = g;
  p.gemm = take(g);
  int64_t nabs = 0;
  (void)pnr_absmax_scratch_floats(&nabs);
  p.absp = take((size_t)nabs * 4);
  p.acp = take((size_t)kAcBlocks * 257 * 4);
  const int kn[4][2] = {{128, 128}, {128, 128}, {128, 256}, {256, 224}};   // the four gemm_nn B operands
  for (int i = 0; i < 4; ++i) p.bsplit[i] = take(nn_b_split_bytes(kn[i][0], kn[i][1]));
  p.total = o;
  return p;
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_group_pairs_scratch_bytes(int64_t m, int64_t n_keys, size_t* out) {
  PNR_CHECK_ARG(out && m >= 0 && n_keys >= 1, "group_pairs_scratch_bytes: bad args");
  *out = group_scratch(m, n_keys);
  return PNR_OK;
}

extern "C" int pnr_group_pairs(const int32_t* prow, int64_t m, const int32_t* key_map, int64_t n_keys,
                               int32_t* prow_sorted, int32_t* pair_of, void* scratch, size_t scratch_bytes,
                               void* stream) {
  return group_pairs(prow, m, key_map, n_keys, prow_sorted, pair_of, scratch, scratch_bytes, as_stream(stream));
}

extern "C" int pnr_alpha_colsum(const float* dpa, const float* h4, int64_t m, float* out_w, float* out_b,
                                float* partials, void* stream) {
  PNR_CHECK_ARG(out_w && out_b && partials && m >= 0 && (m == 0 || (dpa && h4)), "alpha_colsum: bad args");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_alpha_colsum_part, dim3(kAcBlocks), dim3(256), 0, st, dpa, h4, m, partials);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_alpha_colsum_final, dim3(257), dim3(256), 0, st, partials, kAcBlocks, out_w, out_b);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_alpha_colsum_scratch_floats(int64_t* out) {
  PNR_CHECK_ARG(out, "alpha_colsum_scratch_floats: null");
  *out = (int64_t)kAcBlocks * 257;
  return PNR_OK;
}

extern "C" int pnr_aggregate_bwd_step_h2_scratch_bytes(int64_t n, int64_t n_used, size_t* out) {
  PNR_CHECK_ARG(out && n >= 0 && n_used >= 0, "aggregate_bwd_step_h2_scratch_bytes: bad args");
  *out = plan_step(n, n_used).total;
  return PNR_OK;
}

extern "C" int pnr_aggregate_bwd_step_h2(const pnr_points* pts, const pnr_samples* s, const pnr_mlp* w,
                                         const pnr_agg_params* prm, const pnr_agg_saved* saved, const float* d_feat,
                                         int64_t n, int64_t n_used, const pnr_agg_grads* out, void* scratch,
                                         size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(pts && s && w && prm && saved && out && scratch && n >= 0 && n_used >= 0,
                "aggregate_bwd_step_h2: null pointer or negative count");
  PNR_CHECK_ARG(pts->used && pts->used_map && pts->emb, "aggregate_bwd_step_h2: the used-point list is required");
  PNR_CHECK_ARG(saved->dz_absmax && saved->prow && saved->h1 && saved->hid && saved->vpe && saved->hc1 &&
                    saved->hc2 && saved->hc3 && saved->vmask && saved->pe5 && saved->x3e,
                "aggregate_bwd_step_h2: incomplete saved activations");
  for (int i = 0; i < 16; ++i) PNR_CHECK_ARG(prm->p[i] && out->g[i], "aggregate_bwd_step_h2: null parameter %d", i);
  PNR_CHECK_ARG(out->d_emb, "aggregate_bwd_step_h2: d_emb required");
  const StepPlan P = plan_step(n, n_used);
  PNR_CHECK_ARG(scratch_bytes >= P.total && ((uintptr_t)scratch & 255) == 0,
                "aggregate_bwd_step_h2: scratch too small or unaligned (%zu < %zu)", scratch_bytes, P.total);
  hipStream_t st = as_stream(stream);
  void* sv = stream;
  const int64_t N = pts->n;
  const float* const* W = prm->p;
  float* const* G = out->g;
  static const int64_t kParamNumel[16] = {256 * 284, 256, 256 * 256, 256, 256 * 263, 256, 256 * 256, 256,
                                          256,       1,   128 * 280, 128, 128 * 128, 128, 128 * 128, 128};
  if (n == 0) {
    for (float* p : {out->d_emb, out->d_color, out->d_dir, out->d_conf})
      if (p) PNR_HIP(hipMemsetAsync(p, 0, (size_t)N * (p == out->d_emb ? 32 : p == out->d_conf ? 1 : 3) * 4, st));
    for (int i = 0; i < 16; ++i) PNR_HIP(hipMemsetAsync(G[i], 0, (size_t)kParamNumel[i] * 4, st));
    return PNR_OK;
  }
  char* b = static_cast<char*>(scratch);
  auto F = [&](size_t off) { return reinterpret_cast<float*>(b + off); };
  uint32_t* words = reinterpret_cast<uint32_t*>(b + P.words);   // [0] range flag, [1..3] colour-branch maxima
  int32_t* flag = reinterpret_cast<int32_t*>(words);
  const int64_t m = n * kKN;
  const float slope = w->neg_slope;
  int rc;
#define PNR_TRY(x)          \
  do {                      \
    if ((rc = (x))) return rc; \
  } while (0)
  const int64_t nk = n_used > 0 ? n_used : 1;
  float* w3e = F(P.w3e);
  {   // zero fills (gradients, words, the grouping's counts) + the W3 extras gather: one launch
    StepPrep z = {};
    float* ps[kPrepBufs] = {out->d_emb, out->d_color, out->d_dir, out->d_conf, reinterpret_cast<float*>(words),
                            reinterpret_cast<float*>(b + P.grp)};
    const int64_t ns[kPrepBufs] = {N * 32, N * 3, N * 3, N, 16, nk + 1};
    for (int q = 0; q < kPrepBufs; ++q) {
      z.p[q] = ps[q];
      const bool al = ps[q] && ((uintptr_t)ps[q] & 15) == 0;
      z.n4[q] = al ? ns[q] / 4 : 0;
      z.tail[q] = ps[q] ? ns[q] - 4 * z.n4[q] : 0;
    }
    z.w3e = w3e;
    z.w3 = W[4];
    hipLaunchKernelGGL(k_step_prep, dim3(grid_for(N * 8, 256, 8192)), dim3(256), 0, st, z);
    PNR_LAUNCH_CHECK();
  }
  // the four data-gradient products' B operands (colour_branch.4 / .2 / .0[:, :256],
  // block1.0[:, :224]) split into f16 planes once, one launch
  {
    const float* bs[4] = {W[14], W[12], W[10], W[0]};
    const int64_t lds[4] = {128, 128, 280, 284};
    const int ks[4] = {128, 128, 128, 256}, ns[4] = {128, 128, 256, 224};
    void* outs[4] = {b + P.bsplit[0], b + P.bsplit[1], b + P.bsplit[2], b + P.bsplit[3]};
    PNR_TRY(nn_b_split(4, bs, lds, ks, ns, outs, flag, sv));
  }
  // ---- colour branch (color_branch.{0,2,4}: 280 -> 128 -> 128 -> 128, LeakyReLU each)
  float *dzc3 = F(P.dzc3), *dzc2 = F(P.dzc2), *dzc1 = F(P.dzc1), *d_hid = F(P.d_hid);
  PNR_TRY(pnr_color_dz(d_feat, kC + 1, saved->vmask, saved->hc3, 128, n, 128, slope, dzc3, words + 1, sv));
  PNR_TRY(gemm_tn_run(2, dzc3, 128, saved->hc2, 128, n, 128, 128, G[14], 128, 128, G[15], F(P.gemm), P.gemm_bytes,
                      sv, words + 1, flag));
  PNR_TRY(gemm_nn_run(true, dzc3, 128, W[14], 128, n, 128, 128, saved->hc2, 128, slope, dzc2, 128, words + 1, flag,
                      words + 2, sv, b + P.bsplit[0]));
  PNR_TRY(gemm_tn_run(2, dzc2, 128, saved->hc1, 128, n, 128, 128, G[12], 128, 128, G[13], F(P.gemm), P.gemm_bytes,
                      sv, words + 2, flag));
  PNR_TRY(gemm_nn_run(true, dzc2, 128, W[12], 128, n, 128, 128, saved->hc1, 128, slope, dzc1, 128, words + 2, flag,
                      words + 3, sv, b + P.bsplit[1]));
  PNR_TRY(gemm_tn_run(2, dzc1, 128, saved->hid, 256, n, 128, 256, G[10], 280, 256, G[11], F(P.gemm), P.gemm_bytes,
                      sv, words + 3, flag));
  float* vpe32 = F(P.vpe32);
  hipLaunchKernelGGL(k_pad_rows32, dim3(grid_for(n * 32, 256, 1024)), dim3(256), 0, st, saved->vpe, n, 24, vpe32);
  PNR_LAUNCH_CHECK();
  PNR_TRY(gemm_tn_run(2, dzc1, 128, vpe32, 32, n, 128, 32, G[10] + 256, 280, 24, nullptr, F(P.gemm), P.gemm_bytes,
                      sv, words + 3, flag));
  PNR_TRY(gemm_nn_run(true, dzc1, 128, W[10], 280, n, 128, 256, nullptr, 0, 0.f, d_hid, 256, words + 3, flag, nullptr,
                      sv, b + P.bsplit[2]));
  // ---- per-pair chain (k_pairs_bwd<2>), dX packs from the current weights
  float* pscale = F(P.pscale);
  char* packs = b + P.packs;
  const size_t per = (size_t)(16 + 3) * 2048 * 8;
  PNR_TRY(pnr_pack_bwd_h2(W[6], W[4], 263, W[2], 3, pscale, packs, 3 * per, sv));
  pnr_mlp_bwd wb = {nullptr, nullptr, nullptr, nullptr};   // extras per point below
  pnr_mlp_bwd_h2 wbh = {packs, packs + per, packs + 2 * per, pscale};
  float* dz[4] = {F(P.dz[0]), F(P.dz[1]), F(P.dz[2]), F(P.dz[3])};
  float* dpa = F(P.dpa);
  PNR_TRY(pnr_aggregate_bwd_pairs_h2(pts, s, w, &wb, &wbh, saved, d_feat, d_hid, dz[0], dz[1], dz[2], dz[3], dpa,
                                     nullptr, nullptr, nullptr, out->d_conf, sv));
  // ---- per-point sums of dz1 and of the block3.0 extras (pairs grouped by point, pair order)
  int32_t* prow_sorted = reinterpret_cast<int32_t*>(b + P.prow_sorted);
  int32_t* pair_of = reinterpret_cast<int32_t*>(b + P.pair_of);
  const int32_t* off = nullptr;
  PNR_TRY(group_pairs(saved->prow, m, pts->used_map, nk, prow_sorted, pair_of, b + P.grp, P.grp_bytes, st, &off,
                      true));
  float* g_pair = F(P.g_pair);
  PNR_TRY(pnr_aggregate_bwd_extras_rows(pts, s, w, saved, w3e, dz[2], g_pair, sv));
  float* d_p1 = F(P.d_p1);
  // per used point over its group (= pnr_pairs_to_points_ex's sums, 16 lanes per point)
  hipLaunchKernelGGL(k_points_from_groups, dim3(grid_for(nk * 16, 256, 4096)), dim3(256), 0, st, off, pair_of, nk,
                     pts->used, dz[0], d_p1, saved->dz_absmax + 5, g_pair, w->rw2c, pts->rw2c, out->d_color,
                     out->d_dir);
  PNR_LAUNCH_CHECK();
  // ---- weight gradients dW = dZ^T X over the pairs (A scales from k_pairs_bwd's maxima)
  const uint32_t* am = saved->dz_absmax;
  PNR_TRY(gemm_tn_run(2, dz[3], 256, saved->h3, 256, m, 256, 256, G[6], 256, 256, G[7], F(P.gemm), P.gemm_bytes, sv,
                      am + 3, flag));
  PNR_TRY(gemm_tn_run(2, dz[2], 256, saved->h2, 256, m, 256, 256, G[4], 263, 256, G[5], F(P.gemm), P.gemm_bytes, sv,
                      am + 2, flag));
  PNR_TRY(gemm_tn_run(2, dz[2], 256, saved->x3e, 32, m, 256, 32, G[4] + 256, 263, 7, nullptr, F(P.gemm),
                      P.gemm_bytes, sv, am + 2, flag));
  PNR_TRY(gemm_tn_run(2, dz[1], 256, saved->h1, 256, m, 256, 256, G[2], 256, 256, G[3], F(P.gemm), P.gemm_bytes, sv,
                      am + 1, flag));
  PNR_TRY(pnr_alpha_colsum(dpa, saved->h4, m, G[8], G[9], F(P.acp), sv));
  // ---- block1.0: the point half from dP1 / X1 (used rows), the pair half from dz1 / PE_5
  float *x1 = saved->x1 ? saved->x1 : F(P.x1), *dx1 = F(P.dx1);
  if (!saved->x1) PNR_TRY(pnr_point_pe3_rows(pts->emb, pts->used, n_used, x1, sv));   // else the forward's rows
  PNR_TRY(gemm_tn_run(2, d_p1, 256, x1, 224, n_used, 256, 224, G[0], 284, 224, G[1], F(P.gemm), P.gemm_bytes, sv,
                      am + 5, flag));
  PNR_TRY(gemm_tn_run(2, dz[0], 256, saved->pe5, 64, m, 256, 64, G[0] + 224, 284, 60, nullptr, F(P.gemm),
                      P.gemm_bytes, sv, am + 0, flag));
  // (a d emb pass over every row, zeros for the unreferenced ones, measured 176 us
  // against 35 + 42-69 us for the fill and the used-row pass)
  if (n_used > 0) {
    PNR_TRY(gemm_nn_run(true, d_p1, 256, W[0], 284, n_used, 256, 224, nullptr, 0, 0.f, dx1, 224, am + 5, flag,
                        nullptr, sv, b + P.bsplit[3]));
    PNR_TRY(pnr_point_pe3_bwd_rows(pts->emb, pts->used, dx1, n_used, out->d_emb, sv));
  }
#undef PNR_TRY
  return PNR_OK;
}
