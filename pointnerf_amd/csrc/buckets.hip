// Pair-tile buckets for sparse neighbour lists (the reference's masked holders,
// point_aggregators.py:608-628, evaluate only the valid (sample, neighbour)
// pairs; fixed K = 8 tiles spend their MFMA columns on empty slots when a scene
// averages ~2 neighbours per sample, BASELINE config c5).
//
// Every sample of the aggregate's sample list gets the bucket b = 0..3 of its
// "need" (last filled neighbour slot + 1): KT = 1, 2, 4, 8 slots per sample.
// A stable partition of the sample indices by bucket (per-chunk histograms ->
// one scan -> per-chunk scatter, no atomics on the output) lets the pairs kernel
// run each bucket with tiles of 128 / KT samples x KT slots: the slots a bucket
// drops are empty in every one of its samples (the KNN fills slots in order,
// qpiw.py:497-512), so the per-pair outputs and the K-sums are the same numbers
// (sums of the same non-zero terms in the same pairing order).
//
// Layout of the int32 scratch (bucket_scratch_ints): list [n_max] (bucket b's
// samples at [info[b], info[b] + info[4 + b])) | info [8] | hist [nchunks][4].
#include "agg_common.h"

namespace pnr {

constexpr int kBkBlock = 256;
constexpr int kBkItems = 8;
constexpr int kBkChunk = kBkBlock * kBkItems;   // samples per chunk (one workgroup)

__device__ __forceinline__ int sample_bucket(const pnr_samples& s, int64_t v) {
  const int64_t row = sample_row(s, v);
  const int K = s.K;
  int need = 0;
  for (int k = 0; k < K; ++k)
    if (s.pidx[row * K + k] >= 0) need = k + 1;
  return need <= 1 ? 0 : (need <= 2 ? 1 : (need <= 4 ? 2 : 3));
}

__global__ void __launch_bounds__(kBkBlock) k_bucket_hist(pnr_samples s, int32_t* __restrict__ hist) {
  __shared__ int cnt[4];
  if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t n = eff_n(s);
  const int64_t base = (int64_t)blockIdx.x * kBkChunk + threadIdx.x * kBkItems;
  int c[4] = {0, 0, 0, 0};
  for (int i = 0; i < kBkItems; ++i) {
    const int64_t v = base + i;
    if (v < n) {
      const int b = sample_bucket(s, v);
      c[0] += b == 0;
      c[1] += b == 1;
      c[2] += b == 2;
      c[3] += b == 3;
    }
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    int x = c[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if ((threadIdx.x & 63) == 0 && x) atomicAdd(&cnt[b], x);
  }
  __syncthreads();
  if (threadIdx.x < 4) hist[(int64_t)blockIdx.x * 4 + threadIdx.x] = cnt[threadIdx.x];
}

// One workgroup: hist[chunk][b] -> absolute start of the chunk's bucket-b run
// in the list; info[b] = bucket start, info[4 + b] = bucket size.
constexpr int kBkScan = 1024;
__global__ void __launch_bounds__(kBkScan) k_bucket_scan(int32_t* __restrict__ hist, int64_t nchunks,
                                                         int32_t* __restrict__ info) {
  __shared__ int part[4][kBkScan];
  __shared__ int start[4];
  const int t = threadIdx.x;
  const int64_t per = cdiv(nchunks, kBkScan);
  const int64_t c0 = t * per, c1 = c0 + per < nchunks ? c0 + per : nchunks;
  int loc[4] = {0, 0, 0, 0};
  for (int64_t ch = c0; ch < c1; ++ch)
#pragma unroll
    for (int b = 0; b < 4; ++b) loc[b] += hist[ch * 4 + b];
#pragma unroll
  for (int b = 0; b < 4; ++b) part[b][t] = loc[b];
  __syncthreads();
  // Hillis-Steele inclusive scan of the 1024 partials, per bucket
  for (int o = 1; o < kBkScan; o <<= 1) {
    int x[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) x[b] = t >= o ? part[b][t - o] : 0;
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 4; ++b) part[b][t] += x[b];
    __syncthreads();
  }
  if (t == 0) {
    int acc = 0;
    for (int b = 0; b < 4; ++b) {
      start[b] = acc;
      info[b] = acc;
      info[4 + b] = part[b][kBkScan - 1];
      acc += part[b][kBkScan - 1];
    }
  }
  __syncthreads();
  int off[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) off[b] = start[b] + part[b][t] - loc[b];
  for (int64_t ch = c0; ch < c1; ++ch)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int h = hist[ch * 4 + b];
      hist[ch * 4 + b] = off[b];
      off[b] += h;
    }
}

__global__ void __launch_bounds__(kBkBlock) k_bucket_scatter(pnr_samples s, const int32_t* __restrict__ hist,
                                                            int32_t* __restrict__ list) {
  __shared__ int wsum[4][kBkBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n = eff_n(s);
  const int64_t base = (int64_t)blockIdx.x * kBkChunk + threadIdx.x * kBkItems;
  int bk[kBkItems];
  int c[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < kBkItems; ++i) {
    const int64_t v = base + i;
    bk[i] = v < n ? sample_bucket(s, v) : -1;
    c[0] += bk[i] == 0;
    c[1] += bk[i] == 1;
    c[2] += bk[i] == 2;
    c[3] += bk[i] == 3;
  }
  // exclusive prefix of each bucket's count over the block's threads (in thread order)
  int pre[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    int x = c[b];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[b][w] = x;
    pre[b] = x - c[b];
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    int add = hist[(int64_t)blockIdx.x * 4 + b];
    for (int i = 0; i < w; ++i) add += wsum[b][i];
    pre[b] += add;
  }
#pragma unroll
  for (int i = 0; i < kBkItems; ++i) {
    const int b = bk[i];
    if (b < 0) continue;
    int pos = pre[0];
    pos = b == 1 ? pre[1] : pos;
    pos = b == 2 ? pre[2] : pos;
    pos = b == 3 ? pre[3] : pos;
    list[pos] = (int32_t)(base + i);
    pre[0] += b == 0;
    pre[1] += b == 1;
    pre[2] += b == 2;
    pre[3] += b == 3;
  }
}

int64_t bucket_scratch_ints(int64_t n_max) {
  const int64_t nm = n_max > 0 ? n_max : 1;
  return cdiv(nm, 4) * 4 + 8 + cdiv(nm, kBkChunk) * 4;
}

int launch_buckets(const pnr_samples& s, int32_t* scratch, PairBuckets* out, hipStream_t st) {
  const int64_t nm = s.n_max > 0 ? s.n_max : 1;
  const int64_t nchunks = cdiv(nm, kBkChunk);
  out->list = scratch;
  out->info = scratch + cdiv(nm, 4) * 4;
  int32_t* hist = out->info + 8;
  hipLaunchKernelGGL(k_bucket_hist, dim3((unsigned)nchunks), dim3(kBkBlock), 0, st, s, hist);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(kBkScan), 0, st, hist, nchunks, out->info);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bucket_scatter, dim3((unsigned)nchunks), dim3(kBkBlock), 0, st, s, hist, out->list);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

}  // namespace pnr
