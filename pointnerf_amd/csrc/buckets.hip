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
// samples at [info[b], info[b] + info[4 + b])) | info [8] | hist [nchunks][4] |
// bucket of every sample (bytes, padded to 16 B).
#include "agg_common.h"

namespace pnr {

constexpr int kBkBlock = 256;
constexpr int kBkItems = 8;
constexpr int kBkChunk = kBkBlock * kBkItems;   // samples per chunk (one workgroup)

__device__ __forceinline__ int sample_bucket(const pnr_samples& s, int64_t v) {
  const int64_t row = sample_row(s, v);
  const int K = s.K;
  int need = 0;
  if (K == 8 && ((uintptr_t)s.pidx & 15) == 0) {   // one 32-B row: two 16-B loads
    const int4* p = reinterpret_cast<const int4*>(s.pidx + row * 8);
    const int4 a = p[0], b = p[1];
    const int q[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (q[k] >= 0) need = k + 1;
  } else {
    for (int k = 0; k < K; ++k)
      if (s.pidx[row * K + k] >= 0) need = k + 1;
  }
  return need <= 1 ? 0 : (need <= 2 ? 1 : (need <= 4 ? 2 : 3));
}

// Pass 1: bucket of every sample (one byte, read back by the scatter) and the
// chunk's per-bucket counts.  Consecutive threads take consecutive samples, so
// a wave's pidx rows are neighbours in the (ordered) sample list.
__global__ void __launch_bounds__(kBkBlock) k_bucket_hist(pnr_samples s, uint8_t* __restrict__ bkt,
                                                          int32_t* __restrict__ hist) {
  __shared__ int cnt[4];
  if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t n = eff_n(s);
  const int64_t base = (int64_t)blockIdx.x * kBkChunk + threadIdx.x;
  int c[4] = {0, 0, 0, 0};
  for (int i = 0; i < kBkItems; ++i) {
    const int64_t v = base + i * kBkBlock;
    if (v < n) {
      const int b = sample_bucket(s, v);
      bkt[v] = (uint8_t)b;
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

// Pass 3: stable scatter.  The chunk's samples go in 8 rounds of 256
// consecutive ones; within a round a sample's slot is its rank among the lower
// lanes of its wave with the same bucket (ballot + popcount) after the lower
// waves' counts and the earlier rounds' totals -- sample order within every
// bucket, no atomics.
__global__ void __launch_bounds__(kBkBlock) k_bucket_scatter(pnr_samples s, const uint8_t* __restrict__ bkt,
                                                            const int32_t* __restrict__ hist,
                                                            int32_t* __restrict__ list) {
  constexpr int kW = kBkBlock / 64;
  __shared__ int wcnt[kW][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n = eff_n(s);
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;   // lanes below this one
  int run[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) run[b] = hist[(int64_t)blockIdx.x * 4 + b];
  for (int i = 0; i < kBkItems; ++i) {
    const int64_t v = (int64_t)blockIdx.x * kBkChunk + i * kBkBlock + threadIdx.x;
    const int b = v < n ? (int)bkt[v] : -1;
    int rank = 0;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const uint64_t m = __ballot(b == bb);
      if (b == bb) rank = __popcll(m & lt);
      if (lane == 0) wcnt[w][bb] = __popcll(m);
    }
    __syncthreads();
    if (b >= 0) {
      int pos = rank;
      for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][b];
      pos += b == 0 ? run[0] : (b == 1 ? run[1] : (b == 2 ? run[2] : run[3]));
      list[pos] = (int32_t)v;
    }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int ww = 0; ww < kW; ++ww) run[bb] += wcnt[ww][bb];
    __syncthreads();
  }
}

int64_t bucket_scratch_ints(int64_t n_max) {
  const int64_t nm = n_max > 0 ? n_max : 1;
  return cdiv(nm, 4) * 4 + 8 + cdiv(nm, kBkChunk) * 4 + cdiv(nm, 16) * 4;   // .. | bucket bytes
}

int launch_buckets(const pnr_samples& s, int32_t* scratch, PairBuckets* out, hipStream_t st) {
  const int64_t nm = s.n_max > 0 ? s.n_max : 1;
  const int64_t nchunks = cdiv(nm, kBkChunk);
  out->list = scratch;
  out->info = scratch + cdiv(nm, 4) * 4;
  int32_t* hist = out->info + 8;
  uint8_t* bkt = reinterpret_cast<uint8_t*>(hist + nchunks * 4);
  hipLaunchKernelGGL(k_bucket_hist, dim3((unsigned)nchunks), dim3(kBkBlock), 0, st, s, bkt, hist);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(kBkScan), 0, st, hist, nchunks, out->info);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bucket_scatter, dim3((unsigned)nchunks), dim3(kBkBlock), 0, st, s, bkt, hist, out->list);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

}  // namespace pnr
