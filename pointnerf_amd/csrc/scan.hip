// Device-wide exclusive scan of int32 (three-pass: tile reduce, scan of tile
// sums, tile scan + offset), optionally with the stream compaction it sizes
// (list[out[i]] = i for every nonzero in[i], written by the last pass).  Used for every data-dependent compaction of the
// query (R -> R' -> R'' and the SR pick of qpiw.py:655-719), so none of them
// needs a host round trip.
#include "pnr_common.h"

namespace pnr {

constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanBlock * kScanItems;  // 2048

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

// Exclusive scan of one value per thread over a 256-thread block; returns the
// block total through *total.
__device__ __forceinline__ int block_excl_scan(int v, int* lds4, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = wave_incl_scan(v);
  if (lane == 63) lds4[w] = inc;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kScanBlock / 64; ++i) {
    int x = lds4[i];
    base += (i < w) ? x : 0;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

__device__ __forceinline__ int64_t eff_len(int64_t n, const int32_t* n_dev) {
  if (!n_dev) return n;
  int64_t m = *n_dev;
  return m < n ? (m < 0 ? 0 : m) : n;
}

__device__ __forceinline__ int load_item(const int32_t* in, int64_t i, int64_t ne, int as_flag) {
  if (i >= ne) return 0;
  int v = in[i];
  return as_flag ? (v != 0) : v;
}

__global__ void __launch_bounds__(kScanBlock) k_scan_reduce(const int32_t* __restrict__ in, int64_t n,
                                                            const int32_t* n_dev, int as_flag,
                                                            int32_t* __restrict__ sums, const int32_t* run_if) {
  __shared__ int lds4[4];
  if (run_if && *run_if == 0) return;
  const int64_t ne = eff_len(n, n_dev);
  const int64_t start = (int64_t)blockIdx.x * kScanTile;
  if (start >= ne) {
    if (threadIdx.x == 0) sums[blockIdx.x] = 0;
    return;
  }
  int acc = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = start + j * kScanBlock + threadIdx.x;
    acc += load_item(in, i, ne, as_flag);
  }
  int tot;
  block_excl_scan(acc, lds4, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// One block scans all tile sums in place (exclusive); writes the grand total
// to out[n_eff] and total_dev.
__global__ void __launch_bounds__(kScanBlock) k_scan_sums(int32_t* sums, int64_t nb, int64_t n,
                                                          const int32_t* n_dev, int32_t* out,
                                                          int32_t* total_dev, const int32_t* run_if) {
  __shared__ int lds4[4];
  if (run_if && *run_if == 0) return;
  // only the tiles below the effective length hold sums (k_scan_reduce zeroed the
  // rest and k_scan_final skips them): a device length far below n (the query's
  // vflag scan over R * SR slots, ~11 % filled at the headline) then costs its own
  // tiles, not n's (41.7 -> ~5 us)
  const int64_t nbe = cdiv(eff_len(n, n_dev), kScanTile);
  if (nbe < nb) nb = nbe;
  const int64_t per = cdiv(nb, kScanBlock);
  const int64_t b0 = threadIdx.x * per;
  const int64_t b1 = b0 + per < nb ? b0 + per : nb;
  // this thread's segment in batches of 8 loads in flight (one at a time, c5's
  // 22 k tile sums took 30 us of round trips); the adds stay in element order
  constexpr int kB = 8;
  int acc = 0;
  int64_t i = b0;
  for (; i + kB <= b1; i += kB) {
    int x[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) x[j] = sums[i + j];
#pragma unroll
    for (int j = 0; j < kB; ++j) acc += x[j];
  }
  for (; i < b1; ++i) acc += sums[i];
  int tot;
  int base = block_excl_scan(acc, lds4, &tot);
  for (i = b0; i + kB <= b1; i += kB) {
    int x[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) x[j] = sums[i + j];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      sums[i + j] = base;
      base += x[j];
    }
  }
  for (; i < b1; ++i) {
    int x = sums[i];
    sums[i] = base;
    base += x;
  }
  if (threadIdx.x == 0) {
    out[eff_len(n, n_dev)] = tot;
    if (total_dev) *total_dev = tot;
  }
}

__global__ void __launch_bounds__(kScanBlock) k_scan_final(const int32_t* __restrict__ in, int64_t n,
                                                           const int32_t* n_dev, int as_flag,
                                                           const int32_t* __restrict__ sums,
                                                           int32_t* __restrict__ out, const int32_t* run_if,
                                                           int32_t* __restrict__ list) {
  __shared__ int tile[kScanTile];
  __shared__ int lds4[4];
  if (run_if && *run_if == 0) return;
  const int64_t ne = eff_len(n, n_dev);
  const int64_t start = (int64_t)blockIdx.x * kScanTile;
  if (start >= ne) return;
  int lv[kScanItems];   // this thread's loaded items (the list's flags)
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = start + j * kScanBlock + threadIdx.x;
    lv[j] = load_item(in, i, ne, as_flag);
    tile[j * kScanBlock + threadIdx.x] = lv[j];
  }
  __syncthreads();
  int v[kScanItems];
  int acc = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = tile[threadIdx.x * kScanItems + j];
    acc += v[j];
  }
  int tot;
  int base = block_excl_scan(acc, lds4, &tot) + sums[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    tile[threadIdx.x * kScanItems + j] = base;
    base += v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = start + j * kScanBlock + threadIdx.x;
    if (i < ne) {
      const int o = tile[j * kScanBlock + threadIdx.x];
      out[i] = o;
      if (list && lv[j]) list[o] = (int)i;
    }
  }
}

// Two-launch variant for up to kScanDirect tiles (every query compaction and
// grid-build scan at the headline's sizes): each block sums the tile totals before it
// itself (<= kScanDirect / 256 loads per thread) instead of a one-block scan of
// the sums between the passes -- one dependent launch fewer per scan.  The
// block holding the last element writes the grand total.
constexpr int64_t kScanDirect = 4096;   // <= 16 tile totals per thread (the headline's 5.7 M-sample vflag scan: 2 768 tiles)
__global__ void __launch_bounds__(kScanBlock) k_scan_final_direct(const int32_t* __restrict__ in, int64_t n,
                                                                  const int32_t* n_dev, int as_flag,
                                                                  const int32_t* __restrict__ sums,
                                                                  int32_t* __restrict__ out, int32_t* total_dev,
                                                                  const int32_t* run_if, int32_t* __restrict__ list) {
  __shared__ int tile[kScanTile];
  __shared__ int lds4[4];
  if (run_if && *run_if == 0) return;
  const int64_t ne = eff_len(n, n_dev);
  const int64_t start = (int64_t)blockIdx.x * kScanTile;
  if (ne == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      out[0] = 0;
      if (total_dev) *total_dev = 0;
    }
    return;
  }
  if (start >= ne) return;
  int pre = 0;
  for (int i = threadIdx.x; i < (int)blockIdx.x; i += kScanBlock) pre += sums[i];
  int pre_tot;
  block_excl_scan(pre, lds4, &pre_tot);   // (block_excl_scan's barriers also order the tile loads below)
  int lv[kScanItems];   // this thread's loaded items (the list's flags)
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = start + j * kScanBlock + threadIdx.x;
    lv[j] = load_item(in, i, ne, as_flag);
    tile[j * kScanBlock + threadIdx.x] = lv[j];
  }
  __syncthreads();
  int v[kScanItems];
  int acc = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = tile[threadIdx.x * kScanItems + j];
    acc += v[j];
  }
  int tot;
  int base = block_excl_scan(acc, lds4, &tot) + pre_tot;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    tile[threadIdx.x * kScanItems + j] = base;
    base += v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = start + j * kScanBlock + threadIdx.x;
    if (i < ne) {
      const int o = tile[j * kScanBlock + threadIdx.x];
      out[i] = o;
      if (list && lv[j]) list[o] = (int)i;
    }
  }
  if (start + kScanTile >= ne && threadIdx.x == 0) {   // the tile of the last element
    out[ne] = pre_tot + tot;
    if (total_dev) *total_dev = pre_tot + tot;
  }
}

int64_t scan_blocks(int64_t n) { return cdiv(n > 0 ? n : 1, kScanTile); }

size_t scan_scratch_bytes(int64_t n) { return (size_t)(scan_blocks(n) + 1) * sizeof(int32_t); }

int exclusive_scan(const int32_t* in, int64_t n, const int32_t* n_dev, int32_t* out, int64_t out_cap,
                   int32_t* total_dev, void* scratch, size_t scratch_bytes, hipStream_t st,
                   int as_flag, const int32_t* run_if, int32_t* list) {
  PNR_CHECK_ARG(in && out && scratch, "scan: null pointer");
  PNR_CHECK_ARG(n >= 0, "scan: negative length");
  // the grand total is stored at out[n_eff] (n_eff <= n): out needs n + 1 entries
  PNR_CHECK_ARG(out_cap >= n + 1, "scan: out holds %lld entries, the scan of %lld writes %lld",
                (long long)out_cap, (long long)n, (long long)n + 1);
  const int64_t nb = scan_blocks(n);
  PNR_CHECK_ARG(scratch_bytes >= scan_scratch_bytes(n), "scan: scratch too small (%zu < %zu)",
                scratch_bytes, scan_scratch_bytes(n));
  PNR_CHECK_ARG(nb < (int64_t)1 << 31, "scan: too many tiles");
  int32_t* sums = static_cast<int32_t*>(scratch);
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, n_dev, as_flag, sums, run_if);
  PNR_LAUNCH_CHECK();
  if (nb <= kScanDirect) {
    hipLaunchKernelGGL(k_scan_final_direct, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, n_dev, as_flag, sums,
                       out, total_dev, run_if, list);
    PNR_LAUNCH_CHECK();
    return PNR_OK;
  }
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kScanBlock), 0, st, sums, nb, n, n_dev, out, total_dev, run_if);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_scan_final, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, n_dev, as_flag, sums, out, run_if,
                     list);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

}  // namespace pnr

extern "C" int pnr_scan_scratch_bytes(int64_t n, size_t* out) {
  PNR_CHECK_ARG(out, "null out");
  *out = pnr::scan_scratch_bytes(n);
  return PNR_OK;
}

extern "C" int pnr_exclusive_scan_i32(const int32_t* in, int64_t n, const int32_t* n_dev,
                                      int32_t* out, int64_t out_len, int32_t* total_dev, void* scratch,
                                      size_t scratch_bytes, void* stream) {
  return pnr::exclusive_scan(in, n, n_dev, out, out_len, total_dev, scratch, scratch_bytes,
                             pnr::as_stream(stream), 0);
}
