// Ray-march alpha composite.
//
// k_composite fuses, for every ray of the batch:
//   ray_dist = cummax(sample_loc z) differences, unit-voxel clamp, x ray_valid
//                                   neural_points_volumetric_model.py:293-301
//   ray_march + radiance_render + alpha_blend + tone_map 'off'
//                                   diff_ray_marching.py:509-555, diff_render_func.py:36-63
//   fill_invalid (background rays)  neural_points_volumetric_model.py:354-389
// One wave per ray: lane s owns shading slots s and s+64 for the per-slot
// scalars (z, sigma, opacity) and the cummax / exclusive cumprod run as
// wave scans; then lane c owns colour channels c and c+64 and the wave walks
// the valid slots once, reading each sample's 129-float feature row with two
// coalesced 256-B loads.  Empty and invalid slots cost no feature traffic.
#include "pnr_common.h"

namespace pnr {

constexpr int kCBlock = 256;
// feature rows in flight per ray (a ray has ~8 valid samples; A/B: 4 rows 0.94 ms,
// 8 rows 0.93, 16 rows 1.12 on the bench frame, identical checksums)
constexpr int kCRows = 8;

__device__ __forceinline__ float wave_max_scan_incl(float v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    float t = __shfl_up(v, o);
    if (lane >= o) v = fmaxf(v, t);
  }
  return v;
}

__device__ __forceinline__ float wave_prod_scan_incl(float v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    float t = __shfl_up(v, o);
    if (lane >= o) v = v * t;
  }
  return v;
}

// Per-slot scalars -> opacity, exclusive transmittance, blend weight, bg T.
// Inputs per lane for slots s0 = lane, s1 = lane + 64 (SR <= 128).
struct SlotOut {
  float op0, op1, T0, T1, bgT;
};

__device__ __forceinline__ SlotOut march_slots(float sig0, float dist0, float sig1, float dist1, int SR) {
  const int lane = threadIdx.x & 63;
  // sigma = features[...,0] * ray_valid; opacity = 1 - exp(-sigma * dist)
  const float op0 = 1.f - expf(-sig0 * dist0);
  const float op1 = 1.f - expf(-sig1 * dist1);
  // cumprod(1 - opacity + 1e-10), made exclusive (diff_ray_marching.py:534-539)
  float f0 = (lane < SR) ? (1.f - op0 + 1e-10f) : 1.f;
  float f1 = (lane + 64 < SR) ? (1.f - op1 + 1e-10f) : 1.f;
  float i0 = wave_prod_scan_incl(f0);
  float tot0 = __shfl(i0, 63);
  float i1 = wave_prod_scan_incl(f1) * tot0;
  float e0 = __shfl_up(i0, 1);
  float e1 = __shfl_up(i1, 1);
  if (lane == 0) {
    e0 = 1.f;
    e1 = tot0;
  }
  SlotOut o;
  o.op0 = op0;
  o.op1 = op1;
  o.T0 = e0;
  o.T1 = e1;
  // background transmission = inclusive product at slot SR-1
  const int last = SR - 1;
  o.bgT = last < 64 ? __shfl(i0, last) : __shfl(i1, last - 64);
  return o;
}

struct CompArgs {
  const float* campos;
  const float* camrot;
  const int32_t* ray_cam;   // NULL: one camera; else camera index per ray
  int64_t R;
  int SR;
  const int32_t* n_filled;
  const int32_t* ray_off;
  const int32_t* ray_vcnt;
  const int32_t* vflag;
  const int32_t* valid_off;
  const float* sample_p;
  const float* feat;
  const uint16_t* feat_h;   // pnr_composite_fwd_hf: bf16 rows (PNR_FEAT_H_PITCH) instead of feat
  int64_t feat_rows;   // rows of feat: valid samples at or past it are not read (capacity overflow)
  float vsize_z;
  int unit;
  int C;
  const float* bg;
  float* ray_color;
  float* opacity;
  float* is_bg;
  int8_t* ray_mask;
};

// Camera-space depth of the world origin: the z of every unfilled slot
// (sample_loc_w = 0, neural_points_volumetric_model.py:293) for camera `cam`.
__device__ float origin_depth(const CompArgs& a, int64_t cam) {
  float c[3], Rm[9];
#pragma unroll
  for (int i = 0; i < 3; ++i) c[i] = a.campos[cam * 3 + i];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rm[i] = a.camrot[cam * 9 + i];
  const float zero[3] = {0.f, 0.f, 0.f};
  float pc[3];
  world_to_cam(zero, c, Rm, pc);
  return pc[2];
}

// HF: features from pnr_aggregate_fwd_bf16_hf's bf16 rows -- lane l holds
// channels 2l and 2l + 1 (one 4-B load per row), alpha the row's fp32 head.
template <bool HF>
__global__ void __launch_bounds__(kCBlock) k_composite(CompArgs a) {
  constexpr int NRW = kCRows;   // feature rows in flight (bf16 rows too: 12 / 16 measured slower at c5)
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int SR = a.SR, C = a.C, CF = C + 1;
  // depth of the world origin: the z of every unfilled slot (sample_loc_w = 0)
  const float zo0 = origin_depth(a, 0);
  const float vz = a.vsize_z, two_vz = 2.f * a.vsize_z;
  for (int64_t r = wave0; r < a.R; r += nwaves) {
    const bool mask = a.ray_vcnt[r] > 0;
    if (!mask) {  // fill_invalid: background ray
      for (int c = lane; c < C; c += 64) a.ray_color[r * C + c] = a.bg ? a.bg[c] : 0.f;
      for (int s = lane; s < SR; s += 64) a.opacity[r * SR + s] = 0.f;
      if (lane == 0) {
        a.is_bg[r] = 1.f;
        a.ray_mask[r] = 0;
      }
      continue;
    }
    const int n = a.n_filled[r], off = a.ray_off[r];
    const float zo = a.ray_cam ? origin_depth(a, a.ray_cam[r]) : zo0;
    float z[2], sig[2];
    int vrow[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s = lane + 64 * q;
      const bool filled = s < n;
      const int64_t i = off + s;
      z[q] = filled ? a.sample_p[i * 3 + 2] : (s < SR ? zo : -INFINITY);
      const bool val = filled && a.vflag[i];
      vrow[q] = val ? a.valid_off[i] : -1;
      if (vrow[q] >= a.feat_rows) vrow[q] = -1;   // capacity overflow: the caller re-renders
      if constexpr (HF)
        sig[q] = vrow[q] >= 0 ? *reinterpret_cast<const float*>(a.feat_h + (int64_t)vrow[q] * PNR_FEAT_H_PITCH) : 0.f;
      else
        sig[q] = vrow[q] >= 0 ? a.feat[(int64_t)vrow[q] * CF] : 0.f;
    }
    // the first NRW valid rows' channels are loaded now, beside sigma, before the
    // slot scans below (their weights are applied after them): one round trip
    // fewer on a ray's dependent chain (A/B, identical checksums: c5 4.00 -> 3.46
    // ms, the headline unchanged at 0.89 ms -- profiles/r06_composite_prefetch_ab.jsonl)
    unsigned long long m0 = __ballot(vrow[0] >= 0), m1 = __ballot(vrow[1] >= 0);
    int vr[NRW], sl[NRW];   // row and source slot (wave-uniform) of each row in flight
    float f0[NRW], f1[NRW];
    auto pick = [&]() {
#pragma unroll
      for (int u = 0; u < NRW; ++u) {
        vr[u] = -1;
        sl[u] = -1;
        if (m0) {
          const int src = __builtin_ctzll(m0);
          m0 &= m0 - 1;
          vr[u] = __shfl(vrow[0], src);
          sl[u] = src;
        } else if (m1) {
          const int src = __builtin_ctzll(m1);
          m1 &= m1 - 1;
          vr[u] = __shfl(vrow[1], src);
          sl[u] = 64 + src;
        }
      }
    };
    auto load_rows = [&]() {
#pragma unroll
      for (int u = 0; u < NRW; ++u) {
        if constexpr (HF) {
          const uint32_t* f = reinterpret_cast<const uint32_t*>(
              a.feat_h + (int64_t)(vr[u] < 0 ? 0 : vr[u]) * PNR_FEAT_H_PITCH + 8);
          const uint32_t v = (vr[u] >= 0 && 2 * lane < C) ? f[lane] : 0u;
          f0[u] = __uint_as_float(v << 16);            // channel 2 lane
          f1[u] = __uint_as_float(v & 0xffff0000u);    // channel 2 lane + 1
        } else {
          const float* f = a.feat + (int64_t)(vr[u] < 0 ? 0 : vr[u]) * CF + 1;
          f0[u] = (vr[u] >= 0 && lane < C) ? f[lane] : 0.f;
          f1[u] = (vr[u] >= 0 && lane + 64 < C) ? f[lane + 64] : 0.f;
        }
      }
    };
    pick();
    load_rows();
    // cummax over slots (neural_points_volumetric_model.py:293)
    float cm0 = wave_max_scan_incl(z[0]);
    float cm1 = fmaxf(wave_max_scan_incl(z[1]), __shfl(cm0, 63));
    // next slot's cummax
    float nx0 = __shfl_down(cm0, 1), nx1 = __shfl_down(cm1, 1);
    const float cm1_first = __shfl(cm1, 0);
    if (lane == 63) nx0 = cm1_first;
    float dist[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s = lane + 64 * q;
      const float cm = q ? cm1 : cm0, nx = q ? nx1 : nx0;
      float d = (s < SR - 1) ? (nx - cm) : vz;
      const bool msk = (d < 1e-8f) || (a.unit && d > two_vz);
      d = msk ? vz : d;
      dist[q] = vrow[q] >= 0 ? d : 0.f;  // ray_dist *= ray_valid
    }
    const SlotOut so = march_slots(sig[0], dist[0], sig[1], dist[1], SR);
    if (lane < SR) a.opacity[r * SR + lane] = so.op0;
    if (lane + 64 < SR) a.opacity[r * SR + lane + 64] = so.op1;
    const float w0 = so.op0 * so.T0, w1 = so.op1 * so.T1;
    // colour = sum_s w_s * features[s, 1:] + bg * T_bg  (lane = channel)
    // valid slots in slot order, NRW feature rows in flight per iteration
    // (same accumulation order as a plain slot loop)
    float col0 = 0.f, col1 = 0.f;
    for (;;) {
#pragma unroll
      for (int u = 0; u < NRW; ++u) {
        if (vr[u] < 0) break;
        const float w = sl[u] < 64 ? __shfl(w0, sl[u]) : __shfl(w1, sl[u] - 64);
        col0 += w * f0[u];
        col1 += w * f1[u];
      }
      if (!(m0 | m1)) break;
      pick();
      load_rows();
    }
    if constexpr (HF) {
      if (2 * lane < C) {
        float v0 = col0, v1 = col1;
        if (a.bg) {
          v0 += a.bg[2 * lane] * so.bgT;
          v1 += a.bg[2 * lane + 1] * so.bgT;
        }
        a.ray_color[r * C + 2 * lane] = v0;
        a.ray_color[r * C + 2 * lane + 1] = v1;
      }
    } else {
      for (int c = lane, q = 0; c < C; c += 64, ++q) {
        float v = q == 0 ? col0 : (q == 1 ? col1 : 0.f);
        if (a.bg) v += a.bg[c] * so.bgT;
        a.ray_color[r * C + c] = v;
      }
    }
    if (lane == 0) {
      a.is_bg[r] = so.bgT;
      a.ray_mask[r] = 1;
    }
  }
}

// ray_march on dense [NR, SR, C+1] features (mirror path).
__global__ void __launch_bounds__(kCBlock) k_ray_march_dense(const float* __restrict__ ray_dist,
                                                             const uint8_t* __restrict__ ray_valid,
                                                             const float* __restrict__ feat,
                                                             const float* __restrict__ bg, int64_t NR,
                                                             int SR, int C, float* ray_color,
                                                             float* opacity, float* acc_T,
                                                             float* blend_w, float* bg_T) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int CF = C + 1;
  for (int64_t r = wave0; r < NR; r += nwaves) {
    float sig[2], dist[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s = lane + 64 * q;
      const bool in = s < SR;
      const int64_t e = r * SR + s;
      const float v = (in && ray_valid[e]) ? 1.f : 0.f;
      sig[q] = in ? feat[e * CF] * v : 0.f;
      dist[q] = in ? ray_dist[e] : 0.f;
    }
    const SlotOut so = march_slots(sig[0], dist[0], sig[1], dist[1], SR);
    const float w0 = so.op0 * so.T0, w1 = so.op1 * so.T1;
    if (lane < SR) {
      opacity[r * SR + lane] = so.op0;
      acc_T[r * SR + lane] = so.T0;
      blend_w[r * SR + lane] = w0;
    }
    if (lane + 64 < SR) {
      opacity[r * SR + lane + 64] = so.op1;
      acc_T[r * SR + lane + 64] = so.T1;
      blend_w[r * SR + lane + 64] = w1;
    }
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + lane;
      float v = 0.f;
      for (int s = 0; s < SR; ++s) {
        const int q = s >> 6, src = s & 63;
        const float w = __shfl(q ? w1 : w0, src);
        if (c < C) v += w * feat[(r * SR + s) * CF + 1 + c];
      }
      if (c < C) {
        if (bg) v += bg[c] * so.bgT;
        ray_color[r * C + c] = v;
      }
    }
    if (lane == 0) bg_T[r] = so.bgT;
  }
}

// ---------------------------------------------------------------- backward
// Reverse-mode of march_slots + the colour sum (autograd of
// diff_ray_marching.py:530-555): gw = <d colour, c_s> per slot, dbgT =
// <d colour, bg>.  With f_s = 1 - o_s + 1e-10, P = cumprod(f) (inclusive),
// T_s = P_{s-1} (exclusive), w_s = o_s T_s, bgT = P_{SR-1}:
//   dP_i = dT_{i+1} (i < SR-1), dP_{SR-1} = dbgT          (made-exclusive shift)
//   df_j = sum_{i >= j} dP_i P_i / f_j                   (torch cumprod backward)
//   do_j = gw_j T_j - df_j,  dsigma_j = do_j exp(-sigma_j d_j) d_j.
__device__ __forceinline__ float wave_sum_suffix_incl(float v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    float t = __shfl_down(v, o);
    if (lane + o < 64) v += t;
  }
  return v;
}

// Extra per-slot output gradients of the dense ray_march (all differentiable in
// the reference): dox = d opacity, dTx = d acc_transmission (exclusive T); a d
// blend_weight is folded into gw by the caller.  d_dist (NULL = not wanted) is
// the gradient with respect to ray_dist.
__device__ __forceinline__ void march_slots_bwd(const float sig[2], const float dist[2], const float gw[2], float dbgT,
                                                int SR, float dsig[2], const float dox[2] = nullptr,
                                                const float dTx[2] = nullptr, float* ddist = nullptr) {
  const int lane = threadIdx.x & 63;
  const float op0 = 1.f - expf(-sig[0] * dist[0]);
  const float op1 = 1.f - expf(-sig[1] * dist[1]);
  const float f0 = (lane < SR) ? (1.f - op0 + 1e-10f) : 1.f;
  const float f1 = (lane + 64 < SR) ? (1.f - op1 + 1e-10f) : 1.f;
  const float i0 = wave_prod_scan_incl(f0);
  const float tot0 = __shfl(i0, 63);
  const float i1 = wave_prod_scan_incl(f1) * tot0;
  float e0 = __shfl_up(i0, 1), e1 = __shfl_up(i1, 1);
  if (lane == 0) {
    e0 = 1.f;
    e1 = tot0;
  }
  // dT (exclusive) per slot, then dP_i = dT_{i+1}
  const float dT0 = gw[0] * op0 + (dTx ? dTx[0] : 0.f), dT1 = gw[1] * op1 + (dTx ? dTx[1] : 0.f);
  float dP0 = __shfl_down(dT0, 1), dP1 = __shfl_down(dT1, 1);
  const float dT1_first = __shfl(dT1, 0);
  if (lane == 63) {
    dP0 = dT1_first;
    dP1 = 0.f;
  }
  const int last = SR - 1;
  if (lane == last) dP0 = dbgT;
  if (lane + 64 == last) dP1 = dbgT;
  if (lane > last) dP0 = 0.f;
  if (lane + 64 > last) dP1 = 0.f;
  // suffix sums of dP_i P_i (slots 64.. first, then 0..63 plus the upper total)
  const float s1 = wave_sum_suffix_incl(dP1 * i1);
  const float tot1 = __shfl(s1, 0);
  const float s0 = wave_sum_suffix_incl(dP0 * i0) + tot1;
  const float df0 = (lane < SR) ? s0 / f0 : 0.f;
  const float df1 = (lane + 64 < SR) ? s1 / f1 : 0.f;
  const float do0 = gw[0] * e0 - df0 + (dox ? dox[0] : 0.f), do1 = gw[1] * e1 - df1 + (dox ? dox[1] : 0.f);
  const float x0 = expf(-sig[0] * dist[0]), x1 = expf(-sig[1] * dist[1]);
  dsig[0] = do0 * x0 * dist[0];
  dsig[1] = do1 * x1 * dist[1];
  if (ddist) {   // opacity = 1 - exp(-sigma dist): d dist = d opacity exp(-sigma dist) sigma
    ddist[0] = do0 * x0 * sig[0];
    ddist[1] = do1 * x1 * sig[1];
  }
}

struct CompBwdArgs {
  CompArgs f;
  const float* d_color;   // [R,C]
  float* d_feat;          // [S_valid,C+1]
};

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ void __launch_bounds__(kCBlock) k_composite_bwd(CompBwdArgs A) {
  const CompArgs& a = A.f;
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int SR = a.SR, C = a.C, CF = C + 1;
  const float zo0 = origin_depth(a, 0);
  const float vz = a.vsize_z, two_vz = 2.f * a.vsize_z;
  for (int64_t r = wave0; r < a.R; r += nwaves) {
    if (a.ray_vcnt[r] <= 0) continue;   // background ray: no feature gradient
    // forward recompute (same as k_composite)
    const int n = a.n_filled[r], off = a.ray_off[r];
    const float zo = a.ray_cam ? origin_depth(a, a.ray_cam[r]) : zo0;
    float z[2], sig[2];
    int vrow[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s = lane + 64 * q;
      const bool filled = s < n;
      const int64_t i = off + s;
      z[q] = filled ? a.sample_p[i * 3 + 2] : (s < SR ? zo : -INFINITY);
      const bool val = filled && a.vflag[i];
      vrow[q] = val ? a.valid_off[i] : -1;
      if (vrow[q] >= a.feat_rows) vrow[q] = -1;   // capacity overflow: the caller re-renders
      sig[q] = vrow[q] >= 0 ? a.feat[(int64_t)vrow[q] * CF] : 0.f;
    }
    float cm0 = wave_max_scan_incl(z[0]);
    float cm1 = fmaxf(wave_max_scan_incl(z[1]), __shfl(cm0, 63));
    float nx0 = __shfl_down(cm0, 1), nx1 = __shfl_down(cm1, 1);
    const float cm1_first = __shfl(cm1, 0);
    if (lane == 63) nx0 = cm1_first;
    float dist[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s = lane + 64 * q;
      const float cm = q ? cm1 : cm0, nx = q ? nx1 : nx0;
      float d = (s < SR - 1) ? (nx - cm) : vz;
      const bool msk = (d < 1e-8f) || (a.unit && d > two_vz);
      d = msk ? vz : d;
      dist[q] = vrow[q] >= 0 ? d : 0.f;
    }
    const SlotOut so = march_slots(sig[0], dist[0], sig[1], dist[1], SR);
    const float w0 = so.op0 * so.T0, w1 = so.op1 * so.T1;
    // colour part: lane = channel
    const float* dc = A.d_color + r * C;
    const float dc0 = lane < C ? dc[lane] : 0.f, dc1 = lane + 64 < C ? dc[lane + 64] : 0.f;
    float dbgT = 0.f;
    if (a.bg) dbgT = wave_sum_f32((lane < C ? dc0 * a.bg[lane] : 0.f) + (lane + 64 < C ? dc1 * a.bg[lane + 64] : 0.f));
    float gw[2] = {0.f, 0.f};
    const int smax = n < SR ? n : SR;
    for (int s = 0; s < smax; ++s) {
      const int q = s >> 6, src = s & 63;
      const int vr = __shfl(q ? vrow[1] : vrow[0], src);
      if (vr < 0) continue;
      const float w = __shfl(q ? w1 : w0, src);
      const float* f = a.feat + (int64_t)vr * CF + 1;
      float* g = A.d_feat + (int64_t)vr * CF + 1;
      float part = 0.f;
      if (lane < C) {
        part += dc0 * f[lane];
        g[lane] = w * dc0;
      }
      if (lane + 64 < C) {
        part += dc1 * f[lane + 64];
        g[lane + 64] = w * dc1;
      }
      const float gws = wave_sum_f32(part);
      if (lane == src) gw[q] = gws;
    }
    float dsig[2];
    march_slots_bwd(sig, dist, gw, dbgT, SR, dsig);
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (vrow[q] >= 0) A.d_feat[(int64_t)vrow[q] * CF] = dsig[q];
  }
}

// Backward of k_ray_march_dense with respect to feat (and ray_dist), from the
// gradients of every output: d ray_color [NR,C] and, each optional (NULL = 0),
// d opacity / d acc_T / d blend_w [NR,SR] and d bg_T [NR].
struct MarchBwdArgs {
  const float* ray_dist;
  const uint8_t* ray_valid;
  const float* feat;
  const float* bg;
  int64_t NR;
  int SR, C;
  const float* d_color;
  const float* d_opacity;
  const float* d_acc_T;
  const float* d_blend;
  const float* d_bgT;
  float* d_feat;
  float* d_dist;
};

__global__ void __launch_bounds__(kCBlock) k_ray_march_dense_bwd(MarchBwdArgs A) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int SR = A.SR, C = A.C, CF = C + 1;
  for (int64_t r = wave0; r < A.NR; r += nwaves) {
    float sig[2], dist[2], vv[2], dox[2] = {0.f, 0.f}, dTx[2] = {0.f, 0.f}, gb[2] = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s = lane + 64 * q;
      const bool in = s < SR;
      const int64_t e = r * SR + s;
      vv[q] = (in && A.ray_valid[e]) ? 1.f : 0.f;
      sig[q] = in ? A.feat[e * CF] * vv[q] : 0.f;
      dist[q] = in ? A.ray_dist[e] : 0.f;
      if (in) {
        if (A.d_opacity) dox[q] = A.d_opacity[e];
        if (A.d_acc_T) dTx[q] = A.d_acc_T[e];
        if (A.d_blend) gb[q] = A.d_blend[e];
      }
    }
    const SlotOut so = march_slots(sig[0], dist[0], sig[1], dist[1], SR);
    const float w0 = so.op0 * so.T0, w1 = so.op1 * so.T1;
    float gw[2] = {0.f, 0.f};
    float dbgT = A.d_bgT ? A.d_bgT[r] : 0.f;
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + lane;
      const float dcv = c < C ? A.d_color[r * C + c] : 0.f;
      if (A.bg) dbgT += wave_sum_f32(c < C ? dcv * A.bg[c] : 0.f);
      for (int s = 0; s < SR; ++s) {
        const int q = s >> 6, src = s & 63;
        const float w = __shfl(q ? w1 : w0, src);
        const int64_t e = (r * SR + s) * CF + 1 + c;
        const float gws = wave_sum_f32(c < C ? dcv * A.feat[e] : 0.f);
        if (lane == src) gw[q] += gws;
        if (c < C) A.d_feat[e] = w * dcv;
      }
    }
    gw[0] += gb[0];   // blend_weight = opacity * acc_T
    gw[1] += gb[1];
    float dsig[2], dd[2];
    march_slots_bwd(sig, dist, gw, dbgT, SR, dsig, dox, dTx, A.d_dist ? dd : nullptr);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s = lane + 64 * q;
      if (s < SR) {
        A.d_feat[(r * SR + s) * CF] = dsig[q] * vv[q];
        if (A.d_dist) A.d_dist[r * SR + s] = dd[q];
      }
    }
  }
}

// out[c] = sum_r w[r] x[r, c] -- the background colour's gradient (w = is_bg of
// k_composite: bg_T for a hit ray, 1 for a background ray, so both the ray_march
// term bg * bg_T and fill_invalid's bg rows are covered; w = bg_T for the dense
// ray_march).  Block b sums a contiguous ray range in a fixed order (4 waves over
// strided rays, combined in wave order), then one block sums the block partials in
// order: bitwise repeatable.
constexpr int kColsumBlocks = 256;

__global__ void __launch_bounds__(256) k_wcolsum_part(const float* __restrict__ w, const float* __restrict__ x,
                                                      int64_t R, int C, float* __restrict__ part) {
  __shared__ float red[4][128];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t per = cdiv(R, kColsumBlocks);
  const int64_t r0 = blockIdx.x * per, r1 = r0 + per < R ? r0 + per : R;
  float a0 = 0.f, a1 = 0.f;
  for (int64_t r = r0 + wid; r < r1; r += 4) {
    const float wr = w[r];
    if (lane < C) a0 += wr * x[r * C + lane];
    if (lane + 64 < C) a1 += wr * x[r * C + lane + 64];
  }
  red[wid][lane] = a0;
  red[wid][lane + 64] = a1;
  __syncthreads();
  if (wid == 0) {
    for (int c = lane; c < C; c += 64)
      part[(int64_t)blockIdx.x * C + c] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
  }
}

__global__ void __launch_bounds__(128) k_wcolsum_final(const float* __restrict__ part, int C, float* __restrict__ out) {
  const int c = threadIdx.x;
  if (c >= C) return;
  float a = 0.f;
  for (int b = 0; b < kColsumBlocks; ++b) a += part[(int64_t)b * C + c];
  out[c] = a;
}

// Training aux outputs of NeuralPointsRayMarching.forward
// (neural_points_volumetric_model.py:335-338) in the reference's compact layout
// [R'', SR, ...] (rays with ray_vcnt > 0, in ray order): the aggregator's
// normalised inverse-distance weight (point_aggregators.py:421-429, 803-804; the
// value before the conf factor) and ray_march's blend_weight = opacity * acc_T
// from the composite's opacity.  One wave per ray; lane = shading slot.
struct AuxArgs {
  int64_t R;
  int SR, K;
  const int32_t* n_filled;
  const int32_t* ray_off;
  const int32_t* ray_vcnt;
  const int32_t* ray_row;
  const int32_t* pidx;
  const float* sample_w;
  const float* xyz;
  const float* opacity;
  int64_t rows_max;
  float* weight;
  float* blend;
};

__global__ void __launch_bounds__(kCBlock) k_march_aux(AuxArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int SR = a.SR, K = a.K;
  for (int64_t r = wave0; r < a.R; r += nwaves) {
    if (a.ray_vcnt[r] <= 0) continue;
    const int64_t row = a.ray_row[r];
    if (row >= a.rows_max) continue;
    if (a.blend) {
      float op[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int s = lane + 64 * q;
        op[q] = s < SR ? a.opacity[r * SR + s] : 0.f;
      }
      // the exclusive cumprod of k_composite's march_slots on the same opacities
      const float f0 = (lane < SR) ? (1.f - op[0] + 1e-10f) : 1.f;
      const float f1 = (lane + 64 < SR) ? (1.f - op[1] + 1e-10f) : 1.f;
      const float i0 = wave_prod_scan_incl(f0);
      const float tot0 = __shfl(i0, 63);
      const float i1 = wave_prod_scan_incl(f1) * tot0;
      float e0 = __shfl_up(i0, 1), e1 = __shfl_up(i1, 1);
      if (lane == 0) {
        e0 = 1.f;
        e1 = tot0;
      }
      if (lane < SR) a.blend[row * SR + lane] = op[0] * e0;
      if (lane + 64 < SR) a.blend[row * SR + lane + 64] = op[1] * e1;
    }
    if (a.weight) {
      const int n = a.n_filled[r], off = a.ray_off[r];
      for (int s = lane; s < SR; s += 64) {
        float* wo = a.weight + (row * SR + s) * K;
        if (s >= n) {
          for (int k = 0; k < K; ++k) wo[k] = 0.f;
          continue;
        }
        const int64_t i = off + s;
        const float sw[3] = {a.sample_w[i * 3], a.sample_w[i * 3 + 1], a.sample_w[i * 3 + 2]};
        float wl[16];
        float sum = 0.f;
        for (int k = 0; k < K; ++k) {
          const int32_t p = a.pidx[i * K + k];
          float v = 0.f;
          if (p >= 0) {
            const float d0 = a.xyz[(int64_t)p * 3] - sw[0], d1 = a.xyz[(int64_t)p * 3 + 1] - sw[1],
                        d2 = a.xyz[(int64_t)p * 3 + 2] - sw[2];
            v = 1.f / fmaxf(sqrtf(d0 * d0 + d1 * d1 + d2 * d2), 1e-6f);
          }
          wl[k] = v;
          sum += v;
        }
        const float den = fmaxf(sum, 1e-8f);
        for (int k = 0; k < K; ++k) wo[k] = wl[k] / den;
      }
    }
  }
}

}  // namespace pnr

using namespace pnr;

static int composite_fwd(const pnr_rays* rays, const pnr_query_params* q, const pnr_query_bufs* b,
                         const pnr_composite_params* c, const float* feat, const uint16_t* feat_h, float* ray_color,
                         float* opacity, float* is_bg, int8_t* ray_mask, void* stream) {
  PNR_CHECK_ARG(rays && q && b && c && ray_color && opacity && is_bg && ray_mask,
                "composite: null pointer");
  PNR_CHECK_ARG(rays->campos_dev && rays->camrot_dev, "composite: camera required");
  PNR_CHECK_ARG(q->SR >= 1 && q->SR <= 128, "composite: SR=%d unsupported (1..128)", q->SR);
  PNR_CHECK_ARG(c->C >= 1 && c->C <= 128, "composite: C=%d unsupported (1..128)", c->C);
  if (rays->R == 0) return PNR_OK;
  CompArgs a;
  a.campos = rays->campos_dev;
  a.camrot = rays->camrot_dev;
  a.ray_cam = rays->ray_cam;
  a.R = rays->R;
  a.SR = q->SR;
  a.n_filled = b->n_filled;
  a.ray_off = b->ray_off;
  a.ray_vcnt = b->ray_vcnt;
  a.vflag = b->vflag;
  a.valid_off = b->valid_off;
  a.sample_p = b->sample_p;
  a.feat = feat;
  a.feat_h = feat_h;
  a.feat_rows = c->feat_rows > 0 ? c->feat_rows : INT64_MAX;
  a.vsize_z = c->vsize_z;
  a.unit = c->raydist_mode_unit;
  a.C = c->C;
  a.bg = c->bg_color;
  a.ray_color = ray_color;
  a.opacity = opacity;
  a.is_bg = is_bg;
  a.ray_mask = ray_mask;
  const unsigned grid = grid_for(rays->R * 64, kCBlock, 256 * 16);
  if (feat_h)
    hipLaunchKernelGGL(k_composite<true>, dim3(grid), dim3(kCBlock), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(k_composite<false>, dim3(grid), dim3(kCBlock), 0, as_stream(stream), a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_composite_fwd(const pnr_rays* rays, const pnr_query_params* q,
                                 const pnr_query_bufs* b, const pnr_composite_params* c,
                                 const float* feat, float* ray_color, float* opacity, float* is_bg,
                                 int8_t* ray_mask, void* stream) {
  return composite_fwd(rays, q, b, c, feat, nullptr, ray_color, opacity, is_bg, ray_mask, stream);
}

extern "C" int pnr_composite_fwd_hf(const pnr_rays* rays, const pnr_query_params* q,
                                    const pnr_query_bufs* b, const pnr_composite_params* c,
                                    const uint16_t* feat_h, float* ray_color, float* opacity, float* is_bg,
                                    int8_t* ray_mask, void* stream) {
  PNR_CHECK_ARG(feat_h && c && (c->C % 2) == 0, "composite_hf: feat_h required, C even");
  PNR_CHECK_ARG(((uintptr_t)feat_h & 15) == 0, "composite_hf: feat_h must be 16-B aligned");
  return composite_fwd(rays, q, b, c, nullptr, feat_h, ray_color, opacity, is_bg, ray_mask, stream);
}

extern "C" int pnr_ray_march_fwd(const float* ray_dist, const uint8_t* ray_valid, const float* feat,
                                 const float* bg, int64_t NR, int32_t SR, int32_t C, float* ray_color,
                                 float* opacity, float* acc_T, float* blend_w, float* bg_T,
                                 void* stream) {
  PNR_CHECK_ARG(ray_dist && ray_valid && feat && ray_color && opacity && acc_T && blend_w && bg_T,
                "ray_march: null pointer");
  PNR_CHECK_ARG(SR >= 1 && SR <= 128, "ray_march: SR=%d unsupported (1..128)", SR);
  PNR_CHECK_ARG(C >= 1, "ray_march: C must be >= 1");
  if (NR == 0) return PNR_OK;
  const unsigned grid = grid_for(NR * 64, kCBlock, 256 * 16);
  hipLaunchKernelGGL(k_ray_march_dense, dim3(grid), dim3(kCBlock), 0, as_stream(stream), ray_dist,
                     ray_valid, feat, bg, NR, SR, C, ray_color, opacity, acc_T, blend_w, bg_T);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_composite_bwd(const pnr_rays* rays, const pnr_query_params* q, const pnr_query_bufs* b,
                                 const pnr_composite_params* c, const float* feat, const float* d_ray_color,
                                 float* d_feat, void* stream) {
  PNR_CHECK_ARG(rays && q && b && c && feat && d_ray_color && d_feat, "composite_bwd: null pointer");
  PNR_CHECK_ARG(rays->campos_dev && rays->camrot_dev, "composite_bwd: camera required");
  PNR_CHECK_ARG(q->SR >= 1 && q->SR <= 128, "composite_bwd: SR=%d unsupported (1..128)", q->SR);
  PNR_CHECK_ARG(c->C >= 1 && c->C <= 128, "composite_bwd: C=%d unsupported (1..128)", c->C);
  if (rays->R == 0) return PNR_OK;
  CompBwdArgs a;
  a.f.campos = rays->campos_dev;
  a.f.camrot = rays->camrot_dev;
  a.f.ray_cam = rays->ray_cam;
  a.f.R = rays->R;
  a.f.SR = q->SR;
  a.f.n_filled = b->n_filled;
  a.f.ray_off = b->ray_off;
  a.f.ray_vcnt = b->ray_vcnt;
  a.f.vflag = b->vflag;
  a.f.valid_off = b->valid_off;
  a.f.sample_p = b->sample_p;
  a.f.feat = feat;
  a.f.feat_rows = c->feat_rows > 0 ? c->feat_rows : INT64_MAX;
  a.f.vsize_z = c->vsize_z;
  a.f.unit = c->raydist_mode_unit;
  a.f.C = c->C;
  a.f.bg = c->bg_color;
  a.f.ray_color = nullptr;
  a.f.opacity = nullptr;
  a.f.is_bg = nullptr;
  a.f.ray_mask = nullptr;
  a.d_color = d_ray_color;
  a.d_feat = d_feat;
  const unsigned grid = grid_for(rays->R * 64, kCBlock, 256 * 16);
  hipLaunchKernelGGL(k_composite_bwd, dim3(grid), dim3(kCBlock), 0, as_stream(stream), a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_ray_march_bwd_ex(const float* ray_dist, const uint8_t* ray_valid, const float* feat,
                                    const float* bg, int64_t NR, int32_t SR, int32_t C, const float* d_ray_color,
                                    const float* d_opacity, const float* d_acc_T, const float* d_blend_w,
                                    const float* d_bg_T, float* d_feat, float* d_ray_dist, void* stream) {
  PNR_CHECK_ARG(ray_dist && ray_valid && feat && d_ray_color && d_feat, "ray_march_bwd: null pointer");
  PNR_CHECK_ARG(SR >= 1 && SR <= 128, "ray_march_bwd: SR=%d unsupported (1..128)", SR);
  PNR_CHECK_ARG(C >= 1, "ray_march_bwd: C must be >= 1");
  if (NR == 0) return PNR_OK;
  MarchBwdArgs a = {ray_dist, ray_valid, feat, bg, NR, SR, C, d_ray_color, d_opacity, d_acc_T, d_blend_w, d_bg_T,
                    d_feat, d_ray_dist};
  const unsigned grid = grid_for(NR * 64, kCBlock, 256 * 16);
  hipLaunchKernelGGL(k_ray_march_dense_bwd, dim3(grid), dim3(kCBlock), 0, as_stream(stream), a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_ray_march_bwd(const float* ray_dist, const uint8_t* ray_valid, const float* feat,
                                 const float* bg, int64_t NR, int32_t SR, int32_t C, const float* d_ray_color,
                                 float* d_feat, void* stream) {
  return pnr_ray_march_bwd_ex(ray_dist, ray_valid, feat, bg, NR, SR, C, d_ray_color, nullptr, nullptr, nullptr,
                              nullptr, d_feat, nullptr, stream);
}

// Zero the device-counted rows of a capacity-sized buffer (pnr_zero_rows).
__global__ void __launch_bounds__(256) k_zero_rows(uint32_t* __restrict__ p, int64_t row_words,
                                                   const int32_t* __restrict__ n_dev, int64_t n_cap) {
  int64_t n = *n_dev;
  n = n < n_cap ? n : n_cap;
  const int64_t words = n * row_words;
  const int64_t w4 = words >> 2;
  uint4* q = reinterpret_cast<uint4*>(p);
  const bool vec = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (vec) {
    for (int64_t j = i; j < w4; j += stride) q[j] = make_uint4(0u, 0u, 0u, 0u);
    for (int64_t j = 4 * w4 + i; j < words; j += stride) p[j] = 0u;
  } else {
    for (int64_t j = i; j < words; j += stride) p[j] = 0u;
  }
}

extern "C" int pnr_zero_rows(void* p, int64_t row_bytes, const int32_t* n_dev, int64_t n_cap, void* stream) {
  PNR_CHECK_ARG(n_dev && n_cap >= 0 && row_bytes > 0 && row_bytes % 4 == 0 && (p || n_cap == 0),
                "zero_rows: bad args");
  if (n_cap == 0) return PNR_OK;
  const int64_t words = n_cap * (row_bytes / 4);
  const int64_t blocks = cdiv(cdiv(words, 4), 256);
  hipLaunchKernelGGL(k_zero_rows, dim3((unsigned)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048)), dim3(256), 0,
                     as_stream(stream), static_cast<uint32_t*>(p), row_bytes / 4, n_dev, n_cap);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// zero_one_loss of conf_coefficient (base_rendering_model.py:634-639: mean of
// log(v) + log(1 - v), v = clamp(cc, eps, 1 - eps)) from per-point entry counts
// (pnr_zero_one_loss_fwd / _bwd): cc_p = clamp(conf_p, 1e-4, 1) (gradiant_clamp's
// value, point_aggregators.py:724-726; its gradient passes straight through),
// E = R'' SR K entries, the empty ones gathered as point 0.  Per-block partials
// of (sum c_p f(v_p), sum c_p) in fixed order, then one block.
constexpr int kZoBlocks = 512;
__device__ __forceinline__ float zo_v(float conf, float eps) {
  const float cc = fminf(fmaxf(conf, 1e-4f), 1.f);
  return fminf(fmaxf(cc, eps), 1.f - eps);
}
__global__ void __launch_bounds__(256) k_zero_one_part(const float* __restrict__ conf, const float* __restrict__ cnt,
                                                       int64_t N, float eps, float* __restrict__ part) {
  __shared__ float r1[4], r0[4];
  float s1 = 0.f, s0 = 0.f;
  const int64_t per = cdiv(N, (int64_t)kZoBlocks);
  const int64_t b0 = blockIdx.x * per, b1 = b0 + per < N ? b0 + per : N;
  for (int64_t p = b0 + threadIdx.x; p < b1; p += 256) {
    const float c = cnt[p];
    if (c != 0.f) {
      const float v = zo_v(conf[p], eps);
      s1 += c * (logf(v) + logf(1.f - v));
      s0 += c;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s0 += __shfl_xor(s0, o);
  }
  if ((threadIdx.x & 63) == 0) {
    r1[threadIdx.x >> 6] = s1;
    r0[threadIdx.x >> 6] = s0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ((r1[0] + r1[1]) + r1[2]) + r1[3];
    part[2 * blockIdx.x + 1] = ((r0[0] + r0[1]) + r0[2]) + r0[3];
  }
}
// out[0] = loss, out[1] = the empty entries E - sum c (gathered as point 0), out[2] = E
__global__ void __launch_bounds__(64) k_zero_one_final(const float* __restrict__ part, const float* __restrict__ conf,
                                                       const int32_t* __restrict__ r_valid, int64_t srk, float eps,
                                                       float* __restrict__ out) {
  float s1 = 0.f, s0 = 0.f;
  for (int i = threadIdx.x; i < kZoBlocks; i += 64) {
    s1 += part[2 * i];
    s0 += part[2 * i + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s0 += __shfl_xor(s0, o);
  }
  if (threadIdx.x == 0) {
    const float E = (float)((double)*r_valid * (double)srk);
    const float empty = E - s0;
    const float v0 = zo_v(conf[0], eps);
    out[0] = E > 0.f ? (s1 + empty * (logf(v0) + logf(1.f - v0))) / E : 0.f;
    out[1] = empty;
    out[2] = E;
  }
}
__global__ void __launch_bounds__(256) k_zero_one_bwd(const float* __restrict__ conf, const float* __restrict__ cnt,
                                                      int64_t N, float eps, const float* __restrict__ fwd_out,
                                                      const float* __restrict__ g, float* __restrict__ d_conf) {
  const float E = fwd_out[2];
  const float scale = E > 0.f ? g[0] / E : 0.f;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
    const float c = cnt[p] + (p == 0 ? fwd_out[1] : 0.f);
    float d = 0.f;
    if (c != 0.f) {
      const float cc = fminf(fmaxf(conf[p], 1e-4f), 1.f);
      if (cc >= eps && cc <= 1.f - eps) {   // torch.clamp's gradient mask (inclusive)
        const float v = cc;
        d = c * scale * (1.f / v - 1.f / (1.f - v));
      }
    }
    d_conf[p] = d;
  }
}

extern "C" int pnr_zero_one_loss_fwd(const float* conf, const float* counts, int64_t N, const int32_t* r_valid,
                                     int64_t srk, float eps, float* partials, float* out, void* stream) {
  PNR_CHECK_ARG(conf && counts && r_valid && partials && out && N > 0 && srk > 0, "zero_one_loss_fwd: bad args");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_zero_one_part, dim3(kZoBlocks), dim3(256), 0, st, conf, counts, N, eps, partials);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_zero_one_final, dim3(1), dim3(64), 0, st, partials, conf, r_valid, srk, eps, out);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_zero_one_loss_bwd(const float* conf, const float* counts, int64_t N, float eps,
                                     const float* fwd_out, const float* g, float* d_conf, void* stream) {
  PNR_CHECK_ARG(conf && counts && fwd_out && g && d_conf && N > 0, "zero_one_loss_bwd: bad args");
  hipLaunchKernelGGL(k_zero_one_bwd, dim3(grid_for(N, 256, 2048)), dim3(256), 0, as_stream(stream), conf, counts, N,
                     eps, fwd_out, g, d_conf);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_weighted_colsum_scratch_floats(int32_t C, int64_t* out) {
  PNR_CHECK_ARG(out && C >= 1 && C <= 128, "weighted_colsum: C=%d unsupported (1..128)", C);
  *out = (int64_t)kColsumBlocks * C;
  return PNR_OK;
}

extern "C" int pnr_weighted_colsum(const float* w, const float* x, int64_t R, int32_t C, float* out, float* partials,
                                   void* stream) {
  PNR_CHECK_ARG(((w && x) || R == 0) && out && partials, "weighted_colsum: null pointer");
  PNR_CHECK_ARG(C >= 1 && C <= 128, "weighted_colsum: C=%d unsupported (1..128)", C);
  PNR_CHECK_ARG(R >= 0, "weighted_colsum: R < 0");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_wcolsum_part, dim3(kColsumBlocks), dim3(256), 0, st, w, x, R, C, partials);
  PNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_wcolsum_final, dim3(1), dim3(128), 0, st, partials, C, out);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

extern "C" int pnr_march_aux(const pnr_rays* rays, const pnr_query_params* q, const pnr_query_bufs* b,
                             const float* xyz, const float* opacity, int64_t rows_max, float* weight,
                             float* blend_weight, void* stream) {
  PNR_CHECK_ARG(rays && q && b, "march_aux: null pointer");
  PNR_CHECK_ARG(q->SR >= 1 && q->SR <= 128, "march_aux: SR=%d unsupported (1..128)", q->SR);
  PNR_CHECK_ARG(q->K >= 1 && q->K <= 16, "march_aux: K=%d unsupported (1..16)", q->K);
  PNR_CHECK_ARG(!weight || xyz, "march_aux: weight needs xyz");
  PNR_CHECK_ARG(!blend_weight || opacity, "march_aux: blend_weight needs opacity");
  if (rays->R == 0 || rows_max <= 0 || (!weight && !blend_weight)) return PNR_OK;
  AuxArgs a = {rays->R, q->SR, q->K, b->n_filled, b->ray_off, b->ray_vcnt, b->ray_row, b->pidx, b->sample_w,
               xyz, opacity, rows_max, weight, blend_weight};
  const unsigned grid = grid_for(rays->R * 64, kCBlock, 256 * 16);
  hipLaunchKernelGGL(k_march_aux, dim3(grid), dim3(kCBlock), 0, as_stream(stream), a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
