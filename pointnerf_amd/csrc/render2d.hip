// The fork's 2-D neural renderer: NeuralRenderer(input_dim
// = 128) of models/neural_render/neural_renderer.py:24-104 applied to the
// composited [H, W, 128] feature image (neural_points_volumetric_model.py:343-344):
//   rgb  = conv_rgb0(x)                      3x3, 128 -> 3
//   net0 = lrelu_0.2(conv0(x))               3x3, 128 -> 64
//   rgb += conv_rgb1(net0)                   3x3, 64 -> 3
//   net1 = lrelu_0.2(conv1(net0))            3x3, 64 -> 32
//   rgb += conv_rgb2(net1)                   3x3, 32 -> 3
//   out  = sigmoid(rgb)                      (final_actvn)
// (n_feat == input_dim, so conv_in is the identity; img_size 64 -> 2 blocks,
// no norm, no upsampling.)
//
// CDNA4 mapping: each stage is one launch of k_conv3x3, an implicit GEMM on
// v_mfma_f32_32x32x2_f32 (exact fp32): rows = output channels of the stage's
// trunk conv (64, 32, none), columns = 32 consecutive pixels of an image row,
// k = (tap, input channel); the 3-channel rgb skip conv runs on VALU in the
// MFMAs' shadow (each lane already holds the B operand value it needs: 3 FMAs
// per k-step) instead of as a 32-row MFMA tile with 29 zero rows.
// A 4-wave workgroup owns 128 pixels of one row; the 3 input rows x 130
// pixels of a 32-channel slice are staged in LDS (pixel pitch 33 floats,
// conflict-free B reads), so each input element is read from HBM ~3 times
// (once per output row) instead of 9.  Zero padding 1 as in the reference.
#include "pnr_common.h"
#include "agg_common.h"

namespace pnr {

typedef float f32x16r __attribute__((ext_vector_type(16)));

constexpr int kRPx = 128;              // pixels per workgroup (4 waves x 32)
// input channels staged per LDS chunk (16: half the LDS, more workgroups per
// CU, twice the barriers -- measured 2.50 -> 3.18 ms forward, not kept)
constexpr int kRCh = 32;
constexpr int kRPitch = kRCh + 1;      // floats per staged pixel
constexpr int kRRowPx = kRPx + 2;      // staged pixels per input row (halo 1)
// Output rows per workgroup tile.  2 (every weight fragment feeding two rows'
// MFMAs, 4 staged input rows) measured 3.01 vs 2.93 ms for the 800x800 forward,
// 4 rows 3.56 ms: weight fetch is not what bounds the kernel; 1 is kept.
constexpr int kROut = 1;
// Timing ablations (tools/build_variant.sh, 800x800 forward 2.95 ms): 1 = weight
// fragments from L1 (2.01 ms), 2 = fixed B rows (2.53), 4 = no input staging
// (2.53), 7 = all three (1.71).  Staging the weight fragments in LDS per 8
// k-steps for the 4 waves (double-buffered) measured 3.19 ms: the extra barriers
// cost more than the L2 fetch they save; not kept.
constexpr int kConvRW = 6;   // weight-fragment prefetch depth in k-steps (12 / 18: same 2.94 ms)
constexpr int kRRows = kROut + 2;      // staged input rows
constexpr size_t kRLds = (size_t)kRRows * kRRowPx * kRPitch * sizeof(float);

struct ConvArgs {
  const float* in;     // [H, W, Cin]
  int H, W, Cin;
  const float* wf;     // fragment-packed [ROWS, 9 * Cin] (k = tap * Cin + ci), ROWS = 32 * NT
  const float* bias;   // [ROWS] (trunk bias, rgb bias, zeros)
  int cout;            // trunk output channels (0 = rgb only)
  float* out;          // [H, W, ldo] = lrelu(trunk)   (cout > 0)
  float* rgb;          // [H, W, 3] accumulated (first stage writes, later add)
  int rgb_mode;        // 0: rgb = part, 1: rgb += part, 2: out_rgb = sigmoid(rgb + part),
                       // (BWD kernels: data gradient, out = acc * lrelu'(act), act may be NULL, no bias)
  float slope;
  int ldo;             // floats per output pixel row (>= cout)
  const float* act;    // [H, W, cout] forward activation whose LeakyReLU mask applies (mode 3)
  int cin_real;        // input channels >= cin_real are zero padding: their k-steps are skipped
  const float* wrgb;   // forward: the stage's rgb conv [3, 9 * Cin] (k = tap * Cin + ci), on VALU
  const float* brgb;   // [3]
};

// BWD: 0 forward, 1 data gradient, 2 data gradient times the LeakyReLU mask of a.act
// (Cin as a template constant, folding every address to immediates, measured
// 2.57 vs 2.50 ms forward: the runtime Cin is kept.)
template <int NT, int BWD>
__global__ void __launch_bounds__(256, 2) k_conv3x3(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_r[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int segs = (a.W + kRPx - 1) / kRPx;
  const int64_t ntiles = (int64_t)((a.H + kROut - 1) / kROut) * segs;
  constexpr int NTA = NT > 0 ? NT : 1;   // (NT = 0: the rgb-only last forward stage)
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int y0 = (int)(tile / segs) * kROut;
    const int x0 = (int)(tile % segs) * kRPx;
    f32x16r acc[kROut][NTA];
    float racc[3] = {0.f, 0.f, 0.f};   // forward: this lane's half of the pixel's rgb sums
#pragma unroll
    for (int o = 0; o < kROut; ++o)
#pragma unroll
      for (int T = 0; T < NT; ++T) acc[o][T] = (f32x16r){0.f};
    for (int ci0 = 0; ci0 < a.Cin; ci0 += kRCh) {
      // stage rows y0-1 .. y0+kROut, pixels x0-1 .. x0+128, channels ci0 .. ci0+31 (zero padded)
      for (int i = threadIdx.x; i < kRRows * kRRowPx * (kRCh / 4); i += blockDim.x) {
        const int q = i % (kRCh / 4);
        const int px = (i / (kRCh / 4)) % kRRowPx;
        const int r = i / ((kRCh / 4) * kRRowPx);
        const int yy = y0 - 1 + r, xx = x0 - 1 + px;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
          v = *reinterpret_cast<const float4*>(a.in + ((int64_t)yy * a.W + xx) * a.Cin + ci0 + 4 * q);
        float* d = lds_r + (r * kRRowPx + px) * kRPitch + 4 * q;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
      }
      __syncthreads();
      // this wave's 32 pixels: x0 + 32 wid + c, of both output rows: every weight
      // fragment feeds kROut * NT MFMAs
      const int pcol = 32 * wid + c;
      // k-steps of this chunk in (tap, channel-pair) order; weight fragments
      // are software-pipelined kRW steps ahead across tap boundaries
      constexpr int kRW = kConvRW;
      constexpr int kSteps = 9 * (kRCh / 2);
      const float* wp = a.wf + lane;
      auto wstep = [&](int i) {   // global k-step of chunk step i
        const int tap = i / (kRCh / 2), s = i % (kRCh / 2);
        return (tap * a.Cin + ci0) / 2 + s;
      };
      float wr[kRW][NTA];
#pragma unroll
      for (int d = 0; d < kRW; ++d)
#pragma unroll
        for (int T = 0; T < NT; ++T) wr[d][T] = wp[(wstep(d) * NT + T) * 64];
      (void)wr;
#pragma unroll
      for (int i0 = 0; i0 < kSteps; i0 += kRW) {
#pragma unroll
        for (int d = 0; d < kRW; ++d) {
          const int i = i0 + d;
          // (channel pairs wholly in the zero padding of the backward's cat images
          // -- the 3 rgb-gradient channels padded to 32 -- add nothing: their
          // MFMAs are skipped)
          if (i < kSteps) {
            const int tap = i / (kRCh / 2), s = i % (kRCh / 2);
            const int dy = tap / 3, dx = tap % 3;
            if (BWD == 0 || ci0 + 2 * s < a.cin_real) {
#pragma unroll
              for (int o = 0; o < kROut; ++o) {
                const float b = lds_r[((dy + o) * kRRowPx + pcol + dx) * kRPitch + h + 2 * s];
#pragma unroll
                for (int T = 0; T < NT; ++T)
                  acc[o][T] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[d][T], b, acc[o][T], 0, 0, 0);
                if (BWD == 0) {
                  // the 3 rgb rows on VALU in the MFMAs' shadow: lane (c, h) holds
                  // channel ci0 + 2 s + h of its pixel's tap; both weights are uniform
                  // (scalar loads), the lane picks its own
                  const float* wq = a.wrgb + tap * a.Cin + ci0 + 2 * s;
#pragma unroll
                  for (int j = 0; j < 3; ++j) {
                    const float w0 = wq[j * 9 * a.Cin], w1 = wq[j * 9 * a.Cin + 1];
                    racc[j] = fmaf(h ? w1 : w0, b, racc[j]);
                  }
                }
              }
            }
            if (i + kRW < kSteps) {   // the ring refill runs for skipped steps too
#pragma unroll
              for (int T = 0; T < NT; ++T) wr[d][T] = wp[(wstep(i + kRW) * NT + T) * 64];
            }
          }
        }
      }
      __syncthreads();
    }
    // epilogue: trunk rows 0..cout-1 (lrelu) from the MFMA tiles; forward: the
    // rgb sums of the lane halves (even / odd channels) combined, + bias
    const int xo = x0 + 32 * wid + c;
#pragma unroll
    for (int j = 0; j < 3; ++j) racc[j] += __shfl_xor(racc[j], 32);
#pragma unroll
    for (int o = 0; o < kROut; ++o) {
      const int y = y0 + o;
      if (xo >= a.W || y >= a.H) continue;
      const int64_t pix = (int64_t)y * a.W + xo;
      if (BWD) {
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = 32 * T + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (co < a.cout) {
              // LeakyReLU'(z) from the saved output: sign(lrelu(z)) = sign(z), slope > 0
              const float m = BWD == 1 || a.act[pix * a.cout + co] > 0.f ? 1.f : a.slope;
              a.out[pix * a.ldo + co] = acc[o][T][r] * m;
            }
          }
      } else {
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = 32 * T + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float v = acc[o][T][r] + a.bias[co];
            a.out[pix * a.ldo + co] = v > 0.f ? v : v * a.slope;
          }
        if (h == 0) {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const float v = racc[j] + a.brgb[j];
            float* op = a.rgb + pix * 3 + j;
            if (a.rgb_mode == 0) *op = v;
            else if (a.rgb_mode == 1) *op += v;
            else *op = 1.f / (1.f + expf(-(*op + v)));
          }
        }
      }
    }
  }
}

constexpr int kConvGrid = 256 * 3;   // workgroups of the persistent tile loop (one per tile: same time)
template <int NT, int BWD = 0>
static int launch_conv(const ConvArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3x3<NT, BWD>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRLds));
    attr = true;
  }
  const int64_t tiles = (int64_t)((a.H + kROut - 1) / kROut) * ((a.W + kRPx - 1) / kRPx);
  hipLaunchKernelGGL((k_conv3x3<NT, BWD>), dim3(grid_for(tiles, 1, kConvGrid)), dim3(256), kRLds, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// ------------------------------------------------------------------ backward
// Per stage the stacked rows' output gradient dY = [d trunk (pre-activation),
// d rgb, zeros] is one [H, W, M] image ("cat" buffer, M = the stage's stacked
// rows).  Its data gradient is a forward 3x3 convolution of dY with the
// flipped, channel-transposed weights (k_conv3x3 in mode 3, the LeakyReLU mask
// of the layer below in the epilogue); its weight gradient
//   dW[m, tap, ci] = sum_p dY[p, m] X[p + off(tap), ci],  db[m] = sum_p dY[p, m]
// is k_conv_wgrad: an implicit-GEMM A^T B over the pixels on fp32 MFMA, dY and
// X chunks staged in LDS (below), partials summed over the pixel splits in a
// fixed order (deterministic).

// g = d_out * s (1 - s) (the sigmoid's gradient on the saved output s) into the
// rgb slots of the three cat buffers; their pad channels zeroed.
__global__ void k_nr_rgb_grad(const float* __restrict__ d_out, const float* __restrict__ out_rgb, int64_t npix,
                              float* __restrict__ cat2, float* __restrict__ cat1, float* __restrict__ cat0) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    float g[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float s = out_rgb[p * 3 + j];
      g[j] = d_out[p * 3 + j] * (s * (1.f - s));
    }
    float* c2 = cat2 + p * 32;   // [g, 0 x 29]
    float* c1 = cat1 + p * 64;   // [dz1 (32), g, 0 x 29]
    float* c0 = cat0 + p * 96;   // [dz0 (64), g, 0 x 29]
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const float v = j < 3 ? g[j] : 0.f;
      c2[j] = v;
      c1[32 + j] = v;
      c0[64 + j] = v;
    }
  }
}

struct WgradArgs {
  const float* dy;     // [npix, M]
  const float* x;      // [npix, Cin] forward input of the stage
  int H, W, M, Cin;
  int64_t chunk;       // pixels per split (multiple of 32)
  float* part;         // [nsplit][M * 9 * Cin + M]
};

// One 4-wave workgroup per (pixel split, kernel row ky): all M rows x the 3 taps
// (ky, 0..2) x all Cin columns of dW.  Per 32-pixel chunk the dY rows
// (32 x M, contiguous) and the 34 source pixels of the row above / at / below
// (p0 + (ky-1) W - 1 .. +33, contiguous, zero outside the image) are staged in LDS
// with float4 loads, the next chunk's loads in flight during this chunk's MFMAs;
// a lane's B operand for tap kx is the staged pixel (p - p0) + kx, zeroed when
// x + kx - 1 leaves the row.  So every dY element is read from HBM 3 times and
// every X element 3 times (not 9 x Cin/32 and 9 x M/32 as one wave per tap and
// tile would).  Wave w: column tiles j = w, w + 4, w + 8 of the 3 Cin/32
// (tap, channel-tile) pairs, all M/32 row tiles.
// (Dealing stage 1's 12 (column, row) tile pairs 3 per wave instead of 4 / 4 /
// 2 / 2 measured no faster: fwd + bwd 8.17 vs 8.10 ms.)
template <int MT, int NC, bool VR>
__global__ void __launch_bounds__(256, 2) k_conv_wgrad(WgradArgs a) {
  constexpr int M = 32 * MT, C = 32 * NC;
  constexpr int PA = M % 64 == 0 ? M + 32 : M;      // LDS pitches: half-waves 32 banks apart
  constexpr int PB = C % 64 == 0 ? C + 32 : C;
  constexpr int NA4 = 32 * M / 4, NB4 = 34 * C / 4;
  constexpr int RA = (NA4 + 255) / 256, RB = (NB4 + 255) / 256;
  constexpr int NJ = 3 * NC, JW = (NJ + 3) / 4;     // column tiles, per wave
  __shared__ __attribute__((aligned(16))) float as[32 * PA];
  __shared__ __attribute__((aligned(16))) float bs[34 * PB];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int split = blockIdx.x, ky = blockIdx.y;
  const int npix = a.H * a.W;                 // < 2^30 (checked by the caller)
  const int pbeg = split * (int)a.chunk;
  const int pend = pbeg + (int)a.chunk < npix ? pbeg + (int)a.chunk : npix;
  float4 ra[RA], rb[RB];
  auto load = [&](int p0) {
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      const int i = tid + 256 * j, e = 4 * i, r = e / M;
      ra[j] = i < NA4 && p0 + r < pend ? *reinterpret_cast<const float4*>(a.dy + (int64_t)p0 * M + e)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int s0 = p0 + (ky - 1) * a.W - 1;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int i = tid + 256 * j, e = 4 * i, r = e / C, ci = e - r * C;
      const int sp = s0 + r;
      rb[j] = i < NB4 && sp >= 0 && sp < npix ? *reinterpret_cast<const float4*>(a.x + (int64_t)sp * C + ci)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      const int i = tid + 256 * j, e = 4 * i, r = e / M, m = e - r * M;
      if (i < NA4) *reinterpret_cast<float4*>(as + r * PA + m) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int i = tid + 256 * j, e = 4 * i, r = e / C, ci = e - r * C;
      if (i < NB4) *reinterpret_cast<float4*>(bs + r * PB + ci) = rb[j];
    }
  };
  // VR: row tiles 0 .. MT-2 (the trunk's dz rows) on MFMA; the last tile holds
  // the 3 rgb-gradient rows (+ 29 zero rows): those 3 rows run on VALU, each lane
  // multiplying its B value by the 3 g values of its pixel (LDS broadcasts).
  // (stage 1, MT = 2: measured 0.85 -> 1.0 ms with VR, so there all rows stay on MFMA)
  constexpr int MTM = VR ? MT - 1 : MT, MTA = MTM > 0 ? MTM : 1, NR = VR ? 3 : 0;
  f32x16r acc[JW][MTA];
#pragma unroll
  for (int u = 0; u < JW; ++u)
#pragma unroll
    for (int t = 0; t < MTM; ++t) acc[u][t] = (f32x16r){0.f};
  float racc[JW][3];
#pragma unroll
  for (int u = 0; u < JW; ++u)
#pragma unroll
    for (int j = 0; j < 3; ++j) racc[u][j] = 0.f;
  (void)racc;
  float cs = 0.f;
  load(pbeg);
  put();
  __syncthreads();
  for (int p0 = pbeg; p0 < pend; p0 += 32) {
    const bool more = p0 + 32 < pend;
    if (more) load(p0 + 32);   // in flight during the MFMAs
    if (ky == 0 && tid < M) {
#pragma unroll 8
      for (int r = 0; r < 32; ++r) cs += as[r * PA + tid];
    }
#pragma unroll 4
    for (int s2 = 0; s2 < 16; ++s2) {
      const int kp = 2 * s2 + h;
      const int x = (p0 + kp) % a.W;
      float av[MTA], gv[3];
#pragma unroll
      for (int t = 0; t < MTM; ++t) av[t] = as[kp * PA + 32 * t + c];
#pragma unroll
      for (int jj = 0; jj < NR; ++jj) gv[jj] = as[kp * PA + 32 * MTM + jj];
#pragma unroll
      for (int u = 0; u < JW; ++u) {
        const int j = wid + 4 * u;
        if (j < NJ) {
          const int kx = j / NC, nc = j - kx * NC;
          const int xs = x + kx - 1;
          const float b = xs >= 0 && xs < a.W ? bs[(kp + kx) * PB + 32 * nc + c] : 0.f;
#pragma unroll
          for (int t = 0; t < MTM; ++t) acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], b, acc[u][t], 0, 0, 0);
#pragma unroll
          for (int jj = 0; jj < NR; ++jj) racc[u][jj] = fmaf(gv[jj], b, racc[u][jj]);
        }
      }
    }
    __syncthreads();
    if (more) {
      put();
      __syncthreads();
    }
  }
  const int N = 9 * C;
  float* out = a.part + (int64_t)split * ((int64_t)M * N + M);
  // C/D layout: row = (r&3) + 8(r>>2) + 4h, col = c
#pragma unroll
  for (int u = 0; u < JW; ++u) {
    const int j = wid + 4 * u;
    if (j >= NJ) continue;
    const int kx = j / NC, nc = j - kx * NC;
    const int col = (3 * ky + kx) * C + 32 * nc + c;
#pragma unroll
    for (int t = 0; t < MTM; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) out[(int64_t)(32 * t + (r & 3) + 8 * (r >> 2) + 4 * h) * N + col] = acc[u][t][r];
#pragma unroll
    for (int jj = 0; jj < NR; ++jj) {   // the two lane halves' pixels combined
      const float v = racc[u][jj] + __shfl_xor(racc[u][jj], 32);
      if (h == 0) out[(int64_t)(32 * MTM + jj) * N + col] = v;
    }
  }
  if (ky == 0 && tid < M) out[(int64_t)M * N + tid] = cs;
}

// out[i] = sum_s part[s][i], s ascending (fixed order); entries [z0, z1) (the
// zero-padding rows no split writes) are 0.
__global__ void k_sum_splits(const float* __restrict__ part, int64_t n, int nsplit, float* __restrict__ out,
                             int64_t z0, int64_t z1) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    if (i >= z0 && i < z1) {
      out[i] = 0.f;
      continue;
    }
    for (int q = 0; q < nsplit; ++q) s += part[(int64_t)q * n + i];
    out[i] = s;
  }
}

static void wgrad_plan(int64_t npix, int M, int Cin, int* nsplit, int64_t* chunk, int px = 32) {
  // ~2 workgroups per CU over the 3 kernel rows, >= 8 chunks of px pixels per split
  int64_t s = cdiv((int64_t)512, (int64_t)3);
  const int64_t maxs = cdiv(npix > 0 ? npix : 1, (int64_t)8 * px);
  if (s > maxs) s = maxs;
  int64_t ch = cdiv(npix > 0 ? npix : 1, s);
  ch = cdiv(ch, px) * px;
  *chunk = ch;
  *nsplit = (int)(npix > 0 ? cdiv(npix, ch) : 1);
  (void)M;
  (void)Cin;
}

static size_t wgrad_scratch(int64_t npix, int M, int Cin) {
  int ns;
  int64_t ch;
  wgrad_plan(npix, M, Cin, &ns, &ch);
  return (size_t)ns * ((size_t)M * 9 * Cin + M) * sizeof(float);
}

template <int MT, int NC, bool VR>
static int launch_wgrad(const float* dyb, const float* x, int H, int W, int Cin, float* part, float* dw,
                        hipStream_t st) {
  WgradArgs g;
  g.dy = dyb;
  g.x = x;
  g.H = H;
  g.W = W;
  g.M = 32 * MT;
  g.Cin = Cin;
  int ns;
  wgrad_plan((int64_t)H * W, g.M, Cin, &ns, &g.chunk);
  g.part = part;
  hipLaunchKernelGGL((k_conv_wgrad<MT, NC, VR>), dim3(ns, 3), dim3(256), 0, st, g);
  PNR_LAUNCH_CHECK();
  const int64_t n = (int64_t)g.M * 9 * Cin + g.M;
  const int64_t z0 = VR ? (int64_t)(g.M - 32 + 3) * 9 * Cin : 0, z1 = VR ? (int64_t)g.M * 9 * Cin : 0;   // pad rows
  hipLaunchKernelGGL(k_sum_splits, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, part, n, ns, dw, z0, z1);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// ------------------------------------------------------------- fp32h2 convs
// The same convolutions with fp32 accuracy on v_mfma_f32_32x32x16_f16 (the
// MLP's fp32h2 split, DESIGN §13, applied to the 2-D renderer): every staged
// input value x is split as x = xh + 2^-11 xl (f16 planes, splith) and every
// weight as W' = Wh + 2^-11 Wl (frag_pack_h2, per-stage scale 2^-s so
// |W'| < 16), and W.x = 2^-11 (Ws.xh + Wl.xh + Wh.xl), Ws = 2^11 Wh: three f16
// products with fp32 accumulation per 16 k, instead of eight 32x32x2 fp32
// MFMAs (5.3x the MFMA rate).
// Range: each image is staged times 2^e (exact), e chosen on the device from
// the image's max |value| (an absmax word its producer atomicMax-es: the
// previous stage's epilogue, k_nr_absmax, or the rgb-gradient kernel) so that
// max |x 2^e| lies in [2^14, 2^15): no f16 overflow for any input magnitude,
// and tiny images (gradients) keep their relative precision; no host sync and
// no fallback path.  The stacked rows [trunk; rgb; 0] all run as MFMA tiles
// (the rgb rows' tile: 3 live rows of 32; the MFMAs are cheap at this rate).
constexpr int kHPx = 128;                 // pixels per tile (4 waves x 32)
// conv tile: output rows x staged channels per chunk (A/B on one box, 800^2
// forward / forward + backward: 1 x 32 1.35 / 4.55 ms, 1 x 16 1.23 / 4.68,
// 2 x 16 1.00 / 4.31 -- kept; 2 x 32 spills at NT = 3)
constexpr int kConvRO = 2, kConvCH = 16;
constexpr int kHRowPx = kHPx + 2;
constexpr int kHWD = 3;                   // weight fragments prefetched this many k-steps ahead
constexpr int kWS = 16;                   // absmax words 64 B apart (no shared L2 line between them)
// staged f16 per pixel per plane for a CH-channel chunk: 80 B (32 ch) / 48 B (16 ch)
// rows, 5 / 3 16-B slots: the ds_read_b128 lane groups hit 16 distinct slots
template <int CH>
constexpr int conv_pitch() { return CH + 8; }
template <int RO, int CH>
constexpr size_t conv_h2_lds() {
  return (size_t)(RO + 2) * kHRowPx * 2 * conv_pitch<CH>() * sizeof(_Float16);
}

// 2^e with max|x| 2^e in [2^14, 2^15) from the image's absmax bits (1 for an
// all-zero or non-finite image, whose infs / NaNs then propagate as in fp32).
__device__ __forceinline__ float img_scale(const unsigned* w) {
  const float m = __uint_as_float(*w);
  if (!(m > 0.f) || !(m <= 3.0e38f)) return 1.f;
  int E;
  (void)frexpf(m, &E);
  int e = 15 - E;
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  return ldexpf(1.f, e);
}
// running max |v|; a NaN counts as +inf (its image then stages unscaled)
__device__ __forceinline__ float amax_upd(float m, float v) {
  const float a = fabsf(v);
  return a != a ? __builtin_inff() : fmaxf(m, a);
}
__device__ __forceinline__ void amax_commit(float m, unsigned* w) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(w, __float_as_uint(m));
}

__device__ __forceinline__ void amax_commit_block(float& m, unsigned* w, float* red);

__global__ void k_nr_absmax(const float4* __restrict__ x, int64_t n4, unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    m = amax_upd(amax_upd(amax_upd(amax_upd(m, v.x), v.y), v.z), v.w);
  }
  amax_commit_block(m, out, red);
}

struct ConvH2Args {
  const float* in;          // [H, W, Cin] fp32, Cin % 32 == 0
  int H, W, Cin;
  const unsigned* in_max;   // absmax bits of `in`
  const uint4* wp;          // frag_pack_h2 of the stacked rows [32 NT, 9 Cin] (k = tap * Cin + ci)
  const float* wscale;      // its 2^(s - 11) (device)
  const float* bias;        // forward: [32 NT] stacked biases (trunk, rgb, 0)
  int cout;                 // trunk rows (forward) / rows written (data gradient)
  float* out;               // [H, W, ldo]
  int ldo;
  unsigned* out_max;        // absmax bits of `out` (may be NULL)
  float* rgb;               // forward: [H, W, 3], rows cout .. cout + 2 (rgb_mode as ConvArgs)
  int rgb_mode;
  float slope;
  const float* act;         // BWD 2: [H, W, cout] forward activation whose LeakyReLU mask applies
  int cin_real;             // BWD: input channels >= cin_real are zero padding (skipped)
};

// Block max of per-thread |value| maxima -> one atomicMax per workgroup (every
// wave's atomic to one word serialises in L2: measured +0.2 ms per launch).
__device__ __forceinline__ void amax_commit_block(float& m, unsigned* w, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
    if (m > 0.f) atomicMax(w, __float_as_uint(m));
  }
}

// BWD: 0 forward, 1 data gradient, 2 data gradient times lrelu'(act).  RO
// output rows per tile; a 4-wave workgroup owns RO rows x 128 pixels, wave w
// pixels 32 w .. 32 w + 31 of every row.  The (tile, chunk) sequence is
// software-pipelined: the next chunk's global loads (the next tile's first
// chunk after a tile's last) are issued into registers before this chunk's
// MFMAs and split into the LDS planes after them.
template <int NT, int BWD, int RO, int CH>
__global__ void __launch_bounds__(256, 2) k_conv3x3_h2(ConvH2Args a) {
  extern __shared__ __attribute__((aligned(16))) _Float16 lds_h[];
  constexpr int PH = conv_pitch<CH>();
  constexpr int PL = (RO + 2) * kHRowPx * PH;    // f16 per plane
  constexpr int NST = ((RO + 2) * kHRowPx * (CH / 4) + 255) / 256;   // staged float4 per thread
  constexpr int KS = 9 * (CH / 16);              // k-steps per chunk
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int segs = (a.W + kHPx - 1) / kHPx;
  const int64_t ntiles = (int64_t)((a.H + RO - 1) / RO) * segs;
  const float xs = img_scale(a.in_max);
  const float osc = *a.wscale / xs;
  const int ktap = a.Cin / 16;             // k-steps per tap
  const uint4* wp = a.wp + lane;
  constexpr int WD = NT * RO >= 4 ? 2 : kHWD;   // weight ring depth (2 k-steps where 3 would spill)
  float amax = 0.f;
  // staged channels of chunk ci0 (the backward's cat images: zero-padding tails skipped)
  auto nreal_of = [&](int ci0) {
    if (!BWD) return ci0 < a.Cin ? CH : 0;
    const int r = (ci0 < a.Cin ? a.cin_real : 0) - ci0;
    return r <= 0 ? 0 : (r >= CH ? CH : (r + 15) / 16 * 16);
  };
  float4 pre[NST];
  // branch-free: every lane loads (an in-image pixel for the halo / padding
  // slots) and zeroes afterwards, so the loads issue back to back and stay in
  // flight across the MFMAs (sched_barrier: not sunk to their use)
  unsigned pre_ok = 0;
  auto load = [&](int64_t tile, int ci0, int nq) {
    const int y0 = (int)(tile / segs) * RO, x0 = (int)(tile % segs) * kHPx;
    pre_ok = 0;
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int q = i % nq, px = (i / nq) % kHRowPx, r = i / (nq * kHRowPx);
      const int yy = y0 - 1 + r, xx = x0 - 1 + px;
      const bool ok = r < RO + 2 && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      const int yc = ok ? yy : 0, xc = ok ? xx : 0;
      pre[u] = *reinterpret_cast<const float4*>(a.in + ((int64_t)yc * a.W + xc) * a.Cin + ci0 + 4 * (ok ? q : 0));
      pre_ok |= (unsigned)ok << u;
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto put = [&](int nq) {
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int q = i % nq, px = (i / nq) % kHRowPx, r = i / (nq * kHRowPx);
      if (r >= RO + 2) continue;
      const float sc = (pre_ok >> u) & 1u ? xs : 0.f;   // (a NaN / inf pixel of the halo: 0 * x is not 0)
      const float4 v = (pre_ok >> u) & 1u ? pre[u] : make_float4(0.f, 0.f, 0.f, 0.f);
      unsigned h0, h1, l0, l1;
      splith(v.x * sc, v.y * sc, h0, l0);
      splith(v.z * sc, v.w * sc, h1, l1);
      _Float16* d = lds_h + (r * kHRowPx + px) * PH + 4 * q;
      *reinterpret_cast<uint2*>(d) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(d + PL) = make_uint2(l0, l1);
    }
  };
  f32x16 acc[RO][NT];
  int64_t tile = blockIdx.x;
  int ci0 = 0, nreal = nreal_of(0);
  if (tile < ntiles) load(tile, 0, nreal / 4);
  while (tile < ntiles) {
    if (ci0 == 0) {
#pragma unroll
      for (int o = 0; o < RO; ++o)
#pragma unroll
        for (int T = 0; T < NT; ++T) acc[o][T] = (f32x16){0.f};
    }
    put(nreal / 4);
    __syncthreads();
    int nci0 = ci0 + CH;
    int64_t ntile = tile;
    int nnreal = nreal_of(nci0);
    if (nnreal == 0) {
      nci0 = 0;
      ntile = tile + gridDim.x;
      nnreal = nreal_of(0);
    }
    const int pcol = 32 * wid + c;
    // chunk step i = (CH / 16) tap + s: k-step tap * ktap + ci0 / 16 + s; weights WD steps ahead
    auto wstep = [&](int i) { return (i / (CH / 16)) * ktap + (ci0 >> 4) + i % (CH / 16); };
    uint4 wh[WD][NT], wl[WD][NT];
#pragma unroll
    for (int d = 0; d < WD; ++d)
#pragma unroll
      for (int T = 0; T < NT; ++T) {
        wh[d][T] = wp[((wstep(d) * NT + T) * 2 + 0) * 64];
        wl[d][T] = wp[((wstep(d) * NT + T) * 2 + 1) * 64];
      }
    __builtin_amdgcn_sched_barrier(0);
    // the next chunk's staging loads, in flight during the MFMAs (issued after the
    // weight ring's first loads: vmcnt counts in order, so the first MFMAs do not
    // wait for them; the ring's refills still do, WD steps later)
    if (ntile < ntiles) load(ntile, nci0, nnreal / 4);
#pragma unroll
    for (int i0 = 0; i0 < KS; i0 += WD) {
#pragma unroll
      for (int d = 0; d < WD; ++d) {
        const int i = i0 + d;
        if (i >= KS) break;
        const int tap = i / (CH / 16), s = i % (CH / 16);
        const int dy = tap / 3, dx = tap % 3;
        if (!BWD || 16 * s < nreal) {
          uint4 xh[RO], xl[RO];
#pragma unroll
          for (int o = 0; o < RO; ++o) {
            const _Float16* b = lds_h + ((dy + o) * kHRowPx + pcol + dx) * PH + 16 * s + 8 * h;
            xh[o] = *reinterpret_cast<const uint4*>(b);
            xl[o] = *reinterpret_cast<const uint4*>(b + PL);
          }
#pragma unroll
          for (int T = 0; T < NT; ++T) {
            const uint4 ws = f16x8_scale2048(wh[d][T]);
#pragma unroll
            for (int o = 0; o < RO; ++o) {
              acc[o][T] = mfma_f16(ws, xh[o], acc[o][T]);
              acc[o][T] = mfma_f16(wl[d][T], xh[o], acc[o][T]);
              acc[o][T] = mfma_f16(wh[d][T], xl[o], acc[o][T]);
            }
          }
        }
        if (i + WD < KS) {   // refills run for skipped steps too (in-bounds: the pack's zero tail)
#pragma unroll
          for (int T = 0; T < NT; ++T) {
            wh[d][T] = wp[((wstep(i + WD) * NT + T) * 2 + 0) * 64];
            wl[d][T] = wp[((wstep(i + WD) * NT + T) * 2 + 1) * 64];
          }
        }
        __builtin_amdgcn_sched_barrier(0);   // the refills stay WD steps ahead of their use
      }
    }
    __syncthreads();
    if (nci0 == 0) {
      // epilogue.  C/D layout: register r of lane (c, h) = row (r&3) + 8(r>>2) + 4h, pixel c
      const int y0 = (int)(tile / segs) * RO, x0 = (int)(tile % segs) * kHPx;
      const int xo = x0 + 32 * wid + c;
#pragma unroll
      for (int o = 0; o < RO; ++o) {
        const int y = y0 + o;
        if (xo >= a.W || y >= a.H) continue;
        const int64_t pix = (int64_t)y * a.W + xo;
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = 32 * T + (r & 3) + 8 * (r >> 2) + 4 * h;
            float v = acc[o][T][r] * osc;
            if (BWD) {
              if (co < a.cout) {
                // LeakyReLU'(z) from the saved output: sign(lrelu(z)) = sign(z), slope > 0
                if (BWD == 2 && !(a.act[pix * a.cout + co] > 0.f)) v *= a.slope;
                a.out[pix * a.ldo + co] = v;
                amax = amax_upd(amax, v);
              }
            } else if (co < a.cout) {
              v += a.bias[co];
              v = v > 0.f ? v : v * a.slope;
              a.out[pix * a.ldo + co] = v;
              amax = amax_upd(amax, v);
            } else if (co < a.cout + 3) {
              v += a.bias[co];
              float* op = a.rgb + pix * 3 + (co - a.cout);
              if (a.rgb_mode == 0) *op = v;
              else if (a.rgb_mode == 1) *op += v;
              else *op = 1.f / (1.f + expf(-(*op + v)));
            }
          }
      }
    }
    tile = ntile;
    ci0 = nci0;
    nreal = nnreal;
  }
  if (a.out_max) amax_commit_block(amax, a.out_max, red);
}

// Tile shape per stage (RO output rows, CH-channel chunks): measured in DESIGN §12.
template <int NT, int BWD>
static int launch_conv_h2(const ConvH2Args& a, hipStream_t st) {
  constexpr int RO = NT >= 4 ? 1 : kConvRO, CH = kConvCH;   // (NT = 4 at RO = 2 spills)
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3x3_h2<NT, BWD, RO, CH>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)conv_h2_lds<RO, CH>()));
    attr = true;
  }
  const int64_t tiles = (int64_t)((a.H + RO - 1) / RO) * ((a.W + kHPx - 1) / kHPx);
  constexpr size_t lds = conv_h2_lds<RO, CH>();
  hipLaunchKernelGGL((k_conv3x3_h2<NT, BWD, RO, CH>), dim3(grid_for(tiles, 1, 256 * 4)), dim3(256), lds, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// Weight gradient on fp32h2: dW[m, (3 ky + kx) C + ci] = sum_p dY[p, m] X[p + (ky-1) W + kx - 1, ci]
// (zero where x + kx - 1 leaves the row or the source leaves the image), db[m] = sum_p dY[p, m].
// Both operands are activations, so both are split and scaled: dY staged times
// 2^e with max in [8, 16) (so Ys = 2^11 Yh stays in f16), X times 2^e' with max
// in [2^14, 2^15); dW = 2^-11 (Ys.Xh + Yl.Xh + Yh.Xl) / (2^e 2^e').  k = pixel:
// per PX-pixel chunk (PX / 16 k-steps; 64 for the two small stages, whose
// chunks are otherwise latency-bound, 32 for stage 0's 224 staging tasks) dY is
// staged transposed as [plane][m][PX px] and X as three kx-shifted copies
// [kx][plane][ci][PX px]
// (the row-edge and image-edge zeros applied while staging), each lane
// transposing 8 pixels x 4 channels in registers; 80-B / 144-B rows (5 / 9
// 16-B slots, odd: conflict-free ds_read_b128 A and B fragments).  One 4-wave workgroup per (pixel split, ky);
// wave w takes column tiles j = w, w + 4, w + 8 of the 3 NC (kx, channel-tile)
// pairs x all MT row tiles.  db from the fp32 values while staging (ky = 0
// blocks).  Partials per split, summed in fixed order (k_sum_splits).
template <int MT, int NC, int PX>
__global__ void __launch_bounds__(256, 2) k_conv_wgrad_h2(WgradArgs a, const unsigned* y_max, const unsigned* x_max) {
  constexpr int M = 32 * MT, C = 32 * NC;
  constexpr int NO = PX / 8;                            // pixel octets per chunk
  static_assert((M + C) / 4 * NO <= 256, "one staging task per thread");
  constexpr int PIT = PX + 8;                           // f16 per staged row: 80 B (32 px) / 144 B (64 px)
  constexpr int PA = M * PIT, PB = C * PIT;             // f16 per plane
  constexpr int NJ = 3 * NC, JW = (NJ + 3) / 4;
  __shared__ __attribute__((aligned(16))) _Float16 as_h[2 * PA];
  __shared__ __attribute__((aligned(16))) _Float16 bs_h[3 * 2 * PB];
  __shared__ float dbs[NO][M];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int split = blockIdx.x, ky = blockIdx.y;
  const int npix = a.H * a.W;
  const int pbeg = split * (int)a.chunk;
  const int pend = pbeg + (int)a.chunk < npix ? pbeg + (int)a.chunk : npix;
  // dY to max [8, 16), X to max [2^14, 2^15)
  const float ys = img_scale(y_max) * (1.f / 2048.f);
  const float xs = img_scale(x_max);
  const float osc = 1.f / (2048.f * ys * xs);
  f32x16 acc[JW][MT];
#pragma unroll
  for (int u = 0; u < JW; ++u)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[u][t] = (f32x16){0.f};
  float db[4] = {0.f, 0.f, 0.f, 0.f};
  // staging task of this thread (one per chunk): tid < C -> X channel quad qb of
  // pixel octet ob: the 10 source pixels p - 1 .. p + 8 of its 8 pixels (one load
  // each), from which the three kx-shifted copies are cut; C <= tid < C + M -> dY
  // channel quad qa of pixel octet oa.
  const bool tb = tid < C / 4 * NO, ta = !tb && tid < (C + M) / 4 * NO;
  const int qb = tid % (C / 4), ob = tid / (C / 4);
  const int ta_i = tid - C / 4 * NO;
  const int qa = ta_i % (M / 4), oa = ta_i / (M / 4);
  float4 v[10];
  auto load = [&](int p0) {
    if (tb) {
      const int s0 = p0 + 8 * ob + (ky - 1) * a.W - 1;
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const int sp = s0 + j;
        v[j] = sp >= 0 && sp < npix ? *reinterpret_cast<const float4*>(a.x + (int64_t)sp * C + 4 * qb)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else if (ta) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = p0 + 8 * oa + j;
        v[j] = p < pend ? *reinterpret_cast<const float4*>(a.dy + (int64_t)p * M + 4 * qa)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  // 8 pixels x 4 channels (pixel jj = v[jj + sh], zero where !(ok >> jj & 1)) ->
  // per channel k: [hi 8 px] at base + k * PIT, lo at + pitch_pl
  auto put8x4 = [&](_Float16* base, int pitch_pl, int sh, unsigned ok, float sc) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      unsigned hi[4], lo[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* f0 = reinterpret_cast<const float*>(&v[2 * j + sh]);
        const float* f1 = reinterpret_cast<const float*>(&v[2 * j + 1 + sh]);
        const float e0 = (ok >> (2 * j)) & 1u ? f0[k] * sc : 0.f;
        const float e1 = (ok >> (2 * j + 1)) & 1u ? f1[k] * sc : 0.f;
        splith(e0, e1, hi[j], lo[j]);
      }
      *reinterpret_cast<uint4*>(base + k * PIT) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
      *reinterpret_cast<uint4*>(base + k * PIT + pitch_pl) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    }
  };
  auto put = [&](int p0) {
    if (tb) {
      // output pixel p = p0 + 8 ob + jj takes source jj + kx for copy kx: zero where
      // p >= pend or x(p) + kx - 1 leaves the row (the image edges were zeroed by the load)
      const int pf = p0 + 8 * ob;
      unsigned okp = 0, okl = 0, okr = 0;   // p < pend; x > 0 (kx = 0); x < W - 1 (kx = 2)
      int x = pf % a.W;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        okp |= (unsigned)(pf + jj < pend) << jj;
        okl |= (unsigned)(x > 0) << jj;
        okr |= (unsigned)(x < a.W - 1) << jj;
        x = x + 1 == a.W ? 0 : x + 1;
      }
      _Float16* base = bs_h + (4 * qb) * PIT + 8 * ob;
      put8x4(base, PB, 0, okp & okl, xs);
      put8x4(base + 2 * PB, PB, 1, okp, xs);
      put8x4(base + 4 * PB, PB, 2, okp & okr, xs);
    } else if (ta) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        db[0] += v[j].x;
        db[1] += v[j].y;
        db[2] += v[j].z;
        db[3] += v[j].w;
      }
      put8x4(as_h + (4 * qa) * PIT + 8 * oa, PA, 0, 0xffu, ys);
    }
  };
  if (pbeg < pend) load(pbeg);
  for (int p0 = pbeg; p0 < pend; p0 += PX) {
    put(p0);
    __syncthreads();
    if (p0 + PX < pend) load(p0 + PX);   // in flight during the MFMAs
#pragma unroll
    for (int s = 0; s < PX / 16; ++s) {
      uint4 yl_[MT], yh_[MT];   // (Ys = 2^11 Yh made per use: 4 v_pk_mul, 12 fewer VGPRs live)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const _Float16* pa = as_h + (32 * t + c) * PIT + 16 * s + 8 * h;
        yh_[t] = *reinterpret_cast<const uint4*>(pa);
        yl_[t] = *reinterpret_cast<const uint4*>(pa + PA);
      }
#pragma unroll
      for (int u = 0; u < JW; ++u) {
        const int j = wid + 4 * u;
        if (j < NJ) {
          const int kx = j / NC, nc = j - kx * NC;
          const _Float16* pb = bs_h + kx * 2 * PB + (32 * nc + c) * PIT + 16 * s + 8 * h;
          const uint4 xh = *reinterpret_cast<const uint4*>(pb);
          const uint4 xl = *reinterpret_cast<const uint4*>(pb + PB);
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            acc[u][t] = mfma_f16(f16x8_scale2048(yh_[t]), xh, acc[u][t]);
            acc[u][t] = mfma_f16(yl_[t], xh, acc[u][t]);
            acc[u][t] = mfma_f16(yh_[t], xl, acc[u][t]);
          }
        }
      }
    }
    __syncthreads();
  }
  const int N = 9 * C;
  float* out = a.part + (int64_t)split * ((int64_t)M * N + M);
#pragma unroll
  for (int u = 0; u < JW; ++u) {
    const int j = wid + 4 * u;
    if (j >= NJ) continue;
    const int kx = j / NC, nc = j - kx * NC;
    const int col = (3 * ky + kx) * C + 32 * nc + c;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(int64_t)(32 * t + (r & 3) + 8 * (r >> 2) + 4 * h) * N + col] = acc[u][t][r] * osc;
  }
  if (ky == 0) {   // db: the pixel octets' sums per channel, octet order
    if (ta) {
#pragma unroll
      for (int k = 0; k < 4; ++k) dbs[oa][4 * qa + k] = db[k];
    }
    __syncthreads();
    if (tid < M) {
      float sdb = dbs[0][tid];
#pragma unroll
      for (int o = 1; o < NO; ++o) sdb += dbs[o][tid];
      out[(int64_t)M * N + tid] = sdb;
    }
  }
}

template <int MT, int NC, int PX>
static int launch_wgrad_h2(const float* dyb, const unsigned* y_max, const float* x, const unsigned* x_max, int H,
                           int W, float* part, float* dw, hipStream_t st) {
  WgradArgs g;
  g.dy = dyb;
  g.x = x;
  g.H = H;
  g.W = W;
  g.M = 32 * MT;
  g.Cin = 32 * NC;
  int ns;
  wgrad_plan((int64_t)H * W, g.M, g.Cin, &ns, &g.chunk, PX);
  g.part = part;
  hipLaunchKernelGGL((k_conv_wgrad_h2<MT, NC, PX>), dim3(ns, 3), dim3(256), 0, st, g, y_max, x_max);
  PNR_LAUNCH_CHECK();
  const int64_t n = (int64_t)g.M * 9 * g.Cin + g.M;
  hipLaunchKernelGGL(k_sum_splits, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, part, n, ns, dw, (int64_t)0,
                     (int64_t)0);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}

// k_nr_rgb_grad plus max |g| into the absmax words of the three cat images
__global__ void k_nr_rgb_grad_h2(const float* __restrict__ d_out, const float* __restrict__ out_rgb, int64_t npix,
                                 float* __restrict__ cat2, float* __restrict__ cat1, float* __restrict__ cat0,
                                 unsigned* __restrict__ words) {
  float m = 0.f;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    float g[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float s = out_rgb[p * 3 + j];
      g[j] = d_out[p * 3 + j] * (s * (1.f - s));
      m = amax_upd(m, g[j]);
    }
    float* c2 = cat2 + p * 32;
    float* c1 = cat1 + p * 64;
    float* c0 = cat0 + p * 96;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const float v = j < 3 ? g[j] : 0.f;
      c2[j] = v;
      c1[32 + j] = v;
      c0[64 + j] = v;
    }
  }
  __shared__ float red[4];
  amax_commit_block(m, words + 0 * kWS, red);
  if (threadIdx.x == 0 && m > 0.f) {   // (m: the block max after the commit's reduction)
    atomicMax(words + 1 * kWS, __float_as_uint(m));
    atomicMax(words + 2 * kWS, __float_as_uint(m));
  }
}

}  // namespace pnr

using namespace pnr;

extern "C" int pnr_neural_render_scratch_bytes(int32_t H, int32_t W, size_t* out) {
  PNR_CHECK_ARG(out && H >= 0 && W >= 0, "neural_render_scratch_bytes: bad args");
  *out = (size_t)H * W * (64 + 32 + 4) * sizeof(float);
  return PNR_OK;
}

extern "C" int pnr_neural_render_fwd(const float* x, int32_t H, int32_t W, const pnr_neural_render_w* w,
                                     float* out_rgb, void* scratch, size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(x && w && out_rgb && scratch, "neural_render: null pointer");
  PNR_CHECK_ARG(w->wf0 && w->b0 && w->wf1 && w->b1 && w->wrgb0 && w->brgb0 && w->wrgb1 && w->brgb1 && w->wrgb2 &&
                    w->brgb2,
                "neural_render: null weight");
  PNR_CHECK_ARG(H >= 0 && W >= 0, "neural_render: bad image size");
  PNR_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)scratch & 15) == 0,
                "neural_render: x and scratch must be 16-B aligned");
  PNR_CHECK_ARG(scratch_bytes >= (size_t)H * W * 100 * sizeof(float), "neural_render: scratch too small");
  if (H == 0 || W == 0) return PNR_OK;
  hipStream_t st = as_stream(stream);
  float* net0 = static_cast<float*>(scratch);
  float* net1 = net0 + (size_t)H * W * 64;
  int rc;
  ConvArgs a;
  a.H = H;
  a.W = W;
  a.slope = w->neg_slope;
  a.act = nullptr;
  a.cin_real = 1 << 30;
  // stage 0: x (128) -> net0 (64) on MFMA + rgb = conv_rgb0(x) on VALU
  a.in = x;
  a.Cin = 128;
  a.wf = w->wf0;
  a.bias = w->b0;
  a.cout = 64;
  a.ldo = 64;
  a.out = net0;
  a.rgb = out_rgb;
  a.rgb_mode = 0;
  a.wrgb = w->wrgb0;
  a.brgb = w->brgb0;
  if ((rc = launch_conv<2>(a, st))) return rc;
  // stage 1: net0 (64) -> net1 (32), rgb += conv_rgb1(net0)
  a.in = net0;
  a.Cin = 64;
  a.wf = w->wf1;
  a.bias = w->b1;
  a.cout = 32;
  a.ldo = 32;
  a.out = net1;
  a.rgb_mode = 1;
  a.wrgb = w->wrgb1;
  a.brgb = w->brgb1;
  if ((rc = launch_conv<1>(a, st))) return rc;
  // stage 2: out = sigmoid(rgb + conv_rgb2(net1)), rgb only
  a.in = net1;
  a.Cin = 32;
  a.wf = nullptr;
  a.bias = nullptr;
  a.cout = 0;
  a.ldo = 0;
  a.out = nullptr;
  a.rgb_mode = 2;
  a.wrgb = w->wrgb2;
  a.brgb = w->brgb2;
  return launch_conv<0>(a, st);
}

extern "C" int pnr_neural_render_bwd_scratch_bytes(int32_t H, int32_t W, size_t* out) {
  PNR_CHECK_ARG(out && H >= 0 && W >= 0, "neural_render_bwd_scratch_bytes: bad args");
  const int64_t npix = (int64_t)H * W;
  size_t part = wgrad_scratch(npix, 96, 128);
  const size_t p1 = wgrad_scratch(npix, 64, 64), p2 = wgrad_scratch(npix, 32, 32);
  if (p1 > part) part = p1;
  if (p2 > part) part = p2;
  *out = (size_t)npix * (32 + 64 + 96) * sizeof(float) + part;
  return PNR_OK;
}

extern "C" int pnr_neural_render_bwd(const float* x, const float* fwd_scratch, const float* out_rgb,
                                     const float* d_out, int32_t H, int32_t W, const pnr_neural_render_wt* wt,
                                     float* d_x, float* dw0, float* dw1, float* dw2, void* scratch,
                                     size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(x && fwd_scratch && out_rgb && d_out && wt && d_x && dw0 && dw1 && dw2 && scratch,
                "neural_render_bwd: null pointer");
  PNR_CHECK_ARG(wt->wt0 && wt->wt1 && wt->wt2, "neural_render_bwd: null weight");
  PNR_CHECK_ARG(H >= 0 && W >= 0 && (int64_t)H * W < (1ll << 30), "neural_render_bwd: bad image size");
  PNR_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)fwd_scratch & 15) == 0 && ((uintptr_t)scratch & 15) == 0,
                "neural_render_bwd: x, fwd_scratch and scratch must be 16-B aligned");
  size_t need;
  pnr_neural_render_bwd_scratch_bytes(H, W, &need);
  PNR_CHECK_ARG(scratch_bytes >= need, "neural_render_bwd: scratch too small");
  hipStream_t st = as_stream(stream);
  const int64_t npix = (int64_t)H * W;
  if (npix == 0) {
    PNR_HIP(hipMemsetAsync(dw0, 0, (96 * 9 * 128 + 96) * sizeof(float), st));
    PNR_HIP(hipMemsetAsync(dw1, 0, (64 * 9 * 64 + 64) * sizeof(float), st));
    PNR_HIP(hipMemsetAsync(dw2, 0, (32 * 9 * 32 + 32) * sizeof(float), st));
    return PNR_OK;
  }
  const float* net0 = fwd_scratch;
  const float* net1 = fwd_scratch + (size_t)npix * 64;
  float* cat2 = static_cast<float*>(scratch);
  float* cat1 = cat2 + (size_t)npix * 32;
  float* cat0 = cat1 + (size_t)npix * 64;
  float* part = cat0 + (size_t)npix * 96;
  hipLaunchKernelGGL(k_nr_rgb_grad, dim3(grid_for(npix, 256, 2048)), dim3(256), 0, st, d_out, out_rgb, npix, cat2,
                     cat1, cat0);
  PNR_LAUNCH_CHECK();
  int rc;
  ConvArgs a;
  a.H = H;
  a.W = W;
  a.slope = wt->neg_slope;
  a.bias = nullptr;
  a.rgb = nullptr;
  a.rgb_mode = 3;
  // stage 2: d net1 = conv(cat2 = [g, 0], flipped conv_rgb.2), masked by net1 -> cat1[:, :32]
  a.in = cat2;
  a.Cin = 32;
  a.cin_real = 3;         // [g, 0 x 29]
  a.wf = wt->wt2;
  a.cout = 32;
  a.ldo = 64;
  a.out = cat1;
  a.act = net1;
  if ((rc = launch_conv<1, 2>(a, st))) return rc;
  if ((rc = launch_wgrad<1, 1, true>(cat2, net1, H, W, 32, part, dw2, st))) return rc;
  // stage 1: d net0 = conv(cat1 = [dz1, g, 0], flipped [conv_layers.1; conv_rgb.1]), masked by net0
  a.in = cat1;
  a.Cin = 64;
  a.cin_real = 32 + 3;    // [dz1, g, 0 x 29]
  a.wf = wt->wt1;
  a.cout = 64;
  a.ldo = 96;
  a.out = cat0;
  a.act = net0;
  if ((rc = launch_conv<2, 2>(a, st))) return rc;
  if ((rc = launch_wgrad<2, 2, false>(cat1, net0, H, W, 64, part, dw1, st))) return rc;
  // stage 0: d x = conv(cat0 = [dz0, g, 0], flipped [conv_layers.0; conv_rgb.0])
  a.in = cat0;
  a.Cin = 96;
  a.cin_real = 64 + 3;    // [dz0, g, 0 x 29]
  a.wf = wt->wt0;
  a.cout = 128;
  a.ldo = 128;
  a.out = d_x;
  a.act = nullptr;
  if ((rc = launch_conv<4, 1>(a, st))) return rc;
  return launch_wgrad<3, 4, true>(cat0, x, H, W, 128, part, dw0, st);
}

// ---------------------------------------------------------------- fp32h2 ABI
extern "C" int pnr_neural_render_h2_scratch_bytes(int32_t H, int32_t W, size_t* out) {
  PNR_CHECK_ARG(out && H >= 0 && W >= 0, "neural_render_h2_scratch_bytes: bad args");
  *out = (size_t)H * W * (64 + 32) * sizeof(float) + 256;
  return PNR_OK;
}

extern "C" int pnr_neural_render_fwd_h2(const float* x, int32_t H, int32_t W, const pnr_neural_render_h2w* w,
                                        float* out_rgb, void* scratch, size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(x && w && out_rgb && scratch, "neural_render_h2: null pointer");
  PNR_CHECK_ARG(w->wp0 && w->wp1 && w->wp2 && w->ws && w->b0 && w->b1 && w->b2, "neural_render_h2: null weight");
  PNR_CHECK_ARG(H >= 0 && W >= 0, "neural_render_h2: bad image size");
  PNR_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)scratch & 15) == 0,
                "neural_render_h2: x and scratch must be 16-B aligned");
  size_t need;
  pnr_neural_render_h2_scratch_bytes(H, W, &need);
  PNR_CHECK_ARG(scratch_bytes >= need, "neural_render_h2: scratch too small");
  if (H == 0 || W == 0) return PNR_OK;
  hipStream_t st = as_stream(stream);
  const int64_t npix = (int64_t)H * W;
  float* net0 = static_cast<float*>(scratch);
  float* net1 = net0 + (size_t)npix * 64;
  unsigned* words = reinterpret_cast<unsigned*>(net1 + (size_t)npix * 32);   // max |x|, |net0|, |net1|
  PNR_HIP(hipMemsetAsync(words, 0, 256, st));
  hipLaunchKernelGGL(k_nr_absmax, dim3(grid_for(npix * 32, 256, 1024)), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(x), npix * 32, words);
  PNR_LAUNCH_CHECK();
  int rc;
  ConvH2Args a;
  a.H = H;
  a.W = W;
  a.slope = w->neg_slope;
  a.act = nullptr;
  a.cin_real = 1 << 30;
  a.rgb = out_rgb;
  // stage 0: x (128) -> [net0 (64), rgb = conv_rgb0(x)]
  a.in = x;
  a.Cin = 128;
  a.in_max = words + 0 * kWS;
  a.wp = static_cast<const uint4*>(w->wp0);
  a.wscale = w->ws + 0;
  a.bias = w->b0;
  a.cout = 64;
  a.out = net0;
  a.ldo = 64;
  a.out_max = words + 1 * kWS;
  a.rgb_mode = 0;
  if ((rc = launch_conv_h2<3, 0>(a, st))) return rc;
  // stage 1: net0 (64) -> [net1 (32), rgb += conv_rgb1(net0)]
  a.in = net0;
  a.Cin = 64;
  a.in_max = words + 1 * kWS;
  a.wp = static_cast<const uint4*>(w->wp1);
  a.wscale = w->ws + 4;
  a.bias = w->b1;
  a.cout = 32;
  a.out = net1;
  a.ldo = 32;
  a.out_max = words + 2 * kWS;
  a.rgb_mode = 1;
  if ((rc = launch_conv_h2<2, 0>(a, st))) return rc;
  // stage 2: out = sigmoid(rgb + conv_rgb2(net1))
  a.in = net1;
  a.Cin = 32;
  a.in_max = words + 2 * kWS;
  a.wp = static_cast<const uint4*>(w->wp2);
  a.wscale = w->ws + 4;
  a.bias = w->b2;
  a.cout = 0;
  a.out = nullptr;
  a.ldo = 0;
  a.out_max = nullptr;
  a.rgb_mode = 2;
  return launch_conv_h2<1, 0>(a, st);
}

extern "C" int pnr_neural_render_bwd_h2_scratch_bytes(int32_t H, int32_t W, size_t* out) {
  PNR_CHECK_ARG(out && H >= 0 && W >= 0, "neural_render_bwd_h2_scratch_bytes: bad args");
  return pnr_neural_render_bwd_scratch_bytes(H, W, out) == PNR_OK ? (*out += 256, PNR_OK) : PNR_EINVAL;
}

extern "C" int pnr_neural_render_bwd_h2(const float* x, const float* fwd_scratch, const float* out_rgb,
                                        const float* d_out, int32_t H, int32_t W, const pnr_neural_render_h2wt* wt,
                                        float* d_x, float* dw0, float* dw1, float* dw2, void* scratch,
                                        size_t scratch_bytes, void* stream) {
  PNR_CHECK_ARG(x && fwd_scratch && out_rgb && d_out && wt && d_x && dw0 && dw1 && dw2 && scratch,
                "neural_render_bwd_h2: null pointer");
  PNR_CHECK_ARG(wt->wt0 && wt->wt1 && wt->wt2 && wt->ws, "neural_render_bwd_h2: null weight");
  PNR_CHECK_ARG(H >= 0 && W >= 0 && (int64_t)H * W < (1ll << 30), "neural_render_bwd_h2: bad image size");
  PNR_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)fwd_scratch & 15) == 0 && ((uintptr_t)scratch & 15) == 0,
                "neural_render_bwd_h2: x, fwd_scratch and scratch must be 16-B aligned");
  size_t need;
  pnr_neural_render_bwd_h2_scratch_bytes(H, W, &need);
  PNR_CHECK_ARG(scratch_bytes >= need, "neural_render_bwd_h2: scratch too small");
  hipStream_t st = as_stream(stream);
  const int64_t npix = (int64_t)H * W;
  if (npix == 0) {
    PNR_HIP(hipMemsetAsync(dw0, 0, (96 * 9 * 128 + 96) * sizeof(float), st));
    PNR_HIP(hipMemsetAsync(dw1, 0, (64 * 9 * 64 + 64) * sizeof(float), st));
    PNR_HIP(hipMemsetAsync(dw2, 0, (32 * 9 * 32 + 32) * sizeof(float), st));
    return PNR_OK;
  }
  const float* net0 = fwd_scratch;
  const float* net1 = fwd_scratch + (size_t)npix * 64;
  const unsigned* fwords = reinterpret_cast<const unsigned*>(net1 + (size_t)npix * 32);   // the forward's max words
  float* cat2 = static_cast<float*>(scratch);
  float* cat1 = cat2 + (size_t)npix * 32;
  float* cat0 = cat1 + (size_t)npix * 64;
  unsigned* words = reinterpret_cast<unsigned*>(cat0 + (size_t)npix * 96);   // max |cat2|, |cat1|, |cat0|
  float* part = cat0 + (size_t)npix * 96 + 64;
  PNR_HIP(hipMemsetAsync(words, 0, 256, st));
  hipLaunchKernelGGL(k_nr_rgb_grad_h2, dim3(grid_for(npix, 256, 512)), dim3(256), 0, st, d_out, out_rgb, npix, cat2,
                     cat1, cat0, words);
  PNR_LAUNCH_CHECK();
  int rc;
  ConvH2Args a;
  a.H = H;
  a.W = W;
  a.slope = wt->neg_slope;
  a.bias = nullptr;
  a.rgb = nullptr;
  a.rgb_mode = 3;
  // stage 2: d net1 = conv(cat2 = [g, 0], flipped conv_rgb.2), masked by net1 -> cat1[:, :32]
  a.in = cat2;
  a.Cin = 32;
  a.in_max = words + 0 * kWS;
  a.cin_real = 3;
  a.wp = static_cast<const uint4*>(wt->wt2);
  a.wscale = wt->ws + 4;
  a.cout = 32;
  a.ldo = 64;
  a.out = cat1;
  a.out_max = words + 1 * kWS;
  a.act = net1;
  if ((rc = launch_conv_h2<1, 2>(a, st))) return rc;
  if ((rc = launch_wgrad_h2<1, 1, 64>(cat2, words + 0, net1, fwords + 2 * kWS, H, W, part, dw2, st))) return rc;
  // stage 1: d net0 = conv(cat1 = [dz1, g, 0], flipped [conv_layers.1; conv_rgb.1]), masked by net0
  a.in = cat1;
  a.Cin = 64;
  a.in_max = words + 1 * kWS;
  a.cin_real = 32 + 3;
  a.wp = static_cast<const uint4*>(wt->wt1);
  a.wscale = wt->ws + 4;
  a.cout = 64;
  a.ldo = 96;
  a.out = cat0;
  a.out_max = words + 2 * kWS;
  a.act = net0;
  if ((rc = launch_conv_h2<2, 2>(a, st))) return rc;
  if ((rc = launch_wgrad_h2<2, 2, 64>(cat1, words + 1 * kWS, net0, fwords + 1 * kWS, H, W, part, dw1, st))) return rc;
  // stage 0: d x = conv(cat0 = [dz0, g, 0], flipped [conv_layers.0; conv_rgb.0])
  a.in = cat0;
  a.Cin = 96;
  a.in_max = words + 2 * kWS;
  a.cin_real = 64 + 3;
  a.wp = static_cast<const uint4*>(wt->wt0);
  a.wscale = wt->ws + 0;
  a.cout = 128;
  a.ldo = 128;
  a.out = d_x;
  a.out_max = nullptr;
  a.act = nullptr;
  if ((rc = launch_conv_h2<4, 1>(a, st))) return rc;
  return launch_wgrad_h2<3, 4, 32>(cat0, words + 2 * kWS, x, fwords + 0 * kWS, H, W, part, dw0, st);
}
