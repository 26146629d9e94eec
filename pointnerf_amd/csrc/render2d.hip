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
// trunk conv AND its rgb skip conv stacked (64+3 -> 96, 32+3 -> 64, 0+3 -> 32),
// columns = 32 consecutive pixels of an image row, k = (tap, input channel).
// A 4-wave workgroup owns 128 pixels of one row; the 3 input rows x 130
// pixels of a 32-channel slice are staged in LDS (pixel pitch 33 floats,
// conflict-free B reads), so each input element is read from HBM ~3 times
// (once per output row) instead of 9.  Zero padding 1 as in the reference.
#include "pnr_common.h"

namespace pnr {

typedef float f32x16r __attribute__((ext_vector_type(16)));

constexpr int kRPx = 128;              // pixels per workgroup (4 waves x 32)
constexpr int kRCh = 32;               // input channels staged per LDS chunk
constexpr int kRPitch = kRCh + 1;      // floats per staged pixel
constexpr int kRRowPx = kRPx + 2;      // staged pixels per input row (halo 1)
constexpr size_t kRLds = (size_t)3 * kRRowPx * kRPitch * sizeof(float);

struct ConvArgs {
  const float* in;     // [H, W, Cin]
  int H, W, Cin;
  const float* wf;     // fragment-packed [ROWS, 9 * Cin] (k = tap * Cin + ci), ROWS = 32 * NT
  const float* bias;   // [ROWS] (trunk bias, rgb bias, zeros)
  int cout;            // trunk output channels (0 = rgb only)
  float* out;          // [H, W, cout] = lrelu(trunk)   (cout > 0)
  float* rgb;          // [H, W, 3] accumulated (first stage writes, later add)
  int rgb_mode;        // 0: rgb = part, 1: rgb += part, 2: out_rgb = sigmoid(rgb + part)
  float slope;
};

template <int NT>
__global__ void __launch_bounds__(256, 2) k_conv3x3(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_r[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int segs = (a.W + kRPx - 1) / kRPx;
  const int64_t ntiles = (int64_t)a.H * segs;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int y = (int)(tile / segs);
    const int x0 = (int)(tile % segs) * kRPx;
    f32x16r acc[NT];
#pragma unroll
    for (int T = 0; T < NT; ++T) acc[T] = (f32x16r){0.f};
    for (int ci0 = 0; ci0 < a.Cin; ci0 += kRCh) {
      // stage rows y-1..y+1, pixels x0-1 .. x0+128, channels ci0 .. ci0+31 (zero padded)
      for (int i = threadIdx.x; i < 3 * kRRowPx * (kRCh / 4); i += blockDim.x) {
        const int q = i % (kRCh / 4);
        const int px = (i / (kRCh / 4)) % kRRowPx;
        const int r = i / ((kRCh / 4) * kRRowPx);
        const int yy = y - 1 + r, xx = x0 - 1 + px;
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
      // this wave's 32 pixels: x0 + 32 wid + c
      const int pcol = 32 * wid + c;
      // k-steps of this chunk in (tap, channel-pair) order; weight fragments
      // are software-pipelined kRW steps ahead across tap boundaries
      constexpr int kRW = 6;
      constexpr int kSteps = 9 * (kRCh / 2);
      const float* wp = a.wf + lane;
      auto wstep = [&](int i) {   // global k-step of chunk step i
        const int tap = i / (kRCh / 2), s = i % (kRCh / 2);
        return (tap * a.Cin + ci0) / 2 + s;
      };
      float wr[kRW][NT];
#pragma unroll
      for (int d = 0; d < kRW; ++d)
#pragma unroll
        for (int T = 0; T < NT; ++T) wr[d][T] = wp[(wstep(d) * NT + T) * 64];
#pragma unroll
      for (int i0 = 0; i0 < kSteps; i0 += kRW) {
#pragma unroll
        for (int d = 0; d < kRW; ++d) {
          const int i = i0 + d;
          if (i < kSteps) {
            const int tap = i / (kRCh / 2), s = i % (kRCh / 2);
            const int dy = tap / 3, dx = tap % 3;
            const float b = lds_r[(dy * kRRowPx + pcol + dx) * kRPitch + h + 2 * s];
#pragma unroll
            for (int T = 0; T < NT; ++T) acc[T] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[d][T], b, acc[T], 0, 0, 0);
            if (i + kRW < kSteps) {
#pragma unroll
              for (int T = 0; T < NT; ++T) wr[d][T] = wp[(wstep(i + kRW) * NT + T) * 64];
            }
          }
        }
      }
      __syncthreads();
    }
    // epilogue: rows 0..cout-1 trunk (lrelu), rows cout..cout+2 rgb
    const int xo = x0 + 32 * wid + c;
    if (xo < a.W) {
      const int64_t pix = (int64_t)y * a.W + xo;
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = 32 * T + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float v = acc[T][r] + a.bias[co];
          if (co < a.cout) {
            a.out[pix * a.cout + co] = v > 0.f ? v : v * a.slope;
          } else if (co < a.cout + 3) {
            float* o = a.rgb + pix * 3 + (co - a.cout);
            if (a.rgb_mode == 0) *o = v;
            else if (a.rgb_mode == 1) *o += v;
            else *o = 1.f / (1.f + expf(-(*o + v)));
          }
        }
    }
  }
}

template <int NT>
static int launch_conv(const ConvArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    PNR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3x3<NT>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRLds));
    attr = true;
  }
  const int64_t tiles = (int64_t)a.H * ((a.W + kRPx - 1) / kRPx);
  hipLaunchKernelGGL(k_conv3x3<NT>, dim3(grid_for(tiles, 1, 256 * 3)), dim3(256), kRLds, st, a);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
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
  PNR_CHECK_ARG(w->wf0 && w->b0 && w->wf1 && w->b1 && w->wf2 && w->b2, "neural_render: null weight");
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
  // stage 0: x (128) -> net0 (64) + rgb = conv_rgb0(x)
  a.in = x;
  a.Cin = 128;
  a.wf = w->wf0;
  a.bias = w->b0;
  a.cout = 64;
  a.out = net0;
  a.rgb = out_rgb;
  a.rgb_mode = 0;
  if ((rc = launch_conv<3>(a, st))) return rc;
  // stage 1: net0 (64) -> net1 (32), rgb += conv_rgb1(net0)
  a.in = net0;
  a.Cin = 64;
  a.wf = w->wf1;
  a.bias = w->b1;
  a.cout = 32;
  a.out = net1;
  a.rgb_mode = 1;
  if ((rc = launch_conv<2>(a, st))) return rc;
  // stage 2: out = sigmoid(rgb + conv_rgb2(net1))
  a.in = net1;
  a.Cin = 32;
  a.wf = w->wf2;
  a.bias = w->b2;
  a.cout = 0;
  a.out = nullptr;
  a.rgb_mode = 2;
  return launch_conv<1>(a, st);
}
