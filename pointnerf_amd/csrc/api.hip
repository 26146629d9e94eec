// Handle lifetime, error reporting and ABI version of libpnr.so.
#include <cstdarg>

#include "pnr_common.h"

namespace pnr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace pnr

extern "C" int pnr_abi_version(void) { return PNR_ABI_VERSION; }

extern "C" const char* pnr_last_error(void) { return pnr::g_err; }

extern "C" int pnr_create(int device, pnr_handle** out) {
  PNR_CHECK_ARG(out, "create: null out");
  *out = nullptr;
  int count = 0;
  PNR_HIP(hipGetDeviceCount(&count));
  PNR_CHECK_ARG(device >= 0 && device < count, "create: device %d not in [0, %d)", device, count);
  PNR_HIP(hipSetDevice(device));
  pnr_handle* h = new (std::nothrow) pnr_handle();
  if (!h) {
    pnr::set_error("create: out of host memory");
    return PNR_ENOMEM;
  }
  h->device = device;
  *out = h;
  return PNR_OK;
}

extern "C" int pnr_destroy(pnr_handle* h) {
  if (!h) return PNR_OK;
  (void)hipSetDevice(h->device);
  h->release_all();
  delete h;
  return PNR_OK;
}

// Shader clock under load (bench diagnostics): one wave spins for `spins`
// s_sleep slices between two (s_memtime, s_memrealtime) pairs; out[0] = shader
// cycles / (100 MHz real-time ticks) * 100 = the SCLK in MHz the wave saw
// (MI355X_MICROARCH "DVFS give-back" item 6).  Launched on a side stream while
// the timed kernels run, it reports the clock they ran at.
__global__ void k_clock_probe(float* out, int spins) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < spins; ++i) __builtin_amdgcn_s_sleep(8);
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[0] = r1 > r0 ? (float)(c1 - c0) / (float)(r1 - r0) * 100.f : 0.f;
}

extern "C" int pnr_clock_probe(float* out_dev, int32_t spins, void* stream) {
  PNR_CHECK_ARG(out_dev && spins > 0, "clock_probe: bad arguments");
  hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, pnr::as_stream(stream), out_dev, spins);
  PNR_LAUNCH_CHECK();
  return PNR_OK;
}
