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
