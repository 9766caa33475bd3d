// libkrca: version, error reporting and device queries (host-only translation unit).
#include <stdarg.h>
#include <stdio.h>

#include <hip/hip_runtime.h>

#include "krca_common.h"

namespace krca {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace krca

extern "C" {

int krca_version(void) { return 100; }  // 0.1.0

const char* krca_last_error(void) { return krca::g_err; }

int krca_device_count(int* n_host) {
  KRCA_CHECK_ARG(n_host != nullptr, "krca_device_count: null out pointer");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *n_host = 0;
    krca::set_error("hipGetDeviceCount: %s", hipGetErrorString(e));
    return KRCA_EDEVICE;
  }
  *n_host = n;
  return KRCA_OK;
}

}  // extern "C"
