// Error reporting and small host utilities of the C ABI.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/dlamd.h"

namespace dl {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace dl

extern "C" int dl_abi_version(void) { return DL_ABI_VERSION; }

extern "C" const char* dl_last_error(void) { return dl::g_err; }

extern "C" int dl_device_sync(void) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    dl::set_error("hipDeviceSynchronize: %s", hipGetErrorString(e));
    return 1000 + (int)e;
  }
  e = hipGetLastError();
  if (e != hipSuccess) {
    dl::set_error("device error: %s", hipGetErrorString(e));
    return 1000 + (int)e;
  }
  return 0;
}
