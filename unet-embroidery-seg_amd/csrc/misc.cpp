// Error reporting and library identity for the unetseg C ABI.
#include <cstdarg>
#include <cstdio>

#include "common.h"

static thread_local char g_err[1024] = "";

void unetseg_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

UNETSEG_API const char* unetseg_last_error(void) { return g_err; }

UNETSEG_API int unetseg_abi_version(void) { return 1; }

UNETSEG_API int unetseg_device_arch(char* buf, int n) {
  hipDeviceProp_t prop;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    unetseg_set_error("no HIP device");
    return 1;
  }
  snprintf(buf, n, "%s", prop.gcnArchName);
  return 0;
}
