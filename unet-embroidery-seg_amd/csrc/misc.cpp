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

// A stream restricted to the CUs whose bits are set in mask[0 .. n_words) (bit i of word w = CU 32 w + i):
// the weight-gradient stream's persistent kernels hold a CU's LDS for their whole life, and a
// compute-stream kernel that needs a large LDS image cannot start a block beside them
// (UNETSEG_SIDE_CUMASK, ops.side_stream).  *out receives the hipStream_t.
UNETSEG_API int unetseg_stream_create_cumask(const unsigned* mask, int n_words, void** out) {
  US_CHECK_ARG(mask != nullptr && out != nullptr && n_words > 0, "stream_create_cumask: bad arguments");
  hipStream_t s = nullptr;
  const hipError_t err = hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask);
  if (err != hipSuccess) {
    unetseg_set_error("stream_create_cumask: %s", hipGetErrorString(err));
    return 2;
  }
  *out = (void*)s;
  return 0;
}

// Cross-stream ordering for the op layer's weight-gradient stream: `waiter` waits for the work
// enqueued so far on `signaler`.  The events carry a device-scope release only (both streams are
// on one device): the default system-scope fence costs ~6 us of idle compute stream per sync.
UNETSEG_API int unetseg_stream_wait(void* waiter, void* signaler) {
  constexpr int kRing = 64;
  static thread_local hipEvent_t ring[kRing];
  static thread_local int next = -1;
  if (next < 0) {
    for (int i = 0; i < kRing; ++i) {
      const hipError_t err = hipEventCreateWithFlags(&ring[i], hipEventDisableTiming | hipEventReleaseToDevice);
      if (err != hipSuccess) {
        unetseg_set_error("stream_wait: hipEventCreateWithFlags failed: %s", hipGetErrorString(err));
        return 2;
      }
    }
    next = 0;
  }
  hipEvent_t e = ring[next];
  next = (next + 1) % kRing;
  if (hipEventRecord(e, (hipStream_t)signaler) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)waiter, e, 0) != hipSuccess) {
    unetseg_set_error("stream_wait: record/wait failed");
    return 2;
  }
  return 0;
}
