// Library-level C ABI: thread-local error string, version, device probe.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/mapa.h"

static thread_local char g_err[512] = "";

int mapa_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return 1;
}

extern "C" const char* mapa_last_error(void) { return g_err; }

extern "C" int mapa_version(void) { return 1; }

extern "C" int mapa_device_check(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device) {
    mapa_set_error("mapa_device_check: no HIP device %d (count %d)", device, n);
    return 0;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    mapa_set_error("mapa_device_check: hipGetDeviceProperties failed");
    return 0;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    mapa_set_error("mapa_device_check: device %d is %s, library is built for gfx950", device, prop.gcnArchName);
    return 0;
  }
  return 1;
}

// Debug / serialize mode (MAPA_SERIALIZE=1, or AMD_SERIALIZE_KERNEL / HIP_LAUNCH_BLOCKING set): the binding calls
// this after every launch, so a faulting or failing kernel is reported by the launch that caused it instead of by
// whatever synchronises next.  Launch errors are already reported (and cleared) by each entry point's own
// hipGetLastError (MAPA_CHECK_LAUNCH), so this only synchronises and PEEKS: a sticky error left by an unrelated
// earlier call is reported as such but not cleared, so the caller still sees the real error state.
// It also reads (and clears) the library's sticky fault word: a LayerNorm band barrier that gave up is reported here
// as the failure of the launch being checked.
extern "C" int mapa_stream_check(hipStream_t stream, const char* what) {
  const hipError_t s = hipStreamSynchronize(stream);
  const hipError_t e = s != hipSuccess ? s : hipPeekAtLastError();
  if (e != hipSuccess)
    return mapa_set_error("%s: device error after launch: %s (hipError %d)", what ? what : "launch",
                          hipGetErrorString(e), (int)e);
  const int f = mapa_fault_status(1);
  if (f < 0) return 1;  // message already set
  if (f & MAPA_FAULT_LN_BARRIER)
    return mapa_set_error("%s: a LayerNorm-fused GEMM band barrier timed out (its LayerNorm rows are invalid)",
                          what ? what : "launch");
  if (f) return mapa_set_error("%s: device fault word 0x%x", what ? what : "launch", (unsigned)f);
  return 0;
}
