// capi.hip — library-wide C-ABI entry points (errors, version, device probe).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../../include/ruserf_amd.h"
#include "rsf_internal.h"

namespace {
thread_local char g_err[512] = "ok";
}

namespace rsf {
int set_error(int code, const char* msg) {
  std::snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}
int set_hip_error(hipError_t e, const char* what, const char* file, int line) {
  std::snprintf(g_err, sizeof(g_err), "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
  (void)hipGetLastError();
  return RSF_ERR_HIP;
}
}  // namespace rsf

extern "C" {
const char* rsf_last_error(void) { return g_err; }
const char* rsf_version(void) { return "ruserf_amd 0.1.0 (gfx950)"; }
int rsf_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}
}
