// rsf_internal.h — error plumbing and small device-memory helpers shared by
// the C-ABI translation units.  Nothing here crosses the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/ruserf_amd.h"

namespace rsf {

int set_error(int code, const char* msg);
int set_hip_error(hipError_t e, const char* what, const char* file, int line);

inline int dmalloc(void** p, size_t bytes) {
  *p = nullptr;
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();
    return set_error(RSF_ERR_NOMEM, "hipMalloc failed");
  }
  return RSF_OK;
}

// Grow-only device scratch used to stage host batches.
struct DeviceScratch {
  void* base = nullptr;
  size_t cap = 0;
  void* extra = nullptr;
  size_t extra_cap = 0;
  int take(const size_t* bytes, int n, void** out) {
    size_t total = 0;
    for (int i = 0; i < n; ++i) total += (bytes[i] + 255) & ~(size_t)255;
    if (total > cap) {
      if (base) hipFree(base);
      base = nullptr;
      cap = 0;
      int rc = dmalloc(&base, total);
      if (rc) return rc;
      cap = total;
    }
    char* c = (char*)base;
    for (int i = 0; i < n; ++i) {
      out[i] = c;
      c += (bytes[i] + 255) & ~(size_t)255;
    }
    return RSF_OK;
  }
  int take_extra(size_t bytes, void** out) {
    if (bytes > extra_cap) {
      if (extra) hipFree(extra);
      extra = nullptr;
      extra_cap = 0;
      int rc = dmalloc(&extra, bytes);
      if (rc) return rc;
      extra_cap = bytes;
    }
    *out = extra;
    return RSF_OK;
  }
  void release() {
    if (base) hipFree(base);
    if (extra) hipFree(extra);
    base = extra = nullptr;
    cap = extra_cap = 0;
  }
};

}  // namespace rsf

#define RSF_HIP(call)                                                         \
  do {                                                                        \
    hipError_t rsf_e_ = (call);                                               \
    if (rsf_e_ != hipSuccess) return rsf::set_hip_error(rsf_e_, #call, __FILE__, __LINE__); \
  } while (0)
