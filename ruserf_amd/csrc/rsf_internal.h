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

// hipCUB temporary storage.  hipcub does not check the size it is handed, and a call's
// requirement depends on the algorithm, the item count and the types, so no size queried
// for one call may be used for another: every call goes through cub_run, which queries
// that call's own requirement and grows the buffer to it.  A kCanary-byte 0xA5 canary is
// written past the requested bytes at every allocation; canary_intact() reads it back
// (diagnostics and tests: an overrun of the temporary storage changes it).
struct CubTemp {
  static constexpr size_t kCanary = 256;
  void* p = nullptr;
  size_t bytes = 0;  // usable bytes; the canary follows them
  int ensure(size_t need, hipStream_t st) {
    if (p && need <= bytes) return RSF_OK;
    if (p) {
      (void)hipStreamSynchronize(st);  // the old buffer may be in use by queued work
      (void)hipFree(p);
    }
    p = nullptr;
    bytes = 0;
    int rc = dmalloc(&p, need + kCanary);
    if (rc) return rc;
    if (hipMemsetAsync((char*)p + need, 0xA5, kCanary, st) != hipSuccess)
      return set_error(RSF_ERR_HIP, "canary initialisation failed");
    bytes = need;
    return RSF_OK;
  }
  // 1 if the canary is untouched (or nothing was allocated), 0 if not, <0 on a HIP error;
  // synchronises the stream
  int canary_intact(hipStream_t st) const {
    if (!p) return 1;
    unsigned char h[kCanary];
    if (hipMemcpyAsync(h, (const char*)p + bytes, kCanary, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return set_error(RSF_ERR_HIP, "canary read failed");
    for (size_t i = 0; i < kCanary; ++i)
      if (h[i] != 0xA5) return 0;
    return 1;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// One hipCUB device-wide call: f(void* tmp, size_t& bytes) -> hipError_t is invoked once
// with tmp == nullptr to size the call, then with storage of at least that size.
template <class F>
inline int cub_run(CubTemp& t, hipStream_t st, F&& f, const char* what) {
  size_t need = 0;
  hipError_t e = f(nullptr, need);
  if (e != hipSuccess) return set_hip_error(e, what, __FILE__, __LINE__);
  int rc = t.ensure(need, st);
  if (rc) return rc;
  size_t b = t.bytes;
  e = f(t.p, b);
  if (e != hipSuccess) return set_hip_error(e, what, __FILE__, __LINE__);
  return RSF_OK;
}

}  // namespace rsf

#define RSF_HIP(call)                                                       \
  do {                                                                        \
    hipError_t rsf_e_ = (call);                                               \
    if (rsf_e_ != hipSuccess) return rsf::set_hip_error(rsf_e_, #call, __FILE__, __LINE__); \
  } while (0)
