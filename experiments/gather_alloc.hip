// Random 96-B gathers over a 6 GiB table allocated three ways: does the allocation
// (fragment size / physical contiguity) move the TLB cliff?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ inline uint32_t mix(uint64_t i) {
  uint64_t z = i * 0x9E3779B97F4A7C15ull; z ^= z >> 29; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 32; return (uint32_t)z;
}
__global__ void __launch_bounds__(256) gather96(const double2* __restrict__ t, uint64_t nrows, uint64_t lanes, double* sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lanes) return;
  const double2* r = t + (uint64_t)(mix(i) % nrows) * 6;
  double acc = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) { double2 v = r[k]; acc += v.x + v.y; }
  if (acc == 1.2345) sink[0] = acc;
}
static void run(const char* name, double2* t, uint64_t bytes, double* sink) {
  const uint64_t lanes = 64ull << 20;
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipMemset(t, 0, bytes);
  float best = 1e9;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(gather96, dim3(lanes / 256), dim3(256), 0, 0, t, bytes / 96, lanes, sink);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
  }
  printf("%-28s %.3f ms  %.0f GB/s useful\n", name, best, lanes * 96.0 / best / 1e6);
}
int main() {
  const uint64_t bytes = 6ull << 30;
  double* sink; (void)hipMalloc(&sink, 8);
  double2* t = nullptr;
  if (hipMalloc(&t, bytes) == hipSuccess) { run("hipMalloc", t, bytes, sink); (void)hipFree(t); }
  if (hipExtMallocWithFlags((void**)&t, bytes, hipDeviceMallocContiguous) == hipSuccess) {
    run("hipExtMalloc contiguous", t, bytes, sink); (void)hipFree(t);
  } else printf("contiguous alloc failed\n");
  // virtual memory management API with the largest recommended granularity
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gmin = 0, grec = 0;
  (void)hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum);
  (void)hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended);
  printf("VMM granularity min %zu rec %zu\n", gmin, grec);
  hipMemGenericAllocationHandle_t h;
  void* va = nullptr;
  if (hipMemCreate(&h, bytes, &prop, 0) == hipSuccess &&
      hipMemAddressReserve(&va, bytes, 1ull << 30, nullptr, 0) == hipSuccess &&
      hipMemMap(va, bytes, 0, h, 0) == hipSuccess) {
    hipMemAccessDesc d = {};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemSetAccess(va, bytes, &d, 1) == hipSuccess) run("VMM 1GiB-aligned", (double2*)va, bytes, sink);
    (void)hipMemUnmap(va, bytes);
    (void)hipMemAddressFree(va, bytes);
    (void)hipMemRelease(h);
  } else printf("VMM path failed\n");
  return 0;
}
