// Random 96-B gathers over a 6 GiB table: which span restriction restores throughput?
//  mode 0: uniform over the whole table
//  mode 1: block b gathers only from octant (b % 8)  -> per-XCD span of 768 MiB
//  mode 2: block b gathers from sub-span (b * P / nblocks) -> all CUs on one span at a time
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ inline uint32_t mix(uint64_t i) {
  uint64_t z = i * 0x9E3779B97F4A7C15ull; z ^= z >> 29; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 32; return (uint32_t)z;
}
__global__ void __launch_bounds__(256) gather96(const double2* __restrict__ t, uint64_t nrows, uint64_t lanes,
                                                int mode, int P, double* sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lanes) return;
  uint64_t row;
  if (mode == 0) row = mix(i) % nrows;
  else if (mode == 1) { uint64_t sub = nrows / 8; row = (blockIdx.x % 8) * sub + mix(i) % sub; }
  else { uint64_t sub = nrows / P; row = ((uint64_t)blockIdx.x * P / gridDim.x) * sub + mix(i) % sub; }
  const double2* r = t + row * 6;
  double acc = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) { double2 v = r[k]; acc += v.x + v.y; }
  if (acc == 1.2345) sink[0] = acc;
}
int main() {
  const uint64_t bytes = 6ull << 30, nrows = bytes / 96;
  double2* t; double* sink;
  if (hipMalloc(&t, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
  (void)hipMemset(t, 0, bytes);
  const uint64_t lanes = 64ull << 20;
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  struct { int mode, P; } cfg[] = {{0, 1}, {1, 8}, {2, 2}, {2, 3}, {2, 4}, {2, 8}, {2, 16}};
  for (auto c : cfg) {
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(gather96, dim3(lanes / 256), dim3(256), 0, 0, t, nrows, lanes, c.mode, c.P, sink);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    printf("mode %d P %2d: %.3f ms  %.0f GB/s useful\n", c.mode, c.P, best, lanes * 96.0 / best / 1e6);
  }
  return 0;
}
