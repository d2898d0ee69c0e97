// Random 96-B row gathers over a 6 GiB table (the Vivaldi peer-row gather at 64M
// members): does spreading ONE row over several lanes (fewer distinct pages per
// wave-instruction) move the TLB-reach cliff?
//  L = lanes per row (1: each lane loads its own 6 x 16 B; 2: 3 x 16 B per lane;
//      6: one 16-B piece per lane, 10 rows per wave-instruction)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
__device__ inline uint32_t mix(uint64_t i) {
  uint64_t z = i * 0x9E3779B97F4A7C15ull;
  z ^= z >> 29;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 32;
  return (uint32_t)z;
}
template <int L>
__global__ void __launch_bounds__(256) gather(const double2* __restrict__ t, uint64_t nrows, uint64_t rows,
                                             uint64_t span_rows, double* sink) {
  // wave w gathers rows [w*RPW, (w+1)*RPW); RPW = 64 / L rounded down to whole rows
  constexpr int RPW = 64 / L;  // rows per wave-instruction group
  const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = gt / 64;
  double acc = 0;
  if (L == 1) {
    if (wave * 64 + lane >= rows) return;
    const uint64_t row = mix(wave * 64 + lane) % span_rows;
    const double2* r = t + row * 6;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      double2 v = r[k];
      acc += v.x + v.y;
    }
  } else {
    // the wave covers 64 rows (one per member) in L passes of RPW rows each
    const uint32_t sub = lane % L, rw = lane / L;
#pragma unroll
    for (int p = 0; p < (64 + RPW - 1) / RPW; ++p) {
      const uint32_t ri = p * RPW + rw;
      if (rw < RPW && ri < 64) {
        const uint64_t row = mix(wave * 64 + ri) % span_rows;
        const double2* r = t + row * 6;
#pragma unroll
        for (int k = sub; k < 6; k += L) {
          double2 v = r[k];
          acc += v.x + v.y;
        }
      }
    }
  }
  if (acc == 1.2345) sink[0] = acc;
}
int main() {
  const uint64_t bytes = 6ull << 30, nrows = bytes / 96;
  double2* t;
  double* sink;
  if (hipMalloc(&t, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
  (void)hipMemset(t, 0, bytes);
  const uint64_t rows = 64ull << 20;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (uint64_t span : {nrows / 4, nrows}) {
    for (int L : {1, 2, 3, 6}) {
      float best = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        const unsigned blocks = (unsigned)(rows / 256);
        if (L == 1) hipLaunchKernelGGL(gather<1>, dim3(blocks), dim3(256), 0, 0, t, nrows, rows, span, sink);
        if (L == 2) hipLaunchKernelGGL(gather<2>, dim3(blocks), dim3(256), 0, 0, t, nrows, rows, span, sink);
        if (L == 3) hipLaunchKernelGGL(gather<3>, dim3(blocks), dim3(256), 0, 0, t, nrows, rows, span, sink);
        if (L == 6) hipLaunchKernelGGL(gather<6>, dim3(blocks), dim3(256), 0, 0, t, nrows, rows, span, sink);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("span %5.2f GB  lanes/row %d: %.3f ms  %.0f GB/s useful\n", span * 96.0 / 1e9, L, best,
             rows * 96.0 / best / 1e6);
    }
  }
  return 0;
}
