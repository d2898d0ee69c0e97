// Floor of the merge kernel's memory pattern: per receiver row of S view
// entries, ~27 record slots streamed (8 B: rumor id + decoration), then one random view
// entry per record read (a dependent round trip), ~20 of them written back.  No protocol
// logic: this prices the access pattern alone, at the bench's 2M members x 4096 subjects.
//   V0 records only | V1 + view reads | V2 + write-back | V3 as V2 with 8-B entries
//   V4 as V2, two receivers per wave (half-waves) | V5 as V2 with one receiver per wave
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr uint32_t S = 4096, SLOTS = 27, DIRTY = 20;
__device__ inline uint32_t mix(uint64_t i) {
  uint64_t z = i * 0x9E3779B97F4A7C15ull; z ^= z >> 29; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 32; return (uint32_t)z;
}
__global__ void fill_rec(uint2* rec, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) rec[i] = make_uint2(mix(i), mix(i + 0x1234567ull) % S);
}
// MODE 0: records only; 1: + reads; 2: + writes; 3: writes of the whole aligned SPAN-byte
// piece holding the entry (read whole, one entry modified, written whole: full-sector writes
// need no read-modify-write below L2).  E: entry type.  HALF: 2 rows per wave.
// PEND: + an append of the lanes < PEND_N to the row's 128-entry pending list, 12 B each:
// 1 = three SoA arrays (rid, dec, len|queue), 2 = one AoS array of 12-B entries
constexpr uint32_t PEND_N = 13, KPEND = 128;
__device__ uint32_t* g_pend;
template <int MODE, typename E, bool HALF, int RPW, int SPAN = 64, int PEND = 0, uint32_t DW = DIRTY, uint32_t PN = PEND_N>
__global__ void __launch_bounds__(256) floor_kernel(const uint2* __restrict__ rec, E* __restrict__ view, uint64_t n,
                                                    uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const uint32_t sub = HALF ? lane & 31 : lane;
  const uint32_t half = HALF ? lane >> 5 : 0;
  const uint64_t r0 = w * RPW * (HALF ? 2 : 1);
  uint32_t acc = 0;
  for (int k = 0; k < RPW; ++k) {
    const uint64_t row = r0 + (uint64_t)k * (HALF ? 2 : 1) + half;
    if (row >= n || sub >= SLOTS) continue;  // (PEND appends below, per row)
    const uint2 r = rec[row * SLOTS + sub];
    acc ^= r.x;
    if (MODE == 3) {
      constexpr uint32_t K = SPAN / 16;
      uint4* p = (uint4*)view + row * S + (r.y & ~(K - 1));
      uint4 v[K];
#pragma unroll
      for (uint32_t i = 0; i < K; ++i) v[i] = p[i];
      acc ^= v[r.y & (K - 1)].x;
      if (sub < DW) {
        v[r.y & (K - 1)].x += r.x;
#pragma unroll
        for (uint32_t i = 0; i < K; ++i) p[i] = v[i];
      }
    } else if (MODE >= 1) {
      E* p = view + row * S + r.y;
      E v = *p;
      if constexpr (sizeof(E) == 16) {
        acc ^= ((const uint4*)&v)->x;
        if (MODE >= 2 && sub < DW) { ((uint4*)&v)->x += r.x; *p = v; }
      } else {
        acc ^= (uint32_t)(*(const uint64_t*)&v);
        if (MODE >= 2 && sub < DW) { *(uint64_t*)&v += r.x; *p = v; }
      }
    }
    if (PEND && sub < PN) {
      const uint32_t at = (uint32_t)(row & 7) * 8;  // a list already part-filled
      if (PEND == 1) {
        g_pend[row * KPEND + at + sub] = r.x;
        g_pend[(n + row) * KPEND + at + sub] = r.y;
        g_pend[(2 * n + row) * KPEND + at + sub] = sub;
      } else {
        uint3* p = (uint3*)g_pend + row * KPEND + at + sub;
        *p = make_uint3(r.x, r.y, sub);
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int MODE, typename E, bool HALF, int RPW, int SPAN = 64, int PEND = 0, uint32_t DW = DIRTY, uint32_t PN = PEND_N>
float run(const char* name, const uint2* rec, void* view, uint64_t n, uint32_t* sink) {
  const uint64_t waves = (n + RPW * (HALF ? 2 : 1) - 1) / (RPW * (HALF ? 2 : 1));
  const dim3 grid((unsigned)((waves + 3) / 4));
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e9;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL((floor_kernel<MODE, E, HALF, RPW, SPAN, PEND, DW, PN>), grid, dim3(256), 0, 0, rec, (E*)view, n, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (rep && ms < best) best = ms;
  }
  const double recs = (double)n * SLOTS;
  printf("%-34s %7.3f ms  (%.2f G records/s; view sectors read %.2f TB/s)\n", name, best, recs / best / 1e6,
         MODE >= 1 ? recs * 64 / best / 1e9 : 0.0);
  return best;
}

int main() {
  const uint64_t n = 2000000;
  uint2* rec;
  void* view;
  uint32_t* sink;
  if (hipMalloc(&rec, n * SLOTS * 8) || hipMalloc(&view, n * S * 16) || hipMalloc(&sink, 64)) {
    printf("alloc failed\n");
    return 1;
  }
  hipLaunchKernelGGL(fill_rec, dim3((unsigned)((n * SLOTS + 255) / 256)), dim3(256), 0, 0, rec, n * SLOTS);
  hipMemset(view, 0, n * S * 16);
  hipDeviceSynchronize();
  uint32_t* pend;
  if (hipMalloc(&pend, 3 * n * KPEND * 4)) return 1;
  hipMemcpyToSymbol(HIP_SYMBOL(g_pend), &pend, sizeof(pend));
  // the bench's measured mix: 27 records per receiver, ~91% of them newer than the view
  // (written back and re-queued: ~49M of 54M per round)
  run<2, uint4, false, 8, 64, 2, 24, 24>("V14 bench mix: 24 writes + 24 AoS appends", rec, view, n, sink);
  run<2, uint4, false, 8, 64, 0, 24, 24>("V15 bench mix without appends", rec, view, n, sink);
  run<2, uint4, false, 8, 64, 1>("V10 V2 + pending appends, 3 SoA", rec, view, n, sink);
  run<2, uint4, false, 8, 64, 2>("V11 V2 + pending appends, AoS 12B", rec, view, n, sink);
  run<0, uint4, false, 8, 64, 1>("V12 V0 + pending appends, 3 SoA", rec, view, n, sink);
  run<0, uint4, false, 8, 64, 2>("V13 V0 + pending appends, AoS 12B", rec, view, n, sink);
  run<2, uint4, false, 8>("V2 + write-back (merge pattern)", rec, view, n, sink);
  run<0, uint4, false, 8>("V0 records only", rec, view, n, sink);
  run<1, uint4, false, 8>("V1 + 16-B view reads", rec, view, n, sink);
  run<2, uint4, false, 8>("V2 + write-back (merge pattern)", rec, view, n, sink);
  return 0;
}
