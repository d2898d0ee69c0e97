// PMC calibration: FETCH_SIZE / WRITE_SIZE against KNOWN byte counts for the access
// shapes the engine uses (coalesced 4/8/16-B-per-lane streams, random 16/32/64/96-B
// record gathers and scatters).  Run under
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o run -- ./pmc_calib
// and the same with WRITE_SIZE; experiments/pmc_calib.py turns the two CSVs into
// counter/true-byte ratios.  Buffers are 2 GiB, far past the 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ inline uint32_t mix(uint64_t i) {
  uint64_t z = i * 0x9E3779B97F4A7C15ull;
  z ^= z >> 29; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 32;
  return (uint32_t)z;
}

// NT: non-temporal loads / stores (the Vivaldi round kernel's member-side streams)
template <typename T, bool NT = false>
__global__ void stream_read(const T* __restrict__ a, uint64_t n, uint64_t* sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  T v;
  if constexpr (NT) v = __builtin_nontemporal_load(a + i); else v = a[i];
  uint64_t x = 0;
  if constexpr (sizeof(T) < 4) {
    x = (uint64_t)v;
  } else {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
    for (unsigned k = 0; k < sizeof(T) / 4; ++k) x ^= w[k];
  }
  if (x == 0x12345679u) sink[0] = x;
}

template <typename T, bool NT = false>
__global__ void stream_write(T* __restrict__ a, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  T v;
  if constexpr (sizeof(T) < 4) {
    v = (T)i;
  } else {
    uint32_t* w = reinterpret_cast<uint32_t*>(&v);
    for (unsigned k = 0; k < sizeof(T) / 4; ++k) w[k] = (uint32_t)i + k;
  }
  if constexpr (NT) __builtin_nontemporal_store(v, a + i); else a[i] = v;
}
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

// random record gather: REC bytes per lane from a random REC-aligned slot (16-B loads)
template <int REC>
__global__ void gather(const uint4* __restrict__ a, uint64_t nrec, uint64_t lanes, uint64_t* sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lanes) return;
  const uint64_t r = mix(i) % nrec;
  const uint4* p = a + r * (REC / 16);
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < REC / 16; ++k) {
    uint4 v = p[k];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345679u) sink[0] = x;
}

template <int REC>
__global__ void scatter(uint4* __restrict__ a, uint64_t nrec, uint64_t lanes) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lanes) return;
  const uint64_t r = mix(i) % nrec;
  uint4* p = a + r * (REC / 16);
#pragma unroll
  for (int k = 0; k < REC / 16; ++k) p[k] = make_uint4((uint32_t)i, k, 1, 2);
}

int main() {
  const uint64_t bytes = 2ull << 30;
  void* buf;
  uint64_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(buf, 1, bytes));
  auto grid = [](uint64_t n) { return dim3((unsigned)((n + 255) / 256)); };
  // order matters: pmc_calib.py maps dispatch k to (name, true bytes)
  printf("calib stream_read4 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(stream_read<uint32_t>, grid(bytes / 4), dim3(256), 0, 0, (const uint32_t*)buf, bytes / 4, sink);
  printf("calib stream_read8 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(stream_read<uint2>, grid(bytes / 8), dim3(256), 0, 0, (const uint2*)buf, bytes / 8, sink);
  printf("calib stream_read16 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(stream_read<uint4>, grid(bytes / 16), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, sink);
  const uint64_t lanes = 16ull << 20;  // 16M random records per gather/scatter
  printf("calib gather16 %llu\n", (unsigned long long)(lanes * 16));
  hipLaunchKernelGGL(gather<16>, grid(lanes), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, lanes, sink);
  printf("calib gather32 %llu\n", (unsigned long long)(lanes * 32));
  hipLaunchKernelGGL(gather<32>, grid(lanes), dim3(256), 0, 0, (const uint4*)buf, bytes / 32, lanes, sink);
  printf("calib gather64 %llu\n", (unsigned long long)(lanes * 64));
  hipLaunchKernelGGL(gather<64>, grid(lanes), dim3(256), 0, 0, (const uint4*)buf, bytes / 64, lanes, sink);
  printf("calib gather96 %llu\n", (unsigned long long)(lanes * 96));
  hipLaunchKernelGGL(gather<96>, grid(lanes), dim3(256), 0, 0, (const uint4*)buf, bytes / 96, lanes, sink);
  printf("calib stream_write4 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(stream_write<uint32_t>, grid(bytes / 4), dim3(256), 0, 0, (uint32_t*)buf, bytes / 4);
  printf("calib stream_write8 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(stream_write<uint2>, grid(bytes / 8), dim3(256), 0, 0, (uint2*)buf, bytes / 8);
  printf("calib stream_write16 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(stream_write<uint4>, grid(bytes / 16), dim3(256), 0, 0, (uint4*)buf, bytes / 16);
  printf("calib scatter16 %llu\n", (unsigned long long)(lanes * 16));
  hipLaunchKernelGGL(scatter<16>, grid(lanes), dim3(256), 0, 0, (uint4*)buf, bytes / 16, lanes);
  printf("calib scatter32 %llu\n", (unsigned long long)(lanes * 32));
  hipLaunchKernelGGL(scatter<32>, grid(lanes), dim3(256), 0, 0, (uint4*)buf, bytes / 32, lanes);
  printf("calib scatter64 %llu\n", (unsigned long long)(lanes * 64));
  hipLaunchKernelGGL(scatter<64>, grid(lanes), dim3(256), 0, 0, (uint4*)buf, bytes / 64, lanes);
  // appended shapes (keep the order above stable for older summaries)
  printf("calib stream_read1 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_read<uint8_t>), grid(bytes), dim3(256), 0, 0, (const uint8_t*)buf, bytes, sink);
  printf("calib stream_read1_nt %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_read<uint8_t, true>), grid(bytes), dim3(256), 0, 0, (const uint8_t*)buf, bytes, sink);
  printf("calib stream_read4_nt %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_read<uint32_t, true>), grid(bytes / 4), dim3(256), 0, 0, (const uint32_t*)buf, bytes / 4, sink);
  printf("calib stream_read8_nt %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_read<u32x2v, true>), grid(bytes / 8), dim3(256), 0, 0, (const u32x2v*)buf, bytes / 8, sink);
  printf("calib stream_read16_nt %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_read<u32x4v, true>), grid(bytes / 16), dim3(256), 0, 0, (const u32x4v*)buf, bytes / 16, sink);
  printf("calib stream_write1 %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_write<uint8_t>), grid(bytes), dim3(256), 0, 0, (uint8_t*)buf, bytes);
  printf("calib stream_write1_nt %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_write<uint8_t, true>), grid(bytes), dim3(256), 0, 0, (uint8_t*)buf, bytes);
  printf("calib stream_write8_nt %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_write<u32x2v, true>), grid(bytes / 8), dim3(256), 0, 0, (u32x2v*)buf, bytes / 8);
  printf("calib stream_write16_nt %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL((stream_write<u32x4v, true>), grid(bytes / 16), dim3(256), 0, 0, (u32x4v*)buf, bytes / 16);
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  printf("calib done\n");
  return 0;
}
