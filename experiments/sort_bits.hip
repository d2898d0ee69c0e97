// Group sort of the gossip round (6M (receiver, group id) pairs, 21-bit receiver keys) with
// rocPRIM onesweep at 8 bits per pass (the gfx950 tuned default: 3 passes) against 11 bits
// per pass (2 passes); checks the outputs are identical.  Build: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace rocprim;
template <unsigned B, unsigned BS, unsigned IPT>
using ocfg = radix_sort_config<default_config, default_config,
                               radix_sort_onesweep_config<kernel_config<BS, IPT>, kernel_config<BS, IPT>, B,
                                                          block_radix_rank_algorithm::match>>;
template <class Cfg>
float run(const char* name, unsigned* k, unsigned* v, unsigned* ko, unsigned* vo, size_t n, int bits, std::vector<unsigned>& out) {
  size_t tmp = 0;
  CK(radix_sort_pairs<Cfg>(nullptr, tmp, k, ko, v, vo, n, 0, bits, 0));
  void* t;
  CK(hipMalloc(&t, tmp));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) CK(radix_sort_pairs<Cfg>(t, tmp, k, ko, v, vo, n, 0, bits, 0));
  CK(hipEventRecord(a, 0));
  const int R = 20;
  for (int r = 0; r < R; ++r) CK(radix_sort_pairs<Cfg>(t, tmp, k, ko, v, vo, n, 0, bits, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  out.resize(2 * n);
  CK(hipMemcpy(out.data(), ko, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(out.data() + n, vo, n * 4, hipMemcpyDeviceToHost));
  printf("%-28s %.4f ms per sort (temp %zu B)\n", name, ms / R, tmp);
  CK(hipFree(t));
  return ms / R;
}
int main() {
  const size_t n = 6000000;
  const int bits = 21;
  std::vector<unsigned> hk(n), hv(n);
  unsigned s = 12345;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    hk[i] = (s >> 8) % 2000000u;
    hv[i] = (unsigned)i;
  }
  unsigned *k, *v, *ko, *vo;
  CK(hipMalloc(&k, n * 4)); CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&ko, n * 4)); CK(hipMalloc(&vo, n * 4));
  CK(hipMemcpy(k, hk.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, hv.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<unsigned> r0, r1, r2, r3;
  run<default_config>("default (tuned, 8 bits)", k, v, ko, vo, n, bits, r0);
  run<ocfg<11, 1024, 8>>("onesweep 11 bits 1024x8", k, v, ko, vo, n, bits, r1);
  run<ocfg<11, 512, 8>>("onesweep 11 bits 512x8", k, v, ko, vo, n, bits, r2);
  run<ocfg<7, 1024, 12>>("onesweep 7 bits 1024x12", k, v, ko, vo, n, bits, r3);
  printf("identical: %d %d %d\n", r1 == r0, r2 == r0, r3 == r0);
  return 0;
}
