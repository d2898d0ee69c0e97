// common.h — device/host helpers shared by the ruserf_amd HIP kernels.
//
// Philox4x32-10 is the counter-based generator that replaces the reference's
// thread_rng (coordinate.rs:812-821) and memberlist's peer shuffles, so that a
// run is a pure function of (seed, round, member, purpose, draw).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RSF_HD __host__ __device__ __forceinline__

namespace rsf {

// purpose tags (ctr[1] bits 24..31); the oracle uses the same numbering
enum : uint32_t {
  kPurposeUnit = 1,    // rand_f64 draws of unit_vector_at
  kPurposePeer = 2,    // gossip peer selection (kRandomNodes model)
  kPurposeVProbe = 3,  // Vivaldi synthetic probe: neighbour slot + jitter
  kPurposeNbr = 5,     // Vivaldi fixed neighbour set
  kPurposePos = 6,     // Vivaldi ground-truth positions
  kPurposeReconnect = 7,  // Reconnector: throttle draw + failed-member pick
};

struct u32x4 {
  uint32_t x, y, z, w;
};

RSF_HD u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                           uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return {c0, c1, c2, c3};
}

RSF_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

// `f64 as u64` in Rust: truncate toward zero, saturate, NaN -> 0
RSF_HD uint64_t sat_u64(double x) {
  if (!(x > 0.0)) return 0;
  if (x >= 18446744073709551616.0) return UINT64_MAX;
  return (uint64_t)x;
}

// Duration::as_secs_f64 = secs as f64 + nanos as f64 / 1e9.  The division is done as
// q0 = x * RN(1e-9), then one FMA correction: for every integer x in [0, 1e9) -- the whole
// domain of nanos -- this equals the correctly rounded x / 1e9 (checked exhaustively,
// tests/test_div1e9.py), in 3 f64 operations instead of the ~10 of a general division.
RSF_HD double as_secs_f64(uint64_t ns) {
  uint64_t secs = ns / 1000000000ull;
  uint32_t nanos = (uint32_t)(ns - secs * 1000000000ull);
  const double x = (double)nanos, r = 1.0 / 1e9;
  const double q0 = x * r;
  const double q = __builtin_fma(__builtin_fma(-q0, 1e9, x), r, q0);
  return (double)secs + q;
}

// f64::max / f64::min (non-NaN operand wins) == IEEE maxNum/minNum
RSF_HD double rmax(double a, double b) { return fmax(a, b); }
RSF_HD double rmin(double a, double b) { return fmin(a, b); }

// XCD-aware block order.  The dispatcher hands block b to XCD b % 8 (each XCD has its
// own L2 and translation caches); remapping gives every XCD one contiguous range of
// the logical blocks, so neighbouring members (adjacent records, segment bounds, rows
// in the same 2 MB page) are served by one L2 instead of eight.  A bijection on
// [0, nb) for any nb.
#ifndef RSF_XCD_REMAP
#define RSF_XCD_REMAP 0  // measured ~1% slower for merge/emit and Vivaldi
#endif
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
#if RSF_XCD_REMAP
  constexpr uint32_t kXcd = 8;
  const uint32_t x = b % kXcd, i = b / kXcd, q = nb / kXcd, r = nb % kXcd;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
#else
  (void)nb;
  return b;
#endif
}

}  // namespace rsf
