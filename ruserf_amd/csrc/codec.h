// codec.h — device restatement of ruserf's wire formats (scalar, one lane per
// item; the batched kernels are in codec.hip).
//
//   varint      LEB128 u64 (transformable 0.1 utils::encode_varint / decode_varint,
//               used for LamportTime, types/src/clock.rs:109-127; un-vendored:
//               restated from its published algorithm, parity unpinned)
//   Coordinate  u32 BE total length | error | adjustment | height | portion[]
//               all f64 big-endian (core/src/coordinate.rs:663-745)
//   strings     SmolStr / Bytes: u32 BE byte length | bytes (transformable 0.1,
//               un-vendored; parity unpinned)
//   frames      [MessageType tag u8][message] (core/src/serf/base.rs:373,
//               api.rs:293; tags types/src/message.rs:17-24)
//               JoinMessage      u32 BE len | varint ltime | id           (types/src/join.rs:82-135)
//               LeaveMessage     u32 BE len | prune u8 | varint ltime | id (types/src/leave.rs:58-120)
//               UserEventMessage u32 BE len | cc u8 | varint ltime | name | payload
//                                                                         (types/src/user_event.rs:303-370)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ruserf_amd.h"

namespace rsf {

constexpr uint8_t kPingVersion = 1;  // core/src/serf/delegate.rs:34
constexpr uint32_t kCoordHdr = 4 + 3 * 8;

__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
__device__ __forceinline__ void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}
__device__ __forceinline__ double be_f64(const uint8_t* p) {
  uint64_t u = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) u = (u << 8) | p[i];
  return __longlong_as_double((long long)u);
}
__device__ __forceinline__ void put_be_f64(uint8_t* p, double d) {
  uint64_t u = (uint64_t)__double_as_longlong(d);
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    p[i] = (uint8_t)u;
    u >>= 8;
  }
}

__device__ __forceinline__ uint32_t dvarint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}
__device__ __forceinline__ uint32_t put_varint(uint8_t* p, uint64_t v) {
  uint32_t n = 0;
  while (v >= 0x80) {
    p[n++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  p[n++] = (uint8_t)v;
  return n;
}
// returns bytes read, or 0 with *err set (buffer underflow -> SHORT; more than
// 10 bytes or a 10th byte above 1 -> VARINT)
__device__ __forceinline__ uint32_t get_varint(const uint8_t* p, uint64_t avail, uint64_t* v, int* err) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < 10; ++i) {
    if (i >= avail) {
      *err = RSF_ERR_CODEC_SHORT;
      return 0;
    }
    const uint8_t b = p[i];
    if (i == 9 && b > 1) {
      *err = RSF_ERR_CODEC_VARINT;
      return 0;
    }
    x |= (uint64_t)(b & 0x7F) << (7 * i);
    if (b < 0x80) {
      *v = x;
      return i + 1;
    }
  }
  *err = RSF_ERR_CODEC_VARINT;
  return 0;
}

// Coordinate::encode (coordinate.rs:666-692); returns bytes written
__device__ __forceinline__ uint32_t coord_encode(uint8_t* dst, const double* row, uint32_t dim) {
  const uint32_t len = kCoordHdr + 8 * dim;
  put_be32(dst, len);
  put_be_f64(dst + 4, row[dim]);       // error
  put_be_f64(dst + 12, row[dim + 1]);  // adjustment
  put_be_f64(dst + 20, row[dim + 2]);  // height
  for (uint32_t i = 0; i < dim; ++i) put_be_f64(dst + kCoordHdr + 8 * i, row[i]);
  return len;
}

// Coordinate::decode (coordinate.rs:698-745) into a row (portion[dim], error,
// adjustment, height).  Release-build semantics: the portion count is
// floor((len - 28) / 8) and the returned length is the header's.  A header
// below 28 bytes (the reference would underflow and panic) or a portion count
// above max_dim are RSF_ERR_CODEC_LEN.
__device__ __forceinline__ int coord_decode(const uint8_t* src, uint64_t src_len, uint32_t max_dim, double* row,
                                            uint32_t* dim_out) {
  if (src_len < kCoordHdr) return RSF_ERR_CODEC_SHORT;
  const uint32_t len = be32(src);
  if (src_len < len) return RSF_ERR_CODEC_SHORT;
  if (len < kCoordHdr) return RSF_ERR_CODEC_LEN;
  const uint32_t dim = (len - kCoordHdr) / 8;
  if (dim > max_dim) return RSF_ERR_CODEC_LEN;
  for (uint32_t i = 0; i < dim; ++i) row[i] = be_f64(src + kCoordHdr + 8 * i);
  row[dim] = be_f64(src + 4);
  row[dim + 1] = be_f64(src + 12);
  row[dim + 2] = be_f64(src + 20);
  *dim_out = dim;
  return RSF_OK;
}

}  // namespace rsf
