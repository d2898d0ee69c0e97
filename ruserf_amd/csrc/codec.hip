// codec.hip — batched wire codecs on CDNA4: Coordinate
// big-endian codec, ping ack payloads, and serf message frames (Join / Leave /
// UserEvent).  One lane per item: an item is 20-100 bytes, the lanes of a wave
// write neighbouring items, so stores merge into full lines in L2.  Variable
// frame sizes are placed with a device-wide exclusive scan (hipcub).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "../../include/ruserf_amd.h"
#include "codec.h"
#include "rsf_internal.h"

using namespace rsf;

namespace {

inline unsigned grid1(uint64_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }

__device__ __forceinline__ uint32_t str_len(uint32_t n) { return 4 + n; }

// encoded length of one frame: tag byte + message (join.rs:132-134, leave.rs:88-90, user_event.rs:330-332)
__device__ __forceinline__ uint32_t frame_len(const rsf_wire_msg& m) {
  const uint32_t vl = dvarint_len(m.ltime);
  switch (m.type) {
    case RSF_MSG_JOIN: return 1 + 4 + vl + str_len(m.a_len);
    case RSF_MSG_LEAVE: return 1 + 4 + 1 + str_len(m.a_len) + vl;
    case RSF_MSG_USER_EVENT: return 1 + 4 + vl + str_len(m.a_len) + str_len(m.b_len) + 1;
    default: return 0;
  }
}

__global__ void __launch_bounds__(256) wire_len_kernel(const rsf_wire_msg* __restrict__ msgs, uint64_t n,
                                                       uint64_t* __restrict__ off) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) off[0] = 0;
  if (i < n) off[i + 1] = frame_len(msgs[i]);
}

__device__ __forceinline__ uint32_t put_str(uint8_t* d, const uint8_t* blob, uint64_t o, uint32_t n) {
  put_be32(d, n);
  for (uint32_t k = 0; k < n; ++k) d[4 + k] = blob[o + k];
  return 4 + n;
}

// Transformable::encode of the message after its tag (join.rs:82-104, leave.rs:62-86,
// user_event.rs:306-328; tag: base.rs:373 / api.rs:293 write raw[0] then encode into raw[1..])
__global__ void __launch_bounds__(256) wire_encode_kernel(const rsf_wire_msg* __restrict__ msgs, uint64_t n,
                                                          const uint8_t* __restrict__ blob,
                                                          const uint64_t* __restrict__ off, uint8_t* __restrict__ out,
                                                          int32_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const rsf_wire_msg m = msgs[i];
  uint8_t* d = out + off[i];
  const uint32_t fl = frame_len(m);
  if (fl == 0) {
    if (status) status[i] = RSF_ERR_CODEC_TYPE;
    return;
  }
  d[0] = m.type;
  uint8_t* b = d + 1;
  put_be32(b, fl - 1);
  uint32_t o = 4;
  switch (m.type) {
    case RSF_MSG_JOIN:
      o += put_varint(b + o, m.ltime);
      o += put_str(b + o, blob, m.a_off, m.a_len);
      break;
    case RSF_MSG_LEAVE:
      b[o++] = m.flag ? 1 : 0;
      o += put_varint(b + o, m.ltime);
      o += put_str(b + o, blob, m.a_off, m.a_len);
      break;
    default:  // RSF_MSG_USER_EVENT
      b[o++] = m.flag ? 1 : 0;
      o += put_varint(b + o, m.ltime);
      o += put_str(b + o, blob, m.a_off, m.a_len);
      o += put_str(b + o, blob, m.b_off, m.b_len);
      break;
  }
  if (status) status[i] = RSF_OK;
}

// a SmolStr / Bytes at body[o] (avail bytes left in the body)
__device__ __forceinline__ int get_str(const uint8_t* body, uint64_t blen, uint64_t o, uint64_t base, uint64_t* s_off,
                                       uint32_t* s_len, uint64_t* end) {
  if (o > blen || blen - o < 4) return RSF_ERR_CODEC_SHORT;
  const uint32_t n = be32(body + o);
  if (blen - o - 4 < n) return RSF_ERR_CODEC_SHORT;
  *s_off = base + o + 4;
  *s_len = n;
  *end = o + 4 + n;
  return RSF_OK;
}

// notify_message's dispatch (delegate.rs:157-305: empty -> ignored, MessageType::try_from(msg[0]))
// and decode_message (transform.rs:266-300) for the Join / Leave / UserEvent arms
__device__ __forceinline__ void decode_frame(const uint8_t* __restrict__ buf, uint64_t fo, uint64_t flen,
                                             rsf_wire_msg& m) {
  m = rsf_wire_msg{};
  if (flen == 0) {
    m.status = RSF_SKIPPED;
    return;
  }
  const uint8_t* f = buf + fo;
  m.type = f[0];
  const uint8_t* body = f + 1;
  const uint64_t blen = flen - 1, base = fo + 1;
  int err = RSF_OK;
  switch (m.type) {
    case RSF_MSG_JOIN: {  // join.rs:106-130
      if (blen < 4) { m.status = RSF_ERR_CODEC_SHORT; return; }
      const uint32_t len = be32(body);
      if (blen < len) { m.status = RSF_ERR_CODEC_SHORT; return; }
      uint64_t o = 4, end;
      const uint32_t r = get_varint(body + o, blen - o, &m.ltime, &err);
      if (!r) { m.status = err; return; }
      o += r;
      if ((err = get_str(body, blen, o, base, &m.a_off, &m.a_len, &end))) { m.status = err; return; }
      m.frame_len = 1 + len;  // returns the header's length
      m.status = RSF_OK;
      return;
    }
    case RSF_MSG_LEAVE: {  // leave.rs:92-120
      if (blen < 5) { m.status = RSF_ERR_CODEC_SHORT; return; }
      const uint32_t len = be32(body);
      if (blen + 5 < len) { m.status = RSF_ERR_CODEC_SHORT; return; }  // the reference's check, verbatim
      m.flag = body[4] != 0;
      uint64_t o = 5, end;
      const uint32_t r = get_varint(body + o, blen - o, &m.ltime, &err);
      if (!r) { m.status = err; return; }
      o += r;
      if ((err = get_str(body, blen, o, base, &m.a_off, &m.a_len, &end))) { m.status = err; return; }
      m.frame_len = (uint32_t)(1 + end);  // returns the bytes read
      m.status = RSF_OK;
      return;
    }
    case RSF_MSG_USER_EVENT: {  // user_event.rs:334-370
      if (blen < 4) { m.status = RSF_ERR_CODEC_SHORT; return; }
      const uint32_t len = be32(body);
      if (blen < len || blen < 5) { m.status = RSF_ERR_CODEC_SHORT; return; }
      m.flag = body[4] != 0;
      uint64_t o = 5, end;
      const uint32_t r = get_varint(body + o, blen - o, &m.ltime, &err);
      if (!r) { m.status = err; return; }
      o += r;
      if ((err = get_str(body, blen, o, base, &m.a_off, &m.a_len, &end))) { m.status = err; return; }
      if ((err = get_str(body, blen, end, base, &m.b_off, &m.b_len, &end))) { m.status = err; return; }
      m.frame_len = 1 + len;
      m.status = RSF_OK;
      return;
    }
    default:
      m.status = RSF_ERR_CODEC_TYPE;  // unknown tag, or a message kind this codec does not carry
      return;
  }
}

__global__ void __launch_bounds__(256) wire_decode_kernel(const uint8_t* __restrict__ buf,
                                                          const uint64_t* __restrict__ off, uint64_t n,
                                                          rsf_wire_msg* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = off[i], b = off[i + 1];
  rsf_wire_msg m;
  if (b < a) {
    m = rsf_wire_msg{};
    m.status = RSF_ERR_ARG;
  } else {
    decode_frame(buf, a, b - a, m);
  }
  out[i] = m;
}

__global__ void __launch_bounds__(256) coord_encode_kernel(const double* __restrict__ rows, uint32_t dim,
                                                           uint32_t stride, uint64_t n, uint8_t* __restrict__ out,
                                                           uint64_t out_stride, uint32_t ping) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* d = out + i * out_stride;
  if (ping) *d++ = kPingVersion;
  coord_encode(d, rows + i * stride, dim);
}

__global__ void __launch_bounds__(256) coord_decode_kernel(const uint8_t* __restrict__ in,
                                                           const uint64_t* __restrict__ off, uint64_t n,
                                                           uint32_t ping, double* __restrict__ rows, uint32_t stride,
                                                           uint32_t max_dim, uint32_t* __restrict__ dim_out,
                                                           int32_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = off[i], b = off[i + 1];
  int st;
  uint32_t dim = 0;
  if (b < a) {
    st = RSF_ERR_ARG;
  } else {
    const uint8_t* p = in + a;
    uint64_t len = b - a;
    st = RSF_OK;
    if (ping) {  // notify_ping_complete (delegate.rs:704-725): empty -> ignored, version byte first
      if (len == 0) st = RSF_SKIPPED;
      else if (p[0] != kPingVersion) st = RSF_ERR_CODEC_TYPE;
      p++;
      len = len ? len - 1 : 0;
    }
    if (st == RSF_OK) st = coord_decode(p, len, max_dim, rows + i * stride, &dim);
  }
  if (dim_out) dim_out[i] = dim;
  status[i] = st;
}

int scan_lengths(uint64_t* off, uint64_t n, hipStream_t st) {
  size_t tb = 0;
  RSF_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, off + 1, off + 1, (int)n, st));
  void* tmp = nullptr;
  RSF_HIP(hipMallocAsync(&tmp, tb ? tb : 16, st));
  hipError_t e = hipcub::DeviceScan::InclusiveSum(tmp, tb, off + 1, off + 1, (int)n, st);
  hipFreeAsync(tmp, st);
  RSF_HIP(e);
  return RSF_OK;
}

}  // namespace

extern "C" {

int rsf_wire_encoded_lengths(const rsf_wire_msg* msgs, uint64_t n, uint64_t* off, void* stream) {
  if ((n && !msgs) || !off) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (n >= 0x7FFFFFFFull) return rsf::set_error(RSF_ERR_ARG, "batch too large");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(wire_len_kernel, dim3(grid1(n ? n : 1)), dim3(256), 0, st, msgs, n, off);
  RSF_HIP(hipGetLastError());
  if (n) return scan_lengths(off, n, st);
  return RSF_OK;
}

int rsf_wire_encode(const rsf_wire_msg* msgs, uint64_t n, const uint8_t* blob, const uint64_t* off, uint8_t* out,
                    int32_t* status, void* stream) {
  if (n && (!msgs || !off || !out)) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (!n) return RSF_OK;
  hipLaunchKernelGGL(wire_encode_kernel, dim3(grid1(n)), dim3(256), 0, (hipStream_t)stream, msgs, n, blob, off, out,
                     status);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_wire_decode(const uint8_t* buf, const uint64_t* off, uint64_t n, rsf_wire_msg* out, void* stream) {
  if (n && (!buf || !off || !out)) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (!n) return RSF_OK;
  hipLaunchKernelGGL(wire_decode_kernel, dim3(grid1(n)), dim3(256), 0, (hipStream_t)stream, buf, off, n, out);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_coord_encode(const double* rows, uint32_t dim, uint32_t row_stride, uint64_t n, uint8_t* out,
                     uint64_t out_stride, int ping_version_prefix, void* stream) {
  if (n && (!rows || !out)) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (dim == 0 || dim > 64 || row_stride < dim + 3) return rsf::set_error(RSF_ERR_ARG, "bad dimensionality/stride");
  if (out_stride < (uint64_t)(ping_version_prefix ? 1 : 0) + kCoordHdr + 8ull * dim)
    return rsf::set_error(RSF_ERR_ARG, "output stride too small");
  if (!n) return RSF_OK;
  hipLaunchKernelGGL(coord_encode_kernel, dim3(grid1(n)), dim3(256), 0, (hipStream_t)stream, rows, dim, row_stride, n,
                     out, out_stride, (uint32_t)(ping_version_prefix != 0));
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_coord_decode(const uint8_t* in, const uint64_t* off, uint64_t n, int ping_version_prefix, double* rows,
                     uint32_t row_stride, uint32_t max_dim, uint32_t* dim_out, int32_t* status, void* stream) {
  if (n && (!in || !off || !rows || !status)) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (max_dim == 0 || row_stride < max_dim + 3) return rsf::set_error(RSF_ERR_ARG, "row stride below max_dim + 3");
  if (!n) return RSF_OK;
  hipLaunchKernelGGL(coord_decode_kernel, dim3(grid1(n)), dim3(256), 0, (hipStream_t)stream, in, off, n,
                     (uint32_t)(ping_version_prefix != 0), rows, row_stride, max_dim, dim_out, status);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

}  // extern "C"
