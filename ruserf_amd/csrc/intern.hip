// intern.hip — device-side interning of byte strings (user-event names and payloads),
// so a user event's identity can be computed from wire bytes without the host.
//
// The reference compares a user event's identity by value: `prev.name == name &&
// prev.payload == payload` in handle_user_event (core/src/serf/base.rs:801-806), and the
// coalescer keys its IndexMap by the name (coalesce/user.rs:60-75).  The engine carries
// that identity as an exact 64-bit key (name_id << 32 | payload_id).  This table assigns
// the ids on the device: equal bytes <-> equal id (bytes are compared, a hash only picks
// the probe start), and new strings get ids in order of first occurrence in the batch, so
// the result equals a host interner that walks the strings in order (deterministic, not
// scheduling dependent).
//
// One batch of n strings:
//   1. FNV-1a 64 of every string; stable radix sort of (hash, index)
//   2. per sorted element, its representative: the first element of its hash run with
//      equal bytes (the run's first, except on a real collision) -- the smallest index
//   3. each representative probes the persistent table (open addressing): found -> id;
//      otherwise it is new
//   4. new representatives, flagged at their batch index, are ranked by an exclusive scan
//      (ids = n_ids + rank) and their bytes packed into the arena (scan of lengths)
//   5. new representatives claim table slots (CAS on the hash word) and copy their bytes;
//      every string takes its representative's id
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "../../include/ruserf_amd.h"
#include "rsf_internal.h"

struct rsf_interner {
  int device = 0;
  uint32_t cap = 0;          // table slots (power of two, 2x the id capacity)
  uint32_t max_ids = 0;
  uint64_t arena_cap = 0;
  uint32_t n_ids = 0;        // host mirror of the committed count
  uint64_t arena_used = 0;   // host mirror
  unsigned long long* key = nullptr;  // slot hash (0 = empty)
  uint32_t* sid = nullptr;            // slot id
  uint32_t* slen = nullptr;           // slot string length
  uint64_t* soff = nullptr;           // slot arena offset
  uint8_t* arena = nullptr;
};

namespace {

inline unsigned grid1(uint64_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }

__device__ __forceinline__ uint64_t fnv1a(const uint8_t* p, uint32_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
  return h ? h : 1ull;  // 0 marks an empty slot
}
__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

constexpr uint32_t kNoString = 0xFFFFFFFFu;  // a length marking "nothing to intern" (id kNoString)
__global__ void in_hash_kernel(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                               const uint32_t* __restrict__ len, uint64_t n, uint64_t* __restrict__ h,
                               uint32_t* __restrict__ idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  h[i] = len[i] == kNoString ? 0ull : fnv1a(buf + off[i], len[i]);
  idx[i] = (uint32_t)i;
}
// run starts of the sorted hashes: head position or 0, then an inclusive max-scan
__global__ void in_heads_kernel(const uint64_t* __restrict__ h_s, uint64_t n, uint32_t* __restrict__ head) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  head[j] = (j == 0 || h_s[j - 1] != h_s[j]) ? (uint32_t)j : 0u;
}

// per sorted element j: rep[j] = sorted position of the first element of its hash run
// with equal bytes; a representative looks itself up in the table (found id, or new:
// flagged at its batch index with its length)
__global__ void in_group_kernel(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                const uint32_t* __restrict__ len, const uint64_t* __restrict__ h_s,
                                const uint32_t* __restrict__ idx_s, const uint32_t* __restrict__ run_start,
                                uint64_t n, rsf_interner t,
                                uint32_t* __restrict__ rep, uint32_t* __restrict__ found,
                                uint32_t* __restrict__ is_new, uint64_t* __restrict__ new_len) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t h = h_s[j];
  const uint32_t me = idx_s[j], L = len[me];
  if (L == kNoString) {
    rep[j] = (uint32_t)j;
    found[j] = kNoString;
    return;
  }
  const uint64_t s = run_start[j];  // equal strings: one comparison, with the run's first
  const uint8_t* mine = buf + off[me];
  uint64_t r = j;
  for (uint64_t k = s; k < j; ++k) {
    const uint32_t o = idx_s[k];
    if (len[o] == L && bytes_eq(buf + off[o], mine, L)) {
      r = k;
      break;
    }
  }
  rep[j] = (uint32_t)r;
  if (r != j) return;
  // a representative: probe the committed table
  uint32_t p = (uint32_t)h & (t.cap - 1), id = 0xFFFFFFFFu;
  for (;;) {
    const unsigned long long k = t.key[p];
    if (k == 0) break;
    if (k == h && t.slen[p] == L && bytes_eq(t.arena + t.soff[p], mine, L)) {
      id = t.sid[p];
      break;
    }
    p = (p + 1) & (t.cap - 1);
  }
  found[j] = id;
  if (id == 0xFFFFFFFFu) {
    is_new[me] = 1u;
    new_len[me] = L;
  }
}

// new representatives: id = n_ids + rank (by batch index), bytes into the arena, a table
// slot claimed by CAS (distinct new strings may share a hash: each takes its own slot)
__global__ void in_insert_kernel(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                 const uint32_t* __restrict__ len, const uint64_t* __restrict__ h_s,
                                 const uint32_t* __restrict__ idx_s, const uint32_t* __restrict__ rep, uint64_t n,
                                 rsf_interner t, const uint32_t* __restrict__ rank,
                                 const uint64_t* __restrict__ arena_off, uint32_t* __restrict__ found) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || rep[j] != j || found[j] != 0xFFFFFFFFu) return;
  const uint32_t me = idx_s[j], L = len[me];
  if (L == kNoString) return;
  const uint32_t id = t.n_ids + rank[me];
  const uint64_t ao = t.arena_used + arena_off[me];
  for (uint32_t i = 0; i < L; ++i) t.arena[ao + i] = buf[off[me] + i];
  const unsigned long long h = h_s[j];
  uint32_t p = (uint32_t)h & (t.cap - 1);
  while (atomicCAS(t.key + p, 0ull, h) != 0ull) p = (p + 1) & (t.cap - 1);
  t.sid[p] = id;
  t.slen[p] = L;
  t.soff[p] = ao;
  found[j] = id;
}

__global__ void in_ids_kernel(const uint32_t* __restrict__ idx_s, const uint32_t* __restrict__ rep,
                              const uint32_t* __restrict__ found, uint64_t n, uint32_t* __restrict__ ids) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  ids[idx_s[j]] = found[rep[j]];
}

// decoded wire messages -> the strings to intern (names, payloads); non-events: empty
__global__ void in_wire_kernel(const rsf_wire_msg* __restrict__ m, uint64_t n, uint64_t* __restrict__ noff,
                               uint32_t* __restrict__ nlen, uint64_t* __restrict__ poff, uint32_t* __restrict__ plen) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const rsf_wire_msg x = m[i];
  const bool ev = x.type == RSF_MSG_USER_EVENT && x.status == RSF_OK;
  noff[i] = ev ? x.a_off : 0;
  nlen[i] = ev ? x.a_len : kNoString;
  poff[i] = ev ? x.b_off : 0;
  plen[i] = ev ? x.b_len : kNoString;
}
__global__ void in_keys_kernel(const rsf_wire_msg* __restrict__ m, const uint32_t* __restrict__ nid,
                               const uint32_t* __restrict__ pid, uint64_t n, uint64_t* __restrict__ keys) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool ev = m[i].type == RSF_MSG_USER_EVENT && m[i].status == RSF_OK;
  keys[i] = ev ? ((uint64_t)nid[i] << 32) | pid[i] : 0ull;
}

struct Scratch {
  hipStream_t st;
  void* p = nullptr;
  explicit Scratch(hipStream_t s) : st(s) {}
  ~Scratch() {
    if (p) hipFreeAsync(p, st);
  }
};

}  // namespace

extern "C" {

int rsf_interner_create(rsf_interner** out, uint32_t max_ids, uint64_t arena_bytes, int device) {
  if (!out) return rsf::set_error(RSF_ERR_ARG, "null argument");
  *out = nullptr;
  if (max_ids == 0 || max_ids > (1u << 30)) return rsf::set_error(RSF_ERR_ARG, "max_ids must be in [1, 2^30]");
  RSF_HIP(hipSetDevice(device));
  rsf_interner* t = new rsf_interner();
  t->device = device;
  t->max_ids = max_ids;
  t->cap = 2;
  while (t->cap < 2ull * max_ids) t->cap <<= 1;
  t->arena_cap = arena_bytes;
  int rc;
  if ((rc = rsf::dmalloc((void**)&t->key, (size_t)t->cap * 8)) || (rc = rsf::dmalloc((void**)&t->sid, (size_t)t->cap * 4)) ||
      (rc = rsf::dmalloc((void**)&t->slen, (size_t)t->cap * 4)) ||
      (rc = rsf::dmalloc((void**)&t->soff, (size_t)t->cap * 8)) || (rc = rsf::dmalloc((void**)&t->arena, arena_bytes))) {
    rsf_interner_destroy(t);
    return rc;
  }
  if (hipMemset(t->key, 0, (size_t)t->cap * 8) != hipSuccess) {
    rsf_interner_destroy(t);
    return rsf::set_error(RSF_ERR_HIP, "hipMemset failed");
  }
  *out = t;
  return RSF_OK;
}

int rsf_interner_destroy(rsf_interner* t) {
  if (!t) return RSF_OK;
  hipSetDevice(t->device);
  for (void* p : {(void*)t->key, (void*)t->sid, (void*)t->slen, (void*)t->soff, (void*)t->arena})
    if (p) hipFree(p);
  delete t;
  return RSF_OK;
}

int rsf_interner_count(const rsf_interner* t, uint32_t* n_ids, uint64_t* arena_used) {
  if (!t) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (n_ids) *n_ids = t->n_ids;
  if (arena_used) *arena_used = t->arena_used;
  return RSF_OK;
}

}  // extern "C"

namespace {
// One batch through an interner in two steps, so that a caller interning into several
// tables can check every capacity before committing any (rsf_wire_event_keys).
// plan: hashes, sort, equal-bytes runs, lookups of the existing table, the new ids' ranks
// and arena offsets -> n_new, bytes_new.  commit: insert and write the ids.
struct InternPlan {
  rsf_interner* t = nullptr;
  const uint8_t* buf = nullptr;
  const uint64_t* off = nullptr;
  const uint32_t* len = nullptr;
  uint64_t n = 0;
  hipStream_t st = nullptr;
  void* mem = nullptr;  // scratch (hipMallocAsync on st), freed by ~InternPlan
  uint64_t *h = nullptr, *h_s = nullptr, *new_len = nullptr, *aoff = nullptr;
  uint32_t *idx = nullptr, *idx_s = nullptr, *rep = nullptr, *found = nullptr, *is_new = nullptr, *rank = nullptr,
           *head = nullptr, *run_start = nullptr;
  uint64_t n_new = 0, bytes_new = 0;
  ~InternPlan() {
    if (mem) hipFreeAsync(mem, st);
  }
};

int intern_plan(InternPlan& P) {
  const uint64_t n = P.n;
  hipStream_t st = P.st;
  rsf_interner* t = P.t;
  const int ni = (int)n;
  size_t t_sort = 0, t_scan4 = 0, t_scan8 = 0, t_max = 0;
  // every hipCUB call below is sized here for its own types and count; the temporary
  // storage is the largest of them
  RSF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, P.h, P.h_s, P.idx, P.idx_s, ni, 0, 64, st));
  RSF_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan4, P.is_new, P.rank, ni, st));
  RSF_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan8, P.new_len, P.aoff, ni, st));
  RSF_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, t_max, P.head, P.run_start, hipcub::Max(), ni, st));
  const size_t tmp = std::max(std::max(t_sort, t_max), std::max(t_scan4, t_scan8));
  const size_t n8 = ((size_t)n * 8 + 255) & ~(size_t)255, n4 = ((size_t)n * 4 + 255) & ~(size_t)255;
  RSF_HIP(hipMallocAsync(&P.mem, 4 * n8 + 8 * n4 + ((tmp + 255) & ~(size_t)255), st));
  char* b = (char*)P.mem;
  auto take8 = [&](uint64_t** pp) { *pp = (uint64_t*)b; b += n8; };
  auto take4 = [&](uint32_t** pp) { *pp = (uint32_t*)b; b += n4; };
  take8(&P.h); take8(&P.h_s); take8(&P.new_len); take8(&P.aoff);
  take4(&P.idx); take4(&P.idx_s); take4(&P.rep); take4(&P.found); take4(&P.is_new); take4(&P.rank); take4(&P.head);
  take4(&P.run_start);
  void* tp = b;
  const unsigned g = grid1(n);
  hipLaunchKernelGGL(in_hash_kernel, dim3(g), dim3(256), 0, st, P.buf, P.off, P.len, n, P.h, P.idx);
  size_t tb = tmp;
  RSF_HIP(hipcub::DeviceRadixSort::SortPairs(tp, tb, P.h, P.h_s, P.idx, P.idx_s, ni, 0, 64, st));
  hipLaunchKernelGGL(in_heads_kernel, dim3(g), dim3(256), 0, st, P.h_s, n, P.head);
  tb = tmp;
  RSF_HIP(hipcub::DeviceScan::InclusiveScan(tp, tb, P.head, P.run_start, hipcub::Max(), ni, st));
  RSF_HIP(hipMemsetAsync(P.is_new, 0, (size_t)n * 4, st));
  RSF_HIP(hipMemsetAsync(P.new_len, 0, (size_t)n * 8, st));
  hipLaunchKernelGGL(in_group_kernel, dim3(g), dim3(256), 0, st, P.buf, P.off, P.len, P.h_s, P.idx_s, P.run_start, n,
                     *t, P.rep, P.found, P.is_new, P.new_len);
  tb = tmp;
  RSF_HIP(hipcub::DeviceScan::ExclusiveSum(tp, tb, P.is_new, P.rank, ni, st));
  tb = tmp;
  RSF_HIP(hipcub::DeviceScan::ExclusiveSum(tp, tb, P.new_len, P.aoff, ni, st));
  // totals: last rank + last flag, last offset + last length
  uint32_t last[2];
  uint64_t lastb[2];
  RSF_HIP(hipMemcpyAsync(&last[0], P.rank + n - 1, 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(&last[1], P.is_new + n - 1, 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(&lastb[0], P.aoff + n - 1, 8, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(&lastb[1], P.new_len + n - 1, 8, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  P.n_new = (uint64_t)last[0] + last[1];
  P.bytes_new = lastb[0] + lastb[1];
  return RSF_OK;
}

bool intern_fits(const InternPlan& P) {
  return P.t->n_ids + P.n_new <= P.t->max_ids && P.t->arena_used + P.bytes_new <= P.t->arena_cap;
}

int intern_commit(InternPlan& P, uint32_t* ids) {
  rsf_interner* t = P.t;
  const unsigned g = grid1(P.n);
  hipLaunchKernelGGL(in_insert_kernel, dim3(g), dim3(256), 0, P.st, P.buf, P.off, P.len, P.h_s, P.idx_s, P.rep, P.n,
                     *t, P.rank, P.aoff, P.found);
  hipLaunchKernelGGL(in_ids_kernel, dim3(g), dim3(256), 0, P.st, P.idx_s, P.rep, P.found, P.n, ids);
  RSF_HIP(hipGetLastError());
  t->n_ids += (uint32_t)P.n_new;
  t->arena_used += P.bytes_new;
  return RSF_OK;
}
}  // namespace

extern "C" {

int rsf_intern(rsf_interner* t, const uint8_t* buf, const uint64_t* off, const uint32_t* len, uint64_t n,
               uint32_t* ids, void* stream) {
  if (!t || (n && (!buf || !off || !len || !ids))) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (n == 0) return RSF_OK;
  if (n >= 0x7FFFFFFFull) return rsf::set_error(RSF_ERR_ARG, "batch too large");
  RSF_HIP(hipSetDevice(t->device));
  InternPlan P;
  P.t = t, P.buf = buf, P.off = off, P.len = len, P.n = n, P.st = (hipStream_t)stream;
  int rc = intern_plan(P);
  if (rc) return rc;
  if (!intern_fits(P)) return rsf::set_error(RSF_ERR_OVERFLOW, "interner full (max_ids or arena bytes)");
  return intern_commit(P, ids);
}

// Both interners are planned before either is committed: a batch that would overflow
// either one fails with neither table changed.
int rsf_wire_event_keys(rsf_interner* names, rsf_interner* payloads, const uint8_t* buf, const rsf_wire_msg* msgs,
                        uint64_t n, uint64_t* keys, void* stream) {
  if (!names || !payloads || (n && (!buf || !msgs || !keys))) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (n == 0) return RSF_OK;
  if (n >= 0x7FFFFFFFull) return rsf::set_error(RSF_ERR_ARG, "batch too large");
  if (names == payloads) return rsf::set_error(RSF_ERR_ARG, "names and payloads need separate interners");
  hipStream_t st = (hipStream_t)stream;
  const size_t n8 = ((size_t)n * 8 + 255) & ~(size_t)255, n4 = ((size_t)n * 4 + 255) & ~(size_t)255;
  Scratch sc(st);
  RSF_HIP(hipMallocAsync(&sc.p, 2 * n8 + 4 * n4, st));
  char* b = (char*)sc.p;
  uint64_t* noff = (uint64_t*)b;
  uint64_t* poff = (uint64_t*)(b + n8);
  uint32_t* nlen = (uint32_t*)(b + 2 * n8);
  uint32_t* plen = (uint32_t*)(b + 2 * n8 + n4);
  uint32_t* nid = (uint32_t*)(b + 2 * n8 + 2 * n4);
  uint32_t* pid = (uint32_t*)(b + 2 * n8 + 3 * n4);
  hipLaunchKernelGGL(in_wire_kernel, dim3(grid1(n)), dim3(256), 0, st, msgs, n, noff, nlen, poff, plen);
  RSF_HIP(hipGetLastError());
  InternPlan pn, pp;
  pn.t = names, pn.buf = buf, pn.off = noff, pn.len = nlen, pn.n = n, pn.st = st;
  pp.t = payloads, pp.buf = buf, pp.off = poff, pp.len = plen, pp.n = n, pp.st = st;
  int rc;
  if ((rc = intern_plan(pn)) || (rc = intern_plan(pp))) return rc;
  if (!intern_fits(pn) || !intern_fits(pp))
    return rsf::set_error(RSF_ERR_OVERFLOW, "interner full (max_ids or arena bytes); neither table changed");
  if ((rc = intern_commit(pn, nid)) || (rc = intern_commit(pp, pid))) return rc;
  hipLaunchKernelGGL(in_keys_kernel, dim3(grid1(n)), dim3(256), 0, st, msgs, nid, pid, n, keys);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

}  // extern "C"
