// coalesce.hip — UserEventCoalescer (core/src/coalesce/user.rs:52-97) for many
// coalescers at once (one per member's event stream), as sorts and scans.
//
// Per coalescer the reference keeps an IndexMap name -> (latest ltime, events):
// an event with a larger ltime clears the name's list, an equal ltime appends,
// an older one is dropped; flush drains names in first-insertion order.  So an
// event survives iff its ltime equals its name's final maximum, and the flush
// order is (name's first arrival, arrival).  On the GPU:
//   1. stable radix sort of (group, name) keys, arrival index as value
//   2. segment heads -> segment ids (scan), segmented max of ltime, first arrival
//   3. survivors keyed (group, first arrival of their name), stable sort, gather.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <new>

#include "../../include/ruserf_amd.h"
#include "rsf_internal.h"

namespace {

inline unsigned grid1(uint64_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }

__global__ void ce_keys_kernel(const rsf_user_event* __restrict__ in, uint64_t n, uint64_t* __restrict__ key,
                               uint32_t* __restrict__ idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = ((uint64_t)in[i].group << 32) | in[i].name;
  idx[i] = (uint32_t)i;
}

// head flags (as u32 for the scan) and the ltimes in sorted order
__global__ void ce_heads_kernel(const rsf_user_event* __restrict__ in, const uint64_t* __restrict__ key,
                                const uint32_t* __restrict__ idx, uint64_t n, uint32_t* __restrict__ head,
                                uint64_t* __restrict__ lt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  head[i] = (i == 0 || key[i] != key[i - 1]) ? 1u : 0u;
  lt[i] = in[idx[i]].ltime;
}

// seg[i] = inclusive scan of heads (1-based segment id); per segment: start index
__global__ void ce_starts_kernel(const uint32_t* __restrict__ head, const uint32_t* __restrict__ seg, uint64_t n,
                                 uint32_t* __restrict__ start) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (head[i]) start[seg[i] - 1] = (uint32_t)i;
}

// per segment: max ltime (a serial walk per segment would be unbounded; this is
// an atomic max over the segment's elements instead)
__global__ void ce_segmax_kernel(const uint32_t* __restrict__ seg, const uint64_t* __restrict__ lt, uint64_t n,
                                 unsigned long long* __restrict__ segmax) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = seg[i] - 1;
  // most segments are runs of one: skip the atomic unless a neighbour shares the segment
  const bool alone = (i == 0 || seg[i - 1] != seg[i]) && (i + 1 == n || seg[i + 1] != seg[i]);
  if (alone) segmax[s] = lt[i];
  else atomicMax(&segmax[s], (unsigned long long)lt[i]);
}

// survivors: key2 = (group, first arrival of the name), value = arrival index
__global__ void ce_survivors_kernel(const uint64_t* __restrict__ key, const uint32_t* __restrict__ idx,
                                    const uint32_t* __restrict__ seg, const uint32_t* __restrict__ start,
                                    const uint64_t* __restrict__ lt, const unsigned long long* __restrict__ segmax,
                                    uint64_t n, uint64_t* __restrict__ key2, uint32_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = seg[i] - 1;
  flag[i] = lt[i] == (uint64_t)segmax[s] ? 1u : 0u;
  key2[i] = (key[i] & 0xFFFFFFFF00000000ull) | idx[start[s]];  // stable sort: the segment's first = first arrival
}

__global__ void ce_gather_kernel(const rsf_user_event* __restrict__ in, const uint32_t* __restrict__ order,
                                 uint64_t n, rsf_user_event* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = in[order[i]];
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

extern "C" int rsf_coalesce_user_events(const rsf_user_event* in, uint64_t n, rsf_user_event* out, uint64_t* n_out,
                                        void* stream) {
  if (!n_out || (n && (!in || !out))) return rsf::set_error(RSF_ERR_ARG, "null argument");
  *n_out = 0;
  if (n == 0) return RSF_OK;
  if (n >= 0x7FFFFFFFull) return rsf::set_error(RSF_ERR_ARG, "batch too large");
  hipStream_t st = (hipStream_t)stream;
  const int ni = (int)n;
  // buffers: key/key_s/key2/key2_s/lt/segmax u64 x6, idx/idx_s/head/seg/start/flag/sel_v/ord u32 x8
  uint64_t *key = nullptr, *key_s = nullptr, *key2 = nullptr, *key2_s = nullptr, *lt = nullptr;
  uint32_t *idx = nullptr, *idx_s = nullptr, *head = nullptr, *seg = nullptr, *start = nullptr, *flag = nullptr,
           *sel_v = nullptr, *ord = nullptr;
  unsigned long long* segmax = nullptr;
  const size_t n8 = ((size_t)n * 8 + 255) & ~(size_t)255, n4 = ((size_t)n * 4 + 255) & ~(size_t)255;
  Scratch sc(st);
  RSF_HIP(hipMallocAsync(&sc.p, 6 * n8 + 8 * n4 + 256, st));
  char* b = (char*)sc.p;
  auto take8 = [&](void* pp) { *(char**)pp = b; b += n8; };
  auto take4 = [&](void* pp) { *(char**)pp = b; b += n4; };
  take8(&key); take8(&key_s); take8(&key2); take8(&key2_s); take8(&lt); take8(&segmax);
  take4(&idx); take4(&idx_s); take4(&head); take4(&seg); take4(&start); take4(&flag); take4(&sel_v); take4(&ord);
  int* d_nsel = (int*)b;
  uint64_t* sel_k = key2_s;  // the selected survivor keys land here, then sort back into key2
  // every hipCUB call sized for its own item count and types (rsf::cub_run)
  rsf::CubTemp tmp;
  struct Free {
    rsf::CubTemp& t;
    ~Free() { t.release(); }
  } free_tmp{tmp};
  const unsigned g = grid1(n);
  hipLaunchKernelGGL(ce_keys_kernel, dim3(g), dim3(256), 0, st, in, n, key, idx);
  int rc = rsf::cub_run(
      tmp, st,
      [&](void* t, size_t& bytes) { return hipcub::DeviceRadixSort::SortPairs(t, bytes, key, key_s, idx, idx_s, ni, 0, 64, st); },
      "user event sort");
  if (rc) return rc;
  hipLaunchKernelGGL(ce_heads_kernel, dim3(g), dim3(256), 0, st, in, key_s, idx_s, n, head, lt);
  rc = rsf::cub_run(
      tmp, st, [&](void* t, size_t& bytes) { return hipcub::DeviceScan::InclusiveSum(t, bytes, head, seg, ni, st); },
      "user event segment scan");
  if (rc) return rc;
  RSF_HIP(hipMemsetAsync(segmax, 0, (size_t)n * 8, st));
  hipLaunchKernelGGL(ce_starts_kernel, dim3(g), dim3(256), 0, st, head, seg, n, start);
  hipLaunchKernelGGL(ce_segmax_kernel, dim3(g), dim3(256), 0, st, seg, lt, n, segmax);
  hipLaunchKernelGGL(ce_survivors_kernel, dim3(g), dim3(256), 0, st, key_s, idx_s, seg, start, lt, segmax, n, key2,
                     flag);
  RSF_HIP(hipGetLastError());
  rc = rsf::cub_run(
      tmp, st,
      [&](void* t, size_t& bytes) { return hipcub::DeviceSelect::Flagged(t, bytes, key2, flag, sel_k, d_nsel, ni, st); },
      "user event survivor keys");
  if (rc) return rc;
  rc = rsf::cub_run(
      tmp, st,
      [&](void* t, size_t& bytes) { return hipcub::DeviceSelect::Flagged(t, bytes, idx_s, flag, sel_v, d_nsel, ni, st); },
      "user event survivor indices");
  if (rc) return rc;
  int nsel = 0;
  RSF_HIP(hipMemcpyAsync(&nsel, d_nsel, sizeof(int), hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  if (nsel > 0) {
    rc = rsf::cub_run(
        tmp, st,
        [&](void* t, size_t& bytes) {
          return hipcub::DeviceRadixSort::SortPairs(t, bytes, sel_k, key2, sel_v, ord, nsel, 0, 64, st);
        },
        "user event output sort");
    if (rc) return rc;
    hipLaunchKernelGGL(ce_gather_kernel, dim3(grid1((uint64_t)nsel)), dim3(256), 0, st, in, ord, (uint64_t)nsel, out);
    RSF_HIP(hipGetLastError());
    RSF_HIP(hipStreamSynchronize(st));
  }
  *n_out = (uint64_t)nsel;
  return RSF_OK;
}

// ---- MemberEventCoalescer (core/src/coalesce/member.rs:60-118) ------------------------
// coalesce(): latest_events.insert(node, ev) in arrival order, so per (group, node) the
// last arrival wins; flush(): a node whose type equals last_events[node] is skipped
// unless it is an Update, otherwise last_events[node] = type and the member goes out in
// its type's event.  On the GPU: stable radix sort of (group, node) keys with the arrival
// index as value; the last element of each run is the latest event; one thread per run
// checks and updates last_events (each (group, node) has one run, so no races); the
// flushed events are selected and sorted by (group, type, node).
struct rsf_member_coalescer {
  int device = 0;
  uint32_t n_groups = 0, n_nodes = 0;
  uint8_t* last = nullptr;  // [n_groups][n_nodes], 0xFF = none
};

namespace {
constexpr uint8_t kNoEvent = 0xFF;
constexpr uint32_t kMevUpdate = RSF_MEMBER_EVENT_UPDATE;

__global__ void mc_keys_kernel(const rsf_member_event* __restrict__ in, uint64_t n, uint32_t n_groups,
                               uint32_t n_nodes, uint64_t* __restrict__ key, uint32_t* __restrict__ idx,
                               unsigned int* __restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const rsf_member_event e = in[i];
  if (e.group >= n_groups || e.node >= n_nodes || e.type > kMevUpdate) atomicOr(bad, 1u);
  key[i] = ((uint64_t)e.group << 32) | e.node;
  idx[i] = (uint32_t)i;
}

// the last arrival of each (group, node) run against last_events; flushed events keyed
// (group << 35 | type << 32 | node) for the output order
__global__ void mc_flush_kernel(const rsf_member_event* __restrict__ in, const uint64_t* __restrict__ key,
                                const uint32_t* __restrict__ idx, uint64_t n, uint32_t n_nodes,
                                const uint8_t* __restrict__ last, uint64_t* __restrict__ okey, uint32_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool latest = i + 1 == n || key[i + 1] != key[i];
  uint32_t f = 0;
  if (latest) {
    const rsf_member_event e = in[idx[i]];
    const uint8_t* lp = last + (uint64_t)e.group * n_nodes + e.node;
    const uint8_t prev = *lp;
    if (!(prev == e.type && e.type != kMevUpdate)) f = 1;  // recorded by mc_commit_kernel
    okey[i] = ((uint64_t)e.group << 35) | ((uint64_t)e.type << 32) | e.node;
  }
  flag[i] = f;
}

// last_events[node] = type for the flushed events, once every step of the flush has succeeded
// (a failed call leaves the table as it was, so the quantum can be flushed again)
__global__ void mc_commit_kernel(const rsf_member_event* __restrict__ in, const uint32_t* __restrict__ idx,
                                 const uint32_t* __restrict__ flag, uint64_t n, uint32_t n_nodes,
                                 uint8_t* __restrict__ last) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !flag[i]) return;
  const rsf_member_event e = in[idx[i]];
  last[(uint64_t)e.group * n_nodes + e.node] = (uint8_t)e.type;
}

__global__ void mc_gather_kernel(const rsf_member_event* __restrict__ in, const uint32_t* __restrict__ order,
                                 uint64_t n, rsf_member_event* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = in[order[i]];
}
}  // namespace

extern "C" int rsf_member_coalescer_create(rsf_member_coalescer** out, uint32_t n_groups, uint32_t n_nodes,
                                           int device) {
  if (!out) return rsf::set_error(RSF_ERR_ARG, "null argument");
  *out = nullptr;
  if (n_groups == 0 || n_nodes == 0 || n_groups >= (1u << 29))
    return rsf::set_error(RSF_ERR_ARG, "n_groups must be in [1, 2^29), n_nodes >= 1");
  RSF_HIP(hipSetDevice(device));
  rsf_member_coalescer* mc = new (std::nothrow) rsf_member_coalescer();
  if (!mc) return rsf::set_error(RSF_ERR_NOMEM, "host allocation failed");
  mc->device = device;
  mc->n_groups = n_groups;
  mc->n_nodes = n_nodes;
  const size_t bytes = (size_t)n_groups * n_nodes;
  int rc = rsf::dmalloc((void**)&mc->last, bytes);
  if (rc || hipMemset(mc->last, kNoEvent, bytes) != hipSuccess) {
    rsf_member_coalescer_destroy(mc);
    return rc ? rc : rsf::set_error(RSF_ERR_HIP, "hipMemset failed");
  }
  *out = mc;
  return RSF_OK;
}

extern "C" int rsf_member_coalescer_destroy(rsf_member_coalescer* mc) {
  if (!mc) return RSF_OK;
  hipSetDevice(mc->device);
  if (mc->last) hipFree(mc->last);
  delete mc;
  return RSF_OK;
}

extern "C" int rsf_member_coalescer_dump(rsf_member_coalescer* mc, uint8_t* last_out) {
  if (!mc || !last_out) return rsf::set_error(RSF_ERR_ARG, "null argument");
  RSF_HIP(hipSetDevice(mc->device));
  RSF_HIP(hipMemcpy(last_out, mc->last, (size_t)mc->n_groups * mc->n_nodes, hipMemcpyDeviceToHost));
  return RSF_OK;
}

extern "C" int rsf_member_coalescer_flush(rsf_member_coalescer* mc, const rsf_member_event* in, uint64_t n,
                                          rsf_member_event* out, uint64_t* n_out, void* stream) {
  if (!mc || !n_out || (n && (!in || !out))) return rsf::set_error(RSF_ERR_ARG, "null argument");
  *n_out = 0;
  if (n == 0) return RSF_OK;
  if (n >= 0x7FFFFFFFull) return rsf::set_error(RSF_ERR_ARG, "batch too large");
  RSF_HIP(hipSetDevice(mc->device));
  hipStream_t st = (hipStream_t)stream;
  const int ni = (int)n;
  const size_t n8 = ((size_t)n * 8 + 255) & ~(size_t)255, n4 = ((size_t)n * 4 + 255) & ~(size_t)255;
  Scratch sc(st);
  RSF_HIP(hipMallocAsync(&sc.p, 4 * n8 + 4 * n4 + 256, st));
  char* b = (char*)sc.p;
  uint64_t *key = (uint64_t*)b, *key_s = (uint64_t*)(b + n8), *okey = (uint64_t*)(b + 2 * n8),
           *okey_s = (uint64_t*)(b + 3 * n8);
  uint32_t *idx = (uint32_t*)(b + 4 * n8), *idx_s = (uint32_t*)(b + 4 * n8 + n4), *flag = (uint32_t*)(b + 4 * n8 + 2 * n4);
  uint32_t* ord = (uint32_t*)(b + 4 * n8 + 3 * n4);  // the output order (flag stays intact for the commit)
  unsigned int* dv = (unsigned int*)(b + 4 * n8 + 4 * n4);  // [0] bad input, [1] selected count
  RSF_HIP(hipMemsetAsync(dv, 0, 8, st));
  const unsigned g = grid1(n);
  hipLaunchKernelGGL(mc_keys_kernel, dim3(g), dim3(256), 0, st, in, n, mc->n_groups, mc->n_nodes, key, idx, dv);
  RSF_HIP(hipGetLastError());
  unsigned int bad = 0;
  RSF_HIP(hipMemcpyAsync(&bad, dv, 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  if (bad) return rsf::set_error(RSF_ERR_ARG, "member event outside the group / node / type ranges");
  rsf::CubTemp tmp;
  struct Free {
    rsf::CubTemp& t;
    ~Free() { t.release(); }
  } free_tmp{tmp};
  int rc = rsf::cub_run(
      tmp, st,
      [&](void* t, size_t& bytes) { return hipcub::DeviceRadixSort::SortPairs(t, bytes, key, key_s, idx, idx_s, ni, 0, 64, st); },
      "member event sort");
  if (rc) return rc;
  hipLaunchKernelGGL(mc_flush_kernel, dim3(g), dim3(256), 0, st, in, key_s, idx_s, n, mc->n_nodes, mc->last, okey,
                     flag);
  RSF_HIP(hipGetLastError());
  // the flushed events' output keys (into `key`) and arrival indices (into `idx`), then
  // sorted by key with the index riding along, then gathered: the latest event's member
  // (its payload word) is the one sent, as latest_events keeps the last CoalesceEvent
  int* nsel_d = (int*)(dv + 1);
  rc = rsf::cub_run(
      tmp, st,
      [&](void* t, size_t& bytes) { return hipcub::DeviceSelect::Flagged(t, bytes, okey, flag, key, nsel_d, ni, st); },
      "member event select");
  if (rc) return rc;
  rc = rsf::cub_run(
      tmp, st,
      [&](void* t, size_t& bytes) { return hipcub::DeviceSelect::Flagged(t, bytes, idx_s, flag, idx, nsel_d, ni, st); },
      "member event select");
  if (rc) return rc;
  int nsel = 0;
  RSF_HIP(hipMemcpyAsync(&nsel, nsel_d, 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  if (nsel > 0) {
    rc = rsf::cub_run(
        tmp, st,
        [&](void* t, size_t& bytes) {
          return hipcub::DeviceRadixSort::SortPairs(t, bytes, key, okey_s, idx, ord, nsel, 0, 64, st);
        },
        "member event output sort");
    if (rc) return rc;
    hipLaunchKernelGGL(mc_gather_kernel, dim3(grid1((uint64_t)nsel)), dim3(256), 0, st, in, (const uint32_t*)ord,
                       (uint64_t)nsel, out);
    RSF_HIP(hipGetLastError());
    hipLaunchKernelGGL(mc_commit_kernel, dim3(g), dim3(256), 0, st, in, idx_s, flag, n, mc->n_nodes, mc->last);
    RSF_HIP(hipGetLastError());
    RSF_HIP(hipStreamSynchronize(st));
  }
  *n_out = (uint64_t)nsel;
  return RSF_OK;
}
