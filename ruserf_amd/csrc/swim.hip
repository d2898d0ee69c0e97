// swim.hip — memberlist's failure-detector state machine for many members at once
// (SURVEY §8(f)3, row M9): the incarnation merge of alive / suspect / dead messages,
// self-refutation and the suspicion timers, batched over (receiver, subject) entries.
//
// The reference does not vendor memberlist (memberlist-core 0.2; serf reaches it from
// core/src/serf/base.rs:208-225 and the delegate hooks in delegate.rs): PARITY UNPINNED.
// The rules restate memberlist's published state machine (aliveNode, suspectNode,
// deadNode, refute, suspicion.Confirm); oracle/oracle.c holds the same restatement.
//
// Layout: one 32-B entry per (receiver, subject), row-major [n_loc][S]; a receiver's
// messages are stably sorted by receiver, then one thread per receiver applies its
// messages in order (messages of different receivers touch disjoint rows).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <vector>

#include "../../include/ruserf_amd.h"
#include "rsf_internal.h"

namespace {

inline unsigned grid1(uint64_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }

constexpr uint32_t kK = RSF_SWIM_MAX_CONFIRM;

// nodeState + its suspicion timer (conf[0] = the first accuser, conf[1..n] = confirmations)
struct SwimE {
  uint32_t inc, change;
  uint8_t state, nconf, _p0, _p1;
  uint32_t conf[kK + 1];
};
static_assert(sizeof(SwimE) == 32, "entry is 32 B");

struct SwimDev {
  SwimE* view;          // [n_loc][S]
  uint32_t* self_inc;   // [n_loc] m.incarnation
  uint8_t* left;        // [n_loc] m.hasLeft()
  uint32_t* subj_member;// [S]
};

struct SwimCfg {
  uint64_t lo, n_loc;
  uint32_t S, k;
  uint32_t timeout[kK + 1];
};

// refute(me, accusedInc): nextIncarnation, then skip past the accusation
__device__ __forceinline__ uint32_t sw_refute(SwimE& e, uint32_t& self_inc, uint32_t accused) {
  uint32_t inc = self_inc + 1;
  if (accused >= inc) inc = accused + 1;
  self_inc = inc;
  e.inc = inc;
  return inc;
}

__device__ __forceinline__ void sw_clear_timer(SwimE& e) { e.nconf = 0; }

// aliveNode (bootstrap = false; the model carries no meta, so an equal-incarnation
// alive about ourselves is always the "same values" case)
__device__ __forceinline__ int sw_alive(SwimE& e, bool local, uint32_t& self_inc, uint32_t inc, uint32_t now,
                                        uint32_t& ref) {
  if (e.state == RSF_SWIM_UNKNOWN) {  // new node: added to nodeMap as dead, incarnation 0
    e.state = RSF_SWIM_DEAD;
    e.inc = 0;
    e.change = 0;
    e.nconf = 0;
  }
  if (inc <= e.inc && !local) return 0;
  if (inc < e.inc && local) return 0;
  sw_clear_timer(e);
  const uint8_t old = e.state;
  int f = 0;
  if (local) {
    if (inc == e.inc) return 0;
    ref = sw_refute(e, self_inc, inc);
    f |= RSF_SWIM_F_REFUTE;
  } else {
    f |= RSF_SWIM_F_REBROADCAST;
    e.inc = inc;
    if (e.state != RSF_SWIM_ALIVE) {
      e.state = RSF_SWIM_ALIVE;
      e.change = now;
    }
  }
  if (old == RSF_SWIM_DEAD || old == RSF_SWIM_LEFT) f |= RSF_SWIM_F_NOTIFY_JOIN;
  return f;
}

// suspectNode
__device__ __forceinline__ int sw_suspect(SwimE& e, bool local, uint32_t& self_inc, uint32_t inc, uint32_t from,
                                          uint32_t k, uint32_t now, uint32_t& ref) {
  if (e.state == RSF_SWIM_UNKNOWN) return 0;
  if (inc < e.inc) return 0;
  if (e.state == RSF_SWIM_SUSPECT) {  // a running timer: suspicion.Confirm(from)
    if (e.nconf >= k) return 0;
    for (uint32_t i = 0; i <= e.nconf; ++i)
      if (e.conf[i] == from) return 0;
    e.conf[++e.nconf] = from;
    return RSF_SWIM_F_REBROADCAST | RSF_SWIM_F_CONFIRM;
  }
  if (e.state != RSF_SWIM_ALIVE) return 0;
  if (local) {
    ref = sw_refute(e, self_inc, inc);
    return RSF_SWIM_F_REFUTE;
  }
  e.inc = inc;
  e.state = RSF_SWIM_SUSPECT;
  e.change = now;
  e.conf[0] = from;
  e.nconf = 0;
  return RSF_SWIM_F_REBROADCAST | RSF_SWIM_F_SUSPECT;
}

// deadNode
__device__ __forceinline__ int sw_dead(SwimE& e, bool local, bool has_left, uint32_t& self_inc, uint32_t inc,
                                       bool from_self_node, uint32_t now, uint32_t& ref) {
  if (e.state == RSF_SWIM_UNKNOWN) return 0;
  if (inc < e.inc) return 0;
  sw_clear_timer(e);
  if (e.state == RSF_SWIM_DEAD || e.state == RSF_SWIM_LEFT) return 0;
  if (local && !has_left) {
    ref = sw_refute(e, self_inc, inc);
    return RSF_SWIM_F_REFUTE;
  }
  e.inc = inc;
  e.state = from_self_node ? RSF_SWIM_LEFT : RSF_SWIM_DEAD;
  e.change = now;
  return RSF_SWIM_F_REBROADCAST | RSF_SWIM_F_NOTIFY_LEAVE;
}

__global__ void sw_keys_kernel(const rsf_swim_msg* __restrict__ m, uint64_t n, uint64_t lo, uint32_t* __restrict__ key,
                               uint32_t* __restrict__ idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = (uint32_t)(m[i].receiver - lo);
  idx[i] = (uint32_t)i;
}

__global__ void sw_segment_kernel(const uint32_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ seg_start,
                                  uint32_t* __restrict__ seg_end) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = key[i];
  if (i == 0 || key[i - 1] != k) seg_start[k] = (uint32_t)i;
  if (i + 1 == n || key[i + 1] != k) seg_end[k] = (uint32_t)(i + 1);
}

// one thread per receiver, its messages in (stable) array order
__global__ void __launch_bounds__(256) sw_apply_kernel(SwimCfg c, SwimDev d, const rsf_swim_msg* __restrict__ m,
                                                       const uint32_t* __restrict__ idx,
                                                       const uint32_t* __restrict__ seg_start,
                                                       const uint32_t* __restrict__ seg_end, uint32_t now,
                                                       int32_t* __restrict__ flags, uint32_t* __restrict__ ref_out) {
  const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= c.n_loc) return;
  const uint32_t b = seg_start[l], e_ = seg_end[l];
  if (b >= e_) return;
  const uint32_t me = (uint32_t)(c.lo + l);
  uint32_t self_inc = d.self_inc[l];
  const bool has_left = d.left[l] != 0;
  SwimE* row = d.view + l * c.S;
  for (uint32_t j = b; j < e_; ++j) {
    const uint32_t i = idx[j];
    const rsf_swim_msg msg = m[i];
    SwimE e = row[msg.subject];
    const uint32_t node = d.subj_member[msg.subject];
    const bool local = node == me;
    uint32_t ref = 0;
    int f = 0;
    if (msg.type == RSF_SWIM_MSG_ALIVE) f = sw_alive(e, local, self_inc, msg.incarnation, now, ref);
    else if (msg.type == RSF_SWIM_MSG_SUSPECT) f = sw_suspect(e, local, self_inc, msg.incarnation, msg.from, c.k, now, ref);
    else if (msg.type == RSF_SWIM_MSG_DEAD)
      f = sw_dead(e, local, has_left, self_inc, msg.incarnation, node == msg.from, now, ref);
    row[msg.subject] = e;
    flags[i] = f;
    ref_out[i] = ref;
  }
  d.self_inc[l] = self_inc;
}

// suspicion timers: one thread per entry; a due timer runs deadNode{inc, from = receiver}
__global__ void __launch_bounds__(256) sw_tick_kernel(SwimCfg c, SwimDev d, uint32_t now,
                                                      unsigned long long* __restrict__ fired) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= c.n_loc * c.S) return;
  SwimE e = d.view[t];
  if (e.state != RSF_SWIM_SUSPECT) return;
  const uint32_t nconf = e.nconf <= c.k ? e.nconf : c.k;
  if (now - e.change < c.timeout[nconf]) return;
  const uint64_t l = t / c.S;
  const uint32_t me = (uint32_t)(c.lo + l), node = d.subj_member[t - l * c.S];
  uint32_t self_inc = d.self_inc[l], ref = 0;
  // suspectNode refutes instead of suspecting ourselves, but an entry about ourselves can
  // start out suspect (rsf_swim_init): its timer then refutes.  One subject per member,
  // so at most one thread per receiver writes self_inc.
  const bool local = node == me;
  sw_dead(e, local, d.left[l] != 0, self_inc, e.inc, local, now, ref);
  if (local) d.self_inc[l] = self_inc;
  d.view[t] = e;
  atomicAdd(fired, 1ull);
}

// memberlist probeNode's failure path: a receiver whose probe of `target` got no ack runs
// suspectNode{incarnation = its entry's, node = target, from = itself} (a tracked subject
// only; a dead prober process does not probe).  flags[l] = RSF_SWIM_F_* (0: no suspicion)
__global__ void __launch_bounds__(256) sw_probe_fail_kernel(SwimCfg c, SwimDev d, const int32_t* __restrict__ msubj,
                                                            const uint32_t* __restrict__ target,
                                                            const uint8_t* __restrict__ acked,
                                                            const uint8_t* __restrict__ up, uint32_t now,
                                                            int32_t* __restrict__ flags) {
  const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= c.n_loc) return;
  const uint32_t me = (uint32_t)(c.lo + l), t = target[l];
  int f = 0;
  const int32_t j = msubj[t];
  if (!acked[l] && (!up || up[me]) && t != me && j >= 0) {
    SwimE e = d.view[l * c.S + (uint32_t)j];
    uint32_t self_inc = d.self_inc[l], ref = 0;
    f = sw_suspect(e, false, self_inc, e.inc, me, c.k, now, ref);
    d.view[l * c.S + (uint32_t)j] = e;
  }
  if (flags) flags[l] = f;
}

__global__ void sw_init_kernel(SwimE* __restrict__ view, uint64_t n_loc, uint32_t S, const uint8_t* __restrict__ st,
                               const uint32_t* __restrict__ inc, uint32_t* __restrict__ self_inc, uint32_t self0) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n_loc) self_inc[t] = self0;
  if (t >= n_loc * S) return;
  const uint32_t s = (uint32_t)(t % S);
  SwimE e{};
  e.state = st[s];
  e.inc = inc[s];
  view[t] = e;
}

}  // namespace

struct rsf_swim {
  SwimCfg c{};
  SwimDev d{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  unsigned long long* d_fired = nullptr;
  int32_t* d_msubj = nullptr;  // [N] member id -> subject slot (-1: untracked)
  uint64_t N = 0;
  rsf::DeviceScratch scratch;
};

extern "C" {

int rsf_swim_create(rsf_swim** out, const rsf_swim_cfg* cfg, int device) {
  if (!out || !cfg) return rsf::set_error(RSF_ERR_ARG, "null argument");
  *out = nullptr;
  if (cfg->shard_hi <= cfg->shard_lo || cfg->shard_hi > cfg->n_members || cfg->n_members > 0xFFFFFFFFull ||
      cfg->n_subjects == 0 || cfg->suspicion_k > RSF_SWIM_MAX_CONFIRM ||
      (cfg->shard_hi - cfg->shard_lo) * (uint64_t)cfg->n_subjects > (1ull << 36))
    return rsf::set_error(RSF_ERR_ARG, "bad swim config");
  RSF_HIP(hipSetDevice(device));
  rsf_swim* w = new rsf_swim();
  w->device = device;
  w->N = cfg->n_members;
  w->c.lo = cfg->shard_lo;
  w->c.n_loc = cfg->shard_hi - cfg->shard_lo;
  w->c.S = cfg->n_subjects;
  w->c.k = cfg->suspicion_k;
  for (uint32_t i = 0; i <= kK; ++i) w->c.timeout[i] = cfg->timeout[i];
  int rc = RSF_OK;
  if (!rc) rc = rsf::dmalloc((void**)&w->d.view, w->c.n_loc * w->c.S * sizeof(SwimE));
  if (!rc) rc = rsf::dmalloc((void**)&w->d.self_inc, w->c.n_loc * 4);
  if (!rc) rc = rsf::dmalloc((void**)&w->d.left, w->c.n_loc);
  if (!rc) rc = rsf::dmalloc((void**)&w->d.subj_member, (uint64_t)w->c.S * 4);
  if (!rc) rc = rsf::dmalloc((void**)&w->d_fired, 8);
  if (!rc && hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess)
    rc = rsf::set_error(RSF_ERR_HIP, "hipStreamCreate failed");
  if (rc) {
    rsf_swim_destroy(w);
    return rc;
  }
  w->own_stream = true;
  RSF_HIP(hipMemsetAsync(w->d.view, 0xFF, w->c.n_loc * w->c.S * sizeof(SwimE), w->stream));  // all unknown
  RSF_HIP(hipMemsetAsync(w->d.self_inc, 0, w->c.n_loc * 4, w->stream));
  RSF_HIP(hipMemsetAsync(w->d.left, 0, w->c.n_loc, w->stream));
  RSF_HIP(hipMemsetAsync(w->d.subj_member, 0xFF, (uint64_t)w->c.S * 4, w->stream));
  RSF_HIP(hipStreamSynchronize(w->stream));
  *out = w;
  return RSF_OK;
}

int rsf_swim_destroy(rsf_swim* w) {
  if (!w) return RSF_OK;
  hipSetDevice(w->device);
  if (w->stream) hipStreamSynchronize(w->stream);
  hipFree(w->d.view);
  hipFree(w->d.self_inc);
  hipFree(w->d.left);
  hipFree(w->d.subj_member);
  hipFree(w->d_fired);
  if (w->d_msubj) hipFree(w->d_msubj);
  w->scratch.release();
  if (w->own_stream && w->stream) hipStreamDestroy(w->stream);
  delete w;
  return RSF_OK;
}

int rsf_swim_set_stream(rsf_swim* w, void* s) {
  if (!w) return rsf::set_error(RSF_ERR_ARG, "null context");
  if (w->own_stream && w->stream) {
    hipStreamSynchronize(w->stream);
    hipStreamDestroy(w->stream);
  }
  w->own_stream = s == nullptr;
  if (s) w->stream = (hipStream_t)s;
  else RSF_HIP(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
  return RSF_OK;
}

int rsf_swim_set_subjects(rsf_swim* w, const uint32_t* subject_member) {
  if (!w || !subject_member) return rsf::set_error(RSF_ERR_ARG, "null argument");
  RSF_HIP(hipSetDevice(w->device));
  std::vector<int32_t> msubj(w->N, -1);
  for (uint32_t s = 0; s < w->c.S; ++s) {
    if (subject_member[s] >= w->N) return rsf::set_error(RSF_ERR_ARG, "subject member out of range");
    msubj[subject_member[s]] = (int32_t)s;
  }
  if (!w->d_msubj) {
    int rc = rsf::dmalloc((void**)&w->d_msubj, w->N * 4);
    if (rc) return rc;
  }
  RSF_HIP(hipMemcpyAsync(w->d.subj_member, subject_member, (uint64_t)w->c.S * 4, hipMemcpyHostToDevice, w->stream));
  RSF_HIP(hipMemcpyAsync(w->d_msubj, msubj.data(), w->N * 4, hipMemcpyHostToDevice, w->stream));
  RSF_HIP(hipStreamSynchronize(w->stream));
  return RSF_OK;
}

int rsf_swim_probe_failures(rsf_swim* w, const uint32_t* target, const uint8_t* acked, const uint8_t* up,
                            uint32_t now, int32_t* flags_out) {
  if (!w || !target || !acked) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (!w->d_msubj) return rsf::set_error(RSF_ERR_ARG, "call rsf_swim_set_subjects first");
  RSF_HIP(hipSetDevice(w->device));
  hipLaunchKernelGGL(sw_probe_fail_kernel, dim3(grid1(w->c.n_loc)), dim3(256), 0, w->stream, w->c, w->d,
                     (const int32_t*)w->d_msubj, target, acked, up, now, flags_out);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_swim_init(rsf_swim* w, const uint8_t* state, const uint32_t* incarnation, uint32_t self_incarnation) {
  if (!w || !state || !incarnation) return rsf::set_error(RSF_ERR_ARG, "null argument");
  for (uint32_t s = 0; s < w->c.S; ++s)
    if (state[s] > RSF_SWIM_LEFT && state[s] != RSF_SWIM_UNKNOWN) return rsf::set_error(RSF_ERR_ARG, "bad state");
  RSF_HIP(hipSetDevice(w->device));
  void* p[2];
  const size_t b[2] = {w->c.S, (size_t)w->c.S * 4};
  int rc = w->scratch.take(b, 2, p);
  if (rc) return rc;
  RSF_HIP(hipMemcpyAsync(p[0], state, b[0], hipMemcpyHostToDevice, w->stream));
  RSF_HIP(hipMemcpyAsync(p[1], incarnation, b[1], hipMemcpyHostToDevice, w->stream));
  const uint64_t n = w->c.n_loc * w->c.S;
  hipLaunchKernelGGL(sw_init_kernel, dim3(grid1(n > w->c.n_loc ? n : w->c.n_loc)), dim3(256), 0, w->stream,
                     w->d.view, w->c.n_loc, w->c.S, (const uint8_t*)p[0], (const uint32_t*)p[1], w->d.self_inc,
                     self_incarnation);
  RSF_HIP(hipGetLastError());
  RSF_HIP(hipStreamSynchronize(w->stream));
  return RSF_OK;
}

int rsf_swim_set_left(rsf_swim* w, uint64_t member, uint8_t left) {
  if (!w || member < w->c.lo || member >= w->c.lo + w->c.n_loc) return rsf::set_error(RSF_ERR_ARG, "bad member");
  RSF_HIP(hipSetDevice(w->device));
  RSF_HIP(hipMemcpyAsync(w->d.left + (member - w->c.lo), &left, 1, hipMemcpyHostToDevice, w->stream));
  RSF_HIP(hipStreamSynchronize(w->stream));
  return RSF_OK;
}

int rsf_swim_apply_batch(rsf_swim* w, const rsf_swim_msg* msgs, uint64_t n, uint32_t now, int32_t* flags_out,
                         uint32_t* refute_inc_out) {
  if (!w || (n && (!msgs || !flags_out))) return rsf::set_error(RSF_ERR_ARG, "null argument");
  if (n == 0) return RSF_OK;
  if (n > 0xFFFFFFFFull) return rsf::set_error(RSF_ERR_ARG, "batch too large");
  // host-side shape checks before anything reaches the kernel (indices it trusts)
  for (uint64_t i = 0; i < n; ++i) {
    const rsf_swim_msg& m = msgs[i];
    if (m.receiver < w->c.lo || m.receiver >= w->c.lo + w->c.n_loc || m.subject >= w->c.S ||
        m.type > RSF_SWIM_MSG_DEAD)
      return rsf::set_error(RSF_ERR_ARG, "message outside the shard / subject range / type");
  }
  RSF_HIP(hipSetDevice(w->device));
  hipStream_t st = w->stream;
  // the sort's temporary storage is queried for exactly the call made below (same count and bits)
  int bits = 1;
  while (bits < 32 && (w->c.n_loc >> bits)) ++bits;
  size_t sort_bytes = 0;
  RSF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, bits, st));
  void* p[9];
  const size_t b[9] = {n * sizeof(rsf_swim_msg), n * 4, n * 4, n * 4, n * 4, w->c.n_loc * 4, w->c.n_loc * 4,
                       n * 4, n * 4};
  int rc = w->scratch.take(b, 9, p);
  if (rc) return rc;
  void* tmp = nullptr;
  rc = w->scratch.take_extra(sort_bytes, &tmp);
  if (rc) return rc;
  rsf_swim_msg* dm = (rsf_swim_msg*)p[0];
  uint32_t *key = (uint32_t*)p[1], *idx = (uint32_t*)p[2], *key_s = (uint32_t*)p[3], *idx_s = (uint32_t*)p[4];
  uint32_t *seg_start = (uint32_t*)p[5], *seg_end = (uint32_t*)p[6];
  int32_t* dflags = (int32_t*)p[7];
  uint32_t* dref = (uint32_t*)p[8];
  RSF_HIP(hipMemcpyAsync(dm, msgs, b[0], hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(sw_keys_kernel, dim3(grid1(n)), dim3(256), 0, st, dm, n, w->c.lo, key, idx);
  RSF_HIP(hipGetLastError());
  RSF_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, sort_bytes, key, key_s, idx, idx_s, (int)n, 0, bits, st));
  RSF_HIP(hipMemsetAsync(seg_start, 0, b[5], st));
  RSF_HIP(hipMemsetAsync(seg_end, 0, b[6], st));
  hipLaunchKernelGGL(sw_segment_kernel, dim3(grid1(n)), dim3(256), 0, st, key_s, n, seg_start, seg_end);
  RSF_HIP(hipGetLastError());
  hipLaunchKernelGGL(sw_apply_kernel, dim3(grid1(w->c.n_loc)), dim3(256), 0, st, w->c, w->d, dm, idx_s, seg_start,
                     seg_end, now, dflags, dref);
  RSF_HIP(hipGetLastError());
  RSF_HIP(hipMemcpyAsync(flags_out, dflags, n * 4, hipMemcpyDeviceToHost, st));
  if (refute_inc_out) RSF_HIP(hipMemcpyAsync(refute_inc_out, dref, n * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  return RSF_OK;
}

int rsf_swim_tick(rsf_swim* w, uint32_t now, uint64_t* n_fired) {
  if (!w) return rsf::set_error(RSF_ERR_ARG, "null context");
  RSF_HIP(hipSetDevice(w->device));
  RSF_HIP(hipMemsetAsync(w->d_fired, 0, 8, w->stream));
  hipLaunchKernelGGL(sw_tick_kernel, dim3(grid1(w->c.n_loc * w->c.S)), dim3(256), 0, w->stream, w->c, w->d, now,
                     w->d_fired);
  RSF_HIP(hipGetLastError());
  unsigned long long f = 0;
  RSF_HIP(hipMemcpyAsync(&f, w->d_fired, 8, hipMemcpyDeviceToHost, w->stream));
  RSF_HIP(hipStreamSynchronize(w->stream));
  if (n_fired) *n_fired = f;
  return RSF_OK;
}

int rsf_swim_dump(rsf_swim* w, uint64_t first, uint64_t count, uint8_t* state, uint32_t* incarnation,
                  uint32_t* change, uint8_t* n_confirm, uint32_t* self_incarnation) {
  if (!w || first + count > w->c.n_loc) return rsf::set_error(RSF_ERR_ARG, "bad range");
  RSF_HIP(hipSetDevice(w->device));
  const uint64_t ne = count * w->c.S;
  SwimE* h = (SwimE*)malloc(ne * sizeof(SwimE) + 1);
  if (!h) return rsf::set_error(RSF_ERR_NOMEM, "host buffer");
  hipError_t e = hipMemcpyAsync(h, w->d.view + first * w->c.S, ne * sizeof(SwimE), hipMemcpyDeviceToHost, w->stream);
  if (e == hipSuccess && self_incarnation)
    e = hipMemcpyAsync(self_incarnation, w->d.self_inc + first, count * 4, hipMemcpyDeviceToHost, w->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(w->stream);
  if (e != hipSuccess) {
    free(h);
    return rsf::set_hip_error(e, "rsf_swim_dump copy", __FILE__, __LINE__);
  }
  for (uint64_t i = 0; i < ne; ++i) {  // an unknown entry reads as (UNKNOWN, 0, 0, 0)
    const bool known = h[i].state != RSF_SWIM_UNKNOWN;
    if (state) state[i] = h[i].state;
    if (incarnation) incarnation[i] = known ? h[i].inc : 0u;
    if (change) change[i] = known ? h[i].change : 0u;
    if (n_confirm) n_confirm[i] = h[i].state == RSF_SWIM_SUSPECT ? h[i].nconf : 0;
  }
  free(h);
  return RSF_OK;
}

}  // extern "C"
