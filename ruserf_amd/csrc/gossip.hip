// gossip.hip — the batched gossip round on CDNA4 (gfx950): Lamport-clock
// member-state merge + retransmit-limited dissemination.
//
// One round (see DESIGN.md "Round model"):
//   ml_kernel        memberlist transitions at every live member (handle_node_join/leave)
//   refute_kernel    broadcast_join for refutations spawned last round (base.rs:1437-1447)
//   originate_kernel api entry points: join/leave/force_leave/user_event/query
//   emit_kernel      ONE WAVE PER SENDER: the three queues live in registers (lane = queue slot);
//                    k distinct live peers (Philox); per peer broadcast_messages drains
//                    intent -> query -> event under the byte budget with wave argmin
//                    selection (TransmitLimitedQueue::get_broadcasts model)
//   radix sort       stable by receiver (hipCUB onesweep) -> canonical (sender, position) order
//   segment_kernel   receiver segment bounds in the sorted record stream
//   merge_kernel     ONE WAVE PER RECEIVER: lane 0 runs the handlers in canonical order, the
//                    wave re-queues rebroadcasts (ballot for a free slot / wave max for the prune)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/ruserf_amd.h"
#include "common.h"
#include "gossip_handlers.h"
#include "rsf_internal.h"

using namespace rsf;

namespace {

constexpr int kWave = 64;
#ifndef RSF_WPB
#define RSF_WPB 4  // waves per block of the merge and the other wave-per-member kernels
#endif
constexpr int kWavesPerBlock = RSF_WPB;
constexpr uint32_t kSentinel = 0xFFFFFFFFu;
// record decoration (what merge_kernel needs to address the view entry before the rumor
// body arrives): the subject slot of an intent, or the queue of a query / user event
constexpr uint32_t kDecQuery = 0xFFFFFFFEu, kDecEvent = 0xFFFFFFFDu, kDecViewMax = 0xFFFFFFF0u;
// Range guards on the round kernels' data-dependent indices (record slot, subject and
// pending-list index in the merge, sorted group ids): a violation is recorded
// (g_merge_prof[0] bit k, the value in [1 + k % 7], readable through rsf_gossip_merge_prof)
// and the access skipped.  They never fire on valid input; RSF_CHECKS=2 adds guards on every
// other data-dependent index (diagnostic builds; DESIGN.md §5, open issue at 1M x 4096).
#ifndef RSF_CHECKS
#define RSF_CHECKS 1
#endif
#if RSF_MERGE_PROF || RSF_EMIT_PROF || RSF_CHECKS
__device__ unsigned long long g_merge_prof[8];
#endif
// diagnostic build (experiments/deep_prof.py): why emit_run deferred members to the deep path
// ([0..7]), the deep wave kernel's per-phase shader-clock totals ([8..15]) and its queue sizes
// (a histogram by 128 items, [32..63]); read by rsf_gossip_deep_prof
#ifndef RSF_DEEP_PROF
#define RSF_DEEP_PROF 0
#endif
#if RSF_DEEP_PROF
__device__ unsigned long long g_deep_prof[80];
#define RSF_DEEP_WHY(k) \
  do {                  \
    if (lane == 0) atomicAdd(&g_deep_prof[(k)], 1ull); \
  } while (0)
#else
#define RSF_DEEP_WHY(k) \
  do {                  \
  } while (0)
#endif
#if RSF_CHECKS
#define RSF_BAD(k, cond, val) \
  ((cond) ? (atomicOr(&g_merge_prof[0], 1ull << (k)), g_merge_prof[1 + ((k) % 7)] = (unsigned long long)(val), true) : false)
#else
#define RSF_BAD(k, cond, val) false
#endif
// RSF_CHECKS >= 2 (diagnostic builds): further guards on every data-dependent index
#if RSF_CHECKS >= 2
#define RSF_BAD2(k, cond, val) RSF_BAD(k, cond, val)
#else
#define RSF_BAD2(k, cond, val) false
#endif
// wave-uniform forms for per-lane conditions: the whole wave records and skips together, so
// no lane leaves while the others go on through wave-wide ballots and shuffles.  Only in
// converged code (every lane of the wave active).
#if RSF_CHECKS
#define RSF_BAD_W(k, cond, val) (ballot(RSF_BAD(k, cond, val)) != 0)
#else
#define RSF_BAD_W(k, cond, val) false
#endif
#if RSF_CHECKS >= 2
#define RSF_BAD2_W(k, cond, val) RSF_BAD_W(k, cond, val)
#else
#define RSF_BAD2_W(k, cond, val) false
#endif

// Ballot of a per-lane condition straight from its compare.  HIP's __ballot takes an int, so
// the condition is first materialised as 0/1 in a VGPR and compared again (two extra vector
// instructions per ballot, and the emission and merge kernels take dozens per member).
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Wave-wide u64 min/max through DPP (row_ror inside 16-lane rows, then
// row_bcast15 / row_bcast31 across rows, result in lane 63): VALU-only data
// movement, no LDS permute round trips.  Every lane of the wave must be active.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = (uint32_t)__builtin_amdgcn_update_dpp((int)lo, (int)lo, CTRL, ROWMASK, 0xF, false);
  hi = (uint32_t)__builtin_amdgcn_update_dpp((int)hi, (int)hi, CTRL, ROWMASK, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t lane63_u64(uint64_t v) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}
#define RSF_DPP_STEP(OP, CTRL, RM)        \
  {                                       \
    uint64_t o_ = dpp64<CTRL, RM>(v);     \
    v = (o_ OP v) ? o_ : v;               \
  }
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  RSF_DPP_STEP(<, 0xB1, 0xF)   // quad_perm [1,0,3,2]
  RSF_DPP_STEP(<, 0x4E, 0xF)   // quad_perm [2,3,0,1]
  RSF_DPP_STEP(<, 0x124, 0xF)  // row_ror:4
  RSF_DPP_STEP(<, 0x128, 0xF)  // row_ror:8
  RSF_DPP_STEP(<, 0x142, 0xA)  // row_bcast:15 into rows 1,3
  RSF_DPP_STEP(<, 0x143, 0xC)  // row_bcast:31 into rows 2,3
  return lane63_u64(v);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  RSF_DPP_STEP(>, 0xB1, 0xF)
  RSF_DPP_STEP(>, 0x4E, 0xF)
  RSF_DPP_STEP(>, 0x124, 0xF)
  RSF_DPP_STEP(>, 0x128, 0xF)
  RSF_DPP_STEP(>, 0x142, 0xA)
  RSF_DPP_STEP(>, 0x143, 0xC)
  return lane63_u64(v);
}
#undef RSF_DPP_STEP
#define RSF_DPP_STEP32(CTRL, RM)                                                               \
  {                                                                                            \
    const uint32_t o_ = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, RM, 0xF, false); \
    v = o_ < v ? o_ : v;                                                                       \
  }
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  RSF_DPP_STEP32(0xB1, 0xF)
  RSF_DPP_STEP32(0x4E, 0xF)
  RSF_DPP_STEP32(0x124, 0xF)
  RSF_DPP_STEP32(0x128, 0xF)
  RSF_DPP_STEP32(0x142, 0xA)
  RSF_DPP_STEP32(0x143, 0xC)
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
#undef RSF_DPP_STEP32

// inclusive prefix max over the wave (lane 0 first); identity 0
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t dpp64_id0(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, ROWMASK, 0xF, false);
  hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, ROWMASK, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}
#define RSF_SCAN_STEP(CTRL, RM)            \
  {                                        \
    uint64_t o_ = dpp64_id0<CTRL, RM>(v);  \
    v = o_ > v ? o_ : v;                   \
  }
__device__ __forceinline__ uint64_t wave_inclusive_max_u64(uint64_t v) {
  RSF_SCAN_STEP(0x111, 0xF)  // row_shr:1
  RSF_SCAN_STEP(0x112, 0xF)  // row_shr:2
  RSF_SCAN_STEP(0x114, 0xF)  // row_shr:4
  RSF_SCAN_STEP(0x118, 0xF)  // row_shr:8
  RSF_SCAN_STEP(0x142, 0xA)  // row_bcast:15
  RSF_SCAN_STEP(0x143, 0xC)  // row_bcast:31
  return v;
}
#undef RSF_SCAN_STEP
// inclusive prefix sum over the wave (u32, identity 0)
__device__ __forceinline__ uint32_t wave_inclusive_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return v;
}

// value of the previous lane (lane 0 gets 0): wave_shr:1
__device__ __forceinline__ uint64_t wave_shr1_u64(uint64_t v) { return dpp64_id0<0x138, 0xF>(v); }

__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int lane) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// one transmit-limited queue held in registers: lane i owns slot i
struct QRegs {
  uint32_t r, sq, tl;  // rumor id (kEmpty = free), insertion seq, transmits | len << 16
  uint32_t dec = 0;    // emit only: the item's record decoration (subject / kDecQuery / kDecEvent)
};

#ifndef RSF_Q_NT
#define RSF_Q_NT 0  // broadcast queues (touched once by emit, once by merge per round) read / written non-temporally
#endif
// The intent queue also keeps each item's record decoration (its subject slot, q_dec);
// the query / event queues' decoration is the queue itself.
__device__ __forceinline__ void q_load(const GCfg& c, const GState& s, uint64_t l, uint32_t q, uint32_t lane,
                                       QRegs& Q) {
  Q.dec = q == 1 ? kDecQuery : kDecEvent;
  if (lane < c.qcap) {
    uint64_t i = (l * 3 + q) * c.qcap + lane;
#if RSF_Q_NT
    Q.r = __builtin_nontemporal_load(s.q_rumor + i);
    Q.sq = __builtin_nontemporal_load(s.q_seq + i);
    Q.tl = __builtin_nontemporal_load(s.q_txlen + i);
#else
    Q.r = s.q_rumor[i];
    Q.sq = s.q_seq[i];
    Q.tl = s.q_txlen[i];
#endif
    if (q == 0) Q.dec = s.q_dec[l * c.qcap + lane];
  } else {
    Q.r = kEmpty;
    Q.sq = 0;
    Q.tl = 0;
  }
}
__device__ __forceinline__ void q_store(const GCfg& c, const GState& s, uint64_t l, uint32_t q, uint32_t lane,
                                        const QRegs& Q, bool with_seq) {
  if (lane < c.qcap) {
    uint64_t i = (l * 3 + q) * c.qcap + lane;
#if RSF_Q_NT
    __builtin_nontemporal_store(Q.r, s.q_rumor + i);
    __builtin_nontemporal_store(Q.tl, s.q_txlen + i);
    if (with_seq) __builtin_nontemporal_store(Q.sq, s.q_seq + i);
#else
    s.q_rumor[i] = Q.r;
    s.q_txlen[i] = Q.tl;
    if (with_seq) s.q_seq[i] = Q.sq;
#endif
    if (q == 0) s.q_dec[l * c.qcap + lane] = Q.dec;
  }
}

// Queues are kept SORTED in send order: lane i of a queue holds the item with
// the i-th smallest key (transmits, ~len, ~seq); free slots (kEmpty) follow the
// live items.  The content is exactly the reference model's (first-free-slot /
// prune-the-last-item), only the slot order is canonical.

__device__ __forceinline__ uint64_t below_mask(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
// popcount of m over the lanes below this one (v_mbcnt: two vector instructions, no mask build)
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// this lane's bit of a wave-uniform mask (the mask is used as the lane condition directly)
__device__ __forceinline__ bool lane_bit(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// popcount of m over the lanes above this one
__device__ __forceinline__ uint32_t mbcnt_above(uint64_t m) {
  return (uint32_t)__popcll(m) - mbcnt(m) - (lane_bit(m) ? 1u : 0u);
}

// insert: position = number of smaller live keys; lanes at/after it shift by
// one, so on a full queue the last lane (the largest key) falls off = memberlist
// Prune; a new item that would land past the end is itself the pruned one.
// Returns 1 when the queue was full (a live item, possibly the new one, was dropped).
__device__ __forceinline__ uint32_t q_insert_wave(const GCfg& c, QRegs& Q, uint32_t lane, uint32_t rid, uint32_t len,
                                                  uint32_t seq) {
  const bool valid = lane < c.qcap;
  const bool live = valid && Q.r != kEmpty;
  const uint64_t newkey = tlq_key(0, len, seq);
  const uint64_t k = live ? tlq_key(Q.tl & 0xFFFF, Q.tl >> 16, Q.sq) : ~0ull;
  const uint32_t full = (uint32_t)__popcll(ballot(live)) == c.qcap ? 1u : 0u;
  const uint32_t pos = (uint32_t)__popcll(ballot(live && k < newkey));
  if (pos >= c.qcap) return full;
  const int src = lane ? (int)lane - 1 : 0;
  const uint32_t pr = (uint32_t)__shfl((int)Q.r, src), ps = (uint32_t)__shfl((int)Q.sq, src),
                 pt = (uint32_t)__shfl((int)Q.tl, src);
  if (valid && lane > pos) {
    Q.r = pr;
    Q.sq = ps;
    Q.tl = pt;
  }
  if (lane == pos) {
    Q.r = rid;
    Q.sq = seq;
    Q.tl = len << 16;
  }
  return full;
}

// Batched insert of new items (transmits 0) into a sorted queue, equivalent to
// q_insert_wave on each of them in lane order (seq = seq0, seq0+1, ...):
// inserting into a bounded sorted queue and pruning the largest key keeps the
// qcap smallest keys of everything inserted so far, so the result is the qcap
// smallest of (queue items U new items).  Keys are distinct (seqs are unique).
//   existing item i (sorted lane i) lands at i + #(new keys below it);
//   new item j lands at #(existing keys below it) + #(new keys below it).
// One pass over the new items counts both, then every slot PULLS its item
// (ds_bpermute): slots taken by new items are marked in a 64-bit mask, the
// others take the existing items in order.  Returns the number of live items
// that did not fit (memberlist Prune of the queue's tail).
__device__ __forceinline__ uint32_t q_insert_batch(const GCfg& c, QRegs& Q, uint32_t lane, bool ins, uint32_t rid,
                                                   uint32_t len, uint32_t seq0, uint64_t newmask) {
  const bool valid = lane < c.qcap;
  const bool live = valid && Q.r != kEmpty;
  const uint32_t n_live = (uint32_t)__popcll(ballot(live));
  const uint32_t myseq = seq0 + mbcnt(newmask);
  const uint64_t nkey = ins ? tlq_key(0, len, myseq) : ~0ull;
  const uint64_t ekey = live ? tlq_key(Q.tl & 0xFFFF, Q.tl >> 16, Q.sq) : ~0ull;
  uint32_t n_rank = 0, e_less = 0;
  uint64_t mm = newmask;
  while (mm) {
    const int k = __ffsll((long long)mm) - 1;
    mm &= mm - 1;
    const uint64_t bk = shfl_u64(nkey, k);
    const bool eb = live && bk < ekey;
    n_rank += (ins && bk < nkey) ? 1u : 0u;
    const uint32_t el = n_live - (uint32_t)__popcll(ballot(eb));
    e_less = (int)lane == k ? el : e_less;
  }
  const uint32_t pos_n = e_less + n_rank;
  // destinations of the surviving new items and, per destination, its source lane
  uint64_t dm = 0;
  uint32_t srcn = 0;
  mm = ballot(ins && pos_n < c.qcap);
  while (mm) {
    const int k = __ffsll((long long)mm) - 1;
    mm &= mm - 1;
    const uint32_t d = shfl_u32(pos_n, k);
    dm |= 1ull << d;
    srcn = lane == d ? (uint32_t)k : srcn;
  }
  const bool is_new = lane_bit(dm);
  const uint32_t ei = lane - mbcnt(dm);
  const bool is_old = !is_new && valid && ei < n_live;
  const int a_new = (int)(srcn * 4), a_old = (int)((is_old ? ei : lane) * 4);
  const uint32_t nr = (uint32_t)__builtin_amdgcn_ds_bpermute(a_new, (int)rid);
  const uint32_t ns = (uint32_t)__builtin_amdgcn_ds_bpermute(a_new, (int)myseq);
  const uint32_t nl = (uint32_t)__builtin_amdgcn_ds_bpermute(a_new, (int)len);
  const uint32_t orr = (uint32_t)__builtin_amdgcn_ds_bpermute(a_old, (int)Q.r);
  const uint32_t os = (uint32_t)__builtin_amdgcn_ds_bpermute(a_old, (int)Q.sq);
  const uint32_t ot = (uint32_t)__builtin_amdgcn_ds_bpermute(a_old, (int)Q.tl);
  if (valid) {
    Q.r = is_new ? nr : (is_old ? orr : kEmpty);
    Q.sq = is_new ? ns : (is_old ? os : 0u);
    Q.tl = is_new ? (nl << 16) : (is_old ? ot : 0u);
  }
  const uint32_t total = n_live + (uint32_t)__popcll(newmask);
  return total > c.qcap ? total - c.qcap : 0u;
}

// Items whose rumor slot was recycled (the slot's generation is no longer the id's)
// expire: they are dropped and the survivors keep their sorted order at the front.
// Returns the number dropped (wave-uniform).
__device__ __forceinline__ uint32_t q_expire(const GCfg& c, QRegs& Q, uint32_t lane, bool stale, bool permute_dec) {
  const bool valid = lane < c.qcap;
  const bool live = valid && Q.r != kEmpty;
  const uint64_t sm = ballot(live && stale);
  if (!sm) return 0;
  const bool keep = live && !stale;
  const uint64_t km = ballot(keep), vm = ballot(valid);
  const uint32_t mb_k = mbcnt(km), mb_f = mbcnt(vm & ~km);
  const uint32_t pos = keep ? mb_k : (valid ? (uint32_t)__popcll(km) + mb_f : lane);
  if (valid && !keep) {
    Q.r = kEmpty;
    Q.sq = 0;
    Q.tl = 0;
  }
  const int addr = (int)(pos * 4);
  Q.r = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.r);
  Q.sq = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.sq);
  Q.tl = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.tl);
  if (permute_dec) Q.dec = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.dec);
  return (uint32_t)__popcll(sm);
}

// One LDS row per wave: scratch of the batched insert (q_insert_batch_lds) and of the
// re-rank after a pick (q_get_broadcasts).
struct alignas(16) QLds {
  uint32_t r[kWave], sq[kWave], tl[kWave], dec[kWave];
};

// Re-rank after picks: the unpicked keepers (np_m) and the bumped keepers (pk_m) are each
// still sorted in lane order; merge them, free lanes after.  Each list's keys go to the
// wave's LDS row in order, and every keeper counts the other list's keys below its own by a
// binary search there (keys are distinct), all lanes at once: a handful of LDS reads
// instead of a wave-wide pass per bumped item.
template <bool PERMUTE_DEC>
__device__ __forceinline__ void q_rerank(const GCfg& c, QRegs& Q, uint32_t lane, uint64_t pk_m, uint64_t np_m,
                                         QLds& row) {
  const bool valid = lane < c.qcap;
  const uint64_t kept_m = pk_m | np_m;
  const bool np = lane_bit(np_m), kept = lane_bit(kept_m);
  const uint64_t mykey = tlq_key(Q.tl & 0xFFFF, Q.tl >> 16, Q.sq);
  uint64_t* const keys_np = reinterpret_cast<uint64_t*>(row.r);  // r + sq: 64 keys
  uint64_t* const keys_pk = reinterpret_cast<uint64_t*>(row.tl);  // tl + dec: 64 keys
  // (mbcnt is convergent: computed outside any select arm, or the select becomes a branch)
  const uint32_t mb_np = mbcnt(np_m), mb_pk = mbcnt(pk_m), mb_free = mbcnt(~kept_m);
  const uint32_t r_own = np ? mb_np : mb_pk;
  // both lists padded with keys above every real one (LDS writes of a wave land in order, so
  // the real keys overwrite the padding): the search needs no bounds test
  keys_np[lane] = ~0ull;
  keys_pk[lane] = ~0ull;
  if (kept) (np ? keys_np : keys_pk)[r_own] = mykey;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // lower_bound of mykey in the other list, branchless: a keeper's other list holds at most 63
  // keys (both lists share the wave's 64 lanes), so steps 32 .. 1 reach every count, and the
  // probes stay inside the 64-key row
  const uint64_t* const other = np ? keys_pk : keys_np;
  const uint32_t n_pk = (uint32_t)__popcll(pk_m), n_np = (uint32_t)__popcll(np_m);
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = 32; step; step >>= 1) lo = other[lo + step - 1] < mykey ? lo + step : lo;
  const uint32_t pos_free = valid ? n_pk + n_np + mb_free : lane;
  const uint32_t pos = kept ? r_own + lo : pos_free;
  __builtin_amdgcn_wave_barrier();  // the row is free once every lane has searched it
  const int addr = (int)(pos * 4);
  Q.r = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.r);
  Q.sq = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.sq);
  Q.tl = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.tl);
  if (PERMUTE_DEC) Q.dec = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)Q.dec);
}

// one get_broadcasts call on a sorted register-resident queue; returns bytes used.
// The lowest unpicked lane that fits IS the reference's pick (lowest transmits, then
// longest fitting, then newest): every skipped lower lane did not fit and never will.
// Written over wave-uniform lane masks (live, picked, kept): the selection loops are
// scalar work on one 64-bit mask instead of per-lane flags under exec masking.
#ifndef RSF_EMIT_NT
#define RSF_EMIT_NT 0  // emit: records written non-temporally
#endif
// DEEP (a tail behind the head, its key / length lower bounds tmin / tminlen): the call is
// exact only if every pick's key is below tmin and every stop with budget left is one no tail
// item could fit; otherwise *unsafe is set and the caller abandons the emission (the member
// then takes emit_deep_wave_kernel's whole-queue path).  Picks are checked before they are bumped.
template <bool PERMUTE_DEC, bool DEEP = false>
__device__ __forceinline__ int64_t q_get_broadcasts(const GCfg& c, QRegs& Q, uint32_t lane, int64_t limit,
                                                    uint32_t* stage_val, uint32_t* stage_dec,
                                                    uint64_t out_base, uint32_t& nrec, uint32_t& err, bool& dirty,
                                                    QLds& row, uint64_t tmin = ~0ull, uint32_t tminlen = ~0u,
                                                    bool* unsafe = nullptr) {
  const bool valid = lane < c.qcap;
  const uint64_t live_m = ballot(valid && Q.r != kEmpty);  // a sorted queue: a prefix
  if (!live_m) {
    if (DEEP && tmin != ~0ull && limit - (int64_t)c.overhead >= (int64_t)tminlen) {
      *unsafe = true;
      RSF_DEEP_WHY(3);
    }
    return 0;
  }
  const bool live = lane_bit(live_m);
  const uint32_t len = Q.tl >> 16;
  // Live items are the sorted prefix.  If every earlier item was taken, item i fits iff
  // the inclusive prefix sum of (overhead + len) is <= limit, so the leading run of picks
  // comes out of one wave scan; the remaining budget is then offered to later (shorter)
  // items one by one, as the reference does.
  if (limit < 0) return 0;
  const uint32_t lim = (uint32_t)limit;  // 32-bit budget arithmetic below (used <= lim)
  const uint32_t incl = wave_inclusive_sum_u32(live ? c.overhead + len : 0u);
  uint64_t pick_m = ballot(incl <= lim) & live_m;
  uint32_t used = pick_m ? shfl_u32(incl, 63 - __clzll((long long)pick_m)) : 0u;
  for (;;) {
    const int32_t free_b = (int32_t)(lim - used - c.overhead);
    if (free_b <= 0) break;
    const uint64_t cand = ballot(len <= (uint32_t)free_b) & live_m & ~pick_m;
    if (!cand) {
      if (DEEP && tminlen <= (uint32_t)free_b) {  // a tail item might fit
        *unsafe = true;
        RSF_DEEP_WHY(4);
      }
      break;
    }
    const int win = __ffsll((long long)cand) - 1;
    pick_m |= 1ull << win;
    used += c.overhead + shfl_u32(len, win);
  }
  if (DEEP && pick_m) {  // the largest pick (the highest lane: the head is sorted) below the tail
    const int hl = 63 - __clzll((long long)pick_m);
    const uint32_t tl = shfl_u32(Q.tl, hl);
    if (tlq_key(tl & 0xFFFF, tl >> 16, shfl_u32(Q.sq, hl)) >= tmin) {
      *unsafe = true;
      RSF_DEEP_WHY(5);
#if RSF_DEEP_PROF
      {  // diagnostic: is the first pick past the tail bound in the leading run (24) or a later
         // fit (25); would "no tail item fits the budget left before it" have decided it (26)
        const uint64_t below = ballot(live && tlq_key(Q.tl & 0xFFFF, Q.tl >> 16, Q.sq) < tmin);
        const uint64_t cross = pick_m & ~below;
        const int fc = __ffsll((long long)cross) - 1;
        const uint64_t before = fc > 0 ? (~0ull >> (64 - fc)) : 0ull;
        RSF_DEEP_WHY((pick_m & before) == before ? 24 : 25);
        RSF_DEEP_WHY((shfl_u32(Q.tl, fc) & 0xFFFF) == 0 ? 27 : 28);  // the crossing pick's transmit class
        if ((tmin >> 48) == 0) RSF_DEEP_WHY(7);  // the tail's bound is a transmits-0 key
        const uint32_t ub = wave_inclusive_sum_u32(lane_bit(pick_m & before) ? c.overhead + len : 0u);
        const int32_t f0 = (int32_t)lim - (int32_t)shfl_u32(ub, 63) - (int32_t)c.overhead;
        if (f0 < (int32_t)tminlen) RSF_DEEP_WHY(26);
      }
#endif
    }
  }
  if (DEEP && *unsafe) return used;
  if (!pick_m) return used;
  // picks are in ascending lane (= send) order: record rank = picked lanes below
  const bool picked = lane_bit(pick_m);
  const uint32_t npick = (uint32_t)__popcll(pick_m);
  const uint32_t rank = mbcnt(pick_m);
  if (picked && nrec + rank < c.cap_t && stage_val) {
#if RSF_EMIT_NT
    __builtin_nontemporal_store(Q.r, stage_val + out_base + nrec + rank);
    if (stage_dec) __builtin_nontemporal_store(Q.dec, stage_dec + out_base + nrec + rank);
#else
    stage_val[out_base + nrec + rank] = Q.r;
    if (stage_dec) stage_dec[out_base + nrec + rank] = Q.dec;
#endif
  }
  if (nrec + npick > c.cap_t) err |= kErrStage;
  nrec += npick;
  dirty = true;
  // transmits+1, or retire at the retransmit limit
  const bool retire = picked && (Q.tl & 0xFFFF) + 1 >= c.tx_limit;
  const uint64_t ret_m = ballot(retire);
  Q.r = retire ? kEmpty : Q.r;
  Q.tl = (picked && !retire) ? Q.tl + 1 : Q.tl;
  q_rerank<PERMUTE_DEC>(c, Q, lane, pick_m & ~ret_m, live_m & ~pick_m, row);
  return used;
}

// All the fanout peers' get_broadcasts calls on ONE queue in one pass (queue-major emission).
// A peer's picks from queue q depend only on q's state after the earlier peers' picks from q
// and on what the peer's earlier queues left of its byte budget, so running queue 0 for every
// peer, then queue 1, then queue 2 picks exactly what the reference's peer-major
// broadcast_messages loop picks.  Within a queue, for every peer: while all picks come from the queue's lowest transmit class t0 (the leading run
// of the sorted queue), the send order is [unpicked class-t0 items in lane order] followed by
// everything else, so ONE prefix sum of the run's costs serves every peer (each peer's prefix
// is a further stretch of the same sums), the picked items are bumped in place and the re-rank
// runs once at the end.  Picks are recorded per lane (peer, slot in the peer's group) and
// written together after the last peer.  When a peer's next candidate could lie past the run,
// the deferred picks are written and re-ranked into place and the remaining peers run the
// exact q_get_broadcasts one by one.
// Per-peer state is lane-distributed: lane j (< np) holds peer j's bytes used so far (used_v),
// records written so far (nrec_v) and the element offset of its group's record slots from
// ov / od (off_v; ~0 = no output: a bucket over capacity).
// DEEP: as q_get_broadcasts -- abandoned (*unsafe) as soon as the head alone cannot decide.
template <bool PERMUTE_DEC, bool DEEP = false>
__device__ __forceinline__ void q_pick_peers(const GCfg& c, QRegs& Q, uint32_t lane, uint32_t np, uint32_t& used_v,
                                             uint32_t& nrec_v, uint64_t off_v, uint32_t* ov, uint32_t* od,
                                             uint32_t& err, bool& dirty, QLds& row, uint64_t* ep = nullptr,
                                             uint64_t tmin = ~0ull, uint32_t tminlen = ~0u, bool* unsafe = nullptr) {
  const bool valid = lane < c.qcap;
  const uint64_t live_m = ballot(valid && Q.r != kEmpty);  // a sorted queue: a prefix
  if (!live_m) {
    if (DEEP && tmin != ~0ull) {  // only the tail holds items
      *unsafe = true;
      RSF_DEEP_WHY(0);
    }
    return;
  }
#if RSF_EMIT_PROF
  const uint64_t pp0 = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t t0 = shfl_u32(Q.tl, 0) & 0xFFFF;  // lane 0 holds the smallest key
  const uint32_t len = Q.tl >> 16;
  const uint64_t a_m = ballot((Q.tl & 0xFFFF) == t0) & live_m;
  const bool retire_all = t0 + 1 >= c.tx_limit;  // every pick of class t0 retires (or none does)
  uint32_t incl = wave_inclusive_sum_u32(lane_bit(a_m) ? c.overhead + len : 0u);
  uint32_t base = 0;      // the sums consumed by the picks so far (while they are a prefix of the run)
  bool prefix = true;     // the picks so far are a prefix of the class-t0 run
  uint64_t cons = 0;      // picked so far (all of class t0), bumped in place, not yet written
  uint64_t gone = 0;      // picked and retiring: no longer candidates
  uint32_t pk_peer = 0, pk_pos = 0;  // a picked lane: its peer and its slot in the peer's group
  uint32_t j = 0;
  bool exact = false;
  for (; j < np; ++j) {
    // 32-bit budget arithmetic (a peer's bytes used never exceed the limit): scalar 32-bit
    // operations instead of 64-bit pairs in the loop the emission spends most of its scalar
    // issue on
    const uint32_t limit = c.limit - shfl_u32(used_v, j);
    const uint64_t rem = a_m & ~cons;
    if (!prefix) {  // a skip broke the run's prefix: sums of what is left of it
      incl = wave_inclusive_sum_u32(lane_bit(rem) ? c.overhead + len : 0u);
      base = 0;
      prefix = true;
    }
    // (lanes before the consumed prefix wrap to huge sums and fail the compare; masked anyway)
    uint64_t pick = ballot(incl - base <= limit) & rem;
    const uint32_t top = pick ? shfl_u32(incl, 63 - __clzll((long long)pick)) : base;
    uint32_t used = top - base;
    bool skipped = false;
    const uint64_t avail = live_m & ~gone;
    for (;;) {
      const int32_t free_b = (int32_t)(limit - used - c.overhead);
      if (free_b <= 0) break;
      const uint64_t fit = ballot(len <= (uint32_t)free_b) & avail & ~pick;
      if (!fit) {
        if (DEEP && tminlen <= (uint32_t)free_b) {  // a tail item might fit
          *unsafe = true;
          RSF_DEEP_WHY(1);
        }
        break;
      }
      const uint64_t cand = fit & rem;
      if (!cand) {  // the next candidate lies past the class-t0 run (or is a bumped pick)
        exact = true;
        break;
      }
      const int win = __ffsll((long long)cand) - 1;
      pick |= 1ull << win;
      used += c.overhead + shfl_u32(len, win);
      skipped = true;
    }
    if (exact) break;
    if (DEEP && *unsafe) return;
    if (pick) {
      const uint32_t npick = (uint32_t)__popcll(pick);
      const uint32_t nrec = shfl_u32(nrec_v, j);
      const bool pb = lane_bit(pick);
      const uint32_t mb = mbcnt(pick);
      pk_peer = pb ? j : pk_peer;
      pk_pos = pb ? nrec + mb : pk_pos;  // picks in ascending lane (= send) order
      if (nrec + npick > c.cap_t) err |= kErrStage;
      nrec_v = lane == j ? nrec + npick : nrec_v;
      cons |= pick;
      if (retire_all) gone |= pick;
      dirty = true;
      if (skipped) prefix = false;
      else base = top;
    }
    used_v += lane == j ? used : 0u;
  }
#if RSF_EMIT_PROF
  const uint64_t pp1 = __builtin_amdgcn_s_memtime();
  ep[0] += pp1 - pp0;  // picks (prefix sums, fit loops)
  if (exact) ep[4] += 1;  // emissions that needed the exact path
#endif
  if (DEEP && cons) {  // the largest deferred pick (highest lane) below the tail
    const int hl = 63 - __clzll((long long)cons);
    const uint32_t tl = shfl_u32(Q.tl, hl);
    if (tlq_key(tl & 0xFFFF, tl >> 16, shfl_u32(Q.sq, hl)) >= tmin) {
      *unsafe = true;
      RSF_DEEP_WHY(2);
      RSF_DEEP_WHY((tl & 0xFFFF) == 0 ? 27 : 28);  // (diagnostic) the crossing pick's transmit class
      return;
    }
  }
  if (cons) {
    // the deferred picks: records to their groups, then transmits + 1 or retired
    const bool picked = lane_bit(cons);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)off_v, (int)pk_peer);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(off_v >> 32), (int)pk_peer);
    const uint64_t off = ((uint64_t)hi << 32) | lo;
    if (picked && pk_pos < c.cap_t && off != ~0ull) {
#if RSF_EMIT_NT
      __builtin_nontemporal_store(Q.r, ov + off + pk_pos);
      if (od) __builtin_nontemporal_store(Q.dec, od + off + pk_pos);
#else
      ov[off + pk_pos] = Q.r;
      if (od) od[off + pk_pos] = Q.dec;
#endif
    }
    Q.r = (picked && retire_all) ? kEmpty : Q.r;
    Q.tl = (picked && !retire_all) ? Q.tl + 1 : Q.tl;
#if RSF_EMIT_PROF
    const uint64_t pp2 = __builtin_amdgcn_s_memtime();
    ep[1] += pp2 - pp1;  // deferred stores + bumps
#endif
    q_rerank<PERMUTE_DEC>(c, Q, lane, cons & ~gone, live_m & ~cons, row);
#if RSF_EMIT_PROF
    ep[2] += __builtin_amdgcn_s_memtime() - pp2;  // re-rank
#endif
  }
#if RSF_EMIT_PROF
  const uint64_t pp3 = __builtin_amdgcn_s_memtime();
#endif
  // the remaining peers exactly, one re-rank after each
  for (; j < np; ++j) {
    const int64_t limit = (int64_t)c.limit - (int64_t)shfl_u32(used_v, j);
    uint32_t nrec = shfl_u32(nrec_v, j);
    const uint64_t off = shfl_u64(off_v, j);
    const bool out = off != ~0ull;
    const int64_t used = q_get_broadcasts<PERMUTE_DEC, DEEP>(c, Q, lane, limit, out ? ov : nullptr, out ? od : nullptr,
                                                             out ? off : 0ull, nrec, err, dirty, row, tmin, tminlen,
                                                             unsafe);
    if (DEEP && *unsafe) return;
    used_v += lane == j ? (uint32_t)used : 0u;
    nrec_v = lane == j ? nrec : nrec_v;
  }
#if RSF_EMIT_PROF
  ep[3] += __builtin_amdgcn_s_memtime() - pp3;  // exact tail
#endif
}

// Deep queues: the running tail of one (member, queue) while a wave works on its head.  cnt,
// minlen, minkey mirror tsum (wave-uniform); spills are written at t[cnt ...] (the row has
// kTailSlack slots past the capacity) and counted in only by the caller's commit.
struct Spill {
  uint4* t = nullptr;      // the query / event queues' 16-B items
  uint64_t* t8 = nullptr;  // the intent queue's packed items (tail_pack)
  uint32_t cnt = 0, minlen = 0xFFFFFFFFu;
  uint64_t minkey = ~0ull;
};
__device__ __forceinline__ void spill_row(const GCfg& c, const GState& s, uint64_t l, uint32_t q, Spill& sp) {
  if (q == 0) sp.t8 = tail8(s, c, l);
  else sp.t = tail16(s, q) + l * tstride_of(c, q);
}
__device__ __forceinline__ void spill_put(const GCfg& c, const Spill& sp, uint32_t i, uint32_t rid, uint32_t seq,
                                          uint32_t tl, uint32_t dec) {
  if (sp.t8) sp.t8[i] = tail_pack(c, rid, seq, tl);
  else sp.t[i] = make_uint4(rid, seq, tl, dec);
}
__device__ __forceinline__ Spill spill_of(const GCfg& c, const GState& s, uint64_t l, uint32_t q, uint4 sm) {
  Spill sp;
  spill_row(c, s, l, q, sp);
  sp.cnt = sm.x;
  sp.minlen = sm.y;
  sp.minkey = ((uint64_t)sm.w << 32) | sm.z;
  return sp;
}
__device__ __forceinline__ uint4 spill_sum(const Spill& sp) {
  return make_uint4(sp.cnt, sp.minlen, (uint32_t)sp.minkey, (uint32_t)(sp.minkey >> 32));
}
constexpr uint4 kTSumEmpty = {0u, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

// Batched insert of new items (transmits 0, seqs seq0, seq0 + 1, ... in lane order over
// `newmask`) into a sorted register-resident queue: the result is the qcap smallest keys of
// (queue items U new items), exactly memberlist's insert-then-prune one at a time.  Done
// over the DISTINCT LENGTHS of the new items instead of the items.  New items all have
// transmits 0 and newer seqs than anything queued, so:
//   new j lands at  #{queued: tx 0, len > len_j} + #{new: len > len_j} + #{new: len == len_j, later lane}
//   queued i (lane i) lands at  i + (tx_i > 0 ? n_new : #{new: len >= len_i})
// -- one pass per distinct new length (the message-length model has a handful), then
// every item is written to its place in the wave's LDS row and read back in order.
// DEC: the items' record decorations (Q.dec / dec) move with them.
// Returns the number of live items that did not fit (memberlist Prune of the tail).
// SPILL (deep queues): the items that do not fit the head go to the tail instead (sp), and
// the return value is 0; the caller checks the tail's capacity.
template <bool DEC, bool SPILL = false>
__device__ __forceinline__ uint32_t q_insert_batch_lds(const GCfg& c, QRegs& Q, uint32_t lane, bool ins, uint32_t rid,
                                                       uint32_t dec, uint32_t len, uint32_t seq0, uint64_t newmask,
                                                       QLds& row, Spill* sp = nullptr) {
  const bool valid = lane < c.qcap;
  const uint64_t live_m = ballot(valid && Q.r != kEmpty);
  const bool live = lane_bit(live_m);
  const uint32_t n_live = (uint32_t)__popcll(live_m);
  const uint32_t n_new = (uint32_t)__popcll(newmask);
  const uint32_t myseq = seq0 + mbcnt(newmask);
  const uint64_t etx0_m = ballot((Q.tl & 0xFFFF) == 0) & live_m;  // queued items of transmits 0
  const uint32_t elen = Q.tl >> 16;
  uint32_t pos_n = 0, pos_e = lane + (lane_bit(live_m & ~etx0_m) ? n_new : 0u);
  // one pass per distinct new length, over wave-uniform masks (ins == this lane's bit of newmask)
  uint64_t rem = newmask;
  while (rem) {
    const uint32_t L = shfl_u32(len, __ffsll((long long)rem) - 1);
    const uint64_t same = ballot(len == L) & newmask;
    rem &= ~same;
    const uint64_t gt_old_m = ballot(elen > L) & etx0_m;
    const uint32_t base = (uint32_t)__popcll(ballot(len > L) & newmask) + (uint32_t)__popcll(gt_old_m);
    const uint32_t ab = mbcnt_above(same);
    pos_n = lane_bit(same) ? base + ab : pos_n;
    pos_e += lane_bit(etx0_m & ~gt_old_m) ? (uint32_t)__popcll(same) : 0u;
  }
  if (SPILL && n_live + n_new > c.qcap) {
    // positions past the head are the largest keys, in order: they go to the tail, the one at
    // position qcap being the smallest of them
    const bool sn = ins && pos_n >= c.qcap, se = live && pos_e >= c.qcap;
    // (ordinary stores: non-temporal ones measured 1.37 -> 2.24 ms of emission, later spills
    // landing in the same partly written sectors)
    if (sn) spill_put(c, *sp, sp->cnt + (pos_n - c.qcap), rid, myseq, len << 16, DEC ? dec : 0u);
    if (se) spill_put(c, *sp, sp->cnt + (pos_e - c.qcap), Q.r, Q.sq, Q.tl, DEC ? Q.dec : 0u);
    const uint64_t at_n = ballot(ins && pos_n == c.qcap), at_e = ballot(live && pos_e == c.qcap);
    const int w = __ffsll((long long)(at_n | at_e)) - 1;
    const uint32_t tl_w = at_n ? (shfl_u32(len, w) << 16) : shfl_u32(Q.tl, w);
    const uint32_t sq_w = at_n ? shfl_u32(myseq, w) : shfl_u32(Q.sq, w);
    const uint64_t kmin = tlq_key(tl_w & 0xFFFF, tl_w >> 16, sq_w);
    const uint32_t lmin = wave_min_u32(min(sn ? len : 0xFFFFFFFFu, se ? elen : 0xFFFFFFFFu));
    sp->cnt += n_live + n_new - c.qcap;
    sp->minkey = kmin < sp->minkey ? kmin : sp->minkey;
    sp->minlen = lmin < sp->minlen ? lmin : sp->minlen;
  }
  if (ins && pos_n < c.qcap) {
    row.r[pos_n] = rid;
    row.sq[pos_n] = myseq;
    row.tl[pos_n] = len << 16;
    if (DEC) row.dec[pos_n] = dec;
  }
  if (live && pos_e < c.qcap) {
    row.r[pos_e] = Q.r;
    row.sq[pos_e] = Q.sq;
    row.tl[pos_e] = Q.tl;
    if (DEC) row.dec[pos_e] = Q.dec;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t total = n_live + n_new;
  {
    // every lane reads its slot; lanes past the items (or the queue) select the free value
    const bool take = valid && lane < total;
    const uint32_t r = row.r[lane], sq = row.sq[lane], tl = row.tl[lane];
    const uint32_t fr = valid ? kEmpty : Q.r, fs = valid ? 0u : Q.sq, ft = valid ? 0u : Q.tl;
    Q.r = take ? r : fr;
    Q.sq = take ? sq : fs;
    Q.tl = take ? tl : ft;
    if (DEC) {
      const uint32_t d = row.dec[lane];
      Q.dec = take ? d : Q.dec;
    }
  }
  __builtin_amdgcn_wave_barrier();  // the row is free once every lane has read it
  return (!SPILL && total > c.qcap) ? total - c.qcap : 0u;
}

// A member's pending re-queues (pc: their packed counts, which the caller may hold in
// registers) applied to its queues by one wave (lane = slot / entry):
// per queue, its entries in insertion order take the next seqs and go in as one batch.
// Adds the live items dropped to q_pruned and returns their number (the caller flags
// kErrQueue).  merge_kernel calls it only when a list would overflow.
// The entries of one queue from the wave's two batches of the list (lanes 0..63 hold
// entries lane and 64 + lane) go in as one batch after the other, seqs continuing.
struct PendRegs {
  uint32_t rid[2], dec[2], lq[2];
};
__device__ __forceinline__ void pend_load(const GState& s, uint64_t l, uint32_t lane, uint32_t n, PendRegs& p) {
#pragma unroll
  for (uint32_t b = 0; b < 2; ++b) {
    p.rid[b] = p.dec[b] = p.lq[b] = 0;
    if (b * kWave + lane < n) {
      const GState::PendE e = s.p_ent[l * kPend + b * kWave + lane];
      p.rid[b] = e.rid;
      p.dec[b] = e.dec;
      p.lq[b] = e.lq;
    }
  }
}
template <bool DEC, bool SPILL = false>
__device__ __forceinline__ uint32_t pend_apply(const GCfg& c, QRegs& Q, uint32_t lane, uint32_t q, uint32_t n,
                                               const PendRegs& p, uint32_t seq0, QLds& row, Spill* sp = nullptr) {
  uint32_t drops = 0, seq = seq0;
#pragma unroll
  for (uint32_t b = 0; b < 2; ++b) {
    if (b * kWave >= n) break;
    const bool ins = b * kWave + lane < n && (p.lq[b] >> 16) == q;
    const uint64_t m = ballot(ins);
    if (!m) continue;
    drops += q_insert_batch_lds<DEC, SPILL>(c, Q, lane, ins, p.rid[b], p.dec[b], p.lq[b] & 0xFFFF, seq, m, row, sp);
    seq += (uint32_t)__popcll(m);
  }
  return drops;
}

// Deep queues: while the tail holds more than its capacity (head + tail over the queue's
// depth), drop the largest key of the two -- the bounded queue's prune, rare (a queue at its
// full depth).  That key is always in the tail: the tail only goes past its capacity by this
// call's spills, and a spilled item is, by construction, at least every key left in the
// head (the items whose sorted position among head and new items is >= queue_cap).  So one
// pass over the tail finds it.  One wave; returns the number dropped.
// nseq: the queue's next seq after the spills (every tail item is older)
__device__ __forceinline__ uint32_t deep_prune_wave(const GCfg& c, QRegs& Q, uint32_t lane, uint32_t q, Spill& sp,
                                                    uint32_t nseq) {
  (void)Q;
  uint32_t drops = 0;
  while (sp.cnt > tcap_of(c, q)) {
    uint64_t tk = 0;
    uint32_t ti = 0;
    for (uint32_t b = 0; b < sp.cnt; b += kWave) {  // the tail holds items (cnt > tcap >= 1)
      const bool in = b + lane < sp.cnt;
      uint64_t k = 0ull;
      if (sp.t8) {
        const uint64_t x = in ? sp.t8[b + lane] : 0ull;
        const uint32_t tl = tail_tl(x);
        k = in ? tlq_key(tl & 0xFFFF, tl >> 16, tail_seq(x, nseq)) : 0ull;
      } else {
        const uint4 e = in ? sp.t[b + lane] : make_uint4(0u, 0u, 0u, 0u);
        k = in ? tlq_key(e.z & 0xFFFF, e.z >> 16, e.y) : 0ull;
      }
      const uint64_t m = wave_max_u64(k);
      const uint64_t at = ballot(in && k == m);
      if (at && (b == 0 || m > tk)) {
        tk = m;
        ti = b + (uint32_t)(__ffsll((long long)at) - 1);
      }
    }
    if (sp.t8) {
      const uint64_t last = sp.t8[sp.cnt - 1];
      if (lane == 0) sp.t8[ti] = last;
    } else {
      const uint4 last = sp.t[sp.cnt - 1];
      if (lane == 0) sp.t[ti] = last;
    }
    __threadfence_block();  // the next pass reads the moved item
    sp.cnt--;
    drops++;
  }
  return drops;
}

__device__ __forceinline__ uint32_t pend_flush_wave(const GCfg& c, const GState& s, uint64_t l, uint32_t lane,
                                                    uint32_t pc, QLds& row) {
  const uint32_t n = pend_total(pc);
  if (n == 0) return 0;
  PendRegs p;
  pend_load(s, l, lane, n, p);
  uint32_t drops = 0;
#pragma unroll
  for (uint32_t q = 0; q < 3; ++q) {
    const uint32_t nq = (pc >> (8 * q)) & 0xFF;
    if (!nq) continue;
    QRegs Q{kEmpty, 0, 0};
    q_load(c, s, l, q, lane, Q);
    const uint32_t seq0 = s.q_next_seq[l * 3 + q];
    if (tcap_of(c, q)) {  // deep queue: the head's overflow spills into the tail
      Spill sp = spill_of(c, s, l, q, s.tsum[l * 3 + q]);
      pend_apply<true, true>(c, Q, lane, q, n, p, seq0, row, &sp);
      const uint32_t pd = deep_prune_wave(c, Q, lane, q, sp, seq0 + nq);
      drops += pd;
      if (lane == 0) {
        s.tsum[l * 3 + q] = spill_sum(sp);
        if (pd) s.tseal[l * 3 + q].x = 0u;  // the prune moved items inside the tail: no seal
      }
    } else {
      drops += pend_apply<true>(c, Q, lane, q, n, p, seq0, row);
    }
    q_store(c, s, l, q, lane, Q, true);
    if (lane == 0) s.q_next_seq[l * 3 + q] = seq0 + nq;
  }
  if (lane == 0) {
    s.p_cnt[l] = 0;
    if (drops) s.q_pruned[l] += drops;
  }
  return drops;
}

#include "gossip_queue4.h"

// a member's pending list applied to queues of either layout (qcap <= 64: one slot per
// lane; up to 256: four, gossip_queue4.h); `row` is a QLds4 (which holds a QLds)
__device__ __forceinline__ uint32_t pend_flush_any(const GCfg& c, const GState& s, uint64_t l, uint32_t lane,
                                                   uint32_t pc, QLds4& row) {
  if (c.qcap > kWave) return q4_pend_flush_wave(c, s, l, lane, pc, row);
  return pend_flush_wave(c, s, l, lane, pc, *reinterpret_cast<QLds*>(&row));
}
static_assert(sizeof(QLds4) >= sizeof(QLds), "a QLds4 row holds a QLds");

// every member's pending re-queues applied (before anything but emission reads the queues)
// period > 1: only the members whose global id is phase mod period (a staggered checker tick);
// the grids run over those members only: local ids phase_first + i * period
__host__ __device__ inline uint64_t phase_first(const GCfg& c, uint32_t period, uint32_t phase) {
  return (phase + period - (uint32_t)(c.lo % period)) % period;
}
__host__ __device__ inline uint64_t phase_count(const GCfg& c, uint32_t period, uint32_t phase) {
  const uint64_t l0 = phase_first(c, period, phase);
  return c.n_loc > l0 ? (c.n_loc - l0 + period - 1) / period : 0;
}
__global__ void __launch_bounds__(256) pend_flush_kernel(GCfg c, GState s, uint32_t period, uint32_t phase) {
  __shared__ QLds4 rows[kWavesPerBlock];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t l = phase_first(c, period, phase) +
                     ((uint64_t)blockIdx.x * kWavesPerBlock + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave)) *
                         period;
  if (l >= c.n_loc) return;
  const uint32_t pc = s.p_cnt[l];
  if (!pc) return;
  if (pend_flush_any(c, s, l, lane, pc, rows[threadIdx.x / kWave]) && lane == 0) s.err[l] |= kErrQueue;
}

// ---------------------------------------------------------------- kernels
__global__ void __launch_bounds__(256) ml_kernel(GCfg c, GState s, const rsf_ml_event* __restrict__ ml,
                                                 uint32_t n_ml) {
  uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= c.n_loc) return;
  const uint32_t m = (uint32_t)(c.lo + l);
  bool al = s.alive[m] != 0;
  MRegs r;
  load_regs(s, l, r);
  bool touched = false;
  for (uint32_t e = 0; e < n_ml; ++e) {
    uint32_t subj = ml[e].subject, sm = s.subj_member[subj];
    if (sm == m && ml[e].set_alive == 1) {
      al = true;
      r.serf_state = kSerfAlive;
      touched = true;
    }
    if (al && m != sm) {
      ViewS* v = vent(s, c, l, subj);
      if (ml[e].kind == RSF_ML_JOIN) {
        h_node_join(v, r, subj);
        snap_member(c, s, l, subj, true);
        mlog_put(c, s, l, r.err, kEvJoin, subj);
      } else if (ml[e].kind == RSF_ML_UPDATE) {
        if (h_node_update(v, r, subj)) mlog_put(c, s, l, r.err, kEvUpdate, subj);
      } else {
        const int f = h_node_leave(v, r, subj, c.now);
        if (f & RSF_F_MEMBER_EVENT) {
          snap_member(c, s, l, subj, false);
          mlog_put(c, s, l, r.err, (uint32_t)f >> kFEvShift, subj);
        }
      }
      touched = true;
    }
    if (sm == m && ml[e].set_alive == 0) al = false;
  }
  if (touched) store_regs(s, l, r);
  s.alive[m] = al ? 1 : 0;
}

// liveness of every member (replicated array): last set_alive per subject wins
__global__ void ml_alive_kernel(GState s, const rsf_ml_event* __restrict__ ml, uint32_t n_ml) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (uint32_t e = 0; e < n_ml; ++e) {
    uint32_t sm = s.subj_member[ml[e].subject];
    if (ml[e].set_alive == 1) s.alive[sm] = 1;
    if (ml[e].set_alive == 0) s.alive[sm] = 0;
  }
}

__device__ __forceinline__ void put_rumor(const GCfg& c, const GState& s, uint32_t rid, uint8_t type, uint8_t flags, uint32_t subj,
                                          uint64_t L, uint64_t key, uint32_t len) {
  rsf_rumor ru;
  ru.ltime = L;
  ru.key = key;
  ru.subject = subj;
  ru.type = type;
  ru.flags = flags;
  ru.msg_len = (uint16_t)len;
  s.rumors[rid & c.rmask] = ru;
}

__device__ __forceinline__ void push_refute(const GCfg& c, const GState& s, MRegs& r, uint64_t ltime) {
  if (r.subj < 0) return;
  if (RSF_BAD2(11, (uint32_t)r.subj >= c.S, r.subj)) return;
  uint32_t cnt = s.refute_cnt[r.subj];
  if (cnt < c.max_refute) {
    s.refute_ltime[(uint64_t)r.subj * c.max_refute + cnt] = ltime;
    s.refute_cnt[r.subj] = cnt + 1;
  } else {
    r.err |= kErrRefute;
  }
}

// broadcast_join (base.rs:396-412)
__device__ __forceinline__ void broadcast_join(const GCfg& c, const GState& s, uint64_t l, MRegs& r, uint64_t L,
                                               uint32_t rid) {
  uint32_t subj = (uint32_t)r.subj;
  witness(r.clock, L);
  h_join_intent(vent(s, c, l, subj), r, L, c.now);
  uint32_t len = msg_len(RSF_MSG_JOIN, L, 0, 0);
  put_rumor(c, s, rid, RSF_MSG_JOIN, 0, subj, L, 0, len);
  pend_push_serial(c, s, l, kQIntent, rid, subj, len, r);
}

__global__ void __launch_bounds__(256) refute_kernel(GCfg c, GState s, uint32_t base) {
  uint32_t subj = blockIdx.x * blockDim.x + threadIdx.x;
  if (subj >= c.S) return;
  uint32_t m = s.subj_member[subj];
  if (m < c.lo || m >= c.lo + c.n_loc) return;
  uint32_t cnt = s.refute_cnt[subj];
  if (!cnt) return;
  s.refute_cnt[subj] = 0;
  if (!s.alive[m]) return;
  uint64_t l = m - c.lo;
  MRegs r;
  load_regs(s, l, r);
  for (uint32_t i = 0; i < cnt; ++i)
    broadcast_join(c, s, l, r, s.refute_ltime[(uint64_t)subj * c.max_refute + i], base + subj * c.max_refute + i);
  store_regs(s, l, r);
}

// status[a] = the entry point's result (rsf_gossip_action_status): RSF_OK, RSF_SKIPPED (not
// this shard's member, or its process is down), or a size-limit error, in which case the
// action does nothing at all (the reference returns before any clock or queue moves).
__global__ void __launch_bounds__(256) originate_kernel(GCfg c, GState s, const rsf_action* __restrict__ acts,
                                                        uint32_t n_acts, uint32_t abase, int32_t* __restrict__ status) {
  uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n_acts) return;
  rsf_action x = acts[a];
  uint32_t m = x.member;
  if (m < c.lo || m >= c.lo + c.n_loc || !s.alive[m]) {
    status[a] = RSF_SKIPPED;
    return;
  }
  uint64_t l = m - c.lo;
  uint32_t rid = abase + a;
  if (x.act == RSF_ACT_USER_EVENT || x.act == RSF_ACT_QUERY) {
    const int32_t e = x.act == RSF_ACT_USER_EVENT
                          ? user_event_size_check(c.max_ue, s.eclock[l], x.name_len, x.payload_len)
                          : query_size_check(c.query_limit, s.qclock[l], x.name_len, x.payload_len);
    if (e) {
      status[a] = e;
      return;
    }
  }
  MRegs r;
  load_regs(s, l, r);
  // join / leave of the member itself: only a tracked subject has a view entry about itself
  // (rsf_gossip_round_begin rejects the call on the host; this keeps the status truthful)
  if ((x.act == RSF_ACT_JOIN_SELF || x.act == RSF_ACT_LEAVE_SELF) && (uint32_t)r.subj >= c.S) {
    status[a] = RSF_ERR_ARG;
    return;
  }
  status[a] = RSF_OK;
  uint64_t ref = 0;
  switch (x.act) {
    case RSF_ACT_JOIN_SELF:
      r.serf_state = kSerfAlive;
      broadcast_join(c, s, l, r, r.clock, rid);
      break;
    case RSF_ACT_LEAVE_SELF: {
      r.serf_state = kSerfLeaving;
      uint64_t lt = r.clock;
      if (s.snap_sn && !(s.snap_sn[l * 4 + 3] & 1)) {
        // Snapshot::leave (snapshot.rs:568-586): the clock ticker's last value, then the
        // alive set is dropped (unless rejoin_after_leave) and recording stops
        s.snap_sn[l * 4 + 2] = lt ? lt - 1 : 0;
        s.snap_sn[l * 4 + 3] |= 1;
        if (!c.snap_rejoin)
          for (uint32_t k = 0; k < c.snap_w; ++k) s.snap_bits[l * c.snap_w + k] = 0;
      }
      r.clock++;
      uint32_t subj = (uint32_t)r.subj;
      mlog_intent(c, s, l, r.err, h_leave_intent(vent(s, c, l, subj), r, subj, lt, false, ref, c.now), subj);
      uint32_t len = msg_len(RSF_MSG_LEAVE, lt, 0, 0);
      put_rumor(c, s, rid, RSF_MSG_LEAVE, 0, subj, lt, 0, len);
      pend_push_serial(c, s, l, kQIntent, rid, subj, len, r);
      break;
    }
    case RSF_ACT_FORCE_LEAVE: {
      uint64_t lt = r.clock;
      bool prune = x.flags & 1;
      int f = h_leave_intent(vent(s, c, l, x.subject), r, x.subject, lt, prune, ref, c.now);
      mlog_intent(c, s, l, r.err, f, x.subject);
      if (f & RSF_F_REFUTE) push_refute(c, s, r, ref);
      uint32_t len = msg_len(RSF_MSG_LEAVE, lt, 0, 0);
      put_rumor(c, s, rid, RSF_MSG_LEAVE, prune ? 1 : 0, x.subject, lt, 0, len);
      pend_push_serial(c, s, l, kQIntent, rid, x.subject, len, r);
      break;
    }
    case RSF_ACT_USER_EVENT: {
      uint64_t lt = r.eclock;
      r.eclock++;
      const bool cc = x.flags & 1;
      h_user_event(c, s, l, r, lt, x.key, cc);
      uint32_t len = msg_len(RSF_MSG_USER_EVENT, lt, x.name_len, x.payload_len);
      put_rumor(c, s, rid, RSF_MSG_USER_EVENT, cc ? 1 : 0, 0, lt, x.key, len);
      pend_push_serial(c, s, l, kQEvent, rid, kDecEvent, len, r);
      break;
    }
    case RSF_ACT_QUERY: {
      uint64_t lt = r.qclock;
      bool nb = x.flags & 1;
      h_query(c, s, l, r, lt, (uint32_t)x.key, nb);
      uint32_t len = msg_len(RSF_MSG_QUERY, lt, x.name_len, x.payload_len);
      put_rumor(c, s, rid, RSF_MSG_QUERY, nb ? 1 : 0, 0, lt, (uint32_t)x.key, len);
      pend_push_serial(c, s, l, kQQuery, rid, kDecQuery, len, r);
      break;
    }
    default: break;
  }
  store_regs(s, l, r);
}

// Peer selection (memberlist kRandomNodes model): attempts a = 0,1,2,... in order, each a
// Philox draw over the other N-1 members, kept if live and not yet chosen, until `fanout`
// peers.  One thread per member; grp_key[l*fanout + j] = j-th peer (kSentinel: none, or a
// dead sender).  Sender l's records to its j-th peer form GROUP l*fanout + j.
constexpr uint32_t kPeerBatch = 4;
__global__ void __launch_bounds__(256) peers_kernel(GCfg c, GState s, uint32_t round, uint32_t* __restrict__ grp_key) {
  const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= c.n_loc) return;
  const uint32_t m = (uint32_t)(c.lo + l);
  uint32_t peers[8];
  uint32_t np = 0;
  if (s.alive[m]) {
    const uint32_t attempts = 64 * c.fanout;
    for (uint32_t a0 = 0; a0 < attempts && np < c.fanout; a0 += kPeerBatch) {
      uint32_t p[kPeerBatch];
      bool ok[kPeerBatch];
#pragma unroll
      for (uint32_t b = 0; b < kPeerBatch; ++b) {  // the batch's liveness loads go out together
        u32x4 o = philox4x32_10(a0 + b, kPurposePeer << 24, m, round, c.k0, c.k1);
        p[b] = mulhi32(o.x, (uint32_t)(c.N - 1));
        if (p[b] >= m) p[b]++;
        ok[b] = a0 + b < attempts && s.alive[p[b]] != 0;
      }
#pragma unroll
      for (uint32_t b = 0; b < kPeerBatch; ++b) {
        if (!ok[b] || np >= c.fanout) continue;
        bool dup = false;
        for (uint32_t j = 0; j < np; ++j) dup |= peers[j] == p[b];
        if (!dup) peers[np++] = p[b];
      }
    }
  }
  for (uint32_t j = 0; j < c.fanout; ++j) grp_key[l * c.fanout + j] = j < np ? peers[j] : kSentinel;
}

// After the stable sort of the groups by receiver: slot[gid] = the group's position in
// receiver order (where emit_kernel writes its records: cap_t slots per group), and, for
// a context that merges its own records, each receiver's range of groups.
// Bucket emission (wstart non-null): a group's slot word is its destination shard w (top
// kBktWBits bits) and its place in that shard's bucket (i - wstart[w]), so emission needs
// neither a division nor a dependent load of wstart.
constexpr uint32_t kBktWShift = 26, kBktIdxMask = (1u << kBktWShift) - 1;
__global__ void __launch_bounds__(256) grp_index_kernel(const uint32_t* __restrict__ key_s,
                                                        const uint32_t* __restrict__ id_s, uint64_t n, uint64_t lo,
                                                        uint32_t* __restrict__ slot, uint32_t* __restrict__ seg_start,
                                                        uint32_t* __restrict__ seg_end,
                                                        const uint32_t* __restrict__ wstart = nullptr, uint32_t per = 0,
                                                        uint32_t* __restrict__ bkt_keys = nullptr, uint64_t bstride = 0,
                                                        uint32_t gcap = 0) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = key_s[i];
  if (key == kSentinel) return;
  if (RSF_BAD(2, id_s[i] >= n, id_s[i]) || RSF_BAD(3, seg_start && key - lo >= n, key)) return;
  if (wstart) {
    const uint32_t w = key / per;
    // a place past the field (an overflowing bucket) saturates to kBktIdxMask, which is >= the
    // bucket capacity (rsf_gossip_bucket_buffers), so emission skips it instead of wrapping
    const uint64_t place = (uint64_t)i - wstart[w];
    slot[id_s[i]] = (w << kBktWShift) | (uint32_t)(place < kBktIdxMask ? place : kBktIdxMask);
    // the bucket's receiver keys, in sorted order: coalesced here instead of scattered from
    // the emission (one 4-B write per group into a random sector)
    if (place < gcap) bkt_keys[(uint64_t)w * bstride + place] = key;
    return;
  }
  slot[id_s[i]] = (uint32_t)i;
  if (seg_start) {
    if (i == 0 || key_s[i - 1] != key) seg_start[key - lo] = (uint32_t)i;
    if (i + 1 == n || key_s[i + 1] != key) seg_end[key - lo] = (uint32_t)(i + 1);
  }
}

// ONE WAVE PER SENDER: lane i owns slot i of each of its three queues.  For each peer
// (grp_key, from peers_kernel) broadcast_messages drains intent -> query -> event under
// one byte budget; the group's records (rumor id + decoration) go to cap_t slots at the
// group's sorted position, its record count to cnt_s.
// Members per wave in emit_kernel / merge_kernel: with more than one, a wave issues the
// first round trip of every member it owns before working through them, so the loads
// of the next member are in flight while the current one runs (the kernels run at the
// 8-waves/SIMD hardware cap and wait on memory half the time).
#ifndef RSF_EMIT_WPB
#define RSF_EMIT_WPB 1  // waves per emit_kernel block (1 measured ~1% faster than 2 or 4; 16: +8%)
#endif
#ifndef RSF_EMIT_PER_WAVE
#define RSF_EMIT_PER_WAVE 1  // emit: 2, 8 and 16 per wave measured slower
#endif
#ifndef RSF_MERGE_PER_WAVE
#define RSF_MERGE_PER_WAVE 8  // merge: 8 receivers per wave measured fastest (4.30 -> 4.06 ms at 2M; 2, 4, 16, 32 between)
#endif

// Multi-GPU exchange buckets (rsf_gossip_round_emit_buckets): one bucket per destination
// shard, u32 layout [n_groups, 3 x pad | keys[gcap] | cnt[gcap] | vals[gcap * cap_t] |
// decs[gcap * cap_t]]; the groups of a bucket are sorted by receiver.  On the receive side the world's buckets arrive
// back to back in source-rank order = runs.  The bucket a shard addresses to itself never
// travels: the receive side reads run `self_run` from the send buffer (the receive buffer's
// slot for it is left as it is), so the exchange moves (world - 1) buckets per rank.
// Record decorations travel with the rumor ids (80 B per group of 9 slots instead of 44):
// emission has them in registers, while rebuilding them on the receive side from the
// replicated rumor table cost a random 64-B sector per record -- 0.24 ms per round at 1M
// members in the reference regime, whose picks span millions of rumor ids (the merge looking
// them up itself, a separate pass per slot or per group: all slower).
constexpr uint32_t kMaxRuns = 8;
struct Buckets {
  const uint32_t* base;  // receive buffer (RUNS merge); emission writes through `send`
  uint32_t* send;        // send buffer (emission into buckets)
  const uint32_t* wstart;  // emission: per destination shard, its first group in sorted order
  uint64_t per;            // members per shard
  uint64_t stride_u32;   // one bucket
  uint32_t keys_off, cnt_off, vals_off, decs_off, gcap, n_runs, self_run;
  // run r's bucket on the receive side
  __device__ __forceinline__ const uint32_t* run(uint32_t r) const {
    return (r == self_run ? (const uint32_t*)send : base) + (uint64_t)r * stride_u32;
  }
};

#ifndef RSF_MERGE_PROF
#define RSF_MERGE_PROF 0  // diagnostic build: per-phase shader-clock totals of merge_kernel
#endif
#ifndef RSF_EMIT_PROF
#define RSF_EMIT_PROF 0  // diagnostic build: per-phase shader-clock totals of emit_kernel (same counters)
#endif
#if RSF_MERGE_PROF
#define MPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define MPROF_ADD(i, a, b) \
  if (lane == 0) atomicAdd(&g_merge_prof[i], (unsigned long long)((b) - (a)))
#else
#define MPROF_T(v)
#define MPROF_ADD(i, a, b)
#endif
#if RSF_EMIT_PROF
// phase times accumulate in the wave's own (scalar) registers and go out once at the end,
// spread over 512 counter rows: an atomic on one shared address per phase would make every
// following phase wait for that contended atomic (vmcnt also counts it)
__device__ unsigned long long g_eprof[512 * 8];
__device__ unsigned long long g_eprof2[512 * 8];  // q_pick_peers' own split
#define EPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define EPROF_ADD(i, a, b) ep_acc[i] += (uint64_t)((b) - (a))
#else
#define EPROF_T(v)
#define EPROF_ADD(i, a, b)
#endif

// a sender's first round trip: the intent queue (the common case; a sorted queue is
// empty iff its slot 0 is free), the peers and their group slots, and one lane-distributed
// word per lane (`head`): lanes 1, 2 the query / event queue heads, kEhPend the pending
// re-queue counts, kEhSeq + q the queues' next insertion seqs, kEhPruned, kEhErr
enum : uint32_t { kEhPend = 3, kEhSeq = 4, kEhPruned = 7, kEhErr = 8 };
struct EmitIn {
  QRegs Q0;
  uint32_t head, gk, gs;
  uint4 ts;  // deep queues: lane q < 3 holds queue q's tail summary (tsum)
};
template <uint32_t DEEP = 0>
__device__ __forceinline__ void emit_load(const GCfg& c, const GState& s, const uint32_t* __restrict__ grp_key,
                                          const uint32_t* __restrict__ slot, uint64_t l, uint32_t lane, EmitIn& e) {
  e.Q0 = QRegs{kEmpty, 0, 0};
  e.head = kEmpty;
  e.gk = kSentinel;
  e.gs = 0;
  e.ts = kTSumEmpty;
  if (l >= c.n_loc) return;  // wave-uniform: a wave's last member may lie past the shard
  q_load(c, s, l, 0, lane, e.Q0);
  if (DEEP && lane < 3) e.ts = s.tsum[l * 3 + lane];
  const uint32_t* hp = nullptr;
  if (lane == 1 || lane == 2) hp = s.q_rumor + (l * 3 + lane) * c.qcap;
  else if (lane == kEhPend) hp = s.p_cnt + l;
  else if (lane >= kEhSeq && lane < kEhSeq + 3) hp = s.q_next_seq + l * 3 + (lane - kEhSeq);
  else if (lane == kEhPruned) hp = s.q_pruned + l;
  else if (lane == kEhErr) hp = s.err + l;
  if (hp) e.head = *hp;
  e.gk = lane < c.fanout ? grp_key[l * c.fanout + lane] : kSentinel;
  e.gs = lane < c.fanout ? slot[l * c.fanout + lane] : 0u;
}
// buckets: when nothing will be emitted, lanes < np write their group's zero count into the
// destination bucket (the groups' receiver keys are written by grp_index_kernel, in sorted order)
__device__ __forceinline__ void bkt_zero_counts(const Buckets& bk, uint32_t lane, uint32_t np, uint32_t gs) {
  if (lane >= np) return;
  const uint32_t w = gs >> kBktWShift, idx = gs & kBktIdxMask;  // pre-encoded by grp_index_kernel
  if (idx >= bk.gcap) return;  // over the bucket capacity: flagged by the bounds kernel
  bk.send[(uint64_t)w * bk.stride_u32 + bk.cnt_off + idx] = 0u;
}
// DEEP (queues with an HBM tail): the emission runs on the heads as below; it is committed
// only if every pick was decided by the head alone (q_pick_peers' checks against the tails'
// bounds) and every spill fits its tail -- otherwise nothing is stored (records written to the
// group slots are rewritten) and the member is listed for emit_deep_wave_kernel.
// DEEP: bit q set = queue q may have a tail (1: the intent queue only, 7: all three); the
// other queues' tail code is compiled away
template <bool BKT, uint32_t DEEP = 0>
__device__ __forceinline__ void emit_run(const GCfg& c, const GState& s, uint64_t l, uint32_t lane, EmitIn& e,
                                         uint32_t* __restrict__ cnt_s, uint32_t* __restrict__ out_val,
                                         uint32_t* __restrict__ out_dec, const Buckets& bk, QLds& row) {
#if RSF_EMIT_PROF
  uint64_t ep_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t g_eprof_sub[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // inside q_pick_peers (intent queue)
#endif
  EPROF_T(t0);
  QRegs& Q0 = e.Q0;
  QRegs Q1{kEmpty, 0, 0, kDecQuery}, Q2{kEmpty, 0, 0, kDecEvent};
  const uint64_t pm = ballot(e.gk != kSentinel);  // peers are a prefix of the fanout slots
  const uint32_t np = (uint32_t)__popcll(pm);
  const uint32_t pc = shfl_u32(e.head, kEhPend), npend = pend_total(pc);
  if (RSF_BAD2(8, npend > kPend || ((pc >> 24) != 0), pc)) return;
  // deep queues: a queue is non-empty if its tail holds items too
  constexpr bool D0 = DEEP & 1, D1 = DEEP & 2, D2 = DEEP & 4;
  const uint32_t tc0 = D0 ? shfl_u32(e.ts.x, 0) : 0u, tc1 = D1 ? shfl_u32(e.ts.x, 1) : 0u,
                 tc2 = D2 ? shfl_u32(e.ts.x, 2) : 0u;
  const bool ne0 = shfl_u32(Q0.r, 0) != kEmpty || (pc & 0xFF) || tc0,
             ne1 = shfl_u32(e.head, 1) != kEmpty || ((pc >> 8) & 0xFF) || tc1,
             ne2 = shfl_u32(e.head, 2) != kEmpty || ((pc >> 16) & 0xFF) || tc2;
  // no peers: nothing is sent, and the pending re-queues wait for the next emission
  if (np == 0 || !(ne0 || ne1 || ne2)) {
    if (BKT) bkt_zero_counts(bk, lane, np, e.gs);
    return;
  }
  // (three named tails, not an array: a dynamically indexed array goes to scratch)
  Spill sp0, sp1, sp2;
  bool unsafe = false;
  if (DEEP) {
    auto get = [&](Spill& x, uint32_t q) {
      spill_row(c, s, l, q, x);
      x.cnt = shfl_u32(e.ts.x, q);
      x.minlen = shfl_u32(e.ts.y, q);
      x.minkey = ((uint64_t)shfl_u32(e.ts.w, q) << 32) | shfl_u32(e.ts.z, q);
    };
    if (D0 && c.tcap0) get(sp0, 0);
    if (D1 && c.tcap1) get(sp1, 1);
    if (D2 && c.tcap2) get(sp2, 2);
  }
  EPROF_T(t1);
  EPROF_ADD(0, t0, t1);
  bool d0 = false, d1 = false, d2 = false;
  uint32_t err = 0;
  // the pending re-queues (merge_kernel's and the originations' since the last emission)
  PendRegs pr;
  pend_load(s, l, lane, npend, pr);
  // buckets: each peer's destination shard (the slot word holds the shard and the bucket place)
  uint32_t wdst = 0;
  if (BKT && lane < np) wdst = e.gs >> kBktWShift;
  if (ne1) q_load(c, s, l, 1, lane, Q1);
  if (ne2) q_load(c, s, l, 2, lane, Q2);
#if RSF_EMIT_PROF
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic split: round trip 2 vs the apply
  EPROF_T(t1b);
  EPROF_ADD(1, t1, t1b);
#endif
  uint32_t drops_all = 0;
  if (npend) {
    // applied first: in the reference they were queued when the messages arrived
    uint32_t& drops = drops_all;
    if (pc & 0xFF) {
      if (D0 && c.tcap0) pend_apply<true, true>(c, Q0, lane, 0, npend, pr, shfl_u32(e.head, kEhSeq), row, &sp0);
      else drops += pend_apply<true>(c, Q0, lane, 0, npend, pr, shfl_u32(e.head, kEhSeq), row);
      d0 = true;
    }
    if ((pc >> 8) & 0xFF) {
      if (D1 && c.tcap1) pend_apply<false, true>(c, Q1, lane, 1, npend, pr, shfl_u32(e.head, kEhSeq + 1), row, &sp1);
      else drops += pend_apply<false>(c, Q1, lane, 1, npend, pr, shfl_u32(e.head, kEhSeq + 1), row);
      d1 = true;
    }
    if ((pc >> 16) & 0xFF) {
      if (D2 && c.tcap2) pend_apply<false, true>(c, Q2, lane, 2, npend, pr, shfl_u32(e.head, kEhSeq + 2), row, &sp2);
      else drops += pend_apply<false>(c, Q2, lane, 2, npend, pr, shfl_u32(e.head, kEhSeq + 2), row);
      d2 = true;
    }
    if (drops) err |= kErrQueue;
    // a tail past its capacity needs the bounded queue's exact prune over head and tail
    if (DEEP) unsafe = (D0 && sp0.cnt > c.tcap0) || (D1 && sp1.cnt > c.tcap1) || (D2 && sp2.cnt > c.tcap2);
    if (DEEP && unsafe) RSF_DEEP_WHY(6);
    // (the list's bookkeeping -- count, next seqs, prune count -- is written at the end: a store
    // here would make the compiler wait for it before reusing its registers)
  }
  EPROF_T(t2);
#if RSF_EMIT_PROF
  EPROF_ADD(2, t1b, t2);
#endif
  {
    // queue-major: every peer's picks from the intent queue, then the query queue, then the
    // event queue (q_pick_peers).  Lane j < np holds peer j's group: where its records go
    // (off: element offset from the output base) and where its count goes (oc).
    if (RSF_BAD2_W(7, !BKT && lane < np && e.gs >= c.n_loc * c.fanout, e.gs)) return;
    uint64_t off = ~0ull;
    uint32_t* ov = out_val;
    uint32_t* od = out_dec;
    uint32_t* oc = nullptr;
    if (lane < np) {
      if (BKT) {
        const uint32_t idx = e.gs & kBktIdxMask;
        if (idx < bk.gcap) {
          off = (uint64_t)wdst * bk.stride_u32 + bk.vals_off + (uint64_t)idx * c.cap_t;
          oc = bk.send + (uint64_t)wdst * bk.stride_u32 + bk.cnt_off + idx;
        }
      } else {
        off = (uint64_t)e.gs * c.cap_t;
        oc = cnt_s + e.gs;
      }
    }
    if (BKT) {
      ov = bk.send;
      od = bk.send + (bk.decs_off - bk.vals_off);  // (off addresses the vals: the decs sit a fixed distance on)
    }
    uint32_t used_v = 0, nrec_v = 0;
#if RSF_EMIT_PROF
    uint64_t* const ep = g_eprof_sub;
#else
    uint64_t* const ep = nullptr;
#endif
    if (DEEP) {
      // a tail's bounds (~0: empty) as of after the spills above
#define RSF_TB(q) (sp##q.cnt ? sp##q.minkey : ~0ull), (sp##q.cnt ? sp##q.minlen : ~0u)
      if (ne0 && !unsafe) {
        if (D0) q_pick_peers<true, true>(c, Q0, lane, np, used_v, nrec_v, off, ov, od, err, d0, row, ep, RSF_TB(0), &unsafe);
        else q_pick_peers<true>(c, Q0, lane, np, used_v, nrec_v, off, ov, od, err, d0, row, ep);
      }
      if (ne1 && !unsafe) {
        if (D1) q_pick_peers<false, true>(c, Q1, lane, np, used_v, nrec_v, off, ov, od, err, d1, row, nullptr, RSF_TB(1), &unsafe);
        else q_pick_peers<false>(c, Q1, lane, np, used_v, nrec_v, off, ov, od, err, d1, row);
      }
      if (ne2 && !unsafe) {
        if (D2) q_pick_peers<false, true>(c, Q2, lane, np, used_v, nrec_v, off, ov, od, err, d2, row, nullptr, RSF_TB(2), &unsafe);
        else q_pick_peers<false>(c, Q2, lane, np, used_v, nrec_v, off, ov, od, err, d2, row);
      }
#undef RSF_TB
      if (unsafe) {  // nothing committed: the whole-queue path redoes this member's emission
        // by the LDS capacity its largest queue needs: list 2 (kDeepTiny; from n_loc), list 0
        // (kDeepSmall; from the front), list 3 (kDeepMid; from 3 n_loc), list 1 (the full depth;
        // from 3 n_loc - 1 down)
        uint32_t need = c.qcap + max(max(tc0 + (pc & 0xFF), tc1 + ((pc >> 8) & 0xFF)), tc2 + ((pc >> 16) & 0xFF));
        // only the intent queue in use with a sealed tail prefix: the deferred path reads the
        // tail's recent part only (deep_wave_member's recent mode; it re-lists the member for the
        // full depth if that cannot decide)
        if (D0 && c.tcap0 && !ne1 && !ne2 && tc0 + (pc & 0xFF) <= c.tcap0) {
          const uint32_t m0 = s.tseal[l * 3].x;
          if (m0 && m0 <= tc0) need = c.qcap + (tc0 - m0) + (pc & 0xFF);
        }
        if (lane == 0) {
          if (need <= kDeepTiny) s.deep_ids[c.n_loc + atomicAdd(s.deep_n + 2, 1u)] = (uint32_t)l;
          else if (need <= kDeepSmall) s.deep_ids[atomicAdd(s.deep_n, 1u)] = (uint32_t)l;
          else if (need <= kDeepMid) s.deep_ids[c.n_loc * 3 + atomicAdd(s.deep_n + 3, 1u)] = (uint32_t)l;
          else s.deep_ids[c.n_loc * 3 - 1 - atomicAdd(s.deep_n + 1, 1u)] = (uint32_t)l;
        }
        return;
      }
    } else {
      if (ne0) q_pick_peers<true>(c, Q0, lane, np, used_v, nrec_v, off, ov, od, err, d0, row, ep);
      if (ne1) q_pick_peers<false>(c, Q1, lane, np, used_v, nrec_v, off, ov, od, err, d1, row);
      if (ne2) q_pick_peers<false>(c, Q2, lane, np, used_v, nrec_v, off, ov, od, err, d2, row);
    }
    if (oc && (BKT || nrec_v)) *oc = min(nrec_v, c.cap_t);  // buckets: every group's count
  }
  EPROF_T(t2b);
  EPROF_ADD(3, t2, t2b);
  EPROF_T(t3);
  EPROF_ADD(4, t2b, t3);
  if (d0) q_store(c, s, l, 0, lane, Q0, true);
  if (d1) q_store(c, s, l, 1, lane, Q1, true);
  if (d2) q_store(c, s, l, 2, lane, Q2, true);
  if (DEEP) {  // the tails' new counts and bounds (their spilled items are written), lane q for queue q
    const bool l0 = lane == 0, l1 = lane == 1;
    const uint32_t tc = l0 ? tc0 : l1 ? tc1 : tc2;
    const uint32_t tcap = l0 ? (D0 ? c.tcap0 : 0u) : l1 ? (D1 ? c.tcap1 : 0u) : (D2 ? c.tcap2 : 0u);
    const uint32_t cnt = l0 ? sp0.cnt : l1 ? sp1.cnt : sp2.cnt, mlen = l0 ? sp0.minlen : l1 ? sp1.minlen : sp2.minlen;
    const uint64_t mkey = l0 ? sp0.minkey : l1 ? sp1.minkey : sp2.minkey;
    if (lane < 3 && tcap && cnt != tc) s.tsum[l * 3 + lane] = make_uint4(cnt, mlen, (uint32_t)mkey, (uint32_t)(mkey >> 32));
  }
  // the member's bookkeeping as ONE lane-distributed store (each lane of `head` writes its own
  // word back where it changed): the applied pending list's count (0) and the queues' next
  // seqs, the prune count, the error flags (a queue prune, a stage overflow; only when new)
  {
    const uint32_t qi = lane - kEhSeq;
    const uint32_t nq = qi < 3 ? (pc >> (8 * qi)) & 0xFF : 0u;
    const bool w_pend = npend && lane == kEhPend, w_seq = npend && nq != 0;
    const bool w_pr = drops_all && lane == kEhPruned, w_err = lane == kEhErr && (err & ~e.head);
    uint32_t* const base = w_pend ? s.p_cnt : w_seq ? s.q_next_seq : w_pr ? s.q_pruned : s.err;
    const uint64_t idx = w_seq ? l * 3 + qi : l;
    const uint32_t v = w_pend ? 0u : w_seq ? e.head + nq : w_pr ? e.head + drops_all : (e.head | err);
    if (w_pend || w_seq || w_pr || w_err) base[idx] = v;
  }

  EPROF_T(t4);
  EPROF_ADD(7, t3, t4);
  EPROF_ADD(5, t0, t4);
#if RSF_EMIT_PROF
  ep_acc[6] = 1;
  if (lane == 0)
    for (int i = 0; i < 8; ++i)
      if (ep_acc[i]) atomicAdd(&g_eprof[(blockIdx.x & 511) * 8 + i], (unsigned long long)ep_acc[i]);
  if (lane == 0)
    for (int i = 0; i < 5; ++i)
      if (g_eprof_sub[i]) atomicAdd(&g_eprof2[(blockIdx.x & 511) * 8 + i], (unsigned long long)g_eprof_sub[i]);
#endif
}

// emission for queues of 65..256 slots (gossip_queue4.h): emit_run's steps with four slots
// per lane; no prefetch of the next sender and no deferred re-rank
template <bool BKT>
__device__ __forceinline__ void emit_run4(const GCfg& c, const GState& s, const uint32_t* __restrict__ grp_key,
                                          const uint32_t* __restrict__ slot, uint64_t l, uint32_t lane,
                                          uint32_t* __restrict__ cnt_s, uint32_t* __restrict__ out_val,
                                          uint32_t* __restrict__ out_dec, const Buckets& bk, QLds4& row) {
  // one lane-distributed word (emit_load's `head`, lane 0 = the intent queue's slot 0)
  const uint32_t* hp = nullptr;
  if (lane < 3) hp = s.q_rumor + (l * 3 + lane) * c.qcap;
  else if (lane == kEhPend) hp = s.p_cnt + l;
  else if (lane >= kEhSeq && lane < kEhSeq + 3) hp = s.q_next_seq + l * 3 + (lane - kEhSeq);
  else if (lane == kEhPruned) hp = s.q_pruned + l;
  else if (lane == kEhErr) hp = s.err + l;
  const uint32_t head = hp ? *hp : kEmpty;
  const uint32_t gk = lane < c.fanout ? grp_key[l * c.fanout + lane] : kSentinel;
  const uint32_t gs = lane < c.fanout ? slot[l * c.fanout + lane] : 0u;
  const uint32_t np = (uint32_t)__popcll(ballot(gk != kSentinel));
  const uint32_t pc = shfl_u32(head, kEhPend), npend = pend_total(pc);
  const bool ne0 = shfl_u32(head, 0) != kEmpty || (pc & 0xFF), ne1 = shfl_u32(head, 1) != kEmpty || ((pc >> 8) & 0xFF),
             ne2 = shfl_u32(head, 2) != kEmpty || ((pc >> 16) & 0xFF);
  if (np == 0 || !(ne0 || ne1 || ne2)) {
    if (BKT) bkt_zero_counts(bk, lane, np, gs);
    return;
  }
  bool d0 = false, d1 = false, d2 = false;
  uint32_t err = 0;
  PendRegs pr;
  pend_load(s, l, lane, npend, pr);
  uint32_t wdst = 0;
  if (BKT && lane < np) wdst = gs >> kBktWShift;
  Q4 Q0, Q1, Q2;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    Q0.r[k] = Q1.r[k] = Q2.r[k] = kEmpty;
    Q0.sq[k] = Q1.sq[k] = Q2.sq[k] = Q0.tl[k] = Q1.tl[k] = Q2.tl[k] = 0;
    Q0.dec[k] = 0;
    Q1.dec[k] = kDecQuery;
    Q2.dec[k] = kDecEvent;
  }
  if (ne0) q4_load(c, s, l, 0, lane, Q0);
  if (ne1) q4_load(c, s, l, 1, lane, Q1);
  if (ne2) q4_load(c, s, l, 2, lane, Q2);
  if (npend) {
    uint32_t drops = 0;
    if (pc & 0xFF) {
      drops += q4_pend_apply<true>(c, Q0, lane, 0, npend, pr, shfl_u32(head, kEhSeq), row);
      d0 = true;
    }
    if ((pc >> 8) & 0xFF) {
      drops += q4_pend_apply<false>(c, Q1, lane, 1, npend, pr, shfl_u32(head, kEhSeq + 1), row);
      d1 = true;
    }
    if ((pc >> 16) & 0xFF) {
      drops += q4_pend_apply<false>(c, Q2, lane, 2, npend, pr, shfl_u32(head, kEhSeq + 2), row);
      d2 = true;
    }
    if (lane == kEhPend) s.p_cnt[l] = 0;
    if (lane >= kEhSeq && lane < kEhSeq + 3) {
      const uint32_t nq = (pc >> (8 * (lane - kEhSeq))) & 0xFF;
      if (nq) s.q_next_seq[l * 3 + (lane - kEhSeq)] = head + nq;
    }
    if (drops) {
      if (lane == kEhPruned) s.q_pruned[l] = head + drops;
      err |= kErrQueue;
    }
  }
  {
    // queue-major, as emit_run: every peer's picks from each queue in one pass (q4_pick_peers)
    uint64_t off = ~0ull;
    uint32_t* ov = out_val;
    uint32_t* od = out_dec;
    uint32_t* oc = nullptr;
    if (lane < np) {
      if (BKT) {
        const uint32_t idx = gs & kBktIdxMask;
        if (idx < bk.gcap) {
          off = (uint64_t)wdst * bk.stride_u32 + bk.vals_off + (uint64_t)idx * c.cap_t;
          oc = bk.send + (uint64_t)wdst * bk.stride_u32 + bk.cnt_off + idx;
        }
      } else {
        off = (uint64_t)gs * c.cap_t;
        oc = cnt_s + gs;
      }
    }
    if (BKT) {
      ov = bk.send;
      od = bk.send + (bk.decs_off - bk.vals_off);
    }
    uint32_t used_v = 0, nrec_v = 0;
    if (ne0) q4_pick_peers<true>(c, Q0, lane, np, used_v, nrec_v, off, ov, od, err, d0, row);
    if (ne1) q4_pick_peers<false>(c, Q1, lane, np, used_v, nrec_v, off, ov, od, err, d1, row);
    if (ne2) q4_pick_peers<false>(c, Q2, lane, np, used_v, nrec_v, off, ov, od, err, d2, row);
    if (oc && (BKT || nrec_v)) *oc = min(nrec_v, c.cap_t);
  }
  if (d0) q4_store(c, s, l, 0, lane, Q0);
  if (d1) q4_store(c, s, l, 1, lane, Q1);
  if (d2) q4_store(c, s, l, 2, lane, Q2);
  if (lane == kEhErr && (err & ~head)) s.err[l] = head | err;
}

template <bool BKT>
__global__ void __launch_bounds__(64) emit4_kernel(GCfg c, GState s, const uint32_t* __restrict__ grp_key,
                                                   const uint32_t* __restrict__ slot, uint32_t* __restrict__ cnt_s,
                                                   uint32_t* __restrict__ out_val, uint32_t* __restrict__ out_dec,
                                                   Buckets bk) {
  __shared__ QLds4 row;
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t l = blockIdx.x;
  if (l >= c.n_loc) return;
  emit_run4<BKT>(c, s, grp_key, slot, l, lane, cnt_s, out_val, out_dec, bk, row);
}

// FULL: queue_cap == 64 (one slot per lane of the wave), known at compile time -- every
// `lane < qcap` test and its branch fold away (the bench configuration)
#ifndef RSF_EMIT_DEEP_SGPR
#define RSF_EMIT_DEEP_SGPR 94  // SGPR cap for the deep emission: occupancy 8 instead of 7 (11 SGPRs spilled to VGPR lanes; 1.45 -> 1.40 ms at 1M, same box x2); 0: none
#endif
template <bool BKT, bool FULL, uint32_t DEEP>
__device__ __forceinline__ void emit_body(GCfg c, const GState& s, const uint32_t* __restrict__ grp_key,
                                          const uint32_t* __restrict__ slot, uint32_t* __restrict__ cnt_s,
                                          uint32_t* __restrict__ out_val, uint32_t* __restrict__ out_dec,
                                          const Buckets& bk) {
  if (FULL) c.qcap = kWave;
  __shared__ QLds rows[RSF_EMIT_WPB];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  QLds& row = rows[threadIdx.x / kWave];
  const uint64_t l = ((uint64_t)xcd_block(blockIdx.x, gridDim.x) * RSF_EMIT_WPB +
                      (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave)) * RSF_EMIT_PER_WAVE;
  if (l >= c.n_loc) return;
  EmitIn cur, nxt;
  emit_load<DEEP>(c, s, grp_key, slot, l, lane, cur);
  if (RSF_EMIT_PER_WAVE == 1) {
    emit_run<BKT, DEEP>(c, s, l, lane, cur, cnt_s, out_val, out_dec, bk, row);
    return;
  }
  for (uint32_t k = 0; k < RSF_EMIT_PER_WAVE; ++k) {
    if (k + 1 < RSF_EMIT_PER_WAVE) emit_load<DEEP>(c, s, grp_key, slot, l + k + 1, lane, nxt);
    if (l + k < c.n_loc) emit_run<BKT, DEEP>(c, s, l + k, lane, cur, cnt_s, out_val, out_dec, bk, row);
    cur = nxt;
  }
}
template <bool BKT, bool FULL>
__global__ void __launch_bounds__(64 * RSF_EMIT_WPB) emit_kernel(GCfg c, GState s, const uint32_t* __restrict__ grp_key,
                                                                 const uint32_t* __restrict__ slot,
                                                                 uint32_t* __restrict__ cnt_s,
                                                                 uint32_t* __restrict__ out_val,
                                                                 uint32_t* __restrict__ out_dec, Buckets bk) {
  emit_body<BKT, FULL, 0>(c, s, grp_key, slot, cnt_s, out_val, out_dec, bk);
}
// deep queues (DEEP: the queues with a tail, bit q)
template <bool BKT, bool FULL, uint32_t DEEP>
__global__ void __launch_bounds__(64 * RSF_EMIT_WPB)
#if RSF_EMIT_DEEP_SGPR
    __attribute__((amdgpu_num_sgpr(RSF_EMIT_DEEP_SGPR)))
#endif
    emit_kernel_deep(GCfg c, GState s, const uint32_t* __restrict__ grp_key, const uint32_t* __restrict__ slot,
                     uint32_t* __restrict__ cnt_s, uint32_t* __restrict__ out_val, uint32_t* __restrict__ out_dec,
                     Buckets bk) {
  emit_body<BKT, FULL, DEEP>(c, s, grp_key, slot, cnt_s, out_val, out_dec, bk);
}

}  // namespace
#include "gossip_deep.h"
namespace {

// Record decoration: what merge_kernel needs to address the view entry (the
// subject) and to pick the queue, written beside the sorted rumor ids so the
// merge issues its view-entry load in the same round trip as the rumor-body
// load instead of after it.
__device__ __forceinline__ uint32_t decorate(const rsf_rumor* __restrict__ rumors, uint32_t rid) {
  // subject and type share one aligned 8-B word (offset 16): one load, no dependent second one
  static_assert(offsetof(rsf_rumor, subject) == 16 && offsetof(rsf_rumor, type) == 20, "rumor layout");
  const uint2 w = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(rumors + rid) + 16);
  const uint8_t t = (uint8_t)w.y;
  if (t == RSF_MSG_QUERY) return kDecQuery;
  if (t == RSF_MSG_USER_EVENT) return kDecEvent;
  return w.x;
}

// The round's rumor block decorated once into a dense 4-B table (rdec): emission and the
// receive side look a record's decoration up there instead of in the 24-B rumor bodies,
// a table 6x denser in L2 / Infinity Cache.  Run after the block is complete (after the
// all-reduce on the multi-GPU path).
// The same pass keeps the rumor bodies without their 8-B key (only user events and
// queries need it) as aligned 16-B records for the merge kernel's gather.
__global__ void __launch_bounds__(256) dec_fill_kernel(const rsf_rumor* __restrict__ rumors, uint32_t* __restrict__ rdec,
                                                       uint4* __restrict__ rbody, uint64_t base, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  rdec[base + i] = decorate(rumors, (uint32_t)(base + i));
  const uint2* w = reinterpret_cast<const uint2*>(rumors + base + i);  // ltime | key | subject..msg_len
  const uint2 lt = w[0], tail = w[2];
  rbody[base + i] = make_uint4(lt.x, lt.y, tail.x, tail.y);
}
// a rumor rebuilt from its 16-B body (+ the key when the record needs it)
__device__ __forceinline__ rsf_rumor rumor_from_body(uint4 b, uint64_t key) {
  rsf_rumor ru;
  ru.ltime = ((uint64_t)b.y << 32) | b.x;
  ru.key = key;
  ru.subject = b.z;
  ru.type = (uint8_t)(b.w & 0xFF);
  ru.flags = (uint8_t)((b.w >> 8) & 0xFF);
  ru.msg_len = (uint16_t)(b.w >> 16);
  return ru;
}

// segment bounds per receiver + record decoration (keys == nullptr: decoration only)
__global__ void __launch_bounds__(256) segment_kernel(const uint32_t* __restrict__ keys, uint64_t n, uint64_t lo,
                                                      uint32_t* __restrict__ seg_start, uint32_t* __restrict__ seg_end,
                                                      const uint32_t* __restrict__ vals,
                                                      const uint32_t* __restrict__ rdec,
                                                      uint32_t* __restrict__ dec, uint32_t rmask) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k = keys[i];
  if (k == kSentinel) return;
  if (i == 0 || keys[i - 1] != k) seg_start[k - lo] = (uint32_t)i;
  if (i + 1 == n || keys[i + 1] != k) seg_end[k - lo] = (uint32_t)(i + 1);
  if (dec) dec[i] = rdec[vals[i] & rmask];
}

// ---- multi-GPU send side: the records of the receiver-sorted groups (cap_t slots each,
// cnt[i] used) compacted into one receiver-ordered record stream [end[i-1], end[i])
// (end = inclusive scan of cnt); the last valid group publishes the record count.
// kLanesPerGroup lanes per group, one record per lane.
constexpr uint32_t kLanesPerGroup = 16;
// The records go out packed as (receiver << 32 | rumor id): the exchange's send format.
__global__ void __launch_bounds__(256) grp_expand_kernel(const uint32_t* __restrict__ key_s,
                                                         const uint32_t* __restrict__ end, uint64_t n,
                                                         uint32_t cap_t, const uint32_t* __restrict__ slots,
                                                         uint64_t* __restrict__ out, unsigned long long* n_valid) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i = t / kLanesPerGroup;
  const uint32_t sub = (uint32_t)t % kLanesPerGroup;
  if (i >= n) return;
  const uint32_t key = key_s[i];
  if (key == kSentinel) return;
  const uint32_t o = i ? end[i - 1] : 0u, e = end[i];
  const uint32_t* src = slots + i * cap_t;
  for (uint32_t k = sub; o + k < e; k += kLanesPerGroup) out[o + k] = ((uint64_t)key << 32) | src[k];
  if (sub == 0 && (i + 1 == n || key_s[i + 1] == kSentinel)) *n_valid = e;
}

// One wave per receiver, lane = record.  Records arrive in canonical
// (sender, position) order in [seg_start, seg_end); a chunk of up to 64 is
// prefetched lane-parallel (rumor id, rumor body, the receiver's view entry of
// the subject).  The intent handlers then run IN PARALLEL across lanes:
//   * LamportClock::witness(t) is c = max(c, t+1), associative, so the clock a
//     record sees is an exclusive prefix max over earlier intents (DPP scan);
//   * records about the same subject form a chain (prev/next lane); chains are
//     walked in depth order, each link taking its predecessor's output entry;
//   * digest contributions (member events, deliveries), refutations and
//     re-queues are then applied serially in record order.
// User events / queries (dedup rings in HBM) run serially in lane 0.
// the merge's record streams are read once per round
__device__ __forceinline__ uint32_t rec_ld(const uint32_t* p) {
  return *p;
}
#ifndef RSF_MERGE_WAVES
#define RSF_MERGE_WAVES 7  // min waves/SIMD for merge_kernel (register cap; 7 measured fastest with 8 receivers per wave, 8 before)
#endif
#ifndef RSF_MERGE_CHAIN_BY_SUBJECT
#define RSF_MERGE_CHAIN_BY_SUBJECT 1  // 1: chain detection loops over distinct subjects, not records
#endif
// What a receiver's merge needs before its records: segment bounds, liveness, the pending
// re-queue counts and the member's registers, issued a receiver AHEAD (merge_kernel)
// as ONE lane-distributed load: lane j fetches dword j of the setup (kSu* below) from its
// own array, so the prefetch holds one vector register until merge_one reads the fields
// out with readlane.
enum : uint32_t {
  kSuStart, kSuEnd, kSuAlive, kSuPend, kSuClock, kSuEClock = kSuClock + 2,
  kSuQClock = kSuEClock + 2, kSuEMin = kSuQClock + 2, kSuQMin = kSuEMin + 2, kSuDigest = kSuQMin + 2,
  kSuErr = kSuDigest + 2, kSuSerf, kSuSubj, kSuRun,  // kSuRun + 2r, + 2r + 1: run r's groups
  kSuLanes = kSuRun + 2 * kMaxRuns
};
// per-lane source: byte address = base + l * mult + off (alive / serf_state: the aligned
// dword holding the byte)
struct MSetupLane {
  const char* base;
  uint32_t mult, off;
};
__device__ __forceinline__ MSetupLane merge_setup_lane(const GCfg& c, const GState& s,
                                                       const uint32_t* __restrict__ seg_start,
                                                       const uint32_t* __restrict__ seg_end, uint32_t lane,
                                                       uint32_t n_runs) {
  const char* b = (const char*)seg_start;
  uint32_t mult = 4, off = 0;
  if (lane == kSuEnd) b = (const char*)seg_end;
  // bucket input: seg_start / seg_end are [run][n_loc] group ranges
  if (lane >= kSuRun && lane < kSuRun + 2 * n_runs) {
    const uint32_t r = (lane - kSuRun) >> 1;
    b = (const char*)((lane - kSuRun) & 1 ? seg_end : seg_start);
    off = (uint32_t)(r * c.n_loc * 4);
  }
  if (lane == kSuAlive) b = (const char*)s.alive + c.lo, mult = 1;
  if (lane == kSuPend) b = (const char*)s.p_cnt;
  const uint64_t* u64s[6] = {s.clock, s.eclock, s.qclock, s.emin, s.qmin, s.digest};
#pragma unroll
  for (uint32_t k = 0; k < 6; ++k)
    if (lane == kSuClock + 2 * k || lane == kSuClock + 2 * k + 1)
      b = (const char*)u64s[k], mult = 8, off = 4 * (lane - kSuClock - 2 * k);
  if (lane == kSuErr) b = (const char*)s.err;
  if (lane == kSuSerf) b = (const char*)s.serf_state, mult = 1;
  if (lane == kSuSubj) b = (const char*)s.member_subj;
  return MSetupLane{b, mult, off};
}
__device__ __forceinline__ uint32_t merge_setup(const MSetupLane& sl, uint64_t l, uint32_t lane) {
  uint32_t v = 0;
  if (lane < kSuLanes && sl.base) {
    const uintptr_t a = (uintptr_t)(sl.base + l * sl.mult + sl.off);
    // a global (not flat) load: flat loads also count on lgkmcnt, which every ds_bpermute
    // wait of the current receiver would then drain
    v = *(const __attribute__((address_space(1))) uint32_t*)(a & ~(uintptr_t)3);
    v >>= 8 * (uint32_t)(a & 3);  // byte fields: shift the byte down
  }
  return v;
}
__device__ __forceinline__ uint64_t su64(uint32_t v, uint32_t k) {
  return ((uint64_t)shfl_u32(v, k + 1) << 32) | shfl_u32(v, k);
}

// One receiver (one wave).  Input layouts: flat (gcnt == nullptr, stride 1): records
// [seg_start, seg_end) in canonical order; grouped (emit_kernel's): groups [seg_start,
// seg_end) of `stride` slots each, group g holding gcnt[g] records, so lane = slot and the
// empty slots of a group are holes (invalid lanes) in an otherwise canonical lane order.
// Re-queues go to the member's pending list (applied at its next emission); the merge
// never reads or writes the queues themselves, except to apply a list that would overflow.
// Receivers whose pending list might overflow during the merge (pending + slots > kPend)
// are not merged by merge_kernel: they go to a list that merge_big_kernel works through
// afterwards with the in-merge list application compiled in (BIG), which the common path
// then need not carry (its registers).  Receivers are independent, so the order is free.
struct BigList {
  uint32_t* ids;            // [n_loc]
  unsigned long long* n;    // count (reset before each merge)
};
template <bool RUNS, bool BIG>
__device__ __forceinline__ void merge_one(const GCfg& c, const GState& s, const uint32_t* __restrict__ vals,
                                          const uint32_t* __restrict__ dec, const uint32_t* __restrict__ gcnt,
                                          uint32_t stride, uint64_t l, uint32_t lane, uint32_t su, QLds4* row,
                                          uint32_t* __restrict__ sbits, const Buckets& bk, const BigList& big) {
  MPROF_T(t_start);
  uint32_t st = 0, en = 0, total;
  uint32_t rcum[kMaxRuns + 1], rst[kMaxRuns];  // runs: cumulative slots, first group per run
  if (RUNS) {
    rcum[0] = 0;
#pragma unroll
    for (uint32_t r = 0; r < kMaxRuns; ++r) {
      const uint32_t a = r < bk.n_runs ? shfl_u32(su, kSuRun + 2 * r) : 0u;
      const uint32_t b = r < bk.n_runs ? shfl_u32(su, kSuRun + 2 * r + 1) : 0u;
      rst[r] = a;
      rcum[r + 1] = rcum[r] + (b - a) * stride;
    }
    total = rcum[kMaxRuns];
  } else {
    st = shfl_u32(su, kSuStart);
    en = shfl_u32(su, kSuEnd);
    if (RSF_BAD2(10, st > en || en > c.n_loc * c.fanout, ((uint64_t)st << 32) | en)) return;
    total = st < en ? (en - st) * stride : 0u;
  }
  if (total == 0 || (shfl_u32(su, kSuAlive) & 0xFF) == 0) return;
  // pending re-queues: packed per-queue counts and their total (wave-uniform)
  const uint32_t pc0 = shfl_u32(su, kSuPend);
  uint32_t pc = pc0, pn = pend_total(pc0);
  if (RSF_BAD2(12, pn > kPend || (pc0 >> 24) != 0, pc0)) return;
  if (!BIG && pn + total > kPendMerge) {  // at most one re-queue per record slot: might not fit
    if (lane == 0) big.ids[atomicAdd(big.n, 1ull)] = (uint32_t)l;
    return;
  }
  uint32_t qdrop = 0;  // live queue items dropped by full queues (a list applied here)
  GState::PendE* const p_ent = s.p_ent + l * kPend;
  MRegs r;
  r.clock = su64(su, kSuClock);
  r.eclock = su64(su, kSuEClock);
  r.qclock = su64(su, kSuQClock);
  r.emin = su64(su, kSuEMin);
  r.qmin = su64(su, kSuQMin);
  r.digest = su64(su, kSuDigest);
  r.err = shfl_u32(su, kSuErr);
  r.serf_state = (uint8_t)shfl_u32(su, kSuSerf);
  r.subj = (int32_t)shfl_u32(su, kSuSubj);
  ViewS* vrow = vrow_of(s, c, l);
  MPROF_T(t_setup);
  MPROF_ADD(0, t_start, t_setup);
  const uint64_t vs = (uint64_t)st * stride;
  for (uint32_t vb = 0; vb < total; vb += kWave) {
    MPROF_T(t_c0);
    const uint32_t cnt = min((uint32_t)kWave, total - vb);  // lanes in this chunk
    if (BIG && pn + cnt > kPendMerge) {
      // the chunk's re-queues (at most one per record) might not fit the pending list:
      // apply the list to the queues first (rare: a receiver of many records)
      __threadfence_block();
      qdrop += pend_flush_any(c, s, l, lane, pc, *row);
      pc = pn = 0;
    }
    const bool in = lane < cnt;
    const uint32_t vi = vb + lane;  // this lane's slot in the receiver's slot list
    uint32_t rid0 = 0, dsub0 = kEmpty, gk = 1, gc = 1;
    if (RUNS) {
      // the run holding slot v, then its group and place in the group
      uint32_t r = 0;
#pragma unroll
      for (uint32_t q = 1; q < kMaxRuns; ++q) r = vi >= rcum[q] ? q : r;
      uint32_t cr = 0, sr = 0;
#pragma unroll
      for (uint32_t q = 0; q < kMaxRuns; ++q) {
        cr = q == r ? rcum[q] : cr;
        sr = q == r ? rst[q] : sr;
      }
      const uint32_t rel = vi - cr, gr = rel / stride;
      gk = rel - gr * stride;
      const uint64_t g = (uint64_t)sr + gr;
      const uint32_t* b = bk.run(r);
      if (in) {
        rid0 = rec_ld(b + bk.vals_off + g * stride + gk);
        dsub0 = rec_ld(b + bk.decs_off + g * stride + gk);
        gc = rec_ld(b + bk.cnt_off + g);
      }
    } else {
      // slot contents and the group's record count in one round trip (holes read stale ids)
      const uint64_t slot = vs + vi;
      if (RSF_BAD_W(6, in && slot >= (uint64_t)c.n_loc * c.fanout * c.cap_t, slot)) return;
      rid0 = in ? rec_ld(vals + slot) : 0;
      if (gcnt) {
        // group of the slot relative to the receiver's first group: a 32-bit division
        // (a receiver's slot range is small) instead of a 64-bit one
        const uint32_t gr = vi / stride;
        if (RSF_BAD2_W(9, in && (uint64_t)st + gr >= c.n_loc * c.fanout, st + gr)) return;
        if (in) {
          gk = vi - gr * stride;
          gc = rec_ld(gcnt + st + gr);
        }
      }
      // decoration (same round trip as the rumor ids): subject of an intent, or the
      // queue of an event / query; invalid lanes read as neither
      dsub0 = in ? rec_ld(dec + slot) : kEmpty;
    }
    const bool valid = in && (!(RUNS || gcnt) || gk < gc);
    const uint32_t rid = valid ? rid0 : 0;
    const uint32_t dsub = valid ? dsub0 : kEmpty;
    const bool is_view = dsub < kDecViewMax && !RSF_BAD(4, dsub < kDecViewMax && dsub >= c.S, dsub);
    rsf_rumor ru{};
    if (valid) {  // the key only for user events / queries (the decoration says which)
      const uint4 b = s.rbody[rid & c.rmask];
      const uint64_t key = (dsub == kDecQuery || dsub == kDecEvent) ? s.rumors[rid & c.rmask].key : 0ull;
      ru = rumor_from_body(b, key);
    }
    ViewE pre{};
    if (is_view) pre = *view_at(vrow, dsub);  // issued beside the rumor-body load (a non-temporal load measured far slower)
    const uint32_t my_subj = is_view ? dsub : 0xFFFFFFFFu;
    // chains: previous / next record of the same subject in this chunk
    int prev = -1, next = -1;
#if RSF_MERGE_CHAIN_BY_SUBJECT
    // fast path: chunk subjects hashed into the wave's 4096-bit LDS map; no clash means
    // every subject is distinct in the chunk, so there are no chains to link
    bool clash = false;
    if (is_view) {
      const uint32_t h = my_subj & 4095u;
      const uint32_t old = atomicOr(sbits + (h >> 5), 1u << (h & 31));
      clash = (old >> (h & 31)) & 1u;
      sbits[h >> 5] = 0u;  // LDS ops of a wave run in order: every lane's OR has returned
    }
    if (ballot(clash)) {
      // one pass per DISTINCT subject: the ballot of the lanes holding it is the chain,
      // each lane's neighbours are the nearest set bits below and above it
      uint64_t mm = ballot(is_view), same = 0;
      while (mm) {
        const uint32_t sj = shfl_u32(my_subj, __ffsll((long long)mm) - 1);
        const bool hit = my_subj == sj;  // non-view lanes hold 0xFFFFFFFF, never a subject
        const uint64_t grp = ballot(hit);
        if (hit) same = grp;
        mm &= ~grp;
      }
      const uint64_t below = same & ((1ull << lane) - 1), above = same & ~((2ull << lane) - 1);
      prev = below ? 63 - __clzll((long long)below) : -1;
      next = above ? __ffsll((long long)above) - 1 : -1;
    }
#else
    {
      const uint64_t vmask = ballot(is_view);
      uint64_t mm = vmask;
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const uint32_t sj = shfl_u32(my_subj, j);
        if (is_view && sj == my_subj) {
          if (j < (int)lane) prev = j;
          if (j > (int)lane && next < 0) next = j;
        }
      }
    }
#endif
    // Lamport clock each intent record witnesses against: exclusive prefix max
    const uint64_t wit = is_view ? ru.ltime + 1 : 0;
    const uint64_t incl = wave_inclusive_max_u64(wit);
    const uint64_t excl = wave_shr1_u64(incl);
    const uint64_t clock_before = excl > r.clock ? excl : r.clock;
    const uint64_t chunk_max = lane63_u64(incl);
    MPROF_T(t_c1);
    MPROF_ADD(1, t_c0, t_c1);
    // walk chains in depth order
    ViewE v = pre;
    int f = 0;
    uint64_t ref = 0, contrib = 0;  // digest word of a MemberEvent (Failed -> Left)
    bool done = !is_view, dirty = false;
    // bounded: a chain has at most cnt links, so cnt passes always finish it
    for (uint32_t pass = 0; pass < cnt; ++pass) {
      // every lane takes part in each ds_bpermute (an exec-masked source lane reads as 0)
      const int src = prev < 0 ? (int)lane : prev;
      const int pdone = __shfl((int)done, src);  // NOT inside `||`: short-circuit would exec-mask it
      const bool prev_done = prev < 0 || pdone != 0;
      const uint64_t pl = __shfl(v.ltime, src);
      // meta uses 16 bits: the predecessor's dirty flag rides in bit 31
      const uint32_t pmd = (uint32_t)__shfl((int)(v.meta | (dirty ? 0x80000000u : 0u)), src);
      const uint32_t pt = (uint32_t)__shfl((int)v.t, src);
      const bool go = !done && prev_done;
      if (go) {
        if (prev >= 0) {
          v.ltime = pl;
          v.meta = pmd & 0x7FFFFFFFu;
          v.t = pt;
          dirty = (pmd >> 31) != 0;
        }
        MRegs rr = r;
        rr.clock = clock_before;
        rr.digest = 0;
        const uint64_t lt0 = v.ltime;
        const uint32_t mt0 = v.meta, t0 = v.t;
        if (ru.type == RSF_MSG_JOIN) f = hv_join_intent(v, rr, ru.ltime, c.now);
        else f = hv_leave_intent<false>(v, rr, ru.subject, ru.ltime, ru.flags & 1, ref, c.now);
        if (f & RSF_F_MEMBER_EVENT) contrib = kDigMember | ((uint64_t)kEvLeave << 32) | ru.subject;
        dirty = dirty || v.ltime != lt0 || v.meta != mt0 || v.t != t0;
        done = true;
      }
      if (!ballot(!done)) break;
    }
    if (next < 0 && is_view && dirty) *view_at(vrow, my_subj) = v;  // last link writes the subject back
    if (chunk_max > r.clock) r.clock = chunk_max;
    MPROF_T(t_c2);
    MPROF_ADD(2, t_c1, t_c2);
    // intent re-queues of the chunk appended to the pending list in one batch (record order)
    const bool ins = is_view && (f & RSF_F_REBROADCAST);
    const uint64_t newmask = ballot(ins);
    if (newmask) {
      const uint32_t k = (uint32_t)__popcll(newmask);
      const uint32_t i = pn + mbcnt(newmask);
      if (RSF_BAD_W(5, ins && i >= kPend, i)) return;
      if (ins) p_ent[i] = GState::PendE{rid, dsub, ru.msg_len};  // queue 0
      pn += k;
      pc += k;
    }
    // serial part, record order: events/queries (lane 0 handlers), digest, refutes
    const uint64_t serial =
        ballot(valid && (!is_view || (f & (RSF_F_MEMBER_EVENT | RSF_F_REFUTE | RSF_F_PRUNE))));
    uint64_t mm = serial;
    while (mm) {
      const int i = __ffsll((long long)mm) - 1;
      mm &= mm - 1;
      const uint32_t tf = shfl_u32((uint32_t)ru.type | ((uint32_t)ru.flags << 8) | ((uint32_t)ru.msg_len << 16), i);
      const uint8_t type = (uint8_t)(tf & 0xFF);
      int fi;
      if (type == RSF_MSG_JOIN || type == RSF_MSG_LEAVE) {
        fi = (int)shfl_u32((uint32_t)f, i);
        if (fi & RSF_F_MEMBER_EVENT) r.digest = digest_mix(r.digest, shfl_u64(contrib, i));
        if (fi & RSF_F_PRUNE)  // handle_prune's Reap event, after the Leave event of a Failed member
          r.digest = digest_mix(r.digest, kDigMember | ((uint64_t)kEvReap << 32) | shfl_u32(ru.subject, i));
        if (c.dcap && (fi & (RSF_F_MEMBER_EVENT | RSF_F_PRUNE))) {
          const uint32_t sj = shfl_u32(ru.subject, i);
          if (lane == 0) mlog_intent(c, s, l, r.err, fi, sj);
          r.err = shfl_u32(r.err, 0);
        }
        if (fi & RSF_F_REFUTE) {
          const uint64_t rf = shfl_u64(ref, i);
          if (lane == 0) push_refute(c, s, r, rf);
          r.err = shfl_u32(r.err, 0);
        }
      } else {
        const uint64_t L = shfl_u64(ru.ltime, i);
        const uint64_t key = shfl_u64(ru.key, i);
        fi = 0;
        if (lane == 0) {
          if (type == RSF_MSG_USER_EVENT) fi = h_user_event(c, s, l, r, L, key, (tf >> 8) & 1);
          else if (type == RSF_MSG_QUERY) fi = h_query(c, s, l, r, L, (uint32_t)key, (tf >> 8) & 1);
        }
        fi = (int)shfl_u32((uint32_t)fi, 0);
        r.eclock = shfl_u64(r.eclock, 0);
        r.qclock = shfl_u64(r.qclock, 0);
        r.digest = shfl_u64(r.digest, 0);
        r.err = shfl_u32(r.err, 0);
      }
      const uint32_t q = queue_of(type);
      if ((fi & RSF_F_REBROADCAST) && q != kQIntent) {  // intents went in above, batched per chunk
        if (lane == 0) {
          p_ent[pn] = GState::PendE{shfl_u32(rid, i), q == kQQuery ? kDecQuery : kDecEvent, (tf >> 16) | (q << 16)};
        }
        pn++;
        pc += 1u << (8 * q);
      }
    }
    MPROF_T(t_c3);
    MPROF_ADD(3, t_c2, t_c3);
    if (vb + kWave < total) __threadfence_block();  // next chunk's prefetch must see this chunk's view stores
  }
  MPROF_T(t_st0);
  if (BIG && pn > kPendMerge) {  // leave the originations' headroom (kPendMerge)
    __threadfence_block();
    qdrop += pend_flush_any(c, s, l, lane, pc, *row);
    pc = pn = 0;
  }
  if (qdrop) r.err |= kErrQueue;
  // registers go back only where they changed (the setup lanes hold the old values)
  const bool w_clock = r.clock != su64(su, kSuClock), w_eclock = r.eclock != su64(su, kSuEClock),
             w_qclock = r.qclock != su64(su, kSuQClock), w_digest = r.digest != su64(su, kSuDigest),
             w_err = r.err != shfl_u32(su, kSuErr);
  if (lane == 0) {
    if (w_clock) s.clock[l] = r.clock;
    if (w_eclock) s.eclock[l] = r.eclock;
    if (w_qclock) s.qclock[l] = r.qclock;
    if (w_digest) s.digest[l] = r.digest;
    if (w_err) s.err[l] = r.err;
    if (pc != pc0 || qdrop) s.p_cnt[l] = pc;
  }
  MPROF_T(t_end);
  MPROF_ADD(4, t_st0, t_end);
  MPROF_ADD(5, t_start, t_end);
  if (lane == 0) { MPROF_ADD(6, 0, 1); }
}

template <bool RUNS>
__global__ void __launch_bounds__(256, RSF_MERGE_WAVES) merge_kernel(GCfg c, GState s, const uint32_t* __restrict__ vals,
                                                    const uint32_t* __restrict__ dec,
                                                    const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ seg_end,
                                                    const uint32_t* __restrict__ gcnt, uint32_t stride, Buckets bk,
                                                    BigList big) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  __shared__ uint32_t subj_bits[kWavesPerBlock][128];  // chain detection (zero between chunks)
  uint32_t* sbits = subj_bits[threadIdx.x / kWave];
  for (uint32_t i = threadIdx.x & (kWave - 1); i < 128; i += kWave) sbits[i] = 0u;
  const uint64_t l = ((uint64_t)xcd_block(blockIdx.x, gridDim.x) * kWavesPerBlock +
                      (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave)) * RSF_MERGE_PER_WAVE;
  if (l >= c.n_loc) return;
  const MSetupLane sl = merge_setup_lane(c, s, seg_start, seg_end, lane, RUNS ? bk.n_runs : 0u);
  uint32_t cur = merge_setup(sl, l, lane);
  // every owned receiver's setup is in flight one receiver ahead of its merge
  for (uint32_t k = 0; k < RSF_MERGE_PER_WAVE && l + k < c.n_loc; ++k) {
    const uint32_t nxt = k + 1 < RSF_MERGE_PER_WAVE && l + k + 1 < c.n_loc ? merge_setup(sl, l + k + 1, lane) : 0u;
    merge_one<RUNS, false>(c, s, vals, dec, gcnt, stride, l + k, lane, cur, nullptr, sbits, bk, big);
    cur = nxt;
  }
}

// the receivers merge_kernel deferred (BigList), grid-stride over the list
template <bool RUNS>
__global__ void __launch_bounds__(256) merge_big_kernel(GCfg c, GState s, const uint32_t* __restrict__ vals,
                                                        const uint32_t* __restrict__ dec,
                                                        const uint32_t* __restrict__ seg_start,
                                                        const uint32_t* __restrict__ seg_end,
                                                        const uint32_t* __restrict__ gcnt, uint32_t stride, Buckets bk,
                                                        BigList big) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  __shared__ QLds4 qlds[kWavesPerBlock];  // scratch of a pending list applied here
  __shared__ uint32_t subj_bits[kWavesPerBlock][128];
  QLds4& ql = qlds[threadIdx.x / kWave];
  uint32_t* sbits = subj_bits[threadIdx.x / kWave];
  for (uint32_t i = lane; i < 128; i += kWave) sbits[i] = 0u;
  const uint64_t n = *big.n;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  const MSetupLane sl = merge_setup_lane(c, s, seg_start, seg_end, lane, RUNS ? bk.n_runs : 0u);
  for (uint64_t i = (uint64_t)blockIdx.x * kWavesPerBlock + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
       i < n; i += nw) {
    const uint64_t l = big.ids[i];
    merge_one<RUNS, true>(c, s, vals, dec, gcnt, stride, l, lane, merge_setup(sl, l, lane), &ql, sbits, bk, big);
  }
}

// ---- push/pull anti-entropy (M7): merge_remote_state of a sender's local_state
// (core/src/serf/delegate.rs:376-554).  Snapshot semantics: memberlist sends its
// local state before it merges the remote one, so every sender's state is copied
// to a slab first (streaming, one block per pair), then merged.
struct PPSlab {
  ViewS* view;        // [pair][S]
  uint64_t* eb_ltime; // [pair][ebuf]
  uint32_t* eb_cnt;   // [pair][ebuf]
  uint64_t* eb_keys;  // [pair][ebuf * slot_k]
  uint64_t* clocks;   // [pair][4]: clock, event clock, query clock, -
};

__global__ void __launch_bounds__(256) pp_snapshot_kernel(GCfg c, GState s, const rsf_pp_pair* __restrict__ pairs,
                                                          PPSlab sl) {
  const uint64_t p = blockIdx.x;
  const uint64_t l = pairs[p].sender - c.lo;
  const uint4* vsrc = reinterpret_cast<const uint4*>(vrow_of(s, c, l));
  uint4* vdst = reinterpret_cast<uint4*>(view_row(sl.view, c.vrow, p));
  for (uint32_t i = threadIdx.x; i < c.vrow / 16; i += blockDim.x) vdst[i] = vsrc[i];
  for (uint32_t i = threadIdx.x; i < c.ebuf; i += blockDim.x) {
    sl.eb_ltime[p * c.ebuf + i] = s.eb_ltime[l * c.ebuf + i];
    sl.eb_cnt[p * c.ebuf + i] = s.eb_cnt[l * c.ebuf + i];
  }
  const uint64_t nk = (uint64_t)c.ebuf * c.slot_k;
  for (uint64_t i = threadIdx.x; i < nk; i += blockDim.x) sl.eb_keys[p * nk + i] = s.eb_keys[l * nk + i];
  if (threadIdx.x == 0) {
    sl.clocks[p * 4 + 0] = s.clock[l];
    sl.clocks[p * 4 + 1] = s.eclock[l];
    sl.clocks[p * 4 + 2] = s.qclock[l];
  }
}

// One wave per pair (receiver).  Lanes walk the subject slots 64 at a time:
// left members run handle_node_leave_intent(status_time + 1), the other known
// entries handle_node_join_intent(status_time); subjects are distinct, so lanes
// are independent except for the Lamport clock, whose value at each leave is an
// inclusive prefix max over the left members before it (all leaves precede all
// joins, delegate.rs:477-511).  The event buffer is walked the same way: sender
// slot i holds events of ltime = i (mod B), so it lands in receiver slot i and
// lanes touch distinct slots; the event clock is again a prefix max.  Member
// events, refutations and deliveries are digested serially in order.
__global__ void __launch_bounds__(256) pp_merge_kernel(GCfg c, GState s, const rsf_pp_pair* __restrict__ pairs,
                                                       uint64_t n_pairs, PPSlab sl, uint32_t flags) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t p = (uint64_t)blockIdx.x * kWavesPerBlock + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  if (p >= n_pairs) return;
  const uint32_t m = pairs[p].receiver;
  const uint64_t l = m - c.lo;
  if (!s.alive[m]) return;
  MRegs r;
  load_regs(s, l, r);
  const uint64_t pl = sl.clocks[p * 4 + 0], pel = sl.clocks[p * 4 + 1], pql = sl.clocks[p * 4 + 2];
  if (pl > 0) witness(r.clock, pl - 1);
  if (pel > 0) witness(r.eclock, pel - 1);
  if (pql > 0) witness(r.qclock, pql - 1);
  // ---- status_ltimes / left_members
  const ViewS* sv = view_row(sl.view, c.vrow, p);
  ViewS* vrow = vrow_of(s, c, l);
  uint64_t c_leave = r.clock, c_join = r.clock;
  for (uint32_t base = 0; base < c.S; base += kWave) {
    const uint32_t subj = base + lane;
    const bool valid = subj < c.S;
    ViewE se{};
    if (valid) se = *view_at(sv, subj);
    const bool known = valid && vkind(se.meta) == RSF_KIND_KNOWN;
    const bool left = known && vstatus(se.meta) == RSF_STATUS_LEFT;
    const bool join = known && !left;
    ViewE v{};
    if (known) v = *view_at(vrow, subj);
    const uint64_t L = left ? se.ltime + 1 : se.ltime;
    const uint64_t incl = wave_inclusive_max_u64(left ? L + 1 : 0);
    const uint64_t excl = wave_shr1_u64(incl);
    int f = 0;
    uint64_t ref = 0;
    if (known) {
      MRegs rr = r;
      rr.clock = excl > c_leave ? excl : c_leave;
      rr.digest = 0;
      const uint64_t lt0 = v.ltime;
      const uint32_t mt0 = v.meta;
      const uint32_t t0 = v.t;
      if (left) f = hv_leave_intent(v, rr, subj, L, false, ref, c.now);
      else f = hv_join_intent(v, rr, L, c.now);
      if (v.ltime != lt0 || v.meta != mt0 || v.t != t0) *view_at(vrow, subj) = v;
    }
    const uint64_t lmax = lane63_u64(incl);
    if (lmax > c_leave) c_leave = lmax;
    const uint64_t jmax = wave_max_u64(join ? L + 1 : 0);
    if (jmax > c_join) c_join = jmax;
    uint64_t mm = ballot(f & (RSF_F_MEMBER_EVENT | RSF_F_REFUTE));
    while (mm) {
      const int i = __ffsll((long long)mm) - 1;
      mm &= mm - 1;
      const uint32_t fi = shfl_u32((uint32_t)f, i);
      if (fi & RSF_F_MEMBER_EVENT) {
        r.digest = digest_mix(r.digest, kDigMember | ((uint64_t)kEvLeave << 32) | (base + (uint32_t)i));
        if (lane == 0) mlog_put(c, s, l, r.err, kEvLeave, base + (uint32_t)i);
        r.err = shfl_u32(r.err, 0);
      }
      if (fi & RSF_F_REFUTE) {
        const uint64_t rf = shfl_u64(ref, i);
        if (lane == 0) push_refute(c, s, r, rf);
        r.err = shfl_u32(r.err, 0);
      }
    }
  }
  r.clock = c_leave > c_join ? c_leave : c_join;
  // ---- eventJoinIgnore (delegate.rs:513-521)
  if ((flags & 3) == 3 && pel > r.emin) r.emin = pel;
  // ---- the sender's event buffer, index order (delegate.rs:523-541)
  const uint64_t B = c.ebuf;
  uint64_t ec = r.eclock;
  for (uint32_t base = 0; base < c.ebuf; base += kWave) {
    const uint32_t i = base + lane;
    const bool valid = i < c.ebuf;
    const uint32_t cnt = valid ? sl.eb_cnt[p * c.ebuf + i] : 0u;
    const uint64_t L = cnt ? sl.eb_ltime[p * c.ebuf + i] : 0ull;
    const uint64_t incl = wave_inclusive_max_u64(cnt ? L + 1 : 0);
    const uint64_t excl = wave_shr1_u64(incl);
    uint64_t cur = excl > ec ? excl : ec;
    if (cnt && L + 1 > cur) cur = L + 1;  // witness(L) of this slot's events
    uint64_t dmask = 0;  // delivered keys of this slot (slot_k <= 64)
    uint32_t e_err = 0;
    if (cnt && !(L < r.emin) && !(cur > B && L < cur - B)) {
      const uint64_t rs = l * c.ebuf + (L % B);
      if ((L % B) != i) {
        e_err = kErrEvSlot;  // a ring slot not at ltime mod B: never produced by handle_user_event
      } else {
        uint64_t* rk = s.eb_keys + rs * c.slot_k;
        const uint64_t* sk = sl.eb_keys + (p * c.ebuf + i) * c.slot_k;
        uint32_t rc = s.eb_cnt[rs];
        const uint32_t rc0 = rc;
        for (uint32_t k = 0; k < cnt; ++k) {
          const uint64_t key = sk[k];
          bool dup = false;
          for (uint32_t j = 0; j < rc; ++j) dup |= rk[j] == key;
          if (dup) continue;
          if (rc == 0) {
            s.eb_ltime[rs] = L;
            rk[0] = key;
            rc = 1;
          } else if (rc < c.slot_k) {
            rk[rc++] = key;
          } else {
            e_err |= kErrEvSlot;
          }
          dmask |= 1ull << k;
        }
        if (rc != rc0) s.eb_cnt[rs] = rc;
      }
    }
    const uint64_t emax = lane63_u64(incl);
    if (emax > ec) ec = emax;
    uint64_t mm = ballot(dmask != 0 || e_err != 0);
    while (mm) {
      const int j = __ffsll((long long)mm) - 1;
      mm &= mm - 1;
      r.err |= shfl_u32(e_err, j);
      uint64_t dm = shfl_u64(dmask, j);
      const uint64_t Lj = shfl_u64(L, j);
      const uint64_t* skj = sl.eb_keys + (p * c.ebuf + base + (uint32_t)j) * c.slot_k;
      while (dm) {
        const int k = __ffsll((long long)dm) - 1;
        dm &= dm - 1;
        r.digest = digest_mix(digest_mix(r.digest, kDigUser ^ skj[k]), Lj);
        if (lane == 0) dlog_put(c, s, l, r, Lj, skj[k], false);
        r.err = shfl_u32(r.err, 0);
      }
    }
  }
  r.eclock = ec;
  if (lane == 0) {
    store_regs(s, l, r);
    s.emin[l] = r.emin;
  }
}

// ---- Reaper (M8; core/src/serf/base.rs:519-601, 1782-1784).  One wave per live
// member, lanes over subject slots (16-B coalesced view reads).  Pass 1 erases
// failed members past reconnect_timeout and intents past recent_intent_timeout
// and digests the failed reaps in slot order; pass 2 (only where a left member
// is due) erases left members past tombstone_timeout and digests them, so every
// failed Reap event precedes every left one, as reap_failed precedes reap_left.
__global__ void __launch_bounds__(256) reap_kernel(GCfg c, GState s, uint32_t now, uint32_t rc_to, uint32_t ts_to,
                                                   uint32_t in_to) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t l = (uint64_t)blockIdx.x * kWavesPerBlock + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  if (l >= c.n_loc) return;
  if (!s.alive[c.lo + l]) return;
  ViewS* vrow = vrow_of(s, c, l);
  uint64_t dig = s.digest[l];
  const uint64_t d0 = dig;
  uint32_t lerr = 0;  // delivery-log overflow
  bool any_left = false;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1 && !any_left) break;
    for (uint32_t base = 0; base < c.S; base += kWave) {
      const uint32_t subj = base + lane;
      ViewE v{};
      if (subj < c.S) v = *view_at(vrow, subj);
      // (stamps are kept mod 2^27: the age is exact below 2^27 rounds)
      const uint32_t kind = vkind(v.meta), st = vstatus(v.meta), age = (now - v.t) & kViewTMask;
      const bool known = subj < c.S && kind == RSF_KIND_KNOWN;
      const bool failed = known && st == RSF_STATUS_FAILED && age > rc_to;   // leave_time.elapsed() > timeout
      const bool left = known && st == RSF_STATUS_LEFT && age > ts_to;
      const bool intent = subj < c.S && (kind == RSF_KIND_INTENT_JOIN || kind == RSF_KIND_INTENT_LEAVE) && age > in_to;
      const bool reap = pass == 0 ? failed : left;
      if (reap || (pass == 0 && intent)) *view_at(vrow, subj) = ViewE{0ull, 0u, 0u};  // erase_node / reap_intents
      if (pass == 0) any_left = any_left || ballot(left) != 0;
      uint64_t mm = ballot(reap);
      while (mm) {  // Reap member events, slot order
        const int i = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        dig = digest_mix(dig, kDigMember | ((uint64_t)kEvReap << 32) | (base + (uint32_t)i));
        if (lane == 0) mlog_put(c, s, l, lerr, kEvReap, base + (uint32_t)i);
      }
    }
  }
  if (lane == 0 && dig != d0) s.digest[l] = dig;
  if (lane == 0 && lerr) s.err[l] |= lerr;
}

// direct-handler batch: one thread per receiver segment (array order within a receiver)
__global__ void __launch_bounds__(256) apply_kernel(GCfg c, GState s, const rsf_msg* __restrict__ msgs,
                                                    const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ seg_end, int32_t* __restrict__ flags,
                                                    uint64_t* __restrict__ refute) {
  uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= c.n_loc) return;
  uint32_t st = seg_start[l], en = seg_end[l];
  if (st >= en) return;
  MRegs r;
  load_regs(s, l, r);
  ViewS* vrow = vrow_of(s, c, l);
  for (uint32_t i = st; i < en; ++i) {
    uint32_t k = order[i];
    rsf_msg x = msgs[k];
    uint64_t ref = 0;
    int f = 0;
    switch (x.type) {
      case RSF_MSG_JOIN: f = h_join_intent(view_at(vrow, x.subject), r, x.ltime, c.now); break;
      case RSF_MSG_LEAVE:
        f = h_leave_intent(view_at(vrow, x.subject), r, x.subject, x.ltime, x.flags & 1, ref, c.now);
        mlog_intent(c, s, l, r.err, f, x.subject);
        break;
      case RSF_MSG_USER_EVENT: f = h_user_event(c, s, l, r, x.ltime, x.key, x.flags & 1); break;
      case RSF_MSG_QUERY: f = h_query(c, s, l, r, x.ltime, (uint32_t)x.key, x.flags & 1); break;
      default: f = 0; break;
    }
    flags[k] = f;
    refute[k] = ref;
  }
  store_regs(s, l, r);
}

__global__ void keys_from_msgs_kernel(const rsf_msg* __restrict__ msgs, uint64_t n, uint64_t lo,
                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = (uint32_t)(msgs[i].receiver - lo);
  idx[i] = (uint32_t)i;
}

__global__ void init_views_kernel(ViewS* view, uint64_t vrow, uint64_t n_loc, uint32_t S, const uint8_t* kind,
                                  const uint8_t* status, const uint64_t* ltime) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_loc * S) return;
  uint32_t subj = (uint32_t)(i % S);
  ViewE v;
  v.ltime = ltime[subj];
  v.meta = vmeta(status[subj], kind[subj]);
  v.t = 0;
  *view_at(view_row(view, vrow, i / S), subj) = v;
}

__global__ void tsum_init_kernel(uint4* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = kTSumEmpty;
}

__global__ void iota_u32_kernel(uint32_t* p, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

__global__ void fill_u64_kernel(uint64_t* p, uint64_t n, uint64_t v) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void shard_bounds_kernel(const uint64_t* __restrict__ rec, const unsigned long long* n_valid,
                                    uint64_t per, uint32_t world, unsigned long long* __restrict__ bounds) {
  uint32_t w = threadIdx.x;
  if (w > world) return;
  uint64_t nv = *n_valid;
  uint64_t target = (uint64_t)w * per;  // first key >= target
  uint64_t lo = 0, hi = nv;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if ((rec[mid] >> 32) < target) lo = mid + 1;
    else hi = mid;
  }
  bounds[w] = (w == world) ? nv : lo;
}

__global__ void unpack_kernel(const uint64_t* __restrict__ in, uint64_t n, uint32_t* __restrict__ keys,
                              uint32_t* __restrict__ vals) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = in[i];
  keys[i] = (uint32_t)(x >> 32);
  vals[i] = (uint32_t)x;
}

// ---- multi-GPU receive side without a second sort.  The received buffer is n_runs
// runs (one per source shard, concatenated in source-rank = ascending-sender order),
// each already sorted (stably) by receiver.  The canonical merge order is (receiver,
// run, position in run); it is built from run boundaries, per-(run, receiver) counts,
// one scan over receivers and an ordered scatter.
__device__ __forceinline__ uint32_t run_of(const uint64_t* __restrict__ off, uint32_t n_runs, uint64_t i) {
  uint32_t lo = 0, hi = n_runs;  // largest r with off[r] <= i (an empty run is never chosen)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(256) runs_bounds_kernel(const uint64_t* __restrict__ rec, uint64_t n,
                                                          const uint64_t* __restrict__ off, uint32_t n_runs,
                                                          uint64_t lo, uint64_t n_loc, uint32_t* __restrict__ rstart,
                                                          uint32_t* __restrict__ rend,
                                                          unsigned long long* __restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = run_of(off, n_runs, i);
  const uint32_t k = (uint32_t)(rec[i] >> 32);
  const uint64_t l = (uint64_t)k - lo;
  const bool first = i == off[r] || (uint32_t)(rec[i - 1] >> 32) != k;
  const bool last = i + 1 == off[r + 1] || (uint32_t)(rec[i + 1] >> 32) != k;
  if (l >= n_loc || (i > off[r] && (uint32_t)(rec[i - 1] >> 32) > k)) {  // not ours / run not sorted
    atomicOr(bad, 1ull);
    return;
  }
  if (first) rstart[r * n_loc + l] = (uint32_t)i;
  if (last) rend[r * n_loc + l] = (uint32_t)(i + 1);
}

__global__ void __launch_bounds__(256) runs_base_kernel(uint32_t n_runs, uint64_t n_loc,
                                                        const uint32_t* __restrict__ rstart,
                                                        const uint32_t* __restrict__ rend, uint32_t* __restrict__ rbase,
                                                        uint32_t* __restrict__ total) {
  const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n_loc) return;
  uint32_t acc = 0;
  for (uint32_t r = 0; r < n_runs; ++r) {
    const uint64_t idx = r * n_loc + l;
    rbase[idx] = acc;
    acc += rend[idx] - rstart[idx];
  }
  total[l] = acc;
}

__global__ void __launch_bounds__(256) runs_scatter_kernel(const uint64_t* __restrict__ rec, uint64_t n,
                                                           const uint64_t* __restrict__ off, uint32_t n_runs,
                                                           uint64_t lo, uint64_t n_loc,
                                                           const uint32_t* __restrict__ rstart,
                                                           const uint32_t* __restrict__ rbase,
                                                           const uint32_t* __restrict__ seg_start,
                                                           uint32_t* __restrict__ vals,
                                                           const uint32_t* __restrict__ rdec,
                                                           uint32_t* __restrict__ dec, uint32_t rmask) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = run_of(off, n_runs, i);
  const uint64_t x = rec[i];
  const uint64_t l = (uint64_t)(uint32_t)(x >> 32) - lo;
  if (l >= n_loc) return;
  const uint64_t idx = r * n_loc + l;
  const uint32_t pos = seg_start[l] + rbase[idx] + (uint32_t)(i - rstart[idx]);
  vals[pos] = (uint32_t)x;
  dec[pos] = rdec[(uint32_t)x & rmask];
}

__global__ void __launch_bounds__(256) seg_end_kernel(uint64_t n_loc, const uint32_t* __restrict__ seg_start,
                                                      const uint32_t* __restrict__ total,
                                                      uint32_t* __restrict__ seg_end) {
  const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l < n_loc) seg_end[l] = seg_start[l] + total[l];
}

// QueueChecker tick (base.rs:703-760): one thread per (member, queue).  A sorted queue's
// live items are its leading slots, so num_queued is the first free slot; prune(max)
// drops the items past `max`, the last ones in send order (memberlist
// TransmitLimitedQueue::prune).  stats[q] = queued, stats[3 + q] = members at or above
// the warning depth, stats[6 + q] = pruned.
// Deep queues: numq counts the tail too, and a queue to prune is listed (s.deep_ids) for
// check_stream_kernel, which keeps the max smallest keys of head and tail.
// qmax (non-null when min_queue_depth > 0): each member's own get_queue_max (queue_max_kernel).
constexpr uint32_t kOccBin = 64, kOccBins = 160;  // occupancy histogram: 64-item bins up to 10240, then one overflow bin
// One wave per member (lane = head slot; 65..256-slot queues in chunks of 64), a grid-stride
// loop over the phase's members: a queue's head count is its leading run of live slots, one
// ballot per chunk.  The counts and the occupancy histogram are summed per block in LDS and
// added to HBM once per block (one global atomic per member on the same few addresses took
// 0.25 ms for 6.7k members).
__global__ void __launch_bounds__(256) check_queues_kernel(GCfg c, GState s, uint32_t max_depth, uint32_t warn,
                                                           unsigned long long* __restrict__ stats,
                                                           const uint32_t* __restrict__ qmax,
                                                           uint32_t* __restrict__ hist, uint32_t period,
                                                           uint32_t phase) {
  __shared__ unsigned long long bst[9];
  __shared__ uint32_t bh[3 * (kOccBins + 1) + 3];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  for (uint32_t i = threadIdx.x; i < 3 * (kOccBins + 1) + 3; i += blockDim.x) bh[i] = 0;
  if (threadIdx.x < 9) bst[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t l0 = phase_first(c, period, phase);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
  for (uint64_t wi = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;; wi += nw) {
    const uint64_t l = l0 + wi * period;
    if (l >= c.n_loc) break;
    const uint32_t mx = qmax ? qmax[l] : max_depth;
    uint32_t nq[3];
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      const uint64_t base = (l * 3 + q) * c.qcap;
      uint32_t n = 0;
      for (uint32_t j = 0; j < c.qcap; j += kWave) {
        const bool live = j + lane < c.qcap && s.q_rumor[base + j + lane] != kEmpty;
        const uint64_t m = ballot(live);
        const uint32_t run = m == ~0ull ? kWave : (uint32_t)__builtin_ctzll(~m);
        n = j + run;
        if (run < kWave) break;
      }
      if (tcap_of(c, q)) n += s.tsum[l * 3 + q].x;
      nq[q] = n;
    }
    if (lane < 3) {
      const uint32_t q = lane, n = q == 0 ? nq[0] : q == 1 ? nq[1] : nq[2];
      atomicAdd(&bh[q * (kOccBins + 1) + min(n / kOccBin, kOccBins)], 1u);  // occupancy before the prune
      atomicMax(&bh[3 * (kOccBins + 1) + q], n);
      if (n) atomicAdd(&bst[q], (unsigned long long)n);
      if (n >= warn) atomicAdd(&bst[3 + q], 1ull);
      if (n > mx) atomicAdd(&bst[6 + q], (unsigned long long)(n - mx));
      // the deep queues' entries for check_stream_kernel at fixed places (kEmpty: under the
      // max): one atomic per listed queue on a single counter took most of this kernel's time
      if (tcap_of(c, q)) s.deep_ids[wi * deep_queues(c) + deep_rank(c, q)] = n > mx ? (uint32_t)(l * 3 + q) : kEmpty;
    }
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      if (tcap_of(c, q) || nq[q] <= mx) continue;  // numq >= max -> prune(max): retain max
      const uint64_t base = (l * 3 + q) * c.qcap;
      for (uint32_t i = mx + lane; i < nq[q]; i += kWave) {
        s.q_rumor[base + i] = kEmpty;
        s.q_seq[base + i] = 0;
        s.q_txlen[base + i] = 0;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 9 && bst[threadIdx.x]) atomicAdd(stats + threadIdx.x, bst[threadIdx.x]);
  if (hist) {
    for (uint32_t i = threadIdx.x; i < 3 * (kOccBins + 1); i += blockDim.x)
      if (bh[i]) atomicAdd(hist + i, bh[i]);
    if (threadIdx.x < 3 && bh[3 * (kOccBins + 1) + threadIdx.x])
      atomicMax(hist + 3 * (kOccBins + 1) + threadIdx.x, bh[3 * (kOccBins + 1) + threadIdx.x]);
  }
}

// get_queue_max with min_queue_depth > 0 (base.rs:748-759): max(2 * members.states.len(),
// min_queue_depth), per member, since each node's checker reads its own member map.
// states.len() is every member the node knows, as the Reconnector counts it
// (reconnect_kernel): the N - S untracked members, the local node when it is a subject, and
// the tracked subjects whose entry is KNOWN.  One wave per member; out[l] saturates at 2^32-1.
__global__ void __launch_bounds__(256) queue_max_kernel(GCfg c, GState s, uint32_t min_depth,
                                                        uint32_t* __restrict__ out, uint32_t period, uint32_t phase) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t l = phase_first(c, period, phase) + ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave * period;
  if (l >= c.n_loc) return;
  const int32_t own = s.member_subj[l];
  const ViewS* row = vrow_of(s, c, l);
  uint64_t known = (c.N - c.S) + (own >= 0 ? 1u : 0u);
  for (uint32_t j0 = 0; j0 < c.S; j0 += kWave) {
    const uint32_t j = j0 + lane;
    const bool kn = j < c.S && (int32_t)j != own && vkind(ViewE(*view_at(row, j)).meta) == RSF_KIND_KNOWN;
    known += (uint32_t)__popcll(ballot(kn));
  }
  uint64_t mx = 2 * known;
  if (mx < min_depth) mx = min_depth;
  if (lane == 0) out[l] = (uint32_t)(mx < 0xFFFFFFFFull ? mx : 0xFFFFFFFFull);
}

// Generations alive: gen and gen - 1 (modulo the generation count, even so that the
// parity alternates across the wrap).

// At the start of generation `gen` (the ring wrapped): every queue drops its items of
// generation gen - 2, whose table half this generation overwrites.  One wave per
// (member, queue), lane = queue slot; the survivors keep their sorted order.
__global__ void __launch_bounds__(256) expire_kernel(GCfg c, GState s, uint32_t gen) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  if (t >= c.n_loc * 3) return;
  const uint64_t l = t / 3;
  const uint32_t q = (uint32_t)(t % 3);
  const uint32_t G = rumor_generations(c);
  if (c.qcap > kWave) {
    __shared__ QLds4 rows[kWavesPerBlock];
    Q4 Q;
    q4_load(c, s, l, q, lane, Q);
    bool stale[kQK];
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) stale[k] = (gen + G - (Q.r[k] >> c.rbits) % G) % G >= 2;
    const uint32_t x = q4_expire(c, Q, lane, stale, q == 0, rows[threadIdx.x / kWave]);
    if (!x) return;
    q4_store(c, s, l, q, lane, Q);
    if (lane == 0) atomicAdd(s.q_expired + l, x);
    return;
  }
  QRegs Q{kEmpty, 0, 0};
  q_load(c, s, l, q, lane, Q);
  const uint32_t age = (gen + G - (Q.r >> c.rbits) % G) % G;
  const uint32_t x = q_expire(c, Q, lane, age >= 2, q == 0);
  if (x) q_store(c, s, l, q, lane, Q, true);
  const uint32_t xt = tail_expire_wave(c, s, l, q, lane, gen, G);  // deep queues: the tail too
  if ((x + xt) && lane == 0) atomicAdd(s.q_expired + l, x + xt);
}

// ---- multi-GPU exchange buckets: the sorted groups split by destination shard.
// bounds: wstart[w] = first sorted group whose receiver is in shard w (sentinel groups,
// dead senders, sort last); each bucket's header = its group count (overflow flagged).
__global__ void bucket_bounds_kernel(const uint32_t* __restrict__ key_s, uint64_t n, uint64_t per, uint32_t world,
                                     uint32_t* __restrict__ wstart, uint32_t* __restrict__ send, uint64_t stride_u32,
                                     uint32_t gcap, unsigned long long* __restrict__ flags) {
  const uint32_t w = threadIdx.x;
  if (w > world) return;
  auto first_ge = [&](uint64_t target) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if ((uint64_t)key_s[mid] < target) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  const uint64_t a = first_ge((uint64_t)w * per);
  wstart[w] = (uint32_t)a;
  if (w == world) return;
  const uint64_t b = first_ge((uint64_t)(w + 1) * per), ng = b - a;
  send[(uint64_t)w * stride_u32] = (uint32_t)(ng < gcap ? ng : gcap);
  if (ng > gcap) atomicOr(flags, 1ull);
}
// receive side: per (run r, receiver) the range of its groups in bucket r; the records
// merged (group counts) summed for the statistics; a receiver outside the shard or an
// unsorted bucket is flagged.  Grid-stride over a bounded grid: one atomic per block (an
// atomic per 256 groups on one address serialised into ~0.25 ms at 6M groups).
constexpr unsigned kBucketIndexBlocks = 1024;
__global__ void __launch_bounds__(256) bucket_index_kernel(Buckets bk, uint64_t lo, uint64_t n_loc,
                                                           uint32_t* __restrict__ rstart, uint32_t* __restrict__ rend,
                                                           unsigned long long* __restrict__ merged,
                                                           unsigned long long* __restrict__ flags) {
  // 32-bit indices: n_runs <= 8 buckets of < 2^26 groups (checked at rsf_gossip_bucket_buffers);
  // the 64-bit division per group was most of this kernel's time
  const uint32_t n = bk.n_runs * bk.gcap;
  uint64_t sum = 0;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    const uint32_t r = t / bk.gcap, i = t - r * bk.gcap;
    const uint32_t* b = bk.run(r);
    const uint32_t ng = b[0];
    if (i >= ng) continue;
    const uint32_t key = b[bk.keys_off + i];
    const uint64_t l = (uint64_t)key - lo;
    if (l >= n_loc || (i > 0 && b[bk.keys_off + i - 1] > key)) {
      atomicOr(flags, 2ull);
      continue;
    }
    const uint32_t cnt = b[bk.cnt_off + i];
    sum += cnt;
    if (i == 0 || b[bk.keys_off + i - 1] != key) rstart[(uint64_t)r * n_loc + l] = i;
    if (i + 1 == ng || b[bk.keys_off + i + 1] != key) rend[(uint64_t)r * n_loc + l] = i + 1;
  }
  __shared__ uint64_t part[4];
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long tot = part[0] + part[1] + part[2] + part[3];
    if (tot) atomicAdd(merged, tot);
  }
}
// several device buffers cleared by one launch (each hipMemsetAsync is a launch of its own,
// ~5 us on the stream however small the buffer): up to kZeroSpans spans of 4-B words
constexpr int kZeroSpans = 4;
struct ZeroSpans {
  uint32_t* p[kZeroSpans];
  uint64_t words[kZeroSpans];
};
__global__ void __launch_bounds__(256) zero_spans_kernel(ZeroSpans z) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
#pragma unroll
  for (int k = 0; k < kZeroSpans; ++k)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < z.words[k]; i += stride) z.p[k][i] = 0u;
}

// counters[60] (records merged since creation) += counters[from] (this round's)
__global__ void accumulate_kernel(unsigned long long* counters, uint32_t from) {
  if (threadIdx.x == 0 && blockIdx.x == 0) counters[60] += counters[from];
}

inline unsigned grid1(uint64_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }
#ifndef RSF_SYNC_DEBUG
#define RSF_SYNC_DEBUG 0  // diagnostic build: synchronise after every launch of the round and name a failing one
#endif
#define RSF_DBG_SYNC(st, name)                                                                 \
  do {                                                                                         \
    if (RSF_SYNC_DEBUG) {                                                                      \
      const hipError_t e_ = hipStreamSynchronize(st);                                          \
      if (e_ != hipSuccess) {                                                                  \
        fprintf(stderr, "RSF_SYNC_DEBUG: after %s: %s\n", name, hipGetErrorString(e_));        \
        return rsf::set_hip_error(e_, name, __FILE__, __LINE__);                              \
      }                                                                                        \
    }                                                                                          \
  } while (0)
inline int bits_for(uint64_t n) {
  int b = 1;
  while (b < 32 && ((1ull << b) <= n)) ++b;
  return b;
}

}  // namespace

struct rsf_gossip {
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  GCfg c{};
  GState s{};
  // rumor ring: cursor (next free slot) and generation; the round's block is slots
  // [round_slot, round_slot + round_need), its ids round_base + i (gen << rbits | slot)
  uint32_t n_rumors = 0, max_rumors = 0, gen = 0;
  std::vector<uint32_t> subj_sorted;  // the tracked subjects' members, sorted (action checks)
  uint32_t round_slot = 0, round_base = 0, round_abase = 0, round_need = 0;
  // per-round device lists
  rsf_ml_event* d_ml = nullptr;
  rsf_action* d_acts = nullptr;
  int32_t* d_act_status = nullptr;  // [cap_acts] originate_kernel's per-action result
  uint32_t cap_ml = 0, cap_acts = 0, last_n_acts = 0;
  // the round's host lists go to the device from pinned staging (two slots, each reused
  // once the copy issued from it two rounds earlier has completed): a copy from pageable
  // memory would block the host until the stream drained, leaving the GPU idle while the
  // next round is prepared and launched
#ifndef RSF_PIN_STAGING
#define RSF_PIN_STAGING 1
#endif
  void* pin[2] = {nullptr, nullptr};
  size_t pin_cap[2] = {0, 0};
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  bool pin_used[2] = {false, false};
  int pin_next = 0;
  // record pipeline
  uint64_t stage_cap = 0, recv_cap = 0;
  uint32_t *stage_key = nullptr, *stage_val = nullptr, *sort_key = nullptr, *sort_val = nullptr;
  uint32_t *seg_start = nullptr, *seg_end = nullptr;
  void* pp_buf = nullptr;  // push/pull snapshot slab (grow-only)
  uint64_t pp_cap = 0;
  uint32_t* rec_dec = nullptr;  // record decoration beside sort_val (segment_kernel / runs_scatter_kernel)
  // record groups (emit_kernel): [n_loc * fanout] receiver / count, sorted copies, ids, offsets
  uint64_t n_groups = 0;
  // record groups: [n_loc * fanout] peers (emit order) -> sorted by receiver (key_s, id_s);
  // slot[gid] = sorted position; cnt[sorted] = records; off = inclusive scan of cnt (multi-GPU)
  uint32_t *grp_key = nullptr, *grp_cnt = nullptr, *grp_key_s = nullptr, *grp_id = nullptr, *grp_id_s = nullptr,
           *grp_slot = nullptr, *grp_off = nullptr, *stage_dec = nullptr;
  rsf::CubTemp grp_tmp;  // the group count reduce / scan (each call sized by cub_run)
  unsigned merge_blocks = 1;  // merge_big_kernel's grid: merge_kernel's resident blocks per CU x CUs
  unsigned deep_blocks = 1;   // emit_deep_wave_kernel<kDeepSmall> grid (resident waves x CUs)
  unsigned deep_blocks_big = 1;  // emit_deep_wave_kernel<kDeepBig> grid
  unsigned deep_blocks_tiny = 1;  // emit_deep_wave_kernel<kDeepTiny> grid
  unsigned deep_blocks_mid = 1;   // emit_deep_wave_kernel<kDeepMid> grid
  unsigned deep_check_blocks = 1;  // check_stream_kernel grid
  uint64_t deep_last = 0;     // rsf_gossip_deep_stats' previous total
  uint32_t* big_ids = nullptr;  // receivers deferred to merge_big_kernel (count: d_counters[52])
  uint32_t* qmax = nullptr;     // [n_loc] per-member get_queue_max (rsf_gossip_check_queues, min_queue_depth > 0)
  uint32_t* occ_hist = nullptr; // the last checker tick's occupancy histogram + maxima (check_queues_kernel)
  // RSF_GUARD_ZONES (diagnostic builds): 0xA5-filled zones before and after big_ids and
  // stage_dec and after the sort's storage; rsf_gossip_debug_zones counts changed bytes
  char *big_base = nullptr, *dec_base = nullptr;
  uint64_t* send_buf = nullptr;
  unsigned long long* d_counters = nullptr;  // [0] n_valid, [1..] shard bounds
  rsf::CubTemp sort_tmp;  // every radix sort of the round (sort_pairs)
  // Peers ahead: once round t's emission has consumed the groups, round t + 1's peer draw and
  // group sort (they depend on nothing but liveness and the round number) run on a second
  // stream, under round t's merge / bucket exchange.  Round t + 1 uses them if nothing changed
  // liveness in between (ahead_valid), else redraws.  RSF_PEERS_AHEAD=0 turns it off.
  hipStream_t side = nullptr;
  hipEvent_t ev_emitted = nullptr, ev_ahead = nullptr;
  // in-round checker ticks (rsf_gossip_set_checker): period 0 = off
  uint32_t chk_period = 0, chk_max = 0, chk_min = 0, chk_warn = 0;
  bool ahead_launched = false, ahead_valid = false, ahead_on = true;
  uint32_t ahead_round = 0;
  int end_bit = 32;
  uint64_t last_sent = 0, last_merged = 0;
  uint32_t cur_round = 0;
  bool merged_from_stage = true, merged_from_buckets = false;
  // bucket exchange: send / receive buffers (world buckets each), group ranges per run
  uint32_t *bkt_send = nullptr, *bkt_recv = nullptr, *d_rstart = nullptr, *d_rend = nullptr, *d_wstart = nullptr;
  uint32_t bkt_world = 0, bkt_gcap = 0;
  uint64_t total_merged_host = 0;  // multi-GPU merges (n_recv known on host)
  // run-merge tables of rsf_gossip_round_merge_runs: [run_cap][n_loc] u32 x3, [n_loc] u32
  uint32_t *run_start = nullptr, *run_end = nullptr, *run_base = nullptr, *run_total = nullptr;
  uint64_t* d_run_off = nullptr;
  uint32_t run_cap = 0;
  rsf::CubTemp scan_tmp;  // rsf_gossip_round_merge_runs' segment scan
  // phase profiling: marks per round [begin, after begin, after emit, after sort, after merge]
  bool profiling = false;
  static constexpr int kMarks = 5, kMaxProfRounds = 256;
  hipEvent_t ev[kMaxProfRounds][kMarks] = {};
  int prof_rounds = 0;
  bool events_made = false;
  DeviceScratch scratch;
};

static int gerr(const char* m) { return rsf::set_error(RSF_ERR_ARG, m); }

static void mark(rsf_gossip* g, int k) {
  if (!g->profiling || g->prof_rounds >= rsf_gossip::kMaxProfRounds) return;
  hipEventRecord(g->ev[g->prof_rounds][k], g->stream);
  if (k == rsf_gossip::kMarks - 1) g->prof_rounds++;
}

// Every member's pending re-queues applied to its queues: before anything other than
// emission reads the queues, the queue-prune counters or the error flags.
static int flush_pending(rsf_gossip* g, uint32_t period = 1, uint32_t phase = 0) {
  const uint64_t cnt = phase_count(g->c, period, phase);
  if (!cnt) return RSF_OK;
  hipLaunchKernelGGL(pend_flush_kernel, dim3(grid1(cnt, kWavesPerBlock)), dim3(kWave * kWavesPerBlock), 0,
                     g->stream, g->c, g->s, period, phase);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

static int ensure_lists(rsf_gossip* g, uint32_t n_ml, uint32_t n_acts) {
  int rc;
  if (n_ml > g->cap_ml) {
    hipFree(g->d_ml);
    g->d_ml = nullptr;
    uint32_t cap = std::max<uint32_t>(n_ml, 64);
    if ((rc = dmalloc((void**)&g->d_ml, cap * sizeof(rsf_ml_event)))) return rc;
    g->cap_ml = cap;
  }
  if (n_acts > g->cap_acts) {
    hipFree(g->d_acts);
    hipFree(g->d_act_status);
    g->d_acts = nullptr;
    g->d_act_status = nullptr;
    g->cap_acts = 0;
    uint32_t cap = std::max<uint32_t>(n_acts, 1024);
    if ((rc = dmalloc((void**)&g->d_acts, (size_t)cap * sizeof(rsf_action)))) return rc;
    if ((rc = dmalloc((void**)&g->d_act_status, (size_t)cap * sizeof(int32_t)))) return rc;
    g->cap_acts = cap;
  }
  return RSF_OK;
}

#ifndef RSF_GUARD_ZONES
#define RSF_GUARD_ZONES 0  // diagnostic builds: 0xA5 zones around stage_dec and big_ids
#endif
constexpr size_t kZone = RSF_GUARD_ZONES ? (2u << 20) : 0;
// every radix sort sizes its own temporary storage (rsf::cub_run)
static int sort_pairs(rsf_gossip* g, const uint32_t* kin, uint32_t* kout, const uint32_t* vin, uint32_t* vout,
                      uint64_t n, hipStream_t on = nullptr) {
  const int end_bit = g->end_bit;
  hipStream_t st = on ? on : g->stream;
  return rsf::cub_run(
      g->sort_tmp, st,
      [&](void* t, size_t& b) {
        return hipcub::DeviceRadixSort::SortPairs(t, b, kin, kout, vin, vout, (int)n, 0, end_bit, st);
      },
      "group/record radix sort");
}

// the peers-ahead work in flight (if any) is joined by the context stream and dropped: before
// anything changes liveness, or uses the group arrays / sort storage another way
static int ahead_drop(rsf_gossip* g) {
  if (g->ahead_launched) RSF_HIP(hipStreamWaitEvent(g->stream, g->ev_ahead, 0));
  g->ahead_launched = g->ahead_valid = false;
  return RSF_OK;
}

// peer draw + stable sort of the groups by receiver, on stream `st`
static int peers_and_sort(rsf_gossip* g, uint32_t round, hipStream_t st) {
  const GCfg& c = g->c;
  hipLaunchKernelGGL(peers_kernel, dim3(grid1(c.n_loc)), dim3(256), 0, st, c, g->s, round, g->grp_key);
  RSF_HIP(hipGetLastError());
  RSF_DBG_SYNC(st, "peers_kernel");
  int rc = sort_pairs(g, g->grp_key, g->grp_key_s, g->grp_id, g->grp_id_s, g->n_groups, st);
  if (rc) return rc;
  RSF_DBG_SYNC(st, "group sort");
  return RSF_OK;
}

extern "C" {

int rsf_gossip_create(rsf_gossip** out, const rsf_gossip_cfg* cfg, int device) {
  if (!out || !cfg) return gerr("null argument");
  *out = nullptr;
  const uint64_t N = cfg->n_members;
  if (N < 2 || N >= 0xFFFFFFFFull) return gerr("n_members must be in [2, 2^32-1)");
  if (cfg->shard_lo >= cfg->shard_hi || cfg->shard_hi > N) return gerr("bad shard range");
  if (cfg->n_subjects == 0 || cfg->n_subjects > N) return gerr("n_subjects must be in [1, n_members]");
  if (cfg->queue_cap == 0 || cfg->queue_cap > 256) return gerr("queue_cap must be 1..256");
  if (cfg->event_buffer_size == 0 || cfg->query_buffer_size == 0) return gerr("dedup buffers must be non-empty");
  if (cfg->slot_k == 0 || cfg->slot_k > 64) return gerr("slot_k must be 1..64");
  if (cfg->fanout == 0 || cfg->fanout > 8 || cfg->fanout >= N) return gerr("fanout must be 1..8 and < n_members");
  if (cfg->gossip_limit > 0xFFFFFF || cfg->gossip_overhead > 0xFFFF) return gerr("gossip budget too large");
  if (cfg->max_refute == 0 || cfg->max_refute > 4) return gerr("max_refute must be 1..4");
  if (cfg->max_rumors == 0 || (cfg->max_rumors & (cfg->max_rumors - 1)) || cfg->max_rumors > (1u << 30))
    return gerr("max_rumors must be a power of two <= 2^30 (the rumor ring)");
  if (cfg->max_user_event_size > RSF_USER_EVENT_SIZE_LIMIT)  // Serf::new_in (base.rs:69-70)
    return rsf::set_error(RSF_ERR_USER_EVENT_LIMIT, "max_user_event_size exceeds USER_EVENT_SIZE_LIMIT (9 KiB)");
  if (cfg->query_size_limit > 0xFFFE) return gerr("query_size_limit must be <= 65534 (16-bit message lengths)");
  for (int q = 0; q < 3; ++q) {
    const uint32_t d = cfg->queue_depth[q];
    if (d && d < cfg->queue_cap) return gerr("queue_depth must be 0 or >= queue_cap");
    if (d > cfg->queue_cap && cfg->queue_cap > kWave) return gerr("deep queues need queue_cap <= 64 (the register head)");
    if (d > RSF_MAX_QUEUE_DEPTH) return gerr("queue_depth exceeds RSF_MAX_QUEUE_DEPTH");
  }
  RSF_HIP(hipSetDevice(device));
  rsf_gossip* g = new (std::nothrow) rsf_gossip();
  if (!g) return rsf::set_error(RSF_ERR_NOMEM, "host allocation failed");
  g->device = device;
  GCfg& c = g->c;
  c.N = N;
  c.lo = cfg->shard_lo;
  c.n_loc = cfg->shard_hi - cfg->shard_lo;
  c.S = cfg->n_subjects;
  c.vrow = view_row_bytes(c.S);
  c.qcap = cfg->queue_cap;
  c.ebuf = cfg->event_buffer_size;
  c.qbuf = cfg->query_buffer_size;
  c.slot_k = cfg->slot_k;
  c.fanout = cfg->fanout;
  c.limit = cfg->gossip_limit;
  c.overhead = cfg->gossip_overhead;
  {  // memberlist retransmitLimit = mult * ceil(log10(n+1))
    uint64_t x = N + 1, p = 1;
    uint32_t d = 0;
    while (p < x) {
      p *= 10;
      d++;
    }
    c.tx_limit = cfg->retransmit_mult * d;
  }
  c.max_refute = cfg->max_refute;
  c.max_ue = cfg->max_user_event_size ? cfg->max_user_event_size : 512u;  // options.rs:526
  c.query_limit = cfg->query_size_limit ? cfg->query_size_limit : 1024u;  // options.rs:519
  uint32_t max_depth = c.qcap;
  {  // deep queues: the tail behind the register head
    uint32_t tc[3];
    for (int q = 0; q < 3; ++q) {
      const uint32_t d = cfg->queue_depth[q];
      tc[q] = d > c.qcap ? d - c.qcap : 0u;
      c.deep |= tc[q] ? 1u : 0u;
      max_depth = std::max(max_depth, c.qcap + tc[q]);
    }
    c.tcap0 = tc[0];
    c.tcap1 = tc[1];
    c.tcap2 = tc[2];
    c.tstride0 = tc[0] ? tc[0] + kTailSlack : 0u;
    c.tstride1 = tc[1] ? tc[1] + kTailSlack : 0u;
    c.tstride2 = tc[2] ? tc[2] + kTailSlack : 0u;
  }
  {
    uint64_t per = c.limit / (c.overhead + kMinMsgLen);
    c.cap_t = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(3ull * max_depth, per));
  }
  c.k0 = (uint32_t)cfg->seed;
  c.k1 = (uint32_t)(cfg->seed >> 32);
  g->max_rumors = cfg->max_rumors;
  c.rbits = 0;
  while ((1u << c.rbits) < cfg->max_rumors) c.rbits++;
  c.rmask = (cfg->max_rumors << 1) - 1;
  c.gen = 0;
  g->end_bit = bits_for(N);
  auto fail = [&](int code) {
    rsf_gossip_destroy(g);
    return code;
  };
  // the intent queue's packed tail items (tail_pack): the ring slot and parity in 27 bits,
  // transmits in 6
  if (c.tcap0 && c.rbits > 26) return fail(gerr("a deep intent queue needs max_rumors <= 2^26 (packed tail items)"));
  if (c.tcap0 && c.tx_limit > 64)
    return fail(gerr("a deep intent queue needs a retransmit limit <= 64 (packed tail items)"));
  if (hipStreamCreateWithFlags(&g->own, hipStreamNonBlocking) != hipSuccess)
    return fail(rsf::set_error(RSF_ERR_HIP, "hipStreamCreate failed"));
  g->stream = g->own;
  if (hipStreamCreateWithFlags(&g->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev_emitted, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev_ahead, hipEventDisableTiming) != hipSuccess)
    return fail(rsf::set_error(RSF_ERR_HIP, "hipStreamCreate / hipEventCreate failed"));
  {
    const char* e = getenv("RSF_PEERS_AHEAD");
    g->ahead_on = !(e && e[0] == '0');
  }
  GState& s = g->s;
  const uint64_t n = c.n_loc, S = c.S;
  int rc;
#define GA(p, bytes) ((rc = dmalloc((void**)&(p), (bytes))) != 0)
  if (GA(s.clock, n * 8) || GA(s.eclock, n * 8) || GA(s.qclock, n * 8) || GA(s.emin, n * 8) || GA(s.qmin, n * 8) ||
      GA(s.digest, n * 8) || GA(s.err, n * 4) || GA(s.alive, N) || GA(s.serf_state, n) || GA(s.member_subj, n * 4) ||
      GA(s.subj_member, S * 4) || GA(s.refute_cnt, S * 4) || GA(s.refute_ltime, S * c.max_refute * 8) ||
      GA(s.view, n * c.vrow) || GA(s.q_rumor, n * 3 * c.qcap * 4) || GA(s.q_seq, n * 3 * c.qcap * 4) ||
      GA(s.q_txlen, n * 3 * c.qcap * 4) || GA(s.q_dec, n * c.qcap * 4) || GA(s.q_next_seq, n * 3 * 4) || GA(s.q_pruned, n * 4) || GA(s.q_expired, n * 4) || GA(s.eb_ltime, n * c.ebuf * 8) ||
      GA(s.eb_cnt, n * c.ebuf * 4) || GA(s.eb_keys, n * c.ebuf * c.slot_k * 8) || GA(s.qb_ltime, n * c.qbuf * 8) ||
      GA(s.qb_cnt, n * c.qbuf * 4) || GA(s.qb_ids, n * c.qbuf * c.slot_k * 4) ||
      GA(s.rumors, (size_t)cfg->max_rumors * 2 * sizeof(rsf_rumor)) ||
      GA(s.rdec, (size_t)cfg->max_rumors * 2 * 4) || GA(s.rbody, (size_t)cfg->max_rumors * 2 * 16) ||
      GA(s.p_ent, n * kPend * sizeof(GState::PendE)) || GA(s.p_cnt, n * 4))
    return fail(rc);
  if (c.deep) {  // tails, their summaries, the deferred-member list (also the checker's, 3 per member)
    for (int q = 0; q < 3; ++q)
      if (tcap_of(c, q) && (q == 0 ? GA(s.tail0, n * c.tstride0 * sizeof(uint64_t))
                                   : GA(q == 1 ? s.tail1 : s.tail2, n * tstride_of(c, q) * sizeof(uint4))))
        return fail(rc);
    if (GA(s.tsum, n * 3 * sizeof(uint4)) || GA(s.tseal, n * 3 * sizeof(uint4)) || GA(s.deep_ids, n * 5 * 4))
      return fail(rc);
  }
  g->stage_cap = n * c.fanout * c.cap_t;
  if (g->stage_cap >= 0xFFFFFFFFull) return fail(gerr("n_members x fanout x per-target records must fit 32 bits"));
  g->recv_cap = g->stage_cap + g->stage_cap / 2 + 4096;
  const uint64_t pipe = std::max(g->stage_cap, g->recv_cap);
  if (GA(g->stage_key, pipe * 4) || GA(g->stage_val, pipe * 4) || GA(g->sort_key, pipe * 4) ||
      GA(g->sort_val, pipe * 4) || GA(g->seg_start, n * 4) || GA(g->seg_end, n * 4) || GA(g->send_buf, pipe * 8) || GA(g->rec_dec, pipe * 4) ||
      GA(g->d_counters, 72 * 8))
    return fail(rc);
  g->n_groups = n * c.fanout;
  if (GA(g->grp_key, g->n_groups * 4) || GA(g->grp_cnt, g->n_groups * 4) || GA(g->grp_key_s, g->n_groups * 4) ||
      GA(g->grp_id, g->n_groups * 4) || GA(g->grp_id_s, g->n_groups * 4) || GA(g->grp_slot, g->n_groups * 4) ||
      GA(g->grp_off, g->n_groups * 4) || GA(g->dec_base, g->stage_cap * 4 + 2 * kZone) ||
      GA(g->big_base, n * 4 + 2 * kZone))
    return fail(rc);
  g->stage_dec = (uint32_t*)(g->dec_base + kZone);
  g->big_ids = (uint32_t*)(g->big_base + kZone);
  if (kZone) {
    bool zok = true;
    for (char* z : {g->dec_base, g->dec_base + kZone + g->stage_cap * 4, g->big_base, g->big_base + kZone + n * 4})
      zok = zok && hipMemset(z, 0xA5, kZone) == hipSuccess;
    if (!zok) return fail(rsf::set_error(RSF_ERR_HIP, "guard zone init failed"));
  }
#undef GA
  {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, merge_kernel<false>, kWave * kWavesPerBlock, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
      return fail(rsf::set_error(RSF_ERR_HIP, "occupancy query failed"));
    g->merge_blocks = (unsigned)std::max(1, per_cu * cus);
    if (c.deep) {
      int dpc = 0, dpb = 0, dpk = 0, dpt = 0, dpm = 0;
      if (
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&dpc, emit_deep_wave_kernel<false, kDeepSmall>, kWave, 0) !=
              hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&dpt, emit_deep_wave_kernel<false, kDeepTiny>, kWave, 0) !=
              hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&dpm, emit_deep_block_kernel<false, kDeepMid>, kDeepBlkThreads, 0) !=
              hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&dpb, emit_deep_block_kernel<false, kDeepBig>, kDeepBlkThreads, 0) !=
              hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&dpk, check_stream_kernel, kDeepThreads, 0) != hipSuccess)
        return fail(rsf::set_error(RSF_ERR_HIP, "occupancy query failed"));
      g->deep_blocks = (unsigned)std::max(1, dpc * cus);
      g->deep_blocks_big = (unsigned)std::max(1, dpb * cus);
      g->deep_blocks_tiny = (unsigned)std::max(1, dpt * cus);
      g->deep_blocks_mid = (unsigned)std::max(1, dpm * cus);
      g->deep_check_blocks = (unsigned)std::max(1, dpk * cus);
    }
  }
  // the hipCUB temporaries are sized per call at their first use (rsf::cub_run)
  hipStream_t st = g->stream;
  bool ok = true;
  auto ms = [&](void* p, int v, size_t b) { ok = ok && hipMemsetAsync(p, v, b, st) == hipSuccess; };
  ms(g->d_counters, 0, 72 * 8);  // status flags and running totals start at zero
  // deferred members: the counts of lists 0..4 (words 64-66; [55] their total)
  s.deep_n = reinterpret_cast<uint32_t*>(g->d_counters + 64);
  ms(s.emin, 0, n * 8);
  ms(s.qmin, 0, n * 8);
  ms(s.digest, 0, n * 8);
  ms(s.err, 0, n * 4);
  ms(s.alive, 1, N);
  ms(s.serf_state, 0, n);
  ms(s.member_subj, 0xFF, n * 4);
  ms(s.subj_member, 0, S * 4);
  ms(s.refute_cnt, 0, S * 4);
  ms(s.refute_ltime, 0, S * c.max_refute * 8);
  ms(s.view, 0, n * c.vrow);
  ms(s.q_rumor, 0xFF, n * 3 * c.qcap * 4);
  ms(s.q_seq, 0, n * 3 * c.qcap * 4);
  ms(s.q_txlen, 0, n * 3 * c.qcap * 4);
  ms(s.q_dec, 0, n * c.qcap * 4);
  ms(s.q_next_seq, 0, n * 3 * 4);
  ms(s.q_pruned, 0, n * 4);
  ms(s.q_expired, 0, n * 4);
  ms(s.p_cnt, 0, n * 4);
  ms(s.eb_ltime, 0, n * c.ebuf * 8);
  ms(s.eb_cnt, 0, n * c.ebuf * 4);
  ms(s.eb_keys, 0, n * c.ebuf * c.slot_k * 8);
  ms(s.qb_ltime, 0, n * c.qbuf * 8);
  ms(s.qb_cnt, 0, n * c.qbuf * 4);
  ms(s.qb_ids, 0, n * c.qbuf * c.slot_k * 4);
  ms(s.rumors, 0, (size_t)cfg->max_rumors * 2 * sizeof(rsf_rumor));
  ms(s.rdec, 0, (size_t)cfg->max_rumors * 2 * 4);
  ms(s.rbody, 0, (size_t)cfg->max_rumors * 2 * 16);
  // emission's group slots and the record stage start defined (grp_index_kernel writes the
  // slot of every group with a receiver each round; a slot it did not write stays in range)
  ms(g->grp_slot, 0, g->n_groups * 4);
  ms(g->stage_val, 0, g->stage_cap * 4);
  ms(g->stage_dec, 0xFF, g->stage_cap * 4);
  if (!ok) return fail(rsf::set_error(RSF_ERR_HIP, "context initialisation failed"));
  // Serf::new increments every clock once (base.rs:195-199)
  hipLaunchKernelGGL(fill_u64_kernel, dim3(grid1(n)), dim3(256), 0, st, s.clock, n, 1ull);
  hipLaunchKernelGGL(fill_u64_kernel, dim3(grid1(n)), dim3(256), 0, st, s.eclock, n, 1ull);
  hipLaunchKernelGGL(fill_u64_kernel, dim3(grid1(n)), dim3(256), 0, st, s.qclock, n, 1ull);
  hipLaunchKernelGGL(iota_u32_kernel, dim3(grid1(g->n_groups)), dim3(256), 0, st, g->grp_id, g->n_groups);
  if (c.deep) {  // empty tails, no sealed prefix (m = 0)
    hipLaunchKernelGGL(tsum_init_kernel, dim3(grid1(n * 3)), dim3(256), 0, st, s.tsum, n * 3);
    hipLaunchKernelGGL(tsum_init_kernel, dim3(grid1(n * 3)), dim3(256), 0, st, s.tseal, n * 3);
  }
  if (hipStreamSynchronize(st) != hipSuccess) return fail(rsf::set_error(RSF_ERR_HIP, "context init sync failed"));
  *out = g;
  return RSF_OK;
}

int rsf_gossip_destroy(rsf_gossip* g) {
  if (!g) return RSF_OK;
  hipSetDevice(g->device);
  if (g->side) hipStreamSynchronize(g->side);
  if (g->stream) hipStreamSynchronize(g->stream);
  GState& s = g->s;
  void* ptrs[] = {s.clock,  s.eclock,      s.qclock,       s.emin,        s.qmin,     s.digest,     s.err,
                  s.alive,  s.serf_state,  s.member_subj,  s.subj_member, s.refute_cnt, s.refute_ltime, s.view,
                  s.q_rumor, s.q_seq,      s.q_txlen,      s.q_dec,      s.q_next_seq,  s.q_pruned, s.q_expired,  s.eb_ltime, s.eb_cnt,     s.eb_keys,
                  s.qb_ltime, s.qb_cnt,    s.qb_ids,       s.rumors,      s.rdec,       s.rbody,      g->d_ml,    g->d_acts,    g->stage_key,
                  g->stage_val, g->sort_key, g->sort_val,  g->seg_start,  g->seg_end, g->send_buf,  g->d_counters, g->rec_dec, g->pp_buf,
                  g->run_start, g->run_end, g->run_base, g->run_total, g->d_run_off,
                  g->grp_key, g->grp_cnt, g->grp_key_s, g->grp_id, g->grp_id_s,
                  g->grp_slot, g->grp_off, g->dec_base, s.dlog, s.dmeta, s.dcnt,
                  g->bkt_send, g->bkt_recv, g->d_rstart, g->d_rend, g->d_wstart, s.snap_bits, s.snap_sn,
                  s.p_ent, s.p_cnt, g->big_base, s.tail0, s.tail1, s.tail2, s.tsum, s.deep_ids,
                  s.tseal, g->qmax, g->d_act_status, g->occ_hist};
  for (void* p : ptrs)
    if (p) hipFree(p);
  g->scratch.release();
  for (int k = 0; k < 2; ++k) {
    if (g->pin[k]) hipHostFree(g->pin[k]);
    if (g->pin_ev[k]) hipEventDestroy(g->pin_ev[k]);
  }
  g->sort_tmp.release();
  g->grp_tmp.release();
  g->scan_tmp.release();
  if (g->events_made)
    for (auto& row : g->ev)
      for (auto& e : row) hipEventDestroy(e);
  if (g->own) hipStreamDestroy(g->own);
  if (g->side) hipStreamDestroy(g->side);
  if (g->ev_emitted) hipEventDestroy(g->ev_emitted);
  if (g->ev_ahead) hipEventDestroy(g->ev_ahead);
  delete g;
  return RSF_OK;
}

int rsf_gossip_set_stream(rsf_gossip* g, void* st) {
  if (!g) return gerr("null context");
  g->stream = st ? (hipStream_t)st : g->own;
  return RSF_OK;
}

int rsf_gossip_sync(rsf_gossip* g) {
  if (!g) return gerr("null context");
  RSF_HIP(hipSetDevice(g->device));
  if (g->ahead_launched) RSF_HIP(hipStreamSynchronize(g->side));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_set_subjects(rsf_gossip* g, const uint32_t* subj_member) {
  if (!g || !subj_member) return gerr("null argument");
  const GCfg& c = g->c;
  std::vector<int32_t> ms(c.n_loc, -1);
  std::vector<uint8_t> seen(c.N, 0);
  for (uint32_t s = 0; s < c.S; ++s) {
    uint32_t m = subj_member[s];
    if (m >= c.N) return gerr("subject member out of range");
    if (seen[m]++) return gerr("a member is the subject of two slots");
    if (m >= c.lo && m < c.lo + c.n_loc) ms[m - c.lo] = (int32_t)s;
  }
  g->subj_sorted.assign(subj_member, subj_member + c.S);
  std::sort(g->subj_sorted.begin(), g->subj_sorted.end());
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(g->s.subj_member, subj_member, c.S * 4, hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipMemcpyAsync(g->s.member_subj, ms.data(), c.n_loc * 4, hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_init_views(rsf_gossip* g, const uint8_t* kind, const uint8_t* status, const uint64_t* ltime) {
  if (!g || !kind || !status || !ltime) return gerr("null argument");
  const GCfg& c = g->c;
  for (uint32_t i = 0; i < c.S; ++i)
    if (kind[i] > RSF_KIND_KNOWN || status[i] > RSF_STATUS_FAILED) return gerr("bad view kind/status");
  RSF_HIP(hipSetDevice(g->device));
  size_t b[3] = {c.S, c.S, (size_t)c.S * 8};
  void* d[3];
  int rc = g->scratch.take(b, 3, d);
  if (rc) return rc;
  RSF_HIP(hipMemcpyAsync(d[0], kind, c.S, hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipMemcpyAsync(d[1], status, c.S, hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipMemcpyAsync(d[2], ltime, (size_t)c.S * 8, hipMemcpyHostToDevice, g->stream));
  hipLaunchKernelGGL(init_views_kernel, dim3(grid1(c.n_loc * c.S)), dim3(256), 0, g->stream, g->s.view, c.vrow, c.n_loc, c.S,
                     (const uint8_t*)d[0], (const uint8_t*)d[1], (const uint64_t*)d[2]);
  RSF_HIP(hipGetLastError());
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_set_view(rsf_gossip* g, uint64_t m, uint32_t subj, uint8_t kind, uint8_t status, uint64_t ltime) {
  if (!g) return gerr("null context");
  const GCfg& c = g->c;
  if (m < c.lo || m >= c.lo + c.n_loc || subj >= c.S) return gerr("member/subject out of range");
  if (kind > RSF_KIND_KNOWN || status > RSF_STATUS_FAILED) return gerr("bad view kind/status");
  ViewE e;
  e.ltime = ltime;
  e.meta = status | ((uint32_t)kind << 8);
  e.t = 0;
  ViewS v;
  v = e;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(vent(g->s, c, m - c.lo, subj), &v, sizeof(v), hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_set_alive(rsf_gossip* g, const uint8_t* alive) {
  if (!g || !alive) return gerr("null argument");
  RSF_HIP(hipSetDevice(g->device));
  int rc = ahead_drop(g);  // liveness changes: peers drawn ahead are stale
  if (rc) return rc;
  RSF_HIP(hipMemcpyAsync(g->s.alive, alive, g->c.N, hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

static int set_u64(rsf_gossip* g, uint64_t* dst, uint64_t v) {
  RSF_HIP(hipMemcpyAsync(dst, &v, 8, hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_set_clocks(rsf_gossip* g, uint64_t m, uint64_t clock, uint64_t ec, uint64_t qc) {
  if (!g) return gerr("null context");
  if (m < g->c.lo || m >= g->c.lo + g->c.n_loc) return gerr("member out of shard");
  uint64_t l = m - g->c.lo;
  RSF_HIP(hipSetDevice(g->device));
  int rc;
  if ((rc = set_u64(g, g->s.clock + l, clock)) || (rc = set_u64(g, g->s.eclock + l, ec)) ||
      (rc = set_u64(g, g->s.qclock + l, qc)))
    return rc;
  return RSF_OK;
}

int rsf_gossip_set_min_times(rsf_gossip* g, uint64_t m, uint64_t emin, uint64_t qmin) {
  if (!g) return gerr("null context");
  if (m < g->c.lo || m >= g->c.lo + g->c.n_loc) return gerr("member out of shard");
  uint64_t l = m - g->c.lo;
  RSF_HIP(hipSetDevice(g->device));
  int rc;
  if ((rc = set_u64(g, g->s.emin + l, emin)) || (rc = set_u64(g, g->s.qmin + l, qmin))) return rc;
  return RSF_OK;
}

int rsf_gossip_set_serf_state(rsf_gossip* g, uint64_t m, uint8_t state) {
  if (!g) return gerr("null context");
  if (m < g->c.lo || m >= g->c.lo + g->c.n_loc || state > 3) return gerr("bad member/state");
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(g->s.serf_state + (m - g->c.lo), &state, 1, hipMemcpyHostToDevice, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_apply_batch(rsf_gossip* g, const rsf_msg* msgs, uint64_t n, int32_t* flags_out, uint64_t* refute_out) {
  if (!g || (n && (!msgs || !flags_out))) return gerr("null argument");
  if (n == 0) return RSF_OK;
  const GCfg& c = g->c;
  if (n > 0xFFFFFFFFull) return gerr("batch too large");
  for (uint64_t i = 0; i < n; ++i) {
    if (msgs[i].receiver < c.lo || msgs[i].receiver >= c.lo + c.n_loc) return gerr("receiver outside shard");
    uint8_t t = msgs[i].type;
    if (t != RSF_MSG_JOIN && t != RSF_MSG_LEAVE && t != RSF_MSG_USER_EVENT && t != RSF_MSG_QUERY)
      return gerr("unsupported message type");
    if ((t == RSF_MSG_JOIN || t == RSF_MSG_LEAVE) && msgs[i].subject >= c.S) return gerr("subject out of range");
  }
  RSF_HIP(hipSetDevice(g->device));
  size_t b[7] = {n * sizeof(rsf_msg), n * 4, n * 4, n * 4, n * 4, n * 4, n * 8};
  void* d[7];
  int rc = g->scratch.take(b, 7, d);
  if (rc) return rc;
  size_t tmp = 0;
  RSF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (uint32_t*)d[1], (uint32_t*)d[2], (uint32_t*)d[3],
                                             (uint32_t*)d[4], (int)n, 0, bits_for(c.n_loc), g->stream));
  void* tmpbuf;
  if ((rc = g->scratch.take_extra(tmp, &tmpbuf))) return rc;
  RSF_HIP(hipMemcpyAsync(d[0], msgs, n * sizeof(rsf_msg), hipMemcpyHostToDevice, g->stream));
  hipLaunchKernelGGL(keys_from_msgs_kernel, dim3(grid1(n)), dim3(256), 0, g->stream, (const rsf_msg*)d[0], n, c.lo,
                     (uint32_t*)d[1], (uint32_t*)d[3]);
  RSF_HIP(hipcub::DeviceRadixSort::SortPairs(tmpbuf, tmp, (uint32_t*)d[1], (uint32_t*)d[2], (uint32_t*)d[3],
                                             (uint32_t*)d[4], (int)n, 0, bits_for(c.n_loc), g->stream));
  RSF_HIP(hipMemsetAsync(g->seg_start, 0, c.n_loc * 4, g->stream));
  RSF_HIP(hipMemsetAsync(g->seg_end, 0, c.n_loc * 4, g->stream));
  hipLaunchKernelGGL(segment_kernel, dim3(grid1(n)), dim3(256), 0, g->stream, (const uint32_t*)d[2], n, 0ull,
                     g->seg_start, g->seg_end, (const uint32_t*)nullptr, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                     0u);
  hipLaunchKernelGGL(apply_kernel, dim3(grid1(c.n_loc)), dim3(256), 0, g->stream, c, g->s, (const rsf_msg*)d[0],
                     (const uint32_t*)d[4], g->seg_start, g->seg_end, (int32_t*)d[5], (uint64_t*)d[6]);
  RSF_HIP(hipGetLastError());
  RSF_HIP(hipMemcpyAsync(flags_out, d[5], n * 4, hipMemcpyDeviceToHost, g->stream));
  if (refute_out) RSF_HIP(hipMemcpyAsync(refute_out, d[6], n * 8, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

// phases 1-3 (everything before emission)
int rsf_gossip_round_begin(rsf_gossip* g, uint32_t round, const rsf_ml_event* ml, uint32_t n_ml,
                           const rsf_action* acts, uint32_t n_acts) {
  if (!g || (n_ml && !ml) || (n_acts && !acts)) return gerr("null argument");
  const GCfg& c = g->c;
  for (uint32_t e = 0; e < n_ml; ++e)
    if (ml[e].subject >= c.S || (ml[e].kind != RSF_ML_JOIN && ml[e].kind != RSF_ML_LEAVE && ml[e].kind != RSF_ML_UPDATE) || ml[e].set_alive > 2)
      return gerr("bad memberlist event");
  // actions: known kinds, members in range, distinct members
  {
    std::vector<uint32_t> ms;
    ms.reserve(n_acts);
    for (uint32_t a = 0; a < n_acts; ++a) {
      const rsf_action& x = acts[a];
      if (x.member >= c.N || x.act < RSF_ACT_JOIN_SELF || x.act > RSF_ACT_QUERY) return gerr("bad action");
      if (x.act == RSF_ACT_FORCE_LEAVE && x.subject >= c.S) return gerr("force_leave subject out of range");
      if ((x.act == RSF_ACT_JOIN_SELF || x.act == RSF_ACT_LEAVE_SELF) &&
          !std::binary_search(g->subj_sorted.begin(), g->subj_sorted.end(), x.member))
        return gerr("join / leave of a member that is not a tracked subject");
      ms.push_back(x.member);
    }
    std::sort(ms.begin(), ms.end());
    if (std::adjacent_find(ms.begin(), ms.end()) != ms.end()) return gerr("actions of one round must name distinct members");
  }
  uint64_t need = (uint64_t)c.S * c.max_refute + n_acts;
  if (need > g->max_rumors) return rsf::set_error(RSF_ERR_OVERFLOW, "one round's rumors exceed the rumor ring");
  RSF_HIP(hipSetDevice(g->device));
  int rc = ensure_lists(g, n_ml, n_acts);
  if (rc) return rc;
  for (uint32_t e = 0; e < n_ml; ++e)  // liveness changes: peers drawn ahead are stale
    if (ml[e].set_alive != 2 && (rc = ahead_drop(g))) return rc;
  hipStream_t st = g->stream;
  mark(g, 0);
  g->cur_round = round;
  g->c.now = round;  // handlers stamp leave / intent times with the round
  if ((uint64_t)g->n_rumors + need > g->max_rumors) {  // the block restarts the ring, next generation
    g->n_rumors = 0;
    g->gen = (g->gen + 1) % rumor_generations(c);
    g->c.gen = g->gen;
    // this generation reuses the half of the table of generation gen - 2: queued ids of
    // that generation expire now, before anything reads or re-queues them
    if ((rc = flush_pending(g))) return rc;
    hipLaunchKernelGGL(expire_kernel, dim3(grid1(c.n_loc * 3, kWavesPerBlock)), dim3(kWave * kWavesPerBlock), 0,
                       g->stream, c, g->s, g->gen);
  }
  g->round_slot = g->n_rumors;
  g->round_base = (uint32_t)(((uint64_t)g->gen << c.rbits) | g->round_slot);
  g->round_abase = g->round_base + c.S * c.max_refute;
  g->round_need = (uint32_t)need;
  g->n_rumors += (uint32_t)need;
  const uint32_t round_pidx = g->round_base & c.rmask;  // physical index: generation parity | slot
  RSF_HIP(hipMemsetAsync(g->s.rumors + round_pidx, 0, need * sizeof(rsf_rumor), st));
  if (g->c.dcap) RSF_HIP(hipMemsetAsync(g->s.dcnt, 0, c.n_loc * 4, st));  // the round's delivery log
  const size_t b_ml = (size_t)n_ml * sizeof(rsf_ml_event), b_acts = (size_t)n_acts * sizeof(rsf_action);
  const char* pin_ml = nullptr;
  const char* pin_acts = nullptr;
  int pin_k = -1;
  if (!RSF_PIN_STAGING) {
    pin_ml = (const char*)ml;
    pin_acts = (const char*)acts;
  } else if (b_ml + b_acts) {
    const int k = pin_k = g->pin_next;
    g->pin_next ^= 1;
    if (g->pin_used[k]) RSF_HIP(hipEventSynchronize(g->pin_ev[k]));  // its previous copy has landed
    if (!g->pin_ev[k]) RSF_HIP(hipEventCreateWithFlags(&g->pin_ev[k], hipEventDisableTiming));
    if (b_ml + b_acts > g->pin_cap[k]) {
      if (g->pin[k]) RSF_HIP(hipHostFree(g->pin[k]));
      g->pin[k] = nullptr;
      g->pin_cap[k] = 0;
      const size_t cap = std::max<size_t>(b_ml + b_acts, 1 << 20);
      RSF_HIP(hipHostMalloc(&g->pin[k], cap, hipHostMallocDefault));
      g->pin_cap[k] = cap;
    }
    char* p = (char*)g->pin[k];
    if (b_ml) memcpy(p, ml, b_ml);
    if (b_acts) memcpy(p + b_ml, acts, b_acts);
    pin_ml = p;
    pin_acts = p + b_ml;
  }
  if (n_ml) {
    RSF_HIP(hipMemcpyAsync(g->d_ml, pin_ml, b_ml, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(ml_kernel, dim3(grid1(c.n_loc)), dim3(256), 0, st, c, g->s, g->d_ml, n_ml);
    hipLaunchKernelGGL(ml_alive_kernel, dim3(1), dim3(64), 0, st, g->s, g->d_ml, n_ml);
  }
  hipLaunchKernelGGL(refute_kernel, dim3(grid1(c.S)), dim3(256), 0, st, c, g->s, g->round_base);
  RSF_DBG_SYNC(st, "refute_kernel");
  if (n_acts) {
    RSF_HIP(hipMemcpyAsync(g->d_acts, pin_acts, b_acts, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(originate_kernel, dim3(grid1(n_acts)), dim3(256), 0, st, c, g->s, g->d_acts, n_acts,
                       g->round_abase, g->d_act_status);
    RSF_DBG_SYNC(st, "originate_kernel");
  }
  g->last_n_acts = n_acts;
  if (pin_k >= 0) {  // the slot is free again once the stream has passed this point
    RSF_HIP(hipEventRecord(g->pin_ev[pin_k], st));
    g->pin_used[pin_k] = true;
  }
  RSF_HIP(hipGetLastError());
  mark(g, 1);
  return RSF_OK;
}

int rsf_gossip_rumor_block(rsf_gossip* g, void** p, uint64_t* bytes) {
  if (!g || !p || !bytes) return gerr("null argument");
  *p = g->s.rumors + (g->round_base & g->c.rmask);
  *bytes = (uint64_t)g->round_need * sizeof(rsf_rumor);
  return RSF_OK;
}

}  // extern "C"

// Emission in canonical order.  peers_kernel draws every sender's peers; a stable radix
// sort of the GROUPS (sender, peer) by receiver (n_loc * fanout keys, not records) fixes
// where each group's records go, so emit_kernel writes them in merge order directly:
// cap_t slots per group, in (receiver; sender, position) order, with the group's count.
// local: this context merges its own records (single context): also each receiver's
// range of groups for merge_kernel.  Otherwise the groups are compacted into one
// receiver-ordered record stream (packed into send_buf, n_valid) for the exchange.
// bucket mode (world > 0): emission straight into the destination shards' buckets
static Buckets send_buckets(rsf_gossip* g);
// emission by the queue layout: four slots per lane (65..256), one (64: FULL, or fewer); deep
// queues then run the members the heads could not decide through emit_deep_wave_kernel
template <bool BKT>
static int launch_emit(rsf_gossip* g, dim3 egrid, const Buckets& bk) {
  const GCfg& c = g->c;
  hipStream_t st = g->stream;
  const dim3 eb(kWave * RSF_EMIT_WPB);
  if (c.qcap > kWave) {
    hipLaunchKernelGGL(emit4_kernel<BKT>, dim3((unsigned)c.n_loc), dim3(kWave), 0, st, c, g->s, g->grp_key, g->grp_slot,
                       g->grp_cnt, g->stage_val, g->stage_dec, bk);
  } else if (c.deep) {
    // (the deferred-member lists were emptied by peers_kernel)
    // only the intent queue deep (the common configuration): the other queues' tail code is
    // compiled out of the emission
    const bool q0_only = c.tcap1 == 0 && c.tcap2 == 0;
#define RSF_EMIT_DEEP(FULL, M)                                                                                         \
  hipLaunchKernelGGL((emit_kernel_deep<BKT, FULL, M>), egrid, eb, 0, st, c, g->s, g->grp_key, g->grp_slot, g->grp_cnt, \
                     g->stage_val, g->stage_dec, bk)
    if (c.qcap == kWave) {
      if (q0_only) RSF_EMIT_DEEP(true, 1u);
      else RSF_EMIT_DEEP(true, 7u);
    } else {
      if (q0_only) RSF_EMIT_DEEP(false, 1u);
      else RSF_EMIT_DEEP(false, 7u);
    }
#undef RSF_EMIT_DEEP
    RSF_HIP(hipGetLastError());
    RSF_DBG_SYNC(st, "emit_kernel (deep)");
    // by capacity; the full depth last, with the members the smaller classes re-list (list 4)
    // after its own in the same launch.  (Run beside each other on two streams, the classes
    // were slower: a full-depth wave holds most of its CU's LDS, so the small classes' waves
    // could not share the CU.)
    hipLaunchKernelGGL((emit_deep_wave_kernel<BKT, kDeepTiny>), dim3(g->deep_blocks_tiny), dim3(kWave), 0, st, c, g->s,
                       g->grp_key, g->grp_slot, g->grp_cnt, g->stage_val, g->stage_dec, bk, 2u, g->d_counters + 55);
    hipLaunchKernelGGL((emit_deep_wave_kernel<BKT, kDeepSmall>), dim3(g->deep_blocks), dim3(kWave), 0, st, c, g->s,
                       g->grp_key, g->grp_slot, g->grp_cnt, g->stage_val, g->stage_dec, bk, 0u, g->d_counters + 55);
    hipLaunchKernelGGL((emit_deep_block_kernel<BKT, kDeepMid>), dim3(g->deep_blocks_mid), dim3(kDeepBlkThreads), 0, st, c,
                       g->s, g->grp_key, g->grp_slot, g->grp_cnt, g->stage_val, g->stage_dec, bk, 3u, g->d_counters + 55);
    hipLaunchKernelGGL((emit_deep_block_kernel<BKT, kDeepBig>), dim3(g->deep_blocks_big), dim3(kDeepBlkThreads), 0, st, c,
                       g->s, g->grp_key, g->grp_slot, g->grp_cnt, g->stage_val, g->stage_dec, bk, 1u, g->d_counters + 55);
  } else if (c.qcap == kWave) {
    hipLaunchKernelGGL((emit_kernel<BKT, true>), egrid, eb, 0, st, c, g->s, g->grp_key, g->grp_slot, g->grp_cnt,
                       g->stage_val, g->stage_dec, bk);
  } else {
    hipLaunchKernelGGL((emit_kernel<BKT, false>), egrid, eb, 0, st, c, g->s, g->grp_key, g->grp_slot, g->grp_cnt,
                       g->stage_val, g->stage_dec, bk);
  }
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

// after round t's emission (the last reader of grp_key / grp_slot): round t + 1's peers and
// group sort on the side stream
static int launch_ahead(rsf_gossip* g, uint32_t round) {
  if (!g->ahead_on) return RSF_OK;
  RSF_HIP(hipEventRecord(g->ev_emitted, g->stream));
  RSF_HIP(hipStreamWaitEvent(g->side, g->ev_emitted, 0));
  int rc = peers_and_sort(g, round + 1, g->side);
  // (also on an error: work already queued on the side stream may still write the group keys,
  // so the main stream must wait for it before their next use -- ahead_drop does)
  RSF_HIP(hipEventRecord(g->ev_ahead, g->side));
  g->ahead_launched = true;
  g->ahead_valid = rc == RSF_OK;
  if (rc) return rc;
  g->ahead_round = round + 1;
  return RSF_OK;
}

static int check_in_round(rsf_gossip* g, uint32_t round);
static int emit_and_sort(rsf_gossip* g, uint32_t round, bool local, uint32_t world = 0) {
  const GCfg& c = g->c;
  hipStream_t st = g->stream;
  const uint64_t ng = g->n_groups;
  if (g->round_need)
    hipLaunchKernelGGL(dec_fill_kernel, dim3(grid1(g->round_need)), dim3(256), 0, st, (const rsf_rumor*)g->s.rumors,
                       g->s.rdec, g->s.rbody, (uint64_t)(g->round_base & c.rmask), (uint64_t)g->round_need);
  RSF_DBG_SYNC(st, "dec_fill_kernel");
  // this round's peers and group order: drawn ahead under the previous round, or now
  const bool use_ahead = g->ahead_valid && g->ahead_round == round;
  if (g->ahead_launched) RSF_HIP(hipStreamWaitEvent(st, g->ev_ahead, 0));
  g->ahead_launched = g->ahead_valid = false;
  int rc;
  if (!use_ahead && (rc = peers_and_sort(g, round, st))) return rc;
  {
    // the emission's deferred-member lists, the group counts (buckets carry their own), the
    // segment bounds of the single-context merge: one launch
    ZeroSpans z{};
    int k = 0;
    if (c.deep) z.p[k] = g->s.deep_n, z.words[k++] = kDeepLists;
    if (!world) z.p[k] = g->grp_cnt, z.words[k++] = ng;
    if (local) {
      z.p[k] = g->seg_start, z.words[k++] = c.n_loc;
      z.p[k] = g->seg_end, z.words[k++] = c.n_loc;
    }
    uint64_t most = 0;
    for (int i = 0; i < k; ++i) most = std::max(most, z.words[i]);
    if (most) {
      hipLaunchKernelGGL(zero_spans_kernel, dim3((unsigned)std::min<uint64_t>(grid1(most), 2048)), dim3(256), 0, st, z);
      RSF_HIP(hipGetLastError());
    }
  }
  const dim3 egrid(grid1((c.n_loc + RSF_EMIT_PER_WAVE - 1) / RSF_EMIT_PER_WAVE, RSF_EMIT_WPB));
  if (world) {
    // buckets: the shard bounds first, then every group's slot word = (shard, place in bucket)
    // only a group's place inside its bucket must fit the slot word's index field
    if (g->bkt_gcap >= kBktIdxMask || world >= (1u << (32 - kBktWShift)))
      return gerr("bucket capacity too large for the slot encoding");
    const Buckets bk = send_buckets(g);
    hipLaunchKernelGGL(bucket_bounds_kernel, dim3(1), dim3(64), 0, st, (const uint32_t*)g->grp_key_s, ng, bk.per, world,
                       g->d_wstart, g->bkt_send, bk.stride_u32, bk.gcap, g->d_counters + 58);
    hipLaunchKernelGGL(grp_index_kernel, dim3(grid1(ng)), dim3(256), 0, st, g->grp_key_s, g->grp_id_s, ng, c.lo,
                       g->grp_slot, nullptr, nullptr, (const uint32_t*)g->d_wstart, (uint32_t)bk.per,
                       g->bkt_send + bk.keys_off, bk.stride_u32, bk.gcap);
    RSF_HIP(hipGetLastError());
    RSF_DBG_SYNC(st, "grp_index_kernel");
    mark(g, 2);
    if ((rc = launch_emit<true>(g, egrid, bk))) return rc;
    // the tick before the next round's peers start on the side stream: the prune's blocks
    // hold most of a CU's LDS and would only trade places with the sort's
    if ((rc = check_in_round(g, round))) return rc;
    if ((rc = launch_ahead(g, round))) return rc;
    mark(g, 3);
    return RSF_OK;
  }
  hipLaunchKernelGGL(grp_index_kernel, dim3(grid1(ng)), dim3(256), 0, st, g->grp_key_s, g->grp_id_s, ng, c.lo,
                     g->grp_slot, local ? g->seg_start : nullptr, local ? g->seg_end : nullptr);
  RSF_HIP(hipGetLastError());
  RSF_DBG_SYNC(st, "grp_index_kernel");
  mark(g, 2);
  if ((rc = launch_emit<false>(g, egrid, Buckets{}))) return rc;
  RSF_DBG_SYNC(st, "emit_kernel");
  // the counts path reads the sorted groups after the emission (grp_expand_kernel): no ahead
  if ((rc = check_in_round(g, round))) return rc;
  if (local && (rc = launch_ahead(g, round))) return rc;
  if (local) {
    unsigned long long* sum = (unsigned long long*)g->d_counters;
    const uint32_t* cnt = g->grp_cnt;
    int rc2 = rsf::cub_run(
        g->grp_tmp, st,
        [&](void* t, size_t& b) { return hipcub::DeviceReduce::Sum(t, b, cnt, sum, (int)ng, st); },
        "group count reduce");
    if (rc2) return rc2;
    RSF_DBG_SYNC(st, "group count reduce");
  } else {
    const uint32_t* cnt = g->grp_cnt;
    uint32_t* off = g->grp_off;
    int rc2 = rsf::cub_run(
        g->grp_tmp, st, [&](void* t, size_t& b) { return hipcub::DeviceScan::InclusiveSum(t, b, cnt, off, (int)ng, st); },
        "group count scan");
    if (rc2) return rc2;
    RSF_DBG_SYNC(st, "group count scan");
    RSF_HIP(hipMemsetAsync(g->d_counters, 0, 8, st));
    hipLaunchKernelGGL(grp_expand_kernel, dim3(grid1(ng * kLanesPerGroup)), dim3(256), 0, st, g->grp_key_s,
                       g->grp_off, ng, c.cap_t, g->stage_val, g->send_buf, g->d_counters);
    RSF_HIP(hipGetLastError());
  }
  mark(g, 3);
  return RSF_OK;
}

// grouped: the records are emit_kernel's groups (stage_val / stage_dec, cap_t slots, grp_cnt);
// otherwise a flat record stream (vals, rec_dec)
static BigList big_list(rsf_gossip* g) { return BigList{g->big_ids, g->d_counters + 52}; }
// merge_kernel over every receiver, then merge_big_kernel over the ones it deferred
template <bool RUNS>
static int merge_launch(rsf_gossip* g, const uint32_t* vals, const uint32_t* dec, const uint32_t* start,
                        const uint32_t* end, const uint32_t* gcnt, uint32_t stride, const Buckets& bk) {
  const GCfg& c = g->c;
  const BigList big = big_list(g);
  RSF_HIP(hipMemsetAsync(big.n, 0, 8, g->stream));
  const unsigned blocks = grid1((c.n_loc + RSF_MERGE_PER_WAVE - 1) / RSF_MERGE_PER_WAVE, kWavesPerBlock);
  hipLaunchKernelGGL(merge_kernel<RUNS>, dim3(blocks), dim3(kWave * kWavesPerBlock), 0, g->stream, c, g->s, vals, dec,
                     start, end, gcnt, stride, bk, big);
  RSF_DBG_SYNC(g->stream, "merge_kernel");
  hipLaunchKernelGGL(merge_big_kernel<RUNS>, dim3(std::min(g->merge_blocks, blocks)), dim3(kWave * kWavesPerBlock), 0,
                     g->stream, c, g->s, vals, dec, start, end, gcnt, stride, bk, big);
  RSF_HIP(hipGetLastError());
  RSF_DBG_SYNC(g->stream, "merge_big_kernel");
  return RSF_OK;
}

// grouped: the records are emit_kernel's groups (stage_val / stage_dec, cap_t slots, grp_cnt);
// otherwise a flat record stream (vals, rec_dec)
static int launch_merge(rsf_gossip* g, const uint32_t* vals, bool grouped = false) {
  const GCfg& c = g->c;
  int rc = merge_launch<false>(g, grouped ? g->stage_val : vals, grouped ? g->stage_dec : (const uint32_t*)g->rec_dec,
                               g->seg_start, g->seg_end, grouped ? g->grp_cnt : nullptr, grouped ? c.cap_t : 1u,
                               Buckets{});
  if (rc) return rc;
  mark(g, 4);
  return RSF_OK;
}

// ---- bucket exchange (multi-GPU without host synchronisation) -------------------------
static Buckets bucket_layout(const rsf_gossip* g, uint32_t world) {
  const GCfg& c = g->c;
  Buckets b{};
  b.gcap = g->bkt_gcap;
  b.keys_off = 4;
  b.cnt_off = b.keys_off + b.gcap;
  b.vals_off = b.cnt_off + b.gcap;
  b.decs_off = b.vals_off + b.gcap * c.cap_t;
  b.stride_u32 = ((uint64_t)b.decs_off + (uint64_t)b.gcap * c.cap_t + 63) & ~63ull;  // 256-B aligned buckets
  b.per = world ? c.N / world : c.N;
  b.n_runs = world;
  b.self_run = (uint32_t)(c.lo / b.per);
  return b;
}
static Buckets send_buckets(rsf_gossip* g) {
  Buckets b = bucket_layout(g, g->bkt_world);
  b.send = g->bkt_send;
  b.wstart = g->d_wstart;
  b.base = g->bkt_recv;
  return b;
}

static int segment_and_merge(rsf_gossip* g, const uint32_t* keys, const uint32_t* vals, uint64_t n) {
  const GCfg& c = g->c;
  hipStream_t st = g->stream;
  RSF_HIP(hipMemsetAsync(g->seg_start, 0, c.n_loc * 4, st));
  RSF_HIP(hipMemsetAsync(g->seg_end, 0, c.n_loc * 4, st));
  if (n) {
    hipLaunchKernelGGL(segment_kernel, dim3(grid1(n)), dim3(256), 0, st, keys, n, c.lo, g->seg_start, g->seg_end,
                       vals, (const uint32_t*)g->s.rdec, g->rec_dec, c.rmask);
  }
  return launch_merge(g, vals);
}

extern "C" {

int rsf_gossip_round(rsf_gossip* g, uint32_t round, const rsf_ml_event* ml, uint32_t n_ml, const rsf_action* acts,
                     uint32_t n_acts) {
  if (!g) return gerr("null context");
  if (g->c.n_loc != g->c.N) return gerr("sharded context: use round_begin / round_emit / round_merge");
  int rc = rsf_gossip_round_begin(g, round, ml, n_ml, acts, n_acts);
  if (rc) return rc;
  if ((rc = emit_and_sort(g, round, true))) return rc;
  g->merged_from_stage = true;
  g->merged_from_buckets = false;
  hipLaunchKernelGGL(accumulate_kernel, dim3(1), dim3(64), 0, g->stream, g->d_counters, 0u);
  return launch_merge(g, nullptr, true);
}

int rsf_gossip_bucket_buffers(rsf_gossip* g, uint32_t world, void** send, void** recv, uint64_t* bucket_bytes) {
  if (!g || !send || !recv || !bucket_bytes || world == 0 || world > kMaxRuns) return gerr("bad argument");
  const GCfg& c = g->c;
  if (c.N % world || c.n_loc != c.N / world) return gerr("shards must be equal contiguous ranges of n_members");
  if (world != g->bkt_world) {
    RSF_HIP(hipSetDevice(g->device));
    RSF_HIP(hipStreamSynchronize(g->stream));
    for (void* p : {(void*)g->bkt_send, (void*)g->bkt_recv, (void*)g->d_rstart, (void*)g->d_rend})
      if (p) hipFree(p);
    g->bkt_send = g->bkt_recv = g->d_rstart = g->d_rend = nullptr;
    g->bkt_world = 0;
    // groups per destination: n_loc * fanout / world for uniform peers; the capacity holds
    // 1/8 more plus 4096 (overflow is flagged, rsf_gossip_bucket_status)
    const uint64_t expect = (c.n_loc * c.fanout + world - 1) / world;
    const uint64_t gcap = std::min<uint64_t>(expect + expect / 8 + 4096, c.n_loc * c.fanout);
    if (gcap >= kBktIdxMask) return gerr("bucket capacity exceeds the slot word's 26-bit place field");
    if (gcap * (2 * c.cap_t + 2) + 64 >= (1ull << 32)) return gerr("a bucket exceeds 32-bit word offsets");
    g->bkt_gcap = (uint32_t)gcap;
    const Buckets b = bucket_layout(g, world);
    const size_t bytes = (size_t)b.stride_u32 * 4 * world;
    int rc;
    if ((rc = rsf::dmalloc((void**)&g->bkt_send, bytes)) || (rc = rsf::dmalloc((void**)&g->bkt_recv, bytes)) ||
        (rc = rsf::dmalloc((void**)&g->d_rstart, (size_t)world * c.n_loc * 4)) ||
        (rc = rsf::dmalloc((void**)&g->d_rend, (size_t)world * c.n_loc * 4)))
      return rc;
    if (!g->d_wstart && (rc = rsf::dmalloc((void**)&g->d_wstart, (kMaxRuns + 1) * 4))) return rc;
    RSF_HIP(hipMemset(g->bkt_send, 0, bytes));
    RSF_HIP(hipMemset(g->bkt_recv, 0, bytes));
    g->bkt_world = world;
  }
  *send = g->bkt_send;
  *recv = g->bkt_recv;
  *bucket_bytes = bucket_layout(g, world).stride_u32 * 4;
  return RSF_OK;
}

int rsf_gossip_round_emit_buckets(rsf_gossip* g, uint32_t world) {
  if (!g || world == 0 || world != g->bkt_world) return gerr("call rsf_gossip_bucket_buffers(world) first");
  RSF_HIP(hipSetDevice(g->device));
  int rc = emit_and_sort(g, g->cur_round, false, world);
  if (rc) return rc;
  g->merged_from_stage = false;
  g->merged_from_buckets = true;
  return RSF_OK;
}

int rsf_gossip_round_merge_buckets(rsf_gossip* g, uint32_t world) {
  if (!g || world == 0 || world != g->bkt_world) return gerr("call rsf_gossip_bucket_buffers(world) first");
  const GCfg& c = g->c;
  RSF_HIP(hipSetDevice(g->device));
  hipStream_t st = g->stream;
  const Buckets bk = send_buckets(g);
  {  // the runs' receiver ranges and the records-merged counter: one launch
    ZeroSpans z{};
    z.p[0] = g->d_rstart, z.words[0] = (uint64_t)world * c.n_loc;
    z.p[1] = g->d_rend, z.words[1] = (uint64_t)world * c.n_loc;
    z.p[2] = reinterpret_cast<uint32_t*>(g->d_counters + 57), z.words[2] = 2;
    hipLaunchKernelGGL(zero_spans_kernel, dim3((unsigned)std::min<uint64_t>(grid1(z.words[0]), 2048)), dim3(256), 0, st, z);
    RSF_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(bucket_index_kernel, dim3(std::min<uint64_t>(grid1((uint64_t)world * bk.gcap), kBucketIndexBlocks)),
                     dim3(256), 0, st, bk, c.lo, c.n_loc, g->d_rstart, g->d_rend, g->d_counters + 57,
                     g->d_counters + 58);
  hipLaunchKernelGGL(accumulate_kernel, dim3(1), dim3(64), 0, st, g->d_counters, 57u);
  if (g->profiling && g->prof_rounds < rsf_gossip::kMaxProfRounds)
    hipEventRecord(g->ev[g->prof_rounds][3], g->stream);  // exchange time lands in the sort slot
  int rc = merge_launch<true>(g, nullptr, nullptr, g->d_rstart, g->d_rend, nullptr, c.cap_t, bk);
  if (rc) return rc;
  mark(g, 4);
  return RSF_OK;
}

int rsf_gossip_bucket_status(rsf_gossip* g, int* ok) {
  if (!g || !ok) return gerr("null argument");
  unsigned long long f = 0;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(&f, g->d_counters + 58, 8, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  *ok = f == 0;
  return RSF_OK;
}

int rsf_gossip_round_emit(rsf_gossip* g, uint32_t world, uint64_t* send_counts) {
  if (!g || !send_counts || world == 0 || world > 32) return gerr("bad argument");  // d_counters[1..world+1]
  const GCfg& c = g->c;
  if (c.N % world || c.n_loc != c.N / world) return gerr("shards must be equal contiguous ranges of n_members");
  RSF_HIP(hipSetDevice(g->device));
  int rc = emit_and_sort(g, g->cur_round, false);
  if (rc) return rc;
  hipStream_t st = g->stream;
  // emit_and_sort left the stream packed in send_buf (grp_expand_kernel)
  hipLaunchKernelGGL(shard_bounds_kernel, dim3(1), dim3(64), 0, st, g->send_buf, g->d_counters, c.N / world, world,
                     g->d_counters + 1);
  RSF_HIP(hipGetLastError());
  unsigned long long b[64];
  RSF_HIP(hipMemcpyAsync(b, g->d_counters, (world + 2) * 8, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  for (uint32_t w = 0; w < world; ++w) send_counts[w] = b[1 + w + 1] - b[1 + w];
  g->merged_from_stage = false;
  g->merged_from_buckets = false;
  return RSF_OK;
}

int rsf_gossip_send_buffer(rsf_gossip* g, void** p, uint64_t* cap) {
  if (!g || !p) return gerr("null argument");
  *p = g->send_buf;
  if (cap) *cap = std::max(g->stage_cap, g->recv_cap);
  return RSF_OK;
}

// diagnostic (RSF_GUARD_ZONES builds): changed bytes in the guard zones, in the order before
// stage_dec, after stage_dec, before big_ids, after big_ids (synchronises); -1 without zones
int rsf_gossip_debug_zones(rsf_gossip* g, uint64_t* out4) {
  if (!g || !out4) return gerr("null argument");
  if (!kZone) return -1;
  RSF_HIP(hipStreamSynchronize(g->stream));
  const char* z[4] = {g->dec_base, g->dec_base + kZone + g->stage_cap * 4, g->big_base,
                      g->big_base + kZone + g->c.n_loc * 4};
  std::vector<uint8_t> v(kZone);
  for (int k = 0; k < 4; ++k) {
    RSF_HIP(hipMemcpy(v.data(), z[k], kZone, hipMemcpyDeviceToHost));
    uint64_t c = 0;
    for (uint8_t b : v) c += b != 0xA5;
    out4[k] = c;
  }
  return RSF_OK;
}

// the canaries past the hipCUB temporaries (rsf::CubTemp): radix sorts, group count
// reduce/scan, run-merge scan; 1 = intact (or never allocated), 0 = overrun (synchronises)
int rsf_gossip_debug_canaries(rsf_gossip* g, int* out3) {
  if (!g || !out3) return gerr("null argument");
  RSF_HIP(hipSetDevice(g->device));
  const rsf::CubTemp* t[3] = {&g->sort_tmp, &g->grp_tmp, &g->scan_tmp};
  for (int k = 0; k < 3; ++k) {
    const int r = t[k]->canary_intact(g->stream);
    if (r < 0) return r;
    out3[k] = r;
  }
  return RSF_OK;
}

// diagnostic only: device addresses of the context's main buffers and of a global in the
// library's code object (open issue: an address-dependent fault).  Order:
// view, p_ent, q_rumor, stage_val, stage_dec, grp_slot, grp_cnt, seg_start, rbody, rumors,
// rdec, clock, code-object global (0 without one), big_ids, sort_tmp, grp_tmp, d_counters,
// d_acts, grp_key, grp_key_s, grp_id, grp_id_s, grp_off, stage_key, sort_key, sort_val,
// send_buf, rec_dec, seg_end, p_cnt, err, member_subj.  Returns the count written.
int rsf_gossip_debug_ptrs(rsf_gossip* g, uint64_t* out, uint32_t n) {
  if (!g || !out) return gerr("null argument");
  const void* p[32] = {g->s.view, g->s.p_ent, g->s.q_rumor, g->stage_val, g->stage_dec, g->grp_slot, g->grp_cnt,
                       g->seg_start, g->s.rbody, g->s.rumors, g->s.rdec, g->s.clock, nullptr,
                       g->big_ids, g->sort_tmp.p, g->grp_tmp.p, g->d_counters, g->d_acts, g->grp_key, g->grp_key_s,
                       g->grp_id, g->grp_id_s, g->grp_off, g->stage_key, g->sort_key, g->sort_val, g->send_buf,
                       g->rec_dec, g->seg_end, g->s.p_cnt, g->s.err, g->s.member_subj};
#if RSF_MERGE_PROF || RSF_EMIT_PROF || RSF_CHECKS
  void* sym = nullptr;
  if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_merge_prof)) == hipSuccess) p[12] = sym;
#endif
  const uint32_t k = n < 32 ? n : 32;
  for (uint32_t i = 0; i < k; ++i) out[i] = (uint64_t)(uintptr_t)p[i];
  return (int)k;
}

// diagnostic only (experiments/deep_prof.py, builds with -DRSF_DEEP_PROF=1): reads and clears
// the deferral reasons, the deep wave kernel's phase totals and queue-size histogram (64 words);
// returns -1 in normal builds
int rsf_gossip_deep_prof(uint64_t* out64) {
#if RSF_DEEP_PROF
  RSF_HIP(hipDeviceSynchronize());
  RSF_HIP(hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_deep_prof), 80 * sizeof(uint64_t)));
  unsigned long long z[80] = {};
  RSF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_deep_prof), z, sizeof(z)));
  return 0;
#else
  (void)out64;
  return -1;
#endif
}

// diagnostic only (experiments/merge_prof.py, builds with -DRSF_MERGE_PROF=1): reads and
// clears merge_kernel's per-phase shader-clock totals; returns -1 in normal builds
int rsf_gossip_merge_prof(uint64_t* out8) {
#if RSF_MERGE_PROF || RSF_EMIT_PROF || RSF_CHECKS
  RSF_HIP(hipDeviceSynchronize());
  RSF_HIP(hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_merge_prof), 8 * sizeof(uint64_t)));
  unsigned long long z[8] = {};
  RSF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_merge_prof), z, sizeof(z)));
#if RSF_EMIT_PROF
  {
    std::vector<unsigned long long> w(512 * 8), zw(512 * 8, 0ull);
    RSF_HIP(hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_eprof), w.size() * sizeof(unsigned long long)));
    RSF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_eprof), zw.data(), zw.size() * sizeof(unsigned long long)));
    for (int i = 0; i < 8; ++i) {
      out8[i] = 0;
      for (int r = 0; r < 512; ++r) out8[i] += w[r * 8 + i];
    }
    RSF_HIP(hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_eprof2), w.size() * sizeof(unsigned long long)));
    RSF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_eprof2), zw.data(), zw.size() * sizeof(unsigned long long)));
    for (int i = 0; i < 5; ++i) {
      unsigned long long t = 0;
      for (int r = 0; r < 512; ++r) t += w[r * 8 + i];
      fprintf(stderr, "eprof2[%d] %llu\n", i, t);
    }
  }
#endif
  return RSF_OK;
#else
  (void)out8;
  return -1;
#endif
}

int rsf_gossip_round_merge(rsf_gossip* g, const uint64_t* recv, uint64_t n_recv) {
  if (!g || (n_recv && !recv)) return gerr("null argument");
  if (n_recv > g->recv_cap) return rsf::set_error(RSF_ERR_OVERFLOW, "receive buffer capacity exceeded");
  RSF_HIP(hipSetDevice(g->device));
  hipStream_t st = g->stream;
  if (n_recv) {
    hipLaunchKernelGGL(unpack_kernel, dim3(grid1(n_recv)), dim3(256), 0, st, recv, n_recv, g->stage_key, g->stage_val);
    int rc = sort_pairs(g, g->stage_key, g->sort_key, g->stage_val, g->sort_val, n_recv);
    if (rc) return rc;
  }
  g->last_merged = n_recv;
  g->total_merged_host += n_recv;
  if (!g->profiling) {
  } else if (g->prof_rounds < rsf_gossip::kMaxProfRounds) {
    hipEventRecord(g->ev[g->prof_rounds][3], g->stream);  // exchange time lands in the sort slot
  }
  return segment_and_merge(g, g->sort_key, g->sort_val, n_recv);
}

int rsf_gossip_round_merge_runs(rsf_gossip* g, const uint64_t* recv, const uint64_t* run_counts, uint32_t n_runs) {
  if (!g || (n_runs && !run_counts) || n_runs > 32) return gerr("bad argument");
  const GCfg& c = g->c;
  uint64_t off[63];
  off[0] = 0;
  for (uint32_t r = 0; r < n_runs; ++r) off[r + 1] = off[r] + run_counts[r];
  const uint64_t n = n_runs ? off[n_runs] : 0;
  if (n && !recv) return gerr("null argument");
  if (n > g->recv_cap) return rsf::set_error(RSF_ERR_OVERFLOW, "receive buffer capacity exceeded");
  RSF_HIP(hipSetDevice(g->device));
  hipStream_t st = g->stream;
  if (n_runs > g->run_cap) {
    for (void* p : {(void*)g->run_start, (void*)g->run_end, (void*)g->run_base})
      if (p) hipFree(p);
    g->run_start = g->run_end = g->run_base = nullptr;
    g->run_cap = 0;
    const size_t tab = (size_t)n_runs * c.n_loc * 4;
    int rc;
    if ((rc = rsf::dmalloc((void**)&g->run_start, tab)) || (rc = rsf::dmalloc((void**)&g->run_end, tab)) ||
        (rc = rsf::dmalloc((void**)&g->run_base, tab)))
      return rc;
    g->run_cap = n_runs;
  }
  if (!g->run_total) {
    int rc;
    if ((rc = rsf::dmalloc((void**)&g->run_total, c.n_loc * 4)) || (rc = rsf::dmalloc((void**)&g->d_run_off, 63 * 8)))
      return rc;
  }
  RSF_HIP(hipMemcpyAsync(g->d_run_off, off, (n_runs + 1) * 8, hipMemcpyHostToDevice, st));
  const size_t tab = (size_t)n_runs * c.n_loc * 4;
  RSF_HIP(hipMemsetAsync(g->run_start, 0, tab, st));
  RSF_HIP(hipMemsetAsync(g->run_end, 0, tab, st));
  RSF_HIP(hipMemsetAsync(g->d_counters + 62, 0, 8, st));
  if (n)
    hipLaunchKernelGGL(runs_bounds_kernel, dim3(grid1(n)), dim3(256), 0, st, recv, n, g->d_run_off, n_runs, c.lo,
                       c.n_loc, g->run_start, g->run_end, g->d_counters + 62);
  hipLaunchKernelGGL(runs_base_kernel, dim3(grid1(c.n_loc)), dim3(256), 0, st, n_runs, c.n_loc, g->run_start,
                     g->run_end, g->run_base, g->run_total);
  {
    const uint32_t* tot = g->run_total;
    uint32_t* seg = g->seg_start;
    const int nl = (int)c.n_loc;
    int rc = rsf::cub_run(
        g->scan_tmp, st, [&](void* t, size_t& b) { return hipcub::DeviceScan::ExclusiveSum(t, b, tot, seg, nl, st); },
        "run-merge segment scan");
    if (rc) return rc;
  }
  if (n)
    hipLaunchKernelGGL(runs_scatter_kernel, dim3(grid1(n)), dim3(256), 0, st, recv, n, g->d_run_off, n_runs, c.lo,
                       c.n_loc, g->run_start, g->run_base, g->seg_start, g->sort_val, (const uint32_t*)g->s.rdec,
                       g->rec_dec, c.rmask);
  hipLaunchKernelGGL(seg_end_kernel, dim3(grid1(c.n_loc)), dim3(256), 0, st, c.n_loc, g->seg_start, g->run_total,
                     g->seg_end);
  RSF_HIP(hipGetLastError());
  g->last_merged = n;
  g->total_merged_host += n;
  if (g->profiling && g->prof_rounds < rsf_gossip::kMaxProfRounds)
    hipEventRecord(g->ev[g->prof_rounds][3], g->stream);  // exchange time lands in the sort slot
  return launch_merge(g, g->sort_val);
}

static size_t pp_bytes_per_pair(const GCfg& c) {
  return (size_t)c.vrow + (size_t)c.ebuf * 12 + (size_t)c.ebuf * c.slot_k * 8 + 32;
}

int rsf_gossip_push_pull_device(rsf_gossip* g, const rsf_pp_pair* pairs, uint64_t n, uint32_t flags) {
  if (!g || (n && !pairs)) return gerr("null argument");
  if (n == 0) return RSF_OK;
  const GCfg& c = g->c;
  RSF_HIP(hipSetDevice(g->device));
  if (n > g->pp_cap) {
    if (g->pp_buf) {
      RSF_HIP(hipStreamSynchronize(g->stream));
      hipFree(g->pp_buf);
    }
    g->pp_buf = nullptr;
    g->pp_cap = 0;
    int rc = rsf::dmalloc(&g->pp_buf, pp_bytes_per_pair(c) * n);
    if (rc) return rc;
    g->pp_cap = n;
  }
  // slab regions, each 16-byte aligned
  char* b = (char*)g->pp_buf;
  PPSlab sl;
  sl.view = (ViewS*)b;
  b += (size_t)c.vrow * n;
  sl.eb_keys = (uint64_t*)b;
  b += (size_t)c.ebuf * c.slot_k * 8 * n;
  sl.eb_ltime = (uint64_t*)b;
  b += (size_t)c.ebuf * 8 * n;
  sl.clocks = (uint64_t*)b;
  b += (size_t)32 * n;
  sl.eb_cnt = (uint32_t*)b;
  hipLaunchKernelGGL(pp_snapshot_kernel, dim3((unsigned)n), dim3(256), 0, g->stream, c, g->s, pairs, sl);
  hipLaunchKernelGGL(pp_merge_kernel, dim3(grid1(n, kWavesPerBlock)), dim3(kWave * kWavesPerBlock), 0, g->stream, c,
                     g->s, pairs, n, sl, flags);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_gossip_push_pull(rsf_gossip* g, const rsf_pp_pair* pairs, uint64_t n, uint32_t flags) {
  if (!g || (n && !pairs)) return gerr("null argument");
  if (n == 0) return RSF_OK;
  if (n > 0x7FFFFFFFull) return gerr("batch too large");
  const GCfg& c = g->c;
  std::vector<uint32_t> rs(n);
  for (uint64_t i = 0; i < n; ++i) {
    const rsf_pp_pair& x = pairs[i];
    if (x.receiver < c.lo || x.receiver >= c.lo + c.n_loc || x.sender < c.lo || x.sender >= c.lo + c.n_loc)
      return gerr("push/pull members must be in the shard");
    rs[i] = x.receiver;
  }
  std::sort(rs.begin(), rs.end());
  if (std::adjacent_find(rs.begin(), rs.end()) != rs.end()) return gerr("receivers of one push/pull batch must be distinct");
  RSF_HIP(hipSetDevice(g->device));
  size_t bytes[1] = {n * sizeof(rsf_pp_pair)};
  void* d[1];
  int rc = g->scratch.take(bytes, 1, d);
  if (rc) return rc;
  RSF_HIP(hipMemcpyAsync(d[0], pairs, bytes[0], hipMemcpyHostToDevice, g->stream));
  if ((rc = rsf_gossip_push_pull_device(g, (const rsf_pp_pair*)d[0], n, flags))) return rc;
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_reap(rsf_gossip* g, uint32_t now, uint32_t reconnect_timeout, uint32_t tombstone_timeout,
                    uint32_t recent_intent_timeout) {
  if (!g) return gerr("null context");
  const GCfg& c = g->c;
  RSF_HIP(hipSetDevice(g->device));
  hipLaunchKernelGGL(reap_kernel, dim3(grid1(c.n_loc, kWavesPerBlock)), dim3(kWave * kWavesPerBlock), 0, g->stream, c,
                     g->s, now, reconnect_timeout, tombstone_timeout, recent_intent_timeout);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_gossip_set_now(rsf_gossip* g, uint32_t now) {
  if (!g) return gerr("null context");
  g->c.now = now;
  return RSF_OK;
}

// one checker tick at the members whose global id is phase mod period (period 1: all), on
// the engine's stream; reset: the stats block and the occupancy histogram start from zero
static int check_launch(rsf_gossip* g, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                        uint32_t period, uint32_t phase, bool reset) {
  hipStream_t rs = g->stream;
  const GCfg& c = g->c;
  // get_queue_max (base.rs:748-759): max_queue_depth, or (min_queue_depth > 0) per member
  // max(2 * members.states.len(), min_queue_depth) -- queue_max_kernel
  const uint32_t max_depth = max_queue_depth;
  RSF_HIP(hipSetDevice(g->device));
  int rc = flush_pending(g, period, phase);
  if (rc) return rc;
  if (min_queue_depth > 0) {
    if (!g->qmax && (rc = dmalloc((void**)&g->qmax, c.n_loc * 4))) return rc;
    hipLaunchKernelGGL(queue_max_kernel, dim3(grid1(std::max<uint64_t>(1, phase_count(c, period, phase)), 256 / kWave)),
                       dim3(256), 0, g->stream, c, g->s, min_queue_depth, g->qmax, period, phase);
    RSF_HIP(hipGetLastError());
  }
  const uint32_t* qmax = min_queue_depth > 0 ? g->qmax : nullptr;
  const size_t hist_words = 3 * (kOccBins + 1) + 3;
  if (!g->occ_hist) {
    if ((rc = dmalloc((void**)&g->occ_hist, hist_words * 4))) return rc;
    reset = true;
  }
  if (reset) {
    RSF_HIP(hipMemsetAsync(g->occ_hist, 0, hist_words * 4, rs));
    RSF_HIP(hipMemsetAsync(g->d_counters + 40, 0, 9 * 8, rs));
  }
  hipLaunchKernelGGL(check_queues_kernel,
                     dim3((unsigned)std::min<uint64_t>(1024, grid1(std::max<uint64_t>(1, phase_count(c, period, phase)),
                                                                   256 / kWave))),
                     dim3(256), 0, rs, c, g->s, max_depth, depth_warning, g->d_counters + 40, qmax, g->occ_hist, period,
                     phase);
  RSF_HIP(hipGetLastError());
  if (c.deep) {  // the deep queues over the max: the smallest max keys of head and tail kept
    const uint64_t n_list = phase_count(c, period, phase) * deep_queues(c);
    hipLaunchKernelGGL(check_stream_kernel, dim3(g->deep_check_blocks), dim3(kDeepThreads), 0, rs, c, g->s, max_depth,
                       qmax, (uint32_t)n_list);
    RSF_HIP(hipGetLastError());
  }
  return RSF_OK;
}

// the in-round checker ticks (rsf_gossip_set_checker): after round `round`'s emission, before
// its merge.  (Run on a second stream beside the merge, the prune and the merge each took
// longer and the round did not shorten: the prune's blocks hold most of a CU's LDS.)
static int check_in_round(rsf_gossip* g, uint32_t round) {
  if (!g->chk_period) return RSF_OK;
  return check_launch(g, g->chk_max, g->chk_min, g->chk_warn, g->chk_period, round % g->chk_period, false);
}

static int check_stats(rsf_gossip* g, uint64_t* num_queued, uint64_t* n_warn, uint64_t* n_pruned) {
  unsigned long long st[9];
  RSF_HIP(hipMemcpyAsync(st, g->d_counters + 40, sizeof(st), hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  for (int q = 0; q < 3; ++q) {
    if (num_queued) num_queued[q] = st[q];
    if (n_warn) n_warn[q] = st[3 + q];
    if (n_pruned) n_pruned[q] = st[6 + q];
  }
  return RSF_OK;
}

int rsf_gossip_check_queues(rsf_gossip* g, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                            uint64_t* num_queued, uint64_t* n_warn, uint64_t* n_pruned) {
  if (!g) return gerr("null context");
  int rc = check_launch(g, max_queue_depth, min_queue_depth, depth_warning, 1, 0, true);
  return rc ? rc : check_stats(g, num_queued, n_warn, n_pruned);
}

int rsf_gossip_check_queues_phase(rsf_gossip* g, uint32_t max_queue_depth, uint32_t min_queue_depth,
                                  uint32_t depth_warning, uint32_t period, uint32_t phase) {
  if (!g) return gerr("null context");
  if (!period || phase >= period) return gerr("phase must be below a non-zero period");
  return check_launch(g, max_queue_depth, min_queue_depth, depth_warning, period, phase, false);
}

int rsf_gossip_set_checker(rsf_gossip* g, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                           uint32_t period) {
  if (!g) return gerr("null context");
  RSF_HIP(hipSetDevice(g->device));
  g->chk_period = period;
  g->chk_max = max_queue_depth;
  g->chk_min = min_queue_depth;
  g->chk_warn = depth_warning;
  return rsf_gossip_checker_stats(g, nullptr, nullptr, nullptr, 1);
}

int rsf_gossip_checker_stats(rsf_gossip* g, uint64_t* num_queued, uint64_t* n_warn, uint64_t* n_pruned, int reset) {
  if (!g) return gerr("null context");
  RSF_HIP(hipSetDevice(g->device));
  const bool have = g->occ_hist != nullptr;
  int rc = RSF_OK;
  if (have) {
    rc = check_stats(g, num_queued, n_warn, n_pruned);
  } else {
    for (int q = 0; q < 3; ++q) {
      if (num_queued) num_queued[q] = 0;
      if (n_warn) n_warn[q] = 0;
      if (n_pruned) n_pruned[q] = 0;
    }
  }
  if (!rc && reset && have) {
    RSF_HIP(hipMemsetAsync(g->occ_hist, 0, (3 * (kOccBins + 1) + 3) * 4, g->stream));
    RSF_HIP(hipMemsetAsync(g->d_counters + 40, 0, 9 * 8, g->stream));
  }
  return rc;
}

int rsf_gossip_action_status(rsf_gossip* g, int32_t* status, uint32_t n) {
  if (!g || (n && !status)) return gerr("null argument");
  if (n > g->last_n_acts) return gerr("n exceeds the last round's action count");
  if (!n) return RSF_OK;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(status, g->d_act_status, (size_t)n * 4, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_checker_occupancy(rsf_gossip* g, uint32_t* hist, uint32_t* max3, uint32_t* bin, uint32_t* bins) {
  if (!g) return gerr("null context");
  if (bin) *bin = kOccBin;
  if (bins) *bins = kOccBins + 1;
  if (!hist && !max3) return RSF_OK;
  std::vector<uint32_t> h(3 * (kOccBins + 1) + 3, 0u);
  if (g->occ_hist) {
    RSF_HIP(hipSetDevice(g->device));
    RSF_HIP(hipMemcpyAsync(h.data(), g->occ_hist, h.size() * 4, hipMemcpyDeviceToHost, g->stream));
    RSF_HIP(hipStreamSynchronize(g->stream));
  }
  if (hist) std::copy(h.begin(), h.begin() + 3 * (kOccBins + 1), hist);
  if (max3) std::copy(h.begin() + 3 * (kOccBins + 1), h.end(), max3);
  return RSF_OK;
}

int rsf_gossip_flush(rsf_gossip* g) {
  if (!g) return gerr("null context");
  RSF_HIP(hipSetDevice(g->device));
  return flush_pending(g);
}

int rsf_gossip_pruned_total(rsf_gossip* g, int flush, uint64_t* total) {
  if (!g || !total) return gerr("null argument");
  RSF_HIP(hipSetDevice(g->device));
  int rc;
  if (flush && (rc = flush_pending(g))) return rc;
  std::vector<uint32_t> v(g->c.n_loc);
  RSF_HIP(hipMemcpyAsync(v.data(), g->s.q_pruned, g->c.n_loc * 4, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  uint64_t t = 0;
  for (uint32_t x : v) t += x;
  *total = t;
  return RSF_OK;
}

int rsf_gossip_dump_pruned(rsf_gossip* g, uint32_t* pruned, uint32_t* expired) {
  if (!g) return gerr("null context");
  RSF_HIP(hipSetDevice(g->device));
  int rc = flush_pending(g);
  if (rc) return rc;
  if (pruned) RSF_HIP(hipMemcpyAsync(pruned, g->s.q_pruned, g->c.n_loc * 4, hipMemcpyDeviceToHost, g->stream));
  if (expired) RSF_HIP(hipMemcpyAsync(expired, g->s.q_expired, g->c.n_loc * 4, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_set_delivery_log(rsf_gossip* g, uint32_t per_member) {
  if (!g) return gerr("null context");
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipStreamSynchronize(g->stream));
  if (g->s.dlog) hipFree(g->s.dlog);
  if (g->s.dmeta) hipFree(g->s.dmeta);
  if (g->s.dcnt) hipFree(g->s.dcnt);
  g->s.dlog = nullptr;
  g->s.dmeta = nullptr;
  g->s.dcnt = nullptr;
  g->c.dcap = 0;
  if (!per_member) return RSF_OK;
  int rc;
  if ((rc = rsf::dmalloc((void**)&g->s.dlog, (size_t)g->c.n_loc * per_member * 16)) ||
      (rc = rsf::dmalloc((void**)&g->s.dmeta, (size_t)g->c.n_loc * per_member)) ||
      (rc = rsf::dmalloc((void**)&g->s.dcnt, g->c.n_loc * 4)))
    return rc;
  RSF_HIP(hipMemsetAsync(g->s.dcnt, 0, g->c.n_loc * 4, g->stream));
  g->c.dcap = per_member;
  return RSF_OK;
}

int rsf_gossip_dump_deliveries(rsf_gossip* g, rsf_delivery* out, uint64_t cap, uint64_t* n_out) {
  if (!g || !n_out || (cap && !out)) return gerr("null argument");
  *n_out = 0;
  const GCfg& c = g->c;
  if (!c.dcap) return RSF_OK;
  std::vector<uint32_t> cnt(c.n_loc);
  std::vector<uint4> log((size_t)c.n_loc * c.dcap);
  std::vector<uint8_t> meta((size_t)c.n_loc * c.dcap);
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(cnt.data(), g->s.dcnt, c.n_loc * 4, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipMemcpyAsync(log.data(), g->s.dlog, log.size() * 16, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipMemcpyAsync(meta.data(), g->s.dmeta, meta.size(), hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  uint64_t o = 0;
  for (uint64_t l = 0; l < c.n_loc; ++l)
    for (uint32_t k = 0; k < std::min(cnt[l], c.dcap); ++k) {
      if (o >= cap) return rsf::set_error(RSF_ERR_OVERFLOW, "delivery dump capacity exceeded");
      const uint4 e = log[l * c.dcap + k];
      const uint64_t lt = ((uint64_t)e.y << 32) | e.x;
      rsf_delivery& d = out[o++];
      const uint8_t f = meta[l * c.dcap + k];
      const bool mev = (f & kLogMember) != 0;
      d.ltime = lt;
      d.key = ((uint64_t)e.w << 32) | e.z;
      d.member = (uint32_t)(c.lo + l);
      d.cc = (f & kLogCc) ? 1 : 0;
      d.kind = mev ? RSF_DELIVERY_MEMBER_EVENT : RSF_DELIVERY_USER_EVENT;
      d._r[0] = d._r[1] = 0;
    }
  *n_out = o;
  return RSF_OK;
}

int rsf_gossip_check_runs(rsf_gossip* g, int* ok) {
  if (!g || !ok) return gerr("null argument");
  unsigned long long bad = 0;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(&bad, g->d_counters + 62, 8, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  *ok = bad == 0;
  return RSF_OK;
}

int rsf_gossip_dump_members(rsf_gossip* g, uint64_t* clock, uint64_t* ec, uint64_t* qc, uint64_t* digest, uint32_t* err,
                            uint8_t* serf_state) {
  if (!g) return gerr("null context");
  const uint64_t n = g->c.n_loc;
  hipStream_t st = g->stream;
  RSF_HIP(hipSetDevice(g->device));
  int rc = flush_pending(g);  // queue-prune flags
  if (rc) return rc;
  if (clock) RSF_HIP(hipMemcpyAsync(clock, g->s.clock, n * 8, hipMemcpyDeviceToHost, st));
  if (ec) RSF_HIP(hipMemcpyAsync(ec, g->s.eclock, n * 8, hipMemcpyDeviceToHost, st));
  if (qc) RSF_HIP(hipMemcpyAsync(qc, g->s.qclock, n * 8, hipMemcpyDeviceToHost, st));
  if (digest) RSF_HIP(hipMemcpyAsync(digest, g->s.digest, n * 8, hipMemcpyDeviceToHost, st));
  if (err) RSF_HIP(hipMemcpyAsync(err, g->s.err, n * 4, hipMemcpyDeviceToHost, st));
  if (serf_state) RSF_HIP(hipMemcpyAsync(serf_state, g->s.serf_state, n, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  return RSF_OK;
}

int rsf_gossip_dump_view_rows(rsf_gossip* g, uint64_t row0, uint64_t rows, uint64_t* ltime, uint8_t* status,
                              uint8_t* kind, uint32_t* time) {
  if (!g || !ltime || !status || !kind) return gerr("null argument");
  if (row0 > g->c.n_loc || rows > g->c.n_loc - row0) return gerr("rows outside the shard");
  const uint64_t cnt = rows * g->c.S;
  const GCfg& c = g->c;
  std::vector<uint4> raw(rows * c.vrow / 16);
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(raw.data(), vrow_of(g->s, c, row0), rows * c.vrow, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  ViewS* const base = reinterpret_cast<ViewS*>(raw.data());
  for (uint64_t i = 0; i < cnt; ++i) {
    const ViewE v = *view_at(view_row(base, c.vrow, i / c.S), (uint32_t)(i % c.S));
    ltime[i] = v.ltime;
    status[i] = (uint8_t)(v.meta & 0xFF);
    kind[i] = (uint8_t)((v.meta >> 8) & 0xFF);
    if (time) time[i] = v.t;  // (mod 2^27)
  }
  return RSF_OK;
}

int rsf_gossip_dump_view(rsf_gossip* g, uint64_t* ltime, uint8_t* status, uint8_t* kind, uint32_t* time) {
  if (!g) return gerr("null argument");
  return rsf_gossip_dump_view_rows(g, 0, g->c.n_loc, ltime, status, kind, time);
}

// head and tail merged on the host into [n_loc][3][D] in send order
// every queue of local rows [r0, r0 + n) merged from head and tail (tail only on deep
// contexts), sorted, first D items; output row 0 = local row r0
static int dump_queues_deep(rsf_gossip* g, uint32_t D, uint32_t* rumor, uint32_t* seq, uint16_t* tx, uint16_t* len,
                            uint32_t* max_live, uint64_t r0 = 0, uint64_t rows = ~0ull) {
  const GCfg& c = g->c;
  const uint64_t n = std::min<uint64_t>(rows, c.n_loc - r0), hc = n * 3 * c.qcap;
  uint32_t most = 0;
  std::vector<uint32_t> hr(hc), hs(hc), ht(hc);
  std::vector<uint4> sum(n * 3);
  std::vector<std::vector<uint4>> tail(3);
  std::vector<uint64_t> tail0;  // the intent queue's packed items
  std::vector<uint32_t> nseq(n * 3);
  hipStream_t st = g->stream;
  const uint64_t h0 = r0 * 3 * c.qcap;
  RSF_HIP(hipMemcpyAsync(hr.data(), g->s.q_rumor + h0, hc * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(hs.data(), g->s.q_seq + h0, hc * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(ht.data(), g->s.q_txlen + h0, hc * 4, hipMemcpyDeviceToHost, st));
  // tails and their summaries exist only on deep contexts; otherwise every queue is its head
  if (c.deep) RSF_HIP(hipMemcpyAsync(sum.data(), g->s.tsum + r0 * 3, n * 3 * 16, hipMemcpyDeviceToHost, st));
  for (uint32_t q = 0; q < 3; ++q)
    if (tcap_of(c, q)) {
      if (q == 0) {
        tail0.resize(n * c.tstride0);
        RSF_HIP(hipMemcpyAsync(tail0.data(), g->s.tail0 + r0 * c.tstride0, tail0.size() * 8, hipMemcpyDeviceToHost, st));
      } else {
        tail[q].resize(n * tstride_of(c, q));
        RSF_HIP(hipMemcpyAsync(tail[q].data(), tail16(g->s, q) + r0 * tstride_of(c, q), tail[q].size() * 16,
                               hipMemcpyDeviceToHost, st));
      }
    }
  RSF_HIP(hipMemcpyAsync(nseq.data(), g->s.q_next_seq + r0 * 3, n * 3 * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  std::vector<std::pair<uint64_t, uint32_t>> items;
  for (uint64_t l = 0; l < n; ++l)
    for (uint32_t q = 0; q < 3; ++q) {
      items.clear();
      const uint64_t hb = (l * 3 + q) * c.qcap;
      for (uint32_t i = 0; i < c.qcap; ++i)
        if (hr[hb + i] != kEmpty) items.push_back({tlq_key(ht[hb + i] & 0xFFFF, ht[hb + i] >> 16, hs[hb + i]), hr[hb + i]});
      if (tcap_of(c, q))
        for (uint32_t i = 0; i < sum[l * 3 + q].x; ++i) {
          const uint4 e = q == 0 ? tail_unpack(c, tail0[l * c.tstride0 + i], nseq[l * 3])
                                 : tail[q][l * tstride_of(c, q) + i];
          items.push_back({tlq_key(e.z & 0xFFFF, e.z >> 16, e.y), e.x});
        }
      std::sort(items.begin(), items.end());
      most = std::max<uint32_t>(most, (uint32_t)items.size());
      const uint64_t ob = (l * 3 + q) * D;
      for (uint32_t i = 0; i < D; ++i) {
        const bool live = i < items.size();
        const uint64_t k = live ? items[i].first : 0ull;
        rumor[ob + i] = live ? items[i].second : kEmpty;
        seq[ob + i] = live ? 0xFFFFFFFFu - (uint32_t)k : 0u;
        tx[ob + i] = live ? (uint16_t)(k >> 48) : 0;
        len[ob + i] = live ? (uint16_t)(0xFFFF - ((k >> 32) & 0xFFFF)) : 0;
      }
    }
  if (max_live) *max_live = most;
  return RSF_OK;
}

int rsf_gossip_dump_queues_width(rsf_gossip* g, uint32_t width, uint32_t* rumor, uint32_t* seq, uint16_t* tx,
                                 uint16_t* len, uint32_t* next_seq, uint32_t* max_live) {
  if (!g || !rumor || !seq || !tx || !len || !next_seq || !width) return gerr("null argument");
  RSF_HIP(hipSetDevice(g->device));
  int rc = flush_pending(g);
  if (rc) return rc;
  RSF_HIP(hipMemcpyAsync(next_seq, g->s.q_next_seq, g->c.n_loc * 3 * 4, hipMemcpyDeviceToHost, g->stream));
  return dump_queues_deep(g, width, rumor, seq, tx, len, max_live);
}

int rsf_gossip_dump_queues_rows(rsf_gossip* g, uint64_t row0, uint64_t rows, uint32_t width, uint32_t* rumor,
                                uint32_t* seq, uint16_t* tx, uint16_t* len, uint32_t* max_live) {
  if (!g || !rumor || !seq || !tx || !len || !width || row0 + rows > g->c.n_loc) return gerr("bad argument");
  RSF_HIP(hipSetDevice(g->device));
  int rc = flush_pending(g);
  if (rc) return rc;
  return dump_queues_deep(g, width, rumor, seq, tx, len, max_live, row0, rows);
}

int rsf_gossip_dump_queues(rsf_gossip* g, uint32_t* rumor, uint32_t* seq, uint16_t* tx, uint16_t* len,
                           uint32_t* next_seq) {
  if (!g || !rumor || !seq || !tx || !len || !next_seq) return gerr("null argument");
  if (g->c.deep) {
    const uint32_t D = g->c.qcap + std::max(g->c.tcap0, std::max(g->c.tcap1, g->c.tcap2));
    return rsf_gossip_dump_queues_width(g, D, rumor, seq, tx, len, next_seq, nullptr);
  }
  const uint64_t cnt = g->c.n_loc * 3 * g->c.qcap;
  std::vector<uint32_t> tl(cnt);
  hipStream_t st = g->stream;
  RSF_HIP(hipSetDevice(g->device));
  int rc = flush_pending(g);
  if (rc) return rc;
  RSF_HIP(hipMemcpyAsync(rumor, g->s.q_rumor, cnt * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(seq, g->s.q_seq, cnt * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(tl.data(), g->s.q_txlen, cnt * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipMemcpyAsync(next_seq, g->s.q_next_seq, g->c.n_loc * 3 * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  for (uint64_t i = 0; i < cnt; ++i) {
    tx[i] = (uint16_t)(tl[i] & 0xFFFF);
    len[i] = (uint16_t)(tl[i] >> 16);
  }
  return RSF_OK;
}

int rsf_gossip_deep_stats(rsf_gossip* g, uint64_t* slow_total, uint64_t* slow_since_last) {
  if (!g) return gerr("null context");
  unsigned long long t = 0;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(&t, g->d_counters + 55, 8, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  if (slow_total) *slow_total = t;
  if (slow_since_last) *slow_since_last = t - g->deep_last;
  g->deep_last = t;
  return RSF_OK;
}

int rsf_gossip_deep_class_stats(rsf_gossip* g, uint64_t* out4) {
  if (!g || !out4) return gerr("null argument");
  unsigned long long t[8];
  RSF_HIP(hipSetDevice(g->device));
  // lists 0 (kDeepSmall), 1 (the full depth), 2 (kDeepTiny) at counters 55 - kDeepClassOff + list,
  // list 3 (kDeepMid) at 56
  RSF_HIP(hipMemcpyAsync(t, g->d_counters + 55 - kDeepClassOff, sizeof(t), hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  out4[0] = t[2];
  out4[1] = t[0];
  out4[2] = t[7];
  out4[3] = t[1];
  return RSF_OK;
}

int rsf_gossip_deep_full_items(rsf_gossip* g, uint64_t* sum, uint64_t* max) {
  if (!g || !sum || !max) return gerr("null argument");
  unsigned long long t[2] = {0, 0};
  RSF_HIP(hipSetDevice(g->device));
  if (g->c.deep) {
    RSF_HIP(hipMemcpyAsync(t, g->s.deep_n + kDeepFullItems, sizeof(t), hipMemcpyDeviceToHost, g->stream));
    RSF_HIP(hipStreamSynchronize(g->stream));
  }
  *sum = t[0];
  *max = t[1];
  return RSF_OK;
}

int rsf_gossip_dump_tails(rsf_gossip* g, uint32_t q, uint32_t* count, uint32_t* sealed) {
  if (!g || q > 2) return gerr("bad argument");
  const GCfg& c = g->c;
  const uint64_t n = c.n_loc;
  RSF_HIP(hipSetDevice(g->device));
  std::vector<uint4> ts(n * 3), tz(n * 3);
  if (c.deep) {
    RSF_HIP(hipMemcpyAsync(ts.data(), g->s.tsum, n * 3 * sizeof(uint4), hipMemcpyDeviceToHost, g->stream));
    RSF_HIP(hipMemcpyAsync(tz.data(), g->s.tseal, n * 3 * sizeof(uint4), hipMemcpyDeviceToHost, g->stream));
    RSF_HIP(hipStreamSynchronize(g->stream));
  }
  const bool dq = c.deep && tcap_of(c, q);
  for (uint64_t l = 0; l < n; ++l) {
    if (count) count[l] = dq ? ts[l * 3 + q].x : 0u;
    if (sealed) sealed[l] = dq ? std::min(tz[l * 3 + q].x, ts[l * 3 + q].x) : 0u;
  }
  return RSF_OK;
}

// per (member, queue): live items of the head (its leading slots) plus the tail's count
__global__ void __launch_bounds__(256) queue_lengths_kernel(GCfg c, GState s, uint32_t* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= c.n_loc * 3) return;
  const uint64_t base = t * c.qcap;
  uint32_t n = 0;
  while (n < c.qcap && s.q_rumor[base + n] != kEmpty) n++;
  if (tcap_of(c, (uint32_t)(t % 3))) n += s.tsum[t].x;
  out[t] = n;
}

int rsf_gossip_queue_lengths(rsf_gossip* g, uint32_t* out) {
  if (!g || !out) return gerr("null argument");
  const GCfg& c = g->c;
  RSF_HIP(hipSetDevice(g->device));
  int rc = flush_pending(g);
  if (rc) return rc;
  void* dv = nullptr;
  const size_t bytes = c.n_loc * 3 * sizeof(uint32_t);
  if ((rc = g->scratch.take(&bytes, 1, &dv))) return rc;
  uint32_t* d = (uint32_t*)dv;
  hipLaunchKernelGGL(queue_lengths_kernel, dim3(grid1(c.n_loc * 3)), dim3(256), 0, g->stream, c, g->s, d);
  RSF_HIP(hipGetLastError());
  RSF_HIP(hipMemcpyAsync(out, d, c.n_loc * 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_dump_buffers(rsf_gossip* g, uint64_t* eb_ltime, uint32_t* eb_cnt, uint64_t* eb_keys, uint64_t* qb_ltime,
                            uint32_t* qb_cnt, uint32_t* qb_ids) {
  if (!g) return gerr("null context");
  const GCfg& c = g->c;
  hipStream_t st = g->stream;
  RSF_HIP(hipSetDevice(g->device));
  if (eb_ltime) RSF_HIP(hipMemcpyAsync(eb_ltime, g->s.eb_ltime, c.n_loc * c.ebuf * 8, hipMemcpyDeviceToHost, st));
  if (eb_cnt) RSF_HIP(hipMemcpyAsync(eb_cnt, g->s.eb_cnt, c.n_loc * c.ebuf * 4, hipMemcpyDeviceToHost, st));
  if (eb_keys)
    RSF_HIP(hipMemcpyAsync(eb_keys, g->s.eb_keys, c.n_loc * c.ebuf * c.slot_k * 8, hipMemcpyDeviceToHost, st));
  if (qb_ltime) RSF_HIP(hipMemcpyAsync(qb_ltime, g->s.qb_ltime, c.n_loc * c.qbuf * 8, hipMemcpyDeviceToHost, st));
  if (qb_cnt) RSF_HIP(hipMemcpyAsync(qb_cnt, g->s.qb_cnt, c.n_loc * c.qbuf * 4, hipMemcpyDeviceToHost, st));
  if (qb_ids)
    RSF_HIP(hipMemcpyAsync(qb_ids, g->s.qb_ids, c.n_loc * c.qbuf * c.slot_k * 4, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  return RSF_OK;
}

int rsf_gossip_dump_rumors(rsf_gossip* g, uint32_t first, uint32_t count, rsf_rumor* out) {
  if (!g || (count && !out)) return gerr("null argument");
  if ((uint64_t)first + count > 2ull * g->max_rumors) return gerr("rumor range out of bounds");
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(out, g->s.rumors + first, (size_t)count * sizeof(rsf_rumor), hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_dump_refutes(rsf_gossip* g, uint32_t* count, uint64_t* ltimes) {
  if (!g || !count || !ltimes) return gerr("null argument");
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(count, g->s.refute_cnt, g->c.S * 4, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipMemcpyAsync(ltimes, g->s.refute_ltime, (size_t)g->c.S * g->c.max_refute * 8, hipMemcpyDeviceToHost,
                         g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

int rsf_gossip_set_profiling(rsf_gossip* g, int on) {
  if (!g) return gerr("null context");
  RSF_HIP(hipSetDevice(g->device));
  if (on && !g->events_made) {
    for (auto& row : g->ev)
      for (auto& e : row) RSF_HIP(hipEventCreate(&e));
    g->events_made = true;
  }
  g->profiling = on != 0;
  g->prof_rounds = 0;
  return RSF_OK;
}

int rsf_gossip_phase_times(rsf_gossip* g, double* ms_out, uint32_t* rounds_out) {
  if (!g || !ms_out) return gerr("null argument");
  for (int k = 0; k < rsf_gossip::kMarks - 1; ++k) ms_out[k] = 0.0;
  RSF_HIP(hipSetDevice(g->device));
  for (int r = 0; r < g->prof_rounds; ++r) {
    RSF_HIP(hipEventSynchronize(g->ev[r][rsf_gossip::kMarks - 1]));
    for (int k = 0; k + 1 < rsf_gossip::kMarks; ++k) {
      float ms = 0.f;
      RSF_HIP(hipEventElapsedTime(&ms, g->ev[r][k], g->ev[r][k + 1]));
      ms_out[k] += ms;
    }
  }
  if (rounds_out) *rounds_out = (uint32_t)g->prof_rounds;
  g->prof_rounds = 0;
  return RSF_OK;
}

int rsf_gossip_totals(rsf_gossip* g, uint64_t* merged_total) {
  if (!g || !merged_total) return gerr("null argument");
  unsigned long long t = 0;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(&t, g->d_counters + 60, 8, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  *merged_total = t + g->total_merged_host;
  return RSF_OK;
}

int rsf_gossip_last_round_stats(rsf_gossip* g, uint64_t* sent, uint64_t* merged) {
  if (!g) return gerr("null context");
  unsigned long long nv = 0;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(&nv, g->d_counters, 8, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  if (g->merged_from_buckets) {  // bucket exchange: this shard's merged records; emission is not summed
    RSF_HIP(hipMemcpyAsync(&nv, g->d_counters + 57, 8, hipMemcpyDeviceToHost, g->stream));
    RSF_HIP(hipStreamSynchronize(g->stream));
    if (sent) *sent = 0;
    if (merged) *merged = nv;
    return RSF_OK;
  }
  if (sent) *sent = nv;
  if (merged) *merged = g->merged_from_stage ? nv : g->last_merged;
  return RSF_OK;
}

}  // extern "C"

// ======================================================================================
// Snapshot log (core/src/snapshot.rs) and Reconnector (core/src/serf/base.rs:632-701)
// ======================================================================================
// Per member, the snapshotter's state lives beside the member state: the alive set as a
// bitset over subjects (updated by ml_kernel's Join / Leave / Failed member events), the
// largest delivered event / query ltime (h_user_event / h_query), the clock at a leave.
// The snapshot file is produced on demand in its compacted form (snapshot.rs:786-880):
// [Alive node]* Clock EventClock QueryClock, then after a leave: Leave and the shutdown
// clock.  Records: node [tag][u32 LE 4][u32 LE subject], clocks [tag][u64 LE].
namespace {

constexpr uint8_t kSnapAlive = 0, kSnapClock = 2, kSnapEventClock = 3, kSnapQueryClock = 4, kSnapLeave = 6;

__global__ void __launch_bounds__(256) snap_init_kernel(GCfg c, GState s) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= c.n_loc * c.snap_w) return;
  const uint64_t l = t / c.snap_w;
  const uint32_t k = (uint32_t)(t % c.snap_w);
  uint32_t bits = 0;
  for (uint32_t b = 0; b < 32; ++b) {
    const uint32_t j = k * 32 + b;
    if (j >= c.S) break;
    const uint32_t meta = ViewE(*vent(s, c, l, j)).meta;
    const uint32_t st = vstatus(meta);
    if (vkind(meta) == RSF_KIND_KNOWN && (st == RSF_STATUS_ALIVE || st == RSF_STATUS_LEAVING)) bits |= 1u << b;
  }
  s.snap_bits[t] = bits;
  if (k == 0) {
    for (int i = 0; i < 4; ++i) s.snap_sn[l * 4 + i] = 0;
  }
}

__device__ __forceinline__ uint64_t snap_now_clock(const GState& s, uint64_t l) {
  const uint64_t ck = s.clock[l];
  return ck ? ck - 1 : 0;  // update_clock: clock.time() - 1, saturating (snapshot.rs:713-720)
}

__global__ void __launch_bounds__(256) snap_size_kernel(GCfg c, GState s, uint64_t l0, uint64_t count,
                                                        uint64_t* __restrict__ sizes) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > count) return;
  if (i == count) {
    sizes[i] = 0;
    return;
  }
  const uint64_t l = l0 + i;
  uint64_t alive = 0;
  for (uint32_t k = 0; k < c.snap_w; ++k) alive += __popc(s.snap_bits[l * c.snap_w + k]);
  uint64_t b = alive * 9 + 27;
  const uint64_t* sn = s.snap_sn + l * 4;
  if (sn[3] & 1) b += 1 + (snap_now_clock(s, l) > sn[2] ? 9 : 0);
  sizes[i] = b;
}

__device__ __forceinline__ uint8_t* snap_put_clock(uint8_t* p, uint8_t tag, uint64_t t) {
  p[0] = tag;
  for (int i = 0; i < 8; ++i) p[1 + i] = (uint8_t)(t >> (8 * i));
  return p + 9;
}

__global__ void __launch_bounds__(256) snap_encode_kernel(GCfg c, GState s, uint64_t l0, uint64_t count,
                                                          const uint64_t* __restrict__ offs, uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint64_t l = l0 + i;
  uint8_t* p = out + offs[i];
  for (uint32_t k = 0; k < c.snap_w; ++k) {
    uint32_t w = s.snap_bits[l * c.snap_w + k];
    while (w) {
      const uint32_t j = k * 32 + (uint32_t)__builtin_ctz(w);
      w &= w - 1;
      p[0] = kSnapAlive;
      p[1] = 4;
      p[2] = p[3] = p[4] = 0;
      p[5] = (uint8_t)j;
      p[6] = (uint8_t)(j >> 8);
      p[7] = (uint8_t)(j >> 16);
      p[8] = (uint8_t)(j >> 24);
      p += 9;
    }
  }
  const uint64_t* sn = s.snap_sn + l * 4;
  const bool leaving = sn[3] & 1;
  const uint64_t now = snap_now_clock(s, l);
  p = snap_put_clock(p, kSnapClock, leaving ? sn[2] : now);
  p = snap_put_clock(p, kSnapEventClock, sn[0]);
  p = snap_put_clock(p, kSnapQueryClock, sn[1]);
  if (leaving) {
    *p++ = kSnapLeave;
    if (now > sn[2]) p = snap_put_clock(p, kSnapClock, now);  // the shutdown's update_clock
  }
}

// open_and_replay_snapshot (snapshot.rs:233-345) of one restarted member's file into
// scratch (bits, clocks); res = 0 or RSF_SNAP_ERR_*
__global__ void __launch_bounds__(256) snap_replay_kernel(GCfg c, const uint8_t* __restrict__ files,
                                                          const uint64_t* __restrict__ offs, uint32_t n,
                                                          uint32_t* __restrict__ bits, uint64_t* __restrict__ clk,
                                                          int32_t* __restrict__ res) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t* b = bits + (uint64_t)i * c.snap_w;
  uint64_t* ck = clk + (uint64_t)i * 3;
  for (uint32_t k = 0; k < c.snap_w; ++k) b[k] = 0;
  ck[0] = ck[1] = ck[2] = 0;
  const uint8_t* f = files + offs[i];
  const uint64_t len = offs[i + 1] - offs[i];
  uint64_t p = 0;
  int32_t rc = 0;
  while (p < len && !rc) {
    const uint8_t tag = f[p++];
    if (tag == 0 || tag == 1) {
      if (len - p < 4) { rc = RSF_SNAP_ERR_TRUNCATED; break; }
      const uint32_t nl = f[p] | f[p + 1] << 8 | f[p + 2] << 16 | (uint32_t)f[p + 3] << 24;
      p += 4;
      if (len - p < nl) { rc = RSF_SNAP_ERR_TRUNCATED; break; }
      if (nl != 4) { rc = RSF_SNAP_ERR_NODE; break; }
      const uint32_t j = f[p] | f[p + 1] << 8 | f[p + 2] << 16 | (uint32_t)f[p + 3] << 24;
      p += 4;
      if (j >= c.S) { rc = RSF_SNAP_ERR_NODE; break; }
      if (tag == 0) b[j >> 5] |= 1u << (j & 31);
      else b[j >> 5] &= ~(1u << (j & 31));
    } else if (tag >= 2 && tag <= 4) {
      if (len - p < 8) { rc = RSF_SNAP_ERR_TRUNCATED; break; }
      uint64_t t = 0;
      for (int k = 7; k >= 0; --k) t = (t << 8) | f[p + k];
      ck[tag - 2] = t;
      p += 8;
    } else if (tag == 5 || tag == 7) {
      // Coordinate / Comment: nothing to replay
    } else if (tag == 6) {
      if (c.snap_rejoin) continue;  // a previous leave is ignored when re-joining
      for (uint32_t k = 0; k < c.snap_w; ++k) b[k] = 0;
      ck[0] = ck[1] = ck[2] = 0;
    } else {
      rc = RSF_SNAP_ERR_RECORD;
    }
  }
  res[i] = rc;
}

// a fresh process for every restarted member whose file replayed: no member states or
// intents, no queued broadcasts, empty event / query buffers (one block per member)
__global__ void __launch_bounds__(256) snap_reset_kernel(GCfg c, GState s, const uint32_t* __restrict__ members,
                                                         const int32_t* __restrict__ res) {
  const uint32_t i = blockIdx.x;
  if (res[i] < 0) return;
  const uint64_t l = members[i] - c.lo;
  for (uint32_t j = threadIdx.x; j < c.S; j += blockDim.x) *vent(s, c, l, j) = ViewE{0ull, 0u, 0u};
  for (uint32_t j = threadIdx.x; j < 3 * c.qcap; j += blockDim.x) {
    s.q_rumor[l * 3 * c.qcap + j] = kEmpty;
    s.q_seq[l * 3 * c.qcap + j] = 0;
    s.q_txlen[l * 3 * c.qcap + j] = 0;
  }
  if (threadIdx.x < 3) s.q_next_seq[l * 3 + threadIdx.x] = 0;
  if (threadIdx.x < 3 && s.tsum) {  // deep queues: empty tails
    s.tsum[l * 3 + threadIdx.x] = kTSumEmpty;
    s.tseal[l * 3 + threadIdx.x] = kTSumEmpty;
  }
  if (threadIdx.x == 0) s.p_cnt[l] = 0;  // nothing pending either
  for (uint32_t j = threadIdx.x; j < c.ebuf; j += blockDim.x) {
    s.eb_ltime[l * c.ebuf + j] = 0;
    s.eb_cnt[l * c.ebuf + j] = 0;
  }
  for (uint32_t j = threadIdx.x; j < c.ebuf * c.slot_k; j += blockDim.x) s.eb_keys[l * c.ebuf * c.slot_k + j] = 0;
  for (uint32_t j = threadIdx.x; j < c.qbuf; j += blockDim.x) {
    s.qb_ltime[l * c.qbuf + j] = 0;
    s.qb_cnt[l * c.qbuf + j] = 0;
  }
  for (uint32_t j = threadIdx.x; j < c.qbuf * c.slot_k; j += blockDim.x) s.qb_ids[l * c.qbuf * c.slot_k + j] = 0;
}

// Serf::new with a snapshot (base.rs:122-204): clocks start at 1 and witness the replayed
// ones, events / queries up to the replayed clocks are not delivered again, the
// snapshotter continues from the replay; then handle_rejoin (base.rs:1741-1770):
// memberlist.join to the replayed nodes until one is up, after which memberlist's state
// exchange notifies a join of every live member (res = 1 rejoined, 0 alone)
__global__ void __launch_bounds__(256) snap_restart_kernel(GCfg c, GState s, const uint32_t* __restrict__ members,
                                                           uint32_t n, const uint32_t* __restrict__ bits,
                                                           const uint64_t* __restrict__ clk,
                                                           int32_t* __restrict__ res) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || res[i] < 0) return;
  const uint64_t l = members[i] - c.lo;
  const uint64_t* ck = clk + (uint64_t)i * 3;
  MRegs r;
  load_regs(s, l, r);
  r.clock = r.eclock = r.qclock = 1;
  witness(r.clock, ck[0]);
  witness(r.eclock, ck[1]);
  witness(r.qclock, ck[2]);
  r.serf_state = kSerfAlive;
  s.emin[l] = ck[1] + 1;
  s.qmin[l] = ck[2] + 1;
  if (r.subj >= 0) s.refute_cnt[r.subj] = 0;
  uint32_t* row = s.snap_bits + l * c.snap_w;
  for (uint32_t k = 0; k < c.snap_w; ++k) row[k] = bits[(uint64_t)i * c.snap_w + k];
  uint64_t* sn = s.snap_sn + l * 4;
  sn[0] = ck[1];
  sn[1] = ck[2];
  sn[2] = 0;
  sn[3] = 0;
  bool joined = false;
  for (uint32_t j = 0; j < c.S && !joined; ++j)
    if ((row[j >> 5] >> (j & 31) & 1) && (int32_t)j != r.subj && s.alive[s.subj_member[j]]) joined = true;
  if (joined)
    for (uint32_t j = 0; j < c.S; ++j)
      if ((int32_t)j != r.subj && s.alive[s.subj_member[j]]) {
        h_node_join(vent(s, c, l, j), r, j);
        snap_member(c, s, l, j, true);
        mlog_put(c, s, l, r.err, kEvJoin, j);
      }
  store_regs(s, l, r);
  res[i] = joined ? 1 : 0;
}

// Reconnector tick (base.rs:647-690), one wave per member: count the failed / left
// members of the view; with probability num_failed / max(states.len() - failed - left, 1)
// (base.rs:670-671) try a uniformly drawn failed member; the try succeeds when that member
// is up, and memberlist's join then notifies handle_node_join.  states.len() is every
// member the node knows: the N - S untracked members (implicitly Alive, the local node
// among them when it is not a subject), the local node when it is a subject, and the
// tracked subjects whose entry is KNOWN.
__global__ void __launch_bounds__(256) reconnect_kernel(GCfg c, GState s, uint32_t tick, uint32_t* __restrict__ target) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t l = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  if (l >= c.n_loc) return;
  const uint32_t m = (uint32_t)(c.lo + l);
  if (target && lane == 0) target[l] = kEmpty;
  if (!s.alive[m]) return;
  const int32_t own = s.member_subj[l];
  const ViewS* row = vrow_of(s, c, l);
  uint32_t failed = 0, left = 0;
  uint64_t known = (c.N - c.S) + (own >= 0 ? 1u : 0u);  // members.states: see above
  for (uint32_t j0 = 0; j0 < c.S; j0 += kWave) {
    const uint32_t j = j0 + lane;
    uint32_t meta = 0;
    if (j < c.S && (int32_t)j != own) meta = ViewE(*view_at(row, j)).meta;
    const bool kn = vkind(meta) == RSF_KIND_KNOWN;
    known += (uint32_t)__popcll(ballot(kn));
    failed += (uint32_t)__popcll(ballot(kn && vstatus(meta) == RSF_STATUS_FAILED));
    left += (uint32_t)__popcll(ballot(kn && vstatus(meta) == RSF_STATUS_LEFT));
  }
  if (!failed) return;
  uint64_t alive_n = known - failed - left;
  if (alive_n < 1) alive_n = 1;
  const float prob = __fdiv_rn((float)failed, (float)alive_n);  // usize as f32: round to nearest
  const u32x4 o = philox4x32_10(0, kPurposeReconnect << 24, m, tick, c.k0, c.k1);
  const float rr = (float)(o.x >> 8) * (1.0f / 16777216.0f);  // rng.gen::<f32>()
  if (rr > prob) return;
  uint32_t idx = mulhi32(o.y, failed);  // gen_range(0..num_failed)
  uint32_t tj = kEmpty;
  for (uint32_t j0 = 0; j0 < c.S && tj == kEmpty; j0 += kWave) {
    const uint32_t j = j0 + lane;
    uint32_t meta = 0;
    if (j < c.S && (int32_t)j != own) meta = ViewE(*view_at(row, j)).meta;
    const bool fa = vkind(meta) == RSF_KIND_KNOWN && vstatus(meta) == RSF_STATUS_FAILED;
    const unsigned long long mask = ballot(fa);
    const uint32_t cnt = (uint32_t)__popcll(mask);
    if (idx < cnt) {
      const bool hit = fa && (uint32_t)__popcll(mask & ((1ull << lane) - 1)) == idx;
      const unsigned long long hm = ballot(hit);
      tj = j0 + (uint32_t)__builtin_ctzll(hm);
    } else {
      idx -= cnt;
    }
  }
  if (lane != 0) return;
  if (target) target[l] = tj;
  if (!s.alive[s.subj_member[tj]]) return;
  MRegs r;
  load_regs(s, l, r);
  h_node_join(vent(s, c, l, tj), r, tj);
  snap_member(c, s, l, tj, true);
  mlog_put(c, s, l, r.err, kEvJoin, tj);
  store_regs(s, l, r);
}

}  // namespace

extern "C" {

int rsf_gossip_enable_snapshot(rsf_gossip* g, int rejoin_after_leave) {
  if (!g) return gerr("null context");
  GCfg& c = g->c;
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipStreamSynchronize(g->stream));
  if (g->s.snap_bits) hipFree(g->s.snap_bits);
  if (g->s.snap_sn) hipFree(g->s.snap_sn);
  g->s.snap_bits = nullptr;
  g->s.snap_sn = nullptr;
  c.snap_w = (c.S + 31) / 32;
  c.snap_rejoin = rejoin_after_leave ? 1 : 0;
  int rc;
  if ((rc = rsf::dmalloc((void**)&g->s.snap_bits, c.n_loc * c.snap_w * 4)) ||
      (rc = rsf::dmalloc((void**)&g->s.snap_sn, c.n_loc * 32)))
    return rc;
  const uint64_t nt = c.n_loc * c.snap_w;
  hipLaunchKernelGGL(snap_init_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, g->stream, c, g->s);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_gossip_snapshot_encode(rsf_gossip* g, uint64_t first, uint64_t count, uint64_t* offsets, uint8_t* out,
                               uint64_t out_cap, uint64_t* total) {
  if (!g || !offsets || !total) return gerr("null argument");
  const GCfg& c = g->c;
  if (!g->s.snap_bits) return gerr("snapshot not enabled (rsf_gossip_enable_snapshot)");
  if (first < c.lo || first + count > c.lo + c.n_loc || count == 0 || count > 0x7FFFFFFFull)
    return gerr("member range outside this context's shard");
  RSF_HIP(hipSetDevice(g->device));
  hipStream_t st = g->stream;
  const uint64_t l0 = first - c.lo;
  uint64_t* sizes = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  int rc;
  if ((rc = rsf::dmalloc((void**)&sizes, (count + 1) * 8))) return rc;
  hipLaunchKernelGGL(snap_size_kernel, dim3((unsigned)((count + 256) / 256)), dim3(256), 0, st, c, g->s, l0, count,
                     sizes);
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb, sizes, offsets, (int)(count + 1), st) != hipSuccess ||
      (rc = rsf::dmalloc(&tmp, tb)) ||
      hipcub::DeviceScan::ExclusiveSum(tmp, tb, sizes, offsets, (int)(count + 1), st) != hipSuccess) {
    hipFree(sizes);
    if (tmp) hipFree(tmp);
    return rc ? rc : rsf::set_error(RSF_ERR_HIP, "snapshot offset scan failed");
  }
  RSF_HIP(hipMemcpyAsync(total, offsets + count, 8, hipMemcpyDeviceToHost, st));
  RSF_HIP(hipStreamSynchronize(st));
  hipFree(sizes);
  hipFree(tmp);
  if (!out) return RSF_OK;
  if (*total > out_cap) return rsf::set_error(RSF_ERR_OVERFLOW, "snapshot output capacity exceeded");
  hipLaunchKernelGGL(snap_encode_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, c, g->s, l0, count,
                     (const uint64_t*)offsets, out);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_gossip_restart(rsf_gossip* g, const uint32_t* members, uint32_t n, const uint8_t* files,
                       const uint64_t* offsets, int32_t* result) {
  if (!g || (n && (!members || !offsets || !result))) return gerr("null argument");
  const GCfg& c = g->c;
  if (!g->s.snap_bits) return gerr("snapshot not enabled (rsf_gossip_enable_snapshot)");
  if (!n) return RSF_OK;
  std::vector<uint32_t> sorted(members, members + n);
  std::sort(sorted.begin(), sorted.end());
  for (uint32_t i = 0; i < n; ++i) {
    if (sorted[i] < c.lo || sorted[i] >= c.lo + c.n_loc) return gerr("restarted member outside this shard");
    if (i && sorted[i] == sorted[i - 1]) return gerr("a member is restarted twice in one call");
    if (offsets[i + 1] < offsets[i]) return gerr("snapshot offsets must not decrease");
  }
  const uint64_t bytes = offsets[n] - offsets[0];
  if (bytes && !files) return gerr("null snapshot files");
  std::vector<uint64_t> offs(n + 1);
  for (uint32_t i = 0; i <= n; ++i) offs[i] = offsets[i] - offsets[0];
  RSF_HIP(hipSetDevice(g->device));
  // the restarted processes' queues are dropped: what was pending reaches them first, as
  // the reference queued it when the messages arrived (its prunes are counted)
  int frc = flush_pending(g);
  if (frc) return frc;
  hipStream_t st = g->stream;
  uint32_t *d_mem = nullptr, *d_bits = nullptr;
  uint64_t *d_offs = nullptr, *d_clk = nullptr;
  uint8_t* d_files = nullptr;
  int32_t* d_res = nullptr;
  int rc;
  auto release = [&]() {
    for (void* p : {(void*)d_mem, (void*)d_bits, (void*)d_offs, (void*)d_clk, (void*)d_files, (void*)d_res})
      if (p) hipFree(p);
  };
  if ((rc = rsf::dmalloc((void**)&d_mem, (size_t)n * 4)) || (rc = rsf::dmalloc((void**)&d_bits, (size_t)n * c.snap_w * 4)) ||
      (rc = rsf::dmalloc((void**)&d_offs, (size_t)(n + 1) * 8)) || (rc = rsf::dmalloc((void**)&d_clk, (size_t)n * 24)) ||
      (rc = rsf::dmalloc((void**)&d_files, std::max<uint64_t>(bytes, 1))) || (rc = rsf::dmalloc((void**)&d_res, (size_t)n * 4))) {
    release();
    return rc;
  }
  bool ok = hipMemcpyAsync(d_mem, members, (size_t)n * 4, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_offs, offs.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, st) == hipSuccess &&
            (!bytes || hipMemcpyAsync(d_files, files + offsets[0], bytes, hipMemcpyHostToDevice, st) == hipSuccess);
  if (ok) {
    hipLaunchKernelGGL(snap_replay_kernel, dim3((n + 255) / 256), dim3(256), 0, st, c, (const uint8_t*)d_files,
                       (const uint64_t*)d_offs, n, d_bits, d_clk, d_res);
    hipLaunchKernelGGL(snap_reset_kernel, dim3(n), dim3(256), 0, st, c, g->s, (const uint32_t*)d_mem,
                       (const int32_t*)d_res);
    hipLaunchKernelGGL(snap_restart_kernel, dim3((n + 255) / 256), dim3(256), 0, st, c, g->s, (const uint32_t*)d_mem,
                       n, (const uint32_t*)d_bits, (const uint64_t*)d_clk, d_res);
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(result, d_res, (size_t)n * 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
  }
  release();
  return ok ? RSF_OK : rsf::set_error(RSF_ERR_HIP, "snapshot restart failed");
}

int rsf_gossip_reconnect(rsf_gossip* g, uint32_t tick, uint32_t* target) {
  if (!g) return gerr("null context");
  const GCfg& c = g->c;
  RSF_HIP(hipSetDevice(g->device));
  const uint64_t threads = c.n_loc * kWave;
  hipLaunchKernelGGL(reconnect_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, g->stream, c, g->s, tick,
                     target);
  RSF_HIP(hipGetLastError());
  return RSF_OK;
}

int rsf_gossip_dump_snapshot(rsf_gossip* g, uint32_t* bits, uint64_t* state) {
  if (!g || !bits || !state) return gerr("null argument");
  const GCfg& c = g->c;
  if (!g->s.snap_bits) return gerr("snapshot not enabled (rsf_gossip_enable_snapshot)");
  RSF_HIP(hipSetDevice(g->device));
  RSF_HIP(hipMemcpyAsync(bits, g->s.snap_bits, c.n_loc * c.snap_w * 4, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipMemcpyAsync(state, g->s.snap_sn, c.n_loc * 32, hipMemcpyDeviceToHost, g->stream));
  RSF_HIP(hipStreamSynchronize(g->stream));
  return RSF_OK;
}

}  // extern "C"
