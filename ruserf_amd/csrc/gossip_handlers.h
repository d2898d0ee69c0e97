// gossip_handlers.h — device restatement of ruserf's member-state merge and
// dissemination handlers.  Scalar (one lane) code; the kernels in gossip.hip
// call it from thread-per-item or lane-0-of-a-wave contexts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ruserf_amd.h"
#include "common.h"

namespace rsf {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint32_t kMinMsgLen = 18;  // smallest encoded message of the length model
constexpr uint64_t kDigUser = 0x1000000000000000ull;
constexpr uint64_t kDigQuery = 0x2000000000000000ull;
constexpr uint64_t kDigMember = 0x3000000000000000ull;
enum : uint32_t { kEvJoin = 0, kEvLeave = 1, kEvFailed = 2, kEvReap = 3, kEvUpdate = 4 };
constexpr uint32_t kFEvShift = 8;  // h_node_leave: its MemberEventType in bits 8..10 of the result
enum : uint32_t { kQIntent = 0, kQQuery = 1, kQEvent = 2 };
enum : uint32_t {
  kErrEvSlot = RSF_E_EVSLOT,
  kErrQSlot = RSF_E_QSLOT,
  kErrRefute = RSF_E_REFUTE,
  kErrStage = RSF_E_STAGE,
  kErrQueue = RSF_E_QUEUE_PRUNE,
  kErrDlog = RSF_E_DELIVERY_LOG
};
enum : uint8_t { kSerfAlive = 0, kSerfLeaving = 1, kSerfLeft = 2, kSerfShutdown = 3 };

struct GCfg {
  uint64_t N, lo, n_loc;
  uint32_t S, qcap, ebuf, qbuf, slot_k, fanout, limit, overhead, tx_limit, max_refute, cap_t;
  uint32_t k0, k1;
  uint32_t now;  // time stamped into view entries (leave_time / intent wall time); = the round
  // rumor ring: max_rumors = 2^rbits slots per generation; a rumor id is generation << rbits | slot,
  // stored at id & rmask (rmask = 2^(rbits+1) - 1: two generations resident, by parity)
  uint32_t rbits, rmask;
  uint32_t dcap;  // delivery log entries per member (0: log off)
  uint32_t snap_w, snap_rejoin;  // snapshotter: bitset words per member, rejoin_after_leave
  // deep queues (qcap <= 64 head + HBM tail): tail capacity per queue (0: none) and the tail
  // row stride (capacity + room for one emission's spills before its capacity check)
  // (named per queue, not arrays: a select between array elements is compiled back into a
  // dynamic index of a private copy, which goes to scratch or LDS)
  uint32_t tcap0, tcap1, tcap2, tstride0, tstride1, tstride2;
  uint32_t deep;  // any tail
  uint32_t max_ue, query_limit;  // Options::max_user_event_size / query_size_limit (origination checks)
  uint32_t gen;  // the rumor ring's current generation (rebuilds the intent tail's packed rumor ids)
  uint64_t vrow;  // bytes of a member's view row (view_row_bytes(S))
};

// view entry: members.states[subject] (status, status_time) or recent_intents[subject] --
// the register form the handlers work on
struct ViewE {
  uint64_t ltime;
  uint32_t meta;  // status | kind << 8
  uint32_t t;     // leave_time of a Failed/Left member, wall time of a buffered intent (base.rs:1355, 1364, 1813)
};
// ... and its 12-B form in HBM: the Lamport time whole, and one word for the time stamp (27 bits),
// the status (3 bits) and the kind (2 bits).  Time stamps are kept mod 2^27 (rounds): the
// reaper's ages (now - stamp) are exact while below 2^27 rounds, and the dumps return the
// stamp mod 2^27.
constexpr uint32_t kViewTBits = 27;
constexpr uint32_t kViewTMask = (1u << kViewTBits) - 1;
struct ViewS {
  uint32_t lo, hi, mt;
  RSF_HD operator ViewE() const {
    ViewE v;
    v.ltime = ((uint64_t)hi << 32) | lo;
    v.meta = ((mt >> 27) & 7u) | ((mt >> 30) << 8);
    v.t = mt & kViewTMask;
    return v;
  }
  RSF_HD ViewS& operator=(const ViewE& v) {
    lo = (uint32_t)v.ltime;
    hi = (uint32_t)(v.ltime >> 32);
    mt = (v.t & kViewTMask) | ((v.meta & 7u) << 27) | (((v.meta >> 8) & 3u) << 30);
    return *this;
  }
};
static_assert(sizeof(ViewS) == 12, "12-B view entries");
// A member's row: five entries to each 64-B sector (60 B + 4 B of padding), so no entry
// straddles a sector (a random entry is one sector read and one written back, as with 16-B
// entries) at 12.8 B per entry.
constexpr uint32_t kViewPerSector = 5;
RSF_HD uint64_t view_row_bytes(uint32_t S) { return (uint64_t)((S + kViewPerSector - 1) / kViewPerSector) * 64u; }
RSF_HD ViewS* view_at(ViewS* row, uint32_t subj) {
  return reinterpret_cast<ViewS*>(reinterpret_cast<char*>(row) + (uint64_t)(subj / kViewPerSector) * 64u +
                                  (subj % kViewPerSector) * 12u);
}
RSF_HD const ViewS* view_at(const ViewS* row, uint32_t subj) {
  return reinterpret_cast<const ViewS*>(reinterpret_cast<const char*>(row) + (uint64_t)(subj / kViewPerSector) * 64u +
                                        (subj % kViewPerSector) * 12u);
}
RSF_HD ViewS* view_row(ViewS* base, uint64_t row_bytes, uint64_t l) {
  return reinterpret_cast<ViewS*>(reinterpret_cast<char*>(base) + l * row_bytes);
}

struct GState {
  uint64_t *clock, *eclock, *qclock, *emin, *qmin, *digest;
  uint32_t* err;
  uint8_t* alive;  // [N] global liveness
  uint8_t* serf_state;
  int32_t* member_subj;
  uint32_t* subj_member;  // [S]
  uint32_t* refute_cnt;   // [S]
  uint64_t* refute_ltime; // [S][max_refute]
  ViewS* view;            // [n_loc] rows of vrow bytes: S 12-B entries, five to a 64-B sector
  uint32_t *q_rumor, *q_seq, *q_txlen, *q_next_seq;  // [n_loc][3][qcap], next_seq [n_loc][3]
  uint32_t* q_dec;        // [n_loc][qcap] intent queue: each item's record decoration (subject slot)
  uint32_t* q_pruned;     // [n_loc] live queue items dropped by a full queue (memberlist Prune), cumulative
  uint32_t* q_expired;    // [n_loc] queue items dropped when the rumor ring wrapped onto their generation
  uint64_t* eb_ltime;
  uint32_t* eb_cnt;
  uint64_t* eb_keys;
  uint64_t* qb_ltime;
  uint32_t* qb_cnt;
  uint32_t* qb_ids;
  rsf_rumor* rumors;
  uint32_t* rdec;  // per rumor: its record decoration (subject / kDecQuery / kDecEvent), 4 B
  uint4* rbody;    // per rumor id: the rumor without its key (ltime, subject, type, flags, msg_len), 16 B
  uint4* dlog;     // [n_loc][dcap] events delivered to the application: ltime (member event: its type), key
  uint8_t* dmeta;  // [n_loc][dcap] each entry's flags: kLogCc, kLogMember (a byte of its own: an ltime is a full u64)
  uint32_t* dcnt;  // [n_loc] deliveries since the log was cleared
  // snapshotter per member (rsf_gossip_enable_snapshot; null: off): the alive set as a bitset
  // over subjects, and {last event clock, last query clock, last clock at leave, flags}
  uint32_t* snap_bits;  // [n_loc][snap_w]
  uint64_t* snap_sn;    // [n_loc][4]; flags bit 0: leaving (recording stopped)
  // Pending re-queues (deferred TransmitLimitedQueue inserts).  A handler's "rebroadcast"
  // appends (rumor id, record decoration, msg_len | queue << 16) to the member's list in
  // insertion order; the list is applied to the queues as one batch per queue at the
  // member's next emission (emit_kernel, which holds the queues in registers anyway), or by
  // pend_flush_* before anything else reads the queues.  Inserting new items and pruning
  // the largest key is order-free between picks (the queue keeps the qcap smallest keys of
  // everything inserted), so the deferred batch is exactly the reference's one-by-one
  // insert.  p_cnt[l] packs the entries per queue: n0 | n1 << 8 | n2 << 16 (sum <= kPend).
  struct PendE { uint32_t rid, dec, lq; } * p_ent;  // [n_loc][kPend], 12-B entries: one contiguous append
  uint32_t* p_cnt;                 // [n_loc]
  // Deep queues: each queue is its register head (the q_* slots above, sorted) plus an
  // UNORDERED tail in HBM, tail[q][l * tstride[q] + i], i < tsum[l * 3 + q].x: for the query and
  // event queues 16-B items {rumor, seq, transmits | len << 16, decoration}; for the intent queue
  // 8-B packed items (tail_pack below: the rumor's ring slot and generation parity, transmits,
  // length and the seq's low bits; the decoration is the rumor's, s.rdec).  tsum = {count, a
  // lower bound of the tail's smallest
  // message length, a lower bound of its smallest key (lo, hi)}: emission picks from the head
  // only while a pick's key is below the tail's bound and every stop is decided by a length
  // the tail cannot fit; any other member takes the exact whole-queue path (emit_deep_wave_kernel).
  uint64_t* tail0;  // the intent queue's tail: packed 8-B items
  uint4 *tail1, *tail2;
  uint4* tsum;       // [n_loc][3]
  // Sealed tail prefix (a hint for the deferred path): tseal[l * 3 + q] = {m, B lo, B hi, -}:
  // every item of tail[0, m) has a key >= B.  The deferred path then refills the head from the
  // head, the pending list and only the RECENT part tail[m, count) -- the items spilled since
  // the last refill -- whenever the qcap-th smallest of those is below B (no sealed item can
  // precede it), instead of reading the whole tail; each refill seals what it leaves.  Spills
  // append past m and keep it valid; any writer that moves items inside [0, m) reseals (exact)
  // or sets m = 0.
  uint4* tseal;      // [n_loc][3]
  uint32_t* deep_ids;  // [n_loc * 3] members deferred to emit_deep_wave_kernel (two lists), or queues to prune
  uint32_t* deep_n;    // [kDeepLists] the lists' lengths (reset before each emission)
};
// deferred-member lists: 0 small, 1 full depth, 2 tiny, 3 middle, 4 re-listed to the full depth
constexpr uint32_t kDeepLists = 5;
constexpr uint32_t kDeepClassOff = 6;  // the per-list deferral counters sit at (total counter) - 6 + list
// past the lists' counts (u32 words of deep_n): two u64 counters of the full-depth class, the
// items its members held (sum, max) since creation
constexpr uint32_t kDeepFullItems = 8;
constexpr uint32_t kTailSlack = 192;  // tail row room past its capacity: one emission's spills (2 x 64) + 64
// per-queue deep-queue fields by a select on q
RSF_HD uint32_t tcap_of(const GCfg& c, uint32_t q) { return q == 0 ? c.tcap0 : q == 1 ? c.tcap1 : c.tcap2; }
// the deep queues (those with a tail): how many, and queue q's place among them
RSF_HD uint32_t deep_queues(const GCfg& c) { return (c.tcap0 ? 1u : 0u) + (c.tcap1 ? 1u : 0u) + (c.tcap2 ? 1u : 0u); }
RSF_HD uint32_t deep_rank(const GCfg& c, uint32_t q) {
  return (q > 0 && c.tcap0 ? 1u : 0u) + (q > 1 && c.tcap1 ? 1u : 0u);
}
RSF_HD uint32_t tstride_of(const GCfg& c, uint32_t q) { return q == 0 ? c.tstride0 : q == 1 ? c.tstride1 : c.tstride2; }
// the query / event queues' 16-B tails (q = 1, 2); the intent queue's is s.tail0 (tail8)
RSF_HD uint4* tail16(const GState& s, uint32_t q) { return q == 1 ? s.tail1 : s.tail2; }
RSF_HD uint64_t* tail8(const GState& s, const GCfg& c, uint64_t l) { return s.tail0 + l * c.tstride0; }
RSF_HD uint32_t rumor_generations(const GCfg& c) { return (uint32_t)((1ull << (32 - c.rbits)) - 2); }

// The intent queue's packed tail item (8 B), low bits first:
//   seq mod 2^25 | transmits (6 bits) << 25 | length (6 bits) << 31 | (rumor & rmask) << 37.
// Intent messages are at most 28 bytes long (msg_len), transmits stay below the retransmit
// limit (<= 64, checked at create), and rumor & rmask is the ring slot plus the generation's
// parity (rbits + 1 <= 27 bits, checked at create).  Unpacking rebuilds
//   * the rumor id from the parity: only the current generation and the one before hold live
//     items (the ring's wrap expires the older one first, expire_kernel), so the id's
//     generation is `gen` if the parities agree, else gen - 1;
//   * the seq from the queue's next seq: every queued item is older, and an item whose age
//     (next seq - seq) reaches 2^24 insertions is flagged (RSF_E_DEEP_INVARIANT) by the
//     QueueChecker's and the ring expiry's passes, long before the 2^25 window could alias;
//   * the decoration, which is the rumor's (s.rdec), only when the item enters the head.
constexpr uint32_t kTailSeqBits = 25;
constexpr uint32_t kTailSeqMask = (1u << kTailSeqBits) - 1;
constexpr uint32_t kTailAgeFlag = 1u << 24;
constexpr uint32_t kDecLookup = 0xFFFFFFFCu;  // a decoration still to be read from s.rdec
RSF_HD uint64_t tail_pack(const GCfg& c, uint32_t rid, uint32_t seq, uint32_t tl) {
  return (uint64_t)(seq & kTailSeqMask) | ((uint64_t)(tl & 0x3F) << 25) | ((uint64_t)((tl >> 16) & 0x3F) << 31) |
         ((uint64_t)(rid & c.rmask) << 37);
}
RSF_HD uint32_t tail_seq(uint64_t x, uint32_t nseq) { return nseq - ((nseq - (uint32_t)x) & kTailSeqMask); }
RSF_HD uint32_t tail_tl(uint64_t x) { return ((uint32_t)(x >> 25) & 0x3F) | (((uint32_t)(x >> 31) & 0x3F) << 16); }
// gen: the generation the rebuild is relative to (the newest whose items may be queued)
RSF_HD uint32_t tail_rid(const GCfg& c, uint64_t x, uint32_t gen) {
  const uint32_t sl = (uint32_t)(x >> 37);
  const uint32_t par = (sl >> c.rbits) & 1u;
  const uint32_t g = par == (gen & 1u) ? gen : (gen == 0 ? rumor_generations(c) - 1 : gen - 1);
  return (g << c.rbits) | (sl & ((1u << c.rbits) - 1));
}
// the unpacked form of the 16-B items (decoration kDecLookup)
RSF_HD uint4 tail_unpack(const GCfg& c, uint64_t x, uint32_t nseq) {
  return make_uint4(tail_rid(c, x, c.gen), tail_seq(x, nseq), tail_tl(x), kDecLookup);
}
RSF_HD bool tail_age_over(uint64_t x, uint32_t nseq) { return ((nseq - (uint32_t)x) & kTailSeqMask) >= kTailAgeFlag; }
constexpr uint32_t kPend = 128;  // pending entries per member (two per lane of a wave)
// The merge leaves a member at most kPendMerge entries, so the round's originations and
// refutations (at most 1 + max_refute <= 5 per member) append without applying the list
// serially; a member that emits nothing for many rounds can still fill it (then the
// serial application runs, slow but exact).
constexpr uint32_t kPendMerge = kPend - 8;
// items of one queue the deferred-emission path holds in LDS: the full depth plus a pending
// list (kDeepItems, 1 wave per CU), and three smaller capacities for the common cases -- with a
// sealed tail prefix the path reads only the head, the reserve, the items spilled since the last
// refill and the pending list (kDeepTiny and kDeepSmall 8 waves per CU, kDeepMid 4; no per-item decoration in LDS)
constexpr uint32_t kDeepItems = RSF_MAX_QUEUE_DEPTH + kPend;
constexpr uint32_t kDeepTiny = 640 + 64 + kPend;
constexpr uint32_t kDeepSmall = 1024 + 64 + kPend;
constexpr uint32_t kDeepMid = 2240 + 64 + kPend;
RSF_HD uint32_t pend_total(uint32_t pc) { return (pc & 0xFF) + ((pc >> 8) & 0xFF) + ((pc >> 16) & 0xFF); }

RSF_HD ViewS* vrow_of(const GState& s, const GCfg& c, uint64_t l) { return view_row(s.view, c.vrow, l); }
RSF_HD ViewS* vent(const GState& s, const GCfg& c, uint64_t l, uint32_t subj) { return view_at(vrow_of(s, c, l), subj); }

// per-member scalar state held in registers while a kernel works on it
struct MRegs {
  uint64_t clock, eclock, qclock, emin, qmin, digest;
  uint32_t err;
  uint8_t serf_state;
  int32_t subj;
};

__device__ __forceinline__ void load_regs(const GState& s, uint64_t l, MRegs& r) {
  r.clock = s.clock[l];
  r.eclock = s.eclock[l];
  r.qclock = s.qclock[l];
  r.emin = s.emin[l];
  r.qmin = s.qmin[l];
  r.digest = s.digest[l];
  r.err = s.err[l];
  r.serf_state = s.serf_state[l];
  r.subj = s.member_subj[l];
}
__device__ __forceinline__ void store_regs(const GState& s, uint64_t l, const MRegs& r) {
  s.clock[l] = r.clock;
  s.eclock[l] = r.eclock;
  s.qclock[l] = r.qclock;
  s.digest[l] = r.digest;
  s.err[l] = r.err;
  s.serf_state[l] = r.serf_state;
}

// LamportClock::witness (types/src/clock.rs:164-181)
RSF_HD void witness(uint64_t& c, uint64_t t) {
  if (t < c) return;
  c = t + 1;
}

RSF_HD uint64_t digest_mix(uint64_t d, uint64_t x) {
  d ^= x;
  d *= 0x100000001B3ull;
  d ^= d >> 29;
  return d;
}

RSF_HD uint32_t varint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}

// encoded length model (oracle orc_msg_len)
RSF_HD uint32_t msg_len(uint8_t type, uint64_t ltime, uint32_t name_len, uint32_t payload_len) {
  uint32_t base = 1 + 4 + varint_len(ltime);
  switch (type) {
    case RSF_MSG_JOIN: return base + 12;
    case RSF_MSG_LEAVE: return base + 12 + 1;
    case RSF_MSG_USER_EVENT: return base + (4 + name_len) + (4 + payload_len) + 1;
    case RSF_MSG_QUERY: return base + 4 + 28 + 4 + 1 + 8 + (4 + name_len) + (4 + payload_len);
    default: return base;
  }
}

// Serf::user_event's size checks (api.rs:255-287), all before the event clock moves:
// name + payload against max_user_event_size, then against USER_EVENT_SIZE_LIMIT, then the
// encoded length (message_encoded_len: the model's length without the type byte) against
// both.  0 or the SerfError's status.
RSF_HD int32_t user_event_size_check(uint32_t max_ue, uint64_t ltime, uint32_t name_len, uint32_t payload_len) {
  const uint64_t before = (uint64_t)name_len + payload_len;
  if (before > max_ue) return RSF_ERR_USER_EVENT_LIMIT;
  if (before > RSF_USER_EVENT_SIZE_LIMIT) return RSF_ERR_USER_EVENT_TOO_LARGE;
  const uint32_t enc = msg_len(RSF_MSG_USER_EVENT, ltime, name_len, payload_len) - 1;
  if (enc > max_ue || enc > RSF_USER_EVENT_SIZE_LIMIT) return RSF_ERR_RAW_USER_EVENT_TOO_LARGE;
  return 0;
}

// query_in's size check (base.rs:916-921): the encoded query against query_size_limit.  The
// encoding holds name and payload, so a sum past the limit is rejected before msg_len's
// 32-bit arithmetic sees it.
RSF_HD int32_t query_size_check(uint32_t limit, uint64_t ltime, uint32_t name_len, uint32_t payload_len) {
  if ((uint64_t)name_len + payload_len > limit) return RSF_ERR_QUERY_TOO_LARGE;
  const uint32_t enc = msg_len(RSF_MSG_QUERY, ltime, name_len, payload_len) - 1;
  return enc > limit ? RSF_ERR_QUERY_TOO_LARGE : 0;
}

RSF_HD uint64_t tlq_key(uint32_t tx, uint32_t len, uint32_t seq) {
  return ((uint64_t)tx << 48) | ((uint64_t)(0xFFFFu - len) << 32) | (uint64_t)(0xFFFFFFFFu - seq);
}

__device__ __forceinline__ uint32_t vstatus(uint32_t meta) { return meta & 0xFF; }
__device__ __forceinline__ uint32_t vkind(uint32_t meta) { return (meta >> 8) & 0xFF; }
__device__ __forceinline__ uint32_t vmeta(uint32_t status, uint32_t kind) { return status | (kind << 8); }

// upsert_intent (base.rs:1797-1828)
__device__ __forceinline__ bool upsert_intent(ViewS* e, uint32_t kind, uint64_t L, uint32_t now) {
  ViewE v = *e;
  if (vkind(v.meta) == RSF_KIND_UNKNOWN || L > v.ltime) {
    v.ltime = L;
    v.meta = vmeta(vstatus(v.meta), kind);
    v.t = now;
    *e = v;
    return true;
  }
  return false;
}

// upsert_intent on a register copy
__device__ __forceinline__ bool upsert_intent_v(ViewE& v, uint32_t kind, uint64_t L, uint32_t now) {
  if (vkind(v.meta) == RSF_KIND_UNKNOWN || L > v.ltime) {
    v.ltime = L;
    v.meta = vmeta(vstatus(v.meta), kind);
    v.t = now;  // wall_time = stamper() (base.rs:1813, 1822)
    return true;
  }
  return false;
}

// handle_node_join_intent (base.rs:1302-1337) on a register copy of the view entry
__device__ __forceinline__ int hv_join_intent(ViewE& v, MRegs& r, uint64_t L, uint32_t now) {
  witness(r.clock, L);
  if (vkind(v.meta) == RSF_KIND_KNOWN) {
    if (L <= v.ltime) return 0;
    v.ltime = L;
    uint32_t st = vstatus(v.meta);
    if (st == RSF_STATUS_LEAVING) st = RSF_STATUS_ALIVE;
    v.meta = vmeta(st, RSF_KIND_KNOWN);
    return RSF_F_REBROADCAST;
  }
  return upsert_intent_v(v, RSF_KIND_INTENT_JOIN, L, now) ? RSF_F_REBROADCAST : 0;
}
__device__ __forceinline__ int h_join_intent(ViewS* e, MRegs& r, uint64_t L, uint32_t now) {
  ViewE v = *e;
  int f = hv_join_intent(v, r, L, now);
  *e = v;
  return f;
}

// handle_node_leave_intent (base.rs:1409-1528) on a register copy of the view entry.
// DIGEST = false: the caller digests the member events itself from the returned flags
// (merge_kernel's chain walk, which runs the handlers lane-parallel).
template <bool DIGEST = true>
__device__ __forceinline__ int hv_leave_intent(ViewE& v, MRegs& r, uint32_t subj, uint64_t L, bool prune,
                                               uint64_t& refute, uint32_t now) {
  uint8_t state = r.serf_state;
  witness(r.clock, L);
  if (vkind(v.meta) != RSF_KIND_KNOWN) return upsert_intent_v(v, RSF_KIND_INTENT_LEAVE, L, now) ? RSF_F_REBROADCAST : 0;
  if (L <= v.ltime) return 0;
  if (r.subj == (int32_t)subj && state == kSerfAlive) {
    refute = r.clock;
    return RSF_F_REFUTE;
  }
  v.ltime = L;
  int pf = prune ? RSF_F_PRUNE : 0;
  uint32_t st = vstatus(v.meta);
  int f;
  switch (st) {
    case RSF_STATUS_NONE: f = 0; break;
    case RSF_STATUS_ALIVE: st = RSF_STATUS_LEAVING; f = RSF_F_REBROADCAST | pf; break;
    case RSF_STATUS_LEAVING:
    case RSF_STATUS_LEFT: f = RSF_F_REBROADCAST | pf; break;
    case RSF_STATUS_FAILED:
      st = RSF_STATUS_LEFT;
      if (DIGEST) r.digest = digest_mix(r.digest, kDigMember | ((uint64_t)kEvLeave << 32) | subj);
      f = RSF_F_REBROADCAST | RSF_F_MEMBER_EVENT | pf;
      break;
    default: f = 0; break;
  }
  v.meta = vmeta(st, RSF_KIND_KNOWN);
  if (f & RSF_F_PRUNE) {
    // handle_prune (base.rs:1587-1612): erase_node! removes the member's state (and it
    // leaves the left list), then a Reap MemberEvent.  The reference sleeps
    // broadcast_timeout + leave_propagate_delay first when the member is Leaving; the
    // round model erases at once.
    v = ViewE{0ull, vmeta(RSF_STATUS_NONE, RSF_KIND_UNKNOWN), 0u};
    if (DIGEST) r.digest = digest_mix(r.digest, kDigMember | ((uint64_t)kEvReap << 32) | subj);
  }
  return f;
}
__device__ __forceinline__ int h_leave_intent(ViewS* e, MRegs& r, uint32_t subj, uint64_t L, bool prune,
                                              uint64_t& refute, uint32_t now) {
  ViewE v = *e;
  int f = hv_leave_intent(v, r, subj, L, prune, refute, now);
  *e = v;
  return f;
}

// handle_node_join (base.rs:1167-1298)
__device__ __forceinline__ int h_node_join(ViewS* e, MRegs& r, uint32_t subj) {
  ViewE v = *e;
  uint32_t kind = vkind(v.meta);
  v.t = 0;  // leave_time: None (base.rs:1226, 1265)
  if (kind == RSF_KIND_KNOWN) {
    v.meta = vmeta(RSF_STATUS_ALIVE, RSF_KIND_KNOWN);
  } else {
    uint32_t st = RSF_STATUS_ALIVE;
    uint64_t t = 0;
    if (kind == RSF_KIND_INTENT_JOIN) t = v.ltime;
    if (kind == RSF_KIND_INTENT_LEAVE) {
      t = v.ltime;
      st = RSF_STATUS_LEAVING;
    }
    v.ltime = t;
    v.meta = vmeta(st, RSF_KIND_KNOWN);
  }
  *e = v;
  r.digest = digest_mix(r.digest, kDigMember | ((uint64_t)kEvJoin << 32) | subj);
  return RSF_F_MEMBER_EVENT;
}

// handle_node_update (base.rs:1532-1583): a member with state gets the Update event
__device__ __forceinline__ int h_node_update(const ViewS* e, MRegs& r, uint32_t subj) {
  if (vkind(ViewE(*e).meta) != RSF_KIND_KNOWN) return 0;
  r.digest = digest_mix(r.digest, kDigMember | ((uint64_t)kEvUpdate << 32) | subj);
  return RSF_F_MEMBER_EVENT;
}

// handle_node_leave (base.rs:1339-1407)
__device__ __forceinline__ int h_node_leave(ViewS* e, MRegs& r, uint32_t subj, uint32_t now) {
  ViewE v = *e;
  if (vkind(v.meta) != RSF_KIND_KNOWN) return 0;
  uint32_t st = vstatus(v.meta), ev;
  if (st == RSF_STATUS_LEAVING) {
    st = RSF_STATUS_LEFT;
    ev = kEvLeave;
  } else if (st == RSF_STATUS_ALIVE) {
    st = RSF_STATUS_FAILED;
    ev = kEvFailed;
  } else {
    return 0;
  }
  v.meta = vmeta(st, RSF_KIND_KNOWN);
  v.t = now;  // leave_time = now (base.rs:1355, 1364)
  *e = v;
  r.digest = digest_mix(r.digest, kDigMember | ((uint64_t)ev << 32) | subj);
  return RSF_F_MEMBER_EVENT | (int)(ev << kFEvShift);  // the event type rides above the flags (internal)
}

// the snapshotter's process_user_event / process_query_event (snapshot.rs:663-684): the
// largest ltime handed to the application (which = 0: events, 1: queries)
__device__ __forceinline__ void snap_clock(const GState& s, uint64_t l, int which, uint64_t L) {
  if (!s.snap_sn) return;
  uint64_t* sn = s.snap_sn + l * 4;
  if (!(sn[3] & 1) && L > sn[which]) sn[which] = L;
}
// process_member_event (snapshot.rs:686-711): Join adds the node, Leave / Failed remove it
__device__ __forceinline__ void snap_member(const GCfg& c, const GState& s, uint64_t l, uint32_t subj, bool join) {
  if (!s.snap_bits || (s.snap_sn[l * 4 + 3] & 1)) return;
  uint32_t* w = s.snap_bits + l * c.snap_w + (subj >> 5);
  const uint32_t b = 1u << (subj & 31);
  *w = join ? (*w | b) : (*w & ~b);
}

// one delivery (event_tx.send of a UserEvent, base.rs:831-835) into the member's log slot
constexpr uint8_t kLogCc = 1, kLogMember = 2;
__device__ __forceinline__ void dlog_put_raw(const GCfg& c, const GState& s, uint64_t l, uint32_t& err, uint64_t lt,
                                             uint64_t key, uint8_t meta) {
  const uint32_t k = s.dcnt[l];
  if (k < c.dcap) {
    s.dlog[l * c.dcap + k] = make_uint4((uint32_t)lt, (uint32_t)(lt >> 32), (uint32_t)key, (uint32_t)(key >> 32));
    s.dmeta[l * c.dcap + k] = meta;
  } else {
    err |= kErrDlog;
  }
  s.dcnt[l] = k + 1;
}
__device__ __forceinline__ void dlog_put(const GCfg& c, const GState& s, uint64_t l, MRegs& r, uint64_t L,
                                         uint64_t key, bool cc) {
  if (!c.dcap) return;
  dlog_put_raw(c, s, l, r.err, L, key, cc ? kLogCc : 0);
}
// a MemberEvent (event_tx.send of a MemberEvent: handle_node_join / leave / update, the
// Failed -> Left leave intent, handle_prune, the Reaper) into the same log, so the
// application's stream keeps member and user events in the order they were produced;
// tagged kLogMember, the time word holds the type, the key the subject
__device__ __forceinline__ void mlog_put(const GCfg& c, const GState& s, uint64_t l, uint32_t& err, uint32_t ev,
                                         uint32_t subj) {
  if (!c.dcap) return;
  dlog_put_raw(c, s, l, err, ev, subj, kLogMember);
}
// the member events of an intent handler's result: Failed -> Left (Leave), then handle_prune (Reap)
__device__ __forceinline__ void mlog_intent(const GCfg& c, const GState& s, uint64_t l, uint32_t& err, int f,
                                            uint32_t subj) {
  if (!c.dcap) return;
  if (f & RSF_F_MEMBER_EVENT) mlog_put(c, s, l, err, kEvLeave, subj);
  if (f & RSF_F_PRUNE) mlog_put(c, s, l, err, kEvReap, subj);
}

// handle_user_event (base.rs:770-837); cc = the message's coalesce flag (delivery log only)
__device__ __forceinline__ int h_user_event(const GCfg& c, const GState& s, uint64_t l, MRegs& r, uint64_t L,
                                            uint64_t key, bool cc) {
  witness(r.eclock, L);
  if (L < r.emin) return 0;
  uint64_t B = c.ebuf, cur = r.eclock;
  if (cur > B && L < cur - B) return 0;
  uint64_t slot = l * c.ebuf + (L % B);
  uint64_t* keys = s.eb_keys + slot * c.slot_k;
  uint32_t cnt = s.eb_cnt[slot];
  if (cnt) {
    for (uint32_t i = 0; i < cnt; ++i)
      if (keys[i] == key) return 0;
    if (cnt < c.slot_k) {
      keys[cnt] = key;
      s.eb_cnt[slot] = cnt + 1;
    } else {
      r.err |= kErrEvSlot;
    }
  } else {
    s.eb_ltime[slot] = L;
    keys[0] = key;
    s.eb_cnt[slot] = 1;
  }
  r.digest = digest_mix(digest_mix(r.digest, kDigUser ^ key), L);
  dlog_put(c, s, l, r, L, key, cc);
  snap_clock(s, l, 0, L);
  return RSF_F_REBROADCAST | RSF_F_DELIVER;
}

// handle_query (base.rs:981-1119): dedup + rebroadcast decision; filters pass
__device__ __forceinline__ int h_query(const GCfg& c, const GState& s, uint64_t l, MRegs& r, uint64_t L,
                                       uint32_t id, bool no_broadcast) {
  witness(r.qclock, L);
  if (L < r.qmin) return 0;
  uint64_t cur = r.qclock, B = c.qbuf;
  if (cur > B && B < cur - B) return 0;  // reference quirk (base.rs:999)
  uint64_t slot = l * c.qbuf + (L % B);
  uint32_t* ids = s.qb_ids + slot * c.slot_k;
  uint32_t cnt = s.qb_cnt[slot];
  if (cnt) {
    if (s.qb_ltime[slot] == L)
      for (uint32_t i = 0; i < cnt; ++i)
        if (ids[i] == id) return 0;
    if (cnt < c.slot_k) {
      ids[cnt] = id;
      s.qb_cnt[slot] = cnt + 1;
    } else {
      r.err |= kErrQSlot;
    }
  } else {
    s.qb_ltime[slot] = L;
    ids[0] = id;
    s.qb_cnt[slot] = 1;
  }
  r.digest = digest_mix(digest_mix(r.digest, kDigQuery ^ id), L);
  snap_clock(s, l, 1, L);
  return (no_broadcast ? 0 : RSF_F_REBROADCAST) | RSF_F_DELIVER;
}

__device__ __forceinline__ uint32_t queue_of(uint8_t type) {
  return type == RSF_MSG_USER_EVENT ? kQEvent : (type == RSF_MSG_QUERY ? kQQuery : kQIntent);
}

// TransmitLimitedQueue insert, one thread, on a key-sorted queue (live items
// first, ascending (transmits, ~len, ~seq); then free slots): shift the tail by
// one; on a full queue the largest item falls off (memberlist Prune), and a new
// item that would land past the end is itself the pruned one.
// A full queue loses one live item: counted in q_pruned[l] and flagged (kErrQueue).
// Deep queues (a tail, tcap[q] > 0): the item that falls off the full head -- its largest, or
// the new one -- is appended to the tail; past the tail's capacity the largest item of head and
// tail is pruned (tail_prune_serial).
__device__ __forceinline__ void tail_append_serial(const GCfg& c, const GState& s, uint64_t l, uint32_t q, uint32_t rid,
                                                   uint32_t dec, uint32_t seq, uint32_t tl) {
  // (plain scalars, not a uint4 local: HIP's vector type is a union, which keeps a modified
  // copy out of registers)
  const uint4 sm = s.tsum[l * 3 + q];
  const uint32_t cnt = sm.x;
  if (q == 0) tail8(s, c, l)[cnt] = tail_pack(c, rid, seq, tl);
  else (tail16(s, q) + l * tstride_of(c, q))[cnt] = make_uint4(rid, seq, tl, dec);
  const uint64_t k = tlq_key(tl & 0xFFFF, tl >> 16, seq), mk = ((uint64_t)sm.w << 32) | sm.z;
  const uint64_t nk = k < mk ? k : mk;
  s.tsum[l * 3 + q] = make_uint4(cnt + 1, min(sm.y, tl >> 16), (uint32_t)nk, (uint32_t)(nk >> 32));
}
// over the queue's depth: drop the largest key of head and tail; true if one was dropped.
// That key is in the tail: the tail only exceeds its capacity right after an append, and
// the appended item (the head's largest, or a new item past it) is at least every key left
// in the head.  The tail's bounds stay lower bounds.
__device__ __forceinline__ bool tail_prune_serial(const GCfg& c, const GState& s, uint64_t l, uint32_t q) {
  const uint4 sm = s.tsum[l * 3 + q];
  const uint32_t cnt = sm.x;
  if (cnt <= tcap_of(c, q)) return false;
  uint32_t ti = 0;
  uint64_t tk = 0;
  if (q == 0) {
    uint64_t* const t = tail8(s, c, l);
    const uint32_t nseq = s.q_next_seq[l * 3];  // (every tail item is older)
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint64_t e = t[i];
      const uint32_t tl = tail_tl(e);
      const uint64_t x = tlq_key(tl & 0xFFFF, tl >> 16, tail_seq(e, nseq));
      if (x >= tk) {
        tk = x;
        ti = i;
      }
    }
    t[ti] = t[cnt - 1];
  } else {
    uint4* const t = tail16(s, q) + l * tstride_of(c, q);
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint4 e = t[i];
      const uint64_t x = tlq_key(e.z & 0xFFFF, e.z >> 16, e.y);
      if (x >= tk) {
        tk = x;
        ti = i;
      }
    }
    t[ti] = t[cnt - 1];
  }
  s.tsum[l * 3 + q] = make_uint4(cnt - 1, sm.y, sm.z, sm.w);
  s.tseal[l * 3 + q].x = 0u;  // an item moved into the sealed prefix: no seal
  return true;
}

__device__ __forceinline__ void queue_insert_item(const GCfg& c, const GState& s, uint64_t l, uint32_t q,
                                                  uint32_t rid, uint32_t dec, uint32_t len, uint32_t seq, MRegs& r) {
  const uint64_t base = (l * 3 + q) * c.qcap;
  const uint64_t newkey = tlq_key(0, len, seq);
  uint32_t cnt = 0, pos = kEmpty;
  while (cnt < c.qcap && s.q_rumor[base + cnt] != kEmpty) {
    const uint32_t tl = s.q_txlen[base + cnt];
    if (pos == kEmpty && tlq_key(tl & 0xFFFF, tl >> 16, s.q_seq[base + cnt]) > newkey) pos = cnt;
    cnt++;
  }
  if (cnt == c.qcap && tcap_of(c, q)) {
    if (pos == kEmpty) {  // the new item is the head's largest: straight to the tail
      tail_append_serial(c, s, l, q, rid, dec, seq, len << 16);
    } else {  // the head's largest falls into the tail, the new item shifts in
      const uint64_t last = base + c.qcap - 1;
      tail_append_serial(c, s, l, q, s.q_rumor[last], q == 0 ? s.q_dec[l * c.qcap + c.qcap - 1] : 0u, s.q_seq[last],
                         s.q_txlen[last]);
      for (uint32_t i = c.qcap - 1; i > pos; --i) {
        s.q_rumor[base + i] = s.q_rumor[base + i - 1];
        s.q_seq[base + i] = s.q_seq[base + i - 1];
        s.q_txlen[base + i] = s.q_txlen[base + i - 1];
        if (q == 0) s.q_dec[l * c.qcap + i] = s.q_dec[l * c.qcap + i - 1];
      }
      if (q == 0) s.q_dec[l * c.qcap + pos] = dec;
      s.q_rumor[base + pos] = rid;
      s.q_seq[base + pos] = seq;
      s.q_txlen[base + pos] = (len << 16);
    }
    if (tail_prune_serial(c, s, l, q)) {
      s.q_pruned[l] += 1;
      r.err |= kErrQueue;
    }
    return;
  }
  if (cnt == c.qcap) {
    s.q_pruned[l] += 1;
    r.err |= kErrQueue;
  }
  if (pos == kEmpty) pos = cnt;
  if (pos >= c.qcap) return;
  for (uint32_t i = (cnt < c.qcap ? cnt : c.qcap - 1); i > pos; --i) {
    s.q_rumor[base + i] = s.q_rumor[base + i - 1];
    s.q_seq[base + i] = s.q_seq[base + i - 1];
    s.q_txlen[base + i] = s.q_txlen[base + i - 1];
    if (q == 0) s.q_dec[l * c.qcap + i] = s.q_dec[l * c.qcap + i - 1];
  }
  if (q == 0) s.q_dec[l * c.qcap + pos] = dec;
  s.q_rumor[base + pos] = rid;
  s.q_seq[base + pos] = seq;
  s.q_txlen[base + pos] = (len << 16);
}

// the member's pending re-queues applied one by one, in insertion order (one thread)
__device__ __forceinline__ void pend_flush_serial(const GCfg& c, const GState& s, uint64_t l, MRegs& r) {
  const uint32_t n = pend_total(s.p_cnt[l]);
  for (uint32_t i = 0; i < n; ++i) {
    const GState::PendE e = s.p_ent[l * kPend + i];
    const uint32_t q = e.lq >> 16;
    queue_insert_item(c, s, l, q, e.rid, e.dec, e.lq & 0xFFFF,
                      s.q_next_seq[l * 3 + q]++, r);
  }
  s.p_cnt[l] = 0;
}

// re-queue on queue q (one thread): appended to the pending list (a full list is applied first)
__device__ __forceinline__ void pend_push_serial(const GCfg& c, const GState& s, uint64_t l, uint32_t q,
                                                 uint32_t rid, uint32_t dec, uint32_t len, MRegs& r) {
  uint32_t pc = s.p_cnt[l];
  if (pend_total(pc) >= kPend) {
    pend_flush_serial(c, s, l, r);
    pc = 0;
  }
  const uint32_t i = pend_total(pc);
  s.p_ent[l * kPend + i] = GState::PendE{rid, dec, len | (q << 16)};
  s.p_cnt[l] = pc + (1u << (8 * q));
}

}  // namespace rsf
