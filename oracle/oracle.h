/*
 * oracle.h — CPU restatement of the ruserf gossip-round hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under ruserf_amd/ links, imports or
 * executes this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load liboracle.so, and only as the checker / the timed
 * CPU baseline.  The product path (HIP kernels behind include/ruserf_amd.h)
 * never routes through it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - Vivaldi (V1-V14), Lamport clock (M1), intent merge (M3-M6) and the
 *     event/query dedup (D1, D2) and user-event coalescer (D8) are
 *     line-for-line restatements of the Rust reference (cited per function in
 *     oracle.c) and are PINNED by the reference's own unit-test known answers
 *     (tests/golden/ fixtures, tests/test_oracle_kat.py).
 *   - The TransmitLimitedQueue selection/prune model and peer selection live
 *     in the un-vendored memberlist crate: PARITY UNPINNED (restated from the
 *     published memberlist design; documented in DESIGN.md).
 *
 * The reference is Rust and cannot be compiled here (no cargo/rustc), so there
 * is no oracle/_ref build.
 */
#ifndef RUSERF_ORACLE_H
#define RUSERF_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_DIM 16
#define ORC_MAX_WINDOW 64
#define ORC_MAX_FILTER 8

/* ---- Philox4x32-10 (counter-based RNG shared, as a spec, with the kernels) */
void orc_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* ---- CoordinateError codes (coordinate.rs:29-40, variant order) ---------- */
enum {
  ORC_OK = 0,
  ORC_ERR_DIM_MISMATCH = 1,
  ORC_ERR_INVALID_COORD = 2,
  ORC_ERR_INVALID_RTT = 3,
};

/* CoordinateOptions (coordinate.rs:62-213) */
typedef struct {
  uint32_t dimensionality;
  uint32_t adjustment_window_size;
  uint32_t latency_filter_size;
  uint32_t _pad;
  double vivaldi_error_max;
  double vivaldi_ce;
  double vivaldi_cc;
  double height_min;
  double gravity_rho;
} orc_coord_opts;

/* Coordinate (coordinate.rs:508-548) */
typedef struct {
  double portion[ORC_MAX_DIM];
  uint32_t dim;
  uint32_t _pad;
  double error;
  double adjustment;
  double height;
} orc_coord;

/* RNG stream used by unit_vector_at's degenerate branch (rand_f64,
 * coordinate.rs:812-821).  The reference uses thread_rng; the build replaces
 * it with Philox keyed by (seed, round, member, call) so the kernel and the
 * oracle draw identical values. */
typedef struct {
  uint32_t key[2];
  uint32_t member;
  uint32_t round;
  uint32_t call;   /* which unit_vector_at call inside one update */
  uint32_t draw;   /* draw counter inside the call */
} orc_rng;

void orc_coord_opts_default(orc_coord_opts* o);
void orc_coord_with_options(const orc_coord_opts* o, orc_coord* c);
int orc_coord_is_valid(const orc_coord* c);
uint64_t orc_coord_distance_ns(const orc_coord* a, const orc_coord* b);
double orc_coord_raw_distance(const orc_coord* a, const orc_coord* b);
double orc_magnitude(const double* v, uint32_t n);
double orc_rand_f64(orc_rng* r);
double orc_unit_vector_at(const double* v1, const double* v2, uint32_t n, double* out, orc_rng* r);
void orc_apply_force_in_place(orc_coord* self, double height_min, double force,
                              const orc_coord* other, orc_rng* r);
double orc_as_secs_f64(uint64_t ns);

/* One CoordinateClient (coordinate.rs:252-500).  Latency-filter samples are
 * kept per peer slot (the reference keys a HashMap by node id). */
typedef struct {
  double s[ORC_MAX_FILTER + 1];
  uint32_t len;
} orc_filter;

typedef struct {
  orc_coord coord;
  orc_coord origin;
  orc_coord_opts opts;
  uint32_t adjustment_index;
  uint32_t n_slots;
  double adjustment_samples[ORC_MAX_WINDOW];
  orc_filter* filters; /* n_slots entries */
  uint64_t resets;
} orc_client;

int orc_client_init(orc_client* c, const orc_coord_opts* o, uint32_t n_slots);
void orc_client_free(orc_client* c);
int orc_client_set_coordinate(orc_client* c, const orc_coord* coord);
void orc_client_forget_node(orc_client* c, uint32_t slot);
double orc_client_latency_filter(orc_client* c, uint32_t slot, double rtt_seconds);
int orc_client_update(orc_client* c, uint32_t slot, const orc_coord* other, uint64_t rtt_ns,
                      orc_rng* rng, orc_coord* out);

/* ---- Vivaldi population round (BASELINE configs 1 and 5) ----------------
 * State in the same flat layout the kernels use so results compare directly:
 *   rows  : [n][row_stride] doubles = portion[dim], error, adjustment, height
 *   adj   : [window][n] doubles, adj_idx [n]
 *   filt  : [n][peers][filter_size] doubles, filt_len [n][peers]
 *   nbr   : [n][peers] member ids                                        */
typedef struct {
  uint32_t n, peers, row_stride;
  orc_coord_opts opts;
  uint64_t seed;
  double* rows_cur;
  double* rows_nxt;
  double* adj;
  uint32_t* adj_idx;
  double* filt;
  uint32_t* filt_len;
  uint32_t* nbr;
  uint64_t resets;
} orc_vivaldi_pop;

uint32_t orc_row_stride(uint32_t dim);
int orc_vivaldi_pop_init(orc_vivaldi_pop* p, uint32_t n, uint32_t peers, const orc_coord_opts* o,
                         uint64_t seed);
void orc_vivaldi_pop_free(orc_vivaldi_pop* p);
/* the synthetic probe of member m in round t: neighbour slot + rtt in ns */
void orc_vivaldi_probe(uint64_t seed, uint32_t n, uint32_t peers, const uint32_t* nbr, uint32_t m,
                       uint32_t round, uint32_t* slot_out, uint64_t* rtt_out);
void orc_true_position(uint64_t seed, uint32_t m, double* x, double* y, double* h);
/* Run rounds [round0, round0+rounds) over members [m_lo, m_hi) using nthreads threads.
 * Every member probes once per round; peers are read from the previous-round table. */
int orc_vivaldi_pop_rounds(orc_vivaldi_pop* p, uint32_t round0, uint32_t rounds, int nthreads);
void orc_gen_neighbors(uint64_t seed, uint32_t n, uint32_t peers, uint32_t* nbr);
/* The rounds of members sharded into ranges of shard_n whose coordinate table is refreshed
 * by an all-gather after every refresh_every-th round (SURVEY §8(d) C5, R = 8): a member reads
 * a peer of its own shard from the previous round's table and a peer of another shard from
 * `stale`, the [n][row_stride] rows as of the last refresh (the caller initialises it to the
 * population's rows; it is updated at every refresh). */
int orc_vivaldi_pop_rounds_stale(orc_vivaldi_pop* p, uint32_t round0, uint32_t rounds, int nthreads, double* stale,
                                 uint32_t shard_n, uint32_t refresh_every);
/* SURVEY §8(d) C1's accuracy figure over the population's current coordinates: the median
 * over all pairs i < j of |est - true| / true, est = distance_to (ns, coordinate.rs:630-644),
 * true = the synthetic network's noiseless rtt |x_i - x_j| + h_i + h_j in ns */
double orc_vivaldi_pop_median_rel_error(const orc_vivaldi_pop* p);

/* ---- Lamport clock (types/src/clock.rs:142-182) ------------------------- */
static inline void orc_clock_witness(uint64_t* clock, uint64_t t) {
  if (t < *clock) return;
  *clock = t + 1;
}
static inline uint64_t orc_clock_increment(uint64_t* clock) { return ++(*clock); }

/* ---- Gossip world (member-state merge + dissemination) ------------------ */
enum { ORC_ST_NONE = 0, ORC_ST_ALIVE = 1, ORC_ST_LEAVING = 2, ORC_ST_LEFT = 3, ORC_ST_FAILED = 4 };
/* view entry kind: unknown member (no state), unknown + buffered intent, known */
enum { ORC_K_UNKNOWN = 0, ORC_K_INTENT_JOIN = 1, ORC_K_INTENT_LEAVE = 2, ORC_K_KNOWN = 3 };
/* serf state of a member process (SerfState) */
enum { ORC_SERF_ALIVE = 0, ORC_SERF_LEAVING = 1, ORC_SERF_LEFT = 2, ORC_SERF_SHUTDOWN = 3 };
/* rumor / message kinds (types/src/message.rs tags) */
enum { ORC_MSG_LEAVE = 0, ORC_MSG_JOIN = 1, ORC_MSG_USER_EVENT = 3, ORC_MSG_QUERY = 4 };
/* queue index: order in which broadcast_messages drains them (delegate.rs:307-374) */
enum { ORC_Q_INTENT = 0, ORC_Q_QUERY = 1, ORC_Q_EVENT = 2 };
/* merge result flags */
enum {
  ORC_F_REBROADCAST = 1,
  ORC_F_REFUTE = 2,       /* leave intent about self while alive: broadcast_join(ltime) scheduled */
  ORC_F_PRUNE = 4,        /* prune requested (handle_prune) */
  ORC_F_DELIVER = 8,      /* event/query delivered to the application */
  ORC_F_MEMBER_EVENT = 16 /* a MemberEvent was emitted */
};
/* world error bits */
enum { ORC_E_EVSLOT_FULL = 1, ORC_E_QSLOT_FULL = 2, ORC_E_REFUTE_FULL = 4, ORC_E_QUEUE_PRUNE = 16, ORC_E_DLOG = 32 };

typedef struct {
  uint8_t type;     /* ORC_MSG_* */
  uint8_t flags;    /* leave: bit0 prune; query: bit0 no_broadcast */
  uint16_t msg_len; /* encoded length used by the transmit-limited queue byte budget */
  uint32_t subject; /* intents: subject slot */
  uint64_t ltime;
  uint64_t key;     /* events: (name_id<<32)|payload_id ; queries: id */
} orc_rumor;

typedef struct {
  /* config */
  uint32_t n, s, qcap, ebuf, qbuf, slot_k, fanout, limit, overhead, tx_limit, max_refute;
  uint64_t seed;
  /* per member */
  uint64_t *clock, *eclock, *qclock, *emin, *qmin, *digest;
  uint8_t *alive, *serf_state;
  uint32_t* err;
  /* subjects */
  uint32_t* subj_member;     /* [s] */
  int32_t* member_subj;      /* [n] */
  uint32_t* refute_cnt;      /* [s] */
  uint64_t* refute_ltime;    /* [s][max_refute] */
  /* view [n][s] */
  uint64_t* v_ltime;
  uint8_t* v_status;
  uint8_t* v_kind;
  /* queues [n][3][qcap] */
  uint32_t* q_rumor; /* 0xFFFFFFFF = empty */
  uint32_t* q_seq;
  uint16_t* q_tx;
  uint16_t* q_len;
  uint32_t* q_next_seq; /* [n][3] */
  /* user-event dedup ring [n][ebuf]: ltime, count, keys[slot_k] */
  uint64_t* eb_ltime;
  uint32_t* eb_cnt; /* 0 = empty slot (reference Option::None) */
  uint64_t* eb_keys;
  /* query dedup ring [n][qbuf] */
  uint64_t* qb_ltime;
  uint32_t* qb_cnt;
  uint32_t* qb_ids;
  /* rumor table */
  orc_rumor* rumors;
  uint32_t n_rumors, cap_rumors;
  /* stats */
  uint64_t merges, sends, deliveries;
  /* [n][s] leave_time of a Failed/Left member or wall time of a buffered intent
   * (base.rs:1355, 1364, 1813, 1822), in the caller's time unit (rounds) */
  uint32_t* v_time;
  uint32_t now; /* the current time stamped by the handlers (orc_world_round sets it to the round) */
  uint32_t* q_pruned; /* [n] live items dropped by a full queue (cumulative) */
  /* rumor ring: cap_rumors (a power of two) slots per generation; a rumor id is
   * generation << rbits | slot, stored at index id & (2 cap - 1) (two generations
   * resident, by parity).  n_rumors is the ring cursor (next free slot). */
  uint32_t* q_expired; /* [n] queue items dropped when the ring wrapped onto their generation's half */
  uint32_t gen, rbits;
  /* delivery log (rsf_gossip_set_delivery_log): per member up to dcap UserEvents sent to
   * the application since the round began, {ltime, key, cc} */
  uint64_t* dlog;  /* [n][dcap][3] */
  uint32_t* dcnt;  /* [n] */
  uint32_t dcap;
  /* snapshotter per member (orc_world_enable_snapshot; snapshot.rs): the alive set as a
   * bitset over subjects, and {last event clock, last query clock, last clock at leave,
   * flags (bit 0: leaving -- recording stopped)} */
  uint32_t* snap_bits; /* [n][snap_w] */
  uint32_t snap_w;
  int32_t snap_rejoin; /* Options::rejoin_after_leave */
  uint64_t* snap_sn;   /* [n][4] */
  /* queue capacity per queue (intent, query, event): qd[q] <= qcap, the slot stride.  The
   * reference's TransmitLimitedQueue is unbounded between QueueChecker ticks; a capacity
   * deeper than any queue gets between ticks is exactly that (base.rs:720-760). */
  uint32_t qd[3];
  uint32_t* q_hwm; /* [n][3] slots [0, hwm) may be live, [hwm, qd) are free (scan bound) */
  /* Options::max_user_event_size / query_size_limit (the origination size checks) */
  uint32_t max_ue, query_limit;
  /* the last round's per-action results (orc_world_action_status), act_cap entries */
  int32_t* act_status;
  uint32_t act_cap, last_n_acts;
  /* in-round staggered QueueChecker (orc_world_set_checker): in round r, after the emission
   * and before the merge, the tick of the members with id mod chk_period == r mod chk_period;
   * chk_stats accumulates its counts (orc_check_queues' layout).  chk_period 0: off. */
  uint32_t chk_period, chk_max, chk_min, chk_warn;
  uint64_t chk_stats[9];
  /* [n][3] no slot below it is free (a scan-start hint for orc_queue_insert's first-free-slot
   * search; every writer that frees a slot lowers it).  The oracle's speed only. */
  uint32_t* q_hole;
} orc_world;

typedef struct {
  uint32_t n, s, qcap, ebuf, qbuf, slot_k, fanout, limit, overhead, retransmit_mult, max_refute;
  uint32_t cap_rumors;
  uint64_t seed;
  uint32_t qdepth[3]; /* per-queue capacity (intent, query, event); 0 = qcap */
  uint32_t max_user_event_size; /* Options::max_user_event_size, 0 = 512 (options.rs:526); > 9 KiB fails init */
  uint32_t query_size_limit;    /* Options::query_size_limit, 0 = 1024 (options.rs:519) */
  uint32_t _pad;
} orc_world_cfg;

int orc_world_init(orc_world* w, const orc_world_cfg* cfg);
void orc_world_free(orc_world* w);
uint32_t orc_retransmit_limit(uint32_t mult, uint64_t n);

/* handlers (one receiver) — return ORC_F_* flags */
int orc_handle_join_intent(orc_world* w, uint32_t m, uint32_t subj, uint64_t ltime);
int orc_handle_leave_intent(orc_world* w, uint32_t m, uint32_t subj, uint64_t ltime, int prune,
                            uint64_t* refute_ltime);
int orc_handle_node_join(orc_world* w, uint32_t m, uint32_t subj);
int orc_handle_node_leave(orc_world* w, uint32_t m, uint32_t subj);
int orc_handle_node_update(orc_world* w, uint32_t m, uint32_t subj);
int orc_handle_user_event(orc_world* w, uint32_t m, uint64_t ltime, uint64_t key);
/* the same with the message's cc flag, which only the delivery log records */
int orc_handle_user_event_cc(orc_world* w, uint32_t m, uint64_t ltime, uint64_t key, int cc);
/* Delivery log: per member up to per_member entries per round of its event stream in
 * production order, 3 u64 each: user events (ltime, key, cc); member events
 * (MemberEventType, subject, ORC_LOG_MEMBER); the third word holds the flags */
#define ORC_LOG_CC 1ull         /* a user event's cc flag */
#define ORC_LOG_MEMBER 0x100ull /* a member event */
#define ORC_MAX_QCAP 8832 /* slots per transmit-limited queue (the engine's head + tail depth range) */
int orc_world_set_delivery_log(orc_world* w, uint32_t per_member);
int orc_handle_query(orc_world* w, uint32_t m, uint64_t ltime, uint32_t id, int no_broadcast);
int orc_upsert_intent(orc_world* w, uint32_t m, uint32_t subj, uint8_t kind, uint64_t ltime);

/* rumor ring: generations per cycle, table index and liveness of an id, expiry of a member's queue */
uint32_t orc_rumor_generations(const orc_world* w);
uint32_t orc_rumor_index(const orc_world* w, uint32_t rid);
int orc_rumor_live(const orc_world* w, uint32_t rid);
uint32_t orc_queue_expire(orc_world* w, uint32_t m, uint32_t q);

/* transmit-limited queue model */
void orc_queue_insert(orc_world* w, uint32_t m, uint32_t q, uint32_t rumor);
uint32_t orc_queue_get_broadcasts(orc_world* w, uint32_t m, uint32_t q, uint32_t limit,
                                  uint32_t* out, uint32_t max_out, uint32_t* bytes_used);
/* members.states.len() of member m: the n - s untracked members, itself, its KNOWN subjects */
uint64_t orc_states_len(const orc_world* w, uint32_t m);
/* QueueChecker tick (core/src/serf/base.rs:703-760) over every member's queues: max =
 * max_queue_depth, or max(2 * states.len(), min_queue_depth) of that member when
 * min_queue_depth > 0; a queue with
 * >= max items is pruned to max (the last items in send order).  stats[9] (optional):
 * per queue queued items, members at/above depth_warning, items pruned. */
void orc_check_queues(orc_world* w, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                      uint64_t* stats);
/* The same tick at the members whose id is phase mod period only (each node's QueueChecker
 * runs on its own timer, base.rs:703-735: staggered ticks, one phase per round). */
void orc_check_queues_phase(orc_world* w, uint32_t max_queue_depth, uint32_t min_queue_depth,
                            uint32_t depth_warning, uint32_t period, uint32_t phase, uint64_t* stats);
void orc_world_set_checker(orc_world* w, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                           uint32_t period);

uint32_t orc_msg_len(uint8_t type, uint64_t ltime, uint32_t name_len, uint32_t payload_len);
/* origination size checks: 0 or the status (include/ruserf_amd.h RSF_ERR_USER_EVENT_* = -20..-22,
 * RSF_ERR_QUERY_TOO_LARGE = -23); ltime = the clock the message would carry */
enum { ORC_E_UE_LIMIT = -20, ORC_E_UE_TOO_LARGE = -21, ORC_E_UE_RAW = -22, ORC_E_QUERY_TOO_LARGE = -23 };
#define ORC_USER_EVENT_SIZE_LIMIT 9216u /* USER_EVENT_SIZE_LIMIT, core/src/serf.rs:42 */
int32_t orc_user_event_check(uint32_t max_ue, uint64_t ltime, uint32_t name_len, uint32_t payload_len);
int32_t orc_query_check(uint32_t limit, uint64_t ltime, uint32_t name_len, uint32_t payload_len);
/* the last orc_world_round's action results (0 ok, 4 skipped: member down, or an ORC_E_* size
 * error); n <= that round's n_acts; returns -1 otherwise */
int orc_world_action_status(const orc_world* w, int32_t* out, uint32_t n);
uint64_t orc_digest_mix(uint64_t d, uint64_t x);

/* one origination (workload action) */
enum {
  ORC_ACT_JOIN_SELF = 1,
  ORC_ACT_LEAVE_SELF = 2,
  ORC_ACT_FORCE_LEAVE = 3,
  ORC_ACT_USER_EVENT = 4,
  ORC_ACT_QUERY = 5
};
typedef struct {
  uint32_t member;
  uint32_t act;
  uint32_t subject;  /* FORCE_LEAVE target */
  uint32_t name_len; /* events/queries */
  uint32_t payload_len;
  uint32_t flags;    /* query: no_broadcast */
  uint64_t key;      /* events: content key; queries: id */
} orc_action;

/* memberlist-detected transitions (M6) applied at every live member */
enum { ORC_ML_JOIN = 1, ORC_ML_LEAVE = 2, ORC_ML_UPDATE = 3 };
typedef struct {
  uint32_t subject;
  uint32_t kind;     /* ORC_ML_* */
  uint32_t set_alive;/* after applying: 1 subject's member becomes live, 0 dead, 2 unchanged */
  uint32_t _pad;
} orc_ml_event;

/* One full gossip round (see DESIGN.md "Round model"):
 *   1. memberlist transitions, 2. pending refutations, 3. originations,
 *   4. emission (k peers x 3 queues under the byte budget), 5. merge at
 *   receivers in canonical (sender, position) order. */
int orc_world_round(orc_world* w, uint32_t round, const orc_ml_event* ml, uint32_t n_ml,
                    const orc_action* acts, uint32_t n_acts);
/* the same round with its member loops (memberlist transitions, emission, merge)
 * partitioned over nthreads pthreads: identical results (the CPU baseline's all-core rate) */
int orc_world_round_mt(orc_world* w, uint32_t round, const orc_ml_event* ml, uint32_t n_ml,
                       const orc_action* acts, uint32_t n_acts, int nthreads);
uint32_t orc_pick_peers(uint64_t seed, uint32_t n, const uint8_t* alive, uint32_t m, uint32_t round,
                        uint32_t k, uint32_t* out);

/* ---- push/pull anti-entropy (M7; core/src/serf/delegate.rs:376-554) ----- */
/* A member's local_state (delegate.rs:376-420) as the merge reads it: clocks,
 * status_ltimes (the KNOWN view entries), left_members (KNOWN entries with
 * status Left) and the user-event buffer.  Untracked members are implicitly
 * Alive with status_time 0: their artificial join intents are no-ops. */
typedef struct {
  uint64_t clock, eclock, qclock;
  const uint64_t* v_ltime; /* [s] */
  const uint8_t* v_status; /* [s] */
  const uint8_t* v_kind;   /* [s] */
  const uint64_t* eb_ltime;/* [ebuf] */
  const uint32_t* eb_cnt;  /* [ebuf] */
  const uint64_t* eb_keys; /* [ebuf * slot_k] */
} orc_pp_state;
/* merge_remote_state (delegate.rs:422-554) of `pp` at receiver r.  Canonical
 * order: left members in subject-slot order, then the other status_ltimes in
 * slot order (the reference iterates an IndexSet and a HashMap), then the event
 * buffer in index order.  A dead receiver ignores the message.  Returns 0. */
int orc_merge_remote_state(orc_world* w, uint32_t r, const orc_pp_state* pp, int is_join, int event_join_ignore);
/* A batch of push/pull merges: every sender's local_state is taken at batch
 * start (memberlist sends its local state before merging the remote one),
 * then receiver recv[i] merges sender send[i]'s state, in batch order. */
int orc_push_pull(orc_world* w, const uint32_t* recv, const uint32_t* send, uint32_t n, int is_join,
                  int event_join_ignore);

/* ---- Reaper (M8; core/src/serf/base.rs:519-601, 1782-1784) -------------- */
/* One reaper tick at every live member: failed members whose leave time is
 * more than reconnect_timeout old, then left members older than
 * tombstone_timeout, are erased (erase_node: the state is removed and a Reap
 * MemberEvent emitted, in subject-slot order; the reference walks its
 * failed/left lists), then intents older than recent_intent_timeout are
 * dropped (reap_intents).  `elapsed <= timeout` keeps an entry, as reap! does. */
int orc_reap(orc_world* w, uint32_t now, uint32_t reconnect_timeout, uint32_t tombstone_timeout,
             uint32_t recent_intent_timeout);

/* ---- wire codecs ----------------------------------------- */
/* status codes as include/ruserf_amd.h: 0 ok, 4 skipped, -10 short, -11 type, -12 varint, -13 len */
enum { ORC_SKIPPED = 4, ORC_E_SHORT = -10, ORC_E_TYPE = -11, ORC_E_VARINT = -12, ORC_E_LEN = -13 };
/* same layout as rsf_wire_msg */
typedef struct {
  uint8_t type, flag;
  uint16_t _r0;
  int32_t status;
  uint64_t ltime, a_off, b_off;
  uint32_t a_len, b_len, frame_len, _r1;
} orc_wire_msg;
uint32_t orc_varint_len(uint64_t v);
uint32_t orc_varint_encode(uint64_t v, uint8_t* dst);
/* returns bytes read (0 on error, *err set) */
uint32_t orc_varint_decode(const uint8_t* src, uint64_t n, uint64_t* v, int* err);
/* Coordinate codec (core/src/coordinate.rs:663-745); row = portion[dim], error, adjustment, height */
uint32_t orc_coord_encode(const double* row, uint32_t dim, uint8_t* dst);
int orc_coord_decode(const uint8_t* src, uint64_t n, uint32_t max_dim, double* row, uint32_t* dim);
/* serf frames [tag][Join | Leave | UserEvent] */
uint32_t orc_wire_frame_len(const orc_wire_msg* m);
uint32_t orc_wire_encode(const orc_wire_msg* m, const uint8_t* blob, uint8_t* dst);
void orc_wire_decode(const uint8_t* buf, uint64_t frame_off, uint64_t frame_len, orc_wire_msg* m);

/* ---- user-event coalescer (core/src/coalesce/user.rs:52-97) ------------- */
typedef struct {
  uint32_t name;
  uint64_t ltime;
  uint64_t payload;
} orc_uevent;
/* Coalesce a batch of cc events, then flush; out receives flushed events in
 * IndexMap insertion order.  Returns number written. */
uint32_t orc_coalesce_user_events(const orc_uevent* in, uint32_t n, orc_uevent* out);

/* ---- memberlist SWIM layer model -------------------- */
/* memberlist-core 0.2 is not vendored in the reference: PARITY UNPINNED.  A restatement
 * of memberlist's published state machine -- aliveNode, suspectNode, deadNode, refute,
 * suspicion.Confirm and the suspicion timeout -- for the entries (receiver, subject) of
 * a shard.  Message layout = rsf_swim_msg; states / flags as include/ruserf_amd.h. */
typedef struct orc_swim_msg {
  uint32_t receiver, subject, incarnation, from, type, reserved;
} orc_swim_msg;
typedef struct orc_swim {
  uint64_t lo, n_loc;
  uint32_t S, k;
  uint32_t timeout[5];
  uint8_t* state;    /* [n_loc * S], 255 = not in nodeMap */
  uint32_t* inc;     /* [n_loc * S] */
  uint32_t* change;  /* [n_loc * S] state-change tick */
  uint8_t* nconf;    /* [n_loc * S] confirmations of the running suspicion */
  uint32_t* accuser; /* [n_loc * S * 5] first accuser, then the confirmers */
  uint32_t* self_inc;/* [n_loc] m.incarnation */
  uint8_t* left;     /* [n_loc] m.hasLeft() */
  uint32_t* subject_member; /* [S] */
} orc_swim;
int orc_swim_init(orc_swim* w, uint64_t lo, uint64_t n_loc, uint32_t S, uint32_t k, const uint32_t* timeout,
                  const uint32_t* subject_member, const uint8_t* state0, const uint32_t* inc0, uint32_t self_inc0);
void orc_swim_free(orc_swim* w);
void orc_swim_set_left(orc_swim* w, uint64_t member, uint8_t left);
/* messages applied one by one in array order at tick now */
void orc_swim_apply(orc_swim* w, const orc_swim_msg* m, uint64_t n, uint32_t now, int32_t* flags, uint32_t* refute_inc);
/* suspicion timers due at now fire deadNode{inc, from = receiver}; returns how many */
uint64_t orc_swim_tick(orc_swim* w, uint32_t now);
/* as rsf_swim_dump: unknown entries read as (255, 0, 0, 0); confirmations only while suspect */
void orc_swim_dump(const orc_swim* w, uint64_t first, uint64_t count, uint8_t* state, uint32_t* inc, uint32_t* change,
                   uint8_t* nconf, uint32_t* self_inc);

/* ---- Snapshot log (core/src/snapshot.rs) --------------------------------- */
/* record tags (snapshot.rs:196-203); a node is [u32 LE len][node bytes], here the node
 * bytes are the subject index as u32 LE (the model's node identity) */
enum { ORC_SNAP_ALIVE = 0, ORC_SNAP_NOT_ALIVE = 1, ORC_SNAP_CLOCK = 2, ORC_SNAP_EVENT_CLOCK = 3,
       ORC_SNAP_QUERY_CLOCK = 4, ORC_SNAP_COORDINATE = 5, ORC_SNAP_LEAVE = 6, ORC_SNAP_COMMENT = 7 };
enum { ORC_SNAP_ERR_RECORD = -1, ORC_SNAP_ERR_TRUNCATED = -2, ORC_SNAP_ERR_NODE = -3 };
/* open_and_replay_snapshot (snapshot.rs:233-345): alive bitset over s subjects and the
 * last clock / event clock / query clock; 0 or ORC_SNAP_ERR_* */
int orc_snapshot_replay(const uint8_t* file, uint64_t len, int rejoin_after_leave, uint32_t s, uint32_t* alive_bits,
                        uint64_t clocks[3]);
/* one Snapshotter writing an append-only log in memory (Snapshot::stream and the
 * process_* handlers, snapshot.rs:588-800, compaction included) */
typedef struct {
  uint8_t* buf;
  uint64_t len, cap, offset, min_compact, compactions;
  uint32_t* alive;
  uint32_t s;
  uint64_t last_clock, last_event_clock, last_query_clock;
  int leaving, rejoin;
} orc_snapshotter;
/* replays `file` (may be empty) and continues its log: open_and_replay_snapshot + from_replay_result */
int orc_snapshotter_open(orc_snapshotter* sp, uint32_t s, const uint8_t* file, uint64_t len, uint64_t min_compact,
                         int rejoin_after_leave);
void orc_snapshotter_free(orc_snapshotter* sp);
void orc_snapshotter_user_event(orc_snapshotter* sp, uint64_t ltime);
void orc_snapshotter_query(orc_snapshotter* sp, uint64_t ltime);
/* MemberEvent (ev: 0 join, 1 leave, 2 failed, others ignored) with the clock's current time */
void orc_snapshotter_member_event(orc_snapshotter* sp, uint32_t ev, uint32_t subj, uint64_t clock_time);
void orc_snapshotter_update_clock(orc_snapshotter* sp, uint64_t clock_time);
void orc_snapshotter_leave(orc_snapshotter* sp);

/* the world's snapshotters: enable (alive set = each member's known Alive/Leaving
 * subjects), the member's snapshot file as it would be at shutdown (a compacted
 * prefix; after a leave the Leave record and the shutdown clock), and a restart of a
 * member from a file (Serf::new with snapshot_path, base.rs:122-204: replay, clocks
 * witnessed, event/query min times, fresh state, rejoin of the replayed nodes) */
int orc_world_enable_snapshot(orc_world* w, int rejoin_after_leave);
uint64_t orc_world_snapshot_encode(const orc_world* w, uint32_t m, uint8_t* out);
int orc_world_restart(orc_world* w, uint32_t m, const uint8_t* file, uint64_t len);

/* Reconnector tick (base.rs:632-701) at every live member; target[m] = the failed subject
 * it tried (0xFFFFFFFF: none).  A try succeeds when the target member is up, and then
 * memberlist's join notifies handle_node_join.  Returns the successful joins. */
uint32_t orc_world_reconnect(orc_world* w, uint32_t tick, uint32_t* target);
/* the Reconnector's throttle probability given members.states.len(), the failed and left
 * counts (base.rs:670-671) */
float orc_reconnect_prob(uint64_t states, uint64_t failed, uint64_t left);

/* MemberEventCoalescer (coalesce/member.rs:60-118), one per group.  last: the groups'
 * last_events tables [n_groups][n_nodes] (0xFF = none), updated.  coalesce() of the n events
 * in arrival order (latest_events.insert: the last event per (group, node) wins), then
 * flush(): skip a node whose type equals its last flushed type unless it is Update (4),
 * else record the type and send the member.  The flushed events go to out sorted by
 * (group, type, node) (the reference's HashMap order is unspecified); returns their count. */
typedef struct orc_mevent {
  uint32_t group, node, type, member; /* member: opaque, carried through (the Member clone) */
} orc_mevent;
uint64_t orc_member_coalesce(uint8_t* last, uint32_t n_nodes, const orc_mevent* in, uint64_t n, orc_mevent* out);

#ifdef __cplusplus
}
#endif
#endif
