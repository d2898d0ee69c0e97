/*
 * ruserf_amd.h — C ABI of the MI355X-native engine for ruserf's data-parallel
 * hot path (a batched gossip round over very large membership sets).
 *
 * Drop-in boundary.  Every entry point names the reference interface it
 * replaces (al8n/ruserf @ v2, file:line).  Plain pointers and sizes only; no
 * torch or HIP types in signatures (streams are passed as void*).  Errors are
 * returned as int codes, never thrown or aborted across the boundary.  A
 * context is NOT thread-safe: like the reference's RwLock write section the
 * caller serialises calls on one context (coordinate.rs:356-360, 468).
 *
 * Pointer conventions: arguments documented "host" are host memory and are
 * copied; "device" arguments are HBM pointers on the context's device.
 * Calls are asynchronous on the context stream unless they return data to
 * host memory, which synchronises that stream.
 */
#ifndef RUSERF_AMD_H
#define RUSERF_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
/* 1..3 mirror CoordinateError in variant order (core/src/coordinate.rs:29-40) */
#define RSF_OK 0
#define RSF_ERR_DIM_MISMATCH 1   /* CoordinateError::DimensionalityMismatch */
#define RSF_ERR_INVALID_COORD 2  /* CoordinateError::InvalidCoordinate */
#define RSF_ERR_INVALID_RTT 3    /* CoordinateError::InvalidRTT(rtt > 10 s) */
#define RSF_ERR_ARG (-1)         /* bad argument / precondition (reference would panic) */
#define RSF_ERR_HIP (-2)         /* HIP runtime error; see rsf_last_error() */
#define RSF_ERR_NOMEM (-3)       /* device allocation failed */
#define RSF_ERR_OVERFLOW (-4)    /* a fixed-capacity device structure overflowed */
/* wire codecs (per item) */
#define RSF_SKIPPED 4              /* empty message / ping payload: the reference returns early */
#define RSF_ERR_CODEC_SHORT (-10)  /* NotEnoughBytes / varint buffer underflow */
#define RSF_ERR_CODEC_TYPE (-11)   /* unknown MessageType tag, a kind this codec does not carry, or a bad PING_VERSION */
#define RSF_ERR_CODEC_VARINT (-12) /* varint longer than 10 bytes / overflowing u64 */
#define RSF_ERR_CODEC_LEN (-13)    /* length field the reference would panic on (< header) or dim > max */
/* origination size limits (SerfError, core/src/error.rs:292-311): an action's status in
 * rsf_gossip_action_status; the action did nothing (no clock moved, nothing delivered or queued) */
#define RSF_ERR_USER_EVENT_LIMIT (-20)     /* UserEventLimitTooLarge: name + payload > max_user_event_size
                                              (api.rs:258-262); also rsf_gossip_create with
                                              max_user_event_size > 9 KiB (base.rs:69-70) */
#define RSF_ERR_USER_EVENT_TOO_LARGE (-21) /* UserEventTooLarge: name + payload > USER_EVENT_SIZE_LIMIT
                                              9 KiB (api.rs:264-266; serf.rs:42) */
#define RSF_ERR_RAW_USER_EVENT_TOO_LARGE (-22) /* RawUserEventTooLarge: encoded length > max_user_event_size
                                                  or > 9 KiB (api.rs:281-287) */
#define RSF_ERR_QUERY_TOO_LARGE (-23)      /* QueryTooLarge: encoded query > query_size_limit (base.rs:919-921) */
#define RSF_USER_EVENT_SIZE_LIMIT 9216     /* USER_EVENT_SIZE_LIMIT (core/src/serf.rs:42) */

/* Last error message of the calling thread (static storage, never NULL). */
const char* rsf_last_error(void);
/* Library version string. */
const char* rsf_version(void);
/* Number of visible devices (0 when no GPU): lets a caller probe without HIP headers. */
int rsf_device_count(void);

/* ======================================================================== */
/* Vivaldi network coordinates                                              */
/* ======================================================================== */

/* = CoordinateOptions (core/src/coordinate.rs:62-188; defaults 200-213) */
typedef struct rsf_coord_opts {
  uint32_t dimensionality;         /* 1..16 (kernels specialised for 8) */
  uint32_t adjustment_window_size; /* 0..64; 0 disables adjustment (coordinate.rs:335) */
  uint32_t latency_filter_size;    /* 1..7 */
  uint32_t _reserved;
  double vivaldi_error_max;
  double vivaldi_ce;
  double vivaldi_cc;
  double height_min;
  double gravity_rho;
} rsf_coord_opts;

/* Fills CoordinateOptions::new() (coordinate.rs:200-213). */
void rsf_coord_opts_default(rsf_coord_opts* opts);

/* Row layout of one Coordinate in HBM and in host buffers:
 *   row[0..dim) = portion, row[dim] = error, row[dim+1] = adjustment,
 *   row[dim+2] = height, padded to rsf_coord_row_stride(dim) doubles. */
uint32_t rsf_coord_row_stride(uint32_t dimensionality);

/* A population of CoordinateClients, one per member (coordinate.rs:356-500;
 * Serf builds one per node, core/src/serf/base.rs:166-173).  Each member keeps
 * latency-filter samples for `peer_slots` peers (the reference keys them by
 * node id in a HashMap, coordinate.rs:272). */
typedef struct rsf_vivaldi rsf_vivaldi;

/* n_members rows are allocated; this context updates members [shard_lo, shard_hi)
 * (a full table is kept so peers on other shards can be read after an
 * all-gather, see rsf_vivaldi_table).  seed keys the Philox streams that
 * replace thread_rng (coordinate.rs:812-821). */
int rsf_vivaldi_create(rsf_vivaldi** out, uint64_t n_members, uint64_t shard_lo, uint64_t shard_hi,
                       uint32_t peer_slots, const rsf_coord_opts* opts, uint64_t seed, int device);
int rsf_vivaldi_destroy(rsf_vivaldi* v);
/* Use a caller-provided hipStream_t (NULL = the context's own stream). */
int rsf_vivaldi_set_stream(rsf_vivaldi* v, void* hip_stream);
int rsf_vivaldi_sync(rsf_vivaldi* v);

/* = CoordinateClient::get_coordinate (coordinate.rs:406-408), for members
 * [first, first+count); rows_out is host memory, count*row_stride doubles. */
int rsf_vivaldi_get_coordinates(rsf_vivaldi* v, uint64_t first, uint64_t count, double* rows_out);
/* = CoordinateClient::set_coordinate (coordinate.rs:412-415): returns
 * RSF_ERR_DIM_MISMATCH / RSF_ERR_INVALID_COORD exactly as check_coordinate. */
int rsf_vivaldi_set_coordinate(rsf_vivaldi* v, uint64_t member, const double* portion, uint32_t dim,
                               double error, double adjustment, double height);
/* = CoordinateClient::forget_node (coordinate.rs:455-457) */
int rsf_vivaldi_forget_node(rsf_vivaldi* v, uint64_t member, uint32_t peer_slot);
/* = CoordinateClient::stats().resets summed over the population (coordinate.rs:419-423) */
int rsf_vivaldi_resets(rsf_vivaldi* v, uint64_t* resets_out);

/* Batched CoordinateClient::update (coordinate.rs:462-499), one item per
 * (member, peer observation).  All pointers are host memory.
 *   member[i]     : the client being updated (members must be distinct in one batch)
 *   peer_slot[i]  : latency-filter key of the observed node (< peer_slots)
 *   other_rows    : n rows (row_stride doubles each) = the `other` Coordinate
 *   other_dim     : n dims (NULL = all equal to the context's dimensionality)
 *   rtt_ns[i]     : the observed rtt as Duration nanoseconds
 *   round         : keys the Philox stream of unit_vector_at's random branch
 *   status_out[i] : RSF_OK or the CoordinateError code of that item
 *   rows_out      : optional; the updated coordinate (the reference returns a clone) */
int rsf_vivaldi_update_batch(rsf_vivaldi* v, const uint32_t* member, const uint32_t* peer_slot,
                             const double* other_rows, const uint32_t* other_dim,
                             const uint64_t* rtt_ns, uint64_t n, uint32_t round,
                             int32_t* status_out, double* rows_out);

/* Batched Coordinate::distance_to = estimate_rtt (coordinate.rs:630-644).
 * From member a[i]'s coordinate to member b[i]'s; ns_out[i] = Duration nanos.
 * Host pointers. */
int rsf_vivaldi_estimate_rtt_batch(rsf_vivaldi* v, const uint32_t* a, const uint32_t* b, uint64_t n,
                                   uint64_t* ns_out);
/* Same, device pointers, asynchronous (the throughput path). */
int rsf_vivaldi_estimate_rtt_device(rsf_vivaldi* v, const uint32_t* a, const uint32_t* b, uint64_t n,
                                    uint64_t* ns_out);

/* One population round on the synthetic network of BASELINE configs 1/5:
 * every member of the shard probes neighbour slot (round mod `peer_slots`) of
 * its fixed, Philox-drawn neighbour list (memberlist's round-robin probe loop),
 * observes rtt = true distance x (1 + U[0,0.1)),
 * and runs CoordinateClient::update with the neighbour's coordinate as of the
 * END OF THE PREVIOUS ROUND (the ack carries the peer's last coordinate,
 * core/src/serf/delegate.rs:659-779).  Asynchronous; flips the table buffers. */
int rsf_vivaldi_round(rsf_vivaldi* v, uint32_t round);

/* The two halves of rsf_vivaldi_round, for callers that bring their own probes.
 *
 * rsf_vivaldi_gen_probes: the synthetic network's observations for `round`
 * (slot round mod peer_slots): peer_out[i] = neighbour of shard member lo+i,
 * rtt_ns_out[i] its observed RTT.  Device pointers, shard_n entries each.
 *
 * rsf_vivaldi_observe: one CoordinateClient::update (coordinate.rs:462-499) per
 * shard member lo+i with node = the neighbour held in latency-filter slot `slot`,
 * other = row peer[i] of the table as of the end of the previous round, rtt =
 * rtt_ns[i] (the batched form of notify_ping_complete, delegate.rs:704-779).
 * Device pointers, shard_n entries each; status_out (nullable) receives RSF_OK or
 * RSF_ERR_INVALID_RTT (rtt > 10 s) / RSF_ERR_INVALID_COORD per member, or
 * RSF_ERR_ARG for peer[i] >= n_members; on an error the member's coordinate and
 * filter are unchanged.  `round` keys the Philox stream of the degenerate
 * unit-vector draws (coordinate.rs:812-821).  Asynchronous; flips the tables. */
int rsf_vivaldi_gen_probes(rsf_vivaldi* v, uint32_t round, uint32_t* peer_out, uint64_t* rtt_ns_out);
int rsf_vivaldi_observe(rsf_vivaldi* v, uint32_t slot, const uint32_t* peer, const uint64_t* rtt_ns,
                        int32_t* status_out, uint32_t round);
/* rsf_vivaldi_observe over the shard members lo+first .. lo+first+count-1 only (first a
 * multiple of 64; the arrays are still indexed by shard member), WITHOUT flipping the tables:
 * a round pipelined by member chunks (each chunk observed as soon as its peers' rows are in
 * the current table) calls it once per chunk, then rsf_vivaldi_flip.  Chunks of one round must
 * not overlap.  Asynchronous. */
int rsf_vivaldi_observe_range(rsf_vivaldi* v, uint32_t slot, const uint32_t* peer, const uint64_t* rtt_ns,
                              int32_t* status_out, uint32_t round, uint64_t first, uint64_t count);
int rsf_vivaldi_flip(rsf_vivaldi* v);

/* memberlist's probe loop feeding the coordinates (memberlist is not
 * vendored: parity unpinned).  rsf_vivaldi_probe: member lo+i probes neighbour slot
 * (round mod peer_slots) on the synthetic network; the probe is acked when both processes
 * are up (up: device, N bytes of global liveness), with rtt as rsf_vivaldi_gen_probes;
 * a timed-out probe gets rtt UINT64_MAX (rsf_vivaldi_observe then leaves the member
 * unchanged, as no notify_ping_complete happens) and acked 0.  Device pointers, shard_n
 * each.  rsf_vivaldi_probe_acks: the acks on the wire -- for each acked probe the
 * target's ack_payload ([PING_VERSION][Coordinate] of its current row) at off_out[i]
 * (off_out: shard_n+1, an empty range for a timeout) in payload_out (>= shard_n x
 * (29 + 8 dim) bytes), ready for rsf_vivaldi_observe_acks over members lo..lo+shard_n.
 * Timed-out probes feed rsf_swim_probe_failures.  Asynchronous. */
int rsf_vivaldi_probe(rsf_vivaldi* v, uint32_t round, const uint8_t* up, uint32_t* peer_out, uint64_t* rtt_ns_out,
                      uint8_t* acked_out);
int rsf_vivaldi_probe_acks(rsf_vivaldi* v, const uint32_t* peer, const uint8_t* acked, uint64_t* off_out,
                           uint8_t* payload_out, uint64_t payload_cap);

/* = SerfDelegate::ack_payload (core/src/serf/delegate.rs:659-701) for n members:
 * out + i*out_stride receives [PING_VERSION=1][Coordinate encoding] of member[i]'s
 * current coordinate (29 + 8*dim bytes).  Device pointers, asynchronous. */
int rsf_vivaldi_ack_payloads(rsf_vivaldi* v, const uint32_t* member, uint64_t n, uint8_t* out, uint64_t out_stride);
/* = SerfDelegate::notify_ping_complete (delegate.rs:704-779) over n acks: member[i]
 * (in the shard; distinct in a batch) received payload bytes [off[i], off[i+1]) of
 * `payload` with round-trip rtt_ns[i] from the node in latency-filter slot slot[i].
 * status[i]: RSF_SKIPPED (empty payload), RSF_ERR_CODEC_TYPE (version byte),
 * RSF_ERR_CODEC_* (Coordinate::decode), else CoordinateClient::update's result.
 * Device pointers, asynchronous; updates the current table in place. */
int rsf_vivaldi_observe_acks(rsf_vivaldi* v, const uint32_t* member, const uint32_t* slot, const uint8_t* payload,
                             const uint64_t* off, const uint64_t* rtt_ns, uint64_t n, uint32_t round,
                             int32_t* status);

/* Device pointer of the current full coordinate table (n_members rows) and of
 * this shard's slice, for an all-gather between rounds on multi-GPU runs. */
int rsf_vivaldi_table(rsf_vivaldi* v, double** table_out, uint64_t* row_stride_out);

/* Targeted peer-row exchange (multi-GPU): per round each shard fetches
 * only the rows of its members' remote peers from their owners, in place of a full-table
 * all-gather.  Shards are equal contiguous ranges.  Buffers are fixed-capacity buckets,
 * one per shard (device memory, allocated once per world size):
 *   req_send / req_recv : world buckets of req_bucket_bytes (u32 count + peer ids)
 *   rep_send / rep_recv : world buckets of rep_bucket_bytes (rows, row_stride doubles)
 * A round: exchange_requests(peer) -> all-to-all req_send -> req_recv (equal splits) ->
 * exchange_serve (copies the requested rows of this shard's current table) ->
 * all-to-all rep_send -> rep_recv -> exchange_apply (writes each row into this shard's
 * current table at its peer's place) -> rsf_vivaldi_observe.  Capacity overflow or a
 * request for a row the shard does not own is reported by exchange_status (ok = 0). */
typedef struct rsf_vivaldi_xbufs {
  void *req_send, *req_recv, *rep_send, *rep_recv;
  uint64_t req_bucket_bytes, rep_bucket_bytes;
} rsf_vivaldi_xbufs;
int rsf_vivaldi_exchange_buffers(rsf_vivaldi* v, uint32_t world, rsf_vivaldi_xbufs* out);
int rsf_vivaldi_exchange_requests(rsf_vivaldi* v, uint32_t world, const uint32_t* peer);
/* the requests of shard members lo+first .. lo+first+count-1 only (peer indexed by shard member):
 * one chunk of a pipelined round, whose serve / apply follow as above */
int rsf_vivaldi_exchange_requests_range(rsf_vivaldi* v, uint32_t world, const uint32_t* peer, uint64_t first,
                                        uint64_t count);
int rsf_vivaldi_exchange_serve(rsf_vivaldi* v, uint32_t world);
int rsf_vivaldi_exchange_apply(rsf_vivaldi* v, uint32_t world);
int rsf_vivaldi_exchange_status(rsf_vivaldi* v, int* ok);

/* Ground truth of the synthetic network (for convergence reporting). */
int rsf_vivaldi_true_rtt_ns(rsf_vivaldi* v, uint32_t a, uint32_t b, uint64_t* ns_out);

/* ======================================================================== */
/* Gossip round: Lamport-clock member-state merge + dissemination           */
/* ======================================================================== */
/* Model (DESIGN.md "Round model"): N members; S tracked subjects (members
 * whose status churns).  Every member holds a view entry per subject
 * (= members.states / recent_intents, core/src/types/member.rs:13-34), three
 * Lamport clocks (types/src/clock.rs:134-182), three transmit-limited queues
 * (core/src/serf/base.rs:178-189) and the user-event / query dedup rings
 * (core/src/serf.rs:185-201). */

/* view entry kind / member status / message type encodings */
#define RSF_KIND_UNKNOWN 0      /* no state, no buffered intent */
#define RSF_KIND_INTENT_JOIN 1  /* unknown member with a buffered join intent (upsert_intent) */
#define RSF_KIND_INTENT_LEAVE 2 /* unknown member with a buffered leave intent */
#define RSF_KIND_KNOWN 3        /* members.states entry exists */
#define RSF_STATUS_NONE 0       /* MemberStatus (types/src/member.rs:16-27) */
#define RSF_STATUS_ALIVE 1
#define RSF_STATUS_LEAVING 2
#define RSF_STATUS_LEFT 3
#define RSF_STATUS_FAILED 4
#define RSF_MSG_LEAVE 0         /* MessageType tags (types/src/message.rs:17-24) */
#define RSF_MSG_JOIN 1
#define RSF_MSG_USER_EVENT 3
#define RSF_MSG_QUERY 4
/* per-message result flags */
#define RSF_F_REBROADCAST 1     /* handler returned true: notify_message re-queues (delegate.rs:297-304) */
#define RSF_F_REFUTE 2          /* leave intent about self while alive: broadcast_join scheduled (base.rs:1437-1447) */
#define RSF_F_PRUNE 4           /* prune requested (base.rs:1472-1523) */
#define RSF_F_DELIVER 8         /* event/query delivered to the application (event_tx) */
#define RSF_F_MEMBER_EVENT 16   /* a MemberEvent was emitted */
/* per-member error bits (rsf_gossip_dump_members err[]): a fixed capacity of the
 * round model was exceeded.  RSF_E_QUEUE_PRUNE is the model's bounded queue dropping
 * a live item (the largest in send order, as memberlist's Prune would); the count of
 * such drops is rsf_gossip_dump_pruned's. */
#define RSF_E_EVSLOT 1          /* a user-event dedup slot held slot_k keys already */
#define RSF_E_QSLOT 2           /* a query dedup slot held slot_k ids already */
#define RSF_E_REFUTE 4          /* more than max_refute refutations of a subject in one round */
#define RSF_E_STAGE 8           /* a (sender, peer) message held more than cap_t records */
#define RSF_E_QUEUE_PRUNE 16    /* a transmit-limited queue was full: a live item was dropped */
#define RSF_E_DELIVERY_LOG 32   /* the delivery log of a member was full (deliveries happened, unlogged) */
#define RSF_E_DEEP_INVARIANT 64 /* a deep queue broke an engine invariant (a tail past the checker's LDS
                                   capacity): the QueueChecker could not prune it (never set in a valid run) */

typedef struct rsf_gossip_cfg {
  uint64_t n_members;          /* N (global) */
  uint64_t shard_lo, shard_hi; /* members owned by this context */
  uint32_t n_subjects;         /* S */
  uint32_t queue_cap;          /* slots per transmit-limited queue, 1..256 (65..256: four slots per lane) */
  uint32_t event_buffer_size;  /* Options::event_buffer_size (default 512) */
  uint32_t query_buffer_size;  /* Options::query_buffer_size (default 512) */
  uint32_t slot_k;             /* events / query ids kept per dedup slot, 1..64 (the reference's
                                  slot list is unbounded; overflow sets RSF_E_EVSLOT / RSF_E_QSLOT) */
  uint32_t fanout;             /* gossip targets per round (memberlist gossip_nodes), 1..8 */
  uint32_t gossip_limit;       /* byte budget per gossip message (memberlist UDP budget) */
  uint32_t gossip_overhead;    /* per-message compound overhead */
  uint32_t retransmit_mult;    /* memberlist retransmit_mult (LAN: 4) */
  uint32_t max_refute;         /* refutations buffered per subject per round, 1..4 */
  uint32_t max_rumors;         /* rumor ring capacity, a power of two: every round takes a block of
                                  n_subjects * max_refute + n_acts ids; a queue item whose slot has
                                  been recycled since expires at its member's next emission */
  uint32_t max_user_event_size; /* Options::max_user_event_size (0 = the default 512, options.rs:526);
                                   > 9 KiB is RSF_ERR_USER_EVENT_LIMIT at create (base.rs:69-70) */
  uint64_t seed;               /* Philox key of peer selection */
  /* Deep queues: capacity of the intent / query / event queue (0 = queue_cap).  A depth above
   * queue_cap (which must then be <= 64) keeps the queue's first queue_cap slots as the
   * register head emission works on and the rest as an unordered HBM tail of depth - queue_cap
   * items, up to RSF_MAX_QUEUE_DEPTH.  The reference's TransmitLimitedQueue is unbounded between
   * QueueChecker ticks (max_queue_depth 4096, core/src/options.rs:512; pruned only by the checker,
   * core/src/serf/base.rs:720-760): a depth no queue reaches between ticks is that queue exactly;
   * past it the bounded-queue prune applies (RSF_E_QUEUE_PRUNE, counted). */
  uint32_t queue_depth[3];
  uint32_t query_size_limit;   /* Options::query_size_limit (0 = the default 1024, options.rs:519); at most
                                  65534 (the model keeps a message's length in 16 bits) */
} rsf_gossip_cfg;
#define RSF_MAX_QUEUE_DEPTH 8768 /* head (<= 64) + tail: max_queue_depth 4096 plus what 150 rounds between
                                    QueueChecker ticks add at the saturated bench workload (~24 a round) */

/* One rumor (a broadcast message body; SerfBroadcast, core/src/broadcast.rs:153-183). 24 bytes. */
typedef struct rsf_rumor {
  uint64_t ltime;
  uint64_t key;      /* user event: (name_id << 32) | payload_id; query: id */
  uint32_t subject;  /* intents: subject slot */
  uint8_t type;      /* RSF_MSG_* */
  uint8_t flags;     /* leave: bit0 prune; query: bit0 no_broadcast */
  uint16_t msg_len;  /* encoded length (queue byte budget); 0 = unused table entry */
} rsf_rumor;

/* Origination actions (api.rs / base.rs entry points) */
#define RSF_ACT_JOIN_SELF 1   /* Serf::join -> broadcast_join(clock.time()) (base.rs:396-412) */
#define RSF_ACT_LEAVE_SELF 2  /* Serf::leave (api.rs:473-503) */
#define RSF_ACT_FORCE_LEAVE 3 /* force_leave / remove_failed_node (base.rs:474-500) */
#define RSF_ACT_USER_EVENT 4  /* Serf::user_event (api.rs:247-315): size-checked first (RSF_ERR_USER_EVENT_*) */
#define RSF_ACT_QUERY 5       /* query_in (base.rs:869-953): size-checked first (RSF_ERR_QUERY_TOO_LARGE) */
typedef struct rsf_action {
  uint32_t member, act, subject, name_len, payload_len, flags;
  uint64_t key;
} rsf_action;

/* memberlist-detected transitions applied at every live member (NotifyJoin /
 * NotifyLeave / NotifyUpdate -> handle_node_join / handle_node_leave / handle_node_update,
 * base.rs:1167-1407, 1532-1583; an update emits the Update member event for a known member,
 * tags are the host's) */
#define RSF_ML_JOIN 1
#define RSF_ML_LEAVE 2
#define RSF_ML_UPDATE 3
typedef struct rsf_ml_event {
  uint32_t subject, kind;
  uint32_t set_alive; /* 1: the subject's process becomes live first; 0: dead afterwards; 2: unchanged */
  uint32_t _reserved;
} rsf_ml_event;

/* One received message for the direct-handler batch (notify_message dispatch). 32 bytes. */
typedef struct rsf_msg {
  uint32_t receiver; /* member id (must be in the shard) */
  uint32_t subject;  /* intents: subject slot */
  uint64_t ltime;
  uint64_t key;
  uint8_t type;      /* RSF_MSG_* */
  uint8_t flags;     /* leave: prune; query: no_broadcast; user event: cc (coalesce) */
  uint16_t _r0;
  uint32_t _r1;
} rsf_msg;

typedef struct rsf_gossip rsf_gossip;

int rsf_gossip_create(rsf_gossip** out, const rsf_gossip_cfg* cfg, int device);
int rsf_gossip_destroy(rsf_gossip* g);
int rsf_gossip_set_stream(rsf_gossip* g, void* hip_stream);
int rsf_gossip_sync(rsf_gossip* g);
/* subject slot -> member id (S entries, host); defines which member a subject is */
int rsf_gossip_set_subjects(rsf_gossip* g, const uint32_t* subject_member);
/* initial view of every subject, replicated into every member's row (S entries each, host) */
int rsf_gossip_init_views(rsf_gossip* g, const uint8_t* kind, const uint8_t* status, const uint64_t* ltime);
/* one view entry (test / snapshot-restore hook) */
int rsf_gossip_set_view(rsf_gossip* g, uint64_t member, uint32_t subject, uint8_t kind, uint8_t status,
                        uint64_t ltime);
/* process liveness of all N members (host, N bytes) */
int rsf_gossip_set_alive(rsf_gossip* g, const uint8_t* alive);
/* LamportClock values (e.g. restored from a snapshot, base.rs:195-204) */
int rsf_gossip_set_clocks(rsf_gossip* g, uint64_t member, uint64_t clock, uint64_t event_clock,
                          uint64_t query_clock);
/* EventCore/QueryCore min_time (base.rs:777, 992) */
int rsf_gossip_set_min_times(rsf_gossip* g, uint64_t member, uint64_t event_min, uint64_t query_min);
/* SerfState of a member process (0 alive, 1 leaving, 2 left, 3 shutdown) */
int rsf_gossip_set_serf_state(rsf_gossip* g, uint64_t member, uint8_t state);

/* Direct handlers (notify_message, core/src/serf/delegate.rs:157-305):
 * handle_node_join_intent / handle_node_leave_intent / handle_user_event /
 * handle_query for n messages (host).  Messages of one receiver are applied in
 * array order; receivers run in parallel.  flags_out[i] = RSF_F_*;
 * refute_out[i] (optional) = the clock captured for a refuting broadcast_join.
 * Re-queueing is left to the caller, as the reference's caller does it. */
int rsf_gossip_apply_batch(rsf_gossip* g, const rsf_msg* msgs, uint64_t n, int32_t* flags_out,
                           uint64_t* refute_out);

/* One full round (single context): memberlist transitions, pending
 * refutations, originations, emission (k peers x intent/query/event queues
 * under the byte budget, broadcast_messages delegate.rs:307-374), exchange,
 * and the canonical-order merge at every receiver.  ml/acts are host arrays;
 * actions of one round must name distinct members. */
int rsf_gossip_round(rsf_gossip* g, uint32_t round, const rsf_ml_event* ml, uint32_t n_ml,
                     const rsf_action* acts, uint32_t n_acts);
/* The result of each action of the last rsf_gossip_round / rsf_gossip_round_begin (host,
 * n <= that call's n_acts), what the reference's entry point returns: RSF_OK; RSF_SKIPPED
 * (the member is not in this shard, or its process is down); or the size error of
 * Serf::user_event (api.rs:255-287: the name + payload checks, then the encoded length,
 * all before event_clock.increment, api.rs:301) / query_in (base.rs:919-921: the encoded
 * length, before anything is queued), RSF_ERR_USER_EVENT_* / RSF_ERR_QUERY_TOO_LARGE.  A
 * rejected action changes nothing: no clock, delivery, queue item or rumor entry (its id
 * in the round's block stays unused).  The encoded length is the model's (msg_len, without
 * the type byte), which depends on the clock's varint width, so the check runs on the
 * device.  Synchronises. */
int rsf_gossip_action_status(rsf_gossip* g, int32_t* status, uint32_t n);

/* Multi-GPU split of rsf_gossip_round (one context per GPU, members sharded):
 *   begin : phases 1-3 for the shard; writes this round's rumor block, whose
 *           entries are owned by exactly one shard (others zero) -> the caller
 *           sums it across ranks (all-reduce over rsf_gossip_rumor_block)
 *   emit  : emission + stable sort by global receiver; send_counts[w] records
 *           go to shard w (shards are equal contiguous ranges); the packed
 *           records ((receiver << 32) | rumor) are at rsf_gossip_send_buffer
 *   merge : recv (device, n_recv packed records, concatenated in source-rank
 *           order) -> stable sort by receiver -> canonical merge */
int rsf_gossip_round_begin(rsf_gossip* g, uint32_t round, const rsf_ml_event* ml, uint32_t n_ml,
                           const rsf_action* acts, uint32_t n_acts);
int rsf_gossip_rumor_block(rsf_gossip* g, void** dev_ptr, uint64_t* bytes);
int rsf_gossip_round_emit(rsf_gossip* g, uint32_t world, uint64_t* send_counts);
int rsf_gossip_send_buffer(rsf_gossip* g, void** dev_ptr, uint64_t* capacity_records);
int rsf_gossip_round_merge(rsf_gossip* g, const uint64_t* recv_dev, uint64_t n_recv);
/* Same merge without the receive-side sort: recv_dev holds n_runs runs back to back
 * (run r = what source shard r sent, run_counts[r] records, runs in source-rank order),
 * each sorted stably by receiver, as rsf_gossip_round_emit produces them.  The
 * canonical order (receiver, run, position) is rebuilt by counts + scan + an ordered
 * scatter.  n_runs <= 32.  A record for a receiver outside this shard, or an unsorted
 * run, is skipped and reported by rsf_gossip_check_runs (ok = 0). */
int rsf_gossip_round_merge_runs(rsf_gossip* g, const uint64_t* recv_dev, const uint64_t* run_counts,
                                uint32_t n_runs);
int rsf_gossip_check_runs(rsf_gossip* g, int* ok);
/* The exchange without host synchronisation (the multi-GPU bench path): fixed-capacity
 * buckets, one per destination shard.  rsf_gossip_bucket_buffers allocates (once per
 * world size) and returns the send and receive buffers, `world` buckets of bucket_bytes
 * each, device memory.  round_emit_buckets emits straight into the send buckets (each
 * holds its shard's (sender, peer) groups sorted by receiver: a header with the group
 * count, the receivers, record counts, rumor ids and the records' decorations).  The caller moves bucket w of
 * every rank r to slot r of rank w's receive buffer (source-rank order), for every w other
 * than r itself -- a shard's own bucket is read from its send buffer, so its receive slot is
 * never read and need not be filled (grouped point-to-point sends/receives, or an
 * all-to-all of equal splits, which also copies the unused self slot); then
 * round_merge_buckets merges straight from the buckets: per receiver its groups of every
 * source in source-rank order = the canonical (receiver; sender, position) order.  A bucket over
 * its capacity, or a receiver outside the shard, is recorded and reported by
 * rsf_gossip_bucket_status (ok = 0 from then on: the rounds since are not valid). */
int rsf_gossip_bucket_buffers(rsf_gossip* g, uint32_t world, void** send, void** recv, uint64_t* bucket_bytes);
int rsf_gossip_round_emit_buckets(rsf_gossip* g, uint32_t world);
int rsf_gossip_round_merge_buckets(rsf_gossip* g, uint32_t world);
int rsf_gossip_bucket_status(rsf_gossip* g, int* ok);
/* diagnostic: device addresses of the context's main buffers (order in gossip.hip); returns
 * the count written */
int rsf_gossip_debug_ptrs(rsf_gossip* g, uint64_t* out, uint32_t n);
/* diagnostic (builds with RSF_GUARD_ZONES): bytes changed in the guard zones before / after
 * stage_dec and before / after big_ids; -1 without zones */
int rsf_gossip_debug_zones(rsf_gossip* g, uint64_t* out4);
/* diagnostic: every hipCUB temporary is sized per call and followed by a 256-B canary;
 * out3[k] = 1 if the canary after the radix-sort, group reduce/scan and run-merge scan
 * storage is intact (or the buffer was never used), 0 if something wrote past the end.
 * Synchronises the context's stream. */
int rsf_gossip_debug_canaries(rsf_gossip* g, int* out3);

/* ---- push/pull anti-entropy (SerfDelegate::local_state / merge_remote_state,
 * core/src/serf/delegate.rs:376-554) ---------------------------------------
 * Receiver `receiver` merges the local_state of `sender`: the three Lamport
 * clocks (witnessed minus one), status_ltimes (its KNOWN view entries, as
 * artificial join intents), left_members (KNOWN entries with status Left, as
 * leave intents one past their status time) and its user-event buffer (as
 * handle_user_event with cc = false).  Every sender's state is snapshotted
 * before any merge of the batch (memberlist sends its local state before it
 * merges the remote one), so a symmetric exchange is the pair (a<-b, b<-a) in
 * one batch.  Canonical order inside one merge: left members in subject-slot
 * order, then the other entries in slot order, then the buffer in index order
 * (the reference iterates an IndexSet and a HashMap).  Both members must be in
 * the shard; receivers of one batch must be distinct; dead receivers skip. */
typedef struct rsf_pp_pair {
  uint32_t receiver, sender;
} rsf_pp_pair;
#define RSF_PP_JOIN 1               /* merge_remote_state(is_join = true) */
#define RSF_PP_EVENT_JOIN_IGNORE 2  /* Options::event_join_ignore (min_time = event_ltime on a join) */
/* host pairs; validated; synchronises */
int rsf_gossip_push_pull(rsf_gossip* g, const rsf_pp_pair* pairs, uint64_t n, uint32_t flags);
/* device pairs, asynchronous, not validated (the throughput path) */
int rsf_gossip_push_pull_device(rsf_gossip* g, const rsf_pp_pair* pairs_dev, uint64_t n, uint32_t flags);

/* ---- Reaper (Serf's reaper tick, core/src/serf/base.rs:519-601, 1782-1784) ----
 * Times are in the engine's clock, which rsf_gossip_round / _round_begin set to
 * the round number (rsf_gossip_set_now sets it for rsf_gossip_apply_batch).
 * Handlers stamp it as a member's leave_time (Alive -> Failed, Leaving -> Left,
 * base.rs:1355, 1364; kept when Failed -> Left by a leave intent) and as a
 * buffered intent's wall time (upsert_intent, base.rs:1813, 1822).  At every
 * live member: failed members with now - leave_time > reconnect_timeout, then
 * left members past tombstone_timeout, are erased (the view entry returns to
 * unknown) with a Reap MemberEvent each (subject-slot order; the reference walks
 * its failed/left lists); intents past recent_intent_timeout are dropped.
 * Asynchronous.  (erase_node's CoordinateClient::forget_node is the caller's:
 * rsf_vivaldi_forget_node.) */
int rsf_gossip_reap(rsf_gossip* g, uint32_t now, uint32_t reconnect_timeout, uint32_t tombstone_timeout,
                    uint32_t recent_intent_timeout);
int rsf_gossip_set_now(rsf_gossip* g, uint32_t now);

/* ---- delivery log: the events a member's Serf sends to the application on its
 * event channel (event_tx) -- what a consumer, e.g. the coalesce_loop
 * (core/src/coalesce.rs:66-155), reads: the UserEvents handle_user_event delivers
 * (core/src/serf/base.rs:831-835) and the MemberEvents of handle_node_join /
 * handle_node_leave / handle_node_update, of a leave intent that moves a Failed
 * member to Left, of handle_prune and of the Reaper (base.rs:1167-1612, 519-601), in
 * the order the member produced them.  Each member logs up to per_member entries
 * since the last round_begin: its own memberlist transitions and originations, then
 * the round's merges; rsf_gossip_apply_batch, push/pull, the Reaper, the Reconnector
 * and restarts append to the current log.  Overflow sets RSF_E_DELIVERY_LOG.
 * per_member = 0 turns it off. */
enum {
  RSF_DELIVERY_USER_EVENT = 0,
  RSF_DELIVERY_MEMBER_EVENT = 1
};
/* MemberEventType (core/src/event.rs) of a RSF_DELIVERY_MEMBER_EVENT entry */
enum {
  RSF_MEMBER_EVENT_JOIN = 0,
  RSF_MEMBER_EVENT_LEAVE = 1,
  RSF_MEMBER_EVENT_FAILED = 2,
  RSF_MEMBER_EVENT_REAP = 3,
  RSF_MEMBER_EVENT_UPDATE = 4
};
typedef struct rsf_delivery {
  uint64_t ltime;    /* user event: its Lamport time; member event: the RSF_MEMBER_EVENT_* type */
  uint64_t key;      /* user event: (name_id << 32) | payload_id, as rsf_action.key; member event: the subject slot */
  uint32_t member;
  uint8_t cc;        /* UserEventMessage::cc: the coalescer's handle() (coalesce/user.rs:30-34) */
  uint8_t kind;      /* RSF_DELIVERY_USER_EVENT / RSF_DELIVERY_MEMBER_EVENT */
  uint8_t _r[2];
} rsf_delivery;
int rsf_gossip_set_delivery_log(rsf_gossip* g, uint32_t per_member);
/* The log, member by member (ascending id), each member's deliveries in order, into
 * out (host, capacity `cap` entries); *n_out = entries written.  Synchronises. */
int rsf_gossip_dump_deliveries(rsf_gossip* g, rsf_delivery* out, uint64_t cap, uint64_t* n_out);

/* ---- Snapshot log (core/src/snapshot.rs) and restart (core/src/serf/base.rs:122-204)
 * Replaces Options::snapshot_path + Snapshot::from_replay_result / open_and_replay_snapshot
 * (snapshot.rs:233-530) and Serf::new's clock replay (base.rs:128-204).  Every member gets a
 * snapshotter: its alive set follows the Join / Leave / Failed member events (process_member_event,
 * snapshot.rs:686-711), its event / query clocks the largest delivered ltimes (663-684), and a
 * member's Serf::leave stops it (handle_leave, 568-586).  Node records carry the subject index
 * as the node bytes: [tag][u32 LE 4][u32 LE subject]; clock records [tag][u64 LE].
 *   enable_snapshot : allocate and start (alive set = each member's known Alive / Leaving members)
 *   snapshot_encode : members [first, first+count) as compacted snapshot files (compact(),
 *                     786-880; after a leave also the Leave record and the shutdown clock):
 *                     offsets (device, count+1 u64) = each file's start, *total = bytes; with
 *                     out = NULL only the sizes; out (device) needs out_cap >= *total
 *   restart         : members (host, distinct, this shard) restart from their files (host bytes,
 *                     offsets[n+1]): replay, clocks 1 then witness(old), event/query min time =
 *                     old + 1, fresh member state, then handle_rejoin (1741-1770).  result[i] =
 *                     1 rejoined, 0 alone, RSF_SNAP_ERR_* (the member is left unchanged).
 *   dump_snapshot   : the snapshotters' state (bits [n_loc][ceil(S/32)], state [n_loc][4] =
 *                     {event clock, query clock, clock at leave, flags bit0 leaving}) */
#define RSF_SNAP_ERR_RECORD (-1)    /* SnapshotError::UnknownRecordType */
#define RSF_SNAP_ERR_TRUNCATED (-2) /* SnapshotError::Replay (unexpected end of a record) */
#define RSF_SNAP_ERR_NODE (-3)      /* a node record that does not decode */
int rsf_gossip_enable_snapshot(rsf_gossip* g, int rejoin_after_leave);
int rsf_gossip_snapshot_encode(rsf_gossip* g, uint64_t first, uint64_t count, uint64_t* offsets, uint8_t* out,
                               uint64_t out_cap, uint64_t* total);
int rsf_gossip_restart(rsf_gossip* g, const uint32_t* members, uint32_t n, const uint8_t* files,
                       const uint64_t* offsets, int32_t* result);
int rsf_gossip_dump_snapshot(rsf_gossip* g, uint32_t* bits, uint64_t* state);

/* Reconnector tick (core/src/serf/base.rs:632-701; replaces Reconnector::spawn's loop body).
 * At every live member: num_failed / num_alive over its view (num_alive = states - failed - left,
 * at least 1); with that probability (rng.gen::<f32>(), a Philox draw of (seed, member, tick))
 * it tries one failed member (gen_range(0..num_failed), ascending subject order).  The try
 * succeeds when that member is up, and memberlist's join then notifies handle_node_join.
 * target (device, n_loc u32, may be NULL) = the tried subject, 0xFFFFFFFF none. */
int rsf_gossip_reconnect(rsf_gossip* g, uint32_t tick, uint32_t* target);

/* ---- QueueChecker (core/src/serf/base.rs:703-760) ---------------------------
 * One checker tick over the three queues of every shard member: max =
 * max_queue_depth, or, when min_queue_depth > 0, max(2 * states.len(), min_queue_depth)
 * per member (get_queue_max, base.rs:748-759; states.len() = the members that node knows:
 * the N - S untracked ones, itself, its KNOWN subjects); a queue holding >= max items is
 * pruned to max (memberlist
 * TransmitLimitedQueue::prune drops the last items in send order).  depth_warning
 * is the log threshold.  Host outputs (optional, 3 entries each, per queue
 * intent / query / event): items queued over the shard, members at or above the
 * warning depth, items pruned.  Synchronises. */
int rsf_gossip_check_queues(rsf_gossip* g, uint32_t max_queue_depth, uint32_t min_queue_depth,
                            uint32_t depth_warning, uint64_t* num_queued, uint64_t* n_warn, uint64_t* n_pruned);
/* Staggered ticks: each node's QueueChecker runs on its own interval timer
 * (base.rs:703-735), so the nodes' ticks need not coincide.  This runs the same tick at the
 * shard members whose global id is phase mod period only; called after every round with
 * phase = (round + 1) mod period, every member ticks once per period rounds and each round
 * carries 1/period of the ticks.  Asynchronous: the counts accumulate (with the occupancy
 * histogram) until rsf_gossip_checker_stats resets them; rsf_gossip_check_queues resets
 * them at its start.  Errors: period 0 or phase >= period. */
int rsf_gossip_check_queues_phase(rsf_gossip* g, uint32_t max_queue_depth, uint32_t min_queue_depth,
                                  uint32_t depth_warning, uint32_t period, uint32_t phase);
/* In-round staggered ticks (period > 0; 0 turns them off): from the next round on, every
 * round r runs the tick of the members whose global id is r mod period, after the round's
 * emission and before its merge.  The oracle's orc_world_set_checker places its tick at the
 * same point.  Resets the counts (rsf_gossip_checker_stats). */
int rsf_gossip_set_checker(rsf_gossip* g, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                           uint32_t period);
/* The checker counts since the last reset (host, 3 entries each, may be NULL; as
 * rsf_gossip_check_queues reports them); reset != 0 zeroes them and the occupancy
 * histogram afterwards.  Synchronises. */
int rsf_gossip_checker_stats(rsf_gossip* g, uint64_t* num_queued, uint64_t* n_warn, uint64_t* n_pruned, int reset);
/* Occupancy at the checker ticks since the last reset (rsf_gossip_check_queues, or
 * rsf_gossip_checker_stats with reset), before their prunes: hist (host, [3][bins], may be NULL)
 * counts the shard's members per queue whose item count falls in [b * bin, (b + 1) * bin),
 * the last bin everything above; max3 (host, 3, may be NULL) = the most items any member's
 * queue held.  bin / bins (may be NULL) return the histogram's geometry. */
int rsf_gossip_checker_occupancy(rsf_gossip* g, uint32_t* hist, uint32_t* max3, uint32_t* bin, uint32_t* bins);
/* Per shard member (host, n_loc each, cumulative; either may be NULL): pruned = live
 * items its bounded queues dropped when full; expired = queue items dropped at
 * emission because their rumor slot was recycled (see max_rumors). */
int rsf_gossip_dump_pruned(rsf_gossip* g, uint32_t* pruned, uint32_t* expired);
/* Re-queues are deferred: a handler's rebroadcast (and an origination's enqueue) is
 * appended to the member's pending list and applied to its queues as one batch at the
 * member's next emission -- exactly the reference's one-by-one inserts, since inserting
 * into a bounded sorted queue without picks in between keeps the qcap smallest keys of
 * everything inserted.  rsf_gossip_flush applies every pending list now; the inspection
 * calls (dump_queues / dump_members / dump_pruned) and check_queues flush first, so they
 * always show the reference's state.  Asynchronous. */
int rsf_gossip_flush(rsf_gossip* g);
/* Sum of dump_pruned's counts over the shard (flush = 0: without applying the pending
 * lists first, i.e. as of every member's last emission).  Synchronises. */
int rsf_gossip_pruned_total(rsf_gossip* g, int flush, uint64_t* total);

/* Inspection (host copies; synchronise).  Arrays are over the shard's members. */
int rsf_gossip_dump_members(rsf_gossip* g, uint64_t* clock, uint64_t* event_clock, uint64_t* query_clock,
                            uint64_t* digest, uint32_t* err, uint8_t* serf_state);
/* time (optional): the leave time of a Failed/Left entry or the wall time of a buffered intent */
int rsf_gossip_dump_view(rsf_gossip* g, uint64_t* ltime, uint8_t* status, uint8_t* kind, uint32_t* time);
/* the same for local rows [row0, row0 + rows) only (rows x n_subjects entries) */
int rsf_gossip_dump_view_rows(rsf_gossip* g, uint64_t row0, uint64_t rows, uint64_t* ltime, uint8_t* status,
                              uint8_t* kind, uint32_t* time);
/* queues [n_loc][3][D] in send order (live items first, then free slots: rumor 0xFFFFFFFF),
 * D = the deepest queue's capacity (queue_cap, or max(queue_depth)); next_seq [n_loc][3] */
int rsf_gossip_dump_queues(rsf_gossip* g, uint32_t* rumor, uint32_t* seq, uint16_t* transmits, uint16_t* len,
                           uint32_t* next_seq);
/* the same with `width` slots per queue ([n_loc][3][width]: each queue's first width items in
 * send order); *max_live (optional) = the most items any queue holds (> width: truncated) */
int rsf_gossip_dump_queues_width(rsf_gossip* g, uint32_t width, uint32_t* rumor, uint32_t* seq, uint16_t* transmits,
                                 uint16_t* len, uint32_t* next_seq, uint32_t* max_live);
/* the same for local rows [row0, row0 + rows) only ([rows][3][width], no next_seq) */
int rsf_gossip_dump_queues_rows(rsf_gossip* g, uint64_t row0, uint64_t rows, uint32_t width, uint32_t* rumor,
                                uint32_t* seq, uint16_t* tx, uint16_t* len, uint32_t* max_live);
/* deep queues: members whose emission took the exact whole-queue path (the head alone could
 * not decide a pick; emit_deep_wave_kernel) since creation, and since the last call */
int rsf_gossip_deep_stats(rsf_gossip* g, uint64_t* slow_total, uint64_t* slow_since_last);
/* the same since creation per LDS capacity class of emit_deep_wave_kernel (host, 4 entries):
 * [0] the smallest class, [1] the small one, [2] the middle one, [3] the full depth (members the
 * smaller classes re-list to it count twice).  Synchronises. */
int rsf_gossip_deep_class_stats(rsf_gossip* g, uint64_t* out4);
/* the full-depth class's members since creation: the items their queues held in its LDS (sum
 * and the largest; head, tail and pending list).  Diagnostics of the deferred path (engine
 * state, no reference counterpart).  Synchronises. */
int rsf_gossip_deep_full_items(rsf_gossip* g, uint64_t* sum, uint64_t* max);
/* queue q's HBM tail per shard member (host, [n_loc] each, either may be NULL): its item count
 * and the length of its sealed prefix, as the engine holds them (the pending
 * lists are NOT applied first).  Engine state, no reference counterpart.  Synchronises. */
int rsf_gossip_dump_tails(rsf_gossip* g, uint32_t q, uint32_t* count, uint32_t* sealed);
/* items queued per shard member and queue (host, [n_loc][3]: intent, query, event; head + tail),
 * after applying the pending lists (the QueueChecker's num_queued per node).  Synchronises. */
int rsf_gossip_queue_lengths(rsf_gossip* g, uint32_t* out);
int rsf_gossip_dump_buffers(rsf_gossip* g, uint64_t* eb_ltime, uint32_t* eb_cnt, uint64_t* eb_keys,
                            uint64_t* qb_ltime, uint32_t* qb_cnt, uint32_t* qb_ids);
int rsf_gossip_dump_rumors(rsf_gossip* g, uint32_t first, uint32_t count, rsf_rumor* out);
int rsf_gossip_dump_refutes(rsf_gossip* g, uint32_t* count, uint64_t* ltimes);
/* Phase profiling with HIP events on the context stream (no host sync while
 * rounds run): ms_out[0..3] = summed device time of [memberlist + refute +
 * originate], [emit kernel], [sort (+ exchange on multi-GPU)], [segment +
 * merge kernel] over the rounds recorded since the last call. */
int rsf_gossip_set_profiling(rsf_gossip* g, int on);
int rsf_gossip_phase_times(rsf_gossip* g, double* ms_out, uint32_t* rounds_out);
/* records merged by this shard since creation */
int rsf_gossip_totals(rsf_gossip* g, uint64_t* merged_total);
/* records emitted / merged by the last round (this shard) */
int rsf_gossip_last_round_stats(rsf_gossip* g, uint64_t* records_sent, uint64_t* records_merged);

/* ======================================================================== */
/* User-event coalescer (UserEventCoalescer, core/src/coalesce/user.rs:52-97) */
/* ======================================================================== */
/* One event handed to a coalescer (handle() == true: cc events only); 24 bytes.
 * `group` names the coalescer (e.g. the member whose event stream it is), `name`
 * the event name (interned), `payload` an opaque key carried through. */
typedef struct rsf_user_event {
  uint32_t group, name;
  uint64_t ltime;
  uint64_t payload;
} rsf_user_event;
/* coalesce() of every event in array order, then flush(), for all groups at once:
 * out receives, group by ascending group, the flushed events — names in first-
 * insertion (IndexMap) order, each name's events with its final maximum ltime in
 * arrival order (a larger ltime clears the name's list, an equal one appends, an
 * older one is dropped).  Device pointers; *n_out (host) = events written;
 * synchronises the stream. */
int rsf_coalesce_user_events(const rsf_user_event* in, uint64_t n, rsf_user_event* out, uint64_t* n_out,
                             void* stream);

/* ---- MemberEventCoalescer (core/src/coalesce/member.rs:60-118) for many coalescers at
 * once.  A coalescer (`group`, e.g. the member whose event stream it reads) keeps
 * last_events[node] = the type it last flushed for that node (none at first); one
 * quantum's events are coalesced (latest_events: per node the LAST event in arrival
 * order wins) and flushed: a node's event is dropped when its type equals the node's
 * last flushed type, unless the type is Update (a tag update always passes); otherwise
 * it is sent (with the latest event's member) and becomes the node's last type.  The
 * reference groups the flushed
 * members by type in HashMap order (unspecified); here the flushed events come out
 * sorted by (group, type, node).  Types are RSF_MEMBER_EVENT_*; nodes < n_nodes,
 * groups < n_groups.  The coalesce_loop's quantum / quiescent timers are the caller's:
 * a call is one flush over the events of one quantum. */
typedef struct rsf_member_event {
  uint32_t group, node, type;
  uint32_t member;  /* opaque, carried through: the Member the event holds (e.g. an id of its
                     * tags); the flushed event carries the latest arrival's */
} rsf_member_event;
typedef struct rsf_member_coalescer rsf_member_coalescer;
int rsf_member_coalescer_create(rsf_member_coalescer** out, uint32_t n_groups, uint32_t n_nodes, int device);
int rsf_member_coalescer_destroy(rsf_member_coalescer* mc);
/* in / out: device pointers (out holds up to n events); *n_out (host) = events flushed.
 * An event outside the group / node / type ranges is an RSF_ERR_ARG (nothing is
 * flushed).  Synchronises the stream. */
int rsf_member_coalescer_flush(rsf_member_coalescer* mc, const rsf_member_event* in, uint64_t n,
                               rsf_member_event* out, uint64_t* n_out, void* stream);
/* the coalescers' last_events table, [n_groups][n_nodes] bytes (0xFF = none), to host */
int rsf_member_coalescer_dump(rsf_member_coalescer* mc, uint8_t* last_out);

/* ======================================================================== */
/* Wire codecs                                              */
/* ======================================================================== */
/* All pointers are device memory; calls are asynchronous on `stream`
 * (hipStream_t, NULL = default stream).  Formats (ruserf_amd/csrc/codec.h):
 *   Coordinate  u32 BE total length | error | adjustment | height | portion[], f64 BE
 *               (core/src/coordinate.rs:663-745)
 *   frame       [MessageType tag][message]; Join = u32 BE len | varint ltime | id,
 *               Leave = u32 BE len | prune | varint ltime | id, UserEvent = u32 BE len |
 *               cc | varint ltime | name | payload (types/src/{join,leave,user_event}.rs)
 *   id / name / payload: u32 BE byte length | bytes; varint: LEB128 (transformable 0.1,
 *               un-vendored: restated, parity unpinned) */

/* one Join / Leave / UserEvent message; strings are (offset, length) into a byte
 * buffer: the caller's blob on encode, the decoded frame buffer on decode */
typedef struct rsf_wire_msg {
  uint8_t type;       /* RSF_MSG_LEAVE / RSF_MSG_JOIN / RSF_MSG_USER_EVENT (tag byte) */
  uint8_t flag;       /* leave: prune; user event: cc */
  uint16_t _r0;
  int32_t status;     /* decode: RSF_OK / RSF_SKIPPED / RSF_ERR_CODEC_* */
  uint64_t ltime;
  uint64_t a_off;     /* join/leave: node id; user event: name */
  uint64_t b_off;     /* user event: payload */
  uint32_t a_len, b_len;
  uint32_t frame_len; /* decode: 1 + the length the reference's decode returns */
  uint32_t _r1;
} rsf_wire_msg;

/* off[0] = 0, off[i+1] = off[i] + encoded frame length of msgs[i] (n+1 entries) */
int rsf_wire_encoded_lengths(const rsf_wire_msg* msgs, uint64_t n, uint64_t* off, void* stream);
/* frames of msgs[i] at out + off[i] (off from rsf_wire_encoded_lengths); status optional */
int rsf_wire_encode(const rsf_wire_msg* msgs, uint64_t n, const uint8_t* blob, const uint64_t* off, uint8_t* out,
                    int32_t* status, void* stream);
/* notify_message's frame dispatch + decode_message (delegate.rs:157-305,
 * transform.rs:266-300) for frames [off[i], off[i+1]) of buf */
int rsf_wire_decode(const uint8_t* buf, const uint64_t* off, uint64_t n, rsf_wire_msg* out, void* stream);
/* Coordinate::encode of n rows (portion[dim], error, adjustment, height; row_stride
 * doubles apart) to out + i*out_stride, optionally behind the PING_VERSION byte */
int rsf_coord_encode(const double* rows, uint32_t dim, uint32_t row_stride, uint64_t n, uint8_t* out,
                     uint64_t out_stride, int ping_version_prefix, void* stream);
/* Coordinate::decode of [off[i], off[i+1]) into rows (row_stride >= max_dim + 3);
 * dim_out optional; status RSF_OK / RSF_SKIPPED (empty ping payload) / RSF_ERR_CODEC_* */
int rsf_coord_decode(const uint8_t* in, const uint64_t* off, uint64_t n, int ping_version_prefix, double* rows,
                     uint32_t row_stride, uint32_t max_dim, uint32_t* dim_out, int32_t* status, void* stream);

/* Device-side interning of user-event names and payloads: a user event's identity
 * `(name, payload)`, compared by value in handle_user_event (core/src/serf/base.rs:801-806)
 * and by name in the coalescer (coalesce/user.rs:60-75), becomes the exact key
 * (name_id << 32) | payload_id of rsf_action.key / rsf_msg.key without a host table.
 * Equal bytes <-> equal id (bytes are compared; FNV-1a only picks the probe start);
 * new strings take ids in order of first occurrence in the batch, so ids equal those
 * of a host interner walking the strings in order. */
typedef struct rsf_interner rsf_interner;
int rsf_interner_create(rsf_interner** out, uint32_t max_ids, uint64_t arena_bytes, int device);
int rsf_interner_destroy(rsf_interner* t);
/* ids committed so far and arena bytes used (host values; no synchronisation) */
int rsf_interner_count(const rsf_interner* t, uint32_t* n_ids, uint64_t* arena_used);
/* ids[i] = id of bytes [buf + off[i], + len[i]); len[i] == 0xFFFFFFFF: nothing to intern,
 * ids[i] = 0xFFFFFFFF.  Device pointers; synchronises `stream` once (to size the new
 * strings); RSF_ERR_OVERFLOW (nothing committed) when max_ids or the arena would overflow */
int rsf_intern(rsf_interner* t, const uint8_t* buf, const uint64_t* off, const uint32_t* len, uint64_t n,
               uint32_t* ids, void* stream);
/* decoded frames (rsf_wire_decode over buf) -> keys[i] = (name_id << 32) | payload_id for a
 * decoded user event, 0 otherwise: the wire-bytes -> identity step of notify_message
 * (delegate.rs:157-305) on the device */
int rsf_wire_event_keys(rsf_interner* names, rsf_interner* payloads, const uint8_t* buf, const rsf_wire_msg* msgs,
                        uint64_t n, uint64_t* keys, void* stream);

/* ======================================================================== */
/* memberlist SWIM layer model                        */
/* ======================================================================== */
/* memberlist's failure detector state per (member, subject): the incarnation merge of
 * alive / suspect / dead messages and the suspicion timers.  The reference does not
 * vendor memberlist (memberlist-core 0.2, a semver range with no lockfile; called from
 * core/src/serf/base.rs:208-225 and delegate.rs notify_join/leave): PARITY UNPINNED.
 * Restated from memberlist's published state machine (state aliveNode / suspectNode /
 * deadNode / refute and the suspicion timer), identically in oracle/oracle.c.
 * Time is an integer tick (the caller's clock, e.g. ms). */
#define RSF_SWIM_ALIVE 0
#define RSF_SWIM_SUSPECT 1
#define RSF_SWIM_DEAD 2
#define RSF_SWIM_LEFT 3
#define RSF_SWIM_UNKNOWN 255      /* not in nodeMap */
#define RSF_SWIM_MSG_ALIVE 0      /* alive{incarnation, node} */
#define RSF_SWIM_MSG_SUSPECT 1    /* suspect{incarnation, node, from} */
#define RSF_SWIM_MSG_DEAD 2       /* dead{incarnation, node, from}; from == node: the node left */
#define RSF_SWIM_MAX_CONFIRM 4    /* suspicion confirmations tracked per entry (k <= 4) */
/* result flags per message */
#define RSF_SWIM_F_REBROADCAST 1  /* encodeAndBroadcast of the message */
#define RSF_SWIM_F_REFUTE 2       /* about the receiver itself: refute() broadcast alive{new incarnation} */
#define RSF_SWIM_F_NOTIFY_JOIN 4  /* Events.NotifyJoin (unknown/dead/left -> alive) */
#define RSF_SWIM_F_NOTIFY_LEAVE 8 /* Events.NotifyLeave (-> dead / left) */
#define RSF_SWIM_F_SUSPECT 16     /* alive -> suspect: a suspicion timer started */
#define RSF_SWIM_F_CONFIRM 32     /* a new independent confirmation of a running suspicion */

typedef struct rsf_swim_cfg {
  uint64_t n_members;              /* N (member ids are global) */
  uint64_t shard_lo, shard_hi;     /* receivers owned by this context */
  uint32_t n_subjects;             /* S: the members whose entries are tracked */
  uint32_t suspicion_k;            /* SuspicionMult - 2 confirmations (0 .. RSF_SWIM_MAX_CONFIRM) */
  /* suspicion timeout after c confirmations, c = 0..k, in ticks: memberlist's
   * max - log(c+1)/log(k+1) * (max - min), floored, at least min (host-computed) */
  uint32_t timeout[RSF_SWIM_MAX_CONFIRM + 1];
  uint32_t _reserved;
} rsf_swim_cfg;

/* one received message for rsf_swim_apply_batch; 24 bytes */
typedef struct rsf_swim_msg {
  uint32_t receiver;    /* member id (in the shard) */
  uint32_t subject;     /* subject slot the message is about */
  uint32_t incarnation;
  uint32_t from;        /* member id of the accuser (suspect / dead) */
  uint32_t type;        /* RSF_SWIM_MSG_* */
  uint32_t _reserved;
} rsf_swim_msg;

typedef struct rsf_swim rsf_swim;
int rsf_swim_create(rsf_swim** out, const rsf_swim_cfg* cfg, int device);
int rsf_swim_destroy(rsf_swim* w);
int rsf_swim_set_stream(rsf_swim* w, void* hip_stream);
/* subject slot -> member id (S entries, host) */
int rsf_swim_set_subjects(rsf_swim* w, const uint32_t* subject_member);
/* initial entry of every subject replicated into every receiver's row (S each, host);
 * and every receiver's own incarnation (m.incarnation) = self_incarnation */
int rsf_swim_init(rsf_swim* w, const uint8_t* state, const uint32_t* incarnation, uint32_t self_incarnation);
/* per-receiver "left" flag (m.hasLeft(): a dead message about self is not refuted) */
int rsf_swim_set_left(rsf_swim* w, uint64_t member, uint8_t left);
/* aliveNode / suspectNode / deadNode for n messages (host).  A receiver's messages are
 * applied in array order at tick `now`; receivers run in parallel.  flags_out[i] =
 * RSF_SWIM_F_*; refute_inc_out[i] (optional) = the incarnation a refutation broadcast. */
int rsf_swim_apply_batch(rsf_swim* w, const rsf_swim_msg* msgs, uint64_t n, uint32_t now, int32_t* flags_out,
                         uint32_t* refute_inc_out);
/* suspicion timers due at `now` (now - state_change >= timeout[confirmations]) fire:
 * deadNode{entry incarnation, from = the receiver}.  *n_fired (host) = timers fired. */
int rsf_swim_tick(rsf_swim* w, uint32_t now, uint64_t* n_fired);
/* rows of receivers [first, first + count): per entry state, incarnation, state-change
 * tick, confirmations; and those receivers' own incarnations (host buffers) */
int rsf_swim_dump(rsf_swim* w, uint64_t first, uint64_t count, uint8_t* state, uint32_t* incarnation,
                  uint32_t* change, uint8_t* n_confirm, uint32_t* self_incarnation);
/* memberlist probeNode's failure path: receiver lo+i probed member target[i]
 * and got no ack (acked[i] == 0): suspectNode{its entry's incarnation, target, from =
 * receiver} when target is a tracked subject; a receiver whose process is down (up[] of
 * N bytes, nullable) does not probe.  Device pointers (n_loc entries; flags_out nullable:
 * RSF_SWIM_F_* per receiver), asynchronous.  Feed it rsf_vivaldi_probe's peer / acked. */
int rsf_swim_probe_failures(rsf_swim* w, const uint32_t* target, const uint8_t* acked, const uint8_t* up,
                            uint32_t now, int32_t* flags_out);

#ifdef __cplusplus
}
#endif
#endif
