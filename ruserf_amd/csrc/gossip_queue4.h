// gossip_queue4.h — transmit-limited queues of 65..256 slots (queue_cap up to 256; the
// reference's max_queue_depth is 4096, core/src/options.rs:249).  Included by gossip.hip
// after the one-slot-per-lane queue functions, whose invariants these keep exactly:
//   * a queue is SORTED in send order by the key (transmits, ~len, ~seq), live items first;
//   * get_broadcasts picks the leading run that fits the byte budget, then offers what is
//     left to later (shorter) items one by one, bumps the picks (or retires them at the
//     retransmit limit) and re-ranks;
//   * a batch of new items (transmits 0, increasing seqs) keeps the qcap smallest keys of
//     (queue U batch), the rest are counted as pruned (memberlist Prune of the tail).
// Layout in registers: lane i holds the four sorted slots 4i .. 4i + 3 (slot order is lane
// major, so prefix operations are a four-step local prefix plus one wave scan of the lanes'
// totals).  Re-orderings go through the wave's 256-entry LDS row (QLds4): every item is
// written to its new slot and read back in blocked order.
#pragma once

constexpr uint32_t kQK = 4;              // slots per lane
constexpr uint32_t kQ4Cap = kWave * kQK;  // 256

struct Q4 {
  uint32_t r[kQK], sq[kQK], tl[kQK], dec[kQK];
};
struct alignas(16) QLds4 {
  uint32_t r[kQ4Cap], sq[kQ4Cap], tl[kQ4Cap], dec[kQ4Cap];
};

// Orders the wave's LDS accesses before it against those after it.  The fences are what
// the compiler honours: wave_barrier alone does not order memory operations, and the row is
// accessed through different types (u32 fields, u64 keys), so type-based alias analysis
// would otherwise let it move a store of one kind across a load of the other.  Every
// operation below starts and ends its use of the row with one.
__device__ __forceinline__ void lds_fence_wave() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// exclusive prefix over the lanes of a per-lane count (lane 0 first); `total` = the sum
__device__ __forceinline__ uint32_t lanes_excl(uint32_t v, uint32_t& total) {
  const uint32_t inc = wave_inclusive_sum_u32(v);
  total = shfl_u32(inc, kWave - 1);
  return inc - v;
}
// register k of a uniform slot index's lane (k wave-uniform): select, then readlane
__device__ __forceinline__ uint32_t q4_pick(const uint32_t (&a)[kQK], uint32_t k) {
  return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3];
}

__device__ __forceinline__ void q4_load(const GCfg& c, const GState& s, uint64_t l, uint32_t q, uint32_t lane, Q4& Q) {
  const uint64_t base = (l * 3 + q) * c.qcap;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    const uint32_t slot = lane * kQK + k;
    Q.dec[k] = q == 1 ? kDecQuery : kDecEvent;
    if (slot < c.qcap) {
      Q.r[k] = s.q_rumor[base + slot];
      Q.sq[k] = s.q_seq[base + slot];
      Q.tl[k] = s.q_txlen[base + slot];
      if (q == 0) Q.dec[k] = s.q_dec[l * c.qcap + slot];
    } else {
      Q.r[k] = kEmpty;
      Q.sq[k] = 0;
      Q.tl[k] = 0;
    }
  }
}
__device__ __forceinline__ void q4_store(const GCfg& c, const GState& s, uint64_t l, uint32_t q, uint32_t lane,
                                         const Q4& Q) {
  const uint64_t base = (l * 3 + q) * c.qcap;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    const uint32_t slot = lane * kQK + k;
    if (slot < c.qcap) {
      s.q_rumor[base + slot] = Q.r[k];
      s.q_seq[base + slot] = Q.sq[k];
      s.q_txlen[base + slot] = Q.tl[k];
      if (q == 0) s.q_dec[l * c.qcap + slot] = Q.dec[k];
    }
  }
}
__device__ __forceinline__ bool q4_live(const GCfg& c, const Q4& Q, uint32_t lane, uint32_t k) {
  return lane * kQK + k < c.qcap && Q.r[k] != kEmpty;
}

// every item with dst[k] < qcap written to slot dst[k] of the row, then read back in
// blocked order; slots >= n_fill become free
template <bool DEC>
__device__ __forceinline__ void q4_scatter(const GCfg& c, Q4& Q, uint32_t lane, const uint32_t (&dst)[kQK],
                                           uint32_t n_fill, QLds4& row) {
  lds_fence_wave();  // earlier reads of the row (keys, a previous read-back) come first
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    if (dst[k] < c.qcap) {
      row.r[dst[k]] = Q.r[k];
      row.sq[dst[k]] = Q.sq[k];
      row.tl[dst[k]] = Q.tl[k];
      if (DEC) row.dec[dst[k]] = Q.dec[k];
    }
  }
  lds_fence_wave();
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    const uint32_t slot = lane * kQK + k;
    if (slot < n_fill && slot < c.qcap) {
      Q.r[k] = row.r[slot];
      Q.sq[k] = row.sq[slot];
      Q.tl[k] = row.tl[slot];
      if (DEC) Q.dec[k] = row.dec[slot];
    } else if (slot < c.qcap) {
      Q.r[k] = kEmpty;
      Q.sq[k] = 0;
      Q.tl[k] = 0;
    }
  }
  lds_fence_wave();  // the row is free once every lane has read it
}

// Re-rank after picks (q_rerank): the unpicked keepers np and the bumped keepers pk are
// each sorted in slot order; each keeper's new slot = its rank in its list + the number of
// the other list's keys below its own (binary search over the other list's keys in LDS).
template <bool DEC>
__device__ __forceinline__ void q4_rerank(const GCfg& c, Q4& Q, uint32_t lane, const bool (&np)[kQK],
                                          const bool (&pk)[kQK], QLds4& row) {
  uint32_t c_np = 0, c_pk = 0;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    c_np += np[k];
    c_pk += pk[k];
  }
  uint32_t n_np, n_pk;
  uint32_t r_np = lanes_excl(c_np, n_np), r_pk = lanes_excl(c_pk, n_pk);
  uint64_t* const keys_np = reinterpret_cast<uint64_t*>(row.r);   // r + sq: 256 keys
  uint64_t* const keys_pk = reinterpret_cast<uint64_t*>(row.tl);  // tl + dec: 256 keys
  lds_fence_wave();
  // both lists padded with keys above every real one (the real keys overwrite the padding:
  // LDS writes of a wave land in order), so the search needs no bounds test
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    keys_np[lane * kQK + k] = ~0ull;
    keys_pk[lane * kQK + k] = ~0ull;
  }
  uint64_t key[kQK];
  uint32_t rk[kQK];
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    key[k] = tlq_key(Q.tl[k] & 0xFFFF, Q.tl[k] >> 16, Q.sq[k]);
    rk[k] = np[k] ? r_np : r_pk;
    if (np[k]) keys_np[r_np++] = key[k];
    if (pk[k]) keys_pk[r_pk++] = key[k];
  }
  lds_fence_wave();
  uint32_t dst[kQK];
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    // lower_bound of the key in the other list, branchless (a keeper's other list holds at
    // most 255 keys: steps 128 .. 1 reach every count); non-keepers search harmlessly
    const uint64_t* other = np[k] ? keys_pk : keys_np;
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 128; step; step >>= 1) lo = other[lo + step - 1] < key[k] ? lo + step : lo;
    dst[k] = (np[k] || pk[k]) ? rk[k] + lo : kEmpty;
  }
  q4_scatter<DEC>(c, Q, lane, dst, n_np + n_pk, row);  // (it fences the searches first)
}

// one get_broadcasts call (q_get_broadcasts) on a sorted four-slot-per-lane queue
template <bool DEC>
__device__ __forceinline__ int64_t q4_get_broadcasts(const GCfg& c, Q4& Q, uint32_t lane, int64_t limit,
                                                     uint32_t* stage_val, uint32_t* stage_dec, uint64_t out_base,
                                                     uint32_t& nrec, uint32_t& err, bool& dirty, QLds4& row) {
  bool live[kQK];
  uint32_t len[kQK], incl[kQK], a = 0;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    live[k] = q4_live(c, Q, lane, k);
    len[k] = Q.tl[k] >> 16;
    a += live[k] ? c.overhead + len[k] : 0u;
    incl[k] = a;
  }
  uint32_t tot;
  const uint32_t base = lanes_excl(a, tot);
  if (!ballot(live[0])) return 0;  // a sorted queue: empty iff slot 0 is free
  bool pick[kQK];
  uint32_t lead = 0;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    incl[k] += base;
    pick[k] = limit >= 0 && live[k] && (int64_t)incl[k] <= limit;
    lead += pick[k];
  }
  uint32_t n_lead;
  (void)lanes_excl(lead, n_lead);
  // the leading run is the first n_lead slots: used = the prefix sum at its last slot
  int64_t used = 0;
  if (n_lead) {
    const uint32_t s = n_lead - 1;
    used = (int64_t)shfl_u32(q4_pick(incl, s % kQK), (int)(s / kQK));
  }
  for (;;) {
    const int64_t free_b = limit - used - (int64_t)c.overhead;
    if (free_b <= 0) break;
    uint32_t first = kQK;  // this lane's first candidate slot
#pragma unroll
    for (int k = kQK - 1; k >= 0; --k)
      if (live[k] && !pick[k] && (int64_t)len[k] <= free_b) first = (uint32_t)k;
    const uint64_t cm = ballot(first < kQK);
    if (!cm) break;
    const int wl = __ffsll((long long)cm) - 1;
    const uint32_t wk = shfl_u32(first, wl);
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k)
      if ((int)lane == wl && k == wk) pick[k] = true;
    used += (int64_t)c.overhead + shfl_u32(q4_pick(len, wk), wl);
  }
  uint32_t pl = 0;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) pl += pick[k];
  uint32_t npick;
  uint32_t rank = lanes_excl(pl, npick);
  if (!npick) return used;
  bool np[kQK], pk[kQK];
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    if (pick[k]) {
      if (nrec + rank < c.cap_t && stage_val) {
        stage_val[out_base + nrec + rank] = Q.r[k];
        if (stage_dec) stage_dec[out_base + nrec + rank] = Q.dec[k];
      }
      rank++;
    }
    const bool retire = pick[k] && (Q.tl[k] & 0xFFFF) + 1 >= c.tx_limit;
    if (retire) Q.r[k] = kEmpty;
    else if (pick[k]) Q.tl[k] = Q.tl[k] + 1;
    np[k] = live[k] && !pick[k];
    pk[k] = pick[k] && !retire;
  }
  if (nrec + npick > c.cap_t) err |= kErrStage;
  nrec += npick;
  dirty = true;
  q4_rerank<DEC>(c, Q, lane, np, pk, row);
  return used;
}

// All the fanout peers' picks from one four-slot-per-lane queue in one pass (q_pick_peers):
// while every pick comes from the lowest transmit class t0 (the leading run of the sorted
// queue) one prefix sum serves every peer, picks are bumped in place and written together,
// and the re-rank runs once; a peer whose next candidate could lie past the run sends the
// rest through the exact q4_get_broadcasts.  Lane-distributed per-peer state as in
// q_pick_peers (used_v, nrec_v, off_v).
template <bool DEC>
__device__ __forceinline__ void q4_pick_peers(const GCfg& c, Q4& Q, uint32_t lane, uint32_t np, uint32_t& used_v,
                                              uint32_t& nrec_v, uint64_t off_v, uint32_t* ov, uint32_t* od,
                                              uint32_t& err, bool& dirty, QLds4& row) {
  bool live[kQK], a[kQK], cons[kQK], gone[kQK];
  uint32_t len[kQK], incl[kQK], pk_peer[kQK], pk_pos[kQK];
  if (!ballot(q4_live(c, Q, lane, 0))) return;  // a sorted queue: empty iff slot 0 is free
  const uint32_t t0 = shfl_u32(Q.tl[0], 0) & 0xFFFF;  // slot 0 holds the smallest key
  const bool retire_all = t0 + 1 >= c.tx_limit;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    live[k] = q4_live(c, Q, lane, k);
    len[k] = Q.tl[k] >> 16;
    a[k] = live[k] && (Q.tl[k] & 0xFFFF) == t0;
    cons[k] = gone[k] = false;
    pk_peer[k] = pk_pos[k] = 0;
  }
  // inclusive prefix sums of the costs over the slots of `m` (slot order = lane major)
  auto scan = [&](const bool (&m)[kQK]) {
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) {
      acc += m[k] ? c.overhead + len[k] : 0u;
      incl[k] = acc;
    }
    uint32_t tot;
    const uint32_t b = lanes_excl(acc, tot);
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) incl[k] += b;
  };
  scan(a);
  uint32_t base = 0;
  bool prefix = true;
  uint32_t j = 0;
  bool exact = false;
  for (; j < np; ++j) {
    const uint32_t limit = c.limit - shfl_u32(used_v, j);  // (a peer's bytes used never exceed the limit)
    bool rem[kQK], pick[kQK];
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) rem[k] = a[k] && !cons[k];
    if (!prefix) {
      scan(rem);
      base = 0;
      prefix = true;
    }
    uint32_t mx = 0;  // the prefix sum at the last slot of the leading run that fits
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) {
      pick[k] = rem[k] && incl[k] - base <= limit;
      mx = pick[k] ? incl[k] : mx;
    }
    const uint32_t top = ballot(mx != 0) ? (uint32_t)wave_max_u64(mx) : base;
    uint32_t used = top - base;
    bool skipped = false;
    for (;;) {
      const int32_t free_b = (int32_t)(limit - used - c.overhead);
      if (free_b <= 0) break;
      uint32_t first_fit = kQK, first_cand = kQK;  // this lane's first fitting / candidate slot
#pragma unroll
      for (int k = kQK - 1; k >= 0; --k) {
        const bool f = live[k] && !gone[k] && !pick[k] && len[k] <= (uint32_t)free_b;
        first_fit = f ? (uint32_t)k : first_fit;
        first_cand = (f && rem[k]) ? (uint32_t)k : first_cand;
      }
      if (!ballot(first_fit < kQK)) break;
      const uint64_t cm = ballot(first_cand < kQK);
      if (!cm) {  // the next candidate lies past the class-t0 run (or is a bumped pick)
        exact = true;
        break;
      }
      const int wl = __ffsll((long long)cm) - 1;
      const uint32_t wk = shfl_u32(first_cand, wl);
#pragma unroll
      for (uint32_t k = 0; k < kQK; ++k) pick[k] = pick[k] || ((int)lane == wl && k == wk);
      used += c.overhead + shfl_u32(q4_pick(len, wk), wl);
      skipped = true;
    }
    if (exact) break;
    uint32_t pl = 0;
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) pl += pick[k];
    uint32_t npick;
    uint32_t rank = lanes_excl(pl, npick);
    if (npick) {
      const uint32_t nrec = shfl_u32(nrec_v, j);
#pragma unroll
      for (uint32_t k = 0; k < kQK; ++k) {
        pk_peer[k] = pick[k] ? j : pk_peer[k];
        pk_pos[k] = pick[k] ? nrec + rank : pk_pos[k];  // picks in slot (= send) order
        rank += pick[k] ? 1u : 0u;
        cons[k] = cons[k] || pick[k];
        gone[k] = gone[k] || (pick[k] && retire_all);
      }
      if (nrec + npick > c.cap_t) err |= kErrStage;
      nrec_v = lane == j ? nrec + npick : nrec_v;
      dirty = true;
      if (skipped) prefix = false;
      else base = top;
    }
    used_v += lane == j ? used : 0u;
  }
  bool any = false;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) any = any || cons[k];
  if (ballot(any)) {
    // the deferred picks: records to their groups, then transmits + 1 or retired, one re-rank
    bool npk[kQK], pkk[kQK];
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) {
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)off_v, (int)pk_peer[k]);
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(off_v >> 32), (int)pk_peer[k]);
      const uint64_t off = ((uint64_t)hi << 32) | lo;
      if (cons[k] && pk_pos[k] < c.cap_t && off != ~0ull) {
        ov[off + pk_pos[k]] = Q.r[k];
        if (od) od[off + pk_pos[k]] = Q.dec[k];
      }
      npk[k] = live[k] && !cons[k];
      pkk[k] = cons[k] && !gone[k];
      Q.r[k] = (cons[k] && retire_all) ? kEmpty : Q.r[k];
      Q.tl[k] = (cons[k] && !retire_all) ? Q.tl[k] + 1 : Q.tl[k];
    }
    q4_rerank<DEC>(c, Q, lane, npk, pkk, row);
  }
  for (; j < np; ++j) {  // the remaining peers exactly, one re-rank after each
    const int64_t limit = (int64_t)c.limit - (int64_t)shfl_u32(used_v, j);
    uint32_t nrec = shfl_u32(nrec_v, j);
    const uint64_t off = shfl_u64(off_v, j);
    const bool out = off != ~0ull;
    const int64_t used = q4_get_broadcasts<DEC>(c, Q, lane, limit, out ? ov : nullptr, out ? od : nullptr,
                                                out ? off : 0ull, nrec, err, dirty, row);
    used_v += lane == j ? (uint32_t)used : 0u;
    nrec_v = lane == j ? nrec : nrec_v;
  }
}

// Batched insert of new items (q_insert_batch_lds): lane i offers at most one new item
// (ins, rid, dec, len; seqs seq0, seq0 + 1, ... in lane order over `newmask`).  Returns the
// live items that did not fit.
template <bool DEC>
__device__ __forceinline__ uint32_t q4_insert_batch(const GCfg& c, Q4& Q, uint32_t lane, bool ins, uint32_t rid,
                                                    uint32_t dec, uint32_t len, uint32_t seq0, uint64_t newmask,
                                                    QLds4& row) {
  bool live[kQK], etx0[kQK];
  uint32_t elen[kQK], pos_e[kQK], cl = 0;
  const uint32_t n_new = (uint32_t)__popcll(newmask);
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    live[k] = q4_live(c, Q, lane, k);
    cl += live[k];
    etx0[k] = live[k] && (Q.tl[k] & 0xFFFF) == 0;
    elen[k] = Q.tl[k] >> 16;
    pos_e[k] = lane * kQK + k + ((live[k] && !etx0[k]) ? n_new : 0u);
  }
  uint32_t n_live;
  (void)lanes_excl(cl, n_live);
  const uint32_t myseq = seq0 + mbcnt(newmask);
  uint32_t pos_n = 0;
  uint64_t rem = newmask;
  while (rem) {
    const uint32_t L = shfl_u32(len, __ffsll((long long)rem) - 1);
    const uint64_t same = ballot(ins && len == L);
    rem &= ~same;
    const uint32_t gt_new = (uint32_t)__popcll(ballot(ins && len > L));
    uint32_t go = 0;
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k) go += (etx0[k] && elen[k] > L) ? 1u : 0u;
    uint32_t gt_old;
    (void)lanes_excl(go, gt_old);
    if (ins && len == L) pos_n = gt_old + gt_new + mbcnt_above(same);
#pragma unroll
    for (uint32_t k = 0; k < kQK; ++k)
      if (etx0[k] && elen[k] <= L) pos_e[k] += (uint32_t)__popcll(same);
  }
  lds_fence_wave();
  if (ins && pos_n < c.qcap) {
    row.r[pos_n] = rid;
    row.sq[pos_n] = myseq;
    row.tl[pos_n] = len << 16;
    if (DEC) row.dec[pos_n] = dec;
  }
  uint32_t dst[kQK];
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) dst[k] = live[k] ? pos_e[k] : kEmpty;
  const uint32_t total = n_live + n_new;
  q4_scatter<DEC>(c, Q, lane, dst, total, row);
  return total > c.qcap ? total - c.qcap : 0u;
}

template <bool DEC>
__device__ __forceinline__ uint32_t q4_pend_apply(const GCfg& c, Q4& Q, uint32_t lane, uint32_t q, uint32_t n,
                                                  const PendRegs& p, uint32_t seq0, QLds4& row) {
  uint32_t drops = 0, seq = seq0;
#pragma unroll
  for (uint32_t b = 0; b < 2; ++b) {
    if (b * kWave >= n) break;
    const bool ins = b * kWave + lane < n && (p.lq[b] >> 16) == q;
    const uint64_t m = ballot(ins);
    if (!m) continue;
    drops += q4_insert_batch<DEC>(c, Q, lane, ins, p.rid[b], p.dec[b], p.lq[b] & 0xFFFF, seq, m, row);
    seq += (uint32_t)__popcll(m);
  }
  return drops;
}

// pend_flush_wave for queues of more than 64 slots
__device__ __forceinline__ uint32_t q4_pend_flush_wave(const GCfg& c, const GState& s, uint64_t l, uint32_t lane,
                                                       uint32_t pc, QLds4& row) {
  const uint32_t n = pend_total(pc);
  if (n == 0) return 0;
  PendRegs p;
  pend_load(s, l, lane, n, p);
  uint32_t drops = 0;
  for (uint32_t q = 0; q < 3; ++q) {
    const uint32_t nq = (pc >> (8 * q)) & 0xFF;
    if (!nq) continue;
    Q4 Q;
    q4_load(c, s, l, q, lane, Q);
    const uint32_t seq0 = s.q_next_seq[l * 3 + q];
    drops += q4_pend_apply<true>(c, Q, lane, q, n, p, seq0, row);
    q4_store(c, s, l, q, lane, Q);
    if (lane == 0) s.q_next_seq[l * 3 + q] = seq0 + nq;
  }
  if (lane == 0) {
    s.p_cnt[l] = 0;
    if (drops) s.q_pruned[l] += drops;
  }
  return drops;
}

// q_expire: stale items dropped, the survivors keep their order at the front
__device__ __forceinline__ uint32_t q4_expire(const GCfg& c, Q4& Q, uint32_t lane, const bool (&stale)[kQK], bool dec,
                                              QLds4& row) {
  bool keep[kQK];
  uint32_t ck = 0, cs = 0;
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) {
    const bool live = q4_live(c, Q, lane, k);
    keep[k] = live && !stale[k];
    ck += keep[k];
    cs += live && stale[k];
  }
  uint32_t n_stale;
  (void)lanes_excl(cs, n_stale);
  if (!n_stale) return 0;
  uint32_t n_keep;
  uint32_t r = lanes_excl(ck, n_keep);
  uint32_t dst[kQK];
#pragma unroll
  for (uint32_t k = 0; k < kQK; ++k) dst[k] = keep[k] ? r++ : kEmpty;
  if (dec) q4_scatter<true>(c, Q, lane, dst, n_keep, row);
  else q4_scatter<false>(c, Q, lane, dst, n_keep, row);
  return n_stale;
}
