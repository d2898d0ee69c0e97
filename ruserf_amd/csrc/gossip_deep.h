// gossip_deep.h — deep transmit-limited queues: the whole-queue paths (included by gossip.hip).
//
// A deep queue (queue_depth > queue_cap) is its sorted register head (the q_* slots emission
// works on) plus an UNORDERED tail in HBM with a summary {count, length bound, key bound}.  The
// reference's TransmitLimitedQueue (memberlist, un-vendored; core/src/serf/base.rs:178-189) is
// unbounded between QueueChecker ticks, which prune it to max_queue_depth = 4096
// (options.rs:512, base.rs:720-760) -- far more than a register head holds.  emit_run decides a
// member's picks from the head alone when the tail provably cannot change them (every pick's key
// below the tail's key bound, every stop one no tail item could fit) and commits; otherwise it
// stores nothing and lists the member here.  emit_deep_kernel then redoes that member's whole
// emission exactly, one block per member, with the queue's every item in LDS:
//   pending re-queues appended (transmits 0, next seqs) -> bounded-queue prune to the depth ->
//   per peer, queue-major, get_broadcasts = repeated block argmin of the fitting unpicked keys,
//   then transmits + 1 or retire -> head = the queue_cap smallest keys in order, tail = the rest.
// The same block routines run the QueueChecker's prune (check_deep_kernel).
#pragma once

namespace {

constexpr uint32_t kDeepThreads = 256;
constexpr uint32_t kDeepWaves = kDeepThreads / kWave;
// a queue's items in LDS: head + tail (<= RSF_MAX_QUEUE_DEPTH) + one pending list's new items
constexpr uint32_t kDeepItems = RSF_MAX_QUEUE_DEPTH + kPend;
enum : uint8_t { kDeepDead = 0, kDeepLive = 1, kDeepPicked = 2 };

struct DeepLds {
  uint64_t key[kDeepItems];
  uint32_t rid[kDeepItems];
  uint32_t dec[kDeepItems];
  uint8_t st[kDeepItems];
  GState::PendE pend[kPend];
  uint32_t hist[256];
  uint64_t hkey[kWave];
  uint32_t hrid[kWave], hdec[kWave];
  uint64_t w64[kDeepWaves];
  uint32_t w32[kDeepWaves];
  uint64_t off[8];
  uint32_t* oc[8];
  uint32_t used[8], nrec[8];
  uint32_t sel_digit, sel_need, sel_idx, hn, tn, np, err, drops;
};

__device__ __forceinline__ uint32_t key_len(uint64_t k) { return 0xFFFFu - (uint32_t)((k >> 32) & 0xFFFF); }
__device__ __forceinline__ uint32_t key_seq(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }
__device__ __forceinline__ uint32_t key_tl(uint64_t k) { return (uint32_t)(k >> 48) | (key_len(k) << 16); }

// block-wide reductions (every thread calls; the result is block-uniform)
__device__ __forceinline__ uint64_t blk_min_u64(uint64_t v, DeepLds& d) {
  v = wave_min_u64(v);
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) d.w64[threadIdx.x / kWave] = v;
  __syncthreads();
  uint64_t m = d.w64[0];
#pragma unroll
  for (uint32_t w = 1; w < kDeepWaves; ++w) m = d.w64[w] < m ? d.w64[w] : m;
  return m;
}
__device__ __forceinline__ uint32_t blk_min_u32(uint32_t v, DeepLds& d) {
  v = wave_min_u32(v);
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) d.w32[threadIdx.x / kWave] = v;
  __syncthreads();
  uint32_t m = d.w32[0];
#pragma unroll
  for (uint32_t w = 1; w < kDeepWaves; ++w) m = min(m, d.w32[w]);
  return m;
}
__device__ __forceinline__ uint32_t blk_sum_u32(uint32_t v, DeepLds& d) {
  v = wave_inclusive_sum_u32(v);
  v = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) d.w32[threadIdx.x / kWave] = v;
  __syncthreads();
  uint32_t m = 0;
#pragma unroll
  for (uint32_t w = 0; w < kDeepWaves; ++w) m += d.w32[w];
  return m;
}

// The k-th smallest (1-based) key of the live items [0, n) -- keys are distinct -- by an 8-bit
// radix select: per digit a histogram of the candidates still matching the decided prefix,
// then the digit where the running count reaches k.
__device__ uint64_t blk_select_kth(DeepLds& d, uint32_t n, uint32_t k) {
  const uint32_t tid = threadIdx.x;
  uint64_t prefix = 0, mask = 0;
  uint32_t need = k;
  for (int shift = 56; shift >= 0; shift -= 8) {
    __syncthreads();
    for (uint32_t i = tid; i < 256; i += kDeepThreads) d.hist[i] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kDeepThreads)
      if (d.st[i] != kDeepDead && (d.key[i] & mask) == prefix) atomicAdd(&d.hist[(d.key[i] >> shift) & 0xFF], 1u);
    __syncthreads();
    if (tid < kWave) {  // running counts over the 256 bins, four per lane
      const uint32_t h0 = d.hist[4 * tid], h1 = d.hist[4 * tid + 1], h2 = d.hist[4 * tid + 2], h3 = d.hist[4 * tid + 3];
      const uint32_t sum = h0 + h1 + h2 + h3, incl = wave_inclusive_sum_u32(sum), excl = incl - sum;
      if (excl < need && need <= incl) {
        uint32_t b = 0, acc = excl;
        if (acc + h0 < need) {
          acc += h0;
          b = 1;
          if (acc + h1 < need) {
            acc += h1;
            b = 2;
            if (acc + h2 < need) {
              acc += h2;
              b = 3;
            }
          }
        }
        d.sel_digit = 4 * tid + b;
        d.sel_need = need - acc;
      }
    }
    __syncthreads();
    prefix |= (uint64_t)d.sel_digit << shift;
    mask |= 0xFFull << shift;
    need = d.sel_need;
  }
  return prefix;
}

// the queue's live items into LDS: the head's live prefix at [0, hn), the tail after it;
// returns n = hn + tail count (block-uniform)
__device__ uint32_t deep_load_queue(const GCfg& c, const GState& s, uint64_t l, uint32_t q, DeepLds& d) {
  const uint32_t tid = threadIdx.x;
  if (tid < kWave) {
    QRegs Q{kEmpty, 0, 0};
    q_load(c, s, l, q, tid, Q);
    const bool live = tid < c.qcap && Q.r != kEmpty;
    if (live) {
      d.key[tid] = tlq_key(Q.tl & 0xFFFF, Q.tl >> 16, Q.sq);
      d.rid[tid] = Q.r;
      d.dec[tid] = Q.dec;
      d.st[tid] = kDeepLive;
    }
    const uint64_t m = ballot(live);
    if (tid == 0) d.hn = (uint32_t)__popcll(m);
  }
  __syncthreads();
  const uint32_t hn = d.hn;
  const uint32_t tc = tcap_of(c, q) ? s.tsum[l * 3 + q].x : 0u;
  const uint4* t = tcap_of(c, q) ? tail_of(s, q) + l * tstride_of(c, q) : nullptr;
  const uint32_t qdec = q == 1 ? kDecQuery : kDecEvent;
  for (uint32_t i = tid; i < tc; i += kDeepThreads) {
    const uint4 e = t[i];
    d.key[hn + i] = tlq_key(e.z & 0xFFFF, e.z >> 16, e.y);
    d.rid[hn + i] = e.x;
    d.dec[hn + i] = q == 0 ? e.w : qdec;
    d.st[hn + i] = kDeepLive;
  }
  __syncthreads();
  return hn + tc;
}

// keep the `keep` smallest live keys (the bounded queue's prune); returns how many it dropped
__device__ uint32_t deep_keep_smallest(DeepLds& d, uint32_t n, uint32_t keep) {
  uint32_t live = 0;
  for (uint32_t i = threadIdx.x; i < n; i += kDeepThreads) live += d.st[i] != kDeepDead;
  live = blk_sum_u32(live, d);
  if (live <= keep) return 0;
  const uint64_t T = keep ? blk_select_kth(d, n, keep) : 0ull;
  for (uint32_t i = threadIdx.x; i < n; i += kDeepThreads)
    if (d.st[i] != kDeepDead && (keep == 0 || d.key[i] > T)) d.st[i] = kDeepDead;
  __syncthreads();
  return live - keep;
}

// the queue back to HBM: head = the qcap smallest live keys in send order (free slots after
// them), tail = every other live item (any order) with its exact bounds
__device__ void deep_store_queue(const GCfg& c, const GState& s, uint64_t l, uint32_t q, DeepLds& d, uint32_t n) {
  const uint32_t tid = threadIdx.x;
  uint32_t live = 0;
  for (uint32_t i = tid; i < n; i += kDeepThreads) live += d.st[i] != kDeepDead;
  live = blk_sum_u32(live, d);
  const uint64_t T = live > c.qcap ? blk_select_kth(d, n, c.qcap) : ~0ull;
  if (tid == 0) {
    d.hn = 0;
    d.tn = 0;
  }
  __syncthreads();
  uint4* const t = tcap_of(c, q) ? tail_of(s, q) + l * tstride_of(c, q) : nullptr;
  uint64_t tmin = ~0ull;
  uint32_t tlmin = ~0u;
  for (uint32_t i = tid; i < n; i += kDeepThreads) {
    if (d.st[i] == kDeepDead) continue;
    const uint64_t k = d.key[i];
    if (k <= T) {
      const uint32_t h = atomicAdd(&d.hn, 1u);
      d.hkey[h] = k;
      d.hrid[h] = d.rid[i];
      d.hdec[h] = d.dec[i];
    } else {  // only a deep queue holds more live items than its head
      const uint32_t j = atomicAdd(&d.tn, 1u);
      t[j] = make_uint4(d.rid[i], key_seq(k), key_tl(k), d.dec[i]);
      tmin = k < tmin ? k : tmin;
      tlmin = min(tlmin, key_len(k));
    }
  }
  tmin = blk_min_u64(tmin, d);
  tlmin = blk_min_u32(tlmin, d);
  if (tid < kWave) {  // wave 0: the head in key order (rank = smaller keys among the head's)
    const uint32_t hn = d.hn;
    const uint64_t mk = tid < hn ? d.hkey[tid] : ~0ull;
    uint32_t rank = 0;
    for (uint32_t j = 0; j < hn; ++j) rank += d.hkey[j] < mk ? 1u : 0u;
    if (tid < c.qcap) {
      const uint32_t slot = tid < hn ? rank : tid;
      const uint64_t i = (l * 3 + q) * c.qcap + slot;
      const bool h = tid < hn;
      s.q_rumor[i] = h ? d.hrid[tid] : kEmpty;
      s.q_seq[i] = h ? key_seq(mk) : 0u;
      s.q_txlen[i] = h ? key_tl(mk) : 0u;
      if (q == 0) s.q_dec[l * c.qcap + slot] = h ? d.hdec[tid] : 0u;
    }
  }
  if (tid == 0 && tcap_of(c, q)) s.tsum[l * 3 + q] = d.tn ? make_uint4(d.tn, tlmin, (uint32_t)tmin, (uint32_t)(tmin >> 32))
                                                      : kTSumEmpty;
  __syncthreads();
}

// one member's whole emission (emit_run's semantics over every item of every queue)
template <bool BKT>
__device__ void deep_emit_member(const GCfg& c, const GState& s, uint64_t l, const uint32_t* __restrict__ grp_key,
                                 const uint32_t* __restrict__ slot, uint32_t* __restrict__ cnt_s,
                                 uint32_t* __restrict__ out_val, uint32_t* __restrict__ out_dec, const Buckets& bk,
                                 DeepLds& d) {
  const uint32_t tid = threadIdx.x;
  const uint32_t pc = s.p_cnt[l], npend = pend_total(pc);
  if (tid < kWave) {  // the peers (a prefix of the fanout slots): where each one's records go
    const uint32_t gk = tid < c.fanout ? grp_key[l * c.fanout + tid] : kSentinel;
    const uint32_t gs = tid < c.fanout ? slot[l * c.fanout + tid] : 0u;
    const uint64_t pm = ballot(gk != kSentinel);
    if (tid == 0) {
      d.np = (uint32_t)__popcll(pm);
      d.err = 0;
      d.drops = 0;
    }
    if (tid < c.fanout) {
      uint64_t off = ~0ull;
      uint32_t* oc = nullptr;
      if (gk != kSentinel) {
        if (BKT) {
          const uint32_t w = gs >> kBktWShift, idx = gs & kBktIdxMask;
          if (idx < bk.gcap) {
            off = (uint64_t)w * bk.stride_u32 + bk.vals_off + (uint64_t)idx * c.cap_t;
            oc = bk.send + (uint64_t)w * bk.stride_u32 + bk.cnt_off + idx;
          }
        } else {
          off = (uint64_t)gs * c.cap_t;
          oc = cnt_s + gs;
        }
      }
      d.off[tid] = off;
      d.oc[tid] = oc;
      d.used[tid] = 0;
      d.nrec[tid] = 0;
    }
  }
  for (uint32_t i = tid; i < npend; i += kDeepThreads) d.pend[i] = s.p_ent[l * kPend + i];
  __syncthreads();
  const uint32_t np = d.np;
  uint32_t* const ov = BKT ? bk.send : out_val;
  uint32_t* const od = BKT ? nullptr : out_dec;
  for (uint32_t q = 0; q < 3; ++q) {
    const uint32_t nq = (pc >> (8 * q)) & 0xFF;
    uint32_t n = deep_load_queue(c, s, l, q, d);
    if (n == 0 && nq == 0) continue;
    // the pending re-queues of this queue, in list order, transmits 0 and the next seqs
    if (tid < kWave) {
      const uint32_t seq0 = s.q_next_seq[l * 3 + q];
      const uint32_t qdec = q == 1 ? kDecQuery : kDecEvent;
      uint32_t rank0 = 0;
      for (uint32_t b = 0; b < kPend / kWave; ++b) {
        const uint32_t i = b * kWave + tid;
        const bool in = i < npend && (d.pend[i].lq >> 16) == q;
        const uint64_t m = ballot(in);
        if (in) {
          const uint32_t r = rank0 + mbcnt(m), j = n + r;
          d.key[j] = tlq_key(0, d.pend[i].lq & 0xFFFF, seq0 + r);
          d.rid[j] = d.pend[i].rid;
          d.dec[j] = q == 0 ? d.pend[i].dec : qdec;
          d.st[j] = kDeepLive;
        }
        rank0 += (uint32_t)__popcll(m);
      }
    }
    __syncthreads();
    n += nq;
    // inserting into a bounded queue with no pick in between keeps its depth smallest keys
    const uint32_t dropped = deep_keep_smallest(d, n, c.qcap + tcap_of(c, q));
    if (tid == 0) d.drops += dropped;
    // get_broadcasts for every peer, queue-major: the smallest fitting unpicked key, repeated
    for (uint32_t j = 0; j < np; ++j) {
      const uint32_t lim = c.limit - d.used[j];
      uint32_t used = 0, k = 0;
      for (;;) {
        const int32_t free_b = (int32_t)(lim - used - c.overhead);
        if (free_b <= 0) break;
        uint64_t best = ~0ull;
        for (uint32_t i = tid; i < n; i += kDeepThreads)
          if (d.st[i] == kDeepLive) {
            const uint64_t x = d.key[i];
            if (key_len(x) <= (uint32_t)free_b && x < best) best = x;
          }
        best = blk_min_u64(best, d);
        if (best == ~0ull) break;
        for (uint32_t i = tid; i < n; i += kDeepThreads)
          if (d.st[i] == kDeepLive && d.key[i] == best) d.sel_idx = i;
        __syncthreads();
        if (tid == 0) {
          const uint32_t w = d.sel_idx, pos = d.nrec[j] + k;
          d.st[w] = kDeepPicked;
          if (pos < c.cap_t && d.off[j] != ~0ull) {
            ov[d.off[j] + pos] = d.rid[w];
            if (od) od[d.off[j] + pos] = d.dec[w];
          }
        }
        k++;
        used += c.overhead + key_len(best);
        __syncthreads();
      }
      for (uint32_t i = tid; i < n; i += kDeepThreads)  // transmits + 1, or retired at the limit
        if (d.st[i] == kDeepPicked) {
          if ((uint32_t)(d.key[i] >> 48) + 1 >= c.tx_limit) {
            d.st[i] = kDeepDead;
          } else {
            d.key[i] += 1ull << 48;
            d.st[i] = kDeepLive;
          }
        }
      if (tid == 0) {
        if (d.nrec[j] + k > c.cap_t) d.err |= kErrStage;
        d.nrec[j] += k;
        d.used[j] += used;
      }
      __syncthreads();
    }
    deep_store_queue(c, s, l, q, d, n);
    if (tid < kWave) {  // clear the state flags for the next queue
      for (uint32_t i = tid; i < n; i += kWave) d.st[i] = kDeepDead;
    }
    __syncthreads();
  }
  // the groups' counts and the member's bookkeeping (emit_run's)
  if (tid < np) {
    uint32_t* oc = d.oc[tid];
    if (oc && (BKT || d.nrec[tid])) *oc = min(d.nrec[tid], c.cap_t);
  }
  if (tid == 0) {
    if (npend) {
      s.p_cnt[l] = 0;
      for (uint32_t q = 0; q < 3; ++q) s.q_next_seq[l * 3 + q] += (pc >> (8 * q)) & 0xFF;
    }
    uint32_t err = d.err;
    if (d.drops) {
      s.q_pruned[l] += d.drops;
      err |= kErrQueue;
    }
    if (err) s.err[l] |= err;
  }
  __syncthreads();
}

// the members emit_run deferred (s.deep_ids, count *s.deep_n): one block each; every block
// walks the list with a stride of the grid, so each one reaches the end
template <bool BKT>
__global__ void __launch_bounds__(kDeepThreads) emit_deep_kernel(GCfg c, GState s, const uint32_t* __restrict__ grp_key,
                                                                const uint32_t* __restrict__ slot,
                                                                uint32_t* __restrict__ cnt_s,
                                                                uint32_t* __restrict__ out_val,
                                                                uint32_t* __restrict__ out_dec, Buckets bk,
                                                                unsigned long long* __restrict__ total) {
  __shared__ DeepLds d;
  const uint32_t n_list = *s.deep_n;
  if (blockIdx.x == 0 && threadIdx.x == 0 && n_list) atomicAdd(total, (unsigned long long)n_list);
  for (uint32_t i = 0; i < kDeepItems; i += kDeepThreads)
    if (i + threadIdx.x < kDeepItems) d.st[i + threadIdx.x] = kDeepDead;
  __syncthreads();
  for (uint32_t it = blockIdx.x; it < n_list; it += gridDim.x) {
    const uint64_t l = s.deep_ids[it];
    if (l >= c.n_loc) continue;  // block-uniform
    deep_emit_member<BKT>(c, s, l, grp_key, slot, cnt_s, out_val, out_dec, bk, d);
  }
}

// QueueChecker prune of deep queues listed by check_queues_kernel (entries l * 3 + q): keep the
// max_depth smallest keys of head and tail
__global__ void __launch_bounds__(kDeepThreads) check_deep_kernel(GCfg c, GState s, uint32_t max_depth) {
  __shared__ DeepLds d;
  const uint32_t n_list = *s.deep_n;
  for (uint32_t i = 0; i < kDeepItems; i += kDeepThreads)
    if (i + threadIdx.x < kDeepItems) d.st[i + threadIdx.x] = kDeepDead;
  __syncthreads();
  for (uint32_t it = blockIdx.x; it < n_list; it += gridDim.x) {
    const uint32_t e = s.deep_ids[it];
    const uint64_t l = e / 3;
    const uint32_t q = e % 3;
    if (l >= c.n_loc) continue;
    const uint32_t n = deep_load_queue(c, s, l, q, d);
    deep_keep_smallest(d, n, max_depth);
    deep_store_queue(c, s, l, q, d, n);
    for (uint32_t i = threadIdx.x; i < n; i += kDeepThreads) d.st[i] = kDeepDead;
    __syncthreads();
  }
}

// ring wrap: a deep queue's tail drops its items of the recycled generation (one wave per
// (member, queue), in place, order kept); returns the number dropped; exact new bounds
__device__ __forceinline__ uint32_t tail_expire_wave(const GCfg& c, const GState& s, uint64_t l, uint32_t q,
                                                     uint32_t lane, uint32_t gen, uint32_t G) {
  if (!tcap_of(c, q)) return 0;
  const uint4 sm = s.tsum[l * 3 + q];
  if (!sm.x) return 0;
  uint4* const t = tail_of(s, q) + l * tstride_of(c, q);
  uint32_t kept = 0, gone = 0, lmin = ~0u;
  uint64_t kmin = ~0ull;
  for (uint32_t b = 0; b < sm.x; b += kWave) {
    const bool in = b + lane < sm.x;
    const uint4 e = in ? t[b + lane] : make_uint4(kEmpty, 0u, 0u, 0u);
    const bool stale = in && (gen + G - (e.x >> c.rbits) % G) % G >= 2;
    const bool keep = in && !stale;
    const uint64_t km = ballot(keep);
    __threadfence_block();  // every lane has read its item before any is overwritten
    if (keep) t[kept + mbcnt(km)] = e;
    const uint64_t k = keep ? tlq_key(e.z & 0xFFFF, e.z >> 16, e.y) : ~0ull;
    const uint64_t mk = wave_min_u64(k);
    kmin = mk < kmin ? mk : kmin;
    lmin = min(lmin, wave_min_u32(keep ? (e.z >> 16) : ~0u));
    kept += (uint32_t)__popcll(km);
    gone += (uint32_t)__popcll(ballot(stale));
  }
  if (gone && lane == 0)
    s.tsum[l * 3 + q] = kept ? make_uint4(kept, lmin, (uint32_t)kmin, (uint32_t)(kmin >> 32)) : kTSumEmpty;
  return gone;
}

}  // namespace
