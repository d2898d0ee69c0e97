// gossip_deep.h — deep transmit-limited queues: the whole-queue paths (included by gossip.hip).
//
// A deep queue (queue_depth > queue_cap) is its sorted register head (the q_* slots emission
// works on) plus an UNORDERED tail in HBM with a summary {count, length bound, key bound}.  The
// reference's TransmitLimitedQueue (memberlist, un-vendored; core/src/serf/base.rs:178-189) is
// unbounded between QueueChecker ticks, which prune it to max_queue_depth = 4096
// (options.rs:512, base.rs:720-760) -- far more than a register head holds.  emit_run decides a
// member's picks from the head alone when the tail provably cannot change them (every pick's key
// below the tail's key bound, every stop one no tail item could fit) and commits; otherwise it
// stores nothing and lists the member for emit_deep_wave_kernel (below), which redoes that
// member's emission with every item of its queues in LDS.  The block routines first in this file
// run the QueueChecker's prune (check_stream_kernel).
#pragma once

namespace {

constexpr uint32_t kDeepThreads = 256;
// tail items a refill leaves unsealed past the head (w_store_tail, check_stream_kernel)
#ifndef RSF_DEEP_RESERVE
#define RSF_DEEP_RESERVE 128  // 64 and 256 measured slower (profiles/r06/ab_tunables/)
#endif
constexpr uint32_t kDeepReserve = RSF_DEEP_RESERVE;
// items per thread / lane in flight in the tail loads and LDS scans
#ifndef RSF_DEEP_U
#define RSF_DEEP_U 4  // 4 and 6: emission phase -0.035 ms against 8 and 2, same box x3 (profiles/r06/ab_deep_u/)
#endif
constexpr uint32_t kDeepU = RSF_DEEP_U;
constexpr uint32_t kDeepWaves = kDeepThreads / kWave;
enum : uint8_t { kDeepDead = 0, kDeepLive = 1, kDeepPicked = 2 };

__device__ __forceinline__ uint32_t key_len(uint64_t k) { return 0xFFFFu - (uint32_t)((k >> 32) & 0xFFFF); }
__device__ __forceinline__ uint32_t key_seq(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }
__device__ __forceinline__ uint32_t key_tl(uint64_t k) { return (uint32_t)(k >> 48) | (key_len(k) << 16); }

// wave AND / OR by butterfly shuffles (every lane gets the result)
__device__ __forceinline__ uint64_t wave_and_u64_blk(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v &= (uint64_t)__shfl_xor((long long)v, o);
  return v;
}
__device__ __forceinline__ uint64_t wave_or_u64_blk(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= (uint64_t)__shfl_xor((long long)v, o);
  return v;
}
// ---- one wave per deferred member ------------------------------------------------------
#if RSF_DEEP_PROF
// per-wave totals (one wave per block), added to g_deep_prof once at the kernel's end
__shared__ unsigned long long s_dprof[64];
#endif
// The path emit_run defers to (a member whose picks its head could not decide).  Per queue:
// every item (head, tail, the pending re-queues) into the wave's LDS, the bounded prune to the
// depth, then the REFILL: the queue_cap smallest keys become the register head (sorted) and the
// rest the tail with exact bounds, and the ordinary head emission (q_pick_peers with the deep
// checks) runs again -- with the true smallest keys in the head it almost always decides.  If
// it still cannot, the picks are made over the LDS items directly (repeated wave argmin of the
// fitting unpicked keys, as get_broadcasts restated), and head / tail are rebuilt after them.
// Capacities: kDeepTiny items (15 KB of LDS), kDeepSmall (20 KB) and kDeepMid (35 KB) for the common cases,
// the full depth (117 KB) for the rest; emit_run lists a member by the size its largest queue
// needs.
constexpr uint32_t kDeepBig = kDeepItems;
constexpr uint8_t kDeepInHead = 3;

// No per-item decoration: an item's decoration is a function of its queue and rumor (the
// intent queue's is the rumor's record decoration, s.rdec; the query / event queues' a
// constant), so it is read when the item enters the head (head_dec) or is picked by the
// per-peer fallback -- 4 B per item less LDS (the middle class 4 waves per CU instead of 3).
template <uint32_t CAP>
struct DeepWave {
  uint64_t key[CAP];
  uint32_t rid[CAP];
  uint8_t st[CAP];
  GState::PendE pend[kPend];
  uint32_t hist[256];
  uint64_t hkey[kWave];
  uint32_t hrid[kWave];
  QLds row;  // q_pick_peers' re-rank scratch
};

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t wave_and_u64(uint64_t v) {
  v &= dpp64<0xB1, 0xF>(v);
  v &= dpp64<0x4E, 0xF>(v);
  v &= dpp64<0x124, 0xF>(v);
  v &= dpp64<0x128, 0xF>(v);
  v &= dpp64<0x142, 0xA>(v);
  v &= dpp64<0x143, 0xC>(v);
  return lane63_u64(v);
}
__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
  v |= dpp64<0xB1, 0xF>(v);
  v |= dpp64<0x4E, 0xF>(v);
  v |= dpp64<0x124, 0xF>(v);
  v |= dpp64<0x128, 0xF>(v);
  v |= dpp64<0x142, 0xA>(v);
  v |= dpp64<0x143, 0xC>(v);
  return lane63_u64(v);
}

// The LDS scans below read kDeepU items per lane before using any (one LDS round trip per
// kDeepU * 64 items instead of one per 64).

// kDeepU items per lane from LDS: every load issued (in-range indices) before any is used;
// v[u]: item b + u * 64 + lane exists and is in state `state`, x[u] its key
template <uint32_t CAP>
__device__ __forceinline__ void w_chunk(const DeepWave<CAP>& d, uint32_t lane, uint32_t n, uint32_t b, uint8_t state,
                                        uint64_t (&x)[kDeepU], bool (&v)[kDeepU]) {
  uint32_t sv[kDeepU];
#pragma unroll
  for (uint32_t u = 0; u < kDeepU; ++u) {
    const uint32_t i = b + u * kWave + lane;
    const uint32_t ii = i < n ? i : 0u;
    sv[u] = d.st[ii];
    x[u] = d.key[ii];
  }
#pragma unroll
  for (uint32_t u = 0; u < kDeepU; ++u) v[u] = (b + u * kWave + lane < n) & (sv[u] == state);
}

// the items in state `state`: count, smallest and largest key, AND and OR of the keys
struct WRange {
  uint32_t cnt, cnt_t0;  // cnt_t0: those of transmits 0
  uint64_t lo, hi, an, orr;
};
template <uint32_t CAP>
__device__ WRange w_range(const DeepWave<CAP>& d, uint32_t lane, uint32_t n, uint8_t state) {
  uint32_t cnt = 0, c0 = 0;
  uint64_t lo = ~0ull, hi = 0, an = ~0ull, orr = 0;
  for (uint32_t b = 0; b < n; b += kDeepU * kWave) {
    uint64_t x[kDeepU];
    bool v[kDeepU];
    w_chunk(d, lane, n, b, state, x, v);
#pragma unroll
    for (uint32_t u = 0; u < kDeepU; ++u)
      if (v[u]) {
        cnt++;
        c0 += (x[u] >> 48) == 0 ? 1u : 0u;
        lo = x[u] < lo ? x[u] : lo;
        hi = x[u] > hi ? x[u] : hi;
        an &= x[u];
        orr |= x[u];
      }
  }
  WRange r;
  r.cnt = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum_u32(cnt), 63);
  r.cnt_t0 = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum_u32(c0), 63);
  r.lo = wave_min_u64(lo);
  r.hi = wave_max_u64(hi);
  r.an = wave_and_u64(an);
  r.orr = wave_or_u64(orr);
  return r;
}

// the k-th smallest (1-based) key among the items in state `state` (distinct keys; rg their
// w_range): 8-bit radix select, one wave.  Bytes every candidate key shares (the top bytes, the
// high byte of the length and of the seq) are taken from rg without a pass; a digit's lanes
// that agree with the first active lane's digit (the common case: one transmit class, few
// lengths) are counted by that lane alone; the select stops as soon as the chosen bucket holds
// one key.
// Register variant for the smaller capacities (<= kDeepSmall items: <= 19 keys per lane): the
// keys stay in registers and the k-th is built one VARYING bit at a time (the bits where the
// candidates' AND and OR differ), each bit one compare + ballot popcount per key -- no LDS
// histogram, no atomics.  Non-candidates hold ~0, which never matches a prefix: every
// candidate key has bit 63 clear (transmits < 2^15), checked by the caller.
#ifndef RSF_DEEP_SELECT_REG
#define RSF_DEEP_SELECT_REG 1
#endif
template <uint32_t R>
__device__ uint64_t w_select_kth_keys(const uint64_t (&kr)[R], uint32_t k, const WRange& rg) {
  const uint64_t var = rg.an ^ rg.orr;
  uint64_t mask = ~var, prefix = rg.an & ~var;  // the bits every candidate shares
  uint32_t need = k, match = rg.cnt;
  uint64_t rem = var;
  while (rem) {
    const int b = 63 - __clzll((long long)rem);
    rem &= ~(1ull << b);
    const uint64_t mb = mask | (1ull << b);
    uint32_t c0 = 0;  // candidates under the prefix with bit b clear
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) c0 += (uint32_t)__popcll(ballot((kr[r] & mb) == prefix));
    mask = mb;
    if (need <= c0) {
      match = c0;
    } else {
      need -= c0;
      match -= c0;
      prefix |= 1ull << b;
    }
    if (match == 1 && rem) {  // one candidate left under the prefix: it is the k-th
      uint64_t best = ~0ull;
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) best = (kr[r] & mask) == prefix ? kr[r] : best;
      return wave_min_u64(best);
    }
  }
  return prefix;
}

// the keys of LDS items lane, 64 + lane, ... in state `state` (~0 for the others) and their range
template <uint32_t CAP, uint32_t R>
__device__ __forceinline__ WRange w_keys(const DeepWave<CAP>& d, uint32_t lane, uint32_t n, uint8_t state,
                                         uint64_t (&kr)[R], uint32_t* vbits = nullptr) {
  uint32_t cnt = 0, c0 = 0, vb = 0;
  uint64_t lo = ~0ull, hi = 0, an = ~0ull, orr = 0;
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t i = r * kWave + lane;
    const uint32_t ii = i < n ? i : 0u;
    const uint8_t st = d.st[ii];
    const uint64_t x = d.key[ii];
    const bool v = i < n && st == state;
    kr[r] = v ? x : ~0ull;
    vb |= v ? 1u << r : 0u;
    cnt += v ? 1u : 0u;
    c0 += (v && (x >> 48) == 0) ? 1u : 0u;
    lo = v && x < lo ? x : lo;
    hi = v && x > hi ? x : hi;
    an &= v ? x : ~0ull;
    orr |= v ? x : 0ull;
  }
  WRange g;
  g.cnt = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum_u32(cnt), 63);
  g.cnt_t0 = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum_u32(c0), 63);
  g.lo = wave_min_u64(lo);
  g.hi = wave_max_u64(hi);
  g.an = wave_and_u64(an);
  g.orr = wave_or_u64(orr);
  if (vbits) *vbits = vb;
  return g;
}

template <uint32_t CAP>
__device__ uint64_t w_select_kth(DeepWave<CAP>& d, uint32_t lane, uint32_t n, uint32_t k, uint8_t state,
                                 const WRange& rg) {
  if (k <= 1 || rg.lo == rg.hi) return rg.lo;
  // (the smallest class only: at kDeepSmall the second register-resident key set beside
  // w_take_head's spills to scratch)
  if constexpr (RSF_DEEP_SELECT_REG && CAP <= kDeepTiny) {
    if (!(rg.orr >> 63)) {
      constexpr uint32_t R = (CAP + kWave - 1) / kWave;
      uint64_t kr[R];
      w_keys(d, lane, n, state, kr);
      return w_select_kth_keys(kr, k, rg);
    }
  }
  const uint64_t var = rg.an ^ rg.orr;  // the bits that differ between candidates
  uint64_t prefix = 0, mask = 0;
  uint32_t need = k;
  // at least k items of transmits 0: the k-th is one of them (the transmit bytes need no pass)
  const bool t0 = rg.cnt_t0 >= k;
  if (t0) mask = 0xFFFFull << 48;
#if RSF_DEEP_PROF
  if (lane == 0) s_dprof[19] += 1ull;
#endif
  for (int shift = 56; shift >= 0; shift -= 8) {
    const uint64_t bm = 0xFFull << shift;
    if (t0 && shift >= 48) continue;  // (prefix bytes 0)
    if (!(var & bm)) {  // every candidate has this byte
      prefix |= rg.an & bm;
      mask |= bm;
      continue;
    }
#if RSF_DEEP_PROF
    if (lane == 0) s_dprof[18] += 1ull;
#endif
    for (uint32_t i = lane; i < 256; i += kWave) d.hist[i] = 0;
    wsync();
    for (uint32_t b = 0; b < n; b += kDeepU * kWave) {
      uint64_t x[kDeepU];
      bool v[kDeepU];
      w_chunk(d, lane, n, b, state, x, v);
#pragma unroll
      for (uint32_t u = 0; u < kDeepU; ++u) {
        const bool in = v[u] && (x[u] & mask) == prefix;
        const uint32_t dg = (uint32_t)(x[u] >> shift) & 0xFF;
        const uint64_t am = ballot(in);
        if (!am) continue;
        const int f = __ffsll((long long)am) - 1;
        const uint32_t d0 = shfl_u32(dg, f);
        const uint64_t same = ballot(in && dg == d0);
        if (lane == (uint32_t)f) atomicAdd(&d.hist[d0], (uint32_t)__popcll(same));
        else if (in && dg != d0) atomicAdd(&d.hist[dg], 1u);
      }
    }
    wsync();
    const uint32_t h0 = d.hist[4 * lane], h1 = d.hist[4 * lane + 1], h2 = d.hist[4 * lane + 2], h3 = d.hist[4 * lane + 3];
    const uint32_t sum = h0 + h1 + h2 + h3, incl = wave_inclusive_sum_u32(sum), excl = incl - sum;
    const bool here = excl < need && need <= incl;
    uint32_t b = 0, acc = excl, hb = h0;
    if (acc + h0 < need) {
      acc += h0;
      b = 1;
      hb = h1;
      if (acc + h1 < need) {
        acc += h1;
        b = 2;
        hb = h2;
        if (acc + h2 < need) {
          acc += h2;
          b = 3;
          hb = h3;
        }
      }
    }
    const int w = __ffsll((long long)ballot(here)) - 1;
    const uint32_t digit = shfl_u32(4 * lane + b, w);
    const uint32_t cnt = shfl_u32(hb, w);
    need = shfl_u32(need - acc, w);
    prefix |= (uint64_t)digit << shift;
    mask |= bm;
    wsync();
    if (cnt == 1 && shift > 0) {  // one key left in the bucket: it is the k-th
      uint64_t best = ~0ull;
      for (uint32_t i = lane; i < n; i += kWave)
        if (d.st[i] == state && (d.key[i] & mask) == prefix) best = d.key[i];
      return wave_min_u64(best);
    }
  }
  return prefix;
}

// the intent queue's head items get their rumor's record decoration (w_take_head leaves
// kDecLookup; the query / event queues' decorations are constants)
__device__ __forceinline__ void head_dec_fix(const GCfg& c, const GState& s, QRegs& Q) {
  if (Q.dec == kDecLookup && Q.r != kEmpty) Q.dec = s.rdec[Q.r & c.rmask];
}

// head = the qcap smallest live keys, sorted into the lanes of Q (marked kDeepInHead in LDS);
// returns the bounds of the live items left (the tail): (min key, min length), ~0 if none, and
// for w_store_tail the reserve's largest key rres (the (qcap + kDeepReserve)-th smallest: the
// head's picks leave the other items' keys as they are; ~0 when every item left is reserve)
template <uint32_t CAP>
__device__ __forceinline__ void w_take_head(const GCfg& c, DeepWave<CAP>& d, uint32_t lane, uint32_t n, uint32_t q, QRegs& Q,
                            uint64_t& tmin, uint32_t& tminlen, uint64_t& rres) {
#if RSF_DEEP_PROF
  uint64_t tt = __builtin_amdgcn_s_memtime();
#define RSF_TH_T(k)                                                     \
  do {                                                                  \
    const uint64_t tn = __builtin_amdgcn_s_memtime();                   \
    if (lane == 0) s_dprof[(k)] += (unsigned long long)(tn - tt); \
    tt = tn;                                                            \
  } while (0)
#else
#define RSF_TH_T(k) \
  do {              \
  } while (0)
#endif
  uint32_t base = 0;
  uint64_t km = ~0ull;
  uint32_t lm = ~0u;
  // (keys in registers up to kDeepSmall: at kDeepMid, 38 keys per lane, the wave needs 256
  // VGPRs and spills 204 B to scratch)
  if constexpr (RSF_DEEP_SELECT_REG && CAP <= kDeepSmall) {
    // the keys read once into registers: range, select and gather from them
    constexpr uint32_t R = (CAP + kWave - 1) / kWave;
    uint64_t kr[R];
    uint32_t vb;
    static_assert(R <= 32, "validity bits");
    const WRange rg = w_keys(d, lane, n, kDeepLive, kr, &vb);
    RSF_TH_T(20);
    uint64_t T = ~0ull;
    rres = ~0ull;
    // the head's largest, then the reserve's: one select routine in a loop (two inlined copies
    // spill to scratch)
#pragma unroll 1
    for (uint32_t j = 0; j < 2; ++j) {
      const uint32_t k = j ? c.qcap + kDeepReserve : c.qcap;
      if (rg.cnt <= k) break;
      const uint64_t x = (rg.orr >> 63) ? w_select_kth(d, lane, n, k, kDeepLive, rg) : w_select_kth_keys(kr, k, rg);
      if (j) rres = x;
      else T = x;
    }
    RSF_TH_T(21);
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t i = r * kWave + lane;
      const bool v = (vb >> r) & 1u;
      const bool sel = v && kr[r] <= T;
      const uint64_t m = ballot(sel);
      if (sel) {
        const uint32_t pos = base + mbcnt(m);
        d.hkey[pos] = kr[r];
        d.hrid[pos] = d.rid[i];
        d.st[i] = kDeepInHead;
      } else if (v) {  // stays in the tail
        km = kr[r] < km ? kr[r] : km;
        lm = min(lm, key_len(kr[r]));
      }
      base += (uint32_t)__popcll(m);
    }
  } else {
  const WRange rg = w_range(d, lane, n, kDeepLive);
  RSF_TH_T(20);
  uint64_t T = ~0ull;
  rres = ~0ull;
#pragma unroll 1
  for (uint32_t j = 0; j < 2; ++j) {
    const uint32_t k = j ? c.qcap + kDeepReserve : c.qcap;
    if (rg.cnt <= k) break;
    const uint64_t x = w_select_kth(d, lane, n, k, kDeepLive, rg);
    if (j) rres = x;
    else T = x;
  }
  RSF_TH_T(21);
  for (uint32_t b0 = 0; b0 < n; b0 += kDeepU * kWave) {
    uint64_t x[kDeepU];
    bool v[kDeepU];
    w_chunk(d, lane, n, b0, kDeepLive, x, v);
#pragma unroll
    for (uint32_t u = 0; u < kDeepU; ++u) {
      const uint32_t i = b0 + u * kWave + lane;
      const bool sel = v[u] && x[u] <= T;
      const uint64_t m = ballot(sel);
      if (sel) {
        const uint32_t pos = base + mbcnt(m);
        d.hkey[pos] = x[u];
        d.hrid[pos] = d.rid[i];
        d.st[i] = kDeepInHead;
      } else if (v[u]) {  // stays in the tail
        km = x[u] < km ? x[u] : km;
        lm = min(lm, key_len(x[u]));
      }
      base += (uint32_t)__popcll(m);
    }
  }
  }
  tmin = wave_min_u64(km);
  tminlen = wave_min_u32(lm);
  wsync();
  RSF_TH_T(22);
  const uint32_t hn = base;
  const bool h = lane < hn;
  const uint64_t mk = h ? d.hkey[lane] : ~0ull;
  uint32_t rank = 0;
#pragma unroll 8
  for (uint32_t j = 0; j < hn; ++j) rank += d.hkey[j] < mk ? 1u : 0u;
  const uint64_t hm = ballot(h);
  const uint32_t dest = h ? rank : hn + mbcnt(~hm);
  const int addr = (int)(dest * 4);
  const uint32_t r = h ? d.hrid[lane] : kEmpty, sq = h ? key_seq(mk) : 0u, tl = h ? key_tl(mk) : 0u,
                 dc = q == 0 ? kDecLookup : (q == 1 ? kDecQuery : kDecEvent);  // (head_dec fills the intents')
  Q.r = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)r);
  Q.sq = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)sq);
  Q.tl = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)tl);
  Q.dec = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)dc);
  wsync();
  RSF_TH_T(23);
#undef RSF_TH_T
}

// U * 64 tail items [b + u * 64 + lane] of (l, q) in the unpacked 16-B form, all loads issued
// before any is used; indices at or past `end` give zeros.  The intent queue's packed items
// (q == 0) come back with decoration kDecLookup.
template <uint32_t U>
__device__ __forceinline__ void tail_chunk(const GCfg& c, const GState& s, uint64_t l, uint32_t q, uint32_t b,
                                           uint32_t end, uint32_t lane, uint32_t nseq, uint4 (&e)[U]) {
  if (q == 0) {
    const uint64_t* const t = tail8(s, c, l);
    uint64_t x[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = b + u * kWave + lane;
      x[u] = i < end ? t[i] : 0ull;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u)
      e[u] = b + u * kWave + lane < end ? tail_unpack(c, x[u], nseq) : make_uint4(0, 0, 0, 0);
  } else {
    const uint4* const t = tail16(s, q) + l * tstride_of(c, q);
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = b + u * kWave + lane;
      e[u] = i < end ? t[i] : make_uint4(0, 0, 0, 0);
    }
  }
}

// the live items not in the head back to the tail (compacted) at tail[t_lo ...], in two
// groups: first every item above the kDeepReserve-th smallest of them (they join the sealed
// prefix), then the kDeepReserve smallest (the RESERVE: left in the recent part, so the next
// refill -- which usually needs exactly the items just past the head, e.g. a backlog of
// transmits-0 items -- finds them without the sealed prefix).  Returns the count; *nb = the
// sealed group's size, *bmin = its smallest key (~0 if none).
template <uint32_t CAP>
__device__ __forceinline__ uint32_t w_store_tail(const GCfg& c, const GState& s, uint64_t l, uint32_t q, DeepWave<CAP>& d,
                                 uint32_t lane, uint32_t n, uint32_t t_lo, uint64_t R, uint32_t* nb, uint64_t* bmin) {
  // (q == 0: the intent queue's packed items; only a deep queue holds more live items than its head)
  uint4* const t = q && tcap_of(c, q) ? tail16(s, q) + l * tstride_of(c, q) + t_lo : nullptr;
  uint64_t* const t8 = q == 0 && c.tcap0 ? tail8(s, c, l) + t_lo : nullptr;
  // the sealed group's size first (one count pass: the reserve is R's items and below)
  uint32_t ns = 0;
  for (uint32_t b = 0; b < n; b += kWave) {
    const uint32_t i = b + lane;
    ns += (uint32_t)__popcll(ballot(i < n && d.st[i] == kDeepLive && d.key[i] > R));
  }
  // one pass writes both groups: sealed (> R) at [0, ns), the reserve (<= R) from ns on
  uint32_t bs = 0, br = ns;
  uint64_t bm = ~0ull;
  for (uint32_t b = 0; b < n; b += kWave) {
    const uint32_t i = b + lane;
    const uint64_t k = i < n ? d.key[i] : 0ull;
    const bool live = i < n && d.st[i] == kDeepLive;
    const bool sealed = live && k > R, res = live && k <= R;
    const uint64_t ms = ballot(sealed), mr = ballot(res);
    if (live) {
      const uint32_t at = sealed ? bs + mbcnt(ms) : br + mbcnt(mr);
      if (q == 0) t8[at] = tail_pack(c, d.rid[i], key_seq(k), key_tl(k));
      else t[at] = make_uint4(d.rid[i], key_seq(k), key_tl(k), q == 1 ? kDecQuery : kDecEvent);
    }
    if (sealed) bm = k < bm ? k : bm;
    bs += (uint32_t)__popcll(ms);
    br += (uint32_t)__popcll(mr);
  }
  *nb = ns;
  *bmin = wave_min_u64(bm);
  return br;
}

// the sealed prefix tail[0, sm) into LDS after the n items there (live): the recent mode could
// not decide, the member continues with every item; returns the new item count
// nseq: the queue's next seq before this emission (every tail item is older)
template <uint32_t CAP>
__device__ __forceinline__ uint32_t w_load_sealed(const GCfg& c, const GState& s, uint64_t l, uint32_t q, DeepWave<CAP>& d,
                                  uint32_t lane, uint32_t n, uint32_t sm, uint32_t nseq) {
  for (uint32_t i = lane; i < n; i += kWave)
    if (d.st[i] == kDeepInHead) d.st[i] = kDeepLive;
  for (uint32_t b = 0; b < sm; b += kDeepU * kWave) {
    uint4 e[kDeepU];
    tail_chunk<kDeepU>(c, s, l, q, b, sm, lane, nseq, e);
#pragma unroll
    for (uint32_t u = 0; u < kDeepU; ++u) {
      const uint32_t i = b + u * kWave + lane;
      if (i < sm) {
        d.key[n + i] = tlq_key(e[u].z & 0xFFFF, e[u].z >> 16, e[u].y);
        d.rid[n + i] = e[u].x;
        d.st[n + i] = kDeepLive;
      }
    }
  }
  wsync();
  return n + sm;
}

// A member's first round trip, issued while the wave still works on the member before it:
// its pending count, its peers' group keys and slots (lane j < fanout), and per queue (lane
// q < 3) the next seq, whether the head is non-empty (bit 0) and the tail count (<< 1), so
// empty queues cost nothing and the tail loads start at once.
struct DeepPre {
  uint32_t pc, gk, gs, qinfo, qseq;
  uint32_t sm;  // lane q < 3: the sealed prefix's count (tseal.x)
};
__device__ __forceinline__ DeepPre deep_pre(const GCfg& c, const GState& s, uint64_t l, uint32_t lane,
                                            const uint32_t* __restrict__ grp_key,
                                            const uint32_t* __restrict__ slot) {
  DeepPre p{0u, kSentinel, 0u, 0u, 0u, 0u};
  if (l >= c.n_loc) return p;
  p.pc = s.p_cnt[l];
  if (lane < c.fanout) {
    p.gk = grp_key[l * c.fanout + lane];
    p.gs = slot[l * c.fanout + lane];
  }
  if (lane < 3) {
    p.qseq = s.q_next_seq[l * 3 + lane];
    const uint32_t r0 = s.q_rumor[(l * 3 + lane) * c.qcap];
    const bool dq = tcap_of(c, lane) != 0;
    const uint32_t tcq = dq ? s.tsum[l * 3 + lane].x : 0u;
    p.qinfo = (r0 != kEmpty ? 1u : 0u) | (tcq << 1);
    p.sm = dq ? s.tseal[l * 3 + lane].x : 0u;
  }
  return p;
}

// recent mode could not decide: nothing of the member is stored yet, the full-depth class
// (launched after this one) redoes it; the wave's LDS items are cleared for the next member
template <uint32_t CAP>
__device__ __forceinline__ void deep_relist_full(const GCfg& c, const GState& s, uint64_t l, uint32_t lane, uint32_t n,
                                                 DeepWave<CAP>& d) {
  for (uint32_t i = lane; i < n; i += kWave) d.st[i] = kDeepDead;
  wsync();
  if (lane == 0) s.deep_ids[c.n_loc * 4 + atomicAdd(s.deep_n + 4, 1u)] = (uint32_t)l;  // list 4
#if RSF_DEEP_PROF
  if (lane == 0) s_dprof[30] += 1ull;
#endif
}

template <bool BKT, uint32_t CAP>
__device__ __forceinline__ void deep_wave_member(const GCfg& c, const GState& s, uint64_t l, uint32_t lane, const DeepPre& pre,
                                 uint32_t* __restrict__ cnt_s, uint32_t* __restrict__ out_val,
                                 uint32_t* __restrict__ out_dec, const Buckets& bk, DeepWave<CAP>& d) {
  const uint32_t pc = pre.pc, npend = pend_total(pc);
  // the peers (a prefix of the fanout slots); lane j < np: peer j's record offset and count word
  const uint32_t gk = pre.gk, gs = pre.gs;
  const uint32_t np = (uint32_t)__popcll(ballot(gk != kSentinel));
  uint64_t off_v = ~0ull;
  uint32_t* oc = nullptr;
  if (lane < np) {
    if (BKT) {
      const uint32_t w = gs >> kBktWShift, idx = gs & kBktIdxMask;
      if (idx < bk.gcap) {
        off_v = (uint64_t)w * bk.stride_u32 + bk.vals_off + (uint64_t)idx * c.cap_t;
        oc = bk.send + (uint64_t)w * bk.stride_u32 + bk.cnt_off + idx;
      }
    } else {
      off_v = (uint64_t)gs * c.cap_t;
      oc = cnt_s + gs;
    }
  }
#if RSF_DEEP_PROF
  uint64_t pt = __builtin_amdgcn_s_memtime();
  const uint64_t pt_start = pt;
#define RSF_DEEP_T(k)                                                   \
  do {                                                                  \
    const uint64_t pn = __builtin_amdgcn_s_memtime();                   \
    if (lane == 0) s_dprof[(k)] += (unsigned long long)(pn - pt); \
    pt = pn;                                                            \
  } while (0)
#else
#define RSF_DEEP_T(k) \
  do {                \
  } while (0)
#endif
  const uint32_t qinfo = pre.qinfo, qseq = pre.qseq;
  // the pending entries (two per lane) into registers now, into LDS once the first queue's
  // head and tail loads are in flight too: one round trip for all three
  static_assert(kPend == 2 * kWave, "two pending entries per lane");
  // (named scalars: a struct copy here is promoted to an LDS or scratch array)
  uint32_t pr0 = 0, pd0 = 0, pl0 = 0, pr1 = 0, pd1 = 0, pl1 = 0;
  if (lane < npend) {
    const GState::PendE* e = s.p_ent + l * kPend + lane;
    pr0 = e->rid;
    pd0 = e->dec;
    pl0 = e->lq;
  }
  if (kWave + lane < npend) {
    const GState::PendE* e = s.p_ent + l * kPend + kWave + lane;
    pr1 = e->rid;
    pd1 = e->dec;
    pl1 = e->lq;
  }
  bool pend_lds = false;
  uint32_t* const ov = BKT ? bk.send : out_val;
  uint32_t* const od = BKT ? bk.send + (bk.decs_off - bk.vals_off) : out_dec;
  uint32_t used_v = 0, nrec_v = 0, err = 0, drops = 0;
  for (uint32_t q = 0; q < 3; ++q) {
    const uint32_t nq = (pc >> (8 * q)) & 0xFF;
    const uint32_t qi = shfl_u32(qinfo, (int)q);
    if (qi == 0 && nq == 0) continue;  // nothing in head, tail or pending list
    // every item of the queue into LDS: the head's live prefix, the tail, then the pending
    // re-queues in list order (transmits 0, the next seqs)
    // issued together: the head, the tail's first kDeepU * 64 items; then the LDS writes
    QRegs Q{kEmpty, 0, 0};
    q_load(c, s, l, q, lane, Q);
    const uint32_t tc = qi >> 1;
    // RECENT mode (tseal): only the intent queue in use and a sealed tail prefix: load the
    // tail's recent part tail[sm, tc) only; valid if the refilled head is full and its largest
    // key is below the seal's bound (else the member is re-listed for the full depth before
    // anything is stored -- the intent queue is the first one processed).  The full-depth class
    // always loads everything.
    const uint32_t sm = shfl_u32(pre.sm, (int)q);
    const bool others_empty = q == 0 && shfl_u32(qinfo, 1) == 0 && shfl_u32(qinfo, 2) == 0 && ((pc >> 8) & 0xFFFF) == 0;
    bool recent = others_empty && sm > 0 && sm <= tc && tc + nq <= tcap_of(c, q);
    uint32_t t_lo = recent ? sm : 0u;
    const uint32_t tn = tc - t_lo;  // tail items loaded
    // the full depth fits this class: a recent mode that cannot decide continues in place
    const bool fits_all = c.qcap + tc + nq <= CAP;
    if (q == 0 && !recent && !fits_all) {  // (emit_run listed it by the recent part's need)
      if (lane == 0) s.deep_ids[c.n_loc * 4 + atomicAdd(s.deep_n + 4, 1u)] = (uint32_t)l;  // list 4
      return;
    }
    const uint32_t nseq = shfl_u32(qseq, (int)q);  // (every tail item is older)
    uint4 e[kDeepU];
    tail_chunk<kDeepU>(c, s, l, q, t_lo, tc, lane, nseq, e);
    if (!pend_lds) {
      d.pend[lane].rid = pr0;
      d.pend[lane].dec = pd0;
      d.pend[lane].lq = pl0;
      d.pend[kWave + lane].rid = pr1;
      d.pend[kWave + lane].dec = pd1;
      d.pend[kWave + lane].lq = pl1;
      pend_lds = true;
    }
    const bool hl = lane < c.qcap && Q.r != kEmpty;
    const uint32_t hn = (uint32_t)__popcll(ballot(hl));
    if (hl) {
      d.key[lane] = tlq_key(Q.tl & 0xFFFF, Q.tl >> 16, Q.sq);
      d.rid[lane] = Q.r;
      d.st[lane] = kDeepLive;
    }
    for (uint32_t b = 0;;) {
#pragma unroll
      for (uint32_t u = 0; u < kDeepU; ++u) {
        const uint32_t i = b + u * kWave + lane;
        if (i < tn) {
          d.key[hn + i] = tlq_key(e[u].z & 0xFFFF, e[u].z >> 16, e[u].y);
          d.rid[hn + i] = e[u].x;
          d.st[hn + i] = kDeepLive;
        }
      }
      b += kDeepU * kWave;
      if (b >= tn) break;
      tail_chunk<kDeepU>(c, s, l, q, t_lo + b, tc, lane, nseq, e);  // the next kDeepU * 64 (queues past kDeepU * 64 items)
    }
    uint32_t n = hn + tn;
    if (n == 0 && nq == 0) continue;
    wsync();
    if (nq) {
      const uint32_t seq0 = shfl_u32(qseq, (int)q);
      uint32_t rank0 = 0;
      for (uint32_t b = 0; b < kPend / kWave; ++b) {
        const uint32_t i = b * kWave + lane;
        const bool in = i < npend && (d.pend[i].lq >> 16) == q;
        const uint64_t m = ballot(in);
        if (in) {
          const uint32_t r = rank0 + mbcnt(m), j = n + r;
          d.key[j] = tlq_key(0, d.pend[i].lq & 0xFFFF, seq0 + r);
          d.rid[j] = d.pend[i].rid;
          d.st[j] = kDeepLive;
        }
        rank0 += (uint32_t)__popcll(m);
      }
      n += nq;
      wsync();
    }
#if RSF_DEEP_PROF
    if (lane == 0) s_dprof[32 + min(n / 128u, 31u)] += 1ull;
#endif
    RSF_DEEP_T(8);
    // inserting into a bounded queue with no pick in between keeps its depth smallest keys
    const uint32_t depth = c.qcap + tcap_of(c, q);
    if (n > depth) {
      const uint64_t T = w_select_kth(d, lane, n, depth, kDeepLive, w_range(d, lane, n, kDeepLive));
      for (uint32_t i = lane; i < n; i += kWave)
        if (d.st[i] == kDeepLive && d.key[i] > T) d.st[i] = kDeepDead;
      drops += n - depth;
      wsync();
    }
    // the refill, then the head's own emission with the deep checks
    uint64_t tmin, rres;
    uint32_t tminlen;
    RSF_DEEP_T(9);
    w_take_head(c, d, lane, n, q, Q, tmin, tminlen, rres);
    head_dec_fix(c, s, Q);
    RSF_DEEP_T(10);
    // recent mode: exact only if the head is full and below every sealed key; the sealed
    // prefix stays in the tail, so the tail's bounds include the seal's
    uint64_t sb = ~0ull;  // the kept sealed prefix's key bound (recent mode)
    if (recent) {
      const uint4 se = s.tseal[l * 3 + q];
      sb = ((uint64_t)se.z << 32) | se.y;
      const uint64_t hm = ballot(lane < c.qcap && Q.r != kEmpty);
      const bool full = (uint32_t)__popcll(hm) == c.qcap;
      bool ok = full;
      if (full) {
        const int hl = 63 - __clzll((long long)hm);
        const uint32_t tlh = shfl_u32(Q.tl, hl);
        ok = tlq_key(tlh & 0xFFFF, tlh >> 16, shfl_u32(Q.sq, hl)) < sb;
      }
      bool redo = false;  // one refill call site (another inlined copy spills)
      if (!ok && !fits_all) {
        deep_relist_full(c, s, l, lane, n, d);
        return;
      }
      if (!ok) {  // every item after all: the sealed prefix joins, the refill is redone
#if RSF_DEEP_PROF
        if (lane == 0) s_dprof[30] += 1ull;
#endif
        n = w_load_sealed(c, s, l, q, d, lane, n, t_lo, shfl_u32(qseq, (int)q));
        recent = false;
        t_lo = 0;
        sb = ~0ull;
        redo = true;
      }
      if (redo) {
        for (uint32_t i = lane; i < n; i += kWave)
          if (d.st[i] == kDeepInHead) d.st[i] = kDeepLive;
        wsync();
        w_take_head(c, d, lane, n, q, Q, tmin, tminlen, rres);
        head_dec_fix(c, s, Q);
      }
    }
    if (recent) {
      tmin = sb < tmin ? sb : tmin;
      tminlen = min(tminlen, s.tsum[l * 3 + q].y);  // (a bound over the whole tail: covers the sealed part)
#if RSF_DEEP_PROF
      if (lane == 0) s_dprof[29] += 1ull;
#endif
    }
    const uint32_t used_0 = used_v, nrec_0 = nrec_v;
    bool unsafe = false, dirty = false;
    uint32_t errq = 0;
    if (q == 0)
      q_pick_peers<true, true>(c, Q, lane, np, used_v, nrec_v, off_v, ov, od, errq, dirty, d.row, nullptr, tmin, tminlen,
                               &unsafe);
    else
      q_pick_peers<false, true>(c, Q, lane, np, used_v, nrec_v, off_v, ov, od, errq, dirty, d.row, nullptr, tmin,
                                tminlen, &unsafe);
    RSF_DEEP_T(11);
    if (unsafe && recent) {
      if (!fits_all) {
        deep_relist_full(c, s, l, lane, n, d);
        return;
      }
      // the head cannot decide even now: every item (the sealed prefix joins) for the fallback
      n = w_load_sealed(c, s, l, q, d, lane, n, t_lo, shfl_u32(qseq, (int)q));
      recent = false;
      t_lo = 0;
      sb = ~0ull;
    }
    if (!unsafe) {
      err |= errq;
      q_store(c, s, l, q, lane, Q, true);
      uint32_t nb = 0;
      uint64_t bmin = ~0ull;
      const uint32_t cnt = t_lo + w_store_tail(c, s, l, q, d, lane, n, t_lo, rres, &nb, &bmin);
      if (lane == 0 && tcap_of(c, q)) {
        s.tsum[l * 3 + q] = cnt ? make_uint4(cnt, tminlen, (uint32_t)tmin, (uint32_t)(tmin >> 32)) : kTSumEmpty;
        // sealed: the kept prefix and the group written above the reserve (key bound: the
        // smaller of their bounds); the reserve stays in the recent part
        const uint64_t b = bmin < sb ? bmin : sb;
        s.tseal[l * 3 + q] = t_lo + nb ? make_uint4(t_lo + nb, (uint32_t)b, (uint32_t)(b >> 32), 0u) : kTSumEmpty;
      }
      RSF_DEEP_T(12);
    } else {
      // the head still cannot decide: get_broadcasts over every item, peer by peer
      used_v = used_0;
      nrec_v = nrec_0;
      for (uint32_t i = lane; i < n; i += kWave)
        if (d.st[i] == kDeepInHead) d.st[i] = kDeepLive;
      wsync();
      for (uint32_t j = 0; j < np; ++j) {
        const uint32_t lim = c.limit - shfl_u32(used_v, j), nrec = shfl_u32(nrec_v, j);
        const uint64_t off = shfl_u64(off_v, j);
        uint32_t used = 0, k = 0;
        for (;;) {
          const int32_t free_b = (int32_t)(lim - used - c.overhead);
          if (free_b <= 0) break;
          uint64_t best = ~0ull;
          for (uint32_t i = lane; i < n; i += kWave)
            if (d.st[i] == kDeepLive) {
              const uint64_t x = d.key[i];
              if (key_len(x) <= (uint32_t)free_b && x < best) best = x;
            }
          best = wave_min_u64(best);
          if (best == ~0ull) break;
          uint32_t wi = kEmpty;
          for (uint32_t i = lane; i < n; i += kWave)
            if (d.st[i] == kDeepLive && d.key[i] == best) wi = i;
          const uint64_t owner = ballot(wi != kEmpty);
          wi = shfl_u32(wi, __ffsll((long long)owner) - 1);
          if (lane == 0) {
            d.st[wi] = kDeepPicked;
            if (nrec + k < c.cap_t && off != ~0ull) {
              ov[off + nrec + k] = d.rid[wi];
              if (od) od[off + nrec + k] = q == 0 ? s.rdec[d.rid[wi] & c.rmask] : (q == 1 ? kDecQuery : kDecEvent);
            }
          }
          k++;
          used += c.overhead + key_len(best);
          wsync();
        }
        for (uint32_t i = lane; i < n; i += kWave)  // transmits + 1, or retired at the limit
          if (d.st[i] == kDeepPicked) {
            if ((uint32_t)(d.key[i] >> 48) + 1 >= c.tx_limit) {
              d.st[i] = kDeepDead;
            } else {
              d.key[i] += 1ull << 48;
              d.st[i] = kDeepLive;
            }
          }
        if (nrec + k > c.cap_t) err |= kErrStage;
        used_v += lane == j ? used : 0u;
        nrec_v += lane == j ? k : 0u;
        wsync();
      }
      RSF_DEEP_T(13);
      w_take_head(c, d, lane, n, q, Q, tmin, tminlen, rres);
      head_dec_fix(c, s, Q);
      q_store(c, s, l, q, lane, Q, true);
      uint32_t nb = 0;
      uint64_t bmin = ~0ull;
      const uint32_t cnt = w_store_tail(c, s, l, q, d, lane, n, 0u, rres, &nb, &bmin);
      if (lane == 0 && tcap_of(c, q)) {
        s.tsum[l * 3 + q] = cnt ? make_uint4(cnt, tminlen, (uint32_t)tmin, (uint32_t)(tmin >> 32)) : kTSumEmpty;
        s.tseal[l * 3 + q] = nb ? make_uint4(nb, (uint32_t)bmin, (uint32_t)(bmin >> 32), 0u) : kTSumEmpty;
      }
      RSF_DEEP_T(14);
#if RSF_DEEP_PROF
      if (lane == 0) s_dprof[15] += 1ull;
#endif
    }
    if (CAP == kDeepBig && lane == 0) {  // the full-depth class: items it held (rsf_gossip_deep_full_items)
      unsigned long long* const fi = reinterpret_cast<unsigned long long*>(s.deep_n + kDeepFullItems);
      atomicAdd(fi, (unsigned long long)n);
      atomicMax(fi + 1, (unsigned long long)n);
    }
    for (uint32_t i = lane; i < n; i += kWave) d.st[i] = kDeepDead;  // clean for the next queue
    wsync();
  }
  // the groups' counts and the member's bookkeeping (emit_run's)
  if (oc && (BKT || nrec_v)) *oc = min(nrec_v, c.cap_t);
  if (lane == 0) {
    if (npend) {
      s.p_cnt[l] = 0;
      for (uint32_t q = 0; q < 3; ++q) s.q_next_seq[l * 3 + q] += (pc >> (8 * q)) & 0xFF;
    }
    if (drops) {
      s.q_pruned[l] += drops;
      err |= kErrQueue;
    }
    if (err) s.err[l] |= err;
  }
#if RSF_DEEP_PROF
  if (lane == 0) {
    s_dprof[16] += 1ull;
    s_dprof[17] += (unsigned long long)(__builtin_amdgcn_s_memtime() - pt_start);
  }
#endif
#undef RSF_DEEP_T
}

// the members emit_run deferred to the two smaller classes, one wave per member: list 2 (those
// that fit kDeepTiny items) and list 0 (kDeepSmall), the grid striding over the list so every
// wave reaches its end.  (The middle class and the full depth run one block per member,
// emit_deep_block_kernel below; this kernel still takes any list, as it did before them.)
template <bool BKT, uint32_t CAP>
__global__ void __launch_bounds__(kWave) emit_deep_wave_kernel(GCfg c, GState s, const uint32_t* __restrict__ grp_key,
                                                              const uint32_t* __restrict__ slot,
                                                              uint32_t* __restrict__ cnt_s,
                                                              uint32_t* __restrict__ out_val,
                                                              uint32_t* __restrict__ out_dec, Buckets bk, uint32_t list,
                                                              unsigned long long* __restrict__ total) {
  __shared__ DeepWave<CAP> d;
  const uint32_t lane = threadIdx.x;
#if RSF_DEEP_PROF
  s_dprof[lane] = 0;
#endif
  // list 1 (the full depth) also takes list 4 (the members the smaller classes re-listed),
  // after its own: one launch, one tail
  const uint32_t n_own = s.deep_n[list], n_re = list == 1 ? s.deep_n[4] : 0u, n_list = n_own + n_re;
  if (blockIdx.x == 0 && lane == 0 && n_list) {
    atomicAdd(total, (unsigned long long)n_list);
    // per class (the re-listed members count with the full depth)
    atomicAdd(list == 3 ? total + 1 : total - kDeepClassOff + list, (unsigned long long)n_list);
  }
  for (uint32_t i = lane; i < CAP; i += kWave) d.st[i] = kDeepDead;
  wsync();
  const uint64_t last = c.n_loc * 3 - 1;
  const uint32_t* const ids = list == 1 ? s.deep_ids + last
                                        : s.deep_ids + (list == 2 ? c.n_loc : list == 3 ? c.n_loc * 3 : 0ull);
  const uint32_t* const re = s.deep_ids + c.n_loc * 4;
  const int64_t dir = list == 1 ? -1 : 1;
  auto id_at = [&](uint32_t i) -> uint64_t {
    if (i >= n_list) return ~0ull;
    return i < n_own ? ids[dir * (int64_t)i] : re[i - n_own];
  };
  // software pipeline over the wave's members: the next member's first round trip (deep_pre)
  // and the id after it are read while this member is worked on
  const uint32_t G = gridDim.x;
  uint64_t l = id_at(blockIdx.x);
  DeepPre pre = deep_pre(c, s, l, lane, grp_key, slot);
  uint64_t l_next = id_at(blockIdx.x + G);
  for (uint32_t it = blockIdx.x; it < n_list; it += G) {
    const DeepPre pre_next = deep_pre(c, s, l_next, lane, grp_key, slot);
    const uint64_t l_after = id_at(it + 2 * G);
    if (l < c.n_loc) deep_wave_member<BKT, CAP>(c, s, l, lane, pre, cnt_s, out_val, out_dec, bk, d);  // wave-uniform
    l = l_next;
    pre = pre_next;
    l_next = l_after;
  }
#if RSF_DEEP_PROF
  wsync();
  if (s_dprof[lane]) atomicAdd(&g_deep_prof[lane], s_dprof[lane]);
  if (lane == 0) {  // per class: [70 + c] cycles, [74 + c] members (c: tiny, small, middle, full)
    constexpr uint32_t cls = CAP == kDeepTiny ? 0u : CAP == kDeepSmall ? 1u : CAP == kDeepMid ? 2u : 3u;
    atomicAdd(&g_deep_prof[70 + cls], s_dprof[17]);
    atomicAdd(&g_deep_prof[74 + cls], s_dprof[16]);
  }
#endif
}

// ---- the larger classes: one 256-thread block per member -------------------------------------
// The members whose queues need the middle or the full depth ran one wave each at four waves
// (middle) or one wave (full depth: 117 KB of LDS) per CU, each pass over their 1.2-9k items a
// long one-wave loop.  Here the block's four waves share the streaming work -- the tail load,
// the key range, the radix selects, the head gather and the tail store -- while the head's
// register work (q_load, the picks, q_store and the rare per-peer fallback) stays with wave 0.
// The same decisions as deep_wave_member (recent mode, re-listing); the tail's slot order may
// differ from the one-wave path's (it is unordered: nothing reads its order).
constexpr uint32_t kDeepBlkWaves = 4, kDeepBlkThreads = kDeepBlkWaves * kWave;
struct DeepBlk {
  uint64_t r64[kDeepBlkWaves][4];  // per-wave partials of the block reductions
  uint32_t r32[kDeepBlkWaves][4];
  uint64_t hk[kDeepBlkWaves][kWave];  // the head gather: each wave's items, in its range's order
  uint32_t hr[kDeepBlkWaves][kWave];
  uint32_t u[8];  // wave 0's broadcasts: [0..2] select digit / need / bucket count, [4] hn, [5] unsafe, [6] recent ok
};
__device__ __forceinline__ uint64_t b_min_u64(uint64_t v, DeepBlk& x, uint32_t tid) {
  v = wave_min_u64(v);
  if ((tid & (kWave - 1)) == 0) x.r64[tid / kWave][3] = v;
  __syncthreads();
  uint64_t m = x.r64[0][3];
#pragma unroll
  for (uint32_t w = 1; w < kDeepBlkWaves; ++w) m = x.r64[w][3] < m ? x.r64[w][3] : m;
  __syncthreads();
  return m;
}
// items [lo, hi) of wave w's contiguous range (a multiple of 64 per wave): deterministic
// compaction orders without a block scan per 64 items
__device__ __forceinline__ void b_wave_range(uint32_t n, uint32_t w, uint32_t& lo, uint32_t& hi) {
  const uint32_t per = ((n + kDeepBlkThreads - 1) / kDeepBlkThreads) * kWave;
  lo = min(n, w * per);
  hi = min(n, lo + per);
}
template <uint32_t CAP>
__device__ WRange b_range(const DeepWave<CAP>& d, DeepBlk& x, uint32_t tid, uint32_t n, uint8_t state) {
  uint32_t cnt = 0, c0 = 0;
  uint64_t lo = ~0ull, hi = 0, an = ~0ull, orr = 0;
  for (uint32_t b = 0; b < n; b += kDeepU * kDeepBlkThreads) {
    uint64_t xk[kDeepU];
    uint32_t sv[kDeepU];
#pragma unroll
    for (uint32_t u = 0; u < kDeepU; ++u) {
      const uint32_t i = b + u * kDeepBlkThreads + tid, ii = i < n ? i : 0u;
      sv[u] = d.st[ii];
      xk[u] = d.key[ii];
    }
#pragma unroll
    for (uint32_t u = 0; u < kDeepU; ++u)
      if (b + u * kDeepBlkThreads + tid < n && sv[u] == state) {
        cnt++;
        c0 += (xk[u] >> 48) == 0 ? 1u : 0u;
        lo = xk[u] < lo ? xk[u] : lo;
        hi = xk[u] > hi ? xk[u] : hi;
        an &= xk[u];
        orr |= xk[u];
      }
  }
  const uint32_t w = tid / kWave;
  cnt = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum_u32(cnt), 63);
  c0 = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum_u32(c0), 63);
  lo = wave_min_u64(lo);
  hi = wave_max_u64(hi);
  an = wave_and_u64(an);
  orr = wave_or_u64(orr);
  if ((tid & (kWave - 1)) == 0) {
    x.r64[w][0] = lo;
    x.r64[w][1] = hi;
    x.r64[w][2] = an;
    x.r64[w][3] = orr;
    x.r32[w][0] = cnt;
    x.r32[w][1] = c0;
  }
  __syncthreads();
  WRange r{0u, 0u, ~0ull, 0ull, ~0ull, 0ull};
#pragma unroll
  for (uint32_t v = 0; v < kDeepBlkWaves; ++v) {
    r.cnt += x.r32[v][0];
    r.cnt_t0 += x.r32[v][1];
    r.lo = x.r64[v][0] < r.lo ? x.r64[v][0] : r.lo;
    r.hi = x.r64[v][1] > r.hi ? x.r64[v][1] : r.hi;
    r.an &= x.r64[v][2];
    r.orr |= x.r64[v][3];
  }
  __syncthreads();
  return r;
}
// w_select_kth's LDS radix select, the key passes shared by the block's waves
template <uint32_t CAP>
__device__ uint64_t b_select_kth(DeepWave<CAP>& d, DeepBlk& x, uint32_t tid, uint32_t n, uint32_t k, uint8_t state,
                                 const WRange& rg) {
  if (k <= 1 || rg.lo == rg.hi) return rg.lo;
  const uint32_t lane = tid & (kWave - 1), w = tid / kWave;
  const uint64_t var = rg.an ^ rg.orr;
  uint64_t prefix = 0, mask = 0;
  uint32_t need = k;
  const bool t0 = rg.cnt_t0 >= k;
  if (t0) mask = 0xFFFFull << 48;
  for (int shift = 56; shift >= 0; shift -= 8) {
    const uint64_t bm = 0xFFull << shift;
    if (t0 && shift >= 48) continue;
    if (!(var & bm)) {
      prefix |= rg.an & bm;
      mask |= bm;
      continue;
    }
    d.hist[tid] = 0;  // (256 threads, 256 bins)
    __syncthreads();
    for (uint32_t b = 0; b < n; b += kDeepU * kDeepBlkThreads) {
      uint64_t xk[kDeepU];
      uint32_t sv[kDeepU];
#pragma unroll
      for (uint32_t u = 0; u < kDeepU; ++u) {
        const uint32_t i = b + u * kDeepBlkThreads + tid, ii = i < n ? i : 0u;
        sv[u] = d.st[ii];
        xk[u] = d.key[ii];
      }
#pragma unroll
      for (uint32_t u = 0; u < kDeepU; ++u) {
        const bool in = b + u * kDeepBlkThreads + tid < n && sv[u] == state && (xk[u] & mask) == prefix;
        const uint32_t dg = (uint32_t)(xk[u] >> shift) & 0xFF;
        const uint64_t am = ballot(in);
        if (!am) continue;
        const int f = __ffsll((long long)am) - 1;
        const uint32_t d0 = shfl_u32(dg, f);
        const uint64_t same = ballot(in && dg == d0);
        if (lane == (uint32_t)f) atomicAdd(&d.hist[d0], (uint32_t)__popcll(same));
        else if (in && dg != d0) atomicAdd(&d.hist[dg], 1u);
      }
    }
    __syncthreads();
    if (w == 0) {  // the digit holding the need-th key: running counts, four bins per lane
      const uint32_t h0 = d.hist[4 * lane], h1 = d.hist[4 * lane + 1], h2 = d.hist[4 * lane + 2], h3 = d.hist[4 * lane + 3];
      const uint32_t sum = h0 + h1 + h2 + h3, incl = wave_inclusive_sum_u32(sum), excl = incl - sum;
      if (excl < need && need <= incl) {
        uint32_t b = 0, acc = excl, hb = h0;
        if (acc + h0 < need) {
          acc += h0;
          b = 1;
          hb = h1;
          if (acc + h1 < need) {
            acc += h1;
            b = 2;
            hb = h2;
            if (acc + h2 < need) {
              acc += h2;
              b = 3;
              hb = h3;
            }
          }
        }
        x.u[0] = 4 * lane + b;
        x.u[1] = need - acc;
        x.u[2] = hb;
      }
    }
    __syncthreads();
    const uint32_t digit = x.u[0], cnt = x.u[2];
    need = x.u[1];
    prefix |= (uint64_t)digit << shift;
    mask |= bm;
    if (cnt == 1 && shift > 0) {  // one key left in the bucket: it is the k-th
      uint64_t best = ~0ull;
      for (uint32_t i = tid; i < n; i += kDeepBlkThreads)
        if (d.st[i] == state && (d.key[i] & mask) == prefix) best = d.key[i];
      return b_min_u64(best, x, tid);
    }
  }
  return prefix;
}
// w_take_head with the block: the range, the two selects and the gather shared; wave 0 ranks
// the head's keys and permutes them into its register head Q.  tmin / tminlen / rres are
// block-uniform.
template <uint32_t CAP>
__device__ __forceinline__ void b_take_head(const GCfg& c, DeepWave<CAP>& d, DeepBlk& x, uint32_t tid, uint32_t n,
                                            uint32_t q, QRegs& Q, uint64_t& tmin, uint32_t& tminlen, uint64_t& rres) {
  const uint32_t lane = tid & (kWave - 1), w = tid / kWave;
  const WRange rg = b_range(d, x, tid, n, kDeepLive);
  uint64_t T = ~0ull;
  rres = ~0ull;
#pragma unroll 1
  for (uint32_t j = 0; j < 2; ++j) {
    const uint32_t k = j ? c.qcap + kDeepReserve : c.qcap;
    if (rg.cnt <= k) break;
    const uint64_t v = b_select_kth(d, x, tid, n, k, kDeepLive, rg);
    if (j) rres = v;
    else T = v;
  }
  // the head's items (at most qcap <= 64: keys are distinct) gathered per wave range
  uint32_t lo, hi, base = 0;
  b_wave_range(n, w, lo, hi);
  uint64_t km = ~0ull;
  uint32_t lm = ~0u;
  for (uint32_t b = lo; b < hi; b += kWave) {
    const uint32_t i = b + lane;
    const bool v = i < hi && d.st[i] == kDeepLive;
    const uint64_t k = v ? d.key[i] : ~0ull;
    const bool sel = v && k <= T;
    const uint64_t m = ballot(sel);
    if (sel) {
      const uint32_t pos = base + mbcnt(m);
      x.hk[w][pos] = k;
      x.hr[w][pos] = d.rid[i];
      d.st[i] = kDeepInHead;
    } else if (v) {  // stays in the tail
      km = k < km ? k : km;
      lm = min(lm, key_len(k));
    }
    base += (uint32_t)__popcll(m);
  }
  if (lane == 0) x.r32[w][2] = base;
  tmin = b_min_u64(km, x, tid);  // (its barriers publish the gather)
  tminlen = (uint32_t)b_min_u64(lm, x, tid);
  if (w == 0) {
    uint32_t hn = 0, src_w = 0, src_i = lane;
#pragma unroll
    for (uint32_t v = 0; v < kDeepBlkWaves; ++v) {
      const uint32_t cv = x.r32[v][2];
      if (lane >= hn && lane < hn + cv) {
        src_w = v;
        src_i = lane - hn;
      }
      hn += cv;
    }
    const bool h = lane < hn;
    const uint64_t mk = h ? x.hk[src_w][src_i] : ~0ull;
    const uint32_t hr = h ? x.hr[src_w][src_i] : kEmpty;
    d.hkey[lane] = mk;
    wsync();
    uint32_t rank = 0;
#pragma unroll 8
    for (uint32_t j = 0; j < hn; ++j) rank += d.hkey[j] < mk ? 1u : 0u;
    const uint64_t hm = ballot(h);
    const uint32_t dest = h ? rank : hn + mbcnt(~hm);
    const int addr = (int)(dest * 4);
    const uint32_t sq = h ? key_seq(mk) : 0u, tl = h ? key_tl(mk) : 0u,
                   dc = q == 0 ? kDecLookup : (q == 1 ? kDecQuery : kDecEvent);
    Q.r = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)hr);
    Q.sq = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)sq);
    Q.tl = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)tl);
    Q.dec = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)dc);
    wsync();
  }
}
// w_store_tail with the block, at tail[t_lo ...]: per wave range, a count pass, one block scan, a
// write pass -- the sealed group (keys > R) first, the reserve after it.  Block-uniform result.
template <uint32_t CAP>
__device__ __forceinline__ uint32_t b_store_tail(const GCfg& c, const GState& s, uint64_t l, uint32_t q,
                                                 DeepWave<CAP>& d, DeepBlk& x, uint32_t tid, uint32_t n, uint32_t t_lo,
                                                 uint64_t R, uint32_t* nb, uint64_t* bmin) {
  const uint32_t lane = tid & (kWave - 1), w = tid / kWave;
  uint4* const t = q && tcap_of(c, q) ? tail16(s, q) + l * tstride_of(c, q) + t_lo : nullptr;
  uint64_t* const t8 = q == 0 && c.tcap0 ? tail8(s, c, l) + t_lo : nullptr;
  uint32_t lo, hi;
  b_wave_range(n, w, lo, hi);
  uint32_t ns = 0, nr = 0;
  for (uint32_t b = lo; b < hi; b += kWave) {
    const uint32_t i = b + lane;
    const bool live = i < hi && d.st[i] == kDeepLive;
    const bool sealed = live && d.key[i] > R;
    ns += (uint32_t)__popcll(ballot(sealed));
    nr += (uint32_t)__popcll(ballot(live && !sealed));
  }
  if (lane == 0) {
    x.r32[w][0] = ns;
    x.r32[w][1] = nr;
  }
  __syncthreads();
  uint32_t ns_all = 0, so = 0, ro = 0, total = 0;
#pragma unroll
  for (uint32_t v = 0; v < kDeepBlkWaves; ++v) {
    ns_all += x.r32[v][0];
    total += x.r32[v][0] + x.r32[v][1];
    so += v < w ? x.r32[v][0] : 0u;
    ro += v < w ? x.r32[v][1] : 0u;
  }
  __syncthreads();
  uint32_t bs = so, br = ns_all + ro;
  uint64_t bm = ~0ull;
  for (uint32_t b = lo; b < hi; b += kWave) {
    const uint32_t i = b + lane;
    const uint64_t k = i < hi ? d.key[i] : 0ull;
    const bool live = i < hi && d.st[i] == kDeepLive;
    const bool sealed = live && k > R, res = live && k <= R;
    const uint64_t ms = ballot(sealed), mr = ballot(res);
    if (live) {
      const uint32_t at = sealed ? bs + mbcnt(ms) : br + mbcnt(mr);
      if (q == 0) t8[at] = tail_pack(c, d.rid[i], key_seq(k), key_tl(k));
      else t[at] = make_uint4(d.rid[i], key_seq(k), key_tl(k), q == 1 ? kDecQuery : kDecEvent);
    }
    if (sealed) bm = k < bm ? k : bm;
    bs += (uint32_t)__popcll(ms);
    br += (uint32_t)__popcll(mr);
  }
  *nb = ns_all;
  *bmin = b_min_u64(bm, x, tid);
  return total;
}

// tail[t_lo, t_hi) of (l, q) into LDS items [at, ...) (live), every thread kDeepU items in flight
template <uint32_t CAP>
__device__ __forceinline__ void b_tail_load(const GCfg& c, const GState& s, uint64_t l, uint32_t q, DeepWave<CAP>& d,
                                            uint32_t tid, uint32_t t_lo, uint32_t t_hi, uint32_t at, uint32_t nseq) {
  const uint32_t tn = t_hi - t_lo;
  for (uint32_t b = 0; b < tn; b += kDeepU * kDeepBlkThreads) {
    uint4 e[kDeepU];
    if (q == 0) {
      const uint64_t* const t8 = tail8(s, c, l) + t_lo;
      uint64_t v[kDeepU];
#pragma unroll
      for (uint32_t u = 0; u < kDeepU; ++u) {
        const uint32_t i = b + u * kDeepBlkThreads + tid;
        v[u] = i < tn ? t8[i] : 0ull;
      }
#pragma unroll
      for (uint32_t u = 0; u < kDeepU; ++u) e[u] = tail_unpack(c, v[u], nseq);
    } else {
      const uint4* const t16 = tail16(s, q) + l * tstride_of(c, q) + t_lo;
#pragma unroll
      for (uint32_t u = 0; u < kDeepU; ++u) {
        const uint32_t i = b + u * kDeepBlkThreads + tid;
        e[u] = i < tn ? t16[i] : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kDeepU; ++u) {
      const uint32_t i = b + u * kDeepBlkThreads + tid;
      if (i < tn) {
        d.key[at + i] = tlq_key(e[u].z & 0xFFFF, e[u].z >> 16, e[u].y);
        d.rid[at + i] = e[u].x;
        d.st[at + i] = kDeepLive;
      }
    }
  }
}
// the sealed prefix tail[0, sm) into LDS after the n items there (w_load_sealed with the block);
// returns the new item count
template <uint32_t CAP>
__device__ __forceinline__ uint32_t b_load_sealed(const GCfg& c, const GState& s, uint64_t l, uint32_t q,
                                                  DeepWave<CAP>& d, uint32_t tid, uint32_t n, uint32_t sm,
                                                  uint32_t nseq) {
  for (uint32_t i = tid; i < n; i += kDeepBlkThreads)
    if (d.st[i] == kDeepInHead) d.st[i] = kDeepLive;
  b_tail_load(c, s, l, q, d, tid, 0u, sm, n, nseq);
  __syncthreads();
  return n + sm;
}
// recent mode could not decide and the class cannot hold the whole queue: nothing of the member
// is stored yet; the LDS items are cleared and the member re-listed for the full depth (list 4)
template <uint32_t CAP>
__device__ __forceinline__ void b_relist_full(const GCfg& c, const GState& s, uint64_t l, uint32_t tid, uint32_t n,
                                              DeepWave<CAP>& d) {
  for (uint32_t i = tid; i < n; i += kDeepBlkThreads) d.st[i] = kDeepDead;
  if (tid == 0) s.deep_ids[c.n_loc * 4 + atomicAdd(s.deep_n + 4, 1u)] = (uint32_t)l;
  __syncthreads();
}

template <bool BKT, uint32_t CAP>
__device__ __forceinline__ void deep_block_member(const GCfg& c, const GState& s, uint64_t l, uint32_t tid,
                                                  const DeepPre& pre, uint32_t* __restrict__ cnt_s,
                                                  uint32_t* __restrict__ out_val, uint32_t* __restrict__ out_dec,
                                                  const Buckets& bk, DeepWave<CAP>& d, DeepBlk& x) {
  const uint32_t lane = tid & (kWave - 1), w = tid / kWave;
  const uint32_t pc = pre.pc, npend = pend_total(pc);
  const uint32_t gk = pre.gk, gs = pre.gs;
  const uint32_t np = (uint32_t)__popcll(ballot(gk != kSentinel));
  uint64_t off_v = ~0ull;
  uint32_t* oc = nullptr;
  if (lane < np) {
    if (BKT) {
      const uint32_t wd = gs >> kBktWShift, idx = gs & kBktIdxMask;
      if (idx < bk.gcap) {
        off_v = (uint64_t)wd * bk.stride_u32 + bk.vals_off + (uint64_t)idx * c.cap_t;
        oc = bk.send + (uint64_t)wd * bk.stride_u32 + bk.cnt_off + idx;
      }
    } else {
      off_v = (uint64_t)gs * c.cap_t;
      oc = cnt_s + gs;
    }
  }
  const uint32_t qinfo = pre.qinfo, qseq = pre.qseq;
  static_assert(kPend <= kDeepBlkThreads, "one pending entry per thread");
  if (tid < npend) d.pend[tid] = s.p_ent[l * kPend + tid];
  uint32_t* const ov = BKT ? bk.send : out_val;
  uint32_t* const od = BKT ? bk.send + (bk.decs_off - bk.vals_off) : out_dec;
  uint32_t used_v = 0, nrec_v = 0, err = 0, drops = 0;  // (wave 0's)
  __syncthreads();
  for (uint32_t q = 0; q < 3; ++q) {
    const uint32_t nq = (pc >> (8 * q)) & 0xFF;
    const uint32_t qi = shfl_u32(qinfo, (int)q);
    if (qi == 0 && nq == 0) continue;  // (block-uniform: every wave read the same first round trip)
    const uint32_t tc = qi >> 1, nseq = shfl_u32(qseq, (int)q);
    // RECENT mode as deep_wave_member's: only the intent queue in use and a sealed tail prefix
    const uint32_t sm = shfl_u32(pre.sm, (int)q);
    const bool others_empty = q == 0 && shfl_u32(qinfo, 1) == 0 && shfl_u32(qinfo, 2) == 0 && ((pc >> 8) & 0xFFFF) == 0;
    bool recent = others_empty && sm > 0 && sm <= tc && tc + nq <= tcap_of(c, q);
    uint32_t t_lo = recent ? sm : 0u;
    const bool fits_all = c.qcap + tc + nq <= CAP;
    if (!recent && !fits_all) {
      if (q == 0 && CAP < kDeepBig) {  // (emit_run listed it by the recent part's need)
        if (tid == 0) s.deep_ids[c.n_loc * 4 + atomicAdd(s.deep_n + 4, 1u)] = (uint32_t)l;  // list 4
        __syncthreads();
        return;
      }
      if (tid == 0) atomicOr(s.err + l, (uint32_t)RSF_E_DEEP_INVARIANT);  // (the tail's capacity is below it)
      continue;
    }
    QRegs Q{kEmpty, 0, 0};
    if (w == 0) {
      q_load(c, s, l, q, lane, Q);
      const bool hl = lane < c.qcap && Q.r != kEmpty;
      const uint64_t hm = ballot(hl);
      if (hl) {
        d.key[lane] = tlq_key(Q.tl & 0xFFFF, Q.tl >> 16, Q.sq);
        d.rid[lane] = Q.r;
        d.st[lane] = kDeepLive;
      }
      if (lane == 0) x.u[4] = (uint32_t)__popcll(hm);
    }
    __syncthreads();
    const uint32_t hn = x.u[4];
    b_tail_load(c, s, l, q, d, tid, t_lo, tc, hn, nseq);
    const uint32_t tn = tc - t_lo;
    uint32_t n = hn + tn;
    if (n == 0 && nq == 0) continue;
    if (nq && w == 0) {  // the pending re-queues after them, in list order (transmits 0, the next seqs)
      uint32_t rank0 = 0;
      for (uint32_t b = 0; b < kPend / kWave; ++b) {
        const uint32_t i = b * kWave + lane;
        const bool in = i < npend && (d.pend[i].lq >> 16) == q;
        const uint64_t m = ballot(in);
        if (in) {
          const uint32_t r = rank0 + mbcnt(m), j = n + r;
          d.key[j] = tlq_key(0, d.pend[i].lq & 0xFFFF, nseq + r);
          d.rid[j] = d.pend[i].rid;
          d.st[j] = kDeepLive;
        }
        rank0 += (uint32_t)__popcll(m);
      }
    }
    n += nq;
    __syncthreads();
    // the bounded prune to the depth (inserts with no pick in between keep the smallest keys)
    const uint32_t depth = c.qcap + tcap_of(c, q);
    if (n > depth) {
      const uint64_t T = b_select_kth(d, x, tid, n, depth, kDeepLive, b_range(d, x, tid, n, kDeepLive));
      for (uint32_t i = tid; i < n; i += kDeepBlkThreads)
        if (d.st[i] == kDeepLive && d.key[i] > T) d.st[i] = kDeepDead;
      drops += n - depth;
      __syncthreads();
    }
    uint64_t tmin, rres;
    uint32_t tminlen;
    b_take_head(c, d, x, tid, n, q, Q, tmin, tminlen, rres);
    // recent mode: exact only if the head is full and below every sealed key; the sealed prefix
    // stays in the tail, so the tail's bounds include the seal's
    uint64_t sb = ~0ull;
    if (recent) {
      const uint4 se = s.tseal[l * 3 + q];
      sb = ((uint64_t)se.z << 32) | se.y;
      if (w == 0) {
        const uint64_t hm = ballot(lane < c.qcap && Q.r != kEmpty);
        bool ok = (uint32_t)__popcll(hm) == c.qcap;
        if (ok) {
          const int hl = 63 - __clzll((long long)hm);
          const uint32_t tlh = shfl_u32(Q.tl, hl);
          ok = tlq_key(tlh & 0xFFFF, tlh >> 16, shfl_u32(Q.sq, hl)) < sb;
        }
        if (lane == 0) x.u[6] = ok ? 1u : 0u;
      }
      __syncthreads();
      if (!x.u[6]) {
        if (!fits_all) {
          b_relist_full(c, s, l, tid, n, d);
          return;
        }
        // every item after all: the sealed prefix joins, the refill is redone
        n = b_load_sealed(c, s, l, q, d, tid, n, t_lo, nseq);
        recent = false;
        t_lo = 0;
        sb = ~0ull;
        b_take_head(c, d, x, tid, n, q, Q, tmin, tminlen, rres);
      }
    }
    if (recent) {
      tmin = sb < tmin ? sb : tmin;
      tminlen = min(tminlen, s.tsum[l * 3 + q].y);  // (a bound over the whole tail: covers the sealed part)
    }
    const uint32_t used_0 = used_v, nrec_0 = nrec_v;
    uint32_t errq = 0;
    if (w == 0) {
      head_dec_fix(c, s, Q);
      bool unsafe = false, dirty = false;
      if (q == 0)
        q_pick_peers<true, true>(c, Q, lane, np, used_v, nrec_v, off_v, ov, od, errq, dirty, d.row, nullptr, tmin,
                                 tminlen, &unsafe);
      else
        q_pick_peers<false, true>(c, Q, lane, np, used_v, nrec_v, off_v, ov, od, errq, dirty, d.row, nullptr, tmin,
                                  tminlen, &unsafe);
      if (lane == 0) x.u[5] = unsafe ? 1u : 0u;
    }
    __syncthreads();
    const bool unsafe = x.u[5] != 0;
    if (unsafe && recent) {
      if (!fits_all) {
        b_relist_full(c, s, l, tid, n, d);
        return;
      }
      // the head cannot decide even now: every item (the sealed prefix joins) for the fallback
      n = b_load_sealed(c, s, l, q, d, tid, n, t_lo, nseq);
      recent = false;
      t_lo = 0;
      sb = ~0ull;
    }
    if (unsafe) {
      // the head still cannot decide: get_broadcasts over every item, peer by peer (wave 0; rare)
      if (w == 0) {
        used_v = used_0;
        nrec_v = nrec_0;
        for (uint32_t i = lane; i < n; i += kWave)
          if (d.st[i] == kDeepInHead) d.st[i] = kDeepLive;
        wsync();
        for (uint32_t j = 0; j < np; ++j) {
          const uint32_t lim = c.limit - shfl_u32(used_v, j), nrec = shfl_u32(nrec_v, j);
          const uint64_t off = shfl_u64(off_v, j);
          uint32_t used = 0, k = 0;
          for (;;) {
            const int32_t free_b = (int32_t)(lim - used - c.overhead);
            if (free_b <= 0) break;
            uint64_t best = ~0ull;
            for (uint32_t i = lane; i < n; i += kWave)
              if (d.st[i] == kDeepLive) {
                const uint64_t kx = d.key[i];
                if (key_len(kx) <= (uint32_t)free_b && kx < best) best = kx;
              }
            best = wave_min_u64(best);
            if (best == ~0ull) break;
            uint32_t wi = kEmpty;
            for (uint32_t i = lane; i < n; i += kWave)
              if (d.st[i] == kDeepLive && d.key[i] == best) wi = i;
            const uint64_t owner = ballot(wi != kEmpty);
            wi = shfl_u32(wi, __ffsll((long long)owner) - 1);
            if (lane == 0) {
              d.st[wi] = kDeepPicked;
              if (nrec + k < c.cap_t && off != ~0ull) {
                ov[off + nrec + k] = d.rid[wi];
                if (od) od[off + nrec + k] = q == 0 ? s.rdec[d.rid[wi] & c.rmask] : (q == 1 ? kDecQuery : kDecEvent);
              }
            }
            k++;
            used += c.overhead + key_len(best);
            wsync();
          }
          for (uint32_t i = lane; i < n; i += kWave)  // transmits + 1, or retired at the limit
            if (d.st[i] == kDeepPicked) {
              if ((uint32_t)(d.key[i] >> 48) + 1 >= c.tx_limit) {
                d.st[i] = kDeepDead;
              } else {
                d.key[i] += 1ull << 48;
                d.st[i] = kDeepLive;
              }
            }
          if (nrec + k > c.cap_t) err |= kErrStage;
          used_v += lane == j ? used : 0u;
          nrec_v += lane == j ? k : 0u;
          wsync();
        }
      }
      __syncthreads();
      b_take_head(c, d, x, tid, n, q, Q, tmin, tminlen, rres);
      if (w == 0) head_dec_fix(c, s, Q);
    } else if (w == 0) {
      err |= errq;
    }
    if (w == 0) q_store(c, s, l, q, lane, Q, true);
    uint32_t nb = 0;
    uint64_t bmin = ~0ull;
    const uint32_t cnt = t_lo + b_store_tail(c, s, l, q, d, x, tid, n, t_lo, rres, &nb, &bmin);
    if (tid == 0) {
      if (tcap_of(c, q)) {
        s.tsum[l * 3 + q] = cnt ? make_uint4(cnt, tminlen, (uint32_t)tmin, (uint32_t)(tmin >> 32)) : kTSumEmpty;
        // sealed: the kept prefix (recent mode) and the group written above the reserve
        const uint64_t b = bmin < sb ? bmin : sb;
        s.tseal[l * 3 + q] = t_lo + nb ? make_uint4(t_lo + nb, (uint32_t)b, (uint32_t)(b >> 32), 0u) : kTSumEmpty;
      }
      if (CAP == kDeepBig) {  // the items the full-depth class held (rsf_gossip_deep_full_items)
        unsigned long long* const fi = reinterpret_cast<unsigned long long*>(s.deep_n + kDeepFullItems);
        atomicAdd(fi, (unsigned long long)n);
        atomicMax(fi + 1, (unsigned long long)n);
      }
    }
    for (uint32_t i = tid; i < n; i += kDeepBlkThreads) d.st[i] = kDeepDead;  // clean for the next queue
    __syncthreads();
  }
  if (w == 0) {  // the groups' counts and the member's bookkeeping (emit_run's)
    if (oc && (BKT || nrec_v)) *oc = min(nrec_v, c.cap_t);
    if (lane == 0) {
      if (npend) {
        s.p_cnt[l] = 0;
        for (uint32_t q = 0; q < 3; ++q) s.q_next_seq[l * 3 + q] += (pc >> (8 * q)) & 0xFF;
      }
      if (drops) {
        s.q_pruned[l] += drops;
        err |= kErrQueue;
      }
      if (err) s.err[l] |= err;
    }
  }
  __syncthreads();
}

// emit_deep_wave_kernel's lists with one block per member: list 2 / 0 / 3 (the tiny / small /
// middle class), or list 1 (the full depth, from the back of s.deep_ids) followed by list 4 (the
// members the smaller classes re-listed); the grid strides over them
template <bool BKT, uint32_t CAP>
__global__ void __launch_bounds__(kDeepBlkThreads) emit_deep_block_kernel(
    GCfg c, GState s, const uint32_t* __restrict__ grp_key, const uint32_t* __restrict__ slot,
    uint32_t* __restrict__ cnt_s, uint32_t* __restrict__ out_val, uint32_t* __restrict__ out_dec, Buckets bk,
    uint32_t list, unsigned long long* __restrict__ total) {
  __shared__ DeepWave<CAP> d;
  __shared__ DeepBlk x;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1);
  const uint32_t n_own = s.deep_n[list], n_re = list == 1 ? s.deep_n[4] : 0u, n_list = n_own + n_re;
  if (blockIdx.x == 0 && tid == 0 && n_list) {
    atomicAdd(total, (unsigned long long)n_list);
    atomicAdd(list == 3 ? total + 1 : total - kDeepClassOff + list, (unsigned long long)n_list);  // per class
  }
  for (uint32_t i = tid; i < CAP; i += kDeepBlkThreads) d.st[i] = kDeepDead;
  __syncthreads();
  const uint32_t* const ids = list == 1 ? s.deep_ids + (c.n_loc * 3 - 1)
                                        : s.deep_ids + (list == 2 ? c.n_loc : list == 3 ? c.n_loc * 3 : 0ull);
  const int64_t dir = list == 1 ? -1 : 1;
  const uint32_t* const re = s.deep_ids + c.n_loc * 4;
  for (uint32_t it = blockIdx.x; it < n_list; it += gridDim.x) {
    const uint64_t l = it < n_own ? ids[dir * (int64_t)it] : re[it - n_own];
    if (l >= c.n_loc) continue;  // (block-uniform)
    const DeepPre pre = deep_pre(c, s, l, lane, grp_key, slot);  // (every wave reads the same)
    deep_block_member<BKT, CAP>(c, s, l, tid, pre, cnt_s, out_val, out_dec, bk, d, x);
  }
}

// ---- the QueueChecker's prune (check_stream_kernel) --------------------------------------
// One block per listed (member, queue).  Pass 1 streams head and tail once and keeps only the
// 8-B keys in LDS (live head keys first, then the tail's in index order); one select over the
// LDS keys finds the max-th key; pass 2 streams the tail again and compacts it in place.  Two
// blocks per CU (the keys of a full queue are 70 KB).
#ifndef RSF_CHK_U1
#define RSF_CHK_U1 32  // check_stream_kernel's pass 1: 16-B loads in flight per thread (16: 99.2 ms per 1M-member tick, 32: 97.3)
#endif
#ifndef RSF_CHK_U2
#define RSF_CHK_U2 16  // its pass 2 (the compaction): items per thread per batch
#endif
constexpr uint32_t kChkU2 = RSF_CHK_U2;
struct CheckLds {
  uint32_t hist[3][256];
  uint64_t w64[kDeepWaves], w64b[kDeepWaves];
  uint32_t wcnt[kChkU2][kDeepWaves];
  uint32_t sel_digit[3], sel_need[3], nb, hn;
};

// block-uniform minimum (every thread calls)
__device__ __forceinline__ uint64_t blk_min_u64(uint64_t v, CheckLds& d) {
  v = wave_min_u64(v);
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) d.w64[threadIdx.x / kWave] = v;
  __syncthreads();
  uint64_t m = d.w64[0];
#pragma unroll
  for (uint32_t w = 1; w < kDeepWaves; ++w) m = d.w64[w] < m ? d.w64[w] : m;
  return m;
}

// the ks[j]-th smallest of the n LDS keys for each active j (1 <= ks[j] <= n), by a radix
// select over the bytes where the keys differ (from the caller's AND / OR), the three selects
// sharing each pass over the keys.  A digit's lanes that agree with the wave's first active
// lane are counted by that lane alone (a saturated queue's keys share their transmit byte: one
// LDS address would take thousands of atomics).
// pre48: d.hist[0] already holds every key's byte 6 (bits 48..55; the caller's pass 1 counted
// them, valid when byte 7 is the same in every key), so that byte takes no pass here
__device__ void lds_select3(const uint64_t* __restrict__ keys, uint32_t n, CheckLds& d, const uint32_t ks[3],
                            const bool act[3], uint64_t an, uint64_t orr, bool pre48, uint64_t out[3]) {
  constexpr uint32_t U = 4;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const uint64_t var = an ^ orr;
  uint64_t prefix[3] = {0, 0, 0}, mask = 0;
  uint32_t need[3] = {ks[0], ks[1], ks[2]};
  for (int shift = 56; shift >= 0; shift -= 8) {
    const uint64_t bm = 0xFFull << shift;
    if (!(var & bm)) {
#pragma unroll
      for (int j = 0; j < 3; ++j) prefix[j] |= an & bm;
      mask |= bm;
      continue;
    }
    // selects whose prefixes agree share one histogram (always at the first varying byte)
    const uint32_t al1 = act[1] && !(act[0] && prefix[1] == prefix[0]) ? 1u : 0u;
    const uint32_t al2 = act[2] && !(act[0] && prefix[2] == prefix[0]) ? (act[1] && prefix[2] == prefix[1] ? al1 : 2u) : 0u;
    const bool own[3] = {act[0], al1 == 1, al2 == 2};
    const bool counted = pre48 && shift == 48;  // (all three prefixes agree there: al1 = al2 = 0)
    __syncthreads();
    for (uint32_t i = counted ? 3 * 256 : tid; i < 3 * 256; i += kDeepThreads) (&d.hist[0][0])[i] = 0;
    __syncthreads();
    for (uint32_t i0 = 0; i0 < (counted ? 0u : n); i0 += U * kDeepThreads) {
      uint64_t x[U];
      bool v[U];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * kDeepThreads + tid;
        v[u] = i < n;
        x[u] = v[u] ? keys[i] : 0ull;
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t dg = (uint32_t)(x[u] >> shift) & 0xFF;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (!own[j]) continue;
          const bool in = v[u] && (x[u] & mask) == prefix[j];
          const uint64_t am = ballot(in);
          if (!am) continue;
          const int f = __ffsll((long long)am) - 1;
          const uint32_t d0 = shfl_u32(dg, f);
          const uint64_t same = ballot(in && dg == d0);
          if (lane == (uint32_t)f) atomicAdd(&d.hist[j][d0], (uint32_t)__popcll(same));
          else if (in && dg != d0) atomicAdd(&d.hist[j][dg], 1u);
        }
      }
    }
    __syncthreads();
    const bool aw = w == 0 ? act[0] : w == 1 ? act[1] : w == 2 ? act[2] : false;
    if (aw) {  // wave j picks select j's digit: running counts, four bins per lane
      const uint32_t* h = d.hist[w == 0 ? 0u : w == 1 ? al1 : al2];
      const uint32_t h0 = h[4 * lane], h1 = h[4 * lane + 1], h2 = h[4 * lane + 2], h3 = h[4 * lane + 3];
      const uint32_t sum = h0 + h1 + h2 + h3, incl = wave_inclusive_sum_u32(sum), excl = incl - sum;
      const uint32_t nd = w == 0 ? need[0] : w == 1 ? need[1] : need[2];
      if (excl < nd && nd <= incl) {
        uint32_t b = 0, acc = excl;
        if (acc + h0 < nd) {
          acc += h0;
          b = 1;
          if (acc + h1 < nd) {
            acc += h1;
            b = 2;
            if (acc + h2 < nd) {
              acc += h2;
              b = 3;
            }
          }
        }
        d.sel_digit[w] = 4 * lane + b;
        d.sel_need[w] = nd - acc;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (act[j]) {
        prefix[j] |= (uint64_t)d.sel_digit[j] << shift;
        need[j] = d.sel_need[j];
      }
    mask |= bm;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) out[j] = prefix[j];
}

// QueueChecker prune of the deep queues check_queues_kernel listed (entries l * 3 + q): keep the
// `max` smallest keys of head and tail (each member's own max with qmax) and drop the rest.
// One 256-thread block per (member, queue):
//   pass 1 streams the head and the tail once and keeps only their 8-B keys in LDS (plus, with
//          transmit counts below 256, the histogram of the keys' first varying byte);
//   one radix select over the LDS keys finds the max-th smallest key T;
//   pass 2 compacts the tail's kept items (key <= T) in place in index order (each batch is read
//          whole before any of its positions is rewritten; an item moves only downwards), so a
//          sealed prefix stays a prefix with its bound intact and only its length changes; the
//          head is sorted, so its items past T are a suffix of its slots and are cleared.
// No refill: the head may be left part-full with a non-empty tail.  That is a valid state --
// emission then cannot decide from the head and the member takes the deferred whole-queue path,
// which refills the head with the queue's smallest keys (emit_deep_wave_kernel).
__global__ void __launch_bounds__(kDeepThreads) check_stream_kernel(GCfg c, GState s, uint32_t max_depth,
                                                                    const uint32_t* __restrict__ qmax, uint32_t n_list) {
  __shared__ CheckLds d;
  __shared__ uint64_t keys[kDeepItems];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
#if RSF_DEEP_PROF
  uint64_t pf[5] = {0, 0, 0, 0, 0}, pc = 0;
#define RSF_CK(i) const uint64_t ck##i = clock64()
#else
#define RSF_CK(i)
#endif
  // check_queues_kernel's entries at fixed places, kEmpty for a queue under its max; the next
  // entry is read while this one is worked on
  uint32_t e_next = blockIdx.x < n_list ? s.deep_ids[blockIdx.x] : kEmpty;
  for (uint32_t it = blockIdx.x; it < n_list; it += gridDim.x) {
    RSF_CK(0);
    const uint32_t e = e_next;
    e_next = it + gridDim.x < n_list ? s.deep_ids[it + gridDim.x] : kEmpty;
    const uint64_t l = e / 3;
    const uint32_t q = e % 3;
    if (l >= c.n_loc || !tcap_of(c, q)) continue;
    const uint32_t keep = qmax ? qmax[l] : max_depth;
    const uint64_t hb = (l * 3 + q) * c.qcap;
    const uint32_t tc = s.tsum[l * 3 + q].x;
    if (c.qcap + tc > kDeepItems) {  // (the tail's capacity is below it: an engine invariant broke)
      if (tid == 0) atomicOr(s.err + l, (uint32_t)RSF_E_DEEP_INVARIANT);
      continue;
    }
    // the intent queue's packed items (q == 0) or the 16-B items of the others
    uint4* const t = q ? tail16(s, q) + l * tstride_of(c, q) : nullptr;
    uint64_t* const t8 = q ? nullptr : tail8(s, c, l);
    const uint32_t nseq = s.q_next_seq[l * 3 + q];  // (every tail item is older)
    // pass 1: the keys into LDS, AND / OR of them, and (transmit counts below 256: byte 7 is
    // zero in every key) the histogram of byte 6 -- the first radix pass of the selects
    const bool fuse = c.tx_limit < 256;
    for (uint32_t i = tid; i < 256; i += kDeepThreads) d.hist[0][i] = 0;
    __syncthreads();
    uint64_t an = ~0ull, orr = 0;
    if (w == 0) {
      const bool live_h = lane < c.qcap && s.q_rumor[hb + lane] != kEmpty;
      const uint64_t lm = ballot(live_h);
      if (live_h) {
        const uint32_t tl = s.q_txlen[hb + lane];
        const uint64_t k = tlq_key(tl & 0xFFFF, tl >> 16, s.q_seq[hb + lane]);
        keys[mbcnt(lm)] = k;
        an = k;
        orr = k;
        if (fuse) atomicAdd(&d.hist[0][(uint32_t)(k >> 48) & 0xFF], 1u);
      }
      if (lane == 0) d.hn = (uint32_t)__popcll(lm);
    }
    __syncthreads();
    const uint32_t hn = d.hn, n = hn + tc;
    constexpr uint32_t U1 = RSF_CHK_U1;
    auto put = [&](uint32_t i, bool in, uint64_t k) {
      if (in) {
        keys[hn + i] = k;
        an &= k;
        orr |= k;
      }
      if (fuse) {  // one atomic for the lanes that agree with the first active lane
        const uint32_t dg = (uint32_t)(k >> 48) & 0xFF;
        const uint64_t am = ballot(in);
        if (am) {
          const int f = __ffsll((long long)am) - 1;
          const uint32_t d0 = shfl_u32(dg, f);
          const uint64_t same = ballot(in && dg == d0);
          if (lane == (uint32_t)f) atomicAdd(&d.hist[0][d0], (uint32_t)__popcll(same));
          else if (in && dg != d0) atomicAdd(&d.hist[0][dg], 1u);
        }
      }
    };
    if (t8) {
      bool old_item = false;  // an item near the end of the packed seq window
      for (uint32_t b = 0; b < tc; b += U1 * kDeepThreads) {
        uint64_t x[U1];
#pragma unroll
        for (uint32_t u = 0; u < U1; ++u) {
          const uint32_t i = b + u * kDeepThreads + tid;
          x[u] = i < tc ? t8[i] : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < U1; ++u) {
          const uint32_t i = b + u * kDeepThreads + tid;
          const uint32_t tl = tail_tl(x[u]);
          old_item |= i < tc && tail_age_over(x[u], nseq);
          put(i, i < tc, tlq_key(tl & 0xFFFF, tl >> 16, tail_seq(x[u], nseq)));
        }
      }
      if (old_item) atomicOr(s.err + l, (uint32_t)RSF_E_DEEP_INVARIANT);
    } else {
      for (uint32_t b = 0; b < tc; b += U1 * kDeepThreads) {
        uint4 x[U1];
#pragma unroll
        for (uint32_t u = 0; u < U1; ++u) {
          const uint32_t i = b + u * kDeepThreads + tid;
          x[u] = i < tc ? t[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t u = 0; u < U1; ++u) {
          const uint32_t i = b + u * kDeepThreads + tid;
          put(i, i < tc, tlq_key(x[u].z & 0xFFFF, x[u].z >> 16, x[u].y));
        }
      }
    }
    an = wave_and_u64_blk(an);
    orr = wave_or_u64_blk(orr);
    __syncthreads();
    if (lane == 0) {
      d.w64[w] = an;
      d.w64b[w] = orr;
    }
    if (tid == 0) d.nb = 0;
    __syncthreads();
    an = d.w64[0];
    orr = d.w64b[0];
#pragma unroll
    for (uint32_t v = 1; v < kDeepWaves; ++v) {
      an &= d.w64[v];
      orr |= d.w64b[v];
    }
    if (n <= keep) continue;  // (listed by the same count: cannot happen)
    RSF_CK(1);
    // the largest key kept
    const uint32_t kk[3] = {keep, 0u, 0u};
    const bool act[3] = {keep > 0, false, false};
    uint64_t sel[3];
    lds_select3(keys, n, d, kk, act, an, orr, fuse, sel);
    const uint64_t T = act[0] ? sel[0] : 0ull;
    const bool any = act[0];
    RSF_CK(2);
    // pass 2: the tail's kept items (key <= T) compacted in place in index order, so the sealed
    // prefix stays a prefix (its bound still holds) and the unsealed items follow it
    const uint32_t m = min(s.tseal[l * 3 + q].x, tc);
    uint32_t kept_sealed = 0;
    for (uint32_t b = 0; b < tc; b += kChkU2 * kDeepThreads) {
      // (the items move as they are: 8 B packed or 16 B; the keys come from pass 1)
      uint4 x[kChkU2];
#pragma unroll
      for (uint32_t u = 0; u < kChkU2; ++u) {
        const uint32_t i = b + u * kDeepThreads + tid;
        if (t8) {
          const uint64_t v = i < tc ? t8[i] : 0ull;
          x[u] = make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u);
        } else {
          x[u] = i < tc ? t[i] : make_uint4(0, 0, 0, 0);
        }
      }
      uint64_t km[kChkU2];
#pragma unroll
      for (uint32_t u = 0; u < kChkU2; ++u) {
        const uint32_t i = b + u * kDeepThreads + tid;
        const bool kp = any && i < tc && keys[hn + i] <= T;
        km[u] = ballot(kp);
        if (lane == 0) d.wcnt[u][w] = (uint32_t)__popcll(km[u]);
        kept_sealed += kp && i < m ? 1u : 0u;
      }
      __syncthreads();  // every thread has read its batch: the batch's positions may be rewritten
      uint32_t base = d.nb, tot = 0;
#pragma unroll
      for (uint32_t u = 0; u < kChkU2; ++u)
#pragma unroll
        for (uint32_t v = 0; v < kDeepWaves; ++v) tot += d.wcnt[u][v];
#pragma unroll
      for (uint32_t u = 0; u < kChkU2; ++u) {
        uint32_t before = 0;
#pragma unroll
        for (uint32_t v = 0; v < kDeepWaves; ++v) before += v < w ? d.wcnt[u][v] : 0u;
        if ((km[u] >> lane) & 1ull) {
          const uint32_t at = base + before + mbcnt(km[u]);
          if (t8) t8[at] = ((uint64_t)x[u].y << 32) | x[u].x;
          else t[at] = x[u];
        }
#pragma unroll
        for (uint32_t v = 0; v < kDeepWaves; ++v) base += d.wcnt[u][v];
      }
      __syncthreads();
      if (tid == 0) d.nb += tot;
      __syncthreads();
    }
    RSF_CK(3);
    // the head is sorted: the items past T are a suffix of its slots
    if (tid < c.qcap && s.q_rumor[hb + tid] != kEmpty &&
        (!any || tlq_key(s.q_txlen[hb + tid] & 0xFFFF, s.q_txlen[hb + tid] >> 16, s.q_seq[hb + tid]) > T)) {
      s.q_rumor[hb + tid] = kEmpty;
      s.q_seq[hb + tid] = 0;
      s.q_txlen[hb + tid] = 0;
    }
    kept_sealed = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum_u32(kept_sealed), 63);
    __syncthreads();
    if (lane == 0) d.wcnt[0][w] = kept_sealed;
    __syncthreads();
    if (tid == 0) {
      uint32_t ms = 0;
      for (uint32_t v = 0; v < kDeepWaves; ++v) ms += d.wcnt[0][v];
      const uint32_t cnt = d.nb;
      const uint4 old = s.tsum[l * 3 + q], os = s.tseal[l * 3 + q];
      // the bounds stay valid lower bounds (only items left)
      s.tsum[l * 3 + q] = cnt ? make_uint4(cnt, old.y, old.z, old.w) : kTSumEmpty;
      s.tseal[l * 3 + q] = ms ? make_uint4(ms, os.y, os.z, os.w) : kTSumEmpty;
    }
    __syncthreads();
#if RSF_DEEP_PROF
    const uint64_t ck4 = clock64();
    pf[0] += ck1 - ck0;
    pf[1] += ck2 - ck1;
    pf[2] += ck3 - ck2;
    pf[3] += ck4 - ck3;
    pf[4] += n;
    pc++;
#endif
  }
#if RSF_DEEP_PROF
  if (tid == 0) {
    for (int i = 0; i < 5; ++i) atomicAdd(&g_deep_prof[64 + i], pf[i]);
    atomicAdd(&g_deep_prof[69], pc);
  }
#endif
#undef RSF_CK
}

// ring wrap: a deep queue's tail drops its items of the recycled generation (one wave per
// (member, queue), in place, order kept); returns the number dropped; exact new bounds
__device__ __forceinline__ uint32_t tail_expire_wave(const GCfg& c, const GState& s, uint64_t l, uint32_t q,
                                                     uint32_t lane, uint32_t gen, uint32_t G) {
  if (!tcap_of(c, q)) return 0;
  const uint4 sm = s.tsum[l * 3 + q];
  if (!sm.x) return 0;
  uint4* const t = q ? tail16(s, q) + l * tstride_of(c, q) : nullptr;
  uint64_t* const t8 = q ? nullptr : tail8(s, c, l);
  const uint32_t nseq = s.q_next_seq[l * 3 + q];
  // packed items hold the generation's parity only: rebuilt against the previous generation
  // (gen - 1), the newest any queued item can have before this wrap, an item is of gen - 1 or
  // of gen - 2 -- the stale one
  const uint32_t gprev = gen == 0 ? G - 1 : gen - 1;
  uint32_t kept = 0, gone = 0, lmin = ~0u;
  uint64_t kmin = ~0ull;
  bool old_item = false;
  for (uint32_t b = 0; b < sm.x; b += kWave) {
    const bool in = b + lane < sm.x;
    uint4 e;
    uint64_t x = 0ull;
    if (t8) {
      x = in ? t8[b + lane] : 0ull;
      e = make_uint4(tail_rid(c, x, gprev), tail_seq(x, nseq), tail_tl(x), 0u);
      old_item |= in && tail_age_over(x, nseq);
    } else {
      e = in ? t[b + lane] : make_uint4(kEmpty, 0u, 0u, 0u);
    }
    const bool stale = in && (gen + G - (e.x >> c.rbits) % G) % G >= 2;
    const bool keep = in && !stale;
    const uint64_t km = ballot(keep);
    __threadfence_block();  // every lane has read its item before any is overwritten
    if (keep) {
      if (t8) t8[kept + mbcnt(km)] = x;
      else t[kept + mbcnt(km)] = e;
    }
    const uint64_t k = keep ? tlq_key(e.z & 0xFFFF, e.z >> 16, e.y) : ~0ull;
    const uint64_t mk = wave_min_u64(k);
    kmin = mk < kmin ? mk : kmin;
    lmin = min(lmin, wave_min_u32(keep ? (e.z >> 16) : ~0u));
    kept += (uint32_t)__popcll(km);
    gone += (uint32_t)__popcll(ballot(stale));
  }
  if (ballot(old_item) && lane == 0) atomicOr(s.err + l, (uint32_t)RSF_E_DEEP_INVARIANT);
  if (gone && lane == 0) {  // exact bounds over what is kept; the whole tail sealed
    s.tsum[l * 3 + q] = kept ? make_uint4(kept, lmin, (uint32_t)kmin, (uint32_t)(kmin >> 32)) : kTSumEmpty;
    s.tseal[l * 3 + q] = kept ? make_uint4(kept, (uint32_t)kmin, (uint32_t)(kmin >> 32), 0u) : kTSumEmpty;
  }
  return gone;
}

}  // namespace
