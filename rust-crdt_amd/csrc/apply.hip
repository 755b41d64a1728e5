// Batched op path: CmRDT::apply for Orswot (src/orswot.rs:61-85) over a batch
// of canonical records, each with its own ordered op list. SURVEY.md §8(f)
// rank 2 ("the adjacent step to state merge").
//
//   Op::Add { dot, member }: no-op if clock[dot.actor] >= dot.counter; else
//     entries[member].witness(dot); clock.witness(dot); apply_deferred()
//   Op::Rm { clock, member }: apply_remove(member, clock) (src/orswot.rs:195-211):
//     if !(clock <= self.clock) deferred[clock] += member;
//     entries[member].subtract(clock), dropped when empty
//   apply_deferred (:235-243): every deferred (D, S) is re-applied; since the
//     subtracts commute and `D <= clock` does not depend on the member, this is
//     "subtract D from every member of S, then drop the (D, S) with D <= clock".
//
// One wave per object (one wave per block): the record is unpacked into LDS
// arrays (the canonical sections with spare capacity), every op edits them in
// place with wave-cooperative gap inserts / deletes, and the final state is
// written back as a canonical record at
//     out_off[i] = self_off[i] + 32 * (ops before i) + 16 * (Rm clock pairs before i) + 32 * i
// (16-B aligned) which bounds every growth (an Add adds <= 24 B, an Rm <= 12 per clock pair
// + 16, padding <= 32).
#include <hip/hip_runtime.h>

#include <atomic>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "sched.h"
#include "record_layout.h"

namespace crdts_hip {
namespace {

constexpr uint32_t kAW = 64;
// Workspace capacities. Every object is first run in the small workspace
// (8 KB of LDS: ~20 resident waves per CU); an object that outgrows it is
// listed and redone from its input in the large one (16 KB).
template <uint32_t CK, uint32_t MEM, uint32_t DOT, uint32_t DEF, uint32_t FDOT, uint32_t FMEM, uint32_t TMP,
          bool G = false>
struct Caps {
  static constexpr bool kG = G;            // the workspace lives in HBM (hand-offs wait for stores)
  static constexpr uint32_t kCk = CK;      // top clock: dense slots (n_actors <= kCk) or sparse entries
  static constexpr uint32_t kMem = MEM;    // members
  static constexpr uint32_t kDot = DOT;    // member dots
  static constexpr uint32_t kDef = DEF;    // deferred clocks
  static constexpr uint32_t kFDot = FDOT;  // deferred clock entries
  static constexpr uint32_t kFMem = FMEM;  // deferred members
  static constexpr uint32_t kTmp = TMP;    // the clock an Rm / a deferred re-apply subtracts
};
using SmallCaps = Caps<64, 64, 256, 16, 128, 128, 64>;
using BigCaps = Caps<128, 128, 512, 32, 256, 256, 128>;
// the third tier: a workspace in HBM (one per wave of a 64-wave launch) for
// objects past BigCaps — member clocks of any length up to kCk entries
using HugeCaps = Caps<2048, 4096, 16384, 256, 4096, 4096, 2048, true>;
constexpr uint32_t kApHugeWaves = 64;
constexpr uint64_t kApPending = 1ull << 63;  // out_off flag: object left for the large workspace
constexpr uint64_t kApPendingHuge = 1ull << 62;  // ... left for the HBM workspace
constexpr uint64_t kApOpBytesDense = 32;   // output bytes reserved per op, dense top clocks
constexpr uint64_t kApOpBytesSparse = 48;  // ... CSR top clocks (a new clock entry: +12 B)

template <class C>
struct Ws {
  uint64_t cctr[C::kCk];
  uint64_t key[C::kMem];
  uint64_t dctr[C::kDot];
  uint64_t fctr[C::kFDot];
  uint64_t fkey[C::kFMem];
  uint64_t tctr[C::kTmp];
  uint32_t cact[C::kCk];
  uint32_t dend[C::kMem];
  uint32_t dact[C::kDot];
  uint32_t fact[C::kFDot];
  uint32_t fdend[C::kDef];
  uint32_t fmend[C::kDef];
  uint32_t tact[C::kTmp];
  uint32_t dead[C::kDef];
};

struct Cnt {
  uint32_t clk, mem, dot, def, fdot, fmem, tmp;
};

// hand-off between the lanes of the wave through the workspace: LDS, or
// (G) HBM, whose stores must have completed before another lane reads
template <bool G = false>
__device__ __forceinline__ void ap_sync() {
  if constexpr (G) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}
__device__ __forceinline__ uint32_t ap_uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t ap_uni64(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}
__device__ __forceinline__ uint32_t ap_count(bool p) { return (uint32_t)__popcll(__ballot(p)); }
__device__ __forceinline__ uint32_t ap_sum(uint32_t v) {
  for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kAW);
  return ap_uni(v);
}

// a[pos..n) -> a[pos+cnt..n+cnt): chunks from the top, so no chunk's stores
// land on a later chunk's loads
template <bool G = false, class T>
__device__ void ins_gap(T* a, uint32_t n, uint32_t pos, uint32_t cnt, uint32_t lane) {
  for (int32_t base = (int32_t)n; base > (int32_t)pos; base -= (int32_t)kAW) {
    const int32_t i = base - 1 - (int32_t)lane;
    if (i >= (int32_t)pos) {
      const T v = a[i];
      a[i + cnt] = v;
    }
  }
  ap_sync<G>();
}
// a[pos+cnt..n) -> a[pos..n-cnt)
template <bool G = false, class T>
__device__ void del_gap(T* a, uint32_t n, uint32_t pos, uint32_t cnt, uint32_t lane) {
  for (uint32_t base = pos; base + cnt < n; base += kAW) {
    const uint32_t i = base + lane;
    if (i + cnt < n) {
      const T v = a[i + cnt];
      a[i] = v;
    }
  }
  ap_sync<G>();
}
template <bool G = false, class T>
__device__ void add_range(T* a, uint32_t b, uint32_t e, T d, uint32_t lane) {
  for (uint32_t i = b + lane; i < e; i += kAW) a[i] += d;
  ap_sync<G>();
}
// # of a[b..e) < x (a sorted or not: a plain count)
template <class T>
__device__ uint32_t count_less(const T* a, uint32_t b, uint32_t e, T x, uint32_t lane) {
  uint32_t c = 0;
  for (uint32_t i = b; i < e; i += kAW) c += ap_count(i + lane < e && a[i + lane] < x);
  return c;
}
// per-lane lookup of actor x in a sorted (act, ctr) list of n entries
__device__ __forceinline__ uint64_t list_get(const uint32_t* act, const uint64_t* ctr, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (act[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && act[lo] == x ? ctr[lo] : 0ull;
}
template <class C>
__device__ __forceinline__ uint64_t clock_get(const Ws<C>& w, const Cnt& c, bool sparse, uint32_t x) {
  return sparse ? list_get(w.cact, w.cctr, c.clk, x) : (x < c.clk ? w.cctr[x] : 0ull);
}

// tmp <= top clock (for canonical clocks: every tmp entry <= the clock's)
template <class C>
__device__ bool tmp_le_clock(const Ws<C>& w, const Cnt& c, bool sparse, uint32_t lane) {
  bool bad = false;
  for (uint32_t i = lane; i < c.tmp; i += kAW) bad = bad || w.tctr[i] > clock_get(w, c, sparse, w.tact[i]);
  return __ballot(bad) == 0ull;
}

// entries[m].subtract(tmp) (src/vclock.rs:236-242); drop the entry if empty
template <class C>
__device__ void entry_subtract(Ws<C>& w, Cnt& c, uint64_t m, uint32_t lane) {
  const uint32_t pos = count_less(w.key, 0u, c.mem, m, lane);
  if (pos >= c.mem || w.key[pos] != m) return;
  const uint32_t b = pos ? w.dend[pos - 1] : 0u, e = w.dend[pos], n = e - b;
  uint32_t kept = 0;
  if constexpr (C::kCk > 2u * kAW) {
    // the HBM workspace: runs of any length, compacted in place 64 dots at a
    // time (a chunk's writes land at or below its own reads, never on a later
    // chunk's)
    for (uint32_t base = 0; base < n; base += kAW) {
      const bool h = base + lane < n;
      uint32_t x = 0;
      uint64_t v = 0;
      if (h) { x = w.dact[b + base + lane]; v = w.dctr[b + base + lane]; }
      const bool k = h && !(list_get(w.tact, w.tctr, c.tmp, x) >= v);
      const uint64_t K = __ballot(k);
      ap_sync<C::kG>();
      const uint32_t r = kept + __builtin_amdgcn_mbcnt_hi((uint32_t)(K >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K, 0u));
      if (k && kept + (uint32_t)__popcll(K) < n + 1u) { w.dact[b + r] = x; w.dctr[b + r] = v; }
      kept += (uint32_t)__popcll(K);
      ap_sync<C::kG>();
    }
    if (kept == n) return;
  } else {
    // the run has <= C::kCk dots (one per actor): two per lane at most
    uint32_t x0 = 0, x1 = 0;
    uint64_t v0 = 0, v1 = 0;
    const bool h0 = lane < n, h1 = lane + kAW < n;
    if (h0) { x0 = w.dact[b + lane]; v0 = w.dctr[b + lane]; }
    if (h1) { x1 = w.dact[b + kAW + lane]; v1 = w.dctr[b + kAW + lane]; }
    const bool k0 = h0 && !(list_get(w.tact, w.tctr, c.tmp, x0) >= v0);
    const bool k1 = h1 && !(list_get(w.tact, w.tctr, c.tmp, x1) >= v1);
    const uint64_t K0 = __ballot(k0), K1 = __ballot(k1);
    kept = (uint32_t)__popcll(K0) + (uint32_t)__popcll(K1);
    if (kept == n) return;
    ap_sync<C::kG>();
    const uint32_t r0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(K0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K0, 0u));
    const uint32_t r1 = (uint32_t)__popcll(K0) +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(K1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K1, 0u));
    if (k0) { w.dact[b + r0] = x0; w.dctr[b + r0] = v0; }
    if (k1) { w.dact[b + r1] = x1; w.dctr[b + r1] = v1; }
    ap_sync<C::kG>();
  }
  const uint32_t drop = n - kept;
  del_gap<C::kG>(w.dact, c.dot, b + kept, drop, lane);
  del_gap<C::kG>(w.dctr, c.dot, b + kept, drop, lane);
  c.dot -= drop;
  add_range<C::kG>(w.dend, pos, c.mem, 0u - drop, lane);
  if (kept == 0u) {  // an empty member clock is removed (src/orswot.rs:206-208)
    del_gap<C::kG>(w.key, c.mem, pos, 1u, lane);
    del_gap<C::kG>(w.dend, c.mem, pos, 1u, lane);
    c.mem -= 1u;
  }
}

// lexicographic (actor, counter) compare of deferred clock k with tmp, a
// proper prefix first: -1, 0, 1 (per lane: k = the lane's clock)
template <class C>
__device__ int def_cmp_tmp(const Ws<C>& w, const Cnt& c, uint32_t k) {
  const uint32_t b = k ? w.fdend[k - 1] : 0u, n = w.fdend[k] - b;
  const uint32_t m = n < c.tmp ? n : c.tmp;
  for (uint32_t i = 0; i < m; ++i) {
    const uint32_t xa = w.fact[b + i], xb = w.tact[i];
    if (xa != xb) return xa < xb ? -1 : 1;
    const uint64_t ca = w.fctr[b + i], cb = w.tctr[i];
    if (ca != cb) return ca < cb ? -1 : 1;
  }
  return n == c.tmp ? 0 : (n < c.tmp ? -1 : 1);
}

// deferred[tmp] += {m}; returns an error code on capacity overflow
template <class C>
__device__ int deferred_add(Ws<C>& w, Cnt& c, uint64_t m, uint32_t lane) {
  // the deferred clocks are in CLOCK ORDER: walk them 64 at a time, counting
  // the ones ordered before tmp and stopping at the first chunk that holds an
  // equal clock (kDef > 64 in the HBM tier)
  uint32_t kk = 0u, keq = ~0u;
  for (uint32_t k0 = 0; k0 < c.def; k0 += kAW) {
    const bool h = k0 + lane < c.def;
    const int cm = h ? def_cmp_tmp(w, c, k0 + lane) : 1;
    const uint64_t eq = __ballot(h && cm == 0);
    kk += ap_count(h && cm < 0);
    if (eq) { keq = k0 + (uint32_t)__builtin_ctzll(eq); break; }
    if (kk < k0 + kAW) break;  // a clock ordered after tmp: the rest are too
  }
  if (keq != ~0u) {
    const uint32_t k = keq;
    const uint32_t ms = k ? w.fmend[k - 1] : 0u, me = w.fmend[k];
    const uint32_t r = count_less(w.fkey, ms, me, m, lane);
    if (ms + r < me && w.fkey[ms + r] == m) return 0;  // already in the set
    if (c.fmem + 1u > C::kFMem) return CRDT_ECAPACITY;
    ins_gap<C::kG>(w.fkey, c.fmem, ms + r, 1u, lane);
    if (lane == 0u) w.fkey[ms + r] = m;
    ap_sync<C::kG>();
    add_range<C::kG>(w.fmend, k, c.def, 1u, lane);
    c.fmem += 1u;
    return 0;
  }
  if (c.def + 1u > C::kDef || c.fdot + c.tmp > C::kFDot || c.fmem + 1u > C::kFMem) return CRDT_ECAPACITY;
  const uint32_t o =kk ? w.fdend[kk - 1] : 0u, om = kk ? w.fmend[kk - 1] : 0u;
  ins_gap<C::kG>(w.fact, c.fdot, o, c.tmp, lane);
  ins_gap<C::kG>(w.fctr, c.fdot, o, c.tmp, lane);
  for (uint32_t i = lane; i < c.tmp; i += kAW) { w.fact[o + i] = w.tact[i]; w.fctr[o + i] = w.tctr[i]; }
  ins_gap<C::kG>(w.fkey, c.fmem, om, 1u, lane);
  if (lane == 0u) w.fkey[om] = m;
  ins_gap<C::kG>(w.fdend, c.def, kk, 1u, lane);
  ins_gap<C::kG>(w.fmend, c.def, kk, 1u, lane);
  if (lane == 0u) { w.fdend[kk] = o + c.tmp; w.fmend[kk] = om + 1u; }
  ap_sync<C::kG>();
  add_range<C::kG>(w.fdend, kk + 1u, c.def + 1u, c.tmp, lane);
  add_range<C::kG>(w.fmend, kk + 1u, c.def + 1u, 1u, lane);
  c.def += 1u;
  c.fdot += c.tmp;
  c.fmem += 1u;
  return 0;
}

// apply_deferred (src/orswot.rs:235-243)
template <class C>
__device__ void apply_deferred(Ws<C>& w, Cnt& c, bool sparse, uint32_t lane) {
  if (c.def == 0u) return;
  for (uint32_t k = 0; k < c.def; ++k) {
    const uint32_t b = k ? w.fdend[k - 1] : 0u, e = w.fdend[k];
    const uint32_t ms = k ? w.fmend[k - 1] : 0u, me = w.fmend[k];
    for (uint32_t i = lane; i < e - b; i += kAW) { w.tact[i] = w.fact[b + i]; w.tctr[i] = w.fctr[b + i]; }
    c.tmp = e - b;
    ap_sync<C::kG>();
    for (uint32_t j = ms; j < me; ++j) entry_subtract(w, c, w.fkey[j], lane);
    const bool applied = tmp_le_clock(w, c, sparse, lane);
    if (lane == 0u) w.dead[k] = applied ? 1u : 0u;
    ap_sync<C::kG>();
  }
  for (int32_t k = (int32_t)c.def - 1; k >= 0; --k) {  // drop the applied ones (top down keeps indices valid)
    if (!w.dead[k]) continue;
    const uint32_t b = k ? w.fdend[k - 1] : 0u, e = w.fdend[k];
    const uint32_t ms = k ? w.fmend[k - 1] : 0u, me = w.fmend[k];
    del_gap<C::kG>(w.fact, c.fdot, b, e - b, lane);
    del_gap<C::kG>(w.fctr, c.fdot, b, e - b, lane);
    del_gap<C::kG>(w.fkey, c.fmem, ms, me - ms, lane);
    add_range<C::kG>(w.fdend, (uint32_t)k + 1u, c.def, 0u - (e - b), lane);
    add_range<C::kG>(w.fmend, (uint32_t)k + 1u, c.def, 0u - (me - ms), lane);
    del_gap<C::kG>(w.fdend, c.def, (uint32_t)k, 1u, lane);
    del_gap<C::kG>(w.fmend, c.def, (uint32_t)k, 1u, lane);
    c.fdot -= e - b;
    c.fmem -= me - ms;
    c.def -= 1u;
  }
}

// Op::Add (src/orswot.rs:66-79)
template <class C>
__device__ int op_add(Ws<C>& w, Cnt& c, bool sparse, uint32_t A, uint32_t a, uint64_t ctr, uint64_t m, uint32_t lane) {
  if (a >= A) return CRDT_ENONCANON;
  uint64_t cur = 0;
  uint32_t cpos = 0;
  if (sparse) {
    cpos = count_less(w.cact, 0u, c.clk, a, lane);
    cur = cpos < c.clk && w.cact[cpos] == a ? w.cctr[cpos] : 0ull;
  } else {
    cur = w.cctr[a];
  }
  cur = ap_uni64(cur);
  if (cur >= ctr) return 0;  // already seen
  // entries[m] (inserted empty when absent) .witness(dot)
  uint32_t pos = count_less(w.key, 0u, c.mem, m, lane);
  if (pos >= c.mem || w.key[pos] != m) {
    if (c.mem + 1u > C::kMem) return CRDT_ECAPACITY;
    const uint32_t at = pos ? w.dend[pos - 1] : 0u;
    ins_gap<C::kG>(w.key, c.mem, pos, 1u, lane);
    ins_gap<C::kG>(w.dend, c.mem, pos, 1u, lane);
    if (lane == 0u) { w.key[pos] = m; w.dend[pos] = at; }
    ap_sync<C::kG>();
    c.mem += 1u;
  }
  const uint32_t b = pos ? w.dend[pos - 1] : 0u, e = w.dend[pos];
  const uint32_t r = count_less(w.dact, b, e, a, lane);
  if (C::kCk <= 2u * kAW && e - b + 1u > 2u * kAW) return CRDT_ECAPACITY;  // LDS tiers: a run in two registers per lane
  if (b + r < e && w.dact[b + r] == a) {
    if (lane == 0u && w.dctr[b + r] < ctr) w.dctr[b + r] = ctr;
    ap_sync<C::kG>();
  } else {
    if (c.dot + 1u > C::kDot) return CRDT_ECAPACITY;
    ins_gap<C::kG>(w.dact, c.dot, b + r, 1u, lane);
    ins_gap<C::kG>(w.dctr, c.dot, b + r, 1u, lane);
    if (lane == 0u) { w.dact[b + r] = a; w.dctr[b + r] = ctr; }
    ap_sync<C::kG>();
    add_range<C::kG>(w.dend, pos, c.mem, 1u, lane);
    c.dot += 1u;
  }
  // clock.witness(dot)
  if (sparse) {
    if (cpos < c.clk && w.cact[cpos] == a) {
      if (lane == 0u) w.cctr[cpos] = ctr;
    } else {
      if (c.clk + 1u > C::kCk) return CRDT_ECAPACITY;
      ins_gap<C::kG>(w.cact, c.clk, cpos, 1u, lane);
      ins_gap<C::kG>(w.cctr, c.clk, cpos, 1u, lane);
      if (lane == 0u) { w.cact[cpos] = a; w.cctr[cpos] = ctr; }
      c.clk += 1u;
    }
  } else if (lane == 0u) {
    w.cctr[a] = ctr;
  }
  ap_sync<C::kG>();
  apply_deferred(w, c, sparse, lane);
  return 0;
}

// Op::Rm -> apply_remove (src/orswot.rs:195-211); the op clock is in tmp
template <class C>
__device__ int op_rm(Ws<C>& w, Cnt& c, bool sparse, uint64_t m, uint32_t lane) {
  if (!tmp_le_clock(w, c, sparse, lane)) {
    const int rc = deferred_add(w, c, m, lane);
    if (rc) return rc;
  }
  entry_subtract(w, c, m, lane);
  return 0;
}

// Wave-uniform read of an input that no kernel of the launch writes, through
// the constant address space: the compiler emits a scalar (SMEM) load, whose
// wait (lgkmcnt) does not also wait for this wave's earlier vector stores, as
// a vector load's vmcnt wait would (the counter drains in order).
template <class T>
__device__ __forceinline__ T ldc(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}

// the record header (8 u32, already read) is consistent with the record's bounds
__device__ bool rec_ok_h(const uint32_t (&h)[8], uint64_t bytes, uint64_t off, uint32_t A, uint32_t flags) {
  const bool sparse = (flags & kSparseClock) != 0u;
  if (h[7] != flags || (sparse ? h[1] > A : h[1] != A)) return false;
  const uint64_t sz = record_size64(h[1], h[2], h[3], h[4], h[5], h[6], sparse);
  return sz == h[0] && off + sz <= bytes;
}

__device__ bool rec_ok(const uint8_t* base, uint64_t bytes, uint64_t off, uint32_t A, uint32_t flags) {
  if ((off & 15u) || off + kHdrBytes > bytes) return false;
  const uint32_t* h = (const uint32_t*)(base + off);
  const bool sparse = (flags & kSparseClock) != 0u;
  if (h[7] != flags || (sparse ? h[1] > A : h[1] != A)) return false;
  const uint64_t sz = record_size64(h[1], h[2], h[3], h[4], h[5], h[6], sparse);
  return sz == h[0] && off + sz <= bytes;
}

struct ApArgs {
  const uint8_t* sb;
  uint64_t sbytes;
  const uint64_t* soff;
  uint64_t n_obj;
  const uint64_t* obj_end;
  const uint32_t* kind;
  const uint64_t* member;
  const uint32_t* actor;
  const uint64_t* counter;
  const uint64_t* clk_end;
  const uint32_t* clk_act;
  const uint64_t* clk_ctr;
  uint64_t n_ops, n_clk;  // sizes of the op arrays / of the clock-pair arrays
  uint32_t A, flags;
  uint8_t* out;
  uint64_t* ooff;
  uint64_t out_bytes;
  int* status;
  uint32_t* ctl;      // [0]: # objects left for the large workspace
  uint64_t* list;     // their indices (list_cap of them; beyond that, out_off flags)
  uint32_t list_cap;
};

__device__ __forceinline__ uint32_t ap_lane(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t ap_lane64(uint64_t v, uint32_t l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
}
// ops q0 .. min(q0 + 64, oe) - 1: lane i holds op q0 + i
__device__ __forceinline__ void op_fetch(const ApArgs& g, uint64_t q0, uint64_t oe, uint32_t lane, uint32_t& rk,
                                         uint64_t& rm, uint32_t& ra, uint64_t& rn, uint64_t& re) {
  const uint64_t q = q0 + lane;
  if (q < oe && q < g.n_ops) {
    rk = g.kind[q];
    rm = g.member[q];
    ra = g.actor[q];
    rn = g.counter[q];
    re = g.clk_end[q];
  }
}

// clock pairs c0 .. min(c0 + 127, ce - 1) (the first Rm clocks of an object;
// ce = its pairs' end): lane i holds pairs c0 + i and c0 + 64 + i. Bounded by
// the object's own pairs: reading a fixed 128-pair window re-read the
// neighbours' pairs (~1.5 KB per object, on another XCD's L2 for the next
// object), ~1 GB of the launch's 2.3 GB of reads (profiles/r03_apply_*)
__device__ __forceinline__ void clk_fetch(const ApArgs& g, uint64_t c0, uint64_t ce, uint32_t lane, uint32_t& xa0,
                                          uint64_t& xc0, uint32_t& xa1, uint64_t& xc1) {
  const uint64_t e = ce < g.n_clk ? ce : g.n_clk;
  if (c0 + lane < e) { xa0 = g.clk_act[c0 + lane]; xc0 = g.clk_ctr[c0 + lane]; }
  if (c0 + kAW + lane < e) { xa1 = g.clk_act[c0 + kAW + lane]; xc1 = g.clk_ctr[c0 + kAW + lane]; }
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t j) {
  return ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)j, kAW) << 32) |
         (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, (int)j, kAW);
}

// One object: unpack, run its ops in order, write the canonical record.
template <class C>
__device__ int apply_one(Ws<C>& w, const ApArgs& g, uint64_t o, uint32_t lane) {
  const uint8_t* __restrict__ sb = g.sb;
  const uint64_t sbytes = g.sbytes, out_bytes = g.out_bytes;
  const uint64_t* __restrict__ soff = g.soff;
  const uint64_t* __restrict__ obj_end = g.obj_end;
  const uint64_t* __restrict__ clk_end = g.clk_end;
  const uint32_t A = g.A, flags = g.flags;
  uint8_t* __restrict__ out = g.out;
  uint64_t* __restrict__ ooff = g.ooff;
  const bool sparse = (flags & kSparseClock) != 0u;
  const uint64_t so = ldc(soff + o);
  const uint64_t ob = o ? ldc(obj_end + o - 1) : 0u, oe = ldc(obj_end + o);
  const uint64_t cb = ob ? ldc(clk_end + ob - 1) : 0u;
  uint32_t h[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};  // the record header, by scalar loads
  const bool hdr_in = (so & 15u) == 0u && so + kHdrBytes <= sbytes;
  if (hdr_in) {
    const uint32_t* hp = (const uint32_t*)(sb + so);
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = ldc(hp + k);
  }
  // output placement: an op grows a record by at most 32 B in the dense form
  // (new member key + run end + dot, or a deferred key + its two run ends)
  // and 36 B in the sparse form (a new top-clock entry on top: 48 B keeps the
  // 16-B alignment); each Rm clock pair by 16 B; padding by < 32 B per object
  const uint64_t per_op = sparse ? kApOpBytesSparse : kApOpBytesDense;
  const uint64_t oo = so + per_op * ob + 16u * cb + 32u * o;
  const uint64_t ce = oe ? ldc(clk_end + oe - 1) : 0u;
  if (lane == 0u) ooff[o] = oo;  // also clears a pending flag
  // the object's first 64 ops -> registers (lane i: op ob + i), loaded
  // together with the record so the op loop waits on no global load
  uint32_t rk = 0, ra = 0;
  uint64_t rm = 0, rn = 0, re = 0, pe = cb;
  op_fetch(g, ob, oe, lane, rk, rm, ra, rn, re);
  uint32_t xa0 = 0, xa1 = 0;
  uint64_t xc0 = 0, xc1 = 0;
  clk_fetch(g, cb, ce, lane, xa0, xc0, xa1, xc1);
  int rc = 0;
  if (!hdr_in || !rec_ok_h(h, sbytes, so, A, flags) || oe < ob || oe > g.n_ops) rc = CRDT_ENONCANON;
  const uint8_t* r = sb + so;
  Cnt c{};
  if (!rc) {
    c = Cnt{ap_uni(h[1]), ap_uni(h[2]), ap_uni(h[3]), ap_uni(h[4]), ap_uni(h[5]), ap_uni(h[6]), 0u};
    if (c.clk > C::kCk || c.mem > C::kMem || c.dot > C::kDot || c.def > C::kDef || c.fdot > C::kFDot ||
        c.fmem > C::kFMem)
      rc = CRDT_ECAPACITY;
  }
  if (!rc) {  // unpack the record into the workspace
    RecLayout L;
    rec_layout(L, c.clk, c.mem, c.dot, c.def, c.fdot, c.fmem, sparse);
    // element `lane` of every section first: all loads in flight together, one
    // wait, then the workspace stores (the rest, past 64, after)
    {
      const uint32_t i = lane;
      uint64_t v0 = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0;
      uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0, u4 = 0, u5 = 0;
      if (i < c.clk) {
        v0 = ((const uint64_t*)(r + L.o_clk))[i];
        if (sparse) u0 = ((const uint32_t*)(r + L.o_cact))[i];
      }
      if (i < c.mem) { v1 = ((const uint64_t*)(r + L.o_key))[i]; u1 = ((const uint32_t*)(r + L.o_mdend))[i]; }
      if (i < c.dot) { v2 = ((const uint64_t*)(r + L.o_dctr))[i]; u2 = ((const uint32_t*)(r + L.o_dact))[i]; }
      if (i < c.fdot) { v3 = ((const uint64_t*)(r + L.o_fctr))[i]; u3 = ((const uint32_t*)(r + L.o_fact))[i]; }
      if (i < c.fmem) v4 = ((const uint64_t*)(r + L.o_fkey))[i];
      if (i < c.def) { u4 = ((const uint32_t*)(r + L.o_fdend))[i]; u5 = ((const uint32_t*)(r + L.o_fmend))[i]; }
      if (i < c.clk) { w.cctr[i] = v0; if (sparse) w.cact[i] = u0; }
      if (i < c.mem) { w.key[i] = v1; w.dend[i] = u1; }
      if (i < c.dot) { w.dctr[i] = v2; w.dact[i] = u2; }
      if (i < c.fdot) { w.fctr[i] = v3; w.fact[i] = u3; }
      if (i < c.fmem) w.fkey[i] = v4;
      if (i < c.def) { w.fdend[i] = u4; w.fmend[i] = u5; }
    }
    for (uint32_t i = kAW + lane; i < c.clk; i += kAW) {
      w.cctr[i] = ((const uint64_t*)(r + L.o_clk))[i];
      if (sparse) w.cact[i] = ((const uint32_t*)(r + L.o_cact))[i];
    }
    for (uint32_t i = kAW + lane; i < c.mem; i += kAW) {
      w.key[i] = ((const uint64_t*)(r + L.o_key))[i];
      w.dend[i] = ((const uint32_t*)(r + L.o_mdend))[i];
    }
    for (uint32_t i = kAW + lane; i < c.dot; i += kAW) {
      w.dctr[i] = ((const uint64_t*)(r + L.o_dctr))[i];
      w.dact[i] = ((const uint32_t*)(r + L.o_dact))[i];
    }
    for (uint32_t i = kAW + lane; i < c.fdot; i += kAW) {
      w.fctr[i] = ((const uint64_t*)(r + L.o_fctr))[i];
      w.fact[i] = ((const uint32_t*)(r + L.o_fact))[i];
    }
    for (uint32_t i = kAW + lane; i < c.fmem; i += kAW) w.fkey[i] = ((const uint64_t*)(r + L.o_fkey))[i];
    for (uint32_t i = kAW + lane; i < c.def; i += kAW) {
      w.fdend[i] = ((const uint32_t*)(r + L.o_fdend))[i];
      w.fmend[i] = ((const uint32_t*)(r + L.o_fmend))[i];
    }
    ap_sync<C::kG>();
    if constexpr (C::kCk <= 2u * kAW) {  // the LDS tiers hold a member's run in two registers per lane
      bool big = false;
      for (uint32_t i = lane; i < c.mem; i += kAW) big = big || w.dend[i] - (i ? w.dend[i - 1] : 0u) > 2u * kAW;
      if (__ballot(big)) rc = CRDT_ECAPACITY;
    }
  }
  for (uint64_t q = ob; q < oe && !rc; ++q) {  // the object's ops, in order
    const uint32_t qi = (uint32_t)(q - ob) & (kAW - 1u);
    if (qi == 0u && q != ob) {
      op_fetch(g, q, oe, lane, rk, rm, ra, rn, re);
      pe = ap_uni64(clk_end[q - 1]);
    }
    const uint32_t k = ap_lane(rk, qi);
    const uint64_t m = ap_lane64(rm, qi);
    if (k == CRDT_OP_ADD) {
      rc = op_add(w, c, sparse, A, ap_lane(ra, qi), ap_lane64(rn, qi), m, lane);
      if (qi == kAW - 1u) pe = ap_lane64(re, qi);
    } else if (k == CRDT_OP_RM) {
      const uint64_t b = qi ? ap_lane64(re, qi - 1u) : pe, e = ap_lane64(re, qi);
      if (qi == kAW - 1u) pe = e;
      if (e < b || e - b > C::kTmp) { rc = e < b ? CRDT_ENONCANON : CRDT_ECAPACITY; break; }
      if (e > g.n_clk) { rc = CRDT_ENONCANON; break; }
      bool bad = false;
      if (e - cb <= 2u * kAW) {  // the pairs are in registers (clk_fetch)
        uint32_t xlast = 0;  // the previous pass's last actor
        for (uint32_t base = 0; base < (uint32_t)(e - b); base += kAW) {
          const uint32_t i = base + lane;
          const uint32_t j = (uint32_t)(b - cb) + i;  // pair j of the object's first 128
          const uint32_t jl = j & (kAW - 1u);
          const uint32_t a0 = (uint32_t)__shfl((int)xa0, (int)jl, kAW), a1 = (uint32_t)__shfl((int)xa1, (int)jl, kAW);
          const uint64_t c0 = shfl64(xc0, jl), c1 = shfl64(xc1, jl);
          const uint32_t x = j < kAW ? a0 : a1;
          const uint64_t v = j < kAW ? c0 : c1;
          uint32_t xp = (uint32_t)__shfl((int)x, (int)((lane - 1u) & (kAW - 1u)), kAW);
          if (lane == 0u) xp = xlast;
          if (i < (uint32_t)(e - b)) {
            bad = bad || x >= A || v == 0u || (i && xp >= x);  // canonical VClock
            w.tact[i] = x;
            w.tctr[i] = v;
          }
          xlast = (uint32_t)__shfl((int)x, (int)(kAW - 1u), kAW);
        }
      } else {
        for (uint32_t i = lane; i < (uint32_t)(e - b); i += kAW) {
          const uint32_t x = g.clk_act[b + i];
          const uint64_t v = g.clk_ctr[b + i];
          bad = bad || x >= A || v == 0u || (i && g.clk_act[b + i - 1] >= x);  // canonical VClock
          w.tact[i] = x;
          w.tctr[i] = v;
        }
      }
      c.tmp = (uint32_t)(e - b);
      ap_sync<C::kG>();
      if (__ballot(bad)) { rc = CRDT_ENONCANON; break; }
      rc = op_rm(w, c, sparse, m, lane);
    } else {
      rc = CRDT_ENONCANON;
    }
  }
  if (!rc) {  // write the canonical record
    uint32_t n_clk = c.clk;
    RecLayout L;
    rec_layout(L, n_clk, c.mem, c.dot, c.def, c.fdot, c.fmem, sparse);
    // never past this object's own reserved span (the next object's output
    // starts right after it when the input records are packed in order)
    const uint64_t span = (uint64_t)h[0] + per_op * (oe - ob) + 16u * (ce >= cb ? ce - cb : 0u) + 32u;
    if (oo + L.size > out_bytes || (oo & 15u) || L.size > span) {
      rc = CRDT_ECAPACITY;
    } else {
      uint8_t* O = out + oo;
      for (uint32_t i = lane; i < n_clk; i += kAW) {
        ((uint64_t*)(O + L.o_clk))[i] = w.cctr[i];
        if (sparse) ((uint32_t*)(O + L.o_cact))[i] = w.cact[i];
      }
      if (sparse && lane == 0u && (n_clk & 1u)) *(uint32_t*)(O + L.o_cact + 4u * n_clk) = 0u;
      for (uint32_t i = lane; i < c.mem; i += kAW) {
        ((uint64_t*)(O + L.o_key))[i] = w.key[i];
        ((uint32_t*)(O + L.o_mdend))[i] = w.dend[i];
      }
      for (uint32_t i = lane; i < c.dot; i += kAW) {
        ((uint64_t*)(O + L.o_dctr))[i] = w.dctr[i];
        ((uint32_t*)(O + L.o_dact))[i] = w.dact[i];
      }
      for (uint32_t i = lane; i < c.fdot; i += kAW) {
        ((uint64_t*)(O + L.o_fctr))[i] = w.fctr[i];
        ((uint32_t*)(O + L.o_fact))[i] = w.fact[i];
      }
      for (uint32_t i = lane; i < c.fmem; i += kAW) ((uint64_t*)(O + L.o_fkey))[i] = w.fkey[i];
      for (uint32_t i = lane; i < c.def; i += kAW) {
        ((uint32_t*)(O + L.o_fdend))[i] = w.fdend[i];
        ((uint32_t*)(O + L.o_fmend))[i] = w.fmend[i];
      }
      if (lane == 0u && L.o_def != L.o_mpad) *(uint32_t*)(O + L.o_mpad) = 0u;
      if (lane >= 1u && lane < 4u && L.o_end + 4u * (lane - 1u) < L.size)
        *(uint32_t*)(O + L.o_end + 4u * (lane - 1u)) = 0u;
      if (lane == 0u) {
        uint32_t* oh = (uint32_t*)O;
        oh[0] = L.size; oh[1] = n_clk; oh[2] = c.mem; oh[3] = c.dot;
        oh[4] = c.def; oh[5] = c.fdot; oh[6] = c.fmem; oh[7] = sparse ? kSparseClock : 0u;
      }
    }
  }
  return rc;
}

// TIER 0: every object in the small workspace; one that outgrows it is listed
// (and flagged in out_off) instead of failing. TIER 1: the large workspace
// over the listed objects (or over the flagged ones when the list overflowed);
// one that outgrows it is listed again for TIER 2: the HBM workspace (one per
// block of a kApHugeWaves-block launch). The two lists are the halves of the
// context's list: [0, cap/2) with count ctl[0], [cap/2, cap) with ctl[1].
template <class C, int TIER>
__device__ __forceinline__ Ws<C>& ap_workspace(uint8_t* huge_ws) {
  if constexpr (TIER == 2) {
    return *(Ws<C>*)(huge_ws + (uint64_t)blockIdx.x * sizeof(Ws<C>));
  } else {
    __shared__ Ws<C> w_lds;
    return w_lds;
  }
}

template <class C, int TIER>
__global__ __launch_bounds__(kAW) void orswot_apply_kernel(ApArgs g, uint8_t* huge_ws) {
  static_assert(TIER != 2 || C::kG, "the HBM tier needs the HBM-fenced caps");
  Ws<C>& w = ap_workspace<C, TIER>(huge_ws);
  const uint32_t lane = threadIdx.x;
  const uint32_t half = g.list_cap / 2u;
  if (TIER == 0) {
    // BlockTickets (sched.h): half the objects by block index, the rest in
    // 4-object atomic tickets (ctl[3]) — one call site, so apply_one is
    // inlined once (two call sites doubled the kernel's VGPRs). (An
    // XCD-aware split — contiguous object ranges per XCD — measured slower:
    // 3.47 vs 2.67 ms)
    BlockTickets<4> sched(g.n_obj, g.ctl + 3, lane);
    for (uint64_t o = sched.first(); o < g.n_obj; o = sched.next(o)) {
      const int rc = apply_one<C>(w, g, o, lane);
      if (rc && lane == 0u) {
        if (rc == CRDT_ECAPACITY) {
          g.ooff[o] |= kApPending;
          const uint32_t e = atomicAdd(&g.ctl[0], 1u);
          if (e < half) g.list[e] = o;
        } else {
          atomicCAS(g.status, 0, rc);
        }
      }
      ap_sync<C::kG>();
    }
    return;
  }
  const uint64_t flag = TIER == 1 ? kApPending : kApPendingHuge;
  const uint32_t n = ap_uni(__hip_atomic_load(&g.ctl[TIER - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (n == 0u) return;
  const bool listed = n <= half;
  const uint64_t* lst = g.list + (TIER == 1 ? 0u : half);
  const uint64_t m = listed ? n : g.n_obj;
  for (uint64_t e = blockIdx.x; e < m; e += gridDim.x) {
    const uint64_t o = listed ? ap_uni64(lst[e]) : e;
    if (!listed && !(ap_uni64(g.ooff[o]) & flag)) continue;
    const int rc = apply_one<C>(w, g, o, lane);
    if (rc && lane == 0u) {
      if (TIER == 1 && rc == CRDT_ECAPACITY) {
        g.ooff[o] |= kApPendingHuge;
        const uint32_t e2 = atomicAdd(&g.ctl[1], 1u);
        if (e2 < half) g.list[half + e2] = o;
      } else {
        atomicCAS(g.status, 0, rc);
      }
    }
    ap_sync<C::kG>();
  }
}

}  // namespace

size_t launch_apply_huge_scratch_bytes() { return sizeof(Ws<HugeCaps>) * (size_t)kApHugeWaves; }

int launch_orswot_apply(const uint8_t* sb, uint64_t sbytes, const uint64_t* soff, uint64_t n_obj,
                        const uint64_t* obj_end, const uint32_t* kind, const uint64_t* member, const uint32_t* actor,
                        const uint64_t* counter, const uint64_t* clk_end, const uint32_t* clk_act,
                        const uint64_t* clk_ctr, uint64_t n_ops, uint64_t n_clk, uint32_t A, uint32_t flags,
                        uint8_t* out, uint64_t* ooff,
                        uint64_t out_bytes, int* status, uint32_t* ctl, uint64_t* list, uint32_t list_cap,
                        uint8_t* huge_ws, hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  if (!huge_ws) return CRDT_EINVAL;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  static std::atomic<int> occ_small{0}, occ_big{0};
  auto occ_of = [](std::atomic<int>& slot, const void* fn) {
    int occ = slot.load(std::memory_order_relaxed);
    if (occ == 0) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kAW, 0) != hipSuccess || occ < 1) occ = 8;
      slot.store(occ, std::memory_order_relaxed);
    }
    return (uint64_t)occ;
  };
  const void* fs = (const void*)orswot_apply_kernel<SmallCaps, 0>;
  const void* fb = (const void*)orswot_apply_kernel<BigCaps, 1>;
  const void* fh = (const void*)orswot_apply_kernel<HugeCaps, 2>;
  ApArgs g{sb, sbytes, soff, n_obj, obj_end, kind, member, actor, counter, clk_end, clk_act, clk_ctr, n_ops, n_clk,
           A, flags, out, ooff, out_bytes, status, ctl, list, list_cap};
  void* args[] = {&g, &huge_ws};
  if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;  // ctl[3]: tickets
  const bool dense_big = !(flags & kSparseClock) && A > SmallCaps::kCk;  // nothing fits the small workspace
  if (dense_big) {  // every object in the large workspace: the "list overflowed" path with all objects flagged
    if (hipMemsetD32Async((hipDeviceptr_t)ctl, 0xFFFFFFFF, 1, stream) != hipSuccess) return CRDT_EHIP;
    if (hipMemsetAsync(ooff, 0xFF, 8 * n_obj, stream) != hipSuccess) return CRDT_EHIP;
  } else {
    const uint64_t cap = (uint64_t)cus * occ_of(occ_small, fs);
    const uint32_t blocks = (uint32_t)(n_obj < cap ? n_obj : cap);
    if (hipLaunchKernel(fs, dim3(blocks), dim3(kAW), args, 0, stream) != hipSuccess) return CRDT_EHIP;
  }
  const uint64_t capb = (uint64_t)cus * occ_of(occ_big, fb);
  const uint32_t bb = (uint32_t)(n_obj < capb ? n_obj : capb);
  if (hipLaunchKernel(fb, dim3(bb), dim3(kAW), args, 0, stream) != hipSuccess) return CRDT_EHIP;
  if (hipLaunchKernel(fh, dim3(kApHugeWaves), dim3(kAW), args, 0, stream) != hipSuccess) return CRDT_EHIP;
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
