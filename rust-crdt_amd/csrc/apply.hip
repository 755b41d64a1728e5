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

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "record_layout.h"

namespace crdts_hip {
namespace {

constexpr uint32_t kAW = 64;
constexpr uint32_t kApCk = 128;      // top clock: dense slots (n_actors <= 128) or sparse entries
constexpr uint32_t kApMem = 128;     // members
constexpr uint32_t kApDot = 512;     // member dots
constexpr uint32_t kApDef = 32;      // deferred clocks
constexpr uint32_t kApFDot = 256;    // deferred clock entries
constexpr uint32_t kApFMem = 256;    // deferred members
constexpr uint32_t kApTmp = 128;     // the clock an Rm / a deferred re-apply subtracts

struct Ws {
  uint64_t cctr[kApCk];
  uint64_t key[kApMem];
  uint64_t dctr[kApDot];
  uint64_t fctr[kApFDot];
  uint64_t fkey[kApFMem];
  uint64_t tctr[kApTmp];
  uint32_t cact[kApCk];
  uint32_t dend[kApMem];
  uint32_t dact[kApDot];
  uint32_t fact[kApFDot];
  uint32_t fdend[kApDef];
  uint32_t fmend[kApDef];
  uint32_t tact[kApTmp];
  uint32_t dead[kApDef];
};

struct Cnt {
  uint32_t clk, mem, dot, def, fdot, fmem, tmp;
};

__device__ __forceinline__ void ap_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
template <class T>
__device__ void ins_gap(T* a, uint32_t n, uint32_t pos, uint32_t cnt, uint32_t lane) {
  for (int32_t base = (int32_t)n; base > (int32_t)pos; base -= (int32_t)kAW) {
    const int32_t i = base - 1 - (int32_t)lane;
    if (i >= (int32_t)pos) {
      const T v = a[i];
      a[i + cnt] = v;
    }
  }
  ap_sync();
}
// a[pos+cnt..n) -> a[pos..n-cnt)
template <class T>
__device__ void del_gap(T* a, uint32_t n, uint32_t pos, uint32_t cnt, uint32_t lane) {
  for (uint32_t base = pos; base + cnt < n; base += kAW) {
    const uint32_t i = base + lane;
    if (i + cnt < n) {
      const T v = a[i + cnt];
      a[i] = v;
    }
  }
  ap_sync();
}
template <class T>
__device__ void add_range(T* a, uint32_t b, uint32_t e, T d, uint32_t lane) {
  for (uint32_t i = b + lane; i < e; i += kAW) a[i] += d;
  ap_sync();
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
__device__ __forceinline__ uint64_t clock_get(const Ws& w, const Cnt& c, bool sparse, uint32_t x) {
  return sparse ? list_get(w.cact, w.cctr, c.clk, x) : (x < c.clk ? w.cctr[x] : 0ull);
}

// tmp <= top clock (for canonical clocks: every tmp entry <= the clock's)
__device__ bool tmp_le_clock(const Ws& w, const Cnt& c, bool sparse, uint32_t lane) {
  bool bad = false;
  for (uint32_t i = lane; i < c.tmp; i += kAW) bad = bad || w.tctr[i] > clock_get(w, c, sparse, w.tact[i]);
  return __ballot(bad) == 0ull;
}

// entries[m].subtract(tmp) (src/vclock.rs:236-242); drop the entry if empty
__device__ void entry_subtract(Ws& w, Cnt& c, uint64_t m, uint32_t lane) {
  const uint32_t pos = count_less(w.key, 0u, c.mem, m, lane);
  if (pos >= c.mem || w.key[pos] != m) return;
  const uint32_t b = pos ? w.dend[pos - 1] : 0u, e = w.dend[pos], n = e - b;
  // the run has <= kApCk dots (one per actor): two per lane at most
  uint32_t x0 = 0, x1 = 0;
  uint64_t v0 = 0, v1 = 0;
  const bool h0 = lane < n, h1 = lane + kAW < n;
  if (h0) { x0 = w.dact[b + lane]; v0 = w.dctr[b + lane]; }
  if (h1) { x1 = w.dact[b + kAW + lane]; v1 = w.dctr[b + kAW + lane]; }
  const bool k0 = h0 && !(list_get(w.tact, w.tctr, c.tmp, x0) >= v0);
  const bool k1 = h1 && !(list_get(w.tact, w.tctr, c.tmp, x1) >= v1);
  const uint64_t K0 = __ballot(k0), K1 = __ballot(k1);
  const uint32_t kept = (uint32_t)__popcll(K0) + (uint32_t)__popcll(K1);
  if (kept == n) return;
  ap_sync();
  const uint32_t r0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(K0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K0, 0u));
  const uint32_t r1 = (uint32_t)__popcll(K0) +
                      __builtin_amdgcn_mbcnt_hi((uint32_t)(K1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K1, 0u));
  if (k0) { w.dact[b + r0] = x0; w.dctr[b + r0] = v0; }
  if (k1) { w.dact[b + r1] = x1; w.dctr[b + r1] = v1; }
  ap_sync();
  const uint32_t drop = n - kept;
  del_gap(w.dact, c.dot, b + kept, drop, lane);
  del_gap(w.dctr, c.dot, b + kept, drop, lane);
  c.dot -= drop;
  add_range(w.dend, pos, c.mem, 0u - drop, lane);
  if (kept == 0u) {  // an empty member clock is removed (src/orswot.rs:206-208)
    del_gap(w.key, c.mem, pos, 1u, lane);
    del_gap(w.dend, c.mem, pos, 1u, lane);
    c.mem -= 1u;
  }
}

// lexicographic (actor, counter) compare of deferred clock k with tmp, a
// proper prefix first: -1, 0, 1 (per lane: k = the lane's clock)
__device__ int def_cmp_tmp(const Ws& w, const Cnt& c, uint32_t k) {
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
__device__ int deferred_add(Ws& w, Cnt& c, uint64_t m, uint32_t lane) {
  int cm = 1;
  if (lane < c.def) cm = def_cmp_tmp(w, c, lane);
  const uint64_t eq = __ballot(lane < c.def && cm == 0);
  if (eq) {
    const uint32_t k = (uint32_t)__builtin_ctzll(eq);
    const uint32_t ms = k ? w.fmend[k - 1] : 0u, me = w.fmend[k];
    const uint32_t r = count_less(w.fkey, ms, me, m, lane);
    if (ms + r < me && w.fkey[ms + r] == m) return 0;  // already in the set
    if (c.fmem + 1u > kApFMem) return CRDT_ECAPACITY;
    ins_gap(w.fkey, c.fmem, ms + r, 1u, lane);
    if (lane == 0u) w.fkey[ms + r] = m;
    ap_sync();
    add_range(w.fmend, k, c.def, 1u, lane);
    c.fmem += 1u;
    return 0;
  }
  if (c.def + 1u > kApDef || c.fdot + c.tmp > kApFDot || c.fmem + 1u > kApFMem) return CRDT_ECAPACITY;
  const uint32_t kk = ap_count(lane < c.def && cm < 0);  // clocks ordered before tmp
  const uint32_t o = kk ? w.fdend[kk - 1] : 0u, om = kk ? w.fmend[kk - 1] : 0u;
  ins_gap(w.fact, c.fdot, o, c.tmp, lane);
  ins_gap(w.fctr, c.fdot, o, c.tmp, lane);
  for (uint32_t i = lane; i < c.tmp; i += kAW) { w.fact[o + i] = w.tact[i]; w.fctr[o + i] = w.tctr[i]; }
  ins_gap(w.fkey, c.fmem, om, 1u, lane);
  if (lane == 0u) w.fkey[om] = m;
  ins_gap(w.fdend, c.def, kk, 1u, lane);
  ins_gap(w.fmend, c.def, kk, 1u, lane);
  if (lane == 0u) { w.fdend[kk] = o + c.tmp; w.fmend[kk] = om + 1u; }
  ap_sync();
  add_range(w.fdend, kk + 1u, c.def + 1u, c.tmp, lane);
  add_range(w.fmend, kk + 1u, c.def + 1u, 1u, lane);
  c.def += 1u;
  c.fdot += c.tmp;
  c.fmem += 1u;
  return 0;
}

// apply_deferred (src/orswot.rs:235-243)
__device__ void apply_deferred(Ws& w, Cnt& c, bool sparse, uint32_t lane) {
  if (c.def == 0u) return;
  for (uint32_t k = 0; k < c.def; ++k) {
    const uint32_t b = k ? w.fdend[k - 1] : 0u, e = w.fdend[k];
    const uint32_t ms = k ? w.fmend[k - 1] : 0u, me = w.fmend[k];
    for (uint32_t i = lane; i < e - b; i += kAW) { w.tact[i] = w.fact[b + i]; w.tctr[i] = w.fctr[b + i]; }
    c.tmp = e - b;
    ap_sync();
    for (uint32_t j = ms; j < me; ++j) entry_subtract(w, c, w.fkey[j], lane);
    const bool applied = tmp_le_clock(w, c, sparse, lane);
    if (lane == 0u) w.dead[k] = applied ? 1u : 0u;
    ap_sync();
  }
  for (int32_t k = (int32_t)c.def - 1; k >= 0; --k) {  // drop the applied ones (top down keeps indices valid)
    if (!w.dead[k]) continue;
    const uint32_t b = k ? w.fdend[k - 1] : 0u, e = w.fdend[k];
    const uint32_t ms = k ? w.fmend[k - 1] : 0u, me = w.fmend[k];
    del_gap(w.fact, c.fdot, b, e - b, lane);
    del_gap(w.fctr, c.fdot, b, e - b, lane);
    del_gap(w.fkey, c.fmem, ms, me - ms, lane);
    add_range(w.fdend, (uint32_t)k + 1u, c.def, 0u - (e - b), lane);
    add_range(w.fmend, (uint32_t)k + 1u, c.def, 0u - (me - ms), lane);
    del_gap(w.fdend, c.def, (uint32_t)k, 1u, lane);
    del_gap(w.fmend, c.def, (uint32_t)k, 1u, lane);
    c.fdot -= e - b;
    c.fmem -= me - ms;
    c.def -= 1u;
  }
}

// Op::Add (src/orswot.rs:66-79)
__device__ int op_add(Ws& w, Cnt& c, bool sparse, uint32_t A, uint32_t a, uint64_t ctr, uint64_t m, uint32_t lane) {
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
    if (c.mem + 1u > kApMem) return CRDT_ECAPACITY;
    const uint32_t at = pos ? w.dend[pos - 1] : 0u;
    ins_gap(w.key, c.mem, pos, 1u, lane);
    ins_gap(w.dend, c.mem, pos, 1u, lane);
    if (lane == 0u) { w.key[pos] = m; w.dend[pos] = at; }
    ap_sync();
    c.mem += 1u;
  }
  const uint32_t b = pos ? w.dend[pos - 1] : 0u, e = w.dend[pos];
  const uint32_t r = count_less(w.dact, b, e, a, lane);
  if (e - b + 1u > 2u * kAW) return CRDT_ECAPACITY;  // entry_subtract holds a run in two registers per lane
  if (b + r < e && w.dact[b + r] == a) {
    if (lane == 0u && w.dctr[b + r] < ctr) w.dctr[b + r] = ctr;
    ap_sync();
  } else {
    if (c.dot + 1u > kApDot) return CRDT_ECAPACITY;
    ins_gap(w.dact, c.dot, b + r, 1u, lane);
    ins_gap(w.dctr, c.dot, b + r, 1u, lane);
    if (lane == 0u) { w.dact[b + r] = a; w.dctr[b + r] = ctr; }
    ap_sync();
    add_range(w.dend, pos, c.mem, 1u, lane);
    c.dot += 1u;
  }
  // clock.witness(dot)
  if (sparse) {
    if (cpos < c.clk && w.cact[cpos] == a) {
      if (lane == 0u) w.cctr[cpos] = ctr;
    } else {
      if (c.clk + 1u > kApCk) return CRDT_ECAPACITY;
      ins_gap(w.cact, c.clk, cpos, 1u, lane);
      ins_gap(w.cctr, c.clk, cpos, 1u, lane);
      if (lane == 0u) { w.cact[cpos] = a; w.cctr[cpos] = ctr; }
      c.clk += 1u;
    }
  } else if (lane == 0u) {
    w.cctr[a] = ctr;
  }
  ap_sync();
  apply_deferred(w, c, sparse, lane);
  return 0;
}

// Op::Rm -> apply_remove (src/orswot.rs:195-211); the op clock is in tmp
__device__ int op_rm(Ws& w, Cnt& c, bool sparse, uint64_t m, uint32_t lane) {
  if (!tmp_le_clock(w, c, sparse, lane)) {
    const int rc = deferred_add(w, c, m, lane);
    if (rc) return rc;
  }
  entry_subtract(w, c, m, lane);
  return 0;
}

__device__ bool rec_ok(const uint8_t* base, uint64_t bytes, uint64_t off, uint32_t A, uint32_t flags) {
  if ((off & 15u) || off + kHdrBytes > bytes) return false;
  const uint32_t* h = (const uint32_t*)(base + off);
  const bool sparse = (flags & kSparseClock) != 0u;
  if (h[7] != flags || (sparse ? h[1] > A : h[1] != A)) return false;
  const uint64_t sz = record_size64(h[1], h[2], h[3], h[4], h[5], h[6], sparse);
  return sz == h[0] && off + sz <= bytes;
}

__global__ __launch_bounds__(kAW) void orswot_apply_kernel(
    const uint8_t* __restrict__ sb, uint64_t sbytes, const uint64_t* __restrict__ soff, uint64_t n_obj,
    const uint64_t* __restrict__ obj_end, const uint32_t* __restrict__ kind, const uint64_t* __restrict__ member,
    const uint32_t* __restrict__ actor, const uint64_t* __restrict__ counter, const uint64_t* __restrict__ clk_end,
    const uint32_t* __restrict__ clk_act, const uint64_t* __restrict__ clk_ctr, uint32_t A, uint32_t flags,
    uint8_t* __restrict__ out, uint64_t* __restrict__ ooff, uint64_t out_bytes, int* __restrict__ status) {
  __shared__ Ws w;
  const uint32_t lane = threadIdx.x;
  const bool sparse = (flags & kSparseClock) != 0u;
  for (uint64_t o = blockIdx.x; o < n_obj; o += gridDim.x) {
    const uint64_t so = soff[o];
    const uint64_t ob = o ? obj_end[o - 1] : 0u, oe = obj_end[o];
    const uint64_t cb = ob ? clk_end[ob - 1] : 0u;
    const uint64_t oo = so + 32u * ob + 16u * cb + 32u * o;
    if (lane == 0u) ooff[o] = oo;
    int rc = 0;
    if (!rec_ok(sb, sbytes, so, A, flags) || oe < ob) rc = CRDT_ENONCANON;
    const uint8_t* r = sb + so;
    const uint32_t* h = (const uint32_t*)r;
    Cnt c{};
    if (!rc) {
      c = Cnt{ap_uni(h[1]), ap_uni(h[2]), ap_uni(h[3]), ap_uni(h[4]), ap_uni(h[5]), ap_uni(h[6]), 0u};
      if (c.clk > kApCk || c.mem > kApMem || c.dot > kApDot || c.def > kApDef || c.fdot > kApFDot ||
          c.fmem > kApFMem)
        rc = CRDT_ECAPACITY;
    }
    if (!rc) {  // unpack the record into the workspace
      RecLayout L;
      rec_layout(L, c.clk, c.mem, c.dot, c.def, c.fdot, c.fmem, sparse);
      for (uint32_t i = lane; i < c.clk; i += kAW) {
        w.cctr[i] = ((const uint64_t*)(r + L.o_clk))[i];
        if (sparse) w.cact[i] = ((const uint32_t*)(r + L.o_cact))[i];
      }
      for (uint32_t i = lane; i < c.mem; i += kAW) {
        w.key[i] = ((const uint64_t*)(r + L.o_key))[i];
        w.dend[i] = ((const uint32_t*)(r + L.o_mdend))[i];
      }
      for (uint32_t i = lane; i < c.dot; i += kAW) {
        w.dctr[i] = ((const uint64_t*)(r + L.o_dctr))[i];
        w.dact[i] = ((const uint32_t*)(r + L.o_dact))[i];
      }
      for (uint32_t i = lane; i < c.fdot; i += kAW) {
        w.fctr[i] = ((const uint64_t*)(r + L.o_fctr))[i];
        w.fact[i] = ((const uint32_t*)(r + L.o_fact))[i];
      }
      for (uint32_t i = lane; i < c.fmem; i += kAW) w.fkey[i] = ((const uint64_t*)(r + L.o_fkey))[i];
      for (uint32_t i = lane; i < c.def; i += kAW) {
        w.fdend[i] = ((const uint32_t*)(r + L.o_fdend))[i];
        w.fmend[i] = ((const uint32_t*)(r + L.o_fmend))[i];
      }
      ap_sync();
      bool big = false;
      for (uint32_t i = lane; i < c.mem; i += kAW) big = big || w.dend[i] - (i ? w.dend[i - 1] : 0u) > 2u * kAW;
      if (__ballot(big)) rc = CRDT_ECAPACITY;
    }
    for (uint64_t q = ob; q < oe && !rc; ++q) {  // the object's ops, in order
      const uint32_t k = ap_uni(kind[q]);
      const uint64_t m = ap_uni64(member[q]);
      if (k == CRDT_OP_ADD) {
        rc = op_add(w, c, sparse, A, ap_uni(actor[q]), ap_uni64(counter[q]), m, lane);
      } else if (k == CRDT_OP_RM) {
        const uint64_t b = q ? clk_end[q - 1] : 0u, e = clk_end[q];
        if (e < b || e - b > kApTmp) { rc = e < b ? CRDT_ENONCANON : CRDT_ECAPACITY; break; }
        bool bad = false;
        for (uint32_t i = lane; i < (uint32_t)(e - b); i += kAW) {
          const uint32_t x = clk_act[b + i];
          const uint64_t v = clk_ctr[b + i];
          bad = bad || x >= A || v == 0u || (i && clk_act[b + i - 1] >= x);  // canonical VClock
          w.tact[i] = x;
          w.tctr[i] = v;
        }
        c.tmp = (uint32_t)(e - b);
        ap_sync();
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
      if (oo + L.size > out_bytes || (oo & 15u)) {
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
    if (rc && lane == 0u) atomicCAS(status, 0, rc);
    ap_sync();
  }
}

}  // namespace

int launch_orswot_apply(const uint8_t* sb, uint64_t sbytes, const uint64_t* soff, uint64_t n_obj,
                        const uint64_t* obj_end, const uint32_t* kind, const uint64_t* member, const uint32_t* actor,
                        const uint64_t* counter, const uint64_t* clk_end, const uint32_t* clk_act,
                        const uint64_t* clk_ctr, uint32_t A, uint32_t flags, uint8_t* out, uint64_t* ooff,
                        uint64_t out_bytes, int* status, hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t cap = (uint64_t)cus * 9u;
  const uint32_t blocks = (uint32_t)(n_obj < cap ? n_obj : cap);
  hipLaunchKernelGGL(orswot_apply_kernel, dim3(blocks), dim3(kAW), 0, stream, sb, sbytes, soff, n_obj, obj_end, kind,
                     member, actor, counter, clk_end, clk_act, clk_ctr, A, flags, out, ooff, out_bytes, status);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
