// Orswot batch join on gfx950: one wavefront per object pair.
//
// out[i] = self[i].merge(&other[i]) — CvRDT for Orswot, src/orswot.rs:87-157,
// including apply_deferred (:235-243) / apply_remove (:195-211).
//
// Work assignment: each wave owns chunks of 64 consecutive objects. Per chunk
// lane k loads object k's two offsets and two record headers in one
// coalesced step (2 dependent HBM round trips per 64 objects), and writes the
// chunk's 64 output offsets in one store. Per object, the wave then
//  1. copies both input records HBM -> registers -> LDS with 16-B loads; the
//     loads for object t+1 are issued before object t is computed, so their
//     HBM latency hides behind the join (software pipeline, 1 object deep);
//  2. merges the two sorted member-key lists by MERGE PATH, one union
//     position per lane (self first on ties: a key present on both sides is
//     handled by the self lane, its twin lane idles), and per position runs
//     one join loop over the two actor-sorted dot runs implementing the
//     reference's rules — self-only :94-104, both :105-128, other-only
//     :132-138 — followed by the deferred subtraction (:195-211);
//  3. a count pass fixes the output section offsets (wave ballot + prefix
//     sum), a write pass stores keys / dots / ends straight to the final
//     place of the output record in HBM;
//  4. deferred maps: union keyed by clock (:141-148), kept iff
//     !(D <= merged clock) (:197); rare, done by lane 0;
//  5. top clock = pointwise max (:153), written by lanes < n_actors.
// Records larger than the LDS stage (kStageBytes) are flagged in the output
// offset (bit 63) and joined by orswot_merge_big_kernel with the same code
// (staged through a larger LDS buffer, or straight from HBM).
//
// Canonical record layout: include/crdts_hip.h, record_layout.h.
#include <hip/hip_runtime.h>

#include <atomic>

#include "../../include/crdts_hip.h"
#include "ctx.h"
#include "kernels.h"
#include "sched.h"
#include "record_layout.h"

namespace crdts_hip {
namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum : uint32_t { kNone = 0, kSelf = 1, kOther = 2, kBoth = 3 };

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Diagnostic in-kernel stamps (ABL == 9 builds only; never in the real
// kernel): s_memtime with its own lgkmcnt wait, fenced by sched barriers.
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
struct Stamps {
  uint64_t acc[16];
  uint64_t last;
};
template <int ABL>
__device__ __forceinline__ void mark(Stamps& st, int k) {
  if (ABL == 9) {
    const uint64_t t = stamp();
    st.acc[k] += t - st.last;
    st.last = t;
  }
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}
__device__ __forceinline__ uint32_t lane_of(uint32_t v, uint32_t t) { return __builtin_amdgcn_readlane(v, t); }
__device__ __forceinline__ uint64_t lane_of64(uint64_t v, uint32_t t) {
  // readlane yields int: widen through uint32_t, or a low half with bit 31
  // set sign-extends over the high half (offsets >= 2 GiB)
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), t) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, t);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    uint32_t t = __shfl_up(v, off, kWave);
    if (lane >= (uint32_t)off) v += t;
  }
  return v;
}

// Byte offsets of one record's sections (wave-uniform), relative to its base.
struct RV {
  uint32_t clk, cact, key, dctr, dact, mdend, fctr, fkey, fact, fdend, fmend;
  uint32_t n_mem, n_def, n_clk, n_dm;  // (n_dm: deferred member entries, all clocks)
};

__device__ __forceinline__ RV make_rv(const RecLayout& L) {
  RV v;
  v.clk = L.o_clk; v.cact = L.o_cact; v.n_clk = L.n_clk; v.key = L.o_key; v.dctr = L.o_dctr; v.dact = L.o_dact; v.mdend = L.o_mdend;
  v.fctr = L.o_fctr; v.fkey = L.o_fkey; v.fact = L.o_fact; v.fdend = L.o_fdend; v.fmend = L.o_fmend;
  v.n_mem = L.n_mem; v.n_def = L.n_def; v.n_dm = L.n_def_mem;
  return v;
}

// Record accessors (base = LDS stage or HBM record; offsets in bytes). The
// base is a generic pointer, or an LDS-typed one (lds_cu8: ds_* loads, no
// flat round trip) where the record is known to sit in the wave's stage.
typedef const __attribute__((address_space(3))) uint8_t lds_cu8;
__device__ __forceinline__ uint64_t g64(const uint8_t* b, uint32_t off, uint32_t i) {
  return *(const uint64_t*)(b + off + 8u * i);
}
__device__ __forceinline__ uint32_t g32(const uint8_t* b, uint32_t off, uint32_t i) {
  return *(const uint32_t*)(b + off + 4u * i);
}
__device__ __forceinline__ uint64_t g64(lds_cu8* b, uint32_t off, uint32_t i) {
  return *(const __attribute__((address_space(3))) uint64_t*)(b + off + 8u * i);
}
__device__ __forceinline__ uint32_t g32(lds_cu8* b, uint32_t off, uint32_t i) {
  return *(const __attribute__((address_space(3))) uint32_t*)(b + off + 4u * i);
}
// VClock::get on a dense top clock, absent = 0 (src/vclock.rs:206-210)
template <class P>
__device__ __forceinline__ uint64_t top(P b, const RV& v, uint32_t a, uint32_t A) {
  return a < A ? g64(b, v.clk, a) : 0ull;
}
// First index k in [0, n) of the sparse clock's actor list with act[k] >= a.
template <class P>
__device__ __forceinline__ uint32_t clk_lower_bound(P b, const RV& v, uint32_t a) {
  uint32_t lo = 0, n = v.n_clk;
  while (n) {
    const uint32_t h = n >> 1;
    if (g32(b, v.cact, lo + h) < a) { lo += h + 1; n -= h + 1; } else { n = h; }
  }
  return lo;
}
// VClock::get for either clock form: a CSR clock is searched (sorted actors).
template <bool SP, class P>
__device__ __forceinline__ uint64_t topv(P b, const RV& v, uint32_t a, uint32_t A) {
  if (!SP) return top(b, v, a, A);
  const uint32_t k = clk_lower_bound(b, v, a);
  return (k < v.n_clk && g32(b, v.cact, k) == a) ? g64(b, v.clk, k) : 0ull;
}
// The same with an actor -> rank table of the clock (u8 k + 1 per actor id
// < kRankTab, 0 = absent; orswot_big_kernel<true>'s per-object LDS table):
// two dependent LDS reads instead of the binary search.
constexpr uint32_t kRankTab = 1024;
template <bool SP, class P>
__device__ __forceinline__ uint64_t topr(P b, const RV& v, uint32_t a, uint32_t A, lds_cu8* rk) {
  if (!SP || rk == nullptr || a >= kRankTab) return topv<SP>(b, v, a, A);
  const uint32_t k = rk[a];
  return k ? g64(b, v.clk, k - 1u) : 0ull;
}
template <class P>
__device__ __forceinline__ uint32_t run_begin(P b, uint32_t off, uint32_t k) {
  return k ? g32(b, off, k - 1) : 0u;
}

template <class P>
struct SideT {
  P b;
  RV v;
};
typedef SideT<const uint8_t*> Side;
typedef SideT<lds_cu8*> SideL;  // a record in the wave's LDS stage

// D[x] for deferred clock k (actor-sorted run), 0 if absent.
template <class S>
__device__ __forceinline__ uint64_t def_get(const S& s, uint32_t k, uint32_t x) {
  uint32_t e = g32(s.b, s.v.fdend, k);
  for (uint32_t d = run_begin(s.b, s.v.fdend, k); d < e; ++d) {
    uint32_t a = g32(s.b, s.v.fact, d);
    if (a >= x) return a == x ? g64(s.b, s.v.fctr, d) : 0ull;
  }
  return 0ull;
}

template <class S>
__device__ __forceinline__ bool def_has_member(const S& s, uint32_t k, uint64_t m) {
  // the run is clamped to the n_dm keys in_any_deferred scans, so the two
  // agree on a record whose member run ends overrun n_dm (not canonical)
  uint32_t hi = g32(s.b, s.v.fmend, k), lo = run_begin(s.b, s.v.fmend, k);
  hi = hi < s.v.n_dm ? hi : s.v.n_dm;
  lo = lo < hi ? lo : hi;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    uint64_t km = g64(s.b, s.v.fkey, mid);
    if (km == m) return true;
    if (km < m) lo = mid + 1; else hi = mid;
  }
  return false;
}

// apply_deferred over the union of both deferred maps (src/orswot.rs:235-243):
// apply_remove subtracts D from entries[m] for every (D, m) — whether or not
// D is re-deferred — dropping dot (x, v) iff D[x] >= v (VClock::subtract,
// src/vclock.rs:236-242). Order-independent, and duplicates are harmless.
template <class S>
__device__ __forceinline__ bool killed(const S& L, const S& R, uint64_t m, uint32_t x, uint64_t v) {
  for (uint32_t k = 0; k < L.v.n_def; ++k)
    if (def_has_member(L, k, m) && def_get(L, k, x) >= v) return true;
  for (uint32_t k = 0; k < R.v.n_def; ++k)
    if (def_has_member(R, k, m) && def_get(R, k, x) >= v) return true;
  return false;
}

// Whether member m appears in any deferred clock's member set of either
// side: a linear pass over both flat fkey arrays (independent loads; both are
// short), so killed() runs only for the members it can hit.
template <class S>
__device__ __forceinline__ bool in_any_deferred(const S& L, const S& R, uint64_t m) {
  bool hit = false;
  for (uint32_t k = 0; k < L.v.n_dm; ++k) hit = hit || g64(L.b, L.v.fkey, k) == m;
  for (uint32_t k = 0; k < R.v.n_dm; ++k) hit = hit || g64(R.b, R.v.fkey, k) == m;
  return hit;
}

// A 1024-bit filter over both sides' deferred member keys (big-object
// kernel): a member whose bit is clear is in no deferred member set.
__device__ __forceinline__ uint32_t dm_hash(uint64_t m) { return (uint32_t)((m * 0x9E3779B97F4A7C15ull) >> 54); }
__device__ __forceinline__ bool dm_maybe(const uint32_t* bloom, uint64_t m) {
  const uint32_t h = dm_hash(m);
  return ((bloom[h >> 5] >> (h & 31u)) & 1u) != 0u;
}

// Merge path: the candidate at union position p (self first on ties).
// Branch-free binary search with a fixed trip count (no per-lane loop
// control): i = number of self keys among the first p union positions.
template <class S>
__device__ __forceinline__ uint32_t merge_path(const S& L, const S& R, uint32_t p, uint32_t& i, uint32_t& j) {
  const uint32_t nL = L.v.n_mem, nR = R.v.n_mem;
  uint32_t lo = p > nR ? p - nR : 0, len = (p < nL ? p : nL) - lo;
  const uint32_t steps = 32u - __builtin_clz(uni(nL < nR ? nL : nR) | 1u);  // >= log2(len + 1)
  for (uint32_t s = 0; s <= steps; ++s) {
    const uint32_t half = len >> 1, mid = lo + half;
    const bool go = len != 0 && g64(L.b, L.v.key, mid) <= g64(R.b, R.v.key, p - 1 - mid);
    lo = go ? mid + 1 : lo;
    len = len == 0 ? 0 : (go ? len - half - 1 : half);
  }
  i = lo;
  j = p - lo;
  const uint64_t kl = i < nL ? g64(L.b, L.v.key, i) : ~0ull;
  const uint64_t kr = j < nR ? g64(R.b, R.v.key, j) : ~0ull;
  if (i < nL && (j >= nR || kl <= kr)) return (j < nR && kl == kr) ? kBoth : kSelf;
  if (i > 0 && g64(L.b, L.v.key, i - 1) == kr) return kNone;  // twin of a kBoth at p-1
  return kOther;
}

// The joined dot run of one member; returns its length. MODE 0 counts and
// captures the first output dot in (x0, v0); MODE 1 also stores the run at
// oact/octr[d0..]. Lc/Rc are the PRE-merge top clocks. One loop step per
// actor of the union of both runs, branch-free inside.
template <int MODE, bool SP = false, class S>
__device__ __forceinline__ uint32_t join(const S& L, const S& R, uint32_t type, uint32_t i,
                                         uint32_t j, uint32_t A, bool has_def, uint32_t& x0, uint64_t& v0,
                                         uint32_t* oact, uint64_t* octr, uint32_t d0,
                                         const uint32_t* bloom = nullptr, lds_cu8* crank = nullptr) {
  // crank (SP): actor -> rank tables of L's and R's top clocks (topr), or null
  lds_cu8* const rkL = crank;
  lds_cu8* const rkR = crank ? crank + kRankTab : nullptr;
  uint32_t a = 0, ae = 0, b = 0, be = 0;
  if (type & kSelf) { a = run_begin(L.b, L.v.mdend, i); ae = g32(L.b, L.v.mdend, i); }
  if (type & kOther) { b = run_begin(R.b, R.v.mdend, j); be = g32(R.b, R.v.mdend, j); }
  if (type == kSelf) {
    // a self-only entry is kept UNCHANGED iff !(clock <= other.clock) (:98-103)
    bool any = false;
    for (uint32_t d = a; d < ae && !any; ++d)
      any = g64(L.b, L.v.dctr, d) > topr<SP>(R.b, R.v, g32(L.b, L.v.dact, d), A, rkR);
    if (!any) ae = a;
  }
  uint64_t m = 0;
  bool mk = false;  // m is in some deferred member set: its dots face the kill test
  if (has_def) {
    m = (type & kSelf) ? g64(L.b, L.v.key, i) : g64(R.b, R.v.key, j);
    mk = (bloom == nullptr || dm_maybe(bloom, m)) && in_any_deferred(L, R, m);
  }
  uint32_t c = 0;
  while (a < ae || b < be) {
    const bool ha = a < ae, hb = b < be;
    const uint32_t xa = ha ? g32(L.b, L.v.dact, a) : 0xFFFFFFFFu;
    const uint32_t xb = hb ? g32(R.b, R.v.dact, b) : 0xFFFFFFFFu;
    const bool ta = xa <= xb, tb = xb <= xa;  // which run(s) hold actor x
    const uint32_t x = ta ? xa : xb;
    const uint64_t va = ta ? g64(L.b, L.v.dctr, a) : 0ull;
    const uint64_t vb = tb ? g64(R.b, R.v.dctr, b) : 0ull;
    const uint64_t rc = topr<SP>(R.b, R.v, x, A, rkR), lc = topr<SP>(L.b, L.v, x, A, rkL);
    // self-only: the whole run (kept); otherwise L[x] survives iff > Rc[x]
    // (:112, :133 analogue), R[x] iff > Lc[x] (:113, :133); a dot equal on
    // both sides is common (:109) and survives as is; result = max (:115-116)
    const uint64_t lp = (ta && (type == kSelf || va > rc)) ? va : 0ull;
    const uint64_t rp = (tb && vb > lc) ? vb : 0ull;
    uint64_t v = (ta && tb && va == vb) ? va : (lp > rp ? lp : rp);
    a += ta ? 1u : 0u;
    b += tb ? 1u : 0u;
    if (v != 0 && mk && killed(L, R, m, x, v)) v = 0;
    if (v != 0) {
      if (MODE == 1) {
        oact[d0 + c] = x;
        octr[d0 + c] = v;
      } else if (c == 0) {
        x0 = x;
        v0 = v;
      }
      ++c;
    }
  }
  return c;
}

// CLOCK ORDER compare of deferred clock k of X with deferred clock l of Y.
__device__ __forceinline__ int clock_cmp(const Side& X, uint32_t k, const Side& Y, uint32_t l) {
  uint32_t a = run_begin(X.b, X.v.fdend, k), ae = g32(X.b, X.v.fdend, k);
  uint32_t b = run_begin(Y.b, Y.v.fdend, l), be = g32(Y.b, Y.v.fdend, l);
  for (; a < ae && b < be; ++a, ++b) {
    uint32_t xa = g32(X.b, X.v.fact, a), xb = g32(Y.b, Y.v.fact, b);
    if (xa != xb) return xa < xb ? -1 : 1;
    uint64_t va = g64(X.b, X.v.fctr, a), vb = g64(Y.b, Y.v.fctr, b);
    if (va != vb) return va < vb ? -1 : 1;
  }
  if (a == ae && b == be) return 0;
  return a == ae ? -1 : 1;
}

// !(D <= merged clock): some dot of D exceeds max(Lc, Rc)  (src/orswot.rs:197)
template <bool SP = false>
__device__ __forceinline__ bool def_survives(const Side& X, uint32_t k, const Side& L, const Side& R,
                                             uint32_t A) {
  uint32_t e = g32(X.b, X.v.fdend, k);
  for (uint32_t d = run_begin(X.b, X.v.fdend, k); d < e; ++d) {
    uint32_t x = g32(X.b, X.v.fact, d);
    uint64_t lc = topv<SP>(L.b, L.v, x, A), rc = topv<SP>(R.b, R.v, x, A);
    if (g64(X.b, X.v.fctr, d) > (lc > rc ? lc : rc)) return true;
  }
  return false;
}

struct DefOut {
  uint64_t* fctr;
  uint64_t* fkey;
  uint32_t* fact;
  uint32_t* fdend;
  uint32_t* fmend;
};

// Deferred union + filter (src/orswot.rs:141-148, then :155 -> :197-203),
// single lane. With w == nullptr only counts.
template <bool SP = false>
__device__ void deferred_pass(const Side& L, const Side& R, uint32_t A, uint32_t& nd, uint32_t& ndd,
                              uint32_t& ndm, const DefOut* w) {
  uint32_t k = 0, l = 0;
  nd = ndd = ndm = 0;
  while (k < L.v.n_def || l < R.v.n_def) {
    const int c = k >= L.v.n_def ? 1 : (l >= R.v.n_def ? -1 : clock_cmp(L, k, R, l));
    const Side& X = c <= 0 ? L : R;
    const uint32_t kx = c <= 0 ? k : l;
    if (def_survives<SP>(X, kx, L, R, A)) {
      uint32_t e = g32(X.b, X.v.fdend, kx);
      for (uint32_t d = run_begin(X.b, X.v.fdend, kx); d < e; ++d) {
        if (w) { w->fact[ndd] = g32(X.b, X.v.fact, d); w->fctr[ndd] = g64(X.b, X.v.fctr, d); }
        ++ndd;
      }
      // member set: self's, other's, or the sorted union of both (c == 0)
      uint32_t a = 0, ae = 0, b = 0, be = 0;
      if (c <= 0) { a = run_begin(L.b, L.v.fmend, k); ae = g32(L.b, L.v.fmend, k); }
      if (c >= 0) { b = run_begin(R.b, R.v.fmend, l); be = g32(R.b, R.v.fmend, l); }
      while (a < ae || b < be) {
        const uint64_t ka = a < ae ? g64(L.b, L.v.fkey, a) : ~0ull;
        const uint64_t kb = b < be ? g64(R.b, R.v.fkey, b) : ~0ull;
        uint64_t km;
        if (a < ae && (b >= be || ka < kb)) { km = ka; ++a; }
        else if (b < be && (a >= ae || kb < ka)) { km = kb; ++b; }
        else { km = ka; ++a; ++b; }
        if (w) w->fkey[ndm] = km;
        ++ndm;
      }
      if (w) { w->fdend[nd] = ndd; w->fmend[nd] = ndm; }
      ++nd;
    }
    if (c <= 0) ++k;
    if (c >= 0) ++l;
  }
}

// Wave-cooperative deferred union + filter (same semantics as deferred_pass:
// src/orswot.rs:141-148, then :155 -> :197-203). Entries are walked in CLOCK
// ORDER by a wave-uniform loop; per entry the dot-level work (clock compare,
// survival test, copies) is spread over the lanes. With w == nullptr only
// counts. Every lane returns the same counts.
template <class S>
__device__ __forceinline__ int clock_cmp_wave(const S& X, uint32_t k, const S& Y, uint32_t l, uint32_t lane) {
  const uint32_t a0 = uni(run_begin(X.b, X.v.fdend, k)), na = uni(g32(X.b, X.v.fdend, k)) - a0;
  const uint32_t b0 = uni(run_begin(Y.b, Y.v.fdend, l)), nb = uni(g32(Y.b, Y.v.fdend, l)) - b0;
  const uint32_t n = na < nb ? na : nb;
  for (uint32_t base = 0; base < n; base += kWave) {
    const uint32_t d = base + lane;
    int c = 0;
    if (d < n) {
      const uint32_t xa = g32(X.b, X.v.fact, a0 + d), xb = g32(Y.b, Y.v.fact, b0 + d);
      const uint64_t va = g64(X.b, X.v.fctr, a0 + d), vb = g64(Y.b, Y.v.fctr, b0 + d);
      c = xa != xb ? (xa < xb ? -1 : 1) : (va != vb ? (va < vb ? -1 : 1) : 0);
    }
    const uint64_t diff = __ballot(c != 0);
    if (diff) return (int)__builtin_amdgcn_readlane((uint32_t)c, (uint32_t)__builtin_ctzll(diff));
  }
  return na == nb ? 0 : (na < nb ? -1 : 1);
}

template <bool SP = false, class S>
__device__ __forceinline__ bool def_survives_wave(const S& X, uint32_t k, const S& L, const S& R, uint32_t A,
                                                  uint32_t lane) {
  const uint32_t s = uni(run_begin(X.b, X.v.fdend, k)), e = uni(g32(X.b, X.v.fdend, k));
  bool any = false;
  for (uint32_t d = s + lane; d < e; d += kWave) {
    const uint32_t x = g32(X.b, X.v.fact, d);
    const uint64_t lc = topv<SP>(L.b, L.v, x, A), rc = topv<SP>(R.b, R.v, x, A);
    any = any || g64(X.b, X.v.fctr, d) > (lc > rc ? lc : rc);
  }
  return __ballot(any) != 0ull;
}

// One surviving deferred entry: clock kx of side X (c: -1 L only, 1 R only,
// 0 on both sides — member sets united), written at the running counts.
template <class S>
__device__ __forceinline__ void deferred_emit(const S& L, const S& R, int c, uint32_t k, uint32_t l,
                                              uint32_t lane, uint32_t& nd, uint32_t& ndd, uint32_t& ndm,
                                              const DefOut* w) {
  const S& X = c <= 0 ? L : R;
  const uint32_t kx = c <= 0 ? k : l;
  const uint32_t s = uni(run_begin(X.b, X.v.fdend, kx)), e = uni(g32(X.b, X.v.fdend, kx));
  if (w)
    for (uint32_t d = s + lane; d < e; d += kWave) {
      w->fact[ndd + d - s] = g32(X.b, X.v.fact, d);
      w->fctr[ndd + d - s] = g64(X.b, X.v.fctr, d);
    }
  ndd += e - s;
  // member set: self's, other's (copied by the lanes), or — for a clock
  // present on both sides — the sorted union of both (lane 0, rare)
  if (c != 0) {
    const uint32_t ms = uni(run_begin(X.b, X.v.fmend, kx)), me = uni(g32(X.b, X.v.fmend, kx));
    if (w)
      for (uint32_t j = ms + lane; j < me; j += kWave) w->fkey[ndm + j - ms] = g64(X.b, X.v.fkey, j);
    ndm += me - ms;
  } else {
    uint32_t cnt = 0;
    if (lane == 0u) {
      uint32_t a = run_begin(L.b, L.v.fmend, k), ae = g32(L.b, L.v.fmend, k);
      uint32_t b = run_begin(R.b, R.v.fmend, l), be = g32(R.b, R.v.fmend, l);
      while (a < ae || b < be) {
        const uint64_t ka = a < ae ? g64(L.b, L.v.fkey, a) : ~0ull;
        const uint64_t kb = b < be ? g64(R.b, R.v.fkey, b) : ~0ull;
        uint64_t km;
        if (a < ae && (b >= be || ka < kb)) { km = ka; ++a; }
        else if (b < be && (a >= ae || kb < ka)) { km = kb; ++b; }
        else { km = ka; ++a; ++b; }
        if (w) w->fkey[ndm + cnt] = km;
        ++cnt;
      }
    }
    ndm += lane_of(cnt, 0);
  }
  if (w && lane == 0u) { w->fdend[nd] = ndd; w->fmend[nd] = ndm; }
  ++nd;
}

// The union walk. With `cache` (LDS, one u32 per survivor): a counting walk
// (w == nullptr) records each survivor as k | l << 8 | (c + 1) << 16, and a
// writing walk given the recorded count replays them without the clock
// compares and survival tests.
template <bool SP = false, class S = Side>
__device__ void deferred_pass_wave(const S& L, const S& R, uint32_t A, uint32_t lane, uint32_t& nd,
                                   uint32_t& ndd, uint32_t& ndm, const DefOut* w, uint32_t* cache = nullptr,
                                   uint32_t n_cached = 0) {
  if (w && cache) {
    nd = ndd = ndm = 0;
    for (uint32_t i = 0; i < n_cached; ++i) {
      const uint32_t e = cache[i];
      deferred_emit(L, R, (int)(e >> 16) - 1, e & 0xFFu, (e >> 8) & 0xFFu, lane, nd, ndd, ndm, w);
    }
    return;
  }
  uint32_t k = 0, l = 0;
  nd = ndd = ndm = 0;
  const uint32_t nfL = uni(L.v.n_def), nfR = uni(R.v.n_def);
  while (k < nfL || l < nfR) {
    const int c = k >= nfL ? 1 : (l >= nfR ? -1 : clock_cmp_wave(L, k, R, l, lane));
    const S& X = c <= 0 ? L : R;
    const uint32_t kx = c <= 0 ? k : l;
    if (def_survives_wave<SP>(X, kx, L, R, A, lane)) {
      if (cache && lane == 0u) cache[nd] = k | (l << 8) | ((uint32_t)(c + 1) << 16);
      deferred_emit(L, R, c, k, l, lane, nd, ndd, ndm, w);
    }
    if (c <= 0) ++k;
    if (c >= 0) ++l;
  }
}

__device__ __forceinline__ RecLayout layout_at(const uint8_t* rec) {
  const uint32_t* h = (const uint32_t*)rec;
  RecLayout L;
  rec_layout(L, uni(h[1]), uni(h[2]), uni(h[3]), uni(h[4]), uni(h[5]), uni(h[6]), (uni(h[7]) & kSparseClock) != 0u);
  return L;
}

// Sparse (CSR) top-clock join, src/orswot.rs:153 -> VClock::merge
// (src/vclock.rs:131-137): the sorted union of both actor lists, max on
// common actors. Counts the union (every lane gets it); with O != nullptr
// also writes ctr/act at O's clock section for a union of n_out entries.
template <class S>
__device__ __forceinline__ uint32_t sparse_clock_join(const S& L, const S& R, uint8_t* O, uint32_t n_out,
                                                      uint32_t lane) {
  // union index of actor x = #L acts < x + #R acts < x - #common acts < x;
  // the common count below an entry is a running wave prefix over its side.
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t common = 0;
  for (uint32_t base = 0; base < L.v.n_clk; base += kWave) {
    const uint32_t k = base + lane;
    const bool valid = k < L.v.n_clk;
    const uint32_t x = valid ? g32(L.b, L.v.cact, k) : 0u;
    const uint32_t r = valid ? clk_lower_bound(R.b, R.v, x) : 0u;
    const bool eq = valid && r < R.v.n_clk && g32(R.b, R.v.cact, r) == x;
    const uint64_t em = __ballot(eq);
    if (O && valid) {
      const uint32_t idx = k + r - (common + (uint32_t)__popcll(em & lt));
      const uint64_t a = g64(L.b, L.v.clk, k), c = eq ? g64(R.b, R.v.clk, r) : 0ull;
      ((uint64_t*)(O + kHdrBytes))[idx] = a > c ? a : c;
      ((uint32_t*)(O + kHdrBytes + 8u * n_out))[idx] = x;
    }
    common += (uint32_t)__popcll(em);
  }
  if (O) {
    uint32_t rc = 0;
    for (uint32_t base = 0; base < R.v.n_clk; base += kWave) {
      const uint32_t k = base + lane;
      const bool valid = k < R.v.n_clk;
      const uint32_t x = valid ? g32(R.b, R.v.cact, k) : 0u;
      const uint32_t l = valid ? clk_lower_bound(L.b, L.v, x) : 0u;
      const bool eq = valid && l < L.v.n_clk && g32(L.b, L.v.cact, l) == x;
      const uint64_t em = __ballot(eq);
      if (valid && !eq) {  // common actors were written by the self side
        const uint32_t idx = k + l - (rc + (uint32_t)__popcll(em & lt));
        ((uint64_t*)(O + kHdrBytes))[idx] = g64(R.b, R.v.clk, k);
        ((uint32_t*)(O + kHdrBytes + 8u * n_out))[idx] = x;
      }
      rc += (uint32_t)__popcll(em);
    }
  }
  return L.v.n_clk + R.v.n_clk - common;
}

// Join one object pair whose records sit at Ls / Rs (LDS stage or HBM) into
// the output record at O (HBM). SP: both records carry CSR top clocks (and
// so does the output).
template <bool SP = false>
__device__ __forceinline__ void merge_object(const uint8_t* Ls, const uint8_t* Rs, uint8_t* O, uint32_t A,
                                             uint32_t lane) {
  const RecLayout LL = layout_at(Ls), RL = layout_at(Rs);
  const Side L{Ls, make_rv(LL)}, R{Rs, make_rv(RL)};
  const bool has_def = (L.v.n_def | R.v.n_def) != 0;
  const uint32_t P = L.v.n_mem + R.v.n_mem;
  const uint32_t n_clk = SP ? uni(sparse_clock_join(L, R, nullptr, 0u, lane)) : A;

  // ---- pass 1: per-position join -> member / dot totals. For the first
  // two 64-wide chunks each lane keeps its candidate, count and first output
  // dot in registers for pass 2; later chunks are recomputed.
  uint32_t q0 = 0, c0 = 0, x0 = 0, q1 = 0, c1 = 0, x1 = 0;
  uint64_t v0 = 0, v1 = 0;
  uint32_t tot_mem = 0, tot_dot = 0;
  for (uint32_t base = 0; base < P; base += kWave) {
    const uint32_t p = base + lane;
    uint32_t type = kNone, i = 0, j = 0, cnt = 0, x = 0;
    uint64_t v = 0;
    if (p < P) {
      type = merge_path(L, R, p, i, j);
      if (type != kNone) cnt = join<0, SP>(L, R, type, i, j, A, has_def, x, v, nullptr, nullptr, 0);
    }
    const uint32_t q = (type << 30) | (i << 15) | j;
    if (base == 0) { q0 = q; c0 = cnt; x0 = x; v0 = v; }
    else if (base == kWave) { q1 = q; c1 = cnt; x1 = x; v1 = v; }
    tot_mem += (uint32_t)__popcll(__ballot(cnt != 0));
    tot_dot += wave_sum(cnt);
  }
  tot_mem = uni(tot_mem);
  tot_dot = uni(tot_dot);

  // ---- output member block (its offsets depend on the member totals only)
  const uint32_t o_key = kHdrBytes + clock_bytes(n_clk, SP);
  const uint32_t o_dctr = o_key + 8u * tot_mem;
  const uint32_t o_dact = o_dctr + 8u * tot_dot;
  const uint32_t o_mdend = o_dact + 4u * tot_dot;
  const uint32_t o_mpad = o_mdend + 4u * tot_mem;
  const uint32_t o_def = (o_mpad + 7u) & ~7u;
  uint64_t* okey = (uint64_t*)(O + o_key);
  uint64_t* odctr = (uint64_t*)(O + o_dctr);
  uint32_t* odact = (uint32_t*)(O + o_dact);
  uint32_t* omdend = (uint32_t*)(O + o_mdend);

  // top clock: pointwise max (src/orswot.rs:153 -> src/vclock.rs:131-137)
  if (SP) {
    sparse_clock_join(L, R, O, n_clk, lane);
    if (lane == 0u && (n_clk & 1u)) *(uint32_t*)(O + kHdrBytes + 12u * n_clk) = 0u;  // pad to 8
  } else {
    for (uint32_t a = lane; a < A; a += kWave) {
      const uint64_t x = g64(Ls, L.v.clk, a), y = g64(Rs, R.v.clk, a);
      ((uint64_t*)(O + kHdrBytes))[a] = x > y ? x : y;
    }
  }

  // ---- pass 2: write kept members and their joined dot runs
  uint32_t mem_base = 0, dot_base = 0;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (uint32_t base = 0; base < P; base += kWave) {
    const uint32_t p = base + lane;
    // (cached chunks: positions < 128, so i, j fit the 15-bit fields of q;
    // later chunks keep i, j whole — a side may hold 32 768+ members)
    uint32_t type = kNone, i = 0, j = 0, cnt = 0, x = 0;
    uint64_t v = 0;
    if (base < 2u * kWave) {
      const uint32_t q = base == 0 ? q0 : q1;
      cnt = base == 0 ? c0 : c1; x = base == 0 ? x0 : x1; v = base == 0 ? v0 : v1;
      type = q >> 30; i = (q >> 15) & 0x7FFFu; j = q & 0x7FFFu;
    } else if (p < P) {
      type = merge_path(L, R, p, i, j);
      if (type != kNone) cnt = join<0, SP>(L, R, type, i, j, A, has_def, x, v, nullptr, nullptr, 0);
    }
    const uint64_t keep = __ballot(cnt != 0);
    const uint32_t incl = wave_incl_scan(cnt, lane);
    if (cnt != 0) {
      const uint32_t midx = mem_base + (uint32_t)__popcll(keep & lt_mask);
      const uint32_t d0 = dot_base + incl - cnt;
      okey[midx] = (type & kSelf) ? g64(Ls, L.v.key, i) : g64(Rs, R.v.key, j);
      if (cnt == 1) {
        odact[d0] = x;
        odctr[d0] = v;
      } else {
        join<1, SP>(L, R, type, i, j, A, has_def, x, v, odact, odctr, d0);
      }
      omdend[midx] = d0 + cnt;
    }
    mem_base += (uint32_t)__popcll(keep);
    dot_base += __shfl(incl, kWave - 1, kWave);
  }

  // ---- deferred block + header + padding (lane 0)
  if (lane == 0) {
    uint32_t nd = 0, ndd = 0, ndm = 0;
    if (o_def != o_mpad) *(uint32_t*)(O + o_mpad) = 0u;
    if (has_def) {
      deferred_pass<SP>(L, R, A, nd, ndd, ndm, nullptr);
      RecLayout OL;
      rec_layout(OL, n_clk, tot_mem, tot_dot, nd, ndd, ndm, SP);
      DefOut w{(uint64_t*)(O + OL.o_fctr), (uint64_t*)(O + OL.o_fkey), (uint32_t*)(O + OL.o_fact),
               (uint32_t*)(O + OL.o_fdend), (uint32_t*)(O + OL.o_fmend)};
      deferred_pass<SP>(L, R, A, nd, ndd, ndm, &w);
    }
    RecLayout OL;
    rec_layout(OL, n_clk, tot_mem, tot_dot, nd, ndd, ndm, SP);
    for (uint32_t b = OL.o_end; b < OL.size; b += 4) *(uint32_t*)(O + b) = 0u;
    u32x4* h = (u32x4*)O;
    h[0] = u32x4{OL.size, n_clk, tot_mem, tot_dot};
    h[1] = u32x4{nd, ndd, ndm, SP ? kSparseClock : 0u};
  }
}

// Header sanity for a record of the batch: size matches the counts, the
// top-clock width is the batch's, flags are clear, it lies in the buffer.
__device__ __forceinline__ bool header_ok(u32x4 h0, u32x4 h1, uint64_t off, uint64_t bytes, uint32_t A) {
  const uint64_t sz = record_size64(h0.y, h0.z, h0.w, h1.x, h1.y, h1.z);
  return (off & 15u) == 0 && off + kHdrBytes <= bytes && sz == h0.x && h0.y == A && h1.w == 0u &&
         (h1.x != 0u || (h1.y | h1.z) == 0u) && off + sz <= bytes;
}

// ======================================================================
// Fast path: objects whose records fit the LDS stage, with at most 32
// deferred clocks per side, and whose merge has at most 128 union positions
// (two 64-wide chunks) — all of config 3. Same rules as merge_object, written
// for the issue rate: every LDS load is unconditional (indices clamped or
// garbage-then-selected: LDS reads never fault), selects instead of branches,
// DPP wave scans, and all per-position state stays in registers between the
// count and the write pass.
// ======================================================================
constexpr uint32_t kFastStage = 2048;                 // LDS stage per input record per wave
constexpr uint32_t kOutStage = 3072;                  // LDS stage for the output record per wave (4 blocks/CU at 40 KB)
constexpr uint32_t kPer = kFastStage / 16 / kWave;    // 16-B pieces per lane per record
constexpr uint64_t kPending = 1ull << 63;             // Ooff flag: object left for the general kernel

// Wave-wide inclusive prefix sum: DPP row shifts then row broadcasts (gfx9).
__device__ __forceinline__ uint32_t scan_incl(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ uint64_t ld64(const uint8_t* b, uint32_t off) { return *(const uint64_t*)(b + off); }
__device__ __forceinline__ uint32_t ld32(const uint8_t* b, uint32_t off) { return *(const uint32_t*)(b + off); }

// One staged record: LDS base and (wave-uniform) section offsets.
struct FSide {
  const uint8_t* b;
  uint32_t n, key, ctr, act, end;
};

__device__ __forceinline__ FSide fside(const uint8_t* b, uint32_t A, uint32_t n_mem, uint32_t n_dot) {
  FSide s;
  s.b = b;
  s.n = n_mem;
  s.key = kHdrBytes + 8u * A;
  s.ctr = s.key + 8u * n_mem;
  s.act = s.ctr + 8u * n_dot;
  s.end = s.act + 4u * n_dot;
  return s;
}

// Merge path at union position p (p <= nL + nR), branch-free: i = the
// number of self keys among the first p union positions = the first mid in
// [lo, hi] with !(L[mid] <= R[p-1-mid]); found with wave-uniform power-of-two
// steps (`top` = the largest power of two <= min(nL, nR), or 0).
__device__ __forceinline__ uint32_t fpath(const FSide& L, const FSide& R, uint32_t p, uint32_t top, uint32_t& i,
                                          uint32_t& j) {
  const uint32_t lo = p > R.n ? p - R.n : 0u;
  const uint32_t hi = p < L.n ? p : L.n;
  uint32_t base = lo;
  for (uint32_t step = top; step != 0u; step >>= 1) {
    const uint32_t cand = base + step;  // test mid = cand - 1
    const uint64_t kl = ld64(L.b, L.key + 8u * cand - 8u), kr = ld64(R.b, R.key + 8u * (p - cand));
    base = (cand <= hi && kl <= kr) ? cand : base;
  }
  i = base;
  j = p - base;
  const uint64_t kl = ld64(L.b, L.key + 8u * i), kr = ld64(R.b, R.key + 8u * j);
  const uint64_t kp = ld64(L.b, L.key + 8u * i - 8u);
  const bool hl = i < L.n, hr = j < R.n;
  if (hl && (!hr || kl <= kr)) return (hr && kl == kr) ? kBoth : kSelf;
  return (i > 0u && hr && kp == kr) ? kNone : kOther;
}

// Deferred removes on the fast path (objects with any, ~10 % in config 3):
// bit k (k < 32) / 32+k of the mask says deferred clock k of self / other
// lists this member, so each output dot is checked only against those
// clocks (apply_remove via apply_deferred, src/orswot.rs:195-211, 235-243).
template <class S>
__device__ __forceinline__ uint64_t dmask_of(const S& DL, const S& DR, uint64_t m) {
  uint64_t mask = 0;
  for (uint32_t k = 0; k < DL.v.n_def; ++k) mask |= def_has_member(DL, k, m) ? (1ull << k) : 0ull;
  for (uint32_t k = 0; k < DR.v.n_def; ++k) mask |= def_has_member(DR, k, m) ? (1ull << (32 + k)) : 0ull;
  return mask;
}

template <class S>
__device__ __forceinline__ bool dkilled(const S& DL, const S& DR, uint64_t mask, uint32_t x, uint64_t v) {
  for (; mask; mask &= mask - 1) {
    const uint32_t k = (uint32_t)__builtin_ctzll(mask);
    if ((k < 32 ? def_get(DL, k, x) : def_get(DR, k - 32, x)) >= v) return true;
  }
  return false;
}

// Joined dot run of one member (rules of join<> above / src/orswot.rs:94-138).
// COUNT: returns the run length and captures the first two dots in (x0, v0),
// (x1, v1);
// WRITE: stores the run at oact/octr[d0..] (the entry is known to survive).
template <bool WRITE, bool HD>
__device__ __forceinline__ uint32_t fjoin(const FSide& L, const FSide& R, uint32_t A, uint32_t type, uint32_t i,
                                          uint32_t j, uint32_t& x0, uint64_t& v0, uint32_t& x1, uint64_t& v1,
                                          uint32_t* oact, uint64_t* octr, uint32_t d0, uint64_t dmask, const Side& DL,
                                          const Side& DR) {
  const bool hs = (type & kSelf) != 0u, ho = (type & kOther) != 0u, self_only = type == kSelf;
  const uint32_t ab = ld32(L.b, L.end + 4u * i - 4u), ae_ = ld32(L.b, L.end + 4u * i);
  const uint32_t bb = ld32(R.b, R.end + 4u * j - 4u), be_ = ld32(R.b, R.end + 4u * j);
  uint32_t a = hs && i ? ab : 0u, ae = hs ? ae_ : 0u;
  uint32_t b = ho && j ? bb : 0u, be = ho ? be_ : 0u;
  bool any = false;
  uint32_t c = 0;
  while (a < ae || b < be) {
    const uint32_t xa_ = ld32(L.b, L.act + 4u * a), xb_ = ld32(R.b, R.act + 4u * b);
    const uint64_t va = ld64(L.b, L.ctr + 8u * a), vb = ld64(R.b, R.ctr + 8u * b);
    const uint32_t xa = a < ae ? xa_ : 0xFFFFFFFFu, xb = b < be ? xb_ : 0xFFFFFFFFu;
    const bool ta = xa <= xb, tb = xb <= xa;
    const uint32_t x = ta ? xa : xb;
    const bool in = x < A;
    const uint32_t xo = kHdrBytes + 8u * (in ? x : 0u);
    const uint64_t rc_ = ld64(R.b, xo), lc_ = ld64(L.b, xo);
    const uint64_t rc = in ? rc_ : 0ull, lc = in ? lc_ : 0ull;
    any = any || (self_only && ta && va > rc);
    const uint64_t lp = (ta && (self_only || va > rc)) ? va : 0ull;
    const uint64_t rp = (tb && vb > lc) ? vb : 0ull;
    uint64_t v = (ta && tb && va == vb) ? va : (lp > rp ? lp : rp);
    a += ta ? 1u : 0u;
    b += tb ? 1u : 0u;
    if (HD && v != 0ull && dmask != 0ull && dkilled(DL, DR, dmask, x, v)) v = 0ull;
    const bool keep = v != 0ull;
    if (WRITE) {
      if (keep) {
        oact[d0 + c] = x;
        octr[d0 + c] = v;
      }
    } else {
      const bool first = keep && c == 0u, second = keep && c == 1u;
      x0 = first ? x : x0;
      v0 = first ? v : v0;
      x1 = second ? x : x1;
      v1 = second ? v : v1;
    }
    c += keep ? 1u : 0u;
  }
  if (!WRITE && self_only && !any) c = 0u;  // self-only entry dropped as a whole (:98-100)
  return c;
}

template <bool HD>
__device__ __forceinline__ void fwrite_member(const FSide& L, const FSide& R, uint32_t A, uint32_t q, uint32_t cnt,
                                              uint32_t x, uint64_t v, uint32_t xb, uint64_t vb, uint32_t midx,
                                              uint32_t d0, uint64_t* okey, uint32_t* odact, uint64_t* odctr,
                                              uint32_t* omdend, uint64_t dmask, const Side& DL, const Side& DR) {
  const uint32_t type = q >> 30, i = (q >> 15) & 0x7FFFu, j = q & 0x7FFFu;
  const uint64_t kl = ld64(L.b, L.key + 8u * i), kr = ld64(R.b, R.key + 8u * j);
  okey[midx] = (type & kSelf) ? kl : kr;
  if (cnt <= 2u) {
    odact[d0] = x;
    odctr[d0] = v;
    if (cnt == 2u) {
      odact[d0 + 1] = xb;
      odctr[d0 + 1] = vb;
    }
  } else {
    fjoin<true, HD>(L, R, A, type, i, j, x, v, xb, vb, odact, odctr, d0, dmask, DL, DR);
  }
  omdend[midx] = d0 + cnt;
}

// Record-wide section offsets of a staged record (general accessor form),
// used for its deferred block.
__device__ __forceinline__ Side side_of(const uint8_t* b) { return Side{b, make_rv(layout_at(b))}; }

// HD: the object has deferred removes (either side; <= 32 clocks per side).
// ABL (ablation builds for timing only; outputs are NOT valid): 1 = stage
// only, 2 = + merge path, 3 = + counting join, 0 = the real kernel.
// Where a fast-path object's output goes: built in the wave's LDS output
// stage `Os`, then copied to `Og` in HBM with 16-B coalesced stores. An
// output larger than the stage is handed to the general kernel instead.
struct FOut {
  u32x4* Os;
  uint8_t* Og;
  uint64_t obj;
  uint64_t* Ooff;
  uint32_t* ctl;
  uint64_t* list;
  uint32_t list_cap;
};

// Returns the output record's size in 16-B pieces (built in fo.Os; the caller
// copies it to fo.Og later), or 0 if nothing is left to copy.
// OUTCAP: bytes of the output stage. GEN (general kernel): an output larger
// than the stage returns ~0u instead of flagging the object.
template <bool HD, int ABL, uint32_t OUTCAP = kOutStage, bool GEN = false>
__device__ __forceinline__ uint32_t fast_object(const uint8_t* Ls, const uint8_t* Rs, const FOut& fo, uint32_t A,
                                            uint32_t nL, uint32_t dL, uint32_t nR, uint32_t dR, uint32_t lane,
                                            Stamps& st) {
  if (ABL == 1) {
    if (lane == 0) *(u32x4*)fo.Og = u32x4{ld32(Ls, 4), ld32(Rs, 4), nL, nR};
    return 0u;
  }
  const FSide L = fside(Ls, A, nL, dL), R = fside(Rs, A, nR, dR);
  Side DL{Ls, RV{}}, DR{Rs, RV{}};
  if (HD) { DL = side_of(Ls); DR = side_of(Rs); }
  const uint32_t P = nL + nR;
  const uint32_t mn = nL < nR ? nL : nR;
  const uint32_t top = mn ? 1u << (31u - __builtin_clz(mn)) : 0u;
  // chunk 0: positions 0..63
  uint32_t i = 0, j = 0, x0 = 0, y0 = 0, c0 = 0, q0 = 0;
  uint64_t v0 = 0, w0 = 0, m0k = 0;
  {
    const uint32_t p = lane < P ? lane : P;
    uint32_t type = fpath(L, R, p, top, i, j);
    type = lane < P ? type : kNone;
    if (HD && type != kNone) m0k = dmask_of(DL, DR, (type & kSelf) ? ld64(Ls, L.key + 8u * i) : ld64(Rs, R.key + 8u * j));
    mark<ABL>(st, 2);
    if (ABL != 2) c0 = fjoin<false, HD>(L, R, A, type, i, j, x0, v0, y0, w0, nullptr, nullptr, 0u, m0k, DL, DR);
    q0 = (type << 30) | (i << 15) | j;
    mark<ABL>(st, 3);
  }
  // chunk 1: positions 64..127 (P <= 128 on this path)
  uint32_t x1 = 0, y1 = 0, c1 = 0, q1 = 0;
  uint64_t v1 = 0, w1 = 0, m1k = 0;
  if (P > (uint32_t)kWave) {
    const uint32_t p = lane + kWave < P ? lane + kWave : P;
    uint32_t type = fpath(L, R, p, top, i, j);
    type = lane + kWave < P ? type : kNone;
    if (HD && type != kNone) m1k = dmask_of(DL, DR, (type & kSelf) ? ld64(Ls, L.key + 8u * i) : ld64(Rs, R.key + 8u * j));
    mark<ABL>(st, 2);
    if (ABL != 2) c1 = fjoin<false, HD>(L, R, A, type, i, j, x1, v1, y1, w1, nullptr, nullptr, 0u, m1k, DL, DR);
    q1 = (type << 30) | (i << 15) | j;
    mark<ABL>(st, 3);
  }
  if (ABL == 2 || ABL == 3) {  // keep the phase's results live, skip the writes
    const uint32_t k = q0 + q1 + c0 + c1 + x0 + x1 + y0 + y1 + (uint32_t)(v0 ^ v1 ^ w0 ^ w1);
    if (__ballot(k == 0x12345u) != 0ull && lane == 0) *(uint32_t*)fo.Og = k;
    if (lane == 0) *(u32x4*)fo.Og = u32x4{nL, nR, 0u, 0u};
    return 0u;
  }
  const uint32_t inc0 = scan_incl(c0), inc1 = scan_incl(c1);
  const uint64_t k0 = __ballot(c0 != 0u), k1 = __ballot(c1 != 0u);
  const uint32_t tot0 = lane_of(inc0, kWave - 1), tot1 = lane_of(inc1, kWave - 1);
  const uint32_t m0 = (uint32_t)__popcll(k0);
  const uint32_t tot_mem = m0 + (uint32_t)__popcll(k1), tot_dot = tot0 + tot1;

  // deferred counts first (lane 0), so the output size is known up front
  uint32_t nd = 0, ndd = 0, ndm = 0;
  if (HD) deferred_pass_wave(DL, DR, A, lane, nd, ndd, ndm, nullptr);
  RecLayout OL;
  rec_layout(OL, A, tot_mem, tot_dot, nd, ndd, ndm);
  mark<ABL>(st, 4);
  if (OL.size > OUTCAP) {  // rare: let the general kernel write it
    if (GEN) return ~0u;
    if (lane == 0u) {
      fo.Ooff[fo.obj] |= kPending;
      const uint32_t e = atomicAdd(&fo.ctl[0], 1u);
      if (e < fo.list_cap) fo.list[e] = fo.obj;
    }
    return 0u;
  }
  uint8_t* O = (uint8_t*)fo.Os;
  uint64_t* okey = (uint64_t*)(O + OL.o_key);
  uint64_t* odctr = (uint64_t*)(O + OL.o_dctr);
  uint32_t* odact = (uint32_t*)(O + OL.o_dact);
  uint32_t* omdend = (uint32_t*)(O + OL.o_mdend);

  wave_sync();  // the copy-out of the object that last used this stage has read it
  // top clock: pointwise max (src/orswot.rs:153 -> src/vclock.rs:131-137)
  for (uint32_t a = lane; a < A; a += kWave) {
    const uint64_t x = ld64(Ls, kHdrBytes + 8u * a), y = ld64(Rs, kHdrBytes + 8u * a);
    ((uint64_t*)(O + kHdrBytes))[a] = x > y ? x : y;
  }
  const uint64_t lt = (1ull << lane) - 1ull;
  if (c0 != 0u)
    fwrite_member<HD>(L, R, A, q0, c0, x0, v0, y0, w0, (uint32_t)__popcll(k0 & lt), inc0 - c0, okey, odact, odctr,
                      omdend, m0k, DL, DR);
  if (c1 != 0u)
    fwrite_member<HD>(L, R, A, q1, c1, x1, v1, y1, w1, m0 + (uint32_t)__popcll(k1 & lt), tot0 + inc1 - c1, okey,
                      odact, odctr, omdend, m1k, DL, DR);
  if (HD) {
    // deferred union keyed by clock (:141-148), kept iff !(D <= clock) (:197)
    DefOut w{(uint64_t*)(O + OL.o_fctr), (uint64_t*)(O + OL.o_fkey), (uint32_t*)(O + OL.o_fact),
             (uint32_t*)(O + OL.o_fdend), (uint32_t*)(O + OL.o_fmend)};
    deferred_pass_wave(DL, DR, A, lane, nd, ndd, ndm, &w);
  }
  if (lane == 0u) {
    if (OL.o_def != OL.o_mpad) *(uint32_t*)(O + OL.o_mpad) = 0u;
    for (uint32_t b = OL.o_end; b < OL.size; b += 4) *(uint32_t*)(O + b) = 0u;
    u32x4* h = (u32x4*)O;
    h[0] = u32x4{OL.size, A, tot_mem, tot_dot};
    h[1] = u32x4{nd, ndd, ndm, 0u};
  }
  mark<ABL>(st, 5);
  return OL.size / 16u;
}

// Returned by a fast join when the object is outside its limits.
constexpr uint32_t kLeanFallback = 0xFFFFFFFFu;



// ======================================================================
// Mask path (v6): objects without deferred removes, A <= 32 actors, at most
// 64 members and 64 dots per side and 64 union members (all of config 3 but
// the ~7 % with deferred removes). Loop-free rework of the join for the
// VALU issue rate, with the same rules as merge_object:
//  1. dot-parallel pass per side: the member of each dot (run-head flags +
//     mbcnt), its actor / counter kept in registers, and LDS atomic ORs
//     building per member a 32-bit actor mask and a "survives" mask (the
//     dot's counter is above the OTHER side's pre-merge top clock);
//  2. member alignment by rank: every self member binary-searches its key
//     among the other side's keys and vice versa; the union position is
//     rank arithmetic (no merge-path twins, no scan);
//  3. one dot-parallel pass over the other side's dots records, for actors
//     present on both sides of a shared member, "equal" and "self >= other";
//  4. per union member the join is pure mask logic (src/orswot.rs:94-138):
//       lp = ML & (self_only ? ~0 : FL)   rp = MR & FR
//       useA = (ML & MR & EQ) | (lp & (~rp | GE))   keep = useA | rp
//     (self-only entries dropped as a whole iff ML & FL == 0, :98-103);
//  5. every kept dot writes itself at its member's output base + the rank
//     of its actor in the keep mask — no per-member loop anywhere.
// Scratch: kMask1Scratch bytes of LDS per wave. Returns output 16-B pieces,
// or kLeanFallback (union > 64 members, or an actor id >= 32).
// ======================================================================
// LDS hand-off between lanes of one wave with every LDS op drained (lgkmcnt(0)).
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t below(uint32_t mask, uint32_t x) { return __popc(mask & ((1u << x) - 1u)); }

// Both member-alignment ranks in one loop (the two searches' LDS round trips
// overlap): rl = # other keys < kl, rr = # self keys < kr.
__device__ __forceinline__ void rank_both(const uint8_t* Ls, const uint8_t* Rs, uint32_t key, uint32_t nL,
                                          uint32_t nR, uint64_t kl, uint64_t kr, uint32_t& rl, uint32_t& rr) {
  const uint32_t n = nL > nR ? nL : nR;
  uint32_t bl = 0, br = 0;
  for (uint32_t step = n ? 1u << (31u - __builtin_clz(n)) : 0u; step != 0u; step >>= 1) {
    const uint32_t cl = bl + step, cr = br + step;
    const uint64_t kcl = ld64(Rs, key + 8u * (cl - 1u)), kcr = ld64(Ls, key + 8u * (cr - 1u));
    bl = (cl <= nR && kcl < kl) ? cl : bl;
    br = (cr <= nL && kcr < kr) ? cr : br;
  }
  rl = bl;
  rr = br;
}

// #keys of the sorted list at `off` (n of them, n <= 64) strictly below k.
__device__ __forceinline__ uint32_t rank_below(const uint8_t* b, uint32_t off, uint32_t n, uint64_t k) {
  uint32_t base = 0;
  for (uint32_t step = n ? 1u << (31u - __builtin_clz(n)) : 0u; step != 0u; step >>= 1) {  // binary lifting
    const uint32_t cand = base + step;
    const uint64_t kc = ld64(b, off + 8u * (cand - 1u));  // garbage beyond n, masked by cand <= n
    base = (cand <= n && kc < k) ? cand : base;
  }
  return base;
}

#ifdef CRDT_DIAG
#include "diag/orswot_mask_diag.inc"  // mask_object (the v6 join): diagnostic kernels only
#endif


// ======================================================================
// Mask path v8 (mask3_object): mask_object's join for objects without
// deferred removes, rewritten for the instruction count. Same rules
// (src/orswot.rs:94-138) and same output bytes; what changed:
//  - every LDS access is a raw 32-bit LDS address kept in a VGPR (no
//    generic-pointer arithmetic per access);
//  - the rank searches clamp their probe address instead of testing the
//    bound (a probe past the other list reads its last key: if that key is
//    below, the rank is that list's length anyway), so a step is add / min
//    / read / compare / select;
//  - ballots come straight from the compares (one v_cmp into an SGPR pair)
//    and every lane-conditional value is a select on such a mask: no
//    divergent branches before the output stores;
//  - the run-head flags of both sides are ds_permute scatters (lanes that
//    own no member send to lane 0, which always starts a run), not LDS
//    stores + loads;
//  - values the next phase needs from another lane (the other side's top
//    clock at a dot's actor, a run start, a member's partner / union slot)
//    are ds_bpermute gathers from registers;
//  - the union descriptor is one u16 per union slot (L index + 1 | R index
//    + 1 << 8): both sides store their byte, shared keys land in one slot.
// LDS scratch (per wave, k3Scratch bytes): msL / msR member masks (the
// output table overlays them once read), equal/>= masks by union slot, the
// union descriptors, a per-lane sink for the atomics of lanes with nothing
// to add. Returns the output's 16-B pieces, or kLeanFallback (a dot actor
// >= A, or a union of more than 64 members).
// ======================================================================
constexpr uint32_t k3Desc = 1536, k3Trash = 1664;  // (the rest of mask3's layout: M3Lay)
constexpr uint32_t k3Scratch = 2176;  // <= kMask1Scratch: the kernel's scratch also serves mask_object
constexpr uint32_t k3DefMask = k3Scratch;  // u32 [64] (HK 1): actor mask per deferred clock
static_assert(k3DefMask + 256u <= 2560u, "the deferred clock masks fit in the wave's scratch");

typedef const __attribute__((address_space(3))) uint64_t lds_cu64;
typedef const __attribute__((address_space(3))) uint32_t lds_cu32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ uint64_t lr64(uint32_t a) { return *(lds_cu64*)(size_t)a; }
__device__ __forceinline__ uint32_t lr32(uint32_t a) { return *(lds_cu32*)(size_t)a; }
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p;
}
// ballots of compares: one v_cmp writing the wave mask (LLVM icmp predicates)
constexpr int kEQ = 32, kNE = 33, kUGT = 34, kUGE = 35;
template <int P>
__device__ __forceinline__ uint64_t cmp64(uint64_t a, uint64_t b) {
  return __builtin_amdgcn_uicmpl(a, b, P);
}
template <int P>
__device__ __forceinline__ uint64_t cmp32(uint32_t a, uint32_t b) {
  return __builtin_amdgcn_uicmp(a, b, P);
}
// this lane's bit of a wave mask, used straight as the select condition (no VALU)
__device__ __forceinline__ bool bit_of(uint64_t m, uint32_t) { return __builtin_amdgcn_inverse_ballot_w64(m); }
__device__ __forceinline__ uint64_t lanes_below(uint32_t n) { return n >= 64u ? ~0ull : (1ull << n) - 1ull; }
__device__ __forceinline__ uint32_t gather32(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}
__device__ __forceinline__ uint64_t gather64(uint64_t v, uint32_t src_lane) {
  return ((uint64_t)gather32((uint32_t)(v >> 32), src_lane) << 32) | gather32((uint32_t)v, src_lane);
}
// lane k's value moved to lane k + 1 (lane 0 gets 0): DPP wave_shr:1 (gfx9)
__device__ __forceinline__ uint32_t shift_up1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// Copy an LDS-assembled record of n16 16-B pieces (1 <= n16 <= 128) to HBM:
// two stores per lane, always; lanes past the record repeat its last piece
// (the same bytes to the same address), so no lane needs a branch or a sink.
// After a fallback the caller passes n16 = 1: piece 0 of the object's output
// region gets garbage that the general kernel overwrites.
__device__ __forceinline__ void copy_record_out(uint32_t src, uint8_t* O, uint32_t n16, uint32_t lane) {
  const uint32_t i0 = lane < n16 ? lane : n16 - 1u, i1 = lane + kWave < n16 ? lane + kWave : n16 - 1u;
  const u32x4 p0 = *(const __attribute__((address_space(3))) u32x4*)(size_t)(src + 16u * i0);
  const u32x4 p1 = *(const __attribute__((address_space(3))) u32x4*)(size_t)(src + 16u * i1);
  __builtin_nontemporal_store(p0, (u32x4*)(O + 16u * i0));
  __builtin_nontemporal_store(p1, (u32x4*)(O + 16u * i1));
}

// mask3_object's per-wave scratch by actor-mask width: {actor mask, survives
// mask} per member of each side, {equal, >=} per union slot, the union
// descriptors and the sink (BK layout). Out ({keep, useK} by union slot, the
// deferred-remove objects) overlays the member masks once they are read.
template <int AW> struct M3Lay;
template <> struct M3Lay<32> {
  using MT = uint32_t;
  static constexpr uint32_t MsL = 0, MsR = 512, Out = 0, EqGe = 1024, Desc = 1536, TrBK = 1792;
  static constexpr uint32_t Bytes = 2560;  // == kMask1Scratch
};
template <> struct M3Lay<64> {
  using MT = uint64_t;
  static constexpr uint32_t MsL = 0, MsR = 1024, Out = 0, EqGe = 2048, Desc = 3072, TrBK = 3328;
  static constexpr uint32_t Bytes = 3840;
};

// HD (with OUT 0 only): objects with deferred removes — kept dots that a
// deferred clock listing their member covers are cleared from the keep masks
// (apply_deferred -> apply_remove, src/orswot.rs:235-243, :195-211) and the
// deferred block (the union of both deferred maps in CLOCK ORDER, kept iff
// !(D <= merged clock), :141-148, :197) is written after the member block.
__device__ __forceinline__ const uint8_t* gptr(uint32_t a) {
  return (const uint8_t*)(const __attribute__((address_space(3))) uint8_t*)(size_t)a;
}
// RT: member ranks searched in padded key tables (else clamped probes of the stage)
// HK (with HD): 1 = the kill pass finds a deferred member's union slot by one
// search of a union key table and a clock's D[x] by its actor presence mask
// PK: objects with nL + nR <= 64 members search both sides' ranks in ONE
// 64-lane pass (L members in lanes [0, nL), R members in [nL, nL + nR)), half
// the search instructions of the two-sided form
template <uint32_t OUTCAP, int OUT = 0, bool HD = false, int HABL = 0, bool RT = true, int HK = 0, bool PK = false,
          int BK = 0, int AW = 32>  // OUT: 0 direct stores, 1 sink-predicated, 2 LDS-assembled; AW: actor mask bits
__device__ __forceinline__ uint32_t mask3_object(uint32_t uL, uint32_t uR, uint32_t uX, uint8_t* O, uint32_t A,
                                                 uint32_t nL, uint32_t dL, uint32_t nR, uint32_t dR, uint32_t lane,
                                                 bool& big, uint8_t* sink = nullptr) {
#ifndef CRDT_DIAG
  static_assert(HABL == 0, "timing-only ablations (HABL != 0) exist in -DCRDT_DIAG builds only");
#endif
  // BK: LDS bank conflicts — union descriptors one dword per slot (L index in
  // byte 0, R index in byte 1: no two lanes' byte stores share a dword), the
  // sink moved past them, 4-byte sink stores at a 4-byte lane stride (an
  // 8-byte stride put two lanes in every bank), the header written under exec
  static_assert(!(BK && HK == 1), "BK moves the sink over HK 1's deferred clock masks");
  constexpr uint32_t TR = BK ? 1792u : k3Trash;  // the wave's sink (512 B)
  constexpr uint32_t DS = BK ? 4u : 2u;          // bytes per union descriptor
  static_assert(!BK || TR >= k3Desc + 256u, "BK descriptors: 64 dwords before the sink");
  // AW 64 (dense top clocks of 33-64 actors): 64-bit actor masks, the mask
  // tables twice as wide (M3Lay<64>), the BK layout only
  static_assert(AW == 32 || (AW == 64 && BK && HK == 0), "AW 64: the product's BK form");
  using MT = typename M3Lay<AW>::MT;
  constexpr uint32_t MsL = M3Lay<AW>::MsL, MsR = M3Lay<AW>::MsR, EqGe = M3Lay<AW>::EqGe, Desc = M3Lay<AW>::Desc;
  constexpr uint32_t Out = M3Lay<AW>::Out, MW = sizeof(MT), ME = 2u * MW;  // mask word, {mask, mask} entry
  constexpr uint32_t TRW = AW == 64 ? M3Lay<AW>::TrBK : TR;  // the wave's sink
  big = false;
  const uint32_t key = kHdrBytes + 8u * A;
  const uint32_t ctrL = key + 8u * nL, actL = ctrL + 8u * dL, endL = actL + 4u * dL;
  const uint32_t ctrR = key + 8u * nR, actR = ctrR + 8u * dR, endR = actR + 4u * dR;
  const uint32_t l4 = 4u * lane, l8 = 8u * lane;
  const uint64_t mnL = lanes_below(nL), mnR = lanes_below(nR), mdL = lanes_below(dL), mdR = lanes_below(dR);

  // ---- every lane-indexed element of both records: dots (actor, counter),
  // member keys and run ends, top-clock entries (all loads independent)
  const uint32_t xl = lr32(uL + actL + l4), xr = lr32(uR + actR + l4);
  const uint64_t vl = lr64(uL + ctrL + l8), vr = lr64(uR + ctrR + l8);
  const uint64_t kl = lr64(uL + key + l8), kr = lr64(uR + key + l8);
  const uint32_t el = lr32(uL + endL + l4), er = lr32(uR + endR + l4);
  const uint64_t tl = lr64(uL + kHdrBytes + l8), tr = lr64(uR + kHdrBytes + l8);  // lane a: actor a's counter
  // fallback: a dot actor >= A (here) or a union past 64 members (below).
  // With OUT != 0 the join runs on (every access stays in the wave's scratch /
  // 64-lane ranges) and only its stores go to the sink, so that every object
  // issues the same stores; otherwise it returns at once.
  bool fb = ((cmp32<kUGE>(xl, A) & mdL) | (cmp32<kUGE>(xr, A) & mdR)) != 0ull;
  if (OUT == 0 && fb) return kLeanFallback;

  // ---- member alignment by rank (self first on equal keys): L lanes count
  // R keys < kl, R lanes count L keys < kr; probe address = key[b - 1]
  const uint32_t rk0 = uR + key - 8u, rkmax = uR + key + 8u * nR - 8u;
  const uint32_t lk0 = uL + key - 8u, lkmax = uL + key + 8u * nL - 8u;
  uint32_t rl, rr;  // # R keys < kl, # L keys < kr
  uint64_t EL, ER;
  if (RT) {
    // both key lists copied into 64-slot tables padded with ~0 (in the mask
    // scratch, dead until the masks are zeroed below): the probes need no
    // bound, and every probe address is the lane's position + an immediate
    const uint32_t tL = uX + MsL, tR = uX + MsR;
    *(lds_u64*)(size_t)(tL + l8) = bit_of(mnL, lane) ? kl : ~0ull;
    *(lds_u64*)(size_t)(tR + l8) = bit_of(mnR, lane) ? kr : ~0ull;
    wave_sync();
    const uint32_t n = nL > nR ? nL : nR;
    if (PK && nL + nR <= (uint32_t)kWave) {
      // lane i < nL: L member i (searches tR); nL <= lane < nL + nR: R member
      // lane - nL (searches tL); the rest search tR for ~0 (masked out)
      const bool isR = lane >= nL;
      const uint64_t k = isR ? lr64(tR + 8u * ((lane - nL) & 63u)) : kl;
      const uint32_t t0 = isR ? tL : tR;
      uint32_t q = t0;
      if (n >= 64u) q = lr64(q + 504u) < k ? q + 512u : q;
      if (n >= 32u) q = lr64(q + 248u) < k ? q + 256u : q;
#pragma unroll
      for (uint32_t step = 128u; step >= 8u; step >>= 1) q = lr64(q + step - 8u) < k ? q + step : q;
      const uint32_t r = (q - t0) >> 3;
      const uint64_t E = cmp64<kEQ>(lr64(q), k) & cmp32<kUGT>(isR ? nL : nR, r) & lanes_below(nL + nR);
      rl = r;
      rr = gather32(r, (nL + lane) & 63u);
      EL = E & mnL;
      ER = nL < 64u ? (E >> nL) & mnR : 0ull;
    } else {
    uint32_t ql = tR, qr = tL;  // address of the first key not known to be below the lane's key
    if (n >= 64u) {
      ql = lr64(ql + 504u) < kl ? ql + 512u : ql;
      qr = lr64(qr + 504u) < kr ? qr + 512u : qr;
    }
    if (n >= 32u) {
      ql = lr64(ql + 248u) < kl ? ql + 256u : ql;
      qr = lr64(qr + 248u) < kr ? qr + 256u : qr;
    }
#pragma unroll
    for (uint32_t step = 128u; step >= 8u; step >>= 1) {
      const uint64_t a = lr64(ql + step - 8u), b = lr64(qr + step - 8u);
      ql = a < kl ? ql + step : ql;
      qr = b < kr ? qr + step : qr;
    }
    rl = (ql - tR) >> 3;
    rr = (qr - tL) >> 3;
    // the first key >= the lane's: equal only inside the other list (a real
    // key may be ~0 too, so the padding is excluded by position)
    const uint64_t kel = lr64(ql), ker = lr64(qr);
    EL = cmp64<kEQ>(kel, kl) & cmp32<kUGT>(nR, rl) & mnL;
    ER = cmp64<kEQ>(ker, kr) & cmp32<kUGT>(nL, rr) & mnR;
    }
  } else {
    uint32_t pl = rk0, pr = lk0;
    {
      const uint32_t n = nL > nR ? nL : nR;
      for (uint32_t step = n ? 8u << (31u - __builtin_clz(n)) : 0u; step >= 8u; step >>= 1) {
        const uint32_t cl = pl + step, cr = pr + step;
        const uint64_t kcl = lr64(cl < rkmax ? cl : rkmax), kcr = lr64(cr < lkmax ? cr : lkmax);
        pl = kcl < kl ? cl : pl;
        pr = kcr < kr ? cr : pr;
      }
    }
    pl = pl < rkmax ? pl : rkmax;
    pr = pr < lkmax ? pr : lkmax;
    rl = (pl - rk0) >> 3;
    rr = (pr - lk0) >> 3;
    const uint64_t kel = lr64(pl + 8u < rkmax ? pl + 8u : rkmax), ker = lr64(pr + 8u < lkmax ? pr + 8u : lkmax);
    // (an empty other side has no key to be equal to: the clamped probe read
    // the word before its key section)
    EL = nR ? cmp64<kEQ>(kel, kl) & mnL : 0ull;
    ER = nL ? cmp64<kEQ>(ker, kr) & mnR : 0ull;
  }
  const uint32_t U = nL + nR - (uint32_t)__popcll(EL);
  fb = fb || U > (uint32_t)kWave;
  if (OUT == 0 && fb) return kLeanFallback;
  const uint32_t ul = lane + rl - mbcnt64(EL), ur = lane + rr - mbcnt64(ER);  // union slots

  // ---- the member of every dot: run heads scattered by ds_permute (lanes
  // without a member target lane 0, a head whenever there is a member)
  const uint32_t sl = shift_up1(el), sr = shift_up1(er);  // run starts
  const uint32_t hl = (uint32_t)__builtin_amdgcn_ds_permute((int)((bit_of(mnL, lane) ? sl : 0u) << 2), 1);
  const uint32_t hr = (uint32_t)__builtin_amdgcn_ds_permute((int)((bit_of(mnR, lane) ? sr : 0u) << 2), 1);
  const uint64_t HL = cmp32<kNE>(hl, 0u) & mdL, HR = cmp32<kNE>(hr, 0u) & mdR;
  const uint32_t ml = __builtin_amdgcn_mbcnt_hi((uint32_t)(HL >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)HL, hl - 1u));
  const uint32_t mr = __builtin_amdgcn_mbcnt_hi((uint32_t)(HR >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)HR, hr - 1u));

  // ---- dots above the OTHER side's pre-merge top clock (survives masks)
  const uint64_t SL = cmp64<kUGT>(vl, gather64(tr, xl & (AW - 1u))) & mdL;
  const uint64_t SR = cmp64<kUGT>(vr, gather64(tl, xr & (AW - 1u))) & mdR;

  // ---- scratch: zero the mask tables and union descriptors, then the
  // per-member {actor mask, survives mask} by 64-bit atomic ORs
  const uint32_t trash = uX + TRW + l8;
  *(lds_u64*)(size_t)(uX + MsL + l8) = 0ull;
  *(lds_u64*)(size_t)(uX + MsR + l8) = 0ull;
  *(lds_u64*)(size_t)(uX + EqGe + l8) = 0ull;
  if (AW == 64) {
    *(lds_u64*)(size_t)(uX + MsL + 512u + l8) = 0ull;
    *(lds_u64*)(size_t)(uX + MsR + 512u + l8) = 0ull;
    *(lds_u64*)(size_t)(uX + EqGe + 512u + l8) = 0ull;
  }
  if (BK)
    *(lds_u32*)(size_t)(uX + Desc + 4u * lane) = 0u;
  else
    *(lds_u16*)(size_t)(uX + Desc + 2u * lane) = (uint16_t)0;
  wave_sync();
  const MT bl = (MT)1 << (xl & (AW - 1u)), br = (MT)1 << (xr & (AW - 1u));
  if (AW == 64) {  // {actor mask, survives mask} as two 64-bit words per member
    const uint32_t al = bit_of(mdL, lane) ? uX + MsL + ME * ml : trash, ar = bit_of(mdR, lane) ? uX + MsR + ME * mr : trash;
    __hip_atomic_fetch_or((lds_u64*)(size_t)al, bit_of(mdL, lane) ? (uint64_t)bl : 0ull, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or((lds_u64*)(size_t)(al + (bit_of(mdL, lane) ? 8u : 0u)), bit_of(SL, lane) ? (uint64_t)bl : 0ull,
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or((lds_u64*)(size_t)ar, bit_of(mdR, lane) ? (uint64_t)br : 0ull, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or((lds_u64*)(size_t)(ar + (bit_of(mdR, lane) ? 8u : 0u)), bit_of(SR, lane) ? (uint64_t)br : 0ull,
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    const uint64_t ol = ((uint64_t)(bit_of(SL, lane) ? bl : 0u) << 32) | (bit_of(mdL, lane) ? bl : 0u);
    const uint64_t orr = ((uint64_t)(bit_of(SR, lane) ? br : 0u) << 32) | (bit_of(mdR, lane) ? br : 0u);
    __hip_atomic_fetch_or((lds_u64*)(size_t)(bit_of(mdL, lane) ? uX + MsL + 8u * ml : trash), ol,
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or((lds_u64*)(size_t)(bit_of(mdR, lane) ? uX + MsR + 8u * mr : trash), orr,
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  {
    // union descriptors: L lanes store index + 1 in the low byte of their
    // slot, R lanes in the high byte (a shared key: both, same slot)
    const uint32_t trash1 = BK ? uX + TRW + 4u * lane : trash;
    *(lds_u8*)(size_t)(bit_of(mnL, lane) ? uX + Desc + DS * ul : trash1) = (uint8_t)(lane + 1u);
    *(lds_u8*)(size_t)(bit_of(mnR, lane) ? uX + Desc + DS * ur + 1u : trash1) = (uint8_t)(lane + 1u);
  }
  wave_sync();

  // ---- actors on both sides of a shared member: equal / self >= other,
  // by the R dots (partner L member i and union slot u of the dot's member
  // come from the R member lane; L's dot of the same actor by rank in ML)
  const uint32_t pj = bit_of(ER, lane) ? (0x10000u | (ur << 8) | rr) : 0u;
  const uint32_t q = gather32(pj, mr);
  {
    const uint32_t i = q & 63u, u = (q >> 8) & 63u;
    const MT MLi = AW == 64 ? (MT)lr64(uX + MsL + ME * i) : (MT)lr32(uX + MsL + 8u * i);
    const uint32_t a0 = gather32(sl, i);
    const uint32_t idx = a0 + (uint32_t)__builtin_popcountg(MLi & (br - (MT)1));
    const uint64_t va = lr64(uL + ctrL + 8u * idx);
    const uint64_t SH = cmp32<kNE>(q & 0x10000u, 0u) &
                        (AW == 64 ? cmp64<kNE>((uint64_t)(MLi & br), 0ull) : cmp32<kNE>((uint32_t)(MLi & br), 0u)) & mdR;
    const uint64_t EQ = cmp64<kEQ>(va, vr) & SH, GE = cmp64<kUGE>(va, vr) & SH;
    if (AW == 64) {  // {equal, >=} as two 64-bit words per union slot
      const uint32_t ae = bit_of(SH, lane) ? uX + EqGe + ME * u : trash;
      __hip_atomic_fetch_or((lds_u64*)(size_t)ae, bit_of(EQ, lane) ? (uint64_t)br : 0ull, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_or((lds_u64*)(size_t)(ae + (bit_of(SH, lane) ? 8u : 0u)), bit_of(GE, lane) ? (uint64_t)br : 0ull,
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      const uint64_t o = ((uint64_t)(bit_of(GE, lane) ? br : 0u) << 32) | (bit_of(EQ, lane) ? br : 0u);
      __hip_atomic_fetch_or((lds_u64*)(size_t)(bit_of(SH, lane) ? uX + EqGe + 8u * u : trash), o, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  wave_sync();

  // ---- per union member: the mask join
  const uint32_t dsc = BK ? lr32(uX + Desc + 4u * lane)
                          : *(const __attribute__((address_space(3))) uint16_t*)(size_t)(uX + Desc + 2u * lane);
  const uint32_t mi = (dsc - 1u) & 63u, mj = ((dsc >> 8) - 1u) & 63u;
  const uint64_t mU = lanes_below(U);
  const uint64_t hasL = cmp32<kNE>(dsc & 0xFFu, 0u) & mU, hasR = cmp32<kNE>(dsc >> 8, 0u) & mU;
  const uint64_t selfonly = hasL & ~hasR;
  MT ML, FL, MR, FR, EQm, GEm;  // EQm / GEm: zero unless both sides
  if (AW == 64) {
    const uint64_t pL0 = lr64(uX + MsL + ME * mi), pL1 = lr64(uX + MsL + ME * mi + 8u);
    const uint64_t pR0 = lr64(uX + MsR + ME * mj), pR1 = lr64(uX + MsR + ME * mj + 8u);
    EQm = (MT)lr64(uX + EqGe + ME * lane);
    GEm = (MT)lr64(uX + EqGe + ME * lane + 8u);
    ML = bit_of(hasL, lane) ? (MT)pL0 : (MT)0;
    FL = (MT)pL1 & ML;
    MR = bit_of(hasR, lane) ? (MT)pR0 : (MT)0;
    FR = (MT)pR1 & MR;
  } else {
    const uint64_t pL = lr64(uX + MsL + 8u * mi), pR = lr64(uX + MsR + 8u * mj), pE = lr64(uX + EqGe + l8);
    ML = bit_of(hasL, lane) ? (MT)(uint32_t)pL : (MT)0;
    FL = (MT)(uint32_t)(pL >> 32) & ML;
    MR = bit_of(hasR, lane) ? (MT)(uint32_t)pR : (MT)0;
    FR = (MT)(uint32_t)(pR >> 32) & MR;
    EQm = (MT)(uint32_t)pE;
    GEm = (MT)(uint32_t)(pE >> 32);
  }
  const MT lp = bit_of(selfonly, lane) ? ML : FL, rp = FR;
  const MT useA = (ML & MR & EQm) | (lp & (~rp | GEm));
  const uint64_t dropS = (AW == 64 ? cmp64<kEQ>((uint64_t)FL, 0ull) : cmp32<kEQ>((uint32_t)FL, 0u)) &
                         selfonly;  // self-only entry not above R's clock: dropped whole
  MT keep = (bit_of(dropS, lane) || !bit_of(mU, lane)) ? (MT)0 : (useA | rp);
  MT useK = useA & keep;
  Side DL{nullptr, RV{}}, DR{nullptr, RV{}};
  if (HD && HABL != 1) {  // (HABL: timing-only ablations, diagnostic builds)
    static_assert(!HD || OUT == 0, "deferred removes: direct stores only");
    DL = side_of(gptr(uL));
    DR = side_of(gptr(uR));
    // {keep, useK} by union slot (over the member masks, read above), and by
    // union slot the deferred clocks naming that member (bit k: self's clock
    // k, 32 + k: other's) — built from the deferred member lists, one lane per
    // (clock, member) item: the clock by a search over the run ends, the
    // union slot by a search of the key among each side's members
    const uint32_t dmt = uX + EqGe;
    if (AW == 64) {
      *(lds_u64*)(size_t)(uX + Out + ME * lane) = (uint64_t)keep;
      *(lds_u64*)(size_t)(uX + Out + ME * lane + 8u) = (uint64_t)useK;
    } else {
      *(lds_u64*)(size_t)(uX + Out + l8) = (uint64_t)keep | ((uint64_t)useK << 32);
    }
    *(lds_u64*)(size_t)(dmt + l8) = 0ull;
    wave_sync();
    const uint32_t nfL = DL.v.n_def, nfR = DR.v.n_def;
    const uint32_t nmL = nfL ? uni(lr32(uL + DL.v.fmend + 4u * (nfL - 1u))) : 0u;
    const uint32_t nmR = nfR ? uni(lr32(uR + DR.v.fmend + 4u * (nfR - 1u))) : 0u;
    if (HK == 1) {
      // the union keys by slot (slots are in key order), over the R member
      // masks read above, padded with ~0; and per deferred clock (lanes 0-31:
      // self's, 32-63: other's) the mask of the actors it holds
      const uint32_t ut = uX + MsR;
      const uint64_t ukey = lr64(bit_of(hasL, lane) ? uL + key + 8u * mi : uR + key + 8u * mj);
      *(lds_u64*)(size_t)(ut + l8) = bit_of(mU, lane) ? ukey : ~0ull;
      // the masks: one lane per deferred clock entry of either side (its
      // clock by a search of the run ends), OR-ed into its clock's slot
      *(lds_u32*)(size_t)(uX + k3DefMask + 4u * lane) = 0u;
      wave_sync();
      const uint32_t ndL = nfL ? uni(lr32(uL + DL.v.fdend + 4u * (nfL - 1u))) : 0u;
      const uint32_t ndR = nfR ? uni(lr32(uR + DR.v.fdend + 4u * (nfR - 1u))) : 0u;
      bool wide = false;  // an actor >= 32 (not canonical here): the general kernel joins the object
      for (uint32_t base = 0; base < ndL + ndR; base += kWave) {
        const uint32_t it = base + lane;
        const bool isL = it < ndL, act = it < ndL + ndR;
        const uint32_t us = isL ? uL : uR, e = act ? (isL ? it : it - ndL) : 0u;
        const uint32_t fd = us + (isL ? DL.v.fdend : DR.v.fdend), nf = isL ? nfL : nfR;
        uint32_t k = 0;  // # run ends <= e
        for (uint32_t step = 32u; step; step >>= 1)
          k = (k + step <= nf && lr32(fd + 4u * (k + step - 1u)) <= e) ? k + step : k;
        const uint32_t a = lr32(us + (isL ? DL.v.fact : DR.v.fact) + 4u * e);
        wide = wide || (act && a >= 32u);
        const bool put = act && a < 32u;
        __hip_atomic_fetch_or((lds_u32*)(size_t)(put ? uX + k3DefMask + 4u * (isL ? k : 32u + k) : uX + TRW + l8),
                              put ? 1u << a : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (__ballot(wide) != 0ull) return kLeanFallback;
      wave_sync();
      for (uint32_t base = 0; base < nmL + nmR; base += kWave) {
        const uint32_t it = base + lane;
        const bool isL = it < nmL, act = it < nmL + nmR;
        const uint32_t us = isL ? uL : uR, j = act ? (isL ? it : it - nmL) : 0u;
        const uint32_t fk = isL ? DL.v.fkey : DR.v.fkey, fm = isL ? DL.v.fmend : DR.v.fmend;
        const uint32_t nf = isL ? nfL : nfR;
        const uint64_t m = lr64(us + fk + 8u * j);
        uint32_t k = 0;  // # run ends <= j (n_def <= 32 per side)
        for (uint32_t step = 32u; step; step >>= 1)
          k = (k + step <= nf && lr32(us + fm + 4u * (k + step - 1u)) <= j) ? k + step : k;
        uint32_t q = ut;  // the first union key >= m (the table is 64 slots)
#pragma unroll
        for (uint32_t step = 256u; step >= 8u; step >>= 1) q = lr64(q + step - 8u) < m ? q + step : q;
        const uint32_t su = (q - ut) >> 3;
        const bool hit = act && su < U && lr64(q) == m;
        __hip_atomic_fetch_or((lds_u64*)(size_t)(hit ? dmt + 8u * su : uX + TRW + l8),
                              hit ? 1ull << (isL ? k : 32u + k) : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else
    for (uint32_t base = 0; base < nmL + nmR; base += kWave) {
      const uint32_t it = base + lane;
      const bool isL = it < nmL, act = it < nmL + nmR;
      const uint32_t us = isL ? uL : uR, j = act ? (isL ? it : it - nmL) : 0u;
      const uint32_t fk = isL ? DL.v.fkey : DR.v.fkey, fm = isL ? DL.v.fmend : DR.v.fmend;
      const uint32_t nf = isL ? nfL : nfR;
      const uint64_t m = lr64(us + fk + 8u * j);
      uint32_t k = 0;  // # run ends <= j (n_def <= 32 per side)
      for (uint32_t step = 32u; step; step >>= 1)
        k = (k + step <= nf && lr32(us + fm + 4u * (k + step - 1u)) <= j) ? k + step : k;
      // rank of m among each side's member keys (clamped probes), then equality
      uint32_t ql = lk0, qr = rk0;
      {
        const uint32_t n = nL > nR ? nL : nR;
        for (uint32_t step = n ? 8u << (31u - __builtin_clz(n)) : 0u; step >= 8u; step >>= 1) {
          const uint32_t cl = ql + step, cr = qr + step;
          ql = lr64(cl < lkmax ? cl : lkmax) < m ? cl : ql;
          qr = lr64(cr < rkmax ? cr : rkmax) < m ? cr : qr;
        }
      }
      ql = ql < lkmax ? ql : lkmax;
      qr = qr < rkmax ? qr : rkmax;
      const uint32_t il = (ql - lk0) >> 3, ir = (qr - rk0) >> 3;
      const bool eqL = nL && il < nL && lr64(ql + 8u < lkmax ? ql + 8u : lkmax) == m;
      const bool eqR = nR && ir < nR && lr64(qr + 8u < rkmax ? qr + 8u : rkmax) == m;
      const uint32_t sul = gather32(ul, il & 63u), sur = gather32(ur, ir & 63u);  // every lane: bpermute sources
      const uint32_t su = eqL ? sul : sur;
      const bool hit = act && (eqL || eqR);
      __hip_atomic_fetch_or((lds_u64*)(size_t)(hit ? dmt + 8u * (su & 63u) : uX + TRW + l8),
                            hit ? 1ull << (isL ? k : 32u + k) : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    wave_sync();
    // a surviving self dot / kept other dot of a named member: killed if D[x] >= v
    const uint32_t gl = gather32(ul, ml) & 63u, gr = gather32(ur, mr) & 63u;
    MT kpl, ukl, kpr, ukr;  // {keep, useK} of the dot's union slot
    if (AW == 64) {
      kpl = (MT)lr64(uX + Out + ME * gl);
      ukl = (MT)lr64(uX + Out + ME * gl + 8u);
      kpr = (MT)lr64(uX + Out + ME * gr);
      ukr = (MT)lr64(uX + Out + ME * gr + 8u);
    } else {
      const uint64_t okl = lr64(uX + Out + 8u * gl), okr = lr64(uX + Out + 8u * gr);
      kpl = (MT)(uint32_t)okl;
      ukl = (MT)(uint32_t)(okl >> 32);
      kpr = (MT)(uint32_t)okr;
      ukr = (MT)(uint32_t)(okr >> 32);
    }
    uint64_t bitsl = (bit_of(mdL, lane) && (ukl & bl)) ? lr64(dmt + 8u * gl) : 0ull;
    uint64_t bitsr = (bit_of(mdR, lane) && ((kpr & ~ukr) & br)) ? lr64(dmt + 8u * gr) : 0ull;
    // section addresses of both sides (scalars: no struct selected at run time)
    const uint32_t fdL = uL + DL.v.fdend, faL = uL + DL.v.fact, fcL = uL + DL.v.fctr;
    const uint32_t fdR = uR + DR.v.fdend, faR = uR + DR.v.fact, fcR = uR + DR.v.fctr;
    // D[x] of clock bit kb: a fixed-trip binary search of its actor-sorted run
    // (a deferred clock of an object on this path has <= A <= 32 entries)
    auto dget = [&](uint32_t kb, uint32_t x) -> uint64_t {
      if (HK == 1) {  // D[x] by the clock's actor mask: its rank among the clock's actors
        const bool sL = kb < 32u;
        const uint32_t kk = kb & 31u, fd = sL ? fdL : fdR, fc = sL ? fcL : fcR;
        const uint32_t msk = lr32(uX + k3DefMask + 4u * kb);
        const uint32_t lo = kk ? lr32(fd + 4u * (kk - 1u)) : 0u;
        return (msk >> x) & 1u ? lr64(fc + 8u * (lo + __popc(msk & ((1u << x) - 1u)))) : 0ull;
      }
      const bool sL = kb < 32u;
      const uint32_t kk = kb & 31u, fd = sL ? fdL : fdR, fa = sL ? faL : faR, fc = sL ? fcL : fcR;
      uint32_t lo = kk ? lr32(fd + 4u * (kk - 1u)) : 0u;
      const uint32_t e = lr32(fd + 4u * kk);
      uint32_t len = e - lo;
#pragma unroll
      for (int st = 0; st < (AW == 64 ? 7 : 6); ++st) {  // a clock of <= AW entries
        const uint32_t half = len >> 1, mid = lo + half;
        const bool go = len != 0u && lr32(fa + 4u * mid) < x;
        lo = go ? mid + 1u : lo;
        len = len == 0u ? 0u : (go ? len - half - 1u : half);
      }
      return (lo < e && lr32(fa + 4u * lo) == x) ? lr64(fc + 8u * lo) : 0ull;
    };
    bool kl2 = false, kr2 = false;
    while (bitsl | bitsr) {  // both dots' clocks in the same trips
      const uint64_t dl = bitsl ? dget((uint32_t)__builtin_ctzll(bitsl), xl & (AW - 1u)) : 0ull;
      const uint64_t dr = bitsr ? dget((uint32_t)__builtin_ctzll(bitsr), xr & (AW - 1u)) : 0ull;
      kl2 = kl2 || (bitsl && dl >= vl);
      kr2 = kr2 || (bitsr && dr >= vr);
      bitsl &= bitsl - 1u;
      bitsr &= bitsr - 1u;
    }
    __hip_atomic_fetch_and((lds_u64*)(size_t)(kl2 ? uX + Out + ME * gl : uX + TRW + l8), kl2 ? ~(uint64_t)bl : ~0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_and((lds_u64*)(size_t)(kr2 ? uX + Out + ME * gr : uX + TRW + l8), kr2 ? ~(uint64_t)br : ~0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    wave_sync();
    keep = bit_of(mU, lane) ? (MT)lr64(uX + Out + ME * lane) : (MT)0;
    useK &= keep;
  }
  const uint32_t c = (uint32_t)__builtin_popcountg(keep);

  // ---- output layout
  const uint64_t keepm = cmp32<kNE>(c, 0u);
  const uint32_t tot_mem = (uint32_t)__popcll(keepm);
  const uint32_t cincl = scan_incl(c);
  const uint32_t tot_dot = lane_of(cincl, kWave - 1);
  // HD: the deferred union is counted first; its walk records the survivors
  // (in the equal / >= area, read above) for the writing walk to replay
  uint32_t nd = 0, ndd = 0, ndm = 0;
  uint32_t* const dcache = HD ? (uint32_t*)gptr(uX + EqGe) : nullptr;
  const SideL WL{(lds_cu8*)(size_t)uL, DL.v}, WR{(lds_cu8*)(size_t)uR, DR.v};  // the walks read LDS directly
  if (HD && HABL != 2) deferred_pass_wave(WL, WR, A, lane, nd, ndd, ndm, nullptr, dcache);
  const uint32_t o_key = kHdrBytes + 8u * A, o_dctr = o_key + 8u * tot_mem, o_dact = o_dctr + 8u * tot_dot;
  const uint32_t o_mdend = o_dact + 4u * tot_dot, o_mpad = o_mdend + 4u * tot_mem;
  const uint32_t o_def = (o_mpad + 7u) & ~7u;
  const uint32_t o_end = o_def + 12u * ndd + 8u * ndm + 8u * nd;  // == o_def without deferred removes
  const uint32_t size = (o_end + 15u) & ~15u;
  if (OUT == 0 && size > OUTCAP) {
    big = true;
    return 0u;
  }
  const uint32_t d0 = cincl - c;
  if (OUT < 2 && AW == 32)
    *(__attribute__((address_space(3))) u32x4*)(size_t)(uX + Out + 16u * lane) = u32x4{(uint32_t)keep, (uint32_t)useK, d0, 0u};
  const uint32_t midx = mbcnt64(keepm);
  const uint64_t kk = lr64(bit_of(hasL, lane) ? uL + key + 8u * mi : uR + key + 8u * mj);
  const uint32_t xl2 = xl, xr2 = xr;
  const uint64_t vl2 = vl, vr2 = vr;
  const uint64_t top = tl > tr ? tl : tr;  // top clock: pointwise max (:153)
  wave_sync();
  // every kept dot at its member's base + the rank of its actor in keep
  const uint32_t gl = gather32(ul, ml), gr = gather32(ur, mr);
  MT okl, oul, okr, our;  // {keep, useK} of the dot's member
  uint32_t obl, obr;      // and its output dot base
  if (OUT >= 2 || AW == 64) {  // straight from the union lane's registers
    if (AW == 64) {
      okl = (MT)gather64((uint64_t)keep, gl);
      oul = (MT)gather64((uint64_t)useK, gl);
      okr = (MT)gather64((uint64_t)keep, gr);
      our = (MT)gather64((uint64_t)useK, gr);
    } else {
      okl = (MT)gather32((uint32_t)keep, gl);
      oul = (MT)gather32((uint32_t)useK, gl);
      okr = (MT)gather32((uint32_t)keep, gr);
      our = (MT)gather32((uint32_t)useK, gr);
    }
    obl = gather32(d0, gl);
    obr = gather32(d0, gr);
  } else {
    const u32x4 ol = *(const __attribute__((address_space(3))) u32x4*)(size_t)(uX + Out + 16u * (gl & 63u));
    const u32x4 orr = *(const __attribute__((address_space(3))) u32x4*)(size_t)(uX + Out + 16u * (gr & 63u));
    okl = (MT)ol.x;
    oul = (MT)ol.y;
    obl = ol.z;
    okr = (MT)orr.x;
    our = (MT)orr.y;
    obr = orr.z;
  }
  const uint32_t il = obl + (uint32_t)__builtin_popcountg(okl & (bl - (MT)1));
  const uint32_t ir = obr + (uint32_t)__builtin_popcountg(okr & (br - (MT)1));
  const bool wl = bit_of(mdL, lane) && (oul & bl) != (MT)0;          // self dots that survive
  const bool wr = bit_of(mdR, lane) && (okr & ~our & br) != (MT)0;  // other dots kept, not under a self dot
  if (OUT >= 2) {
    // the record is assembled in LDS over the (now dead) input stage, then
    // copied out with two 16-B stores per lane (sink-predicated): 2 vector
    // store instructions per object instead of ~10 scattered ones, which
    // occupied the texture-address unit (TA_BUSY 62-65 % of the kernel)
    fb = fb || size > 2u * 16u * kWave;  // larger outputs: the general kernel
    wave_sync();  // every read of the input stage (kk above) is done
    const uint32_t tw = uX + TRW + l8, tw4 = BK ? uX + TRW + 4u * lane : tw;
    *(lds_u64*)(size_t)(bit_of(keepm, lane) ? uL + o_key + 8u * midx : tw) = kk;
    *(lds_u32*)(size_t)(bit_of(keepm, lane) ? uL + o_mdend + 4u * midx : tw4) = d0 + c;
    *(lds_u64*)(size_t)(lane < A ? uL + kHdrBytes + l8 : tw) = top;
    *(lds_u32*)(size_t)(wl ? uL + o_dact + 4u * il : tw4) = xl2;
    *(lds_u64*)(size_t)(wl ? uL + o_dctr + 8u * il : tw) = vl2;
    *(lds_u32*)(size_t)(wr ? uL + o_dact + 4u * ir : tw4) = xr2;
    *(lds_u64*)(size_t)(wr ? uL + o_dctr + 8u * ir : tw) = vr2;
    const bool mp = lane == 0u && o_def != o_mpad;
    const bool rp = lane >= 1u && lane < 4u && o_def + 4u * (lane - 1u) < size;
    *(lds_u32*)(size_t)(mp ? uL + o_mpad : rp ? uL + o_def + 4u * (lane - 1u) : tw4) = 0u;
    const u32x4 hv = lane == 0u ? u32x4{size, A, tot_mem, tot_dot} : u32x4{0u, 0u, 0u, 0u};
    if (BK) {
      if (lane < 2u) *(__attribute__((address_space(3))) u32x4*)(size_t)(uL + 16u * lane) = hv;
    } else {
      *(__attribute__((address_space(3))) u32x4*)(size_t)(lane < 2u ? uL + 16u * lane : uX + TRW + 16u * (lane & 31u)) =
          hv;  // (16-B sink slots: lanes l and l + 32 share one, inside the 512-B sink)
    }
    if (OUT == 2) {  // OUT 3: the caller copies the record out
      wave_sync();
      copy_record_out(uL, O, fb ? 1u : size / 16u, lane);
    }
  } else if (OUT == 1) {
    // every store below is issued by every object: a lane with nothing to
    // store writes the wave's sink instead (selects, no branches)
    const bool kc = bit_of(keepm, lane) && !fb;
    *(uint64_t*)(kc ? O + o_key + 8u * midx : sink) = kk;
    *(uint32_t*)(kc ? O + o_mdend + 4u * midx : sink + 8) = d0 + c;
    *(uint64_t*)(lane < A && !fb ? O + kHdrBytes + l8 : sink + 16) = top;
    uint32_t* oact = (uint32_t*)(O + o_dact);
    uint64_t* octr = (uint64_t*)(O + o_dctr);
    *(uint32_t*)(wl && !fb ? (uint8_t*)(oact + il) : sink + 24) = xl2;
    *(uint64_t*)(wl && !fb ? (uint8_t*)(octr + il) : sink + 32) = vl2;
    *(uint32_t*)(wr && !fb ? (uint8_t*)(oact + ir) : sink + 24) = xr2;
    *(uint64_t*)(wr && !fb ? (uint8_t*)(octr + ir) : sink + 32) = vr2;
    // zero padding (member block to 8: <= 4 B, record to 16: <= 12 B) and the header
    const bool mp = lane == 0u && o_def != o_mpad && !fb;
    const bool rp = lane >= 1u && lane < 4u && o_def + 4u * (lane - 1u) < size && !fb;
    *(uint32_t*)(mp ? O + o_mpad : rp ? O + o_def + 4u * (lane - 1u) : sink + 40) = 0u;
    const u32x4 hv = lane == 0u ? u32x4{size, A, tot_mem, tot_dot} : u32x4{0u, 0u, 0u, 0u};
    *(u32x4*)(lane < 2u && !fb ? O + 16u * lane : sink + 48) = hv;
  } else {
    if (c != 0u) {
      *(uint64_t*)(O + o_key + 8u * midx) = kk;
      *(uint32_t*)(O + o_mdend + 4u * midx) = d0 + c;
    }
    if (lane < A) *(uint64_t*)(O + kHdrBytes + l8) = top;
    uint32_t* oact = (uint32_t*)(O + o_dact);
    uint64_t* octr = (uint64_t*)(O + o_dctr);
    if (wl) {
      oact[il] = xl2;
      octr[il] = vl2;
    }
    if (wr) {
      oact[ir] = xr2;
      octr[ir] = vr2;
    }
    if (lane == 0u && o_def != o_mpad) *(uint32_t*)(O + o_mpad) = 0u;
    if (lane >= 1u && lane < 4u && o_end + 4u * (lane - 1u) < size) *(uint32_t*)(O + o_end + 4u * (lane - 1u)) = 0u;
    if (lane == 0u) {
      u32x4* h = (u32x4*)O;
      h[0] = u32x4{size, A, tot_mem, tot_dot};
      h[1] = u32x4{nd, ndd, ndm, 0u};
    }
    if (HD && HABL != 2) {  // the deferred block (rec_layout's order: ctr, key, act, dend, mend)
      const uint32_t o_fkey = o_def + 8u * ndd, o_fact = o_fkey + 8u * ndm, o_fdend = o_fact + 4u * ndd;
      DefOut w{(uint64_t*)(O + o_def), (uint64_t*)(O + o_fkey), (uint32_t*)(O + o_fact), (uint32_t*)(O + o_fdend),
               (uint32_t*)(O + o_fdend + 4u * nd)};
      uint32_t a1, a2, a3;
      deferred_pass_wave(WL, WR, A, lane, a1, a2, a3, &w, dcache, nd);
    }
  }
  return OUT != 0 && fb ? kLeanFallback : size / 16u;
}



// ======================================================================
// Sparse mask path: the mask join (mask_object) for CSR top clocks over an
// actor universe of up to 1 024 ids (config 5). Actors are renumbered per
// object by their rank in the union of the two top clocks (<= 64 entries,
// sorted by actor id, so bit order is actor order): the union bitmap's bits
// below the actor, read from its prefix table (a dot actor whose bit is clear
// is outside both top clocks and falls back to the generic join; r06: this
// replaced a u8 actor -> rank table and its verify read, 13.71 -> 13.44 ms
// per 8-replica fold). Masks
// are 64-bit; everything else is mask_object's rules and layout, with the
// output's top clock the union list itself (pointwise max, sparse form).
// ======================================================================
constexpr uint32_t kSpTableN = 1024;
// scratch byte offsets; run heads cover 128 dots per side (two 64-dot rounds)
constexpr uint32_t kSpMsL = 0, kSpMsR = 1024, kSpOut = 0, kSpEq = 2048, kSpDesc = 3072, kSpHeadL = 3328,
                   kSpHeadR = 3456, kSpUofI = 3584, kSpUofJ = 3648, kSpUcAct = 3712, kSpUcL = 3968, kSpUcR = 4480,
                   kSpTrash = 4992;
// the clock-union bitmap and its prefix table overlay the equal/>= masks
// (zeroed once every dot has its rank)
constexpr uint32_t kSpUbm = kSpEq, kSpUpre = kSpEq + 256u;
// 7 040 B per wave: the CSR join takes 6 016 (kSpTrash + 1 KB); the DN
// kernel's wide_mask_object runs on the same scratch (6 944 B)
constexpr uint32_t kSpScratch = 7040;
static_assert(kSpTrash + 16u * kWave <= kSpScratch, "sparse join scratch");

__device__ __forceinline__ uint32_t below64(uint64_t mask, uint32_t b) {
  return (uint32_t)__popcll(mask & ((1ull << b) - 1ull));
}

// # of the n sorted u32 actor ids at `off` strictly below x (n <= 64).
__device__ __forceinline__ uint32_t rank32(const uint8_t* b, uint32_t off, uint32_t n, uint32_t x) {
  uint32_t base = 0;
  for (uint32_t step = n ? 1u << (31u - __builtin_clz(n)) : 0u; step != 0u; step >>= 1) {
    const uint32_t cand = base + step;
    base = (cand <= n && ld32(b, off + 4u * (cand - 1u)) < x) ? cand : base;
  }
  return base;
}

// ASM (objects without deferred removes, Ls the start of a pair stage that
// can hold the output: the sparse mask kernel's): the output record is
// assembled over the pair stage once every read of it is done and copied out
// with 16-B stores, instead of scattered 4- / 8-B stores to HBM (as mask3's
// OUT 2 does for the dense join); with O == nullptr it stays in the stage
// (the fused fold's accumulator)
// (Dense top clocks of 65..1 024 actors take wide_mask_object, below.)
template <bool HD, int ABL = 0, bool ASM = false>
__device__ __forceinline__ uint32_t sparse_mask_object(const uint8_t* Ls, const uint8_t* Rs, uint8_t* X, uint8_t* O,
                                                       uint32_t A, uint32_t ncL, uint32_t nL, uint32_t dL,
                                                       uint32_t ncR, uint32_t nR, uint32_t dR, uint32_t lane,
                                                       Stamps* st = nullptr) {
  const uint32_t keyL = kHdrBytes + clock_bytes(ncL, true), keyR = kHdrBytes + clock_bytes(ncR, true);
  const uint32_t caL = kHdrBytes + 8u * ncL, caR = kHdrBytes + 8u * ncR;  // clock actor lists (CSR)
  const uint32_t ctrL = keyL + 8u * nL, actL = ctrL + 8u * dL, endL = actL + 4u * dL;
  const uint32_t ctrR = keyR + 8u * nR, actR = ctrR + 8u * dR, endR = actR + 4u * dR;
  const uint32_t tr = kSpTrash + 16u * lane;

  // ---- union of the two top clocks: an actor's union position is the
  // number of union-bitmap bits below it (both sides agree on a common actor)
  const bool hcl = lane < ncL, hcr = lane < ncR;
  const uint32_t cxl = ld32(Ls, caL + 4u * lane), cxr = ld32(Rs, caR + 4u * lane);
  const uint64_t cvl = ld64(Ls, kHdrBytes + 8u * lane), cvr = ld64(Rs, kHdrBytes + 8u * lane);
  if (__ballot((hcl && cxl >= kSpTableN) || (hcr && cxr >= kSpTableN)) != 0ull) return kLeanFallback;
  wave_sync();  // the previous object's readers of this scratch are done
  if (lane < kSpTableN / 64u) *(uint64_t*)(X + kSpUbm + 8u * lane) = 0ull;
  atomicOr((unsigned long long*)(X + (hcl ? kSpUbm + 8u * (cxl >> 6) : tr)), 1ull << (cxl & 63u));
  atomicOr((unsigned long long*)(X + (hcr ? kSpUbm + 8u * (cxr >> 6) : tr)), 1ull << (cxr & 63u));
  wave_sync();
  const uint64_t bw = lane < kSpTableN / 64u ? *(const uint64_t*)(X + kSpUbm + 8u * lane) : 0ull;
  const uint32_t bpc = (uint32_t)__popcll(bw), bin = scan_incl(bpc);
  const uint32_t Uc = lane_of(bin, kSpTableN / 64u - 1u);
  if (Uc > (uint32_t)kWave) return kLeanFallback;
  if (lane < kSpTableN / 64u)
    *(u32x4*)(X + kSpUpre + 16u * lane) = u32x4{(uint32_t)bw, (uint32_t)(bw >> 32), bin - bpc, 0u};
  *(uint64_t*)(X + kSpUcL + 8u * lane) = 0ull;
  *(uint64_t*)(X + kSpUcR + 8u * lane) = 0ull;
  wave_sync();
  const u32x4 pwl = *(const u32x4*)(X + kSpUpre + 16u * (cxl >> 6 & 15u));
  const u32x4 pwr = *(const u32x4*)(X + kSpUpre + 16u * (cxr >> 6 & 15u));
  const uint32_t ucl = pwl.z + below64(((uint64_t)pwl.y << 32) | pwl.x, cxl & 63u);
  const uint32_t ucr = pwr.z + below64(((uint64_t)pwr.y << 32) | pwr.x, cxr & 63u);
  if (ABL == 9) mark<ABL>(*st, 2);

  // ---- members (as mask_object); dots are handled in rounds of 64 (<= 128 per side)
  const bool hml = lane < nL, hmr = lane < nR;
  const uint32_t nrnd = (dL > dR ? dL : dR) > 64u ? 2u : 1u;
  const uint64_t kl = ld64(Ls, keyL + 8u * lane), kr = ld64(Rs, keyR + 8u * lane);
  uint32_t rl = 0, rr = 0;
  {
    const uint32_t n = nL > nR ? nL : nR;
    for (uint32_t step = n ? 1u << (31u - __builtin_clz(n)) : 0u; step != 0u; step >>= 1) {
      const uint32_t cl = rl + step, cr = rr + step;
      const uint64_t kcl = ld64(Rs, keyR + 8u * (cl - 1u)), kcr = ld64(Ls, keyL + 8u * (cr - 1u));
      rl = (cl <= nR && kcl < kl) ? cl : rl;
      rr = (cr <= nL && kcr < kr) ? cr : rr;
    }
  }
  const bool eql = hml && rl < nR && ld64(Rs, keyR + 8u * rl) == kl;
  const bool eqr = hmr && rr < nL && ld64(Ls, keyL + 8u * rr) == kr;
  const uint64_t EL = __ballot(eql), ER = __ballot(eqr);
  const uint32_t U = nL + nR - (uint32_t)__popcll(EL);
  if (U > (uint32_t)kWave) return kLeanFallback;
  const uint32_t ul = lane + rl - mbcnt64(EL), ur = lane + rr - mbcnt64(ER);

  wave_sync();  // the previous object's readers of this scratch are done
  // union clock entries (each side its own counter) + actor table
  *(uint32_t*)(X + (hcl ? kSpUcAct + 4u * (ucl & 63u) : tr)) = cxl;
  *(uint64_t*)(X + (hcl ? kSpUcL + 8u * (ucl & 63u) : tr)) = cvl;
  *(uint32_t*)(X + (hcr ? kSpUcAct + 4u * (ucr & 63u) : tr)) = cxr;
  *(uint64_t*)(X + (hcr ? kSpUcR + 8u * (ucr & 63u) : tr)) = cvr;
  // member masks (zeroed), run heads, descriptors
  *(u32x4*)(X + kSpMsL + 16u * lane) = u32x4{0u, 0u, 0u, 0u};
  *(u32x4*)(X + kSpMsR + 16u * lane) = u32x4{0u, 0u, 0u, 0u};
  X[kSpHeadL + lane] = 0u;
  X[kSpHeadL + 64u + lane] = 0u;
  X[kSpHeadR + lane] = 0u;
  X[kSpHeadR + 64u + lane] = 0u;
  const uint32_t el0 = ld32(Ls, endL + 4u * lane - 4u), er0 = ld32(Rs, endR + 4u * lane - 4u);
  const uint32_t sl = lane ? el0 : 0u, sr = lane ? er0 : 0u;
  X[(hml && sl < 128u) ? kSpHeadL + sl : tr] = 1u;
  X[(hmr && sr < 128u) ? kSpHeadR + sr : tr] = 1u;
  *(uint32_t*)(X + (hml ? kSpDesc + 4u * (ul & 63u) : tr)) = ((eql ? kBoth : kSelf) << 16) | (lane << 8) | (eql ? rl : 0u);
  *(uint32_t*)(X + ((hmr && !eqr) ? kSpDesc + 4u * (ur & 63u) : tr)) = (kOther << 16) | (rr << 8) | lane;
  X[kSpUofI + lane] = (uint8_t)ul;
  X[kSpUofJ + lane] = (uint8_t)ur;
  wave_sync();
  if (ABL == 9) mark<ABL>(*st, 3);
  // run-head masks of both rounds; the member of dot 64r + lane is
  // (#heads at or below it) - 1
  const uint64_t HL0 = __ballot(lane < dL && X[kSpHeadL + lane] != 0u);
  const uint64_t HL1 = __ballot(64u + lane < dL && X[kSpHeadL + 64u + lane] != 0u);
  const uint64_t HR0 = __ballot(lane < dR && X[kSpHeadR + lane] != 0u);
  const uint64_t HR1 = __ballot(64u + lane < dR && X[kSpHeadR + 64u + lane] != 0u);
  bool foreign = false;
  // each dot's actor, counter, union-clock bit and member, per round, kept in
  // registers for the later passes (two rounds at most)
  uint32_t rXL[2] = {0u, 0u}, rXR[2] = {0u, 0u}, rBL[2] = {0u, 0u}, rBR[2] = {0u, 0u};
  uint32_t rML[2] = {0u, 0u}, rMR[2] = {0u, 0u};
  uint64_t rVL[2] = {0ull, 0ull}, rVR[2] = {0ull, 0ull};
#pragma unroll
  for (uint32_t rd = 0; rd < 2u; ++rd) {  // dot -> union clock bit (verified) -> member masks
    if (rd >= nrnd) break;
    const uint32_t d = 64u * rd + lane;
    const bool hdl = d < dL, hdr = d < dR;
    const uint32_t xl = ld32(Ls, actL + 4u * d), xr = ld32(Rs, actR + 4u * d);
    const uint64_t vl = ld64(Ls, ctrL + 8u * d), vr = ld64(Rs, ctrR + 8u * d);
    const uint64_t HL = rd ? HL1 : HL0, HR = rd ? HR1 : HR0;
    const uint32_t ml = (rd ? (uint32_t)__popcll(HL0) : 0u) + mbcnt64(HL) + ((HL >> lane) & 1ull ? 1u : 0u) - 1u;
    const uint32_t mr = (rd ? (uint32_t)__popcll(HR0) : 0u) + mbcnt64(HR) + ((HR >> lane) & 1ull ? 1u : 0u) - 1u;
    // rank = the union bitmap's bits below the actor (its prefix-table row);
    // in the union iff its bit is set
    const u32x4 pwl = *(const u32x4*)(X + kSpUpre + 16u * ((xl >> 6) & 15u));
    const u32x4 pwr = *(const u32x4*)(X + kSpUpre + 16u * ((xr >> 6) & 15u));
    const uint64_t bwl = ((uint64_t)pwl.y << 32) | pwl.x, bwr = ((uint64_t)pwr.y << 32) | pwr.x;
    const uint32_t bl = (pwl.z + below64(bwl, xl & 63u)) & 63u, br = (pwr.z + below64(bwr, xr & 63u)) & 63u;
    foreign = foreign || (hdl && (xl >= kSpTableN || ((bwl >> (xl & 63u)) & 1ull) == 0ull)) ||
              (hdr && (xr >= kSpTableN || ((bwr >> (xr & 63u)) & 1ull) == 0ull));
    rXL[rd] = xl; rXR[rd] = xr; rVL[rd] = vl; rVR[rd] = vr; rBL[rd] = bl; rBR[rd] = br; rML[rd] = ml; rMR[rd] = mr;
    const uint64_t rc = *(const uint64_t*)(X + kSpUcR + 8u * bl), lc = *(const uint64_t*)(X + kSpUcL + 8u * br);
    const uint64_t mbl = hdl ? 1ull << bl : 0ull, mbr = hdr ? 1ull << br : 0ull;
    unsigned long long* pl = (unsigned long long*)(X + (hdl ? kSpMsL + 16u * (ml & 63u) : tr));
    unsigned long long* pr = (unsigned long long*)(X + (hdr ? kSpMsR + 16u * (mr & 63u) : tr));
    atomicOr(pl, (unsigned long long)mbl);
    atomicOr(pl + 1, (unsigned long long)(vl > rc ? mbl : 0ull));
    atomicOr(pr, (unsigned long long)mbr);
    atomicOr(pr + 1, (unsigned long long)(vr > lc ? mbr : 0ull));
  }
  if (__ballot(foreign) != 0ull) return kLeanFallback;  // a dot actor outside both top clocks
  wave_sync();
  // every dot has its rank: the prefix table's words become the equal / >= masks
  *(u32x4*)(X + kSpEq + 16u * lane) = u32x4{0u, 0u, 0u, 0u};
  wave_sync();
  if (ABL == 9) mark<ABL>(*st, 4);
#pragma unroll
  for (uint32_t rd = 0; rd < 2u; ++rd) {  // actors on both sides of a shared member: equal / self >= other
    if (rd >= nrnd) break;
    const uint32_t dd = 64u * rd + lane;
    const bool hdr = dd < dR;
    const uint64_t vr = rVR[rd];
    const uint32_t br = rBR[rd], mr = rMR[rd];
    const uint32_t u = X[kSpUofJ + (mr & 63u)] & 63u;
    const uint32_t d = *(const uint32_t*)(X + kSpDesc + 4u * u);
    const uint32_t i = (d >> 8) & 63u;
    const uint64_t ML = *(const uint64_t*)(X + kSpMsL + 16u * i);
    const bool sh = hdr && (d >> 16) == kBoth && ((ML >> br) & 1ull);
    const uint32_t a0 = i ? ld32(Ls, endL + 4u * i - 4u) : 0u;
    const uint64_t va = ld64(Ls, ctrL + 8u * ((a0 + below64(ML, br)) & 127u));
    unsigned long long* pe = (unsigned long long*)(X + (sh ? kSpEq + 16u * u : tr));
    atomicOr(pe, (unsigned long long)(sh && va == vr ? 1ull << br : 0ull));
    atomicOr(pe + 1, (unsigned long long)(sh && va >= vr ? 1ull << br : 0ull));
  }
  wave_sync();
  if (ABL == 9) mark<ABL>(*st, 5);
  // ---- per union member: mask join (src/orswot.rs:94-138)
  const bool hu = lane < U;
  const uint32_t dsc = hu ? *(const uint32_t*)(X + kSpDesc + 4u * lane) : 0u;
  const uint32_t ty = dsc >> 16, mi = (dsc >> 8) & 63u, mj = dsc & 63u;
  const u32x4 pl4 = *(const u32x4*)(X + kSpMsL + 16u * mi), pr4 = *(const u32x4*)(X + kSpMsR + 16u * mj);
  const u32x4 pe4 = *(const u32x4*)(X + kSpEq + 16u * lane);
  const uint64_t zl = ((uint64_t)pl4.y << 32) | pl4.x, zfl = ((uint64_t)pl4.w << 32) | pl4.z;
  const uint64_t zr = ((uint64_t)pr4.y << 32) | pr4.x, zfr = ((uint64_t)pr4.w << 32) | pr4.z;
  const uint64_t ML = (ty & kSelf) ? zl : 0ull, FL = (ty & kSelf) ? zfl : 0ull;
  const uint64_t MR = (ty & kOther) ? zr : 0ull, FR = (ty & kOther) ? zfr : 0ull;
  const uint64_t EQ = ty == kBoth ? (((uint64_t)pe4.y << 32) | pe4.x) : 0ull;
  const uint64_t GE = ty == kBoth ? (((uint64_t)pe4.w << 32) | pe4.z) : 0ull;
  const bool self_only = ty == kSelf;
  const uint64_t lp = self_only ? ML : (ML & FL), rp = MR & FR;
  const uint64_t useA = (ML & MR & EQ) | (lp & (~rp | GE));
  uint64_t keep = useA | rp;
  keep = (self_only && (ML & FL) == 0ull) ? 0ull : keep;
  keep = hu ? keep : 0ull;
  uint64_t useK = useA & keep;
  SideL DL{(lds_cu8*)(size_t)lds_addr(Ls), RV{}}, DR{(lds_cu8*)(size_t)lds_addr(Rs), RV{}};  // LDS stages: ds_* reads
  if (HD) {  // deferred removes (apply_deferred -> apply_remove, src/orswot.rs:235-243, 195-211)
    DL.v = make_rv(layout_at(Ls));
    DR.v = make_rv(layout_at(Rs));
    wave_sync();
    *(uint64_t*)(X + kSpOut + 32u * lane) = keep;
    *(uint64_t*)(X + kSpOut + 32u * lane + 8u) = useK;
    wave_sync();
#pragma unroll
    for (uint32_t rd = 0; rd < 2u; ++rd) {
      if (rd >= nrnd) break;
      const uint32_t d = 64u * rd + lane;
      const bool hdl = d < dL, hdr = d < dR;
      const uint32_t xl = rXL[rd], xr = rXR[rd], bl = rBL[rd], br = rBR[rd], ml = rML[rd], mr = rMR[rd];
      const uint64_t vl = rVL[rd], vr = rVR[rd];
      if (hdl) {
        unsigned long long* ok = (unsigned long long*)(X + kSpOut + 32u * X[kSpUofI + (ml & 63u)]);
        if ((ok[1] >> bl) & 1ull) {
          const uint64_t mk = dmask_of(DL, DR, ld64(Ls, keyL + 8u * (ml & 63u)));
          if (mk && dkilled(DL, DR, mk, xl, vl)) atomicAnd(ok, ~(1ull << bl));
        }
      }
      if (hdr) {
        unsigned long long* ok = (unsigned long long*)(X + kSpOut + 32u * X[kSpUofJ + (mr & 63u)]);
        if (((ok[0] & ~ok[1]) >> br) & 1ull) {
          const uint64_t mk = dmask_of(DL, DR, ld64(Rs, keyR + 8u * (mr & 63u)));
          if (mk && dkilled(DL, DR, mk, xr, vr)) atomicAnd(ok, ~(1ull << br));
        }
      }
    }
    wave_sync();
    keep = *(const uint64_t*)(X + kSpOut + 32u * lane);
    useK &= keep;
    if (ABL == 9) mark<ABL>(*st, 10);
  }
  const uint32_t c = (uint32_t)__popcll(keep);
  // ---- output layout (sparse top clock of Uc entries)
  const uint64_t keepm = __ballot(c != 0u);
  const uint32_t tot_mem = (uint32_t)__popcll(keepm);
  const uint32_t cincl = scan_incl(c);
  const uint32_t tot_dot = lane_of(cincl, kWave - 1);
  uint32_t nd = 0, ndd = 0, ndm = 0;
  if (ABL == 9) mark<ABL>(*st, 6);
  // survivors cached in the run-head area (free once the head ballots are taken; 64 entries)
  uint32_t* dcache = (uint32_t*)(X + kSpHeadL);
  if (HD) deferred_pass_wave<true>(DL, DR, A, lane, nd, ndd, ndm, nullptr, dcache);
  if (ABL == 9) mark<ABL>(*st, 8);
  RecLayout OL;
  rec_layout(OL, Uc, tot_mem, tot_dot, nd, ndd, ndm, true);
  const uint32_t size = OL.size;
  const uint32_t d0 = cincl - c;
  if (ABL == 9) mark<ABL>(*st, 6);
  static_assert(!(ASM && HD), "ASM: objects without deferred removes (the deferred walk reads the stages)");
  uint8_t* const O_ = O;
  if (ASM) {
    // the last read of the pair stage (the kept members' keys; the dots are
    // in registers), then the record is written over the stage
    const uint64_t kk = c != 0u ? ((ty & kSelf) ? ld64(Ls, keyL + 8u * mi) : ld64(Rs, keyR + 8u * mj)) : 0ull;
    wave_sync();
    O = const_cast<uint8_t*>(Ls);
    *(uint64_t*)(X + kSpOut + 32u * lane) = hu ? keep : 0ull;
    *(uint64_t*)(X + kSpOut + 32u * lane + 8u) = hu ? useK : 0ull;
    *(uint32_t*)(X + kSpOut + 32u * lane + 16u) = d0;
    if (c != 0u) {
      const uint32_t midx = mbcnt64(keepm);
      *(uint64_t*)(O + OL.o_key + 8u * midx) = kk;
      *(uint32_t*)(O + OL.o_mdend + 4u * midx) = d0 + c;
    }
  } else {
    wave_sync();
    *(uint64_t*)(X + kSpOut + 32u * lane) = hu ? keep : 0ull;
    *(uint64_t*)(X + kSpOut + 32u * lane + 8u) = hu ? useK : 0ull;
    *(uint32_t*)(X + kSpOut + 32u * lane + 16u) = d0;
    if (c != 0u) {
      const uint32_t midx = mbcnt64(keepm);
      const uint64_t kk = (ty & kSelf) ? ld64(Ls, keyL + 8u * mi) : ld64(Rs, keyR + 8u * mj);
      *(uint64_t*)(O + OL.o_key + 8u * midx) = kk;
      *(uint32_t*)(O + OL.o_mdend + 4u * midx) = d0 + c;
    }
  }
  if (lane < Uc) {  // top clock: the union list, pointwise max (src/orswot.rs:153)
    const uint64_t a = *(const uint64_t*)(X + kSpUcL + 8u * lane), b = *(const uint64_t*)(X + kSpUcR + 8u * lane);
    *(uint64_t*)(O + kHdrBytes + 8u * lane) = a > b ? a : b;
    *(uint32_t*)(O + kHdrBytes + 8u * Uc + 4u * lane) = *(const uint32_t*)(X + kSpUcAct + 4u * lane);
  }
  if (lane == 0u && (Uc & 1u)) *(uint32_t*)(O + kHdrBytes + 12u * Uc) = 0u;  // clock section pad to 8
  wave_sync();
  uint32_t* oact = (uint32_t*)(O + OL.o_dact);
  uint64_t* octr = (uint64_t*)(O + OL.o_dctr);
#pragma unroll
  for (uint32_t rd = 0; rd < 2u; ++rd) {  // every kept dot at its member's base + actor rank
    if (rd >= nrnd) break;
    const uint32_t d = 64u * rd + lane;
    const bool hdl = d < dL, hdr = d < dR;
    const uint32_t xl = rXL[rd], xr = rXR[rd], bl = rBL[rd], br = rBR[rd], ml = rML[rd], mr = rMR[rd];
    const uint64_t vl = rVL[rd], vr = rVR[rd];
    if (hdl) {
      const uint8_t* ob = X + kSpOut + 32u * X[kSpUofI + (ml & 63u)];
      const uint64_t k = *(const uint64_t*)ob, ua = *(const uint64_t*)(ob + 8);
      if ((ua >> bl) & 1ull) {
        const uint32_t idx = *(const uint32_t*)(ob + 16) + below64(k, bl);
        oact[idx] = xl;
        octr[idx] = vl;
      }
    }
    if (hdr) {
      const uint8_t* ob = X + kSpOut + 32u * X[kSpUofJ + (mr & 63u)];
      const uint64_t k = *(const uint64_t*)ob, ua = *(const uint64_t*)(ob + 8);
      if (((k & ~ua) >> br) & 1ull) {
        const uint32_t idx = *(const uint32_t*)(ob + 16) + below64(k, br);
        oact[idx] = xr;
        octr[idx] = vr;
      }
    }
  }
  if (ABL == 9) mark<ABL>(*st, 7);
  if (HD) {
    DefOut w{(uint64_t*)(O + OL.o_fctr), (uint64_t*)(O + OL.o_fkey), (uint32_t*)(O + OL.o_fact),
             (uint32_t*)(O + OL.o_fdend), (uint32_t*)(O + OL.o_fmend)};
    wave_sync();
    deferred_pass_wave<true>(DL, DR, A, lane, nd, ndd, ndm, &w, dcache, nd);
  }
  if (ABL == 9) mark<ABL>(*st, 9);
  if (lane == 0u && OL.o_def != OL.o_mpad) *(uint32_t*)(O + OL.o_mpad) = 0u;
  if (lane >= 1u && lane < 4u && OL.o_end + 4u * (lane - 1u) < size) *(uint32_t*)(O + OL.o_end + 4u * (lane - 1u)) = 0u;
  if (lane == 0u) {
    u32x4* h = (u32x4*)O;
    h[0] = u32x4{size, Uc, tot_mem, tot_dot};
    h[1] = u32x4{nd, ndd, ndm, kSparseClock};
  }
  if (ASM && O_ != nullptr) {  // the assembled record out of the stage: 16-B coalesced non-temporal stores
    wave_sync();
    for (uint32_t k = lane; k < size / 16u; k += kWave) __builtin_nontemporal_store(((const u32x4*)O)[k], (u32x4*)O_ + k);
  }
  if (ABL == 9) mark<ABL>(*st, 7);
  return size / 16u;
}

// ======================================================================
// Dense-wide join (dense top clocks of 65..1 024 actors): the mask join over
// each object's union of PRESENT actors (a dense clock stores 0 for an absent
// actor, src/vclock.rs:159-163), W words of actor masks: W = 1 for a union of
// <= 64 actors, W = 2 (word b >> 6, bit b & 63) for 65..128. An actor's rank
// is read from the union bitmap's prefix table (a dense dot actor is in the
// union iff its bitmap bit is set, so no actor table and no union clock
// lists), the other side's counter at a dot's actor from its dense row, and
// the joined top clock is written dense (pointwise max, src/orswot.rs:153).
// Same rules as mask_object (src/orswot.rs:94-138; apply_deferred
// :235-243 -> apply_remove :195-211); members <= 64 per side and in the
// union, dots <= 128 per side, deferred clocks <= 32 per side.
// ======================================================================
// scratch byte offsets (per wave, laid out for W = 2; fits the sparse join's
// kSpScratch): member masks {M, F} of W words per member; the
// per-union-member {keep, useK, d0} (48 B; W = 1: 32) over them once
// they are read, the deferred walk's survivor cache after it; the union
// bitmap's prefix table over the equal / >= masks until the dots have their
// ranks; run heads as bits (2 words per side); u16 union descriptors; an
// 8-byte trash slot per lane for masked-off stores
constexpr uint32_t kWdMsL = 0, kWdMsR = 2048, kWdOut = 0, kWdCache = 3072, kWdEq = 4096, kWdUpre = kWdEq,
                   kWdDesc = 6144, kWdHeads = 6272, kWdUofI = 6304, kWdUofJ = 6368, kWdTrash = 6432;
constexpr uint32_t kWdScratch = kWdTrash + 8u * kWave;  // 6 944 B per wave
static_assert(kWdScratch <= kSpScratch, "the DN mask kernel's scratch holds the wide join's");
constexpr uint32_t kWdOutStride = 48;
// W = 1 (64-bit masks): {M, F} 16 B per member, {keep, useK, d0} 32 B per
// union member, the survivor cache over the equal / >= masks after the join
constexpr uint32_t kWd1MsR = 1024, kWd1Eq = 2048, kWd1Desc = 3072, kWd1Heads = 3200, kWd1UofI = 3232, kWd1UofJ = 3296,
                   kWd1Trash = 3360;
constexpr uint32_t kWd1Scratch = kWd1Trash + 8u * kWave;  // 3 872 B per wave
static_assert(kWd1Scratch <= kWdScratch, "W = 1 fits the W = 2 scratch");

__device__ __forceinline__ bool bit128(uint64_t lo, uint64_t hi, uint32_t b) {
  return ((b < 64u ? lo : hi) >> (b & 63u)) & 1ull;
}
// # of set bits of the 128-bit mask below bit b (b < 128)
__device__ __forceinline__ uint32_t below128(uint64_t lo, uint64_t hi, uint32_t b) {
  return b < 64u ? below64(lo, b) : (uint32_t)__popcll(lo) + below64(hi, b - 64u);
}
__device__ __forceinline__ uint64_t ldm64(const uint8_t* X, uint32_t off) { return *(const uint64_t*)(X + off); }
// bits [0, n) of a word (n as a signed count: <= 0 -> none, >= 64 -> all)
__device__ __forceinline__ uint64_t lowmask64(uint32_t n) {
  return (int32_t)n <= 0 ? 0ull : n >= 64u ? ~0ull : (1ull << n) - 1ull;
}

template <bool HD, uint32_t W = 2>
__device__ __forceinline__ uint32_t wide_mask_object(const uint8_t* Ls, const uint8_t* Rs, uint8_t* X, uint8_t* O,
                                                     uint32_t A, uint32_t nL, uint32_t dL, uint32_t nR, uint32_t dR,
                                                     uint32_t lane) {
  const uint32_t keyL = kHdrBytes + 8u * A, keyR = keyL;
  const uint32_t ctrL = keyL + 8u * nL, actL = ctrL + 8u * dL, endL = actL + 4u * dL;
  const uint32_t ctrR = keyR + 8u * nR, actR = ctrR + 8u * dR, endR = actR + 4u * dR;
  static_assert(W == 1u || W == 2u, "64- or 128-bit actor masks");
  // scratch offsets: kWd* (W = 2), or the 3 872-B W = 1 layout (kWd1*)
  constexpr uint32_t oMsL = kWdMsL, oOut = kWdOut, oMsR = W == 2u ? kWdMsR : kWd1MsR, oEq = W == 2u ? kWdEq : kWd1Eq;
  constexpr uint32_t oCache = W == 2u ? kWdCache : kWd1Eq, oUpre = W == 2u ? kWdUpre : kWd1Eq;
  constexpr uint32_t oDesc = W == 2u ? kWdDesc : kWd1Desc;
  constexpr uint32_t oHeads = W == 2u ? kWdHeads : kWd1Heads, oUofI = W == 2u ? kWdUofI : kWd1UofI;
  constexpr uint32_t oUofJ = W == 2u ? kWdUofJ : kWd1UofJ, oTrash = W == 2u ? kWdTrash : kWd1Trash;
  const uint32_t tr = oTrash + 8u * lane;
  // per member: {M, F} of W words; per union member: {EQ, GE} of W words,
  // then {keep, useK, d0} over the member masks
  constexpr uint32_t MS = 16u * W, OS = W == 2u ? kWdOutStride : 32u;

  // ---- union of present actors (a dense clock stores 0 for an absent
  // actor, src/vclock.rs:159-163): lane q keeps bitmap word q (actors 64 q ..)
  uint64_t bw = 0ull;
  for (uint32_t q = 0; q < (A + 63u) / 64u; ++q) {
    const uint32_t a = 64u * q + lane;
    const bool p = a < A && (ld64(Ls, kHdrBytes + 8u * a) | ld64(Rs, kHdrBytes + 8u * a)) != 0ull;
    const uint64_t w = __ballot(p);
    bw = lane == q ? w : bw;
  }
  const uint32_t bpc = (uint32_t)__popcll(bw), bin = scan_incl(bpc);
  const uint32_t Uc = lane_of(bin, kSpTableN / 64u - 1u);
  if (Uc > W * kWave) return kLeanFallback;

  // ---- members (as mask_object); dots in rounds of 64 (<= 128 per side)
  const bool hml = lane < nL, hmr = lane < nR;
  const uint32_t nrnd = (dL > dR ? dL : dR) > 64u ? 2u : 1u;
  const uint64_t kl = ld64(Ls, keyL + 8u * lane), kr = ld64(Rs, keyR + 8u * lane);
  uint32_t rl = 0, rr = 0;
  {
    const uint32_t n = nL > nR ? nL : nR;
    for (uint32_t step = n ? 1u << (31u - __builtin_clz(n)) : 0u; step != 0u; step >>= 1) {
      const uint32_t cl = rl + step, cr = rr + step;
      const uint64_t kcl = ld64(Rs, keyR + 8u * (cl - 1u)), kcr = ld64(Ls, keyL + 8u * (cr - 1u));
      rl = (cl <= nR && kcl < kl) ? cl : rl;
      rr = (cr <= nL && kcr < kr) ? cr : rr;
    }
  }
  const bool eql = hml && rl < nR && ld64(Rs, keyR + 8u * rl) == kl;
  const bool eqr = hmr && rr < nL && ld64(Ls, keyL + 8u * rr) == kr;
  const uint64_t EL = __ballot(eql), ER = __ballot(eqr);
  const uint32_t U = nL + nR - (uint32_t)__popcll(EL);
  if (U > (uint32_t)kWave) return kLeanFallback;
  const uint32_t ul = lane + rl - mbcnt64(EL), ur = lane + rr - mbcnt64(ER);

  wave_sync();  // the previous object's readers of this scratch are done
  if (lane < kSpTableN / 64u)
    *(u32x4*)(X + oUpre + 16u * lane) = u32x4{(uint32_t)bw, (uint32_t)(bw >> 32), bin - bpc, 0u};
  const u32x4 z4{0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t q = 0; q < W; ++q) {
    *(u32x4*)(X + oMsL + MS * lane + 16u * q) = z4;
    *(u32x4*)(X + oMsR + MS * lane + 16u * q) = z4;
  }
  if (lane < 4u) *(uint64_t*)(X + oHeads + 8u * lane) = 0ull;
  const uint32_t el0 = ld32(Ls, endL + 4u * lane - 4u), er0 = ld32(Rs, endR + 4u * lane - 4u);
  const uint32_t sl = lane ? el0 : 0u, sr = lane ? er0 : 0u;
  *(uint16_t*)(X + (hml ? oDesc + 2u * (ul & 63u) : tr)) =
      (uint16_t)(((eql ? kBoth : kSelf) << 12) | (lane << 6) | (eql ? rl : 0u));
  *(uint16_t*)(X + ((hmr && !eqr) ? oDesc + 2u * (ur & 63u) : tr)) = (uint16_t)((kOther << 12) | ((rr & 63u) << 6) | lane);
  X[oUofI + lane] = (uint8_t)ul;
  X[oUofJ + lane] = (uint8_t)ur;
  wave_sync();
  // run heads as bits: dot words 0 / 1 of each side (members' first dots)
  atomicOr((unsigned long long*)(X + ((hml && sl < 128u) ? oHeads + 8u * (sl >> 6) : tr)), 1ull << (sl & 63u));
  atomicOr((unsigned long long*)(X + ((hmr && sr < 128u) ? oHeads + 16u + 8u * (sr >> 6) : tr)), 1ull << (sr & 63u));
  wave_sync();
  // run-head masks of both rounds; the member of dot 64 r + lane is
  // (#heads at or below it) - 1
  const uint64_t HL0 = ldm64(X, oHeads) & lowmask64(dL), HL1 = ldm64(X, oHeads + 8u) & lowmask64(dL - 64u);
  const uint64_t HR0 = ldm64(X, oHeads + 16u) & lowmask64(dR), HR1 = ldm64(X, oHeads + 24u) & lowmask64(dR - 64u);
  bool foreign = false;
  uint32_t rXL[2] = {0u, 0u}, rXR[2] = {0u, 0u}, rBL[2] = {0u, 0u}, rBR[2] = {0u, 0u};
  uint32_t rML[2] = {0u, 0u}, rMR[2] = {0u, 0u};
  uint64_t rVL[2] = {0ull, 0ull}, rVR[2] = {0ull, 0ull};
#pragma unroll
  for (uint32_t rd = 0; rd < 2u; ++rd) {  // dot -> union rank (its bitmap bit checked) -> member masks
    if (rd >= nrnd) break;
    const uint32_t d = 64u * rd + lane;
    const bool hdl = d < dL, hdr = d < dR;
    const uint32_t xl = ld32(Ls, actL + 4u * d), xr = ld32(Rs, actR + 4u * d);
    const uint64_t vl = ld64(Ls, ctrL + 8u * d), vr = ld64(Rs, ctrR + 8u * d);
    const uint64_t HL = rd ? HL1 : HL0, HR = rd ? HR1 : HR0;
    const uint32_t ml = (rd ? (uint32_t)__popcll(HL0) : 0u) + mbcnt64(HL) + ((HL >> lane) & 1ull ? 1u : 0u) - 1u;
    const uint32_t mr = (rd ? (uint32_t)__popcll(HR0) : 0u) + mbcnt64(HR) + ((HR >> lane) & 1ull ? 1u : 0u) - 1u;
    const uint32_t xlc = xl < A ? xl : 0u, xrc = xr < A ? xr : 0u;
    const u32x4 pwl = *(const u32x4*)(X + oUpre + 16u * (xlc >> 6)), pwr = *(const u32x4*)(X + oUpre + 16u * (xrc >> 6));
    const uint64_t bwl = ((uint64_t)pwl.y << 32) | pwl.x, bwr = ((uint64_t)pwr.y << 32) | pwr.x;
    const uint32_t bl = (pwl.z + below64(bwl, xlc & 63u)) & 127u, br = (pwr.z + below64(bwr, xrc & 63u)) & 127u;
    rXL[rd] = xl; rXR[rd] = xr; rVL[rd] = vl; rVR[rd] = vr; rBL[rd] = bl; rBR[rd] = br; rML[rd] = ml; rMR[rd] = mr;
    foreign = foreign || (hdl && (xl >= A || ((bwl >> (xlc & 63u)) & 1ull) == 0ull)) ||
              (hdr && (xr >= A || ((bwr >> (xrc & 63u)) & 1ull) == 0ull));
    const uint64_t rc = ld64(Rs, kHdrBytes + 8u * xlc), lc = ld64(Ls, kHdrBytes + 8u * xrc);
    const uint64_t mbl = hdl ? 1ull << (bl & 63u) : 0ull, mbr = hdr ? 1ull << (br & 63u) : 0ull;
    const uint32_t ol = oMsL + MS * (ml & 63u) + 8u * (bl >> 6), orr = oMsR + MS * (mr & 63u) + 8u * (br >> 6);
    atomicOr((unsigned long long*)(X + (hdl ? ol : tr)), (unsigned long long)mbl);
    atomicOr((unsigned long long*)(X + (hdl ? ol + 8u * W : tr)), (unsigned long long)(vl > rc ? mbl : 0ull));
    atomicOr((unsigned long long*)(X + (hdr ? orr : tr)), (unsigned long long)mbr);
    atomicOr((unsigned long long*)(X + (hdr ? orr + 8u * W : tr)), (unsigned long long)(vr > lc ? mbr : 0ull));
  }
  if (__ballot(foreign) != 0ull) return kLeanFallback;  // a dot actor absent from both top clocks
  wave_sync();  // every dot has its rank: the prefix table's words are free
#pragma unroll
  for (uint32_t q = 0; q < W; ++q) *(u32x4*)(X + oEq + MS * lane + 16u * q) = z4;
  wave_sync();
#pragma unroll
  for (uint32_t rd = 0; rd < 2u; ++rd) {  // actors on both sides of a shared member: equal / self >= other
    if (rd >= nrnd) break;
    const bool hdr = 64u * rd + lane < dR;
    const uint64_t vr = rVR[rd];
    const uint32_t br = rBR[rd], mr = rMR[rd];
    const uint32_t u = X[oUofJ + (mr & 63u)] & 63u;
    const uint32_t d = *(const uint16_t*)(X + oDesc + 2u * u);
    const uint32_t i = (d >> 6) & 63u;
    const uint64_t mlo = ldm64(X, oMsL + MS * i), mhi = W == 2u ? ldm64(X, oMsL + MS * i + 8u) : 0ull;
    const bool sh = hdr && (d >> 12) == kBoth && bit128(mlo, mhi, br);
    const uint32_t a0 = i ? ld32(Ls, endL + 4u * i - 4u) : 0u;
    const uint64_t va = ld64(Ls, ctrL + 8u * ((a0 + below128(mlo, mhi, br)) & 127u));
    const uint32_t oe = oEq + MS * u + 8u * (br >> 6);
    const uint64_t bb = 1ull << (br & 63u);
    atomicOr((unsigned long long*)(X + (sh ? oe : tr)), (unsigned long long)(sh && va == vr ? bb : 0ull));
    atomicOr((unsigned long long*)(X + (sh ? oe + 8u * W : tr)), (unsigned long long)(sh && va >= vr ? bb : 0ull));
  }
  wave_sync();
  // ---- per union member: mask join (src/orswot.rs:94-138), word by word
  const bool hu = lane < U;
  const uint32_t dsc = hu ? *(const uint16_t*)(X + oDesc + 2u * lane) : 0u;
  const uint32_t ty = dsc >> 12, mi = (dsc >> 6) & 63u, mj = dsc & 63u;
  const bool self_only = ty == kSelf;
  uint64_t keep[2] = {0ull, 0ull}, useK[2] = {0ull, 0ull}, lpf = 0ull;
#pragma unroll
  for (uint32_t w = 0; w < W; ++w) {
    const uint64_t ML = (ty & kSelf) ? ldm64(X, oMsL + MS * mi + 8u * w) : 0ull;
    const uint64_t FL = (ty & kSelf) ? ldm64(X, oMsL + MS * mi + 8u * W + 8u * w) : 0ull;
    const uint64_t MR = (ty & kOther) ? ldm64(X, oMsR + MS * mj + 8u * w) : 0ull;
    const uint64_t FR = (ty & kOther) ? ldm64(X, oMsR + MS * mj + 8u * W + 8u * w) : 0ull;
    const uint64_t EQ = ty == kBoth ? ldm64(X, oEq + MS * lane + 8u * w) : 0ull;
    const uint64_t GE = ty == kBoth ? ldm64(X, oEq + MS * lane + 8u * W + 8u * w) : 0ull;
    const uint64_t lp = self_only ? ML : (ML & FL), rp = MR & FR;
    const uint64_t useA = (ML & MR & EQ) | (lp & (~rp | GE));
    keep[w] = useA | rp;
    useK[w] = useA;
    lpf |= ML & FL;
  }
#pragma unroll
  for (uint32_t w = 0; w < W; ++w) {
    keep[w] = (!hu || (self_only && lpf == 0ull)) ? 0ull : keep[w];
    useK[w] &= keep[w];
  }
  SideL DL{(lds_cu8*)(size_t)lds_addr(Ls), RV{}}, DR{(lds_cu8*)(size_t)lds_addr(Rs), RV{}};  // LDS stages: ds_* reads
  if (HD) {  // deferred removes (apply_deferred -> apply_remove, src/orswot.rs:235-243, 195-211)
    DL.v = make_rv(layout_at(Ls));
    DR.v = make_rv(layout_at(Rs));
    wave_sync();
    uint64_t* ow = (uint64_t*)(X + oOut + OS * lane);
    ow[0] = keep[0]; ow[W] = useK[0];
    if (W == 2u) { ow[1] = keep[1]; ow[3] = useK[1]; }
    wave_sync();
#pragma unroll
    for (uint32_t rd = 0; rd < 2u; ++rd) {
      if (rd >= nrnd) break;
      const uint32_t d = 64u * rd + lane;
      const bool hdl = d < dL, hdr = d < dR;
      const uint32_t bl = rBL[rd], br = rBR[rd], ml = rML[rd], mr = rMR[rd];
      if (hdl) {
        unsigned long long* ok = (unsigned long long*)(X + oOut + OS * X[oUofI + (ml & 63u)]);
        if (bit128(ok[W], W == 2u ? ok[3] : 0ull, bl)) {
          const uint64_t mk = dmask_of(DL, DR, ld64(Ls, keyL + 8u * (ml & 63u)));
          if (mk && dkilled(DL, DR, mk, rXL[rd], rVL[rd])) atomicAnd(ok + (bl >> 6), ~(1ull << (bl & 63u)));
        }
      }
      if (hdr) {
        unsigned long long* ok = (unsigned long long*)(X + oOut + OS * X[oUofJ + (mr & 63u)]);
        if (bit128(ok[0] & ~ok[W], W == 2u ? ok[1] & ~ok[3] : 0ull, br)) {
          const uint64_t mk = dmask_of(DL, DR, ld64(Rs, keyR + 8u * (mr & 63u)));
          if (mk && dkilled(DL, DR, mk, rXR[rd], rVR[rd])) atomicAnd(ok + (br >> 6), ~(1ull << (br & 63u)));
        }
      }
    }
    wave_sync();
    keep[0] = ow[0];
    keep[1] = W == 2u ? ow[1] : 0ull;
    useK[0] &= keep[0];
    useK[1] &= keep[1];
  }
  const uint32_t c = (uint32_t)__popcll(keep[0]) + (uint32_t)__popcll(keep[1]);
  // ---- output layout (dense top clock of A entries)
  const uint64_t keepm = __ballot(c != 0u);
  const uint32_t tot_mem = (uint32_t)__popcll(keepm);
  const uint32_t cincl = scan_incl(c);
  const uint32_t tot_dot = lane_of(cincl, kWave - 1);
  uint32_t nd = 0, ndd = 0, ndm = 0;
  // survivors cached past the {keep, useK, d0} rows (64 entries)
  uint32_t* dcache = (uint32_t*)(X + oCache);
  if (HD) deferred_pass_wave<false>(DL, DR, A, lane, nd, ndd, ndm, nullptr, dcache);
  RecLayout OL;
  rec_layout(OL, A, tot_mem, tot_dot, nd, ndd, ndm, false);
  const uint32_t size = OL.size;
  const uint32_t d0 = cincl - c;
  wave_sync();
  {
    uint64_t* ow = (uint64_t*)(X + oOut + OS * lane);
    ow[0] = keep[0]; ow[W] = useK[0];
    if (W == 2u) { ow[1] = keep[1]; ow[3] = useK[1]; }
    *(uint32_t*)(ow + 2u * W) = d0;
  }
  if (c != 0u) {
    const uint32_t midx = mbcnt64(keepm);
    const uint64_t kk = (ty & kSelf) ? ld64(Ls, keyL + 8u * mi) : ld64(Rs, keyR + 8u * mj);
    *(uint64_t*)(O + OL.o_key + 8u * midx) = kk;
    *(uint32_t*)(O + OL.o_mdend + 4u * midx) = d0 + c;
  }
  for (uint32_t a = lane; a < A; a += kWave) {  // top clock: dense, pointwise max of the rows (src/orswot.rs:153)
    const uint64_t l = ld64(Ls, kHdrBytes + 8u * a), r = ld64(Rs, kHdrBytes + 8u * a);
    *(uint64_t*)(O + kHdrBytes + 8u * a) = l > r ? l : r;
  }
  wave_sync();
  uint32_t* oact = (uint32_t*)(O + OL.o_dact);
  uint64_t* octr = (uint64_t*)(O + OL.o_dctr);
#pragma unroll
  for (uint32_t rd = 0; rd < 2u; ++rd) {  // every kept dot at its member's base + actor rank
    if (rd >= nrnd) break;
    const uint32_t d = 64u * rd + lane;
    const bool hdl = d < dL, hdr = d < dR;
    const uint32_t bl = rBL[rd], br = rBR[rd], ml = rML[rd], mr = rMR[rd];
    if (hdl) {
      const uint64_t* ob = (const uint64_t*)(X + oOut + OS * X[oUofI + (ml & 63u)]);
      const uint64_t k0 = ob[0], k1 = W == 2u ? ob[1] : 0ull, u0 = ob[W], u1 = W == 2u ? ob[3] : 0ull;
      if (bit128(u0, u1, bl)) {
        const uint32_t idx = *(const uint32_t*)(ob + 2u * W) + below128(k0, k1, bl);
        oact[idx] = rXL[rd];
        octr[idx] = rVL[rd];
      }
    }
    if (hdr) {
      const uint64_t* ob = (const uint64_t*)(X + oOut + OS * X[oUofJ + (mr & 63u)]);
      const uint64_t k0 = ob[0], k1 = W == 2u ? ob[1] : 0ull, u0 = ob[W], u1 = W == 2u ? ob[3] : 0ull;
      if (bit128(k0 & ~u0, k1 & ~u1, br)) {
        const uint32_t idx = *(const uint32_t*)(ob + 2u * W) + below128(k0, k1, br);
        oact[idx] = rXR[rd];
        octr[idx] = rVR[rd];
      }
    }
  }
  if (HD) {
    DefOut w{(uint64_t*)(O + OL.o_fctr), (uint64_t*)(O + OL.o_fkey), (uint32_t*)(O + OL.o_fact),
             (uint32_t*)(O + OL.o_fdend), (uint32_t*)(O + OL.o_fmend)};
    wave_sync();
    deferred_pass_wave<false>(DL, DR, A, lane, nd, ndd, ndm, &w, dcache, nd);
  }
  if (lane == 0u && OL.o_def != OL.o_mpad) *(uint32_t*)(O + OL.o_mpad) = 0u;
  if (lane >= 1u && lane < 4u && OL.o_end + 4u * (lane - 1u) < size) *(uint32_t*)(O + OL.o_end + 4u * (lane - 1u)) = 0u;
  if (lane == 0u) {
    u32x4* h = (u32x4*)O;
    h[0] = u32x4{size, A, tot_mem, tot_dot};
    h[1] = u32x4{nd, ndd, ndm, 0u};
  }
  return size / 16u;
}

// Copy an output record from its LDS stage to HBM: 16-B coalesced,
// non-temporal stores (the output is not re-read by this kernel).
__device__ __forceinline__ void copy_out(const u32x4* src, uint8_t* dst, uint32_t n16, uint32_t lane) {
  wave_sync();
  for (uint32_t k = lane; k < n16; k += kWave) __builtin_nontemporal_store(src[k], (u32x4*)dst + k);
}


// Branch-free forms for the mask kernel: every lane loads (indices past the
// record re-read its last piece, in bounds, merged by the address coalescer)
// and stores its pieces into the 2 KB stage (bytes past the record are never
// read as record data).
__device__ __forceinline__ void prefetch_all(u32x4 (&r)[kPer], const uint8_t* src, uint32_t n16, uint32_t lane) {
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t idx = lane + k * kWave;
    r[k] = __builtin_nontemporal_load((const u32x4*)src + (idx < n16 ? idx : n16 - 1u));
  }
}
__device__ __forceinline__ void stage_all(u32x4* dst, const u32x4 (&r)[kPer], uint32_t lane) {
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) dst[lane + k * kWave] = r[k];
}
// The same through a buffer resource over the record (base and size
// wave-uniform, in SGPRs): pieces past the record are out of range, so they
// return zeros without a memory access, and every lane's offset is a constant
// (no per-object clamp or 64-bit address arithmetic in VGPRs).
constexpr int kBufWord3 = 0x00020000;  // gfx9 buffer resource word 3: raw bytes
constexpr int kBufNT = 2;              // cache policy: nontemporal (gfx94x/gfx950 NT bit)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bytes_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, kBufWord3);
}
template <int AUX = kBufNT>
__device__ __forceinline__ void prefetch_buf(u32x4 (&r)[kPer], const uint8_t* src, uint32_t n16, uint32_t lane) {
  const __amdgpu_buffer_rsrc_t rs = bytes_rsrc(src, 16u * n16);
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) r[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * (lane + k * kWave)), 0, AUX);
}
// prefetch_all with the record base and its last piece made wave-uniform
// (SGPRs): each load is the SGPR base + a 32-bit lane offset (saddr form),
// so the per-load VALU is the clamp and the shift, no 64-bit address add
template <bool NT = true>  // (NT: non-temporal loads; false: default policy)
__device__ __forceinline__ void prefetch_sa(u32x4 (&r)[kPer], const uint8_t* src, uint32_t n16, uint32_t lane) {
  const uint64_t b = (uint64_t)src;
  typedef const __attribute__((address_space(1))) u32x4 gu32x4;
  const __attribute__((address_space(1))) uint8_t* s = (const __attribute__((address_space(1))) uint8_t*)(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b));  // (int -> u32 first: no sign extension)
  const uint32_t last = __builtin_amdgcn_readfirstlane(n16 - 1u);
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t idx = lane + k * kWave;
    if constexpr (NT) r[k] = __builtin_nontemporal_load((gu32x4*)(s + 16u * (idx < last ? idx : last)));
    else r[k] = *(gu32x4*)(s + 16u * (idx < last ? idx : last));
  }
}
// prefetch_sa with the clamp done on byte offsets (one v_min per load: the
// lane's offset against the wave-uniform offset of the last piece)
__device__ __forceinline__ void prefetch_sb(u32x4 (&r)[kPer], const uint8_t* src, uint32_t n16, uint32_t lane) {
  const uint64_t b = (uint64_t)src;
  typedef const __attribute__((address_space(1))) u32x4 gu32x4;
  const __attribute__((address_space(1))) uint8_t* s = (const __attribute__((address_space(1))) uint8_t*)(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b));  // (int -> u32 first: no sign extension)
  const uint32_t lastb = 16u * __builtin_amdgcn_readfirstlane(n16 - 1u);
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t ob = 16u * (lane + k * kWave);
    r[k] = __builtin_nontemporal_load((gu32x4*)(s + (ob < lastb ? ob : lastb)));
  }
}
// copy_record_out with the clamp on byte offsets (wave-uniform last piece)
__device__ __forceinline__ void copy_record_sb(uint32_t src, uint8_t* O, uint32_t n16, uint32_t lane) {
  const uint32_t lastb = 16u * __builtin_amdgcn_readfirstlane(n16 - 1u);
  const uint32_t b0 = 16u * lane, b1 = 16u * (lane + kWave);
  const uint32_t o0 = b0 < lastb ? b0 : lastb, o1 = b1 < lastb ? b1 : lastb;
  const u32x4 p0 = *(const __attribute__((address_space(3))) u32x4*)(size_t)(src + o0);
  const u32x4 p1 = *(const __attribute__((address_space(3))) u32x4*)(size_t)(src + o1);
  __builtin_nontemporal_store(p0, (u32x4*)(O + o0));
  __builtin_nontemporal_store(p1, (u32x4*)(O + o1));
}
// copy_record_out through a buffer resource of the record's n16 pieces: the
// stores of lanes past the record are dropped (the instruction count is fixed)
__device__ __forceinline__ void copy_record_buf(uint32_t src, uint8_t* O, uint32_t n16, uint32_t lane) {
  const __amdgpu_buffer_rsrc_t rs = bytes_rsrc(O, 16u * n16);
  const u32x4 p0 = *(const __attribute__((address_space(3))) u32x4*)(size_t)(src + 16u * lane);
  const u32x4 p1 = *(const __attribute__((address_space(3))) u32x4*)(size_t)(src + 16u * (lane + kWave));
  __builtin_amdgcn_raw_buffer_store_b128(p0, rs, (int)(16u * lane), 0, kBufNT);
  __builtin_amdgcn_raw_buffer_store_b128(p1, rs, (int)(16u * (lane + kWave)), 0, kBufNT);
}
// The join kernel's record prefetch / copy-out by its IO variant (see
// orswot_join_kernel): 0 clamped global loads / stores, 1-3 buffer
// resources, 4 and 7 the saddr prefetch, 5-6 the byte-clamped prefetch;
// copy-out byte-clamped for 5 and 7 (a carried-offset form, the current
// object's offsets kept in SGPRs from the iteration that prefetched it,
// spilled SGPRs: 0.789 vs 0.753 ms)
template <int IO>
__device__ __forceinline__ void prefetch_io(u32x4 (&r)[kPer], const uint8_t* src, uint32_t n16, uint32_t lane) {
  if constexpr (IO >= 1 && IO <= 3)
    prefetch_buf<IO == 3 ? 0 : kBufNT>(r, src, n16, lane);
  else if constexpr (IO == 4 || IO == 7)
    prefetch_sa(r, src, n16, lane);
  else if constexpr (IO == 5 || IO == 6)
    prefetch_sb(r, src, n16, lane);
  else
    prefetch_all(r, src, n16, lane);
}
template <int IO>
__device__ __forceinline__ void copy_io(uint32_t src, uint8_t* O, uint32_t n16, uint32_t lane) {
  if constexpr (IO == 2)
    copy_record_buf(src, O, n16, lane);
  else if constexpr (IO == 5 || IO == 7)
    copy_record_sb(src, O, n16, lane);
  else
    copy_record_out(src, O, n16, lane);
}
// Only the 64-piece rounds a record of n16 pieces reaches (n16 wave-uniform).
__device__ __forceinline__ void stage_used(u32x4* dst, const u32x4 (&r)[kPer], uint32_t n16, uint32_t lane) {
  dst[lane] = r[0];
#pragma unroll
  for (uint32_t k = 1; k < kPer; ++k)
    if (n16 > k * kWave) dst[lane + k * kWave] = r[k];
}


#ifdef CRDT_DIAG
#include "diag/orswot_kernels_diag.inc"  // the v6 mask kernel, orswot_join_kernel<...>
#endif


constexpr uint32_t kGenStage = 8192;
constexpr uint32_t kGenBlocks = 1536;  // 6 resident 24 KB-LDS blocks per CU

// (the big-object kernel's share of the general list: see orswot_big_kernel)
constexpr uint32_t kBigW = 8;           // waves per block
constexpr uint32_t kBigStage = 32768;   // LDS stage per record

#ifndef CRDT_BIG_MIN_POS
#define CRDT_BIG_MIN_POS 128
#endif
constexpr uint32_t kBigMinPos = CRDT_BIG_MIN_POS;  // union positions past which an object takes the block join

__device__ __forceinline__ bool is_big(u32x4 hl0, u32x4 hr0) {
  return hl0.z + hr0.z > kBigMinPos || hl0.x > kGenStage || hr0.x > kGenStage;
}


// ---- the object lists behind a join launch. The context's list buffer is
// split in two halves of list_cap entries each (the launchers halve the
// context's capacity): [0, list_cap) the general kernel's list (count ctl[0]),
// [list_cap, 2 list_cap) the big-object list (count ctl[2] & kBigCount).
// Objects are appended with one atomic per wave and list (a per-lane atomic
// on one address serialises at the memory side: 49k of them cost the join
// ~80 us, r06). Past a half's capacity the consumers scan the pending flags.
constexpr uint32_t kBigCount = 0x7FFFFFFFu;  // ctl[2]: big-list count; bit 31: the general kernel left big objects
constexpr uint32_t kBigLeft = 0x80000000u;
__device__ __forceinline__ void list_append(bool put, uint64_t obj, uint32_t* ctr, uint64_t* dst, uint32_t cap,
                                            uint32_t lane) {
  const uint64_t m = __ballot(put);
  if (m == 0ull) return;
  uint32_t base = 0u;
  if (lane == 0u) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = (uint32_t)__builtin_amdgcn_readfirstlane(base);
  const uint32_t e = base + mbcnt64(m);
  if (put && e < cap) dst[e] = obj;
}

// ======================================================================
// The product join (round 5 form): orswot_join_kernel's product
// instantiation written out with only the product's choices — one pass,
// the guided split (5/8 static chunks, 20-object tickets), the saddr record
// prefetch one object ahead into registers, mask3_object for every object
// (its HD form with direct stores for the ~5 % with deferred removes), the
// packed two-sided rank search and the bank-conflict scratch layout.
// FL (diagnostic knobs, measured and not kept): 1 the chunk's
// output offsets in one coalesced store at its end; 8 record loads with the
// default (temporal) cache policy. (Whole-line output heads / tails, FL 2 / 4
// in round 5, were removed: 0.739-0.784 vs 0.736 ms.)
// ======================================================================
template <int MINW, int AW, int FL>
__global__ __launch_bounds__(kWave * kWavesPerBlock, MINW) void orswot_join5_kernel(
    const uint8_t* __restrict__ Lb, const uint64_t* __restrict__ Loff, uint64_t Lbytes,
    const uint8_t* __restrict__ Rb, const uint64_t* __restrict__ Roff, uint64_t Rbytes,
    uint8_t* __restrict__ Ob, uint64_t* __restrict__ Ooff, uint64_t Obytes, uint64_t n_obj, uint32_t A,
    int* __restrict__ status, uint32_t* __restrict__ ctl, uint64_t* __restrict__ list, uint32_t list_cap) {
#ifndef CRDT_DIAG
  static_assert(FL == 0, "FL knobs exist in -DCRDT_DIAG builds only");
#endif
  __shared__ u32x4 stage_s[kWavesPerBlock][2][kFastStage / 16];
  __shared__ u32x4 scr_s[kWavesPerBlock][M3Lay<AW>::Bytes / 16];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wave = uni(threadIdx.x / kWave);  // wave-uniform: LDS bases in SGPRs
  u32x4* const sL = stage_s[wave][0];
  u32x4* const sR = stage_s[wave][1];
  const uint32_t uX = lds_addr(scr_s[wave]);
  const uint64_t wave_id = (uint64_t)blockIdx.x * kWavesPerBlock + wave;
  const uint64_t n_waves = (uint64_t)gridDim.x * kWavesPerBlock;
  uint8_t* const sink = (uint8_t*)(list + kDefaultListCap) + 64u * (uint32_t)(wave_id % kTrashWaves);
  GuidedSplit<20u, 5u, 0u> gs(n_obj, wave_id, n_waves);
  uint64_t cbase, cend;
  while (gs.next(cbase, cend, &ctl[3], lane)) {
    // ---- chunk step: lane k <-> object cbase + k (offsets, headers, verdicts)
    u32x4 pl[kPer], pr[kPer];  // record prefetch registers
    const uint64_t obj = cbase + lane;
    const bool valid = obj < cend;
    uint64_t lo = 0, ro = 0;
    u32x4 hl0 = {0, 0, 0, 0}, hl1 = hl0, hr0 = hl0, hr1 = hl0;
    uint64_t nlo = Lbytes, nro = Rbytes;
    if (valid) { lo = Loff[obj]; ro = Roff[obj]; }
    if (valid && obj + 1u < n_obj) { nlo = Loff[obj + 1u]; nro = Roff[obj + 1u]; }  // same lines: coalesced
    bool ok = valid && (lo & 15u) == 0 && (ro & 15u) == 0 && lo + kHdrBytes <= Lbytes && ro + kHdrBytes <= Rbytes;
    if (ok) {
      hl0 = ((const u32x4*)(Lb + lo))[0]; hl1 = ((const u32x4*)(Lb + lo))[1];
      hr0 = ((const u32x4*)(Rb + ro))[0]; hr1 = ((const u32x4*)(Rb + ro))[1];
    }
    ok = ok && header_ok(hl0, hl1, lo, Lbytes, A) && header_ok(hr0, hr1, ro, Rbytes, A) &&
         lo + ro + (uint64_t)hl0.x + hr0.x <= Obytes;
    // output placement precondition (out[i] at self.off[i] + other.off[i]):
    // each side's records in increasing offset order, none overlapping the next
    const bool placed = !ok || (nlo >= lo + hl0.x && nro >= ro + hr0.x);
    if (__ballot(!placed) != 0ull && lane == 0) atomicCAS(status, 0, CRDT_EINVAL);
    ok = ok && placed;
    const bool fits = ok && hl0.x <= kFastStage && hr0.x <= kFastStage && A <= (uint32_t)AW && hl0.z <= 64u &&
                      hr0.z <= 64u && hl0.w <= 64u && hr0.w <= 64u;
    const bool hd = fits && (hl1.x | hr1.x) != 0u && hl1.x <= 32u && hr1.x <= 32u;
    const bool fast = (fits && (hl1.x | hr1.x) == 0u) || hd;
    const uint64_t defs = __ballot(hd);
    const bool gen = ok && !fast;
    // objects the general kernel joins (listed here, or falling back in the
    // loop): FL 1 keeps them as a wave mask and stores the chunk's offsets
    // once, at its end (no per-lane 64-bit value kept across the loop)
    uint64_t pendm = __ballot(gen);
    if (!(FL & 1) && valid) Ooff[obj] = (lo + ro) | (gen ? kPending : 0ull);
    // hand the object to the general kernel, or straight to orswot_big_kernel
    // when its headers already say it is big (is_big)
    const bool bigo = gen && is_big(hl0, hr0);
    list_append(gen && !bigo, obj, &ctl[0], list, list_cap, lane);
    list_append(bigo, obj, &ctl[2], list + list_cap, list_cap, lane);
    if (__ballot(valid && !ok && placed) != 0ull && lane == 0) atomicCAS(status, 0, CRDT_ENONCANON);
    const uint64_t runs = __ballot(fast);
    if (runs == 0ull) {
      if ((FL & 1) && valid) Ooff[obj] = (lo + ro) | (gen ? kPending : 0ull);
      continue;
    }
    const uint32_t n16 = fast ? (hl0.x / 16u) | ((hr0.x / 16u) << 16) : 0u;
    const uint32_t nm = hl0.z | (hr0.z << 16), nd = hl0.w | (hr0.w << 16);

    // ---- software pipeline: the next object's records are in flight while
    // the current one is joined from LDS (loop rotated: the wait for a
    // prefetch has one predecessor, the previous object's stores)
    uint64_t pend = runs;
    uint32_t t = (uint32_t)__builtin_ctzll(pend);
    pend &= pend - 1;
    {
      const uint32_t nn = lane_of(n16, t);
      prefetch_sa<!(FL & 8)>(pl, Lb + lane_of64(lo, t), nn & 0xFFFFu, lane);
      prefetch_sa<!(FL & 8)>(pr, Rb + lane_of64(ro, t), nn >> 16, lane);
    }
    wave_sync();  // the previous chunk's last LDS reads are done
    stage_all(sL, pl, lane);
    stage_all(sR, pr, lane);
    wave_sync();
    for (;;) {
      const uint64_t oo = lane_of64(lo, t) + lane_of64(ro, t);
      const uint32_t m = lane_of(nm, t), d = lane_of(nd, t);
      // the next object, or this one again after the chunk's last (a constant load count)
      const uint32_t u = pend ? (uint32_t)__builtin_ctzll(pend) : t;
      const uint32_t nu = lane_of(n16, u);
      prefetch_sa<!(FL & 8)>(pl, Lb + lane_of64(lo, u), nu & 0xFFFFu, lane);
      prefetch_sa<!(FL & 8)>(pr, Rb + lane_of64(ro, u), nu >> 16, lane);
      bool big = false;
      uint32_t r;
      const bool dt = (defs >> t) & 1ull;
      if (dt) {
        r = mask3_object<0xFFFFFFFFu, 0, true, 0, true, 0, true, 1, AW>(lds_addr(sL), lds_addr(sR), uX, Ob + oo, A,
                                                                       m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16,
                                                                       lane, big);
      } else {
        r = mask3_object<0xFFFFFFFFu, 3, false, 0, true, 0, true, 1, AW>(lds_addr(sL), lds_addr(sR), uX, Ob + oo, A,
                                                                        m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16,
                                                                        lane, big, sink);
      }
      const bool fbu = big || r == kLeanFallback;  // wave-uniform
      wave_sync();
      if (dt) {  // the same two stores, to the sink (a constant store count per object)
        const u32x4 z = {0u, 0u, 0u, 0u};
        __builtin_nontemporal_store(z, (u32x4*)sink);
        __builtin_nontemporal_store(z, (u32x4*)sink + 1);
      } else {
        copy_io<7>(lds_addr(sL), Ob + oo, fbu ? 1u : r, lane);
      }
      if (FL & 1) {
        pendm |= fbu ? 1ull << t : 0ull;
      } else {
        *(Ooff + cbase + t) = oo | (fbu ? kPending : 0ull);
      }
      if (fbu && lane == 0u) {  // listed for the general kernel (rare)
        const uint32_t e = atomicAdd(&ctl[0], 1u);
        if (e < list_cap) list[e] = cbase + t;
      }
      if (pend == 0ull) break;
      t = u;
      pend &= pend - 1;
      wave_sync();  // this object's LDS reads are done
      stage_used(sL, pl, nu & 0xFFFFu, lane);
      stage_used(sR, pr, nu >> 16, lane);
      wave_sync();
    }
    if ((FL & 1) && valid) Ooff[obj] = (lo + ro) | ((pendm >> lane) & 1ull ? kPending : 0ull);  // one coalesced store
  }
}

#ifdef CRDT_DIAG
#include "diag/orswot_ring_diag.inc"  // the LDS-DMA ring kernel (r05, not kept)
#endif

// ======================================================================
// General path: objects the fast kernel flagged (records larger than its
// stage, > 64 members or dots on a side, > 32 deferred clocks on a side). The
// fast kernel appends them to a list; a grid of single-wave blocks (6 per CU,
// LDS-bound) joins each one from LDS stages of kGenStage per record, the next
// listed object's offsets and headers in flight meanwhile, and clears its
// flag. Objects past 128 union positions or the stage (is_big) are left
// flagged for orswot_big_kernel, launched after it. If the list overflowed,
// both kernels scan every output offset for flags instead. The list counter
// is cleared by the alternating control-word sets (launch_join_passes).
// ======================================================================
// A listed object's offsets and headers, loaded ahead of its join.
struct GenPre {
  uint64_t o, oo;
  bool pend;  // still flagged (orswot_dense_wide_kernel clears the objects it joins)
  const uint8_t* lr;
  const uint8_t* rr;
  u32x4 hl0, hl1, hr0, hr1;
};
// the offsets (one round trip), then the header loads issued (not waited on)
__device__ __forceinline__ void gen_pre(GenPre& g, const uint8_t* Lb, const uint64_t* Loff, const uint8_t* Rb,
                                        const uint64_t* Roff, const uint64_t* Ooff, uint64_t o) {
  g.o = o;
  const uint64_t f = Ooff[o];
  g.oo = f & ~kPending;
  g.pend = (f & kPending) != 0ull;
  g.lr = Lb + Loff[o];
  g.rr = Rb + Roff[o];
  g.hl0 = ((const u32x4*)g.lr)[0];
  g.hl1 = ((const u32x4*)g.lr)[1];
  g.hr0 = ((const u32x4*)g.rr)[0];
  g.hr1 = ((const u32x4*)g.rr)[1];
}

// One listed object; `mid` runs once the records are staged (or at once for
// an object this kernel leaves to orswot_big_kernel): the caller's loads for
// the next object, in flight during this one's join.
// (returns true for an object it leaves to orswot_big_kernel)
template <class Mid>
__device__ __forceinline__ bool general_one(const GenPre& g, uint8_t* Ob, uint64_t* Ooff, uint32_t A, u32x4* sl,
                                            u32x4* sr, u32x4* so, uint32_t lane, Mid&& mid) {
  const uint64_t o = g.o, oo = g.oo;
  const uint8_t* lr = g.lr;
  const uint8_t* rr = g.rr;
  const u32x4 hl0 = g.hl0, hl1 = g.hl1, hr0 = g.hr0, hr1 = g.hr1;
  const uint32_t szl = uni(hl0.x), szr = uni(hr0.x);
  if (!uni((uint32_t)g.pend)) {  // listed, then joined by orswot_dense_wide_kernel
    mid();
    return false;
  }
  if (is_big(u32x4{szl, 0u, uni(hl0.z), 0u}, u32x4{szr, 0u, uni(hr0.z), 0u})) {  // orswot_big_kernel's
    mid();
    return true;
  }
  if (szl > kGenStage || szr > kGenStage) mid();
  if (szl <= kGenStage && szr <= kGenStage) {
    wave_sync();
    // both records staged 4 KB per side at a time: every load of a round is
    // issued before its stores (one memory round trip per 4 KB, not per 1 KB)
    {
      constexpr uint32_t kB = 4;
      const uint32_t nl = szl / 16, nr = szr / 16, nmax = nl > nr ? nl : nr;
      for (uint32_t k0 = 0; k0 < nmax; k0 += kB * kWave) {
        u32x4 tl[kB], tr[kB];
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
          const uint32_t k = k0 + j * kWave + lane;
          if (k < nl) tl[j] = ((const u32x4*)lr)[k];
          if (k < nr) tr[j] = ((const u32x4*)rr)[k];
        }
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
          const uint32_t k = k0 + j * kWave + lane;
          if (k < nl) sl[k] = tl[j];
          if (k < nr) sr[k] = tr[j];
        }
      }
    }
    mid();
    wave_sync();
    // the join kernel's mask3 join when its limits hold (<= 64 members and
    // dots per side, <= 32 deferred clocks per side, A <= 64: in config 3 the
    // objects sent here are records just past the join kernel's 2 KB stage),
    // else the older fast join, with the general kernel's larger stages
    uint32_t n16 = ~0u;
    const uint32_t nL = uni(hl0.z), nR = uni(hr0.z), dL = uni(hl0.w), dR = uni(hr0.w);
    bool done = false;
    if (A <= 64u && nL <= 64u && nR <= 64u && dL <= 64u && dR <= 64u && uni(hl1.x) <= 32u && uni(hr1.x) <= 32u) {
      bool big = false;
      const bool hd = (uni(hl1.x) | uni(hr1.x)) != 0u;
      uint32_t r;
      if (A <= 32u)
        r = hd ? mask3_object<0xFFFFFFFFu, 0, true>(lds_addr(sl), lds_addr(sr), lds_addr(so), Ob + oo, A, nL, dL, nR,
                                                    dR, lane, big)
               : mask3_object<0xFFFFFFFFu, 0, false>(lds_addr(sl), lds_addr(sr), lds_addr(so), Ob + oo, A, nL, dL, nR,
                                                     dR, lane, big);
      else  // 33-64 actors: the 64-bit actor-mask form of join5<5, 64> (M3Lay<64> fits the scratch)
        r = hd ? mask3_object<0xFFFFFFFFu, 0, true, 0, true, 0, true, 1, 64>(lds_addr(sl), lds_addr(sr), lds_addr(so),
                                                                             Ob + oo, A, nL, dL, nR, dR, lane, big)
               : mask3_object<0xFFFFFFFFu, 0, false, 0, true, 0, true, 1, 64>(lds_addr(sl), lds_addr(sr), lds_addr(so),
                                                                              Ob + oo, A, nL, dL, nR, dR, lane, big);
      done = r != kLeanFallback && !big;
      wave_sync();  // the scratch (so) is reused below
    }
    if (!done && nL + nR <= 2u * kWave && uni(hl1.x) <= 32u && uni(hr1.x) <= 32u) {
      const FOut fo{so, Ob + oo, o, Ooff, nullptr, nullptr, 0u};
      Stamps st{};
      if ((uni(hl1.x) | uni(hr1.x)) != 0u)
        n16 = fast_object<true, 0, kGenStage, true>((const uint8_t*)sl, (const uint8_t*)sr, fo, A, nL, dL, nR, dR,
                                                    lane, st);
      else
        n16 = fast_object<false, 0, kGenStage, true>((const uint8_t*)sl, (const uint8_t*)sr, fo, A, nL, dL, nR, dR,
                                                     lane, st);
    }
    if (done) {
    } else if (n16 != ~0u) {
      copy_out(so, Ob + oo, n16, lane);
    } else {
      merge_object((const uint8_t*)sl, (const uint8_t*)sr, Ob + oo, A, lane);
    }
  } else {
    merge_object(lr, rr, Ob + oo, A, lane);
  }
  if (lane == 0) Ooff[o] = oo;
  return false;
}

// ======================================================================
// Big objects (round 5): the general path's objects with more than 128 union
// positions or a record past the general stage (kGenStage) — the heavy tail
// of a batch (the reference's entries map is unbounded, src/orswot.rs:26-30)
// — joined by a whole workgroup of kBigW waves per object instead of one
// wave: merge_object's two passes with the 64-position chunks of the member
// union dealt round-robin to the waves. Between them a block-wide exclusive
// scan of the per-chunk member / dot totals. A boundary table (the self-key
// count at every 64th union position, one full merge-path search per chunk)
// narrows each position's search to a 65-entry window (7 steps), and pass 1
// leaves each position's candidate and dot count in LDS for pass 2 (which
// then runs only the joins of kept members). Both records are staged in LDS
// when each fits kBigStage; larger ones are read from HBM, the tables then
// carved from the unused stage. Same rules and output as merge_object
// (src/orswot.rs:87-157 with apply_deferred).
// ======================================================================
constexpr uint32_t kBigChS = 96;     // chunk capacity, staged records (<= 86 possible: 12 B a member at least)
constexpr uint32_t kBigChH = 4096;   // chunk capacity, records from HBM (P <= 262 144; past it: one wave)
constexpr uint32_t kBigPos = 4096;   // positions whose candidate / count pass 1 keeps in LDS

// ABL 8 (diag): wave 0's per-phase cycles of the big-object join, summed over
// objects (crdt_debug_big_stamps reads and clears them)
#ifdef CRDT_DIAG
__device__ unsigned long long g_big_st[16];
#endif
template <int ABL>
__device__ __forceinline__ void bst(uint64_t& last, uint32_t k, uint32_t wave, uint32_t lane) {
#ifdef CRDT_DIAG
  if constexpr (ABL == 8) {
    if (wave == 0u) {
      const uint64_t t = stamp();
      if (lane == 0u) atomicAdd(&g_big_st[k], (unsigned long long)(t - last));
      last = t;
    }
  }
#endif
}

struct BigTabs {
  uint32_t* tot;  // 2 x cap: per-chunk kept members, then dots (then their exclusive prefixes)
  uint32_t* spl;  // cap + 1: self keys before each chunk's first position
  uint16_t* pq;   // kBigPos: (type << 14) | i of each position
  uint8_t* pc;    // kBigPos: its joined dot count (255: count again)
  uint32_t* bc;   // 4: grand totals
  uint32_t cap;
  uint32_t* bloom;  // 32: the deferred member filter (dm_maybe)
  uint64_t* last;   // (ABL 8: wave 0's stamp)
  uint8_t* crank;   // SP: 2 x kRankTab actor -> rank tables of both top clocks (topr), or null
};

// merge_path with the answer known to lie in [ilo, ihi], ihi - ilo <= 64.
template <class S>
__device__ __forceinline__ uint32_t merge_path_in(const S& L, const S& R, uint32_t p, uint32_t ilo, uint32_t ihi,
                                                  uint32_t& i, uint32_t& j) {
  const uint32_t nL = L.v.n_mem, nR = R.v.n_mem;
  uint32_t lo = p > nR ? p - nR : 0u, hi = p < nL ? p : nL;
  lo = lo > ilo ? lo : ilo;
  hi = hi < ihi ? hi : ihi;
  uint32_t len = hi > lo ? hi - lo : 0u;
#pragma unroll
  for (uint32_t s = 0; s < 7u; ++s) {
    const uint32_t half = len >> 1, mid = lo + half;
    const bool go = len != 0 && g64(L.b, L.v.key, mid) <= g64(R.b, R.v.key, p - 1 - mid);
    lo = go ? mid + 1 : lo;
    len = len == 0 ? 0 : (go ? len - half - 1 : half);
  }
  i = lo;
  j = p - lo;
  const uint64_t kl = i < nL ? g64(L.b, L.v.key, i) : ~0ull;
  const uint64_t kr = j < nR ? g64(R.b, R.v.key, j) : ~0ull;
  if (i < nL && (j >= nR || kl <= kr)) return (j < nR && kl == kr) ? kBoth : kSelf;
  if (i > 0 && g64(L.b, L.v.key, i - 1) == kr) return kNone;  // twin of a kBoth at p-1
  return kOther;
}

// (ABL, timing only in diag variants: 1 no kill test, 2 no deferred block,
// 3 no pass 2, 4 no pass 1 join; 6 — a real variant — no register cache of
// the first two chunks, pass 2 from the LDS cache only)
template <bool SP, int ABL = 0, class S>
__device__ __forceinline__ void merge_object_block(const S& L, const S& R, uint8_t* O, uint32_t A, uint32_t lane,
                                                   uint32_t wave, const BigTabs& T) {
  const bool has_def = ABL != 1 && (L.v.n_def | R.v.n_def) != 0;
  const uint32_t P = L.v.n_mem + R.v.n_mem;
  const uint32_t nch = (P + kWave - 1) / kWave;
  uint32_t n_clk = A;
  if constexpr (SP) n_clk = uni(sparse_clock_join(L, R, nullptr, 0u, lane));
  // SP: both top clocks' actor -> rank tables (clocks of <= 255 entries over
  // actor ids < kRankTab; others keep the binary search)
  lds_cu8* crank = nullptr;
  if (SP && T.crank != nullptr && L.v.n_clk <= 255u && R.v.n_clk <= 255u) {
    uint32_t* z = (uint32_t*)T.crank;
    for (uint32_t k = threadIdx.x; k < 2u * kRankTab / 4u; k += kWave * kBigW) z[k] = 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < L.v.n_clk + R.v.n_clk; k += kWave * kBigW) {
      const bool isL = k < L.v.n_clk;
      const uint32_t e = isL ? k : k - L.v.n_clk;
      const uint32_t x = isL ? g32(L.b, L.v.cact, e) : g32(R.b, R.v.cact, e);
      if (x < kRankTab) T.crank[(isL ? 0u : kRankTab) + x] = (uint8_t)(e + 1u);
    }
    crank = (lds_cu8*)(size_t)lds_addr(T.crank);
  }
  // ---- the deferred member filter (both sides' deferred member keys)
  if (has_def) {
    if (threadIdx.x < 32u) T.bloom[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < L.v.n_dm + R.v.n_dm; k += kWave * kBigW) {
      const uint64_t m = k < L.v.n_dm ? g64(L.b, L.v.fkey, k) : g64(R.b, R.v.fkey, k - L.v.n_dm);
      const uint32_t h = dm_hash(m);
      atomicOr(&T.bloom[h >> 5], 1u << (h & 31u));
    }
  }
  // ---- chunk boundaries: the merge-path split at every 64th position
  for (uint32_t c = threadIdx.x; c <= nch; c += kWave * kBigW) {
    const uint32_t p = kWave * c < P ? kWave * c : P;
    uint32_t i, j;
    merge_path(L, R, p, i, j);
    T.spl[c] = i;
  }
  __syncthreads();
  if (T.last) bst<ABL>(*T.last, 2, wave, lane);
  // ---- pass 1: per chunk (64 union positions) its kept members and dots;
  // a wave's first two chunks stay in registers for pass 2, every position
  // below kBigPos leaves its candidate and count in LDS
  uint32_t q0 = 0, c0 = 0, x0 = 0, q1 = 0, c1 = 0, x1 = 0;
  uint64_t v0 = 0, v1 = 0;
  for (uint32_t ch = wave, k = 0; ch < nch; ch += kBigW, ++k) {
    const uint32_t p = kWave * ch + lane;
    const uint32_t ilo = uni(T.spl[ch]), ihi = uni(T.spl[ch + 1]);
    uint32_t type = kNone, i = 0, j = 0, cnt = 0, x = 0;
    uint64_t v = 0;
    if (p < P) {
      type = merge_path_in(L, R, p, ilo, ihi, i, j);
      if (ABL == 4) cnt = type != kNone;
      else if (type != kNone) cnt = join<0, SP>(L, R, type, i, j, A, has_def, x, v, nullptr, nullptr, 0, T.bloom, crank);
      if (p < kBigPos) {
        T.pq[p] = (uint16_t)((type << 14) | i);
        T.pc[p] = (uint8_t)(cnt < 255u ? cnt : 255u);
      }
    }
    const uint32_t q = (type << 30) | (i << 15) | j;  // (k < 2: p < 1024)
    if (ABL != 6 && k == 0) { q0 = q; c0 = cnt; x0 = x; v0 = v; }
    else if (ABL != 6 && k == 1) { q1 = q; c1 = cnt; x1 = x; v1 = v; }
    const uint32_t m = (uint32_t)__popcll(__ballot(cnt != 0)), d = wave_sum(cnt);
    if (lane == 0u) { T.tot[ch] = m; T.tot[T.cap + ch] = d; }
  }
  __syncthreads();
  if (T.last) bst<ABL>(*T.last, 3, wave, lane);
  // ---- exclusive prefix of the chunk totals (wave 0), and the grand totals
  // (every wave scanning the table itself, no barrier, measured the same:
  // the CU's two objects are bound by their joins, not by this wait)
  if (wave == 0u) {
    uint32_t cm = 0, cd = 0;
    for (uint32_t b = 0; b < nch; b += kWave) {
      const uint32_t ch = b + lane;
      const uint32_t m = ch < nch ? T.tot[ch] : 0u, d = ch < nch ? T.tot[T.cap + ch] : 0u;
      const uint32_t im = wave_incl_scan(m, lane), id = wave_incl_scan(d, lane);
      if (ch < nch) { T.tot[ch] = cm + im - m; T.tot[T.cap + ch] = cd + id - d; }
      cm += lane_of(im, kWave - 1);
      cd += lane_of(id, kWave - 1);
    }
    if (lane == 0u) { T.bc[0] = cm; T.bc[1] = cd; }
  }
  __syncthreads();
  const uint32_t tot_mem = uni(T.bc[0]), tot_dot = uni(T.bc[1]);
  if (T.last) bst<ABL>(*T.last, 4, wave, lane);
  const uint32_t o_key = kHdrBytes + clock_bytes(n_clk, SP);
  const uint32_t o_dctr = o_key + 8u * tot_mem;
  const uint32_t o_dact = o_dctr + 8u * tot_dot;
  const uint32_t o_mdend = o_dact + 4u * tot_dot;
  const uint32_t o_mpad = o_mdend + 4u * tot_mem;
  const uint32_t o_def = (o_mpad + 7u) & ~7u;
  uint64_t* okey = (uint64_t*)(O + o_key);
  uint64_t* odctr = (uint64_t*)(O + o_dctr);
  uint32_t* odact = (uint32_t*)(O + o_dact);
  uint32_t* omdend = (uint32_t*)(O + o_mdend);
  // top clock: pointwise max (src/orswot.rs:153 -> src/vclock.rs:131-137)
  if constexpr (SP) {
    if (wave == 0u) {
      sparse_clock_join(L, R, O, n_clk, lane);
      if (lane == 0u && (n_clk & 1u)) *(uint32_t*)(O + kHdrBytes + 12u * n_clk) = 0u;  // pad to 8
    }
  } else {
    for (uint32_t a = wave * kWave + lane; a < A; a += kBigW * kWave) {
      const uint64_t x = g64(L.b, L.v.clk, a), y = g64(R.b, R.v.clk, a);
      ((uint64_t*)(O + kHdrBytes))[a] = x > y ? x : y;
    }
  }
  // ---- deferred block + header + padding: the last wave (the fewest pass-2
  // chunks), before its chunks, while the others write theirs; the deferred
  // walk wave-cooperative
  if (wave == kBigW - 1u) {
    uint32_t nd = 0, ndd = 0, ndm = 0;
    if (lane == 0u && o_def != o_mpad) *(uint32_t*)(O + o_mpad) = 0u;
    if (ABL != 2 && has_def) {
      deferred_pass_wave<SP>(L, R, A, lane, nd, ndd, ndm, nullptr);
      RecLayout OL;
      rec_layout(OL, n_clk, tot_mem, tot_dot, nd, ndd, ndm, SP);
      DefOut w{(uint64_t*)(O + OL.o_fctr), (uint64_t*)(O + OL.o_fkey), (uint32_t*)(O + OL.o_fact),
               (uint32_t*)(O + OL.o_fdend), (uint32_t*)(O + OL.o_fmend)};
      deferred_pass_wave<SP>(L, R, A, lane, nd, ndd, ndm, &w);
    }
    if (lane == 0u) {
      RecLayout OL;
      rec_layout(OL, n_clk, tot_mem, tot_dot, nd, ndd, ndm, SP);
      for (uint32_t b = OL.o_end; b < OL.size; b += 4) *(uint32_t*)(O + b) = 0u;
      u32x4* h = (u32x4*)O;
      h[0] = u32x4{OL.size, n_clk, tot_mem, tot_dot};
      h[1] = u32x4{nd, ndd, ndm, SP ? kSparseClock : 0u};
    }
  }
  // ---- pass 2: kept members and their joined dot runs at their chunk's base
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (uint32_t ch = wave, k = 0; ch < (ABL == 3 ? 0u : nch); ch += kBigW, ++k) {
    const uint32_t p = kWave * ch + lane;
    uint32_t type = kNone, i = 0, j = 0, cnt = 0, x = 0;
    uint64_t v = 0;
    bool xv = false;  // (x, v) hold the run's only dot
    if (ABL != 6 && k < 2u) {
      const uint32_t q = k == 0 ? q0 : q1;
      cnt = k == 0 ? c0 : c1; x = k == 0 ? x0 : x1; v = k == 0 ? v0 : v1;
      type = q >> 30; i = (q >> 15) & 0x7FFFu; j = q & 0x7FFFu;
      xv = true;
    } else if (p < P && p < kBigPos) {
      const uint32_t u = T.pq[p];
      type = u >> 14; i = u & 0x3FFFu; j = p - i;
      cnt = T.pc[p];
      if (cnt == 255u) cnt = join<0, SP>(L, R, type, i, j, A, has_def, x, v, nullptr, nullptr, 0, T.bloom, crank);
    } else if (p < P) {
      type = merge_path_in(L, R, p, uni(T.spl[ch]), uni(T.spl[ch + 1]), i, j);
      if (type != kNone) cnt = join<0, SP>(L, R, type, i, j, A, has_def, x, v, nullptr, nullptr, 0, T.bloom, crank);
      xv = true;
    }
    const uint64_t keep = __ballot(cnt != 0);
    const uint32_t incl = wave_incl_scan(cnt, lane);
    const uint32_t mem_base = uni(T.tot[ch]), dot_base = uni(T.tot[T.cap + ch]);
    if (cnt != 0) {
      const uint32_t midx = mem_base + (uint32_t)__popcll(keep & lt_mask);
      const uint32_t d0 = dot_base + incl - cnt;
      okey[midx] = (type & kSelf) ? g64(L.b, L.v.key, i) : g64(R.b, R.v.key, j);
      if (cnt == 1 && xv) {
        odact[d0] = x;
        odctr[d0] = v;
      } else {
        join<1, SP>(L, R, type, i, j, A, has_def, x, v, odact, odctr, d0, T.bloom, crank);
      }
      omdend[midx] = d0 + cnt;
    }
  }
  if (T.last) bst<ABL>(*T.last, 5, wave, lane);
  __syncthreads();  // the stages and the tables are free for the next object
  if (T.last) bst<ABL>(*T.last, 6, wave, lane);
}

template <bool SP, int ABL>
__device__ __noinline__ void big_from_hbm(const uint8_t* lr, const uint8_t* rr, uint8_t* O, uint32_t A,
                                          uint32_t lane, uint32_t wave, u32x4* st, uint32_t* bc, uint8_t* crank) {
  uint8_t* sb = (uint8_t*)st;
  const BigTabs H{(uint32_t*)sb, (uint32_t*)(sb + 8u * kBigChH), (uint16_t*)(sb + 12u * kBigChH + 16u),
                  (uint8_t*)(sb + 12u * kBigChH + 16u + 2u * kBigPos), bc, kBigChH,
                  (uint32_t*)(sb + 12u * kBigChH + 16u + 3u * kBigPos), nullptr, crank};
  static_assert(12u * kBigChH + 16u + 3u * kBigPos + 128u <= 2u * kBigStage, "HBM-path tables fit the stage");
  const RecLayout LL = layout_at(lr), RL = layout_at(rr);
  const Side L{lr, make_rv(LL)}, R{rr, make_rv(RL)};
  merge_object_block<SP, ABL>(L, R, O, A, lane, wave, H);
}
template <bool SP>
__device__ __noinline__ void huge_one_wave(const uint8_t* lr, const uint8_t* rr, uint8_t* O, uint32_t A,
                                           uint32_t lane) {
  merge_object<SP>(lr, rr, O, A, lane);
}

// One big object o (listed for the general path) joined by the whole block.
// st: the 2 x kBigStage stage; T: the staged path's tables.
template <bool SP, int ABL = 0>
__device__ __forceinline__ void big_one(const uint8_t* Lb, const uint64_t* Loff, const uint8_t* Rb,
                                        const uint64_t* Roff, uint8_t* Ob, uint64_t* Ooff, uint64_t o, uint32_t A,
                                        u32x4* st, const BigTabs& T, uint32_t lane, uint32_t wave) {
  if (T.last) bst<ABL>(*T.last, 8, wave, lane);  // (8: between objects: the list walk)
  const uint64_t ow = Ooff[o];
  // only a pending object is this kernel's: after the general kernel every
  // pending object of either list is big (the general kernel cleared the rest)
  if ((ow & kPending) == 0ull) return;
  const uint64_t oo = ow & ~kPending;
  const uint8_t* lr = Lb + Loff[o];
  const uint8_t* rr = Rb + Roff[o];
  const RecLayout LL = layout_at(lr), RL = layout_at(rr);
  const uint32_t szl = LL.size, szr = RL.size, P = LL.n_mem + RL.n_mem;
  const bool staged = szl <= kBigStage && szr <= kBigStage && P <= kWave * kBigChS;
  if (T.last) bst<ABL>(*T.last, 0, wave, lane);
  u32x4* sl = st;
  u32x4* sr = st + kBigStage / 16u;
  if (P > kWave * kBigChH) {  // (past the HBM tables: one wave, merge_object)
    if (wave == 0u) huge_one_wave<SP>(lr, rr, Ob + oo, A, lane);
  } else {
    if (staged) {
      // both records staged: every load of the thread issued before its stores
      constexpr uint32_t kPer = kBigStage / 16u / (kWave * kBigW);
      const uint32_t nl = szl / 16u, nr = szr / 16u;
      u32x4 tl[kPer], tr[kPer];
#pragma unroll
      for (uint32_t u = 0; u < kPer; ++u) {
        const uint32_t k = threadIdx.x + u * kWave * kBigW;
        if (k < nl) tl[u] = ((const u32x4*)lr)[k];
        if (k < nr) tr[u] = ((const u32x4*)rr)[k];
      }
#pragma unroll
      for (uint32_t u = 0; u < kPer; ++u) {
        const uint32_t k = threadIdx.x + u * kWave * kBigW;
        if (k < nl) sl[k] = tl[u];
        if (k < nr) sr[k] = tr[u];
      }
      __syncthreads();
      if (T.last) bst<ABL>(*T.last, 1, wave, lane);
    }
    if (staged) {
      const SideL L{(lds_cu8*)(size_t)lds_addr(sl), make_rv(LL)}, R{(lds_cu8*)(size_t)lds_addr(sr), make_rv(RL)};
      if constexpr (ABL != 5) merge_object_block<SP, ABL>(L, R, Ob + oo, A, lane, wave, T);  // (5: staging only)
    } else {  // from HBM; the tables in the stage
      big_from_hbm<SP, ABL>(lr, rr, Ob + oo, A, lane, wave, st, T.bc, T.crank);
    }
  }
  if (threadIdx.x == 0u) Ooff[o] = oo;
  __syncthreads();
  if (T.last) bst<ABL>(*T.last, 7, wave, lane);
#ifdef CRDT_DIAG
  if (ABL == 8 && threadIdx.x == 0u) atomicAdd(&g_big_st[15], 1ull);
#endif
}

// The big objects, one block per object: the join's big list (objects whose
// headers already said big) and the general list's objects is_big() picks
// (the general kernel, launched before, skipped them). With an overflowed
// list every pending flag left is one.
template <bool SP, int MINW = 4, int ABL = 0>
__global__ __launch_bounds__(kWave * kBigW, MINW) void orswot_big_kernel(
    const uint8_t* __restrict__ Lb, const uint64_t* __restrict__ Loff, const uint8_t* __restrict__ Rb,
    const uint64_t* __restrict__ Roff, uint8_t* __restrict__ Ob, uint64_t* __restrict__ Ooff, uint64_t n_obj,
    uint32_t A, uint32_t* __restrict__ ctl, const uint64_t* __restrict__ list, uint32_t list_cap) {
  __shared__ u32x4 st_s[2 * kBigStage / 16];
  __shared__ uint32_t tot_s[2 * kBigChS], spl_s[kBigChS + 4], bc_s[4];
  __shared__ uint16_t pq_s[kBigPos];
  __shared__ uint8_t pc_s[kBigPos];
  __shared__ uint32_t bloom_s[32];
  uint64_t last = 0;
  if (ABL == 8) last = stamp();
  __shared__ uint8_t crank_s[SP ? 2u * kRankTab : 4u];  // (SP: the top clocks' actor -> rank tables)
  const BigTabs T{tot_s, spl_s, pq_s, pc_s, bc_s, kBigChS, bloom_s, ABL == 8 ? &last : nullptr, SP ? crank_s : nullptr};
  const uint32_t lane = threadIdx.x & (kWave - 1), wave = uni(threadIdx.x / kWave);
  const uint32_t n = uni(__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t scan = uni(__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  // ctl[2] (list_append): the big list's count, | kBigLeft when the general
  // kernel left big objects in its own list (zeroed between launches, so 0
  // means none)
  const uint32_t w2 = uni(__hip_atomic_load(&ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t nb = w2 & kBigCount, ng = (w2 & kBigLeft) ? n : 0u;
  if (nb == 0u && ng == 0u) return;
  // listed: the big list, then (when the general kernel left some) the
  // general list, one entry at a time dealt round-robin to the blocks (an
  // entry is one object: a block's share differs by at most one object; the
  // next entry is loaded while the current object is joined); big_one takes
  // only pending objects. A list past its half's capacity / a scan request:
  // every pending object left is big, found by a walk of the flags.
  const bool listed = n <= list_cap && nb <= list_cap && scan == 0u;
  const uint64_t units = listed ? (uint64_t)nb + ng : n_obj;
  // listed: entry e goes to block e % grid (rounds of 64 of the block's
  // entries: the block's share differs from another's by at most one
  // object); the flag walk: 64-object chunks round-robin
  for (uint64_t k0 = 0;; k0 += kWave) {
    const uint64_t e = listed ? (k0 + lane) * gridDim.x + blockIdx.x : (k0 / kWave * gridDim.x + blockIdx.x) * kWave + lane;
    if (uni64(e) >= units) break;  // (lane 0's is the round's smallest)
    bool big = false;
    uint64_t o = e;
    if (listed) {
      if (e < units) {
        o = e < nb ? list[list_cap + e] : list[e - nb];
        big = o < n_obj;  // (big_one takes only pending objects)
      }
    } else {
      big = e < n_obj && (Ooff[e] & kPending) != 0ull;
    }
    for (uint64_t m = __ballot(big); m; m &= m - 1)
      big_one<SP, ABL>(Lb, Loff, Rb, Roff, Ob, Ooff, lane_of64(o, (uint32_t)__builtin_ctzll(m)), A, st_s, T, lane,
                       wave);
  }
}

__global__ __launch_bounds__(kWave) void orswot_merge_general_kernel(
    const uint8_t* __restrict__ Lb, const uint64_t* __restrict__ Loff, const uint8_t* __restrict__ Rb,
    const uint64_t* __restrict__ Roff, uint8_t* __restrict__ Ob, uint64_t* __restrict__ Ooff, uint64_t n_obj,
    uint32_t A, uint32_t* __restrict__ ctl, const uint64_t* __restrict__ list, uint32_t list_cap,
    uint32_t* __restrict__ zero4) {
  __shared__ u32x4 gen_s[3][kGenStage / 16];
  const uint32_t lane = threadIdx.x;
  // NM: the control words of the other parity (the launch before this one
  // used them; the launch after it will) are zeroed here, so no memset
  // precedes a join launch (launch_join_passes)
  if (zero4 && blockIdx.x == 0u && lane < 4u) zero4[lane] = 0u;
  const uint32_t n = uni(__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t scan = uni(__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  // (the block's first entry is read with the count, a round trip less; an
  // entry past the count is stale and not used)
  const uint64_t first = blockIdx.x < list_cap ? list[blockIdx.x] : 0ull;
  if (n <= list_cap && scan == 0u) {
    // one object ahead: its list entry at the top of this one, its offsets
    // and headers while this one's records are staged and joined
    if (blockIdx.x >= n) return;
    GenPre cur, nxt;
    gen_pre(cur, Lb, Loff, Rb, Roff, Ooff, first);
    bool big = false;
    for (uint32_t e = blockIdx.x; e < n; e += gridDim.x) {
      const uint32_t en = e + gridDim.x;
      const uint64_t on = en < n ? list[en] : 0ull;
      big |= general_one(cur, Ob, Ooff, A, gen_s[0], gen_s[1], gen_s[2], lane, [&]() {
        if (en < n) gen_pre(nxt, Lb, Loff, Rb, Roff, Ooff, on);
      });
      cur = nxt;
    }
    // one store per wave that left a big object (not one atomic per object:
    // same-address atomics serialise at the memory side)
    if (big && lane == 0u) __hip_atomic_fetch_or(&ctl[2], kBigLeft, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {  // list overflow, or objects flagged without a list entry: scan the flags
    const uint64_t n_chunks = (n_obj + kWave - 1) / kWave;
    for (uint64_t chunk = blockIdx.x; chunk < n_chunks; chunk += gridDim.x) {
      const uint64_t obj = chunk * kWave + lane;
      const uint64_t oo = obj < n_obj ? Ooff[obj] : 0ull;
      for (uint64_t pend = __ballot((oo & kPending) != 0ull); pend; pend &= pend - 1) {
        GenPre g;
        gen_pre(g, Lb, Loff, Rb, Roff, Ooff, chunk * kWave + (uint32_t)__builtin_ctzll(pend));
        if (general_one(g, Ob, Ooff, A, gen_s[0], gen_s[1], gen_s[2], lane, []() {}) && lane == 0u)
          __hip_atomic_fetch_or(&ctl[2], kBigLeft, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

constexpr uint32_t kBigBlocks = 512;  // two 8-wave, 72 KB-LDS blocks per CU
#ifdef CRDT_DIAG
int g_big_variant = 0;  // diag variants 330..: the big kernel's knobs
#endif

// The big-object pass, queued after every general kernel launch (the objects
// it leaves flagged are this kernel's).
// SP: CSR top clocks (after the sparse general kernel)
template <bool SP = false>
__host__ inline hipError_t launch_big(const uint8_t* Lb, const uint64_t* Loff, const uint8_t* Rb, const uint64_t* Roff,
                                      uint8_t* Ob, uint64_t* Ooff, uint64_t n_obj, uint32_t A, uint32_t* ctl,
                                      const uint64_t* list, uint32_t list_cap, hipStream_t stream) {
  const void* fn = (const void*)orswot_big_kernel<SP, 4>;
  uint32_t blocks = kBigBlocks;
#ifdef CRDT_DIAG
  if (!SP) {
  if (g_big_variant == 1) { fn = (const void*)orswot_big_kernel<false, 1>; blocks = 256; }
  if (g_big_variant == 2) { fn = (const void*)orswot_big_kernel<false, 2>; blocks = 256; }
  if (g_big_variant == 3) blocks = 256;
  if (g_big_variant == 4) fn = (const void*)orswot_big_kernel<false, 4, 1>;
  if (g_big_variant == 5) fn = (const void*)orswot_big_kernel<false, 4, 2>;
  if (g_big_variant == 6) fn = (const void*)orswot_big_kernel<false, 4, 3>;
  if (g_big_variant == 7) fn = (const void*)orswot_big_kernel<false, 4, 4>;
  if (g_big_variant == 8) fn = (const void*)orswot_big_kernel<false, 4, 5>;
  if (g_big_variant == 9) fn = (const void*)orswot_big_kernel<false, 4, 6>;
  if (g_big_variant == 11) fn = (const void*)orswot_big_kernel<false, 4, 8>;
  }
#endif
  void* args[] = {&Lb, &Loff, &Rb, &Roff, &Ob, &Ooff, &n_obj, &A, &ctl, &list, &list_cap};
  return hipLaunchKernel(fn, dim3(blocks), dim3(kWave * kBigW), args, 0, stream);
}

// ======================================================================
// Sparse (CSR) top-clock batches (config 5: 1024-actor universe): one wave
// per object pair, grid-stride over objects, both records staged through
// LDS when they fit (else read from HBM), joined by merge_object<true>.
// ======================================================================

__device__ __forceinline__ bool sparse_header_ok(u32x4 h0, u32x4 h1, uint64_t off, uint64_t bytes, uint32_t A) {
  const uint64_t sz = record_size64(h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, true);
  return (off & 15u) == 0 && off + kHdrBytes <= bytes && sz == h0.x && h0.y <= A && h1.w == kSparseClock &&
         off + sz <= bytes;
}


// Sparse mask kernel: the dense mask kernel's structure for CSR batches.
// Lane k of a chunk owns object cbase + k's header; objects that fit the
// sparse mask join (both records together <= kSpPair, <= 64 clock entries /
// members, <= 128 dots, <= 32 deferred clocks per side, A <= kSpTableN) are
// joined one per wave from a single LDS pair stage (L at 0, R right after it)
// while the next object's pair is in flight in registers; everything else is
// flagged and listed for orswot_sparse_general_kernel.
constexpr uint32_t kSpPair = 6144;
constexpr uint32_t kSpPer = kSpPair / 16 / kWave;
// CSR batches: the join's 6 016-B scratch leaves room for a 7 KB pair stage
// at the same 3 four-wave blocks per CU (the DN kernel keeps 6 KB + 7 040 B)
constexpr uint32_t kSpPairCsr = 7168, kSpScratchCsr = kSpTrash + 16u * kWave;

template <uint32_t PER = kSpPer>
__device__ __forceinline__ void prefetch_pair(u32x4 (&r)[PER], const uint8_t* L, const uint8_t* R, uint32_t nl,
                                              uint32_t nr, uint32_t lane) {
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t idx = lane + k * kWave;
    const uint32_t j = idx - nl < nr ? idx - nl : nr - 1u;
    r[k] = __builtin_nontemporal_load(idx < nl ? (const u32x4*)L + idx : (const u32x4*)R + j);
  }
}

template <uint32_t PER = kSpPer>
__device__ __forceinline__ void stage_pair(u32x4* dst, const u32x4 (&r)[PER], uint32_t lane) {
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) dst[lane + k * kWave] = r[k];
}

// DN: dense batches of 65..1024 actors (wide_mask_object, 64- then 128-bit
// masks; a union of > 128 present actors goes to the general kernel)
template <int MINW, int ABL = 0, uint32_t DYN = 0, uint32_t SF = 5, bool SASM = false, bool DN = false>  // ABL 9: phase stamps into the list buffer (no general path)
__global__ __launch_bounds__(kWave * kWavesPerBlock, MINW) void orswot_sparse_mask_kernel(
    const uint8_t* __restrict__ Lb, const uint64_t* __restrict__ Loff, uint64_t Lbytes,
    const uint8_t* __restrict__ Rb, const uint64_t* __restrict__ Roff, uint64_t Rbytes,
    uint8_t* __restrict__ Ob, uint64_t* __restrict__ Ooff, uint64_t Obytes, uint64_t n_obj, uint32_t A,
    int* __restrict__ status, uint32_t* __restrict__ ctl, uint64_t* __restrict__ list, uint32_t list_cap) {
  constexpr uint32_t PAIR = DN ? kSpPair : kSpPairCsr, PER = PAIR / 16 / kWave;
  __shared__ u32x4 pair_s[kWavesPerBlock][PAIR / 16];
  __shared__ u32x4 scr_s[kWavesPerBlock][(DN ? kSpScratch : kSpScratchCsr) / 16];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wave = threadIdx.x / kWave;
  u32x4* const S = pair_s[wave];
  uint8_t* const X = (uint8_t*)scr_s[wave];
  const uint64_t wave_id = (uint64_t)blockIdx.x * kWavesPerBlock + wave;
  const uint64_t n_waves = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint64_t rounds = (n_obj + n_waves * kWave - 1) / (n_waves * kWave);
  const uint64_t cs = (n_obj + n_waves * rounds - 1) / (n_waves * rounds);
  Stamps st{};
  if (ABL == 9) st.last = stamp();
  // DYN: the guided split (GuidedSplit); else static rounds of cs-object chunks
  GuidedSplit<DYN ? DYN : 1u, SF> gs(n_obj, wave_id, n_waves);
  uint64_t cbase = wave_id * cs, cend = n_obj;
  for (uint32_t it = 0u;; ++it) {
    if (DYN) {
      if (!gs.next(cbase, cend, &ctl[3], lane)) break;
    } else {
      if (it > 0u) cbase += n_waves * cs;
      if (cbase >= n_obj) break;
    }
    const uint64_t obj = cbase + lane;
    const bool valid = DYN ? obj < cend : lane < cs && obj < n_obj;
    uint64_t lo = 0, ro = 0, nlo = Lbytes, nro = Rbytes;
    if (valid) { lo = Loff[obj]; ro = Roff[obj]; }
    if (valid && obj + 1u < n_obj) { nlo = Loff[obj + 1u]; nro = Roff[obj + 1u]; }
    u32x4 hl0 = {0, 0, 0, 0}, hl1 = hl0, hr0 = hl0, hr1 = hl0;
    bool ok = valid && (lo & 15u) == 0 && (ro & 15u) == 0 && lo + kHdrBytes <= Lbytes && ro + kHdrBytes <= Rbytes;
    if (ok) {
      hl0 = ((const u32x4*)(Lb + lo))[0]; hl1 = ((const u32x4*)(Lb + lo))[1];
      hr0 = ((const u32x4*)(Rb + ro))[0]; hr1 = ((const u32x4*)(Rb + ro))[1];
    }
    ok = ok && (DN ? header_ok(hl0, hl1, lo, Lbytes, A) && header_ok(hr0, hr1, ro, Rbytes, A)
                   : sparse_header_ok(hl0, hl1, lo, Lbytes, A) && sparse_header_ok(hr0, hr1, ro, Rbytes, A)) &&
         lo + ro + (uint64_t)hl0.x + hr0.x <= Obytes;
    const bool placed = !ok || (nlo >= lo + hl0.x && nro >= ro + hr0.x);  // as in orswot_mask_kernel
    if (__ballot(!placed) != 0ull && lane == 0) atomicCAS(status, 0, CRDT_EINVAL);
    ok = ok && placed;
    const bool fast = ok && hl0.x + hr0.x <= PAIR && A <= kSpTableN && (DN || (hl0.y <= 64u && hr0.y <= 64u)) &&
                      hl0.z <= 64u && hr0.z <= 64u && hl0.w <= 128u && hr0.w <= 128u && hl1.x <= 32u &&
                      hr1.x <= 32u;
    if (valid) Ooff[obj] = (lo + ro) | ((ok && !fast) ? kPending : 0ull);
    if (ABL != 9) {  // the general kernel's objects, big ones straight to orswot_big_kernel<true>
      const bool bigo = ok && !fast && is_big(hl0, hr0);
      list_append(ok && !fast && !bigo, obj, &ctl[0], list, list_cap, lane);
      list_append(bigo, obj, &ctl[2], list + list_cap, list_cap, lane);
    }
    if (__ballot(valid && !ok && placed) != 0ull && lane == 0) atomicCAS(status, 0, CRDT_ENONCANON);
    uint64_t pend = __ballot(fast);
    if (pend == 0ull) continue;
    const uint32_t n16 = fast ? (hl0.x / 16u) | ((hr0.x / 16u) << 16) : 0u;
    const uint32_t ncl = hl0.y | (hr0.y << 16), nm = hl0.z | (hr0.z << 16), nd = hl0.w | (hr0.w << 16);
    const uint64_t defs = __ballot(fast && (hl1.x | hr1.x) != 0u);
    uint32_t t = (uint32_t)__builtin_ctzll(pend);
    uint64_t fbm = 0ull;  // the chunk's objects the join left (kLeanFallback)
    u32x4 pf[PER];
    uint32_t nn = lane_of(n16, t);
    prefetch_pair<PER>(pf, Lb + lane_of64(lo, t), Rb + lane_of64(ro, t), nn & 0xFFFFu, nn >> 16, lane);
    while (pend) {
      t = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      nn = lane_of(n16, t);
      wave_sync();  // previous object's LDS reads are done
      stage_pair<PER>(S, pf, lane);
      wave_sync();
      mark<ABL>(st, 0);
      const uint64_t oo = lane_of64(lo, t) + lane_of64(ro, t);
      const uint32_t c = lane_of(ncl, t), m = lane_of(nm, t), d = lane_of(nd, t);
      if (pend) {
        const uint32_t u = (uint32_t)__builtin_ctzll(pend);
        const uint32_t nu = lane_of(n16, u);
        prefetch_pair<PER>(pf, Lb + lane_of64(lo, u), Rb + lane_of64(ro, u), nu & 0xFFFFu, nu >> 16, lane);
      }
      mark<ABL>(st, 1);
      const uint8_t* Ls = (const uint8_t*)S;
      const uint8_t* Rs = Ls + 16u * (nn & 0xFFFFu);
      uint32_t r;
      if (DN) {  // dense-wide: 64-bit actor masks, then 128-bit for a union of 65..128 present actors
        const bool hd = (defs >> t) & 1ull;
        r = hd ? wide_mask_object<true, 1>(Ls, Rs, X, Ob + oo, A, m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16, lane)
               : wide_mask_object<false, 1>(Ls, Rs, X, Ob + oo, A, m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16, lane);
        if (r == kLeanFallback)  // (on the same stage)
          r = hd ? wide_mask_object<true, 2>(Ls, Rs, X, Ob + oo, A, m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16, lane)
                 : wide_mask_object<false, 2>(Ls, Rs, X, Ob + oo, A, m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16,
                                              lane);
      } else if ((defs >> t) & 1ull) {
        r = sparse_mask_object<true, ABL>(Ls, Rs, X, Ob + oo, A, c & 0xFFFFu, m & 0xFFFFu, d & 0xFFFFu, c >> 16,
                                          m >> 16, d >> 16, lane, &st);
      } else {
        r = sparse_mask_object<false, ABL, SASM>(Ls, Rs, X, Ob + oo, A, c & 0xFFFFu, m & 0xFFFFu, d & 0xFFFFu,
                                                 c >> 16, m >> 16, d >> 16, lane, &st);
      }
      fbm |= r == kLeanFallback ? 1ull << t : 0ull;  // union clock / members > 64 or a foreign dot actor
    }
    // the chunk's fallbacks to the general kernel: flagged and listed with
    // one atomic (a per-object atomic on one address serialises: the wide
    // dense distribution lists nearly every object)
    if (ABL != 9 && fbm != 0ull) {
      const bool fb = (fbm >> lane) & 1ull;
      if (fb) Ooff[obj] = (lo + ro) | kPending;
      list_append(fb, obj, &ctl[0], list, list_cap, lane);
    }
  }
  if (ABL == 9 && lane < 16u) {  // per-wave phase sums -> the context's list buffer
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) v = lane == (uint32_t)q ? st.acc[q] : v;
    list[wave_id * 16u + lane] = v;
  }
}

// Wide dense kernel (dense batches of 65..1024 actors, after the DN mask
// kernel): the objects it left flagged whose pair fits the pair stage with
// <= 64 members, <= 128 dots and <= 32 deferred clocks per side are joined by
// wide_mask_object (union of present actors <= 128) and their flag cleared;
// the rest stay flagged for the general kernel (which skips a listed object
// whose flag is clear). The DN kernel's list is dealt in chunks of up to 64
// entries per wave (past its capacity: every object's flag is scanned, 64
// objects per chunk), the next candidate's pair in flight in registers during
// a join; the kernel returns at once when the DN kernel listed nothing.
constexpr uint32_t kWdWaves = 2;
constexpr uint32_t kWdPair = 16384, kWdPer = kWdPair / 16 / kWave;  // pairs the DN kernel's 6 KB stage cannot take
constexpr int kWdMinW = 1;  // (LDS: 23.3 KB per wave, three 2-wave blocks per CU)
template <int MINW>
__global__ __launch_bounds__(kWave * kWdWaves, MINW) void orswot_dense_wide_kernel(
    const uint8_t* __restrict__ Lb, const uint64_t* __restrict__ Loff, const uint8_t* __restrict__ Rb,
    const uint64_t* __restrict__ Roff, uint8_t* __restrict__ Ob, uint64_t* __restrict__ Ooff, uint64_t n_obj,
    uint32_t A, const uint32_t* __restrict__ ctl, const uint64_t* __restrict__ list, uint32_t list_cap) {
  __shared__ u32x4 pair_s[kWdWaves][kWdPair / 16];
  __shared__ u32x4 scr_s[kWdWaves][kWdScratch / 16];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wave = threadIdx.x / kWave;
  u32x4* const S = pair_s[wave];
  uint8_t* const X = (uint8_t*)scr_s[wave];
  const uint32_t n = uni(__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (n == 0u) return;
  const bool listed = n <= list_cap;
  const uint64_t wave_id = (uint64_t)blockIdx.x * kWdWaves + wave;
  const uint64_t n_waves = (uint64_t)gridDim.x * kWdWaves;
  // listed: chunks of `per` list entries (the list spread over every wave)
  const uint64_t per = listed ? (n + n_waves - 1) / n_waves < kWave ? (n + n_waves - 1) / n_waves : kWave : kWave;
  const uint64_t n_chunks = ((listed ? n : n_obj) + per - 1) / per;
  for (uint64_t chunk = wave_id; chunk < n_chunks; chunk += n_waves) {
    const uint64_t e = chunk * per + lane;
    const bool in = lane < per && e < (listed ? (uint64_t)n : n_obj);
    const uint64_t obj = !in ? 0ull : listed ? list[e] : e;
    const bool pending = in && (Ooff[obj] & kPending) != 0ull;
    if (__ballot(pending) == 0ull) continue;
    uint64_t lo = 0, ro = 0;
    u32x4 hl0 = {0, 0, 0, 0}, hl1 = hl0, hr0 = hl0, hr1 = hl0;
    if (pending) {  // (the DN kernel flags only objects whose headers it checked)
      lo = Loff[obj];
      ro = Roff[obj];
      hl0 = ((const u32x4*)(Lb + lo))[0]; hl1 = ((const u32x4*)(Lb + lo))[1];
      hr0 = ((const u32x4*)(Rb + ro))[0]; hr1 = ((const u32x4*)(Rb + ro))[1];
    }
    const bool cand = pending && hl0.x + hr0.x <= kWdPair && hl0.z <= 64u && hr0.z <= 64u && hl0.w <= 128u &&
                      hr0.w <= 128u && hl1.x <= 32u && hr1.x <= 32u;
    uint64_t pend = __ballot(cand);
    if (pend == 0ull) continue;
    const uint32_t n16 = cand ? (hl0.x / 16u) | ((hr0.x / 16u) << 16) : 0u;
    const uint32_t nm = hl0.z | (hr0.z << 16), nd = hl0.w | (hr0.w << 16);
    const uint64_t defs = __ballot(cand && (hl1.x | hr1.x) != 0u);
    uint64_t donem = 0ull;
    u32x4 pf[kWdPer];
    uint32_t t = (uint32_t)__builtin_ctzll(pend);
    uint32_t nn = lane_of(n16, t);
    prefetch_pair<kWdPer>(pf, Lb + lane_of64(lo, t), Rb + lane_of64(ro, t), nn & 0xFFFFu, nn >> 16, lane);
    while (pend) {
      t = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      nn = lane_of(n16, t);
      wave_sync();  // previous object's LDS reads are done
      stage_pair<kWdPer>(S, pf, lane);
      wave_sync();
      const uint64_t oo = lane_of64(lo, t) + lane_of64(ro, t);
      const uint32_t m = lane_of(nm, t), d = lane_of(nd, t);
      if (pend) {
        const uint32_t u = (uint32_t)__builtin_ctzll(pend);
        const uint32_t nu = lane_of(n16, u);
        prefetch_pair<kWdPer>(pf, Lb + lane_of64(lo, u), Rb + lane_of64(ro, u), nu & 0xFFFFu, nu >> 16, lane);
      }
      const uint8_t* Ls = (const uint8_t*)S;
      const uint8_t* Rs = Ls + 16u * (nn & 0xFFFFu);
      const uint32_t r = (defs >> t) & 1ull
                             ? wide_mask_object<true>(Ls, Rs, X, Ob + oo, A, m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16, lane)
                             : wide_mask_object<false>(Ls, Rs, X, Ob + oo, A, m & 0xFFFFu, d & 0xFFFFu, m >> 16, d >> 16,
                                                       lane);
      donem |= r != kLeanFallback ? 1ull << t : 0ull;
    }
    if ((donem >> lane) & 1ull) Ooff[obj] = lo + ro;  // joined: the flag cleared (one coalesced store)
  }
}

// The sparse kernel's general path: one wave per listed object (pairs larger
// than the pair stage, or a union past 64 clock entries / members), staged
// through LDS when both records fit kGenStage: joined by sparse_mask_object
// when its limits hold, else by merge_object<true>.
// One sparse join of the pre-loaded object g (GenPre: offsets, headers) into
// its output place (any sizes); `mid` runs once the records are staged (the
// caller's loads for the next listed object, in flight during this join).
// (returns true for an object it leaves to orswot_big_kernel<true>: past
// kBigMinPos union positions or the general stage, as general_one)
template <class Mid>
__device__ __forceinline__ bool sparse_general_one(const GenPre& g, uint8_t* Ob, uint64_t* Ooff, uint32_t A,
                                                   u32x4* sl, u32x4* sr, uint8_t* X, uint32_t lane, Mid&& mid) {
  const uint8_t* lr = g.lr;
  const uint8_t* rr = g.rr;
  uint8_t* O = Ob + g.oo;
  const u32x4 hl0 = g.hl0, hl1 = g.hl1, hr0 = g.hr0, hr1 = g.hr1;
  const uint32_t szl = uni(hl0.x), szr = uni(hr0.x);
  if (is_big(u32x4{szl, 0u, uni(hl0.z), 0u}, u32x4{szr, 0u, uni(hr0.z), 0u})) {  // orswot_big_kernel<true>'s
    mid();
    return true;
  }
  if (szl > kGenStage || szr > kGenStage) mid();
  if (szl <= kGenStage && szr <= kGenStage) {
    wave_sync();
    // both records staged 4 KB per side at a time: every load of a round is
    // issued before its stores (one memory round trip per 4 KB, not per 1 KB)
    {
      constexpr uint32_t kB = 4;
      const uint32_t nl = szl / 16, nr = szr / 16, nmax = nl > nr ? nl : nr;
      for (uint32_t k0 = 0; k0 < nmax; k0 += kB * kWave) {
        u32x4 tl[kB], tr[kB];
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
          const uint32_t k = k0 + j * kWave + lane;
          if (k < nl) tl[j] = ((const u32x4*)lr)[k];
          if (k < nr) tr[j] = ((const u32x4*)rr)[k];
        }
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
          const uint32_t k = k0 + j * kWave + lane;
          if (k < nl) sl[k] = tl[j];
          if (k < nr) sr[k] = tr[j];
        }
      }
    }
    mid();
    wave_sync();
    uint32_t r = kLeanFallback;
    const uint32_t cL = uni(hl0.y), nL = uni(hl0.z), dL = uni(hl0.w), cR = uni(hr0.y), nR = uni(hr0.z),
                   dR = uni(hr0.w);
    if (A <= kSpTableN && cL <= 64u && cR <= 64u && nL <= 64u && nR <= 64u && dL <= 128u && dR <= 128u &&
        uni(hl1.x) <= 32u && uni(hr1.x) <= 32u) {
      if ((uni(hl1.x) | uni(hr1.x)) != 0u)
        r = sparse_mask_object<true>((const uint8_t*)sl, (const uint8_t*)sr, X, O, A, cL, nL, dL, cR, nR, dR,
                                     lane);
      else
        r = sparse_mask_object<false>((const uint8_t*)sl, (const uint8_t*)sr, X, O, A, cL, nL, dL, cR, nR,
                                      dR, lane);
    }
    if (r == kLeanFallback) merge_object<true>((const uint8_t*)sl, (const uint8_t*)sr, O, A, lane);
  } else {
    merge_object<true>(lr, rr, O, A, lane);
  }
  if (lane == 0) Ooff[g.o] = g.oo;
  return false;
}

__global__ __launch_bounds__(kWave) void orswot_sparse_general_kernel(
    const uint8_t* __restrict__ Lb, const uint64_t* __restrict__ Loff, const uint8_t* __restrict__ Rb,
    const uint64_t* __restrict__ Roff, uint8_t* __restrict__ Ob, uint64_t* __restrict__ Ooff, uint64_t n_obj,
    uint32_t A, uint32_t* __restrict__ ctl, const uint64_t* __restrict__ list, uint32_t list_cap,
    uint32_t* __restrict__ zero4) {
  __shared__ u32x4 gen_s[2][kGenStage / 16];
  __shared__ u32x4 gx_s[kSpScratch / 16];
  const uint32_t lane = threadIdx.x;
  if (zero4 && blockIdx.x == 0u && lane < 4u) zero4[lane] = 0u;  // (the next launch's words: as the dense path)
  const uint32_t n = uni(__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (n <= list_cap) {
    // one object ahead, as the dense general kernel
    if (blockIdx.x >= n) return;
    GenPre cur, nxt;
    gen_pre(cur, Lb, Loff, Rb, Roff, Ooff, list[blockIdx.x]);
    bool big = false;
    for (uint32_t e = blockIdx.x; e < n; e += gridDim.x) {
      const uint32_t en = e + gridDim.x;
      const uint64_t on = en < n ? list[en] : 0ull;
      big |= sparse_general_one(cur, Ob, Ooff, A, gen_s[0], gen_s[1], (uint8_t*)gx_s, lane, [&]() {
        if (en < n) gen_pre(nxt, Lb, Loff, Rb, Roff, Ooff, on);
      });
      cur = nxt;
    }
    // one store per wave that left a big object (as the dense general kernel)
    if (big && lane == 0u) __hip_atomic_fetch_or(&ctl[2], kBigLeft, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {  // list overflow: scan the flags
    const uint64_t n_chunks = (n_obj + kWave - 1) / kWave;
    bool big = false;
    for (uint64_t chunk = blockIdx.x; chunk < n_chunks; chunk += gridDim.x) {
      const uint64_t obj = chunk * kWave + lane;
      const uint64_t oo = obj < n_obj ? Ooff[obj] : 0ull;
      for (uint64_t pend = __ballot((oo & kPending) != 0ull); pend; pend &= pend - 1) {
        GenPre g;
        gen_pre(g, Lb, Loff, Rb, Roff, Ooff, chunk * kWave + (uint32_t)__builtin_ctzll(pend));
        big |= sparse_general_one(g, Ob, Ooff, A, gen_s[0], gen_s[1], (uint8_t*)gx_s, lane, []() {});
      }
    }
    if (big && lane == 0u) __hip_atomic_fetch_or(&ctl[2], kBigLeft, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


}  // namespace

#ifdef CRDT_DIAG
#include "diag/orswot_launch_diag.inc"  // their launchers
#endif

namespace {
// The ring join launch (orswot_ring_kernel, then the general kernel), with
// launch_join_passes' alternating control-word sets (no memset before it).
template <const void* (*KF)(), bool WIDE = false>
int launch_join_kernel(const uint8_t* Lb, const uint64_t* Loff, uint64_t Lbytes, const uint8_t* Rb,
                       const uint64_t* Roff, uint64_t Rbytes, uint8_t* Ob, uint64_t* Ooff, uint64_t Obytes,
                       uint64_t n_obj, uint32_t n_actors, int* status, uint32_t* ctl, uint64_t* list, uint32_t list_cap,
                       hipStream_t stream, int blocks_per_cu, JoinSeq* js) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const void* fn = KF();
  static std::atomic<int> occ_cache{0};  // per kernel
  int occ = occ_cache.load(std::memory_order_relaxed);
  if (occ == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kWave * kWavesPerBlock, 0) != hipSuccess || occ < 1)
      occ = 4;
    occ_cache.store(occ, std::memory_order_relaxed);
  }
  const uint64_t chunks = (n_obj + kWave - 1) / kWave;
  const uint64_t want = (chunks + kWavesPerBlock - 1) / kWavesPerBlock;
  const uint64_t cap = (uint64_t)cus * (blocks_per_cu > 0 ? blocks_per_cu : occ);
  const uint32_t blocks = (uint32_t)(want < cap ? want : cap);
  uint32_t* set = ctl + 4u + 4u * (js->seq & 1u);
  uint32_t* const other = ctl + 4u + 4u * (~js->seq & 1u);
  if (js->dirty && hipMemsetAsync(ctl + 4, 0, 8 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;
  js->dirty = true;  // until both kernels are launched
  void* args[] = {&Lb, &Loff, &Lbytes, &Rb, &Roff, &Rbytes, &Ob, &Ooff, &Obytes, &n_obj, &n_actors, &status,
                  &set, &list, &list_cap};
  if (hipLaunchKernel(fn, dim3(blocks), dim3(kWave * kWavesPerBlock), args, 0, stream) != hipSuccess)
    return CRDT_EHIP;
  if (WIDE) {  // dense-wide: unions of 65..128 present actors before the general kernel
    const void* wf = (const void*)orswot_dense_wide_kernel<kWdMinW>;
    const uint64_t* wlist = list;
    static std::atomic<int> wocc_cache{0};
    int wocc = wocc_cache.load(std::memory_order_relaxed);
    if (wocc == 0) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&wocc, wf, kWave * kWdWaves, 0) != hipSuccess || wocc < 1)
        wocc = 2;
      wocc_cache.store(wocc, std::memory_order_relaxed);
    }
    const uint64_t wwant = ((n_obj + kWave - 1) / kWave + kWdWaves - 1) / kWdWaves;
    const uint64_t wcap = (uint64_t)cus * wocc;
    const uint32_t wblocks = (uint32_t)(wwant < wcap ? wwant : wcap);
    const uint32_t* cset = set;
    void* wargs[] = {&Lb, &Loff, &Rb, &Roff, &Ob, &Ooff, &n_obj, &n_actors, &cset, &wlist, &list_cap};
    if (hipLaunchKernel(wf, dim3(wblocks), dim3(kWave * kWdWaves), wargs, 0, stream) != hipSuccess) return CRDT_EHIP;
  }
  hipLaunchKernelGGL(orswot_merge_general_kernel, dim3(kGenBlocks), dim3(kWave), 0, stream, Lb, Loff, Rb, Roff, Ob,
                     Ooff, n_obj, n_actors, set, list, list_cap, other);
  if (hipGetLastError() != hipSuccess) return CRDT_EHIP;
  if (launch_big(Lb, Loff, Rb, Roff, Ob, Ooff, n_obj, n_actors, set, list, list_cap, stream) != hipSuccess)
    return CRDT_EHIP;
  ++js->seq;
  js->dirty = false;
  return CRDT_OK;
}
template <int MINW, int AW, int FL>
const void* join5_fn() { return (const void*)orswot_join5_kernel<MINW, AW, FL>; }
template <int MINW, int AW, int FL>
constexpr auto launch_join5 = launch_join_kernel<join5_fn<MINW, AW, FL>>;
// dense top clocks of 65..1024 actors: the mask join over the per-object
// union of present actors (DN: wide_mask_object), orswot_dense_wide_kernel
// for pairs past its stage, then the dense general kernel
const void* dense_wide_fn() { return (const void*)orswot_sparse_mask_kernel<3, 0, 16, 5, false, true>; }
constexpr auto launch_dense_wide = launch_join_kernel<dense_wide_fn, true>;
}  // namespace
#ifdef CRDT_DIAG
#include "diag/orswot_variants_diag.inc"  // the diagnostic variant table
#endif

int launch_orswot_merge(const uint8_t* Lb, const uint64_t* Loff, uint64_t Lbytes, const uint8_t* Rb,
                        const uint64_t* Roff, uint64_t Rbytes, uint8_t* Ob, uint64_t* Ooff,
                        uint64_t Obytes, uint64_t n_obj, uint32_t n_actors, int* status, uint32_t* ctl,
                        uint64_t* list, uint32_t list_cap, hipStream_t stream, int blocks_per_cu, int variant,
                        JoinSeq* js) {
  if (n_obj == 0) return CRDT_OK;
  list_cap /= 2u;  // the context's list: the general half, then the big half (list_append)
  JoinSeq local{0u, true};
  if (!js) js = &local;  // (no context state: the words are zeroed first)
  auto go = [&](auto f) {
    return f(Lb, Loff, Lbytes, Rb, Roff, Rbytes, Ob, Ooff, Obytes, n_obj, n_actors, status, ctl, list, list_cap,
             stream, blocks_per_cu, js);
  };
#ifdef CRDT_DIAG
  // diagnostic builds: the kernel variants of tools/ (csrc/diag/orswot_variants_diag.inc);
  // variant 0 is the product path below
  g_big_variant = 0;
  if (variant != 0)
    return launch_orswot_merge_diag(go, Lb, Loff, Lbytes, Rb, Roff, Rbytes, Ob, Ooff, Obytes, n_obj, n_actors,
                                    status, ctl, list, list_cap, stream, blocks_per_cu, variant);
#endif
  (void)variant;
  // dense top clocks wider than the 64-bit actor masks (65..1024 actors):
  // every object whose union of present actors holds <= 128 actors takes the
  // dense-wide mask join (DN), the rest the general kernel
  if (n_actors > 64u && n_actors <= kSpTableN) return go(launch_dense_wide);
  // The product path: orswot_join5_kernel — one pass (mask3_object for every
  // object; those with deferred removes take its HD form, direct stores) at 6
  // waves per SIMD with the guided split (5/8 of the objects in static chunks,
  // the rest in 20-object ticket chunks), record prefetch one object ahead in
  // the saddr form and the copy-out clamped on byte offsets, both sides'
  // member ranks in one packed pass when nL + nR <= 64 and mask3's
  // bank-conflict layout, then the general kernel (measured best,
  // tools/ab_bench.py).
  if (n_actors > 32u)  // dense top clocks of 33-64 actors: the same join with 64-bit actor masks, 5 waves/SIMD
    return go(launch_join5<5, 64, 0>);
  return go(launch_join5<6, 32, 0>);
}

int launch_orswot_merge_sparse(const uint8_t* Lb, const uint64_t* Loff, uint64_t Lbytes, const uint8_t* Rb,
                               const uint64_t* Roff, uint64_t Rbytes, uint8_t* Ob, uint64_t* Ooff, uint64_t Obytes,
                               uint64_t n_obj, uint32_t n_actors, int* status, uint32_t* ctl, uint64_t* list,
                               uint32_t list_cap, hipStream_t stream, int sparse_variant, JoinSeq* js) {
  if (n_obj == 0) return CRDT_OK;
  list_cap /= 2u;  // the context's list: the general half, then the big half (list_append)
  JoinSeq local{0u, true};
  if (!js) js = &local;
  int dev = 0, cus = 256, occ = 0;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
#ifdef CRDT_DIAG
  const void* fn = sparse_variant == 4 ? (const void*)orswot_sparse_mask_kernel<3, 9>
                   : sparse_variant == 5 ? (const void*)orswot_sparse_mask_kernel<3, 0, 20, 5>
                   : sparse_variant == 6 ? (const void*)orswot_sparse_mask_kernel<3, 0, 24, 4>
                   : sparse_variant == 7 ? (const void*)orswot_sparse_mask_kernel<3, 0, 16, 5>
                   : sparse_variant == 8 ? (const void*)orswot_sparse_mask_kernel<3, 0, 32, 5>
                   : sparse_variant == 9 ? (const void*)orswot_sparse_mask_kernel<3, 0, 12, 5>
                   : sparse_variant == 10 ? (const void*)orswot_sparse_mask_kernel<3>  // r02e: static split
                   : sparse_variant == 11 ? (const void*)orswot_sparse_mask_kernel<3, 0, 16, 5, true>  // r04: + SASM
                                        : (const void*)orswot_sparse_mask_kernel<3, 0, 16, 5>;
#else
  sparse_variant = 0;
  // the guided split (GuidedSplit: 5/8 static, the rest in 16-object ticket
  // chunks): 15.3 -> 13.5 ms per 8-replica fold of 1M objects (tools/ab_sparse.py)
  const void* fn = (const void*)orswot_sparse_mask_kernel<3, 0, 16, 5>;
#endif
  static std::atomic<int> occ_cache[16];  // per variant (the product: 0)
  const int oslot = sparse_variant >= 0 && sparse_variant < 16 ? sparse_variant : 0;
  occ = occ_cache[oslot].load(std::memory_order_relaxed);
  if (occ == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kWave * kWavesPerBlock, 0) != hipSuccess || occ < 1)
      occ = 2;
    occ_cache[oslot].store(occ, std::memory_order_relaxed);
  }
  const uint64_t chunks = (n_obj + kWave - 1) / kWave;
  const uint64_t want = (chunks + kWavesPerBlock - 1) / kWavesPerBlock;
  const uint64_t cap = (uint64_t)cus * occ;
  const uint32_t blocks = (uint32_t)(want < cap ? want : cap);
  // the product (sparse_variant 0) takes the dense join's alternating
  // control-word sets (launch_join_passes NM: no memset before the launch);
  // diagnostic variants keep ctl[0..3] and the memset
  const bool nm = sparse_variant == 0;
  uint32_t* set = nm ? ctl + 4u + 4u * (js->seq & 1u) : ctl;
  uint32_t* const other = nm ? ctl + 4u + 4u * (~js->seq & 1u) : nullptr;
  void* args[] = {&Lb, &Loff, &Lbytes, &Rb, &Roff, &Rbytes, &Ob, &Ooff, &Obytes, &n_obj, &n_actors, &status,
                  &set, &list, &list_cap};
  if (nm) {
    if (js->dirty && hipMemsetAsync(ctl + 4, 0, 8 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;
    js->dirty = true;  // until both kernels are launched
  } else if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) {  // ctl[3]: tickets
    return CRDT_EHIP;
  }
  if (hipLaunchKernel(fn, dim3(blocks), dim3(kWave * kWavesPerBlock), args, 0, stream) != hipSuccess)
    return CRDT_EHIP;
  if (sparse_variant == 3 || sparse_variant == 4) return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;  // diagnostics: no general pass
  // one block per resident slot (6 single-wave blocks per CU fit its 23 KB of
  // LDS): a fold step lists ~0.6 % of its objects here (pairs past the 6 KB
  // stage), so the listed objects spread over every CU
  hipLaunchKernelGGL(orswot_sparse_general_kernel, dim3((uint32_t)cus * 6u), dim3(kWave), 0, stream, Lb, Loff, Rb,
                     Roff, Ob, Ooff, n_obj, n_actors, set, list, list_cap, other);
  if (hipGetLastError() != hipSuccess) return CRDT_EHIP;
  // objects past 128 union positions or the general stage: one block each
  // (orswot_big_kernel<true>; it exits at once when the general kernel left none)
  if (launch_big<true>(Lb, Loff, Rb, Roff, Ob, Ooff, n_obj, n_actors, set, list, list_cap, stream) != hipSuccess)
    return CRDT_EHIP;
  if (nm) {
    ++js->seq;
    js->dirty = false;
  }
  return CRDT_OK;
}


}  // namespace crdts_hip

#ifdef CRDT_DIAG
// Diagnostic build only: wave 0's per-phase cycle sums of orswot_big_kernel's
// ABL 8 variant (diag variant 341), [15] = objects; read and cleared.
extern "C" int crdt_debug_big_stamps(uint64_t* h16) {
  unsigned long long z[16] = {};
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(h16, HIP_SYMBOL(crdts_hip::g_big_st), sizeof(z)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(crdts_hip::g_big_st), z, sizeof(z)) != hipSuccess)
    return CRDT_EHIP;
  return CRDT_OK;
}
#endif
