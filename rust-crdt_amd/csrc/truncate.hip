// Batched Causal::truncate for Orswot records (src/orswot.rs:159-172):
//
//     let mut empty_set = Orswot::new(); empty_set.clock = clock.clone();
//     self.merge(&empty_set);            // :87-157 with apply_deferred :235-243
//     self.clock.subtract(&clock);       // vclock.rs:236-242
//     for (_, member_clock) in self.entries.iter_mut() { member_clock.subtract(&clock); }
//
// Spelled out per record (c = the truncating clock, T = the top clock,
// M = max(T, c) the merged clock; canonical clocks: `a <= b` iff every
// a[x] <= b[x], vclock.rs:59-71):
//  - a member (every entry is self-only against the empty set, :94-104) is
//    kept by the merge iff some dot (x, v) of its clock has v > c[x];
//  - apply_deferred: every deferred (D, S) is re-deferred iff !(D <= M)
//    (the member set S unchanged), and every member of S loses the dots with
//    D[x] >= v (apply_remove :195-211), dropped if that empties its clock;
//  - the top clock keeps T[x] iff T[x] > c[x] (M[x] == c[x] otherwise);
//  - a kept member keeps the dots with v > c[x] — possibly none: the
//    reference keeps the member with an EMPTY clock then (it subtracts without
//    dropping). Such a record is written with header flag
//    CRDT_ORSWOT_EMPTY_MEMBER_CLOCK (an empty run), which the merge / apply /
//    codec kernels do not accept (not canonical for them).
// The output is never larger than the input (a subset of every section), so
// record i is written at out_off[i] := self.off[i].
//
// One wave per record, lane = member (runs walked per lane) / deferred clock
// in 64-wide chunks, two passes (count, write); lookups of c[x] and D[x]
// binary-search the sorted runs. Not the hot path: latency-bound, any size.
#include <hip/hip_runtime.h>

#include <atomic>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "record_layout.h"
#include "sched.h"

namespace crdts_hip {
namespace {

constexpr uint32_t kW = 64;
constexpr uint32_t kEmptyClockFlag = 2u;  // CRDT_ORSWOT_EMPTY_MEMBER_CLOCK

__device__ __forceinline__ void fail(int* status, int code) { atomicCAS(status, 0, code); }
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (uint32_t s = 32u; s; s >>= 1) v += __shfl_xor(v, (int)s);
  return v;
}
// exclusive prefix over lanes
__device__ __forceinline__ uint32_t wave_excl(uint32_t v, uint32_t lane) {
  uint32_t x = v;
  for (uint32_t s = 1u; s < kW; s <<= 1) {
    const uint32_t y = __shfl_up(x, (int)s);
    x += lane >= s ? y : 0u;
  }
  return x - v;
}

// A sorted (actor, counter) run in memory; get(x) = its counter or 0.
struct Run {
  const uint32_t* a;
  const uint64_t* c;
  uint32_t n;
  __device__ uint64_t get(uint32_t x) const {
    uint32_t lo = 0, len = n;
    while (len) {
      const uint32_t h = len >> 1;
      if (a[lo + h] < x) {
        lo += h + 1u;
        len -= h + 1u;
      } else {
        len = h;
      }
    }
    return lo < n && a[lo] == x ? c[lo] : 0ull;
  }
};

__device__ __forceinline__ bool has_key(const uint64_t* k, uint32_t n, uint64_t key) {
  uint32_t lo = 0, len = n;
  while (len) {
    const uint32_t h = len >> 1;
    if (k[lo + h] < key) {
      lo += h + 1u;
      len -= h + 1u;
    } else {
      len = h;
    }
  }
  return lo < n && k[lo] == key;
}

// Is the truncating clock run canonical — actors strictly increasing,
// counters > 0 (crdts_hip.h: a malformed run latches CRDT_ENONCANON)? Both
// lookups (Run::get's binary search, the LDS form's dense row) assume it.
// a0 / c0: this lane's entry of the first 64 (any value past the run).
__device__ __forceinline__ bool run_canonical(const Run& c, uint32_t a0, uint64_t c0, uint32_t lane) {
  bool bad = false;
  for (uint32_t b = 0; b < c.n; b += kW) {
    const uint32_t e = b + lane;
    uint32_t a = a0;
    uint64_t v = c0;
    if (b) {
      a = e < c.n ? c.a[e] : 0u;
      v = e < c.n ? c.c[e] : 1ull;
    }
    uint32_t prev = __shfl_up(a, 1);
    if (lane == 0u && b) prev = c.a[b - 1u];
    bad = bad || (e < c.n && (v == 0ull || (e > 0u && a <= prev)));
  }
  return __ballot(bad) == 0ull;
}

struct Rec {
  const uint8_t* r;
  RecLayout L;
  bool sparse;
  __device__ const uint64_t* key() const { return (const uint64_t*)(r + L.o_key); }
  __device__ const uint64_t* dctr() const { return (const uint64_t*)(r + L.o_dctr); }
  __device__ const uint32_t* dact() const { return (const uint32_t*)(r + L.o_dact); }
  __device__ const uint32_t* mdend() const { return (const uint32_t*)(r + L.o_mdend); }
  __device__ const uint64_t* fctr() const { return (const uint64_t*)(r + L.o_fctr); }
  __device__ const uint64_t* fkey() const { return (const uint64_t*)(r + L.o_fkey); }
  __device__ const uint32_t* fact() const { return (const uint32_t*)(r + L.o_fact); }
  __device__ const uint32_t* fdend() const { return (const uint32_t*)(r + L.o_fdend); }
  __device__ const uint32_t* fmend() const { return (const uint32_t*)(r + L.o_fmend); }
  // top clock T[x]
  __device__ uint64_t top(uint32_t x) const {
    if (!sparse) return x < L.n_clk ? ((const uint64_t*)(r + L.o_clk))[x] : 0ull;
    return Run{(const uint32_t*)(r + L.o_cact), (const uint64_t*)(r + L.o_clk), L.n_clk}.get(x);
  }
  // run ends clamped to their section, begins to their end: a malformed
  // record cannot send a lane outside its sections or a count negative
  __device__ uint32_t m_end(uint32_t m) const { return min(mdend()[m], L.n_dot); }
  __device__ uint32_t m_begin(uint32_t m) const { return m ? min(m_end(m - 1u), m_end(m)) : 0u; }
  __device__ uint32_t fd_end(uint32_t k) const { return min(fdend()[k], L.n_def_dot); }
  __device__ uint32_t fd_begin(uint32_t k) const { return k ? min(fd_end(k - 1u), fd_end(k)) : 0u; }
  __device__ uint32_t fm_end(uint32_t k) const { return min(fmend()[k], L.n_def_mem); }
  __device__ uint32_t fm_begin(uint32_t k) const { return k ? min(fm_end(k - 1u), fm_end(k)) : 0u; }
};

// Is the dot (x, v) of member `key` removed by a deferred clock naming the
// member (apply_remove's subtract: D[x] >= v)?
__device__ bool deferred_kills(const Rec& R, uint64_t key, uint32_t x, uint64_t v) {
  for (uint32_t k = 0; k < R.L.n_def; ++k) {
    const uint32_t m0 = R.fm_begin(k), m1 = R.fm_end(k);
    if (!has_key(R.fkey() + m0, m1 - m0, key)) continue;
    const uint32_t d0 = R.fd_begin(k), d1 = R.fd_end(k);
    if (Run{R.fact() + d0, R.fctr() + d0, d1 - d0}.get(x) >= v) return true;
  }
  return false;
}

struct TruncArgs {
  const uint8_t* base;
  const uint64_t* off;
  uint64_t bytes, n_obj;
  const uint64_t* coff;
  const uint32_t* clen;
  const uint32_t* cact;
  const uint64_t* cctr;
  uint64_t c_entries;
  uint32_t A, flags;
  uint8_t* out;
  uint64_t* out_off;
  uint64_t out_bytes;
  int* status;
};

// The general form: every read straight from HBM (any record size, dense or
// CSR top clock, any number of deferred clocks).
__device__ void truncate_global(const TruncArgs& g, const Rec& R, const Run& c, uint64_t o, uint32_t lane) {
  const bool sparse = R.sparse;
  const uint32_t flags = g.flags;
  int* const status = g.status;
  uint8_t* const out = g.out;
  {
    const RecLayout& L = R.L;
    // run ends of member / deferred runs are clamped: a malformed record cannot
    // send a lane past its sections

    // ---- pass 1: counts
    // top clock: T[x] kept iff T[x] > c[x]
    uint32_t n_clk = 0;
    for (uint32_t b = 0; b < L.n_clk; b += kW) {
      const uint32_t k = b + lane;
      uint64_t t = 0;
      uint32_t x = k;
      if (k < L.n_clk) {
        if (sparse) x = ((const uint32_t*)(R.r + L.o_cact))[k];
        t = ((const uint64_t*)(R.r + L.o_clk))[k];
      }
      n_clk += (uint32_t)__popcll(__ballot(k < L.n_clk && t > c.get(x)));
    }
    if (!sparse) n_clk = L.n_clk;  // dense: every slot is written (0 = absent)
    // deferred: (D, S) re-deferred iff !(D <= M), M = max(T, c)
    uint32_t n_def = 0, n_fdot = 0, n_fmem = 0;
    for (uint32_t b = 0; b < L.n_def; b += kW) {
      const uint32_t k = b + lane;
      bool keepd = false;
      uint32_t nd = 0, nm = 0;
      if (k < L.n_def) {
        const uint32_t d0 = R.fd_begin(k), d1 = R.fd_end(k);
        for (uint32_t d = d0; d < d1; ++d) {
          const uint32_t x = R.fact()[d];
          const uint64_t t = R.top(x), cx = c.get(x);
          keepd = keepd || R.fctr()[d] > (t > cx ? t : cx);
        }
        nd = d1 - d0;
        nm = R.fm_end(k) - R.fm_begin(k);
      }
      n_def += (uint32_t)__popcll(__ballot(keepd));
      n_fdot += wave_sum(keepd ? nd : 0u);
      n_fmem += wave_sum(keepd ? nm : 0u);
    }
    // members: kept iff some dot v > c[x] and some dot survives the deferred
    // subtracts; final dots: v > c[x] and not removed by a deferred clock
    uint32_t n_mem = 0, n_dot = 0;
    bool empty_clock = false;
    for (uint32_t b = 0; b < L.n_mem; b += kW) {
      const uint32_t m = b + lane;
      uint32_t fin = 0;
      bool above = false, alive = false;
      if (m < L.n_mem) {
        const uint64_t key = R.key()[m];
        for (uint32_t d = R.m_begin(m); d < R.m_end(m); ++d) {
          const uint32_t x = R.dact()[d];
          const uint64_t v = R.dctr()[d];
          const bool gt = v > c.get(x);
          const bool dk = L.n_def && deferred_kills(R, key, x, v);
          above = above || gt;
          alive = alive || !dk;
          fin += gt && !dk ? 1u : 0u;
        }
      }
      const bool kept = above && alive;
      n_mem += (uint32_t)__popcll(__ballot(kept));
      n_dot += wave_sum(kept ? fin : 0u);
      empty_clock = empty_clock || __ballot(kept && fin == 0u) != 0ull;
    }
    RecLayout O;
    rec_layout(O, n_clk, n_mem, n_dot, n_def, n_fdot, n_fmem, sparse);
    if (O.size > L.size) {  // cannot happen for a canonical record
      if (lane == 0u) fail(status, CRDT_ENONCANON);
      return;
    }
    uint8_t* w = out + o;

    // ---- pass 2: write
    // top clock
    {
      uint32_t at = 0;
      for (uint32_t b = 0; b < L.n_clk; b += kW) {
        const uint32_t k = b + lane;
        uint64_t t = 0;
        uint32_t x = k;
        if (k < L.n_clk) {
          if (sparse) x = ((const uint32_t*)(R.r + L.o_cact))[k];
          t = ((const uint64_t*)(R.r + L.o_clk))[k];
        }
        const bool keep = k < L.n_clk && t > c.get(x);
        if (!sparse) {
          if (k < L.n_clk) ((uint64_t*)(w + O.o_clk))[k] = keep ? t : 0ull;
        } else {
          const uint64_t K = __ballot(keep);
          const uint32_t p = at + mbcnt(K);
          if (keep) {
            ((uint64_t*)(w + O.o_clk))[p] = t;
            ((uint32_t*)(w + O.o_cact))[p] = x;
          }
          at += (uint32_t)__popcll(K);
        }
      }
      if (sparse && lane == 0u && O.o_key != O.o_cact + 4u * n_clk)
        *(uint32_t*)(w + O.o_cact + 4u * n_clk) = 0u;  // pad to 8
    }
    // members
    {
      uint32_t at_m = 0, at_d = 0;
      for (uint32_t b = 0; b < L.n_mem; b += kW) {
        const uint32_t m = b + lane;
        uint32_t fin = 0;
        bool above = false, alive = false;
        uint64_t key = 0;
        const uint32_t d0 = m < L.n_mem ? R.m_begin(m) : 0u;
        const uint32_t d1 = m < L.n_mem ? R.m_end(m) : 0u;
        if (m < L.n_mem) {
          key = R.key()[m];
          for (uint32_t d = d0; d < d1; ++d) {
            const uint32_t x = R.dact()[d];
            const uint64_t v = R.dctr()[d];
            const bool gt = v > c.get(x);
            const bool dk = L.n_def && deferred_kills(R, key, x, v);
            above = above || gt;
            alive = alive || !dk;
            fin += gt && !dk ? 1u : 0u;
          }
        }
        const bool kept = above && alive;
        const uint64_t K = __ballot(kept);
        const uint32_t pm = at_m + mbcnt(K);
        const uint32_t cnt = kept ? fin : 0u;
        const uint32_t pd = at_d + wave_excl(cnt, lane);
        if (kept) {
          ((uint64_t*)(w + O.o_key))[pm] = key;
          ((uint32_t*)(w + O.o_mdend))[pm] = pd + cnt;
          uint32_t q = pd;
          for (uint32_t d = d0; d < d1; ++d) {
            const uint32_t x = R.dact()[d];
            const uint64_t v = R.dctr()[d];
            if (v > c.get(x) && !(L.n_def && deferred_kills(R, key, x, v))) {
              ((uint64_t*)(w + O.o_dctr))[q] = v;
              ((uint32_t*)(w + O.o_dact))[q] = x;
              ++q;
            }
          }
        }
        at_m += (uint32_t)__popcll(K);
        at_d += wave_sum(cnt);
      }
    }
    // deferred (kept ones, in their CLOCK ORDER, sets unchanged)
    {
      uint32_t at = 0, at_d = 0, at_m = 0;
      for (uint32_t b = 0; b < L.n_def; b += kW) {
        const uint32_t k = b + lane;
        bool keepd = false;
        uint32_t d0 = 0, d1 = 0, m0 = 0, m1 = 0;
        if (k < L.n_def) {
          d0 = R.fd_begin(k);
          d1 = R.fd_end(k);
          m0 = R.fm_begin(k);
          m1 = R.fm_end(k);
          for (uint32_t d = d0; d < d1; ++d) {
            const uint32_t x = R.fact()[d];
            const uint64_t t = R.top(x), cx = c.get(x);
            keepd = keepd || R.fctr()[d] > (t > cx ? t : cx);
          }
        }
        const uint64_t K = __ballot(keepd);
        const uint32_t nd = keepd ? d1 - d0 : 0u, nm = keepd ? m1 - m0 : 0u;
        const uint32_t p = at + mbcnt(K), pd = at_d + wave_excl(nd, lane), pmm = at_m + wave_excl(nm, lane);
        if (keepd) {
          for (uint32_t d = 0; d < nd; ++d) {
            ((uint64_t*)(w + O.o_fctr))[pd + d] = R.fctr()[d0 + d];
            ((uint32_t*)(w + O.o_fact))[pd + d] = R.fact()[d0 + d];
          }
          for (uint32_t j = 0; j < nm; ++j) ((uint64_t*)(w + O.o_fkey))[pmm + j] = R.fkey()[m0 + j];
          ((uint32_t*)(w + O.o_fdend))[p] = pd + nd;
          ((uint32_t*)(w + O.o_fmend))[p] = pmm + nm;
        }
        at += (uint32_t)__popcll(K);
        at_d += wave_sum(nd);
        at_m += wave_sum(nm);
      }
    }
    // zero padding (member block to 8, record to 16) and the header
    if (lane == 0u && O.o_def != O.o_mpad) *(uint32_t*)(w + O.o_mpad) = 0u;
    if (lane >= 1u && lane < 4u && O.o_end + 4u * (lane - 1u) < O.size) *(uint32_t*)(w + O.o_end + 4u * (lane - 1u)) = 0u;
    if (lane == 0u) {
      uint32_t* hw = (uint32_t*)w;
      hw[0] = O.size;
      hw[1] = n_clk;
      hw[2] = n_mem;
      hw[3] = n_dot;
      hw[4] = n_def;
      hw[5] = n_fdot;
      hw[6] = n_fmem;
      hw[7] = flags | (empty_clock ? kEmptyClockFlag : 0u);
    }
  }
}

// ---------------------------------------------------------------- LDS form
// Records of dense top clocks over A <= 32 actors, <= kTStage bytes and <= 8
// deferred clocks (config 3: every record) are staged in LDS with the
// truncating clock as a dense row c[x] and every deferred clock as a dense row
// D_k[x]; each member carries the mask of the deferred clocks naming it. The
// same two passes then read only LDS: c[x] and D_k[x] are one read each
// instead of binary searches through HBM. Everything else takes
// truncate_global.
constexpr uint32_t kTStage = 4096;
constexpr uint32_t kTDef = 8;
constexpr uint32_t kTA = 32;
constexpr uint32_t kTWaves = 4;
struct TWs {
  uint32_t stage[kTStage / 4];
  uint64_t ct[kTA];
  uint64_t drow[kTDef][kTA];
  uint32_t nm[kTStage / 24];  // per member: the deferred clocks naming it (a member takes >= 24 B of a record)
};

__device__ __forceinline__ void tsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr uint32_t kTPer = kTStage / 16u / kW;  // 16-B record pieces per lane
typedef uint32_t tu32x4 __attribute__((ext_vector_type(4)));
// An LDS-form object's record (every 16-B piece, clamped to its last) and the
// first 64 entries of its clock, in registers one object ahead
struct TPre {
  tu32x4 r[kTPer];
  uint32_t a;
  uint64_t c;
};
__device__ __forceinline__ void tfetch(TPre& p, const uint8_t* rec, uint32_t n16, const Run& c, uint32_t lane) {
#pragma unroll
  for (uint32_t k = 0; k < kTPer; ++k) {
    const uint32_t i = lane + k * kW;
    p.r[k] = __builtin_nontemporal_load((const tu32x4*)rec + (i < n16 ? i : n16 - 1u));
  }
  p.a = 0xFFFFFFFFu;
  p.c = 0ull;
  if (lane < c.n) { p.a = c.a[lane]; p.c = c.c[lane]; }
}

// Stage an LDS-form record (p: its prefetched pieces and first 64 clock
// entries; c: its clock run, for entries past those) and zero the tables.
__device__ void tstage(TWs& w, const RecLayout& L, const TPre& p, const Run& c, uint32_t lane) {
  const uint32_t n16 = L.size / 16u;
#pragma unroll
  for (uint32_t k = 0; k < kTPer; ++k)
    if (lane + k * kW < n16) ((tu32x4*)w.stage)[lane + k * kW] = p.r[k];
  if (lane < kTA) w.ct[lane] = 0ull;
  for (uint32_t k = lane; k < kTDef * kTA; k += kW) w.drow[k / kTA][k % kTA] = 0ull;
  for (uint32_t m = lane; m < L.n_mem; m += kW) w.nm[m] = 0u;
  tsync();
  if (p.a < kTA) w.ct[p.a] = p.c;  // actors >= A name nothing a dense record holds
  for (uint32_t e = kW + lane; e < c.n; e += kW) {
    const uint32_t x = c.a[e];
    if (x < kTA) w.ct[x] = c.c[e];
  }
}

// The LDS form of one staged record. wide: a dot or deferred actor >= A (not
// canonical here): nothing written, the HBM form decides.
__device__ void truncate_lds(const TruncArgs& g, const Rec& R, uint64_t o, uint32_t lane, TWs& w, bool& wide) {
  const RecLayout& L = R.L;
  const uint32_t A = L.n_clk;
  const uint8_t* S = (const uint8_t*)w.stage;
  {
    bool wd = false;
    for (uint32_t d = lane; d < L.n_dot; d += kW) wd = wd || ((const uint32_t*)(S + L.o_dact))[d] >= A;
    for (uint32_t d = lane; d < L.n_def_dot; d += kW) wd = wd || ((const uint32_t*)(S + L.o_fact))[d] >= A;
    if (__ballot(wd) != 0ull) {
      wide = true;
      tsync();
      return;
    }
  }
  const uint32_t* fdend = (const uint32_t*)(S + L.o_fdend);
  const uint32_t* fmend = (const uint32_t*)(S + L.o_fmend);
  const uint32_t* fact = (const uint32_t*)(S + L.o_fact);
  const uint64_t* fctr = (const uint64_t*)(S + L.o_fctr);
  const uint64_t* fkey = (const uint64_t*)(S + L.o_fkey);
  const uint64_t* key = (const uint64_t*)(S + L.o_key);
  const uint32_t* dact = (const uint32_t*)(S + L.o_dact);
  const uint64_t* dctr = (const uint64_t*)(S + L.o_dctr);
  const uint32_t* mdend = (const uint32_t*)(S + L.o_mdend);
  const uint64_t* top = (const uint64_t*)(S + L.o_clk);
  auto clock_of = [&](const uint32_t* ends, uint32_t j) {  // # run ends <= j: the clock of item j (<= kTDef runs)
    uint32_t k = 0;
    for (uint32_t t = 0; t < L.n_def; ++t) k += ends[t] <= j ? 1u : 0u;
    return k;
  };
  for (uint32_t e = lane; e < L.n_def_dot; e += kW) {
    const uint32_t k = clock_of(fdend, e), x = fact[e];
    if (k < kTDef && x < kTA) w.drow[k][x] = fctr[e];
  }
  for (uint32_t j = lane; j < L.n_def_mem; j += kW) {
    const uint32_t k = clock_of(fmend, j);
    const uint64_t m = fkey[j];
    uint32_t lo = 0, len = L.n_mem;  // the member's index (absent: no member to name)
    while (len) {
      const uint32_t h = len >> 1;
      if (key[lo + h] < m) { lo += h + 1u; len -= h + 1u; } else { len = h; }
    }
    if (lo < L.n_mem && key[lo] == m && k < kTDef) atomicOr(&w.nm[lo], 1u << k);
  }
  tsync();
  auto mend = [&](uint32_t m) { return min(mdend[m], L.n_dot); };
  auto mbeg = [&](uint32_t m) { return m ? min(mend(m - 1u), mend(m)) : 0u; };
  auto fdb = [&](uint32_t k) { return k ? min(min(fdend[k - 1u], L.n_def_dot), min(fdend[k], L.n_def_dot)) : 0u; };
  auto fde = [&](uint32_t k) { return min(fdend[k], L.n_def_dot); };
  auto fmb = [&](uint32_t k) { return k ? min(min(fmend[k - 1u], L.n_def_mem), min(fmend[k], L.n_def_mem)) : 0u; };
  auto fme = [&](uint32_t k) { return min(fmend[k], L.n_def_mem); };
  auto killed = [&](uint32_t names, uint32_t x, uint64_t v) {
    bool dk = false;
    for (uint32_t b = names; b; b &= b - 1u) dk = dk || w.drow[__builtin_ctz(b)][x] >= v;
    return dk;
  };

  // ---- one pass for records without deferred removes, <= 64 members of <=
  // 4 dots (config 3's common record): every lane reads its member's key and
  // dots into registers, counts and layout follow from two wave reductions,
  // then the output record is assembled over the stage (all reads are done,
  // so writing in place is safe) and copied out with 16-B stores — the
  // scattered 4- / 8-B HBM stores of the general write pass below kept the
  // texture-address unit busy (as they did in the join). With
  // no deferred clock nothing is killed, so a kept member keeps >= 1 dot.
  constexpr uint32_t kTK = 4;  // dots per member held in registers
  if (L.n_def == 0u && L.n_mem <= kW &&
      __ballot(lane < L.n_mem && mend(lane) - mbeg(lane) > kTK) == 0ull) {
    const bool hm = lane < L.n_mem;
    const uint32_t d0 = hm ? mbeg(lane) : 0u, nd = hm ? mend(lane) - d0 : 0u;
    const uint64_t kk = hm ? key[lane] : 0ull;
    uint32_t xs[kTK];
    uint64_t vs[kTK];
    uint32_t keepb = 0u, fin = 0u;  // bit j: dot j is kept (above c, none of these records kills)
    bool above = false;
#pragma unroll
    for (uint32_t j = 0; j < kTK; ++j) {
      xs[j] = j < nd ? dact[d0 + j] : 0u;
      vs[j] = j < nd ? dctr[d0 + j] : 0ull;
      const bool gt = j < nd && vs[j] > w.ct[xs[j] & (kTA - 1u)];
      above = above || gt;
      keepb |= gt ? 1u << j : 0u;
      fin += gt ? 1u : 0u;
    }
    const uint64_t tx = lane < A ? top[lane] : 0ull, cx = lane < A ? w.ct[lane] : 0ull;
    const bool kept = hm && above;  // (alive: no deferred clock names a member here)
    const uint64_t K = __ballot(kept);
    const uint32_t pm = mbcnt(K), cnt = kept ? fin : 0u, pd = wave_excl(cnt, lane);
    const uint32_t n_mem = (uint32_t)__popcll(K), n_dot = wave_sum(cnt);
    RecLayout O;
    rec_layout(O, A, n_mem, n_dot, 0u, 0u, 0u, false);
    if (O.size > L.size) {  // cannot happen for a canonical record
      if (lane == 0u) fail(g.status, CRDT_ENONCANON);
      tsync();
      return;
    }
    uint8_t* wout = g.out + o;
    tsync();  // every read of the stage is done: the output is assembled over it
    uint8_t* S8 = (uint8_t*)w.stage;
    if (lane < A) ((uint64_t*)(S8 + O.o_clk))[lane] = tx > cx ? tx : 0ull;
    if (kept) {
      ((uint64_t*)(S8 + O.o_key))[pm] = kk;
      ((uint32_t*)(S8 + O.o_mdend))[pm] = pd + cnt;
      uint32_t q = pd;
#pragma unroll
      for (uint32_t j = 0; j < kTK; ++j) {
        if ((keepb >> j) & 1u) {
          ((uint64_t*)(S8 + O.o_dctr))[q] = vs[j];
          ((uint32_t*)(S8 + O.o_dact))[q] = xs[j];
          ++q;
        }
      }
    }
    if (lane == 0u && O.o_def != O.o_mpad) *(uint32_t*)(S8 + O.o_mpad) = 0u;
    if (lane >= 1u && lane < 4u && O.o_end + 4u * (lane - 1u) < O.size) *(uint32_t*)(S8 + O.o_end + 4u * (lane - 1u)) = 0u;
    if (lane < 8u) {
      const uint32_t hv[8] = {O.size, A, n_mem, n_dot, 0u, 0u, 0u, g.flags};
      uint32_t h = 0u;
#pragma unroll
      for (uint32_t t = 0; t < 8u; ++t) h = lane == t ? hv[t] : h;
      ((uint32_t*)S8)[lane] = h;
    }
    tsync();
    for (uint32_t k = lane; k < O.size / 16u; k += kW)
      __builtin_nontemporal_store(((const tu32x4*)S8)[k], (tu32x4*)wout + k);
    tsync();  // the stage is reused by the wave's next record
    return;
  }

  // ---- pass 1: counts (the dense top clock keeps all A slots)
  uint32_t n_def = 0, n_fdot = 0, n_fmem = 0;
  for (uint32_t b = 0; b < L.n_def; b += kW) {
    const uint32_t k = b + lane;
    bool keepd = false;
    uint32_t nd = 0, nmm = 0;
    if (k < L.n_def) {
      for (uint32_t d = fdb(k); d < fde(k); ++d) {
        const uint32_t x = fact[d];
        const uint64_t t = x < A ? top[x] : 0ull, cx = x < kTA ? w.ct[x] : 0ull;
        keepd = keepd || fctr[d] > (t > cx ? t : cx);
      }
      nd = fde(k) - fdb(k);
      nmm = fme(k) - fmb(k);
    }
    n_def += (uint32_t)__popcll(__ballot(keepd));
    n_fdot += wave_sum(keepd ? nd : 0u);
    n_fmem += wave_sum(keepd ? nmm : 0u);
  }
  uint32_t n_mem = 0, n_dot = 0;
  bool empty_clock = false;
  for (uint32_t b = 0; b < L.n_mem; b += kW) {
    const uint32_t m = b + lane;
    uint32_t fin = 0;
    bool above = false, alive = false;
    if (m < L.n_mem) {
      const uint32_t names = w.nm[m];
      for (uint32_t d = mbeg(m); d < mend(m); ++d) {
        const uint32_t x = dact[d];
        const uint64_t v = dctr[d];
        const bool gt = v > w.ct[x & (kTA - 1u)];
        const bool dk = killed(names, x & (kTA - 1u), v);
        above = above || gt;
        alive = alive || !dk;
        fin += gt && !dk ? 1u : 0u;
      }
    }
    const bool kept = above && alive;
    n_mem += (uint32_t)__popcll(__ballot(kept));
    n_dot += wave_sum(kept ? fin : 0u);
    empty_clock = empty_clock || __ballot(kept && fin == 0u) != 0ull;
  }
  RecLayout O;
  rec_layout(O, A, n_mem, n_dot, n_def, n_fdot, n_fmem, false);
  if (O.size > L.size) {  // cannot happen for a canonical record
    if (lane == 0u) fail(g.status, CRDT_ENONCANON);
    return;
  }
  uint8_t* wout = g.out + o;

  // ---- pass 2: write (HBM)
  if (lane < A) ((uint64_t*)(wout + O.o_clk))[lane] = top[lane] > w.ct[lane] ? top[lane] : 0ull;
  {
    uint32_t at_m = 0, at_d = 0;
    for (uint32_t b = 0; b < L.n_mem; b += kW) {
      const uint32_t m = b + lane;
      uint32_t fin = 0, names = 0;
      bool above = false, alive = false;
      const uint32_t d0 = m < L.n_mem ? mbeg(m) : 0u, d1 = m < L.n_mem ? mend(m) : 0u;
      if (m < L.n_mem) {
        names = w.nm[m];
        for (uint32_t d = d0; d < d1; ++d) {
          const uint32_t x = dact[d] & (kTA - 1u);
          const uint64_t v = dctr[d];
          const bool gt = v > w.ct[x];
          const bool dk = killed(names, x, v);
          above = above || gt;
          alive = alive || !dk;
          fin += gt && !dk ? 1u : 0u;
        }
      }
      const bool kept = above && alive;
      const uint64_t K = __ballot(kept);
      const uint32_t pm = at_m + mbcnt(K);
      const uint32_t cnt = kept ? fin : 0u;
      const uint32_t pd = at_d + wave_excl(cnt, lane);
      if (kept) {
        ((uint64_t*)(wout + O.o_key))[pm] = key[m];
        ((uint32_t*)(wout + O.o_mdend))[pm] = pd + cnt;
        uint32_t q = pd;
        for (uint32_t d = d0; d < d1; ++d) {
          const uint32_t x = dact[d] & (kTA - 1u);
          const uint64_t v = dctr[d];
          if (v > w.ct[x] && !killed(names, x, v)) {
            ((uint64_t*)(wout + O.o_dctr))[q] = v;
            ((uint32_t*)(wout + O.o_dact))[q] = dact[d];
            ++q;
          }
        }
      }
      at_m += (uint32_t)__popcll(K);
      at_d += wave_sum(cnt);
    }
  }
  {
    uint32_t at = 0, at_d = 0, at_m = 0;
    for (uint32_t b = 0; b < L.n_def; b += kW) {
      const uint32_t k = b + lane;
      bool keepd = false;
      uint32_t d0 = 0, d1 = 0, m0 = 0, m1 = 0;
      if (k < L.n_def) {
        d0 = fdb(k);
        d1 = fde(k);
        m0 = fmb(k);
        m1 = fme(k);
        for (uint32_t d = d0; d < d1; ++d) {
          const uint32_t x = fact[d];
          const uint64_t t = x < A ? top[x] : 0ull, cx = x < kTA ? w.ct[x] : 0ull;
          keepd = keepd || fctr[d] > (t > cx ? t : cx);
        }
      }
      const uint64_t K = __ballot(keepd);
      const uint32_t nd = keepd ? d1 - d0 : 0u, nmm = keepd ? m1 - m0 : 0u;
      const uint32_t p = at + mbcnt(K), pd = at_d + wave_excl(nd, lane), pmm = at_m + wave_excl(nmm, lane);
      if (keepd) {
        for (uint32_t d = 0; d < nd; ++d) {
          ((uint64_t*)(wout + O.o_fctr))[pd + d] = fctr[d0 + d];
          ((uint32_t*)(wout + O.o_fact))[pd + d] = fact[d0 + d];
        }
        for (uint32_t j = 0; j < nmm; ++j) ((uint64_t*)(wout + O.o_fkey))[pmm + j] = fkey[m0 + j];
        ((uint32_t*)(wout + O.o_fdend))[p] = pd + nd;
        ((uint32_t*)(wout + O.o_fmend))[p] = pmm + nmm;
      }
      at += (uint32_t)__popcll(K);
      at_d += wave_sum(nd);
      at_m += wave_sum(nmm);
    }
  }
  if (lane == 0u && O.o_def != O.o_mpad) *(uint32_t*)(wout + O.o_mpad) = 0u;
  if (lane >= 1u && lane < 4u && O.o_end + 4u * (lane - 1u) < O.size) *(uint32_t*)(wout + O.o_end + 4u * (lane - 1u)) = 0u;
  if (lane == 0u) {
    uint32_t* hw = (uint32_t*)wout;
    hw[0] = O.size;
    hw[1] = A;
    hw[2] = n_mem;
    hw[3] = n_dot;
    hw[4] = n_def;
    hw[5] = n_fdot;
    hw[6] = n_fmem;
    hw[7] = g.flags | (empty_clock ? kEmptyClockFlag : 0u);
  }
  tsync();  // the stage is reused by the wave's next record
}

// One wave per 64-record chunk: lane k reads record cbase + k's offset, clock
// run and header (one round trip for the chunk); then the chunk's LDS-form
// records are truncated one by one with the next one's record and clock in
// flight in registers, and the others (CSR top clocks, records past the LDS
// limits or not canonical here) in the HBM form.
// FLAGGED (after orswot_truncate_fast_kernel): only the records whose output
// offset the fast kernel left flagged (kTPend) are this kernel's; the flag is
// cleared when the record is written here.
constexpr uint64_t kTPend = 1ull << 63;
template <bool FLAGGED>
__global__ __launch_bounds__(kW * kTWaves, 4) void orswot_truncate_kernel(TruncArgs g, const uint32_t* flagged,
                                                                          const uint64_t* list, uint32_t list_cap) {
  // FLAGGED: flagged[0] counts the records the fast kernel left (none: done),
  // listed at list[0, count) unless the count passed list_cap (then every
  // output offset's flag is scanned)
  const uint32_t nfl =
      FLAGGED ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(flagged, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0u;
  if (FLAGGED && nfl == 0u) return;
  const bool listed = FLAGGED && nfl <= list_cap;
  const uint64_t n_units = listed ? (uint64_t)nfl : g.n_obj;
  __shared__ TWs ws[kTWaves];
  const uint32_t lane = threadIdx.x & (kW - 1u), wv = threadIdx.x / kW;
  TWs& w = ws[wv];
  const uint64_t wave = (uint64_t)blockIdx.x * kTWaves + wv;
  const uint64_t n_waves = (uint64_t)gridDim.x * kTWaves;
  const bool sparse = (g.flags & kSparseClock) != 0u;
  // listed: one entry per wave at a time (the few listed records spread over
  // every wave, not 64 to a wave); else 64-record chunks
  const uint64_t per = listed ? 1u : kW;
  for (uint64_t cb = wave * per; cb < n_units; cb += n_waves * per) {
    const uint64_t obj = listed ? (lane == 0u ? list[cb] : g.n_obj) : cb + lane;
    const bool valid = obj < g.n_obj && (!FLAGGED || (g.out_off[obj] & kTPend) != 0ull);
    if (FLAGGED && __ballot(valid) == 0ull) continue;
    uint64_t o = 0, c0 = 0;
    uint32_t cn = 0;
    if (valid) {
      o = g.off[obj];
      c0 = g.coff[obj];
      cn = g.clen[obj];
      g.out_off[obj] = o;
    }
    bool ok = valid && (o & 15u) == 0u && o <= g.bytes && g.bytes - o >= kHdrBytes;
    tu32x4 h0 = {0u, 0u, 0u, 0u}, h1 = h0;
    if (ok) {
      h0 = ((const tu32x4*)(g.base + o))[0];
      h1 = ((const tu32x4*)(g.base + o))[1];
    }
    RecLayout L;
    rec_layout(L, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, sparse);
    // a record truncate wrote may hold empty member clocks (flag bit 1): truncating
    // it again drops them (empty <= c), as the reference's repeated truncates do
    ok = ok && h0.x == L.size && (h1.w & ~kEmptyClockFlag) == g.flags && (sparse ? h0.y <= g.A : h0.y == g.A) && L.size <= g.bytes - o &&
         o + L.size <= g.out_bytes && c0 <= g.c_entries && cn <= g.c_entries - c0;
    if (__ballot(valid && !ok) != 0ull && lane == 0u) fail(g.status, CRDT_ENONCANON);
    const bool lds = ok && !sparse && h0.y <= kTA && L.size <= kTStage && h1.x <= kTDef && h0.z <= kTStage / 24u;
    auto rec_of = [&](uint32_t t, Rec& R, Run& c, uint64_t& ot) {
      ot = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)o, t) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(o >> 32), t) << 32);
      const uint64_t ct0 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)c0, t) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(c0 >> 32), t) << 32);
      R = Rec{g.base + ot, {}, sparse};
      rec_layout(R.L, __builtin_amdgcn_readlane(h0.y, t), __builtin_amdgcn_readlane(h0.z, t),
                 __builtin_amdgcn_readlane(h0.w, t), __builtin_amdgcn_readlane(h1.x, t),
                 __builtin_amdgcn_readlane(h1.y, t), __builtin_amdgcn_readlane(h1.z, t), sparse);
      c = Run{g.cact + ct0, g.cctr + ct0, (uint32_t)__builtin_amdgcn_readlane(cn, t)};
    };
    // the HBM form (rare on dense batches)
    for (uint64_t m = __ballot(ok && !lds); m; m &= m - 1u) {
      Rec R;
      Run c;
      uint64_t ot;
      rec_of((uint32_t)__builtin_ctzll(m), R, c, ot);
      const bool cok = run_canonical(c, lane < c.n ? c.a[lane] : 0u, lane < c.n ? c.c[lane] : 1ull, lane);
      if (cok) truncate_global(g, R, c, ot, lane);
      else if (lane == 0u) fail(g.status, CRDT_ENONCANON);
    }
    // the LDS form, one record ahead
    uint64_t pend = __ballot(lds);
    if (pend == 0ull) continue;
    uint32_t t = (uint32_t)__builtin_ctzll(pend);
    pend &= pend - 1u;
    Rec R;
    Run c;
    uint64_t ot;
    rec_of(t, R, c, ot);
    TPre p;
    tfetch(p, R.r, R.L.size / 16u, c, lane);
    for (;;) {
      const Rec Rc = R;
      const uint64_t oc = ot;
      const Run cc = c;
      tstage(w, Rc.L, p, cc, lane);
      const bool cok = run_canonical(cc, p.a, p.c, lane);
      const bool more = pend != 0ull;
      if (more) {  // the next record's loads, in flight while this one is truncated
        t = (uint32_t)__builtin_ctzll(pend);
        pend &= pend - 1u;
        rec_of(t, R, c, ot);
        tfetch(p, R.r, R.L.size / 16u, c, lane);
      }
      bool wide = false;
      if (cok) {
        truncate_lds(g, Rc, oc, lane, w, wide);
        if (wide) truncate_global(g, Rc, cc, oc, lane);
      } else {
        if (lane == 0u) fail(g.status, CRDT_ENONCANON);
        tsync();  // the stage is reused by the wave's next record
      }
      if (!more) break;
    }
  }
}


// ---------------------------------------------------------------- fast form
// The common record — dense top clock over A <= 32 actors, <= 64 members, <= 64
// dots, <= 8 deferred clocks of <= 64 entries and <= 64 named members in
// total, <= 2 KB, a truncating clock run of <= 64 entries — with the join
// kernel's skeleton (orswot_join5_kernel): a resident grid with the guided
// split, the chunk's offsets, clock runs and headers in one step (lane =
// object), the next record and clock run prefetched into registers while the
// current one is done from LDS, the output assembled over the stage and
// copied out with 16-B stores. Lane = dot / member / deferred entry; every
// per-member and per-clock quantity is a ballot over run masks.
// Truncate (src/orswot.rs:159-172: merge with the empty set :94-104 +
// apply_deferred :235-243, then VClock::subtract src/vclock.rs:236-242), with
// M = max(T, c):
//  - a dot (x, v) is above iff v > c[x], killed iff a deferred clock naming
//    its member has D[x] >= v;
//  - a member is kept iff one of its dots is above and one is not killed; it
//    keeps its dots that are above and not killed (possibly none: an empty
//    clock, header flag bit 1, as the reference keeps it);
//  - a deferred clock is kept (entries and member set unchanged) iff one of
//    its entries (x, d) has d > M[x];
//  - the top clock keeps T[x] iff T[x] > c[x].
// Every other record is flagged (kTPend on its output offset) for
// orswot_truncate_kernel<true>, which also latches every error.
constexpr uint32_t kTFStage = 2048;               // record bytes staged per wave
constexpr uint32_t kTFPer = kTFStage / 16u / kW;  // 16-B pieces per lane
constexpr uint32_t kTFDef = 8;                    // deferred clocks
struct TFWs {
  tu32x4 stage[kTFStage / 16];
  uint64_t ct[kTA];            // the truncating clock, dense
  uint64_t drow[kTFDef][kTA];  // the deferred clocks, dense
  uint32_t names[kW];          // per member: the deferred clocks naming it
};
__device__ __forceinline__ void tf_sync() { tsync(); }
__device__ __forceinline__ uint64_t lane64(uint64_t v, uint32_t t) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), t) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, t);
}
__device__ __forceinline__ uint64_t below_mask(uint32_t n) { return n >= 64u ? ~0ull : (1ull << n) - 1ull; }

__global__ __launch_bounds__(kW * kTWaves, 8) void orswot_truncate_fast_kernel(TruncArgs g, uint32_t* ctl,
                                                                               uint64_t* list, uint32_t list_cap) {
  __shared__ TFWs ws[kTWaves];
  const uint32_t lane = threadIdx.x & (kW - 1u), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kW);
  TFWs& w = ws[wv];
  const uint64_t wave_id = (uint64_t)blockIdx.x * kTWaves + wv, n_waves = (uint64_t)gridDim.x * kTWaves;
  const uint32_t A = g.A;
  const uint64_t lt = (1ull << lane) - 1ull;
  GuidedSplit<20u, 5u> gs(g.n_obj, wave_id, n_waves);
  uint64_t cbase, cend;
  while (gs.next(cbase, cend, &ctl[3], lane)) {
    // ---- chunk step: lane k <-> object cbase + k
    const uint64_t obj = cbase + lane;
    const bool valid = obj < cend;
    uint64_t o = 0, c0 = 0;
    uint32_t cn = 0;
    if (valid) {
      o = g.off[obj];
      c0 = g.coff[obj];
      cn = g.clen[obj];
    }
    bool ok = valid && (o & 15u) == 0u && o <= g.bytes && g.bytes - o >= kHdrBytes;
    tu32x4 h0 = {0u, 0u, 0u, 0u}, h1 = h0;
    if (ok) {
      h0 = ((const tu32x4*)(g.base + o))[0];
      h1 = ((const tu32x4*)(g.base + o))[1];
    }
    // the fast form's own verdict (the rest, well-formed or not, is the
    // general kernel's: it latches the errors). A record with empty member
    // clocks takes it only without deferred removes.
    const bool lim = h0.y == A && A <= kTA && h0.z <= kW && h0.w <= kW && h1.x <= kTFDef && h1.y <= kW && h1.z <= kW &&
                     h0.x <= kTFStage && (h1.w == 0u || (h1.w == kEmptyClockFlag && h1.x == 0u));
    uint32_t want = 0u;
    if (lim) {
      RecLayout L;
      rec_layout(L, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, false);
      want = L.size;
    }
    const bool fast = ok && lim && h0.x == want && h0.x <= g.bytes - o && o + h0.x <= g.out_bytes &&
                      c0 <= g.c_entries && cn <= g.c_entries - c0 && cn <= kW;
    if (valid) g.out_off[obj] = o | (fast ? 0ull : kTPend);
    // listed for the general kernel (one atomic per wave)
    const uint64_t left = __ballot(valid && !fast);
    if (left != 0ull) {
      uint32_t base = 0u;
      if (lane == 0u) base = atomicAdd(&ctl[0], (uint32_t)__popcll(left));
      base = __builtin_amdgcn_readfirstlane(base);
      const uint32_t e = base + (uint32_t)__popcll(left & lt);
      if (valid && !fast && e < list_cap) list[e] = obj;
    }
    uint64_t pend = __ballot(fast);
    if (pend == 0ull) continue;
    const uint32_t n16 = fast ? h0.x / 16u : 1u;
    const uint32_t nmd = h0.z | (h0.w << 16);
    const uint32_t nf = h1.x | (h1.y << 8) | (h1.z << 16) | (h1.w << 24);  // (each <= 64; flags <= 2)
    // ---- one record ahead in registers: its pieces and its clock run
    tu32x4 pr[kTFPer];
    uint32_t pa;
    uint64_t pc;
    auto fetch = [&](uint32_t t) {
      const uint8_t* rec = g.base + lane64(o, t);
      const uint32_t n = (uint32_t)__builtin_amdgcn_readlane(n16, t);
#pragma unroll
      for (uint32_t k = 0; k < kTFPer; ++k) {
        const uint32_t i = lane + k * kW;
        pr[k] = __builtin_nontemporal_load((const tu32x4*)rec + (i < n ? i : n - 1u));
      }
      const uint64_t ct0 = lane64(c0, t);
      const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane(cn, t);
      pa = lane < cnt ? g.cact[ct0 + lane] : 0xFFFFFFFFu;
      pc = lane < cnt ? g.cctr[ct0 + lane] : 0ull;
    };
    uint32_t t = (uint32_t)__builtin_ctzll(pend);
    pend &= pend - 1u;
    fetch(t);
    for (;;) {
      // ---- stage the record, zero the tables (the previous record's LDS
      // reads are done: its copy-out waited for them)
      const uint32_t n = (uint32_t)__builtin_amdgcn_readlane(n16, t);
#pragma unroll
      for (uint32_t k = 0; k < kTFPer; ++k)
        if (lane + k * kW < n) w.stage[lane + k * kW] = pr[k];
      const uint32_t fw = (uint32_t)__builtin_amdgcn_readlane(nf, t);
      const uint32_t nF = fw & 0xFFu, nFD = (fw >> 8) & 0xFFu, nFM = (fw >> 16) & 0xFFu, iflags = fw >> 24;
      if (lane < kTA) w.ct[lane] = 0ull;
      if (nF) {
#pragma unroll
        for (uint32_t k = 0; k < kTFDef * kTA / kW; ++k) (&w.drow[0][0])[lane + k * kW] = 0ull;
        w.names[lane] = 0u;
      }
      const uint32_t ra = pa;
      const uint64_t rc = pc;
      const uint32_t prev = __shfl_up(ra, 1);
      const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane(cn, t);
      // canonical run: actors strictly increasing, counters > 0
      const bool cbad = lane < cnt && (rc == 0ull || (lane > 0u && ra <= prev));
      tf_sync();
      if (lane < cnt && ra < kTA) w.ct[ra] = rc;
      const uint64_t oo = lane64(o, t);
      const uint32_t md = (uint32_t)__builtin_amdgcn_readlane(nmd, t);
      const uint32_t nM = md & 0xFFFFu, nD = md >> 16;
      RecLayout L;
      rec_layout(L, A, nM, nD, nF, nFD, nFM, false);
      const uint8_t* S = (const uint8_t*)w.stage;
      // the deferred clocks into their dense rows; the members they name
      uint32_t fx = 0u, fk = 0u, gk = 0u;
      uint64_t fd = 0ull, fm = 0ull;
      bool dbad = false;
      if (nF) {
        const uint32_t* fdend = (const uint32_t*)(S + L.o_fdend);
        const uint32_t* fmend = (const uint32_t*)(S + L.o_fmend);
        uint32_t pd = 0u, pm = 0u;
        for (uint32_t k = 0; k < nF; ++k) {  // clock of entry e: # run ends <= e
          const uint32_t ed = fdend[k], emk = fmend[k];
          fk += lane >= ed ? 1u : 0u;
          gk += lane >= emk ? 1u : 0u;
          dbad = dbad || ed <= pd || emk <= pm;  // canonical: no empty clock or member set
          pd = ed;
          pm = emk;
        }
        dbad = dbad || pd != nFD || pm != nFM;
        if (lane < nFD) {
          fx = ((const uint32_t*)(S + L.o_fact))[lane];
          fd = ((const uint64_t*)(S + L.o_fctr))[lane];
          dbad = dbad || fx >= A || fk >= nF;
          if (fx < kTA && fk < kTFDef) w.drow[fk][fx] = fd;
        }
        if (lane < nFM) {
          fm = ((const uint64_t*)(S + L.o_fkey))[lane];
          uint32_t lo = 0, len = nM;  // the named member's index (absent: no member to name)
          const uint64_t* key = (const uint64_t*)(S + L.o_key);
          while (len) {
            const uint32_t h = len >> 1;
            if (key[lo + h] < fm) { lo += h + 1u; len -= h + 1u; } else { len = h; }
          }
          if (lo < nM && key[lo] == fm && gk < kTFDef) atomicOr(&w.names[lo], 1u << gk);
        }
      }
      // the next record's loads, in flight while this one is done
      const bool more = pend != 0ull;
      const uint32_t u = more ? (uint32_t)__builtin_ctzll(pend) : t;
      pend &= pend - 1u;
      fetch(u);
      tf_sync();
      // ---- members and dots
      const bool hm = lane < nM, hd = lane < nD;
      const uint64_t km = hm ? ((const uint64_t*)(S + L.o_key))[lane] : 0ull;
      const uint32_t em = hm ? ((const uint32_t*)(S + L.o_mdend))[lane] : 0u;
      const uint32_t xd = hd ? ((const uint32_t*)(S + L.o_dact))[lane] : 0u;
      const uint64_t vd = hd ? ((const uint64_t*)(S + L.o_dctr))[lane] : 0ull;
      const uint64_t tx = lane < A ? ((const uint64_t*)(S + kHdrBytes))[lane] : 0ull;
      const uint64_t cx = lane < A ? w.ct[lane] : 0ull;
      const uint64_t cd = hd ? w.ct[xd & (kTA - 1u)] : 0ull;
      // run ends within [previous end, n_dot], the last one n_dot; strictly
      // increasing with deferred clocks (no empty clock among the inputs
      // then); dot actors < A: else not canonical here (the general kernel)
      const uint32_t emp = __shfl_up(em, 1);
      const bool rbad = (hm && (em > nD || (lane > 0u && (nF ? em <= emp : em < emp)) || (lane == 0u && nF && em == 0u) ||
                                (lane + 1u == nM && em != nD))) ||
                        (hd && xd >= A) || (lane == 0u && nM == 0u && nD != 0u);
      // the member of each dot: run starts marked by ds_permute (a start is
      // the previous member's run end; runs are non-empty here)
      bool dk = false;
      if (nF) {
        const uint32_t h = (uint32_t)__builtin_amdgcn_ds_permute((int)((hm && lane + 1u < nM ? em : 0u) << 2), 1);
        const uint64_t HD = (__ballot(h != 0u) | 1ull) & below_mask(nD);
        const uint32_t mem = (uint32_t)__popcll(HD & lt) + (uint32_t)((HD >> lane) & 1ull) - 1u;
        const uint32_t nm = hd ? w.names[mem & (kW - 1u)] : 0u;
        for (uint32_t b = nm; b; b &= b - 1u) dk = dk || w.drow[__builtin_ctz(b)][xd & (kTA - 1u)] >= vd;
      }
      const uint64_t G = __ballot(hd && vd > cd), NK = __ballot(hd && !dk), F = G & NK;
      const uint32_t s_m = hm ? (lane ? emp : 0u) : 0u;
      const uint64_t run = hm ? below_mask(em) & ~below_mask(s_m) : 0ull;
      const bool kept = (G & run) != 0ull && (NK & run) != 0ull;
      const uint32_t ne = (uint32_t)__popcll(F & below_mask(em));  // kept dots before this run's end
      const uint64_t K = __ballot(kept);
      const uint32_t n_mem = (uint32_t)__popcll(K), n_dot = (uint32_t)__popcll(F);
      const bool empty = __ballot(kept && (F & run) == 0ull) != 0ull;
      // deferred clocks kept: an entry above max(T, c)
      uint32_t KD = 0u;
      uint64_t FE = 0ull, ME = 0ull;
      uint32_t n_fd = 0u, n_fm = 0u;
      if (nF) {
        const uint64_t mx = ((const uint64_t*)(S + kHdrBytes))[fx & (kTA - 1u)] > w.ct[fx & (kTA - 1u)]
                                ? ((const uint64_t*)(S + kHdrBytes))[fx & (kTA - 1u)]
                                : w.ct[fx & (kTA - 1u)];
        const uint64_t AB = __ballot(lane < nFD && fd > mx);
        const uint32_t* fdend = (const uint32_t*)(S + L.o_fdend);
        for (uint32_t k = 0; k < nF; ++k) {
          const uint32_t b0 = k ? fdend[k - 1u] : 0u, b1 = fdend[k];
          KD |= (AB & below_mask(b1) & ~below_mask(b0)) != 0ull ? 1u << k : 0u;
        }
        KD = __builtin_amdgcn_readfirstlane(KD);
        FE = __ballot(lane < nFD && fk < kTFDef && ((KD >> fk) & 1u));
        ME = __ballot(lane < nFM && gk < kTFDef && ((KD >> gk) & 1u));
        n_fd = (uint32_t)__popcll(FE);
        n_fm = (uint32_t)__popcll(ME);
      }
      const uint32_t n_def = (uint32_t)__popcll(KD);
      const bool bad = __ballot(cbad || rbad || dbad) != 0ull;
      RecLayout O;
      rec_layout(O, A, n_mem, n_dot, n_def, n_fd, n_fm, false);
      // the kept clocks' cumulative ends (lane k: clock k)
      uint32_t oe_d = 0u, oe_m = 0u;
      if (nF && lane < nF) {
        oe_d = (uint32_t)__popcll(FE & below_mask(((const uint32_t*)(S + L.o_fdend))[lane]));
        oe_m = (uint32_t)__popcll(ME & below_mask(((const uint32_t*)(S + L.o_fmend))[lane]));
      }
      tf_sync();  // every read of the stage is done: the output is assembled over it
      if (!bad) {
        uint8_t* W = (uint8_t*)w.stage;
        if (lane < A) ((uint64_t*)(W + kHdrBytes))[lane] = tx > cx ? tx : 0ull;
        if (kept) {
          const uint32_t pm = (uint32_t)__popcll(K & lt);
          ((uint64_t*)(W + O.o_key))[pm] = km;
          ((uint32_t*)(W + O.o_mdend))[pm] = ne;
        }
        if ((F >> lane) & 1ull) {
          const uint32_t pd = (uint32_t)__popcll(F & lt);
          ((uint64_t*)(W + O.o_dctr))[pd] = vd;
          ((uint32_t*)(W + O.o_dact))[pd] = xd;
        }
        if ((FE >> lane) & 1ull) {
          const uint32_t q = (uint32_t)__popcll(FE & lt);
          ((uint64_t*)(W + O.o_fctr))[q] = fd;
          ((uint32_t*)(W + O.o_fact))[q] = fx;
        }
        if ((ME >> lane) & 1ull) ((uint64_t*)(W + O.o_fkey))[(uint32_t)__popcll(ME & lt)] = fm;
        if (lane < nF && ((KD >> lane) & 1u)) {
          const uint32_t q = (uint32_t)__popcll(KD & (uint32_t)lt);
          ((uint32_t*)(W + O.o_fdend))[q] = oe_d;
          ((uint32_t*)(W + O.o_fmend))[q] = oe_m;
        }
        if (lane == 0u && O.o_def != O.o_mpad) *(uint32_t*)(W + O.o_mpad) = 0u;
        if (lane >= 1u && lane < 4u && O.o_end + 4u * (lane - 1u) < O.size) *(uint32_t*)(W + O.o_end + 4u * (lane - 1u)) = 0u;
        if (lane < 8u) {
          const uint32_t hv = lane == 0u ? O.size : lane == 1u ? A : lane == 2u ? n_mem : lane == 3u ? n_dot
                              : lane == 4u ? n_def : lane == 5u ? n_fd : lane == 6u ? n_fm
                              : g.flags | (empty ? kEmptyClockFlag : 0u);
          ((uint32_t*)W)[lane] = hv;
        }
        tf_sync();
        const uint32_t n16o = O.size / 16u;  // <= the input's pieces: at most 2 per lane
        const uint32_t i0 = lane < n16o ? lane : n16o - 1u, i1 = lane + kW < n16o ? lane + kW : n16o - 1u;
        const tu32x4 q0 = w.stage[i0], q1 = w.stage[i1];
        __builtin_nontemporal_store(q0, (tu32x4*)(g.out + oo) + i0);
        __builtin_nontemporal_store(q1, (tu32x4*)(g.out + oo) + i1);
      } else if (lane == 0u) {  // the general kernel takes it (and latches the error)
        g.out_off[cbase + t] = oo | kTPend;
        const uint32_t e = atomicAdd(&ctl[0], 1u);
        if (e < list_cap) list[e] = cbase + t;
      }
      (void)iflags;
      tf_sync();  // the copy-out's reads of the stage are done
      if (!more) break;
      t = u;
    }
  }
}

}  // namespace

int launch_orswot_truncate(const crdt_orswot_batch& self, const crdt_clock_csr& clocks, uint32_t A, uint32_t flags,
                           uint8_t* out, uint64_t* out_off, uint64_t out_bytes, int* status, uint32_t* ctl,
                           uint64_t* list, uint32_t list_cap, hipStream_t stream) {
  if (self.n_obj == 0) return CRDT_OK;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // dense batches of <= 32 actors: the fast form first (resident grid, its
  // ticket counter ctl[3] zeroed), then the general form over the records it
  // flagged; other batches: the general form over every record
  const bool fast = (flags & kSparseClock) == 0u && A <= kTA && ctl != nullptr;
  static std::atomic<int> occ[3];
  auto occupancy = [&](int k, const void* fn) {
    int o = occ[k].load(std::memory_order_relaxed);
    if (o == 0) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, kW * kTWaves, 0) != hipSuccess || o < 1) o = 2;
      occ[k].store(o, std::memory_order_relaxed);
    }
    return o;
  };
  const uint64_t want = (self.n_obj + kTWaves - 1) / kTWaves;
  const TruncArgs g{self.base, self.off, (uint64_t)self.bytes, (uint64_t)self.n_obj, clocks.off, clocks.len,
                    clocks.act, clocks.ctr, (uint64_t)clocks.n_entries, A, flags, out, out_off, out_bytes, status};
  if (fast) {
    const uint64_t chunks = (self.n_obj + kW - 1) / kW;
    const uint64_t fwant = (chunks + kTWaves - 1) / kTWaves;
    const uint64_t fcap = (uint64_t)cus * (uint64_t)occupancy(2, (const void*)orswot_truncate_fast_kernel);
    if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;
    hipLaunchKernelGGL(orswot_truncate_fast_kernel, dim3((uint32_t)(fwant < fcap ? fwant : fcap)), dim3(kW * kTWaves),
                       0, stream, g, ctl, list, list_cap);
    if (hipGetLastError() != hipSuccess) return CRDT_EHIP;
  }
  const void* fn = fast ? (const void*)orswot_truncate_kernel<true> : (const void*)orswot_truncate_kernel<false>;
  const uint64_t cap = (uint64_t)cus * (uint64_t)occupancy(fast ? 1 : 0, fn);
  const uint32_t blocks = (uint32_t)(want < cap ? want : cap);
  const uint32_t* flagged = ctl;
  const uint64_t* clist = list;
  void* args[] = {(void*)&g, (void*)&flagged, (void*)&clist, (void*)&list_cap};
  if (hipLaunchKernel(fn, dim3(blocks), dim3(kW * kTWaves), args, 0, stream) != hipSuccess) return CRDT_EHIP;
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
