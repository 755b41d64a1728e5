// Ingest / egest codec between the reference's binary form of an Orswot and
// the canonical record (include/crdts_hip.h). SURVEY.md §8(f) rank 1.
//
// The reference form is `to_binary(&orswot)` = bincode 0.9 of the serde
// derives (src/lib.rs:62-83; struct Orswot src/orswot.rs:26-30, VClock
// src/vclock.rs:54-57): fields in order, maps and sets as a u64 length +
// elements, fixed-width little-endian integers; HashMap / HashSet iteration
// order is arbitrary, BTreeMap order ascending. Actors and members are
// unsigned integers of 1, 2, 4 or 8 bytes, used as the record's actor ids /
// member keys directly (an order-preserving intern).
//
// Ingest canonicalises: members sorted by key, deferred clocks sorted in
// CLOCK ORDER, deferred member sets sorted; it rejects what a record cannot
// hold (zero counters, empty clocks or sets, actors >= n_actors, duplicates,
// out-of-order BTreeMap keys, truncated or trailing bytes).
//
// One wave per object, grid-stride. A blob that fits the wave's LDS window is
// staged there (16-B loads of the aligned span); the walk over its variable-
// length entries is wave-uniform (every lane reads the same bytes), the
// per-member / per-deferred-clock work is lane-parallel.
#include <hip/hip_runtime.h>

#include <atomic>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "sched.h"
#include "record_layout.h"

namespace crdts_hip {
namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr uint32_t kBcWave = 64;
constexpr uint32_t kBcWaves = 4;        // waves per block
constexpr uint32_t kBcStage = 4096;     // LDS window per wave (blob for ingest, blob for egest)
// Ingest scratch of one wave (bytes), for objects of up to MEM members and DEF
// deferred clocks: the walk writes only the first `Walk` bytes. The fast path
// keeps it in LDS (XS: 256 members, 64 deferred clocks); objects past that are
// listed and decoded by the large-object kernel from an HBM scratch (XB).
template <uint32_t MEM, uint32_t DEF, bool GLOBAL>
struct XLay {
  static constexpr uint32_t kMem = MEM, kDef = DEF;
  static constexpr bool kGlobal = GLOBAL;  // scratch in HBM (its hand-offs need vmcnt waits)
  static constexpr uint32_t Pm = 0;                 // u32 member entry position [MEM]
  static constexpr uint32_t Lm = Pm + 4 * MEM;      // u32 member dot count
  static constexpr uint32_t Pd = Lm + 4 * MEM;      // u32 deferred clock position (its length word)
  static constexpr uint32_t Ld = Pd + 4 * DEF;      // u32 deferred clock entries
  static constexpr uint32_t Ps = Ld + 4 * DEF;      // u32 deferred set position (its length word)
  static constexpr uint32_t Ls = Ps + 4 * DEF;      // u32 deferred set size
  static constexpr uint32_t Walk = Ls + 4 * DEF;
  static constexpr uint32_t Rm = Walk;              // u32 member rank
  static constexpr uint32_t Kc = Rm;                // u64 dense top clock scatter (before the ranking)
  static constexpr uint32_t Sm = Rm + 4 * MEM;      // u32 dot counts / offsets in sorted order
  static constexpr uint32_t Sd = Sm + 4 * MEM;      // u32 sorted deferred clock entries -> offsets
  static constexpr uint32_t Ss = Sd + 4 * DEF;      // u32 sorted deferred set sizes -> offsets
  static constexpr uint32_t Rd = Ss + 4 * DEF;      // u32 deferred rank
  static constexpr uint32_t Kk = Rd + 4 * DEF;      // u64 member keys (HBM scratch only: the ranking's operands)
  static constexpr uint32_t Bytes = GLOBAL ? Kk + 8 * MEM : Kk;
  static_assert(8 * MEM <= Sd - Kc, "dense clock scatter fits the rank + offset arrays");
};
using XS = XLay<256, 64, false>;      // 5 888 B of LDS per wave
using XS5 = XLay<128, 32, false>;     // 2 944 B: five 4-wave blocks per CU
using XB = XLay<16384, 1024, true>;   // 409 600 B of HBM per large-object wave
constexpr uint32_t kXWalk = XS::Walk;
constexpr uint32_t kXBytes = XS::Bytes;
constexpr uint32_t kBcBigWaves = 64;      // waves (one per block) of the large-object decode

// Diagnostic phase stamps (ST builds only, variant 301): s_memtime deltas.
struct BcStamps {
  uint64_t acc[8];
  uint64_t last;
};
__device__ __forceinline__ uint64_t bc_now() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
template <bool ST>
__device__ __forceinline__ void bc_mark(BcStamps* st, int k) {
  if (ST) {
    const uint64_t t = bc_now();
    st->acc[k] += t - st->last;
    st->last = t;
  }
}

__device__ __forceinline__ void bc_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// hand-off between the lanes of one wave through the scratch: LDS (the fast
// path) or HBM (the large-object path, whose stores must have landed)
template <class XL>
__device__ __forceinline__ void bc_xsync() {
  if constexpr (XL::kGlobal) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    bc_sync();
  }
}

__device__ __forceinline__ uint32_t bc_uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t bc_uni64(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

__device__ __forceinline__ uint64_t bc_lane64(uint64_t v, uint32_t t) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), t) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, t);
}

__device__ __forceinline__ uint32_t bc_scan_incl(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < kBcWave; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, kBcWave);
    v += lane >= d ? t : 0u;
  }
  return v;
}

// Blob bytes, read as little-endian unsigned integers of w bytes at a blob
// position. LDS window (S = true): b is the window's 16-B aligned base and
// the blob starts at b + d; a field is two aligned u64 reads and a funnel
// shift (the window has >= 16 spare bytes past the blob). Global (S =
// false, blobs too large for the window): byte loads.
template <bool S>
struct Src;
template <>
struct Src<true> {
  static constexpr bool kWindow = true;
  const uint8_t* b;
  uint32_t d;
  __device__ __forceinline__ uint64_t get(uint64_t pos, uint32_t w) const {
    const uint32_t a = d + (uint32_t)pos;
    const uint64_t* q = (const uint64_t*)(b + (a & ~7u));
    const uint32_t sh = 8u * (a & 7u);
    const uint64_t lo = q[0], hi = q[1];
    const uint64_t v = sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
    return w >= 8u ? v : v & ((1ull << (8u * w)) - 1u);
  }
  // the low 32 bits of the field at pos: two aligned u32 reads + v_alignbit
  __device__ __forceinline__ uint32_t lo32(uint32_t pos) const {
    const uint32_t a = d + pos;
    const uint32_t* q = (const uint32_t*)(b + (a & ~3u));
    return __builtin_amdgcn_alignbit(q[1], q[0], (a & 3u) * 8u);
  }
};
template <>
struct Src<false> {
  static constexpr bool kWindow = false;
  const uint8_t* b;
  __device__ __forceinline__ uint64_t get(uint64_t pos, uint32_t w) const {
    uint64_t v = 0;
    for (uint32_t i = 0; i < w; ++i) v |= (uint64_t)b[pos + i] << (8u * i);
    return v;
  }
};
__device__ __forceinline__ void wrw(uint8_t* p, uint64_t pos, uint64_t v, uint32_t w) {
  for (uint32_t i = 0; i < w; ++i) p[pos + i] = (uint8_t)(v >> (8u * i));
}

// lexicographic (actor, counter) order of two bincode clocks, a proper prefix
// first (the record's CLOCK ORDER): -1, 0, 1
template <class SRC>
__device__ __forceinline__ int bc_clock_cmp(const SRC& B, uint64_t pa, uint32_t na, uint64_t pb, uint32_t nb, uint32_t wa) {
  const uint32_t n = na < nb ? na : nb, st = wa + 8u;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t xa = B.get(pa + (uint64_t)st * i, wa), xb = B.get(pb + (uint64_t)st * i, wa);
    if (xa != xb) return xa < xb ? -1 : 1;
    const uint64_t ca = B.get(pa + (uint64_t)st * i + wa, 8), cb = B.get(pb + (uint64_t)st * i + wa, 8);
    if (ca != cb) return ca < cb ? -1 : 1;
  }
  return na == nb ? 0 : (na < nb ? -1 : 1);
}

struct BcWalk {
  uint32_t n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem;
  int err;
};

// Wave-uniform walk over one blob: bounds, counts, entry positions (into X).
template <class XL, class SRC>
__device__ __forceinline__ BcWalk bc_walk(const SRC& B, uint64_t len, uint32_t wa, uint32_t wm, uint32_t A, uint8_t* X,
                          uint32_t lane) {
  BcWalk w{0, 0, 0, 0, 0, 0, 0};
  const uint64_t sa = wa + 8u;
  if (len < 24u || len >= (1ull << 31)) { w.err = CRDT_ENONCANON; return w; }
  const uint64_t nclk = bc_uni64(B.get(0, 8));
  if (nclk > A || nclk * sa > len - 24u) { w.err = CRDT_ENONCANON; return w; }
  w.n_clk = (uint32_t)nclk;
  uint64_t p = 8u + nclk * sa;
  const uint64_t nent = bc_uni64(B.get(p, 8));
  p += 8u;
  if (nent > XL::kMem) { w.err = CRDT_ECAPACITY; return w; }
  w.n_mem = (uint32_t)nent;
  if constexpr (SRC::kWindow) {
    // the chain of entry positions is the only serial part: one LDS round
    // trip and three dependent ALU steps per entry, carried on the window
    // byte offset of each entry's length field (clamped into the blob); every
    // length is then validated lane-parallel
    const uint32_t L32 = (uint32_t)len, step = wm + 8u, lim = B.d + L32, sa32 = (uint32_t)sa;
    uint32_t a = bc_uni(B.d + (uint32_t)p + wm);
    for (uint32_t e0 = 0; e0 < (uint32_t)nent; e0 += kBcWave) {
      // lane j keeps entry e0 + j's length-field offset (a select per step, no stores in the chain)
      uint32_t mine = 0;
      const uint32_t ne = bc_uni((uint32_t)nent - e0 < kBcWave ? (uint32_t)nent - e0 : kBcWave);
      for (uint32_t j = 0; j < ne; ++j) {
        mine = lane == j ? a : mine;
        const uint32_t ac = a < lim ? a : lim;
        const uint32_t* q = (const uint32_t*)(B.b + (ac & ~3u));
        const uint32_t l = __builtin_amdgcn_alignbit(q[1], q[0], ac * 8u);
        a = __builtin_amdgcn_readfirstlane(__umul24(l < 0xFFFFu ? l : 0xFFFFu, sa32) + a + step);
      }
      if (lane < ne) ((uint32_t*)(X + XL::Pm))[e0 + lane] = mine - B.d - wm;
    }
    const uint32_t q = a - B.d - wm;
    bc_xsync<XL>();
    for (uint32_t e = lane; e < (uint32_t)nent; e += kBcWave) {  // the full 64-bit lengths, in parallel
      const uint32_t pe = ((const uint32_t*)(X + XL::Pm))[e];
      const uint64_t l = B.get(pe + wm < L32 ? pe + wm : L32, 8);
      ((uint32_t*)(X + XL::Lm))[e] = (l >> 32) ? 0xFFFFFFFFu : (uint32_t)l;
    }
    bc_xsync<XL>();
    bool bad = false;
    uint32_t nd = 0;
    for (uint32_t e = lane; e < (uint32_t)nent; e += kBcWave) {
      const uint32_t pe = ((const uint32_t*)(X + XL::Pm))[e], l = ((const uint32_t*)(X + XL::Lm))[e];
      bad = bad || l == 0u || l > A || (uint64_t)pe + wm + 8u + (uint64_t)l * sa > len;
      nd += l;
    }
    if (__ballot(bad)) { w.err = CRDT_ENONCANON; return w; }
    for (uint32_t dd = 32; dd >= 1; dd >>= 1) nd += __shfl_xor(nd, dd, kBcWave);
    w.n_dot = bc_uni(nd);
    p = q;
  } else {
    for (uint32_t e = 0; e < (uint32_t)nent; ++e) {
      if (p + wm + 8u > len) { w.err = CRDT_ENONCANON; return w; }
      const uint64_t l = bc_uni64(B.get(p + wm, 8));
      if (l == 0u || l > A || l * sa > len - (p + wm + 8u)) { w.err = CRDT_ENONCANON; return w; }
      if (lane == (e & (kBcWave - 1u))) {
        ((uint32_t*)(X + XL::Pm))[e] = (uint32_t)p;
        ((uint32_t*)(X + XL::Lm))[e] = (uint32_t)l;
      }
      w.n_dot += (uint32_t)l;
      p += wm + 8u + l * sa;
    }
  }
  if (p + 8u > len) { w.err = CRDT_ENONCANON; return w; }
  const uint64_t ndef = bc_uni64(B.get(p, 8));
  p += 8u;
  if (ndef > XL::kDef) { w.err = CRDT_ECAPACITY; return w; }
  w.n_def = (uint32_t)ndef;
  for (uint32_t d = 0; d < (uint32_t)ndef; ++d) {
    if (p + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t lc = bc_uni64(B.get(p, 8));
    if (lc == 0u || lc > A || lc * sa > len - (p + 8u)) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t q = p + 8u + lc * sa;
    if (q + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t ls = bc_uni64(B.get(q, 8));
    if (ls == 0u || ls > len || ls * wm > len - (q + 8u)) { w.err = CRDT_ENONCANON; return w; }
    if (lane == (d & (kBcWave - 1u))) {
      ((uint32_t*)(X + XL::Pd))[d] = (uint32_t)p;
      ((uint32_t*)(X + XL::Ld))[d] = (uint32_t)lc;
      ((uint32_t*)(X + XL::Ps))[d] = (uint32_t)q;
      ((uint32_t*)(X + XL::Ls))[d] = (uint32_t)ls;
    }
    w.n_def_dot += (uint32_t)lc;
    w.n_def_mem += (uint32_t)ls;
    p = q + 8u + ls * wm;
  }
  if (p != len) w.err = CRDT_ENONCANON;  // trailing bytes
  return w;
}

// The deferred part of the walk alone (positions into X), from the deferred
// map's length word at p; counts and bounds were checked by the lane walk.
template <class XL = XS, class SRC>
__device__ __forceinline__ void bc_walk_deferred(const SRC& B, uint64_t p, uint32_t wa, uint32_t wm, uint8_t* X,
                                                 uint32_t lane) {
  const uint64_t sa = wa + 8u;
  const uint32_t ndef = (uint32_t)bc_uni64(B.get(p, 8));
  p += 8u;
  for (uint32_t d = 0; d < ndef; ++d) {
    const uint64_t lc = bc_uni64(B.get(p, 8));
    const uint64_t q = p + 8u + lc * sa;
    const uint64_t ls = bc_uni64(B.get(q, 8));
    if (lane == (d & (kBcWave - 1u))) {
      ((uint32_t*)(X + XL::Pd))[d] = (uint32_t)p;
      ((uint32_t*)(X + XL::Ld))[d] = (uint32_t)lc;
      ((uint32_t*)(X + XL::Ps))[d] = (uint32_t)q;
      ((uint32_t*)(X + XL::Ls))[d] = (uint32_t)ls;
    }
    p = q + 8u + ls * wm;
  }
}

// Exclusive prefix sum, in place, of n u32 at S (256 per round, carried).
template <class XL = XS>
__device__ void bc_scan_excl(uint32_t* S, uint32_t n, uint32_t lane) {
  uint32_t carry = 0;
  for (uint32_t b = 0; b < n; b += 4u * kBcWave) {
    uint32_t v[4], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
      const uint32_t i = b + 4u * lane + k;
      v[k] = i < n ? S[i] : 0u;
      s += v[k];
    }
    const uint32_t incl = bc_scan_incl(s, lane);
    uint32_t run = carry + incl - s;
    carry += __shfl(incl, (int)(kBcWave - 1u), kBcWave);
    bc_xsync<XL>();
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
      const uint32_t i = b + 4u * lane + k;
      if (i < n) S[i] = run;
      run += v[k];
    }
    bc_xsync<XL>();
  }
}

// Decode one blob (already walked) into its canonical record at O. Returns 0
// or a CRDT_E* code (the record is then not valid).
template <bool ST = false, class XL = XS, class SRC>
__device__ __forceinline__ int bc_write_record(const SRC& B, const BcWalk& w, uint32_t wa, uint32_t wm, uint32_t A, bool sparse,
                               uint8_t* X, uint8_t* O, uint32_t lane, BcStamps* st = nullptr,
                               uint32_t moff = 0) {
  RecLayout L;
  rec_layout(L, sparse ? w.n_clk : A, w.n_mem, w.n_dot, w.n_def, w.n_def_dot, w.n_def_mem, sparse);
  const uint64_t sa = wa + 8u;
  bool bad = false;
  // ---- top clock: BTreeMap order = strictly increasing actors. Dense: the
  // counters are scattered into LDS (the member-key area, free until the
  // ranking) and the A slots written once, coalesced
  const bool lds_clk = !sparse && A <= XL::kMem;
  uint64_t* Kc = (uint64_t*)(X + XL::Kc);
  if (lds_clk) {
    for (uint32_t a = lane; a < A; a += kBcWave) Kc[a] = 0ull;
    bc_xsync<XL>();
  } else if (!sparse) {
    for (uint32_t a = lane; a < A; a += kBcWave) ((uint64_t*)(O + L.o_clk))[a] = 0ull;
    __threadfence_block();
  }
  uint64_t carry = 0;  // the actor before this round's first entry
  for (uint32_t k0 = 0; k0 < w.n_clk; k0 += kBcWave) {
    const uint32_t k = k0 + lane;
    const bool on = k < w.n_clk;
    const uint64_t e = 8u + k * sa;
    uint64_t x = 0, c = 0;
    if (on) {
      x = B.get(e, wa);
      c = B.get(e + wa, 8);
    }
    // the previous entry's actor from the lane below (BTreeMap order: strictly increasing)
    uint64_t px = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(x >> 32), 1, kBcWave) << 32) |
                  (uint32_t)__shfl_up((int)(uint32_t)x, 1, kBcWave);
    if (lane == 0u) px = carry;
    carry = bc_lane64(x, kBcWave - 1u);
    if (!on) continue;
    bad = bad || x >= A || c == 0u || (k && px >= x);
    if (x < A) {
      if (sparse) {
        ((uint64_t*)(O + L.o_clk))[k] = c;
        ((uint32_t*)(O + L.o_cact))[k] = (uint32_t)x;
      } else if (lds_clk) {
        Kc[x] = c;
      } else {
        ((uint64_t*)(O + L.o_clk))[x] = c;
      }
    }
  }
  if (lds_clk) {
    bc_xsync<XL>();
    for (uint32_t a = lane; a < A; a += kBcWave) ((uint64_t*)(O + L.o_clk))[a] = Kc[a];
    bc_xsync<XL>();
  }
  if (sparse && lane == 0u && (w.n_clk & 1u)) *(uint32_t*)(O + L.o_cact + 4u * w.n_clk) = 0u;
  bc_mark<ST>(st, 2);
  // ---- members: rank by key (HashMap order is arbitrary), dot offsets in key order
  uint32_t* Pm = (uint32_t*)(X + XL::Pm) + moff;  // (moff: the group walk's slice of the entry arrays)
  uint32_t* Lm = (uint32_t*)(X + XL::Lm) + moff;
  uint32_t* Rm = (uint32_t*)(X + XL::Rm);
  uint32_t* Sm = (uint32_t*)(X + XL::Sm);
  bc_xsync<XL>();
  if (w.n_mem <= kBcWave) {  // every key in one register: broadcast by readlane
    const uint64_t k = lane < w.n_mem ? B.get(Pm[lane], wm) : 0ull;
    uint32_t r = 0;
    for (uint32_t f = 0; f < w.n_mem; ++f) r += bc_lane64(k, f) < k ? 1u : 0u;
    // the ranks (# keys below) sum to n (n - 1) / 2 exactly when no two keys are equal
    uint32_t rs = lane < w.n_mem ? r : 0u;
    for (uint32_t dd = 32; dd >= 1; dd >>= 1) rs += __shfl_xor(rs, dd, kBcWave);
    bad = bad || bc_uni(rs) != w.n_mem * (w.n_mem - 1u) / 2u;
    if (lane < w.n_mem) {
      Rm[lane] = r;
      Sm[r < XL::kMem ? r : 0u] = Lm[lane];
    }
  } else {
    // HBM scratch: the keys are read out of the blob once (u64 array), so the
    // quadratic ranking reads 8-B words, not wm byte loads per comparison
    uint64_t* Kk = (uint64_t*)(X + (XL::kGlobal ? XL::Kk : 0u));
    if constexpr (XL::kGlobal) {
      for (uint32_t e = lane; e < w.n_mem; e += kBcWave) Kk[e] = B.get(Pm[e], wm);
      bc_xsync<XL>();
    }
    for (uint32_t e = lane; e < w.n_mem; e += kBcWave) {
      const uint64_t k = XL::kGlobal ? Kk[e] : B.get(Pm[e], wm);
      uint32_t r = 0, eq = 0;
      for (uint32_t f = 0; f < w.n_mem; ++f) {
        const uint64_t kf = XL::kGlobal ? Kk[f] : B.get(Pm[f], wm);
        r += kf < k ? 1u : 0u;
        eq += kf == k ? 1u : 0u;
      }
      bad = bad || eq != 1u;
      Rm[e] = r;
      Sm[r < XL::kMem ? r : 0u] = Lm[e];
    }
  }
  bc_xsync<XL>();
  bc_scan_excl<XL>(Sm, w.n_mem, lane);
  bc_mark<ST>(st, 3);
  for (uint32_t e = lane; e < w.n_mem; e += kBcWave) {
    const uint32_t r = Rm[e], d0 = Sm[r], l = Lm[e];
    ((uint64_t*)(O + L.o_key))[r] = B.get(Pm[e], wm);
    ((uint32_t*)(O + L.o_mdend))[r] = d0 + l;
    const uint64_t p = Pm[e] + wm + 8u;
    uint64_t prev = 0;
    for (uint32_t i = 0; i < l; ++i) {
      const uint64_t x = B.get(p + i * sa, wa), c = B.get(p + i * sa + wa, 8);
      bad = bad || x >= A || c == 0u || (i && prev >= x);
      prev = x;
      ((uint32_t*)(O + L.o_dact))[d0 + i] = (uint32_t)x;
      ((uint64_t*)(O + L.o_dctr))[d0 + i] = c;
    }
  }
  bc_mark<ST>(st, 4);
  // ---- deferred: clocks sorted in CLOCK ORDER, member sets sorted
  uint32_t* Pd = (uint32_t*)(X + XL::Pd);
  uint32_t* Ld = (uint32_t*)(X + XL::Ld);
  uint32_t* Ps = (uint32_t*)(X + XL::Ps);
  uint32_t* Ls = (uint32_t*)(X + XL::Ls);
  uint32_t* Sd = (uint32_t*)(X + XL::Sd);
  uint32_t* Ss = (uint32_t*)(X + XL::Ss);
  uint32_t* Rd = (uint32_t*)(X + XL::Rd);
  if (w.n_def) {
    for (uint32_t d = lane; d < w.n_def; d += kBcWave) {
      uint32_t r = 0;
      for (uint32_t f = 0; f < w.n_def; ++f) {
        if (f == d) continue;
        const int c = bc_clock_cmp(B, Pd[f] + 8u, Ld[f], Pd[d] + 8u, Ld[d], wa);
        r += c < 0 ? 1u : 0u;
        bad = bad || c == 0;  // structurally equal HashMap keys
      }
      Rd[d] = r;
      Sd[r < XL::kDef ? r : 0u] = Ld[d];
      Ss[r < XL::kDef ? r : 0u] = Ls[d];
    }
    bc_xsync<XL>();
    bc_scan_excl<XL>(Sd, w.n_def, lane);
    bc_scan_excl<XL>(Ss, w.n_def, lane);
    for (uint32_t d = lane; d < w.n_def; d += kBcWave) {
      const uint32_t r = Rd[d], a0 = Sd[r], m0 = Ss[r], lc = Ld[d], ls = Ls[d];
      ((uint32_t*)(O + L.o_fdend))[r] = a0 + lc;
      ((uint32_t*)(O + L.o_fmend))[r] = m0 + ls;
      const uint64_t p = Pd[d] + 8u;
      uint64_t prev = 0;
      for (uint32_t i = 0; i < lc; ++i) {
        const uint64_t x = B.get(p + i * sa, wa), c = B.get(p + i * sa + wa, 8);
        bad = bad || x >= A || c == 0u || (i && prev >= x);
        prev = x;
        ((uint32_t*)(O + L.o_fact))[a0 + i] = (uint32_t)x;
        ((uint64_t*)(O + L.o_fctr))[a0 + i] = c;
      }
      const uint64_t q = Ps[d] + 8u;
      for (uint32_t i = 0; i < ls; ++i) {  // the set's elements by rank (HashSet order is arbitrary)
        const uint64_t m = B.get(q + (uint64_t)i * wm, wm);
        uint32_t rk = 0, eq = 0;
        for (uint32_t j = 0; j < ls; ++j) {
          const uint64_t mj = B.get(q + (uint64_t)j * wm, wm);
          rk += mj < m ? 1u : 0u;
          eq += mj == m ? 1u : 0u;
        }
        bad = bad || eq != 1u;
        ((uint64_t*)(O + L.o_fkey))[m0 + (rk < ls ? rk : 0u)] = m;
      }
    }
  }
  // ---- padding and header
  if (lane == 0u && L.o_def != L.o_mpad) *(uint32_t*)(O + L.o_mpad) = 0u;
  if (lane >= 1u && lane < 4u && L.o_end + 4u * (lane - 1u) < L.size) *(uint32_t*)(O + L.o_end + 4u * (lane - 1u)) = 0u;
  if (lane == 0u) {
    uint32_t* h = (uint32_t*)O;
    h[0] = L.size; h[1] = L.n_clk; h[2] = L.n_mem; h[3] = L.n_dot;
    h[4] = L.n_def; h[5] = L.n_def_dot; h[6] = L.n_def_mem; h[7] = sparse ? kSparseClock : 0u;
  }
  const int rc = __ballot(bad) ? CRDT_ENONCANON : 0;
  bc_mark<ST>(st, 5);
  return rc;
}

template <bool WRITE, bool ST = false, class XL = XS, class SRC>
__device__ __forceinline__ int bc_object(const SRC& B, uint64_t o, uint64_t len, uint32_t wa, uint32_t wm, uint32_t A,
                                         bool sparse, uint8_t* X, uint64_t* sizes, uint8_t* out, const uint64_t* ooff,
                                         uint64_t out_bytes, uint32_t lane, BcStamps* st = nullptr) {
  const BcWalk w = bc_walk<XL>(B, len, wa, wm, A, X, lane);
  bc_mark<ST>(st, 1);
  if (w.err) return w.err;
  const uint64_t size = record_size64(sparse ? w.n_clk : A, w.n_mem, w.n_dot, w.n_def, w.n_def_dot, w.n_def_mem,
                                      sparse);
  if (!WRITE) {
    if (lane == 0u) sizes[o] = size;
    return 0;
  }
  const uint64_t oo = ooff[o];
  if ((oo & 15u) || oo > out_bytes || size > out_bytes - oo) return CRDT_ECAPACITY;
  bc_xsync<XL>();
  return bc_write_record<ST, XL>(B, w, wa, wm, A, sparse, X, out + oo, lane, st);
}

constexpr uint32_t kBcPer = kBcStage / 16u / kBcWave;  // window lines per lane

// The aligned 16-B lines covering one blob, into registers (lines past the
// buffer's end, and the buffer's last partial line, byte by byte).
__device__ __forceinline__ void bc_prefetch(v4u (&r)[kBcPer], const uint8_t* base, uint64_t bytes, uint64_t a0,
                                            uint32_t n16, uint32_t lane) {
#pragma unroll
  for (uint32_t k = 0; k < kBcPer; ++k) {
    const uint32_t idx = lane + k * kBcWave;
    const uint64_t g = a0 + 16ull * idx;
    if (idx < n16) {
      if (g + 16u <= bytes) {
        r[k] = __builtin_nontemporal_load((const v4u*)(base + g));
      } else {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (uint32_t i = 0; i < 16u; ++i)
          if (g + i < bytes) w[i / 4u] |= (uint32_t)base[g + i] << (8u * (i & 3u));
        r[k] = v4u{w[0], w[1], w[2], w[3]};
      }
    }
  }
}

// One wave per 64-object chunk: lane k holds object cbase + k's blob extent;
// the objects are then walked (and, WRITE, decoded) one by one from the LDS
// window while the next windowed blob is in flight in registers.
template <bool WRITE, bool ST = false>
__global__ __launch_bounds__(kBcWave * kBcWaves, WRITE ? 4 : 5) void bincode_ingest_kernel(
    const uint8_t* __restrict__ blobs, uint64_t blob_bytes, const uint64_t* __restrict__ boff,
    const uint64_t* __restrict__ blen, uint64_t n_obj, uint32_t wa, uint32_t wm, uint32_t A, uint32_t flags,
    uint64_t* __restrict__ sizes, uint8_t* __restrict__ out, const uint64_t* __restrict__ ooff, uint64_t out_bytes,
    int* __restrict__ status) {
  __shared__ v4u st_s[kBcWaves][kBcStage / 16];
  __shared__ v4u sx_s[kBcWaves][(WRITE ? kXBytes : kXWalk) / 16];
  const uint32_t lane = threadIdx.x & (kBcWave - 1u), wave = threadIdx.x / kBcWave;
  uint8_t* X = (uint8_t*)sx_s[wave];
  const bool sparse = (flags & kSparseClock) != 0u;
  const uint64_t n_waves = (uint64_t)gridDim.x * kBcWaves;
  const uint64_t wave_id = (uint64_t)blockIdx.x * kBcWaves + wave;
  BcStamps stv{};
  BcStamps* st = ST ? &stv : nullptr;
  if (ST) stv.last = bc_now();
  for (uint64_t cbase = wave_id * kBcWave; cbase < n_obj; cbase += n_waves * kBcWave) {
    const uint64_t obj = cbase + lane;
    const bool valid = obj < n_obj;
    uint64_t off = 0, len = 0;
    if (valid) { off = boff[obj]; len = blen[obj]; }
    const bool inb = valid && off <= blob_bytes && len <= blob_bytes - off;
    if (valid && !inb) {
      atomicCAS(status, 0, CRDT_ENONCANON);
      if (!WRITE) sizes[obj] = 0u;
    }
    const bool win = inb && len + 32u <= kBcStage;
    const uint64_t a0 = off & ~15ull;
    const uint32_t n16 = win ? (uint32_t)((((off + len + 15u) & ~15ull) - a0) / 16u) : 0u;
    const uint64_t wins = __ballot(win);
    uint64_t pend = __ballot(inb);
    v4u pf[kBcPer];
    uint64_t nxt = wins;
    if (nxt) {
      const uint32_t t = (uint32_t)__builtin_ctzll(nxt);
      bc_prefetch(pf, blobs, blob_bytes, bc_lane64(a0, t), __builtin_amdgcn_readlane(n16, t), lane);
    }
    while (pend) {
      const uint32_t t = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      const uint64_t o = cbase + t, ot = bc_lane64(off, t), lt = bc_lane64(len, t);
      int rc;
      if ((wins >> t) & 1ull) {
        bc_sync();  // the previous object's window readers are done
#pragma unroll
        for (uint32_t k = 0; k < kBcPer; ++k) st_s[wave][lane + k * kBcWave] = pf[k];
        bc_sync();
        nxt &= nxt - 1;  // t was the lowest pending windowed object
        if (nxt) {
          const uint32_t u = (uint32_t)__builtin_ctzll(nxt);
          bc_prefetch(pf, blobs, blob_bytes, bc_lane64(a0, u), __builtin_amdgcn_readlane(n16, u), lane);
        }
        const Src<true> B{(const uint8_t*)st_s[wave], (uint32_t)(ot & 15u)};
        bc_mark<ST>(st, 0);
        rc = bc_object<WRITE, ST>(B, o, lt, wa, wm, A, sparse, X, sizes, out, ooff, out_bytes, lane, st);
      } else {
        const Src<false> B{blobs + ot};
        rc = bc_object<WRITE>(B, o, lt, wa, wm, A, sparse, X, sizes, out, ooff, out_bytes, lane);
      }
      if (rc && lane == 0u) {
        atomicCAS(status, 0, rc);
        if (!WRITE) sizes[o] = 0u;
      }
      bc_mark<ST>(st, 6);
    }
  }
  if (ST && lane < 8u) {  // per-wave phase sums -> the debug buffer (sizes slot of the stamp build)
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) v = lane == (uint32_t)q ? stv.acc[q] : v;
    sizes[wave_id * 8u + lane] = v;
  }
}

// ---------------------------------------------------------------- ingest sizes
// The sizes pass needs only the walk's counts, so each LANE walks its own blob
// (64 independent chains per wave instead of one): u64 fields are two aligned
// 8-B loads and a funnel shift (byte loads within 16 B of the buffer's end).
// Same checks, in the same order, as bc_walk.
__device__ __forceinline__ uint64_t lane_get(const uint8_t* base, uint64_t bytes, uint64_t at, uint32_t w) {
  uint64_t v;
  if (at + 16u <= bytes) {
    const uint64_t* q = (const uint64_t*)(base + (at & ~7ull));
    const uint32_t sh = 8u * (uint32_t)(at & 7u);
    const uint64_t lo = q[0], hi = q[1];
    v = sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
  } else {
    v = 0;
    for (uint32_t i = 0; i < 8u && at + i < bytes; ++i) v |= (uint64_t)base[at + i] << (8u * i);
  }
  return w >= 8u ? v : v & ((1ull << (8u * w)) - 1u);
}

struct LaneWalk {
  uint32_t n_clk, n_mem, n_dot, n_def, n_fdot, n_fmem;
  uint64_t p_def;  // position of the deferred map's length word
  int err;
};

// One lane's walk over its own blob. EMIT: every member entry's (position,
// dot count) is also stored as a u64 at emit[e] (bounded by emit_end).
template <bool EMIT>
__device__ __forceinline__ LaneWalk lane_walk(const uint8_t* blobs, uint64_t blob_bytes, uint64_t off, uint64_t len,
                                              uint32_t wa, uint32_t wm, uint32_t A, uint64_t* emit,
                                              const uint8_t* emit_end) {
  LaneWalk w{0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t sa = wa + 8u;
  if (off > blob_bytes || len > blob_bytes - off || len < 24u || len >= (1ull << 31)) {
    w.err = CRDT_ENONCANON;
    return w;
  }
  const uint64_t nclk = lane_get(blobs, blob_bytes, off, 8);
  if (nclk > A || nclk * sa > len - 24u) { w.err = CRDT_ENONCANON; return w; }
  w.n_clk = (uint32_t)nclk;
  uint64_t p = 8u + nclk * sa;
  const uint64_t nent = lane_get(blobs, blob_bytes, off + p, 8);
  p += 8u;
  if (nent > XB::kMem) { w.err = CRDT_ECAPACITY; return w; }
  for (uint64_t e = 0; e < nent; ++e) {
    if (p + wm + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t l = lane_get(blobs, blob_bytes, off + p + wm, 8);
    if (l == 0u || l > A || l * sa > len - (p + wm + 8u)) { w.err = CRDT_ENONCANON; return w; }
    if (EMIT) {
      if ((const uint8_t*)(emit + e + 1) > emit_end) { w.err = CRDT_ECAPACITY; return w; }
      emit[e] = p | (l << 32);
    }
    w.n_dot += (uint32_t)l;
    p += wm + 8u + l * sa;
  }
  w.n_mem = (uint32_t)nent;
  if (p + 8u > len) { w.err = CRDT_ENONCANON; return w; }
  w.p_def = p;
  const uint64_t ndef = lane_get(blobs, blob_bytes, off + p, 8);
  p += 8u;
  if (ndef > XB::kDef) { w.err = CRDT_ECAPACITY; return w; }
  for (uint64_t d = 0; d < ndef; ++d) {
    if (p + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t lc = lane_get(blobs, blob_bytes, off + p, 8);
    if (lc == 0u || lc > A || lc * sa > len - (p + 8u)) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t q = p + 8u + lc * sa;
    if (q + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t ls = lane_get(blobs, blob_bytes, off + q, 8);
    if (ls == 0u || ls > len || ls * wm > len - (q + 8u)) { w.err = CRDT_ENONCANON; return w; }
    w.n_fdot += (uint32_t)lc;
    w.n_fmem += (uint32_t)ls;
    p = q + 8u + ls * wm;
  }
  w.n_def = (uint32_t)ndef;
  if (p != len) w.err = CRDT_ENONCANON;
  return w;
}

__global__ __launch_bounds__(256) void bincode_sizes_lane_kernel(
    const uint8_t* __restrict__ blobs, uint64_t blob_bytes, const uint64_t* __restrict__ boff,
    const uint64_t* __restrict__ blen, uint64_t n_obj, uint32_t wa, uint32_t wm, uint32_t A, uint32_t flags,
    uint64_t* __restrict__ sizes, int* __restrict__ status) {
  const bool sparse = (flags & kSparseClock) != 0u;
  for (uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n_obj; o += (uint64_t)gridDim.x * blockDim.x) {
    const LaneWalk w = lane_walk<false>(blobs, blob_bytes, boff[o], blen[o], wa, wm, A, nullptr, nullptr);
    if (w.err) {
      sizes[o] = 0u;
      atomicCAS(status, 0, w.err);
    } else {
      sizes[o] = record_size64(sparse ? w.n_clk : A, w.n_mem, w.n_dot, w.n_def, w.n_fdot, w.n_fmem, sparse);
    }
  }
}

// The group walk of the read-once decode pass: each lane walks its own blob
// out of the LDS window that holds a group of blobs (bc_walk's checks, in
// lane_walk's order), and with `write` parks every member entry's position
// and dot count at Pm / Lm[base + e]: one entry chain per lane, the group's
// chains in parallel instead of one after another.
__device__ __forceinline__ LaneWalk bc_lane_walk_window(const Src<true>& B, uint64_t len, uint32_t wa, uint32_t wm,
                                                        uint32_t A, uint32_t* Pm, uint32_t* Lm, uint32_t base,
                                                        bool write) {
  LaneWalk w{0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t sa = wa + 8u;
  if (len < 24u || len >= (1ull << 31)) { w.err = CRDT_ENONCANON; return w; }
  const uint64_t nclk = B.get(0, 8);
  if (nclk > A || nclk * sa > len - 24u) { w.err = CRDT_ENONCANON; return w; }
  w.n_clk = (uint32_t)nclk;
  uint64_t p = 8u + nclk * sa;
  const uint64_t nent = B.get(p, 8);
  p += 8u;
  if (nent > XS::kMem) { w.err = CRDT_ECAPACITY; return w; }
  for (uint32_t e = 0; e < (uint32_t)nent; ++e) {
    if (p + wm + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t l = B.get(p + wm, 8);
    if (l == 0u || l > A || l * sa > len - (p + wm + 8u)) { w.err = CRDT_ENONCANON; return w; }
    if (write) {
      Pm[base + e] = (uint32_t)p;
      Lm[base + e] = (uint32_t)l;
    }
    w.n_dot += (uint32_t)l;
    p += wm + 8u + l * sa;
  }
  w.n_mem = (uint32_t)nent;
  if (p + 8u > len) { w.err = CRDT_ENONCANON; return w; }
  w.p_def = p;
  const uint64_t ndef = B.get(p, 8);
  p += 8u;
  if (ndef > XS::kDef) { w.err = CRDT_ECAPACITY; return w; }
  for (uint64_t d = 0; d < ndef; ++d) {
    if (p + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t lc = B.get(p, 8);
    if (lc == 0u || lc > A || lc * sa > len - (p + 8u)) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t q = p + 8u + lc * sa;
    if (q + 8u > len) { w.err = CRDT_ENONCANON; return w; }
    const uint64_t ls = B.get(q, 8);
    if (ls == 0u || ls > len || ls * wm > len - (q + 8u)) { w.err = CRDT_ENONCANON; return w; }
    w.n_fdot += (uint32_t)lc;
    w.n_fmem += (uint32_t)ls;
    p = q + 8u + ls * wm;
  }
  w.n_def = (uint32_t)ndef;
  if (p != len) w.err = CRDT_ENONCANON;
  return w;
}

// One object of the read-once decode pass: the wave-uniform walk (bc_walk)
// and the record writer over the same source; an object past the LDS scratch
// (XL: members or deferred clocks) is listed for the large-object kernel
// (ctl[0]; past the list: CRDT_ECAPACITY).
template <class XL, class SRC>
__device__ __forceinline__ int bc_decode_listed(const SRC& B, uint64_t o, uint64_t len, uint32_t wa, uint32_t wm,
                                                uint32_t A, bool sparse, uint8_t* X, uint8_t* out, uint64_t oo,
                                                uint64_t out_bytes, uint32_t* ctl, uint64_t* list, uint32_t list_cap,
                                                uint32_t lane) {
  const BcWalk w = bc_walk<XL>(B, len, wa, wm, A, X, lane);
  if (w.err == CRDT_ECAPACITY) {
    uint32_t e = 0u;
    if (lane == 0u) {
      e = atomicAdd(&ctl[0], 1u);
      if (e < list_cap) list[e] = o;
    }
    return bc_uni(e) < list_cap ? 0 : CRDT_ECAPACITY;
  }
  if (w.err) return w.err;
  const uint64_t size = record_size64(sparse ? w.n_clk : A, w.n_mem, w.n_dot, w.n_def, w.n_def_dot, w.n_def_mem,
                                      sparse);
  if (size > out_bytes - oo) return CRDT_ECAPACITY;
  bc_xsync<XL>();
  return bc_write_record<false, XL>(B, w, wa, wm, A, sparse, X, out + oo, lane);
}

// Decode pass, one wave per chunk of objects (guided split). Product (LW =
// false): every blob is read from HBM once — its aligned lines prefetched
// into registers while the previous object is decoded, staged in the LDS
// window, walked there by the wave (bc_walk: the entry chain, then every
// length lane-parallel) and decoded from it; an object past the LDS scratch
// is listed for the large-object kernel. Diagnostic (LW = true, variant 305,
// the round-3 product): each lane first walks its own blob of the chunk over
// HBM (as in the sizes pass) and parks every member entry's (position, dot
// count) in its output record's key section; the wave then decodes from the
// window reading those pairs — faster by 4 % on config 3 but every blob is
// read twice and the pairs written and read back (2.3x the algorithmic bytes,
// DESIGN.md §9).
template <bool LW, class XL = XS, int OCC = 4, bool GW = false>
__global__ __launch_bounds__(kBcWave * kBcWaves, OCC) void bincode_decode_kernel(
    const uint8_t* __restrict__ blobs, uint64_t blob_bytes, const uint64_t* __restrict__ boff,
    const uint64_t* __restrict__ blen, uint64_t n_obj, uint32_t wa, uint32_t wm, uint32_t A, uint32_t flags,
    uint8_t* __restrict__ out, const uint64_t* __restrict__ ooff, uint64_t out_bytes, int* __restrict__ status,
    uint32_t* __restrict__ ctl, uint64_t* __restrict__ list, uint32_t list_cap) {
  __shared__ v4u st_s[kBcWaves][kBcStage / 16];
  static_assert(!LW || XL::kMem == XS::kMem, "the lane walk's listing uses XS");
  __shared__ v4u sx_s[kBcWaves][XL::Bytes / 16];
  const uint32_t lane = threadIdx.x & (kBcWave - 1u), wave = threadIdx.x / kBcWave;
  uint8_t* X = (uint8_t*)sx_s[wave];
  const bool sparse = (flags & kSparseClock) != 0u;
  const uint64_t n_waves = (uint64_t)gridDim.x * kBcWaves;
  const uint64_t wave_id = (uint64_t)blockIdx.x * kBcWaves + wave;
  // the guided split (sched.h): 5/8 of the objects in static chunks by wave
  // index, the rest in 20-object atomic tickets (ctl[3])
  GuidedSplit<20, 5> gs(n_obj, wave_id, n_waves);
  uint64_t cbase = 0, cend = 0;
  while (gs.next(cbase, cend, ctl + 3, lane)) {
    const uint64_t obj = cbase + lane;
    const bool valid = obj < cend;
    uint64_t off = 0, len = 0, oo = 0;
    if (valid) { off = boff[obj]; len = blen[obj]; oo = ooff[obj]; }
    LaneWalk lw{0, 0, 0, 0, 0, 0, 0, 0};
    if (!LW) {  // bounds only: each object is walked from its window
      if (valid) {
        if ((oo & 15u) || oo > out_bytes) lw.err = CRDT_ECAPACITY;
        else if (off > blob_bytes || len > blob_bytes - off) lw.err = CRDT_ENONCANON;
        if (lw.err) atomicCAS(status, 0, lw.err);
      }
    } else if (valid) {
      if ((oo & 15u) || oo > out_bytes) {
        lw.err = CRDT_ECAPACITY;
      } else {
        // the key section follows the top clock; a sparse clock's size is the
        // blob's first field (peeked here, re-checked by the walk)
        const uint64_t nclk = (off <= blob_bytes && len >= 8u && len <= blob_bytes - off)
                                  ? lane_get(blobs, blob_bytes, off, 8) : 0u;
        const uint32_t kc = sparse ? (uint32_t)(nclk < A ? nclk : A) : A;
        uint64_t* emit = (uint64_t*)(out + oo + kHdrBytes + clock_bytes(kc, sparse));
        lw = lane_walk<true>(blobs, blob_bytes, off, len, wa, wm, A, emit, out + out_bytes);
      }
      if (!lw.err) {
        const uint64_t sz = record_size64(sparse ? lw.n_clk : A, lw.n_mem, lw.n_dot, lw.n_def, lw.n_fdot, lw.n_fmem,
                                          sparse);
        if (sz > out_bytes - oo) lw.err = CRDT_ECAPACITY;
      }
      if (lw.err) atomicCAS(status, 0, lw.err);
    }
    if (LW) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the parked pairs are visible to the whole wave
    // objects past the LDS scratch (> 256 members or > 64 deferred clocks) are
    // listed for the large-object kernel (ctl[0]); past the list: CRDT_ECAPACITY
    const bool big = LW && valid && !lw.err && (lw.n_mem > XS::kMem || lw.n_def > XS::kDef);
    if (big) {
      const uint32_t e = atomicAdd(&ctl[0], 1u);
      if (e < list_cap) list[e] = obj;
      else atomicCAS(status, 0, CRDT_ECAPACITY);
    }
    const bool ok = valid && !lw.err && !big;
    const bool win = ok && len + 32u <= kBcStage;
    const uint64_t a0 = off & ~15ull;
    const uint32_t n16 = win ? (uint32_t)((((off + len + 15u) & ~15ull) - a0) / 16u) : 0u;
    const uint64_t wins = __ballot(win);
    uint64_t pend = __ballot(ok);
    v4u pf[kBcPer];
    if constexpr (GW && !LW) {
      // GW: groups of windowed objects whose blobs fit one window together;
      // the group's entry chains are walked lane-parallel, then its objects
      // decoded one by one from the window (read once, one chain step per
      // group step instead of per object)
      static_assert(XL::kMem == XS::kMem, "the group walk parks its entries in XS's arrays");
      uint64_t rem = wins;
      auto group_of = [&](uint64_t& g, uint64_t& ga, uint32_t& gn) {
        const uint32_t t = (uint32_t)__builtin_ctzll(rem);
        ga = bc_lane64(a0, t);
        const bool fit = ((rem >> lane) & 1ull) && off >= ga && off + len + 16u <= ga + kBcStage;
        g = __ballot(fit);
        uint32_t e = fit ? (uint32_t)(off + len - ga) : 0u;  // the group's end, < kBcStage past ga
        for (uint32_t dd = 32; dd >= 1; dd >>= 1) e = max(e, (uint32_t)__shfl_xor((int)e, (int)dd, kBcWave));
        gn = (bc_uni(e) + 15u) / 16u;
        rem &= ~g;
      };
      uint64_t gc = 0ull, ga = 0ull;
      uint32_t gn = 0u;
      if (rem) {
        group_of(gc, ga, gn);
        bc_prefetch(pf, blobs, blob_bytes, ga, gn, lane);
      }
      uint32_t* Pm = (uint32_t*)(X + XS::Pm);
      uint32_t* Lm = (uint32_t*)(X + XS::Lm);
      const uint8_t* wb = (const uint8_t*)st_s[wave];
      uint64_t slow = pend & ~wins;  // decoded one by one from HBM after the groups
      while (gc) {
        bc_sync();  // the previous group's window and scratch readers are done
#pragma unroll
        for (uint32_t k = 0; k < kBcPer; ++k) st_s[wave][lane + k * kBcWave] = pf[k];
        bc_sync();
        const uint64_t gcur = gc, acur = ga;
        gc = 0ull;
        if (rem) {  // the next group's span in flight while this one is decoded
          group_of(gc, ga, gn);
          bc_prefetch(pf, blobs, blob_bytes, ga, gn, lane);
        }
        const bool mine = (gcur >> lane) & 1ull;
        const Src<true> Bm{wb, (uint32_t)(off - acur)};
        // the entry counts first (each lane's blob header), their offsets in
        // the entry arrays by a scan, then every chain walked and parked
        uint32_t cnt = 0u;
        if (mine && len >= 24u && len < (1ull << 31)) {
          const uint64_t nclk = Bm.get(0, 8);
          if (nclk <= A && nclk * (wa + 8u) <= len - 24u) {
            const uint64_t ne = Bm.get(8u + nclk * (wa + 8u), 8);
            cnt = ne <= XS::kMem ? (uint32_t)ne : 0u;
          }
        }
        const uint32_t incl = bc_scan_incl(cnt, lane), base = incl - cnt;
        const bool fits = __builtin_amdgcn_readlane(incl, kBcWave - 1u) <= XS::kMem;
        LaneWalk lw2{0, 0, 0, 0, 0, 0, 0, 0};
        if (mine) lw2 = bc_lane_walk_window(Bm, len, wa, wm, A, Pm, Lm, base, fits);
        bc_xsync<XS>();
        if (!fits) {  // (entry arrays overflowed: a malformed or oversized group) one object at a time
          slow |= gcur;
          continue;
        }
        for (uint64_t pend2 = gcur; pend2; pend2 &= pend2 - 1) {
          const uint32_t t = (uint32_t)__builtin_ctzll(pend2);
          const uint64_t o = cbase + t, oot = bc_lane64(oo, t);
          const Src<true> B{wb, (uint32_t)(bc_lane64(off, t) - acur)};
          int rc;
          {
            const int err = __builtin_amdgcn_readlane(lw2.err, t);
            if (err == CRDT_ECAPACITY) {  // past the LDS scratch: the large-object kernel
              uint32_t e = 0u;
              if (lane == 0u) {
                e = atomicAdd(&ctl[0], 1u);
                if (e < list_cap) list[e] = o;
              }
              rc = bc_uni(e) < list_cap ? 0 : CRDT_ECAPACITY;
            } else if (err) {
              rc = err;
            } else {
              BcWalk w;
              w.n_clk = __builtin_amdgcn_readlane(lw2.n_clk, t);
              w.n_mem = __builtin_amdgcn_readlane(lw2.n_mem, t);
              w.n_dot = __builtin_amdgcn_readlane(lw2.n_dot, t);
              w.n_def = __builtin_amdgcn_readlane(lw2.n_def, t);
              w.n_def_dot = __builtin_amdgcn_readlane(lw2.n_fdot, t);
              w.n_def_mem = __builtin_amdgcn_readlane(lw2.n_fmem, t);
              w.err = 0;
              const uint64_t size = record_size64(sparse ? w.n_clk : A, w.n_mem, w.n_dot, w.n_def, w.n_def_dot,
                                                  w.n_def_mem, sparse);
              if (size > out_bytes - oot) {
                rc = CRDT_ECAPACITY;
              } else {
                bc_sync();  // the previous object's readers of the deferred arrays are done
                if (w.n_def) bc_walk_deferred(B, bc_lane64(lw2.p_def, t), wa, wm, X, lane);
                bc_sync();
                rc = bc_write_record<false, XL>(B, w, wa, wm, A, sparse, X, out + oot, lane, nullptr,
                                                __builtin_amdgcn_readlane(base, t));
              }
            }
          }
          if (rc && lane == 0u) atomicCAS(status, 0, rc);
        }
      }
      // the blobs past the window (len + 32 > 4 KB): one by one from HBM
      for (uint64_t pend2 = slow; pend2; pend2 &= pend2 - 1) {
        const uint32_t t = (uint32_t)__builtin_ctzll(pend2);
        const uint64_t o = cbase + t, ot = bc_lane64(off, t), oot = bc_lane64(oo, t), lt = bc_lane64(len, t);
        const Src<false> B{blobs + ot};
        const int rc = bc_decode_listed<XL>(B, o, lt, wa, wm, A, sparse, X, out, oot, out_bytes, ctl, list, list_cap,
                                            lane);
        if (rc && lane == 0u) atomicCAS(status, 0, rc);
      }
      continue;
    }
    uint64_t nxt = wins;
    if (nxt) {
      const uint32_t t = (uint32_t)__builtin_ctzll(nxt);
      bc_prefetch(pf, blobs, blob_bytes, bc_lane64(a0, t), __builtin_amdgcn_readlane(n16, t), lane);
    }
    while (pend && !LW) {  // read once: walk + decode from the window
      const uint32_t t = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      const uint64_t o = cbase + t, ot = bc_lane64(off, t), oot = bc_lane64(oo, t), lt = bc_lane64(len, t);
      int rc;
      if ((wins >> t) & 1ull) {
        bc_sync();  // the previous object's window readers are done
#pragma unroll
        for (uint32_t k = 0; k < kBcPer; ++k) st_s[wave][lane + k * kBcWave] = pf[k];
        bc_sync();
        nxt &= nxt - 1;  // t was the lowest pending windowed object
        if (nxt) {
          const uint32_t u = (uint32_t)__builtin_ctzll(nxt);
          bc_prefetch(pf, blobs, blob_bytes, bc_lane64(a0, u), __builtin_amdgcn_readlane(n16, u), lane);
        }
        const Src<true> B{(const uint8_t*)st_s[wave], (uint32_t)(ot & 15u)};
        rc = bc_decode_listed<XL>(B, o, lt, wa, wm, A, sparse, X, out, oot, out_bytes, ctl, list, list_cap, lane);
      } else {
        const Src<false> B{blobs + ot};
        rc = bc_decode_listed<XL>(B, o, lt, wa, wm, A, sparse, X, out, oot, out_bytes, ctl, list, list_cap, lane);
      }
      if (rc && lane == 0u) atomicCAS(status, 0, rc);
    }
    while (pend && LW) {
      const uint32_t t = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      const uint64_t ot = bc_lane64(off, t), oot = bc_lane64(oo, t);
      BcWalk w;
      w.n_clk = __builtin_amdgcn_readlane(lw.n_clk, t);
      w.n_mem = __builtin_amdgcn_readlane(lw.n_mem, t);
      w.n_dot = __builtin_amdgcn_readlane(lw.n_dot, t);
      w.n_def = __builtin_amdgcn_readlane(lw.n_def, t);
      w.n_def_dot = __builtin_amdgcn_readlane(lw.n_fdot, t);
      w.n_def_mem = __builtin_amdgcn_readlane(lw.n_fmem, t);
      w.err = 0;
      const uint64_t pdef = bc_lane64(lw.p_def, t);
      // the parked (position, dot count) pairs -> the walk's LDS arrays
      const uint64_t* keyarea = (const uint64_t*)(out + oot + kHdrBytes + clock_bytes(sparse ? w.n_clk : A, sparse));
      bc_sync();
      for (uint32_t e = lane; e < w.n_mem; e += kBcWave) {
        const uint64_t pr = keyarea[e];
        ((uint32_t*)(X + XS::Pm))[e] = (uint32_t)pr;
        ((uint32_t*)(X + XS::Lm))[e] = (uint32_t)(pr >> 32);
      }
      int rc;
      if ((wins >> t) & 1ull) {
#pragma unroll
        for (uint32_t k = 0; k < kBcPer; ++k) st_s[wave][lane + k * kBcWave] = pf[k];
        bc_sync();
        nxt &= nxt - 1;  // t was the lowest pending windowed object
        if (nxt) {
          const uint32_t u = (uint32_t)__builtin_ctzll(nxt);
          bc_prefetch(pf, blobs, blob_bytes, bc_lane64(a0, u), __builtin_amdgcn_readlane(n16, u), lane);
        }
        const Src<true> B{(const uint8_t*)st_s[wave], (uint32_t)(ot & 15u)};
        if (w.n_def) bc_walk_deferred(B, pdef, wa, wm, X, lane);
        bc_sync();
        rc = bc_write_record(B, w, wa, wm, A, sparse, X, out + oot, lane);
      } else {
        const Src<false> B{blobs + ot};
        if (w.n_def) bc_walk_deferred(B, pdef, wa, wm, X, lane);
        bc_sync();
        rc = bc_write_record(B, w, wa, wm, A, sparse, X, out + oot, lane);
      }
      if (rc && lane == 0u) atomicCAS(status, 0, rc);
    }
  }
}

// Large objects (listed by the decode pass): one wave per block, the walk and
// the decode from HBM (Src<false>) with the wave's scratch in HBM (XB: up to
// 16 384 members and 1 024 deferred clocks per object).
__global__ __launch_bounds__(kBcWave) void bincode_decode_big_kernel(
    const uint8_t* __restrict__ blobs, const uint64_t* __restrict__ boff, const uint64_t* __restrict__ blen,
    uint32_t wa, uint32_t wm, uint32_t A, uint32_t flags, uint8_t* __restrict__ out, const uint64_t* __restrict__ ooff,
    uint64_t out_bytes, int* __restrict__ status, const uint32_t* __restrict__ ctl, const uint64_t* __restrict__ list,
    uint32_t list_cap, uint8_t* __restrict__ scratch) {
  const uint32_t lane = threadIdx.x;
  uint8_t* X = scratch + (uint64_t)blockIdx.x * XB::Bytes;
  const bool sparse = (flags & kSparseClock) != 0u;
  const uint32_t n = bc_uni(__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t m = n < list_cap ? n : list_cap;
  for (uint32_t e = blockIdx.x; e < m; e += gridDim.x) {
    const uint64_t o = bc_uni64(list[e]);
    const Src<false> B{blobs + boff[o]};
    const int rc = bc_object<true, false, XB>(B, o, blen[o], wa, wm, A, sparse, X, nullptr, out, ooff, out_bytes, lane);
    if (rc && lane == 0u) atomicCAS(status, 0, rc);
  }
}

size_t bincode_big_scratch_bytes() { return (size_t)XB::Bytes * kBcBigWaves; }

// ---------------------------------------------------------------- egest
// Blob writers. LDS window (zeroed first): a field is OR-ed in as the aligned
// u32 pieces it covers (ds_or_b32; neighbouring fields of other lanes may
// share a dword). Global (blobs too large for the window): byte stores.
template <bool S>
struct Dst;
template <>
struct Dst<true> {
  uint8_t* t;
  __device__ __forceinline__ void put(uint64_t pos, uint64_t v, uint32_t w) const {
    const uint32_t a = (uint32_t)pos, sh = 8u * (a & 3u);
    uint32_t* q = (uint32_t*)(t + (a & ~3u));
    if (w == 8u) {
      const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
      atomicOr(q, lo << sh);
      atomicOr(q + 1, sh ? (hi << sh) | (lo >> (32u - sh)) : hi);
      if (sh) atomicOr(q + 2, hi >> (32u - sh));
    } else {
      const uint32_t m = w == 4u ? (uint32_t)v : (uint32_t)v & ((1u << (8u * w)) - 1u);
      atomicOr(q, m << sh);
      if (sh + 8u * w > 32u) atomicOr(q + 1, m >> (32u - sh));
    }
  }
};
template <>
struct Dst<false> {
  uint8_t* t;
  __device__ __forceinline__ void put(uint64_t pos, uint64_t v, uint32_t w) const {
    for (uint32_t i = 0; i < w; ++i) t[pos + i] = (uint8_t)(v >> (8u * i));
  }
};

__device__ __forceinline__ uint64_t bc_blob_len(const uint32_t* h, uint32_t wa, uint32_t wm, uint32_t nnz) {
  const uint64_t sa = wa + 8u;
  return 8u + nnz * sa + 8u + (uint64_t)h[2] * (wm + 8u) + (uint64_t)h[3] * sa + 8u + 16ull * h[4] +
         (uint64_t)h[5] * sa + (uint64_t)h[6] * wm;
}

// nonzero top-clock entries of a record (dense: count of nonzero slots)
__device__ __forceinline__ uint32_t bc_nnz(const uint8_t* r, uint32_t lane) {
  const uint32_t* h = (const uint32_t*)r;
  if (h[7] & kSparseClock) return bc_uni(h[1]);
  const uint32_t n_clk = bc_uni(h[1]);
  uint32_t n = 0;
  for (uint32_t a = lane; a < n_clk; a += kBcWave) n += ((const uint64_t*)(r + kHdrBytes))[a] != 0u ? 1u : 0u;
  for (uint32_t d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d, kBcWave);
  return bc_uni(n);
}

__device__ bool bc_record_ok(const uint8_t* base, uint64_t bytes, uint64_t off, uint32_t A, uint32_t flags) {
  if ((off & 15u) || off + kHdrBytes > bytes) return false;
  const uint32_t* h = (const uint32_t*)(base + off);
  const bool sparse = (flags & kSparseClock) != 0u;
  if (h[7] != flags || (sparse ? h[1] > A : h[1] != A)) return false;
  const uint64_t sz = record_size64(h[1], h[2], h[3], h[4], h[5], h[6], sparse);
  return sz == h[0] && off + sz <= bytes;
}

// to_binary of one record r (header already validated) into T; returns
// true when a value is wider than its field.
template <class DST>
__device__ __forceinline__ bool bc_emit(const uint8_t* r, const DST& T, uint32_t nnz, uint32_t wa, uint32_t wm,
                                        uint64_t amax, uint64_t mmax, uint32_t lane) {
  const uint32_t* h = (const uint32_t*)r;
  const uint32_t n_clk = bc_uni(h[1]), n_mem = bc_uni(h[2]), n_dot = bc_uni(h[3]), n_def = bc_uni(h[4]);
  const bool sparse = (bc_uni(h[7]) & kSparseClock) != 0u;
  RecLayout L;
  rec_layout(L, n_clk, n_mem, n_dot, n_def, bc_uni(h[5]), bc_uni(h[6]), sparse);
  const uint64_t sa = wa + 8u;
  bool bad = false;
  // top clock: BTreeMap<A, u64> = length, then (actor, counter) ascending
  if (lane == 0u) T.put(0, nnz, 8);
  if (sparse) {
    for (uint32_t k = lane; k < n_clk; k += kBcWave) {
      const uint32_t x = ((const uint32_t*)(r + L.o_cact))[k];
      bad = bad || x > amax;
      T.put(8u + k * sa, x, wa);
      T.put(8u + k * sa + wa, ((const uint64_t*)(r + L.o_clk))[k], 8);
    }
  } else {
    uint32_t run = 0;
    for (uint32_t a0 = 0; a0 < n_clk; a0 += kBcWave) {
      const uint32_t a = a0 + lane;
      const uint64_t c = a < n_clk ? ((const uint64_t*)(r + L.o_clk))[a] : 0ull;
      const uint64_t nz = __ballot(c != 0u);
      const uint32_t k = run + __builtin_amdgcn_mbcnt_hi((uint32_t)(nz >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nz, 0u));
      if (c != 0u) {
        bad = bad || a > amax;
        T.put(8u + k * sa, a, wa);
        T.put(8u + k * sa + wa, c, 8);
      }
      run += (uint32_t)__popcll(nz);
    }
  }
  // entries: HashMap<M, VClock<A>> = length, then (member, clock) in key order
  const uint64_t E = 8u + nnz * sa;
  if (lane == 0u) T.put(E, n_mem, 8);
  for (uint32_t m = lane; m < n_mem; m += kBcWave) {
    const uint32_t b0 = m ? ((const uint32_t*)(r + L.o_mdend))[m - 1] : 0u, e = ((const uint32_t*)(r + L.o_mdend))[m];
    const uint64_t p = E + 8u + (uint64_t)m * (wm + 8u) + (uint64_t)b0 * sa;
    const uint64_t key = ((const uint64_t*)(r + L.o_key))[m];
    bad = bad || key > mmax;
    T.put(p, key, wm);
    T.put(p + wm, e - b0, 8);
    for (uint32_t i = b0; i < e; ++i) {
      const uint32_t x = ((const uint32_t*)(r + L.o_dact))[i];
      bad = bad || x > amax;
      T.put(p + wm + 8u + (i - b0) * sa, x, wa);
      T.put(p + wm + 8u + (i - b0) * sa + wa, ((const uint64_t*)(r + L.o_dctr))[i], 8);
    }
  }
  // deferred: HashMap<VClock<A>, HashSet<M>> = length, then (clock, set) in clock order
  const uint64_t F = E + 8u + (uint64_t)n_mem * (wm + 8u) + (uint64_t)n_dot * sa;
  if (lane == 0u) T.put(F, n_def, 8);
  for (uint32_t d = lane; d < n_def; d += kBcWave) {
    const uint32_t b0 = d ? ((const uint32_t*)(r + L.o_fdend))[d - 1] : 0u, e = ((const uint32_t*)(r + L.o_fdend))[d];
    const uint32_t ms = d ? ((const uint32_t*)(r + L.o_fmend))[d - 1] : 0u, me = ((const uint32_t*)(r + L.o_fmend))[d];
    const uint64_t p = F + 8u + 16ull * d + (uint64_t)b0 * sa + (uint64_t)ms * wm;
    T.put(p, e - b0, 8);
    for (uint32_t i = b0; i < e; ++i) {
      const uint32_t x = ((const uint32_t*)(r + L.o_fact))[i];
      bad = bad || x > amax;
      T.put(p + 8u + (i - b0) * sa, x, wa);
      T.put(p + 8u + (i - b0) * sa + wa, ((const uint64_t*)(r + L.o_fctr))[i], 8);
    }
    const uint64_t q = p + 8u + (uint64_t)(e - b0) * sa;
    T.put(q, me - ms, 8);
    for (uint32_t j = ms; j < me; ++j) {
      const uint64_t key = ((const uint64_t*)(r + L.o_fkey))[j];
      bad = bad || key > mmax;
      T.put(q + 8u + (uint64_t)(j - ms) * wm, key, wm);
    }
  }
  return __ballot(bad) != 0ull;
}

// One wave per 64-record chunk. Sizes pass: blob length from the header and
// the dense clock. Write pass: each record is prefetched into registers,
// staged in an LDS window, its blob assembled in a second (zeroed) window
// and copied out with 16-B stores; records or blobs larger than a window go
// straight from / to HBM.
template <bool WRITE>
__global__ __launch_bounds__(kBcWave * kBcWaves, WRITE ? 4 : 8) void bincode_egest_kernel(
    const uint8_t* __restrict__ rb, uint64_t rbytes, const uint64_t* __restrict__ roff, uint64_t n_obj, uint32_t A,
    uint32_t flags, uint32_t wa, uint32_t wm, uint64_t* __restrict__ sizes, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ ooff, uint64_t out_bytes, int* __restrict__ status, uint32_t* __restrict__ ctl) {
  __shared__ v4u rs_s[kBcWaves][WRITE ? kBcStage / 16 : 1];
  __shared__ v4u ts_s[kBcWaves][WRITE ? kBcStage / 16 : 1];
  const uint32_t lane = threadIdx.x & (kBcWave - 1u), wave = threadIdx.x / kBcWave;
  const uint64_t amax = wa >= 8u ? ~0ull : (1ull << (8u * wa)) - 1u, mmax = wm >= 8u ? ~0ull : (1ull << (8u * wm)) - 1u;
  const uint64_t n_waves = (uint64_t)gridDim.x * kBcWaves;
  const uint64_t wave_id = (uint64_t)blockIdx.x * kBcWaves + wave;
  // static rounds of 64-object chunks by wave index (the guided split measured
  // slower here: 0.73 -> 0.67 G objects/s)
  for (uint64_t cbase = wave_id * kBcWave; cbase < n_obj; cbase += n_waves * kBcWave) {
    const uint64_t obj = cbase + lane;
    const bool valid = obj < n_obj;
    const uint64_t ro = valid ? roff[obj] : 0ull;
    const bool ok = valid && bc_record_ok(rb, rbytes, ro, A, flags);
    if (valid && !ok) {
      atomicCAS(status, 0, CRDT_ENONCANON);
      if (!WRITE) sizes[obj] = 0u;
    }
    const uint32_t rsz = ok ? ((const uint32_t*)(rb + ro))[0] : 0u;
    uint64_t pend = __ballot(ok);
    if (!WRITE) {
      while (pend) {
        const uint32_t t = (uint32_t)__builtin_ctzll(pend);
        pend &= pend - 1;
        const uint8_t* r = rb + bc_lane64(ro, t);
        const uint32_t nnz = bc_nnz(r, lane);
        if (lane == 0u) sizes[cbase + t] = bc_blob_len((const uint32_t*)r, wa, wm, nnz);
      }
      continue;
    }
    const bool win = ok && rsz <= kBcStage;
    const uint64_t wins = __ballot(win);
    v4u pf[kBcPer];
    uint64_t nxt = wins;
    if (nxt) {
      const uint32_t t = (uint32_t)__builtin_ctzll(nxt);
      bc_prefetch(pf, rb, rbytes, bc_lane64(ro, t), __builtin_amdgcn_readlane(rsz, t) / 16u, lane);
    }
    bool bad = (uint64_t)(A - 1u) > amax;
    while (pend) {
      const uint32_t t = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      const uint64_t o = cbase + t, oo = ooff[o];
      if ((wins >> t) & 1ull) {
        bc_sync();  // the previous object's window readers are done
#pragma unroll
        for (uint32_t k = 0; k < kBcPer; ++k) rs_s[wave][lane + k * kBcWave] = pf[k];
        bc_sync();
        nxt &= nxt - 1;
        if (nxt) {
          const uint32_t u = (uint32_t)__builtin_ctzll(nxt);
          bc_prefetch(pf, rb, rbytes, bc_lane64(ro, u), __builtin_amdgcn_readlane(rsz, u) / 16u, lane);
        }
        const uint8_t* r = (const uint8_t*)rs_s[wave];
        const uint32_t nnz = bc_nnz(r, lane);
        const uint64_t len = bc_blob_len((const uint32_t*)r, wa, wm, nnz), padded = (len + 15u) & ~15ull;
        if ((oo & 15u) || oo > out_bytes || padded > out_bytes - oo) {
          if (lane == 0u) atomicCAS(status, 0, CRDT_ECAPACITY);
          continue;
        }
        if (padded <= kBcStage) {
          for (uint32_t k = lane; k < (uint32_t)(padded / 16u); k += kBcWave) ts_s[wave][k] = v4u{0u, 0u, 0u, 0u};
          bc_sync();
          bad = bc_emit(r, Dst<true>{(uint8_t*)ts_s[wave]}, nnz, wa, wm, amax, mmax, lane) || bad;
          bc_sync();
          for (uint32_t k = lane; k < (uint32_t)(padded / 16u); k += kBcWave)
            __builtin_nontemporal_store(ts_s[wave][k], (v4u*)(out + oo) + k);
        } else {
          for (uint64_t k = len + lane; k < padded; k += kBcWave) out[oo + k] = 0u;
          bad = bc_emit(r, Dst<false>{out + oo}, nnz, wa, wm, amax, mmax, lane) || bad;
        }
      } else {
        const uint8_t* r = rb + bc_lane64(ro, t);
        const uint32_t nnz = bc_nnz(r, lane);
        const uint64_t len = bc_blob_len((const uint32_t*)r, wa, wm, nnz), padded = (len + 15u) & ~15ull;
        if ((oo & 15u) || oo > out_bytes || padded > out_bytes - oo) {
          if (lane == 0u) atomicCAS(status, 0, CRDT_ECAPACITY);
          continue;
        }
        for (uint64_t k = len + lane; k < padded; k += kBcWave) out[oo + k] = 0u;
        bad = bc_emit(r, Dst<false>{out + oo}, nnz, wa, wm, amax, mmax, lane) || bad;
      }
    }
    if (bad && lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);  // a value wider than its field
  }
}

// A resident grid for the guided split (every wave's static chunks start at
// once): the kernel's occupancy in blocks per CU, cached per kernel.
uint32_t bc_resident_blocks(uint64_t n_obj, const void* fn, std::atomic<int>& occ_cache) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int occ = occ_cache.load(std::memory_order_relaxed);
  if (occ == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kBcWave * kBcWaves, 0) != hipSuccess || occ < 1)
      occ = 2;
    occ_cache.store(occ, std::memory_order_relaxed);
  }
  const uint64_t want = (n_obj + kBcWave * kBcWaves - 1) / (kBcWave * kBcWaves), cap = (uint64_t)cus * occ;
  return (uint32_t)(want < cap ? want : cap);
}

uint32_t bc_blocks(uint64_t n_obj) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t want = (n_obj + kBcWaves - 1) / kBcWaves, cap = (uint64_t)cus * 8u;
  return (uint32_t)(want < cap ? want : cap);
}

// Record placement without reading the blobs: a bound on the record size of
// blob i from its length alone (crdt_orswot_bincode_record_bounds). Against
// the blob's bytes (u64 lengths before the clock, entries and deferred maps;
// wa / wm bytes per actor / member; 8 per counter), every record section is
// at most c times the blob bytes it comes from, c = max(12 / (wa + 8),
// 12 / (wm + 8), 8 / wm): a member (12 B: key + run end) vs wm + 8, a dot
// (12 B) vs wa + 8, a deferred clock's two ends (8 B) vs its 16 B of
// lengths, a deferred member (8 B) vs wm, a sparse top-clock entry (12 B) vs
// wa + 8. The header, a dense clock and the paddings add 48 + 8 A at most.
__device__ __forceinline__ uint64_t bc_record_bound(uint64_t L, uint32_t wa, uint32_t wm, uint32_t A, bool sparse) {
  const uint64_t m1 = (12u * L + wa + 7u) / (wa + 8u), m2 = (12u * L + wm + 7u) / (wm + 8u),
                 m3 = (8u * L + wm - 1u) / wm;
  uint64_t c = m1 > m2 ? m1 : m2;
  c = c > m3 ? c : m3;
  return (48u + (sparse ? 0ull : 8ull * A) + c + 15u) & ~15ull;
}

__global__ __launch_bounds__(256) void bincode_bounds_kernel(const uint64_t* __restrict__ blen, uint64_t n_obj,
                                                             uint32_t wa, uint32_t wm, uint32_t A, uint32_t flags,
                                                             uint64_t* __restrict__ bounds) {
  const bool sparse = (flags & kSparseClock) != 0u;
  for (uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n_obj; o += (uint64_t)gridDim.x * blockDim.x)
    bounds[o] = bc_record_bound(blen[o], wa, wm, A, sparse);
}

}  // namespace

int launch_bincode_bounds(const uint64_t* blen, uint64_t n_obj, uint32_t wa, uint32_t wm, uint32_t A,
                          uint32_t flags, uint64_t* bounds, hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  const uint64_t want = (n_obj + 255u) / 256u;
  const uint32_t blocks = (uint32_t)(want < 4096u ? want : 4096u);
  hipLaunchKernelGGL(bincode_bounds_kernel, dim3(blocks), dim3(256), 0, stream, blen, n_obj, wa, wm, A, flags, bounds);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

size_t launch_bincode_big_scratch_bytes() { return bincode_big_scratch_bytes(); }

int launch_bincode_ingest(const uint8_t* blobs, uint64_t blob_bytes, const uint64_t* boff, const uint64_t* blen,
                          uint64_t n_obj, uint32_t wa, uint32_t wm, uint32_t A, uint32_t flags, uint64_t* sizes,
                          uint8_t* out, const uint64_t* ooff, uint64_t out_bytes, int* status, uint32_t* ctl,
                          hipStream_t stream, uint64_t* dbg, uint64_t* list, uint32_t list_cap, uint8_t* big_scratch,
                          int walk) {
  if (n_obj == 0) return CRDT_OK;
  const uint32_t blocks = bc_blocks(n_obj);
  if (dbg && !sizes) {  // diagnostic: decode pass with phase stamps into dbg (8 u64 per wave)
    hipLaunchKernelGGL((bincode_ingest_kernel<true, true>), dim3(blocks), dim3(kBcWave * kBcWaves), 0, stream, blobs,
                       blob_bytes, boff, blen, n_obj, wa, wm, A, flags, dbg, out, ooff, out_bytes, status);
    return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
  }
  if (sizes) {  // one lane per blob
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t want = (n_obj + 255u) / 256u, cap = (uint64_t)cus * 8u;
    hipLaunchKernelGGL(bincode_sizes_lane_kernel, dim3((uint32_t)(want < cap ? want : cap)), dim3(256), 0, stream,
                       blobs, blob_bytes, boff, blen, n_obj, wa, wm, A, flags, sizes, status);
  } else {
    if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;  // ctl[3]: tickets
    static std::atomic<int> occ_d{0}, occ_r{0}, occ_5{0}, occ_g{0};
    if (!list || !big_scratch) return CRDT_EINVAL;
    if (walk == 1) {
#ifdef CRDT_DIAG
      const uint32_t rblocks = bc_resident_blocks(n_obj, (const void*)bincode_decode_kernel<true>, occ_d);
      hipLaunchKernelGGL(bincode_decode_kernel<true>, dim3(rblocks), dim3(kBcWave * kBcWaves), 0, stream, blobs,
                         blob_bytes, boff, blen, n_obj, wa, wm, A, flags, out, ooff, out_bytes, status, ctl, list,
                         list_cap);
#else
      (void)occ_d;
      return CRDT_EINVAL;
#endif
    } else if (walk == 3) {
#ifdef CRDT_DIAG
      // the per-object read-once walk (the r04 product before the group walk)
      const uint32_t rblocks = bc_resident_blocks(n_obj, (const void*)bincode_decode_kernel<false>, occ_r);
      hipLaunchKernelGGL(bincode_decode_kernel<false>, dim3(rblocks), dim3(kBcWave * kBcWaves), 0, stream, blobs,
                         blob_bytes, boff, blen, n_obj, wa, wm, A, flags, out, ooff, out_bytes, status, ctl, list,
                         list_cap);
#else
      (void)occ_r;
      return CRDT_EINVAL;
#endif
    } else if (walk == 2) {
#ifdef CRDT_DIAG
      const uint32_t rblocks = bc_resident_blocks(n_obj, (const void*)bincode_decode_kernel<false, XS5, 5>, occ_5);
      hipLaunchKernelGGL((bincode_decode_kernel<false, XS5, 5>), dim3(rblocks), dim3(kBcWave * kBcWaves), 0, stream,
                         blobs, blob_bytes, boff, blen, n_obj, wa, wm, A, flags, out, ooff, out_bytes, status, ctl,
                         list, list_cap);
#else
      (void)occ_5;
      return CRDT_EINVAL;
#endif
    } else {  // product: the read-once group walk
      const uint32_t rblocks = bc_resident_blocks(n_obj, (const void*)bincode_decode_kernel<false, XS, 4, true>, occ_g);
      hipLaunchKernelGGL((bincode_decode_kernel<false, XS, 4, true>), dim3(rblocks), dim3(kBcWave * kBcWaves), 0,
                         stream, blobs, blob_bytes, boff, blen, n_obj, wa, wm, A, flags, out, ooff, out_bytes, status,
                         ctl, list, list_cap);
    }
    hipLaunchKernelGGL(bincode_decode_big_kernel, dim3(kBcBigWaves), dim3(kBcWave), 0, stream, blobs, boff, blen, wa,
                       wm, A, flags, out, ooff, out_bytes, status, ctl, list, list_cap, big_scratch);
  }
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

int launch_bincode_egest(const uint8_t* rb, uint64_t rbytes, const uint64_t* roff, uint64_t n_obj, uint32_t A,
                         uint32_t flags, uint32_t wa, uint32_t wm, uint64_t* sizes, uint8_t* out,
                         const uint64_t* ooff, uint64_t out_bytes, int* status, uint32_t* ctl, hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  (void)ctl;
  const uint32_t blocks = bc_blocks(n_obj);
  if (sizes) {
    hipLaunchKernelGGL(bincode_egest_kernel<false>, dim3(blocks), dim3(kBcWave * kBcWaves), 0, stream, rb, rbytes,
                       roff, n_obj, A, flags, wa, wm, sizes, out, ooff, out_bytes, status, ctl);
  } else {
    hipLaunchKernelGGL(bincode_egest_kernel<true>, dim3(blocks), dim3(kBcWave * kBcWaves), 0, stream, rb, rbytes,
                       roff, n_obj, A, flags, wa, wm, sizes, out, ooff, out_bytes, status, ctl);
  }
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
