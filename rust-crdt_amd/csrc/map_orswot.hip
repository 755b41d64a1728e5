// Map<u64, Orswot<u64, A>, A>::merge, batched (SURVEY.md §8(f) rank 3 as written).
//
// Reference: Map::merge (src/map.rs:192-269) — per key the entry clocks are
// reconciled against both map clocks (self-only :198-211, both :213-240,
// other-only :244-253); a key in both maps merges its nested sets
// (Orswot::merge, src/orswot.rs:87-157) and every kept value is truncated by
// the clock of the actors that removed the entry (Orswot::truncate,
// src/orswot.rs:159-172: merge with an empty set carrying that clock, then
// subtract it from the top clock and from every member clock). Other's
// deferred removes are re-deferred against self's pre-merge clock (apply_rm,
// :336-350: its entry edits land on the entries the merge then replaces), the
// clocks merge, and apply_deferred (:325-333) runs every deferred clock over
// its keys: the entry clock loses the clock and, if still non-empty, its set
// is truncated by it. Unlike the MVReg map (map.hip), a key named by several
// deferred clocks is truncated by each in turn, in CLOCK ORDER (the reference
// iterates a HashMap there; DESIGN.md §5e shows the order can matter).
//
// One wave per map pair; lane = actor slot, NS slots per lane (NS = 1 for
// n_actors <= 64, 2 for <= 128: lane l holds actors l and l + 64), so every
// VClock operation on dense rows is NS lane-parallel ops plus a ballot. The nested
// set being built lives in an LDS workspace (member keys + member clock rows
// + deferred clocks + their member sets); a key's two nested sets are staged
// into it by wide loads (one round trip per side), the merge writes a third;
// the object's map deferred sets are staged once per object when they fit
// kMoStageMax. Keys, members and deferred entries are then
// walked by wave-uniform loops over LDS, not over HBM round trips.
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "map_rows.h"
#include "sched.h"

namespace crdts_hip {
namespace {

constexpr uint32_t kMoW = 64;
constexpr uint32_t kMoLdsMax = 65536;  // workspace limit per wave
constexpr uint32_t kMoStageMax = 16384;  // map deferred staging area limit per wave

__device__ __forceinline__ void mo_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | (uint64_t)uni((uint32_t)v);
}
using namespace maprow;  // Row<NS> and the VClock ops on it (map_rows.h)
__device__ __forceinline__ bool set_has(const uint64_t* set, uint32_t n, uint64_t key, uint32_t lane) {
  bool f = false;
  for (uint32_t j = lane; j < n; j += kMoW) f = f || set[j] == key;
  return __ballot(f) != 0ull;
}

// dst[e] = at(e) for e < n, all lanes: 16-B non-temporal stores when dst is
// 16-B aligned and n even, 8-B stores otherwise.
typedef uint64_t mo_u64x2 __attribute__((ext_vector_type(2)));
template <class F>
__device__ __forceinline__ void fill64(uint64_t* dst, uint64_t n, uint32_t lane, F at) {
  if ((((uintptr_t)dst) & 15u) == 0u && (n & 1u) == 0u) {
    for (uint64_t p = lane; p < n / 2u; p += kMoW) {
      const mo_u64x2 v = {at(2u * p), at(2u * p + 1u)};
      __builtin_nontemporal_store(v, (mo_u64x2*)(dst + 2u * p));
    }
  } else {
    for (uint64_t e = lane; e < n; e += kMoW) dst[e] = at(e);
  }
}

// A nested Orswot under construction (LDS). The top clock is a register
// (lane = actor) held by the caller.
struct Ws {
  uint64_t* key;   // [MW] members, ascending
  uint64_t* row;   // [MW][A] member clocks
  uint64_t* dclk;  // [DW][A] deferred clocks, CLOCK ORDER
  uint32_t* dn;    // [DW] set sizes
  uint64_t* dset;  // [DW][sw] member sets, ascending
  uint32_t nm, nd, sw;
};
struct Caps {
  uint32_t MW, DW, SW, A;
};

// Load key slot ki of a slab's nested set into W.
// Key slot ki of a slab's nested set into W: its two counts (ws_counts, from
// the key walk's registers), then every array (ws_copy: each load
// independent of the others' results — the deferred sets copied
// capacity-strided, their sizes by one lane each — so both sides' slots cost
// one round trip), then the caller's mo_sync.
__device__ __forceinline__ void ws_counts(Ws& W, const crdt_map_orswot_slab& X, uint64_t ki, uint32_t k, uint32_t vm,
                                          uint32_t vd) {
  // key k's counts: lane k of the registers the key walk loaded (k < 64)
  W.nm = k < kMoW ? (uint32_t)__builtin_amdgcn_readlane(vm, k) : uni(X.vn_mem[ki]);
  W.nd = k < kMoW ? (uint32_t)__builtin_amdgcn_readlane(vd, k) : uni(X.vn_def[ki]);
}
__device__ void ws_copy(Ws& W, const crdt_map_orswot_slab& X, uint64_t ki, const Caps& c, uint32_t lane) {
  for (uint32_t j = lane; j < W.nm; j += kMoW) W.key[j] = X.vmem[ki * X.mcap + j];
  for (uint32_t e = lane; e < W.nm * c.A; e += kMoW) W.row[e] = X.vmclock[ki * X.mcap * c.A + e];
  for (uint32_t e = lane; e < W.nd * c.A; e += kMoW) W.dclk[e] = X.vdclock[ki * X.vdcap * c.A + e];
  for (uint32_t d = lane; d < W.nd; d += kMoW) W.dn[d] = X.vdset_n[ki * X.vdcap + d];
  const uint32_t vs = X.vscap;
  for (uint32_t e = lane; e < W.nd * vs; e += kMoW) {  // capacity-strided: no wait for the sizes
    const uint32_t d = e / vs;
    W.dset[d * W.sw + (e - d * vs)] = X.vdset[ki * X.vdcap * vs + e];
  }
}

// Orswot::apply_deferred (src/orswot.rs:235-243) on W under top clock `clk`,
// after the members flagged in mdead are dropped: every deferred clock is
// subtracted from the members of its set (a member left empty is dropped),
// and kept only if `clk` does not cover it. Then both lists are compacted.
template <int NS>
__device__ void ws_apply_deferred(Ws& W, Row<NS> clk, uint32_t* mdead, uint32_t* ddead, const Caps& c,
                                  uint32_t lane) {
  for (uint32_t d = 0; d < W.nd; ++d) {
    const Row<NS> D = ldrow<NS>(W.dclk + d * c.A, c.A, lane);
    const uint32_t n = uni(W.dn[d]);
    for (uint32_t j = 0; j < n; ++j) {
      const uint64_t m = uni64(W.dset[d * W.sw + j]);
      uint32_t lo = 0, hi = W.nm;  // binary search over the (sorted) members
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (uni64(W.key[mid]) < m) lo = mid + 1u;
        else hi = mid;
      }
      if (lo >= W.nm || uni64(W.key[lo]) != m || uni(mdead[lo])) continue;
      const Row<NS> r = vsub(ldrow<NS>(W.row + lo * c.A, c.A, lane), D);
      strow(W.row + lo * c.A, r, c.A, lane);
      const bool gone = !vany(r);
      mo_sync();
      if (gone && lane == 0u) mdead[lo] = 1u;
      mo_sync();
    }
    const bool drop = vle(D, clk);
    if (lane == 0u) ddead[d] = drop ? 1u : 0u;
  }
  mo_sync();
  // compaction, in place (destination <= source)
  uint32_t k = 0;
  for (uint32_t j = 0; j < W.nm; ++j) {
    if (uni(mdead[j])) continue;
    if (k != j) {
      const uint64_t key = W.key[j];
      const Row<NS> r = ldrow<NS>(W.row + j * c.A, c.A, lane);
      mo_sync();
      if (lane == 0u) W.key[k] = key;
      strow(W.row + k * c.A, r, c.A, lane);
      mo_sync();
    }
    ++k;
  }
  W.nm = k;
  k = 0;
  for (uint32_t d = 0; d < W.nd; ++d) {
    if (uni(ddead[d])) continue;
    if (k != d) {
      const Row<NS> D = ldrow<NS>(W.dclk + d * c.A, c.A, lane);
      const uint32_t n = uni(W.dn[d]);
      mo_sync();
      strow(W.dclk + k * c.A, D, c.A, lane);
      if (lane == 0u) W.dn[k] = n;
      for (uint32_t j = lane; j < n; j += kMoW) W.dset[k * W.sw + j] = W.dset[d * W.sw + j];  // (rows k < d)
      mo_sync();
    }
    ++k;
  }
  W.nd = k;
  for (uint32_t j = lane; j < c.MW; j += kMoW) mdead[j] = 0u;
  for (uint32_t j = lane; j < c.DW; j += kMoW) ddead[j] = 0u;
  mo_sync();
}

// Orswot::merge (src/orswot.rs:87-157): Wn = Wc.merge(&Wo), Wo's top clock
// oclk. `sclk` (Wc's top clock) becomes the merged clock.
template <int NS>
__device__ void ws_merge(const Ws& Wc, const Ws& Wo, Ws& Wn, Row<NS>& sclk, Row<NS> oclk, uint32_t* mdead,
                         uint32_t* ddead, const Caps& c, uint32_t lane) {
  const uint32_t no = Wo.nm;
  uint32_t a = 0, b = 0, n = 0;
  while (a < Wc.nm || b < no) {
    const uint64_t ka = a < Wc.nm ? uni64(Wc.key[a]) : ~0ull;
    const uint64_t kb = b < no ? uni64(Wo.key[b]) : ~0ull;
    const bool hs = a < Wc.nm && (b >= no || ka <= kb), ho = b < no && (a >= Wc.nm || kb <= ka);
    const Row<NS> r = hs ? ldrow<NS>(Wc.row + a * c.A, c.A, lane) : zrow<NS>();
    const Row<NS> orow = ho ? ldrow<NS>(Wo.row + b * c.A, c.A, lane) : zrow<NS>();
    Row<NS> out;
    bool keep;
    if (hs && !ho) {  // :94-104: dropped iff other has seen all of it
      out = r;
      keep = !vle(r, oclk);
    } else if (ho && !hs) {  // :132-138
      out = vsub(orow, sclk);
      keep = vany(out);
    } else {  // :105-128
      const Row<NS> common = vcommon(r, orow);  // VClock::intersection
      const Row<NS> e1 = vsub(vsub(r, common), oclk), e2 = vsub(vsub(orow, common), sclk);
      out = vmax(vmax(common, e1), e2);
      keep = vany(out);
    }
    if (keep) {
      if (lane == 0u) Wn.key[n] = hs ? ka : kb;
      strow(Wn.row + n * c.A, out, c.A, lane);
      ++n;
    }
    if (hs) ++a;
    if (ho) ++b;
  }
  Wn.nm = n;
  // deferred: union by clock (:141-148), sets united — CLOCK ORDER merge of both lists
  const uint32_t od = Wo.nd;
  uint32_t p = 0, q = 0, nd = 0;
  while (p < Wc.nd || q < od) {
    const Row<NS> dp = p < Wc.nd ? ldrow<NS>(Wc.dclk + p * c.A, c.A, lane) : zrow<NS>();
    const Row<NS> dq = q < od ? ldrow<NS>(Wo.dclk + q * c.A, c.A, lane) : zrow<NS>();
    int ord;
    if (p >= Wc.nd) ord = 1;
    else if (q >= od) ord = -1;
    else ord = vorder(dp, dq, lane);
    strow(Wn.dclk + nd * c.A, ord <= 0 ? dp : dq, c.A, lane);
    if (lane == 0u) {  // sorted union of the member sets
      const uint64_t* xs = ord <= 0 ? Wc.dset + p * Wc.sw : nullptr;
      const uint32_t nx = ord <= 0 ? Wc.dn[p] : 0u;
      const uint64_t* ys = ord >= 0 ? Wo.dset + q * Wo.sw : nullptr;
      const uint32_t ny = ord >= 0 ? Wo.dn[q] : 0u;
      uint32_t i = 0, j = 0, k = 0;
      while (i < nx || j < ny) {
        const uint64_t kx = i < nx ? xs[i] : ~0ull, ky = j < ny ? ys[j] : ~0ull;
        const uint64_t m = kx < ky ? kx : ky;
        if (kx == m) ++i;
        if (ky == m) ++j;
        Wn.dset[nd * Wn.sw + k++] = m;
      }
      Wn.dn[nd] = k;
    }
    ++nd;
    if (ord <= 0) ++p;
    if (ord >= 0) ++q;
  }
  Wn.nd = nd;
  sclk = vmax(sclk, oclk);  // :153
  mo_sync();
  ws_apply_deferred(Wn, sclk, mdead, ddead, c, lane);  // :155
}

// Orswot::truncate (src/orswot.rs:159-172) of W (top clock `clk`) by `t`.
template <int NS>
__device__ void ws_truncate(Ws& W, Row<NS>& clk, Row<NS> t, uint32_t* mdead, uint32_t* ddead, const Caps& c,
                            uint32_t lane) {
  // merge with an empty set whose clock is t: members t covers are dropped
  // (:94-104); it has no entries or deferred removes; the clocks merge
  for (uint32_t j = 0; j < W.nm; ++j) {
    const bool covered = vle(ldrow<NS>(W.row + j * c.A, c.A, lane), t);
    if (covered && lane == 0u) mdead[j] = 1u;
  }
  clk = vmax(clk, t);
  mo_sync();
  ws_apply_deferred(W, clk, mdead, ddead, c, lane);
  // forget t from the top clock and every member clock (an emptied member stays)
  clk = vsub(clk, t);
  for (uint32_t j = 0; j < W.nm; ++j) strow(W.row + j * c.A, vsub(ldrow<NS>(W.row + j * c.A, c.A, lane), t), c.A, lane);
  mo_sync();
}

// Write W (top clock clk) into key slot kr of R; false if a capacity is exceeded.
template <int NS>
__device__ bool ws_store(const Ws& W, Row<NS> clk, const crdt_map_orswot_slab& R, uint64_t kr, const Caps& c,
                         uint32_t lane) {
  bool fits = W.nm <= R.mcap && W.nd <= R.vdcap;
  for (uint32_t d = 0; d < W.nd; ++d) fits = fits && uni(W.dn[d]) <= R.vscap;
  if (!fits) return false;
  strow(R.vclock + kr * c.A, clk, c.A, lane);
  if (lane == 0u) { R.vn_mem[kr] = W.nm; R.vn_def[kr] = W.nd; }
  const uint32_t nm = W.nm, nmA = W.nm * c.A, ndA = W.nd * c.A, nd = W.nd, vs = R.vscap, SW = W.sw;
  const uint64_t* key = W.key;
  const uint64_t* row = W.row;
  const uint64_t* dclk = W.dclk;
  const uint64_t* dset = W.dset;
  const uint32_t* dn = W.dn;
  // only the used slots are written (the capacity past the counts is left
  // as it was: include/crdts_hip.h)
  fill64(R.vmem + kr * R.mcap, nm, lane, [&](uint64_t j) { return key[j]; });
  fill64(R.vmclock + kr * R.mcap * c.A, nmA, lane, [&](uint64_t e) { return row[e]; });
  fill64(R.vdclock + kr * R.vdcap * c.A, ndA, lane, [&](uint64_t e) { return dclk[e]; });
  for (uint32_t d = lane; d < nd; d += kMoW) R.vdset_n[kr * R.vdcap + d] = dn[d];
  for (uint32_t d = 0; d < nd; ++d)
    fill64(R.vdset + (kr * R.vdcap + d) * vs, uni(dn[d]), lane, [&](uint64_t j) { return dset[d * SW + j]; });
  return true;
}

template <int NS, int MINW = 4>
__global__ __launch_bounds__(kMoW, MINW) void map_orswot_merge_kernel(crdt_map_orswot_slab S, crdt_map_orswot_slab O,
                                                                crdt_map_orswot_slab R, uint64_t n_obj, uint32_t A,
                                                                uint32_t md_cap, int* __restrict__ status,
                                                                uint32_t* __restrict__ ctl) {
  extern __shared__ uint64_t mo_lds[];
  const uint32_t lane = threadIdx.x;
  const Caps c{S.mcap + O.mcap, S.vdcap + O.vdcap, S.vscap + O.vscap, A};
  // workspaces: self's key slot (W0), other's (W2), their merge (W1); then the
  // member / deferred drop flags and the map deferred staging area
  Ws W0, W1, W2;
  uint32_t* mdead;
  uint64_t* md;
  {
    uint64_t* p = mo_lds;
    auto carve = [&](Ws& W, uint32_t m, uint32_t d, uint32_t sw) {  // (no indexed array: W stays in registers)
      W.key = p; p += m;
      W.row = p; p += m * A;
      W.dclk = p; p += d * A;
      W.dset = p; p += d * sw;
      W.sw = sw;
      W.nm = W.nd = 0u;
    };
    carve(W0, S.mcap, S.vdcap, S.vscap);
    carve(W1, c.MW, c.DW, c.SW);
    carve(W2, O.mcap, O.vdcap, O.vscap);
    mdead = (uint32_t*)p;
    for (uint32_t j = lane; j < c.MW + c.DW; j += kMoW) mdead[j] = 0u;
    md = p + (c.MW + c.DW + 1u) / 2u;
  }
  // the map deferred bookkeeping (dcap_s + dcap_o <= 512 entries each, after
  // the staging area): the combined list, (self deferred idx + 1) | (other
  // deferred idx + 1) << 16; both sides' set sizes; the entries naming a key
  const uint32_t DC = S.dcap + O.dcap;
  uint32_t* const comb = (uint32_t*)(md + md_cap);
  uint32_t* const mdn0 = comb + DC;
  uint32_t* const mdn1 = mdn0 + S.dcap;
  uint32_t* const nl = mdn0 + DC;
  // then the three workspaces' nested deferred set sizes (vdcap_s, DW, vdcap_o)
  W0.dn = nl + DC;
  W1.dn = W0.dn + S.vdcap;
  W2.dn = W1.dn + c.DW;
  uint32_t* const ddead = mdead + c.MW;
  mo_sync();
  BlockTickets<4> sched(n_obj, ctl + 3, lane);  // (sched.h)
  for (uint64_t i = sched.first(); i < n_obj; i = sched.next(i)) {
    const Row<NS> cS = rowv<NS>(S.clock, i, A, lane), cO = rowv<NS>(O.clock, i, A, lane);
    const Row<NS> cM = vmax(cS, cO);  // VClock::merge
    const uint32_t nS = uni(S.n_keys[i]), nO = uni(O.n_keys[i]);
    const uint32_t dS = uni(S.n_def[i]), dO = uni(O.n_def[i]);
    if (nS > S.kcap || nO > O.kcap || dS > S.dcap || dO > O.dcap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    // the first 64 keys of each side and their nested counts in registers
    // (lane k: key k), one round trip
    const bool ls = lane < nS, lo = lane < nO;
    const uint64_t kregS = ls ? S.keys[i * S.kcap + lane] : 0ull, kregO = lo ? O.keys[i * O.kcap + lane] : 0ull;
    const uint32_t vmS = ls ? S.vn_mem[i * S.kcap + lane] : 0u, vdS = ls ? S.vn_def[i * S.kcap + lane] : 0u;
    const uint32_t vmO = lo ? O.vn_mem[i * O.kcap + lane] : 0u, vdO = lo ? O.vn_def[i * O.kcap + lane] : 0u;
    // every count the loops below trust, within its capacity (the nested
    // deferred set sizes up to the wave's largest count, so their loads
    // issue together and no unused slot is read)
    bool bad = vmS > S.mcap || vdS > S.vdcap || vmO > O.mcap || vdO > O.vdcap;
    uint32_t mvd = (vdS < S.vdcap ? vdS : S.vdcap) > (vdO < O.vdcap ? vdO : O.vdcap) ? (vdS < S.vdcap ? vdS : S.vdcap)
                                                                                   : (vdO < O.vdcap ? vdO : O.vdcap);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const uint32_t t = __shfl_xor(mvd, off, kMoW);
      mvd = t > mvd ? t : mvd;
    }
    mvd = uni(mvd);
    for (uint32_t d = 0; d < mvd; ++d) {
      if (ls && d < vdS) bad = bad || S.vdset_n[(i * S.kcap + lane) * S.vdcap + d] > S.vscap;
      if (lo && d < vdO) bad = bad || O.vdset_n[(i * O.kcap + lane) * O.vdcap + d] > O.vscap;
    }
    for (uint32_t k = kMoW + lane; k < nS; k += kMoW) {
      const uint64_t ki = i * S.kcap + k;
      bad = bad || S.vn_mem[ki] > S.mcap || S.vn_def[ki] > S.vdcap;
      for (uint32_t d = 0; !bad && d < S.vn_def[ki]; ++d) bad = S.vdset_n[ki * S.vdcap + d] > S.vscap;
    }
    for (uint32_t k = kMoW + lane; k < nO; k += kMoW) {
      const uint64_t ki = i * O.kcap + k;
      bad = bad || O.vn_mem[ki] > O.mcap || O.vn_def[ki] > O.vdcap;
      for (uint32_t d = 0; !bad && d < O.vn_def[ki]; ++d) bad = O.vdset_n[ki * O.vdcap + d] > O.vscap;
    }
    // the map deferred set sizes, one lane per entry
    for (uint32_t d = lane; d < dS; d += kMoW) {
      const uint32_t x = S.dset_n[i * S.dcap + d];
      mdn0[d] = x;
      bad = bad || x > S.scap;
    }
    for (uint32_t d = lane; d < dO; d += kMoW) {
      const uint32_t x = O.dset_n[i * O.dcap + d];
      mdn1[d] = x;
      bad = bad || x > O.scap;
    }
    if (__ballot(bad) != 0ull) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    mo_sync();
    // the map deferred sets staged in LDS when they fit (md_cap words): the
    // key loop asks each of them about every key. (Staging their clocks too
    // cost more occupancy than the round trips it saved: DESIGN.md §9.)
    const uint32_t sS = S.scap, sO = O.scap;
    const bool st = (uint64_t)dS * sS + (uint64_t)dO * sO <= md_cap;
    uint64_t* const mdS = md;
    uint64_t* const mdO = mdS + dS * sS;
    if (st) {  // the used entries of each set
      for (uint32_t e = lane; e < dS * sS; e += kMoW) {
        const uint32_t d = e / sS;
        if (e - d * sS < mdn0[d]) mdS[e] = S.dset[i * S.dcap * sS + e];
      }
      for (uint32_t e = lane; e < dO * sO; e += kMoW) {
        const uint32_t d = e / sO;
        if (e - d * sO < mdn1[d]) mdO[e] = O.dset[i * O.dcap * sO + e];
      }
    }
    mo_sync();
    auto sdc = [&](uint32_t a) -> Row<NS> { return rowv<NS>(S.dclock, i * S.dcap + a, A, lane); };
    auto odc = [&](uint32_t b) -> Row<NS> { return rowv<NS>(O.dclock, i * O.dcap + b, A, lane); };
    // ---- combined map deferred list: self's, plus other's that self's clock does not cover
    //      (apply_rm's deferral, against the pre-merge clock), united in CLOCK ORDER
    uint32_t nc = 0;
    {
      uint32_t a = 0, b = 0;
      while (a < dS || b < dO) {
        if (b < dO && vle(odc(b), cS)) { ++b; continue; }
        int o;
        if (a >= dS) o = 1;
        else if (b >= dO) o = -1;
        else o = vorder(sdc(a), odc(b), lane);
        if (lane == 0u) comb[nc] = (o <= 0 ? a + 1u : 0u) | ((o >= 0 ? b + 1u : 0u) << 16);
        ++nc;
        if (o <= 0) ++a;
        if (o >= 0) ++b;
      }
    }
    mo_sync();
    auto comb_clock = [&](uint32_t e) -> Row<NS> {
      const uint32_t sa = e & 0xFFFFu, sb = e >> 16;
      return sa ? sdc(sa - 1u) : odc(sb - 1u);
    };
    // the combined entries naming `key`, ascending, into nl; returns their count
    auto comb_named = [&](uint64_t key) -> uint32_t {
      uint32_t nn = 0;
      for (uint32_t k = 0; k < nc; ++k) {
        const uint32_t e = uni(comb[k]), sa = e & 0xFFFFu, sb = e >> 16;
        bool f = false;
        if (sa)
          f = set_has(st ? mdS + (sa - 1u) * sS : S.dset + (i * S.dcap + sa - 1u) * sS, uni(mdn0[sa - 1u]), key, lane);
        if (!f && sb)
          f = set_has(st ? mdO + (sb - 1u) * sO : O.dset + (i * O.dcap + sb - 1u) * sO, uni(mdn1[sb - 1u]), key, lane);
        if (f) {
          if (lane == 0u) nl[nn] = k;
          ++nn;
        }
      }
      mo_sync();
      return nn;
    };
    // ---- entries, key by key in ascending order
    uint32_t nk = 0, a = 0, b = 0;
    bool over = false;
    while (a < nS || b < nO) {
      const uint64_t ka = a < nS ? (a < kMoW ? lane64(kregS, a) : uni64(S.keys[i * S.kcap + a])) : ~0ull;
      const uint64_t kb = b < nO ? (b < kMoW ? lane64(kregO, b) : uni64(O.keys[i * O.kcap + b])) : ~0ull;
      const bool chs = a < nS && (b >= nO || ka <= kb), cho = b < nO && (a >= nS || kb <= ka);
      const uint64_t ckey = chs ? ka : kb;
      const uint64_t ia = i * S.kcap + a, ib = i * O.kcap + b;
      const uint32_t ca = a, cb = b;
      if (chs) ++a;
      if (cho) ++b;
      // both entry clocks and both nested top clocks in one round trip
      const Row<NS> eS = chs ? rowv<NS>(S.eclock, ia, A, lane) : zrow<NS>();
      const Row<NS> eO = cho ? rowv<NS>(O.eclock, ib, A, lane) : zrow<NS>();
      const Row<NS> vS = chs ? rowv<NS>(S.vclock, ia, A, lane) : zrow<NS>();
      const Row<NS> vO = cho ? rowv<NS>(O.vclock, ib, A, lane) : zrow<NS>();
      Row<NS> ec, del;
      if (chs && !cho) {  // other has not seen it, or saw it and dropped it
        ec = vsub(eS, cO);
        del = vsub(cO, ec);
      } else if (cho && !chs) {
        ec = vsub(eO, cS);
        del = vsub(cS, ec);
      } else {
        const Row<NS> common = vcommon(eS, eO);  // VClock::intersection
        const Row<NS> e1 = vsub(vsub(eS, common), cO), e2 = vsub(vsub(eO, common), cS);
        ec = vmax(vmax(common, e1), e2);
        del = vsub(vmax(e1, e2), ec);
      }
      bool keep = vany(ec);
      // apply_deferred: the entry clock loses every combined clock naming the key
      // (subtracts commute; an entry emptied at any step is gone for good)
      const uint32_t nn = keep && nc ? comb_named(ckey) : 0u;
      if (keep) {
        for (uint32_t t = 0; t < nn; ++t) ec = vsub(ec, comb_clock(uni(comb[uni(nl[t])])));
        keep = vany(ec);
      }
      if (keep && nk >= R.kcap) {
        over = true;
        keep = false;
      }
      if (keep) {
        // the nested set: self's (merged with other's when both have the key) ...
        if (chs) ws_counts(W0, S, ia, ca, vmS, vdS);
        if (cho) ws_counts(W2, O, ib, cb, vmO, vdO);
        if (chs) ws_copy(W0, S, ia, c, lane);
        if (cho) ws_copy(W2, O, ib, c, lane);
        mo_sync();
        Row<NS> vclk = chs ? vS : vO;
        Ws Wk = chs ? W0 : W2;
        if (chs && cho) {
          ws_merge(W0, W2, W1, vclk, vO, mdead, ddead, c, lane);
          Wk = W1;
        }
        // ... truncated by the removers' clock (Map::merge), then by each deferred
        // clock naming the key, in CLOCK ORDER (apply_deferred -> apply_rm)
        ws_truncate(Wk, vclk, del, mdead, ddead, c, lane);
        for (uint32_t t = 0; t < nn; ++t)
          ws_truncate(Wk, vclk, comb_clock(uni(comb[uni(nl[t])])), mdead, ddead, c, lane);
        const uint64_t ir = i * R.kcap + nk;
        if (ws_store(Wk, vclk, R, ir, c, lane)) {
          if (lane == 0u) R.keys[ir] = ckey;
          strow(R.eclock + ir * A, ec, A, lane);
          ++nk;
        } else {
          over = true;
        }
        mo_sync();
      }
    }
    if (lane == 0u) R.n_keys[i] = nk;
    strow(R.clock + i * A, cM, A, lane);
    // ---- map deferred kept: the combined clocks the merged clock does not cover, sets united
    uint32_t nd = 0;
    for (uint32_t k = 0; k < nc; ++k) {
      const uint32_t e = uni(comb[k]);
      const uint32_t sa = e & 0xFFFFu, sb = e >> 16;
      const Row<NS> D = comb_clock(e);
      if (vle(D, cM)) continue;
      if (nd >= R.dcap) { over = true; break; }
      const uint64_t dr = i * R.dcap + nd;
      strow(R.dclock + dr * A, D, A, lane);
      uint32_t cnt = 0;
      if (lane == 0u) {  // sorted union of the two key sets
        const uint64_t* xs = sa ? (st ? mdS + (sa - 1u) * sS : S.dset + (i * S.dcap + sa - 1u) * sS) : nullptr;
        const uint64_t* ys = sb ? (st ? mdO + (sb - 1u) * sO : O.dset + (i * O.dcap + sb - 1u) * sO) : nullptr;
        const uint32_t nx = sa ? mdn0[sa - 1u] : 0u, ny = sb ? mdn1[sb - 1u] : 0u;
        uint32_t p = 0, q = 0;
        while (p < nx || q < ny) {
          const uint64_t kx = p < nx ? xs[p] : ~0ull, ky = q < ny ? ys[q] : ~0ull;
          const uint64_t kk = kx < ky ? kx : ky;
          if (kx == kk) ++p;
          if (ky == kk) ++q;
          if (cnt < R.scap) R.dset[dr * R.scap + cnt] = kk;
          ++cnt;
        }
        R.dset_n[dr] = cnt < R.scap ? cnt : R.scap;
      }
      over = over || uni(cnt) > R.scap;
      ++nd;
    }
    if (lane == 0u) R.n_def[i] = nd;
    if (over && lane == 0u) atomicCAS(status, 0, CRDT_ECAPACITY);
    mo_sync();
  }
}

}  // namespace

// The kernel's dynamic workspace: self's and other's key slots and their
// merge (W0, W2, W1), the drop flags, the map deferred bookkeeping (3 x
// (dcap_s + dcap_o) u32) and the workspaces' nested deferred set sizes
// (2 x (vdcap_s + vdcap_o) u32). This is the bound crdt_map_orswot_merge
// checks against 64 KB.
size_t map_orswot_lds_bytes(const crdt_map_orswot_slab& S, const crdt_map_orswot_slab& O, uint32_t A) {
  auto per = [&](size_t m, size_t d, size_t s) { return 8 * (m + m * A + d * A + d * s); };
  const size_t MW = S.mcap + O.mcap, DW = S.vdcap + O.vdcap, SW = S.vscap + O.vscap;
  return per(S.mcap, S.vdcap, S.vscap) + per(O.mcap, O.vdcap, O.vscap) + per(MW, DW, SW) + 8 * ((MW + DW + 1) / 2) +
         8 * ((3 * ((size_t)S.dcap + O.dcap) + 2 * DW + 1) / 2);
}

int launch_map_orswot_merge(const crdt_map_orswot_slab& S, const crdt_map_orswot_slab& O,
                            const crdt_map_orswot_slab& R, uint64_t n_obj, uint32_t A, int* status, uint32_t* ctl,
                            hipStream_t stream, int variant) {
  if (n_obj == 0) return CRDT_OK;
  const size_t lds = map_orswot_lds_bytes(S, O, A);
  if (lds > kMoLdsMax) return CRDT_EINVAL;
  // the map deferred staging area: the capacity's sets when they fit
  // kMoStageMax (diag variant 401: none, the sets read from HBM)
  const size_t md = 8 * ((size_t)S.dcap * S.scap + (size_t)O.dcap * O.scap);
  const size_t md_bytes = (variant == 401 || md > kMoStageMax || lds + md > kMoLdsMax) ? 0 : md;
  const uint32_t md_cap = (uint32_t)(md_bytes / 8);
  // (diag variant 402: no register bound — 3 waves/SIMD, no spill)
  const void* fn = A > 64u ? (const void*)map_orswot_merge_kernel<2>
                   : variant == 402 ? (const void*)map_orswot_merge_kernel<1, 1>
                                    : (const void*)map_orswot_merge_kernel<1>;
  int dev = 0, cus = 256, occ = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // one single-wave block per resident slot (LDS-bound: the workspace sizes it)
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kMoW, lds + md_bytes) != hipSuccess || occ < 1) occ = 16;
  const uint64_t cap = (uint64_t)cus * (uint32_t)occ;
  const uint32_t blocks = (uint32_t)(n_obj < cap ? n_obj : cap);
  if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;  // ctl[3]: tickets
  void* args[] = {(void*)&S, (void*)&O, (void*)&R, &n_obj, &A, (void*)&md_cap, &status, &ctl};
  if (hipLaunchKernel(fn, dim3(blocks), dim3(kMoW), args, lds + md_bytes, stream) != hipSuccess) return CRDT_EHIP;
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
