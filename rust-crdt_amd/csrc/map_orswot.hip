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
// + deferred clocks + their member sets), double-buffered for the set merge;
// keys, members and deferred entries are walked by wave-uniform loops.
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "map_rows.h"
#include "sched.h"

namespace crdts_hip {
namespace {

constexpr uint32_t kMoW = 64;
constexpr uint32_t kMoComb = 64;       // combined map deferred entries (<= dcap_self + dcap_other)
constexpr uint32_t kMoLdsMax = 65536;  // workspace limit per wave

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
  uint64_t* dset;  // [DW][SW] member sets, ascending
  uint32_t nm, nd;
};
struct Caps {
  uint32_t MW, DW, SW, A;
};

// Load key slot ki of a slab's nested set into W.
__device__ void ws_load(Ws& W, const crdt_map_orswot_slab& X, uint64_t ki, const Caps& c, uint32_t lane) {
  W.nm = uni(X.vn_mem[ki]);
  W.nd = uni(X.vn_def[ki]);
  for (uint32_t j = lane; j < W.nm; j += kMoW) W.key[j] = X.vmem[ki * X.mcap + j];
  for (uint32_t e = lane; e < W.nm * c.A; e += kMoW) W.row[e] = X.vmclock[ki * X.mcap * c.A + e];
  for (uint32_t e = lane; e < W.nd * c.A; e += kMoW) W.dclk[e] = X.vdclock[ki * X.vdcap * c.A + e];
  for (uint32_t d = 0; d < W.nd; ++d) {
    const uint64_t di = ki * X.vdcap + d;
    const uint32_t n = uni(X.vdset_n[di]);
    if (lane == 0u) W.dn[d] = n;
    for (uint32_t j = lane; j < n; j += kMoW) W.dset[d * c.SW + j] = X.vdset[di * X.vscap + j];
  }
  mo_sync();
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
      const uint64_t m = uni64(W.dset[d * c.SW + j]);
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
      uint64_t s0 = lane < n ? W.dset[d * c.SW + lane] : 0ull;
      mo_sync();
      strow(W.dclk + k * c.A, D, c.A, lane);
      if (lane == 0u) W.dn[k] = n;
      if (lane < n) W.dset[k * c.SW + lane] = s0;  // SW <= 64
      mo_sync();
    }
    ++k;
  }
  W.nd = k;
  for (uint32_t j = lane; j < c.MW; j += kMoW) mdead[j] = 0u;
  for (uint32_t j = lane; j < c.DW; j += kMoW) ddead[j] = 0u;
  mo_sync();
}

// Orswot::merge (src/orswot.rs:87-157): Wn = Wc.merge(&other), other = key
// slot ko of O. `sclk` (Wc's top clock) becomes the merged clock.
template <int NS>
__device__ void ws_merge(const Ws& Wc, Ws& Wn, Row<NS>& sclk, const crdt_map_orswot_slab& O, uint64_t ko,
                         uint32_t* mdead, uint32_t* ddead, const Caps& c, uint32_t lane) {
  const Row<NS> oclk = rowv<NS>(O.vclock, ko, c.A, lane);
  const uint32_t no = uni(O.vn_mem[ko]);
  uint32_t a = 0, b = 0, n = 0;
  while (a < Wc.nm || b < no) {
    const uint64_t ka = a < Wc.nm ? uni64(Wc.key[a]) : ~0ull;
    const uint64_t kb = b < no ? uni64(O.vmem[ko * O.mcap + b]) : ~0ull;
    const bool hs = a < Wc.nm && (b >= no || ka <= kb), ho = b < no && (a >= Wc.nm || kb <= ka);
    const Row<NS> r = hs ? ldrow<NS>(Wc.row + a * c.A, c.A, lane) : zrow<NS>();
    const Row<NS> orow = ho ? rowv<NS>(O.vmclock, ko * O.mcap + b, c.A, lane) : zrow<NS>();
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
  const uint32_t od = uni(O.vn_def[ko]);
  uint32_t p = 0, q = 0, nd = 0;
  while (p < Wc.nd || q < od) {
    const Row<NS> dp = p < Wc.nd ? ldrow<NS>(Wc.dclk + p * c.A, c.A, lane) : zrow<NS>();
    const Row<NS> dq = q < od ? rowv<NS>(O.vdclock, ko * O.vdcap + q, c.A, lane) : zrow<NS>();
    int ord;
    if (p >= Wc.nd) ord = 1;
    else if (q >= od) ord = -1;
    else ord = vorder(dp, dq, lane);
    strow(Wn.dclk + nd * c.A, ord <= 0 ? dp : dq, c.A, lane);
    if (lane == 0u) {  // sorted union of the member sets
      const uint64_t* xs = ord <= 0 ? Wc.dset + p * c.SW : nullptr;
      const uint32_t nx = ord <= 0 ? Wc.dn[p] : 0u;
      const uint64_t* ys = ord >= 0 ? O.vdset + (ko * O.vdcap + q) * O.vscap : nullptr;
      const uint32_t ny = ord >= 0 ? O.vdset_n[ko * O.vdcap + q] : 0u;
      uint32_t i = 0, j = 0, k = 0;
      while (i < nx || j < ny) {
        const uint64_t kx = i < nx ? xs[i] : ~0ull, ky = j < ny ? ys[j] : ~0ull;
        const uint64_t m = kx < ky ? kx : ky;
        if (kx == m) ++i;
        if (ky == m) ++j;
        Wn.dset[nd * c.SW + k++] = m;
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
  const uint32_t nm = W.nm, nmA = W.nm * c.A, ndA = W.nd * c.A, nd = W.nd, vs = R.vscap, SW = c.SW;
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

template <int NS>
__global__ __launch_bounds__(kMoW) void map_orswot_merge_kernel(crdt_map_orswot_slab S, crdt_map_orswot_slab O,
                                                                crdt_map_orswot_slab R, uint64_t n_obj, uint32_t A,
                                                                int* __restrict__ status, uint32_t* __restrict__ ctl) {
  extern __shared__ uint64_t mo_lds[];
  __shared__ uint32_t comb[kMoComb];  // (self deferred idx + 1) | (other deferred idx + 1) << 8
  const uint32_t lane = threadIdx.x;
  const Caps c{S.mcap + O.mcap, S.vdcap + O.vdcap, S.vscap + O.vscap, A};
  // workspace: two nested sets, then the member / deferred drop flags
  Ws W0, W1;
  uint32_t* mdead;
  {
    uint64_t* p = mo_lds;
    for (Ws* w : {&W0, &W1}) {
      w->key = p; p += c.MW;
      w->row = p; p += c.MW * A;
      w->dclk = p; p += c.DW * A;
      w->dset = p; p += c.DW * c.SW;
      w->dn = (uint32_t*)p; p += (c.DW + 1u) / 2u;
      w->nm = w->nd = 0u;
    }
    mdead = (uint32_t*)p;
    for (uint32_t j = lane; j < c.MW + c.DW; j += kMoW) mdead[j] = 0u;
  }
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
    // every count the loops below trust, within its capacity
    bool bad = false;
    for (uint32_t k = lane; k < nS; k += kMoW) {
      const uint64_t ki = i * S.kcap + k;
      bad = bad || S.vn_mem[ki] > S.mcap || S.vn_def[ki] > S.vdcap;
      for (uint32_t d = 0; !bad && d < S.vn_def[ki]; ++d) bad = S.vdset_n[ki * S.vdcap + d] > S.vscap;
    }
    for (uint32_t k = lane; k < nO; k += kMoW) {
      const uint64_t ki = i * O.kcap + k;
      bad = bad || O.vn_mem[ki] > O.mcap || O.vn_def[ki] > O.vdcap;
      for (uint32_t d = 0; !bad && d < O.vn_def[ki]; ++d) bad = O.vdset_n[ki * O.vdcap + d] > O.vscap;
    }
    for (uint32_t k = lane; k < dS; k += kMoW) bad = bad || S.dset_n[i * S.dcap + k] > S.scap;
    for (uint32_t k = lane; k < dO; k += kMoW) bad = bad || O.dset_n[i * O.dcap + k] > O.scap;
    if (__ballot(bad) != 0ull) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    // ---- combined map deferred list: self's, plus other's that self's clock does not cover
    //      (apply_rm's deferral, against the pre-merge clock), united in CLOCK ORDER
    uint32_t nc = 0;
    {
      uint32_t a = 0, b = 0;
      while (a < dS || b < dO) {
        if (b < dO && vle(rowv<NS>(O.dclock, i * O.dcap + b, A, lane), cS)) { ++b; continue; }
        int o;
        if (a >= dS) o = 1;
        else if (b >= dO) o = -1;
        else o = vorder(rowv<NS>(S.dclock, i * S.dcap + a, A, lane), rowv<NS>(O.dclock, i * O.dcap + b, A, lane), lane);
        if (lane == 0u) comb[nc] = (o <= 0 ? a + 1u : 0u) | ((o >= 0 ? b + 1u : 0u) << 8);
        ++nc;
        if (o <= 0) ++a;
        if (o >= 0) ++b;
      }
    }
    mo_sync();
    auto comb_clock = [&](uint32_t e) -> Row<NS> {
      const uint32_t sa = e & 255u, sb = e >> 8;
      return sa ? rowv<NS>(S.dclock, i * S.dcap + sa - 1u, A, lane) : rowv<NS>(O.dclock, i * O.dcap + sb - 1u, A, lane);
    };
    auto comb_names = [&](uint32_t e, uint64_t key) -> bool {
      const uint32_t sa = e & 255u, sb = e >> 8;
      bool named = false;
      if (sa) {
        const uint64_t di = i * S.dcap + sa - 1u;
        named = set_has(S.dset + di * S.scap, S.dset_n[di], key, lane);
      }
      if (!named && sb) {
        const uint64_t di = i * O.dcap + sb - 1u;
        named = set_has(O.dset + di * O.scap, O.dset_n[di], key, lane);
      }
      return named;
    };
    // ---- entries, key by key in ascending order
    uint32_t nk = 0, a = 0, b = 0;
    bool over = false;
    while (a < nS || b < nO) {
      const uint64_t ka = a < nS ? uni64(S.keys[i * S.kcap + a]) : ~0ull;
      const uint64_t kb = b < nO ? uni64(O.keys[i * O.kcap + b]) : ~0ull;
      const bool hs = a < nS && (b >= nO || ka <= kb), ho = b < nO && (a >= nS || kb <= ka);
      const uint64_t key = hs ? ka : kb;
      const uint64_t ia = i * S.kcap + a, ib = i * O.kcap + b;
      const Row<NS> eS = hs ? rowv<NS>(S.eclock, ia, A, lane) : zrow<NS>();
      const Row<NS> eO = ho ? rowv<NS>(O.eclock, ib, A, lane) : zrow<NS>();
      Row<NS> ec, del;
      if (hs && !ho) {  // other has not seen it, or saw it and dropped it
        ec = vsub(eS, cO);
        del = vsub(cO, ec);
      } else if (ho && !hs) {
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
      if (keep) {
        for (uint32_t k = 0; k < nc; ++k)
          if (comb_names(comb[k], key)) ec = vsub(ec, comb_clock(comb[k]));
        keep = vany(ec);
      }
      if (keep && nk >= R.kcap) {
        over = true;
        keep = false;
      }
      if (keep) {
        // the nested set: self's (merged with other's when both have the key) ...
        Row<NS> vclk;
        Ws Wk;
        if (hs) {
          ws_load(W0, S, ia, c, lane);
          vclk = rowv<NS>(S.vclock, ia, A, lane);
          if (ho) {
            ws_merge(W0, W1, vclk, O, ib, mdead, ddead, c, lane);
            Wk = W1;
          } else {
            Wk = W0;
          }
        } else {
          ws_load(W0, O, ib, c, lane);
          vclk = rowv<NS>(O.vclock, ib, A, lane);
          Wk = W0;
        }
        // ... truncated by the removers' clock (Map::merge), then by each deferred
        // clock naming the key, in CLOCK ORDER (apply_deferred -> apply_rm)
        ws_truncate(Wk, vclk, del, mdead, ddead, c, lane);
        for (uint32_t k = 0; k < nc; ++k)
          if (comb_names(comb[k], key)) ws_truncate(Wk, vclk, comb_clock(comb[k]), mdead, ddead, c, lane);
        const uint64_t ir = i * R.kcap + nk;
        if (ws_store(Wk, vclk, R, ir, c, lane)) {
          if (lane == 0u) R.keys[ir] = key;
          strow(R.eclock + ir * A, ec, A, lane);
          ++nk;
        } else {
          over = true;
        }
        mo_sync();
      }
      if (hs) ++a;
      if (ho) ++b;
    }
    if (lane == 0u) R.n_keys[i] = nk;
    strow(R.clock + i * A, cM, A, lane);
    // ---- map deferred kept: the combined clocks the merged clock does not cover, sets united
    uint32_t nd = 0;
    for (uint32_t k = 0; k < nc; ++k) {
      const uint32_t e = comb[k];
      const uint32_t sa = e & 255u, sb = e >> 8;
      const Row<NS> D = comb_clock(e);
      if (vle(D, cM)) continue;
      if (nd >= R.dcap) { over = true; break; }
      const uint64_t dr = i * R.dcap + nd;
      strow(R.dclock + dr * A, D, A, lane);
      uint32_t cnt = 0;
      if (lane == 0u) {  // sorted union of the two key sets
        const uint64_t* xs = sa ? S.dset + (i * S.dcap + sa - 1u) * S.scap : nullptr;
        const uint64_t* ys = sb ? O.dset + (i * O.dcap + sb - 1u) * O.scap : nullptr;
        const uint32_t nx = sa ? S.dset_n[i * S.dcap + sa - 1u] : 0u, ny = sb ? O.dset_n[i * O.dcap + sb - 1u] : 0u;
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

size_t map_orswot_lds_bytes(const crdt_map_orswot_slab& S, const crdt_map_orswot_slab& O, uint32_t A) {
  const size_t MW = S.mcap + O.mcap, DW = S.vdcap + O.vdcap, SW = S.vscap + O.vscap;
  const size_t per = 8 * (MW + MW * A + DW * A + DW * SW + (DW + 1) / 2);
  return 2 * per + 4 * (MW + DW) + 16;
}

int launch_map_orswot_merge(const crdt_map_orswot_slab& S, const crdt_map_orswot_slab& O,
                            const crdt_map_orswot_slab& R, uint64_t n_obj, uint32_t A, int* status, uint32_t* ctl,
                            hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  const size_t lds = map_orswot_lds_bytes(S, O, A);
  if (lds > kMoLdsMax) return CRDT_EINVAL;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t cap = (uint64_t)cus * 16u;
  const uint32_t blocks = (uint32_t)(n_obj < cap ? n_obj : cap);
  if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;  // ctl[3]: tickets
  if (A > 64u)
    hipLaunchKernelGGL(map_orswot_merge_kernel<2>, dim3(blocks), dim3(kMoW), lds, stream, S, O, R, n_obj, A, status,
                       ctl);
  else
    hipLaunchKernelGGL(map_orswot_merge_kernel<1>, dim3(blocks), dim3(kMoW), lds, stream, S, O, R, n_obj, A, status,
                       ctl);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
