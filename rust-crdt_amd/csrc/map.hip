// Map<u64, MVReg<u64, A>, A>::merge, batched.
//
// Reference: Map::merge (src/map.rs:191-268) — per key, the entry clocks are
// reconciled against both map clocks (self-only :198-211, both :212-237,
// other-only :241-250), nested values merged (MVReg::merge,
// src/mvreg.rs:121-153) and truncated by the clock of the actors that removed
// the entry (MVReg::truncate, src/mvreg.rs:71-83); other's deferred removes
// are re-deferred against self's pre-merge clock (apply_rm :336-349 — its
// entry edits land on the entries the merge then replaces, so only the
// deferral survives), the clocks merge, and apply_deferred (:323-333)
// subtracts every deferred clock from its keys' entries, dropping emptied
// entries and truncating the rest, re-deferring the clocks not yet covered.
// Subtracts commute, so each kept key takes all its deferred clocks at once.
//
// One wave per map pair; lane = actor slot, NS slots per lane (NS = 1 for
// n_actors <= 64, 2 for <= 128: map_rows.h), so every VClock operation on
// dense rows is NS lane-parallel ops plus a ballot; keys, values and deferred
// entries are walked by wave-uniform loops.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "map_rows.h"
#include "sched.h"

namespace crdts_hip {
namespace {

using namespace maprow;  // Row<NS> and the VClock ops on it (map_rows.h)

constexpr uint32_t kMpW = 64;
constexpr uint32_t kMpComb = 128;  // combined deferred entries (<= dcap_self + dcap_other, dcap <= 64)
constexpr uint32_t kMpVals = 256;  // kept values of one key (<= mcap_self + mcap_other, mcap <= 128)

__device__ __forceinline__ void mp_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ bool set_has(const uint64_t* set, uint32_t n, uint64_t key, uint32_t lane) {
  bool f = false;
  for (uint32_t j = lane; j < n; j += kMpW) f = f || set[j] == key;
  return __ballot(f) != 0ull;
}

// VS: each key's value clock rows (both sides) are staged in LDS with one
// load per lane per side before the MVReg merge / truncate reads them (the
// launcher picks VS when mcap * A <= kVsRows on both sides); otherwise every
// row read in the dominance loops is its own dependent global load.
constexpr uint32_t kVsRows = 128;  // u64 per side
// the object's map deferred sets are staged in LDS (asked about every key)
// when both sides' fit kMdStage u64
constexpr uint32_t kMdStage = 128;

// G (the nested map's inner pass): n_obj tasks, task t merges S row tsrc[2t]
// with O row tsrc[2t + 1] into R row t; kMpNone marks an absent side (an
// empty map: merge(m, empty) = m for a canonical m), both absent: no task.
constexpr uint64_t kMpNone = ~0ull;

template <bool VS, int NS, bool G = false, int MINW = 7>
__global__ __launch_bounds__(kMpW, MINW) void map_mvreg_merge_kernel(crdt_map_mvreg_slab S, crdt_map_mvreg_slab O,
                                                               crdt_map_mvreg_slab Rout, uint64_t n_obj, uint32_t A,
                                                               int* __restrict__ status, uint32_t* __restrict__ ctl,
                                                               const uint64_t* __restrict__ tsrc = nullptr,
                                                               const uint64_t* __restrict__ Tb = nullptr) {
  __shared__ uint32_t comb[kMpComb];     // (self deferred idx + 1) | (other deferred idx + 1) << 8
  __shared__ uint32_t tk[G ? kMpComb : 1];  // G: the truncated map's deferred survivors (comb index), CLOCK ORDER
  __shared__ uint32_t vals[kMpVals];     // kept value slots of the key: side << 8 | slot
  __shared__ uint64_t vr[2][VS ? kVsRows : 1];  // the key's value clock rows: self, other
  __shared__ uint64_t md[kMdStage];             // the object's map deferred sets (when they fit)
  __shared__ uint32_t mdn[2][64];               // their sizes (dcap <= 64), self / other
  const uint32_t lane = threadIdx.x;
  // (sched.h; G: most tasks are empty slots, a plain stride balances them)
  typename std::conditional<G, GridStride, BlockTickets<4>>::type sched(n_obj, ctl + 3, lane);
  for (uint64_t i = sched.first(); i < n_obj; i = sched.next(i)) {
    const uint64_t si = G ? tsrc[2 * i] : i, oi = G ? tsrc[2 * i + 1] : i, ri = i;
    const bool hasS = !G || si != kMpNone, hasO = !G || oi != kMpNone;
    if (G && !hasS && !hasO) continue;
    // G: the merged map is then truncated by the task's row of Tb when it is
    // non-empty (Causal::truncate, src/map.rs:131-158 — the nested map's
    // removers' clock, from map_map_outer_kernel), fused into the writes below
    const Row<NS> tc = G && Tb != nullptr ? rowv<NS>(Tb, i, A, lane) : zrow<NS>();
    const bool trunc = G && Tb != nullptr && vany(tc);
    const crdt_map_mvreg_slab& R = Rout;
    const Row<NS> cS = hasS ? rowv<NS>(S.clock, si, A, lane) : zrow<NS>();
    const Row<NS> cO = hasO ? rowv<NS>(O.clock, oi, A, lane) : zrow<NS>();
    const Row<NS> cM = vmax(cS, cO);  // VClock::merge
    const uint32_t nS = hasS ? __builtin_amdgcn_readfirstlane(S.n_keys[si]) : 0u;
    const uint32_t nO = hasO ? __builtin_amdgcn_readfirstlane(O.n_keys[oi]) : 0u;
    const uint32_t dS = hasS ? __builtin_amdgcn_readfirstlane(S.n_def[si]) : 0u;
    const uint32_t dO = hasO ? __builtin_amdgcn_readfirstlane(O.n_def[oi]) : 0u;
    if (nS > S.kcap || nO > O.kcap || dS > S.dcap || dO > O.dcap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    // every value count within mcap and deferred set size within scap (the
    // loops below read mv_n / dset_n slots of the slab row as counts); lane k
    // keeps key k's value count (keys < 64), which the value-row stage below
    // reads by readlane (no dependent load on the per-key chain)
    // (and its key; lane d: map deferred entry d's set size, dcap <= 64)
    const uint32_t vnS = lane < nS ? S.mv_n[si * S.kcap + lane] : 0u, vnO = lane < nO ? O.mv_n[oi * O.kcap + lane] : 0u;
    const uint64_t kregS = lane < nS ? S.keys[si * S.kcap + lane] : 0ull;
    const uint64_t kregO = lane < nO ? O.keys[oi * O.kcap + lane] : 0ull;
    const uint32_t dnS = lane < dS ? S.dset_n[si * S.dcap + lane] : 0u, dnO = lane < dO ? O.dset_n[oi * O.dcap + lane] : 0u;
    bool bad = vnS > S.mcap || vnO > O.mcap || dnS > S.scap || dnO > O.scap;
    for (uint32_t k = lane + kMpW; k < nS; k += kMpW) bad = bad || S.mv_n[si * S.kcap + k] > S.mcap;
    for (uint32_t k = lane + kMpW; k < nO; k += kMpW) bad = bad || O.mv_n[oi * O.kcap + k] > O.mcap;
    if (__ballot(bad) != 0ull) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    // the map deferred sets (used entries) staged in LDS when they fit
    const uint32_t sS = S.scap, sO = O.scap;
    const bool st = (uint64_t)dS * sS + (uint64_t)dO * sO <= kMdStage;
    mp_sync();  // the previous object's readers of md / mdn are done
    mdn[0][lane] = dnS;
    mdn[1][lane] = dnO;
    mp_sync();
    if (st) {
      for (uint32_t e = lane; e < dS * sS; e += kMpW) {
        const uint32_t d = e / sS;
        if (e - d * sS < mdn[0][d]) md[e] = S.dset[si * S.dcap * sS + e];
      }
      for (uint32_t e = lane; e < dO * sO; e += kMpW) {
        const uint32_t d = e / sO;
        if (e - d * sO < mdn[1][d]) md[dS * sS + e] = O.dset[oi * O.dcap * sO + e];
      }
    }
    // map deferred entry d's set (x: 0 self, 1 other)
    auto dset_of = [&](uint32_t x, uint32_t d) -> const uint64_t* {
      if (x == 0u) return st ? md + d * sS : S.dset + (si * S.dcap + d) * sS;
      return st ? md + dS * sS + d * sO : O.dset + (oi * O.dcap + d) * sO;
    };
    // ---- combined deferred list: self's, plus other's that self's clock does not cover
    //      (apply_rm's deferral, against the pre-merge clock), united in CLOCK ORDER
    uint32_t nc = 0;
    {
      uint32_t a = 0, b = 0;
      while (a < dS || b < dO) {
        if (b < dO && vle(rowv<NS>(O.dclock, oi * O.dcap + b, A, lane), cS)) { ++b; continue; }
        int c;
        if (a >= dS) c = 1;
        else if (b >= dO) c = -1;
        else c = vorder(rowv<NS>(S.dclock, si * S.dcap + a, A, lane), rowv<NS>(O.dclock, oi * O.dcap + b, A, lane), lane);
        const uint32_t e = (c <= 0 ? a + 1u : 0u) | ((c >= 0 ? b + 1u : 0u) << 8);
        if (lane == 0u) comb[nc] = e;
        ++nc;
        if (c <= 0) ++a;
        if (c >= 0) ++b;
      }
    }
    mp_sync();
    // ---- entries, key by key in ascending order
    uint32_t nk = 0, a = 0, b = 0;
    bool over = false;
    while (a < nS || b < nO) {
      const uint64_t ka = a < nS ? (a < kMpW ? lane64(kregS, a) : S.keys[si * S.kcap + a]) : ~0ull;
      const uint64_t kb = b < nO ? (b < kMpW ? lane64(kregO, b) : O.keys[oi * O.kcap + b]) : ~0ull;
      const bool hs = a < nS && (b >= nO || ka <= kb), ho = b < nO && (a >= nS || kb <= ka);
      const uint64_t key = hs ? ka : kb;
      const uint64_t ia = si * S.kcap + a, ib = oi * O.kcap + b;
      const Row<NS> eS = hs ? rowv<NS>(S.eclock, ia, A, lane) : zrow<NS>();
      const Row<NS> eO = ho ? rowv<NS>(O.eclock, ib, A, lane) : zrow<NS>();
      // the key's value counts (within mcap: checked above)
      const uint32_t ms = !hs ? 0u : a < kMpW ? (uint32_t)__builtin_amdgcn_readlane(vnS, a)
                                             : (uint32_t)__builtin_amdgcn_readfirstlane(S.mv_n[ia]);
      const uint32_t mo = !ho ? 0u : b < kMpW ? (uint32_t)__builtin_amdgcn_readlane(vnO, b)
                                             : (uint32_t)__builtin_amdgcn_readfirstlane(O.mv_n[ib]);
      if (VS) {  // stage the key's used value rows: every load in flight, then the LDS stores
        const uint32_t n0 = ms * A, n1 = mo * A;
        uint64_t x0 = 0, x1 = 0, y0 = 0, y1 = 0;
        if (lane < n0) x0 = S.mv_clock[ia * S.mcap * A + lane];
        if (lane + kMpW < n0) x1 = S.mv_clock[ia * S.mcap * A + lane + kMpW];
        if (lane < n1) y0 = O.mv_clock[ib * O.mcap * A + lane];
        if (lane + kMpW < n1) y1 = O.mv_clock[ib * O.mcap * A + lane + kMpW];
        mp_sync();  // the previous key's reads of the stage are done
        if (lane < n0) vr[0][lane] = x0;
        if (lane + kMpW < n0) vr[0][lane + kMpW] = x1;
        if (lane < n1) vr[1][lane] = y0;
        if (lane + kMpW < n1) vr[1][lane + kMpW] = y1;
        mp_sync();
      }
      // value clock row v of this key on a side
      auto srow = [&](uint32_t v) -> Row<NS> {
        if (VS) return ldrow<NS>(&vr[0][v * A], A, lane);
        return rowv<NS>(S.mv_clock, ia * S.mcap + v, A, lane);
      };
      auto orow = [&](uint32_t v) -> Row<NS> {
        if (VS) return ldrow<NS>(&vr[1][v * A], A, lane);
        return rowv<NS>(O.mv_clock, ib * O.mcap + v, A, lane);
      };
      Row<NS> ec = zrow<NS>(), del = zrow<NS>();
      bool keep;
      uint32_t nv = 0;
      if (hs && !ho) {  // other has not seen it, or saw it and dropped it
        ec = vsub(eS, cO);
        keep = vany(ec);
        del = vsub(cO, ec);
        for (uint32_t v = 0; v < ms; ++v) { if (lane == 0u) vals[nv] = v; ++nv; }
        mp_sync();
      } else if (ho && !hs) {
        ec = vsub(eO, cS);
        keep = vany(ec);
        del = vsub(cS, ec);
        for (uint32_t v = 0; v < mo; ++v) { if (lane == 0u) vals[nv] = 256u | v; ++nv; }
      } else {  // in both
        const Row<NS> common = vcommon(eS, eO);  // VClock::intersection
        const Row<NS> e1 = vsub(vsub(eS, common), cO), e2 = vsub(vsub(eO, common), cS);
        const Row<NS> cm = vmax(vmax(common, e1), e2);
        keep = vany(cm);
        ec = cm;
        del = vsub(vmax(e1, e2), cm);
        // MVReg::merge (src/mvreg.rs:121-153): self's undominated, then other's undominated and new
        for (uint32_t v = 0; v < ms; ++v) {
          const Row<NS> sv = srow(v);
          bool dom = false;
          for (uint32_t w = 0; w < mo && !dom; ++w) dom = vstrict_less(sv, orow(w));
          if (!dom) { if (lane == 0u) vals[nv] = v; ++nv; }
        }
        mp_sync();
        const uint32_t nkeep_s = nv;
        for (uint32_t w = 0; w < mo; ++w) {
          const Row<NS> ov = orow(w);
          bool dom = false;
          for (uint32_t v = 0; v < ms && !dom; ++v) dom = vstrict_less(ov, srow(v));
          if (dom) continue;
          bool dup = false;
          for (uint32_t q = 0; q < nv && !dup; ++q) {
            const uint32_t sl = vals[q];
            dup = veq(q < nkeep_s ? srow(sl & 255u) : orow(sl & 255u), ov);
          }
          if (!dup) { if (lane == 0u) vals[nv] = 256u | w; ++nv; }
          mp_sync();
        }
      }
      mp_sync();
      // ---- apply_deferred on this key: every combined deferred clock naming it
      if (keep) {
        for (uint32_t c = 0; c < nc; ++c) {
          const uint32_t e = comb[c];
          const uint32_t sa = e & 255u, sb = e >> 8;
          bool named = false;
          if (sa) named = set_has(dset_of(0u, sa - 1u), mdn[0][sa - 1u], key, lane);
          if (!named && sb) named = set_has(dset_of(1u, sb - 1u), mdn[1][sb - 1u], key, lane);
          if (!named) continue;
          const Row<NS> D = sa ? rowv<NS>(S.dclock, si * S.dcap + sa - 1u, A, lane)
                               : rowv<NS>(O.dclock, oi * O.dcap + sb - 1u, A, lane);
          ec = vsub(ec, D);
          del = vmax(del, D);  // truncating by several clocks = by their max, slot by slot
        }
        keep = vany(ec);
      }
      // G: Map::truncate of the merged map — the entry clock loses tc (an
      // emptied entry is dropped) and its register is truncated by tc too
      // (subtracting del then tc = subtracting their max, slot by slot)
      if (trunc && keep) {
        ec = vsub(ec, tc);
        keep = vany(ec);
        del = vmax(del, tc);
      }
      if (keep) {
        if (nk >= R.kcap) {
          over = true;
        } else {
          const uint64_t ir = ri * R.kcap + nk;
          if (lane == 0u) R.keys[ir] = key;
          strow<NS>(R.eclock + ir * A, ec, A, lane);
          uint32_t nout = 0;
          for (uint32_t q = 0; q < nv; ++q) {  // MVReg::truncate(del), order kept
            const uint32_t sl = vals[q];
            const bool fromO = sl >= 256u;
            const uint64_t src = fromO ? ib * O.mcap + (sl & 255u) : ia * S.mcap + (sl & 255u);
            const Row<NS> r = vsub(fromO ? orow(sl & 255u) : srow(sl & 255u), del);
            if (!vany(r)) continue;
            if (nout >= R.mcap) { over = true; break; }
            strow<NS>(R.mv_clock + (ir * R.mcap + nout) * A, r, A, lane);
            if (lane == 0u) R.mv_val[ir * R.mcap + nout] = fromO ? O.mv_val[src] : S.mv_val[src];
            ++nout;
          }
          if (lane == 0u) R.mv_n[ir] = nout;  // (slots past the counts are not written: include/crdts_hip.h)
          ++nk;
        }
      }
      mp_sync();
      if (hs) ++a;
      if (ho) ++b;
    }
    if (lane == 0u) R.n_keys[ri] = nk;
    strow<NS>(R.clock + ri * A, trunc ? vsub(cM, tc) : cM, A, lane);
    auto comb_row = [&](uint32_t e) -> Row<NS> {
      const uint32_t sa = e & 255u, sb = e >> 8;
      return sa ? rowv<NS>(S.dclock, si * S.dcap + sa - 1u, A, lane) : rowv<NS>(O.dclock, oi * O.dcap + sb - 1u, A, lane);
    };
    // ---- deferred kept: the combined clocks the merged clock does not cover, sets united
    // (G, truncated: each loses tc, an emptied one is dropped, one that becomes
    // equal to an earlier survivor replaces it — the reference's HashMap
    // insert over the merge's CLOCK ORDER — and the survivors are written in
    // the CLOCK ORDER of the truncated clocks)
    uint32_t nw = nc;
    if constexpr (G) {
      if (trunc) {
        uint32_t ns = 0;
        for (uint32_t c = 0; c < nc; ++c) {
          const Row<NS> D = comb_row(comb[c]);
          if (vle(D, cM)) continue;
          const Row<NS> Dt = vsub(D, tc);
          if (!vany(Dt)) continue;
          uint32_t at = ns, pos = ns;
          for (uint32_t q = 0; q < ns; ++q) {
            const int o = vorder(Dt, vsub(comb_row(comb[tk[q]]), tc), lane);
            if (o == 0) { at = q; break; }    // equal: this (later) one replaces it
            if (o < 0 && pos == ns) pos = q;  // insertion point
          }
          mp_sync();
          if (at < ns) {
            if (lane == 0u) tk[at] = c;
          } else {
            if (lane == 0u) {
              for (uint32_t q = ns; q > pos; --q) tk[q] = tk[q - 1];
              tk[pos] = c;
            }
            ++ns;
          }
          mp_sync();
        }
        nw = ns;
      }
    }
    uint32_t nd = 0;
    for (uint32_t w = 0; w < nw; ++w) {
      const bool tl = G && trunc;
      const uint32_t e = comb[tl ? tk[w] : w];
      const uint32_t sa = e & 255u, sb = e >> 8;
      const Row<NS> D0 = comb_row(e);
      if (!tl && vle(D0, cM)) continue;
      const Row<NS> D = tl ? vsub(D0, tc) : D0;
      if (nd >= R.dcap) { over = true; break; }
      const uint64_t dr = ri * R.dcap + nd;
      strow<NS>(R.dclock + dr * A, D, A, lane);
      uint32_t cnt = 0;
      if (lane == 0u) {  // sorted union of the two key sets
        const uint64_t* xs = sa ? dset_of(0u, sa - 1u) : nullptr;
        const uint64_t* ys = sb ? dset_of(1u, sb - 1u) : nullptr;
        const uint32_t nx = sa ? mdn[0][sa - 1u] : 0u, ny = sb ? mdn[1][sb - 1u] : 0u;
        uint32_t p = 0, q = 0;
        while (p < nx || q < ny) {
          const uint64_t kx = p < nx ? xs[p] : ~0ull, ky = q < ny ? ys[q] : ~0ull;
          const uint64_t k = kx < ky ? kx : ky;
          if (kx == k) ++p;
          if (ky == k) ++q;
          if (cnt < R.scap) R.dset[dr * R.scap + cnt] = k;
          ++cnt;
        }
        R.dset_n[dr] = cnt < R.scap ? cnt : R.scap;
      }
      over = over || __builtin_amdgcn_readfirstlane(cnt) > R.scap;
      ++nd;
    }
    if (lane == 0u) R.n_def[ri] = nd;
    if (over && lane == 0u) atomicCAS(status, 0, CRDT_ECAPACITY);
    mp_sync();
  }
}

}  // namespace

int launch_map_mvreg_merge(const crdt_map_mvreg_slab& S, const crdt_map_mvreg_slab& O, const crdt_map_mvreg_slab& R,
                           uint64_t n_obj, uint32_t A, int* status, uint32_t* ctl, hipStream_t stream, int variant) {
  if (n_obj == 0) return CRDT_OK;
  if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;  // ctl[3]: tickets
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t cap = (uint64_t)cus * 28u;  // 7 single-wave blocks per SIMD
  const uint32_t blocks = (uint32_t)(n_obj < cap ? n_obj : cap);
  const bool vs = (uint64_t)S.mcap * A <= kVsRows && (uint64_t)O.mcap * A <= kVsRows;
  if (A > 64u)  // 65-128 actors: two slots per lane
    hipLaunchKernelGGL((map_mvreg_merge_kernel<false, 2>), dim3(blocks), dim3(kMpW), 0, stream, S, O, R, n_obj, A,
                       status, ctl);
  else if (vs && variant == 501)  // (diag: no register bound, 5 waves/SIMD, no spill)
    hipLaunchKernelGGL((map_mvreg_merge_kernel<true, 1, false, 1>), dim3(blocks), dim3(kMpW), 0, stream, S, O, R,
                       n_obj, A, status, ctl);
  else if (vs && variant == 502)  // (diag: 6 waves/SIMD)
    hipLaunchKernelGGL((map_mvreg_merge_kernel<true, 1, false, 6>), dim3(blocks), dim3(kMpW), 0, stream, S, O, R,
                       n_obj, A, status, ctl);
  else if (vs)
    hipLaunchKernelGGL((map_mvreg_merge_kernel<true, 1>), dim3(blocks), dim3(kMpW), 0, stream, S, O, R, n_obj, A,
                       status, ctl);
  else
    hipLaunchKernelGGL((map_mvreg_merge_kernel<false, 1>), dim3(blocks), dim3(kMpW), 0, stream, S, O, R, n_obj, A,
                       status, ctl);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

int launch_map_mvreg_merge_tasks(const crdt_map_mvreg_slab& S, const crdt_map_mvreg_slab& O,
                                 const crdt_map_mvreg_slab& R, const uint64_t* tsrc, const uint64_t* Tb,
                                 uint64_t n_tasks, uint32_t slots, uint32_t A, int* status, uint32_t* ctl,
                                 hipStream_t stream) {
  if (n_tasks == 0) return CRDT_OK;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t cap = (uint64_t)cus * 28u;
  uint32_t blocks = (uint32_t)(n_tasks < cap ? n_tasks : cap);
  // the kept keys are an object's first slots: a grid stride coprime with the
  // slots per object spreads them over every block (one sharing a factor
  // with it would leave the blocks of the last slots idle)
  auto gcd = [](uint32_t a, uint32_t b) {
    while (b) { const uint32_t t = a % b; a = b; b = t; }
    return a;
  };
  while (blocks > 1u && slots > 1u && gcd(blocks, slots) != 1u) --blocks;
  if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;
  if (A > 64u)
    hipLaunchKernelGGL((map_mvreg_merge_kernel<false, 2, true>), dim3(blocks), dim3(kMpW), 0, stream, S, O, R, n_tasks,
                       A, status, ctl, tsrc, Tb);
  else
    hipLaunchKernelGGL((map_mvreg_merge_kernel<false, 1, true>), dim3(blocks), dim3(kMpW), 0, stream, S, O, R, n_tasks,
                       A, status, ctl, tsrc, Tb);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
