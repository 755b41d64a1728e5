// Map<u64, Map<u64, MVReg<u64, A>, A>, A>::merge, batched — the reference's
// own test type (TestMap, test/map.rs:4-8); beyond SURVEY.md §8(f) rank 3.
//
// Reference: Map::merge (src/map.rs:191-268) with V = the inner map: per
// outer key the entry clocks are reconciled against both map clocks (self-only
// :198-211, both :212-237, other-only :241-250); a kept value is the inner
// maps merged (Map::merge again, for a key in both) and truncated by the clock
// of the actors that removed the entry (Map::truncate, :131-158); other's
// deferred removes are re-deferred against self's pre-merge clock (apply_rm
// :336-350), the clocks merge, and apply_deferred (:325-333) subtracts every
// deferred clock naming a key from its entry and truncates its value by it.
// Subtracts and truncations commute and compose (truncate(c1) then
// truncate(c2) = truncate(max(c1, c2)): every step is a slot-wise subtract
// with emptied rows dropped), so each kept key is truncated once, by the max
// of its removal clock and the deferred clocks naming it.
//
// Two launches, batch-parallel: (1) the outer pass, one wave per map pair
// (lane = actor slot, NS slots per lane: map_rows.h): the outer entries,
// clock and deferred removes, and per output key slot a task — which inner
// map of each side (or none) and the truncating clock; (2) the inner maps
// merged task by task (map.hip's Map<u64, MVReg> kernel in its task form: a
// missing side is the empty map, merge(m, empty) = m for a reachable m) and
// truncated by the task's clock as they are written to the output (round 5:
// no scratch inner slab and no third pass over it).
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "map_rows.h"
#include "sched.h"

namespace crdts_hip {
namespace {

using namespace maprow;

constexpr uint32_t kMmW = 64;
constexpr uint32_t kMmComb = 128;  // combined outer deferred entries (<= dcap_self + dcap_other, dcap <= 64)
constexpr uint32_t kMmStage = 128;  // u64: the map deferred sets staged per object when both sides fit
constexpr uint64_t kMmNone = ~0ull;

__device__ __forceinline__ void mm_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ bool set_has(const uint64_t* set, uint32_t n, uint64_t key, uint32_t lane) {
  bool f = false;
  for (uint32_t j = lane; j < n; j += kMmW) f = f || set[j] == key;
  return __ballot(f) != 0ull;
}

// The outer pass. Writes R's outer part and, for output slot t = i * R.kcap + k,
// tsrc[2t], tsrc[2t + 1] (the inner maps to merge: S row, O row, kMmNone when
// absent; both kMmNone for the unused slots) and Tb row t (the truncating clock).
template <int NS>
__global__ __launch_bounds__(kMmW) void map_map_outer_kernel(crdt_map_map_slab S, crdt_map_map_slab O,
                                                             crdt_map_map_slab R, uint64_t n_obj, uint32_t A,
                                                             uint64_t* __restrict__ tsrc, uint64_t* __restrict__ Tb,
                                                             int* __restrict__ status, uint32_t* __restrict__ ctl) {
  __shared__ uint32_t comb[kMmComb];  // (self deferred idx + 1) | (other deferred idx + 1) << 8
  __shared__ uint64_t md[kMmStage];    // the object's map deferred sets, used entries (when they fit)
  __shared__ uint32_t mdn[2][64];      // their sizes (dcap <= 64), self / other
  const uint32_t lane = threadIdx.x;
  BlockTickets<4> sched(n_obj, ctl + 3, lane);  // (sched.h)
  for (uint64_t i = sched.first(); i < n_obj; i = sched.next(i)) {
    const Row<NS> cS = rowv<NS>(S.clock, i, A, lane), cO = rowv<NS>(O.clock, i, A, lane);
    const Row<NS> cM = vmax(cS, cO);  // VClock::merge
    const uint32_t nS = __builtin_amdgcn_readfirstlane(S.n_keys[i]), nO = __builtin_amdgcn_readfirstlane(O.n_keys[i]);
    const uint32_t dS = __builtin_amdgcn_readfirstlane(S.n_def[i]), dO = __builtin_amdgcn_readfirstlane(O.n_def[i]);
    uint32_t nk = 0;
    bool over = false;
    if (nS > S.kcap || nO > O.kcap || dS > S.dcap || dO > O.dcap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
    } else {
      // lane k: key k (k < 64) and map deferred entry k's set size (dcap <= 64)
      const uint64_t kregS = lane < nS ? S.keys[i * S.kcap + lane] : 0ull;
      const uint64_t kregO = lane < nO ? O.keys[i * O.kcap + lane] : 0ull;
      const uint32_t dnS = lane < dS ? S.dset_n[i * S.dcap + lane] : 0u, dnO = lane < dO ? O.dset_n[i * O.dcap + lane] : 0u;
      if (__ballot(dnS > S.scap || dnO > O.scap) != 0ull) {
        if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      } else {
        // the map deferred sets staged in LDS when they fit (map.hip)
        const uint32_t sS = S.scap, sO = O.scap;
        const bool st = (uint64_t)dS * sS + (uint64_t)dO * sO <= kMmStage;
        mm_sync();  // the previous object's readers of md / mdn are done
        mdn[0][lane] = dnS;
        mdn[1][lane] = dnO;
        mm_sync();
        if (st) {
          for (uint32_t e = lane; e < dS * sS; e += kMmW) {
            const uint32_t d = e / sS;
            if (e - d * sS < mdn[0][d]) md[e] = S.dset[i * S.dcap * sS + e];
          }
          for (uint32_t e = lane; e < dO * sO; e += kMmW) {
            const uint32_t d = e / sO;
            if (e - d * sO < mdn[1][d]) md[dS * sS + e] = O.dset[i * O.dcap * sO + e];
          }
        }
        auto dset_of = [&](uint32_t x, uint32_t d) -> const uint64_t* {
          if (x == 0u) return st ? md + d * sS : S.dset + (i * S.dcap + d) * sS;
          return st ? md + dS * sS + d * sO : O.dset + (i * O.dcap + d) * sO;
        };
        // ---- combined deferred list (map.hip): self's, plus other's that self's clock does not cover
        uint32_t nc = 0;
        {
          uint32_t a = 0, b = 0;
          while (a < dS || b < dO) {
            if (b < dO && vle(rowv<NS>(O.dclock, i * O.dcap + b, A, lane), cS)) { ++b; continue; }
            int c;
            if (a >= dS) c = 1;
            else if (b >= dO) c = -1;
            else c = vorder(rowv<NS>(S.dclock, i * S.dcap + a, A, lane), rowv<NS>(O.dclock, i * O.dcap + b, A, lane),
                            lane);
            if (lane == 0u) comb[nc] = (c <= 0 ? a + 1u : 0u) | ((c >= 0 ? b + 1u : 0u) << 8);
            ++nc;
            if (c <= 0) ++a;
            if (c >= 0) ++b;
          }
        }
        mm_sync();
        // ---- entries, key by key in ascending order
        uint32_t a = 0, b = 0;
        while (a < nS || b < nO) {
          const uint64_t ka = a < nS ? (a < kMmW ? lane64(kregS, a) : S.keys[i * S.kcap + a]) : ~0ull;
          const uint64_t kb = b < nO ? (b < kMmW ? lane64(kregO, b) : O.keys[i * O.kcap + b]) : ~0ull;
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
          } else {  // in both: the inner maps merge
            const Row<NS> common = vcommon(eS, eO);  // VClock::intersection
            const Row<NS> e1 = vsub(vsub(eS, common), cO), e2 = vsub(vsub(eO, common), cS);
            ec = vmax(vmax(common, e1), e2);
            del = vsub(vmax(e1, e2), ec);
          }
          bool keep = vany(ec);
          if (keep) {  // apply_deferred on this key: every combined deferred clock naming it
            for (uint32_t c = 0; c < nc; ++c) {
              const uint32_t e = comb[c];
              const uint32_t sa = e & 255u, sb = e >> 8;
              bool named = false;
              if (sa) named = set_has(dset_of(0u, sa - 1u), mdn[0][sa - 1u], key, lane);
              if (!named && sb) named = set_has(dset_of(1u, sb - 1u), mdn[1][sb - 1u], key, lane);
              if (!named) continue;
              const Row<NS> D = sa ? rowv<NS>(S.dclock, i * S.dcap + sa - 1u, A, lane)
                                   : rowv<NS>(O.dclock, i * O.dcap + sb - 1u, A, lane);
              ec = vsub(ec, D);
              del = vmax(del, D);  // truncations compose: by their max
            }
            keep = vany(ec);
          }
          if (keep) {
            if (nk >= R.kcap) {
              over = true;
            } else {
              const uint64_t ir = i * R.kcap + nk;
              if (lane == 0u) {
                R.keys[ir] = key;
                tsrc[2 * ir] = hs ? ia : kMmNone;
                tsrc[2 * ir + 1] = ho ? ib : kMmNone;
              }
              strow<NS>(R.eclock + ir * A, ec, A, lane);
              strow<NS>(Tb + ir * A, del, A, lane);
              ++nk;
            }
          }
          if (hs) ++a;
          if (ho) ++b;
        }
        if (lane == 0u) R.n_keys[i] = nk;
        strow<NS>(R.clock + i * A, cM, A, lane);
        // ---- deferred kept: the combined clocks the merged clock does not cover, sets united
        uint32_t nd = 0;
        for (uint32_t c = 0; c < nc; ++c) {
          const uint32_t e = comb[c];
          const uint32_t sa = e & 255u, sb = e >> 8;
          const Row<NS> D = sa ? rowv<NS>(S.dclock, i * S.dcap + sa - 1u, A, lane)
                               : rowv<NS>(O.dclock, i * O.dcap + sb - 1u, A, lane);
          if (vle(D, cM)) continue;
          if (nd >= R.dcap) { over = true; break; }
          const uint64_t dr = i * R.dcap + nd;
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
        if (lane == 0u) R.n_def[i] = nd;
      }
    }
    // the slots past the kept keys hold no task (a rejected pair: none at all)
    for (uint32_t k = nk + lane; k < R.kcap; k += kMmW) {
      tsrc[2 * (i * R.kcap + k)] = kMmNone;
      tsrc[2 * (i * R.kcap + k) + 1] = kMmNone;
    }
    if (over && lane == 0u) atomicCAS(status, 0, CRDT_ECAPACITY);
    mm_sync();
  }
}

}  // namespace

size_t map_map_scratch_bytes(const crdt_map_map_slab& R, uint64_t n_obj, uint32_t A) {
  const uint64_t nt = n_obj * R.kcap;
  return 16ull * nt + 8ull * nt * A + 2u * 16u;  // tasks, truncating clocks (each 16-B aligned)
}

int launch_map_map_merge(const crdt_map_map_slab& S, const crdt_map_map_slab& O, const crdt_map_map_slab& R,
                         uint64_t n_obj, uint32_t A, uint8_t* scratch, int* status, uint32_t* ctl,
                         hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  const uint64_t nt = n_obj * R.kcap;
  // scratch: tasks [nt][2] u64, then truncating clocks [nt][A]
  uint8_t* p = scratch;
  auto take = [&](uint64_t bytes) {
    uint8_t* q = p;
    p += (bytes + 15u) & ~15ull;
    return q;
  };
  uint64_t* tsrc = (uint64_t*)take(16ull * nt);
  uint64_t* Tb = (uint64_t*)take(8ull * nt * A);
  if (hipMemsetAsync(ctl, 0, 4 * sizeof(uint32_t), stream) != hipSuccess) return CRDT_EHIP;  // ctl[3]: tickets
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t cap = (uint64_t)cus * 28u;
  const uint32_t blocks = (uint32_t)(n_obj < cap ? n_obj : cap);
  if (A > 64u)
    hipLaunchKernelGGL((map_map_outer_kernel<2>), dim3(blocks), dim3(kMmW), 0, stream, S, O, R, n_obj, A, tsrc, Tb,
                       status, ctl);
  else
    hipLaunchKernelGGL((map_map_outer_kernel<1>), dim3(blocks), dim3(kMmW), 0, stream, S, O, R, n_obj, A, tsrc, Tb,
                       status, ctl);
  if (hipGetLastError() != hipSuccess) return CRDT_EHIP;
  return launch_map_mvreg_merge_tasks(S.inner, O.inner, R.inner, tsrc, Tb, nt, R.kcap, A, status, ctl, stream);
}

}  // namespace crdts_hip
