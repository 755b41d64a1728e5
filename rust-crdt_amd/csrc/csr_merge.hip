// Sparse (CSR) VClock / GCounter / PNCounter join, batched (SURVEY.md §8(a)
// rows A2 and A6 for large actor universes; include/crdts_hip.h "Sparse
// clocks and counters").
//
// The reference clock is a BTreeMap<A, u64> over any actor universe
// (src/vclock.rs:54-57); VClock::merge (:131-137) witnesses every (actor,
// counter) of `other` (:159-163: keep the larger, never store 0), i.e. the
// sorted union of the two actor runs with counters max'ed. GCounter::merge
// (src/gcounter.rs:58-62) delegates to it; PNCounter::merge
// (src/pncounter.rs:90-95) is the same on P and on N. A clock here is a run
// of entries (u32 actor strictly increasing, u64 counter > 0); object i's run
// is [off[i], off[i] + len[i]) of the batch's act / ctr arrays.
//
// One wave per object, a resident grid; a wave takes chunks of 64 objects
// (lane k <-> object c + k: offsets, lengths and the placement checks in one
// coalesced step) and joins them one by one with the NEXT object's two runs
// in flight in registers. The join of runs of <= 64 entries is loop-free:
// lane k holds self entry k and other entry k; every entry finds its rank in
// the other run by a 6-step binary search over the other run's actors held
// in registers (ds_bpermute), equal actors meet (self first), and the union
// position of an entry is its index + its rank - the equal pairs before it
// (mbcnt of the ballot) — the same rank arithmetic as the Orswot member
// alignment. Longer runs take a chunked loop with binary searches in HBM.
// Output record i is written at self.off[i] + other.off[i] (a union is never
// longer than its two runs), so the output needs no scan and is itself a
// valid (gapped) input batch. HBM-bound: 12 B per entry read per side, 12 B
// per union entry written, + 3 x (8 + 4) B of offsets / lengths per object.
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"

namespace crdts_hip {
namespace {

constexpr uint32_t kW = 64;
constexpr uint32_t kBlock = 256;

struct CsrJob {
  const uint64_t* so;
  const uint32_t* sl;
  const uint32_t* sa;
  const uint64_t* sc;
  uint64_t s_entries;
  const uint64_t* oo;
  const uint32_t* ol;
  const uint32_t* oa;
  const uint64_t* oc;
  uint64_t o_entries;
  uint64_t* out_off;
  uint32_t* out_len;
  uint32_t* out_act;
  uint64_t* out_ctr;
  uint64_t out_entries;
  uint64_t n;
};

__device__ __forceinline__ uint32_t rd32(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ uint64_t rd64(uint64_t v, uint32_t src) {
  return ((uint64_t)rd32((uint32_t)(v >> 32), src) << 32) | rd32((uint32_t)v, src);
}
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, uint32_t l) {
  return ((uint64_t)lane_u32((uint32_t)(v >> 32), l) << 32) | lane_u32((uint32_t)v, l);
}
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// lane k's value moved to lane k + 1 (lane 0 gets 0): DPP wave_shr:1
__device__ __forceinline__ uint32_t from_below(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// # of the first n actors held by lanes [0, n) of `a` that are < x
// (n <= 64; lanes past n are never probed): 6-step binary lifting.
__device__ __forceinline__ uint32_t rank_regs(uint32_t a, uint32_t n, uint32_t x) {
  uint32_t b = 0;
#pragma unroll
  for (uint32_t step = 32u; step; step >>= 1) {
    const uint32_t c = b + step;  // candidate count: probe element c - 1
    const uint32_t p = rd32(a, (c - 1u) & 63u);
    b = (c <= n && p < x) ? c : b;
  }
  const uint32_t c = b + 1u;  // the last step (element b) as one more probe
  const uint32_t p = rd32(a, b & 63u);
  return (c <= n && p < x) ? c : b;
}

// # of entries of the sorted run a[0, n) (in HBM) below x.
__device__ __forceinline__ uint64_t rank_mem(const uint32_t* a, uint64_t n, uint32_t x) {
  uint64_t lo = 0, len = n;
  while (len) {
    const uint64_t half = len >> 1;
    if (a[lo + half] < x) {
      lo += half + 1u;
      len -= half + 1u;
    } else {
      len = half;
    }
  }
  return lo;
}

__device__ __forceinline__ void fail(int* status, int code) { atomicCAS(status, 0, code); }

// Runs longer than 64 entries: 64-entry chunks of each side, each entry's
// rank in the other run by binary search in HBM. Returns the union length,
// or ~0u for a non-canonical run (nothing more is written).
__device__ uint32_t join_long(const CsrJob& J, uint64_t s0, uint32_t ns, uint64_t o0, uint32_t no, uint64_t ob,
                              uint32_t lane) {
  const uint32_t* sa = J.sa + s0;
  const uint64_t* sc = J.sc + s0;
  const uint32_t* oa = J.oa + o0;
  const uint64_t* oc = J.oc + o0;
  bool bad = false;
  uint32_t eq_before = 0;
  for (uint32_t base = 0; base < ns; base += kW) {  // self entries: every one is written
    const uint32_t k = base + lane;
    const bool h = k < ns;
    const uint32_t a = h ? sa[k] : 0u;
    const uint64_t c = h ? sc[k] : 1ull;
    bad = bad || (h && (c == 0ull || (k && sa[k - 1u] >= a)));
    const uint64_t r = h ? rank_mem(oa, no, a) : 0ull;
    const bool eq = h && r < no && oa[r] == a;
    const uint64_t E = __ballot(eq);
    const uint64_t v = eq ? (oc[r] > c ? oc[r] : c) : c;
    const uint64_t pos = k + r - (eq_before + mbcnt(E));
    eq_before += (uint32_t)__popcll(E);
    if (h) {
      J.out_act[ob + pos] = a;
      J.out_ctr[ob + pos] = v;
    }
  }
  uint32_t eqo_before = 0;
  for (uint32_t base = 0; base < no; base += kW) {  // other entries not met by a self entry
    const uint32_t k = base + lane;
    const bool h = k < no;
    const uint32_t a = h ? oa[k] : 0u;
    const uint64_t c = h ? oc[k] : 1ull;
    bad = bad || (h && (c == 0ull || (k && oa[k - 1u] >= a)));
    const uint64_t r = h ? rank_mem(sa, ns, a) : 0ull;
    const bool eq = h && r < ns && sa[r] == a;
    const uint64_t E = __ballot(eq);
    const uint64_t pos = k + r - (eqo_before + mbcnt(E));
    eqo_before += (uint32_t)__popcll(E);
    if (h && !eq) {
      J.out_act[ob + pos] = a;
      J.out_ctr[ob + pos] = c;
    }
  }
  if (__ballot(bad)) return ~0u;
  return ns + no - eq_before;
}

// One chunk of 64 objects of job J (lane k <-> object c0 + k).
__device__ __forceinline__ void merge_chunk(const CsrJob& J, uint64_t c0, uint32_t lane, int* status) {
  {
    // ---- chunk state: lane k <-> object c0 + k
    const uint64_t i = c0 + lane;
    const bool valid = i < J.n;
    uint64_t so = 0, oo = 0;
    uint32_t sl = 0, ol = 0;
    if (valid) {
      so = J.so[i];
      oo = J.oo[i];
      sl = J.sl[i];
      ol = J.ol[i];
    }
    // placement precondition: runs of each side in increasing, non-overlapping
    // offset order (the next object's run starts at or after this one's end)
    uint64_t nso = rd64(so, (lane + 1u) & 63u), noo = rd64(oo, (lane + 1u) & 63u);
    if (lane == kW - 1u && i + 1u < J.n) {
      nso = J.so[i + 1u];
      noo = J.oo[i + 1u];
    }
    const bool has_next = i + 1u < J.n;
    const bool inb = so + sl <= J.s_entries && oo + ol <= J.o_entries && so <= J.s_entries && oo <= J.o_entries &&
                     so + oo + sl + ol <= J.out_entries;
    const bool placed = !has_next || (nso >= so + sl && noo >= oo + ol);
    if (__ballot(valid && !placed) && lane == 0u) fail(status, CRDT_EINVAL);
    if (__ballot(valid && !inb) && lane == 0u) fail(status, CRDT_EINVAL);
    const bool ok = valid && placed && inb;
    const uint64_t run = __ballot(ok);
    uint32_t myU = 0u;  // this lane's object's union length (written after the chunk)

    // ---- the chunk's objects one by one, the next one's runs in flight
    uint64_t pend = run;
    uint32_t t = pend ? (uint32_t)__builtin_ctzll(pend) : 0u;
    uint32_t pa = 0u, qa = 0u;
    uint64_t pc = 1ull, qc = 1ull;
    if (pend) {
      const uint32_t ns = lane_u32(sl, t), no = lane_u32(ol, t);
      const uint64_t s0 = lane_u64(so, t), o0 = lane_u64(oo, t);
      if (lane < ns && ns <= kW) { pa = J.sa[s0 + lane]; pc = J.sc[s0 + lane]; }
      if (lane < no && no <= kW) { qa = J.oa[o0 + lane]; qc = J.oc[o0 + lane]; }
    }
    while (pend) {
      t = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1u;
      const uint32_t ns = lane_u32(sl, t), no = lane_u32(ol, t);
      const uint64_t s0 = lane_u64(so, t), o0 = lane_u64(oo, t);
      const uint64_t ob = s0 + o0;
      const uint32_t a = pa, b = qa;
      const uint64_t c = pc, d = qc;
      if (pend) {  // the next object's runs
        const uint32_t u = (uint32_t)__builtin_ctzll(pend);
        const uint32_t nsu = lane_u32(sl, u), nou = lane_u32(ol, u);
        const uint64_t su = lane_u64(so, u), ou = lane_u64(oo, u);
        pa = 0u; qa = 0u; pc = 1ull; qc = 1ull;
        if (lane < nsu && nsu <= kW) { pa = J.sa[su + lane]; pc = J.sc[su + lane]; }
        if (lane < nou && nou <= kW) { qa = J.oa[ou + lane]; qc = J.oc[ou + lane]; }
      }
      uint32_t U;
      if (ns <= kW && no <= kW) {
        const bool hs = lane < ns, ho = lane < no;
        // canonical runs: actors strictly increasing, counters > 0
        const uint32_t ap = from_below(a), bp = from_below(b);
        const bool bad = (hs && (c == 0ull || (lane && ap >= a))) || (ho && (d == 0ull || (lane && bp >= b)));
        // (every lane runs the searches: ds_bpermute sources must be active lanes)
        const uint32_t rs0 = rank_regs(b, no, a), ro0 = rank_regs(a, ns, b);
        const uint32_t rs = hs ? rs0 : 0u;  // # other actors below my self actor
        const uint32_t ro = ho ? ro0 : 0u;  // # self actors below my other actor
        const uint32_t bs = rd32(b, rs & 63u), as = rd32(a, ro & 63u);
        const uint64_t dv = rd64(d, rs & 63u);
        const bool eqs = hs && rs < no && bs == a;
        const bool eqo = ho && ro < ns && as == b;
        const uint64_t ES = __ballot(eqs), EO = __ballot(eqo);
        U = ns + no - (uint32_t)__popcll(ES);
        if (__ballot(bad)) {
          U = 0u;
          if (lane == 0u) fail(status, CRDT_ENONCANON);
        } else {
          const uint32_t ps = lane + rs - mbcnt(ES), po = lane + ro - mbcnt(EO);
          if (hs) {  // VClock::witness: the larger counter (src/vclock.rs:159-163)
            J.out_act[ob + ps] = a;
            J.out_ctr[ob + ps] = eqs && dv > c ? dv : c;
          }
          if (ho && !eqo) {
            J.out_act[ob + po] = b;
            J.out_ctr[ob + po] = d;
          }
        }
      } else {
        U = join_long(J, s0, ns, o0, no, ob, lane);
        if (U == ~0u) {
          U = 0u;
          if (lane == 0u) fail(status, CRDT_ENONCANON);
        }
      }
      myU = lane == t ? U : myU;
    }
    if (valid) {
      J.out_off[i] = so + oo;
      J.out_len[i] = ok ? myU : 0u;
    }
  }
}

__global__ __launch_bounds__(kBlock) void clock_csr_merge_kernel(CsrJob J, uint64_t chunks, int* status) {
  const uint32_t lane = threadIdx.x & (kW - 1u);
  const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / kW) + threadIdx.x / kW;
  const uint64_t n_waves = (uint64_t)gridDim.x * (kBlock / kW);
  for (uint64_t ch = wave; ch < chunks; ch += n_waves) merge_chunk(J, ch * kW, lane, status);
}

}  // namespace

int launch_clock_csr_merge(const crdt_clock_csr* const* self, const crdt_clock_csr* const* other,
                           const crdt_clock_csr_out* const* out, int n_jobs, int* status, hipStream_t stream) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  for (int k = 0; k < n_jobs; ++k) {  // PNCounter: P, then N (independent joins, one stream)
    const CsrJob J{self[k]->off, self[k]->len, self[k]->act, self[k]->ctr, self[k]->n_entries,
                   other[k]->off, other[k]->len, other[k]->act, other[k]->ctr, other[k]->n_entries,
                   out[k]->off, out[k]->len, out[k]->act, out[k]->ctr, out[k]->n_entries, self[k]->n_obj};
    const uint64_t chunks = (self[k]->n_obj + kW - 1) / kW;
    if (chunks == 0) continue;
    const uint64_t want = (chunks + kBlock / kW - 1) / (kBlock / kW);
    const uint64_t cap = (uint64_t)cus * 8;  // 8 blocks of 4 waves per CU: 32 waves
    const uint32_t blocks = (uint32_t)(want < cap ? want : cap);
    hipLaunchKernelGGL(clock_csr_merge_kernel, dim3(blocks), dim3(kBlock), 0, stream, J, chunks, status);
    if (hipGetLastError() != hipSuccess) return CRDT_EHIP;
  }
  return CRDT_OK;
}

}  // namespace crdts_hip
