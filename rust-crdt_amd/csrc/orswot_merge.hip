// Orswot batch join on gfx950: one wavefront per object pair.
//
// out[i] = self[i].merge(&other[i]) — CvRDT for Orswot, src/orswot.rs:87-157,
// including apply_deferred (:235-243) / apply_remove (:195-211).
//
// Per object (one wave64):
//  1. both input records are copied HBM -> LDS with 16-B loads (records are
//     16-B aligned and padded) — the only HBM reads of the object;
//  2. members: the two sorted key lists are merged by MERGE PATH, one union
//     position per lane (ties put self first, so a key present on both sides
//     is handled by the self lane and its twin lane idles). Per position the
//     lane computes the joined dot run with the reference's case rules
//     (self-only :94-104, both :105-128, other-only :132-138) and the
//     deferred-remove subtraction (:195-211), in two passes: a count pass
//     (fixes the output section offsets) and a write pass (wave ballot /
//     prefix sums give each kept member its slot and dot offset);
//  3. deferred: the union of both deferred maps keyed by clock (:141-148),
//     kept iff !(D <= merged clock) (:197); rare, done by lane 0;
//  4. the top clock is the pointwise max (:153), written by lanes < n_actors.
// The output record is written straight to its final place in HBM.
//
// Canonical record layout: include/crdts_hip.h, record_layout.h.
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "record_layout.h"

namespace crdts_hip {
namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr uint32_t kStageBytes = 2048;  // LDS staging per input record per wave
constexpr uint32_t kCache = 128;        // cached union positions per wave

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum : uint32_t { kNone = 0, kSelf = 1, kOther = 2, kBoth = 3 };

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

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

// Read-only view of one record (generic pointers; the staged path points
// into LDS and the compiler's address-space inference keeps ds_* loads).
struct View {
  const uint64_t* clk;
  const uint64_t* key;
  const uint64_t* dctr;
  const uint32_t* dact;
  const uint32_t* mdend;
  const uint64_t* fctr;
  const uint64_t* fkey;
  const uint32_t* fact;
  const uint32_t* fdend;
  const uint32_t* fmend;
  uint32_t n_mem, n_dot, n_def, n_def_dot, n_def_mem;
};

__device__ __forceinline__ View make_view(const uint8_t* rec, const RecLayout& L) {
  View v;
  v.clk = (const uint64_t*)(rec + L.o_clk);
  v.key = (const uint64_t*)(rec + L.o_key);
  v.dctr = (const uint64_t*)(rec + L.o_dctr);
  v.dact = (const uint32_t*)(rec + L.o_dact);
  v.mdend = (const uint32_t*)(rec + L.o_mdend);
  v.fctr = (const uint64_t*)(rec + L.o_fctr);
  v.fkey = (const uint64_t*)(rec + L.o_fkey);
  v.fact = (const uint32_t*)(rec + L.o_fact);
  v.fdend = (const uint32_t*)(rec + L.o_fdend);
  v.fmend = (const uint32_t*)(rec + L.o_fmend);
  v.n_mem = L.n_mem; v.n_dot = L.n_dot; v.n_def = L.n_def;
  v.n_def_dot = L.n_def_dot; v.n_def_mem = L.n_def_mem;
  return v;
}

__device__ __forceinline__ uint64_t top(const View& v, uint32_t a, uint32_t n_actors) {
  return a < n_actors ? v.clk[a] : 0ull;  // VClock::get, absent = 0 (src/vclock.rs:206-210)
}

// D[x] for deferred clock k of side v (sorted run), 0 if absent.
__device__ __forceinline__ uint64_t def_get(const View& v, uint32_t k, uint32_t x) {
  uint32_t s = k ? v.fdend[k - 1] : 0, e = v.fdend[k];
  for (uint32_t d = s; d < e; ++d) {
    uint32_t a = v.fact[d];
    if (a == x) return v.fctr[d];
    if (a > x) break;
  }
  return 0;
}

__device__ __forceinline__ bool def_has_member(const View& v, uint32_t k, uint64_t m) {
  uint32_t lo = k ? v.fmend[k - 1] : 0, hi = v.fmend[k];
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    uint64_t km = v.fkey[mid];
    if (km == m) return true;
    if (km < m) lo = mid + 1; else hi = mid;
  }
  return false;
}

// apply_deferred over the union of both deferred maps (src/orswot.rs:235-243):
// apply_remove subtracts D from entries[m] for every (D, m) — regardless of
// whether D is re-deferred — dropping dot (x, v) iff D[x] >= v
// (VClock::subtract, src/vclock.rs:236-242). Order-independent.
__device__ __forceinline__ bool killed_by_deferred(const View& L, const View& R, uint64_t m,
                                                   uint32_t x, uint64_t v) {
  for (uint32_t k = 0; k < L.n_def; ++k)
    if (def_has_member(L, k, m) && def_get(L, k, x) >= v) return true;
  for (uint32_t k = 0; k < R.n_def; ++k)
    if (def_has_member(R, k, m) && def_get(R, k, x) >= v) return true;
  return false;
}

// Merge path: candidate at union position p of the two sorted key lists
// (self first on ties). Returns type, self index i, other index j.
__device__ __forceinline__ uint32_t merge_path(const View& L, const View& R, uint32_t p,
                                               uint32_t& i, uint32_t& j) {
  uint32_t nL = L.n_mem, nR = R.n_mem;
  uint32_t lo = p > nR ? p - nR : 0, hi = p < nL ? p : nL;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (L.key[mid] <= R.key[p - 1 - mid]) lo = mid + 1; else hi = mid;
  }
  i = lo;
  j = p - lo;
  if (i < nL && (j >= nR || L.key[i] <= R.key[j])) {
    return (j < nR && L.key[i] == R.key[j]) ? kBoth : kSelf;
  }
  if (i > 0 && L.key[i - 1] == R.key[j]) return kNone;  // twin of a kBoth at p-1
  return kOther;
}

// Joined dot run of one member, emitted in actor order: emit(actor, counter).
// Rules: src/orswot.rs:94-104 (self-only), :105-128 (both), :132-138 (other-only);
// then the deferred subtraction. Lc/Rc are the PRE-merge top clocks.
template <class Emit>
__device__ __forceinline__ void join_member(uint32_t type, uint32_t i, uint32_t j, const View& L,
                                            const View& R, uint32_t n_actors, bool has_def,
                                            Emit&& emit) {
  uint64_t m = type == kOther ? R.key[j] : L.key[i];
  auto out = [&](uint32_t x, uint64_t v) {
    if (!has_def || !killed_by_deferred(L, R, m, x, v)) emit(x, v);
  };
  if (type == kSelf) {
    // keep the entry UNCHANGED iff !(clock <= other.clock)  (:98-103)
    uint32_t s = i ? L.mdend[i - 1] : 0, e = L.mdend[i];
    bool le = true;
    for (uint32_t d = s; d < e; ++d)
      if (L.dctr[d] > top(R, L.dact[d], n_actors)) { le = false; break; }
    if (!le)
      for (uint32_t d = s; d < e; ++d) out(L.dact[d], L.dctr[d]);
  } else if (type == kOther) {
    // clock.subtract(&self.clock); keep dots with R[x] > Lc[x]  (:133)
    uint32_t s = j ? R.mdend[j - 1] : 0, e = R.mdend[j];
    for (uint32_t d = s; d < e; ++d) {
      uint32_t x = R.dact[d];
      uint64_t v = R.dctr[d];
      if (v > top(L, x, n_actors)) out(x, v);
    }
  } else {
    // common = intersection; (L - common) - Rc; (R - common) - Lc; max of all (:109-116)
    uint32_t a = i ? L.mdend[i - 1] : 0, ae = L.mdend[i];
    uint32_t b = j ? R.mdend[j - 1] : 0, be = R.mdend[j];
    while (a < ae || b < be) {
      uint32_t xa = a < ae ? L.dact[a] : 0xFFFFFFFFu;
      uint32_t xb = b < be ? R.dact[b] : 0xFFFFFFFFu;
      if (xa < xb) {
        uint64_t v = L.dctr[a++];
        if (v > top(R, xa, n_actors)) out(xa, v);
      } else if (xb < xa) {
        uint64_t v = R.dctr[b++];
        if (v > top(L, xb, n_actors)) out(xb, v);
      } else {
        uint64_t va = L.dctr[a++], vb = R.dctr[b++];
        if (va == vb) {
          out(xa, va);
        } else {
          uint64_t lp = va > top(R, xa, n_actors) ? va : 0;
          uint64_t rp = vb > top(L, xa, n_actors) ? vb : 0;
          uint64_t mx = lp > rp ? lp : rp;
          if (mx) out(xa, mx);
        }
      }
    }
  }
}

__device__ __forceinline__ uint32_t count_member(uint32_t type, uint32_t i, uint32_t j, const View& L,
                                                 const View& R, uint32_t n_actors, bool has_def) {
  if (type == kNone) return 0;
  uint32_t c = 0;
  join_member(type, i, j, L, R, n_actors, has_def, [&](uint32_t, uint64_t) { ++c; });
  return c;
}

// CLOCK ORDER compare of deferred clock k of X with deferred clock l of Y.
__device__ __forceinline__ int clock_cmp(const View& X, uint32_t k, const View& Y, uint32_t l) {
  uint32_t a = k ? X.fdend[k - 1] : 0, ae = X.fdend[k];
  uint32_t b = l ? Y.fdend[l - 1] : 0, be = Y.fdend[l];
  for (; a < ae && b < be; ++a, ++b) {
    uint32_t xa = X.fact[a], xb = Y.fact[b];
    if (xa != xb) return xa < xb ? -1 : 1;
    uint64_t va = X.fctr[a], vb = Y.fctr[b];
    if (va != vb) return va < vb ? -1 : 1;
  }
  if (a == ae && b == be) return 0;
  return a == ae ? -1 : 1;
}

// !(D <= merged clock): some dot of D exceeds max(Lc, Rc)  (src/orswot.rs:197)
__device__ __forceinline__ bool def_survives(const View& X, uint32_t k, const View& L, const View& R,
                                             uint32_t n_actors) {
  uint32_t s = k ? X.fdend[k - 1] : 0, e = X.fdend[k];
  for (uint32_t d = s; d < e; ++d) {
    uint32_t x = X.fact[d];
    uint64_t lc = top(L, x, n_actors), rc = top(R, x, n_actors);
    if (X.fctr[d] > (lc > rc ? lc : rc)) return true;
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
// single lane. If `w` is null only counts.
__device__ void deferred_pass(const View& L, const View& R, uint32_t n_actors, uint32_t& nd,
                              uint32_t& ndd, uint32_t& ndm, const DefOut* w) {
  uint32_t k = 0, l = 0;
  nd = ndd = ndm = 0;
  while (k < L.n_def || l < R.n_def) {
    int c = k >= L.n_def ? 1 : (l >= R.n_def ? -1 : clock_cmp(L, k, R, l));
    const View& X = c <= 0 ? L : R;
    uint32_t kx = c <= 0 ? k : l;
    if (def_survives(X, kx, L, R, n_actors)) {
      uint32_t s = kx ? X.fdend[kx - 1] : 0, e = X.fdend[kx];
      for (uint32_t d = s; d < e; ++d) {
        if (w) { w->fact[ndd] = X.fact[d]; w->fctr[ndd] = X.fctr[d]; }
        ++ndd;
      }
      // member set: self's, other's, or the sorted union of both (c == 0)
      uint32_t a = 0, ae = 0, b = 0, be = 0;
      if (c <= 0) { a = k ? L.fmend[k - 1] : 0; ae = L.fmend[k]; }
      if (c >= 0) { b = l ? R.fmend[l - 1] : 0; be = R.fmend[l]; }
      while (a < ae || b < be) {
        uint64_t ka = a < ae ? L.fkey[a] : ~0ull, kb = b < be ? R.fkey[b] : ~0ull;
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

// Merge one pair; Lr/Rr point at the (staged or global) input records.
__device__ __forceinline__ void merge_pair(const uint8_t* Lr, const RecLayout& LL, const uint8_t* Rr,
                                           const RecLayout& RL, uint8_t* O, uint32_t n_actors,
                                           uint32_t* cid, uint16_t* ccnt, uint32_t lane) {
  const View L = make_view(Lr, LL);
  const View R = make_view(Rr, RL);
  const bool has_def = (L.n_def | R.n_def) != 0;
  const uint32_t P = L.n_mem + R.n_mem;

  // ---- pass 1: per-position join counts -> output member/dot totals
  uint32_t tot_mem = 0, tot_dot = 0;
  for (uint32_t base = 0; base < P; base += kWave) {
    uint32_t p = base + lane;
    uint32_t cnt = 0, type = kNone, i = 0, j = 0;
    if (p < P) {
      type = merge_path(L, R, p, i, j);
      cnt = count_member(type, i, j, L, R, n_actors, has_def);
      if (p < kCache) { cid[p] = (type << 30) | (i << 15) | j; ccnt[p] = (uint16_t)cnt; }
    }
    tot_mem += (uint32_t)__popcll(__ballot(cnt > 0));
    tot_dot += wave_sum(cnt);
  }

  // ---- deferred counts (lane 0, rare) and output layout
  uint32_t nd = 0, ndd = 0, ndm = 0;
  if (has_def) {
    if (lane == 0) deferred_pass(L, R, n_actors, nd, ndd, ndm, nullptr);
    nd = __shfl(nd, 0, kWave);
    ndd = __shfl(ndd, 0, kWave);
    ndm = __shfl(ndm, 0, kWave);
  }
  RecLayout OL;
  rec_layout(OL, n_actors, tot_mem, tot_dot, nd, ndd, ndm);
  uint64_t* okey = (uint64_t*)(O + OL.o_key);
  uint64_t* odctr = (uint64_t*)(O + OL.o_dctr);
  uint32_t* odact = (uint32_t*)(O + OL.o_dact);
  uint32_t* omdend = (uint32_t*)(O + OL.o_mdend);

  // ---- top clock: pointwise max (src/orswot.rs:153, src/vclock.rs:131-137)
  uint64_t* oclk = (uint64_t*)(O + OL.o_clk);
  for (uint32_t a = lane; a < n_actors; a += kWave) {
    uint64_t x = L.clk[a], y = R.clk[a];
    oclk[a] = x > y ? x : y;
  }

  // ---- pass 2: write kept members and their joined dots
  uint32_t mem_base = 0, dot_base = 0;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (uint32_t base = 0; base < P; base += kWave) {
    uint32_t p = base + lane;
    uint32_t cnt = 0, type = kNone, i = 0, j = 0;
    if (p < P) {
      if (p < kCache) {
        uint32_t c = cid[p];
        type = c >> 30; i = (c >> 15) & 0x7FFFu; j = c & 0x7FFFu;
        cnt = ccnt[p];
      } else {
        type = merge_path(L, R, p, i, j);
        cnt = count_member(type, i, j, L, R, n_actors, has_def);
      }
    }
    uint64_t keep = __ballot(cnt > 0);
    uint32_t incl = wave_incl_scan(cnt, lane);
    if (cnt > 0) {
      uint32_t midx = mem_base + (uint32_t)__popcll(keep & lt_mask);
      uint32_t d = dot_base + incl - cnt;
      okey[midx] = type == kOther ? R.key[j] : L.key[i];
      join_member(type, i, j, L, R, n_actors, has_def, [&](uint32_t x, uint64_t v) {
        odact[d] = x;
        odctr[d] = v;
        ++d;
      });
      omdend[midx] = d;
    }
    mem_base += (uint32_t)__popcll(keep);
    dot_base += __shfl(incl, kWave - 1, kWave);
  }

  if (lane == 0) {
    if (OL.o_def != OL.o_mpad) *(uint32_t*)(O + OL.o_mpad) = 0u;  // member-block pad
    if (has_def) {
      DefOut w;
      w.fctr = (uint64_t*)(O + OL.o_fctr);
      w.fkey = (uint64_t*)(O + OL.o_fkey);
      w.fact = (uint32_t*)(O + OL.o_fact);
      w.fdend = (uint32_t*)(O + OL.o_fdend);
      w.fmend = (uint32_t*)(O + OL.o_fmend);
      deferred_pass(L, R, n_actors, nd, ndd, ndm, &w);
    }
    for (uint32_t b = OL.o_end; b < OL.size; b += 4) *(uint32_t*)(O + b) = 0u;  // record pad
    uint4* h = (uint4*)O;
    h[0] = make_uint4(OL.size, n_actors, tot_mem, tot_dot);
    h[1] = make_uint4(nd, ndd, ndm, 0u);
  }
}

__device__ __forceinline__ bool read_layout(const uint8_t* rec, uint64_t avail, uint32_t n_actors,
                                            RecLayout& L) {
  const uint4* h = (const uint4*)rec;
  uint4 a = h[0], b = h[1];
  rec_layout(L, a.y, a.z, a.w, b.x, b.y, b.z);
  return a.x == L.size && a.y == n_actors && b.w == 0u && (uint64_t)L.size <= avail;
}

// Copy one record (size multiple of 16) into LDS: loads first, then stores.
__device__ __forceinline__ void stage_record(u32x4* dst, const u32x4* src, uint32_t n16, uint32_t lane) {
  constexpr uint32_t kPer = kStageBytes / 16 / kWave;  // 16-B chunks per lane
  u32x4 r[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    uint32_t idx = lane + k * kWave;
    if (idx < n16) r[k] = __builtin_nontemporal_load(src + idx);
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    uint32_t idx = lane + k * kWave;
    if (idx < n16) dst[idx] = r[k];
  }
}

__global__ __launch_bounds__(kWave * kWavesPerBlock) void orswot_merge_kernel(
    const uint8_t* __restrict__ Lb, const uint64_t* __restrict__ Loff, uint64_t Lbytes,
    const uint8_t* __restrict__ Rb, const uint64_t* __restrict__ Roff, uint64_t Rbytes,
    uint8_t* __restrict__ Ob, uint64_t* __restrict__ Ooff, uint64_t Obytes, uint64_t n_obj,
    uint32_t n_actors, int* __restrict__ status) {
  __shared__ u32x4 stage[kWavesPerBlock][2][kStageBytes / 16];
  __shared__ uint32_t cid_s[kWavesPerBlock][kCache];
  __shared__ uint16_t ccnt_s[kWavesPerBlock][kCache];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wave = threadIdx.x / kWave;
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t obj = (uint64_t)blockIdx.x * kWavesPerBlock + wave; obj < n_obj; obj += stride) {
    const uint64_t lo = Loff[obj], ro = Roff[obj];
    const uint64_t oo = lo + ro;
    if (lane == 0) Ooff[obj] = oo;
    RecLayout LL, RL;
    bool ok = lo + kHdrBytes <= Lbytes && ro + kHdrBytes <= Rbytes && ((lo | ro) & 15u) == 0;
    ok = ok && read_layout(Lb + lo, Lbytes - lo, n_actors, LL) &&
         read_layout(Rb + ro, Rbytes - ro, n_actors, RL);
    ok = ok && oo + (uint64_t)LL.size + RL.size <= Obytes;
    if (!ok) {
      if (lane == 0) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    if (LL.size <= kStageBytes && RL.size <= kStageBytes) {
      stage_record(stage[wave][0], (const u32x4*)(Lb + lo), LL.size / 16, lane);
      stage_record(stage[wave][1], (const u32x4*)(Rb + ro), RL.size / 16, lane);
      wave_sync();
      merge_pair((const uint8_t*)stage[wave][0], LL, (const uint8_t*)stage[wave][1], RL, Ob + oo,
                 n_actors, cid_s[wave], ccnt_s[wave], lane);
      wave_sync();
    } else {
      merge_pair(Lb + lo, LL, Rb + ro, RL, Ob + oo, n_actors, cid_s[wave], ccnt_s[wave], lane);
      wave_sync();
    }
  }
}

}  // namespace

int launch_orswot_merge(const uint8_t* Lb, const uint64_t* Loff, uint64_t Lbytes, const uint8_t* Rb,
                        const uint64_t* Roff, uint64_t Rbytes, uint8_t* Ob, uint64_t* Ooff,
                        uint64_t Obytes, uint64_t n_obj, uint32_t n_actors, int* status,
                        hipStream_t stream, int blocks_per_cu) {
  if (n_obj == 0) return CRDT_OK;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  uint64_t want = (n_obj + kWavesPerBlock - 1) / kWavesPerBlock;
  uint64_t cap = (uint64_t)cus * (blocks_per_cu > 0 ? blocks_per_cu : 8);
  uint32_t blocks = (uint32_t)(want < cap ? want : cap);
  hipLaunchKernelGGL(orswot_merge_kernel, dim3(blocks), dim3(kWave * kWavesPerBlock), 0, stream,
                     Lb, Loff, Lbytes, Rb, Roff, Rbytes, Ob, Ooff, Obytes, n_obj, n_actors, status);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
