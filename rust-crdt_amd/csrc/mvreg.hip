// MVReg merge and VClock partial order, batched.
//
// VClock `partial_cmp` (src/vclock.rs:59-71) over dense rows (0 = absent):
// Equal when the rows are equal, Greater when other <= self pointwise, Less
// when self <= other pointwise, else None (incomparable). Encoded as
// 0 / 1 / -1 / 2 (crdt_vclock_partial_cmp).
//
// MVReg<V, A>::merge (src/mvreg.rs:121-153), V = u64: self's values that no
// other value strictly dominates (`clock < c`), then other's values that no
// self value strictly dominates and whose clock is not already kept; order
// kept. "Not already kept" needs no sequential scan: an earlier equal clock on
// the other side is either kept (then this one is a duplicate) or dropped for
// a reason that drops this one too.
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"

namespace crdts_hip {
namespace {

constexpr uint32_t kMW = 64;

__device__ __forceinline__ void mv_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// G lanes per pair (G = power of two <= 64); each lane compares a strided
// share of the A slots, the group's flags are combined from two ballots.
__global__ __launch_bounds__(256) void vclock_cmp_kernel(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                         uint64_t n, uint32_t A, uint32_t G, int8_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & (kMW - 1u);
  const uint32_t per_wave = kMW / G, g = lane / G, gl = lane % G;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / kMW) + threadIdx.x / kMW;
  const uint64_t n_waves = (uint64_t)gridDim.x * (blockDim.x / kMW);
  for (uint64_t base = wave * per_wave; base < n; base += n_waves * per_wave) {
    const uint64_t i = base + g;
    bool gt = false, lt = false;
    if (i < n) {
      const uint64_t* ra = a + i * A;
      const uint64_t* rb = b + i * A;
      for (uint32_t x = gl; x < A; x += G) {
        const uint64_t va = ra[x], vb = rb[x];
        gt = gt || va > vb;
        lt = lt || va < vb;
      }
    }
    const uint64_t GT = __ballot(gt), LT = __ballot(lt);
    const uint64_t gm = (G == 64u ? ~0ull : ((1ull << G) - 1ull)) << (g * G);
    if (gl == 0u && i < n) {
      const bool anygt = (GT & gm) != 0ull, anylt = (LT & gm) != 0ull;
      out[i] = (int8_t)(!anygt && !anylt ? 0 : !anylt ? 1 : !anygt ? -1 : 2);
    }
  }
}

// One wave per object, W waves per block, each with its own LDS region
// (dynamic shared memory, `per_wave` bytes: the self / other clock rows, the
// S x O and O x O flag matrices, the output slot table). Output rows are
// written slot-major in one coalesced pass: lane l of the wave writes u64
// l, l + 64, ... of the object's [outcap][A] block, its source row read from
// the slot table (kept self rows first, then kept other rows, order kept).
__global__ __launch_bounds__(256) void mvreg_merge_kernel(
    const uint32_t* __restrict__ sn, const uint64_t* __restrict__ sclk, const uint64_t* __restrict__ sval, uint32_t scap,
    const uint32_t* __restrict__ on, const uint64_t* __restrict__ oclk, const uint64_t* __restrict__ oval, uint32_t ocap,
    uint32_t* __restrict__ outn, uint64_t* __restrict__ outclk, uint64_t* __restrict__ outval, uint32_t outcap,
    uint64_t n_obj, uint32_t A, uint32_t per_wave, int* __restrict__ status) {
  extern __shared__ uint64_t mv_s[];
  const uint32_t lane = threadIdx.x & (kMW - 1u), wave = threadIdx.x / kMW, W = blockDim.x / kMW;
  uint64_t* S = mv_s + (size_t)wave * (per_wave / 8u);
  uint64_t* O = S + (size_t)scap * A;
  uint8_t* fso = (uint8_t*)(O + (size_t)ocap * A);  // [scap][ocap]
  uint8_t* foo = fso + scap * ocap;                   // [ocap][ocap]
  uint8_t* tab = foo + ocap * ocap;                   // [outcap]: output slot -> source row (64 + j: other j)
  const uint32_t AO = outcap * A;
  // Software pipeline: the next register pair's slot counts and the first 64
  // u64 of each side's clock slab (every capacity slot, used or not: the
  // count is not known yet) are loaded while this pair is merged.
  const uint64_t stride = (uint64_t)gridDim.x * W;
  const uint32_t pfS = scap * A < kMW ? scap * A : kMW, pfO = ocap * A < kMW ? ocap * A : kMW;
  uint32_t nsn = 0, non = 0;
  uint64_t nS = 0, nO = 0, nVs = 0, nVo = 0;  // clock elements; values (lane < cap)
  uint64_t o = (uint64_t)blockIdx.x * W + wave;
  if (o < n_obj) {
    nsn = sn[o];
    non = on[o];
    if (lane < scap) nVs = sval[o * scap + lane];
    if (lane < ocap) nVo = oval[o * ocap + lane];
    if (lane < pfS) nS = sclk[o * scap * A + lane];
    if (lane < pfO) nO = oclk[o * ocap * A + lane];
  }
  for (; o < n_obj; o += stride) {
    const uint32_t ns = __builtin_amdgcn_readfirstlane(nsn), no = __builtin_amdgcn_readfirstlane(non);
    const uint64_t cS = nS, cO = nO, cVs = nVs, cVo = nVo;
    if (o + stride < n_obj) {
      const uint64_t u = o + stride;
      nsn = sn[u];
      non = on[u];
      if (lane < scap) nVs = sval[u * scap + lane];
      if (lane < ocap) nVo = oval[u * ocap + lane];
      if (lane < pfS) nS = sclk[u * scap * A + lane];
      if (lane < pfO) nO = oclk[u * ocap * A + lane];
    }
    if (ns > scap || no > ocap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    mv_sync();
    if (lane < ns * A) S[lane] = cS;
    if (lane < no * A) O[lane] = cO;
    for (uint32_t k = kMW + lane; k < ns * A; k += kMW) S[k] = sclk[o * scap * A + k];
    for (uint32_t k = kMW + lane; k < no * A; k += kMW) O[k] = oclk[o * ocap * A + k];
    mv_sync();
    {  // flag matrices: G lanes per clock pair (G | 64, wave-uniform), strided over the actors, OR-reduced
      const uint32_t P1 = ns * no, P = P1 + no * no;
      uint32_t G = 1;
      while (G < kMW && 2u * G * P <= kMW && 2u * G <= A) G *= 2u;
      const uint32_t lg = 31u - __builtin_clz(G);
      for (uint32_t base = 0; base < P * G; base += kMW) {
        const uint32_t id = base + lane, p = id >> lg, gl = id & (G - 1u);
        uint32_t f = 3u;  // O x O entries on or above the diagonal are never read as "equal"
        if (p < P) {
          const uint64_t* pa = nullptr;
          const uint64_t* pb = nullptr;
          if (p < P1) {
            pa = S + (p / no) * A;
            pb = O + (p % no) * A;
          } else {
            const uint32_t q = p - P1, j = q / no, jj = q % no;
            if (jj < j) {
              pa = O + jj * A;
              pb = O + j * A;
            }
          }
          if (pa) {
            f = 0u;
            for (uint32_t x = gl; x < A; x += G) {
              const uint64_t u = pa[x], v = pb[x];
              f |= (u > v ? 1u : 0u) | (u < v ? 2u : 0u);
            }
          }
        }
        for (uint32_t off = 1; off < G; off <<= 1) f |= (uint32_t)__shfl_xor((int)f, (int)off, kMW);
        if (p < P && gl == 0u) {
          if (p < P1) fso[p] = (uint8_t)f;
          else foo[p - P1] = (uint8_t)f;
        }
      }
    }
    mv_sync();
    // self i: kept unless some other clock strictly dominates it (flags == "only <")
    bool ks = false, ko = false;
    if (lane < ns) {
      ks = true;
      for (uint32_t j = 0; j < no; ++j) ks = ks && fso[lane * no + j] != 2u;
    }
    const uint64_t KS = __ballot(ks);
    if (lane < no) {
      ko = true;
      for (uint32_t i = 0; i < ns; ++i) {
        const uint32_t f = fso[i * no + lane];
        ko = ko && f != 1u;                                 // a self clock strictly dominates it
        ko = ko && !(f == 0u && ((KS >> i) & 1ull));         // equal to a kept self clock
      }
      for (uint32_t jj = 0; jj < lane; ++jj) ko = ko && foo[lane * no + jj] != 0u;  // an earlier equal other clock
    }
    const uint64_t KO = __ballot(ko);
    const uint32_t nks = (uint32_t)__popcll(KS), nk = nks + (uint32_t)__popcll(KO);
    if (nk > outcap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ECAPACITY);
      continue;
    }
    const uint32_t rs = __builtin_amdgcn_mbcnt_hi((uint32_t)(KS >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)KS, 0u));
    const uint32_t ro = nks + __builtin_amdgcn_mbcnt_hi((uint32_t)(KO >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)KO, 0u));
    if (ks) tab[rs] = (uint8_t)lane;
    if (ko) tab[ro] = (uint8_t)(64u + lane);
    if (lane == 0u) outn[o] = nk;
    if (ks) outval[o * outcap + rs] = cVs;
    if (ko) outval[o * outcap + ro] = cVo;
    for (uint32_t k = nk + lane; k < outcap; k += kMW) outval[o * outcap + k] = 0u;
    mv_sync();
    uint64_t* oc = outclk + o * (uint64_t)AO;
    uint32_t k = lane / A, x = lane % A;  // slot and actor of this lane's first element
    const uint32_t dk = kMW / A, dx = kMW % A;  // per step of 64 elements
    for (uint32_t e = lane; e < AO; e += kMW) {
      uint64_t v = 0ull;
      if (k < nk) {
        const uint32_t src = tab[k];
        v = src < 64u ? S[src * A + x] : O[(src - 64u) * A + x];
      }
      oc[e] = v;
      k += dk;
      x += dx;
      if (x >= A) { x -= A; ++k; }
    }
  }
}

// Registers past the fast kernel's limits (> 64 slots per side, or rows that
// do not fit its LDS): one wave per pair, the clock rows read from HBM, the
// same keep rules and output form (self's survivors in order, then other's;
// unused slots zeroed); the kept flags of the current pair in LDS.
constexpr uint32_t kMvBigCap = 1024;  // slots per side

__device__ __forceinline__ uint32_t mv_cmp_rows(const uint64_t* a, const uint64_t* b, uint32_t A) {
  uint32_t f = 0u;  // 1: some a > b, 2: some a < b
  for (uint32_t x = 0; x < A; ++x) f |= (a[x] > b[x] ? 1u : 0u) | (a[x] < b[x] ? 2u : 0u);
  return f;
}

__global__ __launch_bounds__(kMW) void mvreg_merge_big_kernel(
    const uint32_t* __restrict__ sn, const uint64_t* __restrict__ sclk, const uint64_t* __restrict__ sval, uint32_t scap,
    const uint32_t* __restrict__ on, const uint64_t* __restrict__ oclk, const uint64_t* __restrict__ oval, uint32_t ocap,
    uint32_t* __restrict__ outn, uint64_t* __restrict__ outclk, uint64_t* __restrict__ outval, uint32_t outcap,
    uint64_t n_obj, uint32_t A, int* __restrict__ status) {
  __shared__ uint8_t ks_s[2 * kMvBigCap];  // kept flags: self slots, then other slots
  const uint32_t lane = threadIdx.x;
  for (uint64_t o = blockIdx.x; o < n_obj; o += gridDim.x) {
    const uint32_t ns = __builtin_amdgcn_readfirstlane(sn[o]), no = __builtin_amdgcn_readfirstlane(on[o]);
    if (ns > scap || no > ocap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    const uint64_t* S = sclk + o * scap * A;
    const uint64_t* O = oclk + o * ocap * A;
    // self i: kept unless some other clock strictly dominates it
    uint32_t nks = 0u;
    mv_sync();  // the previous pair's readers of ks_s are done
    for (uint32_t i = lane; i < ns; i += kMW) {
      bool k = true;
      for (uint32_t j = 0; j < no && k; ++j) k = mv_cmp_rows(S + (uint64_t)i * A, O + (uint64_t)j * A, A) != 2u;
      ks_s[i] = k ? 1u : 0u;
    }
    mv_sync();
    for (uint32_t i = lane; i < ns; i += kMW) nks += ks_s[i];
    // other j: kept unless a self clock strictly dominates it, it equals a kept
    // self clock, or it equals an earlier other clock
    uint32_t nko = 0u;
    for (uint32_t c0 = 0; c0 < no; c0 += kMW) {
      const uint32_t j = c0 + lane;
      bool k = j < no;
      for (uint32_t i = 0; i < ns && k; ++i) {
        const uint32_t f = mv_cmp_rows(S + (uint64_t)i * A, O + (uint64_t)j * A, A);
        k = f != 1u && !(f == 0u && ks_s[i]);
      }
      for (uint32_t jj = 0; jj < j && k; ++jj) k = mv_cmp_rows(O + (uint64_t)jj * A, O + (uint64_t)j * A, A) != 0u;
      nko += (uint32_t)__popcll(__ballot(k));
      if (j < no) ks_s[ns + j] = k ? 1u : 0u;
    }
    for (uint32_t d = 32; d >= 1; d >>= 1) nks += (uint32_t)__shfl_xor((int)nks, (int)d, kMW);
    const uint32_t nk = __builtin_amdgcn_readfirstlane(nks) + nko;
    if (nk > outcap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ECAPACITY);
      continue;
    }
    mv_sync();
    // survivors in order, one row per lane-round; then the unused slots zeroed
    uint64_t* oc = outclk + o * (uint64_t)outcap * A;
    uint32_t pos = 0u;
    for (uint32_t c0 = 0; c0 < ns + no; c0 += kMW) {
      const uint32_t t = c0 + lane;
      const bool k = t < ns + no && ks_s[t];
      const uint64_t m = __ballot(k);
      const uint32_t r = pos + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (k) {
        const uint64_t* src = t < ns ? S + (uint64_t)t * A : O + (uint64_t)(t - ns) * A;
        for (uint32_t x = 0; x < A; ++x) oc[(uint64_t)r * A + x] = src[x];
        outval[o * outcap + r] = t < ns ? sval[o * scap + t] : oval[o * ocap + (t - ns)];
      }
      pos += (uint32_t)__popcll(m);
    }
    for (uint64_t e = (uint64_t)nk * A + lane; e < (uint64_t)outcap * A; e += kMW) oc[e] = 0ull;
    for (uint32_t k = nk + lane; k < outcap; k += kMW) outval[o * outcap + k] = 0u;
    if (lane == 0u) outn[o] = nk;
  }
}

}  // namespace

int launch_vclock_cmp(const uint64_t* a, const uint64_t* b, uint64_t n, uint32_t A, int8_t* out, hipStream_t stream) {
  if (n == 0) return CRDT_OK;
  uint32_t G = 1;
  while (G < 64u && G * 2u <= A) G *= 2u;  // ~one or two slots per lane
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t per_block = 4u * (kMW / G), want = (n + per_block - 1) / per_block, cap = (uint64_t)cus * 16u;
  const uint32_t blocks = (uint32_t)(want < cap ? want : cap);
  hipLaunchKernelGGL(vclock_cmp_kernel, dim3(blocks), dim3(256), 0, stream, a, b, n, A, G, out);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

int launch_mvreg_merge(const uint32_t* sn, const uint64_t* sclk, const uint64_t* sval, uint32_t scap,
                       const uint32_t* on, const uint64_t* oclk, const uint64_t* oval, uint32_t ocap, uint32_t* outn,
                       uint64_t* outclk, uint64_t* outval, uint32_t outcap, uint64_t n_obj, uint32_t A, int* status,
                       hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  // per-wave LDS: clock rows, flag matrices, slot table; 16-B multiple
  const size_t per_wave = (8ull * (scap + ocap) * A + (size_t)scap * ocap + (size_t)ocap * ocap + outcap + 15u) & ~15ull;
  if (scap > kMvBigCap || ocap > kMvBigCap) return CRDT_EINVAL;
  if (per_wave > 60u * 1024u || scap > 64u || ocap > 64u) {  // past the fast kernel's limits
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t cap = (uint64_t)cus * 16u;
    hipLaunchKernelGGL(mvreg_merge_big_kernel, dim3((uint32_t)(n_obj < cap ? n_obj : cap)), dim3(kMW), 0, stream, sn,
                       sclk, sval, scap, on, oclk, oval, ocap, outn, outclk, outval, outcap, n_obj, A, status);
    return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
  }
  uint32_t W = 4;  // waves per block, as many as 60 KB of LDS allow
  while (W > 1u && W * per_wave > 60u * 1024u) --W;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t want = (n_obj + W - 1) / W, cap = (uint64_t)cus * (32u / W);  // ~8 waves per SIMD
  const uint32_t blocks = (uint32_t)(want < cap ? want : cap);
  hipLaunchKernelGGL(mvreg_merge_kernel, dim3(blocks), dim3(kMW * W), W * per_wave, stream, sn, sclk, sval, scap, on,
                     oclk, oval, ocap, outn, outclk, outval, outcap, n_obj, A, (uint32_t)per_wave, status);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
