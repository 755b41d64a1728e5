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

// per-lane: compare two dense rows in LDS: bit0 = some x with p > q, bit1 = some x with p < q
__device__ __forceinline__ uint32_t row_flags(const uint64_t* p, const uint64_t* q, uint32_t A) {
  uint32_t f = 0;
  for (uint32_t x = 0; x < A; ++x) {
    const uint64_t u = p[x], v = q[x];
    f |= (u > v ? 1u : 0u) | (u < v ? 2u : 0u);
  }
  return f;
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
  for (uint64_t o = (uint64_t)blockIdx.x * W + wave; o < n_obj; o += (uint64_t)gridDim.x * W) {
    const uint32_t ns = __builtin_amdgcn_readfirstlane(sn[o]), no = __builtin_amdgcn_readfirstlane(on[o]);
    if (ns > scap || no > ocap) {
      if (lane == 0u) atomicCAS(status, 0, CRDT_ENONCANON);
      continue;
    }
    mv_sync();
    for (uint32_t k = lane; k < ns * A; k += kMW) S[k] = sclk[o * scap * A + k];
    for (uint32_t k = lane; k < no * A; k += kMW) O[k] = oclk[o * ocap * A + k];
    mv_sync();
    for (uint32_t p = lane; p < ns * no; p += kMW) fso[p] = (uint8_t)row_flags(S + (p / no) * A, O + (p % no) * A, A);
    for (uint32_t p = lane; p < no * no; p += kMW) {
      const uint32_t j = p / no, jj = p % no;
      foo[p] = jj < j ? (uint8_t)row_flags(O + jj * A, O + j * A, A) : (uint8_t)3u;
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
    if (ks) outval[o * outcap + rs] = sval[o * scap + lane];
    if (ko) outval[o * outcap + ro] = oval[o * ocap + lane];
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
  if (per_wave > 60u * 1024u || scap > 64u || ocap > 64u) return CRDT_EINVAL;
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
