// Record utilities on the device: deep canonical-form validation, and the
// size / copy kernels behind crdt_orswot_compact (gap removal after a merge).
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"
#include "record_layout.h"

namespace crdts_hip {
namespace {

__device__ __forceinline__ void fail(int* status) { atomicCAS(status, 0, CRDT_ENONCANON); }

// One lane per record. Checks every invariant listed in include/crdts_hip.h.
__global__ void validate_kernel(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                uint64_t bytes, uint64_t n_obj, uint32_t A, uint32_t flags, int* status) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n_obj) return;
  uint64_t o = off[i];
  if ((o & 15u) || o + kHdrBytes > bytes) return fail(status);
  const uint8_t* r = base + o;
  const uint32_t* h = (const uint32_t*)r;
  const bool sparse = (flags & kSparseClock) != 0;
  if (h[7] != flags) return fail(status);
  RecLayout L;
  rec_layout(L, h[1], h[2], h[3], h[4], h[5], h[6], sparse);
  if (h[0] != L.size || (sparse ? h[1] > A : h[1] != A) || o + L.size > bytes) return fail(status);
  if (sparse) {  // CSR top clock: actors strictly increasing and < A, counters > 0
    const uint64_t* cc = (const uint64_t*)(r + L.o_clk);
    const uint32_t* ca = (const uint32_t*)(r + L.o_cact);
    for (uint32_t k = 0; k < L.n_clk; ++k)
      if (ca[k] >= A || cc[k] == 0 || (k && !(ca[k - 1] < ca[k]))) return fail(status);
  }
  const uint64_t* key = (const uint64_t*)(r + L.o_key);
  const uint64_t* dctr = (const uint64_t*)(r + L.o_dctr);
  const uint32_t* dact = (const uint32_t*)(r + L.o_dact);
  const uint32_t* mdend = (const uint32_t*)(r + L.o_mdend);
  const uint64_t* fctr = (const uint64_t*)(r + L.o_fctr);
  const uint64_t* fkey = (const uint64_t*)(r + L.o_fkey);
  const uint32_t* fact = (const uint32_t*)(r + L.o_fact);
  const uint32_t* fdend = (const uint32_t*)(r + L.o_fdend);
  const uint32_t* fmend = (const uint32_t*)(r + L.o_fmend);
  uint32_t s = 0;
  for (uint32_t m = 0; m < L.n_mem; ++m) {
    if (m && !(key[m - 1] < key[m])) return fail(status);
    uint32_t e = mdend[m];
    if (e <= s || e > L.n_dot) return fail(status);
    for (uint32_t d = s; d < e; ++d) {
      if (dact[d] >= A || dctr[d] == 0) return fail(status);
      if (d > s && !(dact[d - 1] < dact[d])) return fail(status);
    }
    s = e;
  }
  if (s != L.n_dot) return fail(status);
  uint32_t fs = 0, ms = 0;
  for (uint32_t k = 0; k < L.n_def; ++k) {
    uint32_t fe = fdend[k], me = fmend[k];
    if (fe <= fs || fe > L.n_def_dot || me <= ms || me > L.n_def_mem) return fail(status);
    for (uint32_t d = fs; d < fe; ++d) {
      if (fact[d] >= A || fctr[d] == 0) return fail(status);
      if (d > fs && !(fact[d - 1] < fact[d])) return fail(status);
    }
    for (uint32_t j = ms + 1; j < me; ++j)
      if (!(fkey[j - 1] < fkey[j])) return fail(status);
    if (k) {  // strictly increasing CLOCK ORDER
      uint32_t ps = k > 1 ? fdend[k - 2] : 0, pe = fs, a = ps, b = fs;
      int c = 0;
      for (; a < pe && b < fe && c == 0; ++a, ++b) {
        if (fact[a] != fact[b]) c = fact[a] < fact[b] ? -1 : 1;
        else if (fctr[a] != fctr[b]) c = fctr[a] < fctr[b] ? -1 : 1;
      }
      if (c == 0) c = (a == pe && b == fe) ? 0 : (a == pe ? -1 : 1);
      if (c >= 0) return fail(status);
    }
    fs = fe;
    ms = me;
  }
  if (fs != L.n_def_dot || ms != L.n_def_mem) return fail(status);
}

// Record sizes, bounds-checked: a record whose header or extent is out of
// [0, bytes), misaligned, or whose size is not a 16-B multiple >= the header
// gets size 0 (nothing is copied for it) and latches CRDT_ENONCANON — e.g.
// an object a merge rejected, whose output offset has no record behind it.
__global__ void sizes_kernel(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off, uint64_t bytes,
                             uint64_t n_obj, uint64_t* __restrict__ sizes, int* status) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n_obj) return;
  const uint64_t o = off[i];
  uint64_t size = 0;
  if (!(o & 15u) && o <= bytes && bytes - o >= kHdrBytes) {
    const uint64_t s = *(const uint32_t*)(base + o);
    if (s >= kHdrBytes && !(s & 15u) && s <= bytes - o) size = s;
  }
  if (!size) fail(status);
  sizes[i] = size;
}

// One wave per record, 16-B copies of sizes[i] bytes (sizes_kernel's).
__global__ __launch_bounds__(256) void copy_kernel(const uint8_t* __restrict__ src,
                                                   const uint64_t* __restrict__ src_off,
                                                   const uint64_t* __restrict__ sizes,
                                                   uint8_t* __restrict__ dst,
                                                   const uint64_t* __restrict__ dst_off,
                                                   uint64_t n_obj, uint64_t dst_bytes) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64; i < n_obj; i += stride) {
    const uint4* s = (const uint4*)(src + src_off[i]);
    const uint64_t o = dst_off[i], sz = sizes[i];
    if (o > dst_bytes || sz > dst_bytes - o) continue;
    uint4* d = (uint4*)(dst + o);
    const uint32_t n16 = (uint32_t)(sz / 16);
    for (uint32_t k = lane; k < n16; k += 64) d[k] = s[k];
  }
}

}  // namespace

int launch_orswot_validate(const uint8_t* base, const uint64_t* off, uint64_t bytes, uint64_t n_obj,
                           uint32_t n_actors, uint32_t flags, int* status, hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  uint32_t blocks = (uint32_t)((n_obj + 255) / 256);
  hipLaunchKernelGGL(validate_kernel, dim3(blocks), dim3(256), 0, stream, base, off, bytes, n_obj,
                     n_actors, flags, status);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

int launch_record_sizes(const uint8_t* base, const uint64_t* off, uint64_t bytes, uint64_t n_obj, uint64_t* sizes,
                        int* status, hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  uint32_t blocks = (uint32_t)((n_obj + 255) / 256);
  hipLaunchKernelGGL(sizes_kernel, dim3(blocks), dim3(256), 0, stream, base, off, bytes, n_obj, sizes, status);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

int launch_record_copy(const uint8_t* src, const uint64_t* src_off, const uint64_t* sizes, uint8_t* dst,
                       const uint64_t* dst_off, uint64_t n_obj, uint64_t dst_bytes, hipStream_t stream) {
  if (n_obj == 0) return CRDT_OK;
  uint64_t want = (n_obj + 3) / 4;
  uint32_t blocks = (uint32_t)(want < 2048 ? want : 2048);
  hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, stream, src, src_off, sizes, dst, dst_off,
                     n_obj, dst_bytes);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
