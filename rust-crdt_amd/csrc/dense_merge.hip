// Dense VClock / GCounter / PNCounter join: self[k] = max(self[k], other[k])
// over u64 slots, in place.
//
// VClock::merge (src/vclock.rs:131-137) witnesses every (actor, counter) of
// `other` (witness = keep the larger, :159-163), i.e. the pointwise max over
// the actor union with absent = 0; GCounter (src/gcounter.rs:58-62) and
// PNCounter (src/pncounter.rs:90-95) delegate to it. On dense rows the whole
// batch is one flat max over n_obj * slots u64 words, so the kernel ignores
// row boundaries: 16-B loads, 4 independent 16-B pairs in flight per lane,
// grid-stride, HBM-bound (24 B of traffic per slot: 2 reads + 1 write).
#include <hip/hip_runtime.h>

#include "../../include/crdts_hip.h"
#include "kernels.h"

namespace crdts_hip {
namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr int kThreads = 256;
constexpr int kUnroll = 4;

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

__global__ __launch_bounds__(kThreads) void dense_max_kernel(u64x2* __restrict__ s,
                                                             const u64x2* __restrict__ o,
                                                             uint64_t n2) {
  const uint64_t tile = (uint64_t)kThreads * kUnroll;
  for (uint64_t base = (uint64_t)blockIdx.x * tile; base < n2; base += (uint64_t)gridDim.x * tile) {
    u64x2 a[kUnroll], b[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      uint64_t k = base + (uint64_t)u * kThreads + threadIdx.x;
      if (k < n2) {
        a[u] = __builtin_nontemporal_load(s + k);
        b[u] = __builtin_nontemporal_load(o + k);
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      uint64_t k = base + (uint64_t)u * kThreads + threadIdx.x;
      if (k < n2) {
        u64x2 r;
        r.x = umax64(a[u].x, b[u].x);
        r.y = umax64(a[u].y, b[u].y);
        __builtin_nontemporal_store(r, s + k);
      }
    }
  }
}

__global__ void dense_max_tail(uint64_t* s, const uint64_t* o, uint64_t n) {
  uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k < n) s[k] = umax64(s[k], o[k]);
}

}  // namespace

int launch_dense_max(uint64_t* self, const uint64_t* other, uint64_t n_words, hipStream_t stream) {
  if (n_words == 0) return CRDT_OK;
  const bool aligned = ((uintptr_t)self % 16 == 0) && ((uintptr_t)other % 16 == 0);
  uint64_t n2 = aligned ? n_words / 2 : 0;
  if (n2) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    uint64_t tiles = (n2 + (uint64_t)kThreads * kUnroll - 1) / ((uint64_t)kThreads * kUnroll);
    uint64_t cap = (uint64_t)cus * 8;
    uint32_t blocks = (uint32_t)(tiles < cap ? tiles : cap);
    hipLaunchKernelGGL(dense_max_kernel, dim3(blocks), dim3(kThreads), 0, stream, (u64x2*)self,
                       (const u64x2*)other, n2);
  }
  uint64_t done = 2 * n2, rest = n_words - done;
  if (rest) {
    uint32_t blocks = (uint32_t)((rest + 255) / 256);
    hipLaunchKernelGGL(dense_max_tail, dim3(blocks), dim3(256), 0, stream, self + done, other + done,
                       rest);
  }
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

}  // namespace crdts_hip
