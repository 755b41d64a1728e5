// Object schedule of the one-object-per-wave kernels (internal).
//
// A resident grid with a static split leaves the youngest waves of every
// SIMD running last: the issue arbiter favours the oldest waves, so with
// equal work the youngest finish last and, at the end, alone (measured on
// the Orswot join, tools/wave_tail.py). BlockTickets gives
// each single-wave block the first half of its objects by block index
// (o = block + k * grid) and the rest in tickets of K consecutive objects
// from an atomic counter (zeroed before the launch); the next ticket is in
// flight while the current one's objects are processed.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace crdts_hip {

template <uint32_t K>
struct BlockTickets {
  uint64_t n, grid, s_rounds, s_total, end = 0, k = 0;
  uint32_t* ctr;
  uint32_t tk = 0u, lane;
  bool dyn = false;
  __device__ BlockTickets(uint64_t n_, uint32_t* ctr_, uint32_t lane_) : n(n_), ctr(ctr_), lane(lane_) {
    grid = gridDim.x;
    s_rounds = n / 2u / grid;
    s_total = s_rounds * grid;
  }
  __device__ uint64_t enter() {  // the next ticket's first object (n: none left)
    dyn = true;
    const uint64_t o0 = s_total + (uint64_t)__builtin_amdgcn_readfirstlane(tk) * K;
    if (o0 >= n) return n;
    end = o0 + K < n ? o0 + K : n;
    if (lane == 0u) tk = atomicAdd(ctr, 1u);  // the ticket after this one
    return o0;
  }
  __device__ uint64_t first() {
    if (lane == 0u) tk = atomicAdd(ctr, 1u);
    return s_rounds ? (uint64_t)blockIdx.x : enter();
  }
  __device__ uint64_t next(uint64_t cur) {
    if (!dyn) {
      if (++k < s_rounds) return blockIdx.x + k * grid;
      return enter();
    }
    return cur + 1u < end ? cur + 1u : enter();
  }
};

}  // namespace crdts_hip
