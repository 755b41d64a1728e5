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
  uint64_t n, unit, units, s_rounds, s_total, end = 0, k = 0;
  uint32_t* ctr;
  uint32_t tk = 0u, lane;
  bool dyn = false;
  // unit / units: this wave's index among the waves sharing the objects
  // (default: one wave per block)
  __device__ BlockTickets(uint64_t n_, uint32_t* ctr_, uint32_t lane_, uint64_t unit_ = blockIdx.x,
                          uint64_t units_ = gridDim.x)
      : n(n_), unit(unit_), units(units_), ctr(ctr_), lane(lane_) {
    s_rounds = n / 2u / units;
    s_total = s_rounds * units;
  }
  __device__ uint64_t enter() {  // the next ticket's first object (n: none left)
    dyn = true;
    const uint64_t o0 = s_total + (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(tk) * K;
    if (o0 >= n) return n;
    end = o0 + K < n ? o0 + K : n;
    if (lane == 0u) tk = atomicAdd(ctr, 1u);  // the ticket after this one
    return o0;
  }
  __device__ uint64_t first() {
    if (lane == 0u) tk = atomicAdd(ctr, 1u);
    return s_rounds ? unit : enter();
  }
  // the object after cur (n: none); may be called one object ahead
  __device__ uint64_t next(uint64_t cur) {
    if (!dyn) {
      if (++k < s_rounds) return unit + k * units;
      return enter();
    }
    return cur + 1u < end ? cur + 1u : enter();
  }
};

// The plain grid-stride schedule with BlockTickets' interface: for the task
// launches whose items are mostly empty (the nested map's per-slot tasks),
// where a ticket atomic per few items would cost more than the imbalance.
struct GridStride {
  uint64_t n;
  __device__ GridStride(uint64_t n_, uint32_t*, uint32_t) : n(n_) {}
  __device__ uint64_t first() const { return blockIdx.x; }
  __device__ uint64_t next(uint64_t cur) const { return cur + gridDim.x; }
};

// Guided chunk schedule of the join kernels: the first SF/8 of n objects in
// static rounds of (<= 64-object) chunks by wave index, the rest in chunks
// of DYN objects handed out by an atomic ticket (ctl[3], zeroed before the
// launch). The issue arbiter favours a SIMD's oldest waves, so with a static
// split the youngest waves finish last and alone (tools/wave_tail.py: the
// median wave was done at 0.77 of the launch); tickets go to the waves that
// are ahead. A wave takes the ticket for its next chunk when the chunk before
// it starts, so the atomic's round trip is hidden behind that chunk.
// (GMIN > 0, diagnostic: ticket chunks shrink from DYN to GMIN as the pool
// drains; the counter then counts objects.)
template <uint32_t DYN, uint32_t SF, uint32_t GMIN = 0>
struct GuidedSplit {
  uint64_t n, wave_id, n_waves, s_total, rounds_s, cs_s;
  uint32_t ticket = 0u, it = 0u, tsz = DYN, seen = 0u;
  bool have_ticket = false;
  __device__ GuidedSplit(uint64_t n_, uint64_t wave_id_, uint64_t n_waves_)
      : n(n_), wave_id(wave_id_), n_waves(n_waves_) {
    s_total = SF >= 8u ? n : n * SF / 8u;
    rounds_s = (s_total + n_waves * 64u - 1) / (n_waves * 64u);  // chunks of <= 64 objects (one per lane)
    cs_s = rounds_s ? (s_total + n_waves * rounds_s - 1) / (n_waves * rounds_s) : 1u;
  }
  __device__ bool is_static(uint32_t k) const { return k < rounds_s && (wave_id + k * n_waves) * cs_s < s_total; }
  __device__ void take(uint32_t* ctr, uint32_t lane) {
    if (GMIN) {
      const uint64_t pool = n - s_total, left = pool > seen ? pool - seen : 0u;
      const uint64_t want = left / (2u * n_waves);
      tsz = want > DYN ? DYN : want < GMIN ? GMIN : (uint32_t)want;
      if (lane == 0u) ticket = atomicAdd(ctr, tsz);
    } else if (lane == 0u) {
      ticket = atomicAdd(ctr, 1u);
    }
  }
  // this wave's next chunk [cb, ce), or false when there is none
  __device__ bool next(uint64_t& cb, uint64_t& ce, uint32_t* ctr, uint32_t lane) {
    if (is_static(it)) {
      cb = (wave_id + it * n_waves) * cs_s;
      ce = cb + cs_s < s_total ? cb + cs_s : s_total;
    } else {
      if (!have_ticket) take(ctr, lane);
      const uint32_t tk = __builtin_amdgcn_readfirstlane(ticket);
      cb = s_total + (GMIN ? (uint64_t)tk : (uint64_t)tk * DYN);
      ce = cb + tsz < n ? cb + tsz : n;
      seen = tk + tsz;
      have_ticket = false;
      if (cb >= n) return false;
    }
    ++it;
    if (!is_static(it)) {  // the next chunk is a ticket: take it now
      take(ctr, lane);
      have_ticket = true;
    }
    return true;
  }
};

}  // namespace crdts_hip
