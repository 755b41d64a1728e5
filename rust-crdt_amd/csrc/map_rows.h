// Dense VClock rows held across a wave (internal; the Map kernels): slot s of
// lane l is actor l + 64 s, NS slots per lane (NS = 1 for n_actors <= 64, 2
// for <= 128), so every VClock operation is NS lane-parallel ops plus a
// ballot. Reference: src/vclock.rs (subtract :236-242, merge :131-137,
// PartialOrd :59-71, intersection :219-228).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace crdts_hip {
namespace maprow {

__device__ __forceinline__ uint64_t lane64(uint64_t v, uint32_t t) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), t) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, t);
}

template <int NS>
struct Row {
  uint64_t v[NS];
};
template <int NS>
__device__ __forceinline__ Row<NS> zrow() {
  Row<NS> r;
  for (int k = 0; k < NS; ++k) r.v[k] = 0ull;
  return r;
}
// VClock::subtract, slot by slot
template <int NS>
__device__ __forceinline__ Row<NS> vsub(Row<NS> e, Row<NS> c) {
  for (int k = 0; k < NS; ++k) e.v[k] = c.v[k] >= e.v[k] ? 0ull : e.v[k];
  return e;
}
// VClock::merge
template <int NS>
__device__ __forceinline__ Row<NS> vmax(Row<NS> a, Row<NS> b) {
  for (int k = 0; k < NS; ++k) a.v[k] = a.v[k] > b.v[k] ? a.v[k] : b.v[k];
  return a;
}
// !is_empty()
template <int NS>
__device__ __forceinline__ bool vany(Row<NS> v) {
  bool a = false;
  for (int k = 0; k < NS; ++k) a = a || v.v[k] != 0ull;
  return __ballot(a) != 0ull;
}
// `d <= c` (PartialOrd) for dense rows: every slot of d within c
template <int NS>
__device__ __forceinline__ bool vle(Row<NS> d, Row<NS> c) {
  bool gt = false;
  for (int k = 0; k < NS; ++k) gt = gt || d.v[k] > c.v[k];
  return __ballot(gt) == 0ull;
}
// partial_cmp(a, b) == Some(Less): a <= b and a != b
template <int NS>
__device__ __forceinline__ bool vstrict_less(Row<NS> a, Row<NS> b) {
  bool gt = false, lt = false;
  for (int k = 0; k < NS; ++k) {
    gt = gt || a.v[k] > b.v[k];
    lt = lt || a.v[k] < b.v[k];
  }
  return __ballot(gt) == 0ull && __ballot(lt) != 0ull;
}
template <int NS>
__device__ __forceinline__ bool veq(Row<NS> a, Row<NS> b) {
  bool ne = false;
  for (int k = 0; k < NS; ++k) ne = ne || a.v[k] != b.v[k];
  return __ballot(ne) == 0ull;
}
// VClock::intersection: the slots equal on both sides
template <int NS>
__device__ __forceinline__ Row<NS> vcommon(Row<NS> a, Row<NS> b) {
  for (int k = 0; k < NS; ++k) a.v[k] = (a.v[k] == b.v[k] && a.v[k] != 0ull) ? a.v[k] : 0ull;
  return a;
}
// CLOCK ORDER of two dense rows (lexicographic over their (actor, counter)
// pairs, a proper prefix first): decided at the first actor where they differ
template <int NS>
__device__ int vorder(Row<NS> p, Row<NS> q, uint32_t lane) {
  for (int k = 0; k < NS; ++k) {
    const uint64_t diff = __ballot(p.v[k] != q.v[k]);
    if (!diff) continue;
    const uint32_t x = (uint32_t)__builtin_ctzll(diff);
    const uint64_t px = lane64(p.v[k], x), qx = lane64(q.v[k], x);
    if (px && qx) return px < qx ? -1 : 1;
    // one side has no entry at actor 64k + x: the other's next entry decides
    bool later = false;  // does the side WITHOUT x hold an actor above it?
    for (int j = k; j < NS; ++j) {
      const uint64_t w = !px ? p.v[j] : q.v[j];
      later = later || (w != 0ull && (j > k || lane > x));
    }
    const bool any = __ballot(later) != 0ull;
    return !px ? (any ? 1 : -1) : (any ? -1 : 1);
  }
  return 0;
}
// a row at `base` / row `row` of a [.][A] array
template <int NS>
__device__ __forceinline__ Row<NS> ldrow(const uint64_t* base, uint32_t A, uint32_t lane) {
  Row<NS> r;
  for (int k = 0; k < NS; ++k) r.v[k] = lane + 64u * k < A ? base[lane + 64u * k] : 0ull;
  return r;
}
template <int NS>
__device__ __forceinline__ Row<NS> rowv(const uint64_t* base, uint64_t row, uint32_t A, uint32_t lane) {
  return ldrow<NS>(base + row * A, A, lane);
}
template <int NS>
__device__ __forceinline__ void strow(uint64_t* base, Row<NS> r, uint32_t A, uint32_t lane) {
  for (int k = 0; k < NS; ++k)
    if (lane + 64u * k < A) base[lane + 64u * k] = r.v[k];
}

}  // namespace maprow
}  // namespace crdts_hip
