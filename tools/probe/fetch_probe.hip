// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths the
// secondary kernels use (MI355X_MICROARCH.md, HBM section: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern"). Each kernel touches exactly kBytes of a buffer far larger than
// the 256 MiB Infinity Cache, once; tools/probe/fetch_calib.py divides the
// counters by kBytes. Diagnostic, not product.
//   hipcc --offload-arch=gfx950 -O3 fetch_probe.hip -o fetch_probe
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o run -- ./fetch_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr uint64_t kBytes = 1ull << 30;  // 1 GiB per pass
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// coalesced: lane i of the grid-stride step reads word i (W bytes per lane)
template <class T>
__global__ void rd_coalesced(const T* __restrict__ p, uint64_t n, uint64_t* out) {
  T acc{};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc[0] == 0x12345u) out[0] = (uint64_t)acc[0];
}
template <>
__global__ void rd_coalesced<uint64_t>(const uint64_t* __restrict__ p, uint64_t n, uint64_t* out) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x123456789ull) out[0] = acc;
}
template <>
__global__ void rd_coalesced<uint32_t>(const uint32_t* __restrict__ p, uint64_t n, uint64_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x12345u) out[0] = acc;
}
// lane walk: every lane reads its own SEG-byte segment front to back with
// 8-B loads (the bincode lane-walk / apply per-lane pattern)
template <uint32_t SEG>
__global__ void rd_lane_walk(const uint64_t* __restrict__ p, uint64_t n_seg, uint64_t* out) {
  uint64_t acc = 0;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < n_seg; s += (uint64_t)gridDim.x * blockDim.x)
    for (uint32_t k = 0; k < SEG / 8; ++k) acc += p[s * (SEG / 8) + k];
  if (acc == 0x123456789ull) out[0] = acc;
}
// wave walk: one wave per SEG-byte segment, 64 lanes x 8 B per step
template <uint32_t SEG>
__global__ void rd_wave_seg8(const uint64_t* __restrict__ p, uint64_t n_seg, uint64_t* out) {
  uint64_t acc = 0;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64u, nw = (uint64_t)gridDim.x * blockDim.x / 64u;
  for (uint64_t s = w; s < n_seg; s += nw)
    for (uint32_t k = lane; k < SEG / 8; k += 64u) acc += p[s * (SEG / 8) + k];
  if (acc == 0x123456789ull) out[0] = acc;
}
template <class T>
__global__ void wr_coalesced(T* __restrict__ p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (T)i;
}
__global__ void wr_coalesced16(u32x4* __restrict__ p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

int main() {
  uint8_t* buf;
  uint64_t* out;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(buf, 1, kBytes) != hipSuccess) return 1;
  const dim3 g(256 * 16), b(256);
  hipLaunchKernelGGL(rd_coalesced<u32x4>, g, b, 0, 0, (const u32x4*)buf, kBytes / 16, out);
  hipLaunchKernelGGL(rd_coalesced<uint64_t>, g, b, 0, 0, (const uint64_t*)buf, kBytes / 8, out);
  hipLaunchKernelGGL(rd_coalesced<uint32_t>, g, b, 0, 0, (const uint32_t*)buf, kBytes / 4, out);
  hipLaunchKernelGGL(rd_lane_walk<1024>, g, b, 0, 0, (const uint64_t*)buf, kBytes / 1024, out);
  hipLaunchKernelGGL(rd_wave_seg8<1024>, g, b, 0, 0, (const uint64_t*)buf, kBytes / 1024, out);
  hipLaunchKernelGGL(wr_coalesced16, g, b, 0, 0, (u32x4*)buf, kBytes / 16);
  hipLaunchKernelGGL(wr_coalesced<uint64_t>, g, b, 0, 0, (uint64_t*)buf, kBytes / 8);
  hipLaunchKernelGGL(wr_coalesced<uint32_t>, g, b, 0, 0, (uint32_t*)buf, kBytes / 4);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("fetch_probe: %llu bytes per kernel\n", (unsigned long long)kBytes);
  return 0;
}
