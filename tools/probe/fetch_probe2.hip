// Round-5 calibration of FETCH_SIZE (and of the HBM cost) for the partial-line
// read patterns of the Map kernels (map.hip / map_orswot.hip / map_map.hip):
// dense 128-B actor rows read by 16 lanes x 8 B, and slots that use only part
// of a 128-B line (counts, keys, set sizes). Each kernel walks a 1 GiB buffer
// (4x the Infinity Cache) once and touches, in every 128-B line, the bytes its
// name says; main() times each (HIP events, best of 5) and prints one JSON
// line. Under `rocprofv3 --pmc FETCH_SIZE` tools/probe/fetch_calib.py gives
// counter bytes / 1 GiB per kernel. Diagnostic, not product.
//   hipcc --offload-arch=gfx950 -O3 fetch_probe2.hip -o fetch_probe2
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr uint64_t kBytes = 1ull << 30;
constexpr uint64_t kLines = kBytes / 128;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// every byte: 16 B per lane, coalesced
__global__ void full16(const u32x4* __restrict__ p, uint64_t n, uint64_t* out) {
  u32x4 acc{};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc[0] == 0x12345u) out[0] = acc[0];
}
// B bytes at the start of every 128-B line, 8 B per lane (B/8 lanes a line):
// B = 128 is a dense actor row read the way rowv reads it (16 lanes x 8 B)
template <uint32_t B>
__global__ void part_line(const uint64_t* __restrict__ p, uint64_t* out) {
  constexpr uint32_t kL = B / 8;  // lanes per line
  uint64_t acc = 0;
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t s = t; s < kLines * kL; s += nt) acc += p[(s / kL) * 16 + (s % kL)];
  if (acc == 0x123456789ull) out[0] = acc;
}
// one 8-B word in every other 64-B half line (the word at offset 64 of each line)
__global__ void second_half8(const uint64_t* __restrict__ p, uint64_t* out) {
  uint64_t acc = 0;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < kLines; s += (uint64_t)gridDim.x * blockDim.x)
    acc += p[s * 16 + 8];
  if (acc == 0x123456789ull) out[0] = acc;
}

typedef void (*Launch)(const void*, uint64_t*);

int main() {
  uint8_t* buf;
  uint64_t* out;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(buf, 1, kBytes) != hipSuccess) return 1;
  const dim3 g(256 * 16), b(256);
  struct K { const char* name; int id; };
  const K ks[] = {{"full16", 0}, {"part_line<128>", 1}, {"part_line<64>", 2}, {"part_line<32>", 3},
                  {"part_line<8>", 4}, {"second_half8", 5}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("{\"bytes\": %llu", (unsigned long long)kBytes);
  for (const K& k : ks) {
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0, 0);
      switch (k.id) {
        case 0: hipLaunchKernelGGL(full16, g, b, 0, 0, (const u32x4*)buf, kBytes / 16, out); break;
        case 1: hipLaunchKernelGGL(part_line<128>, g, b, 0, 0, (const uint64_t*)buf, out); break;
        case 2: hipLaunchKernelGGL(part_line<64>, g, b, 0, 0, (const uint64_t*)buf, out); break;
        case 3: hipLaunchKernelGGL(part_line<32>, g, b, 0, 0, (const uint64_t*)buf, out); break;
        case 4: hipLaunchKernelGGL(part_line<8>, g, b, 0, 0, (const uint64_t*)buf, out); break;
        default: hipLaunchKernelGGL(second_half8, g, b, 0, 0, (const uint64_t*)buf, out); break;
      }
      (void)hipEventRecord(e1, 0);
      if (hipEventSynchronize(e1) != hipSuccess) return 1;
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    printf(", \"%s_ms\": %.4f", k.name, best);
  }
  printf("}\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
