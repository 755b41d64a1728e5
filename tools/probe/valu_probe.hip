// Issue-rate probe of the VALU instructions the merge kernels lean on (run on
// the box; diagnostic, not product): independent instruction streams per wave,
// every SIMD of the chip loaded with W waves; prints ns per wave-instruction
// per SIMD, so ops can be compared (32- vs 64-bit compares, selects, adds).
//   hipcc --offload-arch=gfx950 -O3 valu_probe.hip -o valu_probe && ./valu_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define R16(x) x x x x x x x x x x x x x x x x

template <int OP>
__global__ void valu_kernel(uint64_t* out, int iters) {
  uint32_t c = threadIdx.x, d = threadIdx.x * 5u + 1u, e = 7u;
  uint64_t a = threadIdx.x, b = (uint64_t)threadIdx.x * 3u + 1u;
  uint64_t m = 0;
  for (int i = 0; i < iters; ++i) {
    if (OP == 0) asm volatile(R16("v_cmp_lt_u32_e64 %0, %1, %2\n") : "=s"(m) : "v"(c), "v"(d));
    if (OP == 1) asm volatile(R16("v_cmp_lt_u64_e64 %0, %1, %2\n") : "=s"(m) : "v"(a), "v"(b));
    if (OP == 2) asm volatile(R16("v_cndmask_b32_e64 %0, %1, %2, vcc\n") : "=v"(e) : "v"(c), "v"(d));
    if (OP == 3) asm volatile(R16("v_add_u32_e32 %0, %1, %2\n") : "=v"(e) : "v"(c), "v"(d));
    if (OP == 4) asm volatile(R16("v_mbcnt_lo_u32_b32 %0, %1, %2\n") : "=v"(e) : "s"((uint32_t)m), "v"(d));
    if (OP == 5) asm volatile(R16("v_cmp_eq_u64_e64 %0, %1, %2\n") : "=s"(m) : "v"(a), "v"(b));
    if (OP == 6) asm volatile(R16("v_bcnt_u32_b32 %0, %1, %2\n") : "=v"(e) : "v"(c), "v"(d));
    if (OP == 7) asm volatile(R16("v_lshl_add_u32 %0, %1, 3, %2\n") : "=v"(e) : "v"(c), "v"(d));
  }
  if (threadIdx.x == 0) out[blockIdx.x] = m + e;
}

template <int OP>
float run(int waves_per_simd, int iters, uint64_t* d) {
  const int blocks = 256 * 4 * waves_per_simd;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(valu_kernel<OP>, dim3(blocks), dim3(64), 0, 0, d, iters);  // warm
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(valu_kernel<OP>, dim3(blocks), dim3(64), 0, 0, d, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // ns per wave-instruction per SIMD
  return ms * 1e6f / ((float)waves_per_simd * iters * 16.0f);
}

int main() {
  uint64_t* d;
  if (hipMalloc(&d, 8 << 20) != hipSuccess) return 1;
  const char* names[] = {"v_cmp_lt_u32", "v_cmp_lt_u64", "v_cndmask_b32", "v_add_u32", "v_mbcnt_lo", "v_cmp_eq_u64",
                         "v_bcnt_u32_b32", "v_lshl_add_u32"};
  for (int w : {1, 2, 4, 8}) {
    printf("waves/SIMD %d:", w);
    const int it = 20000;
    float r[8] = {run<0>(w, it, d), run<1>(w, it, d), run<2>(w, it, d), run<3>(w, it, d),
                  run<4>(w, it, d), run<5>(w, it, d), run<6>(w, it, d), run<7>(w, it, d)};
    for (int k = 0; k < 8; ++k) printf(" %s %.3f ns", names[k], r[k]);
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
