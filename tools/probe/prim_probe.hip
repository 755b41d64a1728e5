// Probe of the cross-lane primitives mask3_object relies on (run on the box):
// ds_permute with colliding / missing targets, DPP wave_shr:1, icmp ballots.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(uint32_t* out) {
  const uint32_t l = threadIdx.x;
  // lanes < 20 send (l+1) to lane 2*l (so odd lanes and lanes >= 40 receive nothing), others send 7 to lane 0
  const uint32_t tgt = l < 20 ? 2 * l : 0;
  const uint32_t dat = l < 20 ? l + 1 : 7;
  out[l] = (uint32_t)__builtin_amdgcn_ds_permute((int)(tgt << 2), (int)dat);
  out[64 + l] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(l + 100), 0x138, 0xf, 0xf, false);
  const uint64_t m = __builtin_amdgcn_uicmpl((uint64_t)l << 33, 10ull << 33, 34);  // l > 10
  out[128 + l] = (uint32_t)(m >> 32) ^ (uint32_t)m;
  out[192 + l] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((l + 5) & 63) << 2), (int)(l * 3));
}

int main() {
  uint32_t* d;
  uint32_t h[256];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  printf("permute:");
  for (int i = 0; i < 64; ++i) printf(" %u", h[i]);
  printf("\nwave_shr:");
  for (int i = 0; i < 64; ++i) printf(" %u", h[64 + i]);
  printf("\nicmp ballot (hi^lo): %#x  (expect %#x)\nbpermute:", h[128], (uint32_t)((~0ull << 11) >> 32) ^ (uint32_t)(~0ull << 11));
  for (int i = 0; i < 64; ++i) printf(" %u", h[192 + i]);
  printf("\n");
  return 0;
}
