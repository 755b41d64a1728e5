// Canonical Orswot record layout (spec: include/crdts_hip.h), shared by the
// host codec and the device kernels.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define CRDT_HD __host__ __device__ __forceinline__
#else
#define CRDT_HD inline
#endif

namespace crdts_hip {

constexpr uint32_t kHdrBytes = 32;

// Byte offsets of every section of one record, from its counts.
struct RecLayout {
  uint32_t n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem;
  uint32_t o_clk, o_key, o_dctr, o_dact, o_mdend, o_mpad;  // member block
  uint32_t o_def, o_fctr, o_fkey, o_fact, o_fdend, o_fmend, o_end, size;
};

CRDT_HD uint32_t pad_to(uint32_t x, uint32_t a) { return (x + a - 1) & ~(a - 1); }

// Member-block end (8-aligned) for the given counts.
CRDT_HD uint32_t member_block_end(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot) {
  return pad_to(kHdrBytes + 8u * n_clk + 12u * (n_mem + n_dot), 8);
}

CRDT_HD void rec_layout(RecLayout& L, uint32_t n_clk, uint32_t n_mem, uint32_t n_dot,
                        uint32_t n_def, uint32_t n_def_dot, uint32_t n_def_mem) {
  L.n_clk = n_clk; L.n_mem = n_mem; L.n_dot = n_dot;
  L.n_def = n_def; L.n_def_dot = n_def_dot; L.n_def_mem = n_def_mem;
  L.o_clk = kHdrBytes;
  L.o_key = L.o_clk + 8u * n_clk;
  L.o_dctr = L.o_key + 8u * n_mem;
  L.o_dact = L.o_dctr + 8u * n_dot;
  L.o_mdend = L.o_dact + 4u * n_dot;
  L.o_mpad = L.o_mdend + 4u * n_mem;
  L.o_def = pad_to(L.o_mpad, 8);
  L.o_fctr = L.o_def;
  L.o_fkey = L.o_fctr + 8u * n_def_dot;
  L.o_fact = L.o_fkey + 8u * n_def_mem;
  L.o_fdend = L.o_fact + 4u * n_def_dot;
  L.o_fmend = L.o_fdend + 4u * n_def;
  L.o_end = L.o_fmend + 4u * n_def;
  L.size = pad_to(L.o_end, 16);
}

CRDT_HD uint64_t record_size64(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot, uint32_t n_def,
                               uint32_t n_def_dot, uint32_t n_def_mem) {
  uint64_t b = kHdrBytes + 8ull * n_clk + 12ull * ((uint64_t)n_mem + n_dot);
  b = (b + 7) & ~7ull;
  b += 12ull * n_def_dot + 8ull * n_def_mem + 8ull * n_def;
  return (b + 15) & ~15ull;
}

}  // namespace crdts_hip
