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
constexpr uint32_t kSparseClock = 1;  // header flags bit 0: CSR top clock (CRDT_ORSWOT_SPARSE_CLOCK)

// Byte offsets of every section of one record, from its counts.
struct RecLayout {
  uint32_t n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem;
  uint32_t o_clk, o_cact, o_key, o_dctr, o_dact, o_mdend, o_mpad;  // clock + member block
  uint32_t o_def, o_fctr, o_fkey, o_fact, o_fdend, o_fmend, o_end, size;
};

CRDT_HD uint32_t pad_to(uint32_t x, uint32_t a) { return (x + a - 1) & ~(a - 1); }

// Bytes of the top-clock section: dense u64[n_clk], or sparse (CSR) u64
// ctr[n_clk] + u32 act[n_clk] zero-padded to 8.
CRDT_HD uint32_t clock_bytes(uint32_t n_clk, bool sparse) { return sparse ? pad_to(12u * n_clk, 8) : 8u * n_clk; }

// Member-block end (8-aligned) for the given counts.
CRDT_HD uint32_t member_block_end(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot, bool sparse = false) {
  return pad_to(kHdrBytes + clock_bytes(n_clk, sparse) + 12u * (n_mem + n_dot), 8);
}

CRDT_HD void rec_layout(RecLayout& L, uint32_t n_clk, uint32_t n_mem, uint32_t n_dot,
                        uint32_t n_def, uint32_t n_def_dot, uint32_t n_def_mem, bool sparse = false) {
  L.n_clk = n_clk; L.n_mem = n_mem; L.n_dot = n_dot;
  L.n_def = n_def; L.n_def_dot = n_def_dot; L.n_def_mem = n_def_mem;
  L.o_clk = kHdrBytes;
  L.o_cact = L.o_clk + 8u * n_clk;
  L.o_key = L.o_clk + clock_bytes(n_clk, sparse);
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
                               uint32_t n_def_dot, uint32_t n_def_mem, bool sparse = false) {
  const uint64_t cb = sparse ? ((12ull * n_clk + 7) & ~7ull) : 8ull * n_clk;
  uint64_t b = kHdrBytes + cb + 12ull * ((uint64_t)n_mem + n_dot);
  b = (b + 7) & ~7ull;
  b += 12ull * n_def_dot + 8ull * n_def_mem + 8ull * n_def;
  return (b + 15) & ~15ull;
}

}  // namespace crdts_hip
