// The context behind the opaque crdt_ctx of include/crdts_hip.h (internal).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/crdts_hip.h"
#include "kernels.h"

namespace crdts_hip {
// Device scratch of a context: status word, the general-path object list
// and its control words. A context serves one stream at a time.
constexpr uint32_t kDefaultListCap = 1u << 16;
// Per-wave sink for the lane-predicated global stores of the join kernels
// (a lane with nothing to store writes here instead of branching around the
// store, so every object issues the same stores): kTrashWaves x 64 B, right
// after the list in the context's scratch.
constexpr uint32_t kTrashWaves = 8192;
constexpr size_t kTrashBytes = 64ull * kTrashWaves;
// Objects with deferred removes, listed by the join pass for the deferred
// pass (after the sink); past kDeferListCap entries the deferred pass scans
// the output offsets for their flag instead.
constexpr uint32_t kDeferListCap = 1u << 20;
}  // namespace crdts_hip

struct crdt_ctx {
  int device;
  int* d_status;        // d_scratch + 0
  uint32_t* d_ctl;      // d_scratch + 16: [list count, scan flag, deferred count, chunk tickets] (+ spare)
  uint64_t* d_list;     // d_scratch + 64
  uint32_t list_cap;
  int blocks_per_cu;    // diagnostic builds only (crdt_ctx_set_blocks_per_cu)
  int variant;          // diagnostic builds only (crdt_ctx_set_variant); 0 = the product kernels
  // the Orswot join's launch sequence: alternate launches use the control
  // words ctl[4..7] / ctl[8..11] (launch_orswot_merge, no memset)
  crdts_hip::JoinSeq join_seq{0u, false};
  // replica anti-entropy (replica.hip): the RCCL communicator this context
  // owns (ncclComm_t; null until crdt_comm_init) and a growable device arena
  void* comm = nullptr;
  int n_ranks = 0, rank = 0;
  uint64_t* d_comm_stage = nullptr;  // device staging of the small all-gathers
  uint8_t* d_arena = nullptr;
  size_t arena_bytes = 0;
  size_t arena_limit = 0;  // largest arena the context may allocate (0: no limit; crdt_ctx_set_arena_limit)
  // HBM scratch of the large-object paths (bincode ingest, apply), allocated
  // on first use
  uint8_t* d_big = nullptr;
  size_t big_bytes = 0;
  // host synchronisations made by the replica joins so far (crdt_ctx_host_syncs)
  uint64_t host_syncs = 0;
  // crdt_orswot_fold's intermediate batches (two, ping-pong), grown on demand
  uint8_t* d_fold = nullptr;
  size_t fold_bytes = 0;
};

// Ensures ctx->d_big holds at least `bytes` (api.hip).
int ctx_big_scratch(crdt_ctx* ctx, size_t bytes);
