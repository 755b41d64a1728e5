// Internal launch entry points (the C ABI in api.hip validates and calls these).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/crdts_hip.h"

namespace crdts_hip {

// The join launches' sequence on one context (its control-word set
// alternates per launch; dirty: zero both sets before the next launch).
struct JoinSeq {
  uint32_t seq;
  bool dirty;
};
int launch_orswot_merge(const uint8_t* Lb, const uint64_t* Loff, uint64_t Lbytes, const uint8_t* Rb,
                        const uint64_t* Roff, uint64_t Rbytes, uint8_t* Ob, uint64_t* Ooff,
                        uint64_t Obytes, uint64_t n_obj, uint32_t n_actors, int* status, uint32_t* ctl,
                        uint64_t* list, uint32_t list_cap, hipStream_t stream, int blocks_per_cu,
                        int variant, JoinSeq* js);

int launch_orswot_merge_sparse(const uint8_t* Lb, const uint64_t* Loff, uint64_t Lbytes, const uint8_t* Rb,
                               const uint64_t* Roff, uint64_t Rbytes, uint8_t* Ob, uint64_t* Ooff, uint64_t Obytes,
                               uint64_t n_obj, uint32_t n_actors, int* status, uint32_t* ctl, uint64_t* list,
                               uint32_t list_cap, hipStream_t stream, int sparse_variant, JoinSeq* js);

// Sparse clock joins: n_jobs (1 or 2: PNCounter's P and N) batches in one launch.
int launch_clock_csr_merge(const crdt_clock_csr* const* self, const crdt_clock_csr* const* other,
                           const crdt_clock_csr_out* const* out, int n_jobs, int* status, hipStream_t stream);

int launch_orswot_truncate(const crdt_orswot_batch& self, const crdt_clock_csr& clocks, uint32_t A, uint32_t flags,
                           uint8_t* out, uint64_t* out_off, uint64_t out_bytes, int* status, uint32_t* ctl,
                           uint64_t* list, uint32_t list_cap, hipStream_t stream);

int launch_dense_max(uint64_t* self, const uint64_t* other, uint64_t n_words, hipStream_t stream);

int launch_orswot_validate(const uint8_t* base, const uint64_t* off, uint64_t bytes, uint64_t n_obj,
                           uint32_t n_actors, uint32_t flags, int* status, hipStream_t stream);

// Bounds-checked record sizes (size 0 + CRDT_ENONCANON latched for a record
// out of [0, bytes)), and the copy of sizes[i] bytes per record.
int launch_record_sizes(const uint8_t* base, const uint64_t* off, uint64_t bytes, uint64_t n_obj, uint64_t* sizes,
                        int* status, hipStream_t stream);
// records whose [dst_off, dst_off + size) does not fit dst_bytes are not copied
int launch_record_copy(const uint8_t* src, const uint64_t* src_off, const uint64_t* sizes, uint8_t* dst,
                       const uint64_t* dst_off, uint64_t n_obj, uint64_t dst_bytes, hipStream_t stream);

int launch_bincode_bounds(const uint64_t* blen, uint64_t n_obj, uint32_t wa, uint32_t wm, uint32_t A,
                          uint32_t flags, uint64_t* bounds, hipStream_t stream);
// decode (sizes == null): objects past the LDS scratch are listed (list,
// list_cap) and decoded by a large-object kernel from big_scratch
// (launch_bincode_big_scratch_bytes()).
int launch_bincode_ingest(const uint8_t* blobs, uint64_t blob_bytes, const uint64_t* boff, const uint64_t* blen,
                          uint64_t n_obj, uint32_t wa, uint32_t wm, uint32_t A, uint32_t flags, uint64_t* sizes,
                          uint8_t* out, const uint64_t* ooff, uint64_t out_bytes, int* status, uint32_t* ctl, hipStream_t stream,
                          uint64_t* dbg = nullptr, uint64_t* list = nullptr, uint32_t list_cap = 0,
                          uint8_t* big_scratch = nullptr, int walk = 0);
size_t launch_bincode_big_scratch_bytes();
int launch_bincode_egest(const uint8_t* rb, uint64_t rbytes, const uint64_t* roff, uint64_t n_obj, uint32_t A,
                         uint32_t flags, uint32_t wa, uint32_t wm, uint64_t* sizes, uint8_t* out,
                         const uint64_t* ooff, uint64_t out_bytes, int* status, uint32_t* ctl, hipStream_t stream);

int launch_orswot_apply(const uint8_t* sb, uint64_t sbytes, const uint64_t* soff, uint64_t n_obj,
                        const uint64_t* obj_end, const uint32_t* kind, const uint64_t* member, const uint32_t* actor,
                        const uint64_t* counter, const uint64_t* clk_end, const uint32_t* clk_act,
                        const uint64_t* clk_ctr, uint64_t n_ops, uint64_t n_clk, uint32_t A, uint32_t flags,
                        uint8_t* out, uint64_t* ooff,
                        uint64_t out_bytes, int* status, uint32_t* ctl, uint64_t* list, uint32_t list_cap,
                        uint8_t* huge_ws, hipStream_t stream);
// HBM workspace of the apply's third tier (objects past the LDS workspaces)
size_t launch_apply_huge_scratch_bytes();

int launch_vclock_cmp(const uint64_t* a, const uint64_t* b, uint64_t n, uint32_t A, int8_t* out, hipStream_t stream);
int launch_mvreg_merge(const uint32_t* sn, const uint64_t* sclk, const uint64_t* sval, uint32_t scap,
                       const uint32_t* on, const uint64_t* oclk, const uint64_t* oval, uint32_t ocap, uint32_t* outn,
                       uint64_t* outclk, uint64_t* outval, uint32_t outcap, uint64_t n_obj, uint32_t A, int* status,
                       hipStream_t stream);

int launch_map_mvreg_merge(const crdt_map_mvreg_slab& S, const crdt_map_mvreg_slab& O, const crdt_map_mvreg_slab& R,
                           uint64_t n_obj, uint32_t A, int* status, uint32_t* ctl, hipStream_t stream, int variant = 0);
// The nested map's inner pass (map_map.hip): task t merges S row tsrc[2t]
// with O row tsrc[2t + 1] (~0: an absent side) into R row t, truncated by Tb
// row t when it is non-empty (one pass: no intermediate slab).
int launch_map_mvreg_merge_tasks(const crdt_map_mvreg_slab& S, const crdt_map_mvreg_slab& O,
                                 const crdt_map_mvreg_slab& R, const uint64_t* tsrc, const uint64_t* Tb,
                                 uint64_t n_tasks, uint32_t slots, uint32_t A, int* status, uint32_t* ctl,
                                 hipStream_t stream);
size_t map_map_scratch_bytes(const crdt_map_map_slab& R, uint64_t n_obj, uint32_t A);
int launch_map_map_merge(const crdt_map_map_slab& S, const crdt_map_map_slab& O, const crdt_map_map_slab& R,
                         uint64_t n_obj, uint32_t A, uint8_t* scratch, int* status, uint32_t* ctl,
                         hipStream_t stream);
int launch_map_orswot_merge(const crdt_map_orswot_slab& S, const crdt_map_orswot_slab& O,
                            const crdt_map_orswot_slab& R, uint64_t n_obj, uint32_t A, int* status, uint32_t* ctl,
                            hipStream_t stream, int variant = 0);
size_t map_orswot_lds_bytes(const crdt_map_orswot_slab& S, const crdt_map_orswot_slab& O, uint32_t A);

}  // namespace crdts_hip
