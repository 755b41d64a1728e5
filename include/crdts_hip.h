/*
 * crdts_hip.h — C ABI of the MI355X batched CRDT merge engine.
 *
 * This is the drop-in boundary for ONE path of etsangsplk/rust-crdt (crate
 * `crdts` 1.3.0): the state-based join
 *
 *     pub trait CvRDT { fn merge(&mut self, other: &Self); }   // src/traits.rs:9-12
 *
 * for VClock (src/vclock.rs:131-137), GCounter (src/gcounter.rs:58-62),
 * PNCounter (src/pncounter.rs:90-95) and Orswot incl. deferred removes
 * (src/orswot.rs:87-157, 195-211, 235-243). The reference merges ONE pair per
 * call; every entry point here merges a BATCH of independent pairs
 * (self[i] ⊔= other[i]) on one MI355X, with per-object results bit-exact with
 * calling the reference `merge` on each pair.
 *
 * Conventions
 *  - Plain pointers and sizes only. Pointers named `d_*` are DEVICE pointers
 *    (hipMalloc'd or torch tensors' data_ptr), `h_*` are host pointers.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *  - Return 0 on success, a negative CRDT_E* code otherwise. Nothing aborts.
 *    Launches are asynchronous: argument errors are returned immediately,
 *    record-level errors found by a kernel (non-canonical / oversized input)
 *    are latched in the context and returned by crdt_ctx_status().
 *  - The caller owns every buffer. A crdt_ctx owns only a small device status
 *    word; distinct contexts may be used from distinct threads concurrently.
 *  - Orientation is fixed and matters (Orswot merge is structurally
 *    non-commutative, src/orswot.rs:98-103 vs :132-137):
 *    output = self.merge(&other), exactly.
 *
 * Actors are interned by the caller to dense u32 ids in the same order as the
 * reference's `Ord` on actors (BTreeMap order, src/vclock.rs:54-57); members
 * are interned to u64 keys bijectively (the caller's intern table).
 */
#ifndef CRDTS_HIP_H
#define CRDTS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRDT_ABI_VERSION 1

#define CRDT_OK 0
#define CRDT_EINVAL (-1)     /* bad argument (null pointer, zero actors, misaligned) */
#define CRDT_ENONCANON (-2)  /* an input record is not canonical / inconsistent     */
#define CRDT_EHIP (-3)       /* HIP runtime error                                  */
#define CRDT_ECAPACITY (-4)  /* output capacity too small                          */
#define CRDT_ECOMM (-5)      /* RCCL / communicator error                          */
#define CRDT_ENODEV (-6)     /* no usable gfx950 device                            */

typedef struct crdt_ctx crdt_ctx;

/* Context: binds a device and owns a device-side status word. */
int crdt_ctx_create(crdt_ctx** out, int device);
int crdt_ctx_destroy(crdt_ctx* ctx);
/* Synchronizes `stream`, returns the first record-level error latched by any
 * kernel launched through ctx since the last call (and clears it). */
int crdt_ctx_status(crdt_ctx* ctx, void* stream);
const char* crdt_strerror(int code);
int crdt_abi_version(void);
/* Capacity (<= 65536, the default) of the context's list of objects handed
 * from the fast Orswot / apply kernels to their general kernels (an Orswot
 * merge splits it in two halves: the general kernel's objects and the big
 * objects the join hands straight to the block-per-object kernel). Past a
 * list's capacity the kernels scan every output offset instead; results are
 * identical. Lowering it exercises that overflow path (tests). */
int crdt_ctx_set_list_cap(crdt_ctx* ctx, uint32_t cap);
/* Host synchronisations with the device (stream waits) the context's replica
 * joins have made so far (crdt_orswot_replica_join*: 3 per call in the steady
 * state). A counter for callers that profile the join's per-step cost. */
uint64_t crdt_ctx_host_syncs(const crdt_ctx* ctx);
/* Largest device arena (bytes) the context may allocate for the replica
 * exchanges (crdt_orswot_replica_join*, crdt_replica_*_max_transport);
 * 0 (the default) = no limit. A call whose arena would exceed it returns
 * CRDT_ECAPACITY on every rank of the exchange (the verdict is all-gathered
 * before any data moves), and the context keeps the arena it had. */
int crdt_ctx_set_arena_limit(crdt_ctx* ctx, size_t max_bytes);

/* ------------------------------------------------------------------------ *
 * Dense clocks and counters.
 *
 * Layout: row-major u64[n_obj][n_actors]; row i is one VClock / GCounter, slot
 * a holds the counter of interned actor a, 0 = absent (canonical: the
 * reference never stores a 0, `witness` src/vclock.rs:159-163).
 *
 * self[i] := pointwise max(self[i], other[i]), in place.
 *   VClock::merge   src/vclock.rs:131-137   (witness loop == pointwise max)
 *   GCounter::merge src/gcounter.rs:58-62   (delegates to VClock::merge)
 *   PNCounter::merge src/pncounter.rs:90-95 (P and N rows: pass the [P|N]
 *                    row of 2*n_actors slots, see crdt_pncounter_merge)
 * ------------------------------------------------------------------------ */
int crdt_vclock_dense_merge(crdt_ctx* ctx, uint64_t* d_self, const uint64_t* d_other,
                            size_t n_obj, uint32_t n_actors, void* stream);
int crdt_gcounter_merge(crdt_ctx* ctx, uint64_t* d_self, const uint64_t* d_other,
                        size_t n_obj, uint32_t n_actors, void* stream);
/* PNCounter row = P slots [0, n_actors) then N slots [n_actors, 2*n_actors). */
int crdt_pncounter_merge(crdt_ctx* ctx, uint64_t* d_self, const uint64_t* d_other,
                         size_t n_obj, uint32_t n_actors, void* stream);

/* The same with HOST rows (H2D, merge, D2H, synchronous): the PCIe-inclusive
 * path of a host `merge_batch(&mut [T], &[T])` for VClock / GCounter
 * (n_slots = n_actors) and PNCounter (n_slots = 2 * n_actors, [P|N] rows). */
int crdt_dense_merge_host(crdt_ctx* ctx, uint64_t* h_self, const uint64_t* h_other, size_t n_obj,
                          uint32_t n_slots);

/* ------------------------------------------------------------------------ *
 * Sparse (CSR) clocks and counters, for actor universes too large for dense
 * rows (a 1024-actor universe with ~48 actors per
 * clock is 8 KB dense and ~0.6 KB here). The reference clock is a
 * BTreeMap<A, u64> (src/vclock.rs:54-57): here object i's clock is the run
 * of entries [off[i], off[i] + len[i]) of act / ctr — actors strictly
 * increasing (BTreeMap order of the interned ids), counters > 0 (`witness`
 * never stores 0, :159-163). A batch may have gaps between runs.
 *
 * out[i] := self[i].merge(&other[i]): the sorted union of the two runs with
 * the larger counter per actor — VClock::merge src/vclock.rs:131-137;
 * GCounter::merge src/gcounter.rs:58-62; PNCounter::merge
 * src/pncounter.rs:90-95 (its P and N clocks are two batches). The call
 * writes out.off[i] := self.off[i] + other.off[i] and out.len[i] := the
 * union's length (<= self.len[i] + other.len[i]), and the entries there, so
 * out.n_entries >= self.n_entries + other.n_entries suffices and the output
 * is itself a valid (gapped) input batch.
 * PRECONDITION (checked on the device; a violation latches CRDT_EINVAL and
 * the object's out.len is 0): on each side runs lie inside [0, n_entries)
 * at increasing, non-overlapping offsets (off[i] + len[i] <= off[i+1]). A
 * run that is not canonical (actors not strictly increasing, a zero counter)
 * latches CRDT_ENONCANON (out.len 0). Runs of any length (<= 64 entries per
 * side take the loop-free path).
 * ------------------------------------------------------------------------ */
typedef struct crdt_clock_csr {
  const uint64_t* off;   /* device, n_obj: first entry of object i's run */
  const uint32_t* len;   /* device, n_obj: entries of the run            */
  const uint32_t* act;   /* device, n_entries: interned actor ids          */
  const uint64_t* ctr;   /* device, n_entries: counters                    */
  size_t n_obj;
  size_t n_entries;      /* extent of act / ctr (bounds checks)            */
} crdt_clock_csr;
typedef struct crdt_clock_csr_out {
  uint64_t* off;         /* device, n_obj (written)                        */
  uint32_t* len;         /* device, n_obj (written)                        */
  uint32_t* act;         /* device, n_entries                              */
  uint64_t* ctr;         /* device, n_entries                              */
  size_t n_entries;
} crdt_clock_csr_out;
int crdt_vclock_csr_merge(crdt_ctx* ctx, const crdt_clock_csr* self, const crdt_clock_csr* other,
                          const crdt_clock_csr_out* out, void* stream);
int crdt_gcounter_csr_merge(crdt_ctx* ctx, const crdt_clock_csr* self, const crdt_clock_csr* other,
                            const crdt_clock_csr_out* out, void* stream);
/* PNCounter: its P and N clocks as two batches of the same n_obj (one call). */
int crdt_pncounter_csr_merge(crdt_ctx* ctx, const crdt_clock_csr* self_p, const crdt_clock_csr* self_n,
                             const crdt_clock_csr* other_p, const crdt_clock_csr* other_n,
                             const crdt_clock_csr_out* out_p, const crdt_clock_csr_out* out_n, void* stream);

/* ------------------------------------------------------------------------ *
 * Orswot canonical record (one object = one contiguous, self-describing
 * record; a batch = a byte buffer + a u64 byte offset per object).
 *
 * The reference state is (src/orswot.rs:26-30)
 *     clock:    VClock<A>
 *     entries:  HashMap<M, VClock<A>>
 *     deferred: HashMap<VClock<A>, HashSet<M>>
 * and equality is structural (`#[derive(PartialEq)]`, src/orswot.rs:25). The
 * record is the canonical form of that state: hash-map order is replaced by
 * sorted order, so two states are equal iff their records are byte-equal.
 *
 * Record = header (32 B) followed by a MEMBER block and a DEFERRED block.
 * Every section is densely packed; the member block is zero-padded to a
 * multiple of 8 bytes and the record to a multiple of 16 bytes:
 *   u64 clk_ctr [n_clk]      top clock, DENSE: n_clk == n_actors, 0 = absent
 *   -- member block (entries: HashMap<M, VClock<A>>) --
 *   u64 mem_key [n_mem]      member keys, strictly increasing
 *   u64 dot_ctr [n_dot]      member clocks' counters, member-major
 *   u32 dot_act [n_dot]      member clocks' actors, strictly increasing per member
 *   u32 mem_dend[n_mem]      cumulative end of member m's dots (member m owns
 *                            dots [mem_dend[m-1], mem_dend[m]), mem_dend[-1]=0)
 *   (pad to 8)
 *   -- deferred block (deferred: HashMap<VClock<A>, HashSet<M>>) --
 *   u64 def_ctr [n_def_dot]  deferred clocks' counters, clock-major
 *   u64 def_key [n_def_mem]  deferred member sets, clock-major, each strictly increasing
 *   u32 def_act [n_def_dot]  deferred clocks' actors, strictly increasing per clock
 *   u32 def_dend[n_def]      cumulative end of deferred clock d's dots
 *   u32 def_mend[n_def]      cumulative end of deferred clock d's member keys
 *   (pad to 16)
 * SPARSE (CSR) top clock — header flags bit 0 (CRDT_ORSWOT_SPARSE_CLOCK), for
 * large actor universes (BASELINE.json configs[4]): the
 * top-clock section is instead
 *   u64 clk_ctr [n_clk]      counters of the clock's n_clk = nnz actors
 *   u32 clk_act [n_clk]      their actor ids, strictly increasing, < n_actors
 *   (pad to 8)
 * and everything after it is unchanged. A batch is either all dense (flags 0,
 * n_clk == n_actors) or all sparse (flags 1, counters > 0).
 * Canonical: every counter stored in a run is > 0, every member clock, every
 * deferred clock and every deferred member set is non-empty, and deferred
 * clocks are strictly increasing in CLOCK ORDER = lexicographic order of their
 * (actor, counter) sequences, a proper prefix ordering first.
 * ------------------------------------------------------------------------ */
typedef struct crdt_orswot_hdr {
  uint32_t size;      /* record bytes (header included), multiple of 16 */
  uint32_t n_clk;     /* dense top clock slots (== batch n_actors)      */
  uint32_t n_mem;
  uint32_t n_dot;
  uint32_t n_def;
  uint32_t n_def_dot;
  uint32_t n_def_mem;
  uint32_t flags;     /* 0 (dense top clock) or CRDT_ORSWOT_SPARSE_CLOCK  */
} crdt_orswot_hdr;

#define CRDT_ORSWOT_SPARSE_CLOCK 1u
/* Header flags bit 1: the record holds a member whose clock is EMPTY (an
 * empty run). Only Causal::truncate produces one (crdt_orswot_truncate: the
 * reference keeps such a member, src/orswot.rs:167-169); it is not a
 * canonical input of the merge, apply and codec entry points, which reject
 * it (CRDT_ENONCANON). */
#define CRDT_ORSWOT_EMPTY_MEMBER_CLOCK 2u

#define CRDT_ORSWOT_HDR_BYTES 32u
#define CRDT_RECORD_ALIGN 16u

/* Bytes of a record with these counts (header and padding included). */
size_t crdt_orswot_record_bytes(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot,
                                uint32_t n_def, uint32_t n_def_dot, uint32_t n_def_mem);
/* Same for either clock form (flags: 0 or CRDT_ORSWOT_SPARSE_CLOCK). */
size_t crdt_orswot_record_bytes_ex(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot,
                                   uint32_t n_def, uint32_t n_def_dot, uint32_t n_def_mem,
                                   uint32_t flags);

/* A batch of records: record i starts at d_base + d_off[i] (16-B aligned). */
typedef struct crdt_orswot_batch {
  const uint8_t* base;   /* device */
  const uint64_t* off;   /* device, n_obj entries */
  size_t n_obj;
  size_t bytes;          /* extent of base, for bounds checks */
} crdt_orswot_batch;

/*
 * out[i] := self[i].merge(&other[i])   — src/orswot.rs:87-157 incl.
 * apply_deferred (:235-243) / apply_remove (:195-211).
 *
 * The output record i is written at d_out_base + d_out_off[i] where
 * d_out_off[i] := self.off[i] + other.off[i] (written by the kernel). Because a
 * merged record is never larger than the two inputs together, the output
 * needs at most self.bytes + other.bytes bytes and no prefix scan: the output
 * batch (d_out_base, d_out_off) is itself a valid input batch (it may have
 * gaps between records; crdt_orswot_compact removes them).
 * PRECONDITION (checked on the device; a violation latches CRDT_EINVAL and
 * the offending objects are not written): on each side the records are in
 * increasing offset order and do not overlap, off[i] + size[i] <= off[i+1],
 * so that the output records cannot overlap either. Packed batches, merge
 * outputs (with gaps) and compacted batches all satisfy it.
 * `n_actors` is the dense top-clock width shared by every record.
 */
int crdt_orswot_merge(crdt_ctx* ctx, const crdt_orswot_batch* self,
                      const crdt_orswot_batch* other, uint8_t* d_out_base,
                      uint64_t* d_out_off, size_t out_bytes, uint32_t n_actors,
                      void* stream);

/* crdt_orswot_merge for either clock form: flags = 0 (dense top clocks,
 * n_actors slots) or CRDT_ORSWOT_SPARSE_CLOCK (CSR top clocks over an actor
 * universe of n_actors ids; the output records are sparse too). Same output
 * placement and bounds. */
int crdt_orswot_merge_ex(crdt_ctx* ctx, const crdt_orswot_batch* self,
                         const crdt_orswot_batch* other, uint8_t* d_out_base,
                         uint64_t* d_out_off, size_t out_bytes, uint32_t n_actors,
                         uint32_t flags, void* stream);

/* Same with host buffers: H2D, merge, D2H, synchronous (PCIe-inclusive path
 * used by a host `merge_batch(&mut [T], &[T])`). h_out_off receives offsets
 * into h_out_base (compacted, so h_out_bytes >= sum of merged record sizes
 * suffices; worst case h_self_bytes + h_other_bytes). */
int crdt_orswot_merge_host(crdt_ctx* ctx, const uint8_t* h_self_base,
                           const uint64_t* h_self_off, size_t self_bytes,
                           const uint8_t* h_other_base, const uint64_t* h_other_off,
                           size_t other_bytes, size_t n_obj, uint32_t n_actors,
                           uint8_t* h_out_base, uint64_t* h_out_off, size_t h_out_bytes,
                           size_t* h_out_used);

/* The replica fold, batched: out[i] := ((reps[0][i] ⊔ reps[1][i]) ⊔ reps[2][i])
 * ⊔ ... ⊔ reps[n_reps-1][i] — Orswot::merge (src/orswot.rs:87-157) in rank
 * order, the fold of replica anti-entropy (BASELINE.json configs[4]) — over
 * n_reps batches of the same n_obj objects: n_reps - 1 batched merges
 * (crdt_orswot_merge_ex) with the intermediate batches in a context-owned
 * buffer. flags: 0 (dense top clocks) or CRDT_ORSWOT_SPARSE_CLOCK. Output
 * record i at d_out_off[i] := sum_r reps[r].off[i] (written by the call);
 * out_bytes >= sum_r reps[r].bytes. Each batch: records in increasing offset
 * order, not overlapping (as crdt_orswot_merge). (A fused form — one wave
 * folding an object's records with the accumulator in LDS, no intermediate
 * batch in HBM — measured slower on config 5: the fold is bound by the joins,
 * not by the intermediate bytes; DESIGN.md.) */
int crdt_orswot_fold(crdt_ctx* ctx, const crdt_orswot_batch* reps, uint32_t n_reps, uint32_t n_actors,
                     uint32_t flags, uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, void* stream);

/* Deep canonical-form check of a batch on the device (sortedness, non-zero
 * counters, non-empty runs, section sizes). Result via crdt_ctx_status. */
int crdt_orswot_validate(crdt_ctx* ctx, const crdt_orswot_batch* batch,
                         uint32_t n_actors, void* stream);
int crdt_orswot_validate_ex(crdt_ctx* ctx, const crdt_orswot_batch* batch,
                            uint32_t n_actors, uint32_t flags, void* stream);

/* Remove gaps: copies records into d_dst contiguously; d_dst_off receives the
 * new offsets. d_scratch needs crdt_orswot_compact_scratch_bytes(n_obj). */
size_t crdt_orswot_compact_scratch_bytes(size_t n_obj);
int crdt_orswot_compact(crdt_ctx* ctx, const crdt_orswot_batch* src, uint8_t* d_dst,
                        uint64_t* d_dst_off, size_t dst_bytes, void* d_scratch,
                        void* stream);

/* ------------------------------------------------------------------------ *
 * Replica anti-entropy across GPUs over RCCL (xGMI) — SURVEY.md §8(b),(e);
 * BASELINE.json configs[3] (dense) and configs[4] (Orswot). One process (or
 * thread) per GPU, each holding a full replica of the same n objects. The
 * context owns one RCCL communicator:
 *   rank 0:     crdt_comm_unique_id(id), then the caller distributes the
 *               CRDT_COMM_ID_BYTES bytes to every rank (its own channel);
 *   every rank: crdt_comm_init(ctx, id, n_ranks, rank)     (collective).
 * Every collective entry point below must be called by every rank, in the
 * same order, on the stream each rank passes. A failure found on one rank
 * (bad batch, capacity, a non-canonical record) is returned by all ranks.
 * ------------------------------------------------------------------------ */
#define CRDT_COMM_ID_BYTES 128
int crdt_comm_unique_id(uint8_t* h_id);
int crdt_comm_init(crdt_ctx* ctx, const uint8_t* h_id, int n_ranks, int rank);
/* Also done by crdt_ctx_destroy. */
int crdt_comm_destroy(crdt_ctx* ctx);

/* *h_count := the number of ranks of the context's communicator (ncclCommCount). */
int crdt_comm_count(crdt_ctx* ctx, int* h_count);

/* Dense rows (VClock / GCounter / PNCounter rows, any width): d_rows[k] :=
 * max over ranks of d_rows[k], k < n_words, in place and in u64 order
 * (ncclAllReduce, ncclUint64, ncclMax; chunks of <= 1 GiB). It is
 * VClock::merge (src/vclock.rs:131-137) across replicas: a pointwise max,
 * commutative and associative, so the reduction order cannot change a bit. */
int crdt_replica_allreduce_max(crdt_ctx* ctx, uint64_t* d_rows, size_t n_words, void* stream);
/* The owner-shard variant: rank r receives in
 * d_shard the max over ranks of words [r n/N, (r+1) n/N) of d_rows (one
 * ncclReduceScatter, ncclUint64 + ncclMax); n_words must be a multiple of
 * the rank count. */
int crdt_replica_reduce_scatter_max(crdt_ctx* ctx, const uint64_t* d_rows, size_t n_words, uint64_t* d_shard,
                                    void* stream);

/* Orswot replicas: out[i] = ((r0[i] ⊔ r1[i]) ⊔ r2[i]) ⊔ ... ⊔ r_{N-1}[i], the
 * same bytes on every rank (the join is structurally non-commutative,
 * src/orswot.rs:98-103 vs :132-138, so the fold order is fixed: rank order).
 * Owner-sharded: the objects are split into N contiguous ranges; rank j
 * receives every replica's slice of range j point-to-point, folds it in rank
 * order with the batched merge kernel (crdt_orswot_merge_ex), compacts it,
 * and the folded ranges are exchanged back. Per rank: 1/N of the fold work
 * and about 2(N-1)/N of one replica's bytes sent and received.
 * `mine`: this rank's replica (the same n_obj on every rank; records in
 * increasing, non-overlapping offset order). The output is a packed batch,
 * record i at d_out + d_out_off[i], *h_out_used = its extent in bytes;
 * out_bytes >= crdt_orswot_replica_join_bound() suffices (the sum of every
 * rank's replica bytes, a collective). Synchronous: returns when the output
 * is complete on `stream`. A status an earlier launch on a rank's context
 * latched and the caller has not read (crdt_ctx_status) is that rank's error
 * in the join: every rank returns it, and the status is cleared. */
int crdt_orswot_replica_join_bound(crdt_ctx* ctx, const crdt_orswot_batch* mine, size_t* h_bound, void* stream);
int crdt_orswot_replica_join(crdt_ctx* ctx, const crdt_orswot_batch* mine, uint32_t n_actors, uint32_t flags,
                             uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, size_t* h_out_used,
                             void* stream);
/* The same owner-sharded join over a transport of the caller's (one process
 * per rank; e.g. gloo, MPI or a host network instead of RCCL) — no
 * communicator needed on ctx. The code above the transport is
 * crdt_orswot_replica_join's.
 *   allgather: blocking; every rank contributes n u64 (h_in), h_out receives
 *     n_ranks * n of them in rank order. Returns 0 or non-zero on failure.
 *   exchange: device transfers; every send {peer, src, bytes} is matched, in
 *     list order per peer, by that peer's recv {me, dst, bytes} of the same
 *     size (sends and recvs with peer == rank are local copies, k-th to
 *     k-th). src data is produced on `stream`; the transfers must be
 *     complete, or ordered before later work on `stream`, when it returns.
 *     Zero-byte entries move nothing. Returns 0 or non-zero on failure.
 * A transport failure returns CRDT_ECOMM. */
typedef struct crdt_xfer {
  int peer;
  const void* src;  /* device, sends */
  void* dst;        /* device, recvs */
  size_t bytes;
} crdt_xfer;
typedef struct crdt_transport {
  int n_ranks, rank;
  void* user;
  int (*allgather)(void* user, const uint64_t* h_in, size_t n, uint64_t* h_out);
  int (*exchange)(void* user, const crdt_xfer* sends, size_t n_sends, const crdt_xfer* recvs, size_t n_recvs,
                  void* stream);
} crdt_transport;
int crdt_orswot_replica_join_transport(crdt_ctx* ctx, const crdt_transport* transport,
                                       const crdt_orswot_batch* mine, uint32_t n_actors, uint32_t flags,
                                       uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, size_t* h_out_used,
                                       void* stream);
/* crdt_replica_allreduce_max over a transport of the caller's (above; no
 * communicator needed): rank j owns words [j n/N, (j+1) n/N) (the remainder
 * spread over the first ranks); each rank sends every peer its range, folds
 * the received copies of its own range with the dense max kernel, and sends
 * the result to every peer — the same bits as the RCCL all-reduce on every
 * rank (a pointwise max, src/vclock.rs:131-137). Uses the context's arena
 * for (N - 1) / N of the rows; synchronous: returns when d_rows is complete. */
int crdt_replica_allreduce_max_transport(crdt_ctx* ctx, const crdt_transport* transport, uint64_t* d_rows,
                                         size_t n_words, void* stream);
/* crdt_replica_reduce_scatter_max over a caller transport: rank r receives in
 * d_shard the max over ranks of words [r n/N, (r+1) n/N) of d_rows (n_words a
 * multiple of N) — its own copy of the range maxed with the N - 1 copies its
 * peers send it (the dense max kernel). Synchronous. */
int crdt_replica_reduce_scatter_max_transport(crdt_ctx* ctx, const crdt_transport* transport,
                                              const uint64_t* d_rows, size_t n_words, uint64_t* d_shard,
                                              void* stream);
/* The same owner-sharded join over n_replicas (<= 64) replicas resident on
 * this context's device: each replica is a virtual rank (a host thread with
 * its own context and stream) and device copies are the transport; the code
 * below the transport is crdt_orswot_replica_join's. For single-GPU
 * rehearsal and tests of the exchange. out_bytes >= the sum of the replicas'
 * (16-B aligned) bytes suffices. No communicator needed. */
int crdt_orswot_replica_join_local(crdt_ctx* ctx, const crdt_orswot_batch* replicas, uint32_t n_replicas,
                                   uint32_t n_actors, uint32_t flags, uint8_t* d_out, uint64_t* d_out_off,
                                   size_t out_bytes, size_t* h_out_used, void* stream);

/* ------------------------------------------------------------------------ *
 * Host-side helpers (no device work).
 * ------------------------------------------------------------------------ */

/* Synthetic Orswot pair batches by op simulation (Orswot::apply,
 * src/orswot.rs:61-85), identical for any sharding: object i draws from the
 * SplitMix64 stream seeded with (seed ^ i). Both sides share an ancestor
 * built from `ancestor_adds` adds of distinct members over all actors (each actor starting from a
 * random 40-bit counter base, as after a long history); side L then adds
 * with actors [0, n_actors/2), side R with [n_actors/2, n_actors).
 * Divergent ops per side: pct_add % adds, the rest removes with a read
 * context (Orswot::contains(m).rm_clock); in `pct_deferred_obj` % of objects,
 * `pct_future_rm` % of ops are removes with a FUTURE context (the side's clock
 * advanced on a remote actor), which defer (src/orswot.rs:197-203). In
 * `pct_shared_actor` % of objects side R also adds with actor 0 (the
 * weird_highlight_1 path, test/orswot.rs:84-92). */
typedef struct crdt_orswot_gen_params {
  uint32_t n_actors;         /* dense top-clock width (config 3: 16)            */
  uint32_t member_universe;  /* distinct member keys per object (config 3: 64)  */
  uint32_t ancestor_adds;    /* shared-history adds (config 3: 32)              */
  uint32_t min_div_ops;      /* divergent ops per side, uniform in [min, max]   */
  uint32_t max_div_ops;      /* (config 3: 4..16)                               */
  uint32_t pct_add;          /* (60)                                            */
  uint32_t pct_future_rm;    /* (10)                                            */
  uint32_t pct_deferred_obj; /* (8)                                             */
  uint32_t pct_shared_actor; /* (5)                                             */
} crdt_orswot_gen_params;

typedef struct crdt_orswot_gen crdt_orswot_gen;
/* Generates objects [first_obj, first_obj + n_obj) on n_threads host threads. */
int crdt_orswot_generate(uint64_t seed, size_t first_obj, size_t n_obj,
                         const crdt_orswot_gen_params* params, int n_threads,
                         crdt_orswot_gen** out);
/* side 0 = self (L), 1 = other (R) (or replica r): host base, u64 offsets (n_obj), bytes. */
int crdt_orswot_gen_side(const crdt_orswot_gen* g, int side, const uint8_t** h_base,
                         const uint64_t** h_off, size_t* bytes);
void crdt_orswot_gen_free(crdt_orswot_gen* g);

/* Replica sets for anti-entropy (config 5): per object, a shared ancestor of
 * `ancestor_adds` adds by actors of a per-object pool of `pool_actors` ids
 * drawn from [0, universe); each of the n_replicas replicas then applies
 * min..max divergent ops with its own `own_actors` ids (adds pct_add %,
 * read-context removes, and in pct_deferred_obj % of objects pct_future_rm %
 * removes whose context is advanced on another replica's actor, which
 * defer). Side r of the result (crdt_orswot_gen_side) is replica r. flags:
 * CRDT_ORSWOT_SPARSE_CLOCK encodes CSR top clocks (else dense, universe wide). */
typedef struct crdt_orswot_rep_params {
  uint32_t universe;         /* actor id universe (config 5: 1024)            */
  uint32_t pool_actors;      /* ancestor actors per object (48)               */
  uint32_t own_actors;       /* actors per replica per object (2)             */
  uint32_t member_universe;  /* (64)                                          */
  uint32_t ancestor_adds;    /* (48)                                          */
  uint32_t min_div_ops;      /* (4)                                           */
  uint32_t max_div_ops;      /* (16)                                          */
  uint32_t pct_add;          /* (60)                                          */
  uint32_t pct_future_rm;    /* (10)                                          */
  uint32_t pct_deferred_obj; /* (8)                                           */
} crdt_orswot_rep_params;
int crdt_orswot_generate_replicas(uint64_t seed, size_t first_obj, size_t n_obj,
                                  const crdt_orswot_rep_params* params, uint32_t n_replicas,
                                  uint32_t flags, int n_threads, crdt_orswot_gen** out);
/* The same replica sets, keeping only replicas [keep_first, keep_first +
 * keep_count) (side s of the result = replica keep_first + s): a rank
 * generates the replica it holds without encoding the others. */
int crdt_orswot_generate_replicas_subset(uint64_t seed, size_t first_obj, size_t n_obj,
                                         const crdt_orswot_rep_params* params, uint32_t n_replicas,
                                         uint32_t keep_first, uint32_t keep_count, uint32_t flags, int n_threads,
                                         crdt_orswot_gen** out);

/* ------------------------------------------------------------------------ *
 * Map<K, MVReg<u64, A>, A>::merge, batched (Map
 * src/map.rs:82-98, merge :191-268, apply_rm :336-349, apply_deferred
 * :323-333; MVReg truncate src/mvreg.rs:71-83 as the nested Causal value).
 * Keys are u64. Dense, fixed-capacity slabs, object i owning:
 *   clock[A]                            the map clock (0 = absent)
 *   n_keys, keys[kcap] ascending         entries (BTreeMap order)
 *   eclock[kcap][A]                      entry clocks
 *   mv_n[kcap], mv_clock[kcap][mcap][A], mv_val[kcap][mcap]   nested MVRegs (Vec order)
 *   n_def, dclock[dcap][A]               deferred removes in CLOCK ORDER
 *   dset_n[dcap], dset[dcap][scap]       their key sets, ascending
 * Only the used slots of the output are written (slots past a count keep
 * what the buffer held). Output capacities must be >= the sum of
 * both inputs' (kcap, mcap, dcap, scap); per side kcap <= 4096, mcap <= 128,
 * dcap <= 64, scap <= 4096, n_actors <= 128 (else CRDT_EINVAL); a merged map
 * past the output's capacities latches CRDT_ECAPACITY for that object.       */
typedef struct crdt_map_mvreg_slab {
  uint64_t* clock;
  uint32_t* n_keys;
  uint64_t* keys;
  uint64_t* eclock;
  uint32_t* mv_n;
  uint64_t* mv_clock;
  uint64_t* mv_val;
  uint32_t* n_def;
  uint64_t* dclock;
  uint32_t* dset_n;
  uint64_t* dset;
  uint32_t kcap, mcap, dcap, scap;
} crdt_map_mvreg_slab;
int crdt_map_mvreg_merge(crdt_ctx* ctx, const crdt_map_mvreg_slab* self, const crdt_map_mvreg_slab* other,
                         const crdt_map_mvreg_slab* out, size_t n_obj, uint32_t n_actors, void* stream);

/* ------------------------------------------------------------------------ *
 * Map<K, Map<K, MVReg<u64, A>, A>, A>::merge, batched: the reference's own
 * Map test type (TestMap, test/map.rs:4-8; Map::merge src/map.rs:191-268 with
 * the inner map's merge and Causal::truncate :131-158 as the value's). Keys
 * are u64. Object i's outer map:
 *   clock[A], n_keys, keys[kcap] ascending, eclock[kcap][A]
 *   n_def, dclock[dcap][A] (CLOCK ORDER), dset_n[dcap], dset[dcap][scap]
 * and, for key slot k, its nested map as object i * kcap + k of `inner` (a
 * crdt_map_mvreg_slab of n_obj * kcap maps; its own limits as above).
 * Outer limits per side: kcap <= 4096, dcap <= 64, scap <= 4096; n_actors <=
 * 128; output capacities (outer and inner) >= the sums of the inputs' (else
 * CRDT_EINVAL); a result past them latches CRDT_ECAPACITY. d_scratch needs
 * crdt_map_map_merge_scratch_bytes(out, n_obj, n_actors) bytes (the per-slot
 * merge tasks and their truncating clocks). Only used slots
 * of the output are written. Where two deferred clocks of an inner map
 * become equal under truncation the later one's key set is kept (the
 * reference inserts into a HashMap there). */
typedef struct crdt_map_map_slab {
  uint64_t* clock;
  uint32_t* n_keys;
  uint64_t* keys;
  uint64_t* eclock;
  uint32_t* n_def;
  uint64_t* dclock;
  uint32_t* dset_n;
  uint64_t* dset;
  uint32_t kcap, dcap, scap;
  crdt_map_mvreg_slab inner;
} crdt_map_map_slab;
size_t crdt_map_map_merge_scratch_bytes(const crdt_map_map_slab* out, size_t n_obj, uint32_t n_actors);
int crdt_map_map_merge(crdt_ctx* ctx, const crdt_map_map_slab* self, const crdt_map_map_slab* other,
                       const crdt_map_map_slab* out, size_t n_obj, uint32_t n_actors, void* d_scratch,
                       size_t scratch_bytes, void* stream);

/* ------------------------------------------------------------------------ *
 * Map<K, Orswot<u64, A>, A>::merge, batched (SURVEY.md §8(f) rank 3 as
 * written: src/map.rs:192-269 with the nested value's Causal::truncate,
 * src/orswot.rs:159-172, and Orswot::merge src/orswot.rs:87-157 for keys in
 * both maps). Keys and members are u64. Dense, fixed-capacity slabs, object
 * i owning:
 *   clock[A]                                   the map clock (0 = absent)
 *   n_keys, keys[kcap] ascending               entries (BTreeMap order)
 *   eclock[kcap][A]                            entry clocks
 *   nested Orswot per key:
 *     vclock[kcap][A]                          its top clock
 *     vn_mem[kcap], vmem[kcap][mcap]           members, ascending
 *     vmclock[kcap][mcap][A]                   member clocks (an all-zero row is
 *                                              an empty member clock, which
 *                                              truncate may leave in the
 *                                              reference; reachable states never
 *                                              hold one)
 *     vn_def[kcap], vdclock[kcap][vdcap][A]    deferred removes, CLOCK ORDER
 *     vdset_n[kcap][vdcap], vdset[kcap][vdcap][vscap]   their member sets, ascending
 *   n_def, dclock[dcap][A]                     the map's deferred removes, CLOCK ORDER
 *   dset_n[dcap], dset[dcap][scap]             their key sets, ascending
 * Only the used slots of the output are written: slots past a count keep
 * whatever the buffer held (a reader goes by the counts; zeroing them cost
 * ~10x the state's own bytes in writes). Per side kcap <= 4096, mcap <= 256,
 * vdcap, vscap, dcap <= 256, scap <= 4096, n_actors <= 128, and the
 * kernel's per-wave workspace — two nested sets of (mcap_s + mcap_o) member
 * rows and (vdcap_s + vdcap_o) deferred clocks of n_actors slots with their
 * member sets, plus 12 B per map deferred slot (dcap_s + dcap_o) — within
 * 64 KB
 * (else CRDT_EINVAL); output capacities must hold the result (else
 * CRDT_ECAPACITY is latched for that object). The map's deferred
 * removes are applied in CLOCK ORDER: the reference iterates a HashMap there
 * (src/map.rs:325-333) and, with Orswot values, two deferred clocks naming
 * the same key truncate its set in sequence, which can depend on that order
 * (DESIGN.md §5e); CLOCK ORDER is one of the reference's possible orders. */
typedef struct crdt_map_orswot_slab {
  uint64_t* clock;
  uint32_t* n_keys;
  uint64_t* keys;
  uint64_t* eclock;
  uint64_t* vclock;
  uint32_t* vn_mem;
  uint64_t* vmem;
  uint64_t* vmclock;
  uint32_t* vn_def;
  uint64_t* vdclock;
  uint32_t* vdset_n;
  uint64_t* vdset;
  uint32_t* n_def;
  uint64_t* dclock;
  uint32_t* dset_n;
  uint64_t* dset;
  uint32_t kcap, mcap, vdcap, vscap, dcap, scap;
} crdt_map_orswot_slab;
int crdt_map_orswot_merge(crdt_ctx* ctx, const crdt_map_orswot_slab* self, const crdt_map_orswot_slab* other,
                          const crdt_map_orswot_slab* out, size_t n_obj, uint32_t n_actors, void* stream);

/* ------------------------------------------------------------------------ *
 * VClock partial order and MVReg merge, batched.
 * crdt_vclock_partial_cmp: d_out[i] = partial_cmp(a[i], b[i])
 * (src/vclock.rs:59-71) over dense rows u64[n][n_actors], 0 = absent:
 * 0 Equal, 1 Greater (b <= a), -1 Less (a <= b), 2 None (concurrent).
 * crdt_mvreg_merge: MVReg<u64, A>::merge (src/mvreg.rs:121-153) over slabs
 * of `cap` (clock row, value) slots per object, d_*_n[i] slots in use; the
 * output keeps the reference's order (self's survivors, then other's) and
 * zero-fills unused slots. cap <= 1024 per side (registers of <= 64 slots
 * per side whose rows fit 60 KB of LDS per wave take the fast kernel, the
 * rest a one-wave-per-pair kernel reading the rows from HBM); more survivors
 * than out_cap latch CRDT_ECAPACITY.                                        */
int crdt_vclock_partial_cmp(crdt_ctx* ctx, const uint64_t* d_a, const uint64_t* d_b, size_t n,
                            uint32_t n_actors, int8_t* d_out, void* stream);
int crdt_mvreg_merge(crdt_ctx* ctx, const uint32_t* d_self_n, const uint64_t* d_self_clk,
                     const uint64_t* d_self_val, uint32_t self_cap, const uint32_t* d_other_n,
                     const uint64_t* d_other_clk, const uint64_t* d_other_val, uint32_t other_cap,
                     uint32_t* d_out_n, uint64_t* d_out_clk, uint64_t* d_out_val, uint32_t out_cap,
                     size_t n_obj, uint32_t n_actors, void* stream);

/* ------------------------------------------------------------------------ *
 * Batched op path: CmRDT::apply for Orswot (src/orswot.rs:61-85; Op enum
 * :38-53): out[i] = self[i] after applying object i's ops in order.
 *   Op::Add { dot: (actor, counter), member }   kind CRDT_OP_ADD
 *   Op::Rm  { clock, member }                   kind CRDT_OP_RM; clock i is
 *     pairs [clk_end[i-1], clk_end[i]) of clk_act / clk_ctr (canonical:
 *     actors strictly increasing, counters > 0; Add ops own no pairs)
 * Object i's ops are [obj_end[i-1], obj_end[i]). Record i of the output is
 * written at d_out_off[i] = self.off[i] + P*(ops before i) + 16*(clock pairs
 * before i) + 32*i (set by the call), P = 32 for dense top clocks and 48 for
 * CSR ones (an Add may bring a new actor, member and dot: 36 B), so
 * out_bytes >= self.bytes + P*n_ops + 16*n_clk + 32*n_obj suffices.
 * PRECONDITION: self's records do not overlap and are in increasing offset
 * order (as any packed or merged batch); a record that would outgrow its own
 * span self.size + P*ops + 16*pairs + 32 latches CRDT_ECAPACITY and is not
 * written. Limits per object, at every step of its op list (past one:
 * CRDT_ECAPACITY, the object is not written): <= 2048 top-clock entries (dense:
 * n_actors <= 2048), <= 4096 members, <= 16384 dots, <= 2048 pairs in an Rm
 * clock, <= 256 deferred clocks with <= 4096 entries and <= 4096 members in
 * all. (Objects are joined in an 8 KB LDS workspace, those that outgrow it in
 * a 16 KB one, the rest in an HBM workspace: the limits are the last one's.) */
#define CRDT_OP_ADD 0u
#define CRDT_OP_RM 1u
typedef struct crdt_orswot_ops {
  const uint64_t* obj_end;   /* device, n_obj  */
  const uint32_t* kind;      /* device, n_ops  */
  const uint64_t* member;    /* device, n_ops  */
  const uint32_t* actor;     /* device, n_ops (Add) */
  const uint64_t* counter;   /* device, n_ops (Add) */
  const uint64_t* clk_end;   /* device, n_ops  */
  const uint32_t* clk_act;   /* device, n_clk  */
  const uint64_t* clk_ctr;   /* device, n_clk  */
  size_t n_ops;
  size_t n_clk;
} crdt_orswot_ops;
int crdt_orswot_apply(crdt_ctx* ctx, const crdt_orswot_batch* self, const crdt_orswot_ops* ops,
                      uint32_t n_actors, uint32_t flags, uint8_t* d_out, uint64_t* d_out_off,
                      size_t out_bytes, void* stream);

/* ------------------------------------------------------------------------ *
 * Ingest / egest: the reference's binary form <-> canonical records
 * (SURVEY.md §8(f) rank 1). The reference form of an Orswot<M, A> is
 * `to_binary(&s)` = bincode 0.9 of its serde derives (src/lib.rs:62-83;
 * fields src/orswot.rs:26-30, src/vclock.rs:54-57): u64 little-endian
 * lengths before every map / set, fixed-width little-endian integers, HashMap
 * and HashSet elements in any order, BTreeMap keys ascending. Actors (A) and
 * members (M) are unsigned integers of actor_bytes / member_bytes in
 * {1, 2, 4, 8}; they are the record's actor ids / member keys as they stand.
 * Blob i is bytes [blob_off[i], blob_off[i] + blob_len[i]) of d_blobs
 * (blob_bytes long, any alignment).
 *
 * Ingest = from_binary + canonicalisation; a blob a record cannot hold
 * (zero counter, empty member clock / deferred clock / deferred set, actor
 * >= n_actors, duplicates, BTreeMap keys out of order, truncated or trailing
 * bytes) latches CRDT_ENONCANON; one with more than 16384 members or more
 * than 1024 deferred clocks latches CRDT_ECAPACITY, and so do the objects of
 * one call past its first 65536 with more than 256 members or 64 deferred
 * clocks (those are decoded by a second kernel from an HBM scratch).
 *   1) crdt_orswot_bincode_record_sizes: d_sizes[i] = record bytes (0 if bad)
 *      — or, without reading the blobs, crdt_orswot_bincode_record_bounds:
 *      d_bounds[i] >= the record bytes of any blob of length blob_len[i]
 *      (16-B multiple; <= 48 + 8 n_actors + blob_len * max(12/(wa+8),
 *      12/(wm+8), 8/wm)); records placed by bounds form a gapped batch, a
 *      valid input everywhere (crdt_orswot_compact removes the gaps)
 *   2) the caller places records (16-B aligned offsets, e.g. exclusive scan)
 *   3) crdt_orswot_from_bincode writes record i at d_out + d_out_off[i].
 * Egest = to_binary with HashMap / HashSet elements in ascending key (clock)
 * order — one of the orders the reference may produce, decoded to an equal
 * state by from_binary:
 *   1) crdt_orswot_bincode_sizes: d_sizes[i] = blob bytes
 *   2) the caller places blobs at 16-B aligned offsets (each zero-padded to 16)
 *   3) crdt_orswot_to_bincode writes them.                                    */
int crdt_orswot_bincode_record_sizes(crdt_ctx* ctx, const uint8_t* d_blobs, size_t blob_bytes,
                                     const uint64_t* d_blob_off, const uint64_t* d_blob_len, size_t n_obj,
                                     uint32_t actor_bytes, uint32_t member_bytes, uint32_t n_actors,
                                     uint32_t flags, uint64_t* d_sizes, void* stream);
int crdt_orswot_bincode_record_bounds(crdt_ctx* ctx, const uint64_t* d_blob_len, size_t n_obj,
                                      uint32_t actor_bytes, uint32_t member_bytes, uint32_t n_actors, uint32_t flags,
                                      uint64_t* d_bounds, void* stream);
int crdt_orswot_from_bincode(crdt_ctx* ctx, const uint8_t* d_blobs, size_t blob_bytes,
                             const uint64_t* d_blob_off, const uint64_t* d_blob_len, size_t n_obj,
                             uint32_t actor_bytes, uint32_t member_bytes, uint32_t n_actors, uint32_t flags,
                             uint8_t* d_out, const uint64_t* d_out_off, size_t out_bytes, void* stream);
int crdt_orswot_bincode_sizes(crdt_ctx* ctx, const crdt_orswot_batch* batch, uint32_t n_actors,
                              uint32_t flags, uint32_t actor_bytes, uint32_t member_bytes, uint64_t* d_sizes,
                              void* stream);
int crdt_orswot_to_bincode(crdt_ctx* ctx, const crdt_orswot_batch* batch, uint32_t n_actors, uint32_t flags,
                           uint32_t actor_bytes, uint32_t member_bytes, uint8_t* d_out,
                           const uint64_t* d_out_off, size_t out_bytes, void* stream);

/* Dense synthetic counters: u64[n_obj][n_actors] rows for objects
 * [first_obj, first_obj+n_obj), counter U[0, 2^bits) with `pct_zero` % zeros. */
int crdt_dense_generate(uint64_t seed, size_t first_obj, size_t n_obj, uint32_t n_actors,
                        uint32_t bits, uint32_t pct_zero, int n_threads, uint64_t* h_rows);

/* Causal::truncate, batched (src/orswot.rs:159-172; the Map of Orswots calls it
 * on every value it keeps, src/map.rs): out[i] := self[i] after
 * self[i].truncate(&clock[i]) — merge with an empty Orswot whose clock is
 * clock[i] (incl. apply_deferred), then clock[i] subtracted from the top clock
 * and from every member clock. clocks: a crdt_clock_csr batch of the same
 * n_obj (any clock form of the records: actor ids as in the records).
 * flags: 0 or CRDT_ORSWOT_SPARSE_CLOCK (the batch's record form). A truncated
 * record is never larger than its input: record i is written at
 * d_out_off[i] := self.off[i] (set by the call), so out_bytes >= self.bytes
 * suffices. A member whose clock the subtract empties is kept with an empty
 * clock, as in the reference, and its record carries
 * CRDT_ORSWOT_EMPTY_MEMBER_CLOCK; such a record is a valid input of this call
 * (truncating it again drops those members: empty <= c, src/orswot.rs:98-103).
 * A malformed record or clock run (actors not strictly increasing, a zero
 * counter) latches CRDT_ENONCANON (that record is not written). d_out must
 * not overlap the input records (CRDT_EINVAL): the call is not in place. */
int crdt_orswot_truncate(crdt_ctx* ctx, const crdt_orswot_batch* self, const crdt_clock_csr* clocks,
                         uint32_t n_actors, uint32_t flags, uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes,
                         void* stream);

/* Host op-path builder used to construct states (tests, KAT scripts): an
 * opaque host Orswot with the reference's op semantics (src/orswot.rs:61-85,
 * 195-211, 235-243), encoded to / decoded from canonical records. */
typedef struct crdt_host_orswot crdt_host_orswot;
crdt_host_orswot* crdt_host_orswot_new(void);
crdt_host_orswot* crdt_host_orswot_clone(const crdt_host_orswot* o);
void crdt_host_orswot_free(crdt_host_orswot* o);
/* Op::Add { dot: (actor, counter), member }  (src/orswot.rs:66-79) */
int crdt_host_orswot_apply_add(crdt_host_orswot* o, uint32_t actor, uint64_t counter,
                               uint64_t member);
/* Op::Rm { clock, member }  (src/orswot.rs:80-82) — clock as sorted runs */
int crdt_host_orswot_apply_rm(crdt_host_orswot* o, uint64_t member, const uint32_t* actors,
                              const uint64_t* counters, uint32_t n);
/* Encode into h_rec (capacity cap); returns bytes written or a negative code. */
long crdt_host_orswot_encode(const crdt_host_orswot* o, uint32_t n_actors, uint8_t* h_rec,
                             size_t cap);
/* flags: 0 (dense, n_actors slots) or CRDT_ORSWOT_SPARSE_CLOCK (CSR top clock). */
long crdt_host_orswot_encode_ex(const crdt_host_orswot* o, uint32_t n_actors, uint32_t flags,
                                uint8_t* h_rec, size_t cap);
crdt_host_orswot* crdt_host_orswot_decode(const uint8_t* h_rec, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* CRDTS_HIP_H */
