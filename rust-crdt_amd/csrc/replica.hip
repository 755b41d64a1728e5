// Replica anti-entropy across GPUs (SURVEY.md §8(b),(e); BASELINE.json
// configs[3] and configs[4]) behind the C ABI, on RCCL over xGMI.
//
// Dense clocks / counters: one in-place ncclAllReduce(ncclUint64, ncclMax).
// The join is VClock::merge (src/vclock.rs:131-137), a pointwise max: any
// reduction order gives the same bits, and RCCL reduces u64 natively.
//
// Orswot: the join is structurally NON-commutative (self-only entries kept
// as they are, src/orswot.rs:98-103; other-only entries subtracted by the
// self clock, :132-138), so the result is defined as the rank-order fold
// ((r0 ⊔ r1) ⊔ r2) ⊔ ... and every rank must end with the same bytes. It is
// computed owner-sharded: the n objects are split into N contiguous ranges,
// rank j owns range j and
//   1. learns every rank's byte extent of every range (all-gather of 2N u64);
//   2. receives every replica's slice of range j — records and offsets —
//      point-to-point from each peer (one grouped send/recv round: the 8-GPU
//      node is fully connected, so each pair of GPUs uses its own xGMI link);
//   3. folds the N slices in rank order with the batched merge kernel, then
//      compacts the result (gaps removed);
//   4. sends its folded range to every peer and receives theirs (grouped
//      send/recv again), and rebases the gathered offsets.
// Per rank that is 1/N of the fold work and ~2(N-1)/N replica sizes on the
// wire, instead of N-1 replicas in and N-1 merges of everything.
//
// The per-rank code is written once against a Transport; RcclTransport is
// the product, ThreadTransport runs the same code with one host thread per
// virtual rank on ONE device (crdt_orswot_replica_join_local), which is how
// the exchange logic is tested without a multi-GPU node.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/crdts_hip.h"
#include "ctx.h"
#include "kernels.h"

using namespace crdts_hip;

namespace {

inline hipStream_t S(void* s) { return (hipStream_t)s; }
inline uint64_t al16(uint64_t x) { return (x + 15u) & ~uint64_t(15); }
inline uint64_t al256(uint64_t x) { return (x + 255u) & ~uint64_t(255); }

constexpr size_t kAllReduceChunk = size_t(1) << 27;  // u64 words per collective (1 GiB)

// ---------------------------------------------------------------- kernels
// Step 1's all-gather row of this rank, written on the device so that the
// slice bounds need no host round trip of their own: d[2j], d[2j+1] = byte
// extent of object range j = [b_j, b_{j+1}), b_j = j*n/N, of this replica
// (0, 0 for an empty range; ~0 as the end of a range whose last record
// header lies out of bounds), then the host-known fields of the row.
// Row word 2R + 1 is the error word: a status an earlier launch on this
// context latched and the caller has not read is reported through it (every
// rank then fails the join with it) and cleared.
__global__ void slice_bounds_kernel(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                    uint64_t bytes, uint64_t n, uint32_t R, uint64_t* __restrict__ d, uint64_t f0,
                                    int* __restrict__ status, uint64_t f2, uint64_t f3) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) {
    const int st = *status;
    *status = 0;
    d[2u * R] = f0;
    d[2u * R + 1u] = (uint64_t)(int64_t)-st;
    d[2u * R + 2u] = f2;
    d[2u * R + 3u] = f3;
  }
  if (j >= R) return;
  const uint64_t b0 = n * j / R, b1 = n * (j + 1u) / R;
  uint64_t s = 0, e = 0;
  if (b1 > b0) {
    s = off[b0];
    const uint64_t last = off[b1 - 1u];
    e = last + 32u <= bytes ? last + *(const uint32_t*)(base + last) : ~0ull;  // ~0: out of bounds
  }
  d[2u * j] = s;
  d[2u * j + 1u] = e;
}

// off[i] := off[i] - sub[piece(i)] + add[piece(i)] for pieces of `per` objects
// (piece p = objects [p*per, (p+1)*per)); or, with first != null, pieces
// [first[p], first[p+1]).
__global__ void rebase_kernel(uint64_t* __restrict__ off, uint64_t n, uint64_t per,
                              const uint64_t* __restrict__ first, const uint64_t* __restrict__ sub,
                              const uint64_t* __restrict__ add, uint32_t R) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t p;
  if (first) {
    p = 0;
    while (p + 1u < R && first[p + 1u] <= i) ++p;
  } else {
    p = (uint32_t)(i / per);
  }
  off[i] = off[i] - sub[p] + add[p];
}

// The step-4 row of the owner-sharded join, on the device: {E = bytes of the
// compacted folded range, out_bytes, error word (the fold's latched status, or
// CRDT_ENONCANON when E outgrows the inputs)} — all-gathered straight from
// here, so the compaction's sizes and the status need no read of their own.
__global__ void join_row_kernel(const uint64_t* __restrict__ shard_off, const uint64_t* __restrict__ sizes,
                                uint64_t nr, uint64_t total, uint64_t out_bytes, int* __restrict__ status,
                                uint64_t* __restrict__ row) {
  if (threadIdx.x != 0) return;
  const uint64_t E = nr ? shard_off[nr - 1u] + sizes[nr - 1u] : 0ull;
  const int st = *status;
  row[0] = E;
  row[1] = out_bytes;
  row[2] = st ? (uint64_t)(int64_t)-st : (E > total ? (uint64_t)(int64_t)-CRDT_ENONCANON : 0ull);
}

int launch_rebase(uint64_t* off, uint64_t n, uint64_t per, const uint64_t* first, const uint64_t* sub,
                  const uint64_t* add, uint32_t R, hipStream_t st) {
  if (n == 0) return CRDT_OK;
  hipLaunchKernelGGL(rebase_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, off, n, per, first, sub,
                     add, R);
  return hipGetLastError() == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

// ---------------------------------------------------------------- transports
using Xfer = crdt_xfer;

struct Transport {
  int R = 1, me = 0;
  uint64_t syncs = 0;  // host synchronisations with the device made here
  virtual ~Transport() = default;
  int sync(hipStream_t st) {
    ++syncs;
    return hipStreamSynchronize(st) == hipSuccess ? CRDT_OK : CRDT_EHIP;
  }
  // blocking: every rank contributes n u64 (host), receives R*n in rank order
  virtual int allgather(const uint64_t* h_in, size_t n, uint64_t* h_out, hipStream_t st) = 0;
  // the same with the contribution in DEVICE memory, produced on st (one
  // host synchronisation in all)
  virtual int allgather_dev(const uint64_t* d_in, size_t n, uint64_t* h_out, hipStream_t st) {
    std::vector<uint64_t> h(n);
    if (n && (hipMemcpyAsync(h.data(), d_in, 8 * n, hipMemcpyDeviceToHost, st) != hipSuccess || sync(st)))
      return CRDT_EHIP;
    return allgather(h.data(), n, h_out, st);
  }
  // enqueued on st: every send matched by the peer's recv of the same size
  virtual int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) = 0;
};

int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? CRDT_OK : CRDT_ECOMM; }

// Device staging of the small all-gathers (ctx-owned, crdt_comm_init):
// kStageRow u64 per rank and contribution.
inline size_t stage_row(int R) { return 2ull * R + 8; }
inline size_t stage_words(int R) { return (size_t)(R + 1) * stage_row(R); }

struct RcclTransport : Transport {
  ncclComm_t comm;
  uint64_t* d_buf;
  RcclTransport(crdt_ctx* ctx, uint64_t* d) : comm((ncclComm_t)ctx->comm), d_buf(d) {
    R = ctx->n_ranks;
    me = ctx->rank;
  }
  int gather_out(const uint64_t* d_in, size_t n, uint64_t* h_out, hipStream_t st) {
    if (n > stage_row(R)) return CRDT_EINVAL;
    int rc = nccl_rc(ncclAllGather(d_in, d_buf + stage_row(R), n, ncclUint64, comm, st));
    if (rc) return rc;
    if (hipMemcpyAsync(h_out, d_buf + stage_row(R), 8 * n * R, hipMemcpyDeviceToHost, st) != hipSuccess || sync(st))
      return CRDT_EHIP;
    return CRDT_OK;
  }
  int allgather(const uint64_t* h_in, size_t n, uint64_t* h_out, hipStream_t st) override {
    if (n > stage_row(R)) return CRDT_EINVAL;
    if (hipMemcpyAsync(d_buf, h_in, 8 * n, hipMemcpyHostToDevice, st) != hipSuccess) return CRDT_EHIP;
    return gather_out(d_buf, n, h_out, st);
  }
  int allgather_dev(const uint64_t* d_in, size_t n, uint64_t* h_out, hipStream_t st) override {
    return gather_out(d_in, n, h_out, st);
  }
  int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) override {
    // the self part as device copies (k-th self send -> k-th self recv), the
    // rest as one group of point-to-point transfers (xGMI is point-to-point:
    // each peer pair has its own link)
    size_t k = 0;
    for (const Xfer& y : recvs) {
      if (y.peer != me) continue;
      while (k < sends.size() && sends[k].peer != me) ++k;
      if (k == sends.size() || sends[k].bytes != y.bytes) return CRDT_ECOMM;
      if (y.bytes && hipMemcpyAsync(y.dst, sends[k].src, y.bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return CRDT_EHIP;
      ++k;
    }
    int rc = nccl_rc(ncclGroupStart());
    if (rc) return rc;
    for (size_t q = 0; q < sends.size() && !rc; ++q)
      if (sends[q].peer != me && sends[q].bytes)
        rc = nccl_rc(ncclSend(sends[q].src, sends[q].bytes, ncclUint8, sends[q].peer, comm, st));
    for (size_t q = 0; q < recvs.size() && !rc; ++q)
      if (recvs[q].peer != me && recvs[q].bytes)
        rc = nccl_rc(ncclRecv(recvs[q].dst, recvs[q].bytes, ncclUint8, recvs[q].peer, comm, st));
    const int rc2 = nccl_rc(ncclGroupEnd());
    return rc ? rc : rc2;
  }
};

// The caller's own transport (crdt_transport callbacks: e.g. gloo, MPI, a
// host network), one process per rank; the data path is its business.
struct CallbackTransport : Transport {
  const crdt_transport* t;
  explicit CallbackTransport(const crdt_transport* tt) : t(tt) {
    R = tt->n_ranks;
    me = tt->rank;
  }
  int allgather(const uint64_t* h_in, size_t n, uint64_t* h_out, hipStream_t) override {
    return t->allgather(t->user, h_in, n, h_out) ? CRDT_ECOMM : CRDT_OK;
  }
  int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) override {
    return t->exchange(t->user, sends.data(), sends.size(), recvs.data(), recvs.size(), (void*)st) ? CRDT_ECOMM
                                                                                                  : CRDT_OK;
  }
};

// R virtual ranks in one process, one host thread each, all on one device.
struct ThreadGroup {
  int R;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<uint64_t> gather;                 // allgather staging
  std::vector<std::vector<Xfer>> sends;         // per rank: its published sends
  std::vector<hipEvent_t> ready, done;          // per rank: data ready / copies done
  explicit ThreadGroup(int r) : R(r), sends(r), ready(r, nullptr), done(r, nullptr) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived == R) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

struct ThreadTransport : Transport {
  ThreadGroup* g;
  ThreadTransport(ThreadGroup* grp, int rank) : g(grp) {
    R = grp->R;
    me = rank;
  }
  int allgather(const uint64_t* h_in, size_t n, uint64_t* h_out, hipStream_t) override {
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if (g->gather.size() < n * R) g->gather.resize(n * R);
    }
    g->barrier();
    std::memcpy(g->gather.data() + n * me, h_in, 8 * n);
    g->barrier();
    std::memcpy(h_out, g->gather.data(), 8 * n * R);
    g->barrier();
    return CRDT_OK;
  }
  int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) override {
    g->sends[me] = sends;
    int rc = hipEventRecord(g->ready[me], st) == hipSuccess ? CRDT_OK : CRDT_EHIP;
    g->barrier();
    for (const Xfer& y : recvs) {  // pull each peer's matching send (same order of sends to one peer)
      if (!y.bytes || rc) continue;
      size_t k = 0;
      for (const Xfer& x : recvs) {
        if (&x == &y) break;
        if (x.peer == y.peer && x.bytes) ++k;
      }
      const Xfer* src = nullptr;
      for (const Xfer& x : g->sends[y.peer])
        if (x.peer == me && x.bytes && k-- == 0) { src = &x; break; }
      if (!src || src->bytes != y.bytes) { rc = CRDT_ECOMM; continue; }
      if (hipStreamWaitEvent(st, g->ready[y.peer], 0) != hipSuccess ||
          hipMemcpyAsync(y.dst, src->src, y.bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
        rc = CRDT_EHIP;
    }
    if (hipEventRecord(g->done[me], st) != hipSuccess) rc = CRDT_EHIP;
    g->barrier();
    for (int p = 0; p < R; ++p)  // our send buffers stay untouched until every reader copied them
      if (hipStreamWaitEvent(st, g->done[p], 0) != hipSuccess) rc = CRDT_EHIP;
    g->barrier();
    return rc;
  }
};

// ---------------------------------------------------------------- per-rank join
int ensure_arena(crdt_ctx* ctx, size_t bytes) {
  if (ctx->arena_bytes >= bytes) return CRDT_OK;
  if (ctx->arena_limit && bytes > ctx->arena_limit) return CRDT_ECAPACITY;
  (void)hipFree(ctx->d_arena);
  ctx->d_arena = nullptr;
  ctx->arena_bytes = 0;
  if (hipMalloc(&ctx->d_arena, bytes) != hipSuccess) return CRDT_EHIP;
  ctx->arena_bytes = bytes;
  return CRDT_OK;
}

// Arena layout of rank j's part of a join (every rank can compute every
// rank's, from the step-1 all-gather): head = step-1 row (2R + 4 u64), the
// rebase table (3R u64) and the step-4 row (3 u64); then every replica's slice of range j, their
// offsets, two fold buffers (ping-pong), sizes and scan scratch.
struct Plan {
  size_t head, o_recv, o_roff, o_fa, o_fb, o_oa, o_ob, o_sz, o_cub, cub_temp, end;
};
inline size_t plan_head(int R) { return al256(8ull * (2 * R + 4) + 8ull * 3 * R + 8ull * 3); }  // + the step-4 row
Plan make_plan(int R, uint64_t nr, uint64_t total) {
  Plan P;
  P.head = plan_head(R);
  P.cub_temp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, P.cub_temp, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                         (int)(nr ? nr : 1));
  size_t at = P.head;
  auto take = [&](size_t bytes) { size_t o = at; at = al256(at + bytes); return o; };
  P.o_recv = take(total);
  P.o_roff = take(8 * R * nr);
  P.o_fa = take(total);
  P.o_fb = take(total);
  P.o_oa = take(8 * nr);
  P.o_ob = take(8 * nr);
  P.o_sz = take(8 * nr);
  P.o_cub = take(P.cub_temp);
  P.end = at;
  return P;
}

// The owner-sharded join, one rank's part. `out` may be null (the rank takes
// part in the exchange but does not gather the result). Every verdict that
// decides whether a rank goes on to the next collective is taken from
// all-gathered data, so all ranks leave at the same step (none is left
// waiting in a collective another has left). Host synchronisations per call
// in the steady state (arena large enough on every rank): 3 — the step-1
// all-gather, the step-4 all-gather (its row — the compacted range's size and
// the fold's status — is produced on the device), and the final one (the call
// is synchronous). They are counted in ctx->host_syncs.
int orswot_join_rank_body(crdt_ctx* ctx, Transport& T, const crdt_orswot_batch* mine, uint32_t A, uint32_t flags,
                          uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, size_t* h_used, hipStream_t st) {
  const int R = T.R, me = T.me;
  const uint64_t n = mine->n_obj;
  const bool want = d_out != nullptr;
  auto b = [&](int j) { return n * (uint64_t)j / (uint64_t)R; };
  const size_t W = 2 * (size_t)R + 4;

  // 1. my byte extents of every range + (n, error, want, arena capacity),
  //    all-gathered straight from the device. A status an earlier launch on
  //    this context latched and the caller has not read goes out as this
  //    rank's error word (slice_bounds_kernel reads and clears it): every rank
  //    fails this join with that code (include/crdts_hip.h).
  int err = ensure_arena(ctx, plan_head(R));
  if (!err && n && (!mine->base || !mine->off)) err = CRDT_EINVAL;
  if (err) {
    std::vector<uint64_t> mb(W, 0), G(W * R);
    mb[2 * R] = n;
    mb[2 * R + 1] = (uint64_t)-err;
    int rc = T.allgather(mb.data(), W, G.data(), st);
    return rc ? rc : err;
  }
  uint64_t* d_row = (uint64_t*)ctx->d_arena;
  uint64_t* d_tab = d_row + W;
  hipLaunchKernelGGL(slice_bounds_kernel, dim3((R + 63) / 64), dim3(64), 0, st, n ? mine->base : nullptr,
                     n ? mine->off : nullptr, (uint64_t)mine->bytes, n, (uint32_t)R, d_row, n, ctx->d_status,
                     want ? 1ull : 0ull, (uint64_t)ctx->arena_bytes);
  if (hipGetLastError() != hipSuccess) return CRDT_EHIP;
  std::vector<uint64_t> G(W * R);
  int rc = T.allgather_dev(d_row, W, G.data(), st);
  if (rc) return rc;
  auto gs = [&](int p, int j) { return G[W * p + 2 * j]; };  // rank p's start of range j
  auto gsz = [&](int p, int j) { return G[W * p + 2 * j + 1] - G[W * p + 2 * j]; };
  auto wants = [&](int p) { return G[W * p + 2 * R + 2] != 0; };
  for (int p = 0; p < R; ++p) {  // the same verdict on every rank
    if (G[W * p + 2 * R] != n) return CRDT_EINVAL;  // the same object count on every rank
    if (G[W * p + 2 * R + 1]) return -(int)G[W * p + 2 * R + 1];
    uint64_t prev_end = 0;
    for (int j = 0; j < R; ++j) {  // ranges in increasing, non-overlapping order, 16-B aligned
      if (b(j + 1) == b(j)) continue;
      const uint64_t s0 = gs(p, j), e0 = G[W * p + 2 * j + 1];
      if (e0 == ~0ull || e0 < s0 || s0 < prev_end || ((s0 | e0) & 15u)) return CRDT_EINVAL;
      prev_end = e0;
    }
  }
  auto plan_of = [&](int j) {
    uint64_t total = 0;
    for (int p = 0; p < R; ++p) total += al16(gsz(p, j));
    return make_plan(R, b(j + 1) - b(j), total);
  };

  // 2. the arena (grown only where some rank must: then every rank agrees
  //    on the outcome before any data moves), and every replica's slice of
  //    my range, point-to-point
  bool grow = false;
  for (int p = 0; p < R; ++p) grow |= plan_of(p).end > G[W * p + 2 * R + 3];
  Plan P = plan_of(me);
  if (grow) {
    err = ensure_arena(ctx, P.end);
    uint64_t e1 = (uint64_t)-err;
    std::vector<uint64_t> E1(R);
    if ((rc = T.allgather(&e1, 1, E1.data(), st))) return rc;
    for (int p = 0; p < R; ++p)
      if (E1[p]) return -(int)E1[p];
    d_row = (uint64_t*)ctx->d_arena;  // the arena may have moved
    d_tab = d_row + W;
  }
  const uint64_t nr = b(me + 1) - b(me);
  std::vector<uint64_t> pos(R + 1, 0);
  for (int p = 0; p < R; ++p) pos[p + 1] = pos[p] + al16(gsz(p, me));
  const uint64_t total = pos[R];
  uint8_t* A8 = ctx->d_arena;
  uint8_t* recv = A8 + P.o_recv;
  uint64_t* roff = (uint64_t*)(A8 + P.o_roff);
  std::vector<Xfer> sends, recvs;
  for (int p = 0; p < R; ++p) {  // per peer: the records, then the offsets (same order on both ends)
    const uint64_t np = b(p + 1) - b(p);
    sends.push_back({p, n ? mine->base + gs(me, p) : nullptr, nullptr, gsz(me, p)});
    sends.push_back({p, n ? mine->off + b(p) : nullptr, nullptr, 8 * np});
    recvs.push_back({p, nullptr, recv + pos[p], gsz(p, me)});
    recvs.push_back({p, nullptr, roff + nr * p, 8 * nr});
  }
  if ((rc = T.exchange(sends, recvs, st))) return rc;

  // 3. offsets relative to each slice's own base, the rank-order fold, and
  //    compaction into the fold buffer the result is not in
  std::vector<uint64_t> tab(3 * R, 0);
  for (int p = 0; p < R; ++p) tab[R + p] = gs(p, me);  // sub
  if (hipMemcpyAsync(d_tab, tab.data(), 8ull * 3 * R, hipMemcpyHostToDevice, st) != hipSuccess) err = CRDT_EHIP;
  if (!err) err = launch_rebase(roff, nr * R, nr ? nr : 1, nullptr, d_tab + R, d_tab + 2 * R, (uint32_t)R, st);
  const uint8_t* acc = recv;
  const uint64_t* acc_off = roff;
  uint64_t acc_bytes = gsz(0, me);
  // one replica: nothing is merged, so the slice is checked in full here
  if (!err && R == 1 && nr) err = launch_orswot_validate(acc, acc_off, acc_bytes, nr, A, flags, ctx->d_status, st);
  for (int p = 1; p < R && nr && !err; ++p) {
    uint8_t* o = A8 + (p % 2 ? P.o_fa : P.o_fb);
    uint64_t* oo = (uint64_t*)(A8 + (p % 2 ? P.o_oa : P.o_ob));
    const uint8_t* rb = recv + pos[p];
    const uint64_t* ro = roff + nr * p;
    const uint64_t cap = acc_bytes + gsz(p, me);
    err = (flags & CRDT_ORSWOT_SPARSE_CLOCK)
              ? launch_orswot_merge_sparse(acc, acc_off, acc_bytes, rb, ro, gsz(p, me), o, oo, cap, nr, A,
                                           ctx->d_status, ctx->d_ctl, ctx->d_list, ctx->list_cap, st, 0, &ctx->join_seq)
              : launch_orswot_merge(acc, acc_off, acc_bytes, rb, ro, gsz(p, me), o, oo, cap, nr, A, ctx->d_status,
                                    ctx->d_ctl, ctx->d_list, ctx->list_cap, st, 0, 0, &ctx->join_seq);
    acc = o;
    acc_off = oo;
    acc_bytes = cap;
  }
  const bool in_a = acc == A8 + P.o_fa;
  uint8_t* shard = A8 + (in_a ? P.o_fb : P.o_fa);
  uint64_t* shard_off = (uint64_t*)(A8 + (in_a ? P.o_ob : P.o_oa));
  uint64_t* sizes = (uint64_t*)(A8 + P.o_sz);
  if (nr && !err) {
    // record sizes, bounds-checked (an object the fold rejected leaves no
    // record behind its offset: size 0 and CRDT_ENONCANON latched), the scan,
    // and the copy (each record only where it fits the shard buffer); the
    // compacted size and the fold's status go out with the step-4 row
    err = launch_record_sizes(acc, acc_off, acc_bytes, nr, sizes, ctx->d_status, st);
    if (!err && hipcub::DeviceScan::ExclusiveSum(A8 + P.o_cub, P.cub_temp, sizes, shard_off, (int)nr, st) !=
                    hipSuccess)
      err = CRDT_EHIP;
    if (!err) err = launch_record_copy(acc, acc_off, sizes, shard, shard_off, nr, total, st);
  }

  // 4. every rank's folded range to every rank that gathers the result: the
  //    row {E, out_bytes, error} all-gathered from the device (from the host
  //    when a launch failed here)
  std::vector<uint64_t> G2(3 * R);
  if (!err) {
    uint64_t* d_row2 = d_tab + 3 * R;
    hipLaunchKernelGGL(join_row_kernel, dim3(1), dim3(64), 0, st, shard_off, sizes, nr, (uint64_t)total,
                       (uint64_t)out_bytes, ctx->d_status, d_row2);
    if (hipGetLastError() != hipSuccess) err = CRDT_EHIP;
    if (!err && (rc = T.allgather_dev(d_row2, 3, G2.data(), st))) return rc;
  }
  if (err) {
    uint64_t m2[3] = {0, (uint64_t)out_bytes, (uint64_t)-err};
    if ((rc = T.allgather(m2, 3, G2.data(), st))) return rc;
  }
  const uint64_t E = G2[3 * me];
  std::vector<uint64_t> Pq(R + 1, 0);
  for (int q = 0; q < R; ++q) {
    if (G2[3 * q + 2]) return -(int)G2[3 * q + 2];
    Pq[q + 1] = Pq[q] + G2[3 * q];
  }
  for (int q = 0; q < R; ++q)
    if (wants(q) && G2[3 * q + 1] < Pq[R]) return CRDT_ECAPACITY;  // every rank sees the same verdict
  sends.clear();
  recvs.clear();
  for (int q = 0; q < R; ++q) {
    if (wants(q)) {
      sends.push_back({q, shard, nullptr, E});
      sends.push_back({q, shard_off, nullptr, 8 * nr});
    }
    if (want) {
      const uint64_t nq = b(q + 1) - b(q);
      recvs.push_back({q, nullptr, d_out + Pq[q], G2[3 * q]});
      recvs.push_back({q, nullptr, d_out_off + b(q), 8 * nq});
    }
  }
  rc = T.exchange(sends, recvs, st);
  if (!rc && want) {
    for (int q = 0; q < R; ++q) {
      tab[q] = b(q);
      tab[R + q] = 0;
      tab[2 * R + q] = Pq[q];
    }
    if (hipMemcpyAsync(d_tab, tab.data(), 8ull * 3 * R, hipMemcpyHostToDevice, st) != hipSuccess) rc = CRDT_EHIP;
    if (!rc) rc = launch_rebase(d_out_off, n, 1, d_tab, d_tab + R, d_tab + 2 * R, (uint32_t)R, st);
    if (!rc && h_used) *h_used = Pq[R];
  }
  // the tables are read by kernels on st: finished before a later call reuses them
  if (T.sync(st) && !rc) rc = CRDT_EHIP;
  return rc;
}

// A failed join leaves no latched status behind (the next call starts clean).
int orswot_join_rank(crdt_ctx* ctx, Transport& T, const crdt_orswot_batch* mine, uint32_t A, uint32_t flags,
                     uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, size_t* h_used, hipStream_t st) {
  const int rc = orswot_join_rank_body(ctx, T, mine, A, flags, d_out, d_out_off, out_bytes, h_used, st);
  ctx->host_syncs += T.syncs;
  if (rc) {
    (void)hipStreamSynchronize(st);
    (void)hipMemsetAsync(ctx->d_status, 0, sizeof(int), st);
    (void)hipStreamSynchronize(st);
  }
  return rc;
}

int set_dev(crdt_ctx* ctx) { return hipSetDevice(ctx->device) == hipSuccess ? CRDT_OK : CRDT_EHIP; }

}  // namespace

extern "C" {

int crdt_comm_unique_id(uint8_t* h_id) {
  if (!h_id) return CRDT_EINVAL;
  static_assert(sizeof(ncclUniqueId) == CRDT_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return CRDT_ECOMM;
  std::memcpy(h_id, &id, sizeof id);
  return CRDT_OK;
}

int crdt_comm_init(crdt_ctx* ctx, const uint8_t* h_id, int n_ranks, int rank) {
  if (!ctx || !h_id || n_ranks < 1 || rank < 0 || rank >= n_ranks || ctx->comm) return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc) return rc;
  ncclUniqueId id;
  std::memcpy(&id, h_id, sizeof id);
  uint64_t* stage = nullptr;
  if (hipMalloc(&stage, 8ull * stage_words(n_ranks)) != hipSuccess) return CRDT_EHIP;
  ncclComm_t comm = nullptr;
  if (ncclCommInitRank(&comm, n_ranks, id, rank) != ncclSuccess) {
    (void)hipFree(stage);
    return CRDT_ECOMM;
  }
  ctx->comm = comm;
  ctx->d_comm_stage = stage;
  ctx->n_ranks = n_ranks;
  ctx->rank = rank;
  return CRDT_OK;
}

int crdt_comm_destroy(crdt_ctx* ctx) {
  if (!ctx) return CRDT_EINVAL;
  if (!ctx->comm) return CRDT_OK;
  (void)set_dev(ctx);
  const ncclResult_t r = ncclCommDestroy((ncclComm_t)ctx->comm);
  (void)hipFree(ctx->d_comm_stage);
  ctx->d_comm_stage = nullptr;
  ctx->comm = nullptr;
  ctx->n_ranks = 0;
  return r == ncclSuccess ? CRDT_OK : CRDT_ECOMM;
}

int crdt_comm_count(crdt_ctx* ctx, int* h_count) {
  if (!ctx || !ctx->comm || !h_count) return CRDT_EINVAL;
  return nccl_rc(ncclCommCount((ncclComm_t)ctx->comm, h_count));
}

int crdt_replica_allreduce_max(crdt_ctx* ctx, uint64_t* d_rows, size_t n_words, void* stream) {
  if (!ctx || !ctx->comm || (n_words && !d_rows)) return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc) return rc;
  for (size_t s = 0; s < n_words && !rc; s += kAllReduceChunk) {
    const size_t cnt = std::min(kAllReduceChunk, n_words - s);
    rc = nccl_rc(ncclAllReduce(d_rows + s, d_rows + s, cnt, ncclUint64, ncclMax, (ncclComm_t)ctx->comm,
                               S(stream)));
  }
  return rc;
}

int crdt_replica_reduce_scatter_max(crdt_ctx* ctx, const uint64_t* d_rows, size_t n_words, uint64_t* d_shard,
                                    void* stream) {
  if (!ctx || !ctx->comm || ctx->n_ranks <= 0 || n_words % (size_t)ctx->n_ranks || (n_words && (!d_rows || !d_shard)))
    return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc) return rc;
  if (n_words == 0) return CRDT_OK;
  return nccl_rc(ncclReduceScatter(d_rows, d_shard, n_words / (size_t)ctx->n_ranks, ncclUint64, ncclMax,
                                   (ncclComm_t)ctx->comm, S(stream)));
}

// Dense rows over a caller transport (config 4 without RCCL): ring-free
// owner-sharded all-reduce — rank j owns words [lo(j), lo(j+1)); every rank
// sends each peer that peer's range (reduce-scatter), folds the R - 1
// received copies of its own range with dense_max_kernel, then sends its range
// to every peer (all-gather). Per rank 2(R - 1)/R of the rows sent and
// received; the max is order-free, so the result is bit-identical to
// ncclAllReduce(ncclMax) on every rank.
int dense_allreduce_rank(crdt_ctx* ctx, Transport& T, uint64_t* d_rows, size_t n, hipStream_t st) {
  const int R = T.R, me = T.me;
  if (R == 1) return CRDT_OK;
  auto lo = [&](int j) -> size_t { return (n / (size_t)R) * (size_t)j + std::min((size_t)j, n % (size_t)R); };
  const size_t my0 = lo(me), myn = lo(me + 1) - my0;
  // 0. every rank's (row count, arena verdict), all-gathered: every rank
  //    takes the same decision before any data moves (a rank that left here
  //    alone would leave its peers waiting in the exchange)
  int rc = n ? ensure_arena(ctx, al256(8 * myn * (size_t)(R - 1)) + 256) : CRDT_OK;
  {
    uint64_t mine[2] = {(uint64_t)n, (uint64_t)-rc};
    std::vector<uint64_t> G(2 * (size_t)R);
    const int trc = T.allgather(mine, 2, G.data(), st);
    if (trc) return trc;
    for (int p = 0; p < R; ++p) {
      if (G[2 * p] != n) return CRDT_EINVAL;  // the same row count on every rank
      if (G[2 * p + 1]) return -(int)G[2 * p + 1];
    }
  }
  if (n == 0) return CRDT_OK;
  uint64_t* scratch = (uint64_t*)ctx->d_arena;
  std::vector<Xfer> sends, recvs;
  for (int p = 0, k = 0; p < R; ++p) {
    if (p == me) continue;
    sends.push_back(Xfer{p, d_rows + lo(p), nullptr, 8 * (lo(p + 1) - lo(p))});
    recvs.push_back(Xfer{p, nullptr, scratch + (size_t)k * myn, 8 * myn});
    ++k;
  }
  if ((rc = T.exchange(sends, recvs, st))) return rc;
  for (int k = 0; k < R - 1 && !rc; ++k) rc = launch_dense_max(d_rows + my0, scratch + (size_t)k * myn, myn, st);
  // 1. the fold's launch verdict, all-gathered: no rank enters the all-gather
  //    exchange while a peer has left with an error
  {
    uint64_t e = (uint64_t)-rc;
    std::vector<uint64_t> E((size_t)R);
    const int trc = T.allgather(&e, 1, E.data(), st);
    if (trc) return trc;
    for (int p = 0; p < R; ++p)
      if (E[p]) return -(int)E[p];
  }
  sends.clear();
  recvs.clear();
  for (int p = 0; p < R; ++p) {
    if (p == me) continue;
    sends.push_back(Xfer{p, d_rows + my0, nullptr, 8 * myn});
    recvs.push_back(Xfer{p, nullptr, d_rows + lo(p), 8 * (lo(p + 1) - lo(p))});
  }
  if ((rc = T.exchange(sends, recvs, st))) return rc;
  return hipStreamSynchronize(st) == hipSuccess ? CRDT_OK : CRDT_EHIP;  // the arena is free again
}

// The owner-shard variant over a caller transport: the reduce-scatter half
// of dense_allreduce_rank. Rank j's shard is words [j n/R, (j+1) n/R) (n a
// multiple of R, as ncclReduceScatter): its own copy is the fold's start, the
// R - 1 received copies are maxed into it.
int dense_reduce_scatter_rank(crdt_ctx* ctx, Transport& T, const uint64_t* d_rows, size_t n, uint64_t* d_shard,
                              hipStream_t st) {
  const int R = T.R, me = T.me;
  const size_t w = n / (size_t)R;
  // a word count that does not split into R shards fails on every rank: it is
  // part of the all-gathered verdict, not a local early return that would
  // leave the peers waiting in the all-gather
  int rc = n % (size_t)R ? CRDT_EINVAL
           : w && R > 1  ? ensure_arena(ctx, al256(8 * w * (size_t)(R - 1)) + 256)
                         : CRDT_OK;
  if (R == 1 && rc) return rc;
  if (R > 1) {  // every rank's (word count, verdict) before any data moves
    uint64_t mine[2] = {(uint64_t)n, (uint64_t)-rc};
    std::vector<uint64_t> G(2 * (size_t)R);
    const int trc = T.allgather(mine, 2, G.data(), st);
    if (trc) return trc;
    for (int p = 0; p < R; ++p) {
      if (G[2 * p] != n) return CRDT_EINVAL;
      if (G[2 * p + 1]) return -(int)G[2 * p + 1];
    }
  }
  if (w == 0) return CRDT_OK;
  if (hipMemcpyAsync(d_shard, d_rows + w * (size_t)me, 8 * w, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return CRDT_EHIP;
  if (R == 1) return hipStreamSynchronize(st) == hipSuccess ? CRDT_OK : CRDT_EHIP;
  uint64_t* scratch = (uint64_t*)ctx->d_arena;
  std::vector<Xfer> sends, recvs;
  for (int p = 0, k = 0; p < R; ++p) {
    if (p == me) continue;
    sends.push_back(Xfer{p, d_rows + w * (size_t)p, nullptr, 8 * w});
    recvs.push_back(Xfer{p, nullptr, scratch + (size_t)k * w, 8 * w});
    ++k;
  }
  if ((rc = T.exchange(sends, recvs, st))) return rc;
  for (int k = 0; k < R - 1 && !rc; ++k) rc = launch_dense_max(d_shard, scratch + (size_t)k * w, w, st);
  if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = CRDT_EHIP;  // the arena is free again
  return rc;  // (no exchange follows: a local launch failure is this rank's alone)
}

int crdt_replica_reduce_scatter_max_transport(crdt_ctx* ctx, const crdt_transport* transport,
                                              const uint64_t* d_rows, size_t n_words, uint64_t* d_shard,
                                              void* stream) {
  if (!ctx || !transport || !transport->allgather || !transport->exchange || transport->n_ranks < 1 ||
      transport->rank < 0 || transport->rank >= transport->n_ranks || (n_words && (!d_rows || !d_shard)))
    return CRDT_EINVAL;  // (n_words % n_ranks is checked with the peers, dense_reduce_scatter_rank)
  int rc = set_dev(ctx);
  if (rc) return rc;
  CallbackTransport T(transport);
  return dense_reduce_scatter_rank(ctx, T, d_rows, n_words, d_shard, S(stream));
}

int crdt_replica_allreduce_max_transport(crdt_ctx* ctx, const crdt_transport* transport, uint64_t* d_rows,
                                         size_t n_words, void* stream) {
  if (!ctx || !transport || !transport->allgather || !transport->exchange || transport->n_ranks < 1 ||
      transport->rank < 0 || transport->rank >= transport->n_ranks || (n_words && !d_rows))
    return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc) return rc;
  CallbackTransport T(transport);
  return dense_allreduce_rank(ctx, T, d_rows, n_words, S(stream));
}

int crdt_orswot_replica_join_bound(crdt_ctx* ctx, const crdt_orswot_batch* mine, size_t* h_bound, void* stream) {
  if (!ctx || !ctx->comm || !mine || !h_bound) return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc || (rc = ensure_arena(ctx, 256))) return rc;
  const uint64_t v = al16(mine->bytes);
  uint64_t* d = (uint64_t*)ctx->d_arena;
  uint64_t sum = 0;
  if (hipMemcpyAsync(d, &v, 8, hipMemcpyHostToDevice, S(stream)) != hipSuccess) return CRDT_EHIP;
  if ((rc = nccl_rc(ncclAllReduce(d, d + 1, 1, ncclUint64, ncclSum, (ncclComm_t)ctx->comm, S(stream))))) return rc;
  if (hipMemcpyAsync(&sum, d + 1, 8, hipMemcpyDeviceToHost, S(stream)) != hipSuccess ||
      hipStreamSynchronize(S(stream)) != hipSuccess)
    return CRDT_EHIP;
  *h_bound = sum;
  return CRDT_OK;
}

int crdt_orswot_replica_join(crdt_ctx* ctx, const crdt_orswot_batch* mine, uint32_t n_actors, uint32_t flags,
                             uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, size_t* h_out_used,
                             void* stream) {
  if (!ctx || !ctx->comm || !mine || n_actors == 0 || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK)) return CRDT_EINVAL;
  if (mine->n_obj && (!d_out || !d_out_off || ((uintptr_t)d_out & 15u))) return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc) return rc;
  RcclTransport T(ctx, ctx->d_comm_stage);
  if (h_out_used) *h_out_used = 0;
  return orswot_join_rank(ctx, T, mine, n_actors, flags, d_out, d_out_off, out_bytes, h_out_used, S(stream));
}

int crdt_orswot_replica_join_transport(crdt_ctx* ctx, const crdt_transport* transport,
                                       const crdt_orswot_batch* mine, uint32_t n_actors, uint32_t flags,
                                       uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, size_t* h_out_used,
                                       void* stream) {
  if (!ctx || !transport || !transport->allgather || !transport->exchange || transport->n_ranks < 1 ||
      transport->rank < 0 || transport->rank >= transport->n_ranks || !mine || n_actors == 0 ||
      (flags & ~CRDT_ORSWOT_SPARSE_CLOCK))
    return CRDT_EINVAL;
  if (mine->n_obj && (!d_out || !d_out_off || ((uintptr_t)d_out & 15u))) return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc) return rc;
  CallbackTransport T(transport);
  if (h_out_used) *h_out_used = 0;
  return orswot_join_rank(ctx, T, mine, n_actors, flags, d_out, d_out_off, out_bytes, h_out_used, S(stream));
}

int crdt_orswot_replica_join_local(crdt_ctx* ctx, const crdt_orswot_batch* replicas, uint32_t n_replicas,
                                   uint32_t n_actors, uint32_t flags, uint8_t* d_out, uint64_t* d_out_off,
                                   size_t out_bytes, size_t* h_out_used, void* stream) {
  if (!ctx || !replicas || n_replicas == 0 || n_replicas > 64 || n_actors == 0 ||
      (flags & ~CRDT_ORSWOT_SPARSE_CLOCK))
    return CRDT_EINVAL;
  int rc = set_dev(ctx);
  if (rc) return rc;
  const int R = (int)n_replicas;
  ThreadGroup g(R);
  std::vector<crdt_ctx*> ctxs(R, nullptr);
  std::vector<hipStream_t> streams(R, nullptr);
  ctxs[0] = ctx;
  streams[0] = S(stream);
  for (int r = 0; r < R && !rc; ++r) {
    if (r && (rc = crdt_ctx_create(&ctxs[r], ctx->device))) break;
    if (r && hipStreamCreate(&streams[r]) != hipSuccess) rc = CRDT_EHIP;
    if (hipEventCreateWithFlags(&g.ready[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g.done[r], hipEventDisableTiming) != hipSuccess)
      rc = CRDT_EHIP;
  }
  std::vector<int> rcs(R, CRDT_OK);
  if (!rc) {
    if (h_out_used) *h_out_used = 0;
    auto run = [&](int r) {
      (void)hipSetDevice(ctx->device);
      ThreadTransport T(&g, r);
      rcs[r] = orswot_join_rank(ctxs[r], T, &replicas[r], n_actors, flags, r == 0 ? d_out : nullptr,
                                r == 0 ? d_out_off : nullptr, out_bytes, r == 0 ? h_out_used : nullptr, streams[r]);
    };
    std::vector<std::thread> th;
    for (int r = 1; r < R; ++r) th.emplace_back(run, r);
    run(0);
    for (auto& t : th) t.join();
    for (int r = 0; r < R && !rc; ++r) rc = rcs[r];
  }
  for (int r = 0; r < R; ++r) {
    if (streams[r]) (void)hipStreamSynchronize(streams[r]);
    if (r && streams[r]) (void)hipStreamDestroy(streams[r]);
    if (r && ctxs[r]) (void)crdt_ctx_destroy(ctxs[r]);
    if (g.ready[r]) (void)hipEventDestroy(g.ready[r]);
    if (g.done[r]) (void)hipEventDestroy(g.done[r]);
  }
  return rc;
}

}  // extern "C"
