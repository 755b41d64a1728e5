// C ABI of crdts_hip (include/crdts_hip.h): argument validation, the context,
// and launches. Nothing here falls back to a CPU implementation: without a
// usable gfx950 device every device entry point returns CRDT_ENODEV/EHIP.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <vector>

#include "../../include/crdts_hip.h"
#include "ctx.h"
#include "kernels.h"
#include "record_layout.h"

using namespace crdts_hip;


namespace {

inline hipStream_t S(void* s) { return (hipStream_t)s; }

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int set_device(crdt_ctx* ctx) {
  if (!ctx) return CRDT_EINVAL;
  return hipSetDevice(ctx->device) == hipSuccess ? CRDT_OK : CRDT_EHIP;
}

int dense(crdt_ctx* ctx, uint64_t* self, const uint64_t* other, size_t n_obj, uint64_t slots,
          void* stream) {
  if (!ctx || (n_obj && (!self || !other)) || slots == 0) return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_dense_max(self, other, (uint64_t)n_obj * slots, S(stream));
}

}  // namespace

int ctx_big_scratch(crdt_ctx* ctx, size_t bytes) {
  if (ctx->big_bytes >= bytes) return CRDT_OK;
  // the previous scratch may still be read by queued kernels of this context:
  // hipFree synchronises the device first
  (void)hipFree(ctx->d_big);
  ctx->d_big = nullptr;
  ctx->big_bytes = 0;
  if (hipMalloc(&ctx->d_big, bytes) != hipSuccess) return CRDT_EHIP;
  ctx->big_bytes = bytes;
  return CRDT_OK;
}

extern "C" {

int crdt_abi_version(void) { return CRDT_ABI_VERSION; }

const char* crdt_strerror(int code) {
  switch (code) {
    case CRDT_OK: return "ok";
    case CRDT_EINVAL: return "invalid argument";
    case CRDT_ENONCANON: return "non-canonical or inconsistent record";
    case CRDT_EHIP: return "HIP runtime error";
    case CRDT_ECAPACITY: return "output capacity too small";
    case CRDT_ECOMM: return "communicator error";
    case CRDT_ENODEV: return "no usable gfx950 device";
    default: return "unknown error";
  }
}

int crdt_ctx_create(crdt_ctx** out, int device) {
  if (!out) return CRDT_EINVAL;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice || (e == hipSuccess && (device < 0 || device >= n))) return CRDT_ENODEV;
  if (e != hipSuccess) return CRDT_EHIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return CRDT_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CRDT_ENODEV;
  if (hipSetDevice(device) != hipSuccess) return CRDT_EHIP;
  auto* c = new crdt_ctx();
  c->device = device;
  c->blocks_per_cu = 0;
  c->list_cap = kDefaultListCap;
  c->variant = 0;
  // status, ctl, the general-path list, the per-wave store sink; the deferred
  // list after it is read and written only by the two-pass join variants of
  // the diagnostic build
#ifdef CRDT_DIAG
  const size_t bytes = 64 + 8ull * kDefaultListCap + kTrashBytes + 8ull * kDeferListCap;
#else
  const size_t bytes = 64 + 8ull * kDefaultListCap + kTrashBytes;
#endif
  uint8_t* scratch = nullptr;
  if (hipMalloc(&scratch, bytes) != hipSuccess || hipMemset(scratch, 0, bytes) != hipSuccess) {
    (void)hipFree(scratch);
    delete c;
    return CRDT_EHIP;
  }
  c->d_status = (int*)scratch;
  c->d_ctl = (uint32_t*)(scratch + 16);
  c->d_list = (uint64_t*)(scratch + 64);
  *out = c;
  return CRDT_OK;
}

int crdt_ctx_destroy(crdt_ctx* ctx) {
  if (!ctx) return CRDT_EINVAL;
  (void)hipSetDevice(ctx->device);
  (void)crdt_comm_destroy(ctx);
  (void)hipFree(ctx->d_big);
  (void)hipFree(ctx->d_arena);
  (void)hipFree(ctx->d_fold);
  (void)hipFree(ctx->d_status);
  delete ctx;
  return CRDT_OK;
}

int crdt_ctx_status(crdt_ctx* ctx, void* stream) {
  int rc = set_device(ctx);
  if (rc) return rc;
  if (hipStreamSynchronize(S(stream)) != hipSuccess) return CRDT_EHIP;
  int st = 0;
  if (hipMemcpy(&st, ctx->d_status, sizeof st, hipMemcpyDeviceToHost) != hipSuccess) return CRDT_EHIP;
  if (st != 0 && hipMemset(ctx->d_status, 0, sizeof(int)) != hipSuccess) return CRDT_EHIP;
  return st;
}

int crdt_ctx_set_arena_limit(crdt_ctx* ctx, size_t max_bytes) {
  if (!ctx) return CRDT_EINVAL;
  ctx->arena_limit = max_bytes;
  return CRDT_OK;
}

int crdt_ctx_set_list_cap(crdt_ctx* ctx, uint32_t cap) {
  if (!ctx || cap > kDefaultListCap) return CRDT_EINVAL;
  ctx->list_cap = cap;
  return CRDT_OK;
}

#ifdef CRDT_DIAG
// Diagnostic build only (-DCRDT_DIAG, lib/libcrdts_hip_diag.so, used by
// tools/): copy the context's list buffer
// (holds per-wave phase stamps after a variant-109 launch).
int crdt_ctx_debug_read(crdt_ctx* ctx, uint64_t* h_out, size_t n, void* stream) {
  if (!ctx || !h_out || n > 8ull * kDefaultListCap / 8) return CRDT_EINVAL;
  if (hipMemcpyAsync(h_out, ctx->d_list, 8 * n, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
      hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
    return CRDT_EHIP;
  return CRDT_OK;
}

// Orswot kernel variant (diagnostic build only).
int crdt_ctx_set_variant(crdt_ctx* ctx, int v) {
  if (!ctx || v < 0) return CRDT_EINVAL;
  ctx->variant = v;
  return CRDT_OK;
}

// Workgroups per CU for the Orswot kernel (diagnostic build only).
int crdt_ctx_set_blocks_per_cu(crdt_ctx* ctx, int k) {
  if (!ctx || k < 0 || k > 64) return CRDT_EINVAL;  // 0 = the variant's occupancy
  ctx->blocks_per_cu = k;
  return CRDT_OK;
}
#endif  // CRDT_DIAG

int crdt_vclock_dense_merge(crdt_ctx* ctx, uint64_t* d_self, const uint64_t* d_other, size_t n_obj,
                            uint32_t n_actors, void* stream) {
  return dense(ctx, d_self, d_other, n_obj, n_actors, stream);
}
int crdt_gcounter_merge(crdt_ctx* ctx, uint64_t* d_self, const uint64_t* d_other, size_t n_obj,
                        uint32_t n_actors, void* stream) {
  return dense(ctx, d_self, d_other, n_obj, n_actors, stream);
}
int crdt_pncounter_merge(crdt_ctx* ctx, uint64_t* d_self, const uint64_t* d_other, size_t n_obj,
                         uint32_t n_actors, void* stream) {
  return dense(ctx, d_self, d_other, n_obj, 2ull * n_actors, stream);
}

namespace {
int csr_args_ok(const crdt_clock_csr* s, const crdt_clock_csr* o, const crdt_clock_csr_out* out) {
  if (!s || !o || !out || s->n_obj != o->n_obj) return CRDT_EINVAL;
  if (s->n_obj && (!s->off || !s->len || !o->off || !o->len || !out->off || !out->len)) return CRDT_EINVAL;
  if (s->n_entries && (!s->act || !s->ctr)) return CRDT_EINVAL;
  if (o->n_entries && (!o->act || !o->ctr)) return CRDT_EINVAL;
  if (out->n_entries && (!out->act || !out->ctr)) return CRDT_EINVAL;
  if (out->n_entries < s->n_entries + o->n_entries) return CRDT_ECAPACITY;
  return CRDT_OK;
}
}  // namespace

int crdt_vclock_csr_merge(crdt_ctx* ctx, const crdt_clock_csr* self, const crdt_clock_csr* other,
                          const crdt_clock_csr_out* out, void* stream) {
  if (!ctx) return CRDT_EINVAL;
  int rc = csr_args_ok(self, other, out);
  if (rc || (rc = set_device(ctx))) return rc;
  return launch_clock_csr_merge(&self, &other, &out, 1, ctx->d_status, S(stream));
}
int crdt_gcounter_csr_merge(crdt_ctx* ctx, const crdt_clock_csr* self, const crdt_clock_csr* other,
                            const crdt_clock_csr_out* out, void* stream) {
  return crdt_vclock_csr_merge(ctx, self, other, out, stream);
}
int crdt_pncounter_csr_merge(crdt_ctx* ctx, const crdt_clock_csr* self_p, const crdt_clock_csr* self_n,
                             const crdt_clock_csr* other_p, const crdt_clock_csr* other_n,
                             const crdt_clock_csr_out* out_p, const crdt_clock_csr_out* out_n, void* stream) {
  if (!ctx || !self_p || !self_n || self_p->n_obj != self_n->n_obj) return CRDT_EINVAL;
  int rc = csr_args_ok(self_p, other_p, out_p);
  if (rc || (rc = csr_args_ok(self_n, other_n, out_n)) || (rc = set_device(ctx))) return rc;
  const crdt_clock_csr* s[2] = {self_p, self_n};
  const crdt_clock_csr* o[2] = {other_p, other_n};
  const crdt_clock_csr_out* w[2] = {out_p, out_n};
  return launch_clock_csr_merge(s, o, w, 2, ctx->d_status, S(stream));
}

int crdt_orswot_truncate(crdt_ctx* ctx, const crdt_orswot_batch* self, const crdt_clock_csr* clocks,
                         uint32_t n_actors, uint32_t flags, uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes,
                         void* stream) {
  if (!ctx || !self || !clocks || n_actors == 0 || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK) ||
      clocks->n_obj != self->n_obj)
    return CRDT_EINVAL;
  if (self->n_obj == 0) return CRDT_OK;
  if (!self->base || !self->off || !clocks->off || !clocks->len || !d_out || !d_out_off || !aligned16(d_out))
    return CRDT_EINVAL;
  if (clocks->n_entries && (!clocks->act || !clocks->ctr)) return CRDT_EINVAL;
  if (out_bytes < self->bytes) return CRDT_ECAPACITY;
  // out must not alias the input: the HBM form compacts sections toward lower
  // offsets while other lanes still read them
  const uintptr_t ib = (uintptr_t)self->base, ob = (uintptr_t)d_out;
  if (ob < ib + self->bytes && ib < ob + out_bytes) return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_orswot_truncate(*self, *clocks, n_actors, flags, d_out, d_out_off, out_bytes, ctx->d_status,
                                ctx->d_ctl, ctx->d_list, ctx->list_cap, S(stream));
}

int crdt_dense_merge_host(crdt_ctx* ctx, uint64_t* h_self, const uint64_t* h_other, size_t n_obj, uint32_t n_slots) {
  if (!ctx || n_slots == 0 || (n_obj && (!h_self || !h_other))) return CRDT_EINVAL;
  if (n_obj == 0) return CRDT_OK;
  int rc = set_device(ctx);
  if (rc) return rc;
  const size_t bytes = 8ull * n_obj * n_slots;
  uint64_t *dS = nullptr, *dO = nullptr;
  hipStream_t st = nullptr;
  bool ok = hipStreamCreate(&st) == hipSuccess && hipMalloc(&dS, bytes) == hipSuccess &&
            hipMalloc(&dO, bytes) == hipSuccess &&
            hipMemcpyAsync(dS, h_self, bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(dO, h_other, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
  if (ok) rc = launch_dense_max(dS, dO, (uint64_t)n_obj * n_slots, st);
  ok = ok && rc == CRDT_OK && hipMemcpyAsync(h_self, dS, bytes, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipStreamSynchronize(st) == hipSuccess;
  (void)hipFree(dS);
  (void)hipFree(dO);
  if (st) (void)hipStreamDestroy(st);
  return ok ? CRDT_OK : (rc ? rc : CRDT_EHIP);
}

int crdt_orswot_merge(crdt_ctx* ctx, const crdt_orswot_batch* self, const crdt_orswot_batch* other,
                      uint8_t* d_out_base, uint64_t* d_out_off, size_t out_bytes, uint32_t n_actors,
                      void* stream) {
  return crdt_orswot_merge_ex(ctx, self, other, d_out_base, d_out_off, out_bytes, n_actors, 0u, stream);
}

int crdt_orswot_merge_ex(crdt_ctx* ctx, const crdt_orswot_batch* self, const crdt_orswot_batch* other,
                         uint8_t* d_out_base, uint64_t* d_out_off, size_t out_bytes, uint32_t n_actors,
                         uint32_t flags, void* stream) {
  if (!ctx || !self || !other || n_actors == 0 || self->n_obj != other->n_obj) return CRDT_EINVAL;
  if (flags & ~CRDT_ORSWOT_SPARSE_CLOCK) return CRDT_EINVAL;
  if (self->n_obj == 0) return CRDT_OK;
  if (!self->base || !self->off || !other->base || !other->off || !d_out_base || !d_out_off)
    return CRDT_EINVAL;
  if (!aligned16(self->base) || !aligned16(other->base) || !aligned16(d_out_base)) return CRDT_EINVAL;
  if (out_bytes < self->bytes + other->bytes) return CRDT_ECAPACITY;
  int rc = set_device(ctx);
  if (rc) return rc;
  if (flags & CRDT_ORSWOT_SPARSE_CLOCK)
    return launch_orswot_merge_sparse(self->base, self->off, self->bytes, other->base, other->off, other->bytes,
                                      d_out_base, d_out_off, out_bytes, self->n_obj, n_actors, ctx->d_status,
                                      ctx->d_ctl, ctx->d_list, ctx->list_cap, S(stream),
                                      ctx->variant >= 201 && ctx->variant <= 211 ? ctx->variant - 200 : 0,
                                      &ctx->join_seq);
  return launch_orswot_merge(self->base, self->off, self->bytes, other->base, other->off,
                             other->bytes, d_out_base, d_out_off, out_bytes, self->n_obj, n_actors,
                             ctx->d_status, ctx->d_ctl, ctx->d_list, ctx->list_cap, S(stream),
                             ctx->blocks_per_cu, ctx->variant, &ctx->join_seq);
}

int crdt_orswot_fold(crdt_ctx* ctx, const crdt_orswot_batch* reps, uint32_t n_reps, uint32_t n_actors,
                     uint32_t flags, uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, void* stream) {
  if (!ctx || !reps || n_reps == 0 || n_actors == 0 || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK)) return CRDT_EINVAL;
  const size_t n = reps[0].n_obj;
  size_t total = 0;
  for (uint32_t r = 0; r < n_reps; ++r) {
    if (reps[r].n_obj != n) return CRDT_EINVAL;
    if (n && (!reps[r].base || !reps[r].off || !aligned16(reps[r].base))) return CRDT_EINVAL;
    total += reps[r].bytes;
  }
  if (n == 0) return CRDT_OK;
  if (!d_out || !d_out_off || !aligned16(d_out)) return CRDT_EINVAL;
  if (out_bytes < total) return CRDT_ECAPACITY;
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = S(stream);
  if (n_reps == 1) {  // the batch itself, at its own offsets
    if (hipMemcpyAsync(d_out, reps[0].base, reps[0].bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_out_off, reps[0].off, 8 * n, hipMemcpyDeviceToDevice, st) != hipSuccess)
      return CRDT_EHIP;
    return launch_orswot_validate(d_out, d_out_off, out_bytes, n, n_actors, flags, ctx->d_status, st);
  }
  // intermediate batches: two of the first n_reps - 1 batches' bytes together
  // (an accumulator never outgrows its inputs) plus their offsets
  const size_t acc_cap = (total - reps[n_reps - 1].bytes + 255) & ~size_t(255);
  const size_t need = 2 * acc_cap + 2 * ((8 * n + 255) & ~size_t(255));
  if (n_reps > 2 && ctx->fold_bytes < need) {
    (void)hipFree(ctx->d_fold);
    ctx->d_fold = nullptr;
    ctx->fold_bytes = 0;
    if (hipMalloc(&ctx->d_fold, need) != hipSuccess) return CRDT_EHIP;
    ctx->fold_bytes = need;
  }
  uint8_t* buf[2] = {ctx->d_fold, ctx->d_fold + acc_cap};
  uint64_t* boff[2] = {(uint64_t*)(ctx->d_fold + 2 * acc_cap),
                       (uint64_t*)(ctx->d_fold + 2 * acc_cap + ((8 * n + 255) & ~size_t(255)))};
  const uint8_t* acc = reps[0].base;
  const uint64_t* acc_off = reps[0].off;
  uint64_t acc_bytes = reps[0].bytes;
  for (uint32_t r = 1; r < n_reps && !rc; ++r) {  // ((r0 ⊔ r1) ⊔ r2) ⊔ ..., each step one batched merge
    const bool last = r + 1 == n_reps;
    uint8_t* o = last ? d_out : buf[r & 1u];
    uint64_t* oo = last ? d_out_off : boff[r & 1u];
    const uint64_t cap = last ? out_bytes : acc_bytes + reps[r].bytes;
    rc = (flags & CRDT_ORSWOT_SPARSE_CLOCK)
             ? launch_orswot_merge_sparse(acc, acc_off, acc_bytes, reps[r].base, reps[r].off, reps[r].bytes, o, oo,
                                          cap, n, n_actors, ctx->d_status, ctx->d_ctl, ctx->d_list, ctx->list_cap,
                                          st, 0, &ctx->join_seq)
             : launch_orswot_merge(acc, acc_off, acc_bytes, reps[r].base, reps[r].off, reps[r].bytes, o, oo, cap, n,
                                   n_actors, ctx->d_status, ctx->d_ctl, ctx->d_list, ctx->list_cap, st, 0, 0,
                                   &ctx->join_seq);
    acc = o;
    acc_off = oo;
    acc_bytes = cap;
  }
  return rc;
}

int crdt_orswot_validate(crdt_ctx* ctx, const crdt_orswot_batch* batch, uint32_t n_actors,
                         void* stream) {
  return crdt_orswot_validate_ex(ctx, batch, n_actors, 0u, stream);
}

int crdt_orswot_validate_ex(crdt_ctx* ctx, const crdt_orswot_batch* batch, uint32_t n_actors, uint32_t flags,
                            void* stream) {
  if (!ctx || !batch || n_actors == 0 || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK)) return CRDT_EINVAL;
  if (batch->n_obj && (!batch->base || !batch->off)) return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_orswot_validate(batch->base, batch->off, batch->bytes, batch->n_obj, n_actors, flags,
                                ctx->d_status, S(stream));
}

size_t crdt_orswot_compact_scratch_bytes(size_t n_obj) {
  size_t temp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                   (int)(n_obj ? n_obj : 1));
  return ((8 * n_obj + 255) & ~size_t(255)) + temp + 256;
}

uint64_t crdt_ctx_host_syncs(const crdt_ctx* ctx) { return ctx ? ctx->host_syncs : 0ull; }

int crdt_orswot_compact(crdt_ctx* ctx, const crdt_orswot_batch* src, uint8_t* d_dst,
                        uint64_t* d_dst_off, size_t dst_bytes, void* d_scratch, void* stream) {
  if (!ctx || !src || (src->n_obj && (!src->base || !src->off || !d_dst || !d_dst_off || !d_scratch)))
    return CRDT_EINVAL;
  if (src->n_obj == 0) return CRDT_OK;
  if (src->n_obj > 0x7FFFFFFFull) return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  uint64_t* sizes = (uint64_t*)d_scratch;
  uint8_t* temp = (uint8_t*)d_scratch + ((8 * src->n_obj + 255) & ~size_t(255));
  size_t temp_bytes = crdt_orswot_compact_scratch_bytes(src->n_obj) -
                      ((8 * src->n_obj + 255) & ~size_t(255)) - 256;
  if ((rc = launch_record_sizes(src->base, src->off, src->bytes, src->n_obj, sizes, ctx->d_status, S(stream))))
    return rc;
  if (hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, sizes, d_dst_off, (int)src->n_obj,
                                       S(stream)) != hipSuccess)
    return CRDT_EHIP;
  // bound check: last offset + last size <= dst_bytes (host round trip is fine here)
  uint64_t last_off = 0, last_size = 0;
  if (hipMemcpyAsync(&last_off, d_dst_off + src->n_obj - 1, 8, hipMemcpyDeviceToHost, S(stream)) !=
          hipSuccess ||
      hipMemcpyAsync(&last_size, sizes + src->n_obj - 1, 8, hipMemcpyDeviceToHost, S(stream)) !=
          hipSuccess ||
      hipStreamSynchronize(S(stream)) != hipSuccess)
    return CRDT_EHIP;
  if (last_off + last_size > dst_bytes) return CRDT_ECAPACITY;
  return launch_record_copy(src->base, src->off, sizes, d_dst, d_dst_off, src->n_obj, dst_bytes, S(stream));
}

int crdt_orswot_merge_host(crdt_ctx* ctx, const uint8_t* h_self_base, const uint64_t* h_self_off,
                           size_t self_bytes, const uint8_t* h_other_base,
                           const uint64_t* h_other_off, size_t other_bytes, size_t n_obj,
                           uint32_t n_actors, uint8_t* h_out_base, uint64_t* h_out_off,
                           size_t h_out_bytes, size_t* h_out_used) {
  if (!ctx || n_actors == 0) return CRDT_EINVAL;
  if (n_obj == 0) {
    if (h_out_used) *h_out_used = 0;
    return CRDT_OK;
  }
  if (!h_self_base || !h_self_off || !h_other_base || !h_other_off || !h_out_base || !h_out_off)
    return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  size_t sb = (self_bytes + 15) & ~size_t(15), ob = (other_bytes + 15) & ~size_t(15);
  size_t outb = sb + ob;
  uint8_t *dL = nullptr, *dR = nullptr, *dO = nullptr;
  uint64_t *dLo = nullptr, *dRo = nullptr, *dOo = nullptr;
  hipStream_t st = nullptr;
  auto cleanup = [&]() {
    (void)hipFree(dL); (void)hipFree(dR); (void)hipFree(dO);
    (void)hipFree(dLo); (void)hipFree(dRo); (void)hipFree(dOo);
    if (st) (void)hipStreamDestroy(st);
  };
  if (hipStreamCreate(&st) != hipSuccess || hipMalloc(&dL, sb) != hipSuccess ||
      hipMalloc(&dR, ob) != hipSuccess || hipMalloc(&dO, outb) != hipSuccess ||
      hipMalloc(&dLo, 8 * n_obj) != hipSuccess || hipMalloc(&dRo, 8 * n_obj) != hipSuccess ||
      hipMalloc(&dOo, 8 * n_obj) != hipSuccess) {
    cleanup();
    return CRDT_EHIP;
  }
  bool ok = hipMemcpyAsync(dL, h_self_base, self_bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(dR, h_other_base, other_bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(dLo, h_self_off, 8 * n_obj, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(dRo, h_other_off, 8 * n_obj, hipMemcpyHostToDevice, st) == hipSuccess;
  if (!ok) { cleanup(); return CRDT_EHIP; }
  crdt_orswot_batch Lb = {dL, dLo, n_obj, sb}, Rb = {dR, dRo, n_obj, ob};
  rc = crdt_orswot_merge(ctx, &Lb, &Rb, dO, dOo, outb, n_actors, st);
  if (rc == CRDT_OK) rc = crdt_ctx_status(ctx, st);
  if (rc != CRDT_OK) { cleanup(); return rc; }
  std::vector<uint64_t> offs(n_obj);
  std::vector<uint8_t> out(outb);
  ok = hipMemcpyAsync(offs.data(), dOo, 8 * n_obj, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(out.data(), dO, outb, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipStreamSynchronize(st) == hipSuccess;
  cleanup();
  if (!ok) return CRDT_EHIP;
  size_t pos = 0;
  for (size_t i = 0; i < n_obj; ++i) {
    uint32_t size;
    std::memcpy(&size, out.data() + offs[i], 4);
    if (pos + size > h_out_bytes) return CRDT_ECAPACITY;
    std::memcpy(h_out_base + pos, out.data() + offs[i], size);
    h_out_off[i] = pos;
    pos += size;
  }
  if (h_out_used) *h_out_used = pos;
  return CRDT_OK;
}

// ---------------------------------------------------------------- bincode codec
namespace {
bool bc_width_ok(uint32_t w) { return w == 1u || w == 2u || w == 4u || w == 8u; }
}  // namespace

int crdt_orswot_bincode_record_sizes(crdt_ctx* ctx, const uint8_t* d_blobs, size_t blob_bytes,
                                     const uint64_t* d_blob_off, const uint64_t* d_blob_len, size_t n_obj,
                                     uint32_t actor_bytes, uint32_t member_bytes, uint32_t n_actors,
                                     uint32_t flags, uint64_t* d_sizes, void* stream) {
  if (!ctx || (n_obj && (!d_blobs || !d_blob_off || !d_blob_len || !d_sizes)) || n_actors == 0 ||
      !bc_width_ok(actor_bytes) || !bc_width_ok(member_bytes) || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK))
    return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_bincode_ingest(d_blobs, blob_bytes, d_blob_off, d_blob_len, n_obj, actor_bytes, member_bytes,
                               n_actors, flags, d_sizes, nullptr, nullptr, 0, ctx->d_status, ctx->d_ctl, S(stream));
}

int crdt_orswot_bincode_record_bounds(crdt_ctx* ctx, const uint64_t* d_blob_len, size_t n_obj,
                                      uint32_t actor_bytes, uint32_t member_bytes, uint32_t n_actors, uint32_t flags,
                                      uint64_t* d_bounds, void* stream) {
  if (!ctx || (n_obj && (!d_blob_len || !d_bounds)) || !bc_width_ok(actor_bytes) || !bc_width_ok(member_bytes) ||
      n_actors == 0 || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK))
    return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_bincode_bounds(d_blob_len, n_obj, actor_bytes, member_bytes, n_actors, flags, d_bounds, S(stream));
}

int crdt_orswot_from_bincode(crdt_ctx* ctx, const uint8_t* d_blobs, size_t blob_bytes,
                             const uint64_t* d_blob_off, const uint64_t* d_blob_len, size_t n_obj,
                             uint32_t actor_bytes, uint32_t member_bytes, uint32_t n_actors, uint32_t flags,
                             uint8_t* d_out, const uint64_t* d_out_off, size_t out_bytes, void* stream) {
  if (!ctx || (n_obj && (!d_blobs || !d_blob_off || !d_blob_len || !d_out || !d_out_off)) || n_actors == 0 ||
      !bc_width_ok(actor_bytes) || !bc_width_ok(member_bytes) || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK) ||
      !aligned16(d_out))
    return CRDT_EINVAL;
  int rc = set_device(ctx);
  const size_t big = launch_apply_huge_scratch_bytes() > launch_bincode_big_scratch_bytes()
                         ? launch_apply_huge_scratch_bytes() : launch_bincode_big_scratch_bytes();
  if (rc || (rc = ctx_big_scratch(ctx, big))) return rc;
  return launch_bincode_ingest(d_blobs, blob_bytes, d_blob_off, d_blob_len, n_obj, actor_bytes, member_bytes,
                               n_actors, flags, nullptr, d_out, d_out_off, out_bytes, ctx->d_status, ctx->d_ctl, S(stream),
                               ctx->variant == 301 ? ctx->d_list : nullptr, ctx->d_list, ctx->list_cap, ctx->d_big,
                               ctx->variant == 305 ? 1 : ctx->variant == 304 ? 2 : ctx->variant == 306 ? 3 : 0);
}

int crdt_orswot_bincode_sizes(crdt_ctx* ctx, const crdt_orswot_batch* batch, uint32_t n_actors, uint32_t flags,
                              uint32_t actor_bytes, uint32_t member_bytes, uint64_t* d_sizes, void* stream) {
  if (!ctx || !batch || (batch->n_obj && (!batch->base || !batch->off || !d_sizes)) || n_actors == 0 ||
      !bc_width_ok(actor_bytes) || !bc_width_ok(member_bytes) || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK) ||
      (batch->n_obj && !aligned16(batch->base)))
    return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_bincode_egest(batch->base, batch->bytes, batch->off, batch->n_obj, n_actors, flags, actor_bytes,
                              member_bytes, d_sizes, nullptr, nullptr, 0, ctx->d_status, ctx->d_ctl, S(stream));
}

int crdt_orswot_to_bincode(crdt_ctx* ctx, const crdt_orswot_batch* batch, uint32_t n_actors, uint32_t flags,
                           uint32_t actor_bytes, uint32_t member_bytes, uint8_t* d_out,
                           const uint64_t* d_out_off, size_t out_bytes, void* stream) {
  if (!ctx || !batch || (batch->n_obj && (!batch->base || !batch->off || !d_out || !d_out_off)) ||
      n_actors == 0 || !bc_width_ok(actor_bytes) || !bc_width_ok(member_bytes) ||
      (flags & ~CRDT_ORSWOT_SPARSE_CLOCK) || (batch->n_obj && (!aligned16(batch->base) || !aligned16(d_out))))
    return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_bincode_egest(batch->base, batch->bytes, batch->off, batch->n_obj, n_actors, flags, actor_bytes,
                              member_bytes, nullptr, d_out, d_out_off, out_bytes, ctx->d_status, ctx->d_ctl, S(stream));
}

int crdt_orswot_apply(crdt_ctx* ctx, const crdt_orswot_batch* self, const crdt_orswot_ops* ops, uint32_t n_actors,
                      uint32_t flags, uint8_t* d_out, uint64_t* d_out_off, size_t out_bytes, void* stream) {
  if (!ctx || !self || !ops || n_actors == 0 || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK)) return CRDT_EINVAL;
  if (self->n_obj && (!self->base || !self->off || !ops->obj_end || !d_out || !d_out_off || !aligned16(d_out)))
    return CRDT_EINVAL;
  if (ops->n_ops && (!ops->kind || !ops->member || !ops->actor || !ops->counter || !ops->clk_end))
    return CRDT_EINVAL;
  if (ops->n_clk && (!ops->clk_act || !ops->clk_ctr)) return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  const size_t big = launch_apply_huge_scratch_bytes() > launch_bincode_big_scratch_bytes()
                         ? launch_apply_huge_scratch_bytes() : launch_bincode_big_scratch_bytes();
  if ((rc = ctx_big_scratch(ctx, big))) return rc;
  return launch_orswot_apply(self->base, self->bytes, self->off, self->n_obj, ops->obj_end, ops->kind, ops->member,
                             ops->actor, ops->counter, ops->clk_end, ops->clk_act, ops->clk_ctr, ops->n_ops, ops->n_clk,
                             n_actors, flags,
                             d_out, d_out_off, out_bytes, ctx->d_status, ctx->d_ctl, ctx->d_list, ctx->list_cap,
                             ctx->d_big, S(stream));
}

int crdt_vclock_partial_cmp(crdt_ctx* ctx, const uint64_t* d_a, const uint64_t* d_b, size_t n, uint32_t n_actors,
                            int8_t* d_out, void* stream) {
  if (!ctx || n_actors == 0 || (n && (!d_a || !d_b || !d_out))) return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_vclock_cmp(d_a, d_b, n, n_actors, d_out, S(stream));
}

int crdt_mvreg_merge(crdt_ctx* ctx, const uint32_t* d_self_n, const uint64_t* d_self_clk, const uint64_t* d_self_val,
                     uint32_t self_cap, const uint32_t* d_other_n, const uint64_t* d_other_clk,
                     const uint64_t* d_other_val, uint32_t other_cap, uint32_t* d_out_n, uint64_t* d_out_clk,
                     uint64_t* d_out_val, uint32_t out_cap, size_t n_obj, uint32_t n_actors, void* stream) {
  if (!ctx || n_actors == 0 || self_cap == 0 || other_cap == 0 || self_cap > 1024 || other_cap > 1024 || out_cap == 0)
    return CRDT_EINVAL;
  if (n_obj && (!d_self_n || !d_self_clk || !d_self_val || !d_other_n || !d_other_clk || !d_other_val || !d_out_n ||
                !d_out_clk || !d_out_val))
    return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_mvreg_merge(d_self_n, d_self_clk, d_self_val, self_cap, d_other_n, d_other_clk, d_other_val,
                            other_cap, d_out_n, d_out_clk, d_out_val, out_cap, n_obj, n_actors, ctx->d_status,
                            S(stream));
}

int crdt_map_mvreg_merge(crdt_ctx* ctx, const crdt_map_mvreg_slab* self, const crdt_map_mvreg_slab* other,
                         const crdt_map_mvreg_slab* out, size_t n_obj, uint32_t n_actors, void* stream) {
  if (!ctx || !self || !other || !out || n_actors == 0 || n_actors > 128) return CRDT_EINVAL;
  for (const crdt_map_mvreg_slab* x : {self, other})
    if (x->kcap == 0 || x->kcap > 4096 || x->mcap == 0 || x->mcap > 128 || x->dcap == 0 || x->dcap > 64 ||
        x->scap == 0 || x->scap > 4096)
      return CRDT_EINVAL;
  if (out->kcap < self->kcap + other->kcap || out->mcap < self->mcap + other->mcap ||
      out->dcap < self->dcap + other->dcap || out->scap < self->scap + other->scap)
    return CRDT_EINVAL;
  if (n_obj)
    for (const crdt_map_mvreg_slab* x : {self, other, out})
      if (!x->clock || !x->n_keys || !x->keys || !x->eclock || !x->mv_n || !x->mv_clock || !x->mv_val || !x->n_def ||
          !x->dclock || !x->dset_n || !x->dset)
        return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_map_mvreg_merge(*self, *other, *out, n_obj, n_actors, ctx->d_status, ctx->d_ctl, S(stream),
                                ctx->variant);
}

static bool map_mvreg_caps_ok(const crdt_map_mvreg_slab* x) {
  return x->kcap && x->kcap <= 4096 && x->mcap && x->mcap <= 128 && x->dcap && x->dcap <= 64 && x->scap &&
         x->scap <= 4096;
}
static bool map_mvreg_ptrs_ok(const crdt_map_mvreg_slab* x) {
  return x->clock && x->n_keys && x->keys && x->eclock && x->mv_n && x->mv_clock && x->mv_val && x->n_def && x->dclock &&
         x->dset_n && x->dset;
}

size_t crdt_map_map_merge_scratch_bytes(const crdt_map_map_slab* out, size_t n_obj, uint32_t n_actors) {
  return out ? map_map_scratch_bytes(*out, n_obj, n_actors) : 0u;
}

int crdt_map_map_merge(crdt_ctx* ctx, const crdt_map_map_slab* self, const crdt_map_map_slab* other,
                       const crdt_map_map_slab* out, size_t n_obj, uint32_t n_actors, void* d_scratch,
                       size_t scratch_bytes, void* stream) {
  if (!ctx || !self || !other || !out || n_actors == 0 || n_actors > 128) return CRDT_EINVAL;
  for (const crdt_map_map_slab* x : {self, other})
    if (x->kcap == 0 || x->kcap > 4096 || x->dcap == 0 || x->dcap > 64 || x->scap == 0 || x->scap > 4096 ||
        !map_mvreg_caps_ok(&x->inner))
      return CRDT_EINVAL;
  const crdt_map_mvreg_slab &si = self->inner, &oi = other->inner, &ri = out->inner;
  if (out->kcap < self->kcap + other->kcap || out->dcap < self->dcap + other->dcap ||
      out->scap < self->scap + other->scap || ri.kcap < si.kcap + oi.kcap || ri.mcap < si.mcap + oi.mcap ||
      ri.dcap < si.dcap + oi.dcap || ri.scap < si.scap + oi.scap)
    return CRDT_EINVAL;
  if (n_obj) {
    for (const crdt_map_map_slab* x : {self, other, out})
      if (!x->clock || !x->n_keys || !x->keys || !x->eclock || !x->n_def || !x->dclock || !x->dset_n || !x->dset ||
          !map_mvreg_ptrs_ok(&x->inner))
        return CRDT_EINVAL;
    if (!d_scratch || scratch_bytes < map_map_scratch_bytes(*out, n_obj, n_actors) || ((uintptr_t)d_scratch & 15u))
      return CRDT_EINVAL;
  }
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_map_map_merge(*self, *other, *out, n_obj, n_actors, (uint8_t*)d_scratch, ctx->d_status, ctx->d_ctl,
                              S(stream));
}

int crdt_map_orswot_merge(crdt_ctx* ctx, const crdt_map_orswot_slab* self, const crdt_map_orswot_slab* other,
                          const crdt_map_orswot_slab* out, size_t n_obj, uint32_t n_actors, void* stream) {
  if (!ctx || !self || !other || !out || n_actors == 0 || n_actors > 128) return CRDT_EINVAL;
  for (const crdt_map_orswot_slab* x : {self, other})
    if (x->kcap == 0 || x->kcap > 4096 || x->mcap == 0 || x->mcap > 256 || x->vdcap == 0 || x->vdcap > 256 ||
        x->vscap == 0 || x->vscap > 256 || x->dcap == 0 || x->dcap > 256 || x->scap == 0 || x->scap > 4096)
      return CRDT_EINVAL;
  if (out->kcap == 0 || out->mcap == 0 || out->vdcap == 0 || out->vscap == 0 || out->dcap == 0 || out->scap == 0)
    return CRDT_EINVAL;
  if (map_orswot_lds_bytes(*self, *other, n_actors) > 65536) return CRDT_EINVAL;  // the kernel's workspace
  if (n_obj)
    for (const crdt_map_orswot_slab* x : {self, other, out})
      if (!x->clock || !x->n_keys || !x->keys || !x->eclock || !x->vclock || !x->vn_mem || !x->vmem ||
          !x->vmclock || !x->vn_def || !x->vdclock || !x->vdset_n || !x->vdset || !x->n_def || !x->dclock ||
          !x->dset_n || !x->dset)
        return CRDT_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return launch_map_orswot_merge(*self, *other, *out, n_obj, n_actors, ctx->d_status, ctx->d_ctl, S(stream),
                                 ctx->variant);
}

}  // extern "C"
