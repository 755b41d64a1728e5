// Host side of crdts_hip: canonical record codec, the op path used to build
// states (Orswot::apply, src/orswot.rs:61-85, 195-211, 235-243), and the
// synthetic workload generators. No device work happens here.
//
// The host Orswot keeps the canonical form directly (sorted runs, sorted
// member map, deferred keyed in CLOCK ORDER), so encoding is a linear copy.
// Clocks built by the op path never hold a zero counter (`witness`,
// src/vclock.rs:159-163), so `a <= b` reduces to a pointwise test
// (src/vclock.rs:59-71 with canonical clocks).
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <thread>
#include <vector>

#include "../../include/crdts_hip.h"
#include "record_layout.h"

using namespace crdts_hip;

namespace {

struct Clk {
  std::vector<std::pair<uint32_t, uint64_t>> d;  // sorted by actor, counters > 0

  uint64_t get(uint32_t a) const {  // src/vclock.rs:206-210
    auto it = std::lower_bound(d.begin(), d.end(), std::make_pair(a, (uint64_t)0));
    return (it != d.end() && it->first == a) ? it->second : 0;
  }
  void witness(uint32_t a, uint64_t c) {  // src/vclock.rs:159-163
    auto it = std::lower_bound(d.begin(), d.end(), std::make_pair(a, (uint64_t)0));
    if (it != d.end() && it->first == a) {
      if (!(it->second >= c)) it->second = c;
    } else if (c > 0) {
      d.insert(it, {a, c});
    }
  }
  bool le(const Clk& o) const {  // canonical `<=`, src/vclock.rs:59-71
    for (auto& kv : d)
      if (kv.second > o.get(kv.first)) return false;
    return true;
  }
  void subtract(const Clk& o) {  // src/vclock.rs:236-242
    std::vector<std::pair<uint32_t, uint64_t>> r;
    r.reserve(d.size());
    for (auto& kv : d)
      if (!(o.get(kv.first) >= kv.second)) r.push_back(kv);
    d.swap(r);
  }
  bool operator==(const Clk& o) const { return d == o.d; }
  bool operator<(const Clk& o) const { return d < o.d; }  // CLOCK ORDER (lexicographic)
};

struct HOrswot {
  Clk clock;
  std::map<uint64_t, Clk> entries;
  std::map<Clk, std::vector<uint64_t>> deferred;  // member sets kept sorted

  void apply_add(uint32_t actor, uint64_t counter, uint64_t member) {  // src/orswot.rs:66-79
    if (clock.get(actor) >= counter) return;
    entries[member].witness(actor, counter);
    clock.witness(actor, counter);
    apply_deferred();
  }
  void apply_remove(uint64_t member, const Clk& rm) {  // src/orswot.rs:195-211
    if (!rm.le(clock)) {
      auto& s = deferred[rm];
      auto it = std::lower_bound(s.begin(), s.end(), member);
      if (it == s.end() || *it != member) s.insert(it, member);
    }
    auto it = entries.find(member);
    if (it != entries.end()) {
      it->second.subtract(rm);
      if (it->second.d.empty()) entries.erase(it);
    }
  }
  void apply_deferred() {  // src/orswot.rs:235-243
    if (deferred.empty()) return;
    std::map<Clk, std::vector<uint64_t>> d;
    d.swap(deferred);
    for (auto& kv : d)
      for (uint64_t m : kv.second) apply_remove(m, kv.first);
  }
};

// sparse: CSR top clock (flags bit 0): n_clk = nnz, ctr[] then act[] (crdts_hip.h).
long encode(const HOrswot& o, uint32_t n_actors, uint8_t* out, size_t cap, bool sparse = false) {
  uint32_t n_mem = (uint32_t)o.entries.size(), n_dot = 0, n_def = (uint32_t)o.deferred.size();
  uint32_t n_def_dot = 0, n_def_mem = 0;
  for (auto& kv : o.entries) {
    n_dot += (uint32_t)kv.second.d.size();
    for (auto& x : kv.second.d)
      if (x.first >= n_actors) return CRDT_EINVAL;
  }
  for (auto& kv : o.deferred) {
    n_def_dot += (uint32_t)kv.first.d.size();
    n_def_mem += (uint32_t)kv.second.size();
    for (auto& x : kv.first.d)
      if (x.first >= n_actors) return CRDT_EINVAL;
  }
  for (auto& x : o.clock.d)
    if (x.first >= n_actors) return CRDT_EINVAL;
  const uint32_t n_clk = sparse ? (uint32_t)o.clock.d.size() : n_actors;
  RecLayout L;
  rec_layout(L, n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse);
  if (L.size > cap) return CRDT_ECAPACITY;
  std::memset(out, 0, L.size);
  crdt_orswot_hdr h = {L.size, n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse ? kSparseClock : 0u};
  std::memcpy(out, &h, sizeof h);
  uint64_t* clk = (uint64_t*)(out + L.o_clk);
  uint64_t* key = (uint64_t*)(out + L.o_key);
  uint64_t* dctr = (uint64_t*)(out + L.o_dctr);
  uint32_t* dact = (uint32_t*)(out + L.o_dact);
  uint32_t* mdend = (uint32_t*)(out + L.o_mdend);
  uint64_t* fctr = (uint64_t*)(out + L.o_fctr);
  uint64_t* fkey = (uint64_t*)(out + L.o_fkey);
  uint32_t* fact = (uint32_t*)(out + L.o_fact);
  uint32_t* fdend = (uint32_t*)(out + L.o_fdend);
  uint32_t* fmend = (uint32_t*)(out + L.o_fmend);
  if (sparse) {
    uint32_t* cact = (uint32_t*)(out + L.o_cact);
    uint32_t k = 0;
    for (auto& x : o.clock.d) { clk[k] = x.second; cact[k] = x.first; ++k; }
  } else {
    for (auto& x : o.clock.d) clk[x.first] = x.second;
  }
  uint32_t m = 0, d = 0;
  for (auto& kv : o.entries) {
    key[m] = kv.first;
    for (auto& x : kv.second.d) { dact[d] = x.first; dctr[d] = x.second; ++d; }
    mdend[m++] = d;
  }
  uint32_t k = 0, fd = 0, fm = 0;
  for (auto& kv : o.deferred) {
    for (auto& x : kv.first.d) { fact[fd] = x.first; fctr[fd] = x.second; ++fd; }
    for (uint64_t mm : kv.second) fkey[fm++] = mm;
    fdend[k] = fd;
    fmend[k] = fm;
    ++k;
  }
  return (long)L.size;
}

bool decode(const uint8_t* rec, size_t avail, HOrswot& o) {
  if (avail < kHdrBytes) return false;
  crdt_orswot_hdr h;
  std::memcpy(&h, rec, sizeof h);
  if (h.flags & ~kSparseClock) return false;
  const bool sparse = (h.flags & kSparseClock) != 0;
  RecLayout L;
  rec_layout(L, h.n_clk, h.n_mem, h.n_dot, h.n_def, h.n_def_dot, h.n_def_mem, sparse);
  if (L.size != h.size || L.size > avail) return false;
  const uint64_t* clk = (const uint64_t*)(rec + L.o_clk);
  const uint64_t* key = (const uint64_t*)(rec + L.o_key);
  const uint64_t* dctr = (const uint64_t*)(rec + L.o_dctr);
  const uint32_t* dact = (const uint32_t*)(rec + L.o_dact);
  const uint32_t* mdend = (const uint32_t*)(rec + L.o_mdend);
  const uint64_t* fctr = (const uint64_t*)(rec + L.o_fctr);
  const uint64_t* fkey = (const uint64_t*)(rec + L.o_fkey);
  const uint32_t* fact = (const uint32_t*)(rec + L.o_fact);
  const uint32_t* fdend = (const uint32_t*)(rec + L.o_fdend);
  const uint32_t* fmend = (const uint32_t*)(rec + L.o_fmend);
  o = HOrswot();
  if (sparse) {
    const uint32_t* cact = (const uint32_t*)(rec + L.o_cact);
    for (uint32_t k = 0; k < h.n_clk; ++k) {
      if (k && cact[k] <= cact[k - 1]) return false;
      o.clock.d.push_back({cact[k], clk[k]});
    }
  } else {
    for (uint32_t a = 0; a < h.n_clk; ++a)
      if (clk[a]) o.clock.d.push_back({a, clk[a]});
  }
  uint32_t s = 0;
  for (uint32_t m = 0; m < h.n_mem; ++m) {
    if (mdend[m] < s || mdend[m] > h.n_dot) return false;
    Clk c;
    for (uint32_t d = s; d < mdend[m]; ++d) c.d.push_back({dact[d], dctr[d]});
    o.entries[key[m]] = std::move(c);
    s = mdend[m];
  }
  uint32_t fs = 0, ms = 0;
  for (uint32_t k = 0; k < h.n_def; ++k) {
    if (fdend[k] < fs || fdend[k] > h.n_def_dot || fmend[k] < ms || fmend[k] > h.n_def_mem)
      return false;
    Clk c;
    for (uint32_t d = fs; d < fdend[k]; ++d) c.d.push_back({fact[d], fctr[d]});
    o.deferred[c] = std::vector<uint64_t>(fkey + ms, fkey + fmend[k]);
    fs = fdend[k];
    ms = fmend[k];
  }
  return true;
}

// SplitMix64 (Steele, Lea, Flood 2014).
struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }
};

// One synthetic object pair by op simulation (documented in crdts_hip.h).
void gen_pair(uint64_t seed, uint64_t obj, const crdt_orswot_gen_params& P, HOrswot& L,
              HOrswot& R) {
  SplitMix64 rng(seed ^ obj);
  const uint32_t A = P.n_actors, U = P.member_universe;
  std::vector<uint64_t> keys(U);
  for (uint32_t j = 0; j < U; ++j) {
    uint64_t k;
    do {
      k = rng.next();
    } while (std::find(keys.begin(), keys.begin() + j, k) != keys.begin() + j);
    keys[j] = k;
  }
  std::vector<uint64_t> base(A);
  for (uint32_t a = 0; a < A; ++a) base[a] = rng.next() & ((1ull << 40) - 1);
  auto next_ctr = [&](const HOrswot& o, uint32_t a) {
    return std::max(o.clock.get(a), base[a]) + 1;  // derive_add_ctx, src/ctx.rs:599-607
  };
  // Ancestor: `ancestor_adds` adds of distinct members while the universe
  // lasts (a random permutation), by random actors.
  std::vector<uint32_t> perm(U);
  for (uint32_t j = 0; j < U; ++j) perm[j] = j;
  for (uint32_t j = U; j > 1; --j) std::swap(perm[j - 1], perm[rng.below(j)]);
  HOrswot anc;
  for (uint32_t k = 0; k < P.ancestor_adds; ++k) {
    uint32_t a = rng.below(A);
    uint32_t m = k < U ? perm[k] : rng.below(U);
    anc.apply_add(a, next_ctr(anc, a), keys[m]);
  }
  const bool shared = rng.below(100) < P.pct_shared_actor;
  const bool defobj = rng.below(100) < P.pct_deferred_obj;
  const uint32_t half = std::max(1u, A / 2);
  for (int side = 0; side < 2; ++side) {
    HOrswot& o = side == 0 ? L : R;
    o = anc;
    uint32_t span = P.max_div_ops >= P.min_div_ops ? P.max_div_ops - P.min_div_ops + 1 : 1;
    uint32_t nops = P.min_div_ops + rng.below(span);
    uint32_t own0 = side == 0 ? 0 : std::min(half, A - 1);
    uint32_t own_n = side == 0 ? half : std::max(1u, A - half);
    for (uint32_t k = 0; k < nops; ++k) {
      uint32_t r = rng.below(100);
      if (r < P.pct_add) {
        uint32_t a = own0 + rng.below(own_n);
        if (shared && side == 1 && rng.below(2) == 0) a = 0;
        o.apply_add(a, next_ctr(o, a), keys[rng.below(U)]);
      } else if (defobj && r >= 100 - P.pct_future_rm) {
        // remove with a future context: our clock advanced on a remote actor
        Clk c = o.clock;
        uint32_t other0 = side == 0 ? std::min(half, A - 1) : 0;
        uint32_t other_n = side == 0 ? std::max(1u, A - half) : half;
        uint32_t x = other0 + rng.below(other_n);
        c.witness(x, std::max(c.get(x), base[x]) + 1 + rng.below(3));
        o.apply_remove(keys[rng.below(U)], c);
      } else {
        // remove with a read context: contains(m).rm_clock (src/orswot.rs:214-224)
        if (o.entries.empty()) continue;
        auto it = o.entries.begin();
        std::advance(it, rng.below((uint32_t)o.entries.size()));
        Clk c = it->second;
        o.apply_remove(it->first, c);
      }
    }
  }
}

// One object's replicas for replica anti-entropy (config 5, crdts_hip.h):
// a shared ancestor over a per-object pool of actors drawn from a large
// universe, then each replica diverges with its own actors.
void gen_replicas(uint64_t seed, uint64_t obj, const crdt_orswot_rep_params& P, uint32_t n_rep,
                  std::vector<HOrswot>& reps) {
  SplitMix64 rng(seed ^ obj);
  const uint32_t U = P.member_universe;
  std::vector<uint64_t> keys(U);
  for (uint32_t j = 0; j < U; ++j) {
    uint64_t k;
    do {
      k = rng.next();
    } while (std::find(keys.begin(), keys.begin() + j, k) != keys.begin() + j);
    keys[j] = k;
  }
  auto draw_actors = [&](uint32_t n, std::vector<uint32_t>& out) {
    out.clear();
    while (out.size() < std::min(n, P.universe)) {
      uint32_t a = rng.below(P.universe);
      if (std::find(out.begin(), out.end(), a) == out.end()) out.push_back(a);
    }
  };
  std::vector<uint32_t> pool;
  draw_actors(P.pool_actors, pool);
  std::vector<std::vector<uint32_t>> own(n_rep);
  for (uint32_t r = 0; r < n_rep; ++r) draw_actors(P.own_actors, own[r]);
  std::map<uint32_t, uint64_t> base;  // per-actor 40-bit history base
  auto next_ctr = [&](const HOrswot& o, uint32_t a) {
    auto it = base.find(a);
    if (it == base.end()) it = base.emplace(a, rng.next() & ((1ull << 40) - 1)).first;
    return std::max(o.clock.get(a), it->second) + 1;  // derive_add_ctx, src/ctx.rs:599-607
  };
  std::vector<uint32_t> perm(U);
  for (uint32_t j = 0; j < U; ++j) perm[j] = j;
  for (uint32_t j = U; j > 1; --j) std::swap(perm[j - 1], perm[rng.below(j)]);
  HOrswot anc;
  for (uint32_t k = 0; k < P.ancestor_adds && !pool.empty(); ++k) {
    uint32_t a = pool[rng.below((uint32_t)pool.size())];
    uint32_t m = k < U ? perm[k] : rng.below(U);
    anc.apply_add(a, next_ctr(anc, a), keys[m]);
  }
  const bool defobj = rng.below(100) < P.pct_deferred_obj;
  reps.assign(n_rep, anc);
  for (uint32_t r = 0; r < n_rep; ++r) {
    HOrswot& o = reps[r];
    uint32_t span = P.max_div_ops >= P.min_div_ops ? P.max_div_ops - P.min_div_ops + 1 : 1;
    uint32_t nops = P.min_div_ops + rng.below(span);
    for (uint32_t k = 0; k < nops; ++k) {
      uint32_t q = rng.below(100);
      if (q < P.pct_add && !own[r].empty()) {
        uint32_t a = own[r][rng.below((uint32_t)own[r].size())];
        o.apply_add(a, next_ctr(o, a), keys[rng.below(U)]);
      } else if (defobj && q >= 100 - P.pct_future_rm && n_rep > 1) {
        // remove with a future context: advanced on another replica's actor
        uint32_t r2 = (r + 1 + rng.below(n_rep - 1)) % n_rep;
        if (own[r2].empty()) continue;
        Clk c = o.clock;
        uint32_t x = own[r2][rng.below((uint32_t)own[r2].size())];
        c.witness(x, next_ctr(o, x) + rng.below(3));
        o.apply_remove(keys[rng.below(U)], c);
      } else {
        if (o.entries.empty()) continue;
        auto it = o.entries.begin();
        std::advance(it, rng.below((uint32_t)o.entries.size()));
        Clk c = it->second;
        o.apply_remove(it->first, c);
      }
    }
  }
}

template <class F>
void parallel_for(size_t n, int threads, F f) {
  threads = std::max(1, threads);
  if (threads == 1 || n < 64) {
    f(0, n, 0);
    return;
  }
  std::vector<std::thread> ts;
  size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back(f, b, e, t);
  }
  for (auto& t : ts) t.join();
}

}  // namespace

struct crdt_orswot_gen {
  std::vector<std::vector<uint8_t>> base;  // one batch per side / replica
  std::vector<std::vector<uint64_t>> off;
};

namespace {
// Runs gen(i, states) for objects [0, n) on T threads and packs side
// keep_first + s of every object into batch s, s < n_sides (16-B aligned
// records, object order).
template <class G>
int pack_sides(size_t n_obj, uint32_t n_sides, int T, uint32_t n_actors, bool sparse, G gen,
               crdt_orswot_gen** out, uint32_t keep_first = 0) {
  T = std::max(1, T);
  std::vector<std::vector<std::vector<uint8_t>>> buf(n_sides, std::vector<std::vector<uint8_t>>(T));
  std::vector<std::vector<std::vector<uint64_t>>> loc(n_sides, std::vector<std::vector<uint64_t>>(T));
  std::vector<int> err(T, 0);
  parallel_for(n_obj, T, [&](size_t b, size_t e, int t) {
    std::vector<HOrswot> st;
    std::vector<uint8_t> tmp(1 << 16);
    for (size_t i = b; i < e; ++i) {
      gen(i, st);
      for (uint32_t s = 0; s < n_sides; ++s) {
        long n = encode(st[keep_first + s], n_actors, tmp.data(), tmp.size(), sparse);
        while (n == CRDT_ECAPACITY) {
          tmp.resize(tmp.size() * 2);
          n = encode(st[keep_first + s], n_actors, tmp.data(), tmp.size(), sparse);
        }
        if (n < 0) { err[t] = (int)n; return; }
        loc[s][t].push_back(buf[s][t].size());
        buf[s][t].insert(buf[s][t].end(), tmp.begin(), tmp.begin() + n);
      }
    }
  });
  for (int t = 0; t < T; ++t)
    if (err[t]) return err[t];
  auto* g = new crdt_orswot_gen();
  g->base.resize(n_sides);
  g->off.resize(n_sides);
  for (uint32_t s = 0; s < n_sides; ++s) {
    size_t total = 0;
    for (int t = 0; t < T; ++t) total += buf[s][t].size();
    g->base[s].resize(std::max<size_t>(total, 16));
    g->off[s].resize(n_obj);
    size_t pos = 0, k = 0;
    for (int t = 0; t < T; ++t) {
      std::memcpy(g->base[s].data() + pos, buf[s][t].data(), buf[s][t].size());
      for (uint64_t o : loc[s][t]) g->off[s][k++] = pos + o;
      pos += buf[s][t].size();
      std::vector<uint8_t>().swap(buf[s][t]);
    }
    g->base[s].resize(pos);
  }
  *out = g;
  return CRDT_OK;
}
}  // namespace

struct crdt_host_orswot {
  HOrswot o;
};

extern "C" {

size_t crdt_orswot_record_bytes(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot, uint32_t n_def,
                                uint32_t n_def_dot, uint32_t n_def_mem) {
  return (size_t)record_size64(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem);
}
size_t crdt_orswot_record_bytes_ex(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot, uint32_t n_def,
                                   uint32_t n_def_dot, uint32_t n_def_mem, uint32_t flags) {
  return (size_t)record_size64(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem,
                               (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0);
}

int crdt_orswot_generate(uint64_t seed, size_t first_obj, size_t n_obj,
                         const crdt_orswot_gen_params* params, int n_threads,
                         crdt_orswot_gen** out) {
  if (!params || !out || params->n_actors == 0 || params->member_universe == 0)
    return CRDT_EINVAL;
  const crdt_orswot_gen_params P = *params;
  return pack_sides(n_obj, 2, n_threads, P.n_actors, false,
                    [&](size_t i, std::vector<HOrswot>& st) {
                      st.resize(2);
                      gen_pair(seed, first_obj + i, P, st[0], st[1]);
                    },
                    out);
}

int crdt_orswot_generate_replicas(uint64_t seed, size_t first_obj, size_t n_obj,
                                  const crdt_orswot_rep_params* params, uint32_t n_replicas,
                                  uint32_t flags, int n_threads, crdt_orswot_gen** out) {
  if (!params || !out || params->universe == 0 || params->member_universe == 0 || n_replicas == 0 ||
      (flags & ~CRDT_ORSWOT_SPARSE_CLOCK))
    return CRDT_EINVAL;
  const crdt_orswot_rep_params P = *params;
  return pack_sides(n_obj, n_replicas, n_threads, P.universe, (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0,
                    [&](size_t i, std::vector<HOrswot>& st) { gen_replicas(seed, first_obj + i, P, n_replicas, st); },
                    out);
}

int crdt_orswot_generate_replicas_subset(uint64_t seed, size_t first_obj, size_t n_obj,
                                         const crdt_orswot_rep_params* params, uint32_t n_replicas,
                                         uint32_t keep_first, uint32_t keep_count, uint32_t flags, int n_threads,
                                         crdt_orswot_gen** out) {
  if (!params || !out || params->universe == 0 || params->member_universe == 0 || n_replicas == 0 ||
      keep_count == 0 || keep_first >= n_replicas || keep_count > n_replicas - keep_first ||
      (flags & ~CRDT_ORSWOT_SPARSE_CLOCK))
    return CRDT_EINVAL;
  const crdt_orswot_rep_params P = *params;
  return pack_sides(n_obj, keep_count, n_threads, P.universe, (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0,
                    [&](size_t i, std::vector<HOrswot>& st) { gen_replicas(seed, first_obj + i, P, n_replicas, st); },
                    out, keep_first);
}

int crdt_orswot_gen_side(const crdt_orswot_gen* g, int side, const uint8_t** h_base,
                         const uint64_t** h_off, size_t* bytes) {
  if (!g || side < 0 || (size_t)side >= g->base.size()) return CRDT_EINVAL;
  if (h_base) *h_base = g->base[side].data();
  if (h_off) *h_off = g->off[side].data();
  if (bytes) *bytes = g->base[side].size();
  return CRDT_OK;
}

void crdt_orswot_gen_free(crdt_orswot_gen* g) { delete g; }

int crdt_dense_generate(uint64_t seed, size_t first_obj, size_t n_obj, uint32_t n_actors,
                        uint32_t bits, uint32_t pct_zero, int n_threads, uint64_t* h_rows) {
  if (!h_rows || n_actors == 0 || bits == 0 || bits > 64) return CRDT_EINVAL;
  const uint64_t mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
  parallel_for(n_obj, n_threads, [&](size_t b, size_t e, int) {
    for (size_t i = b; i < e; ++i) {
      SplitMix64 rng(seed ^ (first_obj + i));
      uint64_t* row = h_rows + i * (size_t)n_actors;
      for (uint32_t a = 0; a < n_actors; ++a) {
        uint64_t v = rng.next();
        row[a] = (uint32_t)(v % 100) < pct_zero ? 0 : (rng.next() & mask);
      }
    }
  });
  return CRDT_OK;
}

crdt_host_orswot* crdt_host_orswot_new(void) { return new crdt_host_orswot(); }
crdt_host_orswot* crdt_host_orswot_clone(const crdt_host_orswot* o) {
  return o ? new crdt_host_orswot(*o) : nullptr;
}
void crdt_host_orswot_free(crdt_host_orswot* o) { delete o; }
int crdt_host_orswot_apply_add(crdt_host_orswot* o, uint32_t actor, uint64_t counter,
                               uint64_t member) {
  if (!o) return CRDT_EINVAL;
  o->o.apply_add(actor, counter, member);
  return CRDT_OK;
}
int crdt_host_orswot_apply_rm(crdt_host_orswot* o, uint64_t member, const uint32_t* actors,
                              const uint64_t* counters, uint32_t n) {
  if (!o || (n && (!actors || !counters))) return CRDT_EINVAL;
  Clk c;
  for (uint32_t i = 0; i < n; ++i) c.witness(actors[i], counters[i]);  // From<Vec<(A,u64)>>
  o->o.apply_remove(member, c);
  return CRDT_OK;
}
long crdt_host_orswot_encode(const crdt_host_orswot* o, uint32_t n_actors, uint8_t* h_rec,
                             size_t cap) {
  if (!o || !h_rec) return CRDT_EINVAL;
  return encode(o->o, n_actors, h_rec, cap);
}
long crdt_host_orswot_encode_ex(const crdt_host_orswot* o, uint32_t n_actors, uint32_t flags,
                                uint8_t* h_rec, size_t cap) {
  if (!o || !h_rec || (flags & ~CRDT_ORSWOT_SPARSE_CLOCK)) return CRDT_EINVAL;
  return encode(o->o, n_actors, h_rec, cap, (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0);
}
crdt_host_orswot* crdt_host_orswot_decode(const uint8_t* h_rec, size_t bytes) {
  if (!h_rec) return nullptr;
  auto* o = new crdt_host_orswot();
  if (!decode(h_rec, bytes, o->o)) {
    delete o;
    return nullptr;
  }
  return o;
}

}  // extern "C"
