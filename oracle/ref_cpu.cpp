// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the etsangsplk/rust-crdt (crate `crdts` 1.3.0) state-based
// join for VClock, GCounter, PNCounter and Orswot (incl. deferred removes).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library, and only as the checker / CPU baseline — the product
// path (rust-crdt_amd/) never links or calls it.
//
// It mirrors the reference's data structures so that it is also a fair CPU
// baseline ("kind": "port"):
//   BTreeMap<A,u64>            -> std::map<uint32_t,uint64_t>     (src/vclock.rs:54-57)
//   HashMap<M,VClock>          -> std::unordered_map<uint64_t,VClock> (src/orswot.rs:28)
//   HashMap<VClock,HashSet<M>> -> std::unordered_map<VClock,std::unordered_set<uint64_t>>
//                                                                 (src/orswot.rs:29)
// and the reference's clone pattern in Orswot::merge (src/orswot.rs:90-93).
//
// Parity pinning: the reference cannot be compiled in this image (no
// cargo/rustc), so this restatement is pinned by the reference's own
// known-answer tests and properties, transcribed into tests/golden/*.json and
// run by tests/test_oracle_kat.py, and cross-checked against a second,
// independent pure-Python restatement (oracle/crdts_ref.py).
//
// Canonical record encoding follows include/crdts_hip.h (the boundary spec);
// this file has its own encoder/decoder, independent of the product's.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../include/crdts_hip.h"

namespace oracle {

typedef uint32_t Actor;
typedef uint64_t Counter;  // src/vclock.rs:23
typedef uint64_t Member;

// ---------------------------------------------------------------- VClock
// src/vclock.rs:54-57
struct VClock {
  std::map<Actor, Counter> dots;

  bool operator==(const VClock& o) const { return dots == o.dots; }  // derive(PartialEq) :53

  // get — src/vclock.rs:206-210
  Counter get(Actor a) const {
    auto it = dots.find(a);
    return it == dots.end() ? 0 : it->second;
  }
  // witness — src/vclock.rs:159-163
  void witness(Actor a, Counter c) {
    if (!(get(a) >= c)) dots[a] = c;
  }
  // CvRDT::merge — src/vclock.rs:131-137
  void merge(const VClock& other) {
    for (const auto& kv : other.dots) witness(kv.first, kv.second);
  }
  // PartialOrd::partial_cmp — src/vclock.rs:59-71.
  // Returns 0 Equal, 1 Greater, -1 Less, 2 None.
  int partial_cmp(const VClock& other) const {
    if (*this == other) return 0;
    bool all = true;
    for (const auto& kv : other.dots)
      if (!(get(kv.first) >= kv.second)) { all = false; break; }
    if (all) return 1;
    all = true;
    for (const auto& kv : dots)
      if (!(other.get(kv.first) >= kv.second)) { all = false; break; }
    if (all) return -1;
    return 2;
  }
  // `a <= b` on PartialOrd: Some(Less) | Some(Equal)
  bool le(const VClock& other) const {
    int c = partial_cmp(other);
    return c == 0 || c == -1;
  }
  bool is_empty() const { return dots.empty(); }  // :213-215
  // intersection — src/vclock.rs:219-228
  VClock intersection(const VClock& other) const {
    VClock r;
    for (const auto& kv : dots)
      if (other.get(kv.first) == kv.second) r.dots.emplace(kv.first, kv.second);
    return r;
  }
  // subtract — src/vclock.rs:236-242
  void subtract(const VClock& other) {
    for (const auto& kv : other.dots)
      if (kv.second >= get(kv.first)) dots.erase(kv.first);
  }
  // inc — src/vclock.rs:182-185
  Counter inc(Actor a) const { return get(a) + 1; }
};

struct VClockHash {
  size_t operator()(const VClock& v) const {
    uint64_t h = 1469598103934665603ull;
    for (const auto& kv : v.dots) {
      h ^= kv.first; h *= 1099511628211ull;
      h ^= kv.second; h *= 1099511628211ull;
    }
    return (size_t)h;
  }
};

// ---------------------------------------------------------------- Orswot
// src/orswot.rs:26-30
struct Orswot {
  VClock clock;
  std::unordered_map<Member, VClock> entries;
  std::unordered_map<VClock, std::unordered_set<Member>, VClockHash> deferred;

  // CmRDT::apply, Op::Add — src/orswot.rs:66-79
  void apply_add(Actor actor, Counter counter, Member member) {
    if (clock.get(actor) >= counter) return;  // already seen
    entries[member].witness(actor, counter);  // entry().or_insert_with(VClock::new).apply(dot)
    clock.witness(actor, counter);
    apply_deferred();
  }
  // CmRDT::apply, Op::Rm — src/orswot.rs:80-82
  void apply_rm(Member member, const VClock& rm_clock) { apply_remove(member, rm_clock); }

  // apply_remove — src/orswot.rs:195-211
  void apply_remove(Member member, const VClock& rm_clock) {
    if (!rm_clock.le(clock)) {
      std::unordered_set<Member> drops;
      auto it = deferred.find(rm_clock);
      if (it != deferred.end()) { drops = std::move(it->second); deferred.erase(it); }
      drops.insert(member);
      deferred.emplace(rm_clock, std::move(drops));
    }
    auto it = entries.find(member);
    if (it != entries.end()) {
      VClock existing = std::move(it->second);
      entries.erase(it);
      existing.subtract(rm_clock);
      if (!existing.is_empty()) entries.emplace(member, std::move(existing));
    }
  }

  // apply_deferred — src/orswot.rs:235-243
  void apply_deferred() {
    auto d = deferred;  // clone
    deferred.clear();
    for (const auto& kv : d)
      for (Member m : kv.second) apply_remove(m, kv.first);
  }

  // CvRDT::merge — src/orswot.rs:87-157 (clone pattern of :90, :92, :93 kept)
  void merge(const Orswot& other) {
    auto other_remaining = other.entries;                 // :90
    std::unordered_map<Member, VClock> keep;              // :91
    auto self_entries = entries;                          // :92
    for (auto& kv : self_entries) {
      const Member entry = kv.first;
      VClock& eclock = kv.second;
      auto oit = other.entries.find(entry);
      if (oit == other.entries.end()) {                   // :94-104
        if (eclock.le(other.clock)) {
          // other has seen this entry and dropped it
        } else {
          keep.emplace(entry, eclock);
        }
      } else {                                            // :105-128
        VClock other_entry_clock = oit->second;           // .cloned() :93
        VClock common = eclock.intersection(other_entry_clock);  // :109
        eclock.subtract(common);                          // :110
        other_entry_clock.subtract(common);               // :111
        eclock.subtract(other.clock);                     // :112
        other_entry_clock.subtract(clock);                // :113 (pre-merge self.clock)
        common.merge(eclock);                             // :115
        common.merge(other_entry_clock);                  // :116
        if (!common.is_empty()) keep.emplace(entry, std::move(common));  // :120-125
        other_remaining.erase(entry);                     // :127
      }
    }
    for (auto& kv : other_remaining) {                    // :132-138
      VClock c = kv.second;
      c.subtract(clock);
      if (!c.is_empty()) keep.emplace(kv.first, std::move(c));
    }
    for (const auto& kv : other.deferred) {               // :141-148
      std::unordered_set<Member> ours;
      auto it = deferred.find(kv.first);
      if (it != deferred.end()) { ours = std::move(it->second); deferred.erase(it); }
      for (Member e : kv.second) ours.insert(e);
      deferred.emplace(kv.first, std::move(ours));
    }
    entries = std::move(keep);                            // :150
    clock.merge(other.clock);                             // :153
    apply_deferred();                                     // :155
  }

  // Causal::truncate — src/orswot.rs:159-172: merge with an empty set whose
  // clock is `c`, then forget `c` from the top clock and every member clock
  // (kept as is even if that empties one).
  void truncate(const VClock& c) {
    Orswot empty_set;
    empty_set.clock = c;
    merge(empty_set);
    clock.subtract(c);
    for (auto& kv : entries) kv.second.subtract(c);
  }
};

// GCounter — src/gcounter.rs:26-28; merge :58-62
struct GCounter {
  VClock inner;
  void merge(const GCounter& o) { inner.merge(o.inner); }
  uint64_t value() const {  // :76-78 (wrapping like release-mode Rust u64 add)
    uint64_t s = 0;
    for (const auto& kv : inner.dots) s += kv.second;
    return s;
  }
};
// PNCounter — src/pncounter.rs:33-36; merge :90-95
struct PNCounter {
  GCounter p, n;
  void merge(const PNCounter& o) { p.merge(o.p); n.merge(o.n); }
  int64_t value() const { return (int64_t)p.value() - (int64_t)n.value(); }  // :117-119
};

// ------------------------------------------------- canonical record codec
static inline size_t pad16(size_t x) { return (x + 15) & ~size_t(15); }

// sparse: CSR top clock (header flags bit 0): u64 ctr[n_clk], u32 act[n_clk], pad 8.
size_t record_bytes(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot, uint32_t n_def,
                    uint32_t n_def_dot, uint32_t n_def_mem, bool sparse = false) {
  size_t b = CRDT_ORSWOT_HDR_BYTES + (sparse ? ((12ull * n_clk + 7) & ~size_t(7)) : 8ull * n_clk);
  b += 12ull * ((size_t)n_mem + n_dot);                 // member block
  b = (b + 7) & ~size_t(7);
  b += 12ull * n_def_dot + 8ull * n_def_mem + 8ull * n_def;  // deferred block
  return pad16(b);
}

// Section pointers of a record (layout: include/crdts_hip.h).
struct Sections {
  uint64_t *clk, *key, *dctr, *fctr, *fkey;
  uint32_t *cact, *dact, *mdend, *fact, *fdend, *fmend;
};
static Sections sections(uint8_t* rec, const crdt_orswot_hdr& h) {
  Sections s;
  const bool sparse = (h.flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0;
  s.clk = (uint64_t*)(rec + CRDT_ORSWOT_HDR_BYTES);
  s.cact = (uint32_t*)(s.clk + h.n_clk);
  s.key = sparse ? (uint64_t*)(rec + CRDT_ORSWOT_HDR_BYTES + ((12ull * h.n_clk + 7) & ~size_t(7)))
                 : s.clk + h.n_clk;
  s.dctr = s.key + h.n_mem;
  s.dact = (uint32_t*)(s.dctr + h.n_dot);
  s.mdend = s.dact + h.n_dot;
  size_t mb = (size_t)((uint8_t*)(s.mdend + h.n_mem) - rec);
  mb = (mb + 7) & ~size_t(7);
  s.fctr = (uint64_t*)(rec + mb);
  s.fkey = s.fctr + h.n_def_dot;
  s.fact = (uint32_t*)(s.fkey + h.n_def_mem);
  s.fdend = s.fact + h.n_def_dot;
  s.fmend = s.fdend + h.n_def;
  return s;
}

static bool clock_less(const VClock& a, const VClock& b) {
  // CLOCK ORDER: lexicographic over the (actor, counter) sequence, prefix first.
  auto ia = a.dots.begin(), ib = b.dots.begin();
  for (; ia != a.dots.end() && ib != b.dots.end(); ++ia, ++ib) {
    if (ia->first != ib->first) return ia->first < ib->first;
    if (ia->second != ib->second) return ia->second < ib->second;
  }
  return ia == a.dots.end() && ib != b.dots.end();
}

// Encode; returns bytes or negative code. Dense clock of n_actors slots, or
// (sparse) the clock's nnz actors as CSR.
long encode(const Orswot& o, uint32_t n_actors, uint8_t* out, size_t cap, bool sparse = false) {
  std::vector<std::pair<Member, const VClock*>> ents;
  for (const auto& kv : o.entries) ents.emplace_back(kv.first, &kv.second);
  std::sort(ents.begin(), ents.end(),
            [](const auto& x, const auto& y) { return x.first < y.first; });
  std::vector<std::pair<const VClock*, std::vector<Member>>> defs;
  for (const auto& kv : o.deferred) {
    std::vector<Member> ms(kv.second.begin(), kv.second.end());
    std::sort(ms.begin(), ms.end());
    defs.emplace_back(&kv.first, std::move(ms));
  }
  std::sort(defs.begin(), defs.end(),
            [](const auto& x, const auto& y) { return clock_less(*x.first, *y.first); });
  uint32_t n_mem = (uint32_t)ents.size(), n_dot = 0, n_def = (uint32_t)defs.size(),
           n_def_dot = 0, n_def_mem = 0;
  for (auto& e : ents) n_dot += (uint32_t)e.second->dots.size();
  for (auto& d : defs) {
    n_def_dot += (uint32_t)d.first->dots.size();
    n_def_mem += (uint32_t)d.second.size();
  }
  // Dense top clock: every interned actor id (top clock, member clocks,
  // deferred clocks) must be < n_actors.
  for (auto& kv : o.clock.dots)
    if (kv.first >= n_actors) return CRDT_EINVAL;
  for (auto& e : ents)
    for (auto& kv : e.second->dots)
      if (kv.first >= n_actors) return CRDT_EINVAL;
  for (auto& d : defs)
    for (auto& kv : d.first->dots)
      if (kv.first >= n_actors) return CRDT_EINVAL;
  const uint32_t n_clk = sparse ? (uint32_t)o.clock.dots.size() : n_actors;
  size_t bytes = record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse);
  if (bytes > cap) return CRDT_ECAPACITY;
  std::memset(out, 0, bytes);
  // an empty member clock (Causal::truncate can leave one, src/orswot.rs:167-169)
  // is an empty run, flagged in the header
  bool empty_clock = false;
  for (auto& e : ents) empty_clock = empty_clock || e.second->dots.empty();
  crdt_orswot_hdr h = {(uint32_t)bytes, n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem,
                       (sparse ? CRDT_ORSWOT_SPARSE_CLOCK : 0u) |
                           (empty_clock ? CRDT_ORSWOT_EMPTY_MEMBER_CLOCK : 0u)};
  std::memcpy(out, &h, sizeof h);
  Sections S = sections(out, h);
  uint64_t *clk = S.clk, *key = S.key, *dctr = S.dctr, *fctr = S.fctr, *fkey = S.fkey;
  uint32_t *dact = S.dact, *mdend = S.mdend, *fact = S.fact, *fdend = S.fdend, *fmend = S.fmend;
  if (sparse) {
    uint32_t k = 0;
    for (auto& kv : o.clock.dots) { clk[k] = kv.second; S.cact[k] = kv.first; ++k; }  // BTreeMap order
  } else {
    for (auto& kv : o.clock.dots) clk[kv.first] = kv.second;
  }
  uint32_t d = 0;
  for (uint32_t m = 0; m < n_mem; ++m) {
    key[m] = ents[m].first;
    for (auto& kv : ents[m].second->dots) { dact[d] = kv.first; dctr[d] = kv.second; ++d; }
    mdend[m] = d;
  }
  uint32_t fd = 0, fm = 0;
  for (uint32_t k = 0; k < n_def; ++k) {
    for (auto& kv : defs[k].first->dots) { fact[fd] = kv.first; fctr[fd] = kv.second; ++fd; }
    for (Member mm : defs[k].second) fkey[fm++] = mm;
    fdend[k] = fd;
    fmend[k] = fm;
  }
  return (long)bytes;
}

bool decode(const uint8_t* rec, size_t avail, Orswot& o) {
  if (avail < CRDT_ORSWOT_HDR_BYTES) return false;
  crdt_orswot_hdr h;
  std::memcpy(&h, rec, sizeof h);
  const bool sparse = (h.flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0;
  if (h.flags & ~(CRDT_ORSWOT_SPARSE_CLOCK | CRDT_ORSWOT_EMPTY_MEMBER_CLOCK)) return false;
  size_t bytes = record_bytes(h.n_clk, h.n_mem, h.n_dot, h.n_def, h.n_def_dot, h.n_def_mem, sparse);
  if (bytes != h.size || bytes > avail) return false;
  Sections S = sections(const_cast<uint8_t*>(rec), h);
  const uint64_t *clk = S.clk, *key = S.key, *dctr = S.dctr, *fctr = S.fctr, *fkey = S.fkey;
  const uint32_t *dact = S.dact, *mdend = S.mdend, *fact = S.fact, *fdend = S.fdend,
                 *fmend = S.fmend;
  o = Orswot();
  if (sparse) {
    for (uint32_t k = 0; k < h.n_clk; ++k) o.clock.dots[S.cact[k]] = clk[k];
  } else {
    for (uint32_t a = 0; a < h.n_clk; ++a)
      if (clk[a]) o.clock.dots.emplace(a, clk[a]);
  }
  uint32_t d0 = 0;
  for (uint32_t m = 0; m < h.n_mem; ++m) {
    if (mdend[m] < d0 || mdend[m] > h.n_dot) return false;
    VClock c;
    for (uint32_t d = d0; d < mdend[m]; ++d) c.dots[dact[d]] = dctr[d];
    o.entries[key[m]] = std::move(c);
    d0 = mdend[m];
  }
  uint32_t f0 = 0, k0 = 0;
  for (uint32_t k = 0; k < h.n_def; ++k) {
    if (fdend[k] < f0 || fdend[k] > h.n_def_dot || fmend[k] < k0 || fmend[k] > h.n_def_mem)
      return false;
    VClock c;
    for (uint32_t d = f0; d < fdend[k]; ++d) c.dots[fact[d]] = fctr[d];
    auto& s = o.deferred[c];
    for (uint32_t j = k0; j < fmend[k]; ++j) s.insert(fkey[j]);
    f0 = fdend[k];
    k0 = fmend[k];
  }
  return true;
}

template <class F>
static void parallel_for(size_t n, int threads, F f) {
  if (threads <= 1 || n < 2) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back(f, b, e);
  }
  for (auto& t : ts) t.join();
}

static VClock row_to_vclock(const uint64_t* row, uint32_t n) {
  VClock v;
  for (uint32_t a = 0; a < n; ++a)
    if (row[a]) v.dots.emplace(a, row[a]);
  return v;
}
static void vclock_to_row(const VClock& v, uint64_t* row, uint32_t n) {
  std::memset(row, 0, 8ull * n);
  for (auto& kv : v.dots) row[kv.first] = kv.second;
}

}  // namespace oracle

using namespace oracle;

// ---------------------------------------------------------------- binary form
// to_binary / from_binary (src/lib.rs:62-83) = bincode 0.9 of the serde
// derives on Orswot (src/orswot.rs:26-30) / VClock (src/vclock.rs:54-57),
// restated (bincode is not vendored): u64 LE lengths before maps and sets,
// fixed-width LE integers, fields in declaration order. Decoding fills the
// reference-shaped containers (std::map / unordered_map / unordered_set),
// i.e. it pays what `from_binary` pays; encoding walks them in their own
// (hash) order as `to_binary` does.
namespace oracle {
struct BinReader {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  uint64_t get(int w) {
    if (pos + (size_t)w > n) { ok = false; return 0; }
    uint64_t v = 0;
    for (int i = 0; i < w; ++i) v |= (uint64_t)p[pos + i] << (8 * i);
    pos += w;
    return v;
  }
};

static bool bin_vclock(BinReader& r, int wa, VClock& v) {
  const uint64_t n = r.get(8);
  if (!r.ok || n > r.n) return false;
  bool first = true;
  Actor last = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = r.get(wa), c = r.get(8);
    if (!r.ok || a > 0xFFFFFFFFull || (!first && a <= last)) return false;  // BTreeMap: ascending keys
    v.dots.emplace_hint(v.dots.end(), (Actor)a, c);
    last = (Actor)a;
    first = false;
  }
  return true;
}

bool from_binary(const uint8_t* p, size_t n, int wa, int wm, Orswot& o) {
  BinReader r{p, n};
  if (!bin_vclock(r, wa, o.clock)) return false;
  const uint64_t ne = r.get(8);
  if (!r.ok || ne > n) return false;
  for (uint64_t i = 0; i < ne; ++i) {
    const Member m = r.get(wm);
    VClock v;
    if (!r.ok || !bin_vclock(r, wa, v)) return false;
    if (!o.entries.emplace(m, std::move(v)).second) return false;  // duplicate HashMap key
  }
  const uint64_t nd = r.get(8);
  if (!r.ok || nd > n) return false;
  for (uint64_t i = 0; i < nd; ++i) {
    VClock v;
    if (!bin_vclock(r, wa, v)) return false;
    const uint64_t ns = r.get(8);
    if (!r.ok || ns > n) return false;
    std::unordered_set<Member> s;
    for (uint64_t j = 0; j < ns; ++j) {
      const Member m = r.get(wm);
      if (!r.ok || !s.insert(m).second) return false;
    }
    if (!o.deferred.emplace(std::move(v), std::move(s)).second) return false;
  }
  return r.ok && r.pos == n;
}

static void put(std::vector<uint8_t>& out, uint64_t v, int w) {
  for (int i = 0; i < w; ++i) out.push_back((uint8_t)(v >> (8 * i)));
}
static void bin_put_vclock(std::vector<uint8_t>& out, const VClock& v, int wa) {
  put(out, v.dots.size(), 8);
  for (const auto& kv : v.dots) { put(out, kv.first, wa); put(out, kv.second, 8); }
}
void to_binary(const Orswot& o, int wa, int wm, std::vector<uint8_t>& out) {
  bin_put_vclock(out, o.clock, wa);
  put(out, o.entries.size(), 8);
  for (const auto& kv : o.entries) { put(out, kv.first, wm); bin_put_vclock(out, kv.second, wa); }
  put(out, o.deferred.size(), 8);
  for (const auto& kv : o.deferred) {
    bin_put_vclock(out, kv.first, wa);
    put(out, kv.second.size(), 8);
    for (Member m : kv.second) put(out, m, wm);
  }
}
}  // namespace oracle

namespace oracle {
// ---------------------------------------------------------------- MVReg / Map
// MVReg<u64, A> (src/mvreg.rs:14-18): merge :121-153, truncate :71-83,
// apply(Put) :158-185.
struct MVRegO {
  std::vector<std::pair<VClock, uint64_t>> vals;
  void merge(const MVRegO& other) {
    std::vector<std::pair<VClock, uint64_t>> out;
    for (const auto& sv : vals) {
      bool dom = false;
      for (const auto& ov : other.vals) dom = dom || sv.first.partial_cmp(ov.first) == -1;
      if (!dom) out.push_back(sv);
    }
    for (const auto& ov : other.vals) {
      bool dom = false;
      for (const auto& sv : vals) dom = dom || ov.first.partial_cmp(sv.first) == -1;
      if (dom) continue;
      bool is_new = true;
      for (const auto& e : out)
        if (e.first == ov.first) { is_new = false; break; }
      if (is_new) out.push_back(ov);
    }
    vals.swap(out);
  }
  void truncate(const VClock& c) {
    std::vector<std::pair<VClock, uint64_t>> out;
    for (auto v : vals) {
      v.first.subtract(c);
      if (!v.first.is_empty()) out.push_back(v);
    }
    vals.swap(out);
  }
  void apply_put(const VClock& clock, uint64_t val) {
    if (clock.is_empty()) return;
    std::vector<std::pair<VClock, uint64_t>> out;
    for (const auto& v : vals)
      if (!v.first.le(clock)) out.push_back(v);
    vals.swap(out);
    bool add = true;
    for (const auto& v : vals)
      if (v.first.partial_cmp(clock) == 1) add = false;  // existing_clock > clock
    if (add) vals.emplace_back(clock, val);
  }
};

// Map<u64, V, A> (src/map.rs:82-98) over a value V with merge and
// Causal::truncate: merge :191-268, apply :162-188, apply_rm :336-349,
// apply_deferred :323-333, truncate :131-158. std::map<VClock, ...> orders
// deferred clocks lexicographically over (actor, counter): CLOCK ORDER.
// MapO = Map<u64, MVReg>; MapMapO = Map<u64, Map<u64, MVReg>> (the reference's
// TestMap, test/map.rs:4-8).
template <class V>
struct MapEntryT {
  VClock clock;
  V val;
};
template <class V>
struct MapT {
  VClock clock;
  std::map<uint64_t, MapEntryT<V>> entries;
  std::map<std::map<Actor, Counter>, std::set<uint64_t>> deferred;

  void apply_rm(uint64_t key, const VClock& c) {
    if (!c.le(clock)) deferred[c.dots].insert(key);
    auto it = entries.find(key);
    if (it != entries.end()) {
      MapEntryT<V> e = it->second;
      entries.erase(it);
      e.clock.subtract(c);
      if (!e.clock.is_empty()) {
        e.val.truncate(c);
        entries[key] = e;
      }
    }
  }
  void apply_deferred() {
    auto d = deferred;
    deferred.clear();
    for (const auto& kv : d) {
      VClock c;
      c.dots = kv.first;
      for (uint64_t k : kv.second) apply_rm(k, c);
    }
  }
  void apply_up(Actor a, Counter ctr, uint64_t key, const VClock& put_clock, uint64_t val) {  // (V = MVRegO)
    if (clock.get(a) >= ctr) return;
    MapEntryT<V> e;
    auto it = entries.find(key);
    if (it != entries.end()) { e = it->second; entries.erase(it); }
    e.clock.witness(a, ctr);
    e.val.apply_put(put_clock, val);
    entries[key] = e;
    clock.witness(a, ctr);
    apply_deferred();
  }
  // Causal::truncate (:131-158): entry clocks lose `c` (emptied entries
  // dropped, the rest truncate their value), deferred clocks lose it
  // (emptied ones dropped; two that become equal: the later in CLOCK ORDER
  // replaces the earlier, as the reference's HashMap insert), clock loses it
  void truncate(const VClock& c) {
    for (auto it = entries.begin(); it != entries.end();) {
      it->second.clock.subtract(c);
      if (it->second.clock.is_empty()) {
        it = entries.erase(it);
      } else {
        it->second.val.truncate(c);
        ++it;
      }
    }
    std::map<std::map<Actor, Counter>, std::set<uint64_t>> d;
    for (const auto& kv : deferred) {
      VClock rc;
      rc.dots = kv.first;
      rc.subtract(c);
      if (!rc.is_empty()) d[rc.dots] = kv.second;
    }
    deferred.swap(d);
    clock.subtract(c);
  }
  void merge(const MapT& other) {
    std::map<uint64_t, MapEntryT<V>> keep;
    for (const auto& kv : entries) {
      MapEntryT<V> entry = kv.second;
      auto oit = other.entries.find(kv.first);
      if (oit == other.entries.end()) {
        entry.clock.subtract(other.clock);
        if (!entry.clock.is_empty()) {
          VClock del = other.clock;
          del.subtract(entry.clock);
          entry.val.truncate(del);
          keep[kv.first] = entry;
        }
      } else {
        MapEntryT<V> oe = oit->second;
        VClock common = entry.clock.intersection(oe.clock);
        entry.clock.subtract(common);
        oe.clock.subtract(common);
        entry.clock.subtract(other.clock);
        oe.clock.subtract(clock);
        common.merge(entry.clock);
        common.merge(oe.clock);
        if (!common.is_empty()) {
          entry.val.merge(oe.val);
          VClock del = entry.clock;
          del.merge(oe.clock);
          del.subtract(common);
          entry.val.truncate(del);
          entry.clock = common;
          keep[kv.first] = entry;
        }
      }
    }
    for (const auto& kv : other.entries) {
      if (entries.count(kv.first)) continue;
      MapEntryT<V> entry = kv.second;
      entry.clock.subtract(clock);
      if (!entry.clock.is_empty()) {
        VClock del = clock;
        del.subtract(entry.clock);
        entry.val.truncate(del);
        keep[kv.first] = entry;
      }
    }
    for (const auto& kv : other.deferred) {  // apply_rm on the old entries: only the deferral survives
      VClock c;
      c.dots = kv.first;
      for (uint64_t k : kv.second) apply_rm(k, c);
    }
    entries = keep;
    clock.merge(other.clock);
    apply_deferred();
  }
};
using MapEntry = MapEntryT<MVRegO>;
using MapO = MapT<MVRegO>;
using MapMapO = MapT<MapO>;
}  // namespace oracle

extern "C" {

size_t orc_record_bytes(uint32_t n_clk, uint32_t n_mem, uint32_t n_dot, uint32_t n_def,
                        uint32_t n_def_dot, uint32_t n_def_mem) {
  return record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem);
}

// Merge a batch of record pairs; output compacted (out_off computed here).
// Returns 0, or a negative code (first failing object index in *bad).
int orc_orswot_merge_batch_ex(const uint8_t* lb, const uint64_t* loff, size_t lbytes,
                              const uint8_t* rb, const uint64_t* roff, size_t rbytes, size_t n,
                              uint32_t n_actors, uint32_t flags, uint8_t* ob, uint64_t* ooff, size_t ocap,
                              int threads, int64_t* bad) {
  const bool sparse = (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0;
  std::vector<std::vector<uint8_t>> outs(n);
  std::vector<int> err(n, 0);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      Orswot L, R;
      if (!decode(lb + loff[i], lbytes - loff[i], L) || !decode(rb + roff[i], rbytes - roff[i], R)) {
        err[i] = CRDT_ENONCANON;
        continue;
      }
      L.merge(R);
      std::vector<uint8_t> buf(record_bytes(n_actors, L.entries.size(), 0, 0, 0, 0) + 65536);
      long got;
      while ((got = encode(L, n_actors, buf.data(), buf.size(), sparse)) == CRDT_ECAPACITY)
        buf.resize(buf.size() * 2);
      if (got < 0) { err[i] = (int)got; continue; }
      buf.resize(got);
      outs[i] = std::move(buf);
    }
  });
  size_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    if (err[i]) { if (bad) *bad = (int64_t)i; return err[i]; }
    if (pos + outs[i].size() > ocap) { if (bad) *bad = (int64_t)i; return CRDT_ECAPACITY; }
    std::memcpy(ob + pos, outs[i].data(), outs[i].size());
    ooff[i] = pos;
    pos += outs[i].size();
  }
  return 0;
}

// Causal::truncate (src/orswot.rs:159-172) of every record by its clock, the
// clock i being the sorted run [coff[i], coff[i] + clen[i]) of (cact, cctr);
// outputs packed into ob / ooff like orc_orswot_merge_batch_ex.
int orc_orswot_truncate_batch(const uint8_t* lb, const uint64_t* loff, size_t lbytes, size_t n,
                              const uint64_t* coff, const uint32_t* clen, const uint32_t* cact,
                              const uint64_t* cctr, uint32_t n_actors, uint32_t flags, uint8_t* ob,
                              uint64_t* ooff, size_t ocap, int threads, int64_t* bad) {
  const bool sparse = (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0;
  std::vector<std::vector<uint8_t>> outs(n);
  std::vector<int> err(n, 0);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      Orswot L;
      if (!decode(lb + loff[i], lbytes - loff[i], L)) {
        err[i] = CRDT_ENONCANON;
        continue;
      }
      VClock c;
      for (uint32_t k = 0; k < clen[i]; ++k) c.witness(cact[coff[i] + k], cctr[coff[i] + k]);
      L.truncate(c);
      std::vector<uint8_t> buf(record_bytes(n_actors, L.entries.size(), 0, 0, 0, 0) + 65536);
      long got;
      while ((got = encode(L, n_actors, buf.data(), buf.size(), sparse)) == CRDT_ECAPACITY)
        buf.resize(buf.size() * 2);
      if (got < 0) { err[i] = (int)got; continue; }
      buf.resize(got);
      outs[i] = std::move(buf);
    }
  });
  size_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    if (err[i]) { if (bad) *bad = (int64_t)i; return err[i]; }
    if (pos + outs[i].size() > ocap) { if (bad) *bad = (int64_t)i; return CRDT_ECAPACITY; }
    std::memcpy(ob + pos, outs[i].data(), outs[i].size());
    ooff[i] = pos;
    pos += outs[i].size();
  }
  return 0;
}

int orc_orswot_merge_batch(const uint8_t* lb, const uint64_t* loff, size_t lbytes,
                           const uint8_t* rb, const uint64_t* roff, size_t rbytes, size_t n,
                           uint32_t n_actors, uint8_t* ob, uint64_t* ooff, size_t ocap,
                           int threads, int64_t* bad) {
  return orc_orswot_merge_batch_ex(lb, loff, lbytes, rb, roff, rbytes, n, n_actors, 0u, ob, ooff, ocap,
                                   threads, bad);
}

// CPU baseline: decode untimed, time only L[i].merge(&R[i]) for i in [0, n)
// over `threads` std::threads (static partition, standing in for rayon
// par_iter over objects). Returns seconds of the merge loop.
double orc_orswot_bench(const uint8_t* lb, const uint64_t* loff, size_t lbytes,
                        const uint8_t* rb, const uint64_t* roff, size_t rbytes, size_t n,
                        int threads) {
  std::vector<Orswot> L(n), R(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      decode(lb + loff[i], lbytes - loff[i], L[i]);
      decode(rb + roff[i], rbytes - roff[i], R[i]);
    }
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) L[i].merge(R[i]);
  });
  auto t1 = std::chrono::steady_clock::now();
  // keep results alive so the loop is not elided
  volatile size_t sink = 0;
  for (size_t i = 0; i < n; i += 997) sink += L[i].entries.size();
  (void)sink;
  std::vector<Orswot>().swap(L);
  return std::chrono::duration<double>(t1 - t0).count();
}


// Blob -> canonical record (0 ok / -2 not decodable or not canonical / -4 cap).
long orc_bincode_to_record(const uint8_t* blob, size_t n, int wa, int wm, uint32_t n_actors, uint32_t flags,
                           uint8_t* out, size_t cap) {
  Orswot o;
  if (!from_binary(blob, n, wa, wm, o)) return -2;
  for (const auto& kv : o.clock.dots) if (kv.first >= n_actors || kv.second == 0) return -2;
  return encode(o, n_actors, out, cap, (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0);
}

// CPU baseline of ingest: from_binary + canonical encode of n blobs over
// `threads` std::threads; returns seconds (records written to thread-local
// scratch, not kept).
double orc_bincode_ingest_bench(const uint8_t* blobs, const uint64_t* off, const uint64_t* len, size_t n, int wa,
                                int wm, uint32_t n_actors, uint32_t flags, int threads, int64_t* bad) {
  std::atomic<int64_t> nbad{0};
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    std::vector<uint8_t> rec(1 << 16);
    for (size_t i = b; i < e; ++i) {
      Orswot o;
      if (!from_binary(blobs + off[i], len[i], wa, wm, o) ||
          encode(o, n_actors, rec.data(), rec.size(), (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0) < 0)
        nbad++;
    }
  });
  auto t1 = std::chrono::steady_clock::now();
  if (bad) *bad = nbad.load();
  return std::chrono::duration<double>(t1 - t0).count();
}

// CPU baseline of egest: decode records untimed, time to_binary of each.
double orc_bincode_egest_bench(const uint8_t* rb, const uint64_t* roff, size_t rbytes, size_t n, int wa, int wm,
                               int threads) {
  std::vector<Orswot> objs(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) decode(rb + roff[i], rbytes - roff[i], objs[i]);
  });
  std::atomic<size_t> total{0};
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    std::vector<uint8_t> out;
    size_t t = 0;
    for (size_t i = b; i < e; ++i) {
      out.clear();
      to_binary(objs[i], wa, wm, out);
      t += out.size();
    }
    total += t;
  });
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// CPU baseline of the batched op path: decode untimed, then time applying
// every object's ops in order (CmRDT::apply, src/orswot.rs:61-85) over
// `threads` std::threads. Returns seconds.
double orc_orswot_apply_bench(const uint8_t* rb, const uint64_t* roff, size_t rbytes, size_t n,
                              const uint64_t* obj_end, const uint32_t* kind, const uint64_t* member,
                              const uint32_t* actor, const uint64_t* counter, const uint64_t* clk_end,
                              const uint32_t* clk_act, const uint64_t* clk_ctr, int threads) {
  std::vector<Orswot> objs(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) decode(rb + roff[i], rbytes - roff[i], objs[i]);
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      for (uint64_t q = i ? obj_end[i - 1] : 0; q < obj_end[i]; ++q) {
        if (kind[q] == 0) {
          objs[i].apply_add(actor[q], counter[q], member[q]);
        } else {
          VClock c;
          for (uint64_t k = q ? clk_end[q - 1] : 0; k < clk_end[q]; ++k) c.dots.emplace(clk_act[k], clk_ctr[k]);
          objs[i].apply_rm(member[q], c);
        }
      }
    }
  });
  auto t1 = std::chrono::steady_clock::now();
  volatile size_t sink = 0;
  for (size_t i = 0; i < n; i += 997) sink += objs[i].entries.size();
  (void)sink;
  return std::chrono::duration<double>(t1 - t0).count();
}

// CPU baseline of the batched truncate: records and clocks decoded untimed,
// then Orswot::truncate (src/orswot.rs:159-172) timed. Returns seconds.
double orc_orswot_truncate_bench(const uint8_t* rb, const uint64_t* roff, size_t rbytes, size_t n,
                                 const uint64_t* coff, const uint32_t* clen, const uint32_t* cact,
                                 const uint64_t* cctr, int threads) {
  std::vector<Orswot> objs(n);
  std::vector<VClock> clocks(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      decode(rb + roff[i], rbytes - roff[i], objs[i]);
      for (uint32_t k = 0; k < clen[i]; ++k) clocks[i].witness(cact[coff[i] + k], cctr[coff[i] + k]);
    }
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) objs[i].truncate(clocks[i]);
  });
  auto t1 = std::chrono::steady_clock::now();
  volatile size_t sink = 0;
  for (size_t i = 0; i < n; i += 997) sink += objs[i].entries.size();
  (void)sink;
  return std::chrono::duration<double>(t1 - t0).count();
}

// Dense VClock/GCounter rows, through the BTreeMap-style VClock::merge.
int orc_dense_merge(uint64_t* self, const uint64_t* other, size_t n, uint32_t n_actors,
                    int threads) {
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      VClock a = row_to_vclock(self + i * n_actors, n_actors);
      VClock o = row_to_vclock(other + i * n_actors, n_actors);
      a.merge(o);
      vclock_to_row(a, self + i * n_actors, n_actors);
    }
  });
  return 0;
}
// PNCounter rows [P|N], 2*n_actors slots; via PNCounter::merge.
int orc_pncounter_merge(uint64_t* self, const uint64_t* other, size_t n, uint32_t n_actors,
                        int threads) {
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      uint64_t* s = self + i * 2ull * n_actors;
      const uint64_t* o = other + i * 2ull * n_actors;
      PNCounter a, c;
      a.p.inner = row_to_vclock(s, n_actors);
      a.n.inner = row_to_vclock(s + n_actors, n_actors);
      c.p.inner = row_to_vclock(o, n_actors);
      c.n.inner = row_to_vclock(o + n_actors, n_actors);
      a.merge(c);
      vclock_to_row(a.p.inner, s, n_actors);
      vclock_to_row(a.n.inner, s + n_actors, n_actors);
    }
  });
  return 0;
}
// Sparse (CSR) clocks: object i's clock is the run [off[i], off[i] + len[i])
// of (act, ctr) pairs (include/crdts_hip.h "Sparse (CSR) clocks"); merged by
// VClock::merge over std::map (src/vclock.rs:131-137), the result written at
// s_off[i] + o_off[i] (entries), out_len[i] = its length. A run that is not a
// canonical BTreeMap image (actors not strictly increasing, a zero counter)
// returns -2 with *bad = the object.
static bool run_to_vclock(const uint32_t* a, const uint64_t* c, uint64_t n, VClock& v) {
  for (uint64_t k = 0; k < n; ++k) {
    if (c[k] == 0 || (k && a[k - 1] >= a[k])) return false;
    v.dots.emplace_hint(v.dots.end(), a[k], c[k]);  // From<Vec<(A, u64)>>: witness each
  }
  return true;
}
int orc_vclock_csr_merge(const uint64_t* s_off, const uint32_t* s_len, const uint32_t* s_act,
                         const uint64_t* s_ctr, const uint64_t* o_off, const uint32_t* o_len,
                         const uint32_t* o_act, const uint64_t* o_ctr, size_t n, uint32_t* out_act,
                         uint64_t* out_ctr, uint32_t* out_len, int threads, int64_t* bad) {
  std::atomic<int64_t> first_bad{-1};
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      VClock a, o;
      if (!run_to_vclock(s_act + s_off[i], s_ctr + s_off[i], s_len[i], a) ||
          !run_to_vclock(o_act + o_off[i], o_ctr + o_off[i], o_len[i], o)) {
        int64_t exp = -1;
        first_bad.compare_exchange_strong(exp, (int64_t)i);
        out_len[i] = 0;
        continue;
      }
      a.merge(o);
      uint64_t at = s_off[i] + o_off[i];
      for (const auto& kv : a.dots) {
        out_act[at] = kv.first;
        out_ctr[at++] = kv.second;
      }
      out_len[i] = (uint32_t)a.dots.size();
    }
  });
  if (bad) *bad = first_bad.load();
  return first_bad.load() >= 0 ? -2 : 0;
}
// The CPU baseline of the CSR workload: the runs decoded into std::map
// VClocks beforehand (untimed), VClock::merge timed.
double orc_vclock_csr_bench(const uint64_t* s_off, const uint32_t* s_len, const uint32_t* s_act,
                            const uint64_t* s_ctr, const uint64_t* o_off, const uint32_t* o_len,
                            const uint32_t* o_act, const uint64_t* o_ctr, size_t n, int threads) {
  std::vector<VClock> A(n), B(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      run_to_vclock(s_act + s_off[i], s_ctr + s_off[i], s_len[i], A[i]);
      run_to_vclock(o_act + o_off[i], o_ctr + o_off[i], o_len[i], B[i]);
    }
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) A[i].merge(B[i]);
  });
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}
double orc_dense_bench(const uint64_t* self, const uint64_t* other, size_t n, uint32_t n_actors,
                       int threads) {
  std::vector<GCounter> A(n), B(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      A[i].inner = row_to_vclock(self + i * n_actors, n_actors);
      B[i].inner = row_to_vclock(other + i * n_actors, n_actors);
    }
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) A[i].merge(B[i]);
  });
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// --------------------------------------- object handles for KAT scripts
void* orc_obj_new() { return new Orswot(); }
void* orc_obj_clone(const void* h) { return new Orswot(*(const Orswot*)h); }
void orc_obj_free(void* h) { delete (Orswot*)h; }
void orc_obj_apply_add(void* h, uint32_t actor, uint64_t counter, uint64_t member) {
  ((Orswot*)h)->apply_add(actor, counter, member);
}
void orc_obj_apply_rm(void* h, uint64_t member, const uint32_t* act, const uint64_t* ctr,
                      uint32_t n) {
  VClock c;
  for (uint32_t i = 0; i < n; ++i) c.witness(act[i], ctr[i]);  // From<Vec<(A,u64)>>, :267-271
  ((Orswot*)h)->apply_rm(member, c);
}
void orc_obj_merge(void* dst, const void* src) { ((Orswot*)dst)->merge(*(const Orswot*)src); }
long orc_obj_encode(const void* h, uint32_t n_actors, uint8_t* out, size_t cap) {
  return encode(*(const Orswot*)h, n_actors, out, cap);
}
long orc_obj_encode_ex(const void* h, uint32_t n_actors, uint32_t flags, uint8_t* out, size_t cap) {
  return encode(*(const Orswot*)h, n_actors, out, cap, (flags & CRDT_ORSWOT_SPARSE_CLOCK) != 0);
}
void* orc_obj_decode(const uint8_t* rec, size_t bytes) {
  Orswot* o = new Orswot();
  if (!decode(rec, bytes, *o)) { delete o; return nullptr; }
  return o;
}
long orc_obj_deferred_len(const void* h) { return (long)((const Orswot*)h)->deferred.size(); }
// value(): sorted member keys; returns count (writes up to cap).
long orc_obj_value(const void* h, uint64_t* out, size_t cap) {
  const Orswot* o = (const Orswot*)h;
  std::vector<uint64_t> ks;
  for (auto& kv : o->entries) ks.push_back(kv.first);
  std::sort(ks.begin(), ks.end());
  for (size_t i = 0; i < ks.size() && i < cap; ++i) out[i] = ks[i];
  return (long)ks.size();
}
// contains(m).rm_clock: entry clock dots; returns n or -1 if absent.
long orc_obj_entry(const void* h, uint64_t member, uint32_t* act, uint64_t* ctr, size_t cap) {
  const Orswot* o = (const Orswot*)h;
  auto it = o->entries.find(member);
  if (it == o->entries.end()) return -1;
  size_t i = 0;
  for (auto& kv : it->second.dots) {
    if (i < cap) { act[i] = kv.first; ctr[i] = kv.second; }
    ++i;
  }
  return (long)i;
}
long orc_obj_clock(const void* h, uint32_t* act, uint64_t* ctr, size_t cap) {
  const Orswot* o = (const Orswot*)h;
  size_t i = 0;
  for (auto& kv : o->clock.dots) {
    if (i < cap) { act[i] = kv.first; ctr[i] = kv.second; }
    ++i;
  }
  return (long)i;
}

// --------------------------------------- VClock primitives for KATs
// Clocks passed as (actor[], counter[], n) built with witness (From<Vec>).
static VClock mk(const uint32_t* a, const uint64_t* c, uint32_t n) {
  VClock v;
  for (uint32_t i = 0; i < n; ++i) v.witness(a[i], c[i]);
  return v;
}
static long dump(const VClock& v, uint32_t* a, uint64_t* c, size_t cap) {
  size_t i = 0;
  for (auto& kv : v.dots) {
    if (i < cap) { a[i] = kv.first; c[i] = kv.second; }
    ++i;
  }
  return (long)i;
}
// op: 0 merge, 1 subtract, 2 intersection. Result written to (ra, rc).
long orc_vclock_binop(int op, const uint32_t* aa, const uint64_t* ac, uint32_t an,
                      const uint32_t* ba, const uint64_t* bc, uint32_t bn, uint32_t* ra,
                      uint64_t* rc, size_t cap) {
  VClock a = mk(aa, ac, an), b = mk(ba, bc, bn);
  if (op == 0) a.merge(b);
  else if (op == 1) a.subtract(b);
  else if (op == 2) a = a.intersection(b);
  else return CRDT_EINVAL;
  return dump(a, ra, rc, cap);
}
int orc_vclock_partial_cmp(const uint32_t* aa, const uint64_t* ac, uint32_t an,
                           const uint32_t* ba, const uint64_t* bc, uint32_t bn) {
  return mk(aa, ac, an).partial_cmp(mk(ba, bc, bn));
}

// ---------------------------------------------------------------- Map<u64, MVReg>
static MapO map_from_slab(const crdt_map_mvreg_slab& S, size_t i, uint32_t A) {
  MapO m;
  m.clock = row_to_vclock(S.clock + i * A, A);
  for (uint32_t k = 0; k < S.n_keys[i]; ++k) {
    const size_t ki = i * S.kcap + k;
    MapEntry e;
    e.clock = row_to_vclock(S.eclock + ki * A, A);
    for (uint32_t v = 0; v < S.mv_n[ki]; ++v)
      e.val.vals.emplace_back(row_to_vclock(S.mv_clock + (ki * S.mcap + v) * A, A), S.mv_val[ki * S.mcap + v]);
    m.entries[S.keys[ki]] = e;
  }
  for (uint32_t d = 0; d < S.n_def[i]; ++d) {
    const size_t di = i * S.dcap + d;
    auto& set = m.deferred[row_to_vclock(S.dclock + di * A, A).dots];
    for (uint32_t j = 0; j < S.dset_n[di]; ++j) set.insert(S.dset[di * S.scap + j]);
  }
  return m;
}

static bool map_to_slab(const MapO& m, const crdt_map_mvreg_slab& S, size_t i, uint32_t A) {
  if (m.entries.size() > S.kcap || m.deferred.size() > S.dcap) return false;
  vclock_to_row(m.clock, S.clock + i * A, A);
  S.n_keys[i] = (uint32_t)m.entries.size();
  uint32_t k = 0;
  for (uint32_t z = 0; z < S.kcap; ++z) {
    const size_t ki = i * S.kcap + z;
    S.keys[ki] = 0;
    S.mv_n[ki] = 0;
    std::fill(S.eclock + ki * A, S.eclock + (ki + 1) * A, 0ull);
    std::fill(S.mv_clock + ki * S.mcap * A, S.mv_clock + (ki + 1) * S.mcap * A, 0ull);
    std::fill(S.mv_val + ki * S.mcap, S.mv_val + (ki + 1) * S.mcap, 0ull);
  }
  for (const auto& kv : m.entries) {
    const size_t ki = i * S.kcap + k++;
    if (kv.second.val.vals.size() > S.mcap) return false;
    S.keys[ki] = kv.first;
    vclock_to_row(kv.second.clock, S.eclock + ki * A, A);
    S.mv_n[ki] = (uint32_t)kv.second.val.vals.size();
    for (uint32_t v = 0; v < S.mv_n[ki]; ++v) {
      vclock_to_row(kv.second.val.vals[v].first, S.mv_clock + (ki * S.mcap + v) * A, A);
      S.mv_val[ki * S.mcap + v] = kv.second.val.vals[v].second;
    }
  }
  S.n_def[i] = (uint32_t)m.deferred.size();
  for (uint32_t z = 0; z < S.dcap; ++z) {
    const size_t di = i * S.dcap + z;
    S.dset_n[di] = 0;
    std::fill(S.dclock + di * A, S.dclock + (di + 1) * A, 0ull);
    std::fill(S.dset + di * S.scap, S.dset + (di + 1) * S.scap, 0ull);
  }
  uint32_t d = 0;
  for (const auto& kv : m.deferred) {
    const size_t di = i * S.dcap + d++;
    if (kv.second.size() > S.scap) return false;
    VClock c;
    c.dots = kv.first;
    vclock_to_row(c, S.dclock + di * A, A);
    S.dset_n[di] = (uint32_t)kv.second.size();
    uint32_t j = 0;
    for (uint64_t key : kv.second) S.dset[di * S.scap + j++] = key;
  }
  return true;
}

// out[i] = self[i].merge(&other[i]); 0, or -4 when an output capacity is exceeded.
int orc_map_mvreg_merge_batch(const crdt_map_mvreg_slab* s, const crdt_map_mvreg_slab* o,
                              const crdt_map_mvreg_slab* out, size_t n, uint32_t A) {
  for (size_t i = 0; i < n; ++i) {
    MapO m = map_from_slab(*s, i, A);
    m.merge(map_from_slab(*o, i, A));
    if (!map_to_slab(m, *out, i, A)) return -4;
  }
  return 0;
}

// ---------------------------------------------------------------- Map<u64, Map<u64, MVReg>>
// The nested map's slab (include/crdts_hip.h crdt_map_map_slab): the outer
// map's arrays, key slot k of object i's nested map as object i*kcap + k of
// the inner Map<u64, MVReg> slab.
static MapMapO mapmap_from_slab(const crdt_map_map_slab& S, size_t i, uint32_t A) {
  MapMapO m;
  m.clock = row_to_vclock(S.clock + i * A, A);
  for (uint32_t k = 0; k < S.n_keys[i]; ++k) {
    const size_t ki = i * S.kcap + k;
    MapEntryT<MapO> e;
    e.clock = row_to_vclock(S.eclock + ki * A, A);
    e.val = map_from_slab(S.inner, ki, A);
    m.entries[S.keys[ki]] = e;
  }
  for (uint32_t d = 0; d < S.n_def[i]; ++d) {
    const size_t di = i * S.dcap + d;
    auto& set = m.deferred[row_to_vclock(S.dclock + di * A, A).dots];
    for (uint32_t j = 0; j < S.dset_n[di]; ++j) set.insert(S.dset[di * S.scap + j]);
  }
  return m;
}

static bool mapmap_to_slab(const MapMapO& m, const crdt_map_map_slab& S, size_t i, uint32_t A) {
  if (m.entries.size() > S.kcap || m.deferred.size() > S.dcap) return false;
  vclock_to_row(m.clock, S.clock + i * A, A);
  S.n_keys[i] = (uint32_t)m.entries.size();
  const MapO empty;
  for (uint32_t z = 0; z < S.kcap; ++z) {  // every key slot (its nested map emptied)
    const size_t ki = i * S.kcap + z;
    S.keys[ki] = 0;
    std::fill(S.eclock + ki * A, S.eclock + (ki + 1) * A, 0ull);
    if (!map_to_slab(empty, S.inner, ki, A)) return false;
  }
  uint32_t k = 0;
  for (const auto& kv : m.entries) {
    const size_t ki = i * S.kcap + k++;
    S.keys[ki] = kv.first;
    vclock_to_row(kv.second.clock, S.eclock + ki * A, A);
    if (!map_to_slab(kv.second.val, S.inner, ki, A)) return false;
  }
  S.n_def[i] = (uint32_t)m.deferred.size();
  for (uint32_t z = 0; z < S.dcap; ++z) {
    const size_t di = i * S.dcap + z;
    S.dset_n[di] = 0;
    std::fill(S.dclock + di * A, S.dclock + (di + 1) * A, 0ull);
    std::fill(S.dset + di * S.scap, S.dset + (di + 1) * S.scap, 0ull);
  }
  uint32_t d = 0;
  for (const auto& kv : m.deferred) {
    const size_t di = i * S.dcap + d++;
    if (kv.second.size() > S.scap) return false;
    VClock c;
    c.dots = kv.first;
    vclock_to_row(c, S.dclock + di * A, A);
    S.dset_n[di] = (uint32_t)kv.second.size();
    uint32_t j = 0;
    for (uint64_t key : kv.second) S.dset[di * S.scap + j++] = key;
  }
  return true;
}

// out[i] = self[i].merge(&other[i]) for nested maps; 0, or -4 past an output capacity.
int orc_map_map_merge_batch(const crdt_map_map_slab* s, const crdt_map_map_slab* o, const crdt_map_map_slab* out,
                            size_t n, uint32_t A) {
  for (size_t i = 0; i < n; ++i) {
    MapMapO m = mapmap_from_slab(*s, i, A);
    m.merge(mapmap_from_slab(*o, i, A));
    if (!mapmap_to_slab(m, *out, i, A)) return -4;
  }
  return 0;
}

// CPU baseline of the nested map merge: the n pairs decoded (untimed), then
// self.merge(&other) for every pair over `threads` std::threads; seconds.
double orc_map_map_bench(const crdt_map_map_slab* s, const crdt_map_map_slab* o, size_t n, uint32_t A,
                         int threads) {
  std::vector<MapMapO> L(n), R(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      L[i] = mapmap_from_slab(*s, i, A);
      R[i] = mapmap_from_slab(*o, i, A);
    }
  });
  auto t0 = std::chrono::steady_clock::now();
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) L[i].merge(R[i]);
  });
  auto t1 = std::chrono::steady_clock::now();
  volatile size_t sink = 0;
  for (size_t i = 0; i < n; i += 97) sink += L[i].entries.size();
  (void)sink;
  return std::chrono::duration<double>(t1 - t0).count();
}

// Replica pairs by op simulation (the reference's quickcheck shape,
// test/map.rs:520-740): per object a common history of updates
// (update(key, get(key).derive_add_ctx(actor), |reg, ctx| reg.set(v, ctx)),
// src/map.rs:300-313 + src/ctx.rs) and removes (rm(key, get(key)
// .derive_rm_ctx())), then two replicas diverge with their own actors and
// receive part of each other's ops, some out of order (deferred removes).
int orc_map_mvreg_generate(uint64_t seed, size_t n, uint32_t A, uint32_t keys, int ops,
                           const crdt_map_mvreg_slab* left, const crdt_map_mvreg_slab* right) {
  struct Op { int kind; Actor a; Counter c; uint64_t key; VClock clock; uint64_t val; };
  for (size_t i = 0; i < n; ++i) {
    uint64_t st = seed ^ (0x9E3779B97F4A7C15ull * (i + 1));
    auto rnd = [&]() {
      uint64_t z = (st += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      return z ^ (z >> 31);
    };
    MapO rep[2];
    std::vector<Op> log[2];
    auto make = [&](MapO& m, int r, bool shared) {
      Op op;
      const uint64_t key = rnd() % keys;
      if (rnd() % 100 < 70) {
        const Actor a = shared ? (Actor)(rnd() % A) : (Actor)((2 + r) % A);
        VClock cl = m.clock;  // get(key).derive_add_ctx(a): add_clock = the map clock
        const Counter c = cl.inc(a);
        cl.witness(a, c);
        op = Op{0, a, c, key, cl, rnd() >> 8};
      } else {
        auto it = m.entries.find(key);  // get(key).derive_rm_ctx(): the entry clock
        op = Op{1, 0, 0, key, it == m.entries.end() ? VClock() : it->second.clock, 0};
      }
      return op;
    };
    auto apply = [&](MapO& m, const Op& op) {
      if (op.kind == 0) m.apply_up(op.a, op.c, op.key, op.clock, op.val);
      else m.apply_rm(op.key, op.clock);
    };
    const int common = (int)(rnd() % (uint64_t)ops);
    for (int k = 0; k < common; ++k) {
      Op op = make(rep[0], 0, true);
      apply(rep[0], op);
      apply(rep[1], op);
    }
    for (int r = 0; r < 2; ++r) {
      const int div = 1 + (int)(rnd() % (uint64_t)ops);
      for (int k = 0; k < div; ++k) {
        Op op = make(rep[r], r, false);
        apply(rep[r], op);
        log[r].push_back(op);
      }
    }
    for (int r = 0; r < 2; ++r) {  // part of the other's ops, in a shuffled order (out-of-order removes defer)
      std::vector<Op> sub;
      for (const auto& op : log[1 - r])
        if (rnd() % 100 < 40) sub.push_back(op);
      if (rnd() % 100 < 15) {  // a remove from a third replica whose adds neither side has seen
        VClock c = rep[r].clock;
        c.witness((Actor)(A - 1), 1000 + rnd() % 8);
        sub.push_back(Op{1, 0, 0, rnd() % keys, c, 0});
      }
      for (size_t k = sub.size(); k > 1; --k) std::swap(sub[k - 1], sub[rnd() % k]);
      for (const auto& op : sub) apply(rep[r], op);
    }
    if (!map_to_slab(rep[0], *left, i, A) || !map_to_slab(rep[1], *right, i, A)) return -4;
  }
  return 0;
}

// ---------------------------------------------------------------- MVReg
// MVReg<V, A> { vals: Vec<(VClock<A>, V)> } (src/mvreg.rs:14-18), V = u64.
// merge (src/mvreg.rs:121-153): keep self's values no other value strictly
// dominates (`clock < c`, :126), then other's values no self value strictly
// dominates whose clock is not already kept (:136-150); order kept.
// Batch form: dense rows (0 = absent), `cap` slots per object.
int orc_mvreg_merge_batch(const uint32_t* sn, const uint64_t* sclk, const uint64_t* sval, uint32_t scap,
                          const uint32_t* on, const uint64_t* oclk, const uint64_t* oval, uint32_t ocap,
                          uint32_t* outn, uint64_t* oclk_out, uint64_t* oval_out, uint32_t outcap, size_t n,
                          uint32_t n_actors) {
  auto row = [&](const uint64_t* base, size_t obj, uint32_t cap, uint32_t k) {
    return row_to_vclock(base + ((size_t)obj * cap + k) * n_actors, n_actors);
  };
  for (size_t i = 0; i < n; ++i) {
    std::vector<std::pair<VClock, uint64_t>> self, other, vals;
    for (uint32_t k = 0; k < sn[i]; ++k) self.emplace_back(row(sclk, i, scap, k), sval[i * scap + k]);
    for (uint32_t k = 0; k < on[i]; ++k) other.emplace_back(row(oclk, i, ocap, k), oval[i * ocap + k]);
    for (const auto& sv : self) {
      size_t dom = 0;
      for (const auto& ov : other) dom += sv.first.partial_cmp(ov.first) == -1 ? 1 : 0;  // clock < c
      if (dom == 0) vals.push_back(sv);
    }
    for (const auto& ov : other) {
      size_t dom = 0;
      for (const auto& sv : self) dom += ov.first.partial_cmp(sv.first) == -1 ? 1 : 0;
      if (dom == 0) {
        bool is_new = true;
        for (const auto& e : vals)
          if (e.first == ov.first) { is_new = false; break; }
        if (is_new) vals.push_back(ov);
      }
    }
    if (vals.size() > outcap) return -4;
    outn[i] = (uint32_t)vals.size();
    for (uint32_t k = 0; k < outcap; ++k) {
      uint64_t* r = oclk_out + ((size_t)i * outcap + k) * n_actors;
      if (k < vals.size()) {
        vclock_to_row(vals[k].first, r, n_actors);
        oval_out[(size_t)i * outcap + k] = vals[k].second;
      } else {
        std::fill(r, r + n_actors, 0ull);
        oval_out[(size_t)i * outcap + k] = 0;
      }
    }
  }
  return 0;
}

// Dense-row VClock partial_cmp batch (src/vclock.rs:59-71): 0 Equal, 1 Greater, -1 Less, 2 None.
void orc_vclock_partial_cmp_rows(const uint64_t* a, const uint64_t* b, size_t n, uint32_t n_actors, int8_t* out) {
  for (size_t i = 0; i < n; ++i)
    out[i] = (int8_t)row_to_vclock(a + i * n_actors, n_actors).partial_cmp(row_to_vclock(b + i * n_actors, n_actors));
}


}  // extern "C"

namespace oracle {
// ---------------------------------------------------------------- Map<u64, Orswot>
// Map<u64, Orswot<u64, A>, A> (src/map.rs:82-98) — merge :192-269, apply
// :163-189, apply_rm :336-350, apply_deferred :325-333 — with the nested
// Orswot's merge / truncate above. The map's deferred removes are a HashMap
// in the reference; here a std::map (CLOCK ORDER), and apply_deferred takes
// an optional permutation of that order (`perm`, for enumerating the orders
// the reference could take).
struct MapOrEntry {
  VClock clock;
  Orswot val;
};
struct MapOrswotO {
  VClock clock;
  std::map<uint64_t, MapOrEntry> entries;
  std::map<std::map<Actor, Counter>, std::set<uint64_t>> deferred;
  const std::vector<int>* perm = nullptr;

  void apply_rm(uint64_t key, const VClock& c) {  // :336-350
    if (!c.le(clock)) deferred[c.dots].insert(key);
    auto it = entries.find(key);
    if (it != entries.end()) {
      MapOrEntry e = it->second;
      entries.erase(it);
      e.clock.subtract(c);
      if (!e.clock.is_empty()) {
        e.val.truncate(c);
        entries[key] = e;
      }
    }
  }
  void apply_deferred() {  // :325-333
    auto d = deferred;
    deferred.clear();
    std::vector<std::pair<VClock, std::set<uint64_t>>> v;
    for (const auto& kv : d) {
      VClock c;
      c.dots = kv.first;
      v.emplace_back(c, kv.second);
    }
    if (perm && perm->size() == v.size()) {
      auto w = v;
      for (size_t k = 0; k < v.size(); ++k) v[k] = w[(*perm)[k]];
    }
    for (const auto& kv : v)
      for (uint64_t k : kv.second) apply_rm(k, kv.first);
  }
  // Op::Up {dot, key, op} with op = the nested Orswot's Add or Rm (:169-187)
  void apply_up(Actor a, Counter ctr, uint64_t key, int kind, Actor da, Counter dc, uint64_t member,
                const VClock& rm_clock) {
    if (clock.get(a) >= ctr) return;
    MapOrEntry e;
    auto it = entries.find(key);
    if (it != entries.end()) { e = it->second; entries.erase(it); }
    e.clock.witness(a, ctr);
    if (kind == 0) e.val.apply_add(da, dc, member);
    else e.val.apply_rm(member, rm_clock);
    entries[key] = e;
    clock.witness(a, ctr);
    apply_deferred();
  }
  void merge(const MapOrswotO& other) {  // :193-268
    std::map<uint64_t, MapOrEntry> keep;
    for (const auto& kv : entries) {
      MapOrEntry entry = kv.second;
      auto oit = other.entries.find(kv.first);
      if (oit == other.entries.end()) {
        entry.clock.subtract(other.clock);
        if (!entry.clock.is_empty()) {
          VClock del = other.clock;
          del.subtract(entry.clock);
          entry.val.truncate(del);
          keep[kv.first] = entry;
        }
      } else {
        MapOrEntry oe = oit->second;
        VClock common = entry.clock.intersection(oe.clock);
        entry.clock.subtract(common);
        oe.clock.subtract(common);
        entry.clock.subtract(other.clock);
        oe.clock.subtract(clock);
        common.merge(entry.clock);
        common.merge(oe.clock);
        if (!common.is_empty()) {
          entry.val.merge(oe.val);
          VClock del = entry.clock;
          del.merge(oe.clock);
          del.subtract(common);
          entry.val.truncate(del);
          entry.clock = common;
          keep[kv.first] = entry;
        }
      }
    }
    for (const auto& kv : other.entries) {
      if (entries.count(kv.first)) continue;
      MapOrEntry entry = kv.second;
      entry.clock.subtract(clock);
      if (!entry.clock.is_empty()) {
        VClock del = clock;
        del.subtract(entry.clock);
        entry.val.truncate(del);
        keep[kv.first] = entry;
      }
    }
    for (const auto& kv : other.deferred) {  // apply_rm on the old entries: only the deferral survives
      VClock c;
      c.dots = kv.first;
      for (uint64_t k : kv.second) apply_rm(k, c);
    }
    entries = keep;
    clock.merge(other.clock);
    apply_deferred();
  }
};

static bool clock_dots_less(const std::map<Actor, Counter>& a, const std::map<Actor, Counter>& b) { return a < b; }

static Orswot orswot_from_slab(const crdt_map_orswot_slab& S, size_t ki, uint32_t A) {
  Orswot o;
  o.clock = row_to_vclock(S.vclock + ki * A, A);
  for (uint32_t m = 0; m < S.vn_mem[ki]; ++m)
    o.entries[S.vmem[ki * S.mcap + m]] = row_to_vclock(S.vmclock + (ki * S.mcap + m) * A, A);
  for (uint32_t d = 0; d < S.vn_def[ki]; ++d) {
    const size_t di = ki * S.vdcap + d;
    auto& set = o.deferred[row_to_vclock(S.vdclock + di * A, A)];
    for (uint32_t j = 0; j < S.vdset_n[di]; ++j) set.insert(S.vdset[di * S.vscap + j]);
  }
  return o;
}
static MapOrswotO mapor_from_slab(const crdt_map_orswot_slab& S, size_t i, uint32_t A) {
  MapOrswotO m;
  m.clock = row_to_vclock(S.clock + i * A, A);
  for (uint32_t k = 0; k < S.n_keys[i]; ++k) {
    const size_t ki = i * S.kcap + k;
    MapOrEntry e;
    e.clock = row_to_vclock(S.eclock + ki * A, A);
    e.val = orswot_from_slab(S, ki, A);
    m.entries[S.keys[ki]] = e;
  }
  for (uint32_t d = 0; d < S.n_def[i]; ++d) {
    const size_t di = i * S.dcap + d;
    auto& set = m.deferred[row_to_vclock(S.dclock + di * A, A).dots];
    for (uint32_t j = 0; j < S.dset_n[di]; ++j) set.insert(S.dset[di * S.scap + j]);
  }
  return m;
}
// One object's slab row, every slot written (unused ones zero); false when a capacity is exceeded.
static bool mapor_to_slab(const MapOrswotO& m, const crdt_map_orswot_slab& S, size_t i, uint32_t A) {
  if (m.entries.size() > S.kcap || m.deferred.size() > S.dcap) return false;
  vclock_to_row(m.clock, S.clock + i * A, A);
  S.n_keys[i] = (uint32_t)m.entries.size();
  for (uint32_t z = 0; z < S.kcap; ++z) {
    const size_t ki = i * S.kcap + z;
    S.keys[ki] = 0;
    S.vn_mem[ki] = 0;
    S.vn_def[ki] = 0;
    std::fill(S.eclock + ki * A, S.eclock + (ki + 1) * A, 0ull);
    std::fill(S.vclock + ki * A, S.vclock + (ki + 1) * A, 0ull);
    std::fill(S.vmem + ki * S.mcap, S.vmem + (ki + 1) * S.mcap, 0ull);
    std::fill(S.vmclock + ki * S.mcap * A, S.vmclock + (ki + 1) * S.mcap * A, 0ull);
    std::fill(S.vdclock + ki * S.vdcap * A, S.vdclock + (ki + 1) * S.vdcap * A, 0ull);
    std::fill(S.vdset_n + ki * S.vdcap, S.vdset_n + (ki + 1) * S.vdcap, 0u);
    std::fill(S.vdset + ki * S.vdcap * S.vscap, S.vdset + (ki + 1) * S.vdcap * S.vscap, 0ull);
  }
  uint32_t k = 0;
  for (const auto& kv : m.entries) {
    const size_t ki = i * S.kcap + k++;
    const Orswot& o = kv.second.val;
    if (o.entries.size() > S.mcap || o.deferred.size() > S.vdcap) return false;
    S.keys[ki] = kv.first;
    vclock_to_row(kv.second.clock, S.eclock + ki * A, A);
    vclock_to_row(o.clock, S.vclock + ki * A, A);
    std::vector<Member> mem;
    for (const auto& e : o.entries) mem.push_back(e.first);
    std::sort(mem.begin(), mem.end());
    S.vn_mem[ki] = (uint32_t)mem.size();
    for (uint32_t j = 0; j < mem.size(); ++j) {
      S.vmem[ki * S.mcap + j] = mem[j];
      vclock_to_row(o.entries.at(mem[j]), S.vmclock + (ki * S.mcap + j) * A, A);
    }
    std::vector<const VClock*> dk;
    for (const auto& e : o.deferred) dk.push_back(&e.first);
    std::sort(dk.begin(), dk.end(), [](const VClock* x, const VClock* y) { return clock_dots_less(x->dots, y->dots); });
    S.vn_def[ki] = (uint32_t)dk.size();
    for (uint32_t d = 0; d < dk.size(); ++d) {
      const size_t di = ki * S.vdcap + d;
      const auto& set = o.deferred.at(*dk[d]);
      if (set.size() > S.vscap) return false;
      vclock_to_row(*dk[d], S.vdclock + di * A, A);
      std::vector<Member> ms(set.begin(), set.end());
      std::sort(ms.begin(), ms.end());
      S.vdset_n[di] = (uint32_t)ms.size();
      for (uint32_t j = 0; j < ms.size(); ++j) S.vdset[di * S.vscap + j] = ms[j];
    }
  }
  S.n_def[i] = (uint32_t)m.deferred.size();
  for (uint32_t z = 0; z < S.dcap; ++z) {
    const size_t di = i * S.dcap + z;
    S.dset_n[di] = 0;
    std::fill(S.dclock + di * A, S.dclock + (di + 1) * A, 0ull);
    std::fill(S.dset + di * S.scap, S.dset + (di + 1) * S.scap, 0ull);
  }
  uint32_t d = 0;
  for (const auto& kv : m.deferred) {
    const size_t di = i * S.dcap + d++;
    if (kv.second.size() > S.scap) return false;
    VClock c;
    c.dots = kv.first;
    vclock_to_row(c, S.dclock + di * A, A);
    S.dset_n[di] = (uint32_t)kv.second.size();
    uint32_t j = 0;
    for (uint64_t key : kv.second) S.dset[di * S.scap + j++] = key;
  }
  return true;
}

// Canonical text of a map (for comparing outcomes across deferred orders).
static std::string mapor_key(const MapOrswotO& m) {
  std::string s;
  auto put = [&](uint64_t v) { s.append((const char*)&v, 8); };
  auto putc = [&](const VClock& c) { put(c.dots.size()); for (auto& kv : c.dots) { put(kv.first); put(kv.second); } };
  putc(m.clock);
  for (const auto& kv : m.entries) {
    put(kv.first);
    putc(kv.second.clock);
    const Orswot& o = kv.second.val;
    putc(o.clock);
    std::map<Member, const VClock*> es;
    for (const auto& e : o.entries) es[e.first] = &e.second;
    put(es.size());
    for (auto& e : es) { put(e.first); putc(*e.second); }
    std::map<std::map<Actor, Counter>, std::set<Member>> ds;
    for (const auto& e : o.deferred) ds[e.first.dots].insert(e.second.begin(), e.second.end());
    put(ds.size());
    for (auto& e : ds) { VClock c; c.dots = e.first; putc(c); put(e.second.size()); for (Member x : e.second) put(x); }
  }
  put(m.deferred.size());
  for (auto& e : m.deferred) { VClock c; c.dots = e.first; putc(c); put(e.second.size()); for (auto x : e.second) put(x); }
  return s;
}
}  // namespace oracle

extern "C" {

// out[i] = self[i].merge(&other[i]) with apply_deferred in CLOCK ORDER; 0, or
// -4 when an output capacity is exceeded.
int orc_map_orswot_merge_batch(const crdt_map_orswot_slab* s, const crdt_map_orswot_slab* o,
                               const crdt_map_orswot_slab* out, size_t n, uint32_t A) {
  for (size_t i = 0; i < n; ++i) {
    MapOrswotO m = mapor_from_slab(*s, i, A);
    m.merge(mapor_from_slab(*o, i, A));
    if (!mapor_to_slab(m, *out, i, A)) return -4;
  }
  return 0;
}

// Per object: the number of distinct merge results over every order the
// final apply_deferred of Map::merge can take (all permutations of the
// combined deferred clocks; -1 when there are more than `max_k` of them).
int orc_map_orswot_order_outcomes(const crdt_map_orswot_slab* s, const crdt_map_orswot_slab* o, size_t n,
                                  uint32_t A, int max_k, int32_t* outcomes) {
  for (size_t i = 0; i < n; ++i) {
    MapOrswotO a = mapor_from_slab(*s, i, A), b = mapor_from_slab(*o, i, A);
    // the combined deferred count the final apply_deferred sees
    MapOrswotO probe = a;
    {
      // replay merge up to apply_deferred: entries do not matter for the count
      for (const auto& kv : b.deferred) {
        VClock c;
        c.dots = kv.first;
        if (!c.le(probe.clock)) probe.deferred[kv.first];
      }
    }
    const int k = (int)probe.deferred.size();
    if (k > max_k) { outcomes[i] = -1; continue; }
    std::vector<int> perm(k);
    for (int j = 0; j < k; ++j) perm[j] = j;
    std::set<std::string> seen;
    do {
      MapOrswotO m = a;
      m.perm = &perm;
      m.merge(b);
      seen.insert(mapor_key(m));
    } while (std::next_permutation(perm.begin(), perm.end()));
    outcomes[i] = (int32_t)seen.size();
  }
  return 0;
}

// Replica pairs of Map<u64, Orswot<u64>> by op simulation (the shape of the
// reference's own Map tests, test/orswot.rs:270-307 and src/map.rs:38-80):
// a common history, then two replicas diverge with their own actors and get
// part of each other's ops out of order; updates are
//   update(key, get(key).derive_add_ctx(actor), |set, ctx| set.add(m, ctx))
//   update(key, ..., |set, ctx| set.remove(m, set.contains(&m).derive_rm_ctx()))
// and map removes rm(key, get(key).derive_rm_ctx()); with probability
// pct_future a remove carries a clock from a third replica (deferred at the
// map or at the nested set).
int orc_map_orswot_generate(uint64_t seed, size_t n, uint32_t A, uint32_t keys, uint32_t members, int ops,
                            int pct_future, const crdt_map_orswot_slab* left, const crdt_map_orswot_slab* right) {
  struct Op { int kind; Actor a; Counter c; uint64_t key; int vkind; uint64_t member; VClock clock; };
  for (size_t i = 0; i < n; ++i) {
    uint64_t st = seed ^ (0x9E3779B97F4A7C15ull * (i + 1));
    auto rnd = [&]() {
      uint64_t z = (st += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      return z ^ (z >> 31);
    };
    MapOrswotO rep[2];
    std::vector<Op> log[2];
    auto future = [&](VClock c) {
      c.witness((Actor)(A - 1), 1000 + rnd() % 4);
      return c;
    };
    auto make = [&](MapOrswotO& m, int r, bool shared) {
      Op op{};
      op.key = rnd() % keys;
      const uint64_t roll = rnd() % 100;
      if (roll < 75) {  // an update: nested add (60 %) or nested remove (15 %)
        op.kind = 0;
        op.a = shared ? (Actor)(rnd() % (A - 1)) : (Actor)((2 + r) % (A - 1));
        op.c = m.clock.inc(op.a);  // get(key).derive_add_ctx(a): the map clock's next dot
        op.member = rnd() % members;
        if (roll < 60) {
          op.vkind = 0;
        } else {
          op.vkind = 1;
          auto it = m.entries.find(op.key);
          VClock rc;
          if (it != m.entries.end()) {
            auto jt = it->second.val.entries.find(op.member);
            if (jt != it->second.val.entries.end()) rc = jt->second;
          }
          op.clock = (int)(rnd() % 100) < pct_future ? future(rc) : rc;
        }
      } else {  // a map remove with the entry's clock
        op.kind = 1;
        auto it = m.entries.find(op.key);
        VClock rc = it == m.entries.end() ? VClock() : it->second.clock;
        op.clock = (int)(rnd() % 100) < pct_future ? future(rc) : rc;
      }
      return op;
    };
    auto apply = [&](MapOrswotO& m, const Op& op) {
      if (op.kind == 0) m.apply_up(op.a, op.c, op.key, op.vkind, op.a, op.c, op.member, op.clock);
      else m.apply_rm(op.key, op.clock);
    };
    const int common = (int)(rnd() % (uint64_t)ops);
    for (int k = 0; k < common; ++k) {
      Op op = make(rep[0], 0, true);
      apply(rep[0], op);
      apply(rep[1], op);
    }
    for (int r = 0; r < 2; ++r) {
      const int div = 1 + (int)(rnd() % (uint64_t)ops);
      for (int k = 0; k < div; ++k) {
        Op op = make(rep[r], r, false);
        apply(rep[r], op);
        log[r].push_back(op);
      }
    }
    for (int r = 0; r < 2; ++r) {
      std::vector<Op> sub;
      for (const auto& op : log[1 - r])
        if (rnd() % 100 < 40) sub.push_back(op);
      for (size_t k = sub.size(); k > 1; --k) std::swap(sub[k - 1], sub[rnd() % k]);
      for (const auto& op : sub) apply(rep[r], op);
    }
    if (!mapor_to_slab(rep[0], *left, i, A) || !mapor_to_slab(rep[1], *right, i, A)) return -4;
  }
  return 0;
}

// ---- handles (op-path KATs): Map<u64, Orswot> and Map<u64, MVReg>
void* orc_mapor_new() { return new MapOrswotO(); }
void* orc_mapor_clone(const void* h) { return new MapOrswotO(*(const MapOrswotO*)h); }
void orc_mapor_free(void* h) { delete (MapOrswotO*)h; }
// Op::Up{dot (a, c), key, Orswot Op::Add{dot (a, c), member}} (kind 0) or
// Op::Up{dot, key, Orswot Op::Rm{clock, member}} (kind 1)
void orc_mapor_apply_up(void* h, uint32_t a, uint64_t c, uint64_t key, int kind, uint64_t member,
                        const uint32_t* ra, const uint64_t* rc, uint32_t rn) {
  ((MapOrswotO*)h)->apply_up(a, c, key, kind, a, c, member, mk(ra, rc, rn));
}
void orc_mapor_apply_rm(void* h, uint64_t key, const uint32_t* ra, const uint64_t* rc, uint32_t rn) {
  ((MapOrswotO*)h)->apply_rm(key, mk(ra, rc, rn));
}
void orc_mapor_merge(void* dst, const void* src) { ((MapOrswotO*)dst)->merge(*(const MapOrswotO*)src); }
int orc_mapor_to_slab(const void* h, const crdt_map_orswot_slab* S, size_t i, uint32_t A) {
  return mapor_to_slab(*(const MapOrswotO*)h, *S, i, A) ? 0 : -4;
}
void* orc_mapor_from_slab(const crdt_map_orswot_slab* S, size_t i, uint32_t A) {
  return new MapOrswotO(mapor_from_slab(*S, i, A));
}

void* orc_mapmv_new() { return new MapO(); }
void* orc_mapmv_clone(const void* h) { return new MapO(*(const MapO*)h); }
void orc_mapmv_free(void* h) { delete (MapO*)h; }
// Op::Up{dot (a, c), key, MVReg Op::Put{clock, val}}
void orc_mapmv_apply_up(void* h, uint32_t a, uint64_t c, uint64_t key, const uint32_t* pa, const uint64_t* pc,
                        uint32_t pn, uint64_t val) {
  ((MapO*)h)->apply_up(a, c, key, mk(pa, pc, pn), val);
}
void orc_mapmv_apply_rm(void* h, uint64_t key, const uint32_t* ra, const uint64_t* rc, uint32_t rn) {
  ((MapO*)h)->apply_rm(key, mk(ra, rc, rn));
}
void orc_mapmv_merge(void* dst, const void* src) { ((MapO*)dst)->merge(*(const MapO*)src); }
int orc_mapmv_to_slab(const void* h, const crdt_map_mvreg_slab* S, size_t i, uint32_t A) {
  return map_to_slab(*(const MapO*)h, *S, i, A) ? 0 : -4;
}

}  // extern "C"
