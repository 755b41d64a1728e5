"""KAT backend whose states are built by the product's host op path and whose
every `merge` is executed by the HIP kernel (crdts_hip.Orswot.merge)."""
from __future__ import annotations


class GpuBackend:
    def __init__(self, engine, n_actors=16, sparse=False):
        import crdts_hip

        self.m = crdts_hip
        self.eng = engine
        self.n_actors = n_actors
        self.sparse = sparse
        self.merges = 0

    def new(self):
        return self.m.Orswot(self.n_actors, sparse=self.sparse)

    def load(self, state):
        import kat_runner

        rec = kat_runner._state_record(state, self.n_actors)
        return self.m.Orswot(self.n_actors, host=self.m.HostOrswot.decode(rec), sparse=self.sparse)

    def clone(self, o):
        return o.clone()

    def apply_add(self, o, actor, counter, member):
        o.apply_add(actor, counter, member)

    def apply_rm(self, o, member, pairs):
        o.apply_rm(member, pairs)

    def merge(self, dst, src):
        dst.merge(src, engine=self.eng)
        self.merges += 1

    def clock(self, o):
        return o.clock()

    def entry(self, o, member):
        return o.entry(member)

    def value(self, o):
        return o.value()

    def deferred_len(self, o):
        return o.deferred_len()
