"""GPU parity of the ingest / egest codec (crdt_orswot_from_bincode /
crdt_orswot_to_bincode) against the bincode
restatement (oracle/bincode_ref.py): byte-exact records from blobs in any
HashMap / HashSet order and at any byte alignment, byte-exact blobs from
records, the dense (config 3) and sparse (config 5) record forms, every
integer width, malformed input, and the ingest(egest(x)) == x round trip at
the full 1M-object config."""
import os
import random
import sys

import numpy as np
import pytest

import records

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import bincode_ref as BC  # noqa: E402
from test_bincode_oracle import extreme_state, small_members  # noqa: E402

pytestmark = pytest.mark.gpu


def _upload_blobs(blobs, rng=None):
    """Concatenate with 0-5 junk bytes between blobs (any alignment)."""
    import torch

    buf, off, ln = bytearray(), [], []
    for b in blobs:
        if rng is not None:
            buf += bytes(rng.randrange(256) for _ in range(rng.randrange(6)))
        off.append(len(buf))
        ln.append(len(b))
        buf += b
    t = torch.frombuffer(bytearray(buf) or bytearray(1), dtype=torch.uint8).to("cuda:0")
    o = torch.tensor(off, dtype=torch.int64, device="cuda:0")
    n = torch.tensor(ln, dtype=torch.int64, device="cuda:0")
    return t, o, n


def _blobs_of(out, off, lens):
    host = out.cpu().numpy()
    o, n = off.cpu().numpy(), lens.cpu().numpy()
    return [host[a:a + b].tobytes() for a, b in zip(o, n)]


def _state(st):
    return dict(clock=st["clock"], entries=st["entries"], deferred=st["deferred"])


def _rec(st, A, sparse):
    return records.encode(st["clock"], {m: dict(d) for m, d in st["entries"].items()},
                          {tuple(c): set(ms) for c, ms in st["deferred"]}, A, sparse)


def test_ingest_config3_shuffled(gpu):
    import crdts_hip

    (b, o), _ = crdts_hip.generate_orswot(20_000, first_obj=5, threads=16)
    recs = records.unpack_batch(b, o)
    rng = random.Random(7)
    blobs = [BC.encode(_state(records.decode(r)), 1, 8, rng=rng) for r in recs]
    t, bo, bl = _upload_blobs(blobs, rng)
    out = gpu.orswot_from_bincode(t, bo, bl, 16, 1, 8)
    got = out.records()
    bad = [i for i, (g, e) in enumerate(zip(got, recs)) if g != e]
    assert not bad, f"{len(bad)} differ; first {bad[0]}: {records.decode(got[bad[0]])} vs {records.decode(recs[bad[0]])}"
    assert sum(1 for r in recs if records.decode(r)["deferred"]) > 100


def test_egest_config3(gpu):
    import crdts_hip

    (b, o), _ = crdts_hip.generate_orswot(20_000, first_obj=11, threads=16)
    B = crdts_hip.OrswotBatch.from_host(b, o, 16)
    got = _blobs_of(*gpu.orswot_to_bincode(B, 1, 8))
    exp = [BC.encode(_state(records.decode(r)), 1, 8) for r in records.unpack_batch(b, o)]
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not bad, f"{len(bad)} differ; first {bad[0]}"


@pytest.mark.parametrize("wa,wm", [(2, 2), (4, 4), (8, 8), (1, 1)])
def test_widths_both_ways(gpu, wa, wm):
    import crdts_hip

    (b, o), _ = crdts_hip.generate_orswot(3_000, first_obj=wa * 100 + wm, threads=16)
    sts = [small_members(records.decode(r)) for r in records.unpack_batch(b, o)]
    if wm == 1:
        sts = [s for s in sts if max(list(s["entries"]) + [m for _, ms in s["deferred"] for m in ms] + [0]) < 256]
    recs = [_rec(s, 16, False) for s in sts]
    rng = random.Random(wa + wm)
    t, bo, bl = _upload_blobs([BC.encode(s, wa, wm, rng=rng) for s in sts], rng)
    assert gpu.orswot_from_bincode(t, bo, bl, 16, wa, wm).records() == recs
    assert gpu.orswot_from_bincode(t, bo, bl, 16, wa, wm, packed=False).records() == recs
    B = crdts_hip.OrswotBatch.from_records(recs, 16)
    assert _blobs_of(*gpu.orswot_to_bincode(B, wa, wm)) == [BC.encode(s, wa, wm) for s in sts]


def test_sparse_config5_both_ways(gpu):
    import crdts_hip

    b, o = crdts_hip.generate_replicas(5_000, 2, first_obj=3, threads=16)[1]
    recs = records.unpack_batch(b, o)
    sts = [_state(records.decode(r)) for r in recs]
    rng = random.Random(5)
    t, bo, bl = _upload_blobs([BC.encode(s, 2, 8, rng=rng) for s in sts], rng)
    SP = crdts_hip.SPARSE_CLOCK
    out = gpu.orswot_from_bincode(t, bo, bl, 1024, 2, 8, flags=SP)
    assert out.records() == recs
    assert gpu.orswot_from_bincode(t, bo, bl, 1024, 2, 8, flags=SP, packed=False).records() == recs
    B = crdts_hip.OrswotBatch.from_host(b, o, 1024, flags=SP)
    assert _blobs_of(*gpu.orswot_to_bincode(B, 2, 8)) == [BC.encode(s, 2, 8) for s in sts]


def test_round_trip_full_config3(gpu):
    """ingest(egest(batch)) == batch, byte-exact, at BASELINE's 1M objects."""
    import torch

    import crdts_hip

    (b, o), _ = crdts_hip.generate_orswot(1_000_000, threads=16)
    B = crdts_hip.OrswotBatch.from_host(b, o, 16)
    blobs, boff, blen = gpu.orswot_to_bincode(B, 1, 8)
    back = gpu.orswot_from_bincode(blobs, boff, blen, 16, 1, 8)
    assert torch.equal(back.off, B.off)
    n = int(b.nbytes)
    assert torch.equal(back.base[:n], B.base[:n])
    # one-read ingest (records placed by their bounds): the same records with
    # gaps; compacted, the same bytes
    gapped = gpu.orswot_from_bincode(blobs, boff, blen, 16, 1, 8, packed=False)
    sizes = gapped.base.view(torch.int32)[gapped.off // 4].to(torch.int64)
    ref_sizes = B.base.view(torch.int32)[B.off // 4].to(torch.int64)
    assert torch.equal(sizes, ref_sizes)
    assert bool((gapped.off[1:] - gapped.off[:-1] >= sizes[:-1]).all())
    packed = gpu.orswot_compact(gapped)
    assert torch.equal(packed.off, B.off) and torch.equal(packed.base[:n], B.base[:n])


@pytest.mark.parametrize("wa,wm", [(1, 1), (1, 8), (2, 2), (8, 1), (8, 8), (4, 2)])
@pytest.mark.parametrize("sparse", [False, True])
def test_bound_placement_extreme_shapes(gpu, wa, wm, sparse):
    """Records placed by crdt_orswot_bincode_record_bounds for shapes that
    stress each term of the bound (narrow members in big deferred sets, many
    one-dot members, sparse clocks): every record is decoded whole into its
    slot, byte-exact."""
    import crdts_hip

    rng = random.Random(wa * 10 + wm + sparse)
    A = 256 if sparse else 16
    sts = [extreme_state(rng, A, wa, wm) for _ in range(400)]
    t, bo, bl = _upload_blobs([BC.encode(s, wa, wm) for s in sts])
    SP = crdts_hip.SPARSE_CLOCK if sparse else 0
    out = gpu.orswot_from_bincode(t, bo, bl, A, wa, wm, flags=SP, packed=False)
    assert out.records() == [_rec(s, A, sparse) for s in sts]


def test_malformed_blobs(gpu):
    import crdts_hip
    from crdts_hip._lib import CrdtError

    good = dict(clock={1: 3, 2: 4}, entries={7: [(1, 3)], 9: [(2, 4)]}, deferred=[([(3, 1)], [5, 6])])
    g = BC.encode(good, 1, 1)
    cases = {
        "truncated": g[:-1],
        "trailing": g + b"\x00",
        "zero counter": BC.encode(dict(clock={1: 0}, entries={}, deferred=[]), 1, 1),
        "actor >= n_actors": BC.encode(dict(clock={20: 1}, entries={}, deferred=[]), 1, 1),
        "dup member": BC.encode(good, 1, 1).replace(b"\x09\x01\x00", b"\x07\x01\x00", 1),
        "empty member clock": BC.encode(dict(clock={1: 1}, entries={4: []}, deferred=[]), 1, 1),
        "huge length": b"\xff" * 8 + g[8:],
    }
    for name, blob in cases.items():
        t, bo, bl = _upload_blobs([g, blob, g])
        with pytest.raises(CrdtError) as e:
            gpu.orswot_from_bincode(t, bo, bl, 16, 1, 1)
        assert e.value.code in (-2,), name
    # past the LDS path's 256 members the large-object kernel decodes it ...
    big = dict(clock={1: 400}, entries={m: [(1, m + 1)] for m in range(300)}, deferred=[])
    g2 = BC.encode(good, 1, 2)  # the neighbours in the same member width
    t, bo, bl = _upload_blobs([g2, BC.encode(big, 1, 2, rng=random.Random(4)), g2])
    got = gpu.orswot_from_bincode(t, bo, bl, 16, 1, 2).records()
    assert got == [_rec(good, 16, False), _rec(big, 16, False), _rec(good, 16, False)]
    # ... up to 16 384 members (the HBM scratch); past that, CRDT_ECAPACITY
    huge = dict(clock={1: 20_000}, entries={m: [(1, m + 1)] for m in range(16_385)}, deferred=[])
    t, bo, bl = _upload_blobs([BC.encode(huge, 1, 2)])
    with pytest.raises(CrdtError) as e:
        gpu.orswot_from_bincode(t, bo, bl, 16, 1, 2)
    assert e.value.code == -4
    # egest: a member key wider than member_bytes
    B = crdts_hip.OrswotBatch.from_records([_rec(dict(clock={1: 1}, entries={300: [(1, 1)]}, deferred=[]), 16,
                                                 False)], 16)
    with pytest.raises(CrdtError):
        gpu.orswot_to_bincode(B, 1, 1)
    gpu.status()  # latched errors were cleared by the raising calls


def test_group_walk_shapes(gpu):
    """The decode pass walks the blobs that share one 4 KB window as a group
    (lane-parallel entry chains): ~30 small blobs per group, a blob past the
    scratch's deferred limit inside a group (sent to the large-object
    kernel), blobs straddling the window edge — records byte-exact; a
    malformed blob inside a group, and blobs whose claimed entry counts
    overflow the group's entry arrays (the per-object fallback) — errors
    latched. (Valid blobs cannot overflow them: an entry takes >= 18 B, so a
    4 KB window holds < 256.)"""
    from crdts_hip._lib import CrdtError

    rng = random.Random(11)

    def tiny(k, nm):
        return dict(clock={1 + k % 15: 1 + k}, entries={(k * 7 + j) % 250: [(1 + k % 15, 1 + j % (1 + k))]
                                                         for j in range(nm)}, deferred=[])

    # 120 blobs of 5-6 members, ~30 to a window
    sts = [tiny(k, 5 + k % 2) for k in range(120)]
    # a small blob with 100 deferred clocks (past the scratch's deferred limit) among them
    sts[40] = dict(clock={2: 1}, entries={3: [(2, 1)]}, deferred=[([(1, d + 1)], [d % 200]) for d in range(100)])
    # blobs of ~1.3 KB so that groups end at the window edge
    sts += [dict(clock={1: 90}, entries={m: [(1, m + 1)] for m in range(70 + k)}, deferred=[]) for k in range(12)]
    t, bo, bl = _upload_blobs([BC.encode(s, 1, 1, rng=rng) for s in sts], rng)
    exp = [_rec(s, 16, False) for s in sts]
    assert gpu.orswot_from_bincode(t, bo, bl, 16, 1, 1).records() == exp
    assert gpu.orswot_from_bincode(t, bo, bl, 16, 1, 1, packed=False).records() == exp
    # one malformed blob (a trailing byte) in the middle of a group
    blobs = [BC.encode(s, 1, 1) for s in sts[:20]]
    blobs[9] = blobs[9] + b"\x00"
    t, bo, bl = _upload_blobs(blobs)
    with pytest.raises(CrdtError) as e:
        gpu.orswot_from_bincode(t, bo, bl, 16, 1, 1)
    assert e.value.code == -2
    # two blobs claiming 200 entries each in one window
    liar = (0).to_bytes(8, "little") + (200).to_bytes(8, "little") + bytes(40)
    t, bo, bl = _upload_blobs([BC.encode(s, 1, 1) for s in sts[:3]] + [liar, liar] + [BC.encode(sts[3], 1, 1)])
    with pytest.raises(CrdtError) as e:
        gpu.orswot_from_bincode(t, bo, bl, 16, 1, 1)
    assert e.value.code == -2
    gpu.status()
