"""GPU parity of the replica fold (crdt_orswot_fold: ((r0 ⊔ r1) ⊔ r2) ⊔ ...
with Orswot::merge, src/orswot.rs:87-157 — BASELINE.json configs[4]) against
the oracle's sequential fold, byte-exact per record: config-5 CSR replicas
(8, and 1-3 replicas), dense config-3-shaped replicas, records past the join
kernel's stage (its general kernel), deferred-remove objects, the placement
rule, and malformed input."""
import numpy as np
import pytest

import records

pytestmark = pytest.mark.gpu


def _oracle_fold(oracle, reps, U, SP):
    acc = reps[0]
    for b, o in reps[1:]:
        acc = oracle.orswot_merge_batch(acc[0], acc[1], b, o, U, threads=16, flags=SP)
    return records.unpack_batch(*acc)


def _fold(gpu, reps, U, SP):
    import crdts_hip

    B = [crdts_hip.OrswotBatch.from_host(b, o, U, flags=SP) for b, o in reps]
    out = gpu.orswot_fold(B)
    nat = sum(o.astype(np.uint64) for _, o in reps)
    assert (out.off.cpu().numpy().view(np.uint64) == nat).all()  # placement: the sum of the inputs' offsets
    return out.records(), B


@pytest.mark.parametrize("R", [8, 1, 2, 3])
def test_fold_config5(gpu, oracle, R):
    import crdts_hip

    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    reps = crdts_hip.generate_replicas(20_000, R, threads=16)
    got, B = _fold(gpu, reps, U, SP)
    exp = _oracle_fold(oracle, reps, U, SP)
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not bad, f"{len(bad)} objects differ; first {bad[0]}: {records.decode(got[bad[0]])} vs {records.decode(exp[bad[0]])}"
    if R == 8:  # deferred-remove objects in the fold; the same bytes as the step-by-step GPU fold
        assert sum(1 for r in exp if records.decode(r)["deferred"]) > 100
        acc = B[0]
        for b in B[1:]:
            acc = gpu.orswot_merge(acc, b)
        assert acc.records() == got


def test_fold_large_objects_take_the_general_path(gpu, oracle):
    """Replicas with ~130-180 members: records around and past the 4 KB in
    flight and pairs past the 6 KB stage, mixed with config-5 ones."""
    import crdts_hip

    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    big = dict(crdts_hip.CONFIG5, member_universe=256, ancestor_adds=130)
    reps = crdts_hip.generate_replicas(3_000, 4, threads=16, params=big)
    sizes = [len(r) for r in records.unpack_batch(*reps[0])]
    assert max(sizes) > 4096 and min(sizes) < 4096
    got, _ = _fold(gpu, reps, U, SP)
    assert got == _oracle_fold(oracle, reps, U, SP)


def test_fold_rejects_malformed_and_dense(gpu):
    import crdts_hip

    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    reps = crdts_hip.generate_replicas(500, 3, threads=4)
    b, o = reps[1]
    b = b.copy()
    b[int(o[17]) + 4:int(o[17]) + 8] = np.frombuffer(np.uint32(2000).tobytes(), np.uint8)  # n_clk past the universe
    B = [crdts_hip.OrswotBatch.from_host(x, y, U, flags=SP) for x, y in (reps[0], (b, o), reps[2])]
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.orswot_fold(B)
    assert e.value.code == crdts_hip.CRDT_ENONCANON
    gpu.orswot_fold([crdts_hip.OrswotBatch.from_host(x, y, U, flags=SP) for x, y in reps])  # usable again


def test_fold_dense(gpu, oracle):
    """Dense top clocks (config-3 shape over 16 actors): 5 replicas, the
    second of each pair of generated sides standing in for further replicas."""
    import crdts_hip

    sides = []
    for k in range(3):
        (lb, lo), (rb, ro) = crdts_hip.generate_orswot(5_000, threads=8, seed=0xF01D + k)
        sides += [(lb, lo), (rb, ro)]
    reps = sides[:5]
    got, _ = _fold(gpu, reps, 16, 0)
    assert got == _oracle_fold(oracle, reps, 16, 0)
