"""The boundary's documented per-object limits (include/crdts_hip.h), each
exercised at the limit (byte-exact result) and one past it (CRDT_ECAPACITY):
crdt_orswot_apply (members, deferred clocks; src/orswot.rs:61-85, 195-211)
and crdt_orswot_from_bincode (members, deferred clocks; src/lib.rs:79-83)."""
import os
import sys

import pytest

import records

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import bincode_ref as BC  # noqa: E402
from test_gpu_apply import _oracle_apply  # noqa: E402
from test_gpu_bincode import _rec, _upload_blobs  # noqa: E402

pytestmark = pytest.mark.gpu
A = 4
CAP = -4  # CRDT_ECAPACITY


def _apply(gpu, rec, ops):
    import crdts_hip

    B = crdts_hip.OrswotBatch.from_records([rec], A)
    return gpu.orswot_apply(B, crdts_hip.OrswotOps.from_lists([ops])).records()[0]


@pytest.mark.parametrize("n_mem,ok", [(4095, True), (4096, False)])
def test_apply_member_limit(gpu, oracle, n_mem, ok):
    """An Add of a new member to an object of n_mem members: 4096 members after
    it is the HBM workspace's limit (passes), 4097 is past it."""
    import crdts_hip

    rec = records.encode({0: 9000, 1: 3}, {m: {0: m + 1} for m in range(n_mem)}, {}, A)
    ops = [("add", 1, 4, 10**9)]
    if ok:
        assert _apply(gpu, rec, ops) == _oracle_apply(oracle, rec, ops, A, 0)
    else:
        with pytest.raises(crdts_hip.CrdtError) as e:
            _apply(gpu, rec, ops)
        assert e.value.code == CAP


@pytest.mark.parametrize("n_def,ok", [(255, True), (256, False)])
def test_apply_deferred_limit(gpu, oracle, n_def, ok):
    """An Rm with a future context (deferred, src/orswot.rs:197-200) on an
    object holding n_def deferred clocks: 256 after it passes, 257 does not."""
    import crdts_hip

    rec = records.encode({0: 5000}, {m: {0: m + 1} for m in range(40)},
                         {((0, 5001 + k),): {10_000 + k} for k in range(n_def)}, A)
    ops = [("rm", 7, [(0, 5000), (1, 1)])]
    if ok:
        assert _apply(gpu, rec, ops) == _oracle_apply(oracle, rec, ops, A, 0)
    else:
        with pytest.raises(crdts_hip.CrdtError) as e:
            _apply(gpu, rec, ops)
        assert e.value.code == CAP


@pytest.mark.parametrize("n_mem,ok", [(16_384, True), (16_385, False)])
def test_ingest_member_limit(gpu, n_mem, ok):
    import crdts_hip

    st = dict(clock={1: 20_000}, entries={m: [(1, m + 1)] for m in range(n_mem)}, deferred=[])
    t, bo, bl = _upload_blobs([BC.encode(st, 1, 2)])
    if ok:
        assert gpu.orswot_from_bincode(t, bo, bl, 16, 1, 2).records() == [_rec(st, 16, False)]
    else:
        with pytest.raises(crdts_hip.CrdtError) as e:
            gpu.orswot_from_bincode(t, bo, bl, 16, 1, 2)
        assert e.value.code == CAP


@pytest.mark.parametrize("n_def,ok", [(1024, True), (1025, False)])
def test_ingest_deferred_limit(gpu, n_def, ok):
    import crdts_hip

    st = dict(clock={1: 5}, entries={m: [(1, 1 + m % 5)] for m in range(30)},
              deferred=[([(1, 6 + k)], [k, k + 1]) for k in range(n_def)])
    t, bo, bl = _upload_blobs([BC.encode(st, 1, 2)])
    if ok:
        assert gpu.orswot_from_bincode(t, bo, bl, 16, 1, 2).records() == [_rec(st, 16, False)]
    else:
        with pytest.raises(crdts_hip.CrdtError) as e:
            gpu.orswot_from_bincode(t, bo, bl, 16, 1, 2)
        assert e.value.code == CAP
