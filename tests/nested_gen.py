"""Nested-map (TestMap = Map<u8, Map<u8, MVReg<u8, u8>>>, test/map.rs:4-8)
replica pairs by op simulation on the Python restatement — test and bench
infrastructure (tests/test_gpu_map_nested.py, bench.py --workload map_map)."""
import map_kat_runner as mkr


def make_op(m, rng, actor):
    """A nested op as the reference's API makes it from m's read contexts
    (src/map.rs:291-322, src/ctx.rs:45-60): a nested put, an outer remove, an
    inner remove or an update with a no-op inner op."""
    k1, k2 = rng.randrange(4), rng.randrange(4)
    dot = [actor, m.clock.get(actor) + 1]
    clock = sorted({**m.clock.dots, actor: dot[1]}.items())
    e = m.entries.get(k1)
    r = rng.random()
    if r < 0.5 or e is None:
        return {"up": {"dot": dot, "key": k1,
                       "op": {"up": {"dot": dot, "key": k2, "op": {"put": {"clock": clock, "val": rng.randrange(1 << 40)}}}}}}
    if r < 0.7:
        return {"rm": {"clock": sorted(e[0].dots.items()), "key": k1}}
    ie = e[1].entries.get(k2)
    if r < 0.9 and ie is not None:
        return {"up": {"dot": dot, "key": k1, "op": {"rm": {"clock": sorted(ie[0].dots.items()), "key": k2}}}}
    return {"up": {"dot": dot, "key": k1, "op": "nop"}}


def pair(rng, pool):
    m0 = mkr.nested_map()
    for _ in range(rng.randrange(0, 8)):
        mkr.apply_raw(m0, make_op(m0, rng, rng.choice(pool)))
    a1, a2, a3 = rng.sample(pool, 3)
    m1, m2, m3 = m0.clone(), m0.clone(), m0.clone()
    ops1, ops2 = [], []
    for m, a, log in ((m1, a1, ops1), (m2, a2, ops2), (m3, a3, None)):
        for _ in range(rng.randrange(1, 8)):
            op = make_op(m, rng, a)
            mkr.apply_raw(m, op)
            if log is not None:
                log.append(op)
    # a third replica's removes (clocks with its own dots) reach m1 early and
    # stay deferred: outer removes, and inner removes inside an update
    for _ in range(rng.randrange(0, 4)):
        k1, k2 = rng.randrange(4), rng.randrange(4)
        e = m3.entries.get(k1)
        if e is None:
            continue
        ie = e[1].entries.get(k2)
        if ie is not None and rng.random() < 0.5:
            dot = [a3, m3.clock.get(a3) + 1]
            op = {"up": {"dot": dot, "key": k1, "op": {"rm": {"clock": sorted(ie[0].dots.items()), "key": k2}}}}
            mkr.apply_raw(m3, op)
        else:
            op = {"rm": {"clock": sorted(e[0].dots.items()), "key": k1}}
        mkr.apply_raw(m1, op)
    # part of each side's ops reach the other, out of order (concurrent values)
    for src, dst in ((ops1, m2), (ops2, m1)):
        sub = [op for op in src if rng.random() < 0.4]
        rng.shuffle(sub)
        for op in sub:
            mkr.apply_raw(dst, op)
    return m1, m2
