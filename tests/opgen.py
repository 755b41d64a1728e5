"""Seeded stand-ins for the reference's quickcheck generators (test infrastructure).

quickcheck 0.6 draws integers in [0, size) with size = 100 by default, so
`Vec<(u8, u8, u8, u64)>` op primitives (test/orswot.rs:14-34) are tuples of
small integers; the generators below reproduce that shape with a seed.
"""
from __future__ import annotations

import random


def orswot_opvec(rng: random.Random, max_len=40, size=100, actor_range=None, member_range=None):
    """test/orswot.rs:14-34 build_opvec: (actor, member, choice, counter) -> Add | Rm."""
    n = rng.randrange(0, max_len + 1)
    ar = actor_range or size
    mr = member_range or size
    ops = []
    for _ in range(n):
        actor, member, choice, counter = (rng.randrange(ar), rng.randrange(mr), rng.randrange(size),
                                          rng.randrange(size))
        if choice % 2 == 0:
            ops.append((actor, ("add", actor, counter, member)))
        else:
            ops.append((actor, ("rm", member, [(actor, counter)])))  # Dot{actor,counter}.into()
    return ops


def pncounter_opvec(rng: random.Random, max_len=40, size=100, actor_range=11):
    """test/pncounter.rs:6-16 build_op: (actor, counter, dir)."""
    n = rng.randrange(0, max_len + 1)
    return [((rng.randrange(actor_range), rng.randrange(size)), rng.random() < 0.5) for _ in range(n)]


def apply_op(backend, obj, op):
    if op[0] == "add":
        _, actor, counter, member = op
        backend.apply_add(obj, actor, counter, member)
    else:
        _, member, pairs = op
        backend.apply_rm(obj, member, pairs)
