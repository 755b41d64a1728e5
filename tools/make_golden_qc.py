#!/usr/bin/env python3
"""Generate tests/golden/quickcheck_evolution.json from the reference's
quickcheck_evolution.log (run here, where /root/reference exists; the JSON is
committed and the tests read only the JSON).

The log (quickcheck_evolution.log:1-492) catalogues 8 op vectors that once
made prop_merge_converges (test/orswot.rs:37-76) fail, each with the witness
states the failing run printed. Both are INPUTS here: the op vectors are
replayed through the current op API and the witness lists are folded by the
current merge; the logged "merged:" outputs came from the buggy code of the
time and are not used as expected values.

Op vectors are transcribed by hand below (their text format changed between
entries); witness states are parsed from the log text.
"""
import json
import os
import re
import sys

LOG = "/root/reference/quickcheck_evolution.log"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "quickcheck_evolution.json")


def rm(member, actor, ctx=None):
    return {"kind": "rm", "member": member, "actor": actor, "ctx": ctx}


def add(member, actor, dest=None):
    d = {"kind": "add", "member": member, "actor": actor}
    if dest is not None:
        d["dest"] = dest
    return d


# (log lines of the op vector, summary line, ops)
OPS = [
    ("3-5", "when the dots for different adds are the same, the adds don't add up",
     [add(10, 0, dest=1), add(5, 6, dest=0)]),
    ("66-68", "deleting without a context can diverge (post mortem: always use context)",
     [add(0, 6), rm(0, 7, None)]),
    ("94", "BUG: merge compared the other side's top clock instead of its entry clock",
     [add(4, 6), add(4, 5)]),
    ("128-130", "BUG: deferred removes only present in the other set were ignored",
     [add(7, 3), rm(7, 10, [[0, 6], [1, 6], [2, 1], [3, 3]])]),
    ("202-204", "test-suite bug: generated context not modded while the witness was",
     [rm(3, 0, [[0, 3], [1, 2], [2, 6], [3, 3], [4, 4], [5, 4]]), add(3, 8)]),
    ("294-297", "deferred operations are only applied during merges, not during adds",
     [rm(5, 7, [[0, 2], [1, 4], [2, 3], [3, 3], [4, 3], [5, 3]]), add(0, 8), add(5, 4)]),
    ("379-383", "BUG: unseen defers missing from the merged deferred map (descendence vs partial unseen dots)",
     [add(1, 5), rm(1, 9, [[0, 3], [1, 5], [2, 4], [3, 5], [4, 6], [5, 4]]), add(4, 6),
      rm(9, 3, [[0, 6], [1, 1], [2, 6], [3, 1], [4, 4]])]),
    ("435-438", "add blindly overwrote causality info: adds of one element on several replicas diverged",
     [add(2, 7), rm(2, 8, [[0, 2], [1, 2]]), add(2, 0)]),
]


class P:
    """Recursive-descent parser of the log's Debug-printed Orswot states."""

    def __init__(self, s):
        self.s, self.i = s, 0

    def ws(self):
        while self.i < len(self.s) and self.s[self.i] in " \t\r\n":
            self.i += 1

    def eat(self, tok):
        self.ws()
        if not self.s.startswith(tok, self.i):
            raise ValueError(f"expected {tok!r} at {self.s[self.i:self.i + 40]!r}")
        self.i += len(tok)

    def peek(self, tok):
        self.ws()
        return self.s.startswith(tok, self.i)

    def num(self):
        self.ws()
        m = re.compile(r"\d+").match(self.s, self.i)
        self.i = m.end()
        return int(m.group())

    def seq(self, item, close):
        out = []
        while not self.peek(close):
            out.append(item())
            if self.peek(","):
                self.eat(",")
        self.eat(close)
        return out

    def vclock(self):
        self.eat("VClock")
        self.eat("{")
        self.eat("dots:")
        self.eat("{")

        def kv():
            a = self.num()
            self.eat(":")
            return [a, self.num()]

        d = self.seq(kv, "}")
        self.eat("}")
        return sorted(d)

    def orswot(self):
        self.eat("Orswot")
        self.eat("{")
        self.eat("clock:")
        clock = self.vclock()
        self.eat(",")
        self.eat("entries:")
        self.eat("{")

        def entry():
            m = self.num()
            self.eat(":")
            return [m, self.vclock()]

        entries = self.seq(entry, "}")
        self.eat(",")
        self.eat("deferred:")
        self.eat("{")

        def dfr():
            c = self.vclock()
            self.eat(":")
            self.eat("{")
            return [c, sorted(self.seq(self.num, "}"))]

        deferred = self.seq(dfr, "}")
        self.eat("}")
        return {"clock": clock, "entries": sorted(entries), "deferred": sorted(deferred)}


def main():
    with open(LOG) as f:
        lines = f.read().split("\n")
    # scenario k spans from its op vector to the next separator block
    starts = [int(r.split("-")[0]) for r, _, _ in OPS]
    seps = [i + 1 for i, l in enumerate(lines) if l.startswith("~~~~")]
    scen = []
    for k, (rng, summary, ops) in enumerate(OPS):
        lo = starts[k]
        hi = min([s for s in seps if s > lo] + [len(lines)])
        sets = []
        i = lo - 1
        while i < hi - 1:
            if lines[i].lstrip().split(" ")[-1].startswith("witnesses:") or "witnesses:" in lines[i]:
                j = i
                while j < hi - 1 and not lines[j].lstrip().startswith("merged"):
                    j += 1
                text = "".join(lines[i:j])  # wrapped lines split tokens: join without separators
                text = text[text.index("[") + 1:]
                p = P(text)
                states = p.seq(p.orswot, "]")
                sets.append({"log_lines": f"{i + 1}-{j}", "witnesses": states})
                i = j
            i += 1
        scen.append({"name": f"quickcheck_evolution_{k + 1}", "log_lines": rng, "summary": summary,
                     "ops": ops, "witness_sets": sets})
    doc = {
        "_doc": ("INPUTS transcribed from the reference's quickcheck_evolution.log (8 op vectors that once broke "
                 "prop_merge_converges, test/orswot.rs:37-76, with the witness states the failing runs printed). "
                 "The logged merge outputs came from buggy code and are NOT expected values. Replay rule onto the "
                 "current op API (test/orswot.rs:14-34): for i in 2..ACTOR_MAX(11) witnesses, op (member, actor) goes "
                 "to witness actor % i; Add -> Op::Add{dot: Dot{actor, counter: k}, member} with k = 1 + the number "
                 "of earlier Adds by the same actor (one mutator per actor, the post mortem of scenario 1; 'dest' of "
                 "scenario 1 is kept for reference only); Remove with ctx Some(c) -> Op::Rm{clock: c, member}; "
                 "Remove with ctx None -> Op::Rm{clock: the witness's contains(member).rm_clock at that point}. "
                 "Assertion: the reference's convergence property over i. Witness sets are folded in index order "
                 "into a new set plus an empty 'defer plunger', on every backend, and compared across backends. "
                 "Generated by tools/make_golden_qc.py."),
        "scenarios": scen,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(OUT, [len(s["witness_sets"]) for s in scen])


if __name__ == "__main__":
    sys.exit(main())
