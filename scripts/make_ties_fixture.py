"""Generate tests/golden/ties.json: a cluster whose candidate proposals tie
exactly (seven homopolymer-equivalent Insertion(p, A) with the same total),
the tied set and the proposal the documented (pos, kind, base) order picks.

The reference iterates a Julia Set (hash order, model.jl:487,496) before the
stable sort of choose_candidates (proposals.jl:104-115); this engine uses the
sorted order.  The fixture pins that behaviour and records that every tied
choice yields the same consensus.  Generated with the oracle engine
(tests/oracle_engine.py, the KAT-pinned C restatement).

This is a SELF-CONSISTENCY pin, not reference parity: the fixture comes from
this repo's own oracle engine, and which tied proposal the reference's Set
order would pick is unknown without Julia (parity on the tie-break is
unpinned).  What is parity-relevant is the fixture's second record: every
tied choice gives the same consensus."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)


def cluster():
    from rifraf_amd.sample import random_seq
    rng = np.random.default_rng(5)
    t = np.concatenate([random_seq(20, rng), np.zeros(5, np.int8), random_seq(20, rng)]).astype(np.int8)
    r = np.concatenate([t[:22], [0], t[22:]]).astype(np.int8)
    return t, [r.copy() for _ in range(4)], [np.full(len(r), 25, np.int8) for _ in range(4)]


def main():
    import rifraf_amd.model as M
    from oracle_engine import OracleEngine
    from rifraf_amd.model import RifrafParams, rifraf
    t, reads, phreds = cluster()
    seen = []
    orig = M.handle_candidates

    def hook(cands, state, run, params):
        seen.append([(int(c.proposal.kind), int(c.proposal.pos), int(c.proposal.base), c.score) for c in cands])
        return orig(cands, state, run, params)
    M.handle_candidates = hook
    try:
        res = rifraf(reads, phreds, consensus=t, params=RifrafParams(max_iters=5, do_alignment_proposals=False),
                     engine=OracleEngine())
    finally:
        M.handle_candidates = orig
    first = seen[0]
    best = max(s for *_, s in first)
    tied = [c for c in first if c[3] == best]
    out = {"template": t.tolist(), "reads": [r.tolist() for r in reads], "phreds": [p.tolist() for p in phreds],
           "params": {"max_iters": 5, "do_alignment_proposals": False},
           "tied": [c[:3] for c in tied], "tied_score": best.hex(), "chosen_first_iteration": tied[0][:3],
           "consensus": np.asarray(res.consensus).tolist()}
    with open(os.path.join(REPO, "tests", "golden", "ties.json"), "w") as f:
        json.dump(out, f)
    print(len(tied), "tied", tied[0])


if __name__ == "__main__":
    main()
