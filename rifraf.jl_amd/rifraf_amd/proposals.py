"""Proposal types and host-side proposal logic (src/proposals.jl:1-115).

The proposal *types* are the wire format to the engine's scorer
(kind 0 = Substitution, 1 = Insertion, 2 = Deletion; 1-based positions).
apply_proposals / choose_candidates stay on the host (O(P log P))."""
from __future__ import annotations

from typing import NamedTuple

import numpy as np

SUB, INS, DEL = 0, 1, 2


class Proposal(NamedTuple):
    kind: int
    pos: int
    base: int = 0

    def __repr__(self):
        b = "ACGT"[self.base]
        return {SUB: f"Substitution({self.pos}, {b})", INS: f"Insertion({self.pos}, {b})",
                DEL: f"Deletion({self.pos})"}[self.kind]


def Substitution(pos: int, base: int) -> Proposal:
    return Proposal(SUB, int(pos), int(base))


def Insertion(pos: int, base: int) -> Proposal:
    return Proposal(INS, int(pos), int(base))


def Deletion(pos: int) -> Proposal:
    return Proposal(DEL, int(pos), 0)


class ScoredProposal(NamedTuple):
    proposal: Proposal
    score: float


class AmbiguousProposalsError(Exception):
    """proposals.jl:77"""


def are_ambiguous(ms) -> bool:                                     # :41-56
    ins_positions = [m.pos for m in ms if m.kind == INS]
    other_positions = [m.pos for m in ms if m.kind != INS]
    ins_good = len(set(ins_positions)) == len(ins_positions)
    others_good = len(set(other_positions)) == len(other_positions)
    return not ins_good or not others_good


def apply_proposals(seq: np.ndarray, proposals) -> np.ndarray:     # :80-102
    if are_ambiguous(proposals):
        raise AmbiguousProposalsError()
    result = []
    nxt = 1
    last_del_pos = 0
    # stable sort by (pos, deletions first), proposals.jl:91
    for p in sorted(proposals, key=lambda p: (p.pos, 0 if p.kind == DEL else 1)):
        result.append(seq[nxt - 1:max(p.pos - 1, 0)])  # Julia seq[1:-1] is empty
        if p.kind == SUB:                                          # :58-61
            result.append(np.array([p.base], np.uint8))
        elif p.kind == INS:                                        # :63-69
            if p.pos > 0 and last_del_pos != p.pos:
                result.append(np.array([seq[p.pos - 1], p.base], np.uint8))
            else:
                result.append(np.array([p.base], np.uint8))
        nxt = p.pos + 1
        if p.kind == DEL:
            last_del_pos = p.pos
    result.append(seq[nxt - 1:])
    return np.concatenate(result).astype(np.uint8) if result else np.zeros(0, np.uint8)


def choose_candidates(candidates, min_dist: int):                  # :104-115
    final_cands = []
    posns = []
    # Julia sort(..., by=score, rev=true) is a stable merge sort
    for c in sorted(candidates, key=lambda c: -c.score):
        if any(abs(c.proposal.pos - p) < min_dist for p in posns):
            continue
        posns.append(c.proposal.pos)
        final_cands.append(c)
    return final_cands


def to_arrays(props):
    """Proposal list -> (kind u8, pos i32, base u8) arrays for rf_score."""
    n = len(props)
    if n == 0:
        return np.zeros(0, np.uint8), np.zeros(0, np.int32), np.zeros(0, np.uint8)
    a = np.array(props, dtype=np.int64).reshape(n, 3)
    return (np.ascontiguousarray(a[:, 0], np.uint8), np.ascontiguousarray(a[:, 1], np.int32),
            np.ascontiguousarray(a[:, 2], np.uint8))
