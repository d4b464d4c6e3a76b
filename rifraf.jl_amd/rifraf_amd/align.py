"""Pairwise alignment API (src/align.jl).

The DP fills (forward!, forward_moves!, backward!) and backtraces run on the
HIP engine (rf_realign / rf_backtrace).  The move-list helpers below
(moves_to_aligned_seqs, moves_to_indices, moves_to_proposals) are host-side
bookkeeping over the engine's move lists, as in the reference.
"""
from __future__ import annotations

import math

import numpy as np

from .errormodel import ErrorModel, Scores
from .proposals import Deletion, Insertion, Substitution
from .rifrafsequences import RifrafSequence
from .types import DNASeq, dna_str

TRACE_NONE, TRACE_MATCH, TRACE_INSERT, TRACE_DELETE, TRACE_CODON_INSERT, TRACE_CODON_DELETE = range(6)
OFFSETS = {1: (1, 1), 2: (1, 0), 3: (0, 1), 4: (3, 0), 5: (0, 3)}   # align.jl:14-18

_ENGINE = None


def default_engine():
    """Process-wide engine for one-off alignments (device 0, or LOCAL_RANK)."""
    global _ENGINE
    if _ENGINE is None:
        import os

        from .engine import Engine
        _ENGINE = Engine(int(os.environ.get("RIFRAF_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    return _ENGINE


class Scratch:
    """Sequence / template / slot ids an engine reserves for one-off work."""

    def __init__(self, engine=None, seq_id=0, tpl_id=0, slot=0):
        self.engine = engine or default_engine()
        self.seq_id, self.tpl_id, self.slot = seq_id, tpl_id, slot


def _run(t, s: RifrafSequence, flags, scratch: Scratch | None):
    from .engine import RF_BWD, RF_FWD  # noqa: F401
    sc = scratch or Scratch()
    e = sc.engine
    e.set_sequences(sc.seq_id, [s])
    e.set_templates(sc.tpl_id, [DNASeq(t)])
    score = e.realign([sc.slot], [sc.seq_id], [sc.tpl_id], [s.bandwidth], flags)
    return sc, score[0]


def forward_moves(t, s: RifrafSequence, trim=False, skew_matches=False, scratch=None):
    """align.jl:144-153: (A, moves).  A is downloaded; moves come from the
    device backtrace (the trace is recomputed from A)."""
    from .engine import RF_BAND_A, RF_FWD, RF_SKEW, RF_TRIM
    flags = RF_FWD | (RF_SKEW if skew_matches else 0) | (RF_TRIM if trim else 0)
    sc, _ = _run(t, s, flags, scratch)
    A = sc.engine.download_band(sc.slot, RF_BAND_A)
    moves, _ = sc.engine.backtrace([sc.slot])
    return A, moves[0]


def forward(t, s: RifrafSequence, scratch=None):
    """align.jl:185-194 F[i, j]: log probability of s[1:i-1] vs t[1:j-1]."""
    from .engine import RF_BAND_A, RF_FWD
    sc, _ = _run(t, s, RF_FWD, scratch)
    return sc.engine.download_band(sc.slot, RF_BAND_A)


def backward(t, s: RifrafSequence, scratch=None):
    """align.jl:208-212 B[i, j]: log probability of s[i:end] vs t[j:end]."""
    from .engine import RF_BAND_B, RF_BWD
    sc, _ = _run(t, s, RF_BWD, scratch)
    return sc.engine.download_band(sc.slot, RF_BAND_B)


def align_moves(t, s: RifrafSequence, trim=False, skew_matches=False, scratch=None):
    """align.jl:337-344"""
    from .engine import RF_FWD, RF_SKEW, RF_TRIM
    flags = RF_FWD | (RF_SKEW if skew_matches else 0) | (RF_TRIM if trim else 0)
    sc, _ = _run(t, s, flags, scratch)
    moves, _ = sc.engine.backtrace([sc.slot])
    return moves[0]


def align(t, s: RifrafSequence, trim=False, skew_matches=False, scratch=None):
    """align.jl:346-353 -> (aligned t, aligned s) strings with '-' gaps."""
    moves = align_moves(t, s, trim=trim, skew_matches=skew_matches, scratch=scratch)
    return moves_to_aligned_seqs(moves, DNASeq(t), s.seq)


def count_errors(t, s: RifrafSequence, scratch=None):
    """align.jl:247-250: errors of the skewed alignment."""
    from .engine import RF_FWD, RF_SKEW
    sc, _ = _run(t, s, RF_FWD | RF_SKEW, scratch)
    _, nerr = sc.engine.backtrace([sc.slot], want_moves=False)
    return int(nerr[0])


def edit_distance(t, s, scratch=None):
    """align.jl:253-260: skewed alignment with bandwidth ceil(0.5 min(len))."""
    t = DNASeq(t)
    s = DNASeq(s)
    log_ps = np.full(len(s), -1.0)
    bandwidth = int(math.ceil(min(len(t), len(s)) * 0.5))
    scores = Scores.from_errors(ErrorModel(1.0, 1.0, 1.0))
    seq = RifrafSequence(s, log_ps, bandwidth, scores)
    return count_errors(t, seq, scratch=scratch)


# ---------------------------------------------------------------------
# host bookkeeping over move lists
# ---------------------------------------------------------------------

def moves_to_aligned_seqs(moves, t, s):                           # align.jl:286-311
    at, as_ = [], []
    i = j = 0
    tt, ss = dna_str(t), dna_str(s)
    for mv in moves:
        a, b = OFFSETS[int(mv)]
        i, j = i + a, j + b
        if mv == TRACE_MATCH:
            at.append(tt[j - 1])
            as_.append(ss[i - 1])
        elif mv == TRACE_INSERT:
            at.append("-")
            as_.append(ss[i - 1])
        elif mv == TRACE_DELETE:
            at.append(tt[j - 1])
            as_.append("-")
        elif mv == TRACE_CODON_INSERT:
            at.append("---")
            as_.append(ss[i - 3:i])
        elif mv == TRACE_CODON_DELETE:
            at.append(tt[j - 3:j])
            as_.append("---")
    return "".join(at), "".join(as_)


def moves_to_indices(moves, tlen, slen):                          # align.jl:322-335
    result = []
    i = j = 0
    last_j = 0
    for mv in moves:
        a, b = OFFSETS[int(mv)]
        i, j = i + a, j + b
        if j > last_j:
            result.append(i)
            last_j = j
    return result


def moves_to_proposals(moves, consensus, seq: RifrafSequence):   # model.jl:458-480
    """Substitutions / insertions / deletions seen in one read's alignment."""
    props = []
    i = j = 0
    s = seq.seq
    for mv in moves:
        mv = int(mv)
        a, b = OFFSETS[mv]
        i, j = i + a, j + b
        if mv == TRACE_MATCH:
            if s[i - 1] != consensus[j - 1]:
                props.append(Substitution(j, int(s[i - 1])))
        elif mv == TRACE_INSERT:
            props.append(Insertion(j, int(s[i - 1])))
        elif mv == TRACE_DELETE:
            props.append(Deletion(j))
    return props


def moves_to_proposals_np(moves, consensus, s):
    """Vectorised moves_to_proposals -> (kind, pos, base) integer arrays."""
    mv = np.asarray(moves, np.int64)
    di = np.where((mv == 1) | (mv == 2), 1, np.where(mv == 4, 3, 0))
    dj = np.where((mv == 1) | (mv == 3), 1, np.where(mv == 5, 3, 0))
    i = np.cumsum(di)
    j = np.cumsum(dj)
    sub = (mv == 1) & (s[np.maximum(i - 1, 0)] != consensus[np.maximum(j - 1, 0)])
    ins = mv == 2
    dele = mv == 3
    keep = sub | ins | dele
    kind = np.where(sub, 0, np.where(ins, 1, 2))[keep]
    pos = j[keep]
    base = np.where(dele, 0, s[np.maximum(i - 1, 0)])[keep]
    return kind, pos, base
