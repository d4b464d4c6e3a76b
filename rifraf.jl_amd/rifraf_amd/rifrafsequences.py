"""RifrafSequence: a read (or reference) with its per-base FP64 score tables
(src/rifrafsequences.jl:1-108).  Tables are built on the host exactly as the
reference builds them and are uploaded bit-exact to the engine."""
from __future__ import annotations

import math

import numpy as np

from .errormodel import Scores, phred_to_log_p
from .types import DNASeq


def julia_sum(a: np.ndarray) -> float:
    """Julia 0.6 `sum(::Vector{Float64})`: sequential below 16 elements,
    otherwise pairwise with block size 1024 (base/reduce.jl mapreduce_impl)."""
    a = np.asarray(a, dtype=np.float64)
    n = a.shape[0]
    if n == 0:
        return 0.0
    if n == 1:
        return float(a[0])
    if n < 16:
        return float(np.cumsum(a)[-1])

    def impl(lo, hi):  # inclusive
        if lo + 1024 > hi:
            return float(np.cumsum(a[lo:hi + 1])[-1])
        mid = (lo + hi) >> 1
        return impl(lo, mid) + impl(mid + 1, hi)

    return impl(0, n - 1)


def julia_max(x: float, y: float) -> float:
    """Base.max for Float64 (NaN-propagating, +0 > -0)."""
    if math.isnan(x) or math.isnan(y):
        return math.nan
    if y > x or (math.copysign(1.0, y) > math.copysign(1.0, x) and y == x):
        return y
    return x


class RifrafSequence:
    """Mirror of the mutable struct at rifrafsequences.jl:5-17."""

    __slots__ = ("seq", "est_n_errors", "error_log_p", "match_scores", "mismatch_scores",
                 "ins_scores", "del_scores", "codon_ins_scores", "codon_del_scores",
                 "bandwidth", "bandwidth_fixed")

    def __init__(self, seq=None, error_log_p=None, bandwidth: int = 1, scores: Scores | None = None):
        if seq is None:  # empty sequence, rifrafsequences.jl:97-100
            self._empty()
            return
        seq = DNASeq(seq)
        if bandwidth < 1:
            raise ValueError("bandwidth must be positive")
        lp = np.asarray(error_log_p)
        if lp.dtype.kind in "iu":  # Phred constructor, :84-88
            lp = phred_to_log_p(lp)
        lp = np.ascontiguousarray(lp, dtype=np.float64)
        if len(seq) != len(lp):
            raise ValueError("length mismatch")
        if len(seq) == 0:
            self._empty()
            return
        if lp.min() == -math.inf:
            raise ValueError("a log error probability is negative infinity")
        if lp.max() > 0.0:
            raise ValueError(f"a log error probability is > 0: {lp.max()}")
        n = len(lp)
        with np.errstate(divide="ignore"):
            self.match_scores = np.log10(1.0 - np.power(10.0, lp))          # :45
        self.mismatch_scores = lp + scores.mismatch                          # :46
        self.ins_scores = lp + scores.insertion                              # :47
        d = np.empty(n + 1)
        d[0] = lp[0] + scores.deletion                                       # :49
        d[n] = lp[n - 1] + scores.deletion                                   # :50
        if n > 1:
            d[1:n] = np.maximum(lp[:-1], lp[1:]) + scores.deletion            # :51-53
        self.del_scores = d
        self.codon_ins_scores = np.empty(0)
        self.codon_del_scores = np.empty(0)
        if scores.codon_insertion > -math.inf:                               # :57-64
            if n >= 3:
                self.codon_ins_scores = (np.maximum(np.maximum(lp[:-2], lp[1:-1]), lp[2:])
                                         + scores.codon_insertion)
            else:
                self.codon_ins_scores = np.empty(max(n - 2, 0))
        if scores.codon_deletion > -math.inf:                                # :65-72
            cd = np.empty(n + 1)
            cd[0] = lp[0] + scores.codon_deletion
            cd[n] = lp[n - 1] + scores.codon_deletion
            if n > 1:
                cd[1:n] = np.maximum(lp[:-1], lp[1:]) + scores.codon_deletion
            self.codon_del_scores = cd
        self.seq = seq
        self.error_log_p = lp
        self.est_n_errors = julia_sum(np.power(10.0, lp))                    # :74
        self.bandwidth = int(bandwidth)
        self.bandwidth_fixed = False

    def _empty(self):
        self.seq = np.zeros(0, np.uint8)
        self.est_n_errors = 0.0
        self.error_log_p = np.zeros(0)
        self.match_scores = np.zeros(0)
        self.mismatch_scores = np.zeros(0)
        self.ins_scores = np.zeros(0)
        self.del_scores = np.zeros(0)
        self.codon_ins_scores = np.zeros(0)
        self.codon_del_scores = np.zeros(0)
        self.bandwidth = 0
        self.bandwidth_fixed = False

    @classmethod
    def rescored(cls, other: "RifrafSequence", scores: Scores) -> "RifrafSequence":
        """RifrafSequence(seq, scores), rifrafsequences.jl:90-95."""
        r = cls(other.seq, other.error_log_p, other.bandwidth, scores)
        r.bandwidth_fixed = other.bandwidth_fixed
        return r

    def __len__(self):
        return int(self.seq.shape[0])

    def do_codon_ins(self):            # :102
        return len(self.codon_ins_scores) > 0

    def do_codon_del(self):            # :103
        return len(self.codon_del_scores) > 0

    def do_codon_moves(self):          # :104
        return self.do_codon_ins() or self.do_codon_del()
