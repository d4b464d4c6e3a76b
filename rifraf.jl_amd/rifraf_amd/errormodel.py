"""ErrorModel / Scores (src/errormodel.jl:1-81) and phred helpers
(src/phred.jl:1-41).  Host-side parameters: their values flow bit-exact into
the per-read score tables the engine consumes."""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .types import MAX_PHRED


@dataclass(frozen=True)
class ErrorModel:
    """Relative error rates (errormodel.jl:19-30)."""
    mismatch: float
    insertion: float
    deletion: float
    codon_insertion: float = 0.0
    codon_deletion: float = 0.0

    def args(self):
        return [self.mismatch, self.insertion, self.deletion, self.codon_insertion,
                self.codon_deletion]


def normalize(parts):
    """phred.jl:38-41 / errormodel.jl:33-41: parts / sum(parts) (left fold sum)."""
    if isinstance(parts, ErrorModel):
        return ErrorModel(*normalize(parts.args()))
    total = 0.0
    for p in parts:
        total += float(p)
    return [float(p) / total for p in parts]


def _log10(x: float) -> float:
    return -math.inf if x == 0.0 else math.log10(x)


@dataclass(frozen=True)
class Scores:
    """log10 alignment scores (errormodel.jl:43-49)."""
    mismatch: float
    insertion: float
    deletion: float
    codon_insertion: float
    codon_deletion: float

    @staticmethod
    def from_errors(errors: ErrorModel, mismatch=0.0, insertion=0.0, deletion=0.0) -> "Scores":
        """Scores(errors; mismatch, insertion, deletion), errormodel.jl:66-81."""
        m, i, d, ci, cd = (_log10(x) for x in normalize(errors.args()))
        return Scores(m + mismatch, i + insertion, d + deletion, ci + 3 * insertion,
                      cd + 3 * deletion)


def phred_to_log_p(x):
    """phred.jl:14-18: x / (-10.0)."""
    return np.asarray(x, dtype=np.float64) / (-10.0)


def phred_to_p(x):
    return np.power(10.0, phred_to_log_p(x))


def p_to_phred(p):
    """phred.jl:5-8: min(round(-10 log10 p), MAX_PHRED) (round half to even)."""
    p = np.asarray(p, dtype=np.float64)
    return np.minimum(np.round(-10.0 * np.log10(p)), MAX_PHRED).astype(np.int8)


def cap_phreds(phreds, max_phred: int):
    """phred.jl:35-41."""
    if max_phred < 1:
        raise ValueError("max phred value must be positive")
    return np.minimum(np.asarray(phreds, np.int8), np.int8(max_phred))
