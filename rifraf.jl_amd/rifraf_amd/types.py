"""Sequence / score types (src/types.jl:1-6, src/util.jl:1-5).

DNASeq (BioSequence{DNAAlphabet{2}}) is a numpy uint8 array of 2-bit codes
A=0, C=1, G=2, T=3.  Phred = int8, Score = LogProb = Prob = float64.
"""
from __future__ import annotations

import numpy as np

CODON_LENGTH = 3                      # util.jl:2
BASES = np.array([0, 1, 2, 3], np.uint8)   # util.jl:4 "ACGT"
GAP = 4
_ENC = np.full(256, 255, np.uint8)
for _i, _c in enumerate("ACGT"):
    _ENC[ord(_c)] = _i
    _ENC[ord(_c.lower())] = _i
_DEC = np.frombuffer(b"ACGT-", np.uint8)

Phred = np.int8
MIN_PHRED = 1                          # phred.jl:1
MAX_PHRED = ord("~") - 33              # phred.jl:2


def DNASeq(s="") -> np.ndarray:
    """Encode a string (or pass through a code array) as a DNASeq."""
    if isinstance(s, np.ndarray):
        return np.ascontiguousarray(s, dtype=np.uint8)
    if isinstance(s, (list, tuple)):
        return np.asarray(s, dtype=np.uint8)
    b = np.frombuffer(s.encode("ascii"), np.uint8)
    out = _ENC[b]
    if (out == 255).any():
        raise ValueError(f"invalid DNA symbol in {s!r}")
    return out


def dna_str(seq: np.ndarray) -> str:
    return _DEC[np.asarray(seq, np.uint8)].tobytes().decode("ascii")
