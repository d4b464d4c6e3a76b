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


class PackedReads:
    """A read set held as one contiguous array plus offsets: a sequence of
    per-read views (len / indexing / iteration give numpy views, so any
    consumer of a list of reads takes it unchanged).  The batched driver
    reads `buf` and `off` directly instead of concatenating thousands of
    small arrays (batch._wave_native): FASTQ ingest and bench's e2e staging
    hand clusters over in this form."""

    __slots__ = ("buf", "off")

    def __init__(self, buf, off):
        self.buf = np.ascontiguousarray(buf)
        self.off = np.ascontiguousarray(off, np.int64)
        if self.off.ndim != 1 or len(self.off) < 1 or self.off[0] != 0 or self.off[-1] != len(self.buf) \
                or (np.diff(self.off) < 0).any():
            raise ValueError("PackedReads: offsets must rise from 0 to len(buf)")

    @classmethod
    def from_list(cls, arrs, dtype):
        arrs = [np.asarray(a, dtype) for a in arrs]
        off = np.zeros(len(arrs) + 1, np.int64)
        np.cumsum([len(a) for a in arrs], out=off[1:])
        return cls(np.concatenate(arrs) if arrs else np.zeros(0, dtype), off)

    def lens(self):
        return np.diff(self.off)

    def __len__(self):
        return len(self.off) - 1

    def __getitem__(self, k):
        if isinstance(k, slice):
            return [self[i] for i in range(*k.indices(len(self)))]
        n = len(self)
        if k < 0:
            k += n
        if not 0 <= k < n:
            raise IndexError(k)
        return self.buf[self.off[k]:self.off[k + 1]]

    def __iter__(self):
        b, o = self.buf, self.off.tolist()
        return (b[o[k]:o[k + 1]] for k in range(len(o) - 1))
