"""FASTA / FASTQ IO (src/fastxio.jl:1-124), Sanger (+33) qualities."""
from __future__ import annotations

import numpy as np

from .types import DNASeq, dna_str


def read_fasta_records(filename):
    """-> list of (identifier, sequence string)."""
    recs, name, chunks = [], None, []
    with open(filename) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line.startswith(">"):
                if name is not None:
                    recs.append((name, "".join(chunks)))
                name, chunks = line[1:].split()[0] if len(line) > 1 else "", []
            else:
                chunks.append(line)
    if name is not None:
        recs.append((name, "".join(chunks)))
    return recs


def read_fasta(filename):
    return [DNASeq(s) for _, s in read_fasta_records(filename)]


def write_fasta(filename, seqs, names=None):
    if not names:
        names = [f"seq_{i + 1}" for i in range(len(seqs))]
    with open(filename, "w") as f:
        for n, s in zip(names, seqs):
            f.write(f">{n}\n{dna_str(s) if isinstance(s, np.ndarray) else s}\n")


def read_fastq_records(filename):
    """-> list of (identifier, sequence, phred int8 array); rejects negative
    qualities like fastxio.jl:64-74."""
    recs = []
    with open(filename) as f:
        lines = [l.rstrip("\n") for l in f]
    i = 0
    while i < len(lines):
        if not lines[i].strip():
            i += 1
            continue
        if not lines[i].startswith("@"):
            raise ValueError(f"bad FASTQ record at line {i + 1}")
        name = lines[i][1:].split()[0]
        seq = lines[i + 1].strip()
        qual = lines[i + 3].strip()
        q = np.frombuffer(qual.encode("ascii"), np.uint8).astype(np.int16) - 33
        if (q < 0).any():
            raise ValueError(f"{name} in {filename} contains negative phred values")
        recs.append((name, seq, q.astype(np.int8)))
        i += 4
    return recs


def read_fastq(filename):
    """-> (seqs, phreds, names) (fastxio.jl:87-98)."""
    recs = read_fastq_records(filename)
    return [DNASeq(s) for _, s, _ in recs], [q for _, _, q in recs], [n for n, _, _ in recs]


def read_fastq_packed(filename):
    """read_fastq with the reads and Phred scores as PackedReads (one buffer
    + offsets each): the form the batched native driver takes without a
    per-read concatenation (batch._wave_native).  -> (seqs, phreds, names)."""
    from .types import PackedReads
    seqs, phreds, names = read_fastq(filename)
    return PackedReads.from_list(seqs, np.uint8), PackedReads.from_list(phreds, np.int8), names


def write_fastq(filename, seqs, phreds, names=None):
    if not names or len(names) != len(seqs):
        names = [f"seq_{i + 1}" for i in range(len(seqs))]
    with open(filename, "w") as f:
        for n, s, q in zip(names, seqs, phreds):
            qs = (np.asarray(q, np.int16) + 33).astype(np.uint8).tobytes().decode("ascii")
            f.write(f"@{n}\n{dna_str(s)}\n+\n{qs}\n")
