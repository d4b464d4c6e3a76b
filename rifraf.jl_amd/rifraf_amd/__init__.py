"""rifraf_amd -- host mirror of Rifraf.jl's API over the MI355X hot-path engine.

The hot path (banded forward/backward DP, backtrace, proposal scoring) runs
in the HIP kernels of librifraf_hip.so (rifraf.jl_amd/csrc/), reached through
the C-ABI in include/rifraf_hip.h.  This package mirrors the reference's
interface (src/Rifraf.jl:12-45): rifraf(), RifrafParams, RifrafResult,
ErrorModel, Scores, RifrafSequence, BandedArray, the sampler and FASTX IO.
"""
from .bandedarrays import BandedArray, equal_ranges, ndatarows
from .errormodel import ErrorModel, Scores, cap_phreds, normalize, p_to_phred, phred_to_log_p, phred_to_p
from .proposals import (AmbiguousProposalsError, Deletion, Insertion, Proposal, ScoredProposal,
                        Substitution, apply_proposals, choose_candidates)
from .rifrafsequences import RifrafSequence
from .types import BASES, CODON_LENGTH, DNASeq, dna_str

__all__ = ["BandedArray", "equal_ranges", "ndatarows", "ErrorModel", "Scores", "cap_phreds",
           "normalize", "p_to_phred", "phred_to_log_p", "phred_to_p", "AmbiguousProposalsError",
           "Deletion", "Insertion", "Proposal", "ScoredProposal", "Substitution", "apply_proposals",
           "choose_candidates", "RifrafSequence", "BASES", "CODON_LENGTH", "DNASeq", "dna_str"]


def __getattr__(name):
    # engine-backed API is imported lazily so that host-only use (tests of
    # the host mirror, data generation) never needs the GPU library
    if name in ("Engine", "RifrafError"):
        from . import engine
        return getattr(engine, name)
    if name in ("rifraf", "RifrafParams", "RifrafResult", "RifrafState", "correct_shifts",
                "calibrate_phreds"):
        from . import model
        return getattr(model, name)
    if name in ("align", "align_moves", "forward", "backward", "forward_moves", "edit_distance"):
        from . import align
        return getattr(align, name)
    if name in ("sample_sequences", "sample_mixture", "sample_from_template", "sample_reference",
                "random_seq"):
        from . import sample
        return getattr(sample, name)
    if name in ("read_fasta", "read_fastq", "write_fasta", "write_fastq"):
        from . import fastxio
        return getattr(fastxio, name)
    raise AttributeError(name)
