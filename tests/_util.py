"""Shared helpers for the parity tests (engine vs oracle)."""
import numpy as np

from rifraf_amd import ErrorModel, RifrafSequence, Scores
from rifraf_amd.proposals import DEL, INS, SUB
from rifraf_amd.sample import random_seq, sample_from_template

SEQ_SCORES = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0))      # model.jl:98
REF_SCORES = Scores.from_errors(ErrorModel(10.0, 1e-1, 1e-1, 1.0, 1.0))   # model.jl:99


def make_read(template, rng, error_rate=0.02, bandwidth=9, scores=SEQ_SCORES,
              seq_errors=ErrorModel(1, 5, 5)):
    s, _, ph, _, _ = sample_from_template(template, np.full(len(template), error_rate), seq_errors,
                                          1.5, 1.0, 0.3, rng)
    if len(s) == 0:
        s, ph = template[:1].copy(), np.array([20], np.int8)
    return RifrafSequence(s, ph.astype(np.float64) / -10.0, bandwidth, scores)


def inband_mask(nrows, ncols, bw):
    """(H, ncols) boolean mask of the in-band data entries (row_range)."""
    H = 2 * bw + abs(nrows - ncols) + 1
    h_off = max(ncols - nrows, 0)
    v_off = max(nrows - ncols, 0)
    mask = np.zeros((H, ncols), bool)
    for j in range(1, ncols + 1):
        a = max(1, j - h_off - bw)
        b = min(j + v_off + bw, nrows)
        mask[a - j + h_off + bw: b - j + h_off + bw + 1, j - 1] = True
    return mask


def all_proposals_arrays(template):
    """STAGE_SCORE all_proposals (model.jl:401-456), no seeds, as arrays."""
    m = len(template)
    k, p, b = [INS] * 4, [0] * 4, [0, 1, 2, 3]
    for j in range(1, m + 1):
        for base in range(4):
            if template[j - 1] != base:
                k.append(SUB); p.append(j); b.append(base)
        k.append(DEL); p.append(j); b.append(0)
        for base in range(4):
            k.append(INS); p.append(j); b.append(base)
    return np.array(k, np.uint8), np.array(p, np.int32), np.array(b, np.uint8)


def dense_slot(kind, base):
    return np.where(kind == SUB, base, np.where(kind == DEL, 4, 5 + base))


__all__ = ["make_read", "inband_mask", "all_proposals_arrays", "dense_slot", "random_seq",
           "SEQ_SCORES", "REF_SCORES"]
