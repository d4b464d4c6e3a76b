"""Read simulator (src/sample.jl:1-316) restated with a seeded numpy RNG.

Used to generate the synthetic benchmark / test inputs (configs 2-5 of
BASELINE.json).  Distributions follow the reference (HMM errors with
per-base Beta-distributed template error rates, Exponential Phred offset,
Gaussian Phred-domain jitter); the random stream is numpy's, not Julia's.
The per-base loop of hmm_sample is vectorised for non-codon error models
(reads), which draws the same distribution.
"""
from __future__ import annotations

import numpy as np

from .errormodel import ErrorModel, normalize, p_to_phred

MIN_PROB = 1e-10                       # sample.jl:31
MAX_PROB = 0.5                         # sample.jl:32


def rng_of(seed=None) -> np.random.Generator:
    return seed if isinstance(seed, np.random.Generator) else np.random.default_rng(seed)


def rbase(rng):                                                   # :1-3
    return int(rng.integers(0, 4))


def random_seq(n, rng=None):                                      # :26-28
    return rng_of(rng).integers(0, 4, size=int(n)).astype(np.uint8)


def mutate_bases(bases, rng):
    """mutate_base (:5-11) vectorised: uniform over the three other bases."""
    return ((bases.astype(np.int64) + rng.integers(1, 4, size=len(bases))) % 4).astype(np.uint8)


def mutate_seq(seq, n_diffs, rng):                                # :13-20
    seq = seq.copy()
    for i in rng.integers(0, len(seq), size=n_diffs):
        seq[i] = mutate_bases(seq[i:i + 1], rng)[0]
    return seq


def jitter_phred_domain(x, phred_std, rng):                       # :35-42
    error = rng.standard_normal(len(x)) * phred_std / 10.0
    result = np.power(10.0, np.log10(x) + error)
    return np.clip(result, MIN_PROB, MAX_PROB)


def hmm_sample(sequence, error_p, errors: ErrorModel, rng):       # :44-123
    errors = normalize(errors)
    codon = errors.codon_insertion > 0.0 or errors.codon_deletion > 0.0
    if codon and (errors.insertion > 0.0 or errors.deletion > 0.0):
        raise ValueError("codon and non-codon indels are not both allowed")
    sub_ratio = errors.mismatch
    ins_ratio = errors.codon_insertion if codon else errors.insertion
    del_ratio = errors.codon_deletion if codon else errors.deletion
    L = len(sequence)
    if codon:
        return _hmm_sample_codon(sequence, error_p, sub_ratio, ins_ratio, del_ratio, rng)
    # non-codon: independent events per position (skip is always 0)
    p = np.concatenate([error_p, error_p[-1:]])               # i = 1..L+1
    prev_p = np.concatenate([error_p[:1], error_p])
    max_p = np.maximum(p, prev_p)
    ins = rng.random(L + 1) < max_p * ins_ratio
    dele = rng.random(L) < error_p * del_ratio
    sub = rng.random(L) < error_p * sub_ratio
    ins_bases = rng.integers(0, 4, size=L + 1).astype(np.uint8)
    mutated = mutate_bases(sequence, rng)
    out_bases, out_p, sbools, tbools = [], [], [], []
    # assemble in order: [insertion before i] then base i
    keep = ~dele
    base_i = np.where(sub, mutated, sequence)
    # interleave via index arrays
    nins = int(ins.sum())
    nkeep = int(keep.sum())
    total = nins + nkeep
    order_key = np.concatenate([np.nonzero(ins)[0] * 2, np.nonzero(keep)[0] * 2 + 1])
    vals = np.concatenate([ins_bases[ins], base_i[keep]])
    probs = np.concatenate([max_p[ins], error_p[keep]])
    sb = np.concatenate([np.zeros(nins, bool), ~sub[keep]])
    idx = np.argsort(order_key, kind="stable")
    seq = vals[idx].astype(np.uint8)
    final_p = probs[idx]
    seqbools = sb[idx]
    tb = np.where(dele, False, ~sub)
    assert seq.shape[0] == total
    return seq, final_p, seqbools, tb


def _hmm_sample_codon(sequence, error_p, sub_ratio, ins_ratio, del_ratio, rng):
    final_seq, final_p, seqbools, tbools = [], [], [], []
    skip = 0
    L = len(sequence)
    for i in range(1, L + 2):
        p = error_p[i - 2] if i > L else error_p[i - 1]
        prev_p = error_p[0] if i == 1 else error_p[i - 2]
        max_p = max(p, prev_p)
        ins_p = max_p * ins_ratio / 3.0
        if rng.random() < ins_p:
            final_seq.extend(rng.integers(0, 4, size=3).tolist())
            final_p.extend([max_p] * 3)
            seqbools.extend([False] * 3)
        if i > L:
            break
        if skip > 0:
            skip -= 1
            continue
        del_p = 0.0 if i > L - 2 else max(error_p[i - 1:i + 2]) * del_ratio / 3.0
        if rng.random() < del_p:
            skip = 2
            tbools.extend([False] * 3)
        else:
            if rng.random() < p * sub_ratio:
                final_seq.append(int(mutate_bases(sequence[i - 1:i], rng)[0]))
                seqbools.append(False)
                tbools.append(False)
            else:
                final_seq.append(int(sequence[i - 1]))
                seqbools.append(True)
                tbools.append(True)
            final_p.append(p)
    return (np.array(final_seq, np.uint8), np.array(final_p), np.array(seqbools, bool),
            np.array(tbools, bool))


def sample_reference(template, error_rate, errors: ErrorModel, rng=None):   # :125-144
    rng = rng_of(rng)
    e = normalize(errors)
    if e.insertion > 0.0 or e.deletion > 0.0:
        raise ValueError("non-codon indels are not allowed in reference")
    error_p = error_rate * np.ones(len(template))
    reference, _, _, _ = hmm_sample(template, error_p, errors, rng)
    if len(reference) % 3 == 1:
        idx = int(rng.integers(0, len(reference)))
        reference = np.concatenate([reference[:idx], reference[idx + 1:]])
    elif len(reference) % 3 == 2:
        idx = int(rng.integers(0, len(reference) + 1))
        reference = np.concatenate([reference[:idx], np.array([rbase(rng)], np.uint8), reference[idx:]])
    return reference.astype(np.uint8)


def sample_from_template(template, template_error_p, errors: ErrorModel, phred_scale,
                         actual_std, reported_std, rng=None):           # :146-171
    rng = rng_of(rng)
    e = normalize(errors)
    if e.codon_insertion > 0.0 or e.codon_deletion > 0.0:
        raise ValueError("codon indels are not allowed in sequences")
    offset = rng.exponential(phred_scale)
    base_vector = np.power(10.0, (-10.0 * np.log10(template_error_p) + offset) / (-10.0))
    jittered = jitter_phred_domain(base_vector, actual_std, rng)
    seq, actual_error_p, sbools, tbools = hmm_sample(template, jittered, errors, rng)
    reported = jitter_phred_domain(actual_error_p, reported_std, rng)
    phreds = p_to_phred(reported)
    return seq, actual_error_p, phreds, sbools, tbools


def sample_mixture(nseqs, length, n_diffs, ref_error_rate=0.1,
                   ref_errors=ErrorModel(10, 0, 0, 1, 0), error_rate=0.01, alpha=0.1,
                   phred_scale=1.5, actual_std=3.0, reported_std=1.0,
                   seq_errors=ErrorModel(1, 5, 5), rng=None):           # :173-220
    rng = rng_of(rng)
    template1 = random_seq(length, rng)
    template2 = mutate_seq(template1, n_diffs, rng)
    templates = [template1, template2]
    reference = sample_reference(template1, ref_error_rate, ref_errors, rng)
    beta = alpha * (error_rate - MAX_PROB) / (MIN_PROB - error_rate)
    template_error_p = rng.beta(alpha, beta, size=length) * (MAX_PROB - MIN_PROB) + MIN_PROB
    seqs, actual_ps, phreds, sb, tb = [], [], [], [], []
    for t, n in zip(templates, nseqs):
        for _ in range(n):
            s, a, ph, c, d = sample_from_template(t, template_error_p, seq_errors, phred_scale,
                                                  actual_std, reported_std, rng)
            seqs.append(s)
            actual_ps.append(a)
            phreds.append(ph)
            sb.append(c)
            tb.append(d)
    return reference, templates, template_error_p, seqs, actual_ps, phreds, sb, tb


def sample_sequences(nseqs=3, length=90, ref_error_rate=0.1, ref_errors=ErrorModel(10, 0, 0, 1, 1),
                     error_rate=0.01, alpha=0.1, phred_scale=1.5, actual_std=3.0, reported_std=1.0,
                     seq_errors=ErrorModel(1, 5, 5), rng=None):        # :277-298
    """Returns (reference, template, template_error_p, seqs, actual, phreds,
    seqbools, tbools) like the reference."""
    ref, templates, t_p, seqs, actual, phreds, cb, db = sample_mixture(
        (nseqs, 0), length, 0, ref_error_rate=ref_error_rate, ref_errors=ref_errors,
        error_rate=error_rate, alpha=alpha, phred_scale=phred_scale, actual_std=actual_std,
        reported_std=reported_std, seq_errors=seq_errors, rng=rng)
    return ref, templates[0], t_p, seqs, actual, phreds, cb, db
