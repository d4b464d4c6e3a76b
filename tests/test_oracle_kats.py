"""Pin the CPU oracle (oracle/rifraf_oracle.c) against the reference's own
known-answer and property tests.  Each test cites the Julia test it restates.

These run on CPU (no GPU): they establish that the oracle -- the checker for
the HIP engine -- computes what Rifraf.jl computes.
"""
import math

import numpy as np
import pytest

import oracle
from rifraf_amd import (BandedArray, Deletion, ErrorModel, Insertion, RifrafSequence, Scores,
                        Substitution, apply_proposals, DNASeq)
from rifraf_amd.align import moves_to_aligned_seqs, moves_to_indices
from rifraf_amd.errormodel import normalize
from rifraf_amd.sample import random_seq, rbase, sample_from_template


def inv_log10(x):                       # test_utils.jl:1-3
    return math.log10(1.0 - 10.0 ** x)


def fwd(t, s, **kw):
    data, mv = oracle.forward(DNASeq(t), s, **kw)
    A = BandedArray((len(s) + 1, len(t) + 1), s.bandwidth, default=-np.inf, data=np.asfortranarray(data))
    return A, mv


def bwd(t, s):
    data = oracle.backward(DNASeq(t), s)
    return BandedArray((len(s) + 1, len(t) + 1), s.bandwidth, default=-np.inf, data=np.asfortranarray(data))


def check_all_cols(A, B, codon_moves):  # test_utils.jl:6-23
    assert A[A.nrows, A.ncols] == pytest.approx(B[1, 1])
    expected = A[A.nrows, A.ncols]
    FA, FB = A.full(), B.full()
    # out-of-band cells are zeros in full(); the reference test relies on the
    # in-band maximum dominating, which holds for these scores
    for j in range(A.ncols - (2 if codon_moves else 0)):
        cols = slice(j, j + 3) if codon_moves else slice(j, j + 1)
        mask = np.zeros_like(FA, dtype=bool)
        for jj in range(cols.start, cols.stop):
            a, b = A.row_range(jj + 1)
            mask[a - 1:b, jj] = True
        score = (FA + FB)[mask].max()
        assert score == pytest.approx(expected)


SC = Scores(-1.0, -1.0, -1.0, -math.inf, -math.inf)


class TestForwardBackward:          # test_align.jl:16-181
    def test_perfect_forward(self):
        lp = -3.0
        match = inv_log10(lp)
        pseq = RifrafSequence(DNASeq("AA"), np.full(2, lp), 1, SC)
        A, _ = fwd("AA", pseq)
        expected = np.array([[0.0, lp + SC.deletion, 0.0],
                             [lp + SC.insertion, match, match + lp + SC.deletion],
                             [0.0, match + lp + SC.insertion, 2 * match]])
        np.testing.assert_allclose(A.full(), expected)
        A2, _ = fwd("AA", pseq, moves=True)
        np.testing.assert_array_equal(A2.full(), A.full())

    def test_perfect_backward(self):
        lp = -3.0
        match = inv_log10(lp)
        pseq = RifrafSequence(DNASeq("AA"), np.full(2, lp), 1, SC)
        B = bwd("AA", pseq)
        expected = np.array([[2 * match, match + lp + SC.insertion, 0.0],
                             [match + lp + SC.deletion, match, lp + SC.insertion],
                             [0.0, lp + SC.deletion, 0.0]])
        np.testing.assert_allclose(B.full(), expected)

    def test_imperfect_forward(self):
        lp = -3.0
        match = inv_log10(lp)
        pseq = RifrafSequence(DNASeq("AT"), np.full(2, lp), 1, SC)
        A1, _ = fwd("AA", pseq)
        B = bwd("AA", pseq)
        check_all_cols(A1, B, False)
        expected = np.array([[0.0, lp + SC.deletion, 0.0],
                             [lp + SC.insertion, match, match + lp + SC.deletion],
                             [0.0, match + lp + SC.insertion, match + lp + SC.mismatch]])
        np.testing.assert_allclose(A1.full(), expected, atol=0.01)

    def test_imperfect_backward(self):
        lp = -3.0
        match = inv_log10(lp)
        pseq = RifrafSequence(DNASeq("AT"), np.full(2, lp), 1, SC)
        B = bwd("AA", pseq)
        expected = np.array([[lp + SC.mismatch + match, lp + SC.insertion + match, 0.0],
                             [2 * lp + SC.deletion + SC.mismatch, lp + SC.mismatch, lp + SC.insertion],
                             [0.0, lp + SC.deletion, 0.0]])
        np.testing.assert_allclose(B.full(), expected, atol=0.01)

    @pytest.mark.parametrize("t,s,lp", [("TG", "GTCG", [-1.2, -0.8, -0.7, -1.0]),
                                        ("GCACGGTC", "GACAC", [-1.1, -1.1, -0.4, -1.0, -0.7])])
    def test_agreement_codon(self, t, s, lp):
        sc = Scores.from_errors(ErrorModel(2.0, 1.0, 1.0, 3.0, 3.0))
        pseq = RifrafSequence(DNASeq(s), np.array(lp), 5, sc)
        A, _ = fwd(t, pseq)
        B = bwd(t, pseq)
        check_all_cols(A, B, True)
        A2, _ = fwd(t, pseq, moves=True)
        np.testing.assert_array_equal(A.full(), A2.full())

    def test_insertion_agreement(self):
        lp = np.array([-5.0, -1.0, -6.0])
        pseq = RifrafSequence(DNASeq("ATA"), lp, 10, SC)
        A, _ = fwd("AA", pseq)
        B = bwd("AA", pseq)
        score = inv_log10(lp[0]) + lp[1] + SC.insertion + inv_log10(lp[2])
        assert A[A.nrows, A.ncols] == pytest.approx(score)
        check_all_cols(A, B, False)

    def test_deletion_agreement_1(self):
        pseq = RifrafSequence(DNASeq("GAAG"), np.array([-5.0, -2.0, -1.0, -6.0]), 10, SC)
        A, _ = fwd("GATAG", pseq)
        B = bwd("GATAG", pseq)
        m, d = pseq.match_scores, pseq.del_scores
        assert A[A.nrows, A.ncols] == pytest.approx(m[0] + m[1] + d[2] + m[2] + m[3])
        check_all_cols(A, B, False)

    def test_deletion_agreement_2(self):
        pseq = RifrafSequence(DNASeq("AA"), np.array([-2.0, -3.0]), 10, SC)
        A, _ = fwd("ATA", pseq)
        B = bwd("ATA", pseq)
        m, d = pseq.match_scores, pseq.del_scores
        assert A[A.nrows, A.ncols] == pytest.approx(m[0] + d[1] + m[1])
        check_all_cols(A, B, False)


def align_moves(t, s, skew=False):
    A, mv = fwd(t, s, moves=True, skew=skew)
    return oracle.backtrace(mv, A.nrows, A.ncols, A.bandwidth)


class TestAlignment:                 # test_align.jl:183-284
    scores = Scores.from_errors(normalize(ErrorModel(1.0, 1.0, 1.0, 0.0, 0.0)))

    def test_align_1(self):
        pseq = RifrafSequence(DNASeq("AAA"), np.array([-2.0, -3.0, -3.0]), 10, self.scores)
        t, s = moves_to_aligned_seqs(align_moves("ATAA", pseq), DNASeq("ATAA"), pseq.seq)
        assert (t, s) == ("ATAA", "A-AA")

    def test_align_2(self):
        seq = DNASeq("AAACCCTT")
        pseq = RifrafSequence(seq, np.full(len(seq), math.log10(0.1)), 10, self.scores)
        t, s = moves_to_aligned_seqs(align_moves("AACCTT", pseq), DNASeq("AACCTT"), seq)
        assert t[-2:] == "TT"

    @pytest.mark.parametrize("t,s,expected", [("AAA", "AAA", [1, 2, 3]), ("AAA", "AAAT", [1, 2, 3]),
                                              ("AAAT", "AAA", [1, 2, 3, 3]), ("TAAA", "AAA", [0, 1, 2, 3])])
    def test_moves_to_indices(self, t, s, expected):
        pseq = RifrafSequence(DNASeq(s), np.full(len(s), math.log10(0.1)), 10, self.scores)
        assert moves_to_indices(align_moves(t, pseq), len(t), len(s)) == expected

    def test_align_and_skew(self):
        ref_scores = Scores.from_errors(ErrorModel(10.0, 1e-10, 1e-10, 1.0, 1.0))
        cons = RifrafSequence(DNASeq("CTGCCGA"), np.array([-8., -8., -8., -1., -8., -10., -10.]), 10,
                              ref_scores)
        a, b = moves_to_aligned_seqs(align_moves("CGGCGATTT", cons, skew=True), DNASeq("CGGCGATTT"),
                                     cons.seq)
        assert (a, b) == ("CGG-CGATTT", "CTGCCGA---")

    def test_align_with_self(self):
        seq = DNASeq("AAAGGGTTTCCC")
        errors = np.full(len(seq), 0.1)
        errors[:6] = 0.3
        errors[-4:] = 0.45
        rseq = RifrafSequence(seq, np.log10(errors), 3, Scores.from_errors(ErrorModel(1.0, 10.0, 10.0, 0.0, 0.0)))
        a, b = moves_to_aligned_seqs(align_moves(seq, rseq), seq, seq)
        assert a == b == "AAAGGGTTTCCC"


class TestTables:                    # test_rifrafsequences.jl:13-51
    def test_scores(self):
        lp = np.array([-1., -2., -3., -4.])
        sc = Scores(-1., -2., -3., -4., -5.)
        r = RifrafSequence(DNASeq("ACGT"), lp, 10, sc)
        np.testing.assert_array_equal(r.match_scores, np.log10(1.0 - 10.0 ** lp))
        np.testing.assert_array_equal(r.mismatch_scores, lp + sc.mismatch)
        np.testing.assert_array_equal(r.ins_scores, lp + sc.insertion)
        np.testing.assert_array_equal(r.del_scores, np.array([-1., -1., -2., -3., -4.]) + sc.deletion)
        np.testing.assert_array_equal(r.codon_ins_scores, np.array([-1., -2.]) + sc.codon_insertion)
        np.testing.assert_array_equal(r.codon_del_scores, np.array([-1., -1., -2., -3., -4.]) + sc.codon_deletion)
        # the C restatement of the same constructor agrees bit for bit except
        # for libm log10/exp10 (<= 1 ulp)
        (m, mm, ins, d, ci, cd), ne = oracle.seq_tables(lp, sc)
        np.testing.assert_allclose(m, r.match_scores, rtol=1e-15)
        np.testing.assert_array_equal(mm, r.mismatch_scores)
        np.testing.assert_array_equal(ins, r.ins_scores)
        np.testing.assert_array_equal(d, r.del_scores)
        np.testing.assert_array_equal(ci, r.codon_ins_scores)
        np.testing.assert_array_equal(cd, r.codon_del_scores)
        assert ne == pytest.approx(r.est_n_errors, rel=1e-15)

    def test_update_scores(self):
        r = RifrafSequence(DNASeq("ACGT"), np.array([-1., -2., -3., -4.]), 10, Scores(-1., -2., -3., -4., -5.))
        r2 = RifrafSequence.rescored(r, Scores(-1., -1., -1., -1., -1.))
        np.testing.assert_array_equal(r2.ins_scores, r2.mismatch_scores)

    def test_empty(self):
        assert len(RifrafSequence(DNASeq(""), np.zeros(0), 10, Scores(-1., -2., -3., -4., -5.))) == 0
        assert len(RifrafSequence()) == 0


# test_model.jl:39-154: score_proposal == forward(apply(p))[end, end]
def _random_proposal_case(rng, proposal_kind, pos_choice):
    errors = ErrorModel(1.0, 1.0, 1.0, 0.0, 0.0)
    template_len = int(rng.integers(30, 51))
    template = random_seq(template_len, rng)
    codon_moves = bool(rng.integers(0, 2))
    local_errors = ErrorModel(2.0, 0.1, 0.1, 3.0, 3.0) if codon_moves else ErrorModel(2.0, 4.0, 4.0, 0.0, 0.0)
    local_scores = Scores.from_errors(local_errors)
    seq, _, phreds, _, _ = sample_from_template(template, np.full(template_len, 0.1), errors, 3.0, 0.5, 0.5, rng)
    log_p = phreds.astype(np.float64) / (-10.0)
    bandwidth = max(5 * abs(template_len - len(seq)), 30)
    pseq = RifrafSequence(seq, log_p, bandwidth, local_scores)
    pos = pos_choice(template_len)
    if proposal_kind == "sub":
        p = Substitution(pos, rbase(rng))
    elif proposal_kind == "ins":
        p = Insertion(pos, rbase(rng))
    else:
        p = Deletion(pos)
    return template, pseq, p, codon_moves


@pytest.mark.parametrize("kind,choice,count", [
    ("sub", "rand1", 300), ("ins", "rand0", 300), ("del", "rand1", 300),
    ("del", "first", 10), ("del", "last", 10), ("sub", "first", 10), ("sub", "last", 10),
    ("ins", "first0", 10), ("ins", "last", 10)])
def test_score_proposal_property(kind, choice, count):
    rng = np.random.default_rng(1234)
    choosers = {"rand1": lambda L: int(rng.integers(1, L + 1)), "rand0": lambda L: int(rng.integers(0, L + 1)),
                "first": lambda L: 1, "last": lambda L: L, "first0": lambda L: 0}
    for _ in range(count):
        template, pseq, p, codon = _random_proposal_case(rng, kind, choosers[choice])
        new_template = apply_proposals(template, [p])
        Anew, _ = fwd(new_template, pseq)
        Bnew = bwd(new_template, pseq)
        check_all_cols(Anew, Bnew, codon)
        A, _ = fwd(template, pseq)
        B = bwd(template, pseq)
        score = oracle.score_proposal(p.kind, p.pos, p.base, A.data, B.data, template, pseq)
        assert score == pytest.approx(Anew[Anew.nrows, Anew.ncols], rel=1e-9), (p, codon)


class TestCandidateScores:           # test_model.jl:264-323 (single read, bw 9)
    """get_candidates with alignment proposals: exactly one candidate beats the
    current score, and its score is the perfect-alignment sum of match scores
    (the Julia test compares scores only)."""
    scores = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0))

    @pytest.mark.parametrize("cons,seq", [("TTT", "TAT"), ("TTT", "TT"), ("TT", "TAT")])
    def test_candidate(self, cons, seq):
        from rifraf_amd.align import moves_to_proposals
        pseq = RifrafSequence(DNASeq(seq), np.full(len(seq), -1.0), 9, self.scores)
        t = DNASeq(cons)
        A, _ = fwd(t, pseq)
        B = bwd(t, pseq)
        props = set(moves_to_proposals(align_moves(t, pseq), t, pseq))
        state_score = A[A.nrows, A.ncols]
        cands = []
        for p in props:
            sc = oracle.score_total(p, [A.data], [B.data], [pseq], t)
            if sc > state_score:
                cands.append(sc)
        assert len(cands) == 1
        assert cands[0] == pytest.approx(float(np.sum(pseq.match_scores)))


def _single_indel_proposals(consensus, ref):   # model.jl:538-562 over oracle moves
    moves = align_moves(consensus, ref, skew=True)
    results = []
    cons_idx = ref_idx = 0
    for mv in moves:
        if mv == 1:
            cons_idx += 1
            ref_idx += 1
        elif mv == 2:
            ref_idx += 1
            results.append(Insertion(cons_idx, int(ref.seq[ref_idx - 1])))
        elif mv == 3:
            cons_idx += 1
            results.append(Deletion(cons_idx))
        elif mv == 4:
            ref_idx += 3
        elif mv == 5:
            cons_idx += 3
    return results


@pytest.mark.parametrize("cons,ref,expected", [("TTTT", "TTT", "TTT"), ("TT", "TTT", "TTT"),
                                               ("TTTACCC", "TTTCGC", "TTTCCC"),
                                               ("TTTAAACCC", "TTTCGC", "TTTAAACCC")])
def test_correct_shifts(cons, ref, expected):       # test_correct_shifts.jl:8-35, model.jl:1303-1316
    cons, ref = DNASeq(cons), DNASeq(ref)
    bandwidth = int(math.ceil(min(len(cons), len(ref)) * 0.1))
    refseq = RifrafSequence(ref, np.full(len(ref), -1.0), bandwidth,
                            Scores.from_errors(ErrorModel(10.0, 1e-5, 1e-5, 1.0, 1.0)))
    props = _single_indel_proposals(cons, refseq)
    from rifraf_amd.types import dna_str
    assert dna_str(apply_proposals(cons, props)) == expected


def test_single_indel_proposals():                  # test_model.jl:175-189
    ref = RifrafSequence(DNASeq("CGGCGATTT"), np.full(9, -1.0), 10,
                         Scores.from_errors(ErrorModel(10.0, 1e-10, 1e-10, 1.0, 1.0)))
    props = _single_indel_proposals(DNASeq("CTGCCGA"), ref)
    assert len(props) == 1 and props[0] in [Deletion(2), Deletion(4), Deletion(5)]


@pytest.mark.parametrize("template,expect", [("AAACCCGGGTTT", False), ("AAACCCGGGTTTT", True), ("AAA", False)])
def test_has_single_indels(template, expect):       # test_model.jl:156-172
    rseq = RifrafSequence(DNASeq("AAAGGGTTT"), np.full(9, math.log10(0.01)), 6,
                          Scores.from_errors(normalize(ErrorModel(2.0, 0.5, 0.5, 1.0, 1.0))))
    moves = align_moves(template, rseq)
    assert (2 in moves or 3 in moves) == expect


def test_oracle_pass_matches_scalar():
    rng = np.random.default_rng(7)
    t = random_seq(40, rng)
    sc = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0))
    reads = []
    for _ in range(3):
        s, _, ph, _, _ = sample_from_template(t, np.full(40, 0.02), ErrorModel(1, 5, 5), 1.5, 1.0, 0.3, rng)
        reads.append(RifrafSequence(s, ph.astype(np.float64) / -10.0, 9, sc))
    totals, cells = oracle.cpu_pass(t, reads, nthreads=2)
    As = [fwd(t, r)[0].data for r in reads]
    Bs = [bwd(t, r).data for r in reads]
    for pos in (0, 1, 17, 40):
        for b in range(4):
            exp = oracle.score_total((1, pos, b), As, Bs, reads, t)
            assert totals[pos, 5 + b] == exp
        if pos >= 1:
            assert totals[pos, 4] == oracle.score_total((2, pos, 0), As, Bs, reads, t)
    assert cells > 0


def test_cpu_pass_continues_the_fold_chunk_by_chunk():
    """oracle.cpu_pass(totals=...) continues every proposal's left fold from
    the running totals, so chunked folds equal the whole-batch fold bit for bit
    (model.jl:389-397) -- the full-size c5 parity test relies on it."""
    import numpy as np
    import oracle
    from rifraf_amd import ErrorModel, RifrafSequence, Scores
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(3)
    _, t, _, reads, _, ph, _, _ = sample_sequences(12, 200, error_rate=0.03, rng=rng)
    sc = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0))
    seqs = [RifrafSequence(r, p, 9, sc) for r, p in zip(reads, ph)]
    whole, _ = oracle.cpu_pass(t, seqs, nthreads=2)
    tot, _ = oracle.cpu_pass(t, seqs[:5], nthreads=2)
    oracle.cpu_pass(t, seqs[5:9], nthreads=2, totals=tot)
    oracle.cpu_pass(t, seqs[9:], nthreads=2, totals=tot)
    assert np.array_equal(whole, tot)
    assert np.isfinite(whole).sum() == 8 * len(t) + 4
