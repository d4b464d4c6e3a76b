"""End-to-end rifraf() parity (src/model.jl) and the reference's model tests.

Every test runs the host stage machine (rifraf_amd.model) on two engines:
  * "oracle": tests/oracle_engine.py, the CPU oracle behind the Engine API
    (runs in the CPU suite; pins the host logic);
  * "hip": the MI355X engine (marked gpu).
test_gpu_matches_oracle_run additionally compares whole runs (consensus of
every iteration, final score) between the two engines.
"""
import math
import os

import numpy as np
import pytest

from rifraf_amd import ErrorModel, RifrafSequence, Scores, cap_phreds, dna_str, DNASeq
from rifraf_amd.fastxio import read_fasta_records, read_fastq
from rifraf_amd.errormodel import normalize
from rifraf_amd.model import (RifrafParams, Stage, alignment_error_probs, estimate_probs, get_candidates,
                              initial_state, realign_rescore, resample, rifraf, _Run)
from rifraf_amd.proposals import Deletion, Insertion, Substitution
from rifraf_amd.sample import sample_sequences

HERE = os.path.dirname(os.path.abspath(__file__))
G1 = os.path.join(HERE, "golden", "config1")


@pytest.fixture(params=["oracle", pytest.param("hip-lat", marks=pytest.mark.gpu),
                        pytest.param("hip-tp", marks=pytest.mark.gpu)])
def eng(request):
    """hip-lat: the engine's product default DP (latency mode for small
    calls: k_dpx); hip-tp: the throughput classes (conftest.DP_MODES)."""
    if request.param == "oracle":
        from oracle_engine import OracleEngine
        yield OracleEngine()
        return
    e = request.getfixturevalue("engine")
    old = e.set_option("dp_lat", e.product_dp_lat if request.param == "hip-lat" else 0)
    yield e
    e.set_option("dp_lat", old)


def config1_run(f, refid, engine):
    """scripts/rifraf.jl dofile (:71-120) with the docs/src/examples.md:61-68 flags."""
    refs = dict(read_fasta_records(os.path.join(G1, "references.fasta")))
    seqs, phreds, _ = read_fastq(os.path.join(G1, f))
    phreds = [cap_phreds(p, 30) for p in phreds]
    params = RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)),
                          ref_scores=Scores.from_errors(ErrorModel(8, 0.1, 0.1, 1, 1)), max_iters=100)
    return rifraf(seqs, phreds, reference=refs[refid], params=params, engine=engine)


def test_config1_golden_consensus(eng):
    """data/consensus-results.fasta = CLI output for data/input-reads-*.fastq."""
    expected = dict(read_fasta_records(os.path.join(G1, "consensus-results.fasta")))
    refmap = dict(line.split() for line in open(os.path.join(G1, "ref-map.tsv")) if line.strip())
    for f in sorted(refmap):
        res = config1_run(f, refmap[f], eng)
        assert res.state.converged
        assert dna_str(res.consensus) == expected[f]


def _state(eng, consensus, pseqs, params):
    state = initial_state(DNASeq(consensus), pseqs, np.zeros(0, np.uint8), params)
    run = _Run(eng, len(pseqs))
    eng.set_sequences(0, pseqs)
    run.set_consensus(state.consensus)
    resample(state, params, np.random.default_rng(0))
    realign_rescore(state, run, RifrafParams())
    return state, run


@pytest.mark.parametrize("consensus,seqs,lps,expected", [         # test_model.jl:191-262
    ("ACGAG", ["CGTAC", "CGAC", "CGTAG"], None, {Deletion(1), Insertion(3, 3), Substitution(5, 1)}),
    ("AA", ["AAG", "AA", "AAG"], None, {Insertion(2, 2)}),
    ("AA", ["GAA", "AA", "GAA"], None, {Insertion(0, 2)}),
    ("AA", ["AGA", "AA", "AGA"], None, {Insertion(1, 2)}),
    ("AA", ["GAA", "AA", "AA"], [[-10.0, -5.0, -5.0], [-3.0, -5.0], [-3.0, -50.0]], {Insertion(0, 2)}),
])
def test_alignment_proposals(eng, consensus, seqs, lps, expected):
    from rifraf_amd.model import alignment_proposals
    params = RifrafParams(bandwidth=6, batch_fixed=False, batch_size=len(seqs))
    scores = Scores.from_errors(ErrorModel(1.0, 5.0, 5.0, 0.0, 0.0))
    if lps is None:
        lps = [np.full(len(s), -9.0) for s in seqs]
    pseqs = [RifrafSequence(DNASeq(s), np.array(p, float), params.bandwidth, scores) for s, p in zip(seqs, lps)]
    state, run = _state(eng, consensus, pseqs, params)
    assert set(alignment_proposals(state, run, True)) == expected


@pytest.mark.parametrize("consensus,seq", [("TTT", "TAT"), ("TTT", "TT"), ("TT", "TAT")])
def test_candidate_scores(eng, consensus, seq):                     # test_model.jl:264-323
    params = RifrafParams(bandwidth=9, do_alignment_proposals=True)
    scores = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0))
    pseqs = [RifrafSequence(DNASeq(seq), np.full(len(seq), -1.0), params.bandwidth, scores)]
    state, run = _state(eng, consensus, pseqs, params)
    cands = get_candidates(state, run, params)
    assert len(cands) == 1
    assert cands[0].score == pytest.approx(float(np.sum(pseqs[0].match_scores)))


def test_base_probs(eng):                                            # test_model.jl:378-399
    params = RifrafParams(bandwidth=6)
    scores = Scores.from_errors(normalize(ErrorModel(1.0, 1.0, 1.0, 0.0, 0.0)))
    pseqs = [RifrafSequence(DNASeq("CGAC"), np.full(4, -9.0), 6, scores) for _ in range(3)]
    state, run = _state(eng, "CGTAC", pseqs, params)
    probs = estimate_probs(state, run, False)
    assert probs.sub[0, 1] > 0.9
    assert probs.dele[0] < 1e-9
    assert probs.dele[2] > 0.9


def test_ins_probs(eng):                                             # test_model.jl:402-422
    params = RifrafParams(bandwidth=6)
    scores = Scores.from_errors(normalize(ErrorModel(1.0, 1.0, 1.0, 0.0, 0.0)))
    pseqs = [RifrafSequence(DNASeq("CGTAT"), np.full(5, -9.0), 6, scores) for _ in range(3)]
    state, run = _state(eng, "CGAT", pseqs, params)
    probs = estimate_probs(state, run, False)
    assert probs.ins[0, :].max() < 1e-9
    assert probs.ins[2, 3] > 0.9


def test_alignment_error_probs(eng):                                 # test_model.jl:424-449
    params = RifrafParams(bandwidth=6)
    scores = Scores.from_errors(normalize(ErrorModel(1.0, 1.0, 1.0, 0.0, 0.0)))
    ps = [[0.1, 0.1, 0.1, 0.1], [0.2, 0.1, 0.1], [0.2, 0.1, 0.1, 0.1]]
    pseqs = [RifrafSequence(DNASeq(s), np.log10(p), 6, scores) for s, p in zip(["ACGT", "CGT", "CCGT"], ps)]
    state, run = _state(eng, "ACGT", pseqs, params)
    result = alignment_error_probs(4, state, run)
    assert list(np.argsort(result, kind="stable") + 1) == [4, 3, 2, 1]


def test_alignment_error_probs_matches_loop(eng):
    """The vectorised alignment_error_probs equals the reference's per-read,
    per-move loop (model.jl:817-840) bit for bit: ragged noisy reads, so the
    walk sees matches, inserts and deletes and columns get rows from several
    reads in batch order."""
    from rifraf_amd.align import TRACE_MATCH
    from rifraf_amd.model import base_distribution
    rng = np.random.default_rng(31)
    _, t, _, reads, _, phreds, _, _ = sample_sequences(9, 120, error_rate=0.06, rng=rng)
    scores = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0))
    pseqs = [RifrafSequence(r, p, 9, scores) for r, p in zip(reads, phreds)]
    state, run = _state(eng, dna_str(t), pseqs, RifrafParams(bandwidth=9, batch_size=0, batch_fixed=False))
    got = alignment_error_probs(len(t), state, run)
    moves, _ = run.e.backtrace(np.arange(len(state.batch_seqs), dtype=np.int32))
    probs = np.zeros((len(t), 4))
    off = {1: (1, 1), 2: (1, 0), 3: (0, 1), 4: (3, 0), 5: (0, 3)}
    for idx, mv in zip(state.batch_seqs, moves):
        s = state.sequences[idx]
        i, j = 1, 1
        for move in mv.tolist():
            i, j = i + off[move][0], j + off[move][1]
            if move == TRACE_MATCH:
                probs[j - 2] += base_distribution(int(s.seq[i - 2]), float(s.match_scores[i - 2]))
    probs = np.power(10.0, probs)
    expect = 1.0 - (probs / probs.sum(axis=1, keepdims=True)).max(axis=1)
    np.testing.assert_array_equal(got, expect)
    assert np.count_nonzero(got) > 0


def test_smart_forward_moves_widens_band(eng):                       # test_model.jl:451-471
    from rifraf_amd.model import smart_forward_moves
    seq = DNASeq("AAAGGGTTTCCC")
    errors = np.full(len(seq), 0.3)
    errors[-4:] = 0.45
    rseq = RifrafSequence(seq, np.log10(errors), 1, Scores.from_errors(ErrorModel(1.0, 10.0, 10.0, 0.0, 0.0)))
    run = _Run(eng, 1)
    eng.set_sequences(0, [rseq])
    run.set_consensus(DNASeq("AAACCCGGGTTT"))
    smart_forward_moves(run, [(0, 0)], [rseq], 12, 0.1)
    assert rseq.bandwidth > 1


FULL_MODEL = [(use_ref, dap, si, ico, bs) for use_ref in (True, False) for dap in (True, False)
              for si in (True, False) for ico in (True, False) for bs in (3, 6)]


def test_full_model(eng):                                            # test_model.jl:325-375
    """32 parameter combinations, 5 reads x 30 bp; the reference notes it
    "can't guarantee" success (stochastic inputs); require >= 30/32."""
    seq_errors = ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0)
    ok = 0
    rng = np.random.default_rng(1234)
    for use_ref, dap, si, ico, bs in FULL_MODEL:
        ref, template, _, reads, _, phreds, _, _ = sample_sequences(
            5, 30, ref_error_rate=0.1, ref_errors=ErrorModel(8.0, 0.0, 0.0, 1.0, 1.0), error_rate=0.005,
            alpha=1.0, phred_scale=1.5, actual_std=3.0, reported_std=0.3, seq_errors=seq_errors, rng=rng)
        params = RifrafParams(scores=Scores.from_errors(seq_errors),
                              ref_scores=Scores.from_errors(ErrorModel(8.0, 0.1, 0.1, 1.0, 1.0)),
                              do_alignment_proposals=dap, seed_indels=si, indel_correction_only=ico,
                              batch_size=bs, seed=7)
        res = rifraf(reads, phreds, reference=ref if use_ref else None, params=params, engine=eng)
        ok += int(np.array_equal(res.consensus, template))
    assert ok >= 30, f"{ok}/32 runs recovered the template"


@pytest.mark.gpu
def test_gpu_matches_oracle_run(run_engine, oracle_memo):
    """Identical consensus after every iteration and identical final score,
    HIP engine vs oracle engine, on clusters that exercise INIT, FRAME (codon
    reference scoring) and REFINE."""
    from oracle_engine import OracleEngine
    rng = np.random.default_rng(42)
    for case in range(6):
        ref, template, _, reads, _, phreds, _, _ = sample_sequences(
            8, 150, ref_error_rate=0.05, ref_errors=ErrorModel(8.0, 0.0, 0.0, 1.0, 1.0), error_rate=0.02,
            rng=rng)
        params = RifrafParams(batch_size=0 if case % 2 else 20, seed=case)
        a = rifraf(reads, phreds, reference=ref, params=params, engine=run_engine)
        b = oracle_memo(("gpu_matches_oracle_run", case),
                        lambda: rifraf(reads, phreds, reference=ref, params=params, engine=OracleEngine()))
        assert a.state.score == b.state.score
        assert np.array_equal(a.consensus, b.consensus)
        for sa, sb in zip(a.consensus_stages, b.consensus_stages):
            assert len(sa) == len(sb)
            for x, y in zip(sa, sb):
                assert np.array_equal(x, y)


def test_frame_batch_growth_before_single_indel_proposals(eng, monkeypatch):
    """check_score's batch growth (model.jl:1102-1111) realigns the grown
    batch inside a FRAME iteration before single_indel_proposals
    (model.jl:1145-1149): the skewed reference fill that realign()'s B call
    leaves in the scratch slot must be the current one.  Same run as with
    single_indel_proposals filling the scratch slot itself (SIP_CACHE off)."""
    import rifraf_amd.model as model
    rng = np.random.default_rng(2)
    ref, _, _, reads, _, phreds, _, _ = sample_sequences(
        30, 240, error_rate=0.03, ref_error_rate=0.1, ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
    ref = np.concatenate([ref[:100], ref[101:]]).astype(np.uint8)
    params = RifrafParams(batch_size=5, batch_threshold=0.0, batch_fixed=False, seed=1)
    grown = []
    check = model.check_score

    def spy(state, run, p, old, rng_):
        b = state.batch_size
        ok = check(state, run, p, old, rng_)
        grown.append(state.stage == Stage.FRAME and ok and state.batch_size > b)
        return ok

    monkeypatch.setattr(model, "check_score", spy)
    a = rifraf(reads, phreds, reference=ref, params=params, engine=eng)
    assert any(grown)
    monkeypatch.setattr(model, "SIP_CACHE", False)
    b = rifraf(reads, phreds, reference=ref, params=params, engine=eng)
    assert a.state.score == b.state.score
    assert [list(map(dna_str, x)) for x in a.consensus_stages] == [list(map(dna_str, x)) for x in b.consensus_stages]
