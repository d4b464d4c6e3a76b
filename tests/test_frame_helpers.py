"""Reference-frame helpers of the product host (rifraf_amd.model) on both
engines, against the reference's own known answers:

  correct_shifts          model.jl:1303-1316  <- test/test_correct_shifts.jl:8-35
  has_single_indels       model.jl:532-536    <- test/test_model.jl:156-172
  single_indel_proposals  model.jl:538-562    <- test/test_model.jl:175-189

These run the codon-move DP (skew_matches for single_indel_proposals) and the
backtrace on the engine: "oracle" is the CPU stand-in (CPU suite), "hip-lat" /
"hip-tp" the MI355X engine (gpu) in its default DP mode and with the
throughput classes."""
import math

import numpy as np
import pytest

from rifraf_amd import ErrorModel, RifrafSequence, Scores, DNASeq
from rifraf_amd.errormodel import normalize
from rifraf_amd.model import RifrafState, _Run, correct_shifts, has_single_indels, single_indel_proposals
from rifraf_amd.proposals import Deletion
from rifraf_amd.types import dna_str


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


def _state(eng, consensus, rseq):
    run = _Run(eng, 0)
    run.set_consensus(DNASeq(consensus))
    eng.set_sequences(run.REF, [rseq])
    state = RifrafState(consensus=DNASeq(consensus), ref_scores=rseq, reference=rseq, batch_fixed_size=0,
                        batch_size=0, base_batch_size=0, sequences=[], maxlen=0)
    return state, run


@pytest.mark.parametrize("cons,ref,expected", [("TTTT", "TTT", "TTT"), ("TT", "TTT", "TTT"),
                                               ("TTTACCC", "TTTCGC", "TTTCCC"),
                                               ("TTTAAACCC", "TTTCGC", "TTTAAACCC")])
def test_correct_shifts(eng, cons, ref, expected):          # test_correct_shifts.jl:8-35
    assert dna_str(correct_shifts(DNASeq(cons), DNASeq(ref), engine=eng)) == expected


@pytest.mark.parametrize("template,expect", [("AAACCCGGGTTT", False), ("AAACCCGGGTTTT", True), ("AAA", False)])
def test_has_single_indels(eng, template, expect):         # test_model.jl:156-172
    rseq = RifrafSequence(DNASeq("AAAGGGTTT"), np.full(9, math.log10(0.01)), 6,
                          Scores.from_errors(normalize(ErrorModel(2.0, 0.5, 0.5, 1.0, 1.0))))
    state, run = _state(eng, template, rseq)
    assert has_single_indels(state, run) == expect


def test_single_indel_proposals(eng):                      # test_model.jl:175-189
    ref = RifrafSequence(DNASeq("CGGCGATTT"), np.full(9, -1.0), 10,
                         Scores.from_errors(ErrorModel(10.0, 1e-10, 1e-10, 1.0, 1.0)))
    state, run = _state(eng, "CTGCCGA", ref)
    props = single_indel_proposals(state, run)
    assert len(props) == 1 and props[0] in [Deletion(2), Deletion(4), Deletion(5)]
