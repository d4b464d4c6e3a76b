"""Batched multi-cluster driver (rifraf_amd.batch.rifraf_batch, SURVEY.md
§8(f) rank 1): many clusters' stage machines share one engine and one launch
per request kind, and every cluster's result equals its own rifraf() call."""
import os

import numpy as np
import pytest

from test_sharded import G1, assert_same_run, summary

HERE = os.path.dirname(os.path.abspath(__file__))


def _clusters():
    from rifraf_amd import ErrorModel, Scores, cap_phreds
    from rifraf_amd.fastxio import read_fasta_records, read_fastq
    from rifraf_amd.sample import sample_sequences
    out = []
    refs = dict(read_fasta_records(os.path.join(G1, "references.fasta")))
    refmap = dict(line.split() for line in open(os.path.join(G1, "ref-map.tsv")) if line.strip())
    for f in sorted(refmap):
        seqs, phreds, _ = read_fastq(os.path.join(G1, f))
        out.append(dict(dnaseqs=seqs, phreds=[cap_phreds(p, 30) for p in phreds], reference=refs[refmap[f]]))
    rng = np.random.default_rng(31)
    for n, L in [(5, 60), (3, 80), (8, 50), (1, 40)]:
        _, _, _, reads, _, phreds, _, _ = sample_sequences(n, L, error_rate=0.03, rng=rng)
        out.append(dict(dnaseqs=reads, phreds=phreds))
    return out


def _params():
    from rifraf_amd import ErrorModel, Scores
    from rifraf_amd.model import RifrafParams
    return RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)),
                        ref_scores=Scores.from_errors(ErrorModel(8, 0.1, 0.1, 1, 1)), max_iters=60,
                        do_score=True)


def _check(engine_factory):
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import rifraf
    clusters = _clusters()
    params = _params()
    single = [summary(rifraf(params=params, engine=engine_factory(), **kw)) for kw in clusters]
    batched = rifraf_batch(clusters, params=params, engine=engine_factory())
    assert len(batched) == len(clusters)
    for s, b in zip(single, batched):
        assert_same_run(summary(b), s)


def test_batch_matches_separate_runs_oracle():
    from oracle_engine import OracleEngine
    _check(OracleEngine)


def test_batch_waves_and_errors():
    """Waves smaller than the batch, and a cluster error surfaces."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.engine import RifrafError
    clusters = _clusters()
    params = _params()
    a = rifraf_batch(clusters, params=params, engine=OracleEngine(), wave=2)
    b = rifraf_batch(clusters, params=params, engine=OracleEngine())
    for x, y in zip(a, b):
        assert_same_run(summary(x), summary(y))
    bad = clusters[:2] + [dict(dnaseqs=clusters[2]["dnaseqs"], phreds=[-np.ones(len(s)) for s in
                                                                         clusters[2]["dnaseqs"]])]
    with pytest.raises(RifrafError):
        rifraf_batch(bad, params=params, engine=OracleEngine())


@pytest.mark.gpu
def test_batch_matches_separate_runs_hip(engine):
    _check(lambda: engine)


@pytest.mark.gpu
def test_batch_hip_matches_oracle_runs(engine):
    """HIP-batched clusters (one launch per request kind) against separate
    rifraf() runs on the CPU oracle engine: same consensus at every
    iteration, same score, same QVs (error_probs, aln_error_probs)."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import rifraf
    clusters = _clusters()
    params = _params()
    ref = [summary(rifraf(params=params, engine=OracleEngine(), **kw)) for kw in clusters]
    got = rifraf_batch(clusters, params=params, engine=engine)
    for r, g in zip(ref, got):
        assert_same_run(summary(g), r)
