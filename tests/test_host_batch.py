"""Host-side batch helpers of the native batched driver (CPU): the vectorised
RifrafSequence constructor, the library's Julia-order sums and the
vectorised Poisson thresholds equal the per-sequence Python code bit for bit."""
import math

import numpy as np
import pytest

from rifraf_amd import ErrorModel, RifrafSequence, Scores
from rifraf_amd.poisson import cquantile_poisson, cquantile_poisson_many
from rifraf_amd.rifrafsequences import julia_sum


def _reads(rng, n=300):
    seqs, lps = [], []
    for _ in range(n):
        L = int(rng.choice([1, 2, 3, 15, 16, 17, 100, 1023, 1024, 1025, 1500, 2049, 4100]))
        seqs.append(rng.integers(0, 4, L).astype(np.uint8))
        if rng.random() < 0.5:
            lps.append(rng.integers(0, 41, L).astype(np.int8))          # phreds
        else:
            lps.append(-rng.uniform(0.01, 4.0, L))
    return seqs, lps


def test_many_equals_per_sequence_constructor():
    rng = np.random.default_rng(3)
    seqs, lps = _reads(rng)
    sc = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0))
    got = RifrafSequence.many(seqs, lps, 9, sc)
    for g, s, lp in zip(got, seqs, lps):
        e = RifrafSequence(s, lp, 9, sc)
        for f in ("seq", "error_log_p", "match_scores", "mismatch_scores", "ins_scores", "del_scores",
                  "codon_ins_scores", "codon_del_scores"):
            np.testing.assert_array_equal(getattr(g, f), getattr(e, f), err_msg=f)
        assert g.est_n_errors == e.est_n_errors
        assert g.bandwidth == e.bandwidth and g.bandwidth_fixed == e.bandwidth_fixed


def test_many_concat_phred_tables():
    """The per-distinct-Phred evaluation + gather equals the direct tables."""
    from rifraf_amd.errormodel import phred_to_log_p
    rng = np.random.default_rng(4)
    ph = [rng.integers(0, 94, int(n)).astype(np.int8) for n in rng.integers(1, 3000, 40)]
    seqs = [rng.integers(0, 4, len(p)).astype(np.uint8) for p in ph]
    off = np.zeros(len(ph) + 1, np.int64)
    np.cumsum([len(p) for p in ph], out=off[1:])
    sc = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0))
    cat = np.concatenate(ph)
    a, ta = RifrafSequence.many_concat(seqs, phred_to_log_p(cat), off, 9, sc, phreds=cat)
    b, tb = RifrafSequence.many_concat(seqs, phred_to_log_p(cat), off, 9, sc)
    for k in tb:
        np.testing.assert_array_equal(ta[k], tb[k])
    for x, y, s, p in zip(a, b, seqs, ph):
        e = RifrafSequence(s, p, 9, sc)
        assert x.est_n_errors == y.est_n_errors == e.est_n_errors
        np.testing.assert_array_equal(x.match_scores, e.match_scores)
        np.testing.assert_array_equal(x.del_scores, e.del_scores)


def test_host_sums_match_python():
    from rifraf_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(9)
    lens = rng.choice([0, 1, 2, 15, 16, 1024, 1025, 3000, 5000], 80)
    off = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    v = rng.uniform(0, 1, int(off[-1])) ** 7
    a, b = np.empty(len(lens)), np.empty(len(lens))
    lib.rf_host_julia_sums(len(lens), _lib.ptr(v), _lib.ptr(off), _lib.ptr(a))
    lib.rf_host_seq_sums(len(lens), _lib.ptr(v), _lib.ptr(off), _lib.ptr(b))
    for k in range(len(lens)):
        seg = v[off[k]:off[k + 1]]
        assert a[k] == julia_sum(seg)
        assert b[k] == (float(np.cumsum(seg)[-1]) if len(seg) else 0.0)


def test_poisson_thresholds_vectorised():
    rng = np.random.default_rng(2)
    lams = np.concatenate([rng.uniform(0.01, 400, 3000), rng.uniform(0.001, 2, 500), np.arange(1, 401.0)])
    for p in (0.1, 0.01, 0.5):
        np.testing.assert_array_equal(cquantile_poisson_many(lams, p),
                                      [cquantile_poisson(float(x), p) for x in lams])
    assert math.isnan(cquantile_poisson_many(np.array([math.nan]), 0.1)[0])


def test_qvs_many_equals_per_cluster():
    """The stacked QV post-processing equals estimate_probs_from_dense and
    aln_error_probs_from_sums cluster by cluster, bit for bit."""
    from types import SimpleNamespace

    from rifraf_amd.model import aln_error_probs_from_sums, estimate_probs_from_dense, qvs_many
    rng = np.random.default_rng(8)
    states, dense, sums = [], [], []
    for m in rng.integers(1, 400, 30):
        cons = rng.integers(0, 4, m).astype(np.uint8)
        score = -float(rng.uniform(50, 500))
        d = score + rng.uniform(-30, 2, (m + 1, 9))
        d[0, :5] = np.nan
        states.append(SimpleNamespace(consensus=cons, score=score))
        dense.append(d)
        sums.append(-rng.uniform(0, 60, (m, 4)))
    got = qvs_many(states, dense, sums)
    for st, d, sm, (ep, ap) in zip(states, dense, sums, got):
        e = estimate_probs_from_dense(st, d)
        np.testing.assert_array_equal(ep.sub, e.sub)
        np.testing.assert_array_equal(ep.dele, e.dele)
        np.testing.assert_array_equal(ep.ins, e.ins)
        np.testing.assert_array_equal(ap, aln_error_probs_from_sums(sm))


def test_logsumexp10_table_path():
    from rifraf_amd.batch import _logsumexp10_many
    from rifraf_amd.errormodel import phred_to_log_p
    from rifraf_amd.model import logsumexp10
    rng = np.random.default_rng(6)
    ph = [rng.integers(0, 60, int(n)).astype(np.int8) for n in rng.integers(1, 2000, 50)]
    seqs = [rng.integers(0, 4, len(p)).astype(np.uint8) for p in ph]
    off = np.zeros(len(ph) + 1, np.int64)
    np.cumsum([len(p) for p in ph], out=off[1:])
    cat = np.concatenate(ph)
    objs, tabs = RifrafSequence.many_concat(seqs, phred_to_log_p(cat), off, 9,
                                            Scores.from_errors(ErrorModel(1.0, 2.0, 2.0)), phreds=cat)
    a = _logsumexp10_many(tabs["match"], off, codes=tabs["code"], table=tabs["match_table"])
    b = _logsumexp10_many(tabs["match"], off)
    assert a == b == [logsumexp10(o.match_scores) for o in objs]


def test_threaded_power10_is_elementwise():
    from rifraf_amd.model import _power10
    x = -np.random.default_rng(12).uniform(0, 40, (700_001, 3))
    np.testing.assert_array_equal(_power10(x), np.power(10.0, x))


def _qv_inputs(rng, n=30, stacked=False):
    from types import SimpleNamespace
    states, dense, sums = [], [], []
    ms = rng.integers(1, 400, n)
    ms[:3] = [1, 2, 1500]
    for m in ms:
        cons = rng.integers(0, 4, m).astype(np.uint8)
        score = -float(rng.uniform(50, 500))
        d = score + rng.uniform(-30, 2, (m + 1, 9))
        d[0, :5] = np.nan
        d[1 + np.arange(m), cons] = np.nan          # not a proposal: ignored
        d[rng.random((m + 1, 9)) < 0.01] = -np.inf  # empty summax columns
        d[0, :5] = np.nan
        states.append(SimpleNamespace(consensus=cons, score=score))
        dense.append(d)
        s = -rng.uniform(0, 60, (m, 4))
        s[rng.random((m, 4)) < 0.01] = 0.0
        sums.append(s)
    if stacked:   # consecutive views of one array, as engine.score_dense returns
        D, S = np.concatenate(dense), np.concatenate(sums)
        at, bt, dense, sums = 0, 0, [], []
        for m in ms:
            dense.append(D[at:at + m + 1])
            sums.append(S[bt:bt + m])
            at += m + 1
            bt += m
    return states, dense, sums


def test_qvs_many_lib_equals_qvs_many():
    """The C++ passes of the QV post-processing (rf_host_qv_prep /
    rf_host_qv_finish around numpy's power) equal qvs_many bit for bit,
    for stacked views and separate arrays, with -Inf totals and zero sums."""
    from rifraf_amd.model import qvs_many, qvs_many_lib
    for stacked in (False, True):
        states, dense, sums = _qv_inputs(np.random.default_rng(18), stacked=stacked)
        got = qvs_many_lib(states, dense, sums)
        exp = qvs_many(states, dense, sums)
        for (ep, ap), (e, a) in zip(got, exp):
            for f in ("sub", "dele", "ins"):
                assert getattr(ep, f).tobytes() == getattr(e, f).tobytes(), f
            assert ap.tobytes() == a.tobytes()


def test_qvs_many_lib_errors():
    import pytest

    from rifraf_amd.engine import RifrafError
    from rifraf_amd.model import qvs_many, qvs_many_lib
    states, dense, sums = _qv_inputs(np.random.default_rng(19), n=5)
    dense[3][4, 6] = np.nan
    for f in (qvs_many, qvs_many_lib):
        with pytest.raises(RifrafError, match="failed to compute a valid score"):
            f(states, dense, sums)


def test_many_coded_equals_constructor():
    """many_coded's lazily built tables, est_n_errors and logsumexp10 equal the
    per-sequence constructor's and model.logsumexp10's, bit for bit."""
    from rifraf_amd.model import logsumexp10
    from rifraf_amd.rifrafsequences import CodedRifrafSequence
    rng = np.random.default_rng(21)
    ph = [rng.integers(0, 94, int(n)).astype(np.int8) for n in rng.integers(1, 3000, 60)]
    ph[0][:] = 0                                      # all match scores -Inf
    ph += [np.array([7], np.int8), rng.integers(0, 94, 1025).astype(np.int8)]
    seqs = [rng.integers(0, 4, len(p)).astype(np.uint8) for p in ph]
    off = np.zeros(len(ph) + 1, np.int64)
    np.cumsum([len(p) for p in ph], out=off[1:])
    sc = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0))
    objs, tabs, lse = RifrafSequence.many_coded(seqs, np.concatenate(ph), off, 9, sc)
    full = tabs["source"].full()
    for k, (o, s, p) in enumerate(zip(objs, seqs, ph)):
        assert isinstance(o, CodedRifrafSequence)
        e = RifrafSequence(s, p, 9, sc)
        assert o.est_n_errors == e.est_n_errors
        assert lse[k] == logsumexp10(e.match_scores)
        for f in ("error_log_p", "match_scores", "mismatch_scores", "ins_scores", "del_scores"):
            assert getattr(o, f).tobytes() == getattr(e, f).tobytes(), f
        assert full["match"][off[k]:off[k + 1]].tobytes() == e.match_scores.tobytes()
        assert full["del"][off[k] + k:off[k + 1] + k + 1].tobytes() == e.del_scores.tobytes()
        assert len(o) == len(e) and o.bandwidth == 9 and not o.bandwidth_fixed


def test_packed_reads_sequence():
    """PackedReads: one buffer + offsets behaving as a list of read views."""
    from rifraf_amd.types import PackedReads
    reads = [np.array([0, 1, 2], np.uint8), np.array([3], np.uint8), np.array([2, 2], np.uint8)]
    p = PackedReads.from_list(reads, np.uint8)
    assert len(p) == 3 and list(p.lens()) == [3, 1, 2]
    assert all(np.array_equal(a, b) for a, b in zip(p, reads))
    assert np.array_equal(p[-1], reads[-1]) and len(p[0:2]) == 2
    with pytest.raises(IndexError):
        p[3]
    with pytest.raises(ValueError):
        PackedReads(np.zeros(3, np.uint8), [0, 4])


def test_packed_reads_python_stage_machine_oracle():
    """Clusters given as PackedReads run the Python stage machine (the oracle
    engine) exactly as the same reads given as lists."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams
    from rifraf_amd.sample import sample_sequences
    from rifraf_amd.types import PackedReads
    rng = np.random.default_rng(5)
    cl, pk = [], []
    for _ in range(3):
        _, _, _, reads, _, phreds, _, _ = sample_sequences(6, 60, error_rate=0.03, rng=rng)
        cl.append(dict(dnaseqs=reads, phreds=phreds))
        pk.append(dict(dnaseqs=PackedReads.from_list(reads, np.uint8), phreds=PackedReads.from_list(phreds, np.int8)))
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
    a = rifraf_batch(cl, params=params, engine=OracleEngine())
    b = rifraf_batch(pk, params=params, engine=OracleEngine())
    for x, y in zip(a, b):
        assert np.array_equal(x.consensus, y.consensus) and x.state.score == y.state.score
        assert np.array_equal(x.aln_error_probs, y.aln_error_probs)


def test_read_fastq_packed_matches_lists():
    """read_fastq_packed: the same reads and Phred scores as read_fastq, as
    PackedReads (config 1's golden input)."""
    import os
    from rifraf_amd.fastxio import read_fastq, read_fastq_packed
    f = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config1", "input-reads-1.fastq")
    s, p, n = read_fastq(f)
    ps, pp, pn = read_fastq_packed(f)
    assert n == pn and len(ps) == len(s)
    assert all(np.array_equal(a, b) for a, b in zip(ps, s))
    assert all(np.array_equal(a, b) for a, b in zip(pp, p))
