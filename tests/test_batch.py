"""Batched multi-cluster driver (rifraf_amd.batch.rifraf_batch, SURVEY.md
§8(f) rank 1): many clusters' stage machines share one engine and one launch
per request kind, and every cluster's result equals its own rifraf() call."""
import os

import numpy as np
import pytest

from test_sharded import G1, QV_RTOL, assert_same_run, summary

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


def _check(engine_factory, qv_rtol=0.0):
    """qv_rtol: a HIP engine's batch takes the native driver, whose quality
    pass runs on the device (QVs within QV_RTOL of the host evaluation)."""
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import rifraf
    clusters = _clusters()
    params = _params()
    single = [summary(rifraf(params=params, engine=engine_factory(), **kw)) for kw in clusters]
    batched = rifraf_batch(clusters, params=params, engine=engine_factory())
    assert len(batched) == len(clusters)
    for s, b in zip(single, batched):
        assert_same_run(summary(b), s, qv_rtol=qv_rtol)


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


@pytest.mark.parametrize("wave,excl", [(1024, False), (1, True)])
def test_batch_engine_shards_oracle(wave, excl):
    """rifraf_batch(engines=[...]): waves of clusters taken from a shared
    queue by one host thread per engine (one wave per engine, or one cluster
    per wave with the exclusive-stage-machine option) give the single-engine
    results, in input order."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    clusters = _clusters()
    params = _params()
    one = rifraf_batch(clusters, params=params, engine=OracleEngine())
    three = rifraf_batch(clusters, params=params, engines=[OracleEngine() for _ in range(3)], wave=wave,
                         init_exclusive=excl)
    assert len(three) == len(one)
    for x, y in zip(three, one):
        assert_same_run(summary(x), summary(y))


@pytest.mark.gpu
def test_batch_matches_separate_runs_hip(run_engine):
    engine = run_engine
    _check(lambda: engine, qv_rtol=QV_RTOL)


@pytest.mark.gpu
def test_batch_hip_matches_oracle_runs(run_engine):
    """HIP-batched clusters (one launch per request kind) against separate
    rifraf() runs on the CPU oracle engine: same consensus at every
    iteration, same score, same QVs (error_probs, aln_error_probs)."""
    engine = run_engine
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import rifraf
    clusters = _clusters()
    params = _params()
    ref = [summary(rifraf(params=params, engine=OracleEngine(), **kw)) for kw in clusters]
    got = rifraf_batch(clusters, params=params, engine=engine)
    for r, g in zip(ref, got):
        assert_same_run(summary(g), r, qv_rtol=QV_RTOL)


def _ref_free_clusters(seed=97):
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(seed)
    out = []
    for n, L, err in [(12, 150, 0.02), (20, 300, 0.01), (6, 90, 0.05), (1, 40, 0.02), (9, 220, 0.03),
                      (30, 120, 0.02), (3, 400, 0.01), (15, 250, 0.04)]:
        _, _, _, reads, _, phreds, _, _ = sample_sequences(n, L, error_rate=err, rng=rng)
        out.append(dict(dnaseqs=reads, phreds=phreds))
    return out


NATIVE_PARAMS = {
    "default": dict(max_iters=60),                                          # fixed batch of 5
    "all_reads_qv": dict(batch_size=0, batch_fixed=False, do_score=True),
    "fixed3_noaln": dict(batch_fixed_size=3, do_alignment_proposals=False, do_score=True, max_iters=4),
    # random batches (resample!, model.jl:1051-1054): drawn by the native
    # driver with resampling.py's RNG; the second grows its batch on every
    # score drop (check_score, model.jl:1092-1101) and resamples there too
    "random_batch": dict(batch_size=5, batch_fixed=False, seed=7, do_score=True, max_iters=40),
    "random_grow": dict(batch_size=3, batch_fixed=False, batch_threshold=0.0, seed=3, max_iters=30),
}


def _same_batches(a, b):
    """The final batch (the reads of the last random draw, in draw order)."""
    assert [int(i) for i in a.state.batch_seqs] == [int(i) for i in b.state.batch_seqs]


@pytest.mark.gpu
@pytest.mark.parametrize("pset", sorted(NATIVE_PARAMS))
def test_native_batch_matches_hub(run_engine, pset):
    """rf_rifraf_batch (the library's lockstep stage machine) against the
    Python stage machine over the same engine: identical consensus at every
    iteration, score, iteration counts and convergence; QVs bit-identical
    with the host quality pass (device_qv=False) and within 1e-12 with the
    device one (the default)."""
    engine = run_engine
    from rifraf_amd import ErrorModel, Scores
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams
    params = RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)), **NATIVE_PARAMS[pset])
    clusters = _ref_free_clusters()
    from rifraf_amd import batch as B
    hub = rifraf_batch(clusters, params=params, engine=engine, native=False)
    skipped = B.STATS["qv_refill_skipped"]
    nat = rifraf_batch(clusters, params=params, engine=engine, native=True, device_qv=False)
    dqv = rifraf_batch(clusters, params=params, engine=engine, native=True)
    if pset == "all_reads_qv":   # every cluster converged: the QV pass reuses the final bands
        assert B.STATS["qv_refill_skipped"] == skipped + 2
    for a, b, c in zip(nat, hub, dqv):
        assert_same_run(summary(a), summary(b))
        assert_same_run(summary(c), summary(b), qv_rtol=QV_RTOL)
        _same_batches(a, b)
    if pset == "random_batch":      # drawn below the read count
        assert sum(len(r.state.batch_seqs) < len(k["dnaseqs"]) for r, k in zip(nat, clusters)) >= 4
    if pset == "random_grow":       # grown past the initial 3
        assert any(len(r.state.batch_seqs) > 3 for r in nat)


@pytest.mark.gpu
@pytest.mark.parametrize("random", [False, True])
def test_native_batch_matches_oracle_runs(run_engine, random):
    """Native batched clusters against separate rifraf() runs on the CPU
    oracle engine (reference-free clusters, quality scores on; random:
    batches of 4 drawn at random every iteration)."""
    engine = run_engine
    from oracle_engine import OracleEngine
    from rifraf_amd import ErrorModel, Scores
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams, rifraf
    extra = dict(batch_size=4, batch_fixed=False, seed=19) if random else {}
    params = RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)), do_score=True, max_iters=60, **extra)
    clusters = _ref_free_clusters(seed=5)[:5]
    ref = [rifraf(params=params, engine=OracleEngine(), **kw) for kw in clusters]
    got = rifraf_batch(clusters, params=params, engine=engine, native=True)
    for r, g in zip(ref, got):
        assert_same_run(summary(g), summary(r), qv_rtol=QV_RTOL)
        _same_batches(g, r)


def test_native_scope():
    """What takes the Python stage machine: an engine without the native
    driver, INIT disabled, reference QVs, bad reference scores, empty reads or
    mismatched quality vectors.  Random batches run natively."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import native_eligible, rifraf_batch
    from rifraf_amd.engine import RifrafError
    from rifraf_amd.model import RifrafParams
    clusters = _ref_free_clusters()
    assert native_eligible(clusters, RifrafParams())
    assert native_eligible(clusters, RifrafParams(batch_size=0, batch_fixed=False))
    assert native_eligible(clusters, RifrafParams(batch_size=4, batch_fixed=False))
    # references: native unless the QV pass scores the reference
    ref_clusters = _ref_clusters()
    assert native_eligible(ref_clusters, RifrafParams(batch_size=0, batch_fixed=False))
    assert native_eligible(ref_clusters, RifrafParams(batch_size=0))
    assert native_eligible(ref_clusters, RifrafParams(batch_size=5))
    assert native_eligible(ref_clusters, RifrafParams(batch_size=5, do_refine=False))
    assert not native_eligible(ref_clusters, RifrafParams(batch_size=0, do_score=True, use_ref_for_qvs=True))
    from rifraf_amd import ErrorModel, Scores
    bad_ref = RifrafParams(batch_size=0, ref_scores=Scores(-1.0, -1.0, -1.0, 0.0, -1.0))
    assert not native_eligible(ref_clusters, bad_ref)                # check_params: the hub raises it
    assert not native_eligible(clusters, RifrafParams(do_init=False))
    # an empty read or a quality vector of another length: the Python stage
    # machine (RifrafSequence's own handling), never a whole-wave native error
    empty = [dict(c) for c in clusters[:2]]
    empty[1]["dnaseqs"] = list(empty[1]["dnaseqs"][:-1]) + [np.zeros(0, np.int8)]
    empty[1]["phreds"] = list(empty[1]["phreds"][:-1]) + [np.zeros(0, np.int8)]
    assert not native_eligible(empty, RifrafParams())
    short = [dict(c) for c in clusters[:2]]
    short[0]["phreds"] = [p[:-1] if k == 0 else p for k, p in enumerate(short[0]["phreds"])]
    assert not native_eligible(short, RifrafParams())
    with pytest.raises(RifrafError):
        rifraf_batch(clusters[:1], params=RifrafParams(max_iters=2), engine=OracleEngine(), native=True)


def _ref_clusters(seed=41):
    """Clusters with a reference carrying a frameshift (INIT -> FRAME with
    codon scoring, seeded indel proposals, penalty increases -> REFINE),
    mixed with reference-free ones."""
    from rifraf_amd import ErrorModel
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(seed)
    out = []
    for n, L, shift in [(12, 300, 150), (20, 450, 200), (8, 240, 0), (15, 360, 90), (10, 200, -1),
                        (25, 420, 300)]:
        ref, _, _, reads, _, phreds, _, _ = sample_sequences(
            n, L, error_rate=0.02, ref_error_rate=0.1, ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
        ref = np.asarray(ref, np.uint8)
        if shift > 0:   # a one-base deletion and, later, a one-base insertion in the reference
            ref = np.concatenate([ref[:shift], ref[shift + 1:shift + 60], [2], ref[shift + 60:]]).astype(np.uint8)
        kw = dict(dnaseqs=reads, phreds=phreds)
        if shift >= 0:
            kw["reference"] = ref
        out.append(kw)
    return out


REF_PARAMS = {
    "throughput_qv": dict(batch_size=0, batch_fixed=False, do_score=True),
    "fixed_batch": dict(batch_size=0, batch_fixed=True, batch_fixed_size=4, max_iters=40),
    "unseeded_subs": dict(batch_size=0, batch_fixed=False, seed_indels=False, indel_correction_only=False,
                          max_ref_indel_mults=1, do_alignment_proposals=False, max_iters=30),
    "no_refine": dict(batch_size=6, do_refine=False, ref_error_mult=2.0, do_score=True),
    # the default fixed INIT / FRAME batch, then REFINE's random batches of 6
    "random_refine": dict(batch_size=6, seed=11, do_score=True),
}


@pytest.mark.gpu
@pytest.mark.parametrize("pset", sorted(REF_PARAMS))
def test_native_reference_batch_matches_hub(run_engine, pset):
    """rf_rifraf_batch_ref: reference-guided clusters (FRAME, REFINE) in the
    library's stage machine against the Python stage machine on the same
    engine -- consensus per iteration and stage, score, stage iterations,
    convergence, QVs, penalty increases and the reference's error rate."""
    engine = run_engine
    from rifraf_amd import ErrorModel, Scores
    from rifraf_amd.batch import native_eligible, rifraf_batch
    from rifraf_amd.model import RifrafParams
    params = RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)), **REF_PARAMS[pset])
    clusters = _ref_clusters()
    assert native_eligible(clusters, params)
    hub = rifraf_batch(clusters, params=params, engine=engine, native=False)
    nat = rifraf_batch(clusters, params=params, engine=engine, native=True, device_qv=False)
    dqv = rifraf_batch(clusters, params=params, engine=engine, native=True)
    frames = 0
    for a, b, c in zip(nat, hub, dqv):
        assert_same_run(summary(a), summary(b))
        assert_same_run(summary(c), summary(b), qv_rtol=QV_RTOL)
        assert a.state.n_ref_indel_mults == b.state.n_ref_indel_mults
        assert a.state.ref_error_rate == b.state.ref_error_rate or (
            np.isinf(a.state.ref_error_rate) and np.isinf(b.state.ref_error_rate))
        assert a.state.reference.bandwidth == b.state.reference.bandwidth
        _same_batches(a, b)
        frames += a.state.stage_iterations[1] > 0
    assert frames >= 3
    if pset == "throughput_qv":   # the whole FRAME path: penalty increases, then REFINE
        assert any(r.state.n_ref_indel_mults >= 1 for r in nat)
        assert any(r.state.stage_iterations[2] > 0 for r in nat)
    if pset == "random_refine":   # random REFINE batches below the read count
        assert any(r.state.stage_iterations[2] > 0 and len(r.state.batch_seqs) < len(k["dnaseqs"])
                   for r, k in zip(nat, clusters))


@pytest.mark.gpu
def test_native_reference_batch_matches_oracle_runs(run_engine):
    """Native reference-guided clusters against separate rifraf() runs on the
    CPU oracle engine (throughput settings, QVs on)."""
    engine = run_engine
    from oracle_engine import OracleEngine
    from rifraf_amd import ErrorModel, Scores
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams, rifraf
    params = RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)), **REF_PARAMS["throughput_qv"])
    clusters = _ref_clusters(seed=43)[:4]
    ref = [summary(rifraf(params=params, engine=OracleEngine(), **kw)) for kw in clusters]
    got = rifraf_batch(clusters, params=params, engine=engine, native=True)
    for r, g in zip(ref, got):
        assert_same_run(summary(g), r, qv_rtol=QV_RTOL)


@pytest.mark.gpu
def test_native_auto_with_empty_read(run_engine):
    """rifraf_batch's automatic driver choice (native=None) with an empty read
    in one cluster gives what the Python stage machine gives (native=False):
    the same results, or the same error."""
    engine = run_engine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams
    clusters = [dict(c) for c in _ref_free_clusters()[:3]]
    clusters[1]["dnaseqs"] = list(clusters[1]["dnaseqs"]) + [np.zeros(0, np.int8)]
    clusters[1]["phreds"] = list(clusters[1]["phreds"]) + [np.zeros(0, np.int8)]
    params = RifrafParams(batch_size=0, batch_fixed=False, max_iters=10)

    def run(native):
        try:
            return [summary(r) for r in rifraf_batch(clusters, params=params, engine=engine, native=native)]
        except Exception as e:   # noqa: BLE001 - the error itself is compared
            return (type(e).__name__, str(e))
    a, b = run(None), run(False)
    if isinstance(b, tuple):
        assert a == b
    else:
        for x, y in zip(a, b):
            assert_same_run(x, y)


@pytest.mark.gpu
def test_native_scope_error_message(engine):
    """rf_rifraf_batch refuses a cluster outside its scope with its own
    rf_last_error text, not a stale message of an earlier call."""
    from rifraf_amd import _lib
    from rifraf_amd.engine import RifrafError
    bp = _lib.BatchParams(10, 15, 9, 1, 0, 0, 0.1)
    with pytest.raises(RifrafError, match="cluster 1 is outside the native driver's scope .no reads."):
        engine.rifraf_batch_native(bp, [0, 1, 1], [0], [10], [1.0], None, None, [0, 1], [0, 1],
                                   np.zeros(20, np.uint8), [0, 10, 20])


def _doubling_clusters(seed=12):
    """Reference-free clusters in which one read per cluster carries a run of
    deletions: its band doubles (smart_forward_moves!) to H >= 64, so the
    driver's forward, refill and backward calls differ in row padding."""
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(seed)
    out = []
    for n, L, cut in [(10, 400, 30), (8, 300, 26), (12, 350, 0)]:
        _, _, _, reads, _, phreds, _, _ = sample_sequences(n, L, error_rate=0.01, rng=rng)
        reads, phreds = list(reads), list(phreds)
        if cut:
            k = int(rng.integers(0, n))
            at = int(rng.integers(50, L - 50 - cut))
            reads[k] = np.concatenate([reads[k][:at], reads[k][at + cut:]])
            phreds[k] = np.concatenate([phreds[k][:at], phreds[k][at + cut:]])
        out.append(dict(dnaseqs=reads, phreds=phreds))
    return out


@pytest.mark.gpu
def test_native_batch_band_doubling_vs_oracle(run_engine):
    """Native batched driver with band doubling into line-padded layouts (the
    c4 e2e shape's failure mode: A and B of one read filled by calls that
    differ in padding) against separate oracle-engine rifraf() runs, QVs on."""
    engine = run_engine
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams, rifraf
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True, max_iters=20)
    clusters = _doubling_clusters()
    got = rifraf_batch(clusters, params=params, engine=engine, native=True)
    # bw >= 18 with |n - m| ~ 30: H = 2 bw + |n - m| + 1 >= 64 (a padded call)
    assert max(s.bandwidth for r in got for s in r.state.sequences) >= 18
    ref = [summary(rifraf(params=params, engine=OracleEngine(), **kw)) for kw in clusters]
    for r, g in zip(ref, got):
        assert_same_run(summary(g), r, qv_rtol=QV_RTOL)


@pytest.mark.gpu
def test_native_batch_engines_one_gpu(run_engine):
    """Three contexts on one GPU, one host thread each (rifraf_batch(engines=)),
    equal the single-engine native run."""
    engine = run_engine
    from rifraf_amd import ErrorModel, Scores
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.engine import Engine
    from rifraf_amd.model import RifrafParams
    params = RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)), **NATIVE_PARAMS["all_reads_qv"])
    clusters = _ref_free_clusters() + _ref_free_clusters(seed=3)
    one = rifraf_batch(clusters, params=params, engine=engine, native=True)
    engs = [Engine(0) for _ in range(3)]
    try:
        many = rifraf_batch(clusters, params=params, engines=engs, native=True)
        piped = rifraf_batch(clusters, params=params, engines=engs[:2], native=True, wave=3, init_exclusive=True)
    finally:
        for e in engs:
            e.close()
    for a, b, c in zip(many, one, piped):
        assert_same_run(summary(a), summary(b))
        assert_same_run(summary(c), summary(b))


@pytest.mark.gpu
@pytest.mark.parametrize("marks_min", [128, 0])
def test_aln_error_sums_device_equals_host(run_engine, opts, marks_min):
    """alignment_error_probs's sums (model.jl:817-840) folded on the device
    (k_aln_sums, default; with marks_min 0 the per-read marks + per-column
    fold launches that large clusters use) and on host threads
    (RF_OPT_ALN_SUMS_HOST) are the same bits, through the native driver's
    host quality pass (device_qv=False); both equal the Python stage
    machine's."""
    engine = run_engine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True, max_iters=20)
    clusters = _ref_free_clusters(seed=21) + _doubling_clusters()
    opts("aln_marks_min", marks_min)
    dev = rifraf_batch(clusters, params=params, engine=engine, native=True, device_qv=False)
    opts("aln_sums_host", 1)
    host = rifraf_batch(clusters, params=params, engine=engine, native=True, device_qv=False)
    hub = rifraf_batch(clusters, params=params, engine=engine, native=False)
    for a, b, c in zip(dev, host, hub):
        np.testing.assert_array_equal(a.aln_error_probs, b.aln_error_probs)
        assert_same_run(summary(a), summary(c))


@pytest.mark.gpu
def test_native_batch_packed_reads(run_engine):
    """The native driver's packed-input path (PackedReads clusters: one
    buffer + offsets, what bench's e2e staging and FASTQ ingest hand over)
    gives the same runs as the same reads as lists."""
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams
    from rifraf_amd.sample import sample_sequences
    from rifraf_amd.types import PackedReads
    rng = np.random.default_rng(8)
    cl, pk = [], []
    for n, L in [(12, 300), (7, 240), (20, 180)]:
        _, _, _, reads, _, phreds, _, _ = sample_sequences(n, L, error_rate=0.02, rng=rng)
        cl.append(dict(dnaseqs=reads, phreds=phreds))
        pk.append(dict(dnaseqs=PackedReads.from_list(reads, np.uint8), phreds=PackedReads.from_list(phreds, np.int8)))
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
    a = rifraf_batch(cl, params=params, engine=run_engine, native=True)
    b = rifraf_batch(pk, params=params, engine=run_engine, native=True)
    for x, y in zip(a, b):
        assert_same_run(summary(x), summary(y))
