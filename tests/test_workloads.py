"""HIP engine vs the CPU oracle at the BASELINE.json workload shapes.

Every other parity test uses small inputs; these run the configs' own shapes
(SURVEY.md §8(d)):

  c2  sample_sequences(100, 1000; error_rate=0.01), no reference: whole
      rifraf() runs, default params and the throughput settings with the QV
      pass (do_score): same consensus after every iteration, same score bits,
      same accepted proposals, same error_probs / aln_error_probs bits;
  c3  sample_sequences(1000, 2601; error_rate=0.01, ref_error_rate=0.1,
      ref_errors=ErrorModel(10,0,0,1,1)) with a one-base frameshift in the
      reference so that FRAME runs (codon scoring of the reference, penalty
      increases, seeded indel proposals): same run as the oracle engine,
      default params and the throughput settings (all 1000 reads, QVs);
  c4  clusters of 50 reads x 1.5 kb (bench.make_workload): rf_score_dense of
      every STAGE_SCORE proposal vs oracle.cpu_pass, bit-exact; and two
      whole runs at the throughput settings (all reads, QVs) on the Python
      stage machine and the native driver;
  c5  the first 64 / 256 reads of the bench's 10 kb / 3 % error cluster
      (bench.make_read_shard): band doubling (smart_forward_moves!,
      model.jl:643-672) gives the same bandwidth and A[end,end] per read on
      both engines; bands at the doubled widths and the dense totals are
      bit-exact.

The oracle engine is tests/oracle_engine.py (C oracle behind the Engine
API); tolerance everywhere: bit-exact (north_star allows 1e-9 relative).
"""
import copy
import os
from types import SimpleNamespace

import numpy as np
import pytest

import oracle
from rifraf_amd import ErrorModel
from rifraf_amd.engine import RF_BAND_A, RF_BAND_B, RF_BWD, RF_FWD
from rifraf_amd.model import RifrafParams, rifraf, smart_forward_moves
from rifraf_amd.sample import sample_sequences

pytestmark = pytest.mark.gpu
NTHREADS = min(16, os.cpu_count() or 1)


def assert_same_run(a, b, qv_rtol=0.0):
    """qv_rtol > 0: the QVs within that relative tolerance (+ 1e-15
    absolute) -- a native run's device quality pass against a host one."""
    np.testing.assert_array_equal(a.consensus, b.consensus)
    assert a.state.score == b.state.score
    assert a.state.stage_iterations == b.state.stage_iterations
    assert a.state.converged == b.state.converged
    for sa, sb in zip(a.consensus_stages, b.consensus_stages):
        assert len(sa) == len(sb)
        for x, y in zip(sa, sb):
            np.testing.assert_array_equal(x, y)
    if a.error_probs is None:
        assert b.error_probs is None
    else:
        for f in ("sub", "dele", "ins"):
            if qv_rtol:
                np.testing.assert_allclose(getattr(a.error_probs, f), getattr(b.error_probs, f), rtol=qv_rtol,
                                           atol=1e-15, err_msg=f)
            else:
                np.testing.assert_array_equal(getattr(a.error_probs, f), getattr(b.error_probs, f), err_msg=f)
        if qv_rtol:
            np.testing.assert_allclose(a.aln_error_probs, b.aln_error_probs, rtol=qv_rtol, atol=1e-15)
        else:
            np.testing.assert_array_equal(a.aln_error_probs, b.aln_error_probs)


def _masked(got, ref, t):
    mask = np.ones_like(ref, bool)
    mask[0, :5] = False                       # p = 0 has no sub / del
    mask[np.arange(1, len(t) + 1), np.asarray(t, np.int64)] = False   # the consensus base is no proposal
    return got[mask], ref[mask]


@pytest.mark.parametrize("variant", ["default", "throughput_qv"])
def test_c2_run_matches_oracle(run_engine, oracle_memo, variant):
    from oracle_engine import OracleEngine
    rng = np.random.default_rng(2)
    _, template, _, reads, _, phreds, _, _ = sample_sequences(100, 1000, error_rate=0.01, rng=rng)
    params = (RifrafParams(seed=1) if variant == "default" else
              RifrafParams(seed=1, batch_size=0, batch_fixed=False, do_score=True))
    a = rifraf(reads, phreds, params=params, engine=run_engine)
    b = oracle_memo(("c2", variant), lambda: rifraf(reads, phreds, params=params, engine=OracleEngine()))
    assert_same_run(a, b)
    assert a.state.converged and np.array_equal(a.consensus, template)


def test_c3_frame_run_matches_oracle(run_engine, oracle_memo):
    from oracle_engine import OracleEngine
    rng = np.random.default_rng(3)
    ref, template, _, reads, _, phreds, _, _ = sample_sequences(
        1000, 2601, error_rate=0.01, ref_error_rate=0.1, ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
    # a single-base frameshift in the reference: INIT -> FRAME with codon scoring
    ref = np.concatenate([ref[:1300], ref[1301:2000], [2], ref[2000:]]).astype(np.uint8)
    params = RifrafParams(seed=1)
    a = rifraf(reads, phreds, reference=ref, params=params, engine=run_engine)
    b = oracle_memo("c3_default", lambda: rifraf(reads, phreds, reference=ref, params=params,
                                                 engine=OracleEngine()))
    assert_same_run(a, b)
    assert a.state.stage_iterations[1] >= 2          # FRAME ran (with a penalty increase)
    assert a.state.n_ref_indel_mults == b.state.n_ref_indel_mults >= 1
    # the library's stage machine: REFINE's random batches of 20 drawn there
    from rifraf_amd.batch import rifraf_batch
    n = rifraf_batch([dict(dnaseqs=reads, phreds=phreds, reference=ref)], params=params, engine=run_engine,
                     native=True)[0]
    assert_same_run(n, b)
    assert [int(i) for i in n.state.batch_seqs] == [int(i) for i in b.state.batch_seqs]
    assert len(b.state.batch_seqs) < len(reads)


def test_c3_throughput_frame_run_matches_oracle(run_engine, oracle_memo):
    """Config 3 at the throughput settings (SURVEY §8(d) "Parity runs"):
    every one of the 1000 reads in every batch (batch_size 0, batch_fixed
    false, model.jl:569-573) through INIT, FRAME (frameshifted reference:
    codon scoring, seeded indel proposals, penalty increases) and REFINE,
    with the QV pass: the same run as the oracle engine, bit for bit."""
    from oracle_engine import OracleEngine
    rng = np.random.default_rng(3)
    ref, template, _, reads, _, phreds, _, _ = sample_sequences(
        1000, 2601, error_rate=0.01, ref_error_rate=0.1, ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
    ref = np.concatenate([ref[:1300], ref[1301:2000], [2], ref[2000:]]).astype(np.uint8)
    params = RifrafParams(seed=1, batch_size=0, batch_fixed=False, do_score=True)
    engine = run_engine
    a = rifraf(reads, phreds, reference=ref, params=params, engine=engine)
    b = oracle_memo("c3_throughput", lambda: rifraf(reads, phreds, reference=ref, params=params,
                                                    engine=OracleEngine()))
    assert_same_run(a, b)
    assert a.state.batch_size == 1000
    assert a.state.stage_iterations[1] >= 2 and a.state.n_ref_indel_mults >= 1
    assert np.array_equal(a.consensus, template)
    # the same cluster through the library's stage machine (rf_rifraf_batch_ref)
    from rifraf_amd.batch import native_eligible, rifraf_batch
    kw = dict(dnaseqs=reads, phreds=phreds, reference=ref)
    assert native_eligible([kw], params)
    n = rifraf_batch([kw], params=params, engine=engine, native=True)[0]
    assert_same_run(n, b, qv_rtol=1e-12)        # device quality pass
    n0 = rifraf_batch([kw], params=params, engine=engine, native=True, device_qv=False)[0]
    assert_same_run(n0, b)
    assert n.state.n_ref_indel_mults == b.state.n_ref_indel_mults


def test_c3_qv_with_reference_matches_oracle(run_engine, oracle_memo):
    """QV pass scoring the reference's codon moves too (use_ref_for_qvs,
    model.jl:617-628, :737-791), 2.6 kb template, 40 reads."""
    from oracle_engine import OracleEngine
    rng = np.random.default_rng(33)
    ref, _, _, reads, _, phreds, _, _ = sample_sequences(
        40, 2601, error_rate=0.01, ref_error_rate=0.1, ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
    params = RifrafParams(seed=1, do_score=True, use_ref_for_qvs=True)
    a = rifraf(reads, phreds, reference=ref, params=params, engine=run_engine)
    b = oracle_memo("c3_qv_ref", lambda: rifraf(reads, phreds, reference=ref, params=params,
                                                engine=OracleEngine()))
    assert_same_run(a, b)


def _c4_clusters(n, seed=77):
    """c4 cluster shape from the e2e bench leg: sample_sequences(50, 1500)."""
    out = []
    for k in range(n):
        _, t, _, reads, _, phreds, _, _ = sample_sequences(50, 1500, error_rate=0.01,
                                                           rng=np.random.default_rng([seed, k]))
        out.append((t, dict(dnaseqs=reads, phreds=phreds)))
    return out


def test_c4_throughput_runs_match_oracle(run_engine, oracle_memo):
    """SURVEY §8(d) config 4 at its throughput settings (batch = all 50
    reads, QV pass on), two clusters as whole rifraf() runs: the HIP engine
    through the Python stage machine, through rf_rifraf_batch (the native
    lockstep driver), and the oracle engine agree run for run."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
    clusters = _c4_clusters(2)
    nat = rifraf_batch([kw for _, kw in clusters], params=params, engine=run_engine, native=True)
    for c, ((t, kw), n) in enumerate(zip(clusters, nat)):
        a = rifraf(params=params, engine=run_engine, **kw)
        b = oracle_memo(("c4_run", c), lambda: rifraf(params=params, engine=OracleEngine(), **kw))
        assert_same_run(a, b)
        assert_same_run(n, b, qv_rtol=1e-12)    # device quality pass
        assert b.error_probs is not None


def test_c4_clusters_dense_bitexact(run_engine):
    engine = run_engine
    import bench
    clusters = bench.make_workload(4, 50, 1500, 0.01, 9, seed=bench.shard_seed(2024, 0))
    reads = [r for _, rs in clusters for r in rs]
    n = len(reads)
    engine.set_sequences(0, reads)
    engine.set_templates(0, [t for t, _ in clusters])
    tpl = np.repeat(np.arange(len(clusters)), 50)
    engine.realign(np.arange(n), np.arange(n), tpl, [r.bandwidth for r in reads], RF_FWD | RF_BWD)
    groups = [np.arange(50 * c, 50 * c + 50) for c in range(len(clusters))]
    got = engine.score_dense(groups)
    for c, (t, rs) in enumerate(clusters):
        ref, _ = oracle.cpu_pass(t, rs, nthreads=NTHREADS)
        g, e = _masked(got[c], ref, t)
        np.testing.assert_array_equal(g, e, err_msg=f"cluster {c}")


@pytest.mark.parametrize("nreads", [64, 256])
def test_c5_sample_band_doubling_and_scores(run_engine, nreads):
    engine = run_engine
    import bench
    from oracle_engine import OracleEngine
    t, reads = bench.make_read_shard(5000, 10000, 0.03, 9, 2024, 0, nreads)
    m = len(t)
    # band doubling on both engines (each mutates its own RifrafSequence copies)
    rh = [copy.copy(r) for r in reads]
    ro = [copy.copy(r) for r in reads]
    engine.set_sequences(0, rh)
    engine.set_templates(0, [t])
    oe = OracleEngine()
    oe.set_sequences(0, ro)
    oe.set_templates(0, [t])
    jobs = [(k, k) for k in range(len(reads))]
    sh = smart_forward_moves(SimpleNamespace(e=engine), jobs, rh, m, 0.1)
    so = smart_forward_moves(SimpleNamespace(e=oe), jobs, ro, m, 0.1)
    bw_h = [r.bandwidth for r in rh]
    assert bw_h == [r.bandwidth for r in ro]
    np.testing.assert_array_equal(sh, so)
    assert sum(b > 9 for b in bw_h) >= len(reads) // 2      # the config's point: most reads double
    # bands at the doubled widths, and every STAGE_SCORE total
    n = len(rh)
    engine.realign(np.arange(n), np.arange(n), 0, bw_h, RF_FWD | RF_BWD)
    for k in (0, 1, n // 2, n - 1):
        A_exp, _ = oracle.forward(t, rh[k], bandwidth=bw_h[k])
        B_exp = oracle.backward(t, rh[k], bandwidth=bw_h[k])
        from test_gpu_parity import assert_band_equal
        assert_band_equal(engine.download_band(k, RF_BAND_A), A_exp, len(rh[k]) + 1, m + 1, bw_h[k])
        assert_band_equal(engine.download_band(k, RF_BAND_B), B_exp, len(rh[k]) + 1, m + 1, bw_h[k])
    got = engine.score_dense([np.arange(n)])[0]
    ref, _ = oracle.cpu_pass(t, rh, nthreads=NTHREADS)
    g, e = _masked(got, ref, t)
    np.testing.assert_array_equal(g, e)


def _progress(msg):
    """A line per stage under gpurun_out/ (a long test keeps the GPU call's
    output moving; captured stdout would not)."""
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    try:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "c5_full_parity.log"), "a") as f:
            f.write(msg + "\n")
    except OSError:
        pass


@pytest.mark.timeout(600)
def test_c5_full_cluster_dense_bitexact():
    """The bench's whole c5 cluster (5,000 reads x 10 kb, 3 % error) at its
    final bandwidths: band doubling on the GPU (smart_forward_moves!,
    model.jl:643-672), fwd + bwd DP, and the dense fold of all 80,004
    STAGE_SCORE proposals over all 5,000 reads -- the split-mode scorer plus
    its cross-read fold, exactly the path bench --config c5 times -- against
    oracle.cpu_pass folding the same reads in batch order (model.jl:385-399),
    chunk by chunk (oracle.cpu_pass(totals=...) continues the fold), on every
    core.  Bit-exact."""
    import time
    import bench
    from rifraf_amd.bandedarrays import BAND_PAD_H
    from rifraf_amd.engine import Engine
    t0 = time.time()
    t, reads = bench.make_read_shard(5000, 10000, 0.03, 9, 2024, 0, 5000)
    m = len(t)
    n = len(reads)
    _progress(f"generated {n} reads in {time.time() - t0:.0f} s")
    e = Engine(0)
    try:
        e.reserve(sum(bench.band_bytes(len(r), m, 9) + bench.band_bytes(len(r), m, 18, pad=True) for r in reads)
                  + (256 << 20))
        for a in range(0, n, 1024):
            e.set_sequences(a, reads[a:a + 1024])
        e.set_templates(0, [t])
        smart_forward_moves(SimpleNamespace(e=e), [(k, k) for k in range(n)], reads, m, 0.1)
    finally:
        e.close()
    bws = [r.bandwidth for r in reads]
    assert sum(b > 9 for b in bws) >= n // 2
    _progress(f"band doubling done, {sum(b > 9 for b in bws)} reads doubled")
    e = Engine(0)
    try:
        pad = max(2 * r.bandwidth + abs(len(r) - m) + 1 for r in reads) >= BAND_PAD_H
        e.reserve(sum(2 * bench.band_bytes(len(r), m, r.bandwidth, pad) for r in reads) + (256 << 20))
        for a in range(0, n, 1024):
            e.set_sequences(a, reads[a:a + 1024])
        e.set_templates(0, [t])
        e.realign(np.arange(n), np.arange(n), 0, bws, RF_FWD | RF_BWD)
        got = e.score_dense([np.arange(n)])[0]
    finally:
        e.close()
    _progress(f"GPU pass done at {time.time() - t0:.0f} s")
    ref = None
    for a in range(0, n, 400):
        if ref is None:
            ref, _ = oracle.cpu_pass(t, reads[a:a + 400], nthreads=NTHREADS)
        else:
            oracle.cpu_pass(t, reads[a:a + 400], nthreads=NTHREADS, totals=ref)
        _progress(f"oracle reads {a}..{min(a + 400, n)} folded at {time.time() - t0:.0f} s")
    g, x = _masked(got, ref, t)
    np.testing.assert_array_equal(g, x)
