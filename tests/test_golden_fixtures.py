"""Committed golden fixtures (tests/golden/pairs.npz, config2.json, runs.npz; made by
scripts/make_golden.py from the KAT-pinned oracle).

CPU: the oracle still reproduces them (guards the checker against drift).
GPU: the HIP engine reproduces them bit for bit -- bands, A[end,end],
backtrace moves and error counts, every STAGE_SCORE proposal total, and
whole rifraf() runs (consensus, score)."""
import json
import os

import numpy as np
import pytest

import oracle
from _util import REF_SCORES, SEQ_SCORES, inband_mask
from rifraf_amd import RifrafSequence, dna_str
from rifraf_amd.engine import RF_BAND_A, RF_BAND_B, RF_BWD, RF_FWD

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _pairs():
    z = np.load(os.path.join(G, "pairs.npz"))
    out = []
    for k in range(int(z["npairs"])):
        g = {key: z[f"p{k}_{key}"] for key in ("template", "read", "lp", "bw", "codon", "A", "B", "score",
                                               "moves", "nerr", "kind", "pos", "base", "totals")}
        codon = bool(g["codon"])
        g["seq"] = RifrafSequence(g["read"], g["lp"], int(g["bw"]), REF_SCORES if codon else SEQ_SCORES)
        out.append(g)
    return out


PAIRS = _pairs()


def _inband(data, n, m, bw):
    return np.asarray(data).T[inband_mask(n + 1, m + 1, bw).T]


@pytest.mark.parametrize("k", range(len(PAIRS)))
def test_oracle_reproduces_pairs(k):
    g = PAIRS[k]
    t, s, bw = g["template"], g["seq"], int(g["bw"])
    A, mv = oracle.forward(t, s, moves=True)
    B = oracle.backward(t, s)
    n, m = len(s), len(t)
    np.testing.assert_array_equal(_inband(A, n, m, bw), g["A"])
    np.testing.assert_array_equal(_inband(B, n, m, bw), g["B"])
    moves = oracle.backtrace(mv, n + 1, m + 1, bw)
    np.testing.assert_array_equal(moves, g["moves"])
    assert oracle.count_errors(moves, t, s.seq) == int(g["nerr"])
    for i in range(0, len(g["totals"]), 11):
        assert 0.0 + oracle.score_proposal(int(g["kind"][i]), int(g["pos"][i]), int(g["base"][i]),
                                           A, B, t, s) == g["totals"][i]


def test_oracle_engine_reproduces_config2():
    from oracle_engine import OracleEngine
    _check_config2(OracleEngine())


def _check_config2(engine):
    from rifraf_amd.model import RifrafParams, rifraf
    from rifraf_amd.sample import sample_sequences
    runs = json.load(open(os.path.join(G, "config2.json")))["runs"]
    for r in runs:
        rng = np.random.default_rng(r["seed"])
        _, t, _, reads, _, phreds, _, _ = sample_sequences(r["nreads"], r["length"], error_rate=r["error_rate"],
                                                           rng=rng)
        assert dna_str(t) == r["template"]
        res = rifraf(reads, phreds, params=RifrafParams(), engine=engine)
        assert dna_str(res.consensus) == r["consensus"]
        assert res.state.score.hex() == r["score"]
        assert list(res.state.stage_iterations) == r["stage_iterations"]


@pytest.mark.gpu
def test_engine_reproduces_pairs(run_engine):
    engine = run_engine
    seqs = [g["seq"] for g in PAIRS]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [g["template"] for g in PAIRS])
    n = len(PAIRS)
    bws = [int(g["bw"]) for g in PAIRS]
    scores = engine.realign(np.arange(n), np.arange(n), np.arange(n), bws, RF_FWD | RF_BWD)
    moves, nerr = engine.backtrace(np.arange(n))
    for k, g in enumerate(PAIRS):
        nr, m, bw = len(g["seq"]), len(g["template"]), bws[k]
        A = engine.download_band(k, RF_BAND_A)
        B = engine.download_band(k, RF_BAND_B)
        np.testing.assert_array_equal(_inband(A.data, nr, m, bw), g["A"], err_msg=f"pair {k}")
        np.testing.assert_array_equal(_inband(B.data, nr, m, bw), g["B"], err_msg=f"pair {k}")
        assert scores[k] == g["score"]
        np.testing.assert_array_equal(moves[k], g["moves"])
        assert nerr[k] == int(g["nerr"])
        if len(g["totals"]):
            props = (g["kind"], g["pos"], g["base"])
            group = ([], k, props) if bool(g["codon"]) else ([k], -1, props)
            got = engine.score([group])[0]
            np.testing.assert_array_equal(got, g["totals"], err_msg=f"pair {k}")


@pytest.mark.gpu
def test_engine_reproduces_config2(run_engine):
    engine = run_engine
    _check_config2(engine)


def _run_fixture():
    import bench
    return bench, np.load(bench.GOLDEN_RUNS)


@pytest.mark.parametrize("variant", ["default", "throughput"])
def test_oracle_engine_reproduces_runs(variant):
    """tests/golden/runs.npz (bench's c2 / c3 fields check against it): the
    oracle engine still gives configs[1]'s seed-1 runs bit for bit."""
    from oracle_engine import OracleEngine
    from rifraf_amd.model import RifrafParams, rifraf
    bench, z = _run_fixture()
    t, reads, phreds = bench.c2_cluster(1)
    res = rifraf(reads, phreds, params=RifrafParams(**bench.C2_VARIANTS[variant]), engine=OracleEngine())
    assert bench.run_matches(res, bench.golden_run(f"c2_1_{variant}", z), qv_rtol=0)
    assert np.array_equal(res.consensus, t)


def test_oracle_engine_reproduces_c3_default_run():
    """runs.npz's c3_default (bench's c3.default field): configs[2] with the
    default batches -- REFINE draws random batches of 20 (resampling.py) --
    on the oracle engine, final batch included."""
    from oracle_engine import OracleEngine
    from rifraf_amd.model import RifrafParams, rifraf
    bench, z = _run_fixture()
    t, reads, phreds, ref = bench.c3_cluster()
    res = rifraf(reads, phreds, reference=ref, params=RifrafParams(**bench.C3_DEFAULT), engine=OracleEngine())
    rec = bench.golden_run("c3_default", z)
    assert bench.run_matches(res, rec, qv_rtol=0)
    assert res.state.stage_iterations[2] >= 1 and len(rec["batch"]) == 20


@pytest.mark.gpu
def test_engine_reproduces_c3_default_run(run_engine):
    """The same run through the library's stage machine (its own random
    draws) and the Python stage machine on the HIP engine."""
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams, rifraf
    bench, z = _run_fixture()
    t, reads, phreds, ref = bench.c3_cluster()
    params = RifrafParams(**bench.C3_DEFAULT)
    rec = bench.golden_run("c3_default", z)
    nat = rifraf_batch([dict(dnaseqs=reads, phreds=phreds, reference=ref)], params=params, engine=run_engine,
                       native=True)[0]
    assert bench.run_matches(nat, rec)
    py = rifraf(reads, phreds, reference=ref, params=params, engine=run_engine)
    assert bench.run_matches(py, rec, qv_rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["default", "throughput"])
def test_engine_reproduces_runs(run_engine, variant):
    """configs[1] (100 reads x 1 kb), seeds 1..5, through the library's stage
    machine (rf_rifraf_batch: what bench's c2 field times) and, for seed 1,
    the Python stage machine, against the oracle engine's committed runs:
    consensus per stage, score bits, iterations exact; QVs bit-exact on the
    host quality pass, within 1e-12 on the device one."""
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams, rifraf
    bench, z = _run_fixture()
    params = RifrafParams(**bench.C2_VARIANTS[variant])
    for seed in bench.C2_SEEDS:
        t, reads, phreds = bench.c2_cluster(seed)
        rec = bench.golden_run(f"c2_{seed}_{variant}", z)
        nat = rifraf_batch([dict(dnaseqs=reads, phreds=phreds)], params=params, engine=run_engine, native=True)[0]
        assert bench.run_matches(nat, rec), f"seed {seed}"
        if seed == 1:
            py = rifraf(reads, phreds, params=params, engine=run_engine)
            assert bench.run_matches(py, rec, qv_rtol=0)
