"""resample!'s random batch (model.jl:998-1066, rifraf_amd/resampling.py):
the RNG against the published splitmix64 / xoshiro256++ known answers, and
the draw's properties.  The native driver's copy (rifraf_batch.cpp) is
checked against this one on the GPU (test_batch.py: the random-batch runs
and their final batches)."""
import numpy as np

from rifraf_amd.resampling import (BatchRng, cluster_seeds, error_weights, random_batch, reweight, splitmix64,
                                   wsample_norep)


def test_xoshiro256pp_known_answers():
    """The reference implementation (Blackman, Vigna) from state {1, 2, 3, 4}."""
    r = BatchRng(state=[1, 2, 3, 4])
    assert [r.next_u64() for _ in range(10)] == [
        41943041, 58720359, 3588806011781223, 3591011842654386, 9228616714210784205, 9973669472204895162,
        14011001112246962877, 12406186145184390807, 15849039046786891736, 10450023813501588000]


def test_splitmix64_known_answers():
    x, out = 1234567, []
    for _ in range(5):
        x, z = splitmix64(x)
        out.append(z)
    assert out == [6457827717110365317, 3203168211198807973, 9817491932198370423, 4593380528125082431,
                   16408922859458223821]


def test_rand_is_53_bit_uniform():
    r = BatchRng(9)
    u = np.array([r.rand() for _ in range(20000)])
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01
    assert all(float(v * 2.0 ** 53).is_integer() for v in u[:100])


def test_same_seed_same_batches():
    est = np.linspace(0.5, 9.0, 40)
    a, b = BatchRng(123), BatchRng(123)
    for rnd in (0.9, 0.63, 0.441, 0.0):
        x = random_batch(a, est, 7, rnd)
        assert x == random_batch(b, est, 7, rnd)
        assert len(set(x)) == 7 and all(0 <= i < 40 for i in x)
    assert random_batch(BatchRng(1), est, 7, 0.9) != random_batch(BatchRng(2), est, 7, 0.9)


def test_zero_randomness_takes_the_lowest_error_reads():
    """randomness 0: every weight outside the top n is 0 (model.jl:1027-1030),
    so the draw is the n reads of fewest estimated errors, in some order."""
    rng = np.random.default_rng(4)
    est = rng.uniform(1.0, 20.0, 30)
    x = random_batch(BatchRng(5), est, 6, 0.0)
    assert sorted(x) == sorted(np.argsort(est)[:6].tolist())


def test_first_draw_follows_the_weights():
    w = np.array([1.0, 2.0, 3.0, 4.0])
    counts = np.zeros(4)
    r = BatchRng(77)
    for _ in range(20000):
        counts[wsample_norep(r, w, 1)[0]] += 1
    np.testing.assert_allclose(counts / counts.sum(), w / w.sum(), atol=0.015)


def test_reweight_endpoints():
    wv = error_weights([2.0, 4.0, 6.0, 8.0])
    np.testing.assert_allclose(reweight(wv, 2, 1.0), np.full(4, 0.25))
    np.testing.assert_allclose(reweight(wv, 2, 0.5), wv / wv.sum())
    np.testing.assert_allclose(reweight(wv, 2, 0.0), [0.5, 0.5, 0.0, 0.0])


def test_cluster_seeds():
    assert (cluster_seeds(5, 3) == 5).all()
    s = cluster_seeds(None, 64)
    assert s.dtype == np.uint64 and len(set(s.tolist())) == 64


def test_model_resample_draws_from_the_shared_sampler():
    """model.resample's random branch is resampling.random_batch on the
    run's RNG, and sets realign_As (model.jl:1055-1058)."""
    from types import SimpleNamespace

    from rifraf_amd.model import RifrafParams, Stage, resample
    est = [3.0, 1.0, 4.0, 1.5, 9.0, 2.6, 5.0, 3.5]
    st = SimpleNamespace(sequences=[SimpleNamespace(est_n_errors=e) for e in est], stage=Stage.REFINE,
                         batch_size=3, batch_randomness=0.9, batch_seqs=[], realign_As=False,
                         batch_fixed_size=2)
    resample(st, RifrafParams(), BatchRng(31))
    assert st.batch_seqs == random_batch(BatchRng(31), est, 3, 0.9) and st.realign_As
    st.stage = Stage.INIT
    resample(st, RifrafParams(), BatchRng(31))
    assert st.batch_seqs == [1, 3]                    # fixed batch: the two lowest est_n_errors
