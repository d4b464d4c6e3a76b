"""The fused-step prototype (RF_OPT_SCORE_FWD, k_fuse): rf_score_dense with the
forward band filled inside the scorer from the B bands alone.

Bit-exact against the product path (k_dpr A + k_score_ws / k_reduce) and the
oracle on the same seeded inputs: both task classes (16 lanes for H <= 31,
64 lanes for H 32..127, line-padded rows once a call holds an H >= 64 band),
bw 1..30, reads longer and shorter than the template, tiny reads and templates
(the band corners, c > m), the bench's c4 clusters.  Reference:
align.jl:155-179 (forward!), model.jl:242-285 (score_nocodon), :389-393 (fold).
"""
import numpy as np
import pytest

import oracle
from _util import SEQ_SCORES, make_read, random_seq
from rifraf_amd import RifrafSequence
from rifraf_amd.engine import RF_BWD, RF_FWD

pytestmark = pytest.mark.gpu


def _indel_read(t, rng, k, bw=9):
    s = list(t)
    for _ in range(abs(k)):
        j = int(rng.integers(0, len(s) + (1 if k > 0 else 0)))
        if k > 0:
            s.insert(j, int(rng.integers(0, 4)))
        else:
            del s[j]
    s = np.array(s, np.uint8)
    sub = rng.random(len(s)) < 0.01
    s[sub] = (s[sub] + rng.integers(1, 4, int(sub.sum()))) % 4
    ph = rng.integers(8, 40, len(s)).astype(np.float64)
    return RifrafSequence(s, ph / -10.0, bw, SEQ_SCORES)


def _clusters(rng):
    """(template, reads) with every fused-eligible band height."""
    out = []
    for k in list(range(14)) + [17, 30, 44, 60]:          # H = 19 .. 32, 35, 48, 62, 78 at bw 9
        t = random_seq(300, rng)
        out.append((t, [_indel_read(t, rng, k if r % 2 == 0 else -k) for r in range(3)]))
    t = random_seq(200, rng)                              # H 61 .. 127 at bw 30 .. 40
    out.append((t, [_indel_read(t, rng, k, bw=bw) for k, bw in ((0, 30), (5, 33), (-9, 40), (46, 40))]))
    for bw in range(1, 9):                                # narrow bands
        t = random_seq(int(rng.integers(40, 120)), rng)
        out.append((t, [make_read(t, rng, 0.03, bw) for _ in range(int(rng.integers(1, 5)))]))
    for _ in range(6):                                    # tiny reads / templates (c > m, n < bw)
        t = random_seq(int(rng.integers(1, 12)), rng)
        rs = []
        for _ in range(int(rng.integers(1, 4))):
            n = int(rng.integers(1, 12))
            s = random_seq(n, rng)
            rs.append(RifrafSequence(s, rng.integers(5, 40, n) / -10.0, int(rng.integers(1, 6)), SEQ_SCORES))
        out.append((t, rs))
    return out


def _setup(engine, clusters):
    flat = [r for _, rs in clusters for r in rs]
    assert max(2 * r.bandwidth + abs(len(r) - len(t)) + 1 for t, rs in clusters for r in rs) <= 127
    engine.set_sequences(0, flat)
    engine.set_templates(0, [t for t, _ in clusters])
    tpl = np.concatenate([[c] * len(rs) for c, (_, rs) in enumerate(clusters)]).astype(np.int32)
    groups, at = [], 0
    for _, rs in clusters:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    return flat, tpl, groups


def test_fused_forward_equals_product_and_oracle(engine, opts):
    rng = np.random.default_rng(5150)
    clusters = _clusters(rng)
    flat, tpl, groups = _setup(engine, clusters)
    n = len(flat)
    bws = [r.bandwidth for r in flat]
    engine.realign(np.arange(n), np.arange(n), tpl, bws, RF_FWD | RF_BWD)
    ref = engine.score_dense(groups)
    opts("score_fwd", 1)
    got = engine.score_dense(groups)
    for c, (t, rs) in enumerate(clusters):
        np.testing.assert_array_equal(got[c], ref[c], err_msg=f"cluster {c}: m {len(t)}")
    for c in (0, 6, 12, 13, 15, 17, 18, 19, len(clusters) - 1):
        t, rs = clusters[c]
        exp, _ = oracle.cpu_pass(t, rs, nthreads=4)
        mask = np.ones_like(exp, bool)
        mask[0, :5] = False
        for j in range(1, len(t) + 1):
            mask[j, t[j - 1]] = False
        np.testing.assert_array_equal(got[c][mask], exp[mask], err_msg=f"cluster {c} vs oracle")


def test_fused_forward_needs_only_b(engine, opts):
    """After release_bands + an RF_BWD-only realign, the fused path scores
    from B alone; the product path refuses (A not computed)."""
    rng = np.random.default_rng(77)
    clusters = _clusters(rng)[:8]
    flat, tpl, groups = _setup(engine, clusters)
    n = len(flat)
    bws = [r.bandwidth for r in flat]
    engine.realign(np.arange(n), np.arange(n), tpl, bws, RF_FWD | RF_BWD)
    ref = engine.score_dense(groups)
    engine.release_bands()
    engine.realign(np.arange(n), np.arange(n), tpl, bws, RF_BWD)
    opts("score_fwd", 1)
    got = engine.score_dense(groups)
    for c in range(len(clusters)):
        np.testing.assert_array_equal(got[c], ref[c])
    opts("score_fwd", 0)
    with pytest.raises(Exception):
        engine.score_dense(groups)


def test_fused_forward_c4_clusters(engine, opts):
    """c4-shaped clusters (the bench's generator: 50 reads x 1.5 kb at bw 9)
    score identically with and without RF_OPT_SCORE_FWD."""
    import bench
    clusters = bench.make_workload(6, 50, 1500, 0.01, 9, seed=3)
    reads = [r for _, rs in clusters for r in rs]
    engine.set_sequences(0, reads)
    engine.set_templates(0, [t for t, _ in clusters])
    tpl = np.concatenate([[c] * len(rs) for c, (_, rs) in enumerate(clusters)]).astype(np.int32)
    n = len(reads)
    engine.realign(np.arange(n), np.arange(n), tpl, [r.bandwidth for r in reads], RF_FWD | RF_BWD)
    groups, at = [], 0
    for _, rs in clusters:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    ref = engine.score_dense(groups)
    opts("score_fwd", 1)
    got = engine.score_dense(groups)
    for c in range(len(clusters)):
        np.testing.assert_array_equal(got[c], ref[c])
