"""HIP engine parity against the CPU oracle (bit-exact).

Every test calls the engine through the C-ABI (librifraf_hip.so via ctypes)
and the oracle (oracle/rifraf_oracle.c) on the same seeded inputs.  The
oracle is pinned to the reference by tests/test_oracle_kats.py.
Tolerance: bit-exact for bands, moves, error counts and scores (the engine
evaluates the same FP64 sums in the same order as the reference).
"""
import math
import os

import numpy as np
import pytest

import oracle
from _util import (REF_SCORES, SEQ_SCORES, all_proposals_arrays, dense_slot, inband_mask, make_read,
                   random_seq)
from rifraf_amd import ErrorModel, RifrafSequence, Scores
from rifraf_amd.engine import RF_BAND_A, RF_BAND_B, RF_BWD, RF_FWD, RF_SKEW, RF_TRIM, RifrafError

pytestmark = pytest.mark.gpu


def assert_band_equal(got, exp_data, nrows, ncols, bw):
    mask = inband_mask(nrows, ncols, bw)
    g = got.data[mask]
    e = np.asarray(exp_data)[mask]
    bad = ~((g == e) | (np.isnan(g) & np.isnan(e)))
    assert not bad.any(), f"{bad.sum()} of {mask.sum()} in-band cells differ"


DP_CASES = [
    # (template length, error rate, bandwidth, length jitter, codon)
    (5, 0.05, 1, 0, False),
    (30, 0.05, 3, 0, False),
    (60, 0.05, 9, 4, False),
    (120, 0.03, 9, 12, False),      # H up to 32 -> W=16 class
    (200, 0.03, 20, 10, False),     # W=32 class
    (300, 0.05, 40, 30, False),     # H in (64, 128]: register kernel, 4 pairs per lane
    (500, 0.05, 80, 20, False),     # H > 128: LDS-ring kernel (W = 64)
    (90, 0.05, 9, 0, True),         # codon moves (reference-style tables)
    (150, 0.10, 15, 6, True),
    (200, 0.10, 30, 8, True),       # codon moves with 2 pairs per lane
    (260, 0.10, 45, 10, True),      # codon moves with 4 pairs per lane
    (400, 0.10, 70, 10, True),      # codon moves on the LDS-ring kernel
]


@pytest.mark.parametrize("lat", [0, 2048])
@pytest.mark.parametrize("pad", [64, 1])
@pytest.mark.parametrize("L,err,bw,jit,codon,nl64", [c + (1024,) for c in DP_CASES] +
                         [c + (0,) for c in DP_CASES if c[4]])
def test_dp_bands_bitexact(engine, opts, L, err, bw, jit, codon, nl64, pad, lat):
    """Bands, scores, backtraces and error counts vs the oracle, with the
    default row strides and with every band's rows padded to whole 128-B
    lines (RF_OPT_BAND_PAD = 1: even strides in every DP class).  The codon
    cases run twice: a few non-lean tasks of H <= 127 in k_dpx (the default,
    RF_OPT_DP_NL64) and in the 16-lane non-lean kernels (0).  Lean tasks run
    in their throughput classes (lat 0) and in the latency-mode 64-lane class
    (RF_OPT_DP_LAT, round 5)."""
    opts("band_pad", pad)
    opts("dp_nl64", nl64)
    opts("dp_lat", lat)
    rng = np.random.default_rng(L * 7 + bw)
    t = random_seq(L, rng)
    seqs = []
    for k in range(6):
        if codon:
            s = random_seq(max(3, L + int(rng.integers(-jit, jit + 1))), rng)
            lp = np.log10(rng.uniform(0.01, 0.2, len(s)))
            seqs.append(RifrafSequence(s, lp, bw, REF_SCORES))
        else:
            r = make_read(t, rng, err, bw)
            if jit:
                extra = random_seq(int(rng.integers(0, jit + 1)), rng)
                s = np.concatenate([r.seq, extra])
                lp = np.concatenate([r.error_log_p, np.full(len(extra), -1.0)])
                r = RifrafSequence(s, lp, bw, SEQ_SCORES)
            seqs.append(r)
    n = len(seqs)
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    scores = engine.realign(np.arange(n), np.arange(n), 0, [bw] * n, RF_FWD | RF_BWD)
    for k, s in enumerate(seqs):
        A_exp, mv = oracle.forward(t, s, moves=True)
        B_exp = oracle.backward(t, s)
        A = engine.download_band(k, RF_BAND_A)
        B = engine.download_band(k, RF_BAND_B)
        assert_band_equal(A, A_exp, len(s) + 1, L + 1, bw)
        assert_band_equal(B, B_exp, len(s) + 1, L + 1, bw)
        H = A_exp.shape[0]
        d_end = len(s) - L + max(L - len(s), 0) + bw
        assert scores[k] == A_exp[d_end, L]
        # backtrace recomputed from A == reference backtrace of the trace band
        ref_moves = oracle.backtrace(mv, len(s) + 1, L + 1, bw)
        got_moves, nerr = engine.backtrace([k])
        np.testing.assert_array_equal(got_moves[0], ref_moves)
        assert nerr[0] == oracle.count_errors(ref_moves, t, s.seq)


def _check_bands(engine, t, seqs, bws):
    n = len(seqs)
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    scores = engine.realign(np.arange(n), np.arange(n), 0, bws, RF_FWD | RF_BWD)
    L = len(t)
    for k, s in enumerate(seqs):
        A_exp, _ = oracle.forward(t, s, bandwidth=bws[k])
        B_exp = oracle.backward(t, s, bandwidth=bws[k])
        assert_band_equal(engine.download_band(k, RF_BAND_A), A_exp, len(s) + 1, L + 1, bws[k])
        assert_band_equal(engine.download_band(k, RF_BAND_B), B_exp, len(s) + 1, L + 1, bws[k])
        d_end = len(s) - L + max(L - len(s), 0) + bws[k]
        assert scores[k] == A_exp[d_end, L]


@pytest.mark.parametrize("lat", [0, 2048])
@pytest.mark.parametrize("pad", [64, 0, 1])
def test_dp_class_boundaries(engine, opts, pad, lat):
    """H = 2bw + |n-m| + 1 on both sides of every kernel-class edge (31/32,
    63/64, 127/128), reads longer and shorter than the template, mixed in one
    launch so waves hold tasks of different geometry (lean interior bounds are
    the intersection over a wave's four tasks); default, odd-only and
    all-padded row strides; throughput classes and latency mode (lat)."""
    opts("band_pad", pad)
    opts("dp_lat", lat)
    rng = np.random.default_rng(77)
    t = random_seq(180, rng)
    seqs, bws = [], []
    for H in (29, 30, 31, 32, 33, 61, 62, 63, 64, 65, 125, 126, 127, 128, 129, 254, 255, 256, 257):
        for delta in (0, 1, 4, -3):
            bw = (H - 1 - abs(delta)) // 2
            if bw < 1:
                continue
            r = make_read(t, rng, 0.04, bw)
            s = r.seq
            want = len(t) + delta
            if len(s) > want:
                s = s[:want]
                lp = r.error_log_p[:want]
            else:
                extra = random_seq(want - len(s), rng)
                s = np.concatenate([s, extra])
                lp = np.concatenate([r.error_log_p, np.full(len(extra), -1.2)])
            seqs.append(RifrafSequence(s, lp, bw, SEQ_SCORES))
            bws.append(bw)
    _check_bands(engine, t, seqs, bws)


@pytest.mark.parametrize("dp_wide,lat", [(3, 0), (1, 0), (2, 0), (0, 0), (3, 2048)])
def test_dp_wide_task_classes_long_reads(engine, opts, dp_wide, lat):
    """Regression for the round-2 64/32-lane DP task work (RF_OPT_DP_WIDE):
    one rf_realign whose lean tasks straddle every task-width class edge
    (H 62..66 -> 16 / 32 lanes, 125..131 -> 32 / 64 lanes, 250..257 -> 64
    lanes / k_dp<64>) at lengths where the blocked lean interior runs many
    blocks (m = 2400), odd task counts per class (partial waves: padding tasks
    write the sink), reads longer and shorter than the template, both
    directions, padded and unpadded strides in the same context.  Bands and
    A[end,end] bit-exact vs oracle.forward / oracle.backward."""
    opts("dp_wide", dp_wide)
    opts("dp_lat", lat)   # latency mode: H <= 127 in the 64-lane NP = 1 class, wider ones as before
    rng = np.random.default_rng(4242 + dp_wide)
    t = random_seq(2400, rng)
    seqs, bws = [], []
    for H, delta in ((62, 1), (63, 0), (64, -2), (65, 3), (66, 0), (125, 0), (127, 2), (128, -1),
                     (129, 0), (131, 4), (250, 1), (254, 0), (255, 2), (256, -5), (257, 0),
                     (29, 0), (31, 1), (129, -2), (191, 0)):
        bw = (H - 1 - abs(delta)) // 2
        r = make_read(t, rng, 0.02, bw)
        s, lp = r.seq, r.error_log_p
        want = len(t) + delta
        if len(s) > want:
            s, lp = s[:want], lp[:want]
        else:
            extra = random_seq(want - len(s), rng)
            s = np.concatenate([s, extra])
            lp = np.concatenate([lp, np.full(len(extra), -1.2)])
        seqs.append(RifrafSequence(s, lp, bw, SEQ_SCORES))
        bws.append(bw)
    _check_bands(engine, t, seqs, bws)
    # the same jobs split over two calls (forward alone, then backward alone)
    n = len(seqs)
    engine.realign(np.arange(n), np.arange(n), 0, bws, RF_FWD)
    engine.realign(np.arange(n), np.arange(n), 0, bws, RF_BWD)
    for k in (0, 7, 12, n - 1):
        A_exp, _ = oracle.forward(t, seqs[k], bandwidth=bws[k])
        assert_band_equal(engine.download_band(k, RF_BAND_A), A_exp, len(seqs[k]) + 1, len(t) + 1, bws[k])


@pytest.mark.parametrize("pfit", [1, 0])
@pytest.mark.parametrize("pad", [64, 1])
def test_dp_lean_class_stride_fit(engine, opts, pfit, pad):
    """RF_OPT_DP_PFIT (round 6): a lean NP = 2 / 4 / 8 class launched whole
    takes the smallest stride class holding its widest task (fewer flush
    stores per lane) instead of the class maximum.  Calls whose tasks sit in
    the narrowest stride class, the widest, and a mix, for every NP, with the
    throughput classes (no latency mode, no 32/64-lane wide tasks); bands
    and A[end,end] bit-exact, odd and line-padded strides."""
    opts("dp_lat", 0)
    opts("dp_wide", 0)
    opts("dp_pfit", pfit)
    opts("band_pad", pad)
    rng = np.random.default_rng(606 + pfit)
    t = random_seq(700, rng)
    for Hs in ((33, 35, 37), (61, 63), (33, 50, 63), (65, 68, 71), (120, 127), (129, 135, 140), (250, 255)):
        seqs, bws = [], []
        for k, H in enumerate(Hs * 3):
            delta = (k % 3) - 1
            bw = (H - 1 - abs(delta)) // 2
            r = make_read(t, rng, 0.03, bw)
            s, lp = r.seq, r.error_log_p
            want = len(t) + delta
            if len(s) > want:
                s, lp = s[:want], lp[:want]
            else:
                extra = random_seq(want - len(s), rng)
                s = np.concatenate([s, extra])
                lp = np.concatenate([lp, np.full(len(extra), -1.2)])
            seqs.append(RifrafSequence(s, lp, bw, SEQ_SCORES))
            bws.append(bw)
        _check_bands(engine, t, seqs, bws)


@pytest.mark.parametrize("lat", [0, 2048])
@pytest.mark.parametrize("m,n,bw", [(3, 40, 9), (8, 8, 9), (1, 1, 1), (2, 30, 2), (40, 3, 9), (25, 60, 6)])
def test_dp_short_and_skewed_shapes(engine, opts, m, n, bw, lat):
    """Templates shorter than the bandwidth (c > m: no lean interior) and very
    unequal lengths, several copies per launch; both lean DP modes."""
    opts("dp_lat", lat)
    rng = np.random.default_rng(m * 100 + n)
    t = random_seq(m, rng)
    seqs = [RifrafSequence(random_seq(n, rng), np.log10(rng.uniform(0.01, 0.3, n)), bw, SEQ_SCORES)
            for _ in range(7)]
    _check_bands(engine, t, seqs, [bw] * len(seqs))


@pytest.mark.parametrize("flags", [RF_SKEW, RF_TRIM, RF_SKEW | RF_TRIM])
def test_dp_skew_trim(engine, flags):
    rng = np.random.default_rng(flags)
    t = random_seq(80, rng)
    seqs = [make_read(t, rng, 0.08, 5) for _ in range(4)]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    engine.realign(np.arange(4), np.arange(4), 0, [5] * 4, RF_FWD | flags)
    for k, s in enumerate(seqs):
        A_exp, mv = oracle.forward(t, s, moves=True, skew=bool(flags & RF_SKEW), trim=bool(flags & RF_TRIM))
        assert_band_equal(engine.download_band(k, RF_BAND_A), A_exp, len(s) + 1, 81, 5)
        moves, nerr = engine.backtrace([k])
        ref = oracle.backtrace(mv, len(s) + 1, 81, 5)
        np.testing.assert_array_equal(moves[0], ref)


@pytest.mark.parametrize("flags", [0, RF_SKEW, RF_TRIM, RF_SKEW | RF_TRIM])
@pytest.mark.parametrize("m,dn,bw", [(2600, 21, 9), (2000, -3, 9), (700, 40, 30), (1200, 5, 4), (400, 90, 18)])
def test_dpx_long_reference_tasks(engine, opts, m, dn, bw, flags):
    """Round 5: the latency-bound non-lean kernel (k_dpx) on reference-shaped
    tasks -- one or two long codon alignments per call, as rf_rifraf_batch_ref
    and has_single_indels / single_indel_proposals issue them (configs[2]:
    2,622 x 2,601 at bw 9, H ~ 40) -- with skew_matches and trim, H from 9 to
    127 (k_dpx takes every H <= 127), many 64-row staging blocks (ring
    wrap-around), forward alone (flags) and forward + backward.  Bands,
    A[end,end], backtraces and error counts bit-exact vs the oracle."""
    rng = np.random.default_rng(m + dn + 1000 * bw + flags)
    t = random_seq(m, rng)
    # a mutated copy of the template, shifted in frame: codon and single indels
    s = t.copy()
    for _ in range(max(3, m // 200)):
        p = int(rng.integers(0, len(s)))
        op = int(rng.integers(0, 3))
        if op == 0:
            s[p] = (s[p] + 1) % 4
        elif op == 1:
            s = np.concatenate([s[:p], random_seq(int(rng.integers(1, 4)), rng), s[p:]])
        else:
            s = np.concatenate([s[:p], s[p + int(rng.integers(1, 4)):]])
    want = m + dn
    s = s[:want] if len(s) > want else np.concatenate([s, random_seq(want - len(s), rng)])
    ref = RifrafSequence(s, np.full(len(s), math.log10(0.1)), bw, REF_SCORES)
    engine.set_sequences(0, [ref])
    engine.set_templates(0, [t])
    H = 2 * bw + abs(dn) + 1
    assert H <= 127
    skew, trim = bool(flags & RF_SKEW), bool(flags & RF_TRIM)
    score = engine.realign([0], [0], 0, [bw], RF_FWD | flags)
    A_exp, mv = oracle.forward(t, ref, moves=True, skew=skew, trim=trim)
    assert_band_equal(engine.download_band(0, RF_BAND_A), A_exp, len(s) + 1, m + 1, bw)
    d_end = len(s) - m + max(m - len(s), 0) + bw
    assert score[0] == A_exp[d_end, m]
    moves, nerr = engine.backtrace([0])
    exp_moves = oracle.backtrace(mv, len(s) + 1, m + 1, bw)
    np.testing.assert_array_equal(moves[0], exp_moves)
    assert nerr[0] == oracle.count_errors(exp_moves, t, s)
    if not flags:
        engine.realign([0], [0], 0, [bw], RF_FWD | RF_BWD)
        assert_band_equal(engine.download_band(0, RF_BAND_B), oracle.backward(t, ref), len(s) + 1, m + 1, bw)
        assert_band_equal(engine.download_band(0, RF_BAND_A), A_exp, len(s) + 1, m + 1, bw)


def test_realign_jobs_per_job_flags(engine):
    """rf_realign_jobs (round 5): flags per job in one launch set -- reads'
    backward fills beside the reference's skewed forward fill and a trimmed
    one (the native driver's realign_B + single_indel_proposals) -- give the
    bands, scores and walks of separate rf_realign calls."""
    rng = np.random.default_rng(606)
    t = random_seq(900, rng)
    reads = [make_read(t, rng, 0.02, 9) for _ in range(5)]
    ref = RifrafSequence(np.concatenate([t[:400], t[401:]]), np.full(len(t) - 1, math.log10(0.1)), 9, REF_SCORES)
    engine.set_sequences(0, reads + [ref])
    engine.set_templates(0, [t])
    slots = [0, 1, 2, 3, 4, 5, 6, 7]
    seqs = [0, 1, 2, 3, 4, 5, 5, 5]
    flags = [RF_BWD] * 5 + [RF_BWD, RF_FWD | RF_SKEW, RF_FWD | RF_TRIM]
    got = engine.realign(slots, seqs, 0, [9] * 8, flags)
    bands = [engine.download_band(s, RF_BAND_B).data.copy() for s in range(6)]
    bands += [engine.download_band(s, RF_BAND_A).data.copy() for s in (6, 7)]
    mv_got = engine.backtrace([6, 7])[0]
    sep = list(engine.realign(slots[:6], seqs[:6], 0, [9] * 6, RF_BWD))
    sep += list(engine.realign([6], [5], 0, [9], RF_FWD | RF_SKEW))
    sep += list(engine.realign([7], [5], 0, [9], RF_FWD | RF_TRIM))
    np.testing.assert_array_equal(got, np.array(sep))
    for s, b in zip(range(6), bands):
        np.testing.assert_array_equal(engine.download_band(s, RF_BAND_B).data, b)
    for s, b in zip((6, 7), bands[6:]):
        np.testing.assert_array_equal(engine.download_band(s, RF_BAND_A).data, b)
    for a, b in zip(mv_got, engine.backtrace([6, 7])[0]):
        np.testing.assert_array_equal(a, b)
    A_exp, _ = oracle.forward(t, ref, skew=True)
    assert_band_equal(engine.download_band(6, RF_BAND_A), A_exp, len(ref.seq) + 1, len(t) + 1, 9)


def test_dpx_invalid_score_is_loud(engine):
    """A non-lean task whose band holds a cell with no finite predecessor
    (insertions and deletions impossible: ErrorModel(1, 0, 0, 1, 1), a read
    one base longer than the template) raises the reference's "new score is
    invalid" (align.jl:105-107) from k_dpx, as from the other DP kernels."""
    rng = np.random.default_rng(3)
    t = random_seq(300, rng)
    s = np.concatenate([t, random_seq(1, rng)])
    sc = Scores.from_errors(ErrorModel(1.0, 0.0, 0.0, 1.0, 1.0))
    r = RifrafSequence(s, np.full(len(s), -1.0), 9, sc)
    engine.set_sequences(0, [r])
    engine.set_templates(0, [t])
    with pytest.raises(RifrafError, match="new score is invalid"):
        engine.realign([0], [0], 0, [9], RF_FWD)
    with pytest.raises(oracle.OracleError):
        oracle.forward(t, r)


@pytest.mark.parametrize("mc", [1, 0])
@pytest.mark.parametrize("m,dn,flags", [(2601, 21, RF_SKEW), (3000, -40, 0), (3400, 180, RF_SKEW | RF_TRIM),
                                         (2300, 0, RF_TRIM)])
def test_dpm_edit_distance_bands(engine, opts, m, dn, flags, mc):
    """Very wide bands without codon moves (edit_distance, align.jl:253-260:
    bw = ceil(min(m, n) / 2), skew_matches): configs[2]'s shape (2,622 x
    2,601) and wider, skew and trim, forward and (no flags) backward; bands,
    A[end,end], backtraces and error counts bit-exact vs the oracle.  mc 1
    (the default since round 6): k_dpm's slices across CUs (RF_OPT_DP_MC);
    0: one block per band (k_dp)."""
    opts("dp_mc", mc)
    rng = np.random.default_rng(m + dn)
    t = random_seq(m, rng)
    s = make_read(t, rng, 0.1, 9).seq
    want = m + dn
    s = s[:want] if len(s) > want else np.concatenate([s, random_seq(want - len(s), rng)])
    bw = int(math.ceil(min(m, len(s)) * 0.5))
    r = RifrafSequence(s, np.full(len(s), -1.0), bw, Scores.from_errors(ErrorModel(1.0, 1.0, 1.0)))
    H = 2 * bw + abs(len(s) - m) + 1
    assert 2040 < H <= 3600
    engine.set_sequences(0, [r])
    engine.set_templates(0, [t])
    score = engine.realign([0], [0], 0, [bw], RF_FWD | flags)
    A_exp, mv = oracle.forward(t, r, moves=True, skew=bool(flags & RF_SKEW), trim=bool(flags & RF_TRIM))
    assert_band_equal(engine.download_band(0, RF_BAND_A), A_exp, len(s) + 1, m + 1, bw)
    d_end = len(s) - m + max(m - len(s), 0) + bw
    assert score[0] == A_exp[d_end, m]
    moves, nerr = engine.backtrace([0])
    exp_moves = oracle.backtrace(mv, len(s) + 1, m + 1, bw)
    np.testing.assert_array_equal(moves[0], exp_moves)
    assert nerr[0] == oracle.count_errors(exp_moves, t, s)
    if not flags:
        engine.realign([0], [0], 0, [bw], RF_BWD)
        assert_band_equal(engine.download_band(0, RF_BAND_B), oracle.backward(t, r), len(s) + 1, m + 1, bw)


@pytest.mark.parametrize("mc", [1, 0])
def test_dp_huge_band_global_ring(engine, opts, mc):
    """H > 2040 (edit_distance-sized bands): k_dpm's slices across CUs (mc
    1), or one task per block (mc 0)."""
    opts("dp_mc", mc)
    rng = np.random.default_rng(5)
    t = random_seq(2300, rng)
    s = make_read(t, rng, 0.02, 1100)
    engine.set_sequences(0, [s])
    engine.set_templates(0, [t])
    engine.realign([0], [0], 0, [1100], RF_FWD | RF_BWD)
    A_exp, _ = oracle.forward(t, s, moves=True)
    assert_band_equal(engine.download_band(0, RF_BAND_A), A_exp, len(s) + 1, 2301, 1100)
    B_exp = oracle.backward(t, s)
    assert_band_equal(engine.download_band(0, RF_BAND_B), B_exp, len(s) + 1, 2301, 1100)


@pytest.mark.parametrize("mc", [1, 0])
def test_dp_band_beyond_lds_ring(engine, opts, mc):
    """H > DPW_LDS_H (5114): k_dpm (mc 1, 81 slices) or the block-wide DP
    with its ring in global memory (k_dp<256, true, 256>, mc 0); forward and
    backward bands bit-exact."""
    opts("dp_mc", mc)
    rng = np.random.default_rng(6)
    t = random_seq(5300, rng)
    s = make_read(t, rng, 0.02, 2600)
    engine.set_sequences(0, [s])
    engine.set_templates(0, [t])
    engine.realign([0], [0], 0, [2600], RF_FWD | RF_BWD)
    H = 2 * 2600 + abs(len(s) - len(t)) + 1
    assert H > 5114
    A_exp, _ = oracle.forward(t, s, moves=True)
    assert_band_equal(engine.download_band(0, RF_BAND_A), A_exp, len(s) + 1, len(t) + 1, 2600)
    B_exp = oracle.backward(t, s)
    assert_band_equal(engine.download_band(0, RF_BAND_B), B_exp, len(s) + 1, len(t) + 1, 2600)


def test_dpm_several_wide_bands_one_call(engine):
    """Several very wide bands in one rf_realign (k_dpm: every band's slices
    in one launch, bands of different slice counts, H just above the 2,040
    edge and far above), forward and backward, and a narrow read beside
    them; bands and A[end,end] bit-exact."""
    rng = np.random.default_rng(66)
    t = random_seq(2200, rng)
    seqs, bws = [], []
    for bw, dn in ((1025, 2), (1100, -30), (1300, 0), (1021, 1)):
        s = make_read(t, rng, 0.05, bw).seq
        want = len(t) + dn
        s = s[:want] if len(s) > want else np.concatenate([s, random_seq(want - len(s), rng)])
        seqs.append(RifrafSequence(s, np.full(len(s), -1.3), bw, SEQ_SCORES))
        bws.append(bw)
    seqs.append(make_read(t, rng, 0.02, 9))
    bws.append(9)
    assert all(2 * b + abs(len(s) - len(t)) + 1 > 2040 for s, b in zip(seqs[:4], bws[:4]))
    _check_bands(engine, t, seqs, bws)


def test_dpm_bands_sharing_an_xcd(engine):
    """Seventeen very wide bands of 32 slices in one call: k_dpm puts band t
    on XCD t % 8 and takes 64 slices per XCD per launch, so bands 8-15 queue
    behind bands 0-7 on their XCDs inside the first launch (workgroups
    dispatch in order; a band's slices wait only for earlier, whole bands)
    and band 16 runs in a second launch; forward and backward bit-exact."""
    rng = np.random.default_rng(67)
    t = random_seq(2100, rng)
    seqs, bws = [], []
    for i in range(17):
        bw = 1021
        s = make_read(t, rng, 0.04, bw).seq
        want = len(t) + (i % 5) - 2
        s = s[:want] if len(s) > want else np.concatenate([s, random_seq(want - len(s), rng)])
        seqs.append(RifrafSequence(s, np.full(len(s), -1.1), bw, SEQ_SCORES))
        bws.append(bw)
    Hs = [2 * b + abs(len(s) - len(t)) + 1 for s, b in zip(seqs, bws)]
    assert all(2040 < H <= 2047 for H in Hs)   # 32 slices each
    _check_bands(engine, t, seqs, bws)


@pytest.mark.parametrize("mode", ["fused", "split"])
@pytest.mark.parametrize("L,nreads,bw", [(40, 3, 9), (150, 7, 9), (260, 5, 25)])
def test_score_all_proposals_bitexact(engine, opts, mode, L, nreads, bw):
    opts("score_mode", mode)
    rng = np.random.default_rng(L + nreads)
    t = random_seq(L, rng)
    seqs = [make_read(t, rng, 0.03, bw) for _ in range(nreads)]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    engine.realign(np.arange(nreads), np.arange(nreads), 0, [bw] * nreads, RF_FWD | RF_BWD)
    props = all_proposals_arrays(t)
    got = engine.score([(np.arange(nreads), -1, props)])[0]
    ref_tot, _ = oracle.cpu_pass(t, seqs, nthreads=4)
    exp = ref_tot[props[1], dense_slot(props[0], props[2])]
    np.testing.assert_array_equal(got, exp)


def test_score_per_read_bitexact(engine):
    rng = np.random.default_rng(3)
    t = random_seq(70, rng)
    seqs = [make_read(t, rng, 0.04, 9) for _ in range(4)]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    engine.realign(np.arange(4), np.arange(4), 0, [9] * 4, RF_FWD | RF_BWD)
    props = all_proposals_arrays(t)
    tot, per = engine.score([(np.arange(4), -1, props)], per_seq=True)
    As = [oracle.forward(t, s)[0] for s in seqs]
    Bs = [oracle.backward(t, s) for s in seqs]
    for k in range(0, len(props[0]), 7):
        for r, s in enumerate(seqs):
            exp = oracle.score_proposal(props[0][k], props[1][k], props[2][k], As[r], Bs[r], t, s)
            assert per[0][k, r] == exp
        fold = 0.0
        for r in range(4):
            fold += per[0][k, r]
        assert tot[0][k] == fold


def test_score_many_clusters(engine, opts):
    """Batched clusters: one group per consensus, fused ordered fold."""
    opts("score_mode", "fused")
    rng = np.random.default_rng(99)
    templates, seqs, groups = [], [], []
    for c in range(6):
        t = random_seq(int(rng.integers(50, 90)), rng)
        templates.append(t)
        rs = [make_read(t, rng, 0.03, 9) for _ in range(int(rng.integers(2, 5)))]
        seqs.append(rs)
    flat = [r for rs in seqs for r in rs]
    engine.set_sequences(0, flat)
    engine.set_templates(0, templates)
    ids, tpl, at = [], [], 0
    for c, rs in enumerate(seqs):
        ids.append(np.arange(at, at + len(rs)))
        tpl += [c] * len(rs)
        at += len(rs)
    engine.realign(np.arange(at), np.arange(at), np.array(tpl), [9] * at, RF_FWD | RF_BWD)
    groups = [(ids[c], -1, all_proposals_arrays(templates[c])) for c in range(6)]
    got = engine.score(groups)
    for c in range(6):
        ref_tot, _ = oracle.cpu_pass(templates[c], seqs[c], nthreads=4)
        k, p, b = groups[c][2]
        np.testing.assert_array_equal(got[c], ref_tot[p, dense_slot(k, b)])


def test_score_reference_codon(engine):
    """Reference (codon-move) scoring, model.jl:302-383, alone and after reads."""
    rng = np.random.default_rng(21)
    t = random_seq(99, rng)
    ref_s = random_seq(96, rng)
    ref = RifrafSequence(ref_s, np.full(96, math.log10(0.05)), 9, REF_SCORES)
    reads = [make_read(t, rng, 0.03, 9) for _ in range(3)]
    engine.set_sequences(0, reads + [ref])
    engine.set_templates(0, [t])
    engine.realign(np.arange(4), np.arange(4), 0, [9] * 4, RF_FWD | RF_BWD)
    props = all_proposals_arrays(t)
    tot_ref_only, per = engine.score([(np.arange(0), 3, props)], per_seq=True)
    tot_all = engine.score([(np.arange(3), 3, props)])[0]
    Ar, _ = oracle.forward(t, ref)
    Br = oracle.backward(t, ref)
    As = [oracle.forward(t, s)[0] for s in reads]
    Bs = [oracle.backward(t, s) for s in reads]
    for k in range(len(props[0])):
        prop = (int(props[0][k]), int(props[1][k]), int(props[2][k]))
        exp_ref = oracle.score_proposal(*prop, Ar, Br, t, ref)
        assert tot_ref_only[0][k] == 0.0 + exp_ref
        assert per[0][k, 0] == exp_ref
        exp = oracle.score_total(prop, As, Bs, reads, t, Ar, Br, ref)
        assert tot_all[k] == exp, prop


def test_single_sequence_nocodon_group(engine):
    """A group with only a non-codon 'reference' slot runs the per-proposal
    score_nocodon path (model.jl:242-285)."""
    rng = np.random.default_rng(8)
    t = random_seq(45, rng)
    r = make_read(t, rng, 0.05, 9)
    engine.set_sequences(0, [r])
    engine.set_templates(0, [t])
    engine.realign([0], [0], 0, [9], RF_FWD | RF_BWD)
    props = all_proposals_arrays(t)
    got = engine.score([([], 0, props)])[0]
    A, _ = oracle.forward(t, r)
    B = oracle.backward(t, r)
    for k in range(len(props[0])):
        assert got[k] == oracle.score_proposal(props[0][k], props[1][k], props[2][k], A, B, t, r)


def test_errors_are_loud(engine):
    rng = np.random.default_rng(2)
    t = random_seq(20, rng)
    r = make_read(t, rng, 0.05, 3)
    engine.set_sequences(0, [r])
    engine.set_templates(0, [t])
    with pytest.raises(RifrafError, match="bandwidth must be positive"):
        engine.realign([0], [0], 0, [0], RF_FWD)
    engine.realign([0], [0], 0, [3], RF_FWD)
    with pytest.raises(RifrafError):
        engine.score([([0], -1, all_proposals_arrays(t))])  # no B band yet
    codon = RifrafSequence(r.seq, r.error_log_p, 3, REF_SCORES)
    engine.set_sequences(1, [codon])
    engine.realign([1], [1], 0, [3], RF_FWD | RF_BWD)
    with pytest.raises(RifrafError, match="codon"):
        engine.score([([1], -1, all_proposals_arrays(t))])


@pytest.mark.parametrize("mode", ["fused", "split"])
def test_score_dense_clusters(engine, opts, mode):
    """rf_score_dense over several clusters == oracle all-proposals pass."""
    opts("score_mode", mode)
    rng = np.random.default_rng(123)
    templates, seqs = [], []
    for c in range(5):
        t = random_seq(int(rng.integers(60, 140)), rng)
        templates.append(t)
        seqs.append([make_read(t, rng, 0.03, 9) for _ in range(int(rng.integers(1, 6)))])
    flat = [r for rs in seqs for r in rs]
    engine.set_sequences(0, flat)
    engine.set_templates(0, templates)
    tpl = np.concatenate([[c] * len(rs) for c, rs in enumerate(seqs)])
    n = len(flat)
    engine.realign(np.arange(n), np.arange(n), tpl, [9] * n, RF_FWD | RF_BWD)
    groups, at = [], 0
    for rs in seqs:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    got = engine.score_dense(groups)
    for c in range(5):
        ref_tot, _ = oracle.cpu_pass(templates[c], seqs[c], nthreads=4)
        t = templates[c]
        mask = np.ones_like(ref_tot, bool)
        mask[0, :5] = False                       # p = 0 has no sub/del
        for j in range(1, len(t) + 1):
            mask[j, t[j - 1]] = False             # not a proposal
        np.testing.assert_array_equal(got[c][mask], ref_tot[mask])


def _indel_read(t, rng, k, bw=9):
    """t with k bases inserted (k > 0) or -k bases deleted (k < 0) at random
    positions, plus ~1 % substitutions: |n - m| = |k|, so H = |k| + 2 bw + 1."""
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


@pytest.mark.parametrize("mode", ["fused", "split"])
def test_score_dense_fixed_stride_chains(engine, opts, mode):
    """k_score_ws's fixed-stride chains (lean_chain_fix<P>, P = 11, 13, 15,
    17) against the oracle: one cluster per |n - m| = 0..13 (H = 19..32, both
    parities, every c4 stride), reads longer and shorter than the template,
    m = 700 so that most waves are interior and the first / last are not."""
    opts("score_mode", mode)
    rng = np.random.default_rng(2417)
    templates, seqs = [], []
    for k in range(14):
        t = random_seq(700, rng)
        templates.append(t)
        seqs.append([_indel_read(t, rng, k if r % 2 == 0 else -k) for r in range(3)])
    flat = [r for rs in seqs for r in rs]
    assert {r.bandwidth for r in flat} == {9}
    engine.set_sequences(0, flat)
    engine.set_templates(0, templates)
    tpl = np.concatenate([[c] * len(rs) for c, rs in enumerate(seqs)])
    n = len(flat)
    engine.realign(np.arange(n), np.arange(n), tpl, [9] * n, RF_FWD | RF_BWD)
    groups, at = [], 0
    for rs in seqs:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    got = engine.score_dense(groups)
    for c in range(len(templates)):
        ref_tot, _ = oracle.cpu_pass(templates[c], seqs[c], nthreads=4)
        t = templates[c]
        mask = np.ones_like(ref_tot, bool)
        mask[0, :5] = False
        for j in range(1, len(t) + 1):
            mask[j, t[j - 1]] = False
        np.testing.assert_array_equal(got[c][mask], ref_tot[mask], err_msg=f"|n - m| = {c}")


def test_plan_cache_follows_template_content(engine):
    """A repeated realign/score with identical arguments reuses the uploaded
    plan; a same-length consensus change must still be picked up."""
    rng = np.random.default_rng(77)
    t1 = random_seq(90, rng)
    t2 = t1.copy()
    t2[40:45] = (t2[40:45] + 1) % 4
    seqs = [make_read(t1, rng, 0.03, 9) for _ in range(4)]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t1])
    sl = np.arange(4)
    s1 = engine.realign(sl, sl, 0, [9] * 4, RF_FWD | RF_BWD)
    d1 = engine.score_dense([sl])[0]
    engine.set_templates(0, [t2])
    s2 = engine.realign(sl, sl, 0, [9] * 4, RF_FWD | RF_BWD)
    d2 = engine.score_dense([sl])[0]
    ref2, _ = oracle.cpu_pass(t2, seqs, nthreads=2)
    for k, s in enumerate(seqs):
        A_exp, _ = oracle.forward(t2, s)
        assert_band_equal(engine.download_band(k, RF_BAND_A), A_exp, len(s) + 1, 91, 9)
    assert not np.array_equal(s1, s2)
    np.testing.assert_array_equal(d2[1:, 5:], ref2[1:, 5:])
    engine.set_templates(0, [t1])
    s3 = engine.realign(sl, sl, 0, [9] * 4, RF_FWD | RF_BWD)
    np.testing.assert_array_equal(s3, s1)
    np.testing.assert_array_equal(engine.score_dense([sl])[0][1:, 5:], d1[1:, 5:])


SCORER_CONFIGS = [
    # (score_kernel, lean_lds_kb) engine options
    ("general", None),
    ("seg", None),       # row-segment scorer (wide bands) on every shape: k_score_segl (64 columns)
    ("seglodd", None),   # k_score_segl over odd-stride rows only (band_pad 0: 9-chunk loader)
    ("seglpad", None),   # k_score_segl with every band line-padded (band_pad 1)
    (None, None),        # auto: k_score_ws, or k_score_segl when most cells need sub-windows
    ("ws", None),        # k_score_ws whenever it fits
    ("ws", "8"),         # windows exceed the budget: sub-passes over fewer lanes
    ("ws", "12"),
    ("ws", "24"),
    ("ws", "40"),
    ("ws", "60"),
    (None, "24"),        # auto under a small budget: k_score_segl
]


@pytest.mark.parametrize("wgs", [2048, 1])
def test_score_ws_split_read_chunks(engine, opts, wgs):
    """Round 5: split-mode k_score_ws takes several reads per workgroup
    (RF_OPT_SCORE_WGS 1: every read of a group in one workgroup per item,
    sub-window units included), writing each read's partial, so k_reduce's
    ordered fold equals the one-read-per-workgroup launch and the oracle."""
    import oracle
    opts("score_mode", "split")
    opts("score_kernel", "ws")
    opts("score_wgs", wgs)
    rng = np.random.default_rng(77)
    tpls = [random_seq(L, rng) for L in (700, 300)]
    groups, seqs, tpl_of, bws = [], [], [], []
    for c, t in enumerate(tpls):
        rs = [make_read(t, rng, 0.03, 9 if k % 3 else 20) for k in range(9 + 4 * c)]
        groups.append(np.arange(len(seqs), len(seqs) + len(rs)))
        seqs += rs
        tpl_of += [c] * len(rs)
        bws += [r.bandwidth for r in rs]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, tpls)
    n = len(seqs)
    engine.realign(np.arange(n), np.arange(n), np.array(tpl_of), bws, RF_FWD | RF_BWD)
    dense = engine.score_dense(groups)
    for c, t in enumerate(tpls):
        exp, _ = oracle.cpu_pass(t, [seqs[i] for i in groups[c]], nthreads=2)
        mask = np.ones_like(exp, bool)
        mask[0, :5] = False                       # p = 0 has no sub/del
        for j in range(1, len(t) + 1):
            mask[j, t[j - 1]] = False             # not a proposal
        np.testing.assert_array_equal(dense[c][mask], exp[mask])


@pytest.mark.parametrize("kern,lds", SCORER_CONFIGS)
@pytest.mark.parametrize("mode", ["fused", "split"])
def test_score_dense_kernels(engine, opts, kern, lds, mode):
    """The dense scorers (general, k_score_ws, k_score_segl) over ragged
    clusters: n << m, n >> m, wide bands, 1-read groups; bit-exact vs the
    oracle."""
    pad = 64
    if kern in ("seglodd", "seglpad"):
        pad = 0 if kern == "seglodd" else 1
        kern = "seg"
    opts("band_pad", pad)
    opts("score_kernel", kern or "auto")
    opts("lean_lds_kb", int(lds or 0))
    opts("score_mode", mode)
    rng = np.random.default_rng(77)
    templates, seqs, bws = [], [], []
    shapes = [(150, 9, 0), (40, 3, 25), (260, 20, -30), (130, 9, 0), (70, 5, 12), (1, 1, 0)]
    for c, (L, bw, skew) in enumerate(shapes):
        t = random_seq(L, rng)
        templates.append(t)
        rs = []
        for _ in range(int(rng.integers(1, 6))):
            r = make_read(t, rng, 0.04, bw)
            if skew > 0:
                extra = random_seq(int(rng.integers(0, skew + 1)), rng)
                r = RifrafSequence(np.concatenate([r.seq, extra]),
                                   np.concatenate([r.error_log_p, np.full(len(extra), -1.0)]), bw, SEQ_SCORES)
            elif skew < 0 and len(r.seq) > -skew + 5:
                cut = int(rng.integers(0, -skew + 1))
                r = RifrafSequence(r.seq[:len(r.seq) - cut], r.error_log_p[:len(r.seq) - cut], bw, SEQ_SCORES)
            rs.append(r)
        seqs.append(rs)
        bws += [bw] * len(rs)
    flat = [r for rs in seqs for r in rs]
    engine.set_sequences(0, flat)
    engine.set_templates(0, templates)
    tpl = np.concatenate([[c] * len(rs) for c, rs in enumerate(seqs)])
    n = len(flat)
    engine.realign(np.arange(n), np.arange(n), tpl, bws, RF_FWD | RF_BWD)
    groups, at = [], 0
    for rs in seqs:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    got = engine.score_dense(groups)
    for c in range(len(templates)):
        ref_tot, _ = oracle.cpu_pass(templates[c], seqs[c], nthreads=4)
        t = templates[c]
        mask = np.ones_like(ref_tot, bool)
        mask[0, :5] = False
        for j in range(1, len(t) + 1):
            mask[j, t[j - 1]] = False
        np.testing.assert_array_equal(got[c][mask], ref_tot[mask], err_msg=f"cluster {c}")
    # the proposal-list path (rf_score) through the same scorer
    props = [all_proposals_arrays(t) for t in templates]
    tots = engine.score([(groups[c], -1, props[c]) for c in range(len(templates))])
    for c in range(len(templates)):
        ref_tot, _ = oracle.cpu_pass(templates[c], seqs[c], nthreads=4)
        k, p, b = props[c]
        np.testing.assert_array_equal(tots[c], ref_tot[p, dense_slot(k, b)], err_msg=f"cluster {c}")


def test_score_lean_ineligible_tables(engine):
    """A read with an infinite table entry (phred 0 -> match = -Inf) keeps the
    launch on the general scorer; results stay bit-exact."""
    rng = np.random.default_rng(5)
    t = random_seq(90, rng)
    rs = [make_read(t, rng, 0.03, 9) for _ in range(3)]
    lp = rs[1].error_log_p.copy()
    lp[10] = 0.0
    rs[1] = RifrafSequence(rs[1].seq, lp, 9, SEQ_SCORES)
    engine.set_sequences(0, rs)
    engine.set_templates(0, [t])
    engine.realign(np.arange(3), np.arange(3), 0, [9] * 3, RF_FWD | RF_BWD)
    props = all_proposals_arrays(t)
    got = engine.score([(np.arange(3), -1, props)])[0]
    ref_tot, _ = oracle.cpu_pass(t, rs, nthreads=4)
    exp = ref_tot[props[1], dense_slot(props[0], props[2])]
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("mode", ["fused", "split"])
@pytest.mark.parametrize("kern", [None, "seglodd", "seglpad", "seglmix", "general"])
def test_score_wide_bands(engine, opts, mode, kern):
    """Bands whose kappa-row window exceeds LDS (H ~ 90-260, reads longer and
    shorter than the template, plus a narrow read in the same launch): the
    line-aligned row-segment scorer k_score_segl on line-padded rows,
    odd-stride rows and both in one launch, and the in-place k_score
    ("general"), are bit-exact against the oracle."""
    opts("band_pad", 64)
    if kern in (None, "seglmix"):
        opts("score_kernel", "auto")
    elif kern in ("seglodd", "seglpad"):
        opts("score_kernel", "auto")
        opts("band_pad", 0 if kern == "seglodd" else 1)
    else:
        opts("score_kernel", kern)
    opts("score_mode", mode)
    rng = np.random.default_rng(404)
    templates, seqs, bws = [], [], []
    for L, bw_list, skew in [(320, (100, 60, 9), 40), (250, (45, 120), -35), (90, (70,), 0)]:
        t = random_seq(L, rng)
        templates.append(t)
        rs = []
        for bw in bw_list:
            r = make_read(t, rng, 0.05, bw)
            if skew > 0:
                extra = random_seq(int(rng.integers(skew // 2, skew + 1)), rng)
                r = RifrafSequence(np.concatenate([r.seq, extra]),
                                   np.concatenate([r.error_log_p, np.full(len(extra), -1.0)]), bw, SEQ_SCORES)
            elif skew < 0:
                cut = int(rng.integers(-skew // 2, -skew + 1))
                r = RifrafSequence(r.seq[:len(r.seq) - cut], r.error_log_p[:len(r.seq) - cut], bw, SEQ_SCORES)
            rs.append(r)
            bws.append(bw)
        seqs.append(rs)
    flat = [r for rs in seqs for r in rs]
    engine.set_sequences(0, flat)
    engine.set_templates(0, templates)
    tpl = np.concatenate([[c] * len(rs) for c, rs in enumerate(seqs)])
    n = len(flat)
    if kern == "seglmix":
        # line-padded and odd-stride bands in one scoring launch: the even reads
        # realigned in a padded call, the odd ones in an unpadded one
        ev, od = np.arange(0, n, 2), np.arange(1, n, 2)
        opts("band_pad", 1)
        engine.realign(ev, ev, tpl[ev], np.asarray(bws)[ev], RF_FWD | RF_BWD)
        opts("band_pad", 0)
        engine.realign(od, od, tpl[od], np.asarray(bws)[od], RF_FWD | RF_BWD)
    else:
        engine.realign(np.arange(n), np.arange(n), tpl, bws, RF_FWD | RF_BWD)
    groups, at = [], 0
    for rs in seqs:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    got = engine.score_dense(groups)
    for c in range(len(templates)):
        ref_tot, _ = oracle.cpu_pass(templates[c], seqs[c], nthreads=4)
        t = templates[c]
        mask = np.ones_like(ref_tot, bool)
        mask[0, :5] = False
        for j in range(1, len(t) + 1):
            mask[j, t[j - 1]] = False
        np.testing.assert_array_equal(got[c][mask], ref_tot[mask], err_msg=f"cluster {c}")


@pytest.mark.parametrize("order", ["fwd_then_bwd", "bwd_then_fwd"])
def test_split_direction_calls_share_stride(engine, opts, order):
    """smart_forward_moves! + backward! as separate calls: the forward bands of
    narrow reads come from an unpadded call, the band-doubling refill of one
    read makes a line-padded call, and the backward bands of every read come
    from another padded call (its widest band has H >= RF_OPT_BAND_PAD).  A
    and B of one alignment must keep one row stride (the scorers read both
    with one P); dense and proposal-list totals equal the oracle."""
    opts("band_pad", 64)
    rng = np.random.default_rng(515)
    t = random_seq(400, rng)
    reads = [make_read(t, rng, 0.02, 9) for _ in range(6)]
    wide = make_read(t, rng, 0.05, 40)
    seqs = reads + [wide]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    n = len(seqs)
    sl = np.arange(n)
    bws = np.array([9] * (n - 1) + [40])
    if order == "fwd_then_bwd":
        engine.realign(sl, sl, 0, [9] * n, RF_FWD)                   # unpadded (H < 64)
        engine.realign(sl[-1:], sl[-1:], 0, bws[-1:], RF_FWD)       # padded refill
        engine.realign(sl, sl, 0, bws, RF_BWD)                      # padded call
    else:
        engine.realign(sl[:-1], sl[:-1], 0, bws[:-1], RF_BWD)       # unpadded
        engine.realign(sl, sl, 0, bws, RF_FWD)                      # padded call
        engine.realign(sl[-1:], sl[-1:], 0, bws[-1:], RF_BWD)
    got = engine.score_dense([sl])[0]
    ref_tot, _ = oracle.cpu_pass(t, seqs, nthreads=4)
    mask = np.ones_like(ref_tot, bool)
    mask[0, :5] = False
    for j in range(1, len(t) + 1):
        mask[j, t[j - 1]] = False
    np.testing.assert_array_equal(got[mask], ref_tot[mask])
    kinds, poss, bases = all_proposals_arrays(t)
    tot = engine.score([(sl, -1, (kinds, poss, bases))])[0]
    slot = np.where(kinds == 0, bases, np.where(kinds == 2, 4, 5 + bases))
    np.testing.assert_array_equal(tot, ref_tot[poss, slot])


@pytest.mark.parametrize("do_indels", [True, False])
def test_alignment_proposals_device(engine, do_indels):
    """rf_alignment_proposals (device moves_to_proposals + Set union) equals the
    host union of moves_to_proposals over the oracle's backtraces."""
    from rifraf_amd.align import moves_to_proposals_np
    rng = np.random.default_rng(55 + do_indels)
    templates, seqs = [], []
    for c in range(4):
        t = random_seq(int(rng.integers(60, 160)), rng)
        templates.append(t)
        seqs.append([make_read(t, rng, 0.06, 9) for _ in range(int(rng.integers(1, 7)))])
    flat = [r for rs in seqs for r in rs]
    engine.set_sequences(0, flat)
    engine.set_templates(0, templates)
    tpl = np.concatenate([[c] * len(rs) for c, rs in enumerate(seqs)])
    n = len(flat)
    engine.realign(np.arange(n), np.arange(n), tpl, [9] * n, RF_FWD | RF_BWD)
    groups, at = [], 0
    for rs in seqs:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    masks = engine.alignment_proposals(groups, do_indels)
    for c, t in enumerate(templates):
        exp = np.zeros((len(t) + 1, 9), np.uint8)
        for s in seqs[c]:
            _, mv = oracle.forward(t, s, moves=True)
            moves = oracle.backtrace(mv, len(s) + 1, len(t) + 1, 9)
            k, p, b = moves_to_proposals_np(moves, t, s.seq)
            if not do_indels:
                keep = k == 0
                k, p, b = k[keep], p[keep], b[keep]
            exp[p, np.where(k == 0, b, np.where(k == 2, 4, 5 + b))] = 1
        np.testing.assert_array_equal(masks[c], exp, err_msg=f"cluster {c}")


@pytest.mark.parametrize("nw", [4, 1])
@pytest.mark.parametrize("win_kb,pad", [(32, 64), (16, 64), (16, 1)])
@pytest.mark.parametrize("L,bw,skew", [(700, 9, 0), (400, 40, 30), (300, 120, -40), (260, 9, 60), (90, 3, 0)])
def test_backtrace_windowed(engine, opts, L, bw, skew, win_kb, pad, nw):
    """k_bt_win (LDS windows of kappa rows, re-staged as the walk leaves
    them) against the oracle's backtrace and count_errors, and the fused
    proposal marking against the host moves_to_proposals union, on long reads
    (many windows), wide bands (small windows: P up to 129) and reads longer /
    shorter than the template; a walk on 4 waves (RF_OPT_BT_NW, the default
    for launches of few walks) and on one."""
    from rifraf_amd.align import moves_to_proposals_np
    rng = np.random.default_rng(L + bw)
    t = random_seq(L, rng)
    seqs = []
    for _ in range(5):
        r = make_read(t, rng, 0.05, bw)
        if skew > 0:
            extra = random_seq(int(rng.integers(skew // 2, skew + 1)), rng)
            r = RifrafSequence(np.concatenate([r.seq, extra]),
                               np.concatenate([r.error_log_p, np.full(len(extra), -1.0)]), bw, SEQ_SCORES)
        elif skew < 0:
            cut = int(rng.integers(-skew // 2, -skew + 1))
            r = RifrafSequence(r.seq[:len(r.seq) - cut], r.error_log_p[:len(r.seq) - cut], bw, SEQ_SCORES)
        seqs.append(r)
    n = len(seqs)
    opts("band_pad", pad)
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    engine.realign(np.arange(n), np.arange(n), 0, [bw] * n, RF_FWD | RF_BWD)
    opts("bt_win_kb", win_kb)
    opts("bt_nw", nw)
    got, nerr = engine.backtrace(np.arange(n))
    exp_mask = np.zeros((L + 1, 9), np.uint8)
    for k, s in enumerate(seqs):
        _, mv = oracle.forward(t, s, moves=True, bandwidth=bw)
        ref = oracle.backtrace(mv, len(s) + 1, L + 1, bw)
        np.testing.assert_array_equal(got[k], ref)
        assert nerr[k] == oracle.count_errors(ref, t, s.seq)
        kk, p, b = moves_to_proposals_np(ref, t, s.seq)
        exp_mask[p, np.where(kk == 0, b, np.where(kk == 2, 4, 5 + b))] = 1
    np.testing.assert_array_equal(engine.alignment_proposals([np.arange(n)], True)[0], exp_mask)


@pytest.mark.parametrize("nw", [4, 1])
@pytest.mark.parametrize("L,bw,codon", [(90, 9, True), (400, 70, True), (700, 150, False), (520, 140, True)])
def test_backtrace_windowed_codon_and_wide(engine, opts, L, bw, codon, nw):
    """Round 4: k_bt_win also walks codon alignments (reference-style tables:
    TRACE_CODON_INSERT / _DELETE leave the box, the windows cover the +-3
    predecessors) and bands of any height (H = 301 .. 281 here, above the old
    255 limit): moves and error counts against the oracle's trace band, and
    alignment_proposals' fused
    marking against the host union (codon moves propose nothing)."""
    from rifraf_amd.align import moves_to_proposals_np
    rng = np.random.default_rng(L * 3 + bw)
    t = random_seq(L, rng)
    seqs = []
    for k in range(4):
        if codon:
            # a frameshifted copy of the template: codon moves on the path
            r = make_read(t, rng, 0.03, bw).seq
            cut = int(rng.integers(5, len(r) - 5))
            r = np.concatenate([r[:cut], r[cut + 3:]]) if k % 2 else \
                np.concatenate([r[:cut], random_seq(3, rng), r[cut:]])
            lp = np.log10(rng.uniform(0.01, 0.2, len(r)))
            seqs.append(RifrafSequence(r, lp, bw, REF_SCORES))
        else:
            seqs.append(make_read(t, rng, 0.05, bw))
    n = len(seqs)
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    engine.realign(np.arange(n), np.arange(n), 0, [bw] * n, RF_FWD | RF_BWD)
    opts("bt_nw", nw)
    got, nerr = engine.backtrace(np.arange(n))
    exp_mask = np.zeros((L + 1, 9), np.uint8)
    ncod = 0
    for k, s in enumerate(seqs):
        _, mv = oracle.forward(t, s, moves=True, bandwidth=bw)
        ref = oracle.backtrace(mv, len(s) + 1, L + 1, bw)
        ncod += int(np.sum(ref >= 4))
        np.testing.assert_array_equal(got[k], ref)
        assert nerr[k] == oracle.count_errors(ref, t, s.seq)
        kk, p, b = moves_to_proposals_np(ref, t, s.seq)
        exp_mask[p, np.where(kk == 0, b, np.where(kk == 2, 4, 5 + b))] = 1
    if codon:
        assert ncod > 0
    np.testing.assert_array_equal(engine.alignment_proposals([np.arange(n)], True)[0], exp_mask)


def test_validation_skip_follows_state(engine):
    """rf_realign / rf_score_dense skip their per-job checks only for the same
    job / slot list with nothing changed since it was validated: a template
    change must still be refused by a repeated rf_score_dense (stale bands),
    and a re-realign must make it valid again."""
    rng = np.random.default_rng(303)
    t1 = random_seq(100, rng)
    t2 = t1.copy()
    t2[50:53] = (t2[50:53] + 2) % 4
    seqs = [make_read(t1, rng, 0.03, 9) for _ in range(5)]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t1])
    sl = np.arange(5)
    for _ in range(3):                                   # plan built, then reused twice
        engine.realign(sl, sl, 0, [9] * 5, RF_FWD | RF_BWD)
        d1 = engine.score_dense([sl])[0]
    engine.set_templates(0, [t2])
    with pytest.raises(RifrafError):
        engine.score_dense([sl])
    engine.realign(sl, sl, 0, [9] * 5, RF_FWD | RF_BWD)
    d2 = engine.score_dense([sl])[0]
    d2b = engine.score_dense([sl])[0]
    ref2, _ = oracle.cpu_pass(t2, seqs, nthreads=2)
    np.testing.assert_array_equal(d2[1:, 5:], ref2[1:, 5:])
    np.testing.assert_array_equal(d2, d2b)
    assert not np.array_equal(d1[1:, 5:], d2[1:, 5:])


def test_release_bands_then_refill(engine):
    """rf_release_bands drops every band (scoring a dropped slot is refused,
    not read from reused memory), keeps the device memory, and slots filled
    again give the same totals; a second set of alignments then reuses the
    arena from its start."""
    rng = np.random.default_rng(404)
    t = random_seq(150, rng)
    seqs = [make_read(t, rng, 0.03, 9) for _ in range(6)]
    engine.set_sequences(0, seqs)
    engine.set_templates(0, [t])
    sl = np.arange(6)
    engine.realign(sl, sl, 0, [9] * 6, RF_FWD | RF_BWD)
    d1 = engine.score_dense([sl])[0]
    nbytes = engine.device_bytes()
    engine.release_bands()
    assert engine.device_bytes() == nbytes
    with pytest.raises(RifrafError):
        engine.score_dense([sl])
    engine.realign(sl[::-1], sl[::-1], 0, [9] * 6, RF_FWD | RF_BWD)   # other order: other offsets
    d2 = engine.score_dense([sl])[0]
    np.testing.assert_array_equal(d1, d2)
    ref, _ = oracle.cpu_pass(t, seqs, nthreads=2)
    np.testing.assert_array_equal(d2[1:, 5:], ref[1:, 5:])
    assert engine.device_bytes() == nbytes


def test_plan_cache_follows_slot_contents(engine):
    """rf_score_dense reuses its descriptors only while every scored band
    still describes the same alignment: re-filling the same slots with other
    (shorter) reads at the same bandwidth -- bands that fit their old
    regions -- or another bandwidth must rebuild the plan (advisor finding)."""
    rng = np.random.default_rng(91)
    t = random_seq(120, rng)
    long_reads = [make_read(t, rng, 0.03, 9) for _ in range(4)]
    short_reads = [RifrafSequence(r.seq[:-7], r.error_log_p[:-7], 9, SEQ_SCORES)
                   for r in (make_read(t, rng, 0.03, 9) for _ in range(4))]
    sl = np.arange(4)
    engine.set_templates(0, [t])
    engine.set_sequences(0, long_reads)
    engine.set_sequences(4, short_reads)
    for seqs, ids, bw in ((long_reads, sl, 9), (short_reads, sl + 4, 9), (long_reads, sl, 9),
                          (long_reads, sl, 12)):
        engine.realign(sl, ids, 0, [bw] * 4, RF_FWD | RF_BWD)
        got = engine.score_dense([sl])[0]
        ref, _ = oracle.cpu_pass(t, [RifrafSequence(s.seq, s.error_log_p, bw, SEQ_SCORES) for s in seqs],
                                 nthreads=4)
        mask = np.ones_like(ref, bool)
        mask[0, :5] = False
        mask[np.arange(1, len(t) + 1), t.astype(np.int64)] = False
        np.testing.assert_array_equal(got[mask], ref[mask])


def test_row_code_dictionary_overflow():
    """Reads with all-distinct log error probabilities fill the 65 536-entry
    row-code dictionary part way through one upload: later reads stay
    uncoded and their DP reads the tables directly, in the same launches
    (and waves) as coded reads.  Every band stays bit-exact; the overflow is
    counted (rf_code_stats) and a refill of every slot starts a fresh
    dictionary."""
    from rifraf_amd.engine import Engine
    rng = np.random.default_rng(65536)
    L, bw, nreads = 1000, 9, 120   # ~80 continuous reads x 1000 distinct triples > 65 536
    t = random_seq(L, rng)
    seqs = []
    for k in range(nreads):
        r = make_read(t, rng, 0.01, bw)
        lp = -rng.uniform(0.5, 3.0, len(r.seq))   # continuous: every position its own code
        if k % 3 == 0:
            lp = np.round(r.error_log_p, 1)       # phred-like reads interleaved (shared codes)
        seqs.append(RifrafSequence(r.seq, lp, bw, SEQ_SCORES))
    e = Engine(0)
    try:
        _check_bands(e, t, seqs, [bw] * nreads)
        st = e.code_stats()
        assert st["entries3"] == 65536 and st["uncoded_reads"] > 0
        # a refill of every slot: nothing references the old codes, so the
        # dictionary starts afresh and phred-like reads are coded again
        # (the counter keeps its history)
        fresh = [make_read(t, rng, 0.01, bw) for _ in range(nreads)]
        _check_bands(e, t, fresh, [bw] * nreads)
        st2 = e.code_stats()
        assert st2["resets"] >= 1 and st2["entries3"] < 65536
        assert st2["uncoded_reads"] == st["uncoded_reads"]
    finally:
        e.close()


@pytest.mark.parametrize("stage_kb", [16, 262144])
def test_set_sequences_staged_in_chunks(engine, opts, stage_kb):
    """rf_set_sequences stages its tables in bounded chunks (RF_OPT_STAGE_KB):
    with 16 KB chunks this upload of 40 reads spans many chunks; every read's
    bands stay bit-exact (tables and row codes land in the right regions)."""
    opts("stage_kb", stage_kb)
    rng = np.random.default_rng(1601)
    t = random_seq(300, rng)
    seqs = [make_read(t, rng, 0.02, 9) for _ in range(40)]
    _check_bands(engine, t, seqs, [9] * len(seqs))


def test_removed_option_keys_rejected(engine):
    """Scorer-variant keys removed in rounds 3 and 5 (include/rifraf_hip.h)
    are refused with an error, not silently accepted."""
    from rifraf_amd.engine import RifrafError
    for key in (3, 5, 6, 7, 8, 9, 14, 20, 21, 25):
        assert engine.lib.rf_set_option(engine.ctx, key, 1) != 0
        assert "unknown option" in engine.lib.rf_last_error(engine.ctx).decode()
    with pytest.raises(KeyError):
        engine.set_option("seg_ver", 4)
    assert RifrafError is not None


def test_set_sequences_codes_prep_matches_host(engine):
    """Round 5: the native driver's per-read setup values computed on the
    device while uploading (rf_set_sequences_codes_prep, k_code_prep) --
    est_n_errors in Julia 0.6's pairwise order and the initial consensus's
    logsumexp10 (rifrafsequences.jl:19-82, util.jl:28-38) -- equal
    rf_host_code_prep's bit for bit, over lengths on both sides of every
    pairwise-sum edge (16, 1,024, 2,048, 4,096) and of the LDS staging limit
    (32,768), all-Phred-0 reads (an
    infinite maximum match score), and 5,000 reads in one call (two staging
    chunks at 256 KB); the reads' bands equal a plain upload's."""
    rng = np.random.default_rng(2525)
    # (32,768 / 32,769 / 40,000: both sides of k_code_prep's LDS staging limit)
    lens = [1, 2, 15, 16, 17, 1023, 1024, 1025, 1500, 2047, 2048, 2049, 4095, 4096, 4097, 10000, 32768, 32769,
            40000, 3, 3]
    reads = [rng.integers(0, 4, L).astype(np.uint8) for L in lens]
    phreds = [rng.integers(0, 61, L).astype(np.int8) for L in lens]
    phreds[-1][:] = 0                      # every code infinite: lse = match = -Inf
    phreds[-2][1] = 0
    reads += [rng.integers(0, 4, 300).astype(np.uint8) for _ in range(5000)]
    phreds += [rng.integers(5, 45, 300).astype(np.int8) for _ in range(5000)]
    off = np.zeros(len(reads) + 1, np.int64)
    np.cumsum([len(r) for r in reads], out=off[1:])
    cat = np.concatenate(phreds)
    allb = np.concatenate(reads)
    host = RifrafSequence.many_coded(reads, cat, off, 9, SEQ_SCORES)
    got = {}

    def dev(code, lp_t, match_t, p10, grid):
        got["r"] = engine.set_sequences_codes(0, allb, off, code, lp_t, match_t, SEQ_SCORES, prep=(p10, grid))
        return got["r"]
    try:
        engine.set_option("stage_kb", 256)
        devr = RifrafSequence.many_coded(reads, cat, off, 9, SEQ_SCORES, device=dev)
    finally:
        engine.set_option("stage_kb", 262144)
    assert devr[1]["uploaded"] and got["r"] is not False
    est_h = np.array([r.est_n_errors for r in host[0]])
    est_d = np.array([r.est_n_errors for r in devr[0]])
    assert est_h.view(np.int64).tolist() == est_d.view(np.int64).tolist()
    assert host[2].view(np.int64).tolist() == devr[2].view(np.int64).tolist()   # lse, -Inf included
    # the upload itself: bands of a few reads equal a plain rf_set_sequences_codes upload's
    t = reads[len(lens) + 2]
    engine.set_templates(0, [t])
    sl = np.arange(len(lens), len(lens) + 6)     # 300-base reads
    a1 = engine.realign(sl, sl, 0, [9] * 6, RF_FWD)
    tabs = host[1]
    assert engine.set_sequences_codes(0, allb, off, tabs["code"], tabs["lp_table"], tabs["match_table"], SEQ_SCORES)
    a2 = engine.realign(sl, sl, 0, [9] * 6, RF_FWD)
    np.testing.assert_array_equal(a1, a2)


@pytest.mark.parametrize("scores", ["seq", "other"])
def test_set_sequences_codes_matches_host_tables(engine, scores):
    """rf_set_sequences_codes (tables built on the device from Phred codes)
    gives the same bands, A[end,end], backtraces and dense totals as
    rf_set_sequences of the host tables (RifrafSequence.many_concat), and
    both equal the oracle: lengths from 1 to 400, Phred 0 (an infinite
    match score: the general kernels) among them."""
    from rifraf_amd.errormodel import phred_to_log_p
    from rifraf_amd.sample import sample_sequences
    sc = SEQ_SCORES if scores == "seq" else Scores.from_errors(ErrorModel(2.0, 1.0, 3.0, 0.0, 0.0))
    rng = np.random.default_rng(3131)
    _, t, _, reads, _, phreds, _, _ = sample_sequences(24, 400, error_rate=0.03, rng=rng)
    reads, phreds = list(reads), [np.asarray(p, np.int8).copy() for p in phreds]
    reads[3], phreds[3] = reads[3][:1], phreds[3][:1]              # a one-base read
    phreds[5][7] = 0                                                # Phred 0: match = -Inf
    lens = np.array([len(r) for r in reads])
    off = np.zeros(len(reads) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    cat = np.concatenate(phreds)
    seqs, tabs = RifrafSequence.many_concat(reads, phred_to_log_p(cat), off, 9, sc, phreds=cat)
    n = len(seqs)
    sl = np.arange(n)
    bws = [9] * n
    allb = np.concatenate(reads).astype(np.uint8)
    out = []
    for path in ("codes", "host"):
        if path == "codes":
            assert engine.set_sequences_codes(0, allb, off, tabs["code"], tabs["lp_table"], tabs["match_table"], sc)
        else:
            engine.set_sequences_concat(0, allb, off, tabs["match"], tabs["mismatch"], tabs["ins"], tabs["del"])
        engine.set_templates(0, [t])
        scs = engine.realign(sl, sl, 0, bws, RF_FWD | RF_BWD)
        bands = [(engine.download_band(k, RF_BAND_A).data.copy(), engine.download_band(k, RF_BAND_B).data.copy())
                 for k in range(n)]
        mv, ne = engine.backtrace(list(range(n)))
        dense = engine.score_dense([sl])[0]
        out.append((scs, bands, mv, ne, dense))
    (s1, b1, m1, e1, d1), (s2, b2, m2, e2, d2) = out
    np.testing.assert_array_equal(s1, s2)
    for (a1, bb1), (a2, bb2) in zip(b1, b2):
        np.testing.assert_array_equal(a1, a2)
        np.testing.assert_array_equal(bb1, bb2)
    for x, y in zip(m1, m2):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_array_equal(d1, d2)
    for k in (0, 3, 5, n - 1):
        A_exp, _ = oracle.forward(t, seqs[k])
        assert_band_equal(engine.download_band(k, RF_BAND_A), A_exp, len(seqs[k]) + 1, len(t) + 1, 9)
