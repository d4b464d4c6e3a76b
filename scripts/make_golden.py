#!/usr/bin/env python
"""Generate the committed golden fixtures (SURVEY.md §8(c) "Fixtures to
commit") from the CPU oracle, which tests/test_oracle_kats.py pins to the
reference's own known-answer tests:

  tests/golden/pairs.npz      seeded (template, read) pairs with and without
                              codon moves: A / B bands (in-band cells,
                              column-major order), A[end,end], backtrace
                              moves, error counts, and every STAGE_SCORE
                              proposal total (single-read fold)
  tests/golden/config2.json   whole rifraf() runs on config-2-shaped
                              clusters (default params): final consensus,
                              score and stage iterations
  tests/golden/runs.npz       whole rifraf() runs at the BASELINE configs'
                              own shapes, the ones bench.py times: configs[1]
                              (sample_sequences(100, 1000; error_rate=0.01),
                              seeds 1..5, default params and the throughput
                              settings) and configs[2] (bench.c3_cluster(),
                              throughput settings) -- consensus, score, stage
                              iterations, penalty increases, every stage's
                              consensuses and the QVs; bench's c2 / c3 fields
                              check their native runs against these

usage: python scripts/make_golden.py   (deterministic; rerun to refresh)"""
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from _util import REF_SCORES, all_proposals_arrays, dense_slot, inband_mask, make_read, random_seq  # noqa: E402
from oracle_engine import OracleEngine  # noqa: E402
from rifraf_amd import RifrafSequence, dna_str  # noqa: E402
from rifraf_amd.model import RifrafParams, rifraf  # noqa: E402
from rifraf_amd.sample import sample_sequences  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")


def pairs():
    rng = np.random.default_rng(20240101)
    recs = []
    for k in range(20):
        codon = k >= 14
        L = int(rng.integers(12, 70))
        bw = int(rng.integers(2, 12))
        t = random_seq(L, rng)
        if codon:
            s = random_seq(max(4, L + int(rng.integers(-6, 7))), rng)
            seq = RifrafSequence(s, np.log10(rng.uniform(0.02, 0.2, len(s))), bw, REF_SCORES)
        else:
            seq = make_read(t, rng, float(rng.choice([0.02, 0.05, 0.1])), bw)
        A, mv = oracle.forward(t, seq, moves=True)
        B = oracle.backward(t, seq)
        n, m = len(seq), L
        mask = inband_mask(n + 1, m + 1, bw)
        moves = oracle.backtrace(mv, n + 1, m + 1, bw)
        nerr = oracle.count_errors(moves, t, seq.seq)
        d_end = n - m + max(m - n, 0) + bw
        kind, pos, base = all_proposals_arrays(t)
        try:    # single-sequence fold 0.0 + s (model.jl:389-397); a read as batch, codon as reference
            tot = np.array([0.0 + oracle.score_proposal(int(a), int(b), int(c), A, B, t, seq)
                            for a, b, c in zip(kind, pos, base)])
        except oracle.OracleError:
            tot = np.zeros(0)       # the reference raises on some proposal: no totals fixture
        recs.append(dict(template=t, read=seq.seq, lp=seq.error_log_p, bw=bw, codon=codon,
                         A=A.T[mask.T], B=B.T[mask.T], score=A[d_end, m], moves=moves, nerr=nerr,
                         kind=kind, pos=pos, base=base, totals=tot))
    flat = {}
    for k, r in enumerate(recs):
        for key, v in r.items():
            flat[f"p{k}_{key}"] = np.asarray(v)
    flat["npairs"] = np.asarray(len(recs))
    np.savez_compressed(os.path.join(OUT, "pairs.npz"), **flat)


def config2():
    runs = []
    for seed in (1, 2, 3):
        rng = np.random.default_rng(seed)
        _, t, _, reads, _, phreds, _, _ = sample_sequences(20, 200, error_rate=0.02, rng=rng)
        res = rifraf(reads, phreds, params=RifrafParams(), engine=OracleEngine())
        runs.append({"seed": seed, "nreads": 20, "length": 200, "error_rate": 0.02,
                     "template": dna_str(t), "consensus": dna_str(res.consensus), "score": res.state.score.hex(),
                     "stage_iterations": list(res.state.stage_iterations)})
    json.dump({"generator": "scripts/make_golden.py (CPU oracle engine)", "runs": runs},
              open(os.path.join(OUT, "config2.json"), "w"), indent=1)


def run_record(res):
    """A whole rifraf() result as flat arrays (see runs())."""
    st = res.consensus_stages
    rec = dict(consensus=np.asarray(res.consensus, np.uint8), score=np.float64(res.state.score),
               iters=np.asarray(res.state.stage_iterations, np.int64),
               mults=np.int64(res.state.n_ref_indel_mults), converged=np.bool_(res.state.converged),
               stage_counts=np.asarray([len(x) for x in st], np.int64),
               stage_lens=np.asarray([len(c) for x in st for c in x], np.int64),
               stages=np.concatenate([np.asarray(c, np.uint8) for x in st for c in x] or [np.zeros(0, np.uint8)]))
    if res.error_probs is not None:
        rec.update(sub=res.error_probs.sub, dele=res.error_probs.dele, ins=res.error_probs.ins,
                   aln=np.asarray(res.aln_error_probs))
    return rec


C2_VARIANTS = {"default": dict(seed=1),
               "throughput": dict(seed=1, batch_size=0, batch_fixed=False, do_score=True)}


def c2_cluster(seed):
    """configs[1]: sample_sequences(100, 1000; error_rate=0.01) (sample.jl:277-298)."""
    rng = np.random.default_rng(seed)
    _, t, _, reads, _, phreds, _, _ = sample_sequences(100, 1000, error_rate=0.01, rng=rng)
    return t, reads, phreds


def runs():
    sys.path.insert(0, REPO)
    import bench
    out = {}
    for seed in range(1, 6):
        t, reads, phreds = c2_cluster(seed)
        for var, kw in C2_VARIANTS.items():
            res = rifraf(reads, phreds, params=RifrafParams(**kw), engine=OracleEngine())
            for k, v in run_record(res).items():
                out[f"c2_{seed}_{var}_{k}"] = v
    t, reads, phreds, ref = bench.c3_cluster()
    res = rifraf(reads, phreds, reference=ref, params=RifrafParams(**C2_VARIANTS["throughput"]),
                 engine=OracleEngine())
    for k, v in run_record(res).items():
        out[f"c3_throughput_{k}"] = v
    out.update(c3_default_record())
    out["generator"] = np.asarray("scripts/make_golden.py runs() (CPU oracle engine)")
    np.savez_compressed(os.path.join(OUT, "runs.npz"), **out)


C3_DEFAULT = dict(seed=1, do_score=True)


def c3_default_record():
    """configs[2] with the default batches: the fixed 5 lowest-error reads in
    INIT / FRAME, then REFINE's random batches of 20 (resampling.py's RNG,
    seed 1), QVs on."""
    sys.path.insert(0, REPO)
    import bench
    t, reads, phreds, ref = bench.c3_cluster()
    res = rifraf(reads, phreds, reference=ref, params=RifrafParams(**C3_DEFAULT), engine=OracleEngine())
    rec = {f"c3_default_{k}": v for k, v in run_record(res).items()}
    rec["c3_default_batch"] = np.asarray(res.state.batch_seqs, np.int64)
    return rec


def runs_c3_default():
    """Add (or replace) the c3_default record of runs.npz, keeping the rest."""
    path = os.path.join(OUT, "runs.npz")
    with np.load(path) as z:
        out = {k: z[k] for k in z.files}
    out = {k: v for k, v in out.items() if not k.startswith("c3_default_")}
    out.update(c3_default_record())
    np.savez_compressed(path, **out)


if __name__ == "__main__":
    what = sys.argv[1:] or ["pairs", "config2", "runs"]
    for w in what:
        {"pairs": pairs, "config2": config2, "runs": runs, "runs_c3_default": runs_c3_default}[w]()
        print("wrote", w)
