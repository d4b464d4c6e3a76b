#!/usr/bin/env python
"""Classify the bench e2e clusters whose consensus is not the template
(VERDICT r03 Next 5).  CPU only: the whole rifraf() runs go through the
oracle engine (tests/oracle_engine.py, the KAT-pinned C restatement), so the
classification does not depend on the HIP engine under test.

For every cluster of bench.py's e2e field (sample_sequences(50, 1500), error
0.01, seeds [seed, 77, rank, k]; RifrafParams(batch_size=0, batch_fixed=False);
do_score off -- the QV pass runs after convergence and cannot change the
consensus) whose final consensus C differs from the template T:

  * score(C) = the final state.score (the fold of A[end,end] over every read,
    model.jl:630-635) and score(T) = the same fold with T as consensus, every
    read at its final bandwidth;
  * better = every STAGE_SCORE proposal of C whose total beats score(C)
    (score > state.score, model.jl:521) -- the dense totals of all 8m+4
    single edits (oracle.cpu_pass);
  * aln = the INIT alignment-proposal set of C (model.jl:483-497: the union of
    the reads' backtrace differences, indels included);
  * path = the single edits of C that lower edit_distance(C, T) by one.

Classes:
  template_scores_lower   score(T) <= score(C): the model prefers C;
  local_optimum           no proposal in `aln` beats C (the reference's INIT
                          stops exactly here, model.jl:499-526,937-950);
                          sub-labelled by whether an improving edit exists at
                          all and whether one lies on the path to T;
  score_unchanged_stop    the last iteration ended on check_score's
                          'score did not change' rule (model.jl:1081-1086);
  max_iters               the run did not converge;
  SLIP                    a proposal in `aln` beats score(C) although the run
                          converged: the host restatement stopped early.

usage: python scripts/explain_misses.py [--clusters 512] [--procs 8] [--out profiles/r04_e2e_misses.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

os.environ.setdefault("OMP_NUM_THREADS", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def ed_matrix(a, b):
    """F[i, j] = unit-cost edit distance of a[:i] and b[:j], one numpy row at
    a time (the insertion chain of a row is a running minimum)."""
    a = np.asarray(a, np.int64)
    b = np.asarray(b, np.int64)
    nb = len(b)
    ar = np.arange(nb + 1)
    F = np.empty((len(a) + 1, nb + 1), np.int64)
    F[0] = ar
    for i, x in enumerate(a, 1):
        tmp = np.empty(nb + 1, np.int64)
        tmp[0] = F[i - 1, 0] + 1
        tmp[1:] = np.minimum(F[i - 1, 1:] + 1, F[i - 1, :-1] + (b != x))
        F[i] = np.minimum.accumulate(tmp - ar) + ar
    return F


def path_edits(c, t):
    """Single edits of c that lie on an optimal edit script to t (each lowers
    edit_distance(c, t) by one), as (kind, pos, base) proposals in the
    reference's coordinates (Sub/Del 1-based position, Ins after position p).
    F = prefix distances, G = suffix distances: an edit is on a path when
    F[..] + 1 + G[..] == ED at some column."""
    c = np.asarray(c, np.int64)
    t = np.asarray(t, np.int64)
    F = ed_matrix(c, t)
    G = ed_matrix(c[::-1], t[::-1])[::-1, ::-1]    # G[i, j] = ed(c[i:], t[j:])
    ed = int(F[-1, -1])
    n, m = len(c), len(t)
    out = set()
    for p in range(1, n + 1):                      # Del(p), Sub(p, b): c[p-1] edited
        if np.any(F[p - 1, :] + 1 + G[p, :] == ed):
            out.add((2, p, 0))
        j = np.nonzero(F[p - 1, :m] + 1 + G[p, 1:] == ed)[0]
        for jj in j:
            if t[jj] != c[p - 1]:
                out.add((0, p, int(t[jj])))
    for p in range(0, n + 1):                      # Ins(p, b): t[j] inserted after c[p-1]
        j = np.nonzero(F[p, :m] + 1 + G[p, 1:] == ed)[0]
        for jj in j:
            out.add((1, p, int(t[jj])))
    return ed, out


def run_cluster(k, seed, rank):
    from oracle_engine import OracleEngine
    from rifraf_amd.model import RifrafParams, rifraf
    from rifraf_amd.sample import sample_sequences
    _, t, _, reads, _, phreds, _, _ = sample_sequences(
        50, 1500, error_rate=0.01, rng=np.random.default_rng([seed, 77, rank, k]))
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=False, verbose=2)
    import rifraf_amd.model as model
    msgs = []
    model.log = lambda params, level, msg: msgs.append(msg) if level <= params.verbose else None
    res = rifraf(reads, phreds, params=params, engine=OracleEngine())
    stops = [x.strip() for x in msgs if "score did not change" in x or "no candidates found" in x]
    c = np.asarray(res.consensus, np.uint8)
    t = np.asarray(t, np.uint8)
    out = {"cluster": k, "equal": bool(np.array_equal(c, t)), "converged": bool(res.state.converged),
           "iterations": int(sum(res.state.stage_iterations)), "len_c": len(c), "len_t": len(t),
           "stop": stops[-1] if stops else None}
    if out["equal"]:
        return out
    return analyse(out, res, c, t)


def analyse(out, res, c, t):
    import oracle
    from rifraf_amd.align import moves_to_proposals_np
    st = res.state
    seqs = [st.sequences[i] for i in st.batch_seqs]
    out["score_c"] = float(st.score)
    # score(T): the same fold with T as the consensus, reads at their final bandwidths
    tot = 0.0
    for k, s in enumerate(seqs):
        A, _ = oracle.forward(t, s, moves=True, bandwidth=s.bandwidth)
        v = float(A[len(s) - len(t) + max(len(t) - len(s), 0) + s.bandwidth, len(t)])
        tot = v if k == 0 else tot + v
    out["score_t"] = tot
    # all single edits of C (dense STAGE_SCORE totals, slots Sub A..T, Del, Ins A..T)
    dense, _ = oracle.cpu_pass(c, seqs, nthreads=int(os.environ.get("OMP_NUM_THREADS", "1")))
    m = len(c)
    better = set()
    for p in range(m + 1):
        for sl in range(9):
            if sl < 4 and (p == 0 or c[p - 1] == sl):
                continue
            if sl == 4 and p == 0:
                continue
            if dense[p, sl] > st.score:
                kind = 0 if sl < 4 else (2 if sl == 4 else 1)
                base = sl if sl < 4 else (0 if sl == 4 else sl - 5)
                better.add((kind, p, base))
    # INIT alignment proposals of C (union over the batch reads, indels included)
    aln = set()
    for s in seqs:
        _, mv = oracle.forward(c, s, moves=True, bandwidth=s.bandwidth)
        moves = oracle.backtrace(mv, len(s) + 1, m + 1, s.bandwidth)
        kk, pp, bb = moves_to_proposals_np(moves, c, s.seq)
        aln.update(zip(kk.tolist(), pp.tolist(), bb.tolist()))
    # the path: single edits of C that bring it one edit closer to T
    ed, path = path_edits(c, t)
    out.update({
        "edit_distance": ed,
        "n_better": len(better), "n_aln": len(aln), "n_path": len(path),
        "better_in_aln": sorted(better & aln), "better_on_path": sorted(better & path),
        "path": sorted(path)[:12],
        "best_path_total": max((float(dense[p, (b if k == 0 else (4 if k == 2 else 5 + b))])
                                for k, p, b in path), default=None),
    })
    if out["score_t"] <= out["score_c"]:
        cls = "template_scores_lower"
    elif not out["converged"]:
        cls = "max_iters"
    elif better & aln and "score did not change" in (out["stop"] or ""):
        cls = "score_unchanged_stop"
    elif better & aln:
        cls = "SLIP"
    else:
        cls = "local_optimum"
        if not better:
            cls += ":no_single_edit_improves"
        elif better & path:
            cls += ":improving_path_edit_not_proposed_by_reads"
        else:
            cls += ":improving_edits_off_path_not_proposed"
    out["class"] = cls
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=512)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r04_e2e_misses.json"))
    args = ap.parse_args()
    t0 = time.time()
    ks = list(range(args.first, args.first + args.clusters))
    with Pool(args.procs) as pool:
        rows = pool.starmap(run_cluster, [(k, args.seed, args.rank) for k in ks], chunksize=1)
    misses = [r for r in rows if not r["equal"]]
    classes = {}
    for r in misses:
        classes[r["class"]] = classes.get(r["class"], 0) + 1
    summary = {"source": "scripts/explain_misses.py (oracle engine, CPU)",
               "workload": "bench.py e2e: sample_sequences(50, 1500), error 0.01, seeds [seed, 77, rank, k]",
               "seed": args.seed, "rank": args.rank, "clusters": len(rows),
               "consensus_equals_template": len(rows) - len(misses), "misses": len(misses),
               "classes": classes, "seconds": time.time() - t0, "rows": misses}
    with open(args.out, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "rows"}))


if __name__ == "__main__":
    main()
