"""Read-sharded rifraf() (rifraf_amd.sharded) on CPU with
gloo: world sizes 2, 3 and 8 (one node's GPUs), every rank wrapping the
oracle engine.

* whole rifraf() runs through ShardedEngine give the same consensus at every
  iteration, the same final score and the same quality estimates as one
  unsharded engine -- bit-exact, because the per-proposal fold is carried
  from rank to rank in the reference's order (model.jl:389-397);
* the dense exchange (per-rank partial fold + all-gather + rank-order sum)
  agrees with the one-process fold within the north_star's 1e-9 relative.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
G1 = os.path.join(HERE, "golden", "config1")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(fn, world, *args, backend="gloo"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, backend) + args) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    errs = [g for g in got if g[1] == "error"]
    assert not errs, errs[0][2]
    return dict((r, v) for r, _, v in got)


def _entry(fn, rank, world, port, q, backend, *args):
    import traceback
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        torch.cuda.set_device(rank)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        q.put((rank, "ok", fn(rank, world, *args)))
    except Exception:
        q.put((rank, "error", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


# ----------------------------------------------------------------------
def _config1(engine_factory, f, refid):
    from rifraf_amd import ErrorModel, Scores, cap_phreds
    from rifraf_amd.fastxio import read_fasta_records, read_fastq
    from rifraf_amd.model import RifrafParams, rifraf
    refs = dict(read_fasta_records(os.path.join(G1, "references.fasta")))
    seqs, phreds, _ = read_fastq(os.path.join(G1, f))
    phreds = [cap_phreds(p, 30) for p in phreds]
    params = RifrafParams(scores=Scores.from_errors(ErrorModel(1, 2, 2)),
                          ref_scores=Scores.from_errors(ErrorModel(8, 0.1, 0.1, 1, 1)), max_iters=100,
                          do_score=True)
    res = rifraf(seqs, phreds, reference=refs[refid], params=params, engine=engine_factory(len(seqs)))
    return summary(res)


def _sampled(engine_factory, seed):
    from rifraf_amd.model import RifrafParams, rifraf
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(seed)
    _, _, _, reads, _, phreds, _, _ = sample_sequences(7, 70, error_rate=0.03, rng=rng)
    params = RifrafParams(do_score=True, max_iters=30)
    res = rifraf(reads, phreds, params=params, engine=engine_factory(len(reads)))
    return summary(res)


def _grown(engine_factory, seed, out=None):
    """A run whose batch grows (check_score!, model.jl:1094-1112): batch_size 3
    of 12 reads, batch_threshold 0 (any score drop grows the batch), a fixed seed for
    resample!'s weighted draws (seed 1 grows it to all 12 reads)."""
    from rifraf_amd.model import RifrafParams, rifraf
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(seed)
    _, _, _, reads, _, phreds, _, _ = sample_sequences(12, 60, error_rate=0.05, rng=rng)
    params = RifrafParams(batch_size=3, batch_fixed=False, batch_threshold=0.0, max_iters=30, seed=11)
    eng = engine_factory(len(reads))
    res = rifraf(reads, phreds, params=params, engine=eng)
    s = summary(res)
    s["batch_size"] = res.state.batch_size
    if hasattr(eng, "slot_counts"):
        s["counts"] = eng.slot_counts(np.arange(res.state.batch_size))
    return s


def summary(res):
    st = res.state
    return {"consensus": np.asarray(res.consensus).copy(), "score": st.score,
            "stages": [[np.asarray(c).copy() for c in s] for s in res.consensus_stages],
            "iters": list(st.stage_iterations), "converged": st.converged,
            "sub": None if res.error_probs is None else res.error_probs.sub.copy(),
            "ins": None if res.error_probs is None else res.error_probs.ins.copy(),
            "dele": None if res.error_probs is None else res.error_probs.dele.copy(),
            "aln": None if res.aln_error_probs is None else np.asarray(res.aln_error_probs).copy()}


def _sharded_factory(n):
    from oracle_engine import OracleEngine
    from rifraf_amd.sharded import ShardedEngine
    return ShardedEngine(OracleEngine(), n)


def _plain_factory(n):
    from oracle_engine import OracleEngine
    return OracleEngine()


def _w_config1(rank, world, f, refid):
    return _config1(_sharded_factory, f, refid)


def _w_sampled(rank, world, seed):
    return _sampled(_sharded_factory, seed)


# device quality pass (rifraf_batch(device_qv=True): 10^x by the GPU's exp10)
# against a host evaluation: relative / absolute tolerance of the QVs
QV_RTOL, QV_ATOL = 1e-12, 1e-15


def assert_same_run(a, b, qv_rtol=0.0):
    np.testing.assert_array_equal(a["consensus"], b["consensus"])
    assert a["score"] == b["score"]
    assert a["iters"] == b["iters"] and a["converged"] == b["converged"]
    assert len(a["stages"]) == len(b["stages"])
    for x, y in zip(a["stages"], b["stages"]):
        assert len(x) == len(y)
        for c1, c2 in zip(x, y):
            np.testing.assert_array_equal(c1, c2)
    for k in ("sub", "dele", "ins", "aln"):
        if a[k] is None:
            assert b[k] is None
        elif qv_rtol:
            np.testing.assert_allclose(a[k], b[k], rtol=qv_rtol, atol=QV_ATOL, err_msg=k)
        else:
            np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_config1_with_reference(world):
    """Reference-informed run (FRAME stage, codon scoring on the last rank's
    reference slot) with quality scores: identical to one engine.  At world
    8 the 3 reads leave five ranks without a read slot."""
    f = "input-reads-1.fastq"
    refmap = dict(line.split() for line in open(os.path.join(G1, "ref-map.tsv")) if line.strip())
    refid = refmap[f]
    single = _config1(_plain_factory, f, refid)
    got = _spawn(_w_config1, world, f, refid)
    for r in range(world):
        assert_same_run(got[r], single)


def _w_grown(rank, world, seed):
    return _grown(_sharded_factory, seed)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_batch_growth(world):
    """check_score! grows the batch from 3 reads towards all 12: the sharded
    run equals one engine bit for bit, and the grown batch's bands stay
    spread over the ranks (round-robin slots, at most one read apart)."""
    single = _grown(_plain_factory, 1)
    assert single["batch_size"] > 3
    got = _spawn(_w_grown, world, 1)
    for r in range(world):
        g = dict(got[r])
        counts = g.pop("counts")
        assert g.pop("batch_size") == single["batch_size"]
        assert_same_run(g, {k: v for k, v in single.items() if k != "batch_size"})
        assert sum(counts) == single["batch_size"] and max(counts) - min(counts) <= 1


def test_sharded_sampled_cluster():
    single = _sampled(_plain_factory, 5)
    got = _spawn(_w_sampled, 2, 5)
    for r in range(2):
        assert_same_run(got[r], single)


# ----------------------------------------------------------------------
def _w_dense(rank, world, seed):
    from _util import make_read
    from oracle_engine import OracleEngine
    from rifraf_amd.engine import RF_BWD, RF_FWD
    from rifraf_amd.sample import random_seq
    from rifraf_amd.sharded import ShardedEngine
    rng = np.random.default_rng(seed)
    tpls = [random_seq(int(rng.integers(40, 70)), rng) for _ in range(2)]
    reads = [[make_read(t, rng, 0.04, 6) for _ in range(int(rng.integers(3, 7)))] for t in tpls]
    flat = [r for rs in reads for r in rs]
    e = ShardedEngine(OracleEngine(), len(flat))
    e.set_sequences(0, flat)
    e.set_templates(0, tpls)
    tpl_of = np.concatenate([[c] * len(rs) for c, rs in enumerate(reads)])
    n = len(flat)
    e.realign(np.arange(n), np.arange(n), tpl_of, [6] * n, RF_FWD | RF_BWD)
    groups, at = [], 0
    for rs in reads:
        groups.append(np.arange(at, at + len(rs)))
        at += len(rs)
    return e.score_dense(groups), tpls, reads


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_dense_exchange(world):
    import oracle
    got = _spawn(_w_dense, world, 17)
    dense0, tpls, reads = got[0]
    for r in range(1, world):
        for a, b in zip(got[r][0], dense0):
            np.testing.assert_array_equal(a, b)        # every rank holds the same totals
    for c, t in enumerate(tpls):
        exp, _ = oracle.cpu_pass(t, reads[c], nthreads=2)
        mask = np.isfinite(exp)
        assert (np.isfinite(dense0[c]) == mask).all()
        # regrouped sum: 1e-9 relative is the north_star bar; the bound here is far tighter
        np.testing.assert_allclose(dense0[c][mask], exp[mask], rtol=1e-12, atol=0)


def test_shard_bounds_and_owner():
    from rifraf_amd.sharded import shard_bounds
    for n, w in [(10, 3), (5000, 8), (3, 4), (1, 1)]:
        b = shard_bounds(n, w)
        assert b[0] == 0 and b[-1] == n and all(x <= y for x, y in zip(b, b[1:]))
        sizes = np.diff(b)
        assert sizes.max() - sizes.min() <= 1


def _w_counts(rank, world):
    from oracle_engine import OracleEngine
    from rifraf_amd.model import RifrafParams
    from rifraf_amd.sharded import ShardedEngine
    out = {}
    for bs, nreads in [(20, 5000), (0, 5000), (1, 12), (20, 7)]:
        e = ShardedEngine.for_params(OracleEngine(), nreads, RifrafParams(batch_size=bs))
        batch = min(nreads, bs) if bs > 1 else nreads
        out[(bs, nreads)] = (e.slot_counts(np.arange(batch)), e.slot_counts(np.arange(nreads)),
                             e.owner(nreads), e.owner(nreads + 1))
    return out


def test_sharded_slot_balance():
    """ShardedEngine deals the read slots round-robin, so every batch prefix
    rifraf() fills (batch_size, and the larger batches check_score! grows it
    to) is balanced within one read; reference/scratch slots (>= nreads) go
    to the last rank."""
    got = _spawn(_w_counts, 2)
    for r in range(2):
        c = got[r]
        assert c[(20, 5000)][:2] == ([10, 10], [2500, 2500])
        assert c[(0, 5000)][:2] == ([2500, 2500], [2500, 2500])
        assert c[(1, 12)][:2] == ([6, 6], [6, 6])
        assert c[(20, 7)][:2] == ([4, 3], [4, 3])
        for v in c.values():
            assert v[2] == v[3] == 1


def _w_unfilled(rank, world):
    """results of a slot whose bands were never filled through the
    sharded engine, or of an unknown template, raise the engine's error (on
    every rank, before any collective) instead of a KeyError."""
    from _util import make_read
    from oracle_engine import OracleEngine
    from rifraf_amd.engine import RF_BWD, RF_FWD, RifrafError
    from rifraf_amd.sample import random_seq
    from rifraf_amd.sharded import ShardedEngine
    rng = np.random.default_rng(3)
    t = random_seq(50, rng)
    reads = [make_read(t, rng, 0.03, 6) for _ in range(4)]
    e = ShardedEngine(OracleEngine(), len(reads))
    e.set_sequences(0, reads)
    e.set_templates(0, [t])
    msgs = []
    for call in (lambda: e.score_dense([np.arange(4)]),
                 lambda: e.realign(np.arange(4), np.arange(4), 3, [6] * 4, RF_FWD)):
        try:
            call()
        except RifrafError as err:
            msgs.append(str(err))
    e.realign(np.arange(4), np.arange(4), 0, [6] * 4, RF_FWD | RF_BWD)
    shapes = [e.score_dense([np.arange(4)])[0].shape]   # m = 50
    e.set_templates(0, [random_seq(40, rng)])
    e.realign(np.arange(4), np.arange(4), 0, [6] * 4, RF_FWD | RF_BWD)
    shapes.append(e.score_dense([np.arange(4)])[0].shape)   # refilled: m = 40
    return msgs, shapes


def test_sharded_unfilled_slot_and_unknown_template():
    got = _spawn(_w_unfilled, 2)
    for r in range(2):
        msgs, shapes = got[r]
        assert len(msgs) == 2
        assert "no bands filled" in msgs[0] and "unknown template" in msgs[1]
        assert shapes == [(51, 9), (41, 9)]


def _w_queue(rank, world, n, wave):
    """Each rank takes waves from the store-backed queue and runs them on the
    oracle engine (the Python stage machine)."""
    import time
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import ClusterQueue, rifraf_batch_queue
    from rifraf_amd.model import RifrafParams
    if rank == 1:
        ClusterQueue(5, 1)   # a local queue on one rank only must not shift the store-backed keys
    q = ClusterQueue.for_process_group(n, wave)
    params = RifrafParams(max_iters=20)

    def get(i):
        if rank == 0:
            time.sleep(0.05)   # a slow rank: the others take more waves
        return _queue_cluster(i)
    res = rifraf_batch_queue(get, q, params=params, engine=OracleEngine())
    return {i: np.asarray(r.consensus).tolist() for i, r in res.items()}


def _queue_cluster(i):
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng([99, i])
    _, _, _, reads, _, phreds, _, _ = sample_sequences(4, 40, error_rate=0.03, rng=rng)
    return dict(dnaseqs=reads, phreds=phreds)


@pytest.mark.parametrize("world", [3, 8])
def test_cluster_queue_across_ranks(world):
    """The cross-rank cluster queue (pmap's dynamic hand-out,
    scripts/rifraf.jl:190): every cluster runs on exactly one rank (rank 0 is
    made slow, so the hand-out is uneven; how uneven depends on the host's
    load, so only the exactly-once property is asserted) and each result
    equals one process's run."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.model import RifrafParams
    n, wave = 13, 2
    got = _spawn(_w_queue, world, n, wave)
    seen = {}
    for r in range(world):
        for i, c in got[r].items():
            assert i not in seen
            seen[i] = c
    assert sorted(seen) == list(range(n))
    single = rifraf_batch([_queue_cluster(i) for i in range(n)], params=RifrafParams(max_iters=20),
                          engine=OracleEngine())
    for i in range(n):
        assert seen[i] == np.asarray(single[i].consensus).tolist()


def _w_queue_mismatch(rank, world):
    """Ranks that disagree on a queue's shape fail loudly at creation."""
    from rifraf_amd.batch import ClusterQueue
    try:
        ClusterQueue.for_process_group(10 if rank == 0 else 11, 2, key="mismatch")
    except RuntimeError as e:
        return str(e)
    return "ok"


def test_cluster_queue_mismatch_is_loud():
    got = _spawn(_w_queue_mismatch, 3)
    assert got[0] == "ok"
    for r in (1, 2):
        assert "rank 0 published" in got[r]


def _w_queue_fail(rank, world, n, wave):
    """Rank 1 raises inside its first wave: every rank still reaches the
    barrier; rank 1 re-raises its own error, the others a RuntimeError."""
    from oracle_engine import OracleEngine
    from rifraf_amd.batch import ClusterQueue, rifraf_batch_queue
    from rifraf_amd.model import RifrafParams
    q = ClusterQueue.for_process_group(n, wave)

    def get(i):
        if rank == 1:
            raise ValueError(f"bad cluster {i}")
        return _queue_cluster(i)
    try:
        rifraf_batch_queue(get, q, params=RifrafParams(max_iters=20), engine=OracleEngine())
    except Exception as e:  # noqa: BLE001
        return type(e).__name__, str(e)
    return "ok", ""


def test_cluster_queue_failure_reaches_every_rank():
    got = _spawn(_w_queue_fail, 3, 40, 1)
    assert got[1][0] == "ValueError"
    for r in (0, 2):
        assert got[r][0] == "RuntimeError" and "rank 1 failed" in got[r][1]


# ----------------------------------------------------------------------
def _idle_cpus_rank(rank, world):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    allowed = sorted(os.sched_getaffinity(0))
    return bench.idle_cpus(allowed, 2, dist), allowed


def test_bench_pins_ranks_to_disjoint_idle_cpus():
    """bench's pinned e2e passes: each rank takes the 2 idlest of its allowed
    cpus, disjoint across ranks (world 3, gloo); one process takes 2 of its
    allowed cpus."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    allowed = sorted(os.sched_getaffinity(0))
    one = bench.idle_cpus(allowed, 2)
    assert len(set(one)) == min(2, len(allowed)) and set(one) <= set(allowed)
    got = _spawn(_idle_cpus_rank, 3)
    picks = [got[r][0] for r in range(3)]
    if len(allowed) >= 6:
        assert len(set().union(*map(set, picks))) == 6
    for r in range(3):
        assert set(picks[r]) <= set(got[r][1]) and len(picks[r]) == 2
