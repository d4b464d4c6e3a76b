"""Read-sharded rifraf() on the HIP engine.

Two gloo ranks on the one GPU of the test box, each with its own rf_ctx,
run whole rifraf() calls through ShardedEngine; the results must equal one
unsharded HIP engine bit for bit (the proposal fold is carried from rank to
rank in the reference's order).  rf_score_dense_dev (the device-side partial
of the RCCL exchange) must equal rf_score_dense.
"""
import numpy as np
import pytest

from test_sharded import _config1, _sampled, _spawn, assert_same_run, G1

pytestmark = pytest.mark.gpu


def _hip_sharded_factory(n):
    from rifraf_amd.engine import Engine
    from rifraf_amd.sharded import ShardedEngine
    return ShardedEngine(Engine(0), n)


def _w_hip_config1(rank, world, f, refid):
    return _config1(_hip_sharded_factory, f, refid)


def _w_hip_sampled(rank, world, seed):
    return _sampled(_hip_sharded_factory, seed)


def test_sharded_hip_config1_two_ranks(engine):
    import os
    f = "input-reads-2.fastq"
    refmap = dict(line.split() for line in open(os.path.join(G1, "ref-map.tsv")) if line.strip())
    single = _config1(lambda n: engine, f, refmap[f])
    got = _spawn(_w_hip_config1, 2, f, refmap[f])
    for r in range(2):
        assert_same_run(got[r], single)


def test_sharded_hip_sampled_two_ranks(engine):
    single = _sampled(lambda n: engine, 9)
    got = _spawn(_w_hip_sampled, 2, 9)
    for r in range(2):
        assert_same_run(got[r], single)


def test_score_dense_dev_matches_host(engine):
    import torch
    from _util import make_read
    from rifraf_amd.engine import RF_BWD, RF_FWD
    from rifraf_amd.sample import random_seq
    rng = np.random.default_rng(4)
    tpls = [random_seq(120, rng), random_seq(75, rng)]
    reads = [[make_read(t, rng, 0.03, 9) for _ in range(4)] for t in tpls]
    flat = [r for rs in reads for r in rs]
    engine.set_sequences(0, flat)
    engine.set_templates(0, tpls)
    n = len(flat)
    engine.realign(np.arange(n), np.arange(n), np.repeat([0, 1], 4), [9] * n, RF_FWD | RF_BWD)
    groups = [np.arange(0, 4), np.arange(4, 8)]
    host = engine.score_dense(groups)
    buf = torch.full(((121 + 76) * 9,), 7.0, dtype=torch.float64, device="cuda:0")
    engine.score_dense_dev(groups, buf.data_ptr())
    dev = buf.cpu().numpy()
    np.testing.assert_array_equal(dev[:121 * 9].reshape(121, 9), host[0])
    np.testing.assert_array_equal(dev[121 * 9:].reshape(76, 9), host[1])


def _w_rccl_dense(rank, world):
    """One RCCL rank (backend "nccl" on cuda:0): ShardedEngine.realign (object
    all-gather over RCCL) and score_dense (rf_score_dense_dev straight into a
    CUDA tensor, all_gather_into_tensor, device rank-order sum)."""
    import torch
    import torch.distributed as dist
    from _util import make_read
    from rifraf_amd.engine import RF_BWD, RF_FWD, Engine
    from rifraf_amd.sample import random_seq
    from rifraf_amd.sharded import ShardedEngine, allgather_fold
    assert dist.get_backend() == "nccl"
    rng = np.random.default_rng(21)
    tpls = [random_seq(300, rng), random_seq(180, rng)]
    reads = [[make_read(t, rng, 0.03, 9) for _ in range(6)] for t in tpls]
    flat = [r for rs in reads for r in rs]
    n = len(flat)
    groups = [np.arange(0, 6), np.arange(6, 12)]
    plain = Engine(0)
    plain.set_sequences(0, flat)
    plain.set_templates(0, tpls)
    v0 = plain.realign(np.arange(n), np.arange(n), np.repeat([0, 1], 6), [9] * n, RF_FWD | RF_BWD)
    want = plain.score_dense(groups)
    plain.close()
    sh = ShardedEngine(Engine(0), n)
    assert sh.dev.type == "cuda"
    sh.set_sequences(0, flat)
    sh.set_templates(0, tpls)
    v1 = sh.realign(np.arange(n), np.arange(n), np.repeat([0, 1], 6), [9] * n, RF_FWD | RF_BWD)
    got = sh.score_dense(groups)
    assert sh.last_dense.is_cuda
    from _util import all_proposals_arrays
    props = all_proposals_arrays(tpls[0])
    plain2 = Engine(0)
    plain2.set_sequences(0, flat)
    plain2.set_templates(0, tpls)
    plain2.realign(np.arange(n), np.arange(n), np.repeat([0, 1], 6), [9] * n, RF_FWD | RF_BWD)
    want_list = plain2.score([(groups[0], -1, props)])[0]
    plain2.close()
    got_list = sh.score([(groups[0], -1, props)])[0]
    x = torch.arange(10, dtype=torch.float64, device="cuda:0")
    y = allgather_fold(x, dist)
    sh.close()
    return {"v0": v0, "v1": v1, "want": want, "got": got, "fold": y.cpu().numpy(),
            "want_list": want_list, "got_list": got_list}


def test_rccl_world1_dense_exchange():
    """The RCCL branch of the read-sharded exchange (sharded.py allgather_fold
    on CUDA tensors) executes and, at world size 1, equals the plain engine."""
    got = _spawn(_w_rccl_dense, 1, backend="nccl")[0]
    np.testing.assert_array_equal(got["v0"], got["v1"])
    for a, b in zip(got["want"], got["got"]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(got["fold"], np.arange(10, dtype=np.float64))
    np.testing.assert_array_equal(got["want_list"], got["got_list"])
