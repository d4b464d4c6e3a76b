#!/usr/bin/env python
"""bench.py -- RIFRAF hot path on MI355X.

One step = one pass of the hot path over this rank's batch of clusters:
  1. realign: forward (A) + backward (B) banded DP of every read against its
     cluster consensus (forward_moves!/backward!, realign! model.jl:679-714);
  2. score: every STAGE_SCORE proposal of every cluster (all_proposals,
     model.jl:401-456: 8m+4 per cluster) summed over the cluster's reads in
     batch order (score_proposal(state) model.jl:385-399, as estimate_probs
     does, model.jl:737-791).  Totals stay in HBM.

Workload (default "c4"): BASELINE.json configs[3] -- clusters of 50 reads x
1.5 kb (sample_sequences(50, 1500), error_rate 0.01, seq_errors
ErrorModel(1,5,5), default RifrafParams scores, bandwidth 9), sharded by
cluster across ranks with a fixed per-rank share (weak scaling): 1,250
clusters per GPU, so 8 GPUs = the config's 10,000 clusters.  No collective
on the data path (clusters are independent); the only cross-rank traffic is
the timing barrier / max.  "c2" / "c3" select configs[1] / configs[2]
(single cluster; replicas under --gpus N).

Ranks: `bench.py --gpus N` (N > 1) with no RANK / WORLD_SIZE in the
environment starts N child ranks itself, one per GPU, before anything touches
the GPU; under an external launcher (torch.distributed.run) it checks that
WORLD_SIZE == N.  Each rank needs a GPU of its own (`--shared-gpu` rehearses
several ranks on one GPU); `n_gpus` counts distinct devices (PCI ids), `ranks`
the processes.

Prints ONE JSON line on rank 0 (contract in the task statement); metric
value = GCUPS = in-band DP cells (forward + backward) per second over the
whole step; proposals/s and (proposal x read) pairs/s are reported beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rifraf.jl_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_VEC_TFLOPS = 78.6         # half the 157.3 TF FP32 vector spec

CONFIGS = {
    # name: (clusters per rank, reads per cluster, template length, error rate, bandwidth, label)
    "c4": (1250, 50, 1500, 0.01, 9, "configs[3]: clusters x 50 reads x 1.5 kb, per-GPU share of 10k"),
    "c2": (1, 100, 1000, 0.01, 9, "configs[1]: 1 kb template, 100 reads, ~1% error"),
    "c3": (1, 1000, 2601, 0.01, 9, "configs[2]: 2.6 kb amplicon, 1000 reads (read DP + scoring)"),
    "c5": (1, 5000, 10000, 0.03, 9, "configs[4]: 10 kb template, 5000 reads, high indel rate (band "
                                    "doubling), reads sharded over ranks + all-gather of proposal totals"),
}


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nranks: int, argv) -> int:
    """`bench.py --gpus N` without an external launcher: start N child ranks,
    one per GPU (LOCAL_RANK = RANK = 0..N-1, WORLD_SIZE = N, rendezvous on
    127.0.0.1), wait for all of them and return the worst exit code.  Runs
    before anything in this process touches HIP or torch.cuda (the children
    are fresh interpreters, not an exec of this one).  A rank that fails ends
    the others, so a dead peer cannot leave the rest waiting in a collective."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for o in live:
                    o.terminate()
        if live:
            time.sleep(0.2)
    return rc


def device_identity(torch, gpu):
    """Physical identity of this rank's device (PCI domain:bus:device), so
    that n_gpus counts distinct GPUs, not ranks."""
    if torch is not None and torch.cuda.is_available():
        p = torch.cuda.get_device_properties(gpu)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    return f"cpu-rank-device-{gpu}"   # --dry-run on a host without GPUs: the assignment itself


def distinct_devices(dist, ident: str):
    """(distinct physical devices, most ranks on one device) over all ranks."""
    if dist is None:
        return 1, 1
    ids = [None] * dist.get_world_size()
    dist.all_gather_object(ids, ident)
    return len(set(ids)), max(ids.count(i) for i in set(ids))


def band_cells(n: int, m: int, bw: int) -> int:
    """Number of in-band cells: sum_j |row_range(j)| (bandedarrays.jl:133-137)."""
    nrows, ncols = n + 1, m + 1
    h_off, v_off = max(ncols - nrows, 0), max(nrows - ncols, 0)
    j = np.arange(1, ncols + 1)
    start = np.maximum(1, j - h_off - bw)
    stop = np.minimum(j + v_off + bw, nrows)
    return int(np.sum(stop - start + 1))


def band_bytes(n: int, m: int, bw: int, pad: bool = False) -> int:
    """Device bytes of one kappa-major band (rifraf_hip.hip band_K x band_stride, 256-B aligned)."""
    from rifraf_amd.bandedarrays import band_stride
    H = 2 * bw + abs(n - m) + 1
    P = band_stride(H, pad_h=1 if pad else 0)
    return ((H + 2 * m) * P * 8 + 255) // 256 * 256


def make_workload(nclusters, nreads, length, error_rate, bw, seed):
    """Synthetic clusters from the restated sample module (sample.jl)."""
    from rifraf_amd import ErrorModel, RifrafSequence, Scores
    from rifraf_amd.sample import MAX_PROB, MIN_PROB, random_seq, sample_from_template
    rng = np.random.default_rng(seed)
    scores = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0))   # RifrafParams default
    seq_errors = ErrorModel(1, 5, 5)
    alpha = 0.1
    beta = alpha * (error_rate - MAX_PROB) / (MIN_PROB - error_rate)
    clusters = []
    for _ in range(nclusters):
        t = random_seq(length, rng)
        t_p = rng.beta(alpha, beta, size=length) * (MAX_PROB - MIN_PROB) + MIN_PROB
        reads = []
        for _ in range(nreads):
            s, _, ph, _, _ = sample_from_template(t, t_p, seq_errors, 1.5, 3.0, 1.0, rng)
            reads.append(RifrafSequence(s, ph, bw, scores))
        clusters.append((t, reads))
    return clusters


def read_shard_raw(length, error_rate, seed, lo, hi):
    """One cluster's template and raw reads lo..hi-1 (bases, Phred scores)
    from the restated sample module; read k has its own seeded stream, so
    every rank simulates only its reads."""
    from rifraf_amd import ErrorModel
    from rifraf_amd.sample import MAX_PROB, MIN_PROB, random_seq, sample_from_template
    rng = np.random.default_rng(seed)
    alpha = 0.1
    beta = alpha * (error_rate - MAX_PROB) / (MIN_PROB - error_rate)
    t = random_seq(length, rng)
    t_p = rng.beta(alpha, beta, size=length) * (MAX_PROB - MIN_PROB) + MIN_PROB
    seqs, phreds = [], []
    for k in range(lo, hi):
        s, _, ph, _, _ = sample_from_template(t, t_p, ErrorModel(1, 5, 5), 1.5, 3.0, 1.0,
                                              np.random.default_rng([seed, k]))
        seqs.append(s)
        phreds.append(ph)
    return t, seqs, phreds


def make_read_shard(nreads, length, error_rate, bw, seed, lo, hi):
    """One cluster (template + reads lo..hi-1) as RifrafSequences."""
    from rifraf_amd import ErrorModel, RifrafSequence, Scores
    scores = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0))
    t, seqs, phreds = read_shard_raw(length, error_rate, seed, lo, hi)
    return t, [RifrafSequence(s, ph, bw, scores) for s, ph in zip(seqs, phreds)]


def cpu_threads():
    """Host cores usable by this process (affinity mask, capped by a cgroup
    CPU quota when one is set): the CPU baseline runs on all of them."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline_reads(t, reads, budget_s=12.0):
    """Oracle CPU baseline for one read-sharded cluster: realign + all-proposal
    scoring over chunks of this rank's reads (final bandwidths) until the
    budget, on every usable host core.  Also returns the first chunk's totals
    (the bench's parity check)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    threads = cpu_threads()
    chunk = max(16, threads)
    cells = done = 0
    first = None
    t0 = time.perf_counter()
    for a in range(0, len(reads), chunk):
        tot, c = oracle.cpu_pass(t, reads[a:a + chunk], nthreads=threads)
        if first is None:
            first = (a, a + len(reads[a:a + chunk]), tot)
        cells += c
        done += len(reads[a:a + chunk])
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": cells / dt / 1e9, "unit": "GCUPS", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{done} reads x {len(t)} bp (final bandwidths), realign + all-proposal scoring "
                      f"in chunks of {chunk} reads, {dt:.1f} s, OpenMP {threads} threads (all usable cores)"}, first


def cpu_baseline(clusters, budget_s=12.0):
    """The oracle (C restatement of the reference) on every usable host core,
    over a bounded sample of the same workload (whole clusters until the
    budget), plus the same pass on one thread.  Returns the per-cluster
    totals of the all-core sample for the bench's parity check."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    threads = cpu_threads()
    cells = props = done = 0
    totals = []
    t0 = time.perf_counter()
    for t, reads in clusters:
        tot, c = oracle.cpu_pass(t, reads, nthreads=threads)
        totals.append(tot)
        cells += c
        props += 8 * len(t) + 4
        done += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    # the same pass on one thread (1 thread and all cores), shorter budget
    c1 = d1 = 0
    t1 = time.perf_counter()
    for t, reads in clusters:
        _, c = oracle.cpu_pass(t, reads, nthreads=1)
        c1 += c
        d1 += 1
        if time.perf_counter() - t1 >= budget_s / 4:
            break
    dt1 = time.perf_counter() - t1
    return {"value": cells / dt / 1e9, "unit": "GCUPS", "cores": threads, "kind": "port",
            "proposals_per_s": props / dt, "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{done} cluster(s) x {len(clusters[0][1])} reads x {len(clusters[0][0])} bp, "
                      f"realign + all-proposal scoring, {dt:.1f} s, OpenMP {threads} threads (all usable cores)",
            "single_thread": {"value": c1 / dt1 / 1e9, "unit": "GCUPS", "cores": 1,
                              "sample": f"{d1} cluster(s), {dt1:.1f} s"}}, totals


def parity_check(got, expected, templates):
    """Bench self-check: GPU dense totals vs the oracle's for the clusters the
    CPU baseline ran (every STAGE_SCORE proposal slot, bit for bit)."""
    bad = checked = 0
    for g, e, t in zip(got, expected, templates):
        mask = np.ones(e.shape, bool)
        mask[0, :5] = False                                  # p = 0: no sub / del
        mask[np.arange(1, len(t) + 1), np.asarray(t, np.int64)] = False   # the consensus base
        a, b = np.asarray(g)[mask], e[mask]
        bad += int(np.sum(~((a == b) | (np.isnan(a) & np.isnan(b)))))
        checked += int(mask.sum())
    return {"clusters": len(expected), "proposal_totals": checked, "mismatches": bad, "bitexact": bad == 0}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def shard_seed(seed: int, rank: int) -> int:
    """Each rank simulates its own clusters (weak scaling, no shared input)."""
    return seed * 1000003 + rank


def aggregate(elapsed: float, units, device="cpu"):
    """Whole-job figures: the slowest rank's time and the units of all ranks.
    The only cross-rank traffic of the benchmark (clusters are independent)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(u) for u in units], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [float(x) for x in c.tolist()]


def spread(x: float, device="cpu"):
    """(min, max) of a per-rank figure over all ranks (load balance of the
    static cluster shards; one all-gather, outside any timed region)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    v = [float(o.item()) for o in out]
    return min(v), max(v)


def pmc_traffic(config, size, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/pmc_<config>.json, scripts/pmc_summary.py), when it was taken at
    the same size (clusters per rank for c4, reads per rank for c5); else None."""
    pmc_file = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    key = "reads" if config == "c5" else "clusters"
    try:
        pm = json.load(open(pmc_file))
        if pm.get(key) == size and kernel in pm.get("kernels", {}):
            return pm["kernels"][kernel]["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    return None


def pmc_fp64(config, cells=None, dp_ms=None, world=1):
    """FP64 VALU evidence from a PAST rocprof counter run, not this run
    (profiles/pmc_fp64.json, scripts/pmc_fp64_summary.py over
    scripts/pmc_r03.sh's passes): SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 wave
    instructions.  c4: the DP's measured FP64 lane-ops per in-band cell,
    scaled by this run's cells and DP time; both: each DP kernel's longest
    launch in the profiled run against the FP64 peak.  Only quoted for the
    profiled shape: one rank (the profile was taken at world size 1)."""
    if world != 1:
        return None
    try:
        pm = json.load(open(os.path.join(REPO, "profiles", "pmc_fp64.json")))
        ent = pm[config]
    except (OSError, ValueError, KeyError):
        return None
    peak = pm["fp64_lane_ops_peak_per_s"]
    out = {"source": "profiles/pmc_fp64.json (a past rocprofv3 --pmc run at one rank, not this run)",
           "profiled": pm.get("source"),
           "per_kernel_frac_of_fp64_peak": {k: v["longest_launch"]["frac_of_fp64_peak"]
                                            for k, v in ent["kernels"].items() if k.startswith("k_dpr")}}
    if "dp" in ent and cells and dp_ms:
        r = ent["dp"]["f64_lane_ops_per_cell"]
        out.update({"f64_lane_ops_per_cell": r, "achieved_tops": r * cells / (dp_ms * 1e-3) / 1e12,
                    "frac": r * cells / (dp_ms * 1e-3) / peak})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks = GPUs (default: WORLD_SIZE under an external launcher, else 1)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--clusters", type=int, default=None, help="clusters per rank (override)")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="c4 only: skip the secondary c5 (10 kb, band doubling) workload")
    ap.add_argument("--no-c2", action="store_true",
                    help="c4 only: skip the c2 field (configs[1]: whole runs of 100 reads x 1 kb, seeds 1..5)")
    ap.add_argument("--no-c3", action="store_true",
                    help="c4 only: skip the c3 field (configs[2] run with the reference's codon moves)")
    ap.add_argument("--no-sharded-rifraf", action="store_true",
                    help="c5 at N > 1: skip the read-sharded whole-rifraf() rehearsal field")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--e2e-clusters", type=int, default=512,
                    help="c4 only: whole rifraf() runs per rank for the e2e field (0: skip)")
    ap.add_argument("--e2e-pin-cores", type=int, default=2,
                    help="c4 only: also time the e2e run with the rank pinned to this many host cores (0: skip)")
    ap.add_argument("--e2e-engines", type=int, default=2,
                    help="c4 only: contexts (HIP streams) per GPU for the e2e field, one host thread each "
                         "(round 5: two engines, so one wave's host setup runs beside the other's kernels; "
                         "profiles/r05aj_e2e_engines.jsonl)")
    ap.add_argument("--e2e-wave", type=int, default=256,
                    help="c4 only: clusters per wave of the e2e field (waves from a shared queue per engine)")
    ap.add_argument("--e2e-init-exclusive", type=int, default=0,
                    help="c4 only: 1 = at most one engine in its native stage machine at a time (a two-stage "
                         "pipeline of waves: one engine's kernels, the others' host work)")
    ap.add_argument("--e2e-pin-exclusive", type=int, default=-1,
                    help="c4 only: init_exclusive for the pinned e2e run (-1: as the unpinned run)")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process group for N > 1 (auto: nccl = RCCL when GPUs are visible)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal only: allow several ranks on one GPU (n_gpus then counts distinct devices)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch, rendezvous, workload and device assignment only (no engine): checks the "
                         "multi-rank plumbing on a host without GPUs")
    args = ap.parse_args()
    launched = "RANK" in os.environ or "WORLD_SIZE" in os.environ
    if args.gpus is None:
        # under torch.distributed.run without --gpus: the launcher's world size
        args.gpus = int(os.environ.get("WORLD_SIZE", "1")) if launched else 1

    if args.gpus > 1 and not launched:
        # no external launcher: one child process per GPU, started before this
        # process touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    rank, world, local = dist_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    dist = torch = coll = None
    gpu = local
    if world > 1:
        # torch only for the process group (RCCL over xGMI / gloo): the engine
        # calls are synchronous on their own HIP stream
        import torch
        import torch.distributed as dist
        backend = args.backend
        if backend == "auto":
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        ndev = torch.cuda.device_count()
        if ndev and local >= ndev and not args.shared_gpu:
            raise SystemExit(f"bench.py: rank {rank} (local {local}) has no GPU of its own: {ndev} visible "
                             f"for {world} ranks (--shared-gpu rehearses several ranks per GPU)")
        gpu = local % ndev if ndev else local      # --shared-gpu rehearsals: several ranks per GPU
        if backend == "nccl":
            torch.cuda.set_device(gpu)
        # gloo prints its connection report on stdout, which carries only the
        # JSON line: send fd 1 to stderr while the group connects
        sys.stdout.flush()
        fd1 = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend)
        finally:
            sys.stdout.flush()
            os.dup2(fd1, 1)
            os.close(fd1)
        coll = torch.device("cuda", gpu) if backend == "nccl" else torch.device("cpu")
    n_dev, per_dev = distinct_devices(dist, device_identity(torch, gpu)) if world > 1 else (1, 1)
    args.processes_per_gpu = per_dev

    if args.dry_run:
        result = run_dry(args, rank, world, gpu, dist, coll, n_dev)
    elif args.config == "c5":
        result = run_read_sharded(args, rank, world, gpu, dist, torch, coll)
    else:
        result = run_clusters(args, rank, world, gpu, dist, torch, coll)
        if args.config == "c4" and args.e2e_clusters > 0:
            result["e2e"] = run_e2e(args, rank, world, gpu, dist, coll)
        # the rank-0 legs below report a failure in their own field (the
        # other ranks are already on their way to the next collective)
        if args.config == "c4" and not args.no_c2 and rank == 0:
            # configs[1] beside the headline line: whole runs of the 1 kb
            # cluster, latency mode, checked against the oracle's runs
            result["c2"] = rank0_leg(run_c2, args, gpu)
        if args.config == "c4" and not args.no_c3 and rank == 0:
            # configs[2] beside the headline line: the reference-informed path
            # (FRAME, codon moves) end to end, rank 0 only (one cluster)
            result["c3"] = rank0_leg(run_c3, args, gpu)
        if args.config == "c4" and not args.no_secondary:
            # configs[4] beside the headline line: driver-measured 10 kb reads
            # with band doubling, read-sharded over the same ranks
            result["secondary"] = run_read_sharded(args, rank, world, gpu, dist, torch, coll)
    # n_gpus: distinct physical devices the ranks ran on (a rehearsal with
    # several ranks per GPU reports fewer GPUs than ranks)
    result["n_gpus"] = n_dev
    result["ranks"] = world
    if isinstance(result.get("secondary"), dict):
        result["secondary"]["n_gpus"] = n_dev
        result["secondary"]["ranks"] = world
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_dry(args, rank, world, gpu, dist, coll, n_dev):
    """--dry-run: every step of a run except the engine -- launch, rendezvous,
    device assignment, this rank's workload and its cell count, the whole-job
    reduction -- so the multi-rank plumbing is testable on a host without
    GPUs.  Reports no throughput."""
    nclu, nreads, length, err, bw, label = CONFIGS[args.config]
    if args.clusters is not None:
        nclu = args.clusters
    if args.config == "c5":
        from rifraf_amd.sharded import shard_bounds
        lo, hi = shard_bounds(nreads, world)[rank:rank + 2]
        t, reads = make_read_shard(nreads, length, err, bw, args.seed, lo, hi)
        clusters = [(t, reads)]
    else:
        clusters = make_workload(nclu, nreads, length, err, bw, seed=shard_seed(args.seed, rank))
    cells = sum(2 * band_cells(len(r), len(t), r.bandwidth) for t, rs in clusters for r in rs)
    units = [float(cells), float(sum(len(rs) for _, rs in clusters))]
    elapsed = 0.0
    cspread = None
    if dist is not None:
        elapsed, units = aggregate(elapsed, units, coll)
        cspread = spread(float(cells), coll)
    hand_out = None
    if args.config == "c4" and args.e2e_clusters > 0:
        hand_out = dry_hand_out(args, rank, world, dist)
    return {"metric": "banded fwd/bwd GCUPS + candidate proposals scored/sec, 1/2/4/8 MI355X",
            "value": None, "unit": "GCUPS", "dry_run": True, "steps": args.steps, "warmup": args.warmup,
            "e2e_hand_out": hand_out,
            "higher_is_better": True, "scaling": "strong" if args.config == "c5" else "weak",
            "config": {"workload": args.config, "description": label},
            "cells_per_step_all_ranks": int(units[0]), "reads_all_ranks": int(units[1]),
            "rank_cells_min_max": None if cspread is None else [int(x) for x in cspread]}


E2E_SHAPE = (50, 1500, 0.01)     # SURVEY.md §8(d) config 4's cluster shape


def e2e_cluster(seed, k):
    """Global e2e cluster k: sample_sequences(50, 1500; error_rate=0.01)
    seeded by (seed, 77, 0, k) -> (template, rifraf keyword dict)."""
    from rifraf_amd.sample import sample_sequences
    nr, ln, er = E2E_SHAPE
    _, t, _, reads, _, phreds, _, _ = sample_sequences(nr, ln, error_rate=er,
                                                       rng=np.random.default_rng([seed, 77, 0, k]))
    return t, dict(dnaseqs=reads, phreds=phreds)


class E2EClusters:
    """The e2e field's one global list of clusters, n per rank.  At N > 1
    each rank simulates its own block (untimed) and writes it to a staging
    directory on the host (/dev/shm), and every rank maps all blocks, so
    whichever rank the queue hands cluster k to reads it back (as each of the
    reference's pmap workers reads its file, scripts/rifraf.jl:190):
    `get(k)` -> rifraf keyword dict with the reads and Phred scores as
    PackedReads (one buffer + offsets, as FASTQ ingest hands them over),
    `template(k)`."""

    FIELDS = ("bases", "phreds", "lens", "tpl", "tlens")

    def __init__(self, seed, n_per_rank, rank, world, dist=None):
        self.n = n_per_rank * world
        self.dir = None
        lo = rank * n_per_rank
        blk = [e2e_cluster(seed, k) for k in range(lo, lo + n_per_rank)]
        if world == 1:
            from rifraf_amd.types import PackedReads
            self._local = [(t, dict(dnaseqs=PackedReads.from_list(kw["dnaseqs"], np.uint8),
                                    phreds=PackedReads.from_list(kw["phreds"], np.int8))) for t, kw in blk]
            return
        import tempfile
        base = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
        self.dir = os.path.join(base, "rifraf_bench_e2e_%s_%s" % (os.environ.get("MASTER_ADDR", "x"),
                                                                  os.environ.get("MASTER_PORT", "0")))
        os.makedirs(self.dir, exist_ok=True)
        arrs = {"bases": np.concatenate([r for _, kw in blk for r in kw["dnaseqs"]]).astype(np.uint8),
                "phreds": np.concatenate([p for _, kw in blk for p in kw["phreds"]]).astype(np.int8),
                "lens": np.array([len(kw["dnaseqs"]) for _, kw in blk] +
                                 [len(r) for _, kw in blk for r in kw["dnaseqs"]], np.int64),
                "tpl": np.concatenate([t for t, _ in blk]).astype(np.uint8),
                "tlens": np.array([len(t) for t, _ in blk], np.int64)}
        for f, a in arrs.items():
            tmp = os.path.join(self.dir, f"b{rank}_{f}.tmp.npy")
            np.save(tmp, a)
            os.replace(tmp, os.path.join(self.dir, f"b{rank}_{f}.npy"))
        dist.barrier()
        self.blocks = []
        for r in range(world):
            m = {f: np.load(os.path.join(self.dir, f"b{r}_{f}.npy"), mmap_mode="r") for f in self.FIELDS}
            nc = len(m["tlens"])
            counts = np.asarray(m["lens"][:nc])
            rl = np.asarray(m["lens"][nc:])
            roff = np.concatenate([[0], np.cumsum(rl)])
            coff = np.concatenate([[0], np.cumsum(counts)])
            toff = np.concatenate([[0], np.cumsum(m["tlens"])])
            self.blocks.append((m, roff, coff, toff))
        self.per = n_per_rank

    def get(self, k):
        if self.dir is None:
            return self._local[k][1]
        from rifraf_amd.types import PackedReads
        m, roff, coff, toff = self.blocks[k // self.per]
        c = k % self.per
        a, b = roff[coff[c]], roff[coff[c + 1]]
        off = roff[coff[c]:coff[c + 1] + 1] - a
        return dict(dnaseqs=PackedReads(np.array(m["bases"][a:b]), off),
                    phreds=PackedReads(np.array(m["phreds"][a:b]), off))

    def template(self, k):
        if self.dir is None:
            return self._local[k][0]
        m, _, _, toff = self.blocks[k // self.per]
        c = k % self.per
        return np.array(m["tpl"][toff[c]:toff[c + 1]])

    def close(self, rank, dist=None):
        """Drop the maps; after a barrier rank 0 removes the staging files."""
        if self.dir is None:
            return
        self.blocks = None
        if dist is not None:
            dist.barrier()
        if rank == 0:
            import shutil
            shutil.rmtree(self.dir, ignore_errors=True)


def _digest(kw):
    import hashlib
    h = hashlib.sha256()
    for r, p in zip(kw["dnaseqs"], kw["phreds"]):
        h.update(np.asarray(r, np.uint8).tobytes())
        h.update(np.asarray(p, np.int8).tobytes())
        h.update(b"|")
    return h.hexdigest()


def dry_hand_out(args, rank, world, dist, n_max=8):
    """--dry-run: the e2e field's cluster hand-out without the engine -- the
    staged global list (at most n_max clusters per rank), one pass of the
    process group's ClusterQueue, and on rank 0 the check that every cluster
    was taken exactly once and read back identical to what one process
    simulates for it."""
    from rifraf_amd.batch import ClusterQueue
    data = E2EClusters(args.seed, min(args.e2e_clusters, n_max), rank, world, dist)
    q = ClusterQueue.for_process_group(data.n, max(1, min(args.e2e_wave, 2)))
    got = {}
    while True:
        r = q.take()
        if r is None:
            break
        for k in r:
            got[k] = _digest(data.get(k))
    if dist is not None:
        dist.barrier()
        allg = [None] * world
        dist.all_gather_object(allg, got)
    else:
        allg = [got]
    data.close(rank, dist)
    if rank != 0:
        return None
    seen, once = {}, True
    for g in allg:
        for k, d in g.items():
            once = once and k not in seen
            seen[k] = d
    ident = sorted(seen) == list(range(data.n)) and all(seen[k] == _digest(e2e_cluster(args.seed, k)[1])
                                                         for k in range(data.n))
    return {"clusters": data.n, "exactly_once": bool(once and sorted(seen) == list(range(data.n))),
            "identical_to_one_process": bool(ident), "per_rank": [len(g) for g in allg]}


def run_e2e(args, rank, world, gpu, dist, coll):
    """Whole rifraf() runs on the c4 cluster shape (SURVEY.md §8(d) config 4:
    every read in each batch, quality scores on) through rifraf_batch_queue:
    one global list of clusters (--e2e-clusters per rank), handed out in
    waves to whichever engine of whichever rank asks next (ClusterQueue on
    the process group's store: the reference's pmap over files,
    scripts/rifraf.jl:190), each wave through the native lockstep stage
    machine (rf_rifraf_batch).  clusters_per_s = all clusters / the slowest
    rank's wall time (host setup from reads included, read simulation
    excluded).  Two of this rank's clusters are re-run through the Python
    stage machine (the reference restatement) and must match exactly."""
    from rifraf_amd.batch import ClusterQueue, rifraf_batch, rifraf_batch_queue
    from rifraf_amd.engine import Engine
    from rifraf_amd.model import RifrafParams
    data = E2EClusters(args.seed, args.e2e_clusters, rank, world, dist)
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
    ne = max(1, args.e2e_engines)
    engs = [Engine(gpu) for _ in range(ne)]
    warm = [data.get(k) for k in range(min(4, data.n))]
    for e in engs:
        rifraf_batch(warm, params=params, engine=e)        # warm-up (kernels, pinned staging)
    wave = max(1, args.e2e_wave)

    def queued(excl):
        """One full pass over the global list; (wall s, results, stats)."""
        q = ClusterQueue.for_process_group(data.n, wave)
        st = {}
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        res = rifraf_batch_queue(data.get, q, params=params, engines=engs, init_exclusive=excl, stats=st)
        return time.perf_counter() - t0, res, st

    excl = bool(args.e2e_init_exclusive)
    # cold: the first full-size run also sizes each context's band arena; the
    # timed run is the steady state of a stream of waves (the arena is reused,
    # rf_release_bands) -- every stage of every cluster is recomputed
    cold, _, _ = queued(excl)
    # steady state: five rounds of (unpinned run, run with this rank held to
    # 2 host cores -- its share at 8 ranks on the GPU box's 16; every thread
    # of the process pinned in place, no relaunch; the library's worker pools
    # follow the mask), medians of each (one run of either varies by ~10 %
    # between rounds on one box, profiles/r05l_e2e_pinned.jsonl, r05al_bench.json).
    # Every rank decides to pin (or not) the same way, so all ranks make the
    # same number of queue passes and barriers.
    allowed = sorted(os.sched_getaffinity(0))
    k = args.e2e_pin_cores
    can_pin = float(k > 0 and len(allowed) > k)
    if dist is not None:
        import torch
        f = torch.tensor([can_pin], dtype=torch.float64, device=coll)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        can_pin = float(f.item())
    pin = idle_cpus(allowed, k, dist) if can_pin else None
    pin_excl = bool(args.e2e_pin_exclusive) if ne > 1 and args.e2e_pin_exclusive >= 0 else excl
    runs, pin_runs, stats, same_pin, pin_sets = [], [], [], True, []
    res = None
    for p_ in range(5 if pin else 3):
        s_, r_, st = queued(excl)
        runs.append(s_)
        stats.append(st)
        res = res or r_
        if pin:
            # the idlest cpus at this pass (the shared host's load moves
            # between passes: r08h's first three pinned passes ran 0.43 - 0.46 s
            # on cpus picked once, the last two 0.19 - 0.23 s)
            if p_ > 0:
                pin = idle_cpus(allowed, k, dist)
            pin_sets.append([int(c) for c in pin])
            saved = pin_threads(pin)
            try:
                s_, res_pin, _ = queued(pin_excl)
                pin_runs.append(s_)
            finally:
                unpin_threads(saved)
            # the queue hands clusters out afresh: compare the ones this rank ran both times
            same_pin = same_pin and all(np.array_equal(res[i].consensus, res_pin[i].consensus)
                                        for i in set(res) & set(res_pin))
    elapsed = float(np.median(runs))
    mine = sorted(res)
    chk = mine[:2]
    ref = rifraf_batch([data.get(i) for i in chk], params=params, engine=engs[0], native=False)
    same = all(np.array_equal(res[i].consensus, b.consensus) and res[i].state.score == b.state.score and
               qv_close(res[i], b) for i, b in zip(chk, ref))
    for e in engs:
        e.close()
    ok = sum(int(np.array_equal(res[i].consensus, data.template(i))) for i in mine)
    iters = sum(sum(res[i].state.stage_iterations) for i in mine)
    med = stats[int(np.argsort(runs)[len(runs) // 2])]
    tot = [float(len(mine)), float(ok), float(iters), 1.0 if same else 0.0]
    pin_s = float(np.median(pin_runs)) if pin_runs else 0.0
    per_rank = None
    if dist is not None:
        cold, _ = aggregate(cold, [0.0], coll)
        pin_s, _ = aggregate(pin_s, [0.0], coll)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"clusters": med.get("clusters"), "waves": med.get("waves"),
                                          "busy_s": med.get("busy_s"), "barrier_wait_s": med.get("barrier_wait_s")})
        elapsed, tot = aggregate(elapsed, tot, coll)
    data.close(rank, dist)
    n_all = float(data.n)
    best, pin_best = float(min(runs)), (float(min(pin_runs)) if pin_runs else 0.0)
    if dist is not None:
        best, _ = aggregate(best, [0.0], coll)
        pin_best, _ = aggregate(pin_best, [0.0], coll)
    return {"metric": "whole rifraf() runs per second (c4 cluster shape)", "clusters_per_s": n_all / elapsed,
            "clusters_per_s_per_gpu": n_all / elapsed / max(world, 1), "ranks": world,
            "clusters_per_s_best": n_all / best,
            "clusters": int(n_all), "clusters_run_once": int(tot[0]) == int(n_all), "seconds": elapsed,
            "cold_clusters_per_s": n_all / cold,
            "timing": "steady state: the median of five full passes over the clusters after the first ('cold', "
                      "which also allocates the band arena), alternating with the pinned passes; host setup from "
                      "reads included, read simulation excluded",
            "processes_per_gpu": getattr(args, "processes_per_gpu", 1),
            "engines_per_gpu": ne, "wave": wave, "init_exclusive": excl,
            "hand_out": "ClusterQueue (rifraf_amd/batch.py): one global list of clusters, waves handed to "
                        "whichever engine of whichever rank asks next through the process group's store "
                        "(scripts/rifraf.jl:190's pmap); per_rank: clusters / waves taken, seconds running them "
                        "and waiting at the closing barrier, in the median unpinned pass",
            "per_rank": per_rank if per_rank is not None else [{
                "clusters": med.get("clusters"), "waves": med.get("waves"), "busy_s": med.get("busy_s"),
                "barrier_wait_s": med.get("barrier_wait_s")}],
            "driver": "rf_rifraf_batch (native lockstep INIT) + batched quality pass per wave; "
                      "engines_per_gpu contexts (own HIP stream, own host thread) per process, at most one of "
                      "them in its native stage machine at a time when init_exclusive",
            "params": "batch = all 50 reads, do_score (QVs), no reference",
            "consensus_equals_template": int(tot[1]), "stage_iterations": int(tot[2]),
            "consensus_misses_explained": "profiles/r04_e2e_misses.json: every miss converges at a consensus "
                                          "no single edit improves and that scores above the template",
            "same_as_python_stage_machine": tot[3] == world,
            "same_as_python_stage_machine_note": "consensus and score bit-identical; QVs (device quality pass) "
                                                 "within 1e-12 relative + 1e-15 absolute",
            "runs_s": runs, "pinned_runs_s": pin_runs,
            "pinned": None if not pin else {
                "cores": len(pin), "cpus": [int(c) for c in pin], "cpu_nodes": [cpu_node(c) for c in pin],
                "home_node": home_node(), "clusters_per_s": n_all / pin_s,
                "ratio_to_unpinned": elapsed / pin_s,
                "cpus_per_pass": pin_sets,
                "clusters_per_s_best": n_all / pin_best if pin_best > 0 else None,
                "ratio_best": best / pin_best if pin_best > 0 else None,
                "best_note": "the fastest of the five passes of each kind (medians above): the shared host's "
                             "other load reaches either kind of pass",
                "init_exclusive": pin_excl,
                "host_cpus_unpinned": len(os.sched_getaffinity(0)), "same_consensus": bool(same_pin),
                "note": "the same steady-state pass with every thread of the rank pinned to this many cores "
                        "(a rank's share of the box's 16 at 8 ranks): the idlest of its allowed cpus, disjoint "
                        "across ranks (bench.idle_cpus)"}}


def qv_close(a, b, rtol=1e-12, atol=1e-15):
    """QVs of a native run (device quality pass: 10^x by the GPU's exp10)
    against the Python stage machine's host evaluation: every error_probs /
    aln_error_probs array within rtol (+ atol); consensus and scores are
    compared exactly by the callers."""
    if a.error_probs is None or b.error_probs is None:
        return a.error_probs is None and b.error_probs is None
    pairs = [(getattr(a.error_probs, f), getattr(b.error_probs, f)) for f in ("sub", "dele", "ins")]
    pairs.append((a.aln_error_probs, b.aln_error_probs))
    return all(np.shape(x) == np.shape(y) and np.allclose(x, y, rtol=rtol, atol=atol) for x, y in pairs)


def cpu_busy(cpus, dt=0.3):
    """Busy fraction of each cpu over `dt` seconds (/proc/stat)."""
    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    name, *v = line.split()
                    v = [int(x) for x in v]
                    out[int(name[3:])] = (sum(v), v[3] + (v[4] if len(v) > 4 else 0))
        return out
    a = snap()
    time.sleep(dt)
    b = snap()
    busy = {}
    for c in cpus:
        if c in a and c in b and b[c][0] > a[c][0]:
            busy[c] = 1.0 - (b[c][1] - a[c][1]) / (b[c][0] - a[c][0])
        else:
            busy[c] = 1.0
    return busy


def cpu_node(c):
    """NUMA node of cpu c (sysfs), or -1."""
    try:
        for name in os.listdir(f"/sys/devices/system/cpu/cpu{c}"):
            if name.startswith("node") and name[4:].isdigit():
                return int(name[4:])
    except OSError:
        pass
    return -1


def home_node():
    """NUMA node holding most of this process's resident pages
    (/proc/self/numa_maps), else that of the cpu its main thread last ran
    on, or -1."""
    pages = {}
    try:
        with open("/proc/self/numa_maps") as f:
            for line in f:
                for tok in line.split():
                    if tok[0] == "N" and "=" in tok and tok[1:tok.index("=")].isdigit():
                        n = int(tok[1:tok.index("=")])
                        pages[n] = pages.get(n, 0) + int(tok[tok.index("=") + 1:])
    except (OSError, ValueError):
        pages = {}
    if pages:
        return max(pages, key=pages.get)
    try:
        with open("/proc/self/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return cpu_node(int(fields[36]))   # field 39: processor
    except (OSError, ValueError, IndexError):
        return -1


def idle_cpus(allowed, k, dist=None):
    """The k idlest of the rank's allowed cpus on its home NUMA node (the GPU
    box's host is shared: its first cpus carry other work, r06v's pinned
    passes on cpus 0-1 ran 0.17 - 0.32 s; and cpus of another node left the
    first pinned passes of r06w / r07f at 0.25 - 0.41 s against 0.18 - 0.20 s
    for the later ones, its host buffers being remote until they migrate);
    with a process group, ranks take disjoint sets in rank order from the
    gathered measurements."""
    try:
        busy = cpu_busy(allowed)
    except OSError:
        busy = {c: 0.0 for c in allowed}
    home = home_node()
    order = sorted(allowed, key=lambda c: (home >= 0 and cpu_node(c) != home, busy[c], c))
    if dist is None:
        return order[:k]
    lists = [None] * dist.get_world_size()
    dist.all_gather_object(lists, order)
    taken, mine = set(), None
    for r, lst in enumerate(lists):
        pick = [c for c in lst if c not in taken][:k] or lst[:k]
        taken.update(pick)
        if r == dist.get_rank():
            mine = pick
    return mine


def pin_threads(cpus):
    """Pin every thread of this process to `cpus` (in place, no exec);
    returns the previous masks for unpin_threads."""
    saved = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            saved[int(tid)] = os.sched_getaffinity(int(tid))
            os.sched_setaffinity(int(tid), set(cpus))
        except OSError:
            pass
    return saved


def unpin_threads(saved):
    for tid, mask in saved.items():
        try:
            os.sched_setaffinity(tid, mask)
        except OSError:
            pass


def _sync_fn(torch):
    if torch is not None and torch.cuda.is_available():
        return lambda: torch.cuda.synchronize()
    return lambda: None


def run_clusters(args, rank, world, gpu, dist, torch, coll):
    """configs[3] (default): this rank's clusters, realign + dense scoring."""
    nclu, nreads, length, err, bw, label = CONFIGS[args.config]
    if args.clusters is not None:
        nclu = args.clusters
    t_gen = time.perf_counter()
    clusters = make_workload(nclu, nreads, length, err, bw, seed=shard_seed(args.seed, rank))
    gen_s = time.perf_counter() - t_gen

    from rifraf_amd.engine import RF_BWD, RF_FWD, Engine
    eng = Engine(gpu)
    reads = [r for _, rs in clusters for r in rs]
    tpl_of = np.concatenate([[c] * len(rs) for c, (_, rs) in enumerate(clusters)]).astype(np.int32)
    nr = len(reads)
    cells = 0
    band_bytes = 0
    for c, (t, rs) in enumerate(clusters):
        for r in rs:
            cells += 2 * band_cells(len(r), len(t), r.bandwidth)
            band_bytes += 2 * 8 * (2 * r.bandwidth + abs(len(r) - len(t)) + 1) * (len(t) + 1)
    eng.reserve(int(band_bytes * 1.05) + (64 << 20))
    for a in range(0, nr, 4096):
        eng.set_sequences(a, reads[a:a + 4096])
    eng.set_templates(0, [t for t, _ in clusters])
    slots = np.arange(nr, dtype=np.int32)
    bws = np.array([r.bandwidth for r in reads], np.int32)
    groups, at = [], 0
    for _, rs in clusters:
        groups.append(np.arange(at, at + len(rs), dtype=np.int32))
        at += len(rs)
    nprops = sum(8 * len(t) + 4 for t, _ in clusters)
    npairs = sum((8 * len(t) + 4) * len(rs) for t, rs in clusters)
    # algorithmic bytes: DP = 8 B stored per in-band cell;
    # scoring = A + B in-band cells read once + 33 B of tables per read row +
    # 72 B of totals per consensus position
    dp_bytes = 8 * cells
    score_bytes = 8 * cells + sum(33 * (len(r) + 1) for r in reads) + sum(72 * (len(t) + 1) for t, _ in clusters)

    from rifraf_amd.engine import pack_groups
    packed = pack_groups(groups)   # the caller's slot lists, packed once

    dp_flags = RF_FWD | RF_BWD

    def step():
        eng.realign(slots, slots, tpl_of, bws, dp_flags)
        dp_ms, _, _ = eng.last_timing()
        eng.score_dense(packed, to_host=False)
        _, sc_ms, _ = eng.last_timing()
        return dp_ms, sc_ms

    for _ in range(args.warmup):
        step()
    sync = _sync_fn(torch)
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    dps, scs = [], []
    for _ in range(args.steps):
        a, b = step()
        dps.append(a)
        scs.append(b)
    sync()
    work_s = time.perf_counter() - t0   # this rank's own time, before waiting for the others
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-step units of this rank; the timed region ran args.steps steps
    tot_cells, tot_props, tot_pairs = cells * args.steps, nprops * args.steps, npairs * args.steps
    balance = None
    if dist is not None:
        elapsed, (tot_cells, tot_props, tot_pairs) = aggregate(elapsed, [tot_cells, tot_props, tot_pairs], coll)
        lo, hi = spread(work_s, coll)
        balance = {"rank_work_s_min": lo, "rank_work_s_max": hi, "imbalance": hi / lo - 1.0 if lo > 0 else None,
                   "note": "each rank's own timed-region time before the closing barrier: the spread of the "
                           "static per-rank cluster shards (equal shapes, seeded per rank)"}

    ms_step = elapsed / args.steps * 1e3
    dp_ms = float(np.mean(dps))
    sc_ms = float(np.mean(scs))
    dp_gbs = dp_bytes / (dp_ms * 1e-3) / 1e9
    sc_gbs = score_bytes / (sc_ms * 1e-3) / 1e9
    dominant = "k_score" if sc_ms >= dp_ms else "k_dp"
    ach, byt, ms = (sc_gbs, score_bytes, sc_ms) if dominant == "k_score" else (dp_gbs, dp_bytes, dp_ms)
    traffic = pmc_traffic(args.config, nclu, dominant)
    result = {
        "metric": "banded fwd/bwd GCUPS + candidate proposals scored/sec, 1/2/4/8 MI355X",
        "value": tot_cells / elapsed / 1e9,
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (restated sample.jl simulator, seeded)",
        "config": {"workload": args.config, "description": label, "clusters_per_gpu": nclu,
                   "reads_per_cluster": nreads, "template_len": length, "error_rate": err,
                   "bandwidth": bw, "parallelism": f"clusters sharded over {world} rank(s)",
                   "step": "A/B fill + scoring"},
        "rank_balance": balance,
        "proposals_per_s": tot_props / elapsed,
        "pairs_per_s": tot_pairs / elapsed,
        "dp_ms": dp_ms,
        "score_ms": sc_ms,
        "dp_gcups_kernel": cells / (dp_ms * 1e-3) / 1e9,
        # north_star: the DP fill against the FP64 VALU peak (5 non-FMA FP64
        # ops per cell: 3 adds + 2 max; peak = 78.6 TF FMA / 2 = 39.3 T ops/s)
        "dp_valu": {"ops_per_cell": 5, "achieved_tops": 5 * cells / (dp_ms * 1e-3) / 1e12,
                    "peak_tops": FP64_VEC_TFLOPS / 2,
                    "frac": 5 * cells / (dp_ms * 1e-3) / 1e12 / (FP64_VEC_TFLOPS / 2),
                    "counters_from_profile": pmc_fp64(args.config, cells, dp_ms, world)},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": ach, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes": byt, "launch_ms": ms},
        "roofline_other": {"k_dp": {"achieved": dp_gbs, "frac": dp_gbs / HBM_PEAK_GBS,
                                    "bytes": dp_bytes, "ms": dp_ms},
                           "k_score": {"achieved": sc_gbs, "frac": sc_gbs / HBM_PEAK_GBS,
                                       "bytes": score_bytes, "ms": sc_ms}},
        "setup_s": gen_s,
    }
    if rank == 0:
        # the timed launch's totals (same plan: downloaded, not recomputed)
        dense = eng.score_dense(groups, rows=[len(t) + 1 for t, _ in clusters])
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"], ref = cpu_baseline(clusters, budget_s=args.cpu_budget)
        else:
            result["cpu_baseline"] = None
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle  # test infrastructure: the parity check only
            ref = [oracle.cpu_pass(t, rs, nthreads=cpu_threads())[0] for t, rs in clusters[:2]]
        result["parity"] = parity_check(dense[:len(ref)], ref, [t for t, _ in clusters[:len(ref)]])
    eng.close()
    result["stream_read_gbs"], result["stream_write_gbs"] = probe_bandwidth(gpu, band_bytes)
    return result


def probe_bandwidth(gpu, nbytes):
    """Attainable HBM bandwidth on this box (diagnostics, scripts/probe_bw.hip,
    outside the engine): stream reads over a buffer the size of the step's
    band arena, and the DP fill's store pattern (nontemporal 16-B stores,
    16-lane streams of 2.75 KB chunks).  The c4 DP time varies by ~12 %
    between boxes (8.3 / 9.3 ms) at equal read rates.  (None, None) when the
    probe library is not built."""
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    try:
        from probe_bw import Probe
        p = Probe(gpu, nbytes)
    except Exception:  # noqa: BLE001 -- diagnostic only
        return None, None
    try:
        rd = p.read_gbs(3)
        p.write_gbs(4, 2816, 16384)
        return rd, p.write_gbs(4, 2816, 16384)
    except Exception:  # noqa: BLE001 -- diagnostic only
        return None, None
    finally:
        p.close()


C3_SEED = 3   # the c3 parity tests' cluster (tests/test_workloads.py::test_c3_*)
GOLDEN_RUNS = os.path.join(REPO, "tests", "golden", "runs.npz")   # scripts/make_golden.py runs()
C2_SEEDS = (1, 2, 3, 4, 5)
C2_VARIANTS = {"default": dict(seed=1),
               "throughput": dict(seed=1, batch_size=0, batch_fixed=False, do_score=True)}


def rank0_leg(fn, *a):
    """A rank-0-only field of the bench line: its result, or the error it
    raised (type, message, traceback tail) so that the line still prints."""
    import traceback
    try:
        return fn(*a)
    except Exception as e:  # noqa: BLE001 -- reported in the field, not hidden
        return {"error": f"{type(e).__name__}: {e}", "traceback": traceback.format_exc()[-2000:]}


def golden_run(name, z=None):
    """The CPU oracle engine's whole rifraf() run `name` ("c2_<seed>_<variant>",
    "c3_throughput") from tests/golden/runs.npz (committed data, made by
    scripts/make_golden.py; bench checks its runs against it)."""
    z = np.load(GOLDEN_RUNS) if z is None else z
    pre = name + "_"
    return {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}


def run_matches(res, rec, qv_rtol=1e-12, atol=1e-15):
    """A rifraf() result against a golden_run record: consensus, every
    stage's consensuses, score bits, stage iterations, penalty increases and
    convergence exactly; QVs within qv_rtol (the native driver's device
    quality pass uses the GPU's exp10; 0 = bit-exact)."""
    st = res.consensus_stages
    lens = [len(c) for x in st for c in x]
    ok = (np.array_equal(np.asarray(res.consensus, np.uint8), rec["consensus"]) and
          res.state.score == float(rec["score"]) and
          list(res.state.stage_iterations) == rec["iters"].tolist() and
          int(res.state.n_ref_indel_mults) == int(rec["mults"]) and
          bool(res.state.converged) == bool(rec["converged"]) and
          [len(x) for x in st] == rec["stage_counts"].tolist() and lens == rec["stage_lens"].tolist() and
          np.array_equal(np.concatenate([np.asarray(c, np.uint8) for x in st for c in x] or
                                        [np.zeros(0, np.uint8)]), rec["stages"]))
    if not ok:
        return False
    if "batch" in rec and [int(i) for i in res.state.batch_seqs] != rec["batch"].tolist():
        return False     # a random batch (resampling.py): the final draw
    if "sub" not in rec:
        return res.error_probs is None
    if res.error_probs is None:
        return False
    pairs = [(res.error_probs.sub, rec["sub"]), (res.error_probs.dele, rec["dele"]),
             (res.error_probs.ins, rec["ins"]), (res.aln_error_probs, rec["aln"])]
    if qv_rtol == 0:
        return all(np.array_equal(a, b) for a, b in pairs)
    return all(np.shape(a) == np.shape(b) and np.allclose(a, b, rtol=qv_rtol, atol=atol) for a, b in pairs)


def c2_cluster(seed):
    """configs[1]: sample_sequences(100, 1000; error_rate=0.01), no reference
    (sample.jl:277-298)."""
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(seed)
    _, template, _, reads, _, phreds, _, _ = sample_sequences(100, 1000, error_rate=0.01, rng=rng)
    return template, reads, phreds


def c3_cluster(seed=C3_SEED):
    """configs[2]: sample_sequences(1000, 2601; error_rate=0.01,
    ref_error_rate=0.1, ref_errors=ErrorModel(10,0,0,1,1)) with a one-base
    frameshift in the reference, so that FRAME runs (codon scoring of the
    reference, seeded indel proposals, penalty increases)."""
    from rifraf_amd import ErrorModel
    from rifraf_amd.sample import sample_sequences
    rng = np.random.default_rng(seed)
    ref, template, _, reads, _, phreds, _, _ = sample_sequences(
        1000, 2601, error_rate=0.01, ref_error_rate=0.1, ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
    ref = np.concatenate([ref[:1300], ref[1301:2000], [2], ref[2000:]]).astype(np.uint8)
    return template, reads, phreds, ref


class _StageTimer:
    """Engine proxy for one rifraf() run: kernel milliseconds of every engine
    call (HIP events on the engine stream), DP cells and proposals scored,
    attributed to the stage / iteration the stage machine is in
    (rifraf_amd.model.ITERATION_HOOK)."""

    def __init__(self, eng):
        self.e = eng
        self.lens, self.tlen = {}, {}
        self.key = ("INIT", 0)
        self.rec = {}

    def __getattr__(self, name):
        return getattr(self.e, name)

    def hook(self, it, stage):
        self.key = (stage.name, it)

    def _add(self, **kw):
        r = self.rec.setdefault(self.key, {})
        for k, v in kw.items():
            r[k] = r.get(k, 0) + v

    def set_sequences(self, first, seqs):
        for k, s in enumerate(seqs):
            self.lens[first + k] = len(s)
        return self.e.set_sequences(first, seqs)

    def set_templates(self, first, tpls):
        for k, t in enumerate(tpls):
            self.tlen[first + k] = len(t)
        return self.e.set_templates(first, tpls)

    def realign(self, slots, seqs, tpls, bws, flags):
        out = self.e.realign(slots, seqs, tpls, bws, flags)
        n = len(np.atleast_1d(slots))
        sq = np.broadcast_to(seqs, (n,))
        tp = np.broadcast_to(tpls, (n,))
        bw = np.broadcast_to(bws, (n,))
        from rifraf_amd.engine import RF_BWD, RF_FWD
        fl = np.broadcast_to(np.asarray(flags), (n,))   # one value or one per job
        cells = sum((int(bool(f & RF_FWD)) + int(bool(f & RF_BWD))) * band_cells(self.lens[int(a)], self.tlen[int(b)], int(c))
                    for a, b, c, f in zip(sq, tp, bw, fl.tolist()))
        self._add(dp_ms=self.e.last_timing()[0], dp_cells=cells, realign_calls=1)
        return out

    def backtrace(self, slots, want_moves=True):
        out = self.e.backtrace(slots, want_moves)
        self._add(walk_ms=self.e.last_backtrace_ms())
        return out

    def alignment_proposals(self, groups, do_indels):
        out = self.e.alignment_proposals(groups, do_indels)
        self._add(walk_ms=self.e.last_backtrace_ms())
        return out

    def score(self, groups, per_seq=False):
        out = self.e.score(groups, per_seq)
        _, sc, ga = self.e.last_timing()
        props = sum(len(p[0]) if isinstance(p, tuple) else len(p) for _, _, p in groups)
        ref = sum(1 for _, r, _ in groups if r >= 0)
        self._add(score_ms=sc + ga, codon_ms=self.e.last_codon_ms(), proposals=props,
                  codon_proposals=props if ref else 0, score_calls=1)
        return out

    def score_dense(self, groups, to_host=True, rows=None):
        out = self.e.score_dense(groups, to_host, rows)
        self._add(score_ms=self.e.last_timing()[1], proposals=len(groups) * (8 * self.tlen.get(0, 0) + 4),
                  score_calls=1)
        return out


C3_DEFAULT = dict(seed=1, do_score=True)   # scripts/make_golden.py C3_DEFAULT


def run_c3(args, gpu):
    """configs[2] end to end (rank 0): one rifraf() run of the 1000-read
    2.6 kb cluster with its frameshifted reference at the throughput settings
    (every read in every batch, QV pass on) -- INIT, FRAME with the
    reference's codon moves (k_codon), REFINE, SCORE.  Reports the native
    driver's wall time per run (rf_rifraf_batch_ref) and, from a run of the
    Python stage machine on the same engine, every stage's and every FRAME
    iteration's kernel time (DP fill, proposal scoring, the codon scorer,
    walks) and work; both runs must give the same result."""
    import rifraf_amd.model as model
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.engine import Engine
    template, reads, phreds, ref = c3_cluster()
    params = model.RifrafParams(seed=1, batch_size=0, batch_fixed=False, do_score=True)
    kw = dict(dnaseqs=reads, phreds=phreds, reference=ref)
    eng = Engine(gpu)          # the product default options (latency-mode DP for small calls)
    dp_lat = eng.get_option("dp_lat")
    try:
        rifraf_batch([kw], params=params, engine=eng, native=True)        # warm-up (kernels, arena)
        # the median of five runs (one run varies by up to 1.5x on a box,
        # profiles/r06j_c3_repeat.out)
        runs = []
        for _ in range(5):
            t0 = time.perf_counter()
            nat = rifraf_batch([kw], params=params, engine=eng, native=True)[0]
            runs.append(time.perf_counter() - t0)
        native_s = float(np.median(runs))
        # the default batches: fixed 5 in INIT / FRAME, REFINE's random 20
        # (drawn in the native driver, resampling.py's RNG), QVs on
        dparams = model.RifrafParams(**C3_DEFAULT)
        rifraf_batch([kw], params=dparams, engine=eng, native=True)
        druns = []
        for _ in range(5):
            t0 = time.perf_counter()
            dnat = rifraf_batch([kw], params=dparams, engine=eng, native=True)[0]
            druns.append(time.perf_counter() - t0)
        timer = _StageTimer(eng)
        model.ITERATION_HOOK = timer.hook
        try:
            t0 = time.perf_counter()
            py = model.rifraf(reads, phreds, reference=ref, params=params, engine=timer)
            py_s = time.perf_counter() - t0
        finally:
            model.ITERATION_HOOK = None
    finally:
        eng.close()
    same = (np.array_equal(nat.consensus, py.consensus) and nat.state.score == py.state.score and
            nat.state.stage_iterations == py.state.stage_iterations and qv_close(nat, py))
    gold = golden_run("c3_throughput")
    stages, frame, tot = stage_split(timer)
    return {"metric": "one rifraf() run of configs[2] (reference-informed, codon frame correction)",
            "workload": "c3", "reads": len(reads), "template_len": len(template), "reference_len": len(ref),
            "params": "batch = all 1000 reads, do_score (QVs), seed 1; reference with a one-base frameshift",
            "native_seconds_per_run": native_s, "runs_per_s": 1.0 / native_s, "native_seconds": runs,
            "python_stage_machine_seconds": py_s, "same_as_python_stage_machine": bool(same),
            "dp_lat": dp_lat,
            "same_as_oracle": {"native": bool(run_matches(nat, gold)),
                               "python_stage_machine": bool(run_matches(py, gold, qv_rtol=0)),
                               "fixture": "tests/golden/runs.npz c3_throughput (scripts/make_golden.py: the CPU "
                                          "oracle engine's run of this cluster); consensus, every stage's "
                                          "consensuses, score bits, iterations, penalty increases exact; QVs "
                                          "bit-exact (Python stage machine) / within 1e-12 (native driver's "
                                          "device quality pass)"},
            "consensus_equals_template": bool(np.array_equal(nat.consensus, template)),
            "default": {"params": "RifrafParams(%s)" % ", ".join(f"{k}={v}" for k, v in C3_DEFAULT.items()),
                        "batches": "fixed 5 lowest-error reads in INIT / FRAME, then REFINE's random batches of "
                                   "20 drawn by the native driver (rifraf_amd/resampling.py's RNG and draw)",
                        "native_seconds_per_run": float(np.median(druns)), "native_seconds": druns,
                        "stage_iterations": list(dnat.state.stage_iterations),
                        "same_as_oracle": bool(run_matches(dnat, golden_run("c3_default"))),
                        "fixture": "tests/golden/runs.npz c3_default (the CPU oracle engine's rifraf(); the final "
                                   "random batch included)"},
            "stage_iterations": list(nat.state.stage_iterations),
            "penalty_increases": int(nat.state.n_ref_indel_mults),
            "kernel_ms_total": tot, "codon_share_of_kernel_ms": tot["codon_ms"] / max(
                tot["dp_ms"] + tot["score_ms"] + tot["walk_ms"], 1e-9),
            "per_stage": stages, "frame_iterations": frame,
            "timing": "kernel ms: HIP events on the engine stream, summed per stage from the Python stage "
                      "machine's run (score_ms includes codon_ms); native_seconds_per_run: median wall time of "
                      "five runs of the library's stage machine, host work included"}


def stage_split(timer):
    """Per-stage and per-FRAME-iteration kernel time and work of a
    _StageTimer'd run, and their totals."""
    stages = {}
    for (st, it), r in timer.rec.items():
        a = stages.setdefault(st, {"iterations": 0})
        a["iterations"] += 1 if it > 0 else 0
        for k, v in r.items():
            a[k] = a.get(k, 0) + v
    for a in stages.values():
        if a.get("dp_ms"):
            a["dp_gcups"] = a["dp_cells"] / (a["dp_ms"] * 1e-3) / 1e9
    frame = [dict(iteration=it, **r) for (st, it), r in sorted(timer.rec.items(), key=lambda x: x[0][1])
             if st == "FRAME"]
    tot = {k: sum(r.get(k, 0) for r in timer.rec.values())
           for k in ("dp_ms", "score_ms", "codon_ms", "walk_ms", "dp_cells", "proposals", "codon_proposals")}
    return stages, frame, tot


def run_c2(args, gpu):
    """configs[1] end to end (rank 0): rifraf() of sample_sequences(100, 1000;
    error_rate=0.01), no reference, seeds 1..5, with the default params and
    the throughput settings (every read in every batch, QV pass on).  Each
    run goes through the library's stage machine (rf_rifraf_batch, one
    cluster) on an engine with the product default options -- its realigns
    have at most 100 lean tasks, so the DP runs in latency mode (k_dpx) --
    and is checked against the CPU oracle engine's run of the same cluster
    (tests/golden/runs.npz).  Reports the median wall time per run per
    variant, and per-stage kernel ms of seed 1 from the Python stage machine
    on the same engine (which must give the same result)."""
    import rifraf_amd.model as model
    from rifraf_amd.batch import rifraf_batch
    from rifraf_amd.engine import Engine
    z = np.load(GOLDEN_RUNS)
    clusters = {seed: c2_cluster(seed) for seed in C2_SEEDS}
    eng = Engine(gpu)
    dp_lat = eng.get_option("dp_lat")
    out = {"metric": "one rifraf() run of configs[1] (100 reads x 1 kb, no reference)", "workload": "c2",
           "seeds": list(C2_SEEDS), "dp_lat": dp_lat}
    try:
        for var, kw in C2_VARIANTS.items():
            params = model.RifrafParams(**kw)
            t, reads, phreds = clusters[C2_SEEDS[0]]
            rifraf_batch([dict(dnaseqs=reads, phreds=phreds)], params=params, engine=eng, native=True)  # warm-up
            secs, match, tmpl = [], [], []
            for seed in C2_SEEDS:
                t, reads, phreds = clusters[seed]
                t0 = time.perf_counter()
                res = rifraf_batch([dict(dnaseqs=reads, phreds=phreds)], params=params, engine=eng,
                                   native=True)[0]
                secs.append(time.perf_counter() - t0)
                match.append(bool(run_matches(res, golden_run(f"c2_{seed}_{var}", z))))
                tmpl.append(bool(np.array_equal(res.consensus, t)))
            t, reads, phreds = clusters[C2_SEEDS[0]]
            timer = _StageTimer(eng)
            model.ITERATION_HOOK = timer.hook
            try:
                t0 = time.perf_counter()
                py = model.rifraf(reads, phreds, params=params, engine=timer)
                py_s = time.perf_counter() - t0
            finally:
                model.ITERATION_HOOK = None
            stages, _, tot = stage_split(timer)
            out[var] = {"params": "RifrafParams(%s)" % ", ".join(f"{k}={v}" for k, v in kw.items()),
                        "native_seconds_per_run": float(np.median(secs)), "runs_per_s": 1.0 / float(np.median(secs)),
                        "native_seconds": secs, "same_as_oracle": match, "all_same_as_oracle": all(match),
                        "consensus_equals_template": tmpl,
                        "python_stage_machine_seconds_seed1": py_s,
                        "python_stage_machine_same_as_oracle_seed1": bool(
                            run_matches(py, golden_run(f"c2_{C2_SEEDS[0]}_{var}", z), qv_rtol=0)),
                        "kernel_ms_total_seed1": tot, "per_stage_seed1": stages}
    finally:
        eng.close()
    out["timing"] = ("native_seconds_per_run: median wall time of the library's stage machine over the seeds "
                     "(host work included, after one warm-up run); kernel ms: HIP events on the engine stream, "
                     "summed per stage from the Python stage machine's run of seed 1")
    out["oracle_fixture"] = ("tests/golden/runs.npz (scripts/make_golden.py runs(): the CPU oracle engine); "
                             "consensus, stage consensuses, score bits, iterations exact, QVs within 1e-12 "
                             "(device quality pass)")
    return out


class _TimedEngine:
    """Engine proxy for smart_forward_moves!: accumulates the kernel time of
    every band-doubling realign / backtrace and the DP cells it executes."""

    def __init__(self, eng, reads, m):
        self.e, self.reads, self.m = eng, reads, m
        self.dp_ms = self.bt_ms = 0.0
        self.cells = self.rounds = 0

    def realign(self, slots, seqs, tpls, bws, flags):
        out = self.e.realign(slots, seqs, tpls, bws, flags)
        self.dp_ms += self.e.last_timing()[0]
        self.cells += sum(band_cells(len(self.reads[int(k)]), self.m, int(b)) for k, b in zip(seqs, bws))
        self.rounds += 1
        return out

    def backtrace(self, slots, want_moves=True):
        out = self.e.backtrace(slots, want_moves)
        self.bt_ms += self.e.last_backtrace_ms()
        return out


def run_sharded_rifraf(args, rank, world, local, dist, nreads=256):
    """Whole rifraf() runs through ShardedEngine (rifraf_amd.sharded) on the
    first `nreads` reads of the c5 cluster (10 kb, 3 % error; every read in
    every batch): every rank runs the same stage machine, owns every W-th
    read's bands, and exchanges per-read results through fixed-shape tensor
    collectives.  Reports the collectives' time per stage-machine iteration
    and checks the result against one unsharded engine on rank 0."""
    from rifraf_amd.engine import Engine
    from rifraf_amd.model import RifrafParams, rifraf
    from rifraf_amd.sharded import ShardedEngine
    _, _, length, err, bw, _ = CONFIGS["c5"]
    t, seqs, phreds = read_shard_raw(length, err, args.seed, 0, nreads)
    params = RifrafParams(batch_size=0, batch_fixed=False)
    se = ShardedEngine(Engine(local), len(seqs))
    try:
        dist.barrier()
        t0 = time.perf_counter()
        res = rifraf(seqs, phreds, params=params, engine=se)
        wall = time.perf_counter() - t0
        xs, nx = se.exchange_s, se.exchanges
    finally:
        se.close()
    iters = int(sum(res.state.stage_iterations))
    same = None
    if rank == 0:
        e = Engine(local)
        try:
            one = rifraf(seqs, phreds, params=params, engine=e)
        finally:
            e.close()
        same = bool(np.array_equal(one.consensus, res.consensus) and one.state.score == res.state.score
                    and one.state.stage_iterations == res.state.stage_iterations)
    return {"reads": len(seqs), "template_len": len(t), "ranks": world, "iterations": iters,
            "seconds_rank0": wall, "exchange_ms_rank0": 1e3 * xs, "collectives_rank0": nx,
            "exchange_ms_per_iteration": 1e3 * xs / max(iters, 1),
            "collectives_per_iteration": nx / max(iters, 1),
            "same_as_one_gpu": same,
            "note": "ShardedEngine: realign / backtrace / alignment_proposals / score exchange fixed-shape "
                    "tensors (one all-gather or all-reduce per call, error flag in the payload); "
                    "every read in every batch, no QV pass"}


def run_read_sharded(args, rank, world, local, dist, torch, coll=None):
    """configs[4]: ONE cluster whose reads are split over the ranks.  Setup
    (untimed, reported): each rank simulates and uploads its block of reads
    and runs the band-doubling first realign (smart_forward_moves!,
    model.jl:643-672), timed separately with its DP cells.  Step: fwd+bwd DP
    of the rank's reads at their final bandwidths, the rank's partial fold of
    every STAGE_SCORE proposal (rf_score_dense_dev), then the exchange:
    all-gather of the partial totals over RCCL + rank-order sum
    (rifraf_amd.sharded).  Total work is fixed: strong scaling."""
    from types import SimpleNamespace
    from rifraf_amd.engine import RF_BWD, RF_FWD, Engine
    from rifraf_amd.model import smart_forward_moves
    from rifraf_amd.sharded import allgather_fold, shard_bounds
    _, nreads, length, err, bw, label = CONFIGS["c5"]
    lo, hi = shard_bounds(nreads, world)[rank:rank + 2]
    t_gen = time.perf_counter()
    t, reads = make_read_shard(nreads, length, err, bw, args.seed, lo, hi)
    gen_s = time.perf_counter() - t_gen
    nloc = len(reads)
    # band doubling on a first context sized for one forward band per read at
    # bw and 2*bw; the timed context is then sized exactly for A + B at the
    # final bandwidths (an arena that grows by compaction needs old + new)
    eng = Engine(local)
    eng.reserve(sum(band_bytes(len(r), length, bw) + band_bytes(len(r), length, 2 * bw, pad=True) for r in reads)
                + (256 << 20))
    for a in range(0, nloc, 1024):
        eng.set_sequences(a, reads[a:a + 1024])
    eng.set_templates(0, [t])
    timed = _TimedEngine(eng, reads, length)
    t_dbl = time.perf_counter()
    smart_forward_moves(SimpleNamespace(e=timed), [(k, k) for k in range(nloc)], reads, length, 0.1)
    dbl_s = time.perf_counter() - t_dbl
    # alignment_proposals (model.jl:483-497) over the doubled forward bands:
    # the walk + proposal marking of every read, one launch
    sl_all = np.arange(nloc, dtype=np.int32)
    bws0 = np.array([r.bandwidth for r in reads], np.int32)
    eng.realign(sl_all, sl_all, 0, bws0, RF_FWD)
    eng.alignment_proposals([sl_all], True)
    aln_ms = eng.last_backtrace_ms()
    eng.close()
    eng = Engine(local)
    from rifraf_amd.bandedarrays import BAND_PAD_H
    pad = max(2 * r.bandwidth + abs(len(r) - length) + 1 for r in reads) >= BAND_PAD_H   # one realign call
    eng.reserve(sum(2 * band_bytes(len(r), length, r.bandwidth, pad) for r in reads) + (256 << 20))
    for a in range(0, nloc, 1024):
        eng.set_sequences(a, reads[a:a + 1024])
    eng.set_templates(0, [t])
    slots = np.arange(nloc, dtype=np.int32)
    bws = np.array([r.bandwidth for r in reads], np.int32)
    cells = sum(2 * band_cells(len(r), length, r.bandwidth) for r in reads)
    nprops = 8 * length + 4
    dp_bytes = 8 * cells
    score_bytes = 8 * cells + sum(33 * (len(r) + 1) for r in reads) + 72 * (length + 1)
    partial = None
    if world > 1:
        partial = torch.zeros((length + 1) * 9, dtype=torch.float64, device=coll)

    def step():
        eng.realign(slots, slots, 0, bws, RF_FWD | RF_BWD)
        dp_ms, _, _ = eng.last_timing()
        if partial is None:
            eng.score_dense([slots], to_host=False)
            _, sc_ms, _ = eng.last_timing()
            return dp_ms, sc_ms, 0.0
        if partial.is_cuda:
            eng.score_dense_dev([slots], partial.data_ptr())
        else:
            partial.copy_(torch.from_numpy(eng.score_dense([slots])[0].reshape(-1)))
        _, sc_ms, _ = eng.last_timing()
        x0 = time.perf_counter()
        allgather_fold(partial, dist)
        if partial.is_cuda:
            torch.cuda.synchronize()
        return dp_ms, sc_ms, (time.perf_counter() - x0) * 1e3

    for _ in range(args.warmup):
        step()
    sync = _sync_fn(torch)
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    rec = [step() for _ in range(args.steps)]
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    doubled = int(np.sum(bws > bw))
    units = [cells * args.steps, nloc * nprops * args.steps, doubled, nloc, timed.cells, dbl_s,
             timed.dp_ms, timed.bt_ms, aln_ms]
    if dist is not None:
        elapsed, units = aggregate(elapsed, units, coll)
    tot_cells, tot_pairs, tot_doubled, tot_reads, dbl_cells, _, _, _, _ = units
    dp_ms = float(np.mean([r[0] for r in rec]))
    sc_ms = float(np.mean([r[1] for r in rec]))
    xch_ms = float(np.mean([r[2] for r in rec]))
    dp_gbs = dp_bytes / (dp_ms * 1e-3) / 1e9
    sc_gbs = score_bytes / (sc_ms * 1e-3) / 1e9
    dominant = "k_score" if sc_ms >= dp_ms else "k_dp"
    ach, byt, ms = (sc_gbs, score_bytes, sc_ms) if dominant == "k_score" else (dp_gbs, dp_bytes, dp_ms)
    result = {
        "metric": "banded fwd/bwd GCUPS + candidate proposals scored/sec, 1/2/4/8 MI355X",
        "value": tot_cells / elapsed / 1e9,
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (restated sample.jl simulator, seeded per read)",
        "config": {"workload": "c5", "description": label, "reads": nreads, "template_len": length,
                   "error_rate": err, "bandwidth": bw, "parallelism": f"reads sharded over {world} rank(s)"},
        "proposals_per_s": nprops * args.steps / elapsed,
        "pairs_per_s": tot_pairs / elapsed,
        "dp_ms": dp_ms,
        "score_ms": sc_ms,
        "exchange_ms": xch_ms,
        "dp_gcups_kernel": cells / (dp_ms * 1e-3) / 1e9,
        # north_star: the DP fill against the FP64 VALU peak (5 non-FMA FP64
        # ops per cell: 3 adds + 2 max; peak = 78.6 TF FMA / 2 = 39.3 T ops/s)
        "dp_valu": {"ops_per_cell": 5, "achieved_tops": 5 * cells / (dp_ms * 1e-3) / 1e12,
                    "peak_tops": FP64_VEC_TFLOPS / 2,
                    "frac": 5 * cells / (dp_ms * 1e-3) / 1e12 / (FP64_VEC_TFLOPS / 2),
                    "counters_from_profile": pmc_fp64("c5", world=world)},
        # smart_forward_moves! (first realign of every read): forward fills at
        # bw, the backtrace walks that count errors, the redone fills of the
        # reads whose band doubled -- every executed cell counted (rank 0's
        # kernel times; cells summed over ranks)
        "band_doubling": {"reads_doubled": tot_doubled, "reads": tot_reads, "cells_executed": dbl_cells,
                          "rounds_rank0": timed.rounds, "dp_ms_rank0": timed.dp_ms,
                          "backtrace_ms_rank0": timed.bt_ms, "wall_s_rank0": dbl_s,
                          "gcups_kernel_rank0": (timed.cells / (timed.dp_ms * 1e-3) / 1e9) if timed.dp_ms else None},
        # alignment_proposals (model.jl:483-497): walk + mark every read's
        # proposals (one rf_alignment_proposals launch, rank 0)
        "alignment_proposals_ms_rank0": aln_ms,
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": ach, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                     "traffic": pmc_traffic("c5", len(reads), dominant),
                     "algorithmic_bytes": byt, "launch_ms": ms},
        "roofline_other": {"k_dp": {"achieved": dp_gbs, "frac": dp_gbs / HBM_PEAK_GBS, "bytes": dp_bytes,
                                    "ms": dp_ms},
                           "k_score": {"achieved": sc_gbs, "frac": sc_gbs / HBM_PEAK_GBS,
                                       "bytes": score_bytes, "ms": sc_ms}},
        "setup_s": gen_s,
    }
    if world > 1 and not args.no_sharded_rifraf:
        result["sharded_rifraf"] = run_sharded_rifraf(args, rank, world, local, dist)
    if rank == 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"], first = cpu_baseline_reads(t, reads, budget_s=args.cpu_budget)
        else:
            import oracle  # test infrastructure: the parity check only
            result["cpu_baseline"] = None
            first = (0, 16, oracle.cpu_pass(t, reads[:16], nthreads=cpu_threads())[0])
        a, b, ref = first
        got = eng.score_dense([slots[a:b]])[0]
        result["parity"] = parity_check([got], [ref], [t])
        result["parity"]["reads"] = b - a
    eng.close()
    return result


if __name__ == "__main__":
    main()
