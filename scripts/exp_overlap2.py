"""Does the DP fill overlap with dense scoring on one MI355X?  Two engine
contexts (own HIP streams): ctx1 realigns clusters half 1, ctx2 scores
half 2 (bands realigned once), driven from two host threads (ctypes drops
the GIL), against the same work run back to back.  Diagnostic only."""
import sys, os, time, threading, json
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rifraf.jl_amd")]
import numpy as np
import bench
from rifraf_amd.engine import Engine, RF_FWD, RF_BWD

N = int(sys.argv[1]) if len(sys.argv) > 1 else 600
reps = 10
clusters = bench.make_workload(2 * N, 50, 1500, 0.01, 9, seed=7)
def setup(cl):
    e = Engine(0)
    reads = [r for _, rs in cl for r in rs]
    e.reserve(int(sum(2 * 8 * (2 * r.bandwidth + abs(len(r) - 1500) + 1) * 1501 for r in reads) * 1.05) + (64 << 20))
    for a in range(0, len(reads), 4096):
        e.set_sequences(a, reads[a:a + 4096])
    e.set_templates(0, [t for t, _ in cl])
    sl = np.arange(len(reads), dtype=np.int32)
    tpl = np.repeat(np.arange(len(cl), dtype=np.int32), 50)
    bws = np.array([r.bandwidth for r in reads], np.int32)
    groups = [np.arange(50 * c, 50 * c + 50, dtype=np.int32) for c in range(len(cl))]
    e.realign(sl, sl, tpl, bws, RF_FWD | RF_BWD)
    e.score_dense(groups, to_host=False)
    return e, sl, tpl, bws, groups
e1, sl1, tpl1, bw1, g1 = setup(clusters[:N])
e2, sl2, tpl2, bw2, g2 = setup(clusters[N:])
def dp():
    for _ in range(reps):
        e1.realign(sl1, sl1, tpl1, bw1, RF_FWD | RF_BWD)
def sc():
    for _ in range(reps):
        e2.score_dense(g2, to_host=False)
t0 = time.perf_counter(); dp(); t_dp = time.perf_counter() - t0
t0 = time.perf_counter(); sc(); t_sc = time.perf_counter() - t0
th = [threading.Thread(target=dp), threading.Thread(target=sc)]
t0 = time.perf_counter()
for t in th: t.start()
for t in th: t.join()
t_both = time.perf_counter() - t0
print(json.dumps({"clusters_each": N, "reps": reps, "dp_s": t_dp, "score_s": t_sc, "sequential_s": t_dp + t_sc,
                  "concurrent_s": t_both, "gain": (t_dp + t_sc) / t_both}))
