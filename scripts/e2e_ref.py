#!/usr/bin/env python
"""Reference-guided batches (c3-like: frameshifted references, FRAME with
codon scoring, REFINE; throughput settings, QVs on): clusters/s of the
native driver (rf_rifraf_batch_ref) against the Python stage machine on the
same engine, and whether the two agree."""
import json, os, sys, time
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "tests")]
import numpy as np
from rifraf_amd import ErrorModel
from rifraf_amd.batch import rifraf_batch
from rifraf_amd.engine import Engine
from rifraf_amd.model import RifrafParams
from rifraf_amd.sample import sample_sequences
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
nr, L = int(os.environ.get("NREADS", "50")), int(os.environ.get("LEN", "1500"))
cl = []
for k in range(n):
    rng = np.random.default_rng([11, k])
    ref, t, _, reads, _, phreds, _, _ = sample_sequences(nr, L, error_rate=0.01, ref_error_rate=0.1,
                                                         ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
    ref = np.asarray(ref, np.uint8)
    at = int(rng.integers(100, L - 300))
    ref = np.concatenate([ref[:at], ref[at + 1:at + 150], [int(rng.integers(0, 4))], ref[at + 150:]]).astype(np.uint8)
    cl.append(dict(dnaseqs=reads, phreds=phreds, reference=ref))
params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
e = Engine(0)
rifraf_batch(cl[:4], params=params, engine=e)
out = {"clusters": n, "reads": nr, "len": L}
res = {}
for native in (True, False, True):
    t0 = time.perf_counter()
    res[native] = rifraf_batch(cl, params=params, engine=e, native=native)
    out[("native" if native else "hub") + "_clusters_per_s"] = n / (time.perf_counter() - t0)
a, b = res[True], res[False]
out["same"] = all(np.array_equal(x.consensus, y.consensus) and x.state.score == y.state.score and
                  x.state.stage_iterations == y.state.stage_iterations and
                  np.array_equal(x.aln_error_probs, y.aln_error_probs) for x, y in zip(a, b))
out["frame_iters"] = int(sum(r.state.stage_iterations[1] for r in a))
out["refine_iters"] = int(sum(r.state.stage_iterations[2] for r in a))
out["penalty_increases"] = int(sum(r.state.n_ref_indel_mults for r in a))
print(json.dumps(out), flush=True)
