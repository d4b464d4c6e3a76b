"""Final bandwidths of the c5 workload after band doubling (bench.py's setup):
writes gpurun_out/c5_bands.npz with read lengths and bandwidths."""
import os
import sys
from types import SimpleNamespace

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "rifraf.jl_amd"))
import bench  # noqa: E402
from rifraf_amd.engine import Engine  # noqa: E402
from rifraf_amd.model import smart_forward_moves  # noqa: E402

_, nreads, length, err, bw, _ = bench.CONFIGS["c5"]
t, reads = bench.make_read_shard(nreads, length, err, bw, 2024, 0, nreads)
eng = Engine(0)
eng.reserve(sum(bench.band_bytes(len(r), length, bw) + bench.band_bytes(len(r), length, 2 * bw, pad=True)
                for r in reads) + (256 << 20))
for a in range(0, nreads, 1024):
    eng.set_sequences(a, reads[a:a + 1024])
eng.set_templates(0, [t])
smart_forward_moves(SimpleNamespace(e=eng), [(k, k) for k in range(nreads)], reads, length, 0.1)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "c5_bands.npz"), n=np.array([len(r) for r in reads]),
         bw=np.array([r.bandwidth for r in reads]), m=length)
eng.close()
print("ok")
