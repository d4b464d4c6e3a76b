#!/usr/bin/env python
"""DP fill time alone (realign FWD|BWD) at the c4 shape (1,250 clusters x 50
reads x 1.5 kb, bw 9) and the c5 shape (5,000 reads x 10 kb at bw 18, the
band most reads end at), under option settings interleaved in one process:
argv = settings "name=v[+name=v...]" (e.g. dp_sides=3+dp_big=0
dp_sides=2+dp_big=1).  One JSON line per shape: per-setting median ms."""
import json, os, sys
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np
import bench
from rifraf_amd.engine import Engine, RF_BWD, RF_FWD

settings = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split("+")) for a in sys.argv[1:]]


def run(label, e, sl, seqs, tpl, bws):
    ms = {i: [] for i in range(len(settings))}
    for _ in range(3):
        for i, st in enumerate(settings):
            for k, v in st.items():
                e.set_option(k, v)
            for _ in range(4):
                e.realign(sl, seqs, tpl, bws, RF_FWD | RF_BWD)
                ms[i].append(e.last_timing()[0])
    print(json.dumps({"shape": label, "settings": sys.argv[1:],
                      "median_ms": [float(np.median([x for k, x in enumerate(ms[i]) if k % 4]))
                                    for i in range(len(settings))]}), flush=True)


# c4
clusters = bench.make_workload(1250, 50, 1500, 0.01, 9, seed=bench.shard_seed(2024, 0))
reads = [r for _, rs in clusters for r in rs]
e = Engine(0)
e.reserve(sum(2 * bench.band_bytes(len(r), 1500, 9) for r in reads) + (256 << 20))
for a in range(0, len(reads), 4096):
    e.set_sequences(a, reads[a:a + 4096])
e.set_templates(0, [t for t, _ in clusters])
sl = np.arange(len(reads), dtype=np.int32)
run("c4", e, sl, sl, np.repeat(np.arange(1250, dtype=np.int32), 50), np.full(len(reads), 9, np.int32))
e.close()
# c5 (every read at bw 18)
_, nreads, length, err, bw, _ = bench.CONFIGS["c5"]
t, reads = bench.make_read_shard(nreads, length, err, bw, 2024, 0, nreads)
e = Engine(0)
e.reserve(sum(2 * bench.band_bytes(len(r), length, 18, True) for r in reads) + (256 << 20))
for a in range(0, len(reads), 1024):
    e.set_sequences(a, reads[a:a + 1024])
e.set_templates(0, [t])
sl = np.arange(len(reads), dtype=np.int32)
run("c5", e, sl, sl, 0, np.full(len(reads), 18, np.int32))
e.close()
