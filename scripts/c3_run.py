#!/usr/bin/env python
"""bench.py's c3 field alone (configs[2]: one rifraf() run of the 1000-read
2.6 kb cluster with a frameshifted reference, throughput settings), for
rocprofv3 kernel statistics of the reference-informed path."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import bench  # noqa: E402

out = bench.run_c3(None, 0)
print(json.dumps({k: v for k, v in out.items() if k != "frame_iterations"}), flush=True)
