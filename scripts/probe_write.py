#!/usr/bin/env python
"""Write-bandwidth probes over a band arena the size of the c4 bench's (diagnostics)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rifraf.jl_amd"))
from rifraf_amd.engine import Engine
nbytes = int(float(sys.argv[1])) if len(sys.argv) > 1 else 38 << 30
e = Engine(0)
e.reserve(nbytes + (64 << 20))
res = {"bytes": nbytes, "read_gbs": nbytes / (e.probe_stream(nbytes, 3) * 1e-3) / 1e9}
for nt in (0, 2):
    tag = "_nt" if nt else ""
    e.probe_write(1 + nt, nbytes)  # warm
    res[f"write_seq{tag}_gbs"] = nbytes / (e.probe_write(1 + nt, nbytes) * 1e-3) / 1e9
    for chunk in (256, 1664, 2816, 4096, 16384):
        for ns in (8192, 16384, 65536):
            ms = e.probe_write(2 + nt, nbytes, chunk, ns)
            res[f"write{tag}_chunk{chunk}_s{ns}_gbs"] = nbytes / (ms * 1e-3) / 1e9
print(json.dumps(res, indent=1))
e.close()
