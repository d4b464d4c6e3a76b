#!/usr/bin/env python
"""HBM bandwidth probes (diagnostics; scripts/probe_bw.hip -> libprobe_bw.so,
built by __graft_entry__.build()).  Not part of the engine: bench.py uses it
for the stream_read_gbs / stream_write_gbs fields beside its roofline.

    python scripts/probe_bw.py [bytes]   # read + write sweep, one JSON object
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libprobe_bw.so")
SRC = os.path.join(HERE, "probe_bw.hip")


def build(hipcc="/opt/rocm/bin/hipcc"):
    import subprocess
    tmp = LIB + ".tmp"
    subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-shared", SRC,
                           "-o", tmp])
    os.replace(tmp, LIB)


class Probe:
    """A probe buffer of `nbytes` on `device` (its own allocation and stream)."""

    def __init__(self, device: int, nbytes: int):
        lib = ctypes.CDLL(LIB)
        lib.pb_open.restype = ctypes.c_void_p
        lib.pb_open.argtypes = [ctypes.c_int, ctypes.c_int64]
        lib.pb_close.argtypes = [ctypes.c_void_p]
        lib.pb_read.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
        lib.pb_write.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                 ctypes.POINTER(ctypes.c_double)]
        self.lib, self.nbytes = lib, int(nbytes) & ~15
        self.h = lib.pb_open(int(device), self.nbytes)
        if not self.h:
            raise RuntimeError(f"probe_bw: no {nbytes} B buffer on device {device}")

    def read_gbs(self, reps: int = 3) -> float:
        ms = ctypes.c_double()
        if self.lib.pb_read(self.h, int(reps), ctypes.byref(ms)) or ms.value <= 0:
            raise RuntimeError("probe_bw: read failed")
        return self.nbytes / (ms.value * 1e-3) / 1e9

    def write_gbs(self, mode: int, chunk_bytes: int = 0, nstreams: int = 0) -> float:
        ms = ctypes.c_double()
        if self.lib.pb_write(self.h, int(mode), int(chunk_bytes), int(nstreams), ctypes.byref(ms)) or ms.value <= 0:
            raise RuntimeError("probe_bw: write failed")
        return self.nbytes / (ms.value * 1e-3) / 1e9

    def close(self):
        if self.h:
            self.lib.pb_close(self.h)
            self.h = None


if __name__ == "__main__":
    nbytes = int(float(sys.argv[1])) if len(sys.argv) > 1 else 38 << 30
    p = Probe(0, nbytes)
    res = {"bytes": nbytes, "read_gbs": p.read_gbs(3)}
    for nt in (0, 2):
        tag = "_nt" if nt else ""
        p.write_gbs(1 + nt)   # warm
        res[f"write_seq{tag}_gbs"] = p.write_gbs(1 + nt)
        for chunk in (256, 1664, 2816, 4096, 16384):
            for ns in (8192, 16384, 65536):
                res[f"write{tag}_chunk{chunk}_s{ns}_gbs"] = p.write_gbs(2 + nt, chunk, ns)
    print(json.dumps(res, indent=1))
    p.close()
