"""ctypes wrapper of the CPU oracle (oracle/rifraf_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product path (rifraf.jl_amd/) never
imports this module.  Parity of the oracle itself is pinned by the
reference's known-answer tests (tests/test_oracle_kats.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, Structure, c_double, c_int, c_int8, c_int64, c_uint8, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "rifraf_oracle.c")
LIB = os.path.join(HERE, "liboracle.so")


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (seconds)."""
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
            os.path.getmtime(SRC), os.path.getmtime(os.path.join(HERE, "rifraf_oracle.h"))):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-fopenmp", "-std=gnu11",
                               "-o", LIB, SRC, "-lm"])
    return LIB


class OrSeq(Structure):
    _fields_ = [("n", c_int), ("seq", c_void_p), ("match", c_void_p), ("mismatch", c_void_p),
                ("ins", c_void_p), ("del_", c_void_p), ("cins", c_void_p), ("ncins", c_int),
                ("cdel", c_void_p), ("ncdel", c_int), ("bw", c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build())
        L.or_ndatarows.restype = c_int
        L.or_forward.restype = c_int
        L.or_forward.argtypes = [c_void_p, c_int, POINTER(OrSeq), c_int, c_int, c_int, c_void_p, c_void_p]
        L.or_backward.restype = c_int
        L.or_backward.argtypes = [c_void_p, c_int, POINTER(OrSeq), c_void_p]
        L.or_backtrace.restype = c_int
        L.or_backtrace.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p]
        L.or_count_errors.restype = c_int
        L.or_count_errors.argtypes = [c_void_p, c_int, c_void_p, c_void_p]
        L.or_score_proposal.restype = c_int
        L.or_score_proposal.argtypes = [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                        POINTER(OrSeq), c_void_p, POINTER(c_double)]
        L.or_score_total.restype = c_int
        L.or_score_list.restype = c_int
        L.or_score_list.argtypes = [c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int]
        L.or_pass.restype = c_int64
        L.or_pass.argtypes = [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int]
        L.or_pass_continue.restype = c_int64
        L.or_pass_continue.argtypes = [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int]
        L.or_seq_tables.restype = None
        L.or_seq_tables.argtypes = [c_void_p, c_int, c_double, c_double, c_double, c_double, c_double,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    POINTER(c_double)]
        L.or_row_range.argtypes = [c_int, c_int, c_int, c_int, POINTER(c_int), POINTER(c_int)]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


class Seq:
    """Keeps the numpy tables of a RifrafSequence alive for the C struct."""

    def __init__(self, rs, bandwidth=None):
        self.keep = [np.ascontiguousarray(rs.seq, np.uint8),
                     np.ascontiguousarray(rs.match_scores, np.float64),
                     np.ascontiguousarray(rs.mismatch_scores, np.float64),
                     np.ascontiguousarray(rs.ins_scores, np.float64),
                     np.ascontiguousarray(rs.del_scores, np.float64),
                     np.ascontiguousarray(rs.codon_ins_scores, np.float64),
                     np.ascontiguousarray(rs.codon_del_scores, np.float64)]
        s, m, mm, i, d, ci, cd = self.keep
        self.n = len(s)
        self.bw = int(bandwidth if bandwidth is not None else rs.bandwidth)
        self.st = OrSeq(self.n, _p(s), _p(m), _p(mm), _p(i), _p(d),
                        _p(ci) if len(ci) else None, len(ci), _p(cd) if len(cd) else None, len(cd),
                        self.bw)


ERRORS = {1: "new score is invalid", 2: "failed to find a move", 3: "failed to compute a valid score",
          4: "no new columns need to be recomputed.", 5: "wrong column", 6: "bandwidth must be positive"}


class OracleError(Exception):
    pass


def _chk(rc):
    if rc != 0:
        raise OracleError(ERRORS.get(rc, f"oracle error {rc}"))


def ndatarows(nrows, ncols, bw):
    return 2 * bw + abs(nrows - ncols) + 1


def forward(t, rs, doreverse=False, trim=False, skew=False, moves=False, bandwidth=None):
    """forward!/forward_moves! -> (H x ncols data F-order, moves or None)."""
    s = Seq(rs, bandwidth)
    t = np.ascontiguousarray(t, np.uint8)
    m = len(t)
    H = ndatarows(s.n + 1, m + 1, s.bw)
    A = np.zeros((m + 1, H))
    mv = np.zeros((m + 1, H), np.int8) if moves else None
    _chk(lib().or_forward(_p(t), m, ctypes.byref(s.st), int(doreverse), int(trim), int(skew), _p(A), _p(mv)))
    return A.T, (mv.T if moves else None)


def backward(t, rs, bandwidth=None):
    s = Seq(rs, bandwidth)
    t = np.ascontiguousarray(t, np.uint8)
    m = len(t)
    H = ndatarows(s.n + 1, m + 1, s.bw)
    B = np.zeros((m + 1, H))
    _chk(lib().or_backward(_p(t), m, ctypes.byref(s.st), _p(B)))
    return B.T


def backtrace(moves_data, nrows, ncols, bw):
    mv = np.ascontiguousarray(np.asarray(moves_data).T, np.int8)   # column-major buffer
    out = np.zeros(nrows + ncols, np.int8)
    k = lib().or_backtrace(_p(mv), nrows, ncols, bw, _p(out))
    if k < 0:
        raise OracleError("backtrace hit an invalid move")
    return out[:k].copy()


def count_errors(moves, t, s):
    moves = np.ascontiguousarray(moves, np.int8)
    return lib().or_count_errors(_p(moves), len(moves), _p(np.ascontiguousarray(t, np.uint8)),
                                 _p(np.ascontiguousarray(s, np.uint8)))


def score_proposal(kind, pos, base, A, B, t, rs):
    """score_proposal(p, A, B, consensus, pseq, newcols) on column-major data."""
    s = Seq(rs)
    t = np.ascontiguousarray(t, np.uint8)
    Ab = np.ascontiguousarray(np.asarray(A).T)
    Bb = np.ascontiguousarray(np.asarray(B).T)
    nc = np.zeros((4, s.n + 1))
    out = c_double()
    _chk(lib().or_score_proposal(int(kind), int(pos), int(base), _p(Ab), _p(Bb), _p(t), len(t),
                                 ctypes.byref(s.st), _p(nc), ctypes.byref(out)))
    return out.value


def score_total(prop, As, Bs, rss, t, Aref=None, Bref=None, ref=None):
    """model.jl:385-399: 0.0 + s_1 + ... + s_R (+ s_ref)."""
    kind, pos, base = prop
    total = 0.0
    for A, B, rs in zip(As, Bs, rss):
        total += score_proposal(kind, pos, base, A, B, t, rs)
    if ref is not None:
        total += score_proposal(kind, pos, base, Aref, Bref, t, ref)
    return total


def seq_tables(lp, scores):
    """rifrafsequences.jl:19-82 restated in C (for table KATs)."""
    lp = np.ascontiguousarray(lp, np.float64)
    n = len(lp)
    out = [np.zeros(n), np.zeros(n), np.zeros(n), np.zeros(n + 1), np.zeros(max(n - 2, 1)), np.zeros(n + 1)]
    ne = c_double()
    lib().or_seq_tables(_p(lp), n, scores.mismatch, scores.insertion, scores.deletion,
                        scores.codon_insertion, scores.codon_deletion, *[_p(x) for x in out],
                        ctypes.byref(ne))
    return out, ne.value


def score_list(props, As, Bs, rss, t, Aref=None, Bref=None, ref=None, per_seq=False, nthreads=4):
    """model.jl:385-399 over a proposal list (kind, pos, base arrays) with
    column-major A/B data per sequence (as forward()/backward() return).
    Returns totals (and the per-sequence matrix [k, r] if per_seq)."""
    kind, pos, base = (np.ascontiguousarray(x, np.int32) for x in props)
    P = len(kind)
    seqs = [Seq(r) for r in rss]
    keep = [np.ascontiguousarray(np.asarray(A).T) for A in As] + [np.ascontiguousarray(np.asarray(B).T) for B in Bs]
    R = len(seqs)
    aptr = (c_void_p * max(R, 1))(*[k.ctypes.data for k in keep[:R]])
    bptr = (c_void_p * max(R, 1))(*[k.ctypes.data for k in keep[R:]])
    arr = (OrSeq * max(R, 1))(*[s.st for s in seqs])
    rseq = Seq(ref) if ref is not None else None
    ra = np.ascontiguousarray(np.asarray(Aref).T) if ref is not None else None
    rb = np.ascontiguousarray(np.asarray(Bref).T) if ref is not None else None
    width = R + (1 if ref is not None else 0)
    total = np.zeros(max(P, 1))
    per = np.zeros((max(P, 1), max(width, 1))) if per_seq else None
    t = np.ascontiguousarray(t, np.uint8)
    _chk(lib().or_score_list(P, _p(kind), _p(pos), _p(base), R, ctypes.cast(aptr, c_void_p),
                             ctypes.cast(bptr, c_void_p), ctypes.cast(arr, c_void_p), _p(ra), _p(rb),
                             ctypes.cast(ctypes.pointer(rseq.st), c_void_p) if rseq is not None else None, _p(t), len(t),
                             _p(per), _p(total), int(nthreads)))
    if per_seq:
        return total[:P], per[:P, :width]
    return total[:P]


def cpu_pass(t, rss, nthreads=1, totals=None):
    """CPU baseline: realign every read + score every STAGE_SCORE proposal.
    Returns (totals[(m+1), 9], cells).  With `totals` (the running totals of
    the batch's earlier reads, updated in place) the fold continues from
    them, so a large batch can be folded chunk by chunk in batch order."""
    seqs = [Seq(r) for r in rss]
    arr = (OrSeq * len(seqs))(*[s.st for s in seqs])
    t = np.ascontiguousarray(t, np.uint8)
    fn = lib().or_pass
    if totals is None:
        totals = np.zeros((len(t) + 1, 9))
    else:
        assert totals.shape == (len(t) + 1, 9) and totals.dtype == np.float64 and totals.flags.c_contiguous
        fn = lib().or_pass_continue
    cells = fn(_p(t), len(t), len(seqs), ctypes.cast(arr, c_void_p), _p(totals), int(nthreads))
    if cells < 0:
        raise OracleError("oracle pass failed")
    return totals, int(cells)
