"""RifrafSequence: a read (or reference) with its per-base FP64 score tables
(src/rifrafsequences.jl:1-108).  Tables are built on the host exactly as the
reference builds them and are uploaded bit-exact to the engine."""
from __future__ import annotations

import math

import numpy as np

from .errormodel import Scores, phred_to_log_p
from .types import DNASeq


def julia_sum(a: np.ndarray) -> float:
    """Julia 0.6 `sum(::Vector{Float64})`: sequential below 16 elements,
    otherwise pairwise with block size 1024 (base/reduce.jl mapreduce_impl)."""
    a = np.asarray(a, dtype=np.float64)
    n = a.shape[0]
    if n == 0:
        return 0.0
    if n == 1:
        return float(a[0])
    if n < 16:
        return float(np.cumsum(a)[-1])

    def impl(lo, hi):  # inclusive
        if lo + 1024 > hi:
            return float(np.cumsum(a[lo:hi + 1])[-1])
        mid = (lo + hi) >> 1
        return impl(lo, mid) + impl(mid + 1, hi)

    return impl(0, n - 1)


def julia_max(x: float, y: float) -> float:
    """Base.max for Float64 (NaN-propagating, +0 > -0)."""
    if math.isnan(x) or math.isnan(y):
        return math.nan
    if y > x or (math.copysign(1.0, y) > math.copysign(1.0, x) and y == x):
        return y
    return x


def self_objects(cls, seqs, lp, match, mism, ins, dele, est, off, bandwidth):
    """RifrafSequence objects whose tables are views of concatenated arrays
    (del: n + 1 per sequence at off[k] + k)."""
    out = []
    new = object.__new__
    empty = np.empty(0)
    offl, estl = np.asarray(off).tolist(), np.asarray(est).tolist()
    bw = int(bandwidth)
    for k, sq in enumerate(seqs):
        a, b = offl[k], offl[k + 1]
        r = new(cls)
        r.seq = sq
        r.error_log_p = lp[a:b]
        r.match_scores = match[a:b]
        r.mismatch_scores = mism[a:b]
        r.ins_scores = ins[a:b]
        r.del_scores = dele[a + k:b + k + 1]
        r.codon_ins_scores = empty
        r.codon_del_scores = empty
        r.est_n_errors = estl[k]
        r.bandwidth = bw
        r.bandwidth_fixed = False
        out.append(r)
    return out


class RifrafSequence:
    """Mirror of the mutable struct at rifrafsequences.jl:5-17."""

    __slots__ = ("seq", "est_n_errors", "error_log_p", "match_scores", "mismatch_scores",
                 "ins_scores", "del_scores", "codon_ins_scores", "codon_del_scores",
                 "bandwidth", "bandwidth_fixed")

    def __init__(self, seq=None, error_log_p=None, bandwidth: int = 1, scores: Scores | None = None):
        if seq is None:  # empty sequence, rifrafsequences.jl:97-100
            self._empty()
            return
        seq = DNASeq(seq)
        if bandwidth < 1:
            raise ValueError("bandwidth must be positive")
        lp = np.asarray(error_log_p)
        if lp.dtype.kind in "iu":  # Phred constructor, :84-88
            lp = phred_to_log_p(lp)
        lp = np.ascontiguousarray(lp, dtype=np.float64)
        if len(seq) != len(lp):
            raise ValueError("length mismatch")
        if len(seq) == 0:
            self._empty()
            return
        if lp.min() == -math.inf:
            raise ValueError("a log error probability is negative infinity")
        if lp.max() > 0.0:
            raise ValueError(f"a log error probability is > 0: {lp.max()}")
        n = len(lp)
        with np.errstate(divide="ignore"):
            self.match_scores = np.log10(1.0 - np.power(10.0, lp))          # :45
        self.mismatch_scores = lp + scores.mismatch                          # :46
        self.ins_scores = lp + scores.insertion                              # :47
        d = np.empty(n + 1)
        d[0] = lp[0] + scores.deletion                                       # :49
        d[n] = lp[n - 1] + scores.deletion                                   # :50
        if n > 1:
            d[1:n] = np.maximum(lp[:-1], lp[1:]) + scores.deletion            # :51-53
        self.del_scores = d
        self.codon_ins_scores = np.empty(0)
        self.codon_del_scores = np.empty(0)
        if scores.codon_insertion > -math.inf:                               # :57-64
            if n >= 3:
                self.codon_ins_scores = (np.maximum(np.maximum(lp[:-2], lp[1:-1]), lp[2:])
                                         + scores.codon_insertion)
            else:
                self.codon_ins_scores = np.empty(max(n - 2, 0))
        if scores.codon_deletion > -math.inf:                                # :65-72
            cd = np.empty(n + 1)
            cd[0] = lp[0] + scores.codon_deletion
            cd[n] = lp[n - 1] + scores.codon_deletion
            if n > 1:
                cd[1:n] = np.maximum(lp[:-1], lp[1:]) + scores.codon_deletion
            self.codon_del_scores = cd
        self.seq = seq
        self.error_log_p = lp
        self.est_n_errors = julia_sum(np.power(10.0, lp))                    # :74
        self.bandwidth = int(bandwidth)
        self.bandwidth_fixed = False

    def _empty(self):
        self.seq = np.zeros(0, np.uint8)
        self.est_n_errors = 0.0
        self.error_log_p = np.zeros(0)
        self.match_scores = np.zeros(0)
        self.mismatch_scores = np.zeros(0)
        self.ins_scores = np.zeros(0)
        self.del_scores = np.zeros(0)
        self.codon_ins_scores = np.zeros(0)
        self.codon_del_scores = np.zeros(0)
        self.bandwidth = 0
        self.bandwidth_fixed = False

    @classmethod
    def many(cls, seqs, error_log_ps, bandwidth: int, scores: Scores) -> list:
        """[RifrafSequence(s, lp, bandwidth, scores) for ...] with every table
        computed by one numpy call over the concatenated log error
        probabilities (see many_concat)."""
        seqs = [DNASeq(sq) for sq in seqs]
        lps = []
        for sq, lp in zip(seqs, error_log_ps):
            lp = np.asarray(lp)
            if lp.dtype.kind in "iu":
                lp = phred_to_log_p(lp)
            lp = np.asarray(lp, dtype=np.float64)
            if len(sq) != len(lp):
                raise ValueError("length mismatch")
            lps.append(lp)
        if (scores.codon_insertion > -math.inf or scores.codon_deletion > -math.inf or bandwidth < 1
                or not lps or any(len(x) == 0 for x in lps)):
            return [cls(sq, lp, bandwidth, scores) for sq, lp in zip(seqs, lps)]
        off = np.zeros(len(lps) + 1, np.int64)
        np.cumsum([len(x) for x in lps], out=off[1:])
        return cls.many_concat(seqs, np.concatenate(lps), off, bandwidth, scores)[0]

    @classmethod
    def many_concat(cls, seqs, lp, off, bandwidth: int, scores: Scores, phreds=None):
        """Sequences seqs[k] with log error probabilities lp[off[k]:off[k+1]]
        (all non-empty, no codon scores).  numpy evaluates each element of a
        ufunc the same way wherever it sits in an array (checked by
        tests/test_host_batch.py), so every table is bit-identical to the
        per-sequence constructor's; est_n_errors is the same Julia-order sum
        (rf_host_julia_sums; julia_sum without the library).  With `phreds`
        (the int8 Phred scores lp was divided from) the transcendental tables
        are evaluated once per distinct score and gathered: the same values,
        since each element's result depends on its value alone.  Returns the
        objects (their tables are views) and the concatenated tables for a
        single rf_set_sequences upload."""
        lp = np.ascontiguousarray(lp, np.float64)
        K = len(off) - 1
        if lp.min() == -math.inf:
            raise ValueError("a log error probability is negative infinity")
        if lp.max() > 0.0:
            raise ValueError(f"a log error probability is > 0: {lp.max()}")
        if phreds is not None:
            code = np.ascontiguousarray(np.asarray(phreds, np.int8).view(np.uint8))
            vals = phred_to_log_p(np.arange(256, dtype=np.uint8).view(np.int8))
            tp10 = np.power(10.0, vals)
            with np.errstate(divide="ignore", invalid="ignore"):
                tmatch = np.log10(1.0 - tp10)
            extra = {"code": code, "match_table": tmatch, "lp_table": vals}
            lib = None
            try:
                from . import _lib
                lib = _lib.load()
            except Exception:  # noqa: BLE001 -- host-only use without the library: numpy below
                pass
            if lib is not None:
                # gathers + FP64 add / max in C++ (rf_host_tables_from_codes): the
                # same values as the numpy expressions below, without their temporaries
                N, K = len(code), len(off) - 1
                off64 = np.ascontiguousarray(off, np.int64)
                lp2, match, mism, ins = (np.empty(N) for _ in range(4))
                dele, est = np.empty(N + K), np.empty(K)
                P = _lib.ptr
                lib.rf_host_tables_from_codes(K, P(code), P(off64), P(vals), P(tp10), P(tmatch),
                                              float(scores.mismatch), float(scores.insertion),
                                              float(scores.deletion), P(lp2), P(match), P(mism), P(ins),
                                              P(dele), P(est))
                if not np.array_equal(lp2, lp):
                    raise ValueError("phreds do not match the log error probabilities")
                return self_objects(cls, seqs, lp2, match, mism, ins, dele, est, off, bandwidth), \
                    {"match": match, "mismatch": mism, "ins": ins, "del": dele, **extra}
            if not np.array_equal(vals[code], lp):
                raise ValueError("phreds do not match the log error probabilities")
            p10, match = tp10[code], tmatch[code]
        else:
            p10 = np.power(10.0, lp)
            with np.errstate(divide="ignore"):
                match = np.log10(1.0 - p10)
            extra = {}
        mism = lp + scores.mismatch
        ins = lp + scores.insertion
        # del (n + 1 per sequence) = max(left, right) + deletion with left / right the
        # sequence's lp with its first / last element repeated: the ends are
        # max(x, x) = x, the inside the neighbour maximum (rifrafsequences.jl:49-53)
        left = np.insert(lp, off[:-1], lp[off[:-1]])
        right = np.insert(lp, off[1:], lp[off[1:] - 1])
        dele = np.maximum(left, right) + scores.deletion
        est = np.empty(K)
        try:
            from . import _lib
            _lib.load().rf_host_julia_sums(K, _lib.ptr(p10), _lib.ptr(np.ascontiguousarray(off, np.int64)),
                                           _lib.ptr(est))
        except Exception:  # noqa: BLE001 -- library absent (host-only use): the Python sum
            est = np.array([julia_sum(p10[off[k]:off[k + 1]]) for k in range(K)])
        return self_objects(cls, seqs, lp, match, mism, ins, dele, est, off, bandwidth), \
            {"match": match, "mismatch": mism, "ins": ins, "del": dele, **extra}

    @classmethod
    def many_coded(cls, seqs, phreds, off, bandwidth: int, scores: Scores, device=None, bases=None):
        """The native driver's setup (batch._wave_native) from concatenated
        int8 Phred scores, without building host tables: est_n_errors (the
        same Julia-order sum as many_concat) and logsumexp10 of every
        sequence's match scores (the values batch._logsumexp10_many returns)
        from one C++ pass (rf_host_code_prep) -- or, with `device` (a
        callable (codes, lp_table, match_table, p10_table, grid) -> (est,
        ucode, tsum) or None: the
        engine's rf_set_sequences_codes_prep, which uploads the reads and
        sums on the GPU, round 5), from the device's sums and the host's
        log10 (rf_host_lse_finish): the same bits.  The objects build their
        tables from the codes on first access (CodedRifrafSequence: the same
        gathers, adds and maxima as many_concat, so the same bits).  Returns
        (objects, tables-dict with the codes and per-code tables, lse), or
        None when the library is absent; tables-dict["uploaded"] says whether
        `device` uploaded the reads.  seqs None: the objects' sequences are
        views of `bases` (the concatenated reads, cut at `off`), made on
        first access."""
        try:
            from . import _lib
            lib = _lib.load()
        except Exception:  # noqa: BLE001 -- host-only use: the caller takes many_concat
            return None
        code = np.ascontiguousarray(np.asarray(phreds, np.int8).view(np.uint8))
        vals = phred_to_log_p(np.arange(256, dtype=np.uint8).view(np.int8))
        tp10 = np.power(10.0, vals)
        with np.errstate(divide="ignore", invalid="ignore"):
            tmatch = np.log10(1.0 - tp10)
            grid = np.ascontiguousarray(np.power(10.0, tmatch[None, :] - tmatch[:, None]))   # [u code, x code]
        if (code >= 128).any():
            raise ValueError("phred score cannot be negative")
        if not (vals[:128] <= 0.0).all() or np.isinf(vals[:128]).any():
            raise ValueError("a log error probability is out of range")
        K = len(off) - 1
        off64 = np.ascontiguousarray(off, np.int64)
        P = _lib.ptr
        dev = device(code, vals, tmatch, tp10, grid) if device is not None else None
        if dev is not None:
            est, ucode, tsum = dev
            lse = np.empty(K)
            if lib.rf_host_lse_finish(K, P(tsum), P(ucode), P(tmatch), P(lse)) != 0:
                raise ValueError("rf_host_lse_finish: invalid codes")
        else:
            est, lse = np.empty(K), np.empty(K)
            ucode = np.empty(K, np.int32)
            if lib.rf_host_code_prep(K, P(code), P(off64), P(tp10), P(tmatch), P(grid), P(est), P(ucode),
                                     P(lse)) != 0:
                raise ValueError("rf_host_code_prep: invalid segments (empty sequence?)")
        src = _CodeSource(code, off64, vals, tmatch, scores)
        src.bases = bases
        # per-sequence est / bandwidth live in the source's arrays (the
        # objects read and write them through properties), so neither this
        # loop nor a caller's bulk bandwidth update touches every object
        src.est = np.asarray(est, np.float64)
        src.bw = np.full(K, int(bandwidth), np.int64)
        src.bwf = np.zeros(K, bool)
        out = []
        new = object.__new__
        if seqs is None:
            for k in range(K):
                r = new(CodedRifrafSequence)
                r._src = src
                r._k = k
                out.append(r)
        else:
            put = _SEQ_SLOT.__set__
            for k, sq in enumerate(seqs):
                r = new(CodedRifrafSequence)
                put(r, sq)
                r._src = src
                r._k = k
                out.append(r)
        tabs = {"code": code, "match_table": tmatch, "lp_table": vals, "source": src, "uploaded": dev is not None,
                "est": np.asarray(est, np.float64)}
        return out, tabs, lse

    @classmethod
    def rescored(cls, other: "RifrafSequence", scores: Scores) -> "RifrafSequence":
        """RifrafSequence(seq, scores), rifrafsequences.jl:90-95."""
        r = cls(other.seq, other.error_log_p, other.bandwidth, scores)
        r.bandwidth_fixed = other.bandwidth_fixed
        return r

    def __len__(self):
        return int(self.seq.shape[0])

    def do_codon_ins(self):            # :102
        return len(self.codon_ins_scores) > 0

    def do_codon_del(self):            # :103
        return len(self.codon_del_scores) > 0

    def do_codon_moves(self):          # :104
        return self.do_codon_ins() or self.do_codon_del()


_EMPTY = np.empty(0)
_SEQ_SLOT = RifrafSequence.__dict__["seq"]
_TABLES = ("error_log_p", "match_scores", "mismatch_scores", "ins_scores", "del_scores")


class _CodeSource:
    """Codes and per-code tables shared by the CodedRifrafSequence objects of
    one many_coded call; full() gives the concatenated tables of
    many_concat (rf_host_tables_from_codes) when a caller needs them all."""

    def __init__(self, code, off, vals, tmatch, scores):
        self.code, self.off, self.vals, self.tmatch, self.scores = code, off, vals, tmatch, scores
        self._full = None

    def tables(self, k):
        a, b = int(self.off[k]), int(self.off[k + 1])
        lp = self.vals[self.code[a:b]]
        sc = self.scores
        d = np.empty(b - a + 1)
        d[0] = lp[0] + sc.deletion                                         # rifrafsequences.jl:49-53
        d[-1] = lp[-1] + sc.deletion
        if b - a > 1:
            d[1:-1] = np.maximum(lp[:-1], lp[1:]) + sc.deletion
        return lp, self.tmatch[self.code[a:b]], lp + sc.mismatch, lp + sc.insertion, d

    def full(self):
        if self._full is None:
            from . import _lib
            N, K = len(self.code), len(self.off) - 1
            lp, match, mism, ins = (np.empty(N) for _ in range(4))
            dele, est = np.empty(N + K), np.empty(K)
            P = _lib.ptr
            _lib.load().rf_host_tables_from_codes(K, P(self.code), P(self.off), P(self.vals),
                                                  P(np.power(10.0, self.vals)), P(self.tmatch),
                                                  float(self.scores.mismatch), float(self.scores.insertion),
                                                  float(self.scores.deletion), P(lp), P(match), P(mism), P(ins),
                                                  P(dele), P(est))
            self._full = {"match": match, "mismatch": mism, "ins": ins, "del": dele}
        return self._full


def _coded_table(name, idx):
    slot = RifrafSequence.__dict__[name]

    def get(self):
        try:
            return slot.__get__(self)
        except AttributeError:
            for nm, v in zip(_TABLES, self._src.tables(self._k)):
                RifrafSequence.__dict__[nm].__set__(self, v)
            return slot.__get__(self)

    def put(self, v):
        slot.__set__(self, v)
    return property(get, put)


class CodedRifrafSequence(RifrafSequence):
    """A RifrafSequence of RifrafSequence.many_coded: its tables are built
    from the Phred codes on first access (the same values as the eager
    constructor's); est_n_errors and the bandwidth fields are entries of the
    shared source's arrays."""

    __slots__ = ("_src", "_k")
    codon_ins_scores = _EMPTY     # reads have no codon tables
    codon_del_scores = _EMPTY

    @property
    def seq(self):
        slot = RifrafSequence.__dict__["seq"]
        try:
            return slot.__get__(self)
        except AttributeError:   # many_coded(seqs=None): a view of the shared bases
            src = self._src
            v = src.bases[int(src.off[self._k]):int(src.off[self._k + 1])]
            slot.__set__(self, v)
            return v

    @seq.setter
    def seq(self, v):
        RifrafSequence.__dict__["seq"].__set__(self, v)

    @property
    def est_n_errors(self):
        return float(self._src.est[self._k])

    @property
    def bandwidth(self):
        return int(self._src.bw[self._k])

    @bandwidth.setter
    def bandwidth(self, v):
        self._src.bw[self._k] = v

    @property
    def bandwidth_fixed(self):
        return bool(self._src.bwf[self._k])

    @bandwidth_fixed.setter
    def bandwidth_fixed(self, v):
        self._src.bwf[self._k] = v


for _i, _n in enumerate(_TABLES):
    setattr(CodedRifrafSequence, _n, _coded_table(_n, _i))
