"""Batched multi-cluster driver.

The reference polishes many clusters with one `rifraf()` per input file,
distributed over worker processes (`pmap`, scripts/rifraf.jl:71-120,190).
On one GPU that would be thousands of tiny launches.  `rifraf_batch` runs
the clusters' stage machines side by side on ONE engine context instead:

  - every cluster runs the unchanged host stage machine (`model.rifraf`) in
    its own host thread, against a `ClusterEngine` proxy that maps the
    cluster's local sequence / slot / template ids to disjoint global ids;
  - the hub waits until every live cluster is blocked on an engine request,
    then executes the requests as one launch per kind -- all realigns with
    the same flags in one `rf_realign`, all backtraces in one `rf_backtrace`,
    all proposal scorings in one `rf_score` -- and hands each cluster its
    share of the results.

The kernels compute every slot and every proposal group independently, so
each cluster's result is identical to a separate `rifraf()` call.  A failing
batched call is re-run request by request, so a reference `error()` reaches
exactly the cluster that raised it.
"""
from __future__ import annotations

import contextlib
import threading
import time

import numpy as np

from .bandedarrays import band_stride
from .engine import RifrafError
from .proposals import to_arrays
from .resampling import cluster_seeds
from .types import PackedReads


class _Request:
    __slots__ = ("k", "kind", "args", "ev", "result", "error")

    def __init__(self, k, kind, args):
        self.k, self.kind, self.args = k, kind, args
        self.ev = threading.Event()      # set by the hub: only this worker wakes
        self.result = None
        self.error = None


class ClusterEngine:
    """Engine proxy of one cluster inside a batched run (same methods as
    engine.Engine that the stage machine uses)."""

    def __init__(self, hub, k):
        self.hub, self.k = hub, k

    def set_sequences(self, first, seqs):
        return self.hub.call(self.k, "set_sequences", first, seqs)

    def set_templates(self, first, tpls):
        return self.hub.call(self.k, "set_templates", first, tpls)

    def realign(self, slots, seqs, tpls, bws, flags):
        if np.ndim(flags) == 0:
            return self.hub.call(self.k, "realign", slots, seqs, tpls, bws, flags)
        # flags per job: the hub batches requests by flags, so one request
        # per distinct value (the results in job order)
        slots = np.atleast_1d(np.asarray(slots, np.int32))
        n = len(slots)
        fl = np.broadcast_to(np.asarray(flags), (n,))
        seqs, tpls, bws = (np.broadcast_to(np.asarray(x), (n,)) for x in (seqs, tpls, bws))
        out = np.empty(n)
        for f in dict.fromkeys(fl.tolist()):
            idx = np.flatnonzero(fl == f)
            out[idx] = self.hub.call(self.k, "realign", slots[idx], seqs[idx], tpls[idx], bws[idx], int(f))
        return out

    def backtrace(self, slots, want_moves=True):
        return self.hub.call(self.k, "backtrace", slots, want_moves)

    def score(self, groups, per_seq=False):
        return self.hub.call(self.k, "score", groups, per_seq)

    def alignment_proposals(self, groups, do_indels):
        return self.hub.call(self.k, "aln_props", groups, do_indels)

    def geometry(self, slot, which=0):
        return self.hub.call(self.k, "geometry", slot, which)

    def download_band(self, slot, which=0, default=-np.inf):
        return self.hub.call(self.k, "download_band", slot, which, default)

    def close(self):
        pass


class _Hub:
    def __init__(self, engine, nclusters: int, stride: int):
        self.e = engine
        self.K = nclusters
        self.S = stride              # ids per cluster: reads + reference + scratch
        self.cv = threading.Condition()
        self.pending = []
        self.live = 0
        self.launches = 0
        self.engine_s = 0.0          # wall time inside batched engine calls

    # ---------------- id maps (local -> global) ----------------
    def seq(self, k, x):
        x = np.asarray(x, np.int64)
        if (x < 0).any() or (x >= self.S).any():
            raise RifrafError("batched cluster: sequence / slot id out of range")
        return (k * self.S + x).astype(np.int32)

    def tpl(self, k, x):
        x = np.asarray(x, np.int64)
        if (x < 0).any() or (x > 1).any():
            raise RifrafError("batched cluster: template id out of range")
        return (x * self.K + k).astype(np.int32)

    # ---------------- worker side ----------------
    def call(self, k, kind, *args):
        req = _Request(k, kind, args)
        with self.cv:
            self.pending.append(req)
            if len(self.pending) == self.live:
                self.cv.notify()             # the hub is the only waiter on cv
        req.ev.wait()
        if req.error is not None:
            raise req.error
        return req.result

    # ---------------- hub side ----------------
    def serve(self):
        while True:
            with self.cv:
                self.cv.wait_for(lambda: self.live == 0 or len(self.pending) == self.live)
                if self.live == 0 and not self.pending:
                    return
                batch, self.pending = self.pending, []
            t0 = time.perf_counter()
            self._execute(batch)
            self.engine_s += time.perf_counter() - t0
            for r in batch:
                r.ev.set()

    def _execute(self, batch):
        kinds = {}
        for r in batch:
            key = (r.kind, r.args[4]) if r.kind == "realign" else (
                (r.kind, bool(r.args[1])) if r.kind in ("backtrace", "score", "aln_props") else (r.kind, id(r)))
            kinds.setdefault(key, []).append(r)
        for (kind, _), reqs in kinds.items():
            fn = {"realign": self._realign, "backtrace": self._backtrace, "score": self._score,
                  "aln_props": self._aln_props}.get(kind)
            if fn is not None and len(reqs) > 1:
                try:
                    fn(reqs)
                    self.launches += 1
                    continue
                except RifrafError:
                    pass                      # attribute the error: one request at a time
            for r in reqs:
                try:
                    (fn or self._single)([r])
                    self.launches += 1
                except RifrafError as e:
                    r.error = e

    def _single(self, reqs):
        (r,) = reqs
        k, a = r.k, r.args
        if r.kind == "set_sequences":
            self.e.set_sequences(int(self.seq(k, a[0])), a[1])
        elif r.kind == "set_templates":
            ids = self.tpl(k, np.arange(a[0], a[0] + len(a[1])))
            for i, t in zip(ids, a[1]):
                self.e.set_templates(int(i), [t])
        elif r.kind == "geometry":
            r.result = self.e.geometry(int(self.seq(k, a[0])), a[1])
        elif r.kind == "download_band":
            r.result = self.e.download_band(int(self.seq(k, a[0])), a[1], a[2])
        else:
            raise RifrafError(f"batched cluster: unknown request {r.kind}")

    def _realign(self, reqs):
        sl, sq, tp, bw, cnt = [], [], [], [], []
        for r in reqs:
            slots, seqs, tpls, bws, _ = r.args
            slots = np.atleast_1d(np.asarray(slots, np.int32))
            n = len(slots)
            sl.append(self.seq(r.k, slots))
            sq.append(self.seq(r.k, np.broadcast_to(seqs, (n,))))
            tp.append(self.tpl(r.k, np.broadcast_to(tpls, (n,))))
            bw.append(np.broadcast_to(np.asarray(bws, np.int32), (n,)))
            cnt.append(n)
        out = self.e.realign(np.concatenate(sl), np.concatenate(sq), np.concatenate(tp),
                             np.concatenate(bw), reqs[0].args[4])
        at = 0
        for r, n in zip(reqs, cnt):
            r.result = out[at:at + n].copy()
            at += n

    def _backtrace(self, reqs):
        want = bool(reqs[0].args[1])
        sl = [self.seq(r.k, np.atleast_1d(np.asarray(r.args[0], np.int32))) for r in reqs]
        moves, nerr = self.e.backtrace(np.concatenate(sl), want)
        at = 0
        for r, s in zip(reqs, sl):
            n = len(s)
            r.result = (moves[at:at + n] if want else None, nerr[at:at + n].copy())
            at += n

    def _aln_props(self, reqs):
        groups, cnt = [], []
        for r in reqs:
            cnt.append(len(r.args[0]))
            groups += [self.seq(r.k, np.asarray(sl, np.int32)) for sl in r.args[0]]
        res = self.e.alignment_proposals(groups, bool(reqs[0].args[1]))
        at = 0
        for r, n in zip(reqs, cnt):
            r.result = res[at:at + n]
            at += n

    def _score(self, reqs):
        per_seq = bool(reqs[0].args[1])
        groups, cnt = [], []
        for r in reqs:
            gs = r.args[0]
            cnt.append(len(gs))
            for bslots, ref, props in gs:
                p = props if isinstance(props, tuple) else to_arrays(props)
                groups.append((self.seq(r.k, np.asarray(bslots, np.int32)),
                               int(self.seq(r.k, ref)) if ref >= 0 else -1, p))
        res = self.e.score(groups, per_seq=per_seq)
        tot, mats = (res if per_seq else (res, None))
        at = 0
        for r, n in zip(reqs, cnt):
            r.result = (tot[at:at + n], mats[at:at + n]) if per_seq else tot[at:at + n]
            at += n


STATS = {"launches": 0, "engine_s": 0.0, "native_s": 0.0, "score_phase_s": 0.0, "setup_native_s": 0.0,
         "upload_s": 0.0, "qv_refill_skipped": 0}
_STATS_LOCK = threading.Lock()   # waves of several engines update STATS from their own threads


def _stat(key, value):
    with _STATS_LOCK:
        STATS[key] += value


# diagnostics: a list to receive (thread name, phase, t0, t1, thread CPU s) of
# every native wave's phases (setup, upload, prep, native, results, qv), or None
TIMELINE = None
_TL = threading.local()


def _span(phase, t0):
    if TIMELINE is not None:
        c = time.thread_time()
        TIMELINE.append((threading.current_thread().name, phase, t0, time.perf_counter(),
                         c - getattr(_TL, "cpu", c)))
        _TL.cpu = c


def native_eligible(clusters, params) -> bool:
    """Whether rf_rifraf_batch(_ref) (rifraf_batch.cpp) can run these
    clusters: INIT enabled, fixed, full or random batches (the native driver
    draws random ones with resampling.py's RNG and draw).  Clusters with a
    reference run INIT -> FRAME -> REFINE natively when the quality pass does
    not use the reference."""
    if not params.do_init:
        return False
    for kw in clusters:
        n = len(kw["dnaseqs"])
        if n < 1:
            return False
        ref = kw.get("reference")
        if ref is not None and len(ref) > 0:
            if params.do_score and params.use_ref_for_qvs:
                return False
            try:
                from .model import check_params
                check_params(params.scores, ref, params)
            except Exception:  # noqa: BLE001 -- the Python stage machine raises it per cluster
                return False
        # an empty read or a per-base vector of the wrong length keeps the
        # cluster on the Python stage machine, whose RifrafSequence
        # constructor (rifrafsequences.jl:19-35) gives the reference's
        # behaviour for it (empty sequence / ValueError)
        quals = kw.get("error_log_ps")
        if quals is None:
            quals = kw.get("phreds")
        if quals is None or len(quals) != n:
            return False
        ds = kw["dnaseqs"]
        if isinstance(ds, PackedReads) and isinstance(quals, PackedReads):
            if not np.array_equal(ds.off, quals.off) or (ds.lens() == 0).any():
                return False
            continue
        ls = list(map(len, ds))
        if 0 in ls or ls != list(map(len, quals)):
            return False
    return True


def _logsumexp10_many(values, off, codes=None, table=None):
    """model.logsumexp10 of every segment values[off[k]:off[k+1]] (non-empty):
    the same max, the same numpy power of the shifted values (numpy
    evaluates each element alike wherever it sits), the same sequential sum
    (rf_host_seq_sums) and the same math.log10.  With `codes` (values ==
    table[codes], a 256-entry table), 10 ** (x - u) is evaluated once per
    (code of x, code of u) pair and gathered -- the same values."""
    import math

    from . import _lib
    u = np.maximum.reduceat(values, off[:-1])
    lens = np.diff(off)
    p = None
    if codes is not None:
        fin = np.isfinite(table)
        pos = {float(v): c for c, v in enumerate(table.tolist()) if fin[c]}
        if all(float(x) in pos for x in u.tolist() if math.isfinite(x)):
            ucode = np.array([pos.get(float(x), 0) for x in u.tolist()], np.int32)
            with np.errstate(invalid="ignore"):
                grid = np.ascontiguousarray(np.power(10.0, table[None, :] - table[:, None]))   # [u code, x code]
            s = np.empty(len(lens))
            _lib.load().rf_host_code_seq_sums(len(lens), _lib.ptr(np.ascontiguousarray(codes, np.uint8)),
                                              _lib.ptr(np.ascontiguousarray(off, np.int64)), _lib.ptr(ucode),
                                              _lib.ptr(grid), _lib.ptr(s))
            p = True
    if p is None:
        sh = values - np.repeat(u, lens)
        p = np.ascontiguousarray(np.power(10.0, sh))
        s = np.empty(len(lens))
        _lib.load().rf_host_seq_sums(len(lens), _lib.ptr(p), _lib.ptr(np.ascontiguousarray(off, np.int64)),
                                     _lib.ptr(s))
    out = []
    for k in range(len(lens)):
        uk = float(u[k])
        if abs(uk) == math.inf:
            seg = values[off[k]:off[k + 1]]
            out.append(math.nan if np.isnan(seg).any() else uk)
        else:
            out.append(math.log10(float(s[k])) + uk)
    return out


def _native_refs(part, states, refs, params, engine, nseq, nslot):
    """The reference records of a native wave (rf_rifraf_batch_ref), or None
    when no cluster has a reference.  Ids past the reads: cluster j-th
    reference at sequence nseq + j (uploaded by the callback at FRAME entry),
    its edit-distance copy at nseq + nref + j (uploaded here: log p -1,
    ErrorModel(1, 1, 1) scores, as align.edit_distance builds it), slots
    nslot + 2j (A/B) and nslot + 2j + 1 (scratch).  The callback performs the
    two host steps of finish_stage! that need the mirror's numerics."""
    import math

    from . import _lib
    from .errormodel import ErrorModel, Scores
    from .poisson import cquantile_poisson
    from .rifrafsequences import RifrafSequence
    has = [k for k, r in enumerate(refs) if len(r) > 0]
    if not has:
        return None
    nref = len(has)
    recs = (_lib.BatchRef * len(part))()
    ref_id = {}
    bases, at = [], 0
    for k in range(len(part)):
        recs[k].ref_seq = -1
    edit = []
    ed_scores = Scores.from_errors(ErrorModel(1.0, 1.0, 1.0))
    for j, k in enumerate(has):
        r = refs[k]
        ref_id[k] = nseq + j
        recs[k].ref_seq = nseq + j
        recs[k].edit_seq = nseq + nref + j
        recs[k].ref_slot = nslot + 2 * j
        recs[k].scratch_slot = nslot + 2 * j + 1
        recs[k].ref_off = at
        recs[k].ref_len = len(r)
        bases.append(np.asarray(r, np.uint8))
        at += len(r)
        edit.append(RifrafSequence(r, np.full(len(r), -1.0), max(1, (len(r) + 1) // 2), ed_scores))
    engine.set_sequences(nseq + nref, edit)
    errors = {}

    def cb(user, c, event, value, thr):
        try:
            st = states[c]
            if event == 0:                                   # finish_stage!, INIT -> FRAME (model.jl:944-957)
                st.ref_error_rate = value
                lp = np.full(len(st.reference), math.log10(st.ref_error_rate))
                st.reference = RifrafSequence(st.reference.seq, lp, params.bandwidth, st.ref_scores)
                engine.set_sequences(ref_id[c], [st.reference])
                thr[0] = cquantile_poisson(st.reference.est_n_errors, params.bandwidth_pvalue)
            else:                                            # penalty increase (model.jl:973-985)
                st.n_ref_indel_mults = int(value)
                mult = params.ref_indel_mult ** st.n_ref_indel_mults
                rs = st.ref_scores
                st.ref_scores = Scores(rs.mismatch, rs.insertion * mult, rs.deletion * mult, rs.codon_insertion,
                                       rs.codon_deletion)
                st.reference = RifrafSequence.rescored(st.reference, st.ref_scores)
                engine.set_sequences(ref_id[c], [st.reference])
            return 0
        except Exception as e:  # noqa: BLE001 -- the driver fails the cluster
            errors[c] = e
            return 1

    rp = _lib.BatchRefParams(int(params.do_frame), int(params.do_refine), int(params.seed_indels),
                             int(params.indel_correction_only), int(params.max_ref_indel_mults), 0,
                             float(params.ref_error_mult))
    return {"params": rp, "refs": recs, "bases": np.concatenate(bases), "cb": _lib.RefCallback(cb),
            "cb_errors": errors}


def _wave_native(part, params, engine, init_lock=None, device_qv=True, setup_lock=None):
    """One wave through the native stage machine (rf_rifraf_batch), then
    (do_score) the quality pass of every cluster with three batched engine
    calls; host setup is vectorised across the wave's reads.  init_lock
    (several engines, rifraf_batch(init_exclusive=True)): held around the
    native stage machine, so one engine's stage machine runs while the others
    do their host work (setup, quality pass).  device_qv: the quality pass's
    normalisations on the device (engine.qv_probs: 10^x by the GPU's exp10,
    ~1e-15 relative of numpy's, not bit for bit) when every read is
    row-coded; False keeps them on the host (bit-identical to the Python
    stage machine)."""
    from . import _lib
    from .engine import RF_BWD, RF_FWD
    from .errormodel import phred_to_log_p
    from .model import EstimatedProbs, RifrafResult, Stage, check_params, initial_state, qvs_many_lib
    from .poisson import cquantile_poisson_many
    from .proposals import AmbiguousProposalsError
    from .rifrafsequences import RifrafSequence
    from .types import DNASeq

    # setup_lock (several engines): one engine at a time in the host setup,
    # which is mostly Python (the GIL): the first engine's stage machine
    # starts after one setup, not after all of them interleaved
    if TIMELINE is not None:
        _TL.cpu = time.thread_time()
    held = setup_lock is not None and setup_lock.acquire()
    try:
        K = len(part)
        t_setup = time.perf_counter()
        check_params(params.scores, np.zeros(0, np.uint8), params)
        all_s, all_lp, nread = [], [], []
        phred_in = all(kw.get("error_log_ps") is None for kw in part)
        # reads handed over packed (PackedReads: one buffer + offsets per
        # cluster, e.g. FASTQ ingest or bench's e2e staging): one concatenation
        # per cluster instead of one per read, and no per-read objects here
        packed = phred_in and all(isinstance(kw["dnaseqs"], PackedReads) and isinstance(kw["phreds"], PackedReads)
                                  and kw["dnaseqs"].buf.dtype == np.uint8 and kw["phreds"].buf.dtype.kind in "iu"
                                  for kw in part)
        allb = None
        if packed:
            for kw in part:
                if not np.array_equal(kw["dnaseqs"].off, kw["phreds"].off):
                    raise RifrafError("empty read or length mismatch")
            nread = [len(kw["dnaseqs"]) for kw in part]
            lens = np.concatenate([kw["dnaseqs"].lens() for kw in part]) if part else np.zeros(0, np.int64)
            cat_lp = np.concatenate([kw["phreds"].buf for kw in part]) if part else None
            allb = np.concatenate([kw["dnaseqs"].buf for kw in part]) if part else np.zeros(0, np.uint8)
            all_s = None
            if (lens == 0).any():
                raise RifrafError("empty read or length mismatch")
        else:
            for kw in part:                                                 # rifraf(), model.jl:1276-1287
                if phred_in:
                    all_lp += list(kw["phreds"])
                else:
                    elp = kw.get("error_log_ps")
                    all_lp += [phred_to_log_p(p) for p in kw["phreds"]] if elp is None else list(elp)
                # code arrays pass as they are (DNASeq would only re-wrap them)
                all_s += [x if type(x) is np.ndarray and x.dtype == np.uint8 and x.flags.c_contiguous else DNASeq(x)
                          for x in kw["dnaseqs"]]
                nread.append(len(kw["dnaseqs"]))
            cat_lp = np.concatenate(all_lp) if (phred_in and all_lp) else None
            lens = np.fromiter(map(len, all_s), np.int64, len(all_s))
            if (lens == 0).any() or len(all_lp) != len(all_s) or \
                    (lens != np.fromiter(map(len, all_lp), np.int64, len(all_lp))).any():
                raise RifrafError("empty read or length mismatch")
        if cat_lp is not None and len(cat_lp) and int(cat_lp.min()) < 0:
            raise RifrafError("phred score cannot be negative")
        nall = len(lens)
        soff = np.zeros(nall + 1, np.int64)
        np.cumsum(lens, out=soff[1:])
        # integer Phred scores: the codes go to the device and the host builds no
        # tables (est_n_errors and the initial consensus's logsumexp10 in one C++
        # pass; RifrafSequence.many_coded), else the concatenated host tables
        coded = None
        if (phred_in and cat_lp is not None and cat_lp.dtype.kind in "iu" and len(cat_lp)
                and int(cat_lp.max()) <= 127):
            device = None
            if hasattr(engine, "set_sequences_codes"):
                # the reads go to the device first, and the per-read setup sums
                # (est_n_errors, logsumexp10) come back from it (round 5: no
                # per-position host pass; rf_set_sequences_codes_prep)
                if hasattr(engine, "release_bands"):
                    engine.release_bands()
                if allb is None:
                    allb = np.concatenate(all_s)

                def device(code, lp_t, match_t, p10, grid):
                    r = engine.set_sequences_codes(0, allb, soff, code, lp_t, match_t, params.scores, prep=(p10, grid))
                    return r if r is not False else None
            coded = RifrafSequence.many_coded(all_s, cat_lp.astype(np.int8, copy=False), soff, params.bandwidth,
                                              params.scores, device=device, bases=allb)
        if coded is not None:
            allseqs, tabs, lse_all = coded
        else:
            # one division / ufunc pass over every read (elementwise: equal to per-read calls)
            lp = phred_to_log_p(cat_lp) if phred_in else np.concatenate(
                [np.asarray(x, np.float64) for x in all_lp])
            if all_s is None:   # packed reads on the host-table path: per-read views
                all_s = [allb[soff[k]:soff[k + 1]] for k in range(nall)]
            allseqs, tabs = RifrafSequence.many_concat(all_s, lp, soff, params.bandwidth, params.scores,
                                                       phreds=cat_lp.astype(np.int8) if phred_in else None)
            lse_all = None
        nread = np.array(nread, np.int32)
        read_off = np.zeros(K + 1, np.int32)
        np.cumsum(nread, out=read_off[1:])
        # initial consensus where none is given: the read of max logsumexp10(match scores)
        need = [k for k, kw in enumerate(part) if kw.get("consensus") is None or len(kw["consensus"]) == 0]
        first = {}
        if need:
            ridx = np.concatenate([np.arange(read_off[k], read_off[k + 1]) for k in need])
            if lse_all is None:
                ms = [allseqs[r].match_scores for r in ridx]
                moff = np.zeros(len(ms) + 1, np.int64)
                np.cumsum([len(x) for x in ms], out=moff[1:])
            if lse_all is not None:
                lse = lse_all[ridx]
            elif len(need) == K and phred_in:
                lse = _logsumexp10_many(tabs["match"], moff, codes=tabs["code"], table=tabs["match_table"])
            else:
                lse = _logsumexp10_many(np.concatenate(ms), moff)
            at = 0
            for k in need:
                sc = lse[at:at + nread[k]]
                first[k] = allseqs[read_off[k] + int(np.argmax(sc))].seq.copy()
                at += nread[k]
        states = []
        refs_in = [DNASeq(kw["reference"]) if kw.get("reference") is not None and len(kw["reference"]) > 0
                   else np.zeros(0, np.uint8) for kw in part]
        maxlen = np.maximum.reduceat(lens, read_off[:-1]) if K > 0 else lens
        for k, kw in enumerate(part):
            cons = first[k] if k in first else DNASeq(kw["consensus"])
            states.append(initial_state(cons, allseqs[read_off[k]:read_off[k + 1]], refs_in[k], params,
                                        maxlen=int(maxlen[k])))
        # ids: cluster k's reads (and batch slots) are read_off[k] + local index; template k.
        # The bands of every batch read in one arena reservation (growing it in
        # steps would re-allocate and compact tens of GB several times): A and B
        # at the initial bandwidth plus the doubled bandwidth's regions, which a
        # band-doubling realign allocates above them (the arena bump-allocates; a
        # reservation of 1.5x the initial bands grew, and compacted every band,
        # in each c3 run: 1,999 regions, ~1.8 ms of a 45 ms run, r05am trace)
        # batch slots per cluster: the fixed batch and / or the random or full
        # one (a reference-guided cluster's REFINE follows a fixed INIT / FRAME;
        # a batch that check_score grows later grows the arena)
        nb = np.array([max(st_.batch_fixed_size if params.batch_fixed else 0,
                           st_.batch_size if not params.batch_fixed or (len(refs_in[k]) > 0 and params.do_refine)
                           else 0) for k, st_ in enumerate(states)])
        # every read's A/B band (upper bound: padded rows), one vector pass; a
        # cluster whose batch is smaller than its reads counts its largest bands
        mcons = np.fromiter((len(st_.consensus) for st_ in states), np.int64, K)
        mrd = np.repeat(mcons, nread)
        dn = np.abs(lens - mrd)
        band = np.zeros(len(lens), np.int64)
        for bw_ in (params.bandwidth, 2 * params.bandwidth):
            Hs = 2 * bw_ + dn + 1
            band += (Hs + 2 * mrd) * band_stride(Hs, pad_h=1) * 8
        est_bytes = 2 * int(band.sum())
        for k in np.flatnonzero(nb < nread):
            bk = band[read_off[k]:read_off[k + 1]]
            est_bytes -= 2 * int(bk.sum() - np.sort(bk)[::-1][:nb[k]].sum())
        for k, st_ in enumerate(states):
            m = len(st_.consensus)
            L = len(refs_in[k])
            if L > 0:
                # reference-guided cluster (_native_refs): the reference's A and B
                # at the read bandwidth, and the scratch slot's forward band, which
                # at FRAME entry holds edit_distance's band at bw = ceil(min / 2)
                # (align.jl:253-260) -- it grows with the square of the length
                for bw_ in (params.bandwidth, 2 * params.bandwidth):
                    Hr = 2 * bw_ + abs(L - m) + 1
                    est_bytes += 2 * (Hr + 2 * m) * band_stride(Hr, pad_h=1) * 8
                bwe = -(-min(L, m) // 2)
                He = 2 * bwe + abs(L - m) + 1
                est_bytes += (He + 2 * m) * band_stride(He, pad_h=1) * 8
        # a new wave rewrites every slot it uses: the previous wave's bands are
        # dropped and the arena is reused (sized once for a steady stream of waves)
        uploaded = coded is not None and tabs["uploaded"]
        if hasattr(engine, "release_bands") and not uploaded:
            engine.release_bands()
        engine.reserve(int(est_bytes * 1.1) + (64 << 20))
        _stat("setup_native_s", time.perf_counter() - t_setup)
        _span("setup", t_setup)
        t_up = time.perf_counter()
        if allb is None:
            allb = np.concatenate(all_s)
        # Phred-coded reads: 2 B per position to the device, tables built there
        # (rf_set_sequences_codes; the same bits; already done with the setup
        # sums above when `uploaded`); else the host tables
        if not uploaded and not (
                phred_in and hasattr(engine, "set_sequences_codes") and
                engine.set_sequences_codes(0, allb, soff, tabs["code"], tabs["lp_table"], tabs["match_table"],
                                           params.scores)):
            ft = tabs["source"].full() if coded is not None else tabs
            engine.set_sequences_concat(0, allb, soff, ft["match"], ft["mismatch"], ft["ins"], ft["del"])
        engine.set_templates(0, [st_.consensus for st_ in states])
        _stat("upload_s", time.perf_counter() - t_setup)
        _span("upload", t_up)
        t_up = time.perf_counter()
        read_seq = np.arange(nall, dtype=np.int32)
        read_len = lens.astype(np.int32)
        est = tabs["est"] if coded is not None else np.array([s.est_n_errors for s in allseqs])
        thr = cquantile_poisson_many(est, params.bandwidth_pvalue)
        fixed_off = fixed = None
        if params.batch_fixed:
            fb = [np.argsort(est[read_off[k]:read_off[k + 1]], kind="stable")[:st_.batch_fixed_size]
                  for k, st_ in enumerate(states)]                      # resample!, model.jl:1045-1049
            fixed_off = np.zeros(K + 1, np.int32)
            np.cumsum([len(b) for b in fb], out=fixed_off[1:])
            fixed = np.concatenate(fb).astype(np.int32)
        cons = [st_.consensus for st_ in states]
        cons_off = np.zeros(K + 1, np.int64)
        np.cumsum([len(c) for c in cons], out=cons_off[1:])
        # random batches (resample!): every read's est_n_errors and a seed per
        # cluster for the driver's RNG (resampling.py); kept alive in `keep`
        est_c = np.ascontiguousarray(est, np.float64)
        seeds = cluster_seeds(params.seed, K)
        keep = (est_c, seeds)
        bp = _lib.BatchParams(params.max_iters, params.min_dist, params.bandwidth, int(params.do_alignment_proposals),
                              int(params.batch_fixed), params.batch_size, params.batch_threshold,
                              states[0].batch_randomness if K else 0.9, params.batch_mult,
                              est_c.ctypes.data, seeds.ctypes.data)
        ref = _native_refs(part, states, refs_in, params, engine, nall, int(read_off[-1]))
        _span("prep", t_up)
    finally:
        if held:
            setup_lock.release()
    with (init_lock if init_lock is not None else contextlib.nullcontext()):
        t0 = time.perf_counter()   # the stage machine's own time, not the wait for the lock
        res, bw = engine.rifraf_batch_native(bp, read_off, read_seq, read_len, thr, fixed_off, fixed,
                                             read_off[:-1], np.arange(K, dtype=np.int32), np.concatenate(cons),
                                             cons_off, ref=ref)
        _stat("native_s", time.perf_counter() - t0)
        _span("native", t0)
    del keep
    t_res = time.perf_counter()
    cb_errors = ref["cb_errors"] if ref is not None else {}
    if coded is not None:                  # CodedRifrafSequence: the shared arrays
        src = tabs["source"]
        bwa = np.asarray(bw, np.int64)
        src.bw[:] = np.abs(bwa)
        src.bwf[:] = bwa < 0
    else:
        for s, b in zip(allseqs, bw.tolist()):
            s.bandwidth = abs(b)
            s.bandwidth_fixed = b < 0
    results, errors = [], [None] * K
    for k, (st_, r) in enumerate(zip(states, res)):
        if r["status"] == 2:
            errors[k] = (cb_errors[k] if k in cb_errors else AmbiguousProposalsError()
                         if r["error"] == "AmbiguousProposalsError" else RifrafError(r["error"]))
        st_.consensus = DNASeq(r["consensus"])
        st_.score = r["score"]
        st_.stage_iterations = list(r["stage_iters"]) + [0]
        st_.converged = r["status"] == 1
        st_.batch_seqs = r["batch"]
        st_.n_slots = len(r["batch"])
        st_.slot_scores = [0.0] * st_.n_slots
        st_.stage = Stage.SCORE
        if len(st_.reference) > 0:
            st_.ref_score = r["ref_score"]
            st_.reference.bandwidth = abs(r["ref_bw"])
            st_.reference.bandwidth_fixed = r["ref_bw"] < 0
        stages = [[], [], []]
        for c, sg in zip(r["stages"], r["stage_of"]):
            stages[sg - 1].append(DNASeq(c))
        results.append(RifrafResult(consensus=st_.consensus, params=params, state=st_,
                                    consensus_stages=stages))
    _span("results", t_res)
    for e in errors:
        if e is not None:
            raise e
    if params.do_score:                                             # model.jl:1262-1270
        t0 = time.perf_counter()
        # realign_rescore (every batch read is bandwidth_fixed: one fill each),
        # estimate_probs over the dense totals, alignment_error_probs's sums
        groups = [read_off[k] + np.arange(len(st_.batch_seqs), dtype=np.int32) for k, st_ in enumerate(states)]
        # The bands already hold that fill when every cluster converged
        # without changing its consensus in its last iteration and its batch
        # was every read from the start (the slots never changed reads, and
        # every consensus change was followed by an A and B fill): the device
        # templates are the final consensi and the native final score is the
        # same left fold of the same A[end, end] values, so the fill is
        # skipped.  Otherwise (a cluster stopped at max_iters, fixed or random
        # batches) every cluster is refilled as the reference does.
        current = not params.batch_fixed and all(
            (params.batch_size <= 1 or params.batch_size >= int(nread[k])) and r["status"] == 1 and
            len(r["stages"]) > 0 and np.array_equal(np.asarray(r["stages"][-1]), np.asarray(r["consensus"]))
            for k, r in enumerate(res))
        _stat("qv_refill_skipped", 1 if current else 0)
        if not current:
            sq = np.concatenate([read_off[k] + np.asarray(st_.batch_seqs, np.int32) for k, st_ in enumerate(states)])
            tp = np.concatenate([np.full(len(g), k, np.int32) for k, g in enumerate(groups)])
            bws = np.abs(np.asarray(bw, np.int64))[sq].astype(np.int32)   # = the reads' .bandwidth set above
            engine.set_templates(0, [st_.consensus for st_ in states])
            sc = engine.realign(np.concatenate(groups), sq, tp, bws, RF_FWD | RF_BWD)
            at = 0
            for st_ in states:
                n = len(st_.batch_seqs)
                st_.slot_scores = [float(v) for v in sc[at:at + n]]
                total = st_.slot_scores[0]                              # rescore!, model.jl:630-635
                for v in st_.slot_scores[1:st_.n_slots]:
                    total += v
                st_.score = total
                at += n
        tl = [len(st_.consensus) for st_ in states]
        qv = None
        if device_qv and coded is not None and hasattr(engine, "qv_probs") and min(tl) > 0:
            qv = engine.qv_probs(groups, tl, [st_.score for st_ in states])
        if qv is not None:
            pos, ins, aln, err = qv
            if err[0]:
                raise RifrafError({1: "failed to compute a valid score", 2: "sub scores cannot be positive",
                                   3: "deletion scores cannot be positive",
                                   4: "insertion scores cannot be positive"}[int(err[0])])
            row = 0
            for k, m in enumerate(tl):
                results[k].error_probs = EstimatedProbs(pos[row:row + m, :4], pos[row:row + m, 4],
                                                        ins[row + k:row + k + m + 1])
                results[k].aln_error_probs = aln[row:row + m]
                row += m
            _stat("score_phase_s", time.perf_counter() - t0)
            _span("qv", t0)
            return results
        dense = engine.score_dense(groups, rows=[len(st_.consensus) + 1 for st_ in states])
        ridx = np.concatenate([read_off[k] + np.asarray(st_.batch_seqs, np.int64) for k, st_ in enumerate(states)])
        sums = engine.aln_error_sums_ptr(groups, tl, None, None, lens[ridx]) if coded is not None else None
        if sums is None:        # host fold: the reads' bases and match scores
            ft = tabs["source"].full() if coded is not None else tabs
            sums = engine.aln_error_sums_ptr(groups, tl, allb.ctypes.data + soff[ridx].astype(np.uint64),
                                             ft["match"].ctypes.data + 8 * soff[ridx].astype(np.uint64), lens[ridx])
        for k, (ep, ap) in enumerate(qvs_many_lib(states, dense, sums)):
            results[k].error_probs = ep
            results[k].aln_error_probs = ap
        _stat("score_phase_s", time.perf_counter() - t0)
    return results


def rifraf_batch(clusters, params=None, engine=None, wave: int = 1024, native=None, engines=None,
                 init_exclusive: bool = False, device_qv: bool = True, setup_exclusive: bool = True):
    """rifraf() over many independent clusters, batched on one engine.

    engines: several engines (contexts, each with its own HIP stream, e.g.
    on one GPU), one host thread each.  The clusters are cut into waves of at
    most min(wave, ceil(len / len(engines))) clusters, and each thread takes
    the next wave from a shared queue, so one engine's host work (table
    setup, quality pass) overlaps another's kernels.  init_exclusive: at most
    one engine runs its native stage machine at a time (the others meanwhile
    do host work: a two-stage pipeline of waves).  setup_exclusive: at most
    one engine in a native wave's host setup at a time (mostly Python, so
    interleaving two setups only delays both).  Clusters are independent,
    so the results equal one engine's.  device_qv (native driver): the
    quality pass's normalisations on the device (see _wave_native).

    clusters: sequence of dicts with the keyword arguments of model.rifraf
    (`dnaseqs`, `phreds` or `error_log_ps`, optional `consensus`,
    `reference`).  Returns the list of RifrafResult in input order (an
    exception raised by a cluster is re-raised after the wave finishes).
    Clusters run in waves of at most `wave` (their bands share the device).
    native (default: when eligible, see native_eligible): run the INIT stage
    machine in the library (rf_rifraf_batch) instead of one host thread per
    cluster; the results are identical."""
    import os
    from .model import RifrafParams, rifraf
    params = params or RifrafParams()
    if engines is not None and len(engines) > 1:
        E = len(engines)
        wv = max(1, min(wave, -(-len(clusters) // E)))
        starts = list(range(0, len(clusters), wv))
        out = [None] * len(starts)
        errs = [None] * len(starts)
        nxt = [0]
        qlock = threading.Lock()
        ilock = threading.Lock() if init_exclusive else None
        slock = threading.Lock() if setup_exclusive else None

        def worker(i):
            while True:
                with qlock:
                    w = nxt[0]
                    nxt[0] += 1
                if w >= len(starts):
                    return
                part = clusters[starts[w]:starts[w] + wv]
                try:
                    if (ilock is not None or slock is not None) and (native is None or native) and \
                            native_eligible(part, params) and hasattr(engines[i], "rifraf_batch_native"):
                        out[w] = _wave_native(part, params, engines[i], init_lock=ilock, device_qv=device_qv,
                                              setup_lock=slock)
                    else:
                        out[w] = rifraf_batch(part, params=params, engine=engines[i], wave=wv, native=native,
                                              device_qv=device_qv)
                except BaseException as e:  # noqa: BLE001 -- re-raised below in wave order
                    errs[w] = e
        ts = [threading.Thread(target=worker, args=(i,), daemon=True) for i in range(E)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for e in errs:
            if e is not None:
                raise e
        return [r for part in out for r in part]
    if engines is not None and engine is None:
        engine = engines[0]
    profile_dir = os.environ.get("RIFRAF_BATCH_PROFILE")
    if engine is None:
        from .align import default_engine
        engine = default_engine()
    ok = native_eligible(clusters, params) and hasattr(engine, "rifraf_batch_native")
    if native is None:
        native = ok
    elif native and not ok:
        raise RifrafError("rifraf_batch(native=True): clusters or engine outside the native driver's scope")
    results = [None] * len(clusters)
    for w0 in range(0, len(clusters), wave):
        part = clusters[w0:w0 + wave]
        if native:
            results[w0:w0 + len(part)] = _wave_native(part, params, engine, device_qv=device_qv)
            continue
        stride = max(len(c["dnaseqs"]) for c in part) + 2
        hub = _Hub(engine, len(part), stride)
        errors = [None] * len(part)

        def worker(k, kw):
            try:
                if profile_dir and k == 0:       # diagnostics: host profile of one cluster thread
                    import cProfile
                    pr = cProfile.Profile()
                    results[w0 + k] = pr.runcall(rifraf, params=params, engine=ClusterEngine(hub, k), **kw)
                    pr.dump_stats(f"{profile_dir}/batch_worker0.prof")
                else:
                    results[w0 + k] = rifraf(params=params, engine=ClusterEngine(hub, k), **kw)
            except Exception as e:  # noqa: BLE001 -- handed back to the caller
                errors[k] = e
            finally:
                with hub.cv:
                    hub.live -= 1
                    if len(hub.pending) == hub.live:
                        hub.cv.notify()

        hub.live = len(part)
        threads = [threading.Thread(target=worker, args=(k, kw), daemon=True) for k, kw in enumerate(part)]
        for t in threads:
            t.start()
        hub.serve()
        for t in threads:
            t.join()
        _stat("launches", hub.launches)
        _stat("engine_s", hub.engine_s)
        for e in errors:
            if e is not None:
                raise e
    return results


__all__ = ["rifraf_batch", "ClusterEngine"]


class ClusterQueue:
    """Waves of cluster indices [0, n) handed out to whichever rank asks next
    -- the reference's `pmap` over files (scripts/rifraf.jl:190: an idle
    worker takes the next file) across the GPUs of a node.  The counter lives
    in the process group's key-value store (torch.distributed's TCPStore:
    `add` is atomic), so no data-path collective is involved.  Every rank
    must create its store-backed queues in the same order (the key carries a
    generation number counted over store-backed queues only), or pass the
    same explicit `key`; rank 0 publishes each queue's (key, n, wave) and
    the other ranks check theirs against it, so ranks that disagree fail
    loudly instead of each running every cluster.  Without a store (one
    process) the counter is local."""

    _gen = 0

    def __init__(self, n: int, wave: int, store=None, prefix: str = "rifraf_cluster_queue", key=None,
                 rank: int = 0, timeout_s: float = 300.0):
        self.n, self.wave = int(n), max(1, int(wave))
        self.store = store
        self.rank = int(rank)
        self._local = 0
        self._lock = threading.Lock()
        if store is None:
            self.key = f"{prefix}/local" if key is None else str(key)
            return
        if key is None:
            ClusterQueue._gen += 1
            key = f"{prefix}/{ClusterQueue._gen}"
        self.key = str(key)
        desc = f"{self.key} n={self.n} wave={self.wave}"
        if self.rank == 0:
            store.set(self.key + "/desc", desc)
        else:
            import datetime
            try:
                store.wait([self.key + "/desc"], datetime.timedelta(seconds=timeout_s))
                got = store.get(self.key + "/desc").decode()
            except Exception as e:  # noqa: BLE001 -- reported as the queue mismatch it is
                raise RuntimeError(f"ClusterQueue: rank {self.rank} found no queue {self.key} published by "
                                   f"rank 0 ({e}); create queues in the same order on every rank or pass key=")
            if got != desc:
                raise RuntimeError(f"ClusterQueue: rank {self.rank} has '{desc}', rank 0 published '{got}'")

    @classmethod
    def for_process_group(cls, n: int, wave: int, key=None):
        """A queue on the default process group's store (every rank calls
        this in the same order, or with the same `key`), or a local one when
        no group is up."""
        store = None
        rank = 0
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                from torch.distributed import distributed_c10d
                store = distributed_c10d._get_default_store()
                rank = dist.get_rank()
        except Exception:  # noqa: BLE001 -- no process group: one process takes every wave
            store = None
        return cls(n, wave, store, key=key, rank=rank)

    def failed(self):
        """The rank that reported a failure on this queue, or None."""
        if self.store is None or not self.store.check([self.key + "/failed"]):
            return None
        return int(self.store.get(self.key + "/failed").decode())

    def fail(self):
        """Mark the queue failed (this rank raised): no rank takes more waves."""
        if self.store is not None:
            self.store.set(self.key + "/failed", str(self.rank))

    def take(self):
        """The next wave's cluster indices (a range), or None when the queue
        is empty (or a rank has failed)."""
        if self.store is not None:
            if self.failed() is not None:
                return None
            hi = int(self.store.add(self.key, self.wave))
        else:
            with self._lock:
                self._local += self.wave
                hi = self._local
        lo = hi - self.wave
        if lo >= self.n:
            return None
        return range(lo, min(hi, self.n))


def rifraf_batch_queue(get_cluster, queue: ClusterQueue, params=None, engine=None, engines=None,
                       init_exclusive: bool = False, setup_exclusive: bool = True, on_wave=None, stats=None,
                       **kw):
    """rifraf_batch over the waves this process takes from `queue` (a
    ClusterQueue shared by the ranks of a node): `get_cluster(i)` gives
    cluster i's keyword dict (e.g. read from its FASTQ file, as each `pmap`
    worker does).  Returns {cluster index: RifrafResult} for the clusters
    this rank ran; over all ranks every cluster runs exactly once, with the
    result rifraf() gives it alone (clusters are independent).

    engines: several engines of this process (e.g. two contexts on one GPU),
    one host thread each, every thread taking its own waves from the queue
    (init_exclusive: at most one of them in its native stage machine at a
    time; setup_exclusive: at most one in a wave's host setup, as in
    rifraf_batch).  `on_wave(r)` is called with each wave's
    range after it ran; `stats` (a dict) receives waves / clusters taken,
    the seconds spent running them and the seconds waited at the closing
    barrier.  With a store-backed queue every rank reaches that one barrier
    once the queue is empty, also when it failed (rank 0 hosts the store, so
    it must not tear the group down while another rank still takes waves):
    a rank that raises marks the queue failed so the others stop taking
    waves, and after the barrier the error is raised on it and a
    RuntimeError on every other rank."""
    import time
    from .model import RifrafParams
    params = params or RifrafParams()
    engs = list(engines) if engines else [engine]
    out = {}
    errs = []
    lock = threading.Lock()
    ilock = threading.Lock() if init_exclusive and len(engs) > 1 else None
    slock = threading.Lock() if setup_exclusive and len(engs) > 1 else None
    st = {"waves": 0, "clusters": 0, "busy_s": 0.0}

    def worker(e):
        try:
            while True:
                r = queue.take()
                if r is None:
                    return
                t0 = time.perf_counter()
                part = [get_cluster(i) for i in r]
                if (ilock is not None or slock is not None) and kw.get("native", None) is not False and \
                        native_eligible(part, params) and hasattr(e, "rifraf_batch_native"):
                    res = _wave_native(part, params, e, init_lock=ilock, device_qv=kw.get("device_qv", True),
                                       setup_lock=slock)
                else:
                    res = rifraf_batch(part, params=params, engine=e, wave=len(r), **kw)
                with lock:
                    out.update(zip(r, res))
                    st["waves"] += 1
                    st["clusters"] += len(r)
                    st["busy_s"] += time.perf_counter() - t0
                if on_wave is not None:
                    on_wave(r)
        except BaseException as ex:  # noqa: BLE001 -- re-raised below, after the barrier
            with lock:
                errs.append(ex)
            queue.fail()

    if len(engs) == 1:
        worker(engs[0])
    else:
        ts = [threading.Thread(target=worker, args=(e,), daemon=True) for e in engs]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    t0 = time.perf_counter()
    if queue.store is not None:
        import torch.distributed as dist
        dist.barrier()
    st["barrier_wait_s"] = time.perf_counter() - t0
    if stats is not None:
        stats.update(st)
    if errs:
        raise errs[0]
    bad = queue.failed()
    if bad is not None:
        raise RuntimeError(f"rifraf_batch_queue: rank {bad} failed; its waves did not complete")
    return out
