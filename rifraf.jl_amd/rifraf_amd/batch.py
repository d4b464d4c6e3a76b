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

import threading
import time

import numpy as np

from .engine import RifrafError
from .proposals import to_arrays


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
        return self.hub.call(self.k, "realign", slots, seqs, tpls, bws, flags)

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


STATS = {"launches": 0, "engine_s": 0.0}


def rifraf_batch(clusters, params=None, engine=None, wave: int = 1024):
    """rifraf() over many independent clusters, batched on one engine.

    clusters: sequence of dicts with the keyword arguments of model.rifraf
    (`dnaseqs`, `phreds` or `error_log_ps`, optional `consensus`,
    `reference`).  Returns the list of RifrafResult in input order (an
    exception raised by a cluster is re-raised after the wave finishes).
    Clusters run in waves of at most `wave` (their bands share the device)."""
    import os
    from .model import RifrafParams, rifraf
    params = params or RifrafParams()
    profile_dir = os.environ.get("RIFRAF_BATCH_PROFILE")
    if engine is None:
        from .align import default_engine
        engine = default_engine()
    results = [None] * len(clusters)
    for w0 in range(0, len(clusters), wave):
        part = clusters[w0:w0 + wave]
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
        STATS["launches"] += hub.launches
        STATS["engine_s"] += hub.engine_s
        for e in errors:
            if e is not None:
                raise e
    return results


__all__ = ["rifraf_batch", "ClusterEngine"]
