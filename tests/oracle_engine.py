"""CPU stand-in for rifraf_amd.engine.Engine built on the oracle.

TEST INFRASTRUCTURE ONLY: lets the host stage machine (rifraf_amd.model)
run end to end on CPU, and gives GPU-vs-oracle whole-run comparisons.  Same
method signatures and semantics as Engine (slots own A/B bands, forward
flags, left-fold scoring)."""
import copy
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle
from rifraf_amd.bandedarrays import BandedArray
from rifraf_amd.engine import RF_BAND_A, RF_BWD, RF_FWD, RF_SKEW, RF_TRIM, RifrafError
from rifraf_amd.proposals import to_arrays


# host threads for the oracle's C calls (ctypes releases the GIL): the GPU
# box grants 16 cores of a much larger machine
NTHREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))))


class OracleEngine:
    def __init__(self):
        self.seqs, self.tpls, self.slots = {}, {}, {}
        self.version = 0

    def close(self):
        pass

    def set_sequences(self, first, seqs):
        for k, s in enumerate(seqs):
            self.seqs[first + k] = copy.copy(s)

    def set_templates(self, first, tpls):
        for k, t in enumerate(tpls):
            self.version += 1
            self.tpls[first + k] = (np.asarray(t, np.uint8).copy(), self.version)

    def realign(self, slots, seqs, tpls, bws, flags):
        slots = np.atleast_1d(np.asarray(slots, np.int32))
        n = len(slots)
        seqs = np.broadcast_to(seqs, (n,))
        tpls = np.broadcast_to(tpls, (n,))
        bws = np.broadcast_to(bws, (n,))
        fl = np.broadcast_to(np.asarray(flags, np.int64), (n,))   # one value, or one per job (rf_realign_jobs)
        out = np.empty(n)
        for k in range(n):
            if int(bws[k]) < 1:
                raise RifrafError("bandwidth must be positive")

        def one(k):
            flags = int(fl[k])
            s = self.seqs[int(seqs[k])]
            t, ver = self.tpls[int(tpls[k])]
            bw = int(bws[k])
            key = (int(seqs[k]), int(tpls[k]), ver, bw)
            A = B = None
            try:
                if flags & RF_FWD:
                    A = oracle.forward(t, s, moves=True, skew=bool(flags & RF_SKEW),
                                       trim=bool(flags & RF_TRIM), bandwidth=bw)
                if flags & RF_BWD:
                    B = oracle.backward(t, s, bandwidth=bw)
            except oracle.OracleError as e:
                return RifrafError(str(e))
            return key, len(s), len(t), A, B

        if n >= 32 and NTHREADS > 1:
            with ThreadPoolExecutor(NTHREADS) as ex:
                res = list(ex.map(one, range(n)))
        else:
            res = [one(k) for k in range(n)]
        for k, r in enumerate(res):     # in job order: the first error wins, as in a serial loop
            if isinstance(r, RifrafError):
                raise r
            key, ns, nt, A, B = r
            ent = self.slots.setdefault(int(slots[k]), {})
            if A is not None:
                ent["A"] = (A[0], A[1], key, ns, nt)
            if B is not None:
                ent["B"] = (B, None, key, ns, nt)
            bw = key[3]
            flags = int(fl[k])
            data = ent["A"][0] if flags & RF_FWD else ent["B"][0]
            if flags & RF_FWD:
                out[k] = data[ns - nt + max(nt - ns, 0) + bw, nt]
            else:
                out[k] = data[max(nt - ns, 0) + bw, 0]
        return out

    def backtrace(self, slots, want_moves=True):
        def one(sl):
            A, mv, key, n, m = self.slots[int(sl)]["A"]
            moves = oracle.backtrace(mv, n + 1, m + 1, key[3])
            t = self.tpls[key[1]][0]
            s = self.seqs[key[0]]
            return moves, oracle.count_errors(moves, t, s.seq)
        sl = np.atleast_1d(slots)
        if len(sl) >= 32 and NTHREADS > 1:
            with ThreadPoolExecutor(NTHREADS) as ex:
                res = list(ex.map(one, sl))
        else:
            res = [one(x) for x in sl]
        mvs = [r[0] for r in res]
        errs = [r[1] for r in res]
        return (mvs if want_moves else None), np.array(errs, np.int32)

    def _check_slot(self, sl):
        ent = self.slots.get(int(sl), {})
        if "A" not in ent or "B" not in ent or ent["A"][2] != ent["B"][2]:
            raise RifrafError("A and B bands were computed for different alignments")
        return ent

    def score(self, groups, per_seq=False):
        """model.jl:385-399 per proposal (oracle.score_list: the same
        per-proposal left fold, proposals in parallel in C)."""
        totals, mats = [], []
        for bslots, ref, props in groups:
            k, p, b = props if isinstance(props, tuple) else to_arrays(props)
            ents = [self._check_slot(s) for s in bslots]
            reads = [self._seq_bw(e) for e in ents]
            rent = self._check_slot(ref) if ref >= 0 else None
            t = reads[0][1] if reads else None
            kw = {}
            if rent is not None:
                rs, t = self._seq_bw(rent)
                kw = dict(Aref=rent["A"][0], Bref=rent["B"][0], ref=rs)
            if len(k) == 0:
                totals.append(np.zeros(0))
                mats.append(np.zeros((0, len(ents) + (1 if rent else 0))))
                continue
            try:
                tot, mat = oracle.score_list((k, p, b), [e["A"][0] for e in ents], [e["B"][0] for e in ents],
                                             [s for s, _ in reads], t, per_seq=True, nthreads=NTHREADS, **kw)
            except oracle.OracleError as e:
                raise RifrafError(str(e))
            totals.append(tot)
            mats.append(mat)
        return (totals, mats) if per_seq else totals

    @staticmethod
    def _score1(kind, pos, base, A, B, t, s):
        try:
            return oracle.score_proposal(int(kind), int(pos), int(base), A, B, t, s)
        except oracle.OracleError as e:
            raise RifrafError(str(e))

    def _seq_bw(self, ent):
        key = ent["A"][2]
        s = copy.copy(self.seqs[key[0]])
        s.bandwidth = key[3]
        return s, self.tpls[key[1]][0]

    def geometry(self, slot, which=RF_BAND_A):
        A, mv, key, n, m = self.slots[int(slot)]["A" if which == RF_BAND_A else "B"]
        return n + 1, m + 1, key[3], A.shape[0]

    def download_band(self, slot, which=RF_BAND_A, default=-np.inf):
        data, _, key, n, m = self.slots[int(slot)]["A" if which == RF_BAND_A else "B"]
        return BandedArray((n + 1, m + 1), key[3], default=default, data=np.asfortranarray(data))

    def score_dense(self, groups, to_host=True, rows=None):
        """rf_score_dense on the oracle: all STAGE_SCORE proposals, (m+1, 9)
        totals per group (oracle.cpu_pass refills the bands itself)."""
        res = []
        for sl in groups:
            sb = [self._seq_bw(self._check_slot(s)) for s in sl]
            tot, _ = oracle.cpu_pass(sb[0][1], [s for s, _ in sb], nthreads=NTHREADS)
            res.append(tot)
        return res if to_host else None

    def alignment_proposals(self, groups, do_indels):
        """rf_alignment_proposals on the oracle: dense (m+1, 9) masks."""
        from rifraf_amd.align import moves_to_proposals_np
        out = []
        for sl in groups:
            moves, _ = self.backtrace(sl)
            m = self.slots[int(sl[0])]["A"][4]
            mask = np.zeros((m + 1, 9), np.uint8)
            for s, mv in zip(sl, moves):
                key = self.slots[int(s)]["A"][2]
                k, p, b = moves_to_proposals_np(mv, self.tpls[key[1]][0], self.seqs[key[0]].seq)
                if not do_indels:
                    keep = k == 0
                    k, p, b = k[keep], p[keep], b[keep]
                col = np.where(k == 0, b, np.where(k == 2, 4, 5 + b))
                mask[p, col] = 1
            out.append(mask)
        return out
