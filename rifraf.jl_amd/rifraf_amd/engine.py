"""Device engine: one HIP context (rf_ctx) of librifraf_hip.so.

Thin, typed wrapper over the C-ABI of include/rifraf_hip.h.  All numeric
work (DP fills, backtraces, proposal scoring) runs in the HIP kernels; this
module only marshals arrays.  There is no CPU fallback: a missing library or
GPU raises EngineUnavailable.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int64, byref, c_double, c_int32, c_void_p

import numpy as np

from . import _lib
from ._lib import RF_BAND_A, RF_BAND_B, RF_BWD, RF_ERR_NEED_HOST, RF_FWD, RF_SKEW, RF_TRIM, ptr
from .bandedarrays import BandedArray
from .proposals import to_arrays


class RifrafError(Exception):
    """A reference `error(...)` raised on the engine path (same message text)."""


class PackedGroups:
    """Batch-slot groups packed for rf_score_dense: slot_off (G+1, int32) and
    the concatenated slots (int32)."""
    __slots__ = ("n", "slot_off", "slots")

    def __init__(self, slot_off, slots):
        self.slot_off = np.ascontiguousarray(slot_off, np.int32)
        self.slots = np.ascontiguousarray(slots, np.int32)
        self.n = len(self.slot_off) - 1


def pack_groups(groups) -> PackedGroups:
    """Pack a list of batch-slot arrays (one per cluster) once."""
    G = len(groups)
    slot_off = np.zeros(G + 1, np.int32)
    if G:
        np.cumsum([len(s) for s in groups], out=slot_off[1:])
        slots = np.concatenate(groups).astype(np.int32, copy=False)
    else:
        slots = np.zeros(0, np.int32)
    return PackedGroups(slot_off, slots)


class Engine:
    """One device context.  Sequence ids, template ids and slot ids are small
    integers chosen by the caller (see model.py for the RIFRAF mapping)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = c_void_p()
        rc = self.lib.rf_create(int(device), byref(h))
        if rc != 0:
            raise _lib.EngineUnavailable(f"rf_create(device={device}) failed with {rc}: no HIP device?")
        self.ctx = h
        self.device = device

    # ------------------------------------------------------------------
    def close(self):
        if getattr(self, "ctx", None):
            self.lib.rf_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != 0:
            msg = self.lib.rf_last_error(self.ctx).decode()
            raise RifrafError(msg)

    # ------------------------------------------------------------------
    def set_option(self, name: str, value):
        """rf_set_option: select between bit-identical code paths (kernel
        variants, fused/split fold, ...).  Returns the previous value."""
        key = _lib.OPTIONS[name]
        if isinstance(value, str):
            value = _lib.OPTION_VALUES[name][value]
        old = self.get_option(name)
        self._check(self.lib.rf_set_option(self.ctx, key, int(value)))
        return old

    def get_option(self, name: str) -> int:
        v = c_int32()
        self._check(self.lib.rf_get_option(self.ctx, _lib.OPTIONS[name], byref(v)))
        return v.value

    def reserve(self, nbytes: int):
        self._check(self.lib.rf_reserve(self.ctx, int(nbytes)))

    def release_bands(self):
        """rf_release_bands: drop every slot's bands and reuse the band arena
        from its start (the memory stays allocated)."""
        self._check(self.lib.rf_release_bands(self.ctx))

    def device_bytes(self) -> int:
        return int(self.lib.rf_device_bytes(self.ctx))

    def code_stats(self) -> dict:
        """rf_code_stats: the row-code dictionary's size, the reads left
        uncoded because it was full, and its fresh starts."""
        v = [c_int64() for _ in range(4)]
        self._check(self.lib.rf_code_stats(self.ctx, *[byref(x) for x in v]))
        return dict(zip(("entries3", "entries1", "uncoded_reads", "resets"), (x.value for x in v)))

    def set_sequences(self, first: int, seqs):
        """Upload RifrafSequence tables for ids [first, first+len(seqs))."""
        if not seqs:
            return
        lens = np.array([len(s) for s in seqs], np.int64)
        if (lens < 1).any():
            raise ValueError("empty sequence")
        off = np.zeros(len(seqs) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        bases = np.ascontiguousarray(np.concatenate([s.seq for s in seqs]), np.uint8)
        match = np.ascontiguousarray(np.concatenate([s.match_scores for s in seqs]))
        mism = np.ascontiguousarray(np.concatenate([s.mismatch_scores for s in seqs]))
        ins = np.ascontiguousarray(np.concatenate([s.ins_scores for s in seqs]))
        dele = np.ascontiguousarray(np.concatenate([s.del_scores for s in seqs]))
        any_codon = any(s.do_codon_moves() for s in seqs)
        cins = cdel = cins_off = cdel_off = None
        if any_codon:
            ci = [np.asarray(s.codon_ins_scores, np.float64) for s in seqs]
            cd = [np.asarray(s.codon_del_scores, np.float64) for s in seqs]
            cins_off = np.zeros(len(seqs) + 1, np.int64)
            np.cumsum([len(x) for x in ci], out=cins_off[1:])
            cdel_off = np.zeros(len(seqs) + 1, np.int64)
            np.cumsum([len(x) for x in cd], out=cdel_off[1:])
            cins = np.ascontiguousarray(np.concatenate(ci + [np.zeros(1)]))
            cdel = np.ascontiguousarray(np.concatenate(cd + [np.zeros(1)]))
        self._check(self.lib.rf_set_sequences(
            self.ctx, int(first), len(seqs), ptr(bases), ptr(off), ptr(match), ptr(mism), ptr(ins),
            ptr(dele), ptr(cins), ptr(cins_off), ptr(cdel), ptr(cdel_off)))

    def set_sequences_concat(self, first: int, bases, off, match, mismatch, ins, dele):
        """rf_set_sequences from already concatenated tables (no codon moves):
        sequence k = bases / tables at off[k]..off[k+1], del at off[k]+k ..
        off[k+1]+k+1 (the layout RifrafSequence.many_concat returns)."""
        off = np.ascontiguousarray(off, np.int64)
        a = [np.ascontiguousarray(x, np.float64) for x in (match, mismatch, ins, dele)]
        bases = np.ascontiguousarray(bases, np.uint8)
        self._check(self.lib.rf_set_sequences(self.ctx, int(first), len(off) - 1, ptr(bases), ptr(off),
                                              *[ptr(x) for x in a], None, None, None, None))

    def set_sequences_codes(self, first: int, bases, off, codes, lp_table, match_table, scores, prep=None):
        """rf_set_sequences_codes: Phred-coded reads (no codon moves) with
        their tables built on the device from one byte per position.  False
        when the row-code dictionary is full (upload host tables instead).
        prep = (p10_table, grid): rf_set_sequences_codes_prep -- returns
        (est, ucode, tsum) per sequence (the native driver's setup values,
        computed on the device; rifrafsequences.RifrafSequence.many_coded)."""
        off = np.ascontiguousarray(off, np.int64)
        bases = np.ascontiguousarray(bases, np.uint8)
        codes = np.ascontiguousarray(codes, np.uint8)
        lp_t = np.ascontiguousarray(lp_table, np.float64)
        mt = np.ascontiguousarray(match_table, np.float64)
        if lp_t.shape != (256,) or mt.shape != (256,) or len(codes) != len(bases):
            raise ValueError("set_sequences_codes: 256-entry tables and one code per base")
        sc = (float(scores.mismatch), float(scores.insertion), float(scores.deletion))
        if prep is None:
            rc = self.lib.rf_set_sequences_codes(self.ctx, int(first), len(off) - 1, ptr(bases), ptr(off),
                                                 ptr(codes), ptr(lp_t), ptr(mt), *sc)
            out = True
        else:
            p10 = np.ascontiguousarray(prep[0], np.float64)
            grid = np.ascontiguousarray(prep[1], np.float64)
            if p10.shape != (256,) or grid.shape != (256, 256):
                raise ValueError("set_sequences_codes: prep = (256 values of 10^lp, 256 x 256 grid)")
            n = len(off) - 1
            est, tsum, ucode = np.empty(n), np.empty(n), np.empty(n, np.int32)
            rc = self.lib.rf_set_sequences_codes_prep(self.ctx, int(first), n, ptr(bases), ptr(off), ptr(codes),
                                                      ptr(lp_t), ptr(mt), *sc, ptr(p10), ptr(grid), ptr(est),
                                                      ptr(ucode), ptr(tsum))
            out = (est, ucode, tsum)
        if rc == -4:
            return False
        self._check(rc)
        return out

    def set_templates(self, first: int, tpls):
        if not tpls:
            return
        lens = np.array([len(t) for t in tpls], np.int64)
        off = np.zeros(len(tpls) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        bases = np.ascontiguousarray(np.concatenate([np.asarray(t, np.uint8) for t in tpls]), np.uint8)
        self._check(self.lib.rf_set_templates(self.ctx, int(first), len(tpls), ptr(bases), ptr(off)))

    def rifraf_batch_native(self, bparams, read_off, read_seq, read_len, threshold, fixed_off, fixed,
                            slot_base, tpl_id, cons, cons_off, ref=None):
        """rf_rifraf_batch(_ref) + rf_batch_fetch(_ref): the native lockstep
        stage machine over many clusters (rifraf_batch.cpp).  Returns one dict
        per cluster: consensus, score, iters, status, stages, stage_of,
        stage_iters, batch, error (and ref_bw, ref_score, n_ref_indel_mults);
        and the final bandwidth per read (negative once bandwidth_fixed).
        ref: None (no references) or a dict with "params"
        (_lib.BatchRefParams), "refs" (a _lib.BatchRef array, one per
        cluster), "bases" (uint8) and "cb" (a _lib.RefCallback)."""
        nclu = len(slot_base)
        c = lambda a, t: np.ascontiguousarray(a, t)   # noqa: E731
        read_off, read_seq, read_len = c(read_off, np.int32), c(read_seq, np.int32), c(read_len, np.int32)
        threshold = c(threshold, np.float64)
        fixed_off = c(fixed_off, np.int32) if fixed_off is not None else None
        fixed = c(fixed, np.int32) if fixed is not None else None
        slot_base, tpl_id = c(slot_base, np.int32), c(tpl_id, np.int32)
        cons, cons_off = c(cons, np.uint8), c(cons_off, np.int64)
        score = np.empty(max(nclu, 1))
        iters = np.empty(max(nclu, 1), np.int32)
        status = np.empty(max(nclu, 1), np.int32)
        length = np.empty(max(nclu, 1), np.int64)
        bw = np.empty(max(len(read_seq), 1), np.int32)
        if ref is None:
            self._check(self.lib.rf_rifraf_batch(self.ctx, nclu, byref(bparams), ptr(read_off), ptr(read_seq),
                                                 ptr(read_len), ptr(threshold), ptr(fixed_off), ptr(fixed),
                                                 ptr(slot_base), ptr(tpl_id), ptr(cons), ptr(cons_off),
                                                 ptr(score), ptr(iters), ptr(status), ptr(length), ptr(bw)))
        else:
            rb = np.ascontiguousarray(ref["bases"], np.uint8)
            self._check(self.lib.rf_rifraf_batch_ref(
                self.ctx, nclu, byref(bparams), byref(ref["params"]), ptr(read_off), ptr(read_seq),
                ptr(read_len), ptr(threshold), ptr(fixed_off), ptr(fixed), ptr(slot_base), ptr(tpl_id), ptr(cons),
                ptr(cons_off), ctypes.cast(ref["refs"], c_void_p), ptr(rb) if len(rb) else ptr(np.zeros(1, np.uint8)),
                ctypes.cast(ref["cb"], c_void_p), None, ptr(score), ptr(iters), ptr(status), ptr(length),
                ptr(bw)))
        out = []
        err = ctypes.create_string_buffer(512)
        try:
            for k in range(nclu):
                cs = np.empty(int(length[k]), np.uint8)
                slen = np.empty(max(int(iters[k]), 1), np.int64)
                sit = np.zeros(3, np.int32)
                sof = np.zeros(max(int(iters[k]), 1), np.int8)
                rbw, rsc, nmul, nb = ctypes.c_int32(0), ctypes.c_double(0.0), ctypes.c_int32(0), ctypes.c_int32(0)
                self._check(self.lib.rf_batch_fetch_ref(self.ctx, k, ptr(sit), ptr(sof), byref(rbw), byref(rsc),
                                                        byref(nmul), byref(nb)))
                batch = np.empty(max(int(read_off[k + 1] - read_off[k]), int(nb.value), 1), np.int32)
                self._check(self.lib.rf_batch_fetch(self.ctx, k, ptr(cs), ptr(slen), None, ptr(batch), err, 512))
                batch = batch[:int(nb.value)]
                st = np.empty(int(slen[:iters[k]].sum()), np.uint8)
                self._check(self.lib.rf_batch_fetch(self.ctx, k, None, None, ptr(st), None, None, 0))
                cut = np.cumsum(slen[:iters[k]])[:-1]
                out.append({"consensus": cs, "score": float(score[k]), "iters": int(iters[k]),
                            "status": int(status[k]), "stages": np.split(st, cut) if iters[k] else [],
                            "stage_of": sof[:int(iters[k])].tolist(), "stage_iters": sit.tolist(),
                            "ref_bw": int(rbw.value), "ref_score": float(rsc.value),
                            "n_ref_indel_mults": int(nmul.value),
                            "batch": batch.tolist(), "error": err.value.decode() if status[k] == 2 else None})
        finally:
            self.lib.rf_batch_release(self.ctx)
        return out, bw[:len(read_seq)]

    def aln_error_sums(self, groups, tlens, seqs):
        """rf_aln_error_sums: per group (slot list in batch order, consensus
        length, the slots' RifrafSequences) the (m, 4) base-distribution sums
        of alignment_error_probs before its normalisation."""
        keep = [(np.ascontiguousarray(s.seq, np.uint8), np.ascontiguousarray(s.match_scores, np.float64))
                for gs in seqs for s in gs]
        bptr = np.array([b.ctypes.data for b, _ in keep], np.uint64)
        mptr = np.array([m.ctypes.data for _, m in keep], np.uint64)
        slen = np.array([len(b) for b, _ in keep], np.int32)
        return self.aln_error_sums_ptr(groups, tlens, bptr, mptr, slen)

    def aln_error_sums_ptr(self, groups, tlens, bptr, mptr, slen):
        """aln_error_sums with the slots' read bases / match scores given as
        host addresses (uint64 arrays; the caller keeps the memory alive).
        With bptr / mptr None the sums are folded on the device when every
        read is row-coded; None is returned when the host fold is needed."""
        off = np.zeros(len(groups) + 1, np.int32)
        np.cumsum([len(g) for g in groups], out=off[1:])
        slots = np.ascontiguousarray(np.concatenate([np.asarray(g, np.int32) for g in groups])
                                     if groups else np.zeros(0, np.int32))
        bptr = None if bptr is None else np.ascontiguousarray(bptr, np.uint64)
        mptr = None if mptr is None else np.ascontiguousarray(mptr, np.uint64)
        slen = np.ascontiguousarray(slen, np.int32)
        tl = np.ascontiguousarray(tlens, np.int32)
        row = np.zeros(len(groups) + 1, np.int64)
        np.cumsum(tl, out=row[1:])
        out = np.empty((max(int(row[-1]), 1), 4))
        rc = self.lib.rf_aln_error_sums(self.ctx, len(groups), ptr(off), ptr(slots), ptr(tl),
                                        None if bptr is None else ptr(bptr), None if mptr is None else ptr(mptr),
                                        ptr(slen), ptr(out))
        if rc == RF_ERR_NEED_HOST and (bptr is None or mptr is None):
            return None      # the caller passes the host tables and calls again
        self._check(rc)
        return [out[row[g]:row[g + 1]] for g in range(len(groups))]

    def qv_probs(self, groups, tlens, scores):
        """The quality pass on the device (rf_qv_probs): dense totals, the
        alignment sums and estimate_probs' / alignment_error_probs'
        normalisations for every group, without the totals leaving the GPU.
        Returns (pos (M, 5), ins (M + K, 4), aln (M,), err (kind, group)) --
        the arrays rf_host_qv_prep / rf_host_qv_finish produce, with 10^x from
        the device's exp10 (within ~1e-15 relative, not bit for bit) -- or
        None when a read has no row codes (the host path then runs)."""
        off = np.zeros(len(groups) + 1, np.int32)
        np.cumsum([len(g) for g in groups], out=off[1:])
        slots = np.ascontiguousarray(np.concatenate([np.asarray(g, np.int32) for g in groups])
                                     if groups else np.zeros(0, np.int32))
        tl = np.ascontiguousarray(tlens, np.int32)
        sc = np.ascontiguousarray(scores, np.float64)
        M, K = int(tl.sum()), len(groups)
        pos, ins, aln = np.empty((M, 5)), np.empty((M + K, 4)), np.empty(M)
        err = np.zeros(2, np.int32)
        rc = self.lib.rf_qv_probs(self.ctx, K, ptr(off), ptr(slots), ptr(tl), ptr(sc), ptr(pos), ptr(ins),
                                  ptr(aln), ptr(err))
        if rc == 1:
            return None
        self._check(rc)
        return pos, ins, aln, err

    def realign(self, slots, seqs, tpls, bws, flags) -> np.ndarray:
        """Batched forward_moves!/backward! fill; returns A[end,end] (RF_FWD)
        or B[1,1] per job.  flags: one int for every job (rf_realign) or one
        per job (rf_realign_jobs: e.g. backward fills beside a skewed forward
        fill in one launch set)."""
        slots = np.ascontiguousarray(slots, np.int32)
        n = slots.shape[0]
        seqs = np.ascontiguousarray(np.broadcast_to(seqs, (n,)), np.int32)
        tpls = np.ascontiguousarray(np.broadcast_to(tpls, (n,)), np.int32)
        bws = np.ascontiguousarray(np.broadcast_to(bws, (n,)), np.int32)
        out = np.empty(max(n, 1))
        if np.ndim(flags) == 0:
            self._check(self.lib.rf_realign(self.ctx, n, ptr(slots), ptr(seqs), ptr(tpls), ptr(bws),
                                            int(flags), ptr(out)))
        else:
            fl = np.ascontiguousarray(np.broadcast_to(flags, (n,)), np.int32)
            self._check(self.lib.rf_realign_jobs(self.ctx, n, ptr(slots), ptr(seqs), ptr(tpls), ptr(bws),
                                                 ptr(fl), ptr(out)))
        return out[:n]

    def backtrace(self, slots, want_moves: bool = True):
        """backtrace + count_errors of each slot's A band.
        Returns (list of int8 move arrays in alignment order, nerrors)."""
        slots = np.ascontiguousarray(slots, np.int32)
        n = slots.shape[0]
        nmoves = np.empty(max(n, 1), np.int32)
        nerr = np.empty(max(n, 1), np.int32)
        if want_moves:
            caps = np.empty(n, np.int64)
            for k, s in enumerate(slots):
                nrows, ncols, _, _ = self.geometry(int(s), RF_BAND_A)
                caps[k] = nrows + ncols - 2
            moves_off = np.zeros(n + 1, np.int64)
            np.cumsum(caps, out=moves_off[1:])
            moves = np.empty(max(int(moves_off[-1]), 1), np.int8)
            self._check(self.lib.rf_backtrace(self.ctx, n, ptr(slots), ptr(moves), ptr(moves_off),
                                              ptr(nmoves), ptr(nerr)))
            out = [moves[moves_off[k]:moves_off[k] + nmoves[k]].copy() for k in range(n)]
            return out, nerr[:n].copy()
        self._check(self.lib.rf_backtrace(self.ctx, n, ptr(slots), None, None, ptr(nmoves), ptr(nerr)))
        return None, nerr[:n].copy()

    def alignment_proposals(self, groups, do_indels: bool):
        """rf_alignment_proposals: per group (batch slots of one cluster) the
        (m+1, 9) 0/1 mask of the proposals its alignments imply."""
        G = len(groups)
        slot_off = np.zeros(G + 1, np.int32)
        for g, sl in enumerate(groups):
            slot_off[g + 1] = slot_off[g] + len(sl)
        slots = np.ascontiguousarray(np.concatenate([np.asarray(s, np.int32) for s in groups]), np.int32)
        rows = [self.geometry(int(sl[0]), RF_BAND_A)[1] for sl in groups]
        out = np.zeros(max(int(sum(rows)) * 9, 1), np.uint8)
        self._check(self.lib.rf_alignment_proposals(self.ctx, G, ptr(slot_off), ptr(slots), int(bool(do_indels)),
                                                    ptr(out)))
        res, at = [], 0
        for r in rows:
            res.append(out[at * 9:(at + r) * 9].reshape(r, 9))
            at += r
        return res

    def score(self, groups, per_seq: bool = False):
        """Score proposals.  groups: list of (batch_slots, ref_slot, proposals)
        with ref_slot = -1 for none.  Returns a list of total arrays (and of
        per-sequence matrices if per_seq)."""
        G = len(groups)
        slot_off = np.zeros(G + 1, np.int32)
        prop_off = np.zeros(G + 1, np.int64)
        all_slots, refs, ks, ps, bs = [], np.empty(G, np.int32), [], [], []
        widths = []
        for g, (bslots, ref, props) in enumerate(groups):
            bslots = np.asarray(bslots, np.int32)
            all_slots.append(bslots)
            slot_off[g + 1] = slot_off[g] + len(bslots)
            refs[g] = ref
            if isinstance(props, tuple):
                k, p, b = props
            else:
                k, p, b = to_arrays(props)
            ks.append(k)
            ps.append(p)
            bs.append(b)
            prop_off[g + 1] = prop_off[g] + len(k)
            widths.append(len(bslots) + (1 if ref >= 0 else 0))
        slots = np.ascontiguousarray(np.concatenate(all_slots) if all_slots else np.zeros(1, np.int32), np.int32)
        kind = np.ascontiguousarray(np.concatenate(ks) if ks else np.zeros(0), np.uint8)
        pos = np.ascontiguousarray(np.concatenate(ps) if ps else np.zeros(0), np.int32)
        base = np.ascontiguousarray(np.concatenate(bs) if bs else np.zeros(0), np.uint8)
        nprops = int(prop_off[-1])
        total = np.empty(max(nprops, 1))
        per = None
        if per_seq:
            per = np.empty(max(int(sum(w * (prop_off[g + 1] - prop_off[g]) for g, w in enumerate(widths))), 1))
        self._check(self.lib.rf_score(self.ctx, G, ptr(slot_off), ptr(slots), ptr(refs), ptr(prop_off),
                                      ptr(kind) if nprops else None, ptr(pos) if nprops else None,
                                      ptr(base) if nprops else None, ptr(total), ptr(per)))
        totals = [total[prop_off[g]:prop_off[g + 1]].copy() for g in range(G)]
        if not per_seq:
            return totals
        mats, at = [], 0
        for g, w in enumerate(widths):
            cnt = int(prop_off[g + 1] - prop_off[g])
            mats.append(per[at:at + cnt * w].reshape(cnt, w).copy())
            at += cnt * w
        return totals, mats

    def score_dense(self, groups, to_host: bool = True, rows=None):
        """Dense all-proposals scoring (rf_score_dense).  groups: list of
        batch-slot arrays (one per cluster), or the PackedGroups of
        pack_groups(list) when the same groups are scored repeatedly.
        Returns a list of (m_g+1, 9) arrays (or None when to_host is False:
        totals stay in HBM)."""
        pg = groups if isinstance(groups, PackedGroups) else pack_groups(groups)
        G, slot_off, slots = pg.n, pg.slot_off, pg.slots
        groups = pg
        if not to_host:
            self._check(self.lib.rf_score_dense(self.ctx, G, ptr(slot_off), ptr(slots), None))
            return None
        if rows is None:
            # B: computed on both paths (RF_OPT_SCORE_FWD scores without A)
            rows = [self.geometry(int(slots[slot_off[g]]), RF_BAND_B)[1] for g in range(G)]
        out = np.empty((int(sum(rows)), 9))
        self._check(self.lib.rf_score_dense(self.ctx, G, ptr(slot_off), ptr(slots), ptr(out)))
        res, at = [], 0
        for r in rows:
            res.append(out[at:at + r])
            at += r
        return res

    def score_dense_dev(self, groups, dev_ptr: int):
        """rf_score_dense_dev: dense totals written to device memory at
        dev_ptr (sum_g (m_g+1)*9 doubles on this engine's device)."""
        pg = groups if isinstance(groups, PackedGroups) else pack_groups(groups)
        G, slot_off, slots = pg.n, pg.slot_off, pg.slots
        self._check(self.lib.rf_score_dense_dev(self.ctx, G, ptr(slot_off), ptr(slots), c_void_p(int(dev_ptr))))

    def geometry(self, slot: int, which: int = RF_BAND_A):
        nr, nc, bw, H = c_int32(), c_int32(), c_int32(), c_int32()
        self._check(self.lib.rf_slot_geometry(self.ctx, int(slot), int(which), byref(nr), byref(nc),
                                              byref(bw), byref(H)))
        return nr.value, nc.value, bw.value, H.value

    def download_band(self, slot: int, which: int = RF_BAND_A, default=-np.inf) -> BandedArray:
        nrows, ncols, bw, H = self.geometry(slot, which)
        buf = np.empty(H * ncols)
        self._check(self.lib.rf_download_band(self.ctx, int(slot), int(which), ptr(buf)))
        data = np.asfortranarray(buf.reshape(ncols, H).T)
        return BandedArray((nrows, ncols), bw, default=default, data=data)

    def last_backtrace_ms(self) -> float:
        """Kernel ms of the last backtrace / alignment_proposals call."""
        v = c_double()
        self._check(self.lib.rf_last_backtrace_ms(self.ctx, byref(v)))
        return v.value

    def last_codon_ms(self) -> float:
        """k_codon ms of the last score call (the reference's codon moves)."""
        v = c_double()
        self._check(self.lib.rf_last_codon_ms(self.ctx, byref(v)))
        return v.value

    def last_timing(self):
        a, b, c = c_double(), c_double(), c_double()
        self._check(self.lib.rf_last_timing(self.ctx, byref(a), byref(b), byref(c)))
        return a.value, b.value, c.value


__all__ = ["Engine", "RifrafError", "RF_FWD", "RF_BWD", "RF_SKEW", "RF_TRIM", "RF_BAND_A", "RF_BAND_B"]
