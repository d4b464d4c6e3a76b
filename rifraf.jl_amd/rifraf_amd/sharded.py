"""Read-sharded RIFRAF over the ranks of one node.

The reads of one cluster are independent for the banded DP (realign!,
model.jl:679-714) and for the per-read proposal scores (score_nocodon,
model.jl:242-285, seq_score_deletion :227-236).  The one exchange step is
the per-proposal sum over reads (score_proposal(m, state, newcols, use_ref),
model.jl:385-399), plus the per-read A[end,end] values that rescore! folds
(model.jl:630-635).

`ShardedEngine` is a drop-in for `engine.Engine` under the host stage
machine: every rank runs the same `rifraf(..., engine=ShardedEngine(...))`
call on the same inputs, and every method below is collective.

Ownership:
  - sequence tables and templates are replicated (uploaded on every rank);
  - read batch slots [0, nreads) are dealt round-robin: rank r owns the
    slots s with s % W == r, so the A/B bands of a slot live only on its
    owner and band memory is sharded;
  - slots >= nreads (the reference and scratch slots of model._Run) belong
    to the last rank.
  - rifraf() fills batch slots 0..B-1 (model.jl:569-573, :1038-1066) and
    check_score! can grow B by base_batch_size up to the read count
    (model.jl:1094-1112).  A round-robin deal is balanced for every prefix
    [0, B), so the work stays balanced (within one read per rank) as the
    batch grows, and no rank holds more than ceil(nreads / W) reads' bands.

Exchange and exactness:
  - realign / backtrace results are per job; they are gathered verbatim, so
    `rescore!`'s host fold is bit-identical to one GPU;
  - `score` (proposal lists: get_candidates, estimate_probs): each rank
    scores its own reads, one tensor all-gather collects every read's score
    column, and every rank folds them in batch order starting at 0.0, the
    reference last.  This is the reference's own summation order, so totals
    are bit-identical to one GPU (and to model.jl:389-397);
  - `score_dense` (all proposals of a cluster, the throughput path) has every
    rank fold its own reads on the device (rf_score_dense_dev), all-gathers
    the partial vectors over RCCL and sums them in rank order on the device.
    That regroups the sum, so it agrees with the single-GPU fold to
    <= (W-1)*eps*sum|s| (north_star tolerance: 1e-9 relative).
"""
from __future__ import annotations

import time

import numpy as np

from .engine import RF_BAND_A, RifrafError
from .proposals import to_arrays


class ShardedEngine:
    def __init__(self, local, nreads: int, group=None):
        import torch
        import torch.distributed as dist
        self.e = local
        self.nreads = int(nreads)
        self.group = group
        self.dist = dist
        self.torch = torch
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.dev = (torch.device("cuda", torch.cuda.current_device()) if backend == "nccl"
                    else torch.device("cpu"))
        self.last_dense = None
        # template lengths, and the template length each slot's bands were
        # last filled against (replicated: every rank sees every call)
        self.tlen, self.slot_m = {}, {}
        self.exchange_s, self.exchanges = 0.0, 0   # time in (and number of) collectives

    @classmethod
    def for_params(cls, local, nreads: int, params=None, group=None):
        """ShardedEngine for a rifraf() run over `nreads` reads.  Every batch
        size the run may reach (batch_size, grown by check_score! up to all
        reads) is balanced by the round-robin deal, so only the read count
        matters; `params` is accepted for call-site symmetry."""
        return cls(local, nreads, group)

    def slot_counts(self, slots) -> list:
        """Number of the given slots each rank owns (load-balance diagnostics)."""
        counts = [0] * self.world
        for s in np.asarray(slots).ravel():
            counts[self.owner(int(s))] += 1
        return counts

    # ------------------------------------------------------------------
    # ownership
    def owner(self, slot: int) -> int:
        slot = int(slot)
        if slot < 0:
            raise ValueError("negative slot")
        if slot >= self.nreads:
            return self.world - 1
        return slot % self.world

    def owned(self, slots) -> np.ndarray:
        return self.owned_by(self.rank, slots)

    # ------------------------------------------------------------------
    # collectives: fixed-shape tensors (RCCL on GPUs, gloo on CPU).  Every
    # rank knows which rank owns which job (the deal is deterministic) and
    # the shape of every result (template lengths are replicated), so one
    # all-gather or all-reduce per call carries the results, with an error
    # flag as the last element; error messages (Python objects) travel only
    # when a rank actually failed.
    def _timed(self, fn):
        t0 = time.perf_counter()
        out = fn()
        self.exchange_s += time.perf_counter() - t0
        self.exchanges += 1
        return out

    def _allgather(self, arr: np.ndarray, dtype) -> np.ndarray:
        """(W, len) array of every rank's 1-D `arr` (equal lengths)."""
        torch = self.torch

        def go():
            t = torch.from_numpy(np.ascontiguousarray(arr, dtype=dtype)).to(self.dev)
            if self.dev.type == "cuda":
                out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=self.dev)
                self.dist.all_gather_into_tensor(out, t, group=self.group)
                return out.view(self.world, -1).cpu().numpy()
            parts = [torch.empty_like(t) for _ in range(self.world)]
            self.dist.all_gather(parts, t, group=self.group)
            return torch.stack(parts).numpy()
        return self._timed(go)

    def _allreduce_max_u8(self, arr: np.ndarray) -> np.ndarray:
        torch = self.torch

        def go():
            t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.uint8)).to(self.dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
            return t.cpu().numpy()
        return self._timed(go)

    def _gather(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def _raise_first(self, err):
        """Slow path after a flagged collective: the error text of the first
        failing rank (in rank order) is raised on every rank."""
        for e in self._gather(err):
            if e is not None:
                raise RifrafError(e)
        raise RifrafError("sharded engine: a rank reported an error")

    def _raise_any(self, err):
        """Collective error check: a reference error() on any rank is raised on all."""
        flag = self._allreduce_max_u8(np.array([0 if err is None else 1], np.uint8))
        if flag[0]:
            self._raise_first(err)

    def _global(self, r: int) -> int:
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def owners(self, slots) -> np.ndarray:
        """Owner rank of every slot (vectorised owner())."""
        slots = np.asarray(slots, np.int64)
        return np.where(slots < self.nreads, slots % self.world, self.world - 1)

    def _rows(self, slot: int) -> int:
        """m + 1 for the template the slot's bands were last filled against
        (replicated bookkeeping: every rank sees every realign call).  The
        length is recorded at realign time, so a later set_templates of a
        different length cannot mis-shape the result buffer."""
        m = self.slot_m.get(int(slot))
        if m is None:
            raise RifrafError(f"slot {int(slot)} has no bands filled through this ShardedEngine "
                              "(realign it through the sharded engine first)")
        return m + 1

    # ------------------------------------------------------------------
    # replicated state
    def set_sequences(self, first, seqs):
        self.e.set_sequences(first, seqs)

    def set_templates(self, first, tpls):
        for k, t in enumerate(tpls):
            self.tlen[first + k] = len(t)
        self.e.set_templates(first, tpls)

    def reserve(self, nbytes):
        self.e.reserve(nbytes)

    def close(self):
        self.e.close()

    # ------------------------------------------------------------------
    def realign(self, slots, seqs, tpls, bws, flags) -> np.ndarray:
        """Each rank fills the bands of its own slots; per-job scores travel
        in one all-gather of n + 1 doubles (verbatim, so rescore!'s fold is
        exact)."""
        slots = np.atleast_1d(np.asarray(slots, np.int32))
        n = slots.shape[0]
        seqs = np.broadcast_to(np.asarray(seqs, np.int32), (n,))
        tpls = np.broadcast_to(np.asarray(tpls, np.int32), (n,))
        bws = np.broadcast_to(np.asarray(bws, np.int32), (n,))
        for sl, tp in zip(slots.tolist(), tpls.tolist()):
            if tp not in self.tlen:
                raise RifrafError(f"rf_realign: unknown template {tp}")
            self.slot_m[sl] = self.tlen[tp]
        mine = np.flatnonzero(self.owned(slots))
        err = None
        buf = np.zeros(n + 1)
        if len(mine):
            try:
                fl = flags if np.ndim(flags) == 0 else np.broadcast_to(np.asarray(flags), (n,))[mine]
                buf[mine] = self.e.realign(slots[mine], seqs[mine], tpls[mine], bws[mine], fl)
            except RifrafError as e:
                err = str(e)
        buf[n] = 0.0 if err is None else 1.0
        allv = self._allgather(buf, np.float64)
        if allv[:, n].any():
            self._raise_first(err)
        return allv[self.owners(slots), np.arange(n)]

    def backtrace(self, slots, want_moves: bool = True):
        """Error counts (and move lengths) in one all-gather; the moves, when
        wanted, in a second one of padded byte strings."""
        slots = np.atleast_1d(np.asarray(slots, np.int32))
        n = len(slots)
        mine = np.flatnonzero(self.owned(slots))
        err, mv = None, None
        head = np.zeros(2 * n + 1)
        if len(mine):
            try:
                mv, ne = self.e.backtrace(slots[mine], want_moves)
                head[mine] = ne
                if want_moves:
                    head[n + mine] = [len(x) for x in mv]
            except RifrafError as e:
                err = str(e)
        head[2 * n] = 0.0 if err is None else 1.0
        allh = self._allgather(head, np.float64)
        if allh[:, 2 * n].any():
            self._raise_first(err)
        own = self.owners(slots)
        nerr = allh[own, np.arange(n)].astype(np.int32)
        if not want_moves:
            return None, nerr
        lens = allh[own, n + np.arange(n)].astype(np.int64)
        per_rank = [int(lens[own == r].sum()) for r in range(self.world)]
        pay = np.zeros(max(max(per_rank), 1), np.int8)
        if mv is not None and len(mine):
            flat = np.concatenate([np.asarray(x, np.int8) for x in mv])
            pay[:len(flat)] = flat
        allm = self._allgather(pay, np.int8)
        moves = [None] * n
        at = [0] * self.world
        for i in range(n):
            r = int(own[i])
            moves[i] = allm[r, at[r]:at[r] + lens[i]].copy()
            at[r] += int(lens[i])
        return moves, nerr

    def alignment_proposals(self, groups, do_indels: bool):
        """Per-rank masks of the owned batch slots, OR-ed over the ranks by
        one byte-wise MAX all-reduce (the union is order-free, so the result
        equals one GPU's)."""
        rows = [self._rows(np.asarray(sl)[0]) for sl in groups]
        off = np.zeros(len(groups) + 1, np.int64)
        np.cumsum(np.asarray(rows, np.int64) * 9, out=off[1:])
        buf = np.zeros(int(off[-1]) + 1, np.uint8)
        err = None
        local = [(g, np.asarray(sl, np.int32)[self.owned(sl)]) for g, sl in enumerate(groups)]
        local = [(g, s) for g, s in local if len(s)]
        if local:
            try:
                res = self.e.alignment_proposals([s for _, s in local], do_indels)
                for (g, _), mk in zip(local, res):
                    buf[off[g]:off[g + 1]] = np.asarray(mk, np.uint8).reshape(-1)
            except RifrafError as e:
                err = str(e)
        buf[-1] = 0 if err is None else 1
        out = self._allreduce_max_u8(buf)
        if out[-1]:
            self._raise_first(err)
        return [out[off[g]:off[g + 1]].reshape(rows[g], 9).copy() for g in range(len(groups))]

    def geometry(self, slot: int, which: int = RF_BAND_A):
        src = self.owner(slot)
        obj = [self.e.geometry(slot, which) if self.rank == src else None]
        self.dist.broadcast_object_list(obj, src=self._global(src), group=self.group)
        return obj[0]

    def download_band(self, slot: int, which: int = RF_BAND_A, default=-np.inf):
        src = self.owner(slot)
        obj = [self.e.download_band(slot, which, default) if self.rank == src else None]
        self.dist.broadcast_object_list(obj, src=self._global(src), group=self.group)
        return obj[0]

    # ------------------------------------------------------------------
    def owned_by(self, rank: int, slots) -> np.ndarray:
        """Mask of the slots `rank` owns (the same rule as owned())."""
        slots = np.asarray(slots, np.int64)
        if slots.size == 0:
            return np.zeros(0, bool)
        reads = slots < self.nreads
        mine = reads & (slots % self.world == rank)
        if rank == self.world - 1:
            mine |= ~reads
        return mine

    def score(self, groups, per_seq: bool = False):
        """Proposal-list scoring (get_candidates, estimate_probs): every rank
        scores its own reads (and the reference when it owns the reference
        slot) against every proposal; ONE tensor all-gather (RCCL / gloo) of
        the padded per-read score matrices of all groups, with the error flag
        as the last element (every rank knows every rank's payload size from
        the deal); every rank then folds the columns in batch order,
        0.0 + s_1 + ... + s_R, and adds the reference last -- the reference's
        own order (model.jl:389-397), so the totals are bit-identical to one
        GPU."""
        arrs, local, err = [], [], None
        sizes = np.zeros(self.world, np.int64)
        for bslots, ref, props in groups:
            k, p, b = props if isinstance(props, tuple) else to_arrays(props)
            P = len(k)
            bslots = np.asarray(bslots, np.int32)
            own = self.owned(bslots)
            ref_owner = self.owner(ref) if ref >= 0 else -1
            mine_ref = ref_owner == self.rank
            cols = np.bincount(self.owners(bslots), minlength=self.world) if len(bslots) else \
                np.zeros(self.world, np.int64)
            if ref_owner >= 0:
                cols[ref_owner] += 1
            sizes += P * cols
            per = np.zeros((P, int(own.sum()) + (1 if mine_ref else 0)))
            if (own.any() or mine_ref) and P > 0 and err is None:
                try:
                    _, m = self.e.score([(bslots[own], ref if mine_ref else -1, (k, p, b))], per_seq=True)
                    per = np.asarray(m[0], np.float64).reshape(P, -1)
                except RifrafError as e:
                    err = str(e)
            arrs.append((P, bslots, ref, ref_owner))
            local.append(per)
        buf = np.zeros(int(sizes.max()) + 1)
        flat = np.concatenate([x.reshape(-1) for x in local]) if local else np.zeros(0)
        buf[:flat.size] = flat
        buf[-1] = 0.0 if err is None else 1.0
        parts = self._allgather(buf, np.float64)
        if parts[:, -1].any():
            self._raise_first(err)
        at = [0] * self.world
        totals, mats = [], []
        for P, bslots, ref, ref_owner in arrs:
            R = len(bslots)
            full = np.empty((P, R + (1 if ref >= 0 else 0)))
            own = self.owners(bslots)
            for r in range(self.world):
                idx = np.flatnonzero(own == r)
                cols = len(idx) + (1 if r == ref_owner else 0)
                m = parts[r][at[r]:at[r] + P * cols].reshape(P, cols)
                at[r] += P * cols
                full[:, idx] = m[:, :len(idx)]
                if r == ref_owner:
                    full[:, -1] = m[:, -1]
            acc = np.zeros(P)
            for j in range(full.shape[1]):
                acc = acc + full[:, j]
            totals.append(acc)
            mats.append(full)
        return (totals, mats) if per_seq else totals

    # ------------------------------------------------------------------
    def score_dense(self, groups, to_host: bool = True, rows=None):
        """All proposals of every group: per-rank device fold of the owned
        reads, RCCL all-gather of the partial vectors (an error count rides
        as the last element), rank-order sum."""
        torch = self.torch
        G = len(groups)
        if rows is None:
            rows = [self._rows(np.asarray(sl)[0]) for sl in groups]
        off = np.zeros(G + 1, np.int64)
        np.cumsum(np.asarray(rows, np.int64) * 9, out=off[1:])
        partial = torch.zeros(int(off[-1]) + 1, dtype=torch.float64, device=self.dev)
        local = [(g, np.asarray(sl, np.int32)[self.owned(sl)]) for g, sl in enumerate(groups)]
        local = [(g, s) for g, s in local if len(s)]
        err = None
        if local:
            try:
                if self.dev.type == "cuda":
                    lrows = int(sum(rows[g] for g, _ in local)) * 9
                    buf = partial if len(local) == G else torch.empty(lrows, dtype=torch.float64,
                                                                     device=self.dev)
                    self.e.score_dense_dev([s for _, s in local], buf.data_ptr())
                else:
                    res = self.e.score_dense([s for _, s in local], to_host=True,
                                             rows=[rows[g] for g, _ in local])
                    buf = torch.from_numpy(np.concatenate([np.asarray(r).reshape(-1) for r in res]))
                if buf is not partial:
                    at = 0
                    for g, _ in local:
                        w = rows[g] * 9
                        partial[off[g]:off[g] + w] = buf[at:at + w]
                        at += w
            except RifrafError as e:
                err = str(e)
        if err is not None:
            partial[-1] = 1.0
        total = self._timed(lambda: allgather_fold(partial, self.dist, self.group))
        if float(total[-1].item()) != 0.0:
            self._raise_first(err)
        total = total[:-1]
        self.last_dense = total
        if not to_host:
            return None
        host = total.cpu().numpy()
        return [host[off[g]:off[g + 1]].reshape(rows[g], 9) for g in range(G)]


def allgather_fold(partial, dist, group=None):
    """The read-sharded exchange step: all-gather every rank's partial
    per-proposal totals (RCCL all_gather_into_tensor over xGMI on GPUs, gloo
    on CPU) and sum them in rank order on the device."""
    import torch
    world = dist.get_world_size(group)
    if partial.is_cuda:
        out = torch.empty(world * partial.numel(), dtype=partial.dtype, device=partial.device)
        dist.all_gather_into_tensor(out, partial, group=group)
        return fold_partials(list(out.view(world, -1)))
    parts = [torch.empty_like(partial) for _ in range(world)]
    dist.all_gather(parts, partial, group=group)
    return fold_partials(parts)


def fold_partials(parts):
    """Rank-ordered sum of per-rank partial totals: ((P_0 + P_1) + P_2) + ...
    Deterministic for a given world size (no reduction-tree reordering)."""
    acc = parts[0].clone()
    for p in parts[1:]:
        acc += p
    return acc


def shard_bounds(nitems: int, world: int):
    """Contiguous block partition [lo_r, hi_r) used for slots and bench reads."""
    return [r * nitems // world for r in range(world + 1)]


__all__ = ["ShardedEngine", "allgather_fold", "fold_partials", "shard_bounds"]
