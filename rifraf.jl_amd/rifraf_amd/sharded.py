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
    # collectives
    def _gather(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def _raise_any(self, err):
        """Collective error check: a reference error() on any rank is raised on all."""
        errs = self._gather(err)
        for e in errs:
            if e is not None:
                raise RifrafError(e)

    def _global(self, r: int) -> int:
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    # ------------------------------------------------------------------
    # replicated state
    def set_sequences(self, first, seqs):
        self.e.set_sequences(first, seqs)

    def set_templates(self, first, tpls):
        self.e.set_templates(first, tpls)

    def reserve(self, nbytes):
        self.e.reserve(nbytes)

    def close(self):
        self.e.close()

    # ------------------------------------------------------------------
    def realign(self, slots, seqs, tpls, bws, flags: int) -> np.ndarray:
        """Each rank fills the bands of its own slots; per-job scores are
        gathered verbatim (exact)."""
        slots = np.atleast_1d(np.asarray(slots, np.int32))
        n = slots.shape[0]
        seqs = np.broadcast_to(np.asarray(seqs, np.int32), (n,))
        tpls = np.broadcast_to(np.asarray(tpls, np.int32), (n,))
        bws = np.broadcast_to(np.asarray(bws, np.int32), (n,))
        mine = np.flatnonzero(self.owned(slots))
        err, vals = None, None
        if len(mine):
            try:
                vals = self.e.realign(slots[mine], seqs[mine], tpls[mine], bws[mine], flags)
            except RifrafError as e:
                err = str(e)
        parts = self._gather((err, mine, vals))
        out = np.empty(n)
        for e, idx, v in parts:
            if e is not None:
                raise RifrafError(e)
            if v is not None:
                out[idx] = v
        return out

    def backtrace(self, slots, want_moves: bool = True):
        slots = np.atleast_1d(np.asarray(slots, np.int32))
        mine = np.flatnonzero(self.owned(slots))
        err, mv, ne = None, None, None
        if len(mine):
            try:
                mv, ne = self.e.backtrace(slots[mine], want_moves)
            except RifrafError as e:
                err = str(e)
        parts = self._gather((err, mine, mv, ne))
        nerr = np.empty(len(slots), np.int32)
        moves = [None] * len(slots) if want_moves else None
        for e, idx, m, c in parts:
            if e is not None:
                raise RifrafError(e)
            if c is None:
                continue
            nerr[idx] = c
            if want_moves:
                for k, i in enumerate(idx):
                    moves[i] = m[k]
        return moves, nerr

    def alignment_proposals(self, groups, do_indels: bool):
        """Per-rank masks of the owned batch slots, OR-ed over the ranks (the
        union is order-free, so the result equals one GPU's)."""
        err, masks = None, {}
        local = [(g, np.asarray(sl, np.int32)[self.owned(sl)]) for g, sl in enumerate(groups)]
        local = [(g, s) for g, s in local if len(s)]
        if local:
            try:
                res = self.e.alignment_proposals([s for _, s in local], do_indels)
                masks = {g: m for (g, _), m in zip(local, res)}
            except RifrafError as e:
                err = str(e)
        parts = self._gather((err, masks))
        out = [None] * len(groups)
        for e, ms in parts:
            if e is not None:
                raise RifrafError(e)
            for g, m in ms.items():
                out[g] = m.copy() if out[g] is None else (out[g] | m)
        return out

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
        the padded per-read score matrices of all groups; every rank then
        folds the columns in batch order, 0.0 + s_1 + ... + s_R, and adds the
        reference last -- the reference's own order (model.jl:389-397), so the
        totals are bit-identical to one GPU.  Three collectives per call
        (errors, lengths, scores), whatever the world size and group count."""
        torch = self.torch
        arrs, local, err = [], [], None
        for bslots, ref, props in groups:
            k, p, b = props if isinstance(props, tuple) else to_arrays(props)
            P = len(k)
            bslots = np.asarray(bslots, np.int32)
            own = self.owned(bslots)
            mine_ref = ref >= 0 and self.owner(ref) == self.rank
            per = np.zeros((P, int(own.sum()) + (1 if mine_ref else 0)))
            if (own.any() or mine_ref) and P > 0 and err is None:
                try:
                    _, m = self.e.score([(bslots[own], ref if mine_ref else -1, (k, p, b))], per_seq=True)
                    per = np.asarray(m[0], np.float64).reshape(P, -1)
                except RifrafError as e:
                    err = str(e)
            arrs.append((P, bslots, ref))
            local.append(per)
        self._raise_any(err)
        flat = np.concatenate([x.reshape(-1) for x in local]) if local else np.zeros(0)
        n = torch.tensor([flat.size], dtype=torch.int64, device=self.dev)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(ns, n, group=self.group)
        ns = [int(x.item()) for x in ns]
        buf = torch.zeros(max(max(ns), 1), dtype=torch.float64, device=self.dev)
        buf[:flat.size] = torch.from_numpy(flat).to(self.dev)
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        self.dist.all_gather(parts, buf, group=self.group)
        parts = [x.cpu().numpy() for x in parts]
        at = [0] * self.world
        totals, mats = [], []
        for P, bslots, ref in arrs:
            R = len(bslots)
            full = np.empty((P, R + (1 if ref >= 0 else 0)))
            ref_owner = self.owner(ref) if ref >= 0 else -1
            for r in range(self.world):
                idx = np.flatnonzero(self.owned_by(r, bslots))
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
        reads, RCCL all-gather of the partial vectors, rank-order sum."""
        torch = self.torch
        G = len(groups)
        if rows is None:
            rows = self._gather([self.e.geometry(int(s), RF_BAND_A)[1] if self.owned([s])[0] else None
                                 for s in (np.asarray(sl)[0] for sl in groups)])
            rows = [next(r[g] for r in rows if r[g] is not None) for g in range(G)]
        off = np.zeros(G + 1, np.int64)
        np.cumsum(np.asarray(rows, np.int64) * 9, out=off[1:])
        partial = torch.zeros(int(off[-1]), dtype=torch.float64, device=self.dev)
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
        self._raise_any(err)
        total = allgather_fold(partial, self.dist, self.group)
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
