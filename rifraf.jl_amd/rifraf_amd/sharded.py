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
  - batch slots [0, nslots) are split into contiguous blocks, one per rank
    (rank r owns [r*nslots//W, (r+1)*nslots//W)); the A/B bands of a slot
    live only on its owner, so band memory is sharded;
  - slots >= nslots (the reference and scratch slots of model._Run) belong
    to the last rank.
  - `nslots` must be the batch size the run actually uses (rifraf() fills
    batch slots 0..batch_size-1, model.jl:569-573 / :1038-1066), not the
    read count: `ShardedEngine.for_params` derives it from RifrafParams.  A
    block partition over the read count would put every batch slot of a
    20-read batch on rank 0.  The work is then balanced whenever the batch
    holds >= W reads (REFINE / SCORE, and every stage with batch_size <= 1,
    the throughput setting of configs 2-5); the fixed 5-read INIT/FRAME
    batch (batch_fixed_size) is spread over min(W, 5)-ish ranks only.

Exchange and exactness:
  - realign / backtrace results are per job; they are gathered verbatim, so
    `rescore!`'s host fold is bit-identical to one GPU;
  - `score` (proposal lists: get_candidates, estimate_probs) continues ONE
    left fold along the ranks: rank 0 starts at 0.0, adds its reads' scores
    in batch order and hands the running P-vector to rank 1, and so on; the
    reference is added last.  This is the reference's own summation order,
    so totals are bit-identical to one GPU (and to model.jl:389-397);
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
    def __init__(self, local, nslots: int, group=None):
        import torch
        import torch.distributed as dist
        self.e = local
        self.nslots = int(nslots)
        self.group = group
        self.dist = dist
        self.torch = torch
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.dev = (torch.device("cuda", torch.cuda.current_device()) if backend == "nccl"
                    else torch.device("cpu"))
        self.bounds = [r * self.nslots // self.world for r in range(self.world + 1)]
        self.last_dense = None

    @classmethod
    def for_params(cls, local, nreads: int, params=None, group=None):
        """ShardedEngine sized for the batch rifraf() will use: batch_size
        (all reads when batch_size <= 1, model.jl:569-573), capped at nreads."""
        bs = getattr(params, "batch_size", 0) if params is not None else 0
        nslots = nreads if bs <= 1 else min(bs, nreads)
        return cls(local, nslots, group)

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
        if slot >= self.nslots:
            return self.world - 1
        return int(np.searchsorted(self.bounds, slot, side="right")) - 1

    def owned(self, slots) -> np.ndarray:
        slots = np.asarray(slots, np.int64)
        if slots.size == 0:
            return np.zeros(0, bool)
        lo, hi = self.bounds[self.rank], self.bounds[self.rank + 1]
        mine = (slots >= lo) & (slots < hi)
        if self.rank == self.world - 1:
            mine |= slots >= self.nslots
        return mine

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

    def _send(self, vec: np.ndarray, dst: int):
        self.dist.send(self.torch.from_numpy(np.ascontiguousarray(vec)).to(self.dev),
                       dst=self._global(dst), group=self.group)

    def _recv(self, n: int, src: int) -> np.ndarray:
        t = self.torch.empty(n, dtype=self.torch.float64, device=self.dev)
        self.dist.recv(t, src=self._global(src), group=self.group)
        return t.cpu().numpy()

    def _bcast(self, vec, src: int, n: int) -> np.ndarray:
        t = (self.torch.from_numpy(np.ascontiguousarray(vec)).to(self.dev) if self.rank == src
             else self.torch.empty(n, dtype=self.torch.float64, device=self.dev))
        self.dist.broadcast(t, src=self._global(src), group=self.group)
        return t.cpu().numpy()

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
    def score(self, groups, per_seq: bool = False):
        """Proposal-list scoring with the reference's exact left fold carried
        from rank to rank (see the module docstring)."""
        totals, mats = [], []
        for bslots, ref, props in groups:
            k, p, b = props if isinstance(props, tuple) else to_arrays(props)
            P = len(k)
            bslots = np.asarray(bslots, np.int32)
            own = self.owned(bslots)
            mine_ref = ref >= 0 and self.owner(ref) == self.rank
            err, per = None, np.zeros((P, int(own.sum()) + (1 if mine_ref else 0)))
            if (own.any() or mine_ref) and P > 0:
                try:
                    _, m = self.e.score([(bslots[own], ref if mine_ref else -1, (k, p, b))], per_seq=True)
                    per = m[0]
                except RifrafError as e:
                    err = str(e)
            self._raise_any(err)
            n_own = int(own.sum())
            owners = [self.owner(s) for s in bslots]
            chain = all(a <= c for a, c in zip(owners, owners[1:]))
            if per_seq or not chain or P == 0:
                # gather every column and fold in batch order on every rank
                parts = self._gather((np.flatnonzero(own), per))
                full = np.empty((P, len(bslots) + (1 if ref >= 0 else 0)))
                for idx, m in parts:
                    full[:, idx] = m[:, :len(idx)]
                    if m.shape[1] > len(idx):
                        full[:, -1] = m[:, -1]
                acc = np.zeros(P)
                for j in range(full.shape[1]):
                    acc = acc + full[:, j]
                totals.append(acc)
                mats.append(full)
                continue
            # chain: ranks in order continue one left fold; the reference is last
            acc = np.zeros(P) if self.rank == 0 else self._recv(P, self.rank - 1)
            for j in range(n_own):
                acc = acc + per[:, j]
            last = self.world - 1
            ref_owner = self.owner(ref) if ref >= 0 else last
            if self.rank < last:
                self._send(acc, self.rank + 1)
            elif ref_owner != last:
                self._send(acc, ref_owner)
            if ref >= 0 and self.rank == ref_owner:
                if ref_owner != last:
                    acc = self._recv(P, last)
                acc = acc + per[:, -1]
            totals.append(self._bcast(acc, ref_owner, P))
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
