"""resample!'s random batch (src/model.jl:998-1066): the weights, the RNG and
the weighted draw without replacement, defined so that the Python stage
machine and the native one (rifraf_batch.cpp, `BatchRng` / `random_batch`
there) draw the same batches from the same seed, bit for bit.

- Draw: `StatsBase.sample(data, wv, n, replace=false)` with StatsBase 0.31.0
  (Manifest.toml:242-246), an absent dependency, restated: its default
  sampler without replacement, Efraimidis and Spirakis' A-ExpJ
  (`efraimidis_aexpj_wsample_norep!`).  Keys w / Exp(1) for the first n
  positive weights in a min-heap; then exponential jumps X = threshold *
  Exp(1) over the remaining weights; an item that exhausts the jump enters
  with the key -w / log(t + U (1 - t)), t = exp(-w / threshold); the output
  holds the n items by descending (key, index).  A weight that is not > 0
  is skipped, and fewer than n positive weights raise (DimensionMismatch
  there).
- RNG: xoshiro256++ (the algorithm of Julia >= 1.7's default RNG) with its
  four words from splitmix64(seed); rand() = (next() >> 11) * 2^-53 and
  randexp() = -log1p(-rand()) (Julia's ziggurat randexp is not restated).
  The reference drew from Julia's global MersenneTwister, whose stream this
  does not reproduce: which reads a random batch holds is parity-unpinned
  against Julia, and pinned between the two stage machines.
- Sums run sequentially from the first element.  The only transcendental
  functions are libm's log1p / exp / log, which CPython's math module and
  the C++ driver call alike in one process.
"""
from __future__ import annotations

import heapq
import math
import secrets

import numpy as np

from .engine import RifrafError

_M64 = (1 << 64) - 1


def _rotl(x: int, k: int) -> int:
    return ((x << k) | (x >> (64 - k))) & _M64


def splitmix64(x: int):
    """Next (state, output) of splitmix64 (Steele, Lea, Flood 2014)."""
    x = (x + 0x9E3779B97F4A7C15) & _M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return x, z ^ (z >> 31)


class BatchRng:
    """xoshiro256++ seeded by splitmix64 (rifraf_batch.cpp BatchRng)."""

    def __init__(self, seed: int | None = None, state=None):
        if state is not None:
            self.s = [int(v) & _M64 for v in state]
            return
        if seed is None:
            seed = secrets.randbits(64)
        x = int(seed) & _M64
        self.s = []
        for _ in range(4):
            x, z = splitmix64(x)
            self.s.append(z)

    def next_u64(self) -> int:
        s0, s1, s2, s3 = self.s
        result = (_rotl((s0 + s3) & _M64, 23) + s0) & _M64
        t = (s1 << 17) & _M64
        s2 ^= s0
        s3 ^= s1
        s1 ^= s2
        s0 ^= s3
        s2 ^= t
        s3 = _rotl(s3, 45)
        self.s = [s0, s1, s2, s3]
        return result

    def rand(self) -> float:
        """Uniform in [0, 1): the top 53 bits."""
        return (self.next_u64() >> 11) * (1.0 / 9007199254740992.0)


def seq_sum(xs) -> float:
    s = 0.0
    for x in xs:
        s += float(x)
    return s


def error_weights(est_n_errors) -> np.ndarray:
    """1 - err ./ sum(err) (model.jl:1052); IEEE division as in Julia (a
    one-read cluster's weights are NaN; it never draws at random)."""
    e = np.asarray(est_n_errors, np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        return 1.0 - e / seq_sum(e.tolist())


def reweight(wv, n: int, randomness: float) -> np.ndarray:   # model.jl:1017-1036
    if randomness < 0.0 or randomness > 1.0:
        raise RifrafError("randomness must be between 0.0 and 1.0")
    wv = np.asarray(wv, np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        wv = wv / seq_sum(wv.tolist())
    indices = np.argsort(wv, kind="stable")[::-1][:n]   # reverse(sortperm(wv))[1:n]
    endpoint = wv
    weight = 0.0
    if randomness > 0.5:
        weight = (randomness - 0.5) * 2.0
        endpoint = np.full(len(wv), 1.0 / len(wv))
    elif randomness < 0.5:
        weight = 1.0 - randomness * 2.0
        endpoint = np.zeros(len(wv))
        endpoint[indices] = 1.0 / n
    return weight * endpoint + (1.0 - weight) * wv


def randexp(rng: BatchRng) -> float:
    return -math.log1p(-rng.rand())


def wsample_norep(rng: BatchRng, wv, k: int) -> list:
    """k distinct indices of wv (StatsBase efraimidis_aexpj_wsample_norep!),
    by descending key."""
    w = [float(v) for v in wv]
    n = len(w)
    if k <= 0:
        return []
    pq = []
    s = -1
    for s in range(n):
        if w[s] < 0:
            raise RifrafError(f"Negative weight found in weight vector at index {s + 1}")
        if w[s] > 0:
            pq.append((w[s] / randexp(rng), s))
        if len(pq) >= k:
            break
    if len(pq) < k:
        raise RifrafError(f"wv must have at least {k} strictly positive entries (got {len(pq)})")
    heapq.heapify(pq)
    threshold = pq[0][0]
    x = threshold * randexp(rng)
    for i in range(s + 1, n):
        wi = w[i]
        if wi < 0:
            raise RifrafError(f"Negative weight found in weight vector at index {i + 1}")
        if not wi > 0:
            continue
        x -= wi
        if not x <= 0:
            continue
        t = math.exp(-wi / threshold)
        heapq.heapreplace(pq, (-wi / math.log(t + rng.rand() * (1 - t)), i))
        threshold = pq[0][0]
        x = threshold * randexp(rng)
    return [i for _, i in sorted(pq, reverse=True)]


def random_batch(rng: BatchRng, est_n_errors, n: int, randomness: float) -> list:
    """resample!'s draw of n of the reads (model.jl:1051-1054, n < #reads)."""
    return wsample_norep(rng, reweight(error_weights(est_n_errors), n, randomness), n)


def cluster_seeds(seed: int | None, k: int) -> np.ndarray:
    """Per-cluster seeds of a batched run: params.seed for every cluster (as
    k separate rifraf() calls with the same params), else fresh entropy each."""
    if seed is not None:
        return np.full(k, int(seed) & _M64, np.uint64)
    return np.array([secrets.randbits(64) for _ in range(k)], np.uint64)
