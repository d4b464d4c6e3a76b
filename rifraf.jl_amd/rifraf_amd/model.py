"""RIFRAF consensus stage machine (src/model.jl) over the MI355X engine.

Host logic -- RifrafParams, the stage machine (initial -> frame-correction ->
refinement -> scoring), resampling, candidate handling -- follows the
reference function by function (file:line cited on each).  Every alignment
fill, backtrace and proposal score runs on the HIP engine (rf_realign,
rf_backtrace, rf_score); there is no CPU numeric path here.

Engine id mapping for one rifraf() call (N reads):
  sequences 0..N-1 = reads, N = reference, N+1 = scratch (edit_distance)
  template  0      = consensus
  slots     0..    = batch positions (state.As[k] / Bs[k] / Amoves[k]),
            N = reference (A_ref / B_ref), N+1 = scratch
"""
from __future__ import annotations

import math
import sys
from dataclasses import dataclass, field
from enum import IntEnum

import numpy as np

from .align import (TRACE_CODON_DELETE, TRACE_CODON_INSERT, TRACE_DELETE, TRACE_INSERT, TRACE_MATCH,
                    moves_to_proposals_np)
from .engine import RF_BAND_A, RF_BWD, RF_FWD, RF_SKEW, Engine, RifrafError
from .errormodel import ErrorModel, Scores, phred_to_log_p
from .poisson import cquantile_poisson
from .proposals import (DEL, INS, SUB, Deletion, Insertion, Proposal, ScoredProposal, Substitution,
                        apply_proposals, choose_candidates, to_arrays)
from .resampling import BatchRng, error_weights, reweight, wsample_norep
from .rifrafsequences import RifrafSequence
from .types import BASES, CODON_LENGTH, DNASeq, dna_str


class Stage(IntEnum):                          # model.jl:1-5
    INIT = 1
    FRAME = 2
    REFINE = 3
    SCORE = 4


@dataclass
class EstimatedProbs:                          # model.jl:20-24
    sub: np.ndarray
    dele: np.ndarray
    ins: np.ndarray


@dataclass
class RifrafParams:                            # model.jl:97-164
    scores: Scores = field(default_factory=lambda: Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0)))
    ref_scores: Scores = field(default_factory=lambda: Scores.from_errors(ErrorModel(10.0, 1e-1, 1e-1, 1.0, 1.0)))
    ref_indel_mult: float = 3.0
    max_ref_indel_mults: int = 5
    ref_error_mult: float = 1.0
    do_init: bool = True
    do_frame: bool = True
    do_refine: bool = True
    do_score: bool = False
    do_alignment_proposals: bool = True
    seed_indels: bool = True
    indel_correction_only: bool = True
    use_ref_for_qvs: bool = False
    bandwidth: int = 3 * CODON_LENGTH
    bandwidth_pvalue: float = 0.1
    min_dist: int = 5 * CODON_LENGTH
    batch_fixed: bool = True
    batch_fixed_size: int = 5
    batch_size: int = 20
    batch_randomness: float = 0.9
    batch_mult: float = 0.7
    batch_threshold: float = 0.1
    max_iters: int = 100
    verbose: int = 0
    seed: int | None = None                    # RNG for resample! (Julia's global RNG)


@dataclass
class RifrafState:                             # model.jl:167-193
    consensus: np.ndarray
    ref_scores: Scores
    reference: RifrafSequence
    batch_fixed_size: int
    batch_size: int
    base_batch_size: int
    sequences: list
    maxlen: int
    score: float = -math.inf
    ref_error_rate: float = -math.inf
    n_ref_indel_mults: int = 0
    batch_randomness: float = 0.9
    batch_seqs: list = field(default_factory=list)       # indices into sequences
    n_slots: int = 0                                     # length(state.As)
    slot_scores: list = field(default_factory=list)      # A[end, end] per slot
    ref_score: float = -math.inf                         # A_ref[end, end]
    realign_As: bool = True
    realign_Bs: bool = True
    penalties_increased: bool = False
    stage: Stage = Stage.INIT
    stage_iterations: list = field(default_factory=lambda: [0, 0, 0, 0])
    converged: bool = False


@dataclass
class RifrafResult:                            # model.jl:216-225
    consensus: np.ndarray
    params: RifrafParams
    state: RifrafState
    consensus_stages: list
    error_probs: EstimatedProbs | None = None
    aln_error_probs: np.ndarray | None = None


# realign()'s B call also fills single_indel_proposals' skewed reference
# alignment in FRAME (one engine call); False: single_indel_proposals fills
# it itself (the reference's order; tests compare the two)
SIP_CACHE = True


class _Run:
    """Engine bindings of one rifraf() call (ids per the module docstring)."""

    def __init__(self, engine: Engine, nseqs: int):
        self.e = engine
        self.N = nseqs
        self.REF = nseqs
        self.SCRATCH = nseqs + 1
        self.tpl_version = None
        # the scratch slot holds single_indel_proposals' skewed fill of the
        # current reference against the current consensus (filled beside the
        # B realign, realign()); cleared by every consensus / reference upload
        # and by has_single_indels' own fill
        self.sip_ready = False

    def set_consensus(self, cons):
        self.sip_ready = False
        self.e.set_templates(0, [cons])

    def set_ref(self, ref):
        self.sip_ready = False
        self.e.set_sequences(self.REF, [ref])

    def scratch(self):
        """The scratch slot, for any write to it other than realign()'s
        skewed fill (edit_distance, has_single_indels): the cached fill is
        gone once it is written."""
        self.sip_ready = False
        return self.SCRATCH


def log(params, level, msg):
    if params.verbose >= level:
        print(msg, file=sys.stderr)


# ---------------------------------------------------------------------
# checks and initial state
# ---------------------------------------------------------------------

def check_params(scores: Scores, reference, params: RifrafParams):   # model.jl:842-896
    if (scores.mismatch >= 0.0 or scores.mismatch == -math.inf or scores.insertion >= 0.0
            or scores.insertion == -math.inf or scores.deletion >= 0.0 or scores.deletion == -math.inf):
        raise RifrafError("scores must be between -Inf and 0.0")
    if scores.codon_insertion > -math.inf or scores.codon_deletion > -math.inf:
        raise RifrafError("error model cannot allow codon indels")
    if len(reference) > 0:
        if params.ref_error_mult <= 0.0:
            raise RifrafError("ref_error_mult must be > 0.0")
        if params.ref_indel_mult <= 0.0:
            raise RifrafError("ref_indel_mult must be > 0.0")
        rs = params.ref_scores
        if (rs.mismatch >= 0.0 or rs.insertion >= 0.0 or rs.deletion >= 0.0 or rs.codon_insertion >= 0.0
                or rs.codon_deletion >= 0.0):
            raise RifrafError("ref scores cannot be >= 0")
        if -math.inf in (rs.mismatch, rs.insertion, rs.deletion, rs.codon_insertion, rs.codon_deletion):
            raise RifrafError("ref scores cannot be -Inf")
        if params.max_ref_indel_mults < 0:
            raise RifrafError("ref_indel_increases must be >= 0")
    if not any([params.do_init, params.do_frame, params.do_refine, params.do_score]):
        raise RifrafError("no stages enabled")
    if params.max_iters < 1:
        raise RifrafError(f"invalid max iters: {params.max_iters}")
    if params.batch_fixed and params.batch_fixed_size <= 1:
        raise RifrafError("batch_fixed_size must be > 1")
    if params.batch_randomness < 0.0 or params.batch_randomness > 1.0:
        raise RifrafError("batch_randomness must be between 0.0 and 1.0")
    if params.batch_mult < 0.0 or params.batch_mult > 1.0:
        raise RifrafError("batch_mult must be between 0.0 and 1.0")
    if params.batch_threshold < 0.0 or params.batch_mult > 1.0:
        raise RifrafError("batch_threshold must be between 0.0 and 1.0")


def logsumexp10(x):                            # util.jl:28-38
    x = np.asarray(x, np.float64)
    if x.size == 0:
        return -math.inf
    u = float(np.max(x))
    if abs(u) == math.inf:
        return math.nan if np.isnan(x).any() else u
    # sequential accumulation in index order (cumsum), as the reference's loop
    s = float(np.cumsum(np.power(10.0, x - u))[-1])
    return math.log10(s) + u


def initial_state(consensus, sequences, reference, params: RifrafParams, maxlen=None) -> RifrafState:  # :564-615
    batch_size = params.batch_size if params.batch_size > 1 else len(sequences)
    batch_size = min(batch_size, len(sequences))
    batch_fixed_size = min(params.batch_fixed_size, len(sequences))
    if len(consensus) == 0:
        scores = [logsumexp10(s.match_scores) for s in sequences]
        idx = int(np.argmax(scores))              # indmax: first maximum
        consensus = sequences[idx].seq.copy()
    if maxlen is None:                            # (callers with the lengths at hand pass it)
        maxlen = max(len(s) for s in sequences)
    ref_error_log_p = np.zeros(len(reference))    # placeholder, :601-603
    refseq = RifrafSequence(reference, ref_error_log_p, params.bandwidth, params.ref_scores) \
        if len(reference) > 0 else RifrafSequence()
    return RifrafState(consensus=DNASeq(consensus), ref_scores=params.ref_scores, reference=refseq,
                       batch_fixed_size=batch_fixed_size, batch_size=batch_size,
                       base_batch_size=batch_size, sequences=sequences, maxlen=maxlen)
    # batch_randomness keeps RifrafState's default 0.9 (model.jl:177): the
    # reference's initial_state (:604-614) does not pass params.batch_randomness,
    # which check_params validates (:887) and nothing else reads


def use_ref(ref: RifrafSequence, stage: Stage, use_ref_for_qvs: bool) -> bool:   # :617-628
    if len(ref) == 0:
        return False
    if stage == Stage.FRAME:
        return True
    return stage == Stage.SCORE and use_ref_for_qvs


# ---------------------------------------------------------------------
# realign / rescore (model.jl:630-719)
# ---------------------------------------------------------------------

def rescore(state: RifrafState, run: _Run, use_ref_for_qvs: bool):   # :630-635
    # sum over all state.As (left fold, including stale slots), + A_ref
    total = state.slot_scores[0]
    for v in state.slot_scores[1:state.n_slots]:
        total += v
    state.score = total
    if use_ref(state.reference, state.stage, use_ref_for_qvs):
        state.score += state.ref_score


def smart_forward_moves(run: _Run, jobs, seqs, consensus_len, pvalue):   # :643-672
    """Batched smart_forward_moves!: jobs = [(slot, seq_id)], seqs = their
    RifrafSequences.  Returns A[end,end] per job."""
    e = run.e
    n = len(jobs)
    max_bw = [s.bandwidth if s.bandwidth_fixed else min(s.bandwidth * 2 ** 5, consensus_len, len(s))
              for s in seqs]
    scores = np.empty(n)
    old_err = [sys.maxsize] * n
    n_err = [sys.maxsize] * n
    pending = list(range(n))
    while pending:
        sl = np.array([jobs[k][0] for k in pending], np.int32)
        ids = np.array([jobs[k][1] for k in pending], np.int32)
        bws = np.array([seqs[k].bandwidth for k in pending], np.int32)
        out = e.realign(sl, ids, 0, bws, RF_FWD)
        scores[pending] = out
        check = [k for k in pending if not (seqs[k].bandwidth_fixed or seqs[k].bandwidth >= max_bw[k])]
        if not check:
            break
        _, nerr = e.backtrace(np.array([jobs[k][0] for k in check], np.int32), want_moves=False)
        nxt = []
        for k, ne in zip(check, nerr):
            old_err[k] = n_err[k]
            n_err[k] = int(ne)
            threshold = cquantile_poisson(seqs[k].est_n_errors, pvalue)
            if n_err[k] > threshold and n_err[k] < old_err[k]:
                seqs[k].bandwidth = min(seqs[k].bandwidth * 2, max_bw[k])
                nxt.append(k)
        pending = nxt
    for s in seqs:
        s.bandwidth_fixed = True
    return scores


def realign(state: RifrafState, run: _Run, params: RifrafParams):   # :679-714
    seqs = [state.sequences[i] for i in state.batch_seqs]
    while state.n_slots < len(seqs):                 # grow As/Bs/Amoves
        state.slot_scores.append(0.0)                # A[end,end] of a fresh (zero) BandedArray
        state.n_slots += 1
    ref_on = use_ref(state.reference, state.stage, params.use_ref_for_qvs)
    # the reads' and the reference's fills are independent jobs of one engine
    # call each (round 5: the reference's long latency-bound fill runs beside
    # the reads' instead of after them; the same bands and scores)
    if state.realign_As:
        log(params, 2, "    realigning As")
        jobs = [(k, i) for k, i in enumerate(state.batch_seqs)]
        jseqs = list(seqs)
        if ref_on:
            jobs.append((run.REF, run.REF))
            jseqs.append(state.reference)
        sc = smart_forward_moves(run, jobs, jseqs, len(state.consensus), params.bandwidth_pvalue)
        for k in range(len(seqs)):
            state.slot_scores[k] = float(sc[k])
        if ref_on:
            state.ref_score = float(sc[len(seqs)])
    if state.realign_Bs:
        log(params, 2, "    realigning Bs")
        slots = list(range(len(seqs)))
        ids = list(state.batch_seqs)
        bws = [s.bandwidth for s in seqs]
        flags = [RF_BWD] * len(seqs)
        if ref_on:
            slots.append(run.REF)
            ids.append(run.REF)
            bws.append(state.reference.bandwidth)
            flags.append(RF_BWD)
        # FRAME with seeded indels: single_indel_proposals' skewed fill of the
        # reference against this consensus (model.jl:538-562) in the same call
        sip = SIP_CACHE and state.stage == Stage.FRAME and params.seed_indels and len(state.reference) > 0
        if sip:
            slots.append(run.SCRATCH)
            ids.append(run.REF)
            bws.append(state.reference.bandwidth)
            flags.append(RF_FWD | RF_SKEW)
        run.e.realign(np.array(slots, np.int32), np.array(ids, np.int32), 0, np.array(bws, np.int32),
                      np.array(flags, np.int32) if sip else RF_BWD)
        run.sip_ready = sip


def realign_rescore(state, run, params):       # :716-719
    realign(state, run, params)
    rescore(state, run, params.use_ref_for_qvs)


# ---------------------------------------------------------------------
# proposals (model.jl:401-562)
# ---------------------------------------------------------------------

def all_proposals(stage: Stage, consensus, indel_correction_only: bool, indel_seeds=(),
                  seed_neighborhood: int = CODON_LENGTH):           # :401-456
    length = len(consensus)
    ins_positions, del_positions = set(), set()
    for p in indel_seeds:
        if p.kind == INS:
            ins_positions.update(range(max(p.pos - seed_neighborhood, 0), min(p.pos + seed_neighborhood, length) + 1))
        else:
            del_positions.update(range(max(p.pos - seed_neighborhood, 1), min(p.pos + seed_neighborhood, length) + 1))
    do_subs = stage != Stage.FRAME or not indel_correction_only
    do_indels = stage in (Stage.INIT, Stage.FRAME, Stage.SCORE)
    no_seeds = len(indel_seeds) == 0
    results = []
    if do_indels:
        results += [Insertion(0, b) for b in range(4)]
    for j in range(1, length + 1):
        if do_subs:
            results += [Substitution(j, b) for b in range(4) if consensus[j - 1] != b]
        if do_indels:
            if no_seeds or j in del_positions:
                results.append(Deletion(j))
            if no_seeds or j in ins_positions:
                results += [Insertion(j, b) for b in range(4)]
    return results


def alignment_proposals(state: RifrafState, run: _Run, do_indels: bool):   # :483-497
    """Union of the proposals seen in the batch alignments.  The reference
    collects a Julia Set (hash order); this mirror returns them sorted by
    (pos, kind, base), a documented deterministic order.  Engines with a
    device-side union (rf_alignment_proposals) return it as a dense mask."""
    slots = np.arange(len(state.batch_seqs), dtype=np.int32)
    if hasattr(run.e, "alignment_proposals"):
        return mask_to_proposals(run.e.alignment_proposals([slots], do_indels)[0])
    moves, _ = run.e.backtrace(slots)
    cons = state.consensus
    found = set()
    for mv, i in zip(moves, state.batch_seqs):
        k, p, b = moves_to_proposals_np(mv, cons, state.sequences[i].seq)
        if not do_indels:
            keep = k == SUB
            k, p, b = k[keep], p[keep], b[keep]
        found.update(zip(k.tolist(), p.tolist(), b.tolist()))
    return [Proposal(k, p, b) for (k, p, b) in sorted(found, key=lambda t: (t[1], t[0], t[2]))]


# dense slot -> (kind, base) in (kind, base) order within a position: Sub A..T, Ins A..T, Del
_MASK_ORDER = [(0, SUB, 0), (1, SUB, 1), (2, SUB, 2), (3, SUB, 3),
               (5, INS, 0), (6, INS, 1), (7, INS, 2), (8, INS, 3), (4, DEL, 0)]


def mask_to_proposals(mask):
    """(m+1, 9) proposal mask -> Proposal list sorted by (pos, kind, base)."""
    mask = np.asarray(mask)
    order = np.array([c for c, _, _ in _MASK_ORDER])
    kinds = np.array([k for _, k, _ in _MASK_ORDER])
    bases = np.array([b for _, _, b in _MASK_ORDER])
    pos, col = np.nonzero(mask[:, order])
    return [Proposal(int(kinds[c]), int(p), int(bases[c])) for p, c in zip(pos.tolist(), col.tolist())]


def _align_ref_moves(state: RifrafState, run: _Run, skew: bool):
    """align_moves(consensus, reference; skew_matches) on the engine
    (align.jl:337-344): forward_moves! of the reference (rows) against the
    consensus with the reference's own bandwidth, then backtrace.  The
    skewed fill may already be in the scratch slot (realign's B call)."""
    ref = state.reference
    if not (skew and run.sip_ready):
        run.set_ref(ref)
        run.e.realign([run.scratch()], [run.REF], 0, [ref.bandwidth], RF_FWD | (RF_SKEW if skew else 0))
    run.sip_ready = False
    moves, _ = run.e.backtrace([run.SCRATCH])
    return moves[0]


def has_single_indels(state, run) -> bool:                         # :532-536
    moves = _align_ref_moves(state, run, skew=False)
    return bool(((moves == TRACE_INSERT) | (moves == TRACE_DELETE)).any())


def single_indel_proposals(state, run):                            # :538-562
    moves = _align_ref_moves(state, run, skew=True)
    results = []
    cons_idx = ref_idx = 0
    refseq = state.reference.seq
    for mv in moves.tolist():
        if mv == TRACE_MATCH:
            cons_idx += 1
            ref_idx += 1
        elif mv == TRACE_INSERT:
            ref_idx += 1
            results.append(Insertion(cons_idx, int(refseq[ref_idx - 1])))
        elif mv == TRACE_DELETE:
            cons_idx += 1
            results.append(Deletion(cons_idx))
        elif mv == TRACE_CODON_INSERT:
            ref_idx += 3
        elif mv == TRACE_CODON_DELETE:
            cons_idx += 3
    return results


def score_proposals(state: RifrafState, run: _Run, proposals, with_ref: bool):
    """score_proposal(m, state, newcols, use_ref) for a proposal list
    (model.jl:385-399): batch fold (+ reference last) on the engine."""
    if not proposals:
        return np.zeros(0)
    slots = np.arange(len(state.batch_seqs), dtype=np.int32)
    return run.e.score([(slots, run.REF if with_ref else -1, to_arrays(proposals))])[0]


def get_candidates(state: RifrafState, run: _Run, params: RifrafParams, indel_seeds=()):   # :499-526
    use_ref_ = state.stage == Stage.FRAME
    if state.stage in (Stage.INIT, Stage.REFINE) and params.do_alignment_proposals:
        proposals = alignment_proposals(state, run, state.stage == Stage.INIT)
    else:
        proposals = all_proposals(state.stage, state.consensus, params.indel_correction_only, indel_seeds)
    totals = score_proposals(state, run, proposals, use_ref_)
    return [ScoredProposal(p, float(s)) for p, s in zip(proposals, totals) if s > state.score]


# ---------------------------------------------------------------------
# stage machine (model.jl:898-1114)
# ---------------------------------------------------------------------

def _set_consensus(state, run, cons):
    state.consensus = DNASeq(cons)
    run.set_consensus(state.consensus)


def handle_candidates(candidates, state: RifrafState, run: _Run, params: RifrafParams):   # :898-935
    old_consensus = state.consensus
    chosen = choose_candidates(candidates, params.min_dist)
    log(params, 2, f"    found {len(candidates)} candidates; filtered to {len(chosen)}")
    log(params, 3, f"    chosen: {chosen}")
    _set_consensus(state, run, apply_proposals(old_consensus, [c.proposal for c in chosen]))
    state.realign_As = True
    state.realign_Bs = False
    realign_rescore(state, run, params)
    if len(chosen) > 1 and (state.score < chosen[0].score or
                            math.isclose(state.score, chosen[0].score, rel_tol=math.sqrt(sys.float_info.epsilon))):
        log(params, 2, "    rejecting multiple candidates in favor of best")
        chosen = [chosen[0]]
        _set_consensus(state, run, apply_proposals(old_consensus, [c.proposal for c in chosen]))
    else:
        state.realign_As = False
    state.realign_Bs = True
    return chosen


def edit_distance_engine(t, s, run: _Run):                        # align.jl:253-260
    from .align import Scratch, edit_distance
    slot = run.scratch()
    return edit_distance(t, s, scratch=Scratch(run.e, slot, 1, slot))


def finish_stage(state: RifrafState, run: _Run, params: RifrafParams):   # :937-995
    log(params, 2, f"    no candidates found in {state.stage.name}.")
    if state.stage == Stage.INIT:
        if len(state.reference) == 0 or not params.do_frame:
            state.converged = True
        else:
            state.stage = Stage.FRAME
            edit_dist = edit_distance_engine(state.consensus, state.reference.seq, run)
            ref_error_rate = edit_dist / max(len(state.reference), len(state.consensus))
            ref_error_rate *= params.ref_error_mult
            state.ref_error_rate = min(max(ref_error_rate, 1e-10), 0.5)
            ref_error_log_p = np.full(len(state.reference), math.log10(state.ref_error_rate))
            state.reference = RifrafSequence(state.reference.seq, ref_error_log_p, params.bandwidth,
                                             state.ref_scores)
            run.set_ref(state.reference)
            if not has_single_indels(state, run):
                state.converged = True
    elif state.stage == Stage.FRAME:
        if not has_single_indels(state, run):
            state.stage = Stage.REFINE
        elif state.n_ref_indel_mults == params.max_ref_indel_mults:
            log(params, 2, "    NOTE: alignment had single indels but reached penalty limit.")
            state.stage = Stage.REFINE
        else:
            state.penalties_increased = True
            if state.n_ref_indel_mults < params.max_ref_indel_mults:
                state.n_ref_indel_mults += 1
            else:
                raise RifrafError("Tried to illegally increase n_ref_indel_mults")
            mult = params.ref_indel_mult ** state.n_ref_indel_mults
            rs = state.ref_scores
            state.ref_scores = Scores(rs.mismatch, rs.insertion * mult, rs.deletion * mult,
                                      rs.codon_insertion, rs.codon_deletion)
            state.reference = RifrafSequence.rescored(state.reference, state.ref_scores)
            run.set_ref(state.reference)
            log(params, 2, "    NOTE: alignment to reference had single indels. increasing penalty.")
    elif state.stage == Stage.REFINE:
        state.converged = True
    else:
        raise RifrafError(f"  invalid stage: {state.stage}")


def resample(state: RifrafState, params: RifrafParams, rng: BatchRng):   # :1038-1066
    err_weights = np.array([s.est_n_errors for s in state.sequences])
    if state.stage in (Stage.INIT, Stage.FRAME) and params.batch_fixed:
        state.batch_seqs = np.argsort(err_weights, kind="stable")[:state.batch_fixed_size].tolist()
        log(params, 2, "    kept fixed batch")
        return
    n = state.batch_size
    wv = reweight(error_weights(err_weights), n, state.batch_randomness)
    if n < len(state.sequences):
        # StatsBase.sample(data, Weights, n, replace=false): the draw and the
        # RNG of resampling.py, which the native driver shares (the batch
        # Julia's RNG stream would draw is parity-unpinned)
        state.batch_seqs = wsample_norep(rng, wv, n)
        state.realign_As = True
        log(params, 2, f"    sampled {n} new sequences")
    else:
        state.batch_seqs = list(range(len(state.sequences)))
        log(params, 2, "    sampled all sequences")


def check_score(state: RifrafState, run: _Run, params: RifrafParams, old_score: float, rng) -> bool:  # :1074-1114
    log(params, 2, f"    score: {state.score}")
    if (not state.penalties_increased and state.batch_size == len(state.sequences)
            and state.stage_iterations[int(state.stage) - 1] > 1):
        if state.score < old_score:
            log(params, 2, "    WARNING: not using batches, but score decreased.")
        elif state.score == old_score:
            log(params, 2, "    score did not change. ending stage.")
            return False
    # IEEE division as in Julia (x / 0.0 is +-Inf or NaN, never an exception)
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = float(np.float64(state.score - old_score) / np.float64(old_score))
    if (rel > params.batch_threshold and not state.penalties_increased
            and state.batch_size < len(state.sequences) and state.stage_iterations[int(state.stage) - 1] > 1):
        state.batch_size = min(state.batch_size + state.base_batch_size, len(state.sequences))
        log(params, 2, f"    NOTE: increased batch size to {state.batch_size}.")
        resample(state, params, rng)
        state.realign_As = True
        state.realign_Bs = True
        realign_rescore(state, run, params)
        log(params, 2, f"    new score: {state.score}")
    return True


# ---------------------------------------------------------------------
# quality scores (model.jl:721-840)
# ---------------------------------------------------------------------

def normalize_log_differences(sub_scores, del_scores, ins_scores, state_score):   # :722-735
    pos_scores = np.hstack([sub_scores, del_scores[:, None]])
    pos_exp = np.power(10.0, pos_scores)
    pos_probs = pos_exp / pos_exp.sum(axis=1, keepdims=True)
    ins_exp = np.power(10.0, ins_scores)
    ins_probs = ins_exp / (10.0 ** state_score + ins_exp.sum(axis=1, keepdims=True))
    return EstimatedProbs(pos_probs[:, :4], pos_probs[:, 4], ins_probs)


def score_proposal_arrays(m: int, consensus):
    """all_proposals(STAGE_SCORE, consensus, false) without seeds
    (model.jl:401-456) as (kind, pos, base) arrays in the same order:
    Ins(0, ACGT); then per position j: Sub(j, b != cons[j]), Del(j), Ins(j, ACGT)."""
    cons = np.asarray(consensus, np.int64)
    # per position: 4 sub candidates (the consensus base's is dropped), del, 4 ins
    j9 = np.repeat(np.arange(1, m + 1), 9)
    s9 = np.tile(np.arange(9), m)
    keep = ~((s9 < 4) & (s9 == cons[j9 - 1]))
    j9, s9 = j9[keep], s9[keep]
    kind = np.where(s9 < 4, SUB, np.where(s9 == 4, DEL, INS))
    base = np.where(s9 < 4, s9, np.where(s9 == 4, 0, s9 - 5))
    kind = np.concatenate([np.full(4, INS), kind]).astype(np.uint8)
    pos = np.concatenate([np.zeros(4, np.int64), j9]).astype(np.int32)
    base = np.concatenate([np.arange(4), base]).astype(np.uint8)
    return kind, pos, base


def estimate_probs(state: RifrafState, run: _Run, use_ref_for_qvs: bool) -> EstimatedProbs:   # :737-791
    m = len(state.consensus)
    sub_scores = np.zeros((m, 4)) + state.score
    del_scores = np.zeros(m) + state.score
    ins_scores = np.zeros((m + 1, 4))
    use_ref_ = len(state.reference) > 0 and use_ref_for_qvs
    kind, pos, base = score_proposal_arrays(m, state.consensus)
    slots = np.arange(len(state.batch_seqs), dtype=np.int32)
    scores = run.e.score([(slots, run.REF if use_ref_ else -1, (kind, pos, base))])[0]
    k = kind.astype(np.int64)
    p = pos.astype(np.int64)
    b = base.astype(np.int64)
    sub = k == SUB
    dele = k == DEL
    ins = k == INS
    sub_scores[p[sub] - 1, b[sub]] = scores[sub]
    del_scores[p[dele] - 1] = scores[dele]
    ins_scores[p[ins], b[ins]] = scores[ins]
    max_score = max(sub_scores.max(), del_scores.max(), ins_scores.max())
    sub_scores = sub_scores - max_score
    del_scores = del_scores - max_score
    ins_scores = ins_scores - max_score
    if sub_scores.max() > 0.0:
        raise RifrafError("sub scores cannot be positive")
    if del_scores.max() > 0.0:
        raise RifrafError("deletion scores cannot be positive")
    if ins_scores.max() > 0.0:
        raise RifrafError("insertion scores cannot be positive")
    return normalize_log_differences(sub_scores, del_scores, ins_scores, state.score - max_score)


def estimate_probs_from_dense(state: RifrafState, dense) -> EstimatedProbs:
    """estimate_probs (model.jl:737-791) from the cluster's rf_score_dense
    totals instead of an rf_score proposal list: the dense slots are the same
    left folds of the same per-read scores (rf_score gathers them from this
    very table), and every array operation below is estimate_probs's."""
    m = len(state.consensus)
    dense = np.asarray(dense)
    cons = np.asarray(state.consensus, np.int64)
    sub = dense[1:, 0:4].copy()
    own = np.zeros((m, 4), bool)
    own[np.arange(m), cons] = True
    used = np.concatenate([sub[~own], dense[1:, 4], dense[:, 5:9].ravel()])
    if np.isnan(used).any():
        raise RifrafError("failed to compute a valid score")
    sub_scores = np.zeros((m, 4)) + state.score
    sub_scores[~own] = sub[~own]
    del_scores = dense[1:, 4].copy()
    ins_scores = dense[:, 5:9].copy()
    max_score = max(sub_scores.max(), del_scores.max(), ins_scores.max())
    sub_scores = sub_scores - max_score
    del_scores = del_scores - max_score
    ins_scores = ins_scores - max_score
    if sub_scores.max() > 0.0:
        raise RifrafError("sub scores cannot be positive")
    if del_scores.max() > 0.0:
        raise RifrafError("deletion scores cannot be positive")
    if ins_scores.max() > 0.0:
        raise RifrafError("insertion scores cannot be positive")
    return normalize_log_differences(sub_scores, del_scores, ins_scores, state.score - max_score)


def _power10(x):
    """np.power(10.0, x) over row blocks on host threads (numpy drops the GIL
    inside a ufunc; each element's value is the same whichever block holds it)."""
    x = np.ascontiguousarray(x)
    if x.size < (1 << 20):
        return np.power(10.0, x)
    import os
    from concurrent.futures import ThreadPoolExecutor
    out = np.empty_like(x)
    nth = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                     len(os.sched_getaffinity(0))))   # the cores this thread may use
    cut = np.linspace(0, len(x), nth + 1).astype(int)
    with ThreadPoolExecutor(nth) as ex:
        list(ex.map(lambda t: np.power(10.0, x[cut[t]:cut[t + 1]], out=out[cut[t]:cut[t + 1]]), range(nth)))
    return out


def qvs_many(states, dense, sums):
    """estimate_probs_from_dense and aln_error_probs_from_sums for many
    clusters at once: every cluster's arrays are stacked and each numpy
    operation runs once over the stack.  The operations are elementwise, per
    row of a fixed length, or maxima (exact in any order), which numpy
    evaluates identically wherever a row sits; the per-cluster scalars (the
    max score, 10.0 ** state_score) are computed per cluster exactly as the
    single-cluster code does.  Returns [(EstimatedProbs, aln_error_probs)]."""
    K = len(states)
    ms = np.array([len(st.consensus) for st in states], np.int64)
    moff = np.zeros(K + 1, np.int64)
    np.cumsum(ms, out=moff[1:])
    roff = moff + np.arange(K + 1)                                      # rows of the dense tables
    D = np.concatenate([np.asarray(d) for d in dense])                  # (sum(m+1), 9)
    body = np.ones(len(D), bool)
    body[roff[:-1]] = False                                              # rows p >= 1
    Db = D[body]
    cons = np.concatenate([np.asarray(st.consensus, np.int64) for st in states])
    rows = np.arange(len(Db))
    nan = np.isnan(Db[:, 0:5])
    nan[rows, cons] = False                                              # not a proposal
    if nan.any() or np.isnan(D[:, 5:9]).any():
        raise RifrafError("failed to compute a valid score")
    S = Db[:, 0:4].copy()
    S[rows, cons] = np.zeros(len(Db)) + np.repeat(np.array([st.score for st in states]), ms)
    Dl = Db[:, 4].copy()
    I = D[:, 5:9]
    mxS = np.maximum.reduceat(S.max(axis=1), moff[:-1])
    mxD = np.maximum.reduceat(Dl, moff[:-1])
    mxI = np.maximum.reduceat(I.max(axis=1), roff[:-1])
    mx = [max(x, y, z) for x, y, z in zip(mxS, mxD, mxI)]              # max(sub.max(), del.max(), ins.max())
    mxa = np.array(mx, np.float64)
    for k in np.nonzero((mxS - mxa > 0.0) | (mxD - mxa > 0.0) | (mxI - mxa > 0.0))[0][:1]:
        raise RifrafError("sub scores cannot be positive" if mxS[k] - mxa[k] > 0.0 else
                          "deletion scores cannot be positive" if mxD[k] - mxa[k] > 0.0 else
                          "insertion scores cannot be positive")
    mrow = np.repeat(mxa, ms)
    # normalize_log_differences (model.jl:722-735)
    pos_exp = _power10(np.hstack([S - mrow[:, None], (Dl - mrow)[:, None]]))
    pos_probs = pos_exp / pos_exp.sum(axis=1, keepdims=True)
    ins_exp = _power10(I - np.repeat(mxa, ms + 1)[:, None])
    st_pow = np.repeat(np.array([10.0 ** (st.score - mx[k]) for k, st in enumerate(states)]), ms + 1)
    ins_probs = ins_exp / (st_pow[:, None] + ins_exp.sum(axis=1, keepdims=True))
    A = _power10(np.concatenate([np.asarray(x) for x in sums]))         # alignment_error_probs
    aln = 1.0 - (A / A.sum(axis=1, keepdims=True)).max(axis=1)
    out = []
    for k in range(K):
        a, b, c, d = moff[k], moff[k + 1], roff[k], roff[k + 1]
        out.append((EstimatedProbs(pos_probs[a:b, :4], pos_probs[a:b, 4], ins_probs[c:d]), aln[a:b]))
    return out


def _stacked(parts, rows, cols):
    """The arrays of `parts` as one (rows, cols) array: their common base
    when they are consecutive views of it (engine.score_dense /
    aln_error_sums_ptr results), else a concatenation."""
    if parts:
        b = parts[0].base
        if (isinstance(b, np.ndarray) and b.dtype == np.float64 and b.flags.c_contiguous and b.ndim == 2
                and b.shape[1] == cols and b.shape[0] >= rows and parts[0].ctypes.data == b.ctypes.data):
            at, ok = b.ctypes.data, True
            for x in parts:
                if x.base is not b or x.ctypes.data != at:
                    ok = False
                    break
                at += x.shape[0] * cols * 8
            if ok and at == b.ctypes.data + rows * cols * 8:
                return b[:rows]
    return np.ascontiguousarray(np.concatenate([np.asarray(x, np.float64) for x in parts]) if parts
                                else np.zeros((0, cols)))


def qvs_many_lib(states, dense, sums):
    """qvs_many with its passes in C++ (rf_host_qv_prep / rf_host_qv_finish,
    host threads) and numpy's power in between: the same exponents, the same
    10^x, the same sequential row sums and divisions, so the same values
    (tests/test_host_batch.py compares every bit).  Falls back to qvs_many
    without the library or for an empty consensus."""
    K = len(states)
    ms = np.array([len(st.consensus) for st in states], np.int64)
    try:
        from . import _lib
        lib = _lib.load()
    except Exception:  # noqa: BLE001 -- host-only use without the library
        lib = None
    if lib is None or K == 0 or (ms == 0).any():
        return qvs_many(states, dense, sums)
    moff = np.zeros(K + 1, np.int64)
    np.cumsum(ms, out=moff[1:])
    M = int(moff[-1])
    D = _stacked(dense, M + K, 9)
    A = _stacked(sums, M, 4)
    cons = np.ascontiguousarray(np.concatenate([np.asarray(st.consensus, np.uint8) for st in states]))
    score = np.array([st.score for st in states], np.float64)
    xpos, xins, mx = np.empty((M, 5)), np.empty((M + K, 4)), np.empty(K)
    err = np.zeros(2, np.int32)
    P = _lib.ptr
    if lib.rf_host_qv_prep(K, P(moff), P(D), P(cons), P(score), P(xpos), P(xins), P(mx), P(err)) != 0:
        raise RifrafError("rf_host_qv_prep: invalid arguments")
    if err[0]:
        raise RifrafError({1: "failed to compute a valid score", 2: "sub scores cannot be positive",
                           3: "deletion scores cannot be positive",
                           4: "insertion scores cannot be positive"}[int(err[0])])
    epos, eins, ealn = _power10(xpos), _power10(xins), _power10(A)
    # 10.0 ** (score - mx) with mx a numpy float64, as qvs_many evaluates it
    st_pow = np.array([10.0 ** (st.score - mx[k]) for k, st in enumerate(states)])
    aln = np.empty(M)
    if lib.rf_host_qv_finish(K, P(moff), P(st_pow), P(epos), P(eins), P(ealn), P(aln)) != 0:
        raise RifrafError("rf_host_qv_finish: invalid arguments")
    out = []
    for k in range(K):
        a, b, c, d = moff[k], moff[k + 1], moff[k] + k, moff[k + 1] + k + 1
        out.append((EstimatedProbs(epos[a:b, :4], epos[a:b, 4], eins[c:d]), aln[a:b]))
    return out


def aln_error_probs_from_sums(sums):
    """alignment_error_probs's final normalisation (model.jl:835-839) of the
    per-column base-distribution sums (rf_aln_error_sums)."""
    probs = np.power(10.0, np.asarray(sums))
    return 1.0 - (probs / probs.sum(axis=1, keepdims=True)).max(axis=1)


def base_distribution(base, ilp):                                  # :804-809
    lp = math.log10(1.0 - 10.0 ** ilp)
    result = np.full(4, lp - math.log10(3))
    result[base] = ilp
    return result


def alignment_error_probs(tlen, state: RifrafState, run: _Run):   # :817-840
    """Per consensus position, 1 - max normalised base probability over the
    batch alignments.  The move walk is vectorised over all reads at once and
    the base_distribution rows are built once per distinct (base, match
    score); every column still receives its rows in batch order (one fancy
    add per read), so the sums are the reference loop's."""
    probs = np.zeros((tlen, 4))
    slots = np.arange(len(state.batch_seqs), dtype=np.int32)
    moves, _ = run.e.backtrace(slots)
    if moves:
        _add_base_distributions(probs, moves, [state.sequences[idx] for idx in state.batch_seqs])
    probs = np.power(10.0, probs)
    probs = 1.0 - (probs / probs.sum(axis=1, keepdims=True)).max(axis=1)
    return probs


# read / consensus advance of each move code (align.jl:14-18 OFFSETS)
_MOVE_DI = np.array([0, 1, 1, 0, 3, 0], np.int64)
_MOVE_DJ = np.array([0, 1, 0, 1, 0, 3], np.int64)


def _add_base_distributions(probs, moves, seqs):
    nr = len(moves)
    lens = np.array([len(mv) for mv in moves], np.int64)
    mv = np.concatenate(moves)
    start = np.zeros(nr + 1, np.int64)
    np.cumsum(lens, out=start[1:])
    # i, j after each move (align.jl:286-311 walk), restarted at (1, 1) per read
    ci = np.zeros(len(mv) + 1, np.int64)
    cj = np.zeros(len(mv) + 1, np.int64)
    np.cumsum(_MOVE_DI[mv], out=ci[1:])
    np.cumsum(_MOVE_DJ[mv], out=cj[1:])
    match = mv == TRACE_MATCH
    ii = (ci[1:] - np.repeat(ci[start[:-1]], lens))[match] - 1   # matched read base (0-based)
    jj = (cj[1:] - np.repeat(cj[start[:-1]], lens))[match] - 1   # consensus column (0-based)
    owner = np.repeat(np.arange(nr), lens)[match]
    bases = np.concatenate([s.seq for s in seqs])
    mscores = np.concatenate([np.asarray(s.match_scores) for s in seqs])
    soff = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum([len(s.seq) for s in seqs], out=soff[1:])
    gi = soff[owner] + ii
    ilps = mscores[gi]
    ulp, inv = np.unique(ilps, return_inverse=True)
    table = np.empty((4, len(ulp), 4))
    for u, lp in enumerate(ulp.tolist()):
        for b in range(4):
            table[b, u] = base_distribution(b, lp)
    rows = table[bases[gi], inv.reshape(-1)]
    # bincount adds its weights in input order, i.e. per column in batch order
    flat = (jj[:, None] * 4 + np.arange(4)).ravel()
    probs += np.bincount(flat, weights=rows.ravel(), minlength=probs.size).reshape(probs.shape)


# ---------------------------------------------------------------------
# rifraf (model.jl:1116-1287)
# ---------------------------------------------------------------------

# Instrumentation (bench.py's per-stage kernel times): called with
# (iteration, stage) when an iteration starts and with (0, Stage.SCORE) before
# the quality pass.  None in normal use.
ITERATION_HOOK = None


def rifraf(dnaseqs, phreds=None, *, error_log_ps=None, consensus=None, reference=None,
           params: RifrafParams | None = None, engine: Engine | None = None) -> RifrafResult:
    """rifraf(dnaseqs, phreds; consensus, reference, params) -> RifrafResult.
    Pass `error_log_ps` instead of `phreds` for the log-probability method
    (model.jl:1116)."""
    params = params or RifrafParams()
    if error_log_ps is None:                                         # model.jl:1277-1287
        if any(np.min(p) < 0 for p in phreds):
            raise RifrafError("phred score cannot be negative")
        error_log_ps = [phred_to_log_p(p) for p in phreds]
    dnaseqs = [DNASeq(s) for s in dnaseqs]
    consensus = DNASeq(consensus) if consensus is not None else np.zeros(0, np.uint8)
    reference = DNASeq(reference) if reference is not None else np.zeros(0, np.uint8)
    check_params(params.scores, reference, params)
    sequences = [RifrafSequence(s, p, params.bandwidth, params.scores) for s, p in zip(dnaseqs, error_log_ps)]
    state = initial_state(consensus, sequences, reference, params)
    rng = BatchRng(params.seed)
    if engine is None:
        from .align import default_engine
        engine = default_engine()
    run = _Run(engine, len(sequences))
    engine.set_sequences(0, sequences)
    if len(state.reference) > 0:
        engine.set_sequences(run.REF, [state.reference])
    run.set_consensus(state.consensus)

    enabled = set()
    if params.do_init:
        enabled.add(Stage.INIT)
    if params.do_frame:
        enabled.add(Stage.FRAME)
    if params.do_refine:
        enabled.add(Stage.REFINE)
    if params.do_score:
        enabled.add(Stage.SCORE)
    consensus_stages = [[] for _ in range(int(Stage.SCORE) - 1)]
    state.realign_As = True
    state.realign_Bs = True
    old_score = -math.inf

    for it in range(1, params.max_iters + 1):
        while state.stage < Stage.SCORE and state.stage not in enabled:
            state.stage = Stage(int(state.stage) + 1)
        if state.stage == Stage.SCORE:
            break
        state.stage_iterations[int(state.stage) - 1] += 1
        consensus_stages[int(state.stage) - 1].append(state.consensus.copy())
        log(params, 1, f"iteration {it} : {state.stage.name} : {state.score}")
        if ITERATION_HOOK is not None:
            ITERATION_HOOK(it, state.stage)
        if params.verbose >= 3:
            log(params, 3, f"  consensus: {dna_str(state.consensus)}")
        else:
            log(params, 2, f"  consensus length: {len(state.consensus)}")
        log(params, 2, "  step: resample")
        resample(state, params, rng)
        log(params, 2, "  step: realign and rescore")
        realign_rescore(state, run, params)
        log(params, 2, "  step: check score")
        if check_score(state, run, params, old_score, rng):
            old_score = state.score
            state.penalties_increased = False
            indel_seeds = (single_indel_proposals(state, run)
                           if state.stage == Stage.FRAME and params.seed_indels else [])
            candidates = get_candidates(state, run, params, indel_seeds)
            state.realign_As = True
            if candidates:
                log(params, 2, "  step: handle candidates")
                handle_candidates(candidates, state, run, params)
            else:
                log(params, 2, "  step: finish_stage")
                finish_stage(state, run, params)
        else:
            finish_stage(state, run, params)
        if state.converged:
            break
        if ((not params.batch_fixed or (state.stage == Stage.REFINE and state.stage_iterations[2] > 1))
                and state.batch_size < len(state.sequences)):
            state.batch_randomness *= params.batch_mult
            log(params, 2, f"  batch randomness decreased to {state.batch_randomness}")
    state.stage = Stage.SCORE
    if ITERATION_HOOK is not None:
        ITERATION_HOOK(0, Stage.SCORE)
    result = RifrafResult(consensus=state.consensus, params=params, state=state,
                          consensus_stages=consensus_stages)
    if params.do_score:
        log(params, 2, "computing consensus quality scores")
        state.realign_As = True
        state.realign_Bs = True
        realign_rescore(state, run, params)
        result.error_probs = estimate_probs(state, run, params.use_ref_for_qvs)
        result.aln_error_probs = alignment_error_probs(len(state.consensus), state, run)
    log(params, 1, f"done. converged: {state.converged}")
    return result


def correct_shifts(consensus, reference, log_p: float = -1.0, bandwidth: int = -1,
                   scores: Scores | None = None, engine: Engine | None = None):   # :1303-1316
    """rifraf-style fast frameshift correction."""
    scores = scores or Scores.from_errors(ErrorModel(10.0, 1e-5, 1e-5, 1.0, 1.0))
    consensus, reference = DNASeq(consensus), DNASeq(reference)
    log_ps = np.full(len(reference), log_p)
    if bandwidth < 0:
        bandwidth = int(math.ceil(min(len(consensus), len(reference)) * 0.1))
    refseq = RifrafSequence(reference, log_ps, bandwidth, scores)
    if engine is None:
        from .align import default_engine
        engine = default_engine()
    run = _Run(engine, 0)
    run.set_consensus(consensus)
    state = RifrafState(consensus=consensus, ref_scores=scores, reference=refseq, batch_fixed_size=0,
                        batch_size=0, base_batch_size=0, sequences=[], maxlen=0)
    engine.set_sequences(run.REF, [refseq])
    proposals = single_indel_proposals(state, run)
    return apply_proposals(consensus, proposals)


def calibrate_phreds(s, phred, consensus, engine: Engine | None = None):   # :1295-1300
    from .align import Scratch, edit_distance
    e = engine or None
    n_errors = edit_distance(consensus, s, scratch=Scratch(e) if e else None)
    errors = np.power(10.0, phred_to_log_p(phred))
    return errors * float(n_errors) / errors.sum()
