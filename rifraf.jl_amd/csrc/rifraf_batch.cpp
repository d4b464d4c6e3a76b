// rifraf_batch.cpp -- native batched rifraf() stage machine (host C++).
//
// rf_rifraf_batch runs the INIT stage of rifraf() (src/model.jl:1116-1275)
// for many reference-free clusters in lockstep over one engine context: each
// step of the reference's iteration (resample -> realign! / rescore! ->
// check_score -> get_candidates -> handle_candidates! / finish_stage!) is
// executed for every live cluster with ONE batched engine call per kind
// (rf_realign, rf_backtrace, rf_alignment_proposals, rf_score,
// rf_set_templates_ids).  The per-cluster logic is the reference's, line by
// line (cited per function), with the same FP64 operations in the same order,
// so every cluster ends with the consensus, score and iteration count that a
// separate rifraf() call produces.  Python's batch.py hub does the same with
// one host thread per cluster; this driver removes that interpreter cost
// (SURVEY.md §8(f) row 1).
//
// Scope: every stage but SCORE (rf_rifraf_batch_ref adds FRAME and REFINE
// for clusters with a reference), fixed, full or random batches.  Random
// batches (resample!, model.jl:1038-1066) use rifraf_amd/resampling.py's
// RNG and draw (BatchRng, wsample_norep below), so both stage machines draw
// the same reads from the same seed.  Host inputs that need transcendental
// functions (the per-read Poisson thresholds of smart_forward_moves!, the
// fixed batch order) are computed by the caller with the Python mirror's own
// code, so no host libm result here can differ from the Python path's.

#include "../../include/rifraf_hip.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <utility>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>
#include <cstdlib>
#include <chrono>
#include <cstdio>

// rf_last_error text; the device form of rf_aln_error_sums (rifraf_hip.hip)
int rf_internal_fail(rf_ctx *ctx, int code, const char *msg);
// host worker threads (OMP_NUM_THREADS / machine, <= 16, <= the CPUs of this
// thread's affinity mask); defined in rifraf_hip.hip
int rf_internal_host_threads();
void rf_internal_arena_stats(const rf_ctx *ctx, int64_t *grows, double *secs);
int rf_internal_aln_sums_dev(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                             const int32_t *tlen, double *out);

namespace {

constexpr double INF = std::numeric_limits<double>::infinity();
constexpr int SUB = 0, INS = 1, DEL = 2;

struct Prop {
    int32_t kind, pos, base;
};
struct Cand {
    Prop p;
    double score;
};

// xoshiro256++ seeded by splitmix64; rand() = the top 53 bits
// (rifraf_amd/resampling.py BatchRng)
struct BatchRng {
    uint64_t s[4] = {0, 0, 0, 0};
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    void seed(uint64_t x)
    {
        for (int i = 0; i < 4; ++i) {
            x += 0x9E3779B97F4A7C15ull;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            s[i] = z ^ (z >> 31);
        }
    }
    uint64_t next()
    {
        const uint64_t r = rotl(s[0] + s[3], 23) + s[0];
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    double rand() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// resample!'s random batch (model.jl:1051-1054; resampling.py random_batch):
// weights 1 - err ./ sum(err), reweight (:1017-1036), then StatsBase 0.31's
// A-ExpJ draw without replacement (efraimidis_aexpj_wsample_norep!: keys
// w / Exp(1), exponential jumps, a min-heap of (key, index)); the batch is
// the n items by descending (key, index).  Sums run in index order; each
// product is its own statement (no contraction into an FMA); log1p / exp /
// log are the libm calls CPython's math module makes.  Returns false (the
// message in `err`) when fewer than n weights are > 0 or one is negative.
static bool random_batch(BatchRng &rng, const double *est, int n, int k, double randomness,
                         std::vector<int32_t> &out, std::string &err)
{
    double se = 0.0;
    for (int i = 0; i < n; ++i)
        se += est[i];
    std::vector<double> w(n), e(n);
    for (int i = 0; i < n; ++i)
        w[i] = 1.0 - est[i] / se;
    double sw = 0.0;
    for (int i = 0; i < n; ++i)
        sw += w[i];
    for (int i = 0; i < n; ++i)
        w[i] = w[i] / sw;
    double weight = 0.0;
    if (randomness > 0.5) {
        weight = (randomness - 0.5) * 2.0;
        for (int i = 0; i < n; ++i)
            e[i] = 1.0 / n;
    } else if (randomness < 0.5) {
        weight = 1.0 - randomness * 2.0;
        // reverse(sortperm(w))[1:k]: a stable ascending order, read from its end
        std::vector<int32_t> ord(n);
        for (int i = 0; i < n; ++i)
            ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return w[a] < w[b]; });
        std::fill(e.begin(), e.end(), 0.0);
        for (int i = 0; i < k; ++i)
            e[ord[n - 1 - i]] = 1.0 / k;
    } else {
        e = w;
    }
    const double keep = 1.0 - weight;
    for (int i = 0; i < n; ++i) {
        const double a = weight * e[i];
        const double b = keep * w[i];
        w[i] = a + b;
    }
    auto randexp = [&rng] { return -std::log1p(-rng.rand()); };
    using Key = std::pair<double, int32_t>;
    std::priority_queue<Key, std::vector<Key>, std::greater<Key>> pq;   // min-heap of (key, index)
    int s = 0;
    for (; s < n && (int)pq.size() < k; ++s) {
        if (w[s] < 0) {
            err = "Negative weight found in weight vector at index " + std::to_string(s + 1);
            return false;
        }
        if (w[s] > 0)
            pq.push({w[s] / randexp(), s});
    }
    if ((int)pq.size() < k) {
        err = "wv must have at least " + std::to_string(k) + " strictly positive entries (got " +
              std::to_string(pq.size()) + ")";
        return false;
    }
    double threshold = pq.top().first;
    double x = threshold * randexp();
    for (int i = s; i < n; ++i) {
        const double wi = w[i];
        if (wi < 0) {
            err = "Negative weight found in weight vector at index " + std::to_string(i + 1);
            return false;
        }
        if (!(wi > 0))
            continue;
        x -= wi;
        if (!(x <= 0))
            continue;
        const double t = std::exp(-wi / threshold);
        const double m = rng.rand() * (1.0 - t);
        const double key = -wi / std::log(t + m);
        pq.pop();
        pq.push({key, i});
        threshold = pq.top().first;
        x = threshold * randexp();
    }
    out.resize(k);
    for (int d = k - 1; d >= 0; --d) {   // ascending pops fill the batch from its end
        out[d] = pq.top().second;
        pq.pop();
    }
    return true;
}

struct Read {
    int32_t seq = 0, len = 0, bw = 0;
    bool fixed = false;
    double thr = 0.0;   // cquantile(Poisson(est_n_errors), bandwidth_pvalue)
};

// stages (model.jl:1-5)
constexpr int ST_INIT = 1, ST_FRAME = 2, ST_REFINE = 3, ST_SCORE = 4;

struct Clu {
    int32_t r0 = 0, nreads = 0;   // reads [r0, r0 + nreads) of the read table
    int32_t slot0 = 0, tpl = 0;
    std::vector<uint8_t> cons, old_cons;
    std::vector<std::vector<uint8_t>> stages;   // consensus at each iteration
    std::vector<int8_t> stage_of;               // ... and the stage it ran in
    std::vector<int32_t> batch;                 // batch_seqs (local read indices)
    int32_t batch_size = 0, base_batch_size = 0;
    int32_t n_slots = 0;
    std::vector<double> slot_scores;
    double score = -INF, old_score = -INF;
    bool realign_As = true, realign_Bs = true, penalties_increased = false;
    int32_t iters = 0;                          // all stages
    int32_t stage = ST_INIT, stage_iters[3] = {0, 0, 0};
    bool converged = false, failed = false, done = false;
    std::string err;
    std::vector<Prop> props;
    std::vector<Cand> chosen;
    // reference (model.jl:167-193): its read-table entry (sequence id, length,
    // bandwidth, threshold), A/B slot, scratch slot for one-off alignments,
    // the edit-distance copy of its sequence (align.jl:253-260) and its bases
    bool has_ref = false;
    int32_t ref_read = -1, ref_slot = -1, scratch_slot = -1, edit_seq = -1;
    std::vector<uint8_t> ref_bases;
    double ref_score = -INF;
    int32_t n_ref_indel_mults = 0;
    std::vector<Prop> seeds;                    // FRAME indel seeds
    // the scratch slot already holds single_indel_proposals' skewed fill of
    // the reference against this consensus (filled beside the B realign)
    bool sip_pre = false;
    // the reference slot's A band is the forward fill of this consensus at
    // the reference's bandwidth (smart_forward in FRAME): has_single_indels'
    // align_moves (model.jl:532-536) is the same fill, so its walk reads it
    bool ref_a_ok = false;
    double batch_randomness = 0.9;              // state.batch_randomness (model.jl:177)
    BatchRng rng;                               // resample!'s random batches
};

struct Driver {
    rf_ctx *ctx;
    rf_batch_params P;
    rf_batch_ref_params RP{};
    rf_ref_callback cb = nullptr;
    void *cb_user = nullptr;
    std::vector<Read> reads;
    std::vector<Clu> clu;
    std::vector<int32_t> fixed_off, fixed;   // the caller's fixed batches

    // RIFRAF_BATCH_TIMING: wall time and count of each engine call kind
    // (stderr at the end of rf_rifraf_batch; diagnostics only)
    enum { T_FWD, T_BT, T_BWD, T_PROPS, T_SCORE, T_TPL, T_N };
    double tsum[T_N] = {};
    double ksum[T_N] = {};   // the calls' kernel time (HIP events), seconds
    int tcnt[T_N] = {};
    const bool timing = [] {
        const char *tv = std::getenv("RIFRAF_BATCH_TIMING");
        return tv && *tv && *tv != '0';
    }();
    template <class F>
    int timed(int k, F &&call)
    {
        const auto t0 = std::chrono::steady_clock::now();
        const int e = call();
        tsum[k] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        ++tcnt[k];
        if (timing && e == 0) {
            double dp = 0, sc = 0, ga = 0, bt = 0;
            rf_last_timing(ctx, &dp, &sc, &ga);
            rf_last_backtrace_ms(ctx, &bt);
            ksum[k] += 1e-3 * (k == T_FWD || k == T_BWD ? dp : k == T_SCORE ? sc + ga
                               : (k == T_BT || k == T_PROPS) ? bt : 0.0);
        }
        return e;
    }

    void fail_cluster(int c, const std::string &msg)
    {
        clu[c].failed = true;
        clu[c].err = msg;
    }

    // Run `fn` on the clusters `cs` in one batched engine call; if the call
    // fails, run it cluster by cluster so the error reaches exactly the
    // cluster that raised it (batch.py's attribution).  fn returns 0 or an
    // rf error code and must not change cluster state unless it succeeds.
    template <class F>
    void batched(std::vector<int> &cs, F fn)
    {
        if (cs.empty())
            return;
        if (fn(cs) == 0)
            return;
        std::vector<int> ok;
        for (int c : cs) {
            std::vector<int> one{c};
            if (fn(one) == 0)
                ok.push_back(c);
            else
                fail_cluster(c, rf_last_error(ctx));
        }
        cs.swap(ok);
    }

    // ---------------- resample! (model.jl:1038-1066)
    void resample(Clu &C, int c)
    {
        if (P.batch_fixed && (C.stage == ST_INIT || C.stage == ST_FRAME)) {
            C.batch.assign(fixed.begin() + fixed_off[c], fixed.begin() + fixed_off[c + 1]);
        } else if (C.batch_size < C.nreads) {
            std::string err;
            if (!random_batch(C.rng, P.est_n_errors + C.r0, C.nreads, C.batch_size, C.batch_randomness, C.batch,
                              err))
                fail_cluster(c, err);
            C.realign_As = true;
        } else {
            C.batch.resize(C.nreads);
            for (int k = 0; k < C.nreads; ++k)
                C.batch[k] = k;
        }
    }

    // ---------------- smart_forward_moves! (model.jl:643-672) over the
    // batch slots of every cluster in `cs`, then A[end,end] -> slot_scores.
    // use_ref (model.jl:617-628) inside the stage machine: FRAME only
    bool ref_on(const Clu &C) const { return C.has_ref && C.stage == ST_FRAME; }

    int smart_forward(const std::vector<int> &cs)
    {
        struct Job {
            int c, k;          // k = batch index, -1 = the reference
            int32_t slot, ridx;
            int32_t bw, max_bw;
            int64_t old_err, n_err;
        };
        std::vector<Job> jobs;
        for (int c : cs) {
            const Clu &C = clu[c];
            auto add = [&](int k, int32_t slot, int32_t ridx) {
                const Read &R = reads[ridx];
                const int32_t mx = R.fixed ? R.bw
                                           : std::min<int64_t>(std::min<int64_t>((int64_t)R.bw * 32, (int64_t)C.cons.size()),
                                                               (int64_t)R.len);
                jobs.push_back({c, k, slot, ridx, R.bw, mx, INT64_MAX, INT64_MAX});
            };
            for (int k = 0; k < (int)C.batch.size(); ++k)
                add(k, C.slot0 + k, C.r0 + C.batch[k]);
            if (ref_on(C))   // model.jl:695-698: the reference after the batch (independent slots)
                add(-1, C.ref_slot, C.ref_read);
        }
        std::vector<double> score(jobs.size());
        std::vector<int> pending(jobs.size());
        for (size_t j = 0; j < jobs.size(); ++j)
            pending[j] = (int)j;
        std::vector<int32_t> sl, sq, tp, bw, nerr;
        std::vector<double> out;
        while (!pending.empty()) {
            sl.clear(), sq.clear(), tp.clear(), bw.clear();
            for (int j : pending) {
                sl.push_back(jobs[j].slot);
                sq.push_back(reads[jobs[j].ridx].seq);
                tp.push_back(clu[jobs[j].c].tpl);
                bw.push_back(jobs[j].bw);
            }
            out.resize(pending.size());
            if (int e = timed(T_FWD, [&] {
                    return rf_realign(ctx, (int32_t)pending.size(), sl.data(), sq.data(), tp.data(), bw.data(),
                                      RF_FWD, out.data());
                }))
                return e;
            std::vector<int> check;
            for (size_t i = 0; i < pending.size(); ++i) {
                const int j = pending[i];
                score[j] = out[i];
                if (!(reads[jobs[j].ridx].fixed || jobs[j].bw >= jobs[j].max_bw))
                    check.push_back(j);
            }
            if (check.empty())
                break;
            sl.clear();
            for (int j : check)
                sl.push_back(jobs[j].slot);
            nerr.resize(check.size());
            if (int e = timed(T_BT, [&] {
                    return rf_backtrace(ctx, (int32_t)check.size(), sl.data(), nullptr, nullptr, nullptr, nerr.data());
                }))
                return e;
            std::vector<int> nxt;
            for (size_t i = 0; i < check.size(); ++i) {
                Job &J = jobs[check[i]];
                const Read &R = reads[J.ridx];
                J.old_err = J.n_err;
                J.n_err = nerr[i];
                if ((double)J.n_err > R.thr && J.n_err < J.old_err) {
                    J.bw = std::min(J.bw * 2, J.max_bw);
                    nxt.push_back(check[i]);
                }
            }
            pending.swap(nxt);
        }
        // success: commit bandwidths (bandwidth_fixed) and scores
        for (size_t j = 0; j < jobs.size(); ++j) {
            Clu &C = clu[jobs[j].c];
            Read &R = reads[jobs[j].ridx];
            R.bw = jobs[j].bw;
            R.fixed = true;
            if (jobs[j].k >= 0) {
                C.slot_scores[jobs[j].k] = score[j];
            } else {
                C.ref_score = score[j];
                C.ref_a_ok = true;
            }
        }
        return 0;
    }

    // backward! of every batch read (and the reference in FRAME); round 5:
    // in FRAME with seeded indels also single_indel_proposals' skewed
    // forward fill of the reference against the same consensus
    // (model.jl:538-562, align_moves(skew_matches=true)) into the scratch
    // slot, in the same launch set: the reference's long latency-bound fill
    // runs beside the reads' instead of after them.  The stage machine's
    // order is unchanged (the fill reads only the consensus and the
    // reference, which do not change before single_indel_proposals).
    int realign_B(const std::vector<int> &cs)
    {
        std::vector<int32_t> sl, sq, tp, bw, fl;
        std::vector<int> pre;
        for (int c : cs) {
            const Clu &C = clu[c];
            for (int k = 0; k < (int)C.batch.size(); ++k) {
                const Read &R = reads[C.r0 + C.batch[k]];
                sl.push_back(C.slot0 + k);
                sq.push_back(R.seq);
                tp.push_back(C.tpl);
                bw.push_back(R.bw);
                fl.push_back(RF_BWD);
            }
            if (ref_on(C)) {   // model.jl:710-712
                const Read &R = reads[C.ref_read];
                sl.push_back(C.ref_slot);
                sq.push_back(R.seq);
                tp.push_back(C.tpl);
                bw.push_back(R.bw);
                fl.push_back(RF_BWD);
                if (RP.seed_indels) {
                    sl.push_back(C.scratch_slot);
                    sq.push_back(R.seq);
                    tp.push_back(C.tpl);
                    bw.push_back(R.bw);
                    fl.push_back(RF_FWD | RF_SKEW);
                    pre.push_back(c);
                }
            }
        }
        const int e = timed(T_BWD, [&] {
            return rf_realign_jobs(ctx, (int32_t)sl.size(), sl.data(), sq.data(), tp.data(), bw.data(), fl.data(),
                                   nullptr);
        });
        if (e == 0)
            for (int c : pre)
                clu[c].sip_pre = true;
        return e;
    }

    // ---------------- realign! + rescore! (model.jl:630-719), no reference
    void realign_rescore(std::vector<int> cs)
    {
        std::vector<int> a, b;
        for (int c : cs) {
            Clu &C = clu[c];
            if (C.failed)
                continue;
            while (C.n_slots < (int)C.batch.size()) {   // grow As / Bs (fresh A[end,end] = 0.0)
                C.slot_scores.push_back(0.0);
                ++C.n_slots;
            }
            if (C.realign_As)
                a.push_back(c);
            if (C.realign_Bs)
                b.push_back(c);
        }
        batched(a, [&](const std::vector<int> &s) { return smart_forward(s); });
        batched(b, [&](const std::vector<int> &s) { return realign_B(s); });
        for (int c : cs) {
            Clu &C = clu[c];
            if (C.failed)
                continue;
            double total = C.slot_scores[0];   // left fold over every slot, stale ones included
            for (int k = 1; k < C.n_slots; ++k)
                total += C.slot_scores[k];
            if (ref_on(C))                     // rescore!: + A_ref[end, end] (model.jl:630-635)
                total += C.ref_score;
            C.score = total;
        }
    }

    // ---------------- check_score (model.jl:1074-1114); the clusters that
    // increase their batch size are realigned by the caller (`redo`)
    bool check_score(Clu &C, int c, std::vector<int> &redo)
    {
        const bool all = C.batch_size == C.nreads;
        const int32_t sit = C.stage_iters[C.stage - 1];
        if (!C.penalties_increased && all && sit > 1) {
            if (C.score == C.old_score)
                return false;
        }
        const double rel = (C.score - C.old_score) / C.old_score;   // IEEE: +-Inf / NaN, never a trap
        if (rel > P.batch_threshold && !C.penalties_increased && C.batch_size < C.nreads && sit > 1) {
            C.batch_size = std::min(C.batch_size + C.base_batch_size, C.nreads);
            resample(C, c);
            C.realign_As = true;
            C.realign_Bs = true;
            redo.push_back(c);
        }
        return true;
    }

    // ---------------- all_proposals (model.jl:401-456): indel seeds widen to
    // +-CODON_LENGTH positions; subs unless FRAME with indel_correction_only;
    // indels in INIT / FRAME (SCORE does not reach the driver)
    void all_proposals(int stage, const std::vector<uint8_t> &t, const std::vector<Prop> &seeds,
                       std::vector<Prop> &out) const
    {
        const int len = (int)t.size(), nb = 3;
        std::vector<uint8_t> ins_pos(len + 1, 0), del_pos(len + 1, 0);
        for (const Prop &p : seeds) {
            if (p.kind == INS) {
                for (int j = std::max(p.pos - nb, 0); j <= std::min(p.pos + nb, len); ++j)
                    ins_pos[j] = 1;
            } else {
                for (int j = std::max(p.pos - nb, 1); j <= std::min(p.pos + nb, len); ++j)
                    del_pos[j] = 1;
            }
        }
        const bool do_subs = stage != ST_FRAME || !RP.indel_correction_only;
        const bool do_indels = stage == ST_INIT || stage == ST_FRAME;
        const bool no_seeds = seeds.empty();
        out.clear();
        if (do_indels)
            for (int b = 0; b < 4; ++b)
                out.push_back({INS, 0, b});
        for (int j = 1; j <= len; ++j) {
            if (do_subs)
                for (int b = 0; b < 4; ++b)
                    if (t[j - 1] != b)
                        out.push_back({SUB, j, b});
            if (do_indels) {
                if (no_seeds || del_pos[j])
                    out.push_back({DEL, j, 0});
                if (no_seeds || ins_pos[j])
                    for (int b = 0; b < 4; ++b)
                        out.push_back({INS, j, b});
            }
        }
    }

    // ---------------- the reference aligned to the consensus (align_moves,
    // align.jl:337-344; model.jl:532-562): forward fill of the reference
    // (rows) against the consensus in the cluster's scratch slot with the
    // reference's bandwidth, then the backtrace moves
    int ref_moves(const std::vector<int> &cs, bool skew, std::vector<std::vector<int8_t>> &mv,
                  bool filled = false, bool ref_slot = false)
    {
        std::vector<int32_t> sl, sq, tp, bw, nm(cs.size());
        std::vector<int64_t> moff{0};
        for (int c : cs) {
            const Clu &C = clu[c];
            const Read &R = reads[C.ref_read];
            sl.push_back(ref_slot ? C.ref_slot : C.scratch_slot);
            sq.push_back(R.seq);
            tp.push_back(C.tpl);
            bw.push_back(R.bw);
            moff.push_back(moff.back() + R.len + (int64_t)C.cons.size());
        }
        if (!filled) {   // (filled: the scratch slot holds this fill already, realign_B)
            for (int c : cs)
                clu[c].sip_pre = false;   // any other write to the scratch slot ends the cached fill
            if (int e = timed(T_FWD, [&] {
                    return rf_realign(ctx, (int32_t)cs.size(), sl.data(), sq.data(), tp.data(), bw.data(),
                                      RF_FWD | (skew ? RF_SKEW : 0), nullptr);
                }))
                return e;
        }
        std::vector<int8_t> moves((size_t)std::max<int64_t>(moff.back(), 1));
        if (int e = timed(T_BT, [&] {
                return rf_backtrace(ctx, (int32_t)cs.size(), sl.data(), moves.data(), moff.data(), nm.data(), nullptr);
            }))
            return e;
        mv.resize(cs.size());
        for (size_t i = 0; i < cs.size(); ++i)
            mv[i].assign(moves.begin() + moff[i], moves.begin() + moff[i] + nm[i]);
        return 0;
    }

    // has_single_indels (model.jl:532-536) of clusters `cs` -> flags
    // (round 6: a cluster whose reference A band is current -- FRAME, the
    // consensus and reference unchanged since smart_forward -- walks that
    // band instead of refilling the scratch slot: the same fill, so the same
    // moves, one latency-bound codon fill less per FRAME iteration)
    void has_single_indels(std::vector<int> &cs, std::vector<uint8_t> &flag)
    {
        flag.assign(clu.size(), 0);
        std::vector<int> fill, cur;
        for (int c : cs)
            (clu[c].ref_a_ok ? cur : fill).push_back(c);
        for (int pass = 0; pass < 2; ++pass)
            batched(pass ? cur : fill, [&](const std::vector<int> &s) {
                std::vector<std::vector<int8_t>> mv;
                if (int e = ref_moves(s, false, mv, pass == 1, pass == 1))
                    return e;
                for (size_t i = 0; i < s.size(); ++i)
                    for (int8_t m : mv[i])
                        flag[s[i]] |= (m == 2 || m == 3);   // TRACE_INSERT / TRACE_DELETE
                return 0;
            });
        // the clusters left (batched drops a failing one), in the callers' order
        std::vector<uint8_t> left(clu.size(), 0);
        for (int c : fill)
            left[c] = 1;
        for (int c : cur)
            left[c] = 1;
        std::vector<int> kept;
        for (int c : cs)
            if (left[c])
                kept.push_back(c);
        cs.swap(kept);
    }

    // single_indel_proposals (model.jl:538-562) -> clu[c].seeds; clusters whose
    // skewed fill ran beside their B realign (sip_pre) take only the walk
    void single_indel_proposals(std::vector<int> &cs)
    {
        std::vector<int> pre, rest;
        for (int c : cs)
            (clu[c].sip_pre ? pre : rest).push_back(c);
        single_indel_proposals_(pre, true);
        single_indel_proposals_(rest, false);
        cs = pre;
        cs.insert(cs.end(), rest.begin(), rest.end());
    }
    void single_indel_proposals_(std::vector<int> &cs, bool filled)
    {
        batched(cs, [&](const std::vector<int> &s) {
            std::vector<std::vector<int8_t>> mv;
            if (int e = ref_moves(s, true, mv, filled))
                return e;
            for (size_t i = 0; i < s.size(); ++i) {
                Clu &C = clu[s[i]];
                C.seeds.clear();
                int cons_idx = 0, ref_idx = 0;
                for (int8_t m : mv[i]) {
                    switch (m) {
                    case 1: ++cons_idx, ++ref_idx; break;                                   // MATCH
                    case 2: ++ref_idx; C.seeds.push_back({INS, cons_idx, C.ref_bases[ref_idx - 1]}); break;
                    case 3: ++cons_idx; C.seeds.push_back({DEL, cons_idx, 0}); break;       // DELETE
                    case 4: ref_idx += 3; break;                                             // CODON_INSERT
                    case 5: cons_idx += 3; break;                                            // CODON_DELETE
                    default: break;
                    }
                }
            }
            return 0;
        });
    }

    // ---------------- get_candidates (model.jl:499-526) for `cs`; returns the
    // candidates (score > state.score, in proposal order) per cluster
    void get_candidates(std::vector<int> cs, std::vector<std::vector<Cand>> &cands)
    {
        // alignment_proposals (model.jl:483-497) in INIT (with indels) and
        // REFINE (substitutions only): the device union mask of the batch
        // backtraces, read out in (pos, kind, base) order
        for (int indels = 1; indels >= 0; --indels) {
            std::vector<int> ap;
            for (int c : cs)
                if (P.do_alignment_proposals && clu[c].stage == (indels ? ST_INIT : ST_REFINE))
                    ap.push_back(c);
            batched(ap, [&](const std::vector<int> &s) {
                std::vector<int32_t> off{0}, sl;
                int64_t rows = 0;
                for (int c : s) {
                    for (int k = 0; k < (int)clu[c].batch.size(); ++k)
                        sl.push_back(clu[c].slot0 + k);
                    off.push_back((int32_t)sl.size());
                    rows += (int64_t)clu[c].cons.size() + 1;
                }
                std::vector<uint8_t> mask((size_t)rows * 9);
                if (int e = timed(T_PROPS, [&] {
                        return rf_alignment_proposals(ctx, (int32_t)s.size(), off.data(), sl.data(), indels,
                                                      mask.data());
                    }))
                    return e;
                static const int order[9][3] = {{0, SUB, 0}, {1, SUB, 1}, {2, SUB, 2}, {3, SUB, 3}, {5, INS, 0},
                                                {6, INS, 1}, {7, INS, 2}, {8, INS, 3}, {4, DEL, 0}};
                int64_t row = 0;
                for (int c : s) {
                    Clu &C = clu[c];
                    C.props.clear();
                    const int m = (int)C.cons.size();
                    for (int p = 0; p <= m; ++p)
                        for (const auto &o : order)
                            if (mask[(size_t)(row + p) * 9 + o[0]])
                                C.props.push_back({o[1], p, o[2]});
                    row += m + 1;
                }
                return 0;
            });
        }
        for (int c : cs) {
            Clu &C = clu[c];
            if (C.failed || ((C.stage == ST_INIT || C.stage == ST_REFINE) && P.do_alignment_proposals))
                continue;
            static const std::vector<Prop> none;
            all_proposals(C.stage, C.cons, C.stage == ST_FRAME ? C.seeds : none, C.props);
        }
        // score_proposals (model.jl:385-399): batch fold, + the reference in FRAME
        std::vector<int> sc;
        for (int c : cs)
            if (!clu[c].failed && !clu[c].props.empty())
                sc.push_back(c);
        batched(sc, [&](const std::vector<int> &s) {
            std::vector<int32_t> off{0}, sl, ref, pos;
            std::vector<int64_t> poff{0};
            std::vector<uint8_t> kind, base;
            for (int c : s) {
                const Clu &C = clu[c];
                for (int k = 0; k < (int)C.batch.size(); ++k)
                    sl.push_back(C.slot0 + k);
                off.push_back((int32_t)sl.size());
                ref.push_back(C.stage == ST_FRAME ? C.ref_slot : -1);
                for (const Prop &p : C.props) {
                    kind.push_back((uint8_t)p.kind);
                    pos.push_back(p.pos);
                    base.push_back((uint8_t)p.base);
                }
                poff.push_back((int64_t)kind.size());
            }
            std::vector<double> tot(kind.size());
            if (int e = timed(T_SCORE, [&] {
                    return rf_score(ctx, (int32_t)s.size(), off.data(), sl.data(), ref.data(), poff.data(),
                                    kind.data(), pos.data(), base.data(), tot.data(), nullptr);
                }))
                return e;
            for (size_t g = 0; g < s.size(); ++g) {
                const Clu &C = clu[s[g]];
                auto &out = cands[s[g]];
                out.clear();
                for (int64_t i = poff[g]; i < poff[g + 1]; ++i)
                    if (tot[i] > C.score)
                        out.push_back({C.props[i - poff[g]], tot[i]});
            }
            return 0;
        });
    }

    // ---------------- choose_candidates (proposals.jl:104-115)
    std::vector<Cand> choose(std::vector<Cand> cands) const
    {
        std::stable_sort(cands.begin(), cands.end(), [](const Cand &x, const Cand &y) { return x.score > y.score; });
        std::vector<Cand> out;
        for (const Cand &c : cands) {
            bool near = false;
            for (const Cand &o : out)
                near = near || std::abs(c.p.pos - o.p.pos) < P.min_dist;
            if (!near)
                out.push_back(c);
        }
        return out;
    }

    // ---------------- apply_proposals (proposals.jl:41-102); false: ambiguous
    static bool apply(const std::vector<uint8_t> &seq, std::vector<Cand> ps, std::vector<uint8_t> &out)
    {
        std::vector<int> ins, other;
        for (const Cand &c : ps)
            (c.p.kind == INS ? ins : other).push_back(c.p.pos);
        for (auto *v : {&ins, &other}) {
            std::sort(v->begin(), v->end());
            if (std::adjacent_find(v->begin(), v->end()) != v->end())
                return false;
        }
        std::stable_sort(ps.begin(), ps.end(), [](const Cand &x, const Cand &y) {
            const int kx = x.p.kind == DEL ? 0 : 1, ky = y.p.kind == DEL ? 0 : 1;
            return x.p.pos != y.p.pos ? x.p.pos < y.p.pos : kx < ky;
        });
        out.clear();
        int nxt = 1, last_del = 0;
        for (const Cand &c : ps) {
            const Prop &p = c.p;
            for (int i = nxt - 1; i < std::max(p.pos - 1, 0); ++i)
                out.push_back(seq[i]);
            if (p.kind == SUB) {
                out.push_back((uint8_t)p.base);
            } else if (p.kind == INS) {
                if (p.pos > 0 && last_del != p.pos)
                    out.push_back(seq[p.pos - 1]);
                out.push_back((uint8_t)p.base);
            }
            nxt = p.pos + 1;
            if (p.kind == DEL)
                last_del = p.pos;
        }
        for (int i = nxt - 1; i < (int)seq.size(); ++i)
            out.push_back(seq[i]);
        return true;
    }

    int upload_templates(const std::vector<int> &cs)
    {
        std::vector<int32_t> ids;
        std::vector<int64_t> off{0};
        std::vector<uint8_t> bases;
        for (int c : cs) {
            ids.push_back(clu[c].tpl);
            bases.insert(bases.end(), clu[c].cons.begin(), clu[c].cons.end());
            off.push_back((int64_t)bases.size());
        }
        return timed(T_TPL, [&] {
            return rf_set_templates_ids(ctx, (int32_t)ids.size(), ids.data(), bases.data(), off.data());
        });
    }

    // Set the consensus of clusters `cs` (host copy + device template);
    // a cluster whose upload fails keeps its error.
    void set_consensus(std::vector<int> &cs)
    {
        for (int c : cs)
            clu[c].ref_a_ok = false;
        batched(cs, [&](const std::vector<int> &s) { return upload_templates(s); });
    }

    // ---------------- handle_candidates! (model.jl:898-935)
    void handle_candidates(std::vector<int> cs, std::vector<std::vector<Cand>> &cands)
    {
        std::vector<int> up;
        for (int c : cs) {
            Clu &C = clu[c];
            C.old_cons = C.cons;
            C.chosen = choose(cands[c]);
            std::vector<uint8_t> nc;
            if (!apply(C.old_cons, C.chosen, nc)) {
                fail_cluster(c, "AmbiguousProposalsError");
                continue;
            }
            C.cons.swap(nc);
            up.push_back(c);
        }
        set_consensus(up);
        for (int c : up) {
            clu[c].realign_As = true;
            clu[c].realign_Bs = false;
        }
        realign_rescore(up);
        std::vector<int> redo;
        for (int c : up) {
            Clu &C = clu[c];
            if (C.failed)
                continue;
            const double best = C.chosen[0].score;
            const bool close = C.score == best ||
                               (std::isfinite(C.score) && std::isfinite(best) &&
                                std::fabs(C.score - best) <= std::sqrt(DBL_EPSILON_) * std::max(std::fabs(C.score), std::fabs(best)));
            if (C.chosen.size() > 1 && (C.score < best || close)) {
                // reject multiple candidates in favor of the best
                C.chosen.resize(1);
                std::vector<uint8_t> nc;
                apply(C.old_cons, C.chosen, nc);
                C.cons.swap(nc);
                redo.push_back(c);
            } else {
                C.realign_As = false;
            }
            C.realign_Bs = true;
        }
        set_consensus(redo);
    }
    static constexpr double DBL_EPSILON_ = std::numeric_limits<double>::epsilon();

    // ---------------- finish_stage! (model.jl:937-995)
    void finish_stage(std::vector<int> cs)
    {
        std::vector<int> to_frame, in_frame;
        for (int c : cs) {
            Clu &C = clu[c];
            if (C.failed)
                continue;
            if (C.stage == ST_INIT) {
                if (!C.has_ref || !RP.do_frame)
                    C.converged = true;
                else
                    to_frame.push_back(c);
            } else if (C.stage == ST_FRAME) {
                in_frame.push_back(c);
            } else if (C.stage == ST_REFINE) {
                C.converged = true;
            } else {
                fail_cluster(c, "  invalid stage: " + std::to_string(C.stage));
            }
        }
        std::vector<uint8_t> flag;
        if (!to_frame.empty()) {
            // edit_distance(consensus, reference) (align.jl:253-260): the errors of
            // the skewed alignment of the reference's edit-distance copy (log p
            // -1, ErrorModel(1, 1, 1) scores) at bandwidth ceil(min(len) * 0.5)
            std::vector<int64_t> ed(clu.size(), 0);
            batched(to_frame, [&](const std::vector<int> &s) {
                std::vector<int32_t> sl, sq, tp, bw, nerr(s.size());
                for (int c : s) {
                    Clu &C = clu[c];
                    C.sip_pre = false;   // the scratch slot takes edit_distance's band
                    sl.push_back(C.scratch_slot);
                    sq.push_back(C.edit_seq);
                    tp.push_back(C.tpl);
                    const int64_t mn = std::min<int64_t>((int64_t)C.cons.size(), (int64_t)C.ref_bases.size());
                    bw.push_back((int32_t)((mn + 1) / 2));
                }
                if (int e = timed(T_FWD, [&] {
                        return rf_realign(ctx, (int32_t)s.size(), sl.data(), sq.data(), tp.data(), bw.data(),
                                          RF_FWD | RF_SKEW, nullptr);
                    }))
                    return e;
                if (int e = timed(T_BT, [&] {
                        return rf_backtrace(ctx, (int32_t)s.size(), sl.data(), nullptr, nullptr, nullptr, nerr.data());
                    }))
                    return e;
                for (size_t i = 0; i < s.size(); ++i)
                    ed[s[i]] = nerr[i];
                return 0;
            });
            std::vector<int> entered;
            for (int c : to_frame) {
                Clu &C = clu[c];
                C.stage = ST_FRAME;
                double rate = (double)ed[c] / (double)std::max(C.ref_bases.size(), C.cons.size());
                rate *= RP.ref_error_mult;
                rate = std::min(std::max(rate, 1e-10), 0.5);
                double thr = 0.0;
                C.ref_a_ok = false;   // a new reference
                // the caller builds the reference with log p = log10(rate) and
                // uploads it (rifrafsequences.jl constructor), returns its threshold
                if (cb(cb_user, c, 0, rate, &thr) != 0) {
                    fail_cluster(c, "reference callback failed (FRAME entry)");
                    continue;
                }
                Read &R = reads[C.ref_read];
                R.bw = P.bandwidth;
                R.fixed = false;
                R.thr = thr;
                entered.push_back(c);
            }
            has_single_indels(entered, flag);
            for (int c : entered)
                if (!clu[c].failed && !flag[c])
                    clu[c].converged = true;
        }
        if (!in_frame.empty()) {
            has_single_indels(in_frame, flag);
            for (int c : in_frame) {
                Clu &C = clu[c];
                if (C.failed)
                    continue;
                if (!flag[c]) {
                    C.stage = ST_REFINE;
                } else if (C.n_ref_indel_mults == RP.max_ref_indel_mults) {
                    C.stage = ST_REFINE;   // single indels remain, penalty limit reached
                } else {
                    C.penalties_increased = true;
                    if (C.n_ref_indel_mults < RP.max_ref_indel_mults) {
                        C.n_ref_indel_mults += 1;
                    } else {
                        fail_cluster(c, "Tried to illegally increase n_ref_indel_mults");
                        continue;
                    }
                    double thr = 0.0;
                    C.ref_a_ok = false;   // new indel scores
                    // the caller rescales the reference's indel scores and re-uploads it
                    if (cb(cb_user, c, 1, (double)C.n_ref_indel_mults, &thr) != 0)
                        fail_cluster(c, "reference callback failed (penalty increase)");
                }
            }
        }
    }

    bool enabled(int stage) const
    {
        return stage == ST_INIT || (stage == ST_FRAME && RP.do_frame) || (stage == ST_REFINE && RP.do_refine);
    }

    void run()
    {
        std::vector<int> live;
        for (int c = 0; c < (int)clu.size(); ++c)
            live.push_back(c);
        std::vector<std::vector<Cand>> cands(clu.size());
        for (int it = 1; it <= P.max_iters && !live.empty(); ++it) {
            std::vector<int> act;
            for (int c : live) {
                Clu &C = clu[c];
                while (C.stage < ST_SCORE && !enabled(C.stage))
                    ++C.stage;
                if (C.stage == ST_SCORE) {
                    C.done = true;
                    continue;
                }
                C.iters += 1;
                C.stage_iters[C.stage - 1] += 1;
                C.stages.push_back(C.cons);
                C.stage_of.push_back((int8_t)C.stage);
                resample(C, c);
                act.push_back(c);
            }
            realign_rescore(act);
            std::vector<int> ok, redo, fin;
            for (int c : act) {
                if (clu[c].failed)
                    continue;
                if (check_score(clu[c], c, redo))
                    ok.push_back(c);
                else
                    fin.push_back(c);
            }
            if (!redo.empty())
                realign_rescore(redo);
            std::vector<int> gc, sd;
            for (int c : ok) {
                Clu &C = clu[c];
                if (C.failed)
                    continue;
                C.old_score = C.score;
                C.penalties_increased = false;
                gc.push_back(c);
                if (C.stage == ST_FRAME && RP.seed_indels)
                    sd.push_back(c);
                else
                    C.seeds.clear();
            }
            single_indel_proposals(sd);
            for (int c : act)
                clu[c].sip_pre = false;   // the scratch slot is refilled from here on (has_single_indels)
            for (int c : gc)
                cands[c].clear();
            get_candidates(gc, cands);
            std::vector<int> hc;
            for (int c : gc) {
                Clu &C = clu[c];
                if (C.failed)
                    continue;
                C.realign_As = true;
                (cands[c].empty() ? fin : hc).push_back(c);
            }
            handle_candidates(hc, cands);
            finish_stage(fin);
            std::vector<int> nl;
            for (int c : act) {
                Clu &C = clu[c];
                if (C.failed || C.converged || C.done)
                    continue;
                // update batch randomness (model.jl:1217-1226)
                if ((!P.batch_fixed || (C.stage == ST_REFINE && C.stage_iters[ST_REFINE - 1] > 1)) &&
                    C.batch_size < C.nreads)
                    C.batch_randomness *= P.batch_mult;
                nl.push_back(c);
            }
            live.swap(nl);
        }
    }
};

}  // namespace

// result of the last rf_rifraf_batch per context (retrieved by rf_batch_fetch)
struct BatchResult {
    std::vector<Clu> clu;
    std::vector<Read> reads;
};
// contexts may run on different host threads (one ctx per thread): the
// registry is locked, and each result lives in its own heap block so a
// reference stays valid while other contexts are added or released
static std::mutex g_results_mu;
static std::map<const rf_ctx *, std::unique_ptr<BatchResult>> g_results;

static BatchResult &result_of(const rf_ctx *ctx)
{
    std::lock_guard<std::mutex> lk(g_results_mu);
    auto &slot = g_results[ctx];
    if (!slot)
        slot.reset(new BatchResult{});
    return *slot;
}

extern "C" int rf_rifraf_batch(rf_ctx *ctx, int32_t nclusters, const rf_batch_params *params,
                               const int32_t *read_off, const int32_t *read_seq, const int32_t *read_len,
                               const double *threshold, const int32_t *fixed_off, const int32_t *fixed,
                               const int32_t *slot_base, const int32_t *tpl_id, const uint8_t *cons,
                               const int64_t *cons_off, double *out_score, int32_t *out_iters,
                               int32_t *out_status, int64_t *out_len, int32_t *out_bw)
{
    return rf_rifraf_batch_ref(ctx, nclusters, params, nullptr, read_off, read_seq, read_len, threshold, fixed_off,
                               fixed, slot_base, tpl_id, cons, cons_off, nullptr, nullptr, nullptr, nullptr,
                               out_score, out_iters, out_status, out_len, out_bw);
}

extern "C" int rf_rifraf_batch_ref(rf_ctx *ctx, int32_t nclusters, const rf_batch_params *params,
                                   const rf_batch_ref_params *ref_params, const int32_t *read_off,
                                   const int32_t *read_seq, const int32_t *read_len, const double *threshold,
                                   const int32_t *fixed_off, const int32_t *fixed, const int32_t *slot_base,
                                   const int32_t *tpl_id, const uint8_t *cons, const int64_t *cons_off,
                                   const rf_batch_ref *refs, const uint8_t *ref_bases, rf_ref_callback cb,
                                   void *cb_user, double *out_score, int32_t *out_iters, int32_t *out_status,
                                   int64_t *out_len, int32_t *out_bw)
{
    if (!ctx)
        return RF_ERR_ARG;
    if (nclusters < 0 || !params || (nclusters > 0 && (!read_off || !read_seq || !read_len || !threshold ||
                                                       !slot_base || !tpl_id || !cons || !cons_off)))
        return rf_internal_fail(ctx, RF_ERR_ARG, "rf_rifraf_batch: bad arguments");
    if (params->batch_fixed && (!fixed_off || !fixed))
        return rf_internal_fail(ctx, RF_ERR_ARG, "rf_rifraf_batch: batch_fixed needs fixed_off and fixed");
    if (refs && (!ref_params || !ref_bases || !cb))
        return rf_internal_fail(ctx, RF_ERR_ARG, "rf_rifraf_batch_ref: references need ref_params, ref_bases and cb");
    Driver D{};
    D.ctx = ctx;
    D.P = *params;
    if (ref_params)
        D.RP = *ref_params;
    D.cb = cb;
    D.cb_user = cb_user;
    const int32_t nreads = nclusters > 0 ? read_off[nclusters] : 0;
    D.reads.resize(nreads);
    for (int32_t r = 0; r < nreads; ++r)
        D.reads[r] = {read_seq[r], read_len[r], params->bandwidth, false, threshold[r]};
    if (params->batch_fixed) {
        D.fixed_off.assign(fixed_off, fixed_off + nclusters + 1);
        D.fixed.assign(fixed, fixed + fixed_off[nclusters]);
    }
    D.clu.resize(nclusters);
    for (int32_t c = 0; c < nclusters; ++c) {
        Clu &C = D.clu[c];
        C.r0 = read_off[c];
        C.nreads = read_off[c + 1] - read_off[c];
        C.slot0 = slot_base[c];
        C.tpl = tpl_id[c];
        C.cons.assign(cons + cons_off[c], cons + cons_off[c + 1]);
        // initial_state (model.jl:564-615)
        const int32_t bs = params->batch_size > 1 ? std::min(params->batch_size, C.nreads) : C.nreads;
        C.batch_size = C.base_batch_size = bs;
        C.has_ref = refs && refs[c].ref_seq >= 0;
        if (C.has_ref) {
            const rf_batch_ref &F = refs[c];
            C.ref_bases.assign(ref_bases + F.ref_off, ref_bases + F.ref_off + F.ref_len);
            C.ref_slot = F.ref_slot;
            C.scratch_slot = F.scratch_slot;
            C.edit_seq = F.edit_seq;
            C.ref_read = (int32_t)D.reads.size();   // the reference's read-table entry (bandwidth, threshold)
            D.reads.push_back({F.ref_seq, (int32_t)F.ref_len, params->bandwidth, false, 0.0});
        }
        // outside the native driver's scope (the caller checks first)
        const bool ref_ok = !C.has_ref || (refs[c].ref_len > 0 && refs[c].edit_seq >= 0 && refs[c].ref_slot >= 0 &&
                                           refs[c].scratch_slot >= 0);
        C.batch_randomness = params->batch_randomness;
        if (params->seed)
            C.rng.seed(params->seed[c]);
        // random batches: below the read count without batch_fixed, or in REFINE
        const bool random = bs < C.nreads && (!params->batch_fixed || (C.has_ref && D.RP.do_refine));
        const char *why = C.nreads < 1 ? "no reads"
                          : C.cons.empty() ? "empty consensus"
                          : (random && (!params->est_n_errors || !params->seed))
                              ? "a random batch without est_n_errors and seed"
                          : (params->batch_fixed && fixed_off[c + 1] - fixed_off[c] < 1) ? "an empty fixed batch"
                          : !ref_ok ? "an incomplete reference record"
                          : nullptr;
        if (why)
            return rf_internal_fail(ctx, RF_ERR_ARG,
                                    ("rf_rifraf_batch: cluster " + std::to_string(c) +
                                     " is outside the native driver's scope (" + why + ")").c_str());
    }
    const auto t_run = std::chrono::steady_clock::now();
    int64_t g0;
    double gs0;
    rf_internal_arena_stats(ctx, &g0, &gs0);
    D.run();
    if (const char *tv = std::getenv("RIFRAF_BATCH_TIMING"); tv && *tv && *tv != '0') {
        static const char *names[] = {"realign_fwd", "backtrace", "realign_bwd", "aln_props", "score", "templates"};
        double tot = 0;
        std::fprintf(stderr, "rf_rifraf_batch: %d clusters, run %.4f s;", nclusters,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t_run).count());
        for (int k = 0; k < Driver::T_N; ++k) {
            std::fprintf(stderr, " %s %.4f s / %d (kernels %.4f s);", names[k], D.tsum[k], D.tcnt[k], D.ksum[k]);
            tot += D.tsum[k];
        }
        int64_t g1;
        double gs1;
        rf_internal_arena_stats(ctx, &g1, &gs1);
        std::fprintf(stderr, " engine total %.4f s; arena grows %lld (%.4f s)\n", tot, (long long)(g1 - g0),
                     gs1 - gs0);
    }
    BatchResult &R = result_of(ctx);
    R.clu = std::move(D.clu);
    R.reads = std::move(D.reads);
    for (int32_t c = 0; c < nclusters; ++c) {
        const Clu &C = R.clu[c];
        if (out_score)
            out_score[c] = C.score;
        if (out_iters)
            out_iters[c] = C.iters;
        if (out_status)
            out_status[c] = C.failed ? 2 : (C.converged ? 1 : 0);
        if (out_len)
            out_len[c] = (int64_t)C.cons.size();
    }
    if (out_bw)
        for (int32_t r = 0; r < nreads; ++r)
            out_bw[r] = R.reads[r].bw * (R.reads[r].fixed ? -1 : 1);
    return 0;
}

extern "C" int rf_batch_fetch_ref(rf_ctx *ctx, int32_t cluster, int32_t *stage_iters, int8_t *stage_of,
                                  int32_t *ref_bw, double *ref_score, int32_t *n_ref_indel_mults,
                                  int32_t *batch_len)
{
    if (!ctx)
        return RF_ERR_ARG;
    BatchResult &R = result_of(ctx);
    if (cluster < 0 || cluster >= (int32_t)R.clu.size())
        return RF_ERR_ARG;
    const Clu &C = R.clu[cluster];
    if (stage_iters)
        std::copy(C.stage_iters, C.stage_iters + 3, stage_iters);
    if (stage_of)
        std::copy(C.stage_of.begin(), C.stage_of.end(), stage_of);
    if (ref_bw)
        *ref_bw = C.has_ref ? R.reads[C.ref_read].bw * (R.reads[C.ref_read].fixed ? -1 : 1) : 0;
    if (ref_score)
        *ref_score = C.ref_score;
    if (n_ref_indel_mults)
        *n_ref_indel_mults = C.n_ref_indel_mults;
    if (batch_len)
        *batch_len = (int32_t)C.batch.size();
    return 0;
}

extern "C" int rf_batch_fetch(rf_ctx *ctx, int32_t cluster, uint8_t *cons, int64_t *stage_len, uint8_t *stages,
                              int32_t *batch, char *err, int64_t err_cap)
{
    if (!ctx)
        return RF_ERR_ARG;
    BatchResult &R = result_of(ctx);
    if (cluster < 0 || cluster >= (int32_t)R.clu.size())
        return RF_ERR_ARG;
    const Clu &C = R.clu[cluster];
    if (cons)
        std::memcpy(cons, C.cons.data(), C.cons.size());
    int64_t at = 0;
    for (size_t s = 0; s < C.stages.size(); ++s) {
        if (stage_len)
            stage_len[s] = (int64_t)C.stages[s].size();
        if (stages)
            std::memcpy(stages + at, C.stages[s].data(), C.stages[s].size());
        at += (int64_t)C.stages[s].size();
    }
    if (batch)
        std::copy(C.batch.begin(), C.batch.end(), batch);
    if (err && err_cap > 0) {
        const size_t n = std::min<size_t>(C.err.size(), (size_t)err_cap - 1);
        std::memcpy(err, C.err.data(), n);
        err[n] = 0;
    }
    return 0;
}

extern "C" void rf_batch_release(rf_ctx *ctx)
{
    std::lock_guard<std::mutex> lk(g_results_mu);
    g_results.erase(ctx);
}

// ---------------------------------------------------------------------
// Host helpers of the batched driver's setup and quality pass.  Only FP64
// additions and the C library's pow / log10 (the functions Python's float
// ** and math.log10 call), never a vectorised transcendental, so every
// value equals the Python mirror's.
// ---------------------------------------------------------------------

namespace {
// Julia 0.6 sum(::Vector{Float64}) (base/reduce.jl mapreduce_impl; the mirror
// is rifrafsequences.julia_sum): sequential below 16 elements, otherwise
// pairwise halves down to blocks of at most 1024 summed sequentially.
double julia_sum(const double *a, int64_t lo, int64_t hi)   // inclusive
{
    if (lo + 1024 > hi) {
        double s = a[lo];
        for (int64_t i = lo + 1; i <= hi; ++i)
            s += a[i];
        return s;
    }
    const int64_t mid = (lo + hi) >> 1;
    return julia_sum(a, lo, mid) + julia_sum(a, mid + 1, hi);
}
}  // namespace

extern "C" int rf_host_julia_sums(int64_t nseg, const double *values, const int64_t *off, double *out)
{
    if (nseg < 0 || (nseg > 0 && (!values || !off || !out)))
        return RF_ERR_ARG;
    for (int64_t k = 0; k < nseg; ++k) {
        const int64_t n = off[k + 1] - off[k];
        const double *a = values + off[k];
        if (n == 0) {
            out[k] = 0.0;
        } else if (n < 16) {          // cumsum(a)[-1]: sequential
            double s = a[0];
            for (int64_t i = 1; i < n; ++i)
                s += a[i];
            out[k] = s;
        } else {
            out[k] = julia_sum(a, 0, n - 1);
        }
    }
    return 0;
}

extern "C" int rf_host_seq_sums(int64_t nseg, const double *values, const int64_t *off, double *out)
{
    // np.cumsum(a)[-1] per segment: strictly sequential
    if (nseg < 0 || (nseg > 0 && (!values || !off || !out)))
        return RF_ERR_ARG;
    for (int64_t k = 0; k < nseg; ++k) {
        double s = 0.0;
        bool first = true;
        for (int64_t i = off[k]; i < off[k + 1]; ++i) {
            s = first ? values[i] : s + values[i];
            first = false;
        }
        out[k] = s;
    }
    return 0;
}

// alignment_error_probs (model.jl:817-840) up to its final normalisation:
// for group g, out[(row_g + j) * 4 + b] = the batch-order sum over the group's
// reads of base_distribution(read base, match score)[b] at every match move
// onto consensus column j (0-based); row_g = sum over h < g of m_h.  Moves
// come from rf_backtrace; base_distribution (model.jl:804-809) is evaluated
// with pow / log10 exactly as the Python mirror's scalar code.
extern "C" int rf_aln_error_sums(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                                 const int32_t *tlen, const uint8_t *const *bases, const double *const *match,
                                 const int32_t *seq_len, double *out)
{
    if (!ctx || ngroups < 0 || (ngroups > 0 && (!slot_off || !slots || !tlen || !seq_len || !out)))
        return RF_ERR_ARG;
    // every read row-coded: the moves are folded on the device (k_aln_sums),
    // with the same additions in the same order
    {
        const int e = rf_internal_aln_sums_dev(ctx, ngroups, slot_off, slots, tlen, out);
        if (e <= 0)
            return e;
    }
    if (ngroups > 0 && (!bases || !match))   // the host fold needs the reads' bases and match scores
        return RF_ERR_NEED_HOST;
    const int32_t ns = ngroups > 0 ? slot_off[ngroups] : 0;
    std::vector<int64_t> moff(ns + 1, 0);
    std::vector<int32_t> glen(ns);
    for (int32_t g = 0; g < ngroups; ++g)
        for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k)
            glen[k] = tlen[g];
    for (int32_t k = 0; k < ns; ++k)   // capacity n + m per alignment
        moff[k + 1] = moff[k] + seq_len[k] + glen[k];
    std::vector<int8_t> moves((size_t)std::max<int64_t>(moff[ns], 1));
    std::vector<int32_t> nmoves(std::max(ns, 1));
    if (int e = rf_backtrace(ctx, ns, slots, moves.data(), moff.data(), nmoves.data(), nullptr))
        return e;
    const double log3 = std::log10(3.0);
    // base_distribution rows per distinct match score (math.log10(1.0 - 10.0 ** ilp))
    std::vector<int64_t> rows(ngroups + 1, 0);
    for (int32_t g = 0; g < ngroups; ++g)
        rows[g + 1] = rows[g] + tlen[g];
    // groups are independent: ranges of groups on host threads (each with its
    // own base_distribution cache; the values do not depend on the thread)
    const int nth = std::max(1, std::min(rf_internal_host_threads(), std::max(1, (int)(moff[ns] >> 20))));
    auto work = [&](int t) {
    auto cache = std::vector<std::pair<double, double>>(4096, {std::nan(""), 0.0});
    auto err_lp = [&](double ilp) {
        uint64_t u;
        std::memcpy(&u, &ilp, 8);
        auto &c = cache[(u * 0x9E3779B97F4A7C15ull) >> 52];
        uint64_t cu;
        std::memcpy(&cu, &c.first, 8);
        if (cu == u)
            return c.second;
        const double lp = std::log10(1.0 - std::pow(10.0, ilp)) - log3;
        c = {ilp, lp};
        return lp;
    };
    for (int32_t g = (int32_t)((int64_t)ngroups * t / nth); g < (int32_t)((int64_t)ngroups * (t + 1) / nth); ++g) {
        const int64_t row = rows[g];
        double *P = out + row * 4;
        std::fill(P, P + (size_t)tlen[g] * 4, 0.0);
        for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k) {
            const int8_t *mv = moves.data() + moff[k];
            const uint8_t *b = bases[k];
            const double *ms = match[k];
            int64_t i = 0, j = 0;   // read / consensus positions consumed (align.jl OFFSETS)
            for (int32_t t = 0; t < nmoves[k]; ++t) {
                switch (mv[t]) {
                case 1:   // TRACE_MATCH
                {
                    const double ilp = ms[i];
                    const double o = err_lp(ilp);
                    double *p = P + j * 4;
                    for (int q = 0; q < 4; ++q)
                        p[q] += q == b[i] ? ilp : o;
                    ++i, ++j;
                    break;
                }
                case 2: ++i; break;        // TRACE_INSERT
                case 3: ++j; break;        // TRACE_DELETE
                case 4: i += 3; break;     // TRACE_CODON_INSERT
                case 5: j += 3; break;     // TRACE_CODON_DELETE
                default: break;
                }
            }
        }
    }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nth; ++t)
        th.emplace_back(work, t);
    work(0);
    for (auto &x : th)
        x.join();
    return 0;
}

// RifrafSequence tables (rifrafsequences.jl:19-82) of many sequences whose
// log error probabilities are lp_t[code] for one byte code per position
// (Phred scores): per-code values of lp, 10^lp and match (computed by the
// caller with the Python mirror's numpy expressions) are gathered, and the
// rest is FP64 addition and max exactly as the constructor writes it:
//   mismatch = lp + s_mis, ins = lp + s_ins,
//   del[0] = lp[0] + s_del, del[n] = lp[n-1] + s_del,
//   del[i] = max(lp[i-1], lp[i]) + s_del,
//   est_n_errors = Julia-order sum of 10^lp.
// Outputs are concatenated (del: n + 1 per sequence at off[k] + k).
extern "C" int rf_host_tables_from_codes(int64_t nseg, const uint8_t *codes, const int64_t *off, const double *lp_t,
                                         const double *p10_t, const double *match_t, double s_mis, double s_ins,
                                         double s_del, double *lp, double *match, double *mism, double *ins,
                                         double *del, double *est)
{
    if (nseg < 0 || (nseg > 0 && (!codes || !off || !lp_t || !p10_t || !match_t || !lp || !match || !mism || !ins ||
                                  !del || !est)))
        return RF_ERR_ARG;
    const int64_t N = nseg > 0 ? off[nseg] : 0;
    const int nth = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)rf_internal_host_threads(), (N >> 20) + 1));
    auto work = [&](int t) {
        std::vector<double> p10;
        for (int64_t k = nseg * t / nth; k < nseg * (t + 1) / nth; ++k) {
            const int64_t a = off[k], n = off[k + 1] - off[k];
            double *d = del + a + k;
            p10.resize((size_t)n);
            for (int64_t i = 0; i < n; ++i) {
                const uint8_t c = codes[a + i];
                const double x = lp_t[c];
                lp[a + i] = x;
                match[a + i] = match_t[c];
                mism[a + i] = x + s_mis;
                ins[a + i] = x + s_ins;
                p10[(size_t)i] = p10_t[c];
            }
            if (n > 0) {
                d[0] = lp[a] + s_del;
                d[n] = lp[a + n - 1] + s_del;
                for (int64_t i = 1; i < n; ++i) {   // Base.max of two finite / -Inf values = std::max here
                    const double l = lp[a + i - 1], r = lp[a + i];
                    d[i] = (r > l ? r : l) + s_del;
                }
                est[k] = n < 16 ? [&] {
                    double s = p10[0];
                    for (int64_t i = 1; i < n; ++i)
                        s += p10[(size_t)i];
                    return s;
                }() : julia_sum(p10.data(), 0, n - 1);
            } else {
                est[k] = 0.0;
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nth; ++t)
        th.emplace_back(work, t);
    work(0);
    for (auto &x : th)
        x.join();
    return 0;
}

// logsumexp10 sums of many sequences from the same byte codes: segment k's
// sequential sum of grid[ucode[k] * 256 + codes[i]] (grid = 10^(x - u) per
// (u code, x code), evaluated by the caller with numpy).
extern "C" int rf_host_code_seq_sums(int64_t nseg, const uint8_t *codes, const int64_t *off, const int32_t *ucode,
                                     const double *grid, double *out)
{
    if (nseg < 0 || (nseg > 0 && (!codes || !off || !ucode || !grid || !out)))
        return RF_ERR_ARG;
    for (int64_t k = 0; k < nseg; ++k) {
        const double *g = grid + (size_t)ucode[k] * 256;
        double s = 0.0;
        for (int64_t i = off[k]; i < off[k + 1]; ++i)
            s = i == off[k] ? g[codes[i]] : s + g[codes[i]];
        out[k] = s;
    }
    return 0;
}

namespace {
// ranges [lo, hi) of n items over host threads (OMP_NUM_THREADS, at most 16,
// at least `grain` items per thread)
template <class F>
void host_parallel(int64_t n, int64_t grain, F &&fn)
{
    const int nth = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)rf_internal_host_threads(),
                                                                n / std::max<int64_t>(grain, 1)));
    std::vector<std::thread> th;
    for (int t = 1; t < nth; ++t)
        th.emplace_back([&, t] { fn(n * t / nth, n * (t + 1) / nth); });
    fn(0, n / nth);
    for (auto &x : th)
        x.join();
}
}  // namespace

// Setup of the native driver from Phred codes, without building the host
// tables: per sequence k (codes[off[k]:off[k+1]], non-empty)
//   est[k]   = est_n_errors, the Julia-order sum of p10_t[code]
//              (rifrafsequences.jl:74; the same sum as rf_host_tables_from_codes);
//   ucode[k] = a code whose match_t value is the sequence's maximum match score;
//   lse[k]   = logsumexp10 of the match scores (model.jl:1276-1287's initial
//              consensus choice; the Python mirror model.logsumexp10): the
//              sequential sum of grid[ucode * 256 + code] (grid = 10^(x - u) per
//              code pair, evaluated by the caller with numpy), then
//              log10(sum) + u with the C library's log10 (math.log10).
// A sequence whose maximum is infinite gets lse = u (the caller checks NaN).
extern "C" int rf_host_code_prep(int64_t nseg, const uint8_t *codes, const int64_t *off, const double *p10_t,
                                 const double *match_t, const double *grid, double *est, int32_t *ucode, double *lse)
{
    if (nseg < 0 || (nseg > 0 && (!codes || !off || !p10_t || !match_t || !grid || !est || !ucode || !lse)))
        return RF_ERR_ARG;
    for (int64_t k = 0; k < nseg; ++k)
        if (off[k + 1] <= off[k])
            return RF_ERR_ARG;
    host_parallel(nseg, 64, [&](int64_t lo, int64_t hi) {
        std::vector<double> p10;
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t a = off[k], n = off[k + 1] - off[k];
            const uint8_t *c = codes + a;
            p10.resize((size_t)n);
            int32_t uc = c[0];
            for (int64_t i = 0; i < n; ++i) {
                p10[(size_t)i] = p10_t[c[i]];
                if (match_t[c[i]] > match_t[uc])
                    uc = c[i];
            }
            double s = p10[0];
            if (n < 16) {
                for (int64_t i = 1; i < n; ++i)
                    s += p10[(size_t)i];
            } else {
                s = julia_sum(p10.data(), 0, n - 1);
            }
            est[k] = s;
            ucode[k] = uc;
            const double u = match_t[uc];
            if (std::isinf(u)) {
                lse[k] = u;
                continue;
            }
            const double *g = grid + (size_t)uc * 256;
            double t = g[c[0]];
            for (int64_t i = 1; i < n; ++i)
                t += g[c[i]];
            lse[k] = std::log10(t) + u;
        }
    });
    return 0;
}

extern "C" int rf_host_lse_finish(int64_t nseg, const double *tsum, const int32_t *ucode, const double *match_t,
                                  double *lse)
{
    if (nseg < 0 || (nseg > 0 && (!tsum || !ucode || !match_t || !lse)))
        return RF_ERR_ARG;
    for (int64_t k = 0; k < nseg; ++k) {
        if (ucode[k] < 0 || ucode[k] > 255)
            return RF_ERR_ARG;
        const double u = match_t[ucode[k]];
        lse[k] = std::isinf(u) ? u : std::log10(tsum[k]) + u;   // as rf_host_code_prep
    }
    return 0;
}

// estimate_probs (model.jl:742-800 via the dense totals) and the final
// normalisation of alignment_error_probs (model.jl:835-839) for K clusters at
// once, in two passes around the caller's 10^x (numpy's power, so the values
// equal the Python mirror's model.qvs_many, which this restates):
//
// rf_host_qv_prep: D = stacked dense totals, (m_k + 1) rows of 9 per cluster
// (row 0 = position 0: insertions only); cons = stacked consensus bases;
// score = state scores.  Checks NaN (error 1: "failed to compute a valid
// score"), forms S = sub totals with the consensus base's slot = score,
// Dl = deletion totals, I = insertion totals, mx_k = max(max S, max Dl,
// max I) (Python max order), errors 2/3/4 for a positive sub / del / ins
// maximum relative to mx, and writes the exponents
//   xpos[r] = [S - mx, Dl - mx] (M x 5), xins = I - mx ((M + K) x 4).
// err[0] = error kind, err[1] = its cluster.
extern "C" int rf_host_qv_prep(int64_t K, const int64_t *moff, const double *D, const uint8_t *cons,
                               const double *score, double *xpos, double *xins, double *mx, int32_t *err)
{
    if (K < 0 || (K > 0 && (!moff || !D || !cons || !score || !xpos || !xins || !mx || !err)))
        return RF_ERR_ARG;
    for (int64_t k = 0; k < K; ++k)
        if (moff[k + 1] <= moff[k])
            return RF_ERR_ARG;
    std::vector<uint8_t> bad((size_t)K, 0);
    host_parallel(K, 8, [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t r0 = moff[k] + k, m = moff[k + 1] - moff[k];   // dense rows r0 .. r0 + m
            bool nan = false;
            double mS = -INF, mD = -INF, mI = -INF;
            bool firstS = true, firstD = true, firstI = true;
            for (int64_t p = 0; p <= m; ++p) {
                const double *d = D + (r0 + p) * 9;
                for (int q = 5; q < 9; ++q) {
                    nan |= std::isnan(d[q]);
                    mI = firstI ? d[q] : (d[q] > mI ? d[q] : mI);
                    firstI = false;
                }
                if (p == 0)
                    continue;
                const int64_t r = moff[k] + p - 1;
                const int cb = cons[r];
                for (int q = 0; q < 5; ++q)
                    nan |= q != cb && std::isnan(d[q]);
                for (int q = 0; q < 4; ++q) {
                    const double v = q == cb ? 0.0 + score[k] : d[q];
                    mS = firstS ? v : (v > mS ? v : mS);
                    firstS = false;
                }
                mD = firstD ? d[4] : (d[4] > mD ? d[4] : mD);
                firstD = false;
            }
            double x = mS;                       // Python max(mxS, mxD, mxI)
            if (mD > x)
                x = mD;
            if (mI > x)
                x = mI;
            mx[k] = x;
            bad[(size_t)k] = nan ? 1 : mS - x > 0.0 ? 2 : mD - x > 0.0 ? 3 : mI - x > 0.0 ? 4 : 0;
            if (nan)
                continue;
            for (int64_t p = 0; p <= m; ++p) {
                const double *d = D + (r0 + p) * 9;
                double *xi = xins + (r0 + p) * 4;
                for (int q = 0; q < 4; ++q)
                    xi[q] = d[5 + q] - x;
                if (p == 0)
                    continue;
                const int64_t r = moff[k] + p - 1;
                const int cb = cons[r];
                double *xp = xpos + r * 5;
                for (int q = 0; q < 4; ++q)
                    xp[q] = (q == cb ? 0.0 + score[k] : d[q]) - x;
                xp[4] = d[4] - x;
            }
        }
    });
    err[0] = 0;
    err[1] = -1;
    for (int64_t k = 0; k < K; ++k)       // any NaN first (the mirror checks the whole stack), then the first cluster
        if (bad[(size_t)k] == 1) {
            err[0] = 1;
            err[1] = (int32_t)k;
            return 0;
        }
    for (int64_t k = 0; k < K; ++k)
        if (bad[(size_t)k]) {
            err[0] = bad[(size_t)k];
            err[1] = (int32_t)k;
            return 0;
        }
    return 0;
}

// rf_host_qv_finish: epos / eins / ealn = 10^x of the prep's exponents (and of
// the alignment_error_probs sums, M x 4); in place:
//   epos[r] /= epos[r][0] + ... + epos[r][4]                 (pos_probs)
//   eins[r] /= st_pow[k] + (eins[r][0] + ... + eins[r][3])   (ins_probs)
//   aln[r]   = 1.0 - max_b ealn[r][b] / (ealn[r][0] + ... + ealn[r][3])
// with st_pow[k] = 10.0 ** (score_k - mx_k) from the caller; row sums are
// sequential, as numpy's sum(axis=1) over rows of 4 / 5.
extern "C" int rf_host_qv_finish(int64_t K, const int64_t *moff, const double *st_pow, double *epos, double *eins,
                                 const double *ealn, double *aln)
{
    if (K < 0 || (K > 0 && (!moff || !st_pow || !epos || !eins || !ealn || !aln)))
        return RF_ERR_ARG;
    host_parallel(K, 8, [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t m = moff[k + 1] - moff[k];
            for (int64_t p = 0; p <= m; ++p) {
                double *e = eins + (moff[k] + k + p) * 4;
                const double s = st_pow[k] + (((e[0] + e[1]) + e[2]) + e[3]);
                for (int q = 0; q < 4; ++q)
                    e[q] = e[q] / s;
            }
            for (int64_t r = moff[k]; r < moff[k + 1]; ++r) {
                double *e = epos + r * 5;
                const double s = (((e[0] + e[1]) + e[2]) + e[3]) + e[4];
                for (int q = 0; q < 5; ++q)
                    e[q] = e[q] / s;
                const double *a = ealn + r * 4;
                const double t = ((a[0] + a[1]) + a[2]) + a[3];
                double mxq = a[0] / t;
                for (int q = 1; q < 4; ++q) {   // numpy max: NaN propagates
                    const double v = a[q] / t;
                    mxq = (std::isnan(mxq) || !(v <= mxq)) ? (std::isnan(mxq) ? mxq : v) : mxq;
                }
                aln[r] = 1.0 - mxq;
            }
        }
    });
    return 0;
}
