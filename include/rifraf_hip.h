/*
 * rifraf_hip.h -- C-ABI of the MI355X-native RIFRAF hot-path engine
 * (librifraf_hip.so, built from rifraf.jl_amd/csrc/).
 *
 * The reference (Rifraf.jl) has no FFI layer: the hot path is a set of
 * internal Julia functions.  Each entry point below replaces one of them and
 * is what a Julia `ccall` or Python `ctypes` binds:
 *
 *   rf_set_sequences  <- RifrafSequence tables      src/rifrafsequences.jl:19-82
 *   rf_set_templates  <- state.consensus            src/model.jl:169
 *   rf_realign        <- forward_moves!/forward!/backward! over a batch
 *                        src/align.jl:114-141,155-179,196-202;
 *                        realign! src/model.jl:679-714
 *   rf_backtrace      <- backtrace + count_errors   src/align.jl:229-245
 *   rf_alignment_proposals <- alignment_proposals / moves_to_proposals
 *                        src/model.jl:458-497
 *   rf_score          <- score_proposal(m, state, newcols, use_ref) summed
 *                        over the batch, as called by get_candidates and
 *                        estimate_probs  src/model.jl:385-399,499-526,737-791
 *                        (per-sequence: score_nocodon :242-285 / codon
 *                        score_proposal :302-383 / seq_score_deletion :227-236)
 *   rf_download_band  <- BandedArray data (tests)   src/bandedarrays.jl:5-42
 *
 * Conventions
 *  - Every call returns 0 on success and a negative code on failure; the
 *    message is rf_last_error(ctx), using the reference's error text
 *    ("new score is invalid", "failed to compute a valid score", ...).
 *  - Bases are 2-bit codes A=0, C=1, G=2, T=3 (BioSequences DNAAlphabet{2}).
 *  - Sequence tables are FP64 and uploaded bit-exact from the host (the
 *    host computes them exactly as RifrafSequence() does).
 *  - Proposal positions use the reference's 1-based Proposal.pos
 *    (Insertion(0, b) inserts before the first base). kind: 0 = Substitution,
 *    1 = Insertion, 2 = Deletion.
 *  - Bands stay device resident between calls.  A "slot" is one alignment
 *    (sequence x template) owning an A band and a B band: the H x (m+1) FP64
 *    cells of the reference's data[(i-j)+h_off+bw+1, j]
 *    (src/bandedarrays.jl:101-114), H = 2*bw + |n-m| + 1.  On the device a
 *    band is stored anti-diagonal ("kappa") major: cell (d, j) (0-based data
 *    row d, column j) at kappa = d + 2j, element d >> 1 of a kappa row of
 *    P = ((H+1) >> 1) | 1 doubles; the B band is stored
 *    already flipped.  rf_download_band converts to the reference's
 *    column-major data.
 *  - One context per host thread; calls are synchronous on the context's
 *    HIP stream.  No torch types cross this boundary.
 */
#ifndef RIFRAF_HIP_H
#define RIFRAF_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RF_ABI_VERSION 1

/* rf_realign flags */
#define RF_FWD  1   /* A band: forward_moves!/forward!             align.jl:114,155 */
#define RF_BWD  2   /* B band: backward! (reverse forward + flip!) align.jl:196    */
#define RF_SKEW 4   /* skew_matches: mismatch score *= 0.99        align.jl:70-72  */
#define RF_TRIM 8   /* trim: free insertions in first/last column  align.jl:74-76  */

/* rf_download_band `which` */
#define RF_BAND_A 0
#define RF_BAND_B 1

/* error codes */
#define RF_ERR_ARG        (-1)
#define RF_ERR_HIP        (-2)
#define RF_ERR_NUMERIC    (-3)   /* a reference error() on the numeric path */
#define RF_ERR_STATE      (-4)   /* stale / mismatched bands */
#define RF_ERR_NEED_HOST  (-5)   /* rf_aln_error_sums: host bases / match scores needed (passed NULL) */

typedef struct rf_ctx rf_ctx;

int rf_abi_version(void);

/* Create a context on HIP device `device`. */
int rf_create(int device, rf_ctx **out);
int rf_destroy(rf_ctx *ctx);
const char *rf_last_error(const rf_ctx *ctx);

/* Tuning options of a context (rf_set_option / rf_get_option keys).  Every
 * value selects between code paths with bit-identical results; the defaults
 * are read once from the RIFRAF_* environment at rf_create.  No reference
 * counterpart (the reference has one code path). */
#define RF_OPT_SCORE_MODE   1   /* 0 auto, 1 fused in-kernel fold, 2 split + k_reduce  */
#define RF_OPT_SCORE_KERNEL 2   /* 0 auto, 1 general k_score, 2 k_score_segl, 3 k_score_ws whenever it fits */
#define RF_OPT_LEAN_LDS_KB  4   /* k_score_ws LDS budget in KB (0 = default 160)       */
/* key 9 (RF_OPT_BT_GLOBAL: every walk in the one-lane k_backtrace) removed in round 5 */
#define RF_OPT_DP_PSPLIT   10   /* lean DP stride-class split mask (-1 auto)           */
#define RF_OPT_DP_NP8      11   /* 0: H 128..255 bands in k_dp<64> instead of k_dpr<8> */
#define RF_OPT_DP_NP8_LEAN 12   /* 0: k_dpr<8> general steps only                      */
#define RF_OPT_DP_STREAMS  13   /* 0: DP classes serialised on the context stream      */
#define RF_OPT_BT_WIN_KB   15   /* k_bt_win A-window LDS: 16 (default) or 32 KB        */
#define RF_OPT_STAGE_KB    16   /* rf_set_sequences host staging chunk, KB of tables   */
#define RF_OPT_BAND_PAD    17   /* an rf_realign call whose widest band has H >= value
                                    lays out all its bands with kappa rows of whole
                                    128-B lines (default 64; 1 always, 0 never)       */
#define RF_OPT_DP_WIDE     18   /* lean DP task widths: bit 0 H 128..255 as 64-lane
                                    tasks (k_dpr<2,..,64>), bit 1 H 64..127 as 32-lane
                                    tasks (k_dpr<2,..,32>); 0 = 16-lane tasks only   */
#define RF_OPT_ALN_SUMS_HOST 19 /* 1: rf_aln_error_sums folds the moves on host
                                    threads instead of the device (k_aln_sums)     */
#define RF_OPT_ALN_MARKS_MIN 22 /* rf_aln_error_sums on the device: groups of more
                                   than this many reads (default 128) use the
                                   per-read marks + per-column fold launches      */
#define RF_OPT_SYNC_BLOCK  23   /* 1: host waits for the engine's stream yield
                                   the core, then sleep between event polls,
                                   instead of spinning (ranks held to a few
                                   host cores); 2: auto,
                                   sleep when the waiting thread may run on
                                   fewer than 4 CPUs (its affinity mask; the
                                   default)                                     */
#define RF_OPT_DP_NL64     24   /* at most this many non-lean DP tasks of H <= 127
                                   per call (codon / skew / trim) run as one
                                   latency-bound task per wave, k_dpx (default
                                   1024; 0: the 16-lane non-lean kernels)       */
#define RF_OPT_DP_LAT      26   /* latency mode: an rf_realign call with at most
                                   this many lean tasks of H <= 127 runs them all
                                   as one latency-bound task per wave (k_dpx, one
                                   launch; such a call cannot fill the GPU, so a
                                   task's step latency is the time).  Default
                                   2048; 0 never.  align.jl:114-212            */
#define RF_OPT_SCORE_WGS   27   /* split-mode k_score_ws: reads per workgroup chosen
                                   so that about this many workgroups remain
                                   (default 2048; small values: many reads per
                                   workgroup, partials written per read)        */
#define RF_OPT_SEG_WGS     28   /* split-mode k_score_segl: reads per workgroup
                                   chosen so that about this many workgroups
                                   remain (default 262144)                      */
#define RF_OPT_DP_PFIT     29   /* 1 (default): a lean NP >= 2 DP class in one
                                   launch takes the smallest stride class that
                                   holds its widest task (fewer repeated flush
                                   stores); 0: the class maximum                */
#define RF_OPT_DP_MC       30   /* 1 (default): bands of H > 2040 without codon
                                   moves (edit_distance's) filled across CUs in
                                   slices that hand off every 32 anti-diagonals
                                   (k_dpm); 0: one workgroup per band (k_dp)    */
#define RF_OPT_BT_NW       31   /* 4 (default): a backtrace launch of at most 64
                                   walks runs each on 4 waves (k_bt_win<4096, 4>,
                                   a 252-cell box); 1: one wave per walk        */
/* Keys 3, 5-8, 14 and 20 selected scorer variants measured slower and removed
   in round 3 (k_score_lean, the 128-lane k_score_ws, k_score_seg /
   k_score_segc, 16-diagonal k_score_segl, the unspecialised k_score_w2);
   keys 9 (the one-lane k_backtrace walk), 21 (128-column k_score_segw) and 25
   (k_fuse, the fused forward fill + scoring step) in round 5.  rf_set_option rejects them. */
int rf_set_option(rf_ctx *ctx, int32_t key, int32_t value);
int rf_get_option(rf_ctx *ctx, int32_t key, int32_t *value);

/* Pre-size the device band arena (bytes); optional. */
int rf_reserve(rf_ctx *ctx, int64_t band_bytes);
/* Drop every slot's A and B band (each must be filled again before it is
 * read) and reuse the band arena from its start; the device memory is kept.
 * For a caller that starts a new batch of alignments (the batched driver's
 * waves), so an arena sized once serves every later batch. */
int rf_release_bands(rf_ctx *ctx);
/* Bytes currently allocated on the device by this context. */
int64_t rf_device_bytes(const rf_ctx *ctx);
/* Row-code dictionary of the context (the lean DP's 8-B per-row records):
   distinct (match, mismatch, ins) triples and del values held, reads left
   uncoded because the 65,536-entry dictionary was full (their DP reads the
   tables: slower, same values), and fresh starts (an upload that replaces
   every coded sequence resets it).  Engine-internal; no reference analog. */
int rf_code_stats(const rf_ctx *ctx, int64_t *entries3, int64_t *entries1, int64_t *uncoded_reads,
                  int64_t *resets);

/* Sequences (reads or a reference): ids [first, first+nseq).  Replaces any
 * previous content of those ids.  Per sequence k (n_k = off[k+1]-off[k]):
 *   bases    off[k]..off[k+1]                    (n_k codes)
 *   match, mismatch, ins at off[k]..off[k+1]     (rifrafsequences.jl:45-47)
 *   del      at off[k]+k .. off[k+1]+k+1         (n_k+1, :49-53)
 *   cins     cins_off[k]..cins_off[k+1]           (n_k-2 or 0, :57-64)
 *   cdel     cdel_off[k]..cdel_off[k+1]           (n_k+1 or 0, :65-72)
 * cins/cdel/cins_off/cdel_off may be NULL (no codon moves). */
int rf_set_sequences(rf_ctx *ctx, int32_t first, int32_t nseq,
                     const uint8_t *bases, const int64_t *off,
                     const double *match, const double *mismatch,
                     const double *ins, const double *del,
                     const double *cins, const int64_t *cins_off,
                     const double *cdel, const int64_t *cdel_off);
/* The same upload for Phred-coded reads without codon moves, with the
   tables built on the device from one byte per position: codes[off[k]..]
   index lp_t[256] (log10 error probability) and match_t[256]
   (log10(1 - 10^lp), both evaluated by the caller's libm, as the
   RifrafSequence constructor does, rifrafsequences.jl:19-53); mismatch /
   ins / del follow with the scores' mismatch / insertion / deletion by FP64
   addition and maximum -- bit-identical to rf_set_sequences of the host
   tables.  Moves 2 B per position over PCIe instead of ~41.  Returns
   RF_ERR_STATE when the row-code dictionary is full (upload host tables). */
int rf_set_sequences_codes(rf_ctx *ctx, int32_t first, int32_t nseq, const uint8_t *bases, const int64_t *off,
                           const uint8_t *codes, const double *lp_t, const double *match_t, double s_mis,
                           double s_ins, double s_del);
/* rf_set_sequences_codes plus the native driver's per-read setup values,
 * computed on the device from the same staged codes (k_code_prep, round 5;
 * bit-identical to rf_host_code_prep, which it replaces on the driver's
 * path): est[k] = est_n_errors (Julia-order sum of p10_t[code],
 * rifrafsequences.jl:74), ucode[k] = the code of the first maximal match
 * score, tsum[k] = the sequential sum of grid[ucode * 256 + code] --
 * logsumexp10 of the match scores is log10(tsum) + match_t[ucode]
 * (rf_host_lse_finish; util.jl:28-38, model.jl:575-579).  p10_t: 256 values
 * 10^lp; grid: 256 x 256, grid[u * 256 + x] = 10^(match_t[x] - match_t[u]). */
int rf_set_sequences_codes_prep(rf_ctx *ctx, int32_t first, int32_t nseq, const uint8_t *bases, const int64_t *off,
                                const uint8_t *codes, const double *lp_t, const double *match_t, double s_mis,
                                double s_ins, double s_del, const double *p10_t, const double *grid, double *est,
                                int32_t *ucode, double *tsum);

/* Templates (consensus sequences, one per cluster): ids [first, first+n). */
int rf_set_templates(rf_ctx *ctx, int32_t first, int32_t ntpl,
                     const uint8_t *bases, const int64_t *off);

/* Templates with arbitrary ids: ids[k] receives bases off[k]..off[k+1]
 * (rf_set_templates for a sparse set, e.g. the clusters of a batched run
 * whose consensus changed this iteration). */
int rf_set_templates_ids(rf_ctx *ctx, int32_t ntpl, const int32_t *ids,
                         const uint8_t *bases, const int64_t *off);

/* Batched DP fill.  Job k aligns sequence seq[k] (rows) against template
 * tpl[k] (columns) with bandwidth bw[k] into slot slot[k].  flags: RF_FWD
 * and/or RF_BWD, optionally RF_SKEW / RF_TRIM (forward only).
 * out_score[k] (may be NULL) = A[end,end] if RF_FWD else B[1,1]. */
int rf_realign(rf_ctx *ctx, int32_t njobs, const int32_t *slot,
               const int32_t *seq, const int32_t *tpl, const int32_t *bw,
               int32_t flags, double *out_score);
/* rf_realign with flags per job (round 5): independent fills of one stage
 * machine step -- e.g. the reads' backward! and the reference's skewed
 * forward_moves! of single_indel_proposals (model.jl:538-562) -- share one
 * launch set, so a latency-bound task runs beside the others. */
int rf_realign_jobs(rf_ctx *ctx, int32_t njobs, const int32_t *slot,
                    const int32_t *seq, const int32_t *tpl, const int32_t *bw,
                    const int32_t *flags, double *out_score);

/* Backtrace of the A band of each slot (align.jl:229-238), moves in
 * alignment order written at moves[moves_off[k] ...] (capacity n+m each);
 * nmoves[k] = count; nerrors[k] = count_errors (align.jl:240-245).
 * Any of moves/moves_off/nmoves/nerrors may be NULL. */
int rf_backtrace(rf_ctx *ctx, int32_t nslots, const int32_t *slot,
                 int8_t *moves, const int64_t *moves_off,
                 int32_t *nmoves, int32_t *nerrors);

/* alignment_proposals (model.jl:483-497 over moves_to_proposals :458-480)
 * on the device: backtrace every batch slot of each group (one cluster) and
 * mark the proposals its alignment implies -- Substitution at mismatching
 * matches, and if do_indels, Insertion / Deletion -- in the group's dense
 * mask out_mask[(row_g + p) * 9 + k] (0/1 bytes, slots as rf_score_dense,
 * row_g = sum over h < g of (m_h + 1)).  The mask is the reference's Set
 * union over the batch; position-major order is (pos, kind, base) order. */
int rf_alignment_proposals(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off,
                           const int32_t *slots, int32_t do_indels, uint8_t *out_mask);

/* Proposal scoring.  Group g (one cluster) = batch slots
 * slots[slot_off[g] .. slot_off[g+1]) in batch order, an optional
 * reference slot ref_slot[g] (-1: none; scored with codon moves when its
 * sequence has codon tables), and proposals prop_off[g] .. prop_off[g+1].
 * out_total[k] = 0.0 + s_1 + ... + s_R (+ s_ref), the left fold of
 * model.jl:389-397.  out_per_seq (may be NULL) receives s_r for every
 * (proposal, batch slot) pair, row-major [k][r] with r in batch order,
 * followed by s_ref in an extra last column when the group has a
 * reference (row width R_g or R_g + 1). */
int rf_score(rf_ctx *ctx, int32_t ngroups,
             const int32_t *slot_off, const int32_t *slots,
             const int32_t *ref_slot, const int64_t *prop_off,
             const uint8_t *kind, const int32_t *pos, const uint8_t *base,
             double *out_total, double *out_per_seq);

/* Dense scoring of every proposal anchored at every consensus position --
 * the STAGE_SCORE all_proposals set (model.jl:401-456) that estimate_probs
 * scores (model.jl:737-791) -- for batch reads only (no reference):
 * out[(row_g + p) * 9 + k] = 0.0 + s_1 + ... + s_R for p = 0..m_g, with
 * k = 0..3 Substitution(p, A/C/G/T) (the consensus base's own slot is not a
 * proposal), k = 4 Deletion(p), k = 5..8 Insertion(p, A/C/G/T);
 * row_g = sum over h < g of (m_h + 1).  Sub/Del slots of p = 0 are NaN.
 * A failed update or a -Inf sum is reported as NaN in that slot (the
 * reference raises on such a proposal when it scores it).
 * out may be NULL: totals then stay on the device. */
int rf_score_dense(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off,
                   const int32_t *slots, double *out);

/* rf_score_dense with the totals written to DEVICE memory of the context's
 * device (dev_out: at least sum_g (m_g + 1) * 9 doubles, e.g. a torch tensor).
 * For the read-sharded exchange: each rank's partial fold
 * goes straight into the RCCL all-gather buffer without a host round trip. */
int rf_score_dense_dev(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off,
                       const int32_t *slots, double *dev_out);

/* Native batched rifraf() (src/model.jl:1116-1275) for reference-free
 * clusters: the INIT stage of every cluster runs in lockstep on this context
 * with one batched engine call per step kind (rifraf_batch.cpp); each
 * cluster ends exactly as a separate rifraf() call would (consensus, score,
 * iteration count).  The caller (rifraf_amd.batch) uploads the reads and
 * initial consensus first and supplies the host values that need the Python
 * mirror's transcendental functions.
 *   read_off[c]..read_off[c+1]: cluster c's reads; read_seq / read_len per
 *     read: its sequence id and length; threshold per read:
 *     cquantile(Poisson(est_n_errors), bandwidth_pvalue) (model.jl:661)
 *   fixed_off / fixed: the fixed batch per cluster (local read indices in
 *     batch order, sortperm of est_n_errors; required if batch_fixed)
 *   random batches (resample!, model.jl:1038-1066: batch_size below the read
 *     count without batch_fixed, or in REFINE) are drawn here from
 *     params->est_n_errors (per read) and params->seed (per cluster), with
 *     rifraf_amd/resampling.py's RNG and draw; both NULL: such a cluster is
 *     rejected (RF_ERR_ARG)
 *   slot_base[c]: first of the cluster's batch slots; tpl_id[c]: its template
 *   cons / cons_off: the initial consensus per cluster (already uploaded)
 * Outputs per cluster: final score, INIT iterations, status (0 = reached
 * max_iters, 1 = converged, 2 = failed: rf_batch_fetch has the message),
 * consensus length; out_bw per read = final bandwidth, negated once
 * bandwidth_fixed.  Results stay in the context until rf_batch_release. */
typedef struct rf_batch_params {
    int32_t max_iters;
    int32_t min_dist;
    int32_t bandwidth;               /* initial bandwidth of every read */
    int32_t do_alignment_proposals;
    int32_t batch_fixed;
    int32_t batch_size;              /* params.batch_size (<= 1: every read) */
    double batch_threshold;
    double batch_randomness;         /* initial state.batch_randomness (model.jl:592) */
    double batch_mult;               /* its decay per iteration (model.jl:1234-1238) */
    const double *est_n_errors;      /* per read, or NULL: resample!'s weights */
    const uint64_t *seed;            /* per cluster, or NULL: the random batches' RNG */
} rf_batch_params;
int rf_rifraf_batch(rf_ctx *ctx, int32_t nclusters, const rf_batch_params *params,
                    const int32_t *read_off, const int32_t *read_seq, const int32_t *read_len,
                    const double *threshold, const int32_t *fixed_off, const int32_t *fixed,
                    const int32_t *slot_base, const int32_t *tpl_id, const uint8_t *cons,
                    const int64_t *cons_off, double *out_score, int32_t *out_iters,
                    int32_t *out_status, int64_t *out_len, int32_t *out_bw);
/* Reference-guided clusters (FRAME and REFINE, model.jl:937-995, 499-562):
 * rf_rifraf_batch with, per cluster, a reference record (ref_seq < 0: none).
 * The stage machine then runs INIT -> FRAME -> REFINE like rifraf():
 * edit_distance at FRAME entry (align.jl:253-260, on edit_seq: the
 * reference's copy with log p = -1 and ErrorModel(1, 1, 1) scores, uploaded
 * by the caller), has_single_indels / single_indel_proposals (the reference
 * aligned to the consensus in scratch_slot), seeded all_proposals, scoring
 * with the reference's codon moves (ref_slot) and the reference term of
 * rescore!.  The two host steps that need the caller's transcendental
 * functions go through `cb`:
 *   event 0 (FRAME entry), value = ref_error_rate: build the reference with
 *     log p = log10(value) and the current reference scores, upload it at
 *     ref_seq, write *thr = cquantile(Poisson(est_n_errors), bandwidth_pvalue);
 *   event 1 (penalty increase), value = n_ref_indel_mults: rescale the
 *     reference's indel scores by ref_indel_mult^n (model.jl:978-985) and
 *     upload it again.
 * cb returns 0, or nonzero to fail the cluster.  Scope as rf_rifraf_batch. */
typedef struct rf_batch_ref_params {
    int32_t do_frame, do_refine, seed_indels, indel_correction_only;
    int32_t max_ref_indel_mults, pad;
    double ref_error_mult;
} rf_batch_ref_params;
typedef struct rf_batch_ref {
    int32_t ref_seq, edit_seq, ref_slot, scratch_slot;
    int64_t ref_off, ref_len;   /* the reference's bases in ref_bases */
} rf_batch_ref;
typedef int (*rf_ref_callback)(void *user, int32_t cluster, int32_t event, double value, double *thr);
int rf_rifraf_batch_ref(rf_ctx *ctx, int32_t nclusters, const rf_batch_params *params,
                        const rf_batch_ref_params *ref_params, const int32_t *read_off,
                        const int32_t *read_seq, const int32_t *read_len, const double *threshold,
                        const int32_t *fixed_off, const int32_t *fixed, const int32_t *slot_base,
                        const int32_t *tpl_id, const uint8_t *cons, const int64_t *cons_off,
                        const rf_batch_ref *refs, const uint8_t *ref_bases, rf_ref_callback cb,
                        void *cb_user, double *out_score, int32_t *out_iters, int32_t *out_status,
                        int64_t *out_len, int32_t *out_bw);
/* Stage record of cluster c of the last batch: iterations per stage (INIT,
 * FRAME, REFINE), the stage of each recorded consensus (1/2/3, as many as
 * rf_batch_fetch's stages), the reference's final bandwidth (negated once
 * fixed; 0 without one), A_ref[end,end], n_ref_indel_mults and the length
 * of the final batch (what rf_batch_fetch's `batch` receives: REFINE's
 * batch holds every read even when INIT / FRAME used the fixed batch). */
int rf_batch_fetch_ref(rf_ctx *ctx, int32_t cluster, int32_t *stage_iters, int8_t *stage_of,
                       int32_t *ref_bw, double *ref_score, int32_t *n_ref_indel_mults, int32_t *batch_len);
/* Cluster c of the last rf_rifraf_batch: consensus (out_len[c] bytes), the
 * consensus at each INIT iteration (stage_len[i] bytes each, concatenated
 * in `stages`), the final batch (local read indices; room for every read of
 * the cluster, or rf_batch_fetch_ref's batch_len) and the error message of a
 * failed cluster.  Any output may be NULL. */
int rf_batch_fetch(rf_ctx *ctx, int32_t cluster, uint8_t *cons, int64_t *stage_len, uint8_t *stages,
                   int32_t *batch, char *err, int64_t err_cap);
/* Free the context's stored batch results. */
void rf_batch_release(rf_ctx *ctx);
/* alignment_error_probs (model.jl:817-840) before its final normalisation,
 * for many groups at once: backtraces every slot of group g (slots
 * slot_off[g]..slot_off[g+1], batch order) and sums base_distribution(read
 * base, match score) (model.jl:804-809) at each match move, per consensus
 * column, in batch order: out[(row_g + j) * 4 + b], row_g = sum over h < g
 * of tlen[h].  bases[k] / match[k] point at slot k's read bases and match
 * scores (seq_len[k] each, host memory).  When every read is row-coded the
 * sums are folded on the device and bases / match may be NULL; if they are
 * NULL and the host fold is needed, RF_ERR_NEED_HOST. */
int rf_aln_error_sums(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                      const int32_t *tlen, const uint8_t *const *bases, const double *const *match,
                      const int32_t *seq_len, double *out);
/* The quality pass of many groups on the device (model.jl:737-771 estimate_probs
 * over the dense totals, normalize_log_differences :722-735, and
 * alignment_error_probs :817-840): out_pos[(row_g + p) * 5 + s] (p < m_g; s =
 * Sub A..T, Del at position p + 1), out_ins[(row_g + g + p) * 4 + b] (p <= m_g),
 * out_aln[row_g + p]; score[g] = state.score; err_out = {kind, group} (kind 1:
 * "failed to compute a valid score", 2 / 3 / 4: sub / deletion / insertion
 * scores cannot be positive).  10^x is the device's FP64 exp10 (~1e-15
 * relative of the host's).  Returns 1 (nothing done) when a read has no row
 * codes. */
int rf_qv_probs(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                const int32_t *tlen, const double *score, double *out_pos, double *out_ins, double *out_aln,
                int32_t *err_out);
/* Host sums of segments values[off[k]..off[k+1]): Julia 0.6 sum() order
 * (pairwise, blocks of 1024; rifrafsequences.jl:74 est_n_errors) and the
 * plain sequential order (cumsum(...)[end], util.jl:28-38 logsumexp10). */
int rf_host_julia_sums(int64_t nseg, const double *values, const int64_t *off, double *out);
int rf_host_seq_sums(int64_t nseg, const double *values, const int64_t *off, double *out);
/* RifrafSequence tables of many sequences from one byte code per position
 * (Phred scores): lp_t / p10_t / match_t per code, s_* the Scores terms;
 * concatenated outputs (del: n+1 per sequence at off[k]+k), est_n_errors. */
int rf_host_tables_from_codes(int64_t nseg, const uint8_t *codes, const int64_t *off, const double *lp_t,
                              const double *p10_t, const double *match_t, double s_mis, double s_ins,
                              double s_del, double *lp, double *match, double *mism, double *ins,
                              double *del, double *est);
/* Per segment, the sequential sum of grid[ucode[k] * 256 + codes[i]]. */
int rf_host_code_seq_sums(int64_t nseg, const uint8_t *codes, const int64_t *off, const int32_t *ucode,
                          const double *grid, double *out);
/* Native-driver setup from Phred codes without host tables: per sequence
 * est_n_errors (Julia-order sum of p10_t[code], rifrafsequences.jl:74), a
 * code of its maximum match score, and logsumexp10 of its match scores
 * (util.jl:28-38 with grid[u * 256 + x] = 10^(match_t[x] - match_t[u])). */
int rf_host_code_prep(int64_t nseg, const uint8_t *codes, const int64_t *off, const double *p10_t,
                      const double *match_t, const double *grid, double *est, int32_t *ucode, double *lse);
/* logsumexp10 from rf_set_sequences_codes_prep's outputs: lse[k] =
 * log10(tsum[k]) + match_t[ucode[k]] (libm log10), or match_t[ucode[k]] when
 * that is infinite -- the values rf_host_code_prep writes. */
int rf_host_lse_finish(int64_t nseg, const double *tsum, const int32_t *ucode, const double *match_t, double *lse);
/* estimate_probs (model.jl:742-800) and alignment_error_probs's
 * normalisation (model.jl:835-839) for K clusters, around the caller's 10^x:
 * prep checks the stacked dense totals D ((m_k+1) x 9 per cluster) and
 * writes the exponents xpos (M x 5: subs with the consensus slot = score,
 * deletion; minus the cluster maximum mx_k) and xins ((M+K) x 4); err[0] =
 * 1 NaN / 2 sub / 3 del / 4 ins positive, err[1] = cluster.  finish
 * normalises 10^xpos, 10^xins (with st_pow_k = 10^(score_k - mx_k)) and
 * 10^sums (M x 4, -> aln[M]) in place. */
int rf_host_qv_prep(int64_t K, const int64_t *moff, const double *D, const uint8_t *cons, const double *score,
                    double *xpos, double *xins, double *mx, int32_t *err);
int rf_host_qv_finish(int64_t K, const int64_t *moff, const double *st_pow, double *epos, double *eins,
                      const double *ealn, double *aln);

/* Geometry of a slot's band: nrows = n+1, ncols = m+1, bandwidth, H. */
int rf_slot_geometry(rf_ctx *ctx, int32_t slot, int32_t which,
                     int32_t *nrows, int32_t *ncols, int32_t *bw, int32_t *H);

/* Copy a slot's band (H x ncols doubles, column-major) to the host. */
int rf_download_band(rf_ctx *ctx, int32_t slot, int32_t which, double *out);

/* Kernel timing of the last rf_realign / rf_score call (HIP events on the
 * context stream), milliseconds; used by bench.py's roofline. */
int rf_last_timing(const rf_ctx *ctx, double *dp_ms, double *score_ms,
                   double *gather_ms);
/* Kernel time of the walks of the last rf_backtrace / rf_alignment_proposals
 * call (k_bt_win), milliseconds. */
int rf_last_backtrace_ms(const rf_ctx *ctx, double *ms);
/* Kernel time of the reference's codon score_proposal (k_codon,
 * model.jl:287-383) in the last rf_score call, milliseconds (0 when the call
 * scored no reference); it is part of that call's score_ms. */
int rf_last_codon_ms(const rf_ctx *ctx, double *ms);

#ifdef __cplusplus
}
#endif
#endif
