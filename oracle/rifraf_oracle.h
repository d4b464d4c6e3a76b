/*
 * rifraf_oracle.h -- CPU restatement of the Rifraf.jl hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X engine (rifraf.jl_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never links it.
 *
 * Every function restates a reference function; the reference file:line is
 * cited next to each declaration (paths relative to the Rifraf.jl tree).
 * Parity of this restatement is pinned by the reference's own known-answer
 * tests (test/test_align.jl, test/test_utils.jl, test/test_model.jl,
 * test/test_bandedarrays.jl, test/test_rifrafsequences.jl,
 * test/test_correct_shifts.jl) re-run against it in tests/test_oracle_kats.py,
 * and end-to-end by data/consensus-results.fasta (tests/test_model_e2e.py).
 *
 * Conventions: 1-based indices (i, j) exactly as in the Julia source; band
 * storage is the reference's column-major `data[(i-j)+h_off+bw+1, j]` with
 * leading dimension H = 2*bw + |nrows-ncols| + 1 (bandedarrays.jl:101-114).
 * Bases are 2-bit codes A=0 C=1 G=2 T=3; 4 is the gap sentinel.
 */
#ifndef RIFRAF_ORACLE_H
#define RIFRAF_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Trace codes, align.jl:4-12 */
enum { OR_TRACE_NONE = 0, OR_TRACE_MATCH = 1, OR_TRACE_INSERT = 2,
       OR_TRACE_DELETE = 3, OR_TRACE_CODON_INSERT = 4,
       OR_TRACE_CODON_DELETE = 5 };

/* Proposal kinds (proposals.jl:1-15) */
enum { OR_SUB = 0, OR_INS = 1, OR_DEL = 2 };

/* Error codes mirror the reference's error() messages. */
enum { OR_OK = 0, OR_ERR_INVALID_SCORE = 1 /* "new score is invalid" align.jl:105-107 */,
       OR_ERR_NO_MOVE = 2 /* "failed to find a move" align.jl:108-110 */,
       OR_ERR_NO_VALID_SCORE = 3 /* "failed to compute a valid score" model.jl:282,380 */,
       OR_ERR_NO_NEW_COLS = 4 /* "no new columns need to be recomputed." model.jl:337 */,
       OR_ERR_WRONG_COLUMN = 5 /* "wrong column" model.jl:366 */,
       OR_ERR_BANDWIDTH = 6 /* "bandwidth must be positive" bandedarrays.jl:27 */ };

/* RifrafSequence score tables (rifrafsequences.jl:5-17). */
typedef struct {
    int n;                      /* length(seq) */
    const uint8_t *seq;         /* n base codes */
    const double *match;        /* n */
    const double *mismatch;     /* n */
    const double *ins;          /* n */
    const double *del;          /* n+1 */
    const double *cins;         /* n-2 or NULL */
    int ncins;                  /* length(codon_ins_scores) */
    const double *cdel;         /* n+1 or NULL */
    int ncdel;                  /* length(codon_del_scores) */
    int bw;                     /* bandwidth */
} or_seq;

/* bandedarrays.jl:101-104 */
int or_ndatarows(int nrows, int ncols, int bw);
/* bandedarrays.jl:44-53 */
void or_bandlimits(int nrows, int ncols, int bw, int *lower, int *upper);
/* bandedarrays.jl:133-137 */
void or_row_range(int nrows, int ncols, int bw, int j, int *start, int *stop);
/* bandedarrays.jl:151-157 */
int or_inband(int nrows, int ncols, int bw, int i, int j);
/* bandedarrays.jl:109-114 (returns 1-based data row, or 0 if out of band) */
int or_data_row(int nrows, int ncols, int bw, int i, int j);
/* bandedarrays.jl:220-231 */
void or_equal_ranges(int a_start, int a_stop, int b_start, int b_stop,
                     int *amin, int *amax, int *bmin, int *bmax);
/* bandedarrays.jl:176-198 (in place on a H x ncols column-major array) */
void or_flip(double *data, int H, int ncols);

/* rifrafsequences.jl:19-82: tables from log10 error probabilities.
 * cins (n-2) / cdel (n+1) are written only if the codon score > -Inf;
 * returns est_n_errors via *n_errors (Julia pairwise sum, reduce.jl). */
void or_seq_tables(const double *lp, int n, double mismatch, double insertion,
                   double deletion, double codon_insertion, double codon_deletion,
                   double *match, double *mism, double *ins, double *del,
                   double *cins, double *cdel, double *n_errors);

/* align.jl:50-112 -- exposed for unit tests. newcols is column-major with
 * leading dimension nc_ld (may be NULL when acol < 1). */
int or_update(const double *A, int nrows, int ncols, int bw,
              int i, int j, int s_base, int t_base, const or_seq *s,
              const double *newcols, int nc_ld, int doreverse, int acol,
              int trim, int skew, double *score, int *move);

/* align.jl:114-141 forward_moves! (moves may be NULL -> forward!) and
 * align.jl:155-179 forward!(doreverse).  A/moves are H x (m+1) column-major,
 * H = or_ndatarows(n+1, m+1, s->bw).  Out-of-band data entries are left
 * untouched. */
int or_forward(const uint8_t *t, int m, const or_seq *s, int doreverse,
               int trim, int skew, double *A, int8_t *moves);
/* align.jl:196-202 backward! = forward!(doreverse=true) + flip! */
int or_backward(const uint8_t *t, int m, const or_seq *s, double *B);

/* align.jl:229-238 backtrace: writes moves in alignment order, returns
 * the number of moves (<= n+m). */
int or_backtrace(const int8_t *moves, int nrows, int ncols, int bw, int8_t *out);
/* align.jl:240-245 count_errors via moves_to_aligned_seqs (align.jl:286-311) */
int or_count_errors(const int8_t *mv, int nmoves, const uint8_t *t,
                    const uint8_t *s);

/* util.jl:40-48 summax over two equal-length vectors */
double or_summax(const double *a, const double *b, int len);

/* model.jl:227-236 seq_score_deletion, model.jl:242-285 score_nocodon,
 * model.jl:302-383 score_proposal (dispatches on codon moves).
 * pos is the reference's 1-based Proposal.pos (Insertion(0,b) = before the
 * first base). newcols: caller scratch of (n+1) x 4 doubles. */
int or_score_proposal(int kind, int pos, int base,
                      const double *A, const double *B,
                      const uint8_t *t, int m, const or_seq *s,
                      double *newcols, double *score);

/* model.jl:385-399 left fold over reads (+ reference last).
 * A[k]/B[k] point at read k's bands; ref may be NULL. */
int or_score_total(int kind, int pos, int base, int nseqs,
                   const double *const *As, const double *const *Bs,
                   const or_seq *seqs, const double *Aref, const double *Bref,
                   const or_seq *ref, const uint8_t *t, int m,
                   double *newcols, double *total);

/* CPU baseline pass (bench.py cpu_baseline leg): for each read, forward
 * (with trace) + backward, then score the dense all_proposals set
 * (model.jl:401-456, STAGE_SCORE) against every read, totals left-folded.
 * nthreads > 1 parallelises over reads (DP) and positions (scoring).
 * Returns cells computed; totals laid out [pos 0..m][9] (sub A,C,G,T | del |
 * ins A,C,G,T) matching the engine's dense layout. */
/* model.jl:385-399 over a proposal list (the get_candidates / estimate_probs
 * loop, model.jl:519-523, :762-763): total[k] = 0.0 + s_1 + ... + s_R (+ s_ref)
 * and optionally per[k * width + r] = s_r (width = nseqs + (ref != NULL)).
 * Proposals are independent (OpenMP over k); the returned error is the one
 * the reference raises first (the earliest failing proposal, and within it
 * the earliest failing sequence). */
int or_score_list(int nprops, const int32_t *kind, const int32_t *pos, const int32_t *base,
                  int nseqs, const double *const *As, const double *const *Bs,
                  const or_seq *seqs, const double *Aref, const double *Bref,
                  const or_seq *ref, const uint8_t *t, int m,
                  double *per, double *total, int nthreads);

int64_t or_pass(const uint8_t *t, int m, int nseqs, const or_seq *seqs,
                double *totals, int nthreads);
/* or_pass continuing every proposal's fold from totals[] (chunked batches) */
int64_t or_pass_continue(const uint8_t *t, int m, int nseqs, const or_seq *seqs,
                         double *totals, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
