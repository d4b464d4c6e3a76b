/*
 * rifraf_oracle.c -- CPU restatement of the Rifraf.jl hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see rifraf_oracle.h).  Scalar, single-pass,
 * written to follow the Julia source line by line so that a reviewer can
 * check it against the cited file:line.  Parity pinned by the reference's
 * KATs re-run in tests/test_oracle_kats.py.
 */
#define _GNU_SOURCE
#include "rifraf_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define GAP 4
#define CODON_LENGTH 3                          /* util.jl:2 */

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------ */
/* Band geometry: bandedarrays.jl                                       */
/* ------------------------------------------------------------------ */

int or_ndatarows(int nrows, int ncols, int bw)            /* :101-104 */
{
    return 2 * bw + abs(nrows - ncols) + 1;
}

void or_bandlimits(int nrows, int ncols, int bw, int *lower, int *upper) /* :44-53 */
{
    if (ncols > nrows) {
        *lower = nrows - ncols - bw;
        *upper = bw;
    } else {
        *lower = -bw;
        *upper = nrows - ncols + bw;
    }
}

int or_inband(int nrows, int ncols, int bw, int i, int j)  /* :151-157 */
{
    int lower, upper;
    if (i < 1 || j < 1 || i > nrows || j > ncols)
        return 0;
    or_bandlimits(nrows, ncols, bw, &lower, &upper);
    return lower <= i - j && i - j <= upper;
}

int or_data_row(int nrows, int ncols, int bw, int i, int j) /* :109-114 */
{
    int h_offset = imax(ncols - nrows, 0);
    if (!or_inband(nrows, ncols, bw, i, j))
        return 0;                         /* reference: error("[i, j] is not in band") */
    return (i - j) + h_offset + bw + 1;
}

void or_row_range(int nrows, int ncols, int bw, int j, int *start, int *stop) /* :133-137 */
{
    int h_offset = imax(ncols - nrows, 0);
    int v_offset = imax(nrows - ncols, 0);
    *start = imax(1, j - h_offset - bw);
    *stop = imin(j + v_offset + bw, nrows);
}

void or_equal_ranges(int a_start, int a_stop, int b_start, int b_stop,
                     int *amin, int *amax, int *bmin, int *bmax) /* :220-231 */
{
    int alen = a_stop - a_start + 1;
    int blen = b_stop - b_start + 1;
    *amin = imax(b_start - a_start + 1, 1);
    *amax = alen - imax(a_stop - b_stop, 0);
    *bmin = imax(a_start - b_start + 1, 1);
    *bmax = blen - imax(b_stop - a_stop, 0);
}

void or_flip(double *data, int H, int ncols)               /* :176-198 */
{
    int nrows = H;
    int a = ncols / 2, b = ncols % 2;
#define D(i, j) data[(size_t)((i) - 1) + (size_t)H * (size_t)((j) - 1)]
    for (int j = 1; j <= a; j++) {
        for (int i = 1; i <= nrows; i++) {
            double first = D(i, j);
            double second = D(nrows - i + 1, ncols - j + 1);
            D(i, j) = second;
            D(nrows - i + 1, ncols - j + 1) = first;
        }
    }
    if (b == 1) {
        int c = nrows / 2;
        int j = a + 1;
        for (int i = 1; i <= c; i++) {
            double first = D(i, j);
            double second = D(nrows - i + 1, ncols - j + 1);
            D(i, j) = second;
            D(nrows - i + 1, ncols - j + 1) = first;
        }
    }
#undef D
}

/* Band element access with the reference's getindex default (:116-122). */
typedef struct {
    int nrows, ncols, bw, H, h_off;
} geom;

static inline geom mkgeom(int nrows, int ncols, int bw)
{
    geom g;
    g.nrows = nrows;
    g.ncols = ncols;
    g.bw = bw;
    g.H = or_ndatarows(nrows, ncols, bw);
    g.h_off = imax(ncols - nrows, 0);
    return g;
}

static inline size_t gidx(const geom *g, int i, int j)
{
    return (size_t)((i - j) + g->h_off + g->bw) + (size_t)g->H * (size_t)(j - 1);
}

static inline double gget(const double *data, const geom *g, int i, int j, double dflt)
{
    if (or_inband(g->nrows, g->ncols, g->bw, i, j))
        return data[gidx(g, i, j)];
    return dflt;
}

/* ------------------------------------------------------------------ */
/* Julia arithmetic helpers                                             */
/* ------------------------------------------------------------------ */

/* Base.max(::Float64, ::Float64) incl. NaN / signed-zero rules. */
static inline double jl_max(double x, double y)
{
    int take_y = (y > x) || (signbit(y) < signbit(x));
    if (take_y)
        return isnan(x) ? x : y;
    return isnan(y) ? y : x;
}

/* Julia 0.6 sum(::Vector{Float64}): sequential below 16 elements, else
 * pairwise (mapreduce_impl, blocksize 1024). */
static double jl_sum_impl(const double *a, long ifirst, long ilast)
{
    if (ifirst + 1024 > ilast) {
        double v = a[ifirst] + a[ifirst + 1];
        for (long i = ifirst + 2; i <= ilast; i++)
            v += a[i];
        return v;
    }
    long imid = (ifirst + ilast) >> 1;
    return jl_sum_impl(a, ifirst, imid) + jl_sum_impl(a, imid + 1, ilast);
}

static double jl_sum(const double *a, long n)
{
    if (n == 0)
        return 0.0;
    if (n == 1)
        return a[0];
    if (n < 16) {
        double v = a[0] + a[1];
        for (long i = 2; i < n; i++)
            v += a[i];
        return v;
    }
    return jl_sum_impl(a, 0, n - 1);
}

/* rifrafsequences.jl:19-82 */
void or_seq_tables(const double *lp, int n, double mismatch, double insertion,
                   double deletion, double codon_insertion, double codon_deletion,
                   double *match, double *mism, double *ins, double *del,
                   double *cins, double *cdel, double *n_errors)
{
    double *e = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int k = 0; k < n; k++) {
        match[k] = log10(1.0 - exp10(lp[k]));          /* :45 */
        mism[k] = lp[k] + mismatch;                    /* :46 */
        ins[k] = lp[k] + insertion;                    /* :47 */
    }
    del[0] = lp[0] + deletion;                         /* :49 */
    del[n] = lp[n - 1] + deletion;                     /* :50 */
    for (int k = 1; k <= n - 1; k++)                   /* :51-53 */
        del[k] = jl_max(lp[k - 1], lp[k]) + deletion;
    if (codon_insertion > -INFINITY && cins) {         /* :57-64 */
        for (int k = 2; k <= n - 1; k++)
            cins[k - 2] = jl_max(jl_max(lp[k - 2], lp[k - 1]), lp[k]) + codon_insertion;
    }
    if (codon_deletion > -INFINITY && cdel) {          /* :65-72 */
        cdel[0] = lp[0] + codon_deletion;
        cdel[n] = lp[n - 1] + codon_deletion;
        for (int k = 1; k <= n - 1; k++)
            cdel[k] = jl_max(lp[k - 1], lp[k]) + codon_deletion;
    }
    for (int k = 0; k < n; k++)
        e[k] = exp10(lp[k]);
    *n_errors = jl_sum(e, n);                          /* :74 */
    free(e);
}

/* ------------------------------------------------------------------ */
/* align.jl                                                             */
/* ------------------------------------------------------------------ */

static const int OFFSETS[6][2] = {{0, 0}, {1, 1}, {1, 0}, {0, 1}, {3, 0}, {0, 3}}; /* :14-18 */

/* align.jl:30-48 update_helper */
static inline void update_helper(double *final_score, int *final_move,
                                 double move_score, int move,
                                 const double *newcols, int nc_ld,
                                 const double *A, const geom *g,
                                 int i, int j, int acol)
{
    int prev_i = i - OFFSETS[move][0];
    int prev_j = j - OFFSETS[move][1];
    int rangecol = imin(prev_j, g->ncols);
    if (or_inband(g->nrows, g->ncols, g->bw, prev_i, rangecol)) {
        double score;
        if (acol < 1 || prev_j <= acol)
            score = gget(A, g, prev_i, prev_j, -INFINITY) + move_score;
        else
            score = newcols[(size_t)(prev_i - 1) + (size_t)nc_ld * (size_t)(prev_j - acol - 1)] + move_score;
        if (score > *final_score) {
            *final_score = score;
            *final_move = move;
        }
    }
}

static int update_g(const double *A, const geom *g, int i, int j,
                    int s_base, int t_base, const or_seq *s,
                    const double *newcols, int nc_ld, int doreverse, int acol,
                    int trim, int skew, double *score_out, int *move_out)
{
    double final_score = -INFINITY;
    int final_move = OR_TRACE_NONE;
    int nrows = g->nrows, ncols = g->ncols;
    int seqlen = s->n;
    /* align.jl:64-65 */
    int seq_i = doreverse ? imin(seqlen, seqlen - (i - 1) + 1) : imax(i - 1, 1);
    int del_i = doreverse ? nrows - i + 1 : i;
    double match_score = (s_base == t_base) ? s->match[seq_i - 1] : s->mismatch[seq_i - 1];
    double ins_score = s->ins[seq_i - 1];
    double del_score = s->del[del_i - 1];

    if (skew && s_base != t_base)                      /* :70-72 */
        match_score *= 0.99;
    if (trim && (j == 1 || j == ncols))                /* :74-76 */
        ins_score = 0.0;

    update_helper(&final_score, &final_move, match_score, OR_TRACE_MATCH, newcols, nc_ld, A, g, i, j, acol);
    update_helper(&final_score, &final_move, ins_score, OR_TRACE_INSERT, newcols, nc_ld, A, g, i, j, acol);
    update_helper(&final_score, &final_move, del_score, OR_TRACE_DELETE, newcols, nc_ld, A, g, i, j, acol);

    if (s->ncins > 0 || s->ncdel > 0) {                /* :87-104 */
        if (s->ncins > 0 && i > CODON_LENGTH) {
            int codon_i = i - CODON_LENGTH;
            if (doreverse)
                codon_i = s->ncins - codon_i + 1;
            double codon_ins_score = s->cins[codon_i - 1];
            update_helper(&final_score, &final_move, codon_ins_score, OR_TRACE_CODON_INSERT,
                          newcols, nc_ld, A, g, i, j, acol);
        }
        if (s->ncdel > 0 && j > CODON_LENGTH) {
            double codon_del_score = s->cdel[del_i - 1];
            update_helper(&final_score, &final_move, codon_del_score, OR_TRACE_CODON_DELETE,
                          newcols, nc_ld, A, g, i, j, acol);
        }
    }
    *score_out = final_score;
    *move_out = final_move;
    if (final_score == -INFINITY)                      /* :105-107 */
        return OR_ERR_INVALID_SCORE;
    if (final_move == OR_TRACE_NONE)                   /* :108-110 */
        return OR_ERR_NO_MOVE;
    return OR_OK;
}

int or_update(const double *A, int nrows, int ncols, int bw,
              int i, int j, int s_base, int t_base, const or_seq *s,
              const double *newcols, int nc_ld, int doreverse, int acol,
              int trim, int skew, double *score, int *move)
{
    geom g = mkgeom(nrows, ncols, bw);
    return update_g(A, &g, i, j, s_base, t_base, s, newcols, nc_ld, doreverse,
                    acol, trim, skew, score, move);
}

/* align.jl:114-141 (forward_moves!) and :155-179 (forward!) */
int or_forward(const uint8_t *t, int m, const or_seq *s, int doreverse,
               int trim, int skew, double *A, int8_t *moves)
{
    if (s->bw < 1)
        return OR_ERR_BANDWIDTH;
    int n = s->n;
    geom g = mkgeom(n + 1, m + 1, s->bw);
    A[gidx(&g, 1, 1)] = 0.0;
    if (moves)
        moves[gidx(&g, 1, 1)] = OR_TRACE_NONE;
    for (int j = 1; j <= g.ncols; j++) {
        int start, stop;
        or_row_range(g.nrows, g.ncols, g.bw, j, &start, &stop);
        for (int i = start; i <= stop; i++) {
            if (i == 1 && j == 1)
                continue;
            int sbase = i > 1 ? s->seq[doreverse ? n - (i - 1) : i - 2] : GAP;
            int tbase = j > 1 ? t[doreverse ? m - (j - 1) : j - 2] : GAP;
            double sc;
            int mv;
            int err = update_g(A, &g, i, j, sbase, tbase, s, NULL, 0, doreverse, -1,
                               trim, skew, &sc, &mv);
            if (err)
                return err;
            A[gidx(&g, i, j)] = sc;
            if (moves)
                moves[gidx(&g, i, j)] = (int8_t)mv;
        }
    }
    return OR_OK;
}

/* align.jl:196-202 */
int or_backward(const uint8_t *t, int m, const or_seq *s, double *B)
{
    int err = or_forward(t, m, s, 1, 0, 0, B, NULL);
    if (err)
        return err;
    or_flip(B, or_ndatarows(s->n + 1, m + 1, s->bw), m + 1);
    return OR_OK;
}

/* align.jl:229-238 */
int or_backtrace(const int8_t *moves, int nrows, int ncols, int bw, int8_t *out)
{
    geom g = mkgeom(nrows, ncols, bw);
    int i = nrows, j = ncols, k = 0;
    while (i > 1 || j > 1) {
        int mv = or_inband(nrows, ncols, bw, i, j) ? moves[gidx(&g, i, j)] : 0;
        if (mv < 1 || mv > 5)
            return -1;                                   /* Julia BoundsError */
        out[k++] = (int8_t)mv;
        i -= OFFSETS[mv][0];
        j -= OFFSETS[mv][1];
    }
    for (int a = 0, b = k - 1; a < b; a++, b--) {
        int8_t tmp = out[a];
        out[a] = out[b];
        out[b] = tmp;
    }
    return k;
}

/* align.jl:240-245 + moves_to_aligned_seqs :286-311 */
int or_count_errors(const int8_t *mv, int nmoves, const uint8_t *t, const uint8_t *s)
{
    int i = 0, j = 0, errs = 0;
    for (int k = 0; k < nmoves; k++) {
        int m = mv[k];
        i += OFFSETS[m][0];
        j += OFFSETS[m][1];
        switch (m) {
        case OR_TRACE_MATCH:
            errs += (t[j - 1] != s[i - 1]);
            break;
        case OR_TRACE_INSERT:
        case OR_TRACE_DELETE:
            errs += 1;
            break;
        case OR_TRACE_CODON_INSERT:
        case OR_TRACE_CODON_DELETE:
            errs += 3;
            break;
        default:
            break;
        }
    }
    return errs;
}

/* util.jl:40-48 */
double or_summax(const double *a, const double *b, int len)
{
    double result = a[0] + b[0];
    for (int i = 1; i < len; i++)
        result = jl_max(result, a[i] + b[i]);
    return result;
}

/* ------------------------------------------------------------------ */
/* model.jl scoring                                                     */
/* ------------------------------------------------------------------ */

/* sparsecol(B, j)[bmin:bmax] pointer + overlap length against rows (imin, imax) */
static double summax_cols(const double *acol_vals, int imin_, int imax_,
                          const double *B, const geom *g, int bj)
{
    int bstart, bstop, amin, amax, bmin, bmax;
    or_row_range(g->nrows, g->ncols, g->bw, bj, &bstart, &bstop);
    or_equal_ranges(imin_, imax_, bstart, bstop, &amin, &amax, &bmin, &bmax);
    const double *bcol = B + gidx(g, bstart, bj);      /* sparsecol, :146-149 */
    return or_summax(acol_vals + (amin - 1), bcol + (bmin - 1), amax - amin + 1);
}

/* model.jl:227-236 */
static double seq_score_deletion(const double *A, const double *B, const geom *g,
                                 int acol, int bcol)
{
    int astart, astop;
    or_row_range(g->nrows, g->ncols, g->bw, acol, &astart, &astop);
    const double *Acol = A + gidx(g, astart, acol);
    return summax_cols(Acol, astart, astop, B, g, bcol);
}

/* model.jl:242-285 */
static int score_nocodon(int kind, int pos, int base, const double *A, const double *B,
                         const geom *g, const or_seq *s, double *newcols, double *out)
{
    if (kind == OR_DEL) {
        *out = seq_score_deletion(A, B, g, pos, pos + 1);
        return OR_OK;
    }
    int nrows = g->nrows, ncols = g->ncols;
    int acol = pos + (kind == OR_SUB ? 0 : 1);
    int new_acol = acol + 1;
    int amin, amax;
    or_row_range(nrows, ncols, g->bw, imin(new_acol, ncols), &amin, &amax);
    for (int i = amin; i <= amax; i++) {
        int seq_base = i > 1 ? s->seq[i - 2] : GAP;
        double sc;
        int mv;
        int err = update_g(A, g, i, new_acol, seq_base, base, s, newcols, nrows, 0, acol,
                           0, 0, &sc, &mv);
        if (err)
            return err;
        newcols[i - 1] = sc;
    }
    int bj = pos + 1;
    double score = summax_cols(newcols + (amin - 1), amin, amax, B, g, bj);
    if (score == -INFINITY)
        return OR_ERR_NO_VALID_SCORE;
    *out = score;
    return OR_OK;
}

/* model.jl:302-383 */
int or_score_proposal(int kind, int pos, int base,
                      const double *A, const double *B,
                      const uint8_t *t, int m, const or_seq *s,
                      double *newcols, double *score)
{
    geom g = mkgeom(s->n + 1, m + 1, s->bw);
    if (!(s->ncins > 0 || s->ncdel > 0))
        return score_nocodon(kind, pos, base, A, B, &g, s, newcols, score);

    int nrows = g.nrows, ncols = g.ncols;
    int acol_offset = kind == OR_INS ? 0 : -1;                 /* :312 */
    int acol = pos + acol_offset + 1;                          /* :313 */
    int boff = kind == OR_INS ? 1 : 2;                         /* BOFFSETS :238-240 */
    int first_bcol = acol + boff;
    int last_bcol = first_bcol + CODON_LENGTH - 1;

    if (kind == OR_DEL && acol == ncols - 1) {                 /* :320-323 */
        *score = gget(A, &g, nrows, ncols - 1, -INFINITY);
        return OR_OK;
    }
    int just_a = last_bcol >= ncols;                           /* :329 */
    int n_after = !just_a ? CODON_LENGTH : m - pos;            /* :332 */
    int n_new_bases = kind == OR_DEL ? 0 : 1;
    if (n_new_bases == 0 && n_after == 0)
        return OR_ERR_NO_NEW_COLS;
    int n_new = n_new_bases + n_after;

    /* get_consensus_substring, model.jl:287-300 */
    uint8_t sub_consensus[8];
    int nsub = 0;
    if (kind != OR_DEL)
        sub_consensus[nsub++] = (uint8_t)base;
    int stop = imin(pos + 1 + n_after - 1, m);
    for (int k = pos + 1; k <= stop; k++)
        sub_consensus[nsub++] = t[k - 1];
    if (nsub < n_new)
        return -1;                                             /* Julia BoundsError */

    for (int j = 1; j <= n_new; j++) {                        /* :343-352 */
        int range_col = imin(acol + j, ncols);
        int amin, amax;
        or_row_range(nrows, ncols, g.bw, range_col, &amin, &amax);
        for (int i = amin; i <= amax; i++) {
            int seq_base = i > 1 ? s->seq[i - 2] : GAP;
            double sc;
            int mv;
            int err = update_g(A, &g, i, acol + j, seq_base, sub_consensus[j - 1], s,
                               newcols, nrows, 0, acol, 0, 0, &sc, &mv);
            if (err)
                return err;
            newcols[(size_t)(i - 1) + (size_t)nrows * (size_t)(j - 1)] = sc;
        }
    }
    if (just_a) {                                              /* :354-356 */
        *score = newcols[(size_t)(nrows - 1) + (size_t)nrows * (size_t)(n_new - 1)];
        return OR_OK;
    }
    double best_score = -INFINITY;
    for (int j = 1; j <= CODON_LENGTH; j++) {                  /* :360-378 */
        int new_j = n_new - CODON_LENGTH + j;
        int imn, imx;
        or_row_range(nrows, ncols, g.bw, imin(acol + new_j, ncols), &imn, &imx);
        const double *Acol = newcols + (size_t)nrows * (size_t)(new_j - 1) + (imn - 1);
        int bj = first_bcol + j - 1;
        if (bj > ncols)
            return OR_ERR_WRONG_COLUMN;
        double sc = summax_cols(Acol, imn, imx, B, &g, bj);
        if (sc > best_score)
            best_score = sc;
    }
    if (best_score == -INFINITY)
        return OR_ERR_NO_VALID_SCORE;
    *score = best_score;
    return OR_OK;
}

/* model.jl:385-399 */
/* the left fold of model.jl:389-397 continued from `score` (0.0 for a whole
   batch; a running total when a batch is scored chunk by chunk) */
static int score_fold(double score, int kind, int pos, int base, int nseqs,
                      const double *const *As, const double *const *Bs,
                      const or_seq *seqs, const double *Aref, const double *Bref,
                      const or_seq *ref, const uint8_t *t, int m,
                      double *newcols, double *total)
{
    for (int si = 0; si < nseqs; si++) {
        double sc;
        int err = or_score_proposal(kind, pos, base, As[si], Bs[si], t, m, &seqs[si], newcols, &sc);
        if (err)
            return err;
        score += sc;
    }
    if (ref) {
        double sc;
        int err = or_score_proposal(kind, pos, base, Aref, Bref, t, m, ref, newcols, &sc);
        if (err)
            return err;
        score += sc;
    }
    *total = score;
    return OR_OK;
}

int or_score_total(int kind, int pos, int base, int nseqs,
                   const double *const *As, const double *const *Bs,
                   const or_seq *seqs, const double *Aref, const double *Bref,
                   const or_seq *ref, const uint8_t *t, int m,
                   double *newcols, double *total)
{
    return score_fold(0.0, kind, pos, base, nseqs, As, Bs, seqs, Aref, Bref, ref, t, m, newcols, total);
}

/* model.jl:385-399 for a proposal list, proposals in parallel */
int or_score_list(int nprops, const int32_t *kind, const int32_t *pos, const int32_t *base,
                  int nseqs, const double *const *As, const double *const *Bs,
                  const or_seq *seqs, const double *Aref, const double *Bref,
                  const or_seq *ref, const uint8_t *t, int m,
                  double *per, double *total, int nthreads)
{
    const int width = nseqs + (ref ? 1 : 0);
    int maxn = ref ? ref->n : 0;
    for (int r = 0; r < nseqs; r++)
        maxn = imax(maxn, seqs[r].n);
    int *errs = (int *)calloc((size_t)(nprops > 0 ? nprops : 1), sizeof(int));
#ifdef _OPENMP
    if (nthreads < 1)
        nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        double *newcols = (double *)malloc(sizeof(double) * (size_t)(maxn + 1) * (CODON_LENGTH + 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int k = 0; k < nprops; k++) {
            double score = 0.0;
            int err = 0;
            for (int r = 0; r < width && !err; r++) {
                double sc = 0.0;
                if (r < nseqs)
                    err = or_score_proposal(kind[k], pos[k], base[k], As[r], Bs[r], t, m, &seqs[r], newcols, &sc);
                else
                    err = or_score_proposal(kind[k], pos[k], base[k], Aref, Bref, t, m, ref, newcols, &sc);
                if (!err) {
                    score += sc;
                    if (per)
                        per[(size_t)k * width + r] = sc;
                }
            }
            errs[k] = err;
            total[k] = score;
        }
        free(newcols);
    }
    int first = 0;
    for (int k = 0; k < nprops && !first; k++)
        first = errs[k];
    free(errs);
    return first;
}

/* CPU baseline pass: realign (forward_moves! + backward!) every read, then
 * score the dense STAGE_SCORE all_proposals set (model.jl:401-456) with the
 * left-fold total of model.jl:385-399. */
static int64_t pass_fold(const uint8_t *t, int m, int nseqs, const or_seq *seqs,
                         double *totals, int cont, int nthreads);

int64_t or_pass(const uint8_t *t, int m, int nseqs, const or_seq *seqs,
                double *totals, int nthreads)
{
    return pass_fold(t, m, nseqs, seqs, totals, 0, nthreads);
}

/* or_pass over the next chunk of a batch: every proposal's fold continues
   from totals[] (the previous chunks' running totals, in batch order), so a
   batch too large to hold all its bands at once is folded chunk by chunk
   with the reference's order and rounding */
int64_t or_pass_continue(const uint8_t *t, int m, int nseqs, const or_seq *seqs,
                         double *totals, int nthreads)
{
    return pass_fold(t, m, nseqs, seqs, totals, 1, nthreads);
}

static int64_t pass_fold(const uint8_t *t, int m, int nseqs, const or_seq *seqs,
                         double *totals, int cont, int nthreads)
{
    double **As = (double **)calloc((size_t)nseqs, sizeof(double *));
    double **Bs = (double **)calloc((size_t)nseqs, sizeof(double *));
    int64_t cells = 0;
    int failed = 0;
#ifdef _OPENMP
    if (nthreads < 1)
        nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) reduction(+ : cells)
#endif
    for (int r = 0; r < nseqs; r++) {
        int H = or_ndatarows(seqs[r].n + 1, m + 1, seqs[r].bw);
        size_t sz = (size_t)H * (size_t)(m + 1);
        As[r] = (double *)malloc(sz * sizeof(double));
        Bs[r] = (double *)malloc(sz * sizeof(double));
        int8_t *mv = (int8_t *)malloc(sz);
        if (or_forward(t, m, &seqs[r], 0, 0, 0, As[r], mv) || or_backward(t, m, &seqs[r], Bs[r]))
            failed = 1;
        free(mv);
        for (int j = 1; j <= m + 1; j++) {
            int a, b;
            or_row_range(seqs[r].n + 1, m + 1, seqs[r].bw, j, &a, &b);
            cells += 2 * (int64_t)(b - a + 1);
        }
    }
    if (!failed) {
        int maxn = 0;
        for (int r = 0; r < nseqs; r++)
            maxn = imax(maxn, seqs[r].n);
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
        {
            double *newcols = (double *)malloc(sizeof(double) * (size_t)(maxn + 1) * (CODON_LENGTH + 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
            for (int p = 0; p <= m; p++) {
                double *row = totals + (size_t)p * 9;
                double st[9];
                for (int k = 0; k < 9; k++) {
                    st[k] = cont ? row[k] : 0.0;
                    row[k] = -INFINITY;
                }
                for (int b = 0; b < 4 && p >= 1; b++) {
                    if (t[p - 1] == b)
                        continue;
                    if (score_fold(st[b], OR_SUB, p, b, nseqs, (const double *const *)As,
                                   (const double *const *)Bs, seqs, NULL, NULL, NULL,
                                   t, m, newcols, &row[b]))
                        failed = 1;
                }
                if (p >= 1 && score_fold(st[4], OR_DEL, p, 0, nseqs, (const double *const *)As,
                                         (const double *const *)Bs, seqs, NULL, NULL, NULL,
                                         t, m, newcols, &row[4]))
                    failed = 1;
                for (int b = 0; b < 4; b++)
                    if (score_fold(st[5 + b], OR_INS, p, b, nseqs, (const double *const *)As,
                                   (const double *const *)Bs, seqs, NULL, NULL, NULL,
                                   t, m, newcols, &row[5 + b]))
                        failed = 1;
            }
            free(newcols);
        }
    }
    for (int r = 0; r < nseqs; r++) {
        free(As[r]);
        free(Bs[r]);
    }
    free(As);
    free(Bs);
    return failed ? -1 : cells;
}
