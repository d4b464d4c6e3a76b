// rifraf_hip.hip -- MI355X (gfx950) engine for the RIFRAF hot path.
//
// Kernels (all FP64 max-plus, bit-exact with the reference's evaluation
// order; no MFMA: the path has no dense contraction):
//   k_dpr       banded forward / reverse Viterbi fill (forward_moves!,
//               forward!, backward! = reverse forward + flip!), many tasks
//               per launch: 16-, 32- or 64-lane tasks, systolic DPP lanes
//               src/align.jl:50-112 (update), :114-179, :196-202
//   k_dpx       the same fill for a few long tasks (H <= 127), one
//               latency-bound task per wave (the reference's codon DP)
//   k_dpm / k_dp  very wide bands (edit_distance, align.jl:253-260): band
//               slices across the CUs of an XCD / one block per band
//   k_score_ws / k_score_segl / k_score
//               dense per-position proposal scoring of every batch read,
//               left-folded over the batch in batch order
//               src/model.jl:227-285 (seq_score_deletion, score_nocodon),
//               :385-399 (fold)
//   k_codon     codon-move scoring (reference sequence), one lane per
//               proposal  src/model.jl:287-383
//   k_reduce    ordered fold of per-read partials (split mode)
//   k_gather    proposal list -> totals (+ reference score, last)
//   k_bt_win    moves recomputed from the stored A band, backtrace +
//               count_errors (+ alignment_proposals' mask)
//               src/align.jl:229-245, src/model.jl:458-497
//   k_tables / k_code_prep / k_aln_* / k_qv  device setup and QV pass
//
// Host side: device arenas (sequences, templates, bands), descriptor
// upload, the C-ABI of include/rifraf_hip.h.

#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/rifraf_hip.h"

#define RF_INF (__builtin_inf())

// ---------------------------------------------------------------------
// Band storage on the device: anti-diagonal-major ("kappa-major")
//
//   d     = ii - jj + c    0-based data row of the reference layout
//                          (bandedarrays.jl:109-114), c = h_off + bw
//   kappa = d + 2*jj       anti-diagonal of cell (ii, jj)
//   element (d, jj) lives at band[kappa * P + (d >> 1)],
//   P = ceil(H/2) | 1 (odd row stride: the scorer's lanes read LDS at stride
//   2P; an even P measured 3 % slower scoring with no DP gain in a same-box
//   A/B, despite 4-16 % fewer band bytes), kappa in [0, K), K = H + 2m.
//
// A kappa row holds one anti-diagonal (all band rows d of one parity), so the
// DP fill stores every step as one contiguous run, and a window of columns
// is one contiguous block of rows for the scorer.  The reference's
// column-major `data` is produced on download (rf_download_band).
// ---------------------------------------------------------------------

typedef double dvec2 __attribute__((ext_vector_type(2)));

// Band stores of the DP fill: nontemporal (streamed once, read back by the
// scorer much later; measured ~5 % faster than plain stores on MI355X)
#ifndef RIFRAF_DP_PLAIN_STORES
#define DP_STORE(p, v) __builtin_nontemporal_store((v), (p))
#else
#define DP_STORE(p, v) (*(p) = (v))
#endif

__host__ __device__ inline int band_P(int H) { return ((H + 1) >> 1) | 1; }
// Row stride of a band as allocated: H >= pad_h (> 0) gives rows of a whole
// number of 128-B lines, so that the wide-band scorer's 32-diagonal segments
// read exactly one line per kappa row (k_score_segl); else the odd stride.
// rf_realign pads every band of a call whose widest band has H >=
// RF_OPT_BAND_PAD (pad_h 1 for the call), none otherwise.
inline int band_stride(int H, int pad_h)
{
    return (pad_h > 0 && H >= pad_h) ? (((H + 1) >> 1) + 15) & ~15 : band_P(H);
}
__host__ __device__ inline int64_t band_K(int H, int m) { return (int64_t)H + 2 * (int64_t)m; }

__device__ __forceinline__ size_t bidx(int d, int jj, int P)
{
    return (size_t)(d + 2 * jj) * (size_t)P + (size_t)(d >> 1);
}

// ---------------------------------------------------------------------
// device-side descriptors
// ---------------------------------------------------------------------

// One DP fill task = (slot, direction).
struct alignas(16) DPTask {
    int64_t band;   // output band offset (doubles)
    int64_t sb;     // sequence bases offset (bytes)
    int64_t tab;    // sequence tables offset (doubles)
    int64_t tb;     // template bases offset (bytes)
    int32_t n, m, bw, H;
    int32_t c;      // h_off + bw
    int32_t ncins, ncdel;
    int32_t flags;  // 1 = reverse, 2 = skew, 4 = trim
    int32_t out_idx;
    int32_t klen;   // number of anti-diagonals K = H + 2m
    int32_t P;      // kappa row stride
    int32_t pad;
};

// DPTask.flags bit: the read carries row codes (rf_set_sequences) -- one
// 8-B record per read position i: bits 0-15 the code of (match, mismatch,
// ins)[i], 16-31 / 32-47 the codes of del[i] / del[i+1], 48-55 the base.
// Codes index the context's dictionary: RF_CODES entries of 4 doubles
// {match, mismatch, ins, 0}, then RF_CODES del values.
constexpr int RF_TASK_CODED = 1024;
constexpr int RF_CODES = 1 << 16;
// doubles from a read's table start to its row-code records
__host__ __device__ inline int64_t row_code_off(int64_t n, int64_t nci, int64_t ncd) { return 4 * n + 1 + nci + ncd; }

// One batch read of a scoring group.
struct alignas(16) ScoreRead {
    int64_t A, B;     // band offsets (doubles)
    int64_t sb, tab;  // sequence bases / tables
    int32_t n, bw, H, c;
    int32_t vb;       // v_off + bw
    int32_t P, K;
    int32_t flags;    // SR_CODED: row-code records follow the tables (no codon tables)
};
constexpr int SR_CODED = 1;

struct alignas(16) ScoreGroup {
    int64_t tb;         // template bases
    int64_t dense_off;  // totals [m+1][9]
    int64_t split_off;  // per-read partials base (split mode)
    int32_t r0, r1;     // reads [r0, r1) in the ScoreRead list
    int32_t m, pad;
};

struct alignas(8) WorkItem {
    int32_t group, p0;
};

struct alignas(16) CodonTask {
    int64_t A, B, sb, tab, tb;
    int64_t scratch;   // newcols scratch offset (doubles), 4 * (n+1)
    int32_t n, m, bw, H;
    int32_t ncins, ncdel;
    int32_t kind, pos, base;
    int32_t out_idx;
    int32_t P, pad;
};

struct alignas(16) BTTask {
    int64_t A, sb, tab, tb, out;
    int32_t n, m, bw, H;
    int32_t ncins, ncdel, flags, idx;
    int32_t P, pad;
    int64_t mask;   // k_bt_win with a proposal mask: byte offset of the cluster's (m+1) x 9 mask
};

// error word: first error code wins (atomicCAS)
__device__ __forceinline__ void set_err(int *err, int code)
{
    atomicCAS(err, 0, code);
}

// Order LDS traffic between the lanes of one wave: LDS instructions of a
// wave execute in issue order, so only the compiler has to be fenced.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier ordering LDS only: the fences name the local address
// space, so the wait before s_barrier is lgkmcnt(0) -- a wave's global
// stores in flight are not drained (vmcnt counts loads and stores alike).
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---------------------------------------------------------------------
// k_dp: anti-diagonal wavefront DP fill
//
// Cell (ii, jj) depends on kappa-1 (insert: d-1, delete: d+1), kappa-2
// (match: d) and kappa-3 (codon insert d-3, codon delete d+3).  Lane q of a
// W-lane segment owns the pair of band rows {2q, 2q+1}; at anti-diagonal
// kappa it computes d = 2q + (kappa & 1), so every lane produces one cell per
// step (lanes loop over further pairs when H > 2W).  One task per segment,
// 64/W tasks per single-wave workgroup; the last four anti-diagonals live in
// an LDS ring padded with -Inf sentinels.  Out-of-band predecessors read
// -Inf, which never wins the strict '>' (align.jl:43) -- identical to the
// reference's inband() skip.  The candidates are evaluated in the
// reference's order with the same FP64 additions, so A/B are bit-identical
// to the scalar reference.  Each step's cells are one contiguous run of the
// kappa-major band; the reverse pass stores in flip!'ed position
// (bandedarrays.jl:176-198): kappa' = K-1-kappa, d' = H-1-d.
// ---------------------------------------------------------------------

// NT threads per block (64: one wave, 64 / W tasks; W = NT = DPW_NT: one task
// per block of DPW_NT / 64 waves -- the very wide bands of edit_distance,
// H ~ m, whose single task is latency-bound: more lanes per anti-diagonal and
// the ring in LDS (up to DPW_LDS_H) instead of global memory, round 4).
template <int W, bool GRING, int NT = 64>
__global__ void __launch_bounds__(NT)
k_dp(const DPTask *__restrict__ tasks, int ntasks, const uint8_t *__restrict__ bases,
     const double *__restrict__ tabs, double *__restrict__ bands,
     double *__restrict__ out_score, int *__restrict__ err, int ring_ld,
     double *__restrict__ gring)
{
    constexpr int SEGS = NT / W;
    constexpr bool BLOCK_SYNC = GRING || NT > 64;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int seg = threadIdx.x / W;
    const int q = threadIdx.x % W;
    const int tid = blockIdx.x * SEGS + seg;

    DPTask T = {};
    if (tid < ntasks)
        T = tasks[tid];
    double *ring = GRING ? gring + (size_t)blockIdx.x * 4 * ring_ld
                         : smem + (size_t)seg * 4 * ring_ld;
    for (int e = q; e < 4 * ring_ld; e += W)
        ring[e] = -RF_INF;
    int kmax = T.klen;
    for (int off = 32; off >= 1; off >>= 1)
        kmax = max(kmax, __shfl_xor(kmax, off));
    if (BLOCK_SYNC)
        __syncthreads();
    else
        wave_sync();

    const bool rev = T.flags & 1;
    const bool skew = T.flags & 2;
    const bool trim = T.flags & 4;
    const uint8_t *sbase = bases + T.sb;
    const uint8_t *tbase = bases + T.tb;
    const double *tb = tabs + T.tab;
    const double *t_match = tb;
    const double *t_mism = tb + T.n;
    const double *t_ins = tb + 2 * (size_t)T.n;
    const double *t_del = tb + 3 * (size_t)T.n;
    const double *t_cins = tb + 4 * (size_t)T.n + 1;
    const double *t_cdel = t_cins + T.ncins;
    double *band = bands + T.band;

    for (int k = 0; k < kmax; ++k) {
        if (k < T.klen) {
            const int par = k & 1;
            double *r0 = ring + (k & 3) * ring_ld + 3;
            const double *r1 = ring + ((k - 1) & 3) * ring_ld + 3;
            const double *r2 = ring + ((k - 2) & 3) * ring_ld + 3;
            const double *r3 = ring + ((k - 3) & 3) * ring_ld + 3;
            double *row = band + (size_t)(rev ? T.klen - 1 - k : k) * T.P;
            for (int pp = q;; pp += W) {
                const int d = 2 * pp + par;
                if (d >= T.H || d > k)
                    break;
                const int jj = (k - d) >> 1;
                double v = -RF_INF;
                if (jj <= T.m) {
                    const int ii = d + jj - T.c;
                    if (ii >= 0 && ii <= T.n) {
                        if (ii == 0 && jj == 0) {
                            v = 0.0;
                        } else {
                            // align.jl:64-76 score lookups
                            const int sb = ii >= 1 ? sbase[rev ? T.n - ii : ii - 1] : 4;
                            const int tbb = jj >= 1 ? tbase[rev ? T.m - jj : jj - 1] : 4;
                            const int ks = rev ? min(T.n - 1, T.n - ii) : max(ii - 1, 0);
                            const int kd = rev ? T.n - ii : ii;
                            double ms = (sb == tbb) ? t_match[ks] : t_mism[ks];
                            double is = t_ins[ks];
                            const double ds = t_del[kd];
                            if (skew && sb != tbb)
                                ms *= 0.99;
                            if (trim && (jj == 0 || jj == T.m))
                                is = 0.0;
                            // align.jl:77-104, strict '>' in reference order
                            double best = -RF_INF, s;
                            s = r2[d] + ms;
                            if (s > best) best = s;
                            s = r1[d - 1] + is;
                            if (s > best) best = s;
                            s = r1[d + 1] + ds;
                            if (s > best) best = s;
                            if (T.ncins > 0 && ii >= 3) {
                                const int ci = rev ? T.ncins - ii + 2 : ii - 3;
                                s = r3[d - 3] + t_cins[ci];
                                if (s > best) best = s;
                            }
                            if (T.ncdel > 0 && jj >= 3) {
                                s = r3[d + 3] + t_cdel[kd];
                                if (s > best) best = s;
                            }
                            if (best == -RF_INF)
                                set_err(err, 1);  // "new score is invalid"
                            v = best;
                        }
                        if (ii == T.n && jj == T.m && out_score)
                            out_score[T.out_idx] = v;
                    }
                }
                row[(rev ? T.H - 1 - d : d) >> 1] = v;
                r0[d] = v;
            }
        }
        // an LDS ring needs an LDS-only barrier (round 6: __syncthreads also
        // drained the step's band stores); the global ring needs the full one
        if (BLOCK_SYNC && GRING)
            __syncthreads();
        else if (BLOCK_SYNC)
            lds_barrier();
        else
            wave_sync();
    }
}
// widest band whose four-diagonal ring fits the LDS of k_dp<DPW_NT, false, DPW_NT>
constexpr int DPW_LDS_H = 160 * 1024 / 32 - 6;
// lanes of the very-wide-band task (edit_distance's band, H ~ m): each lane
// walks ceil(H/2 / DPW_NT) pairs per anti-diagonal, one dependent table /
// ring round trip each, so the step time falls with the lanes until the
// block barrier dominates (round 4: 256 -> 1024)
#ifndef DPW_NT
#define DPW_NT 1024
#endif

// ---------------------------------------------------------------------
// k_dpr: register-resident variant of k_dp for bands up to H <= 32*NP.
//
// Same recurrence, cell order and FP64 sums as k_dp; the anti-diagonals
// kappa-1..kappa-3 live in registers instead of an LDS ring.  Each task owns
// one 16-lane DPP row (4 tasks per wave); lane q holds band-row pairs
// q*NP .. q*NP+NP-1, and the only cross-lane traffic per step is the pair
// at each block edge, moved with DPP row shifts (v_mov_b32_dpp row_shr /
// row_shl).  Lanes outside the row read the -Inf "bound" value, i.e. an
// out-of-band predecessor, exactly like the ring's sentinels.
// ---------------------------------------------------------------------

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)0xFFF00000, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
#define DPP_FROM_L1 0x111   // row_shr:1 -> value of lane q-1
#define DPP_FROM_L2 0x112   // row_shr:2 -> lane q-2
#define DPP_FROM_R1 0x101   // row_shl:1 -> lane q+1
#define DPP_FROM_R2 0x102   // row_shl:2 -> lane q+2
// Lanes per DP task: 16 (one DPP row, 4 tasks per wave), 32 (two tasks per
// wave) or 64 (the whole wave).  32 and 64 use wave_shr / wave_shl /
// wave_ror / wave_rol, the same moves across DPP rows.  With 32 lanes the
// wave shifts also cross the two tasks: lane 32 (31) would read lane 31's
// (32's) value where it should read its task's edge, so those lanes select
// the edge after the move (EDGE_FIX).  The rotations need no fix: the lanes
// they wrap between hold a task's top pairs, whose diagonals are >= H (the
// host's class bound), i.e. -Inf or masked, exactly as within a DPP row.
template <int LPT>
struct TaskLanes {
    static_assert(LPT == 16 || LPT == 32 || LPT == 64, "tasks are 16, 32 or 64 lanes");
    static constexpr int FROM_L1 = LPT >= 32 ? 0x138 : 0x111;   // lane q-1 (edge lane 0 reads `old`)
    static constexpr int FROM_R1 = LPT >= 32 ? 0x130 : 0x101;   // lane q+1 (edge lane LPT-1 reads `old`)
    static constexpr int ROT_L1 = LPT >= 32 ? 0x13C : 0x121;    // lane (q-1) mod LPT (or mod 64)
    static constexpr int ROT_R1 = LPT >= 32 ? 0x134 : 0x12F;    // lane (q+1) mod LPT (or mod 64)
    static constexpr bool EDGE_FIX = LPT == 32;
};

// Shift an int / double across the 16-lane DPP row (lanes outside the row
// read `bound`).
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int x, int bound)
{
    return __builtin_amdgcn_update_dpp(bound, x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64_any(double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// one {sub A, C, G, T, ins, del} record per read row i (align.jl:60-69)
__device__ __forceinline__ void lean_row(double *rec, int sbse, double mt, double mm, double ins, double del)
{
    double2 *r2 = (double2 *)rec;
    r2[0] = make_double2(sbse == 0 ? mt : mm, sbse == 1 ? mt : mm);
    r2[1] = make_double2(sbse == 2 ? mt : mm, sbse == 3 ? mt : mm);
    r2[2] = make_double2(ins, del);
}

// Per-row inputs of the recurrence (align.jl:64-76, :87-103): the read base
// and the score-table entries row ii uses, in forward or reverse indexing.
struct RowRec {
    int sb;
    double mt, mm, is, ds, ci, cd;
};

__device__ __forceinline__ RowRec load_row(const DPTask &T, bool rev, const uint8_t *sbase,
                                           const double *tb, int ii, bool codon)
{
    RowRec r;
    if (ii < 0 || ii > T.n) {
        r.sb = 4;
        r.mt = r.mm = r.is = r.ds = r.ci = r.cd = -RF_INF;
        return r;
    }
    r.sb = ii >= 1 ? sbase[rev ? T.n - ii : ii - 1] : 4;
    const int ks = rev ? min(T.n - 1, T.n - ii) : max(ii - 1, 0);
    const int kd = rev ? T.n - ii : ii;
    r.mt = tb[ks];
    r.mm = tb[T.n + ks];
    r.is = tb[2 * (size_t)T.n + ks];
    r.ds = tb[3 * (size_t)T.n + kd];
    r.ci = -RF_INF;
    r.cd = -RF_INF;
    if (codon) {
        const double *t_cins = tb + 4 * (size_t)T.n + 1;
        if (T.ncins > 0 && ii >= 3)
            r.ci = t_cins[rev ? T.ncins - ii + 2 : ii - 3];
        if (T.ncdel > 0)
            r.cd = t_cins[T.ncins + kd];
    }
    return r;
}

// A row record as loaded (no select applied yet: selecting right after the
// loads would make the wave wait for them at once) -- RowRec via row_val.
struct RawRow {
    int sb, fl;   // fl: bit 0 row in range, bit 1 base row (ii >= 1), bit 2 codon insert, bit 3 codon delete
    double mt, mm, is, ds, ci, cd;
};
__device__ __forceinline__ RawRow load_row_raw(const DPTask &T, bool rev, const uint8_t *sbase,
                                               const double *tb, int ii, bool codon)
{
    const bool in = ii >= 0 && ii <= T.n;
    const int ic = min(max(ii, 1), T.n);
    const int iz = min(max(ii, 0), T.n);
    // every index >= 0 also for a padding task (T = {}: n = 0), whose loads
    // read the first entries of the arenas and are discarded
    const int ks = max(rev ? min(T.n - 1, T.n - iz) : iz - 1, 0);
    const int kd = rev ? T.n - iz : iz;
    const int ci_i = rev ? T.ncins - iz + 2 : iz - 3;
    const int64_t ci_off = T.ncins > 0 ? 4 * (int64_t)T.n + 1 + min(max(ci_i, 0), T.ncins - 1) : ks;
    const int64_t cd_off = T.ncdel > 0 ? 4 * (int64_t)T.n + 1 + T.ncins + kd : ks;
    RawRow r;
    r.sb = sbase[max(rev ? T.n - ic : ic - 1, 0)];
    r.mt = tb[ks];
    r.mm = tb[T.n + ks];
    r.is = tb[2 * (size_t)T.n + ks];
    r.ds = tb[3 * (size_t)T.n + kd];
    r.ci = tb[ci_off];
    r.cd = tb[cd_off];
    r.fl = (in ? 1 : 0) | ((in && ii >= 1) ? 2 : 0) | ((codon && T.ncins > 0 && ii >= 3 && in) ? 4 : 0) |
           ((codon && T.ncdel > 0 && in) ? 8 : 0);
    return r;
}
__device__ __forceinline__ RowRec row_val(const RawRow &x)
{
    RowRec r;
    const bool in = x.fl & 1;
    r.sb = (x.fl & 2) ? x.sb : 4;
    r.mt = in ? x.mt : -RF_INF;
    r.mm = in ? x.mm : -RF_INF;
    r.is = in ? x.is : -RF_INF;
    r.ds = in ? x.ds : -RF_INF;
    r.ci = (x.fl & 4) ? x.ci : -RF_INF;
    r.cd = (x.fl & 8) ? x.cd : -RF_INF;
    return r;
}

// load_row without branches around its loads (the non-lean kernels): every
// load is issued at a clamped, valid index and the out-of-range values are
// selected afterwards, so each step issues the same loads on every path and
// hipcc's wait for them counts only the memory operations issued after them
// (a load in a branch makes the count path-dependent: vmcnt(0), i.e. a wait
// for every band store as well).  Same values as load_row.
__device__ __forceinline__ RowRec load_row_flat(const DPTask &T, bool rev, const uint8_t *sbase,
                                                const double *tb, int ii, bool codon)
{
    const bool in = ii >= 0 && ii <= T.n;
    const int ic = min(max(ii, 1), T.n);   // a valid read row for the base
    const int iz = min(max(ii, 0), T.n);
    // indices >= 0 for a padding task too (T = {}: n = 0; load_row_raw)
    const int ks = max(rev ? min(T.n - 1, T.n - iz) : iz - 1, 0);
    const int kd = rev ? T.n - iz : iz;
    const int sb = sbase[max(rev ? T.n - ic : ic - 1, 0)];
    const double mt = tb[ks], mm = tb[T.n + ks], is = tb[2 * (size_t)T.n + ks], ds = tb[3 * (size_t)T.n + kd];
    // codon tables (align.jl:87-98): t_cins has n - 2 entries, t_cdel n + 1;
    // a task without them reads the match table instead and discards it
    const double *t_cins = tb + 4 * (size_t)T.n + 1;
    const int ci_i = rev ? T.ncins - iz + 2 : iz - 3;
    const bool has_ci = codon && T.ncins > 0 && ii >= 3 && in;
    const bool has_cd = codon && T.ncdel > 0 && in;
    // one load each at a selected offset (no branch): a task without the
    // table reads its own match entry instead, never past its region
    const int64_t ci_off = T.ncins > 0 ? 4 * (int64_t)T.n + 1 + min(max(ci_i, 0), T.ncins - 1) : ks;
    const int64_t cd_off = T.ncdel > 0 ? 4 * (int64_t)T.n + 1 + T.ncins + kd : ks;
    const double ci = tb[ci_off], cd = tb[cd_off];
    (void)t_cins;
    RowRec r;
    r.sb = (in && ii >= 1) ? sb : 4;
    r.mt = in ? mt : -RF_INF;
    r.mm = in ? mm : -RF_INF;
    r.is = in ? is : -RF_INF;
    r.ds = in ? ds : -RF_INF;
    r.ci = has_ci ? ci : -RF_INF;
    r.cd = has_cd ? cd : -RF_INF;
    return r;
}

__device__ __forceinline__ int load_col(const DPTask &T, bool rev, const uint8_t *tbase, int jj)
{
    return (jj >= 1 && jj <= T.m) ? tbase[rev ? T.m - jj : jj - 1] : 4;
}
// load_col with its load issued unconditionally (load_row_flat)
__device__ __forceinline__ int load_col_flat(const DPTask &T, bool rev, const uint8_t *tbase, int jj)
{
    const int jc = min(max(jj, 1), max(T.m, 1));
    const int b = tbase[rev ? max(T.m - jc, 0) : jc - 1];
    return (jj >= 1 && jj <= T.m) ? b : 4;
}

// Row record of the lane above (row_shl:1 / wave_shl:1); lane LPT-1 receives `edge`.
template <int LPT = 16>
__device__ __forceinline__ RowRec row_from_above(const RowRec &x, const RowRec &edge, bool codon)
{
    constexpr int C = TaskLanes<LPT>::FROM_R1;
    RowRec r;
    r.sb = __builtin_amdgcn_update_dpp(edge.sb, x.sb, C, 0xF, 0xF, false);
    auto sh = [](double v, double e) {
        constexpr int C = TaskLanes<LPT>::FROM_R1;
        const long long b = __double_as_longlong(v), eb = __double_as_longlong(e);
        const int lo = __builtin_amdgcn_update_dpp((int)eb, (int)b, C, 0xF, 0xF, false);
        const int hi = __builtin_amdgcn_update_dpp((int)(eb >> 32), (int)(b >> 32), C, 0xF, 0xF, false);
        return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
    };
    r.mt = sh(x.mt, edge.mt);
    r.mm = sh(x.mm, edge.mm);
    r.is = sh(x.is, edge.is);
    r.ds = sh(x.ds, edge.ds);
    if (TaskLanes<LPT>::EDGE_FIX && (threadIdx.x & (LPT - 1)) == LPT - 1) {
        r.sb = edge.sb;
        r.mt = edge.mt;
        r.mm = edge.mm;
        r.is = edge.is;
        r.ds = edge.ds;
    }
    if (codon) {
        r.ci = sh(x.ci, edge.ci);
        r.cd = sh(x.cd, edge.cd);
    } else {
        r.ci = r.cd = -RF_INF;
    }
    return r;
}

// ---------------------------------------------------------------------
// k_dpr: register-resident, systolic variant of k_dp for H <= 32*NP.
//
// Same recurrence and cell values as k_dp.  Each task owns one 16-lane DPP
// row (4 tasks per wave); lane q holds band-row pairs q*NP .. q*NP+NP-1.
// With pp = q*NP + r the cell of pair pp at anti-diagonal kappa is
//   row ii = pp + ceil(kappa/2) - c,   column jj = floor(kappa/2) - pp,
// so at odd steps every pair moves down one read row and at even steps one
// template column.  The anti-diagonals kappa-1..kappa-3, the per-row score
// tables and the template base all move systolically through registers: a
// pair takes the row record of the pair above it and the column base of the
// pair before it (DPP row_shl / row_shr); the DPP "old" operand hands lane 15
// its prefetched row and lane 0 its new column.  Out-of-row DPP sources read
// -Inf, i.e. an out-of-band predecessor, exactly like the ring's sentinels.
// The loop is unrolled over (even, odd) anti-diagonals so the parity is
// static.  The cell value of the reference's strict-'>' candidate chain
// (align.jl:43, :77-104) is the maximum of the candidates, and FP64 max of
// the same sums is exact (no NaN, no signed zero among candidates), so
// fmax yields bit-identical cells; the move is recomputed in k_bt_win
// with the strict order.
// ---------------------------------------------------------------------

// FLAT (the non-lean kernels): no branch around a store -- a cell outside
// the band goes to the sink -- the final cell's score is kept in a register
// (`fval` / `fset`, stored once after the loop) and the error flag is
// collected in `eflag` and raised once after the loop, so every step issues
// the same memory operations on every path (load_row_flat).
template <int NP, int PAR, int LPT = 16, bool FLAT = false>
__device__ __forceinline__ void dpr_step(const DPTask &T, int q, int k, bool codon, bool rev,
                                         bool skew, bool trim, double (&v1)[NP], double (&v2)[NP],
                                         double (&v3)[NP], const RowRec (&row)[NP],
                                         const int (&col)[NP], double *__restrict__ band,
                                         double *__restrict__ out_score, int *__restrict__ err,
                                         double *__restrict__ sink = nullptr, int *eflag = nullptr,
                                         double *fval = nullptr, int *fset = nullptr)
{
    // block-edge neighbours at kappa-1 (every lane shifts: uniform control flow)
    double E1;
    if (PAR == 0)
        E1 = dpp_f64<TaskLanes<LPT>::FROM_L1>(v1[NP - 1]);   // (d-1) of pair 0 = lane q-1's last pair
    else
        E1 = dpp_f64<TaskLanes<LPT>::FROM_R1>(v1[0]);        // (d+1) of the last pair = lane q+1's pair 0
    double L3a = -RF_INF, L3b = -RF_INF, R3a = -RF_INF, R3b = -RF_INF;
    // (32- and 64-lane tasks are lean: no codon moves; few long non-lean
    // tasks run in k_dpx, the rest as 16-lane tasks here)
    if (LPT == 16 && codon) {
        if (NP == 1) {
            L3a = dpp_f64<DPP_FROM_L1>(v3[0]);
            L3b = dpp_f64<DPP_FROM_L2>(v3[0]);
            R3a = dpp_f64<DPP_FROM_R1>(v3[0]);
            R3b = dpp_f64<DPP_FROM_R2>(v3[0]);
        } else {
            L3a = dpp_f64<DPP_FROM_L1>(v3[NP - 1]);
            L3b = dpp_f64<DPP_FROM_L1>(v3[NP > 1 ? NP - 2 : 0]);
            R3a = dpp_f64<DPP_FROM_R1>(v3[0]);
            R3b = dpp_f64<DPP_FROM_R1>(v3[NP > 1 ? 1 : 0]);
        }
    }
    const bool live = k < T.klen;
    double *orow = band + (size_t)(rev ? T.klen - 1 - k : k) * T.P;
    double nv[NP];
#pragma unroll
    for (int r = 0; r < NP; ++r) {
        const int d = 2 * (q * NP + r) + PAR;
        const int jj = (k - d) >> 1;
        const int ii = d + jj - T.c;
        const bool stored = live && d < T.H && d <= k;
        const bool valid = stored && jj <= T.m && ii >= 0 && ii <= T.n;
        const RowRec &R = row[r];
        const int tbb = col[r];
        double ms = (R.sb == tbb) ? R.mt : R.mm;
        double is = R.is;
        if (skew && R.sb != tbb)
            ms *= 0.99;
        if (trim && (jj == 0 || jj == T.m))
            is = 0.0;
        // insert (d-1, kappa-1) and delete (d+1, kappa-1)
        const double x_ins = PAR ? v1[r] : (r > 0 ? v1[r > 0 ? r - 1 : 0] : E1);
        const double x_del = PAR ? (r < NP - 1 ? v1[r < NP - 1 ? r + 1 : 0] : E1) : v1[r];
        double best = fmax(fmax(v2[r] + ms, x_ins + is), x_del + R.ds);
        if (codon) {
            if (ii >= 3) {   // codon insert: d-3 at kappa-3 = pair q*NP + r - 2 + PAR
                const int idx = r - 2 + PAR;
                const double y = idx >= 0 ? v3[idx >= 0 ? idx : 0] : (idx == -1 ? L3a : L3b);
                best = fmax(best, y + R.ci);
            }
            if (jj >= 3) {   // codon delete: d+3 at kappa-3 = pair q*NP + r + 1 + PAR
                const int idx = r + 1 + PAR;
                const double y = idx < NP ? v3[idx < NP ? idx : 0] : (idx == NP ? R3a : R3b);
                best = fmax(best, y + R.cd);
            }
        }
        const bool origin = ii == 0 && jj == 0;
        const double v = valid ? (origin ? 0.0 : best) : -RF_INF;
        if (FLAT) {
            *eflag |= (valid && !origin && best == -RF_INF) ? 1 : 0;   // "new score is invalid"
            const bool fin = valid && ii == T.n && jj == T.m;
            *fval = fin ? v : *fval;
            *fset |= fin ? 1 : 0;
            *(stored ? orow + ((rev ? T.H - 1 - d : d) >> 1) : sink + 2 * q) = v;
        } else {
            if (valid && !origin && best == -RF_INF)
                set_err(err, 1);  // "new score is invalid"
            if (valid && ii == T.n && jj == T.m && out_score)
                out_score[T.out_idx] = v;
            if (stored)
                orow[(rev ? T.H - 1 - d : d) >> 1] = v;
        }
        nv[r] = v;
    }
#pragma unroll
    for (int r = 0; r < NP; ++r) {
        v3[r] = v2[r];
        v2[r] = v1[r];
        v1[r] = nv[r];
    }
}

// Whole-row DPP rotate of an f64 (no "old" operand: every lane has a source).
template <int CTRL>
__device__ __forceinline__ double dpp_rot_f64(double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
#define DPP_ROT_L1 0x121   // row_ror:1  -> lane (q-1) mod 16
#define DPP_ROT_R1 0x12F   // row_ror:15 -> lane (q+1) mod 16

// One anti-diagonal of the lean interior (LEAN kernels, kappa in [klo, khi]):
// no codon / skew / trim, and every cell of an active diagonal is inside the
// matrix, so the per-cell range checks, the origin and A[end,end] cases of
// dpr_step drop out.  Inactive diagonals (d >= H, or no cell in the matrix)
// get lb = -Inf, which keeps them at -Inf exactly like dpr_step's masking
// (x + 0.0 == x for every cell value: no cell is -0.0).  The block-edge
// neighbour comes from a row *rotate*: the lane it wraps from holds diagonal
// 32*NP-1 >= H (host guarantees H <= 32*NP-1), i.e. -Inf.  Lean tasks have
// finite match/mismatch/ins/del tables, so every in-band cell is finite (each
// has an in-band predecessor chain to the origin) and the "new score is
// invalid" check (align.jl:105-107) cannot fire here; the general steps keep it.
// (An XOR swizzle of the lean blocks' LDS band rows, removing the 4-way bank
// conflicts of the NP = 8 cell stores, was bit-exact but slower at c5:
// 30.2 -> 32.0 ms DP-only, profiles/r02_exp_dp_swz.json.)
template <int NP>
__device__ __forceinline__ dvec2 dpl_rd2(const double *R, int u)   // u even
{
    return *(const dvec2 *)(R + u);
}

template <int NP, int PAR, int LPT = 16>
__device__ __forceinline__ void dpl_step(double (&v1)[NP], double (&v2)[NP], const RowRec (&row)[NP],
                                         const int (&col)[NP], const double (&lb)[NP],
                                         const bool (&st)[NP], double *Rb, int u0, int ostep)
{
    const double E1 = PAR == 0 ? dpp_rot_f64<TaskLanes<LPT>::ROT_L1>(v1[NP - 1])
                               : dpp_rot_f64<TaskLanes<LPT>::ROT_R1>(v1[0]);
    double nv[NP];
#pragma unroll
    for (int r = 0; r < NP; ++r) {
        const RowRec &R = row[r];
        const double ms = (R.sb == col[r]) ? R.mt : R.mm;
        const double x_ins = PAR ? v1[r] : (r > 0 ? v1[r > 0 ? r - 1 : 0] : E1);
        const double x_del = PAR ? (r < NP - 1 ? v1[r < NP - 1 ? r + 1 : 0] : E1) : v1[r];
        // (round 3: the mask on the insert / delete inputs instead of the cell,
        // and the exchanged value entering the max last, were no faster)
        nv[r] = fmax(fmax(v2[r] + ms, x_ins + R.is), x_del + R.ds) + lb[r];
        if (st[r])
            Rb[u0 + r * ostep] = nv[r];
    }
#pragma unroll
    for (int r = 0; r < NP; ++r) {
        v2[r] = v1[r];
        v1[r] = nv[r];
    }
}

// Blocked lean interior: per task an LDS slice of DPL_B edge records (the
// row entering lane 15 and the column entering lane 0 per period) and
// 2*DPL_B kappa rows of band output, flushed as one contiguous chunk.
#ifndef DPL_BLOCK
#define DPL_BLOCK 16
#endif
// periods per block (<= 16: one edge record per lane); NP = 2, 4 take 8 and NP = 8
// takes 4 (measured: NP = 2/4 at 16 need 280/430 VGPRs -> one wave per SIMD), so
// that a 4-task workgroup's LDS slices (rows of up to 129 doubles) leave
// several waves per CU
#ifndef DPL_B64
#define DPL_B64 8   // periods per block of the 64-lane tasks
#endif
__host__ __device__ constexpr int dpl_b(int np, int lpt = 16)
{
    return lpt >= 32 ? DPL_B64 : (np >= 8 ? 4 : (np >= 2 ? 8 : DPL_BLOCK));
}
#ifndef DPL_SPREAD
#define DPL_SPREAD 1   // NP = 1 lean flush spread over the next block's periods
#endif
#define DPL_SPREAD_ON(np, lpt) (DPL_SPREAD && (np) == 1 && (lpt) == 16)
#ifndef DPR_WPE1
#define DPR_WPE1 1   // minimum waves per SIMD requested for the NP = 1 kernels
#endif
struct alignas(16) EdgeRec {
    double mt, mm, is, ds;
    int sb, col, pad0, pad1;
};
__host__ __device__ constexpr int dpl_pmax(int np, int lpt = 16) { return (lpt * np) | 1; }   // band_P(2*LPT*NP-1)
// carry slots on either side of a task's band-output rows: a flush writes
// whole 128-B lines only and carries the partial line into the next block
constexpr int DPL_CARRY = 16;
__host__ __device__ constexpr int dpl_task_bytes(int np, int pm, int lpt = 16)
{
    return (int)(dpl_b(np, lpt) * sizeof(EdgeRec)) + (2 * dpl_b(np, lpt) * pm + 2 * DPL_CARRY + 8) * 8;
}
__host__ __device__ constexpr int dpl_task_bytes(int np) { return dpl_task_bytes(np, dpl_pmax(np)); }
// 16-B stores per lane of one flush: at most 2*DPL_B*P + DPL_CARRY doubles
__host__ __device__ constexpr int dpl_flush_stores(int np, int pm, int lpt = 16)
{
    return (dpl_b(np, lpt) * pm + DPL_CARRY / 2 + lpt - 1) / lpt;
}
// stride classes of the lean DP launches: k_dpr<1 << npi, true, dpr_pm(npi, pmi)>
// takes the lean tasks of NP class npi with P <= dpr_pm (the largest is the
// class maximum 16 * NP | 1)
__host__ __device__ constexpr int dpr_pm(int npi, int pmi)
{
    // NP = 1: P <= 17 (H <= 31); NP = 2: 17..33; NP = 4: 33..65; NP = 8: 65..129
    return npi == 0 ? 11 + 2 * pmi : npi == 1 ? 19 + 4 * pmi + (pmi == 3 ? 2 : 0) : (((16 << npi) * (pmi + 5)) / 8) | 1;
}
extern __shared__ __attribute__((aligned(16))) char dpl_smem[];

// PM: the largest band row stride P of the launch's tasks (default: the
// class maximum).  The lean flush issues a fixed dpl_flush_stores(NP, PM)
// 16-B stores per lane (a static count, so hipcc's wait for the next edge
// load is vmcnt(FL) rather than vmcnt(0)); lanes past a block's end repeat
// its last pair.  For NP = 1 the host splits the lean class by P (11, 13,
// 15, 17), so a c4 task with P = 11 issues 12 stores per lane per block
// instead of 18.
#ifndef DPR_WPE64
#define DPR_WPE64 2   // minimum waves per SIMD requested for the 64-lane kernels
#endif
// PFIX: every task of the launch has row stride exactly PM (the host routes
// only such tasks to it), so the blocked interior's LDS offsets i * P are
// compile-time immediates instead of one address register per step.
#ifndef DPR_PFIX
#define DPR_PFIX 1
#endif
template <int NP, bool LEAN, int PM, int LPT, bool PFIX>
__device__ __forceinline__ void dpr_body(const int blk, const DPTask *__restrict__ tasks, int ntasks,
                                         const uint8_t *__restrict__ bases, const double *__restrict__ tabs,
                                         double *__restrict__ bands, double *__restrict__ out_score,
                                         int *__restrict__ err, double *__restrict__ sink,
                                         const double *__restrict__ lut)
{
    constexpr int DPL_B = dpl_b(NP, LPT);
    const int q = threadIdx.x & (LPT - 1);
    const int tid = blk * (64 / LPT) + threadIdx.x / LPT;
    DPTask T = {};
    if (tid < ntasks)
        T = tasks[tid];
    int kmax = T.klen;
    for (int off = 32; off >= 1; off >>= 1)
        kmax = max(kmax, __shfl_xor(kmax, off));
    kmax = __builtin_amdgcn_readfirstlane(kmax);
    const bool codon = LEAN ? false : __any(T.ncins > 0 || T.ncdel > 0);   // wave-uniform
    const bool rev = T.flags & 1;
    const bool skew = LEAN ? false : (T.flags & 2);
    const bool trim = LEAN ? false : (T.flags & 4);
    const uint8_t *sbase = bases + T.sb;
    const uint8_t *tbase = bases + T.tb;
    const double *tb = tabs + T.tab;
    double *band = bands + T.band;

    double v1[NP], v2[NP], v3[NP];
    RowRec row[NP];
    int col[NP];
#pragma unroll
    for (int r = 0; r < NP; ++r) {
        v1[r] = -RF_INF;
        v2[r] = -RF_INF;
        v3[r] = -RF_INF;
        const int pp = q * NP + r;
        row[r] = load_row(T, rev, sbase, tb, pp - T.c, codon);   // kappa = 0
        col[r] = load_col(T, rev, tbase, -pp);
    }
    const int top = LPT * NP - 1;
    // general steps of the non-lean kernels: branch-free loads and stores
    // (load_row_flat, dpr_step<FLAT>), so hipcc waits for a prefetched
    // load without draining the band stores issued after it
    constexpr bool FLAT = !LEAN;
    auto lrow = [&](int ii, bool cod) {
        return FLAT ? load_row_flat(T, rev, sbase, tb, ii, cod) : load_row(T, rev, sbase, tb, ii, cod);
    };
    auto lcol = [&](int jj) { return FLAT ? load_col_flat(T, rev, tbase, jj) : load_col(T, rev, tbase, jj); };
    int eflag = 0;
    double fval = 0.0;   // FLAT: the final cell's score (the lane that computes it)
    int fset = 0;
    double *gsink = sink + 64 * (threadIdx.x >> 4);   // 32 doubles per 16-lane row of the wave
    if (FLAT) {
        // Non-lean kernels (codon moves, skew / trim, non-finite tables; e.g. the
        // reference's codon DP, often a single long task per launch, whose
        // period is shorter than a load's latency): the edge row entering lane
        // 15 at odd steps and the column base entering lane 0 at even steps are
        // loaded QD periods ahead into QD static slots (the loop is unrolled
        // over QD periods, so no slot is moved between registers), and their
        // selects run at use; stores and loads are branch-free (dpr_step<FLAT>),
        // so every wait counts only the operations issued after its load.
        constexpr int QD = 4;
        RawRow nq[QD];
        int cq[QD];
        bool cv[QD];
#pragma unroll
        for (int j = 0; j < QD; ++j) {
            nq[j] = load_row_raw(T, rev, sbase, tb, top + 1 + j - T.c, codon);   // period j's edge row
            const int jj = 1 + j;                                                // column of period 1 + j
            cq[j] = tbase[rev ? max(T.m - min(max(jj, 1), max(T.m, 1)), 0) : min(max(jj, 1), max(T.m, 1)) - 1];
            cv[j] = jj >= 1 && jj <= T.m;
        }
        for (int k0 = 0; k0 < kmax; k0 += 2 * QD) {
#pragma unroll
            for (int j = 0; j < QD; ++j) {
                const int k = k0 + 2 * j;
                if (k >= kmax)
                    break;
                if (k > 0) {
                    // even step: lane 0 receives column k/2, from slot (k/2 - 1) mod QD
                    const int cs = (j + QD - 1) % QD;   // static after unrolling
                    const int edge = cv[cs] ? cq[cs] : 4;
                    const int jn = k / 2 + QD;
                    const int jc = min(max(jn, 1), max(T.m, 1));
                    cq[cs] = tbase[rev ? max(T.m - jc, 0) : jc - 1];
                    cv[cs] = jn >= 1 && jn <= T.m;
                    int from = __builtin_amdgcn_update_dpp(edge, col[NP - 1], TaskLanes<LPT>::FROM_L1, 0xF, 0xF,
                                                           false);
                    if (TaskLanes<LPT>::EDGE_FIX && q == 0)
                        from = edge;
#pragma unroll
                    for (int r = NP - 1; r > 0; --r)
                        col[r] = col[r - 1];
                    col[0] = from;
                }
                dpr_step<NP, 0, LPT, true>(T, q, k, codon, rev, skew, trim, v1, v2, v3, row, col, band, out_score,
                                           err, gsink, &eflag, &fval, &fset);
                if (k + 1 < kmax) {
                    // odd step: rows advance; lane 15 receives period k/2's row (slot j)
                    const RowRec up = row_from_above<LPT>(row[0], row_val(nq[j]), codon);
#pragma unroll
                    for (int r = 0; r < NP - 1; ++r)
                        row[r] = row[r + 1];
                    row[NP - 1] = up;
                    nq[j] = load_row_raw(T, rev, sbase, tb, top + k / 2 + 1 + QD - T.c, codon);
                    dpr_step<NP, 1, LPT, true>(T, q, k + 1, codon, rev, skew, trim, v1, v2, v3, row, col, band,
                                               out_score, err, gsink, &eflag, &fval, &fset);
                }
            }
        }
        if (eflag)
            set_err(err, 1);  // "new score is invalid"
        if (fset && out_score)
            out_score[T.out_idx] = fval;
        return;
    }
    // lean kernels: the edge row / column of the next period (one ahead)
    constexpr int QD = 1;
    RowRec nq[QD];
    int cq[QD];
    nq[0] = lrow(top + 1 - T.c, codon);   // enters at kappa = 1
    cq[0] = lcol(1);                      // enters at kappa = 2

    // Lean interior [klo, khi]: the kappa range in which every cell of every
    // active diagonal of the wave's four tasks is inside the matrix, minus the
    // origin and the final cell.  Diagonal d holds cells jj in
    // [max(0, c-d), min(m, n+c-d)], i.e. kappa in [d + 2 jlo, d + 2 jhi].
    int klo = INT_MAX, khi = -1;
    double lb[2][NP];
    bool st[2][NP];
    if (LEAN) {
        int lo = 0, hi = INT_MAX;
        bool ok = true;
#pragma unroll
        for (int par = 0; par < 2; ++par)
#pragma unroll
            for (int r = 0; r < NP; ++r) {
                const int d = 2 * (q * NP + r) + par;
                const int jlo = max(0, T.c - d), jhi = min(T.m, T.n + T.c - d);
                const bool a = tid < ntasks && d < T.H && jlo <= jhi;
                st[par][r] = tid < ntasks && d < T.H;
                lb[par][r] = a ? 0.0 : -RF_INF;
                if (a) {
                    lo = max(lo, d + 2 * jlo);
                    hi = min(hi, d + 2 * jhi);
                }
            }
        if (tid < ntasks) {
            lo = max(lo, T.c + 1);
            hi = min(hi, T.klen - 2);
            ok = T.c <= T.m;   // diagonal 0 holds cells: edge rows stay >= 1
        }
        for (int off = 32; off >= 1; off >>= 1) {
            lo = max(lo, __shfl_xor(lo, off));
            hi = min(hi, __shfl_xor(hi, off));
        }
        if (__all(ok)) {
            klo = __builtin_amdgcn_readfirstlane((lo + 1) & ~1);   // wave-uniform: scalar loop
            khi = __builtin_amdgcn_readfirstlane(hi);
        }
    }
    // whole blocks of the interior; the remainder runs as general steps
    const int nblk = (LEAN && khi >= klo) ? (khi - klo + 1) / (2 * DPL_B) : 0;

    for (int k = 0; k < kmax; k += 2) {
        if (LEAN && k == klo && nblk > 0) {
            // ---- blocked lean interior: DPL_B periods (2*DPL_B anti-diagonals)
            // per block, inputs and outputs staged in this task's LDS slice
            const int P = PFIX ? PM : T.P;
            const int t = threadIdx.x / LPT;
            EdgeRec *ein = reinterpret_cast<EdgeRec *>(dpl_smem + t * dpl_task_bytes(NP, PM, LPT));
            // line-aligned flushes: `fl` is the band position (doubles from the
            // band start, which is 256-B aligned) up to which (forward) or down
            // from which (reverse) the interior has been written.  A block's
            // first position g0 is even forward (even kappa x any P) but can be
            // odd in reverse (odd H): `ob` is shifted by g0's parity so that LDS
            // and global 16-B pairs line up.
            const int blk = 2 * DPL_B * P;
            const ptrdiff_t g00 = (ptrdiff_t)(rev ? T.klen - 2 * DPL_B - k : k) * P;
            ptrdiff_t fl = g00 + (rev ? blk : 0);
            // rows region R; slot u of R holds the band value at position
            // g0 + (u - ub) of the block
            double *R = reinterpret_cast<double *>(dpl_smem + t * dpl_task_bytes(NP, PM, LPT) + DPL_B * sizeof(EdgeRec));
            const int ub = DPL_CARRY + (int)(g00 & 1);
            // this lane's LDS slot per parity; a block's 2*DPL_B rows are the
            // contiguous global chunk (reverse: flipped rows)
            const int sl0 = rev ? (T.H - 1 - 2 * q * NP) >> 1 : q * NP;
            const int sl1 = rev ? (T.H - 2 - 2 * q * NP) >> 1 : q * NP;
            const int ostep = rev ? -1 : 1;
            const int top_c = LPT * NP - T.c;
            // Edge records.  A task whose read has row codes (DPTask flag
            // RF_TASK_CODED) reads one 8-B code record per row from HBM and the
            // table values from the context's code dictionary (L2-resident),
            // instead of 4 table doubles per row; the values are the same
            // doubles.  The code record of a block is loaded one block before
            // its dictionary entries, so neither load's wait covers the
            // block's own band stores.
            const bool coded = T.flags & RF_TASK_CODED;
            const uint64_t *codes = (const uint64_t *)(tb + row_code_off(T.n, T.ncins, T.ncdel));
            auto edge_ks = [&](int kb) {   // lane q < DPL_B: the period kb + 2q edge row (clamped: see dpl_step)
                const int kk = kb + 2 * min(q, DPL_B - 1);
                const int ii = max(1, min(top_c + (kk >> 1), T.n));
                return rev ? T.n - ii : ii - 1;
            };
            auto code_load = [&](int kb) -> uint64_t { return coded ? codes[edge_ks(kb)] : 0; };
            auto edge_load = [&](int kb, uint64_t rec) {
                EdgeRec e;
                const int kk = kb + 2 * min(q, DPL_B - 1);
                const int ks = edge_ks(kb);
                const int kd = rev ? ks : ks + 1;
                if (coded) {
                    const double *l3 = lut + 4 * (int)(rec & 0xffff);
                    const dvec2 mt_mm = *(const dvec2 *)l3;
                    e.mt = mt_mm.x;
                    e.mm = mt_mm.y;
                    e.is = l3[2];
                    e.ds = lut[4 * RF_CODES + (int)((rec >> (rev ? 16 : 32)) & 0xffff)];
                    e.sb = (int)(rec >> 48) & 0xff;
                } else {
                    e.sb = sbase[ks];
                    e.mt = tb[ks];
                    e.mm = tb[T.n + ks];
                    e.is = tb[2 * (size_t)T.n + ks];
                    e.ds = tb[3 * (size_t)T.n + kd];
                }
                const int jj = max(1, min(kk >> 1, T.m));
                e.col = tbase[rev ? T.m - jj : jj - 1];
                return e;
            };
            EdgeRec pend = edge_load(k, code_load(k));
            if (q < DPL_B)
                ein[q] = pend;
            pend = edge_load(k + 2 * DPL_B, code_load(k + 2 * DPL_B));
            uint64_t pcode = code_load(k + 4 * DPL_B);
            // spread flush (NP = 1): a block's flush stores are read from LDS
            // into registers at the block end and issued one per period during
            // the next block, so the store stream stays steady instead of one
            // burst per block that stalls the issuing wave behind the memory
            // pipeline.  Before the first block the pending set is the sink.
            constexpr int FL = dpl_flush_stores(NP, PM, LPT);
            constexpr int FLS = DPL_SPREAD_ON(NP, LPT) ? FL : 1;
            dvec2 pv[FLS];
            dvec2 *pg = (dvec2 *)sink;
            int pnu = 0;
            bool preal = false;
#pragma unroll
            for (int j = 0; j < FLS; ++j)
                pv[j] = dvec2{0.0, 0.0};
            if (!DPL_SPREAD_ON(NP, LPT)) {
                // as many stores behind this load as the loop puts behind its
                // own (to the sink), so that hipcc's wait for `pend` is vmcnt(FL)
                // on every path into the loop, not vmcnt(0)
                dvec2 *g = (dvec2 *)sink;
                const dvec2 z = {0.0, 0.0};
#pragma unroll
                for (int j = 0; j < FL; ++j)
                    g[q + LPT * j] = z;
            }
            wave_sync();
            for (int b = 0; b < nblk; ++b) {
                // edge records are LDS broadcasts read one period ahead: a read
                // issued right before its use exposes the full LDS latency on
                // every step (the DP chain has nothing else to issue meanwhile)
                EdgeRec E = ein[0];
#pragma unroll
                for (int p = 0; p < DPL_B; ++p) {
                    EdgeRec En;
                    if (p + 1 < DPL_B)
                        En = ein[p + 1];
                    if (DPL_SPREAD_ON(NP, LPT)) {
#pragma unroll
                        for (int j = p; j < FLS; j += DPL_B) {
                            const int e = preal ? min(q + LPT * j, pnu - 1) : q + LPT * j;
                            DP_STORE(pg + e, pv[j]);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    {   // even step: column k/2 enters lane 0
                        int from = __builtin_amdgcn_update_dpp(E.col, col[NP - 1], TaskLanes<LPT>::FROM_L1, 0xF, 0xF, false);
                        if (TaskLanes<LPT>::EDGE_FIX && q == 0)
                            from = E.col;
#pragma unroll
                        for (int r = NP - 1; r > 0; --r)
                            col[r] = col[r - 1];
                        col[0] = from;
                    }
                    const int i0 = rev ? 2 * DPL_B - 1 - 2 * p : 2 * p;
                    dpl_step<NP, 0, LPT>(v1, v2, row, col, lb[0], st[0], R, ub + i0 * P + sl0, ostep);
                    {   // odd step: rows advance; lane 15 receives the edge row
                        RowRec e;
                        e.sb = E.sb;
                        e.mt = E.mt;
                        e.mm = E.mm;
                        e.is = E.is;
                        e.ds = E.ds;
                        const RowRec up = row_from_above<LPT>(row[0], e, false);
#pragma unroll
                        for (int r = 0; r < NP - 1; ++r)
                            row[r] = row[r + 1];
                        row[NP - 1] = up;
                    }
                    const int i1 = rev ? 2 * DPL_B - 2 - 2 * p : 2 * p + 1;
                    dpl_step<NP, 1, LPT>(v1, v2, row, col, lb[1], st[1], R, ub + i1 * P + sl1, ostep);
                    if (p + 1 < DPL_B)
                        E = En;
                }
                wave_sync();
                // next block's edges (loaded one block ago) -> LDS (harmless past
                // the last block: ein is not read again)
                if (q < DPL_B)
                    ein[q] = pend;
                // the block after next: issued BEFORE this block's stores.  vmcnt
                // is one in-order counter for loads and stores, so a load issued
                // after the stores could only be waited for by draining them
                // (clamped rows: past the interior it reads valid, unused rows)
                pend = edge_load(k + 4 * DPL_B, pcode);
                pcode = code_load(k + 6 * DPL_B);
                // flush: the block's 2*DPL_B kappa rows are one contiguous run of the
                // band [g0, g0 + blk).  Only whole 128-B lines are written (a partial
                // line would leave L2 as a partial HBM write): the part past the last
                // full line is carried into the next block (LDS slots before /
                // after `ob`); the last block writes everything.  A fixed number of
                // 16-B stores per lane (lanes past the end repeat the last pair;
                // tasks past ntasks write the sink) keeps hipcc's wait for the next
                // edge load at vmcnt(FL) instead of draining these stores.
                {
                    const ptrdiff_t g0 = (ptrdiff_t)(rev ? T.klen - 2 * DPL_B - k : k) * P;
                    const bool last = b + 1 == nblk;
                    ptrdiff_t lo, hi;
                    if (!rev) {
                        lo = fl;
                        hi = last ? g0 + blk : ((g0 + blk) & ~(ptrdiff_t)15);
                        fl = hi;
                    } else {
                        hi = fl;
                        lo = last ? g0 : ((g0 + 15) & ~(ptrdiff_t)15);
                        fl = lo;
                    }
                    // whole 16-B pairs [lo2, hi2); an odd end (reverse, odd g0: only
                    // the first and last blocks) is one 8-B store
                    const ptrdiff_t lo2 = (lo + 1) & ~(ptrdiff_t)1, hi2 = hi & ~(ptrdiff_t)1;
                    const int nu = (int)((hi2 - lo2) >> 1);
                    // padding tasks (T = {}: nu = 0) write slots [0, 16*FL) of
                    // the sink -- never index -1
                    const bool task_real = tid < ntasks;
                    const bool real = task_real && nu > 0;
                    dvec2 *g = real ? (dvec2 *)(band + lo2) : (dvec2 *)sink;
                    const int u2 = ub + (int)(lo2 - g0);   // even
                    if (DPL_SPREAD_ON(NP, LPT)) {
#pragma unroll
                        for (int j = 0; j < FLS; ++j)
                            pv[j] = dpl_rd2<NP>(R, u2 + 2 * (real ? min(q + LPT * j, nu - 1) : 0));
                        pg = g;
                        pnu = nu;
                        preal = real;
                        if (last) {   // nothing follows: write the last block now
#pragma unroll
                            for (int j = 0; j < FLS; ++j) {
                                const int e = real ? min(q + LPT * j, nu - 1) : q + LPT * j;
                                DP_STORE(g + e, pv[j]);
                            }
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < FL; ++j) {
                            const int e = real ? min(q + LPT * j, nu - 1) : q + LPT * j;
                            DP_STORE(g + e, dpl_rd2<NP>(R, u2 + 2 * (real ? e : 0)));
                        }
                    }
                    if (task_real && q == 0 && (lo & 1))
                        band[lo] = R[ub + (int)(lo - g0)];
                    if (task_real && q == 1 && (hi & 1))
                        band[hi - 1] = R[ub + (int)(hi - 1 - g0)];
                    // carry the unwritten partial line (fewer than 16 doubles: one
                    // pass of the task's lanes) next to the next block's rows
                    if (!rev) {
                        const int c = (int)(g0 + blk - fl), src = (int)(fl - g0);
                        if (q < c)
                            R[ub + src - blk + q] = R[ub + src + q];
                    } else {
                        const int c = (int)(fl - g0);
                        if (q < c)
                            R[ub + blk + q] = R[ub + q];
                    }
                }
                wave_sync();
                k += 2 * DPL_B;
            }
            // back to the general steps: the edge row and column they expect
            // (lean kernels only, QD = 1)
            nq[0] = lrow(top + k / 2 + 1 - T.c, false);
            cq[0] = lcol(k / 2);
            if (k >= kmax)
                break;
        }
        if (k > 0) {
            // even step: columns advance; lane 0 receives column k/2
            const int edge = cq[0];
#pragma unroll
            for (int j = 0; j + 1 < QD; ++j)
                cq[j] = cq[j + 1];
            cq[QD - 1] = lcol(k / 2 + QD);
            int from = __builtin_amdgcn_update_dpp(edge, col[NP - 1], TaskLanes<LPT>::FROM_L1, 0xF, 0xF, false);
            if (TaskLanes<LPT>::EDGE_FIX && q == 0)
                from = edge;
#pragma unroll
            for (int r = NP - 1; r > 0; --r)
                col[r] = col[r - 1];
            col[0] = from;
        }
        dpr_step<NP, 0, LPT, FLAT>(T, q, k, codon, rev, skew, trim, v1, v2, v3, row, col, band, out_score, err,
                                   gsink, &eflag, &fval, &fset);
        if (k + 1 < kmax) {
            // odd step: rows advance; lane 15 receives the prefetched row
            const RowRec up = row_from_above<LPT>(row[0], nq[0], codon);
#pragma unroll
            for (int r = 0; r < NP - 1; ++r)
                row[r] = row[r + 1];
            row[NP - 1] = up;
#pragma unroll
            for (int j = 0; j + 1 < QD; ++j)
                nq[j] = nq[j + 1];
            nq[QD - 1] = lrow(top + (k + 2) / 2 + QD - T.c, codon);
            dpr_step<NP, 1, LPT, FLAT>(T, q, k + 1, codon, rev, skew, trim, v1, v2, v3, row, col, band,
                                       out_score, err, gsink, &eflag, &fval, &fset);
        }
    }
    if (FLAT && eflag)
        set_err(err, 1);  // "new score is invalid"
}

template <int NP, bool LEAN, int PM = dpl_pmax(NP), int LPT = 16, bool PFIX = false>
__global__ void __launch_bounds__(64)
__attribute__((amdgpu_waves_per_eu(LPT >= 32 ? DPR_WPE64 : (NP == 1 ? DPR_WPE1 : 1))))
k_dpr(const DPTask *__restrict__ tasks, int ntasks, const uint8_t *__restrict__ bases,
      const double *__restrict__ tabs, double *__restrict__ bands,
      double *__restrict__ out_score, int *__restrict__ err, double *__restrict__ sink,
      const double *__restrict__ lut)
{
    dpr_body<NP, LEAN, PM, LPT, PFIX>(blockIdx.x, tasks, ntasks, bases, tabs, bands, out_score, err, sink, lut);
}

// ---------------------------------------------------------------------
// k_dpm: very wide bands without codon moves across several CUs (round 6;
// edit_distance's band, align.jl:253-260: bw = ceil(min(m, n) / 2), H ~ m,
// configs[2]: H = 2,624, one band per call).  Round 5 ran such a band in
// one 1024-thread workgroup (k_dpw: a barrier per anti-diagonal, issue-bound
// on one CU, 3.35 ms per call).  Here the band is cut into slices of DPM_OWN
// band-row pairs, one single-wave workgroup each (no barrier per step),
// which meet only every DPM_B anti-diagonals:
//   - the wave holds 64 * DPM_NPL consecutive pairs: its slice and DPM_B / 2
//     pairs (DPM_B diagonals) of each neighbouring slice.  After a hand-off
//     every pair holds exact values; in the next DPM_B steps a wrong value
//     enters at the wave's outer edges (their outer neighbours are unknown)
//     and spreads inward one diagonal per step, so it never reaches the
//     slice before the next hand-off refreshes the halo pairs;
//   - the kappa-1 values of neighbouring diagonals move between lanes by DPP
//     (wave_shr / wave_shl), within a lane in registers;
//   - row records and template bases come from LDS rings, filled 64 rows /
//     columns at a time one chunk of 64 periods ahead; the rings carry a
//     mirrored tail, so a lane's ring index is its constant plus the
//     period's scalar one (no wrap per read);
//   - a cell is a fixed sequence of selects: its validity is a per-lane
//     range of periods, its store a buffer store whose offset is per-lane
//     (lanes outside the slice or the band get an offset past the band and
//     the range check drops the store); the origin, the final cell and a
//     last period without its odd step are separate (EDGE) periods;
//   - a wave computes only its compute phase, the periods at which some
//     pair it holds is in the DP; before and after, its cells are -Inf
//     stores (configs[2]: 2,602 of the band's 7,826 anti-diagonals);
//   - hand-off through the band itself: the host fills each band with an
//     all-ones pattern (a NaN no sum produces) before the launch; the slice
//     stores every in-band cell it owns (write-through, sc1) and a wave
//     takes its halo pairs' last two values where they are in the DP by
//     polling those cells (sc1 loads, 64-bit single-copy atomic) until none
//     holds the pattern -- one round trip, no flag and no store drain
//     (bounded: error 4 rather than a hang);
//   - a band's slices run on one XCD (workgroup i runs on XCD i % 8), the
//     bands of a launch spread over the eight.
// Same candidates, FP64 sums and strict-'>' values as k_dp: bit-identical;
// cells left of the DP (jj < 0) are stored as -Inf, which k_dp leaves out.
// ---------------------------------------------------------------------
// geometry (profiles/r06p_exp_dpm.out, configs[2]'s band, ms per call):
// 1 pair per lane, hand-off every 32 steps 0.745; every 16 0.822; 2 pairs
// per lane, every 32 1.064, every 64 0.984 (k_dpw: 3.35)
#ifndef DPM_NPL_
#define DPM_NPL_ 1
#endif
#ifndef DPM_B_
#define DPM_B_ 32
#endif
constexpr int DPM_NPL = DPM_NPL_;                 // pairs per lane
constexpr int DPM_B = DPM_B_;                     // anti-diagonals per hand-off
constexpr int DPM_OWN = 64 * DPM_NPL - DPM_B;     // pairs per slice
constexpr int DPM_RING = 512;                     // staged rows / columns (8 blocks of 64)
constexpr int DPM_RINGX = DPM_RING + 64 * DPM_NPL;   // + the mirrored tail
constexpr int DPM_SPIN = 1 << 22;                 // polls before error 4
constexpr unsigned DPM_NOSTORE = 0x80000000u;     // past every band (K * P * 8 < 2^31)
constexpr long long DPM_UNSET = -1;               // the fill pattern of a band not yet stored
constexpr int DPM_SC1 = 16;                       // buffer-store cache policy: sc1 (write-through)
static_assert(DPM_OWN > 0 && (DPM_B / 2) % DPM_NPL == 0 && 128 % DPM_B == 0, "slice geometry");

__host__ __device__ constexpr int dpm_slices(int H) { return ((H + 1) / 2 + DPM_OWN - 1) / DPM_OWN; }
// A band's slices spin on each other, so they must be resident together:
// at most DPM_TASK_SLICES per band (an XCD holds 8 of these 20-KB workgroups
// per CU, 32 CUs: 256).  Workgroups of one launch dispatch in order, so the
// bands of one XCD become resident one after another (each waits only for
// earlier bands, which are whole); wider bands take k_dp.  Launches from
// other streams (a second engine) interleave with it, so one launch keeps
// to DPM_XCD_SLICES per XCD (more bands: further launches on its stream).
constexpr int DPM_TASK_SLICES = 160;
constexpr int DPM_XCD_SLICES = 64;

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double ld_sc1(const double *p)
{
    return __longlong_as_double(
        (long long)__hip_atomic_load((unsigned long long *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <bool TRIM>
__global__ void __launch_bounds__(64)
k_dpm(const DPTask *__restrict__ tasks, int ntasks, int G, const uint8_t *__restrict__ bases,
      const double *__restrict__ tabs, double *__restrict__ bands, double *__restrict__ out_score,
      int *__restrict__ err)
{
    // workgroup i runs on XCD i % 8: task t takes XCD t % 8, its slice g
    // the workgroups 8 ((t / 8) G + g) + t % 8
    const int row = blockIdx.x >> 3, task = (row / G) * 8 + (blockIdx.x & 7), g = row % G;
    if (task >= ntasks)
        return;
    const DPTask T = tasks[task];
    const int npairs = (T.H + 1) >> 1;
    const int Gt = dpm_slices(T.H);
    if (g >= Gt)
        return;
    const int q = threadIdx.x;
    const bool rev = T.flags & 1, skew = T.flags & 2, trim = TRIM && (T.flags & 4);
    const uint8_t *sbase = bases + T.sb;
    const uint8_t *tbase = bases + T.tb;
    const double *tb = tabs + T.tab;
    double *band = bands + T.band;
    const int K = T.klen, H = T.H;
    const int own_lo = g * DPM_OWN, own_hi = min(own_lo + DPM_OWN, npairs);
    const int pb = own_lo - DPM_B / 2;           // the pair of lane 0, r = 0
    const __amdgpu_buffer_rsrc_t brs =
        __builtin_amdgcn_make_buffer_rsrc(band, 0, (int)((int64_t)K * T.P * 8), 0x00020000);
    __shared__ dvec2 s_rec[2 * DPM_RINGX];      // {mt, mm}, {is, ds} per read row
    __shared__ uint8_t s_sb[DPM_RINGX], s_col[DPM_RINGX];
    // pair pp = pb + x at period P reads read row x + P + par + rbase and
    // template column P + 64 DPM_NPL - 1 - x + cbase: ring entries
    // (x + P + par) and (P + 64 DPM_NPL - 1 - x), blocks of 64 entries
    const int rbase = pb - T.c, cbase = -(pb + 64 * DPM_NPL - 1);
    static_assert(64 * (DPM_NPL + 2) <= DPM_RING, "ring holds the chunk's blocks and the next");
    // a block's loads are held raw until it is put in LDS a chunk later (a
    // select right after them would make hipcc wait for them at once; k_dpx)
    struct Blk {
        RawRow r;
        int col;
        bool colok;
    };
    auto blk_load = [&](int b) {
        Blk x;
        x.r = load_row_raw(T, rev, sbase, tb, rbase + 64 * b + q, false);
        const int jj = cbase + 64 * b + q;
        const int jc = min(max(jj, 1), max(T.m, 1));
        x.col = tbase[rev ? max(T.m - jc, 0) : jc - 1];
        x.colok = jj >= 1 && jj <= T.m;
        return x;
    };
    auto blk_put = [&](int b, const Blk &x) {
        const RowRec rr = row_val(x.r);
        const dvec2 m2{rr.mt, skew ? rr.mm * 0.99 : rr.mm}, i2{rr.is, rr.ds};
        const int i = ((64 * b) & (DPM_RING - 1)) + q;
        s_rec[2 * i] = m2;
        s_rec[2 * i + 1] = i2;
        s_sb[i] = (uint8_t)rr.sb;
        s_col[i] = (uint8_t)(x.colok ? x.col : 4);
        if (i < DPM_RINGX - DPM_RING) {          // the mirrored tail
            s_rec[2 * (i + DPM_RING)] = m2;
            s_rec[2 * (i + DPM_RING) + 1] = i2;
            s_sb[i + DPM_RING] = (uint8_t)rr.sb;
            s_col[i + DPM_RING] = (uint8_t)(x.colok ? x.col : 4);
        }
    };
    // per pair and parity: the periods at which the cell is in the DP
    // (d <= k, jj <= m, 0 <= ii <= n: P in [lo, lo + span]), the store offset
    int lo[2][DPM_NPL];
    unsigned span[2][DPM_NPL], vo[2][DPM_NPL];
    bool own[DPM_NPL];
#pragma unroll
    for (int r = 0; r < DPM_NPL; ++r) {
        const int pp = pb + q * DPM_NPL + r;
        own[r] = pp >= own_lo && pp < own_hi;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int d = 2 * pp + a;
            const bool inb = pp >= 0 && d < H;
            const int l = max(pp, T.c - pp - a), h = min(pp + T.m, T.n + T.c - pp - a);
            const bool ok = inb && l <= h;
            lo[a][r] = ok ? l : (1 << 30);
            span[a][r] = ok ? (unsigned)(h - l) : 0u;
            vo[a][r] = (inb && own[r]) ? 8u * (unsigned)((rev ? H - 1 - d : d) >> 1) : DPM_NOSTORE;
        }
    }
    const int porg = T.c >> 1;                       // the origin (ii = jj = 0): pair c / 2, step c
    const int kfin = T.n + T.m + T.c;                // the final cell (ii = n, jj = m)
    // the wave's compute phase [Pa, Pb]: every pair it holds (slice and halo)
    // is outside the DP before Pa and after Pb, i.e. -Inf there -- those
    // periods are stores of -Inf only (for configs[2]'s band, the ~2,600 of
    // 7,826 anti-diagonals before the origin and after the final cell)
    int la = 1 << 30, hb = -1;
#pragma unroll
    for (int r = 0; r < DPM_NPL; ++r)
#pragma unroll
        for (int a = 0; a < 2; ++a)
            if (lo[a][r] != (1 << 30)) {
                la = min(la, lo[a][r]);
                hb = max(hb, lo[a][r] + (int)span[a][r]);
            }
    for (int o = 32; o > 0; o >>= 1) {
        la = min(la, __shfl_xor(la, o));
        hb = max(hb, __shfl_xor(hb, o));
    }
    const int Pa = __builtin_amdgcn_readfirstlane(la), Pb = __builtin_amdgcn_readfirstlane(hb);
    const int NPER = (K + 1) >> 1;                   // periods: steps 2P, 2P + 1 < K
    const unsigned dso = 8u * (unsigned)(rev ? -T.P : T.P);   // band row step in bytes
    const unsigned so_base = 8u * (unsigned)((rev ? K - 1 : 0) * T.P);
    auto so_of = [&](int P) { return so_base + (unsigned)(2 * P) * dso; };
    // a period outside the compute phase: -Inf in every in-band cell the slice owns
    auto blank = [&](int P) {
        const unsigned so0 = so_of(P);
#pragma unroll
        for (int r = 0; r < DPM_NPL; ++r) {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, -RF_INF), brs, vo[0][r], so0, DPM_SC1);
            if (2 * P + 1 < K)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, -RF_INF), brs, vo[1][r], so0 + dso,
                                                      DPM_SC1);
        }
    };
    double vev[DPM_NPL], vod[DPM_NPL];
    // a pair's row record for its even step is the record its odd step read
    // one period earlier (read row pp + P - c either way): carried here
    dvec2 rmt[DPM_NPL], ris[DPM_NPL];
    int rsb[DPM_NPL];
    uint64_t bad[DPM_NPL];                       // lanes with a valid cell of -Inf
    Blk pend;
    if (Pa <= Pb) {
        // chunk t0 of Pa: blocks t0 .. t0 + DPM_NPL in the ring, t0 + DPM_NPL + 1 loading
        const int t0 = Pa >> 6;
        for (int b = t0; b <= t0 + DPM_NPL; ++b)
            blk_put(b, blk_load(b));
        pend = blk_load(t0 + DPM_NPL + 1);
        wave_sync();
    }
#pragma unroll
    for (int r = 0; r < DPM_NPL; ++r) {
        vev[r] = vod[r] = -RF_INF;
        bad[r] = 0;
        const int ri = q * DPM_NPL + r + (Pa & (DPM_RING - 1));
        rmt[r] = s_rec[2 * ri];
        ris[r] = s_rec[2 * ri + 1];
        rsb[r] = s_sb[ri];
    }
    // one period P of the compute phase: the even step 2P and the odd step
    // 2P + 1.  The LDS reads of both (the period's template bases, the odd
    // step's row records) are issued first.  EDGE: the period may hold the
    // origin, the final cell or no odd step (K odd).
    auto period = [&](auto EDGEC, const int P) {
        constexpr bool EDGE = decltype(EDGEC)::value;
        const bool odd_too = !EDGE || 2 * P + 1 < K;
        const unsigned so0 = so_of(P);
        const int s = P & (DPM_RING - 1);
        const int ir = q * DPM_NPL + 1 + s, ic = s + 64 * DPM_NPL - 1 - q * DPM_NPL;
        int tbb[DPM_NPL];
        dvec2 omt[DPM_NPL], ois[DPM_NPL];
        int osb[DPM_NPL];
#pragma unroll
        for (int r = 0; r < DPM_NPL; ++r) {
            tbb[r] = s_col[ic - r];
            omt[r] = s_rec[2 * (ir + r)];
            ois[r] = s_rec[2 * (ir + r) + 1];
            osb[r] = s_sb[ir + r];
        }
        auto cells = [&](auto PARC, const dvec2 (&mt)[DPM_NPL], const dvec2 (&is2)[DPM_NPL], const int (&sbr)[DPM_NPL]) {
            constexpr int par = decltype(PARC)::value;
            const int k = 2 * P + par;
            const unsigned so = par ? so0 + dso : so0;
            // the neighbouring pair's kappa - 1 value across the lane edge
            // (lanes 0 and 63 hold halo pairs or pairs outside the band: what
            // they receive there is never a slice's value)
            const double nbL = par ? 0.0 : dpp_rot_f64<TaskLanes<64>::FROM_L1>(vod[DPM_NPL - 1]);
            const double nbR = par ? dpp_rot_f64<TaskLanes<64>::FROM_R1>(vev[0]) : 0.0;
            double nv[DPM_NPL];
            bool val[DPM_NPL];
#pragma unroll
            for (int r = 0; r < DPM_NPL; ++r) {
                const double a2 = par ? vod[r] : vev[r];
                const double a1l = par ? vev[r] : (r > 0 ? vod[r > 0 ? r - 1 : 0] : nbL);
                const double a1r = par ? (r < DPM_NPL - 1 ? vev[r < DPM_NPL - 1 ? r + 1 : 0] : nbR) : vod[r];
                const double ms = sbr[r] == tbb[r] ? mt[r].x : mt[r].y;
                double is = is2[r].x;
                if (TRIM) {
                    const int jj = P - (pb + q * DPM_NPL + r);
                    is = (trim && (jj == 0 || jj == T.m)) ? 0.0 : is;
                }
                // align.jl:77-104: the maximum of the candidates
                const double best = fmax(fmax(a2 + ms, a1l + is), a1r + is2[r].y);
                val[r] = (unsigned)(P - lo[par][r]) <= span[par][r];
                nv[r] = val[r] ? best : -RF_INF;
            }
            if (EDGE && k == T.c) {
#pragma unroll
                for (int r = 0; r < DPM_NPL; ++r)
                    nv[r] = (pb + q * DPM_NPL + r == porg && val[r]) ? 0.0 : nv[r];
            }
#pragma unroll
            for (int r = 0; r < DPM_NPL; ++r) {
                // "new score is invalid"
                bad[r] |= __builtin_amdgcn_ballot_w64(nv[r] == -RF_INF) & __builtin_amdgcn_ballot_w64(val[r]);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, nv[r]), brs, vo[par][r], so,
                                                      DPM_SC1);
                if (par)
                    vod[r] = nv[r];
                else
                    vev[r] = nv[r];
            }
            if (EDGE && k == kfin && out_score) {
#pragma unroll
                for (int r = 0; r < DPM_NPL; ++r)
                    if (own[r] && val[r] && pb + q * DPM_NPL + r == P - T.m)
                        out_score[T.out_idx] = nv[r];
            }
        };
        cells(std::integral_constant<int, 0>{}, rmt, ris, rsb);
        if (odd_too)
            cells(std::integral_constant<int, 1>{}, omt, ois, osb);
#pragma unroll
        for (int r = 0; r < DPM_NPL; ++r) {
            rmt[r] = omt[r];
            ris[r] = ois[r];
            rsb[r] = osb[r];
        }
    };
    // ---- hand-off after period P: the halo pairs' values at steps 2P (even
    // diagonal) and 2P + 1 (odd), polled from their owners' cells where the
    // cell is in the DP (an owner computes every such cell; -Inf elsewhere)
    auto hand_off = [&](const int P) {
        const unsigned so0 = so_of(P);
        bool pe[DPM_NPL], po[DPM_NPL];
        const double *ae[DPM_NPL], *ao[DPM_NPL];
#pragma unroll
        for (int r = 0; r < DPM_NPL; ++r) {
            pe[r] = !own[r] && (unsigned)(P - lo[0][r]) <= span[0][r];
            po[r] = !own[r] && (unsigned)(P - lo[1][r]) <= span[1][r];
            const int pp = pb + q * DPM_NPL + r, de = 2 * pp, dod = 2 * pp + 1;
            ae[r] = band + (pe[r] ? (so0 >> 3) + ((rev ? H - 1 - de : de) >> 1) : 0);
            ao[r] = band + (po[r] ? ((so0 + dso) >> 3) + ((rev ? H - 1 - dod : dod) >> 1) : 0);
        }
        double he[DPM_NPL], ho[DPM_NPL];
        for (int spins = 0;; ++spins) {
#pragma unroll
            for (int r = 0; r < DPM_NPL; ++r) {
                he[r] = ld_sc1(ae[r]);
                ho[r] = ld_sc1(ao[r]);
            }
            __builtin_amdgcn_s_waitcnt(0);
            int wait = 0;
#pragma unroll
            for (int r = 0; r < DPM_NPL; ++r)
                wait |= ((int)pe[r] & (int)(__double_as_longlong(he[r]) == DPM_UNSET)) |
                        ((int)po[r] & (int)(__double_as_longlong(ho[r]) == DPM_UNSET));
            if (__builtin_amdgcn_ballot_w64(wait != 0) == 0)
                break;
            if (spins >= DPM_SPIN)
                return false;   // a neighbouring slice never arrived
            __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int r = 0; r < DPM_NPL; ++r) {
            if (own[r])
                continue;
            vev[r] = pe[r] ? he[r] : -RF_INF;
            vod[r] = po[r] ? ho[r] : -RF_INF;
        }
        // nothing of the hand-off left in flight: a register still pending at
        // the loop head would make hipcc wait vmcnt(0) -- every band store --
        // once per period
        __builtin_amdgcn_s_waitcnt(0);
        return true;
    };
    // chunk refill at P = 64 t (t > t0), the period, the hand-off every DPM_B steps
    auto body = [&](auto EDGEC, const int P) {
        if ((P & 63) == 0 && P != Pa) {          // chunk t: rows / columns of block t + DPM_NPL
            const int t = P >> 6;
            __builtin_amdgcn_s_waitcnt(0);       // after a hand-off: nothing left in flight
            blk_put(t + DPM_NPL, pend);
            pend = blk_load(t + DPM_NPL + 1);
            wave_sync();
        }
        period(EDGEC, P);
        const int kn = 2 * P + 2;                // steps done
        return !(kn % DPM_B == 0 && P < Pb) || hand_off(P);
    };
    // the compute phase first (its hand-offs pace the neighbours), in runs of
    // plain periods between the special ones
    const int psp[3] = {porg, kfin >> 1, (K & 1) ? NPER - 1 : INT_MAX};
    bool ok = true;
    for (int P = Pa; P <= Pb && ok;) {
        int stop = Pb + 1;
        for (int i = 0; i < 3; ++i)
            if (psp[i] >= P && psp[i] < stop)
                stop = psp[i];
        for (; P < stop && ok; ++P)
            ok = body(std::false_type{}, P);
        if (P <= Pb && ok) {
            ok = body(std::true_type{}, P);
            ++P;
        }
    }
    if (!ok) {
        set_err(err, 4);
        return;
    }
    for (int P = 0; P < min(Pa, NPER); ++P)
        blank(P);
    for (int P = max(Pb + 1, Pa <= Pb ? 0 : NPER); P < NPER; ++P)
        blank(P);
    bool e = false;
#pragma unroll
    for (int r = 0; r < DPM_NPL; ++r)
        e = e || (own[r] && ((bad[r] >> q) & 1));
    if (e)
        set_err(err, 1);
}

// ---------------------------------------------------------------------
// k_dpx: latency-bound non-lean tasks (round 5).
//
// The reference's codon DP (align.jl:77-104 with codon moves; skew_matches
// for single_indel_proposals, model.jl:538-562) is one task of ~5,000
// anti-diagonals per call: nothing else runs beside it, so its time is the
// step latency of one wave, i.e. the instructions one step issues.  k_dpr's
// general step moved every row record through the lanes (7 DPP moves per
// value and period), took the codon neighbours by two wave shifts each and
// waited for its edge loads with vmcnt(0) -- ~900 cycles per anti-diagonal
// (profiles/r05a_kernel_stats_c3.csv).  Here one task owns a single-wave
// workgroup, lane q holds the diagonal pair {2q, 2q+1} (H <= 127), and
//   - the row records {match, mismatch (x 0.99 under skew), ins, del,
//     codon ins, codon del, base} and the template bases are staged in LDS
//     rings of 256 rows / columns, 64 at a time, loaded a block ahead:
//     lane q reads row P + q + par - c and column P - q at period P (one
//     LDS read set per period instead of the systolic moves);
//   - every anti-diagonal's values go to a 4-row LDS ring as well, so the
//     codon neighbours (d -/+ 3 at kappa - 3) are two LDS reads at an
//     immediate offset; only the insert / delete neighbour at kappa - 1
//     (on the step-to-step chain) is a DPP wave shift;
//   - interior steps (every active diagonal inside the matrix, codon moves
//     allowed, no trim column) carry no range checks: inactive diagonals
//     get -Inf by an additive mask, as in the lean kernels.
// Same candidates, same FP64 sums and the same strict-'>' value (the max of
// the candidates; no NaN, no -0.0) as k_dpr / k_dp, stored in the same
// kappa-major positions (reverse: flipped), so bands, scores and errors are
// bit-identical.
// ---------------------------------------------------------------------
constexpr int DPX_W = 72;       // doubles per LDS band row: 2 pad | 64 lanes | 6 pad (-Inf)
#ifndef DPX_STAGE
#define DPX_STAGE 1   // interior rows staged in LDS, four per contiguous flush
#endif
#ifndef DPX_FL16
#define DPX_FL16 1    // the flush in 16-B stores when the run is 16-B aligned
#endif
constexpr int DPX_RING = 256;   // staged rows / columns: 4 blocks of 64
struct DpxStage {
    RawRow r;
    int col;
    bool colok;
};

constexpr unsigned DPX_NOSTORE = 0x80000000u;   // buffer offset past any band: the store is dropped
// a k_dpx task: H <= 127 (lanes hold diagonal pairs) and a band below 2 GiB
// (32-bit buffer offsets, DPX_NOSTORE past it)
inline bool dpx_fits(const DPTask &t) { return t.H <= 127 && (int64_t)t.klen * t.P * 8 < ((int64_t)1 << 31); }

template <int PAR, bool FAST, bool CODON, bool CHECK>
__device__ __forceinline__ double dpx_cell(const DPTask &T, bool trim, int d, int ii, int jj, double v1,
                                           double v2, double xn, double yci, double ycd, const dvec2 &mtmm,
                                           const dvec2 &isds, const dvec2 &cicd, int sb, int tbb, double lbv,
                                           uint64_t actm, uint64_t &emask, int &eflag, double &fval, int &fset)
{
    const double ms = sb == tbb ? mtmm.x : mtmm.y;   // mismatch staged x 0.99 under skew (align.jl:70-72)
    const double x_ins = PAR ? v1 : xn;               // (d-1, kappa-1)
    const double x_del = PAR ? xn : v1;               // (d+1, kappa-1)
    if (FAST) {
        // candidates off the step-to-step chain first, the kappa-1 pair last
        const double t = CODON ? fmax(fmax(v2 + ms, yci + cicd.x), ycd + cicd.y) : v2 + ms;
        const double best = fmax(t, fmax(x_ins + isds.x, x_del + isds.y));
        if (CHECK)
            emask |= __ballot(best == -RF_INF) & actm;   // "new score is invalid" (active diagonals)
        return best + lbv;
    }
    const bool valid = d < T.H && jj >= 0 && jj <= T.m && ii >= 0 && ii <= T.n;
    const double is = (trim && (jj == 0 || jj == T.m)) ? 0.0 : isds.x;   // align.jl:74-76
    double best = fmax(fmax(v2 + ms, x_ins + is), x_del + isds.y);
    if (CODON) {
        const double cd = jj >= 3 ? cicd.y : -RF_INF;       // codon delete needs j > 3
        best = fmax(fmax(best, yci + cicd.x), ycd + cd);   // cicd.x is -Inf unless i > 3 (staged)
    }
    const bool origin = ii == 0 && jj == 0;
    const double v = valid ? (origin ? 0.0 : best) : -RF_INF;
    eflag |= (valid && !origin && best == -RF_INF) ? 1 : 0;
    const bool fin = valid && ii == T.n && jj == T.m;
    fval = fin ? v : fval;
    fset |= fin ? 1 : 0;
    return v;
}

// CODON: the task may have codon moves (ring of the last four anti-diagonals
// in LDS); CHECK: the interior raises "new score is invalid" (non-finite
// tables).  <false, false> takes the latency-mode lean tasks (finite tables,
// no codon / skew / trim, RF_OPT_DP_LAT), <true, true> every other task.
template <bool CODON, bool CHECK>
__global__ void __launch_bounds__(128)
k_dpx(const DPTask *__restrict__ tasks, int ntasks, const uint8_t *__restrict__ bases,
      const double *__restrict__ tabs, double *__restrict__ bands, double *__restrict__ out_score,
      int *__restrict__ err)
{
    __shared__ dvec2 s_mtmm[DPX_RING], s_isds[DPX_RING], s_cicd[CODON ? DPX_RING : 1];
    __shared__ int s_sb[DPX_RING], s_col[DPX_RING];
    __shared__ double s_band[CODON ? 4 * DPX_W : 1];
    // DPX_STAGE: the interior's four rows of a pair of periods, staged here
    // and written as one contiguous run (P <= 65)
    // (lean tasks only: the reference's single codon task, latency-bound on
    // one wave, ran 0.43 -> 0.61 ms with it; 1,000 lean reads 0.52 -> 0.49 ms,
    // profiles/r05bt_exp_dpx_stage.jsonl)
    constexpr bool STAGE = DPX_STAGE && !CODON;
    __shared__ __attribute__((aligned(16))) double s_out[STAGE ? 4 * 72 : 1];
    // wave 0 fills the band; wave 1 stages the edge records (round 5: its
    // loads' waits are its own, so the filling wave never waits on vmcnt,
    // which would drain its band stores too)
    const int q = threadIdx.x & 63;
    const bool loader = threadIdx.x >= 64;
    const DPTask T = tasks[blockIdx.x];   // one task per workgroup
    const bool rev = T.flags & 1, skew = T.flags & 2, trim = T.flags & 4;
    const bool codon = CODON && (T.ncins > 0 || T.ncdel > 0);
    const uint8_t *sbase = bases + T.sb;
    const uint8_t *tbase = bases + T.tb;
    const double *tb = tabs + T.tab;
    const int K = T.klen;
    // band stores through a buffer resource: a lane that stores nothing at a
    // step gets an offset past the band (dropped by the range check), so no
    // step changes exec for its store (the host keeps K * P * 8 < 2^31)
    const __amdgpu_buffer_rsrc_t brs =
        __builtin_amdgcn_make_buffer_rsrc(bands + T.band, 0, (int)((int64_t)K * T.P * 8), 0x00020000);
    if (CODON && !loader)
        for (int e = q; e < 4 * DPX_W; e += 64)
            s_band[e] = -RF_INF;

    // block b: rows R = P + q + par in [64b, 64b + 64) (read row R - c) and
    // columns J = P - q + 64 in [64b, 64b + 64) (template column J - 64)
    // A block's loads are held raw (load_row_raw) until the block is put in
    // LDS a chunk later, and their range selects (and the skew factor) are
    // applied there: a select right after the loads made hipcc wait for them
    // at once, draining every band store in flight (vmcnt counts both).
    auto stage_load = [&](int b) {
        DpxStage s;
        s.r = load_row_raw(T, rev, sbase, tb, 64 * b + q - T.c, codon);
        const int jj = 64 * b + q - 64;
        const int jc = min(max(jj, 1), max(T.m, 1));
        s.col = tbase[rev ? max(T.m - jc, 0) : jc - 1];
        s.colok = jj >= 1 && jj <= T.m;
        return s;
    };
    auto stage_put = [&](int b, const DpxStage &s) {
        const int i = (64 * b + q) & (DPX_RING - 1);
        const RowRec r = row_val(s.r);
        s_mtmm[i] = dvec2{r.mt, skew ? r.mm * 0.99 : r.mm};
        s_isds[i] = dvec2{r.is, r.ds};
        if (CODON)
            s_cicd[i] = dvec2{r.ci, r.cd};
        s_sb[i] = r.sb;
        s_col[i] = s.colok ? s.col : 4;
    };

    // interior [klo, khi]: every diagonal with cells in the matrix has its
    // cell inside the matrix (with i, j > 3: codon moves open) and j in
    // 1..m-1 (trim off); the origin and the final cell lie outside it
    double lb[2];
    bool act[2];
    // kappa of (0, 0) + 1, and at least H: every band diagonal has d <= kappa
    // (stored); kappa of (n, m) - 1
    int lo = max(T.c + 1, T.H), hi = T.n + T.c + T.m - 1;
    bool ok = true;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        const int d = 2 * q + par;
        const int mlo = max(0, T.c - d), mhi = min(T.m, T.n + T.c - d);
        act[par] = d < T.H && mlo <= mhi;
        lb[par] = act[par] ? 0.0 : -RF_INF;
        if (act[par]) {
            const int jlo = CODON ? max(3, T.c + 3 - d) : max(trim ? 1 : 0, T.c - d);
            const int jhi = min(T.m - (trim ? 1 : 0), T.n + T.c - d);
            ok = ok && jlo <= jhi;
            lo = max(lo, d + 2 * jlo);
            hi = min(hi, d + 2 * jhi);
        }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        lo = max(lo, __shfl_xor(lo, off));
        hi = min(hi, __shfl_xor(hi, off));
    }
    const int klo = __builtin_amdgcn_readfirstlane(__all(ok) ? lo : INT_MAX);
    const int khi = __builtin_amdgcn_readfirstlane(hi);

    const int npairs = (K + 3) >> 2;
    if (loader) {
        // blocks 0-2 before the fill starts; block t + 3 during chunk t (ring
        // slot of block t - 1, which chunk t no longer reads), one barrier
        // per chunk boundary 1 .. nch - 1
        stage_put(0, stage_load(0));
        stage_put(1, stage_load(1));
        stage_put(2, stage_load(2));
        lds_barrier();
        const int nch = (npairs + 31) >> 5;
        for (int t = 0; t + 1 < nch; ++t) {
            stage_put(t + 3, stage_load(t + 3));
            lds_barrier();
        }
        return;
    }
    lds_barrier();

    // per parity: byte offset of this lane's band element in a kappa row
    // (reverse: flipped), or past the band when the row does not hold it
    const unsigned vo0 = 2 * q < T.H ? 8u * (unsigned)(rev ? (T.H - 1 - 2 * q) >> 1 : q) : DPX_NOSTORE;
    const unsigned vo1 = 2 * q + 1 < T.H ? 8u * (unsigned)(rev ? (T.H - 2 - 2 * q) >> 1 : q) : DPX_NOSTORE;
    const unsigned rowb = 8u * (unsigned)T.P;
    const uint64_t actm0 = __ballot(act[0]), actm1 = __ballot(act[1]);
    double v1 = -RF_INF, v2 = -RF_INF;
    uint64_t emask = 0;
    int eflag = 0, fset = 0;
    double fval = 0.0;
    // Records of a pair of periods (2u, 2u + 1): rows R = 2u + q (c), 2u + q + 1
    // (a), 2u + q + 2 (b) and columns J = 2u - q + 64, + 1.  Pair u reads the
    // records of pair u + 1 (rows 2u + q + 3, + 4 and the next columns) into
    // set u mod 3; its own a / b are set u - 1 and its c is the b of set u - 2.
    // The loop runs three pairs per iteration with the sets rotated by name,
    // so no record moves between registers (round 5: the one-pair loop copied
    // 17 registers per pair at its end, ~4 of the ~22 instructions per step).
    struct Rec {
        dvec2 mtmm, isds, cicd;
        int sb;
    };
    auto rec_ld = [&](int r) {
        Rec x;
        x.mtmm = s_mtmm[r];
        x.isds = s_isds[r];
        x.cicd = CODON ? s_cicd[r] : dvec2{0.0, 0.0};
        x.sb = s_sb[r];
        return x;
    };
    Rec A0, B0, A1, B1, A2, B2;
    int C00 = 0, C01 = 0, C10 = 0, C11 = 0, C20, C21;
    B1 = rec_ld(q);              // set -2: b = row q
    A2 = rec_ld(q + 1);          // set -1: rows q + 1, q + 2, columns 64 - q, 65 - q
    B2 = rec_ld(q + 2);
    C20 = s_col[(64 - q) & (DPX_RING - 1)];
    C21 = s_col[(65 - q) & (DPX_RING - 1)];
    A0 = A1 = B0 = A2;           // (defined before their first load)
    // the codon neighbours of the next step, read one step ahead (kappa = 0:
    // ring row 1, still -Inf)
    double cy_ci = CODON ? s_band[DPX_W + 2 + q - 2] : 0.0, cy_cd = CODON ? s_band[DPX_W + 2 + q + 1] : 0.0;
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using BT = std::integral_constant<bool, true>;
    using BF = std::integral_constant<bool, false>;
    // byte offset of kappa row 4u (reverse: K - 1 - 4u), advanced once per
    // pair of periods (the per-step select and multiply off the loop)
    const int drow = rev ? -(int)rowb : (int)rowb;
    unsigned rob = rev ? rowb * (unsigned)(K - 1) : 0u;
    auto pair = [&](const int u, const Rec &c, const Rec &a, const Rec &b, const int col0, const int col1, Rec &na,
                    Rec &nb, int &ncol0, int &ncol1) {
        if ((u & 31) == 0 && u > 0)   // chunk t = u / 32 (64 periods): block t + 2 is in
            lds_barrier();
        // the next pair's records (rows <= 2u + 67: block t + 2 at most, in LDS)
        na = rec_ld((2 * u + q + 3) & (DPX_RING - 1));
        nb = rec_ld((2 * u + q + 4) & (DPX_RING - 1));
        ncol0 = s_col[(2 * u - q + 66) & (DPX_RING - 1)];
        ncol1 = s_col[(2 * u - q + 67) & (DPX_RING - 1)];
        // four steps kappa = 4u + s: (period, parity) = (2u, 0), (2u, 1), (2u+1, 0), (2u+1, 1)
        auto step = [&](auto FASTC, auto PARC, auto SC, int per, const Rec &r, int col) {
            constexpr bool FAST = decltype(FASTC)::value;
            constexpr int PAR = decltype(PARC)::value, S = decltype(SC)::value;
            const int k = 4 * u + S;
            if (!FAST && k >= K)
                return;
            // the kappa - 1 neighbour by a wave rotate: lane 0 (63) receives the
            // value of diagonal 127 (0 at kappa - 1 into diagonal 127), and
            // diagonal 127 >= H is -Inf / masked (the host sends H <= 127 only)
            const double xn = PAR ? dpp_rot_f64<TaskLanes<64>::ROT_R1>(v1) : dpp_rot_f64<TaskLanes<64>::ROT_L1>(v1);
            // codon neighbours at kappa - 3: d - 3 / d + 3 = lanes q - 2 / q + 1
            // (even), q - 1 / q + 2 (odd); this step's were read one step ago,
            // the next step's (ring row kappa - 2, the other parity) now
            const double yci = cy_ci, ycd = cy_cd;
            if (CODON) {
                const double *rr = s_band + ((S + 2) & 3) * DPX_W + 2 + q;
                cy_ci = rr[PAR ? -2 : -1];
                cy_cd = rr[PAR ? 1 : 2];
            }
            const int d = 2 * q + PAR;
            const int jj = per - q, ii = per + q + PAR - T.c;
            const double v = dpx_cell<PAR, FAST, CODON, CHECK>(T, trim, d, ii, jj, v1, v2, xn, yci, ycd, r.mtmm,
                                                               r.isds, r.cicd, r.sb, col, lb[PAR],
                                                               PAR ? actm1 : actm0, emask, eflag, fval, fset);
            if (CODON) {
                s_band[S * DPX_W + 2 + q] = v;
                // other lanes read this row two and three steps on: keep hipcc
                // from hoisting those reads above the write (the three-pair loop
                // body gives it the room; LDS is in order within the wave)
                wave_sync();
            }
            const unsigned ro = rob + (unsigned)(S * drow);   // = rowb * (rev ? K - 1 - k : k)
            const unsigned vo = PAR ? vo1 : vo0;
            if (STAGE && FAST) {
                if (vo != DPX_NOSTORE)
                    s_out[(rev ? 3 - S : S) * T.P + (int)(vo >> 3)] = v;
            } else {
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), brs,
                                                      (FAST || d <= k) ? vo + ro : DPX_NOSTORE, 0, 0);
            }
            v2 = v1;
            v1 = v;
        };
        if (4 * u >= klo && 4 * u + 3 <= khi) {
            step(BT{}, I0{}, I0{}, 2 * u, c, col0);
            step(BT{}, I1{}, I1{}, 2 * u, a, col0);
            step(BT{}, I0{}, I2{}, 2 * u + 1, a, col1);
            step(BT{}, I1{}, I3{}, 2 * u + 1, b, col1);
            if (STAGE) {
                // rows 4u .. 4u + 3 (reverse: K - 4 - 4u .. K - 1 - 4u) are one
                // run of 4P doubles.  A 16-B aligned run (forward always; reverse
                // when K is even) goes out as 16-B stores of consecutive lanes,
                // a fixed DPX_FL16 per lane (4P <= 260 doubles: 130 pairs),
                // lanes past the run at an offset past the band; else 8-B
                // stores in a loop (round 6: the loop issued ~30 instructions
                // per pair of periods)
                wave_sync();
                const unsigned base = rev ? rob - 3u * rowb : rob;
                const int n = 4 * T.P;
                if (DPX_FL16 && (base & 15u) == 0) {
                    const dvec2 *s2 = reinterpret_cast<const dvec2 *>(s_out);
                    const int n2 = n >> 1;
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const int t = q + 64 * j;
                        const dvec2 v = s2[min(t, n2 - 1)];
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), brs,
                                                               t < n2 ? base + 16u * (unsigned)t : DPX_NOSTORE, 0,
                                                               0);
                    }
                } else {
                    for (int t = q; t < n; t += 64)
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, s_out[t]), brs,
                                                              base + 8u * (unsigned)t, 0, 0);
                }
                wave_sync();
            }
        } else {
            step(BF{}, I0{}, I0{}, 2 * u, c, col0);
            step(BF{}, I1{}, I1{}, 2 * u, a, col0);
            step(BF{}, I0{}, I2{}, 2 * u + 1, a, col1);
            step(BF{}, I1{}, I3{}, 2 * u + 1, b, col1);
        }
        rob += (unsigned)(4 * drow);
    };
    int u = 0;
    for (; u + 3 <= npairs; u += 3) {
        pair(u, B1, A2, B2, C20, C21, A0, B0, C00, C01);
        pair(u + 1, B2, A0, B0, C00, C01, A1, B1, C10, C11);
        pair(u + 2, B0, A1, B1, C10, C11, A2, B2, C20, C21);
    }
    if (u < npairs)
        pair(u, B1, A2, B2, C20, C21, A0, B0, C00, C01);
    if (u + 1 < npairs)
        pair(u + 1, B2, A0, B0, C00, C01, A1, B1, C10, C11);
    (void)ntasks;
    if (eflag || emask)
        set_err(err, 1);  // "new score is invalid"
    if (fset && out_score)
        out_score[T.out_idx] = fval;
}

// ---------------------------------------------------------------------
// k_score: dense proposal scoring of batch reads (no codon moves)
//
// One lane per consensus position p in [0, m].  For a read it evaluates
// every proposal anchored at p -- Substitution(p, b) (4 bases, the one equal
// to the consensus base is never requested), Deletion(p), Insertion(p, b) --
// from A columns p-1 and p and B column p (0-based), exactly as
// score_nocodon (model.jl:242-285) and seq_score_deletion (:227-236) do,
// with new columns built in the reference's update order.  The per-read
// results are left-folded over the group's reads in batch order
// (model.jl:389-393).  Output slots: 0-3 sub A,C,G,T; 4 del; 5-8 ins A,C,G,T.
// A failed update ("new score is invalid") or a -Inf sum ("failed to compute
// a valid score") is reported as NaN in that slot.
//
// The A/B kappa rows covering the 64 positions of a work item are one
// contiguous block; it is staged through LDS with coalesced loads when it
// fits (the common narrow band), otherwise read in place.
// ---------------------------------------------------------------------

constexpr int SCORE_C = 64;    // positions per work item

// Accessor of a band window: rows [k0, ...) of a kappa-major band.
struct BandWin {
    const double *base;
    int k0, P;
    __device__ __forceinline__ double at(int d, int jj) const
    {
        return base[(size_t)(d + 2 * jj - k0) * P + (d >> 1)];
    }
};

// HALF 0: Substitution(p, b) chains + Deletion(p)  -> out[0..4]
// HALF 1: Insertion(p, b) chains                     -> out[5..8]
// (two waves of one workgroup share the staged A/B window).
// update() of a new column (align.jl:50-112) keeps the first strictly-best
// of {match, insert, delete}; its value is the FP64 max of the three sums
// (no NaN / signed zero among candidates), and the sums are formed from the
// same operands as the reference, so fmax is bit-exact.  A chain that hits
// -Inf ("new score is invalid") is detected by the running minimum.
template <int HALF>
__device__ __forceinline__ void score_half(int p, int m, const ScoreRead &R,
                                           const uint8_t *__restrict__ s,
                                           const double *__restrict__ tb,
                                           const BandWin A, const BandWin B, double out[5])
{
    const int n = R.n, c = R.c, vb = R.vb;
    const double *t_match = tb;
    const double *t_mism = tb + n;
    const double *t_ins = tb + 2 * (size_t)n;
    const double *t_del = tb + 3 * (size_t)n;
    const double qnan = __builtin_nan("");
    // row ranges (bandedarrays.jl:133-137), 0-based rows
    const int s0 = max(0, p - c), s1 = min(p + vb, n);             // rows(p): new Sub col, B col p
    double prev[4], acc[4], mn[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        prev[b] = -RF_INF;
        acc[b] = -RF_INF;
        mn[b] = RF_INF;
    }
    if (HALF == 0) {
        if (p < 1) {
#pragma unroll
            for (int k = 0; k < 5; ++k)
                out[k] = qnan;
            return;
        }
        const int d0 = max(0, p - 1 - c), d1 = min(p - 1 + vb, n);  // rows(p-1): A col p-1
        double del_acc = -RF_INF;
        // A(p-1, ii) in band iff ii in rows(p-1)
        double am1_prev = (s0 - 1 >= d0) ? A.at(s0 - 1 - (p - 1) + c, p - 1) : -RF_INF;
        for (int ii = s0; ii <= s1; ++ii) {
            const double am1 = (ii <= d1) ? A.at(ii - (p - 1) + c, p - 1) : -RF_INF;
            const double b0 = B.at(ii - p + c, p);
            const int sb = ii >= 1 ? s[ii - 1] : 4;
            const int ks = max(ii - 1, 0);
            const double dm = am1_prev + t_match[ks];     // match predecessor (i-1, p)
            const double dx = am1_prev + t_mism[ks];      //   ... mismatching base
            const double is = t_ins[ks];
            const double dl = am1 + t_del[ii];            // delete predecessor (i, p)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const double best = fmax(fmax(sb == b ? dm : dx, prev[b] + is), dl);
                mn[b] = fmin(mn[b], best);
                prev[b] = best;
                acc[b] = fmax(acc[b], best + b0);     // summax, util.jl:40-48
            }
            if (ii <= d1)
                del_acc = fmax(del_acc, am1 + b0);    // seq_score_deletion, model.jl:227-236
            am1_prev = am1;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b)
            out[b] = (mn[b] == -RF_INF || acc[b] == -RF_INF) ? qnan : acc[b];
        out[4] = del_acc;
    } else {
        const int pI = min(p + 1, m);                                // new Ins col's row range
        const int i0 = max(0, pI - c), i1 = min(pI + vb, n);
        // A(p, ii) in band iff ii in rows(p)
        double a0_prev = (i0 - 1 >= s0) ? A.at(i0 - 1 - p + c, p) : -RF_INF;
        for (int ii = i0; ii <= i1; ++ii) {
            const bool in_s = ii <= s1;
            const double a0 = in_s ? A.at(ii - p + c, p) : -RF_INF;
            const double b0 = in_s ? B.at(ii - p + c, p) : -RF_INF;
            const int sb = ii >= 1 ? s[ii - 1] : 4;
            const int ks = max(ii - 1, 0);
            const double dm = a0_prev + t_match[ks];
            const double dx = a0_prev + t_mism[ks];
            const double is = t_ins[ks];
            const double dl = a0 + t_del[ii];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const double best = fmax(fmax(sb == b ? dm : dx, prev[b] + is), dl);
                mn[b] = fmin(mn[b], best);
                prev[b] = best;
                acc[b] = fmax(acc[b], best + b0);
            }
            a0_prev = a0;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b)
            out[b] = (mn[b] == -RF_INF || acc[b] == -RF_INF) ? qnan : acc[b];
    }
}

// One workgroup = 2 waves x 64 lanes: lane l of wave h handles position
// p0 + l, wave 0 the Substitution/Deletion proposals, wave 1 the
// Insertions.  grid.x = work items (group, chunk of SCORE_C positions);
// grid.y = read index in split mode.  Fused mode folds all reads of the
// group in batch order.  lds_elems: doubles the dynamic LDS holds per band.
__global__ void __launch_bounds__(128)
k_score(const WorkItem *__restrict__ items, const ScoreGroup *__restrict__ groups,
        const ScoreRead *__restrict__ reads, const uint8_t *__restrict__ bases,
        const double *__restrict__ tabs, const double *__restrict__ bands,
        double *__restrict__ dense, double *__restrict__ split, int split_mode, int lds_elems)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const WorkItem w = items[blockIdx.x];
    const ScoreGroup G = groups[w.group];
    const int lane = threadIdx.x & 63;
    const int half = threadIdx.x >> 6;
    const int p = w.p0 + lane;
    int r0 = G.r0, r1 = G.r1;
    if (split_mode) {
        r0 = G.r0 + blockIdx.y;
        if (r0 >= G.r1)
            return;
        r1 = r0 + 1;
    }
    double tot[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
        tot[k] = 0.0;
    double *sA = smem;
    double *sB = smem + lds_elems;
    const int k0 = 2 * (w.p0 - 1);                    // window's first kappa row
    for (int r = r0; r < r1; ++r) {
        const ScoreRead R = reads[r];
        const double *A = bands + R.A;
        const double *B = bands + R.B;
        const bool stage = (2 * SCORE_C + R.H) * R.P <= lds_elems;
        double sc[5];
        if (stage) {
            // contiguous kappa rows -> LDS, coalesced, 16 loads in flight per lane
            const int kbeg = max(k0, 0);
            const int kend = min(k0 + 2 * SCORE_C + R.H, R.K);
            const int nel = (kend - kbeg) * R.P;
            const int off = (kbeg - k0) * R.P;
            const double *ga = A + (size_t)kbeg * R.P;
            const double *gb = B + (size_t)kbeg * R.P;
            for (int e0 = 0; e0 < nel; e0 += 128 * 8) {
                double ra[8], rb[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int e = e0 + u * 128 + threadIdx.x;
                    if (e < nel) {
                        ra[u] = ga[e];
                        rb[u] = gb[e];
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int e = e0 + u * 128 + threadIdx.x;
                    if (e < nel) {
                        sA[off + e] = ra[u];
                        sB[off + e] = rb[u];
                    }
                }
            }
            __syncthreads();
            if (p <= G.m) {
                if (half == 0)
                    score_half<0>(p, G.m, R, bases + R.sb, tabs + R.tab, BandWin{sA, k0, R.P},
                                  BandWin{sB, k0, R.P}, sc);
                else
                    score_half<1>(p, G.m, R, bases + R.sb, tabs + R.tab, BandWin{sA, k0, R.P},
                                  BandWin{sB, k0, R.P}, sc);
            }
            __syncthreads();
        } else if (p <= G.m) {
            if (half == 0)
                score_half<0>(p, G.m, R, bases + R.sb, tabs + R.tab, BandWin{A, 0, R.P},
                              BandWin{B, 0, R.P}, sc);
            else
                score_half<1>(p, G.m, R, bases + R.sb, tabs + R.tab, BandWin{A, 0, R.P},
                              BandWin{B, 0, R.P}, sc);
        }
        if (p <= G.m) {
#pragma unroll
            for (int k = 0; k < 5; ++k)
                tot[k] += sc[k];
        }
    }
    if (p > G.m)
        return;
    double *dst = split_mode ? split + G.split_off + ((size_t)blockIdx.y * (G.m + 1) + p) * 9
                             : dense + G.dense_off + (size_t)p * 9;
    if (half == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k)
            dst[k] = tot[k];
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            dst[5 + k] = tot[k];
    }
}

// split mode: ordered fold over reads, one lane per (group position slot).
__global__ void k_reduce(const ScoreGroup *__restrict__ groups, int ngroups,
                         const int64_t *__restrict__ gstart, int64_t total,
                         const double *__restrict__ split, double *__restrict__ dense)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total)
        return;
    // find group (gstart: prefix of (m+1)*9 per group; empty groups skipped)
    int lo = 0, hi = ngroups - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (gstart[mid] <= e)
            lo = mid;
        else
            hi = mid - 1;
    }
    const ScoreGroup G = groups[lo];
    const int64_t local = e - gstart[lo];
    const int64_t stride = (int64_t)(G.m + 1) * 9;
    const double *src = split + G.split_off + local;
    const int nr = G.r1 - G.r0;
    // the left fold in read order (model.jl:389-393); 16 partials are loaded
    // before they are added, so each lane keeps 16 streaming loads in flight
    double acc = 0.0;
    int r = 0;
    for (; r + 16 <= nr; r += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
            v[u] = __builtin_nontemporal_load(src + (int64_t)(r + u) * stride);
#pragma unroll
        for (int u = 0; u < 16; ++u)
            acc += v[u];
    }
    for (; r < nr; ++r)
        acc += __builtin_nontemporal_load(src + (int64_t)r * stride);
    dense[G.dense_off + local] = acc;
}

// ---------------------------------------------------------------------
// Lean dense scoring (k_score_ws, k_score_segl): one new-column chain per lane
//
// A new column built from A column a (0-based) with base b over the rows of
// column min(a+1, m) serves two proposals (model.jl:250-270):
//   Substitution(a+1, b)  acol = a+1 (1-based) -> summax with B column a+1
//   Insertion(a, b)       acol = a+1 (1-based) -> summax with B column a
// (same A column, same rows, same base: the chains are identical), and the
// lane also folds Deletion(a+1) = max_i A(i, a) + B(i, a+1) (model.jl:227-236).
// So lane a writes slots 5-8 of position a and slots 0-4 of position a+1.
//
// Eligible when every read of the launch has finite match / mismatch / ins /
// del tables (the lean DP condition): then every in-band A and B cell is
// finite, a new column can never hold -Inf, and the reference's "new score
// is invalid" check cannot fire; an empty summax still reports NaN.
//
// Per read, the kappa rows of the work item's columns (one contiguous block
// per band) are staged in LDS with 16-B loads -- the next read's block is
// prefetched into VGPRs while the current one is scored -- and the per-row tables are staged once as {sub A,C,G,T, ins, del} records
// (sub_b = match if the read base is b, else mismatch), so the inner loop is
// LDS reads + FP64 max-plus only.  A read whose window exceeds the LDS budget
// is processed in sub-passes over fewer lanes.  Work items are remapped so
// that consecutive chunks of one group run on the same XCD (shared L2 for the
// H overlapping kappa rows of neighbouring chunks).
// ---------------------------------------------------------------------

// doubles of LDS a sub-pass over L lanes needs for a read of band height H

__host__ __device__ inline int lean_need(int L, int H, int P)
{
    const int win = ((2 * L + H + 1) * P + 3) & ~1;   // kappa rows + alignment shift, even
    return 2 * win + (L + H + 1) * 6;
}

// v_max_f64 without the NaN-quieting self-max hipcc adds in front of every
// fmax whose operand is a loop-carried value; the operands here are never NaN
// (finite tables, finite in-band cells, -Inf sentinels), so the result is
// the same FP64 maximum.
__device__ __forceinline__ double vmax(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}


// One row of the four new-column chains of a lane (score_nocodon's update
// over MATCH / INSERT / DELETE, model.jl:262-270, then summax's running max
// against B, util.jl:40-48): best_k = max(aprev + sub_k, prev_k + ins, dl),
// accI_k = max(accI_k, best_k + bI), accS_k = max(accS_k, best_k + bS).
// Issued phase by phase across the four chains, so that no FP64 op waits on
// the op issued right before it (measured: about 1 % faster than chain by
// chain at c5, the same values).
__device__ __forceinline__ void chain_row(double aprev, const double (&sub)[4], double ins, double dl, double bI,
                                          double bS, double (&prev)[4], double (&accI)[4], double (&accS)[4])
{
    double x[4], y[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        x[k] = aprev + sub[k];
        y[k] = prev[k] + ins;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        x[k] = vmax(x[k], y[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        prev[k] = vmax(x[k], dl);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        x[k] = prev[k] + bI;
        y[k] = prev[k] + bS;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        accI[k] = vmax(accI[k], x[k]);
        accS[k] = vmax(accS[k], y[k]);
    }
}

// Geometry of one staged (read, lanes [la0, la1]) window.
struct LeanWin {
    int kw0, shift, n16, win;   // kappa rows from kw0, 16-B chunks per band, doubles per band slot
    int t0, t1;                 // table rows
};

__device__ __forceinline__ LeanWin lean_win(const ScoreRead &R, int m, int la0, int la1)
{
    LeanWin w;
    w.kw0 = 2 * la0;
    const int kw1 = min(2 * (la1 + 1) + R.H, R.K);
    w.shift = (w.kw0 * R.P) & 1;
    w.n16 = (w.shift + (kw1 - w.kw0) * R.P + 1) >> 1;
    w.win = (2 * w.n16 + 1) & ~1;
    w.t0 = max(0, min(la0 + 1, m) - R.c);
    w.t1 = min(min(la1 + 1, m) + R.vb, R.n);
    return w;
}


// Synchronous staging of a window (bands and tables through VGPRs).
template <int Q>
__device__ __forceinline__ void lean_stage(const ScoreRead &R, const LeanWin &w, int tid,
                                           const double *__restrict__ bands, const double *__restrict__ tabs,
                                           const uint8_t *__restrict__ bases, double *sA, double *sB, double *sT)
{
    // plain 16-B loads + ds_write (no LDS-DMA: a global_load_lds anywhere in
    // the kernel makes hipcc wait vmcnt(0) before every LDS read, which would
    // drain the cross-read prefetch at the start of each chain)
    const dvec2 *ga = (const dvec2 *)(bands + R.A + (size_t)w.kw0 * R.P - w.shift);
    const dvec2 *gb = (const dvec2 *)(bands + R.B + (size_t)w.kw0 * R.P - w.shift);
    dvec2 *la = (dvec2 *)sA, *lb = (dvec2 *)sB;
    for (int e0 = 0; e0 < w.n16; e0 += 4 * Q) {
        dvec2 va[4], vb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * Q + tid;
            if (e < w.n16) {
                va[u] = ga[e];
                vb[u] = gb[e];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * Q + tid;
            if (e < w.n16) {
                la[e] = va[u];
                lb[e] = vb[u];
            }
        }
    }
    const int n = R.n;
    const double *tm = tabs + R.tab;
    const uint8_t *sq = bases + R.sb;
    for (int e = tid; e <= w.t1 - w.t0; e += Q) {
        const int i = w.t0 + e;
        const int ks = max(i - 1, 0);
        lean_row(sT + 6 * e, i >= 1 ? sq[i - 1] : 4, tm[ks], tm[n + ks], tm[2 * (size_t)n + ks],
                 tm[3 * (size_t)n + i]);
    }
}

// One new-column chain (lane column a) over the staged window; accumulates
// into the lane's totals.  Row values are software-pipelined one row ahead.
__device__ __forceinline__ void lean_chain(const ScoreRead &R, const LeanWin &w, int a, int m,
                                           const double *sA, const double *sB, const double *sT,
                                           double tI[4], double tS[4], double &tD)
{
    const int c = R.c, vb = R.vb, P = R.P;
    const int jn = min(a + 1, m);
    const int i0 = max(0, jn - c);
    const int i1 = min(jn + vb, R.n);
    const int ilast = min(i1, a + vb);                  // last row of rows(a)
    int d = i0 - a + c;
    int idx = w.shift + (d + 2 * a - w.kw0) * P + (d >> 1);
    double aprev = (d >= 1 && i0 >= 1) ? sA[idx - P - 1 + (d & 1)] : -RF_INF;
    // B(i, a+1) sits at idx + P - 1 + (d & 1); the last column (a = m) has no
    // Substitution(m+1): it reads B(i, a) there and masks the sum to -Inf
    const bool hasS = a < m;
    const int sofs = hasS ? P - 1 : 0;
    const int sodd = hasS ? 1 : 0;
    const double smask = hasS ? 0.0 : -RF_INF;
    const double *tr = sT + 6 * (i0 - w.t0);
    double prev[4], accI[4], accS[4], dd = -RF_INF;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        prev[k] = -RF_INF;
        accI[k] = -RF_INF;
        accS[k] = -RF_INF;
    }
    double ac = sA[idx], bI = sB[idx], bSr = sB[idx + sofs + (sodd & d)];
    double2 u0 = ((const double2 *)tr)[0], u1 = ((const double2 *)tr)[1], u2 = ((const double2 *)tr)[2];
    for (int i = i0; i <= ilast; ++i) {
        // next row's operands (row ilast + 1 is the peeled row below)
        idx += P + (d & 1);
        ++d;
        tr += 6;
        const double acn = sA[idx], bIn = sB[idx], bSn = sB[idx + sofs + (sodd & d)];
        const double2 v0 = ((const double2 *)tr)[0], v1 = ((const double2 *)tr)[1],
                      v2 = ((const double2 *)tr)[2];
        const double bS = bSr + smask;
        const double sub[4] = {u0.x, u0.y, u1.x, u1.y};
        const double dl = ac + u2.y;
        const double dsum = ac + bS;
        chain_row(aprev, sub, u2.x, dl, bI, bS, prev, accI, accS);
        dd = vmax(dd, dsum);
        aprev = ac;
        ac = acn;
        bI = bIn;
        bSr = bSn;
        u0 = v0;
        u1 = v1;
        u2 = v2;
    }
    if (i1 > ilast) {
        // last row of the new column lies below A/B column a's band (a < m)
        const double sub[4] = {u0.x, u0.y, u1.x, u1.y};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            accS[k] = vmax(accS[k], vmax(aprev + sub[k], prev[k] + u2.x) + bSr);
    }
    const double qnan = __builtin_nan("");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        tI[k] += accI[k] == -RF_INF ? qnan : accI[k];
        tS[k] += accS[k] == -RF_INF ? qnan : accS[k];
    }
    tD += dd;
}

// lean_chain for an interior lane of a read with row stride exactly PT (the
// c4 strides 11..17): a < m, a >= c and a + 1 + vb <= n, so the chain runs
// diagonals d = 1 .. H-1 of column a and then the peeled row d = H.  Over two
// rows (d odd, then even) the window index advances by 2 PT + 1, so with the
// stride a template constant every LDS operand of a row pair is at an
// immediate offset from one pointer per array: the per-row index arithmetic
// of lean_chain (about 15 of its 51 VALU ops per row) drops out.  Same
// operands, same FP64 ops in the same order: the same values.
#ifndef WS_UNROLL
#define WS_UNROLL 2   // lean_chain_fix row pairs per loop iteration
#endif
template <int PT>
__device__ __forceinline__ void lean_chain_fix(const ScoreRead &R, const LeanWin &w, int a, const double *sA,
                                               const double *sB, const double *sT, double tI[4], double tS[4],
                                               double &tD)
{
    const int idx0 = w.shift + (1 + 2 * a - w.kw0) * PT;   // d = 1
    const double *pa = sA + idx0, *pb = sB + idx0;
    const double *pt = sT + 6 * (a + 1 - R.c - w.t0);
    double aprev = pa[-PT];
    double prev[4], accI[4], accS[4], dd = -RF_INF;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        prev[k] = -RF_INF;
        accI[k] = -RF_INF;
        accS[k] = -RF_INF;
    }
    // one row: A / B at offset o, B(i, a+1) at offset os, table record at t
    auto row = [&](int o, int os, int t) {
        const double ac = pa[o], bI = pb[o], bS = pb[os];
        const double2 u0 = *(const double2 *)(pt + t), u1 = *(const double2 *)(pt + t + 2),
                      u2 = *(const double2 *)(pt + t + 4);
        const double sub[4] = {u0.x, u0.y, u1.x, u1.y};
        const double dl = ac + u2.y;
        const double dsum = ac + bS;
        chain_row(aprev, sub, u2.x, dl, bI, bS, prev, accI, accS);
        dd = vmax(dd, dsum);
        aprev = ac;
    };
    const int nrows = R.c + R.vb;   // i0 = a + 1 - c .. ilast = a + vb
    // WS_UNROLL row pairs per iteration: hipcc issues an iteration's LDS
    // reads at its top and waits for the first ones at once, so each
    // iteration exposes one LDS round trip; two pairs halve that per row
    int u = 0;
    if (WS_UNROLL > 1) {
        for (; u + WS_UNROLL <= (nrows >> 1); u += WS_UNROLL) {
#pragma unroll
            for (int k = 0; k < WS_UNROLL; ++k) {    // pair k: offsets + k (2 PT + 1)
                const int o = k * (2 * PT + 1);
                row(o, o + PT, 12 * k);                   // d odd
                row(o + PT + 1, o + 2 * PT, 12 * k + 6);  // d even
            }
            pa += WS_UNROLL * (2 * PT + 1);
            pb += WS_UNROLL * (2 * PT + 1);
            pt += 12 * WS_UNROLL;
        }
    }
    for (; u < (nrows >> 1); ++u) {
        row(0, PT, 0);                        // d odd
        row(PT + 1, 2 * PT, 6);               // d even
        pa += 2 * PT + 1;
        pb += 2 * PT + 1;
        pt += 12;
    }
    // the last odd row (H even), then the peeled row d = H below column a's band
    const bool odd_tail = nrows & 1;
    if (odd_tail)
        row(0, PT, 0);
    const double bSr = odd_tail ? pb[2 * PT] : pb[PT];
    const double *tp = pt + (odd_tail ? 6 : 0);
    const double2 u0 = *(const double2 *)tp, u1 = *(const double2 *)(tp + 2), u2 = *(const double2 *)(tp + 4);
    const double sub[4] = {u0.x, u0.y, u1.x, u1.y};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        accS[k] = vmax(accS[k], vmax(aprev + sub[k], prev[k] + u2.x) + bSr);
    const double qnan = __builtin_nan("");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        tI[k] += accI[k] == -RF_INF ? qnan : accI[k];
        tS[k] += accS[k] == -RF_INF ? qnan : accS[k];
    }
    tD += dd;
}

// Whether every chain lane of this wave is interior for read R (lean_chain_fix).
__device__ __forceinline__ bool ws_wave_interior(const ScoreRead &R, int a, int m)
{
    return __all(a < m && a >= R.c && a + 1 + R.vb <= R.n);
}

#ifndef WS_PFIX
#define WS_PFIX 2   // interior waves of reads with stride 11..17 (1) / 11..25 (2) run lean_chain_fix
#endif
// lean_chain, or lean_chain_fix<P> when the wave is interior and P is a c4 stride
__device__ __forceinline__ void lean_chain_any(const ScoreRead &R, const LeanWin &w, int a, int m, const double *sA,
                                               const double *sB, const double *sT, double tI[4], double tS[4],
                                               double &tD)
{
    if (WS_PFIX && ws_wave_interior(R, a, m)) {
        switch (R.P) {
        case 11: lean_chain_fix<11>(R, w, a, sA, sB, sT, tI, tS, tD); return;
        case 13: lean_chain_fix<13>(R, w, a, sA, sB, sT, tI, tS, tD); return;
        case 15: lean_chain_fix<15>(R, w, a, sA, sB, sT, tI, tS, tD); return;
        case 17: lean_chain_fix<17>(R, w, a, sA, sB, sT, tI, tS, tD); return;
#if WS_PFIX > 1
        // doubled bands (bw 18 after smart_forward_moves!, H 37..51)
        case 19: lean_chain_fix<19>(R, w, a, sA, sB, sT, tI, tS, tD); return;
        case 21: lean_chain_fix<21>(R, w, a, sA, sB, sT, tI, tS, tD); return;
        case 23: lean_chain_fix<23>(R, w, a, sA, sB, sT, tI, tS, tD); return;
        case 25: lean_chain_fix<25>(R, w, a, sA, sB, sT, tI, tS, tD); return;
#endif
        default: break;
        }
    }
    lean_chain(R, w, a, m, sA, sB, sT, tI, tS, tD);
}

__device__ __forceinline__ void wg_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---------------------------------------------------------------------
// k_score_ws: the lean scorer with wave specialization (the default)
//
// 512 threads: waves 0-3 are the chain waves (256 chain columns per work
// item, totals in their VGPRs); waves 4-7 are loader waves that hold the
// NEXT read's window and table rows in their own VGPRs while the chain waves
// score the current read from LDS, then write it to LDS between two
// barriers.  The two roles run separate loops (so the loaders' registers
// never constrain the chains) that meet at the same s_barrier sequence:
// two barriers per read, or per sub-pass of a read too wide for the
// prefetch (staged synchronously by the loaders).
// ---------------------------------------------------------------------


#ifndef WS_NPF
#define WS_NPF 19
#endif
#ifndef WS_CODES
#define WS_CODES 1   // loaders read row-coded reads' tables through the code dictionary
#endif

template <int NPF, int Q>
__global__ void __launch_bounds__(2 * Q)
k_score_ws(const WorkItem *__restrict__ items, const ScoreGroup *__restrict__ groups,
           const ScoreRead *__restrict__ reads, const uint8_t *__restrict__ bases,
           const double *__restrict__ tabs, const double *__restrict__ bands,
           double *__restrict__ dense, double *__restrict__ split, int split_mode, int lds_elems,
           const double *__restrict__ lut, int rchunk)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int nb = gridDim.x, b = blockIdx.x;
    const int xq = nb >> 3, xr = nb & 7, x = b & 7;
    const int item = x * xq + min(x, xr) + (b >> 3);
    const WorkItem wi = items[item];
    const ScoreGroup G = groups[wi.group];
    const int m = G.m;
    const int a0 = wi.p0;
    const int la1f = min(a0 + Q - 1, m);
    int r0 = G.r0, r1 = G.r1;
    if (split_mode & 1) {
        // split mode: rchunk consecutive reads per workgroup (round 5: one
        // read per workgroup left a small cluster's launch -- configs[2]'s
        // 1,000 reads x 11 items -- without the loaders' prefetch overlap),
        // each read's own partial written, k_reduce folds them in order
        r0 = G.r0 + blockIdx.y * rchunk;
        if (r0 >= G.r1)
            return;
        r1 = min(r0 + rchunk, G.r1);
    }
    // same decision in both roles (block-uniform)
    auto fast = [&](const ScoreRead &R, const LeanWin &w) {
        return lean_need(Q, R.H, R.P) <= lds_elems && w.n16 <= NPF * Q && w.t1 - w.t0 < 2 * Q;
    };
    auto sub_L = [&](const ScoreRead &R) {
        int L = Q;
        while (L > 1 && lean_need(L, R.H, R.P) > lds_elems)
            L >>= 1;
        return L;
    };
    // Work units: a read whose whole window fits LDS and the loaders'
    // registers is one unit of Q columns; a wider one is split into sub-
    // windows of L columns that fit LDS (sub_L).  Units stream through the
    // same register prefetch as whole reads whenever a unit's window fits the
    // loaders' registers (doubled bands, P 19..25, at L = Q / 2), otherwise
    // they are staged synchronously.  Both roles walk the same sequence.
    struct Unit {
        int r, s0, L;
    };
    auto unit_first = [&](int r) {
        Unit u{r, 0, Q};
        if (r < r1) {
            const ScoreRead R = reads[r];
            if (!fast(R, lean_win(R, m, a0, la1f)))
                u.L = sub_L(R);
        }
        return u;
    };
    auto unit_next = [&](const Unit &u) {
        const int s0 = u.s0 + u.L;
        if (s0 < Q && a0 + s0 <= m)
            return Unit{u.r, s0, u.L};
        return unit_first(u.r + 1);
    };
    auto unit_win = [&](const ScoreRead &R, const Unit &u) {
        return lean_win(R, m, a0 + u.s0, min(a0 + u.s0 + u.L - 1, m));
    };
    auto unit_pf = [&](const ScoreRead &R, const Unit &u, const LeanWin &w) {   // register-prefetched
        return lean_need(u.L, R.H, R.P) <= lds_elems && w.n16 <= NPF * Q && w.t1 - w.t0 < 2 * Q;
    };
    if (threadIdx.x >= Q) {
        // =========================== loader waves ===========================
        const int lt = threadIdx.x - Q;
        dvec2 pa[NPF], pb[NPF];
        double pm[2], px[2], pn[2], pd[2];
        int ps[2];
        auto issue = [&](const ScoreRead &R2, const LeanWin &w2) {
            const double *tm = tabs + R2.tab;
            const int n2 = R2.n;
            // Row-coded reads (SR_CODED): one 8-B code record per row from HBM
            // (issued first, so that the wait for them leaves the band loads in
            // flight) and the values from the context's L2-resident dictionary
            // -- the same doubles as the tables (rf_set_sequences), 8 instead of
            // 33 B per row.  Record of position ks: triple code | del[ks] code
            // << 16 | del[ks+1] code << 32 | base << 48.
            const bool coded = (R2.flags & SR_CODED) && lut != nullptr;
            uint64_t rc[2];
            if (coded) {
                const uint64_t *rec = (const uint64_t *)(tm + row_code_off(n2, 0, 0));
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = min(w2.t0 + lt + k * Q, w2.t1);
                    rc[k] = rec[max(i - 1, 0)];
                }
            }
            const dvec2 *ga = (const dvec2 *)(bands + R2.A + (size_t)w2.kw0 * R2.P - w2.shift);
            const dvec2 *gb = (const dvec2 *)(bands + R2.B + (size_t)w2.kw0 * R2.P - w2.shift);
#pragma unroll
            for (int u = 0; u < NPF; ++u) {
                // predicated: chunks past the window are neither loaded nor
                // committed (the commit's `e < n16` test)
                const int e = u * Q + lt;
                if (e < w2.n16) {
                    pa[u] = ga[e];
                    pb[u] = gb[e];
                }
            }
            if (coded) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = min(w2.t0 + lt + k * Q, w2.t1);
                    const double *l3 = lut + 4 * (size_t)(rc[k] & 0xffff);
                    pm[k] = l3[0];
                    px[k] = l3[1];
                    pn[k] = l3[2];
                    pd[k] = lut[4 * (size_t)RF_CODES + ((rc[k] >> (i == 0 ? 16 : 32)) & 0xffff)];
                    ps[k] = (int)((rc[k] >> 48) & 0xff);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = min(w2.t0 + lt + k * Q, w2.t1);
                    const int ks = max(i - 1, 0);
                    pm[k] = tm[ks];
                    px[k] = tm[n2 + ks];
                    pn[k] = tm[2 * (size_t)n2 + ks];
                    pd[k] = tm[3 * (size_t)n2 + i];
                    ps[k] = bases[R2.sb + ks];
                }
            }
        };
        bool held = false;   // the registers hold the unit
        for (Unit u = unit_first(r0); u.r < r1;) {
            const ScoreRead R = reads[u.r];
            const LeanWin w = unit_win(R, u);
            const Unit nx = unit_next(u);
            if (unit_pf(R, u, w)) {
                if (!held)
                    issue(R, w);
                dvec2 *sA = (dvec2 *)smem;
                dvec2 *sB = (dvec2 *)(smem + w.win);
                double *sT = smem + 2 * w.win;
#pragma unroll
                for (int k = 0; k < NPF; ++k) {
                    const int e = k * Q + lt;
                    if (e < w.n16) {
                        sA[e] = pa[k];
                        sB[e] = pb[k];
                    }
                }
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int e = lt + k * Q;
                    const int i = w.t0 + e;
                    if (i <= w.t1)
                        lean_row(sT + 6 * e, i >= 1 ? ps[k] : 4, pm[k], px[k], pn[k], pd[k]);
                }
                wg_barrier();                        // unit ready
                held = false;
                if (nx.r < r1) {
                    const ScoreRead R2 = reads[nx.r];
                    const LeanWin w2 = unit_win(R2, nx);
                    if (unit_pf(R2, nx, w2)) {
                        issue(R2, w2);
                        held = true;
                    }
                }
                wg_barrier();                        // chains of the unit done
            } else {
                lean_stage<Q>(R, w, lt, bands, tabs, bases, smem, smem + w.win, smem + 2 * w.win);
                wg_barrier();
                wg_barrier();
                held = false;
            }
            u = nx;
        }
        return;
    }
    // ============================ chain waves =============================
    const int tid = threadIdx.x;
    const int a = a0 + tid;
    double tI[4], tS[4], tD = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        tI[k] = 0.0;
        tS[k] = 0.0;
    }
    const double qnan = __builtin_nan("");
    // one position's 9 totals (fused: the group's fold; split: read r's
    // partial, 0.0 + its own sums, and the running values restart at 0.0)
    auto emit = [&](double *base) {
        double *dst = base + (size_t)a * 9;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            dst[5 + k] = tI[k];
        if (a < m) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                dst[9 + k] = tS[k];
            dst[13] = tD;
        }
        if (a == 0) {
#pragma unroll
            for (int k = 0; k < 5; ++k)
                dst[k] = qnan;
        }
    };
    for (Unit u = unit_first(r0); u.r < r1;) {
        const ScoreRead R = reads[u.r];
        const LeanWin w = unit_win(R, u);
        wg_barrier();                                // unit ready
        if (tid >= u.s0 && tid < u.s0 + u.L && a <= m)
            lean_chain_any(R, w, a, m, smem, smem + w.win, smem + 2 * w.win, tI, tS, tD);
        wg_barrier();                                // chains of the unit done
        const Unit nx = unit_next(u);
        if ((split_mode & 1) && nx.r != u.r && a <= m) {
            emit(split + G.split_off + (size_t)(u.r - G.r0) * (m + 1) * 9);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                tI[k] = 0.0;
                tS[k] = 0.0;
            }
            tD = 0.0;
        }
        u = nx;
    }
    if (a > m || (split_mode & 1))
        return;
    emit(dense + G.dense_off);
}

// ---------------------------------------------------------------------
// k_score_segl: the wide-band scorer over line-aligned band rows (default)
//
// Same chains, operands, order and FP64 max-plus as k_score_ws's lean_chain
// (identical results).  Segments are 32 band diagonals [D, D+32) with D a
// multiple of 32, so a kappa row's piece of a segment is elements
// [D/2, D/2 + 16): exactly one 128-B line when the band's rows are padded to
// whole lines (band_stride, P % 16 == 0; band regions are 256-B aligned) --
// no line is shared by two segments, so each is fetched once.  Bands with the
// odd stride (H below RF_OPT_BAND_PAD) take 9 pair-aligned 16-B chunks per
// row instead.  The wave's 65 columns [a0, a0+64] touch kappa rows
// [D + 2*a0, D + 2*a0 + 160).
//
// LDS holds the segment transposed: slot (d - D + 1) * 65 + (a - a0) for
// d in [D-1, D+32) (row 0 is the previous segment's last diagonal), so lane
// a's operands at step d -- A(d, a), B(d, a), B(d-1, a+1) -- are one
// consecutive 512-B run per wave-instruction at an immediate offset, and the
// table records of read row i = a - c + d (three 16-B arrays) likewise.
// The next segment's lines are loaded into registers while this one is
// scored.
// ---------------------------------------------------------------------
#ifndef SEGL_UNROLL
#define SEGL_UNROLL 32
#endif
// an interior wave's last segment runs the unrolled steps over rows staged as
// -Inf past the peel row when it holds at least this many rows (fewer: the
// generic loop, which costs more per step but runs only the real rows)
#ifndef SEGL_MASKED_MIN
#define SEGL_MASKED_MIN 20
#endif
#define SEGL_FENCE() __builtin_amdgcn_sched_barrier(0)
// A kappa row's piece of a segment is one 128-B line.  (Half-line segments
// of 16 diagonals -- 55 % of the LDS, two waves per SIMD -- were bit-exact but
// slower at c5: 30.6 ms at one wave per SIMD, 40.6 ms at two with spills,
// against 27.9 ms; profiles/r02_exp_segl16.json.)
template <int S_>
struct SeglGeo {
    static_assert(S_ == 32, "segments of 32 diagonals");
    static constexpr int S = S_;        // diagonals per segment
    static constexpr int LS = 65;       // LDS row: columns a0 .. a0+64
    static constexpr int NRW = S + 1;   // LDS rows: d = D-1 .. D+S-1
    static constexpr int NROW = S + 128;   // kappa rows per segment
    static constexpr int CPR = S / 4;      // 16-B chunks of a row piece (S/2 doubles), aligned rows
    static constexpr int RPI = 64 / CPR;   // rows per wave-wide load
    static constexpr int NUA = NROW * CPR / 64;          // chunks per lane and band, aligned rows
    static constexpr int NC = CPR + 1;                   // pair-aligned chunks per row, odd stride
    static constexpr int NUG = (NROW * NC + 63) / 64;
    static constexpr int NT = S + 65;   // table rows: i - ib in [0, S + 65)
};

template <int SEGS>
#ifndef SEGL_WPE
#define SEGL_WPE 1
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SEGL_WPE)))
k_score_segl(const WorkItem *__restrict__ items, const ScoreGroup *__restrict__ groups,
             const ScoreRead *__restrict__ reads, const uint8_t *__restrict__ bases,
             const double *__restrict__ tabs, const double *__restrict__ bands,
             double *__restrict__ dense, double *__restrict__ split, int split_mode, int rchunk)
{
    using Gm = SeglGeo<SEGS>;
    constexpr int S = Gm::S, LS = Gm::LS, NUA = Gm::NUA, NUG = Gm::NUG, NT = Gm::NT;
    constexpr int CPR = Gm::CPR, RPI = Gm::RPI, NC = Gm::NC;

    constexpr int SL = (Gm::NRW * LS + 1) & ~1;   // doubles per band slice (16-B multiple)
    __shared__ __attribute__((aligned(16))) double sA[SL];
    __shared__ __attribute__((aligned(16))) double sB[SL];
    __shared__ __attribute__((aligned(16))) dvec2 sT0[NT], sT1[NT], sT2[NT];
    const int nx = gridDim.x;
    const int lin = blockIdx.x + nx * blockIdx.y, ncell = nx * gridDim.y;
    const int xq = ncell >> 3, xr = ncell & 7, x = lin & 7;
    const int cell = x * xq + min(x, xr) + (lin >> 3);
    const int bx = cell % nx, by = cell / nx;
    const WorkItem wi = items[bx];
    const ScoreGroup G = groups[wi.group];
    const int m = G.m;
    const int a0 = wi.p0;
    const int tid = threadIdx.x;
    const int a = a0 + tid;
    const bool active = a <= m;
    int r0 = G.r0, r1 = G.r1;
    if (split_mode & 1) {
        r0 = G.r0 + by * rchunk;
        if (r0 >= G.r1)
            return;
        r1 = min(r0 + rchunk, G.r1);
    }
    const bool hasS = a < m;
    const double smask = hasS ? 0.0 : -RF_INF;
    const bool wave_s = __all(hasS);   // every lane has a Substitution column
    double tI[4], tS[4], tD = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        tI[k] = 0.0;
        tS[k] = 0.0;
    }
    const bool all_act = __all(active) && wave_s;
    // aligned-row loader lane roles: row r8 + RPI j, 16-B chunk cc8 of the row piece
    const int r8 = tid / CPR, cc8 = tid % CPR, p8 = r8 & 1;
    // per-read geometry: wave-uniform fields plus the lane's diagonal range
    struct RG {
        const double *gA;
        const double *tm;
        const uint8_t *sq;
        int64_t dB;
        int c, P, K, n;
        int dfirst, dlast;           // this lane's chain rows as band diagonals
        bool peel;
        int dlo, dhi, dfmax, dlmin;  // wave-wide
        bool uni;                    // every lane active with the same [dfirst, dlast] and peel
    };
    auto setup = [&](int r, RG &g) {
        const ScoreRead R = reads[r];
        g.c = R.c;
        g.P = R.P;
        g.K = R.K;
        g.n = R.n;
        g.gA = bands + R.A;
        g.dB = R.B - R.A;
        g.tm = tabs + R.tab;
        g.sq = bases + R.sb;
        const int jn = min(a + 1, m);
        const int i0 = max(0, jn - g.c);
        const int i1 = min(jn + R.vb, g.n);
        const int ilast = min(i1, a + R.vb);
        g.dfirst = i0 - a + g.c;
        g.dlast = ilast - a + g.c;
        g.peel = i1 > ilast;
        int dlo = active ? g.dfirst : INT_MAX, dhi = active ? g.dlast + (g.peel ? 1 : 0) : -1;
        int dfmax = active ? g.dfirst : INT_MAX, dlmin = active ? g.dlast : -1;
        for (int off = 32; off >= 1; off >>= 1) {
            dlo = min(dlo, __shfl_xor(dlo, off));
            dhi = max(dhi, __shfl_xor(dhi, off));
            dfmax = max(dfmax, __shfl_xor(dfmax, off));
            dlmin = min(dlmin, __shfl_xor(dlmin, off));
        }
        g.dlo = __builtin_amdgcn_readfirstlane(dlo);
        g.dhi = __builtin_amdgcn_readfirstlane(dhi);
        g.dfmax = __builtin_amdgcn_readfirstlane(dfmax);
        g.dlmin = __builtin_amdgcn_readfirstlane(dlmin);
        // interior waves: every lane has the same chain rows [dfirst, dlast]
        // and a peel row dlast + 1 (uniform), so the first and last segments
        // of the read can run the unrolled steps too (see chains)
        g.uni = all_act && __all(g.dfirst == g.dlo && g.dlast == g.dlmin && g.peel);
    };
    // one segment's registers: its band lines, table rows and (a read's
    // first segment) LDS row 0
    struct SegSet {
        dvec2 ra[NUA], rb[NUA];
        double tmt[2], tmm[2], tin[2], tdl[2];
        int tsb[2];
        double z0a, z0b, z1a, z1b;
    };
    // loads of segment D of read g (registers only)
    auto load_seg = [&](SegSet &X, const RG &g, int D, bool first) {
        const int kb = D + 2 * a0, eh = D >> 1;
        if ((g.P & 15) == 0) {
#pragma unroll
            for (int j = 0; j < NUA; ++j) {
                const int kap = min(kb + r8 + RPI * j, g.K - 1);
                const int64_t o = (int64_t)kap * g.P + eh + 2 * cc8;
                X.ra[j] = *(const dvec2 *)(g.gA + o);
                X.rb[j] = *(const dvec2 *)(g.gA + g.dB + o);
            }
        }
        if (first && D > 0) {
            // diagonal D-1 of columns a0 .. a0+64 (the previous segment's last row)
            const int kap = min(D - 1 + 2 * a, g.K - 1);
            const int64_t o = (int64_t)kap * g.P + ((D - 1) >> 1);
            X.z0a = g.gA[o];
            X.z0b = g.gA[g.dB + o];
            if (tid == 0) {
                const int kap1 = min(D - 1 + 2 * (a0 + 64), g.K - 1);
                const int64_t o1 = (int64_t)kap1 * g.P + ((D - 1) >> 1);
                X.z1a = g.gA[o1];
                X.z1b = g.gA[g.dB + o1];
            }
        }
        const int ib = a0 - g.c + D;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = min(max(ib + tid + 64 * u, 0), g.n);
            const int ks = max(i - 1, 0);
            X.tsb[u] = g.sq[ks];   // read row 0 (the gap) is selected at the store
            X.tmt[u] = g.tm[ks];
            X.tmm[u] = g.tm[g.n + ks];
            X.tin[u] = g.tm[2 * (size_t)g.n + ks];
            X.tdl[u] = g.tm[3 * (size_t)g.n + i];
        }
    };
    auto store_seg = [&](const SegSet &X, const RG &g, int D) {
        if ((g.P & 15) == 0) {
            // an interior wave's last segment: rows past the peel row (d >
            // dlast + 1 in A, d > dlast in B beyond column a) read -Inf, so the
            // unrolled steps past the chain's end leave it unchanged (chains)
            const int dm = (g.uni && D > 0 && g.dlmin + 1 < D + S && g.dlmin + 1 - D >= SEGL_MASKED_MIN)
                               ? g.dlmin + 1 - D : INT_MAX;
#pragma unroll
            for (int j = 0; j < NUA; ++j) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int ddl = 4 * cc8 + 2 * h + p8;       // d - D
                    const int col = (r8 + RPI * j - ddl) >> 1;  // a - a0
                    const double v = h ? X.ra[j].y : X.ra[j].x, w = h ? X.rb[j].y : X.rb[j].x;
                    const int l = (ddl + 1) * LS + col;
                    // rows S..127 always land in [0, 64]; the parallelogram's
                    // first / last S rows hold cells of the neighbouring items
                    if ((j * RPI >= S && (j + 1) * RPI <= 128) || (col >= 0 && col <= 64)) {
                        sA[l] = v;
                        sB[l] = w;
                    }
                }
            }
            if (dm != INT_MAX) {
                // LDS rows dm + 1 .. S (diagonals D + dm ..) of both bands: -Inf
                for (int e = tid; e < (S - dm) * LS; e += 64) {
                    const int l = (dm + 1) * LS + e;
                    sA[l] = -RF_INF;
                    sB[l] = -RF_INF;
                }
            }
        } else {
            // odd-stride rows (narrow bands in a wide launch): NC pair-aligned
            // chunks per row, loaded here in groups of 4 (not prefetched)
            const int kb = D + 2 * a0, eh = D >> 1;
#pragma unroll 1
            for (int j0 = 0; j0 < NUG; j0 += 4) {
                dvec2 ga[4], gb[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int t = min(tid + 64 * (j0 + jj), Gm::NROW * NC - 1);
                    const int rr = t / NC, cc = t - NC * rr;
                    const int kap = min(kb + rr, g.K - 1);
                    const int o = ((kap * g.P + eh) & ~1) + 2 * cc;
                    ga[jj] = *(const dvec2 *)(g.gA + o);
                    gb[jj] = *(const dvec2 *)(g.gA + g.dB + o);
                }
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int t = tid + 64 * (j0 + jj);
                    const int rr = t / NC, cc = t - NC * rr;
                    const int sh = (kb + rr + eh) & 1;   // P odd
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int xl = 2 * cc + h - sh;
                        const int ddl = 2 * xl + (rr & 1);
                        const int col = (rr - ddl) >> 1;
                        if (t < Gm::NROW * NC && xl >= 0 && xl < S / 2 && col >= 0 && col <= 64) {
                            const int l = (ddl + 1) * LS + col;
                            sA[l] = h ? ga[jj].y : ga[jj].x;
                            sB[l] = h ? gb[jj].y : gb[jj].x;
                        }
                    }
                }
            }
            // nothing of this path stays in flight: hipcc's wait analysis
            // merges paths, and a load it saw pending here would make it
            // drain the next segment's prefetch before the chains
            __builtin_amdgcn_s_waitcnt(0);
        }
        const int ib = a0 - g.c + D;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int t = tid + 64 * u;
            if (t < NT) {
                const int sb = ib + t >= 1 ? X.tsb[u] : 4;
                const double mt = X.tmt[u], mm = X.tmm[u];
                sT0[t] = dvec2{sb == 0 ? mt : mm, sb == 1 ? mt : mm};
                sT1[t] = dvec2{sb == 2 ? mt : mm, sb == 3 ? mt : mm};
                sT2[t] = dvec2{X.tin[u], X.tdl[u]};
            }
        }
    };
    // a wave with no column (every a > m) writes nothing; any other wave has
    // rows in every read (each band column holds at least one row)
    if (!__any(active))
        return;
    double prev[4], accI[4], accS[4], dd = -RF_INF;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        prev[k] = -RF_INF;
        accI[k] = -RF_INF;
        accS[k] = -RF_INF;
    }
    // the chains of segment D of read g (operands from LDS)
    auto chains = [&](const RG &g, int D) {
        const int c = g.c, dfirst = g.dfirst, dlast = g.dlast;
        const int dfmax = g.dfmax, dlmin = g.dlmin;
        const bool peel = g.peel;
        if (active) {
            const int lo = max(D, dfirst), hi = min(D + S - 1, dlast);
            const double a0v = sA[min(max(lo - D, 0), S) * LS + tid];   // unconditional read, then select
            double aprev = (lo <= hi && lo >= 1 && a - c + lo >= 1) ? a0v : -RF_INF;
            const double *pA = sA + LS + tid;    // row 1 = diagonal D
            const double *pB = sB + LS + tid;
            const double *pS = sB + tid + 1;     // B(d-1, a+1): row d - D, column + 1
            const dvec2 *q0 = sT0 + tid, *q1 = sT1 + tid, *q2 = sT2 + tid;
            // operands of step s; the next step's are read from LDS while this
            // one is scored (software pipeline: a read right before its use
            // exposes the LDS latency on every step at one wave per SIMD)
            struct Ops {
                double ac, bI, bs;
                dvec2 u0, u1, u2;
            };
            auto ld = [&](int s) {
                Ops o;
                o.ac = pA[s * LS];
                o.bI = pB[s * LS];
                o.bs = pS[s * LS];   // in range for every lane
                o.u0 = q0[s];
                o.u1 = q1[s];
                o.u2 = q2[s];
                return o;
            };
            // ALLS: every lane has a Substitution column (hasS; smask = 0)
            auto step = [&](const Ops &o, auto alls) {
                const double bS = ((decltype(alls)::value || hasS) ? o.bs : o.bI) + smask;
                const double sub[4] = {o.u0.x, o.u0.y, o.u1.x, o.u1.y};
                const double dl = o.ac + o.u2.y;
                const double dsum = o.ac + bS;
                chain_row(aprev, sub, o.u2.x, dl, o.bI, bS, prev, accI, accS);
                dd = vmax(dd, dsum);
                aprev = o.ac;
            };
            // unrolled steps s0 .. shi (wave-uniform) of the segment; s0 = 0 or 1
            // the unrolled steps 0 .. S-1 (one copy of the body: instruction
            // cache); skip0 -- a read's first segment in an interior wave,
            // whose chains start at diagonal 1 -- only takes row 0 as the next
            // step's MATCH predecessor (a scalar branch on the first step)
            auto run = [&](bool skip0) {
                Ops cur = ld(0);
#pragma unroll SEGL_UNROLL
                for (int s = 0; s < S; ++s) {
                    const Ops nxt = ld(s + 1 < S ? s + 1 : s);
                    // keep the reads ahead of this step's chain (hipcc's scheduler
                    // otherwise sinks them next to their use); the arithmetic may
                    // still move across (a full sched_barrier costs hazard nops)
                    SEGL_FENCE();
                    if (s == 0 && skip0)
                        aprev = a - c >= 0 ? cur.ac : -RF_INF;   // diagonal 0: read row a - c
                    else
                        step(cur, std::true_type{});
                    cur = nxt;
                }
            };
            // every lane scores all 32 diagonals (no peel inside: dlast >= D+31);
            // all_act includes wave_s, so the bS select is the identity
            const bool full = all_act && dfmax <= D && dlmin >= D + S - 1;
            // interior wave, first segment of the read (round 4): every lane's
            // chain covers diagonals 1 .. S-1 of it
            const bool first_u = g.uni && D == 0 && dfirst == 1 && dlast + 1 >= S && (g.P & 15) == 0;
            // interior wave, last segment with at least SEGL_MASKED_MIN rows
            // (round 4): the rows past the peel row were stored as -Inf
            // (store_seg), so all S unrolled steps give the chain's rows up to
            // dlast, then the peel row dlast + 1 exactly as below (max(x, -Inf)
            // = x; B(dlast, a + 1) is the peel's operand), and leave the state
            // unchanged afterwards
            const bool last_u = g.uni && D > 0 && dlast + 1 < D + S && dlast + 1 - D >= SEGL_MASKED_MIN &&
                                (g.P & 15) == 0;
            if (full || first_u || last_u) {
                run(__builtin_amdgcn_readfirstlane((int)first_u) != 0);   // one call site: one body
            } else {
                const int slo = max(lo - D, 0), shi = hi - D;
                if (slo <= shi) {
                    Ops cur = ld(slo);
                    for (int s = slo; s <= shi; ++s) {
                        const Ops nxt = ld(s < shi ? s + 1 : s);
                        SEGL_FENCE();
                        step(cur, std::false_type{});
                        cur = nxt;
                    }
                }
                const int dp = dlast + 1;
                if (peel && dp >= D && dp < D + S) {
                    // last row of the new column lies below A/B column a's band (a < m)
                    const int sp = dp - D;
                    const double ap = sA[sp * LS + tid];
                    const double bSr = sB[sp * LS + tid + 1];
                    const dvec2 u0 = sT0[tid + sp], u1 = sT1[tid + sp], u2 = sT2[tid + sp];
                    const double sub[4] = {u0.x, u0.y, u1.x, u1.y};
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        accS[k] = vmax(accS[k], vmax(ap + sub[k], prev[k] + u2.x) + bSr);
                }
            }
        }
    };
    // read r's totals (after its last segment) and fresh chain state
    auto finish = [&](int r) {
        if (active) {
            const double qnan = __builtin_nan("");
            if (split_mode & 1) {
                double *dst = split + G.split_off + ((size_t)(r - G.r0) * (m + 1) + a) * 9;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    dst[5 + k] = accI[k] == -RF_INF ? qnan : accI[k];
                if (a < m) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        dst[9 + k] = accS[k] == -RF_INF ? qnan : accS[k];
                    dst[13] = dd;
                }
                if (a == 0) {
#pragma unroll
                    for (int k = 0; k < 5; ++k)
                        dst[k] = qnan;
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    tI[k] += accI[k] == -RF_INF ? qnan : accI[k];
                    tS[k] += accS[k] == -RF_INF ? qnan : accS[k];
                }
                tD += dd;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            prev[k] = -RF_INF;
            accI[k] = -RF_INF;
            accS[k] = -RF_INF;
        }
        dd = -RF_INF;
    };
    // Reads and their segments as one stream: the register prefetch always
    // holds the next segment(s) -- this read's next, or the next read's
    // first -- so no read starts on an exposed load.
    struct Pos {
        int r, D;
        RG g;
    };
    auto first_of = [&](const RG &g) { return g.dlo & ~(S - 1); };
    auto adv = [&](Pos &p) {
        if (p.D + S > p.g.dhi) {
            ++p.r;
            if (p.r < r1) {
                setup(p.r, p.g);
                p.D = first_of(p.g);
            }
        } else {
            p.D += S;
        }
    };
    // one segment: X holds its loads; afterwards X holds the next segment's
    auto step = [&](SegSet &X, Pos &cur) {
        const int D = cur.D;
        const bool first = D == first_of(cur.g);
        wave_sync();   // previous segment's chains are done with LDS
        // LDS row 0 = diagonal D-1: the previous segment's row 32, or prefetched
        if (first) {
            if (D > 0) {
                sA[tid] = X.z0a;
                sB[tid] = X.z0b;
                if (tid == 0) {
                    sA[64] = X.z1a;
                    sB[64] = X.z1b;
                }
            }
        } else {
            const double va = sA[S * LS + tid], vbv = sB[S * LS + tid];
            const double va6 = sA[S * LS + 64], vb6 = sB[S * LS + 64];
            sA[tid] = va;
            sB[tid] = vbv;
            if (tid == 0) {
                sA[64] = va6;
                sB[64] = vb6;
            }
        }
        store_seg(X, cur.g, D);
        wave_sync();
        Pos ahead = cur;
        if (ahead.r < r1)
            adv(ahead);
        if (ahead.r < r1)
            load_seg(X, ahead.g, ahead.D, ahead.D == first_of(ahead.g));
        chains(cur.g, D);
        if (D + S > cur.g.dhi)
            finish(cur.r);
        cur = ahead;
    };
    Pos cur;
    cur.r = r0;
    if (r0 < r1) {
        setup(r0, cur.g);
        cur.D = first_of(cur.g);
    }
    SegSet X0;
    if (r0 < r1)
        load_seg(X0, cur.g, cur.D, true);
    while (cur.r < r1)
        step(X0, cur);
    if (!active || (split_mode & 1))
        return;
    const double qnan = __builtin_nan("");
    double *dst = dense + G.dense_off + (size_t)a * 9;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        dst[5 + k] = tI[k];
    if (a < m) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            dst[9 + k] = tS[k];
        dst[13] = tD;
    }
    if (a == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k)
            dst[k] = qnan;
    }
}

// ---------------------------------------------------------------------
// k_codon: codon-move scoring, one lane per proposal (model.jl:302-383)
// ---------------------------------------------------------------------

struct Geo {
    int n, m, bw, H, P, c;
    __device__ __forceinline__ bool inband(int ii, int jj) const
    {
        // 0-based cell (ii, jj) of an (n+1) x (m+1) band (bandedarrays.jl:151-157)
        if (ii < 0 || jj < 0 || ii > n || jj > m)
            return false;
        const int d = ii - jj + c;
        return d >= 0 && d < H;
    }
    __device__ __forceinline__ double get(const double *band, int ii, int jj) const
    {
        return band[bidx(ii - jj + c, jj, P)];
    }
    __device__ __forceinline__ void rows(int jj, int &a, int &b) const
    {
        a = max(0, jj - max(m - n, 0) - bw);
        b = min(jj + max(n - m, 0) + bw, n);
    }
};

// align.jl:50-112 with newcols / acol (1-based i, j like the reference)
__device__ bool update_nc(const Geo &g, const double *A, const double *nc, int ncld, int acol,
                          int i, int j, int s_base, int t_base, const double *tb, int ncins,
                          int ncdel, double &out)
{
    const int n = g.n, ncols = g.m + 1;
    const int seq_i = max(i - 1, 1);
    const int del_i = i;
    const double ms = (s_base == t_base) ? tb[seq_i - 1] : tb[n + seq_i - 1];
    const double is = tb[2 * n + seq_i - 1];
    const double ds = tb[3 * n + del_i - 1];
    const double *t_cins = tb + 4 * n + 1;
    const double *t_cdel = t_cins + ncins;
    double best = -RF_INF;
    int mv = 0;
    auto helper = [&](double msc, int move, int a, int b) {
        const int pi = i - a, pj = j - b;
        const int rc = min(pj, ncols);
        if (g.inband(pi - 1, rc - 1)) {
            const double v = (acol < 1 || pj <= acol) ? g.get(A, pi - 1, pj - 1)
                                                      : nc[(size_t)(pi - 1) + (size_t)ncld * (pj - acol - 1)];
            const double sc = v + msc;
            if (sc > best) {
                best = sc;
                mv = move;
            }
        }
    };
    helper(ms, 1, 1, 1);
    helper(is, 2, 1, 0);
    helper(ds, 3, 0, 1);
    if (ncins > 0 || ncdel > 0) {
        if (ncins > 0 && i > 3)
            helper(t_cins[i - 3 - 1], 4, 3, 0);
        if (ncdel > 0 && j > 3)
            helper(t_cdel[del_i - 1], 5, 0, 3);
    }
    out = best;
    return best != -RF_INF && mv != 0;
}

// equal_ranges((imn,imx), row_range(B, bj)) then summax (1-based rows);
// acolvals indexed by absolute 1-based row
__device__ double summax_nc(const Geo &g, const double *acolvals, int imn, int imx,
                            const double *B, int bj)
{
    int bs, be;
    g.rows(bj - 1, bs, be);
    bs += 1;
    be += 1;
    const int lo = max(imn, bs), hi = min(imx, be);
    double r = -RF_INF;
    for (int i = lo; i <= hi; ++i) {
        const double x = acolvals[i - 1] + g.get(B, i - 1, bj - 1);
        r = (i == lo) ? x : fmax(r, x);
    }
    return r;
}

__global__ void k_codon(const CodonTask *__restrict__ tasks, int ntasks,
                        const uint8_t *__restrict__ bases, const double *__restrict__ tabs,
                        const double *__restrict__ bands, double *__restrict__ scratch,
                        double *__restrict__ out)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntasks)
        return;
    const CodonTask T = tasks[t];
    const double qnan = __builtin_nan("");
    const double *A = bands + T.A;
    const double *B = bands + T.B;
    const uint8_t *s = bases + T.sb;
    const uint8_t *cons = bases + T.tb;
    const double *tb = tabs + T.tab;
    double *nc = scratch + T.scratch;
    Geo g;
    g.n = T.n;
    g.m = T.m;
    g.bw = T.bw;
    g.H = T.H;
    g.P = T.P;
    g.c = max(T.m - T.n, 0) + T.bw;
    const int n = T.n, m = T.m;
    const int nrows = n + 1, ncols = m + 1;
    const int kind = T.kind, pos = T.pos;

    if (T.ncins == 0 && T.ncdel == 0) {
        // score_nocodon on a single sequence (model.jl:242-285)
        double result = qnan;
        if (kind == 2) {
            // seq_score_deletion: summax(A col pos, B col pos+1) (model.jl:227-236)
            int as, ae, bs, be;
            g.rows(pos - 1, as, ae);
            g.rows(pos, bs, be);
            const int lo = max(as, bs), hi = min(ae, be);
            double r = -RF_INF;
            for (int i = lo; i <= hi; ++i) {
                const double x = g.get(A, i, pos - 1) + g.get(B, i, pos);
                r = (i == lo) ? x : fmax(r, x);
            }
            result = r;
        } else {
            const int acol = pos + (kind == 0 ? 0 : 1);
            const int new_acol = acol + 1;
            int amin, amax;
            g.rows(min(new_acol, ncols) - 1, amin, amax);
            amin += 1;
            amax += 1;
            bool ok = true;
            for (int i = amin; i <= amax && ok; ++i) {
                const int sb = i > 1 ? s[i - 2] : 4;
                double v;
                ok = update_nc(g, A, nc, nrows, acol, i, new_acol, sb, T.base, tb, 0, 0, v);
                nc[i - 1] = v;
            }
            if (ok) {
                const double sc = summax_nc(g, nc, amin, amax, B, pos + 1);
                result = (sc == -RF_INF) ? qnan : sc;
            }
        }
        out[T.out_idx] = result;
        return;
    }

    // codon path (model.jl:310-383)
    const int acol = pos + (kind == 1 ? 0 : -1) + 1;
    const int first_bcol = acol + (kind == 1 ? 1 : 2);
    const int last_bcol = first_bcol + 2;
    if (kind == 2 && acol == ncols - 1) {
        out[T.out_idx] = g.get(A, nrows - 1, ncols - 2);
        return;
    }
    const bool just_a = last_bcol >= ncols;
    const int n_after = !just_a ? 3 : m - pos;
    const int n_new_bases = kind == 2 ? 0 : 1;
    if (n_new_bases == 0 && n_after == 0) {
        out[T.out_idx] = qnan;
        return;
    }
    const int n_new = n_new_bases + n_after;
    int sub[8];
    int nsub = 0;
    if (kind != 2)
        sub[nsub++] = T.base;
    const int stop = min(pos + 1 + n_after - 1, m);
    for (int k = pos + 1; k <= stop && nsub < 8; ++k)
        sub[nsub++] = cons[k - 1];
    if (nsub < n_new) {
        out[T.out_idx] = qnan;
        return;
    }
    bool ok = true;
    for (int j = 1; j <= n_new && ok; ++j) {
        const int range_col = min(acol + j, ncols);
        int amin, amax;
        g.rows(range_col - 1, amin, amax);
        amin += 1;
        amax += 1;
        for (int i = amin; i <= amax && ok; ++i) {
            const int sb = i > 1 ? s[i - 2] : 4;
            double v;
            ok = update_nc(g, A, nc, nrows, acol, i, acol + j, sb, sub[j - 1], tb, T.ncins,
                           T.ncdel, v);
            nc[(size_t)(i - 1) + (size_t)nrows * (j - 1)] = v;
        }
    }
    if (!ok) {
        out[T.out_idx] = qnan;
        return;
    }
    if (just_a) {
        out[T.out_idx] = nc[(size_t)(nrows - 1) + (size_t)nrows * (n_new - 1)];
        return;
    }
    double best = -RF_INF;
    for (int j = 1; j <= 3; ++j) {
        const int new_j = n_new - 3 + j;
        int imn, imx;
        g.rows(min(acol + new_j, ncols) - 1, imn, imx);
        imn += 1;
        imx += 1;
        const int bj = first_bcol + j - 1;
        if (bj > ncols) {
            best = qnan;
            break;
        }
        const double sc = summax_nc(g, nc + (size_t)nrows * (new_j - 1), imn, imx, B, bj);
        if (sc > best)
            best = sc;
    }
    out[T.out_idx] = (best == -RF_INF) ? qnan : best;
}

// totals for the proposal list: reads fold (dense) + reference score last
__global__ void k_gather(int64_t nprops, const int32_t *__restrict__ pgroup,
                         const uint8_t *__restrict__ kind, const int32_t *__restrict__ pos,
                         const uint8_t *__restrict__ base, const ScoreGroup *__restrict__ groups,
                         const int32_t *__restrict__ has_reads, const double *__restrict__ dense,
                         const double *__restrict__ refscore, const int32_t *__restrict__ has_ref,
                         double *__restrict__ out, int *__restrict__ err)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nprops)
        return;
    const int g = pgroup[k];
    const ScoreGroup G = groups[g];
    const int kd = kind[k];
    const int slot = kd == 0 ? base[k] : (kd == 2 ? 4 : 5 + base[k]);
    double tot = 0.0;
    if (has_reads[g])
        tot = dense[G.dense_off + (size_t)pos[k] * 9 + slot];
    if (has_ref[g])
        tot += refscore[k];
    if (tot != tot)
        set_err(err, 3);  // failed to compute a valid score / new score is invalid
    out[k] = tot;
}

// ---------------------------------------------------------------------
// k_bt_win: backtrace + count_errors (align.jl:229-245), one wave per
// alignment, from LDS windows (round 4: codon moves and any band height too --
// the reference's codon alignment and edit_distance's wide bands).
//
// The walk is sequential, so the wave parallelises it across a "box" of the
// cells it can reach next: from the current cell (ii0, jj0) lane l computes
// the move of cell (ii0 - di, jj0 - dj), di = l / 3, dj = di - (l % 3 - 1),
// i.e. the 3 band diagonals around the walk's diagonal for 21 steps
// (63 cells).  Each move is the first strictly-best candidate over the
// stored A values (align.jl:77-104, the same FP64 sums as the forward fill),
// so it equals the trace band's move.  The walk then follows the box with
// one v_readlane per move (the move, the mismatch flag and the read base
// packed in one dword) until it leaves the box, and a new box is computed
// at the cell reached.
//
// Operands come from LDS: a window of kappa rows [klo, khi] of the A band,
// restricted to the elements [e0, e0 + wd) around the walk's diagonal
// (whole rows when P <= BTW_WD), and windows of the table rows and bases.
// The walk only moves to lower kappa; a window is re-staged below when a
// box would leave it.  Staging issues every load of a window before the
// first LDS write (one memory latency per window, not one per element).
// With a mask, the walk also marks the proposals its alignment implies
// (moves_to_proposals, model.jl:458-480; the set union does not depend on
// the walk direction).
// Codon moves (align.jl:77-104, TRACE_CODON_INSERT / _DELETE) reach cells
// 3 diagonals off the walk's: the windows then extend 2 more kappa rows,
// diagonals and table rows, the box evaluates the two codon candidates after
// the three others (the same strict-> order), and a codon move leaves the box
// (|u| = 3), so the next box starts at the cell it reaches.
// ---------------------------------------------------------------------
// The box's walk is ranked in parallel (pointer doubling over the 63
// cells' successors) instead of one readlane step per move (round 4:
// backtrace 19.8 -> 8.0 ms, alignment proposals 36.9 -> 12.9 ms per 512 e2e
// clusters, bit-exact, profiles/r04ab_btw_rank.txt; the sequential walk is
// in git history).
// elements staged per kappa row (the walk's box needs 3 -- 5 with codon
// moves -- around its diagonal): 8 holds twice the kappa rows of 16 in the
// same LDS, so windows are re-staged half as often: with the ranked walk,
// backtrace 8.1 -> 6.9 ms and alignment proposals 12.8 -> 10.7 ms per 512
// e2e clusters (profiles/r04ad_btw_window.txt); a 32-KB window is slower
#ifndef BTW_WD_ELEMS
#define BTW_WD_ELEMS 8
#endif
// window loads in flight per lane (one memory round trip per chunk)
#ifndef BTW_CHUNK
#define BTW_CHUNK 16
#endif
constexpr int BTW_WD = BTW_WD_ELEMS;   // staged elements per kappa row when P > BTW_WD (>= 6: codon boxes)
constexpr int BTW_T = 256;     // staged table rows / template bases per window

// NW > 1 (round 6): a launch of few walks (the reference's, edit_distance's:
// one latency-bound walk each) gives each walk NW waves and a box of
// 3 x (21 NW) cells; the rank's successor tables go through LDS with a block
// barrier per round (8 rounds for 252 cells) and the results are broadcast
// through LDS.  A box then carries ~4x the moves for ~2x the round latency.
constexpr int BTW_FEW = 64;    // launches of at most this many walks take NW = 4

template <int BTW_A, int NW = 1>   // doubles of the A window (4096: 32 KB, 2048: 16 KB); waves per walk
__global__ void __launch_bounds__(64 * NW)
k_bt_win(const BTTask *__restrict__ tasks, const uint8_t *__restrict__ bases, const double *__restrict__ tabs,
         const double *__restrict__ bands, int8_t *__restrict__ moves, int32_t *__restrict__ nmoves,
         int32_t *__restrict__ nerr, int *__restrict__ err, uint8_t *__restrict__ mask, int do_indels)
{
    constexpr int NT = 64 * NW;                         // threads: box cells + the sink
    constexpr int BD = 21 * NW - 1;                     // box depth: cells di = 0 .. BD (3 diagonals)
    constexpr int TT = NW == 1 ? BTW_T : 2 * BTW_T;     // staged table rows / template bases
    constexpr int RB = NW == 1 ? 6 : (NW == 2 ? 7 : 8); // doubling rounds: log2(NT)
    static_assert(NW == 1 || NW == 2 || NW == 4, "1, 2 or 4 waves per walk");
    constexpr int NX = NW > 1 ? NT : 1;                 // LDS rank arrays (NW > 1 only)
    __shared__ double sA[BTW_A];
    __shared__ double sTm[TT], sTx[TT], sTi[TT], sTd[TT];
    __shared__ double sTci[TT], sTcd[TT];   // codon tables (codon alignments only)
    __shared__ uint8_t sS[TT], sTt[TT];
    __shared__ int sJ[2][NX], sPk[NX], sMv[NX], sNi[NX], sNj[NX], sCnt[NW];
    const BTTask T = tasks[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    auto bsync = [&]() {
        if constexpr (NW == 1)
            wave_sync();
        else
            __syncthreads();
    };
    const double *A = bands + T.A;
    const uint8_t *s = bases + T.sb;
    const uint8_t *tt = bases + T.tb;
    const double *tb = tabs + T.tab;
    const int n = T.n, m = T.m, H = T.H, P = T.P;
    const int c = max(m - n, 0) + T.bw;
    const int K = H + 2 * m;
    const bool skew = T.flags & 2, trim = T.flags & 4;
    const bool cod = T.ncins > 0 || T.ncdel > 0;
    const int wd = min(P, cod ? max(BTW_WD, 6) : BTW_WD);   // codon boxes need 5 elements around the walk
    const int W = BTW_A / wd;                          // kappa rows per window (>= 256)
    const int ext = cod ? 2 : 0;                       // codon predecessors: 2 more rows / diagonals
    const double *t_cins = tb + 4 * (size_t)n + 1;     // cins[ii - 3], ncins = n - 2 entries
    const double *t_cdel = t_cins + T.ncins;           // cdel[ii], ncdel = n + 1 entries
    int8_t *out = moves + T.out;
    uint8_t *mk = mask ? mask + T.mask : nullptr;
    // this thread's box cell offsets
    const int bdi = tid / 3, bdj = bdi - (tid % 3 - 1);
    const bool blane = tid < 3 * (BD + 1);
    int ii = n, jj = m, cnt = 0, errs = 0;
    int klo = -1, e0 = 0;                              // A window: rows [klo, klo + W), elements [e0, e0 + wd)
    int q0 = -1, r0 = -1;                              // table rows [q0, q0 + BTW_T), bases [r0, r0 + BTW_T)
    int failed = 0;
    while ((ii > 0 || jj > 0) && !failed) {
        // ---- windows for the box at (ii, jj)
        const int kap0 = ii + jj + c;                  // kappa of the current cell
        const int d0 = ii - jj + c;
        const int klo_need = max(kap0 - 2 * BD - 3 - ext, 0);
        const int elo = max(d0 - 2 - ext, 0) >> 1, ehi = min(d0 + 2 + ext, H - 1) >> 1;
        if (klo < 0 || klo_need < klo || elo < e0 || ehi >= e0 + wd) {
            const int khi = min(kap0 - 1, K - 1);
            klo = max(0, khi - W + 1);
            e0 = min(max((d0 >> 1) - wd / 2, 0), P - wd);
            const int nrow = khi - klo + 1, na = nrow * wd;
            bsync();                                   // every thread is done with the old window
            if (wd == 8 && na == BTW_A) {
                // a whole window of 8-element rows (the common case): thread =
                // NT / 8 rows x 8 columns per u, so each load is the previous
                // one's address plus NT / 8 rows and each LDS slot an immediate
                // offset (round 6: the generic loop spent ~10 instructions per
                // element)
                const double *src = A + (size_t)(klo + (tid >> 3)) * P + e0 + (tid & 7);
                const size_t step = (size_t)(NT / 8) * P;
                for (int u0 = 0; u0 < BTW_A / NT; u0 += BTW_CHUNK) {
                    double v[BTW_CHUNK];
#pragma unroll
                    for (int u = 0; u < BTW_CHUNK; ++u)
                        v[u] = src[(size_t)(u0 + u) * step];
#pragma unroll
                    for (int u = 0; u < BTW_CHUNK; ++u)
                        sA[tid + NT * (u0 + u)] = v[u];
                }
            } else {
                // element t = row * wd + col, t = tid + NT u: incremental row / col
                const int qr = NT / wd, rr = NT % wd;
                int row = tid / wd, col = tid % wd;
                for (int u0 = 0; u0 < BTW_A / NT; u0 += BTW_CHUNK) {
                    double v[BTW_CHUNK];
                    int rw = row, cl = col;
#pragma unroll
                    for (int u = 0; u < BTW_CHUNK; ++u) {   // issue all loads of the chunk
                        const int t = tid + NT * (u0 + u);
                        v[u] = t < na ? A[(size_t)(klo + rw) * P + e0 + cl] : 0.0;
                        rw += qr;
                        cl += rr;
                        if (cl >= wd) {
                            cl -= wd;
                            ++rw;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < BTW_CHUNK; ++u) {
                        const int t = tid + NT * (u0 + u);
                        if (t < na)
                            sA[t] = v[u];
                    }
                    row = rw;
                    col = cl;
                    if (NT * (u0 + BTW_CHUNK) >= na)      // thread 0 holds the chunk's lowest t
                        break;
                }
            }
            bsync();
        }
        const int qlo_need = max(ii - BD - 1 - ext, 0), rlo_need = max(jj - BD - 2, 0);
        if (q0 < 0 || qlo_need < q0 || rlo_need < r0 || ii > q0 + TT - 1 || max(jj - 1, 0) > r0 + TT - 1) {
            q0 = max(0, ii - TT + 1);                  // del index ii .. ; ks = ii - 1 ..
            r0 = max(0, max(jj - 1, 0) - TT + 1);
            bsync();
            constexpr int NU = TT / NT;
            double vm[NU], vx[NU], vi[NU], vd[NU];
            int vs[NU], vt[NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int q = q0 + tid + NT * u;
                const int ks = min(q, n - 1);
                const int qd = min(q, n);
                vm[u] = tb[ks];
                vx[u] = tb[n + ks];
                vi[u] = tb[2 * (size_t)n + ks];
                vd[u] = tb[3 * (size_t)n + qd];
                vs[u] = q < n ? s[q] : 4;
                const int r = r0 + tid + NT * u;
                vt[u] = r < m ? tt[r] : 4;
            }
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int e = tid + NT * u;
                sTm[e] = vm[u];
                sTx[e] = vx[u];
                sTi[e] = vi[u];
                sTd[e] = vd[u];
                sS[e] = (uint8_t)vs[u];
                sTt[e] = (uint8_t)vt[u];
            }
            if (cod) {
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int q = q0 + tid + NT * u;
                    vm[u] = T.ncins > 0 ? t_cins[min(q, T.ncins - 1)] : 0.0;
                    vx[u] = T.ncdel > 0 ? t_cdel[min(q, T.ncdel - 1)] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    sTci[tid + NT * u] = vm[u];
                    sTcd[tid + NT * u] = vx[u];
                }
            }
            bsync();
        }
        // ---- box: the move of cell (ci, cj), packed mv | mismatch << 3 | read base << 4.
        // Branch-free: every LDS read is issued at a selected (valid) index and
        // masked after, so the box is one LDS round trip (round 6; the guarded
        // reads were exec-mask branches and three dependent round trips).
        int pack = 0;
        {
            const int ci = ii - bdi, cj = jj - bdj;
            const int dc = ci - cj + c, kap = ci + cj + c;   // the cell's diagonal and kappa
            const bool valid = blane & (bdj >= 0) & (ci >= 0) & (cj >= 0) & ((ci | cj) != 0) &
                               ((unsigned)dc < (unsigned)H);
            // predecessors in the band: (ci-1, cj-1) diagonal dc, (ci-1, cj) dc-1, (ci, cj-1) dc+1
            const bool in1 = valid & (ci >= 1) & (cj >= 1), in2 = valid & (ci >= 1) & (dc >= 1),
                       in3 = valid & (cj >= 1) & (dc + 1 < H);
            // indices masked to 0 off the band (an and, not a select: hipcc
            // turns selects of computed indices into exec-mask branches)
            const int row1 = (kap - 2 - klo) * wd - e0, row2 = row1 + wd;
            const int a1i = (row1 + (dc >> 1)) & -(int)in1;
            const int a2i = (row2 + ((dc - 1) >> 1)) & -(int)in2;
            const int a3i = (row2 + ((dc + 1) >> 1)) & -(int)in3;
            const double a1 = sA[a1i], a2 = sA[a2i], a3 = sA[a3i];
            const int ks = (max(ci - 1, 0) - q0) & -(int)valid;
            const int kd = (ci - q0) & -(int)valid;
            const bool hs = valid & (ci >= 1), ht = valid & (cj >= 1);
            const int sbr = sS[(ci - 1 - q0) & -(int)hs], tbr = sTt[(cj - 1 - r0) & -(int)ht];
            const double tm = sTm[ks], tx = sTx[ks], ti = sTi[ks], ds = sTd[kd];
            // every read issued before the selects (else hipcc sinks a load
            // into a branch of its own or after another's wait)
            asm volatile("" ::"v"(tm), "v"(tx), "v"(ti), "v"(ds), "v"(a1), "v"(a2), "v"(a3), "v"(sbr), "v"(tbr));
            const int sb = hs ? sbr : 4, tbb = ht ? tbr : 4;
            const bool mis = sb != tbb;
            const double ms = mis ? (skew ? tx * 0.99 : tx) : tm;
            const double is = (trim & ((cj == 0) | (cj == m))) ? 0.0 : ti;
            double best = -RF_INF, x;
            int mv = 0;
            x = a1 + ms;
            if (in1 && x > best) { best = x; mv = 1; }
            x = a2 + is;
            if (in2 && x > best) { best = x; mv = 2; }
            x = a3 + ds;
            if (in3 && x > best) { best = x; mv = 3; }
            if (cod) {
                // TRACE_CODON_INSERT from (ci - 3, cj), TRACE_CODON_DELETE from (ci, cj - 3)
                const bool in4 = valid & (T.ncins > 0) & (ci >= 3) & (dc >= 3);
                const bool in5 = valid & (T.ncdel > 0) & (cj >= 3) & (dc + 3 < H);
                const int row3 = row1 - wd;
                const double a4 = sA[(row3 + ((dc - 3) >> 1)) & -(int)in4];
                const double a5 = sA[(row3 + ((dc + 3) >> 1)) & -(int)in5];
                x = a4 + sTci[(ci - 3 - q0) & -(int)in4];
                if (in4 && x > best) { best = x; mv = 4; }
                x = a5 + sTcd[kd];
                if (in5 && x > best) { best = x; mv = 5; }
            }
            pack = valid ? (mv | (mis ? 8 : 0) | (sb << 4)) : 0;
        }
        // ---- walk the box by ranking its cells in parallel: J0 = each box
        // cell's successor lane (or the sink, lane 63: leaves the box, reaches
        // (0, 0), or no move), J_r = J0^(2^r) by pointer doubling; lane k then
        // finds the k-th cell of the walk from lane 1 (the current cell) by
        // the binary digits of k, and emits the k-th move.  Round r applies
        // J_r to the lane's cell and squares J_r with two independent
        // permutes (round 6: 6 dependent permute rounds instead of 11).  The
        // same moves, marks, error counts and failure points as the
        // sequential walk (git history).
        {
            constexpr int SINK = NT - 1;
            const int mv0 = pack & 7;
            const int bu = tid % 3 - 1;
            const int ndi = bdi + (int)((mv0 == 1) | (mv0 == 2));
            const int nu = bu + (int)(mv0 == 2) - (int)(mv0 == 3);
            const bool inbox = (mv0 >= 1 && mv0 <= 3) && ndi <= BD && nu >= -1 && nu <= 1;
            const int ti = ii - ndi, tj = jj - (ndi - nu);
            int J = (blane && inbox && (ti > 0 || tj > 0)) ? ndi * 3 + nu + 1 : SINK;
            if (tid == SINK)
                J = SINK;
            int cell = 1;   // thread k: the k-th cell of the walk
            int pk;
            if constexpr (NW == 1) {
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int nx = __builtin_amdgcn_ds_bpermute(cell << 2, J);
                    if (r < RB - 1)
                        J = __builtin_amdgcn_ds_bpermute(J << 2, J);
                    cell = ((lane >> r) & 1) ? nx : cell;
                }
                pk = __builtin_amdgcn_ds_bpermute(cell << 2, pack);
            } else {
                // the same rounds through LDS (two tables, a block barrier each)
                sPk[tid] = pack;
                sJ[0][tid] = J;
                bsync();
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int nx = sJ[r & 1][cell];
                    if (r < RB - 1) {
                        J = sJ[r & 1][J];
                        sJ[(r + 1) & 1][tid] = J;
                    }
                    cell = ((tid >> r) & 1) ? nx : cell;
                    bsync();
                }
                pk = sPk[cell];
            }
            // cells reached; a cell with no move (mv 0) ends the walk in failure
            const bool visited = cell != SINK;
            const int mvk = pk & 7;
            const int cdi = cell / 3, cdu = cell % 3 - 1;
            const int ci = ii - cdi, cj = jj - (cdi - cdu);
            // the cell after this move
            const int di = (mvk == 1 || mvk == 2) ? 1 : (mvk == 4 ? 3 : 0);
            const int dj = (mvk == 1 || mvk == 3) ? 1 : (mvk == 5 ? 3 : 0);
            int nvis;
            bool nomove_last;
            if constexpr (NW == 1) {
                nvis = __popcll(__ballot(visited));
                nomove_last = __builtin_amdgcn_readlane(mvk, max(nvis - 1, 0)) == 0;
            } else {
                const int cw = __popcll(__ballot(visited));
                if (lane == 0)
                    sCnt[wv] = cw;
                sMv[tid] = mvk;
                sNi[tid] = ci - di;
                sNj[tid] = cj - dj;
                bsync();
                nvis = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w)
                    nvis += sCnt[w];
                nomove_last = sMv[max(nvis - 1, 0)] == 0;
            }
            int nmv = nomove_last ? nvis - 1 : nvis;
            bool fail_now = nomove_last;
            if (cnt + nmv > n + m) {   // the sequential walk's cnt >= n + m check
                nmv = n + m - cnt;
                fail_now = true;
            }
            const bool emit = tid < nmv;
            const int ksb = pk >> 4;
            const bool mism = pk & 8;
            // the forward step of this move ends at (ci, cj) (moves_to_proposals):
            // a mismatch marks (cj, read base), an insertion (cj, 5 + base), a
            // deletion (cj, 4) -- one store, its slot selected (no branches)
            const bool mark = emit && mk && ((mvk == 1 && mism) || (do_indels && (mvk == 2 || mvk == 3)));
            const int slot9 = cj * 9 + (mvk == 1 ? ksb : (mvk == 2 ? 5 + ksb : 4));
            if (emit)
                out[n + m - 1 - (cnt + tid)] = (int8_t)mvk;
            if (mark)
                mk[(size_t)slot9] = 1;
            // count_errors: 1 per mismatch or indel, 3 per codon move (this
            // wave's threads; the waves' sums are added at the end)
            errs += __popcll(__ballot(emit && (mvk >= 2 || mism))) + 2 * __popcll(__ballot(emit && mvk >= 4));
            if (nmv > 0) {
                if constexpr (NW == 1) {
                    ii = __builtin_amdgcn_readlane(ci - di, nmv - 1);
                    jj = __builtin_amdgcn_readlane(cj - dj, nmv - 1);
                } else {
                    ii = sNi[nmv - 1];
                    jj = sNj[nmv - 1];
                }
            }
            cnt += nmv;
            if (fail_now) {
                if (tid == 0)
                    set_err(err, 2);  // failed to find a move
                failed = 1;
            }
        }
    }
    if constexpr (NW > 1) {
        bsync();
        if (lane == 0)
            sCnt[wv] = errs;
        bsync();
        errs = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w)
            errs += sCnt[w];
    }
    if (tid == 0) {
        nmoves[T.idx] = cnt;
        nerr[T.idx] = errs;
    }
}

// ---------------------------------------------------------------------
// k_aln_sums: alignment_error_probs's per-column sums (model.jl:817-840)
// on the device, from the backtrace moves already there (k_bt_win).  One workgroup per group (cluster); its reads are walked in
// batch order, one read at a time: the 256 threads take 256 consecutive
// moves, a block prefix sum of the (read, consensus) steps gives each move's
// (i, j), and a MATCH move adds base_distribution(s[i], match[i]) to column
// j: out[j][b] += (b == s[i] ? match[i] : errlp(match[i])).  A read matches a
// column at most once, and a barrier separates the reads, so every column
// receives the same FP64 additions in the same order as the host loop
// (rf_aln_error_sums).  errlp = log10(1 - 10^ilp) - log10(3) is evaluated on
// the host (libm) once per row-code dictionary entry; the read's row-code
// record gives its entry and base.
// ---------------------------------------------------------------------
struct alignas(16) AlnSumRead {
    int64_t mv;    // moves slot (bytes in the backtrace move buffer; moves end-aligned in n + m)
    int64_t rec;   // row-code records (doubles offset into the table arena)
    int32_t n, m, idx, pad;
};
struct alignas(16) AlnSumGroup {
    int64_t out;   // doubles offset of the group's m x 4 sums
    int32_t r0, r1, m, pad;
};

__global__ void __launch_bounds__(256) k_aln_sums(const AlnSumGroup *__restrict__ groups,
                                                  const AlnSumRead *__restrict__ reads,
                                                  const double *__restrict__ tabs, const int8_t *__restrict__ moves,
                                                  const int32_t *__restrict__ nmoves, const double *__restrict__ lut,
                                                  const double *__restrict__ errlut, double *__restrict__ out)
{
    __shared__ int wsum[4];
    const AlnSumGroup G = groups[blockIdx.x];
    double *o = out + G.out;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int e = tid; e < 4 * G.m; e += 256)
        o[e] = 0.0;
    __syncthreads();
    for (int r = G.r0; r < G.r1; ++r) {
        const AlnSumRead R = reads[r];
        const int cnt = nmoves[R.idx];
        const int8_t *mv = moves + R.mv + (R.n + R.m - cnt);
        const uint64_t *rec = (const uint64_t *)(tabs + R.rec);
        int ci = 0, cj = 0;   // read / consensus positions consumed before this tile (block-uniform)
        for (int b0 = 0; b0 < cnt; b0 += 256) {
            const int e = b0 + tid;
            const int v = e < cnt ? mv[e] : 0;
            // align.jl OFFSETS: MATCH (1,1), INSERT (1,0), DELETE (0,1), CODON_INSERT (3,0), CODON_DELETE (0,3)
            const int di = (v == 1 || v == 2) ? 1 : (v == 4 ? 3 : 0);
            const int dj = (v == 1 || v == 3) ? 1 : (v == 5 ? 3 : 0);
            // a tile moves (i, j) by at most 3 * 256 each: 16-bit fields of one
            // int hold the tile's prefix sums; the carry across tiles is two ints
            const int x = di | (dj << 16);
            int inc = x;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(inc, off);
                if (lane >= off)
                    inc += y;
            }
            if (lane == 63)
                wsum[w] = inc;
            __syncthreads();
            int before = 0;
            for (int k = 0; k < w; ++k)
                before += wsum[k];
            const int tile = wsum[0] + wsum[1] + wsum[2] + wsum[3];
            __syncthreads();   // wsum is rewritten by the next tile
            if (v == 1) {
                const int ex = before + inc - x;
                const int i = ci + (ex & 0xffff), j = cj + (ex >> 16);
                const uint64_t rc = rec[i];
                const int code = (int)(rc & 0xffff), sb = (int)(rc >> 48) & 0xff;
                const double ilp = lut[4 * code], el = errlut[code];
                double *p = o + (size_t)j * 4;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    p[q] += q == sb ? ilp : el;
            }
            ci += tile & 0xffff;
            cj += tile >> 16;
        }
        __syncthreads();   // this read's additions precede the next read's
    }
}

// Groups with many reads (c3: one cluster of 1,000 reads) leave k_aln_sums
// one workgroup walking every read in turn (16.6 ms per call at c3, round 4
// profile).  There the sums run in two launches instead: k_aln_marks, one
// wave per read, writes each MATCH move's row-code entry and base into a
// (read, column) record; k_aln_fold, one lane per (group, column), adds the
// records of the column's reads in batch order -- the same FP64 additions in
// the same order per column as k_aln_sums and the host loop.
__global__ void __launch_bounds__(64) k_aln_marks(const AlnSumGroup *__restrict__ groups, int ngroups,
                                                  const AlnSumRead *__restrict__ reads,
                                                  const int64_t *__restrict__ rbase,
                                                  const double *__restrict__ tabs, const int8_t *__restrict__ moves,
                                                  const int32_t *__restrict__ nmoves, uint32_t *__restrict__ marks)
{
    const int r = blockIdx.x, lane = threadIdx.x;
    const AlnSumRead R = reads[r];
    const int cnt = nmoves[R.idx];
    const int8_t *mv = moves + R.mv + (R.n + R.m - cnt);
    const uint64_t *rec = (const uint64_t *)(tabs + R.rec);
    uint32_t *row = marks + rbase[r];   // this read's m records
    int ci = 0, cj = 0;
    for (int b0 = 0; b0 < cnt; b0 += 64) {
        const int e = b0 + lane;
        const int v = e < cnt ? mv[e] : 0;
        const int di = (v == 1 || v == 2) ? 1 : (v == 4 ? 3 : 0);
        const int dj = (v == 1 || v == 3) ? 1 : (v == 5 ? 3 : 0);
        const int x = di | (dj << 16);   // a tile moves (i, j) by at most 3 * 64 each
        int inc = x;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(inc, off);
            if (lane >= off)
                inc += y;
        }
        if (v == 1) {
            const int ex = inc - x;
            const int i = ci + (ex & 0xffff), j = cj + (ex >> 16);
            const uint64_t rc = rec[i];
            row[j] = (uint32_t)(rc & 0xffff) | ((uint32_t)((rc >> 48) & 0xff) << 16) | 0x80000000u;
        }
        const int tile = __shfl(inc, 63);
        ci += tile & 0xffff;
        cj += tile >> 16;
    }
}

__global__ void __launch_bounds__(256) k_aln_fold(const AlnSumGroup *__restrict__ groups, int ngroups,
                                                  const int64_t *__restrict__ gcol, const int64_t *__restrict__ gbase,
                                                  const uint32_t *__restrict__ marks, const double *__restrict__ lut,
                                                  const double *__restrict__ errlut, double *__restrict__ out,
                                                  int64_t ncols)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ncols)
        return;
    int lo = 0, hi = ngroups - 1;   // the group whose columns hold e
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (gcol[mid] <= e)
            lo = mid;
        else
            hi = mid - 1;
    }
    const AlnSumGroup G = groups[lo];
    const int j = (int)(e - gcol[lo]);
    const uint32_t *col = marks + gbase[lo] + j;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int r = 0; r < G.r1 - G.r0; ++r) {
        const uint32_t rc = col[(int64_t)r * G.m];
        if (rc & 0x80000000u) {
            const int code = (int)(rc & 0xffff), sb = (int)((rc >> 16) & 0xff);
            const double ilp = lut[4 * code], el = errlut[code];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                acc[q] += q == sb ? ilp : el;
        }
    }
    double *o = out + G.out + (int64_t)j * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        o[q] = acc[q];
}

// ---------------------------------------------------------------------
// k_scatter: one staged upload -> per-object device regions (a block per
// segment), so a batch upload is one H2D copy instead of one per object.
// ---------------------------------------------------------------------
struct alignas(16) Segment {
    int64_t src, dst, len;   // bytes
    int64_t pad;
};

__global__ void k_scatter(const Segment *__restrict__ segs, const uint8_t *__restrict__ src,
                          uint8_t *__restrict__ dst)
{
    const Segment S = segs[blockIdx.x];
    if ((S.src | S.dst | S.len) % 8 == 0) {
        const uint64_t *a = reinterpret_cast<const uint64_t *>(src + S.src);
        uint64_t *b = reinterpret_cast<uint64_t *>(dst + S.dst);
        for (int64_t e = threadIdx.x; e < S.len / 8; e += blockDim.x)
            b[e] = a[e];
    } else {
        for (int64_t e = threadIdx.x; e < S.len; e += blockDim.x)
            dst[S.dst + e] = src[S.src + e];
    }
}

// ---------------------------------------------------------------------
// k_tables: RifrafSequence tables (rifrafsequences.jl:19-82, no codon
// moves) and row-code records of phred-coded reads, built on the device
// from one byte per position (rf_set_sequences_codes).  Per code c the host
// passes lp[c], match[c] (its own libm values), and the dictionary ids of
// the (match, mismatch, ins) triple and of the del value lp[c] + s_del:
//   mismatch = lp + s_mis, ins = lp + s_ins,
//   del[0] = lp[0] + s_del, del[n] = lp[n-1] + s_del,
//   del[i] = max(lp[i-1], lp[i]) + s_del,
// the same FP64 additions and maximum as the host constructor, so the same
// bits.  One block per sequence.
// ---------------------------------------------------------------------
struct alignas(16) CodeSeq {
    int64_t tab;    // doubles offset of the sequence's tables
    int64_t src;    // byte offset of its codes / bases in the staged upload
    int32_t n, pad0;
    int64_t pad1;
};
struct alignas(16) CodeLut {   // per Phred code
    double lp, match;
    int32_t id3, id1;
    int32_t pad0, pad1;
};

__global__ void __launch_bounds__(256) k_tables(const CodeSeq *__restrict__ seqs, const uint8_t *__restrict__ codes,
                                                const uint8_t *__restrict__ bases, const CodeLut *__restrict__ lut,
                                                double s_mis, double s_ins, double s_del, double *__restrict__ tabs)
{
    const CodeSeq S = seqs[blockIdx.x];
    const int n = S.n;
    const uint8_t *cd = codes + S.src;
    const uint8_t *bs = bases + S.src;
    double *t = tabs + S.tab;
    uint64_t *rec = (uint64_t *)(t + row_code_off(n, 0, 0));
    for (int i = threadIdx.x; i <= n; i += blockDim.x) {
        const CodeLut L = lut[cd[min(i, n - 1)]];
        // del[i] and its dictionary id: the neighbour with the larger lp
        int idd;
        double dv;
        if (i == 0 || i == n) {
            dv = L.lp + s_del;
            idd = L.id1;
        } else {
            const CodeLut Lp = lut[cd[i - 1]];
            const double l = Lp.lp, r = L.lp;
            dv = (r > l ? r : l) + s_del;
            idd = r > l ? L.id1 : Lp.id1;
        }
        t[3 * (size_t)n + i] = dv;
        if (i < n) {
            t[i] = L.match;
            t[n + i] = L.lp + s_mis;
            t[2 * (size_t)n + i] = L.lp + s_ins;
        }
        // records need del[i] and del[i+1]: written by position i with the next id
        if (i < n) {
            int idn;
            if (i + 1 == n) {
                idn = L.id1;
            } else {
                const CodeLut Ln = lut[cd[i + 1]];
                idn = Ln.lp > L.lp ? Ln.id1 : L.id1;
            }
            rec[i] = (uint64_t)(uint32_t)L.id3 | ((uint64_t)(uint32_t)idd << 16) | ((uint64_t)(uint32_t)idn << 32) |
                     ((uint64_t)bs[i] << 48);
        }
    }
}

// Per-read setup values of the native driver from the staged Phred codes
// (round 5: formerly rf_host_code_prep's per-position host pass, which
// bounded a rank held to 2 host cores): one thread per sequence,
//   est[k]   = est_n_errors = sum(10^lp) in Julia 0.6's order
//              (rifrafsequences.jl:19-82, base/reduce.jl mapreduce_impl:
//              sequential below 1,024 elements, else pairwise halves);
//   ucode[k] = the code of the first maximal match score;
//   tsum[k]  = sum_i 10^(match[c_i] - match[ucode]) sequentially -- the
//              host finishes logsumexp10 = log10(tsum) + max with libm
//              (rf_host_lse_finish), so the initial consensus (model.jl:
//              575-579) is the one the host pass picks.
// The same table entries and the same FP64 additions in the same order as
// rf_host_code_prep: bit-identical.
constexpr int PREP_STACK = 40;
// sum_{i = lo..hi} tab[c[i]] left to right (the same additions in the same
// order as one loop), with eight entries loaded ahead of their additions:
// from LDS each element was two dependent round trips on lane 0's chain
__device__ __forceinline__ double prep_seq_sum(const uint8_t *c, const double *tab, int64_t lo, int64_t hi)
{
    double a = tab[c[lo]];
    int64_t i = lo + 1;
    for (; i + 8 <= hi + 1; i += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v[u] = tab[c[i + u]];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            a += v[u];
    }
    for (; i <= hi; ++i)
        a += tab[c[i]];
    return a;
}

__device__ double prep_julia_sum(const uint8_t *c, const double *p10, int64_t lo0, int64_t hi0)
{
    // explicit-stack post-order of the pairwise split (no device recursion)
    int64_t slo[PREP_STACK], shi[PREP_STACK];
    double sleft[PREP_STACK];
    int sst[PREP_STACK];
    int sp = 0;
    slo[0] = lo0;
    shi[0] = hi0;
    sst[0] = 0;
    double ret = 0.0;
    while (true) {
        const int64_t lo = slo[sp], hi = shi[sp];
        if (lo + 1024 > hi) {   // leaf: sequential
            ret = prep_seq_sum(c, p10, lo, hi);
            if (--sp < 0)
                return ret;
            continue;
        }
        const int64_t mid = (lo + hi) >> 1;
        if (sst[sp] == 0) {
            sst[sp] = 1;
            ++sp;
            slo[sp] = lo;
            shi[sp] = mid;
            sst[sp] = 0;
        } else if (sst[sp] == 1) {
            sleft[sp] = ret;
            sst[sp] = 2;
            ++sp;
            slo[sp] = mid + 1;
            shi[sp] = hi;
            sst[sp] = 0;
        } else {
            ret = sleft[sp] + ret;
            if (--sp < 0)
                return ret;
        }
    }
}

// One wave per sequence (round 5): the wave stages the sequence's codes in
// LDS with coalesced loads, and lane 0 runs the sequential sums from LDS (a
// thread per sequence read its codes one byte load at a time, dependent
// chains of global loads: 1.2 ms for configs[2]'s 1,000 reads).  The sums
// and their order are unchanged.
constexpr int CP_MAX = 32768;   // codes staged in LDS (longer sequences: read in place)
__global__ void __launch_bounds__(64) k_code_prep(const CodeSeq *__restrict__ seqs, int nseq,
                                                  const uint8_t *__restrict__ codes, const double *__restrict__ tabs3,
                                                  const double *__restrict__ grid, double *__restrict__ est,
                                                  int32_t *__restrict__ ucode, double *__restrict__ tsum)
{
    __shared__ double p10[256], mt[256], gr[256];
    __shared__ __attribute__((aligned(16))) uint8_t sc[CP_MAX];
    __shared__ int s_uc;
    for (int i = threadIdx.x; i < 256; i += 64) {
        p10[i] = tabs3[i];
        mt[i] = tabs3[256 + i];
    }
    const int k = blockIdx.x;
    if (k >= nseq)
        return;
    const CodeSeq S = seqs[k];
    const int64_t n = S.n;
    const uint8_t *cg = codes + S.src;
    if (n <= CP_MAX)
        for (int64_t i = threadIdx.x; i < n; i += 64)
            sc[i] = cg[i];
    __syncthreads();
    const uint8_t *c = n <= CP_MAX ? (const uint8_t *)sc : cg;
    // ucode: the code at the first position whose match score is maximal
    // (the sequential `if (mt[c_i] > mt[uc]) uc = c_i` scan), by a wave
    // reduction of (maximum, first position)
    {
        double best = -RF_INF;
        int64_t at = INT64_MAX;
        for (int64_t i = threadIdx.x; i < n; i += 64) {
            const double v = mt[c[i]];
            if (v > best) {   // strided: a lane's first maximum is its smallest position
                best = v;
                at = i;
            }
        }
        for (int off = 32; off >= 1; off >>= 1) {
            const double ob = __shfl_xor(best, off);
            const int64_t oa = __shfl_xor(at, off);
            if (ob > best || (ob == best && oa < at)) {
                best = ob;
                at = oa;
            }
        }
        if (threadIdx.x == 0) {
            const int uc = c[at == INT64_MAX ? 0 : at];
            est[k] = n <= 1024 ? prep_seq_sum(c, p10, 0, n - 1) : prep_julia_sum(c, p10, 0, n - 1);
            ucode[k] = uc;
            s_uc = uc;
        }
    }
    __syncthreads();
    const int uc = s_uc;
    for (int i = threadIdx.x; i < 256; i += 64)
        gr[i] = grid[(size_t)uc * 256 + i];
    __syncthreads();
    if (threadIdx.x == 0)
        tsum[k] = prep_seq_sum(c, gr, 0, n - 1);
}

// ---------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------

namespace {

// Every arena keeps ARENA_GUARD bytes before its first region and after its
// last: k_score_seg's LDS-DMA staging reads whole 16-B chunks of band rows
// and table rows, which may start up to one row before a region or end past
// it (values never used); the guards keep those reads inside the allocation.
constexpr int64_t ARENA_GUARD = 1 << 16;

struct Region {
    int64_t off = -1;  // bytes
    int64_t cap = 0;
};

struct Arena {
    char *d = nullptr;
    int64_t cap = 0, top = 0;
};

struct SeqObj {
    bool valid = false;
    bool finite = false;   // match / mismatch / ins / del tables hold no -Inf (lean DP eligible)
    bool coded = false;    // row codes written after the tables (RF_TASK_CODED)
    int32_t n = 0, ncins = 0, ncdel = 0;
    Region bases, tabs;
};

struct TplObj {
    bool valid = false;
    int32_t m = 0;
    uint64_t version = 0;
    Region bases;
};

struct Band {
    bool valid = false;
    int32_t seq = -1, tpl = -1, bw = 0, n = 0, m = 0, H = 0, flags = 0;
    int32_t P = 0;   // kappa row stride (band_stride at the fill)
    uint64_t tplver = 0;
    Region r;
};

struct Slot {
    Band a, b;
};

// Choice of dense scorer for one launch.
struct ScorePick {
    bool lean = false;
    bool seg = false;   // k_score_segl: wide bands (window too large for LDS), finite tables
    int lds = 0;    // lean: doubles of dynamic LDS; general: doubles per staged band
    int q() const { return 256; }   // k_score_ws chain columns per work item
    // columns per work item of the chosen scorer (k_score: 64)
    int cols() const { return lean ? q() : 64; }
};

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

}  // namespace

// Host worker threads: OMP_NUM_THREADS when set (the GPU box's CPU share),
// else the machine's, at most 16, and never more than the CPUs this thread
// may run on (sched_getaffinity, read per call: a rank pinned to its share of
// the host's cores -- e.g. 2 of 16 at 8 ranks -- gets that many workers).
// Shared with rifraf_batch.cpp (C++ linkage, not part of the C-ABI).
int rf_internal_host_threads()
{
    static const int cap = [] {
        const char *v = std::getenv("OMP_NUM_THREADS");
        int t = (v && *v) ? std::atoi(v) : (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(t, 16));
    }();
    cpu_set_t cs;
    CPU_ZERO(&cs);
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0)
        return std::max(1, std::min(cap, (int)CPU_COUNT(&cs)));
    return cap;
}

namespace {
inline int host_threads() { return rf_internal_host_threads(); }
template <class F>
void parallel_for(int nth, F fn)
{
    if (nth <= 1) {
        fn(0);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 1; t < nth; ++t)
        th.emplace_back(fn, t);
    fn(0);
    for (auto &x : th)
        x.join();
}

// Code dictionary of the row codes (RF_TASK_CODED): every distinct
// (match, mismatch, ins) triple and del value of the context's reads gets a
// 16-bit code, first come first served, keyed by the exact bit patterns.  A
// read whose values would need a code past RF_CODES - 1 stays uncoded (its
// DP reads the tables directly; counted in `uncoded_reads`, rf_code_stats).
// Entries are only appended while any coded sequence outside an upload is
// still valid, so codes of earlier reads stay valid; an upload that replaces
// every coded sequence of the context starts a fresh dictionary, so a
// long-lived context refilled batch after batch does not fill it up.  `lut`
// is the device copy (RF_CODES x 4 triple doubles, then RF_CODES del doubles).
struct CodeDict {
    struct K3 {
        uint64_t a, b, c;
        bool operator==(const K3 &o) const { return a == o.a && b == o.b && c == o.c; }
    };
    struct H3 {
        size_t operator()(const K3 &k) const
        {
            return (size_t)((k.a * 0x9E3779B97F4A7C15ull) ^ (k.b * 0xC2B2AE3D27D4EB4Full) ^ (k.c * 0x165667B19E3779F9ull));
        }
    };
    std::unordered_map<K3, uint32_t, H3> t3;
    std::unordered_map<uint64_t, uint32_t> d1;
    std::vector<double> t3v, d1v;   // host copies of the entries
    size_t up3 = 0, up1 = 0;        // entries already on the device
    int64_t uncoded_reads = 0;      // reads left uncoded because the dictionary was full
    int64_t resets = 0;
    DevBuf lut;
    // per triple entry: log10(1 - 10^match) - log10(3), the off-base value of
    // base_distribution (model.jl:804-809), host libm; device copy errlut
    std::vector<double> errv;
    size_t uperr = 0;
    DevBuf errlut;

    void reset()
    {
        t3.clear();
        d1.clear();
        t3v.clear();
        d1v.clear();
        errv.clear();
        up3 = up1 = uperr = 0;
        ++resets;
    }

    static uint64_t bits(double x)
    {
        uint64_t u;
        std::memcpy(&u, &x, 8);
        return u;
    }
    // read-only lookups (safe from several threads while nothing is inserted)
    int32_t find3(const K3 &k) const
    {
        auto it = t3.find(k);
        return it == t3.end() ? -1 : (int32_t)it->second;
    }
    int32_t find1(uint64_t k) const
    {
        auto it = d1.find(k);
        return it == d1.end() ? -1 : (int32_t)it->second;
    }
    // per-thread direct-mapped front cache of the lookups (a read set has few
    // distinct values; misses fall through to the maps)
    struct Cache {
        std::vector<std::pair<K3, int32_t>> c3 = std::vector<std::pair<K3, int32_t>>(1024, {K3{}, -2});
        std::vector<std::pair<uint64_t, int32_t>> c1 = std::vector<std::pair<uint64_t, int32_t>>(1024, {0, -2});
    };
    int32_t find3(const K3 &k, Cache &C) const
    {
        auto &e = C.c3[(H3()(k) >> 32) & 1023];
        if (e.second != -2 && e.first == k)
            return e.second;
        const int32_t v = find3(k);
        if (v >= 0)
            e = {k, v};
        return v;
    }
    int32_t find1(uint64_t k, Cache &C) const
    {
        auto &e = C.c1[((k * 0x9E3779B97F4A7C15ull) >> 40) & 1023];
        if (e.second != -2 && e.first == k)
            return e.second;
        const int32_t v = find1(k);
        if (v >= 0)
            e = {k, v};
        return v;
    }
};

// Tuning options (rf_set_option keys, include/rifraf_hip.h).  Every option
// selects between bit-identical code paths; defaults come from the RIFRAF_*
// environment once, at rf_create, and never from a hot path.
#ifndef DP_WIDE_DEFAULT
#define DP_WIDE_DEFAULT 3
#endif
struct Opts {
    int score_mode = 0;     // RF_OPT_SCORE_MODE: 0 auto, 1 fused, 2 split
    int score_kernel = 0;   // RF_OPT_SCORE_KERNEL: 0 auto, 1 general, 2 seg, 3 ws (k_score_ws when it fits)
    int lean_lds_kb = 0;    // RF_OPT_LEAN_LDS_KB: k_score_ws LDS budget (0 = default 160 KB)
    int dp_wide = DP_WIDE_DEFAULT;   // RF_OPT_DP_WIDE: wide lean tasks (bit 0: H 128..255 in 64 lanes,
                                     // bit 1: H 64..127 in 32 lanes)
    int band_pad_h = 64;    // RF_OPT_BAND_PAD: a realign call whose widest band has H >= this gets
                            // 128-B-line rows for all its bands (0: never, 1: always)
    int bt_win_kb = 16;     // RF_OPT_BT_WIN_KB: k_bt_win A window (16 or 32 KB of LDS)
    int stage_kb = 262144;  // RF_OPT_STAGE_KB: rf_set_sequences staging chunk (KB of tables)
    int dp_psplit = -1;     // RF_OPT_DP_PSPLIT: lean stride-class split mask (-1 auto)
    int dp_np8 = 1;         // RF_OPT_DP_NP8: H 128..255 in k_dpr<8> (0: k_dp<64>)
    int dp_np8_lean = 1;    // RF_OPT_DP_NP8_LEAN: lean k_dpr<8> path
    int dp_streams = 1;     // RF_OPT_DP_STREAMS: DP classes on concurrent streams
    int aln_sums_host = 0;  // RF_OPT_ALN_SUMS_HOST: 1 = rf_aln_error_sums folds the moves on the host
    int aln_marks_min = 128;   // RF_OPT_ALN_MARKS_MIN: device QV sums in two launches above this many reads per group
    int sync_block = 2;     // RF_OPT_SYNC_BLOCK: 1 host waits yield / sleep instead of spinning; 2 (default)
                            // auto: when the waiting thread may run on fewer than 4 CPUs
    int dp_nl64 = 1024;     // RF_OPT_DP_NL64: at most this many non-lean H <= 127 tasks run in k_dpx
    int score_wgs = 2048;   // RF_OPT_SCORE_WGS: split-mode k_score_ws takes reads in chunks so that about
                            // this many workgroups remain
    int seg_wgs = 262144;   // RF_OPT_SEG_WGS: split-mode k_score_segl takes reads in chunks so that about
                            // this many workgroups remain
    int dp_mc = 1;          // RF_OPT_DP_MC: H > 2040 bands without codon moves in k_dpm (0: k_dp)
    int bt_nw = 4;          // RF_OPT_BT_NW: waves per walk in launches of at most BTW_FEW walks (4 or 1)
    int dp_pfit = 1;        // RF_OPT_DP_PFIT: lean NP >= 2 class launched at its tasks' stride class
    int dp_lat = 2048;      // RF_OPT_DP_LAT: a call with at most this many lean H <= 127 tasks runs them all as
                            // one k_dpx launch (latency mode: the launch cannot fill the GPU)
};

}  // namespace

struct rf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t side[3] = {};   // concurrent DP class launches (fork/join on `stream`)
    hipEvent_t ev[6];
    hipEvent_t fork = nullptr, join[3] = {};
    std::string err;
    Arena bytes_arena;  // sequence + template bases
    Arena tab_arena;    // sequence tables
    Arena band_arena;   // A / B bands
    CodeDict codes;     // row-code dictionary (RF_TASK_CODED)
    std::vector<SeqObj> seqs;
    std::vector<TplObj> tpls;
    std::vector<Slot> slots;
    uint64_t tpl_counter = 0;
    uint64_t layout_gen = 1;   // bumped whenever a device offset / length may change
    int64_t arena_grows = 0;   // arena_grow calls and their wall seconds (RIFRAF_BATCH_TIMING)
    double arena_grow_s = 0.0;
    // bumped by every call that changes sequences, templates or band metadata:
    // a plan validated at the current epoch with the same job / slot list
    // needs no per-slot validation again
    uint64_t state_epoch = 1;
    DevBuf scratch[28];
    // pinned host staging for sequence uploads (pageable H2D copies of a few
    // MB took ~14 ms per cluster upload on the box: page locking per call)
    void *pinned = nullptr;
    size_t pinned_bytes = 0;
    // pinned landing zone for small per-call results (rf_realign's scores and
    // the error flag): one D2H + one synchronize per call
    void *hout = nullptr;
    size_t hout_bytes = 0;
    // pinned ring for the per-call descriptor uploads (upload()): the runtime
    // stages a pageable H2D copy through a blit of its own
    void *up = nullptr;
    size_t up_bytes = 0, up_off = 0;
    // pinned landing zone for the other calls' downloads (ensure_hdn): the
    // error flag at 0, results from 16
    void *hdn = nullptr;
    size_t hdn_bytes = 0;
    DevBuf grow_segs;   // compaction descriptors (arena_grow may run inside other uploads)
    int *d_err = nullptr;
    double dp_ms = 0, score_ms = 0, gather_ms = 0, bt_ms = 0;
    double codon_ms = 0;        // k_codon of the last rf_score (inside score_ms)
    hipEvent_t ev_codon = nullptr;
    hipEvent_t ev_block = nullptr;   // blocking-sync event (RF_OPT_SYNC_BLOCK)
    Opts opt;
    uint64_t opt_gen = 0;      // bumped by rf_set_option (scorer plan key)
    std::vector<BTTask> bt_win;   // backtrace descriptors of the last launch
    // host-side plan caches: a repeated call with identical arguments and an
    // unchanged layout reuses the uploaded descriptors (steady-state loops)
    struct {
        bool valid = false;
        uint64_t gen = 0;
        uint64_t val_epoch = 0;   // state_epoch at which the job list was last validated
        std::vector<int32_t> slot, seq, tpl, bw, flags;   // flags: per job (rf_realign_jobs)
        size_t nr[4][2] = {};   // k_dpr<1,2,4,8> x {general, lean}
        size_t nrp[4][4] = {};  // lean k_dpr<NP, true, PM> split by band row stride (dpr_pm)
        size_t nw[2] = {};     // lean wide-task classes (RF_OPT_DP_WIDE)
        size_t nx = 0;         // latency-bound non-lean tasks, k_dpx (RF_OPT_DP_NL64)
        size_t nl = 0;         // latency-mode lean tasks, one k_dpx<false, false> class (RF_OPT_DP_LAT)
        size_t nwm = 0;        // very wide bands without codon moves across CUs (k_dpm, RF_OPT_DP_MC)
        int gm = 0;            // their most slices
        size_t n64 = 0, ng = 0;
        int hmax64 = 0, hmaxg = 0;
        std::vector<DPTask> tasks;   // host copy of the uploaded descriptors
    } rplan;
    std::vector<int32_t> jflags;   // rf_realign: the call's flags for every job
    struct {
        bool valid = false;
        uint64_t gen = 0;
        uint64_t val_epoch = 0;   // state_epoch at which the slot list was last validated
        std::vector<int32_t> slot_off, slots;
        size_t nitems = 0;
        int max_reads = 0, ngroups = 0;
        int64_t dense_total = 0, split_total = 0;
        ScorePick pick;
        uint64_t opt_gen = 0;
        // host copies of the uploaded descriptors: alive until the uploads
        // they source have completed (hipMemcpyAsync from pageable memory)
        std::vector<WorkItem> items;
        std::vector<ScoreGroup> groups;
        std::vector<ScoreRead> reads;
        std::vector<int64_t> gstart;
    } dplan;
};

namespace {

const char *numeric_message(int code)
{
    switch (code) {
    case 1: return "new score is invalid";
    case 2: return "failed to find a move";
    case 3: return "failed to compute a valid score";
    case 4: return "internal error: a band slice's neighbour never arrived (k_dpm)";
    default: return "numeric error";
    }
}

int fail(rf_ctx *ctx, int code, const std::string &msg)
{
    if (ctx)
        ctx->err = msg;
    return code;
}

#define HIPCHK(ctx, call)                                                          \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess)                                                      \
            return fail((ctx), RF_ERR_HIP,                                         \
                        std::string(#call ": ") + hipGetErrorString(e_));          \
    } while (0)

int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// The host's wait for the context's stream.  HIP's stream synchronize spins
// on the completion signal; with RF_OPT_SYNC_BLOCK the thread yields its core
// and then sleeps between polls of an event instead, so a rank held to a
// 2-core share leaves the core to its other host work (quality pass, table
// setup, another engine's thread) while its kernels run.  (Round 6: a
// blocking-sync hipEventSynchronize kept the waiting thread on its core --
// the native stage machine's thread CPU time equalled its wall time,
// profiles/r06e_e2e_phases.out.)  2: auto, block when this thread may run on
// fewer than 4 CPUs.
bool host_blocks(const rf_ctx *ctx)
{
    if (ctx->opt.sync_block == 2) {
        cpu_set_t cs;
        return sched_getaffinity(0, sizeof(cs), &cs) == 0 && CPU_COUNT(&cs) < 4;
    }
    return ctx->opt.sync_block == 1;
}

hipError_t stream_wait(rf_ctx *ctx)
{
    if (!ctx->ev_block || !host_blocks(ctx))
        return hipStreamSynchronize(ctx->stream);
    hipError_t e = hipEventRecord(ctx->ev_block, ctx->stream);
    if (e != hipSuccess)
        return e;
    const auto t0 = std::chrono::steady_clock::now();
    while ((e = hipEventQuery(ctx->ev_block)) == hipErrorNotReady) {
        if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200))
            sched_yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(30));
    }
    return e;
}

// before a device-to-host copy into host memory that may be pageable (HIP
// then copies through a staging buffer and spins until the stream reaches
// the copy): a blocking host waits for the stream first, so the copy is
// short
hipError_t pre_d2h(rf_ctx *ctx)
{
    return host_blocks(ctx) ? stream_wait(ctx) : hipSuccess;
}

int ensure_buf(rf_ctx *ctx, DevBuf &b, size_t bytes)
{
    if (b.cap >= bytes)
        return 0;
    if (b.p) {
        HIPCHK(ctx, stream_wait(ctx));
        HIPCHK(ctx, hipFree(b.p));
    }
    size_t cap = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    HIPCHK(ctx, hipMalloc(&b.p, cap));
    b.cap = cap;
    return 0;
}

#ifndef RF_UP_RING
#define RF_UP_RING (32 << 20)   // bytes of the pinned upload ring (0: pageable copies)
#endif
// `bytes` of the pinned upload ring for one H2D copy on the context's stream
// (*h = nullptr: too large for the ring, copy from pageable memory)
int ring_take(rf_ctx *ctx, size_t bytes, char **h)
{
    *h = nullptr;
    if (RF_UP_RING <= 0 || bytes > (size_t)RF_UP_RING / 4)
        return 0;
    if (!ctx->up) {
        if (hipHostMalloc(&ctx->up, RF_UP_RING, hipHostMallocDefault) != hipSuccess)
            return fail(ctx, RF_ERR_HIP, "pinned upload ring allocation failed");
        ctx->up_bytes = RF_UP_RING;
        ctx->up_off = 0;
    }
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (ctx->up_off + need > ctx->up_bytes) {
        // every copy out of the ring is on this stream: once it drains, the
        // ring is free again
        HIPCHK(ctx, stream_wait(ctx));
        ctx->up_off = 0;
    }
    *h = (char *)ctx->up + ctx->up_off;
    ctx->up_off += need;
    return 0;
}

template <class T>
int upload(rf_ctx *ctx, DevBuf &b, const std::vector<T> &v)
{
    const size_t bytes = v.size() * sizeof(T);
    if (int e = ensure_buf(ctx, b, std::max<size_t>(bytes, 16)))
        return e;
    if (!bytes)
        return 0;
    char *h;
    if (int e = ring_take(ctx, bytes, &h))
        return e;
    if (h)
        std::memcpy(h, v.data(), bytes);
    HIPCHK(ctx, hipMemcpyAsync(b.p, h ? (const void *)h : (const void *)v.data(), bytes, hipMemcpyHostToDevice,
                               ctx->stream));
    return 0;
}

// Collect every live region of an arena, for compaction.
void live_regions(rf_ctx *ctx, Arena *a, std::vector<Region *> &out)
{
    out.clear();
    if (a == &ctx->bytes_arena) {
        for (auto &s : ctx->seqs)
            if (s.bases.off >= 0) out.push_back(&s.bases);
        for (auto &t : ctx->tpls)
            if (t.bases.off >= 0) out.push_back(&t.bases);
    } else if (a == &ctx->tab_arena) {
        for (auto &s : ctx->seqs)
            if (s.tabs.off >= 0) out.push_back(&s.tabs);
    } else {
        for (auto &s : ctx->slots) {
            if (s.a.r.off >= 0) out.push_back(&s.a.r);
            if (s.b.r.off >= 0) out.push_back(&s.b.r);
        }
    }
}

// Grow (and compact) an arena so that `need` more bytes fit at the top.
// `skip` is a region about to be rewritten: its content is not preserved.
int arena_grow_impl(rf_ctx *ctx, Arena &a, int64_t need, Region *skip);
int arena_grow(rf_ctx *ctx, Arena &a, int64_t need, Region *skip)
{
    const auto t0 = std::chrono::steady_clock::now();
    const int e = arena_grow_impl(ctx, a, need, skip);
    ctx->arena_grow_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ++ctx->arena_grows;
    return e;
}

int arena_grow_impl(rf_ctx *ctx, Arena &a, int64_t need, Region *skip)
{
    std::vector<Region *> regs;
    live_regions(ctx, &a, regs);
    int64_t live = 0;
    for (auto *r : regs)
        if (r != skip)
            live += r->cap;
    int64_t cap = std::max<int64_t>(live + need + 2 * ARENA_GUARD, (int64_t)(a.cap * 1.5));
    cap = align_up(cap + cap / 8 + (1 << 20), 1 << 20);
    char *d = nullptr;
    HIPCHK(ctx, hipMalloc((void **)&d, cap));
    std::sort(regs.begin(), regs.end(), [](Region *x, Region *y) { return x->off < y->off; });
    // compaction = one scatter launch (one block per live region), not one
    // copy dispatch per region: a batch upload that grows an arena log(N)
    // times would otherwise issue O(N log N) tiny copies
    std::vector<Segment> segs;
    segs.reserve(regs.size());
    int64_t top = ARENA_GUARD;   // guard bytes before the first region
    for (auto *r : regs) {
        if (r == skip) {
            r->off = -1;
            r->cap = 0;
            continue;
        }
        if (r->cap > 0)
            segs.push_back({r->off, top, r->cap, 0});
        r->off = top;
        top += r->cap;
    }
    if (!segs.empty()) {
        if (int e = upload(ctx, ctx->grow_segs, segs))
            return e;
        hipLaunchKernelGGL(k_scatter, dim3((unsigned)segs.size()), dim3(256), 0, ctx->stream,
                           (const Segment *)ctx->grow_segs.p, (const uint8_t *)a.d, (uint8_t *)d);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, stream_wait(ctx));
    if (a.d)
        HIPCHK(ctx, hipFree(a.d));
    a.d = d;
    a.cap = cap;
    a.top = top;
    ++ctx->layout_gen;
    return 0;
}

int region_ensure(rf_ctx *ctx, Arena &a, Region &r, int64_t bytes)
{
    bytes = align_up(std::max<int64_t>(bytes, 16), 256);
    if (r.off >= 0 && r.cap >= bytes)
        return 0;
    if (a.top + bytes + ARENA_GUARD > a.cap)
        if (int e = arena_grow(ctx, a, bytes, &r))
            return e;
    r.off = a.top;
    r.cap = bytes;
    a.top += bytes;
    ++ctx->layout_gen;
    return 0;
}

// The error flag and `bytes` of results land in ctx->hout (pinned, 16-B
// error slot first); returns the results' host address.
int ensure_hout(rf_ctx *ctx, size_t bytes)
{
    const size_t want = 16 + bytes;
    if (ctx->hout_bytes >= want)
        return 0;
    if (ctx->hout)
        (void)hipHostFree(ctx->hout);
    ctx->hout = nullptr;
    ctx->hout_bytes = 0;
    const size_t sz = std::max<size_t>(want, 1 << 20);
    if (hipHostMalloc(&ctx->hout, sz, hipHostMallocDefault) != hipSuccess)
        return fail(ctx, RF_ERR_HIP, "pinned result buffer allocation failed");
    ctx->hout_bytes = sz;
    return 0;
}

// After the stream was synchronized with the error flag copied to hout.
int check_err_landed(rf_ctx *ctx)
{
    const int h = *(const int *)ctx->hout;
    if (h) {
        int z = 0;
        HIPCHK(ctx, hipMemcpy(ctx->d_err, &z, sizeof(int), hipMemcpyHostToDevice));
        return fail(ctx, RF_ERR_NUMERIC, numeric_message(h));
    }
    return 0;
}

// Downloads of a call land in ctx->hdn (pinned: a pageable D2H copy is
// staged by the runtime through a blit and a wait of its own): the error
// flag at offset 0 (land_err), results from HDN_RES; the call queues them
// behind its kernels, waits once, then copies the results out.
constexpr size_t HDN_RES = 16;
int ensure_hdn(rf_ctx *ctx, size_t bytes)
{
    const size_t want = HDN_RES + bytes;
    if (ctx->hdn_bytes >= want)
        return 0;
    if (ctx->hdn) {
        HIPCHK(ctx, stream_wait(ctx));
        (void)hipHostFree(ctx->hdn);
    }
    ctx->hdn = nullptr;
    ctx->hdn_bytes = 0;
    const size_t sz = std::max<size_t>(want + want / 4, 1 << 20);
    if (hipHostMalloc(&ctx->hdn, sz, hipHostMallocDefault) != hipSuccess)
        return fail(ctx, RF_ERR_HIP, "pinned download buffer allocation failed");
    ctx->hdn_bytes = sz;
    return 0;
}

// queue the error flag's copy into ctx->hdn (after ensure_hdn)
hipError_t land_err(rf_ctx *ctx)
{
    return hipMemcpyAsync(ctx->hdn, ctx->d_err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream);
}

// after the stream wait: the landed error flag
int check_err_hdn(rf_ctx *ctx)
{
    const int h = *(const int *)ctx->hdn;
    if (h) {
        int z = 0;
        HIPCHK(ctx, hipMemcpy(ctx->d_err, &z, sizeof(int), hipMemcpyHostToDevice));
        return fail(ctx, RF_ERR_NUMERIC, numeric_message(h));
    }
    return 0;
}

int check_err(rf_ctx *ctx)
{
    if (int e = ensure_hdn(ctx, 0))
        return e;
    HIPCHK(ctx, pre_d2h(ctx));
    HIPCHK(ctx, land_err(ctx));
    HIPCHK(ctx, stream_wait(ctx));
    return check_err_hdn(ctx);
}

int band_rows(int n, int m, int bw) { return 2 * bw + std::abs(n - m) + 1; }

// k_score stages the kappa rows of a work item through LDS; size the
// per-band buffer for the 90th-percentile window (at most 24 KB per band,
// two bands per single-wave block), larger windows read in place.
int score_lds_elems(const std::vector<ScoreRead> &reads)
{
    if (reads.empty())
        return 0;
    std::vector<int> w;
    w.reserve(reads.size());
    for (const auto &R : reads)
        w.push_back((2 * SCORE_C + R.H) * R.P);
    const size_t q = (w.size() * 9) / 10;
    std::nth_element(w.begin(), w.begin() + q, w.end());
    return std::min(w[q], 24 * 1024 / 8);
}


int env_int(const char *name, int dflt)
{
    const char *v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

// option defaults from the environment (rf_create only)
void load_env_opts(Opts &o)
{
    if (const char *k = std::getenv("RIFRAF_SCORE_KERNEL"))
        o.score_kernel = !std::strcmp(k, "general") ? 1 : !std::strcmp(k, "seg") ? 2 : !std::strcmp(k, "ws") ? 3 : 0;
    if (const char *m = std::getenv("RIFRAF_SCORE_MODE"))
        o.score_mode = !std::strcmp(m, "fused") ? 1 : !std::strcmp(m, "split") ? 2 : 0;
    o.lean_lds_kb = env_int("RIFRAF_LEAN_LDS_KB", o.lean_lds_kb);
    o.dp_psplit = env_int("RIFRAF_DP_PSPLIT", o.dp_psplit);
    o.dp_np8 = env_int("RIFRAF_DP_NO_NP8", 0) ? 0 : 1;
    o.dp_np8_lean = env_int("RIFRAF_DP_NP8_LEAN", o.dp_np8_lean);
    o.dp_streams = env_int("RIFRAF_DP_STREAMS", o.dp_streams);
    o.bt_win_kb = env_int("RIFRAF_BT_WIN_KB", o.bt_win_kb);
    o.band_pad_h = env_int("RIFRAF_BAND_PAD", o.band_pad_h);
    o.dp_wide = env_int("RIFRAF_DP_WIDE", o.dp_wide);
    o.aln_sums_host = env_int("RIFRAF_ALN_SUMS_HOST", o.aln_sums_host);
    o.sync_block = env_int("RIFRAF_SYNC_BLOCK", o.sync_block);
    o.dp_nl64 = env_int("RIFRAF_DP_NL64", o.dp_nl64);
    o.dp_lat = env_int("RIFRAF_DP_LAT", o.dp_lat);
    o.score_wgs = env_int("RIFRAF_SCORE_WGS", o.score_wgs);
    o.seg_wgs = env_int("RIFRAF_SEG_WGS", o.seg_wgs);
    o.dp_pfit = env_int("RIFRAF_DP_PFIT", o.dp_pfit);
    o.dp_mc = env_int("RIFRAF_DP_MC", o.dp_mc);
    o.bt_nw = env_int("RIFRAF_BT_NW", o.bt_nw);
}

ScorePick pick_scorer(const Opts &o, const std::vector<ScoreRead> &reads, bool all_finite)
{
    ScorePick p;
    const bool force_general = o.score_kernel == 1;
    const bool force_seg = o.score_kernel == 2;
    if (all_finite && !force_general && !force_seg && !reads.empty()) {
        int need1 = 0;
        for (const auto &R : reads)
            need1 = std::max(need1, lean_need(1, R.H, R.P));
        // k_score_ws: 256 chain lanes + 256 loader lanes, one workgroup per CU
        // (measured at c4: 128 chain lanes (two workgroups per CU) +14 %,
        // 320 / 384 chain lanes +50 % scoring time)
        const int lds = std::max((o.lean_lds_kb > 0 ? o.lean_lds_kb : 160) * 1024 / 8, need1);
        // Round 5: a read whose 256-column window exceeds LDS runs in sub-
        // windows over a half (or less) of the chain lanes, the others idle;
        // when such reads hold most of the launch's cells, the segment scorer
        // (LDS independent of H) is faster -- configs[2]'s doubled bands
        // (bw 18, H ~ 37-51): 1.50 -> 0.65 ms per dense pass,
        // profiles/r05q_c3_score_kernel.jsonl
        double wide = 0.0, all = 0.0;
        for (const auto &R : reads) {
            const double w = (double)R.n * R.H;
            all += w;
            if (lean_need(256, R.H, R.P) > lds)
                wide += w;
        }
        if (lds <= 160 * 1024 / 8 && (o.score_kernel == 3 || !(2.0 * wide > all))) {
            p.lean = true;
            p.lds = lds;
            return p;
        }
    }
    // wide bands: the row-segment scorer (same chains, H-independent LDS)
    if (all_finite && !force_general && !reads.empty()) {
        p.seg = true;
        return p;
    }
    p.lds = score_lds_elems(reads);
    return p;
}

// work items: chunks of q consecutive positions of every group
std::vector<WorkItem> make_items(const std::vector<ScoreGroup> &groups, int q)
{
    std::vector<WorkItem> items;
    for (int g = 0; g < (int)groups.size(); ++g)
        if (groups[g].r1 > groups[g].r0)
            for (int p0 = 0; p0 <= groups[g].m; p0 += q)
                items.push_back({g, p0});
    return items;
}

void launch_scorer(rf_ctx *ctx, const ScorePick &pk, unsigned nitems, unsigned gy, const WorkItem *items,
                   const ScoreGroup *groups, const ScoreRead *reads, double *dense, double *split)
{
    const uint8_t *d_bases = (const uint8_t *)ctx->bytes_arena.d;
    const double *d_tabs = (const double *)ctx->tab_arena.d;
    const double *d_bands = (const double *)ctx->band_arena.d;
    int sm = split ? 1 : 0;
    dim3 grid(nitems, gy);
    if (pk.seg) {
        int rchunk = 1;
        if (split) {
            const int64_t tgt = std::max(ctx->opt.seg_wgs, 1);
            rchunk = (int)std::max<int64_t>(1, ((int64_t)nitems * gy + tgt - 1) / tgt);
            grid.y = (gy + rchunk - 1) / rchunk;
        }
        hipLaunchKernelGGL(k_score_segl<32>, grid, dim3(64), 0, ctx->stream, items, groups, reads, d_bases, d_tabs,
                           d_bands, dense, split, sm, rchunk);
    } else if (!pk.lean) {
        hipLaunchKernelGGL(k_score, grid, dim3(128), 2 * pk.lds * 8, ctx->stream, items, groups, reads,
                           d_bases, d_tabs, d_bands, dense, split, sm, pk.lds);
    } else {
        // split: enough reads per workgroup for the loaders' prefetch to
        // overlap the chains, still >= 2,048 workgroups (one per CU at a time)
        int rchunk = 1;
        if (split) {
            rchunk = (int)std::max<int64_t>(1, ((int64_t)nitems * gy) / std::max(ctx->opt.score_wgs, 1));
            grid.y = (gy + rchunk - 1) / rchunk;
        }
        hipLaunchKernelGGL((k_score_ws<WS_NPF, 256>), grid, dim3(512), pk.lds * 8, ctx->stream, items,
                           groups, reads, d_bases, d_tabs, d_bands, dense, split, sm, pk.lds,
                           WS_CODES ? (const double *)ctx->codes.lut.p : nullptr, rchunk);
    }
}

}  // namespace

// rf_last_error text for the host stage machine in rifraf_batch.cpp (same
// library, C++ linkage, not part of the C-ABI)
int rf_internal_fail(rf_ctx *ctx, int code, const char *msg)
{
    return fail(ctx, code, msg ? msg : "");
}

extern "C" {

int rf_abi_version(void) { return RF_ABI_VERSION; }

int rf_create(int device, rf_ctx **out)
{
    if (!out)
        return RF_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return RF_ERR_HIP;
    if (device < 0 || device >= ndev)
        return RF_ERR_ARG;
    rf_ctx *ctx = new rf_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&ctx->d_err, sizeof(int)) != hipSuccess ||
        hipMemset(ctx->d_err, 0, sizeof(int)) != hipSuccess) {
        delete ctx;
        return RF_ERR_HIP;
    }
    load_env_opts(ctx->opt);
    for (auto &e : ctx->ev)
        (void)hipEventCreate(&e);
    (void)hipEventCreate(&ctx->ev_codon);
    (void)hipEventCreateWithFlags(&ctx->ev_block, hipEventBlockingSync | hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming);
    for (int i = 0; i < 3; ++i) {
        (void)hipStreamCreateWithFlags(&ctx->side[i], hipStreamNonBlocking);
        (void)hipEventCreateWithFlags(&ctx->join[i], hipEventDisableTiming);
    }
    // the lean scorer may use up to the whole 160 KiB LDS of a CU, and so may
    // the block-wide DP's ring
    (void)hipFuncSetAttribute((const void *)k_score_ws<WS_NPF, 256>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void *)k_dp<DPW_NT, false, DPW_NT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    *out = ctx;
    return 0;
}

int rf_destroy(rf_ctx *ctx)
{
    if (!ctx)
        return 0;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (Arena *a : {&ctx->bytes_arena, &ctx->tab_arena, &ctx->band_arena})
        if (a->d)
            (void)hipFree(a->d);
    for (auto &b : ctx->scratch)
        if (b.p)
            (void)hipFree(b.p);
    if (ctx->grow_segs.p)
        (void)hipFree(ctx->grow_segs.p);
    if (ctx->codes.lut.p)
        (void)hipFree(ctx->codes.lut.p);
    if (ctx->codes.errlut.p)
        (void)hipFree(ctx->codes.errlut.p);
    if (ctx->pinned)
        (void)hipHostFree(ctx->pinned);
    if (ctx->hout)
        (void)hipHostFree(ctx->hout);
    if (ctx->up)
        (void)hipHostFree(ctx->up);
    if (ctx->hdn)
        (void)hipHostFree(ctx->hdn);
    if (ctx->d_err)
        (void)hipFree(ctx->d_err);
    for (auto &e : ctx->ev)
        (void)hipEventDestroy(e);
    if (ctx->ev_codon)
        (void)hipEventDestroy(ctx->ev_codon);
    if (ctx->ev_block)
        (void)hipEventDestroy(ctx->ev_block);
    for (int i = 0; i < 3; ++i) {
        if (ctx->side[i]) {
            (void)hipStreamSynchronize(ctx->side[i]);
            (void)hipStreamDestroy(ctx->side[i]);
        }
        if (ctx->join[i])
            (void)hipEventDestroy(ctx->join[i]);
    }
    if (ctx->fork)
        (void)hipEventDestroy(ctx->fork);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return 0;
}

const char *rf_last_error(const rf_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

static int *opt_slot(rf_ctx *ctx, int32_t key)
{
    Opts &o = ctx->opt;
    switch (key) {
    case RF_OPT_SCORE_MODE: return &o.score_mode;
    case RF_OPT_SCORE_KERNEL: return &o.score_kernel;
    case RF_OPT_LEAN_LDS_KB: return &o.lean_lds_kb;
    case RF_OPT_DP_PSPLIT: return &o.dp_psplit;
    case RF_OPT_DP_NP8: return &o.dp_np8;
    case RF_OPT_DP_NP8_LEAN: return &o.dp_np8_lean;
    case RF_OPT_DP_STREAMS: return &o.dp_streams;
    case RF_OPT_BT_WIN_KB: return &o.bt_win_kb;
    case RF_OPT_STAGE_KB: return &o.stage_kb;
    case RF_OPT_BAND_PAD: return &o.band_pad_h;
    case RF_OPT_DP_WIDE: return &o.dp_wide;
    case RF_OPT_ALN_SUMS_HOST: return &o.aln_sums_host;
    case RF_OPT_ALN_MARKS_MIN: return &o.aln_marks_min;
    case RF_OPT_SYNC_BLOCK: return &o.sync_block;
    case RF_OPT_DP_NL64: return &o.dp_nl64;
    case RF_OPT_DP_LAT: return &o.dp_lat;
    case RF_OPT_SCORE_WGS: return &o.score_wgs;
    case RF_OPT_SEG_WGS: return &o.seg_wgs;
    case RF_OPT_DP_PFIT: return &o.dp_pfit;
    case RF_OPT_DP_MC: return &o.dp_mc;
    case RF_OPT_BT_NW: return &o.bt_nw;
    default: return nullptr;
    }
}

int rf_set_option(rf_ctx *ctx, int32_t key, int32_t value)
{
    if (!ctx)
        return RF_ERR_ARG;
    int *s = opt_slot(ctx, key);
    if (!s)
        return fail(ctx, RF_ERR_ARG, "rf_set_option: unknown option");
    if (*s != value) {
        *s = value;
        ++ctx->opt_gen;
        ctx->rplan.valid = false;   // DP class split depends on options
    }
    return 0;
}

int rf_get_option(rf_ctx *ctx, int32_t key, int32_t *value)
{
    if (!ctx || !value)
        return RF_ERR_ARG;
    int *s = opt_slot(ctx, key);
    if (!s)
        return fail(ctx, RF_ERR_ARG, "rf_get_option: unknown option");
    *value = *s;
    return 0;
}

int rf_reserve(rf_ctx *ctx, int64_t band_bytes)
{
    if (!ctx || band_bytes < 0)
        return RF_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    if (ctx->band_arena.cap - ctx->band_arena.top >= band_bytes + ARENA_GUARD)
        return 0;   // room already: nothing moves, cached plans stay valid
    ++ctx->state_epoch;   // regions move (arena_grow also bumps layout_gen)
    return arena_grow(ctx, ctx->band_arena, band_bytes, nullptr);
}

int rf_release_bands(rf_ctx *ctx)
{
    if (!ctx)
        return RF_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    HIPCHK(ctx, stream_wait(ctx));   // no launch still reads or writes a band
    for (auto &s : ctx->slots)
        for (Band *b : {&s.a, &s.b}) {
            b->valid = false;
            b->r.off = -1;
            b->r.cap = 0;
        }
    ctx->band_arena.top = ARENA_GUARD;
    ++ctx->layout_gen;
    ++ctx->state_epoch;
    return 0;
}

int rf_code_stats(const rf_ctx *ctx, int64_t *entries3, int64_t *entries1, int64_t *uncoded_reads,
                  int64_t *resets)
{
    if (!ctx)
        return RF_ERR_ARG;
    if (entries3)
        *entries3 = (int64_t)ctx->codes.t3.size();
    if (entries1)
        *entries1 = (int64_t)ctx->codes.d1.size();
    if (uncoded_reads)
        *uncoded_reads = ctx->codes.uncoded_reads;
    if (resets)
        *resets = ctx->codes.resets;
    return 0;
}

int64_t rf_device_bytes(const rf_ctx *ctx)
{
    if (!ctx)
        return 0;
    int64_t t = ctx->bytes_arena.cap + ctx->tab_arena.cap + ctx->band_arena.cap;
    for (auto &b : ctx->scratch)
        t += (int64_t)b.cap;
    return t;
}

// rf_set_sequences's staging of sequences [k0, k1) of one call (their regions
// exist): host tables + row codes into pinned memory, H2D, device scatter.
int upload_sequence_chunk(rf_ctx *ctx, int32_t first, int32_t k0, int32_t k1, const uint8_t *bases,
                          const int64_t *off, const double *match, const double *mismatch, const double *ins,
                          const double *del, const double *cins, const int64_t *cins_off, const double *cdel,
                          const int64_t *cdel_off)
{
    int64_t nt = 0, nb = 0;
    for (int32_t k = k0; k < k1; ++k) {
        const SeqObj &S = ctx->seqs[first + k];
        nt += row_code_off(S.n, S.ncins, S.ncdel) + S.n;
        nb += S.n;
    }
    const int32_t nseq = k1 - k0;
    const size_t stage_bytes = (size_t)std::max<int64_t>(nt, 1) * 8 + (size_t)std::max<int64_t>(nb, 1);
    if (ctx->pinned_bytes < stage_bytes) {
        if (ctx->pinned)
            (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
        const size_t want = std::max(stage_bytes + stage_bytes / 2, (size_t)1 << 22);
        if (hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault) != hipSuccess)
            return fail(ctx, RF_ERR_HIP, "rf_set_sequences: pinned staging allocation failed");
        ctx->pinned_bytes = want;
    }
    double *host_tabs = (double *)ctx->pinned;
    uint8_t *host_bases = (uint8_t *)ctx->pinned + (size_t)std::max<int64_t>(nt, 1) * 8;
    std::vector<Segment> sb(nseq), st(nseq);
    std::vector<int64_t> at(nseq + 1, 0);
    for (int32_t k = 0; k < nseq; ++k) {
        const SeqObj &S = ctx->seqs[first + k0 + k];
        at[k + 1] = at[k] + row_code_off(S.n, S.ncins, S.ncdel) + S.n;
        st[k] = {at[k] * 8, S.tabs.off, (at[k + 1] - at[k]) * 8, 0};
        sb[k] = {off[k0 + k] - off[k0], S.bases.off, S.n, 0};
    }
    // The host work per position (staging copies, the finiteness test, the
    // row codes) runs on host threads over ranges of sequences.  Row codes in
    // three passes so the dictionary is only written by one thread: new keys
    // per range (read-only lookups), their insertion in range order (= the
    // serial first-occurrence order), then the records (read-only lookups).
    const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), (nt + (1 << 20) - 1) >> 20));
    std::vector<int32_t> rng(nth + 1);
    for (int t = 0; t <= nth; ++t)
        rng[t] = (int32_t)((int64_t)nseq * t / nth);
    CodeDict &D = ctx->codes;
    auto table = [&](int32_t k) { return host_tabs + at[k]; };
    std::vector<std::vector<CodeDict::K3>> new3(nth);
    std::vector<std::vector<uint64_t>> new1(nth);
    parallel_for(nth, [&](int t) {
        std::unordered_set<CodeDict::K3, CodeDict::H3> s3;
        std::unordered_set<uint64_t> s1;
        CodeDict::Cache cache;
        for (int32_t k = rng[t]; k < rng[t + 1]; ++k) {
            const SeqObj &S = ctx->seqs[first + k0 + k];
            const int64_t n = S.n, nci = S.ncins, ncd = S.ncdel;
            double *h = table(k);
            const int32_t kg = k0 + k;   // index into the caller's arrays
            std::memcpy(h, match + off[kg], n * 8);
            std::memcpy(h + n, mismatch + off[kg], n * 8);
            std::memcpy(h + 2 * n, ins + off[kg], n * 8);
            std::memcpy(h + 3 * n, del + off[kg] + kg, (n + 1) * 8);
            if (nci)
                std::memcpy(h + 4 * n + 1, cins + cins_off[kg], nci * 8);
            if (ncd)
                std::memcpy(h + 4 * n + 1 + nci, cdel + cdel_off[kg], ncd * 8);
            bool fin = true;
            for (int64_t e = 0; e < 4 * n + 1; ++e)
                fin = fin && std::isfinite(h[e]);
            ctx->seqs[first + k0 + k].finite = fin;
            for (int64_t i = 0; i < n; ++i) {
                const CodeDict::K3 key{CodeDict::bits(h[i]), CodeDict::bits(h[n + i]), CodeDict::bits(h[2 * n + i])};
                if (D.find3(key, cache) < 0 && s3.insert(key).second)
                    new3[t].push_back(key);
            }
            for (int64_t i = 0; i <= n; ++i) {
                const uint64_t key = CodeDict::bits(h[3 * n + i]);
                if (D.find1(key, cache) < 0 && s1.insert(key).second)
                    new1[t].push_back(key);
            }
        }
    });
    for (int t = 0; t < nth; ++t) {
        for (const auto &key : new3[t])
            if (D.find3(key) < 0 && D.t3.size() < (size_t)RF_CODES) {
                D.t3.emplace(key, (uint32_t)D.t3.size());
                double v[3];
                std::memcpy(v, &key.a, 8), std::memcpy(v + 1, &key.b, 8), std::memcpy(v + 2, &key.c, 8);
                D.t3v.insert(D.t3v.end(), {v[0], v[1], v[2], 0.0});
            }
        for (uint64_t key : new1[t])
            if (D.find1(key) < 0 && D.d1.size() < (size_t)RF_CODES) {
                D.d1.emplace(key, (uint32_t)D.d1.size());
                double v;
                std::memcpy(&v, &key, 8);
                D.d1v.push_back(v);
            }
    }
    parallel_for(nth, [&](int t) {
        CodeDict::Cache cache;
        for (int32_t k = rng[t]; k < rng[t + 1]; ++k) {
            const SeqObj &S = ctx->seqs[first + k0 + k];
            const int64_t n = S.n;
            const double *h = table(k);
            uint64_t *rec = (uint64_t *)(table(k) + row_code_off(n, S.ncins, S.ncdel));
            const uint8_t *bs = bases + off[k0 + k];
            bool ok = true;
            int32_t dprev = D.find1(CodeDict::bits(h[3 * n]), cache);
            ok = dprev >= 0;
            for (int64_t i = 0; i < n && ok; ++i) {
                const int32_t c3 = D.find3({CodeDict::bits(h[i]), CodeDict::bits(h[n + i]), CodeDict::bits(h[2 * n + i])}, cache);
                const int32_t dn = D.find1(CodeDict::bits(h[3 * n + i + 1]), cache);
                ok = c3 >= 0 && dn >= 0;
                rec[i] = (uint64_t)(uint32_t)c3 | ((uint64_t)(uint32_t)dprev << 16) | ((uint64_t)(uint32_t)dn << 32) |
                         ((uint64_t)bs[i] << 48);
                dprev = dn;
            }
            ctx->seqs[first + k0 + k].coded = ok;
        }
    });
    for (int32_t k = 0; k < nseq; ++k)
        D.uncoded_reads += ctx->seqs[first + k0 + k].coded ? 0 : 1;
    // 3. new code-dictionary entries, one H2D copy each + device scatter
    {
        CodeDict &D = ctx->codes;
        if (int e = ensure_buf(ctx, D.lut, (size_t)RF_CODES * 5 * 8)) return e;
        const size_t n3 = D.t3v.size() / 4, n1 = D.d1v.size();
        if (n3 > D.up3)
            HIPCHK(ctx, hipMemcpyAsync((double *)D.lut.p + 4 * D.up3, D.t3v.data() + 4 * D.up3, (n3 - D.up3) * 32,
                                       hipMemcpyHostToDevice, ctx->stream));
        if (n1 > D.up1)
            HIPCHK(ctx, hipMemcpyAsync((double *)D.lut.p + 4 * (size_t)RF_CODES + D.up1, D.d1v.data() + D.up1,
                                       (n1 - D.up1) * 8, hipMemcpyHostToDevice, ctx->stream));
        D.up3 = n3;
        D.up1 = n1;
    }
    if (int e = ensure_buf(ctx, ctx->scratch[6], (size_t)std::max<int64_t>(nt * 8, 16))) return e;
    if (int e = ensure_buf(ctx, ctx->scratch[7], (size_t)std::max<int64_t>(nb, 16))) return e;
    if (nseq > 0) {
        std::memcpy(host_bases, bases + off[k0], nb);
        HIPCHK(ctx, hipMemcpyAsync(ctx->scratch[6].p, host_tabs, nt * 8, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(ctx->scratch[7].p, host_bases, nb, hipMemcpyHostToDevice, ctx->stream));
        if (int e = upload(ctx, ctx->scratch[5], st)) return e;
        hipLaunchKernelGGL(k_scatter, dim3(nseq), dim3(256), 0, ctx->stream, (const Segment *)ctx->scratch[5].p,
                           (const uint8_t *)ctx->scratch[6].p, (uint8_t *)ctx->tab_arena.d);
        HIPCHK(ctx, stream_wait(ctx));   // scratch[5] is reused below
        if (int e = upload(ctx, ctx->scratch[5], sb)) return e;
        hipLaunchKernelGGL(k_scatter, dim3(nseq), dim3(256), 0, ctx->stream, (const Segment *)ctx->scratch[5].p,
                           (const uint8_t *)ctx->scratch[7].p, (uint8_t *)ctx->bytes_arena.d);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, stream_wait(ctx));
    }
    return 0;
}

int rf_set_sequences(rf_ctx *ctx, int32_t first, int32_t nseq, const uint8_t *bases,
                     const int64_t *off, const double *match, const double *mismatch,
                     const double *ins, const double *del, const double *cins,
                     const int64_t *cins_off, const double *cdel, const int64_t *cdel_off)
{
    if (!ctx || first < 0 || nseq < 0 || (nseq > 0 && (!bases || !off || !match || !mismatch || !ins || !del)))
        return fail(ctx, RF_ERR_ARG, "rf_set_sequences: bad arguments");
    (void)hipSetDevice(ctx->device);
    ++ctx->state_epoch;
    if ((int64_t)first + nseq > (int64_t)ctx->seqs.size())
        ctx->seqs.resize(first + nseq);
    // a fresh code dictionary when no coded sequence outside this upload is
    // still valid (nothing references the old codes)
    {
        bool others = false;
        for (size_t k = 0; k < ctx->seqs.size() && !others; ++k)
            others = ((int64_t)k < first || (int64_t)k >= (int64_t)first + nseq) && ctx->seqs[k].valid &&
                     ctx->seqs[k].coded;
        if (!others && !(ctx->codes.t3.empty() && ctx->codes.d1.empty()))
            ctx->codes.reset();
    }
    // 0. grow each arena at most once for the whole batch
    {
        int64_t need_b = 0, need_t = 0;
        for (int32_t k = 0; k < nseq; ++k) {
            const SeqObj &S = ctx->seqs[first + k];
            const int64_t n = off[k + 1] - off[k];
            const int64_t nci = cins_off ? cins_off[k + 1] - cins_off[k] : 0;
            const int64_t ncd = cdel_off ? cdel_off[k + 1] - cdel_off[k] : 0;
            const int64_t bb = align_up(std::max<int64_t>(n, 16), 256);
            const int64_t tb = align_up(std::max<int64_t>((row_code_off(n, nci, ncd) + n) * 8, 16), 256);
            if (!(S.bases.off >= 0 && S.bases.cap >= bb)) need_b += bb;
            if (!(S.tabs.off >= 0 && S.tabs.cap >= tb)) need_t += tb;
        }
        if (ctx->bytes_arena.top + need_b + ARENA_GUARD > ctx->bytes_arena.cap)
            if (int e = arena_grow(ctx, ctx->bytes_arena, need_b, nullptr)) return e;
        if (ctx->tab_arena.top + need_t + ARENA_GUARD > ctx->tab_arena.cap)
            if (int e = arena_grow(ctx, ctx->tab_arena, need_t, nullptr)) return e;
    }
    // 1. regions (arena growth may move earlier regions: offsets are read after)
    int64_t nb = 0, nt = 0;
    for (int32_t k = 0; k < nseq; ++k) {
        SeqObj &S = ctx->seqs[first + k];
        const int64_t n = off[k + 1] - off[k];
        const int64_t nci = cins_off ? cins_off[k + 1] - cins_off[k] : 0;
        const int64_t ncd = cdel_off ? cdel_off[k + 1] - cdel_off[k] : 0;
        if (n < 1 || (nci != 0 && nci != n - 2) || (ncd != 0 && ncd != n + 1))
            return fail(ctx, RF_ERR_ARG, "rf_set_sequences: inconsistent table lengths");
        S.n = (int32_t)n;
        S.ncins = (int32_t)nci;
        S.ncdel = (int32_t)ncd;
        if (int e = region_ensure(ctx, ctx->bytes_arena, S.bases, n))
            return e;
        // tables [match|mismatch|ins|del|cins|cdel], then one row-code record per position
        if (int e = region_ensure(ctx, ctx->tab_arena, S.tabs, (row_code_off(n, nci, ncd) + n) * 8))
            return e;
        nb += n;
        nt += row_code_off(n, nci, ncd) + n;
    }
    // 2.-3. in chunks of at most RF_OPT_STAGE_KB of tables (a bounded pinned
    // staging buffer and device scratch, whatever the batch size): pack the
    // chunk's tables [match|mismatch|ins|del|cins|cdel|row codes] and bases
    // into pinned memory, then one H2D copy each + a device scatter.
    (void)nb;
    (void)nt;
    int32_t k0 = 0;
    while (k0 < nseq) {
        int32_t k1 = k0;
        int64_t ct = 0;
        while (k1 < nseq) {
            const SeqObj &S = ctx->seqs[first + k1];
            const int64_t len = row_code_off(S.n, S.ncins, S.ncdel) + S.n;
            if (k1 > k0 && (ct + len) * 8 > (int64_t)std::max(ctx->opt.stage_kb, 1) * 1024)
                break;
            ct += len;
            ++k1;
        }
        if (int e = upload_sequence_chunk(ctx, first, k0, k1, bases, off, match, mismatch, ins, del, cins, cins_off,
                                          cdel, cdel_off))
            return e;
        k0 = k1;
    }
    for (int32_t k = 0; k < nseq; ++k)
        ctx->seqs[first + k].valid = true;
    ++ctx->layout_gen;
    return 0;
}

static int set_sequences_codes_impl(rf_ctx *ctx, int32_t first, int32_t nseq, const uint8_t *bases,
                                    const int64_t *off, const uint8_t *codes, const double *lp_t,
                                    const double *match_t, double s_mis, double s_ins, double s_del,
                                    const double *p10_t, const double *grid, double *est, int32_t *ucode,
                                    double *tsum)
{
    const bool prep = p10_t != nullptr;
    if (!ctx || first < 0 || nseq < 0 || (nseq > 0 && (!bases || !off || !codes || !lp_t || !match_t)))
        return fail(ctx, RF_ERR_ARG, "rf_set_sequences_codes: bad arguments");
    (void)hipSetDevice(ctx->device);
    ++ctx->state_epoch;
    for (int32_t k = 0; k < nseq; ++k)
        if (off[k + 1] - off[k] < 1)
            return fail(ctx, RF_ERR_ARG, "rf_set_sequences_codes: empty sequence");
    const int64_t N = nseq > 0 ? off[nseq] - off[0] : 0;
    // codes present, per-code values and finiteness
    bool present[256] = {};
    {
        // one byte store per position (~0.5 ns): threads from 512 K positions
        // (c3's 2.6 M: 1.3 ms on one thread)
        const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), (N >> 19) + 1));
        std::vector<std::array<uint8_t, 256>> pr(nth);
        parallel_for(nth, [&](int t) {
            pr[t].fill(0);
            for (int64_t i = off[0] + N * t / nth; i < off[0] + N * (t + 1) / nth; ++i)
                pr[t][codes[i]] = 1;
        });
        for (int t = 0; t < nth; ++t)
            for (int c = 0; c < 256; ++c)
                present[c] = present[c] || pr[t][c];
    }
    double mt[256], mm[256], is[256], dl[256];
    bool fin[256];
    for (int c = 0; c < 256; ++c) {
        mt[c] = match_t[c];
        mm[c] = lp_t[c] + s_mis;
        is[c] = lp_t[c] + s_ins;
        dl[c] = lp_t[c] + s_del;
        fin[c] = std::isfinite(mt[c]) && std::isfinite(mm[c]) && std::isfinite(is[c]) && std::isfinite(dl[c]);
    }
    // a fresh code dictionary when no coded sequence outside this upload is
    // still valid (as rf_set_sequences)
    {
        bool others = false;
        for (size_t k = 0; k < ctx->seqs.size() && !others; ++k)
            others = ((int64_t)k < first || (int64_t)k >= (int64_t)first + nseq) && ctx->seqs[k].valid &&
                     ctx->seqs[k].coded;
        if (!others && !(ctx->codes.t3.empty() && ctx->codes.d1.empty()))
            ctx->codes.reset();
    }
    CodeDict &D = ctx->codes;
    std::vector<CodeLut> lut(256);
    // entries added by this call, dropped again if the dictionary fills up
    // (the caller then uploads host tables; codes no sequence uses must not
    // crowd out later uploads)
    std::vector<CodeDict::K3> added3;
    std::vector<uint64_t> added1;
    for (int c = 0; c < 256; ++c) {
        lut[c] = {lp_t[c], mt[c], 0, 0, 0, 0};
        if (!present[c])
            continue;
        const CodeDict::K3 key{CodeDict::bits(mt[c]), CodeDict::bits(mm[c]), CodeDict::bits(is[c])};
        int32_t i3 = D.find3(key);
        if (i3 < 0 && D.t3.size() < (size_t)RF_CODES) {
            i3 = (int32_t)D.t3.size();
            D.t3.emplace(key, (uint32_t)i3);
            D.t3v.insert(D.t3v.end(), {mt[c], mm[c], is[c], 0.0});
            added3.push_back(key);
        }
        int32_t i1 = D.find1(CodeDict::bits(dl[c]));
        if (i1 < 0 && D.d1.size() < (size_t)RF_CODES) {
            i1 = (int32_t)D.d1.size();
            D.d1.emplace(CodeDict::bits(dl[c]), (uint32_t)i1);
            D.d1v.push_back(dl[c]);
            added1.push_back(CodeDict::bits(dl[c]));
        }
        if (i3 < 0 || i1 < 0) {   // dictionary full: the caller uploads host tables instead
            for (const auto &k : added3)
                D.t3.erase(k);
            for (const auto &k : added1)
                D.d1.erase(k);
            D.t3v.resize(D.t3v.size() - 4 * added3.size());
            D.d1v.resize(D.d1v.size() - added1.size());
            return fail(ctx, RF_ERR_STATE, "rf_set_sequences_codes: row-code dictionary full");
        }
        lut[c].id3 = i3;
        lut[c].id1 = i1;
    }
    if ((int64_t)first + nseq > (int64_t)ctx->seqs.size())
        ctx->seqs.resize(first + nseq);
    // regions: bases + tables [match|mismatch|ins|del|row codes] (arena growth
    // at most once per arena; offsets are read after every allocation)
    {
        int64_t need_b = 0, need_t = 0;
        for (int32_t k = 0; k < nseq; ++k) {
            const SeqObj &S = ctx->seqs[first + k];
            const int64_t n = off[k + 1] - off[k];
            const int64_t bb = align_up(std::max<int64_t>(n, 16), 256);
            const int64_t tb = align_up(std::max<int64_t>((row_code_off(n, 0, 0) + n) * 8, 16), 256);
            if (!(S.bases.off >= 0 && S.bases.cap >= bb)) need_b += bb;
            if (!(S.tabs.off >= 0 && S.tabs.cap >= tb)) need_t += tb;
        }
        if (ctx->bytes_arena.top + need_b + ARENA_GUARD > ctx->bytes_arena.cap)
            if (int e = arena_grow(ctx, ctx->bytes_arena, need_b, nullptr)) return e;
        if (ctx->tab_arena.top + need_t + ARENA_GUARD > ctx->tab_arena.cap)
            if (int e = arena_grow(ctx, ctx->tab_arena, need_t, nullptr)) return e;
    }
    for (int32_t k = 0; k < nseq; ++k) {
        SeqObj &S = ctx->seqs[first + k];
        const int64_t n = off[k + 1] - off[k];
        S.n = (int32_t)n;
        S.ncins = S.ncdel = 0;
        if (int e = region_ensure(ctx, ctx->bytes_arena, S.bases, n)) return e;
        if (int e = region_ensure(ctx, ctx->tab_arena, S.tabs, (row_code_off(n, 0, 0) + n) * 8)) return e;
    }
    // new dictionary entries to the device
    if (int e = ensure_buf(ctx, D.lut, (size_t)RF_CODES * 5 * 8)) return e;
    {
        const size_t n3 = D.t3v.size() / 4, n1 = D.d1v.size();
        if (n3 > D.up3)
            HIPCHK(ctx, hipMemcpyAsync((double *)D.lut.p + 4 * D.up3, D.t3v.data() + 4 * D.up3, (n3 - D.up3) * 32,
                                       hipMemcpyHostToDevice, ctx->stream));
        if (n1 > D.up1)
            HIPCHK(ctx, hipMemcpyAsync((double *)D.lut.p + 4 * (size_t)RF_CODES + D.up1, D.d1v.data() + D.up1,
                                       (n1 - D.up1) * 8, hipMemcpyHostToDevice, ctx->stream));
        D.up3 = n3;
        D.up1 = n1;
    }
    if (int e = upload(ctx, ctx->scratch[20], lut)) return e;
    // prep (rf_set_sequences_codes_prep): p10 | match tables, the 256 x 256
    // grid, then est / tsum (nseq doubles each) and ucode (nseq ints)
    const size_t prep_tab = 512 * 8, prep_grid = 65536 * 8, prep_out = (size_t)std::max(nseq, 1) * 20;
    if (prep) {
        if (int e = ensure_buf(ctx, ctx->scratch[27], prep_tab + prep_grid + prep_out)) return e;
        // the two tables and the grid as one copy out of the pinned ring
        char *h;
        if (int e = ring_take(ctx, prep_tab + prep_grid, &h)) return e;
        if (h) {
            std::memcpy(h, p10_t, 256 * 8);
            std::memcpy(h + 256 * 8, match_t, 256 * 8);
            std::memcpy(h + prep_tab, grid, prep_grid);
            HIPCHK(ctx, hipMemcpyAsync(ctx->scratch[27].p, h, prep_tab + prep_grid, hipMemcpyHostToDevice,
                                       ctx->stream));
        } else {
            HIPCHK(ctx, hipMemcpyAsync(ctx->scratch[27].p, p10_t, 256 * 8, hipMemcpyHostToDevice, ctx->stream));
            HIPCHK(ctx, hipMemcpyAsync((char *)ctx->scratch[27].p + 256 * 8, match_t, 256 * 8,
                                       hipMemcpyHostToDevice, ctx->stream));
            HIPCHK(ctx, hipMemcpyAsync((char *)ctx->scratch[27].p + prep_tab, grid, prep_grid,
                                       hipMemcpyHostToDevice, ctx->stream));
        }
    }
    double *d_est = (double *)((char *)ctx->scratch[27].p + prep_tab + prep_grid);
    double *d_tsum = d_est + std::max(nseq, 1);
    int32_t *d_ucode = (int32_t *)(d_tsum + std::max(nseq, 1));
    // chunks of sequences: codes + bases staged in pinned memory, one H2D,
    // the bases scattered to their regions, the tables built in place
    int32_t k0 = 0;
    const int64_t chunk_bytes = std::max<int64_t>((int64_t)ctx->opt.stage_kb * 1024 / 4, 1 << 20);
    while (k0 < nseq) {
        int32_t k1 = k0 + 1;
        while (k1 < nseq && 2 * (off[k1 + 1] - off[k0]) <= chunk_bytes)
            ++k1;
        const int64_t nb = off[k1] - off[k0];
        const size_t stage = (size_t)(2 * nb);
        if (ctx->pinned_bytes < stage) {
            if (ctx->pinned)
                (void)hipHostFree(ctx->pinned);
            ctx->pinned = nullptr;
            ctx->pinned_bytes = 0;
            const size_t want = std::max(stage + stage / 2, (size_t)1 << 22);
            if (hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault) != hipSuccess)
                return fail(ctx, RF_ERR_HIP, "rf_set_sequences_codes: pinned staging allocation failed");
            ctx->pinned_bytes = want;
        }
        uint8_t *hb = (uint8_t *)ctx->pinned, *hc = hb + nb;
        std::memcpy(hb, bases + off[k0], nb);
        std::memcpy(hc, codes + off[k0], nb);
        std::vector<CodeSeq> cs(k1 - k0);
        std::vector<Segment> sg(k1 - k0);
        for (int32_t k = k0; k < k1; ++k) {
            const SeqObj &S = ctx->seqs[first + k];
            cs[k - k0] = {S.tabs.off / 8, off[k] - off[k0], S.n, 0, 0};
            sg[k - k0] = {off[k] - off[k0], S.bases.off, S.n, 0};
        }
        if (int e = ensure_buf(ctx, ctx->scratch[7], (size_t)std::max<int64_t>(2 * nb, 16))) return e;
        HIPCHK(ctx, hipMemcpyAsync(ctx->scratch[7].p, hb, 2 * nb, hipMemcpyHostToDevice, ctx->stream));
        if (int e = upload(ctx, ctx->scratch[5], sg)) return e;
        if (int e = upload(ctx, ctx->scratch[6], cs)) return e;
        hipLaunchKernelGGL(k_scatter, dim3(k1 - k0), dim3(256), 0, ctx->stream, (const Segment *)ctx->scratch[5].p,
                           (const uint8_t *)ctx->scratch[7].p, (uint8_t *)ctx->bytes_arena.d);
        hipLaunchKernelGGL(k_tables, dim3(k1 - k0), dim3(256), 0, ctx->stream, (const CodeSeq *)ctx->scratch[6].p,
                           (const uint8_t *)ctx->scratch[7].p + nb, (const uint8_t *)ctx->scratch[7].p,
                           (const CodeLut *)ctx->scratch[20].p, s_mis, s_ins, s_del, (double *)ctx->tab_arena.d);
        if (prep)
            hipLaunchKernelGGL(k_code_prep, dim3(k1 - k0), dim3(64), 0, ctx->stream,
                               (const CodeSeq *)ctx->scratch[6].p, k1 - k0, (const uint8_t *)ctx->scratch[7].p + nb,
                               (const double *)ctx->scratch[27].p, (const double *)((char *)ctx->scratch[27].p + prep_tab),
                               d_est + k0, d_ucode + k0, d_tsum + k0);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, stream_wait(ctx));   // staging and descriptors are reused
        k0 = k1;
    }
    // finiteness per sequence (lean DP / scorer eligibility): every sequence
    // is finite when every code present is; else one pass per sequence
    bool all_fin = true;
    for (int c = 0; c < 256; ++c)
        all_fin = all_fin && (!present[c] || fin[c]);
    if (all_fin) {
        for (int32_t k = 0; k < nseq; ++k)
            ctx->seqs[first + k].finite = true;
    } else {
        const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), (N >> 19) + 1));
        parallel_for(nth, [&](int t) {
            for (int32_t k = (int32_t)((int64_t)nseq * t / nth); k < (int32_t)((int64_t)nseq * (t + 1) / nth); ++k) {
                bool f = true;
                for (int64_t i = off[k]; i < off[k + 1] && f; ++i)
                    f = fin[codes[i]];
                ctx->seqs[first + k].finite = f;
            }
        });
    }
    for (int32_t k = 0; k < nseq; ++k) {
        ctx->seqs[first + k].coded = true;
        ctx->seqs[first + k].valid = true;
    }
    ++ctx->layout_gen;
    if (prep && nseq > 0) {
        // est | tsum | ucode are contiguous on the device: one copy into the
        // pinned landing zone
        const size_t ob = (size_t)std::max(nseq, 1) * 20;
        if (int e = ensure_hdn(ctx, ob)) return e;
        char *hl = (char *)ctx->hdn + HDN_RES;
        HIPCHK(ctx, pre_d2h(ctx));
        HIPCHK(ctx, hipMemcpyAsync(hl, d_est, ob, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, stream_wait(ctx));
        const size_t ns = (size_t)std::max(nseq, 1);
        std::memcpy(est, hl, (size_t)nseq * 8);
        std::memcpy(tsum, hl + ns * 8, (size_t)nseq * 8);
        std::memcpy(ucode, hl + ns * 16, (size_t)nseq * 4);
    }
    return 0;
}

int rf_set_sequences_codes(rf_ctx *ctx, int32_t first, int32_t nseq, const uint8_t *bases, const int64_t *off,
                           const uint8_t *codes, const double *lp_t, const double *match_t, double s_mis,
                           double s_ins, double s_del)
{
    return set_sequences_codes_impl(ctx, first, nseq, bases, off, codes, lp_t, match_t, s_mis, s_ins, s_del, nullptr,
                                    nullptr, nullptr, nullptr, nullptr);
}

int rf_set_sequences_codes_prep(rf_ctx *ctx, int32_t first, int32_t nseq, const uint8_t *bases, const int64_t *off,
                                const uint8_t *codes, const double *lp_t, const double *match_t, double s_mis,
                                double s_ins, double s_del, const double *p10_t, const double *grid, double *est,
                                int32_t *ucode, double *tsum)
{
    if (!ctx || (nseq > 0 && (!p10_t || !grid || !est || !ucode || !tsum)))
        return fail(ctx, RF_ERR_ARG, "rf_set_sequences_codes_prep: bad arguments");
    return set_sequences_codes_impl(ctx, first, nseq, bases, off, codes, lp_t, match_t, s_mis, s_ins, s_del, p10_t,
                                    grid, est, ucode, tsum);
}

int rf_set_templates(rf_ctx *ctx, int32_t first, int32_t ntpl, const uint8_t *bases,
                     const int64_t *off)
{
    if (!ctx || first < 0 || ntpl < 0 || (ntpl > 0 && (!bases || !off)))
        return fail(ctx, RF_ERR_ARG, "rf_set_templates: bad arguments");
    std::vector<int32_t> ids(ntpl);
    for (int32_t k = 0; k < ntpl; ++k)
        ids[k] = first + k;
    return rf_set_templates_ids(ctx, ntpl, ids.data(), bases, off);
}

int rf_set_templates_ids(rf_ctx *ctx, int32_t ntpl, const int32_t *ids, const uint8_t *bases,
                         const int64_t *off)
{
    if (!ctx || ntpl < 0 || (ntpl > 0 && (!ids || !bases || !off)))
        return fail(ctx, RF_ERR_ARG, "rf_set_templates: bad arguments");
    (void)hipSetDevice(ctx->device);
    ++ctx->state_epoch;
    int32_t top = 0;
    for (int32_t k = 0; k < ntpl; ++k) {
        if (ids[k] < 0)
            return fail(ctx, RF_ERR_ARG, "rf_set_templates: bad arguments");
        top = std::max(top, ids[k] + 1);
    }
    if ((int64_t)top > (int64_t)ctx->tpls.size())
        ctx->tpls.resize(top);
    for (int32_t k = 0; k < ntpl; ++k) {
        TplObj &T = ctx->tpls[ids[k]];
        const int64_t m = off[k + 1] - off[k];
        if (m < 1)
            return fail(ctx, RF_ERR_ARG, "rf_set_templates: empty template");
        if (int e = region_ensure(ctx, ctx->bytes_arena, T.bases, m))
            return e;
        if (T.m != (int32_t)m)
            ++ctx->layout_gen;
        T.m = (int32_t)m;
        T.version = ++ctx->tpl_counter;
        T.valid = true;
    }
    if (ntpl > 0) {
        // offsets are read after every region_ensure (arena growth moves regions)
        std::vector<Segment> sg(ntpl);
        for (int32_t k = 0; k < ntpl; ++k)
            sg[k] = {off[k] - off[0], ctx->tpls[ids[k]].bases.off, off[k + 1] - off[k], 0};
        const int64_t nb = off[ntpl] - off[0];
        if (int e = ensure_buf(ctx, ctx->scratch[7], (size_t)std::max<int64_t>(nb, 16))) return e;
        HIPCHK(ctx, hipMemcpyAsync(ctx->scratch[7].p, bases + off[0], nb, hipMemcpyHostToDevice, ctx->stream));
        if (int e = upload(ctx, ctx->scratch[5], sg)) return e;
        hipLaunchKernelGGL(k_scatter, dim3(ntpl), dim3(256), 0, ctx->stream, (const Segment *)ctx->scratch[5].p,
                           (const uint8_t *)ctx->scratch[7].p, (uint8_t *)ctx->bytes_arena.d);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, stream_wait(ctx));
    return 0;
}

static int realign_impl(rf_ctx *ctx, int32_t njobs, const int32_t *slot, const int32_t *seq, const int32_t *tpl,
                        const int32_t *bw, const int32_t *jf, double *out_score)
{
    if (!ctx || njobs < 0 || (njobs > 0 && (!slot || !seq || !tpl || !bw || !jf)))
        return fail(ctx, RF_ERR_ARG, "rf_realign: bad arguments");
    for (int32_t k = 0; k < njobs; ++k)
        if (!(jf[k] & (RF_FWD | RF_BWD)))
            return fail(ctx, RF_ERR_ARG, "rf_realign: need RF_FWD and/or RF_BWD");
    (void)hipSetDevice(ctx->device);
    auto &P = ctx->rplan;
    const size_t nb = sizeof(int32_t) * (size_t)njobs;
    const bool same = P.valid && P.gen == ctx->layout_gen &&
                      P.slot.size() == (size_t)njobs && (njobs == 0 ||
                      (!std::memcmp(P.slot.data(), slot, nb) && !std::memcmp(P.seq.data(), seq, nb) &&
                       !std::memcmp(P.tpl.data(), tpl, nb) && !std::memcmp(P.bw.data(), bw, nb) &&
                       !std::memcmp(P.flags.data(), jf, nb)));
    // the same job list, validated with nothing changed since: its checks and
    // its band bookkeeping would come out the same
    const bool fresh = same && P.val_epoch == ctx->state_epoch;
    if (!fresh)
        for (int32_t k = 0; k < njobs; ++k) {
            if (slot[k] < 0 || seq[k] < 0 || seq[k] >= (int32_t)ctx->seqs.size() || !ctx->seqs[seq[k]].valid ||
                tpl[k] < 0 || tpl[k] >= (int32_t)ctx->tpls.size() || !ctx->tpls[tpl[k]].valid)
                return fail(ctx, RF_ERR_ARG, "rf_realign: unknown slot / sequence / template");
            if (bw[k] < 1)
                return fail(ctx, RF_ERR_ARG, "bandwidth must be positive");
        }
    if (same) {
        // identical job list on an unchanged layout: descriptors on the device
        // are still exact; only the band bookkeeping (template version) moves
        if (!fresh) {
            bool changed = false;
            for (int dir = 0; dir < 2; ++dir) {
                for (int32_t k = 0; k < njobs; ++k) {
                    if (!(jf[k] & (dir == 0 ? RF_FWD : RF_BWD)))
                        continue;
                    Band &b = dir == 0 ? ctx->slots[slot[k]].a : ctx->slots[slot[k]].b;
                    const uint64_t v = ctx->tpls[tpl[k]].version;
                    changed = changed || b.tplver != v;
                    b.tplver = v;
                }
            }
            if (changed)
                ++ctx->state_epoch;
            P.val_epoch = ctx->state_epoch;
        }
    } else {
        P.valid = false;
        ++ctx->state_epoch;   // band metadata changes below
        int32_t maxslot = -1;
        for (int32_t k = 0; k < njobs; ++k)
            maxslot = std::max(maxslot, slot[k]);
        if (maxslot >= (int32_t)ctx->slots.size())
            ctx->slots.resize(maxslot + 1);
        bool moved = false;   // a band now describes another alignment
        // RF_OPT_BAND_PAD: a call whose widest band reaches the threshold lays out
        // all its bands with line-padded rows (the wide-band scorer reads them a
        // line per row); narrower calls (c4-like) keep the odd stride, which the
        // window scorer k_score_ws stages in fewer passes
        int hmax_call = 0;
        for (int32_t k = 0; k < njobs; ++k)
            hmax_call = std::max(hmax_call, band_rows(ctx->seqs[seq[k]].n + 1, ctx->tpls[tpl[k]].m + 1, bw[k]));
        const bool pad_call = ctx->opt.band_pad_h > 0 && hmax_call >= ctx->opt.band_pad_h;
        for (int dir = 0; dir < 2; ++dir) {
            for (int32_t k = 0; k < njobs; ++k) {
                if (!(jf[k] & (dir == 0 ? RF_FWD : RF_BWD)))
                    continue;
                const SeqObj &S = ctx->seqs[seq[k]];
                const TplObj &T = ctx->tpls[tpl[k]];
                Band &b = dir == 0 ? ctx->slots[slot[k]].a : ctx->slots[slot[k]].b;
                const int H = band_rows(S.n + 1, T.m + 1, bw[k]);
                // A and B of one alignment share a row stride: every scorer reads
                // both bands with one P, and the two are often filled by different
                // calls (forward_moves with band doubling, then backward!) that
                // may differ in pad_call
                const Band &o = dir == 0 ? ctx->slots[slot[k]].b : ctx->slots[slot[k]].a;
                const bool partner = o.valid && o.seq == seq[k] && o.tpl == tpl[k] && o.bw == bw[k] &&
                                     o.n == S.n && o.m == T.m && o.H == H && o.tplver == T.version;
                const int P = partner ? o.P : band_stride(H, pad_call ? 1 : 0);
                if (int e = region_ensure(ctx, ctx->band_arena, b.r, band_K(H, T.m) * P * 8))
                    return e;
                moved = moved || !b.valid || b.seq != seq[k] || b.tpl != tpl[k] || b.bw != bw[k] ||
                        b.n != S.n || b.m != T.m || b.H != H || b.P != P;
                b.P = P;
                b.valid = true;
                b.seq = seq[k];
                b.tpl = tpl[k];
                b.bw = bw[k];
                b.n = S.n;
                b.m = T.m;
                b.H = H;
                b.flags = dir == 0 ? (jf[k] & (RF_SKEW | RF_TRIM)) : 0;
                b.tplver = T.version;
            }
        }
        // scorer descriptors (rf_score_dense's plan) hold band geometry and
        // sequence offsets: a band that now describes another read, template or
        // bandwidth invalidates them even when its region did not move
        if (moved)
            ++ctx->layout_gen;
        // band offsets are only final after every allocation (arena growth moves them)
        std::vector<DPTask> cr[4][2], c64, cg, cp[4][4], cw[2], cwm;
        int hmax64 = 0, hmaxg = 0, gm = 0;
        // RF_OPT_DP_PSPLIT: bit npi set = split lean class NP = 1 << npi by stride
        // (default: NP = 1 only, and only when that class holds at least half
        // of the tasks -- measured: c4 DP -5..9 %; splitting the wide classes,
        // or a small NP = 1 class next to them (c5), made the fill slower)
        int psplit = ctx->opt.dp_psplit >= 0 ? ctx->opt.dp_psplit : 1;
        if (ctx->opt.dp_psplit < 0) {
            size_t n1 = 0, nall = 0;
            for (int dir = 0; dir < 2; ++dir) {
                for (int32_t k = 0; k < njobs; ++k) {
                    if (!(jf[k] & (dir == 0 ? RF_FWD : RF_BWD)))
                        continue;
                    const Band &b = dir == 0 ? ctx->slots[slot[k]].a : ctx->slots[slot[k]].b;
                    n1 += b.H <= 31;
                    ++nall;
                }
            }
            if (2 * n1 < nall)
                psplit = 0;
        }
        // latency mode (RF_OPT_DP_LAT, round 5): few lean tasks of H <= 127 --
        // e.g. configs[2]'s 1,000 reads, or one cluster -- cannot fill the GPU
        // whatever their class, so each runs at its own step latency; they all
        // go to one 64-lane NP = 1 launch (one task per wave, one band pair
        // per lane: the shortest step), on one stream
        bool latmode = false;
        {
            size_t nl = 0;
            for (int dir = 0; dir < 2; ++dir) {
                for (int32_t k = 0; k < njobs; ++k) {
                    if (!(jf[k] & (dir == 0 ? RF_FWD : RF_BWD)))
                        continue;
                    const SeqObj &S = ctx->seqs[seq[k]];
                    const Band &b = dir == 0 ? ctx->slots[slot[k]].a : ctx->slots[slot[k]].b;
                    const bool ln = S.ncins == 0 && S.ncdel == 0 && S.finite && !(dir == 0 && (jf[k] & (RF_SKEW | RF_TRIM)));
                    nl += ln && b.H <= 127;
                }
            }
            latmode = nl > 0 && nl <= (size_t)std::max(ctx->opt.dp_lat, 0);
        }
        std::vector<DPTask> cl;
        for (int dir = 0; dir < 2; ++dir) {
            for (int32_t k = 0; k < njobs; ++k) {
                if (!(jf[k] & (dir == 0 ? RF_FWD : RF_BWD)))
                    continue;
                const SeqObj &S = ctx->seqs[seq[k]];
                const TplObj &T = ctx->tpls[tpl[k]];
                const Band &b = dir == 0 ? ctx->slots[slot[k]].a : ctx->slots[slot[k]].b;
                DPTask t{};
                t.band = b.r.off / 8;
                t.sb = S.bases.off;
                t.tab = S.tabs.off / 8;
                t.tb = T.bases.off;
                t.n = S.n;
                t.m = T.m;
                t.bw = bw[k];
                t.H = b.H;
                t.c = std::max(T.m - S.n, 0) + bw[k];
                t.ncins = S.ncins;
                t.ncdel = S.ncdel;
                t.flags = (dir == 1 ? 1 : 0) | (dir == 0 && (jf[k] & RF_SKEW) ? 2 : 0) |
                          (dir == 0 && (jf[k] & RF_TRIM) ? 4 : 0) | (S.coded ? RF_TASK_CODED : 0);
                // out_score: forward scores win when both directions run
                t.out_idx = (dir == 0 || !(jf[k] & RF_FWD)) ? k : njobs + k;
                t.klen = t.H + 2 * t.m;
                t.P = b.P;
                // classes: k_dpr<NP> for H <= 32*NP-1 (NP = 1, 2, 4, 8), lean when
                // there are no codon moves and no skew / trim; k_dp beyond
                const int lean = (S.ncins == 0 && S.ncdel == 0 && S.finite && !(t.flags & 6)) ? 1 : 0;
                const int npi = t.H <= 31 ? 0 : t.H <= 63 ? 1 : t.H <= 127 ? 2 : 3;
                const bool np8 = npi < 3 || (t.H <= 255 && ctx->opt.dp_np8 && ctx->opt.dp_np8_lean);
                // wide tasks for the wide lean bands: H 128..255 as one 64-lane
                // task per wave, H 64..127 as two 32-lane tasks per wave, both NP = 2
                // (the 16-lane NP = 4 / 8 kernels need > 256 registers: one wave
                // per SIMD)
                const int wide = npi == 3 && t.H <= 255 ? 0 : (npi == 2 ? 1 : -1);
                if (lean && latmode && t.H <= 127 && dpx_fits(t)) {
                    cl.push_back(t);
                } else if (lean && wide >= 0 && ((ctx->opt.dp_wide >> wide) & 1)) {
                    cw[wide].push_back(t);
                } else if (lean && ((psplit >> npi) & 1) && np8 &&
                           !(npi == 0 && DPR_PFIX && (t.P < dpr_pm(0, 0) || t.P > dpr_pm(0, 3) || !(t.P & 1)))) {
                    // NP = 1 stride classes take exactly P = 11, 13, 15, 17 (PFIX
                    // kernels); other strides stay in the generic lean class
                    int pmi = 0;
                    while (pmi < 3 && t.P > dpr_pm(npi, pmi))
                        ++pmi;
                    cp[npi][pmi].push_back(t);
                } else if (t.H <= 31)
                    cr[0][lean].push_back(t);
                else if (t.H <= 63)
                    cr[1][lean].push_back(t);
                else if (t.H <= 127)
                    cr[2][lean].push_back(t);
                else if (t.H <= 255 && ctx->opt.dp_np8)
                    cr[3][ctx->opt.dp_np8_lean ? lean : 0].push_back(t);
                else if (t.H <= 2040) {
                    c64.push_back(t);
                    hmax64 = std::max(hmax64, t.H);
                } else if (S.ncins == 0 && S.ncdel == 0 && ctx->opt.dp_mc && dpm_slices(t.H) <= DPM_TASK_SLICES &&
                           (int64_t)t.klen * t.P * 8 < ((int64_t)1 << 31)) {
                    cwm.push_back(t);   // k_dpm: across CUs, no codon moves (edit_distance's band)
                    gm = std::max(gm, dpm_slices(t.H));
                } else {
                    cg.push_back(t);
                    hmaxg = std::max(hmaxg, t.H);
                }
            }
        }
        // Few non-lean tasks of H <= 127 (the reference's codon DP: one long
        // task per call) run as one latency-bound task per wave (k_dpx, round
        // 5; round 4: k_dpr's general step in 64 lanes): such a launch cannot
        // fill the GPU, so the step latency is the time
        std::vector<DPTask> cx;
        if (cr[0][0].size() + cr[1][0].size() + cr[2][0].size() <= (size_t)std::max(ctx->opt.dp_nl64, 0)) {
            for (int a = 0; a <= 2; ++a) {
                std::vector<DPTask> keep;
                for (const DPTask &t : cr[a][0])
                    (dpx_fits(t) ? cx : keep).push_back(t);
                cr[a][0].swap(keep);
            }
        }
        // A lean NP >= 2 class launched whole (no stride split) takes the
        // smallest stride class that holds its widest task (RF_OPT_DP_PFIT,
        // round 6): the blocked flush issues dpl_flush_stores(NP, PM) 16-B
        // stores per lane and lanes past a block's end repeat its last pair,
        // so at the class maximum PM = 33 the c4 NP = 2 class (P <= 19)
        // rewrote 18 % of its bytes (0.7 GB per step, r05j PMC)
        if (ctx->opt.dp_pfit)
            for (int a = 1; a <= 3; ++a) {
                if (cr[a][1].empty() || ((psplit >> a) & 1))
                    continue;
                int pmax = 0;
                for (const DPTask &t : cr[a][1])
                    pmax = std::max(pmax, t.P);
                int pmi = 0;
                while (pmi < 3 && pmax > dpr_pm(a, pmi))
                    ++pmi;
                cp[a][pmi].insert(cp[a][pmi].end(), cr[a][1].begin(), cr[a][1].end());
                cr[a][1].clear();
            }
        auto by_len = [](const DPTask &x, const DPTask &y) { return x.klen > y.klen; };
        std::vector<DPTask> &all = P.tasks;
        all.clear();
        for (auto &cc : cr)
            for (auto &c : cc) {
                std::stable_sort(c.begin(), c.end(), by_len);
                all.insert(all.end(), c.begin(), c.end());
            }
        for (auto &cc : cp)
            for (auto &c : cc) {
                std::stable_sort(c.begin(), c.end(), by_len);
                all.insert(all.end(), c.begin(), c.end());
            }
        for (auto &c : cw) {
            std::stable_sort(c.begin(), c.end(), by_len);
            all.insert(all.end(), c.begin(), c.end());
        }
        std::stable_sort(cx.begin(), cx.end(), by_len);
        all.insert(all.end(), cx.begin(), cx.end());
        std::stable_sort(cl.begin(), cl.end(), by_len);
        all.insert(all.end(), cl.begin(), cl.end());
        std::stable_sort(c64.begin(), c64.end(), by_len);
        std::stable_sort(cg.begin(), cg.end(), by_len);
        all.insert(all.end(), c64.begin(), c64.end());
        all.insert(all.end(), cg.begin(), cg.end());
        all.insert(all.end(), cwm.begin(), cwm.end());
        if (int e = upload(ctx, ctx->scratch[8], all))
            return e;
        P.valid = true;
        P.gen = ctx->layout_gen;
        P.val_epoch = ctx->state_epoch;
        P.flags.assign(jf, jf + njobs);
        P.slot.assign(slot, slot + njobs);
        P.seq.assign(seq, seq + njobs);
        P.tpl.assign(tpl, tpl + njobs);
        P.bw.assign(bw, bw + njobs);
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 2; ++b)
                P.nr[a][b] = cr[a][b].size();
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b)
                P.nrp[a][b] = cp[a][b].size();
        for (int a = 0; a < 2; ++a)
            P.nw[a] = cw[a].size();
        P.nx = cx.size();
        P.nl = cl.size();
        P.n64 = c64.size();
        P.ng = cg.size();
        P.nwm = cwm.size();
        P.gm = gm;
        P.hmax64 = hmax64;
        P.hmaxg = hmaxg;
    }
    if (int e = ensure_buf(ctx, ctx->scratch[9], sizeof(double) * 2 * std::max(njobs, 1)))
        return e;
    double *d_out = (double *)ctx->scratch[9].p;
    const DPTask *d_tasks = (const DPTask *)ctx->scratch[8].p;
    const uint8_t *d_bases = (const uint8_t *)ctx->bytes_arena.d;
    const double *d_tabs = (const double *)ctx->tab_arena.d;
    double *d_bands = (double *)ctx->band_arena.d;
    const double *d_lut = (const double *)ctx->codes.lut.p;

    HIPCHK(ctx, hipEventRecord(ctx->ev[0], ctx->stream));
    // Each kernel class is its own launch.  The classes are independent (disjoint
    // bands), so the smaller ones run on side streams concurrently with the
    // largest: the machine stays full through every launch's tail.
    struct Launch {
        int kind;      // 0..7 = k_dpr<1<<(kind>>1), kind&1>, 8 = k_dp<64,false>, 9 = k_dp<DPW_NT,..>, 11 = k_dpm,
                       // 32 / 33 = lean wide tasks, 34 = k_dpx (few non-lean),
                       // 35 = latency-mode lean,
                       // 16 + 4 * npi + pmi = k_dpr<1 << npi, true, dpr_pm(npi, pmi)>
        size_t at, n;
    };
    std::vector<Launch> launches;
    {
        size_t at = 0;
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 2; ++b)
                if (P.nr[a][b]) {
                    launches.push_back({2 * a + b, at, P.nr[a][b]});
                    at += P.nr[a][b];
                }
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b)
                if (P.nrp[a][b]) {
                    launches.push_back({16 + 4 * a + b, at, P.nrp[a][b]});
                    at += P.nrp[a][b];
                }
        for (int a = 0; a < 2; ++a)
            if (P.nw[a]) {
                launches.push_back({32 + a, at, P.nw[a]});
                at += P.nw[a];
            }
        if (P.nx) {
            launches.push_back({34, at, P.nx});
            at += P.nx;
        }
        if (P.nl) {
            launches.push_back({35, at, P.nl});
            at += P.nl;
        }
        if (P.n64) {
            launches.push_back({8, at, P.n64});
            at += P.n64;
        }
        if (P.ng) {
            launches.push_back({9, at, P.ng});
            at += P.ng;
        }
        if (P.nwm)
            launches.push_back({11, at, P.nwm});
    }
    // (Round 5: the lean 16-lane classes as ONE launch -- a kernel choosing the
    // class body per block, dynamic LDS of the largest class -- was slower:
    // c4 DP 9.86 against 8.75 ms, profiles/r05p_exp_dp_merge.jsonl; splitting
    // the lean NP = 2 class by stride too: 9.61 against 8.72 ms,
    // r05o_exp_dp_psplit.jsonl.  Concurrent launches pack workgroups of
    // different LDS sizes on a CU; one launch holds every workgroup to the
    // largest.)
    if (int e = ensure_buf(ctx, ctx->scratch[7], 4 * (size_t)dpl_task_bytes(4)))  // lean padding-task sink
        return e;
    if (P.ng) {
        if (int e = ensure_buf(ctx, ctx->scratch[10], P.ng * 4 * (size_t)(P.hmaxg + 6) * 8))
            return e;
    }
    // The latency-bound classes (few long tasks: k_dpx, k_dp) go first, on
    // the main stream: the others run beside them on the side streams, which
    // may share hardware queues with each other (round 5: the reference's
    // codon DP waited behind a read class on a shared queue, c3).  Otherwise
    // the largest launch stays on the main stream.
    std::stable_partition(launches.begin(), launches.end(),
                          [](const Launch &L) { return L.kind == 34 || (L.kind >= 8 && L.kind <= 11); });
    size_t big = 0;
    const bool lat_first = !launches.empty() &&
                           (launches[0].kind == 34 || (launches[0].kind >= 8 && launches[0].kind <= 11));
    for (size_t i = 1; i < launches.size() && !lat_first; ++i)
        if (launches[i].n > launches[big].n)
            big = i;
    const bool concurrent = launches.size() > 1 && ctx->opt.dp_streams;
    // stream of each launch: -1 = the main stream, else a side stream.  (Round
    // 5: balancing the classes over the main stream and two side streams by
    // their stores, largest or smallest first, was slower at c4: 8.42-8.48
    // against 8.25 ms, profiles/r05l_exp_dp_sched.jsonl.)
    std::vector<int> lstream(launches.size(), -1);
    if (concurrent) {
        int nside = 0;
        for (size_t i = 0; i < launches.size(); ++i)
            if (i != big)
                lstream[i] = nside++ % 3;
    }
    if (concurrent)
        HIPCHK(ctx, hipEventRecord(ctx->fork, ctx->stream));
    std::vector<int> used_side;
    for (size_t i = 0; i < launches.size(); ++i) {
        const Launch &L = launches[i];
        hipStream_t st = ctx->stream;
        if (lstream[i] >= 0) {
            const int si = lstream[i];
            st = ctx->side[si];
            if (std::find(used_side.begin(), used_side.end(), si) == used_side.end()) {
                HIPCHK(ctx, hipStreamWaitEvent(st, ctx->fork, 0));
                used_side.push_back(si);
            }
        }
        const int n = (int)L.n;
        if (L.kind < 8) {
            using KFn = void (*)(const DPTask *, int, const uint8_t *, const double *, double *, double *, int *,
                                 double *, const double *);
            const KFn kr[8] = {k_dpr<1, false>, k_dpr<1, true>, k_dpr<2, false>, k_dpr<2, true>,
                               k_dpr<4, false>, k_dpr<4, true>, k_dpr<8, false>, k_dpr<8, true>};
            const int np = 1 << (L.kind >> 1);
            const size_t lds = (L.kind & 1) ? 4 * (size_t)dpl_task_bytes(np) : 0;
            hipLaunchKernelGGL(kr[L.kind], dim3((n + 3) / 4), dim3(64), lds, st, d_tasks + L.at, n, d_bases,
                               d_tabs, d_bands, d_out, ctx->d_err, (double *)ctx->scratch[7].p, d_lut);
        } else if (L.kind >= 16 && L.kind < 32) {
            using KFn = void (*)(const DPTask *, int, const uint8_t *, const double *, double *, double *, int *,
                                 double *, const double *);
#define KP(a, b) k_dpr<1 << (a), true, dpr_pm(a, b), 16, (a) == 0 && DPR_PFIX>
            const KFn kp[16] = {KP(0, 0), KP(0, 1), KP(0, 2), KP(0, 3), KP(1, 0), KP(1, 1), KP(1, 2), KP(1, 3),
                                KP(2, 0), KP(2, 1), KP(2, 2), KP(2, 3), KP(3, 0), KP(3, 1), KP(3, 2), KP(3, 3)};
#undef KP
            const int c = L.kind - 16, npi = c >> 2, pmi = c & 3;
            hipLaunchKernelGGL(kp[c], dim3((n + 3) / 4), dim3(64), 4 * (size_t)dpl_task_bytes(1 << npi, dpr_pm(npi, pmi)),
                               st, d_tasks + L.at, n, d_bases, d_tabs, d_bands, d_out, ctx->d_err,
                               (double *)ctx->scratch[7].p, d_lut);
        } else if (L.kind == 34) {
            // few non-lean tasks (H <= 127): one latency-bound task per wave (k_dpx)
            hipLaunchKernelGGL((k_dpx<true, true>), dim3(n), dim3(128), 0, st, d_tasks + L.at, n, d_bases, d_tabs,
                               d_bands, d_out, ctx->d_err);
        } else if (L.kind == 35) {
            // latency mode: lean tasks of H <= 127, one latency-bound task per wave
            hipLaunchKernelGGL((k_dpx<false, false>), dim3(n), dim3(128), 0, st, d_tasks + L.at, n, d_bases, d_tabs,
                               d_bands, d_out, ctx->d_err);
        } else if (L.kind >= 32) {
            // task-width classes, both NP 2: 32 = 64 lanes (H <= 255), 33 = 32 lanes
            // (H <= 127)
            using KFn = void (*)(const DPTask *, int, const uint8_t *, const double *, double *, double *, int *,
                                 double *, const double *);
            const KFn kw[2] = {k_dpr<2, true, dpl_pmax(2, 64), 64>, k_dpr<2, true, dpl_pmax(2, 32), 32>};
            const int a = L.kind - 32, lpt = a == 0 ? 64 : 32, tpw = 64 / lpt;
            hipLaunchKernelGGL(kw[a], dim3((n + tpw - 1) / tpw), dim3(64),
                               (size_t)tpw * dpl_task_bytes(2, dpl_pmax(2, lpt), lpt), st, d_tasks + L.at, n,
                               d_bases, d_tabs, d_bands, d_out, ctx->d_err, (double *)ctx->scratch[7].p, d_lut);
        } else if (L.kind == 8) {
            const int ld = P.hmax64 + 6;
            hipLaunchKernelGGL((k_dp<64, false>), dim3(n), dim3(64), 4 * ld * 8, st, d_tasks + L.at, n, d_bases,
                               d_tabs, d_bands, d_out, ctx->d_err, ld, nullptr);
        } else if (L.kind == 11) {
            // H > 2040 without codon moves across CUs (k_dpm): one workgroup per
            // slice, a band's slices on one XCD; each band filled with the
            // not-yet-stored pattern first (the slices poll their halo cells)
            // At most DPM_XCD_SLICES slices per XCD per launch, launches in
            // sequence on this stream: a launch's bands become resident in
            // order, but two launches from different streams interleave, so
            // each keeps to a share of an XCD (four such launches fit at once)
            const int per = 8 * std::max(1, DPM_XCD_SLICES / P.gm);
            for (int c0 = 0; c0 < n; c0 += per) {
                const int nc = std::min(per, n - c0);
                bool trim = false;
                for (int i = c0; i < c0 + nc; ++i) {
                    const DPTask &t = P.tasks[L.at + i];
                    trim = trim || (t.flags & 4);
                    HIPCHK(ctx, hipMemsetAsync(d_bands + t.band, 0xFF, (size_t)t.klen * t.P * 8, st));
                }
                hipLaunchKernelGGL(trim ? k_dpm<true> : k_dpm<false>, dim3((unsigned)(8 * ((nc + 7) / 8) * P.gm)),
                                   dim3(64), 0, st, d_tasks + L.at + c0, nc, P.gm, d_bases, d_tabs, d_bands, d_out,
                                   ctx->d_err);
            }
        } else {
            // H > 2040: one task per DPW_NT-thread block, the ring in LDS when it fits
            const int ld = P.hmaxg + 6;
            if (P.hmaxg <= DPW_LDS_H)
                hipLaunchKernelGGL((k_dp<DPW_NT, false, DPW_NT>), dim3(n), dim3(DPW_NT), 4 * ld * 8, st, d_tasks + L.at, n,
                                   d_bases, d_tabs, d_bands, d_out, ctx->d_err, ld, nullptr);
            else
                hipLaunchKernelGGL((k_dp<DPW_NT, true, DPW_NT>), dim3(n), dim3(DPW_NT), 0, st, d_tasks + L.at, n, d_bases,
                                   d_tabs, d_bands, d_out, ctx->d_err, ld, (double *)ctx->scratch[10].p);
        }
    }
    for (int si : used_side) {
        HIPCHK(ctx, hipEventRecord(ctx->join[si], ctx->side[si]));
        HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->join[si], 0));
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->ev[1], ctx->stream));
    // scores and the error flag into pinned memory, one synchronize
    const size_t ob = (out_score && njobs > 0) ? sizeof(double) * njobs : 0;
    if (int e = ensure_hout(ctx, ob))
        return e;
    HIPCHK(ctx, hipMemcpyAsync(ctx->hout, ctx->d_err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    if (ob)
        HIPCHK(ctx, hipMemcpyAsync((char *)ctx->hout + 16, d_out, ob, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, stream_wait(ctx));
    if (ob)
        std::memcpy(out_score, (const char *)ctx->hout + 16, ob);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]);
    ctx->dp_ms = ms;
    return check_err_landed(ctx);
}

int rf_realign(rf_ctx *ctx, int32_t njobs, const int32_t *slot, const int32_t *seq,
               const int32_t *tpl, const int32_t *bw, int32_t flags, double *out_score)
{
    if (!ctx || njobs < 0)
        return fail(ctx, RF_ERR_ARG, "rf_realign: bad arguments");
    ctx->jflags.assign((size_t)njobs, flags);
    return realign_impl(ctx, njobs, slot, seq, tpl, bw, ctx->jflags.data(), out_score);
}

int rf_realign_jobs(rf_ctx *ctx, int32_t njobs, const int32_t *slot, const int32_t *seq, const int32_t *tpl,
                    const int32_t *bw, const int32_t *flags, double *out_score)
{
    return realign_impl(ctx, njobs, slot, seq, tpl, bw, flags, out_score);
}

// Launch the backtraces of `tasks` (moves into scratch[3] at t.out, counts in
// scratch[4]) in k_bt_win (round 4: codon alignments and bands of any height
// too); with d_mask, the walks also mark alignment proposals.
static int launch_backtraces(rf_ctx *ctx, std::vector<BTTask> &tasks, uint8_t *d_mask, int do_indels)
{
    const int32_t nslots = (int32_t)tasks.size();
    std::vector<BTTask> &win = ctx->bt_win;   // alive until the caller's sync
    win = tasks;
    int32_t *d_cnt = (int32_t *)ctx->scratch[4].p;
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    if (!win.empty()) {
        if (int e = upload(ctx, ctx->scratch[16], win))
            return e;
        // a launch of few walks (the reference's, edit_distance's: one
        // latency-bound walk each) runs each walk on 4 waves (NW = 4)
        const bool few = win.size() <= (size_t)BTW_FEW && ctx->opt.bt_nw != 1;
        auto kern = few ? k_bt_win<4096, 4> : ctx->opt.bt_win_kb == 16 ? k_bt_win<2048> : k_bt_win<4096>;
        hipLaunchKernelGGL(kern, dim3((unsigned)win.size()), dim3(few ? 256 : 64), 0, ctx->stream,
                           (const BTTask *)ctx->scratch[16].p, (const uint8_t *)ctx->bytes_arena.d,
                           (const double *)ctx->tab_arena.d, (const double *)ctx->band_arena.d,
                           (int8_t *)ctx->scratch[3].p, d_cnt, d_cnt + nslots, ctx->d_err, d_mask, do_indels);
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    return 0;
}

// kernel time of the last launch_backtraces (after the caller's sync)
static void note_bt_ms(rf_ctx *ctx)
{
    float ms = 0;
    if (hipEventElapsedTime(&ms, ctx->ev[4], ctx->ev[5]) == hipSuccess)
        ctx->bt_ms = ms;
}

// Backtrace descriptors of `nslots` slots (moves slot k at offs[k], n+m bytes)
// and the scratch buffers for moves and counts.
static int build_bt_tasks(rf_ctx *ctx, int32_t nslots, const int32_t *slot, std::vector<BTTask> &tasks,
                          std::vector<int64_t> &offs)
{
    tasks.assign(nslots, BTTask{});
    offs.assign(nslots, 0);
    int64_t total = 0;
    for (int32_t k = 0; k < nslots; ++k) {
        if (slot[k] < 0 || slot[k] >= (int32_t)ctx->slots.size() || !ctx->slots[slot[k]].a.valid)
            return fail(ctx, RF_ERR_STATE, "rf_backtrace: slot has no A band");
        const Band &b = ctx->slots[slot[k]].a;
        const SeqObj &S = ctx->seqs[b.seq];
        const TplObj &T = ctx->tpls[b.tpl];
        if (T.version != b.tplver)
            return fail(ctx, RF_ERR_STATE, "rf_backtrace: template changed since the A band was computed");
        BTTask &t = tasks[k];
        t.A = b.r.off / 8;
        t.sb = S.bases.off;
        t.tab = S.tabs.off / 8;
        t.tb = T.bases.off;
        t.out = total;
        t.n = b.n;
        t.m = b.m;
        t.bw = b.bw;
        t.H = b.H;
        t.ncins = S.ncins;
        t.ncdel = S.ncdel;
        t.flags = (b.flags & RF_SKEW ? 2 : 0) | (b.flags & RF_TRIM ? 4 : 0);
        t.idx = k;
        t.P = b.P;
        t.mask = 0;
        offs[k] = total;
        total += b.n + b.m;
    }
    if (int e = ensure_buf(ctx, ctx->scratch[3], std::max<int64_t>(total, 16)))
        return e;
    if (int e = ensure_buf(ctx, ctx->scratch[4], sizeof(int32_t) * 2 * std::max(nslots, 1)))
        return e;
    return 0;
}

int rf_backtrace(rf_ctx *ctx, int32_t nslots, const int32_t *slot, int8_t *moves,
                 const int64_t *moves_off, int32_t *nmoves, int32_t *nerrors)
{
    if (!ctx || nslots < 0 || (nslots > 0 && !slot) || (moves && !moves_off))
        return fail(ctx, RF_ERR_ARG, "rf_backtrace: bad arguments");
    (void)hipSetDevice(ctx->device);
    std::vector<BTTask> tasks;
    std::vector<int64_t> offs;
    if (int e = build_bt_tasks(ctx, nslots, slot, tasks, offs))
        return e;
    const int64_t total = nslots > 0 ? offs[nslots - 1] + tasks[nslots - 1].n + tasks[nslots - 1].m : 0;
    int32_t *d_cnt = (int32_t *)ctx->scratch[4].p;
    if (nslots > 0)
        if (int e = launch_backtraces(ctx, tasks, nullptr, 0))
            return e;
    // counts, then the moves, land in ctx->hdn with the error flag: one wait
    const size_t cb = (sizeof(int32_t) * 2 * (size_t)nslots + 15) & ~(size_t)15;
    if (int e = ensure_hdn(ctx, cb + (moves ? (size_t)total : 0)))
        return e;
    const int32_t *cnt = (const int32_t *)((char *)ctx->hdn + HDN_RES);
    const int8_t *all = (const int8_t *)((char *)ctx->hdn + HDN_RES + cb);
    HIPCHK(ctx, pre_d2h(ctx));
    if (nslots > 0)
        HIPCHK(ctx, hipMemcpyAsync((void *)cnt, d_cnt, sizeof(int32_t) * 2 * nslots, hipMemcpyDeviceToHost,
                                   ctx->stream));
    if (moves && total > 0)
        HIPCHK(ctx, hipMemcpyAsync((void *)all, ctx->scratch[3].p, total, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, land_err(ctx));
    HIPCHK(ctx, stream_wait(ctx));
    if (nslots > 0)
        note_bt_ms(ctx);
    if (int e = check_err_hdn(ctx))
        return e;
    for (int32_t k = 0; k < nslots; ++k) {
        if (nmoves)
            nmoves[k] = cnt[k];
        if (nerrors)
            nerrors[k] = cnt[nslots + k];
        if (moves)   // the walk leaves the moves at the end of the read's n+m slot
            std::memcpy(moves + moves_off[k], all + offs[k] + tasks[k].n + tasks[k].m - cnt[k], cnt[k]);
    }
    return 0;
}

int rf_alignment_proposals(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                           int32_t do_indels, uint8_t *out_mask)
{
    if (!ctx || ngroups < 0 || (ngroups > 0 && (!slot_off || !slots || !out_mask)))
        return fail(ctx, RF_ERR_ARG, "rf_alignment_proposals: bad arguments");
    const int32_t nslots = ngroups > 0 ? slot_off[ngroups] : 0;
    (void)hipSetDevice(ctx->device);
    // 1. descriptors: backtrace tasks of every batch slot + each cluster's mask
    std::vector<BTTask> tasks;
    std::vector<int64_t> offs;
    if (int e = build_bt_tasks(ctx, nslots, slots, tasks, offs))
        return e;
    int64_t mask_total = 0;
    for (int32_t g = 0; g < ngroups; ++g) {
        int32_t tpl = -1, m = 0;
        for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k) {
            const Band &b = ctx->slots[slots[k]].a;
            if (tpl >= 0 && b.tpl != tpl)
                return fail(ctx, RF_ERR_ARG, "rf_alignment_proposals: batch slots use different templates");
            tpl = b.tpl;
            m = b.m;
            tasks[k].mask = mask_total;
        }
        if (slot_off[g + 1] > slot_off[g])
            mask_total += (int64_t)(m + 1) * 9;
    }
    if (nslots == 0)
        return 0;
    if (int e = ensure_buf(ctx, ctx->scratch[2], std::max<int64_t>(mask_total, 16)))
        return e;
    HIPCHK(ctx, hipMemsetAsync(ctx->scratch[2].p, 0, mask_total, ctx->stream));
    // 2. the walks mark the mask as they go
    if (int e = launch_backtraces(ctx, tasks, (uint8_t *)ctx->scratch[2].p, do_indels ? 1 : 0))
        return e;
    HIPCHK(ctx, hipGetLastError());
    if (int e = ensure_hdn(ctx, mask_total))
        return e;
    HIPCHK(ctx, pre_d2h(ctx));
    HIPCHK(ctx, hipMemcpyAsync((char *)ctx->hdn + HDN_RES, ctx->scratch[2].p, mask_total, hipMemcpyDeviceToHost,
                               ctx->stream));
    HIPCHK(ctx, land_err(ctx));
    HIPCHK(ctx, stream_wait(ctx));
    note_bt_ms(ctx);
    if (int e = check_err_hdn(ctx))
        return e;
    std::memcpy(out_mask, (char *)ctx->hdn + HDN_RES, mask_total);
    return 0;
}

int rf_score(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
             const int32_t *ref_slot, const int64_t *prop_off, const uint8_t *kind,
             const int32_t *pos, const uint8_t *base, double *out_total, double *out_per_seq)
{
    if (!ctx || ngroups < 0 || (ngroups > 0 && (!slot_off || !prop_off)))
        return fail(ctx, RF_ERR_ARG, "rf_score: bad arguments");
    (void)hipSetDevice(ctx->device);
    const int64_t nprops = ngroups > 0 ? prop_off[ngroups] - prop_off[0] : 0;
    if (nprops > 0 && (!kind || !pos || !base || !out_total))
        return fail(ctx, RF_ERR_ARG, "rf_score: bad proposal arrays");

    auto band_ok = [&](int32_t s, std::string &why) -> bool {
        if (s < 0 || s >= (int32_t)ctx->slots.size()) {
            why = "unknown slot";
            return false;
        }
        const Slot &S = ctx->slots[s];
        if (!S.a.valid || !S.b.valid) {
            why = "slot has no A/B bands";
            return false;
        }
        if (S.a.seq != S.b.seq || S.a.tpl != S.b.tpl || S.a.bw != S.b.bw || S.a.tplver != S.b.tplver ||
            S.a.m != S.b.m) {
            why = "A and B bands were computed for different alignments";
            return false;
        }
        if (S.a.P != S.b.P) {
            why = "A and B bands have different row strides";
            return false;
        }
        if (ctx->tpls[S.a.tpl].version != S.a.tplver) {
            why = "template changed since the bands were computed";
            return false;
        }
        return true;
    };

    std::vector<ScoreGroup> groups(ngroups);
    std::vector<ScoreRead> reads;
    std::vector<int32_t> has_reads(ngroups, 0), has_ref(ngroups, 0);
    std::vector<WorkItem> items;
    std::vector<CodonTask> ctasks;
    std::vector<int64_t> gstart(ngroups + 1, 0);
    int64_t dense_total = 0, split_total = 0, scratch_total = 0;
    int max_reads = 0;
    bool all_finite = true;
    for (int32_t g = 0; g < ngroups; ++g) {
        int32_t tpl = -1;
        std::string why;
        const int32_t r0 = (int32_t)reads.size();
        for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k) {
            if (!band_ok(slots[k], why))
                return fail(ctx, RF_ERR_STATE, "rf_score: " + why);
            const Band &A = ctx->slots[slots[k]].a;
            const Band &B = ctx->slots[slots[k]].b;
            const SeqObj &S = ctx->seqs[A.seq];
            if (S.ncins > 0 || S.ncdel > 0)
                return fail(ctx, RF_ERR_ARG, "error model cannot allow codon indels");
            all_finite = all_finite && S.finite;
            if (tpl >= 0 && A.tpl != tpl)
                return fail(ctx, RF_ERR_ARG, "rf_score: batch slots use different templates");
            tpl = A.tpl;
            ScoreRead R{};
            R.A = A.r.off / 8;
            R.B = B.r.off / 8;
            R.sb = S.bases.off;
            R.tab = S.tabs.off / 8;
            R.n = A.n;
            R.bw = A.bw;
            R.H = A.H;
            R.c = std::max(A.m - A.n, 0) + A.bw;
            R.vb = std::max(A.n - A.m, 0) + A.bw;
            R.P = A.P;
            R.K = (int32_t)band_K(A.H, A.m);
            R.flags = (S.coded && S.ncins == 0 && S.ncdel == 0) ? SR_CODED : 0;
            reads.push_back(R);
        }
        const int32_t r1 = (int32_t)reads.size();
        if (ref_slot && ref_slot[g] >= 0) {
            if (!band_ok(ref_slot[g], why))
                return fail(ctx, RF_ERR_STATE, "rf_score (reference): " + why);
            const int32_t rt = ctx->slots[ref_slot[g]].a.tpl;
            if (tpl >= 0 && rt != tpl)
                return fail(ctx, RF_ERR_ARG, "rf_score: reference uses a different template");
            tpl = rt;
            has_ref[g] = 1;
        }
        ScoreGroup &G = groups[g];
        G.r0 = r0;
        G.r1 = r1;
        has_reads[g] = r1 > r0;
        max_reads = std::max(max_reads, r1 - r0);
        if (tpl < 0) {
            G.m = 0;
            G.tb = 0;
        } else {
            G.m = ctx->tpls[tpl].m;
            G.tb = ctx->tpls[tpl].bases.off;
        }
        G.dense_off = dense_total;
        gstart[g] = dense_total;
        if (has_reads[g]) {
            dense_total += (int64_t)(G.m + 1) * 9;
            G.split_off = split_total;
            split_total += (int64_t)(G.m + 1) * 9 * (r1 - r0);
            for (int p0 = 0; p0 <= G.m; p0 += 64)
                items.push_back({g, p0});
        }
        gstart[g + 1] = dense_total;
        // proposals: validate, build codon tasks for the reference
        for (int64_t k = prop_off[g]; k < prop_off[g + 1]; ++k) {
            const int kd = kind[k], ps = pos[k], b = base[k];
            if (kd > 2 || b > 3 || (kd == 1 ? (ps < 0 || ps > G.m) : (ps < 1 || ps > G.m)))
                return fail(ctx, RF_ERR_ARG, "rf_score: proposal out of range");
            if (!has_reads[g] && !has_ref[g])
                return fail(ctx, RF_ERR_ARG, "rf_score: group has neither reads nor reference");
            if (has_ref[g]) {
                const Band &A = ctx->slots[ref_slot[g]].a;
                const Band &B = ctx->slots[ref_slot[g]].b;
                const SeqObj &S = ctx->seqs[A.seq];
                CodonTask t{};
                t.A = A.r.off / 8;
                t.B = B.r.off / 8;
                t.sb = S.bases.off;
                t.tab = S.tabs.off / 8;
                t.tb = ctx->tpls[A.tpl].bases.off;
                t.scratch = scratch_total;
                scratch_total += 4 * (int64_t)(A.n + 1);
                t.n = A.n;
                t.m = A.m;
                t.bw = A.bw;
                t.H = A.H;
                t.ncins = S.ncins;
                t.ncdel = S.ncdel;
                t.P = A.P;
                t.kind = kd;
                t.pos = ps;
                t.base = b;
                t.out_idx = (int32_t)(k - prop_off[0]);
                ctasks.push_back(t);
            }
        }
    }
    // split mode: not enough (group, chunk) items to fill the chip, or the
    // caller wants per-read scores
    // RF_OPT_SCORE_MODE = fused | split overrides the choice (tests cover both)
    bool split = out_per_seq != nullptr || ((int64_t)items.size() < 2048 && max_reads > 1);
    if (ctx->opt.score_mode == 1 && !out_per_seq)
        split = false;
    else if (ctx->opt.score_mode == 2)
        split = true;

    const ScorePick pick = pick_scorer(ctx->opt, reads, all_finite);
    if (pick.cols() != 64)
        items = make_items(groups, pick.cols());

    std::vector<int32_t> pgroup(nprops);
    for (int32_t g = 0; g < ngroups; ++g)
        for (int64_t k = prop_off[g]; k < prop_off[g + 1]; ++k)
            pgroup[k - prop_off[0]] = g;

    // uploads
    if (int e = upload(ctx, ctx->scratch[0], items)) return e;
    if (int e = upload(ctx, ctx->scratch[1], groups)) return e;
    if (int e = upload(ctx, ctx->scratch[2], reads)) return e;
    if (int e = upload(ctx, ctx->scratch[3], ctasks)) return e;
    // proposal arrays + per-group flags + gstart
    const size_t pbytes = align_up(nprops * 4, 256) * 2 + align_up(nprops, 256) * 2 +
                          align_up(ngroups * 4, 256) * 2 + align_up((ngroups + 1) * 8, 256);
    if (int e = ensure_buf(ctx, ctx->scratch[4], pbytes + 256)) return e;
    char *pb = (char *)ctx->scratch[4].p;
    int32_t *d_pgroup = (int32_t *)pb;  pb += align_up(nprops * 4, 256);
    int32_t *d_pos = (int32_t *)pb;     pb += align_up(nprops * 4, 256);
    uint8_t *d_kind = (uint8_t *)pb;    pb += align_up(nprops, 256);
    uint8_t *d_base = (uint8_t *)pb;    pb += align_up(nprops, 256);
    int32_t *d_hr = (int32_t *)pb;      pb += align_up(ngroups * 4, 256);
    int32_t *d_href = (int32_t *)pb;    pb += align_up(ngroups * 4, 256);
    int64_t *d_gstart = (int64_t *)pb;
    // the seven arrays in their device layout: one copy out of the ring
    const size_t pused = (size_t)((char *)(d_gstart + ngroups + 1) - (char *)ctx->scratch[4].p);
    char *h;
    if (int e = ring_take(ctx, pused, &h))
        return e;
    auto put = [&](void *d, const void *src, size_t n) -> hipError_t {
        if (!n)
            return hipSuccess;
        if (h) {
            std::memcpy(h + ((char *)d - (char *)ctx->scratch[4].p), src, n);
            return hipSuccess;
        }
        return hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, ctx->stream);
    };
    if (nprops > 0) {
        HIPCHK(ctx, put(d_pgroup, pgroup.data(), nprops * 4));
        HIPCHK(ctx, put(d_pos, pos + prop_off[0], nprops * 4));
        HIPCHK(ctx, put(d_kind, kind + prop_off[0], nprops));
        HIPCHK(ctx, put(d_base, base + prop_off[0], nprops));
    }
    if (ngroups > 0) {
        HIPCHK(ctx, put(d_hr, has_reads.data(), ngroups * 4));
        HIPCHK(ctx, put(d_href, has_ref.data(), ngroups * 4));
        HIPCHK(ctx, put(d_gstart, gstart.data(), (ngroups + 1) * 8));
    }
    if (h && (nprops > 0 || ngroups > 0))
        HIPCHK(ctx, hipMemcpyAsync(ctx->scratch[4].p, h, pused, hipMemcpyHostToDevice, ctx->stream));
    // work buffers: dense totals, split partials, codon scratch + outputs, final totals
    const size_t wbytes = align_up(std::max<int64_t>(dense_total, 1) * 8, 256) +
                          (split ? align_up(std::max<int64_t>(split_total, 1) * 8, 256) : 0) +
                          align_up(std::max<int64_t>(scratch_total, 1) * 8, 256) +
                          2 * align_up(std::max<int64_t>(nprops, 1) * 8, 256);
    if (int e = ensure_buf(ctx, ctx->scratch[5], wbytes)) return e;
    char *wb = (char *)ctx->scratch[5].p;
    double *d_dense = (double *)wb;   wb += align_up(std::max<int64_t>(dense_total, 1) * 8, 256);
    double *d_split = nullptr;
    if (split) { d_split = (double *)wb; wb += align_up(std::max<int64_t>(split_total, 1) * 8, 256); }
    double *d_cscr = (double *)wb;    wb += align_up(std::max<int64_t>(scratch_total, 1) * 8, 256);
    double *d_ref = (double *)wb;     wb += align_up(std::max<int64_t>(nprops, 1) * 8, 256);
    double *d_out = (double *)wb;

    const uint8_t *d_bases = (const uint8_t *)ctx->bytes_arena.d;
    const double *d_tabs = (const double *)ctx->tab_arena.d;
    const double *d_bands = (const double *)ctx->band_arena.d;

    HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
    if (!items.empty()) {
        launch_scorer(ctx, pick, (unsigned)items.size(), split ? (unsigned)max_reads : 1u,
                      (const WorkItem *)ctx->scratch[0].p, (const ScoreGroup *)ctx->scratch[1].p,
                      (const ScoreRead *)ctx->scratch[2].p, d_dense, d_split);
        if (split && dense_total > 0)
            hipLaunchKernelGGL(k_reduce, dim3((unsigned)((dense_total + 255) / 256)), dim3(256), 0,
                               ctx->stream, (const ScoreGroup *)ctx->scratch[1].p, ngroups, d_gstart,
                               dense_total, d_split, d_dense);
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev_codon, ctx->stream));
    if (!ctasks.empty())
        hipLaunchKernelGGL(k_codon, dim3((unsigned)((ctasks.size() + 63) / 64)), dim3(64), 0,
                           ctx->stream, (const CodonTask *)ctx->scratch[3].p, (int)ctasks.size(),
                           d_bases, d_tabs, d_bands, d_cscr, d_ref);
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    if (nprops > 0)
        hipLaunchKernelGGL(k_gather, dim3((unsigned)((nprops + 255) / 256)), dim3(256), 0, ctx->stream,
                           nprops, d_pgroup, d_kind, d_pos, d_base, (const ScoreGroup *)ctx->scratch[1].p,
                           d_hr, d_dense, d_ref, d_href, d_out, ctx->d_err);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    // the totals land in ctx->hdn with the error flag (per-read columns, a
    // test / sharding path, stay pageable)
    if (int e = ensure_hdn(ctx, (size_t)std::max<int64_t>(nprops, 0) * 8))
        return e;
    HIPCHK(ctx, pre_d2h(ctx));
    if (nprops > 0)
        HIPCHK(ctx, hipMemcpyAsync((char *)ctx->hdn + HDN_RES, d_out, nprops * 8, hipMemcpyDeviceToHost,
                                   ctx->stream));
    HIPCHK(ctx, land_err(ctx));
    std::vector<double> split_host;
    if (out_per_seq && split_total > 0) {
        split_host.resize(split_total);
        HIPCHK(ctx, hipMemcpyAsync(split_host.data(), d_split, split_total * 8, hipMemcpyDeviceToHost,
                                   ctx->stream));
    }
    std::vector<double> ref_host;
    if (out_per_seq && !ctasks.empty()) {
        ref_host.resize(nprops);
        HIPCHK(ctx, hipMemcpyAsync(ref_host.data(), d_ref, nprops * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(ctx, stream_wait(ctx));
    float a = 0, b = 0, cms = 0;
    (void)hipEventElapsedTime(&a, ctx->ev[2], ctx->ev[3]);
    (void)hipEventElapsedTime(&b, ctx->ev[3], ctx->ev[4]);
    (void)hipEventElapsedTime(&cms, ctx->ev_codon, ctx->ev[3]);
    ctx->score_ms = a;
    ctx->gather_ms = b;
    ctx->codon_ms = ctasks.empty() ? 0.0 : cms;
    if (out_per_seq) {
        // [k][r] rows, r = batch position (+1 column for the reference, if any)
        int64_t row = 0;
        for (int32_t g = 0; g < ngroups; ++g) {
            const ScoreGroup &G = groups[g];
            const int R = G.r1 - G.r0;
            const int width = R + (has_ref[g] ? 1 : 0);
            for (int64_t k = prop_off[g]; k < prop_off[g + 1]; ++k) {
                const int kd = kind[k];
                const int sl = kd == 0 ? base[k] : (kd == 2 ? 4 : 5 + base[k]);
                for (int r = 0; r < R; ++r)
                    out_per_seq[row + r] =
                        split_host[G.split_off + ((int64_t)r * (G.m + 1) + pos[k]) * 9 + sl];
                if (has_ref[g])
                    out_per_seq[row + R] = ref_host[k - prop_off[0]];
                row += width;
            }
        }
    }
    if (int e = check_err_hdn(ctx))
        return e;
    if (nprops > 0)
        std::memcpy(out_total, (char *)ctx->hdn + HDN_RES, nprops * 8);
    return 0;
}

static int score_dense_impl(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                            double *out, hipMemcpyKind out_kind)
{
    if (!ctx || ngroups < 0 || (ngroups > 0 && (!slot_off || !slots)))
        return fail(ctx, RF_ERR_ARG, "rf_score_dense: bad arguments");
    (void)hipSetDevice(ctx->device);
    const int32_t nslots = ngroups > 0 ? slot_off[ngroups] : 0;
    auto &P = ctx->dplan;
    const bool same = P.valid && P.gen == ctx->layout_gen && P.ngroups == ngroups && P.opt_gen == ctx->opt_gen &&
                      P.slots.size() == (size_t)nslots &&
                      !std::memcmp(P.slot_off.data(), slot_off, sizeof(int32_t) * (ngroups + 1)) &&
                      (nslots == 0 || !std::memcmp(P.slots.data(), slots, sizeof(int32_t) * nslots));
    // per-call validation of the bands, unless this very slot list was
    // validated and nothing (sequences, templates, bands) changed since
    if (!(same && P.val_epoch == ctx->state_epoch))
    for (int32_t g = 0; g < ngroups; ++g) {
        if (slot_off[g + 1] <= slot_off[g])
            return fail(ctx, RF_ERR_ARG, "rf_score_dense: empty group");
        int32_t tpl = -1;
        for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k) {
            const int32_t sl = slots[k];
            if (sl < 0 || sl >= (int32_t)ctx->slots.size())
                return fail(ctx, RF_ERR_ARG, "rf_score_dense: unknown slot");
            const Slot &S = ctx->slots[sl];
            if (!S.a.valid || !S.b.valid || S.a.seq != S.b.seq || S.a.tpl != S.b.tpl ||
                S.a.bw != S.b.bw || S.a.tplver != S.b.tplver || S.a.m != S.b.m)
                return fail(ctx, RF_ERR_STATE, "rf_score_dense: A and B bands were computed for different alignments");
            if (S.a.P != S.b.P)
                return fail(ctx, RF_ERR_STATE, "rf_score_dense: A and B bands have different row strides");
            if (ctx->tpls[S.a.tpl].version != S.a.tplver)
                return fail(ctx, RF_ERR_STATE, "rf_score_dense: template changed since the bands were computed");
            const SeqObj &Q = ctx->seqs[S.a.seq];
            if (Q.ncins > 0 || Q.ncdel > 0)
                return fail(ctx, RF_ERR_ARG, "error model cannot allow codon indels");
            if (tpl >= 0 && S.a.tpl != tpl)
                return fail(ctx, RF_ERR_ARG, "rf_score_dense: batch slots use different templates");
            tpl = S.a.tpl;
        }
    }
    P.val_epoch = ctx->state_epoch;
    if (!same) {
        P.valid = false;
        std::vector<ScoreGroup> &groups = P.groups;
        std::vector<ScoreRead> &reads = P.reads;
        std::vector<WorkItem> &items = P.items;
        groups.assign(ngroups, ScoreGroup{});
        reads.clear();
        items.clear();
        reads.reserve(nslots);
        int64_t dense_total = 0, split_total = 0;
        int max_reads = 0;
        bool all_finite = true;
        for (int32_t g = 0; g < ngroups; ++g) {
            ScoreGroup &G = groups[g];
            G.r0 = (int32_t)reads.size();
            for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k) {
                const Band &B = ctx->slots[slots[k]].b;
                const Band &A = ctx->slots[slots[k]].a;
                const SeqObj &S = ctx->seqs[A.seq];
                all_finite = all_finite && S.finite;
                ScoreRead R{};
                R.A = A.r.off / 8;
                R.B = B.r.off / 8;
                R.sb = S.bases.off;
                R.tab = S.tabs.off / 8;
                R.n = A.n;
                R.bw = A.bw;
                R.H = A.H;
                R.c = std::max(A.m - A.n, 0) + A.bw;
                R.vb = std::max(A.n - A.m, 0) + A.bw;
                R.P = A.P;
                R.K = (int32_t)band_K(A.H, A.m);
                R.flags = (S.coded && S.ncins == 0 && S.ncdel == 0) ? SR_CODED : 0;
                reads.push_back(R);
            }
            G.r1 = (int32_t)reads.size();
            const TplObj &T = ctx->tpls[ctx->slots[slots[slot_off[g]]].b.tpl];
            G.m = T.m;
            G.tb = T.bases.off;
            G.dense_off = dense_total;
            dense_total += (int64_t)(G.m + 1) * 9;
            G.split_off = split_total;
            split_total += (int64_t)(G.m + 1) * 9 * (G.r1 - G.r0);
            max_reads = std::max(max_reads, G.r1 - G.r0);
            for (int p0 = 0; p0 <= G.m; p0 += 64)
                items.push_back({g, p0});
        }
        std::vector<int64_t> &gstart = P.gstart;
        gstart.assign(ngroups + 1, 0);
        for (int32_t g = 0; g < ngroups; ++g)
            gstart[g] = groups[g].dense_off;
        gstart[ngroups] = dense_total;
        P.pick = pick_scorer(ctx->opt, reads, all_finite);
        if (P.pick.cols() != 64)
            items = make_items(groups, P.pick.cols());
        if (int e = upload(ctx, ctx->scratch[11], items)) return e;
        if (int e = upload(ctx, ctx->scratch[12], groups)) return e;
        if (int e = upload(ctx, ctx->scratch[13], reads)) return e;
        if (int e = upload(ctx, ctx->scratch[14], gstart)) return e;
        P.valid = true;
        P.gen = ctx->layout_gen;
        P.ngroups = ngroups;
        P.slot_off.assign(slot_off, slot_off + ngroups + 1);
        P.slots.assign(slots, slots + nslots);
        P.nitems = items.size();
        P.max_reads = max_reads;
        P.dense_total = dense_total;
        P.split_total = split_total;
        P.opt_gen = ctx->opt_gen;
    }
    bool split = (int64_t)P.nitems < 2048 && P.max_reads > 1;
    if (ctx->opt.score_mode == 1)
        split = false;
    else if (ctx->opt.score_mode == 2)
        split = true;
    if (int e = ensure_buf(ctx, ctx->scratch[15], sizeof(double) * std::max<int64_t>(P.dense_total, 1)))
        return e;
    if (split)
        if (int e = ensure_buf(ctx, ctx->scratch[10], sizeof(double) * std::max<int64_t>(P.split_total, 1)))
            return e;
    double *d_dense = (double *)ctx->scratch[15].p;
    HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
    if (P.nitems) {
        dim3 grid((unsigned)P.nitems, split ? (unsigned)P.max_reads : 1u);
        launch_scorer(ctx, P.pick, grid.x, grid.y, (const WorkItem *)ctx->scratch[11].p,
                      (const ScoreGroup *)ctx->scratch[12].p, (const ScoreRead *)ctx->scratch[13].p,
                      d_dense, split ? (double *)ctx->scratch[10].p : nullptr);
        if (split)
            hipLaunchKernelGGL(k_reduce, dim3((unsigned)((P.dense_total + 255) / 256)), dim3(256), 0,
                               ctx->stream, (const ScoreGroup *)ctx->scratch[12].p, ngroups,
                               (const int64_t *)ctx->scratch[14].p, P.dense_total,
                               (const double *)ctx->scratch[10].p, d_dense);
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    if (out && P.dense_total > 0) {
        HIPCHK(ctx, pre_d2h(ctx));
        HIPCHK(ctx, hipMemcpyAsync(out, d_dense, sizeof(double) * P.dense_total, out_kind, ctx->stream));
    }
    HIPCHK(ctx, stream_wait(ctx));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ctx->ev[2], ctx->ev[3]);
    ctx->score_ms = ms;
    ctx->gather_ms = 0;
    return 0;
}

int rf_score_dense(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                   double *out)
{
    return score_dense_impl(ctx, ngroups, slot_off, slots, out, hipMemcpyDeviceToHost);
}

int rf_score_dense_dev(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                       double *dev_out)
{
    if (!dev_out)
        return fail(ctx, RF_ERR_ARG, "rf_score_dense_dev: null device buffer");
    return score_dense_impl(ctx, ngroups, slot_off, slots, dev_out, hipMemcpyDeviceToDevice);
}

int rf_slot_geometry(rf_ctx *ctx, int32_t slot, int32_t which, int32_t *nrows, int32_t *ncols,
                     int32_t *bw, int32_t *H)
{
    if (!ctx || slot < 0 || slot >= (int32_t)ctx->slots.size())
        return fail(ctx, RF_ERR_ARG, "rf_slot_geometry: unknown slot");
    const Band &b = which == RF_BAND_A ? ctx->slots[slot].a : ctx->slots[slot].b;
    if (!b.valid)
        return fail(ctx, RF_ERR_STATE, "rf_slot_geometry: band not computed");
    if (nrows) *nrows = b.n + 1;
    if (ncols) *ncols = b.m + 1;
    if (bw) *bw = b.bw;
    if (H) *H = b.H;
    return 0;
}

int rf_download_band(rf_ctx *ctx, int32_t slot, int32_t which, double *out)
{
    if (!ctx || !out || slot < 0 || slot >= (int32_t)ctx->slots.size())
        return fail(ctx, RF_ERR_ARG, "rf_download_band: bad arguments");
    (void)hipSetDevice(ctx->device);
    const Band &b = which == RF_BAND_A ? ctx->slots[slot].a : ctx->slots[slot].b;
    if (!b.valid)
        return fail(ctx, RF_ERR_STATE, "rf_download_band: band not computed");
    // kappa-major device layout -> the reference's column-major data
    const int P = b.P;
    const int64_t K = band_K(b.H, b.m);
    std::vector<double> buf((size_t)K * P);
    HIPCHK(ctx, hipMemcpyAsync(buf.data(), ctx->band_arena.d + b.r.off, buf.size() * 8,
                               hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, stream_wait(ctx));
    for (int jj = 0; jj <= b.m; ++jj)
        for (int d = 0; d < b.H; ++d)
            out[(size_t)jj * b.H + d] = buf[(size_t)(d + 2 * jj) * P + (d >> 1)];
    return 0;
}

int rf_last_backtrace_ms(const rf_ctx *ctx, double *ms)
{
    if (!ctx || !ms)
        return RF_ERR_ARG;
    *ms = ctx->bt_ms;
    return 0;
}

int rf_last_codon_ms(const rf_ctx *ctx, double *ms)
{
    if (!ctx || !ms)
        return RF_ERR_ARG;
    *ms = ctx->codon_ms;
    return 0;
}

int rf_last_timing(const rf_ctx *ctx, double *dp_ms, double *score_ms, double *gather_ms)
{
    if (!ctx)
        return RF_ERR_ARG;
    if (dp_ms) *dp_ms = ctx->dp_ms;
    if (score_ms) *score_ms = ctx->score_ms;
    if (gather_ms) *gather_ms = ctx->gather_ms;
    return 0;
}

}  // extern "C"

// alignment_error_probs's per-column sums on the device (k_aln_sums) for
// rf_aln_error_sums (rifraf_batch.cpp): returns 1 (nothing done) when a read
// has no row codes -- the caller then folds the moves on the host.  out NULL:
// the sums stay on the device (scratch[19], rf_qv_probs).  A launch
// whose largest group has more than ALN_MARKS_MIN_READS reads uses
// k_aln_marks + k_aln_fold (RF_OPT_ALN_MARKS_MIN; tests set 0: always).
int rf_internal_aln_sums_dev(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                             const int32_t *tlen, double *out)
{
    if (ctx->opt.aln_sums_host)
        return 1;
    (void)hipSetDevice(ctx->device);
    const int32_t ns = ngroups > 0 ? slot_off[ngroups] : 0;
    for (int32_t k = 0; k < ns; ++k) {
        if (slots[k] < 0 || slots[k] >= (int32_t)ctx->slots.size() || !ctx->slots[slots[k]].a.valid)
            return fail(ctx, RF_ERR_STATE, "rf_aln_error_sums: slot has no A band");
        const SeqObj &S = ctx->seqs[ctx->slots[slots[k]].a.seq];
        if (!S.coded)
            return 1;
    }
    std::vector<BTTask> tasks;
    std::vector<int64_t> offs;
    if (int e = build_bt_tasks(ctx, ns, slots, tasks, offs))
        return e;
    // errlut for the dictionary entries added since the last call
    CodeDict &D = ctx->codes;
    const size_t n3 = D.t3v.size() / 4;
    const double log3 = std::log10(3.0);
    for (size_t e = D.errv.size(); e < n3; ++e)
        D.errv.push_back(std::log10(1.0 - std::pow(10.0, D.t3v[4 * e])) - log3);
    if (int e = ensure_buf(ctx, D.errlut, (size_t)RF_CODES * 8))
        return e;
    if (n3 > D.uperr)
        HIPCHK(ctx, hipMemcpyAsync((double *)D.errlut.p + D.uperr, D.errv.data() + D.uperr, (n3 - D.uperr) * 8,
                                   hipMemcpyHostToDevice, ctx->stream));
    D.uperr = n3;
    std::vector<AlnSumRead> rd(ns);
    std::vector<AlnSumGroup> gr(ngroups);
    int64_t rows = 0;
    for (int32_t g = 0; g < ngroups; ++g) {
        gr[g] = {rows * 4, slot_off[g], slot_off[g + 1], tlen[g], 0};
        rows += tlen[g];
        for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k) {
            const Band &b = ctx->slots[slots[k]].a;
            const SeqObj &S = ctx->seqs[b.seq];
            if (b.m != tlen[g])
                return fail(ctx, RF_ERR_ARG, "rf_aln_error_sums: consensus length differs from the A band's");
            rd[k] = {offs[k], S.tabs.off / 8 + row_code_off(S.n, S.ncins, S.ncdel), b.n, b.m, k, 0};
        }
    }
    if (ns > 0)
        if (int e = launch_backtraces(ctx, tasks, nullptr, 0))
            return e;
    if (int e = upload(ctx, ctx->scratch[17], rd)) return e;
    if (int e = upload(ctx, ctx->scratch[18], gr)) return e;
    if (int e = ensure_buf(ctx, ctx->scratch[19], (size_t)std::max<int64_t>(rows * 4 * 8, 16))) return e;
    int maxr = 0;
    for (int32_t g = 0; g < ngroups; ++g)
        maxr = std::max(maxr, slot_off[g + 1] - slot_off[g]);
    if (ngroups > 0 && maxr > ctx->opt.aln_marks_min && ns > 0) {
        // two launches: per-read marks, then a per-column ordered fold
        std::vector<int64_t> rbase(ns), gcol(ngroups + 1), gbase(ngroups);
        int64_t nm = 0, nc = 0;
        for (int32_t g = 0; g < ngroups; ++g) {
            gcol[g] = nc;
            gbase[g] = nm;
            nc += tlen[g];
            for (int32_t k = slot_off[g]; k < slot_off[g + 1]; ++k) {
                rbase[k] = nm;
                nm += tlen[g];
            }
        }
        gcol[ngroups] = nc;
        if (int e = upload(ctx, ctx->scratch[21], rbase)) return e;
        if (int e = upload(ctx, ctx->scratch[22], gcol)) return e;
        if (int e = upload(ctx, ctx->scratch[23], gbase)) return e;
        if (int e = ensure_buf(ctx, ctx->scratch[24], (size_t)std::max<int64_t>(nm * 4, 16))) return e;
        HIPCHK(ctx, hipMemsetAsync(ctx->scratch[24].p, 0, (size_t)nm * 4, ctx->stream));
        hipLaunchKernelGGL(k_aln_marks, dim3((unsigned)ns), dim3(64), 0, ctx->stream,
                           (const AlnSumGroup *)ctx->scratch[18].p, ngroups, (const AlnSumRead *)ctx->scratch[17].p,
                           (const int64_t *)ctx->scratch[21].p, (const double *)ctx->tab_arena.d,
                           (const int8_t *)ctx->scratch[3].p, (const int32_t *)ctx->scratch[4].p,
                           (uint32_t *)ctx->scratch[24].p);
        if (nc > 0)
            hipLaunchKernelGGL(k_aln_fold, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, ctx->stream,
                               (const AlnSumGroup *)ctx->scratch[18].p, ngroups, (const int64_t *)ctx->scratch[22].p,
                               (const int64_t *)ctx->scratch[23].p, (const uint32_t *)ctx->scratch[24].p,
                               (const double *)D.lut.p, (const double *)D.errlut.p, (double *)ctx->scratch[19].p, nc);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, pre_d2h(ctx));
        if (out)
            HIPCHK(ctx, hipMemcpyAsync(out, ctx->scratch[19].p, (size_t)rows * 4 * 8, hipMemcpyDeviceToHost,
                                       ctx->stream));
    } else if (ngroups > 0) {
        hipLaunchKernelGGL(k_aln_sums, dim3((unsigned)ngroups), dim3(256), 0, ctx->stream,
                           (const AlnSumGroup *)ctx->scratch[18].p, (const AlnSumRead *)ctx->scratch[17].p,
                           (const double *)ctx->tab_arena.d, (const int8_t *)ctx->scratch[3].p,
                           (const int32_t *)ctx->scratch[4].p, (const double *)D.lut.p, (const double *)D.errlut.p,
                           (double *)ctx->scratch[19].p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, pre_d2h(ctx));
        if (out)
            HIPCHK(ctx, hipMemcpyAsync(out, ctx->scratch[19].p, (size_t)rows * 4 * 8, hipMemcpyDeviceToHost,
                                       ctx->stream));
    }
    HIPCHK(ctx, stream_wait(ctx));
    if (ns > 0)
        note_bt_ms(ctx);
    return check_err(ctx);
}

// arena_grow count and seconds of a context (rf_rifraf_batch's RIFRAF_BATCH_TIMING line)
void rf_internal_arena_stats(const rf_ctx *ctx, int64_t *grows, double *secs)
{
    *grows = ctx ? ctx->arena_grows : 0;
    *secs = ctx ? ctx->arena_grow_s : 0.0;
}


// ---------------------------------------------------------------------
// k_qv: the quality pass's normalisations on the device (round 4)
//
// estimate_probs (model.jl:737-771, normalize_log_differences :722-735) and
// alignment_error_probs' final step (:835-839) for one cluster per
// workgroup, from its dense totals ((m+1) x 9, rf_score_dense's layout) and
// its per-column base-distribution sums (m x 4, k_aln_sums): the maxima,
// the checks and the row sums exactly as rf_host_qv_prep / rf_host_qv_finish
// (same order), with 10^x evaluated by the device's FP64 exp10 instead of the
// host's numpy power -- within 2 ulp of it, so the probabilities agree with
// the host path to ~1e-15 relative (tests/test_batch.py compares them at
// 1e-12), not bit for bit.  The consensus, scores and accepted proposals do
// not depend on this step.
// ---------------------------------------------------------------------
struct alignas(16) QvGroup {
    int64_t dense_off;   // doubles: (m + 1) x 9 dense totals
    int64_t sums_off;    // doubles: m x 4 alignment sums
    int64_t pos_off;     // rows of out_pos (m rows of 5)
    int64_t ins_off;     // rows of out_ins (m + 1 rows of 4)
    int64_t cons_off;    // bytes arena: the consensus bases
    double score;        // state.score
    int32_t m, pad;
};

__global__ void __launch_bounds__(256) k_qv(const QvGroup *__restrict__ groups, const double *__restrict__ dense,
                                            const double *__restrict__ sums, const uint8_t *__restrict__ bases,
                                            double *__restrict__ pos, double *__restrict__ ins,
                                            double *__restrict__ aln, int32_t *__restrict__ gerr)
{
    __shared__ double rS[4], rD[4], rI[4];
    __shared__ int rN[4];
    const QvGroup G = groups[blockIdx.x];
    const double *D = dense + G.dense_off;
    const uint8_t *cons = bases + G.cons_off;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, m = G.m;
    double mS = -RF_INF, mD = -RF_INF, mI = -RF_INF;
    int nan = 0;
    for (int p = tid; p <= m; p += 256) {
        const double *d = D + (size_t)p * 9;
        for (int q = 5; q < 9; ++q) {
            nan |= d[q] != d[q];
            mI = d[q] > mI ? d[q] : mI;
        }
        if (p >= 1) {
            const int cb = cons[p - 1];
            for (int q = 0; q < 5; ++q)
                nan |= (q != cb && d[q] != d[q]) ? 1 : 0;
            for (int q = 0; q < 4; ++q) {
                const double v = q == cb ? 0.0 + G.score : d[q];
                mS = v > mS ? v : mS;
            }
            mD = d[4] > mD ? d[4] : mD;
        }
    }
    // maxima are exact in any order
    for (int off = 32; off >= 1; off >>= 1) {
        mS = fmax(mS, __shfl_xor(mS, off));
        mD = fmax(mD, __shfl_xor(mD, off));
        mI = fmax(mI, __shfl_xor(mI, off));
        nan |= __shfl_xor(nan, off);
    }
    if (lane == 0) {
        rS[w] = mS;
        rD[w] = mD;
        rI[w] = mI;
        rN[w] = nan;
    }
    __syncthreads();
    mS = fmax(fmax(rS[0], rS[1]), fmax(rS[2], rS[3]));
    mD = fmax(fmax(rD[0], rD[1]), fmax(rD[2], rD[3]));
    mI = fmax(fmax(rI[0], rI[1]), fmax(rI[2], rI[3]));
    nan = rN[0] | rN[1] | rN[2] | rN[3];
    double mx = mS;   // Python max(mxS, mxD, mxI)
    if (mD > mx)
        mx = mD;
    if (mI > mx)
        mx = mI;
    const int e = nan ? 1 : mS - mx > 0.0 ? 2 : mD - mx > 0.0 ? 3 : mI - mx > 0.0 ? 4 : 0;
    if (tid == 0)
        gerr[blockIdx.x] = e;
    if (e)
        return;
    const double st_pow = exp10(G.score - mx);
    for (int p = tid; p <= m; p += 256) {
        const double *d = D + (size_t)p * 9;
        double ei[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            ei[q] = exp10(d[5 + q] - mx);
        const double si = st_pow + (((ei[0] + ei[1]) + ei[2]) + ei[3]);
        double *oi = ins + (size_t)(G.ins_off + p) * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            oi[q] = ei[q] / si;
        if (p >= 1) {
            const int cb = cons[p - 1];
            double ep[5];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                ep[q] = exp10((q == cb ? 0.0 + G.score : d[q]) - mx);
            ep[4] = exp10(d[4] - mx);
            const double sp = (((ep[0] + ep[1]) + ep[2]) + ep[3]) + ep[4];
            double *op = pos + (size_t)(G.pos_off + p - 1) * 5;
#pragma unroll
            for (int q = 0; q < 5; ++q)
                op[q] = ep[q] / sp;
            const double *a = sums + G.sums_off + (size_t)(p - 1) * 4;
            double ea[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                ea[q] = exp10(a[q]);
            const double t = ((ea[0] + ea[1]) + ea[2]) + ea[3];
            double mxq = ea[0] / t;
#pragma unroll
            for (int q = 1; q < 4; ++q) {   // numpy max: NaN propagates
                const double v = ea[q] / t;
                mxq = (mxq != mxq || !(v <= mxq)) ? (mxq != mxq ? mxq : v) : mxq;
            }
            aln[G.pos_off + p - 1] = 1.0 - mxq;
        }
    }
}

extern "C" int rf_qv_probs(rf_ctx *ctx, int32_t ngroups, const int32_t *slot_off, const int32_t *slots,
                           const int32_t *tlen, const double *score, double *out_pos, double *out_ins,
                           double *out_aln, int32_t *err_out)
{
    if (!ctx || ngroups < 0 ||
        (ngroups > 0 && (!slot_off || !slots || !tlen || !score || !out_pos || !out_ins || !out_aln || !err_out)))
        return fail(ctx, RF_ERR_ARG, "rf_qv_probs: bad arguments");
    err_out[0] = err_out[1] = 0;
    if (ngroups == 0)
        return 0;
    (void)hipSetDevice(ctx->device);
    // 1. dense totals, kept on the device (scratch[15], dplan's group offsets)
    if (int e = score_dense_impl(ctx, ngroups, slot_off, slots, nullptr, hipMemcpyDeviceToHost))
        return e;
    // 2. the alignment sums, kept on the device (scratch[19]); 1 = a read
    //    without row codes: the caller takes the host path
    if (int e = rf_internal_aln_sums_dev(ctx, ngroups, slot_off, slots, tlen, nullptr))
        return e;
    const auto &P = ctx->dplan;
    std::vector<QvGroup> gq(ngroups);
    int64_t rows = 0;
    for (int32_t g = 0; g < ngroups; ++g) {
        if (P.groups[g].m != tlen[g])
            return fail(ctx, RF_ERR_ARG, "rf_qv_probs: consensus length differs from the bands'");
        QvGroup &q = gq[g];
        q.dense_off = P.groups[g].dense_off;
        q.sums_off = rows * 4;
        q.pos_off = rows;
        q.ins_off = rows + g;
        q.cons_off = P.groups[g].tb;   // the consensus the dense totals were scored against
        q.score = score[g];
        q.m = tlen[g];
        rows += tlen[g];
    }
    if (int e = upload(ctx, ctx->scratch[25], gq)) return e;
    const size_t npos = (size_t)rows * 5, nins = (size_t)(rows + ngroups) * 4, naln = (size_t)rows;
    const size_t ob = align_up((npos + nins + naln) * 8, 256);
    if (int e = ensure_buf(ctx, ctx->scratch[26], ob + (size_t)ngroups * 4)) return e;
    double *d_pos = (double *)ctx->scratch[26].p, *d_ins = d_pos + npos, *d_aln = d_ins + nins;
    int32_t *d_gerr = (int32_t *)((char *)ctx->scratch[26].p + ob);
    hipLaunchKernelGGL(k_qv, dim3((unsigned)ngroups), dim3(256), 0, ctx->stream, (const QvGroup *)ctx->scratch[25].p,
                       (const double *)ctx->scratch[15].p, (const double *)ctx->scratch[19].p,
                       (const uint8_t *)ctx->bytes_arena.d, d_pos, d_ins, d_aln, d_gerr);
    HIPCHK(ctx, hipGetLastError());
    std::vector<int32_t> gerr(ngroups);
    HIPCHK(ctx, pre_d2h(ctx));
    HIPCHK(ctx, hipMemcpyAsync(out_pos, d_pos, npos * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(out_ins, d_ins, nins * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(out_aln, d_aln, naln * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(gerr.data(), d_gerr, (size_t)ngroups * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, stream_wait(ctx));
    for (int32_t g = 0; g < ngroups; ++g)
        if (gerr[g]) {
            err_out[0] = gerr[g];
            err_out[1] = g;
            break;
        }
    return 0;
}
