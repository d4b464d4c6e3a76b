// Diagnostic probe (not part of the product library): HBM read rate of the
// wide-band scorer's segment loads (k_score_segl) under two band layouts.
//
//   mode 1: kappa-major rows of P doubles (today's line-padded layout): a
//           segment D of work item a0 reads one 128-B line per kappa row in
//           [D + 2 a0, D + 2 a0 + 160), rows P*8 B apart;
//   mode 2: segment-major planes: plane D/32 holds the 16 doubles of every
//           kappa row contiguously, so the same 160 lines are one 20-KB run;
//   mode 3: 32-row blocks of kappa rows, segment-major inside a block;
//   mode 4: planes, items 160 rows apart (no overlap between neighbours);
//   mode 0: the same bytes per wave as one contiguous stream.
//
// One wave per work item (64 columns), one wave per SIMD (39 KB of dynamic LDS
// per workgroup, as the scorer), each wave walks its reads and segments in
// the scorer's order with one segment (20 lines per lane and band) in flight.
// usage: probe_seg NREADS H M [XCD_REMAP]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct dvec2 {
    double x, y;
};

template <int MODE>
__global__ void __launch_bounds__(64) k_probe_seg(const dvec2 *__restrict__ arena, long band_elems, int P, int K,
                                                   int nseg, int nitems, int nreads, int rgroups, double *out, int xcd)
{
    extern __shared__ double lds[];
    int lin = blockIdx.x;
    if (xcd) {   // k_score_segl's remap: consecutive cells on one XCD (blocks go round-robin over 8)
        const int ncell = gridDim.x, xq = ncell >> 3, xr = ncell & 7, x = lin & 7;
        lin = x * xq + min(x, xr) + (lin >> 3);
    }
    const int item = lin % nitems, rg = lin / nitems;
    const int r0 = (long)nreads * rg / rgroups, r1 = (long)nreads * (rg + 1) / rgroups;
    const int tid = threadIdx.x, r8 = tid >> 3, cc8 = tid & 7;
    const int a0 = 64 * item;
    double acc = 0;
    for (int r = r0; r < r1; ++r) {
        const double *gA = (const double *)arena + (long)r * 2 * band_elems;
        const double *gB = gA + band_elems;
        for (int s = 0; s < nseg; ++s) {
            const int D = 32 * s;
            dvec2 ra[20], rb[20];
#pragma unroll
            for (int j = 0; j < 20; ++j) {
                const int kap = min(D + 2 * a0 + r8 + 8 * j, K - 1);
                long o;
                if (MODE == 1)
                    o = (long)kap * P + (D >> 1) + 2 * cc8;
                else if (MODE == 2)
                    o = ((long)s * K + kap) * 16 + 2 * cc8;
                else if (MODE == 3)   // 32-row blocks, segment-major inside a block
                    o = (long)(kap >> 5) * 32 * P + (long)s * 512 + (kap & 31) * 16 + 2 * cc8;
                else if (MODE == 4)   // segment-major planes, items without the 32-row overlap
                    o = ((long)s * K + min(160 * item + r8 + 8 * j, K - 1)) * 16 + 2 * cc8;
                else
                    o = ((long)(item * nseg + s) * 160 + r8 + 8 * j) * 16 + 2 * cc8;
                ra[j] = *(const dvec2 *)(gA + o);
                rb[j] = *(const dvec2 *)(gB + o);
            }
#pragma unroll
            for (int j = 0; j < 20; ++j)
                acc += ra[j].x + ra[j].y + rb[j].x + rb[j].y;
        }
    }
    lds[tid] = acc;
    if (acc == 1.2345)
        out[blockIdx.x] = lds[tid ^ 1];
}

int main(int argc, char **argv)
{
    const int nreads = argc > 1 ? atoi(argv[1]) : 2000;
    const int H = argc > 2 ? atoi(argv[2]) : 141;
    const int m = argc > 3 ? atoi(argv[3]) : 10000;
    const int xcd = argc > 4 ? atoi(argv[4]) : 1;
    const int P = (((H + 1) / 2) + 15) & ~15;
    const int K = H + 2 * m;
    const int nseg = (H + 31) / 32;
    const long band_elems = ((long)K * P + 31) & ~31L;   // same bytes in both layouts (nseg*16 >= P)
    const long band_elems2 = (long)nseg * K * 16;
    const int nitems = (m + 1 + 63) / 64;
    const long band_elems0 = (long)nitems * nseg * 160 * 16;
    long be = band_elems > band_elems2 ? band_elems : band_elems2;
    be = be > band_elems0 ? be : band_elems0;
    const size_t bytes = (size_t)nreads * 2 * be * 8;
    dvec2 *arena;
    double *out;
    if (hipMalloc(&arena, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) {
        printf("alloc failed (%zu bytes)\n", bytes);
        return 1;
    }
    (void)hipMemset(arena, 0, bytes);
    const int rgroups = 32;
    const int nblocks = nitems * rgroups;
    const size_t lds = 39 * 1024;
    // algorithmic bytes read: every wave reads nseg * 160 lines per band per read
    const double rd = (double)nreads * nitems * nseg * 160 * 128 * 2;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 0; mode < 5; ++mode) {
            (void)hipEventRecord(e0);
            if (mode == 0)
                hipLaunchKernelGGL(k_probe_seg<0>, dim3(nblocks), dim3(64), lds, 0, arena, be, P, K, nseg, nitems,
                                   nreads, rgroups, out, xcd);
            else if (mode == 1)
                hipLaunchKernelGGL(k_probe_seg<1>, dim3(nblocks), dim3(64), lds, 0, arena, be, P, K, nseg, nitems,
                                   nreads, rgroups, out, xcd);
            else if (mode == 4)
                hipLaunchKernelGGL(k_probe_seg<4>, dim3(nblocks), dim3(64), lds, 0, arena, be, P, K, nseg, nitems,
                                   nreads, rgroups, out, xcd);
            else if (mode == 3)
                hipLaunchKernelGGL(k_probe_seg<3>, dim3(nblocks), dim3(64), lds, 0, arena, be, P, K, nseg, nitems,
                                   nreads, rgroups, out, xcd);
            else
                hipLaunchKernelGGL(k_probe_seg<2>, dim3(nblocks), dim3(64), lds, 0, arena, be, P, K, nseg, nitems,
                                   nreads, rgroups, out, xcd);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("{\"xcd\": %d, \"rep\": %d, \"mode\": %d, \"H\": %d, \"P\": %d, \"reads\": %d, \"ms\": %.3f, \"GBps\": %.1f}\n", xcd, rep,
                   mode, H, P, nreads, ms, rd / (ms * 1e-3) / 1e9);
        }
    }
    (void)hipFree(arena);
    return 0;
}
