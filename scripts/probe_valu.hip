// Diagnostic probe (not part of the product library): issue cost and
// dependent latency of the VALU ops the DP and the scorers are built from,
// on gfx950, at 1 and 2 waves per SIMD.  Each lane runs CH independent chains
// of N dependent ops; cycles per wave-instruction = clock64 delta / (CH * N).
// usage: probe_valu
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double op_add(double a, double b)
{
    double r;
    asm volatile("v_add_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double op_max(double a, double b)
{
    double r;
    asm volatile("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double op_fma(double a, double b)
{
    double r;
    asm volatile("v_fma_f64 %0, %1, %2, %1" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double op_sel(double a, double b)   // cmp + 2 cndmask (max without v_max_f64)
{
    const bool gt = a > b;
    const long long ai = __double_as_longlong(a), bi = __double_as_longlong(b);
    int lo = gt ? (int)ai : (int)bi, hi = gt ? (int)(ai >> 32) : (int)(bi >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double op_addu(double a, double b)   // v_add_u32 pair (integer reference)
{
    const long long ai = __double_as_longlong(a), bi = __double_as_longlong(b);
    int lo = (int)ai + (int)bi, hi = (int)(ai >> 32) + (int)(bi >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double op_dpp(double a, double b)   // two row_shr:1 dpp moves (one f64)
{
    const long long ai = __double_as_longlong(a);
    int lo = __builtin_amdgcn_mov_dpp((int)ai, 0x111, 0xF, 0xF, false);
    int hi = __builtin_amdgcn_mov_dpp((int)(ai >> 32), 0x111, 0xF, 0xF, false);
    asm volatile("" : "+v"(lo), "+v"(hi));
    (void)b;
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

template <int OP, int CH>
__global__ void __launch_bounds__(64) k_valu(double *out, int n, long long *cyc)
{
    double x[CH];
    const double y = 1e-300 * threadIdx.x;
#pragma unroll
    for (int c = 0; c < CH; ++c)
        x[c] = threadIdx.x + c;
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if (OP == 0)
                    x[c] = op_add(x[c], y);
                else if (OP == 1)
                    x[c] = op_max(x[c], y);
                else if (OP == 2)
                    x[c] = op_fma(x[c], y);
                else if (OP == 3)
                    x[c] = op_sel(x[c], y);
                else if (OP == 4)
                    x[c] = op_addu(x[c], y);
                else
                    x[c] = op_dpp(x[c], y);
            }
    }
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c)
        s += x[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0)
        cyc[blockIdx.x] = t1 - t0;
}

template <int OP, int CH>
void run(const char *name, double *out, long long *cyc, int wps)
{
    const int n = 4096;
    const int blocks = 256 * 4 * wps;   // wps waves per SIMD on 256 CUs
    hipLaunchKernelGGL((k_valu<OP, CH>), dim3(blocks), dim3(64), 0, 0, out, n, cyc);   // warm
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_valu<OP, CH>), dim3(blocks), dim3(64), 0, 0, out, n, cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double ops = (double)n * 8 * CH;   // wave-instructions (ops) per wave
    // time-based: wave-ops per SIMD per ns; at 2.4 GHz -> cycles per op
    const double ns_per_op = ms * 1e6 / (ops * wps);
    printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"clock64_per_op\": %.2f, "
           "\"ns_per_op_per_simd\": %.3f, \"cycles_per_op_at_2.4GHz\": %.2f}\n",
           name, CH, wps, ms, (double)c / ops, ns_per_op, ns_per_op * 2.4);
}

int main()
{
    double *out;
    long long *cyc;
    (void)hipMalloc(&out, 256 * 4 * 8 * 64 * 8);
    (void)hipMalloc(&cyc, 256 * 4 * 8 * 8);
    for (int wps = 1; wps <= 2; ++wps) {
        run<0, 1>("v_add_f64", out, cyc, wps);
        run<0, 8>("v_add_f64", out, cyc, wps);
        run<1, 1>("v_max_f64", out, cyc, wps);
        run<1, 8>("v_max_f64", out, cyc, wps);
        run<2, 8>("v_fma_f64", out, cyc, wps);
        run<3, 1>("cmp_f64+2cndmask", out, cyc, wps);
        run<3, 8>("cmp_f64+2cndmask", out, cyc, wps);
        run<4, 8>("2x v_add_u32", out, cyc, wps);
        run<5, 8>("2x v_mov_b32_dpp", out, cyc, wps);
    }
    return 0;
}
