// probe_bw.hip -- HBM bandwidth probes (diagnostics, NOT part of the engine).
//
// bench.py reports the attainable stream-read and store bandwidth of the box
// beside its roofline fractions (stream_read_gbs, stream_write_gbs): the
// scorer's reads and the DP fill's nontemporal 16-B band stores, measured on
// a buffer of the same size as the c4 step's band arena.  Built by
// __graft_entry__.build() into scripts/libprobe_bw.so; scripts/probe_bw.py
// is the ctypes wrapper.  The engine library (librifraf_hip.so) carries no
// probe code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace {

typedef double dvec2 __attribute__((ext_vector_type(2)));

// stream read: grid-stride 16-B loads, 8 in flight per lane
__global__ void __launch_bounds__(256) k_read(const dvec2 *__restrict__ src, int64_t n16, double *__restrict__ sink)
{
    const int64_t stride = (int64_t)gridDim.x * 256 * 8;
    double acc = 0.0;
    for (int64_t base = (int64_t)blockIdx.x * 256 * 8 + threadIdx.x; base < n16; base += stride) {
        dvec2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t e = base + u * 256;
            v[u] = e < n16 ? src[e] : dvec2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            acc += v[u].x + v[u].y;
    }
    if (acc == 12345.678)   // data dependence keeps the loads alive
        sink[0] = acc;
}

// mode 1: grid-stride 16-B stores; mode 2: the DP fill's pattern -- 16-lane
// streams (4 per wave), each writing its own contiguous region in chunks of
// chunk16 16-B units; modes 3 / 4: modes 1 / 2 with nontemporal stores
__global__ void __launch_bounds__(64) k_write(dvec2 *__restrict__ dst, int64_t n16, int mode, int chunk16,
                                              int nstreams)
{
    const dvec2 v = {1.0, 2.0};
    const bool nt = mode >= 3;
    if (mode == 1 || mode == 3) {
        const int64_t stride = (int64_t)gridDim.x * 64;
        for (int64_t e = (int64_t)blockIdx.x * 64 + threadIdx.x; e < n16; e += stride) {
            if (nt)
                __builtin_nontemporal_store(v, dst + e);
            else
                dst[e] = v;
        }
        return;
    }
    const int sid = blockIdx.x * 4 + (threadIdx.x >> 4);
    const int q = threadIdx.x & 15;
    if (sid >= nstreams)
        return;
    const int64_t per = n16 / nstreams;
    dvec2 *g = dst + (int64_t)sid * per;
    for (int64_t c0 = 0; c0 + chunk16 <= per; c0 += chunk16) {
        for (int e = q; e < chunk16; e += 16) {
            if (nt)
                __builtin_nontemporal_store(v, g + c0 + e);
            else
                g[c0 + e] = v;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

struct Probe {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    void *buf = nullptr;
    double *sink = nullptr;
    int64_t bytes = 0;
};

float timed(Probe *p, auto launch, int reps)
{
    (void)hipEventRecord(p->ev[0], p->stream);
    for (int r = 0; r < reps; ++r)
        launch();
    (void)hipEventRecord(p->ev[1], p->stream);
    (void)hipStreamSynchronize(p->stream);
    float t = 0;
    (void)hipEventElapsedTime(&t, p->ev[0], p->ev[1]);
    return t / reps;
}

}  // namespace

extern "C" {

// A probe over `bytes` of fresh device memory on `device`; NULL on failure.
void *pb_open(int device, int64_t bytes)
{
    Probe *p = new Probe;
    p->device = device;
    p->bytes = bytes & ~(int64_t)15;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&p->ev[0]) != hipSuccess || hipEventCreate(&p->ev[1]) != hipSuccess ||
        hipMalloc(&p->buf, std::max<int64_t>(p->bytes, 16)) != hipSuccess ||
        hipMalloc((void **)&p->sink, 64) != hipSuccess) {
        delete p;
        return nullptr;
    }
    return p;
}

void pb_close(void *h)
{
    Probe *p = (Probe *)h;
    if (!p)
        return;
    (void)hipSetDevice(p->device);
    (void)hipFree(p->buf);
    (void)hipFree(p->sink);
    (void)hipEventDestroy(p->ev[0]);
    (void)hipEventDestroy(p->ev[1]);
    (void)hipStreamDestroy(p->stream);
    delete p;
}

// mean ms of one stream-read pass over the buffer (reps passes)
int pb_read(void *h, int32_t reps, double *ms)
{
    Probe *p = (Probe *)h;
    if (!p || reps < 1 || !ms)
        return -1;
    (void)hipSetDevice(p->device);
    *ms = timed(p, [&] {
        hipLaunchKernelGGL(k_read, dim3(256 * 8), dim3(256), 0, p->stream, (const dvec2 *)p->buf, p->bytes / 16,
                           p->sink);
    }, reps);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ms of one write pass (modes above)
int pb_write(void *h, int32_t mode, int32_t chunk_bytes, int32_t nstreams, double *ms)
{
    Probe *p = (Probe *)h;
    if (!p || !ms || mode < 1 || mode > 4 || ((mode & 1) == 0 && (chunk_bytes < 16 || nstreams < 1)))
        return -1;
    (void)hipSetDevice(p->device);
    const unsigned blocks = (mode & 1) ? 256 * 32 : (unsigned)((nstreams + 3) / 4);
    *ms = timed(p, [&] {
        hipLaunchKernelGGL(k_write, dim3(blocks), dim3(64), 0, p->stream, (dvec2 *)p->buf, p->bytes / 16, mode,
                           chunk_bytes / 16, nstreams);
    }, 1);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
