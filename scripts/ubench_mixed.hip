// ubench_mixed.hip -- the random request-rate ceiling the routing kernels are
// compared against (dev tool).  Independent random 16-byte
// requests, a mix of reads and writes (the SSSP slab kernels issue ~55 %
// reads, ~45 % writes per heap pop), over footprints from Infinity-Cache size
// to the C4 slab footprint.  Each thread draws its addresses from a private
// xorshift stream (no index array: the only memory traffic is the measured
// requests); reads are folded into a value that the writes store, so nothing
// is dead code.  Prints median G requests/s of 7 launches per case.
// Every address is taken modulo the footprint; nothing is accessed out of
// bounds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int kB = 8; // requests in flight per thread per step

__device__ __forceinline__ unsigned long long xs(unsigned long long& s) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}

// steps x kB requests per thread; request j of a step is a write iff
// (j * 256 / kB) < wr_frac256
__global__ __launch_bounds__(256) void k_mixed(double2* __restrict__ buf, unsigned long long nent, int steps,
                                               int wr_frac256, double* __restrict__ sink) {
    unsigned long long s = 0x9E3779B97F4A7C15ull ^ ((unsigned long long)(blockIdx.x * blockDim.x + threadIdx.x) * 0xBF58476D1CE4E5B9ull);
    double acc = 0.0;
    for (int st = 0; st < steps; st++) {
        unsigned long long a[kB];
#pragma unroll
        for (int j = 0; j < kB; j++) a[j] = xs(s) % nent;
        double2 v[kB];
#pragma unroll
        for (int j = 0; j < kB; j++)
            if (j * 256 / kB >= wr_frac256) v[j] = buf[a[j]];
#pragma unroll
        for (int j = 0; j < kB; j++) {
            if (j * 256 / kB >= wr_frac256) acc += v[j].x + v[j].y;
            else buf[a[j]] = make_double2(acc, (double)st);
        }
    }
    if (acc == 12345.678) sink[0] = acc; // never true; keeps the reads live
}

int main(int argc, char** argv) {
    const size_t max_gb = argc > 1 ? (size_t)atol(argv[1]) : 32;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const size_t maxb = max_gb << 30;
    double2* buf = nullptr;
    double* sink = nullptr;
    CHECK(hipMalloc((void**)&buf, maxb));
    CHECK(hipMalloc((void**)&sink, 8));
    CHECK(hipMemset(buf, 0, maxb));
    const int grid = prop.multiProcessorCount * 32, steps = 64;
    const double reqs = (double)grid * 256 * steps * kB;
    const size_t foot_mb[] = {64, 1024, 6u << 10, 30u << 10};
    const int wr[] = {0, 96, 128, 160, 256}; // 0, 37.5, 50, 62.5, 100 % writes (kB = 8: whole eighths)
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    printf("%d CUs, grid %d x 256, %d x %d requests per thread (%.3g per launch)\n", prop.multiProcessorCount, grid,
           steps, kB, reqs);
    for (size_t f : foot_mb) {
        if ((f << 20) > maxb) continue;
        const unsigned long long nent = (unsigned long long)((f << 20) / sizeof(double2));
        for (int w : wr) {
            std::vector<float> ts;
            for (int rep = 0; rep < 8; rep++) {
                CHECK(hipEventRecord(a));
                k_mixed<<<grid, 256>>>(buf, nent, steps, w, sink);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                if (rep) ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            const float med = ts[ts.size() / 2];
            printf("footprint %6zu MB  writes %5.1f %%  %.3f ms  %.1f G requests/s\n", f, 100.0 * w / 256.0, med,
                   reqs / (med * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
