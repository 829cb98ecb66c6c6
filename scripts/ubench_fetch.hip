// ubench_fetch.hip -- what a random gather costs on MI355X, and how the PMC
// counters count it (dev tool; VERDICT r03 "calibrate FETCH_SIZE for random
// 8-B gathers").  Each kernel issues a KNOWN number of requests of a known
// width, so rocprofv3 --pmc FETCH_SIZE / TCC_EA0_RDREQ_sum / WRITE_SIZE over
// this binary give bytes per request for each access class:
//   stream_rd   320 MB read once, 16 B per lane, coalesced (the guide's
//               calibrated case: FETCH_SIZE = 1/2 of the bytes)
//   gath<W>     10M gathers of W bytes at random W-aligned offsets of a
//               3.16 GB table (W = 8, 16, 32, 64, 128; W > 16 = W/16 lanes
//               per gather, one 16-B piece each), 10M x 1-B results out
//   scat<F>     10M random 16-B stores into a footprint of F bytes
//               (147 MB: the compact slab; 3.16 GB)
//   atom        10M atomicAdd on 100k counters (the scatter's slot atomic)
// Table allocations: hipMalloc (default), plus uncached and fine-grained
// variants of gath<8> (does a non-caching MTYPE fetch less than a line?).
// Each kernel: one warm launch, then the median of 9 timed launches; every
// index is reduced modulo the table, nothing is out of bounds.
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

constexpr size_t kN = 10000000;

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void k_stream_rd(const uint4* __restrict__ a, size_t n16, unsigned* __restrict__ out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// W-byte gathers; lanes per gather L = max(1, W / 16); gather g is served by
// lanes [g*L, g*L+L) of consecutive threads, each loading its 16-B piece (or
// one 8-B word for W = 8)
template <int W>
__global__ __launch_bounds__(256) void k_gath(const unsigned char* __restrict__ tab, size_t tbytes,
                                              unsigned char* __restrict__ out, size_t n) {
    constexpr int L = W >= 16 ? W / 16 : 1;
    const size_t slots = tbytes / W;
    const size_t nthreads = n * L;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < nthreads; t += (size_t)gridDim.x * blockDim.x) {
        const size_t g = t / L;
        const size_t off = (mix(g * 0x9E3779B97F4A7C15ull + 1) % slots) * W + (t % L) * (W >= 16 ? 16 : 0);
        unsigned v;
        if (W == 8) {
            const uint2 q = *reinterpret_cast<const uint2*>(tab + off);
            v = q.x ^ q.y;
        } else {
            const uint4 q = *reinterpret_cast<const uint4*>(tab + off);
            v = q.x ^ q.w;
        }
        if (t % L == 0) out[g] = (unsigned char)v;
        else if (v == 0x12345678u) out[g] = 1;
    }
}

__global__ __launch_bounds__(256) void k_scat(uint4* __restrict__ buf, size_t nent, size_t n) {
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (size_t)gridDim.x * blockDim.x)
        buf[mix(g * 0x9E3779B97F4A7C15ull + 7) % nent] = make_uint4((unsigned)g, 1u, 2u, 3u);
}

__global__ __launch_bounds__(256) void k_atom(unsigned* __restrict__ cnt, unsigned H, size_t n) {
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (size_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[mix(g * 0x9E3779B97F4A7C15ull + 3) % H], 1u);
}

template <typename F>
float timeit(F launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 9; r++) {
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ts[ts.size() / 2];
}

int main() {
    const size_t A = 19870, tbytes = A * A * 8; // the C3 packet-path table (8-B entries)
    const size_t sbytes = 320000000;             // 10M 32-B records
    unsigned char *tab, *out;
    uint4 *st, *slab;
    unsigned *cnt, *sink;
    CHECK(hipMalloc(&tab, tbytes));
    CHECK(hipMemset(tab, 0x3c, tbytes));
    CHECK(hipMalloc(&out, kN));
    CHECK(hipMalloc(&st, sbytes));
    CHECK(hipMemset(st, 1, sbytes));
    const size_t slab_ent = 100000ull * 128; // 100k hosts x 128 slots x 16 B = 205 MB
    CHECK(hipMalloc(&slab, slab_ent * 16));
    CHECK(hipMalloc(&cnt, 100000 * 4));
    CHECK(hipMemset(cnt, 0, 100000 * 4));
    CHECK(hipMalloc(&sink, 4));
    const int G = 8192;
    printf("requests per launch: 10M (stream_rd: %zu 16-B lane loads)\n", sbytes / 16);
    float t = timeit([&] { hipLaunchKernelGGL(k_stream_rd, dim3(G), dim3(256), 0, 0, st, sbytes / 16, sink); });
    printf("stream_rd     320 MB               %8.4f ms  %7.1f GB/s\n", t, sbytes / (t * 1e6));
    fflush(stdout);
#define GATH(W)                                                                                                   \
    do {                                                                                                          \
        float tt = timeit([&] { hipLaunchKernelGGL(k_gath<W>, dim3(G), dim3(256), 0, 0, tab, tbytes, out, kN); }); \
        printf("gath<%3d>     3.16 GB table       %8.4f ms  %7.1f G gathers/s  %7.1f GB/s at %d B\n", W, tt,         \
               kN / (tt * 1e6), kN * (double)W / (tt * 1e6), W);                                                  \
        fflush(stdout);                                                                                           \
    } while (0)
    GATH(8);
    GATH(16);
    GATH(32);
    GATH(64);
    GATH(128);
    t = timeit([&] { hipLaunchKernelGGL(k_scat, dim3(G), dim3(256), 0, 0, slab, slab_ent, kN); });
    printf("scat          %5.0f MB footprint    %8.4f ms  %7.1f G stores/s\n", slab_ent * 16 / 1e6, t, kN / (t * 1e6));
    t = timeit([&] { hipLaunchKernelGGL(k_scat, dim3(G), dim3(256), 0, 0, (uint4*)tab, tbytes / 16, kN); });
    printf("scat          3.16 GB footprint    %8.4f ms  %7.1f G stores/s\n", t, kN / (t * 1e6));
    t = timeit([&] { hipLaunchKernelGGL(k_atom, dim3(G), dim3(256), 0, 0, cnt, 100000u, kN); });
    printf("atom          100k counters        %8.4f ms  %7.1f G atomics/s\n", t, kN / (t * 1e6));
    fflush(stdout);
    const unsigned flags[] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
    const char* names[] = {"uncached", "finegrained"};
    for (int f = 0; f < 2; f++) {
        unsigned char* t2 = nullptr;
        if (hipExtMallocWithFlags((void**)&t2, tbytes, flags[f]) != hipSuccess) {
            (void)hipGetLastError();
            printf("%s: allocation refused\n", names[f]);
            continue;
        }
        CHECK(hipMemset(t2, 0x3c, tbytes));
        float a8 = timeit([&] { hipLaunchKernelGGL(k_gath<8>, dim3(G), dim3(256), 0, 0, t2, tbytes, out, kN); });
        float a64 = timeit([&] { hipLaunchKernelGGL(k_gath<64>, dim3(G), dim3(256), 0, 0, t2, tbytes, out, kN); });
        printf("%-12s  gath<8> %8.4f ms (%5.1f G/s)  gath<64> %8.4f ms (%5.1f G/s)\n", names[f], a8, kN / (a8 * 1e6),
               a64, kN / (a64 * 1e6));
        fflush(stdout);
        CHECK(hipFree(t2));
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
