// ubench_gather.hip -- random-gather cost of the packet-scatter kernel on
// MI355X (dev tool).  10M 32-B records, host->slot gathers (100k hosts), one
// table gather per record over an A x A table with 16-B {lat, rel} or 8-B
// {delay, threshold} entries.  Prints the median ms of 10 launches.
// Every index is clamped in-kernel; records past n are never dereferenced.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Pkt {
    unsigned long long now, seq;
    unsigned src, dst, rng, pay;
};
struct Ent16 {
    double lat, rel;
};
struct Ent8 {
    unsigned delay, thr;
};

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

template <typename E, int BATCH>
__global__ __launch_bounds__(256) void k(const Pkt* __restrict__ r, size_t n, const int* __restrict__ hs, unsigned H,
                                         const E* __restrict__ tab, unsigned A, unsigned char* __restrict__ st) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * BATCH) {
        unsigned src[BATCH], dst[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; b++) {
            const size_t i = i0 + b * stride;
            src[b] = 0;
            dst[b] = 0;
            if (i < n) {
                src[b] = r[i].src % H;
                dst[b] = r[i].dst % H;
            }
        }
        unsigned si[BATCH], di[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; b++) {
            si[b] = (unsigned)hs[src[b]] % A;
            di[b] = (unsigned)hs[dst[b]] % A;
        }
        E e[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; b++) e[b] = tab[(size_t)si[b] * A + di[b]];
#pragma unroll
        for (int b = 0; b < BATCH; b++) {
            const size_t i = i0 + b * stride;
            if (i < n) st[i] = (unsigned char)(((const unsigned*)&e[b])[0] & 1u);
        }
    }
}

// streaming reference: read the 32-B record, write a 32-B event + status
__global__ __launch_bounds__(256) void k_copy(const Pkt* __restrict__ r, size_t n, Pkt* __restrict__ o,
                                              unsigned char* __restrict__ st) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        Pkt p = r[i];
        p.seq += 1;
        o[i] = p;
        st[i] = 1;
    }
}

// gathers + the 32-B event write (the scatter kernel's traffic without its logic)
template <typename E, int BATCH>
__global__ __launch_bounds__(256) void kw(const Pkt* __restrict__ r, size_t n, const int* __restrict__ hs, unsigned H,
                                          const E* __restrict__ tab, unsigned A, Pkt* __restrict__ o,
                                          unsigned char* __restrict__ st) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * BATCH) {
        Pkt p[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; b++) {
            const size_t i = i0 + b * stride;
            if (i < n) p[b] = r[i];
            else p[b] = Pkt{0, 0, 0, 0, 0, 0};
        }
        unsigned si[BATCH], di[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; b++) {
            si[b] = (unsigned)hs[p[b].src % H] % A;
            di[b] = (unsigned)hs[p[b].dst % H] % A;
        }
        E e[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; b++) e[b] = tab[(size_t)si[b] * A + di[b]];
#pragma unroll
        for (int b = 0; b < BATCH; b++) {
            const size_t i = i0 + b * stride;
            if (i < n) {
                p[b].now += ((const unsigned*)&e[b])[0];
                o[i] = p[b];
                st[i] = 1;
            }
        }
    }
}

template <typename E, int BATCH>
float runw(const Pkt* r, size_t n, const int* hs, unsigned H, const E* tab, unsigned A, Pkt* o, unsigned char* st,
           int grid) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 12; rep++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((kw<E, BATCH>), dim3(grid), dim3(256), 0, 0, r, n, hs, H, tab, A, o, st);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

template <typename E, int BATCH>
float run(const Pkt* r, size_t n, const int* hs, unsigned H, const E* tab, unsigned A, unsigned char* st, int grid) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 12; rep++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((k<E, BATCH>), dim3(grid), dim3(256), 0, 0, r, n, hs, H, tab, A, st);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t n = 10000000;
    const unsigned H = 100000;
    std::vector<Pkt> hp(n);
    unsigned long long s = 88172645463325252ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (size_t i = 0; i < n; i++) hp[i] = Pkt{rnd() % 10000000, i, (unsigned)(rnd() % H), (unsigned)(rnd() % H), 1, 1};
    Pkt* r;
    int* hs;
    unsigned char* st;
    CHECK(hipMalloc(&r, n * sizeof(Pkt)));
    CHECK(hipMalloc(&hs, H * 4));
    CHECK(hipMalloc(&st, n));
    CHECK(hipMemcpy(r, hp.data(), n * sizeof(Pkt), hipMemcpyHostToDevice));
    Pkt* o;
    CHECK(hipMalloc(&o, n * sizeof(Pkt)));
    {
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        std::vector<float> ts;
        for (int rep = 0; rep < 12; rep++) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, r, n, o, st);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (rep >= 2) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("stream copy 32B in + 32B out + 1B status: %.3f ms (%.0f GB/s)\n", ts[ts.size() / 2],
               n * 65.0 / (ts[ts.size() / 2] * 1e6));
    }
    const unsigned As[] = {1000, 4000, 19870};
    const size_t maxA = 19870;
    void* tab;
    CHECK(hipMalloc(&tab, maxA * maxA * 16));
    CHECK(hipMemset(tab, 0x3f, maxA * maxA * 16));
    for (unsigned A : As) {
        {
            std::vector<int> hhs(H);
            for (unsigned h = 0; h < H; h++) hhs[h] = (int)(rnd() % A);
            CHECK(hipMemcpy(hs, hhs.data(), H * 4, hipMemcpyHostToDevice));
            printf("A=%5u | +32B write: 16B b4 %.3f ms  b8 %.3f ms | 8B b4 %.3f ms  b8 %.3f ms\n", A,
                   runw<Ent16, 4>(r, n, hs, H, (const Ent16*)tab, A, o, st, 8192),
                   runw<Ent16, 8>(r, n, hs, H, (const Ent16*)tab, A, o, st, 8192),
                   runw<Ent8, 4>(r, n, hs, H, (const Ent8*)tab, A, o, st, 8192),
                   runw<Ent8, 8>(r, n, hs, H, (const Ent8*)tab, A, o, st, 8192));
        }
        std::vector<int> hhs(H);
        for (unsigned h = 0; h < H; h++) hhs[h] = (int)(rnd() % A);
        CHECK(hipMemcpy(hs, hhs.data(), H * 4, hipMemcpyHostToDevice));
        printf("A=%5u | 16B entries (%.2f GB): b4 %.3f ms  b8 %.3f ms | 8B entries (%.2f GB): b4 %.3f ms  b8 %.3f ms\n",
               A, (double)A * A * 16 / 1e9, run<Ent16, 4>(r, n, hs, H, (const Ent16*)tab, A, st, 8192),
               run<Ent16, 8>(r, n, hs, H, (const Ent16*)tab, A, st, 8192), (double)A * A * 8 / 1e9,
               run<Ent8, 4>(r, n, hs, H, (const Ent8*)tab, A, st, 8192),
               run<Ent8, 8>(r, n, hs, H, (const Ent8*)tab, A, st, 8192));
    }
    // the same A=19870 gathers from tables allocated uncached / fine-grained
    // (MTYPE UC / CC: no L2 line fill on a miss) -- does a random 16-B read
    // then fetch less than a 128-B line?
    {
        std::vector<int> hhs(H);
        for (unsigned h = 0; h < H; h++) hhs[h] = (int)(rnd() % maxA);
        CHECK(hipMemcpy(hs, hhs.data(), H * 4, hipMemcpyHostToDevice));
        const unsigned flags[] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
        const char* names[] = {"uncached", "finegrained"};
        for (int f = 0; f < 2; f++) {
            void* t2 = nullptr;
            if (hipExtMallocWithFlags(&t2, maxA * maxA * 16, flags[f]) != hipSuccess) {
                (void)hipGetLastError();
                printf("%s: allocation refused\n", names[f]);
                continue;
            }
            CHECK(hipMemset(t2, 0x3f, maxA * maxA * 16));
            printf("A=%5u %s | 16B entries: b4 %.3f ms  b8 %.3f ms | +32B write b4 %.3f ms\n", (unsigned)maxA, names[f],
                   run<Ent16, 4>(r, n, hs, H, (const Ent16*)t2, maxA, st, 8192),
                   run<Ent16, 8>(r, n, hs, H, (const Ent16*)t2, maxA, st, 8192),
                   runw<Ent16, 4>(r, n, hs, H, (const Ent16*)t2, maxA, o, st, 8192));
            CHECK(hipFree(t2));
        }
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
