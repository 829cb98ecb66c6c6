// ubench_scatter.hip -- where the packet-scatter kernel's time goes (dev tool).
// 10M 32-B records; variants add one access class at a time:
//   copy      record in, 32-B event + 1-B status out (streaming floor)
//   host4     + 2 x 4-B host->slot gathers (400 KB array, L2-resident)
//   host8     + 2 x 8-B host_info gathers (800 KB, as the product kernel)
//   tab       + the 16-B table gather (A x A entries)
//   tabonly   record in + table gather at a hashed index (no host gathers) + out
// each at several (items per thread, waves per CU) shapes.  Median of 10.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Pkt {
    unsigned long long now, seq;
    unsigned src, dst, rng, pay;
};
struct Ent {
    double lat, rel;
};

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

enum { COPY = 0, HOST4 = 1, HOST8 = 2, TAB = 3, TABONLY = 4 };

template <int MODE, int B>
__global__ __launch_bounds__(256) void k(const Pkt* __restrict__ r, size_t n, const unsigned* __restrict__ h4,
                                         const uint2* __restrict__ h8, unsigned H, const Ent* __restrict__ tab,
                                         unsigned A, Pkt* __restrict__ o, unsigned char* __restrict__ st) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * B) {
        Pkt p[B];
#pragma unroll
        for (int b = 0; b < B; b++) {
            const size_t i = i0 + b * stride;
            if (i < n) p[b] = r[i];
            else p[b] = Pkt{0, 0, 0, 0, 0, 0};
        }
        unsigned si[B], di[B];
#pragma unroll
        for (int b = 0; b < B; b++) {
            if (MODE == HOST4 || MODE == TAB) {
                si[b] = h4[p[b].src % H] % A;
                di[b] = h4[p[b].dst % H] % A;
            } else if (MODE == HOST8) {
                const uint2 a = h8[p[b].src % H], c = h8[p[b].dst % H];
                si[b] = (a.x ^ c.y) % A;
                di[b] = (c.x ^ a.y) % A;
            } else {
                si[b] = (p[b].src * 2654435761u) % A;
                di[b] = (p[b].dst * 40503u + 7u) % A;
            }
        }
        double v[B];
#pragma unroll
        for (int b = 0; b < B; b++) {
            if (MODE == TAB || MODE == TABONLY) {
                const Ent e = tab[(size_t)si[b] * A + di[b]];
                v[b] = e.lat + e.rel;
            } else {
                v[b] = (double)(si[b] + di[b]);
            }
        }
#pragma unroll
        for (int b = 0; b < B; b++) {
            const size_t i = i0 + b * stride;
            if (i < n) {
                p[b].now += (unsigned long long)v[b];
                o[i] = p[b];
                st[i] = (unsigned char)p[b].now;
            }
        }
    }
}

template <int MODE, int B>
float run(const Pkt* r, size_t n, const unsigned* h4, const uint2* h8, unsigned H, const Ent* tab, unsigned A, Pkt* o,
          unsigned char* st, int grid) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 12; rep++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((k<MODE, B>), dim3(grid), dim3(256), 0, 0, r, n, h4, h8, H, tab, A, o, st);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

template <int MODE>
void row(const char* name, const Pkt* r, size_t n, const unsigned* h4, const uint2* h8, unsigned H, const Ent* tab,
         unsigned A, Pkt* o, unsigned char* st) {
    printf("%-8s A=%5u |", name, A);
    const int grids[] = {1024, 2048, 4096, 8192};
    for (int g : grids) printf(" g%d b1 %.3f b4 %.3f b8 %.3f |", g, run<MODE, 1>(r, n, h4, h8, H, tab, A, o, st, g),
                               run<MODE, 4>(r, n, h4, h8, H, tab, A, o, st, g),
                               run<MODE, 8>(r, n, h4, h8, H, tab, A, o, st, g));
    printf("\n");
    fflush(stdout);
}

int main(int argc, char** argv) {
    const size_t n = 10000000;
    const unsigned H = 100000;
    const bool sorted_src = argc > 1;
    std::vector<Pkt> hp(n);
    unsigned long long s = 88172645463325252ull;
    auto rnd = [&]() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    };
    for (size_t i = 0; i < n; i++) hp[i] = Pkt{rnd() % 10000000, i, (unsigned)(rnd() % H), (unsigned)(rnd() % H), 1, 1};
    if (sorted_src) std::sort(hp.begin(), hp.end(), [](const Pkt& a, const Pkt& b) { return a.src < b.src; });
    Pkt *r, *o;
    unsigned* h4;
    uint2* h8;
    unsigned char* st;
    CHECK(hipMalloc(&r, n * sizeof(Pkt)));
    CHECK(hipMalloc(&o, n * sizeof(Pkt)));
    CHECK(hipMalloc(&h4, H * 4));
    CHECK(hipMalloc(&h8, H * 8));
    CHECK(hipMalloc(&st, n));
    CHECK(hipMemcpy(r, hp.data(), n * sizeof(Pkt), hipMemcpyHostToDevice));
    const unsigned As[] = {250, 19870};
    Ent* tab;
    CHECK(hipMalloc(&tab, (size_t)19870 * 19870 * 16));
    CHECK(hipMemset(tab, 0x3f, (size_t)19870 * 19870 * 16));
    printf("records %s; ms per 10M-record launch\n", sorted_src ? "sorted by src" : "in random order");
    for (unsigned A : As) {
        std::vector<unsigned> a4(H);
        std::vector<uint2> a8(H);
        for (unsigned h = 0; h < H; h++) a4[h] = (unsigned)(rnd() % A), a8[h] = make_uint2(a4[h], (unsigned)rnd());
        CHECK(hipMemcpy(h4, a4.data(), H * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(h8, a8.data(), H * 8, hipMemcpyHostToDevice));
        if (A == As[0]) {
            row<COPY>("copy", r, n, h4, h8, H, tab, A, o, st);
            row<HOST4>("host4", r, n, h4, h8, H, tab, A, o, st);
            row<HOST8>("host8", r, n, h4, h8, H, tab, A, o, st);
        }
        row<TAB>("tab", r, n, h4, h8, H, tab, A, o, st);
        row<TABONLY>("tabonly", r, n, h4, h8, H, tab, A, o, st);
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
