// ubench_tlb.hip -- is the packet table gather bound by address translation?
// (dev tool).  10M random 16-B gathers, the packet-scatter kernel's table
// access without its logic, over (a) windows of growing footprint inside one
// large allocation and (b) several separate allocations of the C3 table size
// in one process, and (c) the C3 footprint with the gathers sorted by
// address (same lines, translation locality).  Prints median ms of 9 launches.
// Every index is taken modulo the window; nothing is read out of bounds.
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

constexpr int kB = 4;

// idx[i] = a random 64-bit value; the entry read is idx % nent
__global__ __launch_bounds__(256) void k_gather(const unsigned long long* __restrict__ idx, size_t n,
                                                const double2* __restrict__ tab, unsigned long long nent,
                                                double* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * kB) {
        unsigned long long j[kB];
#pragma unroll
        for (int b = 0; b < kB; b++) {
            const size_t i = i0 + b * stride;
            j[b] = i < n ? idx[i] % nent : 0;
        }
        double2 e[kB];
#pragma unroll
        for (int b = 0; b < kB; b++) e[b] = tab[j[b]];
#pragma unroll
        for (int b = 0; b < kB; b++) {
            const size_t i = i0 + b * stride;
            if (i < n) out[i] = e[b].x + e[b].y;
        }
    }
}

static float run(const unsigned long long* idx, size_t n, const double2* tab, unsigned long long nent, double* out) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 10; rep++) {
        CHECK(hipEventRecord(a));
        k_gather<<<4096, 256>>>(idx, n, tab, nent, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t n = 10'000'000;
    const unsigned long long c3 = 19870ull * 19870ull; // C3 table entries (6.3 GB)
    std::vector<unsigned long long> h(n);
    unsigned long long s = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < n; i++) {
        s += 0x9E3779B97F4A7C15ull;
        unsigned long long z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        h[i] = z ^ (z >> 31);
    }
    unsigned long long* d_idx;
    double* d_out;
    CHECK(hipMalloc(&d_idx, n * 8));
    CHECK(hipMalloc(&d_out, n * 8));
    CHECK(hipMemcpy(d_idx, h.data(), n * 8, hipMemcpyHostToDevice));

    // (a) footprint sweep inside one 25 GB allocation
    const unsigned long long big = 4 * c3;
    double2* tab;
    CHECK(hipMalloc(&tab, big * 16));
    CHECK(hipMemset(tab, 0, big * 16));
    for (unsigned long long mb : {64ull, 256ull, 512ull, 1024ull, 2048ull, 4096ull, 6316ull, 12632ull, 25264ull}) {
        const unsigned long long ne = std::min(big, mb * 1024 * 1024 / 16);
        printf("footprint %6llu MB: %.3f ms\n", mb, run(d_idx, n, tab, ne, d_out));
        fflush(stdout);
    }
    // (c) sorted indices at the C3 footprint (same lines, in address order)
    std::vector<unsigned long long> hs(n);
    for (size_t i = 0; i < n; i++) hs[i] = h[i] % c3;
    std::sort(hs.begin(), hs.end());
    unsigned long long* d_sorted;
    CHECK(hipMalloc(&d_sorted, n * 8));
    CHECK(hipMemcpy(d_sorted, hs.data(), n * 8, hipMemcpyHostToDevice));
    printf("C3 footprint, indices sorted: %.3f ms\n", run(d_sorted, n, tab, c3, d_out));
    // rows of 256 consecutive records share one 1/256th of the table
    for (size_t i = 0; i < n; i++) hs[i] = (h[i] % c3);
    std::sort(hs.begin(), hs.end(), [](unsigned long long x, unsigned long long y) { return (x >> 22) < (y >> 22); });
    CHECK(hipMemcpy(d_sorted, hs.data(), n * 8, hipMemcpyHostToDevice));
    printf("C3 footprint, grouped by 64 MB region: %.3f ms\n", run(d_sorted, n, tab, c3, d_out));
    CHECK(hipFree(tab));

    // (b) separate allocations of the C3 size
    std::vector<double2*> tabs(4);
    for (auto& t : tabs) {
        CHECK(hipMalloc(&t, c3 * 16));
        CHECK(hipMemset(t, 0, c3 * 16));
    }
    for (int r = 0; r < 2; r++)
        for (size_t k = 0; k < tabs.size(); k++)
            printf("allocation %zu (pass %d): %.3f ms\n", k, r, run(d_idx, n, tabs[k], c3, d_out));
    for (auto t : tabs) CHECK(hipFree(t));
    // (d) physically contiguous allocations of the C3 size
    for (auto& t : tabs) {
        if (hipExtMallocWithFlags((void**)&t, c3 * 16, hipDeviceMallocContiguous) != hipSuccess) {
            printf("contiguous allocation refused: %s\n", hipGetErrorString(hipGetLastError()));
            t = nullptr;
            continue;
        }
        CHECK(hipMemset(t, 0, c3 * 16));
    }
    for (int r = 0; r < 2; r++)
        for (size_t k = 0; k < tabs.size(); k++)
            if (tabs[k]) printf("contiguous allocation %zu (pass %d): %.3f ms\n", k, r, run(d_idx, n, tabs[k], c3, d_out));
    for (auto t : tabs)
        if (t) CHECK(hipFree(t));
    CHECK(hipFree(d_idx));
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_sorted));
    return 0;
}
