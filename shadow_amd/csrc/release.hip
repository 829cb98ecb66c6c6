// release.hip -- lazy row release on device-resident routing tables.
//
// The reference computes and stores a source row the first time a lookup
// misses it (topology.c:1900-1981 -> _topology_computeSourcePaths), and
// _topology_storePathInCache (:1217-1265) stores (s, y) only when neither
// (s, y) nor (y, s) is cached yet; every store may lower the running minimum
// that feeds worker_updateMinTimeJump (:1253-1264, controller.c:141-153).
// Here every row is already computed in HBM, so a first touch of row i only
// has to find what the serial store loop would have released: the columns y
// whose row was not touched before i (touch[y] > seq_i; untouched rows hold
// UINT32_MAX), y != i (a row never stores its own vertex, :1744-1752).  The
// minimum over those entries is one streaming pass over the row's 16-B
// entries: HBM-bound, A x 16 B read per released row (C4: 1.4 MB).
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstring>
#include <new>

#include "shd_internal.h"

namespace {

constexpr int kRelBlock = 256;
constexpr int kRelLoads = 4; // entries in flight per thread

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

// One workgroup per listed row (grid-stride over the list).  Latencies are
// non-negative doubles, so their bit patterns order like the values and the
// reduction runs on u64 (~0 = nothing released).
__global__ __launch_bounds__(kRelBlock) void k_release_min(const ShdEntry* __restrict__ base, int A,
                                                           const int32_t* __restrict__ rows,
                                                           const uint32_t* __restrict__ seqs, int n,
                                                           const uint32_t* __restrict__ touch,
                                                           unsigned long long* __restrict__ out) {
    __shared__ unsigned long long wmin[kRelBlock / 64];
    for (int r = blockIdx.x; r < n; r += gridDim.x) {
        const int i = rows[r];
        const uint32_t seq = seqs[r];
        const ShdEntry* __restrict__ row = base + (size_t)i * (size_t)A;
        unsigned long long m = ~0ull;
        for (int j0 = threadIdx.x; j0 < A; j0 += kRelBlock * kRelLoads) {
            double l[kRelLoads];
            uint32_t tj[kRelLoads];
#pragma unroll
            for (int k = 0; k < kRelLoads; k++) {
                const int j = j0 + k * kRelBlock;
                l[k] = j < A ? row[j].lat : -1.0;
                tj[k] = j < A ? touch[j] : 0u;
            }
#pragma unroll
            for (int k = 0; k < kRelLoads; k++) {
                const int j = j0 + k * kRelBlock;
                if (j != i && tj[k] > seq && l[k] >= 0.0) {
                    const unsigned long long b = (unsigned long long)__double_as_longlong(l[k]);
                    m = b < m ? b : m;
                }
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(m, off);
            m = o < m ? o : m;
        }
        if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long b = wmin[0];
            for (int w = 1; w < kRelBlock / 64; w++) b = wmin[w] < b ? wmin[w] : b;
            out[r] = b;
        }
        __syncthreads();
    }
}

// Grow-only device buffers of one release site (a table shard), owned by the
// host side and serialised by its lock.
struct RelScratch {
    int device = -1;
    uint32_t* touch = nullptr;
    size_t cap_a = 0;
    int32_t* rows = nullptr;
    uint32_t* seqs = nullptr;
    unsigned long long* out = nullptr;
    size_t cap_n = 0;
};

void scratch_release_buffers(RelScratch* s) {
    (void)hipFree(s->touch);
    (void)hipFree(s->rows);
    (void)hipFree(s->seqs);
    (void)hipFree(s->out);
    s->touch = nullptr;
    s->rows = nullptr;
    s->seqs = nullptr;
    s->out = nullptr;
    s->cap_a = s->cap_n = 0;
}

} // namespace

extern "C" int shd_dev_release_min(const ShdEntry* base, int A, const int32_t* rows, const uint32_t* seqs, int n,
                                   const uint32_t* touch, double* out, void** scratch) {
    if (n <= 0) return 0;
    if (!base || A <= 0 || !rows || !seqs || !touch || !out || !scratch) return shd_fail(-EINVAL, "release args");
    int dev = 0;
    int rc = hip_status(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    RelScratch* s = static_cast<RelScratch*>(*scratch);
    if (!s) {
        s = new (std::nothrow) RelScratch();
        if (!s) return -ENOMEM;
        *scratch = s;
    }
    if (s->device >= 0 && s->device != dev) scratch_release_buffers(s); // (only freed on its own device below)
    s->device = dev;
    if ((size_t)A > s->cap_a) {
        (void)hipFree(s->touch);
        s->touch = nullptr;
        s->cap_a = 0;
        if ((rc = hip_status(hipMalloc((void**)&s->touch, 4 * (size_t)A), "hipMalloc release touch"))) return rc;
        s->cap_a = (size_t)A;
    }
    if ((size_t)n > s->cap_n) {
        (void)hipFree(s->rows);
        (void)hipFree(s->seqs);
        (void)hipFree(s->out);
        s->rows = nullptr;
        s->seqs = nullptr;
        s->out = nullptr;
        s->cap_n = 0;
        const size_t cap = (size_t)n + (size_t)n / 2 + 64;
        if ((rc = hip_status(hipMalloc((void**)&s->rows, 4 * cap), "hipMalloc release rows")) ||
            (rc = hip_status(hipMalloc((void**)&s->seqs, 4 * cap), "hipMalloc release seqs")) ||
            (rc = hip_status(hipMalloc((void**)&s->out, 8 * cap), "hipMalloc release out")))
            return rc;
        s->cap_n = cap;
    }
    if ((rc = hip_status(hipMemcpy(s->touch, touch, 4 * (size_t)A, hipMemcpyHostToDevice), "release touch H2D")) ||
        (rc = hip_status(hipMemcpy(s->rows, rows, 4 * (size_t)n, hipMemcpyHostToDevice), "release rows H2D")) ||
        (rc = hip_status(hipMemcpy(s->seqs, seqs, 4 * (size_t)n, hipMemcpyHostToDevice), "release seqs H2D")))
        return rc;
    const int grid = n < 8192 ? n : 8192;
    hipLaunchKernelGGL(k_release_min, dim3(grid), dim3(kRelBlock), 0, nullptr, base, A, s->rows, s->seqs, n, s->touch,
                       s->out);
    if ((rc = hip_status(hipGetLastError(), "k_release_min launch"))) return rc;
    unsigned long long* h = new (std::nothrow) unsigned long long[(size_t)n];
    if (!h) return -ENOMEM;
    rc = hip_status(hipMemcpy(h, s->out, 8 * (size_t)n, hipMemcpyDeviceToHost), "release min D2H");
    if (!rc)
        for (int r = 0; r < n; r++) {
            if (h[r] == ~0ull) out[r] = -1.0;
            else std::memcpy(&out[r], &h[r], 8);
        }
    delete[] h;
    return rc;
}

extern "C" void shd_dev_release_scratch_free(void* scratch) {
    if (!scratch) return;
    RelScratch* s = static_cast<RelScratch*>(scratch);
    int cur = -1;
    if (s->device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != s->device) (void)hipSetDevice(s->device);
    scratch_release_buffers(s);
    if (cur >= 0 && cur != s->device) (void)hipSetDevice(cur);
    delete s;
}
