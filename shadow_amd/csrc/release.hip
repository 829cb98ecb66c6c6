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
//
// The answer for row i depends only on which rows were touched BEFORE i, so
// it can be computed any time after i's touch against any later snapshot of
// the touch sequence: releases are queued by the host (topology.c) and
// launched asynchronously in batches on this scratch's own stream
// (shd_dev_release_launch), and their minima are collected in launch order
// at the next point that needs the running minimum (shd_dev_release_collect;
// the controller reads it only at the round boundary, controller.c:390-422).
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstring>
#include <new>

#include "shd_internal.h"

namespace {

constexpr int kRelBlock = 256;
constexpr int kRelLoads = 4;         // entries in flight per thread
constexpr int kRelChunk = 16384;     // columns per work item: 256 KiB of entries
constexpr unsigned kRelMaxGrid = 16384;

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

// Work item w = (row r, column chunk c) of the listed rows, grid-stride: a
// few rows spread over the whole chip as well as 86k rows.  Latencies are
// non-negative doubles, so their bit patterns order like the values and the
// reduction runs on u64 (~0 = nothing released; out[] starts at ~0).
__global__ __launch_bounds__(kRelBlock) void k_release_min(const ShdEntry* __restrict__ base, int A,
                                                           const int32_t* __restrict__ rows,
                                                           const uint32_t* __restrict__ seqs, int n, int nchunk,
                                                           const uint32_t* __restrict__ touch,
                                                           unsigned long long* __restrict__ out) {
    __shared__ unsigned long long wmin[kRelBlock / 64];
    const size_t items = (size_t)n * (size_t)nchunk;
    for (size_t w = blockIdx.x; w < items; w += gridDim.x) {
        const int r = (int)(w / (size_t)nchunk), c = (int)(w % (size_t)nchunk);
        const int i = rows[r];
        const uint32_t seq = seqs[r];
        const ShdEntry* __restrict__ row = base + (size_t)i * (size_t)A;
        const int jb = c * kRelChunk, je = jb + kRelChunk < A ? jb + kRelChunk : A;
        unsigned long long m = ~0ull;
        for (int j0 = jb + threadIdx.x; j0 < je; j0 += kRelBlock * kRelLoads) {
            double l[kRelLoads];
            uint32_t tj[kRelLoads];
#pragma unroll
            for (int k = 0; k < kRelLoads; k++) {
                const int j = j0 + k * kRelBlock;
                l[k] = j < je ? row[j].lat : -1.0;
                tj[k] = j < je ? touch[j] : 0u;
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
            for (int k = 1; k < kRelBlock / 64; k++) b = wmin[k] < b ? wmin[k] : b;
            if (b != ~0ull) atomicMin(&out[r], b);
        }
        __syncthreads();
    }
}

// Grow-only buffers and the stream of one release site (a table shard),
// owned by the host side and serialised by its lock.  Rows launched since the
// last collect ("the epoch") sit at increasing positions of the row / seq /
// result arrays, so every launch has its own pinned staging; the touch
// snapshot alternates between two pinned buffers, each reused only after the
// copy that read it has completed.
struct RelScratch {
    int device = -1;
    hipStream_t stream = nullptr;
    uint32_t* d_touch = nullptr;
    uint32_t* h_snap[2] = {nullptr, nullptr};
    hipEvent_t snap_ev[2] = {nullptr, nullptr};
    int snap_k = 0;
    size_t cap_a = 0;
    int32_t* d_rows = nullptr;
    uint32_t* d_seqs = nullptr;
    unsigned long long* d_out = nullptr;
    int32_t* h_rows = nullptr;
    uint32_t* h_seqs = nullptr;
    unsigned long long* h_out = nullptr;
    size_t cap_n = 0, n = 0;
};

void free_epoch(RelScratch* s) {
    (void)hipFree(s->d_rows);
    (void)hipFree(s->d_seqs);
    (void)hipFree(s->d_out);
    if (s->h_rows) (void)hipHostFree(s->h_rows);
    if (s->h_seqs) (void)hipHostFree(s->h_seqs);
    if (s->h_out) (void)hipHostFree(s->h_out);
    s->d_rows = nullptr;
    s->d_seqs = nullptr;
    s->d_out = nullptr;
    s->h_rows = nullptr;
    s->h_seqs = nullptr;
    s->h_out = nullptr;
    s->cap_n = 0;
}

void free_all(RelScratch* s) {
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    free_epoch(s);
    (void)hipFree(s->d_touch);
    for (int k = 0; k < 2; k++) {
        if (s->h_snap[k]) (void)hipHostFree(s->h_snap[k]);
        if (s->snap_ev[k]) (void)hipEventDestroy(s->snap_ev[k]);
        s->h_snap[k] = nullptr;
        s->snap_ev[k] = nullptr;
    }
    s->d_touch = nullptr;
    s->cap_a = 0;
    if (s->stream) (void)hipStreamDestroy(s->stream);
    s->stream = nullptr;
    s->n = 0;
}

// room for `need` epoch rows (waits for the launches in flight when it grows:
// their results move to the new pinned buffer)
int reserve_epoch(RelScratch* s, size_t need) {
    if (need <= s->cap_n) return 0;
    int rc = hip_status(hipStreamSynchronize(s->stream), "release stream sync");
    if (rc) return rc;
    const size_t cap = 2 * need + 1024;
    unsigned long long* keep = nullptr;
    if (s->n) {
        keep = new (std::nothrow) unsigned long long[s->n];
        if (!keep) return -ENOMEM;
        std::memcpy(keep, s->h_out, 8 * s->n);
    }
    free_epoch(s);
    if ((rc = hip_status(hipMalloc((void**)&s->d_rows, 4 * cap), "hipMalloc release rows")) ||
        (rc = hip_status(hipMalloc((void**)&s->d_seqs, 4 * cap), "hipMalloc release seqs")) ||
        (rc = hip_status(hipMalloc((void**)&s->d_out, 8 * cap), "hipMalloc release out")) ||
        (rc = hip_status(hipHostMalloc((void**)&s->h_rows, 4 * cap, hipHostMallocDefault), "hipHostMalloc rows")) ||
        (rc = hip_status(hipHostMalloc((void**)&s->h_seqs, 4 * cap, hipHostMallocDefault), "hipHostMalloc seqs")) ||
        (rc = hip_status(hipHostMalloc((void**)&s->h_out, 8 * cap, hipHostMallocDefault), "hipHostMalloc out"))) {
        free_epoch(s);
        delete[] keep;
        s->n = 0; // (the lost results surface as this error)
        return rc;
    }
    s->cap_n = cap;
    if (keep) std::memcpy(s->h_out, keep, 8 * s->n);
    delete[] keep;
    return 0;
}

int reserve_touch(RelScratch* s, int A) {
    if ((size_t)A <= s->cap_a) return 0;
    int rc = hip_status(hipStreamSynchronize(s->stream), "release stream sync");
    if (rc) return rc;
    (void)hipFree(s->d_touch);
    s->d_touch = nullptr;
    for (int k = 0; k < 2; k++) {
        if (s->h_snap[k]) (void)hipHostFree(s->h_snap[k]);
        s->h_snap[k] = nullptr;
    }
    s->cap_a = 0;
    if ((rc = hip_status(hipMalloc((void**)&s->d_touch, 4 * (size_t)A), "hipMalloc release touch")) ||
        (rc = hip_status(hipHostMalloc((void**)&s->h_snap[0], 4 * (size_t)A, hipHostMallocDefault), "hipHostMalloc snap")) ||
        (rc = hip_status(hipHostMalloc((void**)&s->h_snap[1], 4 * (size_t)A, hipHostMallocDefault), "hipHostMalloc snap")))
        return rc;
    s->cap_a = (size_t)A;
    return 0;
}

} // namespace

// Queues the releases of n rows (rows[r] absolute slot, touch sequence
// seqs[r]) on the scratch's stream against `touch` (host array of A touch
// sequences taken after every listed row drew its number); returns without
// waiting.  The calling thread's device is the shard's.
extern "C" int shd_dev_release_launch(const ShdEntry* base, int A, const int32_t* rows, const uint32_t* seqs, int n,
                                      const uint32_t* touch, void** scratch) {
    if (n <= 0) return 0;
    if (!base || A <= 0 || !rows || !seqs || !touch || !scratch) return shd_fail(-EINVAL, "release args");
    int dev = 0;
    int rc = hip_status(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    RelScratch* s = static_cast<RelScratch*>(*scratch);
    if (!s) {
        s = new (std::nothrow) RelScratch();
        if (!s) return -ENOMEM;
        *scratch = s;
    }
    if (s->device >= 0 && s->device != dev) return shd_fail(-EINVAL, "release scratch of device %d used on %d", s->device, dev);
    s->device = dev;
    if (!s->stream && (rc = hip_status(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking), "release stream")))
        return rc;
    for (int k = 0; k < 2; k++)
        if (!s->snap_ev[k] && (rc = hip_status(hipEventCreateWithFlags(&s->snap_ev[k], hipEventDisableTiming),
                                               "release event")))
            return rc;
    if ((rc = reserve_touch(s, A)) || (rc = reserve_epoch(s, s->n + (size_t)n))) return rc;
    const size_t at = s->n;
    std::memcpy(s->h_rows + at, rows, 4 * (size_t)n);
    std::memcpy(s->h_seqs + at, seqs, 4 * (size_t)n);
    const int k = s->snap_k ^= 1;
    if ((rc = hip_status(hipEventSynchronize(s->snap_ev[k]), "release snapshot reuse"))) return rc;
    std::memcpy(s->h_snap[k], touch, 4 * (size_t)A);
    hipStream_t st = s->stream;
    if ((rc = hip_status(hipMemcpyAsync(s->d_touch, s->h_snap[k], 4 * (size_t)A, hipMemcpyHostToDevice, st), "touch H2D")) ||
        (rc = hip_status(hipEventRecord(s->snap_ev[k], st), "release event record")) ||
        (rc = hip_status(hipMemcpyAsync(s->d_rows + at, s->h_rows + at, 4 * (size_t)n, hipMemcpyHostToDevice, st), "rows H2D")) ||
        (rc = hip_status(hipMemcpyAsync(s->d_seqs + at, s->h_seqs + at, 4 * (size_t)n, hipMemcpyHostToDevice, st), "seqs H2D")) ||
        (rc = hip_status(hipMemsetAsync(s->d_out + at, 0xff, 8 * (size_t)n, st), "release out init")))
        return rc;
    const int nchunk = (A + kRelChunk - 1) / kRelChunk;
    const size_t items = (size_t)n * (size_t)nchunk;
    hipLaunchKernelGGL(k_release_min, dim3((unsigned)(items < kRelMaxGrid ? items : kRelMaxGrid)), dim3(kRelBlock), 0,
                       st, base, A, s->d_rows + at, s->d_seqs + at, n, nchunk, s->d_touch, s->d_out + at);
    if ((rc = hip_status(hipGetLastError(), "k_release_min launch")) ||
        (rc = hip_status(hipMemcpyAsync(s->h_out + at, s->d_out + at, 8 * (size_t)n, hipMemcpyDeviceToHost, st),
                         "release min D2H")))
        return rc;
    s->n = at + (size_t)n;
    return 0;
}

// Waits for every launch since the last collect and returns their minima in
// launch order (out[r] = -1: nothing released); *n = how many (<= cap).
extern "C" int shd_dev_release_collect(void* scratch, double* out, size_t cap, size_t* n) {
    *n = 0;
    RelScratch* s = static_cast<RelScratch*>(scratch);
    if (!s || !s->n) return 0;
    if (s->n > cap) return shd_fail(-ENOSPC, "release results %zu > %zu", s->n, cap);
    int rc = hip_status(hipStreamSynchronize(s->stream), "release stream sync");
    if (!rc)
        for (size_t r = 0; r < s->n; r++) {
            if (s->h_out[r] == ~0ull) out[r] = -1.0;
            else std::memcpy(&out[r], &s->h_out[r], 8);
        }
    *n = rc ? 0 : s->n;
    s->n = 0;
    return rc;
}

// Rows launched and not yet collected.
extern "C" size_t shd_dev_release_pending(void* scratch) {
    const RelScratch* s = static_cast<const RelScratch*>(scratch);
    return s ? s->n : 0;
}

extern "C" void shd_dev_release_scratch_free(void* scratch) {
    if (!scratch) return;
    RelScratch* s = static_cast<RelScratch*>(scratch);
    int cur = -1;
    if (s->device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != s->device) (void)hipSetDevice(s->device);
    free_all(s);
    if (cur >= 0 && cur != s->device) (void)hipSetDevice(cur);
    delete s;
}
