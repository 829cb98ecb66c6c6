// dev.hip -- device runtime helpers behind the C ABI (HIP runtime calls
// only; kernels live in routing.hip and packet.hip).  gfx950 only: the
// library refuses to run on anything else rather than silently degrading.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstring>

#include "shd_internal.h"

static int hip_err(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

// Selects `device` for the calling thread (HIP's current device is per
// thread: lookups may come from any worker); the device count and the gfx950
// check run once per thread and device.
extern "C" int shd_dev_init(int device) {
    static thread_local int checked = -1;
    if (checked != device) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return shd_fail(-ENODEV, "no HIP device visible");
        if (device < 0 || device >= n) return shd_fail(-ENODEV, "device %d out of range (%d visible)", device, n);
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, device) != hipSuccess) return shd_fail(-ENODEV, "device query failed");
        if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
            return shd_fail(-ENODEV, "device %d is %s, libshdnet is built for gfx950 only", device, p.gcnArchName);
        checked = device;
    }
    return hip_err(hipSetDevice(device), "hipSetDevice");
}

extern "C" int shd_dev_mem_info(size_t* free_bytes, size_t* total_bytes) {
    return hip_err(hipMemGetInfo(free_bytes, total_bytes), "hipMemGetInfo");
}

extern "C" int shd_dev_malloc(void** p, size_t bytes) {
    *p = nullptr;
    return hip_err(hipMalloc(p, bytes ? bytes : 4), "hipMalloc");
}

// Tables: an ordinary device allocation.  (Physically contiguous memory,
// hipDeviceMallocContiguous, was measured: 10M random 16-B gathers over
// 6.3 GB took 0.251-0.255 ms on it vs 0.253-0.272 ms depending on the
// hipMalloc'd allocation, but the write-heavy users were slower -- the C4
// table build 10.3 vs 9.0-9.2 s, per-wave routing slabs and packet slabs far
// more)
extern "C" int shd_dev_malloc_table(void** p, size_t bytes, int* contig) {
    if (contig) *contig = 0;
    return shd_dev_malloc(p, bytes);
}

extern "C" int shd_dev_free(void* p) { return p ? hip_err(hipFree(p), "hipFree") : 0; }

extern "C" int shd_dev_h2d(void* d, const void* h, size_t bytes) {
    return bytes ? hip_err(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice), "hipMemcpy H2D") : 0;
}

extern "C" int shd_dev_d2h(void* h, const void* d, size_t bytes) {
    return bytes ? hip_err(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost), "hipMemcpy D2H") : 0;
}

extern "C" int shd_dev_d2d(void* d, const void* s, size_t bytes) {
    return bytes ? hip_err(hipMemcpy(d, s, bytes, hipMemcpyDeviceToDevice), "hipMemcpy D2D") : 0;
}

extern "C" int shd_dev_h2d_async(void* d, const void* h, size_t bytes, void* s) {
    return bytes ? hip_err(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, (hipStream_t)s), "hipMemcpyAsync H2D") : 0;
}

extern "C" int shd_dev_d2h_async(void* h, const void* d, size_t bytes, void* s) {
    return bytes ? hip_err(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, (hipStream_t)s), "hipMemcpyAsync D2H") : 0;
}

extern "C" int shd_dev_d2d_async(void* d, const void* src, size_t bytes, void* s) {
    return bytes ? hip_err(hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)s), "hipMemcpyAsync D2D")
                 : 0;
}

// events that order one stream after another (no timing)
extern "C" int shd_dev_event_new(void** e) {
    hipEvent_t h = nullptr;
    const int rc = hip_err(hipEventCreateWithFlags(&h, hipEventDisableTiming), "hipEventCreate");
    *e = rc ? nullptr : (void*)h;
    return rc;
}
extern "C" void shd_dev_event_free(void* e) {
    if (e) (void)hipEventDestroy((hipEvent_t)e);
}
// `waiter` waits (on the device) for what `after` has enqueued so far
extern "C" int shd_dev_stream_after(void* waiter, void* after, void* e) {
    int rc = hip_err(hipEventRecord((hipEvent_t)e, (hipStream_t)after), "hipEventRecord");
    return rc ? rc : hip_err(hipStreamWaitEvent((hipStream_t)waiter, (hipEvent_t)e, 0), "hipStreamWaitEvent");
}

// Pinned (page-locked) host memory: the round's staging buffers, so their
// copies run at the link's rate and asynchronously on the round's stream.
extern "C" int shd_host_alloc(void** p, size_t bytes) {
    *p = nullptr;
    return hip_err(hipHostMalloc(p, bytes ? bytes : 4, hipHostMallocDefault), "hipHostMalloc");
}

extern "C" void shd_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

extern "C" int shd_dev_memset(void* d, int v, size_t bytes) {
    return bytes ? hip_err(hipMemset(d, v, bytes), "hipMemset") : 0;
}

extern "C" int shd_dev_sync(void) { return hip_err(hipDeviceSynchronize(), "hipDeviceSynchronize"); }

extern "C" int shd_dev_stream_new(void** s) {
    hipStream_t h = nullptr;
    const int rc = hip_err(hipStreamCreate(&h), "hipStreamCreate");
    *s = rc ? nullptr : (void*)h;
    return rc;
}

extern "C" int shd_dev_stream_sync(void* s) { return hip_err(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize"); }

extern "C" void shd_dev_stream_free(void* s) {
    if (s) (void)hipStreamDestroy((hipStream_t)s);
}
