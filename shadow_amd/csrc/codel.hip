// codel.hip -- destination routers on gfx950: router_enqueue + the CoDel
// queue manager (reference routing/router.c:103-131,
// routing/router_queue_codel.c:113-265).  The step right after the packet
// hand-off: each destination host's upstream router receives that host's
// delivered events in event_compare order and the receive side of its
// network interface dequeues them.  A router is a sequential state machine,
// so the parallelism is across routers: one lane per router, every router
// of a batch at once (100k-200k routers per round at C3/C4 scale).
//
// Arithmetic is the reference's, bit for bit: sojourn = now - enqueueTS in
// u64 ns, the control law round((ts + interval) / sqrt(count)) in f64 with
// correctly rounded division and square root (no fast math, no contraction),
// the u32 drop counters with their wrap-around.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cmath>

#include "codel_dev.h"
#include "shd_internal.h"

namespace {

struct Router {
    ShdCodelEntry* ring;
    uint32_t cap;
    uint64_t* fate;
    uint32_t op; // index of the operation being run (fate records)
    bool bad;    // a dequeue before an entry's enqueue time (utility_assert(now >= ts), :172)
    uint32_t head, len;

    __device__ __forceinline__ bool pop(ShdCodelEntry& e) {
        if (len == 0) return false;
        e = ring[head];
        head = head + 1 == cap ? 0 : head + 1;
        len--;
        return true;
    }
    // _routerqueuecodel_drop (:138-146): PDS_ROUTER_DROPPED
    __device__ __forceinline__ void drop(uint32_t pkt) { fate[pkt] = ((uint64_t)op << 2) | SHD_CODEL_DROPPED; }
};

__global__ __launch_bounds__(256) void k_codel(uint32_t nrouters, const uint32_t* __restrict__ op_off,
                                               const ShdCodelOp* __restrict__ ops, ShdCodelState* __restrict__ states,
                                               ShdCodelEntry* __restrict__ rings, uint32_t ring_cap,
                                               uint32_t* __restrict__ deq_out, uint64_t* __restrict__ fate,
                                               int* __restrict__ err) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrouters) return;
    ShdCodelState st = states[r];
    Router q{rings + (size_t)r * ring_cap, ring_cap, fate, 0, false, st.head, st.len};
    for (uint32_t i = op_off[r]; i < op_off[r + 1]; i++) {
        const ShdCodelOp o = ops[i];
        q.op = i;
        if (o.kind == 0) { // router_enqueue -> _routerqueuecodel_enqueue (:113-137)
            if (q.len == q.cap) {
                atomicOr(err, 1); // the caller's ring is too small (the reference queue is unbounded)
                break;
            }
            uint32_t tail = q.head + q.len;
            if (tail >= q.cap) tail -= q.cap;
            q.ring[tail] = ShdCodelEntry{o.time, o.pkt, o.length};
            q.len++;
            st.total_size += o.length;
            deq_out[i] = o.pkt; // PDS_ROUTER_ENQUEUED
        } else { // router_dequeue
            ShdCodelEntry e;
            const bool got = shd_codel::dequeue(q, st, o.time, e);
            deq_out[i] = got ? e.pkt : 0xffffffffu;
            if (got) fate[e.pkt] = ((uint64_t)i << 2) | SHD_CODEL_DEQUEUED; // PDS_ROUTER_DEQUEUED
            if (q.bad) {
                atomicOr(err, 2);
                break;
            }
        }
    }
    st.head = q.head;
    st.len = q.len;
    states[r] = st;
}

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

} // namespace

extern "C" int shd_codel_run(uint32_t nrouters, const uint32_t* d_op_offsets, const ShdCodelOp* d_ops,
                             ShdCodelState* d_states, ShdCodelEntry* d_rings, uint32_t ring_cap, uint32_t* d_deq_out,
                             uint64_t* d_fate, void* stream) {
    if (!nrouters) return 0;
    if (!ring_cap) return shd_fail(-EINVAL, "ring capacity 0");
    hipStream_t s = (hipStream_t)stream;
    int* d_err = nullptr;
    int rc = hip_status(hipMalloc((void**)&d_err, sizeof(int)), "hipMalloc codel");
    if (rc) return rc;
    int h_err = 0;
    if (!(rc = hip_status(hipMemsetAsync(d_err, 0, sizeof(int), s), "hipMemset codel"))) {
        hipLaunchKernelGGL(k_codel, dim3((nrouters + 255) / 256), dim3(256), 0, s, nrouters, d_op_offsets, d_ops,
                           d_states, d_rings, ring_cap, d_deq_out, d_fate, d_err);
        rc = hip_status(hipGetLastError(), "k_codel launch");
        if (!rc) rc = hip_status(hipMemcpyAsync(&h_err, d_err, sizeof(int), hipMemcpyDeviceToHost, s), "codel D2H");
        if (!rc) rc = hip_status(hipStreamSynchronize(s), "k_codel");
    }
    (void)hipFree(d_err);
    if (!rc && (h_err & 1)) rc = shd_fail(-ENOSPC, "a router queue outgrew its ring (capacity %u)", ring_cap);
    if (!rc && (h_err & 2)) rc = shd_fail(-EINVAL, "a router dequeued before an entry's enqueue time");
    return rc;
}
