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

#include "shd_internal.h"

namespace {

constexpr uint64_t kTarget = 10ull * 1000000ull;    // CODEL_PARAM_TARGET_DELAY_SIMTIME (:38)
constexpr uint64_t kInterval = 100ull * 1000000ull; // CODEL_PARAM_INTERVAL_SIMTIME (:45)
constexpr uint64_t kMtu = 1500;                     // CONFIG_MTU (definitions.h:185)

struct Router {
    ShdCodelState s;
    ShdCodelEntry* ring;
    uint32_t cap;
    uint64_t* fate;
    uint32_t op; // index of the operation being run (fate records)
    bool bad;    // a dequeue ran at a time before an entry's enqueue (utility_assert(now >= ts), :172)
};

__device__ __forceinline__ bool pop_head(Router& q, ShdCodelEntry& e) {
    if (q.s.len == 0) return false;
    e = q.ring[q.s.head];
    q.s.head = q.s.head + 1 == q.cap ? 0 : q.s.head + 1;
    q.s.len--;
    return true;
}

// _routerqueuecodel_drop (:139-147): PDS_ROUTER_DROPPED
__device__ __forceinline__ void drop(Router& q, uint32_t pkt) {
    q.fate[pkt] = ((uint64_t)q.op << 2) | SHD_CODEL_DROPPED;
}

// _routerqueuecodel_dequeueHelper (:149-196); returns the packet or -1
__device__ int64_t dequeue_helper(Router& q, uint64_t now, bool* ok_to_drop) {
    *ok_to_drop = false;
    ShdCodelEntry e;
    if (!pop_head(q, e)) {
        q.s.interval_expire = 0; // empty: cannot be above target
        return -1;
    }
    q.s.total_size -= e.length;
    if (now < e.enqueue_ts) q.bad = true;
    const uint64_t sojourn = now - e.enqueue_ts;
    if (sojourn < kTarget || q.s.total_size < kMtu) {
        q.s.interval_expire = 0;
    } else if (q.s.interval_expire == 0) {
        q.s.interval_expire = now + kInterval;
    } else if (now >= q.s.interval_expire) {
        *ok_to_drop = true;
    }
    return e.pkt;
}

// _routerqueuecodel_controlLaw (:198-204), as written (not RFC 8289's
// ts + interval / sqrt(count))
__device__ __forceinline__ uint64_t control_law(uint32_t count, uint64_t ts) {
    const uint64_t new_ts = ts + kInterval;
    const double result = (double)new_ts / sqrt((double)count);
    return (uint64_t)round(result);
}

// _routerqueuecodel_dequeue (:206-265)
__device__ int64_t dequeue(Router& q, uint64_t now) {
    bool ok = false;
    int64_t pkt = dequeue_helper(q, now, &ok);
    if (pkt < 0) {
        q.s.mode = 0; // empty queue: leave dropping state
        return pkt;
    }
    if (q.s.mode == 1) {
        if (!ok) q.s.mode = 0; // delays low again
        while (now >= q.s.next_drop && q.s.mode == 1) {
            drop(q, (uint32_t)pkt);
            q.s.drop_count++;
            pkt = dequeue_helper(q, now, &ok);
            if (ok) q.s.next_drop = control_law(q.s.drop_count, q.s.next_drop);
            else q.s.mode = 0;
        }
    } else if (ok) {
        drop(q, (uint32_t)pkt);
        pkt = dequeue_helper(q, now, &ok);
        q.s.mode = 1;
        const uint32_t delta = q.s.drop_count - q.s.drop_count_last;
        q.s.drop_count = 1;
        const bool recently = now < q.s.next_drop + 16 * kInterval;
        if (recently && delta > 1) q.s.drop_count = delta;
        q.s.next_drop = control_law(q.s.drop_count, now);
        q.s.drop_count_last = q.s.drop_count;
    }
    return pkt;
}

__global__ __launch_bounds__(256) void k_codel(uint32_t nrouters, const uint32_t* __restrict__ op_off,
                                               const ShdCodelOp* __restrict__ ops, ShdCodelState* __restrict__ states,
                                               ShdCodelEntry* __restrict__ rings, uint32_t ring_cap,
                                               uint32_t* __restrict__ deq_out, uint64_t* __restrict__ fate,
                                               int* __restrict__ err) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrouters) return;
    Router q{states[r], rings + (size_t)r * ring_cap, ring_cap, fate, 0, false};
    for (uint32_t i = op_off[r]; i < op_off[r + 1]; i++) {
        const ShdCodelOp o = ops[i];
        q.op = i;
        if (o.kind == 0) { // router_enqueue -> _routerqueuecodel_enqueue (:113-137)
            if (q.s.len == q.cap) {
                atomicOr(err, 1); // the caller's ring is too small (the reference queue is unbounded)
                break;
            }
            uint32_t tail = q.s.head + q.s.len;
            if (tail >= q.cap) tail -= q.cap;
            q.ring[tail] = ShdCodelEntry{o.time, o.pkt, o.length};
            q.s.len++;
            q.s.total_size += o.length;
            deq_out[i] = o.pkt; // PDS_ROUTER_ENQUEUED
        } else { // router_dequeue
            const int64_t p = dequeue(q, o.time);
            deq_out[i] = p < 0 ? 0xffffffffu : (uint32_t)p;
            if (p >= 0) fate[p] = ((uint64_t)i << 2) | SHD_CODEL_DEQUEUED; // PDS_ROUTER_DEQUEUED
            if (q.bad) {
                atomicOr(err, 2);
                break;
            }
        }
    }
    states[r] = q.s;
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
