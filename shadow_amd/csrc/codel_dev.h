// codel_dev.h -- the CoDel queue manager as device code, shared by the
// router engine (codel.hip) and the interface engine (nic.hip).  A
// restatement of routing/router_queue_codel.c:148-267 over any queue type Q
// providing
//   bool pop(ShdCodelEntry& e)   -- g_queue_pop_head
//   void drop(uint32_t pkt)      -- _routerqueuecodel_drop (:138-146)
//   bool bad                     -- set when an assertion of the reference fails
// Arithmetic is the reference's bit for bit: u64 ns sojourn, the control law
// round((ts + interval) / sqrt(count)) in f64 with correctly rounded division
// and square root (built with -fno-fast-math -ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>

#include "shdnet.h"

namespace shd_codel {

constexpr uint64_t kTarget = 10ull * 1000000ull;    // CODEL_PARAM_TARGET_DELAY_SIMTIME (:42)
constexpr uint64_t kInterval = 100ull * 1000000ull; // CODEL_PARAM_INTERVAL_SIMTIME (:48)
constexpr uint64_t kMtu = 1500;                     // CONFIG_MTU (definitions.h:185)

// _routerqueuecodel_dequeueHelper (:148-196); the popped entry or pkt = -1
template <class Q>
__device__ __forceinline__ bool helper(Q& q, ShdCodelState& s, uint64_t now, bool* ok, ShdCodelEntry& e) {
    *ok = false;
    if (!q.pop(e)) {
        s.interval_expire = 0; // empty: cannot be above target
        return false;
    }
    if (e.length > s.total_size) q.bad = true; // utility_assert(length <= totalSize)
    s.total_size -= e.length;
    if (now < e.enqueue_ts) q.bad = true;      // utility_assert(now >= ts)
    const uint64_t sojourn = now - e.enqueue_ts;
    if (sojourn < kTarget || s.total_size < kMtu) {
        s.interval_expire = 0;
    } else if (s.interval_expire == 0) {
        s.interval_expire = now + kInterval;
    } else if (now >= s.interval_expire) {
        *ok = true;
    }
    return true;
}

// _routerqueuecodel_controlLaw (:198-205), as written (not RFC 8289's
// ts + interval / sqrt(count))
__device__ __forceinline__ uint64_t control_law(uint32_t count, uint64_t ts) {
    const uint64_t new_ts = ts + kInterval;
    const double result = (double)new_ts / sqrt((double)count);
    return (uint64_t)round(result);
}

// _routerqueuecodel_dequeue (:207-267): true and the entry handed to the
// interface, or false (queue empty after the drops)
template <class Q>
__device__ bool dequeue(Q& q, ShdCodelState& s, uint64_t now, ShdCodelEntry& e) {
    bool ok = false;
    bool have = helper(q, s, now, &ok, e);
    if (!have) {
        s.mode = 0; // empty queue: leave dropping state
        return false;
    }
    if (s.mode == 1) {
        if (!ok) s.mode = 0; // delays low again
        while (now >= s.next_drop && s.mode == 1) {
            q.drop(e.pkt);
            s.drop_count++;
            have = helper(q, s, now, &ok, e);
            if (ok) s.next_drop = control_law(s.drop_count, s.next_drop);
            else s.mode = 0;
        }
    } else if (ok) {
        q.drop(e.pkt);
        have = helper(q, s, now, &ok, e);
        s.mode = 1;
        const uint32_t delta = s.drop_count - s.drop_count_last;
        s.drop_count = 1;
        const bool recently = now < s.next_drop + 16 * kInterval;
        if (recently && delta > 1) s.drop_count = delta;
        s.next_drop = control_law(s.drop_count, now);
        s.drop_count_last = s.drop_count;
    }
    return have;
}

} // namespace shd_codel
