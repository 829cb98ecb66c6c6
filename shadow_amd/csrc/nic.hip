// nic.hip -- the hosts' network interfaces on gfx950:
// the upstream router with CoDel (routing/router.c:103-131,
// router_queue_codel.c:113-267) feeding the receive token bucket, and the
// send token bucket shaping the sender side (host/network_interface.c:
// 99-194 buckets and refills, :448-482 receivePackets, :571-631 sendPackets,
// :633-661 wantsSend).  One lane per host, every host of a window at once.
//
// A host's interface is a sequential state machine driven by three event
// streams, merged here in the order the host's event queue would run them
// (event_compare, core/work/event.c:109-152: time, then source host, then
// the source's event id):
//   - arrivals: the host's delivered events from the hand-off, already in
//     event_compare order (shd_round_process_device / shd_deliv_sort_device
//     segments, read in place) -> router_enqueue, and receivePackets when
//     the router queue was empty;
//   - send requests: packets the host's sockets offer to the interface, in
//     qdisc order, each with the time it was offered (wantsSend) ->
//     sendPackets;
//   - refill tasks (every 1 ms on the grid started at
//     networkinterface_startRefillingTokenBuckets, scheduled only while a
//     bucket is below capacity) -> refill both buckets, receivePackets,
//     sendPackets.
// Refill tasks and send requests are the host's own events (source = the
// host); arrivals come from other hosts, so at equal times the source host
// id decides.  Between a refill and a send request at the same nanosecond
// the source event ids decide in the reference; they are not in the inputs,
// and the send request goes first (documented assumption).
//
// Router queue layout: the entries a window leaves queued are kept in a
// per-host ring (ShdCodelEntry); the window's own arrivals are queued in
// place -- the FIFO tail is always a contiguous run of the host's arrival
// segment -- so no entry is copied unless it outlives the window.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "codel_dev.h"
#include "shd_internal.h"

namespace {

constexpr uint64_t kRefillInterval = 1000000ull; // _networkinterface_getRefillInterval (:99-101): 1 ms
constexpr uint64_t kMtu = shd_codel::kMtu;
constexpr uint64_t kNever = ~0ull;

enum { kErrRing = 1, kErrOrder = 2, kErrHost = 4, kErrId = 8, kErrWindow = 16, kErrAssert = 32, kErrArgs = 64 };

// A lane's packet fates (receive time, status) go out in runs: the ids a
// router pops are consecutive (FIFO over the carried run, then over the
// window's arrival segment), so up to kStage of them are staged in LDS and
// stored back to back, where one store per pop left each 128-B line to be
// written back from L2 many times over.  A dropped packet's time is written
// as ~0, the value its slot already holds (shd_nic_run's memset / the
// window that queued it).
constexpr uint32_t kStage = 16;
struct FateStage {
    uint64_t* rtime;
    uint8_t* rstat;
    uint64_t* lt; // this lane's column of the wave's [kStage][64] LDS arrays
    uint8_t* ls;
    uint32_t id0, n;
    __device__ __forceinline__ void flush() {
        for (uint32_t k = 0; k < n; k++) {
            rtime[id0 + k] = lt[64 * k];
            rstat[id0 + k] = ls[64 * k];
        }
        n = 0;
    }
    __device__ __forceinline__ void put(uint32_t id, uint64_t t, uint8_t st) {
        if (n && id != id0 + n) flush();
        if (!n) id0 = id;
        lt[64 * n] = t;
        ls[64 * n] = st;
        if (++n == kStage) flush();
    }
};

struct RouterQ {
    // carried entries (ring) first, then the window's arrivals [qhead, qtail)
    ShdCodelEntry* ring;
    uint32_t cap, head, len;
    const ShdDeliv* ev;
    const uint32_t* evlen;
    uint32_t qhead, qtail, id_base;
    FateStage* out;
    bool bad;
    uint32_t cidx;   // arrival index whose time / length are cached (~0: none)
    uint64_t ctime;
    uint32_t clen;

    __device__ __forceinline__ bool empty() const { return len == 0 && qhead == qtail; }
    __device__ __forceinline__ bool pop(ShdCodelEntry& e) {
        if (len) {
            e = ring[head];
            head = head + 1 == cap ? 0 : head + 1;
            len--;
            return true;
        }
        if (qhead == qtail) return false;
        // (the arrival just enqueued is usually the one popped: no re-read)
        e = qhead == cidx ? ShdCodelEntry{ctime, id_base + qhead, clen}
                          : ShdCodelEntry{ev[qhead].time, id_base + qhead, evlen[qhead]};
        qhead++;
        return true;
    }
    __device__ __forceinline__ void drop(uint32_t id) { // PDS_ROUTER_DROPPED
        out->put(id, ~0ull, SHD_NIC_DROPPED);
    }
};

// _networkinterface_consumeTokenBucket (:117-125)
__device__ __forceinline__ void consume(uint64_t& remaining, uint64_t bytes) {
    remaining = bytes >= remaining ? 0 : remaining - bytes;
}

// _networkinterface_scheduleNextRefillIfNeeded (:151-164)
__device__ __forceinline__ void schedule_if_needed(ShdNicState& s, uint64_t now) {
    const bool need = s.send_remaining < s.send_capacity || s.recv_remaining < s.recv_capacity;
    if (need && !s.refill_pending) {
        const uint64_t since = (now - s.refill_start) % kRefillInterval;
        s.refill_time = now + (kRefillInterval - since);
        s.refill_pending = 1;
    }
}

struct Host {
    ShdNicState s;
    RouterQ q;
    const ShdNicSend* sends;
    uint32_t sq, sk; // send queue: offered but not sent [sq, sk)
    uint64_t* stime;
    uint64_t boot_end;

    // networkinterface_receivePackets (:448-482)
    __device__ void receive(uint64_t now) {
        const bool boot = now < boot_end;
        while (boot || s.recv_remaining >= kMtu) {
            ShdCodelEntry e;
            if (!shd_codel::dequeue(q, s.router, now, e)) break; // router_dequeue (router.c:123-131)
            q.out->put(e.pkt, now, SHD_NIC_RECEIVED);
            if (!boot) {
                consume(s.recv_remaining, e.length);
                schedule_if_needed(s, now);
            }
        }
    }
    // _networkinterface_sendPackets (:571-631); no bootstrap term in the loop
    // condition, but no consumption while bootstrapping
    __device__ void send(uint64_t now) {
        const bool boot = now < boot_end;
        while (s.send_remaining >= kMtu && sq < sk) {
            const ShdNicSend p = sends[sq];
            stime[sq] = now;
            sq++;
            if (!boot) {
                consume(s.send_remaining, p.length);
                schedule_if_needed(s, now);
            }
        }
    }
    // _networkinterface_refillTokenBucketsCB (:166-186)
    __device__ void refill_tokens() {
        s.refill_pending = 0;
        s.recv_remaining += s.recv_refill; // _networkinterface_refillTokenBucket (:108-115)
        if (s.recv_remaining > s.recv_capacity) s.recv_remaining = s.recv_capacity;
        s.send_remaining += s.send_refill;
        if (s.send_remaining > s.send_capacity) s.send_remaining = s.send_capacity;
    }
    __device__ void refill(uint64_t now) {
        refill_tokens();
        receive(now);
        send(now);
        schedule_if_needed(s, now);
    }
};

__global__ __launch_bounds__(256) void k_nic_init(uint32_t n, const uint64_t* __restrict__ down,
                                                  const uint64_t* __restrict__ up, uint64_t start,
                                                  ShdNicState* __restrict__ st) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n) return;
    // _networkinterface_setupTokenBuckets (:196-228): capacity = refill + MTU
    const uint64_t factor = 1000000000ull / kRefillInterval;
    ShdNicState s{};
    s.recv_refill = down[h] * 1024 / factor;
    s.send_refill = up[h] * 1024 / factor;
    s.recv_capacity = s.recv_refill + kMtu;
    s.send_capacity = s.send_refill + kMtu;
    // networkinterface_startRefillingTokenBuckets (:188-194): the first
    // refill runs at once on empty buckets
    s.refill_start = start;
    s.refill_pending = 0;
    s.recv_remaining = s.recv_refill;
    s.send_remaining = s.send_refill;
    schedule_if_needed(s, start);
    st[h] = s;
}

// kMerged: the three event kinds share one call site each for receive, send
// and the refill scheduling (a lane's calls and their order are unchanged:
// arrival -> receive if the router queue was empty; send request -> send;
// refill -> receive, send, schedule), so a wave whose lanes took different
// kinds runs the CoDel dequeue and the send loop once per event, not once
// per kind: window 0.567 vs 0.654 ms on the C3 round output, identical
// fates and states (profiles/r03nicm_merged.log; SHD_NIC_MERGED=0 keeps the
// per-kind calls).
template <bool kMerged>
__global__ __launch_bounds__(64) void k_nic_run(uint32_t n, uint32_t host_base, const ShdDeliv* __restrict__ ev,
                                                const uint32_t* __restrict__ eoff, const uint32_t* __restrict__ elen,
                                                const ShdNicSend* __restrict__ sends,
                                                const uint32_t* __restrict__ soff, uint64_t window_end,
                                                uint64_t boot_end, ShdNicState* __restrict__ states,
                                                ShdCodelEntry* __restrict__ rings, uint32_t ring_cap,
                                                uint32_t id_base, uint64_t* __restrict__ rtime,
                                                uint8_t* __restrict__ rstat, uint64_t fate_cap,
                                                uint64_t* __restrict__ stime, int* __restrict__ err,
                                                uint32_t flush_at, uint32_t opts) {
    const bool inline_refill = opts & 1u, fast_arrival = opts & 2u;
    __shared__ uint64_t stage_t[kStage * 64];
    __shared__ uint8_t stage_s[kStage * 64];
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    // The window's arrivals start as queued (~0, SHD_NIC_QUEUED) and its send
    // requests unsent (~0): the wave's hosts' segments are one contiguous id
    // range, filled by the whole wave in coalesced strides (no offsets read
    // back to the host, no memsets before the launch); the barrier orders
    // these stores before any lane's fates to the same ids (one wave per
    // block: it costs nothing, and unlike a thread-scope fence it is a
    // release/acquire pair under the HIP memory model).
    // (inputs every lane checks alike, so that no host runs when they fail)
    const uint32_t all0 = eoff[0], all1 = eoff[n];
    const int bad_all = ((uint64_t)id_base + all1 > fate_cap ? kErrId : 0) |
                        (all1 > all0 && (!ev || !elen) ? kErrArgs : 0);
    if (!bad_all) {
        const uint32_t h0 = blockIdx.x * blockDim.x, h1 = h0 + 64 < n ? h0 + 64 : n;
        const uint32_t w0 = eoff[h0], w1 = eoff[h1];
        for (uint32_t k = w0 + threadIdx.x; k < w1; k += 64) {
            rtime[id_base + k] = ~0ull;
            rstat[id_base + k] = SHD_NIC_QUEUED;
        }
        if (soff)
            for (uint32_t k = soff[h0] + threadIdx.x; k < soff[h1]; k += 64) stime[k] = ~0ull;
    }
    __syncthreads();
    if (h >= n) return;
    const uint32_t self = host_base + h;
    FateStage out{rtime, rstat, stage_t + threadIdx.x, stage_s + threadIdx.x, 0u, 0u};
    Host H;
    H.s = states[h];
    uint32_t i = eoff[h];
    const uint32_t iend = eoff[h + 1];
    H.q = RouterQ{rings + (size_t)h * ring_cap, ring_cap, H.s.router.head, H.s.router.len, ev, elen, i, i, id_base,
                  &out, false, ~0u, 0, 0};
    H.sends = sends;
    H.sq = H.sk = soff ? soff[h] : 0;
    const uint32_t kend = soff ? soff[h + 1] : 0;
    H.stime = stime;
    H.boot_end = boot_end;
    int bad = bad_all;
    uint64_t last = 0;
    // every lane ends: at most this many events (a host whose bucket refills
    // by 0 bytes per ms schedules a refill every ms for ever, as the reference)
    uint64_t budget = (uint64_t)(iend - i) + (kend - H.sk) + (1ull << 24);
    // the next arrival and its length in registers, the one after it in flight
    ShdDeliv a_cur{}, a_nxt{};
    uint32_t l_cur = 0, l_nxt = 0;
    if (!bad && i < iend) { // (bad: e.g. events without an event array -- nothing is read)
        a_cur = ev[i];
        l_cur = elen[i];
    }
    if (!bad && i + 1 < iend) {
        a_nxt = ev[i + 1];
        l_nxt = elen[i + 1];
    }
    while (!bad) {
        // A refill that comes next in the host's order while its router queue
        // is empty (the common case: the queue drains at each arrival) runs
        // here, in a loop of its own -- the same call, in the same order --
        // so that a wave whose lanes reach their refills at different
        // iterations does not run the whole merged body (arrival, CoDel
        // dequeue, send) once more per lane's refill.
        if (kMerged && inline_refill)
            while (H.s.refill_pending && H.s.refill_time < window_end && H.q.empty()) {
                const uint64_t tr = H.s.refill_time;
                if (H.sk < kend && sends[H.sk].ready <= tr) break; // a send request first
                if (i < iend && (a_cur.time < tr || (a_cur.time == tr && a_cur.src_host < self))) break; // an arrival
                if (budget-- == 0) {
                    bad |= kErrWindow;
                    break;
                }
                H.refill(tr);
            }
        if (bad) break;
        if (budget-- == 0) {
            bad |= kErrWindow;
            break;
        }
        const bool have_a = i < iend;
        const bool have_s = H.sk < kend;
        const bool have_r = H.s.refill_pending && H.s.refill_time < window_end;
        if (!have_a && !have_s && !have_r) break;
        const ShdDeliv a = a_cur;
        const uint64_t ta = have_a ? a.time : kNever;
        const uint64_t ts = have_s ? sends[H.sk].ready : kNever;
        const uint64_t tr = have_r ? H.s.refill_time : kNever;
        // the host's own next event: a send request before a refill at equal times
        const bool own_is_send = have_s && (!have_r || ts <= tr);
        const uint64_t town = own_is_send ? ts : tr;
        const bool own_exists = have_s || have_r;
        uint64_t now = 0;
        bool do_recv = false, do_send = false, do_sched = false;
        if (have_a && (!own_exists || ta < town || (ta == town && a.src_host < self))) {
            if (a.dst_host != self) bad |= kErrHost;
            if (ta < last) bad |= kErrOrder;
            if (ta >= window_end) bad |= kErrWindow;
            if (bad) break;
            last = ta;
            // router_enqueue (router.c:103-121): peek, enqueue, receive if it was empty
            const bool buffered = !H.q.empty();
            H.q.cidx = i;
            H.q.ctime = ta;
            H.q.clen = l_cur;
            H.q.qtail = ++i;
            H.s.router.total_size += l_cur; // _routerqueuecodel_enqueue (:113-136)
            const uint32_t l_prev = l_cur;
            a_cur = a_nxt;
            l_cur = l_nxt;
            if (i + 1 < iend) {
                a_nxt = ev[i + 1];
                l_nxt = elen[i + 1];
            }
            if (kMerged && fast_arrival && !buffered && ta >= boot_end && H.s.recv_remaining >= kMtu &&
                H.s.router.mode == 0) {
                // the common arrival: the queue held nothing before it, the
                // bucket has a packet's tokens and CoDel is not dropping, so
                // receivePackets dequeues exactly this packet (sojourn 0:
                // below target) and then finds the queue empty -- its
                // effects, without the dequeue's general code
                H.q.qhead++;
                H.s.router.total_size -= l_prev;
                H.s.router.interval_expire = 0;
                out.put(id_base + i - 1, ta, SHD_NIC_RECEIVED);
                consume(H.s.recv_remaining, l_prev);
                schedule_if_needed(H.s, ta);
            } else if (kMerged) {
                now = ta, do_recv = !buffered;
            } else if (!buffered) {
                H.receive(ta);
            }
        } else if (own_is_send) {
            if (ts >= window_end) {
                bad |= kErrWindow;
                break;
            }
            H.sk++; // networkinterface_wantsSend (:633-661)
            if (kMerged) now = ts, do_send = true;
            else H.send(ts);
        } else if (kMerged) {
            H.refill_tokens(); // _networkinterface_refillTokenBucketsCB (:166-186)
            now = tr, do_recv = do_send = do_sched = true;
        } else {
            H.refill(tr);
        }
        if (kMerged) {
            if (do_recv) H.receive(now);
            if (do_send) H.send(now);
            if (do_sched) schedule_if_needed(H.s, now);
        }
        if (H.q.bad) bad |= kErrAssert;
        // the wave's lanes flush their staged fates together once one of them
        // holds flush_at: a lane flushing alone (its stage full) makes the
        // whole wave run the store loop for it, 64 times as often
        if (__any(out.n >= flush_at)) out.flush();
    }
    // the window's arrivals still queued move to the ring
    while (!bad && H.q.qhead < H.q.qtail) {
        if (H.q.len == H.q.cap) {
            bad |= kErrRing;
            break;
        }
        const uint32_t k = H.q.qhead++;
        uint32_t tail = H.q.head + H.q.len;
        if (tail >= H.q.cap) tail -= H.q.cap;
        H.q.ring[tail] = ShdCodelEntry{ev[k].time, id_base + k, elen[k]};
        H.q.len++;
    }
    out.flush();
    if (bad) atomicOr(err, bad);
    H.s.router.head = H.q.head;
    H.s.router.len = H.q.len;
    states[h] = H.s;
}

__global__ void k_event_lengths(size_t n, const ShdDeliv* __restrict__ ev, const ShdPkt* __restrict__ pk,
                                uint32_t header, uint32_t* __restrict__ len) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) len[i] = pk[ev[i].pkt_index].payload_len + header;
}

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

} // namespace

extern "C" int shd_nic_init(uint32_t nhosts, const uint64_t* d_bw_down_kibps, const uint64_t* d_bw_up_kibps,
                            uint64_t start_time, ShdNicState* d_states, void* stream) {
    if (!nhosts) return 0;
    if (!d_bw_down_kibps || !d_bw_up_kibps || !d_states) return -EINVAL;
    hipLaunchKernelGGL(k_nic_init, dim3((nhosts + 255) / 256), dim3(256), 0, (hipStream_t)stream, nhosts,
                       d_bw_down_kibps, d_bw_up_kibps, start_time, d_states);
    return hip_status(hipGetLastError(), "k_nic_init launch");
}

extern "C" int shd_event_lengths(const ShdDeliv* d_events, size_t n, const ShdPkt* d_pkts, uint32_t header_bytes,
                                 uint32_t* d_lengths, void* stream) {
    if (!n) return 0;
    hipLaunchKernelGGL(k_event_lengths, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                       d_events, d_pkts, header_bytes, d_lengths);
    return hip_status(hipGetLastError(), "k_event_lengths launch");
}

namespace {
// Per-thread error words (device words per device, one pinned host word).
// A word whose allocation no longer exists (a hipDeviceReset since) is
// allocated again.
struct NicErrWords {
    int* d[64] = {};
    int* h = nullptr;
    ~NicErrWords() {
        for (int* p : d)
            if (p) (void)hipFree(p);
        if (h) (void)hipHostFree(h);
    }
};
thread_local NicErrWords t_nic_err;

int nic_err_words(int dev, int** d_err) {
    int rc = 0;
    hipPointerAttribute_t at;
    if (t_nic_err.h && hipPointerGetAttributes(&at, t_nic_err.h) != hipSuccess) t_nic_err.h = nullptr;
    if (!t_nic_err.h &&
        (rc = hip_status(hipHostMalloc((void**)&t_nic_err.h, sizeof(int), hipHostMallocDefault), "hipHostMalloc nic")))
        return rc;
    int*& w = t_nic_err.d[dev];
    if (w && hipPointerGetAttributes(&at, w) != hipSuccess) w = nullptr;
    if (!w && ((rc = hip_status(hipMalloc((void**)&w, sizeof(int)), "hipMalloc nic")) ||
               (rc = hip_status(hipMemset(w, 0, sizeof(int)), "memset nic"))))
        return rc;
    *d_err = w;
    return 0;
}
} // namespace

extern "C" int shd_nic_run(uint32_t nhosts, uint32_t host_base, const ShdDeliv* d_events,
                           const uint32_t* d_event_offsets, const uint32_t* d_event_lengths, const ShdNicSend* d_sends,
                           const uint32_t* d_send_offsets, uint64_t window_end, uint64_t bootstrap_end,
                           ShdNicState* d_states, ShdCodelEntry* d_rings, uint32_t ring_cap, uint32_t id_base,
                           uint64_t* d_recv_time, uint8_t* d_recv_status, uint64_t fate_cap, uint64_t* d_send_time,
                           void* stream) {
    if (!nhosts) return 0;
    if (!d_event_offsets || !d_states || !d_rings || !ring_cap || !d_recv_time || !d_recv_status)
        return shd_fail(-EINVAL, "missing buffer");
    if (d_send_offsets && (!d_sends || !d_send_time)) return shd_fail(-EINVAL, "send offsets without sends");
    hipStream_t s = (hipStream_t)stream;
    // the error word: one per thread and device, kept (a call allocates
    // nothing), zero between calls (only a call that read a nonzero word
    // clears it), read back into pinned memory; freed when the thread ends.
    // The stream must belong to the calling thread's current device.
    int dev = 0, sdev = 0;
    int rc = hip_status(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    if (dev < 0 || dev >= 64) return shd_fail(-EINVAL, "device %d", dev);
    if (s && (rc = hip_status(hipStreamGetDevice(s, &sdev), "hipStreamGetDevice"))) return rc;
    if (s && sdev != dev) return shd_fail(-EINVAL, "stream of device %d used on device %d", sdev, dev);
    int* d_err = nullptr;
    if ((rc = nic_err_words(dev, &d_err))) return rc;
    int* t_herr = t_nic_err.h;
    // SHD_NIC_FLUSH: the staged-fate count at which a wave flushes together
    // (kStage + 1: each lane on its own when its stage fills)
    const char* fv = getenv("SHD_NIC_FLUSH");
    const uint32_t flush_at = fv ? (uint32_t)atoi(fv) : 12;
    // SHD_NIC_INLINE_REFILL=0: refills only as iterations of the merged loop;
    // SHD_NIC_FAST=0: every arrival's receive through the CoDel dequeue
    const char* iv = getenv("SHD_NIC_INLINE_REFILL");
    const char* fa = getenv("SHD_NIC_FAST");
    const uint32_t opts = (iv && strcmp(iv, "0") == 0 ? 0u : 1u) | (fa && strcmp(fa, "0") == 0 ? 0u : 2u);
    if (!rc) {
        const char* mv = getenv("SHD_NIC_MERGED");
        if (mv && strcmp(mv, "0") == 0)
            hipLaunchKernelGGL(k_nic_run<false>, dim3((nhosts + 63) / 64), dim3(64), 0, s, nhosts, host_base,
                               d_events, d_event_offsets, d_event_lengths, d_sends, d_send_offsets, window_end,
                               bootstrap_end, d_states, d_rings, ring_cap, id_base, d_recv_time, d_recv_status,
                               fate_cap, d_send_time, d_err, flush_at, opts);
        else
            hipLaunchKernelGGL(k_nic_run<true>, dim3((nhosts + 63) / 64), dim3(64), 0, s, nhosts, host_base,
                               d_events, d_event_offsets, d_event_lengths, d_sends, d_send_offsets, window_end,
                               bootstrap_end, d_states, d_rings, ring_cap, id_base, d_recv_time, d_recv_status,
                               fate_cap, d_send_time, d_err, flush_at, opts);
        rc = hip_status(hipGetLastError(), "k_nic_run launch");
    }
    if (!rc) rc = hip_status(hipMemcpyAsync(t_herr, d_err, sizeof(int), hipMemcpyDeviceToHost, s), "D2H");
    if (!rc) rc = hip_status(hipStreamSynchronize(s), "k_nic_run");
    if (rc) {
        (void)hipMemset(d_err, 0, sizeof(int)); // (whatever failed: the next call starts from zero)
        return rc;
    }
    const int h_err = *t_herr;
    if (h_err && (rc = hip_status(hipMemset(d_err, 0, sizeof(int)), "memset nic"))) return rc;
    if (h_err & kErrRing) return shd_fail(-ENOSPC, "a router queue outgrew its ring (capacity %u)", ring_cap);
    if (h_err & kErrHost) return shd_fail(-EINVAL, "an event in a host's segment is addressed to another host");
    if (h_err & kErrOrder) return shd_fail(-EINVAL, "a host's events are not in time order");
    if (h_err & kErrWindow)
        return shd_fail(-EINVAL, "an event or send request at or after the window end, or more than 2^24 refills "
                                 "in one window");
    if (h_err & kErrId) return shd_fail(-ERANGE, "packet ids exceed the fate arrays");
    if (h_err & kErrAssert) return shd_fail(-EINVAL, "router dequeue before an entry's enqueue time");
    if (h_err & kErrArgs) return shd_fail(-EINVAL, "events without lengths");
    return 0;
}
