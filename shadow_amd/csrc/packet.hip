// packet.hip -- the per-round inter-host packet hand-off on gfx950
// (reference core/worker.c:517-576,
// core/scheduler/scheduler.c:232-255, scheduler_policy_host_single.c:174-220,
// core/work/event.c:109-152, utility/random.c:32-43).
//
// Pipeline over one round's batch (all device-resident, one stream):
//   k_pkt_scatter  per record: host->slot gathers, owner resolution of the
//                  reference cache (touch order / pair bits), 16 B table
//                  gather, the sender's reserved rand_r draw, the drop rule,
//                  ceil(lat * 1e6) delay, end-time drop, barrier clamp,
//                  per-destination count and the min delivered time.
//                  This is the HBM-bound kernel the roofline is quoted on.
//   k_scan_*       exclusive scan of the per-destination counts.
//   k_place        places each delivered event into its destination segment.
//   k_segsort_*    orders every segment by event_compare's remaining keys
//                  (time, src host, srcHostEventID): a rank sort in LDS for
//                  segments up to 1024 events, a padded all-ascending bitonic
//                  network in HBM above that.
// Because event_compare is a total order, per-destination heap pop order
// (priority_queue.c) equals this sorted order, so the output is identical to
// pushing every event into its destination's queue.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>

#include "shd_internal.h"

namespace {

constexpr int kScanTile = 4096; // 256 threads x 16
constexpr int kSmallSeg = 512; // wave register sort up to 8 events per lane

__device__ __forceinline__ int glibc_rand_r(uint32_t* state) {
    uint32_t next = *state;
    int result;
    next = next * 1103515245u + 12345u;
    result = (int)((next / 65536u) % 2048u);
    next = next * 1103515245u + 12345u;
    result = (result << 10) ^ (int)((next / 65536u) % 1024u);
    next = next * 1103515245u + 12345u;
    result = (result << 10) ^ (int)((next / 65536u) % 1024u);
    *state = next;
    return result;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o < v ? o : v;
    }
    return v;
}

__global__ __launch_bounds__(256) void k_pkt_scatter(ShdPktCtx c, const ShdPkt* __restrict__ recs, size_t n,
                                                     uint64_t barrier, uint64_t end_time, uint64_t boot_end,
                                                     ShdDeliv* __restrict__ tmp, uint8_t* __restrict__ status,
                                                     uint32_t* __restrict__ cnt, unsigned long long* counters) {
    __shared__ unsigned long long wmin[4];
    unsigned long long mn = ~0ull;
    const size_t A = (size_t)c.A;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const ShdPkt p = recs[i];
        const bool known = p.src_host < c.nhosts && p.dst_host < c.nhosts;
        const int si = known ? c.host_slot[p.src_host] : -1;
        const int di = known ? c.host_slot[p.dst_host] : -1;
        uint8_t st = 0xff; // unregistered host: not delivered
        if (si >= 0 && di >= 0) {
            int oi = si, oj = di;
            if (c.mode == 0) {
                // owner({s,d}) = row touched first (topology.c:1189-1215, 1918-1968)
                if (si != di && c.touch[di] < c.touch[si]) oi = di, oj = si;
            } else if (c.mode == 2) {
                const size_t b = (size_t)si * A + (size_t)di;
                if (!((c.pair_bits[b >> 5] >> (b & 31)) & 1u)) oi = di, oj = si;
            }
            const ShdEntry e = c.tab[(size_t)oi * A + (size_t)oj];
            uint32_t rs = p.rng_state;
            const double chance = (double)glibc_rand_r(&rs) / 2147483647.0; // random_nextDouble
            st = SHD_DROPPED_LOSS;
            if (p.now < boot_end || chance <= e.rel || p.payload_len == 0) { // worker.c:545
                uint64_t t = p.now + (uint64_t)ceil(e.lat * 1000000.0);   // worker.c:548-549
                if (t >= end_time) {                                        // scheduler.c:236-239
                    st = SHD_DROPPED_END;
                } else {
                    if (p.src_host != p.dst_host && t < barrier) t = barrier; // host_single.c:187-192
                    st = SHD_DELIVERED;
                    // the count's old value is this event's slot in its
                    // destination segment (carried in pad; order fixed by the sort)
                    const uint32_t rank = atomicAdd(&cnt[p.dst_host], 1u);
                    tmp[i] = ShdDeliv{t, p.seq, p.src_host, p.dst_host, (uint32_t)i, rank};
                    if (t >= barrier && t < mn) mn = t; // worker.c:350-363
                }
            }
        }
        status[i] = st;
    }
    mn = wave_min_u64(mn);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) wmin[w] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int k = 1; k < (int)(blockDim.x >> 6); k++) m = wmin[k] < m ? wmin[k] : m;
        if (m != ~0ull) atomicMin(&counters[1], m);
    }
}

__global__ __launch_bounds__(256) void k_hist_deliv(const ShdDeliv* __restrict__ in, size_t n, uint32_t host_lo,
                                                    uint32_t H, uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ rank) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t d = in[i].dst_host - host_lo; // out-of-range events are dropped
        rank[i] = d < H ? atomicAdd(&cnt[d], 1u) : ~0u;
    }
}

// ---- exclusive scan of per-destination counts ----

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(v, off);
        if (lane >= off) v += o;
    }
    return v;
}

// block-wide exclusive scan of one value per thread (256 threads)
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
    __shared__ uint32_t ws[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int k = 0; k < 4; k++) {
        if (k < w) base += ws[k];
        tot += ws[k];
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

__global__ __launch_bounds__(256) void k_scan_local(const uint32_t* __restrict__ cnt, uint32_t H,
                                                    uint32_t* __restrict__ off, uint32_t* __restrict__ bsum) {
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * 16;
    uint32_t v[16], s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        v[k] = (base + k < H) ? cnt[base + k] : 0u;
        s += v[k];
    }
    uint32_t total;
    uint32_t pre = block_excl_scan(s, &total);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if (base + k < H) off[base + k] = pre;
        pre += v[k];
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_top(uint32_t* __restrict__ bsum, uint32_t nb) {
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < nb ? bsum[i] : 0u;
        uint32_t total;
        const uint32_t pre = block_excl_scan(v, &total);
        if (i < nb) bsum[i] = carry + pre;
        __syncthreads();
        if (threadIdx.x == 0) carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* __restrict__ off, const uint32_t* __restrict__ cnt, uint32_t H,
                                                  const uint32_t* __restrict__ bsum, uint32_t nb,
                                                  uint32_t* __restrict__ cur, uint32_t* __restrict__ big,
                                                  uint32_t* __restrict__ nbig, unsigned long long* counters) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < H) {
        off[i] += bsum[i / kScanTile];
        cur[i] = 0;
        if (cnt[i] > (uint32_t)kSmallSeg) big[atomicAdd(nbig, 1u)] = (uint32_t)i;
    }
    if (i == 0) {
        off[H] = bsum[nb];
        if (counters) counters[0] = bsum[nb];
    }
}

// Atomic-free placement: every event already holds its slot inside its
// destination segment (returned by the counting atomic), in pad (packet
// path) or in rank[] (regroup path).
__global__ __launch_bounds__(256) void k_place(const ShdDeliv* __restrict__ tmp, const uint8_t* __restrict__ status,
                                               const uint32_t* __restrict__ rank, size_t n, uint32_t host_lo,
                                               uint32_t H, const uint32_t* __restrict__ off,
                                               ShdDeliv* __restrict__ scr) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (status && status[i] != SHD_DELIVERED) continue;
        const ShdDeliv r = tmp[i];
        const uint32_t d = r.dst_host - host_lo;
        if (d >= H) continue;
        scr[off[d] + (rank ? rank[i] : r.pad)] = r;
    }
}

__device__ __forceinline__ bool ev_less(const ShdDeliv& a, const ShdDeliv& b) {
    // event_compare with equal destination: time, src host id, srcHostEventID
    if (a.time != b.time) return a.time < b.time;
    if (a.src_host != b.src_host) return a.src_host < b.src_host;
    return a.seq < b.seq;
}

// Sort key + payload of one event inside a destination segment.
struct Ev {
    unsigned long long t, q; // time, srcHostEventID
    unsigned s, ix;          // src host, packet index
};

__device__ __forceinline__ bool ev_lt(const Ev& a, const Ev& b) {
    if (a.t != b.t) return a.t < b.t;
    if (a.s != b.s) return a.s < b.s;
    return a.q < b.q;
}

__device__ __forceinline__ Ev ev_shfl_xor(const Ev& e, int m) {
    Ev o;
    o.t = __shfl_xor(e.t, m);
    o.q = __shfl_xor(e.q, m);
    o.s = (unsigned)__shfl_xor((int)e.s, m);
    o.ix = (unsigned)__shfl_xor((int)e.ix, m);
    return o;
}

// One wave sorts one segment of n <= 64*E events held in registers
// (element i = e*64 + lane), bitonic network over 64*E slots with +inf
// padding; partner distances < 64 cross lanes by shuffle, >= 64 stay in-lane.
template <int E>
__device__ void wave_sort_segment(const ShdDeliv* __restrict__ scr, uint32_t b, uint32_t n, uint32_t d,
                                  ShdDeliv* __restrict__ out, int lane) {
    Ev v[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        if (i < n) {
            const ShdDeliv r = scr[b + i];
            v[e] = Ev{r.time, r.seq, r.src_host, r.pkt_index};
        } else {
            v[e] = Ev{~0ull, ~0ull, ~0u, ~0u};
        }
    }
#pragma unroll
    for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int p = e ^ (j >> 6);
                    if (p > e) {
                        const bool up = (((e * 64 + lane) & k) == 0);
                        const bool sw = up ? ev_lt(v[p], v[e]) : ev_lt(v[e], v[p]);
                        if (sw) {
                            const Ev tmp = v[e];
                            v[e] = v[p];
                            v[p] = tmp;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const Ev o = ev_shfl_xor(v[e], j);
                    const bool up = (((e * 64 + lane) & k) == 0);
                    const bool lower = (lane & j) == 0;
                    const bool o_lt = ev_lt(o, v[e]);
                    // the lower slot keeps the min when ascending, the max when descending
                    const bool take_o = (lower == up) ? o_lt : ev_lt(v[e], o);
                    if (take_o) v[e] = o;
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        if (i < n) out[b + i] = ShdDeliv{v[e].t, v[e].q, v[e].s, d, v[e].ix, 0u};
    }
}

// Segments of up to kSmallSeg events, one wave each.
__global__ __launch_bounds__(256) void k_segsort_wave(const ShdDeliv* __restrict__ scr, const uint32_t* __restrict__ off,
                                                      uint32_t H, uint32_t host_lo, ShdDeliv* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t d = wave; d < H; d += nwaves) {
        const uint32_t b = off[d], n = off[d + 1] - b;
        const uint32_t dh = d + host_lo;
        if (n == 0) continue;
        if (n <= 64) wave_sort_segment<1>(scr, b, n, dh, out, lane);
        else if (n <= 128) wave_sort_segment<2>(scr, b, n, dh, out, lane);
        else if (n <= 256) wave_sort_segment<4>(scr, b, n, dh, out, lane);
        else if (n <= (uint32_t)kSmallSeg) wave_sort_segment<8>(scr, b, n, dh, out, lane);
    }
}

__device__ __forceinline__ void cmpx(ShdDeliv* v, uint32_t a, uint32_t b) {
    const ShdDeliv x = v[a], y = v[b];
    if (ev_less(y, x)) {
        v[a] = y;
        v[b] = x;
    }
}

// Segments above kSmallSeg events: copy, then an all-ascending bitonic
// network over the next power of two with virtual +inf padding (pairs that
// touch the padding are skipped, which is exact for this network form).
__global__ __launch_bounds__(256) void k_segsort_big(const ShdDeliv* __restrict__ scr, const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ big, const uint32_t* __restrict__ nbig,
                                                     ShdDeliv* __restrict__ out) {
    const uint32_t nb = *nbig;
    for (uint32_t q = blockIdx.x; q < nb; q += gridDim.x) {
        const uint32_t d = big[q];
        const uint32_t b = off[d], n = off[d + 1] - b;
        ShdDeliv* v = out + b;
        for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
            ShdDeliv r = scr[b + k];
            r.pad = 0; // drop the placement rank carried in pad
            v[k] = r;
        }
        __syncthreads();
        uint32_t N = 1;
        while (N < n) N <<= 1;
        for (uint32_t k = 2; k <= N; k <<= 1) {
            const uint32_t half = k >> 1;
            for (uint32_t i = threadIdx.x; i < N / 2; i += blockDim.x) {
                const uint32_t blk = i / half, o = i % half;
                const uint32_t x = blk * k + o, y = blk * k + k - 1 - o;
                if (y < n) cmpx(v, x, y);
            }
            __syncthreads();
            for (uint32_t j = k >> 2; j >= 1; j >>= 1) {
                for (uint32_t i = threadIdx.x; i < N / 2; i += blockDim.x) {
                    const uint32_t blk = i / j, o = i % j;
                    const uint32_t x = blk * 2 * j + o, y = x + j;
                    if (y < n) cmpx(v, x, y);
                }
                __syncthreads();
            }
        }
        __syncthreads();
    }
}

// ---- workspace (grow-only, per process / device) ----
struct Ws {
    size_t cap_n = 0;
    uint32_t cap_h = 0;
    ShdDeliv* tmp = nullptr;
    ShdDeliv* scr = nullptr;
    uint32_t* cnt = nullptr; // cap_h
    uint32_t* cur = nullptr; // cap_h
    uint32_t* bsum = nullptr;
    uint32_t* big = nullptr; // cap_h
    uint32_t* nbig = nullptr;
};
Ws g_ws;

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

int ws_reserve(size_t n, uint32_t H) {
    int rc = 0;
    if (n > g_ws.cap_n) {
        (void)hipFree(g_ws.tmp);
        (void)hipFree(g_ws.scr);
        g_ws.tmp = g_ws.scr = nullptr;
        g_ws.cap_n = 0;
        const size_t cap = n + n / 8 + 1024;
        if ((rc = hip_status(hipMalloc((void**)&g_ws.tmp, sizeof(ShdDeliv) * cap), "hipMalloc ws.tmp")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.scr, sizeof(ShdDeliv) * cap), "hipMalloc ws.scr")))
            return rc;
        g_ws.cap_n = cap;
    }
    if (H + 1 > g_ws.cap_h) {
        (void)hipFree(g_ws.cnt);
        (void)hipFree(g_ws.cur);
        (void)hipFree(g_ws.bsum);
        (void)hipFree(g_ws.big);
        (void)hipFree(g_ws.nbig);
        g_ws.cap_h = 0;
        const uint32_t cap = H + 1 + 1024;
        if ((rc = hip_status(hipMalloc((void**)&g_ws.cnt, 4ull * cap), "hipMalloc ws.cnt")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.cur, 4ull * cap), "hipMalloc ws.cur")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.bsum, 4ull * (cap / kScanTile + 2)), "hipMalloc ws.bsum")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.big, 4ull * cap), "hipMalloc ws.big")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.nbig, 16), "hipMalloc ws.nbig")))
            return rc;
        g_ws.cap_h = cap;
    }
    return 0;
}

unsigned grid_for(size_t n, unsigned block, unsigned cap) {
    size_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

// ---- optional per-stage timing with HIP events on the launch stream ----
constexpr int kStages = 4; // 0 packet-scatter, 1 scan, 2 place, 3 segment sort
constexpr int kMaxTimed = 1024;
struct Timing {
    bool on = false;
    int n = 0;
    hipEvent_t ev[kMaxTimed][kStages + 1];
    bool created = false;
};
Timing g_tm;

void mark(int stage, hipStream_t s) {
    if (g_tm.on && g_tm.n < kMaxTimed) (void)hipEventRecord(g_tm.ev[g_tm.n][stage], s);
}

// scan + place + segment sort, shared by both entry points
int group_and_sort(const ShdDeliv* tmp, const uint8_t* status, const uint32_t* rank, size_t n, uint32_t host_lo,
                   uint32_t H, ShdDeliv* out, uint32_t* offsets, unsigned long long* counters, hipStream_t s) {
    const uint32_t nb = (H + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_local, dim3(nb ? nb : 1), dim3(256), 0, s, g_ws.cnt, H, offsets, g_ws.bsum);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, g_ws.bsum, nb);
    hipLaunchKernelGGL(k_scan_add, dim3(grid_for(H + 1, 256, 1u << 30)), dim3(256), 0, s, offsets, g_ws.cnt, H,
                       g_ws.bsum, nb, g_ws.cur, g_ws.big, g_ws.nbig, counters);
    mark(2, s);
    hipLaunchKernelGGL(k_place, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, tmp, status, rank, n, host_lo, H,
                       offsets, g_ws.scr);
    mark(3, s);
    hipLaunchKernelGGL(k_segsort_wave, dim3(grid_for(H, 4, 16384)), dim3(256), 0, s, g_ws.scr, offsets, H, host_lo,
                       out);
    hipLaunchKernelGGL(k_segsort_big, dim3(64), dim3(256), 0, s, g_ws.scr, offsets, g_ws.big, g_ws.nbig, out);
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    return hip_status(hipGetLastError(), "group_and_sort launch");
}

} // namespace

extern "C" int shd_dev_packet_round(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                                    uint64_t end_time, uint64_t bootstrap_end, ShdDeliv* d_out,
                                    uint32_t* d_dst_offsets, uint8_t* d_status, uint64_t* d_counters, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const uint32_t H = c->nhosts;
    int rc = ws_reserve(n, H);
    if (rc) return rc;
    unsigned long long* counters = (unsigned long long*)d_counters;
    if ((rc = hip_status(hipMemsetAsync(g_ws.cnt, 0, 4ull * (H + 1), s), "memset cnt")) ||
        (rc = hip_status(hipMemsetAsync(g_ws.nbig, 0, 4, s), "memset nbig")) ||
        (rc = hip_status(hipMemsetAsync(counters, 0xff, 16, s), "memset counters")))
        return rc;
    mark(0, s);
    if (n)
        hipLaunchKernelGGL(k_pkt_scatter, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, *c, d_recs, n, barrier,
                           end_time, bootstrap_end, g_ws.tmp, d_status, g_ws.cnt, counters);
    mark(1, s);
    if ((rc = hip_status(hipGetLastError(), "k_pkt_scatter launch"))) return rc;
    rc = group_and_sort(g_ws.tmp, d_status, nullptr, n, 0, H, d_out, d_dst_offsets, counters, s);
    if (rc) return rc;
    return stream ? 0 : hip_status(hipStreamSynchronize(s), "packet round");
}

extern "C" int shd_round_timing_enable(int enable) {
    if (enable && !g_tm.created) {
        for (int i = 0; i < kMaxTimed; i++)
            for (int k = 0; k <= kStages; k++)
                if (hipEventCreate(&g_tm.ev[i][k]) != hipSuccess) return shd_fail(-EIO, "hipEventCreate");
        g_tm.created = true;
    }
    g_tm.on = enable != 0;
    g_tm.n = 0;
    return 0;
}

extern "C" int shd_round_timing_read(double* stage_ms, int nstages, int* launches) {
    if (nstages > kStages) nstages = kStages;
    for (int k = 0; k < nstages; k++) stage_ms[k] = 0.0;
    for (int i = 0; i < g_tm.n; i++) {
        if (hipEventSynchronize(g_tm.ev[i][kStages]) != hipSuccess) return shd_fail(-EIO, "hipEventSynchronize");
        for (int k = 0; k < nstages; k++) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, g_tm.ev[i][k], g_tm.ev[i][k + 1]) != hipSuccess)
                return shd_fail(-EIO, "hipEventElapsedTime");
            stage_ms[k] += ms;
        }
    }
    if (launches) *launches = g_tm.n;
    return 0;
}

extern "C" int shd_dev_deliv_sort(const ShdDeliv* d_in, size_t n, uint32_t host_lo, uint32_t host_hi, ShdDeliv* d_out,
                                  uint32_t* d_dst_offsets, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const uint32_t H = host_hi - host_lo;
    int rc = ws_reserve(n, H);
    if (rc) return rc;
    if ((rc = hip_status(hipMemsetAsync(g_ws.cnt, 0, 4ull * (H + 1), s), "memset cnt")) ||
        (rc = hip_status(hipMemsetAsync(g_ws.nbig, 0, 4, s), "memset nbig")))
        return rc;
    mark(0, s);
    if (n)
        hipLaunchKernelGGL(k_hist_deliv, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, d_in, n, host_lo, H, g_ws.cnt,
                           reinterpret_cast<uint32_t*>(g_ws.tmp)); // tmp is free here: ranks
    mark(1, s);
    rc = group_and_sort(d_in, nullptr, reinterpret_cast<const uint32_t*>(g_ws.tmp), n, host_lo, H, d_out,
                        d_dst_offsets, nullptr, s);
    if (rc) return rc;
    return stream ? 0 : hip_status(hipStreamSynchronize(s), "deliv sort");
}
