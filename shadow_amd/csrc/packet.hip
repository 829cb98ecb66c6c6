// packet.hip -- the per-round inter-host packet hand-off on gfx950
// (reference core/worker.c:517-576,
// core/scheduler/scheduler.c:232-255, scheduler_policy_host_single.c:174-220,
// core/work/event.c:109-152, utility/random.c:32-43).
//
// Pipeline over one round's batch (device-resident, one stream, no global
// atomics on the event path -- device-scope atomics execute memory-side on
// gfx950, ~20 G/s for scattered addresses, which bounded the first version):
//   k_pkt_scatter  tile of 8192 records per workgroup: host->slot gathers,
//                  owner resolution of the reference cache (touch order /
//                  pair bits), 16 B table gather, the sender's reserved
//                  rand_r draw, drop rule, ceil(lat * 1e6) delay, end-time
//                  drop, barrier clamp; writes the event and counts it in an
//                  LDS histogram over destination *buckets* (128 hosts each).
//                  HBM-bound; the roofline is quoted on this kernel.
//   k_scan_*       exclusive scan of the (bucket x tile) count matrix.
//   k_part1        per tile: LDS ranks -> event into its bucket's region.
//   k_part2_sort   per bucket (workgroup): LDS histogram + scan over its
//                  128 destinations -> per-destination offsets, LDS-ranked
//                  placement, then one wave per destination sorts the
//                  segment by event_compare's remaining keys (time, src host,
//                  srcHostEventID) with a register bitonic network.
//   k_segsort_big  destinations with more than 512 events in a round:
//                  padded all-ascending bitonic network in HBM.
// event_compare is a total order, so per-destination heap pop order
// (priority_queue.c) equals this sorted order: the output is identical to
// pushing every event into its destination's queue.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "shd_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 16;
constexpr int kBatch = 4; // records per thread in flight through the gather chain
constexpr int kTile = kBlock * kItems; // records per workgroup in the tile kernels
constexpr int kMaxBuckets = 1024;      // level-1 buckets (LDS histogram size)
constexpr int kScanTile = 4096;        // 256 threads x 16
constexpr int kSmallSeg = 256;         // wave register sort up to 4 events per lane
constexpr int kSortBlock = 512;        // k_part2_sort workgroup (8 waves)
constexpr int kStream = 8;             // loads in flight per thread in the streaming passes
constexpr int kGroup = 8;              // scatter tiles per k_part1 workgroup
constexpr int kPartBlock = 1024;

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

struct Bucketing {
    uint32_t host_lo; // first host id of the range
    uint32_t H;       // hosts in range
    uint32_t shift;   // bucket = (dst - host_lo) >> shift
    uint32_t nb;      // number of buckets
    uint32_t ntiles;
};

// kRank = true ("rank" pipeline): each delivered event takes its slot in its
// destination segment from a per-destination counter (the counter's old
// value, carried in pad); cnt1 is then the per-destination count array.
// kRank = false ("bucket" pipeline): LDS histogram over destination buckets
// per tile; cnt1 is the bucket x tile matrix.
template <bool kRank>
__global__ __launch_bounds__(kBlock) void k_pkt_scatter(ShdPktCtx c, const ShdPkt* __restrict__ recs, size_t n,
                                                        uint64_t barrier, uint64_t end_time, uint64_t boot_end,
                                                        Bucketing bk, ShdDeliv* __restrict__ tmp,
                                                        uint8_t* __restrict__ status, uint32_t* __restrict__ cnt1,
                                                        unsigned long long* counters) {
    __shared__ uint32_t hist[kRank ? 1 : kMaxBuckets];
    __shared__ unsigned long long wmin[kBlock / 64];
    if (!kRank)
        for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock) hist[b] = 0;
    __syncthreads();
    unsigned long long mn = ~0ull;
    const size_t A = (size_t)c.A;
    const size_t base = (size_t)blockIdx.x * kTile;
    const uint2* __restrict__ host_info = reinterpret_cast<const uint2*>(c.host_info);
    const ShdEntry* __restrict__ tab = c.tab;
    // kBatch records per thread go through each gather level together, so a
    // wave keeps kBatch x 64 independent requests in flight per level
    for (int it0 = 0; it0 < kItems; it0 += kBatch) {
        ShdPkt p[kBatch];
        int si[kBatch], di[kBatch];
        size_t idx[kBatch];
        bool live[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            idx[k] = base + (size_t)(it0 + k) * kBlock + threadIdx.x;
            live[k] = idx[k] < n;
            if (live[k]) p[k] = recs[idx[k]];
        }
        uint32_t ts[kBatch], td[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const bool known = live[k] && p[k].src_host < c.nhosts && p[k].dst_host < c.nhosts;
            const uint2 hs = known ? host_info[p[k].src_host] : make_uint2(~0u, ~0u);
            const uint2 hd = known ? host_info[p[k].dst_host] : make_uint2(~0u, ~0u);
            si[k] = hs.x == ~0u ? -1 : (int)hs.x;
            di[k] = hd.x == ~0u ? -1 : (int)hd.x;
            ts[k] = hs.y;
            td[k] = hd.y;
        }
        size_t ei[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            int oi = si[k], oj = di[k];
            if (oi >= 0 && oj >= 0) {
                if (c.mode == 0) {
                    // owner({s,d}) = row touched first (topology.c:1189-1215, 1918-1968)
                    if (oi != oj && td[k] < ts[k]) oi = di[k], oj = si[k];
                } else if (c.mode == 2) {
                    const size_t b = (size_t)oi * A + (size_t)oj;
                    if (!((c.pair_bits[b >> 5] >> (b & 31)) & 1u)) oi = di[k], oj = si[k];
                }
            }
            ei[k] = (size_t)(oi < 0 ? 0 : oi) * A + (size_t)(oj < 0 ? 0 : oj);
        }
        ShdEntry e[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++)
            if (si[k] >= 0 && di[k] >= 0) e[k] = tab[ei[k]];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (!live[k]) continue;
            uint8_t st = 0xff; // unregistered host: not delivered
            if (si[k] >= 0 && di[k] >= 0) {
                uint32_t rs = p[k].rng_state;
                const double chance = (double)glibc_rand_r(&rs) / 2147483647.0; // random_nextDouble
                st = SHD_DROPPED_LOSS;
                if (p[k].now < boot_end || chance <= e[k].rel || p[k].payload_len == 0) { // worker.c:545
                    uint64_t t = p[k].now + (uint64_t)ceil(e[k].lat * 1000000.0);     // worker.c:548-549
                    if (t >= end_time) {                                              // scheduler.c:236-239
                        st = SHD_DROPPED_END;
                    } else {
                        if (p[k].src_host != p[k].dst_host && t < barrier) t = barrier; // host_single.c:187-192
                        st = SHD_DELIVERED;
                        uint32_t rank = 0;
                        if (kRank) rank = atomicAdd(&cnt1[p[k].dst_host], 1u);
                        else atomicAdd(&hist[(p[k].dst_host - bk.host_lo) >> bk.shift], 1u); // LDS
                        tmp[idx[k]] = ShdDeliv{t, p[k].seq, p[k].src_host, p[k].dst_host, (uint32_t)idx[k], rank};
                        if (t >= barrier && t < mn) mn = t; // worker.c:350-363
                    }
                }
            }
            status[idx[k]] = st;
        }
    }
    mn = wave_min_u64(mn);
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (!kRank)
        for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock) cnt1[(size_t)b * bk.ntiles + blockIdx.x] = hist[b];
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int k = 1; k < kBlock / 64; k++) m = wmin[k] < m ? wmin[k] : m;
        if (m != ~0ull) atomicMin(&counters[1], m); // one per workgroup
    }
}

// Regroup path (events already decided, e.g. after the multi-GPU exchange).
__global__ __launch_bounds__(kBlock) void k_hist_tiles(const ShdDeliv* __restrict__ in, size_t n, Bucketing bk,
                                                       uint32_t* __restrict__ cnt1) {
    __shared__ uint32_t hist[kMaxBuckets];
    for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock) hist[b] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kTile;
    for (int it = 0; it < kItems; it++) {
        const size_t i = base + (size_t)it * kBlock + threadIdx.x;
        if (i >= n) break;
        const uint32_t d = in[i].dst_host - bk.host_lo;
        if (d < bk.H) atomicAdd(&hist[d >> bk.shift], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock) cnt1[(size_t)b * bk.ntiles + blockIdx.x] = hist[b];
}

// ---- exclusive scan of u32 counts: out[k] = sum(in[0..k)), out[len] = total ----

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

__global__ __launch_bounds__(256) void k_scan_local(const uint32_t* __restrict__ in, size_t len,
                                                    uint32_t* __restrict__ out, uint32_t* __restrict__ bsum) {
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * 16;
    uint32_t v[16], s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        v[k] = (base + k < len) ? in[base + k] : 0u;
        s += v[k];
    }
    uint32_t total;
    uint32_t pre = block_excl_scan(s, &total);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if (base + k < len) out[base + k] = pre;
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

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* __restrict__ out, size_t len,
                                                  const uint32_t* __restrict__ bsum, uint32_t nb,
                                                  unsigned long long* counters) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) out[i] += bsum[i / kScanTile];
    if (i == 0) {
        out[len] = bsum[nb];
        if (counters) counters[0] = bsum[nb];
    }
}

// ---- level 1: tile -> bucket regions (LDS ranks, no global atomics) ----
// One workgroup covers kGroup consecutive scatter tiles: a bucket's offsets
// are contiguous across consecutive tiles of the (bucket-major) scan, so the
// first tile's offset is the group's base and runs get kGroup x longer.
__global__ __launch_bounds__(kPartBlock) void k_part1(const ShdDeliv* __restrict__ in,
                                                      const uint8_t* __restrict__ status, size_t n, Bucketing bk,
                                                      const uint32_t* __restrict__ off1,
                                                      ShdDeliv* __restrict__ stage) {
    __shared__ uint32_t base[kMaxBuckets];
    __shared__ uint32_t cur[kMaxBuckets];
    const uint32_t t0 = blockIdx.x * kGroup;
    for (uint32_t b = threadIdx.x; b < bk.nb; b += kPartBlock) {
        base[b] = off1[(size_t)b * bk.ntiles + t0];
        cur[b] = 0;
    }
    __syncthreads();
    const size_t tb = (size_t)t0 * kTile;
    constexpr int kPartItems = kGroup * kTile / kPartBlock;
    for (int it0 = 0; it0 < kPartItems; it0 += kBatch) {
        ShdDeliv r[kBatch];
        bool ok[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const size_t i = tb + (size_t)(it0 + k) * kPartBlock + threadIdx.x;
            ok[k] = i < n && (!status || status[i] == SHD_DELIVERED);
            if (ok[k]) r[k] = in[i];
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const uint32_t d = r[k].dst_host - bk.host_lo;
            if (!ok[k] || d >= bk.H) continue;
            const uint32_t b = d >> bk.shift;
            stage[base[b] + atomicAdd(&cur[b], 1u)] = r[k];
        }
    }
}

// ---- level 2 + segment sort ----

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
__device__ void wave_sort_segment(const ShdDeliv* __restrict__ src, uint32_t b, uint32_t n, uint32_t d,
                                  ShdDeliv* __restrict__ out, int lane) {
    Ev v[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        if (i < n) {
            const ShdDeliv r = src[b + i];
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
                    // the lower slot keeps the min when ascending, the max when descending
                    const bool take_o = (lower == up) ? ev_lt(o, v[e]) : ev_lt(v[e], o);
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

// One workgroup per level-1 bucket (<= kMaxBuckets destinations): per-
// destination histogram and offsets in LDS, LDS-ranked placement into
// stage2 (the bucket's region, L2/MALL-resident), then the segments are
// sorted by the workgroup's waves straight into the output.
__global__ __launch_bounds__(kSortBlock) void k_part2_sort(const ShdDeliv* __restrict__ stage1,
                                                           ShdDeliv* __restrict__ stage2, Bucketing bk,
                                                           const uint32_t* __restrict__ off1,
                                                           uint32_t* __restrict__ offsets,
                                                           ShdDeliv* __restrict__ out, uint32_t* __restrict__ big,
                                                           uint32_t* __restrict__ nbig) {
    __shared__ uint32_t cnt[kMaxBuckets];
    __shared__ uint32_t loc[kMaxBuckets];
    __shared__ uint32_t cur[kMaxBuckets];
    __shared__ uint32_t wsum[kSortBlock / 64];
    const uint32_t b = blockIdx.x;
    const uint32_t per = 1u << bk.shift;
    const uint32_t d0 = b << bk.shift;                   // first destination (range-relative)
    const uint32_t nd = min(per, bk.H - d0);             // destinations in this bucket
    const uint32_t s = off1[(size_t)b * bk.ntiles];      // bucket region [s, e)
    const uint32_t e = off1[(size_t)(b + 1) * bk.ntiles];
    for (uint32_t j = threadIdx.x; j < nd; j += kSortBlock) cnt[j] = 0, cur[j] = 0;
    __syncthreads();
    for (uint32_t k0 = s + threadIdx.x; k0 < e; k0 += kSortBlock * kStream) {
        uint32_t dd[kStream];
#pragma unroll
        for (int q = 0; q < kStream; q++) {
            const uint32_t k = k0 + (uint32_t)q * kSortBlock;
            dd[q] = k < e ? stage1[k].dst_host : ~0u;
        }
#pragma unroll
        for (int q = 0; q < kStream; q++)
            if (dd[q] != ~0u) atomicAdd(&cnt[dd[q] - bk.host_lo - d0], 1u);
    }
    __syncthreads();
    // exclusive scan of cnt[0..nd) (nd <= 1024): two values per thread
    {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const uint32_t j0 = 2 * threadIdx.x, j1 = j0 + 1;
        const uint32_t a0 = j0 < nd ? cnt[j0] : 0u, a1 = j1 < nd ? cnt[j1] : 0u;
        const uint32_t inc = wave_incl_scan(a0 + a1, lane);
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t pre = 0;
        for (int k = 0; k < w; k++) pre += wsum[k];
        pre += inc - (a0 + a1);
        if (j0 < nd) loc[j0] = pre;
        if (j1 < nd) loc[j1] = pre + a0;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nd; j += kSortBlock) offsets[d0 + j] = s + loc[j];
    if (b == gridDim.x - 1 && threadIdx.x == 0) offsets[bk.H] = e;
    for (uint32_t k0 = s + threadIdx.x; k0 < e; k0 += kSortBlock * kStream) {
        ShdDeliv r[kStream];
#pragma unroll
        for (int q = 0; q < kStream; q++) {
            const uint32_t k = k0 + (uint32_t)q * kSortBlock;
            if (k < e) r[q] = stage1[k];
        }
#pragma unroll
        for (int q = 0; q < kStream; q++) {
            if (k0 + (uint32_t)q * kSortBlock >= e) break;
            const uint32_t j = r[q].dst_host - bk.host_lo - d0;
            stage2[s + loc[j] + atomicAdd(&cur[j], 1u)] = r[q];
        }
    }
    __syncthreads(); // workgroup-scope release/acquire: stage2 writes visible to the sorting waves
    const int lane = threadIdx.x & 63;
    for (uint32_t j = threadIdx.x >> 6; j < nd; j += kSortBlock / 64) {
        const uint32_t n = cnt[j], o = s + loc[j], dh = bk.host_lo + d0 + j;
        if (n == 0) continue;
        if (n <= 64) wave_sort_segment<1>(stage2, o, n, dh, out, lane);
        else if (n <= 128) wave_sort_segment<2>(stage2, o, n, dh, out, lane);
        else if (n <= (uint32_t)kSmallSeg) wave_sort_segment<4>(stage2, o, n, dh, out, lane);
        else if (lane == 0) big[atomicAdd(nbig, 1u)] = d0 + j;
    }
}

__device__ __forceinline__ bool ev_less(const ShdDeliv& a, const ShdDeliv& b) {
    if (a.time != b.time) return a.time < b.time;
    if (a.src_host != b.src_host) return a.src_host < b.src_host;
    return a.seq < b.seq;
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
__global__ __launch_bounds__(256) void k_segsort_big(const ShdDeliv* __restrict__ stage2,
                                                     const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ big, const uint32_t* __restrict__ nbig,
                                                     ShdDeliv* __restrict__ out) {
    const uint32_t nb = *nbig;
    for (uint32_t q = blockIdx.x; q < nb; q += gridDim.x) {
        const uint32_t d = big[q];
        const uint32_t b = off[d], n = off[d + 1] - b;
        ShdDeliv* v = out + b;
        for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
            ShdDeliv r = stage2[b + k];
            r.pad = 0;
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

// ---- "rank" pipeline: per-destination counters, atomic-free placement ----

// Regroup path: rank of each event inside its destination (counter old value).
__global__ __launch_bounds__(256) void k_hist_rank(const ShdDeliv* __restrict__ in, size_t n, uint32_t host_lo,
                                                   uint32_t H, uint32_t* __restrict__ cnt, uint32_t* __restrict__ rank) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t d = in[i].dst_host - host_lo; // out-of-range events are dropped
        rank[i] = d < H ? atomicAdd(&cnt[d], 1u) : ~0u;
    }
}

// Each event goes to off[dst] + its rank (pad, or rank[] on the regroup path).
__global__ __launch_bounds__(256) void k_place_rank(const ShdDeliv* __restrict__ in, const uint8_t* __restrict__ status,
                                                    const uint32_t* __restrict__ rank, size_t n, uint32_t host_lo,
                                                    uint32_t H, const uint32_t* __restrict__ off,
                                                    ShdDeliv* __restrict__ scr) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * kBatch) {
        ShdDeliv r[kBatch];
        uint32_t rk[kBatch];
        bool ok[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const size_t i = i0 + (size_t)k * stride;
            ok[k] = i < n && (!status || status[i] == SHD_DELIVERED);
            if (ok[k]) {
                r[k] = in[i];
                rk[k] = rank ? rank[i] : r[k].pad;
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const uint32_t d = r[k].dst_host - host_lo;
            if (ok[k] && d < H) scr[off[d] + rk[k]] = r[k];
        }
    }
}

// One wave per destination segment of up to kSmallSeg events; larger ones go
// to the bitonic-in-HBM list.
__global__ __launch_bounds__(256) void k_segsort_dst(const ShdDeliv* __restrict__ scr, const uint32_t* __restrict__ off,
                                                     uint32_t H, uint32_t host_lo, ShdDeliv* __restrict__ out,
                                                     uint32_t* __restrict__ big, uint32_t* __restrict__ nbig) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t d = wave; d < H; d += nwaves) {
        const uint32_t b = off[d], n = off[d + 1] - b;
        const uint32_t dh = d + host_lo;
        if (n == 0) continue;
        if (n <= 64) wave_sort_segment<1>(scr, b, n, dh, out, lane);
        else if (n <= 128) wave_sort_segment<2>(scr, b, n, dh, out, lane);
        else if (n <= (uint32_t)kSmallSeg) wave_sort_segment<4>(scr, b, n, dh, out, lane);
        else if (lane == 0) big[atomicAdd(nbig, 1u)] = d;
    }
}

// ---- workspace (grow-only, per process / device) ----
struct Ws {
    size_t cap_n = 0;
    ShdDeliv* tmp = nullptr;
    ShdDeliv* st1 = nullptr;
    ShdDeliv* st2 = nullptr;
    size_t cap_m = 0; // bucket x tile matrix
    uint32_t* cnt1 = nullptr;
    uint32_t* off1 = nullptr;
    uint32_t* bsum = nullptr;
    uint32_t cap_h = 0;
    uint32_t* big = nullptr;
    uint32_t* nbig = nullptr;
    uint32_t* rnk = nullptr; // per-event rank, regroup path of the rank pipeline
};
Ws g_ws;

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

int ws_reserve(size_t n, size_t m, uint32_t H) {
    int rc = 0;
    if (n > g_ws.cap_n) {
        (void)hipFree(g_ws.tmp);
        (void)hipFree(g_ws.st1);
        (void)hipFree(g_ws.st2);
        (void)hipFree(g_ws.rnk);
        g_ws.tmp = g_ws.st1 = g_ws.st2 = nullptr;
        g_ws.rnk = nullptr;
        g_ws.cap_n = 0;
        const size_t cap = n + n / 8 + 1024;
        if ((rc = hip_status(hipMalloc((void**)&g_ws.tmp, sizeof(ShdDeliv) * cap), "hipMalloc ws.tmp")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.st1, sizeof(ShdDeliv) * cap), "hipMalloc ws.st1")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.st2, sizeof(ShdDeliv) * cap), "hipMalloc ws.st2")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.rnk, sizeof(uint32_t) * cap), "hipMalloc ws.rnk")))
            return rc;
        g_ws.cap_n = cap;
    }
    if (m + 1 > g_ws.cap_m) {
        (void)hipFree(g_ws.cnt1);
        (void)hipFree(g_ws.off1);
        (void)hipFree(g_ws.bsum);
        g_ws.cap_m = 0;
        const size_t cap = m + 1 + (m >> 3) + 4096;
        if ((rc = hip_status(hipMalloc((void**)&g_ws.cnt1, 4 * cap), "hipMalloc ws.cnt1")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.off1, 4 * cap), "hipMalloc ws.off1")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.bsum, 4 * (cap / kScanTile + 2)), "hipMalloc ws.bsum")))
            return rc;
        g_ws.cap_m = cap;
    }
    if (H + 1 > g_ws.cap_h) {
        (void)hipFree(g_ws.big);
        (void)hipFree(g_ws.nbig);
        g_ws.cap_h = 0;
        const uint32_t cap = H + 1 + 1024;
        if ((rc = hip_status(hipMalloc((void**)&g_ws.big, 4ull * cap), "hipMalloc ws.big")) ||
            (rc = hip_status(hipMalloc((void**)&g_ws.nbig, 16), "hipMalloc ws.nbig")))
            return rc;
        g_ws.cap_h = cap;
    }
    return 0;
}

Bucketing make_bucketing(uint32_t host_lo, uint32_t H, size_t n) {
    Bucketing bk;
    bk.host_lo = host_lo;
    bk.H = H;
    bk.shift = 7; // 128 destinations per bucket, up to kMaxBuckets buckets
    while (((size_t)H + (1u << bk.shift) - 1) >> bk.shift > (size_t)kMaxBuckets) bk.shift++;
    bk.nb = (uint32_t)(((size_t)H + (1u << bk.shift) - 1) >> bk.shift);
    if (bk.nb == 0) bk.nb = 1;
    bk.ntiles = (uint32_t)((n + kTile - 1) / kTile);
    if (bk.ntiles == 0) bk.ntiles = 1;
    return bk;
}

unsigned grid_for(size_t n, unsigned block, unsigned cap) {
    size_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

// ---- optional per-stage timing with HIP events on the launch stream ----
constexpr int kStages = 4; // 0 packet-scatter, 1 scan, 2 level-1 partition, 3 level-2 + segment sort
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

// scan + partition + segment sort, shared by both entry points
int group_and_sort(const ShdDeliv* in, const uint8_t* status, size_t n, const Bucketing& bk, ShdDeliv* out,
                   uint32_t* offsets, unsigned long long* counters, hipStream_t s) {
    const size_t m = (size_t)bk.nb * bk.ntiles;
    const uint32_t nb = (uint32_t)((m + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(k_scan_local, dim3(nb ? nb : 1), dim3(256), 0, s, g_ws.cnt1, m, g_ws.off1, g_ws.bsum);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, g_ws.bsum, nb);
    hipLaunchKernelGGL(k_scan_add, dim3(grid_for(m + 1, 256, 1u << 30)), dim3(256), 0, s, g_ws.off1, m, g_ws.bsum,
                       nb, counters);
    mark(2, s);
    hipLaunchKernelGGL(k_part1, dim3((bk.ntiles + kGroup - 1) / kGroup), dim3(kPartBlock), 0, s, in, status, n, bk,
                       g_ws.off1, g_ws.st1);
    mark(3, s);
    hipLaunchKernelGGL(k_part2_sort, dim3(bk.nb), dim3(kSortBlock), 0, s, g_ws.st1, g_ws.st2, bk, g_ws.off1,
                       offsets, out, g_ws.big, g_ws.nbig);
    hipLaunchKernelGGL(k_segsort_big, dim3(64), dim3(256), 0, s, g_ws.st2, offsets, g_ws.big, g_ws.nbig, out);
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    return hip_status(hipGetLastError(), "group_and_sort launch");
}

// scan of per-destination counts straight into the offsets, atomic-free
// placement by rank, one wave per destination segment
int group_and_sort_rank(const ShdDeliv* in, const uint8_t* status, const uint32_t* rank, size_t n,
                        uint32_t host_lo, uint32_t H, ShdDeliv* out, uint32_t* offsets,
                        unsigned long long* counters, hipStream_t s) {
    const uint32_t nb = (uint32_t)((H + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(k_scan_local, dim3(nb ? nb : 1), dim3(256), 0, s, g_ws.cnt1, (size_t)H, offsets, g_ws.bsum);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, g_ws.bsum, nb);
    hipLaunchKernelGGL(k_scan_add, dim3(grid_for((size_t)H + 1, 256, 1u << 30)), dim3(256), 0, s, offsets, (size_t)H,
                       g_ws.bsum, nb, counters);
    mark(2, s);
    if (n)
        hipLaunchKernelGGL(k_place_rank, dim3(grid_for(n, 256 * kBatch, 1u << 20)), dim3(256), 0, s, in, status, rank,
                           n, host_lo, H, offsets, g_ws.st1);
    mark(3, s);
    hipLaunchKernelGGL(k_segsort_dst, dim3(grid_for(H, 4, 16384)), dim3(256), 0, s, g_ws.st1, offsets, H, host_lo,
                       out, g_ws.big, g_ws.nbig);
    hipLaunchKernelGGL(k_segsort_big, dim3(64), dim3(256), 0, s, g_ws.st1, offsets, g_ws.big, g_ws.nbig, out);
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    return hip_status(hipGetLastError(), "group_and_sort_rank launch");
}

// SHD_PACKET_PIPELINE=bucket selects the two-level bucket partition;
// anything else the per-destination rank pipeline.
bool use_rank_pipeline() {
    const char* v = getenv("SHD_PACKET_PIPELINE");
    return !(v && strcmp(v, "bucket") == 0);
}

} // namespace

extern "C" int shd_dev_packet_round(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                                    uint64_t end_time, uint64_t bootstrap_end, ShdDeliv* d_out,
                                    uint32_t* d_dst_offsets, uint8_t* d_status, uint64_t* d_counters, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const uint32_t H = c->nhosts;
    const bool rk = use_rank_pipeline();
    const Bucketing bk = make_bucketing(0, H, n);
    const size_t m = rk ? (size_t)H : (size_t)bk.nb * bk.ntiles;
    int rc = ws_reserve(n, m, H);
    if (rc) return rc;
    unsigned long long* counters = (unsigned long long*)d_counters;
    if ((rc = hip_status(hipMemsetAsync(g_ws.nbig, 0, 4, s), "memset nbig")) ||
        (rc = hip_status(hipMemsetAsync(counters, 0xff, 16, s), "memset counters")))
        return rc;
    // rank: per-destination counters start at zero; bucket: every tile writes
    // its whole histogram column, only an empty batch needs zeros
    if ((rk || !n) && (rc = hip_status(hipMemsetAsync(g_ws.cnt1, 0, 4 * m, s), "memset cnt1"))) return rc;
    mark(0, s);
    if (n) {
        if (rk)
            hipLaunchKernelGGL(k_pkt_scatter<true>, dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier,
                               end_time, bootstrap_end, bk, g_ws.tmp, d_status, g_ws.cnt1, counters);
        else
            hipLaunchKernelGGL(k_pkt_scatter<false>, dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier,
                               end_time, bootstrap_end, bk, g_ws.tmp, d_status, g_ws.cnt1, counters);
    }
    mark(1, s);
    if ((rc = hip_status(hipGetLastError(), "k_pkt_scatter launch"))) return rc;
    rc = rk ? group_and_sort_rank(g_ws.tmp, d_status, nullptr, n, 0, H, d_out, d_dst_offsets, counters, s)
            : group_and_sort(g_ws.tmp, d_status, n, bk, d_out, d_dst_offsets, counters, s);
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
    const bool rk = use_rank_pipeline();
    const Bucketing bk = make_bucketing(host_lo, H, n);
    const size_t m = rk ? (size_t)H : (size_t)bk.nb * bk.ntiles;
    int rc = ws_reserve(n, m, H);
    if (rc) return rc;
    if ((rc = hip_status(hipMemsetAsync(g_ws.nbig, 0, 4, s), "memset nbig"))) return rc;
    if ((rk || !n) && (rc = hip_status(hipMemsetAsync(g_ws.cnt1, 0, 4 * m, s), "memset cnt1"))) return rc;
    mark(0, s);
    if (n) {
        if (rk)
            hipLaunchKernelGGL(k_hist_rank, dim3(grid_for(n, 256, 1u << 20)), dim3(256), 0, s, d_in, n, host_lo, H,
                               g_ws.cnt1, g_ws.rnk);
        else
            hipLaunchKernelGGL(k_hist_tiles, dim3(bk.ntiles), dim3(kBlock), 0, s, d_in, n, bk, g_ws.cnt1);
    }
    mark(1, s);
    rc = rk ? group_and_sort_rank(d_in, nullptr, g_ws.rnk, n, host_lo, H, d_out, d_dst_offsets, nullptr, s)
            : group_and_sort(d_in, nullptr, n, bk, d_out, d_dst_offsets, nullptr, s);
    if (rc) return rc;
    return stream ? 0 : hip_status(hipStreamSynchronize(s), "deliv sort");
}
