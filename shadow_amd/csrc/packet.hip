// packet.hip -- the per-round inter-host packet hand-off on gfx950
// (reference core/worker.c:517-576,
// core/scheduler/scheduler.c:232-255, scheduler_policy_host_single.c:174-220,
// core/work/event.c:109-152, utility/random.c:32-43).
//
// Pipeline over one round's batch (device-resident, one stream): the default
// is "part" (k_part_scatter + k_part_sort, below); the earlier default
// "slab" (SHD_PACKET_PIPELINE=slab), which the regroup after an exchange and
// the exchanged round's sender side still use:
//   k_pkt_scatter<2> per record: host->slot gathers, owner resolution of the
//                  reference cache (touch order / pair bits), 16 B table
//                  gather, the sender's reserved rand_r draw, drop rule,
//                  ceil(lat * 1e6) delay, end-time drop, barrier clamp; the
//                  event's slot = old value of its destination's counter, and
//                  the event goes straight to slab[dst * kSlab + slot] (slots
//                  >= kSlab to an overflow list).  The roofline is quoted on
//                  this kernel.
//   k_scan_*       exclusive scan of the per-destination counts -> offsets.
//   k_place_ovf    overflow events only (grid-stride over a device count).
//   k_segsort_dst  one wave per destination: register rank sort of its slab
//                  by (time, src host, srcHostEventID), written at off[dst].
//   k_segsort_mid  listed segments (> 256 events): 4096-event runs, LDS bitonic, one
//                  workgroup each (a segment up to 4096 events is one run).
//   k_segsort_merge  segments above 4096 events: merge-path passes over the runs,
//                  tiles claimed by persistent workgroups (skewed destinations).
// Alternatives, all bit-exact and parity-tested: "rank" (events in record
// order, then k_place_rank over the whole batch) and "bucket" (LDS
// histograms over destination buckets, k_place_bucket, k_bucket_sort; no
// global atomics).  The multi-GPU regroup (shd_dev_deliv_sort) uses the same
// pipelines (k_hist_slab / k_hist_rank / k_hist_tiles).
// event_compare is a total order, so per-destination heap pop order
// (priority_queue.c) equals this sorted order: the output is identical to
// pushing every event into its destination's queue.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "shd_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kBatch = 4;          // records per thread in flight through the gather chain
constexpr int kChunks = 1536;      // scatter workgroups per launch (columns of the count matrix);
                                   // 1.5 per CU at 4 waves each = 24 of the 20..32 resident waves a
                                   // CU holds at 88 VGPRs, tails of small chunks overlap better
                                   // than 1024 (profiles/r02s_chunks.log: -1% round time)
constexpr int kMaxBuckets = 4096;  // destination buckets (LDS histogram size)
constexpr int kScanTile = 4096;    // 256 threads x 16
constexpr int kSmallSeg = 256;     // wave register sort up to 4 events per lane
constexpr uint32_t kSlab = 128; // "slab" pipeline: event slots reserved per destination
constexpr int kSortBlock = 1024;   // k_bucket_sort workgroup (16 waves)
constexpr int kMaxPerBucket = 2 * kSortBlock; // destinations per bucket (LDS scan width)
constexpr int kBucketCap = 4096;   // events per bucket staged in LDS by k_bucket_sort (30 B each)
constexpr int kBucketLoads = 4;    // events in flight per thread while staging a bucket
constexpr int kStream = 8;         // loads in flight per thread in the streaming passes
constexpr int kPlaceBlock = 256;
constexpr int kStageBlock = 256;   // staged partition passes (block_excl_scan width)
constexpr int kStageItems = 4;
constexpr int kStageTile = kStageBlock * kStageItems; // events staged in LDS per step
constexpr int kMaxParts = 64;      // pass-1 fan-out limit (np <= kMaxParts - 1)
constexpr uint32_t kPartsTarget = 32;
// stage guards of a round (nbig[2], folded into the merge fault word's bits
// 24..30 by k_segsort_mid): overflow event outside its segment, overflow
// count above the list, big-segment list full, offsets above the staging area
enum : uint32_t { kFaultOvfRange = 1u, kFaultOvfCap = 2u, kFaultBigCap = 4u, kFaultOff = 8u };

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

// 32-byte records move as two aligned 16-byte accesses (hipMalloc'd arrays of
// 32-byte structs; the compiler otherwise splits them at 8-byte alignment,
// e.g. into overlapping dwordx4 pairs at offsets 0 and 12).
__device__ __forceinline__ ShdDeliv ld_ev(const ShdDeliv* p) {
    const uint4* q = reinterpret_cast<const uint4*>(__builtin_assume_aligned(p, 16));
    const uint4 a = q[0], b = q[1];
    ShdDeliv r;
    r.time = ((unsigned long long)a.y << 32) | a.x;
    r.seq = ((unsigned long long)a.w << 32) | a.z;
    r.src_host = b.x;
    r.dst_host = b.y;
    r.pkt_index = b.z;
    r.pad = b.w;
    return r;
}
__device__ __forceinline__ void st_ev(ShdDeliv* p, const ShdDeliv& r) {
    uint4* q = reinterpret_cast<uint4*>(__builtin_assume_aligned(p, 16));
    q[0] = make_uint4((uint32_t)r.time, (uint32_t)(r.time >> 32), (uint32_t)r.seq, (uint32_t)(r.seq >> 32));
    q[1] = make_uint4(r.src_host, r.dst_host, r.pkt_index, r.pad);
}
__device__ __forceinline__ ShdPkt ld_pkt(const ShdPkt* p) {
    const uint4* q = reinterpret_cast<const uint4*>(__builtin_assume_aligned(p, 16));
    const uint4 a = q[0], b = q[1];
    ShdPkt r;
    r.now = ((unsigned long long)a.y << 32) | a.x;
    r.seq = ((unsigned long long)a.w << 32) | a.z;
    r.src_host = b.x;
    r.dst_host = b.y;
    r.rng_state = b.z;
    r.payload_len = b.w;
    return r;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o < v ? o : v;
    }
    return v;
}

// Partition geometry of one launch.  The batch is cut into `ntiles`
// contiguous chunks of `chunk` records, one scatter workgroup each; the
// destination range [host_lo, host_lo + H) into `nb` buckets of 2^shift
// hosts.  cnt1 / off1 are the bucket-major nb x ntiles count matrix and its
// exclusive scan: bucket b's region of the partitioned array (and of the
// output) starts at off1[b * ntiles].
struct Bucketing {
    uint32_t host_lo; // first host id of the range
    uint32_t H;       // hosts in range
    uint32_t shift;   // bucket = (dst - host_lo) >> shift
    uint32_t nb;      // number of buckets
    uint32_t ntiles;  // scatter workgroups (matrix columns)
    uint32_t chunk;   // records per scatter workgroup
    uint32_t xcd;     // 1: XCD-grouped column order (see col_of)
    uint32_t rsort;   // segment sort: 1 rank (default), 0 bitonic (see sort_segment)
    uint32_t slab_rm; // slab layout: 1 rank-major (slot r of host d at r * H + d), 0 host-major (d * kSlab + r)
    uint32_t agg;     // wave-aggregated destination slots (dest_slot); SHD_DEST_AGG=0 turns them off
    unsigned long long tbase; // compact slab records: delivery time - tbase in 32 bits (see CSlab)
};

// Matrix column of chunk g.  Workgroups are dealt to the 8 XCDs round-robin
// (g % 8, for speed only -- correctness never depends on it), so with the
// columns of one XCD's chunks adjacent, a bucket's consecutive runs are
// written through ONE XCD's L2 and its partly written lines fill up there
// instead of being written back piecewise from eight L2s.  A bijection of
// [0, ntiles) either way.
__device__ __forceinline__ uint32_t col_of(const Bucketing& bk, uint32_t g) {
    if (!bk.xcd) return g;
    const uint32_t q = bk.ntiles >> 3, r = bk.ntiles & 7, x = g & 7;
    return x * q + (x < r ? x : r) + (g >> 3);
}

// Per-destination slot counters, wave-aggregated.  Every lane that takes a
// slot hashes its destination to one of 64 per-wave LDS slots and writes its
// lane id there; the lanes whose slot holds a lane of the same destination
// form a group: one global atomic per group (by that lane) hands the group a
// base, and each member adds its rank inside the group (an LDS atomic).
// Lanes whose slot was taken by another destination add alone.  With
// uniform destinations every group has one member (a few LDS operations
// more per event); with a hot destination -- a popular server, Zipf -- its
// lanes share one atomic, where one per event serialised on one address.
// The slots a destination's events get are a permutation of [0, count) in
// any arrangement; the segment sort orders them.
struct DestAgg {
    uint32_t* owner; // [64] per wave
    uint32_t* cnt;   // [64] per wave, zero between uses
    uint32_t* base;  // [64] per wave
    uint32_t on;     // 0: one atomic per event (SHD_DEST_AGG=0)
};
__device__ __forceinline__ void agg_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// called by every lane of the wave (want: this lane takes a slot of d)
__device__ __forceinline__ uint32_t dest_slot(bool want, uint32_t d, uint32_t* __restrict__ gcnt, const DestAgg& a,
                                              int lane) {
    if (!a.on) return want ? atomicAdd(&gcnt[d], 1u) : 0u;
    const uint32_t slot = (d * 2654435761u) >> 26;
    if (want) a.owner[slot] = (uint32_t)lane;
    agg_fence();
    const uint32_t ol = want ? a.owner[slot] : (uint32_t)lane;
    const uint32_t od = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ol << 2), (int)d);
    const bool grp = want && od == d;
    uint32_t r = 0;
    if (grp) r = atomicAdd(&a.cnt[slot], 1u);
    agg_fence();
    if (grp && ol == (uint32_t)lane) {
        const uint32_t c = a.cnt[slot];
        a.base[slot] = atomicAdd(&gcnt[d], c);
        a.cnt[slot] = 0;
    }
    agg_fence();
    if (grp) return a.base[slot] + r;
    return want ? atomicAdd(&gcnt[d], 1u) : 0u;
}

// One atomic per wave for the lanes that want a slot of a shared counter
// (the slab overflow list: with a hot destination most of its events
// overflow, and one atomic per event on one address serialised them).
// Called by every lane; returns this lane's slot (want) or 0.
__device__ __forceinline__ uint32_t wave_alloc(bool want, uint32_t* counter, int lane) {
    const unsigned long long m = __ballot(want);
    if (!m) return 0u;
    const int first = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(counter, (uint32_t)__builtin_popcountll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, first);
    return base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
}

// Compact slab record (16 B, one store): {time - tbase, src host,
// pkt_index, srcHostEventID} when the time offset fits 32 bits (below the
// marker) and the srcHostEventID does (a host's event counter); otherwise the
// slot holds the marker and the event goes whole to the same slot of the
// 32-B slab.  Halves the bytes of the scatter's random store and of the sort's
// slab reads (9.2M events: 147 MB instead of 294 MB, inside the 256 MB
// Infinity Cache).  tbase = barrier - 2^31 ns: delays up to ~2.1 s past the
// barrier and self deliveries up to ~2.1 s before it are compact.
constexpr uint32_t kCMark = 0xFFFFFFFFu;
__device__ __forceinline__ bool c_fits(unsigned long long t, unsigned long long tbase, unsigned long long seq) {
    return t >= tbase && t - tbase < kCMark && seq <= 0xFFFFFFFFull;
}

// The round's path packet counter log (ShdPktCtx.plog): record i's key, the
// flat index of its answering pair, or all-ones when the packet was not kept
// (dropped by loss, or not decided here).  One coalesced store per record --
// 4 B (8 B for tables of 2^32 entries or more) instead of a memory-side
// atomic per kept packet: the atomics ran at the chip's ~25 G/s atomic rate
// (+0.365 ms on the 10M-packet round, k_part_scatter 0.43 -> 0.795 ms,
// profiles/r05b_pcnt_atomic_ab.log); the log is added into the dense counters
// in bulk (shd_dev_pcnt_fold).
__device__ __forceinline__ void pcnt_log(const ShdPktCtx& c, size_t i, bool kept, size_t key) {
    if (!c.plog) return;
    if (c.plog64)
        __builtin_nontemporal_store(kept ? (unsigned long long)key : ~0ull,
                                    static_cast<unsigned long long*>(c.plog) + i);
    else
        __builtin_nontemporal_store(kept ? (uint32_t)key : ~0u, static_cast<uint32_t*>(c.plog) + i);
}

// kMode 1 ("rank" pipeline): each delivered event takes its slot in its
// destination segment from a per-destination global counter (the counter's
// old value, carried in pad); cnt1 is then the per-destination count array.
// kMode 2 ("slab" pipeline, default): the same counter, but the event is
// written straight into its destination's slab of kSlab slots,
// tmp[dst * kSlab + slot]; slots >= kSlab go to the overflow list ovf
// (novf = its length), placed later by k_place_ovf.  No record-order copy
// and no placement pass over the whole batch.
// kMode 0 ("bucket" pipeline): the slot inside the (workgroup, bucket) run
// comes from the workgroup's LDS histogram (old value of an LDS atomic,
// carried in pad) -- no global atomics per event; cnt1 is the bucket x tile
// matrix.
// Packet-path table entry (shd_dev_ptab_build): {delay_ns, keep threshold}.
// keep_thr = max{r : (double)r / 2147483647.0 <= rel} over the 31-bit rand_r
// outputs, so `chance <= rel` (worker.c:545) is exactly `r <= keep_thr`, and
// delay_ns = (u64)ceil(lat * 1e6) (worker.c:548); an entry whose delay does
// not fit (or whose rel has no such r) holds kPtabFallback and is decided
// from the f64 entry.  8 B instead of 16: half the random-gather footprint.
constexpr uint32_t kPtabFallback = 0xFFFFFFFFu;

// kProbe (measurement only, SHD_SCATTER_PROBE; outputs are NOT the round's):
// 1 skips the table gather, 2 the host->slot gathers, 3 the event store,
// 4 the destination-slot atomic -- each stage's share of the kernel time.
// kNT: the table gather with the non-temporal (streaming) cache policy
// (default: the gathered lines are not re-read, and streaming them keeps the
// slab lines and the counters in the L2: scatter 0.597 vs 0.617 ms,
// profiles/r03nt_scatter_nt.log).  Measured and not kept there: streaming
// slab stores (0.80 ms: each 16-B store leaves the L2 as its own partial
// write), status stores (no change), record loads (+0.005 ms).
// SHD_SCATTER_NT=0 is the plain form.
typedef unsigned int shd_v4u __attribute__((ext_vector_type(4)));
template <int kMode, int kB = kBatch, int kProbe = 0, bool kNT = true>
__global__ __launch_bounds__(kBlock) void k_pkt_scatter(ShdPktCtx c, const ShdPkt* __restrict__ recs, size_t n,
                                                        uint64_t barrier, uint64_t end_time, uint64_t boot_end,
                                                        Bucketing bk, ShdDeliv* __restrict__ tmp,
                                                        uint8_t* __restrict__ status, uint32_t* __restrict__ cnt1,
                                                        unsigned long long* counters, ShdDeliv* __restrict__ ovf,
                                                        uint32_t* __restrict__ novf, uint4* __restrict__ cslab) {
    constexpr bool kRank = kMode != 0;
    __shared__ uint32_t hist[kRank ? 1 : kMaxBuckets];
    __shared__ unsigned long long wmin[kBlock / 64];
    __shared__ uint32_t agg_s[kRank ? 3 * kBlock : 1];
    const int lane = threadIdx.x & 63;
    const DestAgg agg{agg_s + 3 * (threadIdx.x & ~63u), agg_s + 3 * (threadIdx.x & ~63u) + 64,
                      agg_s + 3 * (threadIdx.x & ~63u) + 128, bk.agg};
    if (kRank) agg.cnt[lane] = 0;
    if (!kRank)
        for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock) hist[b] = 0;
    __syncthreads();
    unsigned long long mn = ~0ull;
    const size_t A = (size_t)c.A;
    const size_t beg = (size_t)blockIdx.x * bk.chunk;
    const size_t end = beg + bk.chunk < n ? beg + bk.chunk : n;
    const uint2* __restrict__ host_info = reinterpret_cast<const uint2*>(c.host_info);
    const ShdEntry* __restrict__ tab = c.tab;
    const uint2* __restrict__ ptab = reinterpret_cast<const uint2*>(c.ptab);
    // kB records per thread go through each gather level together, so a
    // wave keeps kB x 64 independent requests in flight per level
    for (size_t b0 = beg; b0 < end; b0 += (size_t)kBlock * kB) {
        ShdPkt p[kB];
        int si[kB], di[kB];
        size_t idx[kB];
        bool live[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            idx[k] = b0 + (size_t)k * kBlock + threadIdx.x;
            live[k] = idx[k] < end;
            if (live[k]) p[k] = ld_pkt(&recs[idx[k]]);
        }
        uint32_t ts[kB], td[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const bool known = live[k] && p[k].src_host < c.nhosts && p[k].dst_host < c.nhosts;
            uint2 hs = make_uint2(~0u, ~0u), hd = make_uint2(~0u, ~0u);
            if (kProbe == 2) {
                if (known) hs = make_uint2(p[k].src_host % c.A, 0u), hd = make_uint2(p[k].dst_host % c.A, 1u);
            } else if (known) {
                hs = host_info[p[k].src_host];
                hd = host_info[p[k].dst_host];
            }
            si[k] = hs.x == ~0u ? -1 : (int)hs.x;
            di[k] = hd.x == ~0u ? -1 : (int)hd.x;
            ts[k] = hs.y;
            td[k] = hd.y;
        }
        size_t ei[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
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
            // a row-sharded table holds rows [row_lo, row_hi) only: a record
            // answered by another rank's row is not decided here (status 0xff)
            if (oi < c.row_lo || oi >= c.row_hi) si[k] = -1;
            ei[k] = (size_t)(oi < 0 ? 0 : oi) * A + (size_t)(oj < 0 ? 0 : oj);
        }
        ShdEntry e[kB];
        uint2 q[kB];
        if (ptab) { // (uniform) the 8-B packet-path table
#pragma unroll
            for (int k = 0; k < kB; k++) {
                q[k] = make_uint2(kPtabFallback, 0u);
                if (si[k] >= 0 && di[k] >= 0) {
                    if (kProbe == 1) q[k] = ptab[(ei[k] & 1023u) + (size_t)c.row_lo * A];
                    else if (kNT) {
                        const unsigned long long v =
                            __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(ptab) + ei[k]);
                        q[k] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                    } else q[k] = ptab[ei[k]];
                }
            }
#pragma unroll
            for (int k = 0; k < kB; k++) // entries that do not fit the 8-B form (none on the bench graphs)
                if (si[k] >= 0 && di[k] >= 0 && q[k].x == kPtabFallback) e[k] = tab[ei[k]];
        } else {
#pragma unroll
            for (int k = 0; k < kB; k++)
                if (si[k] >= 0 && di[k] >= 0) e[k] = kProbe == 1 ? tab[(ei[k] & 1023u) + (size_t)c.row_lo * A] : tab[ei[k]];
        }
        uint8_t st[kB];
        uint64_t tt[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            st[k] = 0xff; // unregistered host: not delivered
            tt[k] = 0;
            if (live[k] && si[k] >= 0 && di[k] >= 0) {
                uint32_t rs = p[k].rng_state;
                const uint32_t r = (uint32_t)glibc_rand_r(&rs);
                bool keep;
                uint64_t delay;
                if (ptab && q[k].x != kPtabFallback) {
                    keep = r <= q[k].y; // == (chance <= rel), see kPtabFallback
                    delay = q[k].x;
                } else {
                    const double chance = (double)r / 2147483647.0; // random_nextDouble
                    keep = chance <= e[k].rel;
                    delay = (uint64_t)ceil(e[k].lat * 1000000.0);
                }
                st[k] = SHD_DROPPED_LOSS;
                if (p[k].now < boot_end || keep || p[k].payload_len == 0) { // worker.c:545
                    uint64_t t = p[k].now + delay;                          // worker.c:548-549
                    if (t >= end_time) {                                              // scheduler.c:236-239
                        st[k] = SHD_DROPPED_END;
                    } else {
                        if (p[k].src_host != p[k].dst_host && t < barrier) t = barrier; // host_single.c:187-192
                        st[k] = SHD_DELIVERED;
                        tt[k] = t;
                    }
                    // topology_incrementPathPacketCounter (worker.c:551): every kept packet,
                    // before the end-time drop, at its answering pair
                    if (c.pcnt) atomicAdd(c.pcnt + ei[k], 1u);
                }
            }
            if (live[k]) pcnt_log(c, idx[k], st[k] == SHD_DELIVERED || st[k] == SHD_DROPPED_END, ei[k]);
        }
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const bool dl = st[k] == SHD_DELIVERED;
            uint32_t rank = 0;
            if (kProbe == 4) rank = dl ? (uint32_t)(idx[k] & 127u) : 0u;
            else if (kRank) rank = dest_slot(dl, p[k].dst_host, cnt1, agg, lane); // (every lane: wave-level groups)
            const uint32_t oslot = kMode == 2 ? wave_alloc(dl && rank >= kSlab, novf, lane) : 0u;
            if (dl) {
                const uint64_t t = tt[k];
                if (!kRank) rank = atomicAdd(&hist[(p[k].dst_host - bk.host_lo) >> bk.shift], 1u); // LDS
                const ShdDeliv ev{t, p[k].seq, p[k].src_host, p[k].dst_host, (uint32_t)idx[k] + c.idx_base, rank};
                if (kProbe == 3) {
                } else if (kMode < 2) st_ev(&tmp[idx[k]], ev);
                else if (rank < kSlab) {
                    const size_t sl = bk.slab_rm ? (size_t)rank * bk.H + p[k].dst_host
                                                 : (size_t)p[k].dst_host * kSlab + rank;
                    if (!cslab) {
                        st_ev(&tmp[sl], ev);
                    } else if (c_fits(t, bk.tbase, p[k].seq)) {
                        cslab[sl] = make_uint4((uint32_t)(t - bk.tbase), p[k].src_host, ev.pkt_index, (uint32_t)p[k].seq);
                    } else {
                        cslab[sl] = make_uint4(kCMark, 0u, 0u, 0u);
                        st_ev(&tmp[sl], ev);
                    }
                } else st_ev(&ovf[oslot], ev); // segments above kSlab
                if (t >= barrier && t < mn) mn = t; // worker.c:350-363
            }
            if (live[k]) status[idx[k]] = st[k];
        }
    }
    mn = wave_min_u64(mn);
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (!kRank)
        for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock)
            cnt1[(size_t)b * bk.ntiles + col_of(bk, blockIdx.x)] = hist[b];
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int k = 1; k < kBlock / 64; k++) m = wmin[k] < m ? wmin[k] : m;
        if (m != ~0ull) atomicMin(&counters[1], m); // one per workgroup
    }
}

// The round's resets: nbig[0..2] (big-segment count, overflow count, fault
// word) = 0, counters[0..1] = ~0 (the min-time slots), cnt1[0..m) = 0.
__global__ __launch_bounds__(256) void k_round_init(uint32_t* __restrict__ nbig, unsigned long long* __restrict__ counters,
                                                    uint32_t* __restrict__ cnt1, uint32_t m,
                                                    unsigned long long* __restrict__ minw2 = nullptr) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 3) nbig[t] = 0u;
    else if (t < 5) counters[t - 3] = ~0ull;
    else if (t == 5 && minw2) minw2[1] = ~0ull;
    for (uint32_t i = t; i < m; i += gridDim.x * blockDim.x) cnt1[i] = 0u;
}

// Regroup path (events already decided, e.g. after the multi-GPU exchange):
// per-chunk bucket histogram; rank[i] = the event's slot in its
// (chunk, bucket) run, ~0u for events outside the host range.
__global__ __launch_bounds__(kBlock) void k_hist_tiles(const ShdDeliv* __restrict__ in, size_t n, Bucketing bk,
                                                       uint32_t* __restrict__ cnt1, uint32_t* __restrict__ rank) {
    __shared__ uint32_t hist[kMaxBuckets];
    for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock) hist[b] = 0;
    __syncthreads();
    const size_t beg = (size_t)blockIdx.x * bk.chunk;
    const size_t end = beg + bk.chunk < n ? beg + bk.chunk : n;
    for (size_t i = beg + threadIdx.x; i < end; i += kBlock) {
        const uint32_t d = in[i].dst_host - bk.host_lo;
        rank[i] = d < bk.H ? atomicAdd(&hist[d >> bk.shift], 1u) : ~0u;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < bk.nb; b += kBlock) cnt1[(size_t)b * bk.ntiles + col_of(bk, blockIdx.x)] = hist[b];
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

// k_scan_top and k_scan_add in one launch: every workgroup sums the tile
// totals before its tile itself (bsum[0..t), at most a few hundred words,
// L2-warm) instead of reading a prefix array a one-workgroup launch wrote.
// A 256-element group lies in one kScanTile tile; out[len] (the group that
// holds index len) = that sum + the tile's own total when len is inside it.
__global__ __launch_bounds__(256) void k_scan_add_tiles(uint32_t* __restrict__ out, size_t len,
                                                        const uint32_t* __restrict__ bsum, uint32_t nb,
                                                        unsigned long long* counters) {
    const size_t i0 = (size_t)blockIdx.x * blockDim.x;
    const uint32_t t = (uint32_t)(i0 / kScanTile);
    uint32_t v = 0;
    for (uint32_t k = threadIdx.x; k < t && k < nb; k += blockDim.x) v += bsum[k];
    uint32_t pre;
    (void)block_excl_scan(v, &pre);
    const size_t i = i0 + threadIdx.x;
    if (i < len) out[i] += pre;
    if (i == len) {
        const uint32_t tot = pre + (t < nb ? bsum[t] : 0u);
        out[len] = tot;
        if (counters) counters[0] = tot;
    }
}

// The same scan in ONE launch of one 1,024-thread workgroup (len <=
// kScanOneMax): each wave owns a contiguous stretch of whole 256-element
// chunks; pass 1 sums it with 16-B loads, the 16 wave sums are combined
// through LDS, pass 2 re-reads the stretch (L2-warm) and writes the prefixes
// with a wave scan and a running carry.  out[len] = total (and counters[0]).
// Measured at H = 100k it is slower than the three launches (one CU walks
// 0.4 MB twice: round 0.996 vs 0.969 ms, profiles/r03e_scatter_probes.log),
// so it only takes small ranges, where a launch boundary costs more than
// the walk.
constexpr size_t kScanOneMax = 16384;
__global__ __launch_bounds__(1024) void k_scan_one(const uint32_t* __restrict__ in, size_t len,
                                                   uint32_t* __restrict__ out, unsigned long long* counters) {
    __shared__ uint32_t wsum[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t S = (len + 16 * 256 - 1) / (16 * 256) * 256;
    const size_t b0 = (size_t)w * S;
    auto ld4 = [&](size_t i) {
        uint4 v;
        if (i + 3 < len) {
            v = *reinterpret_cast<const uint4*>(in + i);
        } else {
            v.x = i < len ? in[i] : 0u;
            v.y = i + 1 < len ? in[i + 1] : 0u;
            v.z = i + 2 < len ? in[i + 2] : 0u;
            v.w = i + 3 < len ? in[i + 3] : 0u;
        }
        return v;
    };
    uint32_t sum = 0;
    for (size_t c = 0; c < S; c += 256) {
        const uint4 v = ld4(b0 + c + 4 * lane);
        sum += v.x + v.y + v.z + v.w;
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if (lane == 0) wsum[w] = sum;
    __syncthreads();
    uint32_t carry = 0, total = 0;
    for (int k = 0; k < 16; k++) {
        if (k < w) carry += wsum[k];
        total += wsum[k];
    }
    for (size_t c = 0; c < S && b0 + c < len; c += 256) {
        const size_t i = b0 + c + 4 * lane;
        const uint4 v = ld4(i);
        const uint32_t t = v.x + v.y + v.z + v.w;
        const uint32_t inc = wave_incl_scan(t, lane);
        uint32_t e = carry + inc - t;
        if (i < len) out[i] = e;
        e += v.x;
        if (i + 1 < len) out[i + 1] = e;
        e += v.y;
        if (i + 2 < len) out[i + 2] = e;
        e += v.z;
        if (i + 3 < len) out[i + 3] = e;
        carry += (uint32_t)__shfl(inc, 63);
    }
    if (threadIdx.x == 0) {
        out[len] = total;
        if (counters) counters[0] = total;
    }
}

// ---- bucket placement: one workgroup per scatter chunk, atomic-free ----
// The chunk's column of off1 (its run start in every bucket) is staged in
// LDS; every event goes to col[bucket] + its rank, a pure streaming pass.
__global__ __launch_bounds__(kPlaceBlock) void k_place_bucket(const ShdDeliv* __restrict__ in,
                                                              const uint8_t* __restrict__ status,
                                                              const uint32_t* __restrict__ rank, size_t n,
                                                              Bucketing bk, const uint32_t* __restrict__ off1,
                                                              ShdDeliv* __restrict__ stage) {
    __shared__ uint32_t col[kMaxBuckets];
    const uint32_t c = col_of(bk, blockIdx.x);
    for (uint32_t b = threadIdx.x; b < bk.nb; b += kPlaceBlock) col[b] = off1[(size_t)b * bk.ntiles + c];
    __syncthreads();
    const size_t beg = (size_t)blockIdx.x * bk.chunk;
    const size_t end = beg + bk.chunk < n ? beg + bk.chunk : n;
    for (size_t i0 = beg + threadIdx.x; i0 < end; i0 += (size_t)kPlaceBlock * kStream) {
        ShdDeliv r[kStream];
        uint32_t rk[kStream];
        bool ok[kStream];
#pragma unroll
        for (int k = 0; k < kStream; k++) {
            const size_t i = i0 + (size_t)k * kPlaceBlock;
            ok[k] = i < end && (!status || status[i] == SHD_DELIVERED);
            if (ok[k]) {
                r[k] = ld_ev(&in[i]);
                rk[k] = rank ? rank[i] : r[k].pad;
            }
        }
#pragma unroll
        for (int k = 0; k < kStream; k++) {
            const uint32_t d = r[k].dst_host - bk.host_lo;
            if (ok[k] && d < bk.H) st_ev(&stage[col[d >> bk.shift] + rk[k]], r[k]);
        }
    }
}

// ---- two-level staged partition (default): coalesced writes only ----
// Scattered 32-byte stores cost one L2->fabric request each (partial lines
// are written back piecewise), the same price as a random HBM read; a 100k-
// way grouping done in one pass (k_place_bucket / k_place_rank) pays it for
// every event.  Here the grouping is done in two passes of small fan-out,
// each staging a tile in LDS sorted by destination position so that
// consecutive lanes store consecutive events (runs of ~32 events):
//   pass 1 (k_stage_parts): record-order events -> `np` parts (contiguous
//     bucket ranges), chunk-major inside a part, exact positions from the
//     scanned count matrix (deterministic);
//   pass 2 (k_refine): part order -> bucket regions; each tile reserves its
//     run in every bucket it holds with one atomic per (tile, bucket) on
//     the bucket's cursor (coalesced: consecutive buckets), so the order
//     inside a bucket varies, which k_bucket_sort's total order removes.

// poff[p * ntiles + c]: start of column c's run in part p (pass-1 layout);
// cursor[b]: pass-2 write cursor of bucket b, initialised to its start.
__global__ __launch_bounds__(256) void k_part_offsets(const uint32_t* __restrict__ off1, Bucketing bk,
                                                      uint32_t pshift, uint32_t np, uint32_t* __restrict__ poff,
                                                      uint32_t* __restrict__ cursor) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < bk.nb) cursor[i] = off1[i * bk.ntiles];
    if (i >= (size_t)np * bk.ntiles) return;
    const uint32_t p = (uint32_t)(i / bk.ntiles), c = (uint32_t)(i % bk.ntiles);
    const uint32_t b0 = p << pshift, b1 = min(bk.nb, (p + 1) << pshift);
    uint32_t s = off1[(size_t)b0 * bk.ntiles]; // part start
    for (uint32_t b = b0; b < b1; b++) s += off1[(size_t)b * bk.ntiles + c] - off1[(size_t)b * bk.ntiles];
    poff[i] = s;
}

// Stages one tile's events in LDS ordered by their global destination
// position and stores them with consecutive lanes on consecutive slots.
__device__ __forceinline__ void stage_store(ShdDeliv* stg, uint32_t* gpos, uint32_t total, ShdDeliv* __restrict__ out) {
    for (uint32_t k = threadIdx.x; k < total; k += kStageBlock) st_ev(&out[gpos[k]], stg[k]);
}

// pass 1: one workgroup per scatter chunk, kStageTile events per step
__global__ __launch_bounds__(kStageBlock) void k_stage_parts(const ShdDeliv* __restrict__ in,
                                                             const uint8_t* __restrict__ status, size_t n,
                                                             Bucketing bk, uint32_t pshift, uint32_t np,
                                                             const uint32_t* __restrict__ poff,
                                                             ShdDeliv* __restrict__ out) {
    __shared__ uint32_t run[kMaxParts], cnt[kMaxParts], soff[kMaxParts];
    __shared__ ShdDeliv stg[kStageTile];
    __shared__ uint32_t gpos[kStageTile];
    const uint32_t col = col_of(bk, blockIdx.x);
    for (uint32_t p = threadIdx.x; p < np; p += kStageBlock) run[p] = poff[(size_t)p * bk.ntiles + col];
    const size_t beg = (size_t)blockIdx.x * bk.chunk;
    const size_t end = beg + bk.chunk < n ? beg + bk.chunk : n;
    for (size_t t0 = beg; t0 < end; t0 += kStageTile) {
        for (uint32_t p = threadIdx.x; p < np; p += kStageBlock) cnt[p] = 0;
        __syncthreads();
        ShdDeliv r[kStageItems];
        uint32_t part[kStageItems], rk[kStageItems];
#pragma unroll
        for (int k = 0; k < kStageItems; k++) {
            const size_t i = t0 + (size_t)k * kStageBlock + threadIdx.x;
            part[k] = ~0u;
            if (i < end && (!status || status[i] == SHD_DELIVERED)) {
                r[k] = ld_ev(&in[i]);
                const uint32_t d = r[k].dst_host - bk.host_lo;
                if (d < bk.H) part[k] = (d >> bk.shift) >> pshift;
            }
        }
#pragma unroll
        for (int k = 0; k < kStageItems; k++)
            if (part[k] != ~0u) rk[k] = atomicAdd(&cnt[part[k]], 1u);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t s = 0;
            for (uint32_t p = 0; p < np; p++) soff[p] = s, s += cnt[p];
            soff[kMaxParts - 1] = s; // np <= kMaxParts - 1: total in the last entry
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kStageItems; k++) {
            if (part[k] == ~0u) continue;
            const uint32_t slot = soff[part[k]] + rk[k];
            stg[slot] = r[k];
            gpos[slot] = run[part[k]] + rk[k];
        }
        __syncthreads();
        stage_store(stg, gpos, soff[kMaxParts - 1], out);
        __syncthreads();
        for (uint32_t p = threadIdx.x; p < np; p += kStageBlock) run[p] += cnt[p];
    }
}

// pass 2: part order -> bucket regions, one kStageTile tile per workgroup
__global__ __launch_bounds__(kStageBlock) void k_refine(const ShdDeliv* __restrict__ in, Bucketing bk,
                                                        uint32_t pshift, const uint32_t* __restrict__ off1,
                                                        uint32_t* __restrict__ cursor, ShdDeliv* __restrict__ out) {
    __shared__ uint32_t hist[kMaxBuckets], sof[kMaxBuckets];
    __shared__ ShdDeliv stg[kStageTile];
    __shared__ uint32_t gpos[kStageTile];
    __shared__ uint32_t range[2];
    const uint32_t total = off1[(size_t)bk.nb * bk.ntiles];
    const uint32_t t0 = blockIdx.x * kStageTile;
    if (t0 >= total) return;
    const uint32_t cnt = min((uint32_t)kStageTile, total - t0);
    if (threadIdx.x == 0) {
        // the tile is sorted by part: its buckets lie in the parts of its
        // first and last events
        const uint32_t pf = ((in[t0].dst_host - bk.host_lo) >> bk.shift) >> pshift;
        const uint32_t pl = ((in[t0 + cnt - 1].dst_host - bk.host_lo) >> bk.shift) >> pshift;
        range[0] = pf << pshift;
        range[1] = min(bk.nb, (pl + 1) << pshift);
    }
    __syncthreads();
    const uint32_t bmin = range[0], R = range[1] - range[0];
    for (uint32_t b = threadIdx.x; b < R; b += kStageBlock) hist[b] = 0;
    __syncthreads();
    ShdDeliv r[kStageItems];
    uint32_t lb[kStageItems], rk[kStageItems];
#pragma unroll
    for (int k = 0; k < kStageItems; k++) {
        const uint32_t i = (uint32_t)k * kStageBlock + threadIdx.x;
        lb[k] = ~0u;
        if (i < cnt) {
            r[k] = ld_ev(&in[t0 + i]);
            lb[k] = ((r[k].dst_host - bk.host_lo) >> bk.shift) - bmin;
        }
    }
#pragma unroll
    for (int k = 0; k < kStageItems; k++)
        if (lb[k] != ~0u) rk[k] = atomicAdd(&hist[lb[k]], 1u);
    __syncthreads();
    {   // exclusive scan of hist[0..R) -> sof (R <= kMaxBuckets = 16 per thread)
        constexpr int kPer = kMaxBuckets / kStageBlock;
        const uint32_t j0 = threadIdx.x * kPer;
        uint32_t v[kPer], s = 0;
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            v[q] = j0 + q < R ? hist[j0 + q] : 0u;
            s += v[q];
        }
        uint32_t tot;
        uint32_t pre = block_excl_scan(s, &tot);
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            if (j0 + q < R) sof[j0 + q] = pre;
            pre += v[q];
        }
    }
    __syncthreads();
    // reserve this tile's run in every bucket it holds (hist -> run base)
    for (uint32_t b = threadIdx.x; b < R; b += kStageBlock)
        if (hist[b]) hist[b] = atomicAdd(&cursor[bmin + b], hist[b]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kStageItems; k++) {
        if (lb[k] == ~0u) continue;
        const uint32_t slot = sof[lb[k]] + rk[k];
        stg[slot] = r[k];
        gpos[slot] = hist[lb[k]] + rk[k];
    }
    __syncthreads();
    stage_store(stg, gpos, cnt, out);
}

// ---- per-destination segment sort ----

struct Ev {
    unsigned long long t, q; // time, srcHostEventID
    unsigned s, ix;          // src host, packet index
};

// a compact slab slot (CSlab) as an event; the marker sends it to the 32-B slab
template <bool kNT = false>
__device__ __forceinline__ Ev c_load(const uint4* __restrict__ cslab, const ShdDeliv* __restrict__ slab, size_t i,
                                     unsigned long long tbase) {
    uint4 c;
    if (kNT) {
        const shd_v4u v = __builtin_nontemporal_load(reinterpret_cast<const shd_v4u*>(cslab) + i);
        c = make_uint4(v.x, v.y, v.z, v.w);
    } else c = cslab[i];
    if (c.x != kCMark) return Ev{tbase + c.x, (unsigned long long)c.w, c.y, c.z};
    const ShdDeliv r = ld_ev(&slab[i]);
    return Ev{r.time, r.seq, r.src_host, r.pkt_index};
}

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

__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

// One wave sorts one segment of n <= 64*E events held in registers
// (element i = e*64 + lane) by RANK: event_compare is a total order on
// distinct events ((src host, srcHostEventID) is unique), so the final slot of
// an event is the number of segment events that precede it.  Every element is
// broadcast once to the wave with v_readlane (scalar registers, no LDS, no
// shuffles) and compared with the lane's E elements; each event is then
// stored straight to out[o + rank] (the segment's lines are all written by
// this wave, back to back).  Element i is read from src[b + i], or from
// src[b + perm[i]] when perm (an LDS index list) is given.
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o > v ? o : v;
    }
    return v;
}

// The exchange's wire record (24 B): a delivered event without its
// destination (the block and offsets say it) and without the slot word.
// 25 % fewer bytes over xGMI than the 32-B ShdDeliv.
struct Wire {
    unsigned long long t, q;
    uint32_t s, ix;
};
static_assert(sizeof(Wire) == 24, "wire record");
__device__ __forceinline__ Ev ld_wire(const Wire* p) {
    const uint2* w = reinterpret_cast<const uint2*>(p); // 8-B aligned
    const uint2 a = w[0], b = w[1], c = w[2];
    return Ev{((unsigned long long)a.y << 32) | a.x, ((unsigned long long)b.y << 32) | b.x, c.x, c.y};
}
__device__ __forceinline__ void st_wire(Wire* p, unsigned long long t, unsigned long long q, uint32_t src,
                                        uint32_t ix) {
    uint2* w = reinterpret_cast<uint2*>(p);
    w[0] = make_uint2((uint32_t)t, (uint32_t)(t >> 32));
    w[1] = make_uint2((uint32_t)q, (uint32_t)(q >> 32));
    w[2] = make_uint2(src, ix);
}
template <int E, int kNT = 0, typename Load>
__device__ void wave_rank_segment(Load load, uint32_t n, uint32_t d, ShdDeliv* __restrict__ out, uint32_t o,
                                  int lane, unsigned long long* lk = nullptr) {
    Ev v[E];
    uint32_t rank[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        rank[e] = 0;
        v[e] = i < n ? load(i) : Ev{~0ull, ~0ull, ~0u, ~0u};
    }
    // Pass-1 key: (time - tmin) << 24 | src host when the segment's time span
    // is below 2^40 ns and every src id below 2^24 (it then orders by
    // event_compare's first two keys, and equal keys mean same time AND same
    // sender -- rare, unlike equal times, which every barrier-clamped event
    // shares); else the time alone.  Padding lanes are never counted.
    unsigned long long tmin = ~0ull, tmax = 0, smax = 0;
#pragma unroll
    for (int e = 0; e < E; e++)
        if (e * 64 + lane < (int)n) {
            tmin = v[e].t < tmin ? v[e].t : tmin;
            tmax = v[e].t > tmax ? v[e].t : tmax;
            smax = v[e].s > smax ? v[e].s : smax;
        }
    tmin = wave_min_u64(tmin);
    const bool packed = (wave_max_u64(tmax) - tmin) < (1ull << 40) && wave_max_u64(smax) < (1ull << 24);
    unsigned long long key[E];
#pragma unroll
    for (int e = 0; e < E; e++)
        key[e] = (e * 64 + lane < (int)n) ? (packed ? ((v[e].t - tmin) << 24) | v[e].s : v[e].t) : ~0ull;
    // pass 1: one 64-bit compare per pair (rank = number of smaller keys).
    // With a per-wave LDS key array (lk: 64 * E + 8 slots) the other keys
    // come two at a time by broadcast reads (every lane reads the same
    // address) instead of two readlanes each; slots past n hold the maximum
    // key, which is never smaller.
    if (lk) {
#pragma unroll
        for (int e = 0; e < E; e++) lk[e * 64 + lane] = key[e]; // (padding lanes hold ~0ull)
        if (lane < 8) lk[64 * E + lane] = ~0ull;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        const ulonglong2* lk2 = reinterpret_cast<const ulonglong2*>(lk);
        for (uint32_t j = 0; j < n; j += 8) {
            ulonglong2 kk[4];
#pragma unroll
            for (int u = 0; u < 4; u++) kk[u] = lk2[(j >> 1) + u];
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int e = 0; e < E; e++) rank[e] += (uint32_t)(kk[u].x < key[e]) + (uint32_t)(kk[u].y < key[e]);
        }
    } else {
#pragma unroll
        for (int ej = 0; ej < E; ej++) {
            const int lim = (int)n - ej * 64 < 64 ? (int)n - ej * 64 : 64; // wave-uniform
            for (int l = 0; l < lim; l++) {
                const unsigned long long kj = readlane_u64(key[ej], l);
#pragma unroll
                for (int e = 0; e < E; e++) rank[e] += (uint32_t)(kj < key[e]);
            }
        }
    }
    // Ties: the ranks are a permutation of [0, n) -- sum n(n-1)/2 -- iff all
    // keys differ; a group of g equal keys shares its lowest rank, which
    // lowers the sum.  (Replaces an equality count per pair: pass 1 is the
    // VALU-bound part of the segment sort.)
    uint32_t rsum = 0;
#pragma unroll
    for (int e = 0; e < E; e++) rsum += (e * 64 + lane < (int)n) ? rank[e] : 0u;
    for (int off = 32; off > 0; off >>= 1) rsum += (uint32_t)__shfl_xor((int)rsum, off);
    if (rsum != n * (n - 1) / 2) {
        // pass 2 (segments with equal keys only): rank among the events of
        // equal key by event_compare's remaining keys, branch-free
#pragma unroll
        for (int ej = 0; ej < E; ej++) {
            const int lim = (int)n - ej * 64 < 64 ? (int)n - ej * 64 : 64;
            for (int l = 0; l < lim; l++) {
                const unsigned long long kj = readlane_u64(key[ej], l);
                const unsigned long long qj = readlane_u64(v[ej].q, l);
                const unsigned sj = (unsigned)__builtin_amdgcn_readlane((int)v[ej].s, l);
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const bool after = packed ? (qj < v[e].q) : ((sj < v[e].s) | ((sj == v[e].s) & (qj < v[e].q)));
                    rank[e] += (uint32_t)((kj == key[e]) & after);
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        if (i >= n) continue;
        if (kNT == 3) { // the permutation only: out is an LDS index array, element i is item o + i
            reinterpret_cast<uint16_t*>(out)[o + rank[e]] = (uint16_t)(o + i);
        } else if (kNT == 2) { // the exchange's 24-B wire record (out is a Wire array)
            st_wire(reinterpret_cast<Wire*>(out) + o + rank[e], v[e].t, v[e].q, v[e].s, v[e].ix);
        } else if (kNT) {
            shd_v4u* q = reinterpret_cast<shd_v4u*>(&out[o + rank[e]]);
            const shd_v4u a = {(uint32_t)v[e].t, (uint32_t)(v[e].t >> 32), (uint32_t)v[e].q, (uint32_t)(v[e].q >> 32)};
            const shd_v4u b = {v[e].s, d, v[e].ix, 0u};
            __builtin_nontemporal_store(a, q);
            __builtin_nontemporal_store(b, q + 1);
        } else st_ev(&out[o + rank[e]], ShdDeliv{v[e].t, v[e].q, v[e].s, d, v[e].ix, 0u});
    }
}

// One wave sorts one segment of n <= 64*E events held in registers
// (element i = e*64 + lane), bitonic network over 64*E slots with +inf
// padding; partner distances < 64 cross lanes by shuffle, >= 64 stay in-lane.
// Element i is read from src[b + i], or from src[b + perm[i]] when perm
// (an LDS index list) is given; it is written to out[o + i].  (Kept as the
// SHD_SEGSORT=bitonic alternative of wave_rank_segment.)
template <int E>
__device__ void wave_sort_segment(const ShdDeliv* __restrict__ src, uint32_t b, const uint16_t* perm, uint32_t stride,
                                  uint32_t n,
                                  uint32_t d, ShdDeliv* __restrict__ out, uint32_t o, int lane) {
    Ev v[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        if (i < n) {
            const ShdDeliv r = ld_ev(&src[b + (perm ? (uint32_t)perm[i] : i * stride)]);
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
        if (i < n) st_ev(&out[o + i], ShdDeliv{v[e].t, v[e].q, v[e].s, d, v[e].ix, 0u});
    }
}

// Sorts one destination segment of n <= kSmallSeg events with one wave.
// algo: 1 rank sort, 0 bitonic network.
// Element i of the segment is src[b + perm[i]] (LDS index list) or
// src[b + i * stride] (stride 1: contiguous; H: a rank-major slab).
__device__ __forceinline__ void sort_segment(uint32_t algo, const ShdDeliv* __restrict__ src, uint32_t b,
                                             const uint16_t* perm, uint32_t n, uint32_t d,
                                             ShdDeliv* __restrict__ out, uint32_t o, int lane,
                                             uint32_t stride = 1, unsigned long long* lk = nullptr) {
    if (algo == 1) {
        auto load = [&](uint32_t i) {
            const ShdDeliv r = ld_ev(&src[b + (perm ? (uint32_t)perm[i] : i * stride)]);
            return Ev{r.time, r.seq, r.src_host, r.pkt_index};
        };
        if (n <= 64) wave_rank_segment<1>(load, n, d, out, o, lane, lk);
        else if (n <= 128) wave_rank_segment<2>(load, n, d, out, o, lane, lk);
        else wave_rank_segment<4>(load, n, d, out, o, lane, lk);
    } else {
        if (n <= 64) wave_sort_segment<1>(src, b, perm, stride, n, d, out, o, lane);
        else if (n <= 128) wave_sort_segment<2>(src, b, perm, stride, n, d, out, o, lane);
        else wave_sort_segment<4>(src, b, perm, stride, n, d, out, o, lane);
    }
}

// One workgroup per bucket (2^shift destinations, at most kBucketCap events
// on the LDS path).  The bucket's events are read once for their
// destination (LDS histogram, rank = old value of the LDS atomic), the
// per-destination offsets are scanned in LDS, an LDS index list orders the
// events by destination, and each wave sorts whole destination segments by
// (time, src host, srcHostEventID), gathering the events through the index
// list (the bucket region was just read: L2 / Infinity-Cache resident) and
// writing each segment contiguously to its final place.  Segments above
// kSmallSeg events, and every segment of a bucket above kBucketCap events,
// are copied unsorted to their final place and listed for k_segsort_mid /
// k_segsort_merge.
__global__ __launch_bounds__(kSortBlock) void k_bucket_sort(const ShdDeliv* __restrict__ stage, Bucketing bk,
                                                            const uint32_t* __restrict__ off1,
                                                            uint32_t* __restrict__ offsets,
                                                            ShdDeliv* __restrict__ out, uint32_t* __restrict__ big,
                                                            uint32_t* __restrict__ nbig) {
    __shared__ uint32_t cnt[kMaxPerBucket];
    __shared__ uint32_t loc[kMaxPerBucket];
    __shared__ uint32_t wsum[kSortBlock / 64];
    __shared__ uint16_t rk[kBucketCap];
    __shared__ uint16_t dd[kBucketCap];
    __shared__ uint16_t perm[kBucketCap];
    // the bucket's events, structure of arrays (24 B per event; the
    // destination is implied by the segment)
    __shared__ unsigned long long ev_t[kBucketCap], ev_q[kBucketCap];
    __shared__ uint32_t ev_s[kBucketCap], ev_x[kBucketCap];
    const uint32_t b = blockIdx.x;
    const uint32_t d0 = b << bk.shift;                           // first destination (range-relative)
    const uint32_t nd = min(1u << bk.shift, bk.H - d0);          // destinations in this bucket
    const uint32_t s = off1[(size_t)b * bk.ntiles];              // bucket region [s, e)
    const uint32_t e = off1[(size_t)(b + 1) * bk.ntiles];
    const uint32_t ne = e - s;
    const bool fits = ne <= (uint32_t)kBucketCap;
    for (uint32_t j = threadIdx.x; j < nd; j += kSortBlock) cnt[j] = 0;
    __syncthreads();
    for (uint32_t i0 = threadIdx.x; i0 < ne; i0 += kSortBlock * kBucketLoads) {
        ShdDeliv rq[kBucketLoads];
#pragma unroll
        for (int q = 0; q < kBucketLoads; q++) {
            const uint32_t i = i0 + (uint32_t)q * kSortBlock;
            if (i < ne) rq[q] = ld_ev(&stage[s + i]);
        }
#pragma unroll
        for (int q = 0; q < kBucketLoads; q++) {
            const uint32_t i = i0 + (uint32_t)q * kSortBlock;
            if (i >= ne) continue;
            const uint32_t dl = rq[q].dst_host - bk.host_lo - d0;
            const uint32_t r = atomicAdd(&cnt[dl], 1u);
            if (fits) {
                rk[i] = (uint16_t)r;
                dd[i] = (uint16_t)dl;
                ev_t[i] = rq[q].time;
                ev_q[i] = rq[q].seq;
                ev_s[i] = rq[q].src_host;
                ev_x[i] = rq[q].pkt_index;
            }
        }
    }
    __syncthreads();
    // exclusive scan of cnt[0..nd) (nd <= kMaxPerBucket = 2 * kSortBlock)
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
    const int lane = threadIdx.x & 63;
    if (fits) {
        for (uint32_t i = threadIdx.x; i < ne; i += kSortBlock) perm[loc[dd[i]] + rk[i]] = (uint16_t)i;
        __syncthreads();
        for (uint32_t j = threadIdx.x >> 6; j < nd; j += kSortBlock / 64) {
            const uint32_t n = cnt[j], o = loc[j], dh = bk.host_lo + d0 + j;
            if (n == 0) continue;
            const uint16_t* pj = perm + o;
            auto load = [&](uint32_t i) {
                const uint32_t k = pj[i];
                return Ev{ev_t[k], ev_q[k], ev_s[k], ev_x[k]};
            };
            if (n <= 64) wave_rank_segment<1>(load, n, dh, out, s + o, lane);
            else if (n <= 128) wave_rank_segment<2>(load, n, dh, out, s + o, lane);
            else if (n <= (uint32_t)kSmallSeg) wave_rank_segment<4>(load, n, dh, out, s + o, lane);
            else {
                for (uint32_t i = lane; i < n; i += 64) {
                    const Ev v = load(i);
                    st_ev(&out[s + o + i], ShdDeliv{v.t, v.q, v.s, dh, v.ix, 0u});
                }
                if (lane == 0) big[atomicAdd(nbig, 1u)] = d0 + j;
            }
        }
    } else {
        // oversized bucket (skewed destinations): unsorted placement through
        // LDS cursors, every segment then sorted by k_segsort_mid / _merge
        for (uint32_t j = threadIdx.x; j < nd; j += kSortBlock)
            if (cnt[j] > 0) big[atomicAdd(nbig, 1u)] = d0 + j;
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < nd; j += kSortBlock) cnt[j] = 0;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < ne; i += kSortBlock) {
            ShdDeliv r = ld_ev(&stage[s + i]);
            r.pad = 0;
            const uint32_t j = r.dst_host - bk.host_lo - d0;
            st_ev(&out[s + loc[j] + atomicAdd(&cnt[j], 1u)], r);
        }
    }
}

__device__ __forceinline__ bool ev_less(const ShdDeliv& a, const ShdDeliv& b) {
    if (a.time != b.time) return a.time < b.time;
    if (a.src_host != b.src_host) return a.src_host < b.src_host;
    return a.seq < b.seq;
}


// ---- listed segments (above kSmallSeg events) ----
// Segments of up to kChunk events: one workgroup sorts the segment in LDS
// (k_segsort_mid).  Larger segments (skewed destinations: a popular server
// can receive a sizeable share of a round) are cut into kChunk-event runs,
// each sorted in LDS by the same kernel, then merged pairwise by
// k_segsort_merge: merge-path tiles of kMergeTile outputs, claimed from a
// global work counter in (pass, segment, tile) order by persistent
// workgroups; a tile of pass p waits only for its segment's pass p-1 tiles,
// which were claimed before it and so are being processed by running
// workgroups -- no co-residency assumption, no grid barrier.  Runs ping-pong
// between `out` and `scratch`; the chunk sort writes to whichever makes the
// last pass land in `out`.  event_compare is a total order on distinct
// events, so every merge is exact.
constexpr uint32_t kMidSeg = 4096;      // 96 KiB of dynamic LDS
constexpr uint32_t kChunk = kMidSeg;    // sorted runs of the chunk sort
constexpr uint32_t kMergeTile = 2048;   // outputs per merge tile: 256 threads x 8
constexpr uint32_t kMaxPasses = 24;     // 4096 << 24 events per segment
constexpr uint32_t kMidThreads = 1024;

__device__ __forceinline__ uint32_t merge_passes(uint32_t n) {
    const uint32_t c = (n + kChunk - 1) / kChunk;
    uint32_t p = 0;
    while ((1u << p) < c) p++;
    return p;
}

// Merge metadata (one u32 array in the workspace, shd_dev_ws): header, then
// per merge segment {b, n, dst host, passes} sorted by passes descending (so
// the segments taking part in pass p are a prefix), their tile prefix, and
// per (segment, pass) a count of finished tiles.
struct MergeMeta {
    uint32_t* hdr;   // [0] segments, [1] items, [2] work counter, [3] this round's fault word,
                     // [4 + p] first item of pass p (p <= kMaxPasses), [32 + p] segments in pass p,
                     // [kStickyFault] OR of every round's fault word since the host last read it
    uint4* seg;      // cap
    uint32_t* tpre;  // cap + 1
    uint32_t* done;  // cap * kMaxPasses
    uint32_t cap;
    uint32_t cap_big; // entries of the big-segment list (nbig[0] never exceeds it)
    unsigned long long* flag; // the caller's counters[0] (or null): SHD_ROUND_FAULT set in the faulting round
    uint32_t spin_limit;      // merge waits before a tile gives up (SHD_DEBUG_MERGE_SPIN; 0: every wait faults)
    // a synchronous part round's end, done by the merge kernel's last
    // workgroup (fin_host null: none; see fin_body and ws_sync)
    unsigned long long* fin_host = nullptr;
    uint32_t* fin_nbig = nullptr;
    uint32_t* fin_cnt1 = nullptr;
    uint32_t fin_m = 0;
    unsigned long long* fin_minw2 = nullptr;
};
constexpr uint32_t kMetaHdr = 64;
constexpr uint32_t kStickyFault = 60;
constexpr uint32_t kFinCount = 62; // the merge workgroups that finished (the last one ends the round, then resets it)

// A fault of this round: its word into the round's header slot, the sticky
// word the host reads back, and the caller-visible bit of counters[0]
// (include/shdnet.h SHD_ROUND_FAULT), so the call whose round faulted can see
// it without waiting for a later call.
__device__ __forceinline__ void note_fault(const MergeMeta& mm, uint32_t f) {
    if (!f) return;
    atomicOr(&mm.hdr[kStickyFault], f);
    if (mm.flag) atomicOr(mm.flag, (unsigned long long)SHD_ROUND_FAULT);
}

// A synchronous round's end (one workgroup, every thread; after all of the
// round's work): the next part round's resets (m > 0: nbig, cnt1[0, m), the
// min word), then -- every store of the workgroup device-visible first: the
// host may start the next round on another stream as soon as it sees it --
// the sticky fault word and the zero word beside it (the end marker, see
// ws_sync) into pinned host memory with one system-scope 8-B store
__device__ __forceinline__ void fin_body(const uint32_t* src, unsigned long long* host, uint32_t* nbig, uint32_t* cnt1,
                                         uint32_t m, unsigned long long* minw2) {
    // the segments this round listed, reported in the marker's place (below
    // the host-set all-ones: ws_sync's end, and k_segsort_medium's launch
    // decision for the next synchronous round, see sort_listed)
    const uint32_t nb0 = threadIdx.x == 0 ? nbig[0] : 0u;
    if (m) {
        if (threadIdx.x < 3) nbig[threadIdx.x] = 0u;
        if (threadIdx.x == 3) minw2[1] = ~0ull;
        uint4* c4 = reinterpret_cast<uint4*>(cnt1); // (hipMalloc'd: 16-B aligned)
        for (uint32_t i = threadIdx.x; i < m / 4; i += blockDim.x) c4[i] = uint4{0u, 0u, 0u, 0u};
        for (uint32_t i = (m / 4) * 4 + threadIdx.x; i < m; i += blockDim.x) cnt1[i] = 0u;
    }
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long v = (unsigned long long)__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                                     ((unsigned long long)min(nb0, 0xFFFFFFFEu) << 32);
        __hip_atomic_store(host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Block-uniform value read from LDS or memory, made wave-uniform for the
// compiler (an SGPR): loops and branches around barriers must be uniform in
// its divergence analysis too, or the structurizer may split a loop between
// lanes and the waves reach different barriers.
__device__ __forceinline__ uint32_t bu(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// Barrier for global memory written by one wave and read by another in the
// same workgroup: __syncthreads() does not wait for vector stores to land
// (MI355X_MICROARCH.md, hand-off forms), so every wave drains first.
__device__ __forceinline__ void vm_sync() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// block-wide exclusive scan for kMidThreads threads
__device__ __forceinline__ uint32_t block_excl_scan_1k(uint32_t v, uint32_t* total, uint32_t* ws) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int k = 0; k < (int)(kMidThreads / 64); k++) {
        if (k < w) base += ws[k];
        tot += ws[k];
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// LDS bitonic sort of n <= kChunk events read from src[b ...], written to
// dst[b ...] (in place when src == dst: the whole range is in LDS first).
__device__ void lds_sort_run(const ShdDeliv* src, ShdDeliv* dst, uint32_t b, uint32_t n, uint32_t dh, Ev* sv) {
    uint32_t N = 1;
    while (N < n) N <<= 1;
    for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
        if (i < n) {
            const ShdDeliv r = ld_ev(&src[b + i]);
            sv[i] = Ev{r.time, r.seq, r.src_host, r.pkt_index};
        } else {
            sv[i] = Ev{~0ull, ~0ull, ~0u, ~0u};
        }
    }
    __syncthreads();
    for (uint32_t k = 2; k <= N; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const Ev x = sv[i], y = sv[l];
                    const bool up = (i & k) == 0;
                    if (up ? ev_lt(y, x) : ev_lt(x, y)) {
                        sv[i] = y;
                        sv[l] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        st_ev(&dst[b + i], ShdDeliv{sv[i].t, sv[i].q, sv[i].s, dh, sv[i].ix, 0u});
    __syncthreads();
}

// Listed segments of kSmallSeg < n <= kMedSeg events (the owners' segments
// of a weak-scaled exchange: ~92 N events per destination at N ranks): one
// wave each, a bitonic network over the segment in the wave's LDS region
// (padded to a power of two) -- no workgroup barriers: a wave's LDS accesses
// stay in order.  O(n log^2 n) compare-exchanges, against the register rank
// sort's O(n^2) (whose tie pass -- equal time and sender, frequent when most
// deliveries are clamped to the barrier -- is slower still) and
// k_segsort_mid's 1,024-thread network per segment, one segment per
// workgroup at a time.  k_segsort_mid then skips these segments.
constexpr uint32_t kMedSeg = 1024;
constexpr int kMedWaves = 2; // waves per workgroup (LDS: kMedSeg x 24 B each)
__global__ __launch_bounds__(64 * kMedWaves) void k_segsort_medium(const ShdDeliv* __restrict__ unsorted,
                                                                   const uint32_t* __restrict__ off,
                                                                   const uint32_t* __restrict__ big,
                                                                   const uint32_t* __restrict__ nbig,
                                                                   ShdDeliv* __restrict__ out, uint32_t cap_big) {
    __shared__ Ev sv_all[kMedWaves][kMedSeg];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    Ev* sv = sv_all[wv];
    const uint32_t nb_raw = nbig[0];
    const uint32_t nb = nb_raw <= cap_big ? nb_raw : 0u; // (an overfull list is k_segsort_mid's to report)
    const uint32_t wave = blockIdx.x * kMedWaves + wv, nwaves = gridDim.x * kMedWaves;
    for (uint32_t q = wave; q < nb; q += nwaves) {
        const uint32_t d = big[q];
        const uint32_t b = off[d], n = off[d + 1] - b;
        if (n <= (uint32_t)kSmallSeg || n > kMedSeg) continue;
        uint32_t N = 512;
        while (N < n) N <<= 1;
        const uint32_t dh = (uint32_t)__builtin_amdgcn_readfirstlane((int)unsorted[b].dst_host);
        for (uint32_t i = lane; i < N; i += 64) {
            if (i < n) {
                const ShdDeliv r = ld_ev(&unsorted[b + i]);
                sv[i] = Ev{r.time, r.seq, r.src_host, r.pkt_index};
            } else {
                sv[i] = Ev{~0ull, ~0ull, ~0u, ~0u};
            }
        }
        for (uint32_t k = 2; k <= N; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1)
                for (uint32_t p = lane; p < (N >> 1); p += 64) { // pair p: i = its lower index
                    const uint32_t i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), l = i | j;
                    const Ev x = sv[i], y = sv[l];
                    if (((i & k) == 0) ? ev_lt(y, x) : ev_lt(x, y)) {
                        sv[i] = y;
                        sv[l] = x;
                    }
                }
        for (uint32_t i = lane; i < n; i += 64) {
            const Ev e = sv[i];
            shd_v4u* qd = reinterpret_cast<shd_v4u*>(&out[b + i]);
            const shd_v4u a0 = {(uint32_t)e.t, (uint32_t)(e.t >> 32), (uint32_t)e.q, (uint32_t)(e.q >> 32)};
            const shd_v4u a1 = {e.s, dh, e.ix, 0u};
            __builtin_nontemporal_store(a0, qd);
            __builtin_nontemporal_store(a1, qd + 1);
        }
    }
}

// Every listed segment's kChunk-event runs, dealt round-robin over the
// workgroups (a segment of up to kChunk events is one run, sorted straight
// into `out`).  Workgroup 0 also builds the merge metadata.  skip_med:
// segments of kSmallSeg < n <= kMedSeg events are k_segsort_medium's.
__global__ __launch_bounds__(kMidThreads) void k_segsort_mid(const ShdDeliv* unsorted,
                                                             const uint32_t* __restrict__ off,
                                                             const uint32_t* __restrict__ big,
                                                             const uint32_t* __restrict__ nbig, ShdDeliv* out,
                                                             ShdDeliv* scratch, MergeMeta mm, uint32_t rank_small,
                                                             uint32_t skip_med) {
    extern __shared__ __attribute__((aligned(16))) char mid_smem[];
    Ev* sv = reinterpret_cast<Ev*>(mid_smem);
    __shared__ uint32_t sb[kMidThreads], sn[kMidThreads], sst[kMidThreads + 1];
    __shared__ uint32_t ws[kMidThreads / 64];
    __shared__ uint32_t hp[kMaxPasses + 1], cur[kMaxPasses + 1], s_part[kMaxPasses], s_ns;
    // the list holds at most one entry per destination (cap_big): a count
    // above it is a fault of an earlier stage, reported, never followed
    const uint32_t nb_raw = nbig[0], tid = threadIdx.x, grid = gridDim.x;
    const uint32_t nb = nb_raw <= mm.cap_big ? nb_raw : 0u;
    uint32_t base = 0;
    for (uint32_t qb = 0; qb < nb; qb += kMidThreads) {
        const uint32_t q = qb + tid;
        uint32_t b = 0, n = 0;
        if (q < nb) {
            const uint32_t d = big[q];
            b = off[d];
            n = off[d + 1] - b;
        }
        const uint32_t nch = (skip_med && n > (uint32_t)kSmallSeg && n <= kMedSeg) ? 0u : (n + kChunk - 1) / kChunk;
        uint32_t total;
        const uint32_t st = block_excl_scan_1k(nch, &total, ws);
        total = bu(total);
        sb[tid] = b;
        sn[tid] = n;
        sst[tid] = st;
        if (tid == 0) sst[kMidThreads] = total;
        __syncthreads();
        for (uint32_t i = base + (blockIdx.x + grid - base % grid) % grid; i < base + total; i += grid) {
            const uint32_t loc = i - base;
            uint32_t lo = 0, hi = kMidThreads; // last t with sst[t] <= loc (block-uniform search)
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (bu(sst[mid]) <= loc) lo = mid;
                else hi = mid;
            }
            const uint32_t c = loc - bu(sst[lo]), sbb = bu(sb[lo]), snn = bu(sn[lo]);
            const uint32_t cb = sbb + c * kChunk, cn = snn - c * kChunk < kChunk ? snn - c * kChunk : kChunk;
            ShdDeliv* dst = (snn <= kChunk || (merge_passes(snn) & 1u) == 0) ? out : scratch;
            if (rank_small && snn <= (uint32_t)kSmallSeg) {
                // a segment of at most 256 events (the slab pipeline lists
                // every segment above its 128 slab slots): one wave's rank
                // sort, as k_segsort_dst's, instead of the workgroup's
                // 256-wide bitonic network (36 barrier stages)
                if (threadIdx.x < 64) {
                    const uint32_t dh = bu(unsorted[cb].dst_host);
                    auto load = [&](uint32_t i) {
                        const ShdDeliv r = ld_ev(&unsorted[cb + i]);
                        return Ev{r.time, r.seq, r.src_host, r.pkt_index};
                    };
                    unsigned long long* lk = reinterpret_cast<unsigned long long*>(sv); // 64 * 4 + 8 keys
                    if (snn <= 64) wave_rank_segment<1>(load, snn, dh, dst, cb, (int)threadIdx.x, lk);
                    else if (snn <= 128) wave_rank_segment<2>(load, snn, dh, dst, cb, (int)threadIdx.x, lk);
                    else wave_rank_segment<4>(load, snn, dh, dst, cb, (int)threadIdx.x, lk);
                }
                __syncthreads();
            } else {
                lds_sort_run(unsorted, dst, cb, cn, bu(unsorted[cb].dst_host), sv);
            }
        }
        base += total;
        __syncthreads();
    }
    if (blockIdx.x != 0) return;
    // ---- merge metadata (workgroup 0): segments above kChunk by passes, descending
    for (uint32_t k = tid; k <= kMaxPasses; k += kMidThreads) hp[k] = 0;
    __syncthreads();
    for (uint32_t q = tid; q < nb; q += kMidThreads) {
        const uint32_t d = big[q], n = off[d + 1] - off[d];
        if (n > kChunk) atomicAdd(&hp[merge_passes(n)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int p = (int)kMaxPasses; p >= 1; p--) { // descending passes
            cur[p] = acc;
            acc += hp[p];
        }
        s_ns = acc < mm.cap ? acc : mm.cap; // (read back through LDS: see vm_sync)
        mm.hdr[0] = s_ns;
        // this round's fault word: spin-limit hits of the merge (counted by
        // k_segsort_merge) and the metadata overflow bit (cannot happen: cap
        // covers n / (kChunk + 1)); read back by the host (ws_faults)
        const uint32_t fw =
            (acc > mm.cap ? 0x80000000u : 0u) | ((nbig[2] | (nb_raw > mm.cap_big ? kFaultBigCap : 0u)) << 24);
        mm.hdr[3] = fw;
        note_fault(mm, fw);
        // segments taking part in pass p: those with more than p passes
        uint32_t part = 0;
        for (int p = (int)kMaxPasses - 1; p >= 0; p--) {
            part += hp[p + 1];
            s_part[p] = part;
            mm.hdr[32 + p] = part;
        }
    }
    __syncthreads();
    for (uint32_t q = tid; q < nb; q += kMidThreads) {
        const uint32_t d = big[q], b = off[d], n = off[d + 1] - b;
        if (n <= kChunk) continue;
        const uint32_t k = atomicAdd(&cur[merge_passes(n)], 1u);
        if (k < mm.cap) mm.seg[k] = make_uint4(b, n, unsorted[b].dst_host, merge_passes(n));
    }
    vm_sync(); // other waves read these entries next
    // tile prefix over the sorted segments, then the per-pass item bases
    const uint32_t ns = bu(s_ns);
    uint32_t run = 0;
    for (uint32_t kb = 0; kb < ns; kb += kMidThreads) {
        const uint32_t k = kb + tid;
        const uint32_t nt = k < ns ? (mm.seg[k].y + kMergeTile - 1) / kMergeTile : 0u;
        uint32_t total;
        const uint32_t st = block_excl_scan_1k(nt, &total, ws);
        if (k < ns) mm.tpre[k] = run + st;
        run += bu(total);
    }
    vm_sync(); // (thread 0 reads other threads' tpre entries)
    if (tid == 0) {
        mm.tpre[ns] = run;
        uint32_t item = 0;
        for (uint32_t p = 0; p < kMaxPasses; p++) {
            mm.hdr[4 + p] = item;
            item += s_part[p] == ns ? run : mm.tpre[s_part[p]]; // (tpre[ns]: this thread's own store)
        }
        mm.hdr[4 + kMaxPasses] = item;
        mm.hdr[1] = item;
        mm.hdr[2] = 0;
    }
    for (uint32_t k = tid; k < ns * kMaxPasses; k += kMidThreads) mm.done[k] = 0;
}

// Merge-path split for output diagonal `diag` of A (la) and B (lb) in
// global memory: the number of outputs taken from A, i.e. the first m in
// [lo, hi) with B[diag - 1 - m] < A[m] (else hi).  The workgroup probes up
// to blockDim positions per step: one dependent load pair per step, log_256
// of the range.  Block-uniform; sh: one LDS word.
__device__ uint32_t coop_split(const ShdDeliv* A, uint32_t la, const ShdDeliv* B, uint32_t lb, uint32_t diag,
                               uint32_t* sh) {
    uint32_t lo = diag > lb ? diag - lb : 0u, hi = diag < la ? diag : la;
    const uint32_t nt = blockDim.x;
    while (lo < hi) {
        const uint32_t span = hi - lo;
        const bool dense = span <= nt; // probes lo + k, k < span: this step decides
        const uint32_t k = threadIdx.x;
        const uint32_t m = dense ? lo + k : lo + (uint32_t)(((unsigned long long)span * k) / nt);
        bool pred = false;
        if (!dense || k < span) pred = ev_less(ld_ev(&B[diag - 1 - m]), ld_ev(&A[m]));
        if (threadIdx.x == 0) sh[0] = nt;
        __syncthreads();
        if (pred) atomicMin(&sh[0], k);
        __syncthreads();
        const uint32_t f = bu(sh[0]); // first probe that is true (nt: none)
        __syncthreads();
        if (dense) return f == nt ? hi : lo + f;
        auto mk = [&](uint32_t q) { return lo + (uint32_t)(((unsigned long long)span * q) / nt); };
        if (f == nt) {
            lo = mk(nt - 1) + 1;
        } else {
            const uint32_t nlo = f ? mk(f - 1) + 1 : lo;
            hi = mk(f);
            lo = nlo;
        }
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_segsort_merge(ShdDeliv* out, ShdDeliv* scratch, MergeMeta mm) {
    __shared__ Ev tile[kMergeTile];
    __shared__ uint32_t sh[8];
    const uint32_t tid = threadIdx.x;
    const uint32_t items = bu(mm.hdr[1]);
    // no segment above kChunk (every uniform round): leave without touching
    // the claim counter -- 512 same-address atomics cost more than the launch
    // (a synchronous round's end then comes from workgroup 0: nothing else
    // of the round is left)
    if (items == 0) {
        if (mm.fin_host && blockIdx.x == 0)
            fin_body(mm.hdr + kStickyFault, mm.fin_host, mm.fin_nbig, mm.fin_cnt1, mm.fin_m, mm.fin_minw2);
        return;
    }
    uint32_t done_slot = ~0u; // the previous tile's (segment, pass) counter, published at the next claim
    for (;;) {
        // one lane: publish the previous tile (its stores were drained before
        // the barrier that ended it), then claim the next -- a single lane
        // region between barriers (a second one at the end of the body let
        // the compiler split the loop between lanes)
        if (tid == 0) {
            if (done_slot != ~0u) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                atomicAdd(&mm.done[done_slot], 1u);
            }
            sh[1] = atomicAdd(&mm.hdr[2], 1u);
        }
        __syncthreads();
        const uint32_t item = bu(sh[1]);
        __syncthreads();
        if (item >= items) break;
        uint32_t p = 0;
        while (p + 1 < kMaxPasses && bu(mm.hdr[4 + p + 1]) <= item) p++;
        const uint32_t loc = item - bu(mm.hdr[4 + p]);
        uint32_t lo = 0, hi = bu(mm.hdr[32 + p]); // the segment: last k with tpre[k] <= loc
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (bu(mm.tpre[mid]) <= loc) lo = mid;
            else hi = mid;
        }
        const uint32_t sgi = lo;
        const uint4 sg = mm.seg[sgi];
        const uint32_t b = bu(sg.x), n = bu(sg.y), dh = bu(sg.z), P = bu(sg.w);
        const uint32_t t = loc - bu(mm.tpre[sgi]);
        const uint32_t ntile = (n + kMergeTile - 1) / kMergeTile;
        if (p > 0) { // the segment's previous pass must be complete (its tiles were claimed before this one)
            if (tid == 0) {
                uint32_t spins = 0;
                bool gave_up = mm.spin_limit == 0; // (debug knob: every wait gives up)
                while (!gave_up && __hip_atomic_load(&mm.done[sgi * kMaxPasses + p - 1], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) < ntile) {
                    __builtin_amdgcn_s_sleep(2);
                    gave_up = ++spins >= mm.spin_limit; // every wave ends (inputs that never complete would be a bug)
                }
                if (gave_up) {
                    atomicAdd(&mm.hdr[3], 1u);
                    note_fault(mm, 1u);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); // drops this CU's stale lines
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (holds the barrier for the invalidate)
            }
            __syncthreads();
        }
        // pass p reads the buffer the chunk sort (p = 0) or pass p - 1 wrote
        ShdDeliv* x0 = (P & 1u) ? scratch : out;
        ShdDeliv* x1 = (P & 1u) ? out : scratch;
        const ShdDeliv* src = ((p & 1u) ? x1 : x0) + b;
        ShdDeliv* dst = ((p & 1u) ? x0 : x1) + b;
        const uint32_t L = kChunk << p;
        const uint32_t o0 = t * kMergeTile;            // tile outputs [o0, o1) of the segment
        const uint32_t a0 = o0 / (2 * L) * (2 * L);   // its run pair (a tile never straddles two)
        const uint32_t la = n - a0 < L ? n - a0 : L;
        const uint32_t lb = n - a0 - la < L ? n - a0 - la : L;
        const uint32_t d0 = o0 - a0, d1 = (o0 + kMergeTile < n ? o0 + kMergeTile : n) - a0;
        const ShdDeliv* A = src + a0;
        const ShdDeliv* B = A + la;
        const uint32_t s0 = lb ? coop_split(A, la, B, lb, d0, sh + 4) : d0;
        const uint32_t s1 = lb ? coop_split(A, la, B, lb, d1, sh + 4) : d1;
        const uint32_t ta = s1 - s0, tb = (d1 - d0) - ta;
        for (uint32_t i = tid; i < ta + tb; i += blockDim.x) {
            const ShdDeliv r = i < ta ? ld_ev(&A[s0 + i]) : ld_ev(&B[d0 - s0 + (i - ta)]);
            tile[i] = Ev{r.time, r.seq, r.src_host, r.pkt_index};
        }
        __syncthreads();
        const uint32_t k0 = tid * (kMergeTile / 256);
        if (k0 < ta + tb) {
            // this thread's split inside the tile (A part = tile[0, ta), B part = tile[ta, ta + tb))
            uint32_t lo2 = k0 > tb ? k0 - tb : 0u, hi2 = k0 < ta ? k0 : ta;
            while (lo2 < hi2) {
                const uint32_t m = (lo2 + hi2) >> 1;
                if (ev_lt(tile[ta + k0 - 1 - m], tile[m])) hi2 = m;
                else lo2 = m + 1;
            }
            uint32_t i = lo2, j = k0 - lo2;
            const uint32_t kend = k0 + kMergeTile / 256 < ta + tb ? k0 + kMergeTile / 256 : ta + tb;
            for (uint32_t k = k0; k < kend; k++) {
                const bool takeA = j >= tb || (i < ta && !ev_lt(tile[ta + j], tile[i]));
                const Ev e = takeA ? tile[i] : tile[ta + j];
                if (takeA) i++;
                else j++;
                st_ev(&dst[a0 + d0 + k], ShdDeliv{e.t, e.q, e.s, dh, e.ix, 0u});
            }
        }
        // the tile is published at the next claim (MI355X_MICROARCH.md, valid
        // hand-off forms): every storing wave drains its stores, barrier, then
        // one lane's agent release, drain, and the counter add consumers poll
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        done_slot = sgi * kMaxPasses + p;
    }
    // a synchronous round's end: the last workgroup to finish (its output
    // stores drained before the loop's last barrier; a device-scope release
    // before the count)
    if (mm.fin_host) {
        if (tid == 0) {
            __threadfence();
            sh[0] = atomicAdd(&mm.hdr[kFinCount], 1u) == gridDim.x - 1 ? 1u : 0u;
        }
        __syncthreads();
        if (sh[0]) {
            __threadfence();
            if (tid == 0) mm.hdr[kFinCount] = 0u;
            fin_body(mm.hdr + kStickyFault, mm.fin_host, mm.fin_nbig, mm.fin_cnt1, mm.fin_m, mm.fin_minw2);
        }
    }
}

// ---- "rank" pipeline: per-destination counters, atomic-free placement ----

// Regroup path: rank of each event inside its destination (counter old value).
__global__ __launch_bounds__(256) void k_hist_rank(const ShdDeliv* __restrict__ in, size_t n, uint32_t host_lo,
                                                   uint32_t H, uint32_t* __restrict__ cnt, uint32_t* __restrict__ rank,
                                                   uint32_t agg_on) {
    __shared__ uint32_t agg_s[3 * 256];
    const int lane = threadIdx.x & 63;
    const DestAgg agg{agg_s + 3 * (threadIdx.x & ~63u), agg_s + 3 * (threadIdx.x & ~63u) + 64,
                      agg_s + 3 * (threadIdx.x & ~63u) + 128, agg_on};
    agg.cnt[lane] = 0;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t d = in[i].dst_host - host_lo; // out-of-range events are dropped
        const uint32_t r = dest_slot(d < H, d, cnt, agg, lane);
        rank[i] = d < H ? r : ~0u;
    }
}

// Each event goes to off[dst] + its rank (pad, or rank[] on the regroup path).
__global__ __launch_bounds__(256) void k_place_rank(const ShdDeliv* __restrict__ in, const uint8_t* __restrict__ status,
                                                    const uint32_t* __restrict__ rank, size_t n, uint32_t host_lo,
                                                    uint32_t H, const uint32_t* __restrict__ off,
                                                    ShdDeliv* __restrict__ scr, uint32_t flo, uint32_t fhi) {
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
                r[k] = ld_ev(&in[i]);
                rk[k] = rank ? rank[i] : r[k].pad;
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const uint32_t d = r[k].dst_host - host_lo;
            if (ok[k] && d < H && d >= flo && d < fhi) st_ev(&scr[off[d] + rk[k]], r[k]);
        }
    }
}

// "slab" pipeline: the overflow events (slot >= kSlab of a destination with
// more than kSlab events) go to off[dst] + slot of the staging array, where
// k_segsort_dst has put the first kSlab slots.  Grid-stride over the device
// count, so the launch costs nothing when no segment overflowed.
__global__ __launch_bounds__(256) void k_place_ovf(const ShdDeliv* __restrict__ ovf, const uint32_t* __restrict__ novf,
                                                   const uint32_t* __restrict__ off, uint32_t host_lo,
                                                   ShdDeliv* __restrict__ scr) {
    const uint32_t m = *novf;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const ShdDeliv r = ld_ev(&ovf[i]);
        st_ev(&scr[off[r.dst_host - host_lo] + r.pad], r);
    }
}

// Regroup path, slab pipeline: each event in the host range takes its slot
// from its destination's counter and goes straight into the slab (or the
// overflow list); out-of-range events are dropped.
__global__ __launch_bounds__(256) void k_hist_slab(const ShdDeliv* __restrict__ in, size_t n, uint32_t host_lo,
                                                   uint32_t H, uint32_t* __restrict__ cnt, ShdDeliv* __restrict__ slab,
                                                   uint32_t slab_rm, ShdDeliv* __restrict__ ovf,
                                                   uint32_t* __restrict__ novf, uint32_t agg_on) {
    __shared__ uint32_t agg_s[3 * 256];
    const int lane = threadIdx.x & 63;
    const DestAgg agg{agg_s + 3 * (threadIdx.x & ~63u), agg_s + 3 * (threadIdx.x & ~63u) + 64,
                      agg_s + 3 * (threadIdx.x & ~63u) + 128, agg_on};
    agg.cnt[lane] = 0;
    __syncthreads();
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * kBatch) {
        ShdDeliv r[kBatch];
        bool ok[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const size_t i = i0 + (size_t)k * stride;
            ok[k] = i < n;
            if (ok[k]) r[k] = ld_ev(&in[i]);
            else r[k].dst_host = host_lo + H; // (out of range: takes no slot)
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const uint32_t d = r[k].dst_host - host_lo;
            const bool in = ok[k] && d < H;
            const uint32_t rank = dest_slot(in, d, cnt, agg, lane);
            const uint32_t oslot = wave_alloc(in && rank >= kSlab, novf, lane);
            if (!in) continue;
            r[k].pad = rank;
            if (rank < kSlab) st_ev(&slab[slab_rm ? (size_t)rank * H + d : (size_t)d * kSlab + rank], r[k]);
            else st_ev(&ovf[oslot], r[k]);
        }
    }
}

// One wave per destination segment of up to kSmallSeg events; larger ones go
// to the bitonic-in-HBM list.  With a slab (the "slab" pipeline) segment d's
// events are read from slab[d * kSlab ...]; a larger segment first copies its
// kSlab slab slots to the front of its staging range scr[off[d] ...].
//
// Slab pipeline, fused form (ovf != nullptr): the overflow events (slots >=
// kSlab of the listed segments, disjoint from the slab slots copied here) are
// placed by the same launch, as k_place_ovf would.  Guards (cheap, always on):
// an overflow event whose destination or slot falls outside its segment, or
// an overflow count above the list's capacity, is not stored and sets a bit
// of the round's fault word (nbig[2]), which the host reads back (-EIO).
template <int kNT = 0>
__global__ __launch_bounds__(256) void k_segsort_dst(ShdDeliv* __restrict__ scr, const uint32_t* __restrict__ off,
                                                     uint32_t H, uint32_t host_lo, ShdDeliv* __restrict__ out,
                                                     uint32_t* __restrict__ big, uint32_t* __restrict__ nbig,
                                                     uint32_t rsort, uint32_t flo, uint32_t fhi,
                                                     const ShdDeliv* __restrict__ slab, uint32_t slab_rm,
                                                     uint32_t lds_keys, const ShdDeliv* __restrict__ ovf,
                                                     uint32_t ovf_cap, uint32_t scr_cap,
                                                     const uint4* __restrict__ cslab, unsigned long long tbase) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    if (ovf) {
        // overflow events first: the listed segments' k_segsort_mid runs
        // after this launch, so the order inside the launch is free
        const uint32_t m = nbig[1];
        const uint32_t top = off[H];
        uint32_t flag = m > ovf_cap ? kFaultOvfCap : 0u;
        if (top > scr_cap) flag |= kFaultOff;
        for (uint32_t i = wave * 64 + lane; !flag && i < m; i += nwaves * 64) {
            const ShdDeliv r = ld_ev(&ovf[i]);
            const uint32_t d = r.dst_host - host_lo;
            if (d >= H || r.pad < kSlab || r.pad >= off[d + 1] - off[d]) {
                flag |= kFaultOvfRange;
                break;
            }
            st_ev(&scr[off[d] + r.pad], r);
        }
        if (flag) atomicOr(nbig + 2, flag);
    }
    // per-wave pass-1 key array of the rank sort (SHD_SEGSORT_LDS=0: readlanes)
    __shared__ unsigned long long keys[4][64 * 4 + 8];
    unsigned long long* lk = lds_keys ? keys[threadIdx.x >> 6] : nullptr;
    for (uint32_t d = flo + wave; d < fhi; d += nwaves) {
        const uint32_t b = off[d], n = off[d + 1] - b;
        const uint32_t dh = d + host_lo;
        if (n == 0) continue;
        if (slab && cslab) { // compact records (rank sort)
            const size_t base = slab_rm ? d : (size_t)d * kSlab, stride = slab_rm ? H : 1u;
            if (n <= kSlab) {
                auto load = [&](uint32_t i) {
                    return c_load<(kNT & 1) != 0>(cslab, slab, base + (size_t)i * stride, tbase);
                };
                if (n <= 64) wave_rank_segment<1, kNT / 2>(load, n, dh, out, b, lane, lk);
                else if (n <= 128) wave_rank_segment<2, kNT / 2>(load, n, dh, out, b, lane, lk);
                else wave_rank_segment<4, kNT / 2>(load, n, dh, out, b, lane, lk);
            } else {
                for (uint32_t i = lane; i < kSlab; i += 64) {
                    const Ev e = c_load(cslab, slab, base + (size_t)i * stride, tbase);
                    st_ev(&scr[b + i], ShdDeliv{e.t, e.q, e.s, dh, e.ix, i});
                }
                if (lane == 0) {
                    const uint32_t k = atomicAdd(nbig, 1u);
                    if (k < H) big[k] = d;
                    else atomicOr(nbig + 2, kFaultBigCap);
                }
            }
        } else if (slab) {
            const uint32_t base = slab_rm ? d : d * kSlab, stride = slab_rm ? H : 1u;
            if (n <= kSlab) {
                sort_segment(rsort, slab, base, nullptr, n, dh, out, b, lane, stride, lk);
            } else {
                for (uint32_t i = lane; i < kSlab; i += 64) st_ev(&scr[b + i], ld_ev(&slab[base + (size_t)i * stride]));
                if (lane == 0) {
                    const uint32_t k = atomicAdd(nbig, 1u);
                    if (k < H) big[k] = d;
                    else atomicOr(nbig + 2, kFaultBigCap);
                }
            }
        } else if (n <= (uint32_t)kSmallSeg) {
            sort_segment(rsort, scr, b, nullptr, n, dh, out, b, lane, 1u, lk);
        } else if (lane == 0) {
            const uint32_t k = atomicAdd(nbig, 1u);
            if (k < H) big[k] = d;
            else atomicOr(nbig + 2, kFaultBigCap);
        }
    }
}

// ---- multi-GPU regroup from destination-sorted runs ----
// After the destination-owner exchange, the W blocks a rank receives are
// each already grouped by destination and in event_compare order inside
// every destination (the senders' rounds sorted them).  rofs[k * (Hr + 1) +
// d] is destination d's start inside block k (relative to the block, which
// starts at bbase[k] in `in`).  The regroup reads the runs in place: no
// scatter into destination slabs, only the per-destination union of W runs.
constexpr uint32_t kMaxRuns = 64; // = xchg.hip kMaxWorld

// element i of a run-merge input: a ShdDeliv (kFmt 0) or a Wire (kFmt 1)
template <int kFmt>
__device__ __forceinline__ Ev ld_run(const void* in, uint32_t i) {
    if (kFmt == 1) return ld_wire(static_cast<const Wire*>(in) + i);
    const ShdDeliv r = ld_ev(static_cast<const ShdDeliv*>(in) + i);
    return Ev{r.time, r.seq, r.src_host, r.pkt_index};
}

__global__ __launch_bounds__(256) void k_runs_count(const uint32_t* __restrict__ rofs, uint32_t W, uint32_t Hr,
                                                    uint32_t* __restrict__ cnt) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < Hr; d += gridDim.x * blockDim.x) {
        uint32_t c = 0;
        for (uint32_t k = 0; k < W; k++) c += rofs[(size_t)k * (Hr + 1) + d + 1] - rofs[(size_t)k * (Hr + 1) + d];
        cnt[d] = c;
    }
}

// One wave per destination: its W runs (a run table in LDS: segment-local
// start and source index of each run) are read as one segment and ranked
// like a slab segment; segments above kSmallSeg events are copied to their
// final range of the staging array and listed for k_segsort_mid / _merge.
// (self < W: run `self` is read from in_self -- this rank's own block, never
// sent through the transport -- at its element index, the others from in)
template <int kFmt>
__global__ __launch_bounds__(256) void k_runs_sort(const void* __restrict__ in, const void* __restrict__ in_self,
                                                   uint32_t self, const uint32_t* __restrict__ rofs,
                                                   const uint32_t* __restrict__ bbase, uint32_t W, uint32_t Hr,
                                                   const uint32_t* __restrict__ off, uint32_t host_lo,
                                                   ShdDeliv* __restrict__ out, ShdDeliv* __restrict__ scr,
                                                   uint32_t* __restrict__ big, uint32_t* __restrict__ nbig,
                                                   uint32_t lds_keys) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + wv;
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    __shared__ unsigned long long keys[4][64 * 4 + 8];
    __shared__ uint32_t rs_all[4][kMaxRuns + 1], rb_all[4][kMaxRuns];
    uint32_t* rs = rs_all[wv];
    uint32_t* rb = rb_all[wv];
    unsigned long long* lk = lds_keys ? keys[wv] : nullptr;
    for (uint32_t d = wave; d < Hr; d += nwaves) {
        const uint32_t o = off[d], n = off[d + 1] - o;
        if (n == 0) continue;
        uint32_t len = 0, src = 0;
        if ((uint32_t)lane < W) {
            const uint32_t a = rofs[(size_t)lane * (Hr + 1) + d];
            len = rofs[(size_t)lane * (Hr + 1) + d + 1] - a;
            src = ((uint32_t)lane == self ? 0u : bbase[lane]) + a;
        }
        const uint32_t inc = wave_incl_scan(len, lane);
        if ((uint32_t)lane < W) {
            rs[lane] = inc - len;
            rb[lane] = src;
        }
        if (lane == 0) rs[W] = n;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        auto get = [&](uint32_t i) { // segment element i (i < n), from its run
            uint32_t k = 0;
            while (rs[k + 1] <= i) k++;
            return ld_run<kFmt>(k == self ? in_self : in, rb[k] + (i - rs[k]));
        };
        if (n <= (uint32_t)kSmallSeg) {
            auto load = [&](uint32_t i) { return get(i); };
            if (n <= 64) wave_rank_segment<1>(load, n, d + host_lo, out, o, lane, lk);
            else if (n <= 128) wave_rank_segment<2>(load, n, d + host_lo, out, o, lane, lk);
            else wave_rank_segment<4>(load, n, d + host_lo, out, o, lane, lk);
        } else {
            for (uint32_t i = lane; i < n; i += 64) {
                const Ev e = get(i);
                st_ev(&scr[o + i], ShdDeliv{e.t, e.q, e.s, d + host_lo, e.ix, 0u});
            }
            if (lane == 0) {
                const uint32_t k = atomicAdd(nbig, 1u);
                if (k < Hr) big[k] = d;
                else atomicOr(nbig + 2, kFaultBigCap);
            }
        }
        // the run table is rewritten for the next destination
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
}

// rank of x (element i of run k) in the union of sorted runs staged one
// after another in v (run j at [rs[j], rs[j+1])): its index in its run +
// the elements before it in every other run, ties to the lower run (the
// union's stable order).  The binary searches of 8 runs at a time step in
// lockstep: their LDS reads are independent, so one step costs one LDS
// round trip instead of eight (the searches are latency-bound).
// With packed keys (pk != nullptr: pk[i] = (t - tmin) << 24 | src, distinct
// unless time AND sender are equal) a step reads one 8-B key instead of the
// 24-B event, and the event only on a key tie.
__device__ __forceinline__ uint32_t merged_rank(const Ev* v, const uint32_t* rs, uint32_t W, uint32_t k, uint32_t i,
                                                const Ev& x, const unsigned long long* pk = nullptr,
                                                unsigned long long kx = 0) {
    uint32_t rank = i - rs[k];
    for (uint32_t j0 = 0; j0 < W; j0 += 8) {
        uint32_t lo[8], hi[8], b0[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t j = j0 + u;
            const bool on = j < W && j != k;
            lo[u] = b0[u] = on ? rs[j] : 0u;
            hi[u] = on ? rs[j + 1] : 0u;
        }
        for (bool any = true; any;) {
            any = false;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                if (lo[u] < hi[u]) {
                    const uint32_t mid = (lo[u] + hi[u]) >> 1;
                    bool after;
                    const unsigned long long ky = pk ? pk[mid] : 0ull;
                    if (pk && ky != kx) {
                        after = ky < kx;
                    } else {
                        const Ev y = v[mid];
                        after = j0 + u < k ? !ev_lt(x, y) : ev_lt(y, x);
                    }
                    lo[u] = after ? mid + 1 : lo[u];
                    hi[u] = after ? hi[u] : mid;
                    any = true;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) rank += lo[u] - b0[u];
    }
    return rank;
}

__device__ __forceinline__ void st_deliv_nt(ShdDeliv* p, const Ev& x, uint32_t dh) {
    shd_v4u* q = reinterpret_cast<shd_v4u*>(p);
    const shd_v4u a0 = {(uint32_t)x.t, (uint32_t)(x.t >> 32), (uint32_t)x.q, (uint32_t)(x.q >> 32)};
    const shd_v4u a1 = {x.s, dh, x.ix, 0u};
    __builtin_nontemporal_store(a0, q);
    __builtin_nontemporal_store(a1, q + 1);
}

// The merge of sorted runs for segments of up to kSmallSeg events: one wave
// per destination, its runs staged in the wave's LDS, every element placed
// by merged_rank (no workgroup barrier; k_runs_merge takes the longer ones).
template <int kFmt>
__global__ __launch_bounds__(256) void k_runs_merge_wave(const void* __restrict__ in, const void* __restrict__ in_self,
                                                         uint32_t self, const uint32_t* __restrict__ rofs,
                                                         const uint32_t* __restrict__ bbase, uint32_t W, uint32_t Hr,
                                                         const uint32_t* __restrict__ off, uint32_t host_lo,
                                                         ShdDeliv* __restrict__ out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + wv;
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    __shared__ Ev sv_all[4][kSmallSeg];
    __shared__ uint16_t inv_all[4][kSmallSeg];
    __shared__ uint32_t rs_all[4][kMaxRuns + 1], rb_all[4][kMaxRuns];
    Ev* v = sv_all[wv];
    uint16_t* inv = inv_all[wv];
    uint32_t* rs = rs_all[wv];
    uint32_t* rb = rb_all[wv];
    for (uint32_t d = wave; d < Hr; d += nwaves) {
        const uint32_t o = off[d], n = off[d + 1] - o;
        if (n == 0 || n > (uint32_t)kSmallSeg) continue; // (longer: k_runs_merge's)
        uint32_t len = 0, src = 0;
        if ((uint32_t)lane < W) {
            const uint32_t a = rofs[(size_t)lane * (Hr + 1) + d];
            len = rofs[(size_t)lane * (Hr + 1) + d + 1] - a;
            src = ((uint32_t)lane == self ? 0u : bbase[lane]) + a;
        }
        const uint32_t inc = wave_incl_scan(len, lane);
        if ((uint32_t)lane < W) {
            rs[lane] = inc - len;
            rb[lane] = src;
        }
        if (lane == 0) rs[W] = n;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        uint32_t kk[kSmallSeg / 64];
#pragma unroll
        for (int j = 0; j < kSmallSeg / 64; j++) {
            const uint32_t i = lane + 64 * j;
            uint32_t k = 0;
            if (i < n) {
                while (rs[k + 1] <= i) k++;
                v[i] = ld_run<kFmt>(k == self ? in_self : in, rb[k] + (i - rs[k]));
            }
            kk[j] = k;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        // the permutation in LDS, then the segment written in order (whole
        // lines, not 32-B pieces scattered over the segment)
#pragma unroll
        for (int j = 0; j < kSmallSeg / 64; j++) {
            const uint32_t i = lane + 64 * j;
            if (i < n) inv[merged_rank(v, rs, W, kk[j], i, v[i])] = (uint16_t)i;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t dh = d + host_lo;
        for (uint32_t p = lane; p < n; p += 64) st_deliv_nt(&out[o + p], v[inv[p]], dh);
        // the run table and the stage are rewritten for the next destination
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
}

// The owner's merge when every run is sorted (the senders' sorted wire, or
// their sorted rounds), segments above kSmallSeg events: one workgroup per
// destination, a pairwise merge tree over its W runs in LDS -- each level
// places every element at its index in its run + its rank in the partner run
// (one binary search: ties to the lower run, the union's stable order), so an
// element costs log2(W) searches instead of W - 1 (8 runs: ≈24 key reads
// instead of ≈56).  The searches compare packed 8-B keys (t - tmin) << 24 |
// src (the events, re-read from the input, only on a key tie); LDS holds
// keys, indices and each element's input position (24 KiB: six workgroups per
// CU), and the sorted segment is written from the input in order.  A segment
// whose time span or sender ids do not pack, or above kMergeMax events, goes
// unsorted to the staging array and is listed, as in k_runs_sort.
constexpr uint32_t kMergeMax = 1024;
constexpr uint32_t kMergeThreads = 256; // (512: 240 vs 192 us per 8-rank owner merge, profiles/r04av_…)
template <int kFmt>
__global__ __launch_bounds__(kMergeThreads) void k_runs_merge(const void* __restrict__ in, const void* __restrict__ in_self,
                                                    uint32_t self, const uint32_t* __restrict__ rofs,
                                                    const uint32_t* __restrict__ bbase, uint32_t W, uint32_t Hr,
                                                    const uint32_t* __restrict__ off, uint32_t host_lo,
                                                    ShdDeliv* __restrict__ out, ShdDeliv* __restrict__ scr,
                                                    uint32_t* __restrict__ big, uint32_t* __restrict__ nbig,
                                                    uint32_t probe) {
    constexpr int kPer = (int)(kMergeMax / kMergeThreads);
    __shared__ unsigned long long kbuf[2][kMergeMax];
    __shared__ uint16_t ibuf[2][kMergeMax];
    __shared__ uint32_t sa[kMergeMax]; // element -> its input position (bit 31: this rank's own block)
    __shared__ uint32_t rs[kMaxRuns + 1], rb[kMaxRuns];
    __shared__ unsigned long long red[3][kMergeThreads / 64];
    const uint32_t tid = threadIdx.x;
    auto ld_at = [&](uint32_t a) { return ld_run<kFmt>((a >> 31) ? in_self : in, a & 0x7fffffffu); };
    // (the destinations above kSmallSeg events, found by scanning: listing
    // them with one counter would serialise an atomic per destination)
    for (uint32_t d = blockIdx.x; d < Hr; d += gridDim.x) {
        const uint32_t o = off[d], n = off[d + 1] - o;
        if (n <= (uint32_t)kSmallSeg) continue; // (block-uniform)
        if (tid < 64) {
            uint32_t len = 0, src = 0;
            if (tid < W) {
                const uint32_t a = rofs[(size_t)tid * (Hr + 1) + d];
                len = rofs[(size_t)tid * (Hr + 1) + d + 1] - a;
                src = (tid == self ? 0u : bbase[tid]) + a;
            }
            const uint32_t inc = wave_incl_scan(len, (int)tid);
            if (tid < W) {
                rs[tid] = inc - len;
                rb[tid] = src;
            }
            if (tid == 0) rs[W] = n;
        }
        __syncthreads();
        auto run_of = [&](uint32_t i) {
            uint32_t k = 0;
            while (rs[k + 1] <= i) k++;
            return k;
        };
        const uint32_t dh = d + host_lo;
        bool listed = n > kMergeMax; // (block-uniform)
        Ev ev[kPer];
        uint32_t ea[kPer];
        if (!listed) {
            unsigned long long tmn = ~0ull, tmx = 0ull, smx = 0ull;
#pragma unroll
            for (int e = 0; e < kPer; e++) {
                const uint32_t i = tid + kMergeThreads * e;
                if (i < n) {
                    const uint32_t k = run_of(i);
                    ea[e] = (k == self ? 0x80000000u : 0u) | (rb[k] + (i - rs[k]));
                    ev[e] = ld_at(ea[e]);
                    tmn = ev[e].t < tmn ? ev[e].t : tmn;
                    tmx = ev[e].t > tmx ? ev[e].t : tmx;
                    smx = ev[e].s > smx ? ev[e].s : smx;
                }
            }
            tmn = wave_min_u64(tmn);
            tmx = wave_max_u64(tmx);
            smx = wave_max_u64(smx);
            if ((tid & 63) == 0) red[0][tid >> 6] = tmn, red[1][tid >> 6] = tmx, red[2][tid >> 6] = smx;
            __syncthreads();
            unsigned long long a = red[0][0], bx = red[1][0], cx = red[2][0];
#pragma unroll
            for (int q = 1; q < (int)(kMergeThreads / 64); q++) {
                a = red[0][q] < a ? red[0][q] : a;
                bx = red[1][q] > bx ? red[1][q] : bx;
                cx = red[2][q] > cx ? red[2][q] : cx;
            }
            listed = !(bx - a < (1ull << 40) && cx < (1ull << 24)); // (the keys do not pack: listed)
            if (!listed)
#pragma unroll
                for (int e = 0; e < kPer; e++) {
                    const uint32_t i = tid + kMergeThreads * e;
                    if (i < n) {
                        kbuf[0][i] = ((ev[e].t - a) << 24) | ev[e].s;
                        ibuf[0][i] = (uint16_t)i;
                        sa[i] = ea[e];
                    }
                }
        }
        if (listed) { // unsorted (runs one after another) to the staging array, listed
            for (uint32_t i = tid; i < n; i += kMergeThreads) {
                const uint32_t k = run_of(i);
                const Ev e = ld_run<kFmt>(k == self ? in_self : in, rb[k] + (i - rs[k]));
                st_ev(&scr[o + i], ShdDeliv{e.t, e.q, e.s, dh, e.ix, 0u});
            }
            if (tid == 0) {
                const uint32_t k = atomicAdd(nbig, 1u);
                if (k < Hr) big[k] = d;
                else atomicOr(nbig + 2, kFaultBigCap);
            }
            __syncthreads();
            continue;
        }
        __syncthreads();
        // the merge tree: runs [rs[r], rs[r+1]) of the current buffer, pairs
        // (2q, 2q + 1) merged into the other buffer, the boundaries halved
        int cur = 0;
        for (uint32_t R = W; R > 1 && !(probe & 1u); R = (R + 1) >> 1) {
            for (uint32_t i = tid; i < n; i += kMergeThreads) {
                const unsigned long long kx = kbuf[cur][i];
                const uint16_t ix = ibuf[cur][i];
                uint32_t r = 0;
                while (rs[r + 1] <= i) r++;
                const uint32_t p = r ^ 1u;
                uint32_t pos = i;
                if (p < R) {
                    // left element (r even): partner elements strictly before it;
                    // right element: partner elements before or equal (ties: left first)
                    const bool left = (r & 1u) == 0;
                    uint32_t lo = rs[p], hi = rs[p + 1];
                    const uint32_t base = lo;
                    bool have_x = false;
                    Ev ex;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        const unsigned long long ky = kbuf[cur][mid];
                        bool before;
                        if (ky != kx) {
                            before = ky < kx;
                        } else { // a key tie: the events decide
                            if (!have_x) ex = ld_at(sa[ix]), have_x = true;
                            const Ev ey = ld_at(sa[ibuf[cur][mid]]);
                            before = left ? ev_lt(ey, ex) : !ev_lt(ex, ey);
                        }
                        if (before) lo = mid + 1;
                        else hi = mid;
                    }
                    pos = rs[r & ~1u] + (i - rs[r]) + (lo - base);
                }
                kbuf[cur ^ 1][pos] = kx;
                ibuf[cur ^ 1][pos] = ix;
            }
            __syncthreads();
            if (tid == 0) {
                const uint32_t R2 = (R + 1) >> 1;
                for (uint32_t q = 1; q < R2; q++) rs[q] = rs[2 * q];
                rs[R2] = n;
            }
            cur ^= 1;
            __syncthreads();
        }
        for (uint32_t p = tid; p < n; p += kMergeThreads) st_deliv_nt(&out[o + p], ld_at(sa[ibuf[cur][p]]), dh);
        __syncthreads();
    }
}

// The sender's side of a round that is exchanged next
// (shd_round_process_exchange): the decided events grouped by destination
// -- slab slots, then the overflow events at their ranks -- copied to the
// wire array at off[d], unsorted: the owner sorts the union of the runs it
// receives anyway (k_runs_sort), so the sender's segment sort is skipped.
__global__ __launch_bounds__(256) void k_group_wire(const ShdDeliv* __restrict__ slab, uint32_t slab_rm, uint32_t H,
                                                    const uint32_t* __restrict__ off, const ShdDeliv* __restrict__ ovf,
                                                    const uint32_t* __restrict__ nbig, uint32_t* __restrict__ fault,
                                                    uint32_t ovf_cap, Wire* __restrict__ wire,
                                                    const uint4* __restrict__ cslab, unsigned long long tbase) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const uint32_t m = nbig[1];
    if (m > ovf_cap) {
        if (wave == 0 && lane == 0) atomicOr(fault, kFaultOvfCap);
    } else {
        for (uint32_t i = wave * 64 + lane; i < m; i += nwaves * 64) {
            const ShdDeliv r = ld_ev(&ovf[i]);
            if (r.dst_host >= H || r.pad < kSlab || r.pad >= off[r.dst_host + 1] - off[r.dst_host]) {
                atomicOr(fault, kFaultOvfRange);
                continue;
            }
            st_wire(&wire[off[r.dst_host] + r.pad], r.time, r.seq, r.src_host, r.pkt_index);
        }
    }
    for (uint32_t d = wave; d < H; d += nwaves) {
        const uint32_t b = off[d], n = off[d + 1] - b;
        const uint32_t k = n < kSlab ? n : kSlab;
        const size_t base = slab_rm ? d : (size_t)d * kSlab, stride = slab_rm ? H : 1u;
        for (uint32_t i = lane; i < k; i += 64) {
            if (cslab) {
                const Ev e = c_load(cslab, slab, base + (size_t)i * stride, tbase);
                st_wire(&wire[b + i], e.t, e.q, e.s, e.ix);
            } else {
                const ShdDeliv r = ld_ev(&slab[base + (size_t)i * stride]);
                st_wire(&wire[b + i], r.time, r.seq, r.src_host, r.pkt_index);
            }
        }
    }
}

// ---- "part" pipeline: LDS-staged bucket partition, then one LDS sort per bucket ----
// The slab pipeline's scatter pays two random HBM requests per delivered
// event beyond the table gather: the destination counter's atomic and a 16-B
// partial-line store into a 147 MB slab (profiles/r04a_ubench_part.log: the
// gather floor 0.318 ms, with the slab form 0.573 ms).  Here:
//   k_part_scatter  a workgroup decides 4,096 records (the scatter's decision,
//                   unchanged), stages its delivered events in LDS (16 B
//                   each), counts them per destination BUCKET of 2^shift hosts,
//                   reserves one run per nonempty bucket with one atomic on
//                   the bucket's counter, and writes its runs in bucket order
//                   (consecutive lanes store consecutive records) into the
//                   bucket's region of the stage: bucket b at [b * cap, ...).
//   k_part_sort     one workgroup per bucket: its events into registers, a
//                   count per destination (LDS), the bucket's output base (the
//                   sum of the earlier buckets' totals) and the destination
//                   offsets, the events placed into LDS grouped by
//                   destination, then one wave per destination segment ranks
//                   it by event_compare (wave_rank_segment) and writes it at
//                   its final place -- no slab, no separate scan or sort pass.
// Stage record (16 B): {time - tbase, srcHostEventID, pkt_index, src << shift
// | destination - bucket base}.  An event that does not fit it (time offset
// or srcHostEventID of 32 bits or more, src >= 2^(32 - shift)) or that finds
// its bucket's region full goes whole to the wide list (and counts in wcnt[b]);
// a bucket with wide events, or with more events than k_part_sort holds in
// LDS, takes the listed path: its events are placed unsorted at their
// destination ranges of the staging array and every segment is listed for
// k_segsort_mid / k_segsort_merge (skewed destinations).
constexpr uint32_t kPartMaxDst = 64; // destinations per bucket (shift <= 6)
constexpr uint32_t kPartMaxBuckets = 16384; // register-staged scatter: 8 B of LDS per bucket
constexpr uint32_t kTinySeg = 16;           // part sort: segments ranked one thread per event
constexpr uint32_t kPartMaxBucketsLds = 4096; // LDS-staged scatter: + 20 B per record

struct PartGeo {
    uint32_t host_lo, H; // destination host range
    uint32_t shift, nb;  // bucket = (dst - host_lo) >> shift
    uint32_t cap;        // stage records per bucket
    unsigned long long tbase;
    uint32_t b0 = 0;     // the sorts: first bucket of the launch (blockIdx.x + b0)
    uint32_t xbar = 0x80000000u; // the barrier's time offset (barrier - tbase)
};

__device__ __forceinline__ uint32_t block_excl_scan_n(uint32_t v, uint32_t* total, uint32_t* ws) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int k = 0; k < nw; k++) {
        if (k < w) base += ws[k];
        tot += ws[k];
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// kWG threads decide kCH records (kCH / kWG per thread, in batches of 4).
// kLds: the delivered events are staged in LDS and written in bucket order
// (consecutive lanes, consecutive records of a run); else each thread keeps
// its events in registers and stores them at their run positions itself (LDS
// holds only the bucket counts: more workgroups per CU).
// kProbe (SHD_PART_PROBE, measurement only -- outputs deliberately wrong), a
// bit set: 1 no table gather, 2 no run-reservation atomics, 4 no stage
// stores, 8 no host->slot gathers
// kOcc: waves per SIMD the registers are sized for (0: the compiler's
// choice -- 71 VGPRs, one 1,024-thread workgroup per CU; 8: two per CU, with
// spills)
template <int kWG, int kCH, bool kLds, int kProbe = 0, int kOcc = 0>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(kOcc ? kOcc : 4, 8))) void k_part_scatter(ShdPktCtx c, const ShdPkt* __restrict__ recs, size_t n,
                                                      uint64_t barrier, uint64_t end_time, uint64_t boot_end,
                                                      PartGeo g, uint4* __restrict__ stage,
                                                      uint32_t* __restrict__ gcnt, uint32_t* __restrict__ wcnt,
                                                      uint8_t* __restrict__ status, unsigned long long* counters,
                                                      ShdDeliv* __restrict__ wide, uint32_t* __restrict__ nwide,
                                                      uint32_t ch) {
    constexpr int kB = 4;
    constexpr int kR = kCH / kWG; // records per thread
    static_assert(kCH % (kWG * kB) == 0, "chunk");
    extern __shared__ uint4 part_smem[];
    // kLds: ev[kCH] | rk[kCH] u16 | perm[kCH] u16 | hist[nb] | lofs[nb + 1] | gb[nb]; else hist[nb] | gb[nb]
    uint4* ev = part_smem;
    uint16_t* rk = reinterpret_cast<uint16_t*>(ev + (kLds ? kCH : 0));
    uint16_t* perm = rk + (kLds ? kCH : 0);
    uint32_t* hist = reinterpret_cast<uint32_t*>(perm + (kLds ? kCH : 0));
    uint32_t* lofs = hist + g.nb;
    uint32_t* gb = kLds ? lofs + g.nb + 1 : hist + g.nb;
    __shared__ uint32_t wsum[kWG / 64];
    __shared__ unsigned long long wmin[kWG / 64];
    const int lane = threadIdx.x & 63;
    for (uint32_t b = threadIdx.x; b < g.nb; b += kWG) hist[b] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * ch; // (ch <= kCH records per workgroup, see part_front)
    const size_t A = (size_t)c.A;
    const uint2* __restrict__ host_info = reinterpret_cast<const uint2*>(c.host_info);
    const uint2* __restrict__ ptab = reinterpret_cast<const uint2*>(c.ptab);
    const uint32_t smax = g.shift ? (0xFFFFFFFFu >> g.shift) : 0xFFFFFFFFu; // src hosts that fit the record
    const uint32_t mask = (1u << g.shift) - 1u;
    unsigned long long mn = ~0ull;
    uint4 rv[kLds ? 1 : kR]; // register staging: {record fields..., dst}, w = ~0: none
    uint32_t rr[kLds ? 1 : kR];
    for (int k0 = 0; k0 < kR; k0 += kB) {
        ShdPkt p[kB];
        bool live[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const size_t i = base + (size_t)(k0 + k) * kWG + threadIdx.x;
            live[k] = (uint32_t)((k0 + k) * kWG + threadIdx.x) < ch && i < n;
            if (live[k]) p[k] = ld_pkt(&recs[i]);
        }
        int si[kB], di[kB];
        uint32_t ts[kB], td[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const bool known = live[k] && p[k].src_host < c.nhosts && p[k].dst_host < c.nhosts;
            uint2 hs = make_uint2(~0u, ~0u), hd = make_uint2(~0u, ~0u);
            if (known && (kProbe & 8)) {
                hs = make_uint2(p[k].src_host % (uint32_t)A, 0u);
                hd = make_uint2(p[k].dst_host % (uint32_t)A, 1u);
            } else if (known) {
                hs = host_info[p[k].src_host];
                hd = host_info[p[k].dst_host];
            }
            si[k] = hs.x == ~0u ? -1 : (int)hs.x;
            di[k] = hd.x == ~0u ? -1 : (int)hd.x;
            ts[k] = hs.y;
            td[k] = hd.y;
        }
        size_t ei[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            int oi = si[k], oj = di[k];
            if (oi >= 0 && oj >= 0) {
                if (c.mode == 0) {
                    if (oi != oj && td[k] < ts[k]) oi = di[k], oj = si[k]; // owner: row touched first
                } else if (c.mode == 2) {
                    const size_t b = (size_t)oi * A + (size_t)oj;
                    if (!((c.pair_bits[b >> 5] >> (b & 31)) & 1u)) oi = di[k], oj = si[k];
                }
            }
            if (oi < c.row_lo || oi >= c.row_hi) si[k] = -1; // another rank's row: not decided here
            ei[k] = (size_t)(oi < 0 ? 0 : oi) * A + (size_t)(oj < 0 ? 0 : oj);
        }
        ShdEntry e[kB];
        uint2 q[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            q[k] = make_uint2((kProbe & 1) ? 1000000u : kPtabFallback, (kProbe & 1) ? 0xFFFFFFFFu : 0u);
            if (!(kProbe & 1) && ptab && si[k] >= 0 && di[k] >= 0) {
                const unsigned long long v =
                    __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(ptab) + ei[k]);
                q[k] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
            }
        }
#pragma unroll
        for (int k = 0; k < kB; k++)
            if (si[k] >= 0 && di[k] >= 0 && q[k].x == kPtabFallback) e[k] = c.tab[ei[k]];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const uint32_t li = (uint32_t)((k0 + k) * kWG + threadIdx.x);
            uint8_t st = 0xff; // unregistered host: not delivered
            uint64_t t = 0;
            if (live[k] && si[k] >= 0 && di[k] >= 0) {
                uint32_t rs = p[k].rng_state;
                const uint32_t r = (uint32_t)glibc_rand_r(&rs);
                bool keep;
                uint64_t delay;
                if (q[k].x != kPtabFallback) {
                    keep = r <= q[k].y; // == (chance <= rel), see kPtabFallback
                    delay = q[k].x;
                } else {
                    keep = (double)r / 2147483647.0 <= e[k].rel; // random_nextDouble, worker.c:545
                    delay = (uint64_t)ceil(e[k].lat * 1000000.0);
                }
                st = SHD_DROPPED_LOSS;
                if (p[k].now < boot_end || keep || p[k].payload_len == 0) {
                    t = p[k].now + delay;                                   // worker.c:548-549
                    if (t >= end_time) st = SHD_DROPPED_END;                // scheduler.c:236-239
                    else {
                        if (p[k].src_host != p[k].dst_host && t < barrier) t = barrier; // host_single.c:187-192
                        st = SHD_DELIVERED;
                    }
                    // topology_incrementPathPacketCounter (worker.c:551): every kept packet
                    // at its answering pair (SHD_PCNT=atomic: a memory-side atomic each)
                    if (c.pcnt) atomicAdd(c.pcnt + ei[k], 1u);
                }
            }
            if (live[k]) pcnt_log(c, base + li, st == SHD_DELIVERED || st == SHD_DROPPED_END, ei[k]);
            const bool dl = st == SHD_DELIVERED;
            const uint32_t dr = p[k].dst_host - g.host_lo;
            const bool fits = dl && c_fits(t, g.tbase, p[k].seq) && p[k].src_host <= smax && dr < g.H;
            uint4 sv = make_uint4(0u, 0u, 0u, ~0u);
            uint32_t rank = 0;
            if (fits) {
                rank = atomicAdd(&hist[dr >> g.shift], 1u); // LDS
                sv = make_uint4((uint32_t)(t - g.tbase), (uint32_t)p[k].seq, p[k].src_host, p[k].dst_host);
            }
            if (kLds) {
                ev[li] = sv;
                if (fits) rk[li] = (uint16_t)rank;
            } else {
                rv[kLds ? 0 : k0 + k] = sv;
                rr[kLds ? 0 : k0 + k] = rank;
            }
            const uint32_t ws = wave_alloc(dl && !fits, nwide, lane); // (every lane: ballot)
            if (dl && !fits) {
                st_ev(&wide[ws], ShdDeliv{t, p[k].seq, p[k].src_host, p[k].dst_host, (uint32_t)(base + li) + c.idx_base,
                                          0u});
                if (dr < g.H) atomicAdd(&wcnt[dr >> g.shift], 1u);
            }
            if (dl && t >= barrier && t < mn) mn = t; // worker.c:350-363
            if (live[k]) status[base + li] = st;
        }
    }
    __syncthreads();
    // one run per nonempty bucket (and, with LDS staging, bucket order inside the workgroup)
    if (kLds) {
        const uint32_t per = (g.nb + kWG - 1) / kWG, b0 = threadIdx.x * per;
        uint32_t sum = 0;
        for (uint32_t k = 0; k < per && b0 + k < g.nb; k++) sum += hist[b0 + k];
        uint32_t tot;
        uint32_t pre = block_excl_scan_n(sum, &tot, wsum);
        for (uint32_t k = 0; k < per && b0 + k < g.nb; k++) {
            const uint32_t h = hist[b0 + k];
            lofs[b0 + k] = pre;
            gb[b0 + k] = h ? atomicAdd(&gcnt[b0 + k], h) : 0u;
            pre += h;
        }
        if (threadIdx.x == 0) lofs[g.nb] = tot;
    } else {
        for (uint32_t b = threadIdx.x; b < g.nb; b += kWG) {
            const uint32_t h = hist[b];
            if ((kProbe & 2)) gb[b] = (blockIdx.x * 37u + b) % (g.cap > 64 ? g.cap - 64 : 1u);
            else gb[b] = h ? atomicAdd(&gcnt[b], h) : 0u;
        }
    }
    __syncthreads();
    auto put = [&](bool valid, const uint4& e, uint32_t li, size_t j) { // (every lane: ballot inside)
        const uint32_t b = valid ? (e.w - g.host_lo) >> g.shift : 0u;
        const bool in = valid && j < g.cap;
        if (in && !(kProbe & 4)) // runs of a bucket, consecutive records
            stage[(size_t)b * g.cap + j] =
                make_uint4(e.x, e.y, (uint32_t)(base + li) + c.idx_base, (e.z << g.shift) | ((e.w - g.host_lo) & mask));
        const bool full = valid && !in; // the bucket's region is full: whole event to the wide list
        const uint32_t ws = wave_alloc(full, nwide, lane);
        if (full) {
            st_ev(&wide[ws], ShdDeliv{g.tbase + e.x, (unsigned long long)e.y, e.z, e.w,
                                      (uint32_t)(base + li) + c.idx_base, 0u});
            atomicAdd(&wcnt[b], 1u);
        }
    };
    if (kLds) {
        for (uint32_t li = threadIdx.x; li < (uint32_t)kCH; li += kWG) {
            const uint32_t w = ev[li].w;
            if (w != ~0u) perm[lofs[(w - g.host_lo) >> g.shift] + rk[li]] = (uint16_t)li;
        }
        __syncthreads();
        const uint32_t total = lofs[g.nb];
        for (uint32_t p0 = 0; p0 < total; p0 += kWG) { // (uniform trip count)
            const uint32_t pp = p0 + threadIdx.x;
            const bool valid = pp < total;
            uint4 e = make_uint4(0u, 0u, 0u, 0u);
            uint32_t li = 0;
            size_t j = 0;
            if (valid) {
                li = perm[pp];
                e = ev[li];
                const uint32_t b = (e.w - g.host_lo) >> g.shift;
                j = (size_t)gb[b] + (pp - lofs[b]);
            }
            put(valid, e, li, j);
        }
    } else {
#pragma unroll
        for (int k = 0; k < (kLds ? 1 : kR); k++) {
            const bool valid = rv[k].w != ~0u;
            const size_t j = valid ? (size_t)gb[(rv[k].w - g.host_lo) >> g.shift] + rr[k] : 0;
            put(valid, rv[k], (uint32_t)(k * kWG + threadIdx.x), j);
        }
    }
    mn = wave_min_u64(mn);
    if (lane == 0) wmin[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int k = 1; k < kWG / 64; k++) m = wmin[k] < m ? wmin[k] : m;
        if (m != ~0ull) atomicMin(&counters[1], m);
    }
}

// The split scatter (SHD_PART_SCATTER=10): the decision and the partition
// as two kernels.  k_part_decide makes the decision of k_part_scatter
// (identical code path: gathers, rand_r, drop, ceil delay, end-time drop,
// barrier clamp, status, counter log, wide list, min time) in small
// workgroups with no LDS and few registers, so that many waves per SIMD keep
// the table gathers and the record stream in flight together, and writes
// each record's 16-B stage form {time - tbase, seq, src, dst} (w = ~0: not
// staged) in record order -- coalesced.  k_part_place then reads those in
// chunks of kCH and does k_part_scatter's bucket counting, run reservation
// and run stores.  (The one-kernel form waits for each workgroup's gathers
// and then does everything else, one 1,024-thread workgroup per CU: the
// probes add up, profiles/r05g_part_scatter_probe_bits.log.)
template <int kWG, int kB>
__global__ __launch_bounds__(kWG) void k_part_decide(ShdPktCtx c, const ShdPkt* __restrict__ recs, size_t n,
                                                     uint64_t barrier, uint64_t end_time, uint64_t boot_end, PartGeo g,
                                                     uint4* __restrict__ dec, uint32_t* __restrict__ wcnt,
                                                     uint8_t* __restrict__ status, unsigned long long* counters,
                                                     ShdDeliv* __restrict__ wide, uint32_t* __restrict__ nwide) {
    __shared__ unsigned long long wmin[kWG / 64];
    const int lane = threadIdx.x & 63;
    const size_t base = (size_t)blockIdx.x * (kWG * kB);
    const size_t A = (size_t)c.A;
    const uint2* __restrict__ host_info = reinterpret_cast<const uint2*>(c.host_info);
    const uint2* __restrict__ ptab = reinterpret_cast<const uint2*>(c.ptab);
    const uint32_t smax = g.shift ? (0xFFFFFFFFu >> g.shift) : 0xFFFFFFFFu;
    unsigned long long mn = ~0ull;
    ShdPkt p[kB];
    bool live[kB];
#pragma unroll
    for (int k = 0; k < kB; k++) {
        const size_t i = base + (size_t)k * kWG + threadIdx.x;
        live[k] = i < n;
        if (live[k]) p[k] = ld_pkt(&recs[i]);
    }
    int si[kB], di[kB];
    uint32_t ts[kB], td[kB];
#pragma unroll
    for (int k = 0; k < kB; k++) {
        const bool known = live[k] && p[k].src_host < c.nhosts && p[k].dst_host < c.nhosts;
        uint2 hs = make_uint2(~0u, ~0u), hd = make_uint2(~0u, ~0u);
        if (known) {
            hs = host_info[p[k].src_host];
            hd = host_info[p[k].dst_host];
        }
        si[k] = hs.x == ~0u ? -1 : (int)hs.x;
        di[k] = hd.x == ~0u ? -1 : (int)hd.x;
        ts[k] = hs.y;
        td[k] = hd.y;
    }
    size_t ei[kB];
#pragma unroll
    for (int k = 0; k < kB; k++) {
        int oi = si[k], oj = di[k];
        if (oi >= 0 && oj >= 0) {
            if (c.mode == 0) {
                if (oi != oj && td[k] < ts[k]) oi = di[k], oj = si[k]; // owner: row touched first
            } else if (c.mode == 2) {
                const size_t b = (size_t)oi * A + (size_t)oj;
                if (!((c.pair_bits[b >> 5] >> (b & 31)) & 1u)) oi = di[k], oj = si[k];
            }
        }
        if (oi < c.row_lo || oi >= c.row_hi) si[k] = -1; // another rank's row: not decided here
        ei[k] = (size_t)(oi < 0 ? 0 : oi) * A + (size_t)(oj < 0 ? 0 : oj);
    }
    ShdEntry e[kB];
    uint2 q[kB];
#pragma unroll
    for (int k = 0; k < kB; k++) {
        q[k] = make_uint2(kPtabFallback, 0u);
        if (ptab && si[k] >= 0 && di[k] >= 0) {
            const unsigned long long v = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(ptab) + ei[k]);
            q[k] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
        }
    }
#pragma unroll
    for (int k = 0; k < kB; k++)
        if (si[k] >= 0 && di[k] >= 0 && q[k].x == kPtabFallback) e[k] = c.tab[ei[k]];
#pragma unroll
    for (int k = 0; k < kB; k++) {
        const size_t i = base + (size_t)k * kWG + threadIdx.x;
        uint8_t st = 0xff; // unregistered host: not delivered
        uint64_t t = 0;
        if (live[k] && si[k] >= 0 && di[k] >= 0) {
            uint32_t rs = p[k].rng_state;
            const uint32_t r = (uint32_t)glibc_rand_r(&rs);
            bool keep;
            uint64_t delay;
            if (q[k].x != kPtabFallback) {
                keep = r <= q[k].y; // == (chance <= rel), see kPtabFallback
                delay = q[k].x;
            } else {
                keep = (double)r / 2147483647.0 <= e[k].rel; // random_nextDouble, worker.c:545
                delay = (uint64_t)ceil(e[k].lat * 1000000.0);
            }
            st = SHD_DROPPED_LOSS;
            if (p[k].now < boot_end || keep || p[k].payload_len == 0) {
                t = p[k].now + delay;                                   // worker.c:548-549
                if (t >= end_time) st = SHD_DROPPED_END;                // scheduler.c:236-239
                else {
                    if (p[k].src_host != p[k].dst_host && t < barrier) t = barrier; // host_single.c:187-192
                    st = SHD_DELIVERED;
                }
                if (c.pcnt) atomicAdd(c.pcnt + ei[k], 1u); // (SHD_PCNT=atomic) worker.c:551
            }
        }
        if (live[k]) pcnt_log(c, i, st == SHD_DELIVERED || st == SHD_DROPPED_END, ei[k]);
        const bool dl = st == SHD_DELIVERED;
        const uint32_t dr = p[k].dst_host - g.host_lo;
        const bool fits = dl && c_fits(t, g.tbase, p[k].seq) && p[k].src_host <= smax && dr < g.H;
        if (live[k]) {
            const shd_v4u sv = fits ? shd_v4u{(uint32_t)(t - g.tbase), (uint32_t)p[k].seq, p[k].src_host, p[k].dst_host}
                                    : shd_v4u{0u, 0u, 0u, ~0u};
            *reinterpret_cast<shd_v4u*>(dec + i) = sv;
        }
        const uint32_t ws = wave_alloc(dl && !fits, nwide, lane); // (every lane: ballot)
        if (dl && !fits) {
            st_ev(&wide[ws], ShdDeliv{t, p[k].seq, p[k].src_host, p[k].dst_host, (uint32_t)i + c.idx_base, 0u});
            if (dr < g.H) atomicAdd(&wcnt[dr >> g.shift], 1u);
        }
        if (dl && t >= barrier && t < mn) mn = t; // worker.c:350-363
        if (live[k]) status[i] = st;
    }
    mn = wave_min_u64(mn);
    if (lane == 0) wmin[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int k = 1; k < kWG / 64; k++) m = wmin[k] < m ? wmin[k] : m;
        if (m != ~0ull) atomicMin(&counters[1], m);
    }
}

// the split scatter's partition: records [blockIdx.x * ch, + ch) of dec
// counted per bucket (LDS), one run per nonempty bucket reserved, each
// staged record stored at its run position -- k_part_scatter's tail
template <int kWG, int kCH>
__global__ __launch_bounds__(kWG) void k_part_place(const uint4* __restrict__ dec, size_t n, uint32_t idx_base,
                                                    PartGeo g, uint4* __restrict__ stage, uint32_t* __restrict__ gcnt,
                                                    uint32_t* __restrict__ wcnt, ShdDeliv* __restrict__ wide,
                                                    uint32_t* __restrict__ nwide, uint32_t ch) {
    constexpr int kR = kCH / kWG;
    extern __shared__ uint4 part_smem[];
    uint32_t* hist = reinterpret_cast<uint32_t*>(part_smem);
    uint32_t* gb = hist + g.nb;
    const int lane = threadIdx.x & 63;
    for (uint32_t b = threadIdx.x; b < g.nb; b += kWG) hist[b] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * ch;
    const uint32_t mask = (1u << g.shift) - 1u;
    uint4 rv[kR];
    uint32_t rr[kR];
#pragma unroll
    for (int k = 0; k < kR; k++) {
        const uint32_t li = (uint32_t)(k * kWG + threadIdx.x);
        const size_t i = base + li;
        rv[k] = make_uint4(0u, 0u, 0u, ~0u);
        if (li < ch && i < n) {
            const shd_v4u v = __builtin_nontemporal_load(reinterpret_cast<const shd_v4u*>(dec) + i);
            rv[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    }
#pragma unroll
    for (int k = 0; k < kR; k++) rr[k] = rv[k].w != ~0u ? atomicAdd(&hist[(rv[k].w - g.host_lo) >> g.shift], 1u) : 0u;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < g.nb; b += kWG) {
        const uint32_t h = hist[b];
        gb[b] = h ? atomicAdd(&gcnt[b], h) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kR; k++) {
        const uint4 e = rv[k];
        const bool valid = e.w != ~0u;
        const uint32_t b = valid ? (e.w - g.host_lo) >> g.shift : 0u;
        const size_t j = valid ? (size_t)gb[b] + rr[k] : 0;
        const uint32_t li = (uint32_t)(k * kWG + threadIdx.x);
        const bool in = valid && j < g.cap;
        if (in)
            stage[(size_t)b * g.cap + j] =
                make_uint4(e.x, e.y, (uint32_t)(base + li) + idx_base, (e.z << g.shift) | ((e.w - g.host_lo) & mask));
        const bool full = valid && !in; // the bucket's region is full: whole event to the wide list
        const uint32_t ws = wave_alloc(full, nwide, lane);
        if (full) {
            st_ev(&wide[ws], ShdDeliv{g.tbase + e.x, (unsigned long long)e.y, e.z, e.w, (uint32_t)(base + li) + idx_base,
                                      0u});
            atomicAdd(&wcnt[b], 1u);
        }
    }
}

// The software-pipelined scatter (SHD_PART_SCATTER=7): the same decisions,
// runs and outputs as k_part_scatter, but one persistent workgroup per CU
// walks its chunks with the NEXT chunk's table gathers in flight while the
// current chunk is decided, reserved and stored.  Why: the measurement-only
// probes (profiles/r05g_part_scatter_probe_bits.log) show the forms' costs
// adding up -- floor 0.16 ms + table gather 0.22 ms (its whole ceiling time,
// 10M gathers at 46.2 G/s) + stage stores 0.08 ms -- i.e. every CU waits for
// its gathers and then does everything else, so the gathers (the one
// irreducible random request) overlap nothing.  Here they overlap the
// decide, the run reservation and the stores of the chunk before.
//
// Per iteration (a chunk of ch <= kCH records; chunk = blockIdx.x + it *
// gridDim.x, every workgroup the same number of chunks):
//   decide(cur)  -- waits for cur's gathers, issued one iteration earlier;
//                   status, counter log, LDS ranks, the wide list
//   load(next)   -- next chunk's records
//   barrier; run reservation (one atomic per nonempty bucket, results kept
//                   in registers); gather(next) -- host->slot + table
//                   gathers issued; the reservations into LDS
//   barrier; stores of cur's events at their runs
// Vector memory returns count in issue order: reading the reservation
// results waits for the record loads (older) but not for next's table
// gathers (younger), which stay in flight across the barrier and the stores.
// A workgroup barrier ordering LDS only: __syncthreads()'s workgroup fence
// also covers global memory and so waits for every outstanding vector memory
// operation (s_waitcnt vmcnt(0)) -- in-flight table gathers included.  The
// pipelined scatter shares only LDS across its barriers.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

constexpr uint32_t kPartPipeMaxBuckets = 8192; // (the reservations held in registers: 8 per thread)

template <int kR>
struct PartFront {
    ShdPkt p[kR];
    int si[kR], di[kR];
    size_t ei[kR];
    uint2 q[kR];
    bool live[kR];
};

// (No divergent branch around a load whose result waits for a later use: a
// value merged at a branch join is copied there, and the copy waits for the
// load -- dead lanes load a valid address and are masked afterwards.)
template <int kWG, int kR>
__device__ __forceinline__ void part_load(PartFront<kR>& f, const ShdPkt* __restrict__ recs, size_t base,
                                          uint32_t ch, size_t n) {
#pragma unroll
    for (int k = 0; k < kR; k++) {
        const uint32_t li = (uint32_t)(k * kWG + threadIdx.x);
        const size_t i = base + li;
        f.live[k] = li < ch && i < n;
        f.p[k] = ld_pkt(&recs[f.live[k] ? i : n - 1]); // (n >= 1)
    }
}

__device__ unsigned long long g_ptab_none = ((unsigned long long)0u << 32) | kPtabFallback;

template <int kR>
__device__ __forceinline__ void part_gather(PartFront<kR>& f, const ShdPktCtx& c) {
    const size_t A = (size_t)c.A;
    const uint2* __restrict__ host_info = reinterpret_cast<const uint2*>(c.host_info);
    uint32_t ts[kR], td[kR];
#pragma unroll
    for (int k = 0; k < kR; k++) {
        const bool known = f.live[k] && f.p[k].src_host < c.nhosts && f.p[k].dst_host < c.nhosts;
        uint2 hs = host_info[known ? f.p[k].src_host : 0u], hd = host_info[known ? f.p[k].dst_host : 0u];
        if (!known) hs = hd = make_uint2(~0u, ~0u);
        f.si[k] = hs.x == ~0u ? -1 : (int)hs.x;
        f.di[k] = hd.x == ~0u ? -1 : (int)hd.x;
        ts[k] = hs.y;
        td[k] = hd.y;
    }
#pragma unroll
    for (int k = 0; k < kR; k++) {
        int oi = f.si[k], oj = f.di[k];
        if (oi >= 0 && oj >= 0) {
            if (c.mode == 0) {
                if (oi != oj && td[k] < ts[k]) oi = f.di[k], oj = f.si[k]; // owner: row touched first
            } else if (c.mode == 2) {
                const size_t b = (size_t)oi * A + (size_t)oj;
                if (!((c.pair_bits[b >> 5] >> (b & 31)) & 1u)) oi = f.di[k], oj = f.si[k];
            }
        }
        if (oi < c.row_lo || oi >= c.row_hi) f.si[k] = -1; // another rank's row: not decided here
        f.ei[k] = (size_t)(oi < 0 ? 0 : oi) * A + (size_t)(oj < 0 ? 0 : oj);
    }
    // the table gathers, left in flight: read only by the decision (a pair
    // not decided here, or no ptab, reads the fallback marker)
    const unsigned long long* __restrict__ pt =
        c.ptab ? reinterpret_cast<const unsigned long long*>(c.ptab) : &g_ptab_none;
#pragma unroll
    for (int k = 0; k < kR; k++) {
        const bool ok = c.ptab && f.si[k] >= 0 && f.di[k] >= 0;
        const unsigned long long v = __builtin_nontemporal_load(pt + (ok ? f.ei[k] : 0));
        f.q[k] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
    }
}

template <int kWG, int kCH>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_part_scatter_pipe(
    ShdPktCtx c, const ShdPkt* __restrict__ recs, size_t n, uint64_t barrier, uint64_t end_time, uint64_t boot_end,
    PartGeo g, uint4* __restrict__ stage, uint32_t* __restrict__ gcnt, uint32_t* __restrict__ wcnt,
    uint8_t* __restrict__ status, unsigned long long* counters, ShdDeliv* __restrict__ wide,
    uint32_t* __restrict__ nwide, uint32_t ch, uint32_t nchunks) {
    constexpr int kR = kCH / kWG;
    static_assert(kCH % kWG == 0, "chunk");
    extern __shared__ uint4 part_smem[];
    uint32_t* hist = reinterpret_cast<uint32_t*>(part_smem); // hist[nb] | gb[nb]
    uint32_t* gb = hist + g.nb;
    __shared__ unsigned long long wmin[kWG / 64];
    const int lane = threadIdx.x & 63;
    for (uint32_t b = threadIdx.x; b < g.nb; b += kWG) hist[b] = 0;
    __syncthreads();
    const uint32_t smax = g.shift ? (0xFFFFFFFFu >> g.shift) : 0xFFFFFFFFu;
    const uint32_t mask = (1u << g.shift) - 1u;
    unsigned long long mn = ~0ull;
    PartFront<kR> f;
    uint32_t chunk = blockIdx.x; // (< nchunks: the grid is at most the chunk count)
    part_load<kWG>(f, recs, (size_t)chunk * ch, ch, n);
    part_gather(f, c);
    for (; chunk < nchunks; chunk += gridDim.x) {
        const size_t base = (size_t)chunk * ch;
        const uint32_t nxt = chunk + gridDim.x;
        const size_t nbase = (size_t)(nxt < nchunks ? nxt : chunk) * ch; // (the last: a harmless reload)
        uint4 rv[kR];                    // {time - tbase, seq, src, dst}, w = ~0: none
        uint32_t rr[kR];
#pragma unroll
        for (int k = 0; k < kR; k++) {
            const ShdPkt& p = f.p[k];
            const uint32_t li = (uint32_t)(k * kWG + threadIdx.x);
            uint8_t st = 0xff; // unregistered host: not delivered
            uint64_t t = 0;
            if (f.live[k] && f.si[k] >= 0 && f.di[k] >= 0) {
                uint32_t rs = p.rng_state;
                const uint32_t r = (uint32_t)glibc_rand_r(&rs);
                bool keep;
                uint64_t delay;
                if (f.q[k].x != kPtabFallback) {
                    keep = r <= f.q[k].y; // == (chance <= rel), see kPtabFallback
                    delay = f.q[k].x;
                } else {
                    const ShdEntry e = c.tab[f.ei[k]];
                    keep = (double)r / 2147483647.0 <= e.rel; // random_nextDouble, worker.c:545
                    delay = (uint64_t)ceil(e.lat * 1000000.0);
                }
                st = SHD_DROPPED_LOSS;
                if (p.now < boot_end || keep || p.payload_len == 0) {
                    t = p.now + delay;                    // worker.c:548-549
                    if (t >= end_time) st = SHD_DROPPED_END; // scheduler.c:236-239
                    else {
                        if (p.src_host != p.dst_host && t < barrier) t = barrier; // host_single.c:187-192
                        st = SHD_DELIVERED;
                    }
                    if (c.pcnt) atomicAdd(c.pcnt + f.ei[k], 1u); // (SHD_PCNT=atomic) worker.c:551
                }
            }
            if (f.live[k]) pcnt_log(c, base + li, st == SHD_DELIVERED || st == SHD_DROPPED_END, f.ei[k]);
            const bool dl = st == SHD_DELIVERED;
            const uint32_t dr = p.dst_host - g.host_lo;
            const bool fits = dl && c_fits(t, g.tbase, p.seq) && p.src_host <= smax && dr < g.H;
            rv[k] = make_uint4(0u, 0u, 0u, ~0u);
            rr[k] = 0;
            if (fits) {
                rr[k] = atomicAdd(&hist[dr >> g.shift], 1u); // LDS
                rv[k] = make_uint4((uint32_t)(t - g.tbase), (uint32_t)p.seq, p.src_host, p.dst_host);
            }
            const uint32_t ws = wave_alloc(dl && !fits, nwide, lane); // (every lane: ballot)
            if (dl && !fits) {
                st_ev(&wide[ws], ShdDeliv{t, p.seq, p.src_host, p.dst_host, (uint32_t)(base + li) + c.idx_base, 0u});
                if (dr < g.H) atomicAdd(&wcnt[dr >> g.shift], 1u);
            }
            if (dl && t >= barrier && t < mn) mn = t; // worker.c:350-363
            if (f.live[k]) status[base + li] = st;
        }
        part_load<kWG>(f, recs, nbase, ch, n);
        lds_barrier(); // the chunk's ranks are all taken
        // every reservation in flight at once (a loop that stored each result
        // before the next atomic waited for each round trip in turn)
        constexpr int kPer = (int)((kPartPipeMaxBuckets + kWG - 1) / kWG);
        uint32_t res[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t b = threadIdx.x + (uint32_t)k * kWG;
            const uint32_t h = b < g.nb ? hist[b] : 0u;
            res[k] = 0u;
            if (h) res[k] = atomicAdd(&gcnt[b], h);
        }
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t b = threadIdx.x + (uint32_t)k * kWG;
            if (b < g.nb) gb[b] = res[k], hist[b] = 0; // (hist reused after the next barrier)
        }
        part_gather(f, c);
        lds_barrier(); // the runs' bases are published
#pragma unroll
        for (int k = 0; k < kR; k++) {
            const uint32_t li = (uint32_t)(k * kWG + threadIdx.x);
            const bool valid = rv[k].w != ~0u;
            const uint32_t b = valid ? (rv[k].w - g.host_lo) >> g.shift : 0u;
            const size_t j = valid ? (size_t)gb[b] + rr[k] : 0;
            const bool in = valid && j < g.cap;
            if (in)
                stage[(size_t)b * g.cap + j] = make_uint4(rv[k].x, rv[k].y, (uint32_t)(base + li) + c.idx_base,
                                                          (rv[k].z << g.shift) | ((rv[k].w - g.host_lo) & mask));
            const bool full = valid && !in; // the bucket's region is full: whole event to the wide list
            const uint32_t ws = wave_alloc(full, nwide, lane);
            if (full) {
                st_ev(&wide[ws], ShdDeliv{g.tbase + rv[k].x, (unsigned long long)rv[k].y, rv[k].z, rv[k].w,
                                          (uint32_t)(base + li) + c.idx_base, 0u});
                atomicAdd(&wcnt[b], 1u);
            }
        }
        // (gb is next written after the next iteration's first barrier, when
        // every thread has left these stores)
    }
    mn = wave_min_u64(mn);
    if (lane == 0) wmin[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int k = 1; k < kWG / 64; k++) m = wmin[k] < m ? wmin[k] : m;
        if (m != ~0ull) atomicMin(&counters[1], m);
    }
}

// The part round's per-bucket counters (w.cnt1): gcnt[nb] (staged events) |
// wcnt[nb] (wide events) | wcur[nb] (k_wide_group's cursors) | bpre[nb + 1]
// (each bucket's output base: the earlier buckets' totals) | wpre[nb] (its
// first event in the grouped wide list).
constexpr size_t part_cnt_words(uint32_t nb) { return 5 * (size_t)nb + 1; }

// The wide list (events whose record did not fit the 16-B stage form, or
// whose bucket region was full) grouped by bucket into `grouped`, so that a
// bucket reads only its own (wcnt[b] events from the earlier buckets'
// total): every workgroup scans the per-bucket counts into LDS, then places
// its share of the list with per-bucket cursors.  Exits at once when the list
// is empty (the usual round).  Workgroup 0 first writes bpre / wpre (one
// scan here instead of every sort workgroup summing the counts before it).
__global__ __launch_bounds__(1024) void k_wide_group(PartGeo g, const ShdDeliv* __restrict__ wide,
                                                     const uint32_t* __restrict__ nwide, uint32_t wide_cap,
                                                     const uint32_t* __restrict__ gcnt,
                                                     const uint32_t* __restrict__ wcnt, uint32_t* __restrict__ wcur,
                                                     ShdDeliv* __restrict__ grouped, unsigned long long* counters,
                                                     const unsigned long long* __restrict__ minw2) {
    // the scatter's minimum delivered time (into the workspace's word: it
    // needs no per-round initialisation of the caller's counters)
    if (blockIdx.x == 0 && threadIdx.x == 0) counters[1] = minw2[1];
    if (blockIdx.x == 0) {
        __shared__ uint32_t ps[16];
        uint32_t* bpre = wcur + g.nb;
        uint32_t* wpre = bpre + g.nb + 1;
        // (nb <= kPartMaxBuckets: at most 16 counts per thread, all loads in
        // flight at once)
        constexpr int kPer = (int)(kPartMaxBuckets / 1024);
        const uint32_t per = (g.nb + 1023) / 1024, b0 = threadIdx.x * per;
        uint32_t gv[kPer], wv[kPer];
        uint32_t st = 0, sw = 0;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const bool in = (uint32_t)k < per && b0 + k < g.nb;
            gv[k] = in ? min(gcnt[b0 + k], g.cap) : 0u;
            wv[k] = in ? wcnt[b0 + k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < kPer; k++) st += gv[k] + wv[k], sw += wv[k];
        uint32_t tt, tw;
        uint32_t pt = block_excl_scan_n(st, &tt, ps);
        uint32_t pw = block_excl_scan_n(sw, &tw, ps);
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            if ((uint32_t)k < per && b0 + k < g.nb) {
                bpre[b0 + k] = pt;
                wpre[b0 + k] = pw;
            }
            pt += gv[k] + wv[k];
            pw += wv[k];
        }
        if (threadIdx.x == 0) bpre[g.nb] = tt;
    }
    const uint32_t m = *nwide;
    if (m == 0 || m > wide_cap) return; // (block-uniform; an overfull list is the sort's fault to report)
    extern __shared__ uint32_t woff[]; // [nb]
    __shared__ uint32_t wsum[16];
    const uint32_t per = (g.nb + 1023) / 1024, b0 = threadIdx.x * per;
    uint32_t sm = 0;
    for (uint32_t k = 0; k < per && b0 + k < g.nb; k++) sm += wcnt[b0 + k];
    uint32_t tot;
    uint32_t pre = block_excl_scan_n(sm, &tot, wsum);
    for (uint32_t k = 0; k < per && b0 + k < g.nb; k++) {
        woff[b0 + k] = pre;
        pre += wcnt[b0 + k];
    }
    __syncthreads();
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < m; i += gridDim.x * 1024) {
        const ShdDeliv r = ld_ev(&wide[i]);
        const uint32_t dr = r.dst_host - g.host_lo;
        if (dr < g.H) {
            const uint32_t b = dr >> g.shift;
            st_ev(&grouped[woff[b] + atomicAdd(&wcur[b], 1u)], r);
        }
    }
}

// One workgroup of kWG threads per bucket of at most kCap events held in
// LDS (7 per thread; see above).  nbig / big / scr: the listed segments
// (k_segsort_mid); fault: nbig[2] guard bits.
// kKeyE: the per-wave LDS key array holds segments of up to 64 kKeyE events
// (larger ones up to kSmallSeg take the readlane form): 4, or 2 for the
// instance sized for three workgroups per CU
// kWire: the sorted segments go out as the exchange's 24-B wire records
// (`out` is then a Wire array; listed segments are staged and listed as
// always -- their sorted ShdDeliv form is converted by k_listed_wire)
// Segments of kTinySeg < n <= 128 events (the C3 round: ~92 per destination)
// ranked by TIME BUCKET instead of all pairs: the wave spreads the segment's
// time offsets over 64 buckets ((t - tmin) >> sh), counts them in LDS, scans
// the counts (each bucket's first rank) and lists each bucket's events; an
// event's rank is its bucket's first rank plus the events of its own bucket
// before it in event_compare order (time offset, src, srcHostEventID: the
// stage record's fields order as the full values do).  O(n) LDS work and a
// few compares per event instead of the all-pairs rank's 2n 64-bit compares
// per lane (k_part_sort was VALU-bound on those).  Returns
// false (wave-uniform, before any output) when a bucket holds more than
// kBucketRankMax events -- e.g. many events clamped to the barrier, which all
// share one time -- and the caller takes the all-pairs rank.
constexpr uint32_t kBucketRankMax = 8;
constexpr uint32_t kBucketRankSeg = 128;
// per wave, in the wave's LDS key array (the two paths never overlap in time)
struct BucketRankLds {
    uint32_t h[2 * 64]; // [0, 64): counts, then first ranks; [64, 128): fill cursors, then counts
    uint8_t m[128];     // the events of each bucket, at its first rank
};
static_assert(sizeof(BucketRankLds) <= 8 * (64 * 2 + 8), "fits a wave's LDS key array (kKeyE >= 2)");
__device__ __forceinline__ void wave_lds_sync() { // (LDS only: in-flight global stores stay in flight)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off));
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    return v;
}
// rank[e] of element e * 64 + lane (< n) of the segment lev[o, o + n)
__device__ __forceinline__ bool wave_bucket_rank(const uint4* lev, uint32_t o, uint32_t n, uint32_t shift,
                                                 BucketRankLds& w, int lane, uint32_t (&rank)[2]) {
    uint32_t tmin = ~0u, tmax = 0u, tv[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        if (i < n) {
            tv[e] = lev[o + i].x;
            tmin = min(tmin, tv[e]);
            tmax = max(tmax, tv[e]);
        }
    }
    tmin = wave_min_u32(tmin);
    const uint32_t span = wave_max_u32(tmax) - tmin;
    const uint32_t sh = span < 64u ? 0u : 26u - (uint32_t)__clz((int)span); // (span >> sh) < 64
    w.h[lane] = w.h[lane + 64] = 0u;
    wave_lds_sync();
    uint32_t bk[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 2; e++)
        if ((uint32_t)(e * 64 + lane) < n) {
            bk[e] = (tv[e] - tmin) >> sh;
            atomicAdd(&w.h[bk[e]], 1u);
        }
    wave_lds_sync();
    const uint32_t h0 = w.h[lane];
    if (__ballot(h0 > kBucketRankMax)) return false;
    const uint32_t ex = wave_incl_scan(h0, lane) - h0;
    wave_lds_sync(); // (every lane has read its count)
    w.h[lane] = ex;
    wave_lds_sync();
    uint32_t first[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        if (i < n) {
            first[e] = w.h[bk[e]];
            w.m[first[e] + atomicAdd(&w.h[64 + bk[e]], 1u)] = (uint8_t)i;
        }
    }
    wave_lds_sync();
    for (int e = 0; e < 2; e++) { // (not unrolled: one element's compares at a time)
        const uint32_t i = (uint32_t)(e * 64 + lane);
        const uint32_t f = e ? first[1] : first[0], b = e ? bk[1] : bk[0];
        uint32_t rk = f;
        if (i < n) {
            const uint4 me = lev[o + i];
            const uint32_t cb = w.h[64 + b], sr = me.w >> shift;
            for (uint32_t k = 0; k < cb; k++) {
                const uint4 x = lev[o + w.m[f + k]];
                const uint32_t sx = x.w >> shift;
                rk += (uint32_t)(x.x < me.x || (x.x == me.x && (sx < sr || (sx == sr && x.y < me.y))));
            }
        }
        if (e) rank[1] = rk;
        else rank[0] = rk;
    }
    return true;
}

// The part sort's rank of one destination segment lev[o, o + n) (n <= 64 E,
// LDS stage records {time - tbase, seq, pkt_index, src << shift | dl}) by
// event_compare, with 31-bit keys: key = time - barrier (xbar: the
// barrier's offset from tbase), which every inter-host delivery (clamped to
// the barrier) has in [0, 2^31 - 1) unless it lands 2.1 s or more after the
// barrier; kj < key is then the sign bit of kj - key -- a subtract and a shift
// per pair on plain VGPRs, independent of each other, where a 64-bit compare
// writes an SGPR pair that the next instruction must wait for.  Keys come
// four at a time by LDS broadcast.  Returns false (wave-uniform, before any
// output) when an event precedes the barrier (a host's packet to itself) or
// lies that far past it: the caller ranks that segment on 64-bit keys.
// Equal times (rare: 3 of C3's 100,000 segments hold a pair) are ranked
// among themselves by (src, srcHostEventID) in a second pass.  Each event is
// stored at out + its rank (kOut 1: the 32-B event, 2: the 24-B wire record).
template <int E, int kOut>
__device__ __forceinline__ bool wave_rank_x31(const uint4* lev, uint32_t o, uint32_t n, uint32_t xbar, uint32_t shift,
                                              unsigned long long tbase, uint32_t dh, ShdDeliv* __restrict__ out,
                                              uint32_t ob, int lane, uint32_t* lk32) {
    uint4 r[E];
    uint32_t key[E], rank[E];
    bool early = false;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        r[e] = i < n ? lev[o + i] : make_uint4(xbar, 0u, 0u, 0u);
        early |= r[e].x < xbar || r[e].x - xbar >= 0x7FFFFFFFu;
    }
    if (__ballot(early)) return false;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * 64 + lane);
        key[e] = i < n ? r[e].x - xbar : 0x7FFFFFFFu; // (padding: above every key)
        rank[e] = 0;
        lk32[e * 64 + lane] = key[e];
    }
    if (lane < 16) lk32[64 * E + lane] = 0x7FFFFFFFu;
    wave_lds_sync();
    const uint4* lk4 = reinterpret_cast<const uint4*>(lk32);
    for (uint32_t j = 0; j < n; j += 16) {
        uint4 kk[4];
#pragma unroll
        for (int u = 0; u < 4; u++) kk[u] = lk4[(j >> 2) + u];
#pragma unroll
        for (int e = 0; e < E; e++) {
            uint32_t a = 0, c = 0;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                a += ((kk[u].x - key[e]) >> 31) + ((kk[u].y - key[e]) >> 31);
                c += ((kk[u].z - key[e]) >> 31) + ((kk[u].w - key[e]) >> 31);
            }
            rank[e] += a + c;
        }
    }
    // ties (equal keys share their lowest rank: the ranks' sum falls short)
    uint32_t rsum = 0;
#pragma unroll
    for (int e = 0; e < E; e++) rsum += (e * 64 + lane < (int)n) ? rank[e] : 0u;
    for (int off = 32; off > 0; off >>= 1) rsum += (uint32_t)__shfl_xor((int)rsum, off);
    if (rsum != n * (n - 1) / 2) {
#pragma unroll
        for (int ej = 0; ej < E; ej++) {
            const int lim = (int)n - ej * 64 < 64 ? (int)n - ej * 64 : 64;
            for (int l = 0; l < lim; l++) {
                const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key[ej], l);
                const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)(r[ej].w >> shift), l);
                const uint32_t qj = (uint32_t)__builtin_amdgcn_readlane((int)r[ej].y, l);
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const uint32_t se = r[e].w >> shift;
                    rank[e] += (uint32_t)((kj == key[e]) & ((sj < se) | ((sj == se) & (qj < r[e].y))));
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < E; e++) {
        if ((uint32_t)(e * 64 + lane) >= n) continue;
        const unsigned long long t = tbase + r[e].x;
        const uint32_t src = r[e].w >> shift;
        if (kOut == 2) {
            st_wire(reinterpret_cast<Wire*>(out) + ob + rank[e], t, (unsigned long long)r[e].y, src, r[e].z);
        } else {
            shd_v4u* q = reinterpret_cast<shd_v4u*>(&out[ob + rank[e]]);
            const shd_v4u a = {(uint32_t)t, (uint32_t)(t >> 32), r[e].y, 0u};
            const shd_v4u c2 = {src, dh, r[e].z, 0u};
            __builtin_nontemporal_store(a, q);
            __builtin_nontemporal_store(c2, q + 1);
        }
    }
    return true;
}

template <int kWG, int kCap, int kKeyE, bool kWire>
__device__ __forceinline__ void part_sort_body(PartGeo g, const uint4* __restrict__ stage,
                                                          const uint32_t* __restrict__ gcnt,
                                                          const uint32_t* __restrict__ wcnt,
                                                          const ShdDeliv* __restrict__ wide,
                                                          const uint32_t* __restrict__ nwide, uint32_t wide_cap,
                                                          uint32_t* __restrict__ offsets, ShdDeliv* __restrict__ out,
                                                          ShdDeliv* __restrict__ scr, uint32_t* __restrict__ big,
                                                          uint32_t* __restrict__ nbig,
                                                          unsigned long long* __restrict__ counters, uint32_t lds_keys,
                                                          const uint32_t b) {
    // perm: the segments' ranks go to an LDS permutation and the bucket is
    // written in order afterwards -- consecutive lanes, consecutive 16-B (8-B
    // for wire records) pieces of the output, whole lines per instruction
    // instead of every event's two 16-B stores scattered over its segment
    // (the instances whose LDS has room for the 2-B index per event; not the
    // LDS-key-free four-per-CU one)
    constexpr bool kPermOk = kCap <= 2304 && kKeyE > 0;
    __shared__ uint4 lev[kCap];
    __shared__ uint16_t inv[kPermOk ? kCap : 1];
    const bool perm = kPermOk && (lds_keys & 2u);
    __shared__ unsigned long long keys[kWG / 64][kKeyE ? 64 * kKeyE + 8 : 1];
    __shared__ uint32_t cnt[kPartMaxDst], loc[kPartMaxDst + 1], cur[kPartMaxDst];
    const bool brank = kKeyE >= 2 && (lds_keys & 4u);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t d0 = b << g.shift;
    const uint32_t nd = min(1u << g.shift, g.H - d0);
    const uint32_t mask = (1u << g.shift) - 1u;
    const uint32_t ns = min(gcnt[b], g.cap), nw = wcnt[b], tot = ns + nw;
    const bool listed = tot > (uint32_t)kCap || nw > 0; // (block-uniform)
    for (uint32_t j = threadIdx.x; j < kPartMaxDst; j += kWG) cnt[j] = cur[j] = 0;
    const uint4* sb = stage + (size_t)b * g.cap;
    // the bucket's records in registers, kCap / kWG per thread; an instance
    // whose capacity is not a multiple of kWG (512 threads, 2,304 events)
    // reads its last partial row from the stage twice instead (count, place:
    // only buckets above kRegEv events)
    constexpr uint32_t kRegEv = (uint32_t)(kCap / kWG) * kWG;
    uint4 e[kCap / kWG];
    if (!listed) { // the bucket's records
#pragma unroll
        for (int k = 0; k < kCap / kWG; k++) {
            const uint32_t i = (uint32_t)k * kWG + threadIdx.x;
            if (i < ns) {
                const shd_v4u v = __builtin_nontemporal_load(reinterpret_cast<const shd_v4u*>(sb) + i);
                e[k] = make_uint4(v.x, v.y, v.z, v.w);
            }
        }
    }
    // this bucket's output base (the totals of the buckets before it) and
    // its wide events' place in the grouped list, from k_wide_group's scan
    // (the counter layout: part_cnt_words)
    const uint32_t* bpre = gcnt + 3 * (size_t)g.nb;
    const uint32_t obase = bpre[b];
    const ShdDeliv* wb = wide + (nw ? bpre[g.nb + 1 + b] : 0u); // this bucket's wide events (k_wide_group)
    lds_barrier(); // (orders the cnt reset)
    if (!listed) {
#pragma unroll
        for (int k = 0; k < kCap / kWG; k++)
            if ((uint32_t)k * kWG + threadIdx.x < ns) atomicAdd(&cnt[e[k].w & mask], 1u);
        if (kRegEv < (uint32_t)kCap)
            for (uint32_t i = kRegEv + threadIdx.x; i < ns; i += kWG) atomicAdd(&cnt[sb[i].w & mask], 1u);
    } else {
        for (uint32_t i = threadIdx.x; i < ns; i += kWG) atomicAdd(&cnt[sb[i].w & mask], 1u);
        const uint32_t m = *nwide;
        if (m > wide_cap) {
            if (threadIdx.x == 0) atomicOr(nbig + 2, kFaultOvfCap);
        } else {
            for (uint32_t i = threadIdx.x; i < nw; i += kWG) atomicAdd(&cnt[(wb[i].dst_host - g.host_lo) & mask], 1u);
        }
    }
    lds_barrier();
    if (threadIdx.x < 64) { // destination offsets (nd <= 64: one wave)
        const uint32_t v = threadIdx.x < nd ? cnt[threadIdx.x] : 0u;
        const uint32_t inc = wave_incl_scan(v, lane);
        if (threadIdx.x < nd) {
            loc[threadIdx.x] = inc - v;
            offsets[d0 + threadIdx.x] = obase + inc - v;
        }
        if (threadIdx.x == 63) loc[nd] = inc;
    }
    if (b == g.nb - 1 && threadIdx.x == 0) {
        offsets[g.H] = obase + tot;
        counters[0] = obase + tot; // the round's delivered count
    }
    lds_barrier();
    if (!listed) {
#pragma unroll
        for (int k = 0; k < kCap / kWG; k++) {
            const uint32_t i = (uint32_t)k * kWG + threadIdx.x;
            if (i < ns) {
                const uint32_t dl = e[k].w & mask;
                lev[loc[dl] + atomicAdd(&cur[dl], 1u)] = e[k];
            }
        }
        if (kRegEv < (uint32_t)kCap)
            for (uint32_t i = kRegEv + threadIdx.x; i < ns; i += kWG) {
                const uint4 r = sb[i];
                const uint32_t dl = r.w & mask;
                lev[loc[dl] + atomicAdd(&cur[dl], 1u)] = r;
            }
        lds_barrier();
        // segments of at most kTinySeg events (many destinations per bucket,
        // few events each: C4's rounds): one thread per event, its rank the
        // count of its segment's events before it in event_compare order
        // (time, src, srcHostEventID -- the stage record's time offset, src and
        // 32-bit id compare as the full values do)
        for (uint32_t i = threadIdx.x; i < ns; i += kWG) {
            const uint4 r = lev[i];
            const uint32_t dl = r.w & mask, nj = cnt[dl];
            if (nj > kTinySeg) continue;
            const uint32_t o = loc[dl], sr = r.w >> g.shift;
            uint32_t rank = 0;
            for (uint32_t j = o; j < o + nj; j++) {
                const uint4 x = lev[j];
                const uint32_t sx = x.w >> g.shift;
                rank += (uint32_t)(x.x < r.x || (x.x == r.x && (sx < sr || (sx == sr && x.y < r.y))));
            }
            const unsigned long long t = g.tbase + r.x;
            if (perm) {
                inv[o + rank] = (uint16_t)i;
            } else if (kWire) {
                st_wire(reinterpret_cast<Wire*>(out) + obase + o + rank, t, (unsigned long long)r.y, sr, r.z);
            } else {
                shd_v4u* q = reinterpret_cast<shd_v4u*>(&out[obase + o + rank]);
                const shd_v4u a = {(uint32_t)t, (uint32_t)(t >> 32), r.y, 0u};
                const shd_v4u c2 = {sr, g.host_lo + d0 + dl, r.z, 0u};
                __builtin_nontemporal_store(a, q);
                __builtin_nontemporal_store(c2, q + 1);
            }
        }
        unsigned long long* lk = (lds_keys & 1u) && kKeyE ? keys[wv] : nullptr;
        for (uint32_t j = wv; j < nd; j += kWG / 64) {
            const uint32_t nj = cnt[j], o = loc[j], dh = g.host_lo + d0 + j;
            if (nj <= kTinySeg) continue;
            auto load = [&](uint32_t i) {
                const uint4 r = lev[o + i];
                return Ev{g.tbase + r.x, (unsigned long long)r.y, r.w >> g.shift, r.z};
            };
            constexpr int kOut = kWire ? 2 : 1;
            ShdDeliv* const wo = reinterpret_cast<ShdDeliv*>(inv);
            if (brank && nj <= kBucketRankSeg) {
                uint32_t rk[2];
                if (wave_bucket_rank(lev, o, nj, g.shift, *reinterpret_cast<BucketRankLds*>(keys[wv]), lane, rk)) {
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const uint32_t i = (uint32_t)(e * 64 + lane);
                        if (i >= nj) continue;
                        if (perm) {
                            inv[o + rk[e]] = (uint16_t)(o + i);
                            continue;
                        }
                        const uint4 r = lev[o + i];
                        const unsigned long long t = g.tbase + r.x;
                        const uint32_t sr = r.w >> g.shift;
                        if (kWire) {
                            st_wire(reinterpret_cast<Wire*>(out) + obase + o + rk[e], t, (unsigned long long)r.y, sr, r.z);
                        } else {
                            shd_v4u* q = reinterpret_cast<shd_v4u*>(&out[obase + o + rk[e]]);
                            const shd_v4u a = {(uint32_t)t, (uint32_t)(t >> 32), r.y, 0u};
                            const shd_v4u c2 = {sr, dh, r.z, 0u};
                            __builtin_nontemporal_store(a, q);
                            __builtin_nontemporal_store(c2, q + 1);
                        }
                    }
                    continue;
                }
            }
            // 31-bit keys (the time offset from the destination's earliest):
            // the signed difference's sign bit is the compare, no SGPR carry
            // chain (SHD_SORT_X31=0: the packed 64-bit keys)
            if (kKeyE >= 2 && lk && !perm && !(lds_keys & 64u) && nj <= 128) {
                const bool done =
                    nj <= 64 ? wave_rank_x31<1, kOut>(lev, o, nj, g.xbar, g.shift, g.tbase, dh, out, obase + o, lane,
                                                      reinterpret_cast<uint32_t*>(lk))
                             : wave_rank_x31<2, kOut>(lev, o, nj, g.xbar, g.shift, g.tbase, dh, out, obase + o, lane,
                                                      reinterpret_cast<uint32_t*>(lk));
                if (done) continue;
            }
            if (nj <= 64) {
                if (perm) wave_rank_segment<1, 3>(load, nj, dh, wo, o, lane, lk);
                else wave_rank_segment<1, kOut>(load, nj, dh, out, obase + o, lane, lk);
            } else if (nj <= 128) {
                if (perm) wave_rank_segment<2, 3>(load, nj, dh, wo, o, lane, kKeyE >= 2 ? lk : nullptr);
                else wave_rank_segment<2, kOut>(load, nj, dh, out, obase + o, lane, kKeyE >= 2 ? lk : nullptr);
            } else if (nj <= (uint32_t)kSmallSeg) {
                if (perm) wave_rank_segment<4, 3>(load, nj, dh, wo, o, lane, kKeyE >= 4 ? lk : nullptr);
                else wave_rank_segment<4, kOut>(load, nj, dh, out, obase + o, lane, kKeyE >= 4 ? lk : nullptr);
            } else { // a larger segment: unsorted to its range of the staging array, listed
                for (uint32_t i = lane; i < nj; i += 64) {
                    const Ev v = load(i);
                    st_ev(&scr[obase + o + i], ShdDeliv{v.t, v.q, v.s, dh, v.ix, 0u});
                    if (perm) inv[o + i] = 0xFFFFu; // (its place is the listed kernels' to write)
                }
                if (lane == 0) {
                    const uint32_t k = atomicAdd(nbig, 1u);
                    if (k < g.H) big[k] = d0 + j;
                    else atomicOr(nbig + 2, kFaultBigCap);
                }
            }
        }
        if (perm) { // the bucket in output order
            lds_barrier();
            if (kWire) {
                uint2* ob = reinterpret_cast<uint2*>(reinterpret_cast<Wire*>(out) + obase);
                for (uint32_t u = threadIdx.x; u < 3 * ns; u += kWG) {
                    const uint32_t p = u / 3, part = u - 3 * p;
                    const uint32_t i = inv[p];
                    if (i == 0xFFFFu) continue;
                    const uint4 r = lev[i];
                    const unsigned long long t = g.tbase + r.x;
                    ob[u] = part == 0 ? make_uint2((uint32_t)t, (uint32_t)(t >> 32))
                            : part == 1 ? make_uint2(r.y, 0u)
                                        : make_uint2(r.w >> g.shift, r.z);
                }
            } else {
                shd_v4u* ob = reinterpret_cast<shd_v4u*>(out + obase);
                for (uint32_t h = threadIdx.x; h < 2 * ns; h += kWG) {
                    const uint32_t i = inv[h >> 1];
                    if (i == 0xFFFFu) continue;
                    const uint4 r = lev[i];
                    const unsigned long long t = g.tbase + r.x;
                    const shd_v4u a = (h & 1) ? shd_v4u{r.w >> g.shift, g.host_lo + d0 + (r.w & mask), r.z, 0u}
                                              : shd_v4u{(uint32_t)t, (uint32_t)(t >> 32), r.y, 0u};
                    __builtin_nontemporal_store(a, ob + h);
                }
            }
        }
        return;
    }
    // listed bucket: every event unsorted to its destination's range of the
    // staging array, every nonempty segment listed (k_segsort_mid / _merge)
    for (uint32_t i = threadIdx.x; i < ns; i += kWG) {
        const uint4 r = sb[i];
        const uint32_t dl = r.w & mask;
        st_ev(&scr[obase + loc[dl] + atomicAdd(&cur[dl], 1u)],
              ShdDeliv{g.tbase + r.x, (unsigned long long)r.y, r.w >> g.shift, g.host_lo + d0 + dl, r.z, 0u});
    }
    if (nw && *nwide <= wide_cap)
        for (uint32_t i = threadIdx.x; i < nw; i += kWG) {
            ShdDeliv r = ld_ev(&wb[i]);
            const uint32_t dl = (r.dst_host - g.host_lo) & mask;
            r.pad = 0;
            st_ev(&scr[obase + loc[dl] + atomicAdd(&cur[dl], 1u)], r);
        }
    lds_barrier();
    for (uint32_t j = threadIdx.x; j < nd; j += kWG)
        if (cnt[j] > 0) {
            const uint32_t k = atomicAdd(nbig, 1u);
            if (k < g.H) big[k] = d0 + j;
            else atomicOr(nbig + 2, kFaultBigCap);
        }
}

// the kernels: the compiler's register choice, or sized for kOcc waves per
// SIMD (SHD_PART_SORT=4: no LDS keys, 63 VGPRs, four workgroups per CU)
// kMinW: waves per SIMD the registers are held to (instance 3: 6, three
// 512-thread workgroups per CU -- the LDS allows it, the registers must too)
template <int kWG, int kCap, int kKeyE = 4, bool kWire = false, int kMinW = 1>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(kMinW, 8))) void k_part_sort(PartGeo g, const uint4* __restrict__ stage,
                                                          const uint32_t* __restrict__ gcnt,
                                                          const uint32_t* __restrict__ wcnt,
                                                          const ShdDeliv* __restrict__ wide,
                                                          const uint32_t* __restrict__ nwide, uint32_t wide_cap,
                                                          uint32_t* __restrict__ offsets, ShdDeliv* __restrict__ out,
                                                          ShdDeliv* __restrict__ scr, uint32_t* __restrict__ big,
                                                          uint32_t* __restrict__ nbig,
                                                          unsigned long long* __restrict__ counters, uint32_t lds_keys) {
    part_sort_body<kWG, kCap, kKeyE, kWire>(g, stage, gcnt, wcnt, wide, nwide, wide_cap, offsets, out, scr, big, nbig,
                                           counters, lds_keys, g.b0 + blockIdx.x);
}
template <int kWG, int kCap, int kKeyE, int kOcc>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(kOcc, kOcc))) void k_part_sort_occ(PartGeo g, const uint4* __restrict__ stage,
                                                          const uint32_t* __restrict__ gcnt,
                                                          const uint32_t* __restrict__ wcnt,
                                                          const ShdDeliv* __restrict__ wide,
                                                          const uint32_t* __restrict__ nwide, uint32_t wide_cap,
                                                          uint32_t* __restrict__ offsets, ShdDeliv* __restrict__ out,
                                                          ShdDeliv* __restrict__ scr, uint32_t* __restrict__ big,
                                                          uint32_t* __restrict__ nbig,
                                                          unsigned long long* __restrict__ counters, uint32_t lds_keys) {
    part_sort_body<kWG, kCap, kKeyE, false>(g, stage, gcnt, wcnt, wide, nwide, wide_cap, offsets, out, scr, big, nbig,
                                           counters, lds_keys, g.b0 + blockIdx.x);
}

// The sorted wire's listed segments: the listed kernels sorted them as
// ShdDeliv into `sorted` (at their event offsets); copied here into the wire
// array at the same offsets (one wave per listed destination).
__global__ __launch_bounds__(256) void k_listed_wire(const ShdDeliv* __restrict__ sorted, const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ big, const uint32_t* __restrict__ nbig,
                                                     uint32_t cap_big, Wire* __restrict__ wire) {
    const int lane = threadIdx.x & 63;
    const uint32_t nb_raw = nbig[0];
    const uint32_t nb = nb_raw <= cap_big ? nb_raw : 0u;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
    for (uint32_t q = wave; q < nb; q += nwaves) {
        const uint32_t d = big[q];
        for (uint32_t i = off[d] + lane; i < off[d + 1]; i += 64) {
            const ShdDeliv r = ld_ev(&sorted[i]);
            st_wire(&wire[i], r.time, r.seq, r.src_host, r.pkt_index);
        }
    }
}

// The exchanged round's sender side on the part pipeline (see
// k_group_wire): one workgroup per bucket counts its events per destination,
// writes the destination offsets (the bucket's base: k_wide_group's scan of
// the earlier buckets' totals) and places every event, unsorted, at its destination's range of
// the wire array -- the owners sort the union of what they receive.
template <int kWG, int kR>
__global__ __launch_bounds__(kWG) void k_part_wire(PartGeo g, const uint4* __restrict__ stage,
                                                   const uint32_t* __restrict__ gcnt, const uint32_t* __restrict__ wcnt,
                                                   const ShdDeliv* __restrict__ wide, const uint32_t* __restrict__ nwide,
                                                   uint32_t wide_cap, uint32_t* __restrict__ offsets,
                                                   Wire* __restrict__ wire, unsigned long long* __restrict__ counters,
                                                   uint32_t* __restrict__ fault) {
    __shared__ uint32_t cnt[kPartMaxDst], loc[kPartMaxDst + 1], cur[kPartMaxDst];
    const uint32_t b = g.b0 + blockIdx.x;
    const uint32_t d0 = b << g.shift;
    const uint32_t nd = min(1u << g.shift, g.H - d0);
    const uint32_t mask = (1u << g.shift) - 1u;
    const uint32_t ns = min(gcnt[b], g.cap), nw = wcnt[b], tot = ns + nw;
    for (uint32_t j = threadIdx.x; j < kPartMaxDst; j += kWG) cnt[j] = cur[j] = 0;
    // the bucket's records (up to kR per thread in registers, read once: the
    // count pass and the placement use them)
    const uint4* sb = stage + (size_t)b * g.cap;
    const bool held = ns <= (uint32_t)(kWG * kR); // (block-uniform)
    uint4 e[kR];
    if (held) {
#pragma unroll
        for (int k = 0; k < kR; k++) {
            const uint32_t i = (uint32_t)k * kWG + threadIdx.x;
            if (i < ns) {
                const shd_v4u v = __builtin_nontemporal_load(reinterpret_cast<const shd_v4u*>(sb) + i);
                e[k] = make_uint4(v.x, v.y, v.z, v.w);
            }
        }
    }
    const uint32_t* bpre = gcnt + 3 * (size_t)g.nb; // (k_wide_group's scan: part_cnt_words)
    const uint32_t obase = bpre[b];
    const ShdDeliv* wb = wide + (nw ? bpre[g.nb + 1 + b] : 0u); // this bucket's wide events (k_wide_group)
    __syncthreads(); // (orders the cnt reset)
    const uint32_t m = *nwide;
    const bool wide_ok = m <= wide_cap;
    if (!wide_ok && b == 0 && threadIdx.x == 0) atomicOr(fault, kFaultOvfCap);
    if (held) {
#pragma unroll
        for (int k = 0; k < kR; k++)
            if ((uint32_t)k * kWG + threadIdx.x < ns) atomicAdd(&cnt[e[k].w & mask], 1u);
    } else {
        for (uint32_t i = threadIdx.x; i < ns; i += kWG) atomicAdd(&cnt[sb[i].w & mask], 1u);
    }
    if (wide_ok)
        for (uint32_t i = threadIdx.x; i < nw; i += kWG) atomicAdd(&cnt[(wb[i].dst_host - g.host_lo) & mask], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t v = threadIdx.x < nd ? cnt[threadIdx.x] : 0u;
        const uint32_t inc = wave_incl_scan(v, (int)threadIdx.x);
        if (threadIdx.x < nd) {
            loc[threadIdx.x] = inc - v;
            offsets[d0 + threadIdx.x] = obase + inc - v;
        }
    }
    if (b == g.nb - 1 && threadIdx.x == 0) {
        offsets[g.H] = obase + tot;
        counters[0] = obase + tot;
    }
    __syncthreads();
    auto place = [&](const uint4& r) {
        const uint32_t dl = r.w & mask;
        st_wire(&wire[obase + loc[dl] + atomicAdd(&cur[dl], 1u)], g.tbase + r.x, (unsigned long long)r.y,
                r.w >> g.shift, r.z);
    };
    if (held) {
#pragma unroll
        for (int k = 0; k < kR; k++)
            if ((uint32_t)k * kWG + threadIdx.x < ns) place(e[k]);
    } else {
        for (uint32_t i = threadIdx.x; i < ns; i += kWG) place(sb[i]);
    }
    if (wide_ok)
        for (uint32_t i = threadIdx.x; i < nw; i += kWG) {
            const ShdDeliv r = ld_ev(&wb[i]);
            const uint32_t dl = (r.dst_host - g.host_lo) & mask;
            st_wire(&wire[obase + loc[dl] + atomicAdd(&cur[dl], 1u)], r.time, r.seq, r.src_host, r.pkt_index);
        }
}

// The split exchange's per-owner cuts straight from the partition, before
// any bucket is sorted: cuts[r] = the grouped output's offset of host
// bounds[r] -- the earlier buckets' totals (k_wide_group's bpre) plus the
// events of bounds[r]'s bucket below it, staged and wide; what the sorts'
// destination offsets say at that host.  One workgroup per cut.
struct CutArgs {
    uint32_t b[65];
    int W;
};
__global__ __launch_bounds__(256) void k_part_cuts(PartGeo g, const uint4* __restrict__ stage,
                                                   const uint32_t* __restrict__ gcnt, const uint32_t* __restrict__ wcnt,
                                                   const ShdDeliv* __restrict__ wide, const uint32_t* __restrict__ nwide,
                                                   uint32_t wide_cap, CutArgs a, uint32_t* __restrict__ cuts) {
    __shared__ uint32_t ws[4];
    const uint32_t hb = a.b[blockIdx.x];
    const uint32_t* bpre = gcnt + 3 * (size_t)g.nb; // (part_cnt_words)
    if (hb >= g.H) {
        if (threadIdx.x == 0) cuts[blockIdx.x] = bpre[g.nb];
        return;
    }
    const uint32_t mask = (1u << g.shift) - 1u, b = hb >> g.shift, d = hb & mask;
    uint32_t c = 0;
    if (d) {
        const uint32_t ns = min(gcnt[b], g.cap), nw = wcnt[b];
        const uint4* sb = stage + (size_t)b * g.cap;
        for (uint32_t i = threadIdx.x; i < ns; i += 256) c += (sb[i].w & mask) < d ? 1u : 0u;
        if (nw && *nwide <= wide_cap) {
            const ShdDeliv* wb = wide + bpre[g.nb + 1 + b];
            for (uint32_t i = threadIdx.x; i < nw; i += 256)
                c += ((wb[i].dst_host - g.host_lo) & mask) < d ? 1u : 0u;
        }
    }
    for (int off = 32; off > 0; off >>= 1) c += (uint32_t)__shfl_xor((int)c, off);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cuts[blockIdx.x] = bpre[b] + ws[0] + ws[1] + ws[2] + ws[3];
}

// cuts[r] = offsets[bounds[r]] (a sender whose offsets are all written)
__global__ void k_gather_cuts(const uint32_t* __restrict__ offsets, CutArgs a, uint32_t* __restrict__ cuts) {
    if ((int)threadIdx.x <= a.W) cuts[threadIdx.x] = offsets[a.b[threadIdx.x]];
}

// the round's fault word when no merge kernel runs: the stage guards only
__global__ void k_fault_word(const uint32_t* __restrict__ nbig, MergeMeta mm) {
    if (threadIdx.x == 0) {
        mm.hdr[3] = nbig[2] << 24;
        note_fault(mm, nbig[2] << 24);
    }
}

// ---- workspace (grow-only, one per topology; see shd_dev_ws_new) ----
constexpr size_t kXmatWords = 64 * 66; // the exchange's count matrix at the largest world (xchg.hip kMaxWorld)
constexpr int kXchgEvents = 16;
struct Ws {
    int device = -1;           // device the buffers live on
    hipEvent_t done = nullptr; // recorded after the last launch that used the buffers
    hipEvent_t fin = nullptr;  // a synchronous call's end (ws_sync)
    hipStream_t last = nullptr;
    bool used = false;
    bool checked = false; // the fault word of the last (completed) use has been read
    size_t cap_n = 0;
    ShdDeliv* tmp = nullptr; // decided events in record order
    ShdDeliv* st1 = nullptr; // events partitioned by bucket (bucket) / destination (rank)
    uint32_t* rnk = nullptr; // per-event rank, regroup path
    ShdDeliv* st2 = nullptr; // pass-1 (part) layout of the staged partition
    size_t cap_m = 0;        // count matrix (bucket) / per-destination counts (rank)
    uint32_t* cnt1 = nullptr;
    uint32_t* off1 = nullptr;
    uint32_t* poff = nullptr;   // part x column offsets (staged partition)
    uint32_t* cursor = nullptr; // bucket cursors (staged partition)
    uint32_t* bsum = nullptr;
    uint32_t cap_h = 0;
    uint32_t* big = nullptr;
    uint32_t* nbig = nullptr; // [0] big segments, [1] slab overflow events
    size_t cap_slab = 0;      // slab pipeline: H x kSlab event slots
    ShdDeliv* slab = nullptr;
    size_t cap_cslab = 0;     // ... and their compact 16-B form (CSlab)
    uint4* cslab = nullptr;
    size_t cap_pstage = 0;    // part pipeline: the bucket regions of the stage (16-B records)
    uint4* pstage = nullptr;
    uint32_t* meta = nullptr; // big-segment merge metadata (MergeMeta)
    uint32_t cap_meta = 0;    // merge segments it holds
    uint32_t* fault = nullptr; // pinned host buffer the sticky fault word is read into
    hipStream_t rd = nullptr;  // the stream that read uses (non-blocking)
    void* xdev = nullptr;      // exchange scratch (xchg.hip: route counts / offsets, event cuts), grow-only
    size_t cap_xdev = 0;
    void* xhost = nullptr;     // its pinned host side (read back on the launch stream)
    size_t cap_xhost = 0;
    uint64_t* xmat = nullptr;  // the exchange's count matrix (kXmatWords u64), device and pinned host
    uint64_t* hxmat = nullptr;
    bool done_pending = false; // the last use's w.done not recorded yet (done_flush)
    // the part pipeline's round state pre-cleared by the last synchronous
    // round's final kernel (k_fault_out): nbig, cnt1[0, pre_m) and the min
    // word are zero / all-ones; clean_now: this use may rely on it (set by
    // ws_begin, dropped by any regrowth); pre_req: the cnt1 words this use
    // wants cleared at its end (part_front)
    bool pre_clean = false, clean_now = false;
    size_t pre_m = 0, pre_req = 0;
    unsigned long long* minw2 = nullptr; // [1]: the scatter's minimum delivered time (part pipeline)
    // fin_ask: the caller waits for this part round (shd_dev_packet_round on
    // the null stream): its merge kernel may end it (fin_done, fin_m: the
    // resets it did) instead of a k_fault_out launch in ws_sync
    bool fin_ask = false, fin_done = false;
    uint32_t fin_m = 0;
    // the segments the last synchronous round listed (its end word; ~0u:
    // unknown -- an asynchronous use, or the copy form of the end)
    uint32_t last_listed = ~0u;
    hipStream_t xs = nullptr;  // the split exchange's transfer stream (non-blocking) and its events
    hipEvent_t xev[kXchgEvents] = {};
};

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

// w.done is recorded lazily on the null stream: ws_end only notes the use,
// and the first reader records the event there, behind everything it launched.
// A synchronous call that waits for that stream itself never records it
// (ws_sync): an event record holds the stream's next command back ~5 us
// (profiles/r05z_round_trace_gaps.log).
int done_flush(Ws& w) {
    if (!w.done_pending) return 0;
    w.done_pending = false;
    return hip_status(hipEventRecord(w.done, w.last), "hipEventRecord ws");
}

// Before buffers are freed or regrown, the last launch that used them (on
// whatever stream) must have finished.
int ws_quiesce(Ws& w) {
    if (!w.used) return 0;
    if (int rc = done_flush(w)) return rc;
    return hip_status(hipEventSynchronize(w.done), "hipEventSynchronize ws");
}

int ws_faults(Ws& w, bool completed, hipStream_t s);

// SHD_DEBUG_WS_OOM=<tag>: the first growth of the per-bucket counters after
// the tag changes fails with -ENOMEM, once, after the old buffers are freed
// (tests of the callers' retry without the 8-B table, routes.c)
bool dbg_oom_once() {
    static char last[64];
    const char* e = getenv("SHD_DEBUG_WS_OOM");
    if (!e || !*e || strncmp(e, last, sizeof last - 1) == 0) return false;
    strncpy(last, e, sizeof last - 1);
    return true;
}

int ws_reserve(Ws& w, size_t n, size_t m, uint32_t H) {
    int rc = 0;
    if (m + 1 > w.cap_m || H + 1 > w.cap_h) w.clean_now = false; // (new buffers: not cleared)
    if ((n > w.cap_n || m + 1 > w.cap_m || H + 1 > w.cap_h) && (rc = ws_quiesce(w))) return rc;
    if (n > w.cap_n) {
        (void)hipFree(w.tmp);
        (void)hipFree(w.st1);
        (void)hipFree(w.rnk);
        (void)hipFree(w.st2);
        w.tmp = w.st1 = w.st2 = nullptr;
        w.rnk = nullptr;
        w.cap_n = 0;
        const size_t cap = n + n / 8 + 1024;
        if ((rc = hip_status(hipMalloc((void**)&w.tmp, sizeof(ShdDeliv) * cap), "hipMalloc ws.tmp")) ||
            (rc = hip_status(hipMalloc((void**)&w.st1, sizeof(ShdDeliv) * cap), "hipMalloc ws.st1")) ||
            (rc = hip_status(hipMalloc((void**)&w.rnk, sizeof(uint32_t) * cap), "hipMalloc ws.rnk")) ||
            (rc = hip_status(hipMalloc((void**)&w.st2, sizeof(ShdDeliv) * cap), "hipMalloc ws.st2")))
            return rc;
        w.cap_n = cap;
    }
    // merge metadata: segments above kChunk events are at most n / (kChunk + 1)
    const uint32_t cm = (uint32_t)((n + n / 8 + 1024) / (kChunk + 1) + 2);
    if (!w.meta || cm > w.cap_meta) {
        // (an unread fault of the last round lives in the sticky word about to be freed)
        if ((rc = ws_quiesce(w)) || (rc = ws_faults(w, true, nullptr))) return rc;
        (void)hipFree(w.meta);
        w.meta = nullptr;
        w.cap_meta = 0;
        if ((rc = hip_status(hipMalloc((void**)&w.meta, 4 * ((size_t)kMetaHdr + 4ull * cm + cm + 1 +
                                                               (size_t)cm * kMaxPasses)),
                             "hipMalloc ws.meta")))
            return rc;
        if ((rc = hip_status(hipMemset(w.meta, 0, 4 * (size_t)kMetaHdr), "hipMemset ws.meta"))) return rc;
        w.cap_meta = cm;
    }
    if (m + 1 > w.cap_m) {
        (void)hipFree(w.cnt1);
        (void)hipFree(w.off1);
        (void)hipFree(w.bsum);
        (void)hipFree(w.poff);
        (void)hipFree(w.cursor);
        // (nulled at once: a failed allocation below leaves no freed pointer
        // for a retried reserve to free again)
        w.cnt1 = w.off1 = w.bsum = w.poff = w.cursor = nullptr;
        w.cap_m = 0;
        const size_t cap = m + 1 + (m >> 3) + 4096;
        if (dbg_oom_once()) return shd_fail(-ENOMEM, "hipMalloc ws.cnt1: injected (SHD_DEBUG_WS_OOM)");
        if ((rc = hip_status(hipMalloc((void**)&w.cnt1, 4 * cap), "hipMalloc ws.cnt1")) ||
            (rc = hip_status(hipMalloc((void**)&w.off1, 4 * cap), "hipMalloc ws.off1")) ||
            (rc = hip_status(hipMalloc((void**)&w.bsum, 4 * (cap / kScanTile + 2)), "hipMalloc ws.bsum")) ||
            (rc = hip_status(hipMalloc((void**)&w.poff, 4 * cap), "hipMalloc ws.poff")) ||
            (rc = hip_status(hipMalloc((void**)&w.cursor, 4 * (size_t)kMaxBuckets + 64), "hipMalloc ws.cursor")))
            return rc;
        w.cap_m = cap;
    }
    if (H + 1 > w.cap_h) {
        (void)hipFree(w.big);
        (void)hipFree(w.nbig);
        w.big = w.nbig = nullptr;
        w.cap_h = 0;
        const uint32_t cap = H + 1 + 1024;
        if ((rc = hip_status(hipMalloc((void**)&w.big, 4ull * cap), "hipMalloc ws.big")) ||
            (rc = hip_status(hipMalloc((void**)&w.nbig, 16), "hipMalloc ws.nbig")))
            return rc;
        w.cap_h = cap;
    }
    return 0;
}

int cslab_reserve(Ws& w, uint32_t H) {
    const size_t need = (size_t)H * kSlab;
    if (need <= w.cap_cslab) return 0;
    if (int rc = ws_quiesce(w)) return rc;
    (void)hipFree(w.cslab);
    w.cslab = nullptr;
    w.cap_cslab = 0;
    int rc = hip_status(hipMalloc((void**)&w.cslab, sizeof(uint4) * need), "hipMalloc ws.cslab");
    if (!rc) w.cap_cslab = need;
    return rc;
}

int pstage_reserve(Ws& w, size_t need) {
    if (need <= w.cap_pstage) return 0;
    if (int rc = ws_quiesce(w)) return rc;
    (void)hipFree(w.pstage);
    w.pstage = nullptr;
    w.cap_pstage = 0;
    const size_t cap = need + need / 8 + 1024;
    int rc = hip_status(hipMalloc((void**)&w.pstage, sizeof(uint4) * cap), "hipMalloc ws.pstage");
    if (!rc) w.cap_pstage = cap;
    return rc;
}

int slab_reserve(Ws& w, uint32_t H) {
    const size_t need = (size_t)H * kSlab;
    if (need <= w.cap_slab) return 0;
    if (int rc = ws_quiesce(w)) return rc;
    (void)hipFree(w.slab);
    w.slab = nullptr;
    w.cap_slab = 0;
    int rc = hip_status(hipMalloc((void**)&w.slab, sizeof(ShdDeliv) * need), "hipMalloc ws.slab");
    if (!rc) w.cap_slab = need;
    return rc;
}

// SHD_DEBUG_MERGE_SPIN=k: merge waits give up after k spins (0: at once, so
// every multi-pass segment faults -- the test of the fault path); default 2^22
uint32_t merge_spin_limit() {
    const char* v = getenv("SHD_DEBUG_MERGE_SPIN");
    return v ? (uint32_t)strtoul(v, nullptr, 10) : (1u << 22);
}

MergeMeta merge_meta(const Ws& w, unsigned long long* flag) {
    MergeMeta m;
    m.cap_big = w.cap_h;
    m.hdr = w.meta;
    m.seg = reinterpret_cast<uint4*>(w.meta + kMetaHdr);
    m.tpre = w.meta + kMetaHdr + 4ull * w.cap_meta;
    m.done = m.tpre + w.cap_meta + 1;
    m.cap = w.cap_meta;
    m.flag = flag;
    m.spin_limit = merge_spin_limit();
    return m;
}

// k_segsort_mid's dynamic LDS (above the 64 KiB default), set once per process
constexpr size_t kMidLds = sizeof(Ev) * kMidSeg;
int mid_attr() {
    static bool done = false;
    if (done) return 0;
    int rc = hip_status(hipFuncSetAttribute((const void*)k_segsort_mid, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)kMidLds),
                        "hipFuncSetAttribute k_segsort_mid");
    done = rc == 0;
    return rc;
}

// The workspace's sticky fault word (meta hdr[kStickyFault]: the OR of every
// round's fault word since the host last read it) copied to pinned host
// memory at the end of a round, on its stream.  The device only ORs into the
// sticky word, so a round that finishes before the host looked cannot hide
// an earlier round's fault.
// (the sticky word stays on the device; ws_faults reads it once the
// workspace's last use has completed -- nothing on the round's stream)
int copy_faults(Ws&, hipStream_t) { return 0; }

// listed segments: LDS runs, then the merge passes of the larger ones.  A
// round's fault (tiles that gave up waiting for their segment's previous
// pass, a metadata overflow, a stage guard) sets SHD_ROUND_FAULT in the
// caller's counters[0] (flag) during the round and the sticky word, which
// ws_faults reports.
int fault_word_buf(Ws& w);
int sort_listed(Ws& w, const ShdDeliv* unsorted, const uint32_t* offsets, ShdDeliv* out, hipStream_t s,
                unsigned long long* flag) {
    if (int rc = mid_attr()) return rc;
    MergeMeta mm = merge_meta(w, flag);
    // a waited-for part round (w.fin_ask) ends with the merge kernel (see
    // ws_sync): the end marker is set before that launch; SHD_SYNC_COPY /
    // SHD_SYNC_SPIN forms other than the default keep the separate end
    const char* cpv = getenv("SHD_SYNC_COPY");
    const char* spv = getenv("SHD_SYNC_SPIN");
    w.fin_done = false;
    if (w.fin_ask && !(cpv && strcmp(cpv, "memcpy") == 0) && !(spv && (!strcmp(spv, "0") || !strcmp(spv, "event")))) {
        if (int rc = fault_word_buf(w)) return rc;
        w.fault[1] = ~0u;
        mm.fin_host = reinterpret_cast<unsigned long long*>(w.fault);
        mm.fin_m = w.pre_req && w.minw2 && w.pre_req + 1 <= w.cap_m ? (uint32_t)w.pre_req : 0u;
        mm.fin_nbig = w.nbig;
        mm.fin_cnt1 = w.cnt1;
        mm.fin_minw2 = w.minw2;
        w.fin_done = true;
        w.fin_m = mm.fin_m;
    }
    w.fin_ask = false;
    const char* mr = getenv("SHD_MID_RANK");
    // k_segsort_medium (segments of kSmallSeg < n <= kMedSeg events): launched
    // unless this round ends synchronously (fin_done) and the synchronous
    // round before it on this workspace listed no segment at all -- a
    // uniform load, where the launch finds nothing (~4.6 us per round); a
    // medium segment that turns up then is k_segsort_mid's (one workgroup's
    // network per segment, as before the medium kernel), and its round's
    // count launches the kernel again next round.  SHD_MEDIUM_SEG=0: never,
    // 1: always.
    const char* md = getenv("SHD_MEDIUM_SEG");
    const bool med = md && strcmp(md, "0") == 0   ? false
                     : md && strcmp(md, "1") == 0 ? true
                                                  : !(w.fin_done && w.last_listed == 0u);
    if (med) {
        hipLaunchKernelGGL(k_segsort_medium, dim3(2048), dim3(64 * kMedWaves), 0, s, unsorted, offsets, w.big, w.nbig,
                           out, mm.cap_big);
        if (int rc = hip_status(hipGetLastError(), "k_segsort_medium launch")) return rc;
    }
    hipLaunchKernelGGL(k_segsort_mid, dim3(256), dim3(kMidThreads), kMidLds, s, unsorted, offsets, w.big, w.nbig,
                       out, w.st1, mm, (uint32_t)!(mr && strcmp(mr, "0") == 0), (uint32_t)med);
    if (int rc = hip_status(hipGetLastError(), "k_segsort_mid launch")) return rc;
    hipLaunchKernelGGL(k_segsort_merge, dim3(512), dim3(256), 0, s, out, w.st1, mm);
    if (int rc = hip_status(hipGetLastError(), "k_segsort_merge launch")) return rc;
    return copy_faults(w, s);
}

// The sticky fault word as of the workspace's last completed use.  completed:
// the caller has synchronised that use (the report is about the call's own
// round); else non-blocking -- a round still running is checked by a later
// call (an asynchronous caller sees its own round's fault in counters[0]).
// A fault read here is cleared on the device too (s: a stream the next
// launches follow; NULL = synchronously -- nothing is in flight).  -EIO: a
// merge tile hit its spin limit (its input may have been incomplete: the
// destination segment may be mis-sorted), the merge metadata overflowed or a
// stage guard fired.
int fault_word_buf(Ws& w) {
    // (two words: the fault word and, over a host-set all-ones marker, the
    // round's listed-segment count (fin_body) or, in the copy form, meta
    // hdr[kStickyFault + 1] -- never written, so 0: ws_sync's end)
    if (!w.fault && hipHostMalloc((void**)&w.fault, 8, hipHostMallocDefault) != hipSuccess) {
        w.fault = nullptr;
        return shd_fail(-ENOMEM, "hipHostMalloc fault word");
    }
    return 0;
}
int fault_report(Ws& w, hipStream_t s);
int ws_faults(Ws& w, bool completed, hipStream_t s) {
    if (!w.used || !w.meta || w.checked) return 0;
    if (int rc = done_flush(w)) return rc;
    if (!completed && hipEventQuery(w.done) != hipSuccess) return 0;
    // the word, read on a stream of the workspace's own (it waits for nothing
    // else: the use it reports on has completed)
    if (int rc = fault_word_buf(w)) return rc;
    if (!w.rd && hipStreamCreateWithFlags(&w.rd, hipStreamNonBlocking) != hipSuccess) {
        w.rd = nullptr;
        return shd_fail(-EIO, "hipStreamCreate fault read");
    }
    if (int rc = hip_status(hipMemcpyAsync(w.fault, w.meta + kStickyFault, 4, hipMemcpyDeviceToHost, w.rd),
                            "fault word D2H"))
        return rc;
    if (int rc = hip_status(hipStreamSynchronize(w.rd), "fault word read")) return rc;
    return fault_report(w, s);
}
// the synchronous round's last operation: the sticky fault word and the
// zero word beside it (the end marker, see ws_sync) into pinned host memory;
// before it (m > 0) the next part round's resets -- nbig, cnt1[0, m), the
// min word -- so that round launches no k_round_init (every store of this
// workgroup is device-visible before the marker: the host may start the next
// round on another stream as soon as it sees it)
__global__ __launch_bounds__(256) void k_fault_out(const uint32_t* __restrict__ src, unsigned long long* host,
                                                   uint32_t* __restrict__ nbig, uint32_t* __restrict__ cnt1, uint32_t m,
                                                   unsigned long long* __restrict__ minw2) {
    fin_body(src, host, nbig, cnt1, m, minw2);
}
// A synchronous call's end: the fault word copied on the call's own stream
// behind its launches, one wait for both (not a wait for the round and then
// another for the word's copy on a side stream)
int ws_sync(Ws& w, hipStream_t s, const char* what) {
    if (!w.meta) return hip_status(hipStreamSynchronize(s), what);
    if (int rc = fault_word_buf(w)) return rc;
    // SHD_SYNC_SPIN (default 1): the calling thread polls instead of
    // sleeping in hipStreamSynchronize -- the caller waits anyway, and a poll
    // sees the end sooner than a wake-up does (the gap before the next round's
    // launches).  It polls the fault word's copy itself: the copy is the
    // call's last operation on the stream and overwrites a host-set marker
    // with the device's zero word beside the fault word, so the marker's
    // change is the end of every earlier operation of the stream (an event
    // recorded behind it reported the end ~4 us after the copy had landed,
    // profiles/r06u round trace; the GPU idle between rounds 25.6 -> 9.2 us,
    // profiles/r06y_round_gaps.log); the event is still queried every 256 polls
    // so a failed stream ends the wait with its error.  SHD_SYNC_SPIN=event:
    // poll the event alone.
    const char* sp = getenv("SHD_SYNC_SPIN");
    const bool spin = !(sp && strcmp(sp, "0") == 0), marker = !(sp && strcmp(sp, "event") == 0);
    // (the two words are read as one aligned 8-B load: the copy lands them with
    // one 8-B store, so a zero marker comes with its fault word)
    volatile uint64_t* fw = reinterpret_cast<volatile uint64_t*>(w.fault);
    // the copy: one wave storing the 8 B straight into the pinned words (a
    // system-scope store; SHD_SYNC_COPY=memcpy: hipMemcpyAsync, whose blit
    // kernel took 3.7-4.3 us per round in the trace) -- or none at all when
    // the round's merge kernel did that store (fin_done, marker set before
    // its launch: one launch less per round)
    const char* cp = getenv("SHD_SYNC_COPY");
    bool counted = true; // the end word carries the round's listed count (fin_body), not the copy's zero
    if (w.fin_done) {
        w.fin_done = false;
        w.pre_clean = w.fin_m > 0;
        w.pre_m = w.fin_m;
        w.pre_req = 0;
    } else if ((w.fault[1] = ~0u), !(cp && strcmp(cp, "memcpy") == 0)) {
        const uint32_t m = w.pre_req && w.minw2 && w.pre_req + 1 <= w.cap_m ? (uint32_t)w.pre_req : 0u;
        hipLaunchKernelGGL(k_fault_out, dim3(1), dim3(256), 0, s, w.meta + kStickyFault,
                           reinterpret_cast<unsigned long long*>(w.fault), w.nbig, w.cnt1, m, w.minw2);
        if (int rc = hip_status(hipGetLastError(), "fault word store")) return rc;
        w.pre_clean = m > 0;
        w.pre_m = m;
        w.pre_req = 0;
    } else {
        counted = false;
        if (int rc = hip_status(hipMemcpyAsync(w.fault, w.meta + kStickyFault, 8, hipMemcpyDeviceToHost, s),
                                "fault word D2H"))
            return rc;
    }
    if (spin) {
        if (!w.fin && hipEventCreateWithFlags(&w.fin, hipEventDisableTiming) != hipSuccess) w.fin = nullptr;
        if (w.fin && hipEventRecord(w.fin, s) == hipSuccess) {
            hipError_t e = hipErrorNotReady;
            for (uint32_t k = 1;; k++) {
                if (marker && (*fw >> 32) != 0xFFFFFFFFu) {
                    e = hipSuccess;
                    break;
                }
                if ((!marker || (k & 255u) == 0u) && (e = hipEventQuery(w.fin)) != hipErrorNotReady) break;
            }
            if (int rc = hip_status(e, what)) return rc;
            w.last_listed = counted ? (uint32_t)(*fw >> 32) : ~0u;
            if (s == w.last) w.done_pending = false; // (the last use has finished: nothing to record)
            return fault_report(w, s);
        }
    }
    if (int rc = hip_status(hipStreamSynchronize(s), what)) return rc;
    w.last_listed = counted ? (uint32_t)(*fw >> 32) : ~0u;
    if (s == w.last) w.done_pending = false;
    return fault_report(w, s);
}
// *w.fault holds the word of the workspace's last, completed use
int fault_report(Ws& w, hipStream_t s) {
    w.checked = true;
    const uint32_t f = *w.fault;
    if (!f) return 0;
    *w.fault = 0;
    (void)(s ? hipMemsetAsync(w.meta + kStickyFault, 0, 4, s) : hipMemset(w.meta + kStickyFault, 0, 4));
    const uint32_t g = (f >> 24) & 0x7fu;
    return shd_fail(-EIO, "round fault word %#x (%s%s%s%s%s%s)", f,
                    (f & 0xffffffu) ? "merge spin-limit hits" : "", (f & 0x80000000u) ? ", merge metadata overflow" : "",
                    (g & kFaultOvfRange) ? ", overflow event outside its segment" : "",
                    (g & kFaultOvfCap) ? ", overflow count above its list" : "",
                    (g & kFaultBigCap) ? ", big-segment list full" : "",
                    (g & kFaultOff) ? ", offsets above the staging area" : "");
}

// compute units of the current device (cached per device)
int dev_cus() {
    static int cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cus[dev] = v;
    }
    return cus[dev];
}

unsigned grid_for(size_t n, unsigned block, unsigned cap) {
    size_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

// SHD_PLACE=staged selects the two-level staged partition instead of the
// one-pass bucket placement (k_place_bucket, default).
bool staged_partition() {
    const char* v = getenv("SHD_PLACE");
    return v && strcmp(v, "staged") == 0;
}

// SHD_SEGSORT=bitonic selects the bitonic segment network, else rank sort
// SHD_SEGSORT_LDS=0: pass-1 keys by readlane instead of LDS broadcast reads
uint32_t lds_keys() {
    const char* v = getenv("SHD_SEGSORT_LDS");
    return !(v && strcmp(v, "0") == 0);
}
// the part sort's flags word: bit 0 LDS keys, bit 1 (SHD_PART_PERM=1) buckets
// written in order through the LDS permutation -- measured 3-4 us slower per
// round than every event stored at its rank (profiles/r04af_part_perm_probe.log:
// the L2 merges the scattered halves; the extra pass and barrier cost more)
// bit 2 (SHD_SORT_BUCKET=1 sets it): segments of 17..128 events ranked by
// time bucket (wave_bucket_rank) instead of all pairs -- measured slower on
// C3 (sort 0.193-0.195 vs 0.149-0.150 ms in one process,
// profiles/r05c_sort_bucket_rank_probe.log), kept as the A/B form
uint32_t part_sort_flags() {
    const char* v = getenv("SHD_PART_PERM");
    const char* bk = getenv("SHD_SORT_BUCKET");
    const char* x31 = getenv("SHD_SORT_X31");
    return lds_keys() | (v && strcmp(v, "1") == 0 ? 2u : 0u) | (bk && strcmp(bk, "1") == 0 ? 4u : 0u) |
           (x31 && strcmp(x31, "0") == 0 ? 64u : 0u);
}
// Compact 16-B slab records (CSlab) with the rank sort; SHD_SLAB_COMPACT=0
// (or the bitonic segment sort) keeps the 32-B slab
bool compact_slab() {
    const char* v = getenv("SHD_SLAB_COMPACT");
    const char* b = getenv("SHD_SEGSORT");
    return !(v && strcmp(v, "0") == 0) && !(b && strcmp(b, "bitonic") == 0);
}
uint32_t rank_sort() {
    const char* v = getenv("SHD_SEGSORT");
    if (v && strcmp(v, "bitonic") == 0) return 0;
    return 1;
}

constexpr uint32_t kMaxShift = 11; // 2^11 = kMaxPerBucket destinations per bucket

// Buckets: the fewest (widest) that keep a uniform batch's expected events
// per bucket within half the LDS capacity of k_bucket_sort; chunks: about
// kChunks scatter workgroups of whole kBlock-record rows (the last batch of a
// chunk may be partial: the scatter masks it).
int make_bucketing(uint32_t host_lo, uint32_t H, size_t n, Bucketing* out) {
    Bucketing bk;
    bk.host_lo = host_lo;
    bk.H = H;
    bk.shift = 0;
    while ((((size_t)H + (1u << bk.shift) - 1) >> bk.shift) > (size_t)kMaxBuckets) bk.shift++;
    if (bk.shift > kMaxShift) return shd_fail(-E2BIG, "%u destination hosts exceed the partition limit", H);
    while (bk.shift < kMaxShift && H > 0 && (double)n * (double)(2u << bk.shift) / (double)H <= kBucketCap * 0.4)
        bk.shift++;
    bk.nb = (uint32_t)(((size_t)H + (1u << bk.shift) - 1) >> bk.shift);
    if (bk.nb == 0) bk.nb = 1;
    // SHD_SCATTER_CHUNKS=k (64..65536): measurement knob for the workgroup count
    const size_t unit = kBlock;
    size_t nchunks = kChunks;
    if (const char* sc = getenv("SHD_SCATTER_CHUNKS")) {
        const long v = atol(sc);
        if (v >= 64 && v <= 65536) nchunks = (size_t)v;
    }
    size_t chunk = (n + nchunks - 1) / nchunks;
    chunk = (chunk + unit - 1) / unit * unit;
    if (chunk < unit) chunk = unit;
    bk.chunk = (uint32_t)chunk;
    bk.ntiles = (uint32_t)((n + chunk - 1) / chunk);
    if (bk.ntiles == 0) bk.ntiles = 1;
    const char* x = getenv("SHD_XCD_COLS");
    bk.xcd = !(x && strcmp(x, "0") == 0);
    const char* sl = getenv("SHD_SLAB_LAYOUT");
    bk.slab_rm = sl && strcmp(sl, "rank") == 0;
    const char* ag = getenv("SHD_DEST_AGG");
    bk.agg = !(ag && strcmp(ag, "0") == 0);
    bk.rsort = rank_sort();
    *out = bk;
    return 0;
}

// SHD_DEBUG_SYNC=1: synchronise after each stage of a round and name the
// stage whose kernels failed; print the workspace and argument ranges once
// per round and fail on an overlap (diagnostics; asynchronous otherwise)
bool debug_sync() {
    static const bool on = [] {
        const char* v = getenv("SHD_DEBUG_SYNC");
        return v && strcmp(v, "1") == 0;
    }();
    return on;
}
int dbg_sync(hipStream_t s, const char* stage) {
    if (!debug_sync()) return 0;
    const hipError_t e = hipStreamSynchronize(s);
    return e == hipSuccess ? 0 : shd_fail(-EIO, "stage %s: %s", stage, hipGetErrorString(e));
}
int dbg_ranges(const Ws& w, const void* status, size_t n, const void* out, const void* offsets, uint32_t H) {
    if (!debug_sync()) return 0;
    struct R {
        const char* name;
        uintptr_t lo, hi;
    } r[] = {{"ws.tmp", (uintptr_t)w.tmp, (uintptr_t)(w.tmp + w.cap_n)},
             {"ws.st1", (uintptr_t)w.st1, (uintptr_t)(w.st1 + w.cap_n)},
             {"ws.st2", (uintptr_t)w.st2, (uintptr_t)(w.st2 + w.cap_n)},
             {"ws.cnt1", (uintptr_t)w.cnt1, (uintptr_t)(w.cnt1 + w.cap_m)},
             {"ws.big", (uintptr_t)w.big, (uintptr_t)(w.big + w.cap_h)},
             {"ws.nbig", (uintptr_t)w.nbig, (uintptr_t)(w.nbig + 4)},
             {"ws.slab", (uintptr_t)w.slab, (uintptr_t)(w.slab + w.cap_slab)},
             {"status", (uintptr_t)status, (uintptr_t)status + n},
             {"out", (uintptr_t)out, (uintptr_t)out + n * sizeof(ShdDeliv)},
             {"offsets", (uintptr_t)offsets, (uintptr_t)offsets + 4ull * (H + 1)}};
    const int k = (int)(sizeof r / sizeof r[0]);
    for (int i = 0; i < k; i++) fprintf(stderr, "[shd debug] %-8s %#lx..%#lx\n", r[i].name, (unsigned long)r[i].lo,
                                        (unsigned long)r[i].hi);
    for (int i = 0; i < k; i++)
        for (int j = i + 1; j < k; j++)
            if (r[i].lo && r[j].lo && r[i].lo < r[j].hi && r[j].lo < r[i].hi && r[i].hi > r[i].lo && r[j].hi > r[j].lo)
                return shd_fail(-EIO, "debug: %s overlaps %s", r[i].name, r[j].name);
    return 0;
}

// SHD_ROUND_FUSE=0: the three-launch scan and a separate overflow placement
// launch (the launch count before the fused forms; parity-tested)
bool round_fuse() {
    const char* v = getenv("SHD_ROUND_FUSE");
    return !(v && strcmp(v, "0") == 0);
}

// exclusive scan of len counts into out (out[len] = total; counters[0] = total)
void scan_counts(const uint32_t* in, size_t len, uint32_t* out, uint32_t* bsum, unsigned long long* counters,
                 hipStream_t s) {
    if (len <= kScanOneMax && round_fuse()) {
        hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(1024), 0, s, in, len, out, counters);
        return;
    }
    const uint32_t nb = (uint32_t)((len + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(k_scan_local, dim3(nb ? nb : 1), dim3(256), 0, s, in, len, out, bsum);
    const char* s3 = getenv("SHD_SCAN3");
    if (!(s3 && strcmp(s3, "1") == 0)) {
        hipLaunchKernelGGL(k_scan_add_tiles, dim3(grid_for(len + 1, 256, 1u << 30)), dim3(256), 0, s, out, len, bsum,
                           nb, counters);
        return;
    }
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, bsum, nb);
    hipLaunchKernelGGL(k_scan_add, dim3(grid_for(len + 1, 256, 1u << 30)), dim3(256), 0, s, out, len, bsum, nb,
                       counters);
}

// ---- optional per-stage timing with HIP events on the launch stream ----
constexpr int kStages = 4; // 0 packet-scatter, 1 scan, 2 placement, 3 per-bucket / per-destination sort
constexpr int kMaxTimed = 1024;
struct Timing {
    bool on = false;
    int n = 0;
    hipEvent_t ev[kMaxTimed][kStages + 1];
    int8_t at[kMaxTimed][kStages + 1]; // the event a boundary reads (a stage with no kernels: the previous one)
    bool created = false;
    bool enabled = false; // (on: enabled and not paused)
};
Timing g_tm;

void mark(int stage, hipStream_t s) {
    if (g_tm.on && g_tm.n < kMaxTimed) {
        (void)hipEventRecord(g_tm.ev[g_tm.n][stage], s);
        g_tm.at[g_tm.n][stage] = (int8_t)stage;
    }
}
// a boundary with nothing launched since the previous one: no event of its
// own (an event record costs the stream ~5 us)
void mark_same(int stage, int prev) {
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.at[g_tm.n][stage] = g_tm.at[g_tm.n][prev];
}

// scan of the count matrix, atomic-free placement into bucket regions,
// per-bucket LDS sort (shared by both entry points)
int group_and_sort(Ws& w, const ShdDeliv* in, const uint8_t* status, const uint32_t* rank, size_t n, const Bucketing& bk,
                   ShdDeliv* out, uint32_t* offsets, unsigned long long* counters, hipStream_t s) {
    const size_t m = (size_t)bk.nb * bk.ntiles;
    scan_counts(w.cnt1, m, w.off1, w.bsum, counters, s);
    mark(2, s);
    if (staged_partition()) {
        // parts of 2^pshift buckets, at most kPartsTarget of them
        uint32_t pshift = 0;
        while (((bk.nb + (1u << pshift) - 1) >> pshift) > kPartsTarget) pshift++;
        const uint32_t np = (bk.nb + (1u << pshift) - 1) >> pshift;
        const size_t np_cols = (size_t)np * bk.ntiles;
        hipLaunchKernelGGL(k_part_offsets, dim3(grid_for(np_cols > bk.nb ? np_cols : bk.nb, 256, 1u << 30)),
                           dim3(256), 0, s, w.off1, bk, pshift, np, w.poff, w.cursor);
        hipLaunchKernelGGL(k_stage_parts, dim3(bk.ntiles), dim3(kStageBlock), 0, s, in, status, n, bk, pshift, np,
                           w.poff, w.st2);
        hipLaunchKernelGGL(k_refine, dim3(grid_for(n, kStageTile, 1u << 30)), dim3(kStageBlock), 0, s, w.st2, bk,
                           pshift, w.off1, w.cursor, w.st1);
    } else {
        hipLaunchKernelGGL(k_place_bucket, dim3(bk.ntiles), dim3(kPlaceBlock), 0, s, in, status, rank, n, bk,
                           w.off1, w.st1);
    }
    mark(3, s);
    hipLaunchKernelGGL(k_bucket_sort, dim3(bk.nb), dim3(kSortBlock), 0, s, w.st1, bk, w.off1, offsets, out,
                       w.big, w.nbig);
    if (int rc = sort_listed(w, out, offsets, out, s, counters)) return rc; // placed unsorted in out; st1 is free now
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    return hip_status(hipGetLastError(), "group_and_sort launch");
}

// scan of per-destination counts straight into the offsets, atomic-free
// placement by rank, one wave per destination segment
// slab: the scatter already wrote each event to its destination's slab (or
// the overflow list); only overflow events are placed.
int group_and_sort_rank(Ws& w, const ShdDeliv* in, const uint8_t* status, const uint32_t* rank, size_t n,
                        uint32_t host_lo, uint32_t H, ShdDeliv* out, uint32_t* offsets,
                        unsigned long long* counters, hipStream_t s, const ShdDeliv* slab = nullptr,
                        uint32_t slab_rm = 0, const uint4* cslab = nullptr, unsigned long long tbase = 0) {
    scan_counts(w.cnt1, (size_t)H, offsets, w.bsum, counters, s);
    if (int rc = dbg_sync(s, "scan")) return rc;
    mark(2, s);
    const bool fuse = slab && round_fuse();
    if (slab && !fuse)
        hipLaunchKernelGGL(k_place_ovf, dim3(512), dim3(256), 0, s, w.st2, w.nbig + 1, offsets, host_lo,
                           w.st1);
    else if (!slab && n)
        hipLaunchKernelGGL(k_place_rank, dim3(grid_for(n, 256 * kBatch, 1u << 20)), dim3(256), 0, s, in, status, rank,
                           n, host_lo, H, offsets, w.st1, 0u, H);
    if (int rc = dbg_sync(s, "place")) return rc;
    mark(3, s);
    // streaming cache policy (SHD_SEGSORT_NT bits, default 3): 1 the compact
    // slab loads (read once), 2 the output stores (not re-read by the round;
    // streaming them also leaves the next scatter's lines cached): round 0.819
    // -0.826 vs 0.855-0.880 ms in one process (profiles/r03nt_segsort_nt.log)
    const char* ntv = getenv("SHD_SEGSORT_NT");
    const int nt = ntv ? atoi(ntv) : 3;
#define SHD_SEGSORT_LAUNCH(M)                                                                                      \
    hipLaunchKernelGGL(k_segsort_dst<M>, dim3(grid_for(H, 4, 16384)), dim3(256), 0, s, w.st1, offsets, H, host_lo, \
                       out, w.big, w.nbig, rank_sort(), 0u, H, slab, slab_rm, lds_keys(), fuse ? w.st2 : nullptr,   \
                       (uint32_t)w.cap_n, (uint32_t)w.cap_n, cslab, tbase)
    if (nt == 1) SHD_SEGSORT_LAUNCH(1);
    else if (nt == 2) SHD_SEGSORT_LAUNCH(2);
    else if (nt == 3) SHD_SEGSORT_LAUNCH(3);
    else SHD_SEGSORT_LAUNCH(0);
#undef SHD_SEGSORT_LAUNCH
    if (int rc = dbg_sync(s, "k_segsort_dst")) return rc;
    if (int rc = sort_listed(w, w.st1, offsets, out, s, counters)) return rc;
    if (int rc = dbg_sync(s, "k_segsort_mid + k_segsort_merge")) return rc;
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    return hip_status(hipGetLastError(), "group_and_sort_rank launch");
}

// SHD_PACKET_PIPELINE: "slab" (default for the packet round), "rank"
// (per-destination counters + a placement pass over the batch) or "bucket"
// (atomic-free bucket partition).  The slab pipeline needs H x kSlab x 32 B
// of HBM (100k hosts: 0.8 GB); above kMaxSlabBytes it falls back to rank.
enum Pipeline { kBucketPipe = 0, kRankPipe = 1, kSlabPipe = 2, kPartPipe = 3 };
constexpr size_t kMaxSlabBytes = 32ull << 30;

// k_part_sort instances (SHD_PART_SORT, measurement knob): 0: 1024 threads,
// 7,168 events in LDS (one workgroup per CU); 1: 512 threads, 3,584 (two per
// CU); 2: 256 threads, 1,792 (four); 3 (default): 512 threads, 2,304, keys
// for segments up to 128 in LDS (46 KB, 71 VGPRs: three per CU).  The buckets
// are sized for the instance.  C3: round 0.611-0.616 ms with 3 (sort 0.159 ms)
// vs 0.635-0.643 with 1 (sort 0.183, profiles/r04l_part_sort_3wg.log), 0.676
// with 0; 2 needs 12,500 buckets (scatter 0.475 ms, profiles/r04i_part_sort_256.log);
// 4: instance 3 without the LDS keys at 63 VGPRs, four per CU: sort 0.197 ms
// (profiles/r04m_part_sort_occ8.log).
int part_sort_cfg() {
    const char* v = getenv("SHD_PART_SORT");
    const int k = v ? atoi(v) : 3;
    return k >= 0 && k <= 4 ? k : 3;
}
constexpr int kPartSortCap[5] = {7168, 3584, 1792, 2304, 2304};

// Geometry of the part pipeline for n records over H destinations: the
// widest buckets (shift <= 6) whose expected load stays within the LDS sort's
// capacity with room for the spread of a uniform load (6/7 of it); false
// when the buckets would be too many for the scatter's LDS histogram.
bool part_geometry(uint32_t host_lo, uint32_t H, size_t n, unsigned long long tbase, PartGeo* g,
                   unsigned long long barrier) {
    if (!H) return false;
    const double target = kPartSortCap[part_sort_cfg()] * 6.0 / 7.0;
    uint32_t shift = 6;
    while (shift > 0 && (double)n * (double)(1u << shift) / (double)H > target) shift--;
    const uint32_t nb = (uint32_t)(((size_t)H + (1u << shift) - 1) >> shift);
    if (nb > kPartMaxBuckets || (uint64_t)H > (0xFFFFFFFFull >> shift) + 1ull) return false;
    g->host_lo = host_lo;
    g->H = H;
    g->shift = shift;
    g->nb = nb;
    g->cap = (uint32_t)((double)n * (double)(1u << shift) / (double)H * 1.25) + 256u;
    g->tbase = tbase;
    g->xbar = (uint32_t)(barrier - tbase); // (tbase = barrier - 2^31, or 0 below 2^31: <= 2^31)
    return true;
}

// part_ok: the caller runs the part pipeline (the decided round: default; the
// regroup of already-decided events has no part form and takes the slab's)
int pipeline_for(uint32_t H, bool slab_ok, bool part_ok = false) {
    const char* v = getenv("SHD_PACKET_PIPELINE");
    if (v && strcmp(v, "bucket") == 0) return kBucketPipe;
    if (v && strcmp(v, "rank") == 0) return kRankPipe;
    if (part_ok && !(v && strcmp(v, "slab") == 0)) return kPartPipe;
    if (!slab_ok || (size_t)H * kSlab * sizeof(ShdDeliv) > kMaxSlabBytes) return kRankPipe;
    return kSlabPipe;
}

// Orders this call's launches on stream s after the workspace's last use on
// another stream (the buffers are shared); ws_end marks the end of this use.
int ws_begin(Ws& w, hipStream_t s) {
    int dev = 0;
    int rc = hip_status(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    if (w.device >= 0 && w.device != dev) return shd_fail(-EINVAL, "workspace of device %d used on device %d", w.device, dev);
    w.device = dev;
    w.clean_now = w.pre_clean;
    w.pre_clean = false;
    w.pre_req = 0;
    if ((rc = ws_faults(w, false, s))) return rc;
    if ((rc = done_flush(w))) return rc;
    if (!w.done && (rc = hip_status(hipEventCreateWithFlags(&w.done, hipEventDisableTiming), "hipEventCreate ws")))
        return rc;
    if (w.used && w.last != s) return hip_status(hipStreamWaitEvent(s, w.done, 0), "hipStreamWaitEvent ws");
    return 0;
}
int ws_end(Ws& w, hipStream_t s) {
    w.last = s;
    w.used = true;
    w.checked = false;
    // deferred on the null stream only (the synchronous calls' stream, which
    // outlives the workspace; a caller's stream could be destroyed before a
    // deferred record); SHD_WS_LAZY=0: record at once
    const char* e = getenv("SHD_WS_LAZY");
    if (s || (e && strcmp(e, "0") == 0)) return hip_status(hipEventRecord(w.done, s), "hipEventRecord ws");
    w.done_pending = true;
    return 0;
}

} // namespace

// The workspace's faults after its last use, waited for: for callers that
// synchronised their own streams (multi-shard collect, the exchange).
extern "C" int shd_dev_ws_sync(void* ws, void* stream) {
    if (!ws) return hip_status(hipStreamSynchronize((hipStream_t)stream), "stream sync");
    return ws_sync(*static_cast<Ws*>(ws), (hipStream_t)stream, "stream sync");
}

extern "C" int shd_dev_ws_check_faults(void* ws) {
    if (!ws) return 0;
    Ws& w = *static_cast<Ws*>(ws);
    if (!w.used) return 0;
    if (int rc = done_flush(w)) return rc;
    if (int rc = hip_status(hipEventSynchronize(w.done), "hipEventSynchronize ws")) return rc;
    return ws_faults(w, true, nullptr);
}

extern "C" int shd_dev_ws_new(void** ws) {
    *ws = new (std::nothrow) Ws();
    return *ws ? 0 : shd_fail(-ENOMEM, "workspace");
}

extern "C" void shd_dev_ws_free(void* p) {
    if (!p) return;
    Ws* w = static_cast<Ws*>(p);
    if (w->used) {
        (void)done_flush(*w);
        (void)hipEventSynchronize(w->done);
    }
    (void)hipFree(w->tmp);
    (void)hipFree(w->st1);
    (void)hipFree(w->rnk);
    (void)hipFree(w->st2);
    (void)hipFree(w->cnt1);
    (void)hipFree(w->off1);
    (void)hipFree(w->poff);
    (void)hipFree(w->cursor);
    (void)hipFree(w->bsum);
    (void)hipFree(w->big);
    (void)hipFree(w->nbig);
    (void)hipFree(w->slab);
    (void)hipFree(w->cslab);
    (void)hipFree(w->pstage);
    (void)hipFree(w->meta);
    (void)hipFree(w->minw2);
    if (w->fault) (void)hipHostFree(w->fault);
    if (w->rd) (void)hipStreamDestroy(w->rd);
    (void)hipFree(w->xdev);
    if (w->xhost) (void)hipHostFree(w->xhost);
    (void)hipFree(w->xmat);
    if (w->hxmat) (void)hipHostFree(w->hxmat);
    if (w->done) (void)hipEventDestroy(w->done);
    if (w->fin) (void)hipEventDestroy(w->fin);
    if (w->xs) (void)hipStreamDestroy(w->xs);
    for (hipEvent_t e : w->xev)
        if (e) (void)hipEventDestroy(e);
    delete w;
}

// ---- packet-path table (see kPtabFallback) ----
namespace {
__device__ __forceinline__ uint2 ptab_entry(const ShdEntry e) {
    const double d = ceil(e.lat * 1000000.0);
    if (!(e.lat >= 0.0) || !(d < 4294967295.0) || !(e.rel >= 0.0)) return make_uint2(kPtabFallback, 0u);
    // the largest r in [0, 2^31 - 1] with (double)r / 2147483647.0 <= rel: the
    // quotient is monotone in r, so start at floor(rel * (2^31 - 1)) and step
    // to the boundary with the exact test
    double g = floor(e.rel * 2147483647.0);
    int64_t r = g < 0.0 ? 0 : (g > 2147483647.0 ? 2147483647 : (int64_t)g);
    while (r < 2147483647 && (double)(r + 1) / 2147483647.0 <= e.rel) r++;
    while (r >= 0 && (double)r / 2147483647.0 > e.rel) r--;
    if (r < 0) return make_uint2(kPtabFallback, 0u);
    return make_uint2((uint32_t)d, (uint32_t)r);
}
__global__ __launch_bounds__(256) void k_ptab_build(const ShdEntry* __restrict__ tab, size_t n, uint2* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = ptab_entry(tab[i]);
}

// Path packet counters >= thr move to a list (see shd_dev_pcnt_spill): one
// wave-aggregated slot reservation per wave, the appended entries zeroed.
// (d8: the u8 delta layer, NULL: none; a count is cnt + d8, below 2^32)
__global__ __launch_bounds__(256) void k_pcnt_spill(uint32_t* __restrict__ cnt, uint8_t* __restrict__ d8, size_t n,
                                                    uint32_t thr, unsigned long long* __restrict__ list, uint32_t cap,
                                                    uint32_t* __restrict__ nlist) {
    const int lane = threadIdx.x & 63;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    // (uniform trip count over the wave: wave_alloc ballots)
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const size_t i = i0 + threadIdx.x;
        const uint32_t v = i < n ? cnt[i] + (d8 ? (uint32_t)d8[i] : 0u) : 0u;
        const bool hit = i < n && v >= thr && v != 0u;
        const uint32_t slot = wave_alloc(hit, nlist, lane);
        if (hit && slot < cap) {
            list[2 * (size_t)slot] = i;
            list[2 * (size_t)slot + 1] = v;
            cnt[i] = 0u;
            if (d8) d8[i] = 0u;
        }
    }
}

// ---- the counter log's fold (shd_dev_pcnt_fold) ----
// The logged keys (u32 flat entry indices < N <= kFoldMaxN, all-ones = not
// kept) are added into the counters by a two-level partition and one LDS
// accumulation per 32K-counter region:
//   key -> region r = key >> 15 (at most 16,384), coarse c = r >> 7 (<= 128),
//   fine f = r & 127.
// Both levels sort tile-locally -- no histogram pass over the keys and no
// global scan of per-tile counts: each level writes its tiles' digit
// prefixes, and the next level reads runs out of the tiles.
// 1. k_fold_p1: a tile of kFoldT log entries counting-sorted by coarse
//    digit in LDS, written back at the tile's own offset of `part` (kept
//    keys only), with its prefix P1[t][0..128] (P1[t][128]: kept keys).
// 2. k_fold_units: unit (c, g) = coarse digit c over the group g of kFoldG
//    consecutive level-1 tiles; its key count from P1 and the level-2 tiles
//    it needs (ceil(count / kFoldT)); two small scans place every unit's keys
//    (c-major: a coarse digit's units are contiguous) and level-2 tiles.
// 3. k_fold_p2: one workgroup per unit gathers its runs (coarse c of each of
//    its kFoldG tiles, ~60 keys each) in batches of kFoldT, counting-sorts a
//    batch by fine digit in LDS and writes it as u16 region offsets (the
//    coarse and fine digits are implied from here on) at the unit's place,
//    with the level-2 tile's fine prefix F[tile][0..128] and start S[tile].
// 4. k_fold_rn: region r's keys = its fine run in each of its coarse
//    digit's level-2 tiles; rn[r] = its chunks (at most kFoldAddMax keys
//    each, by tile ranges); k_fold_chunks: the chunk list.
// 5. k_fold_add: one workgroup per chunk gathers the region's runs, adds
//    them into LDS counters and the LDS counters into the table: the u8
//    delta layer d8 (a byte past 255 moves into the u32 counter) or the u32
//    counters themselves; a region of several chunks adds with device atomics.
// Every pass streams the keys in whole-line runs; the single-level partition
// over 12k regions (runs of < 1 key per tile) wrote every key as its own
// store: 2.1 ms of a 3.1 ms fold of 184M keys (profiles/r05d_fold_kernel_stats.csv);
// the histogram passes of round 5's two levels took 0.42 of 1.6 ms (r06f).
constexpr uint32_t kFoldRegionBits = 15;          // 32K u32 counters = 128 KB of LDS
constexpr uint32_t kFoldFineBits = 7;              // 128 regions per coarse bucket
constexpr uint32_t kFoldCoarse = 128;              // at most
constexpr unsigned long long kFoldMaxN = 1ull << (kFoldRegionBits + kFoldFineBits + 7); // 2^29 counters
constexpr int kFoldWG = 1024;
constexpr int kFoldPer = 8;                        // keys per thread per tile
constexpr uint32_t kFoldT = kFoldWG * kFoldPer;    // 8,192 keys per tile
constexpr uint32_t kFoldG = 128;                   // level-1 tiles per level-2 unit
constexpr uint32_t kFoldP = kFoldCoarse + 1;       // prefix words per tile
constexpr uint32_t kFoldSent = 0xFFFFFFFFu;
constexpr uint32_t kFoldAddMax = 1u << 18;         // keys per add chunk of a big region (about)
constexpr uint32_t kFoldSmallMax = 65535;          // a small region's keys: its u16 LDS counters cannot wrap
constexpr uint32_t kFoldBig = 0x80000000u;         // rn flag: a big region
constexpr uint32_t kFoldMaxRegions = 1u << 14;

__device__ __forceinline__ uint32_t fold_coarse(uint32_t k) { return k >> (kFoldRegionBits + kFoldFineBits); }
__device__ __forceinline__ uint32_t fold_fine(uint32_t k) { return (k >> kFoldRegionBits) & ((1u << kFoldFineBits) - 1u); }

// the 128 counts h[] of a tile -> exclusive prefix start[] and *tot (64
// threads, two digits per lane; the caller syncs)
__device__ __forceinline__ void fold_prefix128(const uint32_t* h, uint32_t* start, uint32_t* tot) {
    if (threadIdx.x < 64) {
        const uint32_t a = h[2 * threadIdx.x], b = h[2 * threadIdx.x + 1];
        const uint32_t inc = wave_incl_scan(a + b, (int)threadIdx.x);
        start[2 * threadIdx.x] = inc - a - b;
        start[2 * threadIdx.x + 1] = inc - b;
        if (threadIdx.x == 63) *tot = inc;
    }
}

__global__ __launch_bounds__(kFoldWG) void k_fold_p1(const uint32_t* __restrict__ log, size_t L,
                                                     uint32_t* __restrict__ part, uint32_t* __restrict__ P1) {
    __shared__ uint32_t h[kFoldCoarse], start[kFoldCoarse], tot;
    __shared__ uint32_t stage[kFoldT];
    if (threadIdx.x < kFoldCoarse) h[threadIdx.x] = 0u;
    __syncthreads();
    const size_t beg = (size_t)blockIdx.x * kFoldT, end = beg + kFoldT < L ? beg + kFoldT : L;
    uint32_t k[kFoldPer], rk[kFoldPer];
#pragma unroll
    for (int u = 0; u < kFoldPer; u++) {
        const size_t i = beg + (size_t)u * kFoldWG + threadIdx.x;
        k[u] = i < end ? __builtin_nontemporal_load(log + i) : kFoldSent;
    }
#pragma unroll
    for (int u = 0; u < kFoldPer; u++) rk[u] = k[u] != kFoldSent ? atomicAdd(&h[fold_coarse(k[u])], 1u) : 0u;
    __syncthreads();
    fold_prefix128(h, start, &tot);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kFoldPer; u++)
        if (k[u] != kFoldSent) stage[start[fold_coarse(k[u])] + rk[u]] = k[u];
    if (threadIdx.x < kFoldP) P1[(size_t)blockIdx.x * kFoldP + threadIdx.x] = threadIdx.x < kFoldCoarse ? start[threadIdx.x] : tot;
    __syncthreads();
    const uint32_t n = tot;
    for (uint32_t j = threadIdx.x; j < n; j += kFoldWG) part[beg + j] = stage[j];
}

// Group g of kFoldG level-1 tiles (one workgroup): its prefixes through LDS
// (coalesced both ways) into every unit (c, g)'s run table RT[u][i] = {start
// in part, length} of tile g kFoldG + i, and the unit's keys U[u] and level-2
// tiles T2[u] (u = c * ng + g: c-major)
constexpr int kFoldUnitsWG = 1024;
__global__ __launch_bounds__(kFoldUnitsWG) void k_fold_units(const uint32_t* __restrict__ P1, uint32_t nt1, uint32_t C,
                                                             uint32_t ng, uint2* __restrict__ RT,
                                                             uint32_t* __restrict__ U, uint32_t* __restrict__ T2) {
    __shared__ uint32_t P[kFoldG * kFoldP];
    __shared__ uint32_t us[kFoldCoarse];
    const uint32_t g = blockIdx.x, t0 = g * kFoldG, nt = t0 + kFoldG < nt1 ? kFoldG : nt1 - t0;
    for (uint32_t j = threadIdx.x; j < nt * kFoldP; j += kFoldUnitsWG) P[j] = P1[(size_t)t0 * kFoldP + j];
    if (threadIdx.x < kFoldCoarse) us[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < C * kFoldG; j += kFoldUnitsWG) { // (c, i): i fastest
        const uint32_t c = j / kFoldG, i = j - c * kFoldG;
        uint2 e = make_uint2(0u, 0u);
        if (i < nt) {
            const uint32_t a = P[i * kFoldP + c], b = P[i * kFoldP + c + 1];
            e = make_uint2((t0 + i) * kFoldT + a, b - a);
        }
        RT[((size_t)c * ng + g) * kFoldG + i] = e;
        const uint32_t w = wave_incl_scan(e.y, (int)(threadIdx.x & 63)); // (64 i of one c per wave)
        if ((threadIdx.x & 63) == 63) atomicAdd(&us[c], w);
    }
    __syncthreads();
    if (threadIdx.x < C) {
        const uint32_t v = us[threadIdx.x];
        U[(size_t)threadIdx.x * ng + g] = v;
        T2[(size_t)threadIdx.x * ng + g] = (v + kFoldT - 1) / kFoldT;
    }
}

// units blockIdx.x, + gridDim.x, ... (u = (c, g): runs of c out of tiles [g
// kFoldG, ...), RT), each in batches of kFoldT keys (virtual position v: run
// i holds [vs[i], vs[i + 1])).  Persistent, two workgroups per CU, software
// pipelined over its units: while unit i's keys are ranked, sorted and
// written, unit i + 1's keys and unit i + 2's run table are in flight (two
// LDS run tables and two key sets, used in turn; every barrier of the
// processing orders LDS only, so those loads stay in flight).  (One unit at
// a time, waiting on its run table and then its keys: 0.52 ms of a 1.17 ms
// fold, profiles/r06l_fold_timeline.log.)
constexpr int kFoldP2WG = 512;
constexpr int kFoldP2Per = kFoldT / kFoldP2WG; // 16 keys per thread per batch
// a unit's run table in LDS: dl[i] = run i's start in part minus its first
// virtual position, vs[i] = that position (vs[kFoldG] = the unit's keys), pl
// = {key place, first level-2 tile}, map[v - b0] = the run holding virtual
// position v of the batch at b0 (the waves write it run by run: two LDS reads
// per key instead of a binary search's seven)
struct FoldP2Lds {
    uint32_t dl[kFoldG], vs[kFoldG + 1], pl[2];
    uint8_t map[kFoldT];
};
__device__ __forceinline__ void fold_p2_map(FoldP2Lds& L, uint32_t b0) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = wv; i < (int)kFoldG; i += kFoldP2WG / 64) {
        const uint32_t lo = L.vs[i] > b0 ? L.vs[i] : b0, e = b0 + kFoldT, hi = L.vs[i + 1] < e ? L.vs[i + 1] : e;
        for (uint32_t v = lo + (uint32_t)lane; v < hi; v += 64u) L.map[v - b0] = (uint8_t)i;
    }
    lds_barrier();
}
// the keys of batch b0 of the unit whose run table is L, map built for b0
// (sentinel past the unit's keys)
__device__ __forceinline__ void fold_p2_keys(const FoldP2Lds& L, const uint32_t* __restrict__ part, uint32_t b0,
                                             uint32_t (&k)[kFoldP2Per]) {
    const uint32_t U = L.vs[kFoldG];
#pragma unroll
    for (int e = 0; e < kFoldP2Per; e++) {
        const uint32_t j = (uint32_t)e * kFoldP2WG + threadIdx.x, v = b0 + j;
        k[e] = v < U ? part[L.dl[L.map[j]] + v] : kFoldSent;
    }
}
__global__ __launch_bounds__(kFoldP2WG) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_fold_p2(
    const uint32_t* __restrict__ part, const uint2* __restrict__ RT,
                                                       uint32_t units, const uint32_t* __restrict__ Uoff,
                                                       const uint32_t* __restrict__ L2b, uint16_t* __restrict__ out16,
                                                       uint32_t* __restrict__ F, uint32_t* __restrict__ S) {
    __shared__ FoldP2Lds lt[2];
    __shared__ uint32_t h[kFoldCoarse], start[kFoldCoarse], tot;
    __shared__ __attribute__((aligned(16))) uint16_t stage[kFoldT];
    const uint32_t G = gridDim.x;
    uint2 n0 = make_uint2(0u, 0u), n1 = make_uint2(0u, 0u);
    uint32_t np = 0;
    auto fetch = [&](uint32_t u) { // a run table into registers (threads < 64: two runs each; 64, 65: the places)
        if (u >= units) return;
        if (threadIdx.x < 64) {
            n0 = RT[(size_t)u * kFoldG + 2 * threadIdx.x];
            n1 = RT[(size_t)u * kFoldG + 2 * threadIdx.x + 1];
        } else if (threadIdx.x == 64) {
            np = Uoff[u];
        } else if (threadIdx.x == 65) {
            np = L2b[u];
        }
    };
    auto put = [&](FoldP2Lds& L) { // the fetched run table into LDS: runs and their exclusive prefix
        if (threadIdx.x < 64) {
            const uint32_t inc = wave_incl_scan(n0.y + n1.y, (int)threadIdx.x);
            const uint32_t v0 = inc - n0.y - n1.y, v1 = inc - n1.y;
            L.dl[2 * threadIdx.x] = n0.x - v0;
            L.dl[2 * threadIdx.x + 1] = n1.x - v1;
            L.vs[2 * threadIdx.x] = v0;
            L.vs[2 * threadIdx.x + 1] = v1;
            if (threadIdx.x == 63) L.vs[kFoldG] = inc;
        } else if (threadIdx.x < 66) {
            L.pl[threadIdx.x - 64] = np;
        }
    };
    // one batch (keys k) of the unit of L: fine-digit counting sort in LDS,
    // written as u16 region offsets with its prefix and start
    auto batch = [&](const FoldP2Lds& L, uint32_t b0, const uint32_t (&k)[kFoldP2Per]) {
        uint32_t rk[kFoldP2Per];
#pragma unroll
        for (int e = 0; e < kFoldP2Per; e++) rk[e] = k[e] != kFoldSent ? atomicAdd(&h[fold_fine(k[e])], 1u) : 0u;
        lds_barrier();
        fold_prefix128(h, start, &tot);
        lds_barrier();
#pragma unroll
        for (int e = 0; e < kFoldP2Per; e++)
            if (k[e] != kFoldSent)
                stage[start[fold_fine(k[e])] + rk[e]] = (uint16_t)(k[e] & ((1u << kFoldRegionBits) - 1u));
        const uint32_t tile = L.pl[1] + b0 / kFoldT, p0 = L.pl[0] + b0;
        if (threadIdx.x < kFoldP) F[(size_t)tile * kFoldP + threadIdx.x] = threadIdx.x < kFoldCoarse ? start[threadIdx.x] : tot;
        if (threadIdx.x == 0) S[tile] = p0;
        lds_barrier();
        const uint32_t n = tot;
        // (u16 pairs where the batch starts at an even position: kFoldT is even)
        if ((p0 & 1u) == 0u) {
            const uint32_t* st2 = reinterpret_cast<const uint32_t*>(stage);
            uint32_t* o2 = reinterpret_cast<uint32_t*>(out16 + p0);
            for (uint32_t j = threadIdx.x; j < n / 2; j += kFoldP2WG) o2[j] = st2[j];
            if ((n & 1u) && threadIdx.x == 0) out16[p0 + n - 1] = stage[n - 1];
        } else {
            for (uint32_t j = threadIdx.x; j < n; j += kFoldP2WG) out16[p0 + j] = stage[j];
        }
        lds_barrier(); // (stage, h and tot free for the next batch)
        if (threadIdx.x < kFoldCoarse) h[threadIdx.x] = 0u;
        lds_barrier();
    };
    // unit u (run table in Lc, first batch's keys kc, already loaded or in
    // flight) while unit u + G's keys go into kn (its table into Ln) and unit
    // u + 2G's table into registers
    auto step = [&](uint32_t u, FoldP2Lds& Lc, FoldP2Lds& Ln, uint32_t (&kc)[kFoldP2Per], uint32_t (&kn)[kFoldP2Per]) {
        put(Ln); // (unit u + G's table, fetched one step ago)
        lds_barrier();
        if (u + G < units) {
            fold_p2_map(Ln, 0u);
            fold_p2_keys(Ln, part, 0u, kn);
        }
        fetch(u + 2 * G);
        const uint32_t U = Lc.vs[kFoldG];
        if (U) batch(Lc, 0u, kc); // (an empty unit has no level-2 tile: its place is the next unit's)
        for (uint32_t b0 = kFoldT; b0 < U; b0 += kFoldT) { // (block-uniform; units past kFoldT keys: Zipf)
            fold_p2_map(Lc, b0);
            fold_p2_keys(Lc, part, b0, kc);
            batch(Lc, b0, kc);
        }
    };
    if (threadIdx.x < kFoldCoarse) h[threadIdx.x] = 0u;
    uint32_t ka[kFoldP2Per], kb[kFoldP2Per];
    const uint32_t u0 = blockIdx.x;
    fetch(u0);
    put(lt[0]);
    lds_barrier();
    fold_p2_map(lt[0], 0u);
    fold_p2_keys(lt[0], part, 0u, ka);
    fetch(u0 + G);
    for (uint32_t u = u0; u < units; u += 2 * G) { // (block-uniform)
        step(u, lt[0], lt[1], ka, kb);
        if (u + G >= units) break;
        step(u + G, lt[1], lt[0], kb, ka);
    }
}

// coarse digit blockIdx.x: each of its regions' keys over its level-2 tiles
// [L2b[c ng], L2b[(c + 1) ng]) (8 slices of tiles per fine digit, summed in
// LDS) and its chunk count rn[r]
__global__ __launch_bounds__(1024) void k_fold_rn(const uint32_t* __restrict__ F, const uint32_t* __restrict__ L2b,
                                                  uint32_t ng, uint32_t R, uint32_t* __restrict__ rn) {
    __shared__ uint32_t sum[8][kFoldCoarse];
    const uint32_t c = blockIdx.x, f = threadIdx.x & (kFoldCoarse - 1), sl = threadIdx.x >> 7;
    const uint32_t ta = L2b[(size_t)c * ng], tb = L2b[(size_t)(c + 1) * ng];
    uint32_t s = 0;
#pragma unroll 4
    for (uint32_t t = ta + sl; t < tb; t += 8) {
        const uint32_t* p = F + (size_t)t * kFoldP;
        s += p[f + 1] - p[f];
    }
    sum[sl][f] = s;
    __syncthreads();
    const uint32_t r = c * kFoldCoarse + threadIdx.x;
    if (threadIdx.x < kFoldCoarse && r < R) {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) tot += sum[k][threadIdx.x];
        // small: one chunk counted in u16 LDS counters (no count can pass
        // 65,535); else chunks of about kFoldAddMax keys, flagged
        rn[r] = tot <= kFoldSmallMax ? (tot ? 1u : 0u) : ((tot + kFoldAddMax - 1) / kFoldAddMax) | kFoldBig;
    }
}

// The add's work units.  A small region (at most kFoldSmallMax keys: every
// region of a uniform fold of ~20 C3 rounds, ~15k keys) is one chunk of
// list A, counted in u16 LDS counters (64 KB: two workgroups per CU); a big
// region's level-2 tiles go to list B in rn[r] chunks of equal tile ranges,
// counted in u32 LDS counters (a hot region -- Zipf senders, one sender's
// row takes ~10 % of all keys -- spreads over many workgroups that add with
// device atomics instead of one workgroup walking 20M keys while the chip
// idles, the Zipf C3 fold ~4 ms per 20 rounds, profiles/r06b_bench_line.json).
// One workgroup: both lists' exclusive prefixes over the regions; cA[id] =
// r, cB[id] = r | j << 14; n2 = {|A|, |B|}.
__global__ __launch_bounds__(kFoldWG) void k_fold_chunks(const uint32_t* __restrict__ rn, uint32_t R,
                                                         uint32_t* __restrict__ cA, uint32_t* __restrict__ cB,
                                                         uint32_t* __restrict__ n2) {
    __shared__ uint32_t ws[kFoldWG / 64];
    constexpr uint32_t per = kFoldMaxRegions / kFoldWG; // 16 regions per thread
    const uint32_t r0 = threadIdx.x * per;
    uint32_t sa = 0, sb = 0;
    for (uint32_t k = 0; k < per && r0 + k < R; k++) {
        const uint32_t v = rn[r0 + k];
        if (v & kFoldBig) sb += v & ~kFoldBig;
        else sa += v;
    }
    uint32_t ta, tb;
    uint32_t pa = block_excl_scan_n(sa, &ta, ws);
    uint32_t pb = block_excl_scan_n(sb, &tb, ws);
    for (uint32_t k = 0; k < per && r0 + k < R; k++) {
        const uint32_t v = rn[r0 + k];
        if (v & kFoldBig) {
            for (uint32_t j = 0; j < (v & ~kFoldBig); j++) cB[pb++] = (r0 + k) | (j << 14);
        } else if (v) {
            cA[pa++] = r0 + k;
        }
    }
    if (threadIdx.x == 0) n2[0] = ta, n2[1] = tb;
}

// chunk blockIdx.x of list A (kSmall: region r, all its level-2 tiles) or
// B (region r, tiles [ta + j nt / n, ta + (j + 1) nt / n) of coarse c's
// level-2 tiles).  The region's runs are gathered a tile per thread (start,
// length), each wave walking its threads' runs 8 at a time (two keys per
// lane per run in flight; longer runs loop); the keys are region offsets
// (u16).  kSmall: u16 counters packed in pairs (the chunk's keys are at most
// 65,535), 64 KB of LDS.
// kD8: the counts go to the u8 delta layer d8 (16-B aligned at index 0,
// readable up to N rounded up to 16): 16 counters per lane-step, one 16-B
// load (issued before the gathers) and store of their delta bytes; a byte
// whose sum passes 255 moves the whole sum into dense (a device atomic) and
// restarts at 0 -- the region's HBM traffic is its 32 KB of deltas, not its
// 128 KB of u32 counters.  Else the u32 counters are read-modify-written 16 B
// per lane (dense 16-B aligned, the caller checks) or one per lane.
template <bool kD8, bool kVec, bool kSmall>
__device__ __forceinline__ void fold_add_chunk(uint32_t id, const uint16_t* __restrict__ keys,
                                               const uint32_t* __restrict__ F, const uint32_t* __restrict__ S,
                                               const uint32_t* __restrict__ L2b, uint32_t ng,
                                               const uint32_t* __restrict__ rn, const uint32_t* __restrict__ cmap,
                                               uint32_t* __restrict__ dense, unsigned long long N,
                                               unsigned long long n0, uint8_t* __restrict__ d8, uint32_t* fc) {
    const uint32_t cm = cmap[id], r = cm & 0x3FFFu, jc = kSmall ? 0u : cm >> 14;
    const uint32_t c = r >> kFoldFineBits, f = r & ((1u << kFoldFineBits) - 1u);
    const uint32_t ta = L2b[(size_t)c * ng], ntl = L2b[(size_t)(c + 1) * ng] - ta, n = kSmall ? 1u : rn[r] & ~kFoldBig;
    const uint32_t t0 = ta + (uint32_t)((unsigned long long)jc * ntl / n),
                   t1 = ta + (uint32_t)((unsigned long long)(jc + 1) * ntl / n);
    const bool shared_region = n > 1; // (block-uniform) other chunks add to it too
    constexpr uint32_t R = 1u << kFoldRegionBits;
    constexpr int kU = R / 16 / kFoldWG; // 2: 16 counters per lane-step, the whole region
    const unsigned long long rb = (unsigned long long)r << kFoldRegionBits;
    const uint32_t lim = N - rb < R ? (uint32_t)(N - rb) : R;
    const uint32_t lim16 = (lim + 15u) / 16u;
    const int lane = threadIdx.x & 63;
    uint4* d16 = reinterpret_cast<uint4*>(d8 + rb);
    uint4 dv[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
        const uint32_t q = threadIdx.x + (uint32_t)u * kFoldWG;
        // (only groups at or past the first counter's: a shard's first region
        // starts below its rows, where no delta byte is allocated)
        dv[u] = kD8 && !shared_region && q < lim16 && rb + 16u * q >= (n0 & ~15ull) ? d16[q] : uint4{0u, 0u, 0u, 0u};
    }
    constexpr uint32_t kWords = kSmall ? R / 2 : R;
    for (uint32_t j = threadIdx.x; j < kWords / 4; j += kFoldWG) reinterpret_cast<uint4*>(fc)[j] = uint4{0u, 0u, 0u, 0u};
    lds_barrier(); // (LDS only: the delta loads stay in flight)
    // one key into the LDS counters
    auto count = [&](uint32_t k) {
        if (kSmall) atomicAdd(&fc[k >> 1], 1u << ((k & 1u) << 4));
        else atomicAdd(&fc[k], 1u);
    };
    const int wv = threadIdx.x >> 6;
    for (uint32_t tb0 = t0; tb0 < t1; tb0 += kFoldWG) { // (block-uniform)
        // tile tb0 + wv + 16 lane: every wave holds ~1/16 of the runs in its low lanes
        const uint32_t t = tb0 + (uint32_t)wv + 16u * (uint32_t)lane;
        uint32_t rs = 0, rl = 0;
        if (t < t1) {
            const uint32_t* p = F + (size_t)t * kFoldP;
            const uint32_t a = p[f];
            rs = S[t] + a;
            rl = p[f + 1] - a;
        }
        const unsigned long long live = __ballot(t < t1);
        const int nl = live ? 64 - __builtin_clzll(live) : 0; // (wave-uniform)
        for (int l0 = 0; l0 < nl; l0 += 8) { // this wave's runs, 8 at a time
            uint32_t k0[8], k1[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)rs, l0 + e);
                const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)rl, l0 + e);
                k0[e] = (uint32_t)lane < m ? keys[s + lane] : kFoldSent;
                k1[e] = (uint32_t)lane + 64u < m ? keys[s + 64 + lane] : kFoldSent;
            }
#pragma unroll
            for (int e = 0; e < 8; e++) {
                if (k0[e] != kFoldSent) count(k0[e]);
                if (k1[e] != kFoldSent) count(k1[e]);
            }
#pragma unroll
            for (int e = 0; e < 8; e++) { // (runs past 128 keys: hot regions)
                const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)rs, l0 + e);
                const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)rl, l0 + e);
                for (uint32_t i = 128u + (uint32_t)lane; i < m; i += 64u) count(keys[s + i]);
            }
        }
    }
    __syncthreads();
    if (!kSmall && shared_region) { // a hot region's chunk: device atomics for its nonzero counters
        for (uint32_t j = threadIdx.x; j < lim; j += kFoldWG) {
            const uint32_t v = fc[j];
            if (v) atomicAdd(dense + rb + j, v);
        }
        return;
    }
    const uint4* f4 = reinterpret_cast<const uint4*>(fc);
    // counters [4 i, 4 i + 4) of the LDS counters
    auto four = [&](uint32_t i) -> uint4 {
        if (!kSmall) return f4[i];
        const uint2 w = reinterpret_cast<const uint2*>(fc)[i];
        return uint4{w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16};
    };
    if (kD8) {
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * kFoldWG;
            if (q >= lim16) continue;
            uint4 v[4];
            uint32_t o = 0u;
#pragma unroll
            for (int w = 0; w < 4; w++) {
                v[w] = four(4 * q + w);
                o |= v[w].x | v[w].y | v[w].z | v[w].w;
            }
            if (!o) continue;
            uint32_t dw[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w};
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const uint32_t cc[4] = {v[w].x, v[w].y, v[w].z, v[w].w};
                uint32_t nw = 0u;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    uint32_t x = ((dw[w] >> (8 * b)) & 0xFFu) + cc[b];
                    if (x > 0xFFu) { // (rare: a pair past 255 since its last move)
                        atomicAdd(dense + rb + 16u * q + 4u * w + b, x);
                        x = 0u;
                    }
                    nw |= x << (8 * b);
                }
                dw[w] = nw;
            }
            d16[q] = uint4{dw[0], dw[1], dw[2], dw[3]};
        }
        return;
    }
    uint32_t j0 = 0;
    if (kVec) { // eight loads in flight per lane before the stores
        constexpr int kV = R / 4 / kFoldWG; // 8: the whole region in one pass
        const uint32_t lim4 = lim / 4;
        uint4* dd4 = reinterpret_cast<uint4*>(dense + rb);
        uint4 v[kV], d[kV];
#pragma unroll
        for (int u = 0; u < kV; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * kFoldWG;
            v[u] = q < lim4 ? four(q) : uint4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < kV; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * kFoldWG;
            if (q < lim4 && (v[u].x | v[u].y | v[u].z | v[u].w)) d[u] = dd4[q];
        }
#pragma unroll
        for (int u = 0; u < kV; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * kFoldWG;
            if (q < lim4 && (v[u].x | v[u].y | v[u].z | v[u].w))
                dd4[q] = uint4{d[u].x + v[u].x, d[u].y + v[u].y, d[u].z + v[u].z, d[u].w + v[u].w};
        }
        j0 = lim4 * 4; // (a partial last region's tail: one counter per lane)
    }
    for (uint32_t j = j0 + threadIdx.x; j < lim; j += kFoldWG) {
        const uint32_t v = kSmall ? (fc[j >> 1] >> ((j & 1u) << 4)) & 0xFFFFu : fc[j];
        if (v) dense[rb + j] += v;
    }
}

// chunks blockIdx.x, + gridDim.x, ... of the list (list B's grid is a few
// per CU: its length is known on the device only)
template <bool kD8, bool kVec, bool kSmall>
__global__ __launch_bounds__(kFoldWG) void k_fold_add(const uint16_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ F, const uint32_t* __restrict__ S,
                                                      const uint32_t* __restrict__ L2b, uint32_t ng,
                                                      const uint32_t* __restrict__ rn,
                                                      const uint32_t* __restrict__ cmap,
                                                      const uint32_t* __restrict__ nchunks,
                                                      uint32_t* __restrict__ dense, unsigned long long N,
                                                      unsigned long long n0, uint8_t* __restrict__ d8) {
    extern __shared__ uint32_t fc[];
    const uint32_t nc = *nchunks;
    for (uint32_t id = blockIdx.x; id < nc; id += gridDim.x) { // (block-uniform)
        if (id != blockIdx.x) __syncthreads(); // (the last chunk's LDS reads before the reset)
        fold_add_chunk<kD8, kVec, kSmall>(id, keys, F, S, L2b, ng, rn, cmap, dense, N, n0, d8, fc);
    }
}

struct FoldScratch {
    uint32_t* part = nullptr; // level-1 output (L keys)
    size_t cap_part = 0;
    uint32_t* P1 = nullptr; // level-1 prefixes (nt1 x 129)
    size_t cap_P1 = 0;
    uint32_t* un = nullptr; // U | Uoff | T2 | L2b (4 x (units + 1))
    size_t cap_un = 0;
    uint32_t* RT = nullptr; // the units' run tables (units x kFoldG uint2)
    size_t cap_RT = 0;
    uint32_t* F = nullptr; // level-2 prefixes (tiles x 129) | S (tiles)
    size_t cap_F = 0;
    uint32_t* cmap = nullptr; // rn (kFoldMaxRegions) | nchunks | cmap
    size_t cap_cmap = 0;
    uint32_t* bsum = nullptr;
    size_t cap_bsum = 0;
};

int fold_grow(uint32_t** p, size_t* cap, size_t need, const char* what) {
    if (need <= *cap) return 0;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (int r = hip_status(hipMalloc((void**)p, 4 * need), what)) return r;
    *cap = need;
    return 0;
}

struct FoldGeo {
    size_t nt1, ng, units, tiles2; // level-1 tiles, unit groups, units (at most), level-2 tiles (at most)
};
FoldGeo fold_geo(size_t L, uint32_t C) {
    FoldGeo q;
    q.nt1 = (L + kFoldT - 1) / kFoldT;
    q.ng = (q.nt1 + kFoldG - 1) / kFoldG;
    q.units = (size_t)C * q.ng;
    q.tiles2 = q.units + L / kFoldT + 1;
    return q;
}
// the add's chunk list: at most one per region plus one per kFoldAddMax keys
// list B's chunks: at most one per kFoldAddMax keys plus one per big region
size_t fold_max_chunks(size_t L) { return L / kFoldAddMax + L / (kFoldSmallMax + 1) + 1; }

// buffers for folds of up to L keys (grow-only; reserved with the log so that
// a fold inside a timed region allocates nothing)
int fold_reserve(FoldScratch& f, size_t L) {
    const FoldGeo q = fold_geo(L, kFoldCoarse);
    const size_t mb = (q.units + 1) / kScanTile + 2;
    int rc;
    if ((rc = fold_grow(&f.part, &f.cap_part, L ? L : 1, "hipMalloc fold part")) ||
        (rc = fold_grow(&f.P1, &f.cap_P1, q.nt1 * kFoldP + 1, "hipMalloc fold P1")) ||
        (rc = fold_grow(&f.un, &f.cap_un, 4 * (q.units + 1), "hipMalloc fold units")) ||
        (rc = fold_grow(&f.RT, &f.cap_RT, 2 * q.units * kFoldG, "hipMalloc fold runs")) ||
        (rc = fold_grow(&f.F, &f.cap_F, q.tiles2 * (kFoldP + 1), "hipMalloc fold F")) ||
        (rc = fold_grow(&f.bsum, &f.cap_bsum, mb, "hipMalloc fold scan")) ||
        (rc = fold_grow(&f.cmap, &f.cap_cmap, 2 * kFoldMaxRegions + 2 + fold_max_chunks(L), "hipMalloc fold chunks")))
        return rc;
    return 0;
}

// (log: the input and, as u16, the level-2 output -- one scratch array of L
// keys besides it)
int pcnt_fold(uint32_t* log, size_t L, uint32_t* dense, uint8_t* d8, unsigned long long n0, unsigned long long N,
              FoldScratch& f, hipStream_t s) {
    if (N > kFoldMaxN) return shd_fail(-EINVAL, "fold: %llu counters exceed the fold's %llu", N, kFoldMaxN);
    if (d8 && ((uintptr_t)d8 & 15u)) return shd_fail(-EINVAL, "fold: the delta layer is not 16-B aligned");
    if (int rc = fold_reserve(f, L)) return rc;
    static bool attr = false;
    if (!attr) {
        for (const void* fn : {(const void*)k_fold_add<true, false, false>, (const void*)k_fold_add<false, true, false>,
                               (const void*)k_fold_add<false, false, false>, (const void*)k_fold_add<true, false, true>,
                               (const void*)k_fold_add<false, true, true>, (const void*)k_fold_add<false, false, true>})
            if (int rc = hip_status(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                        4 << kFoldRegionBits),
                                    "hipFuncSetAttribute k_fold_add"))
                return rc;
        attr = true;
    }
    const uint32_t R = (uint32_t)(((N - 1) >> kFoldRegionBits) + 1);
    const uint32_t C = ((R - 1) >> kFoldFineBits) + 1;
    const FoldGeo q = fold_geo(L, C);
    const uint32_t units = (uint32_t)q.units, ng = (uint32_t)q.ng;
    uint32_t* U = f.un;
    uint32_t* Uoff = U + (units + 1);
    uint32_t* T2 = Uoff + (units + 1);
    uint32_t* L2b = T2 + (units + 1);
    uint2* RT = reinterpret_cast<uint2*>(f.RT);
    uint32_t* F = f.F;
    uint32_t* S = F + q.tiles2 * kFoldP;
    uint32_t* rn = f.cmap;
    uint32_t* n2 = rn + kFoldMaxRegions;
    uint32_t* cA = n2 + 2;
    uint32_t* cB = cA + kFoldMaxRegions;
    uint16_t* out16 = reinterpret_cast<uint16_t*>(log);
    hipLaunchKernelGGL(k_fold_p1, dim3((unsigned)q.nt1), dim3(kFoldWG), 0, s, log, L, f.part, f.P1);
    hipLaunchKernelGGL(k_fold_units, dim3(ng), dim3(kFoldUnitsWG), 0, s, f.P1, (uint32_t)q.nt1, C, ng, RT, U, T2);
    scan_counts(U, units, Uoff, f.bsum, nullptr, s);
    scan_counts(T2, units, L2b, f.bsum, nullptr, s);
    // SHD_FOLD_P2_GRID: the persistent grid (default two workgroups per CU)
    const char* pg = getenv("SHD_FOLD_P2_GRID");
    const uint32_t g2 = pg && atoi(pg) > 0 ? (uint32_t)atoi(pg) : 2u * (uint32_t)dev_cus();
    hipLaunchKernelGGL(k_fold_p2, dim3(units < g2 ? units : g2), dim3(kFoldP2WG), 0, s, f.part, RT, units, Uoff, L2b,
                       out16, F, S);
    hipLaunchKernelGGL(k_fold_rn, dim3(C), dim3(1024), 0, s, F, L2b, ng, R, rn);
    hipLaunchKernelGGL(k_fold_chunks, dim3(1), dim3(kFoldWG), 0, s, rn, R, cA, cB, n2);
    // (grids: the lists' upper bounds; the rest exit at once)
    const uint32_t gA = R, gB = (uint32_t)(fold_max_chunks(L) < 128 ? fold_max_chunks(L) : 128);
    // SHD_FOLD_VEC=0: the scalar read-modify-write of the u32 counters
    const char* fv = getenv("SHD_FOLD_VEC");
#define SHD_FOLD_ADD(D8, VEC)                                                                                         \
    do {                                                                                                              \
        hipLaunchKernelGGL((k_fold_add<D8, VEC, true>), dim3(gA), dim3(kFoldWG), (size_t)2 << kFoldRegionBits, s,     \
                           out16, F, S, L2b, ng, rn, cA, n2, dense, N, n0, d8);                                       \
        hipLaunchKernelGGL((k_fold_add<D8, VEC, false>), dim3(gB), dim3(kFoldWG), (size_t)4 << kFoldRegionBits, s,    \
                           out16, F, S, L2b, ng, rn, cB, n2 + 1, dense, N, n0, d8);                                   \
    } while (0)
    if (d8) SHD_FOLD_ADD(true, false);
    else if (((uintptr_t)dense & 15u) == 0 && !(fv && strcmp(fv, "0") == 0)) SHD_FOLD_ADD(false, true);
    else SHD_FOLD_ADD(false, false);
#undef SHD_FOLD_ADD
    return hip_status(hipGetLastError(), "pcnt fold launch");
}

} // namespace

extern "C" int shd_dev_pcnt_fold_reserve(size_t L, void** scratch) {
    if (!*scratch && !(*scratch = new (std::nothrow) FoldScratch())) return shd_fail(-ENOMEM, "fold scratch");
    return fold_reserve(*static_cast<FoldScratch*>(*scratch), L);
}

extern "C" int shd_dev_pcnt_fold(void* log, size_t L, uint32_t* dense, uint8_t* d8, uint64_t n0, uint64_t N,
                                 void** scratch, void* stream) {
    if (!L || !N) return 0;
    if (!*scratch && !(*scratch = new (std::nothrow) FoldScratch())) return shd_fail(-ENOMEM, "fold scratch");
    return pcnt_fold(static_cast<uint32_t*>(log), L, dense, d8, n0, N, *static_cast<FoldScratch*>(*scratch),
                     (hipStream_t)stream);
}

extern "C" void shd_dev_pcnt_scratch_free(void* scratch) {
    if (!scratch) return;
    FoldScratch* f = static_cast<FoldScratch*>(scratch);
    (void)hipFree(f->part);
    (void)hipFree(f->P1);
    (void)hipFree(f->un);
    (void)hipFree(f->RT);
    (void)hipFree(f->F);
    (void)hipFree(f->bsum);
    (void)hipFree(f->cmap);
    delete f;
}

extern "C" int shd_dev_pcnt_spill(uint32_t* cnt, uint8_t* d8, size_t n, uint32_t thr, uint64_t* d_list, size_t cap,
                                  uint32_t* d_nlist, size_t* appended) {
    *appended = 0;
    if (!n) return 0;
    if (cap > 0xFFFFFFFFull) cap = 0xFFFFFFFFull;
    int rc = hip_status(hipMemset(d_nlist, 0, 4), "hipMemset spill count");
    if (rc) return rc;
    hipLaunchKernelGGL(k_pcnt_spill, dim3(grid_for(n, 256, 8192)), dim3(256), 0, nullptr, cnt, d8, n, thr,
                       (unsigned long long*)d_list, (uint32_t)cap, d_nlist);
    if ((rc = hip_status(hipGetLastError(), "k_pcnt_spill launch"))) return rc;
    uint32_t m = 0;
    if ((rc = hip_status(hipMemcpy(&m, d_nlist, 4, hipMemcpyDeviceToHost), "spill count D2H"))) return rc;
    *appended = m < cap ? m : cap;
    return 0;
}

extern "C" int shd_dev_ptab_build(const ShdEntry* tab, size_t nent, void* d_out, void* stream) {
    if (!nent) return 0;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_ptab_build, dim3(grid_for(nent, 256, 32768)), dim3(256), 0, s, tab, nent,
                       static_cast<uint2*>(d_out));
    int rc = hip_status(hipGetLastError(), "k_ptab_build launch");
    return rc ? rc : hip_status(hipStreamSynchronize(s), "k_ptab_build");
}

// Grow-only scratch of the multi-GPU exchange (device + pinned host), so a
// round allocates nothing: hipFree / hipHostFree synchronise the device.
// Callers run on one stream and synchronise it before returning, so a grow
// only waits for the workspace's last round.
// The exchange's count matrix (world x (world + 2) u64, device + pinned
// host), allocated once per workspace.
extern "C" int shd_dev_ws_xmat(void* ws, size_t words, uint64_t** d, uint64_t** h) {
    if (!ws) return shd_fail(-ENOMEM, "no round workspace");
    Ws& w = *static_cast<Ws*>(ws);
    if (words > kXmatWords) return shd_fail(-EINVAL, "count matrix of %zu words", words);
    if (!w.xmat) {
        if (int rc = hip_status(hipMalloc((void**)&w.xmat, 8 * kXmatWords), "hipMalloc count matrix")) return rc;
        if (hipHostMalloc((void**)&w.hxmat, 8 * kXmatWords, hipHostMallocDefault) != hipSuccess) {
            w.hxmat = nullptr;
            (void)hipFree(w.xmat);
            w.xmat = nullptr;
            return shd_fail(-ENOMEM, "hipHostMalloc count matrix");
        }
    }
    *d = w.xmat;
    *h = w.hxmat;
    return 0;
}

extern "C" int shd_dev_ws_xchg_sync_objs(void* ws, void** xfer_stream, void** events, int nevents) {
    if (!ws) return shd_fail(-ENOMEM, "no round workspace");
    Ws& w = *static_cast<Ws*>(ws);
    if (nevents > kXchgEvents) return shd_fail(-EINVAL, "%d exchange events > %d", nevents, kXchgEvents);
    int rc = 0;
    if (!w.xs && (rc = hip_status(hipStreamCreateWithFlags(&w.xs, hipStreamNonBlocking), "hipStreamCreate exchange")))
        return rc;
    for (int k = 0; k < nevents; k++) {
        if (!w.xev[k] && (rc = hip_status(hipEventCreate(&w.xev[k]), "hipEventCreate exchange"))) return rc;
        events[k] = w.xev[k];
    }
    *xfer_stream = w.xs;
    return 0;
}

extern "C" int shd_dev_ws_scratch(void* ws, size_t dev_bytes, size_t host_bytes, void** d, void** h) {
    if (!ws) return shd_fail(-ENOMEM, "no round workspace");
    Ws& w = *static_cast<Ws*>(ws);
    int rc = 0;
    if (dev_bytes > w.cap_xdev) {
        if ((rc = ws_quiesce(w))) return rc;
        (void)hipFree(w.xdev);
        w.xdev = nullptr;
        w.cap_xdev = 0;
        const size_t cap = dev_bytes + dev_bytes / 4 + 256;
        if ((rc = hip_status(hipMalloc(&w.xdev, cap), "hipMalloc exchange scratch"))) return rc;
        w.cap_xdev = cap;
    }
    if (host_bytes > w.cap_xhost) {
        if ((rc = ws_quiesce(w))) return rc;
        if (w.xhost) (void)hipHostFree(w.xhost);
        w.xhost = nullptr;
        w.cap_xhost = 0;
        const size_t cap = host_bytes + host_bytes / 4 + 256;
        if ((rc = hip_status(hipHostMalloc(&w.xhost, cap, hipHostMallocDefault), "hipHostMalloc exchange scratch")))
            return rc;
        w.cap_xhost = cap;
    }
    if (d) *d = w.xdev;
    if (h) *h = w.xhost;
    return 0;
}

// The part pipeline's round (see k_part_scatter): reset, partitioned
// scatter, per-bucket LDS sort, listed segments.  Stage timing: 0 scatter, 1
// (no scan), 2 (no placement), 3 the bucket sort and the listed segments.
// k_part_scatter instances (SHD_PART_SCATTER, measurement knob): 0 LDS
// staging, 1024 threads x 4096 records; 1 registers, 1024 x 4096 (default:
// round 0.670 vs 0.734-0.744 ms, profiles/r04b_part_scatter_variants.log);
// 2 registers, 512 x 2048; 3 registers, 256 x 2048 (8 per thread)
struct PartCfg {
    const void* fn;
    int wg, ch;
    bool lds;
    int pipe = 0; // k_part_scatter_pipe: persistent workgroups per CU
    int split = 0; // k_part_decide (records per thread) + k_part_place
};
int part_probe() {
    const char* v = getenv("SHD_PART_PROBE");
    const int k = v ? atoi(v) : 0; // (the instantiated bit sets)
    return k == 1 || k == 2 || k == 4 || k == 8 || k == 6 || k == 5 || k == 7 || k == 15 ? k : 0;
}
PartCfg part_cfg(uint32_t nb) {
    const char* v = getenv("SHD_PART_SCATTER");
    int k = v ? atoi(v) : 1;
    if (k == 0 && nb > kPartMaxBucketsLds) k = 1; // (the LDS-staged form's histogram limit)
    if (k == 1) return {(const void*)k_part_scatter<1024, 4096, false>, 1024, 4096, false};
    if (k == 2) return {(const void*)k_part_scatter<512, 2048, false>, 512, 2048, false};
    if (k == 3) return {(const void*)k_part_scatter<256, 2048, false>, 256, 2048, false};
    if (k == 4) return {(const void*)k_part_scatter<1024, 4096, false, 0, 8>, 1024, 4096, false};
    if (k == 5) return {(const void*)k_part_scatter<512, 4096, false>, 512, 4096, false};
    if (k == 6) return {(const void*)k_part_scatter<1024, 8192, false>, 1024, 8192, false};
    if (k == 12) return {(const void*)k_part_scatter<1024, 16384, false>, 1024, 16384, false};
    if (k == 10 || k == 11) return {(const void*)k_part_place<1024, 4096>, 1024, 4096, false, 0, k == 10 ? 4 : 2};
    if ((k == 7 || k == 8 || k == 9) && nb > kPartPipeMaxBuckets) k = 1;
    if (k == 7) return {(const void*)k_part_scatter_pipe<1024, 2048>, 1024, 2048, false, 1};
    if (k == 8) return {(const void*)k_part_scatter_pipe<512, 1024>, 512, 1024, false, 2};
    if (k == 9) return {(const void*)k_part_scatter_pipe<256, 512>, 256, 512, false, 3};
    return {(const void*)k_part_scatter<1024, 4096, true>, 1024, 4096, true};
}
size_t part_lds(const PartCfg& f, uint32_t nb) {
    return f.lds ? (size_t)f.ch * 20 + 12u * nb + 4 : 8u * nb;
}
int part_attr() {
    static bool done = false;
    if (done) return 0;
    const PartCfg cfgs[] = {{(const void*)k_part_scatter<1024, 4096, true>, 1024, 4096, true},
                            {(const void*)k_part_scatter<1024, 4096, false>, 1024, 4096, false},
                            {(const void*)k_part_scatter<512, 2048, false>, 512, 2048, false},
                            {(const void*)k_part_scatter<256, 2048, false>, 256, 2048, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 0, 8>, 1024, 4096, false},
                            {(const void*)k_part_scatter<512, 4096, false>, 512, 4096, false},
                            {(const void*)k_part_scatter<1024, 8192, false>, 1024, 8192, false},
                            {(const void*)k_part_scatter<1024, 16384, false>, 1024, 16384, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 1>, 1024, 4096, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 2>, 1024, 4096, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 4>, 1024, 4096, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 8>, 1024, 4096, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 6>, 1024, 4096, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 5>, 1024, 4096, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 7>, 1024, 4096, false},
                            {(const void*)k_part_scatter<1024, 4096, false, 15>, 1024, 4096, false},
                            {(const void*)k_part_scatter_pipe<1024, 2048>, 1024, 2048, false},
                            {(const void*)k_part_scatter_pipe<512, 1024>, 512, 1024, false},
                            {(const void*)k_part_scatter_pipe<256, 512>, 256, 512, false},
                            {(const void*)k_part_place<1024, 4096>, 1024, 4096, false}};
    if (int rc = hip_status(hipFuncSetAttribute((const void*)k_wide_group, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                (int)(4 * kPartMaxBuckets)),
                            "hipFuncSetAttribute k_wide_group"))
        return rc;
    for (const PartCfg& f : cfgs)
        if (int rc = hip_status(hipFuncSetAttribute(f.fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)part_lds(f, f.lds ? kPartMaxBucketsLds : kPartMaxBuckets)),
                                "hipFuncSetAttribute k_part_scatter"))
            return rc;
    done = true;
    return 0;
}

// reset + k_part_scatter of a part round (counters, gcnt / wcnt in cnt1)
int part_front(Ws& w, const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier, uint64_t end_time,
               uint64_t bootstrap_end, const PartGeo& g, uint8_t* d_status, unsigned long long* counters,
               hipStream_t s) {
    unsigned long long* const ucounters = counters; // (the caller's)
    uint32_t* gcnt = w.cnt1;
    uint32_t* wcnt = w.cnt1 + g.nb;
    if (!w.minw2) {
        if (int rc = hip_status(hipMalloc((void**)&w.minw2, 16), "hipMalloc ws.minw")) return rc;
        w.clean_now = false;
    }
    // the round's resets: none when the last synchronous round on this
    // workspace left them done (its final kernel clears them: one launch and
    // its gap less per round, ws_sync); SHD_ROUND_PRECLEAN=0: always here
    const char* pcv = getenv("SHD_ROUND_PRECLEAN");
    const bool pre_ok = !(pcv && strcmp(pcv, "0") == 0);
    if (!(pre_ok && w.clean_now && w.pre_m >= 3 * (size_t)g.nb))
        hipLaunchKernelGGL(k_round_init, dim3(grid_for(3 * g.nb, 256, 4096)), dim3(256), 0, s, w.nbig, counters,
                           w.cnt1, 3 * g.nb, w.minw2);
    w.clean_now = false;
    w.pre_req = pre_ok ? 3 * (size_t)g.nb : 0;
    // (the scatters' minimum goes to the workspace word minw2[1]: they take
    // minw2 as their counters; k_wide_group hands it to the caller's)
    counters = w.minw2;
    mark(0, s);
    if (n) {
        const PartCfg f = part_cfg(g.nb);
        // records per workgroup: at most f.ch, spread so that the grid is a
        // whole number of waves of one workgroup per CU (no last, partly
        // filled wave of workgroups: 10M records = 2,560 x 3,907, not
        // 2,442 x 4,096 on 256 CUs); SHD_PART_EVEN=0: f.ch each
        uint32_t ch = (uint32_t)f.ch;
        const char* ev = getenv("SHD_PART_EVEN");
        const size_t ncu = (size_t)dev_cus();
        if (f.pipe) {
            // persistent: f.pipe workgroups per CU, each the same number of
            // chunks of at most f.ch records
            // (SHD_PART_PIPE_GRID: another workgroup count -- tests walk many
            // chunks per workgroup on small batches with it)
            const char* pg = getenv("SHD_PART_PIPE_GRID");
            const size_t nwg = pg && atoi(pg) > 0 ? (size_t)atoi(pg) : ncu * (size_t)f.pipe,
                         iters = (n + nwg * f.ch - 1) / (nwg * f.ch);
            ch = (uint32_t)((n + nwg * iters - 1) / (nwg * iters));
        } else if (!(ev && strcmp(ev, "0") == 0)) {
            const size_t waves = (n + ncu * f.ch - 1) / (ncu * f.ch);
            ch = (uint32_t)((n + ncu * waves - 1) / (ncu * waves));
        }
        const dim3 grid((unsigned)((n + ch - 1) / ch)), blk(f.wg);
        const size_t lds = part_lds(f, g.nb);
        if (f.split) {
            // (dec: w.st1, free until the sort's listed segments)
            uint4* dec = reinterpret_cast<uint4*>(w.st1);
            if (f.split == 4)
                hipLaunchKernelGGL((k_part_decide<256, 4>), dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, s, *c,
                                   d_recs, n, barrier, end_time, bootstrap_end, g, dec, wcnt, d_status, counters, w.st2,
                                   w.nbig + 1);
            else
                hipLaunchKernelGGL((k_part_decide<256, 2>), dim3((unsigned)((n + 511) / 512)), dim3(256), 0, s, *c,
                                   d_recs, n, barrier, end_time, bootstrap_end, g, dec, wcnt, d_status, counters, w.st2,
                                   w.nbig + 1);
            hipLaunchKernelGGL((k_part_place<1024, 4096>), grid, blk, lds, s, dec, n, c->idx_base, g, w.pstage, gcnt, wcnt,
                               w.st2, w.nbig + 1, ch);
        } else if (f.pipe) {
            const char* pg = getenv("SHD_PART_PIPE_GRID");
            const unsigned nch = grid.x,
                           nwg = pg && atoi(pg) > 0 ? (unsigned)atoi(pg) : (unsigned)ncu * (unsigned)f.pipe,
                           ng = nch < nwg ? nch : nwg;
#define SHD_PIPE_LAUNCH(WG, CH)                                                                                       \
    hipLaunchKernelGGL((k_part_scatter_pipe<WG, CH>), dim3(ng), blk, lds, s, *c, d_recs, n, barrier, end_time,         \
                       bootstrap_end, g, w.pstage, gcnt, wcnt, d_status, counters, w.st2, w.nbig + 1, ch, nch)
            if (f.wg == 1024) SHD_PIPE_LAUNCH(1024, 2048);
            else if (f.wg == 512) SHD_PIPE_LAUNCH(512, 1024);
            else SHD_PIPE_LAUNCH(256, 512);
#undef SHD_PIPE_LAUNCH
        } else {
#define SHD_PART_LAUNCH(WG, CH, L, ...)                                                                             \
    hipLaunchKernelGGL((k_part_scatter<WG, CH, L, ##__VA_ARGS__>), grid, blk, lds, s, *c, d_recs, n, barrier, end_time, \
                       bootstrap_end, g, w.pstage, gcnt, wcnt, d_status, counters, w.st2, w.nbig + 1, ch)
        const int pr = part_probe();
        if (pr && !f.lds && f.wg == 1024) {
            if (pr == 1) SHD_PART_LAUNCH(1024, 4096, false, 1);
            else if (pr == 2) SHD_PART_LAUNCH(1024, 4096, false, 2);
            else if (pr == 4) SHD_PART_LAUNCH(1024, 4096, false, 4);
            else if (pr == 8) SHD_PART_LAUNCH(1024, 4096, false, 8);
            else if (pr == 6) SHD_PART_LAUNCH(1024, 4096, false, 6);
            else if (pr == 5) SHD_PART_LAUNCH(1024, 4096, false, 5);
            else if (pr == 7) SHD_PART_LAUNCH(1024, 4096, false, 7);
            else SHD_PART_LAUNCH(1024, 4096, false, 15);
        } else if (f.lds) SHD_PART_LAUNCH(1024, 4096, true);
        else if (f.fn == (const void*)k_part_scatter<1024, 4096, false, 0, 8>) SHD_PART_LAUNCH(1024, 4096, false, 0, 8);
        else if (f.wg == 1024 && f.ch == 8192) SHD_PART_LAUNCH(1024, 8192, false);
        else if (f.wg == 1024 && f.ch == 16384) SHD_PART_LAUNCH(1024, 16384, false);
        else if (f.wg == 1024) SHD_PART_LAUNCH(1024, 4096, false);
        else if (f.wg == 512 && f.ch == 4096) SHD_PART_LAUNCH(512, 4096, false);
        else if (f.wg == 512) SHD_PART_LAUNCH(512, 2048, false);
        else SHD_PART_LAUNCH(256, 2048, false);
        }
#undef SHD_PART_LAUNCH
        // the wide list by bucket (w.tmp: unused by this pipeline), for the
        // second pass to read its buckets' own
    }
    // (also with no records: it writes the sort's bucket bases)
    hipLaunchKernelGGL(k_wide_group, dim3(64), dim3(1024), 4 * (size_t)g.nb, s, g, w.st2, w.nbig + 1, (uint32_t)w.cap_n,
                       gcnt, wcnt, w.cnt1 + 2 * g.nb, w.tmp, ucounters, w.minw2);
    mark(1, s);
    mark_same(2, 1);
    int rc = hip_status(hipGetLastError(), "k_part_scatter launch");
    return rc ? rc : dbg_sync(s, "k_part_scatter");
}

int part_round(Ws& w, const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier, uint64_t end_time,
               uint64_t bootstrap_end, const PartGeo& g, ShdDeliv* d_out, uint32_t* d_dst_offsets, uint8_t* d_status,
               uint64_t* d_counters, hipStream_t s) {
    int rc;
    if ((rc = part_attr()) || (rc = ws_begin(w, s)) || (rc = ws_reserve(w, n, part_cnt_words(g.nb), g.H)) ||
        (rc = pstage_reserve(w, (size_t)g.nb * g.cap)))
        return rc;
    unsigned long long* counters = (unsigned long long*)d_counters;
    uint32_t* gcnt = w.cnt1;
    uint32_t* wcnt = w.cnt1 + g.nb;
    if ((rc = dbg_ranges(w, d_status, n, d_out, d_dst_offsets, g.H))) return rc;
    if ((rc = part_front(w, c, d_recs, n, barrier, end_time, bootstrap_end, g, d_status, counters, s))) return rc;
    mark_same(3, 2);
    {
        const int sc = part_sort_cfg();
#define SHD_PART_SORT_LAUNCH(WG, CAP, ...)                                                                            \
    hipLaunchKernelGGL((k_part_sort<WG, CAP, ##__VA_ARGS__>), dim3(g.nb), dim3(WG), 0, s, g, w.pstage, gcnt, wcnt, w.tmp, w.nbig + 1, \
                       (uint32_t)w.cap_n, d_dst_offsets, d_out, w.st1, w.big, w.nbig, counters, part_sort_flags())
        if (sc == 1) SHD_PART_SORT_LAUNCH(512, 3584);
        else if (sc == 2) SHD_PART_SORT_LAUNCH(256, 1792);
        else if (sc == 3) SHD_PART_SORT_LAUNCH(512, 2304, 2, false, 6);
        else if (sc == 4)
            hipLaunchKernelGGL((k_part_sort_occ<512, 2304, 0, 8>), dim3(g.nb), dim3(512), 0, s, g, w.pstage, gcnt, wcnt,
                               w.tmp, w.nbig + 1, (uint32_t)w.cap_n, d_dst_offsets, d_out, w.st1, w.big, w.nbig, counters,
                               part_sort_flags());
        else SHD_PART_SORT_LAUNCH(1024, 7168);
#undef SHD_PART_SORT_LAUNCH
    }
    if ((rc = hip_status(hipGetLastError(), "k_part_sort launch")) || (rc = dbg_sync(s, "k_part_sort"))) return rc;
    if ((rc = sort_listed(w, w.st1, d_dst_offsets, d_out, s, counters)) || (rc = dbg_sync(s, "listed segments")))
        return rc;
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    return ws_end(w, s);
}

extern "C" int shd_dev_packet_round(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                                    uint64_t end_time, uint64_t bootstrap_end, ShdDeliv* d_out,
                                    uint32_t* d_dst_offsets, uint8_t* d_status, uint64_t* d_counters, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (!c->ws) return shd_fail(-ENOMEM, "no round workspace");
    Ws& w = *static_cast<Ws*>(c->ws);
    const uint32_t H = c->nhosts;
    int pipe = pipeline_for(H, true, true);
    if (pipe == kPartPipe) {
        PartGeo g;
        if (part_geometry(0, H, n, barrier > (1ull << 31) ? barrier - (1ull << 31) : 0ull, &g, barrier)) {
            w.fin_ask = stream == nullptr; // (waited for below: its merge kernel may end it)
            int rc = part_round(w, c, d_recs, n, barrier, end_time, bootstrap_end, g, d_out, d_dst_offsets, d_status,
                                d_counters, s);
            w.fin_ask = false;
            if (rc) w.fin_done = false;
            if (rc || stream) return rc;
            return ws_sync(w, s, "packet round");
        }
        pipe = pipeline_for(H, true); // (buckets too many for the scatter's histogram: the slab form)
    }
    const bool rk = pipe != kBucketPipe;
    Bucketing bk;
    int rc = make_bucketing(0, H, n, &bk);
    if (rc) return rc;
    const size_t m = rk ? (size_t)H : (size_t)bk.nb * bk.ntiles;
    if ((rc = ws_begin(w, s))) return rc;
    if ((rc = ws_reserve(w, n, m, H))) return rc;
    if (pipe == kSlabPipe && (rc = slab_reserve(w, H))) return rc;
    const bool compact = pipe == kSlabPipe && compact_slab();
    if (compact && (rc = cslab_reserve(w, H))) return rc;
    uint4* cs = compact ? w.cslab : nullptr;
    bk.tbase = barrier > (1ull << 31) ? barrier - (1ull << 31) : 0ull;
    unsigned long long* counters = (unsigned long long*)d_counters;
    if ((rc = dbg_ranges(w, d_status, n, d_out, d_dst_offsets, H))) return rc;
    // rank: per-destination counters start at zero; bucket: every tile writes
    // its whole histogram column, only an empty batch needs zeros.  One
    // launch for the three resets (three memsets cost two more kernel
    // boundaries per round: round 0.807-0.811 vs 0.811-0.813 ms in one
    // process, profiles/r03init_round_init.log).
    {
        const uint32_t mz = (rk || !n) ? (uint32_t)m : 0u;
        hipLaunchKernelGGL(k_round_init, dim3(grid_for(mz ? mz : 1, 256, 4096)), dim3(256), 0, s, w.nbig, counters,
                           w.cnt1, mz);
        if ((rc = hip_status(hipGetLastError(), "k_round_init launch"))) return rc;
    }
    mark(0, s);
    if (n) {
        const char* sb = getenv("SHD_SCATTER_BATCH");
        const char* pr = getenv("SHD_SCATTER_PROBE");
        const int probe = pr ? atoi(pr) : 0;
        const char* ntv = getenv("SHD_SCATTER_NT");
        const int nt = ntv ? atoi(ntv) : 1;
#define SHD_PROBE_LAUNCH(P)                                                                                        \
    hipLaunchKernelGGL((k_pkt_scatter<2, kBatch, P>), dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier, \
                       end_time, bootstrap_end, bk, w.slab, d_status, w.cnt1, counters, w.st2, w.nbig + 1, cs)
        if (pipe == kSlabPipe && probe == 1) SHD_PROBE_LAUNCH(1);
        else if (pipe == kSlabPipe && probe == 2) SHD_PROBE_LAUNCH(2);
        else if (pipe == kSlabPipe && probe == 3) SHD_PROBE_LAUNCH(3);
        else if (pipe == kSlabPipe && probe == 4) SHD_PROBE_LAUNCH(4);
#undef SHD_PROBE_LAUNCH
        else if (pipe == kSlabPipe && nt == 0)
            hipLaunchKernelGGL((k_pkt_scatter<2, kBatch, 0, false>), dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n,
                               barrier, end_time, bootstrap_end, bk, w.slab, d_status, w.cnt1, counters, w.st2,
                               w.nbig + 1, cs);
else if (pipe == kSlabPipe && sb && strcmp(sb, "8") == 0)
            hipLaunchKernelGGL((k_pkt_scatter<2, 8>), dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier,
                               end_time, bootstrap_end, bk, w.slab, d_status, w.cnt1, counters, w.st2,
                               w.nbig + 1, cs);
        else if (pipe == kSlabPipe && sb && strcmp(sb, "2") == 0)
            hipLaunchKernelGGL((k_pkt_scatter<2, 2>), dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier,
                               end_time, bootstrap_end, bk, w.slab, d_status, w.cnt1, counters, w.st2,
                               w.nbig + 1, cs);
        else if (pipe == kSlabPipe)
            hipLaunchKernelGGL(k_pkt_scatter<2>, dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier,
                               end_time, bootstrap_end, bk, w.slab, d_status, w.cnt1, counters, w.st2,
                               w.nbig + 1, cs);
        else if (rk)
            hipLaunchKernelGGL(k_pkt_scatter<1>, dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier,
                               end_time, bootstrap_end, bk, w.tmp, d_status, w.cnt1, counters, nullptr,
                               nullptr, nullptr);
        else
            hipLaunchKernelGGL(k_pkt_scatter<0>, dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier,
                               end_time, bootstrap_end, bk, w.tmp, d_status, w.cnt1, counters, nullptr,
                               nullptr, nullptr);
    }
    mark(1, s);
    if ((rc = hip_status(hipGetLastError(), "k_pkt_scatter launch"))) return rc;
    if ((rc = dbg_sync(s, "memsets + k_pkt_scatter"))) return rc;
    rc = pipe == kSlabPipe
             ? group_and_sort_rank(w, w.tmp, d_status, nullptr, n, 0, H, d_out, d_dst_offsets, counters, s, w.slab,
                                   bk.slab_rm, cs, bk.tbase)
         : rk ? group_and_sort_rank(w, w.tmp, d_status, nullptr, n, 0, H, d_out, d_dst_offsets, counters, s)
              : group_and_sort(w, w.tmp, d_status, nullptr, n, bk, d_out, d_dst_offsets, counters, s);
    if (!rc) rc = ws_end(w, s);
    if (rc) return rc;
    if (stream) return 0;
    return ws_sync(w, s, "packet round");
}

// Which grouping pipeline a round of n records over nhosts destinations runs
// (0 bucket, 1 rank, 2 slab, 3 part), for tooling and benchmarks.
extern "C" int shd_round_pipeline_of(uint32_t nhosts, size_t n, int* pipe) {
    if (!pipe) return -EINVAL;
    int p = pipeline_for(nhosts, true, true);
    PartGeo g;
    if (p == kPartPipe && !part_geometry(0, nhosts, n, 0, &g, 0)) p = pipeline_for(nhosts, true);
    *pipe = p;
    return 0;
}

extern "C" int shd_round_timing_enable(int enable) {
    if (enable && !g_tm.created) {
        for (int i = 0; i < kMaxTimed; i++)
            for (int k = 0; k <= kStages; k++)
                if (hipEventCreate(&g_tm.ev[i][k]) != hipSuccess) return shd_fail(-EIO, "hipEventCreate");
        g_tm.created = true;
    }
    g_tm.on = g_tm.enabled = enable != 0;
    g_tm.n = 0;
    return 0;
}

extern "C" int shd_round_timing_pause(int paused) {
    g_tm.on = g_tm.enabled && paused == 0;
    return 0;
}

extern "C" int shd_round_timing_read(double* stage_ms, int nstages, int* launches) {
    if (nstages > kStages) nstages = kStages;
    for (int k = 0; k < nstages; k++) stage_ms[k] = 0.0;
    for (int i = 0; i < g_tm.n; i++) {
        if (hipEventSynchronize(g_tm.ev[i][kStages]) != hipSuccess) return shd_fail(-EIO, "hipEventSynchronize");
        for (int k = 0; k < nstages; k++) {
            float ms = 0.f;
            const int a = g_tm.at[i][k], b = g_tm.at[i][k + 1];
            if (a != b && hipEventElapsedTime(&ms, g_tm.ev[i][a], g_tm.ev[i][b]) != hipSuccess)
                return shd_fail(-EIO, "hipEventElapsedTime");
            stage_ms[k] += ms;
        }
    }
    if (launches) *launches = g_tm.n;
    return 0;
}

extern "C" int shd_dev_deliv_sort(void* ws, const ShdDeliv* d_in, size_t n, uint32_t host_lo, uint32_t host_hi,
                                  ShdDeliv* d_out, uint32_t* d_dst_offsets, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (!ws) return shd_fail(-ENOMEM, "no round workspace");
    Ws& w = *static_cast<Ws*>(ws);
    const uint32_t H = host_hi - host_lo;
    const int pipe = pipeline_for(H, true);
    const bool rk = pipe != kBucketPipe;
    Bucketing bk;
    int rc = make_bucketing(host_lo, H, n, &bk);
    if (rc) return rc;
    const size_t m = rk ? (size_t)H : (size_t)bk.nb * bk.ntiles;
    if ((rc = ws_begin(w, s))) return rc;
    if ((rc = ws_reserve(w, n, m, H))) return rc;
    if (pipe == kSlabPipe && (rc = slab_reserve(w, H))) return rc;
    if ((rc = dbg_ranges(w, nullptr, 0, d_out, d_dst_offsets, H))) return rc;
    if ((rc = hip_status(hipMemsetAsync(w.nbig, 0, 12, s), "memset nbig"))) return rc;
    if ((rk || !n) && (rc = hip_status(hipMemsetAsync(w.cnt1, 0, 4 * m, s), "memset cnt1"))) return rc;
    mark(0, s);
    if (n) {
        if (pipe == kSlabPipe)
            hipLaunchKernelGGL(k_hist_slab, dim3(grid_for(n, 256 * kBatch, 1u << 20)), dim3(256), 0, s, d_in, n,
                               host_lo, H, w.cnt1, w.slab, bk.slab_rm, w.st2, w.nbig + 1, bk.agg);
        else if (rk)
            hipLaunchKernelGGL(k_hist_rank, dim3(grid_for(n, 256, 1u << 20)), dim3(256), 0, s, d_in, n, host_lo, H,
                               w.cnt1, w.rnk, bk.agg);
        else
            hipLaunchKernelGGL(k_hist_tiles, dim3(bk.ntiles), dim3(kBlock), 0, s, d_in, n, bk, w.cnt1, w.rnk);
    }
    mark(1, s);
    rc = pipe == kSlabPipe
             ? group_and_sort_rank(w, d_in, nullptr, w.rnk, n, host_lo, H, d_out, d_dst_offsets, nullptr, s, w.slab,
                                   bk.slab_rm)
         : rk ? group_and_sort_rank(w, d_in, nullptr, w.rnk, n, host_lo, H, d_out, d_dst_offsets, nullptr, s)
              : group_and_sort(w, d_in, nullptr, w.rnk, n, bk, d_out, d_dst_offsets, nullptr, s);
    if (!rc) rc = ws_end(w, s);
    if (rc) return rc;
    if (stream) return 0;
    return ws_sync(w, s, "deliv sort");
}

// Regroup of the exchange's W received blocks (see k_runs_count): d_in holds
// the n events of the blocks back to back (block k from d_bbase[k], a device
// array of W + 1 prefix counts), d_rofs the W per-block offset arrays over
// the host range [host_lo, host_hi).  Output as shd_dev_deliv_sort.
extern "C" int shd_dev_deliv_merge_runs_self(void* ws, const void* d_in, const void* d_self, uint32_t self, int wire,
                                             int sorted, size_t n, const uint32_t* d_rofs, const uint32_t* d_bbase,
                                             uint32_t W, uint32_t host_lo, uint32_t host_hi, ShdDeliv* d_out,
                                             uint32_t* d_dst_offsets, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (!ws) return shd_fail(-ENOMEM, "no round workspace");
    if (W < 1 || W > kMaxRuns) return shd_fail(-EINVAL, "%u runs outside 1..%u", W, kMaxRuns);
    Ws& w = *static_cast<Ws*>(ws);
    const uint32_t H = host_hi - host_lo;
    int rc;
    if ((rc = ws_begin(w, s))) return rc;
    if ((rc = ws_reserve(w, n, H, H))) return rc; // (st1: staging of the listed segments)
    if ((rc = dbg_ranges(w, nullptr, 0, d_out, d_dst_offsets, H))) return rc;
    if ((rc = hip_status(hipMemsetAsync(w.nbig, 0, 12, s), "memset nbig"))) return rc;
    hipLaunchKernelGGL(k_runs_count, dim3(grid_for(H, 256, 4096)), dim3(256), 0, s, d_rofs, W, H, w.cnt1);
    scan_counts(w.cnt1, (size_t)H, d_dst_offsets, w.bsum, nullptr, s);
    if (!d_self) self = 0xffffffffu;
    if (sorted) { // (every run sorted: merge by binary searches)
        const unsigned g = grid_for(H, 1, 8192), gw = grid_for(H, 4, 16384);
        const char* mp = getenv("SHD_MERGE_PROBE"); // (measurement only)
        const uint32_t mprobe = mp ? (uint32_t)atoi(mp) : 0u;
        if (wire) {
            hipLaunchKernelGGL(k_runs_merge_wave<1>, dim3(gw), dim3(256), 0, s, d_in, d_self, self, d_rofs, d_bbase, W,
                               H, d_dst_offsets, host_lo, d_out);
            hipLaunchKernelGGL(k_runs_merge<1>, dim3(g), dim3(kMergeThreads), 0, s, d_in, d_self, self, d_rofs, d_bbase, W, H,
                               d_dst_offsets, host_lo, d_out, w.st1, w.big, w.nbig, mprobe);
        } else {
            hipLaunchKernelGGL(k_runs_merge_wave<0>, dim3(gw), dim3(256), 0, s, d_in, d_self, self, d_rofs, d_bbase, W,
                               H, d_dst_offsets, host_lo, d_out);
            hipLaunchKernelGGL(k_runs_merge<0>, dim3(g), dim3(kMergeThreads), 0, s, d_in, d_self, self, d_rofs, d_bbase, W, H,
                               d_dst_offsets, host_lo, d_out, w.st1, w.big, w.nbig, mprobe);
        }
    } else if (wire)
        hipLaunchKernelGGL(k_runs_sort<1>, dim3(grid_for(H, 4, 16384)), dim3(256), 0, s, d_in, d_self, self, d_rofs,
                           d_bbase, W, H, d_dst_offsets, host_lo, d_out, w.st1, w.big, w.nbig, lds_keys());
    else
        hipLaunchKernelGGL(k_runs_sort<0>, dim3(grid_for(H, 4, 16384)), dim3(256), 0, s, d_in, d_self, self, d_rofs,
                           d_bbase, W, H, d_dst_offsets, host_lo, d_out, w.st1, w.big, w.nbig, lds_keys());
    if ((rc = hip_status(hipGetLastError(), "k_runs_sort launch"))) return rc;
    if ((rc = dbg_sync(s, "k_runs_sort"))) return rc;
    if ((rc = sort_listed(w, w.st1, d_dst_offsets, d_out, s, nullptr))) return rc;
    if ((rc = ws_end(w, s))) return rc; // (not a timed round stage: shd_round_timing_* time the decide side)
    if (stream) return 0;
    return ws_sync(w, s, "merge runs");
}

extern "C" int shd_dev_deliv_merge_runs(void* ws, const void* d_in, int wire, int sorted, size_t n, const uint32_t* d_rofs,
                                        const uint32_t* d_bbase, uint32_t W, uint32_t host_lo, uint32_t host_hi,
                                        ShdDeliv* d_out, uint32_t* d_dst_offsets, void* stream) {
    return shd_dev_deliv_merge_runs_self(ws, d_in, nullptr, 0xffffffffu, wire, sorted, n, d_rofs, d_bbase, W, host_lo,
                                         host_hi, d_out, d_dst_offsets, stream);
}

// The part sender's bucket sorts for buckets [b_lo, b_hi): sort_wire -- every
// destination's run goes out sorted (the part sort writing wire records;
// listed segments sorted later by the listed kernels, grouped_finish), so
// the owners merge sorted runs; else unsorted runs (k_part_wire), the owners
// sort their union.
int grouped_sorts(Ws& w, PartGeo pg, void* d_wire, uint32_t* d_off, unsigned long long* counters, hipStream_t s,
                  bool wsorted, uint32_t b_lo, uint32_t b_hi) {
    if (b_hi <= b_lo) return 0;
    pg.b0 = b_lo;
    const dim3 grid(b_hi - b_lo);
    if (wsorted) {
        ShdDeliv* wout = static_cast<ShdDeliv*>(d_wire); // (a Wire array: kWire)
        const int sc = part_sort_cfg();
#define SHD_WIRE_SORT_LAUNCH(WG, CAP, KE, ...)                                                                        \
    hipLaunchKernelGGL((k_part_sort<WG, CAP, KE, true, ##__VA_ARGS__>), grid, dim3(WG), 0, s, pg, w.pstage, w.cnt1,   \
                       w.cnt1 + pg.nb, w.tmp, w.nbig + 1, (uint32_t)w.cap_n, d_off, wout, w.st1, w.big, w.nbig, counters, \
                       part_sort_flags())
        if (sc == 0) SHD_WIRE_SORT_LAUNCH(1024, 7168, 4);
        else if (sc == 1) SHD_WIRE_SORT_LAUNCH(512, 3584, 4);
        else if (sc == 2) SHD_WIRE_SORT_LAUNCH(256, 1792, 4);
        else SHD_WIRE_SORT_LAUNCH(512, 2304, 2, 6);
#undef SHD_WIRE_SORT_LAUNCH
        return hip_status(hipGetLastError(), "k_part_sort (wire) launch");
    }
    hipLaunchKernelGGL((k_part_wire<512, 5>), grid, dim3(512), 0, s, pg, w.pstage, w.cnt1, w.cnt1 + pg.nb, w.tmp,
                       w.nbig + 1, (uint32_t)w.cap_n, d_off, static_cast<Wire*>(d_wire), counters, w.nbig + 2);
    return hip_status(hipGetLastError(), "k_part_wire launch");
}

// ... and what follows the sorts: the listed segments (sorted into w.st2 --
// the wide list's first copy, free by then -- and converted to wire records)
// and the round's fault word.  (ws_end is the caller's.)
int grouped_finish(Ws& w, const PartGeo& pg, void* d_wire, uint32_t* d_off, unsigned long long* counters,
                   hipStream_t s, bool wsorted) {
    int rc;
    if (wsorted) {
        if ((rc = sort_listed(w, w.st1, d_off, w.st2, s, counters))) return rc;
        hipLaunchKernelGGL(k_listed_wire, dim3(1024), dim3(256), 0, s, w.st2, d_off, w.big, w.nbig,
                           merge_meta(w, counters).cap_big, static_cast<Wire*>(d_wire));
        if ((rc = hip_status(hipGetLastError(), "k_listed_wire launch"))) return rc;
    }
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    if ((rc = dbg_sync(s, "grouped part round"))) return rc;
    hipLaunchKernelGGL(k_fault_word, dim3(1), dim3(64), 0, s, w.nbig, merge_meta(w, counters));
    return copy_faults(w, s);
}

// The sender's side of shd_round_process_exchange: the slab round up to the
// per-destination offsets (d_off, H + 1), then the grouped, unsorted wire
// records (k_group_wire) instead of the segment sort.  Slab pipeline only.
extern "C" int shd_dev_packet_round_grouped(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                                            uint64_t end_time, uint64_t bootstrap_end, void* d_wire, uint32_t* d_off,
                                            uint8_t* d_status, uint64_t* d_counters, void* stream, int sort_wire,
                                            int* sorted_out) {
    hipStream_t s = (hipStream_t)stream;
    if (sorted_out) *sorted_out = 0;
    if (!c->ws) return shd_fail(-ENOMEM, "no round workspace");
    Ws& w = *static_cast<Ws*>(c->ws);
    const uint32_t H = c->nhosts;
    const unsigned long long tb = barrier > (1ull << 31) ? barrier - (1ull << 31) : 0ull;
    PartGeo pg;
    if (pipeline_for(H, true, true) == kPartPipe && part_geometry(0, H, n, tb, &pg, barrier)) {
        // the part scatter, then the bucket's events grouped by destination
        // straight into the wire array (k_part_wire)
        unsigned long long* counters = (unsigned long long*)d_counters;
        int rc;
        if ((rc = part_attr()) || (rc = ws_begin(w, s)) || (rc = ws_reserve(w, n, part_cnt_words(pg.nb), H)) ||
            (rc = pstage_reserve(w, (size_t)pg.nb * pg.cap)) ||
            (rc = part_front(w, c, d_recs, n, barrier, end_time, bootstrap_end, pg, d_status, counters, s)))
            return rc;
        mark_same(3, 2);
        const bool wsorted = sort_wire != 0;
        if ((rc = grouped_sorts(w, pg, d_wire, d_off, counters, s, wsorted, 0, pg.nb)) ||
            (rc = grouped_finish(w, pg, d_wire, d_off, counters, s, wsorted)))
            return rc;
        if (sorted_out) *sorted_out = wsorted ? 1 : 0;
        return ws_end(w, s);
    }
    const int pipe = pipeline_for(H, true);
    if (pipe == kBucketPipe || pipe == kRankPipe) return shd_fail(-ENOTSUP, "the exchanged round needs the slab pipeline");
    Bucketing bk;
    int rc = make_bucketing(0, H, n, &bk);
    if (rc) return rc;
    if ((rc = ws_begin(w, s))) return rc;
    if ((rc = ws_reserve(w, n, H, H)) || (rc = slab_reserve(w, H))) return rc;
    const bool compact = compact_slab();
    if (compact && (rc = cslab_reserve(w, H))) return rc;
    uint4* cs = compact ? w.cslab : nullptr;
    bk.tbase = barrier > (1ull << 31) ? barrier - (1ull << 31) : 0ull;
    unsigned long long* counters = (unsigned long long*)d_counters;
    if ((rc = hip_status(hipMemsetAsync(w.nbig, 0, 12, s), "memset nbig")) ||
        (rc = hip_status(hipMemsetAsync(counters, 0xff, 16, s), "memset counters")) ||
        (rc = hip_status(hipMemsetAsync(w.cnt1, 0, 4 * (size_t)H, s), "memset cnt1")))
        return rc;
    mark(0, s);
    if (n)
        hipLaunchKernelGGL(k_pkt_scatter<2>, dim3(bk.ntiles), dim3(kBlock), 0, s, *c, d_recs, n, barrier, end_time,
                           bootstrap_end, bk, w.slab, d_status, w.cnt1, counters, w.st2, w.nbig + 1, cs);
    mark(1, s);
    if ((rc = hip_status(hipGetLastError(), "k_pkt_scatter launch"))) return rc;
    scan_counts(w.cnt1, (size_t)H, d_off, w.bsum, counters, s);
    mark(2, s);
    mark(3, s);
    hipLaunchKernelGGL(k_group_wire, dim3(grid_for(H, 4, 16384)), dim3(256), 0, s, w.slab, bk.slab_rm, H, d_off, w.st2,
                       w.nbig, w.nbig + 2, (uint32_t)w.cap_n, static_cast<Wire*>(d_wire), cs, bk.tbase);
    if ((rc = hip_status(hipGetLastError(), "k_group_wire launch"))) return rc;
    mark(4, s);
    if (g_tm.on && g_tm.n < kMaxTimed) g_tm.n++;
    if ((rc = dbg_sync(s, "grouped round"))) return rc;
    // the guard bits of this round (nbig[2]) go to the fault word the host
    // reads back (no merge kernel runs on the sender's side)
    hipLaunchKernelGGL(k_fault_word, dim3(1), dim3(64), 0, s, w.nbig, merge_meta(w, counters));
    if ((rc = copy_faults(w, s))) return rc;
    return ws_end(w, s);
}

// shd_dev_packet_round_grouped in two halves (see ShdSplitHooks): the cuts
// from the partition, the front hook, the buckets of the owners below
// bounds[half] (through the bucket holding bounds[half]: the cut there is
// then written by this half too), the listed-segment count so far, the mid
// hook, the other buckets and the listed segments.
extern "C" int shd_dev_packet_round_grouped_split(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n,
                                                  uint64_t barrier, uint64_t end_time, uint64_t bootstrap_end,
                                                  void* d_wire, uint32_t* d_off, uint8_t* d_status,
                                                  uint64_t* d_counters, void* stream, int sort_wire,
                                                  const uint32_t* bounds, int W, int half, uint32_t* d_cuts,
                                                  uint32_t* d_listed_a, const ShdSplitHooks* hooks) {
    hipStream_t s = (hipStream_t)stream;
    if (!c->ws) return shd_fail(-ENOMEM, "no round workspace");
    if (W < 1 || W > 64 || half < 0 || half > W) return shd_fail(-EINVAL, "bad split");
    Ws& w = *static_cast<Ws*>(c->ws);
    const uint32_t H = c->nhosts;
    const unsigned long long tb = barrier > (1ull << 31) ? barrier - (1ull << 31) : 0ull;
    CutArgs ca;
    ca.W = W;
    for (int r = 0; r <= W; r++) ca.b[r] = bounds[r];
    int rc;
    PartGeo pg;
    if (!(pipeline_for(H, true, true) == kPartPipe && part_geometry(0, H, n, tb, &pg, barrier))) {
        // the slab sender: the whole round, then its cuts and both hooks
        int sorted = 0;
        if ((rc = shd_dev_packet_round_grouped(c, d_recs, n, barrier, end_time, bootstrap_end, d_wire, d_off, d_status,
                                               d_counters, stream, sort_wire, &sorted)))
            return rc;
        hipLaunchKernelGGL(k_gather_cuts, dim3(1), dim3(128), 0, s, d_off, ca, d_cuts);
        if ((rc = hip_status(hipGetLastError(), "cuts launch")) ||
            (rc = hip_status(hipMemsetAsync(d_listed_a, 0, 4, s), "memset listed")) ||
            (rc = hooks->front(hooks->user, d_cuts, sorted)))
            return rc;
        return hooks->mid(hooks->user);
    }
    unsigned long long* counters = (unsigned long long*)d_counters;
    if ((rc = part_attr()) || (rc = ws_begin(w, s)) || (rc = ws_reserve(w, n, part_cnt_words(pg.nb), H)) ||
        (rc = pstage_reserve(w, (size_t)pg.nb * pg.cap)) ||
        (rc = part_front(w, c, d_recs, n, barrier, end_time, bootstrap_end, pg, d_status, counters, s)))
        return rc;
    mark_same(3, 2);
    const bool wsorted = sort_wire != 0;
    hipLaunchKernelGGL(k_part_cuts, dim3(W + 1), dim3(256), 0, s, pg, w.pstage, w.cnt1, w.cnt1 + pg.nb, w.tmp,
                       w.nbig + 1, (uint32_t)w.cap_n, ca, d_cuts);
    if ((rc = hip_status(hipGetLastError(), "k_part_cuts launch")) ||
        (rc = hooks->front(hooks->user, d_cuts, wsorted ? 1 : 0)))
        return rc;
    const uint32_t hb = bounds[half];
    const uint32_t b_a = hb >= H ? pg.nb : ((hb >> pg.shift) + 1 < pg.nb ? (hb >> pg.shift) + 1 : pg.nb);
    if ((rc = grouped_sorts(w, pg, d_wire, d_off, counters, s, wsorted, 0, b_a)) ||
        (rc = hip_status(hipMemcpyAsync(d_listed_a, w.nbig, 4, hipMemcpyDeviceToDevice, s), "listed count")) ||
        (rc = hooks->mid(hooks->user)) ||
        (rc = grouped_sorts(w, pg, d_wire, d_off, counters, s, wsorted, b_a, pg.nb)) ||
        (rc = grouped_finish(w, pg, d_wire, d_off, counters, s, wsorted)))
        return rc;
    return ws_end(w, s);
}
