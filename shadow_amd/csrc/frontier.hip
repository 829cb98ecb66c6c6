// frontier.hip -- latency rows by a bucketed frontier SSSP (Dial's algorithm):
// north_star's frontier SSSP for sparse graphs, whole-ms latencies.
//
// As for the min-plus kernel (minplus.hip), the latencies are shortest-path
// distances, independent of which equal-latency path igraph's heap picks, so
// any exact SSSP reproduces them; with every edge latency a whole number of
// ms (ShdGraphDev.sl) every distance is an exact u32 and equals the f64 sum
// the reference forms.  Entries are then formed as
// _topology_computeSourcePaths stores them (topology.c:1744-1791): latency 0
// -> 1 ms, unreachable -1, the self path by _topology_computeShortestPathToSelf
// (topology.c:1431-1576).  The reliabilities need igraph's pop order (DESIGN.md
// §4.1) and stay with the heap kernels.
//
// One wave per source row (persistent waves, rows strided).  Edge latencies
// are at least 1 ms and at most Wmax, so the frontier is a ring of Wmax + 1
// distance buckets (Dial): bucket cur holds the vertices whose tentative
// distance is cur, settled when it is reached; relaxing their edges only
// pushes into the next Wmax buckets, never into cur.  A bucket is a list of
// 64-entry chunks (one entry per lane) from the wave's chunk pool, its head,
// tail and tail fill in LDS; popped chunks return to a free stack.  A chunk
// of up to 64 vertices is relaxed edge-parallel: the wave scans their
// degrees, then takes their edges 64 at a time (each lane finds its vertex by
// a binary search over the scanned offsets in LDS), gathers the neighbours'
// distances and stores the improvements (lanes that improved the same
// neighbour in one batch settle on the minimum by store-and-reread).  A
// vertex is pushed once per strict improvement; entries whose vertex has
// improved since are skipped when popped.  Per wave in HBM: the distances
// (4 B per vertex) and the chunk pool.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <new>

#include "shd_internal.h"

namespace {

constexpr uint32_t kInf = 0xffffffffu;
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kWaves = 4; // waves per workgroup

struct __attribute__((aligned(16))) Ent { // ShdGraphDev.sl entry
    int nbr;
    uint32_t w;
    double rel;
};

__device__ __forceinline__ void wave_sync_mem() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// per-wave LDS: head[nbk] | tail[nbk] | fill[nbk] | offs[64] | starts[64] | htab[64]
__host__ __device__ constexpr size_t dial_lds_words(int nbk) { return 3 * (size_t)nbk + 192; }
// the largest edge latency (ms) whose bucket ring fits the 160 KiB LDS (checked below)
constexpr int kFrontierMaxWms = 3348;
static_assert(dial_lds_words(kFrontierMaxWms + 1) * 4 * kWaves <= 160 * 1024, "ring fits the LDS");
static_assert(dial_lds_words(kFrontierMaxWms + 2) * 4 * kWaves > 160 * 1024, "the limit is the largest that fits");

// rows: rowlist[0 .. nrows) (or row_lo + i when rowlist is null); a row whose
// chunk pool ran out is appended to redo (for a second launch with the
// worst-case pool) and its output left unwritten
__global__ __launch_bounds__(64 * kWaves) void k_sssp_dial(ShdGraphDev g, int row_lo, const int* __restrict__ rowlist,
                                                          int nrows, int nbk, char* __restrict__ slab, size_t stride,
                                                          uint32_t nchunk, int Vp, double* __restrict__ lat,
                                                          int* __restrict__ redo, unsigned* __restrict__ nredo) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dsm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int gw = (int)blockIdx.x * kWaves + w, nw = (int)gridDim.x * kWaves;
    uint32_t* head = dsm + (size_t)w * dial_lds_words(nbk);
    uint32_t* tail = head + nbk;
    uint32_t* fill = tail + nbk;
    uint32_t* offs = fill + nbk;
    uint32_t* starts = offs + 64;
    uint32_t* htab = starts + 64;
    uint32_t* dist = reinterpret_cast<uint32_t*>(slab + (size_t)gw * stride);
    uint32_t* pool = dist + Vp;
    uint32_t* nxt = pool + (size_t)nchunk * 64;
    uint32_t* fstk = nxt + nchunk;
    const Ent* __restrict__ sl = static_cast<const Ent*>(g.sl);
    const int A = g.A;
    const uint32_t maxd = (uint32_t)min((unsigned long long)g.V * (unsigned long long)(nbk - 1), 0xFFFFFFFEull);
    for (int i = gw; i < nrows; i += nw) {
        const int row = rowlist ? rowlist[i] : row_lo + i;
        const int src = g.slot_vertex[row];
        for (int v = lane; v < Vp; v += 64) dist[v] = kInf;
        for (int b = lane; b < nbk; b += 64) head[b] = kNone, fill[b] = 0u;
        wave_sync_mem();
        uint32_t bump = 0, ftop = 0, fsafe = 0; // chunk allocation (wave-uniform); fsafe: free-stack
                                                // entries stored before the last fence
        bool failed = false;
        // the source: bucket 0
        bump = 1;
        if (lane == 0) {
            dist[src] = 0u;
            pool[0] = (uint32_t)src;
            head[0] = tail[0] = 0u;
            fill[0] = 1u;
        }
        wave_sync_mem();
        uint32_t pending = 1, cur = 0;
        while (pending > 0 && !failed) {
            const uint32_t b = cur % (uint32_t)nbk;
            uint32_t c = uni(head[b]);
            while (c != kNone && !failed) {
                const bool last = c == uni(tail[b]);
                const uint32_t n = last ? uni(fill[b]) : 64u;
                const uint32_t nx = last ? kNone : uni(nxt[c]);
                const int v = lane < (int)n ? (int)pool[(size_t)c * 64 + lane] : -1;
                if (lane == 0) {
                    fstk[ftop] = c;
                    if (last) head[b] = kNone, fill[b] = 0u;
                    else head[b] = nx;
                }
                ftop++;
                pending -= n;
                c = nx;
                // settled (stale entries: the vertex improved since it was
                // pushed); its distance and list bounds in one round trip
                uint32_t dv = kInf;
                int a0 = 0, a1 = 0;
                if (v >= 0) {
                    dv = dist[v];
                    a0 = g.inc_off[v];
                    a1 = g.inc_off[v + 1];
                }
                const bool live = v >= 0 && dv == cur;
                const uint32_t deg = live ? (uint32_t)(a1 - a0) : 0u;
                uint32_t incl = deg;
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
                    if (lane >= o) incl += y;
                }
                const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                offs[lane] = incl - deg;
                starts[lane] = (uint32_t)(a0 + v); // (sl: one sentinel per list before it)
                __asm__ volatile("" ::: "memory"); // (LDS: the wave's own accesses stay in order)
                // batch e0's entries (issued one batch ahead of their use)
                auto entry = [&](uint32_t e) {
                    Ent en{-1, 0u, 0.0};
                    if (e < T) {
                        int o = 0; // the last lane whose edges start at or before e
#pragma unroll
                        for (int s = 32; s > 0; s >>= 1)
                            if (offs[o + s] <= e) o += s;
                        en = sl[starts[o] + (e - offs[o])];
                    }
                    return en;
                };
                Ent en = entry((uint32_t)lane);
                for (uint32_t e0 = 0; e0 < T; e0 += 64) {
                    const Ent nx_en = entry(e0 + 64 + (uint32_t)lane);
                    const bool act = e0 + (uint32_t)lane < T;
                    const uint32_t alt = cur + en.w;
                    bool imp = act && alt < dist[en.nbr];
                    bool push = imp;
                    // two lanes improving the same neighbour: found through an
                    // LDS table (neighbour mod 64: a collision is only a false
                    // alarm); then they settle on the minimum by store and re-read
                    if (imp) htab[en.nbr & 63] = (uint32_t)lane;
                    __asm__ volatile("" ::: "memory");
                    const bool clash = imp && htab[en.nbr & 63] != (uint32_t)lane;
                    if (__ballot(clash)) {
                        push = false;
                        while (__ballot(imp)) {
                            if (imp) dist[en.nbr] = alt;
                            wave_sync_mem();
                            if (imp) {
                                const uint32_t now = dist[en.nbr];
                                push |= now == alt;
                                imp = now > alt;
                            }
                        }
                    } else if (imp) {
                        dist[en.nbr] = alt;
                    }
                    // pushes, grouped by bucket
                    const uint32_t bk = b + en.w >= (uint32_t)nbk ? b + en.w - (uint32_t)nbk : b + en.w;
                    unsigned long long m;
                    while ((m = __ballot(push)) != 0ull) {
                        const int l = __builtin_ctzll(m);
                        const uint32_t bb = (uint32_t)__builtin_amdgcn_readlane((int)bk, l);
                        const unsigned long long grp = __ballot(push && bk == bb);
                        const uint32_t cnt = (uint32_t)__builtin_popcountll(grp);
                        const uint32_t r = (uint32_t)__builtin_amdgcn_mbcnt_hi(
                            (unsigned)(grp >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)grp, 0u));
                        uint32_t t = uni(tail[bb]), tc = uni(fill[bb]);
                        const bool empty = uni(head[bb]) == kNone;
                        // chunks: the free stack, else the pool's next unused one
                        uint32_t need = (empty ? 1u : 0u) + ((empty ? 0u : tc) + cnt > 64u ? 1u : 0u);
                        uint32_t got[2] = {kNone, kNone};
                        for (uint32_t q = 0; q < need; q++) {
                            if (ftop > 0) {
                                if (ftop > fsafe) { // (an entry stored since the last fence)
                                    wave_sync_mem();
                                    fsafe = ftop;
                                }
                                got[q] = uni(fstk[--ftop]);
                                fsafe = ftop < fsafe ? ftop : fsafe;
                            } else if (bump < nchunk) {
                                got[q] = bump++;
                            } else {
                                failed = true;
                            }
                        }
                        if (failed) break;
                        if (empty) {
                            t = got[0];
                            tc = 0;
                            if (lane == 0) head[bb] = t;
                        }
                        const uint32_t room = 64u - tc;
                        const uint32_t t2 = empty ? got[1] : got[0];
                        if (push && bk == bb) {
                            if (r < room) pool[(size_t)t * 64 + tc + r] = (uint32_t)en.nbr;
                            else pool[(size_t)t2 * 64 + (r - room)] = (uint32_t)en.nbr;
                        }
                        if (lane == 0) {
                            if (cnt > room) {
                                nxt[t] = t2;
                                tail[bb] = t2;
                                fill[bb] = cnt - room;
                            } else {
                                tail[bb] = t;
                                fill[bb] = tc + cnt;
                            }
                        }
                        pending += cnt;
                        if (bk == bb) push = false;
                    }
                    // the batch's stores seen by the next batch's gathers
                    wave_sync_mem();
                    fsafe = ftop;
                    en = nx_en;
                    if (failed) break;
                }
            }
            // (a guard, not a path: every distance is below V * wmax)
            if (++cur > maxd) failed = true;
        }
        if (failed) {
            if (lane == 0) {
                const unsigned k = atomicAdd(nredo, 1u);
                redo[k] = row;
            }
            continue;
        }
        // the row (topology.c:1744-1791), then the self path (topology.c:1431-1576)
        double* out = lat + (size_t)(rowlist ? row - row_lo : i) * (size_t)A;
        for (int j = lane; j < A; j += 64) {
            if (j == row) continue;
            const uint32_t d = dist[g.slot_vertex[j]];
            out[j] = d == kInf ? -1.0 : (d == 0 ? 1.0 : (double)d);
        }
        double best = 0.0;
        int bk = 0x7fffffff;
        for (int k = g.inc_off[src] + lane; k < g.inc_off[src + 1]; k += 64) {
            double l = g.inc_w[k];
            if (g.inc_nbr[k] != src) l *= 2.0;
            if (bk == 0x7fffffff || l < best) best = l, bk = k;
        }
        for (int o = 32; o > 0; o >>= 1) {
            const double ob = __shfl_xor(best, o);
            const int ok = __shfl_xor(bk, o);
            if (ok != 0x7fffffff && (bk == 0x7fffffff || ob < best || (ob == best && ok < bk))) best = ob, bk = ok;
        }
        if (lane == 0) out[row] = bk == 0x7fffffff ? 0.0 : best;
    }
}

int hip_rc(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

} // namespace

// Rows [row_lo, row_hi) of the latency table into d_lat (row - row_lo major,
// A doubles per row).  wmax: the largest edge latency in ms (every one whole,
// at least 1).  Synchronous: the workspace is allocated for the call.
extern "C" int shd_dev_frontier_latency(const ShdGraphDev* gp, int row_lo, int row_hi, int wmax, double* d_lat,
                                        void* stream) {
    const ShdGraphDev g = *gp;
    if (!g.sl) return shd_fail(-ENOTSUP, "frontier latencies need whole-ms edge latencies");
    // the ring's head / tail / fill words of the 4 waves live in LDS: at most
    // 3,349 buckets, i.e. edge latencies up to kFrontierMaxWms = 3,348 ms
    if (wmax < 1 || wmax > kFrontierMaxWms)
        return shd_fail(-ENOTSUP, "frontier latencies: largest edge latency %d ms (the limit is %d ms)", wmax,
                        kFrontierMaxWms);
    const int nrows = row_hi - row_lo;
    if (nrows <= 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    int dev = 0, cus = 0;
    int rc = hip_rc(hipGetDevice(&dev), "hipGetDevice");
    if (!rc) rc = hip_rc(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
    if (rc) return rc;
    const int nbk = wmax + 1;
    const size_t lds = dial_lds_words(nbk) * 4 * kWaves;
    if (lds > 160 * 1024) return shd_fail(-ENOTSUP, "frontier latencies: %d buckets exceed the LDS", nbk);
    if ((rc = hip_rc(hipFuncSetAttribute((const void*)k_sssp_dial, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                     "hipFuncSetAttribute k_sssp_dial")))
        return rc;
    const int Vp = (g.V + 63) / 64 * 64;
    int* d_redo = nullptr;
    unsigned* d_nredo = nullptr;
    if ((rc = hip_rc(hipMalloc((void**)&d_redo, sizeof(int) * (size_t)nrows + sizeof(unsigned) * 4), "hipMalloc redo")))
        return rc;
    d_nredo = reinterpret_cast<unsigned*>(d_redo + nrows);
    char* slab = nullptr;
    // pass 1: a pool for 1.5 V live entries per wave; pass 2 (the rows whose
    // pool ran out): the worst case, every incidence entry pushed once
    for (int pass = 0; pass < 2 && !rc; pass++) {
        unsigned nr = (unsigned)nrows;
        if (pass == 1) {
            if ((rc = hip_rc(hipMemcpyAsync(&nr, d_nredo, sizeof nr, hipMemcpyDeviceToHost, s), "redo count")) ||
                (rc = hip_rc(hipStreamSynchronize(s), "hipStreamSynchronize")))
                break;
            if (nr == 0) break;
        }
        const uint32_t nchunk = (uint32_t)nbk + 2u +
                                (pass == 0 ? (uint32_t)((3ull * (size_t)g.V / 2 + 63) / 64) : (uint32_t)((size_t)g.M / 64 + 1));
        const size_t stride = ((size_t)Vp * 4 + (size_t)nchunk * (64 * 4 + 8) + 255) & ~(size_t)255;
        size_t fr = 0, tot = 0;
        if ((rc = hip_rc(hipMemGetInfo(&fr, &tot), "hipMemGetInfo"))) break;
        long waves = (long)cus * 32;
        const long fit = (long)((fr / 2) / stride);
        if (waves > fit) waves = fit;
        if (waves > (long)nr) waves = nr;
        if (waves < 1) {
            rc = shd_fail(-ENOMEM, "frontier latencies: no room for one wave's workspace (%zu B)", stride);
            break;
        }
        const int grid = (int)((waves + kWaves - 1) / kWaves);
        if ((rc = hip_rc(hipMalloc((void**)&slab, stride * (size_t)grid * kWaves), "hipMalloc frontier workspace")))
            break;
        if (pass == 0) {
            if ((rc = hip_rc(hipMemsetAsync(d_nredo, 0, sizeof(unsigned), s), "hipMemsetAsync"))) break;
            hipLaunchKernelGGL(k_sssp_dial, dim3(grid), dim3(64 * kWaves), lds, s, g, row_lo, (const int*)nullptr,
                               nrows, nbk, slab, stride, nchunk, Vp, d_lat, d_redo, d_nredo);
        } else {
            // (the redo list is both read and appended to: a row can only fail
            // once more if even the worst-case pool is short, which it is not)
            int* d_list = nullptr;
            if ((rc = hip_rc(hipMalloc((void**)&d_list, sizeof(int) * nr), "hipMalloc redo list")) ||
                (rc = hip_rc(hipMemcpyAsync(d_list, d_redo, sizeof(int) * nr, hipMemcpyDeviceToDevice, s), "copy")) ||
                (rc = hip_rc(hipMemsetAsync(d_nredo, 0, sizeof(unsigned), s), "hipMemsetAsync"))) {
                (void)hipFree(d_list);
                break;
            }
            hipLaunchKernelGGL(k_sssp_dial, dim3(grid), dim3(64 * kWaves), lds, s, g, row_lo, d_list, (int)nr, nbk,
                               slab, stride, nchunk, Vp, d_lat, d_redo, d_nredo);
            rc = hip_rc(hipGetLastError(), "k_sssp_dial launch");
            if (!rc) rc = hip_rc(hipStreamSynchronize(s), "k_sssp_dial");
            unsigned left = 0;
            if (!rc) rc = hip_rc(hipMemcpy(&left, d_nredo, sizeof left, hipMemcpyDeviceToHost), "redo count");
            if (!rc && left) rc = shd_fail(-EIO, "frontier latencies: %u rows overflowed the worst-case pool", left);
            (void)hipFree(d_list);
        }
        if (!rc) rc = hip_rc(hipGetLastError(), "k_sssp_dial launch");
        if (!rc) rc = hip_rc(hipStreamSynchronize(s), "k_sssp_dial");
        (void)hipFree(slab);
        slab = nullptr;
    }
    (void)hipFree(slab);
    (void)hipFree(d_redo);
    return rc;
}
