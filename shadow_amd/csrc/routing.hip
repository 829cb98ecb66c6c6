// routing.hip -- routing-table rows on gfx950.
//
// k_sssp_rows: one 64-lane wave per source slot runs igraph 0.8's
// get_shortest_paths_dijkstra exactly (routing/topology.c:1682 ->
// igraph structural_properties.c): indexed binary max-heap on -dist
// (igraph_2wheap: shift-up swaps while !(x < parent), sink prefers the left
// child when left >= right, modify = sink then shift-up at the original
// position, delete_max = swap root/last, pop, sink), incidence lists in
// igraph_incident(mode OUT) order, "first finite distance" -> push,
// "alt < cur" -> modify, early exit once every attached vertex is popped.
// Reliability is folded along the final parent chain exactly as
// _topology_computePathProperties multiplies it (topology.c:1308-1365): the
// last improvement of v fixes rel[v] = rel[u] * (1 - loss(u,v)) with rel[u]
// already final because u was popped.  Results are therefore bit-identical
// to the reference, ties included, with no CPU fallback.
//
// Parallel structure: sources are independent (one wave each, all of the
// chip's waves in flight); within a pop the wave relaxes 64 incident edges
// per step (coalesced CSR reads, gathered dist reads), a ballot collects
// the improving lanes and the wave applies their heap operations in
// incidence order (the order igraph applies them) with uniform control
// flow.  Small graphs keep dist/rel/heap (32 B per vertex) in LDS; large
// graphs use a per-wave slab in HBM.
#include <hip/hip_runtime.h>

#include <cerrno>

#include "shd_internal.h"

namespace {

struct Heap {
    double* d; // heap keys (= -dist), position order
    int* ix;   // position -> vertex
    int* pos;  // vertex -> position + 2 (igraph index2)
    int n;
};

__device__ __forceinline__ void heap_shift_up(Heap& h, int e) {
    const double x = h.d[e];
    const int xi = h.ix[e];
    while (e > 0) {
        const int p = ((e + 1) >> 1) - 1;
        const double dp = h.d[p];
        if (x < dp) break; // igraph: stop iff data[elem] < data[parent]
        const int pi = h.ix[p];
        h.d[e] = dp;
        h.ix[e] = pi;
        h.pos[pi] = e + 2;
        e = p;
    }
    h.d[e] = x;
    h.ix[e] = xi;
    h.pos[xi] = e + 2;
}

__device__ __forceinline__ void heap_sink(Heap& h, int e) {
    const double x = h.d[e];
    const int xi = h.ix[e];
    for (;;) {
        const int l = 2 * e + 1;
        if (l >= h.n) break;
        const int r = l + 1;
        const double dl = h.d[l];
        int c = l;
        double dc = dl;
        if (r != h.n) {
            const double dr = h.d[r];
            if (!(dl >= dr)) c = r, dc = dr; // left when left >= right
        }
        if (!(x < dc)) break;
        const int ci = h.ix[c];
        h.d[e] = dc;
        h.ix[e] = ci;
        h.pos[ci] = e + 2;
        e = c;
    }
    h.d[e] = x;
    h.ix[e] = xi;
    h.pos[xi] = e + 2;
}

__device__ __forceinline__ void heap_push(Heap& h, int idx, double key) {
    const int s = h.n++;
    h.d[s] = key;
    h.ix[s] = idx;
    h.pos[idx] = s + 2;
    heap_shift_up(h, s);
}

__device__ __forceinline__ int heap_delete_max(Heap& h, double* key) {
    const double top = h.d[0];
    const int ti = h.ix[0];
    const int last = h.n - 1;
    if (last > 0) {
        const int li = h.ix[last];
        h.d[0] = h.d[last];
        h.ix[0] = li;
        h.pos[li] = 2;
    }
    h.n = last;
    h.pos[ti] = 0;
    if (h.n > 0) heap_sink(h, 0);
    *key = top;
    return ti;
}

__device__ __forceinline__ void heap_modify(Heap& h, int idx, double key) {
    const int p = h.pos[idx] - 2;
    h.d[p] = key;
    heap_sink(h, p);
    heap_shift_up(h, p);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// _topology_computeShortestPathToSelf (topology.c:1431-1576): first strict
// minimum over the OUT-incident edges of u, loops at L, other edges at 2L
// (and reliability squared).  Lane-parallel: (lat, k) lexicographic minimum.
__device__ void self_entry(const ShdGraphDev& g, int u, ShdEntry* out, int lane) {
    const int k0 = g.inc_off[u], k1 = g.inc_off[u + 1];
    double best = 0.0;
    int bk = 0x7fffffff;
    for (int k = k0 + lane; k < k1; k += 64) {
        double lat = g.inc_w[k];
        if (g.inc_nbr[k] != u) lat *= 2.0;
        if (bk == 0x7fffffff || lat < best) best = lat, bk = k;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double ob = __shfl_xor(best, off);
        const int ok = __shfl_xor(bk, off);
        if (ok != 0x7fffffff && (bk == 0x7fffffff || ob < best || (ob == best && ok < bk))) best = ob, bk = ok;
    }
    if (lane == 0) {
        ShdEntry e;
        if (bk == 0x7fffffff) {
            e.lat = 0.0; // vertex without edges (topology.c:1516-1519)
            e.rel = 0.0;
        } else {
            double r = g.inc_r[bk];
            if (g.inc_nbr[bk] != u) r = r * r;
            e.lat = best;
            e.rel = r;
        }
        *out = e;
    }
}

template <bool kLds>
__global__ __launch_bounds__(64) void k_sssp_rows(ShdGraphDev g, int row_lo, int row_hi, ShdEntry* __restrict__ tab,
                                                  char* __restrict__ slab, size_t slab_stride) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x;
    const int V = g.V, A = g.A;
    char* base = kLds ? smem : slab + (size_t)blockIdx.x * slab_stride;
    double* dist = reinterpret_cast<double*>(base);
    double* rel = dist + V;
    double* hd = rel + V;
    int* hix = reinterpret_cast<int*>(hd + V);
    int* hpos = hix + V;

    for (int row = row_lo + (int)blockIdx.x; row < row_hi; row += (int)gridDim.x) {
        const int src = g.slot_vertex[row];
        for (int v = lane; v < V; v += 64) dist[v] = -1.0;
        __syncthreads();
        Heap h{hd, hix, hpos, 0};
        dist[src] = 0.0;
        rel[src] = 1.0;
        heap_push(h, src, 0.0);
        int to_reach = A;
        while (h.n > 0 && to_reach > 0) {
            double key;
            const int u = heap_delete_max(h, &key);
            const double mindist = -key;
            if (g.vertex_slot[u] >= 0) --to_reach;
            const double ru = rel[u];
            const int k0 = g.inc_off[u], k1 = g.inc_off[u + 1];
            for (int b = k0; b < k1; b += 64) {
                const int k = b + lane;
                int v = 0;
                double alt = 0.0;
                bool imp = false, fresh = false;
                if (k < k1) {
                    v = g.inc_nbr[k];
                    alt = mindist + g.inc_w[k];
                    const double cur = dist[v];
                    fresh = cur < 0;
                    imp = fresh || alt < cur;
                    if (imp) {
                        dist[v] = alt;
                        rel[v] = ru * g.inc_r[k];
                    }
                }
                unsigned long long m = __ballot(imp);
                const unsigned long long fm = __ballot(fresh);
                while (m) { // heap ops in incidence order, uniform across the wave
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const int vv = __builtin_amdgcn_readlane(v, l);
                    const double aa = readlane_d(alt, l);
                    if ((fm >> l) & 1ull) heap_push(h, vv, -aa);
                    else heap_modify(h, vv, -aa);
                }
            }
            __syncthreads();
        }
        ShdEntry* out = tab + (size_t)row * (size_t)A;
        for (int j = lane; j < A; j += 64) {
            if (j == row) continue;
            const int v = g.slot_vertex[j];
            const double l = dist[v];
            ShdEntry e;
            if (l < 0) {
                e.lat = -1.0; // unreachable: impossible on a validated (strongly connected) graph
                e.rel = 0.0;
            } else {
                e.lat = (l == 0) ? 1.0 : l; // topology.c:1787-1791
                e.rel = rel[v];
            }
            out[j] = e;
        }
        self_entry(g, src, out + row, lane);
        __syncthreads();
    }
}

// _topology_lookupDirectPath (topology.c:1816-1858): the (s,d) edge itself.
__global__ __launch_bounds__(256) void k_direct_rows(ShdGraphDev g, int row_lo, int row_hi, ShdEntry* __restrict__ tab) {
    const int A = g.A;
    for (int row = row_lo + (int)blockIdx.x; row < row_hi; row += (int)gridDim.x) {
        ShdEntry* out = tab + (size_t)row * (size_t)A;
        for (int j = threadIdx.x; j < A; j += blockDim.x) out[j] = ShdEntry{-1.0, 0.0};
        __syncthreads();
        const int u = g.slot_vertex[row];
        for (int k = g.inc_off[u] + threadIdx.x; k < g.inc_off[u + 1]; k += blockDim.x) {
            const int j = g.vertex_slot[g.inc_nbr[k]];
            if (j >= 0) out[j] = ShdEntry{0.0 + g.inc_w[k], 1.0 * g.inc_r[k]};
        }
        __syncthreads();
    }
}

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

constexpr int kLdsMaxV = 4096; // 32 B per vertex -> 128 KiB of the 160 KiB LDS

} // namespace

extern "C" int shd_dev_build_rows(const ShdGraphDev* gp, int use_sp, int row_lo, int row_hi, ShdEntry* tab) {
    const ShdGraphDev g = *gp;
    const int rows = row_hi - row_lo;
    if (rows <= 0) return 0;
    int rc;
    if (!use_sp) {
        const int grid = rows < 4096 ? rows : 4096;
        hipLaunchKernelGGL(k_direct_rows, dim3(grid), dim3(256), 0, nullptr, g, row_lo, row_hi, tab);
        if ((rc = hip_status(hipGetLastError(), "k_direct_rows launch"))) return rc;
        return hip_status(hipDeviceSynchronize(), "k_direct_rows");
    }
    const size_t per_vertex = 3 * sizeof(double) + 2 * sizeof(int);
    if (g.V <= kLdsMaxV) {
        const size_t lds = per_vertex * (size_t)g.V;
        if (lds > 65536 &&
            (rc = hip_status(hipFuncSetAttribute((const void*)k_sssp_rows<true>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                             "hipFuncSetAttribute")))
            return rc;
        hipLaunchKernelGGL(k_sssp_rows<true>, dim3(rows), dim3(64), lds, nullptr, g, row_lo, row_hi, tab,
                           (char*)nullptr, (size_t)0);
        if ((rc = hip_status(hipGetLastError(), "k_sssp_rows<lds> launch"))) return rc;
        return hip_status(hipDeviceSynchronize(), "k_sssp_rows<lds>");
    }
    // large graphs: one HBM slab per resident wave, persistent over rows
    const size_t stride = (per_vertex * (size_t)g.V + 255) & ~(size_t)255;
    int grid = rows < 2048 ? rows : 2048;
    char* slab = nullptr;
    while (hipMalloc((void**)&slab, stride * (size_t)grid) != hipSuccess) {
        (void)hipGetLastError();
        if (grid <= 64) return shd_fail(-ENOMEM, "cannot allocate SSSP workspace");
        grid /= 2;
    }
    hipLaunchKernelGGL(k_sssp_rows<false>, dim3(grid), dim3(64), 0, nullptr, g, row_lo, row_hi, tab, slab, stride);
    rc = hip_status(hipGetLastError(), "k_sssp_rows<hbm> launch");
    if (!rc) rc = hip_status(hipDeviceSynchronize(), "k_sssp_rows<hbm>");
    (void)hipFree(slab);
    return rc;
}
