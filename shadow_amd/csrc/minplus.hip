// minplus.hip -- the latency half of the routing table by blocked min-plus
// Floyd-Warshall (north_star's dense-graph kernel), for whole-ms graphs.
//
// The routing table's latencies are shortest-path distances; they do not
// depend on which of several equal-latency paths igraph's heap picks (only
// the reliabilities do), so any exact all-pairs algorithm
// reproduces them.  With every edge latency a whole number of ms (the
// condition of ShdGraphDev.sl, the integer-key SSSP kernels' condition)
// every path sum is an exact integer below 2^32 - 1, so u32 min-plus gives
// the f64 values bit for bit.  Entries are then formed as
// _topology_computeSourcePaths stores them (topology.c:1744-1791): the self
// path by _topology_computeShortestPathToSelf's rule (loops at L, other
// edges at 2L, topology.c:1431-1576), latency 0 -> 1 ms, unreachable -1.
//
// Layout: a Vp x Vp u32 distance matrix (Vp = V rounded up to 64), 64 x 64
// tiles.  Round kb, two launches: the tiles of row and column kb take one
// min-plus product with the (closed) diagonal tile, then every other tile one
// product of its row-kb and column-kb tiles, both staged in LDS.  The only
// dependent chain -- the next round's diagonal tile closing over its own 64
// vertices -- runs in the one workgroup of the second launch that produced
// that tile, so a round is two product launches deep.  The products are the
// O(V^3) part.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <new>

#include "shd_internal.h"

namespace {

constexpr int kT = 64;                  // tile edge
constexpr uint32_t kInfD = 0x3FFFFFFFu; // unreachable; two of them still fit a u32
constexpr int kMaxV = 16384;            // Vp^2 x 4 B = 1 GiB

// row u of the distance matrix: 0 on the diagonal, the direct edges
// (igraph_incident mode OUT: an undirected edge is in both lists; the
// lightest of parallel edges), unreachable elsewhere -- built in LDS, one
// workgroup per row, stored once
__global__ __launch_bounds__(256) void k_fw_init(ShdGraphDev g, uint32_t* __restrict__ D, int Vp) {
    extern __shared__ __attribute__((aligned(16))) uint32_t row[];
    for (int u = blockIdx.x; u < Vp; u += gridDim.x) {
        for (int j = threadIdx.x; j < Vp; j += 256) row[j] = j == u ? 0u : kInfD;
        __syncthreads();
        if (u < g.V)
            for (int k = g.inc_off[u] + threadIdx.x; k < g.inc_off[u + 1]; k += 256) {
                const int v = g.inc_nbr[k];
                if (v != u) atomicMin(&row[v], (uint32_t)g.inc_w[k]);
            }
        __syncthreads();
        for (int j = threadIdx.x * 4; j < Vp; j += 1024)
            *reinterpret_cast<uint4*>(&D[(size_t)u * Vp + j]) = *reinterpret_cast<const uint4*>(&row[j]);
        __syncthreads();
    }
}

// The diagonal tile's closure keeps each thread's 4 x 4 block in registers;
// step k needs the tile's current row k and column k, which the 16 threads
// owning them publish to a double-buffered LDS line before the step's single
// barrier.
__device__ __forceinline__ void ld_block(uint32_t (&d)[4][4], const uint32_t* D, int Vp, int ti, int tj, int ty, int tx) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint4 v = *reinterpret_cast<const uint4*>(&D[(size_t)(ti * kT + ty * 4 + r) * Vp + tj * kT + tx * 4]);
        d[r][0] = v.x, d[r][1] = v.y, d[r][2] = v.z, d[r][3] = v.w;
    }
}
__device__ __forceinline__ void st_block(const uint32_t (&d)[4][4], uint32_t* D, int Vp, int ti, int tj, int ty, int tx) {
#pragma unroll
    for (int r = 0; r < 4; r++)
        *reinterpret_cast<uint4*>(&D[(size_t)(ti * kT + ty * 4 + r) * Vp + tj * kT + tx * 4]) =
            make_uint4(d[r][0], d[r][1], d[r][2], d[r][3]);
}
__device__ __forceinline__ void relax(uint32_t (&d)[4][4], const uint4 cv, const uint4 rv) {
    const uint32_t a[4] = {cv.x, cv.y, cv.z, cv.w}, b[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t x = a[r] + b[c];
            d[r][c] = x < d[r][c] ? x : d[r][c];
        }
}

// closes the tile held in registers over its own 64 vertices (64 dependent
// steps)
__device__ __forceinline__ void close_regs(uint32_t (&d)[4][4], uint32_t (*rowb)[kT], uint32_t (*colb)[kT], int ty,
                                           int tx) {
    // (k = 4 kk + r with r a compile-time constant: a runtime index into d
    // would put the block in scratch memory)
    for (int kk = 0; kk < kT / 4; kk++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int p = r & 1;
            if (ty == kk) *reinterpret_cast<uint4*>(&rowb[p][tx * 4]) = make_uint4(d[r][0], d[r][1], d[r][2], d[r][3]);
            if (tx == kk) *reinterpret_cast<uint4*>(&colb[p][ty * 4]) = make_uint4(d[0][r], d[1][r], d[2][r], d[3][r]);
            __syncthreads();
            relax(d, *reinterpret_cast<const uint4*>(&colb[p][ty * 4]), *reinterpret_cast<const uint4*>(&rowb[p][tx * 4]));
        }
}

// round 0's diagonal tile (later rounds' are closed by k_fw_tiles)
__global__ __launch_bounds__(256) void k_fw_close(uint32_t* __restrict__ D, int Vp) {
    __shared__ __attribute__((aligned(16))) uint32_t rowb[2][kT], colb[2][kT];
    const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
    uint32_t d[4][4];
    ld_block(d, D, Vp, 0, 0, ty, tx);
    close_regs(d, rowb, colb, ty, tx);
    st_block(d, D, Vp, 0, 0, ty, tx);
}

// Round kb with its diagonal tile C already closed.  Every tile (i, j) takes
// one min-plus product: d = min(d, D[i][kb] (+) D[kb][j]), both operands
// staged in LDS (a 4 x 4 register block per thread, two 16-B LDS reads and
// 32 VALU per k).  cross: the tiles of row and column kb -- for a row tile
// that is C (+) R, for a column tile L (+) C: with C closed (zero diagonal)
// one product is the whole relaxation through block kb, because a path's
// last vertex in block kb splits it into a C part and an R part.  The
// operands are staged before the tile is written, and no workgroup writes
// another's operand (C is not written), so the update is in place.  prod:
// every other tile, through the updated row and column tiles; the workgroup
// of tile (kb + 1, kb + 1) then closes it for the next round (block 0, so
// that the round's dependent chain starts first).
template <bool kCross>
__global__ __launch_bounds__(256) void k_fw_tiles(uint32_t* __restrict__ D, int Vp, int kb, int nb) {
    __shared__ __attribute__((aligned(16))) uint32_t at[kT][kT + 4]; // D[i][kb] transposed: at[k][i]
    __shared__ __attribute__((aligned(16))) uint32_t bt[kT][kT];     // D[kb][j]: bt[k][j]
    int ti, tj;
    bool close = false;
    if (kCross) {
        const int q = (int)blockIdx.x;
        const bool row = q < nb - 1;
        int o = row ? q : q - (nb - 1);
        if (o >= kb) o++;
        ti = row ? kb : o;
        tj = row ? o : kb;
    } else {
        int q = (int)blockIdx.x;
        const int nk = kb + 1 < nb ? kb + 1 : -1; // the next round's diagonal tile, taken by block 0
        if (nk >= 0) {
            const int qn = (nk - (nk > kb)) * (nb - 1) + (nk - (nk > kb)); // its linear index
            if (q == 0) q = qn, close = true;
            else if (q <= qn) q--;
        }
        ti = q / (nb - 1), tj = q % (nb - 1);
        if (ti >= kb) ti++;
        if (tj >= kb) tj++;
    }
    // the three tiles' loads all in flight before the first LDS store
    uint4 av[4], bv[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int q = (int)threadIdx.x + 256 * m, r = q >> 4, c = (q & 15) * 4;
        av[m] = *reinterpret_cast<const uint4*>(&D[(size_t)(ti * kT + r) * Vp + kb * kT + c]);
        bv[m] = *reinterpret_cast<const uint4*>(&D[(size_t)(kb * kT + r) * Vp + tj * kT + c]);
    }
    const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
    uint32_t d[4][4];
    ld_block(d, D, Vp, ti, tj, ty, tx);
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int q = (int)threadIdx.x + 256 * m, r = q >> 4, c = (q & 15) * 4;
        at[c][r] = av[m].x, at[c + 1][r] = av[m].y, at[c + 2][r] = av[m].z, at[c + 3][r] = av[m].w;
        *reinterpret_cast<uint4*>(&bt[r][c]) = bv[m];
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < kT; k++)
        relax(d, *reinterpret_cast<const uint4*>(&at[k][ty * 4]), *reinterpret_cast<const uint4*>(&bt[k][tx * 4]));
    if (!kCross && close) { // (block-uniform)
        __syncthreads();
        close_regs(d, reinterpret_cast<uint32_t(*)[kT]>(&at[0][0]), reinterpret_cast<uint32_t(*)[kT]>(&bt[0][0]), ty,
                   tx);
    }
    st_block(d, D, Vp, ti, tj, ty, tx);
}

// the A x A latency table from the distances (one block per row)
__global__ __launch_bounds__(256) void k_fw_rows(ShdGraphDev g, const uint32_t* __restrict__ D, int Vp,
                                                 double* __restrict__ lat) {
    const int A = g.A;
    for (int i = blockIdx.x; i < A; i += gridDim.x) {
        const int u = g.slot_vertex[i];
        double* out = lat + (size_t)i * A;
        for (int j = threadIdx.x; j < A; j += 256) {
            if (j == i) continue;
            const uint32_t d = D[(size_t)u * Vp + g.slot_vertex[j]];
            out[j] = d >= kInfD ? -1.0 : (d == 0 ? 1.0 : (double)d); // topology.c:1787-1791
        }
        if (threadIdx.x < 64) { // the self path, topology.c:1431-1576 (first strict minimum)
            const int lane = threadIdx.x;
            double best = 0.0;
            int bk = 0x7fffffff;
            for (int k = g.inc_off[u] + lane; k < g.inc_off[u + 1]; k += 64) {
                double l = g.inc_w[k];
                if (g.inc_nbr[k] != u) l *= 2.0;
                if (bk == 0x7fffffff || l < best) best = l, bk = k;
            }
            for (int o = 32; o > 0; o >>= 1) {
                const double ob = __shfl_xor(best, o);
                const int ok = __shfl_xor(bk, o);
                if (ok != 0x7fffffff && (bk == 0x7fffffff || ob < best || (ob == best && ok < bk))) best = ob, bk = ok;
            }
            if (lane == 0) out[i] = bk == 0x7fffffff ? 0.0 : best;
        }
    }
}

int hip_rc(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

} // namespace

// Grow-only distance matrix of a caller (one per topology), and the event
// that marks the end of its last use: a call on another stream waits for it.
struct FwScratch {
    int device = -1;
    uint32_t* D = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool used = false;
};

extern "C" int shd_dev_fw_latency(const ShdGraphDev* gp, double* d_lat, void** scratch, void* stream) {
    const ShdGraphDev g = *gp;
    if (!g.sl) return shd_fail(-ENOTSUP, "min-plus latencies need whole-ms edge latencies");
    if (g.V > kMaxV) return shd_fail(-ENOTSUP, "min-plus latencies: %d vertices > %d", g.V, kMaxV);
    if (!scratch) return shd_fail(-EINVAL, "min-plus scratch");
    const int Vp = (g.V + kT - 1) / kT * kT, nb = Vp / kT;
    hipStream_t s = (hipStream_t)stream;
    int dev = 0;
    int rc = hip_rc(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    FwScratch* w = static_cast<FwScratch*>(*scratch);
    if (!w) {
        w = new (std::nothrow) FwScratch();
        if (!w) return -ENOMEM;
        *scratch = w;
    }
    if (w->device >= 0 && w->device != dev) return shd_fail(-EINVAL, "min-plus scratch of device %d used on %d", w->device, dev);
    w->device = dev;
    if (!w->done && (rc = hip_rc(hipEventCreateWithFlags(&w->done, hipEventDisableTiming), "hipEventCreate"))) return rc;
    const size_t need = (size_t)Vp * Vp;
    if (need > w->cap) {
        if (w->used && (rc = hip_rc(hipEventSynchronize(w->done), "min-plus scratch quiesce"))) return rc;
        (void)hipFree(w->D);
        w->D = nullptr;
        w->cap = 0;
        if ((rc = hip_rc(hipMalloc((void**)&w->D, need * 4), "hipMalloc distances"))) return rc;
        w->cap = need;
    } else if (w->used && (rc = hip_rc(hipStreamWaitEvent(s, w->done, 0), "hipStreamWaitEvent"))) {
        return rc;
    }
    uint32_t* D = w->D;
    hipLaunchKernelGGL(k_fw_init, dim3(Vp < 4096 ? Vp : 4096), dim3(256), (size_t)Vp * 4, s, g, D, Vp);
    hipLaunchKernelGGL(k_fw_close, dim3(1), dim3(256), 0, s, D, Vp);
    for (int kb = 0; nb > 1 && kb < nb; kb++) {
        hipLaunchKernelGGL(k_fw_tiles<true>, dim3(2 * (nb - 1)), dim3(256), 0, s, D, Vp, kb, nb);
        hipLaunchKernelGGL(k_fw_tiles<false>, dim3((nb - 1) * (nb - 1)), dim3(256), 0, s, D, Vp, kb, nb);
    }
    hipLaunchKernelGGL(k_fw_rows, dim3(g.A < 4096 ? g.A : 4096), dim3(256), 0, s, g, D, Vp, d_lat);
    if ((rc = hip_rc(hipGetLastError(), "min-plus launch"))) return rc;
    w->used = true;
    return hip_rc(hipEventRecord(w->done, s), "hipEventRecord");
}

extern "C" void shd_dev_fw_scratch_free(void* scratch) {
    FwScratch* w = static_cast<FwScratch*>(scratch);
    if (!w) return;
    int cur = -1;
    if (w->device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != w->device) (void)hipSetDevice(w->device);
    if (w->used) (void)hipEventSynchronize(w->done);
    (void)hipFree(w->D);
    if (w->done) (void)hipEventDestroy(w->done);
    if (cur >= 0 && cur != w->device) (void)hipSetDevice(cur);
    delete w;
}
