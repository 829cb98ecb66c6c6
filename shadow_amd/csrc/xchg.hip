// xchg.hip -- multi-GPU rounds: the destination-owner event
// exchange, the owner-row routing of records for row-sharded tables, and an
// RCCL transport (ncclSend / ncclRecv over xGMI).  The reference has no
// multi-process or multi-GPU path (one process, pthread workers,
// core/worker.c:132-185); the exchange is what replaces the direct push into
// another host's locked queue (scheduler_policy_host_single.c:198-219) when
// the destination host lives on another GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include <pthread.h>

#include "shd_internal.h"

namespace {

constexpr int kMaxWorld = 64;
constexpr int kRouteBlock = 256;

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

struct RouteArgs {
    uint32_t bounds[kMaxWorld + 1]; // row (slot) bounds per rank
    int world;
};

// Rank holding the row that answers record p: the slot of the endpoint
// touched first (topology.c:1189-1215; touch order = host_info[.].y).
__device__ __forceinline__ int route_rank(const ShdPkt& p, const uint2* __restrict__ host_info, uint32_t nhosts,
                                          const RouteArgs& ra) {
    if (p.src_host >= nhosts || p.dst_host >= nhosts) return 0;
    const uint2 hs = host_info[p.src_host], hd = host_info[p.dst_host];
    if (hs.x == ~0u || hd.x == ~0u) return 0; // unattached: rank 0 reports it undelivered
    const uint32_t owner = (hs.x != hd.x && hd.y < hs.y) ? hd.x : hs.x;
    int r = 0;
    while (r + 1 < ra.world && owner >= ra.bounds[r + 1]) r++;
    return r;
}

// Two passes over the same chunks: pass 0 counts records per (rank, block),
// pass 1 writes each record to its rank's region at off[rank * nblocks +
// block] + its stable position (ballot prefix per tile), so records keep
// their order within each destination rank.
template <int kPass>
__global__ __launch_bounds__(kRouteBlock) void k_route(const ShdPkt* __restrict__ recs, size_t n,
                                                       const uint2* __restrict__ host_info, uint32_t nhosts,
                                                       RouteArgs ra, size_t chunk, uint32_t* __restrict__ cnt,
                                                       const uint32_t* __restrict__ off, ShdPkt* __restrict__ out) {
    __shared__ uint32_t wsum[kRouteBlock / 64][kMaxWorld];
    __shared__ uint32_t base[kMaxWorld];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t nb = gridDim.x;
    for (int r = threadIdx.x; r < ra.world; r += kRouteBlock) base[r] = kPass ? off[(size_t)r * nb + blockIdx.x] : 0u;
    __syncthreads();
    const size_t beg = (size_t)blockIdx.x * chunk;
    const size_t end = beg + chunk < n ? beg + chunk : n;
    for (size_t t0 = beg; t0 < end; t0 += kRouteBlock) {
        const size_t i = t0 + threadIdx.x;
        ShdPkt p;
        int r = -1;
        if (i < end) {
            p = recs[i];
            r = route_rank(p, host_info, nhosts, ra);
        }
        uint32_t prefix = 0;
        for (int rr = 0; rr < ra.world; rr++) {
            const unsigned long long m = __ballot(r == rr);
            if (r == rr) prefix = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (lane == 0) wsum[w][rr] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        if (r >= 0 && kPass) {
            uint32_t pos = base[r] + prefix;
            for (int k = 0; k < w; k++) pos += wsum[k][r];
            out[pos] = p;
        }
        __syncthreads();
        for (int rr = threadIdx.x; rr < ra.world; rr += kRouteBlock) {
            uint32_t s = 0;
            for (int k = 0; k < kRouteBlock / 64; k++) s += wsum[k][rr];
            base[rr] += s;
        }
        __syncthreads();
    }
    if (!kPass)
        for (int r = threadIdx.x; r < ra.world; r += kRouteBlock) cnt[(size_t)r * nb + blockIdx.x] = base[r];
}

// exclusive scan of m counts (one block; m <= world * nblocks, small)
__global__ __launch_bounds__(1024) void k_scan_small(const uint32_t* __restrict__ in, uint32_t m,
                                                     uint32_t* __restrict__ out) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (m + 1023) / 1024;
    const uint32_t b = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t k = 0; k < per && b + k < m; k++) s += in[b + k];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int k = 0; k < 1024; k++) {
            const uint32_t v = part[k];
            part[k] = acc;
            acc += v;
        }
        out[m] = acc;
    }
    __syncthreads();
    uint32_t acc = part[threadIdx.x];
    for (uint32_t k = 0; k < per && b + k < m; k++) {
        out[b + k] = acc;
        acc += in[b + k];
    }
}

// offsets[bounds[r]] for r = 0..world (the per-rank cuts of a CSR array)
__global__ void k_cuts(const uint32_t* __restrict__ offsets, RouteArgs ra, uint32_t* __restrict__ cuts) {
    const int r = threadIdx.x;
    if (r <= ra.world) cuts[r] = offsets[ra.bounds[r]];
}

// This rank's row of the exchange's count matrix: the events for each owner
// rank (the cuts of the destination offsets at the owners' host bounds), its
// receive capacity and whether its own stage failed (then the offsets are
// not read; bit 0 of the flag word) and whether its runs are sorted (bit 1);
// the cuts themselves for the payload's base.
__global__ void k_count_row(const uint32_t* __restrict__ offsets, RouteArgs ra, uint32_t* __restrict__ cuts,
                            uint64_t* __restrict__ row, uint64_t cap, int failed, int sorted) {
    const int r = threadIdx.x, W = ra.world;
    if (failed) {
        if (r < W) row[r] = 0ull;
        if (r == 0) row[W] = cap, row[W + 1] = 1ull;
        return;
    }
    if (r <= W) cuts[r] = offsets[ra.bounds[r]];
    if (r < W) row[r] = (uint64_t)(offsets[ra.bounds[r + 1]] - offsets[ra.bounds[r]]);
    if (r == 0) row[W] = cap, row[W + 1] = sorted ? 2ull : 0ull;
}

// the same row from cuts computed by the sender (the split exchange's
// shd_dev_packet_round_grouped_split)
__global__ void k_count_row_cuts(const uint32_t* __restrict__ cuts, int W, uint64_t* __restrict__ row, uint64_t cap,
                                 int failed, int sorted) {
    const int r = threadIdx.x;
    if (r < W) row[r] = failed ? 0ull : (uint64_t)(cuts[r + 1] - cuts[r]);
    if (r == 0) row[W] = cap, row[W + 1] = failed ? 1ull : sorted ? 2ull : 0ull;
}

int make_args(const uint32_t* bounds, int world, RouteArgs* ra) {
    if (world < 1 || world > kMaxWorld) return shd_fail(-EINVAL, "world %d outside 1..%d", world, kMaxWorld);
    ra->world = world;
    for (int r = 0; r <= world; r++) {
        ra->bounds[r] = bounds[r];
        if (r && bounds[r] < bounds[r - 1]) return shd_fail(-EINVAL, "bounds not ascending");
    }
    return 0;
}

// A count that says "this rank failed before the exchange" (no real count
// comes near it): a rank whose local stage failed still takes part in the
// count all-to-all, so every rank learns it and all of them return together
// instead of leaving the others waiting in the payload collective.
constexpr uint64_t kPeerFailed = ~0ull;

// all-to-all of per-peer element counts, then of the blocks themselves.
// local_rc != 0: this rank failed before the exchange (send_elems unused);
// it returns local_rc and every peer returns -EIO, after the same counts
// all-to-all.
int exchange_blocks(const ShdTransport* x, const void* d_send, const uint64_t* send_elems, size_t elem_bytes,
                    void* d_recv, size_t recv_cap, size_t* n_recv, hipStream_t s, uint64_t* recv_out = nullptr,
                    int local_rc = 0) {
    const int W = x->world;
    std::vector<uint64_t> recv_elems(W), sb(W), rb(W), fail(W, kPeerFailed);
    int rc = x->alltoall_u64(x->user, local_rc ? fail.data() : send_elems, recv_elems.data());
    if (rc) return rc < 0 ? rc : -EIO;
    if (local_rc) return local_rc;
    for (int r = 0; r < W; r++)
        if (recv_elems[r] == kPeerFailed) return shd_fail(-EIO, "rank %d failed before the exchange", r);
    uint64_t total = 0;
    for (int r = 0; r < W; r++) {
        total += recv_elems[r];
        sb[r] = send_elems[r] * elem_bytes;
        rb[r] = recv_elems[r] * elem_bytes;
    }
    // The capacity verdict is collective: a rank that returned here alone
    // would leave its peers waiting in the payload exchange.  Every rank
    // sends its overflow flag to every peer, and all of them fail together.
    const uint64_t over = total > recv_cap ? 1 : 0;
    std::vector<uint64_t> flags(W, over), peer(W);
    rc = x->alltoall_u64(x->user, flags.data(), peer.data());
    if (rc) return rc < 0 ? rc : -EIO;
    uint64_t any = 0;
    for (int r = 0; r < W; r++) any |= peer[r];
    if (over) return shd_fail(-ENOSPC, "receive %llu elements > capacity %zu", (unsigned long long)total, recv_cap);
    if (any) return shd_fail(-ENOSPC, "a peer's receive capacity is too small for this exchange");
    rc = x->alltoallv(x->user, d_send, sb.data(), d_recv, rb.data(), (void*)s);
    if (rc) return rc < 0 ? rc : -EIO;
    *n_recv = (size_t)total;
    if (recv_out)
        for (int r = 0; r < W; r++) recv_out[r] = recv_elems[r];
    return 0;
}

// Peer r's slice of this rank's destination offsets, rebased to its block:
// out[lo_r + r + j] = off[lo_r + j] - off[lo_r], j = 0 .. H_r (the slices of
// all peers back to back: sum of (H_r + 1) = H + W entries).
// (r0, r1: only the slices of owners [r0, r1) -- the split exchange's groups)
__global__ __launch_bounds__(256) void k_offset_slices(const uint32_t* __restrict__ off, RouteArgs ra,
                                                       uint32_t* __restrict__ out, int r0 = 0, int r1 = -1) {
    if (r1 < 0) r1 = ra.world;
    const uint32_t first = ra.bounds[r0] + (uint32_t)r0, total = ra.bounds[r1] + (uint32_t)r1;
    for (uint32_t p = first + blockIdx.x * blockDim.x + threadIdx.x; p < total; p += gridDim.x * blockDim.x) {
        int r = r0;
        while (r + 1 < ra.world && p >= ra.bounds[r + 1] + (uint32_t)(r + 1)) r++;
        const uint32_t lo = ra.bounds[r], j = p - lo - (uint32_t)r;
        out[p] = off[lo + j] - off[lo];
    }
}

// ---- RCCL transport ----
struct Rccl {
    ShdTransport x;
    ncclComm_t comm;
    int device;
    hipStream_t stream; // the count exchange's own stream (never the null stream)
    uint64_t* d_u64;    // 2 x world staging for the count exchange
    uint64_t* h_u64;    // its pinned host side
};

int nccl_status(ncclResult_t r, const char* what) {
    return r == ncclSuccess ? 0 : shd_fail(-EIO, "%s: %s", what, ncclGetErrorString(r));
}

// Counts: pinned staging, stream-ordered copies and the send/recv group on
// the transport's own stream, one synchronisation of that stream (the host
// needs the counts); nothing touches the null stream.
int rccl_alltoall_u64(void* user, const uint64_t* send, uint64_t* recv) {
    Rccl* t = static_cast<Rccl*>(user);
    const int W = t->x.world;
    std::memcpy(t->h_u64, send, 8 * (size_t)W);
    int rc = hip_status(hipMemcpyAsync(t->d_u64, t->h_u64, 8 * (size_t)W, hipMemcpyHostToDevice, t->stream),
                        "counts H2D");
    if (rc) return rc;
    if ((rc = nccl_status(ncclGroupStart(), "ncclGroupStart"))) return rc;
    for (int r = 0; r < W; r++) {
        if ((rc = nccl_status(ncclSend(t->d_u64 + r, 1, ncclUint64, r, t->comm, t->stream), "ncclSend")) ||
            (rc = nccl_status(ncclRecv(t->d_u64 + W + r, 1, ncclUint64, r, t->comm, t->stream), "ncclRecv"))) {
            (void)ncclGroupEnd();
            return rc;
        }
    }
    if ((rc = nccl_status(ncclGroupEnd(), "ncclGroupEnd"))) return rc;
    if ((rc = hip_status(hipMemcpyAsync(t->h_u64 + W, t->d_u64 + W, 8 * (size_t)W, hipMemcpyDeviceToHost, t->stream),
                         "counts D2H")) ||
        (rc = hip_status(hipStreamSynchronize(t->stream), "counts sync")))
        return rc;
    std::memcpy(recv, t->h_u64 + W, 8 * (size_t)W);
    return 0;
}

// send_off: peer r's block at d_send + send_off[r] (NULL: blocks contiguous
// in rank order)
int rccl_alltoallv_off(void* user, const void* d_send, const uint64_t* send_bytes, const uint64_t* send_off,
                       void* d_recv, const uint64_t* recv_bytes, void* stream) {
    Rccl* t = static_cast<Rccl*>(user);
    const int W = t->x.world;
    hipStream_t s = (hipStream_t)stream;
    int rc = nccl_status(ncclGroupStart(), "ncclGroupStart");
    if (rc) return rc;
    uint64_t so = 0, ro = 0;
    for (int r = 0; r < W; r++) {
        const uint64_t at = send_off ? send_off[r] : so;
        if (send_bytes[r] &&
            (rc = nccl_status(ncclSend((const char*)d_send + at, send_bytes[r], ncclChar, r, t->comm, s), "ncclSend")))
            break;
        if (recv_bytes[r] &&
            (rc = nccl_status(ncclRecv((char*)d_recv + ro, recv_bytes[r], ncclChar, r, t->comm, s), "ncclRecv")))
            break;
        so += send_bytes[r];
        ro += recv_bytes[r];
    }
    const int rc2 = nccl_status(ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : rc2;
}
int rccl_alltoallv(void* user, const void* d_send, const uint64_t* send_bytes, void* d_recv,
                   const uint64_t* recv_bytes, void* stream) {
    return rccl_alltoallv_off(user, d_send, send_bytes, nullptr, d_recv, recv_bytes, stream);
}
// The exchange's two all-to-alls -- the payload (explicit send offsets) and
// the destination offset slices (contiguous) -- as ONE send/recv group: one
// RCCL launch per round instead of two back to back on the stream.
int rccl_alltoallv2(void* user, const void* d_send, const uint64_t* send_bytes, const uint64_t* send_off,
                    void* d_recv, const uint64_t* recv_bytes, const void* d_send2, const uint64_t* send2_bytes,
                    void* d_recv2, const uint64_t* recv2_bytes, void* stream, const uint64_t* send2_off = nullptr) {
    Rccl* t = static_cast<Rccl*>(user);
    const int W = t->x.world;
    hipStream_t s = (hipStream_t)stream;
    int rc = nccl_status(ncclGroupStart(), "ncclGroupStart");
    if (rc) return rc;
    uint64_t ro = 0, so2 = 0, ro2 = 0;
    for (int r = 0; r < W && !rc; r++) {
        if (send_bytes[r])
            rc = nccl_status(ncclSend((const char*)d_send + send_off[r], send_bytes[r], ncclChar, r, t->comm, s),
                             "ncclSend");
        if (!rc && recv_bytes[r])
            rc = nccl_status(ncclRecv((char*)d_recv + ro, recv_bytes[r], ncclChar, r, t->comm, s), "ncclRecv");
        if (!rc && send2_bytes[r])
            rc = nccl_status(ncclSend((const char*)d_send2 + (send2_off ? send2_off[r] : so2), send2_bytes[r],
                                      ncclChar, r, t->comm, s),
                             "ncclSend");
        if (!rc && recv2_bytes[r])
            rc = nccl_status(ncclRecv((char*)d_recv2 + ro2, recv2_bytes[r], ncclChar, r, t->comm, s), "ncclRecv");
        ro += recv_bytes[r];
        so2 += send2_bytes[r];
        ro2 += recv2_bytes[r];
    }
    const int rc2 = nccl_status(ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : rc2;
}

// All-gather of variable blocks, in place: rank r's block is bytes
// [off[r], off[r+1]) of buf.  Every rank sends its block straight to every
// peer (one send/recv group): on the fully connected xGMI mesh each block
// crosses one link and the 7 links of a GPU run at once, where a ring would
// pass every block through W - 1 hops.
int rccl_allgatherv(void* user, void* d_buf, const uint64_t* off, void* stream) {
    Rccl* t = static_cast<Rccl*>(user);
    const int W = t->x.world, me = t->x.rank;
    hipStream_t s = (hipStream_t)stream;
    char* b = static_cast<char*>(d_buf);
    const uint64_t mine = off[me + 1] - off[me];
    int rc = nccl_status(ncclGroupStart(), "ncclGroupStart");
    if (rc) return rc;
    for (int r = 0; r < W && !rc; r++) {
        if (r == me) continue;
        if (mine) rc = nccl_status(ncclSend(b + off[me], mine, ncclChar, r, t->comm, s), "ncclSend");
        if (!rc && off[r + 1] > off[r])
            rc = nccl_status(ncclRecv(b + off[r], off[r + 1] - off[r], ncclChar, r, t->comm, s), "ncclRecv");
    }
    const int rc2 = nccl_status(ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : rc2;
}

} // namespace

extern "C" int shd_dev_route_records(const ShdPktCtx* c, const ShdTransport* x, const ShdPkt* d_recs, size_t n,
                                     const uint32_t* row_bounds, ShdPkt* d_part, ShdPkt* d_recv, size_t recv_cap,
                                     size_t* n_recv, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    RouteArgs ra;
    int rc = make_args(row_bounds, x->world, &ra);
    if (rc) return rc;
    const int W = x->world;
    size_t nblocks = n ? (n + 65535) / 65536 : 1;
    if (nblocks > 1024) nblocks = 1024;
    const size_t chunk = n ? (n + nblocks - 1) / nblocks : 1;
    const size_t m = (size_t)W * nblocks;
    // counts and offsets in the workspace's persistent scratch (no per-round
    // hipMalloc / hipFree), offsets read back into its pinned host side
    void *dscr = nullptr, *hscr = nullptr;
    std::vector<uint64_t> send(W);
    // (a failure from here on still goes through the count all-to-all)
    if (!(rc = shd_dev_ws_scratch(c->ws, 4 * (2 * m + 1), 4 * (m + 1), &dscr, &hscr))) {
        uint32_t* d_cnt = static_cast<uint32_t*>(dscr);
        uint32_t* d_off = d_cnt + m;
        const uint32_t* off = static_cast<const uint32_t*>(hscr);
        const uint2* hi = reinterpret_cast<const uint2*>(c->host_info);
        hipLaunchKernelGGL(k_route<0>, dim3(nblocks), dim3(kRouteBlock), 0, s, d_recs, n, hi, c->nhosts, ra, chunk,
                           d_cnt, nullptr, nullptr);
        hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, s, d_cnt, (uint32_t)m, d_off);
        hipLaunchKernelGGL(k_route<1>, dim3(nblocks), dim3(kRouteBlock), 0, s, d_recs, n, hi, c->nhosts, ra, chunk,
                           nullptr, d_off, d_part);
        if (!(rc = hip_status(hipGetLastError(), "k_route launch")) &&
            !(rc = hip_status(hipMemcpyAsync(hscr, d_off, 4 * (m + 1), hipMemcpyDeviceToHost, s), "route D2H")))
            rc = hip_status(hipStreamSynchronize(s), "route sync");
        if (!rc)
            for (int r = 0; r < W; r++) send[r] = off[(size_t)(r + 1) * nblocks] - off[(size_t)r * nblocks];
    }
    rc = exchange_blocks(x, d_part, send.data(), sizeof(ShdPkt), d_recv, recv_cap, n_recv, s, nullptr, rc);
    if (!rc) rc = hip_status(hipStreamSynchronize(s), "route exchange");
    return rc;
}

extern "C" int shd_dev_event_cuts(void* ws, const uint32_t* d_dst_offsets, const uint32_t* host_bounds, int world,
                                  uint64_t* send_elems, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    RouteArgs ra;
    int rc = make_args(host_bounds, world, &ra);
    if (rc) return rc;
    void *dscr = nullptr, *hscr = nullptr;
    if ((rc = shd_dev_ws_scratch(ws, 4 * (kMaxWorld + 1), 4 * (kMaxWorld + 1), &dscr, &hscr))) return rc;
    uint32_t* d_cuts = static_cast<uint32_t*>(dscr);
    const uint32_t* cuts = static_cast<const uint32_t*>(hscr);
    hipLaunchKernelGGL(k_cuts, dim3(1), dim3(kMaxWorld + 1), 0, s, d_dst_offsets, ra, d_cuts);
    rc = hip_status(hipMemcpyAsync(hscr, d_cuts, 4 * (size_t)(world + 1), hipMemcpyDeviceToHost, s), "cuts D2H");
    if (!rc) rc = hip_status(hipStreamSynchronize(s), "cuts sync");
    if (!rc)
        for (int r = 0; r < world; r++) send_elems[r] = cuts[r + 1] - cuts[r];
    return rc;
}

// Destination-owner exchange + regroup by runs: the events of each peer's
// destinations (elem_bytes each: 32-B ShdDeliv or the 24-B wire record) and,
// beside them, the rebased per-destination offsets of that block; the owner
// then merges the W destination-grouped runs in place
// (shd_dev_deliv_merge_runs) instead of scattering every received event into
// destination slabs again.  Scratch (device, caller-sized, see
// xchg_scratch_words): [cuts | H + W slices | W x (H_me + 1) received offsets
// | W + 1 block bases]; host (pinned): [cuts | block bases].
// the count matrix of a rank whose workspace could not allocate its own
// (exchange_runs_core): a static device array, so that rank can still join the
// matrix all-gather and report its failure through it
__device__ uint64_t g_xmat_fallback[64 * 66];
namespace {
int local_allgatherv(void* user, void* d_buf, const uint64_t* off, void* stream);
int local_alltoallv_off(void* user, const void* d_send, const uint64_t* send_bytes, const uint64_t* send_off,
                        void* d_recv, const uint64_t* recv_bytes, void* stream);
size_t xchg_scratch_words(uint32_t H, int W, uint32_t Hm) {
    return (kMaxWorld + 1) + ((size_t)H + W) + (size_t)W * (Hm + 1) + (W + 1);
}
// local_rc != 0: this rank's own round failed; it still joins the count
// all-to-all (exchange_blocks) so that every rank fails together.  sorted:
// this rank's runs are in event_compare order inside every destination; the
// owner merges instead of sorting when every sender's are (the count
// matrix says so; without it only for ShdDeliv runs, sorted by contract).
int exchange_runs_core(void* ws, const ShdTransport* x, const void* d_events, size_t elem_bytes, int wire, int sorted,
                       const uint32_t* d_dst_offsets, const uint32_t* host_bounds, void* d_recv, size_t recv_cap,
                       ShdDeliv* d_out, uint32_t* d_out_offsets, size_t* n_out, hipStream_t s, uint32_t* dscr,
                       uint32_t* hscr, int local_rc = 0) {
    const int W = x->world, me = x->rank;
    RouteArgs ra;
    int rc = make_args(host_bounds, W, &ra); // (checked by every rank alike: no collective yet)
    if (rc) return rc;
    if (!local_rc) { // SHD_DEBUG_FAIL_RANK=r: rank r fails before the exchange (test of the agreement)
        const char* f = getenv("SHD_DEBUG_FAIL_RANK");
        if (f && atoi(f) == me) local_rc = shd_fail(-EIO, "debug: injected failure of rank %d", me);
    }
    // With an all-gather in the transport, one collective carries the whole
    // count matrix (every rank's counts for every owner, its receive capacity
    // and its failure flag): the cuts, the counts and the capacity verdict in
    // one host round trip instead of three; every rank reads the same matrix,
    // so all of them fail together.
    uint64_t *d_mat = nullptr, *h_mat = nullptr;
    // (the library's own transports: their all-gather takes any device
    // buffer; a caller's transport may only know the buffers it registered).
    // The form depends on the transport alone, so every rank takes the same
    // collectives: a rank whose matrix allocation failed still joins the
    // all-gather, with the static fallback matrix, and reports the failure in
    // its row's flag -- every rank then returns an error together.
    const bool own = x->allgatherv == rccl_allgatherv || x->allgatherv == local_allgatherv;
    const bool one_trip = own;
    std::vector<uint64_t> h_fallback;
    if (one_trip) {
        const int xrc = shd_dev_ws_xmat(ws, (size_t)W * (W + 2), &d_mat, &h_mat);
        if (xrc) {
            if (!local_rc) local_rc = xrc;
            if ((rc = hip_status(hipGetSymbolAddress((void**)&d_mat, HIP_SYMBOL(g_xmat_fallback)),
                                 "fallback count matrix")))
                return rc;
            h_fallback.assign((size_t)W * (W + 2), 0);
            h_mat = h_fallback.data();
        }
    }
    if (local_rc && !one_trip) { // only the count all-to-all that tells the peers
        std::vector<uint64_t> none(W, 0);
        size_t nr = 0;
        return exchange_blocks(x, nullptr, none.data(), elem_bytes, nullptr, 0, &nr, s, nullptr, local_rc);
    }
    const uint32_t H = host_bounds[W], lo = host_bounds[me], hi = host_bounds[me + 1], Hm = hi - lo;
    if (one_trip) {
        const size_t rw = (size_t)W + 2;
        uint32_t* d_cuts = local_rc ? nullptr : dscr;
        hipLaunchKernelGGL(k_count_row, dim3(1), dim3(kMaxWorld + 1), 0, s, local_rc ? nullptr : d_dst_offsets, ra,
                           d_cuts, d_mat + (size_t)me * rw, (uint64_t)recv_cap, local_rc ? 1 : 0, sorted);
        uint32_t* d_sl = local_rc ? nullptr : dscr + (kMaxWorld + 1);
        if (!local_rc)
            hipLaunchKernelGGL(k_offset_slices,
                               dim3((unsigned)(((size_t)H + W + 255) / 256 < 4096 ? ((size_t)H + W + 255) / 256 : 4096)),
                               dim3(256), 0, s, d_dst_offsets, ra, d_sl);
        std::vector<uint64_t> moff(W + 1);
        for (int r = 0; r <= W; r++) moff[r] = 8ull * rw * (uint64_t)r;
        int rc2 = hip_status(hipGetLastError(), "count row launch");
        if (!rc2) rc2 = x->allgatherv(x->user, d_mat, moff.data(), (void*)s);
        if (rc2) return rc2 < 0 ? rc2 : -EIO;
        if ((rc2 = hip_status(hipMemcpyAsync(h_mat, d_mat, 8 * rw * (size_t)W, hipMemcpyDeviceToHost, s), "counts D2H")) ||
            (!local_rc && (rc2 = hip_status(hipMemcpyAsync(hscr, dscr, 4 * (size_t)(W + 1), hipMemcpyDeviceToHost, s),
                                            "cuts D2H"))) ||
            (rc2 = hip_status(hipStreamSynchronize(s), "counts sync")))
            return rc2;
        if (local_rc) return local_rc;
        bool over = false;
        int all_sorted = 1;
        for (int r = 0; r < W; r++) {
            if (h_mat[(size_t)r * rw + W + 1] & 1ull) return shd_fail(-EIO, "rank %d failed before the exchange", r);
            if (!(h_mat[(size_t)r * rw + W + 1] & 2ull)) all_sorted = 0;
        }
        for (int t = 0; t < W; t++) {
            uint64_t tot = 0;
            for (int r = 0; r < W; r++) tot += h_mat[(size_t)r * rw + t];
            if (tot > h_mat[(size_t)t * rw + W]) {
                if (t == me) return shd_fail(-ENOSPC, "receive %llu elements > capacity %zu", (unsigned long long)tot, recv_cap);
                over = true;
            }
        }
        if (over) return shd_fail(-ENOSPC, "a peer's receive capacity is too small for this exchange");
        // this rank's own block stays where it is: the merge reads it from
        // the send buffer (no copy through the transport)
        std::vector<uint64_t> sbytes(W), rbytes(W), recv(W), sb(W), rb(W);
        uint64_t nrecv = 0;
        for (int r = 0; r < W; r++) {
            sbytes[r] = r == me ? 0 : h_mat[(size_t)me * rw + r] * elem_bytes;
            recv[r] = h_mat[(size_t)r * rw + me];
            rbytes[r] = r == me ? 0 : recv[r] * elem_bytes;
            nrecv += recv[r];
        }
        uint32_t* h_cuts = hscr;
        std::vector<uint64_t> soff(W);
        for (int r = 0; r < W; r++) soff[r] = (uint64_t)h_cuts[r] * elem_bytes; // (own block skipped, in place)
        // the payload and the offset slices (H_r + 1 words to peer r, H_me + 1
        // from each peer): one group on RCCL
        const size_t n_sl = (size_t)H + W;
        uint32_t* d_ro = d_sl + n_sl;
        uint32_t* d_bb = d_ro + (size_t)W * (Hm + 1);
        uint32_t* h_bb = h_cuts + (kMaxWorld + 1);
        for (int r = 0; r < W; r++) {
            sb[r] = 4ull * (host_bounds[r + 1] - host_bounds[r] + 1);
            rb[r] = 4ull * (Hm + 1);
        }
        int rc3;
        if (x->allgatherv == rccl_allgatherv)
            rc3 = rccl_alltoallv2(x->user, d_events, sbytes.data(), soff.data(), d_recv, rbytes.data(), d_sl,
                                  sb.data(), d_ro, rb.data(), (void*)s);
        else if (!(rc3 = local_alltoallv_off(x->user, d_events, sbytes.data(), soff.data(), d_recv, rbytes.data(),
                                              (void*)s)))
            rc3 = x->alltoallv(x->user, d_sl, sb.data(), d_ro, rb.data(), (void*)s);
        if (rc3) return rc3 < 0 ? rc3 : -EIO;
        h_bb[0] = 0;
        for (int r = 0; r < W; r++) h_bb[r + 1] = h_bb[r] + (r == me ? 0u : (uint32_t)recv[r]);
        const void* self_block = static_cast<const char*>(d_events) + (size_t)h_cuts[me] * elem_bytes;
        if ((rc3 = hip_status(hipMemcpyAsync(d_bb, h_bb, 4 * (size_t)(W + 1), hipMemcpyHostToDevice, s), "bases H2D")) ||
            (rc3 = shd_dev_deliv_merge_runs_self(ws, d_recv, self_block, (uint32_t)me, wire, all_sorted, nrecv, d_ro, d_bb,
                                                 (uint32_t)W, lo, hi, d_out, d_out_offsets, s)) ||
            (rc3 = shd_dev_ws_sync(ws, (void*)s)))
            return rc3;
        *n_out = nrecv;
        return 0;
    }
    const size_t n_sl = (size_t)H + W, n_ro = (size_t)W * (Hm + 1);
    uint32_t* d_cuts = dscr;
    uint32_t* d_sl = d_cuts + (kMaxWorld + 1);
    uint32_t* d_ro = d_sl + n_sl;
    uint32_t* d_bb = d_ro + n_ro;
    uint32_t* h_cuts = hscr;
    uint32_t* h_bb = h_cuts + (kMaxWorld + 1);
    // cuts of the events at the owners' host bounds, and the offset slices
    {
        hipLaunchKernelGGL(k_cuts, dim3(1), dim3(kMaxWorld + 1), 0, s, d_dst_offsets, ra, d_cuts);
        hipLaunchKernelGGL(k_offset_slices, dim3((unsigned)((n_sl + 255) / 256 < 4096 ? (n_sl + 255) / 256 : 4096)),
                           dim3(256), 0, s, d_dst_offsets, ra, d_sl);
        if (!(rc = hip_status(hipGetLastError(), "exchange cuts launch")) &&
            !(rc = hip_status(hipMemcpyAsync(h_cuts, d_cuts, 4 * (size_t)(W + 1), hipMemcpyDeviceToHost, s),
                              "cuts D2H")))
            rc = hip_status(hipStreamSynchronize(s), "cuts sync");
    }
    std::vector<uint64_t> send(W), recv(W), sb(W), rb(W);
    if (!rc)
        for (int r = 0; r < W; r++) send[r] = h_cuts[r + 1] - h_cuts[r];
    size_t nrecv = 0;
    // the events (the capacity verdict is collective inside, and so is a
    // failure of this rank's stages above)
    if ((rc = exchange_blocks(x, static_cast<const char*>(d_events) + (rc ? 0 : (size_t)h_cuts[0] * elem_bytes),
                              send.data(), elem_bytes, d_recv, recv_cap, &nrecv, s, recv.data(), rc)))
        return rc;
    // the offset slices: H_r + 1 words to peer r, H_me + 1 from each peer
    for (int r = 0; r < W; r++) {
        sb[r] = 4ull * (host_bounds[r + 1] - host_bounds[r] + 1);
        rb[r] = 4ull * (Hm + 1);
    }
    rc = x->alltoallv(x->user, d_sl, sb.data(), d_ro, rb.data(), (void*)s);
    if (rc) return rc < 0 ? rc : -EIO;
    h_bb[0] = 0;
    for (int r = 0; r < W; r++) h_bb[r + 1] = h_bb[r] + (uint32_t)recv[r];
    if ((rc = hip_status(hipMemcpyAsync(d_bb, h_bb, 4 * (size_t)(W + 1), hipMemcpyHostToDevice, s), "bases H2D")))
        return rc;
    if ((rc = shd_dev_deliv_merge_runs_self(ws, d_recv, nullptr, 0xffffffffu, wire, wire ? 0 : sorted, nrecv, d_ro,
                                            d_bb, (uint32_t)W, lo, hi, d_out, d_out_offsets, s)))
        return rc;
    // the sender's round and this merge ran on the workspace: their faults
    // are this call's (synchronous) -- reported now, not by a later call
    if ((rc = shd_dev_ws_sync(ws, (void*)s))) return rc;
    *n_out = nrecv;
    return 0;
}

// ---- the split exchange (shd_round_process_exchange on the library's own
// transports, SHD_XCHG_SPLIT != 0) ----
//
// The owners are split in two halves, A = ranks [0, W/2) and B = [W/2, W),
// and the payload goes out in two send/recv groups on a transfer stream of
// its own: A's blocks as soon as the sender has sorted A's buckets, while it
// sorts B's; B's blocks after that, while the A owners merge.  The count
// matrix does not wait for any sort: the per-owner cuts come straight from
// the partition (k_part_cuts), so the matrix all-gather and the host's read
// of it run beside the first half's sort.  Per rank and round (stream s =
// the caller's, x = the transfer stream):
//   s: scatter | cuts | count row | matrix all-gather | sort A | read-back (E)
//      | sort B, listed | (B) ............ | merge (own half's group) | wait G2
//   x:                  wait E (B if A had listed segments) | slices A,
//      group 1 (G1) | wait B | slices B, group 2 (G2)
// Phase times of the last split round of this thread, from HIP events
// (shd_round_exchange_phases): decide (the sender's kernels), counts (the
// matrix all-gather), group 1, group 2, merge, whole call, the time the
// transfers ran beside the sender's sort (group 1's start to the end of
// the sender's kernels) and the merge's time beside group 2.
constexpr int kPhases = 8;
thread_local double t_phase[kPhases];
thread_local int t_phase_valid = 0;

enum { kEvE, kEvB, kEvG1, kEvG2, kEv0, kEvFront, kEvCounts, kEvG1s, kEvG2s, kEvMs, kEvMe, kEvEnd, kEvCount };

struct SplitCtx {
    const ShdTransport* x;
    hipStream_t s;
    int W, me;
    uint64_t *d_mat, *h_mat;
    uint32_t *d_cuts, *h_cuts, *d_listed, *h_listed;
    uint64_t recv_cap;
    hipEvent_t* ev;
    bool front_done, mid_done;
};

int split_front(void* u, const uint32_t* d_cuts, int sorted) {
    SplitCtx* k = static_cast<SplitCtx*>(u);
    const size_t rw = (size_t)k->W + 2;
    (void)hipEventRecord(k->ev[kEvFront], k->s);
    hipLaunchKernelGGL(k_count_row_cuts, dim3(1), dim3(kMaxWorld + 1), 0, k->s, d_cuts, k->W,
                       k->d_mat + (size_t)k->me * rw, k->recv_cap, d_cuts ? 0 : 1, sorted);
    std::vector<uint64_t> moff(k->W + 1);
    for (int r = 0; r <= k->W; r++) moff[r] = 8ull * rw * (uint64_t)r;
    int rc = hip_status(hipGetLastError(), "count row launch");
    if (!rc) rc = k->x->allgatherv(k->x->user, k->d_mat, moff.data(), (void*)k->s);
    k->front_done = true; // (the collective was entered)
    (void)hipEventRecord(k->ev[kEvCounts], k->s);
    return rc ? (rc < 0 ? rc : -EIO) : 0;
}

int split_mid(void* u) {
    SplitCtx* k = static_cast<SplitCtx*>(u);
    k->mid_done = true;
    const size_t rw = (size_t)k->W + 2;
    int rc;
    if ((rc = hip_status(hipMemcpyAsync(k->h_mat, k->d_mat, 8 * rw * (size_t)k->W, hipMemcpyDeviceToHost, k->s),
                         "counts D2H")) ||
        (rc = hip_status(hipMemcpyAsync(k->h_cuts, k->d_cuts, 4 * (size_t)(k->W + 1), hipMemcpyDeviceToHost, k->s),
                         "cuts D2H")) ||
        (rc = hip_status(hipMemcpyAsync(k->h_listed, k->d_listed, 4, hipMemcpyDeviceToHost, k->s), "listed D2H")))
        return rc;
    return hip_status(hipEventRecord(k->ev[kEvE], k->s), "event E");
}

// one group: this rank's blocks for owners [r0, r1) and, when it is one of
// them, its receives (every peer's block and offset slice)
int split_group(const ShdTransport* x, int r0, int r1, int me, const void* d_events, const uint64_t* sbytes,
                const uint64_t* soff, void* d_recv, const uint64_t* rbytes, const uint32_t* d_sl,
                const uint64_t* sl_bytes, const uint64_t* sl_off, uint32_t* d_ro, const uint64_t* ro_bytes,
                hipStream_t xs) {
    const int W = x->world;
    const bool mine = me >= r0 && me < r1;
    std::vector<uint64_t> sb(W, 0), rb(W, 0), s2(W, 0), r2(W, 0);
    for (int r = r0; r < r1; r++) sb[r] = sbytes[r], s2[r] = sl_bytes[r];
    if (mine)
        for (int r = 0; r < W; r++) rb[r] = rbytes[r], r2[r] = ro_bytes[r];
    int rc;
    if (x->allgatherv == rccl_allgatherv)
        rc = rccl_alltoallv2(x->user, d_events, sb.data(), soff, d_recv, rb.data(), d_sl, s2.data(), d_ro, r2.data(),
                             (void*)xs, sl_off);
    else if (!(rc = local_alltoallv_off(x->user, d_events, sb.data(), soff, d_recv, rb.data(), (void*)xs)))
        rc = local_alltoallv_off(x->user, d_sl, s2.data(), sl_off, d_ro, r2.data(), (void*)xs);
    return rc ? (rc < 0 ? rc : -EIO) : 0;
}

float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : -1.f;
}

int exchange_split(const ShdPktCtx* c, const ShdTransport* x, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                   uint64_t end_time, uint64_t bootstrap_end, const uint32_t* host_bounds, void* d_wire_send,
                   uint8_t* d_status, uint64_t* d_counters, void* d_wire_recv, size_t recv_cap, ShdDeliv* d_out,
                   uint32_t* d_out_offsets, size_t* n_out, hipStream_t s, int sort_wire) {
    const int W = x->world, me = x->rank, half = W / 2;
    const uint32_t H = c->nhosts, lo = host_bounds[me], hi = host_bounds[me + 1], Hm = hi - lo;
    constexpr size_t elem = 24; // the wire record
    t_phase_valid = 0;
    RouteArgs ra;
    int rc = make_args(host_bounds, W, &ra);
    if (rc) return rc;
    // scratch: device [d_off H+1 | cuts | slices H+W | received slices W(Hm+1) | bases W+1 | listed]
    //          host   [cuts | bases | listed]
    const size_t dwords = ((size_t)H + 1) + xchg_scratch_words(H, W, Hm) + 1;
    void *dscr = nullptr, *hscr = nullptr, *xsv = nullptr;
    void* evv[kEvCount] = {};
    int local_rc = shd_dev_ws_scratch(c->ws, 4 * dwords, 4 * (2 * kMaxWorld + 4), &dscr, &hscr);
    if (!local_rc) local_rc = shd_dev_ws_xchg_sync_objs(c->ws, &xsv, evv, kEvCount);
    uint64_t *d_mat = nullptr, *h_mat = nullptr;
    std::vector<uint64_t> h_fallback;
    const int xrc = shd_dev_ws_xmat(c->ws, (size_t)W * (W + 2), &d_mat, &h_mat);
    if (xrc) { // (still joins the matrix all-gather, with the static fallback: see exchange_runs_core)
        if (!local_rc) local_rc = xrc;
        if ((rc = hip_status(hipGetSymbolAddress((void**)&d_mat, HIP_SYMBOL(g_xmat_fallback)), "fallback count matrix")))
            return rc;
        h_fallback.assign((size_t)W * (W + 2), 0);
        h_mat = h_fallback.data();
    }
    if (!local_rc) { // SHD_DEBUG_FAIL_RANK=r: rank r fails before the exchange (test of the agreement)
        const char* f = getenv("SHD_DEBUG_FAIL_RANK");
        if (f && atoi(f) == me) local_rc = shd_fail(-EIO, "debug: injected failure of rank %d", me);
    }
    hipEvent_t* ev = reinterpret_cast<hipEvent_t*>(evv);
    const hipStream_t xs = static_cast<hipStream_t>(xsv);
    uint32_t* d_off = static_cast<uint32_t*>(dscr);
    uint32_t* d_cuts = d_off ? d_off + (H + 1) : nullptr;
    uint32_t* d_sl = d_cuts ? d_cuts + (kMaxWorld + 1) : nullptr;
    uint32_t* d_ro = d_sl ? d_sl + ((size_t)H + W) : nullptr;
    uint32_t* d_bb = d_ro ? d_ro + (size_t)W * (Hm + 1) : nullptr;
    uint32_t* d_listed = d_bb ? d_bb + (W + 1) : nullptr;
    uint32_t* h_cuts = static_cast<uint32_t*>(hscr);
    uint32_t* h_bb = h_cuts ? h_cuts + (kMaxWorld + 1) : nullptr;
    uint32_t* h_listed = h_bb ? h_bb + (kMaxWorld + 1) : nullptr;
    SplitCtx k{x, s, W, me, d_mat, h_mat, d_cuts, h_cuts, d_listed, h_listed, (uint64_t)recv_cap, ev, false, false};
    const ShdSplitHooks hooks{split_front, split_mid, &k};
    if (!local_rc) {
        (void)hipEventRecord(ev[kEv0], s);
        local_rc = shd_dev_packet_round_grouped_split(c, d_recs, n, barrier, end_time, bootstrap_end, d_wire_send, d_off,
                                                      d_status, d_counters, (void*)s, sort_wire, host_bounds, W, half,
                                                      d_cuts, d_listed, &hooks);
    }
    if (!k.front_done) { // failed before the matrix went out: tell every peer through it
        std::vector<uint64_t> moff(W + 1);
        const size_t rw = (size_t)W + 2;
        for (int r = 0; r <= W; r++) moff[r] = 8ull * rw * (uint64_t)r;
        hipLaunchKernelGGL(k_count_row_cuts, dim3(1), dim3(kMaxWorld + 1), 0, s, nullptr, W, d_mat + (size_t)me * rw,
                           (uint64_t)recv_cap, 1, 0);
        int rc2 = hip_status(hipGetLastError(), "count row launch");
        if (!rc2) rc2 = x->allgatherv(x->user, d_mat, moff.data(), (void*)s);
        if (!rc2) rc2 = hip_status(hipStreamSynchronize(s), "counts sync");
        return local_rc ? local_rc : rc2;
    }
    // (the matrix went out saying this rank is fine: a later failure still
    // takes part in both groups below and in the closing status agreement)
    if (!local_rc) { // SHD_DEBUG_FAIL_LATE_RANK=r: rank r fails after its matrix row went out
        const char* f = getenv("SHD_DEBUG_FAIL_LATE_RANK");
        if (f && atoi(f) == me) local_rc = shd_fail(-EIO, "debug: injected late failure of rank %d", me);
    }
    if (!k.mid_done && (rc = split_mid(&k))) return rc;
    (void)hipEventRecord(ev[kEvB], s);
    if ((rc = hip_status(hipEventSynchronize(ev[kEvE]), "exchange counts"))) return rc;
    const size_t rw = (size_t)W + 2;
    int all_sorted = 1;
    for (int r = 0; r < W; r++) {
        if (h_mat[(size_t)r * rw + W + 1] & 1ull) {
            (void)hipStreamSynchronize(s);
            return local_rc ? local_rc : shd_fail(-EIO, "rank %d failed before the exchange", r);
        }
        if (!(h_mat[(size_t)r * rw + W + 1] & 2ull)) all_sorted = 0;
    }
    bool over = false;
    for (int t = 0; t < W; t++) {
        uint64_t tot = 0;
        for (int r = 0; r < W; r++) tot += h_mat[(size_t)r * rw + t];
        if (tot > h_mat[(size_t)t * rw + W]) over = true;
    }
    if (over) {
        (void)hipStreamSynchronize(s);
        return shd_fail(-ENOSPC, "a receive capacity is too small for this exchange");
    }
    std::vector<uint64_t> sbytes(W), rbytes(W), recv(W), soff(W), slb(W), sloff(W), rob(W);
    uint64_t nrecv = 0;
    for (int r = 0; r < W; r++) {
        sbytes[r] = r == me ? 0 : h_mat[(size_t)me * rw + r] * elem;
        recv[r] = h_mat[(size_t)r * rw + me];
        rbytes[r] = r == me ? 0 : recv[r] * elem;
        nrecv += recv[r];
        soff[r] = (uint64_t)h_cuts[r] * elem; // (own block skipped: merged in place)
        slb[r] = 4ull * (host_bounds[r + 1] - host_bounds[r] + 1);
        sloff[r] = 4ull * (host_bounds[r] + (uint64_t)r);
        rob[r] = 4ull * (Hm + 1);
    }
    h_bb[0] = 0;
    for (int r = 0; r < W; r++) h_bb[r + 1] = h_bb[r] + (r == me ? 0u : (uint32_t)recv[r]);
    const uint32_t listed_a = *h_listed;
    const void* self_block = static_cast<const char*>(d_wire_send) + (size_t)h_cuts[me] * elem;
    auto merge = [&]() {
        int m;
        (void)hipEventRecord(ev[kEvMs], s);
        if ((m = hip_status(hipMemcpyAsync(d_bb, h_bb, 4 * (size_t)(W + 1), hipMemcpyHostToDevice, s), "bases H2D")) ||
            (m = shd_dev_deliv_merge_runs_self(c->ws, d_wire_recv, self_block, (uint32_t)me, 1, all_sorted, nrecv, d_ro,
                                               d_bb, (uint32_t)W, lo, hi, d_out, d_out_offsets, s)))
            return m;
        return hip_status(hipEventRecord(ev[kEvMe], s), "merge event");
    };
    auto slices = [&](int r0, int r1) {
        const uint32_t m = host_bounds[r1] + (uint32_t)r1 - host_bounds[r0] - (uint32_t)r0;
        hipLaunchKernelGGL(k_offset_slices, dim3(m / 256 + 1 < 4096 ? m / 256 + 1 : 4096), dim3(256), 0, xs, d_off, ra,
                           d_sl, r0, r1);
        return hip_status(hipGetLastError(), "offset slices launch");
    };
    // group 1 (owners of A) once A's buckets are sorted -- after the listed
    // segments too when A had any (they are written at the round's end)
    int g1 = hip_status(hipStreamWaitEvent(xs, listed_a ? ev[kEvB] : ev[kEvE], 0), "wait A");
    (void)hipEventRecord(ev[kEvG1s], xs);
    if (!g1) g1 = slices(0, half);
    if (!g1) g1 = split_group(x, 0, half, me, d_wire_send, sbytes.data(), soff.data(), d_wire_recv, rbytes.data(),
                              d_sl, slb.data(), sloff.data(), d_ro, rob.data(), xs);
    (void)hipEventRecord(ev[kEvG1], xs);
    int mg = 0;
    if (me < half && !g1) mg = hip_status(hipStreamWaitEvent(s, ev[kEvG1], 0), "wait group 1") ?: merge();
    int g2 = hip_status(hipStreamWaitEvent(xs, ev[kEvB], 0), "wait B");
    (void)hipEventRecord(ev[kEvG2s], xs);
    if (!g2) g2 = slices(half, W);
    if (!g2) g2 = split_group(x, half, W, me, d_wire_send, sbytes.data(), soff.data(), d_wire_recv, rbytes.data(),
                              d_sl, slb.data(), sloff.data(), d_ro, rob.data(), xs);
    (void)hipEventRecord(ev[kEvG2], xs);
    if (me >= half && !g2 && !mg) mg = hip_status(hipStreamWaitEvent(s, ev[kEvG2], 0), "wait group 2") ?: merge();
    // the send buffer is the caller's again only when group 2 has gone out
    (void)hipStreamWaitEvent(s, ev[kEvG2], 0);
    (void)hipEventRecord(ev[kEvEnd], s);
    rc = shd_dev_ws_sync(c->ws, (void*)s);
    if (!rc) rc = hip_status(hipStreamSynchronize(xs), "transfer stream");
    // closing agreement: a rank that failed after its matrix row said it was
    // fine has still sent (possibly half-written) blocks in both groups, so
    // every rank learns every rank's final status before any returns, and
    // all of them fail together -- the rule the front all-gather keeps for
    // failures before the exchange
    const int mine_rc = local_rc ? local_rc : g1 ? g1 : g2 ? g2 : mg ? mg : rc;
    int failed_rank = -1;
    {
        std::vector<uint64_t> moff(W + 1);
        for (int r = 0; r <= W; r++) moff[r] = 8ull * rw * (uint64_t)r;
        h_mat[(size_t)me * rw] = mine_rc ? 1ull : 0ull;
        int a = hip_status(hipMemcpyAsync(d_mat + (size_t)me * rw, h_mat + (size_t)me * rw, 8, hipMemcpyHostToDevice, s),
                           "status H2D");
        if (!a) a = x->allgatherv(x->user, d_mat, moff.data(), (void*)s);
        if (!a) a = hip_status(hipMemcpyAsync(h_mat, d_mat, 8 * rw * (size_t)W, hipMemcpyDeviceToHost, s), "status D2H");
        if (!a) a = hip_status(hipStreamSynchronize(s), "status sync");
        if (a) return mine_rc ? mine_rc : (a < 0 ? a : -EIO);
        for (int r = 0; r < W && failed_rank < 0; r++)
            if (h_mat[(size_t)r * rw]) failed_rank = r;
    }
    if (mine_rc) return mine_rc;
    if (failed_rank >= 0) return shd_fail(-EIO, "rank %d failed during the exchange", failed_rank);
    t_phase[0] = ev_ms(ev[kEv0], ev[kEvFront]) + ev_ms(ev[kEvCounts], ev[kEvB]);
    t_phase[1] = ev_ms(ev[kEvFront], ev[kEvCounts]);
    t_phase[2] = ev_ms(ev[kEvG1s], ev[kEvG1]);
    t_phase[3] = ev_ms(ev[kEvG2s], ev[kEvG2]);
    t_phase[4] = ev_ms(ev[kEvMs], ev[kEvMe]);
    t_phase[5] = ev_ms(ev[kEv0], ev[kEvEnd]);
    const float ov = ev_ms(ev[kEvG1s], ev[kEvB]);
    t_phase[6] = ov > 0.f ? ov : 0.0;
    // the merge's time beside group 2 (the intervals' intersection)
    const float ms0 = ev_ms(ev[kEv0], ev[kEvMs]), me0 = ev_ms(ev[kEv0], ev[kEvMe]);
    const float gs0 = ev_ms(ev[kEv0], ev[kEvG2s]), ge0 = ev_ms(ev[kEv0], ev[kEvG2]);
    const float mo = (me0 < ge0 ? me0 : ge0) - (ms0 > gs0 ? ms0 : gs0);
    t_phase[7] = mo > 0.f ? mo : 0.0;
    t_phase_valid = 1;
    *n_out = nrecv;
    return 0;
}

} // namespace

extern "C" int shd_round_exchange_phases(double* ms, int n, int* valid) {
    if (!ms || n < 0) return -EINVAL;
    for (int k = 0; k < n && k < kPhases; k++) ms[k] = t_phase[k];
    if (valid) *valid = t_phase_valid;
    return 0;
}

extern "C" int shd_dev_exchange_runs(void* ws, const ShdTransport* x, const ShdDeliv* d_events,
                                     const uint32_t* d_dst_offsets, const uint32_t* host_bounds, ShdDeliv* d_recv,
                                     size_t recv_cap, ShdDeliv* d_out, uint32_t* d_out_offsets, size_t* n_out,
                                     void* stream) {
    const int W = x->world;
    if (W < 1 || W > kMaxWorld || x->rank < 0 || x->rank >= W) return shd_fail(-EINVAL, "bad world");
    const uint32_t Hm = host_bounds[x->rank + 1] - host_bounds[x->rank];
    void *dscr = nullptr, *hscr = nullptr;
    const int rc = shd_dev_ws_scratch(ws, 4 * xchg_scratch_words(host_bounds[W], W, Hm), 4 * (2 * kMaxWorld + 2),
                                      &dscr, &hscr); // (a failure still joins the first collective)
    return exchange_runs_core(ws, x, d_events, sizeof(ShdDeliv), 0, 1, d_dst_offsets, host_bounds, d_recv, recv_cap,
                              d_out, d_out_offsets, n_out, (hipStream_t)stream, static_cast<uint32_t*>(dscr),
                              static_cast<uint32_t*>(hscr), rc);
}

// A round decided and exchanged in one call (shd_round_process_exchange):
// the sender groups its decided events by destination without sorting them
// and ships 24-B wire records; the owners sort the union of what they get.
extern "C" int shd_dev_round_exchange(const ShdPktCtx* c, const ShdTransport* x, const ShdPkt* d_recs, size_t n,
                                      uint64_t barrier, uint64_t end_time, uint64_t bootstrap_end,
                                      const uint32_t* host_bounds, void* d_wire_send, uint8_t* d_status,
                                      uint64_t* d_counters, void* d_wire_recv, size_t recv_cap, ShdDeliv* d_out,
                                      uint32_t* d_out_offsets, size_t* n_out, void* stream) {
    const int W = x->world;
    if (W < 1 || W > kMaxWorld || x->rank < 0 || x->rank >= W) return shd_fail(-EINVAL, "bad world");
    const uint32_t H = c->nhosts, Hm = host_bounds[x->rank + 1] - host_bounds[x->rank];
    if (host_bounds[0] != 0 || host_bounds[W] != H) return shd_fail(-EINVAL, "host bounds must cover [0, %u)", H);
    const size_t words = ((size_t)H + 1) + xchg_scratch_words(H, W, Hm);
    void *dscr = nullptr, *hscr = nullptr;
    // (a failed local stage still joins the exchange's first collective)
    int rc = shd_dev_ws_scratch(c->ws, 4 * words, 4 * (2 * kMaxWorld + 2), &dscr, &hscr);
    uint32_t* d_off = static_cast<uint32_t*>(dscr); // the sender's destination offsets (H + 1)
    // Sorted wire runs (SHD_WIRE_SORTED=1/0 forces them on/off): by default
    // when an owner's destination would gather more than kSmallSeg events
    // from the W runs on average (W n / H) -- then its union is past the
    // one-wave rank sort and a merge of sorted runs is the cheaper side
    // (profiles/r04y_xchg_probe.log); below, the sender's sort costs more
    // than the owner's.  Ranks may choose differently: the owners merge
    // only when every run is sorted.
    // (a caller's transport takes the three-step exchange, whose owners sort
    // the wire runs anyway: no sender sort there)
    const bool own = x->allgatherv == rccl_allgatherv || x->allgatherv == local_allgatherv;
    const char* sw = getenv("SHD_WIRE_SORTED");
    const int sort_wire = !own                         ? 0
                          : sw && strcmp(sw, "1") == 0 ? 1
                          : sw && strcmp(sw, "0") == 0 ? 0
                                                       : (double)W * (double)n > 256.0 * (double)(H ? H : 1);
    // the split exchange (two send/recv groups overlapping the sender's second
    // half and the first owners' merge): the library's own transports, two
    // ranks or more; SHD_XCHG_SPLIT=0 keeps one group after the whole round.
    // (Every rank takes the same form: it depends on the transport, W and the
    // environment only.)
    const char* sp = getenv("SHD_XCHG_SPLIT");
    if (own && W >= 2 && !(sp && strcmp(sp, "0") == 0))
        return exchange_split(c, x, d_recs, n, barrier, end_time, bootstrap_end, host_bounds, d_wire_send, d_status,
                              d_counters, d_wire_recv, recv_cap, d_out, d_out_offsets, n_out, (hipStream_t)stream,
                              sort_wire);
    int sorted = 0;
    if (!rc)
        rc = shd_dev_packet_round_grouped(c, d_recs, n, barrier, end_time, bootstrap_end, d_wire_send, d_off, d_status,
                                          d_counters, stream, sort_wire, &sorted);
    return exchange_runs_core(c->ws, x, d_wire_send, 24, 1, sorted, d_off, host_bounds, d_wire_recv, recv_cap, d_out,
                              d_out_offsets, n_out, (hipStream_t)stream, rc ? nullptr : d_off + (H + 1),
                              static_cast<uint32_t*>(hscr), rc);
}

extern "C" int shd_dev_exchange_blocks(const ShdTransport* x, const void* d_send, const uint64_t* send_elems,
                                       size_t elem_bytes, void* d_recv, size_t recv_cap, size_t* n_recv,
                                       void* stream) {
    int rc = exchange_blocks(x, d_send, send_elems, elem_bytes, d_recv, recv_cap, n_recv, (hipStream_t)stream);
    if (!rc) rc = hip_status(hipStreamSynchronize((hipStream_t)stream), "exchange");
    return rc;
}

extern "C" int shd_transport_rccl_unique_id(void* id128) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    int rc = nccl_status(ncclGetUniqueId(&id), "ncclGetUniqueId");
    if (!rc) std::memcpy(id128, &id, sizeof id);
    return rc;
}

extern "C" int shd_transport_rccl_new(int rank, int world, const void* id128, int device, ShdTransport** out) {
    if (!out || !id128 || world < 1 || rank < 0 || rank >= world) return shd_fail(-EINVAL, "bad RCCL transport args");
    *out = nullptr;
    int rc = shd_dev_init(device);
    if (rc) return rc;
    Rccl* t = new (std::nothrow) Rccl();
    if (!t) return -ENOMEM;
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof id);
    t->device = device;
    if ((rc = hip_status(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking), "hipStreamCreate transport")) ||
        (rc = hip_status(hipMalloc((void**)&t->d_u64, 16 * (size_t)world), "hipMalloc transport")) ||
        (rc = hip_status(hipHostMalloc((void**)&t->h_u64, 16 * (size_t)world, hipHostMallocDefault),
                         "hipHostMalloc transport")) ||
        (rc = nccl_status(ncclCommInitRank(&t->comm, world, id, rank), "ncclCommInitRank"))) {
        (void)hipFree(t->d_u64);
        if (t->h_u64) (void)hipHostFree(t->h_u64);
        if (t->stream) (void)hipStreamDestroy(t->stream);
        delete t;
        return rc;
    }
    t->x.rank = rank;
    t->x.world = world;
    t->x.user = t;
    t->x.alltoall_u64 = rccl_alltoall_u64;
    t->x.alltoallv = rccl_alltoallv;
    t->x.allgatherv = rccl_allgatherv;
    *out = &t->x;
    return 0;
}

extern "C" void shd_transport_rccl_free(ShdTransport* x) {
    if (!x) return;
    Rccl* t = static_cast<Rccl*>(x->user);
    (void)ncclCommDestroy(t->comm);
    (void)hipFree(t->d_u64);
    if (t->h_u64) (void)hipHostFree(t->h_u64);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

// ---- in-process transports: one process, one thread and one topology per GPU ----
// (Shadow is one process with one manager, core/manager.c:543-577.)
//
// shd_transport_rccl_new_all: one RCCL communicator per device from
// ncclCommInitAll; the thread driving device k uses transport k.
//
// shd_transport_local_new: no RCCL at all -- the ranks are threads of this
// process, so a collective is a barrier plus device-to-device copies that
// each receiver pulls from the senders' published buffers (peer access over
// xGMI between GPUs, a plain copy on one GPU).  Used to rehearse the
// multi-rank rounds with threads on one GPU.
namespace {

struct LocalHub {
    int world;
    pthread_barrier_t bar;
    std::vector<uint64_t> u64;        // world x world count exchange
    std::vector<const char*> src;     // each rank's published send buffer
    std::vector<std::vector<uint64_t>> boff; // each rank's block offsets (alltoallv: per peer; allgatherv: per rank)
    int refs;
    pthread_mutex_t mu;
};

struct Local {
    ShdTransport x;
    LocalHub* hub;
    int device;
};

void hub_wait(LocalHub* h) { pthread_barrier_wait(&h->bar); }

int local_alltoall_u64(void* user, const uint64_t* send, uint64_t* recv) {
    Local* t = static_cast<Local*>(user);
    LocalHub* h = t->hub;
    const int W = h->world, me = t->x.rank;
    for (int r = 0; r < W; r++) h->u64[(size_t)me * W + r] = send[r];
    hub_wait(h);
    for (int r = 0; r < W; r++) recv[r] = h->u64[(size_t)r * W + me];
    hub_wait(h); // (the slots are reused by the next exchange)
    return 0;
}

// every rank publishes its send buffer and per-peer block offsets; each
// receiver copies its blocks out of the senders' buffers, in rank order
// (send_off: as rccl_alltoallv_off)
int local_alltoallv_off(void* user, const void* d_send, const uint64_t* send_bytes, const uint64_t* send_off,
                        void* d_recv, const uint64_t* recv_bytes, void* stream) {
    Local* t = static_cast<Local*>(user);
    LocalHub* h = t->hub;
    const int W = h->world, me = t->x.rank;
    hipStream_t s = (hipStream_t)stream;
    int rc = hip_status(hipStreamSynchronize(s), "local alltoallv (send side ready)");
    h->src[me] = static_cast<const char*>(d_send);
    // boff[me]: block r at [2r] (offset) and [2r + 1] (size)
    std::vector<uint64_t>& o = h->boff[me];
    o.assign(2 * (size_t)W, 0);
    uint64_t so = 0;
    for (int r = 0; r < W; r++) {
        o[2 * (size_t)r] = send_off ? send_off[r] : so;
        o[2 * (size_t)r + 1] = send_bytes[r];
        so += send_bytes[r];
    }
    hub_wait(h);
    uint64_t at = 0;
    for (int r = 0; r < W && !rc; r++) {
        if (recv_bytes[r] != h->boff[r][2 * (size_t)me + 1]) rc = shd_fail(-EIO, "local alltoallv: block sizes disagree");
        else if (recv_bytes[r])
            rc = hip_status(hipMemcpyAsync(static_cast<char*>(d_recv) + at, h->src[r] + h->boff[r][2 * (size_t)me],
                                           recv_bytes[r], hipMemcpyDefault, s),
                            "local alltoallv copy");
        at += recv_bytes[r];
    }
    if (!rc) rc = hip_status(hipStreamSynchronize(s), "local alltoallv");
    hub_wait(h); // (senders keep their buffers until every receiver copied)
    return rc;
}
int local_alltoallv(void* user, const void* d_send, const uint64_t* send_bytes, void* d_recv,
                    const uint64_t* recv_bytes, void* stream) {
    return local_alltoallv_off(user, d_send, send_bytes, nullptr, d_recv, recv_bytes, stream);
}

int local_allgatherv(void* user, void* d_buf, const uint64_t* off, void* stream) {
    Local* t = static_cast<Local*>(user);
    LocalHub* h = t->hub;
    const int W = h->world, me = t->x.rank;
    hipStream_t s = (hipStream_t)stream;
    int rc = hip_status(hipStreamSynchronize(s), "local allgatherv (block ready)");
    h->src[me] = static_cast<const char*>(d_buf);
    hub_wait(h);
    for (int r = 0; r < W && !rc; r++)
        if (r != me && off[r + 1] > off[r])
            rc = hip_status(hipMemcpyAsync(static_cast<char*>(d_buf) + off[r], h->src[r] + off[r], off[r + 1] - off[r],
                                           hipMemcpyDefault, s),
                            "local allgatherv copy");
    if (!rc) rc = hip_status(hipStreamSynchronize(s), "local allgatherv");
    hub_wait(h);
    return rc;
}

} // namespace

extern "C" int shd_transport_local_new(int world, ShdTransport** out) {
    if (!out || world < 1 || world > kMaxWorld) return shd_fail(-EINVAL, "bad local transport args");
    LocalHub* h = new (std::nothrow) LocalHub();
    if (!h) return -ENOMEM;
    h->world = world;
    h->u64.assign((size_t)world * world, 0);
    h->src.assign(world, nullptr);
    h->boff.assign(world, std::vector<uint64_t>(world + 1, 0));
    h->refs = world;
    if (pthread_barrier_init(&h->bar, nullptr, (unsigned)world) != 0) {
        delete h;
        return shd_fail(-EAGAIN, "pthread_barrier_init");
    }
    pthread_mutex_init(&h->mu, nullptr);
    for (int r = 0; r < world; r++) {
        Local* t = new (std::nothrow) Local();
        if (!t) return -ENOMEM; // (the transports made so far stay valid; the caller frees them)
        t->hub = h;
        t->device = -1;
        t->x.rank = r;
        t->x.world = world;
        t->x.user = t;
        t->x.alltoall_u64 = local_alltoall_u64;
        t->x.alltoallv = local_alltoallv;
        t->x.allgatherv = local_allgatherv;
        out[r] = &t->x;
    }
    return 0;
}

extern "C" void shd_transport_local_free(ShdTransport* x) {
    if (!x) return;
    Local* t = static_cast<Local*>(x->user);
    LocalHub* h = t->hub;
    pthread_mutex_lock(&h->mu);
    const int left = --h->refs;
    pthread_mutex_unlock(&h->mu);
    delete t;
    if (left == 0) {
        pthread_barrier_destroy(&h->bar);
        pthread_mutex_destroy(&h->mu);
        delete h;
    }
}

// One communicator per device of this process (ncclCommInitAll); transport
// k drives devices[k] and is used by the thread driving that device.
extern "C" int shd_transport_rccl_new_all(int ndev, const int* devices, ShdTransport** out) {
    if (!out || !devices || ndev < 1 || ndev > kMaxWorld) return shd_fail(-EINVAL, "bad RCCL transport args");
    std::vector<ncclComm_t> comms(ndev);
    int rc = nccl_status(ncclCommInitAll(comms.data(), ndev, devices), "ncclCommInitAll");
    if (rc) return rc;
    for (int k = 0; k < ndev; k++) out[k] = nullptr;
    int made = 0; // transports built so far (they own comms[0, made))
    for (int k = 0; k < ndev && !rc; k++) {
        if ((rc = shd_dev_init(devices[k]))) break;
        Rccl* t = new (std::nothrow) Rccl();
        if (!t) {
            rc = -ENOMEM;
            break;
        }
        t->device = devices[k];
        t->comm = comms[k];
        if ((rc = hip_status(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking), "hipStreamCreate transport")) ||
            (rc = hip_status(hipMalloc((void**)&t->d_u64, 16 * (size_t)ndev), "hipMalloc transport")) ||
            (rc = hip_status(hipHostMalloc((void**)&t->h_u64, 16 * (size_t)ndev, hipHostMallocDefault),
                             "hipHostMalloc transport"))) {
            (void)hipFree(t->d_u64);
            if (t->h_u64) (void)hipHostFree(t->h_u64);
            if (t->stream) (void)hipStreamDestroy(t->stream);
            delete t;
            break;
        }
        t->x.rank = k;
        t->x.world = ndev;
        t->x.user = t;
        t->x.alltoall_u64 = rccl_alltoall_u64;
        t->x.alltoallv = rccl_alltoallv;
        t->x.allgatherv = rccl_allgatherv;
        out[k] = &t->x;
        made = k + 1;
    }
    if (rc) { // all or nothing: free what was built and the communicators no transport took
        for (int k = 0; k < made; k++) {
            shd_transport_rccl_free(out[k]);
            out[k] = nullptr;
        }
        for (int k = made; k < ndev; k++) (void)ncclCommDestroy(comms[k]);
    }
    return rc;
}

namespace {
__global__ __launch_bounds__(256) void k_gather_entries(const ShdEntry* __restrict__ tab,
                                                        const uint64_t* __restrict__ idx, size_t n,
                                                        ShdEntry* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = tab[idx[i]];
}
} // namespace

extern "C" int shd_dev_gather_entries(const ShdEntry* tab, const uint64_t* d_idx, size_t n, ShdEntry* d_out) {
    if (!n) return 0;
    const size_t g = (n + 255) / 256;
    hipLaunchKernelGGL(k_gather_entries, dim3(g < 4096 ? g : 4096), dim3(256), 0, nullptr, tab, d_idx, n, d_out);
    int rc = hip_status(hipGetLastError(), "k_gather_entries launch");
    return rc ? rc : hip_status(hipDeviceSynchronize(), "k_gather_entries");
}

extern "C" int shd_memcpy(void* dst, const void* src, size_t bytes) {
    return bytes ? hip_status(hipMemcpy(dst, src, bytes, hipMemcpyDefault), "hipMemcpy") : 0;
}
