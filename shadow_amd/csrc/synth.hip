// synth.hip -- the load generator of the simulated rounds (benchmarks and
// tests; it stands in for the hosts' applications, which are out of scope --
// SURVEY.md §8 -- and is not part of the hand-off itself).
//
// One round: every sender k of a pool sends m packets.  Packet j of sender k
// reserves the sender's j-th rand_r draw of the round (worker.c:540-541: one
// draw per packet, reserved at send time): its record carries the pre-state
// of that draw, and the sender's state after the round (m draws further) is
// carried to the next round -- a device array, like the hosts' random
// streams.  Destinations, send times and payload sizes come from a
// splitmix64 hash of (seed, round, sender, j), so a round's records are a
// pure function of the carried state and the round index; tests restate the
// generator in numpy (shadow_amd.synth.synth_sends) and compare records bit
// for bit.  Send times: packet j of a sender in the j-th of m equal slices of
// the window [t0, t0 + window), in send order (a host sends in time order).
#include <hip/hip_runtime.h>

#include <cerrno>

#include "shd_internal.h"

namespace {

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// one glibc rand_r call's effect on the state (random.c:32-43 -> rand_r)
__device__ __forceinline__ uint32_t rand_r_advance(uint32_t s) {
    s = s * 1103515245u + 12345u;
    s = s * 1103515245u + 12345u;
    return s * 1103515245u + 12345u;
}

__global__ __launch_bounds__(256) void k_synth_sends(const uint32_t* __restrict__ pool, uint32_t npool, uint32_t m,
                                                     uint64_t key, uint64_t t0, uint64_t window,
                                                     const uint32_t* __restrict__ dst_pool, uint32_t ndst,
                                                     const uint32_t* __restrict__ st_in, uint32_t* __restrict__ st_out,
                                                     const uint64_t* __restrict__ seq_in, uint64_t* __restrict__ seq_out,
                                                     ShdPkt* __restrict__ recs) {
    const size_t n = (size_t)npool * m;
    const uint64_t slice = window / m;
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x) {
        const uint32_t k = (uint32_t)(p / m), j = (uint32_t)(p % m);
        const uint32_t h = pool[k];
        uint32_t s = st_in[k];
        for (uint32_t i = 0; i < j; i++) s = rand_r_advance(s);
        const unsigned long long x = mix64(key + p);
        uint32_t di = (uint32_t)(x % ndst);
        uint32_t d = dst_pool ? dst_pool[di] : di;
        if (d == h && ndst > 1) {
            di = di + 1 == ndst ? 0u : di + 1;
            d = dst_pool ? dst_pool[di] : di;
        }
        ShdPkt r;
        r.now = t0 + (uint64_t)j * slice + (slice ? (x >> 32) % slice : 0);
        r.seq = seq_in[k] + j;
        r.src_host = h;
        r.dst_host = d;
        r.rng_state = s;
        r.payload_len = ((x >> 16) & 1023u) < 922u ? 1448u : 0u; // ~90 % carry a payload (C3's 1448 B)
        recs[p] = r;
        if (j == m - 1) { // the sender's carried state: m draws further
            st_out[k] = rand_r_advance(s);
            seq_out[k] = seq_in[k] + m;
        }
    }
}

} // namespace

extern "C" int shd_synth_sends_device(const uint32_t* d_pool, uint32_t npool, uint32_t m, uint32_t round,
                                      uint64_t seed, uint64_t t0, uint64_t window_ns, const uint32_t* d_dst_pool,
                                      uint32_t ndst, const uint32_t* d_state_in, uint32_t* d_state_out,
                                      const uint64_t* d_seq_in, uint64_t* d_seq_out, ShdPkt* d_recs, void* stream) {
    if (!npool || !m) return 0;
    if (!d_pool || !ndst || !d_state_in || !d_state_out || !d_seq_in || !d_seq_out || !d_recs)
        return shd_fail(-EINVAL, "bad synthetic-send arguments");
    // the carried states are read by every packet's thread while the last one
    // of each sender writes them: input and output arrays must not overlap
    auto overlap = [npool](const void* a, const void* b, size_t elem) {
        const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b, len = (uintptr_t)npool * elem;
        return x < y + len && y < x + len;
    };
    if (overlap(d_state_in, d_state_out, 4) || overlap(d_seq_in, d_seq_out, 8))
        return shd_fail(-EINVAL, "synthetic sends: the carried state arrays in and out overlap");
    const size_t n = (size_t)npool * m;
    const size_t g = (n + 255) / 256;
    // the round's hash key: seed and round index spread apart (splitmix64 of both)
    const uint64_t key = seed * 0xD1B54A32D192ED03ull + (uint64_t)round * 0x8CB92BA72F3D8DD7ull;
    hipLaunchKernelGGL(k_synth_sends, dim3((unsigned)(g < 65536 ? g : 65536)), dim3(256), 0, (hipStream_t)stream,
                       d_pool, npool, m, key, t0, window_ns, d_dst_pool, ndst, d_state_in, d_state_out, d_seq_in,
                       d_seq_out, d_recs);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : shd_fail(-EIO, "k_synth_sends launch: %s", hipGetErrorString(e));
}
