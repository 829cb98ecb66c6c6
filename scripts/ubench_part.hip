// ubench_part.hip -- design probe for the packet-scatter kernel (dev tool).
// The C3 shapes: 10M 32-B records over 100k hosts, an A = 19,870 table of
// 8-B {delay_ns, keep threshold} entries (3.16 GB), the glibc rand_r draw,
// the drop rule and the barrier clamp.  What differs is where a delivered
// event goes:
//   ref0   nowhere (status + decision only): the gather floor
//   ref1   the product's slab form: slot = atomicAdd(cnt[dst]), one random
//          16-B store into a 205 MB per-destination slab
//   part   LDS-staged partition: a workgroup decides CH records, stages the
//          delivered events in LDS, counts them per destination BUCKET of
//          2^BS hosts, reserves one run per nonempty bucket with one atomic,
//          and writes its runs in bucket order (consecutive lanes store
//          consecutive 16-B records)
//   b0     the partition's second half: one workgroup per bucket moves its
//          events into the per-destination slab with LDS counters (the slab
//          lines of a bucket are written by one workgroup, back to back)
// Sanity: the per-destination counts of ref1 and part+b0 must be equal.
// Prints the median of 9 timed launches (resets outside the timed region).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

struct Pkt {
    unsigned long long now, seq;
    unsigned src, dst, rng, pay;
};

constexpr size_t kN = 10000000;
constexpr unsigned kH = 100000, kA = 19870, kSlab = 128;
constexpr unsigned long long kBarrier = 110000000ull, kTbase = kBarrier - (1ull << 31);

__device__ __forceinline__ unsigned rand_r_dev(unsigned s) {
    unsigned next = s;
    int result;
    next = next * 1103515245u + 12345u;
    result = (int)((next / 65536u) % 2048u);
    next = next * 1103515245u + 12345u;
    result = (result << 10) ^ (int)((next / 65536u) % 1024u);
    next = next * 1103515245u + 12345u;
    result = (result << 10) ^ (int)((next / 65536u) % 1024u);
    return (unsigned)result;
}

__device__ __forceinline__ Pkt ld_pkt(const Pkt* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    Pkt r;
    r.now = ((unsigned long long)a.y << 32) | a.x;
    r.seq = ((unsigned long long)a.w << 32) | a.z;
    r.src = b.x;
    r.dst = b.y;
    r.rng = b.z;
    r.pay = b.w;
    return r;
}

// the decision of worker.c:545-549 + host_single.c:187-192 on an 8-B entry
__device__ __forceinline__ bool decide(const Pkt& p, uint2 q, unsigned long long* t) {
    const unsigned r = rand_r_dev(p.rng);
    const bool keep = r <= q.y || p.pay == 0;
    unsigned long long tt = p.now + q.x;
    if (p.src != p.dst && tt < kBarrier) tt = kBarrier;
    *t = tt;
    return keep;
}

__device__ __forceinline__ uint2 gather(const uint2* __restrict__ ptab, size_t i) {
    const unsigned long long v = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(ptab) + i);
    return make_uint2((unsigned)v, (unsigned)(v >> 32));
}

// ---- reference forms: the product's chunked 256-thread scatter ----
template <int MODE>
__global__ __launch_bounds__(256) void k_ref(const Pkt* __restrict__ recs, size_t n, const uint2* __restrict__ hinfo,
                                             const uint2* __restrict__ ptab, size_t chunk, unsigned* __restrict__ cnt,
                                             uint4* __restrict__ cslab, unsigned char* __restrict__ st,
                                             unsigned long long* __restrict__ mnout) {
    constexpr int kB = 4;
    const size_t beg = (size_t)blockIdx.x * chunk, end = beg + chunk < n ? beg + chunk : n;
    unsigned long long mn = ~0ull;
    for (size_t b0 = beg; b0 < end; b0 += 256 * kB) {
        Pkt p[kB];
        bool live[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const size_t i = b0 + (size_t)k * 256 + threadIdx.x;
            live[k] = i < end;
            if (live[k]) p[k] = ld_pkt(&recs[i]);
        }
        uint2 hs[kB], hd[kB];
#pragma unroll
        for (int k = 0; k < kB; k++)
            if (live[k]) hs[k] = hinfo[p[k].src], hd[k] = hinfo[p[k].dst];
        uint2 q[kB];
#pragma unroll
        for (int k = 0; k < kB; k++)
            if (live[k]) {
                unsigned oi = hs[k].x, oj = hd[k].x;
                if (oi != oj && hd[k].y < hs[k].y) oi = hd[k].x, oj = hs[k].x;
                q[k] = gather(ptab, (size_t)oi * kA + oj);
            }
#pragma unroll
        for (int k = 0; k < kB; k++) {
            if (!live[k]) continue;
            const size_t i = b0 + (size_t)k * 256 + threadIdx.x;
            unsigned long long t;
            const bool d = decide(p[k], q[k], &t);
            st[i] = d ? 1 : 2;
            if (d) {
                mn = t < mn ? t : mn;
                if (MODE == 1) {
                    const unsigned s = atomicAdd(&cnt[p[k].dst], 1u);
                    if (s < kSlab)
                        cslab[(size_t)p[k].dst * kSlab + s] =
                            make_uint4((unsigned)(t - kTbase), p[k].src, (unsigned)i, (unsigned)p[k].seq);
                }
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(mn, o);
        mn = v < mn ? v : mn;
    }
    if ((threadIdx.x & 63) == 0 && mn != ~0ull) atomicMin(mnout, mn);
}

// ---- partitioned form ----
template <int WG>
__device__ void block_scan(const unsigned* hist, unsigned* lofs, unsigned nb, unsigned* wsum) {
    const unsigned per = (nb + WG - 1) / WG, b0 = threadIdx.x * per;
    unsigned s = 0;
    for (unsigned k = 0; k < per && b0 + k < nb; k++) s += hist[b0 + k];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = (unsigned)__shfl_up((int)inc, o);
        if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    unsigned pre = inc - s;
    for (int k = 0; k < w; k++) pre += wsum[k];
    for (unsigned k = 0; k < per && b0 + k < nb; k++) {
        lofs[b0 + k] = pre;
        pre += hist[b0 + k];
    }
    if (threadIdx.x == WG - 1) lofs[nb] = pre;
}

template <int WG, int CH, int BS>
__global__ __launch_bounds__(WG) void k_part(const Pkt* __restrict__ recs, size_t n, const uint2* __restrict__ hinfo,
                                             const uint2* __restrict__ ptab, unsigned nb, size_t cap,
                                             unsigned* __restrict__ gcnt, uint4* __restrict__ stage,
                                             unsigned char* __restrict__ st, unsigned long long* __restrict__ mnout,
                                             unsigned* __restrict__ novf) {
    extern __shared__ uint4 smem[];
    uint4* ev = smem;                                            // CH staged events {t_off, src, seq, dst}
    uint16_t* rk = reinterpret_cast<uint16_t*>(ev + CH);         // CH ranks inside their bucket
    uint16_t* perm = rk + CH;                                    // CH: bucket order -> staged slot
    unsigned* hist = reinterpret_cast<unsigned*>(perm + CH);     // nb
    unsigned* lofs = hist + nb;                                  // nb + 1
    unsigned* gb = lofs + nb + 1;                                // nb
    unsigned* wsum = gb + nb;                                    // WG / 64
    __shared__ unsigned long long wmin[WG / 64];
    for (unsigned b = threadIdx.x; b < nb; b += WG) hist[b] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * CH;
    unsigned long long mn = ~0ull;
    constexpr int kB = 4;
    static_assert(CH % (WG * kB) == 0, "chunk");
    for (int k0 = 0; k0 < CH / WG; k0 += kB) {
        Pkt p[kB];
        bool live[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const size_t i = base + (size_t)(k0 + k) * WG + threadIdx.x;
            live[k] = i < n;
            if (live[k]) p[k] = ld_pkt(&recs[i]);
        }
        uint2 hs[kB], hd[kB];
#pragma unroll
        for (int k = 0; k < kB; k++)
            if (live[k]) hs[k] = hinfo[p[k].src], hd[k] = hinfo[p[k].dst];
        uint2 q[kB];
#pragma unroll
        for (int k = 0; k < kB; k++)
            if (live[k]) {
                unsigned oi = hs[k].x, oj = hd[k].x;
                if (oi != oj && hd[k].y < hs[k].y) oi = hd[k].x, oj = hs[k].x;
                q[k] = gather(ptab, (size_t)oi * kA + oj);
            }
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const unsigned li = (unsigned)((k0 + k) * WG + threadIdx.x);
            uint4 e = make_uint4(0u, 0u, 0u, ~0u);
            if (live[k]) {
                unsigned long long t;
                const bool d = decide(p[k], q[k], &t);
                st[base + li] = d ? 1 : 2;
                if (d) {
                    mn = t < mn ? t : mn;
                    rk[li] = (uint16_t)atomicAdd(&hist[p[k].dst >> BS], 1u);
                    e = make_uint4((unsigned)(t - kTbase), p[k].src, (unsigned)p[k].seq, p[k].dst);
                }
            }
            ev[li] = e;
        }
    }
    __syncthreads();
    block_scan<WG>(hist, lofs, nb, wsum);
    for (unsigned b = threadIdx.x; b < nb; b += WG) {
        const unsigned c = hist[b];
        gb[b] = c ? atomicAdd(&gcnt[b], c) : 0u;
    }
    __syncthreads();
    for (unsigned li = threadIdx.x; li < CH; li += WG) {
        const unsigned w = ev[li].w;
        if (w != ~0u) perm[lofs[w >> BS] + rk[li]] = (uint16_t)li;
    }
    __syncthreads();
    const unsigned total = lofs[nb];
    constexpr unsigned kMask = (1u << BS) - 1u;
    for (unsigned p = threadIdx.x; p < total; p += WG) {
        const unsigned li = perm[p];
        const uint4 e = ev[li];
        const unsigned b = e.w >> BS;
        const size_t j = (size_t)gb[b] + (p - lofs[b]);
        if (j < cap) stage[(size_t)b * cap + j] = make_uint4(e.x, e.z, (unsigned)(base + li), (e.y << BS) | (e.w & kMask));
        else atomicAdd(novf, 1u);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(mn, o);
        mn = v < mn ? v : mn;
    }
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int k = 1; k < WG / 64; k++) m = wmin[k] < m ? wmin[k] : m;
        if (m != ~0ull) atomicMin(mnout, m);
    }
}

template <int BS>
__global__ __launch_bounds__(1024) void k_b0(const uint4* __restrict__ stage, size_t cap, const unsigned* __restrict__ gcnt,
                                             unsigned* __restrict__ cnt1, uint4* __restrict__ cslab) {
    __shared__ unsigned c[1u << BS];
    constexpr unsigned kMask = (1u << BS) - 1u;
    const unsigned b = blockIdx.x;
    for (unsigned j = threadIdx.x; j <= kMask; j += 1024) c[j] = 0;
    __syncthreads();
    const unsigned nb_ev = min(gcnt[b], (unsigned)cap);
    const uint4* s = stage + (size_t)b * cap;
    for (unsigned j0 = threadIdx.x; j0 < nb_ev; j0 += 4096) {
        uint4 e[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (j0 + k * 1024 < nb_ev) e[k] = s[j0 + k * 1024];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (j0 + k * 1024 >= nb_ev) continue;
            const unsigned dl = e[k].w & kMask, d = (b << BS) + dl;
            const unsigned r = atomicAdd(&c[dl], 1u);
            if (r < kSlab) cslab[(size_t)d * kSlab + r] = make_uint4(e[k].x, e[k].w >> BS, e[k].z, e[k].y);
        }
    }
    __syncthreads();
    for (unsigned j = threadIdx.x; j <= kMask; j += 1024)
        if ((b << BS) + j < kH) cnt1[(b << BS) + j] = c[j];
}

__global__ void k_fill_ptab(uint2* t, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        t[i] = make_uint2((unsigned)(1000000u * (1u + (unsigned)(i % 97u))), 1975684956u); // 0.92 x 2^31
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
    }
    template <typename P, typename F>
    float run(P prep, F launch) {
        std::vector<float> ts;
        for (int r = 0; r < 10; r++) {
            prep();
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (r) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return ts[ts.size() / 2];
    }
};

int main() {
    std::vector<Pkt> hp(kN);
    unsigned long long s = 88172645463325252ull;
    auto rnd = [&]() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    };
    for (size_t i = 0; i < kN; i++)
        hp[i] = Pkt{100000000ull + rnd() % 10000000ull, i / 100, (unsigned)(rnd() % kH), (unsigned)(rnd() % kH),
                    (unsigned)rnd(), 1u};
    std::vector<uint2> hi(kH);
    for (unsigned h = 0; h < kH; h++) hi[h] = make_uint2((unsigned)(rnd() % kA), (unsigned)rnd());
    Pkt* recs;
    uint2 *hinfo, *ptab;
    unsigned char* st;
    unsigned *cnt, *cnt1, *gcnt, *novf;
    uint4 *cslab, *stage;
    unsigned long long* mn;
    CHECK(hipMalloc(&recs, kN * sizeof(Pkt)));
    CHECK(hipMemcpy(recs, hp.data(), kN * sizeof(Pkt), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&hinfo, kH * 8));
    CHECK(hipMemcpy(hinfo, hi.data(), kH * 8, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&ptab, (size_t)kA * kA * 8));
    hipLaunchKernelGGL(k_fill_ptab, dim3(8192), dim3(256), 0, 0, ptab, (size_t)kA * kA);
    CHECK(hipMalloc(&st, kN));
    CHECK(hipMalloc(&cnt, kH * 4));
    CHECK(hipMalloc(&cnt1, kH * 4));
    CHECK(hipMalloc(&gcnt, 4096 * 4));
    CHECK(hipMalloc(&novf, 4));
    CHECK(hipMalloc(&mn, 8));
    CHECK(hipMalloc(&cslab, (size_t)kH * kSlab * 16));
    const size_t stage_ent = 2 * kN + (1u << 22);
    CHECK(hipMalloc(&stage, stage_ent * 16));
    CHECK(hipDeviceSynchronize());
    Timer tm;
    const size_t chunk = ((kN + 1535) / 1536 + 255) / 256 * 256;
    const unsigned nch = (unsigned)((kN + chunk - 1) / chunk);
    auto reset_ref = [&] {
        CHECK(hipMemsetAsync(cnt, 0, kH * 4));
        CHECK(hipMemsetAsync(mn, 0xff, 8));
    };
    float t0 = tm.run(reset_ref, [&] {
        hipLaunchKernelGGL(k_ref<0>, dim3(nch), dim3(256), 0, 0, recs, kN, hinfo, ptab, chunk, cnt, cslab, st, mn);
    });
    printf("ref0 gather floor (decide + status)          %.4f ms\n", t0);
    float t1 = tm.run(reset_ref, [&] {
        hipLaunchKernelGGL(k_ref<1>, dim3(nch), dim3(256), 0, 0, recs, kN, hinfo, ptab, chunk, cnt, cslab, st, mn);
    });
    printf("ref1 slab (atomic + random 16-B store)       %.4f ms\n", t1);
    fflush(stdout);
    std::vector<unsigned> want(kH), got(kH);
    CHECK(hipMemcpy(want.data(), cnt, kH * 4, hipMemcpyDeviceToHost));
    unsigned long long delivered = 0;
    for (unsigned v : want) delivered += v;
    printf("delivered %llu of %zu\n", delivered, kN);

#define PART(WG, CH, BS)                                                                                               \
    do {                                                                                                               \
        const unsigned nb = (kH + (1u << BS) - 1) >> BS;                                                               \
        const size_t cap = std::min<size_t>((size_t)(kN / nb) * 5 / 4 + 4096, stage_ent / nb);                        \
        const size_t lds = (size_t)CH * 20 + 4 * (3 * (size_t)nb + 1) + 4 * (WG / 64);                                 \
        CHECK(hipFuncSetAttribute((const void*)k_part<WG, CH, BS>, hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                  (int)lds));                                                                          \
        const unsigned g = (unsigned)((kN + CH - 1) / CH);                                                             \
        auto reset = [&] {                                                                                             \
            CHECK(hipMemsetAsync(gcnt, 0, 4096 * 4));                                                                  \
            CHECK(hipMemsetAsync(novf, 0, 4));                                                                         \
            CHECK(hipMemsetAsync(mn, 0xff, 8));                                                                        \
        };                                                                                                             \
        float ta = tm.run(reset, [&] {                                                                                 \
            hipLaunchKernelGGL((k_part<WG, CH, BS>), dim3(g), dim3(WG), lds, 0, recs, kN, hinfo, ptab, nb, cap, gcnt,  \
                               stage, st, mn, novf);                                                                   \
        });                                                                                                            \
        float tb = tm.run([] {}, [&] {                                                                                 \
            hipLaunchKernelGGL(k_b0<BS>, dim3(nb), dim3(1024), 0, 0, stage, cap, gcnt, cnt1, cslab);                   \
        });                                                                                                            \
        CHECK(hipMemcpy(got.data(), cnt1, kH * 4, hipMemcpyDeviceToHost));                                             \
        unsigned ov = 0;                                                                                               \
        CHECK(hipMemcpy(&ov, novf, 4, hipMemcpyDeviceToHost));                                                         \
        printf("part WG=%4d CH=%5d BS=%d (%4u buckets, %5.1f events/run, LDS %6zu B): part %.4f ms  b0 %.4f ms  "     \
               "sum %.4f  counts %s  ovf %u\n",                                                                        \
               WG, CH, BS, nb, (double)delivered / g / nb, lds, ta, tb, ta + tb, got == want ? "match" : "DIFFER", ov); \
        fflush(stdout);                                                                                                \
    } while (0)
    PART(256, 1024, 8);
    PART(256, 2048, 8);
    PART(512, 2048, 8);
    PART(512, 4096, 8);
    PART(512, 4096, 9);
    PART(1024, 4096, 8);
    PART(1024, 4096, 9);
    PART(1024, 4096, 10);
    PART(512, 6144, 9);
    CHECK(hipDeviceSynchronize());
    return 0;
}
