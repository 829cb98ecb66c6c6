// routing.hip -- routing-table rows on gfx950.
//
// Both SSSP kernels run igraph 0.8's get_shortest_paths_dijkstra exactly,
// one 64-lane wave per source (routing/topology.c:1682 -> igraph
// structural_properties.c): indexed binary max-heap on -dist (igraph_2wheap:
// shift-up swaps while !(x < parent), sink prefers the left child when
// left >= right, modify = sink then shift-up at the original position,
// delete_max = swap root/last, pop, sink), incidence lists in
// igraph_incident(mode OUT) order, "first finite distance" -> push,
// "alt < cur" -> modify, early exit once every attached vertex is popped.
// Reliability is folded along the final parent chain exactly as
// _topology_computePathProperties multiplies it (topology.c:1308-1365): the
// last improvement of v fixes rel[v] = rel[u] * (1 - loss(u,v)) with rel[u]
// already final because u was popped.  Results are therefore bit-identical
// to the reference, ties included, with no CPU fallback.
//
// Parallel structure: sources are independent (one wave each, as many in
// flight as the CUs hold); within a pop the wave relaxes 64 incident edges
// per step (coalesced CSR reads, gathered dist reads), a ballot collects the
// improving lanes and the wave applies their updates in incidence order (the
// order igraph applies them) with uniform control flow.  Every heap,
// distance and reliability store inside the pop loop is made by all 64 lanes
// with the same address and value, so each lane reads back its own writes in
// program order and the loop needs no barrier.
//
//  * k_sssp_lds (V <= kLdsMaxV, the dense C1 graphs): everything in LDS
//    (36 B per vertex), one wave per block, 16 batches of 64 incident edges
//    in flight per pop.
//  * k_sssp_slab (larger graphs): a private HBM slab per wave (heap, {dist,
//    rel} records, pos), heap positions [0, kTop) in LDS, persistent waves.
//    A row is a chain of dependent memory round trips (~1-2 us each under
//    load), so the pop is arranged to overlap them: the root node carries
//    the start of its vertex's sentinel-terminated incidence list, so the
//    edge loads of u, the removal's last-node load and rel[u] are issued
//    together the moment u is known, the neighbours' distance gathers are
//    issued as soon as the edges arrive, and the sink's HBM block loads
//    then wait behind them -- the relaxation data is in registers when the
//    sink ends.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <cstdio>

#include "shd_internal.h"

namespace {

constexpr int kTopDefault = 256; // heap positions in LDS for the slab kernel (levels 0..7)
constexpr int kSlabWaves = 4;   // independent waves per slab-kernel block
constexpr int kWavesPerCU = 32; // gfx950: resident waves per CU
constexpr int kLdsMaxV = 4096;  // 36 B per vertex -> 144 KiB of the 160 KiB LDS
constexpr int kSinkLevels = 5;  // heap levels loaded per sink block (62 nodes, one per lane)

// so: in the slab kernel, the start of v's list in the sentinel-terminated
// incidence arrays (g.snb / g.swr); unused by the LDS kernel
struct __attribute__((aligned(16))) HNode {
    double key; // -dist
    int v;
    int so;
};

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ double uni_d(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ HNode uni_n(const HNode& x) { return HNode{uni_d(x.key), uni(x.v), uni(x.so)}; }

// igraph_2wheap over split storage.  kAll: every position in LDS (top).
// Else positions < kTop in LDS and position p >= kTop at rest[p + 1], which
// puts each child pair (2e+1, 2e+2) in one 32-B sector.
//
// pos (igraph's index2, vertex -> position + 2) is what a decrease-key needs
// to find a vertex.  In the slab kernel every pos store is one random HBM
// request and a sink moves a node at every level it passes, most of them in
// the LDS top; so there pos of a node in the LDS top is the marker 1
// ("somewhere in the top"), written only when the node enters the top, and
// a decrease-key of such a node finds it by a wave-wide search of the (at
// most kTop) top positions.  The slab kernel's pop does not clear pos: a
// popped vertex is never decreased again (alt = dist[u] + w >= dist[v] for
// every popped v, weights > 0).  Neither changes a heap operation.
// kDp: sink and shift-up by the data-parallel block forms (sink_dp,
// shift_up_dp) rather than level by level; always on for the slab kernel.
template <bool kAll, int kTop = kTopDefault, bool kDp = !kAll>
struct Heap {
    HNode* top;
    HNode* rest;
    int* pos; // vertex -> position + 2 (slab: 1 = in the LDS top)
    int n;
    int lane;

    // the node at p as loaded (per lane); the slab kernel makes it uniform
    // with uni_n only where it is used, so that the load can be issued early
    __device__ __forceinline__ HNode ld_raw(int p) const {
        HNode x;
        // (distinct asm markers after each access keep the compiler from
        // sinking the LDS and the global access into one flat access)
        if (kAll || p < kTop) {
            x = top[p];
            if (!kAll) __asm__ volatile("; heap lds" ::: "memory");
        } else {
            x = rest[p + 1];
            __asm__ volatile("; heap hbm" ::: "memory");
        }
        return x;
    }
    // every heap operand is wave-uniform: readfirstlane tells the compiler
    // so, and the heap then runs on scalar branches with LDS- or
    // global-specific accesses (not exec-masked flat ones)
    __device__ __forceinline__ HNode ld(int p) const {
        if (kAll) return ld_raw(p); // (the LDS kernel is faster without the readfirstlanes)
        return uni_n(ld_raw(p));
    }
    // stores node x at position p; `from` = its previous position (-1: new)
    __device__ __forceinline__ void st(int p, const HNode& x, int from) {
        if (kAll || p < kTop) {
            top[p] = x;
            if (!kAll) __asm__ volatile("; heap lds st" ::: "memory");
        } else {
            rest[p + 1] = x;
            __asm__ volatile("; heap hbm st" ::: "memory");
        }
        if (kAll || p >= kTop) {
            if (p != from) pos[x.v] = p + 2;
        } else if (from < 0 || from >= kTop) {
            pos[x.v] = 1; // entered the LDS top
        }
    }
    // climb while !(x < parent); x was at position `from` (-1: new)
    __device__ __forceinline__ void shift_up(int e, const HNode& x, int from) {
        while (e > 0) {
            const int p = ((e + 1) >> 1) - 1;
            const HNode pn = ld(p);
            if (x.key < pn.key) break;
            st(e, pn, p);
            e = p;
        }
        st(e, x, from);
    }
    // Shift-up, data-parallel (slab kernel): lane j loads the j-th ancestor
    // of e -- at most 2 from the HBM slab per round (a climb is usually 0-2
    // levels), every LDS one up to the root -- and one ballot says which
    // ancestors x is not smaller than.  The heap order makes that set the
    // nearest c ancestors (parent >= child all the way up), so x climbs c
    // levels: those ancestors each move one level down along the path, by
    // their own lanes in one store (+ one for pos), exactly the moves of
    // shift_up.
    __device__ __forceinline__ void shift_up_dp(int e, const HNode& x, int from) {
        for (;;) {
            if (e == 0) break;
            const int lvl = 31 - __builtin_clz((unsigned)e + 1); // ancestors of e: lvl
            constexpr int kTopLv = kTop >= 512 ? 9 : 8;          // levels wholly in the LDS top
            const int nh = lvl > kTopLv ? lvl - kTopLv : 0;      // ancestors at deeper levels (slab)
            const int K = (!kAll && nh > 2) ? 2 : lvl;           // loaded this round
            const int a = ((e + 1) >> (lane + 1)) - 1;           // lane's ancestor
            const bool ld = lane < K;
            HNode c = HNode{0.0, 0, 0};
            if (ld) {
                if (kAll || a < kTop) {
                    c = top[a];
                    __asm__ volatile("; up lds" ::: "memory");
                } else {
                    c = rest[a + 1];
                    __asm__ volatile("; up hbm" ::: "memory");
                }
            }
            const unsigned long long m = __ballot(ld && !(x.key < c.key)); // x climbs past these
            const int cnt = (int)__builtin_ctzll(~m);
            if (lane < cnt) { // each passed ancestor moves one level down the path
                const int d = ((e + 1) >> lane) - 1;
                if (kAll) {
                    top[d] = c;
                    pos[c.v] = d + 2;
                } else if (d < kTop) {
                    top[d] = c;
                    __asm__ volatile("; up mv lds" ::: "memory");
                } else {
                    rest[d + 1] = c;
                    __asm__ volatile("; up mv hbm" ::: "memory");
                    pos[c.v] = d + 2;
                }
            }
            if (cnt == 0) break;
            e = ((e + 1) >> cnt) - 1;
            if (cnt < K) break;
        }
        st(e, x, from);
    }
    // descend towards the larger child (the left one when left >= right)
    // while x < child, one level at a time
    __device__ __forceinline__ void sink_seq(int e, const HNode& x, int from) {
        for (;;) {
            const int l = 2 * e + 1;
            if (l >= n) break;
            HNode c = ld(l);
            int ci = l;
            if (l + 1 < n) { // (the right child exists: never read past the heap)
                const HNode r = ld(l + 1);
                if (!(c.key >= r.key)) c = r, ci = l + 1;
            }
            if (!(x.key < c.key)) break;
            st(e, c, ci);
            e = ci;
        }
        st(e, x, from);
    }
    // Sink by blocks, data-parallel (slab kernel): the 62 nodes of the next
    // 5 levels under e are loaded one per lane as in sink_blocks; the lanes
    // then make every level's comparisons at once -- each left child lane
    // compares with its sibling (DPP swap), every lane compares with x --
    // and three ballots hand the scalar unit what the sequential walk would
    // read: which children exist, which sibling is the larger one (the left
    // on equality), which children x is smaller than.  The walk down the
    // larger children is then a few scalar bit operations per level, and the
    // nodes it moves are stored by their own lanes, each one level up, in one
    // store instruction (plus one for their pos).  Same moves as sink_seq.
    __device__ __forceinline__ void sink_dp(int e, const HNode& x, int from) {
        const int j = 31 - __builtin_clz((unsigned)lane + 2); // this lane's level under e (1..5)
        const int bi = lane + 2 - (1 << j);                    // ... and index in that level
        const bool inblk = lane < (2 << kSinkLevels) - 2;
        for (;;) {
            if (2 * e + 1 >= n) break;
            const int p = (e + 1) * (1 << j) - 1 + bi;
            const bool valid = inblk && p < n;
            HNode c = HNode{0.0, 0, 0};
            // (uniform tests first: a block is wholly in LDS or in the slab
            // except the one that straddles kTop)
            if (kAll || 32 * e + 62 < kTop) {
                if (valid) c = top[p];
                __asm__ volatile("; sink lds" ::: "memory");
            } else if (2 * e + 1 >= kTop) {
                if (valid) c = rest[p + 1];
                __asm__ volatile("; sink hbm" ::: "memory");
            } else if (valid) {
                if (p < kTop) {
                    c = top[p];
                    __asm__ volatile("; sink lds/hbm" ::: "memory");
                } else {
                    c = rest[p + 1];
                    __asm__ volatile("; sink hbm/lds" ::: "memory");
                }
            }
            // the sibling's key: quad_perm(1, 0, 3, 2) swaps lanes 2i, 2i + 1
            const long long kb = __double_as_longlong(c.key);
            const unsigned slo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(kb & 0xffffffffll), 0xB1, 0xF, 0xF, false);
            const unsigned shi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(kb >> 32), 0xB1, 0xF, 0xF, false);
            const double ks = __longlong_as_double((long long)(((unsigned long long)shi << 32) | slo));
            const unsigned long long vm = __ballot(valid);
            // rm bit at a left child: its right sibling exists and is larger
            const unsigned long long rm =
                __ballot(valid && (lane & 1) == 0 && ((vm >> (lane + 1)) & 1ull) && !(c.key >= ks));
            // g: this lane is the larger child of its pair and x < it -- the
            // walk passes it iff every ancestor of it in the block is g too
            const bool larger = (int)((rm >> (lane & ~1)) & 1ull) == (lane & 1);
            const unsigned long long g = __ballot(valid && larger && x.key < c.key);
            bool mvl = (g >> lane) & 1ull;
#pragma unroll
            for (int i = 1; i < kSinkLevels; i++) // ancestor at level i (lanes at levels > i)
                if (i < j) mvl = mvl && ((g >> ((2 << (i - 1)) - 2 + (bi >> (j - i)))) & 1ull);
            const unsigned long long mv = __ballot(mvl); // one lane per level, levels 1..lv
            const int lv = __builtin_popcountll(mv);
            if (mvl) { // each moved node goes one level up
                const int q = (p - 1) >> 1;
                if (kAll) {
                    top[q] = c;
                    pos[c.v] = q + 2;
                } else if (q < kTop) {
                    top[q] = c;
                    __asm__ volatile("; sink mv lds" ::: "memory");
                } else {
                    rest[q + 1] = c;
                    __asm__ volatile("; sink mv hbm" ::: "memory");
                }
                if (!kAll && p >= kTop) pos[c.v] = q >= kTop ? q + 2 : 1; // (1: entered the LDS top)
            }
            if (lv == 0) break;
            // the hole: the deepest moved node's old position
            const int hl = 63 - __builtin_clzll(mv);
            e = ((e + 1) << lv) - 1 + (hl + 2 - (1 << lv));
            if (lv < kSinkLevels) break;
        }
        st(e, x, from);
    }
    __device__ __forceinline__ void sink(int e, const HNode& x, int from) {
        if (kDp) sink_dp(e, x, from);
        else sink_seq(e, x, from);
    }
    __device__ __forceinline__ void push(int v, double key, int so) {
        const int e = n++;
        if (kDp) shift_up_dp(e, HNode{key, v, so}, -1);
        else shift_up(e, HNode{key, v, so}, -1);
    }
    // delete_max in two halves: the root is read first (top_node), then
    // removed (the last node takes the root and sinks)
    __device__ __forceinline__ HNode top_node() const { return ld(0); }
    __device__ __forceinline__ void pop_top(int v) {
        const int last = --n;
        pos[v] = 0;
        if (last > 0) sink(0, ld(last), last);
    }
    // position of v in the LDS top (slab kernel): every lane compares its
    // share of the occupied top positions, a ballot names the one holding v
    __device__ __forceinline__ int find_top(int v) const {
        const int m = n < kTop ? n : kTop;
        int found = -1;
        for (int q = lane; q < m; q += 64)
            if (top[q].v == v) found = q;
        const unsigned long long b = __ballot(found >= 0);
        return __builtin_amdgcn_readlane(found, b ? __builtin_ctzll(b) : 0);
    }
    // igraph_2wheap_modify with a larger key (Dijkstra only lowers a
    // distance, strictly): its sink step cannot move the node -- the heap
    // keeps parent >= child, so every child is <= the old key < the new key --
    // which leaves the shift-up at the node's position.
    __device__ __forceinline__ void raise(int v, double key, int so) {
        int e;
        if (kAll) {
            e = pos[v] - 2;
        } else {
            const int pv = uni(pos[v]);
            e = pv == 1 ? uni(find_top(v)) : pv - 2;
        }
        if (kDp) shift_up_dp(e, HNode{key, v, so}, e);
        else shift_up(e, HNode{key, v, so}, e);
    }
};

// ---- blocked slab heap (k_sssp_blk) ----------------------------------------
// The same igraph_2wheap (every comparison, move and tie rule of Heap above),
// stored so that a heap operation costs few HBM requests.  Positions
// [0, kBlkTop) -- levels 0..7 -- live in LDS.  Below, the heap is cut into
// 3-level subtrees ("blocks": a root at level 8, 11, 14, ... with its 2
// children and 4 grandchildren) of 7 nodes, stored BFS-ordered in one
// 128-byte line (slot 7 unused).  A sink or shift-up then reads a level
// triple with one line request and writes it back with one full-line store
// (8 lanes x 16 B, no partial-line write), where the flat layout costs a
// request per level for the node and another for its position.
// pos[v]: 0 not queued / popped, 1 in the LDS top, b + 2 in block b: a node
// moving inside its block keeps its pos (only moves across blocks write it);
// a decrease-key loads the block and finds v among its 7 slots.
// Lane-resident working set: lane L holds slot (L & 7) of one block in a
// 16-lane region (a sibling pair of blocks: the children of a level-7 node or
// of a block's bottom node are the roots of two consecutive blocks).
constexpr int kBlkTop = 255;   // LDS heap positions (levels 0..7)
constexpr int kBlkTopLv = 8;   // first HBM level

__host__ __device__ __forceinline__ int blk_base(int k) { return (256 * ((1 << (3 * k)) - 1)) / 7; }

// number of 128-B blocks that positions [kBlkTop, P] occupy (+1: pair loads)
__host__ __forceinline__ size_t blk_count(long P) {
    if (P < kBlkTop) return 2;
    int L = 0;
    while ((2L << L) <= P + 1) L++;
    const int k = (L - kBlkTopLv) / 3, Lr = kBlkTopLv + 3 * k;
    const long roots = P - (1L << Lr) + 2; // roots at level Lr with position <= P
    return (size_t)blk_base(k) + (size_t)(roots < (1L << Lr) ? roots : (1L << Lr)) + 1;
}

struct BHeap {
    HNode* top;   // LDS, kBlkTop (+1) nodes
    HNode* blk;   // HBM blocks, 8 nodes each, 128-B aligned
    int* pos;
    int n;
    int lane;
    // this lane's slot of an operation's working blocks (local to each
    // operation, so that it holds no registers between them)
    struct W {
        double k;
        int v, s;
    };

    // position p >= kBlkTop -> block id and slot
    __device__ __forceinline__ static void locate(int p, int& bid, int& idx) {
        const int L = 31 - __builtin_clz((unsigned)p + 1);
        const int k = (L - kBlkTopLv) / 3, Lr = kBlkTopLv + 3 * k, d = L - Lr;
        const int r1 = (p + 1) >> d;
        bid = blk_base(k) + r1 - (1 << Lr);
        idx = (1 << d) - 1 + ((p + 1) & ((1 << d) - 1));
    }
    // position of the root of block bid
    __device__ __forceinline__ static int root_pos(int bid) {
        int k = 0;
        while (blk_base(k + 1) <= bid) k++;
        return bid - blk_base(k) + (1 << (kBlkTopLv + 3 * k)) - 1;
    }
    __device__ __forceinline__ static int slot_pos(int root, int idx) {
        const int d = 31 - __builtin_clz((unsigned)idx + 1);
        return ((root + 1) << d) + (idx - ((1 << d) - 1)) - 1;
    }
    // node in working lane l (uniform)
    __device__ __forceinline__ static HNode lane_node(const W& w, int l) {
        return HNode{readlane_d(w.k, l), __builtin_amdgcn_readlane(w.v, l), __builtin_amdgcn_readlane(w.s, l)};
    }
    __device__ __forceinline__ void set_lane(W& w, int l, const HNode& x) const {
        if (lane == l) w.k = x.key, w.v = x.v, w.s = x.so;
    }
    // lanes [rb, rb + 8 * nb) <- blocks bid, bid + 1 (nb = 1 or 2)
    __device__ __forceinline__ void load_blocks(W& w, int bid, int rb, int nb) const {
        __asm__ volatile("" ::: "memory");
        if (lane >= rb && lane < rb + 8 * nb) {
            const HNode x = blk[(size_t)bid * 8 + (lane - rb)];
            w.k = x.key, w.v = x.v, w.s = x.so;
        }
        __asm__ volatile("; blk load" ::: "memory");
    }
    // one full-line store of the block in lanes [cb, cb + 8)
    __device__ __forceinline__ void store_block(const W& w, int bid, int cb) const {
        __asm__ volatile("" ::: "memory");
        if (lane >= cb && lane < cb + 8) blk[(size_t)bid * 8 + (lane - cb)] = HNode{w.k, w.v, w.s};
        __asm__ volatile("; blk store" ::: "memory");
    }
    __device__ __forceinline__ void set_pos(int v, int x) {
        pos[v] = x;
        __asm__ volatile("; pos store" ::: "memory");
    }
    __device__ __forceinline__ HNode ld_raw(int p) const {
        HNode x;
        if (p < kBlkTop) {
            x = top[p];
            __asm__ volatile("; heap lds" ::: "memory");
        } else {
            int b, i;
            locate(p, b, i);
            x = blk[(size_t)b * 8 + i];
            __asm__ volatile("; heap hbm" ::: "memory");
        }
        return x;
    }
    __device__ __forceinline__ HNode top_node() const { return uni_n(top[0]); }

    // LDS-only shift-up from e < kBlkTop; x enters the top (pos 1) unless it
    // was there already
    __device__ __forceinline__ void up_lds(int e, const HNode& x, bool was_top) {
        while (e > 0) {
            const int p = ((e + 1) >> 1) - 1;
            const HNode pn = uni_n(top[p]);
            if (x.key < pn.key) break;
            top[e] = pn;
            e = p;
        }
        top[e] = x;
        if (!was_top) set_pos(x.v, 1);
    }

    // shift-up of x from position e (>= kBlkTop) whose block is in lanes
    // [0, 8) already (block cbid, x's slot idx); from_bid = block x was in
    // (-1: new or from the LDS)
    __device__ __forceinline__ void up_blk(W& w, int cbid, int idx, const HNode& x, int from_bid) {
        int cb = 0;
        for (;;) {
            if (idx > 0) {
                const int pi = (idx - 1) >> 1;
                const HNode pn = lane_node(w, cb + pi);
                if (x.key < pn.key) break;
                set_lane(w, cb + idx, pn); // same block: pos unchanged
                idx = pi;
                continue;
            }
            const int rp = root_pos(cbid);
            const int pp = ((rp + 1) >> 1) - 1;
            if (pp < kBlkTop) { // parent in the LDS top
                const HNode pn = uni_n(top[pp]);
                if (x.key < pn.key) break;
                set_lane(w, cb, pn);
                set_pos(pn.v, cbid + 2);
                store_block(w, cbid, cb);
                up_lds(pp, x, false);
                return;
            }
            int pb, pidx;
            locate(pp, pb, pidx);
            const int ob = cb ^ 16;
            load_blocks(w, pb, ob, 1);
            const HNode pn = lane_node(w, ob + pidx);
            if (x.key < pn.key) break;
            set_lane(w, cb, pn);
            set_pos(pn.v, cbid + 2);
            store_block(w, cbid, cb);
            cb = ob, cbid = pb, idx = pidx;
        }
        set_lane(w, cb + idx, x);
        if (from_bid != cbid) set_pos(x.v, cbid + 2);
        store_block(w, cbid, cb);
    }

    __device__ __forceinline__ void push(int v, double key, int so) {
        const int e = n++;
        const HNode x{key, v, so};
        if (e < kBlkTop) {
            up_lds(e, x, false);
            return;
        }
        int b, i;
        locate(e, b, i);
        W w{0.0, 0, 0};
        if (i) load_blocks(w, b, 0, 1); // (a new block root: no slot of its block is live)
        up_blk(w, b, i, x, -1);
    }

    // igraph_2wheap_modify with a larger key: a shift-up at v's position
    __device__ __forceinline__ void raise(int v, double key, int so) {
        const HNode x{key, v, so};
        const int pv = uni(pos[v]);
        if (pv == 1) {
            const int m = n < kBlkTop ? n : kBlkTop;
            int found = -1;
            for (int q = lane; q < m; q += 64)
                if (top[q].v == v) found = q;
            const unsigned long long b = __ballot(found >= 0);
            const int e = uni(__builtin_amdgcn_readlane(found, b ? __builtin_ctzll(b) : 0));
            up_lds(e, x, true);
            return;
        }
        const int bid = pv - 2;
        W w{0.0, 0, 0};
        load_blocks(w, bid, 0, 1);
        const int root = root_pos(bid);
        const bool mine = lane < 8 && w.v == v && slot_pos(root, lane) < n;
        const unsigned long long m = __ballot(mine);
        up_blk(w, bid, __builtin_ctzll(m), x, bid);
    }

    // delete_max's sink of x (the old last node, from position `from`) from
    // the root: LDS levels by blocks of up to 5 levels, then HBM block pairs
    __device__ __forceinline__ void sink(const HNode& x, int from) {
        int e = 0;
        const int j = 31 - __builtin_clz((unsigned)lane + 2);
        const int bi = lane + 2 - (1 << j);
        for (;;) { // LDS phase
            if (2 * e + 1 >= n) {
                top[e] = x;
                if (from >= kBlkTop) set_pos(x.v, 1);
                return;
            }
            if (2 * e + 1 >= kBlkTop) break;
            const int p = (e + 1) * (1 << j) - 1 + bi;
            double ck_l = 0.0;
            int cv_l = 0, cs_l = 0;
            if (lane < (2 << kSinkLevels) - 2 && p < n && p < kBlkTop) {
                const HNode c = top[p];
                ck_l = c.key, cv_l = c.v, cs_l = c.so;
            }
            int lv = 0, li = 0;
            for (; lv < kSinkLevels; lv++) {
                const int l = 2 * e + 1;
                if (l >= n || l >= kBlkTop) break;
                int cl = (2 << lv) - 2 + 2 * li;
                double ck = readlane_d(ck_l, cl);
                int ci = l;
                if (l + 1 < n) {
                    const double rk = readlane_d(ck_l, cl + 1);
                    if (!(ck >= rk)) ck = rk, cl += 1, ci = l + 1;
                }
                if (!(x.key < ck)) {
                    top[e] = x;
                    if (from >= kBlkTop) set_pos(x.v, 1);
                    return;
                }
                top[e] = HNode{ck, __builtin_amdgcn_readlane(cv_l, cl), __builtin_amdgcn_readlane(cs_l, cl)};
                li = 2 * li + (ci - l);
                e = ci;
            }
        }
        // HBM phase: e is a level-7 hole whose children root blocks cb0, cb0 + 1
        int from_bid = -1;
        if (from >= kBlkTop) {
            int fi;
            locate(from, from_bid, fi);
        }
        int rb = 0;
        W w{0.0, 0, 0};
        load_blocks(w, 2 * e + 2 - 256, rb, 2);
        int cbid = -1, cb = 0, idx = 0; // the hole: top[e] (cbid < 0) or slot idx of block cbid
        for (;;) {
            const int l = 2 * e + 1;
            if (l >= n) break;
            int lc, step; // lanes of the two children
            const bool down = cbid < 0 || idx >= 3; // children are the roots of the loaded pair
            if (down) lc = rb, step = 8;
            else lc = cb + 2 * idx + 1, step = 1;
            HNode c = lane_node(w, lc);
            int ci = l;
            if (l + 1 < n) {
                const double rk = readlane_d(w.k, lc + step);
                if (!(c.key >= rk)) c = lane_node(w, lc + step), lc += step, ci = l + 1;
            }
            if (!(x.key < c.key)) break;
            if (cbid < 0) { // into the LDS top
                top[e] = c;
                set_pos(c.v, 1);
            } else {
                set_lane(w, cb + idx, c);
                if (down) set_pos(c.v, cbid + 2);
            }
            e = ci;
            if (down) {
                if (cbid >= 0) store_block(w, cbid, cb);
                cb = lc;
                int i2;
                locate(ci, cbid, i2);
                idx = 0;
            } else {
                idx = 2 * idx + 1 + (ci - l);
            }
            if (idx >= 3 && 2 * e + 1 < n) { // bottom of the block: next pair
                rb = (cb & ~15) ^ 16;
                int b2, i2;
                locate(2 * e + 1, b2, i2);
                load_blocks(w, b2, rb, 2);
            }
        }
        if (cbid < 0) {
            top[e] = x;
            if (from >= kBlkTop) set_pos(x.v, 1);
            return;
        }
        set_lane(w, cb + idx, x);
        if (from_bid != cbid) set_pos(x.v, cbid + 2);
        store_block(w, cbid, cb);
    }
};

// orders one wave's per-lane accesses before its uniform ones (and back)
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
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

// Row output (topology.c:1744-1791): every attached target but the source
// itself -- latency 0 becomes 1 ms -- then the self path.
template <typename DistRel>
__device__ __forceinline__ void write_row(const ShdGraphDev& g, int row, int src, ShdEntry* __restrict__ tab, int lane,
                                          DistRel dist_rel) {
    const int A = g.A;
    ShdEntry* out = tab + (size_t)row * (size_t)A;
    for (int j = lane; j < A; j += 64) {
        if (j == row) continue;
        double l, r;
        dist_rel(g.slot_vertex[j], l, r);
        ShdEntry e;
        if (l < 0) {
            e.lat = -1.0; // unreachable: impossible on a validated (strongly connected) graph
            e.rel = 0.0;
        } else {
            e.lat = (l == 0) ? 1.0 : l; // topology.c:1787-1791
            e.rel = r;
        }
        out[j] = e;
    }
    self_entry(g, src, out + row, lane);
}

// ---- LDS kernel: the whole per-row state in LDS (dense graphs, C1) ----
// The root node carries the start of its vertex's sentinel-terminated list
// (as in the slab kernel), so a pop's only memory round trip is the edge
// loads: kRelax batches of 64 entries are issued together (a complete
// graph's lists are 24 MB: Infinity-Cache round trips); the list's sentinel
// also says whether u is attached.
template <bool kDp>
__global__ __launch_bounds__(64) void k_sssp_lds(ShdGraphDev g, int row_lo, int row_hi, ShdEntry* __restrict__ tab) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int V = g.V, A = g.A;
    constexpr int kRelax = 16;
    HNode* top = reinterpret_cast<HNode*>(smem);
    double* dist = reinterpret_cast<double*>(top + V + 1);
    double* rel = dist + V;
    int* pos = reinterpret_cast<int*>(rel + V);
    const int2* __restrict__ snb = static_cast<const int2*>(g.snb);
    const double2* __restrict__ swr = static_cast<const double2*>(g.swr);
    for (int row = row_lo + (int)blockIdx.x; row < row_hi; row += (int)gridDim.x) {
        const int src = g.slot_vertex[row];
        for (int v = lane; v < V; v += 64) dist[v] = -1.0;
        wave_fence();
        Heap<true, kTopDefault, kDp> h{top, nullptr, pos, 0, lane};
        dist[src] = 0.0;
        rel[src] = 1.0;
        h.push(src, 0.0, g.soff[src]);
        int to_reach = A;
        while (h.n > 0 && to_reach > 0) {
            const HNode t = h.top_node();
            const int u = t.v;
            const double mindist = -t.key;
            const double ru = rel[u];
            // the list's first kRelax batches are loaded before the root is
            // removed: their latency overlaps the (LDS) sink
            int b = (int)((unsigned)t.so >> 8); // (unsigned: starts up to 2^24)
            const int lim = (t.so & 255) == 255 ? 64 * kRelax : (t.so & 255); // entries worth reading
            int2 nb[kRelax];
            double2 wr[kRelax];
#pragma unroll
            for (int q = 0; q < kRelax; q++) { // (entries past the sentinel re-read it)
                const int k = q * 64 + lane < lim ? q * 64 + lane : lim - 1;
                nb[q] = snb[b + k];
                wr[q] = swr[b + k];
            }
            h.pop_top(u);
            // kRelax batches are relaxed together (dist reads, then the
            // updates): an update only writes the dist of its own neighbour,
            // and a neighbour occurs once per list (parallel edges are
            // rejected at load; a loop never improves), so the early reads
            // see exactly what one-at-a-time relaxation would.
            for (;;) {
                int end = 64 * kRelax; // entries of this group before the sentinel
#pragma unroll
                for (int q = kRelax - 1; q >= 0; q--) {
                    const unsigned long long m = __ballot(nb[q].x < 0);
                    if (m) end = q * 64 + __builtin_ctzll(m);
                }
                bool imp[kRelax], fresh[kRelax];
                double alt[kRelax], rv[kRelax];
#pragma unroll
                for (int q = 0; q < kRelax; q++) {
                    const bool ok = q * 64 + lane < end && nb[q].x != u;
                    const double cur = ok ? dist[nb[q].x] : 0.0;
                    alt[q] = mindist + wr[q].x;
                    rv[q] = ru * wr[q].y;
                    fresh[q] = ok && cur < 0;
                    imp[q] = ok && (cur < 0 || alt[q] < cur);
                }
#pragma unroll
                for (int q = 0; q < kRelax; q++) {
                    unsigned long long m = __ballot(imp[q]);
                    const unsigned long long fm = __ballot(fresh[q]);
                    while (m) { // igraph's order: incidence order, one edge at a time
                        const int l = __builtin_ctzll(m);
                        m &= m - 1;
                        const int vv = __builtin_amdgcn_readlane(nb[q].x, l);
                        const double aa = readlane_d(alt[q], l);
                        dist[vv] = aa;
                        rel[vv] = readlane_d(rv[q], l);
                        if ((fm >> l) & 1ull) h.push(vv, -aa, __builtin_amdgcn_readlane(nb[q].y, l));
                        else h.raise(vv, -aa, __builtin_amdgcn_readlane(nb[q].y, l));
                    }
                }
                if (end < 64 * kRelax) {
                    // the sentinel: -2 when u is an attached vertex
                    int sv = 0;
#pragma unroll
                    for (int q = 0; q < kRelax; q++)
                        if (end >= q * 64 && end < q * 64 + 64) sv = __builtin_amdgcn_readlane(nb[q].x, end - q * 64);
                    if (sv == -2) --to_reach;
                    break;
                }
                b += 64 * kRelax; // lists longer than kRelax * 64 entries
#pragma unroll
                for (int q = 0; q < kRelax; q++) {
                    nb[q] = snb[b + q * 64 + lane];
                    wr[q] = swr[b + q * 64 + lane];
                }
            }
        }
        wave_fence();
        write_row(g, row, src, tab, lane, [&](int v, double& l, double& r) {
            l = dist[v];
            r = rel[v];
        });
        wave_fence();
    }
}

// ---- slab kernel: per-wave HBM slab, LDS heap top (sparse graphs, C2/C4) ----
// Incidence lists are read from the sentinel-terminated copy: list of v at
// g.soff[v], entries {nbr, soff[nbr]} in g.snb and {w, 1 - loss} in g.swr,
// closed by {-1 or -2 (v attached), 0}; the arrays are padded by 64 x 16 entries,
// so a 64-lane batch never reads past them.
template <int kTop>
__global__ __launch_bounds__(64 * kSlabWaves) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8, 8))) void k_sssp_slab(ShdGraphDev g, int row_lo, int row_hi,
                                                              ShdEntry* __restrict__ tab, char* __restrict__ slab,
                                                              size_t slab_stride) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const int gw = (int)blockIdx.x * wpb + w, nw = (int)gridDim.x * wpb;
    const int V = g.V, A = g.A;
    HNode* top = reinterpret_cast<HNode*>(smem) + w * kTop;
    HNode* rest = reinterpret_cast<HNode*>(slab + (size_t)gw * slab_stride);
    // one 16-B {dist, rel} record per vertex: the stores after an
    // improvement and the rel[u] read at its pop fall on the line the
    // distance gather fetched
    double2* dr = reinterpret_cast<double2*>(rest + V + 2);
    int* pos = reinterpret_cast<int*>(dr + V);
    const int2* __restrict__ snb = static_cast<const int2*>(g.snb);
    const double2* __restrict__ swr = static_cast<const double2*>(g.swr);

    for (int row = row_lo + gw; row < row_hi; row += nw) {
        const int src = g.slot_vertex[row];
        for (int v = lane; v < V; v += 64) dr[v].x = -1.0;
        wave_fence();
        Heap<false, kTop> h{top, rest, pos, 0, lane};
        dr[src] = make_double2(0.0, 1.0);
        h.push(src, 0.0, uni(g.soff[src]));
        int to_reach = A;
        while (h.n > 0 && to_reach > 0) {
            const HNode t = h.top_node(); // LDS
            const int u = t.v;
            const double mindist = -t.key;
            int b = (int)((unsigned)t.so >> 8); // (unsigned: starts up to 2^24)
            // issued together: u's incidence entries (only as many lanes as
            // the list has entries, sentinel included), the last heap node
            // (the removal sinks it) and rel[u]
            // lanes past the sentinel re-read it: their loads fall on lines
            // the list already fetches, so a short list costs 1-2 requests
            const int li = lane < (t.so & 255) ? lane : (t.so & 255) - 1;
            int2 nb = snb[b + li];
            double2 wr = swr[b + li];
            const int last = --h.n;
            const HNode xl = h.ld_raw(last);
            const double ru_l = dr[u].y;
            bool first = true;
            double ru = 0.0;
            for (;;) {
                // the list ends at the first sentinel; its value says whether
                // u is an attached vertex (a target of the row)
                const unsigned long long sm = __ballot(nb.x < 0);
                const int fs = sm ? __builtin_ctzll(sm) : 64;
                // (a loop entry -- listed twice per loop -- never improves: no gather)
                const bool ok = lane < fs && nb.x != u;
                double cur = ok ? dr[nb.x].x : 0.0; // neighbour distance gathers
                if (first) {
                    // the removal of the root: the sink's HBM block loads
                    // queue behind the gathers just issued
                    if (last > 0) h.sink(0, uni_n(xl), last);
                    ru = uni_d(ru_l);
                    first = false;
                }
                // keeps the gathered values' first use after the sink (else the
                // compiler hoists the compares above it and waits for the
                // gathers before sinking, serialising the two round trips)
                __asm__ volatile("" : "+v"(cur));
                if (fs < 64 && __builtin_amdgcn_readlane(nb.x, fs) == -2) --to_reach;
                const double alt = mindist + wr.x;
                const double rv = ru * wr.y;
                const bool fresh = ok && cur < 0;
                unsigned long long m = __ballot(ok && (cur < 0 || alt < cur));
                const unsigned long long fm = __ballot(fresh);
                // the batch's gathers precede its updates: an update writes
                // only its own neighbour's record and a neighbour occurs once
                // per list (parallel edges rejected; a loop never improves)
                while (m) { // igraph's order: incidence order, one edge at a time
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const int vv = __builtin_amdgcn_readlane(nb.x, l);
                    const int vs = __builtin_amdgcn_readlane(nb.y, l);
                    const double aa = readlane_d(alt, l);
                    dr[vv] = make_double2(aa, readlane_d(rv, l));
                    if ((fm >> l) & 1ull) h.push(vv, -aa, vs);
                    else h.raise(vv, -aa, vs);
                }
                if (fs < 64) break;
                b += 64; // lists longer than 64 entries: next batch
                nb = snb[b + lane];
                wr = swr[b + lane];
            }
        }
        wave_fence();
        write_row(g, row, src, tab, lane, [&](int v, double& l, double& r) {
            const double2 x = dr[v];
            l = x.x;
            r = x.y;
        });
        wave_fence();
    }
}

// ---- blocked-slab kernel: k_sssp_slab's pop loop over BHeap -----------------
// Slab per wave: nblk 128-B heap blocks, then one 16-B {dist, rel} record per
// vertex, then pos.  Same overlap of the pop's round trips as k_sssp_slab.
template <int kWpe> // waves per SIMD the register allocation is held to (8: 32 per CU)
__global__ __launch_bounds__(64 * kSlabWaves) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(kWpe, kWpe))) void k_sssp_blk(
    ShdGraphDev g, int row_lo, int row_hi, ShdEntry* __restrict__ tab, char* __restrict__ slab, size_t slab_stride,
    size_t nblk) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const int gw = (int)blockIdx.x * wpb + w, nw = (int)gridDim.x * wpb;
    const int V = g.V, A = g.A;
    HNode* top = reinterpret_cast<HNode*>(smem) + w * (kBlkTop + 1);
    HNode* blk = reinterpret_cast<HNode*>(slab + (size_t)gw * slab_stride);
    double2* dr = reinterpret_cast<double2*>(blk + nblk * 8);
    int* pos = reinterpret_cast<int*>(dr + V);
    const int2* __restrict__ snb = static_cast<const int2*>(g.snb);
    const double2* __restrict__ swr = static_cast<const double2*>(g.swr);

    for (int row = row_lo + gw; row < row_hi; row += nw) {
        const int src = g.slot_vertex[row];
        for (int v = lane; v < V; v += 64) dr[v].x = -1.0;
        wave_fence();
        BHeap h{top, blk, pos, 0, lane};
        dr[src] = make_double2(0.0, 1.0);
        h.push(src, 0.0, uni(g.soff[src]));
        int to_reach = A;
        while (h.n > 0 && to_reach > 0) {
            const HNode t = h.top_node(); // LDS
            const int u = t.v;
            const double mindist = -t.key;
            int b = (int)((unsigned)t.so >> 8); // (unsigned: starts up to 2^24)
            const int li = lane < (t.so & 255) ? lane : (t.so & 255) - 1;
            int2 nb = snb[b + li];
            double2 wr = swr[b + li];
            const int last = --h.n;
            const HNode xl = h.ld_raw(last);
            const double ru_l = dr[u].y;
            bool first = true;
            double ru = 0.0;
            for (;;) {
                const unsigned long long sm = __ballot(nb.x < 0);
                const int fs = sm ? __builtin_ctzll(sm) : 64;
                const bool ok = lane < fs && nb.x != u;
                double cur = ok ? dr[nb.x].x : 0.0;
                if (first) {
                    if (last > 0) h.sink(uni_n(xl), last);
                    ru = uni_d(ru_l);
                    first = false;
                }
                __asm__ volatile("" : "+v"(cur));
                if (fs < 64 && __builtin_amdgcn_readlane(nb.x, fs) == -2) --to_reach;
                const double alt = mindist + wr.x;
                const double rv = ru * wr.y;
                const bool fresh = ok && cur < 0;
                unsigned long long m = __ballot(ok && (cur < 0 || alt < cur));
                const unsigned long long fm = __ballot(fresh);
                while (m) {
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const int vv = __builtin_amdgcn_readlane(nb.x, l);
                    const int vs = __builtin_amdgcn_readlane(nb.y, l);
                    const double aa = readlane_d(alt, l);
                    dr[vv] = make_double2(aa, readlane_d(rv, l));
                    if ((fm >> l) & 1ull) h.push(vv, -aa, vs);
                    else h.raise(vv, -aa, vs);
                }
                if (fs < 64) break;
                b += 64;
                nb = snb[b + lane];
                wr = swr[b + lane];
            }
        }
        wave_fence();
        write_row(g, row, src, tab, lane, [&](int v, double& l, double& r) {
            const double2 x = dr[v];
            l = x.x;
            r = x.y;
        });
        wave_fence();
    }
}

// ---- integer-key slab kernel (k_sssp_islab): graphs whose latencies are whole ms ----
// When every edge latency is a whole number of ms and V * max latency <
// 2^32 - 1 (ShdGraphDev.sl present), every distance igraph forms -- f64 sums
// of whole numbers below 2^53 -- is exact, so a u32 holds it bit for bit and
// the heap compares u32 dist instead of f64 -dist (x.key < c.key <=> dc < dx;
// ties compare equal in both).  That shrinks a heap node to 8 B {dist, v},
// and the storage is laid out for few HBM requests per heap operation:
//  * positions [0, 511) (levels 0..8) in LDS, 4 KiB per wave;
//  * below, 4-level subtrees ("blocks", roots at levels 9, 13, 17, ...) of 15
//    nodes in one 128-B line each, so a sink reads the two child blocks of
//    its hole (the 4 levels under it) with two line requests, walks them
//    data-parallel, and its moves inside a block all land in that block's line;
//  * each vertex's 16-B record {dist u32, pos u32, rel f64}: pos is the block
//    the vertex's node sits in (1: the LDS top, 0: never queued), so only moves
//    that cross a block boundary write a pos (not every level a node moves),
//    a decrease-key finds its node among the 15 slots of the line it loads
//    anyway for the shift-up, and the neighbour gather of a pop brings the
//    pos of every neighbour with its distance.
// The list handle no longer rides in the node: the pop reads soff[u] (a 4-B
// array shared by every wave, L2-resident).  Heap moves are igraph_2wheap's,
// exactly as in Heap above.
namespace ik {
typedef unsigned long long u64;
constexpr int kTop = 511; // LDS positions: levels 0..8
constexpr int kTopLv = 9; // first HBM level
constexpr uint32_t kInf = 0xffffffffu;

struct __attribute__((aligned(16))) Rec {
    uint32_t d;   // distance in ms (kInf: not reached)
    uint32_t pos; // 0 never queued, 1 LDS top, block id + 2
    double rel;
};
struct __attribute__((aligned(16))) Ent { // one incidence-list entry (ShdGraphDev.sl)
    int nbr;
    uint32_t w;
    double rel;
};

__device__ __forceinline__ uint32_t kd(u64 x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ int kv(u64 x) { return (int)(uint32_t)x; }
__device__ __forceinline__ u64 mk(uint32_t d, int v) { return ((u64)d << 32) | (uint32_t)v; }
__device__ __forceinline__ int lvl(int p) { return 31 - __builtin_clz((unsigned)p + 1); }
// first block id of block level k: 512 * (16^k - 1) / 15 = 512 * 0x11..1 (k hex ones)
__host__ __device__ __forceinline__ int bbase(int k) { return (int)((0x11111111u & ((1u << (4 * k)) - 1u)) << 9); }
__device__ __forceinline__ u64 uni64(u64 x) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 lane64(u64 x, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
    return ((u64)hi << 32) | lo;
}
// HBM position p (>= kTop): its block id; *slot = its slot in the block
__device__ __forceinline__ int bid_of(int p, int* slot) {
    const int t = lvl(p) - kTopLv;
    const int d = t & 3, k = t >> 2;
    const int m = (1 << d) - 1;
    *slot = m + ((p + 1) & m);
    // bbase(k) - 2^(9 + 4k) for the block levels a heap of < 2^21 nodes uses
    const int c = k == 0 ? -512 : k == 1 ? 512 - 8192 : k == 2 ? 8704 - 131072 : 139776 - 2097152;
    return ((p + 1) >> d) + c;
}

// kStats: event counters (SHD_SSSP_STATS=1, measurement only)
enum { kStPops, kStSinkHbm, kStPush, kStRaiseHbm, kStRaiseLds, kStUpRounds, kStUpClimb, kStLogOvf, kStBatches,
       kStHeapSum, kStUpHbmRounds, kStN };
constexpr u64 kSent = ~0ull; // an empty heap slot: dist kInf, vertex -1

// A heap place: b < 0: LDS position s; else slot s of HBM block b.
// Block navigation (no positions needed):
//  * children of LDS position s at level 8: the roots of blocks 2s - 510, 2s - 509;
//  * children of bottom slot s (7..14) of block b: the roots of blocks
//    16b + 2s + 498 and the next one (independent of the block level);
//  * parent of the root of block b: LDS position (b + 510) / 2 when b < 512,
//    else slot 7 + ((b - 512) & 15) / 2 of block (b - 512) / 16.
// Every slot at or past the heap's end holds kSent, so the sink and the
// decrease-key search need no size tests: an empty child is never the
// larger one and never larger than the sinking node.
template <bool kStats>
struct Heap {
    unsigned long long st[kStats ? kStN : 1];
    __device__ __forceinline__ void stat(int i, unsigned long long x = 1) {
        if (kStats) st[i] += x;
    }
    u64* top;    // LDS: position p at top[p + 1] (a sibling pair is one aligned 16-B read); top[0] scratch
    u64* blk;    // 16 u64 per block (slot 15 unused)
    Rec* rec;
    int n;
    int lane;
    int nblk;
    // pos stores made since the current batch's gather (which read the
    // neighbours' pos): lane i holds entry i; nlog > 64 = overflowed
    int log_v;
    uint32_t log_t;
    int nlog;

    __device__ __forceinline__ void set_pos(int v, uint32_t t) {
        rec[v].pos = t;
        __asm__ volatile("; ipos store" ::: "memory");
        if (lane == nlog) log_v = v, log_t = t;
        nlog++;
    }
    // v's pos: the last logged store, else the gathered value g (or a fresh
    // load when the log overflowed)
    __device__ __forceinline__ uint32_t pos_of(int v, uint32_t g) {
        if (nlog > 64) {
            stat(kStLogOvf);
            return (uint32_t)__builtin_amdgcn_readfirstlane((int)rec[v].pos);
        }
        const unsigned long long m = __ballot(lane < nlog && log_v == v);
        if (!m) return g;
        return (uint32_t)__builtin_amdgcn_readlane((int)log_t, 63 - __builtin_clzll(m));
    }
    // the place of position p
    __device__ __forceinline__ static void loc_of(int p, int& b, int& s) {
        if (p < kTop) {
            b = -1, s = p;
        } else {
            b = bid_of(p, &s);
        }
    }
    __device__ __forceinline__ static uint32_t tag(int b) { return b < 0 ? 1u : (uint32_t)b + 2u; }
    // node x into place (b, s) by lane l (l < 0: every lane, same value)
    __device__ __forceinline__ void put(int b, int s, u64 x, int l = -1) {
        if (b < 0) {
            if (l < 0 || lane == l) top[s + 1] = x;
            __asm__ volatile("; iput lds" ::: "memory");
        } else {
            if (l < 0 || lane == l) blk[(size_t)b * 16 + s] = x;
            __asm__ volatile("; iput hbm" ::: "memory");
        }
    }

    // Shift-up of x from place (b, s); returns x's new pos tag.  One round
    // per storage unit: the ancestors from the parent up to the top of the
    // parent's block (or every LDS ancestor) are compared at once, one per
    // lane, a ballot says which x is not smaller than (the nearest cnt, heap
    // order), and those move one level down the path.  se >= 0: (b, s) is in
    // a block whose line the caller holds (lane s = slot s), so a first round
    // inside that block needs no load.
    __device__ __forceinline__ uint32_t up(int b, int s, u64 x, u64 line = 0, bool held = false) {
        const uint32_t dx = kd(x);
        for (;;) {
            if (b < 0 && s == 0) break; // the root
            // the round's unit: ub < 0: LDS, ancestors from position ps up;
            // else block ub, ancestors from slot ps up
            int ub, ps;
            if (b < 0) {
                ub = -1, ps = (s - 1) >> 1;
            } else if (s > 0) {
                ub = b, ps = (s - 1) >> 1;
            } else if (b < 512) {
                ub = -1, ps = (b + 510) >> 1;
            } else {
                ub = (b - 512) >> 4, ps = 7 + (((b - 512) & 15) >> 1);
            }
            const int K = lvl(ps) + 1;
            const int sa = ((ps + 1) >> lane) - 1; // lane j: j-th ancestor in the unit
            u64 c = 0;
            stat(kStUpRounds);
            if (ub < 0) {
                if (lane < K) c = top[sa + 1];
                __asm__ volatile("; iup lds" ::: "memory");
            } else {
                stat(kStUpHbmRounds);
                if (held && ub == b) {
                    const int src = lane < K ? sa : 0;
                    const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(4 * src, (int)(uint32_t)line);
                    const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(4 * src, (int)(uint32_t)(line >> 32));
                    c = ((u64)hi << 32) | lo;
                } else if (lane < K) {
                    c = blk[(size_t)ub * 16 + sa];
                }
                __asm__ volatile("; iup hbm" ::: "memory");
            }
            held = false;
            const unsigned long long m = __ballot(lane < K && dx <= kd(c)); // x climbs past these
            const int cnt = (int)__builtin_ctzll(~m);
            if (cnt == 0) break;
            stat(kStUpClimb);
            // ancestor 0 into x's place, ancestor j >= 1 into ancestor j-1's
            put(b, s, c, 0);
            if (lane >= 1 && lane < cnt) {
                const int q = ((ps + 1) >> (lane - 1)) - 1;
                if (ub < 0) {
                    top[q + 1] = c;
                    __asm__ volatile("; iup mv lds" ::: "memory");
                } else {
                    blk[(size_t)ub * 16 + q] = c;
                    __asm__ volatile("; iup mv hbm" ::: "memory");
                }
            }
            if (b >= 0 && s == 0) set_pos(kv(lane64(c, 0)), tag(b)); // crossed into x's old block
            b = ub, s = ((ps + 1) >> (cnt - 1)) - 1;
            if (cnt < K) break;
        }
        put(b, s, x);
        return tag(b);
    }
    // Shift-up of x from HBM place (b, s) (b >= 0) with the first round
    // fused: the ancestors inside b (from the held line when `held`, lane q
    // = slot q) and those of b's parent unit (b's parent's block, or every
    // LDS ancestor) are compared in one round, so a climb that leaves its
    // block still costs one memory round trip.  Returns x's new pos tag.
    __device__ __forceinline__ uint32_t up2(int b, int s, u64 x, u64 line, bool held) {
        const uint32_t dx = kd(x);
        if (held && s > 0) { // the ancestors inside the held line first: no load
            const int ds = lvl(s);
            const int qa = ((s + 1) >> (lane + 1)) - 1;
            const int src = lane < ds ? qa : 0;
            const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(4 * src, (int)(uint32_t)line);
            const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(4 * src, (int)(uint32_t)(line >> 32));
            const u64 c = ((u64)hi << 32) | lo;
            const unsigned long long m = __ballot(lane < ds && dx <= kd(c));
            const int cnt = (int)__builtin_ctzll(~m);
            if (cnt < ds) { // x stays below the block's root
                if (lane < cnt) {
                    const int q = lane == 0 ? s : ((s + 1) >> lane) - 1;
                    blk[(size_t)b * 16 + q] = c;
                    __asm__ volatile("; iup2h mv blk" ::: "memory");
                }
                put(b, ((s + 1) >> cnt) - 1, x);
                return tag(b);
            }
        }
        const int ds = lvl(s); // ancestors inside b: slots ((s + 1) >> j) - 1, j = 1..ds
        // b's parent unit: pb < 0: the LDS, ancestors from position pp up; else block pb from slot pp up
        int pb, pp;
        if (b < 512) {
            pb = -1, pp = (b + 510) >> 1;
        } else {
            pb = (b - 512) >> 4, pp = 7 + (((b - 512) & 15) >> 1);
        }
        const int pK = lvl(pp) + 1;
        const int K = ds + pK;
        // lane j < ds: in-block ancestor j + 1; ds <= j < K: parent-unit ancestor i = j - ds
        const bool inb = lane < ds;
        const int i = lane - ds;
        const int qa = ((s + 1) >> (lane + 1)) - 1; // in-block ancestor slot (lane < ds)
        const int qp = ((pp + 1) >> (i < 0 ? 0 : i)) - 1; // parent-unit place (lane >= ds)
        u64 c = 0;
        if (held) {
            const int src = inb ? qa : 0;
            const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(4 * src, (int)(uint32_t)line);
            const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(4 * src, (int)(uint32_t)(line >> 32));
            c = ((u64)hi << 32) | lo;
        } else if (inb) {
            c = blk[(size_t)b * 16 + qa];
        }
        if (!inb && lane < K) {
            if (pb < 0) {
                c = top[qp + 1];
                __asm__ volatile("; iup2 lds" ::: "memory");
            } else {
                c = blk[(size_t)pb * 16 + qp];
                __asm__ volatile("; iup2 hbm" ::: "memory");
            }
        }
        stat(kStUpRounds);
        stat(kStUpHbmRounds);
        const unsigned long long m = __ballot(lane < K && dx <= kd(c)); // x climbs past these
        const int cnt = (int)__builtin_ctzll(~m);
        if (cnt == 0) {
            put(b, s, x);
            return tag(b);
        }
        stat(kStUpClimb);
        // ancestor j moves into ancestor j-1's place (j = 0: x's place):
        // in b for j <= ds (j = ds: b's root, a crossing), else in the parent unit
        if (lane < cnt) {
            if (lane <= ds) {
                const int q = lane == 0 ? s : ((s + 1) >> lane) - 1;
                blk[(size_t)b * 16 + q] = c;
                __asm__ volatile("; iup2 mv blk" ::: "memory");
            } else {
                const int q = ((pp + 1) >> (i - 1)) - 1;
                if (pb < 0) {
                    top[q + 1] = c;
                    __asm__ volatile("; iup2 mv lds" ::: "memory");
                } else {
                    blk[(size_t)pb * 16 + q] = c;
                    __asm__ volatile("; iup2 mv pblk" ::: "memory");
                }
            }
        }
        if (cnt > ds) set_pos(kv(lane64(c, ds)), tag(b)); // parent-unit ancestor 0 crossed into b
        if (cnt <= ds) { // x stays in b
            const int q = ((s + 1) >> cnt) - 1;
            put(b, q, x);
            return tag(b);
        }
        const int q = ((pp + 1) >> (cnt - 1 - ds)) - 1; // x's place in the parent unit
        if (cnt < K || pb < 0) {
            put(pb, q, x);
            return tag(pb);
        }
        return up(pb, q, x); // climbed past the whole parent block (q = its root)
    }
    // the place of position n, when the caller knows it (the pop's emptied
    // place is where the first push of the pop goes)
    int cb_p = -1, cb_b = 0, cb_s = 0;
    __device__ __forceinline__ uint32_t push(int v, uint32_t d) {
        stat(kStPush);
        int b, s;
        if (n == cb_p) {
            b = cb_b, s = cb_s;
        } else {
            loc_of(n, b, s);
        }
        n++;
        if (b < 0) return up(b, s, mk(d, v));
        return up2(b, s, mk(d, v), 0, false);
    }
    // igraph_2wheap_modify with a smaller distance: a shift-up at v's node.
    // A node that moved up into the LDS top keeps the block its pos names
    // (no pos store for that move: one write request less per pop), so a
    // block that does not hold v sends the search to the LDS top.  A pos
    // that names neither (never expected) is counted in *err and the update
    // skipped: the launch then fails instead of reading outside the slab.
    __device__ __forceinline__ uint32_t raise(int v, uint32_t d, uint32_t t, unsigned* err) {
        stat(t == 1u ? kStRaiseLds : kStRaiseHbm);
        if (t >= 2u && (int)(t - 2u) < nblk) {
            // the named block, then its ancestors' blocks (a node the sink
            // moved up across a block boundary keeps its old pos)
            for (int b = (int)t - 2; b >= 0; b = b >= 512 ? (b - 512) >> 4 : -1) {
                u64 c = kSent;
                if (lane < 15) c = blk[(size_t)b * 16 + lane];
                __asm__ volatile("; iraise find" ::: "memory");
                const unsigned long long bm = __ballot(lane < 15 && kv(c) == v);
                if (bm) return up2(b, __builtin_ctzll(bm), mk(d, v), c, true);
            }
            t = 1u; // moved up into the LDS top since
        }
        if (t == 1u) {
            int found = -1;
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (q * 64 + lane < kTop && kv(top[q * 64 + lane + 1]) == v) found = q * 64 + lane;
            const unsigned long long bm = __ballot(found >= 0);
            if (!bm) {
                if (lane == 0) atomicOr(err, 1u);
                return t;
            }
            const int e = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(found, __builtin_ctzll(bm)));
            return up(-1, e, mk(d, v));
        }
        if (lane == 0) atomicOr(err, 2u);
        return t;
    }

    // delete_max's sink of x (the old last node, whose place had tag tfrom)
    // from the root: the LDS levels one per step, branch-free on the vector
    // unit (every lane computes the same walk), then the HBM levels four at a
    // time -- the two child blocks of the hole, one node per lane, walked
    // data-parallel (ballots: which sibling is larger, which nodes x is
    // larger than), each moved node stored one level up by its own lane
    __device__ __forceinline__ void sink(u64 x, uint32_t tfrom) {
        const uint32_t dx = kd(x);
        int ev = 0;
        bool alive = true;
        // (no early exit: x is a bottom node and nearly always sinks past
        // all eight levels; a stopped walk just rewrites the scratch slot)
#pragma unroll
        for (int it = 0; it < kTopLv - 1; it++) {
            const int l = 2 * ev + 1;
            const uint4 pr = *reinterpret_cast<const uint4*>(top + l + 1);
            __asm__ volatile("; isink lds" ::: "memory");
            const bool right = pr.w < pr.y;
            const uint32_t dc = right ? pr.w : pr.y;
            const uint32_t vc = right ? pr.z : pr.x;
            const bool mv = alive && dc < dx;
            top[mv ? ev + 1 : 0] = ((u64)dc << 32) | vc;
            __asm__ volatile("; isink mv lds" ::: "memory");
            ev = mv ? l + (right ? 1 : 0) : ev;
            alive = mv;
        }
        int hb = -1, hs = __builtin_amdgcn_readfirstlane(ev);
        if (__ballot(alive) != 0ull) { // the hole reached level 8: HBM blocks
            const int j = 31 - __builtin_clz((unsigned)lane + 2); // lane's level under the hole
            const int bi = lane + 2 - (1 << j);                    // ... and index in that level
            const int sb = bi >> (j - 1);                          // child block 0 / 1
            const int bslot = (1 << (j - 1)) - 1 + (bi & ((1 << (j - 1)) - 1)); // slot in it
            // the lane's ancestors at levels 1..3 under the hole (itself where it has none)
            const int an1 = j > 1 ? (bi >> (j - 1)) : lane;
            const int an2 = j > 2 ? 2 + (bi >> (j - 2)) : lane;
            const int an3 = j > 3 ? 6 + (bi >> (j - 3)) : lane;
            for (;;) {
                const int b0 = hb < 0 ? 2 * hs - 510 : 16 * hb + 2 * hs + 498;
                if (b0 + 1 >= nblk) break; // (no block there: past every possible heap position)
                stat(kStSinkHbm);
                u64 c = kSent;
                if (j <= 4) c = blk[(size_t)(b0 + sb) * 16 + bslot];
                __asm__ volatile("; isink hbm" ::: "memory");
                const uint32_t dc = kd(c);
                const uint32_t dsib = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dc, 0xB1, 0xF, 0xF, false);
                // rm bit at a left child: the right sibling is larger (smaller
                // dist; an empty right sibling never is)
                const unsigned long long rm = __ballot((lane & 1) == 0 && dsib < dc);
                const uint32_t larger = (uint32_t)((rm >> (lane & ~1)) ^ (unsigned long long)lane ^ 1ull) & 1u;
                const unsigned long long g = __ballot(j <= 4 && larger && dc < dx);
                // a lane moves iff it and its ancestors in the block pair are all g
                const uint32_t mvb = (uint32_t)(g >> lane) & (uint32_t)(g >> an1) & (uint32_t)(g >> an2) &
                                     (uint32_t)(g >> an3) & 1u;
                const bool mvl = mvb != 0u;
                const unsigned long long mv = __ballot(mvl);
                if (mv == 0ull) break;
                const int lv = __builtin_popcountll(mv);
                const int l1 = __builtin_ctzll(mv);
                // the level-1 mover into the hole (the LDS or the parent block: a crossing)
                put(hb, hs, c, l1);
                // (the level-1 mover goes up into the hole's block or the LDS:
                // its pos is left naming a block below, see raise)
                if (mvl && j > 1) { // the others one level up inside their block
                    blk[(size_t)(b0 + sb) * 16 + ((bslot - 1) >> 1)] = c;
                    __asm__ volatile("; isink mv blk" ::: "memory");
                }
                const int hl = 63 - __builtin_clzll(mv); // the new hole: the deepest mover's place
                hb = b0 + __builtin_amdgcn_readlane(sb, hl);
                hs = __builtin_amdgcn_readlane(bslot, hl);
                if (lv < 4) break;
            }
        }
        put(hb, hs, x);
        if (hb >= 0 && tag(hb) != tfrom) set_pos(kv(x), tag(hb)); // (into the LDS: pos left stale, see raise)
    }
};

// blocks a wave's heap needs for positions < V (+1: a hole's child pair):
// those of the deepest block level in use hold every root of its top level
// up to position V - 1
__host__ __device__ __forceinline__ int blk_count(long V) {
    if (V <= kTop) return 0;
    const long p = V - 1;
    int L = 0;
    while ((2L << L) <= p + 1) L++;
    const int k = (L - kTopLv) >> 2, Lr = kTopLv + 4 * k;
    long roots = p - (1L << Lr) + 2; // roots at level Lr with position <= p
    if (roots > (1L << Lr)) roots = 1L << Lr;
    return (int)(bbase(k) + roots) + 1;
}
} // namespace ik

// Slab per wave: nblk 128-B heap blocks, then V 16-B records.
// kWpe: waves per SIMD (SHD_SSSP_WPE: 8 default; 7 and 6 trade occupancy for
// fewer register spills -- 8 waves leave 64 VGPRs and 78 SGPRs, and the
// compiler spills 23 VGPRs to scratch and 35 SGPRs to VGPR lanes; 7: 18 and
// 26; 6: 6 and 11)
template <bool kStats, int kWpe = 8>
__global__ __launch_bounds__(64 * kSlabWaves) __attribute__((amdgpu_waves_per_eu(kWpe, kWpe))) void k_sssp_islab(
    ShdGraphDev g, int row_lo, int row_hi, ShdEntry* __restrict__ tab, char* __restrict__ slab, size_t slab_stride,
    size_t nblk, unsigned* __restrict__ err, unsigned long long* __restrict__ stats) {
    using namespace ik;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const int gw = (int)blockIdx.x * wpb + w, nw = (int)gridDim.x * wpb;
    const int V = g.V, A = g.A;
    u64* top = reinterpret_cast<u64*>(smem) + w * (kTop + 1);
    u64* blk = reinterpret_cast<u64*>(slab + (size_t)gw * slab_stride);
    Rec* rec = reinterpret_cast<Rec*>(blk + nblk * 16);
    const Ent* __restrict__ sl = static_cast<const Ent*>(g.sl);
    const int* __restrict__ soff = g.soff;
    // every heap slot starts empty (and is emptied again at the end of a row)
    for (int q = lane; q <= kTop; q += 64) top[q] = kSent;
    for (size_t q = lane; q < nblk * 16; q += 64) blk[q] = kSent;

    for (int row = row_lo + gw; row < row_hi; row += nw) {
        const int src = g.slot_vertex[row];
        for (int v = lane; v < V; v += 64) rec[v] = Rec{kInf, 0u, 0.0};
        wave_fence();
        ik::Heap<kStats> h;
        h.top = top, h.blk = blk, h.rec = rec, h.n = 0, h.lane = lane, h.nblk = (int)nblk;
        h.log_v = 0, h.log_t = 0u, h.nlog = 0;
        if (kStats)
            for (int i = 0; i < kStN; i++) h.st[i] = 0;
        rec[src] = Rec{0u, 1u, 1.0};
        top[1] = mk(0u, src);
        h.n = 1;
        int to_reach = A;
        // the next root's list handle, loaded right after the sink (the
        // updates that follow rarely replace the root): pv = its vertex
        int pv = -1, pso = 0;
        while (h.n > 0 && to_reach > 0) {
            h.stat(kStPops);
            h.stat(kStHeapSum, (unsigned long long)h.n);
            const u64 t = uni64(top[1]); // LDS (the root)
            const int u = kv(t);
            const uint32_t du = kd(t);
            const int so = u == pv ? uni(pso) : uni(soff[u]);
            int b = (int)((unsigned)so >> 8); // (unsigned: starts up to 2^24)
            // issued together: u's entries (lanes past the sentinel re-read
            // it), the last heap node (the removal sinks it) and rel[u]
            const int li = lane < (so & 255) ? lane : (so & 255) - 1;
            Ent en = sl[b + li];
            // the last node (the removal sinks it); its place becomes empty
            const int last = --h.n;
            int lb, ls;
            h.loc_of(last, lb, ls);
            h.cb_p = last, h.cb_b = lb, h.cb_s = ls;
            u64 xl;
            if (lb < 0) {
                xl = top[ls + 1];
                top[ls + 1] = kSent;
                __asm__ volatile("; ilast lds" ::: "memory");
            } else {
                xl = blk[(size_t)lb * 16 + ls];
                blk[(size_t)lb * 16 + ls] = kSent;
                __asm__ volatile("; ilast hbm" ::: "memory");
            }
            const double ru_l = rec[u].rel;
            bool first = true;
            double ru = 0.0;
            for (;;) {
                h.stat(kStBatches);
                const unsigned long long sm = __ballot(en.nbr < 0);
                const int fs = sm ? __builtin_ctzll(sm) : 64;
                const bool ok = lane < fs && en.nbr != u;
                // neighbour {dist, pos} gathers
                u64 cur = ok ? *reinterpret_cast<const u64*>(&rec[en.nbr]) : 0ull;
                h.nlog = 0;
                if (first) {
                    if (last > 0) h.sink(uni64(xl), h.tag(lb));
                    // (the wait for rel[u] covers every load issued so far:
                    // the prefetch goes after it, not into it)
                    ru = uni_d(ru_l);
                    pv = h.n > 0 ? kv(uni64(top[1])) : -1;
                    if (pv >= 0) pso = soff[pv];
                    first = false;
                }
                __asm__ volatile("" : "+v"(cur));
                if (fs < 64 && __builtin_amdgcn_readlane(en.nbr, fs) == -2) --to_reach;
                const uint32_t alt = du + en.w;
                const double rv = ru * en.rel;
                const uint32_t cd = (uint32_t)cur;
                unsigned long long m = __ballot(ok && alt < cd);
                const unsigned long long fm = __ballot(ok && cd == kInf);
                while (m) { // igraph's order: incidence order, one edge at a time
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const int vv = __builtin_amdgcn_readlane(en.nbr, l);
                    const uint32_t aa = (uint32_t)__builtin_amdgcn_readlane((int)alt, l);
                    uint32_t tg;
                    if ((fm >> l) & 1ull) {
                        tg = h.push(vv, aa);
                    } else {
                        const uint32_t gp = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cur >> 32), l);
                        tg = h.raise(vv, aa, h.pos_of(vv, gp), err);
                    }
                    // (not logged: vv occurs once in the list, so no later
                    // update of this batch asks for its pos)
                    rec[vv] = Rec{aa, tg, readlane_d(rv, l)};
                    __asm__ volatile("; irec store" ::: "memory");
                }
                if (fs < 64) break;
                b += 64; // lists longer than 64 entries: next batch
                en = sl[b + lane];
            }
        }
        // empty the heap for the next row (slots past n are empty already)
        for (int q = lane; q <= kTop; q += 64) top[q] = kSent;
        for (int q = lane, e = blk_count(h.n) * 16; q < e; q += 64) blk[q] = kSent;
        wave_fence();
        write_row(g, row, src, tab, lane, [&](int v, double& l, double& r) {
            const Rec x = rec[v];
            l = x.d == kInf ? -1.0 : (double)x.d;
            r = x.rel;
        });
        wave_fence();
        if (kStats && lane == 0)
            for (int i = 0; i < kStN; i++) atomicAdd(&stats[i], h.st[i]);
    }
}

// ---- integer-key LDS kernel (k_sssp_ilds): dense graphs with whole-ms latencies (C1) ----
// k_sssp_lds's structure (one wave per row, the whole row in LDS, kRelax
// batches of 64 list entries in flight per pop) with the integer keys of
// k_sssp_islab: 8-B heap nodes {dist u32, v}, u32 compares, 16-B list
// entries {nbr, w, 1 - loss} (the list handles copied into LDS once per
// wave), the removal's sink as a branch-free walk on the vector unit, and a
// shift-up as one data-parallel round (every ancestor is in LDS).  pos is
// exact (position + 1) -- in LDS every move may as well record it.  LDS: 28 B
// per vertex (k_sssp_lds: 36).
__global__ __launch_bounds__(64) void k_sssp_ilds(ShdGraphDev g, int row_lo, int row_hi, ShdEntry* __restrict__ tab) {
    using namespace ik;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int kRelax = 16;
    const int lane = threadIdx.x & 63;
    const int V = g.V, A = g.A;
    u64* top = reinterpret_cast<u64*>(smem);                      // V + 2: position p at top[p + 1]; top[0] scratch
    uint32_t* dp = reinterpret_cast<uint32_t*>(top + V + 2);      // 2V: {dist, pos + 1} per vertex, + 2 scratch
    double* rel = reinterpret_cast<double*>(dp + 2 * V + 2);       // V
    int* so_l = reinterpret_cast<int*>(rel + V);                  // V: list handles
    const Ent* __restrict__ sl = static_cast<const Ent*>(g.sl);
    uint32_t* const pscr = dp + 2 * V; // scratch for masked-off pos stores
    for (int v = lane; v < V; v += 64) so_l[v] = g.soff[v];
    for (int row = row_lo + (int)blockIdx.x; row < row_hi; row += (int)gridDim.x) {
        const int src = g.slot_vertex[row];
        for (int v = lane; v < V; v += 64) reinterpret_cast<u64*>(dp)[v] = (u64)kInf; // dist kInf, pos 0
        wave_fence();
        top[1] = mk(0u, src);
        reinterpret_cast<u64*>(dp)[src] = 1ull << 32; // dist 0 at position 0
        rel[src] = 1.0;
        int n = 1;
        // shift-up of x from position e (one round: all ancestors in LDS);
        // returns x's final position
        auto up = [&](int e, u64 x) -> int {
            const uint32_t dx = kd(x);
            if (e > 0) {
                const int K = lvl(e);
                const int a = ((e + 1) >> (lane + 1)) - 1;
                u64 c = 0;
                if (lane < K) c = top[a + 1];
                const unsigned long long m = __ballot(lane < K && dx <= kd(c));
                const int cnt = (int)__builtin_ctzll(~m);
                if (lane < cnt) {
                    const int d = ((e + 1) >> lane) - 1;
                    top[d + 1] = c;
                    dp[2 * kv(c) + 1] = (uint32_t)d + 1u;
                }
                e = ((e + 1) >> cnt) - 1;
            }
            top[e + 1] = x;
            return e;
        };
        int to_reach = A;
        while (n > 0 && to_reach > 0) {
            const u64 t = uni64(top[1]);
            const int u = kv(t);
            const uint32_t du = kd(t);
            const int so = uni(so_l[u]);
            int b = (int)((unsigned)so >> 8); // (unsigned: starts up to 2^24)
            const int lim = (so & 255) == 255 ? 64 * kRelax : (so & 255); // entries worth reading
            Ent en[kRelax];
#pragma unroll
            for (int q = 0; q < kRelax; q++) { // (entries past the sentinel re-read it)
                const int k = q * 64 + lane < lim ? q * 64 + lane : lim - 1;
                en[q] = sl[b + k];
            }
            const double ru = rel[u];
            // delete_max: the last node sinks from the root (branch-free walk)
            const int last = --n;
            if (last > 0) {
                const u64 x = uni64(top[last + 1]);
                const uint32_t dx = kd(x);
                int ev = 0;
                bool alive = true;
                for (;;) {
                    const int l = 2 * ev + 1;
                    const bool has = alive && l < n;
                    if (__ballot(has) == 0ull) break;
                    const uint4 pr = *reinterpret_cast<const uint4*>(top + l + 1);
                    const bool right = l + 1 < n && pr.w < pr.y;
                    const uint32_t dc = right ? pr.w : pr.y;
                    const uint32_t vc = right ? pr.z : pr.x;
                    const bool mv = has && dc < dx;
                    top[mv ? ev + 1 : 0] = ((u64)dc << 32) | vc;
                    *(mv ? &dp[2 * vc + 1] : pscr) = (uint32_t)ev + 1u;
                    ev = mv ? l + (right ? 1 : 0) : ev;
                    alive = mv;
                }
                const int e = __builtin_amdgcn_readfirstlane(ev);
                top[e + 1] = x;
                dp[2 * kv(x) + 1] = (uint32_t)e + 1u;
            }
            // kRelax batches are relaxed together (LDS gathers, then the
            // updates in incidence order): an update writes only its own
            // neighbour's dist, and a neighbour occurs once per list
            for (;;) {
                int end = 64 * kRelax;
#pragma unroll
                for (int q = kRelax - 1; q >= 0; q--) {
                    const unsigned long long m = __ballot(en[q].nbr < 0);
                    if (m) end = q * 64 + __builtin_ctzll(m);
                }
                bool imp[kRelax], fresh[kRelax];
                uint32_t alt[kRelax];
                double rv[kRelax];
#pragma unroll
                for (int q = 0; q < kRelax; q++) {
                    const bool ok = q * 64 + lane < end && en[q].nbr != u;
                    const uint32_t cd = ok ? dp[2 * en[q].nbr] : 0u;
                    alt[q] = du + en[q].w;
                    rv[q] = ru * en[q].rel;
                    fresh[q] = ok && cd == kInf;
                    imp[q] = ok && alt[q] < cd;
                }
#pragma unroll
                for (int q = 0; q < kRelax; q++) {
                    unsigned long long m = __ballot(imp[q]);
                    const unsigned long long fm = __ballot(fresh[q]);
                    while (m) { // igraph's order: incidence order, one edge at a time
                        const int l = __builtin_ctzll(m);
                        m &= m - 1;
                        const int vv = __builtin_amdgcn_readlane(en[q].nbr, l);
                        const uint32_t aa = (uint32_t)__builtin_amdgcn_readlane((int)alt[q], l);
                        const int e0 = (fm >> l) & 1ull ? n++ : (int)uni((int)dp[2 * vv + 1]) - 1;
                        const int e = up(e0, mk(aa, vv));
                        reinterpret_cast<u64*>(dp)[vv] = ((u64)(e + 1) << 32) | aa;
                        rel[vv] = readlane_d(rv[q], l);
                    }
                }
                if (end < 64 * kRelax) {
                    // the sentinel: -2 when u is an attached vertex
                    int sv = 0;
#pragma unroll
                    for (int q = 0; q < kRelax; q++)
                        if (end >= q * 64 && end < q * 64 + 64) sv = __builtin_amdgcn_readlane(en[q].nbr, end - q * 64);
                    if (sv == -2) --to_reach;
                    break;
                }
                b += 64 * kRelax; // lists longer than kRelax * 64 entries
#pragma unroll
                for (int q = 0; q < kRelax; q++) en[q] = sl[b + q * 64 + lane];
            }
        }
        wave_fence();
        write_row(g, row, src, tab, lane, [&](int v, double& l, double& r) {
            const uint32_t d = dp[2 * v];
            l = d == kInf ? -1.0 : (double)d;
            r = rel[v];
        });
        wave_fence();
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

// Released minimum of a device-resident table: min lat over (i, j), i < j,
// lat >= 0 (the pairs touch_all's row-by-row release stores).  Latencies
// are >= 0 doubles, whose bit patterns order like u64; ~0 = none.  One
// block per row range; lanes read consecutive entries of a row (coalesced).
__global__ __launch_bounds__(256) void k_min_upper(const ShdEntry* __restrict__ rows, int A, int row_lo, int row_hi,
                                                   unsigned long long* __restrict__ out) {
    unsigned long long m = ~0ull;
    for (int i = row_lo + (int)blockIdx.x; i < row_hi; i += gridDim.x) {
        const ShdEntry* row = rows + (size_t)(i - row_lo) * (size_t)A;
        for (int j = i + 1 + threadIdx.x; j < A; j += blockDim.x) {
            const double l = row[j].lat;
            if (l >= 0.0) {
                const unsigned long long b = (unsigned long long)__double_as_longlong(l);
                m = b < m ? b : m;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off);
        m = o < m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m != ~0ull) atomicMin(out, m);
}

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return shd_fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

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
    const char* kern = getenv("SHD_SSSP_KERNEL");
    // whole-ms latencies: the integer-key LDS kernel (SHD_SSSP_KERNEL=lds: the f64 one)
    if (g.V <= kLdsMaxV && g.sl && !(kern && strcmp(kern, "lds") == 0)) {
        const size_t lds = 8 * ((size_t)g.V + 2) + 8 * (size_t)g.V + 8 + 8 * (size_t)g.V + 4 * (size_t)g.V;
        if (lds > 65536 && (rc = hip_status(hipFuncSetAttribute((const void*)k_sssp_ilds,
                                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                                            "hipFuncSetAttribute")))
            return rc;
        hipLaunchKernelGGL(k_sssp_ilds, dim3(rows), dim3(64), lds, nullptr, g, row_lo, row_hi, tab);
        if ((rc = hip_status(hipGetLastError(), "k_sssp_ilds launch"))) return rc;
        return hip_status(hipDeviceSynchronize(), "k_sssp_ilds");
    }
    if (g.V <= kLdsMaxV) {
        const size_t lds = sizeof(HNode) * ((size_t)g.V + 1) + 20 * (size_t)g.V;
        // SHD_SSSP_LDS_SEQ=1: level-by-level sink and shift-up
        const char* sq = getenv("SHD_SSSP_LDS_SEQ");
        const bool dp = !(sq && atoi(sq) == 1);
        const void* kf = dp ? (const void*)k_sssp_lds<true> : (const void*)k_sssp_lds<false>;
        if (lds > 65536 &&
            (rc = hip_status(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                             "hipFuncSetAttribute")))
            return rc;
        if (dp) hipLaunchKernelGGL(k_sssp_lds<true>, dim3(rows), dim3(64), lds, nullptr, g, row_lo, row_hi, tab);
        else hipLaunchKernelGGL(k_sssp_lds<false>, dim3(rows), dim3(64), lds, nullptr, g, row_lo, row_hi, tab);
        if ((rc = hip_status(hipGetLastError(), "k_sssp_lds launch"))) return rc;
        return hip_status(hipDeviceSynchronize(), "k_sssp_lds");
    }
    if (!g.snb || !g.swr || !g.soff) return shd_fail(-EINVAL, "slab kernel needs the sentinel incidence arrays");
    if (kern && strcmp(kern, "blk") == 0) { // SHD_SSSP_KERNEL=blk: the blocked slab heap
        const size_t nblk = blk_count((long)g.V + 1);
        const size_t bstride = (nblk * 128 + 20 * (size_t)g.V + 255) & ~(size_t)255;
        int dev = 0, cus = 0;
        if ((rc = hip_status(hipGetDevice(&dev), "hipGetDevice")) ||
            (rc = hip_status(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev),
                             "hipDeviceGetAttribute")))
            return rc;
        // SHD_SSSP_WPE=7: 7 waves per SIMD (no register spills) instead of 8
        int wpe = 8;
        if (const char* e = getenv("SHD_SSSP_WPE")) wpe = atoi(e) == 7 ? 7 : 8;
        long waves = (long)cus * 4 * wpe;
        if (const char* e = getenv("SHD_SSSP_WAVES")) {
            const long x = atol(e);
            if (x > 0) waves = x;
        }
        if (waves > rows) waves = rows;
        int grid = (int)((waves + kSlabWaves - 1) / kSlabWaves);
        char* slab = nullptr;
        while (hipMalloc((void**)&slab, bstride * kSlabWaves * (size_t)grid) != hipSuccess) {
            (void)hipGetLastError();
            if (grid <= 16) return shd_fail(-ENOMEM, "cannot allocate SSSP workspace");
            grid /= 2;
        }
        const size_t lds = sizeof(HNode) * (kBlkTop + 1) * kSlabWaves;
        if (wpe == 7)
            hipLaunchKernelGGL(k_sssp_blk<7>, dim3(grid), dim3(64 * kSlabWaves), lds, nullptr, g, row_lo, row_hi, tab,
                               slab, bstride, nblk);
        else
            hipLaunchKernelGGL(k_sssp_blk<8>, dim3(grid), dim3(64 * kSlabWaves), lds, nullptr, g, row_lo, row_hi, tab,
                               slab, bstride, nblk);
        rc = hip_status(hipGetLastError(), "k_sssp_blk launch");
        if (!rc) rc = hip_status(hipDeviceSynchronize(), "k_sssp_blk");
        (void)hipFree(slab);
        return rc;
    }
    // whole-ms latencies: the integer-key blocked heap (SHD_SSSP_KERNEL=slab:
    // the f64 slab kernel for every graph)
    if (g.sl && !(kern && strcmp(kern, "slab") == 0)) {
        const size_t nblk = (size_t)ik::blk_count(g.V) + 1; // (+1: a right sibling block past the last)
        const size_t stride = (nblk * 128 + sizeof(ik::Rec) * (size_t)g.V + 255) & ~(size_t)255;
        int dev = 0, cus = 0;
        if ((rc = hip_status(hipGetDevice(&dev), "hipGetDevice")) ||
            (rc = hip_status(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev),
                             "hipDeviceGetAttribute")))
            return rc;
        int wpe = 8;
        if (const char* e = getenv("SHD_SSSP_WPE")) wpe = atoi(e) == 7 ? 7 : atoi(e) == 6 ? 6 : 8;
        long waves = (long)cus * 4 * wpe;
        if (const char* e = getenv("SHD_SSSP_WAVES")) {
            const long x = atol(e);
            if (x > 0) waves = x;
        }
        if (waves > rows) waves = rows;
        int grid = (int)((waves + kSlabWaves - 1) / kSlabWaves);
        char* slab = nullptr;
        while (hipMalloc((void**)&slab, stride * kSlabWaves * (size_t)grid) != hipSuccess) {
            (void)hipGetLastError();
            if (grid <= 16) return shd_fail(-ENOMEM, "cannot allocate SSSP workspace");
            grid /= 2;
        }
        const size_t lds = sizeof(unsigned long long) * (ik::kTop + 1) * kSlabWaves;
        unsigned* err = nullptr; // heap-consistency fault bits (raise)
        if ((rc = hip_status(hipMalloc((void**)&err, sizeof *err), "hipMalloc")) ||
            (rc = hip_status(hipMemset(err, 0, sizeof *err), "hipMemset"))) {
            (void)hipFree(slab);
            return rc;
        }
        // SHD_SSSP_STATS=1: the counting build of the kernel, totals to stderr
        const char* st_env = getenv("SHD_SSSP_STATS");
        unsigned long long* stats = nullptr;
        if (st_env && atoi(st_env) == 1 && hipMalloc((void**)&stats, 8 * ik::kStN) == hipSuccess) {
            (void)hipMemset(stats, 0, 8 * ik::kStN);
            hipLaunchKernelGGL(k_sssp_islab<true>, dim3(grid), dim3(64 * kSlabWaves), lds, nullptr, g, row_lo, row_hi,
                               tab, slab, stride, nblk, err, stats);
        } else if (wpe == 7) {
            hipLaunchKernelGGL((k_sssp_islab<false, 7>), dim3(grid), dim3(64 * kSlabWaves), lds, nullptr, g, row_lo,
                               row_hi, tab, slab, stride, nblk, err, nullptr);
        } else if (wpe == 6) {
            hipLaunchKernelGGL((k_sssp_islab<false, 6>), dim3(grid), dim3(64 * kSlabWaves), lds, nullptr, g, row_lo,
                               row_hi, tab, slab, stride, nblk, err, nullptr);
        } else {
            hipLaunchKernelGGL(k_sssp_islab<false>, dim3(grid), dim3(64 * kSlabWaves), lds, nullptr, g, row_lo, row_hi,
                               tab, slab, stride, nblk, err, nullptr);
        }
        rc = hip_status(hipGetLastError(), "k_sssp_islab launch");
        if (!rc) rc = hip_status(hipDeviceSynchronize(), "k_sssp_islab");
        if (stats) {
            unsigned long long h[ik::kStN] = {0};
            if (!rc && hipMemcpy(h, stats, sizeof h, hipMemcpyDeviceToHost) == hipSuccess) {
                static const char* nm[ik::kStN] = {"pops",      "sink_hbm_iters", "push",      "raise_hbm",
                                                   "raise_lds", "up_rounds",      "up_climbs", "log_overflow",
                                                   "batches",   "heap_size_sum",  "up_hbm_rounds"};
                for (int i = 0; i < ik::kStN; i++) fprintf(stderr, "islab_stat %s %llu\n", nm[i], h[i]);
            }
            (void)hipFree(stats);
        }
        unsigned herr = 0;
        if (!rc) rc = hip_status(hipMemcpy(&herr, err, sizeof herr, hipMemcpyDeviceToHost), "hipMemcpy");
        if (!rc && herr) rc = shd_fail(-EIO, "k_sssp_islab: heap position fault %#x", herr);
        (void)hipFree(err);
        (void)hipFree(slab);
        return rc;
    }
    // large graphs: persistent waves, one HBM slab each (heap V+2 nodes,
    // {dist, rel}, pos); SHD_SSSP_WAVES overrides the wave count
    const size_t stride = (sizeof(HNode) * ((size_t)g.V + 2) + 20 * (size_t)g.V + 255) & ~(size_t)255;
    int dev = 0, cus = 0;
    if ((rc = hip_status(hipGetDevice(&dev), "hipGetDevice")) ||
        (rc = hip_status(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev),
                         "hipDeviceGetAttribute")))
        return rc;
    // heap positions kept in LDS per wave (256: 32 waves/CU; 512: 20)
    int top_n = kTopDefault;
    if (const char* e = getenv("SHD_SSSP_TOP")) top_n = atoi(e) == 512 ? 512 : kTopDefault;
    long waves = (long)cus * (top_n == 512 ? 20 : kWavesPerCU);
    if (const char* e = getenv("SHD_SSSP_WAVES")) {
        const long x = atol(e);
        if (x > 0) waves = x;
    }
    if (waves > rows) waves = rows;
    int grid = (int)((waves + kSlabWaves - 1) / kSlabWaves);
    char* slab = nullptr;
    while (hipMalloc((void**)&slab, stride * kSlabWaves * (size_t)grid) != hipSuccess) {
        (void)hipGetLastError();
        if (grid <= 16) return shd_fail(-ENOMEM, "cannot allocate SSSP workspace");
        grid /= 2;
    }
    if (top_n == 512) {
        const size_t lds = sizeof(HNode) * 512 * kSlabWaves;
        if ((rc = hip_status(hipFuncSetAttribute((const void*)k_sssp_slab<512>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                             "hipFuncSetAttribute"))) {
            (void)hipFree(slab);
            return rc;
        }
        hipLaunchKernelGGL(k_sssp_slab<512>, dim3(grid), dim3(64 * kSlabWaves), lds, nullptr, g, row_lo, row_hi, tab,
                           slab, stride);
    } else {
        hipLaunchKernelGGL(k_sssp_slab<kTopDefault>, dim3(grid), dim3(64 * kSlabWaves),
                           sizeof(HNode) * kTopDefault * kSlabWaves, nullptr, g, row_lo, row_hi, tab, slab, stride);
    }
    rc = hip_status(hipGetLastError(), "k_sssp_slab launch");
    if (!rc) rc = hip_status(hipDeviceSynchronize(), "k_sssp_slab");
    (void)hipFree(slab);
    return rc;
}

extern "C" int shd_dev_min_upper(const ShdEntry* rows, int A, int row_lo, int row_hi, double* out) {
    *out = -1.0;
    if (A < 2 || row_hi <= row_lo) return 0;
    unsigned long long* d = nullptr;
    int rc = hip_status(hipMalloc((void**)&d, sizeof *d), "hipMalloc min");
    if (rc) return rc;
    unsigned long long h = ~0ull;
    if (!(rc = hip_status(hipMemcpy(d, &h, sizeof h, hipMemcpyHostToDevice), "hipMemcpy min"))) {
        const int nr = row_hi - row_lo;
        hipLaunchKernelGGL(k_min_upper, dim3(nr < 8192 ? nr : 8192), dim3(256), 0, nullptr, rows, A, row_lo, row_hi, d);
        rc = hip_status(hipGetLastError(), "k_min_upper launch");
        if (!rc) rc = hip_status(hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost), "hipMemcpy min");
    }
    (void)hipFree(d);
    if (!rc && h != ~0ull) memcpy(out, &h, sizeof h);
    return rc;
}
