/*
 * routes.c -- building and holding the routing table in HBM.
 *
 * Layout: slots = attached vertices in ascending vertex index; the table is
 * a row-major A x A array of 16-byte {lat_ms, rel} entries, row = source
 * slot.  Row s, column d holds exactly what
 * _topology_computeSourcePaths (topology.c:1578-1814) would store for (s,d)
 * (self path for s == d, topology.c:1431-1576), or the direct edge for
 * use_shortest_path = false (topology.c:1816-1858).  A host mirror is kept
 * for the CPU-side lookups of the drop-in API.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "topology_impl.h"

void shd_topology_release_device(ShdTopology* t) {
    shd_shards_clear(t);
    if (t->d_tab && t->d_tab_owned) shd_dev_free(t->d_tab);
    shd_dev_free(t->d_inc_off);
    shd_dev_free(t->d_inc_nbr);
    shd_dev_free(t->d_inc_w);
    shd_dev_free(t->d_inc_r);
    shd_dev_free(t->d_slot_vertex);
    shd_dev_free(t->d_vertex_slot);
    shd_dev_free(t->d_host_info);
    shd_dev_free(t->d_touch);
    shd_dev_free(t->d_pair_bits);
    shd_dev_free(t->d_snb);
    shd_dev_free(t->d_swr);
    shd_dev_free(t->d_soff);
    shd_dev_free(t->d_sl);
    t->d_sl = NULL;
    t->d_snb = t->d_swr = NULL;
    t->d_soff = NULL;
    t->d_tab = NULL;
    t->d_host_info = NULL;
    t->d_inc_off = t->d_inc_nbr = t->d_slot_vertex = t->d_vertex_slot = NULL;
    t->d_inc_w = t->d_inc_r = NULL;
    t->d_touch = t->d_pair_bits = NULL;
}

#define UPLOAD(dst, src, bytes)                                   \
    do {                                                          \
        rc = shd_dev_malloc((void**)&(dst), ((bytes) != 0) ? (bytes) : 4); \
        if (!rc && ((bytes) != 0)) rc = shd_dev_h2d((dst), (src), (bytes)); \
        if (rc) goto fail;                                        \
    } while (0)

/* Slots, device CSR and host->slot map.  Idempotent until an attach.
 * Caller holds setup_mu. */
static int prepare(ShdTopology* t) {
    if (t->prepared && !t->routes_stale) return 0;
    int rc = shd_dev_init(t->device);
    if (rc) return rc;
    shd_topology_release_device(t);
    free(t->slot_vertex);
    free(t->vertex_slot);
    t->A = 0;
    t->slot_vertex = (int32_t*)malloc(sizeof(int32_t) * ((size_t)t->V + 1));
    t->vertex_slot = (int32_t*)malloc(sizeof(int32_t) * ((size_t)t->V + 1));
    for (int v = 0; v < t->V; v++) {
        t->vertex_slot[v] = t->v_attached[v] ? t->A : -1;
        if (t->v_attached[v]) t->slot_vertex[t->A++] = v;
    }
    if (t->A == 0) return shd_fail(-EINVAL, "no host is attached");
    size_t M = (size_t)t->M;
    double* w = (double*)malloc(sizeof(double) * (M + 1));
    double* r = (double*)malloc(sizeof(double) * (M + 1));
    free(t->h_host_info);
    uint32_t* hs = t->h_host_info = (uint32_t*)malloc(sizeof(uint32_t) * 2 * ((size_t)t->nhosts + 1));
    for (size_t k = 0; k < M; k++) {
        w[k] = t->e_ms[t->inc_eid[k]];
        r[k] = t->e_rel[t->inc_eid[k]];
    }
    for (uint32_t h = 0; h < t->nhosts; h++) {
        hs[2 * h] = t->host_vertex[h] >= 0 ? (uint32_t)t->vertex_slot[t->host_vertex[h]] : SHD_UNTOUCHED;
        hs[2 * h + 1] = SHD_UNTOUCHED;
    }
    UPLOAD(t->d_inc_off, t->inc_off, sizeof(int32_t) * ((size_t)t->V + 1));
    UPLOAD(t->d_inc_nbr, t->inc_nbr, sizeof(int32_t) * M);
    UPLOAD(t->d_inc_w, w, sizeof(double) * M);
    UPLOAD(t->d_inc_r, r, sizeof(double) * M);
    UPLOAD(t->d_slot_vertex, t->slot_vertex, sizeof(int32_t) * (size_t)t->A);
    UPLOAD(t->d_vertex_slot, t->vertex_slot, sizeof(int32_t) * (size_t)t->V);
    UPLOAD(t->d_host_info, hs, sizeof(uint32_t) * 2 * (size_t)t->nhosts);
    {
        /* sentinel-terminated lists for the slab kernel (shd_internal.h) */
        const size_t SM = M + (size_t)t->V + 64 * 16; /* a wave reads up to 16 batches of 64 past a list start */
        int32_t* snb = (int32_t*)calloc(2 * SM, sizeof(int32_t));
        double* swr = (double*)calloc(2 * SM, sizeof(double));
        int32_t* soff = (int32_t*)malloc(sizeof(int32_t) * ((size_t)t->V + 1));
        if (!snb || !swr || !soff) {
            free(snb);
            free(swr);
            free(soff);
            rc = -ENOMEM;
            goto fail;
        }
        /* a list handle packs the start (24 bits) with the number of entries
         * a first read needs, sentinel included (8 bits; 255 = "255 or more":
         * read whole batches) */
        if (SM >= (1u << 24)) {
            free(snb);
            free(swr);
            free(soff);
            rc = shd_fail(-ENOTSUP, "graph too large for 24-bit incidence list handles (%zu entries)", SM);
            goto fail;
        }
        for (int v = 0; v < t->V; v++) {
            const int32_t cnt = t->inc_off[v + 1] - t->inc_off[v] + 1;
            soff[v] = (int32_t)(((uint32_t)(t->inc_off[v] + v) << 8) | (uint32_t)(cnt < 255 ? cnt : 255));
        }
        for (int v = 0; v < t->V; v++) {
            size_t o = (size_t)((uint32_t)soff[v] >> 8);
            for (int32_t k = t->inc_off[v]; k < t->inc_off[v + 1]; k++, o++) {
                snb[2 * o] = t->inc_nbr[k];
                snb[2 * o + 1] = soff[t->inc_nbr[k]];
                swr[2 * o] = w[k];
                swr[2 * o + 1] = r[k];
            }
            snb[2 * o] = t->v_attached[v] ? -2 : -1;
        }
        for (size_t o = M + (size_t)t->V; o < SM; o++) snb[2 * o] = -1;
        /* integer-latency copy for k_sssp_islab: every latency a whole
         * number of ms and every path sum below 2^32 - 1 (a simple path has
         * < V edges) -- then u32 sums equal the f64 sums bit for bit */
        int int_ok = 1;
        double max_w = 0.0;
        for (size_t k = 0; k < M && int_ok; k++) {
            /* (range first: the cast of a value >= 2^32 is undefined) */
            if (!(w[k] >= 0.0 && w[k] < 4294967296.0) || w[k] != (double)(uint32_t)w[k]) int_ok = 0;
            else if (w[k] > max_w) max_w = w[k];
        }
        if (int_ok && (double)t->V * max_w >= 4294967295.0) int_ok = 0;
        if (int_ok) {
            /* {int32 nbr, uint32 w, double rel} */
            unsigned char* sl = (unsigned char*)calloc(SM, 16);
            if (!sl) {
                free(snb);
                free(swr);
                free(soff);
                rc = -ENOMEM;
                goto fail;
            }
            for (size_t o = 0; o < SM; o++) {
                const int32_t nbr = snb[2 * o];
                const uint32_t wi = nbr >= 0 ? (uint32_t)swr[2 * o] : 0u;
                memcpy(sl + 16 * o, &nbr, 4);
                memcpy(sl + 16 * o + 4, &wi, 4);
                memcpy(sl + 16 * o + 8, &swr[2 * o + 1], 8);
            }
            rc = shd_dev_malloc(&t->d_sl, 16 * SM);
            if (!rc) rc = shd_dev_h2d(t->d_sl, sl, 16 * SM);
            free(sl);
        }
        if (!rc) rc = shd_dev_malloc(&t->d_snb, sizeof(int32_t) * 2 * SM);
        if (!rc) rc = shd_dev_h2d(t->d_snb, snb, sizeof(int32_t) * 2 * SM);
        if (!rc) rc = shd_dev_malloc(&t->d_swr, sizeof(double) * 2 * SM);
        if (!rc) rc = shd_dev_h2d(t->d_swr, swr, sizeof(double) * 2 * SM);
        if (!rc) rc = shd_dev_malloc((void**)&t->d_soff, sizeof(int32_t) * (size_t)t->V);
        if (!rc) rc = shd_dev_h2d(t->d_soff, soff, sizeof(int32_t) * (size_t)t->V);
        free(snb);
        free(swr);
        free(soff);
        if (rc) goto fail;
    }
    free(w);
    free(r);
    hs = NULL;
    /* release state */
    free(t->touch);
    free(t->self_released);
    free(t->pair_bits);
    t->touch = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)t->A);
    memset(t->touch, 0xff, sizeof(uint32_t) * (size_t)t->A);
    t->self_released = (uint8_t*)calloc((size_t)t->A, 1);
    size_t nbits = (size_t)t->A * (size_t)t->A;
    t->pair_bits = t->use_sp ? NULL : (uint32_t*)calloc((nbits + 31) / 32, sizeof(uint32_t));
    t->next_touch = 0;
    rc = shd_dev_malloc((void**)&t->d_touch, sizeof(uint32_t) * (size_t)t->A);
    if (!rc && !t->use_sp && t->directed) rc = shd_dev_malloc((void**)&t->d_pair_bits, ((nbits + 31) / 32) * 4);
    if (rc) goto fail_nofree;
    t->touch_dirty = 1;
    t->prepared = 1;
    t->built = 0;
    t->routes_stale = 0;
    __atomic_store_n(&t->ready, 0, __ATOMIC_RELEASE);
    return 0;
fail:
    free(w);
    free(r);
fail_nofree:
    shd_topology_release_device(t);
    return rc;
}

static ShdGraphDev graph_dev(const ShdTopology* t) {
    ShdGraphDev g;
    g.V = t->V;
    g.A = t->A;
    g.M = t->M;
    g.directed = t->directed;
    g.inc_off = t->d_inc_off;
    g.inc_nbr = t->d_inc_nbr;
    g.inc_w = t->d_inc_w;
    g.inc_r = t->d_inc_r;
    g.slot_vertex = t->d_slot_vertex;
    g.vertex_slot = t->d_vertex_slot;
    g.snb = t->d_snb;
    g.swr = t->d_swr;
    g.soff = t->d_soff;
    g.sl = t->d_sl;
    return g;
}

static int adopt(ShdTopology* t, ShdEntry* d_tab, int owned) {
    size_t n = (size_t)t->A * (size_t)t->A;
    shd_shards_clear(t); /* (a device-resident table adopted before) */
    free(t->h_tab);
    t->h_tab = (ShdEntry*)malloc(sizeof(ShdEntry) * n);
    if (!t->h_tab) return -ENOMEM;
    int rc = shd_dev_d2h(t->h_tab, d_tab, sizeof(ShdEntry) * n);
    if (rc) return rc;
    if (t->d_tab && t->d_tab_owned && t->d_tab != d_tab) shd_dev_free(t->d_tab);
    shd_ptab_drop(t);
    if ((rc = shd_pcnt_drop(t, &t->pcnt))) return rc; /* (the counts so far stay, in the host map) */
    t->d_tab = d_tab;
    t->d_tab_owned = owned;
    t->tab_row_lo = 0;
    t->tab_row_hi = t->A;
    t->built = 1;
    __atomic_store_n(&t->ready, 1, __ATOMIC_RELEASE); /* publishes the immutable table to lock-free lookups */
    return 0;
}

static int build_routes_locked(ShdTopology* t) {
    if (t->built && !t->routes_stale) return 0;
    int rc = prepare(t);
    if (rc) return rc;
    ShdEntry* d_tab = NULL;
    rc = shd_dev_malloc_table((void**)&d_tab, sizeof(ShdEntry) * (size_t)t->A * (size_t)t->A, NULL);
    if (rc) return rc;
    ShdGraphDev g = graph_dev(t);
    rc = shd_dev_build_rows(&g, t->use_sp, 0, t->A, d_tab);
    if (!rc) rc = adopt(t, d_tab, 1);
    if (rc) shd_dev_free(d_tab);
    return rc;
}

int shd_topology_build_routes(ShdTopology* t) {
    if (!t) return -EINVAL;
    pthread_mutex_lock(&t->setup_mu);
    int rc = build_routes_locked(t);
    pthread_mutex_unlock(&t->setup_mu);
    return rc;
}

/* The first lookup builds the table (the reference computes rows lazily in
 * whichever worker misses, topology.c:1940-1961); later ones see `ready`. */
int shd_ensure_routes(ShdTopology* t) {
    if (__atomic_load_n(&t->ready, __ATOMIC_ACQUIRE)) return 0;
    return shd_topology_build_routes(t);
}

int shd_topology_slot_count(ShdTopology* t, int* A) {
    if (!t || !A) return -EINVAL;
    pthread_mutex_lock(&t->setup_mu);
    int rc = prepare(t);
    if (!rc) *A = t->A;
    pthread_mutex_unlock(&t->setup_mu);
    return rc;
}

int shd_topology_build_rows_device(ShdTopology* t, int row_lo, int row_hi, void* d_table) {
    if (!t || !d_table) return -EINVAL;
    pthread_mutex_lock(&t->setup_mu);
    int rc = prepare(t);
    if (!rc && (row_lo < 0 || row_hi > t->A || row_lo > row_hi)) rc = shd_fail(-EINVAL, "row range out of bounds");
    ShdGraphDev g = graph_dev(t);
    if (!rc) rc = shd_dev_build_rows(&g, t->use_sp, row_lo, row_hi, (ShdEntry*)d_table);
    pthread_mutex_unlock(&t->setup_mu);
    return rc;
}

int shd_topology_latency_table_fw(ShdTopology* t, void* d_lat, void* stream) {
    if (!t || !d_lat) return -EINVAL;
    pthread_mutex_lock(&t->setup_mu);
    int rc = prepare(t);
    ShdGraphDev g = graph_dev(t);
    if (!rc) rc = shd_dev_init(t->device);
    if (!rc) rc = shd_dev_fw_latency(&g, (double*)d_lat, &t->fw_scratch, stream);
    pthread_mutex_unlock(&t->setup_mu);
    if (!rc && !stream) rc = shd_dev_stream_sync(NULL); /* (NULL stream: the call is synchronous) */
    return rc;
}

int shd_topology_latency_rows_frontier(ShdTopology* t, int row_lo, int row_hi, void* d_lat, void* stream) {
    if (!t || !d_lat) return -EINVAL;
    pthread_mutex_lock(&t->setup_mu);
    int rc = prepare(t);
    if (!rc && (row_lo < 0 || row_hi > t->A || row_lo > row_hi)) rc = shd_fail(-EINVAL, "row range out of bounds");
    ShdGraphDev g = graph_dev(t);
    double wmax = 0.0;
    for (int e = 0; !rc && e < t->E; e++)
        if (t->e_ms[e] > wmax) wmax = t->e_ms[e];
    if (!rc) rc = shd_dev_init(t->device);
    if (!rc) rc = shd_dev_frontier_latency(&g, row_lo, row_hi, wmax > 2147483647.0 ? -1 : (int)wmax, (double*)d_lat,
                                           stream);
    pthread_mutex_unlock(&t->setup_mu);
    return rc;
}

/* ---- single-process multi-GPU build (shd_topology_build_shards) ---- */

/* The device graph arrays of prepare(), with their sizes (bytes). */
#define NGRAPH_ARRAYS 10
static void graph_arrays(ShdTopology* t, const void* src[NGRAPH_ARRAYS], size_t bytes[NGRAPH_ARRAYS]) {
    const size_t M = (size_t)t->M, V = (size_t)t->V, SM = M + V + 64 * 16;
    const void* s[NGRAPH_ARRAYS] = {t->d_inc_off, t->d_inc_nbr, t->d_inc_w, t->d_inc_r, t->d_slot_vertex,
                                    t->d_vertex_slot, t->d_snb, t->d_swr, t->d_soff, t->d_sl};
    const size_t b[NGRAPH_ARRAYS] = {4 * (V + 1), 4 * M, 8 * M, 8 * M, 4 * (size_t)t->A, 4 * V, 8 * SM, 16 * SM, 4 * V,
                                     t->d_sl ? 16 * SM : 0};
    for (int k = 0; k < NGRAPH_ARRAYS; k++) src[k] = s[k], bytes[k] = b[k];
}

typedef struct {
    ShdTopology* t;
    int device, lo, hi;
    ShdEntry* base;
    int rc;
    char err[256];
} ShardJob;

static void* build_shard(void* arg) {
    ShardJob* j = (ShardJob*)arg;
    ShdTopology* t = j->t;
    const void* src[NGRAPH_ARRAYS];
    size_t bytes[NGRAPH_ARRAYS];
    void* dst[NGRAPH_ARRAYS] = {0};
    graph_arrays(t, src, bytes);
    int rc = shd_dev_init(j->device);
    ShdGraphDev g = graph_dev(t);
    if (!rc && j->device != t->device) { /* the graph on this shard's device (peer copies) */
        for (int k = 0; k < NGRAPH_ARRAYS && !rc; k++)
            if (bytes[k] && !(rc = shd_dev_malloc(&dst[k], bytes[k]))) rc = shd_dev_d2d(dst[k], src[k], bytes[k]);
        g.inc_off = (const int32_t*)dst[0];
        g.inc_nbr = (const int32_t*)dst[1];
        g.inc_w = (const double*)dst[2];
        g.inc_r = (const double*)dst[3];
        g.slot_vertex = (const int32_t*)dst[4];
        g.vertex_slot = (const int32_t*)dst[5];
        g.snb = dst[6];
        g.swr = dst[7];
        g.soff = (const int32_t*)dst[8];
        g.sl = dst[9];
    }
    if (!rc) rc = shd_dev_build_rows(&g, t->use_sp, j->lo, j->hi, j->base);
    for (int k = 0; k < NGRAPH_ARRAYS; k++) shd_dev_free(dst[k]);
    j->rc = rc;
    if (rc) snprintf(j->err, sizeof j->err, "%s", shd_last_error());
    return NULL;
}

int shd_topology_build_shards(ShdTopology* t, int n, const int* devices, void* const* d_rows, const int* row_bounds) {
    if (!t || n < 1 || n > SHD_MAX_SHARDS || !devices || !d_rows || !row_bounds)
        return shd_fail(-EINVAL, "bad shard arguments");
    pthread_mutex_lock(&t->setup_mu);
    int rc = prepare(t);
    if (!rc && (row_bounds[0] != 0 || row_bounds[n] != t->A)) rc = shd_fail(-EINVAL, "row bounds must cover [0, %d)", t->A);
    for (int k = 0; k < n && !rc; k++)
        if (row_bounds[k + 1] < row_bounds[k]) rc = shd_fail(-EINVAL, "row bounds not ascending");
    ShardJob jobs[SHD_MAX_SHARDS];
    pthread_t th[SHD_MAX_SHARDS];
    int started[SHD_MAX_SHARDS] = {0};
    for (int k = 0; k < n && !rc; k++) {
        jobs[k] = (ShardJob){t, devices[k], row_bounds[k], row_bounds[k + 1],
                             (ShdEntry*)d_rows[k] - (ptrdiff_t)row_bounds[k] * (ptrdiff_t)t->A, 0, {0}};
        if (row_bounds[k + 1] > row_bounds[k]) started[k] = pthread_create(&th[k], NULL, build_shard, &jobs[k]) == 0;
        if (row_bounds[k + 1] > row_bounds[k] && !started[k]) rc = shd_fail(-EAGAIN, "cannot start a build thread");
    }
    for (int k = 0; k < n; k++)
        if (started[k]) {
            pthread_join(th[k], NULL);
            if (!rc && jobs[k].rc) rc = shd_fail(jobs[k].rc, "shard %d: %s", k, jobs[k].err);
        }
    pthread_mutex_unlock(&t->setup_mu);
    shd_dev_init(t->device);
    return rc;
}

int shd_topology_adopt_table_device(ShdTopology* t, void* d_table) {
    if (!t || !d_table) return -EINVAL;
    pthread_mutex_lock(&t->setup_mu);
    int rc = prepare(t);
    if (!rc) rc = adopt(t, (ShdEntry*)d_table, 0);
    pthread_mutex_unlock(&t->setup_mu);
    return rc;
}

int shd_topology_copy_table(ShdTopology* t, double* lat, double* rel, int32_t* slot_vertex, int cap) {
    if (!t) return -EINVAL;
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    if (cap < t->A) return shd_fail(-ENOSPC, "need %d slots", t->A);
    if (!t->h_tab) return shd_fail(-ENOTSUP, "the table is device-resident (no host mirror)");
    size_t n = (size_t)t->A * (size_t)t->A;
    for (size_t k = 0; k < n; k++) {
        if (lat) lat[k] = t->h_tab[k].lat;
        if (rel) rel[k] = t->h_tab[k].rel;
    }
    if (slot_vertex) memcpy(slot_vertex, t->slot_vertex, sizeof(int32_t) * (size_t)t->A);
    return 0;
}

/* Uploads the release state the packet kernel reads (touch order or pair
 * bits) if it changed since the last upload. */
int shd_sync_touch(ShdTopology* t) {
    if (!__atomic_exchange_n(&t->touch_dirty, 0, __ATOMIC_ACQ_REL)) return 0;
    int rc = shd_dev_h2d(t->d_touch, t->touch, sizeof(uint32_t) * (size_t)t->A);
    /* per-host {slot, touch[slot]} records: one 8-byte gather per endpoint */
    uint32_t* hs = t->h_host_info;
    for (uint32_t h = 0; h < t->nhosts; h++)
        hs[2 * h + 1] = hs[2 * h] != SHD_UNTOUCHED ? t->touch[hs[2 * h]] : SHD_UNTOUCHED;
    if (!rc) rc = shd_dev_h2d(t->d_host_info, hs, sizeof(uint32_t) * 2 * (size_t)t->nhosts);
    if (!rc && t->d_pair_bits) {
        size_t nbits = (size_t)t->A * (size_t)t->A;
        rc = shd_dev_h2d(t->d_pair_bits, t->pair_bits, ((nbits + 31) / 32) * 4);
    }
    if (rc) __atomic_store_n(&t->touch_dirty, 1, __ATOMIC_RELEASE);
    return rc;
}

/* SHD_PTAB=0 keeps the rounds on the 16-B f64 entries (A/B measurements). */
static int ptab_enabled(void) {
    const char* v = getenv("SHD_PTAB");
    return !(v && strcmp(v, "0") == 0);
}

void shd_ptab_drop(ShdTopology* t) {
    shd_dev_free(t->d_ptab_alloc);
    t->d_ptab_alloc = t->d_ptab = NULL;
    t->ptab_unavailable = 0;
}

/* The rounds' 8-byte form of the resident rows (packet.hip kPtabFallback):
 * {delay_ns, keep threshold} per entry, converted once per adopted table.
 * Half the bytes of the random gather's footprint; the f64 table stays for
 * the lookups.  It is an optional copy (C4: 60 GB beside the 120 GB table),
 * so it is built only when it takes at most half of the free device memory
 * and leaves kPtabHeadroom for the round workspace and the caller's buffers;
 * otherwise, or if the allocation fails, the rounds read the f64 entries
 * (and shd_ptab_release_for_retry drops it when a later allocation fails).
 * SHD_PTAB_MAX_BYTES caps it (tests of the f64 path). */
#define SHD_PTAB_HEADROOM (8ull << 30)
int shd_ensure_ptab(ShdTopology* t) {
    if (t->d_ptab || t->ptab_unavailable || !t->d_tab || !ptab_enabled()) return 0;
    const size_t rows = (size_t)(t->tab_row_hi - t->tab_row_lo), A = (size_t)t->A;
    if (!rows) return 0;
    const size_t need = rows * A * 8;
    size_t fr = 0, tot = 0;
    const char* mx = getenv("SHD_PTAB_MAX_BYTES");
    if ((mx && need > (size_t)strtoull(mx, NULL, 10)) || shd_dev_mem_info(&fr, &tot) || need > fr / 2 ||
        fr - need < SHD_PTAB_HEADROOM) {
        t->ptab_unavailable = 1;
        return 0;
    }
    void* d = NULL;
    if (shd_dev_malloc(&d, need)) {
        t->ptab_unavailable = 1;
        return 0;
    }
    int rc = shd_dev_ptab_build(t->d_tab + (size_t)t->tab_row_lo * A, rows * A, d, NULL);
    if (rc) {
        shd_dev_free(d);
        return rc;
    }
    t->d_ptab_alloc = d;
    t->d_ptab = (char*)d - (ptrdiff_t)((size_t)t->tab_row_lo * A * 8);
    return 0;
}

/* A round allocation failed (-ENOMEM) while the optional 8-B table holds
 * device memory: drop it for good (the f64 entries decide) and say whether
 * the caller should retry. */
int shd_ptab_release_for_retry(ShdTopology* t, int rc) {
    if (rc != -ENOMEM || !t->d_ptab_alloc) return 0;
    shd_ptab_drop(t);
    t->ptab_unavailable = 1;
    return 1;
}

/* ---- device path packet counters (topology_incrementPathPacketCounter of
 * every kept packet, worker.c:551 / topology.c:1983-1993, counted by the
 * round kernels) ----
 * Dense u32 counters per resident table entry.  The round kernels log each
 * record's answering-pair key (one coalesced store per record, inside the
 * round) and the log is added into the counters in bulk -- when it is full,
 * before anything reads the counters (shd_pcnt_sync), or when the caller
 * asks (shd_topology_path_counts_sync) -- by shd_dev_pcnt_fold.  The
 * per-packet device atomic (SHD_PCNT=atomic) costs the round +0.365 ms at
 * C3. */

/* SHD_PCNT: "log" (the default where the fold applies: tables of at most
 * SHD_PCNT_FOLD_MAX_N = 2^29 entries, C1-C3), "atomic" (one device atomic
 * per kept packet: the default above, C4's 7.5e9-entry table, whose 1M-packet
 * rounds spend ~0.04 ms on them), "0" (measurement only: counts are not
 * kept). */
static int pcnt_mode_of(const ShdTopology* t, const ShdPcnt* p) {
    const char* v = getenv("SHD_PCNT");
    if (v && strcmp(v, "0") == 0) return 0;
    if (v && strcmp(v, "atomic") == 0) return 2;
    return (uint64_t)p->hi * (uint64_t)t->A <= SHD_PCNT_FOLD_MAX_N ? 1 : 2;
}

/* Spill threshold: counters >= T move to the host map once the packets
 * counted since the last spill could reach T (T + T < 2^32: no counter
 * wraps).  SHD_PCNT_SPILL_AT (tests) lowers T. */
static uint64_t pcnt_spill_at(void) {
    const char* v = getenv("SHD_PCNT_SPILL_AT");
    const uint64_t x = v ? strtoull(v, NULL, 10) : 0;
    return x >= 1 && x <= (1ull << 31) ? x : (1ull << 31);
}

/* Log capacity in records: SHD_PCNT_LOG (tests), else 2^28 (1 GB of u32
 * keys, ~27 rounds of 10M packets), at least one round. */
static size_t pcnt_log_cap(size_t n) {
    const char* v = getenv("SHD_PCNT_LOG");
    size_t c = v ? (size_t)strtoull(v, NULL, 10) : ((size_t)1 << 28);
    if (c < 1) c = 1;
    return c > n ? c : n;
}

static int pcnt_dev(ShdTopology* t, const ShdPcnt* p) {
    for (const ShdShard* s = t->shards; s < t->shards + t->nshards; s++)
        if (p == &s->pcnt) return s->device;
    return t->device;
}

/* Host-log mode: counts every logged key (global row * A + col; all-ones:
 * not kept) into the host map, in chunks of at most 2^22 records. */
static int pcnt_drain_host(ShdTopology* t, ShdPcnt* p) {
    if (!p->log_fill) return 0;
    int rc = shd_dev_init(p->device);
    if (!rc) rc = shd_dev_sync(); /* every round that wrote the log has finished */
    const size_t ksz = p->log64 ? 8 : 4, chunk = (size_t)1 << 22, A = (size_t)t->A;
    void* h = malloc(ksz * (p->log_fill < chunk ? p->log_fill : chunk));
    if (!h && !rc) rc = -ENOMEM;
    for (size_t off = 0; !rc && off < p->log_fill; off += chunk) {
        const size_t m = p->log_fill - off < chunk ? p->log_fill - off : chunk;
        if ((rc = shd_dev_d2h(h, (const char*)p->log + off * ksz, m * ksz))) break;
        pthread_mutex_lock(&t->pkt_mu);
        for (size_t k = 0; k < m && !rc; k++) {
            const uint64_t key = p->log64 ? ((const uint64_t*)h)[k] : ((const uint32_t*)h)[k];
            if (key == (p->log64 ? UINT64_MAX : (uint64_t)UINT32_MAX)) continue;
            rc = shd_count_packet_locked(t, (int)(key / A), (int)(key % A), 1);
        }
        pthread_mutex_unlock(&t->pkt_mu);
    }
    free(h);
    if (!rc) p->log_fill = 0;
    shd_dev_init(t->device);
    return rc;
}

/* Adds the log into the counters (synchronous: every round that wrote it
 * has finished -- they may have run on any stream). */
static int pcnt_fold(ShdTopology* t, ShdPcnt* p) {
    if (p->hostlog) return pcnt_drain_host(t, p);
    if (!p->alloc || !p->log_fill) return 0;
    int rc = shd_dev_init(p->device);
    if (!rc) rc = shd_dev_sync();
    /* SHD_FOLD_D8=0 (A/B): this fold adds into the u32 counters (the deltas
     * already held stay counted: reads sum both) */
    const char* d8v = getenv("SHD_FOLD_D8");
    uint8_t* d8 = d8v && !strcmp(d8v, "0") ? NULL : p->d8;
    if (!rc)
        rc = shd_dev_pcnt_fold(p->log, p->log_fill, p->base, d8, (uint64_t)(p->lo) * (uint64_t)t->A,
                               (uint64_t)(p->hi) * (uint64_t)t->A, &p->fold, NULL);
    if (!rc) rc = shd_dev_sync();
    if (!rc) p->log_fill = 0;
    shd_dev_init(t->device);
    return rc;
}

/* Moves every counter >= thr of p into the host map (pkt_mu taken here). */
static int pcnt_spill(ShdTopology* t, ShdPcnt* p, uint32_t thr) {
    if (!p->alloc || p->hi <= p->lo) return 0;
    int rc = pcnt_fold(t, p);
    if (rc) return rc;
    const size_t A = (size_t)t->A, n = (size_t)(p->hi - p->lo) * A;
    const size_t cap = n < (1u << 22) ? n : (1u << 22);
    rc = shd_dev_init(p->device);
    if (!rc) rc = shd_dev_sync(); /* rounds on any stream have counted */
    uint64_t* d_list = NULL;
    uint32_t* d_n = NULL;
    uint64_t* h = (uint64_t*)malloc(16 * cap);
    if (!h) rc = -ENOMEM;
    if (!rc && !(rc = shd_dev_malloc((void**)&d_list, 16 * cap))) rc = shd_dev_malloc((void**)&d_n, 4);
    for (size_t got = cap; !rc && got == cap;) {
        if ((rc = shd_dev_pcnt_spill(p->alloc, p->d8 ? p->d8 + (size_t)p->lo * A : NULL, n, thr, d_list, cap, d_n,
                                     &got)) ||
            !got)
            break;
        if ((rc = shd_dev_d2h(h, d_list, 16 * got))) break;
        pthread_mutex_lock(&t->pkt_mu);
        if (!(rc = shd_count_reserve_locked(t, got)))
            for (size_t k = 0; k < got && !rc; k++)
                rc = shd_count_packet_locked(t, p->lo + (int)(h[2 * k] / A), (int)(h[2 * k] % A), h[2 * k + 1]);
        pthread_mutex_unlock(&t->pkt_mu);
    }
    shd_dev_free(d_list);
    shd_dev_free(d_n);
    free(h);
    shd_dev_init(t->device);
    return rc;
}

int shd_pcnt_ensure(ShdTopology* t, ShdPcnt* p, int lo, int hi, size_t n) {
    p->cur = NULL;
    p->mode = 0;
    ShdPcnt want = *p;
    want.lo = lo;
    want.hi = hi;
    const int mode = pcnt_mode_of(t, &want);
    if (!mode || hi <= lo) return 0;
    int rc = 0;
    if (p->alloc && (p->lo != lo || p->hi != hi) && (rc = shd_pcnt_drop(t, p))) return rc;
    const int dev = pcnt_dev(t, p);
    /* SHD_DEBUG_PCNT_OOM (tests): "1" the dense counters' allocation fails as
     * on a full device; "64" also with u64 log keys */
    const char* oom = getenv("SHD_DEBUG_PCNT_OOM");
    if (!p->alloc && !p->hostlog) {
        const size_t bytes = (size_t)(hi - lo) * (size_t)t->A * 4;
        void* d = NULL;
        rc = oom && *oom && strcmp(oom, "0") ? -ENOMEM : shd_dev_malloc(&d, bytes);
        if (rc == -ENOMEM && !oom && t->d_ptab_alloc) { /* the counters are worth more than the 8-B table */
            shd_ptab_drop(t);
            t->ptab_unavailable = 1;
            rc = shd_dev_malloc(&d, bytes);
        }
        if (!rc && ((rc = shd_dev_memset(d, 0, bytes)) || (rc = shd_dev_sync()))) shd_dev_free(d);
        if (rc == -ENOMEM) { /* bounded fallback: log on the device, count on the host */
            p->hostlog = 1;
            p->device = dev;
            p->log_fill = 0;
            rc = 0;
        } else if (rc) {
            return rc;
        } else {
            p->alloc = (uint32_t*)d;
            p->base = p->alloc - (ptrdiff_t)lo * (ptrdiff_t)t->A;
            p->lo = lo;
            p->hi = hi;
            p->device = dev;
            p->budget = 0;
            /* the fold's u8 delta layer (log-mode tables only; without it --
             * no memory -- the fold adds into the u32 counters) */
            size_t fr = 0, tot = 0;
            if ((uint64_t)hi * (uint64_t)t->A <= SHD_PCNT_FOLD_MAX_N && !shd_dev_mem_info(&fr, &tot) &&
                fr > bytes / 4 + ((size_t)1 << 30)) { /* (headroom: no failed allocation left behind) */
                const size_t first = (size_t)lo * (size_t)t->A, off = first & 15u;
                void* d8 = NULL;
                if (!shd_dev_malloc(&d8, bytes / 4 + 32)) {
                    if (shd_dev_memset(d8, 0, bytes / 4 + 32) || shd_dev_sync()) {
                        shd_dev_free(d8);
                    } else {
                        p->d8_alloc = (uint8_t*)d8;
                        p->d8 = p->d8_alloc + off - first; /* (16-B aligned: hipMalloc is) */
                    }
                }
            }
        }
    }
    if (p->hostlog) {
        const int log64 = ((uint64_t)hi * (uint64_t)t->A > (uint64_t)UINT32_MAX) || (oom && !strcmp(oom, "64"));
        if (log64 != p->log64 || p->log_fill + n > p->log_cap) { /* drain, then re-size when needed */
            if ((rc = pcnt_drain_host(t, p))) return rc;
            if (log64 != p->log64 || n > p->log_cap || !p->log) {
                shd_dev_init(dev);
                shd_dev_free(p->log);
                p->log = NULL;
                p->log_cap = 0;
                p->log64 = log64;
                size_t cap = pcnt_log_cap(n);
                if (cap > ((size_t)1 << 26) && n <= ((size_t)1 << 26)) cap = (size_t)1 << 26; /* <= 512 MB */
                if ((rc = shd_dev_malloc(&p->log, cap * (log64 ? 8 : 4)))) return rc;
                p->log_cap = cap;
            }
        }
        p->lo = lo; /* (keys are global: a new row range needs no drain) */
        p->hi = hi;
        p->mode = 1;
        p->cur = (char*)p->log + p->log_fill * (p->log64 ? 8 : 4);
        p->cur_n = n;
        return shd_dev_init(dev);
    }
    const uint64_t T = pcnt_spill_at();
    if (p->budget + n >= T) { /* a counter below T could otherwise pass 2^32 - 1 */
        if ((rc = pcnt_spill(t, p, (uint32_t)T))) return rc;
        p->budget = 0;
    }
    p->budget += n;
    p->mode = mode;
    if (mode == 2) return shd_dev_init(dev);
    const size_t ksz = 4; /* (log mode: u32 keys, the table is below 2^29 entries) */
    if (p->log_fill + n > p->log_cap) {
        if ((rc = pcnt_fold(t, p))) return rc;
        if (n > p->log_cap || !p->log) {
            shd_dev_init(dev);
            shd_dev_free(p->log);
            p->log = NULL;
            p->log_cap = 0;
            const size_t cap = pcnt_log_cap(n);
            /* the log and the fold's buffers for a full log: a fold inside a
             * timed region allocates nothing */
            if ((rc = shd_dev_malloc(&p->log, cap * ksz)) || (rc = shd_dev_pcnt_fold_reserve(cap, &p->fold))) return rc;
            p->log_cap = cap;
        }
    }
    /* this round's slice; shd_pcnt_commit adds it to the log once the round
     * is launched (a round that fails before leaves it out) */
    p->cur = (char*)p->log + p->log_fill * ksz;
    p->cur_n = n;
    return shd_dev_init(dev);
}

void shd_pcnt_ctx(const ShdPcnt* p, ShdPktCtx* c) {
    c->plog = p->cur;
    c->plog64 = p->cur ? (uint32_t)p->log64 : 0u;
    c->pcnt = p->mode == 2 ? p->base : NULL;
}

void shd_pcnt_commit(ShdPcnt* p, int rc) {
    if (!rc && p->cur) p->log_fill += p->cur_n;
    p->cur = NULL;
    p->cur_n = 0;
}

/* caller holds round_mu -- and keeps it across its reads of the counters,
 * so no re-adoption (shd_shards_clear) can free them in between */
int shd_pcnt_sync_locked(ShdTopology* t) {
    int rc = pcnt_fold(t, &t->pcnt);
    for (int k = 0; k < t->nshards && !rc; k++) rc = pcnt_fold(t, &t->shards[k].pcnt);
    return rc;
}

int shd_pcnt_sync(ShdTopology* t) {
    pthread_mutex_lock(&t->round_mu);
    int rc = shd_pcnt_sync_locked(t);
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}

int shd_topology_path_counts_sync(ShdTopology* t) {
    if (!t) return -EINVAL;
    return shd_pcnt_sync(t);
}

int shd_pcnt_drop(ShdTopology* t, ShdPcnt* p) {
    if (!p->alloc && !p->hostlog) return 0;
    int rc = p->hostlog ? pcnt_drain_host(t, p) : pcnt_spill(t, p, 1u); /* (folds the log first) */
    shd_dev_init(p->device);
    shd_dev_free(p->alloc);
    shd_dev_free(p->d8_alloc);
    shd_dev_free(p->log);
    shd_dev_pcnt_scratch_free(p->fold);
    memset(p, 0, sizeof *p);
    shd_dev_init(t->device);
    return rc;
}

void shd_pcnt_discard(ShdTopology* t) {
    ShdPcnt* ps[SHD_MAX_SHARDS + 1];
    int n = 0;
    ps[n++] = &t->pcnt;
    for (int k = 0; k < t->nshards; k++) ps[n++] = &t->shards[k].pcnt;
    for (int k = 0; k < n; k++)
        if (ps[k]->alloc || ps[k]->hostlog) {
            shd_dev_init(ps[k]->device);
            shd_dev_free(ps[k]->alloc);
            shd_dev_free(ps[k]->d8_alloc);
            shd_dev_free(ps[k]->log);
            shd_dev_pcnt_scratch_free(ps[k]->fold);
            memset(ps[k], 0, sizeof *ps[k]);
        }
    shd_dev_init(t->device);
}

static ShdPcnt* pcnt_of(ShdTopology* t, int row) {
    ShdPcnt* p = &t->pcnt;
    if (t->nshards > 1) {
        ShdShard* s = shd_shard_of(t, row);
        p = s ? &s->pcnt : NULL;
    }
    return p && p->alloc && row >= p->lo && row < p->hi ? p : NULL;
}

/* (the readers run shd_pcnt_sync first: the log is folded) */
int shd_pcnt_read(ShdTopology* t, int row, int col, uint64_t* v) {
    *v = 0;
    ShdPcnt* p = pcnt_of(t, row);
    if (!p) return 0;
    uint32_t x = 0;
    uint8_t y = 0;
    const size_t k = (size_t)row * (size_t)t->A + (size_t)col;
    int rc = shd_dev_init(p->device);
    if (!rc) rc = shd_dev_sync();
    if (!rc) rc = shd_dev_d2h(&x, p->base + k, 4);
    if (!rc && p->d8) rc = shd_dev_d2h(&y, p->d8 + k, 1); /* (the fold's delta layer) */
    *v = (uint64_t)x + y;
    shd_dev_init(t->device);
    return rc;
}

int shd_pcnt_read_row(ShdTopology* t, int row, uint64_t* out) { return shd_pcnt_read_rows(t, row, row + 1, out); }

int shd_pcnt_read_rows(ShdTopology* t, int lo, int hi, uint64_t* out) {
    const size_t A = (size_t)t->A;
    const size_t chunk_rows = A ? ((size_t)1 << 24) / A + 1 : 1; /* ~64 MB of u32 per copy */
    uint32_t* x = NULL;
    uint8_t* y = NULL;
    int rc = 0;
    for (int i = lo; i < hi && !rc;) {
        ShdPcnt* p = pcnt_of(t, i);
        if (!p) {
            i++;
            continue;
        }
        int e = hi < p->hi ? hi : p->hi;
        if ((size_t)(e - i) > chunk_rows) e = i + (int)chunk_rows;
        const size_t m = (size_t)(e - i) * A;
        if (!x && !(x = (uint32_t*)malloc(4 * (chunk_rows < (size_t)(hi - lo) ? chunk_rows : (size_t)(hi - lo)) * A)))
            return -ENOMEM;
        if (p->d8 && !y && !(y = (uint8_t*)malloc((chunk_rows < (size_t)(hi - lo) ? chunk_rows : (size_t)(hi - lo)) * A))) {
            free(x);
            return -ENOMEM;
        }
        if (!(rc = shd_dev_init(p->device)) && !(rc = shd_dev_sync()))
            rc = shd_dev_d2h(x, p->base + (size_t)i * A, 4 * m);
        if (!rc && p->d8) rc = shd_dev_d2h(y, p->d8 + (size_t)i * A, m); /* (the fold's delta layer) */
        uint64_t* o = out + (size_t)(i - lo) * A;
        for (size_t k = 0; !rc && k < m; k++) o[k] += (uint64_t)x[k] + (p->d8 ? y[k] : 0u);
        i = e;
    }
    free(x);
    free(y);
    shd_dev_init(t->device);
    return rc;
}

void shd_pkt_ctx(ShdTopology* t, ShdPktCtx* c) {
    c->tab = t->d_tab;
    c->A = t->A;
    c->mode = t->use_sp ? 0 : (t->directed ? 2 : 1);
    c->touch = t->d_touch;
    c->pair_bits = t->d_pair_bits;
    c->host_info = t->d_host_info;
    c->nhosts = t->nhosts;
    c->row_lo = t->tab_row_lo;
    c->row_hi = t->tab_row_hi;
    c->idx_base = 0;
    c->ptab = ptab_enabled() ? t->d_ptab : NULL;
    shd_pcnt_ctx(&t->pcnt, c); /* (shd_pcnt_ensure ran first) */
    if (!t->ws) shd_dev_ws_new(&t->ws); /* (a failure leaves ws NULL: the launch reports -ENOMEM) */
    c->ws = t->ws;
}

int shd_device_alloc_table(int device, size_t bytes, void** d_out, int* contiguous) {
    if (!d_out) return -EINVAL;
    *d_out = NULL;
    int rc = shd_dev_init(device);
    return rc ? rc : shd_dev_malloc_table(d_out, bytes, contiguous);
}

int shd_device_free(int device, void* d_ptr) {
    int rc = shd_dev_init(device);
    return rc ? rc : shd_dev_free(d_ptr);
}

int shd_device_copy(int device, void* d_dst, const void* d_src, size_t bytes) {
    if ((!d_dst || !d_src) && bytes) return -EINVAL;
    int rc = shd_dev_init(device);
    return rc ? rc : shd_dev_d2d(d_dst, d_src, bytes);
}
