/*
 * stub_dev.c -- TEST ONLY.  A host-memory stand-in for the device layer of
 * libshdnet (shd_internal.h: shd_dev_*), so that the product's host C
 * (topology.c, routes.c, round.c, gml.c, units.c) can be exercised for
 * thread safety under ThreadSanitizer on a machine without a GPU.  It never
 * ships: the product library links dev.hip / routing.hip / packet.hip.
 *
 * The "routing table" it builds is a fixed synthetic table (asymmetric, so
 * that the owner of a pair matters), not a routing computation: the thread
 * test checks the cache / release bookkeeping around the table, not the
 * table's values (those are checked on the GPU against the oracle).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "shd_internal.h"

int shd_dev_init(int device) { return device == 0 ? 0 : -ENODEV; }
int shd_dev_malloc(void** p, size_t bytes) {
    *p = malloc(bytes ? bytes : 4);
    return *p ? 0 : -ENOMEM;
}
int shd_dev_malloc_table(void** p, size_t bytes, int* contig) {
    if (contig) *contig = 0;
    return shd_dev_malloc(p, bytes);
}
int shd_dev_free(void* p) {
    free(p);
    return 0;
}
int shd_dev_h2d(void* d, const void* h, size_t bytes) {
    if (bytes) memcpy(d, h, bytes);
    return 0;
}
int shd_dev_d2d(void* d, const void* s, size_t bytes) {
    if (bytes) memcpy(d, s, bytes);
    return 0;
}
int shd_dev_d2h(void* h, const void* d, size_t bytes) {
    if (bytes) memcpy(h, d, bytes);
    return 0;
}
int shd_dev_memset(void* d, int v, size_t bytes) {
    memset(d, v, bytes);
    return 0;
}
int shd_dev_sync(void) { return 0; }
int shd_dev_stream_new(void** s) {
    *s = malloc(1);
    return *s ? 0 : -ENOMEM;
}
int shd_dev_stream_sync(void* s) { return 0; }
void shd_dev_stream_free(void* s) { free(s); }

/* entry (i, j) of the synthetic table */
void stub_entry(int i, int j, double* lat, double* rel) {
    uint32_t h = (uint32_t)i * 0x9E3779B1u ^ (uint32_t)j * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    *lat = 1.0 + (double)(h % 1000000u) / 1000.0;
    *rel = 0.5 + (double)((i * 29 + j * 53) % 41) / 100.0;
}

int shd_dev_fw_latency(const ShdGraphDev* g, double* d_lat, void** scratch, void* stream) {
    (void)g;
    (void)d_lat;
    (void)scratch;
    (void)stream;
    return -ENOTSUP;
}
void shd_dev_fw_scratch_free(void* scratch) { (void)scratch; }
int shd_dev_frontier_latency(const ShdGraphDev* g, int row_lo, int row_hi, int wmax, double* d_lat, void* stream) {
    (void)g;
    (void)row_lo;
    (void)row_hi;
    (void)wmax;
    (void)d_lat;
    (void)stream;
    return -ENOTSUP;
}

int shd_dev_build_rows(const ShdGraphDev* g, int use_sp, int row_lo, int row_hi, ShdEntry* tab) {
    (void)use_sp;
    for (int i = row_lo; i < row_hi; i++)
        for (int j = 0; j < g->A; j++) stub_entry(i, j, &tab[(size_t)i * g->A + j].lat, &tab[(size_t)i * g->A + j].rel);
    return 0;
}

int shd_dev_min_upper(const ShdEntry* rows, int A, int row_lo, int row_hi, double* out) {
    *out = -1.0;
    for (int i = row_lo; i < row_hi; i++)
        for (int j = i + 1; j < A; j++) {
            const double l = rows[(size_t)(i - row_lo) * A + j].lat;
            if (l >= 0 && (*out < 0 || l < *out)) *out = l;
        }
    return 0;
}

/* release: computed at launch on the host, kept until collect */
typedef struct {
    double* v;
    size_t n, cap;
} StubRel;
int shd_dev_release_launch(const ShdEntry* base, int A, const int32_t* rows, const uint32_t* seqs, int n,
                           const uint32_t* touch, void** scratch) {
    StubRel* s = (StubRel*)*scratch;
    if (!s && !(s = (StubRel*)calloc(1, sizeof *s))) return -ENOMEM;
    *scratch = s;
    if (s->n + (size_t)n > s->cap) {
        size_t nc = 2 * (s->n + (size_t)n) + 16;
        double* v = (double*)realloc(s->v, sizeof(double) * nc);
        if (!v) return -ENOMEM;
        s->v = v;
        s->cap = nc;
    }
    for (int r = 0; r < n; r++) {
        const ShdEntry* row = base + (size_t)rows[r] * (size_t)A;
        double m = -1.0;
        for (int j = 0; j < A; j++)
            if (j != rows[r] && touch[j] > seqs[r] && row[j].lat >= 0 && (m < 0 || row[j].lat < m)) m = row[j].lat;
        s->v[s->n++] = m;
    }
    return 0;
}
int shd_dev_release_collect(void* scratch, double* out, size_t cap, size_t* n) {
    StubRel* s = (StubRel*)scratch;
    *n = 0;
    if (!s || !s->n) return 0;
    if (s->n > cap) return -ENOSPC;
    memcpy(out, s->v, sizeof(double) * s->n);
    *n = s->n;
    s->n = 0;
    return 0;
}
size_t shd_dev_release_pending(void* scratch) { return scratch ? ((StubRel*)scratch)->n : 0; }
void shd_dev_release_scratch_free(void* scratch) {
    if (scratch) free(((StubRel*)scratch)->v);
    free(scratch);
}

int shd_dev_ws_new(void** ws) {
    *ws = malloc(1);
    return *ws ? 0 : -ENOMEM;
}
void shd_dev_ws_free(void* ws) { free(ws); }
int shd_dev_ws_scratch(void* ws, size_t dev_bytes, size_t host_bytes, void** d, void** h) {
    return shd_fail(-ENOSYS, "stub device: no exchange scratch");
}
int shd_dev_ws_check_faults(void* ws) { return 0; }
int shd_dev_ws_sync(void* ws, void* stream) { return 0; }
int shd_dev_mem_info(size_t* free_bytes, size_t* total_bytes) {
    *free_bytes = *total_bytes = (size_t)1 << 40;
    return 0;
}

int shd_dev_packet_round(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier, uint64_t end_time,
                         uint64_t bootstrap_end, ShdDeliv* d_out, uint32_t* d_dst_offsets, uint8_t* d_status,
                         uint64_t* d_counters, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no packet kernels");
}

int shd_dev_deliv_sort(void* ws, const ShdDeliv* d_in, size_t n, uint32_t host_lo, uint32_t host_hi, ShdDeliv* d_out,
                       uint32_t* d_dst_offsets, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no packet kernels");
}

int shd_dev_deliv_merge_runs(void* ws, const void* d_in, int wire, int sorted, size_t n, const uint32_t* d_rofs,
                             const uint32_t* d_bbase, uint32_t W, uint32_t host_lo, uint32_t host_hi, ShdDeliv* d_out,
                             uint32_t* d_dst_offsets, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no packet kernels");
}
int shd_dev_round_exchange(const ShdPktCtx* c, const ShdTransport* x, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                           uint64_t end_time, uint64_t bootstrap_end, const uint32_t* host_bounds, void* d_wire_send,
                           uint8_t* d_status, uint64_t* d_counters, void* d_wire_recv, size_t recv_cap,
                           ShdDeliv* d_out, uint32_t* d_out_offsets, size_t* n_out, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no exchange");
}

int shd_dev_route_records(const ShdPktCtx* c, const ShdTransport* x, const ShdPkt* d_recs, size_t n,
                          const uint32_t* row_bounds, ShdPkt* d_scratch, ShdPkt* d_recv, size_t recv_cap,
                          size_t* n_recv, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no exchange");
}
int shd_dev_event_cuts(void* ws, const uint32_t* d_dst_offsets, const uint32_t* host_bounds, int world,
                       uint64_t* send_elems, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no exchange");
}
int shd_dev_exchange_runs(void* ws, const ShdTransport* x, const ShdDeliv* d_events, const uint32_t* d_dst_offsets,
                          const uint32_t* host_bounds, ShdDeliv* d_recv, size_t recv_cap, ShdDeliv* d_out,
                          uint32_t* d_out_offsets, size_t* n_out, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no exchange");
}
int shd_dev_exchange_blocks(const ShdTransport* x, const void* d_send, const uint64_t* send_elems, size_t elem_bytes,
                            void* d_recv, size_t recv_cap, size_t* n_recv, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no exchange");
}

int shd_dev_ptab_build(const ShdEntry* tab, size_t nent, void* d_out, void* stream) {
    return shd_fail(-ENOSYS, "stub device: no packet table");
}

int shd_dev_gather_entries(const ShdEntry* tab, const uint64_t* d_idx, size_t n, ShdEntry* d_out) {
    for (size_t i = 0; i < n; i++) d_out[i] = tab[d_idx[i]];
    return 0;
}

int shd_dev_h2d_async(void* d, const void* h, size_t bytes, void* stream) { return shd_dev_h2d(d, h, bytes); }
int shd_dev_d2h_async(void* h, const void* d, size_t bytes, void* stream) { return shd_dev_d2h(h, d, bytes); }
int shd_dev_d2d_async(void* d, const void* s, size_t bytes, void* stream) { return shd_dev_d2d(d, s, bytes); }
int shd_dev_event_new(void** e) {
    *e = malloc(1);
    return *e ? 0 : -ENOMEM;
}
void shd_dev_event_free(void* e) { free(e); }
int shd_dev_stream_after(void* waiter, void* after, void* e) { return 0; }
int shd_host_alloc(void** p, size_t bytes) {
    *p = malloc(bytes ? bytes : 4);
    return *p ? 0 : -ENOMEM;
}
void shd_host_free(void* p) { free(p); }
int shd_dev_pcnt_spill(uint32_t* cnt, uint8_t* d8, size_t n, uint32_t thr, uint64_t* d_list, size_t cap,
                       uint32_t* d_nlist, size_t* appended) {
    size_t k = 0;
    for (size_t i = 0; i < n && k < cap; i++) {
        const uint32_t v = cnt[i] + (d8 ? d8[i] : 0u);
        if (v && v >= thr) {
            d_list[2 * k] = i;
            d_list[2 * k + 1] = v;
            cnt[i] = 0;
            if (d8) d8[i] = 0;
            k++;
        }
    }
    *d_nlist = (uint32_t)k;
    *appended = k;
    return 0;
}
int shd_dev_pcnt_fold(void* log, size_t L, uint32_t* dense, uint8_t* d8, uint64_t n0, uint64_t N, void** scratch,
                      void* stream) {
    for (size_t i = 0; i < L; i++) {
        const uint32_t k = ((const uint32_t*)log)[i];
        if (k == UINT32_MAX) continue;
        if (!d8) {
            dense[k]++;
        } else if (d8[k] == 255) { /* (the device fold moves a byte past 255 into the u32 counter) */
            dense[k] += 256;
            d8[k] = 0;
        } else {
            d8[k]++;
        }
    }
    return 0;
}
int shd_dev_pcnt_fold_reserve(size_t L, void** scratch) { return 0; }
void shd_dev_pcnt_scratch_free(void* scratch) { (void)scratch; }
