/*
 * round.c -- host side of the batched packet hand-off that replaces the body
 * of worker_sendPacket (core/worker.c:517-576) + scheduler_push
 * (core/scheduler/scheduler.c:232-255) + the host-single policy push
 * (scheduler_policy_host_single.c:174-220).
 *
 * At send time each worker thread calls shd_round_append_worker: the lookup
 * side effects of topology_getReliability (row touch, min-jump) happen right
 * there, in send order, exactly where the reference's lookup happens
 * (worker.c:539), and the record -- which carries the sender's reserved
 * rand_r pre-state -- goes to that worker's own buffer (no lock between
 * workers).  At the round boundary (manager.c:563-573, all workers idle)
 * shd_round_collect ships the batch to the GPU, which decides loss, computes
 * and clamps delivery times and groups the events per destination in
 * event_compare order.  Batching is exact because inter-host deliveries are
 * clamped to >= the barrier (host_single.c:187-192), so none of them runs in
 * the round that sent it.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "topology_impl.h"

int shd_round_set_workers(ShdTopology* t, int nworkers) {
    if (!t || nworkers < 1 || nworkers > 4096) return shd_fail(-EINVAL, "worker count %d out of range", nworkers);
    pthread_mutex_lock(&t->round_mu);
    int rc = 0;
    for (int w = 0; w < t->nworkers; w++)
        if (t->wbuf[w].n) rc = shd_fail(-EBUSY, "records are staged; collect the round first");
    if (!rc) {
        ShdWorkerBuf* nb = (ShdWorkerBuf*)calloc((size_t)nworkers, sizeof(ShdWorkerBuf));
        if (!nb) rc = -ENOMEM;
        else {
            for (int w = 0; w < t->nworkers; w++) free(t->wbuf[w].recs);
            free(t->wbuf);
            t->wbuf = nb;
            t->nworkers = nworkers;
        }
    }
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}

int shd_round_begin(ShdTopology* t, uint64_t barrier, uint64_t end_time, uint64_t bootstrap_end) {
    if (!t) return -EINVAL;
    pthread_mutex_lock(&t->round_mu);
    t->barrier = barrier;
    t->end_time = end_time;
    t->bootstrap_end = bootstrap_end;
    for (int w = 0; w < t->nworkers; w++) t->wbuf[w].n = 0;
    pthread_mutex_unlock(&t->round_mu);
    return 0;
}

/* Slots of a record's endpoints, or -ENOENT (no side effect). */
static int rec_slots(const ShdTopology* t, const ShdPkt* p, int* si, int* di) {
    if (p->src_host >= t->nhosts || p->dst_host >= t->nhosts || t->host_vertex[p->src_host] < 0 ||
        t->host_vertex[p->dst_host] < 0)
        return -ENOENT;
    *si = t->vertex_slot[t->host_vertex[p->src_host]];
    *di = t->vertex_slot[t->host_vertex[p->dst_host]];
    return 0;
}

int shd_round_append_worker(ShdTopology* t, int worker, const ShdPkt* recs, size_t n) {
    if (!t || (!recs && n) || worker < 0 || worker >= t->nworkers) return shd_fail(-EINVAL, "bad append arguments");
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    if (!__atomic_load_n(&t->lookups_started, __ATOMIC_RELAXED)) __atomic_store_n(&t->lookups_started, 1, __ATOMIC_RELEASE);
    /* validate the whole batch before any side effect or copy */
    int si, di;
    for (size_t i = 0; i < n; i++)
        if (rec_slots(t, &recs[i], &si, &di)) return shd_fail(-ENOENT, "packet %zu references an unattached host", i);
    ShdWorkerBuf* b = &t->wbuf[worker];
    if (b->n + n > b->cap) {
        size_t nc = b->cap ? b->cap : 4096;
        while (nc < b->n + n) nc *= 2;
        ShdPkt* s = (ShdPkt*)realloc(b->recs, sizeof(ShdPkt) * nc);
        if (!s) return -ENOMEM;
        b->recs = s;
        b->cap = nc;
    }
    for (size_t i = 0; i < n; i++) {
        rec_slots(t, &recs[i], &si, &di);
        int oi, oj;
        rc = shd_resolve(t, si, di, &oi, &oj); /* topology_getReliability's lookup, at send time */
        if (rc) return rc;                     /* (unreachable on a validated graph) */
        b->recs[b->n++] = recs[i];
    }
    return 0;
}

int shd_round_append(ShdTopology* t, const ShdPkt* recs, size_t n) { return shd_round_append_worker(t, 0, recs, n); }

int shd_round_staged(ShdTopology* t, size_t* n) {
    if (!t || !n) return -EINVAL;
    size_t k = 0;
    for (int w = 0; w < t->nworkers; w++) k += t->wbuf[w].n;
    *n = k;
    return 0;
}

/* Concatenates the worker buffers (worker order) into t->staged. */
static int gather_staged(ShdTopology* t, size_t* n_out) {
    size_t n = 0;
    for (int w = 0; w < t->nworkers; w++) n += t->wbuf[w].n;
    if (n > t->capstaged) {
        ShdPkt* s = (ShdPkt*)realloc(t->staged, sizeof(ShdPkt) * n);
        if (!s) return -ENOMEM;
        t->staged = s;
        t->capstaged = n;
    }
    size_t k = 0;
    for (int w = 0; w < t->nworkers; w++) {
        if (t->wbuf[w].n) memcpy(t->staged + k, t->wbuf[w].recs, sizeof(ShdPkt) * t->wbuf[w].n);
        k += t->wbuf[w].n;
    }
    *n_out = n;
    return 0;
}

static int collect_locked(ShdTopology* t, ShdDeliv* out, size_t cap, size_t* n_out, uint32_t* dst_offsets,
                          uint8_t* status, uint64_t* min_time) {
    size_t n = 0;
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    if ((rc = gather_staged(t, &n))) return rc;
    if (cap < n && out) return shd_fail(-ENOSPC, "output capacity %zu < %zu records", cap, n);
    if ((rc = shd_dev_init(t->device))) return rc;
    ShdPkt* d_recs = NULL;
    ShdDeliv* d_out = NULL;
    uint32_t* d_off = NULL;
    uint8_t* d_status = NULL;
    uint64_t* d_cnt = NULL;
    uint8_t* h_status = NULL;
    size_t nn = n ? n : 1;
    if ((rc = shd_dev_malloc((void**)&d_recs, sizeof(ShdPkt) * nn)) ||
        (rc = shd_dev_malloc((void**)&d_out, sizeof(ShdDeliv) * nn)) ||
        (rc = shd_dev_malloc((void**)&d_off, sizeof(uint32_t) * ((size_t)t->nhosts + 1))) ||
        (rc = shd_dev_malloc((void**)&d_status, nn)) || (rc = shd_dev_malloc((void**)&d_cnt, 16)))
        goto done;
    if (n && (rc = shd_dev_h2d(d_recs, t->staged, sizeof(ShdPkt) * n))) goto done;
    if ((rc = shd_sync_touch(t))) goto done;
    ShdPktCtx c;
    shd_pkt_ctx(t, &c);
    rc = shd_dev_packet_round(&c, d_recs, n, t->barrier, t->end_time, t->bootstrap_end, d_out, d_off, d_status,
                              d_cnt, NULL);
    if (rc) goto done;
    uint64_t cnt[2];
    if ((rc = shd_dev_d2h(cnt, d_cnt, 16))) goto done;
    if (n_out) *n_out = (size_t)cnt[0];
    if (min_time) *min_time = cnt[1];
    if (out && cnt[0] && (rc = shd_dev_d2h(out, d_out, sizeof(ShdDeliv) * (size_t)cnt[0]))) goto done;
    if (dst_offsets && (rc = shd_dev_d2h(dst_offsets, d_off, sizeof(uint32_t) * ((size_t)t->nhosts + 1)))) goto done;
    h_status = status ? status : (uint8_t*)malloc(nn);
    if (!h_status) {
        rc = -ENOMEM;
        goto done;
    }
    if ((rc = shd_dev_d2h(h_status, d_status, n))) goto done;
    /* topology_incrementPathPacketCounter for every kept packet (worker.c:551),
     * delivered or discarded at the end time alike; the lookups were already
     * made at append, so this only resolves owners and counts */
    pthread_mutex_lock(&t->pkt_mu);
    for (size_t i = 0; i < n && !rc; i++)
        if (h_status[i] != SHD_DROPPED_LOSS) {
            int si, di, oi, oj;
            rec_slots(t, &t->staged[i], &si, &di);
            if (!(rc = shd_resolve(t, si, di, &oi, &oj))) rc = shd_count_packet_locked(t, oi, oj, 1);
        }
    pthread_mutex_unlock(&t->pkt_mu);
    if (!rc)
        for (int w = 0; w < t->nworkers; w++) t->wbuf[w].n = 0;
done:
    if (h_status != status) free(h_status);
    shd_dev_free(d_recs);
    shd_dev_free(d_out);
    shd_dev_free(d_off);
    shd_dev_free(d_status);
    shd_dev_free(d_cnt);
    return rc;
}

int shd_round_collect(ShdTopology* t, ShdDeliv* out, size_t cap, size_t* n_out, uint32_t* dst_offsets,
                      uint8_t* status, uint64_t* min_time) {
    if (!t) return -EINVAL;
    pthread_mutex_lock(&t->round_mu);
    int rc = collect_locked(t, out, cap, n_out, dst_offsets, status, min_time);
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}

int shd_round_process_device(ShdTopology* t, const ShdPkt* d_recs, size_t n, uint64_t barrier, uint64_t end_time,
                             uint64_t bootstrap_end, ShdDeliv* d_out, uint32_t* d_dst_offsets, uint8_t* d_status,
                             uint64_t* d_counters, void* stream) {
    if (!t) return -EINVAL;
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    if (!__atomic_load_n(&t->lookups_started, __ATOMIC_RELAXED)) __atomic_store_n(&t->lookups_started, 1, __ATOMIC_RELEASE);
    pthread_mutex_lock(&t->round_mu);
    if (!(rc = shd_dev_init(t->device)) && !(rc = shd_sync_touch(t))) {
        ShdPktCtx c;
        shd_pkt_ctx(t, &c);
        rc = shd_dev_packet_round(&c, d_recs, n, barrier, end_time, bootstrap_end, d_out, d_dst_offsets, d_status,
                                  d_counters, stream);
    }
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}

int shd_deliv_sort_device(ShdTopology* t, const ShdDeliv* d_in, size_t n, uint32_t host_lo, uint32_t host_hi,
                          ShdDeliv* d_out, uint32_t* d_dst_offsets, void* stream) {
    if (!t || host_hi < host_lo) return -EINVAL;
    pthread_mutex_lock(&t->round_mu);
    int rc = shd_dev_init(t->device);
    if (!rc && !t->ws) rc = shd_dev_ws_new(&t->ws);
    if (!rc) rc = shd_dev_deliv_sort(t->ws, d_in, n, host_lo, host_hi, d_out, d_dst_offsets, stream);
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}

/* ---- multi-GPU rounds (kernels and RCCL in xchg.hip) ---- */

int shd_round_exchange(ShdTopology* t, const ShdTransport* x, const ShdDeliv* d_events, const uint32_t* d_dst_offsets,
                       const uint32_t* host_bounds, ShdDeliv* d_recv, size_t recv_cap, ShdDeliv* d_out,
                       uint32_t* d_out_offsets, size_t* n_out, void* stream) {
    if (!t || !x || !host_bounds || !n_out || x->world < 1 || x->rank < 0 || x->rank >= x->world)
        return shd_fail(-EINVAL, "bad exchange arguments");
    if (host_bounds[0] != 0 || host_bounds[x->world] != t->nhosts)
        return shd_fail(-EINVAL, "host bounds must cover [0, %u)", t->nhosts);
    int rc = shd_dev_init(t->device);
    if (rc) return rc;
    uint64_t* send = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)x->world);
    if (!send) return -ENOMEM;
    size_t nrecv = 0;
    if (!(rc = shd_dev_event_cuts(d_dst_offsets, host_bounds, x->world, send, stream)) &&
        !(rc = shd_dev_exchange_blocks(x, d_events, send, sizeof(ShdDeliv), d_recv, recv_cap, &nrecv, stream)))
        rc = shd_deliv_sort_device(t, d_recv, nrecv, host_bounds[x->rank], host_bounds[x->rank + 1], d_out,
                                   d_out_offsets, stream);
    free(send);
    if (!rc) *n_out = nrecv;
    return rc;
}

int shd_round_route_records(ShdTopology* t, const ShdTransport* x, const ShdPkt* d_recs, size_t n,
                            const uint32_t* row_bounds, ShdPkt* d_scratch, ShdPkt* d_recv, size_t recv_cap,
                            size_t* n_recv, void* stream) {
    if (!t || !x || !row_bounds || !n_recv || x->world < 1) return shd_fail(-EINVAL, "bad route arguments");
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    if (!t->use_sp) return shd_fail(-ENOTSUP, "row routing needs use_shortest_path (touch order)");
    if (row_bounds[0] != 0 || (int)row_bounds[x->world] != t->A)
        return shd_fail(-EINVAL, "row bounds must cover [0, %d)", t->A);
    pthread_mutex_lock(&t->round_mu);
    if (!(rc = shd_dev_init(t->device)) && !(rc = shd_sync_touch(t))) {
        ShdPktCtx c;
        shd_pkt_ctx(t, &c);
        rc = shd_dev_route_records(&c, x, d_recs, n, row_bounds, d_scratch, d_recv, recv_cap, n_recv, stream);
    }
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}
