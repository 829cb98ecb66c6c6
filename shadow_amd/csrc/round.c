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
            for (int w = 0; w < t->nworkers; w++) shd_wbuf_release(&t->wbuf[w]);
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
    int rc = 0;
    for (int w = 0; w < t->nworkers; w++) {
        ShdWorkerBuf* b = &t->wbuf[w];
        if (b->stream && b->up) { /* (a round dropped without a collect: its uploads finish first) */
            const int r = shd_dev_stream_sync(b->stream);
            if (!rc) rc = r;
        }
        b->n = b->up = 0;
    }
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}

void shd_wbuf_release(ShdWorkerBuf* b) {
    if (b->stream) (void)shd_dev_stream_sync(b->stream);
    shd_host_free(b->recs);
    shd_dev_free(b->d_recs);
    shd_dev_event_free(b->ev);
    shd_dev_stream_free(b->stream);
    memset(b, 0, sizeof *b);
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

/* Grows worker buffer b (pinned host memory: the collect copies it to the
 * device asynchronously at the link's rate) to hold `need` records. */
static int wbuf_reserve(ShdWorkerBuf* b, size_t need) {
    if (need <= b->cap) return 0;
    size_t nc = b->cap ? b->cap : 4096;
    while (nc < need) nc *= 2;
    ShdPkt* s = NULL;
    int rc = 0;
    if (b->stream && b->up && (rc = shd_dev_stream_sync(b->stream))) return rc; /* (uploads read the old buffer) */
    if ((rc = shd_host_alloc((void**)&s, sizeof(ShdPkt) * nc))) return rc;
    if (b->n) memcpy(s, b->recs, sizeof(ShdPkt) * b->n);
    shd_host_free(b->recs);
    b->recs = s;
    b->cap = nc;
    return 0;
}

/* Uploads worker buffer b's records [up, n) to its device mirror on the
 * worker's own stream (the link copies while the round's sends go on).  Not
 * for multi-shard tables (their collect partitions on the host).  A failure
 * here is not the append's: the collect copies whatever was not uploaded. */
static void wbuf_upload(ShdTopology* t, ShdWorkerBuf* b) {
    if (t->nshards > 1 || b->n == b->up) return;
    const char* v = getenv("SHD_APPEND_UPLOAD");
    if (v && strcmp(v, "0") == 0) return;
    if (shd_dev_init(t->device)) return;
    if (!b->stream && shd_dev_stream_new(&b->stream)) return;
    if (!b->ev && shd_dev_event_new(&b->ev)) return;
    if (b->n > b->dcap) { /* grow the mirror, keeping the uploaded prefix */
        ShdPkt* d = NULL;
        if (shd_dev_malloc((void**)&d, sizeof(ShdPkt) * b->cap)) return;
        if (b->up && (shd_dev_d2d_async(d, b->d_recs, sizeof(ShdPkt) * b->up, b->stream) ||
                      shd_dev_stream_sync(b->stream))) {
            shd_dev_free(d);
            return;
        }
        shd_dev_free(b->d_recs);
        b->d_recs = d;
        b->dcap = b->cap;
    }
    if (!shd_dev_h2d_async(b->d_recs + b->up, b->recs + b->up, sizeof(ShdPkt) * (b->n - b->up), b->stream))
        b->up = b->n;
}

int shd_round_append_worker(ShdTopology* t, int worker, const ShdPkt* recs, size_t n) {
    if (!t || (!recs && n) || worker < 0 || worker >= t->nworkers) return shd_fail(-EINVAL, "bad append arguments");
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    if (!__atomic_load_n(&t->lookups_started, __ATOMIC_RELAXED)) __atomic_store_n(&t->lookups_started, 1, __ATOMIC_RELEASE);
    /* validate the whole batch before any side effect or copy; note whether
     * any send can still have a lookup side effect (a first touch of its row,
     * a first self or direct pair) -- none in the steady state, where the
     * batch is then one copy.  (Every attached pair of a validated graph is
     * routable: strongly connected, or complete for direct paths.) */
    const uint32_t* hs = t->h_host_info; /* {slot, -} per host, UINT32_MAX: unattached */
    const uint32_t H = t->nhosts;
    size_t pending = 0;
    for (size_t i = 0; i < n; i++) {
        const uint32_t s = recs[i].src_host, d = recs[i].dst_host;
        if (s >= H || d >= H || hs[2 * (size_t)s] == SHD_UNTOUCHED || hs[2 * (size_t)d] == SHD_UNTOUCHED)
            return shd_fail(-ENOENT, "packet %zu references an unattached host", i);
        pending += (size_t)shd_resolve_pending(t, (int)hs[2 * (size_t)s], (int)hs[2 * (size_t)d]);
    }
    ShdWorkerBuf* b = &t->wbuf[worker];
    if ((rc = wbuf_reserve(b, b->n + n))) return rc;
    if (!pending) { /* in pieces of 4 MB, each uploaded while the next is copied */
        const size_t kPiece = 131072;
        for (size_t i = 0; i < n; i += kPiece) {
            const size_t m = n - i < kPiece ? n - i : kPiece;
            memcpy(b->recs + b->n, recs + i, sizeof(ShdPkt) * m);
            b->n += m;
            wbuf_upload(t, b);
        }
        return 0;
    }
    for (size_t i = 0; i < n && !rc; i++) {
        const int si = (int)hs[2 * (size_t)recs[i].src_host], di = (int)hs[2 * (size_t)recs[i].dst_host];
        int oi, oj;
        if (shd_resolve_pending(t, si, di))
            rc = shd_resolve(t, si, di, &oi, &oj); /* topology_getReliability's lookup, at send time */
        if (!rc) b->recs[b->n++] = recs[i];
    }
    wbuf_upload(t, b);
    /* device-resident rows first touched here are queued; launched in batches
     * (never waited for at send time), folded in touch order at the boundary */
    const int rcf = shd_release_kick(t);
    return rc ? rc : rcf;
}

int shd_round_append(ShdTopology* t, const ShdPkt* recs, size_t n) { return shd_round_append_worker(t, 0, recs, n); }

int shd_host_buffer_alloc(size_t bytes, void** out) {
    if (!out) return -EINVAL;
    return shd_host_alloc(out, bytes);
}

void shd_host_buffer_free(void* p) { shd_host_free(p); }

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

/* The collect's device buffers for n records over H hosts (grow-only; the
 * previous round on the collect stream has completed). */
static int collect_reserve(ShdTopology* t, size_t n, uint32_t H) {
    int rc = 0;
    if (!t->cstream && (rc = shd_dev_stream_new(&t->cstream))) return rc;
    if (!t->h_ccnt && (rc = shd_host_alloc((void**)&t->h_ccnt, 16))) return rc;
    if (!t->d_ccnt && (rc = shd_dev_malloc((void**)&t->d_ccnt, 16))) return rc;
    if (!n) n = 1;
    if (n > t->cap_c) {
        shd_dev_free(t->d_crecs);
        shd_dev_free(t->d_cout);
        shd_dev_free(t->d_cstat);
        t->d_crecs = NULL;
        t->d_cout = NULL;
        t->d_cstat = NULL;
        t->cap_c = 0;
        const size_t cap = n + n / 8 + 1024;
        if ((rc = shd_dev_malloc((void**)&t->d_crecs, sizeof(ShdPkt) * cap)) ||
            (rc = shd_dev_malloc((void**)&t->d_cout, sizeof(ShdDeliv) * cap)) ||
            (rc = shd_dev_malloc((void**)&t->d_cstat, cap)))
            return rc;
        t->cap_c = cap;
    }
    if (H + 1 > t->cap_coff) {
        shd_dev_free(t->d_coff);
        t->d_coff = NULL;
        t->cap_coff = 0;
        if ((rc = shd_dev_malloc((void**)&t->d_coff, sizeof(uint32_t) * ((size_t)H + 1)))) return rc;
        t->cap_coff = H + 1;
    }
    return 0;
}

/* The round boundary on one device: the worker buffers (pinned) go to the
 * device on the collect stream, the round runs there (path packet counters
 * included, on the device), and the outputs come back on the same stream:
 * one wait for the event count, one for the copies.  No allocation in the
 * steady state. */
static int collect_locked(ShdTopology* t, ShdDeliv* out, size_t cap, size_t* n_out, uint32_t* dst_offsets,
                          uint8_t* status, uint64_t* min_time) {
    size_t n = 0;
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    for (int w = 0; w < t->nworkers; w++) n += t->wbuf[w].n;
    if (cap < n && out) return shd_fail(-ENOSPC, "output capacity %zu < %zu records", cap, n);
    if ((rc = shd_dev_init(t->device))) return rc;
    if ((rc = collect_reserve(t, n, t->nhosts))) return rc;
    void* s = t->cstream;
    size_t at = 0;
    for (int w = 0; w < t->nworkers && !rc; w++) {
        ShdWorkerBuf* b = &t->wbuf[w];
        /* uploaded at append time: after the worker's stream, device to
         * device; the rest from the pinned buffer */
        if (b->up && !(rc = shd_dev_stream_after(s, b->stream, b->ev)))
            rc = shd_dev_d2d_async(t->d_crecs + at, b->d_recs, sizeof(ShdPkt) * b->up, s);
        if (!rc && b->n > b->up)
            rc = shd_dev_h2d_async(t->d_crecs + at + b->up, b->recs + b->up, sizeof(ShdPkt) * (b->n - b->up), s);
        at += b->n;
    }
    if (rc) {
        (void)shd_dev_stream_sync(s);
        return rc;
    }
    if ((rc = shd_sync_touch(t)) || (rc = shd_pcnt_ensure(t, &t->pcnt, t->tab_row_lo, t->tab_row_hi, n)) ||
        (rc = shd_ensure_ptab(t)))
        return rc;
    ShdPktCtx c;
    shd_pkt_ctx(t, &c);
    rc = shd_dev_packet_round(&c, t->d_crecs, n, t->barrier, t->end_time, t->bootstrap_end, t->d_cout, t->d_coff,
                              t->d_cstat, t->d_ccnt, s);
    if (shd_ptab_release_for_retry(t, rc)) {
        shd_pkt_ctx(t, &c);
        rc = shd_dev_packet_round(&c, t->d_crecs, n, t->barrier, t->end_time, t->bootstrap_end, t->d_cout, t->d_coff,
                                  t->d_cstat, t->d_ccnt, s);
    }
    shd_pcnt_commit(&t->pcnt, rc);
    if (!rc) rc = shd_dev_d2h_async(t->h_ccnt, t->d_ccnt, 16, s);
    if (!rc) rc = shd_dev_ws_sync(c.ws, s); /* (the round's own fault report) */
    if (rc) {
        (void)shd_dev_stream_sync(s); /* nothing of this round stays in flight */
        return rc;
    }
    /* the round is decided and counted: its records leave the staging
     * buffers whatever happens below (a retried collect must not count them
     * twice) */
    for (int w = 0; w < t->nworkers; w++) t->wbuf[w].n = t->wbuf[w].up = 0;
    const uint64_t nev = t->h_ccnt[0], mt = t->h_ccnt[1];
    if (out && nev) rc = shd_dev_d2h_async(out, t->d_cout, sizeof(ShdDeliv) * (size_t)nev, s);
    if (!rc && dst_offsets)
        rc = shd_dev_d2h_async(dst_offsets, t->d_coff, sizeof(uint32_t) * ((size_t)t->nhosts + 1), s);
    if (!rc && status) rc = shd_dev_d2h_async(status, t->d_cstat, n, s);
    const int rcs = shd_dev_stream_sync(s);
    if (!rc) rc = rcs;
    if (!rc) {
        if (n_out) *n_out = (size_t)nev;
        if (min_time) *min_time = mt;
    }
    return rc;
}

/* ---- single-process multi-GPU round (a multi-shard table) ----
 * The batch is split by the shard holding each record's answering row (the
 * owner row of the touch order, resolved here on the host from the same
 * state the kernel reads); every shard decides its records on its own device
 * and stream, concurrently; the decided events of each shard are cut by
 * destination owner (shard m owns hosts [host_bounds[m], host_bounds[m+1]))
 * and copied device to device (xGMI between GPUs) to the owner, which
 * regroups them into event_compare order (shd_dev_deliv_sort).  The union is
 * the single-GPU round: event_compare is a total order. */

#define GROW(ptr, cap_field, need, elem)                                                      \
    do {                                                                                      \
        if ((need) > (cap_field)) {                                                           \
            shd_dev_free(ptr);                                                                \
            (ptr) = NULL;                                                                     \
            if ((rc = shd_dev_malloc((void**)&(ptr), (elem) * ((need) + (need) / 4 + 64)))) goto done; \
        }                                                                                     \
    } while (0)

/* Uploads the release state to shard s's device if it changed (caller holds round_mu). */
static int sync_shard_touch(ShdTopology* t, ShdShard* s) {
    const uint64_t gen = __atomic_load_n(&t->touch_gen, __ATOMIC_ACQUIRE);
    if (s->d_touch && s->synced_gen == gen && gen) return 0;
    int rc = 0;
    if (!s->d_touch && (rc = shd_dev_malloc((void**)&s->d_touch, sizeof(uint32_t) * (size_t)t->A))) return rc;
    if (!s->d_host_info && (rc = shd_dev_malloc((void**)&s->d_host_info, sizeof(uint32_t) * 2 * ((size_t)t->nhosts + 1))))
        return rc;
    uint32_t* snap = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)t->A);
    uint32_t* hs = (uint32_t*)malloc(sizeof(uint32_t) * 2 * ((size_t)t->nhosts + 1));
    if (!snap || !hs) rc = -ENOMEM;
    for (int i = 0; !rc && i < t->A; i++) snap[i] = __atomic_load_n(&t->touch[i], __ATOMIC_ACQUIRE);
    for (uint32_t h = 0; !rc && h < t->nhosts; h++) {
        hs[2 * h] = t->h_host_info[2 * h];
        hs[2 * h + 1] = hs[2 * h] != SHD_UNTOUCHED ? snap[hs[2 * h]] : SHD_UNTOUCHED;
    }
    if (!rc) rc = shd_dev_h2d(s->d_touch, snap, sizeof(uint32_t) * (size_t)t->A);
    if (!rc) rc = shd_dev_h2d(s->d_host_info, hs, sizeof(uint32_t) * 2 * (size_t)t->nhosts);
    free(snap);
    free(hs);
    if (!rc) s->synced_gen = gen;
    return rc;
}

static int collect_shards_locked(ShdTopology* t, ShdDeliv* out, size_t cap, size_t* n_out, uint32_t* dst_offsets,
                                 uint8_t* status, uint64_t* min_time) {
    const int S = t->nshards;
    const uint32_t H = t->nhosts;
    size_t n = 0;
    int rc = gather_staged(t, &n);
    if (rc) return rc;
    if (cap < n && out) return shd_fail(-ENOSPC, "output capacity %zu < %zu records", cap, n);
    const size_t nn = n ? n : 1;
    uint32_t* perm = (uint32_t*)malloc(sizeof(uint32_t) * nn);    /* partition position -> record */
    uint16_t* owner = (uint16_t*)malloc(sizeof(uint16_t) * nn);   /* record -> shard */
    ShdPkt* part = (ShdPkt*)malloc(sizeof(ShdPkt) * nn);
    uint8_t* pst = (uint8_t*)malloc(nn);
    uint32_t* offk = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)H + 1) * (size_t)S);
    size_t pbeg[SHD_MAX_SHARDS + 1] = {0};
    uint64_t cnt[SHD_MAX_SHARDS][2];
    if (!perm || !owner || !part || !pst || !offk) {
        rc = -ENOMEM;
        goto done;
    }
    /* owner shard of every record: its answering row (use_shortest_path:
     * touch order, as k_pkt_scatter resolves it); unattached -> shard 0,
     * which reports them undelivered */
    for (size_t i = 0; i < n; i++) {
        const ShdPkt* p = &t->staged[i];
        int si, di, k = 0;
        if (!rec_slots(t, p, &si, &di)) {
            int oi = si;
            if (si != di && __atomic_load_n(&t->touch[di], __ATOMIC_ACQUIRE) <
                                __atomic_load_n(&t->touch[si], __ATOMIC_ACQUIRE))
                oi = di;
            ShdShard* s = shd_shard_of(t, oi);
            k = s ? (int)(s - t->shards) : 0;
        }
        owner[i] = (uint16_t)k;
        pbeg[k + 1]++;
    }
    for (int k = 0; k < S; k++) pbeg[k + 1] += pbeg[k];
    {
        size_t fill[SHD_MAX_SHARDS];
        for (int k = 0; k < S; k++) fill[k] = pbeg[k];
        for (size_t i = 0; i < n; i++) {
            const size_t q = fill[owner[i]]++;
            perm[q] = (uint32_t)i;
            part[q] = t->staged[i];
        }
    }
    /* decide: every shard on its device and stream, concurrently */
    for (int k = 0; k < S && !rc; k++) {
        ShdShard* s = &t->shards[k];
        const size_t nk = pbeg[k + 1] - pbeg[k];
        if ((rc = shd_dev_init(s->device))) break;
        if (!s->stream && (rc = shd_dev_stream_new(&s->stream))) break;
        if (!s->ws && (rc = shd_dev_ws_new(&s->ws))) break;
        if ((rc = sync_shard_touch(t, s)) || (rc = shd_pcnt_ensure(t, &s->pcnt, s->lo, s->hi, nk))) break;
        GROW(s->d_recs, s->cap_n, nk, sizeof(ShdPkt));
        GROW(s->d_out, s->cap_n, nk, sizeof(ShdDeliv));
        GROW(s->d_status, s->cap_n, nk, 1);
        if (nk > s->cap_n) s->cap_n = nk + nk / 4 + 64;
        GROW(s->d_off, s->cap_h, (size_t)H + 1, sizeof(uint32_t));
        GROW(s->d_fin_off, s->cap_h, (size_t)H + 1, sizeof(uint32_t));
        if (!s->d_cnt && (rc = shd_dev_malloc((void**)&s->d_cnt, 16))) break;
        if ((size_t)H + 1 > s->cap_h) s->cap_h = H + 1 + (H + 1) / 4 + 64;
        if (nk && (rc = shd_dev_h2d(s->d_recs, part + pbeg[k], sizeof(ShdPkt) * nk))) break;
        ShdPktCtx c;
        c.tab = s->base;
        c.A = t->A;
        c.mode = 0;
        c.touch = s->d_touch;
        c.pair_bits = NULL;
        c.host_info = s->d_host_info;
        c.nhosts = H;
        c.ws = s->ws;
        c.row_lo = s->lo;
        c.row_hi = s->hi;
        c.idx_base = (uint32_t)pbeg[k];
        c.ptab = NULL; /* shards decide from their f64 rows */
        shd_pcnt_ctx(&s->pcnt, &c); /* path packet counters of the shard's rows */
        rc = shd_dev_packet_round(&c, s->d_recs, nk, t->barrier, t->end_time, t->bootstrap_end, s->d_out, s->d_off,
                                  s->d_status, s->d_cnt, s->stream);
        shd_pcnt_commit(&s->pcnt, rc);
    }
    for (int k = 0; k < S && !rc; k++) {
        ShdShard* s = &t->shards[k];
        const size_t nk = pbeg[k + 1] - pbeg[k];
        if (!(rc = shd_dev_init(s->device)) && !(rc = shd_dev_stream_sync(s->stream)) &&
            !(rc = shd_dev_ws_check_faults(s->ws)) && !(rc = shd_dev_d2h(cnt[k], s->d_cnt, 16)) &&
            !(rc = shd_dev_d2h(offk + ((size_t)H + 1) * (size_t)k, s->d_off, sizeof(uint32_t) * ((size_t)H + 1))))
            rc = shd_dev_d2h(pst + pbeg[k], s->d_status, nk);
    }
    /* destination-owner exchange (device to device) and regroup */
    size_t obase = 0;
    for (int m = 0; m < S && !rc; m++) {
        ShdShard* sm = &t->shards[m];
        const uint32_t lo = t->host_bounds[m], hi = t->host_bounds[m + 1];
        size_t tot = 0;
        for (int k = 0; k < S; k++) {
            const uint32_t* o = offk + ((size_t)H + 1) * (size_t)k;
            tot += o[hi] - o[lo];
        }
        if ((rc = shd_dev_init(sm->device))) break;
        GROW(sm->d_recv, sm->cap_r, tot, sizeof(ShdDeliv));
        GROW(sm->d_fin, sm->cap_r, tot, sizeof(ShdDeliv));
        if (tot > sm->cap_r) sm->cap_r = tot + tot / 4 + 64;
        size_t at = 0;
        for (int k = 0; k < S && !rc; k++) {
            const uint32_t* o = offk + ((size_t)H + 1) * (size_t)k;
            const size_t b = o[hi] - o[lo];
            if (b) rc = shd_dev_d2d(sm->d_recv + at, t->shards[k].d_out + o[lo], sizeof(ShdDeliv) * b);
            at += b;
        }
        /* the S received blocks are each grouped by destination in
         * event_compare order: merged as runs (their offsets are on the host) */
        const size_t nro = (size_t)S * (hi - lo + 1) + (size_t)S + 1;
        if (!rc) rc = shd_dev_init(sm->device);
        GROW(sm->d_rofs, sm->cap_rofs, nro, sizeof(uint32_t));
        if (nro > sm->cap_rofs) sm->cap_rofs = nro + nro / 4 + 64;
        if (!rc) {
            uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * nro);
            if (!h) rc = -ENOMEM;
            uint32_t base = 0;
            for (int k = 0; k < S && !rc; k++) {
                const uint32_t* o = offk + ((size_t)H + 1) * (size_t)k;
                for (uint32_t j = 0; j <= hi - lo; j++) h[(size_t)k * (hi - lo + 1) + j] = o[lo + j] - o[lo];
                h[(size_t)S * (hi - lo + 1) + k] = base;
                base += o[hi] - o[lo];
            }
            if (!rc) h[(size_t)S * (hi - lo + 1) + S] = base;
            if (!rc) rc = shd_dev_h2d(sm->d_rofs, h, sizeof(uint32_t) * nro);
            free(h);
        }
        if (!rc)
            rc = shd_dev_deliv_merge_runs(sm->ws, sm->d_recv, 0, 1, tot, sm->d_rofs, sm->d_rofs + (size_t)S * (hi - lo + 1),
                                          (uint32_t)S, lo, hi, sm->d_fin, sm->d_fin_off, sm->stream);
        if (!rc) rc = shd_dev_stream_sync(sm->stream);
        if (!rc) rc = shd_dev_ws_check_faults(sm->ws);
        if (!rc && out && tot) rc = shd_dev_d2h(out + obase, sm->d_fin, sizeof(ShdDeliv) * tot);
        if (!rc && dst_offsets) {
            if ((rc = shd_dev_d2h(dst_offsets + lo, sm->d_fin_off, sizeof(uint32_t) * ((size_t)(hi - lo) + 1))))
                break;
            for (uint32_t h = lo; h <= hi; h++) dst_offsets[h] += (uint32_t)obase;
        }
        obase += tot;
    }
    if (rc) goto done;
    uint64_t mt = UINT64_MAX;
    for (int k = 0; k < S; k++)
        if (pbeg[k + 1] > pbeg[k] && cnt[k][1] < mt) mt = cnt[k][1];
    if (n_out) *n_out = obase;
    if (min_time) *min_time = mt;
    if (out)
        for (size_t i = 0; i < obase; i++) out[i].pkt_index = perm[out[i].pkt_index];
    if (status)
        for (size_t q = 0; q < n; q++) status[perm[q]] = pst[q]; /* partition order -> record order */
    for (int w = 0; w < t->nworkers; w++) t->wbuf[w].n = t->wbuf[w].up = 0; /* decided and counted (see collect_locked) */
done:
    free(perm);
    free(owner);
    free(part);
    free(pst);
    free(offk);
    shd_dev_init(t->device);
    return rc;
}

int shd_round_collect(ShdTopology* t, ShdDeliv* out, size_t cap, size_t* n_out, uint32_t* dst_offsets,
                      uint8_t* status, uint64_t* min_time) {
    if (!t) return -EINVAL;
    pthread_mutex_lock(&t->round_mu);
    /* the round boundary: releases queued by this round's sends and lookups
     * are folded into the running minimum (and the min-jump callback) first,
     * in touch order -- what the controller reads next (controller.c:390-422) */
    int rc = shd_release_sync(t, 1);
    if (!rc)
        rc = t->nshards > 1 ? collect_shards_locked(t, out, cap, n_out, dst_offsets, status, min_time)
                            : collect_locked(t, out, cap, n_out, dst_offsets, status, min_time);
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
    if (t->nshards > 1) return shd_fail(-ENOTSUP, "a multi-shard table runs its rounds with shd_round_process_shards");
    pthread_mutex_lock(&t->round_mu);
    if (!(rc = shd_dev_init(t->device)) && !(rc = shd_sync_touch(t)) &&
        !(rc = shd_pcnt_ensure(t, &t->pcnt, t->tab_row_lo, t->tab_row_hi, n)) && !(rc = shd_ensure_ptab(t))) {
        ShdPktCtx c;
        shd_pkt_ctx(t, &c);
        rc = shd_dev_packet_round(&c, d_recs, n, barrier, end_time, bootstrap_end, d_out, d_dst_offsets, d_status,
                                  d_counters, stream);
        if (shd_ptab_release_for_retry(t, rc)) { /* the workspace did not fit beside the 8-B table */
            shd_pkt_ctx(t, &c);
            rc = shd_dev_packet_round(&c, d_recs, n, barrier, end_time, bootstrap_end, d_out, d_dst_offsets,
                                      d_status, d_counters, stream);
        }
        shd_pcnt_commit(&t->pcnt, rc);
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
    const char* runs = getenv("SHD_XCHG_RUNS"); /* 0: regroup by re-scattering (the round-2 form) */
    if (!(runs && strcmp(runs, "0") == 0)) {
        pthread_mutex_lock(&t->round_mu);
        if (!t->ws) rc = shd_dev_ws_new(&t->ws);
        if (!rc)
            rc = shd_dev_exchange_runs(t->ws, x, d_events, d_dst_offsets, host_bounds, d_recv, recv_cap, d_out,
                                       d_out_offsets, n_out, stream);
        pthread_mutex_unlock(&t->round_mu);
        return rc;
    }
    uint64_t* send = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)x->world);
    if (!send) return -ENOMEM;
    size_t nrecv = 0;
    pthread_mutex_lock(&t->round_mu);
    if (!t->ws) rc = shd_dev_ws_new(&t->ws);
    if (!rc) rc = shd_dev_event_cuts(t->ws, d_dst_offsets, host_bounds, x->world, send, stream);
    pthread_mutex_unlock(&t->round_mu);
    if (!rc &&
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

int shd_topology_allgather_rows(ShdTopology* t, const ShdTransport* x, void* d_table, const uint32_t* row_bounds,
                                void* stream) {
    if (!t || !x || !d_table || !row_bounds || x->world < 1 || x->rank < 0 || x->rank >= x->world)
        return shd_fail(-EINVAL, "bad all-gather arguments");
    if (!x->allgatherv) return shd_fail(-ENOTSUP, "the transport has no allgatherv");
    int A = 0;
    int rc = shd_topology_slot_count(t, &A);
    if (rc) return rc;
    if (row_bounds[0] != 0 || (int)row_bounds[x->world] != A) return shd_fail(-EINVAL, "row bounds must cover [0, %d)", A);
    uint64_t* off = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)x->world + 1));
    if (!off) return -ENOMEM;
    for (int r = 0; r <= x->world && !rc; r++) {
        if (r && row_bounds[r] < row_bounds[r - 1]) rc = shd_fail(-EINVAL, "row bounds not ascending");
        off[r] = (uint64_t)row_bounds[r] * (uint64_t)A * sizeof(ShdEntry);
    }
    if (!rc) rc = shd_dev_init(t->device);
    if (!rc) {
        rc = x->allgatherv(x->user, d_table, off, stream);
        if (rc > 0) rc = -EIO;
    }
    if (!rc) rc = stream ? shd_dev_stream_sync(stream) : shd_dev_sync();
    free(off);
    return rc;
}

int shd_round_process_exchange(ShdTopology* t, const ShdTransport* x, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                               uint64_t end_time, uint64_t bootstrap_end, const uint32_t* host_bounds, void* d_send,
                               uint8_t* d_status, uint64_t* d_counters, void* d_recv, size_t recv_cap,
                               ShdDeliv* d_out, uint32_t* d_out_offsets, size_t* n_out, void* stream) {
    if (!t || !x || !host_bounds || !n_out || !d_send || !d_recv || x->world < 1 || x->rank < 0 ||
        x->rank >= x->world)
        return shd_fail(-EINVAL, "bad exchange arguments");
    int rc = shd_ensure_routes(t);
    if (rc) return rc;
    if (t->nshards > 1) return shd_fail(-ENOTSUP, "a multi-shard table runs its rounds with shd_round_collect");
    if (!__atomic_load_n(&t->lookups_started, __ATOMIC_RELAXED)) __atomic_store_n(&t->lookups_started, 1, __ATOMIC_RELEASE);
    pthread_mutex_lock(&t->round_mu);
    if (!(rc = shd_dev_init(t->device)) && !(rc = shd_sync_touch(t)) &&
        !(rc = shd_pcnt_ensure(t, &t->pcnt, t->tab_row_lo, t->tab_row_hi, n)) && !(rc = shd_ensure_ptab(t))) {
        ShdPktCtx c;
        shd_pkt_ctx(t, &c);
        rc = c.ws ? shd_dev_round_exchange(&c, x, d_recs, n, barrier, end_time, bootstrap_end, host_bounds, d_send,
                                           d_status, d_counters, d_recv, recv_cap, d_out, d_out_offsets, n_out, stream)
                  : -ENOMEM;
        shd_pcnt_commit(&t->pcnt, rc);
    }
    pthread_mutex_unlock(&t->round_mu);
    return rc;
}
