/*
 * round.c -- host side of the batched packet hand-off that replaces the body
 * of worker_sendPacket (core/worker.c:517-576) + scheduler_push
 * (core/scheduler/scheduler.c:232-255) + the host-single policy push
 * (scheduler_policy_host_single.c:174-220).
 *
 * At send time (shd_round_append) the CPU keeps what must stay in send
 * order: the lookup side effects of topology_getReliability (row touch,
 * min-jump) -- the decision itself only needs the sender's reserved rand_r
 * pre-state, recorded in the ShdPkt.  At the round boundary
 * (manager.c:563-573, all workers idle) shd_round_collect ships the batch
 * to the GPU, which decides loss, computes and clamps delivery times and
 * groups the events per destination in event_compare order.  Batching is
 * exact because inter-host deliveries are clamped to >= the barrier
 * (host_single.c:187-192), so none of them runs in the round that sent it.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "topology_impl.h"

int shd_round_begin(ShdTopology* t, uint64_t barrier, uint64_t end_time, uint64_t bootstrap_end) {
    if (!t) return -EINVAL;
    t->barrier = barrier;
    t->end_time = end_time;
    t->bootstrap_end = bootstrap_end;
    t->nstaged = 0;
    return 0;
}

int shd_round_append(ShdTopology* t, const ShdPkt* recs, size_t n) {
    if (!t || (!recs && n)) return -EINVAL;
    int rc = shd_topology_build_routes(t);
    if (rc) return rc;
    t->lookups_started = 1;
    if (t->nstaged + n > t->capstaged) {
        size_t nc = t->capstaged ? t->capstaged : 4096;
        while (nc < t->nstaged + n) nc *= 2;
        ShdPkt* s = (ShdPkt*)realloc(t->staged, sizeof(ShdPkt) * nc);
        if (!s) return -ENOMEM;
        t->staged = s;
        t->capstaged = nc;
    }
    for (size_t i = 0; i < n; i++) {
        const ShdPkt* p = &recs[i];
        if (p->src_host >= t->nhosts || p->dst_host >= t->nhosts || t->host_vertex[p->src_host] < 0 ||
            t->host_vertex[p->dst_host] < 0)
            return shd_fail(-ENOENT, "packet %zu references an unattached host", i);
        int si = t->vertex_slot[t->host_vertex[p->src_host]];
        int di = t->vertex_slot[t->host_vertex[p->dst_host]];
        int oi, oj;
        rc = shd_resolve(t, si, di, &oi, &oj); /* topology_getReliability's lookup */
        if (rc) return rc;
        t->staged[t->nstaged++] = *p;
    }
    return 0;
}

int shd_round_collect(ShdTopology* t, ShdDeliv* out, size_t cap, size_t* n_out, uint32_t* dst_offsets,
                      uint8_t* status, uint64_t* min_time) {
    if (!t) return -EINVAL;
    size_t n = t->nstaged;
    if (cap < n && out) return shd_fail(-ENOSPC, "output capacity %zu < %zu records", cap, n);
    int rc = shd_topology_build_routes(t);
    if (rc) return rc;
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
    if ((rc = shd_dev_d2h(h_status, d_status, n))) goto done;
    /* topology_incrementPathPacketCounter for every kept packet (worker.c:551),
     * delivered or discarded at the end time alike */
    for (size_t i = 0; i < n; i++)
        if (h_status[i] != SHD_DROPPED_LOSS) {
            const ShdPkt* p = &t->staged[i];
            int si = t->vertex_slot[t->host_vertex[p->src_host]];
            int di = t->vertex_slot[t->host_vertex[p->dst_host]];
            int oi, oj;
            if ((rc = shd_resolve(t, si, di, &oi, &oj)) || (rc = shd_count_packet(t, oi, oj, 1))) goto done;
        }
    t->nstaged = 0;
done:
    if (h_status != status) free(h_status);
    shd_dev_free(d_recs);
    shd_dev_free(d_out);
    shd_dev_free(d_off);
    shd_dev_free(d_status);
    shd_dev_free(d_cnt);
    return rc;
}

int shd_round_process_device(ShdTopology* t, const ShdPkt* d_recs, size_t n, uint64_t barrier, uint64_t end_time,
                             uint64_t bootstrap_end, ShdDeliv* d_out, uint32_t* d_dst_offsets, uint8_t* d_status,
                             uint64_t* d_counters, void* stream) {
    if (!t) return -EINVAL;
    int rc = shd_topology_build_routes(t);
    if (rc) return rc;
    t->lookups_started = 1;
    if ((rc = shd_sync_touch(t))) return rc;
    ShdPktCtx c;
    shd_pkt_ctx(t, &c);
    return shd_dev_packet_round(&c, d_recs, n, barrier, end_time, bootstrap_end, d_out, d_dst_offsets, d_status,
                                d_counters, stream);
}

int shd_deliv_sort_device(ShdTopology* t, const ShdDeliv* d_in, size_t n, uint32_t host_lo, uint32_t host_hi,
                          ShdDeliv* d_out, uint32_t* d_dst_offsets, void* stream) {
    if (!t || host_hi < host_lo) return -EINVAL;
    int rc = shd_dev_init(t->device);
    if (rc) return rc;
    return shd_dev_deliv_sort(d_in, n, host_lo, host_hi, d_out, d_dst_offsets, stream);
}
