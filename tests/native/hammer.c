/*
 * hammer.c -- TEST ONLY.  N threads call the drop-in lookup API concurrently
 * (as Shadow's worker threads do: socket.c:808, tcp.c:392-393,
 * worker.c:539-551) and append round records from their own worker slots;
 * afterwards the state is checked for serial consistency:
 *   - every value a lookup returned is the entry of the pair's owner, the
 *     row with the smaller final touch sequence (topology.c:1189-1215);
 *   - the running minimum equals the minimum a serial execution in touch
 *     order releases (topology.c:1253-1264), and the min-jump callback
 *     reported a strictly decreasing sequence ending there;
 *   - path packet counters equal the increments made per owner pair;
 *   - every appended record is staged, in its worker's append order.
 * Built twice by tests/test_threads_cpu.py: plain and -fsanitize=thread,
 * against the product host C and tests/native/stub_dev.c.
 * Usage: hammer GML_PATH USE_SP NHOSTS THREADS OPS [SHARDS]
 *   SHARDS 0 (default): host-mirrored table; 1: device-resident table
 *   (lazy release through shd_release_flush); 2: a two-shard table
 *   (shd_topology_build_shards + adopt_table_shards, both on device 0).
 */
#include <arpa/inet.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "shdnet.h"

void stub_entry(int i, int j, double* lat, double* rel);

typedef struct {
    uint32_t s, d;
    uint8_t kind; /* 0 latency, 1 reliability, 2 routable, 3 increment, 4 append */
    double v;
} Op;

static ShdTopology* g_top;
static int g_nhosts, g_ops, g_use_sp;
static uint32_t* g_ip;
static Op** g_log;

static void* g_extra;
static double g_cb_last = 0;
static int g_cb_calls = 0, g_cb_bad = 0;
static uint64_t g_cb_hash = 1469598103934665603ull; /* FNV-1a over the reported values, in call order */
static void on_min_jump(double ms, void* user) {
    (void)user;
    /* called under the topology's min lock: plain accesses are ordered */
    uint64_t b;
    memcpy(&b, &ms, 8);
    for (int k = 0; k < 8; k++) g_cb_hash = (g_cb_hash ^ ((b >> (8 * k)) & 0xff)) * 1099511628211ull;
    if (g_cb_calls && !(ms < g_cb_last)) g_cb_bad++;
    g_cb_last = ms;
    g_cb_calls++;
}

static uint64_t xs(uint64_t* s) {
    *s ^= *s << 13;
    *s ^= *s >> 7;
    *s ^= *s << 17;
    return *s;
}

static void* worker(void* arg) {
    const int tid = (int)(intptr_t)arg;
    uint64_t r = 0x9E3779B97F4A7C15ull * (uint64_t)(tid + 1);
    for (int k = 0; k < g_ops; k++) {
        Op* o = &g_log[tid][k];
        o->s = (uint32_t)(xs(&r) % (uint64_t)g_nhosts);
        o->d = (uint32_t)(xs(&r) % (uint64_t)g_nhosts);
        o->kind = (uint8_t)(xs(&r) % 5);
        int rc = 0, b = 0;
        switch (o->kind) {
        case 0: rc = shd_topology_get_latency(g_top, g_ip[o->s], g_ip[o->d], &o->v); break;
        case 1: rc = shd_topology_get_reliability(g_top, g_ip[o->s], g_ip[o->d], &o->v); break;
        case 2:
            rc = shd_topology_is_routable(g_top, g_ip[o->s], g_ip[o->d], &b);
            o->v = b;
            break;
        case 3: rc = shd_topology_increment_path_packet_counter(g_top, g_ip[o->s], g_ip[o->d]); break;
        default: {
            ShdPkt p = {(uint64_t)k, (uint64_t)k, o->s, o->d, (uint32_t)tid, (uint32_t)k};
            rc = shd_round_append_worker(g_top, tid, &p, 1);
        }
        }
        if (rc) {
            fprintf(stderr, "thread %d op %d kind %d failed: %d %s\n", tid, k, o->kind, rc, shd_last_error());
            exit(3);
        }
    }
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 6) return 2;
    g_use_sp = atoi(argv[2]);
    g_nhosts = atoi(argv[3]);
    const int T = atoi(argv[4]);
    g_ops = atoi(argv[5]);
    if (shd_topology_new(argv[1], g_use_sp, 0, &g_top)) {
        fprintf(stderr, "load: %s\n", shd_last_error());
        return 3;
    }
    g_ip = malloc(sizeof(uint32_t) * (size_t)g_nhosts);
    int* host_vertex = malloc(sizeof(int) * (size_t)g_nhosts);
    for (int h = 0; h < g_nhosts; h++) {
        g_ip[h] = htonl(0x0B000001u + (uint32_t)h);
        uint32_t st = 2654435761u * (uint32_t)(h + 1);
        if (shd_topology_attach(g_top, (uint32_t)h, g_ip[h], &st, NULL, NULL, NULL, NULL, NULL)) return 3;
        shd_topology_vertex_of_host(g_top, (uint32_t)h, &host_vertex[h]);
    }
    shd_topology_set_min_jump_callback(g_top, on_min_jump, NULL);
    if (shd_round_set_workers(g_top, T) || shd_round_begin(g_top, 100, 1000000, 0)) return 3;
    int A = 0, V = 0;
    shd_topology_info(g_top, &V, NULL, NULL, NULL, NULL);
    shd_topology_slot_count(g_top, &A);
    const int shards = argc > 6 ? atoi(argv[6]) : 0;
    void* d_tab = NULL;
    if (shards == 1) {
        if (shd_device_alloc_table(0, (size_t)A * A * 16, &d_tab, NULL) ||
            shd_topology_build_rows_device(g_top, 0, A, d_tab) || shd_topology_adopt_table_device_resident(g_top, d_tab)) {
            fprintf(stderr, "device-resident: %s\n", shd_last_error());
            return 3;
        }
    } else if (shards == 2) {
        const int bounds[3] = {0, A / 3, A}, devs[2] = {0, 0};
        void* rows[2] = {NULL, NULL};
        if (shd_device_alloc_table(0, (size_t)(A / 3 + 1) * A * 16, &rows[0], NULL) ||
            shd_device_alloc_table(0, (size_t)(A - A / 3) * A * 16, &rows[1], NULL) ||
            shd_topology_build_shards(g_top, 2, devs, rows, bounds) ||
            shd_topology_adopt_table_shards(g_top, 2, devs, rows, bounds)) {
            fprintf(stderr, "shards: %s\n", shd_last_error());
            return 3;
        }
        d_tab = rows[0];
        g_extra = rows[1];
    }
    int* slot_of_v = malloc(sizeof(int) * (size_t)V);
    for (int v = 0; v < V; v++) slot_of_v[v] = -1;
    for (int h = 0; h < g_nhosts; h++) slot_of_v[host_vertex[h]] = 1;
    for (int v = 0, k = 0; v < V; v++)
        if (slot_of_v[v] == 1) slot_of_v[v] = k++;

    g_log = malloc(sizeof(Op*) * (size_t)T);
    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)T);
    for (int i = 0; i < T; i++) g_log[i] = calloc((size_t)g_ops, sizeof(Op));
    for (int i = 0; i < T; i++) pthread_create(&th[i], NULL, worker, (void*)(intptr_t)i);
    for (int i = 0; i < T; i++) pthread_join(th[i], NULL);

    /* ---- serial-consistency checks ---- */
    uint32_t* seq = malloc(sizeof(uint32_t) * (size_t)A);
    uint8_t* self = malloc((size_t)A);
    if (shd_topology_touch_order(g_top, seq, self, A)) return 3;
    int bad = 0, touched = 0;
    uint64_t* cnt = calloc((size_t)A * (size_t)A, sizeof(uint64_t));
    size_t appended = 0;
    for (int i = 0; i < T; i++)
        for (int k = 0; k < g_ops; k++) {
            const Op* o = &g_log[i][k];
            int si = slot_of_v[host_vertex[o->s]], di = slot_of_v[host_vertex[o->d]];
            int oi = si, oj = di;
            if (g_use_sp && si != di && seq[di] < seq[si]) oi = di, oj = si;
            if (g_use_sp && si != di && seq[si] == 0xffffffffu && seq[di] == 0xffffffffu) bad++; /* nobody touched */
            double lat, rel, lat2, rel2;
            stub_entry(oi, oj, &lat, &rel);
            stub_entry(oj, oi, &lat2, &rel2);
            if (o->kind == 0 && o->v != lat && (g_use_sp || o->v != lat2)) bad++;
            if (o->kind == 1 && o->v != rel && (g_use_sp || o->v != rel2)) bad++;
            if (o->kind == 2 && o->v != 1) bad++;
            if (o->kind == 3) cnt[(size_t)oi * A + oj]++;
            if (o->kind == 4) appended++;
        }
    if (bad) fprintf(stderr, "%d lookups returned a value that is not the owner's entry\n", bad);
    /* counters per owner pair (use_shortest_path: owners are fixed by seq) */
    int badc = 0;
    if (g_use_sp)
        for (int i = 0; i < T; i++)
            for (int k = 0; k < g_ops; k++) {
                const Op* o = &g_log[i][k];
                if (o->kind != 3) continue;
                int si = slot_of_v[host_vertex[o->s]], di = slot_of_v[host_vertex[o->d]];
                int oi = si, oj = di;
                if (si != di && seq[di] < seq[si]) oi = di, oj = si;
                uint64_t c = 0;
                shd_topology_get_path_packet_count(g_top, g_ip[o->s], g_ip[o->d], &c);
                if (c != cnt[(size_t)oi * A + oj]) badc++;
            }
    if (badc) fprintf(stderr, "%d packet counters differ\n", badc);
    /* released minimum of the serial execution in touch order */
    double want = 0;
    if (g_use_sp) {
        for (int i = 0; i < A; i++) {
            if (seq[i] != 0xffffffffu) {
                touched++;
                for (int j = 0; j < A; j++)
                    if (j != i && seq[j] > seq[i]) {
                        double l, r;
                        stub_entry(i, j, &l, &r);
                        if (want == 0 || l < want) want = l;
                    }
            }
            if (self[i]) {
                double l, r;
                stub_entry(i, i, &l, &r);
                if (want == 0 || l < want) want = l;
            }
        }
    }
    double got = -1;
    shd_topology_get_min_path_latency(g_top, &got);
    int badm = g_use_sp && (got != want || g_cb_last != got || g_cb_bad);
    if (badm) fprintf(stderr, "min %.17g want %.17g cb_last %.17g cb_bad %d\n", got, want, g_cb_last, g_cb_bad);
    size_t staged = 0;
    shd_round_staged(g_top, &staged);
    int bads = staged != appended;
    if (bads) fprintf(stderr, "staged %zu appended %zu\n", staged, appended);
    printf("threads %d ops %d slots %d touched %d min %.17g cb_calls %d cb_hash %016llx staged %zu bad %d %d %d %d\n",
           T, g_ops, A, touched, got, g_cb_calls, (unsigned long long)g_cb_hash, staged, bad, badc, badm, bads);
    shd_topology_free(g_top);
    if (d_tab) shd_device_free(0, d_tab);
    if (g_extra) shd_device_free(0, g_extra);
    return (bad || badc || badm || bads) ? 1 : 0;
}
