/* topology_impl.h -- the ShdTopology object shared by topology.c, routes.c
 * and round.c (host C side of libshdnet).
 *
 * Threading (the reference is called from every worker thread and guards
 * its cache with a GMutex + 3 GRWLocks, topology.c:26-85):
 *   - setup (load, attach, build, adopt) is serialised by setup_mu, and the
 *     table is immutable once `ready` is published (release store);
 *   - lookups read the table and the release state lock-free (atomic loads
 *     of touch[] / pair_bits[]); a row touch takes touch_mu only to draw its
 *     sequence number, so every released pair is owned by the row with the
 *     smaller sequence -- the state equals the serial execution in sequence
 *     order;
 *   - the running minimum and the min-jump callback are under min_mu, the
 *     path packet counters under pkt_mu, direct-path (pair bit) misses under
 *     pair_mu;
 *   - round staging is per worker (no lock between workers); the round
 *     pipeline (collect / process / regroup) is serialised by round_mu and
 *     its device workspace belongs to this topology. */
#ifndef SHD_TOPOLOGY_IMPL_H
#define SHD_TOPOLOGY_IMPL_H

#include <pthread.h>

#include "shd_internal.h"

#define SHD_UNTOUCHED 0xffffffffu

/* One worker's staged sends for the current round (one cache line: each
 * worker writes only its own).  recs: pinned host buffer; d_recs: its
 * device mirror, records [0, up) already copied there -- each append is
 * uploaded on the worker's own stream while the round's sends go on, so the
 * collect finds them on the device. */
typedef struct {
    ShdPkt* recs;
    size_t n, cap;
    ShdPkt* d_recs;
    size_t dcap, up;
    void* stream; /* the worker's upload stream (hipStream_t) and its event */
    void* ev;
} ShdWorkerBuf;
/* frees a worker buffer's host and device sides (its uploads finished) */
void shd_wbuf_release(ShdWorkerBuf* b);

typedef struct {
    uint32_t ip;
    int32_t vertex;
    uint8_t used; /* 0 empty, 1 live, 2 tombstone */
} IpSlot;

typedef struct {
    IpSlot* slots;
    uint32_t cap, n, tomb;
} IpMap;

/* A queued release of a device-resident table (topology.c "row releases"):
 * a row's first touch (row >= 0, its touch sequence) or a first self lookup
 * (row = -1 - slot).  key orders the fold: 2 * seq + 1 for a row, 2 *
 * next_touch for a self path released while next_touch rows were touched;
 * ord keeps queue order among equal keys. */
typedef struct {
    int32_t row;
    uint32_t seq;
    uint64_t key;
    uint64_t ord;
} ShdRelItem;
typedef struct {
    ShdRelItem* v;
    size_t n, cap;
} ShdRelList;
void shd_rel_list_free(ShdRelList* q);

/* Device path packet counters of resident rows [lo, hi): one u32 per table
 * entry (row r at base + r * A), the rounds' kernels add 1 per kept packet
 * at its answering pair (worker.c:551).  A counter never wraps: before a
 * round could take any counter past 2^32 - 1 (budget: packets counted since
 * the last spill), the counters >= 2^31 move into the host map (u64). */
typedef struct {
    uint32_t* alloc;
    uint32_t* base;
    /* the u8 delta layer of the log mode's fold (NULL: none): a pair's count
     * is base[k] + d8[k]; d8 is 16-B aligned at index 0 (d8_alloc holds
     * rows [lo, hi) plus 32 B of padding) */
    uint8_t* d8_alloc;
    uint8_t* d8;
    int lo, hi;
    int device;
    uint64_t budget;
    /* the counter log (SHD_PCNT=log): log_fill records logged since the last
     * fold, keys u32 (u64 when the table has 2^32 entries or more); cur /
     * cur_n: the slice reserved for the round being launched */
    void* log;
    size_t log_cap, log_fill;
    int log64; /* u64 keys (host-log mode on tables of 2^32 entries or more; the fold takes u32) */
    int mode;  /* this round's: 0 none, 1 log, 2 atomic */
    /* host-log mode: the dense counters did not fit on the device (-ENOMEM
     * even with the 8-B table dropped), so alloc stays NULL and the rounds
     * only log; the log is drained into the host map (u64 counters) when it
     * is full and before every read -- bounded device memory, slower reads */
    int hostlog;
    void* cur;
    size_t cur_n;
    void* fold; /* shd_dev_pcnt_fold scratch */
} ShdPcnt;

/* A device-resident piece of the routing table (no host mirror): rows [lo,
 * hi) on `device`, row r at base + r * A.  One shard for a single-GPU table,
 * several for a single-process multi-GPU table (shd_topology_adopt_table_shards);
 * a multi-process rank holds one shard and no other rows.  mu serialises the
 * shard's release scratch and its round buffers. */
#define SHD_MAX_SHARDS 64
typedef struct {
    int device;
    ShdEntry* base;
    int lo, hi;
    void* rel_scratch; /* shd_dev_release_launch buffers + stream */
    ShdRelList sent;   /* rows launched on this shard, not yet collected (launch order) */
    pthread_mutex_t mu;
    /* per-shard packet-round state (multi-shard topologies, round.c) */
    uint32_t *d_host_info, *d_touch, *d_pair_bits;
    uint64_t synced_gen;
    void* ws;
    void* stream;
    ShdPkt* d_recs;
    ShdDeliv *d_out, *d_recv, *d_fin;
    uint8_t* d_status;
    uint32_t *d_off, *d_fin_off;
    uint64_t* d_cnt;
    uint32_t* d_rofs; /* regroup: per source shard the rebased destination offsets + block bases */
    size_t cap_n, cap_r, cap_rofs;
    uint32_t cap_h;
    ShdPcnt pcnt; /* path packet counters of the shard's rows (multi-shard rounds) */
} ShdShard;


struct ShdTopology {
    int device;
    int use_sp;
    int directed, complete;
    int V, E, M;
    GmlDoc doc; /* owns every attribute string */
    int32_t *efrom, *eto; /* igraph storage order (undirected: from=max, to=min) */
    double* e_ms;         /* edge latency, ms = ns / 1e6 (topology.c:294) */
    double* e_rel;        /* 1 - packet_loss (topology.c:396) */
    int32_t *inc_off, *inc_nbr, *inc_eid; /* igraph_incident(OUT) CSR */
    const char **v_ip, **v_city, **v_country;
    int64_t *v_bw_down, *v_bw_up; /* KiB/s */
    double* v_id;                 /* the GML node id (VERTEX_ATTR_ID) */

    /* attachment */
    IpMap ipmap;
    uint8_t* v_attached;
    int32_t* host_vertex; /* host id -> vertex */
    uint32_t* host_ip;
    uint32_t nhosts, host_cap;
    int lookups_started;
    int routes_stale;

    /* routing table: slots = attached vertices in ascending vertex order */
    int A;
    int32_t* slot_vertex;
    int32_t* vertex_slot;
    ShdEntry* h_tab; /* host mirror of the device table */
    int tab_row_lo, tab_row_hi; /* rows present in d_tab (a rank's shard, else 0..A) */
    int built, prepared;
    int d_tab_owned;

    /* device state */
    ShdEntry* d_tab;
    /* 8-B packet-path form of the resident rows of d_tab (shd_ensure_ptab),
     * indexed like d_tab (d_ptab = allocation - tab_row_lo * A entries) */
    void* d_ptab;
    void* d_ptab_alloc;
    int ptab_unavailable; /* the allocation failed: rounds read d_tab */
    int32_t *d_inc_off, *d_inc_nbr, *d_slot_vertex, *d_vertex_slot;
    uint32_t* d_host_info; /* nhosts x {slot, touch[slot]} for the packet kernel */
    uint32_t* h_host_info;
    double *d_inc_w, *d_inc_r;
    void *d_snb, *d_swr; /* sentinel-terminated incidence lists (slab kernel) */
    void* d_sl;          /* integer-latency form of the same lists (NULL: not eligible) */
    int32_t* d_soff;
    uint32_t *d_touch, *d_pair_bits;

    /* release (cache) state */
    uint32_t* touch; /* per slot, SHD_UNTOUCHED or touch sequence */
    uint32_t next_touch;
    uint8_t* self_released;
    uint32_t* pair_bits; /* use_shortest_path = 0: (i,j) stored, A*A bits */
    int touch_dirty;
    uint64_t touch_gen; /* bumped by every touch (multi-shard uploads) */

    /* device-resident table (h_tab == NULL): its shards */
    int nshards;
    ShdShard shards[SHD_MAX_SHARDS];
    uint32_t* host_bounds; /* nshards + 1: destination hosts owned per shard (multi-shard rounds) */
    ShdRelList relq;    /* queued releases, not launched (under rel_mu) */
    ShdRelList relself; /* self paths of launched batches, read at the fold */
    double min_lat;
    ShdMinJumpFn cb;
    void* cb_user;

    /* path packet counters keyed by the answering (owner) pair: the host map
     * (explicit increments, spilled device counters) plus the device
     * counters of the rounds (pcnt; per shard for multi-shard tables) */
    uint64_t *pkt_keys, *pkt_vals;
    uint64_t pkt_cap, pkt_n;
    ShdPcnt pcnt;

    /* round staging (host API): one pinned buffer per worker */
    uint64_t barrier, end_time, bootstrap_end;
    ShdWorkerBuf* wbuf;
    int nworkers;
    ShdPkt* staged; /* concatenation at collect (worker order; multi-shard rounds) */
    size_t capstaged;
    /* shd_round_collect's device buffers (grow-only), its stream and its
     * pinned counter read-back */
    ShdPkt* d_crecs;
    ShdDeliv* d_cout;
    uint8_t* d_cstat;
    uint32_t* d_coff;
    uint64_t* d_ccnt;
    uint64_t* h_ccnt;
    size_t cap_c;
    uint32_t cap_coff;
    void* cstream;

    /* device workspace of the round pipeline (packet.hip) */
    void* ws;
    void* fw_scratch; /* min-plus Floyd-Warshall distances (minplus.hip) */

    /* synchronisation (see the header comment) */
    int ready; /* table built and adopted: lookups may proceed (atomic) */
    pthread_mutex_t setup_mu, touch_mu, min_mu, pkt_mu, pair_mu, round_mu, rel_mu;
};

void shd_topology_release_device(ShdTopology* t);
void shd_shards_clear(ShdTopology* t);
int shd_resolve(ShdTopology* t, int si, int di, int* oi, int* oj);
/* could shd_resolve(si, di) still have a side effect (read-only) */
int shd_resolve_pending(ShdTopology* t, int si, int di);
/* device-resident releases (topology.c): launch the queue once it is long
 * enough (never waits); wait for everything and fold it in touch order (fold
 * = 1) or drop it (0) */
int shd_release_kick(ShdTopology* t);
int shd_release_sync(ShdTopology* t, int fold);
/* the shard holding row `row` of a device-resident table (NULL: another rank's) */
ShdShard* shd_shard_of(ShdTopology* t, int row);
/* n table entries by flat index (host mirror or the owning shards' devices) */
int shd_read_entries(ShdTopology* t, const uint64_t* idx, size_t n, ShdEntry* out);
int shd_count_packet(ShdTopology* t, int oi, int oj, uint64_t inc);
int shd_count_packet_locked(ShdTopology* t, int oi, int oj, uint64_t inc);
int shd_count_reserve_locked(ShdTopology* t, uint64_t more);
int shd_sync_touch(ShdTopology* t);
void shd_pkt_ctx(ShdTopology* t, ShdPktCtx* c);
/* builds the packet-path table of the resident rows if there is none
 * (caller holds round_mu); a failed allocation leaves the f64 path */
int shd_ensure_ptab(ShdTopology* t);
void shd_ptab_drop(ShdTopology* t);
int shd_ptab_release_for_retry(ShdTopology* t, int rc);
int shd_ensure_routes(ShdTopology* t);
/* device path packet counters (routes.c): allocated (zeroed) for the rows
 * [lo, hi) on the calling thread's device at the first round, spilled ahead
 * of a round of n records when they could wrap (caller holds round_mu);
 * drop folds every counter into the host map and frees them */
int shd_pcnt_ensure(ShdTopology* t, ShdPcnt* p, int lo, int hi, size_t n);
/* after the round's launch: rc == 0 adds its reserved slice to the log */
void shd_pcnt_commit(ShdPcnt* p, int rc);
/* the round context's counter fields for p (its reserved slice / counters) */
void shd_pcnt_ctx(const ShdPcnt* p, ShdPktCtx* c);
/* folds every log of the topology into its counters (takes round_mu; the
 * readers call it before reading) */
int shd_pcnt_sync(ShdTopology* t);
int shd_pcnt_sync_locked(ShdTopology* t); /* (caller holds round_mu) */
int shd_pcnt_drop(ShdTopology* t, ShdPcnt* p);
/* frees every device counter without folding (topology teardown) */
void shd_pcnt_discard(ShdTopology* t);
/* device count of the flat table entry idx (0 if the rows are not resident
 * here or no round counted yet); waits for the device */
int shd_pcnt_read(ShdTopology* t, int row, int col, uint64_t* v);
/* counts of row `row`, columns [0, A), added into out (A values) */
int shd_pcnt_read_row(ShdTopology* t, int row, uint64_t* out);
/* rows [lo, hi), row-major, added into out ((hi - lo) * A values) */
int shd_pcnt_read_rows(ShdTopology* t, int lo, int hi, uint64_t* out);

#endif
