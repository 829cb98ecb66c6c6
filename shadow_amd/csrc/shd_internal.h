/*
 * shd_internal.h -- internal interfaces of libshdnet (host C side and the
 * thin C-ABI to the HIP kernels).  Not installed; see include/shdnet.h.
 */
#ifndef SHD_INTERNAL_H
#define SHD_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "shdnet.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error reporting ---- */
int shd_fail(int code, const char* fmt, ...);

/* ---- units (core/support/units.rs restated) ---- */
int64_t shd_units_time_ns(const char* s);
int64_t shd_units_bandwidth_bits(const char* s);

/* ---- GML document (igraph_read_graph_gml dialect) ---- */
enum { GML_INT = 1, GML_REAL = 2, GML_STR = 3 };

typedef struct {
    const char* key;
    int type;
    long long ival;
    double rval;
    const char* sval;
} GmlKV;

typedef struct {
    int first, count; /* range in kvs[] */
} GmlBlock;

typedef struct {
    char* buf; /* private, NUL-split copy of the text */
    int directed;
    GmlKV* kvs;
    size_t nkv, capkv;
    GmlBlock* nodes;
    int nnodes, capnodes;
    GmlBlock* edges;
    int nedges, capedges;
} GmlDoc;

int shd_gml_parse(const char* text, GmlDoc* doc);
void shd_gml_free(GmlDoc* doc);

/* ---- device graph + launches (implemented in HIP, C ABI) ---- */
typedef struct {
    int V;       /* vertices */
    int A;       /* attached vertices (= table slots) */
    int M;       /* incidence entries */
    int directed;
    const int32_t* inc_off; /* V+1, igraph_incident(mode OUT) order */
    const int32_t* inc_nbr; /* M */
    const double* inc_w;    /* M, edge latency in ms */
    const double* inc_r;    /* M, 1 - packet_loss */
    const int32_t* slot_vertex; /* A */
    const int32_t* vertex_slot; /* V, -1 = not attached */
    /* sentinel-terminated copy of the incidence lists for the SSSP kernels:
     * v's list handle soff[v] = (start << 8) | n, start = inc_off[v] + v and
     * n = min(degree + 1, 255) entries to read first (sentinel included; 255
     * = read whole batches); entries {nbr, soff[nbr]} (snb, int2) and
     * {w_ms, 1 - loss} (swr, double2), closed by {-1, 0} (-2 when v is
     * attached); both padded by 64 x 16 entries */
    const void* snb;
    const void* swr;
    const int32_t* soff; /* V */
    /* integer-latency lists (same offsets and sentinels as snb): 16-B entries
     * {nbr, (uint32) w_ms, 1 - loss}; present only when every edge latency is
     * a whole number of ms and V * max latency < 2^32 - 1, so that every path
     * sum the f64 kernel would form is an exact u32 (k_sssp_islab) */
    const void* sl;
} ShdGraphDev;

typedef struct {
    double lat;
    double rel;
} ShdEntry; /* 16 B table entry, row-major A x A */

int shd_dev_init(int device);
int shd_dev_malloc(void** p, size_t bytes);
/* free and total device memory of the calling thread's device */
int shd_dev_mem_info(size_t* free_bytes, size_t* total_bytes);
int shd_dev_free(void* p);
/* physically contiguous when granted, else hipMalloc; *contig says which */
int shd_dev_malloc_table(void** p, size_t bytes, int* contig);
int shd_dev_d2d(void* d, const void* s, size_t bytes);
int shd_dev_h2d(void* d, const void* h, size_t bytes);
int shd_dev_d2h(void* h, const void* d, size_t bytes);
int shd_dev_memset(void* d, int v, size_t bytes);
/* copies enqueued on a stream (hipStream_t behind void*); the host side
 * should be pinned (shd_host_alloc) for them to be asynchronous */
int shd_dev_h2d_async(void* d, const void* h, size_t bytes, void* stream);
int shd_dev_d2h_async(void* h, const void* d, size_t bytes, void* stream);
int shd_dev_d2d_async(void* d, const void* s, size_t bytes, void* stream);
/* an event (hipEvent_t behind void*, no timing); shd_dev_stream_after:
 * `waiter` waits on the device for everything enqueued on `after` so far */
int shd_dev_event_new(void** e);
void shd_dev_event_free(void* e);
int shd_dev_stream_after(void* waiter, void* after, void* e);
/* pinned host memory */
int shd_host_alloc(void** p, size_t bytes);
void shd_host_free(void* p);
int shd_dev_sync(void);
/* a stream on the calling thread's device (hipStream_t behind void*) */
int shd_dev_stream_new(void** s);
int shd_dev_stream_sync(void* s);
void shd_dev_stream_free(void* s);

/* Routing rows [row_lo, row_hi) of the A x A table (tab already sized A*A
 * on device; rows outside the range are not written).
 * use_sp = 1: igraph-exact Dijkstra per source slot + self path (R-7, R-9);
 * use_sp = 0: direct edge per pair (R-10).  Synchronous. */
int shd_dev_build_rows(const ShdGraphDev* g, int use_sp, int row_lo, int row_hi, ShdEntry* tab);
/* The A x A latency half of the table (lat_ms doubles, row-major) by blocked
 * min-plus Floyd-Warshall (minplus.hip); whole-ms graphs only (-ENOTSUP
 * otherwise), V <= 16384.  Enqueued on stream (hipStream_t or NULL), no
 * waiting; *scratch: the caller's grow-only distance matrix (NULL the first
 * time), freed with shd_dev_fw_scratch_free. */
int shd_dev_fw_latency(const ShdGraphDev* g, double* d_lat, void** scratch, void* stream);
void shd_dev_fw_scratch_free(void* scratch);
/* Latency rows [row_lo, row_hi) by the bucketed frontier SSSP (frontier.hip):
 * whole-ms graphs, wmax = the largest edge latency in ms; synchronous. */
int shd_dev_frontier_latency(const ShdGraphDev* g, int row_lo, int row_hi, int wmax, double* d_lat, void* stream);
/* min latency over the entries (i, j), i < j, lat >= 0, of rows [row_lo,
 * row_hi) of an A-column table (rows: row i at rows + (i - row_lo) * A); -1 if none */
int shd_dev_min_upper(const ShdEntry* rows, int A, int row_lo, int row_hi, double* out);
/* Lazy row release (release.hip), asynchronous: queues on the release
 * scratch's own stream, for each listed row rows[r] (absolute slot, row r at
 * base + rows[r] * A) with touch sequence seqs[r], the minimum latency over
 * columns j != rows[r] with touch[j] > seqs[r] and lat >= 0 (touch: host
 * array of A sequences taken after the listed rows drew theirs); returns
 * without waiting.  Runs on the calling thread's device.  *scratch: grow-only
 * buffers + stream of the caller (NULL the first time), freed with
 * shd_dev_release_scratch_free. */
int shd_dev_release_launch(const ShdEntry* base, int A, const int32_t* rows, const uint32_t* seqs, int n,
                           const uint32_t* touch, void** scratch);
/* Waits for the launches since the last collect; their minima in launch
 * order into out (-1: none released), *n of them (at most cap). */
int shd_dev_release_collect(void* scratch, double* out, size_t cap, size_t* n);
/* rows launched and not yet collected */
size_t shd_dev_release_pending(void* scratch);
void shd_dev_release_scratch_free(void* scratch);

/* Packet round on device arrays (see shd_round_process_device). */
typedef struct {
    const ShdEntry* tab;      /* A x A */
    int A;
    int mode;                 /* 0 = owner by touch order, 1 = direct symmetric, 2 = direct + pair bits */
    const uint32_t* touch;    /* A, touch sequence (UINT32_MAX = never) */
    const uint32_t* pair_bits; /* A*A bits, mode 2 */
    const uint32_t* host_info; /* nhosts x {slot (UINT32_MAX = unattached), touch[slot]}: one 8-B gather */
    uint32_t nhosts;
    void* ws;                  /* the topology's device workspace (shd_dev_ws_new) */
    int row_lo, row_hi;        /* rows of tab present (a shard: others are never read) */
    uint32_t idx_base;         /* added to the record index an event carries (pkt_index) */
    const void* ptab;          /* NULL or the 8-B packet-path table {delay_ns, keep threshold} indexed as tab */
    /* path packet counters (topology_incrementPathPacketCounter, worker.c:551)
     * of every kept packet (delivered or dropped at the end time), at its
     * answering pair's flat entry index (oi * A + oj):
     *   plog: this round's slice of the counter log -- record i writes its
     *         key (u32, or u64 when plog64) or all-ones (not kept) at
     *         plog[i]; shd_dev_pcnt_fold adds logged keys into the dense
     *         counters (default, SHD_PCNT=log);
     *   pcnt: the dense u32 counters themselves, one device atomic per kept
     *         packet (SHD_PCNT=atomic, the A/B form);
     * both NULL: SHD_PCNT=0 (measurement only: counts are not kept). */
    void* plog;
    uint32_t plog64;
    uint32_t* pcnt;
} ShdPktCtx;

/* Path packet counter spill (packet.hip): every entry of cnt[0, n) whose
 * count -- cnt[i], plus d8[i] when the u8 delta layer d8 is not NULL -- is
 * >= thr is appended to list as {index (u64), value (u64)} (at most cap
 * entries; *d_nlist, device, counts all that qualified) and zeroed (both
 * layers) -- only the appended ones.  Synchronous on the calling thread's
 * device.  Returns the number of entries appended in *appended (host). */
int shd_dev_pcnt_spill(uint32_t* cnt, uint8_t* d8, size_t n, uint32_t thr, uint64_t* d_list, size_t cap,
                       uint32_t* d_nlist, size_t* appended);
/* Adds the L logged keys of `log` (u32 flat entry indices below N <=
 * SHD_PCNT_FOLD_MAX_N, all-ones = nothing; the counters of keys [n0, N)
 * exist, n0 = a shard's first row times A) into the counters: a two-level
 * partition of the keys into 32K-counter regions and one workgroup per
 * region that accumulates its keys in LDS and adds its counters to the
 * table.  With d8 (NULL: none) the counts go to the u8 delta layer d8[N]
 * (16-B aligned at index 0; a pair's count is dense + d8): a byte that would
 * pass 255 moves its whole value into dense with one device atomic and
 * restarts at 0, so the fold streams N bytes of deltas instead of 4N of
 * counters.  The log's buffer is overwritten (it holds the second level's
 * output).  Enqueued on stream; *scratch: grow-only buffers (NULL the first
 * time; shd_dev_pcnt_fold_reserve sizes them for L keys ahead), freed with
 * shd_dev_pcnt_scratch_free. */
#define SHD_PCNT_FOLD_MAX_N (1ull << 29)
int shd_dev_pcnt_fold(void* log, size_t L, uint32_t* dense, uint8_t* d8, uint64_t n0, uint64_t N, void** scratch,
                      void* stream);
int shd_dev_pcnt_fold_reserve(size_t L, void** scratch);
void shd_dev_pcnt_scratch_free(void* scratch);

/* The 8-B packet-path table of nent entries of tab ({u32 delay_ns =
 * ceil(lat * 1e6), u32 keep threshold over the 31-bit rand_r output}, or a
 * fallback mark where the f64 entry must decide) into d_out; synchronous. */
int shd_dev_ptab_build(const ShdEntry* tab, size_t nent, void* d_out, void* stream);

/* Round-pipeline workspace (grow-only device buffers + the event that marks
 * the end of its last use), one per topology; callers serialise its use. */
int shd_dev_ws_new(void** ws);
void shd_dev_ws_free(void* ws);
/* grow-only exchange scratch of a workspace: dev_bytes of device memory and
 * host_bytes of pinned host memory (either pointer may be NULL) */
int shd_dev_ws_scratch(void* ws, size_t dev_bytes, size_t host_bytes, void** d, void** h);
/* The exchange's count matrix (words <= 64 x 66 u64: device + pinned host),
 * allocated on first use and kept. */
int shd_dev_ws_xmat(void* ws, size_t words, uint64_t** d, uint64_t** h);
/* The workspace's round faults after its last use (waits for it): 0, or -EIO
 * once per faulted round (merge spin-out, metadata overflow, stage guard). */
int shd_dev_ws_check_faults(void* ws);
/* synchronise `stream` (the workspace's last use was launched on it) and
 * report that use's fault word, copied behind it on the same stream: one wait */
int shd_dev_ws_sync(void* ws, void* stream);
int shd_dev_packet_round(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                         uint64_t end_time, uint64_t bootstrap_end, ShdDeliv* d_out, uint32_t* d_dst_offsets,
                         uint8_t* d_status, uint64_t* d_counters, void* stream);
int shd_dev_deliv_sort(void* ws, const ShdDeliv* d_in, size_t n, uint32_t host_lo, uint32_t host_hi, ShdDeliv* d_out,
                       uint32_t* d_dst_offsets, void* stream);
/* The same regroup from W received blocks that are each grouped by
 * destination in event_compare order (the exchange's output): block k starts
 * at event d_bbase[k] of d_in (W + 1 prefix counts, device), d_rofs holds
 * per block the (host_hi - host_lo + 1) destination offsets relative to the
 * block.  No scatter: the runs are read in place.  sorted: every run is in
 * event_compare order inside each destination (merged, not sorted). */
int shd_dev_deliv_merge_runs(void* ws, const void* d_in, int wire, int sorted, size_t n, const uint32_t* d_rofs,
                             const uint32_t* d_bbase, uint32_t W, uint32_t host_lo, uint32_t host_hi, ShdDeliv* d_out,
                             uint32_t* d_dst_offsets, void* stream);
/* The same with run `self` read from d_self (this rank's own block, at its
 * element index: never sent through the transport); d_self NULL: none.
 * sorted: every run is sorted (a merge instead of the union's sort). */
int shd_dev_deliv_merge_runs_self(void* ws, const void* d_in, const void* d_self, uint32_t self, int wire, int sorted,
                                  size_t n, const uint32_t* d_rofs, const uint32_t* d_bbase, uint32_t W,
                                  uint32_t host_lo, uint32_t host_hi, ShdDeliv* d_out, uint32_t* d_dst_offsets,
                                  void* stream);
/* The sender's side of an exchanged round: decided events grouped by
 * destination as 24-B wire records {time, seq, src, pkt_index} into d_wire,
 * destination offsets (H + 1) into d_off.  sort_wire: each destination's
 * run in event_compare order (the part pipeline only); *sorted_out says
 * whether they are. */
int shd_dev_packet_round_grouped(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                                 uint64_t end_time, uint64_t bootstrap_end, void* d_wire, uint32_t* d_off,
                                 uint8_t* d_status, uint64_t* d_counters, void* stream, int sort_wire,
                                 int* sorted_out);
/* The same sender round in two halves for an exchange that sends in two
 * groups (xchg.hip): the per-owner cuts of the grouped output (d_cuts,
 * W + 1 words) come from the partition before any bucket is sorted and
 * front(user, d_cuts, sorted) is called (the exchange's count matrix goes
 * out on the stream behind them); then the buckets of the owners below
 * bounds[half] are sorted, the listed-segment count so far is copied to
 * d_listed_a and mid(user) is called (the exchange's host read-back);
 * then the rest.  With no part geometry (the slab pipeline) the whole round
 * runs first and both hooks follow it.  A hook's nonzero return stops
 * the round and is returned. */
typedef struct {
    int (*front)(void* user, const uint32_t* d_cuts, int sorted);
    int (*mid)(void* user);
    void* user;
} ShdSplitHooks;
int shd_dev_packet_round_grouped_split(const ShdPktCtx* c, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                                       uint64_t end_time, uint64_t bootstrap_end, void* d_wire, uint32_t* d_off,
                                       uint8_t* d_status, uint64_t* d_counters, void* stream, int sort_wire,
                                       const uint32_t* bounds, int W, int half, uint32_t* d_cuts,
                                       uint32_t* d_listed_a, const ShdSplitHooks* hooks);
/* streams and events of the split exchange (created on first use, kept
 * with the workspace): the transfer stream and four events */
int shd_dev_ws_xchg_sync_objs(void* ws, void** xfer_stream, void** events, int nevents);
/* decide + group + exchange + merge in one call (shd_round_process_exchange) */
int shd_dev_round_exchange(const ShdPktCtx* c, const ShdTransport* x, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                           uint64_t end_time, uint64_t bootstrap_end, const uint32_t* host_bounds, void* d_wire_send,
                           uint8_t* d_status, uint64_t* d_counters, void* d_wire_recv, size_t recv_cap,
                           ShdDeliv* d_out, uint32_t* d_out_offsets, size_t* n_out, void* stream);

/* out[i] = tab[idx[i]] for n entries (device pointers; synchronous; on the
 * calling thread's device) */
int shd_dev_gather_entries(const ShdEntry* tab, const uint64_t* d_idx, size_t n, ShdEntry* d_out);

/* multi-GPU rounds (xchg.hip) */
int shd_dev_route_records(const ShdPktCtx* c, const ShdTransport* x, const ShdPkt* d_recs, size_t n,
                          const uint32_t* row_bounds, ShdPkt* d_scratch, ShdPkt* d_recv, size_t recv_cap,
                          size_t* n_recv, void* stream);
int shd_dev_event_cuts(void* ws, const uint32_t* d_dst_offsets, const uint32_t* host_bounds, int world,
                       uint64_t* send_elems, void* stream);
/* shd_round_exchange's default form: events + per-destination run offsets to
 * every owner, regrouped there by shd_dev_deliv_merge_runs; synchronous */
int shd_dev_exchange_runs(void* ws, const ShdTransport* x, const ShdDeliv* d_events, const uint32_t* d_dst_offsets,
                          const uint32_t* host_bounds, ShdDeliv* d_recv, size_t recv_cap, ShdDeliv* d_out,
                          uint32_t* d_out_offsets, size_t* n_out, void* stream);
int shd_dev_exchange_blocks(const ShdTransport* x, const void* d_send, const uint64_t* send_elems, size_t elem_bytes,
                            void* d_recv, size_t recv_cap, size_t* n_recv, void* stream);

#ifdef __cplusplus
}
#endif
#endif
