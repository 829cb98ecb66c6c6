/*
 * oracle.h -- CPU restatement of Shadow's network plane.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in shadow_amd/ (the product) links,
 * imports or executes this code; it is the checker used by tests/,
 * __graft_entry__.smoke() and the cpu_baseline leg of bench.py.
 *
 * Every function restates a reference function; the citation is on the
 * definition in oracle.c (paths are relative to /root/reference/src/main).
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - rand_r streams and seed chain: pinned against the reference's own
 *     utility/random.c compiled from its sources (oracle/ref_driver.c).
 *   - per-destination event order: pinned against the reference's own
 *     utility/priority_queue.c compiled from its sources, driven with an
 *     event_compare restatement (oracle/ref_driver.c).
 *   - unit strings: pinned against the Rust unit tests in
 *     core/support/units.rs:579-775 (restated as fixture cases).
 *   - self-loop graphs (every graph the reference's tests use): pinned by the
 *     reference test configs (1_gbit_switch, tcp-*-lossy.yaml).
 *   - multi-vertex Dijkstra path choice: igraph is not vendored and absent
 *     from this image -> restatement-pinned (igraph 0.8 2wheap semantics),
 *     fp64 latencies cross-checked against networkx (tie-independent).
 */
#ifndef SHD_ORACLE_H
#define SHD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- units (core/support/units.rs) ---- */
int64_t orc_parse_time_ns(const char* s);
int64_t orc_parse_bandwidth_bits(const char* s);

/* ---- glibc rand_r streams (utility/random.c) ---- */
int orc_rand_r(uint32_t* state);
double orc_next_double(uint32_t* state);
uint32_t orc_next_uint(uint32_t* state);

/* ---- topology (routing/topology.c) ---- */
typedef struct OrcTopo OrcTopo;

/* NULL on an invalid graph (topology_new returns NULL, topology.c:2345-2351). */
OrcTopo* orc_topology_new(const char* gml_text, int use_shortest_path);
void orc_topology_free(OrcTopo* t);
int orc_topology_vertex_count(const OrcTopo* t);
int orc_topology_edge_count(const OrcTopo* t);
int orc_topology_is_directed(const OrcTopo* t);
int orc_topology_is_complete(const OrcTopo* t);

/* Returns the chosen vertex index (>= 0) or -1.  rng_state is the host's
 * Random seedState; exactly the reference's draws are consumed. */
int orc_topology_attach(OrcTopo* t, uint32_t ip_net, uint32_t* rng_state, const char* ip_hint,
                        const char* city_hint, const char* country_hint, uint64_t* bw_down_kibps,
                        uint64_t* bw_up_kibps);
void orc_topology_detach(OrcTopo* t, uint32_t ip_net);

double orc_topology_get_latency(OrcTopo* t, uint32_t src_ip, uint32_t dst_ip);
double orc_topology_get_reliability(OrcTopo* t, uint32_t src_ip, uint32_t dst_ip);
int orc_topology_is_routable(OrcTopo* t, uint32_t src_ip, uint32_t dst_ip);
void orc_topology_increment_path_packet_counter(OrcTopo* t, uint32_t src_ip, uint32_t dst_ip);
uint64_t orc_topology_path_packet_count(OrcTopo* t, uint32_t src_ip, uint32_t dst_ip);

/* Running min of stored path latencies (topology.c:1253-1264) and the number
 * of worker_updateMinTimeJump calls it has produced. */
double orc_topology_min_path_latency(const OrcTopo* t);
int orc_topology_min_jump_updates(const OrcTopo* t);
/* controller_updateMinTimeJump's view: nextMinJumpTime in ns (controller.c:141-153). */
uint64_t orc_controller_next_min_jump_ns(const OrcTopo* t);

/* Stand-alone row computation, no cache side effects: fills lat/rel for the
 * given target vertices exactly as _topology_computeSourcePaths would store
 * them for source `src` (src==target -> the self path of R-9).  Returns 0. */
int orc_compute_row(OrcTopo* t, int src, const int* targets, int ntargets, double* lat,
                    double* rel);
/* use_shortest_path=false value of (src,dst) (topology.c:1816-1858). */
int orc_direct_path(OrcTopo* t, int src, int dst, double* lat, double* rel);
void orc_direct_row(OrcTopo* t, int src, const int* targets, int ntargets, double* lat, double* rel);
int orc_vertex_of_ip(OrcTopo* t, uint32_t ip_net);

/* Seed the cache with a precomputed row table (for CPU baseline timing of the
 * packet hand-off only): row-major nslots x nslots over the attached vertex
 * list `slots`.  Entries are inserted as if rows were touched in slot order. */
int orc_topology_preload_table(OrcTopo* t, const int* slots, int nslots, const double* lat,
                               const double* rel);
/* Full rows (nrows x ncols, columns = the attached vertices `cols`) inserted
 * as if rows[0], rows[1], ... were touched first, in that order. */
int orc_topology_preload_rows(OrcTopo* t, const int* rows, int nrows, const int* cols, int ncols,
                              const double* lat, const double* rel);

/* ---- packet hand-off (core/worker.c:517-576, scheduler push, event order) ---- */
typedef struct OrcPkt {
    uint64_t now;       /* worker_getCurrentTime() at send */
    uint64_t seq;       /* srcHostEventID (per-src monotone) */
    uint32_t src_host;  /* host index = registration order (GQuark order) */
    uint32_t dst_host;
    uint32_t rng_state; /* src host Random seedState before the draw */
    uint32_t payload_len;
} OrcPkt;

typedef struct OrcDeliv {
    uint64_t time;
    uint64_t seq;
    uint32_t src_host;
    uint32_t dst_host;
    uint32_t pkt_index;
    uint32_t pad;
} OrcDeliv;

enum { ORC_DROP_LOSS = 0, ORC_DELIVERED = 1, ORC_DROP_END = 2 };

/* Processes one round's packets in input order against the topology (with the
 * reference's lazy cache side effects), pushes kept events into one binary
 * heap per destination host ordered by event_compare, then pops every heap in
 * host order.  out must hold n entries; returns the number delivered.
 * min_time receives the worker_setMinEventTimeNextRound minimum (UINT64_MAX
 * if none).  host_ips[h] is host h's network-order IP. */
size_t orc_round(OrcTopo* t, const uint32_t* host_ips, uint32_t nhosts, uint64_t barrier,
                 uint64_t end_time, uint64_t bootstrap_end, const OrcPkt* pkts, size_t n,
                 OrcDeliv* out, uint8_t* status, uint64_t* min_time);
/* The same hand-off on nthreads worker threads sharded by source host, with
 * per-destination queue mutexes (host-single policy analogue); every path
 * the packets use must already be cached (else returns (size_t)-1). */
size_t orc_round_mt(OrcTopo* t, const uint32_t* host_ips, uint32_t nhosts, uint64_t barrier, uint64_t end_time,
                    uint64_t bootstrap_end, const OrcPkt* pkts, size_t n, int nthreads, OrcDeliv* out,
                    uint8_t* status, uint64_t* min_time);

/* _topology_logAllCachedPaths: every cached path as one '\n'-terminated line,
 * in (source, destination) vertex order.  Writes at most cap bytes (NUL
 * included) and returns the length the full log needs. */
size_t orc_topology_log_cached_paths(OrcTopo* t, char* buf, size_t cap);

/* Binary heap restating utility/priority_queue.c with event_compare
 * (core/work/event.c:109-152); exposed for the PQ golden test. */
typedef struct OrcEvKey {
    uint64_t time;
    uint32_t dst;
    uint32_t src;
    uint64_t seq;
} OrcEvKey;
/* Pushes keys[0..n) in order, pops all; writes pop order (indices) to order. */
void orc_pq_order(const OrcEvKey* keys, size_t n, uint32_t* order);

/* Destination routers (routing/router.c:103-131) with the CoDel queue
 * manager (routing/router_queue_codel.c:113-265), one router after another.
 * Same record layouts as include/shdnet.h's ShdCodel*; the oracle keeps its
 * queues as growable FIFOs (the reference's GQueue), not rings: entries in
 * flight are carried in and out through `queues`/`qlen` (per router, FIFO
 * order, capacity `qcap` each).  Returns 0, -2 if a queue would exceed qcap,
 * -1 on a dequeue before an entry's enqueue time (utility_assert :172). */
typedef struct OrcCodelState {
    uint64_t interval_expire, next_drop, total_size;
    uint32_t mode, drop_count, drop_count_last, head, len, pad;
} OrcCodelState;
typedef struct OrcCodelEntry {
    uint64_t enqueue_ts;
    uint32_t pkt, length;
} OrcCodelEntry;
typedef struct OrcCodelOp {
    uint64_t time;
    uint32_t kind, pkt, length, pad;
} OrcCodelOp;
int orc_codel_run(uint32_t nrouters, const uint32_t* op_offsets, const OrcCodelOp* ops, OrcCodelState* states,
                  OrcCodelEntry* rings, uint32_t ring_cap, uint32_t* deq_out, uint64_t* fate);

/* Network interfaces with the upstream router (host/network_interface.c,
 * routing/router.c, router_queue_codel.c), as an event-driven simulation per
 * host.  Same records and arguments as include/shdnet.h's shd_nic_*
 * (host arrays).  Returns 0, -1 bad input, -2 ring overflow, -3 no memory. */
typedef struct OrcNicState {
    uint64_t recv_remaining, recv_refill, recv_capacity;
    uint64_t send_remaining, send_refill, send_capacity;
    uint64_t refill_start, refill_time;
    uint32_t refill_pending, pad0;
    uint64_t pad1;
    OrcCodelState router;
} OrcNicState;
typedef struct OrcNicSend {
    uint64_t ready;
    uint32_t id, length;
} OrcNicSend;
int orc_nic_init(uint32_t n, const uint64_t* down, const uint64_t* up, uint64_t start, OrcNicState* st);
int orc_nic_run(uint32_t nhosts, uint32_t host_base, const OrcDeliv* ev, const uint32_t* eoff, const uint32_t* elen,
                const OrcNicSend* sends, const uint32_t* soff, uint64_t window_end, uint64_t boot_end,
                OrcNicState* states, OrcCodelEntry* rings, uint32_t ring_cap, uint32_t id_base, uint64_t* rtime,
                uint8_t* rstat, uint64_t fate_cap, uint64_t* stime);


#ifdef __cplusplus
}
#endif
#endif
