/*
 * shdnet.h -- C ABI of the MI355X-native Shadow network plane (libshdnet.so).
 *
 * Drop-in for two reference paths (citations into /root/reference/src/main):
 *   1. routing/topology.h:17-28 -- topology_new/free/attach/detach/isRoutable/
 *      getLatency/getReliability/incrementPathPacketCounter, including the
 *      worker_updateMinTimeJump side effect (worker.h:89, topology.c:1253-1264).
 *   2. the body of core/worker.c:517-576 worker_sendPacket + core/scheduler/
 *      scheduler.c:232-255 scheduler_push + scheduler_policy_host_single.c:
 *      174-220 push, batched per round: the CPU reserves the
 *      sender's rand_r draw at send time and appends a record; at the round
 *      boundary the GPU decides loss, computes delivery times, clamps to the
 *      barrier and emits per-destination event segments ordered by
 *      event_compare (core/work/event.c:109-152).
 *
 * Conventions: plain C types only; IPv4 addresses are network-order in_addr_t
 * values (address_toNetworkIP); host ids are dense indices in registration
 * order (the order of their GQuarks, manager.c:343), so comparing ids compares
 * GQuarks; times are SimulationTime nanoseconds.  Every entry point returns an
 * int status (0 or a negative errno) and never unwinds across the ABI; the
 * topology_* compatibility values (-1 latency, FALSE routable) are produced by
 * the wrappers shown in INTEGRATION.md.  There is no CPU compute fallback: if
 * no gfx950 device is usable every compute entry point returns -ENODEV.
 */
#ifndef SHDNET_H
#define SHDNET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHDNET_ABI_VERSION 1

typedef struct ShdTopology ShdTopology;

/* Called whenever the running minimum of released path latencies decreases;
 * replaces worker_updateMinTimeJump(gdouble) (worker.c:624-626). */
typedef void (*ShdMinJumpFn)(double min_latency_ms, void* user);

/* ---------------------------------------------------------------------- */
/* Routing (replaces routing/topology.h)                                   */
/* ---------------------------------------------------------------------- */

/* topology_new (topology.h:17, topology.c:2328-2354).  Reads and validates
 * the GML graph at gml_path (igraph GML dialect, validation of
 * topology.c:1040-1063) and extracts edge weights.  -EINVAL on an invalid
 * graph (reference: error() + NULL), -ENOENT if the file cannot be read,
 * -ENOTSUP for graphs with parallel edges (their igraph edge choice is
 * unpinned).  device: HIP device ordinal used for all compute. */
int shd_topology_new(const char* gml_path, int use_shortest_path, int device, ShdTopology** out);
/* Same, from GML text in memory (the controller writes the text to a file
 * only to hand it to igraph, controller.c:155-188). */
int shd_topology_new_from_text(const char* gml_text, int use_shortest_path, int device, ShdTopology** out);
/* topology_free (topology.h:18, topology.c:2283-2326) */
void shd_topology_free(ShdTopology* top);

/* topology_attach (topology.h:20-22, topology.c:2218-2272).  rng_state is
 * the host's Random seedState (random.c:15-18); the reference's draw is
 * consumed from it when the attach is random.  host_id registers the
 * address's host for the packet path.  bw outputs in KiB/s, may be NULL.
 * Attaching after the first path lookup returns -EBUSY (Shadow attaches
 * every host before the simulation starts, controller.c:333-336). */
int shd_topology_attach(ShdTopology* top, uint32_t host_id, uint32_t ip_net, uint32_t* rng_state,
                        const char* ip_hint, const char* city_hint, const char* country_hint,
                        uint64_t* bw_down_kibps, uint64_t* bw_up_kibps);
/* topology_detach (topology.h:23, topology.c:2274-2281): removes the IP only. */
int shd_topology_detach(ShdTopology* top, uint32_t ip_net);

/* Computes every attached source row of the routing table on the GPU
 * (igraph-exact Dijkstra per source) and keeps it
 * resident in HBM.  Called implicitly by the first lookup if not called
 * explicitly.  Rows are only *released* (cache side effects, min-jump) in
 * the reference's lazy touch order, by the lookups below. */
int shd_topology_build_routes(ShdTopology* top);

/* topology_getLatency / getReliability / isRoutable /
 * incrementPathPacketCounter (topology.h:25-28, topology.c:1983-2022).
 * Status -ENOENT when an address is not attached (reference returns -1 /
 * FALSE), -EHOSTUNREACH for an attached pair with no path (reference:
 * utility_panic, topology.c:1970-1976). */
int shd_topology_get_latency(ShdTopology* top, uint32_t src_ip, uint32_t dst_ip, double* latency_ms);
int shd_topology_get_reliability(ShdTopology* top, uint32_t src_ip, uint32_t dst_ip, double* reliability);
int shd_topology_is_routable(ShdTopology* top, uint32_t src_ip, uint32_t dst_ip, int* routable);
int shd_topology_increment_path_packet_counter(ShdTopology* top, uint32_t src_ip, uint32_t dst_ip);
int shd_topology_get_path_packet_count(ShdTopology* top, uint32_t src_ip, uint32_t dst_ip, uint64_t* count);

/* ---- DNS: host address assignment (routing/dns.c) ---------------------- */
/* dns_new (dns.c:294-305): the generator starts after 11.0.0.0. */
typedef struct ShdDns ShdDns;
int shd_dns_new(ShdDns** out);
void shd_dns_free(ShdDns* dns);
/* dns_register (dns.c:125-163): requested_ip may be NULL (generate); an
 * unparsable, reserved (_dns_isRestricted, :89-106) or taken address is
 * replaced by the next free generated one; "127.0.0.1" is a local address
 * and is not stored.  Every call takes the next MAC number.  ip_net is in
 * network byte order. */
int shd_dns_register(ShdDns* dns, const char* name, const char* requested_ip, uint32_t* ip_net, uint32_t* mac,
                     int* is_local);
/* n registrations in order under one lock (startup: 200k hosts); the
 * request array may be NULL (all generated). */
int shd_dns_register_batch(ShdDns* dns, uint32_t n, const char* const* names, const char* const* requested_ips,
                           uint32_t* ip_net, uint32_t* mac, uint8_t* is_local);
/* dns_deregister (dns.c:165-181) of the address (ip_net, name, is_local) */
int shd_dns_deregister(ShdDns* dns, uint32_t ip_net, const char* name, int is_local);
/* dns_resolveIPToAddress / dns_resolveNameToAddress (dns.c:183-203):
 * -ENOENT when absent.  name gets at most cap bytes (NUL included). */
int shd_dns_resolve_ip(ShdDns* dns, uint32_t ip_net, char* name, size_t cap, uint32_t* mac);
int shd_dns_resolve_name(ShdDns* dns, const char* name, uint32_t* ip_net, uint32_t* mac);
/* The hosts file dns_getHostsFilePath writes (dns.c:231-290): "127.0.0.1
 * localhost" then "<ip> <name>" per name mapping, in registration order
 * (the reference's order is glib's hash order).  At most cap bytes (NUL
 * included) into buf; *len = the full length. */
int shd_dns_hosts_file(ShdDns* dns, char* buf, size_t cap, size_t* len);

/* topology_free's teardown log (_topology_logAllCachedPaths,
 * topology.c:1860-1897 called at :2287; path_toString, path.c:62-75): fn gets
 * one line per cached path -- "Found path <srcID>-><dstID> in cache:
 * SourceIndex=.. DestinationIndex=.. Latency=%f Reliability=%f PacketCount=..
 * isDirect=True|False" ("<->" on undirected graphs) -- in (source,
 * destination) vertex order (the reference's order is glib's hash order).
 * The cache is the release state (touched rows, released self paths, stored
 * direct pairs) with the path packet counters.  A device-resident table is
 * read back one row at a time. */
typedef void (*ShdPathLogFn)(const char* line, void* user);
int shd_topology_log_cached_paths(ShdTopology* top, ShdPathLogFn fn, void* user, uint64_t* nlines);

/* n lookups in one call, in order, with the same side effects as n calls of
 * topology_getLatency (the pair's row touch, min-jump): lat_ms / rel (either
 * may be NULL) receive the answers.  For a device-resident table the answers
 * come from one device gather instead of n 16-byte PCIe reads.  Stops at
 * the first unattached address (-ENOENT; earlier lookups took effect). */
int shd_topology_lookup_batch(ShdTopology* top, const uint32_t* src_ips, const uint32_t* dst_ips, size_t n,
                              double* lat_ms, double* rel);

/* The min-jump callback (worker_updateMinTimeJump, worker.h:89) gets every
 * new running minimum, strictly decreasing, in the serial touch order.  On a
 * device-resident table the rows first touched by lookups and sends are
 * reduced on the GPU asynchronously, in batches, and the callback fires when
 * their minima are folded: at the latest at the next round boundary
 * (shd_round_collect), minimum query or teardown log, or at
 * shd_topology_release_sync.  Shadow's controller reads the min jump only at
 * the round boundary (controller.c:390-422), so it sees the same values. */
int shd_topology_set_min_jump_callback(ShdTopology* top, ShdMinJumpFn fn, void* user);
/* Running min of released latencies (topology.c:48, 1253-1264); 0 if none.
 * Folds the queued releases first. */
int shd_topology_get_min_path_latency(ShdTopology* top, double* min_ms);
/* Waits for the queued releases of a device-resident table and folds their
 * minima (callback included) in touch order; for callers of the device round
 * API (shd_round_process_device) at their round boundary. */
int shd_topology_release_sync(ShdTopology* top);

/* Introspection for tests and tooling. */
int shd_topology_info(ShdTopology* top, int* vertices, int* edges, int* directed, int* complete,
                      int* attached_vertices);
/* Vertex index a host id / ip is attached to (-1 if none). */
int shd_topology_vertex_of_host(ShdTopology* top, uint32_t host_id, int* vertex);
/* Copies the full device routing table (row-major over attached vertex
 * slots, slots ordered by vertex index) to host memory: lat_ms/rel each
 * hold slots*slots doubles; slot_vertex receives the slot->vertex map. */
int shd_topology_copy_table(ShdTopology* top, double* lat_ms, double* rel, int32_t* slot_vertex, int cap_slots);
/* Multi-GPU row sharding: number of table slots A, then
 * compute rows [row_lo, row_hi) into a caller-owned device table of A*A
 * 16-byte {lat_ms, rel} entries (e.g. a torch tensor that an RCCL
 * all-gather completes), then adopt the completed table as the resident one
 * (the caller keeps it alive for the topology's lifetime). */
int shd_topology_slot_count(ShdTopology* top, int* slots);
/* Device memory for a caller-owned routing table (or any device array the
 * library should own the placement of): the allocation the library uses for
 * its own tables (shd_topology_build_routes).  *contiguous (may be NULL)
 * reports whether it is physically contiguous (currently never: measured
 * slower for the table build).  Free with shd_device_free. */
int shd_device_alloc_table(int device, size_t bytes, void** d_out, int* contiguous);
int shd_device_free(int device, void* d_ptr);
/* Device-to-device copy (e.g. an all-gathered table into one from
 * shd_device_alloc_table); synchronous. */
int shd_device_copy(int device, void* d_dst, const void* d_src, size_t bytes);
int shd_topology_build_rows_device(ShdTopology* top, int row_lo, int row_hi, void* d_table);
/* Latencies only: the A x A lat_ms column of the table (row-major doubles,
 * slots as above) into device memory d_lat, by blocked min-plus
 * Floyd-Warshall over 64 x 64 LDS tiles -- the shortest-path latencies do
 * not depend on igraph's tie order (the reliabilities do, which is why the
 * table itself is built by the Dijkstra kernels).  Bit-identical to the
 * table's latencies; graphs whose edge latencies are all whole ms and with at
 * most 16,384 vertices (-ENOTSUP otherwise).  Releases nothing (no lookup
 * side effects).  Enqueued on stream (hipStream_t) without waiting, on the
 * topology's persistent distance scratch (calls on other streams wait for its
 * last use); stream NULL: synchronous. */
int shd_topology_latency_table_fw(ShdTopology* top, void* d_lat, void* stream);
/* Latencies only, for sparse graphs: rows [row_lo, row_hi) of the lat_ms
 * column ((row_hi - row_lo) x A doubles, row - row_lo major) into d_lat, by a
 * bucketed frontier SSSP per source (Dial's algorithm: a ring of
 * max-latency + 1 distance buckets, each settled bucket's edges relaxed
 * edge-parallel by one wave; csrc/frontier.hip).  Same entries as the
 * table's latency column (tie-independent, as for the min-plus entry above),
 * no lookup side effects; graphs whose edge latencies are all whole ms and at
 * most 3,348 ms (the per-wave bucket ring lives in LDS) -- -ENOTSUP
 * otherwise.  Synchronous on stream (hipStream_t, NULL: the null stream). */
int shd_topology_latency_rows_frontier(ShdTopology* top, int row_lo, int row_hi, void* d_lat, void* stream);
int shd_topology_adopt_table_device(ShdTopology* top, void* d_table);
/* Adopts a device table WITHOUT a host mirror (tables larger than host RAM
 * wants: A = 86k slots is 120 GB).  Nothing is released at adoption: as in
 * the reference, the first lookup or send that misses row i releases it
 * (topology.c:1189-1265, 1900-1981) -- here a device pass over row i that
 * finds what the reference's store loop would store (columns whose row was
 * not touched before i) and feeds their minimum to the min-jump callback.
 * Host lookups read single entries from the device.  use_shortest_path
 * graphs only (-ENOTSUP), before any lookup (-EBUSY).  The caller keeps
 * d_table alive for the topology's lifetime. */
int shd_topology_adopt_table_device_resident(ShdTopology* top, void* d_table);
/* Single-process multi-GPU table (Shadow is one process with one manager,
 * core/manager.c:543-577): shard k holds rows [row_bounds[k],
 * row_bounds[k+1]) (nshards + 1 slot ids, host memory) in d_rows[k], a device
 * allocation of (row_bounds[k+1] - row_bounds[k]) * A entries on
 * devices[k] (e.g. built by shd_topology_build_rows_device on that device's
 * topology copy, or shd_topology_build_shards).  One release state for the
 * whole table: lookups from any worker thread read the owning shard's
 * device, a row release reduces the row on its shard's device.  Destination
 * hosts are split evenly over the shards for the rounds
 * (shd_topology_set_host_bounds).  Same conditions as above. */
int shd_topology_adopt_table_shards(ShdTopology* top, int nshards, const int* devices, void* const* d_rows,
                                    const int* row_bounds);
/* Builds every row of a single-process multi-GPU table: shard k's rows are
 * computed on devices[k] into d_rows[k] (caller-owned, sized as above), all
 * shards concurrently (one host thread per shard). */
int shd_topology_build_shards(ShdTopology* top, int nshards, const int* devices, void* const* d_rows,
                              const int* row_bounds);
/* Destination hosts owned by each shard of a multi-shard table in its rounds
 * (nshards + 1 host ids, [0, nhosts)); default: an even split. */
int shd_topology_set_host_bounds(ShdTopology* top, const uint32_t* host_bounds);
/* Touches every untouched attached vertex row, in slot order (steady state
 * of a long simulation; used by benchmarks before timing). */
int shd_topology_touch_all(ShdTopology* top);
/* Release state, for tests and tooling: per table slot, the touch sequence
 * number of its row (UINT32_MAX = never touched) and whether its self pair
 * was released; either pointer may be NULL.  The owner of a released pair
 * {X, Y} is the row with the smaller sequence number. */
int shd_topology_touch_order(ShdTopology* top, uint32_t* touch_seq, uint8_t* self_released, int cap_slots);

/* ---------------------------------------------------------------------- */
/* Per-round packet hand-off (replaces worker_sendPacket + scheduler push) */
/* ---------------------------------------------------------------------- */

/* One send, recorded by the CPU at worker_sendPacket time (32 bytes). */
typedef struct ShdPkt {
    uint64_t now;         /* worker_getCurrentTime() */
    uint64_t seq;         /* srcHostEventID (host_getNewEventID, host.c:368-371) */
    uint32_t src_host;    /* host ids (dense, registration order) */
    uint32_t dst_host;
    uint32_t rng_state;   /* sender's Random seedState BEFORE the reserved draw */
    uint32_t payload_len; /* packet_getPayloadLength(); 0 = control packet */
} ShdPkt;

/* One delivered event (32 bytes), ordered by event_compare. */
typedef struct ShdDeliv {
    uint64_t time; /* delivery time after the host-single barrier clamp */
    uint64_t seq;
    uint32_t src_host;
    uint32_t dst_host;
    uint32_t pkt_index; /* index of the record in the round's batch */
    uint32_t pad;
} ShdDeliv;

/* Per-record outcome. */
enum { SHD_DROPPED_LOSS = 0, SHD_DELIVERED = 1, SHD_DROPPED_END = 2 };

/* Round parameters: barrier = current round end (scheduler.c:247),
 * end_time = scheduler endTime (scheduler.c:236), bootstrap_end =
 * bootstrap_end_time (worker.rs:339-341). */
int shd_round_begin(ShdTopology* top, uint64_t barrier, uint64_t end_time, uint64_t bootstrap_end);
/* Number of worker threads that append (Shadow's worker pool size,
 * worker.c:132-185); each gets its own staging buffer.  Default 1.  Only
 * between rounds (-EBUSY while records are staged). */
int shd_round_set_workers(ShdTopology* top, int nworkers);
/* Called by worker `worker` inside worker_sendPacket, at send time: performs
 * the reference's lookup side effects for each send right away, in send
 * order (row touch, min-jump -- topology_getReliability at worker.c:539), and
 * stages the records (host memory, copied) in that worker's own buffer.
 * Workers append concurrently without locking each other; a worker index is
 * used by one thread at a time.  The whole batch is validated first: on
 * -ENOENT (an unattached host) nothing was staged and no side effect ran.
 * pkt_index in shd_round_collect's output counts records in worker order
 * (worker 0's records first, each worker's in append order). */
int shd_round_append_worker(ShdTopology* top, int worker, const ShdPkt* recs, size_t n);
/* shd_round_append_worker(top, 0, recs, n) (single producer). */
int shd_round_append(ShdTopology* top, const ShdPkt* recs, size_t n);
/* Records staged for the current round, over all workers. */
int shd_round_staged(ShdTopology* top, size_t* n);
/* At the round boundary (workers idle): runs the batch on the GPU and
 * returns delivered events grouped by
 * destination host: out[dst_offsets[h] .. dst_offsets[h+1]) is host h's
 * events in event_compare order (dst_offsets has nhosts+1 entries, may be
 * NULL).  status (may be NULL) receives one outcome per appended record.
 * min_time: minimum delivered time >= barrier (worker.c:350-363),
 * UINT64_MAX if none. */
int shd_round_collect(ShdTopology* top, ShdDeliv* out, size_t cap, size_t* n_out, uint32_t* dst_offsets,
                      uint8_t* status, uint64_t* min_time);
/* Pinned (page-locked) host memory, e.g. for shd_round_collect's out /
 * dst_offsets / status: copies into it run at the host link's full rate.
 * Any host memory works there; this is the fast kind.  Worker staging
 * buffers are pinned by the library itself. */
int shd_host_buffer_alloc(size_t bytes, void** out);
void shd_host_buffer_free(void* p);

/* Path packet counters (topology_incrementPathPacketCounter, worker.c:551):
 * every round -- shd_round_collect, shd_round_process_device,
 * shd_round_process_exchange -- counts each kept packet (delivered or
 * dropped at the end time) at its answering pair on the device, inside the
 * round's own kernels; shd_topology_get_path_packet_count and the teardown
 * log read them back.  With a row-sharded table a rank counts the packets
 * it decides (the pair's total is the sum over ranks). */
/* Every counter of table rows [row_lo, row_hi) (slots as in
 * shd_topology_copy_table): counts[(i - row_lo) * A + j] = the packets
 * counted at pair (i, j), host-side increments included (the count the
 * teardown log prints for the cached path (i, j)).  Rows this topology does
 * not hold (another rank's shard) read 0. */
int shd_topology_copy_path_packet_counts(ShdTopology* top, int row_lo, int row_hi, uint64_t* counts);
/* The rounds log each kept packet's pair (one store per record, inside the
 * round's own kernels) and the log is added into the device counters in
 * bulk: when it fills, before any of the readers above, and here.  Waits for
 * every round in flight on the topology's device(s).  A benchmark calls it
 * inside its timed region so that every counted packet is in the time. */
int shd_topology_path_counts_sync(ShdTopology* top);

/* Device-resident variant (inputs already in HBM; used by benchmarks and the
 * multi-GPU exchange).  All pointers are device pointers; stream is a
 * hipStream_t (NULL = default stream).  The lookup side effects (row touch,
 * min-jump) are NOT applied: rows must have been touched (shd_round_append
 * or shd_topology_touch_all); the path packet counters are counted.
 * out needs n entries, dst_offsets nhosts+1, status n; counters[0] =
 * delivered count, counters[1] = min delivered time (both written async).
 * A round whose device-side guards fired (a merge tile that gave up waiting,
 * a metadata overflow, an out-of-range overflow event) has SHD_ROUND_FAULT
 * set in counters[0] -- in that same round, so an asynchronous caller sees
 * it with the count -- and its outputs must not be used; the call returns
 * -EIO itself when stream is NULL (synchronous).  With a stream, counters[0]
 * bit 63 is the authoritative per-round signal; the sticky fault word is
 * also reported (-EIO, once) by some later call on the topology after the
 * faulted round has completed -- not necessarily the next call, which may
 * start while that round still runs. */
#define SHD_ROUND_FAULT (1ull << 63)
int shd_round_process_device(ShdTopology* top, const ShdPkt* d_recs, size_t n, uint64_t barrier,
                             uint64_t end_time, uint64_t bootstrap_end, ShdDeliv* d_out,
                             uint32_t* d_dst_offsets, uint8_t* d_status, uint64_t* d_counters, void* stream);
/* Number of registered hosts (dst_offsets needs this + 1 entries). */
int shd_topology_host_count(ShdTopology* top, uint32_t* nhosts);

/* Regroups already-decided delivered events (e.g. after a multi-GPU
 * all-to-all) into event_compare order per destination host in
 * [host_lo, host_hi).  Device pointers. */
int shd_deliv_sort_device(ShdTopology* top, const ShdDeliv* d_in, size_t n, uint32_t host_lo, uint32_t host_hi,
                          ShdDeliv* d_out, uint32_t* d_dst_offsets, void* stream);

/* ---------------------------------------------------------------------- */
/* Multi-GPU rounds: one topology per GPU / rank           */
/* ---------------------------------------------------------------------- */

/* The collectives a multi-GPU round needs, supplied by the caller: Shadow's
 * C host plugs in RCCL (shd_transport_rccl_new below: ncclSend/ncclRecv over
 * xGMI); tests plug in gloo.  Every call is collective over `world` ranks.
 *   alltoall_u64: host arrays of `world` values; recv[r] = what rank r sent
 *                 to this rank.
 *   alltoallv:    device buffers; this rank's block for peer r is
 *                 send_bytes[r] bytes, blocks contiguous in rank order in
 *                 d_send; the blocks received land contiguous in rank order
 *                 in d_recv.  Enqueued on `stream` (hipStream_t) or completed
 *                 before returning.
 *   allgatherv:   in place on the device buffer d_buf: rank r contributes
 *                 bytes [offsets[r], offsets[r+1]) (world + 1 host values,
 *                 the same on every rank); afterwards every rank holds every
 *                 block.  Enqueued on `stream` or completed before returning.
 *                 Only shd_topology_allgather_rows needs it (may be NULL
 *                 otherwise).
 * Return 0 or a negative errno. */
typedef struct ShdTransport {
    int rank, world;
    void* user;
    int (*alltoall_u64)(void* user, const uint64_t* send, uint64_t* recv);
    int (*alltoallv)(void* user, const void* d_send, const uint64_t* send_bytes, void* d_recv,
                     const uint64_t* recv_bytes, void* stream);
    int (*allgatherv)(void* user, void* d_buf, const uint64_t* offsets, void* stream);
} ShdTransport;

/* Full-matrix export of a row-sharded table ("RCCL
 * all-gather over xGMI only when a full matrix is requested"): d_table is
 * this rank's A x A table (A = shd_topology_slot_count) in which rank r has
 * built rows [row_bounds[r], row_bounds[r+1]) at their own offsets
 * (shd_topology_build_rows_device); on return every rank's d_table holds
 * every row, ready for shd_topology_adopt_table_device.  row_bounds: world +
 * 1 slot ids covering [0, A).  Synchronous (stream: hipStream_t or NULL). */
int shd_topology_allgather_rows(ShdTopology* top, const ShdTransport* xport, void* d_table, const uint32_t* row_bounds,
                                void* stream);

/* Destination-owner exchange of one round's delivered events: rank r owns
 * the destination hosts [host_bounds[r], host_bounds[r+1]) (host memory,
 * world+1 ids).  d_events / d_dst_offsets are this rank's
 * shd_round_process_device output (events grouped by destination over all
 * nhosts).  The events of every rank's destinations are sent there
 * (alltoallv), received into d_recv (capacity recv_cap events) and regrouped
 * into event_compare order per owned destination: d_out (recv_cap events),
 * d_out_offsets (owned hosts + 1).  *n_out = events received.  The union
 * over ranks equals a single-GPU round over all ranks' records (the order
 * is a total order).  Synchronous. */
int shd_round_exchange(ShdTopology* top, const ShdTransport* xport, const ShdDeliv* d_events,
                       const uint32_t* d_dst_offsets, const uint32_t* host_bounds, ShdDeliv* d_recv, size_t recv_cap,
                       ShdDeliv* d_out, uint32_t* d_out_offsets, size_t* n_out, void* stream);
/* One round decided and exchanged in one call (the multi-GPU form of
 * shd_round_process_device + shd_round_exchange): this rank's records are
 * decided, grouped by destination WITHOUT the per-destination sort (the
 * owner sorts the union of what it receives anyway) and shipped as 24-byte
 * wire records {time, srcHostEventID, src host, pkt_index} -- a quarter
 * fewer bytes over xGMI than ShdDeliv -- to the destinations' owners, which
 * merge them into event_compare order: d_out / d_out_offsets / *n_out as
 * shd_round_exchange's.  d_send: >= 24 * n bytes; d_recv: recv_cap wire
 * records (24 * recv_cap bytes); d_status / d_counters as
 * shd_round_process_device (counters[0]: events this rank decided,
 * counters[1]: its min delivered time).  On the library's own transports
 * with two ranks or more the payload goes out in two send/recv groups --
 * the owners below rank W/2 first, while the sender sorts the rest, then the
 * others while the first owners merge (shd_round_exchange_phases).
 * Synchronous. */
int shd_round_process_exchange(ShdTopology* top, const ShdTransport* xport, const ShdPkt* d_recs, size_t n,
                               uint64_t barrier, uint64_t end_time, uint64_t bootstrap_end, const uint32_t* host_bounds,
                               void* d_send, uint8_t* d_status, uint64_t* d_counters, void* d_recv, size_t recv_cap,
                               ShdDeliv* d_out, uint32_t* d_out_offsets, size_t* n_out, void* stream);
/* Row-sharded tables (C4 at N > 1, no full matrix anywhere): rank r holds
 * rows [row_bounds[r], row_bounds[r+1]) (slot ids, host memory).  Each
 * record is sent to the rank holding the row that answers it -- the row of
 * the endpoint touched first (use_shortest_path; records naming unattached
 * hosts go to rank 0, which reports them undelivered) -- preserving record
 * order per source rank (partitioned into d_scratch, n records, which is
 * what the transport sends); received records land in d_recv (recv_cap) in
 * source-rank order, *n_recv set.  The receiver then decides them with
 * shd_round_process_device on its shard and exchanges the events with
 * shd_round_exchange.  Synchronous. */
int shd_round_route_records(ShdTopology* top, const ShdTransport* xport, const ShdPkt* d_recs, size_t n,
                            const uint32_t* row_bounds, ShdPkt* d_scratch, ShdPkt* d_recv, size_t recv_cap,
                            size_t* n_recv, void* stream);
/* Multi-process jobs (one process per GPU): adopts rows [row_lo, row_hi) of
 * the table (d_rows: (row_hi - row_lo) * A entries) as this rank's
 * device-resident shard and releases every row in slot order (the
 * touch_all steady state of a long simulation); lookups and rounds on this
 * topology may then only use pairs whose answering row is in the shard
 * (-EXDEV otherwise).  global_min_ms: the released minimum over the whole
 * table (min over ranks of shd_topology_shard_min_latency), or < 0 to use
 * this shard's.  The lazy release of a single process is
 * shd_topology_adopt_table_shards. */
int shd_topology_adopt_table_shard_device_resident(ShdTopology* top, void* d_rows, int row_lo, int row_hi,
                                                   double global_min_ms);
/* Released minimum over this shard's rows (pairs i < j), -1 if none. */
int shd_topology_shard_min_latency(ShdTopology* top, const void* d_rows, int row_lo, int row_hi, double* min_ms);

/* RCCL transport (xGMI): rank 0 creates the id (128 bytes), every rank gets
 * it out of band and creates its transport on its device; free after use. */
int shd_transport_rccl_unique_id(void* id128);
int shd_transport_rccl_new(int rank, int world, const void* id128, int device, ShdTransport** out);
void shd_transport_rccl_free(ShdTransport* xport);
/* One process, several GPUs (Shadow's process model, core/manager.c:543-577),
 * as ranks that are threads: one topology and one thread per device.
 * rccl_new_all: ndev RCCL transports from ncclCommInitAll (out[k] drives
 * devices[k]); free each with shd_transport_rccl_free.  local_new: world
 * transports with no RCCL -- a collective is a thread barrier plus
 * device-to-device copies each receiver pulls from the senders' buffers
 * (peer access between GPUs; a plain copy on one GPU, e.g. to rehearse the
 * multi-rank rounds with threads on one device); free each with
 * shd_transport_local_free.  Every rank's thread must take part in every
 * collective, as with RCCL. */
int shd_transport_rccl_new_all(int ndev, const int* devices, ShdTransport** out);
int shd_transport_local_new(int world, ShdTransport** out);
void shd_transport_local_free(ShdTransport* xport);

/* ---------------------------------------------------------------------- */
/* Destination routers: router_enqueue + CoDel           */
/* ---------------------------------------------------------------------- */

/* One upstream-router queue (routing/router_queue_codel.c:56-78), with its
 * packets in a caller-provided ring of ShdCodelEntry (ring_cap per router). */
typedef struct ShdCodelState {
    uint64_t interval_expire; /* intervalExpireTS */
    uint64_t next_drop;       /* nextDropTS */
    uint64_t total_size;      /* bytes queued (payload + header) */
    uint32_t mode;            /* 0 store, 1 drop (CoDelMode) */
    uint32_t drop_count, drop_count_last;
    uint32_t head, len;       /* ring position of the oldest entry, entries queued */
    uint32_t pad;
} ShdCodelState;
typedef struct ShdCodelEntry {
    uint64_t enqueue_ts;
    uint32_t pkt, length;
} ShdCodelEntry;
/* One queue operation at simulated time `time`: kind 0 = router_enqueue of
 * packet `pkt` (router.c:103-121; `length` = payload + header bytes), kind 1
 * = router_dequeue (router.c:123-131, what networkinterface_receivePackets
 * calls, network_interface.c:448-478). */
typedef struct ShdCodelOp {
    uint64_t time;
    uint32_t kind, pkt, length, pad;
} ShdCodelOp;
enum { SHD_CODEL_QUEUED = 0, SHD_CODEL_DEQUEUED = 1, SHD_CODEL_DROPPED = 2 };
/* Runs every router's operations in order (device pointers): router r's ops
 * are ops[op_offsets[r] .. op_offsets[r+1]) in time order, its state
 * states[r], its ring rings[r * ring_cap ...].  deq_out[i] = the packet a
 * dequeue op returned (UINT32_MAX: none; enqueue ops get their packet id);
 * fate[pkt] = (op index << 2) | SHD_CODEL_DEQUEUED or SHD_CODEL_DROPPED for
 * every packet that left its queue (PDS_ROUTER_DEQUEUED / _DROPPED), entries
 * of packets still queued untouched.  Exactly the reference's CoDel,
 * control law included (router_queue_codel.c:113-265: target 10 ms, interval
 * 100 ms, MTU 1500, unbounded queue).  Synchronous; -ENOSPC if a ring would
 * overflow (that router's remaining ops are not run). */
int shd_codel_run(uint32_t nrouters, const uint32_t* d_op_offsets, const ShdCodelOp* d_ops, ShdCodelState* d_states,
                  ShdCodelEntry* d_rings, uint32_t ring_cap, uint32_t* d_deq_out, uint64_t* d_fate, void* stream);

/* ---- network interfaces: router + CoDel + token buckets ----------------- */
/* host/network_interface.c (buckets :33-41, 99-228; receivePackets :448-482;
 * sendPackets :571-631; wantsSend :633-661) with the upstream router
 * (routing/router.c:103-131, router_queue_codel.c).  One record per host;
 * refill grid and router state included.  128 bytes. */
typedef struct ShdNicState {
    uint64_t recv_remaining, recv_refill, recv_capacity; /* bytes; refill per 1 ms */
    uint64_t send_remaining, send_refill, send_capacity;
    uint64_t refill_start; /* timeStartedRefillingBuckets */
    uint64_t refill_time;  /* when the pending refill task runs */
    uint32_t refill_pending, pad0;
    uint64_t pad1;
    ShdCodelState router; /* head/len index the host's entry ring */
} ShdNicState;

/* A packet a host's sockets offer to its interface (qdisc order), offered
 * at `ready` (networkinterface_wantsSend); length = payload + header. */
typedef struct ShdNicSend {
    uint64_t ready;
    uint32_t id, length;
} ShdNicSend;

enum { SHD_NIC_QUEUED = 0, SHD_NIC_RECEIVED = 1, SHD_NIC_DROPPED = 2 };

/* _networkinterface_setupTokenBuckets + networkinterface_startRefillingTokenBuckets
 * at start_time for nhosts interfaces (bandwidths in KiB/s, device arrays). */
int shd_nic_init(uint32_t nhosts, const uint64_t* d_bw_down_kibps, const uint64_t* d_bw_up_kibps,
                 uint64_t start_time, ShdNicState* d_states, void* stream);

/* Per-event packet length = the record's payload_len + header_bytes (42 UDP,
 * 66 TCP: CONFIG_HEADER_SIZE_*, definitions.h:173-180). */
int shd_event_lengths(const ShdDeliv* d_events, size_t n, const ShdPkt* d_pkts, uint32_t header_bytes,
                      uint32_t* d_lengths, void* stream);

/* Runs hosts [host_base, host_base + nhosts) up to window_end (exclusive):
 * host h's arrivals are d_events[d_event_offsets[h] .. [h+1]) in
 * event_compare order (a round's per-destination segments, as produced),
 * all with time < window_end; its send requests d_sends[d_send_offsets[h] ..
 * [h+1]) (NULL offsets: none), in offer order.  Arrival k is packet id
 * id_base + k: d_recv_time / d_recv_status[id] (arrays of fate_cap entries,
 * also written for packets queued in earlier windows) get the receive time
 * and SHD_NIC_RECEIVED, or SHD_NIC_DROPPED (CoDel), or stay
 * SHD_NIC_QUEUED / ~0 (still in the router at window_end: the entry moves
 * to the host's ring of ring_cap entries and is carried).  d_send_time[k]
 * gets request k's send time (~0: not sent by window_end -- offer it again,
 * first, in the next window).  Synchronous.  -ENOSPC on a ring overflow,
 * -EINVAL on misaddressed, out-of-order or out-of-window inputs. */
int shd_nic_run(uint32_t nhosts, uint32_t host_base, const ShdDeliv* d_events, const uint32_t* d_event_offsets,
                const uint32_t* d_event_lengths, const ShdNicSend* d_sends, const uint32_t* d_send_offsets,
                uint64_t window_end, uint64_t bootstrap_end, ShdNicState* d_states, ShdCodelEntry* d_rings,
                uint32_t ring_cap, uint32_t id_base, uint64_t* d_recv_time, uint8_t* d_recv_status,
                uint64_t fate_cap, uint64_t* d_send_time, void* stream);


/* Copies between device and/or host memory (unified addressing), e.g. for a
 * transport that bounces device blocks through host memory. */
int shd_memcpy(void* dst, const void* src, size_t bytes);

/* Device timing of the round pipeline with HIP events recorded on the launch
 * stream (for benchmarks): stages 0 packet-scatter (decision + gathers +
 * per-destination count), 1 scan, 2 place, 3 segment sort.  enable resets
 * the record; read sums the elapsed ms per stage over recorded launches. */
int shd_round_timing_enable(int enable);
/* Pauses (paused != 0) or resumes the recording without resetting it: a
 * benchmark times only some rounds' stages (each event record holds the
 * stream's next kernel back a few microseconds). */
int shd_round_timing_pause(int paused);
/* The grouping pipeline a round of n records over nhosts destinations runs
 * (SHD_PACKET_PIPELINE or the default): 0 bucket, 1 rank, 2 slab, 3 part. */
int shd_round_pipeline_of(uint32_t nhosts, size_t n, int* pipe);
int shd_round_timing_read(double* stage_ms, int nstages, int* launches);
/* Phase times (ms, HIP events) of this thread's last shd_round_process_exchange
 * that sent in two groups (the split exchange: the library's own transports,
 * two ranks or more, SHD_XCHG_SPLIT != 0): [0] decide (the sender's
 * kernels), [1] counts (the count-matrix all-gather), [2] group 1 (owners
 * [0, W/2)), [3] group 2, [4] owner merge, [5] the whole call, [6] the
 * transfer time that ran beside the sender's kernels, [7] the merge's time
 * beside group 2.  *valid = 0 when the last call did not complete a split
 * exchange. */
int shd_round_exchange_phases(double* ms, int n, int* valid);

/* Unit strings as the GML loader reads them (replace parse_time_nanosec /
 * parse_bandwidth, bindings.h:279,282, core/support/units.rs:777-837):
 * "<u64>[ ]<unit>", unit default seconds / bits.  -EINVAL on a malformed
 * string (e.g. "10.5 ms", units.rs:632). */
int shd_parse_time_ns(const char* s, uint64_t* ns);
int shd_parse_bandwidth_bits(const char* s, uint64_t* bits_per_s);

/* Synthetic load for simulated rounds (benchmarks and tests: it stands in
 * for the hosts' applications; not part of the hand-off).  Every sender
 * d_pool[k] (k < npool) sends m packets into d_recs (npool * m records,
 * sender-major): packet j reserves the sender's j-th rand_r draw of the round
 * (worker.c:540-541; the record carries that draw's pre-state), goes to
 * d_dst_pool[x % ndst] (or host x % ndst when d_dst_pool is NULL; the next
 * one if that is the sender) at a time in the j-th of m slices of [t0, t0 +
 * window_ns), x a splitmix64 hash of (seed, round, k, j).  The senders'
 * rand_r states and event counters are carried: d_state_in / d_seq_in (per
 * pool position) -> d_state_out / d_seq_out after the round.  Device
 * pointers; stream: hipStream_t or NULL. */
int shd_synth_sends_device(const uint32_t* d_pool, uint32_t npool, uint32_t m, uint32_t round, uint64_t seed,
                           uint64_t t0, uint64_t window_ns, const uint32_t* d_dst_pool, uint32_t ndst,
                           const uint32_t* d_state_in, uint32_t* d_state_out, const uint64_t* d_seq_in,
                           uint64_t* d_seq_out, ShdPkt* d_recs, void* stream);

/* Last error message for this thread (static storage). */
const char* shd_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
