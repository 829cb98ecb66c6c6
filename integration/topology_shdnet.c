/*
 * routing/topology_shdnet.c -- replaces routing/topology.c in a Shadow tree
 * (INTEGRATION.md §2): the reference's routing API (routing/topology.h:17-28)
 * forwarded to libshdnet (include/shdnet.h).  Same header, same signatures,
 * same return conventions; igraph is no longer linked.
 *
 * Compiled against the reference headers by tests/test_integration_cpu.py
 * (gcc -fsyntax-only), so a drift of topology.h or shdnet.h fails there.
 */
#include <errno.h>
#include <glib.h>

#include "lib/logger/logger.h"
#include "main/core/worker.h"
#include "main/routing/address.h"
#include "main/routing/topology.h"
#include "main/utility/random.h"
#include "main/utility/utility.h"
#include "shdnet.h"
#include "shdnet_shadow_helpers.h"

struct _Topology {
    ShdTopology* t;
};

ShdTopology* topology_shdnetHandle(Topology* top) { return top->t; }

/* the running minimum of released path latencies (topology.c:1253-1264) */
static void _topology_minJump(double minMs, void* user) {
    (void)user;
    worker_updateMinTimeJump(minMs); /* worker.h:89 */
}

/* topology.c:2328-2354 */
Topology* topology_new(const gchar* graphPath, gboolean useShortestPath) {
    Topology* top = g_new0(Topology, 1);
    if (shd_topology_new(graphPath, useShortestPath ? 1 : 0, /*device*/ 0, &top->t) != 0) {
        error("we failed to create the simulation topology: %s", shd_last_error());
        g_free(top);
        return NULL;
    }
    shd_topology_set_min_jump_callback(top->t, _topology_minJump, NULL);
    return top;
}

static void _topology_logPath(const char* line, void* user) {
    (void)user;
    debug("%s", line);
}

/* topology.c:2283-2326, including the cached-path log of :2287 */
void topology_free(Topology* top) {
    if (!top) return;
    shd_topology_log_cached_paths(top->t, _topology_logPath, NULL, NULL);
    shd_topology_free(top->t);
    g_free(top);
}

/* topology.c:2218-2272: the attach draw comes from the host's own stream */
void topology_attach(Topology* top, Address* address, Random* randomSourcePool, gchar* ipHint, gchar* citycodeHint,
                     gchar* countrycodeHint, guint64* bwDownOut, guint64* bwUpOut) {
    uint64_t down = 0, up = 0;
    const guint32 host = shadow_host_index_of((GQuark)address_getID(address));
    const int rc = shd_topology_attach(top->t, host, address_toNetworkIP(address), random_seedStatePtr(randomSourcePool),
                                       ipHint, citycodeHint, countrycodeHint, &down, &up);
    if (rc != 0) utility_panic("unable to attach host %u: %s", host, shd_last_error());
    if (bwDownOut) *bwDownOut = down;
    if (bwUpOut) *bwUpOut = up;
}

/* topology.c:2274-2281 */
void topology_detach(Topology* top, Address* address) { shd_topology_detach(top->t, address_toNetworkIP(address)); }

/* topology.c:2019-2022 */
gboolean topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress) {
    int routable = 0;
    const int rc =
        shd_topology_is_routable(top->t, address_toNetworkIP(srcAddress), address_toNetworkIP(dstAddress), &routable);
    return rc == 0 && routable ? TRUE : FALSE;
}

/* topology.c:1995-2005: -1 for an unattached address; an attached pair with
 * no path panics (:1970-1976) */
gdouble topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress) {
    double ms = -1.0;
    const int rc = shd_topology_get_latency(top->t, address_toNetworkIP(srcAddress), address_toNetworkIP(dstAddress), &ms);
    if (rc == -ENOENT) return -1;
    if (rc != 0) utility_panic("unable to find path: %s", shd_last_error());
    return ms;
}

/* topology.c:2007-2017 */
gdouble topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress) {
    double rel = -1.0;
    const int rc =
        shd_topology_get_reliability(top->t, address_toNetworkIP(srcAddress), address_toNetworkIP(dstAddress), &rel);
    if (rc == -ENOENT) return -1;
    if (rc != 0) utility_panic("unable to find path: %s", shd_last_error());
    return rel;
}

/* topology.c:1983-1993 */
void topology_incrementPathPacketCounter(Topology* top, Address* srcAddress, Address* dstAddress) {
    const int rc = shd_topology_increment_path_packet_counter(top->t, address_toNetworkIP(srcAddress),
                                                              address_toNetworkIP(dstAddress));
    if (rc != 0) utility_panic("unable to find path: %s", shd_last_error());
}
