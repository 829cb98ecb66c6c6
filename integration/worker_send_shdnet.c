/*
 * core/worker.c:517-576 -- worker_sendPacket with the libshdnet hand-off
 * (INTEGRATION.md §3).  Replaces the function's body in worker.c; kept here
 * as its own translation unit (with the worker.c internals it needs behind
 * the helpers of shdnet_shadow_helpers.h) so that it compiles against the
 * reference headers (tests/test_integration_cpu.py).
 *
 * What stays at send time, on the sending worker: address resolution, the
 * null-address panic, the topology_getReliability lookup's side effects (row
 * touch, cache direction, min-jump -- inside shd_round_append_worker, in send
 * order), the reserved random draw, the srcHostEventID, and the packet copy.
 * What moves to the round boundary (manager_round_shdnet.c): the drop
 * decision, the delivery time, the end-time drop, the barrier clamp and the
 * queue insertion.
 */
#include <glib.h>
#include <netinet/in.h>

#include "main/core/worker.h"
#include "main/host/host.h"
#include "main/routing/address.h"
#include "main/routing/packet.h"
#include "main/utility/random.h"
#include "main/utility/utility.h"
#include "shdnet.h"
#include "shdnet_shadow_helpers.h"

void worker_sendPacket(Host* srcHost, Packet* packet) {
    utility_assert(packet != NULL);
    if (!worker_schedulerIsRunning()) return; /* the simulation is over (worker.c:520-523) */

    Address* srcAddress = worker_resolveIPToAddress(packet_getSourceIP(packet));
    Address* dstAddress = worker_resolveIPToAddress(packet_getDestinationIP(packet));
    if (!srcAddress || !dstAddress) {
        utility_panic("unable to schedule packet because of null addresses");
        return;
    }

    Random* random = host_getRandom(srcHost);
    ShdPkt rec = {
        .now = worker_getCurrentTime(),
        .seq = host_getNewEventID(srcHost), /* srcHostEventID (host.c:368-371) */
        .src_host = shadow_host_index_of((GQuark)address_getID(srcAddress)),
        .dst_host = shadow_host_index_of((GQuark)address_getID(dstAddress)),
        .rng_state = random_peekState(random), /* pre-state of the reserved draw */
        .payload_len = packet_getPayloadLength(packet),
    };
    (void)random_nextDouble(random); /* the draw is consumed now, as at worker.c:540 */

    const int w = worker_threadIndex();
    const int rc = shd_round_append_worker(topology_shdnetHandle(worker_getTopology()), w, &rec, 1);
    if (rc != 0) utility_panic("unable to schedule packet: %s", shd_last_error());
    /* the copy the deliver task will own is taken now, as at worker.c:565;
     * the sender keeps modifying its own packet afterwards */
    packet_ref(packet);
    worker_roundPacketsPush(w, packet, packet_copy(packet));
}
