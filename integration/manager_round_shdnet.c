/*
 * core/manager.c:552-574 -- the round boundary of manager_run with the
 * libshdnet hand-off.  manager_run calls
 *
 *     shd_round_begin(top, windowEnd, endTime, bootstrapEndTime);   before the workers start the round
 *     ... scheduler_continueNextRound / scheduler_awaitNextRound ...
 *     minNextEventTime = shdnet_manager_finishRound(scheduler, top, windowEnd, minNextEventTime);
 *     keepRunning = controller_managerFinishedCurrentRound(controller, minNextEventTime, ...);
 *
 * on the scheduler thread, with the workers idle.  Compiled against the
 * reference headers by tests/test_integration_cpu.py.
 */
#include "main/core/worker.h" /* first, as core/worker.c has it (the core headers include each other) */

#include <glib.h>

#include "main/core/scheduler/scheduler.h"
#include "main/core/support/definitions.h"
#include "main/core/work/event.h"
#include "main/core/work/task.h"
#include "main/routing/packet.h"
#include "main/utility/utility.h"
#include "shdnet.h"
#include "shdnet_shadow_helpers.h"

/* Decides the round's staged sends on the GPU, applies the sender-side
 * statuses (worker.c:561, 574), pushes every delivered event into its
 * destination's queue in event_compare order and returns the next round's
 * minimum event time with the GPU's minimum folded in (what the senders'
 * worker_setMinEventTimeNextRound calls contributed, worker.c:350-363). */
SimulationTime shdnet_manager_finishRound(Scheduler* scheduler, ShdTopology* top, SimulationTime windowEnd,
                                          SimulationTime minNextEventTime) {
    uint32_t nhosts = 0;
    size_t nrec = 0, ndeliv = 0;
    uint64_t gpuMin = UINT64_MAX;
    if (shd_topology_host_count(top, &nhosts) != 0 || shd_round_staged(top, &nrec) != 0)
        utility_panic("shdnet: %s", shd_last_error());
    ShdDeliv* evs = g_new(ShdDeliv, nrec ? nrec : 1);
    uint32_t* dstOffsets = g_new(uint32_t, (gsize)nhosts + 1);
    uint8_t* status = g_new(uint8_t, nrec ? nrec : 1);
    if (shd_round_collect(top, evs, nrec, &ndeliv, dstOffsets, status, &gpuMin) != 0)
        utility_panic("shdnet round: %s", shd_last_error());
    utility_assert(worker_roundPacketsCount() == nrec);

    /* sender-side statuses; the copy of a dropped packet is released, the
     * copies of kept ones go to their deliver tasks below */
    for (guint64 i = 0; i < nrec; i++) {
        Packet *original = NULL, *copy = NULL;
        worker_roundPacketsGet(i, &original, &copy);
        if (status[i] == SHD_DROPPED_LOSS) {
            packet_addDeliveryStatus(original, PDS_INET_DROPPED);
            packet_unref(copy);
        } else {
            packet_addDeliveryStatus(original, PDS_INET_SENT);
            packet_addDeliveryStatus(copy, PDS_INET_SENT);
            if (status[i] == SHD_DROPPED_END) packet_unref(copy); /* scheduler_push's end-time drop (:236) */
        }
        packet_unref(original);
    }

    /* per destination, already in event_compare order (a total order:
     * inserting the sorted segment equals pushing each event at send time) */
    for (uint32_t h = 0; h < nhosts; h++) {
        Host* dst = scheduler_getHostByIndex(scheduler, h);
        for (uint32_t k = dstOffsets[h]; k < dstOffsets[h + 1]; k++) {
            Packet *original = NULL, *copy = NULL;
            worker_roundPacketsGet(evs[k].pkt_index, &original, &copy);
            Host* src = scheduler_getHostByIndex(scheduler, evs[k].src_host);
            Task* task = worker_newDeliverPacketTask(copy);
            Event* ev = event_newWithID(task, evs[k].time, src, dst, evs[k].seq);
            task_unref(task);
            scheduler_pushDecided(scheduler, ev, src, dst, windowEnd);
        }
    }
    worker_roundPacketsClear();
    g_free(evs);
    g_free(dstOffsets);
    g_free(status);
    return gpuMin < minNextEventTime ? gpuMin : minNextEventTime;
}
