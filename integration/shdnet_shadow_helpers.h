/*
 * shdnet_shadow_helpers.h -- the small helpers a Shadow tree needs beside
 * the libshdnet wrappers of this directory.  Each is a
 * one- or two-line addition to the named reference file; none changes an
 * existing signature.  Declared here so that the wrappers compile against an
 * unmodified Shadow tree (tests/test_integration_cpu.py).
 */
#ifndef SHDNET_SHADOW_HELPERS_H
#define SHDNET_SHADOW_HELPERS_H

#include <glib.h>

#include "main/core/scheduler/scheduler.h"
#include "main/core/support/definitions.h"
#include "main/core/work/event.h"
#include "main/core/work/task.h"
#include "main/host/host.h"
#include "main/routing/packet.h"
#include "main/routing/topology.h"
#include "main/utility/random.h"
#include "shdnet.h"

/* utility/random.c: &random->seedState (random.c:15-18), the state the
 * attach draw of topology_attach consumes in place. */
guint32* random_seedStatePtr(Random* random);
/* utility/random.c: the seedState before the next draw, without drawing
 * (the reserved draw of worker_sendPacket, worker.c:540). */
guint32 random_peekState(Random* random);

/* core/manager.c: the dense registration index of a host (the order
 * manager_addNewVirtualHost registers them, manager.c:339-350, = GQuark
 * order); libshdnet's host ids. */
guint32 shadow_host_index_of(GQuark hostID);
/* core/scheduler/scheduler.c: the host with that dense index. */
Host* scheduler_getHostByIndex(Scheduler* scheduler, guint32 index);

/* core/work/event.c: event_new_ (event.c:27-42) with the srcHostEventID the
 * sender reserved at send time instead of a fresh host_getNewEventID. */
Event* event_newWithID(Task* task, SimulationTime time, gpointer srcHost, gpointer dstHost, guint64 srcHostEventID);

/* core/scheduler/scheduler.c: the policy push of an already decided event
 * from the scheduler thread (time already clamped to >= the barrier and
 * below the end time; scheduler_push's worker_setMinEventTimeNextRound call
 * needs a worker thread, the round's minimum is folded by the caller). */
void scheduler_pushDecided(Scheduler* scheduler, Event* event, Host* sender, Host* receiver, SimulationTime barrier);

/* core/worker.c: the calling worker's index in the pool (0..n-1), whether
 * the manager's scheduler is still running, and the per-worker list of the
 * round's sent packets (original, copy taken at send time), in append order. */
int worker_threadIndex(void);
gboolean worker_schedulerIsRunning(void);
void worker_roundPacketsPush(int worker, Packet* original, Packet* copy);
/* the i-th record of the round (worker-order concatenation) */
void worker_roundPacketsGet(guint64 i, Packet** original, Packet** copy);
guint64 worker_roundPacketsCount(void);
void worker_roundPacketsClear(void);
/* core/worker.c: the deliver task _worker_runDeliverPacketTask (worker.c:
 * 509-515) for a packet copy (the task takes the copy's reference). */
Task* worker_newDeliverPacketTask(Packet* packetCopy);

/* routing/topology_shdnet.c: the libshdnet topology behind Shadow's. */
ShdTopology* topology_shdnetHandle(Topology* top);

#endif
