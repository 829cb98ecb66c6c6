/*
 * ref_driver.c -- drives the REFERENCE's own utility/random.c and
 * utility/priority_queue.c (compiled from /root/reference by
 * oracle/Makefile into oracle/_ref/ref_driver) to emit golden vectors.
 * TEST INFRASTRUCTURE ONLY; run by oracle/gen_golden.py in the build
 * container.  The reference sources are compiled where they lie; nothing
 * is copied.  Output: one JSON object on stdout.
 */
#include <glib.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "main/utility/priority_queue.h"
#include "main/utility/random.h"

/* Event keys as event_compare orders them (core/work/event.c:109-152); the
 * driver supplies the comparator, the reference supplies the heap. */
typedef struct {
    uint64_t time;
    uint32_t dst, src;
    uint64_t seq;
    uint32_t index;
} Ev;

static gint ev_compare(gconstpointer pa, gconstpointer pb, gpointer unused) {
    const Ev* a = pa;
    const Ev* b = pb;
    (void)unused;
    if (a->time > b->time) return 1;
    if (a->time < b->time) return -1;
    if (a->dst > b->dst) return 1;
    if (a->dst < b->dst) return -1;
    if (a->src > b->src) return 1;
    if (a->src < b->src) return -1;
    if (a->seq > b->seq) return 1;
    if (a->seq < b->seq) return -1;
    return 0;
}

static uint64_t sm_state;
static uint64_t splitmix64(void) {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void emit_stream(guint seed, int n, int first) {
    Random* r = random_new(seed);
    printf("%s{\"seed\":%u,\"double\":[", first ? "" : ",", seed);
    for (int i = 0; i < n; i++) printf("%s%.17g", i ? "," : "", random_nextDouble(r));
    random_free(r);
    r = random_new(seed);
    printf("],\"uint\":[");
    for (int i = 0; i < n; i++) printf("%s%u", i ? "," : "", random_nextUInt(r));
    random_free(r);
    r = random_new(seed);
    printf("],\"rand\":[");
    for (int i = 0; i < n; i++) printf("%s%d", i ? "," : "", random_rand(r));
    random_free(r);
    printf("]}");
}

/* controller -> manager -> scheduler -> per-host seed chain
 * (controller.c:91,353; manager.c:178,199,344; host.c:164) */
static void emit_chain(guint seed, int nhosts, int first) {
    Random* c = random_new(seed);
    guint managerSeed = random_nextUInt(c);
    Random* m = random_new(managerSeed);
    guint schedulerSeed = random_nextUInt(m);
    printf("%s{\"seed\":%u,\"manager\":%u,\"scheduler\":%u,\"hosts\":[", first ? "" : ",", seed, managerSeed,
           schedulerSeed);
    for (int h = 0; h < nhosts; h++) printf("%s%u", h ? "," : "", random_nextUInt(m));
    printf("]}");
    random_free(c);
    random_free(m);
}

static void emit_pq(int n, uint64_t seed, int tmod, int hmod, int first) {
    sm_state = seed;
    Ev* evs = malloc(sizeof(Ev) * (size_t)n);
    for (int i = 0; i < n; i++) {
        evs[i].time = splitmix64() % (uint64_t)tmod;
        evs[i].dst = (uint32_t)(splitmix64() % (uint64_t)hmod);
        evs[i].src = (uint32_t)(splitmix64() % (uint64_t)hmod);
        evs[i].seq = splitmix64() % 1000000ull;
        evs[i].index = (uint32_t)i;
    }
    /* make (src, seq) unique as srcHostEventID guarantees */
    for (int i = 0; i < n; i++) evs[i].seq = evs[i].seq * (uint64_t)n + (uint64_t)i;
    PriorityQueue* q = priorityqueue_new(ev_compare, NULL, NULL);
    for (int i = 0; i < n; i++) priorityqueue_push(q, &evs[i]);
    printf("%s{\"n\":%d,\"keys\":[", first ? "" : ",", n);
    for (int i = 0; i < n; i++)
        printf("%s[%llu,%u,%u,%llu]", i ? "," : "", (unsigned long long)evs[i].time, evs[i].dst, evs[i].src,
               (unsigned long long)evs[i].seq);
    printf("],\"order\":[");
    for (int i = 0; i < n; i++) {
        Ev* e = priorityqueue_pop(q);
        printf("%s%u", i ? "," : "", e->index);
    }
    printf("]}");
    priorityqueue_free(q);
    free(evs);
}

int main(void) {
    printf("{\"streams\":[");
    guint seeds[] = {1u, 0u, 2u, 12345u, 0x7fffffffu, 0xffffffffu, 3735928559u};
    for (int i = 0; i < (int)(sizeof seeds / sizeof seeds[0]); i++) emit_stream(seeds[i], 64, i == 0);
    printf("],\"chains\":[");
    emit_chain(1u, 16, 1);
    emit_chain(42u, 16, 0);
    emit_chain(123456789u, 8, 0);
    printf("],\"pq\":[");
    emit_pq(50, 1, 5, 3, 1);
    emit_pq(300, 2, 20, 10, 0);
    emit_pq(1000, 3, 1000000, 100, 0);
    emit_pq(257, 4, 2, 2, 0);
    printf("]}\n");
    return 0;
}
