/* dns.c -- address assignment for the simulated hosts (SURVEY.md §8f-3;
 * reference routing/dns.c:22-163, 175-296).
 *
 * Host C: registration is startup work (one call per host, 200k hosts at
 * C4) and its cost in the reference is the glib hash tables plus sixteen
 * CIDR parses per candidate address (_dns_isRestricted, :89-106).  Here
 * the reserved ranges are precomputed (value, mask) pairs in host order, the
 * two maps are open-addressing tables keyed by the network-order address
 * and by a 64-bit FNV-1a hash of the name, and a batch entry point takes all
 * hosts under one lock acquisition. */
#include <arpa/inet.h>
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "shd_internal.h"

typedef struct {
    uint32_t ip_net, mac;
    char* name;
} DnsAddr;

typedef struct {
    uint64_t key; /* ip_net, or the name hash */
    int32_t idx;  /* -1 empty, -2 tombstone, else entry index */
} DnsSlot;

typedef struct {
    DnsSlot* s;
    uint32_t cap, n, tomb;
} DnsMap;

struct ShdDns {
    pthread_mutex_t mu; /* the reference's dns->lock */
    uint32_t ip_counter; /* host order (ipAddressCounter) */
    uint32_t mac_counter;
    DnsAddr* addr;
    uint32_t naddr, capaddr;
    DnsMap by_ip, by_name;
};

/* _dns_isRestricted (:89-106): reserved IPv4 blocks as (subnet, mask) in host order */
static const struct {
    uint32_t net, bits;
} kReserved[] = {
    {0x00000000u, 8},  {0x0A000000u, 8},  {0x64400000u, 10}, {0x7F000000u, 8},  {0xA9FE0000u, 16}, {0xAC100000u, 12},
    {0xC0000000u, 29}, {0xC0000200u, 24}, {0xC0586300u, 24}, {0xC0A80000u, 16}, {0xC6120000u, 15}, {0xC6336400u, 24},
    {0xCB007100u, 24}, {0xE0000000u, 4},  {0xF0000000u, 4},  {0xFFFFFFFFu, 32},
};

static int restricted(uint32_t ip_net) {
    const uint32_t h = ntohl(ip_net);
    for (size_t i = 0; i < sizeof kReserved / sizeof kReserved[0]; i++) {
        const uint32_t mask = kReserved[i].bits ? ~0u << (32 - kReserved[i].bits) : 0u;
        if ((h & mask) == (kReserved[i].net & mask)) return 1;
    }
    return 0;
}

static uint64_t name_hash(const char* s) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (; *s; s++) h = (h ^ (unsigned char)*s) * 0x100000001b3ull;
    return h;
}

static uint32_t slot_of(uint64_t key, uint32_t cap) { /* splitmix64 finaliser */
    key ^= key >> 30;
    key *= 0xbf58476d1ce4e5b9ull;
    key ^= key >> 27;
    key *= 0x94d049bb133111ebull;
    key ^= key >> 31;
    return (uint32_t)key & (cap - 1);
}

static int map_grow_to(DnsMap* m, uint32_t want) {
    uint32_t ncap = m->cap ? m->cap * 2 : 1024;
    while ((uint64_t)(want + 1) * 2 > ncap) ncap *= 2;
    DnsSlot* ns = (DnsSlot*)malloc(sizeof(DnsSlot) * ncap);
    if (!ns) return -ENOMEM;
    for (uint32_t i = 0; i < ncap; i++) ns[i].idx = -1;
    for (uint32_t i = 0; i < m->cap; i++)
        if (m->s[i].idx >= 0) {
            uint32_t h = slot_of(m->s[i].key, ncap);
            while (ns[h].idx != -1) h = (h + 1) & (ncap - 1);
            ns[h] = m->s[i];
        }
    free(m->s);
    m->s = ns;
    m->cap = ncap;
    m->tomb = 0;
    return 0;
}

static int map_grow(DnsMap* m) { return map_grow_to(m, m->n); }

/* the slot holding an entry accepted by `match`, or NULL */
typedef int (*MatchFn)(const struct ShdDns* d, int32_t idx, const void* want);

static DnsSlot* map_find(const struct ShdDns* d, const DnsMap* m, uint64_t key, MatchFn match, const void* want) {
    if (!m->cap) return NULL;
    for (uint32_t h = slot_of(key, m->cap);; h = (h + 1) & (m->cap - 1)) {
        DnsSlot* s = &m->s[h];
        if (s->idx == -1) return NULL;
        if (s->idx >= 0 && s->key == key && match(d, s->idx, want)) return s;
    }
}

static int match_any(const struct ShdDns* d, int32_t idx, const void* want) { return 1; }
static int match_name(const struct ShdDns* d, int32_t idx, const void* want) {
    return strcmp(d->addr[idx].name, (const char*)want) == 0;
}

/* g_hash_table_replace */
static int map_replace(struct ShdDns* d, DnsMap* m, uint64_t key, int32_t idx, MatchFn match, const void* want) {
    DnsSlot* s = map_find(d, m, key, match, want);
    if (s) {
        s->idx = idx;
        return 0;
    }
    if ((uint64_t)(m->n + m->tomb + 1) * 2 > m->cap) {
        int rc = map_grow(m);
        if (rc) return rc;
    }
    uint32_t h = slot_of(key, m->cap);
    while (m->s[h].idx >= 0) h = (h + 1) & (m->cap - 1);
    if (m->s[h].idx == -2) m->tomb--;
    m->s[h].key = key;
    m->s[h].idx = idx;
    m->n++;
    return 0;
}

static void map_remove(struct ShdDns* d, DnsMap* m, uint64_t key, MatchFn match, const void* want) {
    DnsSlot* s = map_find(d, m, key, match, want);
    if (s) {
        s->idx = -2;
        m->n--;
        m->tomb++;
    }
}

int shd_dns_new(ShdDns** out) {
    if (!out) return -EINVAL;
    ShdDns* d = (ShdDns*)calloc(1, sizeof *d);
    if (!d) return -ENOMEM;
    pthread_mutex_init(&d->mu, NULL);
    d->ip_counter = 0x0B000000u; /* "11.0.0.0" (dns_new, :294-305) */
    *out = d;
    return 0;
}

void shd_dns_free(ShdDns* d) {
    if (!d) return;
    for (uint32_t i = 0; i < d->naddr; i++) free(d->addr[i].name);
    free(d->addr);
    free(d->by_ip.s);
    free(d->by_name.s);
    pthread_mutex_destroy(&d->mu);
    free(d);
}

/* address_stringToIP (address.c:145-152): inet_pton, INADDR_NONE otherwise */
static uint32_t string_to_ip(const char* s) {
    struct in_addr a;
    return inet_pton(AF_INET, s, &a) == 1 ? a.s_addr : 0xFFFFFFFFu;
}

/* _dns_generateIP (:113-123) */
static uint32_t generate_ip(ShdDns* d) {
    uint32_t ip = htonl(++d->ip_counter);
    while (restricted(ip) || map_find(d, &d->by_ip, ip, match_any, NULL)) ip = htonl(++d->ip_counter);
    return ip;
}

/* dns_register (:125-163) without the lock */
static int register_locked(ShdDns* d, const char* name, const char* requested, uint32_t* ip_out, uint32_t* mac_out,
                           int* local_out) {
    uint32_t ip;
    const uint32_t mac = ++d->mac_counter;
    int local = 0;
    if (requested) {
        ip = string_to_ip(requested);
        if (ip == htonl(0x7F000001u)) local = 1;
        else if (restricted(ip) || map_find(d, &d->by_ip, ip, match_any, NULL)) ip = generate_ip(d);
    } else {
        ip = generate_ip(d);
    }
    if (!local) {
        if (d->naddr == d->capaddr) {
            uint32_t ncap = d->capaddr ? d->capaddr * 2 : 1024;
            DnsAddr* na = (DnsAddr*)realloc(d->addr, sizeof(DnsAddr) * ncap);
            if (!na) return -ENOMEM;
            d->addr = na;
            d->capaddr = ncap;
        }
        char* nm = strdup(name);
        if (!nm) return -ENOMEM;
        const int32_t idx = (int32_t)d->naddr++;
        d->addr[idx] = (DnsAddr){ip, mac, nm};
        int rc = map_replace(d, &d->by_ip, ip, idx, match_any, NULL);
        if (!rc) rc = map_replace(d, &d->by_name, name_hash(name), idx, match_name, name);
        if (rc) return rc;
    }
    if (ip_out) *ip_out = ip;
    if (mac_out) *mac_out = mac;
    if (local_out) *local_out = local;
    return 0;
}

int shd_dns_register(ShdDns* d, const char* name, const char* requested_ip, uint32_t* ip_net, uint32_t* mac,
                     int* is_local) {
    if (!d || !name) return -EINVAL;
    pthread_mutex_lock(&d->mu);
    int rc = register_locked(d, name, requested_ip, ip_net, mac, is_local);
    pthread_mutex_unlock(&d->mu);
    return rc;
}

int shd_dns_register_batch(ShdDns* d, uint32_t n, const char* const* names, const char* const* requested_ips,
                           uint32_t* ip_net, uint32_t* mac, uint8_t* is_local) {
    if (!d || (n && !names)) return -EINVAL;
    for (uint32_t i = 0; i < n; i++)
        if (!names[i]) return shd_fail(-EINVAL, "name %u is NULL", i);
    pthread_mutex_lock(&d->mu);
    int rc = 0;
    /* size the maps and the address array for the whole batch up front */
    const uint64_t want = (uint64_t)d->naddr + n;
    if (want > UINT32_MAX / 4) rc = shd_fail(-ENOMEM, "too many addresses");
    if (!rc && (uint64_t)(d->by_ip.n + d->by_ip.tomb + n) * 2 > d->by_ip.cap) rc = map_grow_to(&d->by_ip, d->by_ip.n + n);
    if (!rc && (uint64_t)(d->by_name.n + d->by_name.tomb + n) * 2 > d->by_name.cap)
        rc = map_grow_to(&d->by_name, d->by_name.n + n);
    if (!rc && want > d->capaddr) {
        DnsAddr* na = (DnsAddr*)realloc(d->addr, sizeof(DnsAddr) * want);
        if (!na) rc = -ENOMEM;
        else d->addr = na, d->capaddr = (uint32_t)want;
    }
    for (uint32_t i = 0; i < n && !rc; i++) {
        int local = 0;
        rc = register_locked(d, names[i], requested_ips ? requested_ips[i] : NULL, ip_net ? &ip_net[i] : NULL,
                             mac ? &mac[i] : NULL, &local);
        if (is_local) is_local[i] = (uint8_t)local;
    }
    pthread_mutex_unlock(&d->mu);
    return rc;
}

/* dns_deregister (:165-181): drops the IP's mapping and the name's mapping
 * (whichever address the name maps to now, as g_hash_table_remove does). */
int shd_dns_deregister(ShdDns* d, uint32_t ip_net, const char* name, int is_local) {
    if (!d || !name) return -EINVAL;
    if (is_local) return 0;
    pthread_mutex_lock(&d->mu);
    map_remove(d, &d->by_ip, ip_net, match_any, NULL);
    map_remove(d, &d->by_name, name_hash(name), match_name, name);
    pthread_mutex_unlock(&d->mu);
    return 0;
}

/* dns_resolveIPToAddress (:183-193) */
int shd_dns_resolve_ip(ShdDns* d, uint32_t ip_net, char* name, size_t cap, uint32_t* mac) {
    if (!d) return -EINVAL;
    pthread_mutex_lock(&d->mu);
    DnsSlot* s = map_find(d, &d->by_ip, ip_net, match_any, NULL);
    int rc = 0;
    if (!s) rc = -ENOENT;
    else {
        const DnsAddr* a = &d->addr[s->idx];
        if (name && cap) snprintf(name, cap, "%s", a->name);
        if (mac) *mac = a->mac;
    }
    pthread_mutex_unlock(&d->mu);
    return rc;
}

/* dns_resolveNameToAddress (:195-203) */
int shd_dns_resolve_name(ShdDns* d, const char* name, uint32_t* ip_net, uint32_t* mac) {
    if (!d || !name) return -EINVAL;
    pthread_mutex_lock(&d->mu);
    DnsSlot* s = map_find(d, &d->by_name, name_hash(name), match_name, name);
    int rc = 0;
    if (!s) rc = -ENOENT;
    else {
        if (ip_net) *ip_net = d->addr[s->idx].ip_net;
        if (mac) *mac = d->addr[s->idx].mac;
    }
    pthread_mutex_unlock(&d->mu);
    return rc;
}

/* _dns_writeNewHostsFile's content (:231-265): "127.0.0.1 localhost" then
 * "<ip> <name>" for every name mapping, in registration order (the
 * reference walks its name table in glib hash order).  Writes at most cap
 * bytes including the NUL; *len = the full length. */
int shd_dns_hosts_file(ShdDns* d, char* buf, size_t cap, size_t* len) {
    if (!d || !len) return -EINVAL;
    pthread_mutex_lock(&d->mu);
    size_t used = 0;
    for (int64_t i = -1; i < (int64_t)d->naddr; i++) {
        char ip[INET_ADDRSTRLEN] = "127.0.0.1";
        const char* nm = "localhost";
        if (i >= 0) {
            const DnsAddr* a = &d->addr[i];
            DnsSlot* s = map_find(d, &d->by_name, name_hash(a->name), match_name, a->name);
            if (!s || s->idx != (int32_t)i) continue; /* replaced or removed */
            struct in_addr in = {a->ip_net};
            inet_ntop(AF_INET, &in, ip, sizeof ip);
            nm = a->name;
        }
        const size_t room = buf && used < cap ? cap - used : 0;
        used += (size_t)snprintf(room ? buf + used : NULL, room, "%s %s\n", ip, nm);
    }
    pthread_mutex_unlock(&d->mu);
    *len = used;
    return 0;
}
