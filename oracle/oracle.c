/*
 * oracle.c -- CPU restatement of Shadow's network plane (routing table +
 * per-round packet hand-off).  TEST INFRASTRUCTURE ONLY: the product in
 * shadow_amd/ never links or calls this file.  See oracle.h for the pinning
 * of each part.  Citations are file:line into /root/reference/src/main.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; no fast-math so every
 * fp64 operation is the one the reference performs).
 */
#include "oracle.h"

#include <arpa/inet.h>
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* units: core/support/units.rs                                            */
/* ======================================================================= */

/* Rust str::trim / regex \s on the ASCII subset. */
static int orc_isspace(int c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

/* Splits "<value> <unit>" per the regex ^([+-]?[0-9\.]*)\s*(.*)$ of
 * units.rs:420 and trims both parts (units.rs:422-425).  Returns 0 on match. */
static int split_value_unit(const char* s, char* val, size_t vcap, char* unit, size_t ucap) {
    const char* p = s;
    const char* v0 = p;
    if (*p == '+' || *p == '-') p++;
    while ((*p >= '0' && *p <= '9') || *p == '.') p++;
    const char* v1 = p;
    while (orc_isspace((unsigned char)*p)) p++;
    const char* u0 = p;
    /* (.*)$ : '.' does not match '\n', so the rest must be newline-free */
    for (const char* q = u0; *q; q++)
        if (*q == '\n') return -1;
    const char* u1 = u0 + strlen(u0);
    while (v0 < v1 && orc_isspace((unsigned char)*v0)) v0++;
    while (v1 > v0 && orc_isspace((unsigned char)v1[-1])) v1--;
    while (u0 < u1 && orc_isspace((unsigned char)*u0)) u0++;
    while (u1 > u0 && orc_isspace((unsigned char)u1[-1])) u1--;
    if ((size_t)(v1 - v0) >= vcap || (size_t)(u1 - u0) >= ucap) return -1;
    memcpy(val, v0, (size_t)(v1 - v0));
    val[v1 - v0] = 0;
    memcpy(unit, u0, (size_t)(u1 - u0));
    unit[u1 - u0] = 0;
    return 0;
}

/* Rust u64::from_str: optional '+', at least one ASCII digit, no overflow. */
static int parse_u64_rust(const char* s, uint64_t* out) {
    const char* p = s;
    if (*p == '+') p++;
    if (!*p) return -1;
    uint64_t v = 0;
    for (; *p; p++) {
        if (*p < '0' || *p > '9') return -1;
        uint64_t d = (uint64_t)(*p - '0');
        if (v > (UINT64_MAX - d) / 10) return -1;
        v = v * 10 + d;
    }
    *out = v;
    return 0;
}

/* parse_time_nanosec (units.rs:809-837) over Time<TimePrefix>
 * (units.rs:233-279, unit_impl! from_str :404-437, suffixes [""] :547). */
int64_t orc_parse_time_ns(const char* s) {
    if (!s) return -1;
    char val[128], unit[128];
    if (split_value_unit(s, val, sizeof val, unit, sizeof unit) != 0) return -1;
    uint64_t factor;
    if (unit[0] == 0) factor = 1000000000ull; /* TimePrefix default = Sec (units.rs:227-231) */
    else if (!strcmp(unit, "ns") || !strcmp(unit, "nanosecond") || !strcmp(unit, "nanoseconds")) factor = 1ull;
    else if (!strcmp(unit, "us") || !strcmp(unit, "\xce\xbcs") || !strcmp(unit, "microsecond") ||
             !strcmp(unit, "microseconds")) factor = 1000ull;
    else if (!strcmp(unit, "ms") || !strcmp(unit, "millisecond") || !strcmp(unit, "milliseconds")) factor = 1000000ull;
    else if (!strcmp(unit, "s") || !strcmp(unit, "sec") || !strcmp(unit, "secs") || !strcmp(unit, "second") ||
             !strcmp(unit, "seconds")) factor = 1000000000ull;
    else if (!strcmp(unit, "m") || !strcmp(unit, "min") || !strcmp(unit, "mins") || !strcmp(unit, "minute") ||
             !strcmp(unit, "minutes")) factor = 60000000000ull;
    else if (!strcmp(unit, "h") || !strcmp(unit, "hr") || !strcmp(unit, "hrs") || !strcmp(unit, "hour") ||
             !strcmp(unit, "hours")) factor = 3600000000000ull;
    else return -1;
    uint64_t v;
    if (parse_u64_rust(val, &v) != 0) return -1;
    if (v != 0 && v > UINT64_MAX / factor) return -1; /* checked_mul (units.rs:371-378) */
    uint64_t ns = v * factor;
    if (ns > (uint64_t)INT64_MAX) return -1; /* try_into i64 (units.rs:828-834) */
    return (int64_t)ns;
}

/* parse_bandwidth (units.rs:777-807) over BitsPerSec<SiPrefixUpper>
 * (suffixes ["bit","bits"] units.rs:577, prefixes :141-216). */
int64_t orc_parse_bandwidth_bits(const char* s) {
    if (!s) return -1;
    char val[128], unit[128];
    if (split_value_unit(s, val, sizeof val, unit, sizeof unit) != 0) return -1;
    /* try removing suffixes in order (units.rs:427-433) */
    size_t ul = strlen(unit);
    if (ul >= 3 && !strcmp(unit + ul - 3, "bit")) unit[ul - 3] = 0;
    else if (ul >= 4 && !strcmp(unit + ul - 4, "bits")) unit[ul - 4] = 0;
    uint64_t factor;
    if (unit[0] == 0) factor = 1;
    else if (!strcmp(unit, "K") || !strcmp(unit, "kilo")) factor = 1000ull;
    else if (!strcmp(unit, "Ki") || !strcmp(unit, "kibi")) factor = 1024ull;
    else if (!strcmp(unit, "M") || !strcmp(unit, "mega")) factor = 1000000ull;
    else if (!strcmp(unit, "Mi") || !strcmp(unit, "mebi")) factor = 1048576ull;
    else if (!strcmp(unit, "G") || !strcmp(unit, "giga")) factor = 1000000000ull;
    else if (!strcmp(unit, "Gi") || !strcmp(unit, "gibi")) factor = 1073741824ull;
    else if (!strcmp(unit, "T") || !strcmp(unit, "tera")) factor = 1000000000000ull;
    else if (!strcmp(unit, "Ti") || !strcmp(unit, "tebi")) factor = 1099511627776ull;
    else return -1;
    uint64_t v;
    if (parse_u64_rust(val, &v) != 0) return -1;
    if (v != 0 && v > UINT64_MAX / factor) return -1;
    uint64_t b = v * factor;
    if (b > (uint64_t)INT64_MAX) return -1;
    return (int64_t)b;
}

/* ======================================================================= */
/* rand_r streams: utility/random.c:32-51 over glibc rand_r                 */
/* ======================================================================= */

/* glibc stdlib/rand_r.c (the libc the reference links; published algorithm). */
int orc_rand_r(uint32_t* state) {
    uint32_t next = *state;
    int result;
    next *= 1103515245u;
    next += 12345u;
    result = (int)((next / 65536u) % 2048u);
    next *= 1103515245u;
    next += 12345u;
    result <<= 10;
    result ^= (int)((next / 65536u) % 1024u);
    next *= 1103515245u;
    next += 12345u;
    result <<= 10;
    result ^= (int)((next / 65536u) % 1024u);
    *state = next;
    return result;
}

/* random_nextDouble (random.c:39-43): r / RAND_MAX */
double orc_next_double(uint32_t* state) { return (double)orc_rand_r(state) / 2147483647.0; }

/* random_nextUInt (random.c:45-51) */
uint32_t orc_next_uint(uint32_t* state) {
    double f = orc_next_double(state);
    return (uint32_t)(f * 4294967295.0);
}

/* ======================================================================= */
/* GML reader: igraph_read_graph_gml subset (topology.c:326-360 -> igraph)  */
/* ======================================================================= */

typedef enum { GV_INT, GV_REAL, GV_STR, GV_LIST } GvType;
typedef struct GItem GItem;
typedef struct GList {
    GItem* items;
    int n, cap;
} GList;
struct GItem {
    char* key;
    GvType type;
    long long ival;
    double rval;
    char* sval;
    GList list;
};

typedef struct {
    const char* p;
    int line;
    int err;
} GLex;

static void glist_push(GList* l, GItem it) {
    if (l->n == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 8;
        l->items = (GItem*)realloc(l->items, sizeof(GItem) * (size_t)l->cap);
    }
    l->items[l->n++] = it;
}

static void glist_free(GList* l) {
    for (int i = 0; i < l->n; i++) {
        free(l->items[i].key);
        free(l->items[i].sval);
        if (l->items[i].type == GV_LIST) glist_free(&l->items[i].list);
    }
    free(l->items);
    l->items = NULL;
    l->n = l->cap = 0;
}

static void glex_skip(GLex* L) {
    for (;;) {
        while (*L->p && (orc_isspace((unsigned char)*L->p))) L->p++;
        if (*L->p == '#') { /* comment to end of line */
            while (*L->p && *L->p != '\n') L->p++;
            continue;
        }
        break;
    }
}

/* Parses "key value" pairs until ']' (nested) or end of text (top). */
static int gparse_list(GLex* L, GList* out, int nested) {
    for (;;) {
        glex_skip(L);
        if (!*L->p) return nested ? -1 : 0;
        if (*L->p == ']') {
            if (!nested) return -1;
            L->p++;
            return 0;
        }
        if (!(isalpha((unsigned char)*L->p) || *L->p == '_')) return -1;
        const char* k0 = L->p;
        while (isalnum((unsigned char)*L->p) || *L->p == '_') L->p++;
        GItem it;
        memset(&it, 0, sizeof it);
        it.key = strndup(k0, (size_t)(L->p - k0));
        glex_skip(L);
        const char* p = L->p;
        if (*p == '[') {
            L->p++;
            it.type = GV_LIST;
            if (gparse_list(L, &it.list, 1) != 0) {
                free(it.key);
                glist_free(&it.list);
                return -1;
            }
        } else if (*p == '"') {
            const char* s0 = ++L->p;
            while (*L->p && *L->p != '"') L->p++;
            if (*L->p != '"') {
                free(it.key);
                return -1;
            }
            it.type = GV_STR;
            it.sval = strndup(s0, (size_t)(L->p - s0));
            L->p++;
        } else if (*p == '-' || (*p >= '0' && *p <= '9')) {
            const char* n0 = L->p;
            if (*L->p == '-') L->p++;
            if (!(*L->p >= '0' && *L->p <= '9')) {
                free(it.key);
                return -1;
            }
            while (*L->p >= '0' && *L->p <= '9') L->p++;
            int real = 0;
            if (*L->p == '.' && L->p[1] >= '0' && L->p[1] <= '9') {
                real = 1;
                L->p++;
                while (*L->p >= '0' && *L->p <= '9') L->p++;
            }
            if ((*L->p == 'e' || *L->p == 'E') &&
                ((L->p[1] >= '0' && L->p[1] <= '9') ||
                 ((L->p[1] == '+' || L->p[1] == '-') && L->p[2] >= '0' && L->p[2] <= '9'))) {
                real = 1;
                L->p += 2;
                while (*L->p >= '0' && *L->p <= '9') L->p++;
            }
            char* tok = strndup(n0, (size_t)(L->p - n0));
            if (real) {
                it.type = GV_REAL;
                it.rval = strtod(tok, NULL);
            } else {
                it.type = GV_INT;
                it.ival = strtoll(tok, NULL, 10);
            }
            free(tok);
        } else {
            free(it.key);
            return -1;
        }
        glist_push(out, it);
    }
}

/* ======================================================================= */
/* Graph + attribute tables (what igraph's C attribute handler holds)       */
/* ======================================================================= */

typedef struct {
    char* name;
    int is_string; /* IGRAPH_ATTRIBUTE_STRING vs NUMERIC */
    double* num;   /* NaN when absent */
    char** str;    /* "" when absent */
} Attr;

typedef struct {
    int n;
    Attr* a;
} AttrSet;

static Attr* attr_find(AttrSet* s, const char* name) {
    for (int i = 0; i < s->n; i++)
        if (!strcmp(s->a[i].name, name)) return &s->a[i];
    return NULL;
}

static void attrset_free(AttrSet* s) {
    for (int i = 0; i < s->n; i++) {
        free(s->a[i].name);
        free(s->a[i].num);
        if (s->a[i].str) {
            free(s->a[i].str); /* strings are owned by the GML tree */
        }
    }
    free(s->a);
}

/* Fill attribute table over a sequence of GML blocks (igraph: type is
 * NUMERIC unless any occurrence is a string; missing -> NaN / ""). */
static void attrs_build(AttrSet* s, GItem** blocks, int nb, int skip_src_tgt) {
    s->n = 0;
    s->a = NULL;
    for (int b = 0; b < nb; b++) {
        GList* l = &blocks[b]->list;
        for (int j = 0; j < l->n; j++) {
            GItem* it = &l->items[j];
            if (it->type == GV_LIST) continue; /* composite attributes ignored */
            if (skip_src_tgt && (!strcmp(it->key, "source") || !strcmp(it->key, "target"))) continue;
            Attr* a = attr_find(s, it->key);
            if (!a) {
                s->a = (Attr*)realloc(s->a, sizeof(Attr) * (size_t)(s->n + 1));
                a = &s->a[s->n++];
                memset(a, 0, sizeof *a);
                a->name = strdup(it->key);
                a->is_string = (it->type == GV_STR);
            } else if (it->type == GV_STR) {
                a->is_string = 1;
            }
        }
    }
    static char empty[1] = {0};
    for (int i = 0; i < s->n; i++) {
        Attr* a = &s->a[i];
        if (a->is_string) {
            a->str = (char**)malloc(sizeof(char*) * (size_t)(nb ? nb : 1));
            for (int b = 0; b < nb; b++) a->str[b] = empty;
        } else {
            a->num = (double*)malloc(sizeof(double) * (size_t)(nb ? nb : 1));
            for (int b = 0; b < nb; b++) a->num[b] = NAN;
        }
    }
    for (int b = 0; b < nb; b++) {
        GList* l = &blocks[b]->list;
        for (int j = 0; j < l->n; j++) {
            GItem* it = &l->items[j];
            if (it->type == GV_LIST) continue;
            if (skip_src_tgt && (!strcmp(it->key, "source") || !strcmp(it->key, "target"))) continue;
            Attr* a = attr_find(s, it->key);
            if (a->is_string) {
                if (it->type == GV_STR) a->str[b] = it->sval;
                else {
                    /* numeric value in a string attribute: printed (unpinned corner) */
                    char buf[64];
                    if (it->type == GV_INT) snprintf(buf, sizeof buf, "%lld", it->ival);
                    else snprintf(buf, sizeof buf, "%.17g", it->rval);
                    free(it->sval);
                    it->sval = strdup(buf);
                    a->str[b] = it->sval;
                }
            } else {
                a->num[b] = (it->type == GV_INT) ? (double)it->ival : it->rval;
            }
        }
    }
}

typedef struct {
    int eid;
    int nbr;
} Inc;

struct OrcTopo {
    GList tree;
    int directed;
    int V, E;
    int* efrom; /* igraph storage: directed as given; undirected from=max to=min */
    int* eto;
    AttrSet va, ea;
    /* incidence (igraph_incident mode OUT): CSR */
    int* inc_off;
    Inc* inc;
    double* weight_ms; /* _topology_extractEdgeWeights (topology.c:1065-1122) */
    double* edge_rel;  /* 1.0 - packet_loss (topology.c:396) */
    int is_complete;
    int use_sp;
    /* attach state */
    int nip, capip;
    uint32_t* ip_keys;
    int* ip_vertex;
    unsigned char* v_attached;
    /* path cache: row per source vertex, allocated lazily */
    struct PathE {
        unsigned char present, is_direct;
        double lat, rel;
        uint64_t pkts;
    }** cache;
    /* rows already computed once: on a directed graph the reference recomputes
     * row s on every (s, d) lookup whose pair was stored as (d, s)
     * (topology.c:1940-1968, the (d, s) probe is undirected-only); that
     * recomputation stores nothing (every (s, v) of the row is already stored
     * either way, entries are never removed), so it is skipped here */
    unsigned char* row_done;
    double min_lat;
    int min_updates;
    uint64_t next_min_jump_ns;
    long long* v_ids; /* GML node ids (VERTEX_ATTR_ID) */
};
typedef struct PathE PathE;

static int cmp_inc(const void* a, const void* b) {
    const Inc* x = (const Inc*)a;
    const Inc* y = (const Inc*)b;
    if (x->nbr != y->nbr) return x->nbr < y->nbr ? -1 : 1;
    /* igraph_vector_order leaves parallel edges in descending id order */
    return x->eid > y->eid ? -1 : (x->eid < y->eid);
}

/* igraph_incident(graph, v, IGRAPH_OUT): directed -> out-edges sorted by
 * head; undirected -> ALL: out-part (from==v, by to) then in-part (to==v, by
 * from), i.e. ascending neighbour, undirected loops listed twice. */
static void build_incidence(OrcTopo* t) {
    int V = t->V, E = t->E;
    int* deg = (int*)calloc((size_t)V + 1, sizeof(int));
    for (int e = 0; e < E; e++) {
        deg[t->efrom[e]]++;
        if (!t->directed) deg[t->eto[e]]++;
    }
    t->inc_off = (int*)malloc(sizeof(int) * ((size_t)V + 1));
    t->inc_off[0] = 0;
    for (int v = 0; v < V; v++) t->inc_off[v + 1] = t->inc_off[v] + deg[v];
    t->inc = (Inc*)malloc(sizeof(Inc) * (size_t)(t->inc_off[V] ? t->inc_off[V] : 1));
    int* fill = (int*)calloc((size_t)V, sizeof(int));
    for (int e = 0; e < E; e++) {
        int f = t->efrom[e], g = t->eto[e];
        t->inc[t->inc_off[f] + fill[f]++] = (Inc){e, g};
        if (!t->directed) t->inc[t->inc_off[g] + fill[g]++] = (Inc){e, f};
    }
    for (int v = 0; v < V; v++) {
        /* out-part entries have nbr <= v, in-part nbr >= v: a single sort by
         * (nbr, eid desc) reproduces the concatenation except that the two
         * copies of an undirected loop must stay adjacent (they do: equal nbr). */
        qsort(t->inc + t->inc_off[v], (size_t)deg[v], sizeof(Inc), cmp_inc);
    }
    free(deg);
    free(fill);
}

/* igraph_get_eid(from,to,directed): first edge in incidence order (simple
 * graphs have exactly one; parallel-edge choice is unpinned). -1 if none. */
static int get_eid(const OrcTopo* t, int from, int to) {
    for (int k = t->inc_off[from]; k < t->inc_off[from + 1]; k++)
        if (t->inc[k].nbr == to) return t->inc[k].eid;
    return -1;
}

static const char* vas(const OrcTopo* t, const char* name, int v) {
    Attr* a = attr_find((AttrSet*)&t->va, name);
    if (!a || !a->is_string) return NULL;
    const char* s = a->str[v];
    return (s && s[0]) ? s : NULL;
}

/* _topology_findVertexAttributeStringBandwidth (topology.c:210-233) */
static int vertex_bw(const OrcTopo* t, int v, const char* name, uint64_t* out) {
    const char* s = vas(t, name, v);
    if (!s) return 0;
    int64_t b = orc_parse_bandwidth_bits(s);
    if (b < 0) return 0;
    b /= 8 * 1024;
    *out = (uint64_t)b;
    return 1;
}

/* _topology_findEdgeAttributeStringTimeMs (topology.c:280-302) */
static int edge_time_ms(const OrcTopo* t, int e, const char* name, double* out) {
    Attr* a = attr_find((AttrSet*)&t->ea, name);
    if (!a || !a->is_string) return 0;
    const char* s = a->str[e];
    if (!s || !s[0]) return 0;
    int64_t ns = orc_parse_time_ns(s);
    if (ns < 0) return 0;
    *out = (double)ns / 1000000.0;
    return 1;
}

static int edge_num(const OrcTopo* t, int e, const char* name, double* out) {
    Attr* a = attr_find((AttrSet*)&t->ea, name);
    if (!a || a->is_string) return 0;
    if (isnan(a->num[e])) return 0;
    *out = a->num[e];
    return 1;
}

/* g_ascii_strncasecmp(attrName, expected, strlen(expected)) == 0 */
static int key_is(const char* name, const char* expected) {
    return strncasecmp(name, expected, strlen(expected)) == 0;
}

/* _topology_checkGraphAttributes (topology.c:525-657) */
static int check_attributes(OrcTopo* t) {
    int ok = 1;
    for (int i = 0; i < t->va.n; i++) {
        Attr* a = &t->va.a[i];
        if (key_is(a->name, "id")) ok = ok && !a->is_string;
        else if (key_is(a->name, "ip_address") || key_is(a->name, "city_code") ||
                 key_is(a->name, "country_code") || key_is(a->name, "bandwidth_down") ||
                 key_is(a->name, "bandwidth_up") || key_is(a->name, "label"))
            ok = ok && a->is_string;
        else ok = 0;
    }
    if (!attr_find(&t->va, "id") || !attr_find(&t->va, "bandwidth_down") || !attr_find(&t->va, "bandwidth_up"))
        ok = 0;
    for (int i = 0; i < t->ea.n; i++) {
        Attr* a = &t->ea.a[i];
        if (key_is(a->name, "latency") || key_is(a->name, "jitter") || key_is(a->name, "label"))
            ok = ok && a->is_string;
        else if (key_is(a->name, "packet_loss")) ok = ok && !a->is_string;
        else ok = 0;
    }
    if (!attr_find(&t->ea, "latency") || !attr_find(&t->ea, "packet_loss")) ok = 0;
    return ok;
}

/* igraph_is_connected(IGRAPH_STRONG) && clusters == 1 (topology.c:674-713) */
static int strongly_connected(const OrcTopo* t) {
    int V = t->V;
    if (V == 0) return 0;
    int* seen = (int*)calloc((size_t)V, sizeof(int));
    int* stack = (int*)malloc(sizeof(int) * (size_t)V);
    /* reverse adjacency for the backward pass of a directed graph */
    int* roff = (int*)calloc((size_t)V + 1, sizeof(int));
    int* radj = (int*)malloc(sizeof(int) * (size_t)(t->E + 1));
    for (int e = 0; e < t->E; e++) roff[t->eto[e] + 1]++;
    for (int v = 0; v < V; v++) roff[v + 1] += roff[v];
    int* rf = (int*)calloc((size_t)V, sizeof(int));
    for (int e = 0; e < t->E; e++) radj[roff[t->eto[e]] + rf[t->eto[e]]++] = t->efrom[e];
    int ok = 1;
    for (int pass = 0; pass < (t->directed ? 2 : 1) && ok; pass++) {
        memset(seen, 0, sizeof(int) * (size_t)V);
        int sp = 0, cnt = 1;
        stack[sp++] = 0;
        seen[0] = 1;
        while (sp) {
            int u = stack[--sp];
            int k0 = pass == 0 ? t->inc_off[u] : roff[u];
            int k1 = pass == 0 ? t->inc_off[u + 1] : roff[u + 1];
            for (int k = k0; k < k1; k++) {
                int w = pass == 0 ? t->inc[k].nbr : radj[k];
                if (!seen[w]) {
                    seen[w] = 1;
                    cnt++;
                    stack[sp++] = w;
                }
            }
        }
        if (cnt != V) ok = 0;
    }
    free(seen);
    free(stack);
    free(roff);
    free(radj);
    free(rf);
    return ok;
}

/* _topology_isComplete (topology.c:409-511) */
static int is_complete(const OrcTopo* t) {
    for (int v = 0; v < t->V; v++) {
        int ecount = t->inc_off[v + 1] - t->inc_off[v];
        if (!t->directed && get_eid(t, v, v) >= 0) ecount -= 1;
        if (ecount < t->V) return 0;
    }
    return 1;
}

/* _topology_checkGraphVerticesHelperHook (topology.c:718-829) */
static int check_vertices(const OrcTopo* t) {
    Attr* id = attr_find((AttrSet*)&t->va, "id");
    int ok = 1;
    for (int v = 0; v < t->V; v++) {
        if (!id || id->is_string || isnan(id->num[v])) ok = 0;
        uint64_t bw;
        if (!(vertex_bw(t, v, "bandwidth_down", &bw) && bw > 0)) ok = 0;
        if (!(vertex_bw(t, v, "bandwidth_up", &bw) && bw > 0)) ok = 0;
    }
    return ok;
}

/* _topology_checkGraphEdgesHelperHook (topology.c:892-977) */
static int check_edges(const OrcTopo* t) {
    int ok = 1;
    for (int e = 0; e < t->E; e++) {
        double lat, loss, jit;
        if (!(edge_time_ms(t, e, "latency", &lat) && lat > 0.0)) ok = 0;
        if (!(edge_num(t, e, "packet_loss", &loss) && loss >= 0.0f && loss <= 1.0f)) ok = 0;
        if (attr_find((AttrSet*)&t->ea, "jitter") && edge_time_ms(t, e, "jitter", &jit) && !(jit >= 0.0f)) ok = 0;
    }
    return ok;
}

void orc_topology_free(OrcTopo* t) {
    if (!t) return;
    attrset_free(&t->va);
    attrset_free(&t->ea);
    glist_free(&t->tree);
    free(t->efrom);
    free(t->eto);
    free(t->v_ids);
    free(t->inc_off);
    free(t->inc);
    free(t->weight_ms);
    free(t->edge_rel);
    free(t->ip_keys);
    free(t->ip_vertex);
    free(t->v_attached);
    if (t->cache) {
        for (int v = 0; v < t->V; v++) free(t->cache[v]);
        free(t->cache);
    }
    free(t->row_done);
    free(t);
}

typedef struct {
    long long id;
    int v;
} IdIdx;

static int cmp_ididx(const void* a, const void* b) {
    const IdIdx *x = (const IdIdx*)a, *y = (const IdIdx*)b;
    return x->id < y->id ? -1 : x->id > y->id;
}

static int find_id(const IdIdx* byid, int n, long long id) {
    int lo = 0, hi = n - 1;
    while (lo <= hi) {
        int mid = lo + (hi - lo) / 2;
        if (byid[mid].id == id) return byid[mid].v;
        if (byid[mid].id < id) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

/* topology_new (topology.c:2328-2354): load, check, extract weights. */
OrcTopo* orc_topology_new(const char* text, int use_shortest_path) {
    OrcTopo* t = (OrcTopo*)calloc(1, sizeof(OrcTopo));
    t->use_sp = use_shortest_path ? 1 : 0;
    GLex L = {text, 1, 0};
    if (!text || gparse_list(&L, &t->tree, 0) != 0) goto fail;
    GItem* graph = NULL;
    for (int i = 0; i < t->tree.n; i++)
        if (!strcmp(t->tree.items[i].key, "graph") && t->tree.items[i].type == GV_LIST) {
            graph = &t->tree.items[i];
            break;
        }
    if (!graph) goto fail;
    int nn = 0, ne = 0;
    for (int i = 0; i < graph->list.n; i++) {
        GItem* it = &graph->list.items[i];
        if (!strcmp(it->key, "node")) {
            if (it->type != GV_LIST) goto fail;
            nn++;
        } else if (!strcmp(it->key, "edge")) {
            if (it->type != GV_LIST) goto fail;
            ne++;
        } else if (!strcmp(it->key, "directed") && it->type == GV_INT) {
            t->directed = (it->ival == 1);
        }
    }
    GItem** nodes = (GItem**)malloc(sizeof(GItem*) * (size_t)(nn + 1));
    GItem** edges = (GItem**)malloc(sizeof(GItem*) * (size_t)(ne + 1));
    nn = ne = 0;
    for (int i = 0; i < graph->list.n; i++) {
        GItem* it = &graph->list.items[i];
        if (!strcmp(it->key, "node")) nodes[nn++] = it;
        else if (!strcmp(it->key, "edge")) edges[ne++] = it;
    }
    t->V = nn;
    t->E = ne;
    /* node ids: integer, unique; vertex index = order of node blocks */
    long long* ids = (long long*)malloc(sizeof(long long) * (size_t)(nn + 1));
    int bad = 0;
    for (int v = 0; v < nn; v++) {
        int has = 0;
        for (int j = 0; j < nodes[v]->list.n; j++) {
            GItem* it = &nodes[v]->list.items[j];
            if (!strcmp(it->key, "id")) {
                if (it->type != GV_INT) bad = 1;
                ids[v] = it->ival;
                has = 1;
                break;
            }
        }
        if (!has) bad = 1;
    }
    /* (id, vertex) pairs sorted by id: uniqueness check and endpoint lookup
     * in O(log V) (ids are unique, so the lookup is the one matching vertex) */
    IdIdx* byid = (IdIdx*)malloc(sizeof(IdIdx) * (size_t)(nn + 1));
    for (int v = 0; v < nn; v++) byid[v].id = ids[v], byid[v].v = v;
    qsort(byid, (size_t)nn, sizeof(IdIdx), cmp_ididx);
    for (int v = 1; v < nn && !bad; v++)
        if (byid[v].id == byid[v - 1].id) bad = 1;
    t->efrom = (int*)malloc(sizeof(int) * (size_t)(ne + 1));
    t->eto = (int*)malloc(sizeof(int) * (size_t)(ne + 1));
    for (int e = 0; e < ne && !bad; e++) {
        long long s = 0, g = 0;
        int hs = 0, hg = 0;
        for (int j = 0; j < edges[e]->list.n; j++) {
            GItem* it = &edges[e]->list.items[j];
            if (!strcmp(it->key, "source")) {
                if (it->type != GV_INT) bad = 1;
                s = it->ival;
                hs = 1;
            } else if (!strcmp(it->key, "target")) {
                if (it->type != GV_INT) bad = 1;
                g = it->ival;
                hg = 1;
            }
        }
        if (!hs || !hg) {
            bad = 1;
            break;
        }
        int sv = find_id(byid, nn, s), gv = find_id(byid, nn, g);
        if (sv < 0 || gv < 0) {
            bad = 1;
            break;
        }
        if (t->directed || sv > gv) {
            t->efrom[e] = sv;
            t->eto[e] = gv;
        } else {
            t->efrom[e] = gv;
            t->eto[e] = sv;
        }
    }
    t->v_ids = ids;
    free(byid);
    if (bad) {
        free(nodes);
        free(edges);
        goto fail;
    }
    attrs_build(&t->va, nodes, nn, 0);
    attrs_build(&t->ea, edges, ne, 1);
    free(nodes);
    free(edges);
    build_incidence(t);

    /* _topology_checkGraph (topology.c:1040-1063) */
    if (!check_attributes(t)) goto fail;
    if (!strongly_connected(t)) goto fail;
    t->is_complete = is_complete(t);
    if (!t->is_complete && !t->use_sp) goto fail;
    if (!check_vertices(t) || !check_edges(t)) goto fail;

    /* _topology_extractEdgeWeights + reliabilities */
    t->weight_ms = (double*)malloc(sizeof(double) * (size_t)(ne + 1));
    t->edge_rel = (double*)malloc(sizeof(double) * (size_t)(ne + 1));
    for (int e = 0; e < ne; e++) {
        double loss = 0;
        edge_time_ms(t, e, "latency", &t->weight_ms[e]);
        edge_num(t, e, "packet_loss", &loss);
        t->edge_rel[e] = 1.0f - loss;
    }
    t->v_attached = (unsigned char*)calloc((size_t)t->V, 1);
    t->cache = (PathE**)calloc((size_t)t->V, sizeof(PathE*));
    t->row_done = (unsigned char*)calloc((size_t)t->V, 1);
    return t;
fail:
    orc_topology_free(t);
    return NULL;
}

int orc_topology_vertex_count(const OrcTopo* t) { return t->V; }
int orc_topology_edge_count(const OrcTopo* t) { return t->E; }
int orc_topology_is_directed(const OrcTopo* t) { return t->directed; }
int orc_topology_is_complete(const OrcTopo* t) { return t->is_complete; }

/* ======================================================================= */
/* attach: topology.c:2024-2272                                            */
/* ======================================================================= */

/* address_stringToIP (address.c:145-152): inet_pton, INADDR_NONE on failure */
static uint32_t str_to_ip(const char* s) {
    struct in_addr a;
    if (s && inet_pton(AF_INET, s, &a) == 1) return a.s_addr;
    return 0xffffffffu;
}

/* INADDR_* compared against network-order values, as the reference does */
static int ip_usable(uint32_t ip) { return ip != 0xffffffffu && ip != 0u && ip != 0x7f000001u; }

typedef struct {
    int* v;
    int n;
} Queue;

static void q_push(Queue* q, int v, int cap) {
    (void)cap;
    q->v[q->n++] = v;
}

/* virtualIP hash table (topology.c:40, GHashTable) as linear probing over
 * capip slots; ip_vertex < 0 marks an empty slot, -2 a removed one. */
static uint32_t ip_slot(const OrcTopo* t, uint32_t ip) {
    /* full-avalanche mix: network-order IPs differ only in their high bytes */
    ip ^= ip >> 16;
    ip *= 0x85ebca6bu;
    ip ^= ip >> 13;
    ip *= 0xc2b2ae35u;
    ip ^= ip >> 16;
    return ip & (uint32_t)(t->capip - 1);
}

static void ip_map_set(OrcTopo* t, uint32_t ip, int v);

static void ip_map_grow(OrcTopo* t) {
    int oc = t->capip;
    uint32_t* ok = t->ip_keys;
    int* ov = t->ip_vertex;
    t->capip = oc ? oc * 2 : 1024;
    t->ip_keys = (uint32_t*)calloc((size_t)t->capip, sizeof(uint32_t));
    t->ip_vertex = (int*)malloc(sizeof(int) * (size_t)t->capip);
    for (int i = 0; i < t->capip; i++) t->ip_vertex[i] = -1;
    t->nip = 0;
    for (int i = 0; i < oc; i++)
        if (ov[i] >= 0) ip_map_set(t, ok[i], ov[i]);
    free(ok);
    free(ov);
}

static void ip_map_set(OrcTopo* t, uint32_t ip, int v) {
    if ((t->nip + 1) * 2 > t->capip) ip_map_grow(t);
    uint32_t h = ip_slot(t, ip);
    while (t->ip_vertex[h] != -1 && !(t->ip_vertex[h] >= 0 && t->ip_keys[h] == ip))
        h = (h + 1) & (uint32_t)(t->capip - 1);
    if (t->ip_vertex[h] == -1) t->nip++;
    t->ip_keys[h] = ip;
    t->ip_vertex[h] = v;
}

int orc_vertex_of_ip(OrcTopo* t, uint32_t ip) {
    if (!t->capip) return -1;
    uint32_t h = ip_slot(t, ip);
    while (t->ip_vertex[h] != -1) {
        if (t->ip_vertex[h] >= 0 && t->ip_keys[h] == ip) return t->ip_vertex[h];
        h = (h + 1) & (uint32_t)(t->capip - 1);
    }
    return -1;
}

int orc_topology_attach(OrcTopo* t, uint32_t ip_net, uint32_t* rng_state, const char* ip_hint,
                        const char* city_hint, const char* country_hint, uint64_t* bw_down,
                        uint64_t* bw_up) {
    (void)ip_net;
    int V = t->V;
    Queue city = {(int*)malloc(sizeof(int) * (size_t)V), 0};
    Queue country = {(int*)malloc(sizeof(int) * (size_t)V), 0};
    Queue all = {(int*)malloc(sizeof(int) * (size_t)V), 0};
    unsigned nIPsCity = 0, nIPsCountry = 0, nIPsAll = 0;
    int requestedUsable = 0, exact = 0;
    uint32_t requested = 0;
    if (ip_hint) {
        uint32_t ip = str_to_ip(ip_hint);
        if (ip_usable(ip)) {
            requestedUsable = 1;
            requested = ip;
        }
    }
    /* _topology_findAttachmentVertexHelperHook over all vertices (:2024-2100);
     * without any hint every vertex lands in candidatesAll in order and no
     * LPM applies, so the scan is skipped (same choice, O(1)). */
    if (!ip_hint && !city_hint && !country_hint) {
        double r = orc_next_double(rng_state);
        int chosen = (int)round((double)((V - 1) * r));
        free(city.v);
        free(country.v);
        free(all.v);
        ip_map_set(t, ip_net, chosen);
        t->v_attached[chosen] = 1;
        if (bw_up) vertex_bw(t, chosen, "bandwidth_up", bw_up);
        if (bw_down) vertex_bw(t, chosen, "bandwidth_down", bw_down);
        return chosen;
    }
    for (int v = 0; v < V; v++) {
        const char* ipStr = vas(t, "ip_address", v);
        const char* cc = vas(t, "city_code", v);
        const char* co = vas(t, "country_code", v);
        int cityMatch = cc && city_hint && !strcasecmp(cc, city_hint);
        int countryMatch = co && country_hint && !strcasecmp(co, country_hint);
        int vUsable = 0;
        uint32_t vip = 0xffffffffu;
        if (ipStr) {
            uint32_t ip = str_to_ip(ipStr);
            if (ip_usable(ip)) {
                vUsable = 1;
                vip = ip;
            }
        }
        if (requestedUsable && vUsable && vip == requested) {
            if (!exact) {
                city.n = country.n = all.n = 0;
            }
            exact = 1;
            q_push(&all, v, V);
            nIPsAll++;
        }
        if (exact) continue;
        q_push(&all, v, V);
        if (vUsable) nIPsAll++;
        if (cityMatch) {
            q_push(&city, v, V);
            if (vUsable) nIPsCity++;
        }
        if (countryMatch) {
            q_push(&country, v, V);
            if (vUsable) nIPsCountry++;
        }
    }
    Queue* cand;
    int useLPM;
    if (city.n > 0) {
        cand = &city;
        useLPM = requestedUsable && nIPsCity > 0;
    } else if (country.n > 0) {
        cand = &country;
        useLPM = requestedUsable && nIPsCountry > 0;
    } else {
        cand = &all;
        useLPM = (ip_hint != NULL) && nIPsAll > 0;
    }
    int chosen = -1;
    if (cand->n > 0) {
        if (useLPM && !exact) {
            /* _topology_getLongestPrefixMatch (:2102-2130) */
            uint32_t best = 0;
            for (int i = 0; i < cand->n; i++) {
                const char* s = vas(t, "ip_address", cand->v[i]);
                uint32_t vip = str_to_ip(s ? s : "");
                uint32_t match = ~(vip ^ requested);
                if (match > best || best == 0) {
                    best = match;
                    chosen = cand->v[i];
                }
            }
        } else {
            double r = orc_next_double(rng_state);
            int range = cand->n - 1;
            int idx = (int)round((double)(range * r));
            chosen = cand->v[idx];
        }
    }
    free(city.v);
    free(country.v);
    free(all.v);
    if (chosen < 0) return -1;
    ip_map_set(t, ip_net, chosen);
    t->v_attached[chosen] = 1;
    if (bw_up) vertex_bw(t, chosen, "bandwidth_up", bw_up);
    if (bw_down) vertex_bw(t, chosen, "bandwidth_down", bw_down);
    return chosen;
}

/* topology_detach (topology.c:2274-2281): removes the IP only */
void orc_topology_detach(OrcTopo* t, uint32_t ip) {
    if (!t->capip) return;
    uint32_t h = ip_slot(t, ip);
    while (t->ip_vertex[h] != -1) {
        if (t->ip_vertex[h] >= 0 && t->ip_keys[h] == ip) {
            t->ip_vertex[h] = -2; /* tombstone keeps probe chains intact */
            return;
        }
        h = (h + 1) & (uint32_t)(t->capip - 1);
    }
}

/* ======================================================================= */
/* igraph_2wheap (igraph 0.8 src/core/indheap.c) -- max-heap on -dist      */
/* ======================================================================= */

typedef struct {
    double* data;
    int* index;  /* heap position -> vertex */
    int* index2; /* vertex -> position + 2 (0 = absent) */
    int size;
} Wheap;

#define WH_PARENT(x) ((((x) + 1) / 2) - 1)
#define WH_LEFT(x) (((x) + 1) * 2 - 1)
#define WH_RIGHT(x) (((x) + 1) * 2)

static void wh_switch(Wheap* h, int e1, int e2) {
    if (e1 != e2) {
        double tmp = h->data[e1];
        h->data[e1] = h->data[e2];
        h->data[e2] = tmp;
        int t1 = h->index[e1], t2 = h->index[e2];
        h->index2[t1] = e2 + 2;
        h->index2[t2] = e1 + 2;
        h->index[e1] = t2;
        h->index[e2] = t1;
    }
}

static void wh_shift_up(Wheap* h, int e) {
    while (!(e == 0 || h->data[e] < h->data[WH_PARENT(e)])) {
        wh_switch(h, e, WH_PARENT(e));
        e = WH_PARENT(e);
    }
}

static void wh_sink(Wheap* h, int head) {
    for (;;) {
        int size = h->size;
        if (WH_LEFT(head) >= size) return;
        if (WH_RIGHT(head) == size || h->data[WH_LEFT(head)] >= h->data[WH_RIGHT(head)]) {
            if (h->data[head] < h->data[WH_LEFT(head)]) {
                wh_switch(h, head, WH_LEFT(head));
                head = WH_LEFT(head);
            } else return;
        } else {
            if (h->data[head] < h->data[WH_RIGHT(head)]) {
                wh_switch(h, head, WH_RIGHT(head));
                head = WH_RIGHT(head);
            } else return;
        }
    }
}

static void wh_push(Wheap* h, int idx, double elem) {
    int size = h->size++;
    h->data[size] = elem;
    h->index[size] = idx;
    h->index2[idx] = size + 2;
    wh_shift_up(h, size);
}

static double wh_delete_max(Wheap* h, int* idx) {
    double tmp = h->data[0];
    *idx = h->index[0];
    wh_switch(h, 0, h->size - 1);
    h->size--;
    h->index2[*idx] = 0;
    wh_sink(h, 0);
    return tmp;
}

static void wh_modify(Wheap* h, int idx, double elem) {
    int pos = h->index2[idx] - 2;
    h->data[pos] = elem;
    wh_sink(h, pos);
    wh_shift_up(h, pos);
}

/* igraph_get_shortest_paths_dijkstra (igraph 0.8 structural_properties.c),
 * mode OUT, weights = weight_ms, early exit once every target is popped.
 * Fills dist/rel (reliability folded left-to-right along the parent chain,
 * exactly _topology_computePathProperties' product, topology.c:1308-1365). */
static void dijkstra(const OrcTopo* t, int src, const unsigned char* is_target_in, int ntargets,
                     double* dist, double* rel) {
    int V = t->V;
    Wheap h;
    h.data = (double*)malloc(sizeof(double) * (size_t)V);
    h.index = (int*)malloc(sizeof(int) * (size_t)V);
    h.index2 = (int*)calloc((size_t)V, sizeof(int));
    h.size = 0;
    unsigned char* is_target = (unsigned char*)malloc((size_t)V);
    memcpy(is_target, is_target_in, (size_t)V);
    for (int v = 0; v < V; v++) {
        dist[v] = -1.0;
        rel[v] = 0.0;
    }
    int to_reach = ntargets;
    dist[src] = 0.0;
    rel[src] = 1.0;
    wh_push(&h, src, 0.0);
    while (h.size > 0 && to_reach > 0) {
        int u;
        double mindist = -wh_delete_max(&h, &u);
        if (is_target[u]) {
            is_target[u] = 0;
            to_reach--;
        }
        double ru = rel[u];
        for (int k = t->inc_off[u]; k < t->inc_off[u + 1]; k++) {
            int e = t->inc[k].eid, v = t->inc[k].nbr;
            double alt = mindist + t->weight_ms[e];
            double cur = dist[v];
            if (cur < 0) {
                dist[v] = alt;
                rel[v] = ru * t->edge_rel[e];
                wh_push(&h, v, -alt);
            } else if (alt < cur) {
                dist[v] = alt;
                rel[v] = ru * t->edge_rel[e];
                wh_modify(&h, v, -alt);
            }
        }
    }
    free(h.data);
    free(h.index);
    free(h.index2);
    free(is_target);
}

/* _topology_computeShortestPathToSelf (topology.c:1431-1576) */
static void self_path(const OrcTopo* t, int v, double* lat_out, double* rel_out, int* direct_out) {
    double minLatency = -1.0f, relMin = 0.0f;
    int isDirect = 0;
    for (int k = t->inc_off[v]; k < t->inc_off[v + 1]; k++) {
        int e = t->inc[k].eid;
        double lat = t->weight_ms[e];
        int edgeIsDirect = (t->inc[k].nbr == v);
        if (!edgeIsDirect) lat *= 2.0f;
        if (minLatency == -1 || lat < minLatency) {
            minLatency = lat;
            relMin = t->edge_rel[e];
            isDirect = edgeIsDirect;
        }
    }
    if (minLatency == -1) {
        minLatency = 0;
        isDirect = 1;
    }
    double r = relMin;
    if (!isDirect) r = r * r;
    *lat_out = minLatency;
    *rel_out = r;
    *direct_out = isDirect;
}

int orc_direct_path(OrcTopo* t, int s, int d, double* lat, double* rel) {
    int e = get_eid(t, s, d);
    if (e < 0) return -1;
    double tl = 0.0, tr = 1.0;
    tl += t->weight_ms[e];
    tr *= t->edge_rel[e];
    *lat = tl;
    *rel = tr;
    return 0;
}

/* A row of direct paths (use_shortest_path=false, topology.c:1816-1858):
 * orc_direct_path for every target; -1 / -1 where no edge joins them. */
void orc_direct_row(OrcTopo* t, int src, const int* targets, int ntargets, double* lat, double* rel) {
    for (int i = 0; i < ntargets; i++)
        if (orc_direct_path(t, src, targets[i], &lat[i], &rel[i]) != 0) lat[i] = rel[i] = -1.0;
}

int orc_compute_row(OrcTopo* t, int src, const int* targets, int ntargets, double* lat, double* rel) {
    int V = t->V;
    unsigned char* is_t = (unsigned char*)calloc((size_t)V, 1);
    int distinct = 0;
    for (int i = 0; i < ntargets; i++)
        if (!is_t[targets[i]]) {
            is_t[targets[i]] = 1;
            distinct++;
        }
    double* dist = (double*)malloc(sizeof(double) * (size_t)V);
    double* r = (double*)malloc(sizeof(double) * (size_t)V);
    dijkstra(t, src, is_t, distinct, dist, r);
    for (int i = 0; i < ntargets; i++) {
        int v = targets[i];
        if (v == src) {
            int dd;
            self_path(t, src, &lat[i], &rel[i], &dd);
        } else {
            double l = dist[v];
            if (l == 0) l = 1; /* topology.c:1787-1791 */
            lat[i] = l;
            rel[i] = r[v];
        }
    }
    free(is_t);
    free(dist);
    free(r);
    return 0;
}

/* ======================================================================= */
/* path cache + lookups: topology.c:1166-1265, 1900-2022                    */
/* ======================================================================= */

static PathE* cache_get(OrcTopo* t, int s, int d) {
    if (!t->cache[s]) return NULL;
    PathE* p = &t->cache[s][d];
    return __atomic_load_n(&p->present, __ATOMIC_ACQUIRE) ? p : NULL;
}

/* controller_updateMinTimeJump (controller.c:141-153) */
static void controller_update(OrcTopo* t, double minMs) {
    if (t->next_min_jump_ns == 0 || minMs < (double)t->next_min_jump_ns)
        t->next_min_jump_ns = ((uint64_t)minMs) * 1000000ull;
}

/* _topology_shouldStorePath + _topology_storePathInCache (:1189-1265) */
static void cache_store(OrcTopo* t, int isDirect, int s, int d, double lat, double rel) {
    if (cache_get(t, s, d) || cache_get(t, d, s)) return;
    if (!isDirect && !t->use_sp && get_eid(t, s, d) >= 0) return;
    if (!t->cache[s]) t->cache[s] = (PathE*)calloc((size_t)t->V, sizeof(PathE));
    PathE* p = &t->cache[s][d];
    p->is_direct = (unsigned char)isDirect;
    p->lat = lat;
    p->rel = rel;
    p->pkts = 0;
    __atomic_store_n(&p->present, 1, __ATOMIC_RELEASE); /* last: orc_round_mt readers */
    if (t->min_lat == 0 || lat < t->min_lat) {
        t->min_lat = lat;
        t->min_updates++;
        controller_update(t, t->min_lat);
    }
}

/* _topology_computeSourcePaths (:1578-1814) incl. the self case */
static int compute_source_paths(OrcTopo* t, int s, int d) {
    if (s == d) {
        double l, r;
        int dir;
        self_path(t, s, &l, &r, &dir);
        cache_store(t, dir, s, s, l, r);
        return 1;
    }
    if (t->row_done[s]) return 1; /* a recomputation would store nothing (row_done) */
    int V = t->V, n = 0;
    int* targets = (int*)malloc(sizeof(int) * (size_t)V);
    for (int v = 0; v < V; v++)
        if (t->v_attached[v]) targets[n++] = v;
    unsigned char* is_t = (unsigned char*)calloc((size_t)V, 1);
    for (int i = 0; i < n; i++) is_t[targets[i]] = 1;
    double* dist = (double*)malloc(sizeof(double) * (size_t)V);
    double* r = (double*)malloc(sizeof(double) * (size_t)V);
    dijkstra(t, s, is_t, n, dist, r);
    for (int i = 0; i < n; i++) {
        int v = targets[i];
        if (v == s || dist[v] < 0) continue;
        double l = dist[v];
        if (l == 0) l = 1;
        cache_store(t, 0, s, v, l, r[v]);
    }
    t->row_done[s] = 1;
    free(targets);
    free(is_t);
    free(dist);
    free(r);
    return 1;
}

static PathE* get_path_entry(OrcTopo* t, uint32_t sip, uint32_t dip) {
    int s = orc_vertex_of_ip(t, sip);
    if (s < 0) return NULL;
    int d = orc_vertex_of_ip(t, dip);
    if (d < 0) return NULL;
    PathE* p = cache_get(t, s, d);
    if (!p && !t->directed) p = cache_get(t, d, s);
    if (!p) {
        int ok;
        if (!t->use_sp) {
            double l, r;
            ok = orc_direct_path(t, s, d, &l, &r) == 0;
            if (ok) cache_store(t, 1, s, d, l, r);
        } else {
            ok = compute_source_paths(t, s, d);
        }
        if (ok) {
            p = cache_get(t, s, d);
            if (!p) p = cache_get(t, d, s);
        }
    }
    return p; /* NULL here is utility_panic in the reference (:1970-1976) */
}

double orc_topology_get_latency(OrcTopo* t, uint32_t s, uint32_t d) {
    PathE* p = get_path_entry(t, s, d);
    return p ? p->lat : -1.0;
}

double orc_topology_get_reliability(OrcTopo* t, uint32_t s, uint32_t d) {
    PathE* p = get_path_entry(t, s, d);
    return p ? p->rel : -1.0;
}

int orc_topology_is_routable(OrcTopo* t, uint32_t s, uint32_t d) {
    return orc_topology_get_latency(t, s, d) > -1 ? 1 : 0;
}

void orc_topology_increment_path_packet_counter(OrcTopo* t, uint32_t s, uint32_t d) {
    PathE* p = get_path_entry(t, s, d);
    if (p) p->pkts++;
}

uint64_t orc_topology_path_packet_count(OrcTopo* t, uint32_t s, uint32_t d) {
    int sv = orc_vertex_of_ip(t, s), dv = orc_vertex_of_ip(t, d);
    if (sv < 0 || dv < 0) return 0;
    PathE* p = cache_get(t, sv, dv);
    if (!p) p = cache_get(t, dv, sv);
    return p ? p->pkts : 0;
}

double orc_topology_min_path_latency(const OrcTopo* t) { return t->min_lat; }
int orc_topology_min_jump_updates(const OrcTopo* t) { return t->min_updates; }
uint64_t orc_controller_next_min_jump_ns(const OrcTopo* t) { return t->next_min_jump_ns; }

int orc_topology_preload_table(OrcTopo* t, const int* slots, int nslots, const double* lat, const double* rel) {
    int empty = t->use_sp;
    for (int v = 0; v < t->V && empty; v++) empty = t->cache[v] == NULL;
    if (empty) {
        /* Same stores, same order, without the lookups: on an empty cache
         * row i's store of (s_i, s_j) succeeds exactly for j > i (the
         * reverse (s_j, s_i), j < i, was stored by the earlier row j).  A row
         * never stores its own vertex (topology.c:1744-1752): the self path
         * is computed and stored by the first (X, X) lookup only. */
        for (int i = 0; i < nslots; i++) {
            int s = slots[i];
            if (!t->cache[s]) t->cache[s] = (PathE*)calloc((size_t)t->V, sizeof(PathE));
            for (int j = i + 1; j < nslots; j++) {
                PathE* p = &t->cache[s][slots[j]];
                p->present = 1;
                p->is_direct = 0;
                p->lat = lat[(size_t)i * nslots + j];
                p->rel = rel[(size_t)i * nslots + j];
                p->pkts = 0;
                if (t->min_lat == 0 || p->lat < t->min_lat) {
                    t->min_lat = p->lat;
                    t->min_updates++;
                    controller_update(t, t->min_lat);
                }
            }
        }
        return 0;
    }
    for (int i = 0; i < nslots; i++) {
        int s = slots[i];
        for (int j = 0; j < nslots; j++) {
            if (i == j) continue; /* self paths: first (X, X) lookup only */
            cache_store(t, 0, s, slots[j], lat[(size_t)i * nslots + j], rel[(size_t)i * nslots + j]);
        }
    }
    return 0;
}

/* Rows of a table whose columns are all attached vertices (slot order):
 * stores (rows[i], cols[j]) in row order, i.e. as if rows[0], rows[1], ...
 * had been touched first, in that order (the _topology_storePathInCache rule
 * keeps the first stored direction of a pair).  Used to check a sampled
 * subset of a table too large for preload_table (C4: 86k x 86k). */
int orc_topology_preload_rows(OrcTopo* t, const int* rows, int nrows, const int* cols, int ncols, const double* lat,
                              const double* rel) {
    for (int i = 0; i < nrows; i++)
        for (int j = 0; j < ncols; j++)
            if (rows[i] != cols[j]) /* self paths: first (X, X) lookup only */
                cache_store(t, 0, rows[i], cols[j], lat[(size_t)i * ncols + j], rel[(size_t)i * ncols + j]);
    return 0;
}

/* ======================================================================= */
/* event order: utility/priority_queue.c:91-175 with event_compare          */
/* (core/work/event.c:109-152; host_compare host.c:407-413 = id order)      */
/* ======================================================================= */

static int ev_cmp(const OrcEvKey* a, const OrcEvKey* b) {
    if (a->time != b->time) return a->time > b->time ? 1 : -1;
    if (a->dst != b->dst) return a->dst > b->dst ? 1 : -1;
    if (a->src != b->src) return a->src > b->src ? 1 : -1;
    if (a->seq != b->seq) return a->seq > b->seq ? 1 : -1;
    return 0;
}

typedef struct {
    uint32_t* heap; /* indices into keys */
    size_t size, cap;
    const OrcEvKey* keys;
} Pq;

static int pq_smaller(Pq* q, size_t i, size_t j) { return ev_cmp(&q->keys[q->heap[i]], &q->keys[q->heap[j]]) < 0; }

static void pq_swap(Pq* q, size_t i, size_t j) {
    uint32_t x = q->heap[i];
    q->heap[i] = q->heap[j];
    q->heap[j] = x;
}

static void pq_push(Pq* q, uint32_t idx) {
    if (q->size == q->cap) {
        q->cap = q->cap ? q->cap * 2 : 100;
        q->heap = (uint32_t*)realloc(q->heap, sizeof(uint32_t) * q->cap);
    }
    size_t i = q->size++;
    q->heap[i] = idx;
    while (i > 0 && pq_smaller(q, i, (i - 1) / 2)) {
        pq_swap(q, i, (i - 1) / 2);
        i = (i - 1) / 2;
    }
}

static uint32_t pq_pop(Pq* q) {
    uint32_t top = q->heap[0];
    pq_swap(q, 0, q->size - 1);
    q->size--;
    size_t i = 0, c;
    while ((c = 2 * i + 1) < q->size) {
        if (c + 1 < q->size && pq_smaller(q, c + 1, c)) c = c + 1;
        if (pq_smaller(q, c, i)) {
            pq_swap(q, i, c);
            i = c;
        } else break;
    }
    return top;
}

void orc_pq_order(const OrcEvKey* keys, size_t n, uint32_t* order) {
    Pq q = {NULL, 0, 0, keys};
    for (size_t i = 0; i < n; i++) pq_push(&q, (uint32_t)i);
    for (size_t i = 0; i < n; i++) order[i] = pq_pop(&q);
    free(q.heap);
}

/* ======================================================================= */
/* packet hand-off: worker_sendPacket (worker.c:517-576) -> scheduler_push  */
/* (scheduler.c:232-255) -> host-single push (policy_host_single.c:174-220) */
/* ======================================================================= */

size_t orc_round(OrcTopo* t, const uint32_t* host_ips, uint32_t nhosts, uint64_t barrier, uint64_t end_time,
                 uint64_t bootstrap_end, const OrcPkt* pkts, size_t n, OrcDeliv* out, uint8_t* status,
                 uint64_t* min_time) {
    OrcEvKey* keys = (OrcEvKey*)malloc(sizeof(OrcEvKey) * (n ? n : 1));
    Pq* qs = (Pq*)calloc(nhosts ? nhosts : 1, sizeof(Pq));
    for (uint32_t h = 0; h < nhosts; h++) qs[h].keys = keys;
    uint64_t mn = UINT64_MAX;
    for (size_t i = 0; i < n; i++) {
        const OrcPkt* p = &pkts[i];
        uint32_t sip = host_ips[p->src_host], dip = host_ips[p->dst_host];
        int boot = p->now < bootstrap_end;
        double rel = orc_topology_get_reliability(t, sip, dip);
        uint32_t st = p->rng_state;
        double chance = orc_next_double(&st);
        if (boot || chance <= rel || p->payload_len == 0) {
            double lat = orc_topology_get_latency(t, sip, dip);
            uint64_t delay = (uint64_t)ceil(lat * 1000000.0);
            uint64_t tm = p->now + delay;
            orc_topology_increment_path_packet_counter(t, sip, dip);
            if (tm >= end_time) {
                status[i] = ORC_DROP_END;
                continue;
            }
            if (p->src_host != p->dst_host && tm < barrier) tm = barrier;
            keys[i] = (OrcEvKey){tm, p->dst_host, p->src_host, p->seq};
            pq_push(&qs[p->dst_host], (uint32_t)i);
            if (tm >= barrier && tm < mn) mn = tm; /* worker.c:350-363 */
            status[i] = ORC_DELIVERED;
        } else {
            status[i] = ORC_DROP_LOSS;
        }
    }
    size_t k = 0;
    for (uint32_t h = 0; h < nhosts; h++) {
        while (qs[h].size) {
            uint32_t i = pq_pop(&qs[h]);
            out[k++] = (OrcDeliv){keys[i].time, keys[i].seq, keys[i].src, keys[i].dst, i, 0};
        }
        free(qs[h].heap);
    }
    free(qs);
    free(keys);
    if (min_time) *min_time = mn;
    return k;
}

/* ======================================================================= */
/* the hand-off on N threads (CPU baseline of SURVEY.md §8d C3): Shadow's   */
/* worker pool with the host-single policy -- each worker sends its own     */
/* hosts' packets (sharded by source) and pushes into the destination's     */
/* queue under that queue's mutex (scheduler_policy_host_single.c:207-219). */
/* Needs every row the packets touch already cached (preload): lookups are */
/* then read-only; the path counter increment is atomic.  Output identical  */
/* to orc_round (event_compare is a total order).                           */
/* ======================================================================= */
#include <pthread.h>

typedef struct {
    OrcTopo* t;
    const uint32_t* host_ips;
    uint32_t nhosts;
    uint64_t barrier, end_time, bootstrap_end;
    const OrcPkt* pkts;
    size_t n;
    uint8_t* status;
    OrcEvKey* keys;
    Pq* qs;
    pthread_mutex_t* qlock;
    int nthreads;
    size_t* qoff;
    OrcDeliv* out;
    pthread_mutex_t miss_mu; /* a missing path (a first self path) is computed serially */
} RoundMt;

typedef struct {
    RoundMt* r;
    int tid;
    uint64_t mn;
    int missing;
} RoundMtArg;

static PathE* cached_entry(OrcTopo* t, uint32_t sip, uint32_t dip) {
    int s = orc_vertex_of_ip(t, sip), d = orc_vertex_of_ip(t, dip);
    if (s < 0 || d < 0) return NULL;
    PathE* p = cache_get(t, s, d);
    if (!p && !t->directed) p = cache_get(t, d, s);
    if (!p) p = cache_get(t, d, s); /* the re-read after a (here: no-op) row computation, topology.c:1963-1968 */
    return p;
}

static void* round_mt_send(void* arg) {
    RoundMtArg* a = (RoundMtArg*)arg;
    RoundMt* r = a->r;
    uint64_t mn = UINT64_MAX;
    for (size_t i = 0; i < r->n; i++) {
        const OrcPkt* p = &r->pkts[i];
        if ((int)(p->src_host % (uint32_t)r->nthreads) != a->tid) continue; /* this worker's hosts */
        PathE* e = cached_entry(r->t, r->host_ips[p->src_host], r->host_ips[p->dst_host]);
        if (!e) { /* the reference's lookup (its writer lock): first (X, X) lookups */
            pthread_mutex_lock(&r->miss_mu);
            e = get_path_entry(r->t, r->host_ips[p->src_host], r->host_ips[p->dst_host]);
            pthread_mutex_unlock(&r->miss_mu);
        }
        if (!e) {
            a->missing++;
            continue;
        }
        uint32_t st = p->rng_state;
        double chance = orc_next_double(&st);
        if (p->now < r->bootstrap_end || chance <= e->rel || p->payload_len == 0) {
            uint64_t tm = p->now + (uint64_t)ceil(e->lat * 1000000.0);
            __atomic_fetch_add(&e->pkts, 1, __ATOMIC_RELAXED);
            if (tm >= r->end_time) {
                r->status[i] = ORC_DROP_END;
                continue;
            }
            if (p->src_host != p->dst_host && tm < r->barrier) tm = r->barrier;
            r->keys[i] = (OrcEvKey){tm, p->dst_host, p->src_host, p->seq};
            pthread_mutex_lock(&r->qlock[p->dst_host]);
            pq_push(&r->qs[p->dst_host], (uint32_t)i);
            pthread_mutex_unlock(&r->qlock[p->dst_host]);
            if (tm >= r->barrier && tm < mn) mn = tm;
            r->status[i] = ORC_DELIVERED;
        } else {
            r->status[i] = ORC_DROP_LOSS;
        }
    }
    a->mn = mn;
    return NULL;
}

static void* round_mt_pop(void* arg) {
    RoundMtArg* a = (RoundMtArg*)arg;
    RoundMt* r = a->r;
    for (uint32_t h = (uint32_t)a->tid; h < r->nhosts; h += (uint32_t)r->nthreads) {
        size_t k = r->qoff[h];
        while (r->qs[h].size) {
            uint32_t i = pq_pop(&r->qs[h]);
            r->out[k++] = (OrcDeliv){r->keys[i].time, r->keys[i].seq, r->keys[i].src, r->keys[i].dst, i, 0};
        }
        free(r->qs[h].heap);
    }
    return NULL;
}

/* Returns the number of delivered events, or (size_t)-1 if a packet's path
 * cannot be resolved.  Paths are expected to be preloaded; a missing one (a
 * first self path: rows never store their own vertex) is computed by the
 * serial lookup under miss_mu, as the reference's writer lock would. */
size_t orc_round_mt(OrcTopo* t, const uint32_t* host_ips, uint32_t nhosts, uint64_t barrier, uint64_t end_time,
                    uint64_t bootstrap_end, const OrcPkt* pkts, size_t n, int nthreads, OrcDeliv* out,
                    uint8_t* status, uint64_t* min_time) {
    if (nthreads < 1) nthreads = 1;
    RoundMt r = {t, host_ips, nhosts, barrier, end_time, bootstrap_end, pkts, n, status, NULL, NULL, NULL, nthreads,
                 NULL, out, PTHREAD_MUTEX_INITIALIZER};
    r.keys = (OrcEvKey*)malloc(sizeof(OrcEvKey) * (n ? n : 1));
    r.qs = (Pq*)calloc(nhosts ? nhosts : 1, sizeof(Pq));
    r.qlock = (pthread_mutex_t*)malloc(sizeof(pthread_mutex_t) * (nhosts ? nhosts : 1));
    r.qoff = (size_t*)malloc(sizeof(size_t) * ((size_t)nhosts + 1));
    for (uint32_t h = 0; h < nhosts; h++) {
        r.qs[h].keys = r.keys;
        pthread_mutex_init(&r.qlock[h], NULL);
    }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    RoundMtArg* args = (RoundMtArg*)calloc((size_t)nthreads, sizeof(RoundMtArg));
    for (int i = 0; i < nthreads; i++) {
        args[i].r = &r;
        args[i].tid = i;
        pthread_create(&th[i], NULL, round_mt_send, &args[i]);
    }
    uint64_t mn = UINT64_MAX;
    int missing = 0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        if (args[i].mn < mn) mn = args[i].mn;
        missing += args[i].missing;
    }
    size_t k = 0;
    for (uint32_t h = 0; h < nhosts; h++) {
        r.qoff[h] = k;
        k += r.qs[h].size;
    }
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, round_mt_pop, &args[i]);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    for (uint32_t h = 0; h < nhosts; h++) pthread_mutex_destroy(&r.qlock[h]);
    free(th);
    free(args);
    free(r.qlock);
    free(r.qoff);
    free(r.qs);
    free(r.keys);
    if (min_time) *min_time = mn;
    return missing ? (size_t)-1 : k;
}

/* ---------------------------------------------------------------------------
 * Destination routers with CoDel (routing/router.c:103-131,
 * routing/router_queue_codel.c:113-265).  The router state and the entries
 * still queued travel in the same records as libshdnet's (a ring per router:
 * `head`, `len` index `rings + r * ring_cap`) so that a round can resume from
 * either implementation; inside, each router's queue is a plain FIFO array
 * with a read cursor (g_queue_push_tail / g_queue_pop_head). */

#define ORC_CODEL_TARGET (10ull * 1000000ull)    /* CODEL_PARAM_TARGET_DELAY_SIMTIME, :42 */
#define ORC_CODEL_INTERVAL (100ull * 1000000ull) /* CODEL_PARAM_INTERVAL_SIMTIME, :48 */
#define ORC_CODEL_MTU 1500ull                    /* CONFIG_MTU, core/support/definitions.h:185 */
enum { ORC_STORE = 0, ORC_DROP = 1 };

typedef struct {
    OrcCodelState* st;
    OrcCodelEntry* q; /* FIFO storage */
    size_t rd, wr, cap;
    uint64_t* fate;
    uint32_t op;
    int bad;
    uint8_t* rstat; /* interface engine: drops are recorded per packet id here */
} OrcRouter;

static void orc_codel_drop(OrcRouter* R, uint32_t pkt) { /* :138-146 */
    if (R->rstat) R->rstat[pkt] = 2;
    else R->fate[pkt] = ((uint64_t)R->op << 2) | 2u;
}

/* :148-196 */
static int64_t orc_codel_helper(OrcRouter* R, uint64_t now, int* ok) {
    *ok = 0;
    if (R->rd == R->wr) {
        R->st->interval_expire = 0;
        return -1;
    }
    OrcCodelEntry e = R->q[R->rd++];
    if (e.length > R->st->total_size) R->bad = 1; /* utility_assert(length <= totalSize) */
    R->st->total_size -= e.length;
    if (now < e.enqueue_ts) R->bad = 1; /* utility_assert(now >= ts) */
    uint64_t sojourn = now - e.enqueue_ts;
    if (sojourn < ORC_CODEL_TARGET || R->st->total_size < ORC_CODEL_MTU) {
        R->st->interval_expire = 0;
    } else if (R->st->interval_expire == 0) {
        R->st->interval_expire = now + ORC_CODEL_INTERVAL;
    } else if (now >= R->st->interval_expire) {
        *ok = 1;
    }
    return e.pkt;
}

/* :198-205 */
static uint64_t orc_codel_law(uint32_t count, uint64_t ts) {
    uint64_t nts = ts + ORC_CODEL_INTERVAL;
    double result = ((double)nts) / sqrt((double)count);
    return (uint64_t)round(result);
}

/* :207-267 */
static int64_t orc_codel_dequeue(OrcRouter* R, uint64_t now) {
    OrcCodelState* s = R->st;
    int ok = 0;
    int64_t p = orc_codel_helper(R, now, &ok);
    if (p < 0) {
        s->mode = ORC_STORE;
        return p;
    }
    if (s->mode == ORC_DROP) {
        if (!ok) s->mode = ORC_STORE;
        while (now >= s->next_drop && s->mode == ORC_DROP) {
            orc_codel_drop(R, (uint32_t)p);
            s->drop_count++;
            p = orc_codel_helper(R, now, &ok);
            if (ok)
                s->next_drop = orc_codel_law(s->drop_count, s->next_drop);
            else
                s->mode = ORC_STORE;
        }
    } else if (ok) {
        orc_codel_drop(R, (uint32_t)p);
        p = orc_codel_helper(R, now, &ok);
        s->mode = ORC_DROP;
        uint32_t delta = s->drop_count - s->drop_count_last;
        s->drop_count = 1;
        int recently = now < s->next_drop + (16 * ORC_CODEL_INTERVAL);
        if (recently && delta > 1) s->drop_count = delta;
        s->next_drop = orc_codel_law(s->drop_count, now);
        s->drop_count_last = s->drop_count;
    }
    return p;
}

int orc_codel_run(uint32_t nrouters, const uint32_t* op_offsets, const OrcCodelOp* ops, OrcCodelState* states,
                  OrcCodelEntry* rings, uint32_t ring_cap, uint32_t* deq_out, uint64_t* fate) {
    int rc = 0;
    size_t fcap = 16;
    OrcCodelEntry* fifo = malloc(fcap * sizeof *fifo);
    if (!fifo) return -3;
    for (uint32_t r = 0; r < nrouters; r++) {
        OrcCodelState* st = &states[r];
        OrcCodelEntry* ring = rings + (size_t)r * ring_cap;
        size_t need = (size_t)st->len + (op_offsets[r + 1] - op_offsets[r]);
        if (need > fcap) {
            while (fcap < need) fcap *= 2;
            free(fifo);
            fifo = malloc(fcap * sizeof *fifo);
            if (!fifo) return -3;
        }
        OrcRouter R = {st, fifo, 0, 0, fcap, fate, 0, 0, NULL};
        for (uint32_t k = 0; k < st->len; k++) fifo[R.wr++] = ring[(st->head + k) % ring_cap];
        int failed = 0;
        for (uint32_t i = op_offsets[r]; i < op_offsets[r + 1]; i++) {
            const OrcCodelOp* o = &ops[i];
            R.op = i;
            if (o->kind == 0) { /* router_enqueue (router.c:103-121) -> :113-136 */
                if (R.wr - R.rd == ring_cap) {
                    rc = -2, failed = 1;
                    break;
                }
                fifo[R.wr++] = (OrcCodelEntry){o->time, o->pkt, o->length};
                st->total_size += o->length;
                deq_out[i] = o->pkt;
            } else { /* router_dequeue (router.c:123-131) */
                int64_t p = orc_codel_dequeue(&R, o->time);
                deq_out[i] = p < 0 ? UINT32_MAX : (uint32_t)p;
                if (p >= 0) fate[p] = ((uint64_t)i << 2) | 1u;
                if (R.bad) {
                    rc = rc ? rc : -1, failed = 1;
                    break;
                }
            }
        }
        (void)failed;
        /* hand the remaining entries back in ring form: every pop advanced the head */
        uint32_t n = (uint32_t)(R.wr - R.rd);
        st->head = (uint32_t)((st->head + R.rd) % ring_cap);
        for (uint32_t k = 0; k < n; k++) ring[(st->head + k) % ring_cap] = fifo[R.rd + k];
        st->len = n;
    }
    free(fifo);
    return rc;
}

/* _topology_logAllCachedPaths (topology.c:1860-1897) at topology_free
 * (:2287), over the literal cache: "Found path <srcID><-> or -><dstID> in
 * cache: " + path_toString (path.c:62-75).  Lines in (source, destination)
 * vertex order (the reference's glib hash-table walk has no defined order). */
size_t orc_topology_log_cached_paths(OrcTopo* t, char* buf, size_t cap) {
    size_t used = 0;
    char line[512];
    for (int s = 0; s < t->V; s++) {
        if (!t->cache[s]) continue;
        for (int d = 0; d < t->V; d++) {
            PathE* p = &t->cache[s][d];
            if (!p->present) continue;
            int k = snprintf(line, sizeof line,
                             "Found path %li%s%li in cache: SourceIndex=%ld DestinationIndex=%ld Latency=%f "
                             "Reliability=%f PacketCount=%lu isDirect=%s\n",
                             (long)t->v_ids[s], t->directed ? "->" : "<->", (long)t->v_ids[d], (long)s, (long)d,
                             p->lat, p->rel, (unsigned long)p->pkts, p->is_direct ? "True" : "False");
            if (buf && used + (size_t)k < cap) memcpy(buf + used, line, (size_t)k + 1);
            used += (size_t)k;
        }
    }
    return used;
}

/* ---------------------------------------------------------------------------
 * Network interfaces (host/network_interface.c) with the upstream router,
 * as the reference runs them: a per-host event queue ordered like
 * event_compare (time, source host, then the source's event order), into
 * which the arrivals and send requests are pushed up front and refill tasks
 * are pushed when scheduled (worker_scheduleTask); each popped event runs its
 * callback.  A refill and a send request of the same host at the same time:
 * the send request first (the reference orders them by event id, which the
 * inputs do not carry -- the same assumption as libshdnet's). */

#define ORC_NIC_INTERVAL 1000000ull /* _networkinterface_getRefillInterval, :99-101 */

/* send requests that met a refill task of their host at the same nanosecond
 * in the last orc_nic_run (how often the tie assumption above decided) */
static uint64_t orc_nic_ties;
uint64_t orc_nic_tie_count(void) { return orc_nic_ties; }

typedef struct {
    uint64_t time;
    uint32_t src;
    uint32_t cls; /* 0 arrival, 1 send request, 2 refill */
    uint64_t idx; /* input order within (time, src, cls) */
} OrcNicEv;

static int orc_nicev_less(const OrcNicEv* a, const OrcNicEv* b) {
    if (a->time != b->time) return a->time < b->time;
    if (a->src != b->src) return a->src < b->src;
    if (a->cls != b->cls) return a->cls < b->cls;
    return a->idx < b->idx;
}

typedef struct {
    OrcNicEv* h;
    size_t n, cap;
} OrcNicHeap;

static int orc_nicheap_push(OrcNicHeap* H, OrcNicEv e) {
    if (H->n == H->cap) {
        size_t nc = H->cap ? H->cap * 2 : 64;
        OrcNicEv* nh = (OrcNicEv*)realloc(H->h, nc * sizeof *nh);
        if (!nh) return -1;
        H->h = nh;
        H->cap = nc;
    }
    size_t i = H->n++;
    H->h[i] = e;
    while (i && orc_nicev_less(&H->h[i], &H->h[(i - 1) / 2])) {
        OrcNicEv t = H->h[i];
        H->h[i] = H->h[(i - 1) / 2];
        H->h[(i - 1) / 2] = t;
        i = (i - 1) / 2;
    }
    return 0;
}

static OrcNicEv orc_nicheap_pop(OrcNicHeap* H) {
    OrcNicEv top = H->h[0];
    H->h[0] = H->h[--H->n];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < H->n && orc_nicev_less(&H->h[l], &H->h[m])) m = l;
        if (r < H->n && orc_nicev_less(&H->h[r], &H->h[m])) m = r;
        if (m == i) break;
        OrcNicEv t = H->h[i];
        H->h[i] = H->h[m];
        H->h[m] = t;
        i = m;
    }
    return top;
}

typedef struct {
    OrcNicState* s;
    OrcRouter R;
    OrcNicHeap* H;
    uint32_t self;
    uint64_t boot_end;
    const OrcNicSend* sends;
    size_t sq, sk; /* offered, not yet sent: [sq, sk) */
    uint64_t* stime;
    uint64_t* rtime;
    uint8_t* rstat;
    int oom;
} OrcNic;

static void orc_nic_consume(uint64_t* rem, uint64_t bytes) { /* :117-125 */
    if (bytes >= *rem) *rem = 0;
    else *rem -= bytes;
}

/* _networkinterface_scheduleNextRefillIfNeeded + scheduleNextRefill (:135-164) */
static void orc_nic_schedule(OrcNic* N, uint64_t now) {
    OrcNicState* s = N->s;
    int need = s->send_remaining < s->send_capacity || s->recv_remaining < s->recv_capacity;
    if (!need || s->refill_pending) return;
    uint64_t offset = now - s->refill_start;
    uint64_t since = offset % ORC_NIC_INTERVAL;
    s->refill_time = now + (ORC_NIC_INTERVAL - since);
    s->refill_pending = 1; /* _networkinterface_scheduleRefillTask (:127-133) */
    OrcNicEv e = {s->refill_time, N->self, 2, 0};
    if (orc_nicheap_push(N->H, e)) N->oom = 1;
}

/* networkinterface_receivePackets (:448-482) */
static void orc_nic_receive(OrcNic* N, uint64_t now) {
    int boot = now < N->boot_end;
    while (boot || N->s->recv_remaining >= ORC_CODEL_MTU) {
        int64_t p = orc_codel_dequeue(&N->R, now); /* router_dequeue (router.c:123-131) */
        if (p < 0) break;
        uint32_t len = N->R.q[N->R.rd - 1].length;
        N->rtime[p] = now;
        N->rstat[p] = 1;
        if (!boot) {
            orc_nic_consume(&N->s->recv_remaining, len);
            orc_nic_schedule(N, now);
        }
    }
}

/* _networkinterface_sendPackets (:571-631) */
static void orc_nic_send(OrcNic* N, uint64_t now) {
    int boot = now < N->boot_end;
    while (N->s->send_remaining >= ORC_CODEL_MTU) {
        if (N->sq == N->sk) break; /* no socket has a packet */
        const OrcNicSend* p = &N->sends[N->sq];
        N->stime[N->sq] = now;
        N->sq++;
        if (!boot) {
            orc_nic_consume(&N->s->send_remaining, p->length);
            orc_nic_schedule(N, now);
        }
    }
}

/* _networkinterface_refillTokenBucketsCB (:166-186) */
static void orc_nic_refill(OrcNic* N, uint64_t now) {
    OrcNicState* s = N->s;
    s->refill_pending = 0;
    s->recv_remaining += s->recv_refill; /* :108-115 */
    if (s->recv_remaining > s->recv_capacity) s->recv_remaining = s->recv_capacity;
    s->send_remaining += s->send_refill;
    if (s->send_remaining > s->send_capacity) s->send_remaining = s->send_capacity;
    orc_nic_receive(N, now);
    orc_nic_send(N, now);
    orc_nic_schedule(N, now);
}

int orc_nic_init(uint32_t n, const uint64_t* down, const uint64_t* up, uint64_t start, OrcNicState* st) {
    for (uint32_t h = 0; h < n; h++) {
        OrcNicState* s = &st[h];
        memset(s, 0, sizeof *s);
        uint64_t factor = 1000000000ull / ORC_NIC_INTERVAL; /* _networkinterface_setupTokenBuckets (:196-228) */
        s->recv_refill = down[h] * 1024 / factor;
        s->send_refill = up[h] * 1024 / factor;
        s->recv_capacity = s->recv_refill + ORC_CODEL_MTU;
        s->send_capacity = s->send_refill + ORC_CODEL_MTU;
        /* networkinterface_startRefillingTokenBuckets (:188-194) -> refillCB on empty buckets */
        s->refill_start = start;
        s->recv_remaining = s->recv_refill < s->recv_capacity ? s->recv_refill : s->recv_capacity;
        s->send_remaining = s->send_refill < s->send_capacity ? s->send_refill : s->send_capacity;
        int need = s->send_remaining < s->send_capacity || s->recv_remaining < s->recv_capacity;
        if (need) {
            s->refill_time = start + ORC_NIC_INTERVAL;
            s->refill_pending = 1;
        }
    }
    return 0;
}

int orc_nic_run(uint32_t nhosts, uint32_t host_base, const OrcDeliv* ev, const uint32_t* eoff, const uint32_t* elen,
                const OrcNicSend* sends, const uint32_t* soff, uint64_t window_end, uint64_t boot_end,
                OrcNicState* states, OrcCodelEntry* rings, uint32_t ring_cap, uint32_t id_base, uint64_t* rtime,
                uint8_t* rstat, uint64_t fate_cap, uint64_t* stime) {
    int rc = 0;
    OrcNicHeap H = {0};
    orc_nic_ties = 0;
    for (uint32_t k = eoff[0]; k < eoff[nhosts]; k++) {
        if ((uint64_t)id_base + k >= fate_cap) return -3;
        rtime[id_base + k] = UINT64_MAX;
        rstat[id_base + k] = 0;
    }
    if (soff)
        for (uint32_t k = soff[0]; k < soff[nhosts]; k++) stime[k] = UINT64_MAX;
    for (uint32_t h = 0; h < nhosts && !rc; h++) {
        OrcNicState* s = &states[h];
        const uint32_t self = host_base + h;
        size_t na = eoff[h + 1] - eoff[h], ns = soff ? soff[h + 1] - soff[h] : 0;
        size_t fcap = (size_t)s->router.len + na + 1;
        OrcCodelEntry* fifo = (OrcCodelEntry*)malloc(fcap * sizeof *fifo);
        if (!fifo) return -3;
        OrcCodelEntry* ring = rings + (size_t)h * ring_cap;
        OrcNic N;
        memset(&N, 0, sizeof N);
        N.s = s;
        N.R = (OrcRouter){(OrcCodelState*)&s->router, fifo, 0, 0, fcap, NULL, 0, 0, rstat};
        for (uint32_t k = 0; k < s->router.len; k++) fifo[N.R.wr++] = ring[(s->router.head + k) % ring_cap];
        N.H = &H;
        N.self = self;
        N.boot_end = boot_end;
        N.sends = sends;
        N.sq = N.sk = soff ? soff[h] : 0;
        N.stime = stime;
        N.rtime = rtime;
        N.rstat = rstat;
        H.n = 0;
        for (size_t k = 0; k < na; k++) {
            const OrcDeliv* d = &ev[eoff[h] + k];
            if (d->dst_host != self || d->time >= window_end) rc = -1;
            OrcNicEv e = {d->time, d->src_host, 0, k};
            if (orc_nicheap_push(&H, e)) rc = -3;
        }
        for (size_t k = 0; k < ns; k++) {
            if (sends[soff[h] + k].ready >= window_end) rc = -1;
            OrcNicEv e = {sends[soff[h] + k].ready, self, 1, k};
            if (orc_nicheap_push(&H, e)) rc = -3;
        }
        if (s->refill_pending) {
            OrcNicEv e = {s->refill_time, self, 2, 0};
            if (orc_nicheap_push(&H, e)) rc = -3;
        }
        uint64_t last = 0;
        while (!rc && H.n && H.h[0].time < window_end) {
            OrcNicEv e = orc_nicheap_pop(&H);
            if (e.cls == 0) { /* packet arrival: router_enqueue (router.c:103-121) */
                const uint32_t k = eoff[h] + (uint32_t)e.idx;
                if (e.time < last) rc = -1;
                last = e.time;
                int buffered = N.R.rd != N.R.wr; /* queueHooks->peek */
                N.R.q[N.R.wr++] = (OrcCodelEntry){ev[k].time, id_base + k, elen[k]};
                s->router.total_size += elen[k];
                if (!buffered) orc_nic_receive(&N, e.time);
            } else if (e.cls == 1) { /* networkinterface_wantsSend (:633-661) */
                /* the documented assumption decided this order iff the host's
                 * refill task is due at the very same nanosecond */
                if (H.n && H.h[0].time == e.time && H.h[0].cls == 2) orc_nic_ties++;
                N.sk = soff[h] + (size_t)e.idx + 1;
                orc_nic_send(&N, e.time);
            } else {
                orc_nic_refill(&N, e.time);
            }
            if (N.R.bad) rc = -1;
            if (N.oom) rc = -3;
        }
        /* still queued: back into the ring */
        uint32_t left = (uint32_t)(N.R.wr - N.R.rd);
        if (!rc && left > ring_cap) rc = -2;
        if (!rc) {
            s->router.head = (uint32_t)((s->router.head + (N.R.rd < s->router.len ? N.R.rd : s->router.len)) % ring_cap);
            for (uint32_t k = 0; k < left; k++) ring[(s->router.head + k) % ring_cap] = fifo[N.R.rd + k];
            s->router.len = left;
        }
        free(fifo);
    }
    free(H.h);
    return rc;
}
