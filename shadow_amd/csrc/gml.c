/*
 * gml.c -- reader for the GML dialect Shadow hands to igraph_read_graph_gml
 * (routing/topology.c:326-360; format docs/network_graph_spec.md).
 *
 * Lexical rules follow igraph's GML lexer: keys [A-Za-z_][A-Za-z0-9_]*,
 * integers -?[0-9]+, reals -?[0-9]+(.[0-9]+)?([eE][+-]?[0-9]+)?, strings
 * "..." without escapes, '#' comments to end of line.  The top-level
 * "graph [...]" list yields: directed (integer, 1 = directed, default 0),
 * node and edge blocks in file order (vertex/edge index = order of
 * appearance), all other graph keys ignored.  Nested lists inside node/edge
 * blocks (e.g. graphics) are skipped, as igraph ignores composite values.
 *
 * Single pass; tokens are copied into one arena so the document owns all
 * strings.
 */
#include <ctype.h>
#include <stdlib.h>
#include <string.h>

#include "shd_internal.h"

typedef struct {
    const char* p;
    char* arena;
    size_t used;
} Lex;

static void skip_space(Lex* L) {
    for (;;) {
        while (*L->p && isspace((unsigned char)*L->p)) L->p++;
        if (*L->p != '#') return;
        while (*L->p && *L->p != '\n') L->p++;
    }
}

static const char* keep(Lex* L, const char* s, size_t n) {
    char* d = L->arena + L->used;
    memcpy(d, s, n);
    d[n] = 0;
    L->used += n + 1;
    return d;
}

static int push_kv(GmlDoc* d, GmlKV kv) {
    if (d->nkv == d->capkv) {
        d->capkv = d->capkv ? d->capkv * 2 : 1024;
        GmlKV* k = (GmlKV*)realloc(d->kvs, sizeof(GmlKV) * d->capkv);
        if (!k) return -1;
        d->kvs = k;
    }
    d->kvs[d->nkv++] = kv;
    return 0;
}

static int push_block(GmlBlock** arr, int* n, int* cap, GmlBlock b) {
    if (*n == *cap) {
        *cap = *cap ? *cap * 2 : 256;
        GmlBlock* a = (GmlBlock*)realloc(*arr, sizeof(GmlBlock) * (size_t)*cap);
        if (!a) return -1;
        *arr = a;
    }
    (*arr)[(*n)++] = b;
    return 0;
}

/* Reads one key; returns its length (0 if none). */
static size_t read_key(Lex* L, const char** k0) {
    skip_space(L);
    if (!(isalpha((unsigned char)*L->p) || *L->p == '_')) return 0;
    *k0 = L->p;
    while (isalnum((unsigned char)*L->p) || *L->p == '_') L->p++;
    return (size_t)(L->p - *k0);
}

/* Reads a scalar value into kv, or reports a list opening.
 * Returns 1 scalar, 2 list '[' consumed, -1 error. */
static int read_value(Lex* L, GmlKV* kv) {
    skip_space(L);
    const char* p = L->p;
    if (*p == '[') {
        L->p++;
        return 2;
    }
    if (*p == '"') {
        const char* e = strchr(p + 1, '"');
        if (!e) return -1;
        kv->type = GML_STR;
        kv->sval = keep(L, p + 1, (size_t)(e - p - 1));
        L->p = e + 1;
        return 1;
    }
    const char* q = p + (*p == '-');
    if (!isdigit((unsigned char)*q)) return -1;
    while (isdigit((unsigned char)*q)) q++;
    int real = 0;
    if (*q == '.' && isdigit((unsigned char)q[1])) {
        real = 1;
        q++;
        while (isdigit((unsigned char)*q)) q++;
    }
    if ((*q == 'e' || *q == 'E') &&
        (isdigit((unsigned char)q[1]) || ((q[1] == '+' || q[1] == '-') && isdigit((unsigned char)q[2])))) {
        real = 1;
        q += 2;
        while (isdigit((unsigned char)*q)) q++;
    }
    const char* tok = keep(L, p, (size_t)(q - p));
    if (real) {
        kv->type = GML_REAL;
        kv->rval = strtod(tok, NULL);
    } else {
        kv->type = GML_INT;
        kv->ival = strtoll(tok, NULL, 10);
    }
    L->p = q;
    return 1;
}

/* Skips the rest of a list whose '[' was consumed. */
static int skip_list(Lex* L) {
    for (;;) {
        skip_space(L);
        if (*L->p == ']') {
            L->p++;
            return 0;
        }
        const char* k0;
        if (!read_key(L, &k0)) return -1;
        GmlKV kv;
        int r = read_value(L, &kv);
        if (r < 0) return -1;
        if (r == 2 && skip_list(L)) return -1;
    }
}

/* Reads a node/edge block body (after '['): scalar items kept. */
static int read_block(Lex* L, GmlDoc* d, GmlBlock* b) {
    b->first = (int)d->nkv;
    b->count = 0;
    for (;;) {
        skip_space(L);
        if (*L->p == ']') {
            L->p++;
            return 0;
        }
        const char* k0;
        size_t kl = read_key(L, &k0);
        if (!kl) return -1;
        GmlKV kv = {0};
        kv.key = keep(L, k0, kl);
        int r = read_value(L, &kv);
        if (r < 0) return -1;
        if (r == 2) {
            if (skip_list(L)) return -1;
            continue;
        }
        if (push_kv(d, kv)) return -1;
        b->count++;
    }
}

static int read_graph(Lex* L, GmlDoc* d) {
    for (;;) {
        skip_space(L);
        if (*L->p == ']') {
            L->p++;
            return 0;
        }
        const char* k0;
        size_t kl = read_key(L, &k0);
        if (!kl) return -1;
        int is_node = kl == 4 && !memcmp(k0, "node", 4);
        int is_edge = kl == 4 && !memcmp(k0, "edge", 4);
        int is_dir = kl == 8 && !memcmp(k0, "directed", 8);
        GmlKV kv = {0};
        int r = read_value(L, &kv);
        if (r < 0) return -1;
        if (r == 2) {
            if (is_node || is_edge) {
                GmlBlock b;
                if (read_block(L, d, &b)) return -1;
                if (is_node ? push_block(&d->nodes, &d->nnodes, &d->capnodes, b)
                            : push_block(&d->edges, &d->nedges, &d->capedges, b))
                    return -1;
            } else if (skip_list(L)) {
                return -1;
            }
        } else if (is_node || is_edge) {
            return -1; /* 'node' / 'edge' must be lists */
        } else if (is_dir && kv.type == GML_INT) {
            d->directed = kv.ival == 1;
        }
    }
}

int shd_gml_parse(const char* text, GmlDoc* d) {
    memset(d, 0, sizeof *d);
    size_t n = strlen(text);
    d->buf = (char*)malloc(2 * n + 16);
    if (!d->buf) return -1;
    Lex L = {text, d->buf, 0};
    int found = 0;
    for (;;) {
        skip_space(&L);
        if (!*L.p) break;
        const char* k0;
        size_t kl = read_key(&L, &k0);
        if (!kl) goto bad;
        GmlKV kv = {0};
        int r = read_value(&L, &kv);
        if (r < 0) goto bad;
        if (r == 2) {
            if (!found && kl == 5 && !memcmp(k0, "graph", 5)) {
                if (read_graph(&L, d)) goto bad;
                found = 1;
            } else if (skip_list(&L)) {
                goto bad;
            }
        }
    }
    if (!found) goto bad;
    return 0;
bad:
    shd_gml_free(d);
    return -1;
}

void shd_gml_free(GmlDoc* d) {
    free(d->buf);
    free(d->kvs);
    free(d->nodes);
    free(d->edges);
    memset(d, 0, sizeof *d);
}
