/*
 * units.c -- unit-string parsing restated from the Rust the reference
 * exports to C (core/support/units.rs:777-837 parse_bandwidth /
 * parse_time_nanosec, FromStr :404-437).  Rust is not in this image, so the
 * rule is restated in C: value = regex ^([+-]?[0-9.]*)\s*(.*)$ group 1
 * trimmed, parsed as u64 (optional '+', digits only); unit = group 2
 * trimmed, mapped through the prefix table; value * factor checked in u64,
 * then checked into i64.  Any failure -> -1.
 */
#include <errno.h>
#include <string.h>

#include "shd_internal.h"

typedef struct {
    const char* name;
    uint64_t factor;
} UnitName;

/* TimePrefix::from_str (units.rs:237-256) in ns; default "" = seconds. */
static const UnitName kTime[] = {
    {"", 1000000000ull},         {"ns", 1ull},
    {"nanosecond", 1ull},        {"nanoseconds", 1ull},
    {"us", 1000ull},             {"\xce\xbcs", 1000ull},
    {"microsecond", 1000ull},    {"microseconds", 1000ull},
    {"ms", 1000000ull},          {"millisecond", 1000000ull},
    {"milliseconds", 1000000ull}, {"s", 1000000000ull},
    {"sec", 1000000000ull},      {"secs", 1000000000ull},
    {"second", 1000000000ull},   {"seconds", 1000000000ull},
    {"m", 60000000000ull},       {"min", 60000000000ull},
    {"mins", 60000000000ull},    {"minute", 60000000000ull},
    {"minutes", 60000000000ull}, {"h", 3600000000000ull},
    {"hr", 3600000000000ull},    {"hrs", 3600000000000ull},
    {"hour", 3600000000000ull},  {"hours", 3600000000000ull},
};

/* SiPrefixUpper::from_str (units.rs:159-177) in base units. */
static const UnitName kSiUpper[] = {
    {"", 1ull},
    {"K", 1000ull},
    {"kilo", 1000ull},
    {"Ki", 1024ull},
    {"kibi", 1024ull},
    {"M", 1000000ull},
    {"mega", 1000000ull},
    {"Mi", 1048576ull},
    {"mebi", 1048576ull},
    {"G", 1000000000ull},
    {"giga", 1000000000ull},
    {"Gi", 1073741824ull},
    {"gibi", 1073741824ull},
    {"T", 1000000000000ull},
    {"tera", 1000000000000ull},
    {"Ti", 1099511627776ull},
    {"tebi", 1099511627776ull},
};

static int is_ws(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

typedef struct {
    const char *v0, *v1, *u0, *u1;
} Split;

static int split(const char* s, Split* sp) {
    const char* p = s;
    sp->v0 = p;
    p += (*p == '+' || *p == '-');
    p += strspn(p, "0123456789.");
    sp->v1 = p;
    while (is_ws(*p)) p++;
    sp->u0 = p;
    sp->u1 = p + strlen(p);
    if (memchr(sp->u0, '\n', (size_t)(sp->u1 - sp->u0))) return -1; /* '.' excludes '\n' */
    while (sp->v0 < sp->v1 && is_ws(*sp->v0)) sp->v0++;
    while (sp->v1 > sp->v0 && is_ws(sp->v1[-1])) sp->v1--;
    while (sp->u0 < sp->u1 && is_ws(*sp->u0)) sp->u0++;
    while (sp->u1 > sp->u0 && is_ws(sp->u1[-1])) sp->u1--;
    return 0;
}

static int lookup(const UnitName* t, size_t n, const char* s, size_t len, uint64_t* f) {
    for (size_t i = 0; i < n; i++)
        if (strlen(t[i].name) == len && memcmp(t[i].name, s, len) == 0) {
            *f = t[i].factor;
            return 0;
        }
    return -1;
}

static int64_t scaled(const char* v0, const char* v1, uint64_t factor) {
    const char* p = v0 + (v0 < v1 && *v0 == '+');
    if (p == v1) return -1;
    uint64_t v = 0;
    for (; p < v1; p++) {
        if (*p < '0' || *p > '9') return -1;
        uint64_t d = (uint64_t)(*p - '0');
        if (v > (UINT64_MAX - d) / 10) return -1;
        v = v * 10 + d;
    }
    if (v && v > UINT64_MAX / factor) return -1;
    v *= factor;
    return v > (uint64_t)INT64_MAX ? -1 : (int64_t)v;
}

int64_t shd_units_time_ns(const char* s) {
    Split sp;
    uint64_t f;
    if (!s || split(s, &sp) || lookup(kTime, sizeof kTime / sizeof *kTime, sp.u0, (size_t)(sp.u1 - sp.u0), &f))
        return -1;
    return scaled(sp.v0, sp.v1, f);
}

int64_t shd_units_bandwidth_bits(const char* s) {
    Split sp;
    uint64_t f;
    if (!s || split(s, &sp)) return -1;
    size_t len = (size_t)(sp.u1 - sp.u0);
    /* strip the first matching suffix of ["bit", "bits"] (units.rs:427-433) */
    if (len >= 3 && memcmp(sp.u1 - 3, "bit", 3) == 0) len -= 3;
    else if (len >= 4 && memcmp(sp.u1 - 4, "bits", 4) == 0) len -= 4;
    if (lookup(kSiUpper, sizeof kSiUpper / sizeof *kSiUpper, sp.u0, len, &f)) return -1;
    return scaled(sp.v0, sp.v1, f);
}

/* C-ABI exports (include/shdnet.h): the same rules the GML loader applies. */
int shd_parse_time_ns(const char* s, uint64_t* ns) {
    const int64_t v = shd_units_time_ns(s);
    if (v < 0) return shd_fail(-EINVAL, "invalid time string");
    if (ns) *ns = (uint64_t)v;
    return 0;
}

int shd_parse_bandwidth_bits(const char* s, uint64_t* bits) {
    const int64_t v = shd_units_bandwidth_bits(s);
    if (v < 0) return shd_fail(-EINVAL, "invalid bandwidth string");
    if (bits) *bits = (uint64_t)v;
    return 0;
}
