/*
 * scc_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU checker for the dependency-graph extension: the
 * reference has no cycle checker (its Jepsen harness runs knossos and
 * bank/set checkers, linearizable/jepsen/src/comdb2/core.clj:152-177), so
 * this is "parity unpinned by the reference": edges follow Adya's
 * definitions over a recorded history and SCCs come from Tarjan's algorithm.
 *
 * History: micro-ops (txn, key, read|write, observed writer) of committed
 * transactions; txn ids are commit order, version order of a key is the
 * commit order of its writers.
 *   ww: consecutive writers of a key          (w_i -> w_{i+1})
 *   wr: writer of the observed version -> reader
 *   rw: reader -> writer of the next version after the observed one
 * Self edges are dropped; parallel edges are merged (type bits OR-ed).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { DG_WW = 1, DG_WR = 2, DG_RW = 4 };

typedef struct kv {
    uint64_t key;
    uint32_t txn;
} kv;

static int cmp_kv(const void *a, const void *b)
{
    const kv *x = a, *y = b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    if (x->txn != y->txn) return x->txn < y->txn ? -1 : 1;
    return 0;
}

typedef struct edge {
    uint32_t src, dst;
    uint32_t type;
} edge;

static int cmp_edge(const void *a, const void *b)
{
    const edge *x = a, *y = b;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
    return 0;
}

/* Builds the deduplicated edge list.  Returns the number of edges; the
 * caller frees *src, *dst, *type with dg_free. */
size_t dg_edges(size_t nops, const uint32_t *txn, const uint64_t *key, const uint8_t *is_write,
                const int64_t *observed, uint32_t **src, uint32_t **dst, uint32_t **type)
{
    size_t nw = 0;
    for (size_t i = 0; i < nops; i++) nw += is_write[i] != 0;
    kv *w = malloc(sizeof(kv) * (nw ? nw : 1));
    size_t k = 0;
    for (size_t i = 0; i < nops; i++)
        if (is_write[i]) {
            w[k].key = key[i];
            w[k].txn = txn[i];
            k++;
        }
    qsort(w, nw, sizeof(kv), cmp_kv);
    size_t nu = 0; /* unique (key, writer) */
    for (size_t i = 0; i < nw; i++)
        if (nu == 0 || w[nu - 1].key != w[i].key || w[nu - 1].txn != w[i].txn) w[nu++] = w[i];
    size_t cap = nu + 2 * nops + 1, ne = 0;
    edge *e = malloc(sizeof(edge) * cap);
    for (size_t i = 0; i + 1 < nu; i++)
        if (w[i].key == w[i + 1].key) e[ne++] = (edge){w[i].txn, w[i + 1].txn, DG_WW};
    for (size_t i = 0; i < nops; i++) {
        if (is_write[i]) continue;
        const uint32_t r = txn[i];
        const int64_t ob = observed[i];
        if (ob >= 0 && (uint32_t)ob != r) e[ne++] = (edge){(uint32_t)ob, r, DG_WR};
        /* next writer of key[i] after version ob (ob = -1: the initial one) */
        size_t lo = 0, hi = nu;
        const kv probe = {key[i], ob < 0 ? 0 : (uint32_t)ob};
        while (lo < hi) { /* first (key, txn) > probe, or >= for the initial version */
            size_t mid = (lo + hi) / 2;
            int c = cmp_kv(&w[mid], &probe);
            if (c < 0 || (c == 0 && ob >= 0))
                lo = mid + 1;
            else
                hi = mid;
        }
        if (lo < nu && w[lo].key == key[i] && w[lo].txn != r) e[ne++] = (edge){r, w[lo].txn, DG_RW};
    }
    free(w);
    qsort(e, ne, sizeof(edge), cmp_edge);
    size_t m = 0;
    for (size_t i = 0; i < ne; i++) {
        if (m && e[m - 1].src == e[i].src && e[m - 1].dst == e[i].dst)
            e[m - 1].type |= e[i].type;
        else
            e[m++] = e[i];
    }
    *src = malloc(sizeof(uint32_t) * (m ? m : 1));
    *dst = malloc(sizeof(uint32_t) * (m ? m : 1));
    *type = malloc(sizeof(uint32_t) * (m ? m : 1));
    for (size_t i = 0; i < m; i++) {
        (*src)[i] = e[i].src;
        (*dst)[i] = e[i].dst;
        (*type)[i] = e[i].type;
    }
    free(e);
    return m;
}

void dg_free(void *p) { free(p); }

/* Iterative Tarjan over the edge list (sorted by src).  scc[v] = the
 * largest node id of v's strongly connected component. */
void dg_scc(uint32_t n, size_t ne, const uint32_t *src, const uint32_t *dst, uint32_t *scc)
{
    size_t *off = calloc((size_t)n + 1, sizeof(size_t));
    for (size_t i = 0; i < ne; i++) off[src[i] + 1]++;
    for (uint32_t v = 0; v < n; v++) off[v + 1] += off[v];
    int64_t *index = malloc(sizeof(int64_t) * (n ? n : 1));
    int64_t *low = malloc(sizeof(int64_t) * (n ? n : 1));
    uint8_t *on = calloc(n ? n : 1, 1);
    uint32_t *stack = malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t *cs_v = malloc(sizeof(uint32_t) * (n ? n : 1));
    size_t *cs_e = malloc(sizeof(size_t) * (n ? n : 1));
    for (uint32_t v = 0; v < n; v++) index[v] = -1;
    int64_t counter = 0;
    size_t sp = 0;
    for (uint32_t root = 0; root < n; root++) {
        if (index[root] >= 0) continue;
        size_t csp = 0;
        cs_v[csp] = root;
        cs_e[csp] = off[root];
        csp++;
        index[root] = low[root] = counter++;
        stack[sp++] = root;
        on[root] = 1;
        while (csp) {
            const uint32_t v = cs_v[csp - 1];
            if (cs_e[csp - 1] < off[v + 1]) {
                const uint32_t u = dst[cs_e[csp - 1]++];
                if (index[u] < 0) {
                    index[u] = low[u] = counter++;
                    stack[sp++] = u;
                    on[u] = 1;
                    cs_v[csp] = u;
                    cs_e[csp] = off[u];
                    csp++;
                } else if (on[u] && index[u] < low[v]) {
                    low[v] = index[u];
                }
                continue;
            }
            if (low[v] == index[v]) {
                size_t top = sp;
                uint32_t mx = 0;
                do {
                    const uint32_t x = stack[--top];
                    if (x > mx) mx = x;
                } while (stack[top] != v);
                while (sp > top) {
                    const uint32_t x = stack[--sp];
                    on[x] = 0;
                    scc[x] = mx;
                }
            }
            csp--;
            if (csp) {
                const uint32_t p = cs_v[csp - 1];
                if (low[v] < low[p]) low[p] = low[v];
            }
        }
    }
    free(off);
    free(index);
    free(low);
    free(on);
    free(stack);
    free(cs_v);
    free(cs_e);
}
