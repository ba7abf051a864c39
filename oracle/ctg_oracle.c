/*
 * ctg_oracle.c -- scalar C restatement of the RAG + edge-feature semantics.
 *
 * TEST INFRASTRUCTURE ONLY (the checker and bench.py's cpu_baseline "port"
 * leg).  Written independently of the HIP product code: per-edge Welford
 * accumulation (vigra style) in a plain open-addressing hash map, qsort of
 * the keys, and an array-based restatement of vigra's
 * RangeHistogramBase::computeStandardQuantiles.  Semantics follow
 * oracle/rag_oracle.py (see its header for the reference call sites it
 * restates: graph/initial_sub_graphs.py:124-129,
 * features/block_edge_features.py:113-148, test/graph/test_graph.py:42-115,
 * test/features/test_edge_features.py:32-77).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NB 40
#define NS (NB + 2)

typedef struct {
    uint64_t u, v;
    int64_t n;
    double mean, m2;
    float mn, mx;
    int64_t hist[NS];
    int used;
} Acc;

typedef struct {
    Acc* a;
    int64_t cap, size;
} Map;

static uint64_t mix(uint64_t u, uint64_t v) {
    uint64_t h = u * 0x9E3779B97F4A7C15ull ^ (v + 0x632BE59BD9B4E019ull + (u << 6) + (u >> 2));
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return h;
}

static int map_init(Map* m, int64_t cap) {
    m->cap = 1;
    while (m->cap < cap) m->cap <<= 1;
    m->size = 0;
    m->a = (Acc*)calloc((size_t)m->cap, sizeof(Acc));
    return m->a ? 0 : -1;
}

static Acc* map_get(Map* m, uint64_t u, uint64_t v);

static int map_grow(Map* m) {
    Map n;
    if (map_init(&n, m->cap * 2)) return -1;
    for (int64_t i = 0; i < m->cap; ++i)
        if (m->a[i].used) {
            Acc* d = map_get(&n, m->a[i].u, m->a[i].v);
            *d = m->a[i];
        }
    free(m->a);
    *m = n;
    return 0;
}

static Acc* map_get(Map* m, uint64_t u, uint64_t v) {
    if ((m->size + 1) * 2 > m->cap)
        if (map_grow(m)) return NULL;
    uint64_t h = mix(u, v) & (uint64_t)(m->cap - 1);
    for (;;) {
        Acc* a = &m->a[h];
        if (!a->used) {
            memset(a, 0, sizeof(Acc));
            a->used = 1;
            a->u = u;
            a->v = v;
            a->mn = INFINITY;
            a->mx = -INFINITY;
            m->size++;
            return a;
        }
        if (a->u == u && a->v == v) return a;
        h = (h + 1) & (uint64_t)(m->cap - 1);
    }
}

static int slot_of(double x, double lo, double hi) {
    const double scale = (double)NB / (hi - lo);
    const double m = scale * (x - lo);
    int idx;
    if (m == (double)NB) idx = NB - 1;
    else if (m >= (double)NB) return NB + 1;
    else if (m <= -1.0) return 0;
    else if (m != m) return 0;
    else idx = (int)m;
    if (idx < 0) return 0;
    return idx + 1;
}

static void add_sample(Acc* a, float x, double lo, double hi) {
    const double d = (double)x;
    a->n += 1;
    const double delta = d - a->mean;
    a->mean += delta / (double)a->n;
    a->m2 += delta * (d - a->mean);
    if (x < a->mn) a->mn = x;
    if (x > a->mx) a->mx = x;
    a->hist[slot_of(d, lo, hi)] += 1;
}

/* vigra computeStandardQuantiles, arrays of keypoints as in the original */
static void quantiles(const int64_t* h, double mn, double mx, double count, double lo, double hi, double* res) {
    static const double Q[7] = {0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0};
    double kp[2 * NB + 8], ch[2 * NB + 8];
    int n = 0;
    const double scale = (double)NB / (hi - lo), inv = 1.0 / scale;
    for (int i = 0; i < 7; ++i) res[i] = 0.0;
    if (count == 0.0) return;
    kp[n] = scale * (mn - lo);
    ch[n++] = 0.0;
    const double left = (double)h[0], right = (double)h[NS - 1];
    if (left > 0.0) {
        kp[n] = 0.0;
        ch[n++] = left;
    }
    double cum = left;
    for (int k = 0; k < NB; ++k) {
        if (h[k + 1] > 0) {
            if (kp[n - 1] <= (double)k) {
                kp[n] = (double)k;
                ch[n++] = cum;
            }
            cum += (double)h[k + 1];
            kp[n] = (double)(k + 1);
            ch[n++] = cum;
        }
    }
    if (right > 0.0) {
        if (kp[n - 1] != (double)NB) {
            kp[n] = (double)NB;
            ch[n++] = cum;
        }
        kp[n] = scale * (mx - lo);
        ch[n++] = count;
    } else {
        kp[n - 1] = scale * (mx - lo);
        ch[n - 1] = count;
    }
    int q = 0, end = 7;
    res[0] = mn;
    q = 1;
    res[6] = mx;
    end = 6;
    int p = 0;
    double qc = count * Q[q];
    while (q < end && p + 1 < n) {
        if (ch[p] < qc && ch[p + 1] >= qc) {
            const double t = (qc - ch[p]) / (ch[p + 1] - ch[p]) * (kp[p + 1] - kp[p]);
            res[q] = inv * (t + kp[p]) + lo;
            ++q;
            qc = count * Q[q];
        } else {
            ++p;
        }
    }
}

static int cmp_acc(const void* a, const void* b) {
    const Acc* x = *(const Acc* const*)a;
    const Acc* y = *(const Acc* const*)b;
    if (x->u != y->u) return x->u < y->u ? -1 : 1;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;
    return 0;
}

typedef struct {
    int64_t n_edges;
    uint64_t* edges;   /* 2E */
    double* feats;     /* 10E */
} OracleResult;

/*
 * mode 0: graph only, 1: boundary map (both voxel values per face),
 * 2: affinities (C,Z,Y,X) with offsets (sample aff[c,p] if (L[p],L[p+o]) is a
 * RAG edge).  own_begin: faces / samples whose owning voxel (upper voxel of a
 * face; p of an affinity sample) lies in [own_begin, shape).
 */
int ctgo_features(const uint64_t* L, const float* D, int mode, int n_ch, const int32_t* off,
                  int64_t Z, int64_t Y, int64_t X, const int64_t* own, int ignore_label, double lo,
                  double hi, int64_t* n_edges_out, uint64_t** edges_out, double** feats_out) {
    Map m;
    if (map_init(&m, 1 << 12)) return -1;
    const int64_t sz = Y * X;
    const int64_t oz = own ? own[0] : 0, oy = own ? own[1] : 0, ox = own ? own[2] : 0;
    for (int64_t z = 0; z < Z; ++z)
        for (int64_t y = 0; y < Y; ++y)
            for (int64_t x = 0; x < X; ++x) {
                const int64_t i = z * sz + y * X + x;
                const uint64_t lp = L[i];
                for (int a = 0; a < 3; ++a) {
                    const int64_t qz = z + (a == 0), qy = y + (a == 1), qx = x + (a == 2);
                    if (qz >= Z || qy >= Y || qx >= X) continue;
                    if (qz < oz || qy < oy || qx < ox) continue;
                    const int64_t j = qz * sz + qy * X + qx;
                    const uint64_t lq = L[j];
                    if (lp == lq) continue;
                    if (ignore_label && (lp == 0 || lq == 0)) continue;
                    const uint64_t u = lp < lq ? lp : lq, v = lp < lq ? lq : lp;
                    Acc* acc = map_get(&m, u, v);
                    if (!acc) return -1;
                    if (mode == 1) {
                        add_sample(acc, D[i], lo, hi);
                        add_sample(acc, D[j], lo, hi);
                    }
                }
            }
    if (mode == 2) {
        const int64_t V = Z * sz;
        for (int c = 0; c < n_ch; ++c) {
            const int dz = off[3 * c], dy = off[3 * c + 1], dx = off[3 * c + 2];
            for (int64_t z = oz; z < Z; ++z)
                for (int64_t y = oy; y < Y; ++y)
                    for (int64_t x = ox; x < X; ++x) {
                        const int64_t qz = z + dz, qy = y + dy, qx = x + dx;
                        if (qz < 0 || qz >= Z || qy < 0 || qy >= Y || qx < 0 || qx >= X) continue;
                        const int64_t i = z * sz + y * X + x;
                        const uint64_t lp = L[i], lq = L[qz * sz + qy * X + qx];
                        if (lp == lq) continue;
                        if (ignore_label && (lp == 0 || lq == 0)) continue;
                        const uint64_t u = lp < lq ? lp : lq, v = lp < lq ? lq : lp;
                        /* only RAG edges receive samples: lookup without insert */
                        uint64_t h = mix(u, v) & (uint64_t)(m.cap - 1);
                        Acc* hit = NULL;
                        for (;;) {
                            Acc* e = &m.a[h];
                            if (!e->used) break;
                            if (e->u == u && e->v == v) {
                                hit = e;
                                break;
                            }
                            h = (h + 1) & (uint64_t)(m.cap - 1);
                        }
                        if (hit) add_sample(hit, D[(int64_t)c * V + i], lo, hi);
                    }
        }
    }
    const int64_t E = m.size;
    Acc** list = (Acc**)malloc(sizeof(Acc*) * (size_t)(E ? E : 1));
    int64_t k = 0;
    for (int64_t i = 0; i < m.cap; ++i)
        if (m.a[i].used) list[k++] = &m.a[i];
    qsort(list, (size_t)E, sizeof(Acc*), cmp_acc);
    uint64_t* edges = (uint64_t*)malloc(sizeof(uint64_t) * 2 * (size_t)(E ? E : 1));
    double* feats = (double*)calloc((size_t)(E ? E : 1) * 10, sizeof(double));
    for (int64_t e = 0; e < E; ++e) {
        const Acc* a = list[e];
        edges[2 * e] = a->u;
        edges[2 * e + 1] = a->v;
        if (mode == 0 || a->n == 0) continue;
        double q[7];
        quantiles(a->hist, (double)a->mn, (double)a->mx, (double)a->n, lo, hi, q);
        double* f = feats + 10 * e;
        f[0] = a->mean;
        f[1] = a->m2 / (double)a->n;
        for (int j = 0; j < 7; ++j) f[2 + j] = q[j];
        f[9] = (double)a->n;
    }
    free(list);
    free(m.a);
    *n_edges_out = E;
    *edges_out = edges;
    *feats_out = feats;
    return 0;
}

void ctgo_free(void* p) { free(p); }
