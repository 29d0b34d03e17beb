/*
 * ws_order.c -- TEST INFRASTRUCTURE ONLY (linked into liboracle.so, never into libhrf.so).
 *
 * NOT a restatement of the reference.  This is a CPU model of the tie-exact watershed
 * formulation the GPU kernel (hiprfish_image_analysis_amd/csrc/watershed.hip) implements;
 * tests/test_oracle_golden.py checks it against the heap flood restated from skimage
 * (oracle_watershed in hrf_oracle.c, i.e. skimage.morphology.watershed as called at
 * ecoli measurement.py:113 / multispecies :154) on plateau-heavy integer images.  It
 * exists so the formulation is validated on thousands of cases without a GPU, and so
 * tie statistics of real inputs can be gathered.
 *
 * Formulation (DESIGN.md "Watershed"):
 *  - key(x) = (lambda, h): lambda = minimax flood level, h = FIFO layer inside the level
 *    (entries 0; +1 across a pixel of value lambda; +0 across a "basin" pixel whose value
 *    is below lambda, which the heap fills inside the slot of the pixel that reached it).
 *  - C(x) = in-mask labelled neighbours with the least key (the pixels that can push x).
 *  - the heap pops in the lexicographic order of str(x) = head(x) . min_{c in C(x)} str(c)
 *    (basin pixels: str = min_{c in C(x)} str(c), no head; markers: head . BOTTOM . rank).
 *  - x takes the label of its min-str candidate; candidates of different labels never
 *    share an ancestor, so the push index never matters for labels.
 *  - rank of a marker = raster index.  skimage orders equal-valued markers (all age 0)
 *    by the internal layout of its binary heap; decisions that come down to that are
 *    counted in stats[2] ("heap-layout" decisions), and then -- as libhrf floods such a tile
 *    again with skimage's heap (watershed.hip ws_heap_flood_kernel) -- the model returns the
 *    heap flood's labels (oracle_watershed).
 * stats: [0] contested pixels, [1] walk steps, [2] heap-layout decisions, [3] rounds
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* hrf_oracle.c: the heap flood restated from skimage */
void oracle_watershed(const double *img, const int32_t *markers, const uint8_t *mask, int64_t H, int64_t W,
                      int32_t *out);

typedef struct {
    int64_t *a;
    int64_t n, cap;
} ivec;

static void iv_push(ivec *v, int64_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 64;
        v->a = (int64_t *)realloc(v->a, sizeof(int64_t) * v->cap);
    }
    v->a[v->n++] = x;
}

typedef struct {
    const double *f;
    const uint8_t *mask;
    const int32_t *mk;
    int64_t H, W;
    double *lam;
    int32_t *hop;
    uint32_t *stamp; /* per group */
    uint32_t serial;
} wsctx;

static int inm(const wsctx *c, int64_t i) { return c->mask == NULL || c->mask[i]; }
static int ismarker(const wsctx *c, int64_t i) { return inm(c, i) && c->mk[i] != 0; }
static int kless(double l1, int32_t h1, double l2, int32_t h2) { return l1 < l2 || (l1 == l2 && h1 < h2); }

static int nbrs(const wsctx *c, int64_t i, int64_t *nb) {
    int64_t r = i / c->W, col = i % c->W;
    int k = 0;
    if (r > 0) nb[k++] = i - c->W;
    if (col > 0) nb[k++] = i - 1;
    if (col + 1 < c->W) nb[k++] = i + 1;
    if (r + 1 < c->H) nb[k++] = i + c->W;
    return k;
}

/* candidates of x: labelled in-mask neighbours with the least key */
static int cands(const wsctx *c, int64_t x, int64_t *out) {
    int64_t nb[4];
    int k = nbrs(c, x, nb), m = 0;
    double bl = INFINITY;
    int32_t bh = INT32_MAX;
    for (int j = 0; j < k; ++j) {
        int64_t y = nb[j];
        if (!inm(c, y) || c->lam[y] == INFINITY) continue;
        if (kless(c->lam[y], c->hop[y], bl, bh)) {
            bl = c->lam[y];
            bh = c->hop[y];
            m = 0;
        }
        if (c->lam[y] == bl && c->hop[y] == bh) out[m++] = y;
    }
    return m;
}

static int isbasin(const wsctx *c, int64_t x) { return !ismarker(c, x) && c->f[x] < c->lam[x]; }

/* replace basin members by the non-basin pixels of equal key reachable through the basin */
static void expand(wsctx *c, ivec *g, uint32_t *st, uint32_t ser) {
    ivec q = {0, 0, 0}, out = {0, 0, 0};
    for (int64_t i = 0; i < g->n; ++i) {
        int64_t x = g->a[i];
        if (st[x] == ser) continue;
        st[x] = ser;
        if (isbasin(c, x)) iv_push(&q, x);
        else iv_push(&out, x);
    }
    for (int64_t qi = 0; qi < q.n; ++qi) {
        int64_t cc[4];
        int m = cands(c, q.a[qi], cc);
        for (int j = 0; j < m; ++j) {
            int64_t y = cc[j];
            if (st[y] == ser) continue;
            st[y] = ser;
            if (isbasin(c, y)) iv_push(&q, y);
            else iv_push(&out, y);
        }
    }
    free(q.a);
    free(g->a);
    *g = out;
}

/* index (into cand[]) of the candidate the heap pops first */
static int walk(wsctx *c, const int64_t *cand, int k, int64_t *stats) {
    ivec *g = (ivec *)malloc(sizeof(ivec) * k);
    int *alive = (int *)malloc(sizeof(int) * k);
    double *ml = (double *)malloc(sizeof(double) * k);
    int32_t *mh = (int32_t *)malloc(sizeof(int32_t) * k);
    int64_t *mrank = (int64_t *)malloc(sizeof(int64_t) * k);
    for (int j = 0; j < k; ++j) {
        g[j].a = NULL;
        g[j].n = g[j].cap = 0;
        iv_push(&g[j], cand[j]);
        alive[j] = 1;
    }
    int win = -1;
    for (;;) {
        stats[1] += 1;
        double bl = INFINITY;
        int32_t bh = INT32_MAX;
        for (int j = 0; j < k; ++j) {
            if (!alive[j]) continue;
            c->serial += 1;
            expand(c, &g[j], c->stamp, c->serial);
            ml[j] = INFINITY;
            mh[j] = INT32_MAX;
            for (int64_t i = 0; i < g[j].n; ++i) {
                int64_t x = g[j].a[i];
                if (kless(c->lam[x], c->hop[x], ml[j], mh[j])) {
                    ml[j] = c->lam[x];
                    mh[j] = c->hop[x];
                }
            }
            if (kless(ml[j], mh[j], bl, bh)) {
                bl = ml[j];
                bh = mh[j];
            }
        }
        int nal = 0, last = -1;
        int anym = 0;
        for (int j = 0; j < k; ++j) {
            if (!alive[j]) continue;
            if (ml[j] != bl || mh[j] != bh) {
                alive[j] = 0;
                continue;
            }
            ivec keep = {0, 0, 0};
            mrank[j] = -1;
            for (int64_t i = 0; i < g[j].n; ++i) {
                int64_t x = g[j].a[i];
                if (c->lam[x] != bl || c->hop[x] != bh) continue;
                iv_push(&keep, x);
                if (ismarker(c, x) && (mrank[j] < 0 || x < mrank[j])) mrank[j] = x;
            }
            free(g[j].a);
            g[j] = keep;
            anym |= mrank[j] >= 0;
            ++nal;
            last = j;
        }
        if (nal == 1) {
            win = last;
            break;
        }
        if (anym) {
            int64_t best = -1;
            int nm = 0;
            int32_t l0 = 0, multi = 0;
            for (int j = 0; j < k; ++j) {
                if (!alive[j] || mrank[j] < 0) continue;
                ++nm;
                if (nm == 1) l0 = c->mk[mrank[j]];
                else if (c->mk[mrank[j]] != l0) multi = 1;
                if (best < 0 || mrank[j] < best) {
                    best = mrank[j];
                    win = j;
                }
            }
            if (nm > 1 && multi) stats[2] += 1;
            break;
        }
        /* step: union of the members' candidates */
        for (int j = 0; j < k; ++j) {
            if (!alive[j]) continue;
            c->serial += 1;
            ivec nx = {0, 0, 0};
            for (int64_t i = 0; i < g[j].n; ++i) {
                int64_t cc[4];
                int m = cands(c, g[j].a[i], cc);
                for (int t = 0; t < m; ++t) {
                    if (c->stamp[cc[t]] == c->serial) continue;
                    c->stamp[cc[t]] = c->serial;
                    iv_push(&nx, cc[t]);
                }
            }
            free(g[j].a);
            g[j] = nx;
        }
    }
    for (int j = 0; j < k; ++j) free(g[j].a);
    free(g);
    free(alive);
    free(ml);
    free(mh);
    free(mrank);
    return win;
}

/* the order model alone: the resolution's labels even where a decision came down to the heap
 * layout (stats[2] > 0), where the composed flow below -- like libhrf -- floods with the heap */
static void watershed_ordered(const double *img, const int32_t *markers, const uint8_t *mask, int64_t H, int64_t W,
                              int32_t *out, int64_t *stats, int heap_fallback);

EXPORT void oracle_watershed_ordered(const double *img, const int32_t *markers, const uint8_t *mask, int64_t H,
                                     int64_t W, int32_t *out, int64_t *stats) {
    watershed_ordered(img, markers, mask, H, W, out, stats, 1);
}

EXPORT void oracle_watershed_ordered_raw(const double *img, const int32_t *markers, const uint8_t *mask, int64_t H,
                                         int64_t W, int32_t *out, int64_t *stats) {
    watershed_ordered(img, markers, mask, H, W, out, stats, 0);
}

static void watershed_ordered(const double *img, const int32_t *markers, const uint8_t *mask, int64_t H, int64_t W,
                              int32_t *out, int64_t *stats, int heap_fallback) {
    const int64_t n = H * W;
    wsctx c = {img, mask, markers, H, W, NULL, NULL, NULL, 0};
    c.lam = (double *)malloc(sizeof(double) * n);
    c.hop = (int32_t *)malloc(sizeof(int32_t) * n);
    c.stamp = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
    int64_t *ptr = (int64_t *)malloc(sizeof(int64_t) * n); /* resolved parent, -1 = none */
    for (int j = 0; j < 4; ++j) stats[j] = 0;
    for (int64_t i = 0; i < n; ++i) {
        int m = ismarker(&c, i);
        c.lam[i] = m ? img[i] : INFINITY;
        c.hop[i] = m ? 0 : INT32_MAX;
        out[i] = m ? markers[i] : 0;
        ptr[i] = -1;
    }
    /* keys: least fixed point of the monotone rule, Gauss-Seidel sweeps both ways */
    for (int changed = 1; changed;) {
        changed = 0;
        for (int dir = 0; dir < 2; ++dir)
            for (int64_t t = 0; t < n; ++t) {
                int64_t x = dir ? n - 1 - t : t;
                if (!inm(&c, x) || ismarker(&c, x)) continue;
                int64_t cc[4];
                int m = cands(&c, x, cc);
                if (!m) continue;
                double bl = c.lam[cc[0]];
                int32_t bh = c.hop[cc[0]];
                double nl;
                int32_t nh;
                if (bl < img[x]) nl = img[x], nh = 0;
                else if (bl == img[x]) nl = bl, nh = bh + 1;
                else nl = bl, nh = bh;
                if (nl != c.lam[x] || nh != c.hop[x]) {
                    c.lam[x] = nl;
                    c.hop[x] = nh;
                    changed = 1;
                }
            }
    }
    for (;;) {
        /* labels: resolved pixels copy their parent, others the least candidate label */
        for (int64_t i = 0; i < n; ++i)
            if (!ismarker(&c, i)) out[i] = 0;
        for (int changed = 1; changed;) {
            changed = 0;
            for (int dir = 0; dir < 2; ++dir)
                for (int64_t t = 0; t < n; ++t) {
                    int64_t x = dir ? n - 1 - t : t;
                    if (!inm(&c, x) || ismarker(&c, x) || c.lam[x] == INFINITY) continue;
                    int32_t l = 0;
                    if (ptr[x] >= 0) l = out[ptr[x]];
                    else {
                        int64_t cc[4];
                        int m = cands(&c, x, cc);
                        for (int j = 0; j < m; ++j)
                            if (out[cc[j]] && (!l || out[cc[j]] < l)) l = out[cc[j]];
                    }
                    if (l != out[x]) {
                        out[x] = l;
                        changed = 1;
                    }
                }
        }
        stats[3] += 1;
        int64_t found = 0;
        for (int64_t x = 0; x < n; ++x) {
            if (!inm(&c, x) || ismarker(&c, x) || c.lam[x] == INFINITY || ptr[x] >= 0) continue;
            int64_t cc[4];
            int m = cands(&c, x, cc);
            int diff = 0;
            for (int j = 1; j < m; ++j) diff |= out[cc[j]] != out[cc[0]];
            if (!diff) continue;
            ++found;
            if (!isbasin(&c, x)) {
                ptr[x] = cc[walk(&c, cc, m, stats)];
                continue;
            }
            /* a basin component takes the label of its first-popped slot: every pixel of
             * the component points at the winner among all its equal-key non-basin
             * neighbours (one decision per component, no pointer cycles) */
            ivec comp = {0, 0, 0}, slots = {0, 0, 0};
            c.serial += 1;
            c.stamp[x] = c.serial;
            iv_push(&comp, x);
            for (int64_t qi = 0; qi < comp.n; ++qi) {
                int64_t bc[4];
                int bm = cands(&c, comp.a[qi], bc);
                for (int j = 0; j < bm; ++j) {
                    int64_t y = bc[j];
                    if (c.stamp[y] == c.serial) continue;
                    c.stamp[y] = c.serial;
                    iv_push(isbasin(&c, y) ? &comp : &slots, y);
                }
            }
            int64_t win = slots.a[walk(&c, slots.a, (int)slots.n, stats)];
            for (int64_t qi = 0; qi < comp.n; ++qi) ptr[comp.a[qi]] = win;
            free(comp.a);
            free(slots.a);
        }
        stats[0] += found;
        if (!found) break;
    }
    free(c.lam);
    free(c.hop);
    free(c.stamp);
    free(ptr);
    if (heap_fallback && stats[2] > 0) oracle_watershed(img, markers, mask, H, W, out);
}
