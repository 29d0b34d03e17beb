/*
 * kmeans_sk.c -- TEST INFRASTRUCTURE ONLY (linked into liboracle.so, never into libhrf.so).
 *
 * a8 1-D KMeans: sklearn KMeans(n_clusters=k, random_state=0, n_init=10).fit_predict(
 * x.reshape(-1, 1)) as the reference calls it (ecoli measurement.py:73, :85; multispecies
 * :125, :141), restated from sklearn 1.7.2 (sklearn/cluster/_kmeans.py: KMeans.fit,
 * _kmeans_plusplus, _kmeans_single_lloyd, _relocate_empty_clusters_dense; the 2019 defaults
 * n_init=10, algorithm "lloyd") with its random stream supplied by the caller from
 * numpy.random.RandomState(0) (oracle.py kmeans_sk):
 *
 *  - run r of n_init: first centre = the choice(n, p=1/n) sample (`first[r]`, a rank among
 *    the valid values in raster order); then for each further centre, n_local_trials =
 *    2 + int(log k) candidates: trial t draws u (`draws`), the candidate is the first sample
 *    whose cumulative closest-squared-distance reaches u * (total potential); the candidate
 *    leaving the least potential wins (first on ties);
 *  - Lloyd from those centres: labels = argmin_j (x - c_j)^2 (first minimum, sklearn's centre
 *    order); centres = cluster means; an empty cluster takes the sample farthest from its
 *    centre (its sum/count move, its label does not); stop when the labels repeat (strict
 *    convergence) or the summed squared centre shift is <= tol = 1e-4 * var(x); without
 *    strict convergence the labels are recomputed from the final centres; max_iter 300;
 *  - the run with the least inertia wins (strictly less and a different partition).
 *
 * Where sklearn's result depends on floating-point summation order (BLAS dot products,
 * OpenMP chunked sums) this restatement uses exact integer sums, so its decisions equal
 * sklearn's except when sklearn's own rounding decides (a uniform draw within ~1e-16 of a
 * cumulative boundary, a sample exactly at a midpoint): squared distances d = fl(x - c)^2
 * enter the potentials as floor(d * 2^S) in 128-bit sums (S fixed by the data range, the
 * resolution is 2^-61 of the largest squared distance), values enter the centre sums as
 * llrint(x * 2^s) int64 (as before), and tol / inertia are formed in f64 from those exact
 * sums.  Ties between equally distant samples in the relocation are broken by the lower
 * sorted position.  libhrf's kmeans.hip implements the same definition; tests pin this file
 * to sklearn 1.7.2 itself (tests/golden/kmeans_images.npz and random draws in
 * tests/test_oracle_golden.py).
 *
 * info: [0] winning run, [1] its Lloyd iterations, [2] strict convergence of the winner,
 *       [3] empty-cluster relocations over all runs
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

typedef unsigned __int128 u128;

int oracle_kmeans_scale(double amax, int64_t n);

/* squared distance in fixed point: floor(fl((x - c)^2) * 2^S) */
static uint64_t qd(double x, double c, int S) {
    const double d = x - c;
    return (uint64_t)ldexp(d * d, S);
}

/* ceil(m * T / 2^53), m < 2^53, T < 2^100: exact (192-bit intermediate) */
static u128 thr_of(uint64_t m, u128 T) {
    const uint64_t tl = (uint64_t)T, th = (uint64_t)(T >> 64);
    const u128 a = (u128)m * tl;              /* < 2^117 */
    const u128 b = (u128)m * th;              /* < 2^89 */
    /* P = b * 2^64 + a; want ceil(P / 2^53) */
    const u128 lo = (a & (((u128)1 << 53) - 1));
    const u128 q = (a >> 53) + (b << 11);
    return q + (lo != 0);
}

typedef struct {
    int64_t n;           /* valid samples */
    const double *v;     /* valid values, raster order */
    int S, s;            /* potential / value fixed-point scales */
} kdata;

/* assignment with centres in sklearn order: first minimum */
static int assign(double x, const double *c, int k) {
    int bj = 0;
    double bd = (x - c[0]) * (x - c[0]);
    for (int j = 1; j < k; ++j) {
        const double d = (x - c[j]) * (x - c[j]);
        if (d < bd) {
            bd = d;
            bj = j;
        }
    }
    return bj;
}

/* one run; returns inertia, fills lab (n), cen (k); iters / strict / relocations out */
static double run_one(const kdata *D, int k, int64_t first, const double *u, int nt, int max_iter, double tol,
                      int32_t *lab, double *cen, int *iters, int *strict, int *reloc) {
    const int64_t n = D->n;
    const double *v = D->v;
    /* ---- k-means++ ---- */
    uint64_t *cl = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    cen[0] = v[first];
    u128 T = 0;
    for (int64_t i = 0; i < n; ++i) {
        cl[i] = qd(v[i], cen[0], D->S);
        T += cl[i];
    }
    for (int c = 1; c < k; ++c) {
        double best_v = 0;
        u128 best_P = 0;
        int have = 0;
        for (int t = 0; t < nt; ++t) {
            const uint64_t m = (uint64_t)ldexp(u[(c - 1) * nt + t], 53);
            const u128 thr = thr_of(m, T);
            u128 acc = 0;
            int64_t ci = n - 1;
            for (int64_t i = 0; i < n; ++i) {
                acc += cl[i];
                if (acc >= thr) {
                    ci = i;
                    break;
                }
            }
            const double cv = v[ci];
            u128 P = 0;
            for (int64_t i = 0; i < n; ++i) {
                const uint64_t d = qd(v[i], cv, D->S);
                P += d < cl[i] ? d : cl[i];
            }
            if (!have || P < best_P) {
                have = 1;
                best_P = P;
                best_v = cv;
            }
        }
        cen[c] = best_v;
        for (int64_t i = 0; i < n; ++i) {
            const uint64_t d = qd(v[i], best_v, D->S);
            if (d < cl[i]) cl[i] = d;
        }
        T = best_P;
    }
    free(cl);
    /* ---- Lloyd ---- */
    int32_t *old = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    for (int64_t i = 0; i < n; ++i) old[i] = -1;
    int64_t sum[8], cnt[8];
    double nc[8];
    *strict = 0;
    int it;
    for (it = 0; it < max_iter; ++it) {
        memset(sum, 0, sizeof sum);
        memset(cnt, 0, sizeof cnt);
        for (int64_t i = 0; i < n; ++i) {
            const int j = assign(v[i], cen, k);
            lab[i] = j;
            sum[j] += llrint(ldexp(v[i], D->s));
            cnt[j] += 1;
        }
        /* empty clusters take the samples farthest from their (old) centres */
        int nempty = 0;
        for (int j = 0; j < k; ++j) nempty += cnt[j] == 0;
        if (nempty) {
            *reloc += nempty;
            /* farthest first; ties -> lower sorted position (raster order here is not sorted:
             * sort key = (distance desc, value asc, raster asc)) */
            int64_t pick[8];
            int np = 0;
            for (int e = 0; e < nempty; ++e) {
                int64_t bi = -1;
                double bd = -1;
                for (int64_t i = 0; i < n; ++i) {
                    int taken = 0;
                    for (int q = 0; q < np; ++q) taken |= pick[q] == i;
                    if (taken) continue;
                    const double d = (v[i] - cen[lab[i]]) * (v[i] - cen[lab[i]]);
                    if (d > bd || (d == bd && (v[i] < v[bi] || (v[i] == v[bi] && i < bi)))) {
                        bd = d;
                        bi = i;
                    }
                }
                pick[np++] = bi;
            }
            int q = 0;
            for (int j = 0; j < k; ++j) {
                if (cnt[j]) continue;
                const int64_t fi = pick[q++];
                const long long fq = llrint(ldexp(v[fi], D->s));
                sum[lab[fi]] -= fq;
                cnt[lab[fi]] -= 1;
                sum[j] = fq;
                cnt[j] = 1;
            }
        }
        double shift = 0;
        for (int j = 0; j < k; ++j) {
            nc[j] = cnt[j] ? ldexp((double)sum[j] / (double)cnt[j], -D->s) : cen[j];
            const double d = nc[j] - cen[j];
            shift += d * d;
        }
        for (int j = 0; j < k; ++j) cen[j] = nc[j];
        int same = 1;
        for (int64_t i = 0; i < n && same; ++i) same = lab[i] == old[i];
        if (same) {
            *strict = 1;
            break;
        }
        if (shift <= tol) break;
        memcpy(old, lab, sizeof(int32_t) * (size_t)n);
    }
    *iters = it < max_iter ? it + 1 : max_iter;
    if (!*strict)
        for (int64_t i = 0; i < n; ++i) lab[i] = assign(v[i], cen, k);
    /* inertia from exact per-cluster sums of q and q^2 */
    int64_t s1[8] = {0};
    u128 s2[8] = {0};
    int64_t nn[8] = {0};
    for (int64_t i = 0; i < n; ++i) {
        const long long q = llrint(ldexp(v[i], D->s));
        s1[lab[i]] += q;
        s2[lab[i]] += (u128)((__int128)q * q);
        nn[lab[i]] += 1;
    }
    double I = 0;
    for (int j = 0; j < k; ++j) {
        if (!nn[j]) continue;
        const double cs = ldexp(cen[j], D->s);
        I += ((double)s2[j] - 2.0 * cs * (double)s1[j]) + (double)nn[j] * cs * cs;
    }
    free(old);
    return ldexp(I, -2 * D->s);
}

static int same_partition(const int32_t *a, const int32_t *b, int64_t n, int k) {
    int map[8];
    for (int j = 0; j < 8; ++j) map[j] = -1;
    for (int64_t i = 0; i < n; ++i) {
        if (map[a[i]] < 0) map[a[i]] = b[i];
        else if (map[a[i]] != b[i]) return 0;
    }
    (void)k;
    return 1;
}

EXPORT int oracle_kmeans_sk(const double *x, const uint8_t *valid, int64_t n, int k, int n_init, int max_iter,
                            const int64_t *first, const double *draws, int32_t *labels, double *centers,
                            int64_t *info) {
    int64_t nv = 0;
    for (int64_t i = 0; i < n; ++i) nv += !valid || valid[i];
    double *v = (double *)malloc(sizeof(double) * (size_t)(nv ? nv : 1));
    double mn = INFINITY, mx = -INFINITY, amax = 0;
    nv = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (valid && !valid[i]) continue;
        v[nv++] = x[i];
        mn = x[i] < mn ? x[i] : mn;
        mx = x[i] > mx ? x[i] : mx;
        amax = fabs(x[i]) > amax ? fabs(x[i]) : amax;
    }
    for (int j = 0; j < 4; ++j) info[j] = 0;
    if (nv == 0) {
        for (int64_t i = 0; i < n; ++i) labels[i] = -1;
        free(v);
        return 0;
    }
    kdata D;
    D.n = nv;
    D.v = v;
    D.s = oracle_kmeans_scale(amax, nv);
    const double r = mx - mn, R2 = r * r;
    int e = 0;
    frexp(R2 > 0 ? R2 : 1.0, &e);
    D.S = 61 - e;
    /* tol = 1e-4 * var(x) from exact sums */
    int64_t t1 = 0;
    u128 t2 = 0;
    for (int64_t i = 0; i < nv; ++i) {
        const long long q = llrint(ldexp(v[i], D.s));
        t1 += q;
        t2 += (u128)((__int128)q * q);
    }
    const double m1 = (double)t1 / (double)nv, m2 = (double)t2 / (double)nv;
    const double var = ldexp(m2 - m1 * m1, -2 * D.s);
    const double tol = var * 1e-4;
    const int nt = 2 + (int)log((double)k);
    int32_t *lab = (int32_t *)malloc(sizeof(int32_t) * (size_t)nv);
    int32_t *best = (int32_t *)malloc(sizeof(int32_t) * (size_t)nv);
    double cen[8], bcen[8], binert = 0;
    int have = 0, reloc = 0;
    for (int r0 = 0; r0 < n_init; ++r0) {
        int it = 0, strict = 0;
        const double I = run_one(&D, k, first[r0], draws + (size_t)r0 * (k - 1) * nt, nt, max_iter, tol, lab, cen,
                                 &it, &strict, &reloc);
        if (!have || (I < binert && !same_partition(lab, best, nv, k))) {
            have = 1;
            binert = I;
            memcpy(best, lab, sizeof(int32_t) * (size_t)nv);
            memcpy(bcen, cen, sizeof cen);
            info[0] = r0;
            info[1] = it;
            info[2] = strict;
        }
    }
    info[3] = reloc;
    nv = 0;
    for (int64_t i = 0; i < n; ++i) labels[i] = (valid && !valid[i]) ? -1 : best[nv++];
    for (int j = 0; j < k; ++j) centers[j] = bcen[j];
    free(v);
    free(lab);
    free(best);
    return 0;
}
