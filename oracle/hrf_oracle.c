/*
 * hrf_oracle.c -- CPU restatement of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (hiprfish_image_analysis_amd/,
 * libhrf.so) links, loads or calls this file.  It is the checker used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 *
 * Every function restates (does not copy) one reference algorithm; the file:line it
 * follows is cited above it.  Paths are relative to the reference repository root.
 * Pinning: tests/test_oracle_golden.py checks these functions against fixtures made
 * from the reference's own compiled Cython (oracle/build_ref.sh) and from reference
 * numpy/numba code executed in the build container (tests/golden/make_golden.py).
 *
 * Conventions: row-major arrays, int64 sizes, int32 labels, f64 arithmetic.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../hiprfish_image_analysis_amd/csrc/detmath.h"

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------
 * a5/a7  line-profile sampling tables
 * neighbor2d.pyx:32-55 (2-D), neighbor.pyx:135-169 / :209-243 (3-D, identical)
 * intervals = round-half-even(increment * direction cosines); the line of
 * 2*|max interval|+1 samples is spread over the patch with truncating division and the
 * first/last sample repeated to fill patch_size taps.
 * ---------------------------------------------------------------------------------- */
static int sgn_i(int64_t v) { return (v > 0) - (v < 0); }

static void build_line(int patch, int ndim, const int64_t *iv, int32_t *off /*[patch][ndim]*/) {
    int inc = (patch - 1) / 2;
    int arg = 0;
    for (int k = 1; k < ndim; ++k)
        if (llabs(iv[k]) > llabs(iv[arg])) arg = k;
    int64_t maxint = iv[arg];
    int line_n = (int)(2 * llabs(maxint) + 1);
    int base = 0;
    for (int i = 0; i < patch * ndim; ++i) off[i] = 0;
    if (line_n < patch) base = (patch - line_n) / 2;
    for (int li = 0; li < line_n; ++li) {
        for (int k = 0; k < ndim; ++k) {
            double h = (double)(sgn_i(iv[k]) * (int64_t)li) * (double)(2 * llabs(iv[k]) + 1) / (double)line_n;
            double t = (h > 0 ? 1.0 : (h < 0 ? -1.0 : 0.0)) * floor(fabs(h));
            off[(li + base) * ndim + k] = (int32_t)(t + (double)inc - (double)iv[k]);
        }
    }
    if (line_n < patch) {
        for (int li = 0; li < base; ++li)
            for (int k = 0; k < ndim; ++k) off[li * ndim + k] = off[base * ndim + k];
        for (int li = 0; li < base; ++li)
            for (int k = 0; k < ndim; ++k)
                off[(li + line_n + base) * ndim + k] = off[(line_n + base - 1) * ndim + k];
    }
}

/* off: [nphi][patch][2] */
EXPORT void oracle_lp_table_2d(int patch, int nphi, int32_t *off) {
    int inc = (patch - 1) / 2;
    for (int phi = 0; phi < nphi; ++phi) {
        double a = (double)phi * M_PI / (double)nphi;
        int64_t iv[2] = {(int64_t)nearbyint((double)inc * cos(a)), (int64_t)nearbyint((double)inc * sin(a))};
        build_line(patch, 2, iv, off + (int64_t)phi * patch * 2);
    }
}

/* off: [(ntheta-1)*nphi][patch][3] */
EXPORT void oracle_lp_table_3d(int patch, int ntheta, int nphi, int32_t *off) {
    int inc = (patch - 1) / 2;
    for (int th = 1; th < ntheta; ++th)
        for (int phi = 0; phi < nphi; ++phi) {
            double ap = (double)phi * M_PI / (double)nphi;
            double at = (double)th * M_PI / (double)ntheta;
            int64_t iv[3] = {(int64_t)nearbyint((double)inc * cos(ap) * sin(at)),
                             (int64_t)nearbyint((double)inc * sin(ap) * sin(at)),
                             (int64_t)nearbyint((double)inc * cos(at))};
            build_line(patch, 3, iv, off + (int64_t)((th - 1) * nphi + phi) * patch * 3);
        }
}

/* a5: neighbor2d.pyx:56-63. pad (hp,wp) -> out (hp-patch+1, wp-patch+1, nphi, patch) */
EXPORT void oracle_line_profile_2d(const double *pad, int64_t hp, int64_t wp, int patch, int nphi, double *out) {
    int32_t *off = (int32_t *)malloc(sizeof(int32_t) * nphi * patch * 2);
    oracle_lp_table_2d(patch, nphi, off);
    int64_t H = hp - (patch - 1), W = wp - (patch - 1);
    for (int64_t i = 0; i < H; ++i)
        for (int64_t j = 0; j < W; ++j)
            for (int t = 0; t < nphi; ++t)
                for (int l = 0; l < patch; ++l) {
                    const int32_t *o = off + (t * patch + l) * 2;
                    out[((i * W + j) * nphi + t) * patch + l] = pad[(i + o[0]) * wp + (j + o[1])];
                }
    free(off);
}

/* numpy's pairwise add.reduce for n >= 8 (first 8 seed the accumulators) */
static double np_pairwise_sum(const double *a, int n) {
    if (n < 8) {
        double s = a[0];
        for (int i = 1; i < n; ++i) s += a[i];
        return s;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

static int cmp_double(const void *a, const void *b) {
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

/* numpy.percentile(..., method='linear') incl. its _lerp (t >= 0.5 -> b - diff*(1-t)) */
static double np_percentile_sorted(const double *s, int n, double q) {
    double vi = q / 100.0 * (double)(n - 1);
    double lo = floor(vi);
    int il = (int)lo;
    int ih = il + 1 < n ? il + 1 : n - 1;
    double t = vi - lo;
    double a = s[il], b = s[ih];
    double d = b - a;
    return t >= 0.5 ? b - d * (1.0 - t) : a + d * t;
}

static double nan_to_num(double v) {
    if (isnan(v)) return 0.0;
    if (isinf(v)) return v > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308;
    return v;
}

/* a5+a6: multispecies_spectral_image_measurement.py:110-124 (biofilm :352-366).
 * final = mean_9(rnc) * (1 - qcv), rnc = (centre-min)/(max-min) per direction,
 * qcv = (s[6]-s[2])/(s[6]+s[2]+1e-8) only where s[6] > 0.  NaN kept (flat lines). */
EXPORT void oracle_enhance_2d(const double *pad, int64_t hp, int64_t wp, int patch, int nphi, double *final_) {
    int32_t *off = (int32_t *)malloc(sizeof(int32_t) * nphi * patch * 2);
    oracle_lp_table_2d(patch, nphi, off);
    int64_t H = hp - (patch - 1), W = wp - (patch - 1);
    int inc = (patch - 1) / 2;
    double *rnc = (double *)malloc(sizeof(double) * nphi);
    double *srt = (double *)malloc(sizeof(double) * nphi);
    for (int64_t i = 0; i < H; ++i)
        for (int64_t j = 0; j < W; ++j) {
            int anynan = 0;
            for (int t = 0; t < nphi; ++t) {
                double mn = INFINITY, mx = -INFINITY, c = 0;
                for (int l = 0; l < patch; ++l) {
                    const int32_t *o = off + (t * patch + l) * 2;
                    double v = nan_to_num(pad[(i + o[0]) * wp + (j + o[1])]);
                    mn = v < mn ? v : mn;
                    mx = v > mx ? v : mx;
                    if (l == inc) c = v;
                }
                rnc[t] = (c - mn) / (mx - mn);
                if (isnan(rnc[t])) anynan = 1;
            }
            double avg = np_pairwise_sum(rnc, nphi) / (double)nphi;
            double out;
            if (anynan) {
                out = NAN; /* np.percentile -> nan, uq>0 False -> qcv 0, avg nan */
            } else {
                memcpy(srt, rnc, sizeof(double) * nphi);
                qsort(srt, nphi, sizeof(double), cmp_double);
                double lq = np_percentile_sorted(srt, nphi, 25.0);
                double uq = np_percentile_sorted(srt, nphi, 75.0);
                double qcv = 0.0;
                if (uq > 0) qcv = (uq - lq) / (uq + lq + 1e-8);
                out = avg * (1.0 - qcv);
            }
            final_[i * W + j] = out;
        }
    free(off);
    free(rnc);
    free(srt);
}

/* a7 (unfused): neighbor.pyx:170-180 line_profile_v2 -> (X,Y,Z,ndir,patch) */
EXPORT void oracle_line_profile_3d(const double *pad, int64_t xp, int64_t yp, int64_t zp, int patch, int ntheta,
                                   int nphi, double *out) {
    int ndir = (ntheta - 1) * nphi;
    int32_t *off = (int32_t *)malloc(sizeof(int32_t) * ndir * patch * 3);
    oracle_lp_table_3d(patch, ntheta, nphi, off);
    int64_t X = xp - (patch - 1), Y = yp - (patch - 1), Z = zp - (patch - 1);
    for (int64_t i = 0; i < X; ++i)
        for (int64_t j = 0; j < Y; ++j)
            for (int64_t k = 0; k < Z; ++k)
                for (int t = 0; t < ndir; ++t)
                    for (int l = 0; l < patch; ++l) {
                        const int32_t *o = off + (t * patch + l) * 3;
                        out[(((i * Y + j) * Z + k) * ndir + t) * patch + l] =
                            pad[((i + o[0]) * yp + (j + o[1])) * zp + (k + o[2])];
                    }
    free(off);
}

/* a7: neighbor.pyx:244-262 line_profile_memory_efficient_v2 -> (X,Y,Z,ndir):
 * (centre - min) / max(max - min, 1e-8) per direction. */
static double lp3_norm(const double *pad, int64_t yp, int64_t zp, int64_t i, int64_t j, int64_t k, const int32_t *o,
                       int patch) {
    int inc = (patch - 1) / 2;
    double mn = 0, mx = 0, c = 0;
    for (int l = 0; l < patch; ++l) {
        double v = pad[((i + o[l * 3]) * yp + (j + o[l * 3 + 1])) * zp + (k + o[l * 3 + 2])];
        if (l == 0 || v < mn) mn = v;
        if (l == 0 || v > mx) mx = v;
        if (l == inc) c = v;
    }
    double r = mx - mn;
    if (1e-8 > r) r = 1e-8; /* builtin max(r, 1e-8) keeps r unless 1e-8 > r */
    return (c - mn) / r;
}

EXPORT void oracle_line_profile_3d_norm(const double *pad, int64_t xp, int64_t yp, int64_t zp, int patch, int ntheta,
                                        int nphi, double *out) {
    int ndir = (ntheta - 1) * nphi;
    int32_t *off = (int32_t *)malloc(sizeof(int32_t) * ndir * patch * 3);
    oracle_lp_table_3d(patch, ntheta, nphi, off);
    int64_t X = xp - (patch - 1), Y = yp - (patch - 1), Z = zp - (patch - 1);
    for (int64_t i = 0; i < X; ++i)
        for (int64_t j = 0; j < Y; ++j)
            for (int64_t k = 0; k < Z; ++k)
                for (int t = 0; t < ndir; ++t)
                    out[((i * Y + j) * Z + k) * ndir + t] = lp3_norm(pad, yp, zp, i, j, k, off + t * patch * 3, patch);
    free(off);
}

/* a7 fused: biofilm_analysis.py:811-817. final = mean_72 * (1 - nan_to_num((uq-lq)/(uq+lq))) */
EXPORT void oracle_enhance_3d(const double *pad, int64_t xp, int64_t yp, int64_t zp, int patch, int ntheta, int nphi,
                              double *final_) {
    int ndir = (ntheta - 1) * nphi;
    int32_t *off = (int32_t *)malloc(sizeof(int32_t) * ndir * patch * 3);
    oracle_lp_table_3d(patch, ntheta, nphi, off);
    double *v = (double *)malloc(sizeof(double) * ndir);
    double *s = (double *)malloc(sizeof(double) * ndir);
    int64_t X = xp - (patch - 1), Y = yp - (patch - 1), Z = zp - (patch - 1);
    for (int64_t i = 0; i < X; ++i)
        for (int64_t j = 0; j < Y; ++j)
            for (int64_t k = 0; k < Z; ++k) {
                for (int t = 0; t < ndir; ++t) v[t] = lp3_norm(pad, yp, zp, i, j, k, off + t * patch * 3, patch);
                double avg = np_pairwise_sum(v, ndir) / (double)ndir;
                memcpy(s, v, sizeof(double) * ndir);
                qsort(s, ndir, sizeof(double), cmp_double);
                double lq = np_percentile_sorted(s, ndir, 25.0);
                double uq = np_percentile_sorted(s, ndir, 75.0);
                double qcv = nan_to_num((uq - lq) / (uq + lq));
                final_[(i * Y + j) * Z + k] = avg * (1.0 - qcv);
            }
    free(off);
    free(v);
    free(s);
}

/* ------------------------------------------------------------------------------------
 * neighbor.line_profile_memory_efficient_v3 (neighbor.pyx:268-349).  Table (:293-311): as
 * v2 but the short-line branch rounds (np.round, half to even: no exact halves occur) and
 * the full-length branch floors s*li*(2*iv+1)/line_n with the SIGNED interval.  Per voxel:
 * the 72 min/max-normalised centre taps (range clamped to 1e-8), their mean accumulated in
 * order (:341-343), p25 and p75 (np.percentile, linear), and
 * final = mean * (p25 - p75) / (p25 + p75 + 1e-8) (:344-347: "uq" is the 25th percentile).
 * The table reaches past the patch (offsets up to 18 along x and z); the reference reads
 * image_patch[vli, vlj, vlk] unchecked, i.e. pad[(i+vli)*yp*zp + (j+vlj)*zp + (k+vlk)] as a
 * flat address (z overflow wraps into the next row), and beyond the end of the array for
 * voxels near the far x face, where its result is undefined.  Restated with the same flat
 * addressing; reads past the end of the array give 0.
 * ---------------------------------------------------------------------------------- */
static void build_line_v3(int patch, const int64_t *iv, int32_t *off /*[patch][3]*/) {
    int inc = (patch - 1) / 2;
    int arg = 0;
    for (int k = 1; k < 3; ++k)
        if (llabs(iv[k]) > llabs(iv[arg])) arg = k;
    int line_n = (int)(2 * llabs(iv[arg]) + 1);
    for (int i = 0; i < patch * 3; ++i) off[i] = 0;
    if (line_n < patch) {
        int base = (patch - line_n) / 2;
        for (int li = 0; li < line_n; ++li)
            for (int k = 0; k < 3; ++k) {
                double h = (double)(sgn_i(iv[k]) * (int64_t)li) * (double)(2 * llabs(iv[k]) + 1) / (double)line_n;
                off[(li + base) * 3 + k] = (int32_t)(nearbyint(h) + (double)inc - (double)iv[k]);
            }
        for (int li = 0; li < base; ++li)
            for (int k = 0; k < 3; ++k) off[li * 3 + k] = off[base * 3 + k];
        for (int li = 0; li < base; ++li)
            for (int k = 0; k < 3; ++k) off[(li + line_n + base) * 3 + k] = off[(line_n + base - 1) * 3 + k];
    } else {
        for (int li = 0; li < line_n; ++li)
            for (int k = 0; k < 3; ++k) {
                double h = (double)(sgn_i(iv[k]) * (int64_t)li) * (double)(2 * iv[k] + 1) / (double)line_n;
                off[li * 3 + k] = (int32_t)(floor(h) + (double)inc - (double)iv[k]);
            }
    }
}

EXPORT void oracle_lp_table_3d_v3(int patch, int ntheta, int nphi, int32_t *off) {
    int inc = (patch - 1) / 2;
    for (int th = 1; th < ntheta; ++th)
        for (int phi = 0; phi < nphi; ++phi) {
            double ap = (double)phi * M_PI / (double)nphi;
            double at = (double)th * M_PI / (double)ntheta;
            int64_t iv[3] = {(int64_t)nearbyint((double)inc * cos(ap) * sin(at)),
                             (int64_t)nearbyint((double)inc * sin(ap) * sin(at)),
                             (int64_t)nearbyint((double)inc * cos(at))};
            build_line_v3(patch, iv, off + (int64_t)((th - 1) * nphi + phi) * patch * 3);
        }
}

/* 1 where every read of voxel (i, j, k) stays inside the padded array (the defined part) */
EXPORT void oracle_v3_defined(int64_t xp, int64_t yp, int64_t zp, int patch, int ntheta, int nphi, uint8_t *ok) {
    int ndir = (ntheta - 1) * nphi;
    int32_t *off = (int32_t *)malloc(sizeof(int32_t) * ndir * patch * 3);
    oracle_lp_table_3d_v3(patch, ntheta, nphi, off);
    int64_t X = xp - (patch - 1), Y = yp - (patch - 1), Z = zp - (patch - 1), total = xp * yp * zp;
    for (int64_t i = 0; i < X; ++i)
        for (int64_t j = 0; j < Y; ++j)
            for (int64_t k = 0; k < Z; ++k) {
                int good = 1;
                for (int e = 0; e < ndir * patch && good; ++e)
                    if ((i + off[e * 3]) * yp * zp + (j + off[e * 3 + 1]) * zp + (k + off[e * 3 + 2]) >= total) good = 0;
                ok[(i * Y + j) * Z + k] = (uint8_t)good;
            }
    free(off);
}

EXPORT void oracle_enhance_3d_v3(const double *pad, int64_t xp, int64_t yp, int64_t zp, int patch, int ntheta,
                                 int nphi, double *final_) {
    int ndir = (ntheta - 1) * nphi;
    int32_t *off = (int32_t *)malloc(sizeof(int32_t) * ndir * patch * 3);
    oracle_lp_table_3d_v3(patch, ntheta, nphi, off);
    double *v = (double *)malloc(sizeof(double) * ndir);
    int64_t X = xp - (patch - 1), Y = yp - (patch - 1), Z = zp - (patch - 1);
    for (int64_t i = 0; i < X; ++i)
        for (int64_t j = 0; j < Y; ++j)
            for (int64_t k = 0; k < Z; ++k) {
                double avg = 0.0;
                const int64_t total = xp * yp * zp;
                for (int t = 0; t < ndir; ++t) {
                    const int32_t *o = off + t * patch * 3;
                    double mn = 0, mx = 0, c = 0;
                    for (int l = 0; l < patch; ++l) {
                        const int64_t a = (i + o[l * 3]) * yp * zp + (j + o[l * 3 + 1]) * zp + (k + o[l * 3 + 2]);
                        const double q = a < total ? pad[a] : 0.0;
                        if (l == 0) { mn = q; mx = q; }
                        else { mn = q < mn ? q : mn; mx = q > mx ? q : mx; }
                        if (l == (patch - 1) / 2) c = q;
                    }
                    double r = mx - mn;
                    if (1e-8 > r) r = 1e-8;
                    v[t] = (c - mn) / r;
                    avg += v[t];
                }
                avg /= (double)ndir;
                qsort(v, ndir, sizeof(double), cmp_double);
                double p25 = np_percentile_sorted(v, ndir, 25.0);
                double p75 = np_percentile_sorted(v, ndir, 75.0);
                final_[(i * Y + j) * Z + k] = avg * (p25 - p75) / (p25 + p75 + 1e-8);
            }
    free(off);
    free(v);
}

/* ------------------------------------------------------------------------------------
 * a10 connected components: skimage.measure.label / morphology.label semantics
 * (ecoli measurement.py:97-98,109,111-112; multispecies :140).  Pixels connect when both
 * are non-zero and EQUAL (label of an int image), 4- (conn=1) or 8-connectivity
 * (conn=2, skimage's default).  Labels numbered 1.. in raster order of each component's
 * first pixel (what skimage's union-find + raster relabel and scipy.ndimage.label give).
 * ---------------------------------------------------------------------------------- */
static int64_t uf_find(int64_t *p, int64_t x) {
    while (p[x] != x) {
        p[x] = p[p[x]];
        x = p[x];
    }
    return x;
}
static void uf_union(int64_t *p, int64_t a, int64_t b) {
    a = uf_find(p, a);
    b = uf_find(p, b);
    if (a < b) p[b] = a;
    else if (b < a) p[a] = b;
}

EXPORT int32_t oracle_label(const int32_t *img, int64_t H, int64_t W, int conn, int32_t *out) {
    int64_t n = H * W;
    int64_t *p = (int64_t *)malloc(sizeof(int64_t) * n);
    for (int64_t i = 0; i < n; ++i) p[i] = i;
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            int64_t i = r * W + c;
            int32_t v = img[i];
            if (!v) continue;
            if (c > 0 && img[i - 1] == v) uf_union(p, i, i - 1);
            if (r > 0) {
                if (img[i - W] == v) uf_union(p, i, i - W);
                if (conn == 2) {
                    if (c > 0 && img[i - W - 1] == v) uf_union(p, i, i - W - 1);
                    if (c + 1 < W && img[i - W + 1] == v) uf_union(p, i, i - W + 1);
                }
            }
        }
    int32_t next = 0;
    int32_t *lab = (int32_t *)calloc(n, sizeof(int32_t));
    for (int64_t i = 0; i < n; ++i) {
        if (!img[i]) {
            out[i] = 0;
            continue;
        }
        int64_t rt = uf_find(p, i);
        if (rt == i) lab[i] = ++next;
        out[i] = lab[rt];
    }
    free(p);
    free(lab);
    return next;
}

/* ------------------------------------------------------------------------------------
 * a9 binary morphology (skimage.morphology defaults, cross footprint):
 *   binary_erosion  -> ndi.binary_erosion(border_value=True)   (ecoli :107, :122)
 *   binary_dilation -> ndi.binary_dilation(border_value=False)
 *   binary_opening  = dilation(erosion)                         (ecoli :95, multispecies :136)
 * ---------------------------------------------------------------------------------- */
EXPORT void oracle_erode(const uint8_t *m, int64_t H, int64_t W, int border, uint8_t *o) {
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            int64_t i = r * W + c;
            int v = m[i] != 0;
            v = v && (r > 0 ? m[i - W] != 0 : border);
            v = v && (r + 1 < H ? m[i + W] != 0 : border);
            v = v && (c > 0 ? m[i - 1] != 0 : border);
            v = v && (c + 1 < W ? m[i + 1] != 0 : border);
            o[i] = (uint8_t)v;
        }
}
EXPORT void oracle_dilate(const uint8_t *m, int64_t H, int64_t W, uint8_t *o) {
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            int64_t i = r * W + c;
            int v = m[i] != 0;
            v = v || (r > 0 && m[i - W]) || (r + 1 < H && m[i + W]) || (c > 0 && m[i - 1]) || (c + 1 < W && m[i + 1]);
            o[i] = (uint8_t)v;
        }
}

/* remove_small_objects on a bool image: ndi.label with connectivity `conn`, drop
 * components with size < min_size (ecoli :96 min 50, :108 min 10; multispecies :137) */
EXPORT void oracle_rso_mask(const uint8_t *m, int64_t H, int64_t W, int64_t min_size, int conn, uint8_t *o) {
    int64_t n = H * W;
    int32_t *img = (int32_t *)malloc(sizeof(int32_t) * n), *lab = (int32_t *)malloc(sizeof(int32_t) * n);
    for (int64_t i = 0; i < n; ++i) img[i] = m[i] != 0;
    int32_t nl = oracle_label(img, H, W, conn, lab);
    int64_t *cnt = (int64_t *)calloc(nl + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) cnt[lab[i]]++;
    for (int64_t i = 0; i < n; ++i) o[i] = lab[i] && cnt[lab[i]] >= min_size;
    free(img);
    free(lab);
    free(cnt);
}

/* remove_small_objects on an int label image: bincount of the labels themselves
 * (ecoli :114 min 100, multispecies :155 min 60). Labels < 0 are not allowed. */
EXPORT void oracle_rso_labels(const int32_t *l, int64_t H, int64_t W, int64_t min_size, int32_t *o) {
    int64_t n = H * W;
    int32_t mx = 0;
    for (int64_t i = 0; i < n; ++i) mx = l[i] > mx ? l[i] : mx;
    int64_t *cnt = (int64_t *)calloc((size_t)mx + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) cnt[l[i]]++;
    for (int64_t i = 0; i < n; ++i) o[i] = (l[i] && cnt[l[i]] < min_size) ? 0 : l[i];
    free(cnt);
}

/* remove_small_holes(ar, area_threshold=64, connectivity=1) = ~rso(~ar) (ecoli :95) */
EXPORT void oracle_remove_small_holes(const uint8_t *m, int64_t H, int64_t W, int64_t thr, int conn, uint8_t *o) {
    int64_t n = H * W;
    uint8_t *inv = (uint8_t *)malloc(n);
    for (int64_t i = 0; i < n; ++i) inv[i] = !m[i];
    oracle_rso_mask(inv, H, W, thr, conn, o);
    for (int64_t i = 0; i < n; ++i) o[i] = !o[i];
    free(inv);
}

/* scipy.ndimage.binary_fill_holes (cross structure): background 4-components that
 * do not touch the image border are filled (multispecies :138-139). */
EXPORT void oracle_fill_holes(const uint8_t *m, int64_t H, int64_t W, uint8_t *o) {
    int64_t n = H * W;
    int32_t *img = (int32_t *)malloc(sizeof(int32_t) * n), *lab = (int32_t *)malloc(sizeof(int32_t) * n);
    for (int64_t i = 0; i < n; ++i) img[i] = !m[i];
    int32_t nl = oracle_label(img, H, W, 1, lab);
    uint8_t *edge = (uint8_t *)calloc((size_t)nl + 1, 1);
    for (int64_t c = 0; c < W; ++c) {
        edge[lab[c]] = 1;
        edge[lab[(H - 1) * W + c]] = 1;
    }
    for (int64_t r = 0; r < H; ++r) {
        edge[lab[r * W]] = 1;
        edge[lab[r * W + W - 1]] = 1;
    }
    for (int64_t i = 0; i < n; ++i) o[i] = m[i] || (lab[i] && !edge[lab[i]]);
    free(img);
    free(lab);
    free(edge);
}

/* skimage.segmentation.clear_border(labels): re-label equal-valued 8-components and
 * zero those touching the 1-pixel frame (ecoli :115, multispecies :156). */
EXPORT void oracle_clear_border(const int32_t *l, int64_t H, int64_t W, int32_t *o) {
    int64_t n = H * W;
    int32_t *lab = (int32_t *)malloc(sizeof(int32_t) * n);
    int32_t nl = oracle_label(l, H, W, 2, lab);
    uint8_t *edge = (uint8_t *)calloc((size_t)nl + 1, 1);
    for (int64_t c = 0; c < W; ++c) {
        edge[lab[c]] = 1;
        edge[lab[(H - 1) * W + c]] = 1;
    }
    for (int64_t r = 0; r < H; ++r) {
        edge[lab[r * W]] = 1;
        edge[lab[r * W + W - 1]] = 1;
    }
    for (int64_t i = 0; i < n; ++i) o[i] = (lab[i] && edge[lab[i]]) ? 0 : l[i];
    free(lab);
    free(edge);
}

/* skimage.segmentation.relabel_sequential(l)[0]: unique non-zero labels in ascending
 * order -> 1..N (multispecies :157). Returns N. */
EXPORT int32_t oracle_relabel_sequential(const int32_t *l, int64_t n, int32_t *o) {
    int32_t mx = 0;
    for (int64_t i = 0; i < n; ++i) mx = l[i] > mx ? l[i] : mx;
    int32_t *map = (int32_t *)calloc((size_t)mx + 1, sizeof(int32_t));
    for (int64_t i = 0; i < n; ++i)
        if (l[i] > 0) map[l[i]] = 1;
    map[0] = 0;
    int32_t k = 0;
    for (int32_t v = 1; v <= mx; ++v)
        if (map[v]) map[v] = ++k;
    for (int64_t i = 0; i < n; ++i) o[i] = map[l[i]];
    free(map);
    return k;
}

/* ------------------------------------------------------------------------------------
 * a12 watershed: skimage.morphology.watershed(image, markers, mask) as of the reference
 * era (skimage <= 0.18, _watershed.pyx): markers*mask pushed in raster order with age 0,
 * heap ordered by (value, age), neighbours (cross) visited up, left, right, down, a
 * neighbour is labelled when PUSHED with the popping pixel's label, age += 1 per push.
 * Binary heap restated from skimage heap_general.pxi (strict-less sift up/down).
 * (ecoli :113, multispecies :154)
 * ---------------------------------------------------------------------------------- */
typedef struct {
    double value;
    int64_t age;
    int64_t index;
} hitem;

static int h_smaller(const hitem *a, const hitem *b) {
    if (a->value != b->value) return a->value < b->value;
    return a->age < b->age;
}

typedef struct {
    hitem *d;
    int64_t n, cap;
} heap_t;

static void h_push(heap_t *h, hitem e) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 1024;
        h->d = (hitem *)realloc(h->d, sizeof(hitem) * h->cap);
    }
    int64_t c = h->n++;
    h->d[c] = e;
    while (c > 0) {
        int64_t p = (c + 1) / 2 - 1;
        if (h_smaller(&h->d[c], &h->d[p])) {
            hitem t = h->d[c];
            h->d[c] = h->d[p];
            h->d[p] = t;
            c = p;
        } else
            break;
    }
}

static hitem h_pop(heap_t *h) {
    hitem top = h->d[0];
    h->n -= 1;
    if (h->n == 0) return top;
    h->d[0] = h->d[h->n];
    int64_t i = 0;
    for (;;) {
        int64_t s = i, l = 2 * i + 1, r = 2 * i + 2;
        if (l < h->n) {
            if (h_smaller(&h->d[l], &h->d[i])) s = l;
            if (r < h->n && h_smaller(&h->d[r], &h->d[s])) s = r;
        } else
            break;
        if (s == i) break;
        hitem t = h->d[i];
        h->d[i] = h->d[s];
        h->d[s] = t;
        i = s;
    }
    return top;
}

EXPORT void oracle_watershed(const double *img, const int32_t *markers, const uint8_t *mask, int64_t H, int64_t W,
                             int32_t *out) {
    int64_t n = H * W;
    heap_t h = {0, 0, 0};
    for (int64_t i = 0; i < n; ++i) out[i] = (mask == NULL || mask[i]) ? markers[i] : 0;
    for (int64_t i = 0; i < n; ++i)
        if (out[i]) {
            hitem e = {img[i], 0, i};
            h_push(&h, e);
        }
    int64_t age = 1;
    while (h.n > 0) {
        hitem e = h_pop(&h);
        int64_t r = e.index / W, c = e.index % W;
        int64_t nb[4];
        int ok[4] = {r > 0, c > 0, c + 1 < W, r + 1 < H};
        nb[0] = e.index - W;
        nb[1] = e.index - 1;
        nb[2] = e.index + 1;
        nb[3] = e.index + W;
        for (int k = 0; k < 4; ++k) {
            if (!ok[k]) continue;
            int64_t q = nb[k];
            if (mask && !mask[q]) continue;
            if (out[q]) continue;
            age += 1;
            hitem ne = {img[q], age, q};
            h_push(&h, ne);
            out[q] = out[e.index];
        }
    }
    free(h.d);
}

/* ------------------------------------------------------------------------------------
 * a14/a20 per-label region statistics (skimage.measure.regionprops, reference era):
 * area, centroid, inertia-tensor eigenvalues -> major/minor axis (4*sqrt(l)),
 * eccentricity sqrt(1 - l2/l1), orientation (0.14/0.15 convention
 * -0.5*atan2(-2b, a-c), +-pi/4 when a == c).  Raw moments are exact int64 sums; the
 * central moments come from them in exact 128-bit integer arithmetic.
 * (ecoli :116-123; classify_spectra.py :38-46; biofilm :1234-1241)
 * stats[l] (l = 1..nlab) = {area, cr, cc, major, minor, ecc, orient, present}
 * ---------------------------------------------------------------------------------- */
EXPORT void oracle_region_stats(const int32_t *lab, int64_t H, int64_t W, int32_t nlab, double *stats /*[(nlab+1)*8]*/) {
    int64_t(*m)[6] = calloc((size_t)nlab + 1, sizeof(int64_t[6]));
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            int32_t l = lab[r * W + c];
            if (l <= 0 || l > nlab) continue;
            m[l][0] += 1;
            m[l][1] += r;
            m[l][2] += c;
            m[l][3] += r * r;
            m[l][4] += c * c;
            m[l][5] += r * c;
        }
    for (int32_t l = 0; l <= nlab; ++l) {
        double *s = stats + (int64_t)l * 8;
        memset(s, 0, sizeof(double) * 8);
        int64_t A = m[l][0];
        if (l == 0 || A == 0) continue;
        __int128 a = A, sr = m[l][1], sc = m[l][2];
        double A2 = (double)A * (double)A;
        double mu20 = (double)(a * m[l][3] - sr * sr) / A2; /* sum (r-rbar)^2 / A */
        double mu02 = (double)(a * m[l][4] - sc * sc) / A2;
        double mu11 = (double)(a * m[l][5] - sr * sc) / A2;
        /* skimage inertia tensor [[mu02, -mu11], [-mu11, mu20]] (per-area normalised) */
        double ta = mu02, tb = -mu11, tc = mu20;
        double root = sqrt(4.0 * tb * tb + (ta - tc) * (ta - tc));
        double l1 = (ta + tc) / 2.0 + root / 2.0;
        double l2 = (ta + tc) / 2.0 - root / 2.0;
        if (l1 < 0) l1 = 0;
        if (l2 < 0) l2 = 0;
        s[0] = (double)A;
        s[1] = (double)m[l][1] / (double)A;
        s[2] = (double)m[l][2] / (double)A;
        s[3] = 4.0 * sqrt(l1);
        s[4] = 4.0 * sqrt(l2);
        s[5] = l1 == 0 ? 0.0 : sqrt(1.0 - l2 / l1);
        if (ta - tc == 0) s[6] = tb < 0 ? -M_PI / 4.0 : M_PI / 4.0;
        else s[6] = -0.5 * atan2(-2.0 * tb, ta - tc);
        s[7] = 1.0;
    }
    free(m);
}

/* a15: per-label mean spectrum (regionprops mean_intensity per channel, ecoli :151-155,
 * multispecies :167-171): sums[l][c] = sum of stack[p][c] over label l, counts[l].
 * Accumulated in f64 (stack values are f32). */
EXPORT void oracle_label_sums(const float *stack, const int32_t *lab, int64_t n, int C, int32_t nlab, double *sums,
                              int64_t *counts) {
    memset(sums, 0, sizeof(double) * ((size_t)nlab + 1) * C);
    memset(counts, 0, sizeof(int64_t) * ((size_t)nlab + 1));
    for (int64_t p = 0; p < n; ++p) {
        int32_t l = lab[p];
        if (l <= 0 || l > nlab) continue;
        counts[l]++;
        for (int c = 0; c < C; ++c) sums[(int64_t)l * C + c] += (double)stack[p * C + c];
    }
}

/* ------------------------------------------------------------------------------------
 * a19 segmented cosine distance (train_reference.py):
 *   variant 0 "ungated": mean over segments of per-segment cosine distance
 *             (the all-segment branch of channel_cosine_intensity :333-385)
 *   variant 1 channel_cosine_intensity (:223-386): flags equal (sum|fx-fy| < 0.01) ->
 *             segments with fx==0 contribute 0; always / nseg
 *   variant 2 channel_cosine_intensity_7b_v2 (:993-1072): flags equal -> 0.5*sum/nseg
 *             (segments with fx==0 contribute 0), else 1
 * per-segment: both norms 0 -> 0, one norm 0 -> 1, else 1 - dot/sqrt(nx*ny)
 * ---------------------------------------------------------------------------------- */
static double seg_dist(const double *x, const double *y, int lo, int hi) {
    double d = 0, nx = 0, ny = 0;
    for (int i = lo; i < hi; ++i) {
        d += x[i] * y[i];
        nx += x[i] * x[i];
        ny += y[i] * y[i];
    }
    if (nx == 0.0 && ny == 0.0) return 0.0;
    if (nx == 0.0 || ny == 0.0) return 1.0;
    return 1.0 - d / sqrt(nx * ny);
}

EXPORT double oracle_segcos(const double *x, const double *y, const int32_t *bounds, int nseg, int variant,
                            const double *fx, const double *fy) {
    if (variant == 0) {
        double s = 0;
        for (int k = 0; k < nseg; ++k) s += seg_dist(x, y, bounds[k], bounds[k + 1]);
        return s / nseg;
    }
    double chk = 0;
    for (int k = 0; k < nseg; ++k) chk += fabs(fx[k] - fy[k]);
    if (chk < 0.01) {
        double s = 0;
        for (int k = 0; k < nseg; ++k) s += fx[k] == 0 ? 0.0 : seg_dist(x, y, bounds[k], bounds[k + 1]);
        return variant == 1 ? s / nseg : 0.5 * s / nseg;
    }
    if (variant == 2) return 1.0;
    double s = 0;
    for (int k = 0; k < nseg; ++k) s += seg_dist(x, y, bounds[k], bounds[k + 1]);
    return s / nseg;
}

/* argmin_r d(x_i, ref_r) (first minimum). x: [n][C] f64, ref: [R][C], flags [n][nseg]/[R][nseg] */
EXPORT void oracle_classify(const double *x, int64_t n, const double *ref, int R, int C, const int32_t *bounds,
                            int nseg, int variant, const double *fx, const double *fr, int32_t *arg, double *dmin) {
    (void)C;
    for (int64_t i = 0; i < n; ++i) {
        double best = INFINITY;
        int32_t bi = 0;
        for (int r = 0; r < R; ++r) {
            double d = oracle_segcos(x + i * C, ref + (int64_t)r * C, bounds, nseg, variant,
                                     fx ? fx + i * nseg : NULL, fr ? fr + (int64_t)r * nseg : NULL);
            if (d < best) {
                best = d;
                bi = r;
            }
        }
        arg[i] = bi;
        dmin[i] = best;
    }
}

/* the same search keeping the runner-up distance too (d2[i] = second smallest over r != arg):
 * lets tests require the exact argmin wherever best and runner-up are separated by more than
 * the device's error bound.  Pixels are independent: OpenMP only shortens test wall time. */
EXPORT void oracle_classify_top2(const double *x, int64_t n, const double *ref, int R, int C, const int32_t *bounds,
                                 int nseg, int32_t *arg, double *d1, double *d2) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double best = INFINITY, second = INFINITY;
        int32_t bi = 0;
        for (int r = 0; r < R; ++r) {
            double d = oracle_segcos(x + i * C, ref + (int64_t)r * C, bounds, nseg, 0, NULL, NULL);
            if (d < best) {
                second = best;
                best = d;
                bi = r;
            } else if (d < second) {
                second = d;
            }
        }
        arg[i] = bi;
        d1[i] = best;
        d2[i] = second;
    }
}

/* ------------------------------------------------------------------------------------
 * a8 1-D KMeans: the restatement of sklearn KMeans lives in kmeans_sk.c; this is the
 * fixed-point scale it shares with libhrf: q = llrint(x * 2^s), s chosen so n * max|q| < 2^62.
 * ---------------------------------------------------------------------------------- */
EXPORT int oracle_kmeans_scale(double amax, int64_t n) {
    int e = 0;
    frexp(amax > 0 ? amax : 1.0, &e); /* amax < 2^e */
    int ln = 0;
    while (((int64_t)1 << ln) < (n > 1 ? n : 1)) ++ln;
    return 61 - ln - e;
}

/* ------------------------------------------------------------------------------------
 * a22 label adjacency: skimage.future.graph.rag_boundary(labels, edge_map) edge set
 * (biofilm :1277-1278): per pixel, 3x3 grey erosion/dilation (reflect border == the
 * in-bounds window for 3x3); edges (min, centre) where min != centre and (centre, max)
 * where max != centre.  Writes a dense (nlab+1)^2 uint8 edge matrix, edge[a][b] for a<b.
 * Then barcode adjacency (biofilm :1283-1292): each undirected edge (a,b), a,b >= 1,
 * adds 1 to adj[bc[a]][bc[b]] and 1 to adj[bc[b]][bc[a]].
 * ---------------------------------------------------------------------------------- */
EXPORT void oracle_rag_edges(const int32_t *lab, int64_t H, int64_t W, int32_t nlab, uint8_t *edge) {
    int64_t L = (int64_t)nlab + 1;
    memset(edge, 0, (size_t)(L * L));
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            int32_t v = lab[r * W + c], mn = v, mx = v;
            for (int dr = -1; dr <= 1; ++dr)
                for (int dc = -1; dc <= 1; ++dc) {
                    int64_t rr = r + dr, cc = c + dc;
                    if (rr < 0 || rr >= H || cc < 0 || cc >= W) continue;
                    int32_t u = lab[rr * W + cc];
                    mn = u < mn ? u : mn;
                    mx = u > mx ? u : mx;
                }
            if (mn != v) edge[(int64_t)mn * L + v] = 1;
            if (mx != v) edge[(int64_t)v * L + mx] = 1;
        }
}

EXPORT void oracle_barcode_adjacency(const uint8_t *edge, int32_t nlab, const int32_t *bc, int R, int64_t *adj) {
    int64_t L = (int64_t)nlab + 1;
    memset(adj, 0, sizeof(int64_t) * (size_t)R * R);
    for (int64_t a = 1; a < L; ++a)
        for (int64_t b = a + 1; b < L; ++b)
            if (edge[a * L + b]) {
                /* a label whose row has no barcode in the lookup (bc < 0) is not counted (the
                 * reference's .loc would raise KeyError there) */
                if (bc[a] < 0 || bc[a] >= R || bc[b] < 0 || bc[b] >= R) continue;
                adj[(int64_t)bc[a] * R + bc[b]] += 1;
                adj[(int64_t)bc[b] * R + bc[a]] += 1;
            }
}

/* a23: per-barcode counts (collect_measurement_results.py:92-98 value_counts) */
EXPORT void oracle_barcode_counts(const int32_t *bc, int64_t n, int R, int64_t *counts) {
    memset(counts, 0, sizeof(int64_t) * R);
    for (int64_t i = 0; i < n; ++i)
        if (bc[i] >= 0 && bc[i] < R) counts[bc[i]]++;
}

/* a21: identification map (image_classification.py:65-71): pixels with label L in
 * 1..N take code[L-1] (row L-1 of the cell table, as the reference paints); others 0. */
EXPORT void oracle_paint_ids(const int32_t *lab, int64_t n, const int32_t *code, int32_t ncell, int32_t *out) {
    for (int64_t i = 0; i < n; ++i) {
        int32_t l = lab[i];
        out[i] = (l >= 1 && l <= ncell) ? code[l - 1] : 0;
    }
}

/* ------------------------------------------------------------------------------------
 * a4 non-local means: skimage.restoration.denoise_nl_means(image, patch_size=7,
 * patch_distance=11, h, fast_mode=True, sigma) on a 2-D image (multispecies :108 h=0.02,
 * biofilm :350).  skimage is not installed here and the reference pins no version: the
 * algorithm below is skimage's published fast 2-D path (_nl_means_denoising.pyx,
 * _fast_nl_means_denoising_2d), parity against skimage itself is unpinned.
 * ---------------------------------------------------------------------------------- */
/* numpy.pad(mode='reflect') source index: mirror without repeating the edge */
static int64_t reflect_idx(int64_t i, int64_t n) {
    if (n == 1) return 0;
    int64_t per = 2 * (n - 1), m = i % per;
    if (m < 0) m += per;
    return m < n ? m : per - m;
}

static double *reflect_pad(const double *img, int64_t H, int64_t W, int64_t pw) {
    int64_t hp = H + 2 * pw, wp = W + 2 * pw;
    double *p = (double *)malloc(sizeof(double) * hp * wp);
    for (int64_t r = 0; r < hp; ++r)
        for (int64_t c = 0; c < wp; ++c) p[r * wp + c] = img[reflect_idx(r - pw, H) * W + reflect_idx(c - pw, W)];
    return p;
}

/* The algorithm as skimage runs it: reflect padding by offset + d + 1; for each shift
 * t = (t_row in [-d, d], t_col in [0, d]) the integral image of the per-pixel squared
 * differences between the image and its t-shifted copy (minus var) gives every patch
 * distance in four lookups; a pair within the cutoff (distance / (h^2 s^2) <= 5) adds
 * alpha * exp(-distance) to the weights of BOTH pixels and the other pixel's value to each
 * result (alpha = 0.5 for t_col == 0, t_row != 0, whose pairs are visited twice; the zero
 * shift credits its pixel twice); result / weights, padding cropped.  Rows and columns
 * within offset of the padded border (they only reach cropped pixels) are skipped. */
EXPORT void oracle_nl_means_skimage(const double *img, int64_t H, int64_t W, int patch, int dist, double h,
                                    double sigma, double *out) {
    const int s = patch % 2 == 0 ? patch + 1 : patch;
    const int off = s / 2;
    const int64_t pw = off + dist + 1, nr = H + 2 * pw, nc = W + 2 * pw;
    double *P = reflect_pad(img, H, W, pw);
    double *res = (double *)calloc((size_t)(nr * nc), sizeof(double));
    double *wt = (double *)calloc((size_t)(nr * nc), sizeof(double));
    double *I = (double *)malloc(sizeof(double) * nr * nc);
    const double h2 = h * h, s2 = (double)s * (double)s, h2s2 = 1.0 * h2 * s2, var = sigma * sigma;
    for (int tr = -dist; tr <= dist; ++tr)
        for (int tc = 0; tc <= dist; ++tc) {
            const double alpha = (tc == 0 && tr != 0) ? 0.5 : 1.0;
            memset(I, 0, sizeof(double) * nr * nc);
            const int64_t rs = tr < 0 ? -tr : 1, re = tr > 0 ? nr - tr : nr;
            for (int64_t r = (rs > 1 ? rs : 1); r < re; ++r)
                for (int64_t c = 1; c < nc - tc; ++c) {
                    double t = P[r * nc + c] - P[(r + tr) * nc + c + tc];
                    double d = t * t;
                    d -= 1.0 * var;
                    I[r * nc + c] = d + I[(r - 1) * nc + c] + I[r * nc + c - 1] - I[(r - 1) * nc + c - 1];
                }
            const int64_t r_lo = (off + 1 > off - tr) ? off + 1 : off - tr;
            const int64_t r_hi = (nr - off < nr - off - tr) ? nr - off : nr - off - tr;
            for (int64_t r = r_lo; r < r_hi; ++r)
                for (int64_t c = off + 1; c < nc - off - tc; ++c) {
                    double D = I[(r + off) * nc + c + off] + I[(r - off - 1) * nc + c - off - 1] -
                               I[(r - off - 1) * nc + c + off] - I[(r + off) * nc + c - off - 1];
                    D = (D > 0.0 ? D : 0.0) / h2s2;
                    if (D > 5.0) continue;
                    const double w = alpha * exp(-D);
                    const int64_t q = (r + tr) * nc + c + tc;
                    wt[r * nc + c] += w;
                    wt[q] += w;
                    res[r * nc + c] += w * P[q];
                    res[q] += w * P[r * nc + c];
                }
        }
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            const int64_t i = (r + pw) * nc + c + pw;
            out[r * W + c] = res[i] / wt[i];
        }
    free(P);
    free(res);
    free(wt);
    free(I);
}

/* The same weights per pixel, in the summation order AND arithmetic of libhrf's
 * nl_means_pairs_kernel, so the two are bit-identical (tests/test_nlmeans_gpu.py) and the
 * whole community chain can be compared without handing the GPU image to the oracle:
 * out[p] = (2 P[p] + sum_s w_s P[p+s]) / (2 + sum_s w_s) over the (2d+1)^2 window, s != 0,
 * taken as skimage takes it -- each unordered pair once: for s in the half window H+ (sr > 0,
 * or sr == 0 and sc > 0) in raster order, first the pair (p, p+s), then (p-s, p).  Patch
 * distance of the pair (a, a+s) = sum7 over 7 rows (top to bottom) of the row's sum7 of 7
 * squared differences (left to right), sum7 the kernel's fixed tree -- symmetric in a and
 * a+s, so both ends see the same weight; skimage's cut
 * max(D,0)/h2s2 <= 5 as the exact threshold D <= lim on D (a cut pair adds w = 0);
 * w = e^{-max(D,0) * (1/h2s2)} by hrf_exp_neg_tab (detmath.h, shared with the kernel).
 * Agrees with the integral-image restatement above within 1e-12. */
/* nlmeans.hip sum7: ((v0 + v1) + (v2 + v3)) + ((v4 + v5) + v6) */
static double sum7(const double *v) { return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + v[6]); }

EXPORT void oracle_nl_means(const double *img, int64_t H, int64_t W, int patch, int dist, double h, double sigma,
                            double *out) {
    const int s = patch % 2 == 0 ? patch + 1 : patch;
    const int off = s / 2;
    if (s != 7) { /* sum7: the kernel is built for patch 7 only */
        for (int64_t i = 0; i < H * W; ++i) out[i] = NAN;
        return;
    }
    const int64_t pw = off + dist, wp = W + 2 * pw;
    double *P = reflect_pad(img, H, W, pw);
    const double h2 = h * h, s2 = (double)s * (double)s, h2s2 = 1.0 * h2 * s2, var = sigma * sigma;
    /* the largest D whose quotient fl(D / h2s2) is still <= 5 */
    double lim = 5.0 * h2s2;
    while (lim / h2s2 > 5.0) lim = nextafter(lim, -1.0);
    while (nextafter(lim, 2.0 * lim + 1.0) / h2s2 <= 5.0) lim = nextafter(lim, 2.0 * lim + 1.0);
    const double inv = 1.0 / h2s2;
    /* rows are independent (each pixel's sums run in a fixed order): OpenMP only shortens
     * the wall time of full-size parity tests, the result does not depend on it */
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            const double *p = P + (r + pw) * wp + (c + pw);
            double acc = p[0] + p[0], ws = 2.0;
            for (int sr = 0; sr <= dist; ++sr)
                for (int sc = sr == 0 ? 1 : -dist; sc <= dist; ++sc)
                    for (int end = 0; end < 2; ++end) {
                        /* the pair (a, a + s): a = p first, then a = p - s; the partner's value */
                        const double *a = end == 0 ? p : p - sr * wp - sc;
                        const double *b = a + sr * wp + sc;
                        double hs[7], sq[7];
                        for (int du = -off; du <= off; ++du) {
                            for (int dv = -off; dv <= off; ++dv) {
                                const double t = a[du * wp + dv] - b[du * wp + dv];
                                sq[dv + off] = var == 0.0 ? t * t : t * t - var;
                            }
                            hs[du + off] = sum7(sq);
                        }
                        const double D = sum7(hs);
                        /* a cut pair adds w = 0, as the kernel's pixel phase does */
                        const double w = D <= lim ? hrf_exp_neg_tab(-(D > 0.0 ? D : 0.0) * inv, hrf_exp2tab64) : 0.0;
                        ws += w;
                        const double t = w * (end == 0 ? b[0] : a[0]);
                        acc += t;
                    }
            out[r * W + c] = acc / ws;
        }
    free(P);
}

/* ecoli measurement.py:116-126 (per-cell shape filter + 2x binary_erosion of the cell) */
EXPORT void oracle_shape_filter(const int32_t *lab, int64_t H, int64_t W, const double *stats, int32_t nlab,
                                double lo, double hi, int32_t *out) {
    for (int64_t r = 0; r < H; ++r)
        for (int64_t c = 0; c < W; ++c) {
            int32_t l = lab[r * W + c], o = 0;
            if (l > 0 && l <= nlab && stats[(int64_t)l * 8 + 7] != 0.0) {
                double mn = stats[(int64_t)l * 8 + 4];
                if (!(mn < lo || mn > hi)) {
                    int in = 1;
                    for (int dr = -2; dr <= 2; ++dr)
                        for (int dc = -2; dc <= 2; ++dc) {
                            if (abs(dr) + abs(dc) > 2) continue;
                            int64_t rr = r + dr, cc = c + dc;
                            if (rr < 0 || rr >= H || cc < 0 || cc >= W) continue;
                            in = in && lab[rr * W + cc] == l;
                        }
                    o = in ? l : 0;
                }
            }
            out[r * W + c] = o;
        }
}
