/* oracle/backend.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product path): CPU
 * restatement of the per-cell classifier back-end (a17, a18, f2), in the reference's operation
 * order, f64.
 *
 *  oracle_svc_predict  sklearn SVC.predict / decision_function (ovo): libsvm svm_predict_values
 *                      on dense vectors (sklearn's svm.cpp, _DENSE_REP): kernel values in
 *                      feature order, per pair (a, b) the class-a support vectors with
 *                      coef[b-1] then the class-b ones with coef[a], minus rho; vote a when > 0;
 *                      first maximum.  Pinned to sklearn itself (tests/golden/backend.npz).
 *  oracle_knn          brute-force k nearest rows under channel_cosine_intensity_7b_v2
 *                      (train_reference.py:993-1072) / _violet_derivative_v2 (:569-731, the
 *                      scalar (d + c1..c5)/6 it computes) / euclidean; ties to the lower row.
 *                      The search pinned to sklearn NearestNeighbors(algorithm='brute').
 *  oracle_umap_init    umap-learn transform's initial embedding (umap_.py, 0.4 era):
 *                      smooth_knn_dist (float32 rho / sigma), compute_membership_strengths
 *                      (bipartite, float32), CSR l1 normalisation, init_transform (float32).
 *  oracle_umap_refine  transform's layout refinement (optimize_layout_euclidean, training
 *                      embedding fixed) with per-query seeded negative-sample streams.
 *                      umap-learn is absent here: parity unpinned for both.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../hiprfish_image_analysis_amd/csrc/detmath.h"

static double svc_k(const double *x, const double *y, int f, int kernel, double gamma, double coef0, int degree) {
  double s = 0.0;
  if (kernel == 2) {
    for (int i = 0; i < f; ++i) {
      const double d = x[i] - y[i];
      s += d * d;
    }
    return hrf_det_exp(-gamma * s);
  }
  for (int i = 0; i < f; ++i) s += x[i] * y[i];
  if (kernel == 0) return s;
  if (kernel == 1) {
    double r = 1.0, t = gamma * s + coef0;
    for (int d = degree; d > 0; d /= 2) {
      if (d % 2 == 1) r *= t;
      t = t * t;
    }
    return r;
  }
  return tanh(gamma * s + coef0);
}

void oracle_svc_predict(const double *x, int64_t n, int64_t ldx, int f, const double *sv, int nsv, const double *coef,
                        const double *intercept, const int32_t *start, int n_class, int kernel, double gamma,
                        double coef0, int degree, int32_t *pred, double *dec) {
  double *kv = (double *)malloc(sizeof(double) * (size_t)nsv);
  int *vote = (int *)malloc(sizeof(int) * (size_t)n_class);
  const int npair = n_class * (n_class - 1) / 2;
  for (int64_t i = 0; i < n; ++i) {
    const double *xi = x + i * ldx;
    for (int s = 0; s < nsv; ++s) kv[s] = svc_k(xi, sv + (int64_t)s * f, f, kernel, gamma, coef0, degree);
    memset(vote, 0, sizeof(int) * (size_t)n_class);
    int p = 0;
    for (int a = 0; a < n_class; ++a)
      for (int b = a + 1; b < n_class; ++b, ++p) {
        const double *c1 = coef + (int64_t)(b - 1) * nsv, *c2 = coef + (int64_t)a * nsv;
        double sum = 0.0;
        for (int k = start[a]; k < start[a + 1]; ++k) sum += c1[k] * kv[k];
        for (int k = start[b]; k < start[b + 1]; ++k) sum += c2[k] * kv[k];
        sum += intercept[p];
        if (dec) dec[i * npair + p] = sum;
        ++vote[sum > 0 ? a : b];
      }
    int best = 0;
    for (int c = 1; c < n_class; ++c)
      if (vote[c] > vote[best]) best = c;
    pred[i] = best;
  }
  free(kv);
  free(vote);
}

/* libsvm svm_predict_probability (C_SVC with probA / probB): sigmoid_predict per pair, clamp
 * [1e-7, 1 - 1e-7], multiclass_probability (max(100, k) iterations, eps 0.005 / k) */
static double sigmoid_predict(double dec, double A, double B) {
  const double fApB = dec * A + B;
  if (fApB >= 0) return hrf_det_exp(-fApB) / (1.0 + hrf_det_exp(-fApB));
  return 1.0 / (1 + hrf_det_exp(fApB));
}

/* multiclass_probability follows libsvm's svm.cpp (Wu, Lin and Weng's pairwise coupling, as
 * sklearn vendors it), whose licence asks for this notice:
 *
 * Copyright (c) 2000-2019 Chih-Chung Chang and Chih-Jen Lin.  All rights reserved.
 *
 * Redistribution and use in source and binary forms, with or without modification, are
 * permitted provided that the following conditions are met:
 * 1. Redistributions of source code must retain the above copyright notice, this list of
 *    conditions and the following disclaimer.
 * 2. Redistributions in binary form must reproduce the above copyright notice, this list of
 *    conditions and the following disclaimer in the documentation and/or other materials
 *    provided with the distribution.
 * 3. Neither name of copyright holders nor the names of its contributors may be used to
 *    endorse or promote products derived from this software without specific prior written
 *    permission.
 *
 * THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS" AND ANY EXPRESS
 * OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE IMPLIED WARRANTIES OF
 * MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE DISCLAIMED.  IN NO EVENT SHALL THE
 * REGENTS OR CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY,
 * OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR
 * SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED AND ON ANY
 * THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING NEGLIGENCE OR
 * OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS SOFTWARE, EVEN IF ADVISED OF THE
 * POSSIBILITY OF SUCH DAMAGE. */
static void multiclass_probability(int k, double **r, double *p, double **Q, double *Qp) {
  int t, j, iter, max_iter = k > 100 ? k : 100;
  double pQp, eps = 0.005 / k;
  for (t = 0; t < k; t++) {
    p[t] = 1.0 / k;
    Q[t][t] = 0;
    for (j = 0; j < t; j++) {
      Q[t][t] += r[j][t] * r[j][t];
      Q[t][j] = Q[j][t];
    }
    for (j = t + 1; j < k; j++) {
      Q[t][t] += r[j][t] * r[j][t];
      Q[t][j] = -r[j][t] * r[t][j];
    }
  }
  for (iter = 0; iter < max_iter; iter++) {
    pQp = 0;
    for (t = 0; t < k; t++) {
      Qp[t] = 0;
      for (j = 0; j < k; j++) Qp[t] += Q[t][j] * p[j];
      pQp += p[t] * Qp[t];
    }
    double max_error = 0;
    for (t = 0; t < k; t++) {
      const double error = fabs(Qp[t] - pQp);
      if (error > max_error) max_error = error;
    }
    if (max_error < eps) break;
    for (t = 0; t < k; t++) {
      const double diff = (-Qp[t] + pQp) / Q[t][t];
      p[t] += diff;
      pQp = (pQp + diff * (diff * Q[t][t] + 2 * Qp[t])) / (1 + diff) / (1 + diff);
      for (j = 0; j < k; j++) {
        Qp[j] = (Qp[j] + diff * Q[t][j]) / (1 + diff);
        p[j] /= (1 + diff);
      }
    }
  }
}

void oracle_svc_proba(const double *x, int64_t n, int64_t ldx, int f, const double *sv, int nsv, const double *coef,
                      const double *intercept, const int32_t *start, int n_class, int kernel, double gamma,
                      double coef0, int degree, const double *probA, const double *probB, double *prob) {
  const int k = n_class, npair = k * (k - 1) / 2;
  double *dec = (double *)malloc(sizeof(double) * (size_t)npair);
  int32_t *pred = (int32_t *)malloc(sizeof(int32_t));
  double **r = (double **)malloc(sizeof(double *) * (size_t)k), **Q = (double **)malloc(sizeof(double *) * (size_t)k);
  double *rbuf = (double *)malloc(sizeof(double) * (size_t)k * k), *qbuf = (double *)malloc(sizeof(double) * (size_t)k * k);
  double *Qp = (double *)malloc(sizeof(double) * (size_t)k);
  for (int a = 0; a < k; ++a) {
    r[a] = rbuf + (size_t)a * k;
    Q[a] = qbuf + (size_t)a * k;
  }
  for (int64_t i = 0; i < n; ++i) {
    oracle_svc_predict(x + i * ldx, 1, ldx, f, sv, nsv, coef, intercept, start, n_class, kernel, gamma, coef0, degree,
                       pred, dec);
    int q = 0;
    for (int a = 0; a < k; ++a)
      for (int b = a + 1; b < k; ++b, ++q) {
        double v = sigmoid_predict(dec[q], probA[q], probB[q]);
        v = v < 1e-7 ? 1e-7 : v;
        v = v > 1 - 1e-7 ? 1 - 1e-7 : v;
        r[a][b] = v;
        r[b][a] = 1 - v;
      }
    /* sklearn's libsvm couples two classes too (no k == 2 shortcut) */
    multiclass_probability(k, r, prob + i * k, Q, Qp);
  }
  free(dec);
  free(pred);
  free(r);
  free(Q);
  free(rbuf);
  free(qbuf);
  free(Qp);
}

static double seg_cos(const double *x, const double *y, int lo, int hi) {
  double result = 0.0, nx = 0.0, ny = 0.0;
  for (int i = lo; i < hi; ++i) {
    result += x[i] * y[i];
    nx += x[i] * x[i];
    ny += y[i] * y[i];
  }
  if (nx == 0.0 && ny == 0.0) return 0.0;
  if (nx == 0.0 || ny == 0.0) return 1.0;
  return 1.0 - (result / sqrt(nx * ny));
}

double oracle_knn_metric(int metric, const double *x, const double *y, int f) {
  if (metric == 0) {
    double s = 0.0;
    for (int i = 0; i < f; ++i) s += (x[i] - y[i]) * (x[i] - y[i]);
    return sqrt(s);
  }
  if (metric == 1) {
    double check = 0.0;
    for (int i = 63; i < 67; ++i) check += fabs(x[i] - y[i]);
    if (!(check < 0.01)) return 1.0;
    static const int b[5] = {0, 23, 43, 57, 63};
    double c[4];
    for (int s = 0; s < 4; ++s) c[s] = x[63 + s] == 0 ? 0.0 : seg_cos(x, y, b[s], b[s + 1]);
    return 0.5 * (c[0] + c[1] + c[2] + c[3]) / 4;
  }
  double check = 0.0;
  for (int i = 126; i < 132; ++i) check += fabs(x[i] - y[i]);
  static const int b[6] = {0, 32, 55, 75, 89, 95};
  double c[5], d;
  if (check < 0.01) {
    d = 0.0;
    for (int s = 0; s < 5; ++s) c[s] = x[126 + s] == 0 ? 0.0 : seg_cos(x, y, b[s], b[s + 1]);
  } else {
    d = 1.0;
    for (int s = 0; s < 5; ++s) c[s] = seg_cos(x, y, b[s], b[s + 1]);
  }
  return (d + c[0] + c[1] + c[2] + c[3] + c[4]) / 6;
}

void oracle_knn(const double *q, int64_t nq, int64_t ldq, const double *train, int64_t nt, int f, int metric, int k,
                int32_t *idx, double *dist) {
  for (int64_t i = 0; i < nq; ++i) {
    int n = 0;
    double *bd = dist + i * k;
    int32_t *bi = idx + i * k;
    for (int64_t r = 0; r < nt; ++r) {
      const double d = oracle_knn_metric(metric, q + i * ldq, train + r * f, f);
      if (n == k && !(d < bd[k - 1])) continue;
      int pos = n < k ? n : k - 1;
      while (pos > 0 && d < bd[pos - 1]) {
        bd[pos] = bd[pos - 1];
        bi[pos] = bi[pos - 1];
        --pos;
      }
      bd[pos] = d;
      bi[pos] = (int32_t)r;
      if (n < k) ++n;
    }
    for (int j = n; j < k; ++j) {
      bi[j] = -1;
      bd[j] = INFINITY;
    }
  }
}

void oracle_umap_init(const int32_t *idx, const double *dist, int64_t nq, int k, double n_neighbors,
                      double local_connectivity, const float *emb, int d, float *memb, float *out) {
  double mean_all = 0.0;
  for (int64_t e = 0; e < nq * k; ++e) mean_all += dist[e];
  mean_all /= (double)(nq * k);
  const double target = hrf_det_log(n_neighbors) * 1.4426950408889634;  /* log2 */
  float *w = (float *)malloc(sizeof(float) * (size_t)k);
  int *ord = (int *)malloc(sizeof(int) * (size_t)k);
  for (int64_t i = 0; i < nq; ++i) {
    const double *di = dist + i * k;
    const int32_t *ii = idx + i * k;
    float rho = 0.0f;   /* umap keeps rho and sigma in float32 arrays */
    int nnz = 0;
    for (int j = 0; j < k; ++j) nnz += di[j] > 0.0;
    if (nnz >= local_connectivity) {
      const int index = (int)floor(local_connectivity);
      const double interp = local_connectivity - index;
      double nz[2] = {0, 0}, first = 0;
      int seen = 0, got = 0;
      for (int j = 0; j < k; ++j) {
        if (!(di[j] > 0.0)) continue;
        if (!got) {
          first = di[j];
          got = 1;
        }
        ++seen;
        if (seen == index) nz[0] = di[j];
        if (seen == index + 1) nz[1] = di[j];
      }
      if (index > 0) {
        rho = (float)nz[0];
        if (interp > 1e-5) rho = (float)((double)rho + interp * (nz[1] - nz[0]));
      } else {
        rho = (float)(interp * first);
      }
    } else if (nnz > 0) {
      double mx = -INFINITY;
      for (int j = 0; j < k; ++j)
        if (di[j] > 0.0 && di[j] > mx) mx = di[j];
      rho = (float)mx;
    }
    double lo = 0.0, hi = INFINITY, mid = 1.0;
    for (int it = 0; it < 64; ++it) {
      double psum = 0.0;
      for (int j = 1; j < k; ++j) {
        const double dd = di[j] - (double)rho;
        psum += dd > 0 ? hrf_det_exp(-(dd / mid)) : 1.0;
      }
      if (fabs(psum - target) < 1e-5) break;
      if (psum > target) {
        hi = mid;
        mid = (lo + hi) / 2.0;
      } else {
        lo = mid;
        mid = isinf(hi) ? mid * 2 : (lo + hi) / 2.0;
      }
    }
    float sigma = (float)mid;
    if (rho > 0.0f) {
      double m = 0.0;
      for (int j = 0; j < k; ++j) m += di[j];
      m /= k;
      if ((double)sigma < 1e-3 * m) sigma = (float)(1e-3 * m);
    } else if ((double)sigma < 1e-3 * mean_all) {
      sigma = (float)(1e-3 * mean_all);
    }
    int n = 0;
    for (int j = 0; j < k; ++j) {
      float v = 0.0f;
      if (ii[j] >= 0) {
        const double dd = di[j] - (double)rho;
        v = (dd <= 0.0 || sigma == 0.0f) ? 1.0f : (float)hrf_det_exp(-(dd / (double)sigma));
        w[n] = v;
        ord[n] = j;
        ++n;
      }
      if (memb) memb[i * k + j] = v;
    }
    for (int a = 1; a < n; ++a)
      for (int b = a; b > 0 && ii[ord[b]] < ii[ord[b - 1]]; --b) {
        const int t = ord[b];
        ord[b] = ord[b - 1];
        ord[b - 1] = t;
        const float tw = w[b];
        w[b] = w[b - 1];
        w[b - 1] = tw;
      }
    double s = 0.0;   /* sklearn normalize(norm='l1'): double row sum, float32 store */
    for (int a = 0; a < n; ++a) s += fabs((double)w[a]);
    for (int c = 0; c < d; ++c) out[i * d + c] = 0.0f;
    for (int a = 0; a < n; ++a) {
      const float wn = s != 0.0 ? (float)((double)w[a] / s) : w[a];
      for (int c = 0; c < d; ++c) {
        const volatile float prod = wn * emb[(int64_t)ii[ord[a]] * d + c];
        out[i * d + c] = out[i * d + c] + prod;
      }
    }
  }
  free(w);
  free(ord);
}

/* umap's tau_rand_int on unsigned 32-bit states; per-query streams seeded by splitmix64 of
 * (seed, query) -- the device's stream (backend.hip umap_refine_kernel) */
static uint32_t tau_rand(uint32_t *s) {
  s[0] = ((s[0] & 4294967294u) << 12) ^ (((s[0] << 13) ^ s[0]) >> 19);
  s[1] = ((s[1] & 4294967288u) << 4) ^ (((s[1] << 2) ^ s[1]) >> 25);
  s[2] = ((s[2] & 4294967280u) << 17) ^ (((s[2] << 3) ^ s[2]) >> 11);
  return s[0] ^ s[1] ^ s[2];
}

static uint64_t splitmix64(uint64_t *x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static double uclip(double v) { return v > 4.0 ? 4.0 : (v < -4.0 ? -4.0 : v); }

static double urdist(const float *x, const float *y, int d) {
  double r = 0.0;
  for (int c = 0; c < d; ++c) {
    const float df = x[c] - y[c];
    const volatile float sq = df * df;
    r += (double)sq;
  }
  return r;
}

/* umap_.py transform() after init (0.4): threshold the graph at max / n_epochs,
 * make_epochs_per_sample, optimize_layout_euclidean with the training embedding fixed */
void oracle_umap_refine(const int32_t *idx, const float *memb, int64_t nq, int k, int n_epochs, const float *tail,
                        int64_t ntrain, int d, double a, double b, double gamma, double alpha0, double neg_rate,
                        uint64_t seed, float *emb) {
  float wmax = 0.0f;
  for (int64_t e = 0; e < nq * k; ++e)
    if (memb[e] > wmax) wmax = memb[e];
  const float thr = (float)((double)wmax / (double)n_epochs);
  double *eps = (double *)malloc(sizeof(double) * (size_t)k * 3);
  double *eons = eps + k, *eonns = eps + 2 * k;
  int32_t *tl = (int32_t *)malloc(sizeof(int32_t) * (size_t)k);
  for (int64_t i = 0; i < nq; ++i) {
    int ne = 0;
    for (int j = 0; j < k; ++j) {
      const float w = memb[i * k + j];
      if (idx[i * k + j] < 0 || !(w >= thr) || w == 0.0f) continue;
      const float ratio = w / wmax;
      const float ns = (float)n_epochs * ratio;
      eps[ne] = ns > 0.0f ? (double)((float)n_epochs / ns) : -1.0;
      eons[ne] = eps[ne];
      eonns[ne] = eps[ne] / neg_rate;
      tl[ne] = idx[i * k + j];
      ++ne;
    }
    float *cur = emb + i * d;
    uint64_t sm = seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(i + 1));
    uint32_t st[3];
    st[0] = (uint32_t)splitmix64(&sm) | 2u;
    st[1] = (uint32_t)splitmix64(&sm) | 8u;
    st[2] = (uint32_t)splitmix64(&sm) | 16u;
    double alpha = alpha0;
    for (int n = 0; n < n_epochs; ++n) {
      for (int e = 0; e < ne; ++e) {
        if (!(eons[e] <= n)) continue;
        const float *o = tail + (int64_t)tl[e] * d;
        const double d2 = urdist(cur, o, d);
        double gc = 0.0;
        if (d2 > 0.0) {
          gc = -2.0 * a * b * hrf_det_pow(d2, b - 1.0);
          gc /= a * hrf_det_pow(d2, b) + 1.0;
        }
        for (int c = 0; c < d; ++c) {
          const double g = uclip(gc * (double)(cur[c] - o[c]));
          cur[c] = (float)((double)cur[c] + g * alpha);
        }
        eons[e] += eps[e];
        const double epns = eps[e] / neg_rate;
        const int nneg = (int)(((double)n - eonns[e]) / epns);
        for (int p = 0; p < nneg; ++p) {
          const int64_t kk = (int64_t)(tau_rand(st) % (uint64_t)ntrain);
          const float *on = tail + kk * d;
          const double dn = urdist(cur, on, d);
          double gn;
          if (dn > 0.0) {
            gn = 2.0 * gamma * b;
            gn /= (0.001 + dn) * (a * hrf_det_pow(dn, b) + 1.0);
          } else if (kk == i) {
            continue;
          } else {
            gn = 0.0;
          }
          for (int c = 0; c < d; ++c) {
            const double g = gn > 0.0 ? uclip(gn * (double)(cur[c] - on[c])) : 4.0;
            cur[c] = (float)((double)cur[c] + g * alpha);
          }
        }
        eonns[e] += nneg * epns;
      }
      alpha = alpha0 * (1.0 - (double)n / (double)n_epochs);
    }
  }
  free(eps);
  free(tl);
}

/* correctly rounded log / log10 (detmath.h hrf_cr_log*, the functions libhrf's image_cn uses):
 * image_cn = log(sum + 1e-2) (ecoli measurement.py:72), log10(sum + 1) (biofilm :831).
 * mode 0: log, 1: log10 */
__attribute__((visibility("default"))) void oracle_cr_log(const double *x, int64_t n, int mode, double *out) {
  for (int64_t i = 0; i < n; ++i) out[i] = mode ? hrf_cr_log10(x[i]) : hrf_cr_log(x[i]);
}

/* the C library's own log / log10 (glibc here), element by element: what numpy 1.16 -- the
 * reference era's numpy, whose np.log called libm -- computes for image_cn (ecoli :72).  Used by
 * tests/test_image_cn_log.py to show the segmentation does not depend on the last ulp. */
__attribute__((visibility("default"))) void oracle_libm_log(const double *x, int64_t n, int mode, double *out) {
  for (int64_t i = 0; i < n; ++i) out[i] = mode ? log10(x[i]) : log(x[i]);
}

/* hrf_div_rcp (detmath.h) against the IEEE division on n float32 pairs: random bit patterns
 * (finite, d nonzero), plus directed significands (all ones, 1 + ulp, powers of two) -> the
 * number of pairs whose results differ (tests/test_oracle_golden.py). */
__attribute__((visibility("default"))) int64_t oracle_div_rcp_check(uint64_t seed, int64_t n) {
  uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
  int64_t bad = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t w[2];
    for (int k = 0; k < 2; ++k) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      w[k] = (uint32_t)(s >> 11);
    }
    const int mode = (int)(i & 7);
    if (mode == 1) w[1] |= 0x007FFFFFu;                  /* d significand all ones */
    if (mode == 2) w[1] = (w[1] & 0xFF800000u) | 1u;     /* d = 2^e (1 + ulp) */
    if (mode == 3) w[0] |= 0x007FFFFFu;
    if (mode == 4) w[1] &= 0xFF800000u;                  /* d a power of two */
    if (mode == 5) w[1] = (w[1] & 0x807FFFFFu) | 0x3F000000u;   /* d in [0.5, 1) (flat fields) */
    if (mode == 6) w[0] = (w[0] & 0x007FFFFFu) | 0x3E000000u;   /* x in [0.125, 0.25) */
    float xf, df;
    memcpy(&xf, &w[0], 4);
    memcpy(&df, &w[1], 4);
    if (!isfinite(xf) || !isfinite(df) || df == 0.0f) continue;
    const double x = xf, d = df, r = 1.0 / d;
    const double a = x / d, b = hrf_div_rcp(x, d, r);
    if (memcmp(&a, &b, 8) != 0) ++bad;
  }
  return bad;
}

/* nlmeans.hip's widened-table exponential against detmath.h hrf_exp_neg_tab (the oracle's):
 * n values spread over [-8, 0] plus every rounding boundary k ln2/64 and its neighbours;
 * returns the count of results that differ in any bit. */
__attribute__((visibility("default"))) int64_t oracle_exp_tabw_check(int64_t n) {
  static double tabw[HRF_EXP_WIDE_N];
  for (int i = 0; i < HRF_EXP_WIDE_N; ++i) tabw[i] = ldexp(hrf_exp2tab64[-i & 63], -i >> 6);
  int64_t bad = 0;
  for (int64_t i = 0; i <= n; ++i) {
    const double x = -8.0 * (double)i / (double)n;
    const double a = hrf_exp_neg_tab(x, hrf_exp2tab64), b = hrf_exp_neg_tabw(x, tabw);
    if (memcmp(&a, &b, 8) != 0) ++bad;
  }
  for (int k = 0; k <= 739; ++k) {
    double x = -(k + 0.5) / HRF_EXP_INVL;
    for (int d = 0; d < 5; ++d) x = nextafter(x, 0.0);
    for (int d = 0; d < 10 && x >= -8.0; ++d, x = nextafter(x, -9.0)) {
      const double a = hrf_exp_neg_tab(x, hrf_exp2tab64), b = hrf_exp_neg_tabw(x, tabw);
      if (memcmp(&a, &b, 8) != 0) ++bad;
    }
  }
  return bad;
}
