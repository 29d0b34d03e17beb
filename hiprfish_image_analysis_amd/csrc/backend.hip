// backend.hip -- the per-cell classifier back-end after the spectra (a17, a18, f2).
//
// Reference: ecoli image_classification.py:43-56 and synthetic-community
// classify_spectra.py:27-35 --
//   features   avgint_norm | np.diff(avgint_norm[:, 0:32]) | per-laser check-SVC flags (E. coli,
//              132 columns); avgint_norm | flags (community, 67 columns, the flags from the
//              StandardScaler-scaled segments)                                              (a17)
//   flags      clf[k].predict(segment k)  -- sklearn SVC (libsvm one-vs-one)                   (a18)
//   embedding  umap_transform.transform(features): exact k nearest training rows under the
//              reference metric (channel_cosine_intensity_7b_v2 / _violet_derivative_v2,
//              train_reference.py:993-1072 / :569-731), smooth_knn_dist, l1-normalised
//              membership strengths, weighted mean of the training embedding (umap-learn's
//              init_transform)                                                             (f2)
//   barcode    clf_umap.predict(embedding) -- sklearn SVC                                       (f2)
// The models arrive as arrays (support vectors, coefficients, training table and embedding),
// never as pickles.  Every stage is f64 in the reference's operation order.
//
// MI355X mapping: these run on the N cells of a tile (hundreds to thousands), not on pixels:
// one workgroup per cell; SVC kernel values for the support vectors strided over the threads
// into LDS, then the one-vs-one pair sums strided over the threads (each pair in libsvm's
// order); the kNN streams a feature-major copy of the training table (coalesced) and keeps the
// running k best in LDS, merging a 256-row chunk only when some row beats the current k-th.
#include <cmath>

#include "common.hpp"
#include "detmath.h"

namespace {

// ---- a17 -------------------------------------------------------------------------------------
// E. coli: out (n x 132) = x (n x 95) | diff(x[:, 0:32]) (31) | 0 (6 flag columns)
__global__ void features_ecoli_kernel(const double *__restrict__ x, int64_t n, double *__restrict__ out) {
  const int64_t total = n * 132;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / 132;
    const int c = (int)(e - i * 132);
    const double *r = x + i * 95;
    double v = 0.0;
    if (c < 95) v = r[c];
    else if (c < 126) v = r[c - 95 + 1] - r[c - 95];
    out[e] = v;
  }
}

// community: out (n x 67) = x (n x 63) | 0 (4 flag columns)
__global__ void features_multi_kernel(const double *__restrict__ x, int64_t n, double *__restrict__ out) {
  const int64_t total = n * 67;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / 67;
    const int c = (int)(e - i * 67);
    out[e] = c < 63 ? x[i * 63 + c] : 0.0;
  }
}

// sklearn StandardScaler.transform: (x - mean) / scale, column by column
__global__ void standard_scale_kernel(const double *__restrict__ x, int64_t n, int32_t f, int64_t ldx,
                                      const double *__restrict__ mean, const double *__restrict__ scale,
                                      double *__restrict__ out) {
  const int64_t total = n * f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / f;
    const int c = (int)(e - i * f);
    double v = x[i * ldx + c];
    if (mean) v -= mean[c];
    if (scale) v /= scale[c];
    out[e] = v;
  }
}

// ---- a18 / f2: SVC (libsvm one-vs-one) ---------------------------------------------------------
struct SvcModel {
  const double *sv;         // (nsv, f) row-major
  const double *coef;       // (n_class - 1, nsv), libsvm's sign convention
  const double *intercept;  // (n_pairs), = -rho: pair (i, j) votes i when its sum > 0
  const int32_t *start;     // (n_class + 1) first support vector of each class
  int32_t nsv, f, n_class, kernel, degree;
  double gamma, coef0;
};

// libsvm Kernel::k_function (dense): linear, poly, rbf, sigmoid, in feature order
__device__ double svc_kernel(const double *x, const double *y, const SvcModel &m) {
  double s = 0.0;
  if (m.kernel == 2) {
    for (int i = 0; i < m.f; ++i) {
      const double d = x[i] - y[i];
      s += d * d;
    }
    return hrf_det_exp(-m.gamma * s);
  }
  for (int i = 0; i < m.f; ++i) s += x[i] * y[i];
  if (m.kernel == 0) return s;
  if (m.kernel == 1) {
    const double b = m.gamma * s + m.coef0;
    double r = 1.0, t = b;           // libsvm powi: square-and-multiply
    for (int d = m.degree; d > 0; d /= 2) {
      if (d % 2 == 1) r *= t;
      t = t * t;
    }
    return r;
  }
  return tanh(m.gamma * s + m.coef0);
}

constexpr int SVC_T = 256;

__global__ __launch_bounds__(SVC_T) void svc_predict_kernel(const double *__restrict__ x, int64_t ldx, SvcModel m,
                                                            int32_t *__restrict__ pred, double *__restrict__ dec,
                                                            double *__restrict__ val_out, int64_t val_stride,
                                                            const double *__restrict__ class_values) {
  extern __shared__ double kv[];                // nsv kernel values, then the votes
  const int64_t i = blockIdx.x;
  const double *xi = x + i * ldx;
  for (int s = threadIdx.x; s < m.nsv; s += SVC_T) kv[s] = svc_kernel(xi, m.sv + (int64_t)s * m.f, m);
  int *vote = reinterpret_cast<int *>(kv + m.nsv);
  for (int c = threadIdx.x; c < m.n_class; c += SVC_T) vote[c] = 0;
  __syncthreads();
  const int npair = m.n_class * (m.n_class - 1) / 2;
  for (int p = threadIdx.x; p < npair; p += SVC_T) {
    // pair p = (a, b), a < b, in libsvm's order: row a starts at P(a) = a n - a (a + 1) / 2
    auto P = [&](int64_t a) { return a * m.n_class - a * (a + 1) / 2; };
    const double nn = 2.0 * m.n_class - 1.0;
    int a = (int)floor((nn - sqrt(nn * nn - 8.0 * (double)p)) / 2.0);
    if (a < 0) a = 0;
    while (a > 0 && P(a) > p) --a;
    while (a + 1 < m.n_class && P(a + 1) <= p) ++a;
    const int b = a + 1 + (int)(p - P(a));
    const double *c1 = m.coef + (int64_t)(b - 1) * m.nsv, *c2 = m.coef + (int64_t)a * m.nsv;
    double sum = 0.0;
    for (int k = m.start[a]; k < m.start[a + 1]; ++k) sum += c1[k] * kv[k];
    for (int k = m.start[b]; k < m.start[b + 1]; ++k) sum += c2[k] * kv[k];
    sum += m.intercept[p];
    if (dec) dec[i * npair + p] = sum;
    atomicAdd(&vote[sum > 0 ? a : b], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int best = 0;
    for (int c = 1; c < m.n_class; ++c)
      if (vote[c] > vote[best]) best = c;
    pred[i] = best;
    if (val_out) val_out[i * val_stride] = class_values ? class_values[best] : (double)best;
  }
}

// ---- f2: SVC.predict_proba (libsvm svm_predict_probability) ---------------------------------------
// biofilm_analysis.py:1229 clf_umap.predict_proba: pairwise Platt sigmoids of the one-vs-one
// decision values (sigmoid_predict, clamped to [1e-7, 1 - 1e-7]) coupled by libsvm's
// multiclass_probability (Wu, Lin & Weng's second method: fixed-point iteration on Q p with
// the in-loop renormalisation, max(100, k) iterations, stop at max |Qp_t - pQp| < 0.005 / k).
// One wavefront per cell: the support-vector kernel values and the k x k pairwise matrix r in
// LDS; p and Qp live in registers, two classes per lane (k <= 128), and the sequential sweep
// over t broadcasts Qp[t] / Q[t][t] from the owning lane, so the sweep needs no barrier.  Every
// sum runs in libsvm's order.
constexpr int PROB_T = 64;
constexpr int PROB_KMAX = 128;
constexpr int PROB_SLOTS = PROB_KMAX / PROB_T;

__device__ __forceinline__ double platt(double dec, double A, double B) {
  const double fApB = dec * A + B;
  return fApB >= 0 ? hrf_det_exp(-fApB) / (1.0 + hrf_det_exp(-fApB)) : 1.0 / (1 + hrf_det_exp(fApB));
}

__global__ __launch_bounds__(PROB_T) void svc_proba_kernel(const double *__restrict__ x, int64_t ldx, SvcModel m,
                                                           const double *__restrict__ probA,
                                                           const double *__restrict__ probB,
                                                           double *__restrict__ prob) {
  extern __shared__ double sh[];
  const int k = m.n_class;
  double *kv = sh;
  double *r = kv + m.nsv;          // r[i * k + j]
  double *pl = r + k * k;          // p broadcast copy for the Qp products
  const int lane = threadIdx.x;
  const int64_t i = blockIdx.x;
  const double *xi = x + i * ldx;
  for (int s = lane; s < m.nsv; s += PROB_T) kv[s] = svc_kernel(xi, m.sv + (int64_t)s * m.f, m);
  __syncthreads();
  const int npair = k * (k - 1) / 2;
  for (int q = lane; q < npair; q += PROB_T) {
    auto P = [&](int64_t a) { return a * k - a * (a + 1) / 2; };
    const double nn = 2.0 * k - 1.0;
    int a = (int)floor((nn - sqrt(nn * nn - 8.0 * (double)q)) / 2.0);
    if (a < 0) a = 0;
    while (a > 0 && P(a) > q) --a;
    while (a + 1 < k && P(a + 1) <= q) ++a;
    const int b = a + 1 + (int)(q - P(a));
    const double *c1 = m.coef + (int64_t)(b - 1) * m.nsv, *c2 = m.coef + (int64_t)a * m.nsv;
    double sum = 0.0;
    for (int t = m.start[a]; t < m.start[a + 1]; ++t) sum += c1[t] * kv[t];
    for (int t = m.start[b]; t < m.start[b + 1]; ++t) sum += c2[t] * kv[t];
    sum += m.intercept[q];
    const double rr = fmin(fmax(platt(sum, probA[q], probB[q]), 1e-7), 1 - 1e-7);
    r[a * k + b] = rr;
    r[b * k + a] = 1 - rr;
  }
  __syncthreads();
  double *out = prob + i * k;   // two classes are coupled too (sklearn's libsvm has no k == 2 shortcut)
  double p[PROB_SLOTS], Qp[PROB_SLOTS], Qtt[PROB_SLOTS];
#pragma unroll
  for (int s = 0; s < PROB_SLOTS; ++s) {
    const int t = lane + s * PROB_T;
    p[s] = 1.0 / k;
    double q = 0.0;
    if (t < k) {
      for (int j = 0; j < t; ++j) q += r[j * k + t] * r[j * k + t];
      for (int j = t + 1; j < k; ++j) q += r[j * k + t] * r[j * k + t];
    }
    Qtt[s] = q;
    Qp[s] = 0.0;
  }
  const int max_iter = k > 100 ? k : 100;
  const double eps = 0.005 / k;
  for (int iter = 0; iter < max_iter; ++iter) {
#pragma unroll
    for (int s = 0; s < PROB_SLOTS; ++s)
      if (lane + s * PROB_T < k) pl[lane + s * PROB_T] = p[s];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PROB_SLOTS; ++s) {
      const int t = lane + s * PROB_T;
      double acc = 0.0;
      if (t < k)
        for (int j = 0; j < k; ++j) acc += (j == t ? Qtt[s] : -r[j * k + t] * r[t * k + j]) * pl[j];
      Qp[s] = acc;
    }
    __syncthreads();
    double pQp = 0.0, maxe = 0.0;
    for (int t = 0; t < k; ++t) pQp += pl[t] * __shfl(Qp[t / PROB_T], t % PROB_T, PROB_T);
    for (int t = 0; t < k; ++t) {
      const double e = fabs(__shfl(Qp[t / PROB_T], t % PROB_T, PROB_T) - pQp);
      if (e > maxe) maxe = e;
    }
    if (maxe < eps) break;
    for (int t = 0; t < k; ++t) {
      const double qpt = __shfl(Qp[t / PROB_T], t % PROB_T, PROB_T);
      const double qtt = __shfl(Qtt[t / PROB_T], t % PROB_T, PROB_T);
      const double diff = (-qpt + pQp) / qtt;
      pQp = (pQp + diff * (diff * qtt + 2 * qpt)) / (1 + diff) / (1 + diff);
#pragma unroll
      for (int s = 0; s < PROB_SLOTS; ++s) {
        const int j = lane + s * PROB_T;
        if (j >= k) continue;
        const double qtj = j == t ? qtt : -r[j * k + t] * r[t * k + j];
        Qp[s] = (Qp[s] + diff * qtj) / (1 + diff);
        p[s] = (j == t ? p[s] + diff : p[s]) / (1 + diff);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < PROB_SLOTS; ++s)
    if (lane + s * PROB_T < k) out[lane + s * PROB_T] = p[s];
}

// ---- f2: kNN under the reference metrics ---------------------------------------------------------
// metric 0: euclidean; 1: channel_cosine_intensity_7b_v2 (67 columns); 2: the scalar of
// channel_cosine_intensity_violet_derivative_v2 (132 columns: (d + c1 + ... + c5) / 6 -- the
// reference computes it and returns the six terms as a tuple, train_reference.py:730-731)
template <class Y>
__device__ double seg_cos(const double *x, Y y, int lo, int hi) {
  double result = 0.0, nx = 0.0, ny = 0.0;
  for (int i = lo; i < hi; ++i) {
    const double yi = y(i);
    result += x[i] * yi;
    nx += x[i] * x[i];
    ny += yi * yi;
  }
  if (nx == 0.0 && ny == 0.0) return 0.0;
  if (nx == 0.0 || ny == 0.0) return 1.0;
  return 1.0 - (result / sqrt(nx * ny));
}

template <class Y>
__device__ double knn_metric(int metric, const double *x, Y y, int f) {
  if (metric == 0) {
    double s = 0.0;
    for (int i = 0; i < f; ++i) {
      const double d = x[i] - y(i);
      s += d * d;
    }
    return sqrt(s);
  }
  if (metric == 1) {
    double check = 0.0;
    for (int i = 63; i < 67; ++i) check += fabs(x[i] - y(i));
    if (!(check < 0.01)) return 1.0;
    const int b[5] = {0, 23, 43, 57, 63};
    double c[4];
    for (int s = 0; s < 4; ++s) c[s] = x[63 + s] == 0 ? 0.0 : seg_cos(x, y, b[s], b[s + 1]);
    return 0.5 * (c[0] + c[1] + c[2] + c[3]) / 4;
  }
  double check = 0.0;
  for (int i = 126; i < 132; ++i) check += fabs(x[i] - y(i));
  const int b[6] = {0, 32, 55, 75, 89, 95};
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

constexpr int KNN_T = 256;
constexpr int KNN_KMAX = 64;
constexpr int KNN_FMAX = 160;

// one workgroup per query; trainT is feature-major (f x nt) so a chunk's rows load coalesced
__global__ __launch_bounds__(KNN_T) void knn_kernel(const double *__restrict__ q, int64_t ldq,
                                                    const double *__restrict__ trainT, int64_t nt, int32_t f,
                                                    int32_t metric, int32_t k, int32_t *__restrict__ idx_out,
                                                    double *__restrict__ dist_out) {
  __shared__ double xq[KNN_FMAX];
  __shared__ double bd[KNN_KMAX];
  __shared__ int64_t bi[KNN_KMAX];
  __shared__ double cd[KNN_T];
  __shared__ int64_t ci[KNN_T];
  __shared__ int ncand, nbest;
  const int64_t qi = blockIdx.x;
  for (int c = threadIdx.x; c < f; c += KNN_T) xq[c] = q[qi * ldq + c];
  if (threadIdx.x == 0) {
    ncand = 0;
    nbest = 0;
  }
  __syncthreads();
  for (int64_t base = 0; base < nt; base += KNN_T) {
    const int64_t r = base + threadIdx.x;
    double d = 0.0;
    bool ok = r < nt;
    if (ok) d = knn_metric(metric, xq, [&](int c) { return trainT[(int64_t)c * nt + r]; }, f);
    // a candidate beats the current k-th (ties: the lower row index, always the earlier one)
    const bool cand = ok && (nbest < k || d < bd[k - 1]);
    if (cand) {
      const int s = atomicAdd(&ncand, 1);
      cd[s] = d;
      ci[s] = r;
    }
    __syncthreads();
    if (threadIdx.x == 0 && ncand > 0) {
      // merge in row order (candidates arrived in arbitrary order: sort them by row first)
      for (int a = 1; a < ncand; ++a)
        for (int b2 = a; b2 > 0 && ci[b2] < ci[b2 - 1]; --b2) {
          const double td = cd[b2];
          cd[b2] = cd[b2 - 1];
          cd[b2 - 1] = td;
          const int64_t ti = ci[b2];
          ci[b2] = ci[b2 - 1];
          ci[b2 - 1] = ti;
        }
      for (int a = 0; a < ncand; ++a) {
        const double dv = cd[a];
        if (nbest == k && !(dv < bd[k - 1])) continue;
        int pos = nbest < k ? nbest : k - 1;
        while (pos > 0 && dv < bd[pos - 1]) {   // equal distances keep row order
          bd[pos] = bd[pos - 1];
          bi[pos] = bi[pos - 1];
          --pos;
        }
        bd[pos] = dv;
        bi[pos] = ci[a];
        if (nbest < k) ++nbest;
      }
      ncand = 0;
    }
    __syncthreads();
  }
  for (int j = threadIdx.x; j < k; j += KNN_T) {
    idx_out[qi * k + j] = j < nbest ? (int32_t)bi[j] : -1;
    dist_out[qi * k + j] = j < nbest ? bd[j] : INFINITY;
  }
}

// ---- f2: umap-learn transform (0.4 era, the reference's) ------------------------------------------
// umap_.py transform() after the neighbour search: smooth_knn_dist (n_iter 64,
// SMOOTH_K_TOLERANCE 1e-5, MIN_K_DIST_SCALE 1e-3; rho and sigma live in float32 arrays, so every
// later read sees the f32-rounded value; the psum loop skips the first neighbour),
// compute_membership_strengths (bipartite: no self-edge test; float32 values), the coo -> csr
// conversion (row entries sorted by training index), sklearn's l1 row normalisation (double row
// sum, float32 store) and init_transform (float32 products accumulated in a float32 row).
// One thread per query.
__global__ void umap_init_kernel(const int32_t *__restrict__ idx, const double *__restrict__ dist, int64_t nq,
                                 int32_t k, double n_neighbors, double local_connectivity,
                                 const double *__restrict__ mean_dev, const float *__restrict__ emb, int32_t d,
                                 float *__restrict__ memb_out, float *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const double mean_all = *mean_dev;
  const double *di = dist + i * k;
  const int32_t *ii = idx + i * k;
  const double target = hrf_det_log(n_neighbors) * 1.4426950408889634;  /* log2 */
  float rho = 0.0f;
  int nnz = 0;
  for (int j = 0; j < k; ++j) nnz += di[j] > 0.0;
  if (nnz >= local_connectivity) {
    const int index = (int)floor(local_connectivity);
    const double interp = local_connectivity - index;
    int seen = 0;
    double nz_prev = 0.0, nz_cur = 0.0, nz_first = 0.0;
    bool got_first = false;
    for (int j = 0; j < k; ++j) {
      if (!(di[j] > 0.0)) continue;
      if (!got_first) {
        nz_first = di[j];
        got_first = true;
      }
      ++seen;
      if (seen == index) nz_prev = di[j];
      if (seen == index + 1) nz_cur = di[j];
    }
    if (index > 0) {
      rho = (float)nz_prev;
      if (interp > 1e-5) rho = (float)((double)rho + interp * (nz_cur - nz_prev));
    } else {
      rho = (float)(interp * nz_first);
    }
  } else if (nnz > 0) {
    double mx = -INFINITY;
    for (int j = 0; j < k; ++j)
      if (di[j] > 0.0 && di[j] > mx) mx = di[j];
    rho = (float)mx;
  }
  double lo = 0.0, hi = INFINITY, mid = 1.0;
  for (int n = 0; n < 64; ++n) {
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
      mid = hi == INFINITY ? mid * 2 : (lo + hi) / 2.0;
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
  float w[KNN_KMAX];
  int ord[KNN_KMAX];
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
    if (memb_out) memb_out[i * k + j] = v;
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
  double s = 0.0;
  for (int a = 0; a < n; ++a) s += fabs((double)w[a]);
  for (int c = 0; c < d; ++c) out[i * d + c] = 0.0f;
  for (int a = 0; a < n; ++a) {
    const float wn = s != 0.0 ? (float)((double)w[a] / s) : w[a];
    const float *e = emb + (int64_t)ii[ord[a]] * d;
    for (int c = 0; c < d; ++c) out[i * d + c] = __fadd_rn(out[i * d + c], __fmul_rn(wn, e[c]));
  }
}

// umap's tau_rand_int (three-component Tausworthe) on unsigned 32-bit states
__device__ __forceinline__ uint32_t tau_rand(uint32_t &s0, uint32_t &s1, uint32_t &s2) {
  s0 = ((s0 & 4294967294u) << 12) ^ (((s0 << 13) ^ s0) >> 19);
  s1 = ((s1 & 4294967288u) << 4) ^ (((s1 << 2) ^ s1) >> 25);
  s2 = ((s2 & 4294967280u) << 17) ^ (((s2 << 3) ^ s2) >> 11);
  return s0 ^ s1 ^ s2;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t &x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ double umap_clip(double v) { return v > 4.0 ? 4.0 : (v < -4.0 ? -4.0 : v); }

constexpr int UMAP_DMAX = 8;

// rdist of a float32 pair: float32 differences squared in float32, summed in double (numba's
// inference for umap's rdist)
__device__ __forceinline__ double umap_rdist(const float *cur, const float *__restrict__ o, int d) {
  double r = 0.0;
  for (int c = 0; c < d; ++c) {
    const float df = cur[c] - o[c];
    r += (double)__fmul_rn(df, df);
  }
  return r;
}

// transform()'s layout refinement: the graph's edges below max / n_epochs dropped,
// make_epochs_per_sample (float32 arithmetic as numpy does it on the float32 graph), then
// optimize_layout_euclidean with the training embedding fixed (move_other False), alpha =
// initial_alpha / 4 decayed per epoch.  umap draws the negative samples from ONE sequential
// stream shared by all edges (parallel and unseeded in the reference: random_state None); here
// each query has its own stream seeded from (seed, query), so the result is deterministic and
// independent of batching.  One thread per query; its edges are visited in knn order each epoch.
__global__ void umap_refine_kernel(const int32_t *__restrict__ idx, const float *__restrict__ memb, int64_t nq,
                                   int32_t k, const float *__restrict__ wmax_dev, int32_t n_epochs,
                                   const float *__restrict__ tail, int64_t ntrain, int32_t d, double a, double b,
                                   double gamma, double alpha0, double neg_rate, uint64_t seed,
                                   float *__restrict__ emb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const float wmax = *wmax_dev;
  const float thr = (float)((double)wmax / (double)n_epochs);   // numpy 1.x: f32 max / float -> f64, compared in f32
  double eps[KNN_KMAX], eons[KNN_KMAX], eonns[KNN_KMAX];
  int32_t tl[KNN_KMAX];
  int ne = 0;
  for (int j = 0; j < k; ++j) {
    const float w = memb[i * k + j];
    if (idx[i * k + j] < 0 || !(w >= thr) || w == 0.0f) continue;   // eliminate_zeros after thresholding
    const float ns = __fmul_rn((float)n_epochs, w / wmax);
    eps[ne] = ns > 0.0f ? (double)((float)n_epochs / ns) : -1.0;
    eons[ne] = eps[ne];
    eonns[ne] = eps[ne] / neg_rate;
    tl[ne] = idx[i * k + j];
    ++ne;
  }
  float cur[UMAP_DMAX];
  for (int c = 0; c < d; ++c) cur[c] = emb[i * d + c];
  uint64_t sm = seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(i + 1));
  uint32_t s0 = (uint32_t)splitmix64(sm) | 2u, s1 = (uint32_t)splitmix64(sm) | 8u, s2 = (uint32_t)splitmix64(sm) | 16u;
  const double bm1 = b - 1.0;
  double alpha = alpha0;
  for (int n = 0; n < n_epochs; ++n) {
    for (int e = 0; e < ne; ++e) {
      if (!(eons[e] <= n)) continue;
      const float *o = tail + (int64_t)tl[e] * d;
      const double d2 = umap_rdist(cur, o, d);
      double gc = 0.0;
      if (d2 > 0.0) {
        gc = -2.0 * a * b * hrf_det_pow(d2, bm1);
        gc /= a * hrf_det_pow(d2, b) + 1.0;
      }
      for (int c = 0; c < d; ++c) {
        const double g = umap_clip(gc * (double)(cur[c] - o[c]));
        cur[c] = (float)((double)cur[c] + g * alpha);
      }
      eons[e] += eps[e];
      const double epns = eps[e] / neg_rate;
      const int nneg = (int)(((double)n - eonns[e]) / epns);
      for (int p = 0; p < nneg; ++p) {
        const int64_t kk = (int64_t)(tau_rand(s0, s1, s2) % (uint64_t)ntrain);
        const float *on = tail + kk * d;
        const double dn = umap_rdist(cur, on, d);
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
          const double g = gn > 0.0 ? umap_clip(gn * (double)(cur[c] - on[c])) : 4.0;
          cur[c] = (float)((double)cur[c] + g * alpha);
        }
      }
      eonns[e] += nneg * epns;
    }
    alpha = alpha0 * (1.0 - (double)n / (double)n_epochs);
  }
  for (int c = 0; c < d; ++c) emb[i * d + c] = cur[c];
}

}  // namespace

extern "C" {

hrf_status hrf_features_ecoli(const double *avgint_norm, int64_t n, double *out, hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(avgint_norm && out, "features_ecoli: null buffer");
  features_ecoli_kernel<<<hrf::stream_grid(n * 132), 256, 0, (hipStream_t)stream>>>(avgint_norm, n, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_features_multi(const double *avgint_norm, int64_t n, double *out, hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(avgint_norm && out, "features_multi: null buffer");
  features_multi_kernel<<<hrf::stream_grid(n * 67), 256, 0, (hipStream_t)stream>>>(avgint_norm, n, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_standard_scale(const double *x, int64_t n, int32_t f, int64_t ldx, const double *mean,
                              const double *scale, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(f >= 1 && ldx >= f, "standard_scale: bad shape");
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(x && out, "standard_scale: null buffer");
  standard_scale_kernel<<<hrf::stream_grid(n * f), 256, 0, (hipStream_t)stream>>>(x, n, f, ldx, mean, scale, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_svc_predict(const double *x, int64_t n, int64_t ldx, int32_t f, const double *sv, int32_t nsv,
                           const double *coef, const double *intercept, const int32_t *start, int32_t n_class,
                           int32_t kernel, double gamma, double coef0, int32_t degree, int32_t *pred, double *dec,
                           double *val_out, int64_t val_stride, const double *class_values, hrf_stream_t stream) {
  HRF_REQUIRE(f >= 1 && ldx >= f && nsv >= 1 && n_class >= 2 && kernel >= 0 && kernel <= 3,
              "svc_predict: bad model shape");
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(x && sv && coef && intercept && start && pred, "svc_predict: null buffer");
  const size_t shm = sizeof(double) * (size_t)nsv + sizeof(int) * (size_t)n_class + 16;
  HRF_REQUIRE(shm <= 160 * 1024, "svc_predict: %d support vectors and %d classes exceed the LDS budget", nsv, n_class);
  SvcModel m{sv, coef, intercept, start, nsv, f, n_class, kernel, degree, gamma, coef0};
  hipFuncSetAttribute((const void *)svc_predict_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  svc_predict_kernel<<<(unsigned)n, SVC_T, shm, (hipStream_t)stream>>>(x, ldx, m, pred, dec, val_out, val_stride,
                                                                       class_values);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_svc_predict_proba(const double *x, int64_t n, int64_t ldx, int32_t f, const double *sv, int32_t nsv,
                                 const double *coef, const double *intercept, const int32_t *start, int32_t n_class,
                                 int32_t kernel, double gamma, double coef0, int32_t degree, const double *probA,
                                 const double *probB, double *prob, hrf_stream_t stream) {
  HRF_REQUIRE(f >= 1 && ldx >= f && nsv >= 1 && n_class >= 2 && n_class <= PROB_KMAX && kernel >= 0 && kernel <= 3,
              "svc_predict_proba: bad model shape (2..%d classes)", PROB_KMAX);
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(x && sv && coef && intercept && start && probA && probB && prob, "svc_predict_proba: null buffer");
  const size_t shm = sizeof(double) * ((size_t)nsv + (size_t)n_class * n_class + n_class);
  HRF_REQUIRE(shm <= 160 * 1024, "svc_predict_proba: %d support vectors and %d classes exceed the LDS budget", nsv,
              n_class);
  SvcModel m{sv, coef, intercept, start, nsv, f, n_class, kernel, degree, gamma, coef0};
  hipFuncSetAttribute((const void *)svc_proba_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  svc_proba_kernel<<<(unsigned)n, PROB_T, shm, (hipStream_t)stream>>>(x, ldx, m, probA, probB, prob);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_knn(const double *q, int64_t nq, int64_t ldq, const double *trainT, int64_t nt, int32_t f,
                   int32_t metric, int32_t k, int32_t *idx_out, double *dist_out, hrf_stream_t stream) {
  HRF_REQUIRE(metric >= 0 && metric <= 2, "knn: metric must be 0 (euclidean), 1 (7b_v2) or 2 (violet_derivative_v2)");
  HRF_REQUIRE(f >= 1 && f <= KNN_FMAX && ldq >= f, "knn: 1..%d features", KNN_FMAX);
  HRF_REQUIRE(metric != 1 || f == 67, "knn: channel_cosine_intensity_7b_v2 needs 67 columns");
  HRF_REQUIRE(metric != 2 || f == 132, "knn: channel_cosine_intensity_violet_derivative_v2 needs 132 columns");
  HRF_REQUIRE(k >= 1 && k <= KNN_KMAX && nt >= 1, "knn: 1..%d neighbours of a non-empty table", KNN_KMAX);
  if (nq == 0) return HRF_OK;
  HRF_REQUIRE(q && trainT && idx_out && dist_out, "knn: null buffer");
  knn_kernel<<<(unsigned)nq, KNN_T, 0, (hipStream_t)stream>>>(q, ldq, trainT, nt, f, metric, k, idx_out, dist_out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_umap_init_transform(const int32_t *knn_idx, const double *knn_dist, int64_t nq, int32_t k,
                                   double n_neighbors, double local_connectivity, const double *mean_dist_dev,
                                   const float *embedding, int32_t d, float *memb_out, float *out,
                                   hrf_stream_t stream) {
  HRF_REQUIRE(k >= 1 && k <= KNN_KMAX && d >= 1, "umap_init_transform: bad shape");
  if (nq == 0) return HRF_OK;
  HRF_REQUIRE(knn_idx && knn_dist && mean_dist_dev && embedding && out, "umap_init_transform: null buffer");
  umap_init_kernel<<<(unsigned)hrf::cdiv(nq, 64), 64, 0, (hipStream_t)stream>>>(
      knn_idx, knn_dist, nq, k, n_neighbors, local_connectivity, mean_dist_dev, embedding, d, memb_out, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_umap_refine(const int32_t *knn_idx, const float *memb, int64_t nq, int32_t k, const float *wmax_dev,
                           int32_t n_epochs, const float *tail_embedding, int64_t ntrain, int32_t d, double a,
                           double b, double repulsion_strength, double initial_alpha, double negative_sample_rate,
                           uint64_t seed, float *embedding, hrf_stream_t stream) {
  HRF_REQUIRE(k >= 1 && k <= KNN_KMAX && d >= 1 && d <= UMAP_DMAX, "umap_refine: 1..%d neighbours, 1..%d dims",
              KNN_KMAX, UMAP_DMAX);
  HRF_REQUIRE(n_epochs >= 1 && ntrain >= 1 && negative_sample_rate > 0, "umap_refine: bad schedule");
  if (nq == 0) return HRF_OK;
  HRF_REQUIRE(knn_idx && memb && wmax_dev && tail_embedding && embedding, "umap_refine: null buffer");
  umap_refine_kernel<<<(unsigned)hrf::cdiv(nq, 64), 64, 0, (hipStream_t)stream>>>(
      knn_idx, memb, nq, k, wmax_dev, n_epochs, tail_embedding, ntrain, d, a, b, repulsion_strength, initial_alpha,
      negative_sample_rate, seed, embedding);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
