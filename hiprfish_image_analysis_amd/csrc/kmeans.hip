// kmeans.hip -- 1-D KMeans thresholding (a8).
//
// Reference: sklearn KMeans(n_clusters=k, random_state=0).fit_predict(x.reshape(-1,1))
// (ecoli measurement.py:73,85; multispecies :125,141).  Restated (oracle/hrf_oracle.c
// oracle_kmeans_1d) as Lloyd iterations from a deterministic init with EXACT centre updates:
// each value is mapped to int64 fixed point q = rint(x * 2^s) once per pass and summed with
// integer atomics, so the centres -- and therefore every label -- are independent of the
// reduction order and identical to the CPU restatement bit for bit.
//
// Device-resident loop: ONE launch per Lloyd iteration.  Launch `it` first applies update
// number `it` (every block derives the same centres from the previous launch's integer sums),
// then streams the data once accumulating into a rotating sum buffer; it exits at once when
// converged, so the host launches batches and polls rarely.
//
// Sorted path (hrf_kmeans_1d_sorted, the one the pipelines use): the valid values are sorted
// once by value bucket (2^20 equal-width buckets, rocPRIM radix sort of 20-bit keys with the
// values as payload) and their fixed-point values prefix-summed in that order.  With ascending, well separated centres the label
// argmin_j (x - c_j)^2 (first minimum) is a non-decreasing step function of x, so one Lloyd
// iteration reduces to locating the k - 1 label steps in the bucket-ordered array (a 4096-ary
// search by one 1024-thread workgroup that narrows to whole buckets, then counts the few
// values of the straddling bucket) and reading cluster sums and counts off the prefix array:
// the same integer sums, hence the same centres, as the streaming pass -- with all iterations
// in ONE launch and no per-iteration pass over the data.  A sort can serve several k on the
// same input (E. coli :73 and :85 both cluster image_cn).  Whenever the step-function premise
// cannot be guaranteed (a NaN among the values, centres not strictly ascending or closer than
// 2^-40 of the data range) the call reruns the streaming path.
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.hpp"
#include "wave.hpp"

namespace {

constexpr int KMAX = 8;

struct KmState {
  double center[KMAX];         // final centres (read by the host and km_label_kernel)
  double cen[2][KMAX];         // centres used by launch it live in cen[it & 1]
  long long sum[3][KMAX];      // launch it accumulates into sum[it % 3]
  unsigned long long cnt[3][KMAX];
  unsigned long long lo_bits, hi_bits;  // order-preserving encodings of min / max
  unsigned long long amax_bits;         // |x| max (non-negative doubles order as uint64)
  unsigned long long nvalid;
  unsigned long long nnan;              // NaN values among the valid ones (sorted path: fall back)
  int scale;
  int converged;
  int iters;
  int k;
  int fallback;                         // sorted path could not guarantee the step premise
};

__device__ __forceinline__ unsigned long long ord_enc(double x) {
  const unsigned long long b = __double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double ord_dec(unsigned long long e) {
  const unsigned long long b = (e >> 63) ? (e & 0x7fffffffffffffffull) : ~e;
  return __longlong_as_double((long long)b);
}

__global__ void km_minmax_kernel(const double *__restrict__ x, const uint8_t *__restrict__ valid, int64_t n,
                                 KmState *st) {
  unsigned long long lo = ~0ull, hi = 0ull, am = 0ull, nv = 0ull, nn = 0ull;
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += T * 8) {
    double vv[8];
    bool ok[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t k = i + e * T;
      ok[e] = k < n;
      vv[e] = ok[e] ? x[k] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (!ok[e] || (valid && !valid[i + e * T])) continue;
      const double v = vv[e];
      const unsigned long long en = ord_enc(v);
      lo = en < lo ? en : lo;
      hi = en > hi ? en : hi;
      const unsigned long long a = (unsigned long long)__double_as_longlong(fabs(v));
      am = a > am ? a : am;
      nv += 1;
      nn += v != v;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64), a2 = __shfl_xor(am, o, 64);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
    am = a2 > am ? a2 : am;
    nv += __shfl_xor(nv, o, 64);
    nn += __shfl_xor(nn, o, 64);
  }
  __shared__ unsigned long long red[4][5];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = lo;
    red[w][1] = hi;
    red[w][2] = am;
    red[w][3] = nv;
    red[w][4] = nn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) {
      lo = red[q][0] < lo ? red[q][0] : lo;
      hi = red[q][1] > hi ? red[q][1] : hi;
      am = red[q][2] > am ? red[q][2] : am;
      nv += red[q][3];
      nn += red[q][4];
    }
    atomicMin(&st->lo_bits, lo);
    atomicMax(&st->hi_bits, hi);
    atomicMax(&st->amax_bits, am);
    atomicAdd(&st->nvalid, nv);
    if (nn) atomicAdd(&st->nnan, nn);
  }
}

__global__ void km_init_kernel(KmState *st, int k) {
  const double mn = ord_dec(st->lo_bits), mx = ord_dec(st->hi_bits);
  const double amax = __longlong_as_double((long long)st->amax_bits);
  int e = 0;
  frexp(amax > 0 ? amax : 1.0, &e);
  const unsigned long long nv = st->nvalid;
  int ln = 0;
  while ((1ull << ln) < (nv > 1 ? nv : 1ull)) ++ln;
  st->scale = 61 - ln - e;
  for (int j = 0; j < KMAX; ++j) {
    st->center[j] = j < k ? mn + ((double)j + 0.5) * (mx - mn) / (double)k : 0.0;
    st->cen[0][j] = st->cen[1][j] = st->center[j];  // launch 0 reads cen[1]
    st->sum[0][j] = 0;
    st->cnt[0][j] = 0;
  }
  st->k = k;
  st->converged = nv == 0;
  st->iters = 0;
  st->fallback = 0;
}

constexpr int KM_E = 8;  // elements in flight per thread

template <int K>
__device__ __forceinline__ int km_assign(double v, const double *c) {
  int bj = 0;
  double bd = (v - c[0]) * (v - c[0]);
#pragma unroll
  for (int j = 1; j < K; ++j) {
    const double d = (v - c[j]) * (v - c[j]);
    if (d < bd) {
      bd = d;
      bj = j;
    }
  }
  return bj;
}

template <int K>
__global__ __launch_bounds__(256) void km_step_kernel(const double *__restrict__ x, const uint8_t *__restrict__ valid,
                                                     int64_t n, KmState *st, int it, int max_iter) {
  if (st->converged) return;
  const int s = st->scale;
  double c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) c[j] = st->cen[(it + 1) & 1][j];
  if (it > 0) {
    // update number `it` (the former km_update_kernel), identical in every block
    const int pb = (it + 2) % 3;
    int changed = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const unsigned long long cn = st->cnt[pb][j];
      if (cn) {
        const double cj = ldexp((double)st->sum[pb][j] / (double)cn, -s);
        if (cj != c[j]) changed = 1;
        c[j] = cj;
      }
    }
    if (!changed || it >= max_iter) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int j = 0; j < K; ++j) st->center[j] = c[j];
        st->iters = it;
        st->converged = 1;
      }
      return;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < K) {
    st->cen[it & 1][threadIdx.x] = c[threadIdx.x];
    st->sum[(it + 1) % 3][threadIdx.x] = 0;
    st->cnt[(it + 1) % 3][threadIdx.x] = 0;
  }
  long long sum[K];
  unsigned long long cnt[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    sum[j] = 0;
    cnt[j] = 0;
  }
  // KM_E strided elements per thread per round, all loads issued before any is used: the pass
  // is bound by memory-level parallelism, not arithmetic
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += T * KM_E) {
    double v[KM_E];
    bool ok[KM_E];
#pragma unroll
    for (int e = 0; e < KM_E; ++e) {
      const int64_t k = i + e * T;
      ok[e] = k < n;
      v[e] = ok[e] ? x[k] : 0.0;
    }
    if (valid) {
#pragma unroll
      for (int e = 0; e < KM_E; ++e) ok[e] = ok[e] && valid[i + e * T];
    }
#pragma unroll
    for (int e = 0; e < KM_E; ++e) {
      if (!ok[e]) continue;
      const int bj = km_assign<K>(v[e], c);
      const long long q = (long long)rint(ldexp(v[e], s));
#pragma unroll
      for (int j = 0; j < K; ++j) {
        sum[j] += bj == j ? q : 0;
        cnt[j] += bj == j;
      }
    }
  }
  __shared__ long long ssum[4][K];
  __shared__ unsigned long long scnt[4][K];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const long long a = hrf::wave_sum(sum[j]);
    const unsigned long long b = hrf::wave_sum(cnt[j]);
    if ((threadIdx.x & 63) == 0) {
      ssum[w][j] = a;
      scnt[w][j] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < K) {
    const int j = threadIdx.x;
    const long long a = ssum[0][j] + ssum[1][j] + ssum[2][j] + ssum[3][j];
    const unsigned long long b = scnt[0][j] + scnt[1][j] + scnt[2][j] + scnt[3][j];
    if (b) {
      atomicAdd((unsigned long long *)&st->sum[it % 3][j], (unsigned long long)a);
      atomicAdd(&st->cnt[it % 3][j], b);
    }
  }
}

template <int K>
__global__ void km_label_kernel(const double *__restrict__ x, const uint8_t *__restrict__ valid, int64_t n,
                                const KmState *st, int32_t *__restrict__ labels, uint8_t *__restrict__ top) {
  double c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) c[j] = st->center[j];
  int jt = 0;
#pragma unroll
  for (int j = 1; j < K; ++j)
    if (c[j] > c[jt]) jt = j;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool ok = !valid || valid[i];
    const int bj = ok ? km_assign<K>(x[i], c) : -1;
    if (labels) labels[i] = bj;
    if (top) top[i] = (uint8_t)(bj == jt);
  }
}

template <int K>
hrf_status km_run(const double *x, const uint8_t *valid, int64_t n, int max_iter, int32_t *labels, uint8_t *top,
                  double *centers_host, int32_t *iters_host, KmState *st, hipStream_t s) {
  const unsigned g = hrf::stream_grid(n);
  const unsigned gr = std::min<unsigned>(g, 512);
  KmState init{};
  for (int j = 0; j < KMAX; ++j) init.center[j] = 0;
  init.lo_bits = ~0ull;
  init.hi_bits = 0;
  init.amax_bits = 0;
  init.nvalid = 0;
  HRF_HIP(hipMemcpyAsync(st, &init, sizeof(KmState), hipMemcpyHostToDevice, s));
  if (n > 0) km_minmax_kernel<<<gr, 256, 0, s>>>(x, valid, n, st);
  km_init_kernel<<<1, 1, 0, s>>>(st, K);
  HRF_LAUNCHED();
  int done = 0;
  int launched = 0;
  int batch = 4;
  int conv = 0;
  while (!done) {
    // launch `it` applies update `it`; update max_iter ends the fit, so at most max_iter + 1
    for (int b = 0; b < batch && launched <= max_iter; ++b, ++launched)
      km_step_kernel<K><<<gr, 256, 0, s>>>(x, valid, n, st, launched, max_iter);
    HRF_LAUNCHED();
    HRF_HIP(hipMemcpyAsync(&conv, &st->converged, sizeof(int), hipMemcpyDeviceToHost, s));
    HRF_HIP(hipStreamSynchronize(s));
    done = conv || launched > max_iter;
    batch = batch < 16 ? batch * 2 : 16;
  }
  if (n > 0) km_label_kernel<K><<<g, 256, 0, s>>>(x, valid, n, st, labels, top);
  HRF_LAUNCHED();
  KmState fin;
  HRF_HIP(hipMemcpyAsync(&fin, st, sizeof(KmState), hipMemcpyDeviceToHost, s));
  HRF_HIP(hipStreamSynchronize(s));
  if (centers_host)
    for (int j = 0; j < K; ++j) centers_host[j] = fin.center[j];
  if (iters_host) *iters_host = fin.iters;
  return HRF_OK;
}


// ---- sorted path: sort by value bucket ------------------------------------------------------
// NB value buckets of equal width over [min, max]; bucket(x) is a non-decreasing function of
// x, so every value of bucket b is below every value of bucket b' > b.  The valid values are
// radix sorted by their 20-bit bucket index (rocPRIM pairs, 3 digit passes instead of 8 for
// full 64-bit keys; invalid entries get key NB and land past them), in no particular order
// inside a bucket -- only integer sums are read off the result, so that order never shows.
// off[b] = first position of bucket b, then the fixed-point encodings are prefix-summed.
constexpr int KM_NB = 1 << 20;
constexpr int KM_NB_BITS = 21;  // keys 0..NB inclusive

__device__ __forceinline__ int km_bucket(double x, double mn, double inv) {
  const double t = (x - mn) * inv;
  return t >= 0.0 ? (t < (double)(KM_NB - 1) ? (int)t : KM_NB - 1) : 0;  // NaN -> 0
}

// bucket geometry from the min / max found by km_minmax_kernel
__global__ void km_bucket_init_kernel(KmState *st, double *geo) {
  const double mn = ord_dec(st->lo_bits), mx = ord_dec(st->hi_bits);
  geo[0] = mn;
  geo[1] = mx > mn ? (double)KM_NB / (mx - mn) : 0.0;
}

__global__ void km_bucket_key_kernel(const double *__restrict__ x, const uint8_t *__restrict__ valid, int64_t n,
                                     const double *__restrict__ geo, uint32_t *__restrict__ key) {
  const double mn = geo[0], inv = geo[1];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    key[i] = (!valid || valid[i]) ? (uint32_t)km_bucket(x[i], mn, inv) : (uint32_t)KM_NB;
}

// off[b] = first sorted position whose key is >= b (b = 0..NB, a binary search each, so empty
// stretches of buckets cost nothing extra); q = fixed-point values in sorted order
__global__ void km_bucket_bounds_kernel(const uint32_t *__restrict__ key, const double *__restrict__ xs, int64_t n,
                                        const KmState *st, unsigned long long *__restrict__ off,
                                        long long *__restrict__ q, long long *__restrict__ prefix0) {
  const int s = st->scale;
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t0 == 0) *prefix0 = 0;
  for (int64_t b = t0; b <= KM_NB; b += T) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)key[mid] < b) lo = mid + 1;
      else hi = mid;
    }
    off[b] = (unsigned long long)lo;
  }
  for (int64_t i = t0; i < n; i += T) q[i] = (long long)rint(ldexp(xs[i], s));
}

constexpr int KS_T = 1024;           // threads of the iteration workgroup
constexpr int KS_P = 4;              // probes per thread per round -> 4096-ary search
static_assert(KS_T * KS_P == 4096, "index arithmetic below shifts by 12");

// For label step j (labels <= j versus > j): the number of bucket-ordered values with label
// <= j and the sum of their fixed-point encodings.  Invariant: the range [lo, hi) starts and
// ends on bucket boundaries, every value before it has label <= j and every value after it
// label > j (labels are non-decreasing in the value, buckets are ordered by value).  A round
// probes 4096 evenly spaced values: the range shrinks to [start of the last bucket holding a
// "<= j" probe, end of the first bucket holding a "> j" probe).  A range of <= 4096 values, or
// one that a round could not halve, is counted exhaustively.
template <int K>
__device__ void km_bucket_step(const double *__restrict__ xs, const long long *__restrict__ q,
                               const long long *__restrict__ prefix, const unsigned long long *__restrict__ off,
                               int64_t nv, double mn, double inv, double range, const double *c, int j,
                               int64_t *cnt_le, long long *sum_le) {
  const int t = threadIdx.x;
  __shared__ int64_t lo_sh, hi_sh;
  __shared__ int bf_sh, bt_sh, exh_sh;
  __shared__ unsigned long long nf_sh;
  __shared__ long long sf_sh;
  if (t == 0) {
    // Direct bracket: the label step lies within delta of the midpoint m (the comparison's
    // rounding moves it by ~2^-53 of the centre gap; delta is 2^-40 of the magnitudes), and
    // km_bucket is monotone in the value, so every value in a bucket below bucket(m - delta)
    // has label <= j and every value in a bucket above bucket(m + delta) label > j.  The
    // range then starts on those bucket boundaries instead of [0, nv).
    const double m = 0.5 * c[j] + 0.5 * c[j + 1];
    const double delta = (fabs(c[j]) + fabs(c[j + 1]) + range) * 0x1p-40;
    const int blo = km_bucket(m - delta, mn, inv), bhi = km_bucket(m + delta, mn, inv);
    const int64_t lo = (int64_t)off[blo], hi = (int64_t)off[bhi + 1];
    lo_sh = lo < 0 ? 0 : (lo > nv ? nv : lo);
    hi_sh = hi < lo_sh ? lo_sh : (hi > nv ? nv : hi);
    exh_sh = 0;
  }
  __syncthreads();
  while (true) {
    const int64_t lo = lo_sh, hi = hi_sh;
    const int64_t len = hi - lo;
    if (exh_sh || len <= (int64_t)KS_T * KS_P) {
      // count the range exhaustively: values with label <= j and the sum of their encodings
      if (t == 0) {
        nf_sh = 0;
        sf_sh = 0;
      }
      __syncthreads();
      unsigned long long nf = 0;
      long long sf = 0;
      const long long plo = t == 0 ? prefix[lo] : 0;  // issued before the scan's loads
      for (int64_t idx = lo + t; idx < hi; idx += KS_T)
        if (km_assign<K>(xs[idx], c) <= j) {
          nf += 1;
          sf += q[idx];
        }
      nf = hrf::wave_sum(nf);
      sf = hrf::wave_sum(sf);
      if ((t & 63) == 0 && nf) {
        atomicAdd(&nf_sh, nf);
        atomicAdd((unsigned long long *)&sf_sh, (unsigned long long)sf);
      }
      __syncthreads();
      if (t == 0) {
        *cnt_le = lo + (int64_t)nf_sh;
        *sum_le = plo + sf_sh;
      }
      __syncthreads();
      return;
    }
    if (t == 0) {
      bf_sh = -1;
      bt_sh = KM_NB;
    }
    __syncthreads();
    int bf = -1, bt = KM_NB;
#pragma unroll
    for (int p = 0; p < KS_P; ++p) {
      const int64_t idx = lo + ((len * (t * KS_P + p)) >> 12);  // KS_T * KS_P = 4096; len < 2^51
      const double v = xs[idx];
      const int b = km_bucket(v, mn, inv);
      if (km_assign<K>(v, c) <= j) bf = b > bf ? b : bf;
      else bt = b < bt ? b : bt;
    }
    if (bf >= 0) atomicMax(&bf_sh, bf);
    if (bt < KM_NB) atomicMin(&bt_sh, bt);
    __syncthreads();
    if (t == 0) {
      const int64_t nlo = bf_sh >= 0 ? (int64_t)off[bf_sh] : lo;
      const int64_t nhi = bt_sh < KM_NB ? (int64_t)off[bt_sh + 1] : hi;
      const int64_t clo = nlo > lo ? nlo : lo, chi = nhi < hi ? nhi : hi;
      exh_sh = 2 * (chi - clo) > len;  // few buckets hold the range: no real progress
      lo_sh = clo;
      hi_sh = chi;
    }
    __syncthreads();
  }
}

template <int K>
__global__ __launch_bounds__(KS_T) void km_sorted_iter_kernel(const double *__restrict__ xs,
                                                              const long long *__restrict__ q,
                                                              const long long *__restrict__ prefix,
                                                              const unsigned long long *__restrict__ off,
                                                              const double *__restrict__ geo, KmState *st,
                                                              int max_iter) {
  __shared__ double c[KMAX];
  __shared__ int64_t cle[KMAX];
  __shared__ long long sle[KMAX];
  __shared__ int stop;
  const int t = threadIdx.x;
  const int64_t nv = (int64_t)st->nvalid;
  const int s = st->scale;
  const double mn = geo[0], inv = geo[1];
  if (t < K) c[t] = st->center[t];
  if (t == 0) stop = 0;
  __syncthreads();
  if (nv == 0) {
    if (t == 0) st->iters = 0;
    return;
  }
  if (st->nnan) {
    if (t == 0) st->fallback = 1;
    return;
  }
  const double range = ord_dec(st->hi_bits) - ord_dec(st->lo_bits);
  int it;
  for (it = 1; it <= max_iter; ++it) {
    if (t == 0) {
      // premise of the step search: strictly ascending, well separated centres
      for (int j = 0; j + 1 < K; ++j)
        if (!(c[j + 1] - c[j] > range * 0x1p-40)) stop = 2;
    }
    __syncthreads();
    if (stop) break;
    for (int j = 0; j + 1 < K; ++j) km_bucket_step<K>(xs, q, prefix, off, nv, mn, inv, range, c, j, &cle[j], &sle[j]);
    if (t == 0) {
      int changed = 0;
      int64_t c0 = 0;
      long long s0 = 0;
      for (int j = 0; j < K; ++j) {
        const int64_t c1 = j < K - 1 ? cle[j] : nv;
        const long long s1 = j < K - 1 ? sle[j] : prefix[nv];
        const int64_t cn = c1 - c0;
        if (cn) {
          const double cj = ldexp((double)(s1 - s0) / (double)cn, -s);
          if (cj != c[j]) changed = 1;
          c[j] = cj;
        }
        c0 = c1;
        s0 = s1;
      }
      if (!changed) stop = 1;
    }
    __syncthreads();
    if (stop) break;
  }
  if (t == 0) {
    if (stop == 2) {
      st->fallback = 1;
    } else {
      for (int j = 0; j < K; ++j) st->center[j] = c[j];
      st->iters = it > max_iter ? max_iter : it;
      st->converged = 1;
    }
  }
}

struct SortWs {
  KmState *st;
  double *geo;
  uint32_t *key_in, *key;
  unsigned long long *off;
  double *xs;
  long long *q, *prefix;
  void *tmp;
  size_t tmp_bytes;
};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

hrf_status sort_tmp_bytes(int64_t n, size_t *bytes) {
  size_t a = 0, b = 0;
  const size_t m = (size_t)std::max<int64_t>(n, 1);
  HRF_HIP(rocprim::radix_sort_pairs(nullptr, a, (uint32_t *)nullptr, (uint32_t *)nullptr, (const double *)nullptr,
                                    (double *)nullptr, m, 0, KM_NB_BITS, (hipStream_t)0));
  HRF_HIP(rocprim::inclusive_scan(nullptr, b, (const unsigned long long *)nullptr, (unsigned long long *)nullptr, m,
                                  rocprim::plus<unsigned long long>(), (hipStream_t)0));
  *bytes = std::max(a, b);
  return HRF_OK;
}

int64_t sort_ws_bytes(int64_t n, size_t tmp_bytes) {
  const size_t m = (size_t)std::max<int64_t>(n, 1);
  return (int64_t)(align256(sizeof(KmState)) + 256 + 2 * align256(sizeof(uint32_t) * m) +
                   align256(sizeof(unsigned long long) * (KM_NB + 1)) + 2 * align256(sizeof(double) * m) +
                   align256(sizeof(long long) * (m + 1)) + align256(tmp_bytes));
}

SortWs carve(void *work, int64_t n, size_t tmp_bytes) {
  char *w = (char *)work;
  const size_t m = (size_t)std::max<int64_t>(n, 1);
  SortWs ws{};
  ws.st = (KmState *)w;
  w += align256(sizeof(KmState));
  ws.geo = (double *)w;
  w += 256;
  ws.key_in = (uint32_t *)w;
  w += align256(sizeof(uint32_t) * m);
  ws.key = (uint32_t *)w;
  w += align256(sizeof(uint32_t) * m);
  ws.off = (unsigned long long *)w;
  w += align256(sizeof(unsigned long long) * (KM_NB + 1));
  ws.xs = (double *)w;
  w += align256(sizeof(double) * m);
  ws.q = (long long *)w;
  w += align256(sizeof(double) * m);
  ws.prefix = (long long *)w;
  w += align256(sizeof(long long) * (m + 1));
  ws.tmp = w;
  ws.tmp_bytes = tmp_bytes;
  return ws;
}

// Enqueue the sorted path (sort unless `reuse`, iterations, labels) and the read-back of its
// final state into *fin (host); the caller synchronises before km_sorted_finish reads it.
template <int K>
hrf_status km_sorted_launch(const double *x, const uint8_t *valid, int64_t n, int max_iter, int32_t *labels,
                            uint8_t *top, const SortWs &ws, int reuse, hipStream_t s, KmState *fin) {
  KmState *st = ws.st;
  const unsigned g = hrf::stream_grid(n);
  if (!reuse) {
    KmState init{};
    init.lo_bits = ~0ull;
    HRF_HIP(hipMemcpyAsync(st, &init, sizeof(KmState), hipMemcpyHostToDevice, s));
    if (n > 0) km_minmax_kernel<<<std::min<unsigned>(g, 512), 256, 0, s>>>(x, valid, n, st);
    HRF_LAUNCHED();
  }
  km_init_kernel<<<1, 1, 0, s>>>(st, K);
  HRF_LAUNCHED();
  if (!reuse && n > 0) {
    km_bucket_init_kernel<<<1, 1, 0, s>>>(st, ws.geo);
    km_bucket_key_kernel<<<g, 256, 0, s>>>(x, valid, n, ws.geo, ws.key_in);
    HRF_LAUNCHED();
    size_t tb = ws.tmp_bytes;
    HRF_HIP(rocprim::radix_sort_pairs(ws.tmp, tb, ws.key_in, ws.key, x, ws.xs, (size_t)n, 0, KM_NB_BITS, s));
    km_bucket_bounds_kernel<<<hrf::stream_grid(std::max<int64_t>(n, KM_NB + 1)), 256, 0, s>>>(ws.key, ws.xs, n, st, ws.off, ws.q, ws.prefix);
    HRF_LAUNCHED();
    tb = ws.tmp_bytes;
    // entries past the valid values (invalid ones, sorted last) are never read back: the scan
    // covers all n in unsigned (wrapping) arithmetic; prefixes up to nvalid are the exact sums
    HRF_HIP(rocprim::inclusive_scan(ws.tmp, tb, (const unsigned long long *)ws.q, (unsigned long long *)ws.prefix + 1,
                                    (size_t)n, rocprim::plus<unsigned long long>(), s));
  }
  km_sorted_iter_kernel<K><<<1, KS_T, 0, s>>>(ws.xs, ws.q, ws.prefix, ws.off, ws.geo, st, max_iter);
  HRF_LAUNCHED();
  if (n > 0) km_label_kernel<K><<<g, 256, 0, s>>>(x, valid, n, st, labels, top);
  HRF_LAUNCHED();
  HRF_HIP(hipMemcpyAsync(fin, st, sizeof(KmState), hipMemcpyDeviceToHost, s));
  return HRF_OK;
}

// After the synchronisation: NaN input or merging centres send the call to the streaming
// path, which recomputes everything (labels, top mask) in the workspace's state block.
template <int K>
hrf_status km_sorted_finish(const double *x, const uint8_t *valid, int64_t n, int max_iter, int32_t *labels,
                            uint8_t *top, double *centers_host, int32_t *iters_host, const SortWs &ws,
                            hipStream_t s, const KmState &fin) {
  KmState *st = ws.st;
  if (fin.fallback) {
    // the streaming path recomputes everything from scratch in its own state block
    if (hrf_status r = km_run<K>(x, valid, n, max_iter, labels, top, centers_host, iters_host, st, s)) return r;
    return HRF_OK;
  }
  if (centers_host)
    for (int j = 0; j < K; ++j) centers_host[j] = fin.center[j];
  if (iters_host) *iters_host = fin.iters;
  return HRF_OK;
}

template <int K>
hrf_status km_run_sorted(const double *x, const uint8_t *valid, int64_t n, int max_iter, int32_t *labels,
                         uint8_t *top, double *centers_host, int32_t *iters_host, const SortWs &ws, int reuse,
                         hipStream_t s) {
  KmState fin;
  if (hrf_status r = km_sorted_launch<K>(x, valid, n, max_iter, labels, top, ws, reuse, s, &fin)) return r;
  HRF_HIP(hipStreamSynchronize(s));
  return km_sorted_finish<K>(x, valid, n, max_iter, labels, top, centers_host, iters_host, ws, s, fin);
}

hrf_status km_launch_k(int k, const double *x, const uint8_t *valid, int64_t n, int max_iter, uint8_t *top,
                       const SortWs &ws, int reuse, hipStream_t s, KmState *fin) {
  switch (k) {
#define HRF_KML(KK) \
  case KK: return km_sorted_launch<KK>(x, valid, n, max_iter, nullptr, top, ws, reuse, s, fin);
    HRF_KML(1) HRF_KML(2) HRF_KML(3) HRF_KML(4) HRF_KML(5) HRF_KML(6) HRF_KML(7)
#undef HRF_KML
    default: return km_sorted_launch<8>(x, valid, n, max_iter, nullptr, top, ws, reuse, s, fin);
  }
}

hrf_status km_finish_k(int k, const double *x, const uint8_t *valid, int64_t n, int max_iter, uint8_t *top,
                       const SortWs &ws, hipStream_t s, const KmState &fin) {
  switch (k) {
#define HRF_KMF(KK) \
  case KK: return km_sorted_finish<KK>(x, valid, n, max_iter, nullptr, top, nullptr, nullptr, ws, s, fin);
    HRF_KMF(1) HRF_KMF(2) HRF_KMF(3) HRF_KMF(4) HRF_KMF(5) HRF_KMF(6) HRF_KMF(7)
#undef HRF_KMF
    default: return km_sorted_finish<8>(x, valid, n, max_iter, nullptr, top, nullptr, nullptr, ws, s, fin);
  }
}

}  // namespace

extern "C" {

int64_t hrf_kmeans_state_bytes(void) { return (int64_t)sizeof(KmState); }

hrf_status hrf_kmeans_1d(const double *x, const uint8_t *valid, int64_t n, int32_t k, int32_t max_iter,
                         int32_t *labels, uint8_t *top_mask, double *centers_host, int32_t *iters_host, void *state_ws,
                         hrf_stream_t stream) {
  HRF_REQUIRE(k >= 1 && k <= KMAX, "kmeans_1d: k must be 1..8");
  HRF_REQUIRE(n >= 0 && max_iter >= 1 && state_ws, "kmeans_1d: bad arguments");
  HRF_REQUIRE(n == 0 || x, "kmeans_1d: null input");
  hipStream_t s = (hipStream_t)stream;
  KmState *st = (KmState *)state_ws;
  switch (k) {
    case 1: return km_run<1>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
    case 2: return km_run<2>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
    case 3: return km_run<3>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
    case 4: return km_run<4>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
    case 5: return km_run<5>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
    case 6: return km_run<6>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
    case 7: return km_run<7>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
    default: return km_run<8>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, st, s);
  }
}

int64_t hrf_kmeans_sorted_workspace_bytes(int64_t n) {
  size_t tb = 0;
  if (sort_tmp_bytes(n, &tb) != HRF_OK) return -1;
  return sort_ws_bytes(n, tb);
}

hrf_status hrf_kmeans_1d_sorted(const double *x, const uint8_t *valid, int64_t n, int32_t k, int32_t max_iter,
                                int32_t *labels, uint8_t *top_mask, double *centers_host, int32_t *iters_host,
                                void *work, int64_t work_bytes, int32_t reuse_sort, hrf_stream_t stream) {
  HRF_REQUIRE(k >= 1 && k <= KMAX, "kmeans_1d: k must be 1..8");
  HRF_REQUIRE(n >= 0 && max_iter >= 1 && work, "kmeans_1d: bad arguments");
  HRF_REQUIRE(n == 0 || x, "kmeans_1d: null input");
  const int64_t need = hrf_kmeans_sorted_workspace_bytes(n);
  HRF_REQUIRE(need > 0, "kmeans_1d: workspace size query failed");
  if (work_bytes < need) {
    ::hrf::set_error("kmeans_1d: workspace of %lld bytes, %lld needed", (long long)work_bytes, (long long)need);
    return HRF_ENOMEM;
  }
  size_t tb = 0;
  if (hrf_status r = sort_tmp_bytes(n, &tb)) return r;
  const SortWs ws = carve(work, n, tb);
  hipStream_t s = (hipStream_t)stream;
  switch (k) {
#define HRF_KMS(KK) \
  case KK: return km_run_sorted<KK>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, ws, reuse_sort, s);
    HRF_KMS(1) HRF_KMS(2) HRF_KMS(3) HRF_KMS(4) HRF_KMS(5) HRF_KMS(6) HRF_KMS(7)
#undef HRF_KMS
    default: return km_run_sorted<8>(x, valid, n, max_iter, labels, top_mask, centers_host, iters_host, ws, reuse_sort, s);
  }
}

hrf_status hrf_kmeans_1d_sorted_pair(const double *x, const uint8_t *valid, int64_t n, int32_t k1, int32_t k2,
                                     int32_t max_iter, uint8_t *top1, uint8_t *top2, void *work, int64_t work_bytes,
                                     hrf_stream_t stream) {
  HRF_REQUIRE(k1 >= 1 && k1 <= KMAX && k2 >= 1 && k2 <= KMAX, "kmeans_1d_pair: k must be 1..8");
  HRF_REQUIRE(n >= 0 && max_iter >= 1 && work, "kmeans_1d_pair: bad arguments");
  HRF_REQUIRE(n == 0 || x, "kmeans_1d_pair: null input");
  const int64_t need = hrf_kmeans_sorted_workspace_bytes(n);
  HRF_REQUIRE(need > 0, "kmeans_1d_pair: workspace size query failed");
  if (work_bytes < need) {
    ::hrf::set_error("kmeans_1d_pair: workspace of %lld bytes, %lld needed", (long long)work_bytes, (long long)need);
    return HRF_ENOMEM;
  }
  size_t tb = 0;
  if (hrf_status r = sort_tmp_bytes(n, &tb)) return r;
  const SortWs ws = carve(work, n, tb);
  hipStream_t s = (hipStream_t)stream;
  // both runs enqueued before the one synchronisation; the second reuses the sort.  A
  // fallback of either (rare) then reruns that k on the streaming path, after both.
  // pinned read-back slots (one pair per host thread, kept for the thread's lifetime), so the
  // first state copy does not block the host before the second run is enqueued
  static thread_local KmState *fin = nullptr;
  if (!fin) HRF_HIP(hipHostMalloc((void **)&fin, 2 * sizeof(KmState), hipHostMallocDefault));
  if (hrf_status r = km_launch_k(k1, x, valid, n, max_iter, top1, ws, 0, s, &fin[0])) return r;
  if (hrf_status r = km_launch_k(k2, x, valid, n, max_iter, top2, ws, 1, s, &fin[1])) return r;
  HRF_HIP(hipStreamSynchronize(s));
  const KmState f1 = fin[0], f2 = fin[1];
  if (hrf_status r = km_finish_k(k1, x, valid, n, max_iter, top1, ws, s, f1)) return r;
  return km_finish_k(k2, x, valid, n, max_iter, top2, ws, s, f2);
}

}  // extern "C"
