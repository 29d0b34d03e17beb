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
// Sorted path (hrf_kmeans_1d_sorted, the one the pipelines use): the valid values are radix
// sorted once (rocPRIM, on order-preserving uint64 encodings) and the fixed-point values
// prefix-summed in that order.  With ascending, well separated centres the label
// argmin_j (x - c_j)^2 (first minimum) is a non-decreasing step function of x, so one Lloyd
// iteration reduces to locating the k - 1 label steps in the sorted array (a 4096-ary search
// by one 1024-thread workgroup) and reading cluster sums and counts off the prefix array:
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


// ---- sorted path -------------------------------------------------------------------------
__global__ void km_encode_kernel(const double *__restrict__ x, const uint8_t *__restrict__ valid, int64_t n,
                                 unsigned long long *__restrict__ keys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = (!valid || valid[i]) ? ord_enc(x[i]) : ~0ull;  // invalid entries sort past every value
}

// q[i] = fixed-point value of the i-th smallest valid value (0 past the valid ones)
__global__ void km_fixed_kernel(const unsigned long long *__restrict__ keys, int64_t n, const KmState *st,
                                long long *__restrict__ q, long long *__restrict__ prefix0) {
  const int s = st->scale;
  const int64_t nv = (int64_t)st->nvalid;
  if (blockIdx.x == 0 && threadIdx.x == 0) *prefix0 = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    q[i] = i < nv ? (long long)rint(ldexp(ord_dec(keys[i]), s)) : 0;
}

constexpr int KS_T = 1024;           // threads of the iteration workgroup
constexpr int KS_P = 4;              // probes per thread per round -> 4096-ary search
static_assert(KS_T * KS_P == 4096, "index arithmetic below shifts by 12");

// First index in [lo, hi) of the sorted values whose label exceeds j (hi when none), for all
// boundaries j < K - 1 at once; pos[j] receives the answer.
template <int K>
__device__ void km_find_steps(const unsigned long long *__restrict__ keys, int64_t nv, const double *c,
                              int64_t *pos, int *cnt_sh) {
  const int t = threadIdx.x;
  __shared__ int64_t lo_sh[KMAX], hi_sh[KMAX];
  if (t < K - 1) {
    lo_sh[t] = 0;
    hi_sh[t] = nv;
  }
  __syncthreads();
  for (int j = 0; j < K - 1; ++j) {
    // every boundary is searched with the whole workgroup; its range shrinks 4096-fold per round
    while (true) {
      const int64_t lo = lo_sh[j], hi = hi_sh[j];
      const int64_t len = hi - lo;
      if (len <= 0) break;
      if (t == 0) *cnt_sh = 0;
      __syncthreads();
      const bool exact = len <= (int64_t)KS_T * KS_P;
      int nf = 0;  // probes of this thread whose label is <= j
#pragma unroll
      for (int p = 0; p < KS_P; ++p) {
        const int m = t * KS_P + p;
        int64_t idx;
        if (exact) {
          idx = lo + m;
          if (idx >= hi) continue;
        } else {
          idx = lo + ((len * m) >> 12);  // KS_T * KS_P = 4096; len < 2^51
        }
        nf += km_assign<K>(ord_dec(keys[idx]), c) <= j;
      }
      const int wsum = hrf::wave_sum(nf);
      if ((t & 63) == 0 && wsum) atomicAdd(cnt_sh, wsum);
      __syncthreads();
      const int F = *cnt_sh;
      __syncthreads();
      if (exact) {
        if (t == 0) {
          lo_sh[j] = lo + F;
          hi_sh[j] = lo + F;
        }
        __syncthreads();
        break;
      }
      // probes are a non-decreasing sample: the first F say "<= j", the rest "> j"
      if (t == 0) {
        const int64_t nlo = F == 0 ? lo : lo + ((len * (F - 1)) >> 12) + 1;
        const int64_t nhi = F == KS_T * KS_P ? hi : lo + ((len * F) >> 12);
        lo_sh[j] = nlo;
        hi_sh[j] = nhi;
      }
      __syncthreads();
    }
    // the next boundary lies at or after this one
    if (t == 0 && j + 1 < K - 1) lo_sh[j + 1] = lo_sh[j];
    __syncthreads();
  }
  if (t < K - 1) pos[t] = lo_sh[t];
  __syncthreads();
}

template <int K>
__global__ __launch_bounds__(KS_T) void km_sorted_iter_kernel(const unsigned long long *__restrict__ keys,
                                                              const long long *__restrict__ prefix, KmState *st,
                                                              int max_iter) {
  __shared__ double c[KMAX];
  __shared__ int64_t pos[KMAX];
  __shared__ int cnt_sh, stop;
  const int t = threadIdx.x;
  const int64_t nv = (int64_t)st->nvalid;
  const int s = st->scale;
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
    km_find_steps<K>(keys, nv, c, pos, &cnt_sh);
    if (t == 0) {
      int changed = 0;
      int64_t p0 = 0;
      for (int j = 0; j < K; ++j) {
        const int64_t p1 = j < K - 1 ? pos[j] : nv;
        const int64_t cn = p1 - p0;
        if (cn) {
          const long long sm = prefix[p1] - prefix[p0];
          const double cj = ldexp((double)sm / (double)cn, -s);
          if (cj != c[j]) changed = 1;
          c[j] = cj;
        }
        p0 = p1;
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
  unsigned long long *keys_in, *keys;
  long long *q, *prefix;
  void *tmp;
  size_t tmp_bytes;
};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

hrf_status sort_tmp_bytes(int64_t n, size_t *bytes) {
  size_t a = 0, b = 0;
  HRF_HIP(rocprim::radix_sort_keys(nullptr, a, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                   (size_t)std::max<int64_t>(n, 1), 0, 64, (hipStream_t)0));
  HRF_HIP(rocprim::inclusive_scan(nullptr, b, (long long *)nullptr, (long long *)nullptr,
                                  (size_t)std::max<int64_t>(n, 1), rocprim::plus<long long>(), (hipStream_t)0));
  *bytes = std::max(a, b);
  return HRF_OK;
}

SortWs carve(void *work, int64_t n, size_t tmp_bytes) {
  char *w = (char *)work;
  SortWs ws{};
  const size_t nb = align256(sizeof(unsigned long long) * (size_t)std::max<int64_t>(n, 1));
  ws.st = (KmState *)w;
  w += align256(sizeof(KmState));
  ws.keys_in = (unsigned long long *)w;
  w += nb;
  ws.keys = (unsigned long long *)w;
  w += nb;
  ws.q = (long long *)w;
  w += nb;
  ws.prefix = (long long *)w;
  w += align256(sizeof(long long) * (size_t)(std::max<int64_t>(n, 1) + 1));
  ws.tmp = w;
  ws.tmp_bytes = tmp_bytes;
  return ws;
}

template <int K>
hrf_status km_run_sorted(const double *x, const uint8_t *valid, int64_t n, int max_iter, int32_t *labels,
                         uint8_t *top, double *centers_host, int32_t *iters_host, const SortWs &ws, int reuse,
                         hipStream_t s) {
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
    km_encode_kernel<<<g, 256, 0, s>>>(x, valid, n, ws.keys_in);
    HRF_LAUNCHED();
    size_t tb = ws.tmp_bytes;
    HRF_HIP(rocprim::radix_sort_keys(ws.tmp, tb, ws.keys_in, ws.keys, (size_t)n, 0, 64, s));
    km_fixed_kernel<<<g, 256, 0, s>>>(ws.keys, n, st, ws.q, ws.prefix);
    HRF_LAUNCHED();
    tb = ws.tmp_bytes;
    HRF_HIP(rocprim::inclusive_scan(ws.tmp, tb, ws.q, ws.prefix + 1, (size_t)n, rocprim::plus<long long>(), s));
  }
  km_sorted_iter_kernel<K><<<1, KS_T, 0, s>>>(ws.keys, ws.prefix, st, max_iter);
  HRF_LAUNCHED();
  if (n > 0) km_label_kernel<K><<<g, 256, 0, s>>>(x, valid, n, st, labels, top);
  HRF_LAUNCHED();
  KmState fin;
  HRF_HIP(hipMemcpyAsync(&fin, st, sizeof(KmState), hipMemcpyDeviceToHost, s));
  HRF_HIP(hipStreamSynchronize(s));
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
  const size_t nb = align256(sizeof(unsigned long long) * (size_t)std::max<int64_t>(n, 1));
  return (int64_t)(align256(sizeof(KmState)) + 3 * nb + align256(sizeof(long long) * (size_t)(std::max<int64_t>(n, 1) + 1)) +
                   align256(tb));
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

}  // extern "C"
