// kmeans.hip -- 1-D KMeans thresholding (a8): sklearn's KMeans, k-means++ and all.
//
// Reference: sklearn KMeans(n_clusters=k, random_state=0).fit_predict(x.reshape(-1,1))
// (ecoli measurement.py:73, :85; multispecies :125, :141), n_init=10.  Restated from
// sklearn 1.7.2 -- the sklearn importable here -- (KMeans.fit, _kmeans_plusplus,
// _kmeans_single_lloyd, _relocate_empty_clusters_dense); the CPU restatement is
// oracle/kmeans_sk.c, pinned to sklearn itself in tests/test_oracle_golden.py:
//  * the random stream is numpy's RandomState(0) (MT19937, init_genrand) replayed on the host:
//    per run the first centre (choice(n, p=1/n)) and 2 + int(log k) uniform draws per further
//    centre;
//  * k-means++ picks each further centre as the first sample whose running sum of
//    closest-squared-distances reaches u * total; of a centre's trials the one leaving the
//    least total wins;
//  * Lloyd iterations stop on repeated labels (strict convergence) or a summed squared centre
//    shift <= 1e-4 * var(x); empty clusters take the samples farthest from their centres;
//    without strict convergence the labels are recomputed from the final centres;
//  * of the n_init runs the one with the least inertia wins (strictly less, different
//    partition in sklearn's one-sided sense).
// Where sklearn's outcome hangs on its own floating-point summation order the restatement sums
// exactly instead: squared distances as floor(d^2 * 2^S) in 128-bit integers, values as
// rint(x * 2^s) in int64 (prefix sums over the value-sorted array, plus 128-bit prefix sums of
// their squares), so every decision is independent of reduction order and equal to the CPU
// restatement's bit for bit.
// Parity is pinned to sklearn 1.7.2 only.  The reference ran with the sklearn of its era
// (0.20-0.22: first centre from randint, per-run int32 seeds, Elkan by default), whose random
// streams differ; no fixture in the reference pins that, so parity with the reference-era
// sklearn is unpinned (an ambiguous 1-D split could land differently).
//
// MI355X mapping.  The valid values are bucket sorted once (2^20 value buckets, a two-digit
// counting sort without global atomics) and per-bucket prefix sums of q and q^2 are taken; a
// Lloyd step is then k - 1 label-step searches on the sorted array (one 1024-thread workgroup
// narrows to whole buckets and counts the straddling ones) -- no pass over the data per
// iteration.  The n_init runs proceed in parallel: a k-means++ round is one raster pass for the
// block potentials of all runs, a parallel candidate pick per (run, trial), and one pass over the
// sorted array for every trial's potential (a trial only changes the samples of its candidate's
// value cell, a contiguous range of buckets); the Lloyd loops run one workgroup per run; a last
// kernel picks the winner and a raster pass writes labels / the top-cluster mask.  No host
// synchronisation is needed between the stages (the draws travel as kernel arguments).
#include <algorithm>
#include <cmath>
#include <mutex>
#include <unordered_map>
#include <vector>


#include "common.hpp"
#include "wave.hpp"

namespace {

typedef unsigned __int128 u128;

constexpr int KMAX = 8;
constexpr int NRUN = 10;                 // n_init (the reference era's default)
constexpr int NTMAX = 4;                 // 2 + int(log 8)
constexpr int PB = 4096;                 // samples per potential block
constexpr int PT = 256;                  // threads per potential block (16 samples each)

struct U128 {
  unsigned long long lo, hi;
};
struct U128Plus {
  __host__ __device__ U128 operator()(const U128 &a, const U128 &b) const {
    U128 r;
    r.lo = a.lo + b.lo;
    r.hi = a.hi + b.hi + (r.lo < a.lo ? 1ull : 0ull);
    return r;
  }
};
__host__ __device__ inline u128 U(const U128 &a) { return ((u128)a.hi << 64) | a.lo; }
__host__ __device__ inline U128 P(u128 v) { return U128{(unsigned long long)v, (unsigned long long)(v >> 64)}; }

// correctly rounded (nearest even) u128 -> double, identical on host and device
__host__ __device__ inline double u128_to_double(u128 v) {
  const unsigned long long hi = (unsigned long long)(v >> 64);
  if (!hi) return (double)(unsigned long long)v;
  int z = 0;
  while (!((hi << z) & 0x8000000000000000ull)) ++z;
  const u128 t = v << z;                              // top bit at 127
  const unsigned long long m64 = (unsigned long long)(t >> 64);
  const bool sticky = (unsigned long long)t != 0;
  unsigned long long mant = m64 >> 11;                // 53 bits
  const unsigned long long rem = m64 & 0x7ffull;
  if (rem > 0x400ull || (rem == 0x400ull && (sticky || (mant & 1ull)))) ++mant;
  return ldexp((double)mant, 64 - z + 11);
}

// ceil(m * T / 2^53) for m < 2^53, T < 2^100 (exact)
__host__ __device__ inline u128 thr_of(unsigned long long m, u128 T) {
  const unsigned long long tl = (unsigned long long)T, th = (unsigned long long)(T >> 64);
  const u128 a = (u128)m * tl;
  const u128 b = (u128)m * th;
  const u128 lo = a & ((((u128)1) << 53) - 1);
  return (a >> 53) + (b << 11) + (lo != 0 ? 1 : 0);
}

__host__ __device__ inline unsigned long long qd(double x, double c, double scaleS) {
  const double d = x - c;
  return (unsigned long long)(d * d * scaleS);
}

// ---- host: numpy RandomState replay --------------------------------------------------------
struct Mt19937 {
  uint32_t mt[624];
  int i = 624;
  explicit Mt19937(uint32_t seed) {
    mt[0] = seed;
    for (int k = 1; k < 624; ++k) mt[k] = 1812433253u * (mt[k - 1] ^ (mt[k - 1] >> 30)) + (uint32_t)k;
  }
  uint32_t u32() {
    if (i >= 624) {
      for (int k = 0; k < 624; ++k) {
        const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
        mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      i = 0;
    }
    uint32_t y = mt[i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double random_sample() {  // numpy: (a >> 5, b >> 6) -> 53-bit double in [0, 1)
    const uint32_t a = u32() >> 5, b = u32() >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
  }
};

// numpy RandomState.choice(nv, p = ones(nv) / nv): cdf = cumsum(p) / cdf[-1] (sequential),
// index = searchsorted(cdf, u, side='right').  The cdf depends on nv only: cached.
int64_t choice_uniform(int64_t nv, double u) {
  static std::mutex mu;
  static std::unordered_map<int64_t, std::vector<double>> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(nv);
  if (it == cache.end()) {
    if (cache.size() > 8) cache.clear();
    std::vector<double> cdf((size_t)nv);
    const double p = 1.0 / (double)nv;
    double s = 0.0;
    for (int64_t i = 0; i < nv; ++i) {
      s += p;
      cdf[(size_t)i] = s;
    }
    const double last = cdf[(size_t)nv - 1];
    for (auto &v : cdf) v /= last;
    it = cache.emplace(nv, std::move(cdf)).first;
  }
  const std::vector<double> &cdf = it->second;
  return (int64_t)(std::upper_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
}

struct Draws {  // kernel argument
  long long first[NRUN];                 // rank of each run's first centre among the valid samples
  unsigned long long m[NRUN][KMAX - 1][NTMAX];  // trial draws as integers (u = m / 2^53)
  int nt, nrun;
};

Draws make_draws(int64_t nv, int k, int n_init, uint32_t seed) {
  Draws d{};
  Mt19937 rs(seed);
  d.nt = 2 + (int)std::log((double)k);
  d.nrun = n_init;
  for (int r = 0; r < n_init; ++r) {
    d.first[r] = (long long)choice_uniform(nv, rs.random_sample());
    for (int c = 1; c < k; ++c)
      for (int t = 0; t < d.nt; ++t) d.m[r][c - 1][t] = (unsigned long long)ldexp(rs.random_sample(), 53);
  }
  return d;
}

// ---- device state ----------------------------------------------------------------------------
struct SkRun {
  double cen[KMAX];    // final centres, sklearn order
  double lcen[KMAX];   // centres that produced the final labels
  double cand[NTMAX];  // candidates of the current k-means++ round
  U128 T;              // current potential
  double inertia;
  long long cut[KMAX]; // final labels: samples with sorted rank <= p (value order)
  int ids[KMAX];       // sorted rank -> sklearn id (final labels)
  int iters, strict, reloc, ncen;
};

struct KmState {
  unsigned long long lo_bits, hi_bits, amax_bits, nvalid, nnan;
  int s;          // value fixed point: q = rint(x * 2^s)
  int S;          // potential fixed point: floor(d^2 * 2^S)
  double tol;
  int error;      // 1: NaN input (sklearn raises)
  int best;       // winning run
  int top;        // sklearn id of the top cluster (by the rule)
  long long nle0; // samples <= 0 (rule 1)
  long long sumq; // sums of q and q^2 over the valid samples
  U128 sumq2;
  double center[KMAX];
  int iters;
  SkRun run[NRUN];
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
      if (v != v) {
        nn += 1;
        nv += 1;
        continue;
      }
      const unsigned long long en = ord_enc(v);
      lo = en < lo ? en : lo;
      hi = en > hi ? en : hi;
      const unsigned long long a = (unsigned long long)__double_as_longlong(fabs(v));
      am = a > am ? a : am;
      nv += 1;
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

// value and potential scales (oracle_kmeans_scale / kmeans_sk.c)
__device__ __forceinline__ void km_scale(KmState *st) {
  const double amax = __longlong_as_double((long long)st->amax_bits);
  int e = 0;
  frexp(amax > 0 ? amax : 1.0, &e);
  const unsigned long long nv = st->nvalid;
  int ln = 0;
  while ((1ull << ln) < (nv > 1 ? nv : 1ull)) ++ln;
  st->s = 61 - ln - e;
  const double mn = ord_dec(st->lo_bits), mx = ord_dec(st->hi_bits);
  const double r = nv && !st->nnan ? mx - mn : 0.0, R2 = r * r;
  int e2 = 0;
  frexp(R2 > 0 ? R2 : 1.0, &e2);
  st->S = 61 - e2;
  st->error = st->nnan ? 1 : 0;
}

// ---- exact 128-bit reductions -------------------------------------------------------------
__device__ __forceinline__ U128 wave_sum128(U128 a) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    U128 b;
    b.lo = __shfl_xor(a.lo, o, 64);
    b.hi = __shfl_xor(a.hi, o, 64);
    a = U128Plus()(a, b);
  }
  return a;
}

// block sum of per-thread u128 values (PT threads); result valid in thread 0
__device__ __forceinline__ U128 block_sum128(U128 a, U128 *sh) {
  a = wave_sum128(a);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = a;
  __syncthreads();
  U128 r{0, 0};
  if (threadIdx.x == 0)
    for (int q = 0; q < PT / 64; ++q) r = U128Plus()(r, sh[q]);
  return r;
}

// block exclusive scan of per-thread u128 values (PT threads); *total = the block sum (all threads)
__device__ __forceinline__ u128 block_excl_scan128(u128 v, U128 *sh, u128 *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  u128 inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long lo = __shfl_up((unsigned long long)inc, o, 64);
    const unsigned long long hi = __shfl_up((unsigned long long)(inc >> 64), o, 64);
    if (lane >= o) inc += ((u128)hi << 64) | lo;
  }
  __syncthreads();
  if (lane == 63) sh[w] = P(inc);
  __syncthreads();
  u128 off = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < PT / 64; ++q) {
    const u128 x = U(sh[q]);
    off += q < w ? x : (u128)0;
    tot += x;
  }
  *total = tot;
  return off + inc - v;
}


// ---- bucket-sorted array ----------------------------------------------------------------------
// NB value buckets of equal width over [min, max]; bucket(x) is a non-decreasing function of
// x, so every value of bucket b is below every value of bucket b' > b.  The valid values are
// counting sorted by bucket (xs, in no particular order inside a bucket -- only integer sums and
// counts are read off): off[b] = first position of bucket b (off[NB] = nvalid).  For every
// non-empty bucket b, bq[b] / bq2[b] = the sums of q = rint(x 2^s) and of q^2 over the samples
// before it; the totals are in the state.
//
// The sort is a two-digit MSD counting sort without global atomics: the coarse digit (bucket >>
// 10) per 4096-sample chunk of the raster input (LDS histogram, per-chunk counts written
// digit-major, one scan -> every chunk's run of every digit), scattered into tmp; then the fine
// digit per 4096-sample chunk of each coarse segment the same way into xs.  Ranks inside a chunk
// come from LDS atomics (no order is needed inside a bucket).
constexpr int KM_NB = 1 << 20;
constexpr int KD = 1024;                  // digit values (2 x 10 bits)
constexpr int KS_CH = 4096;               // samples per sort chunk (256 threads x 16)

__device__ __forceinline__ int km_bucket(double x, double mn, double inv) {
  const double t = (x - mn) * inv;
  return t >= 0.0 ? (t < (double)(KM_NB - 1) ? (int)t : KM_NB - 1) : 0;  // NaN -> 0
}

__device__ __forceinline__ long long km_q(double x, int s) { return (long long)rint(ldexp(x, s)); }
__device__ __forceinline__ u128 km_q2(long long v) {
  const unsigned long long a = (unsigned long long)(v < 0 ? -v : v);
  return (u128)a * a;
}

__device__ __forceinline__ void km_bucket_init(KmState *st, double *geo) {
  const double mn = ord_dec(st->lo_bits), mx = ord_dec(st->hi_bits);
  geo[0] = mn;
  geo[1] = mx > mn ? (double)KM_NB / (mx - mn) : 0.0;
}

// the scales and (n > 0) the bucket geometry, one launch
__global__ void km_scale_kernel(KmState *st, double *geo) {
  km_scale(st);
  if (geo) km_bucket_init(st, geo);
}

__device__ __forceinline__ unsigned long long block_excl_scan_u64(unsigned long long v, unsigned long long *sh,
                                                                  unsigned long long *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned long long inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  unsigned long long off = 0, tot = 0;
  for (int q = 0; q < nw; ++q) {
    off += q < w ? sh[q] : 0ull;
    tot += sh[q];
  }
  *total = tot;
  return off + inc - v;
}

// ---- exclusive scan of u32 counts (3 kernels: block sums, their scan, apply; in place) ----
constexpr int KSC_B = 4096;  // entries per scan block (256 threads x 16)

__global__ __launch_bounds__(256) void km_scan_sum_kernel(const unsigned *__restrict__ a, long long n,
                                                          unsigned *__restrict__ bsum) {
  const long long i0 = (long long)blockIdx.x * KSC_B;
  unsigned long long s = 0;
  for (int e = threadIdx.x; e < KSC_B; e += 256)
    if (i0 + e < n) s += a[i0 + e];
  s = hrf::wave_sum(s);
  __shared__ unsigned long long sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = (unsigned)(sh[0] + sh[1] + sh[2] + sh[3]);
}

__global__ __launch_bounds__(256) void km_scan_blocks_kernel(unsigned *__restrict__ bsum, int nb) {
  __shared__ unsigned long long sh[4];
  unsigned long long carry = 0;
  for (int b0 = 0; b0 < nb; b0 += 256) {
    const int i = b0 + threadIdx.x;
    unsigned long long tot;
    const unsigned long long e = block_excl_scan_u64(i < nb ? bsum[i] : 0u, sh, &tot);
    if (i < nb) bsum[i] = (unsigned)(carry + e);
    carry += tot;
  }
}

__global__ __launch_bounds__(256) void km_scan_apply_kernel(unsigned *__restrict__ a, long long n,
                                                            const unsigned *__restrict__ bsum) {
  __shared__ unsigned long long sh[4];
  const long long i0 = (long long)blockIdx.x * KSC_B + threadIdx.x * 16;
  unsigned v[16];
  unsigned long long loc = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    v[e] = i0 + e < n ? a[i0 + e] : 0u;
    loc += v[e];
  }
  unsigned long long tot;
  unsigned long long acc = bsum[blockIdx.x] + block_excl_scan_u64(loc, sh, &tot);
#pragma unroll
  for (int e = 0; e < 16; ++e)
    if (i0 + e < n) {
      a[i0 + e] = (unsigned)acc;
      acc += v[e];
    }
}

// ---- order-preserving compaction of the valid samples (sklearn's sample order) ----
// km_sel_count_kernel: valid samples per KSC_B block; km_scan_blocks_kernel turns the counts into
// block offsets in place; km_sel_scatter_kernel writes each block's valid values in raster order
// (16 consecutive samples per thread, a block scan of the per-thread counts) and the total.
__global__ __launch_bounds__(256) void km_sel_count_kernel(const uint8_t *__restrict__ valid, long long n,
                                                           unsigned *__restrict__ cnt) {
  const long long i0 = (long long)blockIdx.x * KSC_B;
  unsigned long long s = 0;
  for (int e = threadIdx.x; e < KSC_B; e += 256)
    if (i0 + e < n) s += valid[i0 + e] != 0;
  s = hrf::wave_sum(s);
  __shared__ unsigned long long sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = (unsigned)(sh[0] + sh[1] + sh[2] + sh[3]);
}

__global__ __launch_bounds__(256) void km_sel_scatter_kernel(const double *__restrict__ x,
                                                             const uint8_t *__restrict__ valid, long long n,
                                                             const unsigned *__restrict__ boff,
                                                             double *__restrict__ out,
                                                             unsigned long long *__restrict__ nsel) {
  __shared__ unsigned long long sh[4];
  const long long i0 = (long long)blockIdx.x * KSC_B + threadIdx.x * 16;
  unsigned m = 0;
  unsigned long long loc = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const bool v = i0 + e < n && valid[i0 + e] != 0;
    m |= (unsigned)v << e;
    loc += v;
  }
  unsigned long long tot;
  unsigned long long o = boff[blockIdx.x] + block_excl_scan_u64(loc, sh, &tot);
#pragma unroll
  for (int e = 0; e < 16; ++e)
    if ((m >> e) & 1u) out[o++] = x[i0 + e];
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *nsel = boff[blockIdx.x] + tot;
}

// ---- pass A: coarse digit over raster chunks ----
// cntA[d * nchA + c] = samples of chunk c with coarse digit d
// st != nullptr: the scales and the bucket geometry (km_scale_kernel's work) are taken here --
// every block derives the geometry from the min / max itself, block 0 stores both for the
// later kernels (one launch less per fit)
__global__ __launch_bounds__(256) void km_hist_a_kernel(const double *__restrict__ x, const uint8_t *__restrict__ valid,
                                                        int64_t n, double *__restrict__ geo,
                                                        unsigned *__restrict__ cntA, int nchA, KmState *st) {
  __shared__ unsigned h[KD];
  for (int i = threadIdx.x; i < KD; i += 256) h[i] = 0;
  double mn, inv;
  if (st) {
    mn = ord_dec(st->lo_bits);
    const double mx = ord_dec(st->hi_bits);
    inv = mx > mn ? (double)KM_NB / (mx - mn) : 0.0;  // km_bucket_init's expression
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      km_scale(st);
      geo[0] = mn;
      geo[1] = inv;
    }
  } else {
    mn = geo[0];
    inv = geo[1];
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * KS_CH + threadIdx.x;
#pragma unroll 4
  for (int e = 0; e < KS_CH / 256; ++e) {
    const int64_t i = base + (int64_t)e * 256;
    if (i < n && (!valid || valid[i])) atomicAdd(&h[km_bucket(x[i], mn, inv) >> 10], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < KD; i += 256) cntA[(int64_t)i * nchA + blockIdx.x] = h[i];
}

__global__ __launch_bounds__(256) void km_scatter_a_kernel(const double *__restrict__ x,
                                                           const uint8_t *__restrict__ valid, int64_t n,
                                                           const double *__restrict__ geo,
                                                           const unsigned *__restrict__ offA, int nchA,
                                                           double *__restrict__ tmp) {
  __shared__ unsigned h[KD];
  for (int i = threadIdx.x; i < KD; i += 256) h[i] = offA[(int64_t)i * nchA + blockIdx.x];
  __syncthreads();
  const double mn = geo[0], inv = geo[1];
  const int64_t base = (int64_t)blockIdx.x * KS_CH + threadIdx.x;
#pragma unroll 4
  for (int e = 0; e < KS_CH / 256; ++e) {
    const int64_t i = base + (int64_t)e * 256;
    if (i < n && (!valid || valid[i])) {
      const double v = x[i];
      tmp[atomicAdd(&h[km_bucket(v, mn, inv) >> 10], 1u)] = v;
    }
  }
}

// coarse segments: seg[d] = first position of digit d (seg[KD] = nvalid); their 4096-sample
// chunks cB[d] (exclusive prefix, cB[KD] = number of chunks)
__global__ __launch_bounds__(KD) void km_segments_kernel(const unsigned *__restrict__ offA, int nchA,
                                                         const KmState *st, unsigned *__restrict__ seg,
                                                         unsigned *__restrict__ cB) {
  __shared__ unsigned long long sh[16];
  const int d = threadIdx.x;
  const unsigned nv = (unsigned)st->nvalid;
  const unsigned s0 = offA[(int64_t)d * nchA];
  const unsigned s1 = d + 1 < KD ? offA[(int64_t)(d + 1) * nchA] : nv;
  seg[d] = s0;
  if (d == 0) seg[KD] = nv;
  unsigned long long tot;
  const unsigned long long e = block_excl_scan_u64((s1 - s0 + KS_CH - 1) / KS_CH, sh, &tot);
  cB[d] = (unsigned)e;
  if (d == 0) cB[KD] = (unsigned)tot;
}

__device__ __forceinline__ int km_seg_of(const unsigned *cB, int j) {  // cB[d] <= j < cB[d + 1]
  int lo = 0, hi = KD;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cB[mid] <= (unsigned)j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// ---- pass B: fine digit over the chunks of every coarse segment ----
// cntB[f * L + j] = samples of chunk j with fine digit f (L = chunk bound + 1, the spare columns
// zero)
__global__ __launch_bounds__(256) void km_hist_b_kernel(const double *__restrict__ tmp, const double *__restrict__ geo,
                                                        const unsigned *__restrict__ seg,
                                                        const unsigned *__restrict__ cB, unsigned *__restrict__ cntB,
                                                        int L) {
  __shared__ unsigned h[KD];
  for (int i = threadIdx.x; i < KD; i += 256) h[i] = 0;
  __syncthreads();
  const int j = blockIdx.x;
  if (j < (int)cB[KD]) {
    const int d = km_seg_of(cB, j);
    const long long a = (long long)seg[d] + (long long)(j - (int)cB[d]) * KS_CH;
    const long long b = a + KS_CH < (long long)seg[d + 1] ? a + KS_CH : (long long)seg[d + 1];
    const double mn = geo[0], inv = geo[1];
#pragma unroll 4
    for (int e = 0; e < KS_CH / 256; ++e) {
      const long long i = a + (long long)e * 256 + threadIdx.x;
      if (i < b) atomicAdd(&h[km_bucket(tmp[i], mn, inv) & (KD - 1)], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < KD; i += 256) {
    cntB[(int64_t)i * L + j] = h[i];
    if (j == L - 2) cntB[(int64_t)i * L + L - 1] = 0;
  }
}

// bucket starts: off[d * KD + f] = seg[d] + samples of segment d with fine digit < f
__global__ __launch_bounds__(KD) void km_bucket_off_kernel(const unsigned *__restrict__ S, int L,
                                                           const unsigned *__restrict__ seg,
                                                           const unsigned *__restrict__ cB,
                                                           unsigned long long *__restrict__ off) {
  __shared__ unsigned long long sh[16];
  const int d = blockIdx.x, f = threadIdx.x;
  const int j0 = (int)cB[d], j1 = (int)cB[d + 1];
  const unsigned tot = S[(int64_t)f * L + j1] - S[(int64_t)f * L + j0];
  unsigned long long t;
  const unsigned long long e = block_excl_scan_u64(tot, sh, &t);
  off[(int64_t)d * KD + f] = seg[d] + e;
  if (d == KD - 1 && f == 0) off[KM_NB] = seg[KD];
}

__global__ __launch_bounds__(256) void km_scatter_b_kernel(const double *__restrict__ tmp,
                                                           const double *__restrict__ geo,
                                                           const unsigned *__restrict__ seg,
                                                           const unsigned *__restrict__ cB,
                                                           const unsigned *__restrict__ S, int L,
                                                           const unsigned long long *__restrict__ off,
                                                           double *__restrict__ xs) {
  __shared__ unsigned h[KD];
  const int j = blockIdx.x;
  if (j >= (int)cB[KD]) return;
  const int d = km_seg_of(cB, j), j0 = (int)cB[d];
  for (int f = threadIdx.x; f < KD; f += 256)
    h[f] = (unsigned)(off[(int64_t)d * KD + f] - seg[d]) + S[(int64_t)f * L + j] - S[(int64_t)f * L + j0];
  __syncthreads();
  const long long a = (long long)seg[d] + (long long)(j - j0) * KS_CH;
  const long long b = a + KS_CH < (long long)seg[d + 1] ? a + KS_CH : (long long)seg[d + 1];
  const double mn = geo[0], inv = geo[1];
#pragma unroll 4
  for (int e = 0; e < KS_CH / 256; ++e) {
    const long long i = a + (long long)e * 256 + threadIdx.x;
    if (i < b) {
      const double v = tmp[i];
      xs[(long long)seg[d] + atomicAdd(&h[km_bucket(v, mn, inv) & (KD - 1)], 1u)] = v;
    }
  }
}

// bucket prefix sums: per 4096-sample chunk of xs the sums of q and q^2, their scan, then per
// non-empty bucket the sums before its first sample
__global__ __launch_bounds__(PT) void km_chunk_sum_kernel(const double *__restrict__ xs, const KmState *st,
                                                          long long *__restrict__ cq, U128 *__restrict__ cq2) {
  __shared__ U128 sh[PT / 64];
  __shared__ long long sa[PT / 64];
  const int64_t nv = (int64_t)st->nvalid;
  const int s = st->s;
  const int64_t i0 = (int64_t)blockIdx.x * PB + threadIdx.x;
  long long a = 0;
  u128 b = 0;
#pragma unroll
  for (int e = 0; e < PB / PT; ++e) {
    const int64_t i = i0 + (int64_t)e * PT;
    if (i < nv) {
      const long long q = km_q(xs[i], s);
      a += q;
      b += km_q2(q);
    }
  }
  a = hrf::wave_sum(a);
  if ((threadIdx.x & 63) == 0) sa[threadIdx.x >> 6] = a;
  const U128 tb = block_sum128(P(b), sh);
  if (threadIdx.x == 0) {
    cq[blockIdx.x] = sa[0] + sa[1] + sa[2] + sa[3];
    cq2[blockIdx.x] = tb;
  }
}

__global__ __launch_bounds__(PT) void km_chunk_scan_kernel(long long *__restrict__ cq, U128 *__restrict__ cq2,
                                                           int nch, KmState *st) {
  __shared__ U128 sh[PT / 64];
  __shared__ unsigned long long shq[PT / 64];
  unsigned long long carry = 0;
  u128 carry2 = 0;
  for (int b0 = 0; b0 < nch; b0 += PT) {
    const int i = b0 + threadIdx.x;
    const unsigned long long a = i < nch ? (unsigned long long)cq[i] : 0ull;
    const u128 b = i < nch ? U(cq2[i]) : (u128)0;
    unsigned long long ta;
    u128 tb;
    const unsigned long long ea = block_excl_scan_u64(a, shq, &ta);  // two's complement: exact
    const u128 eb = block_excl_scan128(b, sh, &tb);
    if (i < nch) {
      cq[i] = (long long)(carry + ea);
      cq2[i] = P(carry2 + eb);
    }
    carry += ta;
    carry2 += tb;
  }
  if (threadIdx.x == 0) {
    st->sumq = (long long)carry;
    st->sumq2 = P(carry2);
  }
}

__global__ __launch_bounds__(PT) void km_bucket_prefix_kernel(const double *__restrict__ xs, const KmState *st,
                                                              const double *__restrict__ geo,
                                                              const long long *__restrict__ cq,
                                                              const U128 *__restrict__ cq2, long long *__restrict__ bq,
                                                              U128 *__restrict__ bq2) {
  __shared__ U128 sh[PT / 64];
  __shared__ unsigned long long shq[PT / 64];
  const int64_t nv = (int64_t)st->nvalid;
  const int s = st->s;
  const double mn = geo[0], inv = geo[1];
  const int64_t i0 = (int64_t)blockIdx.x * PB + threadIdx.x * (PB / PT);  // 16 consecutive samples
  double v[PB / PT];
  long long q[PB / PT];
  unsigned long long a = 0;
  u128 b = 0;
#pragma unroll
  for (int e = 0; e < PB / PT; ++e) {
    const int64_t i = i0 + e;
    v[e] = i < nv ? xs[i] : 0.0;
    q[e] = i < nv ? km_q(v[e], s) : 0;
    a += (unsigned long long)q[e];
    b += km_q2(q[e]);
  }
  unsigned long long ta;
  u128 tb;
  unsigned long long ra = block_excl_scan_u64(a, shq, &ta) + (unsigned long long)cq[blockIdx.x];
  u128 rb = block_excl_scan128(b, sh, &tb) + U(cq2[blockIdx.x]);
  if (i0 >= nv) return;
  int prev = i0 > 0 ? km_bucket(xs[i0 - 1], mn, inv) : -1;
#pragma unroll
  for (int e = 0; e < PB / PT; ++e) {
    if (i0 + e >= nv) break;
    const int kb = km_bucket(v[e], mn, inv);
    if (kb != prev) {
      bq[kb] = (long long)ra;
      bq2[kb] = P(rb);
    }
    prev = kb;
    ra += (unsigned long long)q[e];
    rb += km_q2(q[e]);
  }
}

// tol = 1e-4 * var(x) from the exact sums (kmeans_sk.c)
__device__ __forceinline__ void km_tol(KmState *st) {
  const long long nv = (long long)st->nvalid;
  if (!nv) {
    st->tol = 0;
    return;
  }
  const double m1 = (double)st->sumq / (double)nv, m2 = u128_to_double(U(st->sumq2)) / (double)nv;
  st->tol = ldexp(m2 - m1 * m1, -2 * st->s) * 1e-4;
}

// ---- k-means++ -------------------------------------------------------------------------------
// closest squared distance of v to the run's first c centres.  floor(. * 2^S) is monotone, so the
// least fixed-point potential is the fixed point of the least square: one conversion per sample.
__device__ __forceinline__ double closest_sq(double v, const double *cen, int c) {
  double b = (v - cen[0]) * (v - cen[0]);
  for (int j = 1; j < c; ++j) {
    const double d = (v - cen[j]) * (v - cen[j]);
    b = d < b ? d : b;
  }
  return b;
}
__device__ __forceinline__ unsigned long long closest_q(double v, const double *cen, int c, double scaleS) {
  return (unsigned long long)(closest_sq(v, cen, c) * scaleS);
}

// the first centre of every run: first[r]-th valid sample in raster order (xr compacted)
__global__ void km_pp_first_kernel(const double *__restrict__ xr, KmState *st, Draws d) {
  const int r = threadIdx.x;
  if (r >= d.nrun) return;
  SkRun &R = st->run[r];
  const long long nv = (long long)st->nvalid;
  long long idx = d.first[r] < nv ? d.first[r] : nv - 1;
  R.cen[0] = nv > 0 ? xr[idx] : 0.0;
  R.ncen = 1;
}

// Every round (one further centre for all runs):
//  pass  -- per run, block sums of the closest potential over the raster-ordered samples;
//  pick  -- per run and trial, the total T and the candidate: the first raster sample whose
//           running potential reaches thr = ceil(m T / 2^53); also the range of the value-sorted
//           array that holds every sample the candidate is closer to than the run's centres;
//  corr  -- per run and trial, the potential the candidate removes: sum over that range of
//           closest - min(closest, candidate) (zero outside its cell);
//  choose-- per run, the trial of least T - corr (the first on ties).
// The candidate's cell is an interval of values (1-D): the range is bounded by whole buckets
// around the midpoints to the neighbouring centres, widened by a margin far above the rounding
// of the squares.  Work per round: one raster pass, one sweep of the cells.
// c == 1: the runs' first centres (km_pp_first_kernel's work) are taken here -- every block
// reads them from the draws, block 0 stores them for the later kernels
__global__ __launch_bounds__(PT) void km_pp_pass_kernel(const double *__restrict__ xr, KmState *st, Draws d,
                                                        U128 *__restrict__ part, int nblk, int c) {
  __shared__ U128 sh[PT / 64];
  __shared__ double cen[NRUN][KMAX];
  if (threadIdx.x < NRUN * KMAX && !(c == 1 && threadIdx.x % KMAX == 0))
    cen[threadIdx.x / KMAX][threadIdx.x % KMAX] = st->run[threadIdx.x / KMAX].cen[threadIdx.x % KMAX];
  const int64_t nv = (int64_t)st->nvalid;
  if (c == 1 && (int)threadIdx.x < d.nrun) {
    const int r = threadIdx.x;
    const long long idx = d.first[r] < nv ? d.first[r] : nv - 1;
    const double c0 = nv > 0 ? xr[idx] : 0.0;
    cen[r][0] = c0;
    if (blockIdx.x == 0) {
      st->run[r].cen[0] = c0;
      st->run[r].ncen = 1;
    }
  }
  const double scaleS = ldexp(1.0, st->S);
  const int64_t base = (int64_t)blockIdx.x * PB + threadIdx.x;
  double v[PB / PT];
  int cnt = 0;
#pragma unroll
  for (int e = 0; e < PB / PT; ++e) {
    const int64_t i = base + e * PT;
    v[e] = i < nv ? xr[i] : 0.0;
    cnt += i < nv;
  }
  __syncthreads();
  for (int r = 0; r < d.nrun; ++r) {
    u128 s = 0;
#pragma unroll
    for (int e = 0; e < PB / PT; ++e) s += e < cnt ? closest_q(v[e], cen[r], c, scaleS) : 0ull;
    const U128 tot = block_sum128(P(s), sh);
    if (threadIdx.x == 0) part[(int64_t)r * nblk + blockIdx.x] = tot;
  }
}

__global__ __launch_bounds__(PT) void km_pp_pick_kernel(const double *__restrict__ xr,
                                                        const unsigned long long *__restrict__ off,
                                                        const double *__restrict__ geo, KmState *st, Draws d,
                                                        const U128 *__restrict__ part, int nblk, int c,
                                                        long long *__restrict__ rng) {
  __shared__ U128 sh[PT / 64];
  __shared__ int first_sh;
  __shared__ long long idx_sh;
  __shared__ int blk_sh;
  __shared__ U128 acc_sh;
  const int r = blockIdx.x / d.nt, t = blockIdx.x % d.nt;
  SkRun &R = st->run[r];
  const int64_t nv = (int64_t)st->nvalid;
  const double scaleS = ldexp(1.0, st->S);
  const int tid = threadIdx.x;
  const U128 *pr = part + (int64_t)r * nblk;
  const int per = (nblk + PT - 1) / PT;
  const int b0 = tid * per, b1 = b0 + per < nblk ? b0 + per : nblk;
  u128 loc = 0;
  for (int b = b0; b < b1; ++b) loc += U(pr[b]);
  u128 T;
  const u128 before = block_excl_scan128(loc, sh, &T);
  const u128 thr = thr_of(d.m[r][c - 1][t], T);
  if (tid == 0) {
    first_sh = PT;
    idx_sh = -1;
    blk_sh = -1;
  }
  __syncthreads();
  // the block whose inclusive running sum first reaches thr: in the range of the first thread
  // whose inclusive sum does
  if (b0 < b1 && before + loc >= thr) atomicMin(&first_sh, tid);
  __syncthreads();
  if (tid == first_sh) {
    u128 acc = before;
    for (int b = b0; b < b1; ++b) {
      const u128 nx = acc + U(pr[b]);
      if (nx >= thr) {
        blk_sh = b;
        break;
      }
      acc = nx;
    }
    acc_sh = P(acc);
  }
  __syncthreads();
  const int b = blk_sh;
  if (b >= 0) {
    const int64_t i0 = (int64_t)b * PB + tid * (PB / PT);
    unsigned long long cl[PB / PT];
    u128 sthr = 0;
#pragma unroll
    for (int e = 0; e < PB / PT; ++e) {
      const int64_t i = i0 + e;
      cl[e] = i < nv ? closest_q(xr[i], R.cen, c, scaleS) : 0ull;
      sthr += cl[e];
    }
    u128 tb;
    const u128 bt = block_excl_scan128(sthr, sh, &tb) + U(acc_sh);
    if (tid == 0) first_sh = PT;
    __syncthreads();
    if (bt + sthr >= thr) atomicMin(&first_sh, tid);
    __syncthreads();
    if (tid == first_sh) {
      u128 acc = bt;
      for (int e = 0; e < PB / PT; ++e) {
        acc += cl[e];
        if (acc >= thr && i0 + e < nv) {
          idx_sh = i0 + e;
          break;
        }
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    // sklearn clips an out-of-range candidate to the last sample
    const long long idx = idx_sh >= 0 ? idx_sh : nv - 1;
    const double cv = nv > 0 ? xr[idx] : 0.0;
    R.cand[t] = cv;
    if (t == 0) R.T = P(T);
    // the sorted range holding the candidate's cell
    bool eq = false, hl = false, hh = false;
    double lo = 0, hi = 0;
    for (int j = 0; j < c; ++j) {
      const double cj = R.cen[j];
      if (cj == cv) eq = true;
      else if (cj < cv) {
        if (!hl || cj > lo) lo = cj;
        hl = true;
      } else if (cj > cv) {
        if (!hh || cj < hi) hi = cj;
        hh = true;
      }
    }
    long long a = 0, e = nv;
    if (eq || nv == 0) e = 0;
    else {
      const double mn = geo[0], inv = geo[1];
      const double range = ord_dec(st->hi_bits) - ord_dec(st->lo_bits);
      const double delta = (fabs(lo) + fabs(cv) + fabs(hi) + range) * 0x1p-40;
      if (hl) a = (long long)off[km_bucket(0.5 * lo + 0.5 * cv - delta, mn, inv)];
      if (hh) e = (long long)off[km_bucket(0.5 * cv + 0.5 * hi + delta, mn, inv) + 1];
      if (e > nv) e = nv;
      if (a > e) a = e;
    }
    rng[2 * (r * NTMAX + t)] = a;
    rng[2 * (r * NTMAX + t) + 1] = e;
  }
}

// per sorted chunk (one pass over xs for all runs and trials): the chunk's part of every trial's
// correction -> part2[(r * NTMAX + t) * nch + chunk] (zero where the cell misses the chunk)
__global__ __launch_bounds__(PT) void km_pp_corr_kernel(const double *__restrict__ xs, const KmState *st, Draws d,
                                                        const long long *__restrict__ rng, U128 *__restrict__ part2,
                                                        int nch, int c) {
  // per (run, trial) the chunk's sum: wave sums added into LDS (exact: carry into the high word)
  __shared__ unsigned long long acc[NRUN * NTMAX][2];
  __shared__ double cen[NRUN][KMAX], cand[NRUN * NTMAX];
  __shared__ long long rg[NRUN * NTMAX][2];
  for (int i = threadIdx.x; i < NRUN * NTMAX; i += PT) {
    acc[i][0] = acc[i][1] = 0;
    cand[i] = st->run[i / NTMAX].cand[i % NTMAX];
    rg[i][0] = rng[2 * i];
    rg[i][1] = rng[2 * i + 1];
  }
  if (threadIdx.x < NRUN * KMAX) cen[threadIdx.x / KMAX][threadIdx.x % KMAX] = st->run[threadIdx.x / KMAX].cen[threadIdx.x % KMAX];
  __syncthreads();
  const int64_t nv = (int64_t)st->nvalid;
  const long long c0 = (long long)blockIdx.x * PB, c1 = c0 + PB < nv ? c0 + PB : nv;
  // a chunk no trial's cell reaches: zero parts, and none of its values is read
  bool reach = false;
  for (int q = 0; q < d.nrun * NTMAX; ++q)
    reach |= q % NTMAX < d.nt && rg[q][0] < c1 && rg[q][1] > c0;
  if (!reach) {
    for (int p = threadIdx.x; p < d.nrun * NTMAX; p += PT)
      if (p % NTMAX < d.nt) part2[(int64_t)p * nch + blockIdx.x] = U128{0ull, 0ull};
    return;
  }
  const double scaleS = ldexp(1.0, st->S);
  double v[PB / PT];
#pragma unroll
  for (int e = 0; e < PB / PT; ++e) {
    const long long i = c0 + (long long)e * PT + threadIdx.x;
    v[e] = i < c1 ? xs[i] : 0.0;
  }
  for (int r = 0; r < d.nrun; ++r) {
    bool any = false;
    for (int t = 0; t < d.nt; ++t) {
      const int q = r * NTMAX + t;
      any |= rg[q][0] < c1 && rg[q][1] > c0;
    }
    if (!any) continue;
    // the closest potentials of the run, in fixed point once for all its trials (the f64 -> u64
    // conversion is a multi-instruction sequence on gfx950)
    double dc[PB / PT];
    unsigned long long dcq[PB / PT];
#pragma unroll
    for (int e = 0; e < PB / PT; ++e) {
      dc[e] = closest_sq(v[e], cen[r], c);
      dcq[e] = (unsigned long long)(dc[e] * scaleS);
    }
    for (int t = 0; t < d.nt; ++t) {
      const int q = r * NTMAX + t;
      const long long a = rg[q][0], b = rg[q][1];
      if (!(a < c1 && b > c0)) continue;
      const double cv = cand[q];
      u128 s = 0;
#pragma unroll
      for (int e = 0; e < PB / PT; ++e) {
        const long long i = c0 + (long long)e * PT + threadIdx.x;
        const double dt = (v[e] - cv) * (v[e] - cv);
        if (i >= a && i < b && i < c1 && dt < dc[e]) s += dcq[e] - (unsigned long long)(dt * scaleS);
      }
      const U128 w = wave_sum128(P(s));
      if ((threadIdx.x & 63) == 0 && (w.lo | w.hi)) {
        const unsigned long long old = atomicAdd(&acc[q][0], w.lo);
        const unsigned long long h = w.hi + (old + w.lo < old ? 1ull : 0ull);
        if (h) atomicAdd(&acc[q][1], h);
      }
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < d.nrun * NTMAX; p += PT)
    if (p % NTMAX < d.nt) part2[(int64_t)p * nch + blockIdx.x] = U128{acc[p][0], acc[p][1]};
}

// per run (one workgroup each): T - corr of every trial, the least (first) wins
__global__ __launch_bounds__(PT) void km_pp_choose_kernel(KmState *st, Draws d, const U128 *__restrict__ part2,
                                                          int nch, int c) {
  __shared__ U128 sh[PT / 64];
  const int r = blockIdx.x;
  SkRun &R = st->run[r];
  const u128 T = U(R.T);
  int bt = 0;
  u128 best = 0;
  for (int t = 0; t < d.nt; ++t) {
    const U128 *p = part2 + (int64_t)(r * NTMAX + t) * nch;
    u128 s = 0;
    for (int b = threadIdx.x; b < nch; b += PT) s += U(p[b]);
    const u128 tt = T - U(block_sum128(P(s), sh));
    if (t == 0 || tt < best) {
      best = tt;
      bt = t;
    }
  }
  if (threadIdx.x == 0) {
    R.cen[c] = R.cand[bt];
    R.T = P(best);
    R.ncen = c + 1;
  }
}

// ---- Lloyd on the sorted array ---------------------------------------------------------------
// 256 threads: one wave per SIMD, so a run's workgroup fits in the registers one retiring
// classifier workgroup frees (a 1024-thread workgroup needs four waves' worth on every SIMD of
// one CU and, with the classifier resident everywhere, waited for its grid to drain: 2.2 ms
// in-bench for a 21 us kernel)
constexpr int KS_T = 256;            // threads of an iteration workgroup
constexpr int KS_P = 16;             // probes per thread per round -> 4096-ary search
static_assert(KS_T * KS_P == 4096, "index arithmetic below shifts by 12");

// label of v: sklearn id of the first minimum of (v - c_j)^2 in sklearn order
template <int K>
__device__ __forceinline__ int sk_assign(double v, const double *c) {
  int bj = 0;
  double bd = (v - c[0]) * (v - c[0]);
#pragma unroll
  for (int j = 1; j < K; ++j) {
    const double dd = (v - c[j]) * (v - c[j]);
    if (dd < bd) {
      bd = dd;
      bj = j;
    }
  }
  return bj;
}

// For sorted boundary j (sorted ranks <= j versus > j): the count of samples with rank <= j,
// the sum of their q and of their q^2.  Invariant: the range [lo, hi) starts and ends on
// bucket boundaries, every sample before it has rank <= j and every sample after it rank > j
// (ranks are non-decreasing in the value, buckets ordered by value).  A round probes 4096
// evenly spaced samples; the range shrinks to [start of the last bucket holding a "<= j"
// probe, end of the first bucket holding a "> j" probe).  A range of <= 4096 samples, or one a
// round could not halve, is counted exhaustively.
template <int K>
__device__ void km_bucket_step(const double *__restrict__ xs, const long long *__restrict__ bq,
                               const U128 *__restrict__ bq2, const unsigned long long *__restrict__ off,
                               const KmState *st, int64_t nv, int s, double mn, double inv, double range,
                               const double *c, const int *pos, const double *cso, int j, int64_t *cnt_le,
                               long long *sum_le, U128 *sq_le) {
  const int t = threadIdx.x;
  __shared__ int64_t lo_sh, hi_sh;
  __shared__ int bf_sh, bt_sh, exh_sh;
  __shared__ unsigned long long nf_sh;
  __shared__ long long sf_sh;
  __shared__ U128 qf_sh[KS_T / 64];
  if (t == 0) {
    // direct bracket: the step lies within delta of the midpoint of the sorted centres j, j+1
    const double m = 0.5 * cso[j] + 0.5 * cso[j + 1];
    const double delta = (fabs(cso[j]) + fabs(cso[j + 1]) + range) * 0x1p-40;
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
      if (t == 0) {
        nf_sh = 0;
        sf_sh = 0;
      }
      __syncthreads();
      unsigned long long nf = 0;
      long long sf = 0;
      u128 qf = 0;
      for (int64_t idx = lo + t; idx < hi; idx += KS_T) {
        const double v = xs[idx];
        if (pos[sk_assign<K>(v, c)] <= j) {
          const long long qi = km_q(v, s);
          nf += 1;
          sf += qi;
          qf += km_q2(qi);
        }
      }
      nf = hrf::wave_sum(nf);
      sf = hrf::wave_sum(sf);
      const U128 qw = wave_sum128(P(qf));
      if ((t & 63) == 0) {
        qf_sh[t >> 6] = qw;
        if (nf) {
          atomicAdd(&nf_sh, nf);
          atomicAdd((unsigned long long *)&sf_sh, (unsigned long long)sf);
        }
      }
      __syncthreads();
      if (t == 0) {
        // lo starts a bucket (or is nv): the sums before it
        long long pa = st->sumq;
        u128 qa = U(st->sumq2);
        if (lo < nv) {
          const int lb = km_bucket(xs[lo], mn, inv);
          pa = bq[lb];
          qa = U(bq2[lb]);
        }
        for (int w = 0; w < KS_T / 64; ++w) qa += U(qf_sh[w]);
        *cnt_le = lo + (int64_t)nf_sh;
        *sum_le = pa + sf_sh;
        *sq_le = P(qa);
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
      if (pos[sk_assign<K>(v, c)] <= j) bf = b > bf ? b : bf;
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

// the assignment for the centres c (sklearn order): per sklearn id count, sum q, sum q^2;
// the label signature (sorted ranks -> ids, cumulative counts)
template <int K>
__device__ void km_assign_all(const double *xs, const long long *bq, const U128 *bq2, const unsigned long long *off,
                              const KmState *st, int64_t nv, int s, double mn, double inv, double range,
                              const double *c, int *ids, int *pos, double *cso, int64_t *cle, long long *sle,
                              U128 *qle, long long *cnt, long long *sum, U128 *sq) {
  const int t = threadIdx.x;
  if (t == 0) {
    // sorted ranks by (value, sklearn id): among equal centres the first id takes the samples
    for (int j = 0; j < K; ++j) ids[j] = j;
    for (int a = 1; a < K; ++a)
      for (int b = a; b > 0; --b) {
        const int x = ids[b - 1], y = ids[b];
        if (c[y] < c[x] || (c[y] == c[x] && y < x)) {
          ids[b - 1] = y;
          ids[b] = x;
        } else
          break;
      }
    for (int p = 0; p < K; ++p) {
      pos[ids[p]] = p;
      cso[p] = c[ids[p]];
    }
  }
  __syncthreads();
  for (int j = 0; j + 1 < K; ++j)
    if (cso[j] != cso[j + 1])
      km_bucket_step<K>(xs, bq, bq2, off, st, nv, s, mn, inv, range, c, pos, cso, j, &cle[j], &sle[j], &qle[j]);
  __syncthreads();
  if (t == 0) {
    cle[K - 1] = nv;
    sle[K - 1] = st->sumq;
    qle[K - 1] = st->sumq2;
    for (int j = K - 2; j >= 0; --j)
      if (cso[j] == cso[j + 1]) {  // rank j+1 is never taken: the same cumulative state
        cle[j] = cle[j + 1];
        sle[j] = sle[j + 1];
        qle[j] = qle[j + 1];
      }
    int64_t c0 = 0;
    long long s0 = 0;
    u128 q0 = 0;
    for (int p = 0; p < K; ++p) {
      cnt[ids[p]] = cle[p] - c0;
      sum[ids[p]] = sle[p] - s0;
      sq[ids[p]] = P(U(qle[p]) - q0);
      c0 = cle[p];
      s0 = sle[p];
      q0 = U(qle[p]);
    }
  }
  __syncthreads();
}

template <int K>
__global__ __launch_bounds__(KS_T) void km_lloyd_kernel(const double *__restrict__ xs,
                                                        const long long *__restrict__ bq,
                                                        const U128 *__restrict__ bq2,
                                                        const unsigned long long *__restrict__ off,
                                                        const double *__restrict__ geo, KmState *st, int max_iter) {
  __shared__ double c[KMAX], cso[KMAX], oldc[KMAX];
  __shared__ int ids[KMAX], pos[KMAX], oids[KMAX];
  __shared__ int64_t cle[KMAX], ocle[KMAX];
  __shared__ long long sle[KMAX], cnt[KMAX], sum[KMAX];
  __shared__ U128 qle[KMAX], sq[KMAX];
  __shared__ int stop, have_old, nempty;
  __shared__ double rd[KS_T / 64][1];
  __shared__ long long ri[KS_T / 64][1];
  __shared__ long long far_sh[KMAX];
  const int t = threadIdx.x;
  const int r = blockIdx.x;
  SkRun &R = st->run[r];
  const int64_t nv = (int64_t)st->nvalid;
  const int s = st->s;
  const double mn = geo[0], inv = geo[1];
  if (nv == 0 || st->error) {
    if (t == 0) {
      R.inertia = 0;
      R.iters = 0;
      for (int j = 0; j < K; ++j) R.cen[j] = R.lcen[j] = 0;
    }
    return;
  }
  const double range = ord_dec(st->hi_bits) - ord_dec(st->lo_bits);
  if (t < K) c[t] = R.cen[t];
  if (t == 0) {
    stop = 0;
    have_old = 0;
    R.reloc = 0;
  }
  __syncthreads();
  int it;
  for (it = 0; it < max_iter; ++it) {
    km_assign_all<K>(xs, bq, bq2, off, st, nv, s, mn, inv, range, c, ids, pos, cso, cle, sle, qle, cnt, sum, sq);
    if (t == 0) {
      nempty = 0;
      for (int j = 0; j < K; ++j) nempty += cnt[j] == 0;
    }
    __syncthreads();
    if (nempty) {
      // the nempty samples farthest from their own centre (ties: lower value, then lower
      // position) over all samples: per-thread ordered lists, then nempty block-wide rounds
      const int m = nempty;
      double bd[KMAX];
      long long bi[KMAX];
      for (int e = 0; e < KMAX; ++e) {
        bd[e] = -1;
        bi[e] = -1;
      }
      for (int64_t i = t; i < nv; i += KS_T) {
        const double v = xs[i];
        const double cc = c[sk_assign<K>(v, c)];
        const double dd = (v - cc) * (v - cc);
        for (int e = 0; e < m; ++e) {
          // later samples of this thread have larger positions: on equal (d, value) the
          // earlier one stays ahead
          if (bi[e] < 0 || dd > bd[e] || (dd == bd[e] && v < xs[bi[e]])) {
            for (int f = m - 1; f > e; --f) {
              bd[f] = bd[f - 1];
              bi[f] = bi[f - 1];
            }
            bd[e] = dd;
            bi[e] = i;
            break;
          }
        }
      }
      for (int e = 0; e < m; ++e) {
        double d0 = bd[0];
        long long i0 = bi[0];
        for (int o = 32; o > 0; o >>= 1) {
          const double d1 = __shfl_xor(d0, o, 64);
          const long long i1 = __shfl_xor(i0, o, 64);
          if (i1 >= 0 && (i0 < 0 || d1 > d0 || (d1 == d0 && (xs[i1] < xs[i0] || (xs[i1] == xs[i0] && i1 < i0))))) {
            d0 = d1;
            i0 = i1;
          }
        }
        if ((t & 63) == 0) {
          rd[t >> 6][0] = d0;
          ri[t >> 6][0] = i0;
        }
        __syncthreads();
        if (t == 0) {
          double db = -1;
          long long ib = -1;
          for (int w = 0; w < KS_T / 64; ++w) {
            const long long i1 = ri[w][0];
            const double d1 = rd[w][0];
            if (i1 >= 0 && (ib < 0 || d1 > db || (d1 == db && (xs[i1] < xs[ib] || (xs[i1] == xs[ib] && i1 < ib))))) {
              db = d1;
              ib = i1;
            }
          }
          far_sh[e] = ib;
        }
        __syncthreads();
        if (far_sh[e] >= 0 && bi[0] == far_sh[e]) {  // the owner drops its head
          for (int f = 0; f + 1 < m; ++f) {
            bd[f] = bd[f + 1];
            bi[f] = bi[f + 1];
          }
          bd[m - 1] = -1;
          bi[m - 1] = -1;
        }
        __syncthreads();
      }
      if (t == 0) {
        // _relocate_empty_clusters_dense: the e-th empty cluster (ascending id) takes the e-th
        // farthest sample; its old cluster loses it (its label stays)
        int pk = 0;
        for (int j = 0; j < K; ++j) {
          if (cnt[j]) continue;
          const long long fi = far_sh[pk++];
          if (fi < 0) continue;
          const int oj = sk_assign<K>(xs[fi], c);
          const long long qf = km_q(xs[fi], s);
          sum[oj] -= qf;
          cnt[oj] -= 1;
          sum[j] = qf;
          cnt[j] = 1;
          R.reloc += 1;
        }
      }
      __syncthreads();
    }
    if (t == 0) {
      double shift = 0;
      double nc[KMAX];
      for (int j = 0; j < K; ++j) {
        nc[j] = cnt[j] ? ldexp((double)sum[j] / (double)cnt[j], -s) : c[j];
        const double dd = nc[j] - c[j];
        shift += dd * dd;
      }
      // labels equal to the previous iteration's: same cumulative counts and ids per
      // non-empty sorted rank
      bool same = have_old;
      if (same) {
        for (int p = 0; p < K && same; ++p) {
          const int64_t a0 = p ? cle[p - 1] : 0, b0 = p ? ocle[p - 1] : 0;
          if (cle[p] != ocle[p]) same = false;
          else if (cle[p] - a0 > 0 && ids[p] != oids[p]) same = false;
          (void)b0;
        }
      }
      for (int j = 0; j < K; ++j) {
        oldc[j] = c[j];
        c[j] = nc[j];
      }
      if (same) stop = 2;
      else if (shift <= st->tol) stop = 1;
      for (int p = 0; p < K; ++p) {
        ocle[p] = cle[p];
        oids[p] = ids[p];
      }
      have_old = 1;
    }
    __syncthreads();
    if (stop) break;
  }
  if (t == 0) {
    R.iters = it < max_iter ? it + 1 : max_iter;
    R.strict = stop == 2;
  }
  __syncthreads();
  // final labels: strict -> the last assignment (made with oldc); else an E-step with c
  if (stop != 2) {
    km_assign_all<K>(xs, bq, bq2, off, st, nv, s, mn, inv, range, c, ids, pos, cso, cle, sle, qle, cnt, sum, sq);
  }
  if (t == 0) {
    // inertia of the final labels (their own sums, before any relocation) and final centres
    long long n_of[KMAX], s_of[KMAX];
    u128 q_of[KMAX];
    int64_t c0 = 0;
    long long s0 = 0;
    u128 q0 = 0;
    for (int p = 0; p < K; ++p) {
      n_of[ids[p]] = cle[p] - c0;
      s_of[ids[p]] = sle[p] - s0;
      q_of[ids[p]] = U(qle[p]) - q0;
      c0 = cle[p];
      s0 = sle[p];
      q0 = U(qle[p]);
    }
    double I = 0;
    for (int j = 0; j < K; ++j) {
      if (!n_of[j]) continue;
      const double cs = ldexp(c[j], s);
      I += (u128_to_double(q_of[j]) - 2.0 * cs * (double)s_of[j]) + (double)n_of[j] * cs * cs;
    }
    R.inertia = ldexp(I, -2 * s);
    for (int j = 0; j < K; ++j) {
      R.cen[j] = c[j];
      R.lcen[j] = stop == 2 ? oldc[j] : c[j];
    }
    for (int p = 0; p < K; ++p) {
      R.cut[p] = cle[p];
      R.ids[p] = ids[p];
    }
  }
}

// sklearn's _is_same_clustering(labels_a, labels_b): every cluster of a lies inside one cluster
// of b, i.e. every cut of b (between non-empty sorted ranks) is a cut of a
template <int K>
__device__ bool same_clustering(const SkRun &a, const SkRun &b) {
  for (int p = 0; p + 1 < K; ++p) {
    const long long cb = b.cut[p];
    if (cb == 0 || cb == b.cut[K - 1]) continue;
    bool found = false;
    for (int q = 0; q + 1 < K; ++q) found |= a.cut[q] == cb;
    if (!found) return false;
  }
  return true;
}

// winner of the n_init runs; top cluster by `rule`: 0 the largest centre among non-empty
// clusters; 1 (k = 2, multispecies :126-135) the cluster of larger mean positive value when
// both hold a positive sample, else sklearn's cluster 0 (the reference's NaN comparison);
// 2 (k = 2, ecoli :75-84) the larger cluster mean when both are non-empty, else cluster 0
template <int K>
__device__ void km_best(KmState *st, int nrun, int rule, bool write, int *best_out, int *top_out) {
  int best = 0;
  for (int r = 1; r < nrun; ++r)
    if (st->run[r].inertia < st->run[best].inertia && !same_clustering<K>(st->run[r], st->run[best])) best = r;
  const SkRun &B = st->run[best];
  if (write) {
    st->best = best;
    for (int j = 0; j < K; ++j) st->center[j] = B.cen[j];
    st->iters = B.iters;
  }
  long long n_of[KMAX];
  long long c0 = 0;
  for (int p = 0; p < K; ++p) {
    n_of[B.ids[p]] = B.cut[p] - c0;
    c0 = B.cut[p];
  }
  int top = -1;
  for (int j = 0; j < K; ++j)
    if (n_of[j] > 0 && (top < 0 || B.lcen[j] > B.lcen[top])) top = j;
  if (top < 0) top = 0;
  if (K == 2 && rule == 2 && (n_of[0] == 0 || n_of[1] == 0)) top = 0;
  if (K == 2 && rule == 1) {
    // lower interval = sorted rank 0; samples <= 0 fill it first
    const int lo_id = B.ids[0], hi_id = B.ids[1];
    const long long nl = n_of[lo_id], nh = n_of[hi_id], z = st->nle0;
    const long long zl = z < nl ? z : nl, zh = z - zl;
    const bool pos_lo = nl - zl > 0, pos_hi = nh - zh > 0;
    top = (pos_lo && pos_hi) ? hi_id : 0;
  }
  if (write) st->top = top;
  *best_out = best;
  *top_out = top;
}

// samples <= 0 (rule 1), counted on the sorted array: whole buckets below, the straddling one
__device__ __forceinline__ void km_count_le0(const double *__restrict__ xs, const unsigned long long *__restrict__ off,
                                             const double *__restrict__ geo, KmState *st) {
  __shared__ unsigned long long acc;
  const int64_t nv = (int64_t)st->nvalid;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  if (nv == 0) {
    if (threadIdx.x == 0) st->nle0 = 0;
    return;
  }
  const double mn = geo[0], inv = geo[1];
  const int b0 = km_bucket(0.0, mn, inv);
  const int64_t lo = mn > 0.0 ? 0 : (int64_t)off[b0], hi = mn > 0.0 ? 0 : (int64_t)off[b0 + 1];
  unsigned long long c = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) c += xs[i] <= 0.0;
  c = hrf::wave_sum(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&acc, c);
  __syncthreads();
  if (threadIdx.x == 0) st->nle0 = mn > 0.0 ? 0 : lo + (long long)acc;
}

// tol, then the samples <= 0: one launch
__global__ void km_tol_le0_kernel(const double *__restrict__ xs, const unsigned long long *__restrict__ off,
                                  const double *__restrict__ geo, KmState *st) {
  if (threadIdx.x == 0) km_tol(st);
  km_count_le0(xs, off, geo, st);
}

// the winner of the runs (every block works it out from the runs' records; block 0 stores it),
// then the labels / top mask
template <int K>
__global__ void km_label_kernel(const double *__restrict__ x, const uint8_t *__restrict__ valid, int64_t n,
                                KmState *st, int32_t *__restrict__ labels, uint8_t *__restrict__ top, int nrun,
                                int rule) {
  __shared__ int sbest, stop;
  if (threadIdx.x == 0) km_best<K>(st, nrun, rule, blockIdx.x == 0, &sbest, &stop);
  __syncthreads();
  double c[K];
  const SkRun &B = st->run[sbest];
#pragma unroll
  for (int j = 0; j < K; ++j) c[j] = B.lcen[j];
  const int jt = stop;
  const bool err = st->error != 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool ok = (!valid || valid[i]) && !err;
    const int bj = ok ? sk_assign<K>(x[i], c) : -1;
    if (labels) labels[i] = bj;
    if (top) top[i] = (uint8_t)(bj == jt);
  }
}

// ---- workspace ---------------------------------------------------------------------------------
struct SortWs {
  KmState *st;
  double *geo;
  unsigned *cntA, *cntB, *seg, *cB, *sbsum;
  unsigned long long *off;
  double *xs, *xr, *tmpx;
  long long *bq, *cq;
  U128 *bq2, *cq2, *part, *corr;
  long long *rng;
  unsigned long long *nsel;
  void *tmp;
  size_t tmp_bytes;
};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

int64_t nblocks(int64_t n) { return std::max<int64_t>(1, (n + PB - 1) / PB); }

// the compaction's per-block offsets
hrf_status sort_tmp_bytes(int64_t n, size_t *bytes) {
  *bytes = sizeof(unsigned) * (size_t)((std::max<int64_t>(n, 1) + KSC_B - 1) / KSC_B);
  return HRF_OK;
}

// one table, carved in order by carve() (sizes kept in one place)
int nch_b(int64_t n) { return (int)nblocks(n) + KD; }         // coarse-segment chunk bound
int64_t scan_blocks(int64_t n) {
  const int64_t a = (int64_t)KD * nblocks(n), b = (int64_t)KD * (nch_b(n) + 1);
  return (std::max(a, b) + KSC_B - 1) / KSC_B;
}

// one table, carved in order by carve() (sizes kept in one place)
template <class F>
void ws_layout(int64_t n, size_t tmp_bytes, F &&f) {
  const size_t m = (size_t)std::max<int64_t>(n, 1), nb = (size_t)nblocks(n);
  f(align256(sizeof(KmState)));                          // st
  f(256);                                                // geo
  f(align256(sizeof(unsigned) * KD * nb));               // cntA
  f(align256(sizeof(unsigned) * KD * (nch_b(n) + 1)));   // cntB
  f(align256(sizeof(unsigned) * (KD + 1)));              // seg
  f(align256(sizeof(unsigned) * (KD + 1)));              // cB
  f(align256(sizeof(unsigned) * scan_blocks(n)));        // sbsum
  f(align256(sizeof(unsigned long long) * (KM_NB + 1))); // off
  f(align256(sizeof(double) * m));                       // xs
  f(align256(sizeof(double) * m));                       // xr
  f(align256(sizeof(double) * m));                       // tmpx
  f(align256(sizeof(long long) * KM_NB));                // bq
  f(align256(sizeof(long long) * nb));                   // cq
  f(align256(sizeof(U128) * KM_NB));                     // bq2
  f(align256(sizeof(U128) * nb));                        // cq2
  f(align256(sizeof(U128) * NRUN * nb));                 // part
  f(align256(sizeof(U128) * NRUN * NTMAX * nb));         // corr (per trial and sorted chunk)
  f(align256(sizeof(long long) * 2 * NRUN * NTMAX));     // rng
  f(256);                                                // nsel
  f(align256(tmp_bytes));                                // tmp
}

int64_t sort_ws_bytes(int64_t n, size_t tmp_bytes) {
  size_t tot = 0;
  ws_layout(n, tmp_bytes, [&](size_t b) { tot += b; });
  return (int64_t)tot;
}

SortWs carve(void *work, int64_t n, size_t tmp_bytes) {
  char *w = (char *)work;
  char *p[24];
  int i = 0;
  ws_layout(n, tmp_bytes, [&](size_t b) {
    p[i++] = w;
    w += b;
  });
  SortWs ws{};
  int k = 0;
  ws.st = (KmState *)p[k++];
  ws.geo = (double *)p[k++];
  ws.cntA = (unsigned *)p[k++];
  ws.cntB = (unsigned *)p[k++];
  ws.seg = (unsigned *)p[k++];
  ws.cB = (unsigned *)p[k++];
  ws.sbsum = (unsigned *)p[k++];
  ws.off = (unsigned long long *)p[k++];
  ws.xs = (double *)p[k++];
  ws.xr = (double *)p[k++];
  ws.tmpx = (double *)p[k++];
  ws.bq = (long long *)p[k++];
  ws.cq = (long long *)p[k++];
  ws.bq2 = (U128 *)p[k++];
  ws.cq2 = (U128 *)p[k++];
  ws.part = (U128 *)p[k++];
  ws.corr = (U128 *)p[k++];
  ws.rng = (long long *)p[k++];
  ws.nsel = (unsigned long long *)p[k++];
  ws.tmp = p[k++];
  ws.tmp_bytes = tmp_bytes;
  return ws;
}

__global__ void km_state_init_kernel(KmState *st) {
  static_assert(sizeof(KmState) % 8 == 0, "KmState is cleared in 8-byte words");
  unsigned long long *w = reinterpret_cast<unsigned long long *>(st);
  for (int i = threadIdx.x; i < (int)(sizeof(KmState) / 8); i += blockDim.x) w[i] = 0ull;
  __syncthreads();
  if (threadIdx.x == 0) st->lo_bits = ~0ull;
}

// (a last-block scan behind an agent-scope ticket saved one launch per scan but wrote back and
// invalidated the XCD's L2 in every block; it cost end to end and was removed in round 5)
hrf_status scan_u32(unsigned *a, int64_t n, unsigned *bsum, hipStream_t s) {
  const int nb = (int)((n + KSC_B - 1) / KSC_B);
  km_scan_sum_kernel<<<nb, 256, 0, s>>>(a, n, bsum);
  km_scan_blocks_kernel<<<1, 256, 0, s>>>(bsum, nb);
  km_scan_apply_kernel<<<nb, 256, 0, s>>>(a, n, bsum);
  HRF_LAUNCHED();
  return HRF_OK;
}

// Enqueue one KMeans(k) fit: sort (unless `reuse`), k-means++ for all runs, Lloyd, winner,
// labels / top mask, and the read-back of the final state into *fin (host).
template <int K>
hrf_status km_sk_launch(const double *x, const uint8_t *valid, int64_t n, int max_iter, int n_init, int rule,
                        int32_t *labels, uint8_t *top, const SortWs &ws, int reuse, hipStream_t s, KmState *fin) {
  KmState *st = ws.st;
  const unsigned g = hrf::stream_grid(n);
  if (!reuse) {
    // initial state written by a kernel: an asynchronous copy from a host stack object may run
    // after this frame is gone
    km_state_init_kernel<<<1, 256, 0, s>>>(st);
    if (n > 0) km_minmax_kernel<<<std::min<unsigned>(g, 512), 256, 0, s>>>(x, valid, n, st);
    // n > 0: km_hist_a_kernel takes the scales and the bucket geometry
    if (n == 0) km_scale_kernel<<<1, 1, 0, s>>>(st, nullptr);
    HRF_LAUNCHED();
    if (n > 0) {
      const unsigned nch = (unsigned)nblocks(n);
      const int L = nch_b(n) + 1;
      km_hist_a_kernel<<<nch, 256, 0, s>>>(x, valid, n, ws.geo, ws.cntA, (int)nch, st);
      if (hrf_status r = scan_u32(ws.cntA, (int64_t)KD * nch, ws.sbsum, s)) return r;
      km_scatter_a_kernel<<<nch, 256, 0, s>>>(x, valid, n, ws.geo, ws.cntA, (int)nch, ws.tmpx);
      km_segments_kernel<<<1, KD, 0, s>>>(ws.cntA, (int)nch, st, ws.seg, ws.cB);
      km_hist_b_kernel<<<L - 1, 256, 0, s>>>(ws.tmpx, ws.geo, ws.seg, ws.cB, ws.cntB, L);
      if (hrf_status r = scan_u32(ws.cntB, (int64_t)KD * L, ws.sbsum, s)) return r;
      km_bucket_off_kernel<<<KD, KD, 0, s>>>(ws.cntB, L, ws.seg, ws.cB, ws.off);
      km_scatter_b_kernel<<<L - 1, 256, 0, s>>>(ws.tmpx, ws.geo, ws.seg, ws.cB, ws.cntB, L, ws.off, ws.xs);
      km_chunk_sum_kernel<<<nch, PT, 0, s>>>(ws.xs, st, ws.cq, ws.cq2);
      km_chunk_scan_kernel<<<1, PT, 0, s>>>(ws.cq, ws.cq2, (int)nch, st);
      km_bucket_prefix_kernel<<<nch, PT, 0, s>>>(ws.xs, st, ws.geo, ws.cq, ws.cq2, ws.bq, ws.bq2);
      HRF_LAUNCHED();
      if (valid) {  // the valid samples in raster order (sklearn's sample order)
        const int nsb = (int)((n + KSC_B - 1) / KSC_B);
        unsigned *boff = (unsigned *)ws.tmp;
        km_sel_count_kernel<<<nsb, 256, 0, s>>>(valid, n, boff);
        km_scan_blocks_kernel<<<1, 256, 0, s>>>(boff, nsb);
        km_sel_scatter_kernel<<<nsb, 256, 0, s>>>(x, valid, n, boff, ws.xr, ws.nsel);
        HRF_LAUNCHED();
      }
      km_tol_le0_kernel<<<1, 1024, 0, s>>>(ws.xs, ws.off, ws.geo, st);
      HRF_LAUNCHED();
    }
  }
  if (n == 0) {
    if (fin) HRF_HIP(hipMemcpyAsync(fin, st, sizeof(KmState), hipMemcpyDeviceToHost, s));
    return HRF_OK;
  }
  // the random stream does not depend on the data, only on the number of valid samples: the
  // host needs it before the launches.  n itself when there is no mask; with a mask the count
  // comes from the device (one synchronisation, masked calls only).
  int64_t nv = n;
  if (valid) {
    unsigned long long h = 0;
    HRF_HIP(hipMemcpyAsync(&h, &st->nvalid, sizeof(h), hipMemcpyDeviceToHost, s));
    HRF_HIP(hipStreamSynchronize(s));
    nv = (int64_t)h;
  }
  const Draws d = make_draws(std::max<int64_t>(nv, 1), K, n_init, 0u);
  const double *xr = valid ? ws.xr : x;
  const int nblk = (int)nblocks(nv);
  if (K == 1) km_pp_first_kernel<<<1, 64, 0, s>>>(xr, st, d);  // K > 1: the first pass takes them
  HRF_LAUNCHED();
  for (int c = 1; c < K; ++c) {
    km_pp_pass_kernel<<<nblk, PT, 0, s>>>(xr, st, d, ws.part, nblk, c);
    km_pp_pick_kernel<<<n_init * d.nt, PT, 0, s>>>(xr, ws.off, ws.geo, st, d, ws.part, nblk, c, ws.rng);
    km_pp_corr_kernel<<<nblk, PT, 0, s>>>(ws.xs, st, d, ws.rng, ws.corr, nblk, c);
    km_pp_choose_kernel<<<n_init, PT, 0, s>>>(st, d, ws.corr, nblk, c);
    HRF_LAUNCHED();
  }
  km_lloyd_kernel<K><<<n_init, KS_T, 0, s>>>(ws.xs, ws.bq, ws.bq2, ws.off, ws.geo, st, max_iter);
  km_label_kernel<K><<<g, 256, 0, s>>>(x, valid, n, st, labels, top, n_init, rule);
  HRF_LAUNCHED();
  if (fin) HRF_HIP(hipMemcpyAsync(fin, st, sizeof(KmState), hipMemcpyDeviceToHost, s));
  return HRF_OK;
}

hrf_status km_launch_k(int k, const double *x, const uint8_t *valid, int64_t n, int max_iter, int n_init, int rule,
                       int32_t *labels, uint8_t *top, const SortWs &ws, int reuse, hipStream_t s, KmState *fin) {
  switch (k) {
#define HRF_KML(KK) \
  case KK: return km_sk_launch<KK>(x, valid, n, max_iter, n_init, rule, labels, top, ws, reuse, s, fin);
    HRF_KML(1) HRF_KML(2) HRF_KML(3) HRF_KML(4) HRF_KML(5) HRF_KML(6) HRF_KML(7)
#undef HRF_KML
    default: return km_sk_launch<8>(x, valid, n, max_iter, n_init, rule, labels, top, ws, reuse, s, fin);
  }
}

hrf_status check_args(int32_t k, int64_t n, int32_t max_iter, int32_t n_init, int32_t rule, const void *work,
                      const double *x) {
  HRF_REQUIRE(k >= 1 && k <= KMAX, "kmeans_1d: k must be 1..8");
  HRF_REQUIRE(n >= 0 && n < ((int64_t)1 << 32) - KS_CH && max_iter >= 1 && work, "kmeans_1d: bad arguments");
  HRF_REQUIRE(n_init >= 1 && n_init <= NRUN, "kmeans_1d: n_init must be 1..10");
  HRF_REQUIRE(rule >= 0 && rule <= 2, "kmeans_1d: top rule must be 0, 1 or 2");
  HRF_REQUIRE(n == 0 || x, "kmeans_1d: null input");
  return HRF_OK;
}

// the final state of this thread's last hrf_kmeans_1d_sorted call (pinned host copy)
KmState *&last_single_state() {
  static thread_local KmState *fin = nullptr;
  return fin;
}

}  // namespace

extern "C" {

hrf_status hrf_kmeans_last_runs(int32_t *iters, int32_t *relocations, int32_t *strict, int32_t n) {
  KmState *f = last_single_state();
  HRF_REQUIRE(f && n >= 1 && n <= NRUN && iters, "kmeans_last_runs: no hrf_kmeans_1d_sorted call on this thread yet");
  for (int r = 0; r < n; ++r) {
    iters[r] = f->run[r].iters;
    if (relocations) relocations[r] = f->run[r].reloc;
    if (strict) strict[r] = f->run[r].strict;
  }
  return HRF_OK;
}

int64_t hrf_kmeans_sorted_workspace_bytes(int64_t n) {
  size_t tb = 0;
  if (sort_tmp_bytes(n, &tb) != HRF_OK) return -1;
  return sort_ws_bytes(n, tb);
}

hrf_status hrf_kmeans_draws(int64_t nv, int32_t k, int32_t n_init, int64_t *first_host, double *draws_host) {
  HRF_REQUIRE(nv >= 1 && k >= 1 && k <= KMAX && n_init >= 1 && n_init <= NRUN, "kmeans_draws: bad arguments");
  const Draws d = make_draws(nv, k, n_init, 0u);
  int64_t o = 0;
  for (int r = 0; r < n_init; ++r) {
    first_host[r] = d.first[r];
    for (int c = 1; c < k; ++c)
      for (int t = 0; t < d.nt; ++t) draws_host[o++] = ldexp((double)d.m[r][c - 1][t], -53);
  }
  return HRF_OK;
}

hrf_status hrf_kmeans_1d_sorted(const double *x, const uint8_t *valid, int64_t n, int32_t k, int32_t max_iter,
                                int32_t n_init, int32_t top_rule, int32_t *labels, uint8_t *top_mask,
                                double *centers_host, int32_t *iters_host, void *work, int64_t work_bytes,
                                int32_t reuse_sort, hrf_stream_t stream) {
  if (hrf_status r = check_args(k, n, max_iter, n_init, top_rule, work, x)) return r;
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
  KmState *&fin = last_single_state();
  if (!fin) HRF_HIP(hipHostMalloc((void **)&fin, sizeof(KmState), hipHostMallocDefault));
  if (hrf_status r = km_launch_k(k, x, valid, n, max_iter, n_init, top_rule, labels, top_mask, ws, reuse_sort, s, fin))
    return r;
  HRF_HIP(hipStreamSynchronize(s));
  HRF_REQUIRE(!fin->error, "kmeans_1d: input contains NaN (sklearn KMeans raises ValueError)");
  if (centers_host)
    for (int j = 0; j < k; ++j) centers_host[j] = fin->center[j];
  if (iters_host) *iters_host = fin->iters;
  return HRF_OK;
}

}  // extern "C"

// The pair without its synchronisation (the native E. coli driver): the NaN flag lands in
// *err_pinned (pinned host memory), or stays on the device for the caller's own read-back
// (err_pinned == nullptr), and the caller checks it after its next synchronisation.
hrf_status hrf::kmeans_1d_sorted_pair_deferred(const double *x, int64_t n, int32_t k1, int32_t k2, int32_t max_iter,
                                               int32_t n_init, int32_t rule1, int32_t rule2, uint8_t *top1,
                                               uint8_t *top2, void *work, int64_t work_bytes, hipStream_t s,
                                               int32_t *err_pinned) {
  if (hrf_status r = check_args(k1, n, max_iter, n_init, rule1, work, x)) return r;
  if (hrf_status r = check_args(k2, n, max_iter, n_init, rule2, work, x)) return r;
  const int64_t need = hrf_kmeans_sorted_workspace_bytes(n);
  HRF_REQUIRE(need > 0 && work_bytes >= need, "kmeans_1d_pair: workspace too small");
  size_t tb = 0;
  if (hrf_status r = sort_tmp_bytes(n, &tb)) return r;
  const SortWs ws = carve(work, n, tb);
  if (hrf_status r = km_launch_k(k1, x, nullptr, n, max_iter, n_init, rule1, nullptr, top1, ws, 0, s, nullptr)) return r;
  if (hrf_status r = km_launch_k(k2, x, nullptr, n, max_iter, n_init, rule2, nullptr, top2, ws, 1, s, nullptr)) return r;
  // err_pinned == nullptr: the caller reads the flag itself (hrf::kmeans_error_flag)
  if (err_pinned) HRF_HIP(hipMemcpyAsync(err_pinned, &ws.st->error, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  return HRF_OK;
}

// device address of the NaN flag of the last fit in this workspace (n values)
const int32_t *hrf::kmeans_error_flag(void *work, int64_t n) {
  size_t tb = 0;
  if (sort_tmp_bytes(n, &tb) != HRF_OK) return nullptr;
  return &carve(work, n, tb).st->error;
}

extern "C" {

hrf_status hrf_kmeans_1d_sorted_pair(const double *x, const uint8_t *valid, int64_t n, int32_t k1, int32_t k2,
                                     int32_t max_iter, int32_t n_init, int32_t rule1, int32_t rule2, uint8_t *top1,
                                     uint8_t *top2, void *work, int64_t work_bytes, hrf_stream_t stream) {
  if (hrf_status r = check_args(k1, n, max_iter, n_init, rule1, work, x)) return r;
  if (hrf_status r = check_args(k2, n, max_iter, n_init, rule2, work, x)) return r;
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
  // both fits enqueued (the second reuses the sort), one synchronisation for the NaN check
  static thread_local KmState *fin = nullptr;
  if (!fin) HRF_HIP(hipHostMalloc((void **)&fin, sizeof(KmState), hipHostMallocDefault));
  if (hrf_status r = km_launch_k(k1, x, valid, n, max_iter, n_init, rule1, nullptr, top1, ws, 0, s, nullptr)) return r;
  if (hrf_status r = km_launch_k(k2, x, valid, n, max_iter, n_init, rule2, nullptr, top2, ws, 1, s, fin)) return r;
  HRF_HIP(hipStreamSynchronize(s));
  HRF_REQUIRE(!fin->error, "kmeans_1d_pair: input contains NaN (sklearn KMeans raises ValueError)");
  return HRF_OK;
}

}  // extern "C"
