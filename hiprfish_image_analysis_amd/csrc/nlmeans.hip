// nlmeans.hip -- 2-D non-local means denoising (a4).
//
// Replaces skimage.restoration.denoise_nl_means(image, h=0.02) on the normalised channel
// sum (multispecies_spectral_image_measurement.py:108; biofilm_analysis.py:350 and the
// other 2-D segmentations): skimage's fast-mode 2-D path with its defaults patch_size 7
// (offset 3), patch_distance 11, sigma 0.  That path (integral images per patch shift, each
// pixel pair visited once and credited to both ends) computes, for every pixel p of the
// reflect-padded image P,
//
//   out[p] = (2 P[p] + sum_{s != 0, d_s <= 5} e^{-d_s} P[p+s]) / (2 + sum_{s != 0, d_s <= 5} e^{-d_s})
//   d_s    = max(sum_{u in 7x7} ((P[p+u] - P[p+s+u])^2 - var), 0) / (n_ch h^2 s^2)
//
// over the (2*11+1)^2 search window; the self term weighs 2 because the zero shift adds its
// weight to the pixel twice.  oracle/hrf_oracle.c holds both the integral-image algorithm
// (oracle_nl_means_skimage) and this formulation in this kernel's summation order
// (oracle_nl_means).
//
// MI355X mapping: one 256-thread workgroup = 64x64 output pixels; the (64+28)^2
// reflect-padded f64 neighbourhood is staged once in LDS (67.7 KB, two workgroups per CU).
// Thread = 2 adjacent columns x 8 rows.  Per shift, each of the 14 rows its patches touch is
// read with 16-byte ds_read_b128 (16 lanes cover 256 contiguous bytes: conflict-free), the
// squared differences of 8 columns are formed once and give both pixels' 7-wide row sums,
// and the 7-high column sums come from registers: ~8.75 b128 reads and ~25 f64 VALU ops per
// (pixel, shift) before the weight.  Sums run in a fixed order (7 columns, then 7 rows) with
// -ffp-contract=off, so the patch distances equal the oracle's bit for bit; exp() may differ
// in the last ulp.  HBM traffic is 16 B per pixel: the kernel is f64-VALU bound (exp).
#include <cmath>

#include "common.hpp"

namespace {

constexpr int NL_OFF = 3;        // patch 7
constexpr int NL_DIST = 11;      // search window 23 x 23
constexpr int NL_HALO = NL_OFF + NL_DIST;          // 14
constexpr int NL_TW = 64, NL_TH = 64;
constexpr int NL_K = 2, NL_R = 8;                  // per-thread block: 2 columns x 8 rows
constexpr int NL_THREADS = (NL_TW / NL_K) * (NL_TH / NL_R);   // 256
constexpr int NL_LW = NL_TW + 2 * NL_HALO;         // 92 doubles: even, rows stay 16-B aligned
constexpr int NL_LH = NL_TH + 2 * NL_HALO;
constexpr int NL_ROWS = NL_R + 2 * NL_OFF;         // 14 rows of squared differences
constexpr double NL_CUTOFF = 5.0;

// exp(x) for x in [-5.0001, 0] (the weights that pass skimage's cut): Cody-Waite reduction
// x = k ln2 + r, |r| <= ln2/2, then the degree-13 Taylor polynomial of e^r in Horner form
// (truncation < 5e-18) and an exact scale by 2^k -- 16 FMAs and no range handling, against
// the library exp's special-case paths.  Within a few ulp of exp(); the weights enter a
// normalised average, so the result moves by ~1e-15 relative.
__device__ __forceinline__ double exp_neg_small(double x) {
  const double k = rint(x * 1.4426950408889634);
  double r = __builtin_fma(-k, 6.93147180369123816490e-01, x);  // ln2 hi (Cody-Waite)
  r = __builtin_fma(-k, 1.90821492927058770002e-10, r);         // ln2 lo
  double p = 1.0 / 6227020800.0;                                // 1/13!
  p = __builtin_fma(p, r, 1.0 / 479001600.0);
  p = __builtin_fma(p, r, 1.0 / 39916800.0);
  p = __builtin_fma(p, r, 1.0 / 3628800.0);
  p = __builtin_fma(p, r, 1.0 / 362880.0);
  p = __builtin_fma(p, r, 1.0 / 40320.0);
  p = __builtin_fma(p, r, 1.0 / 5040.0);
  p = __builtin_fma(p, r, 1.0 / 720.0);
  p = __builtin_fma(p, r, 1.0 / 120.0);
  p = __builtin_fma(p, r, 1.0 / 24.0);
  p = __builtin_fma(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_ldexp(p, (int)k);
}

// numpy.pad(mode='reflect') index: mirror without repeating the edge, period 2(n-1)
__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t n) {
  if (n == 1) return 0;
  const int64_t per = 2 * (n - 1);
  int64_t m = i % per;
  if (m < 0) m += per;
  return m < n ? m : per - m;
}

// Five 16-byte reads = 10 consecutive doubles starting at an even LDS index.
__device__ __forceinline__ void read10(const double *p, double (&v)[10]) {
  const double2 *q = reinterpret_cast<const double2 *>(__builtin_assume_aligned(p, 16));
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const double2 t = q[i];
    v[2 * i] = t.x;
    v[2 * i + 1] = t.y;
  }
}

// One shift (sr, sc) with sc of parity ODD.  The reference window of the thread's 2 columns
// covers LDS columns lc-3 .. lc+4 (lc = 14 + 2g, even), read as the aligned run lc-4 .. lc+5
// (entries 1..8); the shifted window starts at lc-3+sc, aligned when sc is odd (entries
// 0..7), one entry later in the run that starts before it when sc is even (entries 1..8).
template <int ODD, bool VAR>
__device__ __forceinline__ void nl_shift(const double *__restrict__ P, int br, int lc, int sr, int sc, double inv,
                                         double lim, double var, double (&acc)[NL_R][NL_K],
                                         double (&wsum)[NL_R][NL_K]) {
  constexpr int SB = ODD ? 0 : 1;  // first used entry of the shifted run
  double D[NL_R][NL_K];            // running patch distances of the block's rows
  const double *pa = P + (br - NL_OFF) * NL_LW + lc - 4;
  // shifted run start lc-3+sc-SB: written as an even offset so the reads stay ds_read_b128
  const double *pb = pa + sr * NL_LW + (ODD ? 2 * ((sc + 1) >> 1) : 2 * (sc >> 1));
#pragma unroll
  for (int x = 0; x < NL_ROWS; ++x) {
    double a[10], b[10];
    read10(pa + x * NL_LW, a);
    read10(pb + x * NL_LW, b);
    double sq[NL_K + 2 * NL_OFF];
#pragma unroll
    for (int j = 0; j < NL_K + 2 * NL_OFF; ++j) {
      const double t = a[1 + j] - b[SB + j];
      sq[j] = VAR ? t * t - var : t * t;  // sigma = 0 (the reference's call): var is exactly 0
    }
#pragma unroll
    for (int k = 0; k < NL_K; ++k) {
      double s = sq[k];
#pragma unroll
      for (int j = 1; j <= 2 * NL_OFF; ++j) s += sq[k + j];
      // row x enters the distances of output rows x-6 .. x, in increasing row order
#pragma unroll
      for (int i = 0; i < NL_R; ++i) {
        if (i == x) D[i][k] = s;
        else if (i < x && x <= i + 2 * NL_OFF) D[i][k] += s;
      }
    }
    if (x >= 2 * NL_OFF) {  // output row x-6 is complete
      const int i = x - 2 * NL_OFF;
      // P[p + s] of the row's two pixels, re-read from LDS rather than held in registers
      const double *pc = P + (br + i + sr) * NL_LW + lc + sc;
      const double ctr[NL_K] = {pc[0], pc[1]};
#pragma unroll
      for (int k = 0; k < NL_K; ++k) {
        const double Dv = D[i][k];
        // lim = the largest D with fl(D / h2s2) <= 5 (host): exactly skimage's cut, no division
        if (Dv <= lim) {
          const double w = exp_neg_small(-(Dv > 0.0 ? Dv : 0.0) * inv);
          wsum[i][k] += w;
          const double t = w * ctr[k];
          acc[i][k] += t;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool VAR>
__global__ __launch_bounds__(NL_THREADS, 2) void nl_means_kernel(const double *__restrict__ img, int64_t H, int64_t W,
                                                                 double inv, double lim, double var,
                                                                 double *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) double P[NL_LH * NL_LW];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * NL_TH, c0 = (int64_t)blockIdx.x * NL_TW;
  for (int idx = tid; idx < NL_LH * NL_LW; idx += NL_THREADS) {
    const int lr = idx / NL_LW, lc = idx - lr * NL_LW;
    const int64_t gr = reflect_idx(r0 + lr - NL_HALO, H), gc = reflect_idx(c0 + lc - NL_HALO, W);
    P[idx] = img[gr * W + gc];
  }
  __syncthreads();

  // lanes 0-31 of a wave: 32 column pairs (64 columns) of one row strip, lanes 32-63 the next
  const int g = tid & 31, strip = tid >> 5;
  const int lc = NL_HALO + NL_K * g;          // LDS column of the pair's first pixel (even)
  const int br = NL_HALO + NL_R * strip;      // LDS row of the block's first pixel

  double acc[NL_R][NL_K], wsum[NL_R][NL_K];
#pragma unroll
  for (int i = 0; i < NL_R; ++i)
#pragma unroll
    for (int k = 0; k < NL_K; ++k) {
      const double v = P[(br + i) * NL_LW + lc + k];
      acc[i][k] = v + v;  // the zero shift: weight exp(0) = 1, added twice
      wsum[i][k] = 2.0;
    }

#pragma unroll 1
  for (int sr = -NL_DIST; sr <= NL_DIST; ++sr) {
#pragma unroll 1
    for (int sc = -NL_DIST; sc <= NL_DIST; ++sc) {
      if (sc & 1)
        nl_shift<1, VAR>(P, br, lc, sr, sc, inv, lim, var, acc, wsum);
      else if (sr != 0 || sc != 0)
        nl_shift<0, VAR>(P, br, lc, sr, sc, inv, lim, var, acc, wsum);
    }
  }
#pragma unroll
  for (int i = 0; i < NL_R; ++i) {
    const int64_t r = r0 + NL_R * strip + i;
    if (r >= H) continue;
#pragma unroll
    for (int k = 0; k < NL_K; ++k) {
      const int64_t c = c0 + NL_K * g + k;
      if (c < W) out[r * W + c] = acc[i][k] / wsum[i][k];
    }
  }
}

}  // namespace

extern "C" {

hrf_status hrf_nl_means_2d(const double *img, int64_t H, int64_t W, int32_t patch_size, int32_t patch_distance,
                           double h, double sigma, double *out, hrf_stream_t stream) {
  // skimage rounds an even patch size up (s % 2 == 0 -> s + 1)
  const int s = (patch_size % 2 == 0) ? patch_size + 1 : patch_size;
  HRF_REQUIRE(s == 2 * NL_OFF + 1 && patch_distance == NL_DIST,
              "nl_means_2d: only the reference parameters (patch_size 7, patch_distance 11) are built");
  HRF_REQUIRE(H >= 1 && W >= 1 && h > 0.0 && sigma >= 0.0, "nl_means_2d: bad image size or h/sigma");
  HRF_REQUIRE(img && out, "nl_means_2d: null buffer");
  // skimage: h2 = h ** 2, s2 = s ** 2, h2s2 = n_ch * h2 * s2 (n_ch = 1), var = sigma ** 2
  const double h2 = h * h, s2 = (double)s * (double)s;
  const double h2s2 = 1.0 * h2 * s2;
  const double var = sigma * sigma;
  // the cut d = max(D, 0) / h2s2 <= 5 as a threshold on D: fl(D / h2s2) is non-decreasing in D,
  // so walk from 5 h2s2 to the last double whose quotient still rounds to <= 5
  double lim = NL_CUTOFF * h2s2;
  while (lim / h2s2 > NL_CUTOFF) lim = std::nextafter(lim, -1.0);
  while (std::nextafter(lim, 2.0 * lim + 1.0) / h2s2 <= NL_CUTOFF) lim = std::nextafter(lim, 2.0 * lim + 1.0);
  const double inv = 1.0 / h2s2;
  dim3 grid((unsigned)hrf::cdiv(W, NL_TW), (unsigned)hrf::cdiv(H, NL_TH));
  HRF_REQUIRE(grid.y <= 65535, "nl_means_2d: image too tall");
  if (var == 0.0)
    nl_means_kernel<false><<<grid, NL_THREADS, 0, (hipStream_t)stream>>>(img, H, W, inv, lim, var, out);
  else
    nl_means_kernel<true><<<grid, NL_THREADS, 0, (hipStream_t)stream>>>(img, H, W, inv, lim, var, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
