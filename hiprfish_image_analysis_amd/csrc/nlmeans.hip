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
// (oracle_nl_means_skimage) and this formulation in this file's summation order
// (oracle_nl_means).
//
// MI355X mapping (nl_means_pairs_kernel, below): like skimage, each unordered pixel pair once
// -- the patch distance is symmetric, so one weight per pair serves both ends, half the
// exponentials and distances of a per-pixel walk.  One 1024-thread workgroup = 48 x 64 output
// pixels with the (48+28) x (64+28) reflect-padded f64 neighbourhood in LDS; per shift three
// barrier-separated phases build the pair's row sums, distances + weights and the two
// accumulations through LDS (141 KB: one workgroup, 16 waves per CU).  All 7-term sums use one
// fixed tree (sum7) and -ffp-contract=off, the exponential is hrf_exp_neg_tabw (detmath.h, equal
// to the oracle's hrf_exp_neg_tab bit for bit): results are bit-identical.  HBM traffic is 16 B per
// pixel: the kernel is f64-VALU bound.
//
// nl_means_kernel (HRF_NLM_PERPIXEL=1, timing A/B only) is the round-3 per-pixel walk: every
// ordered shift, 2 columns x 8 rows per thread, the patch distances as running row sums.
#include <cmath>
#include <cstdlib>

#include "common.hpp"
#include "detmath.h"

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

// ---- each unordered pixel pair once -------------------------------------------------------
// skimage's own structure: the patch distance of the pair (a, a+s) is the one of (a+s, a-s+s)
// seen from the other end ((P[a+u] - P[a+s+u])^2 is symmetric), so one weight per pair over
// the half window H+ = {(sr, sc): sr > 0, or sr == 0 and sc > 0} (264 shifts) serves both
// pixels.  One 256-thread workgroup = NP_TH x 64 output pixels; per shift s the pairs whose
// first pixel lies in the box B_s = {q : q in the tile or q + s in the tile} are formed in three
// barrier-separated phases over LDS:
//   rows:    HS[y][x] = sum_{dv=-3..3} (P[y][x+dv] - P[y+sr][x+sc+dv])^2 over B_s's rows +- 3
//            (a thread = 8 consecutive columns of one row: 14 squared differences, 8 sums)
//   columns: D[y][x] = sum_{du=-3..3} HS[y+du][x], w = D <= lim ? e^{-max(D,0)/h2s2} : 0 -> WB
//            (a thread = 8 consecutive rows of one column)
//   pixels:  each output p adds w(p, p+s) P[p+s] and then w(p-s, p) P[p-s]
// The sums run in the per-pixel kernel's order (7 columns left to right, then 7 rows top to
// bottom), so every weight is the one nl_means_kernel forms; the accumulation order over the
// shifts is H+ in raster order, the pair (p, p+s) before (p-s, p) -- oracle_nl_means' order.
// The pixel phase of shift s and the row phase of s+1 touch disjoint buffers and share one
// barrier interval: two barriers per shift.  Row strides are odd (93, 77 doubles) so the
// row-per-lane reads of the row phase hit distinct bank pairs.
constexpr int NP_TW = 64;

// The 7-term sums of the patch distance (a row's 7 squared differences, then 7 row sums) in
// the fixed tree ((v0 + v1) + (v2 + v3)) + ((v4 + v5) + v6): position-independent, so the
// oracle restates it per pixel, while overlapping windows of a segment share their pair sums
// (the compiler CSEs v_i + v_{i+1}): 4 adds per window instead of 6.
__device__ __forceinline__ double sum7(const double *v) {
  return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + v[6]);
}
constexpr int NP_SEGMAX = 16;                               // longest row / column segment built
// Buffers are sized so that the row and column segments run unguarded: a segment's reads and
// writes past the box edge (at most NP_SEGMAX - 1 entries) land in padding that is never read
// back as a result.  Row strides stay odd so row-per-lane accesses hit distinct bank pairs.
constexpr int NP_LW = NP_TW + 2 * NL_HALO + 5;              // 97: box cols + 3 + a full last segment
constexpr int NP_BW = 81;                                   // >= 64 + 16 (last segment's end)
// column segments of cseg rows write weights up to row round_up(Hb, cseg) - 1 and read row sums
// 6 rows further; Hb <= TH + 11
constexpr int np_wh(int th, int cseg) { return (th + NL_DIST + cseg - 1) / cseg * cseg; }
constexpr int np_hsh(int th, int cseg) { return np_wh(th, cseg) + 2 * NL_OFF; }
constexpr int np_lds(int th, int cseg) {
  return ((th + 2 * NL_HALO) * NP_LW + (np_hsh(th, cseg) + np_wh(th, cseg)) * NP_BW + HRF_EXP_WIDE_N) * 8;
}

template <bool VAR, int RSEG, int CSEG, int NT, int NP_TH>
__global__ __launch_bounds__(NT, NT == 256 ? 2 : 4) void nl_means_pairs_kernel(const double *__restrict__ img, int64_t H,
                                                                       int64_t W, double inv, double lim, double var,
                                                                       double *__restrict__ out) {
  static_assert(RSEG <= NP_SEGMAX && CSEG <= NP_SEGMAX, "segment padding");
  constexpr int NP_THREADS = NT, NP_OUT = NP_TW * NP_TH / NT;   // outputs per thread
  constexpr int NP_LH = NP_TH + 2 * NL_HALO, NP_HSH = np_hsh(NP_TH, CSEG), NP_WH = np_wh(NP_TH, CSEG);
  static_assert(NP_OUT * NT == NP_TW * NP_TH, "whole outputs per thread");
  static_assert(np_lds(NP_TH, CSEG) <= 160 * 1024, "LDS");
  __shared__ double P[NP_LH * NP_LW];
  __shared__ double HS[NP_HSH * NP_BW];
  __shared__ double WB[NP_WH * NP_BW];
  __shared__ double ET[HRF_EXP_WIDE_N];  // 2^(-i/64): hrf_exp_neg_tabw
  const int tid = threadIdx.x;
  for (int i = tid; i < HRF_EXP_WIDE_N; i += NT) ET[i] = ldexp(hrf_exp2tab64[-i & 63], -i >> 6);
  const int64_t r0 = (int64_t)blockIdx.y * NP_TH, c0 = (int64_t)blockIdx.x * NP_TW;
  for (int idx = tid; idx < NP_LH * NP_LW; idx += NP_THREADS) {
    const int lr = idx / NP_LW, lc = idx - lr * NP_LW;
    const int64_t gr = reflect_idx(r0 + lr - NL_HALO, H), gc = reflect_idx(c0 + lc - NL_HALO, W);
    P[idx] = lc < NP_TW + 2 * NL_HALO ? img[gr * W + gc] : 0.0;
  }
  for (int idx = tid; idx < NP_HSH * NP_BW; idx += NP_THREADS) HS[idx] = 0.0;
  __syncthreads();

  // output j of the thread: tile index tid + j NT, column-major (lanes walk rows: odd strides)
  int wofs[NP_OUT], pofs[NP_OUT];
  double acc[NP_OUT], wsum[NP_OUT];
#pragma unroll
  for (int j = 0; j < NP_OUT; ++j) {
    const int i = tid + j * NT, orow = i % NP_TH, oc = i / NP_TH;
    wofs[j] = orow * NP_BW + oc;
    pofs[j] = (orow + NL_HALO) * NP_LW + oc + NL_HALO;
    const double v = P[pofs[j]];
    acc[j] = v + v;  // the zero shift: weight exp(0) = 1, added twice
    wsum[j] = 2.0;
  }

#pragma unroll 1
  for (int sr = 0; sr <= NL_DIST; ++sr) {
#pragma unroll 1
    for (int sc = sr == 0 ? 1 : -NL_DIST; sc <= NL_DIST; ++sc) {
      // B_s: rows -sr .. NP_TH-1, columns cmin .. cmin+Wb-1 (tile coordinates)
      const int cmin = sc > 0 ? -sc : 0, Wb = NP_TW + (sc > 0 ? sc : -sc), Hb = NP_TH + sr, nr = Hb + 2 * NL_OFF;
      // rows phase: HS row ry <-> tile row ry - sr - 3
      const int nrs = (Wb + RSEG - 1) / RSEG;
      for (int it = tid; it < nr * nrs; it += NP_THREADS) {
        const int seg = it / nr, ry = it - seg * nr, x0 = seg * RSEG;
        const double *pa = P + (ry - sr - NL_OFF + NL_HALO) * NP_LW + (cmin + x0 - NL_OFF + NL_HALO);
        const double *pb = pa + sr * NP_LW + sc;
        double sq[RSEG + 2 * NL_OFF];
#pragma unroll
        for (int k = 0; k < RSEG + 2 * NL_OFF; ++k) {
          const double t = pa[k] - pb[k];
          sq[k] = VAR ? t * t - var : t * t;
        }
        double *hs = HS + ry * NP_BW + x0;
#pragma unroll
        for (int k = 0; k < RSEG; ++k) hs[k] = sum7(sq + k);
      }
      __syncthreads();
      // columns phase: WB row wy <-> tile row wy - sr, its distance from HS rows wy .. wy+6
      const int ncs = (Hb + CSEG - 1) / CSEG;
      for (int it = tid; it < Wb * ncs; it += NP_THREADS) {
        const int seg = it / Wb, cx = it - seg * Wb, y0 = seg * CSEG;
        const double *h = HS + y0 * NP_BW + cx;
        double hv[CSEG + 2 * NL_OFF];
#pragma unroll
        for (int k = 0; k < CSEG + 2 * NL_OFF; ++k) hv[k] = h[k * NP_BW];
        double *wb = WB + y0 * NP_BW + cx;
#pragma unroll
        for (int k = 0; k < CSEG; ++k) {
          const double D = sum7(hv + k);
          // lim = the largest D with fl(D / h2s2) <= 5 (host): exactly skimage's cut, no division
          // branch-free: the CSEG exponentials are independent chains the scheduler can
          // interleave; the clamp only touches cut pairs (x < -5.0001), whose w is 0 anyway
          // sigma = 0: D is a sum of squares, never negative, and max(D, 0) is D itself
          const double x = -(VAR ? (D > 0.0 ? D : 0.0) : D) * inv;
          const double e = hrf_exp_neg_tabw(fmax(x, -8.0), ET);
          wb[k * NP_BW] = D <= lim ? e : 0.0;
        }
      }
      __syncthreads();
      // pixels phase: (p, p+s) then (p-s, p); w == 0 exactly when the pair is cut
#pragma unroll
      for (int j = 0; j < NP_OUT; ++j) {
        const double w1 = WB[wofs[j] + sr * NP_BW - cmin];
        const double w2 = WB[wofs[j] - sc - cmin];
        const double v1 = P[pofs[j] + sr * NP_LW + sc];
        const double v2 = P[pofs[j] - sr * NP_LW - sc];
        // a cut pair adds w = 0 (oracle_nl_means does the same)
        wsum[j] += w1;
        const double t1 = w1 * v1;
        acc[j] += t1;
        wsum[j] += w2;
        const double t2 = w2 * v2;
        acc[j] += t2;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NP_OUT; ++j) {
    const int i = tid + j * NT;
    const int64_t r = r0 + i % NP_TH, c = c0 + i / NP_TH;
    if (r < H && c < W) out[r * W + c] = acc[j] / wsum[j];
  }
}

template <bool VAR>
void launch_pairs(int rseg, int cseg, int nt, int th, hipStream_t st, const double *img, int64_t H, int64_t W, double inv,
                  double lim, double var, double *out) {
#define HRF_NP(R, C, T, TH)                                                                           \
  if (rseg == R && cseg == C && nt == T && th == TH) {                                                \
    dim3 g((unsigned)hrf::cdiv(W, NP_TW), (unsigned)hrf::cdiv(H, TH));                                \
    nl_means_pairs_kernel<VAR, R, C, T, TH><<<g, T, 0, st>>>(img, H, W, inv, lim, var, out);          \
    return;                                                                                           \
  }
  HRF_NP(8, 4, 1024, 32) HRF_NP(8, 4, 1024, 48) HRF_NP(16, 4, 1024, 48) HRF_NP(8, 8, 1024, 48)
  HRF_NP(8, 4, 768, 48)
#undef HRF_NP
  dim3 g((unsigned)hrf::cdiv(W, NP_TW), (unsigned)hrf::cdiv(H, 48));
  nl_means_pairs_kernel<VAR, 8, 4, 1024, 48><<<g, 1024, 0, st>>>(img, H, W, inv, lim, var, out);
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
  // HRF_NLM_PERPIXEL=1: the round-3 per-pixel kernel (every ordered shift, raster order) for
  // timing A/B only -- its summation order is not oracle_nl_means' any more
  static const bool per_pixel = getenv("HRF_NLM_PERPIXEL") != nullptr;
  if (per_pixel) {
    dim3 grid((unsigned)hrf::cdiv(W, NL_TW), (unsigned)hrf::cdiv(H, NL_TH));
    HRF_REQUIRE(grid.y <= 65535, "nl_means_2d: image too tall");
    if (var == 0.0)
      nl_means_kernel<false><<<grid, NL_THREADS, 0, (hipStream_t)stream>>>(img, H, W, inv, lim, var, out);
    else
      nl_means_kernel<true><<<grid, NL_THREADS, 0, (hipStream_t)stream>>>(img, H, W, inv, lim, var, out);
  } else {
    HRF_REQUIRE(hrf::cdiv(H, 16) <= 65535, "nl_means_2d: image too tall");
    // HRF_NLM_SEG=<rows><cols> (e.g. 0804), HRF_NLM_NT=threads: A/B only
    static const int seg = getenv("HRF_NLM_SEG") ? atoi(getenv("HRF_NLM_SEG")) : 804;
    static const int nt = getenv("HRF_NLM_NT") ? atoi(getenv("HRF_NLM_NT")) : 1024;
    static const int th = getenv("HRF_NLM_TH") ? atoi(getenv("HRF_NLM_TH")) : 48;
    if (var == 0.0)
      launch_pairs<false>(seg / 100, seg % 100, nt, th, (hipStream_t)stream, img, H, W, inv, lim, var, out);
    else
      launch_pairs<true>(seg / 100, seg % 100, nt, th, (hipStream_t)stream, img, H, W, inv, lim, var, out);
  }
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
