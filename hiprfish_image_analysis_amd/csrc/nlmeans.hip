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
// exponentials and distances of a per-pixel walk.  One 1024-thread workgroup = 52 x 64 output
// pixels with the (52+28) x (64+28) reflect-padded f64 neighbourhood in LDS; per shift three
// barrier-separated phases build the pair's row sums, distances + weights and the two
// accumulations through LDS (151 KB: one workgroup, 16 waves per CU).  All 7-term sums use one
// fixed tree (sum7) and -ffp-contract=off, the exponential is hrf_exp_neg_tabw (detmath.h, equal
// to the oracle's hrf_exp_neg_tab bit for bit): results are bit-identical.  HBM traffic is 16 B per
// pixel: the kernel is f64-VALU bound.
#include <cmath>
#include <cstdlib>

#include "common.hpp"
#include "detmath.h"

namespace {

constexpr int NL_OFF = 3;        // patch 7
constexpr int NL_DIST = 11;      // search window 23 x 23
constexpr int NL_HALO = NL_OFF + NL_DIST;          // 14
constexpr double NL_CUTOFF = 5.0;

// numpy.pad(mode='reflect') index: mirror without repeating the edge, period 2(n-1)
__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t n) {
  if (n == 1) return 0;
  const int64_t per = 2 * (n - 1);
  int64_t m = i % per;
  if (m < 0) m += per;
  return m < n ? m : per - m;
}

// ---- each unordered pixel pair once -------------------------------------------------------
// skimage's own structure: the patch distance of the pair (a, a+s) is the one of (a+s, a-s+s)
// seen from the other end ((P[a+u] - P[a+s+u])^2 is symmetric), so one weight per pair over
// the half window H+ = {(sr, sc): sr > 0, or sr == 0 and sc > 0} (264 shifts) serves both
// pixels.  One workgroup = NP_TH x 64 output pixels; per shift s the pairs whose
// first pixel lies in the box B_s = {q : q in the tile or q + s in the tile} are formed in three
// barrier-separated phases over LDS:
//   rows:    HS[y][x] = sum_{dv=-3..3} (P[y][x+dv] - P[y+sr][x+sc+dv])^2 over B_s's rows +- 3
//            (a thread = 8 consecutive columns of one row: 14 squared differences, 8 sums)
//   columns: D[y][x] = sum_{du=-3..3} HS[y+du][x], w = D <= lim ? e^{-max(D,0)/h2s2} : 0 -> WB
//            (a thread = 8 consecutive rows of one column)
//   pixels:  each output p adds w(p, p+s) P[p+s] and then w(p-s, p) P[p-s]
// The sums run in the per-pixel kernel's order (7 columns left to right, then 7 rows top to
// bottom), as oracle_nl_means forms every weight; the accumulation order over the
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
  constexpr int NP_THREADS = NT, NP_NO = NP_TW * NP_TH, NP_OUT = (NP_NO + NT - 1) / NT;  // outputs per thread
  constexpr int NP_LH = NP_TH + 2 * NL_HALO, NP_HSH = np_hsh(NP_TH, CSEG), NP_WH = np_wh(NP_TH, CSEG);
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
    // a thread past the tile's last output (NP_NO % NT != 0) shadows output 0: computed, never stored
    const int i = tid + j * NT < NP_NO ? tid + j * NT : 0, orow = i % NP_TH, oc = i / NP_TH;
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
    if (i < NP_NO && r < H && c < W) out[r * W + c] = acc[j] / wsum[j];
  }
}

// 52 x 64 tiles, 8-column row segments, 4-row column segments, 1024 threads (3.25 outputs per
// thread): a 2048^2 image is 40 x 32 = 1280 workgroups, exactly five rounds of one workgroup on
// each of the 256 CUs -- 48-row tiles left the sixth round 3/8 full (3.42 vs 3.80 ms, two
// alternating rounds, profiles/r5_nlm_ab.txt)
constexpr int NL_TILE_H = 52;
#ifndef HRF_NLM_RSEG
#define HRF_NLM_RSEG 8  // row-phase segment (columns per item)
#endif
#ifndef HRF_NLM_CSEG
#define HRF_NLM_CSEG 4  // column-phase segment (rows per item)
#endif

template <bool VAR>
void launch_pairs(hipStream_t st, const double *img, int64_t H, int64_t W, double inv, double lim, double var,
                  double *out) {
  dim3 g((unsigned)hrf::cdiv(W, NP_TW), (unsigned)hrf::cdiv(H, NL_TILE_H));
  nl_means_pairs_kernel<VAR, HRF_NLM_RSEG, HRF_NLM_CSEG, 1024, NL_TILE_H><<<g, 1024, 0, st>>>(img, H, W, inv, lim, var, out);
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
  HRF_REQUIRE(hrf::cdiv(H, NL_TILE_H) <= 65535, "nl_means_2d: image too tall");
  if (var == 0.0)
    launch_pairs<false>((hipStream_t)stream, img, H, W, inv, lim, var, out);
  else
    launch_pairs<true>((hipStream_t)stream, img, H, W, inv, lim, var, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
