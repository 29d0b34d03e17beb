// xcorr.hip -- the registration cross-correlations of a tile in six launches (§8 row f1).
//
// skimage.feature.register_translation(ref, img) (upsample_factor 1): the shift is the location of
// max |ifft2(F(ref) * conj(F(img)))| (first in raster order), wrapped per axis to (-n/2, n/2]
// (ecoli measurement.py:45-57 on channel-max images, multispecies :82-84 on channel sums).  For
// power-of-two image sizes (16..4096 per axis) this file replaces the hipFFT path of register.hip
// (two D2Z, a product launch, one Z2D and two argmax launches per target, ~30 launches and ~2.4 GB
// of f64 traffic per 2048^2 tile of five lasers, a third of it rocFFT's transposes) with one f64
// pipeline whose frequency-domain data never leaves a column-blocked order:
//   1. rows, forward: every image row (W reals) as W/2 complex points (even + i odd), one LDS
//      Stockham FFT, then the real-FFT split -> W/2 + 1 bins per row;
//   2. columns, forward pass A (four-step, H = H1 * H2): for each n2 the H1-point DFT over rows
//      n2 + H2 n1, times exp(-2 pi i n2 k1 / H), in place (rows n2 + H2 k1);
//   3. columns, pass B fused with the product and its inverse: per k1, the H2 rows H2 k1 + n2 of
//      the reference and of every target are transformed over n2, multiplied ref * conj(target)
//      and transformed back -- the spectra of the targets are never written in natural order;
//   4. columns, inverse pass A: conj twiddle, inverse H1-point DFT -> rows in natural order;
//   5. rows, inverse: the inverse real-FFT split, one LDS FFT, |cc| and the first maximum per row;
//   6. per target the first maximum over rows -> the wrapped (and clamped) shift.
// Scale: no 1/N anywhere (a positive power-of-two factor leaves the argmax).  Twiddles are
// exp(-2 pi i j / N) tables per size (host long double, rounded to double).  Every column pass
// moves 32-column tiles (512-byte row segments).  The reference's own ifftn keeps the complex
// result and takes |.| with its ~1e-16 imaginary noise; here the inverse is real -- both differ
// from each other only in rounding, as the hipFFT path did (tests/test_registration_gpu.py).
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include <cstdlib>

#include "common.hpp"

namespace {

constexpr int XT = 256;      // threads per workgroup
constexpr int TCA = 32;      // columns per tile, column pass A (512-byte row segments)
constexpr int TCB = 16;      // columns per tile, fused pass B (two tiles in LDS)

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 conj2(double2 a) { return make_double2(a.x, -a.y); }

// In-place Stockham FFT (radix 4, a final radix 2 when LG is odd) of NB = 2^LGNB transforms of
// M = 2^LG points in LDS.  Rows (NB = 1): element i at buf[i].  Columns (COLS): element i of
// transform b at buf[i * NB + b] (a tile of NB adjacent columns), consecutive lanes on
// consecutive columns so every LDS access is conflict-free.  tw[j * ts] = exp(-2 pi i j / M);
// INV: the conjugate (unnormalised inverse).  Each stage reads its inputs into registers, then
// (after a barrier) writes its outputs; sizes are compile-time, so a thread holds at most
// ceil(NB M / 4 / XT) butterflies.
template <int LG, int LGNB, bool INV>
__device__ __forceinline__ void lds_fft(double2 *buf, const double2 *__restrict__ tw, int ts) {
  constexpr int M = 1 << LG, NB = 1 << LGNB;
  const int tid = threadIdx.x;
#pragma unroll
  for (int lgLs = 0; lgLs + 2 <= LG; lgLs += 2) {
    constexpr int Q = M >= 4 ? M >> 2 : 1;  // (the loop does not run for M < 4)
    constexpr int NBF = NB * Q;
    constexpr int MB = (NBF + XT - 1) / XT;
    const int Ls = 1 << lgLs;
    double2 o[MB][4];
    int ob[MB];
#pragma unroll
    for (int r = 0; r < MB; ++r) {
      const int u = tid + r * XT;
      ob[r] = -1;
      if (NBF % XT == 0 || u < NBF) {
        const int b = u & (NB - 1), j = u >> LGNB;
        const int k = j & (Ls - 1), g = j >> lgLs;
        double2 x0 = buf[j * NB + b], x1 = buf[(j + Q) * NB + b], x2 = buf[(j + 2 * Q) * NB + b],
                x3 = buf[(j + 3 * Q) * NB + b];
        if (lgLs > 0) {  // the first stage's twiddles are all 1
          const int step = (k << (LG - lgLs - 2)) * ts;  // k * M / (4 Ls)
          double2 w1 = tw[step], w2 = tw[2 * step], w3 = tw[3 * step];
          if (INV) {
            w1 = conj2(w1);
            w2 = conj2(w2);
            w3 = conj2(w3);
          }
          x1 = cmul(x1, w1);
          x2 = cmul(x2, w2);
          x3 = cmul(x3, w3);
        }
        const double2 a0 = cadd(x0, x2), a1 = csub(x0, x2), a2 = cadd(x1, x3), a3 = csub(x1, x3);
        // -i a3 = (a3.y, -a3.x); +i a3 = (-a3.y, a3.x)
        const double2 mi = INV ? make_double2(-a3.y, a3.x) : make_double2(a3.y, -a3.x);
        o[r][0] = cadd(a0, a2);
        o[r][1] = cadd(a1, mi);
        o[r][2] = csub(a0, a2);
        o[r][3] = csub(a1, mi);
        ob[r] = ((g << (lgLs + 2)) + k) * NB + b;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MB; ++r)
      if (ob[r] >= 0) {
        const int st = Ls * NB;
        buf[ob[r]] = o[r][0];
        buf[ob[r] + st] = o[r][1];
        buf[ob[r] + 2 * st] = o[r][2];
        buf[ob[r] + 3 * st] = o[r][3];
      }
    __syncthreads();
  }
  if (LG & 1) {  // radix-2 stage, Ls = M / 2
    constexpr int Q = M >> 1;
    constexpr int NBF = NB * Q;
    constexpr int MB = (NBF + XT - 1) / XT;
    double2 o[MB][2];
    int ob[MB];
#pragma unroll
    for (int r = 0; r < MB; ++r) {
      const int u = tid + r * XT;
      ob[r] = -1;
      if (NBF % XT == 0 || u < NBF) {
        const int b = u & (NB - 1), j = u >> LGNB;
        const double2 x0 = buf[j * NB + b];
        double2 w = tw[j * ts];
        if (INV) w = conj2(w);
        const double2 x1 = cmul(buf[(j + Q) * NB + b], w);
        o[r][0] = cadd(x0, x1);
        o[r][1] = csub(x0, x1);
        ob[r] = j * NB + b;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MB; ++r)
      if (ob[r] >= 0) {
        buf[ob[r]] = o[r][0];
        buf[ob[r] + Q * NB] = o[r][1];
      }
    __syncthreads();
  }
}

// 1. forward rows: image img, row y -> spec[(img * H + y) * P + k], k <= M = W / 2 (P = M + 1)
// The row and column passes walk their rows / tiles on a resident grid (round 3: ~1-2 k workgroup
// dispatches per pass instead of ~10 k; under the concurrent classifier each dispatch waits for a
// CU slot).  nrows = all (img, y) rows of the pass.
template <int LGM>
__global__ __launch_bounds__(XT) void xc_row_fwd_kernel(const double *__restrict__ imgs, int64_t H,
                                                        double2 *__restrict__ spec, const double2 *__restrict__ twW,
                                                        int64_t nrows) {
  constexpr int M = 1 << LGM, P = M + 1;
  __shared__ double2 buf[M];
  for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {  // img * H + y
  const double2 *src = reinterpret_cast<const double2 *>(imgs + row * 2 * M);
  for (int n = threadIdx.x; n < M; n += XT) buf[n] = src[n];
  __syncthreads();
  lds_fft<LGM, 0, false>(buf, twW, 2);
  double2 *dst = spec + row * P;
  for (int k = threadIdx.x; k <= M; k += XT) {
    const double2 zk = buf[k & (M - 1)], zc = conj2(buf[(M - k) & (M - 1)]);
    const double2 e = make_double2(0.5 * (zk.x + zc.x), 0.5 * (zk.y + zc.y));
    const double2 d = make_double2(0.5 * (zk.x - zc.x), 0.5 * (zk.y - zc.y));
    const double2 od = make_double2(d.y, -d.x);  // -i d
    dst[k] = cadd(e, cmul(twW[k], od));
  }
  __syncthreads();
  }
}

// load / store one column tile: rows r(i) = r0 + i * rstep (i < n) of columns [c0, c0 + TC)
template <int TC>
__device__ __forceinline__ void tile_load(const double2 *__restrict__ img, int P, int64_t r0, int64_t rstep, int n,
                                          int c0, double2 *buf) {
  for (int e = threadIdx.x; e < n * TC; e += XT) {
    const int i = e / TC, c = e - i * TC;
    buf[e] = c0 + c < P ? img[(r0 + i * rstep) * P + c0 + c] : make_double2(0.0, 0.0);
  }
}
template <int TC>
__device__ __forceinline__ void tile_store(double2 *__restrict__ img, int P, int64_t r0, int64_t rstep, int n, int c0,
                                           const double2 *buf) {
  for (int e = threadIdx.x; e < n * TC; e += XT) {
    const int i = e / TC, c = e - i * TC;
    if (c0 + c < P) img[(r0 + i * rstep) * P + c0 + c] = buf[e];
  }
}

constexpr int lg2c(int n) { return n <= 1 ? 0 : 1 + lg2c(n / 2); }

// 2 / 4. column pass A (forward) or its inverse: image img0 + blockIdx.z, n2 = blockIdx.y,
// tile blockIdx.x; rows n2 + H2 * i, i < H1
template <int LGH1, int LGH2, bool INV>
__global__ __launch_bounds__(XT) void xc_col_a_kernel(double2 *__restrict__ spec, int img0, int P,
                                                      const double2 *__restrict__ twH, int ta, int nimgs) {
  constexpr int H1 = 1 << LGH1, H2 = 1 << LGH2;
  constexpr int64_t H = (int64_t)H1 * H2;
  __shared__ double2 buf[H1 * TCA];
  for (int64_t job = blockIdx.x; job < (int64_t)ta * H2 * nimgs; job += gridDim.x) {  // (img, n2, tile)
  const int tx = (int)(job % ta), n2 = (int)((job / ta) % H2), iz = (int)(job / ((int64_t)ta * H2));
  const int c0 = tx * TCA;
  double2 *img = spec + (int64_t)(img0 + iz) * H * P;
  tile_load<TCA>(img, P, n2, H2, H1, c0, buf);
  __syncthreads();
  if (INV) {  // conj twiddle on element k1, then the inverse DFT over k1
    for (int e = threadIdx.x; e < H1 * TCA; e += XT) buf[e] = cmul(buf[e], conj2(twH[n2 * (e / TCA)]));
    __syncthreads();
    lds_fft<LGH1, lg2c(TCA), true>(buf, twH, H2);
  } else {
    lds_fft<LGH1, lg2c(TCA), false>(buf, twH, H2);
    for (int e = threadIdx.x; e < H1 * TCA; e += XT) buf[e] = cmul(buf[e], twH[n2 * (e / TCA)]);
    __syncthreads();
  }
  tile_store<TCA>(img, P, n2, H2, H1, c0, buf);
  __syncthreads();
  }
}

// 3. column pass B + product + inverse pass B: k1 = blockIdx.y, tile blockIdx.x; rows H2 k1 + n2
template <int LGH1, int LGH2>
__global__ __launch_bounds__(XT) void xc_col_b_kernel(double2 *__restrict__ spec, int nimg, int P,
                                                      const double2 *__restrict__ twH) {
  constexpr int H1 = 1 << LGH1, H2 = 1 << LGH2;
  constexpr int64_t H = (int64_t)H1 * H2;
  __shared__ double2 A[H2 * TCB], B[H2 * TCB];
  const int64_t r0 = (int64_t)blockIdx.y * H2;
  const int c0 = blockIdx.x * TCB;
  tile_load<TCB>(spec, P, r0, 1, H2, c0, A);
  __syncthreads();
  lds_fft<LGH2, lg2c(TCB), false>(A, twH, H1);
  for (int t = 1; t < nimg; ++t) {
    double2 *img = spec + (int64_t)t * H * P;
    tile_load<TCB>(img, P, r0, 1, H2, c0, B);
    __syncthreads();
    lds_fft<LGH2, lg2c(TCB), false>(B, twH, H1);
    // numpy: src_freq * target_freq.conj()
    for (int e = threadIdx.x; e < H2 * TCB; e += XT) {
      const double2 a = A[e], b = B[e];
      B[e] = make_double2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
    }
    __syncthreads();
    lds_fft<LGH2, lg2c(TCB), true>(B, twH, H1);
    tile_store<TCB>(img, P, r0, 1, H2, c0, B);
    __syncthreads();
  }
}

struct RowBest {
  double v;
  int32_t col;
  int32_t pad;
};

// 5. inverse rows of target t = 1 + blockIdx.y, row y = blockIdx.x: the first max |cc| of the row
template <int LGM>
__global__ __launch_bounds__(XT) void xc_row_inv_kernel(const double2 *__restrict__ spec, int64_t H,
                                                        const double2 *__restrict__ twW, RowBest *__restrict__ rowbest,
                                                        double *__restrict__ cc_out, int64_t nrows) {
  constexpr int M = 1 << LGM, P = M + 1;
  __shared__ double2 buf[M];
  __shared__ double rv[XT / 64];
  __shared__ int rc[XT / 64];
  for (int64_t job = blockIdx.x; job < nrows; job += gridDim.x) {  // (target - 1) * H + y
  const int64_t ti = job / H, y = job - ti * H;
  const int t = 1 + (int)ti;
  const double2 *X = spec + ((int64_t)t * H + y) * P;
  for (int k = threadIdx.x; k < M; k += XT) {
    const double2 xk = X[k], xc = conj2(X[M - k]);
    const double2 e = make_double2(0.5 * (xk.x + xc.x), 0.5 * (xk.y + xc.y));
    const double2 d = make_double2(0.5 * (xk.x - xc.x), 0.5 * (xk.y - xc.y));
    const double2 o = cmul(d, conj2(twW[k]));
    buf[k] = make_double2(e.x - o.y, e.y + o.x);  // e + i o
  }
  __syncthreads();
  lds_fft<LGM, 0, true>(buf, twW, 2);
  if (cc_out) {  // the correlation surface itself (tests): H * W / 2 times numpy.fft.ifft2
    double2 *o = reinterpret_cast<double2 *>(cc_out + (ti * H + y) * 2 * M);
    for (int n = threadIdx.x; n < M; n += XT) o[n] = buf[n];
  }
  double bv = -1.0;
  int bc = 0x7fffffff;
  for (int n = threadIdx.x; n < M; n += XT) {  // columns 2n, 2n + 1; increasing per thread
    const double2 z = buf[n];
    const double a = fabs(z.x), b = fabs(z.y);
    if (a > bv) {
      bv = a;
      bc = 2 * n;
    }
    if (b > bv) {
      bv = b;
      bc = 2 * n + 1;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bv, o, 64);
    const int oc = __shfl_xor(bc, o, 64);
    if (ov > bv || (ov == bv && oc < bc)) {
      bv = ov;
      bc = oc;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    rv[threadIdx.x >> 6] = bv;
    rc[threadIdx.x >> 6] = bc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < XT / 64; ++q)
      if (rv[q] > bv || (rv[q] == bv && rc[q] < bc)) {
        bv = rv[q];
        bc = rc[q];
      }
    rowbest[ti * H + y] = RowBest{bv, bc, 0};
  }
  __syncthreads();
  }
}

// 6. per target (blockIdx.x): the first maximum over its rows -> shift[1 + t]; shift[0] = (0, 0)
__global__ __launch_bounds__(XT) void xc_shifts_kernel(const RowBest *__restrict__ rowbest, int64_t H, int64_t W,
                                                       int32_t clamp, int32_t *__restrict__ shift) {
  __shared__ double rv[XT / 64];
  __shared__ long long ri[XT / 64];
  const RowBest *rb = rowbest + (int64_t)blockIdx.x * H;
  double bv = -1.0;
  long long bi = LLONG_MAX;
  for (int64_t y = threadIdx.x; y < H; y += XT) {
    const RowBest q = rb[y];
    if (q.v > bv) {  // increasing rows per thread: the first kept on ties
      bv = q.v;
      bi = y * W + q.col;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bv, o, 64);
    const long long oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    rv[threadIdx.x >> 6] = bv;
    ri[threadIdx.x >> 6] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < XT / 64; ++q)
      if (rv[q] > bv || (rv[q] == bv && ri[q] < bi)) {
        bv = rv[q];
        bi = ri[q];
      }
    int64_t r = bi / W, c = bi % W;
    if (r > H / 2) r -= H;  // midpoints = fix(n / 2)
    if (c > W / 2) c -= W;
    if (clamp >= 0) {
      r = (r > clamp || r < -clamp) ? 0 : r;
      c = (c > clamp || c < -clamp) ? 0 : c;
    }
    shift[2 * (1 + blockIdx.x)] = (int32_t)r;
    shift[2 * (1 + blockIdx.x) + 1] = (int32_t)c;
    if (blockIdx.x == 0) shift[0] = shift[1] = 0;
  }
}

// a resident grid for the walking passes (one workgroup per job lost in round 3's A/B)
template <class Kern>
unsigned xgrid(Kern k, int64_t njobs) {
  return hrf::resident_grid(k, XT, 0, njobs);
}

int ilog2(int64_t n) {
  int l = 0;
  while ((int64_t)1 << l < n) ++l;
  return ((int64_t)1 << l) == n ? l : -1;
}

// exp(-2 pi i j / N), j < N, per (device, N): uploaded once (synchronously, on first use)
std::mutex g_tw_mu;
std::map<std::tuple<int, int64_t>, double2 *> g_tw;

hrf_status twiddles(int64_t N, const double2 **out) {
  int dev = 0;
  HRF_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_tw_mu);
  auto key = std::make_tuple(dev, N);
  auto it = g_tw.find(key);
  if (it != g_tw.end()) {
    *out = it->second;
    return HRF_OK;
  }
  std::vector<double2> h((size_t)N);
  const long double two_pi = 6.283185307179586476925286766559005768L;
  for (int64_t j = 0; j < N; ++j) {
    const long double a = two_pi * (long double)j / (long double)N;
    h[(size_t)j] = make_double2((double)cosl(a), (double)-sinl(a));
  }
  double2 *d = nullptr;
  HRF_HIP(hipMalloc((void **)&d, sizeof(double2) * (size_t)N));
  HRF_HIP(hipMemcpy(d, h.data(), sizeof(double2) * (size_t)N, hipMemcpyHostToDevice));
  g_tw[key] = d;
  *out = d;
  return HRF_OK;
}

bool supported(int32_t nimg, int64_t H, int64_t W) {
  const int lh = ilog2(H), lw = ilog2(W);
  return nimg >= 2 && nimg <= 16 && lh >= 4 && lh <= 12 && lw >= 2 && lw <= 12;
}

}  // namespace

extern "C" {

int64_t hrf_xcorr_workspace_bytes(int32_t nimg, int64_t H, int64_t W) {
  if (!supported(nimg, H, W)) return -1;
  const int64_t P = W / 2 + 1;
  return (int64_t)nimg * H * P * (int64_t)sizeof(double2) + ((int64_t)nimg - 1) * H * (int64_t)sizeof(RowBest) + 256;
}

static hrf_status xcorr_run(const double *imgs, int32_t nimg, int64_t H, int64_t W, void *work, int32_t clamp,
                            int32_t *shifts_dev, double *cc_out, hrf_stream_t stream) {
  HRF_REQUIRE(supported(nimg, H, W), "xcorr_shifts: power-of-two sizes 16..4096 (rows) / 4..4096 (columns), "
                                     "2..16 images");
  HRF_REQUIRE(imgs && work, "xcorr_shifts: null buffer");
  hipStream_t s = (hipStream_t)stream;
  const double2 *twW = nullptr, *twH = nullptr;
  if (hrf_status st = twiddles(W, &twW)) return st;
  if (hrf_status st = twiddles(H, &twH)) return st;
  const int lgH = ilog2(H), lgM = ilog2(W) - 1;
  const int P = (int)(W / 2 + 1);
  double2 *spec = reinterpret_cast<double2 *>(work);
  RowBest *rowbest = reinterpret_cast<RowBest *>(spec + (int64_t)nimg * H * P);
  switch (lgM) {
#define HRF_XR(L)                                                                                        \
  case L:                                                                                                \
    xc_row_fwd_kernel<L><<<xgrid(xc_row_fwd_kernel<L>, nimg * H), XT, 0, s>>>(imgs, H, spec, twW, nimg * H); \
    break;
    HRF_XR(1) HRF_XR(2) HRF_XR(3) HRF_XR(4) HRF_XR(5) HRF_XR(6) HRF_XR(7) HRF_XR(8) HRF_XR(9) HRF_XR(10) HRF_XR(11)
#undef HRF_XR
  }
  const unsigned ta = (unsigned)hrf::cdiv(P, TCA), tb = (unsigned)hrf::cdiv(P, TCB);
  switch (lgH) {
#define HRF_XC(LH)                                                                                        \
  case LH: {                                                                                              \
    constexpr int L1 = LH / 2, L2 = LH - LH / 2;                                                          \
    xc_col_a_kernel<L1, L2, false><<<xgrid(xc_col_a_kernel<L1, L2, false>, (int64_t)ta * (1 << L2) * nimg), XT, 0, \
                                     s>>>(spec, 0, P, twH, (int)ta, nimg);                                  \
    xc_col_b_kernel<L1, L2><<<dim3(tb, 1u << L1), XT, 0, s>>>(spec, nimg, P, twH);                        \
    xc_col_a_kernel<L1, L2, true><<<xgrid(xc_col_a_kernel<L1, L2, true>, (int64_t)ta * (1 << L2) * (nimg - 1)),   \
                                    XT, 0, s>>>(spec, 1, P, twH, (int)ta, nimg - 1);                       \
    break;                                                                                                \
  }
    HRF_XC(4) HRF_XC(5) HRF_XC(6) HRF_XC(7) HRF_XC(8) HRF_XC(9) HRF_XC(10) HRF_XC(11) HRF_XC(12)
#undef HRF_XC
  }
  switch (lgM) {
#define HRF_XI(L)                                                                                           \
  case L:                                                                                                   \
    xc_row_inv_kernel<L><<<xgrid(xc_row_inv_kernel<L>, (nimg - 1) * H), XT, 0, s>>>(spec, H, twW, rowbest, cc_out, \
                                                                                (nimg - 1) * H);           \
    break;
    HRF_XI(1) HRF_XI(2) HRF_XI(3) HRF_XI(4) HRF_XI(5) HRF_XI(6) HRF_XI(7) HRF_XI(8) HRF_XI(9) HRF_XI(10) HRF_XI(11)
#undef HRF_XI
  }
  if (shifts_dev) xc_shifts_kernel<<<(unsigned)(nimg - 1), XT, 0, s>>>(rowbest, H, W, clamp, shifts_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_xcorr_shifts_dev(const double *imgs, int32_t nimg, int64_t H, int64_t W, void *work, int32_t clamp,
                                int32_t *shifts_dev, hrf_stream_t stream) {
  HRF_REQUIRE(shifts_dev, "xcorr_shifts: null buffer");
  return xcorr_run(imgs, nimg, H, W, work, clamp, shifts_dev, nullptr, stream);
}

hrf_status hrf_xcorr_surfaces_dev(const double *imgs, int32_t nimg, int64_t H, int64_t W, void *work, double *cc_out,
                                  hrf_stream_t stream) {
  HRF_REQUIRE(cc_out, "xcorr_surfaces: null buffer");
  return xcorr_run(imgs, nimg, H, W, work, -1, nullptr, cc_out, stream);
}

}  // extern "C"
