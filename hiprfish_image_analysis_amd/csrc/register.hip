// register.hip -- integer registration shift estimate.
//
// skimage.feature.register_translation(src, target) with its defaults (upsample_factor 1,
// space 'real'), as the reference calls it before stack assembly: ecoli
// measurement.py:45-46 (per-laser channel max images), multispecies :82-83 (channel sums),
// biofilm :326-327 (log channel sums).  The cross-correlation ifft(F(src) * conj(F(target)))
// is formed with two real-to-complex f64 FFTs (hipFFT), a pointwise conjugate product over
// the half spectrum and one complex-to-real inverse; the shift is the location of max |cc|
// (first in raster order), wrapped per axis to (-n/2, n/2] (shift > fix(n/2) -> shift - n).
// The argmax is a two-level reduction on (value, index) pairs, deterministic.
#include <hipfft/hipfft.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>

#include "common.hpp"

namespace {

// One plan pair per (device, size), shared by every stream.  The plans' work areas are NOT
// allocated by hipFFT: each call binds a region of its own caller-provided workspace (under
// the mutex, right before it enqueues), so transforms of concurrent tiles on different streams
// never share scratch memory.
struct Plans {
  hipfftHandle fwd, inv;
  size_t work;   // bytes of work area either plan needs
};
std::mutex g_plan_mu;
std::map<std::tuple<int, int64_t, int64_t>, Plans> g_plans;

#define HRF_FFT(expr)                                                               \
  do {                                                                              \
    hipfftResult r_ = (expr);                                                       \
    if (r_ != HIPFFT_SUCCESS) {                                                     \
      ::hrf::set_error("%s failed: hipfft status %d (%s:%d)", #expr, (int)r_,      \
                       __FILE__, __LINE__);                                         \
      return HRF_EHIP;                                                              \
    }                                                                               \
  } while (0)

hrf_status get_plans(int64_t H, int64_t W, Plans *out) {
  int dev = 0;
  HRF_HIP(hipGetDevice(&dev));
  auto key = std::make_tuple(dev, H, W);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) {
    *out = it->second;
    return HRF_OK;
  }
  Plans p{};
  size_t wf = 0, wi = 0;
  HRF_FFT(hipfftCreate(&p.fwd));
  HRF_FFT(hipfftCreate(&p.inv));
  HRF_FFT(hipfftSetAutoAllocation(p.fwd, 0));
  HRF_FFT(hipfftSetAutoAllocation(p.inv, 0));
  HRF_FFT(hipfftMakePlan2d(p.fwd, (int)H, (int)W, HIPFFT_D2Z, &wf));
  HRF_FFT(hipfftMakePlan2d(p.inv, (int)H, (int)W, HIPFFT_Z2D, &wi));
  p.work = std::max(wf, wi);
  g_plans[key] = p;
  *out = p;
  return HRF_OK;
}

// o = a * conj(b) (numpy: src_freq * target_freq.conj())
__global__ void xcorr_product_kernel(const hipfftDoubleComplex *__restrict__ a, const hipfftDoubleComplex *__restrict__ b,
                                     int64_t n, hipfftDoubleComplex *__restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const hipfftDoubleComplex x = a[i], y = b[i];
    o[i] = make_hipDoubleComplex(x.x * y.x + x.y * y.y, x.y * y.x - x.x * y.y);
  }
}

struct Best {
  double v;
  int64_t i;
};
__device__ __forceinline__ Best better(Best a, Best b) {
  // larger |cc| wins, equal values -> smaller raster index (numpy argmax: first occurrence)
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

constexpr int AM_BLOCKS = 1024;

__global__ __launch_bounds__(256) void abs_argmax_partial_kernel(const double *__restrict__ cc, int64_t n,
                                                                 Best *__restrict__ part) {
  Best b{-1.0, INT64_MAX};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = fabs(cc[i]);
    if (v > b.v) b = Best{v, i};  // increasing i per thread: first occurrence kept
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best c{__shfl_xor(b.v, o, 64), (int64_t)__shfl_xor((long long)b.i, o, 64)};
    b = better(b, c);
  }
  __shared__ Best red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) b = better(b, red[q]);
    part[blockIdx.x] = b;
  }
}

__global__ __launch_bounds__(256) void abs_argmax_final_kernel(const Best *__restrict__ part, int nparts,
                                                               int64_t *__restrict__ best_idx) {
  Best b{-1.0, INT64_MAX};
  for (int i = threadIdx.x; i < nparts; i += 256) b = better(b, part[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best c{__shfl_xor(b.v, o, 64), (int64_t)__shfl_xor((long long)b.i, o, 64)};
    b = better(b, c);
  }
  __shared__ Best red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) b = better(b, red[q]);
    *best_idx = b.i;
  }
}

// peak index -> (row, col) shift (midpoints = fix(n / 2)); |component| > clamp -> 0 (clamp >= 0;
// ecoli measurement.py:47-57)
__global__ void shift_of_peak_kernel(const int64_t *__restrict__ bidx, int64_t H, int64_t W, int32_t clamp,
                                     int32_t *__restrict__ shift) {
  const int64_t best = *bidx;
  int64_t r = best / W, c = best % W;
  if (r > H / 2) r -= H;
  if (c > W / 2) c -= W;
  if (clamp >= 0) {
    r = (r > clamp || r < -clamp) ? 0 : r;
    c = (c > clamp || c < -clamp) ? 0 : c;
  }
  shift[0] = (int32_t)r;
  shift[1] = (int32_t)c;
}

// the cross-correlation peak index into bidx (device); the FFT of src is taken unless
// src_fft_ready (then work already holds it, from a previous call with the same src)
hrf_status xcorr_peak(const double *src, const double *target, int64_t H, int64_t W, void *work, bool src_fft_ready,
                      hipStream_t s, int64_t **bidx_out) {
  const int64_t nc = H * (W / 2 + 1);
  char *w = (char *)work;
  hipfftDoubleComplex *fa = (hipfftDoubleComplex *)w;
  hipfftDoubleComplex *fb = fa + nc;
  hipfftDoubleComplex *fp = fb + nc;
  double *cc = (double *)(fp + nc);
  Best *part = (Best *)(cc + H * W);
  int64_t *bidx = (int64_t *)(part + AM_BLOCKS);
  char *fft_work = (char *)(((uintptr_t)(bidx + 1) + 255) & ~(uintptr_t)255);
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);  // plan handles are shared; bind stream + work area, run
    Plans p{};
    if (hrf_status st = get_plans(H, W, &p)) return st;
    HRF_FFT(hipfftSetStream(p.fwd, s));
    HRF_FFT(hipfftSetStream(p.inv, s));
    HRF_FFT(hipfftSetWorkArea(p.fwd, fft_work));
    HRF_FFT(hipfftSetWorkArea(p.inv, fft_work));
    // hipFFT's real-to-complex transform does not modify its input
    if (!src_fft_ready) HRF_FFT(hipfftExecD2Z(p.fwd, const_cast<double *>(src), fa));
    HRF_FFT(hipfftExecD2Z(p.fwd, const_cast<double *>(target), fb));
    xcorr_product_kernel<<<hrf::stream_grid(nc), 256, 0, s>>>(fa, fb, nc, fp);
    HRF_LAUNCHED();
    HRF_FFT(hipfftExecZ2D(p.inv, fp, cc));  // unnormalised: a positive scale leaves the argmax
  }
  const unsigned nb = (unsigned)std::min<int64_t>(AM_BLOCKS, hrf::cdiv(H * W, 256));
  abs_argmax_partial_kernel<<<nb, 256, 0, s>>>(cc, H * W, part);
  abs_argmax_final_kernel<<<1, 256, 0, s>>>(part, (int)nb, bidx);
  HRF_LAUNCHED();
  *bidx_out = bidx;
  return HRF_OK;
}

// ---- all targets of one reference in one batch ------------------------------------------
// One batched D2Z over the nimg images (reference first), one product launch for the nimg - 1
// targets, one batched Z2D, one argmax pass over every correlation surface and one kernel for
// the shifts: a dozen launches per tile set instead of ten per target, and FFT grids nimg
// times larger.
struct BatchPlans {
  hipfftHandle fwd, inv;
  size_t work;
};
std::map<std::tuple<int, int64_t, int64_t, int>, BatchPlans> g_bplans;

hrf_status get_batch_plans(int64_t H, int64_t W, int nimg, BatchPlans *out) {
  int dev = 0;
  HRF_HIP(hipGetDevice(&dev));
  auto key = std::make_tuple(dev, H, W, nimg);
  auto it = g_bplans.find(key);
  if (it != g_bplans.end()) {
    *out = it->second;
    return HRF_OK;
  }
  BatchPlans p{};
  int n[2] = {(int)H, (int)W};
  size_t wf = 0, wi = 0;
  const int real_dist = (int)(H * W), cplx_dist = (int)(H * (W / 2 + 1));
  HRF_FFT(hipfftCreate(&p.fwd));
  HRF_FFT(hipfftCreate(&p.inv));
  HRF_FFT(hipfftSetAutoAllocation(p.fwd, 0));
  HRF_FFT(hipfftSetAutoAllocation(p.inv, 0));
  HRF_FFT(hipfftMakePlanMany(p.fwd, 2, n, nullptr, 1, real_dist, nullptr, 1, cplx_dist, HIPFFT_D2Z, nimg, &wf));
  HRF_FFT(hipfftMakePlanMany(p.inv, 2, n, nullptr, 1, cplx_dist, nullptr, 1, real_dist, HIPFFT_Z2D, nimg - 1, &wi));
  p.work = std::max(wf, wi);
  g_bplans[key] = p;
  *out = p;
  return HRF_OK;
}

// o[t] = F[0] * conj(F[1 + t]) for every target t
__global__ void xcorr_product_batch_kernel(const hipfftDoubleComplex *__restrict__ F, int64_t nc, int ntgt,
                                           hipfftDoubleComplex *__restrict__ o) {
  const int64_t total = nc * ntgt;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / nc, j = i - t * nc;
    const hipfftDoubleComplex x = F[j], y = F[(1 + t) * nc + j];
    o[i] = make_hipDoubleComplex(x.x * y.x + x.y * y.y, x.y * y.x - x.x * y.y);
  }
}

// blockIdx.y = surface; AM_BLOCKS partials per surface
__global__ __launch_bounds__(256) void abs_argmax_partial_batch_kernel(const double *__restrict__ cc, int64_t n,
                                                                       Best *__restrict__ part) {
  const double *c = cc + (int64_t)blockIdx.y * n;
  Best b{-1.0, INT64_MAX};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = fabs(c[i]);
    if (v > b.v) b = Best{v, i};
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best q{__shfl_xor(b.v, o, 64), (int64_t)__shfl_xor((long long)b.i, o, 64)};
    b = better(b, q);
  }
  __shared__ Best red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) b = better(b, red[q]);
    part[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = b;
  }
}

// one workgroup per surface: its peak -> shift[1 + t] (row 0, the reference, = (0, 0))
__global__ __launch_bounds__(256) void shifts_batch_kernel(const Best *__restrict__ part, int nparts, int64_t H,
                                                           int64_t W, int32_t clamp, int32_t *__restrict__ shift) {
  const Best *p = part + (int64_t)blockIdx.x * nparts;
  Best b{-1.0, INT64_MAX};
  for (int i = threadIdx.x; i < nparts; i += 256) b = better(b, p[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best q{__shfl_xor(b.v, o, 64), (int64_t)__shfl_xor((long long)b.i, o, 64)};
    b = better(b, q);
  }
  __shared__ Best red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) b = better(b, red[q]);
    int64_t r = b.i / W, c = b.i % W;
    if (r > H / 2) r -= H;
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

}  // namespace

extern "C" {

int64_t hrf_register_batch_workspace_bytes(int32_t nimg, int64_t H, int64_t W) {
  if (nimg < 2 || nimg > 64 || H < 1 || W < 1 || H > (1 << 15) || W > (1 << 15)) return -1;
  const int64_t nc = H * (W / 2 + 1);
  BatchPlans p{};
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if (get_batch_plans(H, W, nimg, &p) != HRF_OK) return -1;
  }
  const int64_t spectra = (2 * (int64_t)nimg - 1) * nc * (int64_t)sizeof(hipfftDoubleComplex);
  const int64_t surfaces = ((int64_t)nimg - 1) * H * W * (int64_t)sizeof(double);
  const int64_t parts = ((int64_t)nimg - 1) * AM_BLOCKS * (int64_t)sizeof(Best);
  return spectra + surfaces + parts + 512 + (int64_t)p.work;
}

hrf_status hrf_register_translations_batch_dev(const double *imgs, int32_t nimg, int64_t H, int64_t W, void *work,
                                               int32_t clamp, int32_t *shifts_dev, hrf_stream_t stream) {
  HRF_REQUIRE(nimg >= 2 && nimg <= 64 && H >= 1 && W >= 1 && H <= (1 << 15) && W <= (1 << 15),
              "register_translations_batch: bad sizes");
  HRF_REQUIRE(imgs && work && shifts_dev, "register_translations_batch: null buffer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nc = H * (W / 2 + 1), n = H * W;
  char *w = (char *)work;
  hipfftDoubleComplex *F = (hipfftDoubleComplex *)w;           // nimg spectra
  hipfftDoubleComplex *Pr = F + (int64_t)nimg * nc;              // nimg - 1 products
  double *cc = (double *)(Pr + (int64_t)(nimg - 1) * nc);        // nimg - 1 surfaces
  Best *part = (Best *)(cc + (int64_t)(nimg - 1) * n);
  char *fft_work = (char *)(((uintptr_t)(part + (int64_t)(nimg - 1) * AM_BLOCKS) + 255) & ~(uintptr_t)255);
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    BatchPlans p{};
    if (hrf_status st = get_batch_plans(H, W, nimg, &p)) return st;
    HRF_FFT(hipfftSetStream(p.fwd, s));
    HRF_FFT(hipfftSetStream(p.inv, s));
    HRF_FFT(hipfftSetWorkArea(p.fwd, fft_work));
    HRF_FFT(hipfftSetWorkArea(p.inv, fft_work));
    HRF_FFT(hipfftExecD2Z(p.fwd, const_cast<double *>(imgs), F));
    xcorr_product_batch_kernel<<<hrf::stream_grid(nc * (nimg - 1)), 256, 0, s>>>(F, nc, nimg - 1, Pr);
    HRF_LAUNCHED();
    HRF_FFT(hipfftExecZ2D(p.inv, Pr, cc));  // unnormalised: a positive scale leaves the argmax
  }
  const unsigned nb = (unsigned)std::min<int64_t>(AM_BLOCKS, hrf::cdiv(n, 256));
  abs_argmax_partial_batch_kernel<<<dim3(nb, (unsigned)(nimg - 1)), 256, 0, s>>>(cc, n, part);
  shifts_batch_kernel<<<(unsigned)(nimg - 1), 256, 0, s>>>(part, (int)nb, H, W, clamp, shifts_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

int64_t hrf_register_workspace_bytes(int64_t H, int64_t W) {
  if (H < 1 || W < 1 || H > (1 << 20) || W > (1 << 20)) return -1;
  const int64_t nc = H * (W / 2 + 1);
  Plans p{};
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if (get_plans(H, W, &p) != HRF_OK) return -1;
  }
  return 3 * nc * (int64_t)sizeof(hipfftDoubleComplex) + H * W * (int64_t)sizeof(double) +
         AM_BLOCKS * (int64_t)sizeof(Best) + 64 + 256 + (int64_t)p.work;
}

hrf_status hrf_register_translation_dev(const double *src, const double *target, int64_t H, int64_t W, void *work,
                                        int32_t clamp, int32_t *shift_dev, hrf_stream_t stream) {
  HRF_REQUIRE(H >= 1 && W >= 1 && H <= (1 << 20) && W <= (1 << 20), "register_translation: bad image size");
  HRF_REQUIRE(target && work && shift_dev, "register_translation: null buffer");
  hipStream_t s = (hipStream_t)stream;
  int64_t *bidx = nullptr;
  // src == nullptr: the FFT of the reference image is already in the workspace
  if (hrf_status st = xcorr_peak(src, target, H, W, work, src == nullptr, s, &bidx)) return st;
  shift_of_peak_kernel<<<1, 1, 0, s>>>(bidx, H, W, clamp, shift_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_register_translation(const double *src, const double *target, int64_t H, int64_t W, void *work,
                                    int32_t *shift_host, hrf_stream_t stream) {
  HRF_REQUIRE(H >= 1 && W >= 1 && H <= (1 << 20) && W <= (1 << 20), "register_translation: bad image size");
  HRF_REQUIRE(src && target && work && shift_host, "register_translation: null buffer");
  hipStream_t s = (hipStream_t)stream;
  int64_t *bidx = nullptr;
  if (hrf_status st = xcorr_peak(src, target, H, W, work, false, s, &bidx)) return st;
  int64_t best = 0;
  HRF_HIP(hipMemcpyAsync(&best, bidx, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HRF_HIP(hipStreamSynchronize(s));
  int64_t r = best / W, c = best % W;
  if (r > H / 2) r -= H;  // midpoints = fix(n / 2)
  if (c > W / 2) c -= W;
  shift_host[0] = (int32_t)r;
  shift_host[1] = (int32_t)c;
  return HRF_OK;
}

}  // extern "C"
