// stats.hip -- per-label reductions over the (H, W, C) spectral stack and the label map.
//
// a15 hrf_label_sums: the reference computes the per-cell mean spectrum with one skimage
// regionprops pass per channel (ecoli measurement.py:151-155, multispecies :167-171) --
// C passes over the image.  Here one streaming pass that fetches only labelled pixels and
// reduces runs of equal labels per channel in f64, one atomic per (run, channel):
// label_sums_wave_kernel (C <= 128, default) works per wave without LDS or barriers;
// label_sums_kernel (any C) stages 64-pixel chunks through LDS.  Flat-field division
// (ecoli :147-150) is folded into the reduction so the calibrated stack never exists.
// a20 hrf_region_moments/props: exact int64 raw moments (agg. atomics) -> regionprops
// area/centroid/axes/eccentricity/orientation with exact integer central moments.
#include "common.hpp"
#include "wave.hpp"

#include <cstdlib>

namespace {

constexpr int LS_P = 64;  // pixels per chunk

__global__ __launch_bounds__(256) void label_sums_kernel(const float *__restrict__ stack,
                                                         const int32_t *__restrict__ lab, int64_t npix, int C,
                                                         int32_t maxlab, const float *__restrict__ cal, int64_t cal_sp,
                                                         int cal_sc, int cal0, int cal1, double *__restrict__ sums,
                                                         unsigned long long *__restrict__ counts, int vec_ok) {
  extern __shared__ __attribute__((aligned(16))) float sbuf[];
  __shared__ int32_t slab[LS_P];
  __shared__ double scal[LS_P];
  const int tid = threadIdx.x;
  const int64_t nchunks = (npix + LS_P - 1) / LS_P;
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int64_t p0 = ch * LS_P;
    const int np = (int)min((int64_t)LS_P, npix - p0);
    int mine = 0;
    if (tid < LS_P) {
      int32_t l = tid < np ? lab[p0 + tid] : 0;
      if (l < 0 || l > maxlab) l = 0;
      slab[tid] = l;
      scal[tid] = (cal && tid < np && cal_sc == 0) ? (double)cal[(p0 + tid) * cal_sp] : 1.0;
      mine = l != 0;
    }
    if (!__syncthreads_or(mine)) continue;
    const int64_t nel = (int64_t)np * C;
    const float *src = stack + p0 * C;
    if (vec_ok) {
      const int nv = (int)(nel >> 2);
      for (int v = tid; v < nv; v += 256) {
        const int e = v << 2;
        if (slab[e / C] | slab[(e + 3) / C]) reinterpret_cast<float4 *>(sbuf)[v] = reinterpret_cast<const float4 *>(src)[v];
      }
      for (int e = (nv << 2) + tid; e < nel; e += 256)
        if (slab[e / C]) sbuf[e] = src[e];
    } else {
      for (int e = tid; e < nel; e += 256)
        if (slab[e / C]) sbuf[e] = src[e];
    }
    __syncthreads();
    const int half = tid >> 7;
    const int lo = half * (LS_P / 2), hi = min(lo + LS_P / 2, np);
    for (int c = tid & 127; c < C; c += 128) {
      const bool calc = cal && c >= cal0 && c < cal1;
      int32_t run = 0;
      double acc = 0.0;
      for (int i = lo; i < hi; ++i) {
        const int32_t l = slab[i];
        if (l != run) {
          if (run) atomicAdd(&sums[(int64_t)run * C + c], acc);
          run = l;
          acc = 0.0;
        }
        if (l) {
          const double x = (double)sbuf[i * C + c];
          // a plane calibration is staged per pixel; per-channel / full ones are read directly
          acc += calc ? x / (cal_sc == 0 ? scal[i] : (double)cal[(p0 + i) * cal_sp + (int64_t)c * cal_sc]) : x;
        }
      }
      if (run) atomicAdd(&sums[(int64_t)run * C + c], acc);
    }
    if ((tid & 127) == 0) {
      int32_t run = 0;
      unsigned long long n = 0;
      for (int i = lo; i < hi; ++i) {
        const int32_t l = slab[i];
        if (l != run) {
          if (run) atomicAdd(&counts[run], n);
          run = l;
          n = 0;
        }
        n += l != 0;
      }
      if (run) atomicAdd(&counts[run], n);
    }
    __syncthreads();
  }
}

// Wave-per-chunk variant (default): each wave owns a 64-pixel raster chunk at a time, lane =
// pixel for the label read (next chunk's labels prefetched while this one reduces), lane =
// channel (c, c + 64) for the spectra.  Only foreground pixels are fetched, LS_B of them per
// round with every load in flight (each pixel's C floats are contiguous, so a round is LS_B
// coalesced row reads); runs of equal labels accumulate in f64 registers and flush one atomic
// per (run, channel).  No LDS, no workgroup barriers: background chunks cost one ballot.
constexpr int LS_B = 16;

template <int CAL>  // 0 none, 1 per-pixel plane (cal_sc == 0), 2 per-channel / full array
__global__ __launch_bounds__(256) void label_sums_wave_kernel(const float *__restrict__ stack,
                                                              const int32_t *__restrict__ lab, int64_t npix, int C,
                                                              int32_t maxlab, const float *__restrict__ cal,
                                                              int64_t cal_sp, int cal_sc, int cal0, int cal1,
                                                              double *__restrict__ sums,
                                                              unsigned long long *__restrict__ counts) {
  const int lane = hrf::lane_id();
  const int64_t nchunks = (npix + 63) >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t ch = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int c0 = lane, c1 = lane + 64;
  const bool v0 = c0 < C, v1 = c1 < C;
  const bool k0 = CAL != 0 && c0 >= cal0 && c0 < cal1, k1 = CAL != 0 && c1 >= cal0 && c1 < cal1;
  auto load_label = [&](int64_t c) -> int32_t {
    const int64_t p = (c << 6) + lane;
    int32_t l = (c < nchunks && p < npix) ? __builtin_nontemporal_load(lab + p) : 0;
    return (l < 0 || l > maxlab) ? 0 : l;
  };
  int32_t lnext = load_label(ch);
  for (; ch < nchunks; ch += nwaves) {
    const int32_t l = lnext;
    lnext = load_label(ch + nwaves);
    unsigned long long fg = __ballot(l != 0);
    if (!fg) continue;
    const int64_t p0 = ch << 6;
    float pcal = 1.0f;
    if (CAL == 1) pcal = (p0 + lane < npix) ? cal[(p0 + lane) * cal_sp] : 1.0f;
    int32_t run = 0;  // wave-uniform
    unsigned long long n = 0;
    double a0 = 0.0, a1 = 0.0;
    while (fg) {
      int idx[LS_B];
      int nb = 0;
#pragma unroll
      for (int j = 0; j < LS_B; ++j) {
        idx[j] = fg ? __ffsll((long long)fg) - 1 : -1;
        if (fg) { fg &= fg - 1; ++nb; }
      }
      float x0[LS_B], x1[LS_B], q0[LS_B], q1[LS_B];
#pragma unroll
      for (int j = 0; j < LS_B; ++j) {
        x0[j] = x1[j] = 0.0f;
        q0[j] = q1[j] = 1.0f;
        if (j < nb) {
          const int64_t p = p0 + idx[j];
          const float *src = stack + p * C;
          if (v0) x0[j] = __builtin_nontemporal_load(src + c0);
          if (v1) x1[j] = __builtin_nontemporal_load(src + c1);
          if (CAL == 2) {
            if (k0) q0[j] = cal[p * cal_sp + (int64_t)c0 * cal_sc];
            if (k1) q1[j] = cal[p * cal_sp + (int64_t)c1 * cal_sc];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < LS_B; ++j) {
        if (j < nb) {
          const int32_t lj = __builtin_amdgcn_readlane(l, idx[j]);
          if (lj != run) {
            if (run) {
              double *row = sums + (int64_t)run * C;
              if (v0) atomicAdd(row + c0, a0);
              if (v1) atomicAdd(row + c1, a1);
              if (lane == 0) atomicAdd(counts + run, n);
            }
            run = lj;
            a0 = a1 = 0.0;
            n = 0;
          }
          ++n;
          if (CAL == 1) {
            const double d = (double)__builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                 __builtin_bit_cast(int, pcal), idx[j]));
            a0 += k0 ? (double)x0[j] / d : (double)x0[j];
            a1 += k1 ? (double)x1[j] / d : (double)x1[j];
          } else if (CAL == 2) {
            a0 += k0 ? (double)x0[j] / (double)q0[j] : (double)x0[j];
            a1 += k1 ? (double)x1[j] / (double)q1[j] : (double)x1[j];
          } else {
            a0 += (double)x0[j];
            a1 += (double)x1[j];
          }
        }
      }
    }
    double *row = sums + (int64_t)run * C;
    if (v0) atomicAdd(row + c0, a0);
    if (v1) atomicAdd(row + c1, a1);
    if (lane == 0) atomicAdd(counts + run, n);
  }
}

// rows = labels with count > 0, ascending (regionprops order).  One workgroup.
__global__ __launch_bounds__(1024) void cell_rows_kernel(const unsigned long long *__restrict__ counts,
                                                         int32_t maxlab, int32_t *__restrict__ row_of_label,
                                                         int32_t *__restrict__ label_of_row,
                                                         int32_t *__restrict__ nrows) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 1; base <= maxlab; base += 1024) {
    const int64_t l = base + tid;
    const int32_t v = (l <= maxlab && counts[l] > 0) ? 1 : 0;
    const int32_t inc = hrf::wave_inclusive_scan(v);
    if ((tid & 63) == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    if (tid < 64) {
      const int32_t s = tid < 16 ? wsum[tid] : 0;
      const int32_t si = hrf::wave_inclusive_scan(s);
      if (tid < 16) wsum[tid] = si - s;
    }
    __syncthreads();
    const int32_t excl = carry + wsum[tid >> 6] + inc - v;
    if (l <= maxlab) {
      row_of_label[l] = v ? excl : -1;
      if (v) label_of_row[excl] = (int32_t)l;
    }
    __syncthreads();
    if (tid == 1023) carry = excl + v;
    __syncthreads();
  }
  if (tid == 0) {
    row_of_label[0] = -1;
    *nrows = carry;
  }
}

// avgint[row][c] = sums[l][c] / counts[l]; avgint_norm = avgint / max_c(avgint[row])
// one wave per row
__global__ void cell_means_kernel(const double *__restrict__ sums, const unsigned long long *__restrict__ counts,
                                  const int32_t *__restrict__ label_of_row, const int32_t *__restrict__ nrows_dev,
                                  int32_t max_rows, int C, double *__restrict__ avgint, double *__restrict__ avgnorm) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int32_t nrows = *nrows_dev;
  if (row >= nrows || row >= max_rows) return;
  const int32_t l = label_of_row[row];
  const double n = (double)counts[l];
  double mx = -__builtin_inf();
  for (int c = lane; c < C; c += 64) {
    const double m = sums[(int64_t)l * C + c] / n;
    avgint[row * C + c] = m;
    mx = m > mx ? m : mx;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double u = __shfl_xor(mx, o, 64);
    mx = u > mx ? u : mx;
  }
  if (avgnorm)
    for (int c = lane; c < C; c += 64) avgnorm[row * C + c] = avgint[row * C + c] / mx;
}

// raw moments: area, sum r, sum c, sum r^2, sum c^2, sum rc  (exact int64)
__global__ void moments_kernel(const int32_t *__restrict__ lab, int64_t H, int64_t W, int32_t maxlab,
                               unsigned long long *__restrict__ mom) {
  const int64_t n = H * W;
  const int64_t n_up = (n + 63) / 64 * 64;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_up; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = p < n ? lab[p] : 0;
    const bool ok = l > 0 && l <= maxlab;
    const int64_t r = p / W, c = p - (p / W) * W;
    const int64_t key = ok ? (int64_t)l * 6 : 0;
    // six aggregated adds, one per moment, keyed by the label.  When the wave's 64 pixels lie on
    // one image row (always, when 64 divides W), r is uniform: the count is a popcount, the
    // row moments follow from it, and a label's lanes usually form one run [c0, c1] whose column
    // sums have closed forms -- no reductions; otherwise wave sums as before.
    unsigned long long pending = __ballot(ok);
    bool active = ok;
    const int lane = hrf::lane_id();
    const int64_t pb = p - lane, rb = pb / W;
    const bool one_row = pb + 63 < n && (pb + 63) / W == rb;
    while (pending) {
      const int leader = __ffsll((long long)pending) - 1;
      const int64_t k = __shfl(key, leader, 64);
      const bool m = active && key == k;
      const unsigned long long same = __ballot(m);
      unsigned long long a0, a1, a2, a3, a4, a5;
      if (one_row) {
        const unsigned long long cnt = (unsigned long long)__popcll(same);
        const unsigned long long cb = (unsigned long long)(pb - rb * W), rr = (unsigned long long)rb;
        const int hi = 63 - __builtin_clzll(same);
        unsigned long long sc, scc;
        if ((int)cnt == hi - leader + 1) {  // one run: closed forms over [c0, c1]
          const unsigned long long c0 = cb + leader, c1 = cb + hi;
          sc = (c0 + c1) * cnt / 2;
          auto sq = [](unsigned long long x) { return x * (x + 1) * (2 * x + 1) / 6; };
          scc = sq(c1) - (c0 ? sq(c0 - 1) : 0ull);
        } else {
          sc = hrf::wave_sum<unsigned long long>(m ? (unsigned long long)c : 0ull);
          scc = hrf::wave_sum<unsigned long long>(m ? (unsigned long long)(c * c) : 0ull);
        }
        a0 = cnt;
        a1 = cnt * rr;
        a2 = sc;
        a3 = cnt * rr * rr;
        a4 = scc;
        a5 = rr * sc;
      } else {
        a0 = hrf::wave_sum<unsigned long long>(m ? 1ull : 0ull);
        a1 = hrf::wave_sum<unsigned long long>(m ? (unsigned long long)r : 0ull);
        a2 = hrf::wave_sum<unsigned long long>(m ? (unsigned long long)c : 0ull);
        a3 = hrf::wave_sum<unsigned long long>(m ? (unsigned long long)(r * r) : 0ull);
        a4 = hrf::wave_sum<unsigned long long>(m ? (unsigned long long)(c * c) : 0ull);
        a5 = hrf::wave_sum<unsigned long long>(m ? (unsigned long long)(r * c) : 0ull);
      }
      if (lane == leader) {
        atomicAdd(mom + k + 0, a0);
        atomicAdd(mom + k + 1, a1);
        atomicAdd(mom + k + 2, a2);
        atomicAdd(mom + k + 3, a3);
        atomicAdd(mom + k + 4, a4);
        atomicAdd(mom + k + 5, a5);
      }
      if (m) active = false;
      pending &= ~same;
    }
  }
}

__device__ __forceinline__ double exact_central(int64_t A, int64_t s2, int64_t sa, int64_t sb) {
  // (A*s2 - sa*sb) / A^2 with the numerator exact in 128-bit integers
  const __int128 num = (__int128)A * s2 - (__int128)sa * sb;
  const double A2 = (double)A * (double)A;
  return (double)(int64_t)num / A2;
}

// the inertia eigenvalues of label l from its moments (skimage regionprops' inertia_tensor_eigvals)
__device__ __forceinline__ void label_eigvals(const unsigned long long *__restrict__ mom, int64_t l, int64_t A,
                                              double &ta, double &tb, double &tc, double &l1, double &l2) {
  const int64_t sr = (int64_t)mom[l * 6 + 1], sc = (int64_t)mom[l * 6 + 2];
  const double mu20 = exact_central(A, (int64_t)mom[l * 6 + 3], sr, sr);
  const double mu02 = exact_central(A, (int64_t)mom[l * 6 + 4], sc, sc);
  const double mu11 = exact_central(A, (int64_t)mom[l * 6 + 5], sr, sc);
  ta = mu02;
  tb = -mu11;
  tc = mu20;
  const double root = sqrt(4.0 * tb * tb + (ta - tc) * (ta - tc));
  l1 = (ta + tc) / 2.0 + root / 2.0;
  l2 = (ta + tc) / 2.0 - root / 2.0;
  if (l1 < 0) l1 = 0;
  if (l2 < 0) l2 = 0;
}

__global__ void props_kernel(const unsigned long long *__restrict__ mom, int32_t maxlab, double *__restrict__ props) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l > maxlab) return;
  double *s = props + l * 8;
  const int64_t A = (int64_t)mom[l * 6];
  for (int q = 0; q < 8; ++q) s[q] = 0.0;
  if (l == 0 || A == 0) return;
  const int64_t sr = (int64_t)mom[l * 6 + 1], sc = (int64_t)mom[l * 6 + 2];
  double ta, tb, tc, l1, l2;
  label_eigvals(mom, l, A, ta, tb, tc, l1, l2);
  s[0] = (double)A;
  s[1] = (double)sr / (double)A;
  s[2] = (double)sc / (double)A;
  s[3] = 4.0 * sqrt(l1);
  s[4] = 4.0 * sqrt(l2);
  s[5] = l1 == 0 ? 0.0 : sqrt(1.0 - l2 / l1);
  if (ta - tc == 0)
    s[6] = tb < 0 ? -M_PI / 4.0 : M_PI / 4.0;
  else
    s[6] = -0.5 * atan2(-2.0 * tb, ta - tc);
  s[7] = 1.0;
}

__global__ void barcode_counts_kernel(const int32_t *__restrict__ bc, int64_t n, int32_t R,
                                      unsigned long long *__restrict__ counts, const int32_t *__restrict__ n_dev) {
  if (n_dev) n = min(n, (int64_t)*n_dev);
  const int64_t n_up = (n + 63) / 64 * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_up; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t b = i < n ? bc[i] : -1;
    const bool ok = b >= 0 && b < R;
    hrf::agg_atomic_add<unsigned long long>(counts, ok ? b : 0, 1ull, ok);
  }
}

__global__ void paint_kernel(const int32_t *__restrict__ lab, int64_t n, const int32_t *__restrict__ code,
                             int32_t ncell, int32_t *__restrict__ out, const int32_t *__restrict__ ncell_dev,
                             int32_t add) {
  if (ncell_dev) ncell = min(ncell, *ncell_dev);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lab[i];
    out[i] = (l >= 1 && l <= ncell) ? code[l - 1] + add : 0;
  }
}

// ecoli measurement.py:116-126: keep a cell iff !(minor < lo || minor > hi) and paint only its
// interior after two cross erosions of its own mask (border_value True) == every in-image
// pixel within L1 distance 2 carries the same label.
__global__ void shape_filter_kernel(const int32_t *__restrict__ lab, int64_t H, int64_t W,
                                    const double *__restrict__ props, int32_t maxlab, double lo, double hi,
                                    int32_t *__restrict__ out) {
  const int64_t n = H * W;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lab[p];
    int32_t o = 0;
    bool valid = false;
    double mn = 0.0;
    if (l > 0 && l <= maxlab) {
      valid = props[(int64_t)l * 8 + 7] != 0.0;
      mn = props[(int64_t)l * 8 + 4];
    }
    if (valid) {
      if (!(mn < lo || mn > hi)) {
        const int64_t r = p / W, c = p - r * W;
        bool in = true;
#pragma unroll
        for (int dr = -2; dr <= 2; ++dr)
#pragma unroll
          for (int dc = -2; dc <= 2; ++dc) {
            if ((dr < 0 ? -dr : dr) + (dc < 0 ? -dc : dc) > 2) continue;
            const int64_t rr = r + dr, cc = c + dc;
            if (rr < 0 || rr >= H || cc < 0 || cc >= W) continue;
            in = in && lab[rr * W + cc] == l;
          }
        o = in ? l : 0;
      }
    }
    out[p] = o;
  }
}

}  // namespace

extern "C" {

hrf_status hrf_label_sums(const float *stack, const int32_t *labels, int64_t npix, int32_t C, int32_t maxlab,
                          const float *cal, int32_t cal_c0, int32_t cal_c1, double *sums, int64_t *counts,
                          hrf_stream_t stream) {
  return hrf_label_sums_cal(stack, labels, npix, C, maxlab, cal, 1, 0, cal_c0, cal_c1, sums, counts, stream);
}

hrf_status hrf_label_sums_cal(const float *stack, const int32_t *labels, int64_t npix, int32_t C, int32_t maxlab,
                              const float *cal, int64_t cal_sp, int32_t cal_sc, int32_t cal_c0, int32_t cal_c1,
                              double *sums, int64_t *counts, hrf_stream_t stream) {
  HRF_REQUIRE(cal_sp >= 0 && cal_sc >= 0, "label_sums: bad calibration layout");
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(C >= 1 && C <= 512 && maxlab >= 0 && npix >= 0, "label_sums: C must be 1..512");
  HRF_REQUIRE(sums && counts, "label_sums: null output");
  HRF_HIP(hipMemsetAsync(sums, 0, sizeof(double) * ((size_t)maxlab + 1) * C, s));
  HRF_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * ((size_t)maxlab + 1), s));
  if (npix == 0) return HRF_OK;
  HRF_REQUIRE(stack && labels, "label_sums: null input");
  if (C <= 128) {
    const int64_t nchunks = hrf::cdiv(npix, 64);
    const int mode = cal == nullptr ? 0 : (cal_sc == 0 ? 1 : 2);
    const int64_t nblk = hrf::cdiv(nchunks, 4);
#define HRF_LSW(M)                                                                                                 \
  {                                                                                                                \
    const unsigned grid = hrf::resident_grid(label_sums_wave_kernel<M>, 256, 0, nblk);                             \
    label_sums_wave_kernel<M><<<grid, 256, 0, s>>>(stack, labels, npix, C, maxlab, cal, cal_sp, cal_sc, cal_c0,     \
                                                   cal_c1, sums, (unsigned long long *)counts);                   \
  }
    if (mode == 0) HRF_LSW(0) else if (mode == 1) HRF_LSW(1) else HRF_LSW(2)
#undef HRF_LSW
    HRF_LAUNCHED();
    return HRF_OK;
  }
  const int vec_ok = C >= 4 && ((C * LS_P) % 4 == 0) && (((uintptr_t)stack & 15) == 0);
  const size_t shm = sizeof(float) * LS_P * C;
  const int64_t nchunks = hrf::cdiv(npix, LS_P);
  const unsigned grid = hrf::resident_grid(label_sums_kernel, 256, shm, nchunks);
  label_sums_kernel<<<grid, 256, shm, s>>>(stack, labels, npix, C, maxlab, cal, cal_sp, cal_sc, cal_c0, cal_c1, sums,
                                           (unsigned long long *)counts, vec_ok);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_cell_table(const double *sums, const int64_t *counts, int32_t maxlab, int32_t C, int32_t max_rows,
                          int32_t *row_of_label, int32_t *label_of_row, double *avgint, double *avgint_norm,
                          int32_t *nrows_dev, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && C >= 1 && max_rows >= 0, "cell_table: bad sizes");
  HRF_REQUIRE(sums && counts && row_of_label && label_of_row && avgint && nrows_dev, "cell_table: null buffer");
  cell_rows_kernel<<<1, 1024, 0, s>>>((const unsigned long long *)counts, maxlab, row_of_label, label_of_row,
                                      nrows_dev);
  if (max_rows > 0)
    cell_means_kernel<<<(unsigned)hrf::cdiv((int64_t)max_rows * 64, 256), 256, 0, s>>>(
        sums, (const unsigned long long *)counts, label_of_row, nrows_dev, max_rows, C, avgint, avgint_norm);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_region_moments(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, int64_t *mom,
                              hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && mom, "region_moments: bad arguments");
  HRF_HIP(hipMemsetAsync(mom, 0, sizeof(int64_t) * 6 * ((size_t)maxlab + 1), s));
  return hrf::region_moments_zeroed(labels, H, W, maxlab, mom, s);
}

}  // extern "C"

hrf_status hrf::region_moments_zeroed(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, int64_t *mom,
                                      hipStream_t s) {
  HRF_REQUIRE(maxlab >= 0 && mom, "region_moments: bad arguments");
  if (H * W == 0) return HRF_OK;
  moments_kernel<<<hrf::stream_grid(H * W), 256, 0, s>>>(labels, H, W, maxlab, (unsigned long long *)mom);
  HRF_LAUNCHED();
  return HRF_OK;
}

extern "C" {

hrf_status hrf_region_props(const int64_t *mom, int32_t maxlab, double *props, hrf_stream_t stream) {
  HRF_REQUIRE(maxlab >= 0 && mom && props, "region_props: bad arguments");
  props_kernel<<<(unsigned)hrf::cdiv((int64_t)maxlab + 1, 256), 256, 0, (hipStream_t)stream>>>(
      (const unsigned long long *)mom, maxlab, props);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_shape_filter(const int32_t *labels, int64_t H, int64_t W, const double *props, int32_t maxlab,
                            double minor_lo, double minor_hi, int32_t *out, hrf_stream_t stream) {
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(labels && props && out && labels != out && maxlab >= 0, "shape_filter: bad arguments");
  shape_filter_kernel<<<hrf::stream_grid(H * W), 256, 0, (hipStream_t)stream>>>(labels, H, W, props, maxlab,
                                                                                  minor_lo, minor_hi, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_barcode_counts(const int32_t *bc, int64_t n, int32_t R, int64_t *counts, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(R >= 1 && counts, "barcode_counts: bad arguments");
  HRF_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * R, s));
  if (n == 0) return HRF_OK;
  barcode_counts_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(bc, n, R, (unsigned long long *)counts, nullptr);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_paint_ids(const int32_t *labels, int64_t n, const int32_t *code, int32_t ncell, int32_t *out,
                         hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(labels && out && (code || ncell == 0), "paint_ids: null buffer");
  paint_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(labels, n, code, ncell, out, nullptr, 0);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"

namespace hrf {

// hrf_barcode_counts / hrf_paint_ids with the cell count held on the device (hrf_tile_ecoli):
// n_dev <= nmax rows; paint writes code[l - 1] + add
hrf_status barcode_counts_devn(const int32_t *bc, int64_t nmax, const int32_t *n_dev, int32_t R, int64_t *counts,
                               hipStream_t s, bool zeroed) {
  HRF_REQUIRE(R >= 1 && counts, "barcode_counts: bad arguments");
  if (!zeroed) HRF_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * R, s));
  if (nmax == 0) return HRF_OK;
  barcode_counts_kernel<<<hrf::stream_grid(nmax), 256, 0, s>>>(bc, nmax, R, (unsigned long long *)counts, n_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status paint_ids_devn(const int32_t *labels, int64_t n, const int32_t *code, int32_t nmax, const int32_t *ncell_dev,
                          int32_t add, int32_t *out, hipStream_t s) {
  if (n == 0) return HRF_OK;
  paint_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(labels, n, code, nmax, out, ncell_dev, add);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // namespace hrf
