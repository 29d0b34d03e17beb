// enhance.hip -- oriented line-profile stencils (a5-a7).
//
// Replaces the Cython passes neighbor2d.line_profile_2d_v2 (neighbor2d.pyx:8-64),
// neighbor.line_profile_v2 (neighbor.pyx:115-181) and
// neighbor.line_profile_memory_efficient_v2 (neighbor.pyx:186-263), plus the numpy
// post-chains that consume them (multispecies_spectral_image_measurement.py:111-124,
// biofilm_analysis.py:812-817).
//
// Fused kernels stage an f64 tile (+10 halo) in LDS and read the 9x11 (2-D) or 72x11 (3-D)
// taps with compile-time offsets (lp_tables.inc), so every tap is one ds_read_b64 with an
// immediate offset.  Lanes run along the fastest image axis: conflict-free LDS reads and
// coalesced global traffic.  All arithmetic is f64 in the reference's order (numpy's
// 8-accumulator pairwise mean, numpy percentile lerp), compiled with -ffp-contract=off, so
// results are bit-identical to the reference chain.
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "common.hpp"
#include "lp_tables.inc"

namespace {

constexpr double DMAX = 1.7976931348623157e308;

__device__ __forceinline__ double nan_to_num(double v) {
  if (v != v) return 0.0;
  if (v > DMAX) return DMAX;
  if (v < -DMAX) return -DMAX;
  return v;
}

// ------------------------------------------------------------------------------------
// 2-D fused: patch 11, 9 directions.  Tile 16 rows x 64 cols of output, 4 pixels/thread.
// ------------------------------------------------------------------------------------
constexpr int E2_TW = 64, E2_TH = 16, E2_LW = E2_TW + 10, E2_LH = E2_TH + 10;

__global__ __launch_bounds__(256) void enhance2d_kernel(const double *__restrict__ pad, int64_t hp, int64_t wp,
                                                        int64_t ld, double *__restrict__ out, int64_t H, int64_t W) {
  __shared__ double tile[E2_LH * E2_LW];
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.y * E2_TH, j0 = (int64_t)blockIdx.x * E2_TW;
  for (int idx = tid; idx < E2_LH * E2_LW; idx += 256) {
    const int r = idx / E2_LW, c = idx - r * E2_LW;
    const int64_t gi = i0 + r, gj = j0 + c;
    // np.nan_to_num is applied to every tap; applying it once per staged value is equal.
    tile[idx] = (gi < hp && gj < wp) ? nan_to_num(pad[gi * ld + gj]) : 0.0;
  }
  __syncthreads();
  const int jj = tid & 63, rg = tid >> 6;
#pragma unroll 1
  for (int k = 0; k < 4; ++k) {
    const int ii = rg + 4 * k;
    const int64_t i = i0 + ii, j = j0 + jj;
    if (i >= H || j >= W) continue;
    const double *b = tile + ii * E2_LW + jj;
    double v[9];
    bool anynan = false;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      double mn = b[LP2D_11_9[t][0][0] * E2_LW + LP2D_11_9[t][0][1]], mx = mn, c = 0.0;
#pragma unroll
      for (int l = 0; l < 11; ++l) {
        const double x = b[LP2D_11_9[t][l][0] * E2_LW + LP2D_11_9[t][l][1]];
        mn = x < mn ? x : mn;
        mx = x > mx ? x : mx;
        if (l == 5) c = x;
      }
      v[t] = (c - mn) / (mx - mn);
      anynan |= (v[t] != v[t]);
    }
    double res = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    res += v[8];
    const double avg = res / 9.0;
    double o;
    if (anynan) {
      o = __builtin_nan("");
    } else {
#pragma unroll
      for (int q = 0; q < SEL9_N; ++q) {
        const double a = v[SEL9[q][0]], bb = v[SEL9[q][1]];
        v[SEL9[q][0]] = a < bb ? a : bb;
        v[SEL9[q][1]] = a < bb ? bb : a;
      }
      // np.percentile over 9 values: positions 2.0 and 6.0 (t = 0)
      const double lq = v[2] + (v[3] - v[2]) * 0.0;
      const double uq = v[6] + (v[7] - v[6]) * 0.0;
      double qcv = 0.0;
      if (uq > 0) qcv = (uq - lq) / (uq + lq + 1e-8);
      o = avg * (1.0 - qcv);
    }
    out[i * W + j] = o;
  }
}

// ------------------------------------------------------------------------------------
// 3-D fused: patch 11, 72 directions.  Tile 4 x 4 x 32 outputs (z fastest), 2 voxels per
// thread; 14 x 14 x 42 f64 LDS tile (65,856 B, 2 workgroups per CU).
// MODE 0: final (X,Y,Z); MODE 1: per-direction normalised centre (X,Y,Z,72).
// ------------------------------------------------------------------------------------
constexpr int E3_TX = 4, E3_TY = 4, E3_TZ = 32;
constexpr int E3_LX = E3_TX + 10, E3_LY = E3_TY + 10, E3_LZ = E3_TZ + 10;

// One output voxel (b: its centre in the LDS tile).  FAST: the tile holds no NaN, no infinity, no
// negative zero and no magnitude above 2^1023 (so no window's range overflows and every normalised
// tap is a number in [0, 1]), so every `a < b ? a : b` of the reference's min/max and of the
// selection network picks the same value as v_min_f64 / v_max_f64 -- one instruction instead of a
// compare, two 64-bit selects and their hazard nops (values equal => same bits, no signed zeros).
#ifndef E3_GROUP_N
#define E3_GROUP_N 4
#endif
constexpr int E3_GROUP = E3_GROUP_N;

template <int MODE, bool FAST>
__device__ __forceinline__ void enhance3d_voxel(const double *__restrict__ b, int64_t vox,
                                                double *__restrict__ out) {
  double v[72];
#pragma unroll
  for (int t = 0; t < 72; ++t) {
    double mn = 0.0, mx = 0.0, c = 0.0;
#pragma unroll
    for (int l = 0; l < 11; ++l) {
      const double q = b[(LP3D_11_9_9[t][l][0] * E3_LY + LP3D_11_9_9[t][l][1]) * E3_LZ + LP3D_11_9_9[t][l][2]];
      if (l == 0) {
        mn = q;
        mx = q;
      } else if (FAST) {
        mn = __builtin_fmin(q, mn);
        mx = __builtin_fmax(q, mx);
      } else {
        mn = q < mn ? q : mn;
        mx = q > mx ? q : mx;
      }
      if (l == 5) c = q;
    }
    double r = mx - mn;
    if (1e-8 > r) r = 1e-8;  // builtin max(range, 1e-8) (neighbor.pyx:259)
    v[t] = (c - mn) / r;
    // at most E3_GROUP directions' taps in flight: the 72 results stay within the register
    // budget of two waves per SIMD instead of the scheduler hoisting hundreds of LDS reads
    if (t % E3_GROUP == E3_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
  }
  if (MODE == 1) {
#pragma unroll
    for (int t = 0; t < 72; ++t) out[vox * 72 + t] = v[t];
    return;
  }
  // numpy pairwise mean over 72 (8 accumulators seeded with the first 8)
  double acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = v[q];
#pragma unroll
  for (int i = 8; i < 72; i += 8)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += v[i + q];
  const double avg = (((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]))) / 72.0;
#pragma unroll
  for (int q = 0; q < SEL72_N; ++q) {
    const double a = v[SEL72[q][0]], bb = v[SEL72[q][1]];
    if (FAST) {
      v[SEL72[q][0]] = __builtin_fmin(a, bb);
      v[SEL72[q][1]] = __builtin_fmax(a, bb);
    } else {
      v[SEL72[q][0]] = a < bb ? a : bb;
      v[SEL72[q][1]] = a < bb ? bb : a;
    }
  }
  // np.percentile(.., 25/75) over 72: positions 17.75 (t >= .5 form) and 53.25
  const double lq = v[18] - (v[18] - v[17]) * 0.25;
  const double uq = v[53] + (v[54] - v[53]) * 0.25;
  const double qcv = nan_to_num((uq - lq) / (uq + lq));
  out[vox] = avg * (1.0 - qcv);
}

template <int MODE, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void enhance3d_kernel(const double *__restrict__ pad, int64_t xp, int64_t yp,
                                                        int64_t zp, double *__restrict__ out, int64_t X, int64_t Y,
                                                        int64_t Z) {
  __shared__ double tile[E3_LX * E3_LY * E3_LZ];
  const int tid = threadIdx.x;
  const int64_t x0 = (int64_t)blockIdx.z * E3_TX, y0 = (int64_t)blockIdx.y * E3_TY, z0 = (int64_t)blockIdx.x * E3_TZ;
  // a NaN, an infinity, a negative zero -- or a magnitude of 2^1023 or more, where a window's
  // max - min could overflow to inf (2^1023 - (-2^1023) = 2^1024 already does) and (c - mn) / r give
  // inf / inf = NaN, on which fmin / fmax and the reference's `a < b ? a : b` disagree -- sends the
  // tile down the reference's compare-select path
  int special = 0;
  for (int idx = tid; idx < E3_LX * E3_LY * E3_LZ; idx += 256) {
    const int lx = idx / (E3_LY * E3_LZ);
    const int rem = idx - lx * (E3_LY * E3_LZ);
    const int ly = rem / E3_LZ, lz = rem - ly * E3_LZ;
    const int64_t gx = x0 + lx, gy = y0 + ly, gz = z0 + lz;
    const double v = (gx < xp && gy < yp && gz < zp) ? pad[(gx * yp + gy) * zp + gz] : 0.0;
    special |= !(__builtin_fabs(v) < 0x1p1023) || (v == 0.0 && __builtin_signbit(v));
    tile[idx] = v;
  }
  const bool fast = !__syncthreads_or(special);
  const int tz = tid & 31, ty = (tid >> 5) & 3, th = tid >> 7;
#pragma unroll 1
  for (int k = 0; k < 2; ++k) {
    const int tx = th + 2 * k;
    const int64_t x = x0 + tx, y = y0 + ty, z = z0 + tz;
    if (x >= X || y >= Y || z >= Z) continue;
    const double *b = tile + (tx * E3_LY + ty) * E3_LZ + tz;
    const int64_t vox = (x * Y + y) * Z + z;
    if (fast) enhance3d_voxel<MODE, true>(b, vox, out);
    else enhance3d_voxel<MODE, false>(b, vox, out);
  }
}

// ------------------------------------------------------------------------------------
// neighbor.line_profile_memory_efficient_v3 (neighbor.pyx:268-349): its own sampling table
// (LP3D_V3: reaches up to 18 voxels along x and z, past the patch), read the way the
// reference's unchecked memoryview reads it -- flat address (i+a)*yp*zp + (j+b)*zp + (k+c)
// into the padded array, 0 past its end (undefined in the reference) -- the 72 normalised
// centre taps, their mean in loop order, p25 / p75 and mean*(p25-p75)/(p25+p75+1e-8).
// One thread per voxel straight from global memory (L2-resident windows): the reference
// imports this function but never calls it.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enhance3d_v3_kernel(const double *__restrict__ pad, int64_t xp, int64_t yp,
                                                           int64_t zp, double *__restrict__ out, int64_t X, int64_t Y,
                                                           int64_t Z) {
  const int64_t total = xp * yp * zp, n = X * Y * Z;
  for (int64_t vox = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; vox < n; vox += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = vox / (Y * Z), rem = vox - i * (Y * Z), j = rem / Z, k = rem - j * Z;
    double v[72];
    double avg = 0.0;
#pragma unroll
    for (int t = 0; t < 72; ++t) {
      double mn = 0.0, mx = 0.0, c = 0.0;
#pragma unroll
      for (int l = 0; l < 11; ++l) {
        const int64_t a = (i + LP3D_V3_11_9_9[t][l][0]) * yp * zp + (j + LP3D_V3_11_9_9[t][l][1]) * zp +
                          (k + LP3D_V3_11_9_9[t][l][2]);
        const double q = a < total ? pad[a] : 0.0;
        if (l == 0) {
          mn = q;
          mx = q;
        } else {
          mn = q < mn ? q : mn;
          mx = q > mx ? q : mx;
        }
        if (l == 5) c = q;
      }
      double r = mx - mn;
      if (1e-8 > r) r = 1e-8;
      v[t] = (c - mn) / r;
      avg += v[t];  // :341-343, in loop order
    }
    avg /= 72.0;
#pragma unroll
    for (int q = 0; q < SEL72_N; ++q) {
      const double a = v[SEL72[q][0]], bb = v[SEL72[q][1]];
      v[SEL72[q][0]] = a < bb ? a : bb;
      v[SEL72[q][1]] = a < bb ? bb : a;
    }
    const double p25 = v[18] - (v[18] - v[17]) * 0.25;
    const double p75 = v[53] + (v[54] - v[53]) * 0.25;
    out[vox] = avg * (p25 - p75) / (p25 + p75 + 1e-8);
  }
}

// ------------------------------------------------------------------------------------
// Unfused gathers for the drop-in API (outputs the full profile arrays).
// ------------------------------------------------------------------------------------
__global__ void lp2d_gather_kernel(const double *__restrict__ pad, int64_t ld, const int32_t *__restrict__ tab,
                                   int patch, int nphi, double *__restrict__ out, int64_t H, int64_t W) {
  const int64_t n = H * W * nphi * patch;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tl = e % ((int64_t)nphi * patch);
    const int64_t pix = e / ((int64_t)nphi * patch);
    const int64_t i = pix / W, j = pix - i * W;
    out[e] = pad[(i + tab[2 * tl]) * ld + (j + tab[2 * tl + 1])];
  }
}

__global__ void lp3d_gather_kernel(const double *__restrict__ pad, int64_t yp, int64_t zp,
                                   const int32_t *__restrict__ tab, int patch, int ndir, double *__restrict__ out,
                                   int64_t X, int64_t Y, int64_t Z) {
  const int64_t per = (int64_t)ndir * patch;
  const int64_t n = X * Y * Z * per;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tl = e % per;
    const int64_t vox = e / per;
    const int64_t z = vox % Z, y = (vox / Z) % Y, x = vox / (Y * Z);
    out[e] = pad[((x + tab[3 * tl]) * yp + (y + tab[3 * tl + 1])) * zp + (z + tab[3 * tl + 2])];
  }
}

__global__ void lp3d_norm_generic_kernel(const double *__restrict__ pad, int64_t yp, int64_t zp,
                                         const int32_t *__restrict__ tab, int patch, int ndir,
                                         double *__restrict__ out, int64_t X, int64_t Y, int64_t Z) {
  const int64_t n = X * Y * Z * ndir;
  const int inc = (patch - 1) / 2;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e % ndir, vox = e / ndir;
    const int64_t z = vox % Z, y = (vox / Z) % Y, x = vox / (Y * Z);
    double mn = 0, mx = 0, c = 0;
    for (int l = 0; l < patch; ++l) {
      const int32_t *o = tab + (t * patch + l) * 3;
      const double q = pad[((x + o[0]) * yp + (y + o[1])) * zp + (z + o[2])];
      if (l == 0 || q < mn) mn = q;
      if (l == 0 || q > mx) mx = q;
      if (l == inc) c = q;
    }
    double r = mx - mn;
    if (1e-8 > r) r = 1e-8;
    out[e] = (c - mn) / r;
  }
}

// Device copies of runtime tables, uploaded once per parameter set.
std::mutex g_tab_mu;
std::map<std::tuple<int, int, int, int, int>, int32_t *> g_tabs;

hrf_status device_table(int dims, int patch, int ntheta, int nphi, int32_t **out) {
  int dev = 0;
  HRF_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_tab_mu);
  auto key = std::make_tuple(dev, dims, patch, ntheta, nphi);
  auto it = g_tabs.find(key);
  if (it != g_tabs.end()) {
    *out = it->second;
    return HRF_OK;
  }
  const int ndir = dims == 2 ? nphi : (ntheta - 1) * nphi;
  std::vector<int32_t> h((size_t)ndir * patch * dims);
  if (dims == 2)
    hrf::lp_table_2d(patch, nphi, h.data());
  else
    hrf::lp_table_3d(patch, ntheta, nphi, h.data());
  int32_t *d = nullptr;
  HRF_HIP(hipMalloc(&d, h.size() * sizeof(int32_t)));
  HRF_HIP(hipMemcpy(d, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  g_tabs[key] = d;
  *out = d;
  return HRF_OK;
}

}  // namespace

extern "C" {

hrf_status hrf_line_profile_2d(const double *pad, int64_t hp, int64_t wp, int64_t ld, int32_t patch, int32_t nphi,
                               double *out, hrf_stream_t stream) {
  HRF_REQUIRE(patch >= 1 && patch <= 64 && nphi >= 1 && nphi <= 64, "line_profile_2d: patch/phi out of range");
  HRF_REQUIRE(hp >= patch - 1 && wp >= patch - 1 && ld >= wp, "line_profile_2d: padded image smaller than patch");
  const int64_t H = hp - (patch - 1), W = wp - (patch - 1);
  if (H == 0 || W == 0) return HRF_OK;
  HRF_REQUIRE(pad && out, "line_profile_2d: null buffer");
  int32_t *tab = nullptr;
  hrf_status s = device_table(2, patch, 0, nphi, &tab);
  if (s) return s;
  const int64_t n = H * W * nphi * patch;
  lp2d_gather_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(pad, ld, tab, patch, nphi, out, H, W);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_enhance_2d(const double *pad, int64_t hp, int64_t wp, int64_t ld, int32_t patch, int32_t nphi,
                          double *final_, hrf_stream_t stream) {
  HRF_REQUIRE(patch == 11 && nphi == 9, "enhance_2d: only the reference parameters (patch 11, phi 9) are fused");
  HRF_REQUIRE(hp >= 10 && wp >= 10 && ld >= wp, "enhance_2d: padded image smaller than patch");
  const int64_t H = hp - 10, W = wp - 10;
  if (H == 0 || W == 0) return HRF_OK;
  HRF_REQUIRE(pad && final_, "enhance_2d: null buffer");
  dim3 grid((unsigned)hrf::cdiv(W, E2_TW), (unsigned)hrf::cdiv(H, E2_TH));
  HRF_REQUIRE(grid.y <= 65535, "enhance_2d: image too tall");
  enhance2d_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(pad, hp, wp, ld, final_, H, W);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_line_profile_3d(const double *pad, int64_t xp, int64_t yp, int64_t zp, int32_t patch, int32_t ntheta,
                               int32_t nphi, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(patch >= 1 && patch <= 64 && ntheta >= 2 && nphi >= 1 && (ntheta - 1) * nphi <= 512,
              "line_profile_3d: parameters out of range");
  HRF_REQUIRE(xp >= patch - 1 && yp >= patch - 1 && zp >= patch - 1, "line_profile_3d: padded volume smaller than patch");
  const int64_t X = xp - (patch - 1), Y = yp - (patch - 1), Z = zp - (patch - 1);
  if (X == 0 || Y == 0 || Z == 0) return HRF_OK;
  HRF_REQUIRE(pad && out, "line_profile_3d: null buffer");
  int32_t *tab = nullptr;
  hrf_status s = device_table(3, patch, ntheta, nphi, &tab);
  if (s) return s;
  const int ndir = (ntheta - 1) * nphi;
  const int64_t n = X * Y * Z * ndir * patch;
  lp3d_gather_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(pad, yp, zp, tab, patch, ndir, out, X, Y,
                                                                            Z);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_line_profile_3d_norm(const double *pad, int64_t xp, int64_t yp, int64_t zp, int32_t patch,
                                    int32_t ntheta, int32_t nphi, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(patch >= 1 && patch <= 64 && ntheta >= 2 && nphi >= 1 && (ntheta - 1) * nphi <= 512,
              "line_profile_3d_norm: parameters out of range");
  HRF_REQUIRE(xp >= patch - 1 && yp >= patch - 1 && zp >= patch - 1,
              "line_profile_3d_norm: padded volume smaller than patch");
  const int64_t X = xp - (patch - 1), Y = yp - (patch - 1), Z = zp - (patch - 1);
  if (X == 0 || Y == 0 || Z == 0) return HRF_OK;
  HRF_REQUIRE(pad && out, "line_profile_3d_norm: null buffer");
  if (patch == 11 && ntheta == 9 && nphi == 9) {
    dim3 grid((unsigned)hrf::cdiv(Z, E3_TZ), (unsigned)hrf::cdiv(Y, E3_TY), (unsigned)hrf::cdiv(X, E3_TX));
    HRF_REQUIRE(grid.y <= 65535 && grid.z <= 65535, "line_profile_3d_norm: volume too large");
    enhance3d_kernel<1><<<grid, 256, 0, (hipStream_t)stream>>>(pad, xp, yp, zp, out, X, Y, Z);
    HRF_LAUNCHED();
    return HRF_OK;
  }
  int32_t *tab = nullptr;
  hrf_status s = device_table(3, patch, ntheta, nphi, &tab);
  if (s) return s;
  const int ndir = (ntheta - 1) * nphi;
  lp3d_norm_generic_kernel<<<hrf::stream_grid(X * Y * Z * ndir), 256, 0, (hipStream_t)stream>>>(
      pad, yp, zp, tab, patch, ndir, out, X, Y, Z);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_enhance_3d(const double *pad, int64_t xp, int64_t yp, int64_t zp, int32_t patch, int32_t ntheta,
                          int32_t nphi, double *final_, hrf_stream_t stream) {
  HRF_REQUIRE(patch == 11 && ntheta == 9 && nphi == 9,
              "enhance_3d: only the reference parameters (patch 11, theta 9, phi 9) are fused");
  HRF_REQUIRE(xp >= 10 && yp >= 10 && zp >= 10, "enhance_3d: padded volume smaller than patch");
  const int64_t X = xp - 10, Y = yp - 10, Z = zp - 10;
  if (X == 0 || Y == 0 || Z == 0) return HRF_OK;
  HRF_REQUIRE(pad && final_, "enhance_3d: null buffer");
  dim3 grid((unsigned)hrf::cdiv(Z, E3_TZ), (unsigned)hrf::cdiv(Y, E3_TY), (unsigned)hrf::cdiv(X, E3_TX));
  HRF_REQUIRE(grid.y <= 65535 && grid.z <= 65535, "enhance_3d: volume too large");
  // built for two waves per SIMD (106 VGPRs of spills) rather than one: 12.2 vs 17.0 ms on the
  // 1024x1024x64 volume (round 4)
  enhance3d_kernel<0, 2><<<grid, 256, 0, (hipStream_t)stream>>>(pad, xp, yp, zp, final_, X, Y, Z);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_enhance_3d_v3(const double *pad, int64_t xp, int64_t yp, int64_t zp, int32_t patch, int32_t ntheta,
                             int32_t nphi, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(patch == 11 && ntheta == 9 && nphi == 9,
              "line_profile_memory_efficient_v3: only the reference parameters (11, 9, 9) are built");
  HRF_REQUIRE(xp >= 10 && yp >= 10 && zp >= 10, "line_profile_memory_efficient_v3: padded volume smaller than patch");
  const int64_t X = xp - 10, Y = yp - 10, Z = zp - 10;
  if (X == 0 || Y == 0 || Z == 0) return HRF_OK;
  HRF_REQUIRE(pad && out, "line_profile_memory_efficient_v3: null buffer");
  enhance3d_v3_kernel<<<hrf::stream_grid(X * Y * Z), 256, 0, (hipStream_t)stream>>>(pad, xp, yp, zp, out, X, Y, Z);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
