#include <cstdlib>
// stack.hip -- spectral stack assembly and per-pixel channel reductions (a1-a3), plus the
// small elementwise steps between pipeline stages.
//
// a1/a2 hrf_register_assemble: per-laser (H, W, C_l) stacks -> one (H, W, C) stack with each
//   laser shifted by its integer registration vector and zero outside its coverage
//   (ecoli measurement.py:51-70, multispecies :88-102), optionally multiplied by the
//   intersection of all coverage masks (ecoli :69-70).  One pass, lanes along channels.
// a3 hrf_channel_sum: per-pixel sum over C in numpy's pairwise order (8 accumulators,
//   blocks of 128) so the f64 result equals np.sum(stack, axis=2) bit for bit, then
//   log(s + 1e-2) (ecoli :72) / log10(s + 1) (biofilm :831) / identity, optionally negated
//   (watershed input).
#include <algorithm>

#include "common.hpp"
#include "pixtable.hpp"
#include "wave.hpp"
#include "detmath.h"

namespace {

constexpr int LMAX = 8;
struct Lasers {
  const float *src[LMAX];
  int32_t c0[LMAX + 1];  // channel offsets, c0[n] = C
  int32_t dr[LMAX], dc[LMAX];
  int32_t n;
  const int32_t *dsh;  // non-null: the shifts are read from the device (dr, dc pairs)
};

// the shifts in force: from the device buffer when given (no host round trip), else the
// kernel-argument copies
__device__ __forceinline__ void load_shifts(const Lasers &L, int *sdr, int *sdc) {
  if (threadIdx.x < LMAX) {
    const int q = threadIdx.x;
    sdr[q] = q < L.n ? (L.dsh ? L.dsh[2 * q] : L.dr[q]) : 0;
    sdc[q] = q < L.n ? (L.dsh ? L.dsh[2 * q + 1] : L.dc[q]) : 0;
  }
  __syncthreads();
}

__device__ __forceinline__ bool covered(int64_t r, int64_t c, int64_t H, int64_t W, int dr, int dc) {
  // destination rows [max(0,dr), H + min(0,dr)), same for columns
  return r >= (dr > 0 ? dr : 0) && r < H + (dr < 0 ? dr : 0) && c >= (dc > 0 ? dc : 0) && c < W + (dc < 0 ? dc : 0);
}

__global__ void assemble_kernel(Lasers L, int64_t H, int64_t W, int apply_mask, float *__restrict__ dst) {
  __shared__ int sdr[LMAX], sdc[LMAX];
  load_shifts(L, sdr, sdc);
  const int C = L.c0[L.n];
  const int64_t n = H * W * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = e / C;
    const int ch = (int)(e - p * C);
    const int64_t r = p / W, c = p - r * W;
    int li = 0;
#pragma unroll
    for (int q = 1; q < LMAX; ++q)
      if (q < L.n && ch >= L.c0[q]) li = q;
    bool ok = true;
    if (apply_mask) {
#pragma unroll
      for (int q = 0; q < LMAX; ++q)
        if (q < L.n) ok = ok && covered(r, c, H, W, sdr[q], sdc[q]);
    }
    float v = 0.0f;
    if (ok && covered(r, c, H, W, sdr[li], sdc[li])) {
      const int cl = L.c0[li + 1] - L.c0[li];
      v = L.src[li][((r - sdr[li]) * W + (c - sdc[li])) * cl + (ch - L.c0[li])];
    }
    dst[e] = v;
  }
}

// LDS-staged form for C <= 128: one workgroup = 64 consecutive pixels of one row.  Each laser's
// 64 x C_l source block is one contiguous run (a shift moves whole rows and columns), read
// coalesced and scattered into the pixel-major LDS tile at its channel offset; the tile is
// then written out as one contiguous 64 x C run with 16-byte stores.  32-bit index math only.
constexpr int AS_P = 64;
__global__ __launch_bounds__(256) void assemble_lds_kernel(Lasers L, int64_t H, int64_t W, int apply_mask,
                                                           float *__restrict__ dst, int vec_ok,
                                                           double *__restrict__ cn_out, int cn_mode) {
  extern __shared__ __attribute__((aligned(16))) float tile[];
  __shared__ uint8_t okp[AS_P];
  __shared__ int sdr[LMAX], sdc[LMAX];
  load_shifts(L, sdr, sdc);
  const int C = L.c0[L.n];
  const int tid = threadIdx.x;
  const int64_t r = blockIdx.y;
  const int64_t c0 = (int64_t)blockIdx.x * AS_P;
  const int np = (int)min((int64_t)AS_P, W - c0);
  if (tid < AS_P) {
    bool ok = tid < np;
    if (apply_mask)
      for (int q = 0; q < L.n; ++q) ok = ok && covered(r, c0 + tid, H, W, sdr[q], sdc[q]);
    okp[tid] = (uint8_t)ok;
  }
  for (int q = 0; q < L.n; ++q) {
    const int cl = L.c0[q + 1] - L.c0[q], off = L.c0[q];
    const int dr = sdr[q], dc = sdc[q];
    const int64_t rs = r - dr;
    const bool row_ok = r >= (dr > 0 ? dr : 0) && r < H + (dr < 0 ? dr : 0);
    const float *src = L.src[q] + (rs * W + (c0 - dc)) * (int64_t)cl;  // pixel c0's source (may be off-row)
    const int cmin = dc > 0 ? dc : 0, cmax = (int)W + (dc < 0 ? dc : 0);
    const int n = np * cl;
    // four loads in flight per thread per round (the run is at most 64 x 128 floats)
    for (int i0 = tid; i0 < n; i0 += 1024) {
      float v[4];
      int pp[4], cc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 256 * u;
        pp[u] = i / cl;
        cc[u] = i - pp[u] * cl;
        const int64_t c = c0 + pp[u];
        const bool cov = i < n && row_ok && c >= cmin && c < cmax;
        v[u] = cov ? src[i] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + 256 * u < n) tile[pp[u] * C + off + cc[u]] = v[u];
    }
  }
  __syncthreads();
  float *out = dst + (r * W + c0) * (int64_t)C;
  const int n = np * C;
  if (vec_ok) {
    for (int v = tid; v < (n >> 2); v += 256) {
      const int e = v << 2;
      float4 x = reinterpret_cast<const float4 *>(tile)[v];
      if (apply_mask) {
        x.x = okp[e / C] ? x.x : 0.0f;
        x.y = okp[(e + 1) / C] ? x.y : 0.0f;
        x.z = okp[(e + 2) / C] ? x.z : 0.0f;
        x.w = okp[(e + 3) / C] ? x.w : 0.0f;
      }
      reinterpret_cast<float4 *>(out)[v] = x;
    }
    for (int e = ((n >> 2) << 2) + tid; e < n; e += 256) out[e] = (!apply_mask || okp[e / C]) ? tile[e] : 0.0f;
  } else {
    for (int e = tid; e < n; e += 256) out[e] = (!apply_mask || okp[e / C]) ? tile[e] : 0.0f;
  }
  if (cn_out) {
    // the channel sum of the assembled (masked) pixels, numpy's pairwise order as
    // channel_sum_lds_kernel takes it (8 lanes per pixel), from the tile already in LDS:
    // ecoli :71-72 image_cn without a second pass over the stack
    const int j = tid & 7;
    const int main_n = C < 8 ? 0 : C - (C % 8);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int pi = half * 32 + (tid >> 3);
      const float *a = tile + (pi < np ? pi : 0) * C;
      const bool ok = pi < np && (!apply_mask || okp[pi]);
      double res = 0.0;
      if (C >= 8) {
        double rr = ok ? (double)a[j] : 0.0;
        for (int i = 8; i < main_n; i += 8) rr += ok ? (double)a[i + j] : 0.0;
        rr = rr + __shfl_xor(rr, 1, 64);
        rr = rr + __shfl_xor(rr, 2, 64);
        rr = rr + __shfl_xor(rr, 4, 64);
        res = rr;
        if (j == 0)
          for (int i = main_n; i < C; ++i) res += ok ? (double)a[i] : 0.0;
      } else if (j == 0) {
        for (int i = 0; i < C; ++i) res += ok ? (double)a[i] : 0.0;
      }
      if (j == 0 && pi < np) {
        double sv = 0.0 + res;
        if (cn_mode == 1) sv = hrf_cr_log(sv + 1e-2);
        else if (cn_mode == 2) sv = hrf_cr_log10(sv + 1.0);
        cn_out[r * W + c0 + pi] = sv;
      }
    }
  }
}

// E. coli layout (lasers of 32, 23, 20, 14, 6 channels) specialised: every laser's source run
// of the strip is loaded with all reads in flight (25 per thread, divisions by compile-time
// channel counts), then scattered into the tile; the rest as assemble_lds_kernel.
template <int Q>
struct EcoliLasers {
  static constexpr int n = 5;
  static constexpr int cl(int q) { return q == 0 ? 32 : q == 1 ? 23 : q == 2 ? 20 : q == 3 ? 14 : 6; }
  static constexpr int off(int q) { return q == 0 ? 0 : off(q - 1) + cl(q - 1); }
  static constexpr int C = 95;
};

template <int q, int NL>
__device__ __forceinline__ void lay_load(const Lasers &L, const int *sdr, const int *sdc, int64_t r, int64_t c0,
                                         int64_t H, int64_t W, int tid, float *v) {
  constexpr int cl = EcoliLasers<0>::cl(q);
  constexpr int U = (AS_P * cl + 255) / 256;
  const int dr = sdr[q], dc = sdc[q];
  const bool row_ok = r >= (dr > 0 ? dr : 0) && r < H + (dr < 0 ? dr : 0);
  const int64_t cmin = dc > 0 ? dc : 0, cmax = W + (dc < 0 ? dc : 0);
  const float *src = L.src[q] + ((r - dr) * W + (c0 - dc)) * (int64_t)cl;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + 256 * u;
    const int pp = e / cl;
    const int64_t c = c0 + pp;
    v[u] = (e < AS_P * cl && row_ok && c >= cmin && c < cmax && c < W) ? src[e] : 0.0f;
  }
  if constexpr (q + 1 < NL) lay_load<q + 1, NL>(L, sdr, sdc, r, c0, H, W, tid, v + U);
}

// The same loads through buffer descriptors (round 5): an element outside the laser's coverage
// gets an out-of-range offset and reads 0 (the descriptor's range check), so the 25 loads issue
// back to back with no exec-mask branches around them.  Offsets are 32-bit: each laser buffer
// holds < 2 GiB (checked by the launch).  rbase[q] = ((r - dr) * W + c0 - dc) * cl, cok[q] packs
// the strip's valid column range for laser q (wave-uniform, computed once per strip).
template <int q, int NL>
__device__ __forceinline__ void lay_load_buf(const __amdgpu_buffer_rsrc_t *rs, const int *rbase, const int *clo,
                                             const int *chi, int tid, float *v) {
  constexpr int cl = EcoliLasers<0>::cl(q);
  constexpr int U = (AS_P * cl + 255) / 256;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + 256 * u;
    const int pp = e / cl;
    const bool ok = e < AS_P * cl && pp >= clo[q] && pp < chi[q];
    const int off = ok ? (rbase[q] + e) * 4 : -1;
    v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs[q], off, 0, 0));
  }
  if constexpr (q + 1 < NL) lay_load_buf<q + 1, NL>(rs, rbase, clo, chi, tid, v + U);
}

template <int q, int NL>
__device__ __forceinline__ void lay_store(float *tile, int tid, const float *v) {
  constexpr int cl = EcoliLasers<0>::cl(q), off = EcoliLasers<0>::off(q);
  constexpr int U = (AS_P * cl + 255) / 256;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + 256 * u;
    if (e < AS_P * cl) {
      const int pp = e / cl;
      tile[pp * EcoliLasers<0>::C + off + (e - pp * cl)] = v[u];
    }
  }
  if constexpr (q + 1 < NL) lay_store<q + 1, NL>(tile, tid, v + U);
}

// Strips t = blockIdx.x, + gridDim.x, ... (row t / nsx, columns (t % nsx) * 64 ..): launched on a
// resident grid (round 3), a 2048^2 tile is ~1.5 k workgroup dispatches instead of 65 k -- under
// the concurrent classifier every dispatch waits for a CU slot.  Per strip: loads -> barrier ->
// channel sums and segment norms (the tile only read) -> barrier -> flags, image_cn's log and the
// table entries -> barrier.
// (Round 3 also built a prefetching form -- the next strip's loads in flight through this strip's
// image_cn and pixel-table phases -- equal end to end; removed in round 5.)
// Built for four workgroups per CU (128 VGPRs); the lasers are loaded in two rounds (lasers 0-1,
// then 2-4) so fewer values are live at once.
template <bool BUF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void assemble_ecoli_kernel(Lasers L, int64_t H, int64_t W, int apply_mask,
                                                             float *__restrict__ dst, double *__restrict__ cn_out,
                                                             int cn_mode, uint4 *__restrict__ ptab,
                                                             uint8_t *__restrict__ pflags) {
  constexpr int C = EcoliLasers<0>::C;
  __shared__ __attribute__((aligned(16))) float tile[AS_P * C];
  __shared__ uint8_t okp[AS_P];
  __shared__ int sdr[LMAX], sdc[LMAX];
  __shared__ uint32_t fl[AS_P];
  __shared__ double cns[AS_P];  // the strip's channel sums (pixel-table mode: logged in the table phase)
  __shared__ float invs[5 * AS_P];  // reciprocal segment norms (hrf_pix::ecoli_norms)
  load_shifts(L, sdr, sdc);
  const int tid = threadIdx.x;
  constexpr int UT = 8 + 6;  // the larger load round (lasers 0-1)
  float v[UT];
  // strips t = blockIdx.x, + gridDim.x, ...: (row, column strip) stepped incrementally in 32 bits
  // (H * W < 2^31), no per-strip 64-bit division
  const int nsx = (int)((W + AS_P - 1) / AS_P), Hi = (int)H, Wi = (int)W;
  const int gstep_r = (int)(gridDim.x / nsx), gstep_c = (int)(gridDim.x % nsx);
  int ri = (int)(blockIdx.x / nsx), csi = (int)(blockIdx.x % nsx);
  for (; ri < Hi; ri += gstep_r + (csi + gstep_c >= nsx), csi = csi + gstep_c >= nsx ? csi + gstep_c - nsx : csi + gstep_c) {
  const int64_t r = ri;
  const int64_t c0 = (int64_t)csi * AS_P;
  const int np = min(AS_P, Wi - csi * AS_P);
  if (tid < AS_P) {
    bool ok = tid < np;
    if (apply_mask)
      for (int q = 0; q < L.n; ++q) ok = ok && covered(r, c0 + tid, H, W, sdr[q], sdc[q]);
    okp[tid] = (uint8_t)ok;
    fl[tid] = 0;
  }
  if (BUF) {
    // per laser: the strip's source offset and its valid pixel range [clo, chi) (row outside the
    // laser's coverage: empty)
    int rbase[5], clo[5], chi[5];
    __amdgpu_buffer_rsrc_t rs[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int dr = __builtin_amdgcn_readfirstlane(sdr[q]), dc = __builtin_amdgcn_readfirstlane(sdc[q]);
      rs[q] = __builtin_amdgcn_make_buffer_rsrc((void *)L.src[q], (short)0, (int)(H * W * EcoliLasers<0>::cl(q) * 4),
                                                0x00020000);
      const bool row_ok = ri >= (dr > 0 ? dr : 0) && ri < Hi + (dr < 0 ? dr : 0);
      const int cmin = dc > 0 ? dc : 0, cmax = min(Wi + (dc < 0 ? dc : 0), Wi);
      const int c0i = csi * AS_P;
      clo[q] = row_ok ? max(cmin - c0i, 0) : AS_P;
      chi[q] = row_ok ? min(cmax - c0i, np) : 0;
      rbase[q] = ((ri - dr) * Wi + (c0i - dc)) * EcoliLasers<0>::cl(q);
    }
    lay_load_buf<0, 2>(rs, rbase, clo, chi, tid, v);
    lay_store<0, 2>(tile, tid, v);
    lay_load_buf<2, 5>(rs, rbase, clo, chi, tid, v);
    lay_store<2, 5>(tile, tid, v);
  } else {
    lay_load<0, 2>(L, sdr, sdc, r, c0, H, W, tid, v);
    lay_store<0, 2>(tile, tid, v);
    lay_load<2, 5>(L, sdr, sdc, r, c0, H, W, tid, v);
    lay_store<2, 5>(tile, tid, v);
  }
  __syncthreads();
  float *out = dst ? dst + (r * W + c0) * (int64_t)C : nullptr;
  const int n = dst ? np * C : 0;
  if (!dst) {
    // the registered stack is not materialised (the pixel table and image_cn are what the path
    // reads; label sums read the lasers): no store
  } else if (np == AS_P) {   // a full strip: 64 x 95 floats, 16-byte aligned (W multiple of 64)
    for (int vv = tid; vv < (n >> 2); vv += 256) {
      const int e = vv << 2;
      float4 x = reinterpret_cast<const float4 *>(tile)[vv];
      if (apply_mask) {
        x.x = okp[e / C] ? x.x : 0.0f;
        x.y = okp[(e + 1) / C] ? x.y : 0.0f;
        x.z = okp[(e + 2) / C] ? x.z : 0.0f;
        x.w = okp[(e + 3) / C] ? x.w : 0.0f;
      }
      reinterpret_cast<float4 *>(out)[vv] = x;
    }
  } else {
    for (int e = tid; e < n; e += 256) out[e] = (!apply_mask || okp[e / C]) ? tile[e] : 0.0f;
  }
  if (cn_out) {
    // 8 lanes per pixel; a 32-lane group takes pixels g, g + 8, g + 16, g + 24 (g = tid >> 5), so
    // with the odd row stride its reads fall in 32 distinct banks
    const int j = tid & 7;
    constexpr int main_n = C - (C % 8);
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
      const int pi = half * 32 + (tid >> 5) + 8 * ((tid >> 3) & 3);
      const float *a = tile + (pi < np ? pi : 0) * C;
      const bool ok = pi < np && (!apply_mask || okp[pi]);
      double rr = ok ? (double)a[j] : 0.0;
#pragma unroll 2
      for (int i = 8; i < main_n; i += 8) rr += ok ? (double)a[i + j] : 0.0;
      rr = rr + __shfl_xor(rr, 1, 64);
      rr = rr + __shfl_xor(rr, 2, 64);
      rr = rr + __shfl_xor(rr, 4, 64);
      double res = rr;
      if (j == 0)
        for (int i = main_n; i < C; ++i) res += ok ? (double)a[i] : 0.0;
      if (j == 0 && pi < np) {
        if (ptab) {  // the log is taken once per pixel in the table phase
          cns[pi] = res;
        } else {
          double sv = 0.0 + res;
          if (cn_mode == 1) sv = hrf_cr_log(sv + 1e-2);
          else if (cn_mode == 2) sv = hrf_cr_log10(sv + 1.0);
          cn_out[r * W + c0 + pi] = sv;
        }
      }
    }
  }
  if (ptab) {  // the classifier's operands from the same tile (pixtable.hpp); W % 16 == 0
    const uint8_t *okm = apply_mask ? okp : nullptr;
    hrf_pix::ecoli_norms(tile, okm, np, invs, fl);  // beside the channel sums: the tile is only read
    __syncthreads();
    const int64_t p0 = r * W + c0;
    if (tid < np) {
      pflags[p0 + tid] = (uint8_t)fl[tid];
      if (cn_out) {
        double sv = 0.0 + cns[tid];
        if (cn_mode == 1) sv = hrf_cr_log(sv + 1e-2);
        else if (cn_mode == 2) sv = hrf_cr_log10(sv + 1.0);
        cn_out[p0 + tid] = sv;
      }
    }
    hrf_pix::ecoli_table(tile, okm, np, p0, invs, ptab);
  }
  __syncthreads();  // the next strip rewrites tile, okp, fl, invs and cns
  }
}

// E. coli assembly launch: a resident grid of the kernel built for four workgroups per CU (128
// VGPRs, no spills).  Round 5: the pixel-table form no longer normalises the tile in place (the
// norms share the channel sums' barrier interval, the table applies them), the channel-sum reads
// are bank-conflict free and the loads go through buffer descriptors: 0.98 -> 0.92 ms alone,
// per-pixel-off line +4 % (profiles/r5_asm_ab.txt); it was three per CU (165 VGPRs) in rounds 3-4,
// where four spilled.  One workgroup per strip instead of the resident grid lost in round 3.
template <bool BUF>
void launch_assemble_b(const Lasers &L, int64_t H, int64_t W, int apply_mask, float *dst, double *cn_out, int cn_mode,
                       uint4 *table, uint8_t *flags, hipStream_t s) {
  const int64_t nstrip = hrf::cdiv(W, AS_P) * H;
  const unsigned grid = hrf::resident_grid(assemble_ecoli_kernel<BUF>, 256, 0, nstrip);
  assemble_ecoli_kernel<BUF><<<grid, 256, 0, s>>>(L, H, W, apply_mask, dst, cn_out, cn_mode, table, flags);
}

void launch_assemble(const Lasers &L, int64_t H, int64_t W, int apply_mask, float *dst, double *cn_out, int cn_mode,
                     uint4 *table, uint8_t *flags, hipStream_t s) {
  // buffer-descriptor loads while every laser buffer (H W 32 floats at most) is < 2 GiB
  if (H * W * 32 * 4 < ((int64_t)1 << 31))
    launch_assemble_b<true>(L, H, W, apply_mask, dst, cn_out, cn_mode, table, flags, s);
  else
    launch_assemble_b<false>(L, H, W, apply_mask, dst, cn_out, cn_mode, table, flags, s);
}

// numpy pairwise_sum over n f32 values (as f64), n <= 512
__device__ double pw_block(const float *a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += (double)a[i];
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (double)a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += (double)a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += (double)a[i];
  return res;
}
__device__ double pw_l1(const float *a, int n) {
  if (n <= 128) return pw_block(a, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pw_block(a, n2) + pw_block(a + n2, n - n2);
}
__device__ double pw_sum(const float *a, int n) {
  if (n <= 256) return pw_l1(a, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pw_l1(a, n2) + pw_l1(a + n2, n - n2);
}

__global__ void channel_sum_kernel(const float *__restrict__ stack, int64_t npix, int C,
                                   const uint8_t *__restrict__ mask, int mode, int negate, double *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    double s = (mask && !mask[p]) ? 0.0 : 0.0 + pw_sum(stack + p * C, C);
    if (mode == 1) s = hrf_cr_log(s + 1e-2);
    else if (mode == 2) s = hrf_cr_log10(s + 1.0);
    out[p] = negate ? -s : s;
  }
}

// Flat-field calibration folded into a reduction: channels [c0, c1) of pixel p are divided by
// cal[p * sp + c * sc] in f64 (numpy's stack / calibration_image broadcasting: sp = 1, sc = 0
// for an (H, W) plane; sp = 0, sc = 1 for a (C,) vector; sp = C, sc = 1 for (H, W, C)).
struct Cal {
  const float *p;
  int64_t sp;
  int32_t sc, c0, c1;
  __device__ __forceinline__ double apply(double x, int64_t pix, int c) const {
    return (p && c >= c0 && c < c1) ? x / (double)p[pix * sp + (int64_t)c * sc] : x;
  }
};

// C <= 128: 64-pixel chunks staged through LDS with 16-byte loads (coalesced), then 8 lanes per
// pixel: lane j accumulates numpy's r[j] (a[j] + a[j+8] + ...), the three xor-shuffle levels
// are exactly ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), lane 0 adds the tail in order.  The next
// chunk's loads are issued into registers right after this chunk lands in LDS, so they are in
// flight while it is reduced (0.364 -> 0.337 ms at 2048^2 x 95, 56 -> 60 % of HBM peak).
constexpr int CS_P = 64;

// The 16-byte loads of chunk c into eight named registers (an indexed array is not promoted
// out of scratch here), nothing past the last chunk; CS_PUT stores them into LDS.
#define CS_FETCH(c)                                                                                  \
  {                                                                                                  \
    const int64_t q0 = (c) * CS_P;                                                                   \
    const int nvq = (c) < nchunks ? (int)(((int64_t)min((int64_t)CS_P, npix - q0) * C) >> 2) : 0;   \
    const float4 *g = reinterpret_cast<const float4 *>(stack + q0 * C);                             \
    if (tid < nvq) r0 = g[tid];                                                                      \
    if (tid + 256 < nvq) r1 = g[tid + 256];                                                          \
    if (tid + 512 < nvq) r2 = g[tid + 512];                                                          \
    if (tid + 768 < nvq) r3 = g[tid + 768];                                                          \
    if (tid + 1024 < nvq) r4 = g[tid + 1024];                                                        \
    if (tid + 1280 < nvq) r5 = g[tid + 1280];                                                        \
    if (tid + 1536 < nvq) r6 = g[tid + 1536];                                                        \
    if (tid + 1792 < nvq) r7 = g[tid + 1792];                                                        \
  }
#define CS_PUT(nv)                                                                                   \
  {                                                                                                  \
    float4 *d = reinterpret_cast<float4 *>(sb);                                                      \
    if (tid < (nv)) d[tid] = r0;                                                                     \
    if (tid + 256 < (nv)) d[tid + 256] = r1;                                                         \
    if (tid + 512 < (nv)) d[tid + 512] = r2;                                                         \
    if (tid + 768 < (nv)) d[tid + 768] = r3;                                                         \
    if (tid + 1024 < (nv)) d[tid + 1024] = r4;                                                       \
    if (tid + 1280 < (nv)) d[tid + 1280] = r5;                                                       \
    if (tid + 1536 < (nv)) d[tid + 1536] = r6;                                                       \
    if (tid + 1792 < (nv)) d[tid + 1792] = r7;                                                       \
  }
static_assert(CS_P * 128 / 4 == 8 * 256, "CS_FETCH covers 8 float4 per thread");

template <bool CAL>
__global__ __launch_bounds__(256) void channel_sum_lds_kernel(const float *__restrict__ stack, int64_t npix, int C,
                                                              const uint8_t *__restrict__ mask, int mode, int negate,
                                                              double *__restrict__ out, int vec_ok, Cal cal) {
  extern __shared__ __attribute__((aligned(16))) float sb[];
  const int tid = threadIdx.x;
  const int64_t nchunks = (npix + CS_P - 1) / CS_P;
  const int j = tid & 7;
  const int main_n = C < 8 ? 0 : C - (C % 8);
  // Vector path, software-pipelined: the next chunk's 16-byte loads are in flight in
  // registers while this chunk is reduced from LDS (C <= 128: at most 8 per thread).
  float4 r0, r1, r2, r3, r4, r5, r6, r7;
  if (vec_ok) CS_FETCH((int64_t)blockIdx.x)
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int64_t p0 = ch * CS_P;
    const int np = (int)min((int64_t)CS_P, npix - p0);
    const int64_t nel = (int64_t)np * C;
    const float *src = stack + p0 * C;
    if (vec_ok) {
      const int nv = (int)(nel >> 2);
      CS_PUT(nv)
      for (int e = (nv << 2) + tid; e < nel; e += 256) sb[e] = src[e];
    } else {
      for (int e = tid; e < nel; e += 256) sb[e] = src[e];
    }
    __syncthreads();
    if (vec_ok) CS_FETCH(ch + gridDim.x)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int pi = half * 32 + (tid >> 3);
      const float *a = sb + pi * C;
      const int64_t pix = p0 + (pi < np ? pi : 0);
      auto val = [&](int i) { return CAL ? cal.apply((double)a[i], pix, i) : (double)a[i]; };
      double res = 0.0;
      if (C >= 8) {
        double r = val(j);
        for (int i = 8; i < main_n; i += 8) r += val(i + j);
        r = r + __shfl_xor(r, 1, 64);
        r = r + __shfl_xor(r, 2, 64);
        r = r + __shfl_xor(r, 4, 64);
        res = r;
        if (j == 0)
          for (int i = main_n; i < C; ++i) res += val(i);
      } else if (j == 0) {
        for (int i = 0; i < C; ++i) res += val(i);
      }
      if (j == 0 && pi < np) {
        const int64_t p = p0 + pi;
        double sv = (mask && !mask[p]) ? 0.0 : 0.0 + res;
        if (mode == 1) sv = hrf_cr_log(sv + 1e-2);
        else if (mode == 2) sv = hrf_cr_log10(sv + 1.0);
        out[p] = negate ? -sv : sv;
      }
    }
    __syncthreads();
  }
}

#undef CS_FETCH
#undef CS_PUT

__global__ void max_f64_kernel(const double *__restrict__ a, int64_t n, unsigned long long *__restrict__ mx) {
  // order-preserving encoding so atomicMax on uint64 is a max on doubles
  unsigned long long m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long b = __double_as_longlong(a[i]);
    const unsigned long long e = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    m = e > m ? e : m;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long u = __shfl_xor(m, o, 64);
    m = u > m ? u : m;
  }
  __shared__ unsigned long long red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) m = red[q] > m ? red[q] : m;
    if (m) atomicMax(mx, m);
  }
}

__global__ void decode_max_kernel(unsigned long long *mx) {
  const unsigned long long e = *mx;
  const unsigned long long b = (e >> 63) ? (e & 0x7fffffffffffffffull) : ~e;
  *reinterpret_cast<double *>(mx) = __longlong_as_double((long long)b);
}

__global__ void div_scalar_kernel(const double *__restrict__ a, int64_t n, const double *__restrict__ d,
                                  double *__restrict__ o) {
  const double v = *d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = a[i] / v;
}

__global__ void pad_edge_kernel(const double *__restrict__ a, int64_t H, int64_t W, int w, double *__restrict__ o) {
  const int64_t HP = H + 2 * w, WP = W + 2 * w;
  const int64_t n = HP * WP;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / WP, c = i - r * WP;
    int64_t rr = r - w, cc = c - w;
    rr = rr < 0 ? 0 : (rr >= H ? H - 1 : rr);
    cc = cc < 0 ? 0 : (cc >= W ? W - 1 : cc);
    o[i] = a[rr * W + cc];
  }
}

__global__ void pad_edge3_kernel(const double *__restrict__ a, int64_t X, int64_t Y, int64_t Z, int w,
                                 double *__restrict__ o) {
  const int64_t YP = Y + 2 * w, ZP = Z + 2 * w;
  const int64_t n = (X + 2 * w) * YP * ZP;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i / (YP * ZP), r = i - x * YP * ZP, y = r / ZP, z = r - y * ZP;
    int64_t xx = x - w, yy = y - w, zz = z - w;
    xx = xx < 0 ? 0 : (xx >= X ? X - 1 : xx);
    yy = yy < 0 ? 0 : (yy >= Y ? Y - 1 : yy);
    zz = zz < 0 ? 0 : (zz >= Z ? Z - 1 : zz);
    o[i] = a[(xx * Y + yy) * Z + zz];
  }
}

__global__ void mask_mul_kernel(const double *__restrict__ a, const uint8_t *__restrict__ m, int64_t n,
                                double *__restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = a[i] * (double)(m[i] != 0);
}

// np.max(stack, axis=2) as f64 (ecoli measurement.py:45, the registration images)
__global__ void channel_max_kernel(const float *__restrict__ stack, int64_t npix, int C, double *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    const float *a = stack + p * C;
    float m = a[0];
    for (int c = 1; c < C; ++c) m = (a[c] > m || a[c] != a[c]) ? a[c] : m;  // numpy max propagates NaN
    out[p] = (double)m;
  }
}

// 64-pixel chunks staged in LDS with 16-byte loads (a chunk is one contiguous 64 x C run), then
// four lanes per pixel reduce a quarter of its channels each: coalesced, unlike a thread per
// pixel walking its own channels.  Same NaN-propagating max.
constexpr int CM_P = 64;
__global__ __launch_bounds__(256) void channel_max_lds_kernel(const float *__restrict__ stack, int64_t npix, int C,
                                                              double *__restrict__ out, int vec_ok) {
  extern __shared__ __attribute__((aligned(16))) float sb[];
  const int tid = threadIdx.x, pi = tid >> 2, q = tid & 3;
  for (int64_t ch = blockIdx.x; ch * CM_P < npix; ch += gridDim.x) {
    const int64_t p0 = ch * CM_P;
    const int np = (int)min((int64_t)CM_P, npix - p0);
    const int nel = np * C;
    const float *src = stack + p0 * C;
    int e0 = 0;
    if (vec_ok) {
      for (int v = tid; v < (nel >> 2); v += 256) reinterpret_cast<float4 *>(sb)[v] = reinterpret_cast<const float4 *>(src)[v];
      e0 = (nel >> 2) << 2;
    }
    for (int e = e0 + tid; e < nel; e += 256) sb[e] = src[e];
    __syncthreads();
    float m = -__builtin_inff();
    bool any = false;
    if (pi < np) {
      const float *a = sb + pi * C;
      for (int c = q; c < C; c += 4) {
        const float v = a[c];
        m = (!any || v > m || v != v) ? v : m;
        any = true;
      }
    }
#pragma unroll
    for (int o = 1; o <= 2; o <<= 1) {
      const float v = __shfl_xor(m, o, 64);
      const bool va = __shfl_xor((int)any, o, 64) != 0;
      if (va) {
        m = (!any || v > m || v != v || m != m) ? (m != m ? m : v) : m;
        any = true;
      }
    }
    if (q == 0 && pi < np) out[p0 + pi] = (double)m;
    __syncthreads();
  }
}

// All lasers' channel-max projections in one launch (ecoli :45, one per laser before the shift
// estimate): workgroups are split between the lasers in proportion to their channel counts and
// each walks its laser's 64-pixel chunks as channel_max_lds_kernel does.
struct MaxJob {
  const float *src[LMAX];
  double *out[LMAX];
  int32_t C[LMAX];
  int32_t wg0[LMAX + 1];  // first workgroup of each laser; wg0[n] = grid size
  int32_t n;
};

__global__ __launch_bounds__(256) void channel_max_multi_kernel(MaxJob J, int64_t npix) {
  extern __shared__ __attribute__((aligned(16))) float sb[];
  int l = 0;
#pragma unroll
  for (int q = 1; q < LMAX; ++q)
    if (q < J.n && (int)blockIdx.x >= J.wg0[q]) l = q;
  const int C = J.C[l];
  const float *stack = J.src[l];
  double *out = J.out[l];
  const int nwg = J.wg0[l + 1] - J.wg0[l], wg = (int)blockIdx.x - J.wg0[l];
  const int vec_ok = ((uintptr_t)stack & 15) == 0 && (CM_P * C) % 4 == 0;
  const int tid = threadIdx.x, pi = tid >> 2, q = tid & 3;
  for (int64_t ch = wg; ch * CM_P < npix; ch += nwg) {
    const int64_t p0 = ch * CM_P;
    const int np = (int)min((int64_t)CM_P, npix - p0);
    const int nel = np * C;
    const float *src = stack + p0 * C;
    int e0 = 0;
    if (vec_ok) {
      for (int v = tid; v < (nel >> 2); v += 256) reinterpret_cast<float4 *>(sb)[v] = reinterpret_cast<const float4 *>(src)[v];
      e0 = (nel >> 2) << 2;
    }
    for (int e = e0 + tid; e < nel; e += 256) sb[e] = src[e];
    __syncthreads();
    float m = -__builtin_inff();
    bool any = false;
    if (pi < np) {
      const float *a = sb + pi * C;
      for (int c = q; c < C; c += 4) {
        const float v = a[c];
        m = (!any || v > m || v != v) ? v : m;
        any = true;
      }
    }
#pragma unroll
    for (int o = 1; o <= 2; o <<= 1) {
      const float v = __shfl_xor(m, o, 64);
      const bool va = __shfl_xor((int)any, o, 64) != 0;
      if (va) {
        m = (!any || v > m || v != v || m != m) ? (m != m ? m : v) : m;
        any = true;
      }
    }
    if (q == 0 && pi < np) out[p0 + pi] = (double)m;
    __syncthreads();
  }
}

// The same for C <= 32 and whole 128-pixel chunks, software-pipelined: the next chunk's
// 16-byte loads (at most 4 per thread) are in flight in registers while this chunk is reduced
// from LDS; two lanes per pixel.
constexpr int CM_P2 = 128;
__global__ __launch_bounds__(256) void channel_max_multi_pf_kernel(MaxJob J, int64_t npix) {
  __shared__ __attribute__((aligned(16))) float sb[CM_P2 * 32];
  int l = 0;
#pragma unroll
  for (int q = 1; q < LMAX; ++q)
    if (q < J.n && (int)blockIdx.x >= J.wg0[q]) l = q;
  const int C = J.C[l];
  const float4 *g = reinterpret_cast<const float4 *>(J.src[l]);
  double *out = J.out[l];
  const int nwg = J.wg0[l + 1] - J.wg0[l], wg = (int)blockIdx.x - J.wg0[l];
  const int tid = threadIdx.x, pi = tid >> 1, h = tid & 1;
  const int nv = CM_P2 * C / 4;          // float4 per chunk
  const int64_t nch = npix / CM_P2;
  float4 r0, r1, r2, r3;
  auto fetch = [&](int64_t ch) {
    if (ch >= nch) return;
    const float4 *s = g + ch * nv;
    if (tid < nv) r0 = s[tid];
    if (tid + 256 < nv) r1 = s[tid + 256];
    if (tid + 512 < nv) r2 = s[tid + 512];
    if (tid + 768 < nv) r3 = s[tid + 768];
  };
  fetch(wg);
  for (int64_t ch = wg; ch < nch; ch += nwg) {
    float4 *d = reinterpret_cast<float4 *>(sb);
    if (tid < nv) d[tid] = r0;
    if (tid + 256 < nv) d[tid + 256] = r1;
    if (tid + 512 < nv) d[tid + 512] = r2;
    if (tid + 768 < nv) d[tid + 768] = r3;
    __syncthreads();
    fetch(ch + nwg);
    const float *a = sb + pi * C;
    float m = a[h];
    for (int c = h + 2; c < C; c += 2) {
      const float v = a[c];
      m = (v > m || v != v) ? v : m;
    }
    if (C > 1) {
      const float v = __shfl_xor(m, 1, 64);
      m = (m != m) ? m : ((v > m || v != v) ? v : m);
    }
    if (h == 0) out[ch * CM_P2 + pi] = (double)m;
    __syncthreads();
  }
}

__global__ void and_u8_kernel(const uint8_t *__restrict__ a, const uint8_t *__restrict__ b, int64_t n,
                              uint8_t *__restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = (uint8_t)(a[i] != 0 && b[i] != 0);
}

__global__ void mask_labels_kernel(const int32_t *__restrict__ l, const uint8_t *__restrict__ m, int64_t n,
                                   int32_t *__restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = m[i] ? l[i] : 0;
}

// the calibrated stack as f64 (multispecies :104 image_channel, written as _registered.npy :166)
__global__ void calibrate_kernel(const float *__restrict__ stack, int64_t npix, int C, Cal cal,
                                 double *__restrict__ out) {
  const int64_t n = npix * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = e / C;
    out[e] = cal.apply((double)stack[e], p, (int)(e - p * C));
  }
}

// a15 per-label spectra (label_sums_wave_kernel, stats.hip) read straight from the per-laser
// acquisitions: lane = channel c (c, c + 64), its laser q(c) and local channel fixed per lane; a
// foreground pixel's value is its laser's source pixel shifted by (dr_q, dc_q), 0 outside the
// laser's frame or -- apply_mask -- outside any laser's frame (register_assemble's stack, which
// then never has to exist).  CAL: a per-pixel flat field on channels [cal0, cal1).
template <bool CAL>
__global__ __launch_bounds__(256) void label_sums_lasers_kernel(Lasers L, int64_t H, int64_t W, int apply_mask,
                                                                const int32_t *__restrict__ lab, int32_t maxlab,
                                                                const float *__restrict__ cal, int cal0, int cal1,
                                                                double *__restrict__ sums,
                                                                unsigned long long *__restrict__ counts) {
  constexpr int LB = 16;
  __shared__ int sdr[LMAX], sdc[LMAX];
  load_shifts(L, sdr, sdc);
  const int C = L.c0[L.n];
  const int64_t npix = H * W;
  const int lane = hrf::lane_id();
  const int64_t nchunks = (npix + 63) >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t ch = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int c0 = lane, c1 = lane + 64;
  const bool v0 = c0 < C, v1 = c1 < C;
  const bool k0 = CAL && c0 >= cal0 && c0 < cal1, k1 = CAL && c1 >= cal0 && c1 < cal1;
  int q0 = 0, q1 = 0;
#pragma unroll
  for (int q = 1; q < LMAX; ++q) {
    if (q < L.n && c0 >= L.c0[q]) q0 = q;
    if (q < L.n && c1 >= L.c0[q]) q1 = q;
  }
  const int cl0 = L.c0[q0 + 1] - L.c0[q0], cl1 = L.c0[q1 + 1] - L.c0[q1];
  const float *s0 = L.src[q0] + (c0 - L.c0[q0]), *s1 = L.src[q1] + (c1 - L.c0[q1]);
  const int dr0 = sdr[q0], dc0 = sdc[q0], dr1 = sdr[q1], dc1 = sdc[q1];
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
    double prc = 1.0;  // lane = pixel: one division per 64 pixels, 1 / flat field
    if (CAL) {
      pcal = (p0 + lane < npix) ? cal[p0 + lane] : 1.0f;
      prc = 1.0 / (double)pcal;
    }
    // the chunk's pixels: lane = pixel for the coverage of the whole stack (apply_mask), a bit
    // per pixel; the row of every pixel once (no 64-bit division per fetched pixel)
    const int64_t pl = p0 + lane;
    const int64_t rl = pl / W, cl = pl - rl * W;
    bool okl = pl < npix;
    if (apply_mask)
      for (int q = 0; q < L.n; ++q) okl = okl && covered(rl, cl, H, W, sdr[q], sdc[q]);
    const unsigned long long okmask = __ballot(okl);
    int32_t run = 0;  // wave-uniform
    unsigned long long n = 0;
    double a0 = 0.0, a1 = 0.0;
    while (fg) {
      int idx[LB];
      int nb = 0;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        idx[j] = fg ? __ffsll((long long)fg) - 1 : -1;
        if (fg) {
          fg &= fg - 1;
          ++nb;
        }
      }
      float x0[LB], x1[LB];
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        x0[j] = x1[j] = 0.0f;
        if (j < nb) {
          const int64_t r = __shfl(rl, idx[j], 64), c = __shfl(cl, idx[j], 64);
          const bool ok = (okmask >> idx[j]) & 1ull;
          if (ok && v0 && covered(r, c, H, W, dr0, dc0))
            x0[j] = __builtin_nontemporal_load(s0 + ((r - dr0) * W + (c - dc0)) * cl0);
          if (ok && v1 && covered(r, c, H, W, dr1, dc1))
            x1[j] = __builtin_nontemporal_load(s1 + ((r - dr1) * W + (c - dc1)) * cl1);
        }
      }
#pragma unroll
      for (int j = 0; j < LB; ++j) {
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
          if (CAL) {
            // x / d bit for bit through the pixel's reciprocal (detmath.h hrf_div_rcp: x and d
            // are float32 values); d zero or not finite keeps the division
            const float df = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pcal), idx[j]));
            const double d = (double)df;
            const unsigned long long rb = __builtin_bit_cast(unsigned long long, prc);
            const double r = __builtin_bit_cast(
                double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(rb >> 32), idx[j]) << 32) |
                            (unsigned)__builtin_amdgcn_readlane((int)(unsigned)rb, idx[j]));
            if (df != 0.0f && __builtin_isfinite(df)) {
              a0 += k0 ? hrf_div_rcp((double)x0[j], d, r) : (double)x0[j];
              a1 += k1 ? hrf_div_rcp((double)x1[j], d, r) : (double)x1[j];
            } else {
              a0 += k0 ? (double)x0[j] / d : (double)x0[j];
              a1 += k1 ? (double)x1[j] / d : (double)x1[j];
            }
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

// label_sums_lasers_kernel for W % 64 == 0: every 64-pixel chunk lies in one row, so a lane's
// laser covers a contiguous range [lo, lo + span) of the chunk's pixels, and its pixel idx reads
// base + (idx - lo) * cl -- the per-pixel row / column, coverage test and 64-bit address of the
// general kernel (≈100 VALU and 13 quarter-rate 64-bit multiplies per labelled pixel, which
// bound it) become one compare and one 24-bit multiply-add per lane.  Same per-wave partial sums
// as the general kernel (runs of equal labels in raster order, f64 per lane, the same atomics);
// a pixel outside the coverage (apply_mask) counts with a zero spectrum, as there.
template <bool CAL>
__global__ __launch_bounds__(256) void label_sums_lasers_row_kernel(Lasers L, int64_t H, int64_t W, int apply_mask,
                                                                    const int32_t *__restrict__ lab, int32_t maxlab,
                                                                    const float *__restrict__ cal, int cal0, int cal1,
                                                                    double *__restrict__ sums,
                                                                    unsigned long long *__restrict__ counts) {
  constexpr int LB = 16;
  __shared__ int sdr[LMAX], sdc[LMAX];
  load_shifts(L, sdr, sdc);
  const int C = L.c0[L.n];
  const int64_t npix = H * W;
  const int lane = hrf::lane_id();
  const int64_t nchunks = npix >> 6;  // W % 64 == 0
  const int64_t cpr = W >> 6;         // chunks per row
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t ch = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = lane, c1 = lane + 64;
  const bool v0 = c0 < C, v1 = c1 < C;
  const bool k0 = CAL && c0 >= cal0 && c0 < cal1, k1 = CAL && c1 >= cal0 && c1 < cal1;
  int q0 = 0, q1 = 0;
#pragma unroll
  for (int q = 1; q < LMAX; ++q) {
    if (q < L.n && c0 >= L.c0[q]) q0 = q;
    if (q < L.n && c1 >= L.c0[q]) q1 = q;
  }
  const int cl0 = L.c0[q0 + 1] - L.c0[q0], cl1 = L.c0[q1 + 1] - L.c0[q1];
  const float *s0 = L.src[q0] + (c0 - L.c0[q0]), *s1 = L.src[q1] + (c1 - L.c0[q1]);
  const int dr0 = sdr[q0], dc0 = sdc[q0], dr1 = sdr[q1], dc1 = sdc[q1];
  auto load_label = [&](int64_t c) -> int32_t {
    const int64_t p = (c << 6) + lane;
    int32_t l = c < nchunks ? __builtin_nontemporal_load(lab + p) : 0;
    return (l < 0 || l > maxlab) ? 0 : l;
  };
  // the lane's laser over the chunk (row r, columns cs .. cs + 63): pixels [lo, lo + span),
  // pixel lo at base
  auto span_of = [&](int64_t r, int64_t cs, bool v, int dr, int dc, const float *src, int cl, const float **base,
                     int *lo) -> unsigned {
    const int64_t rr = r - dr, col = cs - dc;
    const int64_t a = col < 0 ? -col : 0, b = W - col < 64 ? W - col : 64;
    const bool ok = v && rr >= 0 && rr < H && b > a;
    *lo = ok ? (int)a : 0;
    *base = ok ? src + (rr * W + col + a) * cl : src;
    return ok ? (unsigned)(b - a) : 0u;
  };
  int32_t lnext = load_label(ch);
  for (; ch < nchunks; ch += nwaves) {
    const int32_t l = lnext;
    lnext = load_label(ch + nwaves);
    unsigned long long fg = __ballot(l != 0);
    if (!fg) continue;
    const int64_t p0 = ch << 6;
    const int64_t r = ch / cpr, cs = (ch - r * cpr) << 6;
    float pcal = 1.0f;
    double prc = 1.0;  // lane = pixel: one division per 64 pixels, 1 / flat field
    if (CAL) {
      pcal = cal[p0 + lane];
      prc = 1.0 / (double)pcal;
    }
    unsigned long long okmask = ~0ull;
    if (apply_mask) {
      bool okl = true;
      for (int q = 0; q < L.n; ++q) okl = okl && covered(r, cs + lane, H, W, sdr[q], sdc[q]);
      okmask = __ballot(okl);
    }
    const float *b0, *b1;
    int lo0, lo1;
    const unsigned sp0 = span_of(r, cs, v0, dr0, dc0, s0, cl0, &b0, &lo0);
    const unsigned sp1 = span_of(r, cs, v1, dr1, dc1, s1, cl1, &b1, &lo1);
    int32_t run = 0;  // wave-uniform
    unsigned long long n = 0;
    double a0 = 0.0, a1 = 0.0;
    while (fg) {
      int idx[LB];
      int nb = 0;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        idx[j] = fg ? __ffsll((long long)fg) - 1 : -1;
        if (fg) {
          fg &= fg - 1;
          ++nb;
        }
      }
      float x0[LB], x1[LB];
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        x0[j] = x1[j] = 0.0f;
        if (j < nb && ((okmask >> idx[j]) & 1ull)) {
          const unsigned u0 = (unsigned)(idx[j] - lo0), u1 = (unsigned)(idx[j] - lo1);
          if (u0 < sp0) x0[j] = __builtin_nontemporal_load(b0 + __umul24(u0, (unsigned)cl0));
          if (u1 < sp1) x1[j] = __builtin_nontemporal_load(b1 + __umul24(u1, (unsigned)cl1));
        }
      }
#pragma unroll
      for (int j = 0; j < LB; ++j) {
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
          if (CAL) {
            const float df = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pcal), idx[j]));
            const double d = (double)df;
            const unsigned long long rb = __builtin_bit_cast(unsigned long long, prc);
            const double rc = __builtin_bit_cast(
                double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(rb >> 32), idx[j]) << 32) |
                            (unsigned)__builtin_amdgcn_readlane((int)(unsigned)rb, idx[j]));
            if (df != 0.0f && __builtin_isfinite(df)) {
              a0 += k0 ? hrf_div_rcp((double)x0[j], d, rc) : (double)x0[j];
              // channels 64.. calibrated on no lane (the E. coli flat field covers 0..31): a plain sum
              a1 += (cal1 > 64 && k1) ? hrf_div_rcp((double)x1[j], d, rc) : (double)x1[j];
            } else {
              a0 += k0 ? (double)x0[j] / d : (double)x0[j];
              a1 += k1 ? (double)x1[j] / d : (double)x1[j];
            }
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

}  // namespace

extern "C" {

static hrf_status register_assemble(const float *const *src_host, const int32_t *channels_host,
                                    const int32_t *shifts_host, const int32_t *shifts_dev, int32_t nlaser, int64_t H,
                                    int64_t W, int32_t apply_mask, float *dst, hrf_stream_t stream,
                                    double *cn_out = nullptr, int32_t cn_mode = 0) {
  HRF_REQUIRE(nlaser >= 1 && nlaser <= LMAX && src_host && channels_host && (shifts_host || shifts_dev),
              "register_assemble: bad lasers");
  Lasers L{};
  L.n = nlaser;
  L.c0[0] = 0;
  L.dsh = shifts_dev;
  for (int i = 0; i < nlaser; ++i) {
    HRF_REQUIRE(channels_host[i] >= 1 && src_host[i], "register_assemble: laser %d empty", i);
    L.src[i] = src_host[i];
    L.c0[i + 1] = L.c0[i] + channels_host[i];
    L.dr[i] = shifts_host ? shifts_host[2 * i] : 0;
    L.dc[i] = shifts_host ? shifts_host[2 * i + 1] : 0;
  }
  for (int i = nlaser + 1; i <= LMAX; ++i) L.c0[i] = L.c0[nlaser];
  const int64_t n = H * W * L.c0[nlaser];
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(dst, "register_assemble: null output");
  const int C = L.c0[nlaser];
  if (C <= 128 && H <= 65535) {
    // row runs start at pixel (r, 64 k): 16-byte aligned when W * C is a multiple of 4 floats
    const int vec_ok = ((W * C) % 4 == 0) && (((uintptr_t)dst & 15) == 0);
    dim3 grid((unsigned)hrf::cdiv(W, AS_P), (unsigned)H);
    bool ecoli = nlaser == 5 && W % 4 == 0 && (((uintptr_t)dst & 15) == 0);
    for (int i = 0; i < nlaser && ecoli; ++i) ecoli = channels_host[i] == EcoliLasers<0>::cl(i);
    if (ecoli) {
      launch_assemble(L, H, W, apply_mask, dst, cn_out, cn_mode, nullptr, nullptr, (hipStream_t)stream);
      HRF_LAUNCHED();
      return HRF_OK;
    }
    assemble_lds_kernel<<<grid, 256, sizeof(float) * AS_P * C, (hipStream_t)stream>>>(L, H, W, apply_mask, dst, vec_ok,
                                                                                     cn_out, cn_mode);
  } else {
    assemble_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(L, H, W, apply_mask, dst);
  }
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_register_assemble(const float *const *src_host, const int32_t *channels_host,
                                 const int32_t *shifts_host, int32_t nlaser, int64_t H, int64_t W,
                                 int32_t apply_mask, float *dst, hrf_stream_t stream) {
  HRF_REQUIRE(shifts_host, "register_assemble: null shifts");
  return register_assemble(src_host, channels_host, shifts_host, nullptr, nlaser, H, W, apply_mask, dst, stream);
}

hrf_status hrf_register_assemble_dev(const float *const *src_host, const int32_t *channels_host,
                                     const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                     int32_t apply_mask, float *dst, hrf_stream_t stream) {
  HRF_REQUIRE(shifts_dev, "register_assemble: null device shifts");
  return register_assemble(src_host, channels_host, nullptr, shifts_dev, nlaser, H, W, apply_mask, dst, stream);
}

hrf_status hrf_register_assemble_cn_dev(const float *const *src_host, const int32_t *channels_host,
                                        const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                        int32_t apply_mask, float *dst, double *cn_out, int32_t cn_mode,
                                        hrf_stream_t stream) {
  HRF_REQUIRE(shifts_dev && cn_out && cn_mode >= 0 && cn_mode <= 2, "register_assemble_cn: bad arguments");
  int C = 0;
  for (int i = 0; i < nlaser && channels_host; ++i) C += channels_host[i];
  if (C <= 128 && H <= 65535)
    return register_assemble(src_host, channels_host, nullptr, shifts_dev, nlaser, H, W, apply_mask, dst, stream, cn_out,
                             cn_mode);
  if (hrf_status r = register_assemble(src_host, channels_host, nullptr, shifts_dev, nlaser, H, W, apply_mask, dst,
                                       stream))
    return r;
  return hrf_channel_sum(dst, H * W, C, nullptr, cn_mode, 0, cn_out, stream);
}

static hrf_status lasers_of(const float *const *src_host, const int32_t *channels_host, const int32_t *shifts_dev,
                            int32_t nlaser, Lasers *L) {
  HRF_REQUIRE(nlaser >= 1 && nlaser <= LMAX && src_host && channels_host && shifts_dev, "lasers: bad arguments");
  *L = Lasers{};
  L->n = nlaser;
  L->dsh = shifts_dev;
  for (int i = 0; i < nlaser; ++i) {
    HRF_REQUIRE(channels_host[i] >= 1 && src_host[i], "lasers: laser %d empty", i);
    L->src[i] = src_host[i];
    L->c0[i + 1] = L->c0[i] + channels_host[i];
  }
  for (int i = nlaser + 1; i <= LMAX; ++i) L->c0[i] = L->c0[nlaser];
  return HRF_OK;
}

hrf_status hrf_register_assemble_pixtable(const float *const *src_host, const int32_t *channels_host,
                                          const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                          int32_t apply_mask, float *dst, double *cn_out, int32_t cn_mode, void *table,
                                          uint8_t *flags, hrf_stream_t stream) {
  Lasers L;
  if (hrf_status st = lasers_of(src_host, channels_host, shifts_dev, nlaser, &L)) return st;
  bool ecoli = nlaser == 5;
  for (int i = 0; i < nlaser && ecoli; ++i) ecoli = channels_host[i] == EcoliLasers<0>::cl(i);
  HRF_REQUIRE(ecoli && W % 16 == 0 && H <= 65535 && H >= 1 && W >= 16,
              "register_assemble_pixtable: the five E. coli lasers and W a multiple of 16");
  HRF_REQUIRE(cn_out && cn_mode >= 0 && cn_mode <= 2 && (table != nullptr) == (flags != nullptr),
              "register_assemble_pixtable: null output");
  HRF_REQUIRE(!dst || ((uintptr_t)dst & 15) == 0, "register_assemble_pixtable: dst must be 16-byte aligned");
  launch_assemble(L, H, W, apply_mask, dst, cn_out, cn_mode, (uint4 *)table, flags, (hipStream_t)stream);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_label_sums_lasers(const float *const *src_host, const int32_t *channels_host, const int32_t *shifts_dev,
                                 int32_t nlaser, int64_t H, int64_t W, int32_t apply_mask, const int32_t *labels,
                                 int32_t maxlab, const float *cal, int32_t cal_c0, int32_t cal_c1, double *sums,
                                 int64_t *counts, hrf_stream_t stream) {
  Lasers L;
  if (hrf_status st = lasers_of(src_host, channels_host, shifts_dev, nlaser, &L)) return st;
  const int C = L.c0[nlaser];
  HRF_REQUIRE(C <= 128 && maxlab >= 0 && H >= 0 && W >= 0, "label_sums_lasers: C must be <= 128");
  HRF_REQUIRE(sums && counts, "label_sums_lasers: null output");
  hipStream_t s = (hipStream_t)stream;
  HRF_HIP(hipMemsetAsync(sums, 0, sizeof(double) * ((size_t)maxlab + 1) * C, s));
  HRF_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * ((size_t)maxlab + 1), s));
  return hrf::label_sums_lasers_zeroed(src_host, channels_host, shifts_dev, nlaser, H, W, apply_mask, labels, maxlab,
                                       cal, cal_c0, cal_c1, sums, counts, s);
}

}  // extern "C"

hrf_status hrf::label_sums_lasers_zeroed(const float *const *src_host, const int32_t *channels_host,
                                         const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                         int32_t apply_mask, const int32_t *labels, int32_t maxlab, const float *cal,
                                         int32_t cal_c0, int32_t cal_c1, double *sums, int64_t *counts,
                                         hipStream_t s) {
  Lasers L;
  if (hrf_status st = lasers_of(src_host, channels_host, shifts_dev, nlaser, &L)) return st;
  const int C = L.c0[nlaser];
  HRF_REQUIRE(C <= 128 && maxlab >= 0 && H >= 0 && W >= 0, "label_sums_lasers: C must be <= 128");
  HRF_REQUIRE(sums && counts, "label_sums_lasers: null output");
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(labels, "label_sums_lasers: null labels");
  const int64_t nblk = hrf::cdiv(hrf::cdiv(H * W, 64), 4);
  if (W % 64 == 0) {
    if (cal) {
      const unsigned grid = hrf::resident_grid(label_sums_lasers_row_kernel<true>, 256, 0, nblk);
      label_sums_lasers_row_kernel<true><<<grid, 256, 0, s>>>(L, H, W, apply_mask, labels, maxlab, cal, cal_c0,
                                                              cal_c1, sums, (unsigned long long *)counts);
    } else {
      const unsigned grid = hrf::resident_grid(label_sums_lasers_row_kernel<false>, 256, 0, nblk);
      label_sums_lasers_row_kernel<false><<<grid, 256, 0, s>>>(L, H, W, apply_mask, labels, maxlab, nullptr, 0, 0,
                                                               sums, (unsigned long long *)counts);
    }
    HRF_LAUNCHED();
    return HRF_OK;
  }
  if (cal) {
    const unsigned grid = hrf::resident_grid(label_sums_lasers_kernel<true>, 256, 0, nblk);
    label_sums_lasers_kernel<true><<<grid, 256, 0, s>>>(L, H, W, apply_mask, labels, maxlab, cal, cal_c0, cal_c1, sums,
                                                       (unsigned long long *)counts);
  } else {
    const unsigned grid = hrf::resident_grid(label_sums_lasers_kernel<false>, 256, 0, nblk);
    label_sums_lasers_kernel<false><<<grid, 256, 0, s>>>(L, H, W, apply_mask, labels, maxlab, nullptr, 0, 0, sums,
                                                        (unsigned long long *)counts);
  }
  HRF_LAUNCHED();
  return HRF_OK;
}

extern "C" {

hrf_status hrf_channel_sum(const float *stack, int64_t npix, int32_t C, const uint8_t *mask, int32_t mode,
                           int32_t negate, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(C >= 1 && C <= 512 && mode >= 0 && mode <= 2, "channel_sum: C must be 1..512, mode 0..2");
  if (npix == 0) return HRF_OK;
  HRF_REQUIRE(stack && out, "channel_sum: null buffer");
  if (C <= 128) {
    const int vec_ok = C >= 4 && (((uintptr_t)stack & 15) == 0);
    const int64_t nch = hrf::cdiv(npix, CS_P);
    const size_t shm = sizeof(float) * CS_P * C;
    channel_sum_lds_kernel<false><<<hrf::resident_grid(channel_sum_lds_kernel<false>, 256, shm, nch), 256, shm,
                                    (hipStream_t)stream>>>(stack, npix, C, mask, mode, negate, out, vec_ok, Cal{});
  } else {
    channel_sum_kernel<<<hrf::stream_grid(npix), 256, 0, (hipStream_t)stream>>>(stack, npix, C, mask, mode, negate,
                                                                               out);
  }
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_channel_sum_cal(const float *stack, int64_t npix, int32_t C, const float *cal, int64_t cal_sp,
                               int32_t cal_sc, int32_t cal_c0, int32_t cal_c1, int32_t mode, double *out,
                               hrf_stream_t stream) {
  if (!cal) return hrf_channel_sum(stack, npix, C, nullptr, mode, 0, out, stream);
  HRF_REQUIRE(C >= 1 && C <= 128 && mode >= 0 && mode <= 2, "channel_sum_cal: C must be 1..128, mode 0..2");
  HRF_REQUIRE(cal_sp >= 0 && cal_sc >= 0 && cal_c0 >= 0 && cal_c1 <= C, "channel_sum_cal: bad calibration layout");
  if (npix == 0) return HRF_OK;
  HRF_REQUIRE(stack && out, "channel_sum_cal: null buffer");
  const int vec_ok = C >= 4 && (((uintptr_t)stack & 15) == 0);
  const int64_t nch = hrf::cdiv(npix, CS_P);
  const size_t shm = sizeof(float) * CS_P * C;
  channel_sum_lds_kernel<true><<<hrf::resident_grid(channel_sum_lds_kernel<true>, 256, shm, nch), 256, shm,
                                 (hipStream_t)stream>>>(stack, npix, C, nullptr, mode, 0, out, vec_ok,
                                                        Cal{cal, cal_sp, cal_sc, cal_c0, cal_c1});
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_channel_max(const float *stack, int64_t npix, int32_t C, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(C >= 1, "channel_max: C must be >= 1");
  if (npix == 0) return HRF_OK;
  HRF_REQUIRE(stack && out, "channel_max: null buffer");
  if (C <= 256) {
    const int vec_ok = ((uintptr_t)stack & 15) == 0 && (CM_P * C) % 4 == 0;
    const unsigned g = (unsigned)std::min<int64_t>(hrf::cdiv(npix, CM_P), 4096);
    channel_max_lds_kernel<<<g, 256, sizeof(float) * CM_P * C, (hipStream_t)stream>>>(stack, npix, C, out, vec_ok);
  } else {
    channel_max_kernel<<<hrf::stream_grid(npix), 256, 0, (hipStream_t)stream>>>(stack, npix, C, out);
  }
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_channel_max_multi(const float *const *src_host, const int32_t *channels_host, int32_t nlaser,
                                 int64_t npix, double *const *out_host, hrf_stream_t stream) {
  return hrf_channel_max_multi_grid(src_host, channels_host, nlaser, npix, out_host, 0, stream);
}

hrf_status hrf_channel_max_multi_grid(const float *const *src_host, const int32_t *channels_host, int32_t nlaser,
                                      int64_t npix, double *const *out_host, int32_t max_workgroups,
                                      hrf_stream_t stream) {
  HRF_REQUIRE(nlaser >= 1 && nlaser <= LMAX && src_host && channels_host && out_host, "channel_max_multi: bad lasers");
  HRF_REQUIRE(max_workgroups >= 0, "channel_max_multi: bad workgroup budget");
  if (npix == 0) return HRF_OK;
  MaxJob J{};
  J.n = nlaser;
  int ctot = 0, cmax = 0;
  for (int i = 0; i < nlaser; ++i) {
    HRF_REQUIRE(src_host[i] && out_host[i] && channels_host[i] >= 1, "channel_max_multi: laser %d empty", i);
    if (channels_host[i] > 256)
      for (int k = 0; k < nlaser; ++k)   // wide stacks: one launch each
        if (hrf_status r = hrf_channel_max(src_host[k], npix, channels_host[k], out_host[k], stream)) return r;
    if (channels_host[i] > 256) return HRF_OK;
    J.src[i] = src_host[i];
    J.out[i] = out_host[i];
    J.C[i] = channels_host[i];
    ctot += channels_host[i];
    cmax = std::max(cmax, (int)channels_host[i]);
  }
  const int64_t chunks = hrf::cdiv(npix, CM_P);
  // 4096 workgroups by default (two rounds on 256 CUs, the fastest alone); the tile path passes a
  // smaller budget (tile.hip)
  const int64_t total = std::min<int64_t>(chunks * nlaser, max_workgroups > 0 ? max_workgroups : 4096);
  int wg = 0;
  for (int i = 0; i < nlaser; ++i) {
    J.wg0[i] = wg;
    int64_t share = std::max<int64_t>(1, (total * J.C[i] + ctot - 1) / ctot);
    share = std::min<int64_t>(share, chunks);
    wg += (int)share;
  }
  for (int i = nlaser; i <= LMAX; ++i) J.wg0[i] = wg;
  bool pf = cmax <= 32 && npix % CM_P2 == 0;
  for (int i = 0; i < nlaser && pf; ++i) pf = ((uintptr_t)src_host[i] & 15) == 0;
  if (pf)
    channel_max_multi_pf_kernel<<<(unsigned)wg, 256, 0, (hipStream_t)stream>>>(J, npix);
  else
    channel_max_multi_kernel<<<(unsigned)wg, 256, sizeof(float) * CM_P * cmax, (hipStream_t)stream>>>(J, npix);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_calibrate_f64(const float *stack, int64_t npix, int32_t C, const float *cal, int64_t cal_sp,
                             int32_t cal_sc, int32_t cal_c0, int32_t cal_c1, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(C >= 1 && cal_sp >= 0 && cal_sc >= 0 && cal_c0 >= 0 && cal_c1 <= C, "calibrate: bad arguments");
  if (npix == 0) return HRF_OK;
  HRF_REQUIRE(stack && out, "calibrate: null buffer");
  calibrate_kernel<<<hrf::stream_grid(npix * C), 256, 0, (hipStream_t)stream>>>(stack, npix, C,
                                                                             Cal{cal, cal_sp, cal_sc, cal_c0, cal_c1},
                                                                             out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_and_u8(const uint8_t *a, const uint8_t *b, int64_t n, uint8_t *out, hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(a && b && out, "and_u8: null buffer");
  and_u8_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(a, b, n, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_mask_labels(const int32_t *labels, const uint8_t *mask, int64_t n, int32_t *out, hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(labels && mask && out, "mask_labels: null buffer");
  mask_labels_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(labels, mask, n, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

// *max_dev (an 8-byte device word) receives max(a) as a double
hrf_status hrf_max_f64(const double *a, int64_t n, double *max_dev, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(max_dev && n >= 1 && a, "max_f64: bad arguments");
  HRF_HIP(hipMemsetAsync(max_dev, 0, sizeof(double), s));
  max_f64_kernel<<<std::min<unsigned>(hrf::stream_grid(n), 512), 256, 0, s>>>(a, n, (unsigned long long *)max_dev);
  decode_max_kernel<<<1, 1, 0, s>>>((unsigned long long *)max_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_div_scalar_f64(const double *a, int64_t n, const double *divisor_dev, double *out,
                              hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(a && divisor_dev && out, "div_scalar: null buffer");
  div_scalar_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(a, n, divisor_dev, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_pad_edge_f64(const double *a, int64_t H, int64_t W, int32_t width, double *out, hrf_stream_t stream) {
  HRF_REQUIRE(width >= 0 && H >= 1 && W >= 1 && a && out, "pad_edge: bad arguments");
  pad_edge_kernel<<<hrf::stream_grid((H + 2 * width) * (W + 2 * width)), 256, 0, (hipStream_t)stream>>>(a, H, W, width,
                                                                                                        out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_pad_edge3_f64(const double *a, int64_t X, int64_t Y, int64_t Z, int32_t width, double *out,
                             hrf_stream_t stream) {
  HRF_REQUIRE(width >= 0 && X >= 1 && Y >= 1 && Z >= 1 && a && out, "pad_edge3: bad arguments");
  pad_edge3_kernel<<<hrf::stream_grid((X + 2 * width) * (Y + 2 * width) * (Z + 2 * width)), 256, 0,
                     (hipStream_t)stream>>>(a, X, Y, Z, width, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_mask_mul_f64(const double *a, const uint8_t *mask, int64_t n, double *out, hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(a && mask && out, "mask_mul: null buffer");
  mask_mul_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(a, mask, n, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
