// pixtable.hpp -- the per-pixel classifier's B operands as a table in HBM.
//
// classify_pixels_w16_kernel normalises and splits its pixels in a prologue (staging through LDS,
// one lane per pixel for the segment norms, hi/lo fp16 split).  The same arithmetic, done where
// the registered stack is produced (the E. coli assembly pass holds every 64-pixel strip in LDS
// anyway, stack.hip) or by a standalone pass, writes the operands in the exact register layout of
// the 16x16x32 MFMA B operand: per group of 16 pixels, per k-block t and hi/lo half, one 1 KiB
// block of 64 lanes x 16 B (lane = pixel (lane & 15), columns 32t + 8 (lane >> 4) .. + 7), so the
// classifier's prologue is 2 KT global_load_dwordx4 per group (classify.hip
// classify_pixels_w16t_kernel) and the sweep starts as soon as they land.  A flag byte per pixel
// carries its all-zero segments (bits 0..4) and "has a negative value" (bit 7).  Bit-identical to
// the in-kernel build: same f32 sums in channel order, same v_rsq, same f64 redo on underflow.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "detmath.h"

namespace hrf_pix {

struct LayEcoli {
  static constexpr int C = 95, NSEG = 5;
  static constexpr int PADB = 32;  // row pad bytes: 416-byte rows (see lay_sweep16's bank note)
  __host__ __device__ static constexpr int b(int s) {
    return s <= 0 ? 0 : s == 1 ? 32 : s == 2 ? 55 : s == 3 ? 75 : s == 4 ? 89 : 95;
  }
};
struct LayMulti {
  static constexpr int C = 63, NSEG = 4;
  static constexpr int PADB = 16;
  __host__ __device__ static constexpr int b(int s) { return s <= 0 ? 0 : s == 1 ? 23 : s == 2 ? 43 : s == 3 ? 57 : 63; }
};

template <class L>
__host__ __device__ constexpr int lay_seg(int c) {
  int s = 0;
  for (int t = 1; t < L::NSEG; ++t) s += c >= L::b(t) ? 1 : 0;
  return s;
}

template <class L>
constexpr int lay_kt() {
  return (L::C + 1 + 31) / 32;
}

// uint4 entries per 16-pixel group
template <class L>
constexpr int group_entries() {
  return lay_kt<L>() * 2 * 64;
}

// Pixels [0, np) of an LDS tile (pixel i at tile[i * C], np <= 64 and a multiple of 16 unless it
// ends the image) -> table entries of the 16-pixel groups g16_0 + i / 16, flags[p0 + i].  ok
// (nullable): pixels whose ok byte is 0 are taken as all-zero (the coverage mask).  The tile is
// normalised in place.  All threads of the block call it (256 threads).
template <class L>
__device__ __forceinline__ void prep_tile(float *tile, const uint8_t *ok, int np, int64_t p0, uint4 *__restrict__ table,
                                          uint8_t *__restrict__ flags) {
  constexpr int C = L::C, KT = lay_kt<L>();
  const int tid = threadIdx.x;
  if (tid < np) {
    float *px = tile + tid * C;
    const bool use = !ok || ok[tid];
    float nn[L::NSEG];
#pragma unroll
    for (int s = 0; s < L::NSEG; ++s) nn[s] = 0.0f;
    uint32_t sg = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float x = use ? px[c] : 0.0f;
      nn[lay_seg<L>(c)] = __builtin_fmaf(x, x, nn[lay_seg<L>(c)]);
      sg |= __float_as_uint(x);
    }
    float inv[L::NSEG];
    uint32_t zx = 0;
#pragma unroll
    for (int s = 0; s < L::NSEG; ++s) {
      inv[s] = rsqrtf(nn[s]);
      if (!(nn[s] >= 1e-30f)) {  // zero, or an f32 underflow: decide from the bits, redo in f64
        uint32_t nz = 0;
        double td = 0.0;
        for (int c = L::b(s); c < L::b(s + 1); ++c) {
          const float x = use ? px[c] : 0.0f;
          nz |= __float_as_uint(x) << 1;
          td += (double)x * (double)x;
        }
        inv[s] = nz ? (float)(1.0 / sqrt(td)) : 0.0f;
        zx |= (nz ? 0u : 1u) << s;
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) px[c] = use ? px[c] * inv[lay_seg<L>(c)] : 0.0f;
    flags[p0 + tid] = (uint8_t)(zx | ((sg >> 31) << 7));
  }
  __syncthreads();
  const int ne = (np + 15) / 16 * KT * 2 * 64;
  for (int e = tid; e < ne; e += 256) {
    const int lane = e & 63, hl = (e >> 6) & 1, gt = e >> 7;  // gt = g * KT + t
    const int g = gt / KT, t = gt - g * KT;
    const int i = 16 * g + (lane & 15), Q = lane >> 4;
    const float *pc = tile + (i < np ? i : 0) * C;
    union {
      _Float16 h[8];
      uint4 u;
    } o;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 32 * t + 8 * Q + q;
      float x = k < C ? pc[k] : (k == C ? 1.0f : 0.0f);
      if (i >= np) x = 0.0f;
      const _Float16 hv = (_Float16)x;
      o.h[q] = hl ? (_Float16)(x - (float)hv) : hv;
    }
    table[(p0 / 16 + g) * (int64_t)(KT * 2 * 64) + t * 128 + hl * 64 + lane] = o.u;
  }
}

// The same for the E. coli layout with the norm pass spread over the block's four waves (wave =
// a segment group, lane = pixel: segments 0 | 1 | 2 | 3 + 4, at most 32 channels per wave instead
// of 95 per lane): the assembly kernel calls this on its strip.  Same arithmetic per segment (the
// segments' sums are independent), so the table is bit-identical to prep_tile's.
// workgroup barrier ordering LDS only (s_barrier after the LDS counter drains): unlike
// __syncthreads it does not wait for the wave's global loads, so loads issued before it stay in
// flight across it (the E. coli assembly prefetches its next strip that way)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Caller contract: fl[0..63] is zero and the tile is staged (both ordered by a barrier before
// the call); the f64 channel sums the caller left in cns[0..np) (nullable) are turned into
// image_cn by wave 2 (log(s + 1e-2), cn_mode 1, or log10(s + 1), cn_mode 2) beside its segment.
template <bool LDSB = false>
__device__ __forceinline__ void prep_tile_ecoli(float *tile, const uint8_t *ok, int np, int64_t p0,
                                                uint4 *__restrict__ table, uint8_t *__restrict__ flags,
                                                uint32_t *fl /* LDS, 64 words, zero */, const double *cns,
                                                int cn_mode, double *__restrict__ cn_out) {
  using L = LayEcoli;
  constexpr int C = L::C, KT = lay_kt<L>();
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  auto seg = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (lane >= np) return;
    float *px = tile + lane * C;
    const bool use = !ok || ok[lane];
    float nn = 0.0f;
    uint32_t sg = 0;
#pragma unroll 4
    for (int c = L::b(s); c < L::b(s + 1); ++c) {
      const float x = use ? px[c] : 0.0f;
      nn = __builtin_fmaf(x, x, nn);
      sg |= __float_as_uint(x);
    }
    float inv = rsqrtf(nn);
    uint32_t zx = 0;
    if (!(nn >= 1e-30f)) {  // zero, or an f32 underflow: decide from the bits, redo in f64
      uint32_t nz = 0;
      double td = 0.0;
      for (int c = L::b(s); c < L::b(s + 1); ++c) {
        const float x = use ? px[c] : 0.0f;
        nz |= __float_as_uint(x) << 1;
        td += (double)x * (double)x;
      }
      inv = nz ? (float)(1.0 / sqrt(td)) : 0.0f;
      zx = nz ? 0u : (1u << s);
    }
#pragma unroll 4
    for (int c = L::b(s); c < L::b(s + 1); ++c) px[c] = use ? px[c] * inv : 0.0f;
    const uint32_t f = zx | ((sg >> 31) << 7);
    if (f) atomicOr(&fl[lane], f);
  };
  if (w == 0) seg(std::integral_constant<int, 0>{});
  else if (w == 1) seg(std::integral_constant<int, 1>{});
  else if (w == 2) {
    seg(std::integral_constant<int, 2>{});
    if (cns && lane < np) {
      double sv = 0.0 + cns[lane];
      if (cn_mode == 1) sv = hrf_cr_log(sv + 1e-2);
      else if (cn_mode == 2) sv = hrf_cr_log10(sv + 1.0);
      cn_out[p0 + lane] = sv;
    }
  } else {
    seg(std::integral_constant<int, 3>{});
    seg(std::integral_constant<int, 4>{});
  }
  if (LDSB) lds_barrier();
  else __syncthreads();
  if (tid < np) flags[p0 + tid] = (uint8_t)fl[tid];
  // one item = one (group, k-block, lane): its 8 values once, the hi and the lo entry from them
  const int ne = (np + 15) / 16 * KT * 64;
#pragma unroll 1
  for (int e = tid; e < ne; e += 256) {
    const int ln = e & 63, gt = e >> 6;
    const int g = gt / KT, t = gt - g * KT;
    const int i = 16 * g + (ln & 15), Q = ln >> 4;
    const float *pc = tile + (i < np ? i : 0) * C;
    union {
      _Float16 h[8];
      uint4 u;
    } hi, lo;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 32 * t + 8 * Q + q;
      float x = k < C ? pc[k] : (k == C ? 1.0f : 0.0f);
      if (i >= np) x = 0.0f;
      const _Float16 hv = (_Float16)x;
      hi.h[q] = hv;
      lo.h[q] = (_Float16)(x - (float)hv);
    }
    uint4 *dst = table + (p0 / 16 + g) * (int64_t)(KT * 2 * 64) + t * 128 + ln;
    dst[0] = hi.u;
    dst[64] = lo.u;
  }
}

}  // namespace hrf_pix
