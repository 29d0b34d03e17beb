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

// The same for the E. coli layout, in two phases the assembly kernel runs on its strip (round 5:
// the tile is read, never rewritten, so the norms share a barrier interval with the channel sums):
//  ecoli_norms: the segment norms spread over the block's four waves (wave = a segment group, lane
//    = pixel: segments 0 | 1 | 2 | 3 + 4), each pixel's reciprocal segment norms into invs[s * 64 +
//    pixel] and its flag bits into fl (zero on entry);
//  ecoli_table (after a barrier): the table entries, x = raw * inv of its segment.
// Same arithmetic per segment as prep_tile (f32 sums in channel order, v_rsq, the f64 redo, one f32
// multiply per value), so the table is bit-identical to prep_tile's.
__device__ __forceinline__ void ecoli_norms(const float *tile, const uint8_t *ok, int np, float *invs, uint32_t *fl) {
  using L = LayEcoli;
  constexpr int C = L::C;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  auto seg = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (lane >= np) return;
    const float *px = tile + lane * C;
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
    invs[s * 64 + lane] = inv;
    const uint32_t f = zx | ((sg >> 31) << 7);
    if (f) atomicOr(&fl[lane], f);
  };
  if (w == 0) seg(std::integral_constant<int, 0>{});
  else if (w == 1) seg(std::integral_constant<int, 1>{});
  else if (w == 2) seg(std::integral_constant<int, 2>{});
  else {
    seg(std::integral_constant<int, 3>{});
    seg(std::integral_constant<int, 4>{});
  }
}

// runtime segment of E. coli column k (k < 95) and its segment's end
__device__ __forceinline__ int ecoli_seg(int k) { return (k >= 32) + (k >= 55) + (k >= 75) + (k >= 89); }
__device__ __forceinline__ int ecoli_end(int s) { return s == 0 ? 32 : s == 1 ? 55 : s == 2 ? 75 : s == 3 ? 89 : 95; }

// One item per (group g, k-block t, lane): wave w takes the three (g, t) with 3g + t in {w, w + 4,
// w + 8} -- one per k-block, so t is a compile-time constant in each.
__device__ __forceinline__ void ecoli_table(const float *tile, const uint8_t *ok, int np, int64_t p0, const float *invs,
                                            uint4 *__restrict__ table) {
  constexpr int C = LayEcoli::C, KT = lay_kt<LayEcoli>();
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, Q = lane >> 4;
  const int ng = (np + 15) / 16;
#pragma unroll 1  // (unrolled, the three items' values spill at four waves per SIMD)
  for (int t = 0; t < KT; ++t) {
    const int j = ((t - w) % 3 + 3) % 3;
    const int g = (w + 4 * j - t) / 3;
    if (g >= ng) continue;
    const int i = 16 * g + (lane & 15);
    const int ii = i < np ? i : 0;
    const float *pc = tile + ii * C;
    const bool use = i < np && (!ok || ok[ii]);
    const int k0 = 32 * t + 8 * Q;
    const int sa = ecoli_seg(k0), sb = ecoli_seg(min(k0 + 7, C - 1));
    const float ia = invs[sa * 64 + ii], ib = invs[sb * 64 + ii];
    const int split = ecoli_end(sa) - k0;  // first q of segment sb
    union {
      _Float16 h[8];
      uint4 u;
    } hi, lo;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = k0 + q;
      float x;
      if (32 * t + 24 + q < C) {  // every lane quarter's column is a channel
        x = use ? pc[k] * (q < split ? ia : ib) : 0.0f;
      } else {
        x = k < C ? (use ? pc[k < C ? k : 0] * (q < split ? ia : ib) : 0.0f) : (k == C ? 1.0f : 0.0f);
        if (i >= np) x = 0.0f;
      }
      const _Float16 hv = (_Float16)x;
      hi.h[q] = hv;
      lo.h[q] = (_Float16)(x - (float)hv);
    }
    uint4 *dst = table + (p0 / 16 + g) * (int64_t)(KT * 2 * 64) + t * 128 + lane;
    dst[0] = hi.u;
    dst[64] = lo.u;
  }
}

}  // namespace hrf_pix
