// classify.hip -- segmented-cosine barcode classification (a19).
//
// Metric (train_reference.py channel_cosine_intensity :223-386 / _7b_v2 :993-1072): per
// excitation segment s, d_s = 1 - <x_s, y_s>/(|x_s||y_s|) (0 if both norms are 0, 1 if one
// is); the spectral distance is the mean over segments (gated variants below).
//
// Per pixel (north_star mode, ungated): argmin_r d(x, ref_r) = argmax_r sum_s cos'_s where
// cos'_s is the cosine of the segment-normalised vectors, plus 1 where both segments are
// zero.  Appending the S zero-segment indicators to both operands makes that ONE dense
// GEMM  score = Xext (P x K) . Refext^T (K x R),  K = C + S padded to KP:
//   * v_mfma_f32_32x32x2_f32 (exact f32 fmaf chain, 157 TF/s dense): fp32 because the
//     scores must match the f64 restatement to 1e-5;
//   * each wave keeps its 64 pixels' normalised spectra resident in VGPRs (B operand,
//     KP/2 registers per 32-pixel group) for the whole reference sweep; references stream
//     through LDS in 128-row chunks (A operand, ds_read_b64, conflict-free stride KP+2);
//   * MFMA k-slot h of step s holds channel h*KP/2 + s (a fixed permutation of the shared
//     reduction index), so each lane's operands are contiguous;
//   * the argmax over R is fused into the epilogue (each lane owns one pixel column and 16
//     reference rows of every 32x32 tile), so the P x R score matrix never exists.
// Per cell (reference semantics, gated by presence flags): f64, exact channel order of the
// restatement, one workgroup per cell -- bit-identical to oracle_segcos.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "common.hpp"
#include "pixtable.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int SMAX = 8;
struct Bounds {
  int32_t b[SMAX + 1];
  int32_t nseg;
};

constexpr int RCH = 64;  // references per LDS chunk (prefetched into registers)

// workgroups per CU the 16x16x32 sweeps (w16, w16t) are built for.  Round 6: 2 (256 VGPRs).  The
// runner-up tracking (t2, the refine's certificate) does not fit the 168 VGPRs of three: at three
// the E. coli table sweep reloaded B operands from scratch every chunk, 2.87 ms per 2048^2 tile
// against 1.77 ms at two (gpurun_out/r6b; round 5's three-per-CU kernel without t2: 1.69-1.81).
#ifndef HRF_W16T_OCC
#define HRF_W16T_OCC 2
#endif
// the table screen (hrf_classify_pixels_table): 16-pixel groups per wave and workgroups per CU
// The screens (hrf_classify_pixels_screen mode 2, hrf_classify_pixels_table): three 16-pixel groups
// per wave (72 B-operand VGPRs instead of 96) fit three workgroups per CU with the runner-up keys
// (165 VGPRs, no spills): 1.76-1.78 ms alone against 1.75 at four groups and two per CU, but
// 866 vs 842 Mpix/s in the bench (three interleaved pairs, profiles/r6_screen_ng3_ab.txt).  The
// fused certificate keeps four groups (64 pixels per wave) at two per CU.
#ifndef HRF_W16T_NG
#define HRF_W16T_NG 3
#endif
#ifndef HRF_W16T_SCREEN_OCC
#define HRF_W16T_SCREEN_OCC 3
#endif

// ==== exact per-pixel classification: the f64 refine of the screen (round 6) ==================
// The MFMA sweeps above are a SCREEN: split-fp16 (or f32-MFMA) scores within a bound of the exact
// segmented-cosine score.  Every sweep also reports, per pixel, an upper bound s2 on the device
// score of every library row other than its best row b1 (the runner-up, `second`).  The refine:
//  * rescores b1 in f64 exactly as the restatement does (oracle seg_dist / oracle_segcos variant
//    0: the three sums in channel order, 1 - d / sqrt(nx * ny), the segment mean) from the pixel's
//    f32 values -- the stack, or the five shifted acquisitions of a registered tile -- and the f32
//    library promoted to f64 (the restatement's ref64);
//  * certifies b1 when D(b1) < 1 - (s2 + eps) / nseg - 1e-12, eps the screen's proven error bound
//    (screen_eps below): then every other row r has S_exact(r) <= s2 + eps, i.e. its restated
//    distance exceeds D(b1), so b1 is the restatement's argmin and D(b1) its distance, bit for bit;
//  * answers an all-zero pixel from the library alone (every segment one-zero or both-zero:
//    D(r) = (nonzero segments of r) / nseg, its first argmin precomputed at prepare time);
//  * lists every other pixel (ties, near-ties, NaN / inf values) for refine_list_kernel, which
//    scores all rows in f32 with its own proven bound (fmaf chains on the raw values), keeps the
//    rows within twice that bound of the best, and rescores those in f64 -- lowest row on ties.
// The prepared library (refx) carries the exact section after its MFMA table: a header, the f32
// library row-major (pitch CP = C rounded to 4, float4 rows), channel-major (pitch RT = R rounded
// to 64, coalesced for the list kernel), the f64 segment sums of squares ny (the restatement's
// |y|^2) and f32 reciprocal segment norms iy.
struct ExactHdr {
  int32_t R, C, nseg, idx0;  // idx0 / D0: the all-zero pixel's argmin and distance
  double D0;
  int32_t tiny;              // some row has 0 < ny < 1e-30: the list kernel's f32 pass is not safe
  float zero[4];             // 0: what an uncovered pixel's channel reads (a load that needs no branch)
};
struct ExactLayout {
  int64_t off;  // section offset from the start of refx
  int32_t CP, RT;
  int64_t lib32, libT, ny, iy, total;  // offsets inside the section
};
inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }
int64_t table_rowb(int mode, int lay, int kp);
ExactLayout exact_layout(int mode, int lay, int kp, int rpad, int R, int C, int nseg) {
  ExactLayout e;
  const int64_t rowb = mode == 0 ? 4 * (int64_t)kp : table_rowb(mode, lay, kp);
  e.off = al256((int64_t)rpad * rowb);
  e.CP = (C + 3) & ~3;
  e.RT = (R + 63) & ~63;
  e.lib32 = 256;
  e.libT = al256(e.lib32 + (int64_t)R * e.CP * 4);
  e.ny = al256(e.libT + (int64_t)C * e.RT * 4);
  e.iy = al256(e.ny + (int64_t)R * nseg * 8);
  e.total = al256(e.iy + (int64_t)R * nseg * 4);
  return e;
}
struct ExactPtr {
  const float *lib32, *libT, *iy;
  const double *ny;
  int32_t CP, RT;
};

__global__ __launch_bounds__(256) void exact_prep_kernel(const float *__restrict__ ref, int32_t R, int32_t C,
                                                         Bounds bd, int32_t CP, int32_t RT, float *__restrict__ lib32,
                                                         float *__restrict__ libT, double *__restrict__ ny,
                                                         float *__restrict__ iy) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t e = t0; e < (int64_t)R * CP; e += stride) {
    const int64_t r = e / CP;
    const int c = (int)(e - r * CP);
    lib32[e] = c < C ? ref[r * C + c] : 0.0f;
  }
  for (int64_t e = t0; e < (int64_t)C * RT; e += stride) {
    const int64_t c = e / RT, r = e - c * RT;
    libT[e] = r < R ? ref[r * C + c] : 0.0f;
  }
  for (int64_t e = t0; e < (int64_t)R * bd.nseg; e += stride) {
    const int64_t r = e / bd.nseg;
    const int sg = (int)(e - r * bd.nseg);
    double v = 0.0;
    for (int i = bd.b[sg]; i < bd.b[sg + 1]; ++i) {
      const double y = (double)ref[r * C + i];
      v += y * y;
    }
    ny[e] = v;
    iy[e] = v > 0.0 ? (float)(1.0 / sqrt(v)) : 0.0f;
  }
}

// one thread: the all-zero pixel's answer (oracle_classify's loop on x = 0) and the tiny-row flag
__global__ void exact_hdr_kernel(const double *__restrict__ ny, int32_t R, int32_t C, int32_t nseg,
                                 ExactHdr *__restrict__ hdr) {
  double best = __builtin_inf();
  int32_t bi = 0, tiny = 0;
  for (int r = 0; r < R; ++r) {
    double sum = 0.0;
    for (int sg = 0; sg < nseg; ++sg) {
      const double v = ny[(int64_t)r * nseg + sg];
      sum += v == 0.0 ? 0.0 : 1.0;
      tiny |= (v > 0.0 && v < 1e-30) ? 1 : 0;
    }
    const double d = sum / nseg;
    if (d < best) {
      best = d;
      bi = r;
    }
  }
  hdr->R = R;
  hdr->C = C;
  hdr->nseg = nseg;
  hdr->idx0 = bi;
  hdr->D0 = best;
  hdr->tiny = tiny;
  for (int i = 0; i < 4; ++i) hdr->zero[i] = 0.0f;
}

// Pixel source: the registered value of pixel p (row r = p / W, column c = p % W) at channel k of
// laser q is src[q][((r - dr_q) W + (c - dc_q)) cl_q + (k - c0_q)], 0 outside the laser's frame and,
// with apply_mask, outside any laser's frame (register_assemble's stack; stack.hip).  A plain (P, C)
// stack is one laser with no shift.
constexpr int XLMAX = 8;
struct PixSrc {
  const float *src[XLMAX];
  int32_t c0[XLMAX + 1];
  uint64_t mdiv[XLMAX];  // ceil(2^32 / cl): e / cl = (e * mdiv) >> 32 for e < 2^32 / cl
  int32_t n;
  const int32_t *dsh;    // device (dr, dc) pairs, or null (no shift)
  int64_t H, W;
  int32_t apply_mask;
};

__device__ __forceinline__ bool src_covered(int64_t r, int64_t c, int64_t H, int64_t W, int dr, int dc) {
  return r >= (dr > 0 ? dr : 0) && r < H + (dr < 0 ? dr : 0) && c >= (dc > 0 ? dc : 0) && c < W + (dc < 0 ? dc : 0);
}

// element offsets (from src[q]) of pixel p's run in every laser, -1 where it reads as zero
__device__ __forceinline__ void src_offsets(const PixSrc &S, int64_t p, bool valid, int32_t (&off)[XLMAX]) {
  const int64_t r = p / S.W, c = p - r * S.W;
  bool ok = valid;
  if (S.apply_mask && S.dsh)
    for (int q = 0; q < S.n; ++q) ok = ok && src_covered(r, c, S.H, S.W, S.dsh[2 * q], S.dsh[2 * q + 1]);
#pragma unroll
  for (int q = 0; q < XLMAX; ++q) {
    off[q] = -1;
    if (q < S.n && ok) {
      const int dr = S.dsh ? S.dsh[2 * q] : 0, dc = S.dsh ? S.dsh[2 * q + 1] : 0;
      if (src_covered(r, c, S.H, S.W, dr, dc))
        off[q] = (int32_t)(((r - dr) * S.W + (c - dc)) * (int64_t)(S.c0[q + 1] - S.c0[q]));
    }
  }
}

// f64 restated distance of the pixel (f32 values x[0..C), stride 1) to a library row (yv: its f32
// values, float4-aligned, CP = C rounded to 4; nyr: its segment sums of squares): the
// restatement's seg_dist per segment in channel order, their sum, / nseg.  nz: the pixel's
// all-zero segments; in_range: every non-zero segment's sum of squares lies where the screen's f32
// normalisation is exact to its bound (no f32 overflow, no overflowing f64-redo reciprocal).
// NC > 0: the channel loop unrolled to NC (yv then indexes registers with constants); 0: a loop.
constexpr double NX_MIN = 1e-70, NX_MAX = 1e37;
template <int NC, class YV, class NY>
__device__ __forceinline__ double exact_dist_y(const float *x, YV yv, NY nyr, int C, const Bounds &bd, int *nz,
                                               bool *in_range) {
  double sum = 0.0;
  int zc = 0;
  bool rok = true;
  for (int sg = 0; sg < bd.nseg; ++sg) {
    const double ny = nyr(sg);  // issued before the segment's channels: its latency overlaps them
    double nx = 0.0, dd = 0.0;
    // 16 channels' loads issued together (clamped channel, the sum selected: a branch around the
    // sums would take the loads with it and wait for each), then their sums in channel order
    const int cb = bd.b[sg], ce = bd.b[sg + 1];
    for (int c0 = cb; c0 < ce; c0 += 16) {
      float xv[16], yy[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int c = min(c0 + u, ce - 1);
        xv[u] = x[c];
        yy[u] = yv(c);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const bool ok = c0 + u < ce;
        const double xd = (double)xv[u], yd = (double)yy[u];
        dd = ok ? dd + xd * yd : dd;
        nx = ok ? nx + xd * xd : nx;
      }
    }
    const double sd = (nx == 0.0 && ny == 0.0) ? 0.0 : ((nx == 0.0 || ny == 0.0) ? 1.0 : 1.0 - dd / sqrt(nx * ny));
    sum += sd;
    zc += nx == 0.0 ? 1 : 0;
    rok = rok && (nx == 0.0 || (nx >= NX_MIN && nx <= NX_MAX));
  }
  *nz = zc;
  if (in_range) *in_range = rok;
  return sum / bd.nseg;
}
__device__ __forceinline__ double exact_dist(const float *x, const ExactPtr &E, int r, int C, const Bounds &bd,
                                             int *nz, bool *in_range = nullptr) {
  const float *yr = E.lib32 + (int64_t)r * E.CP;
  const double *nyr = E.ny + (int64_t)r * bd.nseg;
  return exact_dist_y<0>(x, [&](int c) { return yr[c]; }, [&](int sg) { return nyr[sg]; }, C, bd, nz, in_range);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Everything the refine of a screen's output needs (kernel argument of the fused sweep)
struct RefineArgs {
  PixSrc S;
  ExactPtr E;
  const ExactHdr *hdr;
  double eps_base, eps_zero;
  int32_t *list, *cnt;
  Bounds bd;  // (kernel-argument memory: indexed by a runtime segment without a scratch copy)
};

// One wave refines the 64 consecutive pixels p0 .. p0 + 63 (lane = pixel: b1 = its screen row,
// sec2 = the runner-up bound).  The values and rows stream through the wave's LDS slice in chunks
// of RCK channels (lane = (pixel, channel) pairs, every load of a chunk in flight, stored as
// (x, y) pairs), and every lane carries its pixel's f64 sums across the chunks in channel order,
// so the slice stays small (more waves resident) and all 64 lanes do the f64 work.  Then the
// certificate: best_dist (and best_idx with write_idx) for a certified row, the header's answer
// for an all-zero pixel, the list otherwise.
// G chunks' loads are issued together (branch-free: clamped addresses, the value selected after
// the load), so a wave waits for memory once per G chunks rather than once per chunk.
#ifndef HRF_REFINE_WPE
#define HRF_REFINE_WPE 3  // refine_best_kernel: waves per SIMD the register budget allows
#endif
#ifndef HRF_REFINE_RCK
#define HRF_REFINE_RCK 16
#endif
constexpr int RCK = HRF_REFINE_RCK;  // channels per chunk
#ifndef HRF_REFINE_G
#define HRF_REFINE_G 2  // chunks whose loads are in flight together
#endif
__host__ __device__ constexpr int64_t refine_slice_bytes() {
  return (int64_t)64 * (4 * XLMAX + 4) + (int64_t)64 * (RCK + 1) * 8;
}
template <int G>
__device__ __forceinline__ void refine_pixels64(const RefineArgs &A, int C, const Bounds &bd, int64_t p0, int64_t P,
                                                int b1, float sec2, char *slice, int32_t *__restrict__ best_idx,
                                                float *__restrict__ best_dist, bool write_idx) {
  int32_t *offs = reinterpret_cast<int32_t *>(slice);                 // XLMAX x 64
  int32_t *b1s = offs + XLMAX * 64;                                   // 64
  float2 *xy = reinterpret_cast<float2 *>(b1s + 64);                  // 64 x (RCK + 1) (x, y)
  const PixSrc &S = A.S;
  const ExactPtr &E = A.E;
  const int lane = threadIdx.x & 63;
  const int64_t p = p0 + lane;
  const bool valid = p < P;
  const int Rr = A.hdr->R;
  const bool brow = b1 >= 0 && b1 < Rr;
  const int64_t brw = brow ? b1 : 0;
  // the row's segment sums of squares, every load in flight (clamped index, constant register index)
  double nyv[SMAX];
#pragma unroll
  for (int q = 0; q < SMAX; ++q) nyv[q] = E.ny[brw * bd.nseg + (q < bd.nseg ? q : 0)];
  {
    int32_t off[XLMAX];
    src_offsets(S, p, valid, off);
#pragma unroll
    for (int q = 0; q < XLMAX; ++q) offs[q * 64 + lane] = off[q];
    b1s[lane] = (int32_t)brw;
  }
  wave_lds_sync();
  // staging: element lane + 64 u of a chunk = pixel il + 4 u, channel k0 + kl
  const int kl = lane & (RCK - 1), il = lane / RCK;
  double nx = 0.0, dd = 0.0, sum = 0.0;
  int sg = 0, send = bd.b[1], zc = 0;
  bool rok = true;
  for (int k00 = 0; k00 < C; k00 += G * RCK) {
    float xv[G][RCK], yv[G][RCK];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int c = k00 + g * RCK + kl;
      const int ca = c < C ? c : C - 1;  // a readable channel for the padding lanes
      // this lane's laser for channel ca (uniform candidates, per-lane selects: no indexed registers)
      int qc = 0, cq = 0;
      const float *sp = S.src[0];
      for (int q = 1; q < S.n; ++q)
        if (ca >= S.c0[q]) {
          qc = q;
          sp = S.src[q];
          cq = S.c0[q];
        }
      int o[RCK], rb[RCK];
#pragma unroll
      for (int u = 0; u < RCK; ++u) {
        const int i = il + (64 / RCK) * u;
        o[u] = offs[qc * 64 + i];
        rb[u] = b1s[i];
      }
#pragma unroll
      for (int u = 0; u < RCK; ++u) {
        // unconditional loads (a selected address, not a selected value: the compiler would sink a
        // load whose value is selected into a branch and wait for it there); the padding lanes'
        // values are never read
        xv[g][u] = *(o[u] >= 0 ? sp + (o[u] + ca - cq) : A.hdr->zero);
        yv[g][u] = E.lib32[(int64_t)rb[u] * E.CP + ca];
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int k0 = k00 + g * RCK;
      if (k0 >= C) break;
#pragma unroll
      for (int u = 0; u < RCK; ++u) xy[(il + (64 / RCK) * u) * (RCK + 1) + kl] = make_float2(xv[g][u], yv[g][u]);
      wave_lds_sync();
      const float2 *row = xy + lane * (RCK + 1);
#pragma unroll
      for (int k = 0; k < RCK; ++k) {
        if (k0 + k >= C) break;
        const float2 v = row[k];
        const double xd = (double)v.x, yd = (double)v.y;
        dd += xd * yd;
        nx += xd * xd;
        if (k0 + k + 1 == send) {  // the segment's restated distance, in segment order
          double ny = nyv[0];
#pragma unroll
          for (int q = 1; q < SMAX; ++q) ny = sg == q ? nyv[q] : ny;
          const double sd = (nx == 0.0 && ny == 0.0) ? 0.0 : ((nx == 0.0 || ny == 0.0) ? 1.0 : 1.0 - dd / sqrt(nx * ny));
          sum += sd;
          zc += nx == 0.0 ? 1 : 0;
          rok = rok && (nx == 0.0 || (nx >= NX_MIN && nx <= NX_MAX));
          nx = dd = 0.0;
          ++sg;
          send = bd.b[sg + 1];
        }
      }
      wave_lds_sync();  // the chunk is consumed before the next one is staged
    }
  }
  const double D = sum / bd.nseg;
  bool listed = false;
  if (valid) {
    if (!brow) {  // no real row won the screen (cannot happen with R >= 1): list it
      listed = true;
    } else if (zc == bd.nseg) {  // all-zero pixel: the library's own answer
      best_idx[p] = A.hdr->idx0;
      best_dist[p] = (float)A.hdr->D0;
    } else if (!rok) {  // outside the screen bound's premises
      listed = true;
    } else {
      const double eps = A.eps_base + A.eps_zero * zc;
      const double lim = 1.0 - ((double)sec2 + eps) / bd.nseg - 1e-12;
      if (D < lim) {  // certified (NaN anywhere fails the compare)
        if (write_idx) best_idx[p] = b1;
        best_dist[p] = (float)D;
      } else {
        listed = true;
      }
    }
  }
  const unsigned long long m = __ballot(listed);
  if (m) {
    int base = 0;
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(A.cnt, __popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1, 64);
    if (listed) A.list[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)p;
  }
}



// refx[r][0..C) = ref / |ref_seg| (0 if the norm is 0), refx[r][C+s] = (norm_s == 0),
// zero padding to KP columns and to Rpad rows.
__global__ void ref_prep_kernel(const float *__restrict__ ref, int32_t R, int32_t C, Bounds bd, int32_t KP,
                                int32_t Rpad, float *__restrict__ refx) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= Rpad) return;
  float *o = refx + r * KP;
  for (int k = 0; k < KP; ++k) o[k] = 0.0f;
  if (r >= R) return;
  const float *x = ref + r * C;
  for (int s = 0; s < bd.nseg; ++s) {
    double nn = 0.0;
    for (int c = bd.b[s]; c < bd.b[s + 1]; ++c) nn += (double)x[c] * (double)x[c];
    const double inv = nn > 0 ? 1.0 / sqrt(nn) : 0.0;
    for (int c = bd.b[s]; c < bd.b[s + 1]; ++c) o[c] = (float)((double)x[c] * inv);
    o[C + s] = nn > 0 ? 0.0f : 1.0f;
  }
}

template <int KS>
__global__ __launch_bounds__(256) void classify_pixels_kernel(const float *__restrict__ stack, int64_t P, int32_t C,
                                                                  Bounds bd, const float *__restrict__ refx,
                                                                  int32_t R, int32_t Rpad,
                                                                  int32_t *__restrict__ best_idx,
                                                                  float *__restrict__ best_dist,
                                                                  float *__restrict__ second) {
  constexpr int KP = 2 * KS;
  constexpr int STRIDE = KP + 2;  // == 2 (mod 4): conflict-free ds_read_b64 over 32 rows
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * 256 + w * 64;

  // ---- stage this wave's two 32-pixel groups, build the B operand in registers ----
  float bx[2][KS];
  float *stg = lds + w * (32 * C);
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int64_t p0 = pbase + g * 32;
    const int64_t np = std::max<int64_t>(0, std::min<int64_t>(32, P - p0));
    const int64_t nel = np * C;
    const float *src = stack + p0 * C;
    for (int64_t e = lane; e < 32 * C; e += 64) stg[e] = e < nel ? src[e] : 0.0f;
    __syncthreads();
    // segment norms of pixel j (f64 accumulation, as the restatement)
    float inv[SMAX];
    float zf[SMAX];
#pragma unroll
    for (int s = 0; s < SMAX; ++s) {
      inv[s] = 0.0f;
      zf[s] = 0.0f;
      if (s < bd.nseg) {
        double nn = 0.0;
        for (int c = bd.b[s]; c < bd.b[s + 1]; ++c) {
          const double v = (double)stg[j * C + c];
          nn += v * v;
        }
        inv[s] = nn > 0 ? (float)(1.0 / sqrt(nn)) : 0.0f;
        zf[s] = nn > 0 ? 0.0f : 1.0f;
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = h * KS + s;
      float v = 0.0f;
      if (k < C) {
        float iv = inv[0];
#pragma unroll
        for (int q = 1; q < SMAX; ++q)
          if (q < bd.nseg && k >= bd.b[q]) iv = inv[q];
        v = (float)((double)stg[j * C + k] * (double)iv);
      } else if (k < C + bd.nseg) {
        float z = zf[0];
#pragma unroll
        for (int q = 1; q < SMAX; ++q)
          if (q == k - C) z = zf[q];
        v = z;
      }
      bx[g][s] = v;
    }
    __syncthreads();
  }

  float best[2] = {-__builtin_inff(), -__builtin_inff()};
  float sec[2] = {-__builtin_inff(), -__builtin_inff()};  // runner-up score (any row but the best)
  int bidx[2] = {0, 0};

  // ---- sweep the reference library in LDS chunks ----
  // The next chunk is prefetched into registers while the current one feeds the MFMAs, so
  // the L2 latency of the table hides behind ~25K MFMA cycles per chunk.
  constexpr int PF = (RCH * (KP / 2) + 255) / 256;  // float2 per thread per chunk
  float2 pf[PF];
  auto prefetch = [&](int r0) {
    const float2 *gsrc = reinterpret_cast<const float2 *>(refx + (int64_t)r0 * KP);
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int e = tid + q * 256;
      if (e < RCH * (KP / 2)) pf[q] = gsrc[e];
    }
  };
  prefetch(0);
  for (int r0 = 0; r0 < Rpad; r0 += RCH) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int e = tid + q * 256;
      if (e < RCH * (KP / 2)) {
        const int rr = e / (KP / 2), cc = e - rr * (KP / 2);
        reinterpret_cast<float2 *>(lds + rr * STRIDE)[cc] = pf[q];
      }
    }
    __syncthreads();
    if (r0 + RCH < Rpad) prefetch(r0 + RCH);
#pragma unroll 1
    for (int rb = 0; rb < RCH; rb += 32) {
      f32x16 acc0 = {0}, acc1 = {0};
      const float *arow = lds + (rb + j) * STRIDE + h * KS;
#pragma unroll
      for (int s = 0; s < KS; s += 2) {
        const float2 a = *reinterpret_cast<const float2 *>(arow + s);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bx[0][s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bx[1][s], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bx[0][s + 1], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bx[1][s + 1], acc1, 0, 0, 0);
      }
      // rows (references) of this lane: (reg&3) + 8*(reg>>2) + 4*h, increasing in reg
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int r = r0 + rb + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const bool ok = r < R;
        if (ok) {
          sec[0] = fmaxf(sec[0], fminf(best[0], acc0[reg]));
          sec[1] = fmaxf(sec[1], fminf(best[1], acc1[reg]));
        }
        if (ok && acc0[reg] > best[0]) {
          best[0] = acc0[reg];
          bidx[0] = r;
        }
        if (ok && acc1[reg] > best[1]) {
          best[1] = acc1[reg];
          bidx[1] = r;
        }
      }
    }
  }
  // merge the two lane halves holding the same pixel column
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const float ob = __shfl_xor(best[g], 32, 64);
    const int oi = __shfl_xor(bidx[g], 32, 64);
    sec[g] = fmaxf(fmaxf(sec[g], __shfl_xor(sec[g], 32, 64)), fminf(best[g], ob));
    if (ob > best[g] || (ob == best[g] && oi < bidx[g])) {
      best[g] = ob;
      bidx[g] = oi;
    }
    const int64_t p = pbase + g * 32 + j;
    if (h == 0 && p < P) {
      best_idx[p] = bidx[g];
      best_dist[p] = ((float)bd.nseg - best[g]) / (float)bd.nseg;
      if (second) second[p] = sec[g];
    }
  }
}

// ---- mode 1: split-fp16 MFMA ----------------------------------------------------------------
// Each normalised operand value v (|v| <= 1) is carried as hi = fp16(v) and lo = fp16(v - hi);
// score = sum(hi*hi' + hi*lo' + lo*hi') in one f32 accumulator.  Per product the error is the
// dropped lo*lo' (<= 2^-22) plus lo's fp16 rounding (<= 2^-25 absolute, subnormal spacing),
// so a 100-term score is within ~1e-6 of the exact f32 dot product; the three products are
// v_mfma_f32_32x32x16_f16 at 16x the f32-MFMA rate.
//
// Reference table rows (global AND LDS image): {hi[0..KP), lo[0..KP), 16 B pad} fp16, so the
// row pitch 4*KP+16 is 16 x odd (conflict-free ds_read_b128 over 32 rows) and a 64-row chunk
// is a whole number of 1 KiB LDS-DMA pieces.  Column C+nseg is a validity bias: 0 for real
// rows, -1024 for the padding rows past R, against 1.0 on the pixel side, so padding rows
// never win the argmax and the epilogue needs no bounds test.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

__global__ void ref_prep_f16_kernel(const float *__restrict__ ref, int32_t R, int32_t C, Bounds bd, int32_t KP,
                                    int32_t Rpad, _Float16 *__restrict__ refh) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= Rpad) return;
  _Float16 *hi = refh + r * (2 * KP + 8);
  _Float16 *lo = hi + KP;
  for (int k = 0; k < 2 * KP + 8; ++k) hi[k] = (_Float16)0.0f;
  hi[C + bd.nseg] = (_Float16)(r < R ? 0.0f : -1024.0f);
  if (r >= R) return;
  const float *x = ref + r * C;
  for (int s = 0; s < bd.nseg; ++s) {
    double nn = 0.0;
    for (int c = bd.b[s]; c < bd.b[s + 1]; ++c) nn += (double)x[c] * (double)x[c];
    const double inv = nn > 0 ? 1.0 / sqrt(nn) : 0.0;
    for (int c = bd.b[s]; c < bd.b[s + 1]; ++c) {
      const float v = (float)((double)x[c] * inv);
      const _Float16 h = (_Float16)v;
      hi[c] = h;
      lo[c] = (_Float16)(v - (float)h);
    }
    hi[C + s] = (_Float16)(nn > 0 ? 0.0f : 1.0f);
  }
}

// Raw spectra of one 32-pixel group: 32*C floats = 8*C float4, at most 16 per lane (C <= 128).
// All loads of both groups are issued before any is consumed, so a wave pays the HBM latency
// once per tile instead of once per element.
constexpr int LDV = 16;
__device__ __forceinline__ void load_group(const float *__restrict__ stack, int64_t P, int32_t C, int64_t p0, int lane,
                                           float4 (&v)[LDV], int npmax = 32) {
  const int64_t np = std::max<int64_t>(0, std::min<int64_t>(npmax, P - p0));
  const int64_t nel = np * C;  // valid floats of this group
  const float *src = stack + p0 * C;
  const int nv = 8 * C;
#pragma unroll
  for (int i = 0; i < LDV; ++i) {
    const int e4 = lane + 64 * i;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e4 < nv) {
      const int64_t e = 4 * (int64_t)e4;
      if (e + 4 <= nel) {
        x = *reinterpret_cast<const float4 *>(src + e);
      } else {
        x.x = e + 0 < nel ? src[e + 0] : 0.f;
        x.y = e + 1 < nel ? src[e + 1] : 0.f;
        x.z = e + 2 < nel ? src[e + 2] : 0.f;
        x.w = e + 3 < nel ? src[e + 3] : 0.f;
      }
    }
    v[i] = x;
  }
}

// Per-workgroup column map for the B operand: segk[k] = the slot of column k in a pixel's
// 24-float multiplier row {1/norm_s (0..7), zero-indicator_s (8..15), bias 1.0 (16), 0 (17)}.
constexpr int MROW = 24;
__device__ __forceinline__ void build_segk(const Bounds &bd, int32_t C, int KP, uint8_t *segk) {
  for (int k = threadIdx.x; k < KP; k += blockDim.x) {
    int v = 0x80 | 17;  // bit 7: not a channel (the value is the multiplier slot itself)
    if (k < C) {
      v = 0;
      for (int t = 1; t < bd.nseg; ++t) v += k >= bd.b[t];
    } else if (k < C + bd.nseg) {
      v = 0x80 | (8 + (k - C));
    } else if (k == C + bd.nseg) {
      v = 0x80 | 16;
    }
    segk[k] = (uint8_t)v;
  }
}

// Stage one loaded group in LDS and build its split-fp16 B operand (lane = pixel j, half h
// holds columns 16s + 8h + q): column k = raw[k] * mult[segk[k]] (raw = 1 past C), i.e. the
// channel scaled by its segment's 1/norm, then the zero-segment indicators, the bias column
// 1.0 and zeros.  The two half-waves of a pixel split each segment's channels for the norm.
template <int KS16>
__device__ __forceinline__ void build_b_f16(const float4 (&v)[LDV], int32_t C, const Bounds &bd, float *stg,
                                            float *mult, const uint8_t *segk, int lane, int j, int h,
                                            h8 (&bh)[KS16], h8 (&bl)[KS16]) {
  const int nv = 8 * C;
#pragma unroll
  for (int i = 0; i < LDV; ++i) {
    const int e4 = lane + 64 * i;
    if (e4 < nv) reinterpret_cast<float4 *>(stg)[e4] = v[i];
  }
  __syncthreads();
  const float *px = stg + j * C;
  float *mj = mult + j * MROW;
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    if (s < bd.nseg) {
      double n0 = 0.0, n1 = 0.0;
      const int c1 = bd.b[s + 1];
      int c = bd.b[s] + h;
      for (; c + 2 < c1; c += 4) {
        const double x0 = (double)px[c], x1 = (double)px[c + 2];
        n0 += x0 * x0;
        n1 += x1 * x1;
      }
      if (c < c1) {
        const double x0 = (double)px[c];
        n0 += x0 * x0;
      }
      double nn = n0 + n1;
      nn += __shfl_xor(nn, 32, 64);
      if (h == 0) {
        mj[s] = nn > 0 ? (float)(1.0 / sqrt(nn)) : 0.0f;
        mj[8 + s] = nn > 0 ? 0.0f : 1.0f;
      }
    }
  }
  if (h == 0) {
    mj[16] = 1.0f;
    mj[17] = 0.0f;
  }
  __syncthreads();
  // per-lane bases + immediate offsets; the raw read past C lands in LDS and is discarded
  const float *pc = px + 8 * h;
  const uint8_t *sk = segk + 8 * h;
#pragma unroll
  for (int s = 0; s < KS16; ++s) {
    h8 vh, vl;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      // the channel test comes from the column map (a load), not from k < C, which the
      // compiler would hoist out of the tile loop as 56 live masks
      const int code = sk[16 * s + q];
      const float m = mj[code & 31];
      float x = (code & 0x80) ? m : pc[16 * s + q] * m;
      asm volatile("" : "+v"(x));  // round to f32 first: no fused multiply-to-f16
      const _Float16 hv = (_Float16)x;
      vh[q] = hv;
      vl[q] = (_Float16)(x - (float)hv);
    }
    bh[s] = vh;
    bl[s] = vl;
  }
  __syncthreads();
}

// One workgroup = 4 waves x 64 pixels, held as split-fp16 B operands in VGPRs for the whole
// sweep.  The library streams through two LDS chunk buffers by LDS-DMA
// (global_load_lds_dwordx4, no VGPR staging): chunk c+1 is in flight while chunk c feeds the
// MFMAs, one barrier per chunk.  The argmax is fused (lane = pixel column, 16 rows per tile).
template <int KS16>
__global__ __launch_bounds__(256, 2) void classify_pixels_f16_kernel(const float *__restrict__ stack, int64_t P,
                                                                     int32_t C, Bounds bd,
                                                                     const _Float16 *__restrict__ refh, int32_t R,
                                                                     int32_t Rpad, int32_t *__restrict__ best_idx,
                                                                     float *__restrict__ best_dist,
                                                                     float *__restrict__ second) {
  constexpr int KP = 16 * KS16;
  constexpr int ROWB = 4 * KP + 16;
  constexpr int CHB = RCH * ROWB;
  constexpr int NPC = CHB / 1024;  // LDS-DMA pieces per chunk
  static_assert(CHB % 1024 == 0, "chunk must be whole 1 KiB pieces");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  char *ldsb = reinterpret_cast<char *>(lds);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * 256 + w * 64;

  h8 bh0[KS16], bl0[KS16], bh1[KS16], bl1[KS16];
  // staging aliases the chunk buffers (done before the first DMA): raw rows, multiplier rows,
  // column map
  float *stg = lds + w * (32 * C);
  float *mult = lds + 4 * 32 * C + w * (32 * MROW);
  uint8_t *segk = reinterpret_cast<uint8_t *>(lds + 4 * 32 * (C + MROW));
  build_segk(bd, C, KP, segk);
  {
    float4 v0[LDV], v1[LDV];
    load_group(stack, P, C, pbase, lane, v0);
    load_group(stack, P, C, pbase + 32, lane, v1);
    build_b_f16<KS16>(v0, C, bd, stg, mult, segk, lane, j, h, bh0, bl0);
    build_b_f16<KS16>(v1, C, bd, stg, mult, segk, lane, j, h, bh1, bl1);
  }

  const char *gref = reinterpret_cast<const char *>(refh);
  auto issue = [&](int c) {
    const char *g = gref + (int64_t)c * CHB + lane * 16;
    char *l = ldsb + (c & 1) * CHB;
    for (int q = w; q < NPC; q += 4)
      __builtin_amdgcn_global_load_lds((glb_void_t *)(g + q * 1024), (lds_void_t *)(l + q * 1024), 16, 0, 0);
  };
  issue(0);

  float best0 = -__builtin_inff(), best1 = -__builtin_inff();
  float sec0 = -__builtin_inff(), sec1 = -__builtin_inff();  // runner-up scores
  int bi0 = 0, bi1 = 0;  // wave-uniform part of the row index (4h added at the end)
  // Software-pipelined argmax: the scores of block b are compared while block b+1's MFMAs
  // run (a slice of the 16 registers after each k-step), so the epilogue's VALU fills the MFMA
  // issue gaps instead of following them.  Blocks are still consumed in increasing row order.
  f32x16 pv0, pv1;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) pv0[reg] = pv1[reg] = -__builtin_inff();
  int pr = 0;  // first row of the pending block
  auto epi = [&](int lo, int hi) {
#pragma unroll
    for (int reg = lo; reg < hi; ++reg) {
      const int r = pr + (reg & 3) + 8 * (reg >> 2);
      const float s0 = pv0[reg], s1 = pv1[reg];
      sec0 = fmaxf(sec0, fminf(best0, s0));
      sec1 = fmaxf(sec1, fminf(best1, s1));
      if (s0 > best0) {
        best0 = s0;
        bi0 = r;
      }
      if (s1 > best1) {
        best1 = s1;
        bi1 = r;
      }
    }
  };
  const int nch = Rpad / RCH;
  for (int c = 0; c < nch; ++c) {
    // chunk c landed: this wave's LDS-DMA retired (hipcc does not count global_load_lds for the
    // barrier's wait, so the vmcnt(0) is explicit), then the barrier covers every wave's pieces;
    // everyone is past chunk c-1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 1 < nch) issue(c + 1);
    const char *buf = ldsb + (c & 1) * CHB;
#pragma unroll
    for (int rb = 0; rb < RCH; rb += 32) {
      f32x16 acc0 = {0}, acc1 = {0};
      const char *row = buf + (rb + j) * ROWB + 16 * h;
#pragma unroll
      for (int s = 0; s < KS16; ++s) {
        const h8 ah = *reinterpret_cast<const h8 *>(row + 32 * s);
        const h8 al = *reinterpret_cast<const h8 *>(row + 2 * KP + 32 * s);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh0[s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh1[s], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl0[s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl1[s], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh0[s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh1[s], acc1, 0, 0, 0);
        epi((16 * s) / KS16, (16 * (s + 1)) / KS16);  // previous block, slice s
      }
      pv0 = acc0;
      pv1 = acc1;
      pr = c * RCH + rb;
    }
  }
  epi(0, 16);  // the last block
  float best[2] = {best0, best1};
  float sec[2] = {sec0, sec1};
  int bidx[2] = {bi0 + 4 * h, bi1 + 4 * h};
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const float ob = __shfl_xor(best[g], 32, 64);
    const int oi = __shfl_xor(bidx[g], 32, 64);
    sec[g] = fmaxf(fmaxf(sec[g], __shfl_xor(sec[g], 32, 64)), fminf(best[g], ob));
    if (ob > best[g] || (ob == best[g] && oi < bidx[g])) {
      best[g] = ob;
      bidx[g] = oi;
    }
    const int64_t p = pbase + g * 32 + j;
    if (h == 0 && p < P) {
      best_idx[p] = bidx[g];
      best_dist[p] = ((float)bd.nseg - best[g]) / (float)bd.nseg;
      if (second) second[p] = sec[g];
    }
  }
}

// ---- mode 2: split-fp16 MFMA on the reference channel layouts ---------------------------------
// The E. coli (95 channels, lasers 405/488/514/561/633: train_reference.py:1401) and
// synthetic-community (63 channels, 488/514/561/633: :1488) layouts as compile-time segment
// maps.  Every B-operand column's segment is then known at compile time, so the operand build
// is straight-line code (a select only where the two lane halves straddle a segment bound)
// with no LDS table lookups, and K = C + 1 (channels + the validity-bias column) instead of
// C + nseg + 1.  The zero-segment indicator terms (+1 for a segment that is zero in both the
// pixel and the reference row) are one extra hi-only k-step, run only by workgroups holding a
// pixel with an all-zero segment (workgroup-uniform branch to a second copy of the sweep): its
// A operand is the row's pad, which holds the row's indicators as fp16 1/0 (exact products, so
// the sum equals adding the integer count after the products); its B operand is the pixel's
// indicators.  95 -> 96 columns: 6 k-steps per 32-row block instead of 7, 19 MFMAs instead of
// 18 in the zero-segment copy.
using hrf_pix::LayEcoli;  // pixtable.hpp
using hrf_pix::LayMulti;

// segment of B-operand column k: 0..NSEG-1 for a channel, -1 for the bias column (k == C),
// -2 for zero padding
template <class L>
__host__ __device__ constexpr int col_seg(int k) {
  if (k > L::C) return -2;
  if (k == L::C) return -1;
  int s = 0;
  for (int t = 1; t < L::NSEG; ++t) s += k >= L::b(t) ? 1 : 0;
  return s;
}
template <class L>
constexpr int lay_ks16() {
  return (L::C + 1 + 15) / 16;
}

// Stage one loaded group in LDS and build its split-fp16 B operand (lane = pixel j, half h
// holds columns 16s + 8h + q).  Segment norms: f32 sums of the lane's own columns plus the
// other half's (one shuffle), 1/sqrt by v_rsq (both within ~1e-7 of the restatement's f64,
// far inside the classifier's 1e-5); a segment is zero when all its values are +-0 (exact,
// from the bit patterns), and a sum that underflows f32 is redone in f64.  zx = the pixel's
// all-zero segments; neg = some value is negative.
template <class L, int KS>
__device__ __forceinline__ void build_b_lay(const float4 (&v)[LDV], float *stg, int lane, int j, int h,
                                            h8 (&bh)[KS], h8 (&bl)[KS], uint32_t &zx, uint32_t &neg) {
  const int nv = 8 * L::C;
#pragma unroll
  for (int i = 0; i < LDV; ++i) {
    const int e4 = lane + 64 * i;
    if (e4 < nv) reinterpret_cast<float4 *>(stg)[e4] = v[i];
  }
  __syncthreads();
  const float *pc = stg + j * L::C + 8 * h;
  float raw[KS][8];
  float nn[L::NSEG];
  uint32_t nzs[L::NSEG];
  uint32_t sgn = 0;
#pragma unroll
  for (int s = 0; s < L::NSEG; ++s) {
    nn[s] = 0.0f;
    nzs[s] = 0u;
  }
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int sa = col_seg<L>(16 * s + q), sb = col_seg<L>(16 * s + 8 + q);
      const float r = pc[16 * s + q];  // past the row end: another pixel's value, masked here
      const float x = h ? (sb >= 0 ? r : 0.0f) : (sa >= 0 ? r : 0.0f);
      raw[s][q] = x;
      const uint32_t xb = __float_as_uint(x);
      sgn |= xb;
      const uint32_t mag = xb << 1;  // non-zero iff |x| != 0
      if (sa == sb) {
        if (sa >= 0) {
          nn[sa >= 0 ? sa : 0] = __builtin_fmaf(x, x, nn[sa >= 0 ? sa : 0]);
          nzs[sa >= 0 ? sa : 0] |= mag;
        }
      } else {
        const float x2 = x * x;
        if (sa >= 0) {
          nn[sa >= 0 ? sa : 0] += h ? 0.0f : x2;
          nzs[sa >= 0 ? sa : 0] |= h ? 0u : mag;
        }
        if (sb >= 0) {
          nn[sb >= 0 ? sb : 0] += h ? x2 : 0.0f;
          nzs[sb >= 0 ? sb : 0] |= h ? mag : 0u;
        }
      }
    }
  neg = sgn >> 31;
  float inv[L::NSEG];
  zx = 0;
#pragma unroll
  for (int s = 0; s < L::NSEG; ++s) {
    const float t = nn[s] + __shfl_xor(nn[s], 32, 64);
    const uint32_t nz = nzs[s] | __shfl_xor(nzs[s], 32, 64);
    inv[s] = nz ? rsqrtf(t) : 0.0f;
    zx |= (nz ? 0u : 1u) << s;
    if (nz && !(t >= 1e-30f)) {  // f32 underflow (|x| < ~1e-19 throughout): redo in f64
      double td = 0.0;
#pragma unroll
      for (int ss = 0; ss < KS; ++ss)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int sa = col_seg<L>(16 * ss + q), sb = col_seg<L>(16 * ss + 8 + q);
          const double x = (double)raw[ss][q];
          if ((h ? sb : sa) == s) td += x * x;
        }
      td += __shfl_xor(td, 32, 64);
      inv[s] = (float)(1.0 / sqrt(td));
    }
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    h8 vh, vl;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int sa = col_seg<L>(16 * s + q), sb = col_seg<L>(16 * s + 8 + q);
      const float ma = sa >= 0 ? inv[sa >= 0 ? sa : 0] : (sa == -1 ? 1.0f : 0.0f);
      const float mb = sb >= 0 ? inv[sb >= 0 ? sb : 0] : (sb == -1 ? 1.0f : 0.0f);
      float x;
      if (sa >= 0 && sb >= 0)
        x = raw[s][q] * (h ? mb : ma);
      else
        x = h ? (sb >= 0 ? raw[s][q] * mb : mb) : (sa >= 0 ? raw[s][q] * ma : ma);
      asm volatile("" : "+v"(x));  // round to f32 first: no fused multiply-to-f16
      const _Float16 hv = (_Float16)x;
      vh[q] = hv;
      vl[q] = (_Float16)(x - (float)hv);
    }
    bh[s] = vh;
    bl[s] = vl;
  }
  __syncthreads();
}

// The library sweep of one workgroup (see classify_pixels_f16_kernel).  ZS adds the
// zero-segment indicator terms popcount(zx & zr) to every score, as a seventh MFMA per pixel
// group and block: A = the row's indicator fp16s in its pad (every lane reads its row's pad;
// the h = 1 half meets B = 0), B = the pixel's indicators (h = 0 lanes, k < NSEG).  KEYED (all scores >= 0:
// no negative value in the workgroup's pixels or the library) runs the argmax on integer
// keys: score bits with the low 4 mantissa bits replaced by 15 - register (so the max also
// names the register, lower rows winning ties), a max tree per block and one compare per
// block -- about half the VALU of a compare-and-select per score.  The 4 dropped bits are
// <= 2^-19 relative (< 1e-5 of a distance): the keyed score IS the truncated one (it is the
// distance reported), and its argmax keeps the reference's tie rule on it -- within a block the
// code makes the lowest row win equal scores, across blocks (and chunks) only a strictly greater
// score replaces the running best, so equal scores anywhere in the library go to the lowest r.
// Runner-up tracking (the refine's certificate, hrf_classify_pixels_refine): the second-largest key
// of {a >= b} and k is med3(a, b, k) (v_med3_i32); a key's score bits with the 4 position bits set
// bound every untruncated score that truncates to them (negative keys -- padding rows only -- keep
// their truncated value, the larger one)
__device__ __forceinline__ int med3i(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }
__device__ __forceinline__ float key_score_hi(int k) {
  return __int_as_float(k >= 0 ? ((k & -16) | 15) : (k & -16));
}
// the same bound from a truncated score (keyed sweeps) or the exact one (compare-select sweeps)
__device__ __forceinline__ float score_hi(float s, bool keyed) { return keyed ? key_score_hi(__float_as_int(s)) : s; }

template <int KS16, int ROWB, int NW, int NSEG, bool ZS, bool KEYED>
__device__ __forceinline__ void lay_sweep(const char *__restrict__ gref, char *ldsb, int nch, int lane, int w, int h,
                                          const h8 (&bh0)[KS16], const h8 (&bl0)[KS16], const h8 (&bh1)[KS16],
                                          const h8 (&bl1)[KS16], uint32_t zx0, uint32_t zx1, float &best0,
                                          float &best1, int &bi0, int &bi1, float &sec0, float &sec1) {
  constexpr int KP = 16 * KS16;
  constexpr int CHB = RCH * ROWB;
  constexpr int NPC = CHB / 1024;
  const int j = lane & 31;
  auto issue = [&](int c) {
    const char *g = gref + (int64_t)c * CHB + lane * 16;
    char *l = ldsb + (c & 1) * CHB;
    for (int q = w; q < NPC; q += NW)
      __builtin_amdgcn_global_load_lds((glb_void_t *)(g + q * 1024), (lds_void_t *)(l + q * 1024), 16, 0, 0);
  };
  issue(0);
  f32x16 pv0, pv1;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) pv0[reg] = pv1[reg] = -__builtin_inff();
  int pr = 0;  // first row of the pending block
  h8 bz0, bz1;  // ZS: the pixels' zero-segment indicators (B operand of the extra k-step)
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bz0[q] = (_Float16)((h == 0 && q < NSEG && ((zx0 >> q) & 1u)) ? 1.0f : 0.0f);
    bz1[q] = (_Float16)((h == 0 && q < NSEG && ((zx1 >> q) & 1u)) ? 1.0f : 0.0f);
  }
  // KEYED: key = the best so far (a later block's best replaces it on a strictly greater score only);
  // t1 / t2 = the largest / second-largest keys seen (t1 doubles as the block's best, see sweep_w16)
  int key0 = INT32_MIN, key1 = INT32_MIN;
  int t10 = INT32_MIN, t11 = INT32_MIN, t20 = INT32_MIN, t21 = INT32_MIN;
  auto epi = [&](int lo, int hi) {
#pragma unroll
    for (int reg = lo; reg < hi; ++reg) {
      const int r = pr + (reg & 3) + 8 * (reg >> 2);
      const float s0 = pv0[reg], s1 = pv1[reg];
      if (KEYED) {
        const int q0 = (__float_as_int(s0) & -16) | (15 - reg), q1 = (__float_as_int(s1) & -16) | (15 - reg);
        t20 = med3i(t10, t20, q0);
        t21 = med3i(t11, t21, q1);
        t10 = max(t10, q0);
        t11 = max(t11, q1);
      } else {
        sec0 = fmaxf(sec0, fminf(best0, s0));
        sec1 = fmaxf(sec1, fminf(best1, s1));
        if (s0 > best0) {
          best0 = s0;
          bi0 = r;
        }
        if (s1 > best1) {
          best1 = s1;
          bi1 = r;
        }
      }
    }
    if (KEYED && hi == 16) {  // the pending block is complete: a later block wins on a greater score only
      if ((t10 >> 4) > (key0 >> 4)) {
        key0 = t10;
        bi0 = pr;
      }
      if ((t11 >> 4) > (key1 >> 4)) {
        key1 = t11;
        bi1 = pr;
      }
    }
  };
  for (int c = 0; c < nch; ++c) {
    // chunk c landed: this wave's LDS-DMA retired (hipcc does not count global_load_lds for the
    // barrier's wait, so the vmcnt(0) is explicit), then the barrier covers every wave's pieces;
    // everyone is past chunk c-1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 1 < nch) issue(c + 1);
    const char *buf = ldsb + (c & 1) * CHB;
#pragma unroll
    for (int rb = 0; rb < RCH; rb += 32) {
      f32x16 acc0 = {0}, acc1 = {0};
      const char *row = buf + (rb + j) * ROWB + 16 * h;
      h8 az;
      if (ZS) az = *reinterpret_cast<const h8 *>(buf + (rb + j) * ROWB + 4 * KP);
      // the cross products (hi * lo', lo * hi') first, then hi * hi': the small products meet an
      // accumulator of ~2^-10 of a score (screen_eps counts KS16 + 1 full-magnitude MFMAs)
#pragma unroll
      for (int s = 0; s < KS16; ++s) {
        const h8 ah = *reinterpret_cast<const h8 *>(row + 32 * s);
        const h8 al = *reinterpret_cast<const h8 *>(row + 2 * KP + 32 * s);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl0[s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl1[s], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh0[s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh1[s], acc1, 0, 0, 0);
        epi((16 * s) / KS16, (16 * (s + 1)) / KS16);  // previous block, slice s
      }
#pragma unroll
      for (int s = 0; s < KS16; ++s) {
        const h8 ah = *reinterpret_cast<const h8 *>(row + 32 * s);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh0[s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh1[s], acc1, 0, 0, 0);
      }
      if (ZS) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(az, bz0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(az, bz1, acc1, 0, 0, 0);
      }
      pv0 = acc0;
      pv1 = acc1;
      pr = c * RCH + rb;
    }
  }
  epi(0, 16);  // the last block
  if (KEYED) {
    const int g0 = 15 - (key0 & 15), g1 = 15 - (key1 & 15);
    bi0 += (g0 & 3) + 8 * (g0 >> 2);
    bi1 += (g1 & 3) + 8 * (g1 >> 2);
    best0 = __int_as_float(key0 & -16);
    best1 = __int_as_float(key1 & -16);
    sec0 = key_score_hi(t20);
    sec1 = key_score_hi(t21);
  }
}

template <class L, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void classify_pixels_lay_kernel(const float *__restrict__ stack, int64_t P,
                                                                     const _Float16 *__restrict__ refh, int32_t R,
                                                                     int32_t Rpad, int32_t *__restrict__ best_idx,
                                                                     float *__restrict__ best_dist,
                                                                     float *__restrict__ second) {
  constexpr int KS16 = lay_ks16<L>();
  constexpr int KP = 16 * KS16;
  constexpr int ROWB = 4 * KP + L::PADB;
  static_assert((RCH * ROWB) % 1024 == 0, "chunk must be whole 1 KiB pieces");
  static_assert(L::NSEG <= 6, "the pad holds 6 indicators (fp16 6-7 of row 0: the negative flag)");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * (64 * NW) + w * 64;

  h8 bh0[KS16], bl0[KS16], bh1[KS16], bl1[KS16];
  uint32_t zx0 = 0, zx1 = 0, ng0 = 0, ng1 = 0;
  float *stg = lds + w * (32 * L::C);  // staging aliases the chunk buffers (before the first DMA)
  {
    float4 v0[LDV], v1[LDV];
    load_group(stack, P, L::C, pbase, lane, v0);
    load_group(stack, P, L::C, pbase + 32, lane, v1);
    build_b_lay<L, KS16>(v0, stg, lane, j, h, bh0, bl0, zx0, ng0);
    build_b_lay<L, KS16>(v1, stg, lane, j, h, bh1, bl1, zx1, ng1);
  }
  // the library's "has a negative value" flag sits in row 0's pad (ref_negflag_kernel)
  const uint32_t libneg = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(refh) + 4 * KP + 12);
  float best0 = -__builtin_inff(), best1 = -__builtin_inff();
  float sec0 = -__builtin_inff(), sec1 = -__builtin_inff();
  int bi0 = 0, bi1 = 0;  // wave-uniform part of the row index (4h added at the end)
  const char *gref = reinterpret_cast<const char *>(refh);
  char *ldsb = reinterpret_cast<char *>(lds);
  const int nch = Rpad / RCH;
  // every wave of the workgroup takes the same branch (the chunk barriers are shared)
  const bool zs = __syncthreads_or((zx0 | zx1) != 0);
  const bool keyed = !libneg && !__syncthreads_or((ng0 | ng1) != 0);
#define HRF_SWEEP(Z, K) \
  lay_sweep<KS16, ROWB, NW, L::NSEG, Z, K>(gref, ldsb, nch, lane, w, h, bh0, bl0, bh1, bl1, zx0, zx1, best0, best1, bi0, \
                                           bi1, sec0, sec1)
  if (keyed) {
    if (zs) HRF_SWEEP(true, true);
    else HRF_SWEEP(false, true);
  } else {
    if (zs) HRF_SWEEP(true, false);
    else HRF_SWEEP(false, false);
  }
#undef HRF_SWEEP
  float best[2] = {best0, best1};
  float sec[2] = {sec0, sec1};
  int bidx[2] = {bi0 + 4 * h, bi1 + 4 * h};
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const float ob = __shfl_xor(best[g], 32, 64);
    const int oi = __shfl_xor(bidx[g], 32, 64);
    sec[g] = fmaxf(fmaxf(sec[g], __shfl_xor(sec[g], 32, 64)), fminf(score_hi(best[g], keyed), score_hi(ob, keyed)));
    if (ob > best[g] || (ob == best[g] && oi < bidx[g])) {
      best[g] = ob;
      bidx[g] = oi;
    }
    const int64_t p = pbase + g * 32 + j;
    if (h == 0 && p < P) {
      best_idx[p] = bidx[g];
      best_dist[p] = ((float)L::NSEG - best[g]) / (float)L::NSEG;
      if (second) second[p] = sec[g];
    }
  }
}

// ---- the same sweep on v_mfma_f32_16x16x32_f16 (E. coli layout) -------------------------------
// Same table, same split-fp16 products, same argmax rules; the MFMA shape differs: A = 16
// library rows x 32 columns (lane: row lane & 15, columns 32t + 8Q..+7, Q = lane >> 4), B = 32
// columns x 16 pixels (lane: pixel lane & 15, the same columns), C = 16 x 16 (lane: pixel lane &
// 15, rows 4Q..4Q+3).  A wave holds four 16-pixel groups.  At equal cycles per flop, this
// shape holds a higher clock than 32x32x16 under load (MI355X_MICROARCH.md, matrix-core DVFS).
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- round 3: the 16x16x32 sweep with a lane-per-pixel prologue and per-chunk argmax keys ----
// Same table, products, scores and tie rules as the 32x32x16 form; what changes against round 2's
// first 16x16x32 kernel (lay16, removed in round 5 after losing every A/B) is the instruction
// count around the MFMAs (lay16 issued ~2.3 VALU per MFMA over its life, which with two waves per
// SIMD left the matrix pipe idle ~40 % of the time):
//  * prologue: in the B-operand layout a lane's columns 32t + 8Q + q belong to a segment that
//    depends on the lane quarter Q, a runtime value, so lay16's operand build selected among all
//    NSEG segments for every value (~830 v_cndmask per wave).  Here the segment norms are taken by
//    one lane per staged pixel walking its C channels -- every channel's segment a compile-time
//    constant -- and the pixel is normalised in place in LDS; the B-operand lanes then only read
//    and split into hi/lo fp16;
//  * sweep: the argmax folds each block's 16 keys into a per-chunk key with v_max3 and compares
//    with the running best once per chunk (the key's low 4 bits name the row within the chunk:
//    4 * block + register, blocks of 16 rows, CR <= 64), instead of a compare-and-select per
//    block;
//  * NW waves per workgroup share CR-row chunks through NBUF LDS buffers (template parameters;
//    the defaults are the measured best, DESIGN.md "Per-pixel classifier").
using hrf_pix::lay_seg;

// One staged 32-pixel group (row-major, stride C floats, at stg): lanes 0..31 (pixel = lane)
// take the segment norms, flag all-zero segments (zx) and negative values (neg), and rewrite
// the pixel normalised.  Same arithmetic as build_b_lay (f32 sums, v_rsq, f64 redo when a sum
// underflows f32), summed in channel order.
template <class L>
__device__ __forceinline__ void norm_pixels_w16(float *stg, int lane, uint32_t &zx, uint32_t &neg) {
  zx = 0;
  neg = 0;
  if (lane < 32) {
    float *px = stg + lane * L::C;
    float nn[L::NSEG];
#pragma unroll
    for (int s = 0; s < L::NSEG; ++s) nn[s] = 0.0f;
    uint32_t sg = 0;
#pragma unroll
    for (int c = 0; c < L::C; ++c) {
      const float x = px[c];
      nn[lay_seg<L>(c)] = __builtin_fmaf(x, x, nn[lay_seg<L>(c)]);
      sg |= __float_as_uint(x);
    }
    neg = sg >> 31;
    float inv[L::NSEG];
#pragma unroll
    for (int s = 0; s < L::NSEG; ++s) {
      inv[s] = rsqrtf(nn[s]);
      if (!(nn[s] >= 1e-30f)) {  // zero, or an f32 underflow: decide from the bits, redo in f64
        uint32_t nz = 0;
        double td = 0.0;
        for (int c = L::b(s); c < L::b(s + 1); ++c) {
          const float x = px[c];
          nz |= __float_as_uint(x) << 1;
          td += (double)x * (double)x;
        }
        inv[s] = nz ? (float)(1.0 / sqrt(td)) : 0.0f;
        zx |= (nz ? 0u : 1u) << s;
      }
    }
#pragma unroll
    for (int c = 0; c < L::C; ++c) px[c] = px[c] * inv[lay_seg<L>(c)];
  }
}

// B operand of 16-pixel sub-group g of the normalised staged group: lane pixel (lane & 15) + 16g,
// columns 32t + 8Q + q; column C is the validity-bias column (1), columns past it 0.
template <class L, int KT>
__device__ __forceinline__ void split_b_w16(const float *stg, int lane, int g, h8 (&bh)[KT], h8 (&bl)[KT]) {
  const int jj = (lane & 15) + 16 * g, Q = lane >> 4;
  const float *pc = stg + jj * L::C + 8 * Q;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    h8 vh, vl;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float x = pc[32 * t + q];  // past the row end: another pixel's value, replaced below
      if (32 * t + 24 + q >= L::C) {  // only the last columns depend on Q
        const int k = 32 * t + 8 * Q + q;
        x = k < L::C ? x : (k == L::C ? 1.0f : 0.0f);
      }
      const _Float16 hv = (_Float16)x;
      vh[q] = hv;
      vl[q] = (_Float16)(x - (float)hv);
    }
    bh[t] = vh;
    bl[t] = vl;
  }
}

template <int KT, int ROWB, int NW, int NSEG, bool ZS, bool KEYED, int NBUF, int CR, bool PIPE, int NG = 4>
__device__ __forceinline__ void sweep_w16(const char *__restrict__ gref, char *ldsb, int nch, int lane, int w,
                                          const h8 (&bh)[NG][KT], const h8 (&bl)[NG][KT], const uint32_t zxp,
                                          float (&best)[NG], int (&bi)[NG], float (&sec)[NG]) {
  static_assert(NG >= 1 && NG <= 4, "16-pixel groups per wave: 8 bits of zxp / bic each");
  constexpr int KP = 32 * KT;
  constexpr int CHB = CR * ROWB;
  constexpr int NPC = (CHB + 1023) / 1024;  // 1 KiB LDS-DMA pieces per chunk (the last may be partial)
  constexpr int NB = CR / 16;               // 16-row blocks per chunk
  static_assert(CR % 16 == 0 && NB <= 4, "chunk keys hold 4 * block + register in 4 bits");
  const int rl = lane & 15, Q = lane >> 4;
  auto issue = [&](int c) {
    const char *g = gref + (int64_t)c * CHB + lane * 16;
    char *l = ldsb + (c % NBUF) * CHB;
    for (int q = w; q < NPC; q += NW)
      if (CHB % 1024 == 0 || q * 1024 + lane * 16 < CHB)
        __builtin_amdgcn_global_load_lds((glb_void_t *)(g + q * 1024), (lds_void_t *)(l + q * 1024), 16, 0, 0);
  };
  // pieces this wave issues per chunk (the waitcnt below leaves chunk c + 1's outstanding)
  const int mine = (NPC - w + NW - 1) / NW;
  constexpr int MINE_LO = NPC / NW;
  issue(0);
  if (NBUF >= 3 && nch > 1) issue(1);
  f32x4 pv[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[g][i] = -__builtin_inff();
  int pr = 0;  // first row of the pending block
  // ZS: the pixels' indicator B operand (fp16 1.0 = 0x3c00 in slot q < NSEG of quarter 0 where
  // segment q is all zero), rebuilt per use from zxp (group g's all-zero segments in bits 8g..8g+7)
  // instead of held in 16 VGPRs
  auto bz_of = [&](int g) -> h8 {
    const uint32_t m = Q == 0 ? ((zxp >> (8 * g)) & ((1u << NSEG) - 1u)) : 0u;
    uint32_t d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = (((m >> (2 * i)) & 1u) * 0x3c00u) | (((m >> (2 * i + 1)) & 1u) * 0x3c000000u);
    return __builtin_bit_cast(h8, d);
  };
  // keyed: key = the running best (replaced by a chunk's best only on a strictly greater score),
  // t1 / t2 = the largest and second-largest keys seen (t1 also serves as the chunk's best: a key
  // from an earlier chunk that was not adopted has key's score)
  int key[NG], t1[NG], t2[NG];
  uint32_t bic = 0;  // keyed: the chunk of each group's key, 8 bits per group
#pragma unroll
  for (int g = 0; g < NG; ++g) key[g] = t1[g] = t2[g] = INT32_MIN;
  // fold the pending block into the chunk keys, groups [g0, g1); after the chunk's last block,
  // the chunk key against the running best (strictly greater score, the position code left out:
  // earlier chunks win ties, so equal scores keep the lowest row across the whole library)
  auto epi = [&](int g0, int g1) {
    const int pb = (pr / 16) % NB;
#pragma unroll
    for (int g = g0; g < g1; ++g) {
      if (KEYED) {
        const int base = 15 - 4 * pb;
        const int k0 = (__float_as_int(pv[g][0]) & -16) | (base - 0);
        const int k1 = (__float_as_int(pv[g][1]) & -16) | (base - 1);
        const int k2 = (__float_as_int(pv[g][2]) & -16) | (base - 2);
        const int k3 = (__float_as_int(pv[g][3]) & -16) | (base - 3);
        t2[g] = med3i(t1[g], t2[g], k0);
        t1[g] = max(t1[g], k0);
        t2[g] = med3i(t1[g], t2[g], k1);
        t1[g] = max(t1[g], k1);
        t2[g] = med3i(t1[g], t2[g], k2);
        t1[g] = max(t1[g], k2);
        t2[g] = med3i(t1[g], t2[g], k3);
        t1[g] = max(t1[g], k3);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) sec[g] = fmaxf(sec[g], fminf(best[g], pv[g][i]));
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (pv[g][i] > best[g]) {
            best[g] = pv[g][i];
            bi[g] = pr + i;
          }
      }
    }
    if (KEYED && g1 == NG && pb == NB - 1) {
      const uint32_t cc = (uint32_t)(pr / CR);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if ((t1[g] >> 4) > (key[g] >> 4)) {  // t1 is then this chunk's
          key[g] = t1[g];
          bic = (bic & ~(0xffu << (8 * g))) | (cc << (8 * g));
        }
      }
    }
  };
  for (int c = 0; c < nch; ++c) {
    if (NBUF == 2 || c + 1 >= nch) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (mine > MINE_LO) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MINE_LO + 1) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MINE_LO) : "memory");
    if (NW > 1) __syncthreads();  // every wave's pieces of c landed; everyone is past chunk c - 1
    if (c + NBUF - 1 < nch) issue(c + NBUF - 1);
    const char *buf = ldsb + (c % NBUF) * CHB;
#pragma unroll
    for (int rb = 0; rb < CR; rb += 16) {
      f32x4 acc[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char *row = buf + (rb + rl) * ROWB + 16 * Q;
      h8 az;
      if (ZS) az = *reinterpret_cast<const h8 *>(buf + (rb + rl) * ROWB + 4 * KP);
      // the cross products (hi * lo', lo * hi', each ~2^-11 of a score) first, then the hi * hi'
      // products: the accumulator the small products meet stays ~2^-10 of a score, so only KT
      // (+ the indicator step) MFMAs per score round at the score's magnitude (screen_eps)
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const h8 ah = *reinterpret_cast<const h8 *>(row + 64 * t);
        const h8 al = *reinterpret_cast<const h8 *>(row + 2 * KP + 64 * t);
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[g][t], acc[g], 0, 0, 0);
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[g][t], acc[g], 0, 0, 0);
        if (PIPE) epi((NG * t) / KT, (NG * (t + 1)) / KT);  // previous block, slice t
      }
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const h8 ah = *reinterpret_cast<const h8 *>(row + 64 * t);
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[g][t], acc[g], 0, 0, 0);
      }
      if (ZS) {
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(az, bz_of(g), acc[g], 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < NG; ++g) pv[g] = acc[g];
      pr = c * CR + rb;
      if (!PIPE) epi(0, NG);  // this block at once (the other waves on the SIMD cover the MFMA latency)
    }
  }
  if (PIPE) epi(0, NG);  // the last block (the end of the last chunk: finalises its key)
  if (KEYED) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int code = 15 - (key[g] & 15);
      bi[g] = CR * (int)((bic >> (8 * g)) & 0xffu) + 16 * (code >> 2) + (code & 3);
      best[g] = __int_as_float(key[g] & -16);
      sec[g] = key_score_hi(t2[g]);
    }
  }
}

template <class L, int NW, int NBUF, int CR, int OCC, int NG = 4>
__global__ __launch_bounds__(64 * NW, OCC) void classify_pixels_w16_kernel(const float *__restrict__ stack,
                                                                     int64_t P, const _Float16 *__restrict__ refh,
                                                                     int32_t R, int32_t Rpad,
                                                                     int32_t *__restrict__ best_idx,
                                                                     float *__restrict__ best_dist,
                                                                     float *__restrict__ second) {
  constexpr int KT = (L::C + 1 + 31) / 32;
  constexpr int KP = 32 * KT;
  constexpr int ROWB = 4 * KP + L::PADB;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  static_assert(NG == 3 || NG == 4, "a wave holds 3 or 4 16-pixel groups");
  const int64_t pbase = (int64_t)blockIdx.x * (16 * NG * NW) + w * (16 * NG);
  h8 bh[NG][KT], bl[NG][KT];
  uint32_t zxp = 0, ng = 0;  // all-zero segments of the NG 16-pixel groups, 8 bits each
  float *stg = lds + w * (32 * L::C);  // staging aliases the chunk buffers (before the first DMA)
  {
    // both halves' loads in flight at once where the registers allow (two waves per SIMD);
    // at three, the second half is loaded after the first is staged
    constexpr int NV = OCC < 3 ? 2 : 1;
    float4 v[NV][LDV];
    // (NG = 3: the second half is one 16-pixel group; the rest of its staging reads as zero)
    load_group(stack, P, L::C, pbase, lane, v[0]);
    if (NV == 2) load_group(stack, P, L::C, pbase + 32, lane, v[NV - 1], 16 * (NG - 2));
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (NV == 1 && half == 1) load_group(stack, P, L::C, pbase + 32, lane, v[0], 16 * (NG - 2));
#pragma unroll
      for (int i = 0; i < LDV; ++i) {
        const int e4 = lane + 64 * i;
        if (e4 < 8 * L::C) reinterpret_cast<float4 *>(stg)[e4] = v[NV == 2 ? half : 0][i];
      }
      __syncthreads();
      uint32_t zxh, ngp;
      norm_pixels_w16<L>(stg, lane, zxh, ngp);
      ng |= ngp;
      __syncthreads();
      split_b_w16<L, KT>(stg, lane, 0, bh[2 * half], bl[2 * half]);
      if (2 * half + 1 < NG) split_b_w16<L, KT>(stg, lane, 1, bh[(2 * half + 1) % NG], bl[(2 * half + 1) % NG]);
      zxp |= (uint32_t)__shfl(zxh, lane & 15, 64) << (16 * half);
      if (2 * half + 1 < NG) zxp |= (uint32_t)__shfl(zxh, 16 + (lane & 15), 64) << (16 * half + 8);
      __syncthreads();
    }
  }
  const uint32_t libneg = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(refh) + 4 * KP + 12);
  float best[NG], sec[NG];
  int bi[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    best[g] = sec[g] = -__builtin_inff();
    bi[g] = 0;
  }
  const char *gref = reinterpret_cast<const char *>(refh);
  char *ldsb = reinterpret_cast<char *>(lds);
  const int nch = Rpad / CR;
  const bool zs = __syncthreads_or(zxp != 0);
  const bool keyed = !libneg && !__syncthreads_or(ng != 0);
#define HRF_SWEEPW(Z, K) \
  sweep_w16<KT, ROWB, NW, L::NSEG, Z, K, NBUF, CR, (OCC < 3), NG>(gref, ldsb, nch, lane, w, bh, bl, zxp, best, bi, sec)
  if (keyed) {
    if (zs) HRF_SWEEPW(true, true);
    else HRF_SWEEPW(false, true);
  } else {
    if (zs) HRF_SWEEPW(true, false);
    else HRF_SWEEPW(false, false);
  }
#undef HRF_SWEEPW
  const int Q = lane >> 4;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    float b = best[g], sc = sec[g];
    int idx = bi[g] + 4 * Q;
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ob = __shfl_xor(b, o, 64);
      const int oi = __shfl_xor(idx, o, 64);
      sc = fmaxf(fmaxf(sc, __shfl_xor(sc, o, 64)), fminf(score_hi(b, keyed), score_hi(ob, keyed)));
      if (ob > b || (ob == b && oi < idx)) {
        b = ob;
        idx = oi;
      }
    }
    const int64_t p = pbase + 16 * g + (lane & 15);
    if (Q == 0 && p < P) {
      best_idx[p] = idx;
      best_dist[p] = ((float)L::NSEG - b) / (float)L::NSEG;
      if (second) second[p] = sc;
    }
  }
}

// ---- the B operands from a pixel table (pixtable.hpp) ------------------------------------------
// Standalone producer: 64 pixels per workgroup staged through LDS (coalesced float4 loads).
template <class L>
__global__ __launch_bounds__(256) void pixtable_prep_kernel(const float *__restrict__ stack, int64_t P,
                                                            uint4 *__restrict__ table, uint8_t *__restrict__ flags) {
  __shared__ __attribute__((aligned(16))) float tile[64 * L::C];
  const int64_t p0 = (int64_t)blockIdx.x * 64;
  const int np = (int)min((int64_t)64, P - p0);
  const int nel = np * L::C;
  const float *src = stack + p0 * L::C;
  for (int e = threadIdx.x; e < (nel >> 2); e += 256)
    reinterpret_cast<float4 *>(tile)[e] = reinterpret_cast<const float4 *>(src)[e];
  for (int e = ((nel >> 2) << 2) + threadIdx.x; e < nel; e += 256) tile[e] = src[e];
  __syncthreads();
  hrf_pix::prep_tile<L>(tile, nullptr, np, p0, table, flags);
}

// classify_pixels_w16_kernel with the prologue replaced by direct loads of the prepared operands.
// FUSE (round 6): the f64 refine follows the sweep in the same workgroup (refine_pixels on the
// freed chunk buffers, each wave its four 16-pixel groups), so its loads and f64 work overlap the
// other resident workgroup's MFMA sweep, and the screen's rows and bounds never leave registers.
template <class L, int NW, int NBUF, int CR, int OCC, bool FUSE, int NG = 4>
__global__ __launch_bounds__(64 * NW, OCC) void classify_pixels_w16t_kernel(const uint4 *__restrict__ table,
                                                                      const uint8_t *__restrict__ flags, int64_t P,
                                                                      const _Float16 *__restrict__ refh, int32_t R,
                                                                      int32_t Rpad, int32_t *__restrict__ best_idx,
                                                                      float *__restrict__ best_dist,
                                                                      float *__restrict__ second, RefineArgs A) {
  constexpr int KT = (L::C + 1 + 31) / 32;
  constexpr int KP = 32 * KT;
  constexpr int ROWB = 4 * KP + L::PADB;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  static_assert(!FUSE || NG == 4, "the fused refine takes 64 pixels per wave");
  const int64_t pbase = (int64_t)blockIdx.x * (16 * NG * NW) + w * (16 * NG);
  h8 bh[NG][KT], bl[NG][KT];
  uint32_t zxp = 0, ng = 0;  // all-zero segments of the NG 16-pixel groups, 8 bits each
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int64_t g16 = pbase / 16 + g;
    const uint4 *e = table + g16 * (int64_t)(KT * 128) + lane;
    // (NG < 4: the table holds whole 256-pixel blocks, a 16 NG NW-pixel workgroup can pass them)
    const bool gv = NG == 4 || 16 * g16 < P;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const uint4 hv = gv ? e[t * 128] : uint4{0, 0, 0, 0}, lv = gv ? e[t * 128 + 64] : uint4{0, 0, 0, 0};
      bh[g][t] = *reinterpret_cast<const h8 *>(&hv);
      bl[g][t] = *reinterpret_cast<const h8 *>(&lv);
    }
    const int64_t p = pbase + 16 * g + (lane & 15);
    const uint32_t f = p < P ? flags[p] : 0x1fu;
    zxp |= (f & 0x1fu) << (8 * g);
    ng |= f >> 7;
  }
  const uint32_t libneg = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(refh) + 4 * KP + 12);
  float best[NG], sec[NG];
  int bi[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    best[g] = sec[g] = -__builtin_inff();
    bi[g] = 0;
  }
  const char *gref = reinterpret_cast<const char *>(refh);
  char *ldsb = reinterpret_cast<char *>(lds);
  const int nch = Rpad / CR;
  const bool zs = __syncthreads_or(zxp != 0);
  const bool keyed = !libneg && !__syncthreads_or(ng != 0);
#define HRF_SWEEPW(Z, K) \
  sweep_w16<KT, ROWB, NW, L::NSEG, Z, K, NBUF, CR, (OCC < 3), NG>(gref, ldsb, nch, lane, w, bh, bl, zxp, best, bi, sec)
  if (keyed) {
    if (zs) HRF_SWEEPW(true, true);
    else HRF_SWEEPW(false, true);
  } else {
    if (zs) HRF_SWEEPW(true, false);
    else HRF_SWEEPW(false, false);
  }
#undef HRF_SWEEPW
  const int Q = lane >> 4;
  int b1g[NG];
  float s2g[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    float b = best[g], sc = sec[g];
    int idx = bi[g] + 4 * Q;
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ob = __shfl_xor(b, o, 64);
      const int oi = __shfl_xor(idx, o, 64);
      sc = fmaxf(fmaxf(sc, __shfl_xor(sc, o, 64)), fminf(score_hi(b, keyed), score_hi(ob, keyed)));
      if (ob > b || (ob == b && oi < idx)) {
        b = ob;
        idx = oi;
      }
    }
    b1g[g] = idx;  // every quarter lane holds pixel (lane & 15) + 16 g's merged result
    s2g[g] = sc;
    const int64_t p = pbase + 16 * g + (lane & 15);
    if (!FUSE && Q == 0 && p < P) {
      best_idx[p] = idx;
      best_dist[p] = ((float)L::NSEG - b) / (float)L::NSEG;
      if (second) second[p] = sc;
    }
  }
  if constexpr (FUSE) {
    __syncthreads();  // every wave is done with the chunk buffers: they become the refine's slices
    constexpr int64_t SL = (refine_slice_bytes() + 15) / 16 * 16;
    char *slice = ldsb + w * SL;
    // lane l holds pixel pbase + l's merged result in quarter Q = l >> 4's slot
    const int b1 = Q == 0 ? b1g[0] : Q == 1 ? b1g[1 % NG] : Q == 2 ? b1g[2 % NG] : b1g[3 % NG];
    const float s2 = Q == 0 ? s2g[0] : Q == 1 ? s2g[1 % NG] : Q == 2 ? s2g[2 % NG] : s2g[3 % NG];
    refine_pixels64<HRF_REFINE_G>(A, L::C, A.bd, pbase, P, b1, s2, slice, best_idx, best_dist, true);
  }
}

// mode-2 table: {hi[KP], lo[KP], pad 16 B} fp16 per row, KP = 16 * ceil((C + 1) / 16); column C
// is the validity bias (0 real rows, -1024 padding rows); pad fp16 s (s < nseg) = 1 when the row's
// segment s is all zero (the indicator k-step's A operand), fp16 6-7 of row 0 = the library's
// negative-value flag.
__global__ void ref_prep_lay_kernel(const float *__restrict__ ref, int32_t R, int32_t C, Bounds bd, int32_t KP,
                                    int32_t Rpad, int32_t rowh, _Float16 *__restrict__ refh) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= Rpad) return;
  _Float16 *hi = refh + r * rowh;
  _Float16 *lo = hi + KP;
  for (int k = 0; k < rowh; ++k) hi[k] = (_Float16)0.0f;
  hi[C] = (_Float16)(r < R ? 0.0f : -1024.0f);
  if (r >= R) return;
  const float *x = ref + r * C;
  for (int s = 0; s < bd.nseg; ++s) {
    double nn = 0.0;
    for (int c = bd.b[s]; c < bd.b[s + 1]; ++c) nn += (double)x[c] * (double)x[c];
    const double inv = nn > 0 ? 1.0 / sqrt(nn) : 0.0;
    for (int c = bd.b[s]; c < bd.b[s + 1]; ++c) {
      const float v = (float)((double)x[c] * inv);
      const _Float16 h = (_Float16)v;
      hi[c] = h;
      lo[c] = (_Float16)(v - (float)h);
    }
    if (!(nn > 0)) hi[2 * KP + s] = (_Float16)1.0f;
  }
}

// row 0's last pad word (byte 4*KP + 12) = 1 when any library value is negative (the keyed argmax
// needs every score >= 0); one workgroup, after ref_prep_lay_kernel
__global__ __launch_bounds__(256) void ref_negflag_kernel(const float *__restrict__ ref, int64_t n, int32_t KP,
                                                          _Float16 *__restrict__ refh) {
  int neg = 0;
  for (int64_t i = threadIdx.x; i < n; i += 256) neg |= ref[i] < 0.0f;
  neg = __syncthreads_or(neg);
  if (threadIdx.x == 0) *reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(refh) + 4 * KP + 12) = (uint32_t)neg;
}

// presence flags of the gated metrics: out[n][s] = 1.0 when max over segment s of row n > thr (a NaN
// in the segment makes the max NaN, and the comparison false), else 0.0
__global__ __launch_bounds__(256) void segment_flags_kernel(const double *__restrict__ x, int64_t N, int32_t C,
                                                            Bounds bd, double thr, double *__restrict__ out,
                                                            const int32_t *__restrict__ n_dev) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n_dev) N = min(N, (int64_t)*n_dev);
  if (i >= N * bd.nseg) return;
  const int64_t n = i / bd.nseg;
  const int sg = (int)(i - n * bd.nseg);
  bool any = false, nan = false;
  for (int c = bd.b[sg]; c < bd.b[sg + 1]; ++c) {
    const double v = x[n * C + c];
    any |= v > thr;
    nan |= v != v;
  }
  out[i] = (any && !nan) ? 1.0 : 0.0;
}

// 1 = E. coli layout, 2 = synthetic-community layout, 0 = other
template <class L>
bool is_layout(const Bounds &bd, int C) {
  if (C != L::C || bd.nseg != L::NSEG) return false;
  for (int s = 0; s <= L::NSEG; ++s)
    if (bd.b[s] != L::b(s)) return false;
  return true;
}
int layout_id(const Bounds &bd, int C) {
  if (is_layout<LayEcoli>(bd, C)) return 1;
  if (is_layout<LayMulti>(bd, C)) return 2;
  return 0;
}
// bytes per row of a mode-1/2 table: hi | lo | pad (the reference layouts' pads differ)
int64_t table_rowb(int mode, int lay, int kp) {
  if (mode == 2 && lay == 1) return 4 * kp + LayEcoli::PADB;
  if (mode == 2 && lay == 2) return 4 * kp + LayMulti::PADB;
  return 4 * kp + 16;
}

// ---- per cell, f64, gated variants ----
// The library is read channel-major (refT[c * R + r], transposed once per call), so the threads of
// a workgroup -- one library row each -- read consecutive addresses per channel: coalesced,
// instead of 64 cache lines per load with row-major rows.  A segment's distance is
// 1 - x.y / sqrt(|x|^2 |y|^2) with the three sums in channel order (0 when both are zero, 1 when
// one is), the restatement's seg_dist.

// library prep for the blocked kernel: refT = channel-major library (t[c * R + r]) and ny[r * S + s]
// = the segment's sum of squares in channel order (the restatement's |y|^2, bit for bit)
__global__ void cells_lib_prep_kernel(const double *__restrict__ a, int32_t R, int32_t C, Bounds bd,
                                      double *__restrict__ t, double *__restrict__ ny) {
  const int64_t n = (int64_t)R * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / C, c = e - r * C;
    t[c * R + r] = a[e];
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)R * bd.nseg;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / bd.nseg;
    const int sg = (int)(e - r * bd.nseg);
    double v = 0;
    for (int i = bd.b[sg]; i < bd.b[sg + 1]; ++i) {
      const double y = a[r * C + i];
      v += y * y;
    }
    ny[e] = v;
  }
}

// CB cells per workgroup: each library value read from L2 feeds CB cells, and only the dot
// products run per (cell, row) -- the segment norms are taken once, the cells' in the workgroup
// (nx) and the library's by cells_lib_prep_kernel (ny), in channel order, so every distance is the
// restatement's bit for bit (round 1's one-workgroup-per-cell kernel, removed in round 5, computed
// the same values).  Rows are visited in increasing order per thread and ties go to the smaller row.
template <int CB, int NT>
__global__ __launch_bounds__(NT) void classify_cells_blk_kernel(const double *__restrict__ X, int64_t N,
                                                                 const double *__restrict__ refT,
                                                                 const double *__restrict__ ny, int32_t R, int32_t C,
                                                                 Bounds bd, int32_t variant,
                                                                 const double *__restrict__ fx,
                                                                 const double *__restrict__ fr,
                                                                 int32_t *__restrict__ arg, double *__restrict__ dmin,
                                                                 const int32_t *__restrict__ n_dev) {
  extern __shared__ double xs[];  // CB x C
  __shared__ double snx[CB][SMAX];
  __shared__ double sfx[CB][SMAX];
  __shared__ double sbest[NT];
  __shared__ int sidx[NT];
  const int tid = threadIdx.x;
  const int S = bd.nseg;
  const int64_t nmax = n_dev ? min(N, (int64_t)*n_dev) : N;
  const int64_t n0 = (int64_t)blockIdx.x * CB;
  if (n0 >= nmax) return;
  const int nc = (int)min((int64_t)CB, nmax - n0);
  for (int e = tid; e < CB * C; e += NT) {
    const int j = e / C;
    xs[e] = j < nc ? X[(n0 + j) * C + (e - j * C)] : 0.0;
  }
  __syncthreads();
  if (tid < CB * S) {
    const int j = tid / S, sg = tid - j * S;
    double v = 0;
    for (int i = bd.b[sg]; i < bd.b[sg + 1]; ++i) {
      const double x = xs[j * C + i];
      v += x * x;
    }
    snx[j][sg] = v;
    sfx[j][sg] = (variant && j < nc) ? fx[(n0 + j) * S + sg] : 0.0;
  }
  __syncthreads();
  double best[CB];
  int bi[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    best[j] = __builtin_inf();
    bi[j] = 0x7fffffff;
  }
  for (int r = tid; r < R; r += NT) {
    double sd[CB][SMAX];
    for (int sg = 0; sg < S; ++sg) {
      double d[CB];
#pragma unroll
      for (int j = 0; j < CB; ++j) d[j] = 0;
      // the segment's library values in batches of 8 independent loads (the L2 latency of one
      // load per iteration otherwise serialises the walk), accumulated in channel order
      const int lo = bd.b[sg], hi = bd.b[sg + 1];
      for (int i0 = lo; i0 < hi; i0 += 8) {
        double yv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) yv[u] = i0 + u < hi ? refT[(int64_t)(i0 + u) * R + r] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i0 + u < hi)
#pragma unroll
            for (int j = 0; j < CB; ++j) d[j] += xs[j * C + i0 + u] * yv[u];
      }
      const double yy = ny[(int64_t)r * S + sg];
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const double xx = snx[j][sg];
        sd[j][sg] = (xx == 0.0 && yy == 0.0) ? 0.0 : ((xx == 0.0 || yy == 0.0) ? 1.0 : 1.0 - d[j] / sqrt(xx * yy));
      }
    }
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      double dist;
      if (variant == 0) {
        double sum = 0;
        for (int k = 0; k < S; ++k) sum += sd[j][k];
        dist = sum / S;
      } else {
        double chk = 0;
        for (int k = 0; k < S; ++k) chk += fabs(sfx[j][k] - fr[(int64_t)r * S + k]);
        if (chk < 0.01) {
          double sum = 0;
          for (int k = 0; k < S; ++k) sum += sfx[j][k] == 0 ? 0.0 : sd[j][k];
          dist = variant == 1 ? sum / S : 0.5 * sum / S;
        } else if (variant == 2) {
          dist = 1.0;
        } else {
          double sum = 0;
          for (int k = 0; k < S; ++k) sum += sd[j][k];
          dist = sum / S;
        }
      }
      if (dist < best[j]) {
        best[j] = dist;
        bi[j] = r;
      }
    }
  }
  for (int j = 0; j < nc; ++j) {
    sbest[tid] = best[j];
    sidx[tid] = bi[j];
    __syncthreads();
    for (int o = NT / 2; o > 0; o >>= 1) {
      if (tid < o) {
        const double b2 = sbest[tid + o];
        const int i2 = sidx[tid + o];
        if (b2 < sbest[tid] || (b2 == sbest[tid] && i2 < sidx[tid])) {
          sbest[tid] = b2;
          sidx[tid] = i2;
        }
      }
      __syncthreads();
    }
    if (tid == 0) {
      arg[n0 + j] = sidx[0] == 0x7fffffff ? 0 : sidx[0];
      dmin[n0 + j] = sbest[0];
    }
    __syncthreads();
  }
}

constexpr int CELLS_CB = 4;    // cells per workgroup of the blocked kernel
constexpr int CELLS_NT = 1024; // threads (library rows in flight) per workgroup

int choose_ks(int K) {
  static const int ks[] = {8, 16, 18, 24, 32, 34, 40, 50, 56, 64};
  for (int v : ks)
    if (2 * v >= K) return v;
  return -1;
}

template <class L, int NW, int NB, int CR, int OCC, int NG>
hrf_status launch_w16_lay(const float *stack, int64_t P, const void *refx, int32_t R, int32_t rpad, int32_t *best_idx,
                          float *best_dist, float *second, hipStream_t s) {
  constexpr int KT = (L::C + 1 + 31) / 32;
  const size_t shm = std::max<size_t>((size_t)NB * CR * (128 * KT + L::PADB), sizeof(float) * NW * 32 * L::C);
  HRF_REQUIRE(shm * OCC <= 160 * 1024 + 1024, "classify: w16 configuration exceeds the LDS");
  (void)hipFuncSetAttribute((const void *)classify_pixels_w16_kernel<L, NW, NB, CR, OCC, NG>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  classify_pixels_w16_kernel<L, NW, NB, CR, OCC, NG><<<(unsigned)hrf::cdiv(P, 16 * NG * NW), 64 * NW, shm, s>>>(
      stack, P, (const _Float16 *)refx, R, rpad, best_idx, best_dist, second);
  return HRF_OK;
}

hrf_status make_bounds(const int32_t *bounds_host, int32_t nseg, int32_t C, Bounds *bd) {
  HRF_REQUIRE(nseg >= 1 && nseg <= SMAX && bounds_host, "classify: 1..8 segments required");
  HRF_REQUIRE(bounds_host[0] == 0 && bounds_host[nseg] == C, "classify: segment bounds must span [0, C)");
  for (int s = 0; s < nseg; ++s) HRF_REQUIRE(bounds_host[s] < bounds_host[s + 1], "classify: empty segment");
  for (int s = 0; s <= SMAX; ++s) bd->b[s] = s <= nseg ? bounds_host[s] : C;
  bd->nseg = nseg;
  return HRF_OK;
}

// The unfused refine: one wave = 64 consecutive pixels of a screen's output (refine_pixels64).
__global__ __launch_bounds__(64, HRF_REFINE_WPE) void refine_best_kernel(RefineArgs A, int64_t P, int32_t C, Bounds bd,
                                                         const float *__restrict__ second,
                                                         int32_t *__restrict__ best_idx,
                                                         float *__restrict__ best_dist) {
  extern __shared__ __attribute__((aligned(16))) char rslice[];
  const int lane = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * 64, p = p0 + lane;
  const bool valid = p < P;
  const int b1 = valid ? best_idx[p] : 0;
  const float sec2 = valid ? second[p] : 0.0f;
  refine_pixels64<HRF_REFINE_G>(A, C, bd, p0, P, b1, sec2, rslice, best_idx, best_dist, false);
}

// Listed pixels, in batches of LIST_NP per workgroup (grid-strided over the device count), so
// each library value read from L2 serves LIST_NP pixels:
//  1. the batch's values (32 threads per pixel, lane = channel) and finiteness; per pixel and
//     segment the f64 sum of squares nx (channel order) and the f32 reciprocal norm ix;
//  2. every row's f32 score for every pixel of the batch (thread = 4 rows): per segment an fmaf
//     chain of the raw products d, cos = d * ix * iy (both-zero 1, one-zero 0), summed in f32; its
//     error is at most eps32 (screen_eps) -- so only rows within 2 eps32 of a pixel's best f32
//     score can be its restated argmin;
//  3. those rows (every row for a pixel with non-finite values or norms out of the f32 pass's
//     range) rescored exactly (exact_dist), minimum with the lowest row on ties, as
//     oracle_classify's first-minimum loop.
#ifndef HRF_LIST_LV
#define HRF_LIST_LV 4  // list pass: channels whose library loads are in flight together
#endif
constexpr int LIST_NP = 8;     // pixels per batch (stage 1 maps 32 threads per pixel)
constexpr int LIST_NT = 256;   // threads per workgroup
constexpr int LIST_RMAX = 4096;
static_assert(LIST_NP * 32 == LIST_NT, "stage 1 loads one pixel per 32 threads");
__global__ __launch_bounds__(LIST_NT) void refine_list_kernel(PixSrc S, int32_t C, Bounds bd, ExactPtr E,
                                                              const ExactHdr *__restrict__ hdr, int32_t R,
                                                              double eps32, const int32_t *__restrict__ list,
                                                              const int32_t *__restrict__ cnt,
                                                              int32_t *__restrict__ stats,
                                                              int32_t *__restrict__ best_idx,
                                                              float *__restrict__ best_dist) {
  __shared__ float xb[LIST_NP][128];
  __shared__ float ixb[LIST_NP][SMAX];
  __shared__ int fullb[LIST_NP];
  __shared__ float thrb[LIST_NP];
  __shared__ double redd[LIST_NT / 64][LIST_NP];
  __shared__ int redr[LIST_NT / 64][LIST_NP];
  constexpr int CAND = 1024;  // sparse candidates per batch; a pixel that overflows is scored in full
  __shared__ int32_t cand[CAND];
  __shared__ int ncand;
  extern __shared__ float scb[];  // LIST_NP x RT f32 scores
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = *cnt;
  const int nseg = bd.nseg;
  for (int64_t b0 = (int64_t)blockIdx.x * LIST_NP; b0 < n; b0 += (int64_t)gridDim.x * LIST_NP) {
    const int nb = (int)min((int64_t)LIST_NP, n - b0);
    // 1. values: pixel j = t / 32, channels (t & 31) + 32 m
    {
      const int j = t >> 5, k0 = t & 31;
      bool bad = false;
      if (j < nb) {
        const int64_t p = list[b0 + j];
        int32_t off[XLMAX];
        src_offsets(S, p, true, off);
        for (int k = k0; k < C; k += 32) {
          int q = 0;
          for (int qq = 1; qq < S.n; ++qq) q = k >= S.c0[qq] ? qq : q;
          const float v = off[q] >= 0 ? S.src[q][off[q] + k - S.c0[q]] : 0.0f;
          xb[j][k] = v;
          bad = bad || !__builtin_isfinite(v);
        }
      }
      if (t < LIST_NP) fullb[t] = hdr->tiny;
      __syncthreads();
      if (bad) atomicOr(&fullb[j], 1);
    }
    if (t < nb * nseg) {
      const int j = t / nseg, sg = t - j * nseg;
      double v = 0.0;
      for (int i = bd.b[sg]; i < bd.b[sg + 1]; ++i) {
        const double xd = (double)xb[j][i];
        v += xd * xd;
      }
      ixb[j][sg] = v > 0.0 ? (float)(1.0 / sqrt(v)) : 0.0f;
      if (v > 0.0 && (v < 1e-30 || v > 1e30)) atomicOr(&fullb[j], 1);
    }
    __syncthreads();
    // 2. f32 scores, thread = rows r0 + t + 256 u
    for (int r0 = 0; r0 < E.RT; r0 += 4 * LIST_NT) {
      float sc[LIST_NP][4];
#pragma unroll
      for (int j = 0; j < LIST_NP; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) sc[j][u] = 0.0f;
      for (int sg = 0; sg < nseg; ++sg) {
        float d[LIST_NP][4];
#pragma unroll
        for (int j = 0; j < LIST_NP; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u) d[j][u] = 0.0f;
        // LV channels' loads in flight together (clamped addresses, no branch around a load; rows
        // past RT are never stored), then their fmaf chains in channel order
        constexpr int LV = HRF_LIST_LV;
        const int ce = bd.b[sg + 1];
        for (int i0 = bd.b[sg]; i0 < ce; i0 += LV) {
          float y[LV][4];
#pragma unroll
          for (int v = 0; v < LV; ++v) {
            const int i = min(i0 + v, ce - 1);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int r = min(r0 + t + LIST_NT * u, E.RT - 1);
              y[v][u] = E.libT[(int64_t)i * E.RT + r];
            }
          }
#pragma unroll
          for (int v = 0; v < LV; ++v) {
            const bool ok = i0 + v < ce;  // (a select, not a branch: a branch would take the loads with it)
            const int i = ok ? i0 + v : i0;
#pragma unroll
            for (int j = 0; j < LIST_NP; ++j) {
              const float x = xb[j][i];
#pragma unroll
              for (int u = 0; u < 4; ++u) d[j][u] = ok ? __builtin_fmaf(x, y[v][u], d[j][u]) : d[j][u];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = r0 + t + LIST_NT * u;
          const float iyv = r < R ? E.iy[(int64_t)r * nseg + sg] : 0.0f;
#pragma unroll
          for (int j = 0; j < LIST_NP; ++j) {
            const float ix = ixb[j][sg];
            const float c = ix == 0.0f ? (iyv == 0.0f ? 1.0f : 0.0f) : (iyv == 0.0f ? 0.0f : (d[j][u] * ix) * iyv);
            sc[j][u] += c;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + t + LIST_NT * u;
        if (r < E.RT)
#pragma unroll
          for (int j = 0; j < LIST_NP; ++j) scb[j * E.RT + r] = r < R ? sc[j][u] : -__builtin_inff();
      }
    }
    __syncthreads();
    // per pixel: the best f32 score -> the candidate threshold (wave w takes pixels w, w + 4)
    for (int j = w; j < nb; j += LIST_NT / 64) {
      float mx = -__builtin_inff();
      for (int r = lane; r < R; r += 64) mx = fmaxf(mx, scb[j * E.RT + r]);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      if (lane == 0) {
        float th = mx - (float)(2.0 * eps32) * 1.0001f;
        thrb[j] = th - fabsf(th) * 1e-6f;  // the subtraction's own rounding, generously
      }
    }
    __syncthreads();
    // 3. exact distances: the candidates of the other pixels compacted into one list shared by
    //    all threads (a handful per pixel), every row of the full-path pixels; per pixel the
    //    minimum, lowest row on ties, whatever order the rows were visited in
    if (t == 0) ncand = 0;
    __syncthreads();
    for (int j = 0; j < nb; ++j) {
      if (fullb[j]) continue;
      const float th = thrb[j];
      for (int r = t; r < R; r += LIST_NT)
        if (scb[j * E.RT + r] >= th) {
          const int k = atomicAdd(&ncand, 1);
          if (k < CAND) cand[k] = (j << 16) | r;
          else atomicOr(&fullb[j], 2);
        }
    }
    __syncthreads();
    double bdv[LIST_NP];
    int brv[LIST_NP];
#pragma unroll
    for (int j = 0; j < LIST_NP; ++j) {
      bdv[j] = __builtin_inf();
      brv[j] = 0x7fffffff;
    }
    auto take = [&](int j, int r, double D) {
#pragma unroll
      for (int jj = 0; jj < LIST_NP; ++jj)
        if (jj == j && (D < bdv[jj] || (D == bdv[jj] && r < brv[jj]))) {
          bdv[jj] = D;
          brv[jj] = r;
        }
    };
    // sparse candidates, one thread each (all of a batch's candidates at once): the restatement's
    // arithmetic (exact_dist) bit for bit
    const int nc = min(ncand, CAND);
    if (t < nb && fullb[t]) atomicAdd(stats + 1, 1);  // statistics: pixels scored in full
    if (t == 0) atomicAdd(stats, nc);                  // and sparse candidates
    for (int k = t; k < nc; k += LIST_NT) {
      const int j = cand[k] >> 16, r = cand[k] & 0xffff;
      if (fullb[j]) continue;
      int nz = 0;
      take(j, r, exact_dist(xb[j], E, r, C, bd, &nz));
    }
    for (int j = 0; j < nb; ++j)
      if (fullb[j])
        for (int r = t; r < R; r += LIST_NT) {
          int nz = 0;
          take(j, r, exact_dist(xb[j], E, r, C, bd, &nz));
        }
#pragma unroll
    for (int j = 0; j < LIST_NP; ++j) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const double ob = __shfl_xor(bdv[j], o, 64);
        const int orr = __shfl_xor(brv[j], o, 64);
        if (ob < bdv[j] || (ob == bdv[j] && orr < brv[j])) {
          bdv[j] = ob;
          brv[j] = orr;
        }
      }
      if (lane == 0) {
        redd[w][j] = bdv[j];
        redr[w][j] = brv[j];
      }
    }
    __syncthreads();
    if (t < nb) {
      double bv = redd[0][t];
      int br = redr[0][t];
      for (int ww = 1; ww < LIST_NT / 64; ++ww) {
        const double ob = redd[ww][t];
        const int orr = redr[ww][t];
        if (ob < bv || (ob == bv && orr < br)) {
          bv = ob;
          br = orr;
        }
      }
      const int64_t p = list[b0 + t];
      best_idx[p] = br == 0x7fffffff ? 0 : br;
      best_dist[p] = (float)bv;
    }
    __syncthreads();
  }
}

// The screen's proven error bound, in score units (score = sum over segments of the cosine of the
// segment-normalised vectors, plus the zero-segment indicators), for a pixel with no all-zero
// segment (eps_zero per all-zero segment on top).  u = 2^-24.  Terms, per segment s of n_s channels:
//  (a) the pixel's f32 normalisation: f32 sum of squares (<= n_s u), v_rsq (<= 2 u), the product
//      (u): the segment cosine moves by <= (n_s / 2 + 4) u;
//  (b) the library's normalisation (f64, rounded to f32): <= 1.01 u;
//  (c) split fp16 (v = hi + lo + e, |e| <= 2^-22 |v| + 2^-25; lo * lo' dropped):
//      <= 3 * 2^-22 + 2^-24 * 1.01 sqrt(n_s)  (sum |x| <= sqrt(n_s) for a unit segment);
//  (d) the MFMA accumulation: each f16 MFMA output within KMFMA u (|C_in| + sum |a b|) of the exact
//      (hrf_probe_mfma_f16: tests/test_classify_exact_gpu.py measures <= 7.6 on gfx950 and asserts
//      <= 12; the bound uses 16), and every partial sum of an output is <= A = sum |products| <=
//      1.002 nseg (+1 per all-zero segment: the indicator terms), so NM MFMAs per output add
//      <= KMFMA u NM A.  The f32 MFMA (mode 0) is a k-ordered fmaf chain (cdna_hip_programming.md
//      "FP32-input MFMA"): <= KP u A.
// The keyed sweeps' 4 truncated bits are covered by reporting s2 with them set (key_score_hi).
constexpr double KMFMA = 16.0;
constexpr double U24 = 1.0 / 16777216.0;
struct ScreenEps {
  double base, zero, eps32;
};
ScreenEps screen_eps(const Bounds &bd, double nmfma, bool f32chain, int kp) {
  double a = 0.0, c = 0.0, e32 = 0.0;
  for (int sg = 0; sg < bd.nseg; ++sg) {
    const int ns = bd.b[sg + 1] - bd.b[sg];
    a += ns / 2.0 + 4.0 + 1.01;
    c += 12.0 + 1.01 * sqrt((double)ns);
    e32 += ns + 4.01;
  }
  e32 += (double)bd.nseg * bd.nseg;
  const double A = 1.002 * bd.nseg + 0.01;
  const double per = f32chain ? (double)kp : KMFMA * nmfma;
  ScreenEps e;
  e.base = U24 * (a + c + per * A) * 1.01;
  e.zero = U24 * per * 1.01;
  e.eps32 = U24 * e32 * 1.01;
  return e;
}

}  // namespace

extern "C" {

hrf_status hrf_classify_geometry(int32_t C, int32_t nseg, int32_t R, int32_t mode, int32_t *kp_host,
                                 int32_t *rpad_host) {
  HRF_REQUIRE(C >= 1 && nseg >= 1 && nseg <= SMAX && R >= 1, "classify_geometry: bad arguments");
  HRF_REQUIRE(mode >= 0 && mode <= 2,
              "classify_geometry: mode must be 0 (f32 MFMA), 1 (split fp16 MFMA) or 2 (split fp16, reference layouts)");
  if (mode == 2) {
    *kp_host = 16 * (int32_t)hrf::cdiv(C + 1, 16);
  } else if (mode == 0) {
    const int ks = choose_ks(C + nseg);
    HRF_REQUIRE(ks > 0, "classify: C + nseg must be <= 128");
    *kp_host = 2 * ks;
  } else {
    const int ks16 = (int)hrf::cdiv(C + nseg + 1, 16);  // + the validity-bias column
    HRF_REQUIRE(ks16 >= 1 && ks16 <= 8, "classify: C + nseg must be <= 127");
    *kp_host = 16 * ks16;
  }
  *rpad_host = (int32_t)(hrf::cdiv(R, RCH) * RCH);
  return HRF_OK;
}

hrf_status hrf_classify_table_row_bytes(int32_t C, const int32_t *bounds_host, int32_t nseg, int32_t mode,
                                        int32_t *row_bytes_host) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  int32_t kp = 0, rpad = 0;
  if (hrf_status s = hrf_classify_geometry(C, nseg, 1, mode, &kp, &rpad)) return s;
  HRF_REQUIRE(row_bytes_host, "classify_table_row_bytes: null output");
  *row_bytes_host = (int32_t)(mode == 0 ? 4 * kp : table_rowb(mode, layout_id(bd, C), kp));
  return HRF_OK;
}

hrf_status hrf_classify_prepare_refs(const float *ref, int32_t R, int32_t C, const int32_t *bounds_host, int32_t nseg,
                                     int32_t mode, void *refx, hrf_stream_t stream) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  int32_t kp = 0, rpad = 0;
  if (hrf_status s = hrf_classify_geometry(C, nseg, R, mode, &kp, &rpad)) return s;
  HRF_REQUIRE(ref && refx, "classify_prepare_refs: null buffer");
  HRF_REQUIRE(mode != 2 || layout_id(bd, C) != 0,
              "classify: mode 2 needs the E. coli (0,32,55,75,89,95) or multispecies (0,23,43,57,63) layout");
  HRF_REQUIRE(C <= 128 && R <= LIST_RMAX, "classify_prepare_refs: C <= 128 and R <= %d required", LIST_RMAX);
  hipStream_t s = (hipStream_t)stream;
  if (mode == 2) {
    ref_prep_lay_kernel<<<(unsigned)hrf::cdiv(rpad, 128), 128, 0, s>>>(
        ref, R, C, bd, kp, rpad, (int32_t)(table_rowb(2, layout_id(bd, C), kp) / 2), (_Float16 *)refx);
    ref_negflag_kernel<<<1, 256, 0, s>>>(ref, (int64_t)R * C, kp, (_Float16 *)refx);
  } else if (mode == 0)
    ref_prep_kernel<<<(unsigned)hrf::cdiv(rpad, 128), 128, 0, s>>>(ref, R, C, bd, kp, rpad, (float *)refx);
  else
    ref_prep_f16_kernel<<<(unsigned)hrf::cdiv(rpad, 128), 128, 0, s>>>(ref, R, C, bd, kp, rpad, (_Float16 *)refx);
  // the exact section (refine): f32 library row- and channel-major, ny, iy, header
  const ExactLayout el = exact_layout(mode, layout_id(bd, C), kp, rpad, R, C, nseg);
  char *sec = (char *)refx + el.off;
  exact_prep_kernel<<<hrf::stream_grid((int64_t)C * el.RT), 256, 0, s>>>(
      ref, R, C, bd, el.CP, el.RT, (float *)(sec + el.lib32), (float *)(sec + el.libT), (double *)(sec + el.ny),
      (float *)(sec + el.iy));
  exact_hdr_kernel<<<1, 1, 0, s>>>((const double *)(sec + el.ny), R, C, nseg, (ExactHdr *)sec);
  HRF_LAUNCHED();
  return HRF_OK;
}

int64_t hrf_classify_refx_bytes(int32_t C, const int32_t *bounds_host, int32_t nseg, int32_t R, int32_t mode) {
  Bounds bd;
  if (make_bounds(bounds_host, nseg, C, &bd) != HRF_OK) return -1;
  int32_t kp = 0, rpad = 0;
  if (hrf_classify_geometry(C, nseg, R, mode, &kp, &rpad) != HRF_OK) return -1;
  const ExactLayout el = exact_layout(mode, layout_id(bd, C), kp, rpad, R, C, nseg);
  return el.off + el.total;
}

// {listed count (16 B), the list (4 P B)}, then the table sweep's runner-up bounds (4 P B) for
// hrf_classify_pixels_table_exact
int64_t hrf_classify_refine_work_bytes(int64_t P) {
  return P < 0 ? -1 : al256(16 + 4 * (P > 0 ? P : 1)) + 4 * (P > 0 ? P : 1);
}

}  // extern "C"

namespace {

// the sweep of hrf_classify_pixels (`second`: nullable runner-up bound output)
hrf_status screen_stack(const float *stack, int64_t P, int32_t C, const void *refx, int32_t R, const Bounds &bd,
                        int32_t mode, int32_t *best_idx, float *best_dist, float *second, hipStream_t s) {
  int32_t kp = 0, rpad = 0;
  if (hrf_status st = hrf_classify_geometry(C, bd.nseg, R, mode, &kp, &rpad)) return st;
  if (P == 0) return HRF_OK;
  HRF_REQUIRE(stack && refx && best_idx && best_dist, "classify_pixels: null buffer");
  const unsigned grid = (unsigned)hrf::cdiv(P, 256);
  if (mode == 2) {
    const int lay = layout_id(bd, C);
    HRF_REQUIRE(lay != 0, "classify: mode 2 needs the E. coli or multispecies channel layout");
    if (lay == 1) {
      // E. coli layout: the 16x16x32 sweep with the lane-per-pixel prologue
      // (classify_pixels_w16_kernel) -- 4 waves, 2 buffers of 64 rows, HRF_W16T_OCC workgroups per
      // CU (rounds 3-5: three, 1.76 vs 1.83 ms for round 2's lay16 form, 2.13-2.20 for the 32x32x16
      // form, on a 2048^2 tile at R = 1023; DESIGN.md "Per-pixel classifier")
      if (hrf_status st = launch_w16_lay<LayEcoli, 4, 2, 64, HRF_W16T_SCREEN_OCC, HRF_W16T_NG>(stack, P, refx, R, rpad, best_idx, best_dist,
                                                                            second, s))
        return st;
      HRF_LAUNCHED();
      return HRF_OK;
    }
    // community layout (R = 127: a two-chunk sweep, where the 32x32x16 form's shorter prologue
    // wins, 0.34 vs 0.44 ms): 4 waves per workgroup share the library chunks streamed through LDS
    const size_t rowb = (size_t)table_rowb(2, lay, kp);
    const size_t shm = std::max<size_t>((size_t)2 * RCH * rowb, sizeof(float) * 4 * 32 * C);
    (void)hipFuncSetAttribute((const void *)classify_pixels_lay_kernel<LayMulti, 4>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    classify_pixels_lay_kernel<LayMulti, 4><<<(unsigned)hrf::cdiv(P, 256), 256, shm, s>>>(
        stack, P, (const _Float16 *)refx, R, rpad, best_idx, best_dist, second);
    HRF_LAUNCHED();
    return HRF_OK;
  }
  if (mode == 1) {
    const int ks16 = kp / 16;
    const size_t shm = std::max<size_t>((size_t)2 * RCH * (4 * kp + 16), sizeof(float) * 4 * 32 * (C + MROW) + 128);
    HRF_REQUIRE(shm <= 160 * 1024, "classify_pixels: C too large for LDS staging");
#define HRF_CP16(K)                                                                                          \
  case K:                                                                                                    \
    hipFuncSetAttribute((const void *)classify_pixels_f16_kernel<K>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                        (int)shm);                                                                           \
    classify_pixels_f16_kernel<K><<<grid, 256, shm, s>>>(stack, P, C, bd, (const _Float16 *)refx, R, rpad,     \
                                                         best_idx, best_dist, second);                       \
    break;
    switch (ks16) {
      HRF_CP16(1)
      HRF_CP16(2)
      HRF_CP16(3)
      HRF_CP16(4)
      HRF_CP16(5)
      HRF_CP16(6)
      HRF_CP16(7)
      HRF_CP16(8)
      default:
        HRF_REQUIRE(false, "classify_pixels: unsupported K");
    }
#undef HRF_CP16
    HRF_LAUNCHED();
    return HRF_OK;
  }
  const int ks = kp / 2;
  const size_t shm = sizeof(float) * std::max<size_t>((size_t)RCH * (kp + 2), (size_t)4 * 32 * C);
  HRF_REQUIRE(shm <= 160 * 1024, "classify_pixels: C too large for LDS staging");
#define HRF_CP(K)                                                                                          \
  case K:                                                                                                  \
    hipFuncSetAttribute((const void *)classify_pixels_kernel<K>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                        (int)shm);                                                                         \
    classify_pixels_kernel<K><<<grid, 256, shm, s>>>(stack, P, C, bd, (const float *)refx, R, rpad, best_idx,   \
                                                     best_dist, second);                                   \
    break;
  switch (ks) {
    HRF_CP(8)
    HRF_CP(16)
    HRF_CP(18)
    HRF_CP(24)
    HRF_CP(32)
    HRF_CP(34)
    HRF_CP(40)
    HRF_CP(50)
    HRF_CP(56)
    HRF_CP(64)
    default:
      HRF_REQUIRE(false, "classify_pixels: unsupported K");
  }
#undef HRF_CP
  HRF_LAUNCHED();
  return HRF_OK;
}

// MFMAs accumulated into one score by each screen (the bound's NM): screen 0 = mode 0 (f32 chain,
// KP fmas), 1 = mode 1 (32x32x16, indicator columns), 2 = mode 2 in-kernel (E. coli: the 16x16x32
// w16 sweep, community: the 32x32x16 lay sweep; + the indicator k-step), 3 = the pixel-table w16t
ScreenEps eps_of_screen(int screen, const Bounds &bd, int C, int kp) {
  const int lay = layout_id(bd, C);
  if (screen == 0) return screen_eps(bd, 0, true, kp);
  if (screen == 1) return screen_eps(bd, 3 * (kp / 16), false, kp);
  if (screen == 2 && lay == 2) {  // classify_pixels_lay_kernel: cross products first, as w16
    const int ks = (C + 1 + 15) / 16;
    return screen_eps(bd, ks + 1 + 2.0 * ks * 0x1p-9, false, kp);
  }
  // w16 / w16t: the 2 KT cross-product MFMAs meet accumulators below 2^-9 A (their products are
  // <= 2^-10 A in all), then KT hi * hi' MFMAs and the indicator step at full magnitude
  const int kt = (C + 1 + 31) / 32;
  return screen_eps(bd, kt + 1 + 2.0 * kt * 0x1p-9, false, kp);
}

// the refine's arguments for `screen`'s output on refx; fuse: the table sweep (screen 3) runs the
// certificate itself (classify_pixels_w16t_kernel<..., true>), else refine_best_kernel does
hrf_status refine_args(const PixSrc &S, int64_t P, int32_t C, const void *refx, int32_t R, const Bounds &bd,
                       int32_t screen, void *work, int64_t work_bytes, RefineArgs *A, hipStream_t s) {
  HRF_REQUIRE(screen >= 0 && screen <= 3, "classify_refine: screen must be 0..3");
  const int mode = screen == 3 ? 2 : screen;
  int32_t kp = 0, rpad = 0;
  if (hrf_status st = hrf_classify_geometry(C, bd.nseg, R, mode, &kp, &rpad)) return st;
  HRF_REQUIRE(C <= 128 && R <= LIST_RMAX, "classify_refine: C <= 128 and R <= %d required", LIST_RMAX);
  HRF_REQUIRE(work_bytes >= hrf_classify_refine_work_bytes(P), "classify_refine: work buffer too small");
  HRF_REQUIRE(refx && work, "classify_refine: null buffer");
  const ExactLayout el = exact_layout(mode, layout_id(bd, C), kp, rpad, R, C, bd.nseg);
  const char *sec = (const char *)refx + el.off;
  A->S = S;
  A->E.lib32 = (const float *)(sec + el.lib32);
  A->E.libT = (const float *)(sec + el.libT);
  A->E.ny = (const double *)(sec + el.ny);
  A->E.iy = (const float *)(sec + el.iy);
  A->E.CP = el.CP;
  A->E.RT = el.RT;
  A->hdr = (const ExactHdr *)sec;
  const ScreenEps ep = eps_of_screen(screen, bd, C, kp);
  A->eps_base = ep.base;
  A->eps_zero = ep.zero;
  A->cnt = (int32_t *)work;
  A->list = (int32_t *)((char *)work + 16);
  A->bd = bd;
  HRF_HIP(hipMemsetAsync(A->cnt, 0, 4 * sizeof(int32_t), s));  // count + the list pass's statistics
  return HRF_OK;
}

// the list pass over what the certificate left (device-held count)
hrf_status refine_list(const RefineArgs &A, int64_t P, int32_t C, int32_t R, const Bounds &bd, int32_t screen,
                       int32_t *best_idx, float *best_dist, hipStream_t s) {
  int32_t kp = 0, rpad = 0;
  if (hrf_status st = hrf_classify_geometry(C, bd.nseg, R, screen == 3 ? 2 : screen, &kp, &rpad)) return st;
  const ScreenEps ep = eps_of_screen(screen, bd, C, kp);
  const size_t shm = sizeof(float) * LIST_NP * (size_t)A.E.RT;  // 128 KB at R = LIST_RMAX
  (void)hipFuncSetAttribute((const void *)refine_list_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  const unsigned g = hrf::resident_grid(refine_list_kernel, LIST_NT, shm, hrf::cdiv(P, LIST_NP));
  refine_list_kernel<<<g, LIST_NT, shm, s>>>(A.S, C, bd, A.E, A.hdr, R, ep.eps32, A.list, A.cnt, A.cnt + 1, best_idx,
                                             best_dist);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status refine(const PixSrc &S, int64_t P, int32_t C, const void *refx, int32_t R, const Bounds &bd, int32_t screen,
                  const float *second, int32_t *best_idx, float *best_dist, void *work, int64_t work_bytes,
                  hipStream_t s) {
  if (P == 0) return HRF_OK;
  HRF_REQUIRE(second && best_idx && best_dist, "classify_refine: null buffer");
  RefineArgs A;
  if (hrf_status st = refine_args(S, P, C, refx, R, bd, screen, work, work_bytes, &A, s)) return st;
  refine_best_kernel<<<(unsigned)hrf::cdiv(P, 64), 64, (size_t)refine_slice_bytes(), s>>>(
      A, P, C, bd, second, best_idx, best_dist);
  HRF_LAUNCHED();
  return refine_list(A, P, C, R, bd, screen, best_idx, best_dist, s);
}

hrf_status pixsrc_of(const float *const *src_host, const int32_t *channels_host, const int32_t *shifts_dev,
                     int32_t nlaser, int64_t H, int64_t W, int32_t apply_mask, int32_t C, PixSrc *S) {
  HRF_REQUIRE(nlaser >= 1 && nlaser <= XLMAX && src_host && channels_host && H >= 0 && W >= 1,
              "classify_refine: bad pixel source");
  *S = PixSrc{};
  S->n = nlaser;
  S->c0[0] = 0;
  for (int q = 0; q < nlaser; ++q) {
    HRF_REQUIRE(src_host[q] && channels_host[q] >= 1, "classify_refine: laser %d missing", q);
    S->src[q] = src_host[q];
    S->c0[q + 1] = S->c0[q] + channels_host[q];
    S->mdiv[q] = ((uint64_t)1 << 32) / (uint64_t)channels_host[q] + (((uint64_t)1 << 32) % (uint64_t)channels_host[q] ? 1 : 0);
  }
  for (int q = nlaser; q < XLMAX; ++q) S->c0[q + 1] = S->c0[nlaser];
  HRF_REQUIRE(S->c0[nlaser] == C, "classify_refine: the lasers hold %d channels, the library %d", S->c0[nlaser], C);
  HRF_REQUIRE(H * W * (int64_t)C < ((int64_t)1 << 31), "classify_refine: H * W * C must be < 2^31");
  S->dsh = shifts_dev;
  S->H = H;
  S->W = W;
  S->apply_mask = apply_mask;
  return HRF_OK;
}

}  // namespace

extern "C" {

hrf_status hrf_classify_pixels_screen(const float *stack, int64_t P, int32_t C, const void *refx, int32_t R,
                                      const int32_t *bounds_host, int32_t nseg, int32_t mode, int32_t *best_idx,
                                      float *best_dist, float *second, hrf_stream_t stream) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  return screen_stack(stack, P, C, refx, R, bd, mode, best_idx, best_dist, second, (hipStream_t)stream);
}

hrf_status hrf_classify_pixels_refine(const float *const *src_host, const int32_t *channels_host,
                                      const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                      int32_t apply_mask, const void *refx, int32_t R, const int32_t *bounds_host,
                                      int32_t nseg, int32_t screen, const float *second, int32_t *best_idx,
                                      float *best_dist, void *work, int64_t work_bytes, hrf_stream_t stream) {
  Bounds bd;
  const int32_t C = channels_host ? [&] {
    int32_t c = 0;
    for (int q = 0; q < nlaser && q < XLMAX; ++q) c += channels_host[q];
    return c;
  }() : 0;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  PixSrc S;
  if (hrf_status s = pixsrc_of(src_host, channels_host, shifts_dev, nlaser, H, W, apply_mask, C, &S)) return s;
  return refine(S, H * W, C, refx, R, bd, screen, second, best_idx, best_dist, work, work_bytes, (hipStream_t)stream);
}

hrf_status hrf_classify_screen_eps(int32_t C, const int32_t *bounds_host, int32_t nseg, int32_t R, int32_t screen,
                                   double *eps_host) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  HRF_REQUIRE(screen >= 0 && screen <= 3 && eps_host, "classify_screen_eps: bad arguments");
  int32_t kp = 0, rpad = 0;
  if (hrf_status s = hrf_classify_geometry(C, nseg, R, screen == 3 ? 2 : screen, &kp, &rpad)) return s;
  const ScreenEps e = eps_of_screen(screen, bd, C, kp);
  eps_host[0] = e.base;
  eps_host[1] = e.zero;
  eps_host[2] = e.eps32;
  return HRF_OK;
}

hrf_status hrf_classify_pixels(const float *stack, int64_t P, int32_t C, const void *refx, int32_t R,
                               const int32_t *bounds_host, int32_t nseg, int32_t mode, int32_t *best_idx,
                               float *best_dist, hrf_stream_t stream) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  if (P == 0) return HRF_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t wb = hrf_classify_refine_work_bytes(P);
  char *ws = nullptr;
  HRF_HIP(hipMallocAsync((void **)&ws, (size_t)(al256(4 * P) + wb), s));
  float *second = (float *)ws;
  hrf_status st = screen_stack(stack, P, C, refx, R, bd, mode, best_idx, best_dist, second, s);
  if (!st) {
    const float *src[1] = {stack};
    const int32_t ch[1] = {C};
    PixSrc S;
    st = pixsrc_of(src, ch, nullptr, 1, 1, P, 0, C, &S);
    if (!st) st = refine(S, P, C, refx, R, bd, mode, second, best_idx, best_dist, ws + al256(4 * P), wb, s);
  }
  HRF_HIP(hipFreeAsync(ws, s));
  return st;
}

int64_t hrf_pixtable_bytes(int64_t P, int32_t C, const int32_t *bounds_host, int32_t nseg) {
  Bounds bd;
  if (make_bounds(bounds_host, nseg, C, &bd) != HRF_OK) return -1;
  const int lay = layout_id(bd, C);
  if (lay == 0 || P < 0) return -1;
  const int64_t groups = (P + 255) / 256 * 16;  // whole classifier workgroups
  return groups * (lay == 1 ? hrf_pix::group_entries<LayEcoli>() : hrf_pix::group_entries<LayMulti>()) * 16;
}

hrf_status hrf_pixtable_prepare(const float *stack, int64_t P, int32_t C, const int32_t *bounds_host, int32_t nseg,
                                void *table, uint8_t *flags, hrf_stream_t stream) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  const int lay = layout_id(bd, C);
  HRF_REQUIRE(lay != 0, "pixtable: the E. coli or multispecies channel layout only");
  if (P == 0) return HRF_OK;
  HRF_REQUIRE(stack && table && flags, "pixtable: null buffer");
  const unsigned g = (unsigned)hrf::cdiv(P, 64);
  if (lay == 1)
    pixtable_prep_kernel<LayEcoli><<<g, 256, 0, (hipStream_t)stream>>>(stack, P, (uint4 *)table, flags);
  else
    pixtable_prep_kernel<LayMulti><<<g, 256, 0, (hipStream_t)stream>>>(stack, P, (uint4 *)table, flags);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_classify_pixels_table(const void *table, const uint8_t *flags, int64_t P, int32_t C, const void *refx,
                                     int32_t R, const int32_t *bounds_host, int32_t nseg, int32_t *best_idx,
                                     float *best_dist, float *second, hrf_stream_t stream) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  int32_t kp = 0, rpad = 0;
  if (hrf_status s = hrf_classify_geometry(C, nseg, R, 2, &kp, &rpad)) return s;
  const int lay = layout_id(bd, C);
  HRF_REQUIRE(lay != 0, "classify_pixels_table: the E. coli or multispecies channel layout only");
  if (P == 0) return HRF_OK;
  HRF_REQUIRE(table && flags && refx && best_idx && best_dist, "classify_pixels_table: null buffer");
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = (unsigned)hrf::cdiv(P, 64 * HRF_W16T_NG);
  auto go = [&](auto lay_tag) -> hrf_status {
    using L = decltype(lay_tag);
    constexpr int KT = (L::C + 1 + 31) / 32;
    const size_t shm = (size_t)2 * 64 * (128 * KT + L::PADB);
    (void)hipFuncSetAttribute(
        (const void *)classify_pixels_w16t_kernel<L, 4, 2, 64, HRF_W16T_SCREEN_OCC, false, HRF_W16T_NG>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    classify_pixels_w16t_kernel<L, 4, 2, 64, HRF_W16T_SCREEN_OCC, false, HRF_W16T_NG><<<grid, 256, shm, s>>>(
        (const uint4 *)table, flags, P, (const _Float16 *)refx, R, rpad, best_idx, best_dist, second, RefineArgs{});
    return HRF_OK;
  };
  hrf_status st = lay == 1 ? go(LayEcoli{}) : go(LayMulti{});
  if (st) return st;
  HRF_LAUNCHED();
  return HRF_OK;
}

// the table sweep, exact: fused (the sweep certifies its own rows) or the sweep with its runner-up
// bounds, then refine_best_kernel; both followed by the list pass
static hrf_status table_exact(const void *table, const uint8_t *flags, const float *const *src_host,
                              const int32_t *channels_host, const int32_t *shifts_dev, int32_t nlaser, int64_t H,
                              int64_t W, int32_t apply_mask, const void *refx, int32_t R, const int32_t *bounds_host,
                              int32_t nseg, int32_t *best_idx, float *best_dist, void *work, int64_t work_bytes,
                              bool fused, hipStream_t s) {
  const int64_t P = H * W;
  int32_t C = 0;
  for (int q = 0; src_host && channels_host && q < nlaser && q < XLMAX; ++q) C += channels_host[q];
  Bounds bd;
  if (hrf_status st = make_bounds(bounds_host, nseg, C, &bd)) return st;
  int32_t kp = 0, rpad = 0;
  if (hrf_status st = hrf_classify_geometry(C, nseg, R, 2, &kp, &rpad)) return st;
  const int lay = layout_id(bd, C);
  HRF_REQUIRE(lay != 0, "classify_pixels_table_exact: the E. coli or multispecies channel layout only");
  if (P == 0) return HRF_OK;
  HRF_REQUIRE(table && flags && refx && best_idx && best_dist, "classify_pixels_table_exact: null buffer");
  PixSrc S;
  if (hrf_status st = pixsrc_of(src_host, channels_host, shifts_dev, nlaser, H, W, apply_mask, C, &S)) return st;
  if (!fused) {
    HRF_REQUIRE(work && work_bytes >= hrf_classify_refine_work_bytes(P), "classify_pixels_table_exact: work buffer too small");
    float *second = (float *)((char *)work + al256(16 + 4 * P));
    if (hrf_status st = hrf_classify_pixels_table(table, flags, P, C, refx, R, bounds_host, nseg, best_idx, best_dist,
                                                  second, s))
      return st;
    return refine(S, P, C, refx, R, bd, 3, second, best_idx, best_dist, work, work_bytes, s);
  }
  RefineArgs A;
  if (hrf_status st = refine_args(S, P, C, refx, R, bd, 3, work, work_bytes, &A, s)) return st;
  const unsigned grid = (unsigned)hrf::cdiv(P, 256);
  auto go = [&](auto lay_tag) -> hrf_status {
    using L = decltype(lay_tag);
    constexpr int KT = (L::C + 1 + 31) / 32;
    constexpr int64_t SL = (refine_slice_bytes() + 15) / 16 * 16;
    const size_t shm = std::max<size_t>((size_t)2 * 64 * (128 * KT + L::PADB), (size_t)(4 * SL));
    (void)hipFuncSetAttribute((const void *)classify_pixels_w16t_kernel<L, 4, 2, 64, HRF_W16T_OCC, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    classify_pixels_w16t_kernel<L, 4, 2, 64, HRF_W16T_OCC, true><<<grid, 256, shm, s>>>(
        (const uint4 *)table, flags, P, (const _Float16 *)refx, R, rpad, best_idx, best_dist, nullptr, A);
    return HRF_OK;
  };
  hrf_status st = lay == 1 ? go(LayEcoli{}) : go(LayMulti{});
  if (st) return st;
  HRF_LAUNCHED();
  return refine_list(A, P, C, R, bd, 3, best_idx, best_dist, s);
}

hrf_status hrf_classify_pixels_table_exact(const void *table, const uint8_t *flags, const float *const *src_host,
                                           const int32_t *channels_host, const int32_t *shifts_dev, int32_t nlaser,
                                           int64_t H, int64_t W, int32_t apply_mask, const void *refx, int32_t R,
                                           const int32_t *bounds_host, int32_t nseg, int32_t *best_idx,
                                           float *best_dist, void *work, int64_t work_bytes, hrf_stream_t stream) {
  return table_exact(table, flags, src_host, channels_host, shifts_dev, nlaser, H, W, apply_mask, refx, R, bounds_host,
                     nseg, best_idx, best_dist, work, work_bytes, false, (hipStream_t)stream);
}

hrf_status hrf_classify_pixels_table_exact_fused(const void *table, const uint8_t *flags,
                                                 const float *const *src_host, const int32_t *channels_host,
                                                 const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                                 int32_t apply_mask, const void *refx, int32_t R,
                                                 const int32_t *bounds_host, int32_t nseg, int32_t *best_idx,
                                                 float *best_dist, void *work, int64_t work_bytes,
                                                 hrf_stream_t stream) {
  return table_exact(table, flags, src_host, channels_host, shifts_dev, nlaser, H, W, apply_mask, refx, R, bounds_host,
                     nseg, best_idx, best_dist, work, work_bytes, true, (hipStream_t)stream);
}

}  // extern "C"

namespace hrf {

// the per-cell tail of hrf_tile_ecoli: row counts held on the device (nrows_dev <= nmax), no host
// synchronisation; refT = the library transposed to channel-major (transpose_f64)
hrf_status cells_lib_prep(const double *a, int32_t R, int32_t C, const int32_t *bounds_host, int32_t nseg, double *t,
                          double *ny, hipStream_t s) {
  Bounds bd;
  if (hrf_status st = make_bounds(bounds_host, nseg, C, &bd)) return st;
  cells_lib_prep_kernel<<<hrf::stream_grid((int64_t)R * C), 256, 0, s>>>(a, R, C, bd, t, ny);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status segment_flags_devn(const double *x, int64_t nmax, const int32_t *nrows_dev, int32_t C,
                              const int32_t *bounds_host, int32_t nseg, double thr, double *out, hipStream_t s) {
  Bounds bd;
  if (hrf_status st = make_bounds(bounds_host, nseg, C, &bd)) return st;
  if (nmax == 0) return HRF_OK;
  segment_flags_kernel<<<(unsigned)hrf::cdiv(nmax * nseg, 256), 256, 0, s>>>(x, nmax, C, bd, thr, out, nrows_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status classify_cells_devn(const double *x, int64_t nmax, const int32_t *nrows_dev, const double *refT,
                               const double *ny, int32_t R, int32_t C, const int32_t *bounds_host, int32_t nseg,
                               int32_t variant, const double *fx, const double *fr, int32_t *arg, double *dmin,
                               hipStream_t s) {
  Bounds bd;
  if (hrf_status st = make_bounds(bounds_host, nseg, C, &bd)) return st;
  HRF_REQUIRE(variant >= 0 && variant <= 2, "classify_cells: variant must be 0, 1 or 2");
  HRF_REQUIRE(variant == 0 || (fx && fr), "classify_cells: gated variants need presence flags");
  if (nmax == 0) return HRF_OK;
  classify_cells_blk_kernel<CELLS_CB, CELLS_NT><<<(unsigned)hrf::cdiv(nmax, CELLS_CB), CELLS_NT,
                                                  sizeof(double) * CELLS_CB * C, s>>>(
      x, nmax, refT, ny, R, C, bd, variant, fx, fr, arg, dmin, nrows_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // namespace hrf

extern "C" {

hrf_status hrf_segment_flags(const double *x, int64_t N, int32_t C, const int32_t *bounds_host, int32_t nseg,
                             double thr, double *out, hrf_stream_t stream) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  if (N == 0) return HRF_OK;
  HRF_REQUIRE(x && out, "segment_flags: null buffer");
  segment_flags_kernel<<<(unsigned)hrf::cdiv(N * nseg, 256), 256, 0, (hipStream_t)stream>>>(x, N, C, bd, thr, out,
                                                                                             nullptr);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_classify_cells(const double *x, int64_t N, const double *ref, int32_t R, int32_t C,
                              const int32_t *bounds_host, int32_t nseg, int32_t variant, const double *fx,
                              const double *fr, int32_t *arg, double *dmin, hrf_stream_t stream) {
  Bounds bd;
  if (hrf_status s = make_bounds(bounds_host, nseg, C, &bd)) return s;
  HRF_REQUIRE(variant >= 0 && variant <= 2, "classify_cells: variant must be 0, 1 or 2");
  HRF_REQUIRE(variant == 0 || (fx && fr), "classify_cells: gated variants need presence flags");
  HRF_REQUIRE(R >= 1 && C >= 1, "classify_cells: bad sizes");
  if (N == 0) return HRF_OK;
  HRF_REQUIRE(x && ref && arg && dmin, "classify_cells: null buffer");
  hipStream_t s = (hipStream_t)stream;
  double *refT = nullptr;
  HRF_HIP(hipMallocAsync((void **)&refT, sizeof(double) * (size_t)R * (C + bd.nseg), s));
  double *ny = refT + (size_t)R * C;
  cells_lib_prep_kernel<<<hrf::stream_grid((int64_t)R * C), 256, 0, s>>>(ref, R, C, bd, refT, ny);
  classify_cells_blk_kernel<CELLS_CB, CELLS_NT><<<(unsigned)hrf::cdiv(N, CELLS_CB), CELLS_NT,
                                                  sizeof(double) * CELLS_CB * C, s>>>(
      x, N, refT, ny, R, C, bd, variant, fx, fr, arg, dmin, nullptr);
  HRF_LAUNCHED();
  HRF_HIP(hipFreeAsync(refT, s));
  return HRF_OK;
}

}  // extern "C"

// ---- MFMA accumulation probe ------------------------------------------------------------------
// The per-pixel screen's error bound (hrf_classify_pixels_refine) assumes how an f16 MFMA adds
// its products to the f32 accumulator.  This runs ONE v_mfma_f32_16x16x32_f16 (shape 0) or
// v_mfma_f32_32x32x16_f16 (shape 1) per tile on caller data so tests/test_classify_exact_gpu.py
// can pin that model on the device: A (M x K) and B (K x N) f16 row-major, C and D (M x N) f32.
namespace {
__global__ __launch_bounds__(64) void mfma_probe_kernel(int shape, const _Float16 *__restrict__ a,
                                                        const _Float16 *__restrict__ b, const float *__restrict__ c,
                                                        float *__restrict__ d) {
  const int t = blockIdx.x, lane = threadIdx.x;
  h8 av, bv;
  if (shape == 0) {  // 16 x 16 x 32: lane row/col lane & 15, k 8Q..8Q+7, D rows 4Q..4Q+3
    const _Float16 *A = a + (int64_t)t * 16 * 32, *B = b + (int64_t)t * 32 * 16;
    const float *Cm = c + (int64_t)t * 256;
    float *Dm = d + (int64_t)t * 256;
    const int j = lane & 15, Q = lane >> 4;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      av[q] = A[j * 32 + 8 * Q + q];
      bv[q] = B[(8 * Q + q) * 16 + j];
    }
    f32x4 acc;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = Cm[(4 * Q + i) * 16 + j];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) Dm[(4 * Q + i) * 16 + j] = acc[i];
  } else {  // 32 x 32 x 16: lane row/col lane & 31, k 8h..8h+7, D rows (reg & 3) + 8 (reg >> 2) + 4h
    const _Float16 *A = a + (int64_t)t * 32 * 16, *B = b + (int64_t)t * 16 * 32;
    const float *Cm = c + (int64_t)t * 1024;
    float *Dm = d + (int64_t)t * 1024;
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      av[q] = A[j * 16 + 8 * h + q];
      bv[q] = B[(8 * h + q) * 32 + j];
    }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = Cm[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + j];
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) Dm[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + j] = acc[r];
  }
}
}  // namespace

extern "C" hrf_status hrf_probe_mfma_f16(int32_t shape, const void *a, const void *b, const float *c, float *d,
                                         int32_t ntiles, hrf_stream_t stream) {
  HRF_REQUIRE((shape == 0 || shape == 1) && ntiles >= 0 && (ntiles == 0 || (a && b && c && d)),
              "probe_mfma_f16: bad arguments");
  if (ntiles == 0) return HRF_OK;
  mfma_probe_kernel<<<(unsigned)ntiles, 64, 0, (hipStream_t)stream>>>(shape, (const _Float16 *)a,
                                                                      (const _Float16 *)b, c, d);
  HRF_LAUNCHED();
  return HRF_OK;
}
