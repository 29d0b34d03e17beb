// label.hip -- connected components and the binary-morphology / label-cleanup stages
// (a9, a10, a13).
//
// Connected components (skimage.measure.label semantics: non-zero pixels connect when
// EQUAL, 4- or 8-connectivity, raster-first numbering):
//   1. cc_local   : 32x32 tile per workgroup, union-find in LDS with atomicMin linking
//                   (larger root -> smaller root), so each local root is the tile-local
//                   minimum index.
//   2. cc_border  : the same union over tile-crossing neighbour pairs in global memory.
//                   Reads may be stale; correctness comes from atomicMin's returned value
//                   (retry on the true parent, indices strictly decrease).
//   3. cc_compress: parent[p] = root = the component's minimum raster index.
//   4. numbering  : roots ranked in raster order (wave ballots + block scan), which is
//                   exactly "first appearance" numbering -- bit-identical to skimage/scipy.
// Morphology kernels use the cross footprint of skimage's defaults.
#include <algorithm>

#include "common.hpp"
#include "wave.hpp"

namespace {

constexpr int CC_T = 32;  // tile edge

struct MaskV {
  const uint8_t *p;
  int inv;
  __device__ __forceinline__ int32_t operator()(int64_t i) const { return (int32_t)((p[i] != 0) ^ inv); }
};
struct LabelV {
  const int32_t *p;
  __device__ __forceinline__ int32_t operator()(int64_t i) const { return p[i]; }
};

__device__ __forceinline__ int find_lds(volatile int32_t *lp, int x) {
  int y = lp[x];
  while (y != x) {
    x = y;
    y = lp[x];
  }
  return x;
}

__device__ __forceinline__ void union_lds(int32_t *lp, int a, int b) {
  volatile int32_t *v = lp;
  for (;;) {
    a = find_lds(v, a);
    b = find_lds(v, b);
    if (a == b) return;
    if (a < b) {
      const int t = a;
      a = b;
      b = t;
    }
    const int old = atomicMin(&lp[a], b);
    if (old == a) return;
    a = old;
  }
}

__device__ __forceinline__ int32_t find_g(const int32_t *par, int32_t x) {
  int32_t y = par[x];
  while (y != x) {
    x = y;
    y = par[x];
  }
  return x;
}

__device__ __forceinline__ void union_g(int32_t *par, int32_t a, int32_t b) {
  for (;;) {
    a = find_g(par, a);
    b = find_g(par, b);
    if (a == b) return;
    if (a < b) {
      const int32_t t = a;
      a = b;
      b = t;
    }
    const int32_t old = atomicMin(&par[a], b);
    if (old == a) return;
    a = old;
  }
}

// zero != nullptr: also clears that per-pixel array (the component sizes the fused
// compression pass counts into)
template <class V, int CONN>
__global__ __launch_bounds__(256) void cc_local_kernel(V val, int64_t H, int64_t W, int32_t *__restrict__ parent,
                                                       int32_t *__restrict__ zero) {
  __shared__ int32_t lp[CC_T * CC_T];
  __shared__ int32_t lv[CC_T * CC_T];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * CC_T, c0 = (int64_t)blockIdx.x * CC_T;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int li = tid + 256 * k, lr = li >> 5, lc = li & 31;
    const int64_t gr = r0 + lr, gc = c0 + lc;
    const int32_t v = (gr < H && gc < W) ? val(gr * W + gc) : 0;
    lv[li] = v;
  }
  __syncthreads();
  // Horizontal runs come from a ballot: a wave holds two tile rows (lanes 0-31, 32-63); a
  // pixel's initial parent is the start of its run (the run's least index), so no union is
  // spent inside a run.
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int li = tid + 256 * k, lc = li & 31;
    const int32_t v = lv[li];
    const unsigned long long join = __ballot(v && lc > 0 && lv[li - 1] == v);
    const unsigned row = (unsigned)(join >> (threadIdx.x & 32));
    const unsigned starts = ~row & (lc == 31 ? 0xffffffffu : ((2u << lc) - 1u));  // bit 0 never joins
    lp[li] = v ? (li - lc) + (31 - __builtin_clz(starts)) : -1;
  }
  __syncthreads();
  // Vertical links: once per overlap segment of two runs (its first column); a diagonal link
  // only where neither the pixel's own run nor the other row's run already implies it through
  // a vertical one.  Every adjacency of equal values ends up linked, with ~one union per
  // (run, run) contact instead of one per neighbour pair.
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int li = tid + 256 * k, lr = li >> 5, lc = li & 31;
    const int32_t v = lv[li];
    if (!v || lr == 0) continue;
    const bool l = lc > 0 && lv[li - 1] == v, u = lv[li - 32] == v;
    const bool ul = lc > 0 && lv[li - 33] == v, ur = lc < 31 && lv[li - 31] == v;
    if (u && !(l && ul)) union_lds(lp, li, li - 32);
    if (CONN == 2) {
      if (ul && !l && !u) union_lds(lp, li, li - 33);
      if (ur && !u && !(lc < 31 && lv[li + 1] == v)) union_lds(lp, li, li - 31);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int li = tid + 256 * k, lr = li >> 5, lc = li & 31;
    const int64_t gr = r0 + lr, gc = c0 + lc;
    if (gr >= H || gc >= W) continue;
    int32_t g = -1;
    if (lv[li]) {
      const int rt = find_lds(lp, li);
      g = (int32_t)((r0 + (rt >> 5)) * W + c0 + (rt & 31));
    }
    parent[gr * W + gc] = g;
    if (zero) zero[gr * W + gc] = 0;
  }
}

// One thread per tile-border pixel that can have a neighbour in another tile: row 0 of the
// tile (32) and columns 0 and 31 of rows 1..31 (62), 94 per tile -- a grid of 94/1024 of the
// image instead of one thread per pixel that mostly exits at once.
constexpr int CC_BORDER_PX = CC_T + 2 * (CC_T - 1);
template <class V, int CONN>
__global__ void cc_border_kernel(V val, int64_t H, int64_t W, int32_t *__restrict__ parent) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tiles_x = (W + CC_T - 1) / CC_T;
  const int64_t tile = t / CC_BORDER_PX;
  if (tile >= tiles_x * ((H + CC_T - 1) / CC_T)) return;
  const int k = (int)(t - tile * CC_BORDER_PX);
  const int lr = k < CC_T ? 0 : 1 + ((k - CC_T) >> 1);
  const int lc = k < CC_T ? k : (((k - CC_T) & 1) ? CC_T - 1 : 0);
  const int64_t r = (tile / tiles_x) * CC_T + lr, c = (tile % tiles_x) * CC_T + lc;
  if (r >= H || c >= W) return;
  const int64_t p = r * W + c;
  const int32_t v = val(p);
  if (!v) return;
  if (lc == 0 && c > 0 && val(p - 1) == v) union_g(parent, (int32_t)p, (int32_t)(p - 1));
  if (r > 0) {
    if (lr == 0 && val(p - W) == v) union_g(parent, (int32_t)p, (int32_t)(p - W));
    if (CONN == 2) {
      if ((lr == 0 || lc == 0) && c > 0 && val(p - W - 1) == v) union_g(parent, (int32_t)p, (int32_t)(p - W - 1));
      if ((lr == 0 || lc == 31) && c + 1 < W && val(p - W + 1) == v) union_g(parent, (int32_t)p, (int32_t)(p - W + 1));
    }
  }
}

// zero != nullptr: also clears a per-pixel size array for cc_sizes (saves its memset launch)
__global__ void cc_compress_kernel(int32_t *__restrict__ parent, int64_t n, int32_t *__restrict__ zero) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t q = parent[p];
    if (q >= 0 && q != p) parent[p] = find_g(parent, q);
    if (zero) zero[p] = 0;
  }
}

// compression fused with the size count: each wave compresses RUN_PX consecutive pixels and
// counts them at their roots (wave_run_count); size[] was cleared by the tile pass.  The finds
// read ancestors while other waves store roots -- every store is a root, as in cc_compress.
constexpr int RUN = 32;
constexpr int64_t RUN_PX = RUN * 64;
__global__ void cc_compress_sizes_kernel(int32_t *__restrict__ parent, int64_t n, int32_t *__restrict__ size) {
  const int64_t nw = (n + RUN_PX - 1) / RUN_PX;
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t w = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); w < nw; w += (int64_t)gridDim.x * wpb)
    hrf::wave_run_count<RUN>(size, w * RUN_PX, n, [&](int64_t e) {
      int32_t q = parent[e];
      if (q >= 0 && q != e) {
        q = find_g(parent, q);
        parent[e] = q;
      }
      return q;
    });
}

// Numbering.  Block = 256 threads x 4 pixels = 1024 consecutive raster pixels.
constexpr int NB = 1024;

__global__ __launch_bounds__(256) void cc_count_roots_kernel(const int32_t *__restrict__ parent, int64_t n,
                                                             int32_t *__restrict__ blk) {
  __shared__ int32_t ws[4];
  const int tid = threadIdx.x;
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t p = (int64_t)blockIdx.x * NB + k * 256 + tid;
    cnt += (p < n && parent[p] == p);
  }
  cnt = hrf::wave_sum(cnt);
  if ((tid & 63) == 0) ws[tid >> 6] = cnt;
  __syncthreads();
  if (tid == 0) blk[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Exclusive scan of nb block counts in one workgroup; total -> *total.
__global__ __launch_bounds__(1024) void scan_blocks_kernel(int32_t *__restrict__ blk, int64_t nb,
                                                           int32_t *__restrict__ total) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t i = base + tid;
    const int32_t v = i < nb ? blk[i] : 0;
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
    if (i < nb) blk[i] = excl;
    __syncthreads();
    if (tid == 1023) carry = excl + v;
    __syncthreads();
  }
  if (tid == 0) *total = carry;
}

// labels[root] = 1 + rank(root); background 0.  Non-roots filled by cc_fill_kernel.
__global__ __launch_bounds__(256) void cc_rank_roots_kernel(const int32_t *__restrict__ parent, int64_t n,
                                                            const int32_t *__restrict__ blk,
                                                            int32_t *__restrict__ labels) {
  __shared__ int32_t wc[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // pixel order inside the block: k*256 + tid; wave w covers [k*256 + 64w, +64)
  int flags[4];
  int pc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t p = (int64_t)blockIdx.x * NB + k * 256 + tid;
    flags[k] = (p < n && parent[p] == p);
    const unsigned long long b = __ballot(flags[k]);
    pc[k] = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wc[k * 4 + w] = __popcll(b);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t p = (int64_t)blockIdx.x * NB + k * 256 + tid;
    if (p >= n) continue;
    int before = 0;
    for (int q = 0; q < k * 4 + w; ++q) before += wc[q];
    if (flags[k]) labels[p] = blk[blockIdx.x] + before + pc[k] + 1;
    else if (parent[p] < 0) labels[p] = 0;
  }
}

__global__ void cc_fill_kernel(const int32_t *__restrict__ parent, int64_t n, int32_t *__restrict__ labels) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t q = parent[p];
    if (q >= 0 && q != p) labels[p] = labels[q];
  }
}

// component sizes at the root index (size[] zeroed by the caller); each wave counts RUN*64
// consecutive pixels (wave_run_count) so a giant component is one atomic per wave
__global__ void cc_sizes_kernel(const int32_t *__restrict__ parent, int64_t n, int32_t *__restrict__ size) {
  const int64_t nw = (n + RUN_PX - 1) / RUN_PX;
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t w = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); w < nw; w += (int64_t)gridDim.x * wpb)
    hrf::wave_run_count<RUN>(size, w * RUN_PX, n, [&](int64_t e) { return parent[e]; });
}

// rso / remove_small_holes finish: out = (fg && size[root] >= thr) ^ inv
__global__ void cc_keep_kernel(const int32_t *__restrict__ parent, const int32_t *__restrict__ size, int64_t n,
                               int64_t thr, int inv, uint8_t *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t q = parent[p];
    const int keep = q >= 0 && (int64_t)size[q] >= thr;
    out[p] = (uint8_t)(keep ^ inv);
  }
}

// erosion-seed freeze step (ecoli measurement.py:102-106): components smaller than thr
// join the seed mask, the others stay in play.
__global__ void split_by_size_kernel(const int32_t *__restrict__ parent, const int32_t *__restrict__ size, int64_t n,
                                     int64_t thr, uint8_t *__restrict__ small_or, uint8_t *__restrict__ large) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t q = parent[p];
    const bool fg = q >= 0;
    const bool sm = fg && (int64_t)size[q] < thr;
    if (sm) small_or[p] = 1;
    large[p] = (uint8_t)(fg && !sm);
  }
}

// flag[root] = 1 for components with a pixel on the 1-pixel frame
__global__ void border_roots_kernel(const int32_t *__restrict__ parent, int64_t H, int64_t W,
                                    int32_t *__restrict__ flag) {
  const int64_t nb = 2 * W + 2 * H;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nb; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p;
    if (e < W) p = e;
    else if (e < 2 * W) p = (H - 1) * W + (e - W);
    else if (e < 2 * W + H) p = (e - 2 * W) * W;
    else p = (e - 2 * W - H) * W + (W - 1);
    const int32_t q = parent[p];
    if (q >= 0) flag[q] = 1;
  }
}

__global__ void fill_holes_finish_kernel(const uint8_t *__restrict__ mask, const int32_t *__restrict__ parent,
                                         const int32_t *__restrict__ flag, int64_t n, uint8_t *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t q = parent[p];  // component of the background
    out[p] = (uint8_t)(mask[p] != 0 || (q >= 0 && !flag[q]));
  }
}

__global__ void clear_border_finish_kernel(const int32_t *__restrict__ lab, const int32_t *__restrict__ parent,
                                           const int32_t *__restrict__ flag, int64_t n, int32_t *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t q = parent[p];
    out[p] = (q >= 0 && flag[q]) ? 0 : lab[p];
  }
}

// rso on an int label image: counts per label value
__global__ void label_counts_kernel(const int32_t *__restrict__ lab, int64_t n, int32_t maxlab,
                                    int32_t *__restrict__ cnt) {
  const int64_t nw = (n + RUN_PX - 1) / RUN_PX;
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t w = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); w < nw; w += (int64_t)gridDim.x * wpb)
    hrf::wave_run_count<RUN>(cnt, w * RUN_PX, n, [&](int64_t e) {
      const int32_t l = lab[e];
      return (l > 0 && l <= maxlab) ? l : -1;
    });
}

__global__ void rso_labels_finish_kernel(const int32_t *__restrict__ lab, const int32_t *__restrict__ cnt,
                                         int64_t n, int32_t maxlab, int64_t thr, int32_t *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lab[p];
    out[p] = (l > 0 && l <= maxlab && (int64_t)cnt[l] < thr) ? 0 : l;
  }
}

// relabel_sequential: present flags -> exclusive scan -> map
__global__ void present_kernel(const int32_t *__restrict__ lab, int64_t n, int32_t maxlab,
                               int32_t *__restrict__ present) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lab[p];
    if (l > 0 && l <= maxlab) present[l] = 1;
  }
}

__global__ __launch_bounds__(1024) void scan_present_kernel(int32_t *__restrict__ m, int64_t len,
                                                            int32_t *__restrict__ total) {
  // in-place inclusive scan of flags -> map[l] = rank (1-based) for present labels, 0 else
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < len; base += 1024) {
    const int64_t i = base + tid;
    const int32_t v = i < len ? m[i] : 0;
    const int32_t inc = hrf::wave_inclusive_scan(v);
    if ((tid & 63) == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    if (tid < 64) {
      const int32_t s = tid < 16 ? wsum[tid] : 0;
      const int32_t si = hrf::wave_inclusive_scan(s);
      if (tid < 16) wsum[tid] = si - s;
    }
    __syncthreads();
    const int32_t incl = carry + wsum[tid >> 6] + inc;
    if (i < len) m[i] = v ? incl : 0;
    __syncthreads();
    if (tid == 1023) carry = incl;
    __syncthreads();
  }
  if (tid == 0) *total = carry;
}

__global__ void apply_map_kernel(const int32_t *__restrict__ lab, int64_t n, int32_t maxlab,
                                 const int32_t *__restrict__ map, int32_t *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lab[p];
    out[p] = (l > 0 && l <= maxlab) ? map[l] : 0;
  }
}

// ---- morphology (cross footprint) ------------------------------------------------------
__global__ void erode_kernel(const uint8_t *__restrict__ m, int64_t H, int64_t W, int border,
                             uint8_t *__restrict__ o) {
  const int64_t n = H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / W, c = i - r * W;
    int v = m[i] != 0;
    v = v && (r > 0 ? m[i - W] != 0 : border);
    v = v && (r + 1 < H ? m[i + W] != 0 : border);
    v = v && (c > 0 ? m[i - 1] != 0 : border);
    v = v && (c + 1 < W ? m[i + 1] != 0 : border);
    o[i] = (uint8_t)v;
  }
}

__global__ void dilate_kernel(const uint8_t *__restrict__ m, int64_t H, int64_t W, uint8_t *__restrict__ o) {
  const int64_t n = H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / W, c = i - r * W;
    const int v = m[i] || (r > 0 && m[i - W]) || (r + 1 < H && m[i + W]) || (c > 0 && m[i - 1]) ||
                  (c + 1 < W && m[i + 1]);
    o[i] = (uint8_t)v;
  }
}

// dilate(erode(m)) with the cross in one pass (the eroded image is not stored): a pixel is set
// when it or one of its in-image 4-neighbours q survives the erosion, q's erosion reading its
// own 4-neighbours with `border` outside the image -- erode_kernel then dilate_kernel, fused
__device__ __forceinline__ int eroded_at(const uint8_t *__restrict__ m, int64_t H, int64_t W, int border, int64_t r,
                                         int64_t c) {
  const int64_t i = r * W + c;
  int v = m[i] != 0;
  v = v && (r > 0 ? m[i - W] != 0 : border);
  v = v && (r + 1 < H ? m[i + W] != 0 : border);
  v = v && (c > 0 ? m[i - 1] != 0 : border);
  v = v && (c + 1 < W ? m[i + 1] != 0 : border);
  return v;
}

__global__ void opening_kernel(const uint8_t *__restrict__ m, int64_t H, int64_t W, int border,
                               uint8_t *__restrict__ o) {
  const int64_t n = H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / W, c = i - r * W;
    const int v = eroded_at(m, H, W, border, r, c) || (r > 0 && eroded_at(m, H, W, border, r - 1, c)) ||
                  (r + 1 < H && eroded_at(m, H, W, border, r + 1, c)) ||
                  (c > 0 && eroded_at(m, H, W, border, r, c - 1)) ||
                  (c + 1 < W && eroded_at(m, H, W, border, r, c + 1));
    o[i] = (uint8_t)v;
  }
}

__global__ void count_u8_kernel(const uint8_t *__restrict__ m, int64_t n, unsigned long long *__restrict__ cnt) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += m[i] != 0;
  c = hrf::wave_sum(c);
  __shared__ unsigned long long red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    c = red[0] + red[1] + red[2] + red[3];
    if (c) atomicAdd(cnt, c);
  }
}

__global__ void max_i32_kernel(const int32_t *__restrict__ a, int64_t n, int32_t *__restrict__ mx) {
  int32_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = a[i] > m ? a[i] : m;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t u = __shfl_xor(m, o, 64);
    m = u > m ? u : m;
  }
  __shared__ int32_t red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) m = red[q] > m ? red[q] : m;
    atomicMax(mx, m);
  }
}

// zero: an array the compression pass clears; sizes: component sizes counted at the roots by
// the compression pass itself (cleared by the tile pass)
template <class V>
hrf_status run_cc(V val, int64_t H, int64_t W, int conn, int32_t *parent, hipStream_t s, int32_t *zero = nullptr,
                  int32_t *sizes = nullptr) {
  dim3 g((unsigned)hrf::cdiv(W, CC_T), (unsigned)hrf::cdiv(H, CC_T));
  const unsigned gb = (unsigned)hrf::cdiv(hrf::cdiv(W, CC_T) * hrf::cdiv(H, CC_T) * CC_BORDER_PX, 256);
  if (conn == 2) {
    cc_local_kernel<V, 2><<<g, 256, 0, s>>>(val, H, W, parent, sizes);
    cc_border_kernel<V, 2><<<gb, 256, 0, s>>>(val, H, W, parent);
  } else {
    cc_local_kernel<V, 1><<<g, 256, 0, s>>>(val, H, W, parent, sizes);
    cc_border_kernel<V, 1><<<gb, 256, 0, s>>>(val, H, W, parent);
  }
  if (sizes)
    cc_compress_sizes_kernel<<<(unsigned)std::min<int64_t>(hrf::cdiv(H * W, RUN_PX * 4), 4096), 256, 0, s>>>(
        parent, H * W, sizes);
  else
    cc_compress_kernel<<<hrf::stream_grid(H * W), 256, 0, s>>>(parent, H * W, zero);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status check_hw(int64_t H, int64_t W, const char *who) {
  HRF_REQUIRE(H >= 0 && W >= 0 && H * W < (int64_t)INT32_MAX && H <= 65535, "%s: image too large (%lld x %lld)",
              who, (long long)H, (long long)W);
  return HRF_OK;
}

}  // namespace

extern "C" {

hrf_status hrf_cc_roots(const void *img, int32_t dtype, int64_t H, int64_t W, int32_t conn, int32_t *parent,
                        hrf_stream_t stream) {
  if (hrf_status s = check_hw(H, W, "cc_roots")) return s;
  HRF_REQUIRE(conn == 1 || conn == 2, "cc_roots: connectivity must be 1 or 2");
  HRF_REQUIRE(dtype == 0 || dtype == 1 || dtype == 2, "cc_roots: dtype must be 0 (u8), 1 (i32) or 2 (u8 inverted)");
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(img && parent, "cc_roots: null buffer");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) return run_cc(LabelV{(const int32_t *)img}, H, W, conn, parent, s);
  return run_cc(MaskV{(const uint8_t *)img, dtype == 2}, H, W, conn, parent, s);
}

hrf_status hrf_cc_number(const int32_t *parent, int64_t n, int32_t *labels, int32_t *blk_ws, int32_t *nlab_dev,
                         hrf_stream_t stream) {
  HRF_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "cc_number: size out of range");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    if (nlab_dev) HRF_HIP(hipMemsetAsync(nlab_dev, 0, sizeof(int32_t), s));
    return HRF_OK;
  }
  HRF_REQUIRE(parent && labels && blk_ws && nlab_dev, "cc_number: null buffer");
  const int64_t nb = hrf::cdiv(n, NB);
  cc_count_roots_kernel<<<(unsigned)nb, 256, 0, s>>>(parent, n, blk_ws);
  scan_blocks_kernel<<<1, 1024, 0, s>>>(blk_ws, nb, nlab_dev);
  cc_rank_roots_kernel<<<(unsigned)nb, 256, 0, s>>>(parent, n, blk_ws, labels);
  cc_fill_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(parent, n, labels);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_label(const void *img, int32_t dtype, int64_t H, int64_t W, int32_t conn, int32_t *labels,
                     int32_t *parent_ws, int32_t *blk_ws, int32_t *nlab_dev, hrf_stream_t stream) {
  if (hrf_status st = hrf_cc_roots(img, dtype, H, W, conn, parent_ws, stream)) return st;
  return hrf_cc_number(parent_ws, H * W, labels, blk_ws, nlab_dev, stream);
}

}  // extern "C"

extern "C" {

hrf_status hrf_cc_sizes(const int32_t *parent, int64_t n, int32_t *size, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(parent && size, "cc_sizes: null buffer");
  HRF_HIP(hipMemsetAsync(size, 0, sizeof(int32_t) * n, s));
  cc_sizes_kernel<<<(unsigned)std::min<int64_t>(hrf::cdiv(n, RUN_PX * 4), 4096), 256, 0, s>>>(parent, n, size);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"

namespace {
// hrf_cc_roots + hrf_cc_sizes with the size array cleared by the compression pass
hrf_status cc_roots_sizes(const uint8_t *mask, int dtype, int64_t H, int64_t W, int conn, int32_t *parent,
                          int32_t *size, hipStream_t s) {
  if (hrf_status st = check_hw(H, W, "cc_roots")) return st;
  HRF_REQUIRE(conn == 1 || conn == 2, "cc_roots: connectivity must be 1 or 2");
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(mask && parent && size, "cc_roots: null buffer");
  return run_cc(MaskV{mask, dtype == 2}, H, W, conn, parent, s, nullptr, size);
}
}  // namespace

extern "C" {

hrf_status hrf_remove_small_objects_mask(const uint8_t *mask, int64_t H, int64_t W, int64_t min_size, int32_t conn,
                                         uint8_t *out, int32_t *parent_ws, int32_t *size_ws, hrf_stream_t stream) {
  const int64_t n = H * W;
  if (n == 0) return HRF_OK;
  if (hrf_status st = cc_roots_sizes(mask, 0, H, W, conn, parent_ws, size_ws, (hipStream_t)stream)) return st;
  cc_keep_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(parent_ws, size_ws, n, min_size, 0, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_remove_small_holes(const uint8_t *mask, int64_t H, int64_t W, int64_t area_threshold, int32_t conn,
                                  uint8_t *out, int32_t *parent_ws, int32_t *size_ws, hrf_stream_t stream) {
  const int64_t n = H * W;
  if (n == 0) return HRF_OK;
  if (hrf_status st = cc_roots_sizes(mask, 2, H, W, conn, parent_ws, size_ws, (hipStream_t)stream)) return st;
  cc_keep_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(parent_ws, size_ws, n, area_threshold, 1,
                                                                        out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_split_by_size(const uint8_t *mask, int64_t H, int64_t W, int32_t conn, int64_t thr, uint8_t *small_or,
                             uint8_t *large, int32_t *parent_ws, int32_t *size_ws, hrf_stream_t stream) {
  const int64_t n = H * W;
  if (n == 0) return HRF_OK;
  if (hrf_status st = cc_roots_sizes(mask, 0, H, W, conn, parent_ws, size_ws, (hipStream_t)stream)) return st;
  split_by_size_kernel<<<hrf::stream_grid(n), 256, 0, (hipStream_t)stream>>>(parent_ws, size_ws, n, thr, small_or,
                                                                              large);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_fill_holes(const uint8_t *mask, int64_t H, int64_t W, uint8_t *out, int32_t *parent_ws,
                          int32_t *flag_ws, hrf_stream_t stream) {
  const int64_t n = H * W;
  hipStream_t s = (hipStream_t)stream;
  if (hrf_status st = check_hw(H, W, "fill_holes")) return st;
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(mask && out && parent_ws && flag_ws, "fill_holes: null buffer");
  // the compression pass clears the root flags (no memset launch)
  if (hrf_status st = run_cc(MaskV{mask, 1}, H, W, 1, parent_ws, s, flag_ws)) return st;
  border_roots_kernel<<<hrf::stream_grid(2 * (H + W)), 256, 0, s>>>(parent_ws, H, W, flag_ws);
  fill_holes_finish_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(mask, parent_ws, flag_ws, n, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_clear_border(const int32_t *labels, int64_t H, int64_t W, int32_t *out, int32_t *parent_ws,
                            int32_t *flag_ws, hrf_stream_t stream) {
  const int64_t n = H * W;
  hipStream_t s = (hipStream_t)stream;
  if (hrf_status st = check_hw(H, W, "clear_border")) return st;
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(labels && out && parent_ws && flag_ws, "clear_border: null buffer");
  if (hrf_status st = run_cc(LabelV{labels}, H, W, 2, parent_ws, s, flag_ws)) return st;
  border_roots_kernel<<<hrf::stream_grid(2 * (H + W)), 256, 0, s>>>(parent_ws, H, W, flag_ws);
  clear_border_finish_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(labels, parent_ws, flag_ws, n, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_remove_small_objects_labels(const int32_t *labels, int64_t n, int32_t maxlab, int64_t min_size,
                                           int32_t *out, int32_t *cnt_ws, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(cnt_ws && maxlab >= 0, "remove_small_objects_labels: bad arguments");
  HRF_HIP(hipMemsetAsync(cnt_ws, 0, sizeof(int32_t) * ((size_t)maxlab + 1), s));
  return hrf::remove_small_objects_labels_zeroed(labels, n, maxlab, min_size, out, cnt_ws, s);
}

}  // extern "C"

hrf_status hrf::remove_small_objects_labels_zeroed(const int32_t *labels, int64_t n, int32_t maxlab,
                                                   int64_t min_size, int32_t *out, int32_t *cnt_ws, hipStream_t s) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(labels && out && cnt_ws && maxlab >= 0, "remove_small_objects_labels: bad arguments");
  label_counts_kernel<<<(unsigned)std::min<int64_t>(hrf::cdiv(n, RUN_PX * 4), 4096), 256, 0, s>>>(labels, n, maxlab, cnt_ws);
  rso_labels_finish_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(labels, cnt_ws, n, maxlab, min_size, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

extern "C" {

hrf_status hrf_relabel_sequential(const int32_t *labels, int64_t n, int32_t maxlab, int32_t *out, int32_t *map_ws,
                                  int32_t *nlab_dev, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && map_ws && nlab_dev, "relabel_sequential: bad arguments");
  HRF_HIP(hipMemsetAsync(map_ws, 0, sizeof(int32_t) * ((size_t)maxlab + 1), s));
  if (n > 0) present_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(labels, n, maxlab, map_ws);
  scan_present_kernel<<<1, 1024, 0, s>>>(map_ws, (int64_t)maxlab + 1, nlab_dev);
  if (n > 0) apply_map_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(labels, n, maxlab, map_ws, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_binary_erosion(const uint8_t *mask, int64_t H, int64_t W, int32_t border_value, uint8_t *out,
                              hrf_stream_t stream) {
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(mask && out && mask != out, "binary_erosion: bad buffers (in-place not supported)");
  erode_kernel<<<hrf::stream_grid(H * W), 256, 0, (hipStream_t)stream>>>(mask, H, W, border_value != 0, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"

// hrf_label(mask, u8) with the component count left in device memory (nlab_dev) for a later
// read-back.  blk_ws: label_dev_ws_words(n) int32.  (Round 4 also built a last-block scan behind
// an agent-scope ticket here -- one launch less, an L2 write-back + invalidate per block; it lost
// end to end and was removed in round 5, profiles/r4h_ticket_ab.txt, r4i_fusion_ab.txt.)
int64_t hrf::label_dev_ws_words(int64_t n) { return hrf::cdiv(n, NB) + 4; }

hrf_status hrf::label_dev(const uint8_t *mask, int64_t H, int64_t W, int32_t conn, int32_t *labels,
                          int32_t *parent_ws, int32_t *blk_ws, int32_t *nlab_dev, hipStream_t s) {
  if (hrf_status st = check_hw(H, W, "label")) return st;
  HRF_REQUIRE(conn == 1 || conn == 2, "label: connectivity must be 1 or 2");
  const int64_t n = H * W;
  HRF_REQUIRE(n > 0 && mask && labels && parent_ws && blk_ws && nlab_dev, "label: bad arguments");
  const int64_t nb = hrf::cdiv(n, NB);
  if (hrf_status st = run_cc(MaskV{mask, false}, H, W, conn, parent_ws, s)) return st;
  cc_count_roots_kernel<<<(unsigned)nb, 256, 0, s>>>(parent_ws, n, blk_ws);
  scan_blocks_kernel<<<1, 1024, 0, s>>>(blk_ws, nb, nlab_dev);
  cc_rank_roots_kernel<<<(unsigned)nb, 256, 0, s>>>(parent_ws, n, blk_ws, labels);
  cc_fill_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(parent_ws, n, labels);
  HRF_LAUNCHED();
  return HRF_OK;
}

// hrf_binary_erosion(mask, border_value) then hrf_binary_dilation, one launch
hrf_status hrf::binary_opening(const uint8_t *mask, int64_t H, int64_t W, int32_t border_value, uint8_t *out,
                               hipStream_t s) {
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(mask && out && mask != out, "binary_opening: bad buffers (in-place not supported)");
  opening_kernel<<<hrf::stream_grid(H * W), 256, 0, s>>>(mask, H, W, border_value != 0, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

extern "C" {

hrf_status hrf_binary_dilation(const uint8_t *mask, int64_t H, int64_t W, uint8_t *out, hrf_stream_t stream) {
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(mask && out && mask != out, "binary_dilation: bad buffers (in-place not supported)");
  dilate_kernel<<<hrf::stream_grid(H * W), 256, 0, (hipStream_t)stream>>>(mask, H, W, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_count_nonzero_u8(const uint8_t *mask, int64_t n, int64_t *count_dev, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(count_dev, "count_nonzero: null output");
  HRF_HIP(hipMemsetAsync(count_dev, 0, sizeof(int64_t), s));
  if (n == 0) return HRF_OK;
  count_u8_kernel<<<std::min<unsigned>(hrf::stream_grid(n), 512), 256, 0, s>>>(mask, n, (unsigned long long *)count_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_max_i32(const int32_t *a, int64_t n, int32_t *max_dev, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(max_dev, "max_i32: null output");
  HRF_HIP(hipMemsetAsync(max_dev, 0, sizeof(int32_t), s));
  if (n == 0) return HRF_OK;
  max_i32_kernel<<<std::min<unsigned>(hrf::stream_grid(n), 512), 256, 0, s>>>(a, n, max_dev);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
