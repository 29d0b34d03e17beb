// seeds.hip -- the E. coli erosion-seeding loop (a11) in ONE launch.
//
// Reference (ecoli measurement.py:97-110): while any region is left: regions (8-connected)
// with area < 600 become seeds and leave the mask; the rest is eroded (cross, border True);
// 4-connected fragments < 10 px are dropped; relabel; repeat.
// None of these steps lets information cross an 8-connected component of the starting mask:
// a pixel's cross neighbours are 8-adjacent (same component), 4-components and 8-components
// of a subset stay inside the component, and each component's loop ends when it is empty.
// So every component of `cell_sm` runs the loop independently, to the end, in one workgroup:
//  * erosion_seed_runs_kernel (one workgroup per component, 32 KB LDS): the box as bit planes,
//    connected components over horizontal runs -- every component whose planes fit, large
//    boxes included (SEED_BIG_RUNS);
//  * erosion_seed_kernel: the components the run kernel hands over (its run arrays full, or
//    planes that do not fit), 1 flag byte + parent + size per pixel of the box (<= 18176 px)
//    in a global scratch slice per workgroup;
//  * whole-image passes over a crop holding the rest (boxes above 18176 px whose planes do not
//    fit, or every large box when a large-box component overflowed the run kernel and the
//    caller redoes the stage), padded with one background row/column wherever the crop edge is
//    not the image edge (so the erosion's border_value=True applies only at the true border).
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "wave.hpp"

namespace {

// the pixel kernel's box capacity (9 B per pixel of scratch: the 160 KB it once took in LDS)
constexpr int SEED_LDS_PX_MAX = 18176;

constexpr int RS_T = 256;
constexpr int RS_LDS = 32768;
constexpr int RS_MIN_CAP = 96;

struct RunBox {
  uint64_t *m, *t, *sd;
  int *off, *part;
  uint16_t *c0, *c1, *row;
  int *par, *sz;
  int cap;
};

__host__ __device__ inline int rs_bytes_fixed(int bh, int w64) {
  return 24 * bh * w64 + 4 * (bh + 1) + 4 * RS_T + 64;
}

// 0: run-length kernel (32 KB LDS), 1: pixel kernel (160 KB LDS), 2: whole-image loop on a
// crop; -1: no pixels.  Evaluated on the host (dispatch) and in the kernels from the same
// boxes, so no class table travels host -> device.  mode bit 0: the run kernel is in use
// (HRF_SEEDS_RUNS); bit 1 (SEED_BIG_RUNS): a box above the pixel kernel's capacity still goes
// to the run kernel when its bit planes fit -- a clump of cells on a diagonal has a large box
// but few pixels and runs.  Should such a component overflow its run arrays, the run kernel
// counts it (it has no device fallback) and the caller redoes the stage without bit 1.
constexpr int SEED_BIG_RUNS = 2;
__host__ __device__ inline int seed_class(const int32_t *box, int comp, int mode) {
  const int64_t bh = (int64_t)box[comp * 4 + 2] - box[comp * 4 + 0] + 1;
  const int64_t bw = (int64_t)box[comp * 4 + 3] - box[comp * 4 + 1] + 1;
  if (bh <= 0 || bw <= 0) return -1;
  const bool runs_fit = (mode & 1) && bw <= 65535 && bh <= 65535 &&
                        rs_bytes_fixed((int)bh, (int)((bw + 63) >> 6)) + 14 * RS_MIN_CAP <= RS_LDS;
  if (runs_fit && (mode & SEED_BIG_RUNS)) return 0;
  if (bh * bw > SEED_LDS_PX_MAX) return 2;
  return runs_fit ? 0 : 1;
}


// find with path halving: a box is up to 18K px and the raster-order unions would otherwise
// build parent chains as long as a row run (quadratic finds).  A halving store only ever
// points a node at one of its ancestors (all links go to smaller indices, so no cycles); a
// concurrent atomicMin it overwrites belongs to a union that saw a non-root and retries.
__device__ __forceinline__ int sfind(int32_t *par, int x) {
  volatile int32_t *v = par;
  for (;;) {
    const int y = v[x];
    if (y == x) return x;
    const int z = v[y];
    if (z == y) return y;
    v[x] = z;
    x = z;
  }
}

// read-only find for the flatten pass.  A flatten store (par[x] = root) racing with a
// path-halving store from another thread's find (par[x] = a stale grandparent) could leave x
// pointing at a non-root and its size counted there; with no halving during the flatten, every
// store is a root and concurrent walks still end at it.
__device__ __forceinline__ int sfind_ro(const int32_t *par, int x) {
  const volatile int32_t *v = par;
  int y = v[x];
  while (y != x) {
    x = y;
    y = v[x];
  }
  return x;
}

__device__ __forceinline__ void sunion(int32_t *par, int a, int b) {
  for (;;) {
    a = sfind(par, a);
    b = sfind(par, b);
    if (a == b) return;
    if (a < b) {
      const int t = a;
      a = b;
      b = t;
    }
    const int old = atomicMin(&par[a], b);
    if (old == a) return;
    a = old;
  }
}

// components of flag bit0 inside the box; par[p] = root, sz[root] = size
__device__ void box_cc(uint8_t *fl, int32_t *par, int32_t *sz, int bh, int bw, bool conn8) {
  const int n = bh * bw;
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    par[p] = (fl[p] & 1) ? p : -1;
    sz[p] = 0;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    if (!(fl[p] & 1)) continue;
    const int r = p / bw, c = p - r * bw;
    if (c > 0 && (fl[p - 1] & 1)) sunion(par, p, p - 1);
    if (r > 0) {
      if (fl[p - bw] & 1) sunion(par, p, p - bw);
      if (conn8) {
        if (c > 0 && (fl[p - bw - 1] & 1)) sunion(par, p, p - bw - 1);
        if (c + 1 < bw && (fl[p - bw + 1] & 1)) sunion(par, p, p - bw + 1);
      }
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < n; p += blockDim.x)
    if (fl[p] & 1) par[p] = sfind_ro(par, p);
  __syncthreads();
  const int n_up = (n + 63) & ~63;  // whole waves: one LDS atomic per distinct root per wave
  for (int p = threadIdx.x; p < n_up; p += blockDim.x) {
    const bool in = p < n && (fl[p] & 1);
    hrf::agg_atomic_add<int32_t>(sz, in ? par[p] : 0, 1, in);
  }
  __syncthreads();
}

// flags: bit0 = in play (dist_lab != 0), bit1 = seed (dist_be), bit2 = erosion result
// one component in a scratch slice (box <= SEED_LDS_PX_MAX pixels)
__device__ void seed_component_px(char *lds, const int32_t *__restrict__ labels, int64_t H, int64_t W,
                                  const int32_t *__restrict__ box, int comp, int32_t area_max, int32_t min_obj,
                                  uint8_t *__restrict__ be_out) {
  const int r0 = box[comp * 4 + 0], c0 = box[comp * 4 + 1], r1 = box[comp * 4 + 2], c1 = box[comp * 4 + 3];
  if (r1 < r0 || c1 < c0) return;
  const int bh = r1 - r0 + 1, bw = c1 - c0 + 1, n = bh * bw;
  uint8_t *fl = reinterpret_cast<uint8_t *>(lds);
  int32_t *par = reinterpret_cast<int32_t *>(lds + ((n + 15) & ~15));
  int32_t *sz = par + n;
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    const int r = p / bw, c = p - r * bw;
    fl[p] = labels[(int64_t)(r0 + r) * W + (c0 + c)] == comp ? 1 : 0;
  }
  __syncthreads();
  for (int it = 0; it < 4 * (bh + bw) + 8; ++it) {
    // :102-106 regions (8-connected) below area_max become seeds
    box_cc(fl, par, sz, bh, bw, true);
    for (int p = threadIdx.x; p < n; p += blockDim.x)
      if ((fl[p] & 1) && sz[par[p]] < area_max) fl[p] = (uint8_t)((fl[p] & ~1) | 2);
    __syncthreads();
    // :107 binary_erosion (cross, border_value True at the image edge; outside the box but
    // inside the image is another component's or background territory -> False)
    for (int p = threadIdx.x; p < n; p += blockDim.x) {
      const int r = p / bw, c = p - r * bw;
      bool v = fl[p] & 1;
      if (v) {
        v = v && (r > 0 ? (fl[p - bw] & 1) != 0 : (r0 == 0));
        v = v && (r + 1 < bh ? (fl[p + bw] & 1) != 0 : (r1 == H - 1));
        v = v && (c > 0 ? (fl[p - 1] & 1) != 0 : (c0 == 0));
        v = v && (c + 1 < bw ? (fl[p + 1] & 1) != 0 : (c1 == W - 1));
      }
      if (v) fl[p] |= 4;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < n; p += blockDim.x) fl[p] = (uint8_t)((fl[p] & 2) | ((fl[p] >> 2) & 1));
    __syncthreads();
    // :108 remove_small_objects(., min_obj), 4-connected
    box_cc(fl, par, sz, bh, bw, false);
    int any = 0;
    for (int p = threadIdx.x; p < n; p += blockDim.x)
      if (fl[p] & 1) {
        if (sz[par[p]] < min_obj)
          fl[p] &= (uint8_t)~1;
        else
          any = 1;
      }
    if (!__syncthreads_or(any)) break;
  }
  for (int p = threadIdx.x; p < n; p += blockDim.x)
    if (fl[p] & 2) {
      const int r = p / bw, c = p - r * bw;
      be_out[(int64_t)(r0 + r) * W + (c0 + c)] = 1;
    }
}

// the components the run kernel hands over (class 1, or over its run capacity), listed on the
// device: a few 256-thread workgroups walk the list, each with a 164 KB slice of global scratch.  Not LDS:
// the kernel is launched for every tile but usually finds the list empty (no component of the
// bench tiles reaches it), and a 160 KB-LDS workgroup cannot be dispatched until a whole CU's
// LDS is free -- with the classifier's workgroups resident that wait was 0.2-1.6 ms of an
// empty launch in the segmentation chain.  The rare real work pays L2 atomics instead.
constexpr size_t SEED_SLICE = ((SEED_LDS_PX_MAX + 15) & ~15) + 8 * (size_t)SEED_LDS_PX_MAX;
constexpr int SEED_PX_WG = 16;
__global__ __launch_bounds__(256) void erosion_seed_kernel(const int32_t *__restrict__ labels, int64_t H, int64_t W,
                                                           const int32_t *__restrict__ box,
                                                           const int32_t *__restrict__ list,
                                                           const int32_t *__restrict__ count, int32_t area_max,
                                                           int32_t min_obj, char *__restrict__ scratch,
                                                           uint8_t *__restrict__ be_out) {
  const int n = *count;
  char *mem = scratch + (size_t)blockIdx.x * SEED_SLICE;
  for (int idx = blockIdx.x; idx < n; idx += gridDim.x) {
    seed_component_px(mem, labels, H, W, box, list[idx], area_max, min_obj, be_out);
    __syncthreads();
  }
}

// ---- run-length variant -----------------------------------------------------------------------
// The same per-component loop on a bit-packed box (one u64 word = 64 columns of a row) with
// connected components over horizontal RUNS instead of pixels: a run is a node, runs of
// adjacent rows that overlap (4-connected) or touch diagonally (8-connected) are united, a
// component's size is the sum of its run lengths.  The erosion is word-parallel bit
// arithmetic, freezing / sieving clears whole runs with LDS word atomics.  A box of a few
// touching cells holds a few hundred runs against thousands of pixels, so an iteration is a
// handful of short passes.  Run arrays have a fixed LDS capacity; a component whose run count
// exceeds it at any iteration stops without writing and is flagged for the pixel kernel.
__device__ __forceinline__ uint64_t rs_valid(int w, int w64, int bw) {
  return (w < w64 - 1 || (bw & 63) == 0) ? ~0ull : ((1ull << (bw & 63)) - 1);
}

// block-wide exclusive scan of off[0..bh) in place; off[bh] = total.  Returns the total.
__device__ int rs_scan_rows(int *off, int *part, int bh) {
  const int t = threadIdx.x;
  const int chunk = (bh + RS_T - 1) / RS_T;
  const int lo = t * chunk, hi = min(bh, lo + chunk);
  int acc = 0;
  for (int r = lo; r < hi; ++r) acc += off[r];
  // exclusive scan of the per-thread sums: shuffles within each wave, wave totals in part[]
  const int incl = hrf::wave_inclusive_scan(acc);
  const int wave = t >> 6;
  if ((t & 63) == 63) part[wave] = incl;
  __syncthreads();
  int wbase = 0, all = 0;
#pragma unroll
  for (int i = 0; i < RS_T / 64; ++i) {
    const int v = part[i];
    wbase += i < wave ? v : 0;
    all += v;
  }
  if (t == 0) off[bh] = all;
  int base = wbase + incl - acc;
  for (int r = lo; r < hi; ++r) {
    const int v = off[r];
    off[r] = base;
    base += v;
  }
  __syncthreads();
  return off[bh];
}

// runs of the current mask, row-major, ascending columns within a row.  -1: over capacity.
__device__ int rs_extract(RunBox &B, int bh, int w64) {
  for (int r = threadIdx.x; r < bh; r += RS_T) {
    int cnt = 0;
    uint64_t prev = 0;
    for (int w = 0; w < w64; ++w) {
      const uint64_t x = B.m[r * w64 + w];
      cnt += __popcll(x & ~((x << 1) | prev));
      prev = x >> 63;
    }
    B.off[r] = cnt;
  }
  __syncthreads();
  const int total = rs_scan_rows(B.off, B.part, bh);
  if (total > B.cap) return -1;
  for (int r = threadIdx.x; r < bh; r += RS_T) {
    int k = B.off[r], start = 0;
    uint64_t prev = 0;
    for (int w = 0; w < w64; ++w) {
      const uint64_t x = B.m[r * w64 + w];
      const uint64_t nxt = w + 1 < w64 ? B.m[r * w64 + w + 1] : 0ull;
      uint64_t st = x & ~((x << 1) | prev);
      uint64_t en = x & ~((x >> 1) | (nxt << 63));
      prev = x >> 63;
      while (st | en) {
        const int bs = st ? __ffsll((long long)st) - 1 : 64;
        const int be = en ? __ffsll((long long)en) - 1 : 64;
        if (bs <= be) {
          start = w * 64 + bs;
          st &= st - 1;
        } else {
          B.c0[k] = (uint16_t)start;
          B.c1[k] = (uint16_t)(w * 64 + be);
          B.row[k] = (uint16_t)r;
          ++k;
          en &= en - 1;
        }
      }
    }
  }
  __syncthreads();
  return total;
}

// union of runs in adjacent rows (d = 1: 8-connected, 0: 4-connected); par[i] = root,
// sz[root] = pixels
__device__ void rs_components(RunBox &B, int total, int d) {
  for (int i = threadIdx.x; i < total; i += RS_T) {
    B.par[i] = i;
    B.sz[i] = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < total; i += RS_T) {
    const int r = B.row[i];
    if (r == 0) continue;
    int lo = B.off[r - 1], hi = B.off[r];
    const int a = (int)B.c0[i] - d, b = (int)B.c1[i] + d;
    while (lo < hi) {   // first run of the previous row ending at or after a
      const int mid = (lo + hi) >> 1;
      if ((int)B.c1[mid] < a) lo = mid + 1;
      else hi = mid;
    }
    for (int j = lo; j < B.off[r] && (int)B.c0[j] <= b; ++j) sunion(B.par, i, j);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < total; i += RS_T) B.par[i] = sfind_ro(B.par, i);
  __syncthreads();
  for (int i = threadIdx.x; i < total; i += RS_T) atomicAdd(&B.sz[B.par[i]], (int)B.c1[i] - (int)B.c0[i] + 1);
  __syncthreads();
}

__device__ void rs_clear_run(uint64_t *m, uint64_t *sd, int base, int c0, int c1) {
  for (int w = c0 >> 6; w <= (c1 >> 6); ++w) {
    const int lo = w == (c0 >> 6) ? (c0 & 63) : 0;
    const int hi = w == (c1 >> 6) ? (c1 & 63) : 63;
    const uint64_t mask = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
    atomicAnd((unsigned long long *)&m[base + w], (unsigned long long)~mask);
    if (sd) atomicOr((unsigned long long *)&sd[base + w], (unsigned long long)mask);
  }
}

__global__ __launch_bounds__(RS_T) void erosion_seed_runs_kernel(const int32_t *__restrict__ labels, int64_t H,
                                                                 int64_t W, const int32_t *__restrict__ box,
                                                                 int32_t mode, int32_t area_max,
                                                                 int32_t min_obj, int32_t *__restrict__ list,
                                                                 int32_t *__restrict__ count,
                                                                 uint8_t *__restrict__ be_out,
                                                                 int32_t *__restrict__ ovf) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int comp = blockIdx.x + 1;
  const int cls = seed_class(box, comp, mode);
  if (cls == 1 && threadIdx.x == 0) list[atomicAdd(count, 1)] = comp;
  if (cls != 0) return;
  const int r0 = box[comp * 4 + 0], c0 = box[comp * 4 + 1], r1 = box[comp * 4 + 2], c1 = box[comp * 4 + 3];
  if (r1 < r0 || c1 < c0) return;
  const int bh = r1 - r0 + 1, bw = c1 - c0 + 1, w64 = (bw + 63) >> 6, nw = bh * w64;
  RunBox B;
  B.m = reinterpret_cast<uint64_t *>(lds);
  B.t = B.m + nw;
  B.sd = B.t + nw;
  B.off = reinterpret_cast<int *>(B.sd + nw);
  B.part = B.off + bh + 1;
  char *rp = reinterpret_cast<char *>(B.part + RS_T);
  B.cap = (RS_LDS - rs_bytes_fixed(bh, w64)) / 14;
  B.par = reinterpret_cast<int *>(rp);
  B.sz = B.par + B.cap;
  B.c0 = reinterpret_cast<uint16_t *>(B.sz + B.cap);
  B.c1 = B.c0 + B.cap;
  B.row = B.c1 + B.cap;
  // the component's pixels as bits, one wave per (row, word)
  const int lane = hrf::lane_id(), wave = threadIdx.x >> 6;
  for (int q = wave; q < nw; q += RS_T / 64) {
    const int r = q / w64, w = q - r * w64;
    const int c = w * 64 + lane;
    const bool in = c < bw && labels[(int64_t)(r0 + r) * W + (c0 + c)] == comp;
    const uint64_t word = __ballot(in);
    if (lane == 0) {
      B.m[q] = word;
      B.sd[q] = 0;
    }
  }
  __syncthreads();
  const uint64_t up_border = r0 == 0 ? ~0ull : 0ull, down_border = r1 == H - 1 ? ~0ull : 0ull;
  const uint64_t left_border = c0 == 0 ? 1ull : 0ull, right_border = c1 == W - 1 ? 1ull : 0ull;
  for (int it = 0; it < 4 * (bh + bw) + 8; ++it) {
    // :102-106 regions (8-connected) below area_max become seeds
    int total = rs_extract(B, bh, w64);
    if (total < 0) break;
    rs_components(B, total, 1);
    for (int i = threadIdx.x; i < total; i += RS_T)
      if (B.sz[B.par[i]] < area_max) rs_clear_run(B.m, B.sd, B.row[i] * w64, B.c0[i], B.c1[i]);
    __syncthreads();
    // :107 binary_erosion (cross; border True only at the image edge)
    for (int q = threadIdx.x; q < nw; q += RS_T) {
      const int r = q / w64, w = q - r * w64;
      uint64_t x = B.m[q];
      const uint64_t up = r > 0 ? B.m[q - w64] : up_border;
      const uint64_t dn = r + 1 < bh ? B.m[q + w64] : down_border;
      const uint64_t lft = (x << 1) | (w > 0 ? (B.m[q - 1] >> 63) : left_border);
      uint64_t xe = x;
      uint64_t nb;
      if (w + 1 < w64) {
        nb = B.m[q + 1] & 1ull;
      } else if (bw & 63) {
        xe |= right_border << (bw & 63);   // the column right of the box, as a padding bit
        nb = 0;
      } else {
        nb = right_border;
      }
      const uint64_t rgt = (xe >> 1) | (nb << 63);
      B.t[q] = x & up & dn & lft & rgt & rs_valid(w, w64, bw);
    }
    __syncthreads();
    {
      uint64_t *tmp = B.m;
      B.m = B.t;
      B.t = tmp;
    }
    // :108 remove_small_objects(., min_obj), 4-connected
    total = rs_extract(B, bh, w64);
    if (total < 0) break;
    rs_components(B, total, 0);
    int any = 0;
    for (int i = threadIdx.x; i < total; i += RS_T) {
      if (B.sz[B.par[i]] < min_obj) rs_clear_run(B.m, nullptr, B.row[i] * w64, B.c0[i], B.c1[i]);
      else any = 1;
    }
    if (!__syncthreads_or(any)) {
      // done: write the seeds
      for (int q = threadIdx.x; q < nw; q += RS_T) {
        uint64_t x = B.sd[q];
        const int r = q / w64, w = q - r * w64;
        while (x) {
          const int b = __ffsll((long long)x) - 1;
          x &= x - 1;
          be_out[(int64_t)(r0 + r) * W + (c0 + w * 64 + b)] = 1;
        }
      }
      return;
    }
  }
  // over capacity (or the iteration cap): the pixel kernel redoes this component -- unless its
  // box exceeds the pixel kernel's capacity (SEED_BIG_RUNS): then count[1] tells the caller
  if (threadIdx.x == 0) {
    if ((int64_t)bh * bw > SEED_LDS_PX_MAX) {
      atomicAdd(count + 1, 1);
      if (ovf) atomicAdd(ovf, 1);  // the caller's copy of count[1] (no device-to-device copy)
    } else {
      list[atomicAdd(count, 1)] = comp;
    }
  }
}

// crop (with padding) of the oversized components' pixels
__global__ void big_crop_kernel(const int32_t *__restrict__ labels, int64_t H, int64_t W, const int32_t *__restrict__ box,
                                int32_t ncomp, int mode, int64_t r0, int64_t c0, int64_t h, int64_t w,
                                uint8_t *__restrict__ m) {
  const int64_t n = h * w;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = r0 + i / w, c = c0 + i % w;
    uint8_t v = 0;
    if (r >= 0 && r < H && c >= 0 && c < W) {
      const int32_t l = labels[r * W + c];
      v = l > 0 && l <= ncomp && seed_class(box, l, mode) == 2;
    }
    m[i] = v;
  }
}

__global__ void big_paste_kernel(const uint8_t *__restrict__ be_crop, int64_t H, int64_t W, int64_t r0, int64_t c0,
                                 int64_t h, int64_t w, uint8_t *__restrict__ be_out) {
  const int64_t n = h * w;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = r0 + i / w, c = c0 + i % w;
    if (be_crop[i] && r >= 0 && r < H && c >= 0 && c < W) be_out[r * W + c] = 1;
  }
}

__global__ void box_init_kernel(int32_t *box, int32_t maxlab) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l > maxlab) return;
  box[l * 4 + 0] = 0x7fffffff;
  box[l * 4 + 1] = 0x7fffffff;
  box[l * 4 + 2] = -1;
  box[l * 4 + 3] = -1;
}

// per-label bounding boxes; atomics aggregated per distinct label in the wave
__global__ void box_kernel(const int32_t *__restrict__ lab, int64_t H, int64_t W, int32_t maxlab,
                           int32_t *__restrict__ box) {
  const int64_t n = H * W;
  const int64_t n_up = (n + 63) / 64 * 64;
  const int lane = hrf::lane_id();
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_up; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = p < n ? lab[p] : 0;
    bool active = l > 0 && l <= maxlab;
    const int32_t r = (int32_t)(p / W), c = (int32_t)(p - (p / W) * W);
    // the wave's 64 pixels on one image row (always, when 64 divides W): a label's box within
    // the wave is its first and last lane -- no reductions
    const int64_t pb = p - lane, rb = pb / W;
    const bool one_row = pb + 63 < n && (pb + 63) / W == rb;
    unsigned long long pending = __ballot(active);
    while (pending) {
      const int leader = __ffsll((long long)pending) - 1;
      const int32_t k = __shfl(l, leader, 64);
      const bool m = active && l == k;
      const unsigned long long same = __ballot(m);
      int32_t rmin, cmin, rmax, cmax;
      if (one_row) {
        const int32_t cb = (int32_t)(pb - rb * W);
        rmin = rmax = (int32_t)rb;
        cmin = cb + leader;
        cmax = cb + 63 - __builtin_clzll(same);
      } else {
        rmin = m ? r : 0x7fffffff, cmin = m ? c : 0x7fffffff, rmax = m ? r : -1, cmax = m ? c : -1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          rmin = min(rmin, __shfl_xor(rmin, o, 64));
          cmin = min(cmin, __shfl_xor(cmin, o, 64));
          rmax = max(rmax, __shfl_xor(rmax, o, 64));
          cmax = max(cmax, __shfl_xor(cmax, o, 64));
        }
      }
      if (lane == leader) {
        atomicMin(&box[k * 4 + 0], rmin);
        atomicMin(&box[k * 4 + 1], cmin);
        atomicMax(&box[k * 4 + 2], rmax);
        atomicMax(&box[k * 4 + 3], cmax);
      }
      if (m) active = false;
      pending &= ~same;
    }
  }
}

// Pool of pixel-kernel scratch buffers for the standalone hrf_erosion_seeds (the native
// drivers pass their context's).  A buffer is leased for one call; the lease's destructor
// synchronises the call's stream and returns the buffer only if that succeeded (a stream in
// error keeps its buffer out of circulation).  Pool size = the peak number of concurrent
// calls per device; the buffers live for the process.
struct PxScratchPool {
  std::mutex mu;
  std::map<int, std::vector<char *>> idle;
};
PxScratchPool &px_pool() {
  static PxScratchPool *p = new PxScratchPool;  // never destroyed: outlives late callers
  return *p;
}
struct PxScratchLease {
  int dev;
  hipStream_t s;
  char *buf = nullptr;
  PxScratchLease(int d, hipStream_t st) : dev(d), s(st) {}
  hipError_t acquire() {
    {
      std::lock_guard<std::mutex> g(px_pool().mu);
      auto &v = px_pool().idle[dev];
      if (!v.empty()) {
        buf = v.back();
        v.pop_back();
        return hipSuccess;
      }
    }
    return hipMalloc((void **)&buf, (size_t)::hrf::seed_px_scratch_bytes());
  }
  ~PxScratchLease() {
    if (!buf) return;
    if (hipStreamSynchronize(s) != hipSuccess) return;
    std::lock_guard<std::mutex> g(px_pool().mu);
    px_pool().idle[dev].push_back(buf);
  }
};

}  // namespace

extern "C" {

hrf_status hrf_label_boxes(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, int32_t *box,
                           hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && box, "label_boxes: bad arguments");
  box_init_kernel<<<(unsigned)hrf::cdiv((int64_t)maxlab + 1, 256), 256, 0, s>>>(box, maxlab);
  if (H * W > 0) box_kernel<<<hrf::stream_grid(H * W), 256, 0, s>>>(labels, H, W, maxlab, box);
  HRF_LAUNCHED();
  return HRF_OK;
}

// labels: 8-connected components 1..ncomp of the starting mask (hrf_label output);
// box: hrf_label_boxes output.  Synchronises once to read the boxes, and once per iteration
// of the whole-image loop when oversized components exist.
hrf_status hrf_erosion_seeds(const int32_t *labels, int64_t H, int64_t W, int32_t ncomp, const int32_t *box,
                             int32_t area_max, int32_t min_obj, uint8_t *be_out, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(ncomp >= 0 && be_out && (ncomp == 0 || (labels && box)), "erosion_seeds: bad arguments");
  if (ncomp == 0) {
    HRF_HIP(hipMemsetAsync(be_out, 0, (size_t)(H * W), s));
    return HRF_OK;
  }
  std::vector<int32_t> hb((size_t)(ncomp + 1) * 4);
  HRF_HIP(hipMemcpyAsync(hb.data(), box, hb.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HRF_HIP(hipStreamSynchronize(s));
  // the pixel kernel's scratch: checked out of a per-device pool for this call and returned
  // by the guard on every return path, after the stream has drained -- so no later call, from
  // any thread or stream, can receive a buffer a kernel of this call may still touch
  int dev = 0;
  HRF_HIP(hipGetDevice(&dev));
  PxScratchLease pxl(dev, s);
  HRF_HIP(pxl.acquire());
  char *pxs = pxl.buf;
  int32_t *ovf = nullptr;
  HRF_HIP(hipMallocAsync((void **)&ovf, sizeof(int32_t), s));
  hrf_status st =
      ::hrf::erosion_seeds_hostbox(labels, H, W, ncomp, box, hb.data(), area_max, min_obj, be_out, s, ovf, pxs);
  int32_t novf = 0;
  if (st == HRF_OK) {
    HRF_HIP(hipMemcpyAsync(&novf, ovf, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HRF_HIP(hipStreamSynchronize(s));
  }
  HRF_HIP(hipFreeAsync(ovf, s));
  // a large-box component overflowed the run kernel: redo the classic way
  if (st == HRF_OK && novf > 0) {
    st = ::hrf::erosion_seeds_hostbox(labels, H, W, ncomp, box, hb.data(), area_max, min_obj, be_out, s, nullptr,
                                      pxs);
  }
  if (st == HRF_OK) HRF_HIP(hipStreamSynchronize(s));  // (the lease synchronises on error paths)
  return st;
}

}  // extern "C"

int64_t hrf::seed_px_scratch_bytes() { return (int64_t)SEED_PX_WG * (int64_t)SEED_SLICE; }

// The same with the boxes already on the host (hb: (ncomp + 1) x 4, as hrf_label_boxes
// writes them): the native E. coli driver reads them back at its component-count
// synchronisation instead of a second one here.
hrf_status hrf::erosion_seeds_hostbox(const int32_t *labels, int64_t H, int64_t W, int32_t ncomp, const int32_t *box,
                                      const int32_t *hb, int32_t area_max, int32_t min_obj, uint8_t *be_out,
                                      hipStream_t s, int32_t *ovf_dev, char *px_scratch) {
  if (ncomp == 0) {
    HRF_HIP(hipMemsetAsync(be_out, 0, (size_t)(H * W), s));
    if (ovf_dev) HRF_HIP(hipMemsetAsync(ovf_dev, 0, sizeof(int32_t), s));
    return HRF_OK;
  }
  // 0: run-length kernel (32 KB LDS), 1: pixel kernel (160 KB LDS), 2: whole-image loop.
  // Components the run kernel cannot hold (run arrays over capacity) are listed with the
  // class-1 ones and redone by the pixel kernel, so every box it receives fits SEED_LDS_PX_MAX.
  // ovf_dev given: large boxes may go to the run kernel; ovf_dev receives the number of those
  // that overflowed it (then the caller redoes the stage with ovf_dev == nullptr)
  const int mode = 1 | (ovf_dev ? SEED_BIG_RUNS : 0);
  int64_t br0 = H, bc0 = W, br1 = -1, bc1 = -1;
  for (int c = 1; c <= ncomp; ++c) {
    if (seed_class(hb, c, mode) != 2) continue;
    br0 = std::min<int64_t>(br0, hb[c * 4 + 0]);
    bc0 = std::min<int64_t>(bc0, hb[c * 4 + 1]);
    br1 = std::max<int64_t>(br1, hb[c * 4 + 2]);
    bc1 = std::max<int64_t>(bc1, hb[c * 4 + 3]);
  }
  // the run kernel lists, on the device, the components it hands to the pixel kernel (nothing
  // is copied from host memory, whose lifetime an asynchronous copy would outlive)
  int32_t *dlist = nullptr;
  const size_t nl = (size_t)ncomp + 3;
  const int npx_wg = std::min(ncomp, SEED_PX_WG);
  const size_t list_bytes = (sizeof(int32_t) * nl + 255) & ~(size_t)255;
  // the pixel kernel's scratch: the caller's (the native driver's context holds one), else
  // allocated with the list
  HRF_HIP(hipMallocAsync((void **)&dlist, list_bytes + (px_scratch ? 0 : (size_t)npx_wg * SEED_SLICE), s));
  if (!px_scratch) px_scratch = reinterpret_cast<char *>(dlist) + list_bytes;
  int32_t *dcount = dlist + ncomp + 1;  // [0] pixel-kernel list length, [1] large-box overflows
  // the seed image, the counters and the caller's overflow slot cleared by one launch
  ZeroPub zp;
  HRF_REQUIRE(zp.zero(dcount, 2 * sizeof(int32_t)) && zp.zero(ovf_dev, sizeof(int32_t)),
              "erosion_seeds: clear list");
  if ((H * W) % 4 == 0) {
    HRF_REQUIRE(zp.zero(be_out, H * W), "erosion_seeds: clear seeds");
  } else {
    HRF_HIP(hipMemsetAsync(be_out, 0, (size_t)(H * W), s));
  }
  if (hrf_status r_ = zero_publish(zp, s)) return r_;
  erosion_seed_runs_kernel<<<(unsigned)ncomp, RS_T, RS_LDS, s>>>(labels, H, W, box, mode, area_max, min_obj, dlist,
                                                                 dcount, be_out, ovf_dev);
  erosion_seed_kernel<<<(unsigned)npx_wg, 256, 0, s>>>(labels, H, W, box, dlist, dcount, area_max, min_obj,
                                                        px_scratch, be_out);
  HRF_LAUNCHED();
  hrf_status st = HRF_OK;
  if (br1 >= 0) {
    // pad by one background pixel where the crop edge is interior to the image
    const int64_t r0 = br0 > 0 ? br0 - 1 : 0, c0 = bc0 > 0 ? bc0 - 1 : 0;
    const int64_t r1 = br1 < H - 1 ? br1 + 1 : H - 1, c1 = bc1 < W - 1 ? bc1 + 1 : W - 1;
    const int64_t h = r1 - r0 + 1, w = c1 - c0 + 1, n = h * w;
    char *ws = nullptr;
    HRF_HIP(hipMallocAsync((void **)&ws, (size_t)(3 * n + 8 * n + 64), s));
    uint8_t *m = (uint8_t *)ws, *m2 = m + n, *bec = m2 + n;
    int32_t *par = (int32_t *)(ws + ((3 * n + 15) & ~(int64_t)15)), *sz = par + n;
    int64_t *cnt_dev = nullptr;
    HRF_HIP(hipMallocAsync((void **)&cnt_dev, sizeof(int64_t), s));
    HRF_HIP(hipMemsetAsync(bec, 0, (size_t)n, s));
    big_crop_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(labels, H, W, box, ncomp, mode, r0, c0, h, w, m);
    HRF_LAUNCHED();
    for (int64_t it = 0; it < 4 * (h + w) + 8; ++it) {
      int64_t cnt = 0;
      if ((st = hrf_count_nonzero_u8(m, n, cnt_dev, s))) break;
      HRF_HIP(hipMemcpyAsync(&cnt, cnt_dev, sizeof(int64_t), hipMemcpyDeviceToHost, s));
      HRF_HIP(hipStreamSynchronize(s));
      if (cnt == 0) break;
      if ((st = hrf_split_by_size(m, h, w, 2, area_max, bec, m2, par, sz, s))) break;
      if ((st = hrf_binary_erosion(m2, h, w, 1, m, s))) break;
      if ((st = hrf_remove_small_objects_mask(m, h, w, min_obj, 1, m2, par, sz, s))) break;
      std::swap(m, m2);
    }
    if (st == HRF_OK) {
      big_paste_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(bec, H, W, r0, c0, h, w, be_out);
      HRF_LAUNCHED();
    }
    HRF_HIP(hipFreeAsync(cnt_dev, s));
    HRF_HIP(hipFreeAsync(ws, s));
  }
  HRF_HIP(hipFreeAsync(dlist, s));
  return st;
}
