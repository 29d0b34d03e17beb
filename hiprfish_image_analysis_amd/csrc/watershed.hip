// watershed.hip -- marker-controlled watershed (a12), tie-exact, as a parallel relaxation
// plus an exact resolution of the (rare) pixels whose label depends on the heap's order.
//
// Reference: skimage.morphology.watershed(image, markers, mask) (ecoli measurement.py:113,
// multispecies :154): a sequential binary-heap flood ordered by (value, age), a pixel
// labelled when it is PUSHED, with the label of the pixel being popped.
//
// Order theorem used here (derivation in DESIGN.md "Watershed"; CPU model oracle/ws_order.c,
// checked against the restated heap on plateau-heavy integer images):
//  * the heap pops in non-decreasing flood level lambda(q) = min over marker paths of the
//    path maximum, and within one level in FIFO layers: key(q) = (lambda, h) with h = 0 at
//    a level's entries and markers, h + 1 across a pixel whose value equals the level, h + 0
//    across a "basin" pixel whose value is below it (the heap fills a basin inside the slot
//    of the plateau pixel that reached it);
//  * C(q) = the in-mask labelled neighbours with the least key are the pixels that can push
//    q; q takes the label of the first of them popped.  Their pop order is the lexicographic
//    order of str(x) = key(x) . min_{c in C(x)} str(c) (a basin pixel: min_{c in C(x)} str(c);
//    a marker: key . BOTTOM . raster index).  Candidates of different labels never share an
//    ancestor, so the age a push receives inside one slot never decides a label.
// Execution:
//  1. relaxation of (lambda, h, label) -- ties to the smaller label -- in 32x32 LDS tiles,
//     ping-pong global passes until no tile changes (ws_pass_kernel);
//  2. ws_contest_kernel lists the pixels whose candidates carry different labels.  None (every
//     input without competing equal values, and the quantised E. coli tiles measured) -> done;
//  3. otherwise ws_resolve_wave_kernel decides each listed pixel by walking the candidates'
//     strings (one 64-lane workgroup per walker, sets of tied ancestors, hash-deduplicated, a
//     basin component at once), fixes its parent, labels are re-propagated from the markers (ws_pass_kernel in
//     relabel mode: resolved pixels copy their parent, others the least candidate label) and
//     step 2 repeats until no undecided contest is left.
//  4. when two competing strings are equal down to markers of the same value (counted in
//     ties_host[2]), skimage's choice depends on where its binary heap happens to hold the two
//     age-0 items; the resolver then takes the smaller raster index and the tile is flooded
//     once more by ws_heap_flood_kernel, one workgroup running skimage's heap itself, whose
//     labels replace the relaxation's.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "ws_core.hpp"
#ifdef HRF_WSW_DEBUG
__device__ int g_wsw_dbg = 0;
#define WSW_DBG(...) do { if (g_wsw_dbg && threadIdx.x == 0 && blockIdx.x == 0) printf(__VA_ARGS__); } while (0)
#endif
#include "ws_wave.hpp"

namespace {

using namespace hrf_ws;
constexpr int WT = 32, WL = WT + 2;

struct WsState {
  double *lam;
  int32_t *hop;
  int32_t *lab;
  int32_t *dst;  // basin distance (relaxation tie-break only, see ws_pass_kernel)
};

// One workgroup per 32x32 tile: both ping-pong buffers get the initial state (so a tile that
// never runs keeps a valid copy in each), and tile_work[t] = 1 iff the tile holds a pixel the
// relaxation can change (in the mask and not a marker).  Tiles without one -- the background
// beyond the rough mask, about a quarter of an E. coli tile -- are skipped by every pass.
// tile_marker[t] = 1 iff the tile holds a marker: the first pass of a relaxation (labels only
// flow out of markers then) takes these flags as "changed in the previous pass", so tiles with
// no marker in their 3x3 tile neighbourhood skip it.
__global__ __launch_bounds__(256) void ws_init_kernel(const double *__restrict__ f, int negate,
                                                      const int32_t *__restrict__ markers,
                                                      const uint8_t *__restrict__ mask, int64_t H, int64_t W,
                                                      WsState a, WsState b, int32_t *__restrict__ ptr,
                                                      int32_t *__restrict__ tile_work,
                                                      int32_t *__restrict__ tile_marker,
                                                      int32_t *__restrict__ tile_flags, int32_t *__restrict__ flags) {
  // the first pass batch's zeroed state, instead of fills: this tile's change flags of
  // generations 0 and 1, and (block 0) the 8 host-read flags
  const int tid = threadIdx.x;
  const int64_t ntl = (int64_t)gridDim.x * gridDim.y, tl = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  if (tid < 2) tile_flags[tid * ntl + tl] = 0;
  if (tl == 0 && tid < 8) flags[tid] = 0;
  int work = 0, mark = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t gr = (int64_t)blockIdx.y * WT + (tid >> 5) + 8 * k, gc = (int64_t)blockIdx.x * WT + (tid & 31);
    if (gr >= H || gc >= W) continue;
    const int64_t i = gr * W + gc;
    const bool in = !mask || mask[i];
    const int32_t m = in ? markers[i] : 0;
    const double l = m ? (negate ? -f[i] : f[i]) : __builtin_inf();
    const int32_t h = m ? 0 : HOP_INF;
    a.lam[i] = l;
    b.lam[i] = l;
    a.hop[i] = h;
    b.hop[i] = h;
    a.dst[i] = h;
    b.dst[i] = h;
    a.lab[i] = m;
    b.lab[i] = m;
    ptr[i] = -1;
    work |= in && !m;
    mark |= m != 0;
  }
  work = __syncthreads_or(work);
  mark = __syncthreads_or(mark);
  if (tid == 0) {
    tile_work[blockIdx.y * gridDim.x + blockIdx.x] = work;
    tile_marker[blockIdx.y * gridDim.x + blockIdx.x] = mark;
  }
}

__device__ __forceinline__ bool better(double l1, int32_t h1, int32_t d1, int32_t b1, double l2, int32_t h2,
                                       int32_t d2, int32_t b2) {
  if (l1 != l2) return l1 < l2;
  if (h1 != h2) return h1 < h2;
  if (d1 != d2) return d1 < d2;
  return b1 < b2;
}

// One global pass.  RELABEL = false: relax (lambda, h, d, label) from the least labelled
// neighbour (ties -> smaller label).  d, the distance into a basin from its slot, is not part
// of the order the heap uses; it only makes the pointer relation strictly increasing inside a
// basin (equal (lambda, h) there), without which simultaneous (Jacobi) updates of two basin
// neighbours can swap stale labels forever.  RELABEL = true: keys are final; a pixel with a resolved
// parent copies its label, any other takes the least non-zero label of its candidates (0 =
// not yet reached, so labels flow out of the markers again after a reset).
// The pass walks the tiles persistently: a resident grid of workgroups takes tiles t = blockIdx.x,
// + gridDim.x, ... (ntx x nty tiles), so a pass costs a resident grid's dispatches instead of one
// per tile -- most tiles are skipped after the first passes, and under the concurrent classifier
// every dispatch waits for a CU's LDS.
template <bool RELABEL>
__global__ __launch_bounds__(256) void ws_pass_kernel(const double *__restrict__ f, int negate,
                                                      const int32_t *__restrict__ markers,
                                                      const uint8_t *__restrict__ mask, int64_t H, int64_t W,
                                                      WsState in, WsState out, const int32_t *__restrict__ ptr,
                                                      int32_t *__restrict__ changed,
                                                      const int32_t *__restrict__ prev_tile,
                                                      int32_t *__restrict__ cur_tile,
                                                      int32_t *__restrict__ next_tile,
                                                      const int32_t *__restrict__ tile_work, int ntx, int nty) {
  __shared__ double sl[WL * WL];
  __shared__ int32_t sh[WL * WL];
  __shared__ int32_t sd[WL * WL];
  __shared__ int32_t sb[WL * WL];
  __shared__ uint8_t sm[WL * WL];
  const int tid = threadIdx.x;
  for (int tile = blockIdx.x; tile < ntx * nty; tile += gridDim.x) {
  const int bx = tile % ntx, by = tile / ntx;
  const int64_t r0 = (int64_t)by * WT - 1, c0 = (int64_t)bx * WT - 1;
  // Tile flags rotate through three generations: this pass reads prev, sets cur, and clears
  // next for the following pass (last read as prev by the pass before this one, which has
  // finished), so no memset is needed between passes.
  if (tid == 0) next_tile[tile] = 0;
  if (!tile_work[tile]) continue;  // nothing relaxable: state fixed
  // A tile whose 3x3 tile neighbourhood did not change in the previous pass is skipped: its
  // own state did not change either, so both ping-pong buffers already hold it.
  if (prev_tile) {
    int act = 0;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int ty = by + dy, tx = bx + dx;
        if (ty >= 0 && ty < nty && tx >= 0 && tx < ntx) act |= prev_tile[ty * ntx + tx];
      }
    if (!act) continue;
  }
  for (int idx = tid; idx < WL * WL; idx += 256) {
    const int lr = idx / WL, lc = idx - lr * WL;
    const int64_t gr = r0 + lr, gc = c0 + lc;
    if (gr >= 0 && gr < H && gc >= 0 && gc < W) {
      const int64_t g = gr * W + gc;
      const bool inm = !mask || mask[g];
      sl[idx] = in.lam[g];
      sh[idx] = in.hop[g];
      sd[idx] = RELABEL ? 0 : in.dst[g];
      sb[idx] = in.lab[g];
      sm[idx] = (uint8_t)((inm ? 1 : 0) | ((inm && markers[g]) ? 2 : 0));
    } else {
      sl[idx] = __builtin_inf();
      sh[idx] = HOP_INF;
      sd[idx] = HOP_INF;
      sb[idx] = 0;
      sm[idx] = 0;
    }
  }
  __syncthreads();
  // each thread owns 4 interior pixels, row = 4 (tid/32) + k, col = tid%32, so a thread's pixels
  // alternate in colour with k (red-black order below).
  // The owned pixels' own values stay in registers (only a pixel's own value is ever read:
  // 9 KB less LDS per workgroup, room beside the classifier's workgroups on a CU).
  int own[4];
  int32_t par[4];
  double fvk[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    own[k] = (4 * (tid >> 5) + k + 1) * WL + (tid & 31) + 1;
    par[k] = -1;
    {
      const int64_t gr = r0 + (own[k] / WL), gc = c0 + (own[k] % WL);
      fvk[k] = (gr < H && gc < W) ? (negate ? -f[gr * W + gc] : f[gr * W + gc]) : 0.0;
    }
    if (RELABEL) {
      const int64_t gr = r0 + (own[k] / WL), gc = c0 + (own[k] % WL);
      if (gr < H && gc < W) par[k] = ptr[gr * W + gc];
    }
  }
  // the new state of pixel i from its neighbours' current state; true if it changes
  auto relax = [&](int i, double fv, int32_t parent, double &nl, int32_t &nh, int32_t &nd, int32_t &nb) -> bool {
    nl = sl[i];
    nh = sh[i];
    nd = sd[i];
    nb = sb[i];
    if ((sm[i] & 3) != 1) return false;  // outside mask or a marker
    const int nbr[4] = {i - WL, i - 1, i + 1, i + WL};
    if (!RELABEL) {
      // first-popped neighbour = least (lambda, h) among labelled in-mask neighbours
      double bl = __builtin_inf();
      int32_t bh = HOP_INF, bd = HOP_INF, bb = 0;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int j = nbr[d];
        const int32_t bj = sb[j];
        if (!bj || !(sm[j] & 1)) continue;
        if (better(sl[j], sh[j], sd[j], bj, bl, bh, bd, bb)) {
          bl = sl[j];
          bh = sh[j];
          bd = sd[j];
          bb = bj;
        }
      }
      if (bb) {
        if (bl < fv) {  // entry of level fv
          nl = fv;
          nh = 0;
          nd = 0;
        } else if (bl == fv) {  // plateau pixel: next FIFO layer
          nl = bl;
          nh = bh + 1;
          nd = 0;
        } else {  // basin pixel: filled in the slot that reached it
          nl = bl;
          nh = bh;
          nd = bd + 1;
        }
        nb = bb;
      }
      return (nb != sb[i]) || (nl != sl[i]) || (nh != sh[i]) || (nd != sd[i]);
    }
    int32_t lb = 0;
    if (parent >= 0) {
      const int64_t pr = parent / W - r0, pc = parent % W - c0;
      lb = (pr >= 0 && pr < WL && pc >= 0 && pc < WL) ? sb[pr * WL + pc] : in.lab[parent];
    } else {
      double bl = __builtin_inf();
      int32_t bh = HOP_INF;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int j = nbr[d];
        if (!(sm[j] & 1) || sl[j] == __builtin_inf()) continue;
        const int32_t bj = sb[j];
        if (sl[j] < bl || (sl[j] == bl && sh[j] < bh)) {
          bl = sl[j];
          bh = sh[j];
          lb = bj;
        } else if (sl[j] == bl && sh[j] == bh && bj && (!lb || bj < lb)) {
          lb = bj;
        }
      }
    }
    nb = lb;
    return nb != sb[i];
  };
  auto store = [&](int i, double nl, int32_t nh, int32_t nd, int32_t nb) {
    if (!RELABEL) {
      sl[i] = nl;
      sh[i] = nh;
      sd[i] = nd;
    }
    sb[i] = nb;
  };
  bool any_change = false;
  for (int it = 0; it < 4 * WT * WT; ++it) {
    bool ch = false;
    // Red-black (checkerboard) relaxation: a pixel's four neighbours have the other colour, so
    // one colour's pixels update in place from the other's current state (no two neighbours
    // ever update together, nothing is staged) and a label travels two pixels per iteration.
    // The update is monotone, so it reaches the Jacobi form's least fixpoint (the Jacobi form
    // was 3.03 vs 2.16 ms per tile in the bench; removed in round 5).  Colour of pixel k:
    // (k + tid) & 1; every lane updates two pixels per colour.
#pragma unroll
    for (int colour = 0; colour < 2; ++colour) {
      const bool odd = (colour ^ (tid & 1)) != 0;  // this lane's pixels of the colour: k = odd, odd + 2
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int i = odd ? own[2 * j + 1] : own[2 * j];
        const double fv = odd ? fvk[2 * j + 1] : fvk[2 * j];
        const int32_t pa = odd ? par[2 * j + 1] : par[2 * j];
        double nl;
        int32_t nh, nd, nb;
        if (relax(i, fv, pa, nl, nh, nd, nb)) {
          store(i, nl, nh, nd, nb);
          ch = true;
        }
      }
      if (colour == 0) __syncthreads();  // red written before black reads it
    }
    any_change |= ch;
    if (!__syncthreads_or(ch)) break;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = own[k];
    const int lr = i / WL, lc = i - lr * WL;
    const int64_t gr = r0 + lr, gc = c0 + lc;
    if (gr < H && gc < W) {
      const int64_t g = gr * W + gc;
      if (!RELABEL) {
        out.lam[g] = sl[i];
        out.hop[g] = sh[i];
        out.dst[g] = sd[i];
      }
      out.lab[g] = sb[i];
    }
  }
  if (__syncthreads_or(any_change) && tid == 0) {
    *changed = 1;
    cur_tile[tile] = 1;
  }
  }
}

__global__ void ws_contest_kernel(WsGeom g, const int32_t *__restrict__ lab, const int32_t *__restrict__ ptr,
                                  int32_t *__restrict__ list, int32_t *__restrict__ count) {
  const int64_t n = g.H * g.W;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
    if (!g_in(g, x) || g.mk[x] || g.lam[x] == __builtin_inf() || ptr[x] >= 0) continue;
    int32_t cc[4];
    const int m = g_cands(g, x, cc);
    bool diff = false;
    for (int j = 1; j < m; ++j) diff |= lab[cc[j]] != lab[cc[0]];
    if (diff) list[atomicAdd(count, 1)] = (int32_t)x;
  }
}

// One thread per listed pixel (grid-strided).  A plateau/entry pixel gets the winning
// candidate as parent; a basin pixel decides its whole basin component (every pixel of the
// component points at the winning slot, so the component stays one label, no cycles).
__global__ void ws_resolve_kernel(WsGeom g, const int32_t *__restrict__ list, int32_t count, int32_t *__restrict__ ptr,
                                  char *__restrict__ scratch, int64_t stride, int64_t nt, int32_t cap, int32_t hcap,
                                  int32_t gcap, int32_t *__restrict__ retry, int32_t *__restrict__ nretry,
                                  int32_t *__restrict__ layout) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt) return;  // scratch exists for nt threads only
  char *base = scratch + t * stride;
  Walker w;
  w.pa = (int32_t *)base;
  w.ga = w.pa + cap;
  w.pb = w.ga + cap;
  w.gb = w.pb + cap;
  w.slots = w.gb + cap;
  w.hkey = (uint64_t *)(w.slots + cap);
  w.hgen = (uint32_t *)(w.hkey + hcap);
  w.ml = (double *)(w.hgen + hcap);
  w.mh = (int32_t *)(w.ml + gcap);
  w.mr = w.mh + gcap;
  w.alive = (uint8_t *)(w.mr + gcap);
  w.cap = cap;
  w.hcap = hcap;
  w.gcap = gcap;
  w.gen = 0;
  w.hcount = 0;
  for (int32_t i = 0; i < hcap; ++i) w.hgen[i] = 0;
  int32_t lay = 0;
  for (int64_t li = t; li < count; li += nt) {
    const int32_t x = list[li];
    if (ptr[x] >= 0) continue;  // decided with its basin component by another thread
    const bool fail = !ws_resolve_one(g, x, ptr, w, &lay);
    if (fail) retry[atomicAdd(nretry, 1)] = x;
  }
  if (lay) atomicAdd(layout, lay);
}

// ws_resolve_kernel with one 64-lane workgroup per walker (ws_wave.hpp): the same decisions, each
// walk's frontier processed 64 members at a time.  Scratch layout as ws_resolve_kernel's (the
// hash is the hkey array; hgen and ml are unused).
__global__ __launch_bounds__(64) void ws_resolve_wave_kernel(WsGeom g, const int32_t *__restrict__ list,
                                                             int32_t count, int32_t *__restrict__ ptr,
                                                             char *__restrict__ scratch, int64_t stride, int64_t nw,
                                                             int32_t cap, int32_t hcap, int32_t gcap, int pbits,
                                                             int gbits, int32_t *__restrict__ retry,
                                                             int32_t *__restrict__ nretry, int32_t *__restrict__ layout) {
  const int64_t t = blockIdx.x;
  if (t >= nw) return;  // scratch exists for nw walkers only
  char *base = scratch + t * stride;
  WalkerW w;
  w.pa = (int32_t *)base;
  w.ga = w.pa + cap;
  w.pb = w.ga + cap;
  w.gb = w.pb + cap;
  w.slots = w.gb + cap;
  w.hs = (unsigned long long *)(w.slots + cap);
  uint32_t *hgen = (uint32_t *)(w.hs + hcap);
  double *ml = (double *)(hgen + hcap);
  w.hit = (int32_t *)(ml + gcap);
  w.mr = w.hit + gcap;
  w.alive = (uint8_t *)(w.mr + gcap);
  w.cap = cap;
  w.hcap = hcap;
  w.gcap = gcap;
  w.pbits = pbits;
  w.gbits = gbits;
  w.genb = 64 - pbits - gbits;
  w.gen = 1;
  for (int32_t i = threadIdx.x; i < hcap; i += 64) w.hs[i] = 0ull;
  __syncthreads();
  int32_t lay = 0;
  for (int64_t li = t; li < count; li += nw) {
    const int32_t x = list[li];
    if (ptr[x] >= 0) continue;  // decided with its basin component by another walker (uniform read)
    const bool ok = ws_resolve_one_wave(g, x, ptr, w, &lay);
    if (!ok && threadIdx.x == 0) retry[atomicAdd(nretry, 1)] = x;
    __syncthreads();
  }
  if (threadIdx.x == 0 && lay) atomicAdd(layout, lay);
}

// labels of every non-marker pixel back to 0 (both ping-pong buffers): relabel from markers
__global__ void ws_reset_labels_kernel(const int32_t *__restrict__ markers, const uint8_t *__restrict__ mask, int64_t n,
                                       int32_t *__restrict__ la, int32_t *__restrict__ lb) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t m = (!mask || mask[i]) ? markers[i] : 0;
    la[i] = m;
    lb[i] = m;
  }
}

// ---- exact replay of skimage's binary heap (equal-valued markers) ------------------------
// When a decision comes down to equal-valued markers of different labels (all age 0), skimage
// pops them in whatever order its binary heap holds them -- a function of every push and pop
// before.  No parallel formulation reproduces that, so such a tile is flooded once more by one
// workgroup that runs skimage's algorithm itself (_watershed.pyx / heap_general.pxi of the
// reference era, restated in oracle_watershed): markers pushed in raster order with age 0,
// (value, age) binary heap with strict-less sift up and down, the four neighbours visited up,
// left, right, down, a pixel labelled when pushed.  The top 13 levels of the heap (8191 items)
// live in LDS, deeper items in global memory (16 B each).
// The flood is serial; one wave runs it, its lanes spreading each heap operation's loads and
// compares (below).  Rare: no bench tile needs it.
struct alignas(16) HeapItem {
  double v;
  uint32_t age;
  int32_t idx;
};
constexpr int32_t HEAP_LDS = 8191;
constexpr size_t HEAP_LDS_BYTES = (size_t)HEAP_LDS * 16;

// LDS-qualified pointer: through a plain pointer the compiler emits FLAT instructions for the
// heap's LDS levels (the generic address path, with global-memory latency).  An item is one
// 16-byte read or write on either side (ds_read_b128 / global_load_dwordx4).
#define HRF_LDS __attribute__((address_space(3)))
typedef uint32_t heap_u4 __attribute__((ext_vector_type(4)));
struct HeapView {
  HRF_LDS heap_u4 *l;  // positions < HEAP_LDS
  HeapItem *g;         // indexed by heap position (positions < HEAP_LDS unused)
  __device__ __forceinline__ HeapItem get(int32_t p) const {
    return p < HEAP_LDS ? __builtin_bit_cast(HeapItem, l[p]) : g[p];
  }
  __device__ __forceinline__ void put(int32_t p, const HeapItem &x) const {
    if (p < HEAP_LDS)
      l[p] = __builtin_bit_cast(heap_u4, x);
    else
      g[p] = x;
  }
  // per lane, position p where valid: the LDS read is issued by every lane (its index clamped
  // into the LDS levels), the global read only by the lanes whose item lies deeper, each into
  // its own registers -- with one destination for both the compiler waits on the global reads
  // in flight before issuing the LDS one
  __device__ __forceinline__ HeapItem load(int32_t p, bool valid) const {
    const HeapItem a = __builtin_bit_cast(HeapItem, l[p < HEAP_LDS ? p : 0]);
    HeapItem b{0.0, 0u, 0};
    if (valid && p >= HEAP_LDS) b = g[p];
    return p < HEAP_LDS ? a : b;
  }
};

// heap_general.pxi smaller(): value first (IEEE compare, NaN never smaller), then age
__device__ __forceinline__ bool heap_smaller(const HeapItem &a, const HeapItem &b) {
  if (a.v != b.v) return a.v < b.v;
  return a.age < b.age;
}

__device__ __forceinline__ int32_t heap_uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double heap_uni(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                                        (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b));
}
__device__ __forceinline__ double heap_lane(double v, int src) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  return __builtin_bit_cast(double,
                            ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(b >> 32), src) << 32) |
                                (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src));
}

// heap_smaller for every lane as a lane mask: the three primitive compares are the compare
// instructions' own masks (no per-lane booleans to materialise), combined by scalar operations
__device__ __forceinline__ unsigned long long heap_smaller_mask(const HeapItem &a, const HeapItem &b) {
  const unsigned long long ne = __ballot(a.v != b.v), lt = __ballot(a.v < b.v), al = __ballot(a.age < b.age);
  return (ne & lt) | (~ne & al);
}

// heappush, one wave: the new item x sifts up while strictly smaller than its parent.  The
// ancestors do not change while it climbs (each only moves down one level), so every "x smaller
// than ancestor j" is decided at once: lane j loads ancestor j of the new slot c, one ballot
// gives the climb height t (the run of ones from bit 1), lanes 1..t move their ancestors down
// one level in one store, lane 0 stores x.  One round trip per push instead of one per level.
// LDS_ONLY (the new slot lies in LDS, so do all its ancestors): no global access, hence no wait
// on the label store just issued.
template <bool LDS_ONLY>
__device__ __forceinline__ void heap_push_w(const HeapView &h, int32_t c, const HeapItem &x, int lane) {
  const int32_t pj = lane < 32 ? ((c + 1) >> lane) - 1 : -1;  // ancestor lane of c (lane 0: c)
  const bool va = lane >= 1 && pj >= 0;
  const HeapItem A = LDS_ONLY ? __builtin_bit_cast(HeapItem, h.l[pj < 0 ? 0 : pj]) : h.load(pj < 0 ? 0 : pj, va);
  const unsigned long long m = __ballot(va) & heap_smaller_mask(x, A);
  const int t = __builtin_ctzll(~(m >> 1));  // bits 1..t set: x climbs t levels
  if (LDS_ONLY) {
    if (lane >= 1 && lane <= t) h.l[((c + 1) >> (lane - 1)) - 1] = __builtin_bit_cast(heap_u4, A);
    if (lane == 0) h.l[((c + 1) >> t) - 1] = __builtin_bit_cast(heap_u4, x);
  } else {
    if (lane >= 1 && lane <= t) h.put(((c + 1) >> (lane - 1)) - 1, A);
    if (lane == 0) h.put(((c + 1) >> t) - 1, x);
  }
}
__device__ __forceinline__ void heap_push_w(const HeapView &h, int32_t &n, const HeapItem &x, int lane) {
  const int32_t c = n++;
  if (c < HEAP_LDS)
    heap_push_w<true>(h, c, x, lane);
  else
    heap_push_w<false>(h, c, x, lane);
}

// heappop's sift-down of x (the heap's former last item) from the hole at the root, n items
// left, one wave: SD_LEV levels per round trip.  Lane k < 2^SD_LEV - 1 takes the node k places
// below the hole in breadth-first order (depth d = log2(k + 1), position hole * 2^d + k), loads
// its two children and decides the three compares the sift can ask there -- left child smaller
// than x, right child smaller than x, right smaller than left -- into three ballots.  The path
// is then walked on those bits alone (the rule of heap_general.pxi: the hole moves to the left
// child if it is smaller than x, unless the right one is smaller still; to the right child if
// only it is smaller than x; else x stays), and every moved child is written into its parent by
// the lane that holds it: one store per side.  A child at or past n is never smaller.
// LDS_ONLY: the whole heap lies in LDS (n <= HEAP_LDS), so the step holds no global load -- a
// global load anywhere in the loop makes the compiler wait for every load in flight (the popped
// pixel's neighbours included) before the first compare.
constexpr int SD_LEV = 6;
// the steps whose nodes all lie on the LDS levels 0..12: a step from a hole on depth
// s * SD_LEV reaches depth (s + 1) * SD_LEV
constexpr int SD_LDS_STEPS = 12 / SD_LEV;

// one step from `hole`; false once x has found its place (hole then holds its position)
template <bool LDS_STEP>
__device__ __forceinline__ bool heap_sift_step(const HeapView &h, int32_t n, const HeapItem &x, int lane,
                                               int64_t &hole) {
  const int k = lane;
  const bool kl = k < (1 << SD_LEV) - 1;
  const int d = 31 - __builtin_clz((unsigned)k + 1u);
  const int64_t a = (hole << d) + k, l = 2 * a + 1, r = l + 1;
  const bool vl = kl && l < n, vr = kl && r < n;
  HeapItem L, R;
  if (LDS_STEP) {
    L = __builtin_bit_cast(HeapItem, h.l[vl ? (int32_t)l : 0]);
    R = __builtin_bit_cast(HeapItem, h.l[vr ? (int32_t)r : 0]);
  } else {
    L = h.load(vl ? (int32_t)l : 0, vl);
    R = h.load(vr ? (int32_t)r : 0, vr);
  }
  const unsigned long long bl = __ballot(vl), br = __ballot(vr);
  const unsigned long long mlx = bl & heap_smaller_mask(L, x);
  const unsigned long long mrx = br & heap_smaller_mask(R, x);
  const unsigned long long mrl = br & heap_smaller_mask(R, L);
  // per node, where the hole would go from there: left if the left child is smaller than x and
  // the right one not smaller than it; right if the right one is smaller than the better of the two
  const unsigned long long gol = mlx & ~mrl, gor = (mlx & mrl) | (~mlx & mrx);
  // the walk, branch-free (scalar selects): `act` stays 1 while the hole keeps moving
  unsigned long long mvl = 0, mvr = 0;
  int kk = 0, dep = 0;
  unsigned act = 1u;
#pragma unroll
  for (int lev = 0; lev < SD_LEV; ++lev) {
    const unsigned ml = act & (unsigned)(gol >> kk) & 1u, mr = act & (unsigned)(gor >> kk) & 1u;
    mvl |= (unsigned long long)ml << kk;
    mvr |= (unsigned long long)mr << kk;
    act = ml | mr;
    kk = act ? 2 * kk + 1 + (int)mr : kk;
    dep += (int)act;
  }
  if (LDS_STEP) {
    if ((mvl >> lane) & 1ull) h.l[(int32_t)a] = __builtin_bit_cast(heap_u4, L);
    if ((mvr >> lane) & 1ull) h.l[(int32_t)a] = __builtin_bit_cast(heap_u4, R);
  } else {
    if ((mvl >> lane) & 1ull) h.put((int32_t)a, L);
    if ((mvr >> lane) & 1ull) h.put((int32_t)a, R);
  }
  // relative node kk at depth dep: position hole * 2^dep + kk
  hole = (hole << dep) + kk;
  return dep == SD_LEV;
}

// LDS_ONLY: the whole heap lies in LDS.  Otherwise the first SD_LDS_STEPS steps still read LDS
// only, in code of their own: the global reads of the later steps are waited for in order, and
// in shared code that wait would take in the popped pixel's neighbour loads before the first
// compare.
template <bool LDS_ONLY>
__device__ __forceinline__ void heap_sift_down_w(const HeapView &h, int32_t n, const HeapItem &x, int lane) {
  int64_t hole = 0;  // wave-uniform
  if (LDS_ONLY) {
    while (heap_sift_step<true>(h, n, x, lane, hole)) {
    }
  } else {
    bool more = true;
#pragma unroll
    for (int s = 0; s < SD_LDS_STEPS && more; ++s) more = heap_sift_step<true>(h, n, x, lane, hole);
    while (more) more = heap_sift_step<false>(h, n, x, lane, hole);
  }
  if (lane == 0) h.put((int32_t)hole, x);
}

// One 1024-thread workgroup.  Phase 1 (all threads): out = markers where in the mask, and the
// list of marker pixels in raster order (order-preserving compaction by ballots + a 16-wave
// scan).  Phase 2 (wave 0): the flood.  heap: (n + 2) items; list: n int32.
template <bool HASMASK>
__global__ __launch_bounds__(1024) void ws_heap_flood_kernel(const double *__restrict__ f, int negate,
                                                             const int32_t *__restrict__ markers,
                                                             const uint8_t *__restrict__ mask, int32_t H, int32_t W,
                                                             int32_t *__restrict__ out, HeapItem *__restrict__ heap,
                                                             int32_t *__restrict__ list) {
  extern __shared__ HeapItem heap_smem[];
  __shared__ int32_t wsum[16];
  __shared__ int32_t base_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int32_t n = H * W;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int32_t c0 = 0; c0 < n; c0 += 1024) {
    const int32_t i = c0 + tid;
    int32_t m = 0;
    if (i < n) {
      m = (!mask || mask[i]) ? markers[i] : 0;
      out[i] = m;
    }
    const uint64_t bal = __ballot(m != 0);
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int32_t off = base_s;
    for (int k = 0; k < wv; ++k) off += wsum[k];
    if (m) list[off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    __syncthreads();
    if (tid == 0) {
      int32_t t = base_s;
      for (int k = 0; k < 16; ++k) t += wsum[k];
      base_s = t;
    }
    __syncthreads();
  }
  if (wv != 0) return;
  __threadfence_block();  // the other waves' list and label stores, seen by wave 0's loads
  HeapView h{(HRF_LDS heap_u4 *)heap_smem, heap};
  const int32_t nm = heap_uni(base_s);
  int32_t hn = 0;
  for (int32_t k = 0; k < nm; ++k) {
    const int32_t i = heap_uni(list[k]);
    const double fv = heap_uni(f[i]);
    heap_push_w(h, hn, HeapItem{negate ? -fv : fv, 0u, i}, lane);
  }
  uint32_t age = 1;
  const double invW = 1.0 / (double)W;
#ifdef HRF_HEAP_PROF
  unsigned long long tp_top = 0, tp_sift = 0, tp_push = 0, npop = 0;
#define HP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define HP_T(v)
#endif
  while (hn > 0) {
    HP_T(t0);
    // the popped pixel x (the root) and its four neighbours, up, left, right, down: lane d & 3
    // loads neighbour d's state, read before any of them is written (distinct pixels); a
    // neighbour off the image reads the pixel itself and is never free
    const int32_t x = heap_uni(h.get(0).idx);
    // a last item in global memory is loaded before the neighbours: its wait then takes only it
    // (loads complete in order)
    HeapItem lastg{0.0, 0u, 0};
    if (hn - 1 >= HEAP_LDS) lastg = h.g[hn - 1];
    int32_t r = (int32_t)((double)x * invW);  // within one of x / W; corrected exactly
    r -= (int64_t)r * W > x;
    r += (int64_t)(r + 1) * W <= x;
    const int32_t c = x - r * W;
    const int dn = lane & 3;
    const bool okd = dn == 0 ? r > 0 : dn == 1 ? c > 0 : dn == 2 ? c + 1 < W : r + 1 < H;
    const int32_t nbd = dn == 0 ? x - W : dn == 1 ? x - 1 : dn == 2 ? x + 1 : x + W;
    const int32_t q = okd ? nbd : x;
    const uint32_t mq = HASMASK ? mask[q] : 1u;
    const int32_t oq = out[q];
    const double vq = f[q];
    const int32_t labv = out[x];  // read back after the sift-down: the load's wait would hold it up
    HP_T(t1);
    hn -= 1;
    if (hn > 0 && hn < HEAP_LDS) {  // the heap (positions < hn) and its last item (position hn) in LDS
      const HeapItem last = __builtin_bit_cast(HeapItem, h.l[hn]);
      heap_sift_down_w<true>(h, hn, HeapItem{heap_uni(last.v), (uint32_t)heap_uni((int32_t)last.age), heap_uni(last.idx)},
                             lane);
    } else if (hn > 0) {
      heap_sift_down_w<false>(
          h, hn, HeapItem{heap_uni(lastg.v), (uint32_t)heap_uni((int32_t)lastg.age), heap_uni(lastg.idx)}, lane);
    }
    HP_T(t2);
    const unsigned long long fm = __ballot(lane < 4 && okd && mq != 0u && oq == 0);
    const int32_t lab = heap_uni(labv);
    const double vn = negate ? -vq : vq;
#pragma unroll
    for (int dd = 0; dd < 4; ++dd) {
      if (!((fm >> dd) & 1ull)) continue;
      const int32_t nb = dd == 0 ? x - W : dd == 1 ? x - 1 : dd == 2 ? x + 1 : x + W;
      age += 1;
      heap_push_w(h, hn, HeapItem{heap_lane(vn, dd), age, nb}, lane);
    }
    // the pushed neighbours' labels, one store by their lanes after the pushes (a store before a
    // push's global loads would be waited for with them)
    if ((fm >> lane) & 1ull) out[nbd] = lab;
#ifdef HRF_HEAP_PROF
    HP_T(t3);
    tp_top += t1 - t0;
    tp_sift += t2 - t1;
    tp_push += t3 - t2;
    ++npop;
#endif
  }
#ifdef HRF_HEAP_PROF
  if (lane == 0)
    printf("heap prof: pops %llu cycles/pop: top+loads %.0f sift %.0f wait+push %.0f\n", npop, (double)tp_top / npop,
           (double)tp_sift / npop, (double)tp_push / npop);
#endif
}

int64_t heap_flood_scratch_bytes(int64_t n) { return ((n + 2) * 16 + n * 4 + 255) & ~(int64_t)255; }

hrf_status heap_flood(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask, int64_t H,
                      int64_t W, int32_t *out, hipStream_t s) {
  const int64_t n = H * W;
  HRF_REQUIRE(n < ((int64_t)1 << 31) - 2, "watershed heap replay: image too large");
  if (n == 0) return HRF_OK;
  char *scratch = nullptr;
  HRF_HIP(hipMallocAsync((void **)&scratch, (size_t)heap_flood_scratch_bytes(n), s));
  static const bool attr = [] {
    return hipFuncSetAttribute((const void *)ws_heap_flood_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)HEAP_LDS_BYTES) == hipSuccess &&
           hipFuncSetAttribute((const void *)ws_heap_flood_kernel<false>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)HEAP_LDS_BYTES) == hipSuccess;
  }();
  hrf_status st = HRF_OK;
  if (!attr) {
    ::hrf::set_error("watershed heap replay: cannot reserve %d bytes of LDS", (int)HEAP_LDS_BYTES);
    st = HRF_EHIP;
  } else {
    HeapItem *hp = (HeapItem *)scratch;
    int32_t *lp = (int32_t *)(scratch + (n + 2) * 16);
    if (mask)
      ws_heap_flood_kernel<true><<<1, 1024, HEAP_LDS_BYTES, s>>>(image, negate, markers, mask, (int32_t)H, (int32_t)W,
                                                                 out, hp, lp);
    else
      ws_heap_flood_kernel<false><<<1, 1024, HEAP_LDS_BYTES, s>>>(image, negate, markers, mask, (int32_t)H,
                                                                  (int32_t)W, out, hp, lp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      ::hrf::set_error("watershed heap replay: launch failed: %s", hipGetErrorString(e));
      st = HRF_EHIP;
    }
  }
  HRF_HIP(hipFreeAsync(scratch, s));
  return st;
}

int64_t walker_bytes(int32_t cap, int32_t hcap, int32_t gcap) {
  int64_t b = 5 * (int64_t)cap * 4 + (int64_t)hcap * 12 + (int64_t)gcap * (8 + 4 + 4 + 1);
  return (b + 255) & ~(int64_t)255;
}

struct WsBuffers {
  WsState a, b;
  int32_t *ptr, *list, *retry, *tf, *tw, *tm;
};

WsBuffers carve(void *state_ws, int64_t n, int64_t ntiles) {
  char *ws = (char *)state_ws;
  WsBuffers B;
  B.a = WsState{(double *)ws, (int32_t *)(ws + 8 * n), (int32_t *)(ws + 12 * n), (int32_t *)(ws + 16 * n)};
  B.b = WsState{(double *)(ws + 24 * n), (int32_t *)(ws + 32 * n), (int32_t *)(ws + 36 * n), (int32_t *)(ws + 40 * n)};
  B.ptr = (int32_t *)(ws + 44 * n);
  B.list = (int32_t *)(ws + 48 * n);
  B.retry = (int32_t *)(ws + 52 * n);
  B.tf = (int32_t *)(ws + 56 * n);
  B.tw = B.tf + 3 * ntiles;
  B.tm = B.tw + ntiles;
  return B;
}

}  // namespace

extern "C" {

int64_t hrf_watershed_workspace_bytes(int64_t H, int64_t W) {
  if (H < 0 || W < 0) return -1;
  const int64_t ntiles = hrf::cdiv(W, WT) * hrf::cdiv(H, WT);
  return 56 * H * W + 20 * ntiles + 256;
}

// flag_ws (>= 8 int32): [0] change flag of a batch's last pass, [1] the other passes',
// [2] contest count, [3] retry count, [4] heap-layout decisions
hrf_status hrf_watershed_ex(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask, int64_t H,
                            int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws, int32_t max_passes,
                            int32_t *passes_host, int32_t *ties_host, hrf_stream_t stream) {
  return hrf::watershed_ex_extra(image, negate, markers, mask, H, W, out_labels, state_ws, flag_ws, max_passes,
                                 passes_host, ties_host, (hipStream_t)stream, nullptr);
}

}  // extern "C"

// hrf_watershed_ex whose batch read-backs also run the caller's clears and read-backs (extra:
// the native chains fold theirs into the watershed's synchronisation, common.hpp ZeroPub)
hrf_status hrf::watershed_ex_extra(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask,
                                   int64_t H, int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws,
                                   int32_t max_passes, int32_t *passes_host, int32_t *ties_host, hipStream_t s,
                                   const ZeroPub *extra) {
  const int64_t n = H * W;
  HRF_REQUIRE(H >= 0 && W >= 0 && H <= 65535 * (int64_t)WT && W <= 65535 * (int64_t)WT && n < ((int64_t)1 << 31),
              "watershed: bad shape");
  if (ties_host) ties_host[0] = ties_host[1] = ties_host[2] = 0;
  if (passes_host) *passes_host = 0;
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(image && markers && out_labels && state_ws && flag_ws, "watershed: null buffer");
  // the batch flags' pinned host slots (one set per host thread, kept for the process)
  static thread_local int32_t *pin = nullptr;
  if (!pin) HRF_HIP(host_alloc_mapped((void **)&pin, 64));
  int32_t *pin_dev = mapped(pin);
  HRF_REQUIRE(pin_dev, "watershed: pinned flags have no device address");
  dim3 grid((unsigned)hrf::cdiv(W, WT), (unsigned)hrf::cdiv(H, WT));
  const int64_t ntiles = (int64_t)grid.x * grid.y;
  WsBuffers B = carve(state_ws, n, ntiles);
  // Buffer a's labels live in out_labels: every batch runs an even number of passes, so the
  // converged labels end in a, and no final copy is needed (kept as a fallback below).
  HRF_REQUIRE(out_labels != markers, "watershed: out_labels must not alias markers");
  B.a.lab = out_labels;
  WsState a = B.a, b = B.b;
  int32_t *tf = B.tf;  // per-tile change flags, three rotating generations
  ws_init_kernel<<<grid, 256, 0, s>>>(image, negate, markers, mask, H, W, a, b, B.ptr, B.tw, B.tm, tf, flag_ws);
  HRF_LAUNCHED();
  int32_t hflag[4] = {0, 0, 0, 0};  // host copies of flag_ws[0..3]
  bool zeroed = true;  // ws_init_kernel zeroed tf's generations 0/1 and flag_ws[0..7]
  int passes = 0;
  // persistent pass grids (one workgroup per tile lost in round 3)
  const unsigned pgrid_t = hrf::resident_grid(ws_pass_kernel<true>, 256, 0, ntiles);
  const unsigned pgrid_f = hrf::resident_grid(ws_pass_kernel<false>, 256, 0, ntiles);

  // Passes run in batches with one host read per batch (change flag + contest count): the
  // first batch of 8 covers the typical tile (~7 passes) with a single synchronisation, later
  // batches 4.  Passes after convergence skip every tile (no tile changed).
  auto run = [&](bool relabel, int32_t *count_out) -> hrf_status {
    if (!zeroed) HRF_HIP(hipMemsetAsync(tf, 0, sizeof(int32_t) * 2 * ntiles, s));  // generations 0 and 1
    int local = 0;
    for (int batch = 8;; batch = 4) {
      if (!zeroed) HRF_HIP(hipMemsetAsync(flag_ws, 0, sizeof(int32_t) * 3, s));
      zeroed = false;
      for (int k = 0; k < batch; ++k) {
        int32_t *cur = tf + (local % 3) * ntiles;
        const int32_t *prev = local == 0 ? B.tm : tf + ((local + 2) % 3) * ntiles;
        int32_t *next = tf + ((local + 1) % 3) * ntiles;
        int32_t *chg = flag_ws + (k == batch - 1 ? 0 : 1);
        if (relabel)
          ws_pass_kernel<true><<<pgrid_t, 256, 0, s>>>(image, negate, markers, mask, H, W, a, b, B.ptr, chg, prev,
                                                       cur, next, B.tw, (int)grid.x, (int)grid.y);
        else
          ws_pass_kernel<false><<<pgrid_f, 256, 0, s>>>(image, negate, markers, mask, H, W, a, b, B.ptr, chg, prev,
                                                        cur, next, B.tw, (int)grid.x, (int)grid.y);
        WsState t = a;
        a = b;
        b = t;
        ++local;
        ++passes;
      }
      HRF_LAUNCHED();
      WsGeom g{image, negate, markers, mask, H, W, a.lam, a.hop};
      ws_contest_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(g, a.lab, B.ptr, B.list, flag_ws + 2);
      HRF_LAUNCHED();
      {  // the batch's flags (and the caller's extras) in one launch, read after the synchronisation
        ZeroPub zp = extra ? *extra : ZeroPub();
        HRF_REQUIRE(zp.pub(flag_ws, pin_dev, 3), "watershed: too many read-backs");
        if (hrf_status r = zero_publish(zp, s)) return r;
        HRF_HIP(hipStreamSynchronize(s));
        for (int k = 0; k < 3; ++k) hflag[k] = pin[k];
      }
      if (!hflag[0]) {
        *count_out = hflag[2];
        return HRF_OK;
      }
      if (passes >= max_passes) {
        ::hrf::set_error("watershed: not converged after %d passes (max_passes)", passes);
        return HRF_EINVAL;
      }
    }
  };

  int32_t ncontest = 0;
  if (hrf_status r = run(false, &ncontest)) return r;
  int32_t total = 0, rounds = 0;
  char *scratch = nullptr;
  int64_t scratch_bytes = 0;
  // stream-ordered: a tile with contests must not stall the other tiles' streams (hipFree
  // would synchronise the whole device)
  struct Scratch {
    char **p;
    hipStream_t s;
    ~Scratch() {
      if (*p) (void)hipFreeAsync(*p, s);
    }
  } sguard{&scratch, s};
  while (ncontest > 0) {
    total += ncontest;
    ++rounds;
    WsGeom g{image, negate, markers, mask, H, W, a.lam, a.hop};
    const int32_t *todo = B.list;
    int32_t ntodo = ncontest;
    // as many walkers as a 1 GB scratch budget holds (~4 k walkers of 244 KB at the first
    // capacity; round 3 ran 256), each deciding its share of the list
    constexpr int64_t budget = (int64_t)1024 << 20;
    for (int32_t cap = 4096;; cap *= 16) {
      const int32_t hcap = 2 * cap, gcap = cap;
      const int64_t stride = walker_bytes(cap, hcap, gcap);
      const int64_t threads = budget / stride > 0 ? budget / stride : 1;
      const int64_t nth = ntodo < threads ? ntodo : threads;
      if (nth * stride > scratch_bytes) {
        const hipError_t fe = scratch ? hipFreeAsync(scratch, s) : hipSuccess;
        scratch = nullptr;  // before the status check: the guard must not free it again
        scratch_bytes = 0;
        HRF_HIP(fe);
        HRF_HIP(hipMallocAsync((void **)&scratch, (size_t)(nth * stride), s));
        scratch_bytes = nth * stride;
      }
      HRF_HIP(hipMemsetAsync(flag_ws + 3, 0, sizeof(int32_t), s));
      // one 64-lane workgroup per walker; one thread per walker (the serial walk of ws_core.hpp,
      // 28x slower on the adversarial image) only when the hash slots' [generation | group |
      // pixel] words cannot hold 8 generation bits
      int pbits = 1, gbits = 1;
      while (pbits < 31 && ((int64_t)1 << pbits) < n) ++pbits;
      while (gbits < 31 && ((int64_t)1 << gbits) <= gcap) ++gbits;
      if (64 - pbits - gbits >= 8)
        ws_resolve_wave_kernel<<<(unsigned)nth, 64, 0, s>>>(g, todo, ntodo, B.ptr, scratch, stride, nth, cap, hcap,
                                                            gcap, pbits, gbits, B.retry, flag_ws + 3, flag_ws + 4);
      else
        ws_resolve_kernel<<<(unsigned)hrf::cdiv(nth, 64), 64, 0, s>>>(g, todo, ntodo, B.ptr, scratch, stride, nth,
                                                                       cap, hcap, gcap, B.retry, flag_ws + 3,
                                                                       flag_ws + 4);
      HRF_LAUNCHED();
      HRF_HIP(hipMemcpyAsync(hflag + 3, flag_ws + 3, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      HRF_HIP(hipStreamSynchronize(s));
      if (!hflag[3]) break;
      // a group holds at most n pixels, and the queue each at most 4 times: beyond that an
      // overflow means a corrupted state, not a large plateau
      HRF_REQUIRE((int64_t)cap <= 16 * n + 65536, "watershed: tie resolution exceeded its scratch (%d entries)", cap);
      // retry list -> list (the retry buffer is rewritten by the next launch)
      HRF_HIP(hipMemcpyAsync(B.list, B.retry, sizeof(int32_t) * hflag[3], hipMemcpyDeviceToDevice, s));
      todo = B.list;
      ntodo = hflag[3];
    }
    ws_reset_labels_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(markers, mask, n, a.lab, b.lab);
    HRF_LAUNCHED();
    if (hrf_status r = run(true, &ncontest)) return r;
    HRF_REQUIRE(rounds < 4096, "watershed: tie resolution does not terminate");
  }
  int32_t layout = 0;  // decisions between equal-valued markers of different labels
  if (rounds) {
    HRF_HIP(hipMemcpyAsync(hflag + 3, flag_ws + 4, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HRF_HIP(hipStreamSynchronize(s));
    layout = hflag[3];
  }
  if (ties_host) {
    ties_host[0] = total;
    ties_host[1] = rounds;
    ties_host[2] = layout;
  }
  if (a.lab != out_labels) HRF_HIP(hipMemcpyAsync(out_labels, a.lab, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
  // skimage decides those by its heap's layout: flood the tile again with the heap itself
  if (layout > 0)
    if (hrf_status r = heap_flood(image, negate, markers, mask, H, W, out_labels, s)) return r;
  if (passes_host) *passes_host = passes;
  return HRF_OK;
}

extern "C" {

hrf_status hrf_watershed(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask, int64_t H,
                         int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws, int32_t max_passes,
                         int32_t *passes_host, hrf_stream_t stream) {
  return hrf_watershed_ex(image, negate, markers, mask, H, W, out_labels, state_ws, flag_ws, max_passes, passes_host,
                          nullptr, stream);
}

hrf_status hrf_watershed_heap(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask,
                              int64_t H, int64_t W, int32_t *out_labels, hrf_stream_t stream) {
  HRF_REQUIRE(H >= 0 && W >= 0, "watershed_heap: bad shape");
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(image && markers && out_labels, "watershed_heap: null buffer");
  HRF_REQUIRE(out_labels != markers, "watershed_heap: out_labels must not alias markers");
  return heap_flood(image, negate, markers, mask, H, W, out_labels, (hipStream_t)stream);
}

}  // extern "C"
