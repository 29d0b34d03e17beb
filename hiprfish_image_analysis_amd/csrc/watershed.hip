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
//  3. otherwise ws_resolve_kernel decides each listed pixel by walking the candidates' strings
//     (one thread per pixel, sets of tied ancestors, hash-deduplicated, a basin component at
//     once), fixes its parent, labels are re-propagated from the markers (ws_pass_kernel in
//     relabel mode: resolved pixels copy their parent, others the least candidate label) and
//     step 2 repeats until no undecided contest is left.
// One departure from skimage remains, reported in ties_host[2]: when two competing strings
// are equal down to markers of the same value, skimage's choice depends on where its binary
// heap happens to hold the two age-0 items; here the marker with the smaller raster index wins.
#include "common.hpp"

namespace {

constexpr int WT = 32, WL = WT + 2;
constexpr int32_t HOP_INF = 0x7fffffff;

struct WsState {
  double *lam;
  int32_t *hop;
  int32_t *lab;
};

__global__ void ws_init_kernel(const double *__restrict__ f, int negate, const int32_t *__restrict__ markers,
                               const uint8_t *__restrict__ mask, int64_t n, double *__restrict__ lam,
                               int32_t *__restrict__ hop, int32_t *__restrict__ lab, int32_t *__restrict__ ptr) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool in = !mask || mask[i];
    const int32_t m = in ? markers[i] : 0;
    lam[i] = m ? (negate ? -f[i] : f[i]) : __builtin_inf();
    hop[i] = m ? 0 : HOP_INF;
    lab[i] = m;
    ptr[i] = -1;
  }
}

__device__ __forceinline__ bool better(double l1, int32_t h1, int32_t b1, double l2, int32_t h2, int32_t b2) {
  if (l1 != l2) return l1 < l2;
  if (h1 != h2) return h1 < h2;
  return b1 < b2;
}

// One global pass.  RELABEL = false: relax (lambda, h, label) from the least-key labelled
// neighbour (ties -> smaller label).  RELABEL = true: keys are final; a pixel with a resolved
// parent copies its label, any other takes the least non-zero label of its candidates (0 =
// not yet reached, so labels flow out of the markers again after a reset).
template <bool RELABEL>
__global__ __launch_bounds__(256) void ws_pass_kernel(const double *__restrict__ f, int negate,
                                                      const int32_t *__restrict__ markers,
                                                      const uint8_t *__restrict__ mask, int64_t H, int64_t W,
                                                      WsState in, WsState out, const int32_t *__restrict__ ptr,
                                                      int32_t *__restrict__ changed,
                                                      const int32_t *__restrict__ prev_tile,
                                                      int32_t *__restrict__ cur_tile,
                                                      int32_t *__restrict__ next_tile) {
  __shared__ double sl[WL * WL];
  __shared__ double sf[WL * WL];
  __shared__ int32_t sh[WL * WL];
  __shared__ int32_t sb[WL * WL];
  __shared__ uint8_t sm[WL * WL];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * WT - 1, c0 = (int64_t)blockIdx.x * WT - 1;
  // Tile flags rotate through three generations: this pass reads prev, sets cur, and clears
  // next for the following pass (last read as prev by the pass before this one, which has
  // finished), so no memset is needed between passes.
  if (tid == 0) next_tile[blockIdx.y * gridDim.x + blockIdx.x] = 0;
  // A tile whose 3x3 tile neighbourhood did not change in the previous pass is skipped: its
  // own state did not change either, so both ping-pong buffers already hold it.
  if (prev_tile) {
    int act = 0;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int ty = (int)blockIdx.y + dy, tx = (int)blockIdx.x + dx;
        if (ty >= 0 && ty < (int)gridDim.y && tx >= 0 && tx < (int)gridDim.x) act |= prev_tile[ty * gridDim.x + tx];
      }
    if (!act) return;
  }
  for (int idx = tid; idx < WL * WL; idx += 256) {
    const int lr = idx / WL, lc = idx - lr * WL;
    const int64_t gr = r0 + lr, gc = c0 + lc;
    if (gr >= 0 && gr < H && gc >= 0 && gc < W) {
      const int64_t g = gr * W + gc;
      const bool inm = !mask || mask[g];
      sl[idx] = in.lam[g];
      sh[idx] = in.hop[g];
      sb[idx] = in.lab[g];
      sf[idx] = negate ? -f[g] : f[g];
      sm[idx] = (uint8_t)((inm ? 1 : 0) | ((inm && markers[g]) ? 2 : 0));
    } else {
      sl[idx] = __builtin_inf();
      sh[idx] = HOP_INF;
      sb[idx] = 0;
      sf[idx] = 0.0;
      sm[idx] = 0;
    }
  }
  __syncthreads();
  // each thread owns 4 interior pixels: (row = tid/32 + 8k, col = tid%32)
  int own[4];
  int32_t par[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    own[k] = ((tid >> 5) + 8 * k + 1) * WL + (tid & 31) + 1;
    par[k] = -1;
    if (RELABEL) {
      const int64_t gr = r0 + (own[k] / WL), gc = c0 + (own[k] % WL);
      if (gr < H && gc < W) par[k] = ptr[gr * W + gc];
    }
  }
  bool any_change = false;
  for (int it = 0; it < 4 * WT * WT; ++it) {
    double nl[4];
    int32_t nh[4], nb[4];
    bool ch = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = own[k];
      nl[k] = sl[i];
      nh[k] = sh[i];
      nb[k] = sb[i];
      if ((sm[i] & 3) != 1) continue;  // outside mask or a marker
      const int nbr[4] = {i - WL, i - 1, i + 1, i + WL};
      if (!RELABEL) {
        // first-popped neighbour = least (lambda, h) among labelled in-mask neighbours
        double bl = __builtin_inf();
        int32_t bh = HOP_INF, bb = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int j = nbr[d];
          const int32_t bj = sb[j];
          if (!bj || !(sm[j] & 1)) continue;
          if (better(sl[j], sh[j], bj, bl, bh, bb)) {
            bl = sl[j];
            bh = sh[j];
            bb = bj;
          }
        }
        if (bb) {
          const double fv = sf[i];
          if (bl < fv) {  // entry of level fv
            nl[k] = fv;
            nh[k] = 0;
          } else if (bl == fv) {  // plateau pixel: next FIFO layer
            nl[k] = bl;
            nh[k] = bh + 1;
          } else {  // basin pixel: filled in the slot that reached it
            nl[k] = bl;
            nh[k] = bh;
          }
          nb[k] = bb;
        }
        ch |= (nb[k] != sb[i]) || (nl[k] != sl[i]) || (nh[k] != sh[i]);
      } else {
        int32_t lb = 0;
        if (par[k] >= 0) {
          const int64_t pr = par[k] / W - r0, pc = par[k] % W - c0;
          lb = (pr >= 0 && pr < WL && pc >= 0 && pc < WL) ? sb[pr * WL + pc] : in.lab[par[k]];
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
        nb[k] = lb;
        ch |= nb[k] != sb[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!RELABEL) {
        sl[own[k]] = nl[k];
        sh[own[k]] = nh[k];
      }
      sb[own[k]] = nb[k];
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
      }
      out.lab[g] = sb[i];
    }
  }
  if (__syncthreads_or(any_change) && tid == 0) {
    *changed = 1;
    cur_tile[blockIdx.y * gridDim.x + blockIdx.x] = 1;
  }
}

// ---- exact resolution -----------------------------------------------------------------------
struct WsGeom {
  const double *f;
  int negate;
  const int32_t *mk;
  const uint8_t *mask;
  int64_t H, W;
  const double *lam;
  const int32_t *hop;
};

__device__ __forceinline__ bool g_in(const WsGeom &g, int64_t i) { return !g.mask || g.mask[i]; }
__device__ __forceinline__ bool g_marker(const WsGeom &g, int64_t i) { return g_in(g, i) && g.mk[i] != 0; }
__device__ __forceinline__ double g_f(const WsGeom &g, int64_t i) { return g.negate ? -g.f[i] : g.f[i]; }
__device__ __forceinline__ bool g_basin(const WsGeom &g, int64_t i) { return !g_marker(g, i) && g_f(g, i) < g.lam[i]; }
__device__ __forceinline__ bool kless(double l1, int32_t h1, double l2, int32_t h2) {
  return l1 < l2 || (l1 == l2 && h1 < h2);
}

// candidates of x: in-mask reached neighbours with the least key
__device__ int g_cands(const WsGeom &g, int64_t x, int32_t *out) {
  const int64_t r = x / g.W, c = x - r * g.W;
  int64_t nb[4];
  int k = 0;
  if (r > 0) nb[k++] = x - g.W;
  if (c > 0) nb[k++] = x - 1;
  if (c + 1 < g.W) nb[k++] = x + 1;
  if (r + 1 < g.H) nb[k++] = x + g.W;
  double bl = __builtin_inf();
  int32_t bh = HOP_INF;
  int m = 0;
  for (int j = 0; j < k; ++j) {
    const int64_t y = nb[j];
    if (!g_in(g, y)) continue;
    const double ly = g.lam[y];
    if (ly == __builtin_inf()) continue;
    const int32_t hy = g.hop[y];
    if (kless(ly, hy, bl, bh)) {
      bl = ly;
      bh = hy;
      m = 0;
    }
    if (ly == bl && hy == bh) out[m++] = (int32_t)y;
  }
  return m;
}

// Per-thread scratch: two member buffers (pixel, group), the basin slot list, a generation
// hash set of (pixel, group) and per-group state.  Sized by the host; overflow -> retry larger.
struct Walker {
  int32_t *pa, *ga, *pb, *gb, *slots;
  uint64_t *hkey;
  uint32_t *hgen;
  double *ml;
  int32_t *mh, *mr;
  uint8_t *alive;
  int32_t cap, hcap, gcap;
  uint32_t gen;
  int32_t hcount;

  __device__ void new_gen() {
    ++gen;
    hcount = 0;
  }
  // true if (p, grp) was not yet in this generation's set (then inserted); false if present
  // or the table is full (*ovf set)
  __device__ bool insert(int32_t p, int32_t grp, bool *ovf) {
    const uint64_t key = ((uint64_t)(uint32_t)p << 32) | (uint32_t)grp;
    if (2 * (hcount + 1) > hcap) {
      *ovf = true;
      return false;
    }
    uint64_t h = key * 0x9E3779B97F4A7C15ull;
    uint32_t s = (uint32_t)(h >> 33) & (uint32_t)(hcap - 1);
    for (;;) {
      if (hgen[s] != gen) {
        hgen[s] = gen;
        hkey[s] = key;
        ++hcount;
        return true;
      }
      if (hkey[s] == key) return false;
      s = (s + 1) & (uint32_t)(hcap - 1);
    }
  }
};

// index into cand[] of the candidate whose string is least (the one the heap pops first);
// -1 on scratch overflow.  *layout += 1 when equal strings down to markers of different labels
// are decided by raster index.
__device__ int ws_walk(const WsGeom &g, const int32_t *cand, int k, Walker &w, int32_t *layout) {
  if (k <= 0 || k > w.gcap || k > w.cap) return -1;
  if (k == 1) return 0;
  bool ovf = false;
  int32_t *cp = w.pa, *cg = w.ga, *op = w.pb, *og = w.gb;
  int32_t ncur = 0;
  for (int j = 0; j < k; ++j) {
    cp[ncur] = cand[j];
    cg[ncur] = j;
    ++ncur;
    w.alive[j] = 1;
  }
  for (;;) {
    // 1. basin members -> the non-basin pixels of equal key reachable through the basin
    w.new_gen();
    int32_t nout = 0;
    for (int32_t i = 0; i < ncur; ++i) {
      const int32_t x = cp[i], gr = cg[i];
      if (!w.insert(x, gr, &ovf)) {
        if (ovf) return -1;
        continue;
      }
      if (g_basin(g, x)) {
        int32_t cc[4];
        const int m = g_cands(g, x, cc);
        for (int t = 0; t < m; ++t) {
          if (ncur >= w.cap) return -1;
          cp[ncur] = cc[t];
          cg[ncur] = gr;
          ++ncur;
        }
      } else {
        if (nout >= w.cap) return -1;
        op[nout] = x;
        og[nout] = gr;
        ++nout;
      }
    }
    if (nout == 0) return -1;  // cannot happen (every string ends at a marker)
    // 2. least key per group; groups above the overall least drop out
    for (int j = 0; j < k; ++j) {
      w.ml[j] = __builtin_inf();
      w.mh[j] = HOP_INF;
      w.mr[j] = -1;
    }
    double bl = __builtin_inf();
    int32_t bh = HOP_INF;
    for (int32_t i = 0; i < nout; ++i) {
      const int32_t x = op[i], gr = og[i];
      const double lx = g.lam[x];
      const int32_t hx = g.hop[x];
      if (kless(lx, hx, w.ml[gr], w.mh[gr])) {
        w.ml[gr] = lx;
        w.mh[gr] = hx;
      }
      if (kless(lx, hx, bl, bh)) {
        bl = lx;
        bh = hx;
      }
    }
    int nal = 0, last = -1;
    for (int j = 0; j < k; ++j) {
      if (!w.alive[j]) continue;
      if (w.ml[j] != bl || w.mh[j] != bh) {
        w.alive[j] = 0;
        continue;
      }
      ++nal;
      last = j;
    }
    if (nal == 1) return last;
    // 3. members at the least key; markers among them end their string (BOTTOM . rank)
    int32_t nkeep = 0;
    bool anym = false;
    for (int32_t i = 0; i < nout; ++i) {
      const int32_t x = op[i], gr = og[i];
      if (!w.alive[gr] || g.lam[x] != bl || g.hop[x] != bh) continue;
      cp[nkeep] = x;
      cg[nkeep] = gr;
      ++nkeep;
      if (g_marker(g, x)) {
        anym = true;
        if (w.mr[gr] < 0 || x < w.mr[gr]) w.mr[gr] = x;
      }
    }
    if (anym) {
      int win = -1, nm = 0;
      int32_t l0 = 0;
      bool multi = false;
      for (int j = 0; j < k; ++j) {
        if (!w.alive[j] || w.mr[j] < 0) continue;
        ++nm;
        if (nm == 1) l0 = g.mk[w.mr[j]];
        else if (g.mk[w.mr[j]] != l0) multi = true;
        if (win < 0 || w.mr[j] < w.mr[win]) win = j;
      }
      if (nm > 1 && multi) atomicAdd(layout, 1);
      return win;
    }
    // 4. one symbol further: the union of the kept members' candidates, per group
    w.new_gen();
    int32_t nn = 0;
    for (int32_t i = 0; i < nkeep; ++i) {
      int32_t cc[4];
      const int m = g_cands(g, cp[i], cc);
      for (int t = 0; t < m; ++t) {
        if (!w.insert(cc[t], cg[i], &ovf)) {
          if (ovf) return -1;
          continue;
        }
        if (nn >= w.cap) return -1;
        op[nn] = cc[t];
        og[nn] = cg[i];
        ++nn;
      }
    }
    int32_t *t0 = cp, *t1 = cg;
    cp = op;
    cg = og;
    op = t0;
    og = t1;
    ncur = nn;
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
                                  char *__restrict__ scratch, int64_t stride, int32_t cap, int32_t hcap, int32_t gcap,
                                  int32_t *__restrict__ retry, int32_t *__restrict__ nretry,
                                  int32_t *__restrict__ layout) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nt = (int64_t)gridDim.x * blockDim.x;
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
  for (int64_t li = t; li < count; li += nt) {
    const int32_t x = list[li];
    if (ptr[x] >= 0) continue;  // decided with its basin component by another thread
    bool fail = false;
    if (!g_basin(g, x)) {
      int32_t cc[4];
      const int m = g_cands(g, x, cc);
      const int win = ws_walk(g, cc, m, w, layout);
      if (win < 0) fail = true;
      else ptr[x] = cc[win];
    } else {
      // component of equal-key basin pixels and its slots (equal-key non-basin neighbours)
      bool ovf = false;
      w.new_gen();
      int32_t nq = 0, ns = 0;
      w.insert(x, 0, &ovf);
      w.pa[nq++] = x;
      for (int32_t qi = 0; qi < nq && !fail; ++qi) {
        int32_t cc[4];
        const int m = g_cands(g, w.pa[qi], cc);
        for (int j = 0; j < m; ++j) {
          if (!w.insert(cc[j], 0, &ovf)) {
            if (ovf) fail = true;
            continue;
          }
          if (g_basin(g, cc[j])) {
            if (nq >= cap) fail = true;
            else w.pa[nq++] = cc[j];
          } else {
            if (ns >= cap) fail = true;
            else w.slots[ns++] = cc[j];
          }
        }
      }
      int win = -1;
      if (!fail) {
        // ws_walk reuses pa/ga: move the component out of the way by re-deriving it afterwards
        win = ws_walk(g, w.slots, ns, w, layout);
        if (win < 0) fail = true;
      }
      if (!fail) {
        const int32_t wp = w.slots[win];
        w.new_gen();
        nq = 0;
        w.insert(x, 0, &ovf);
        w.pa[nq++] = x;
        for (int32_t qi = 0; qi < nq; ++qi) {
          const int32_t b = w.pa[qi];
          ptr[b] = wp;
          int32_t cc[4];
          const int m = g_cands(g, b, cc);
          for (int j = 0; j < m; ++j)
            if (g_basin(g, cc[j]) && w.insert(cc[j], 0, &ovf)) w.pa[nq++] = cc[j];
        }
      }
    }
    if (fail) retry[atomicAdd(nretry, 1)] = x;
  }
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

int64_t walker_bytes(int32_t cap, int32_t hcap, int32_t gcap) {
  int64_t b = 5 * (int64_t)cap * 4 + (int64_t)hcap * 12 + (int64_t)gcap * (8 + 4 + 4 + 1);
  return (b + 255) & ~(int64_t)255;
}

struct WsBuffers {
  WsState a, b;
  int32_t *ptr, *list, *retry, *tf;
};

WsBuffers carve(void *state_ws, int64_t n, int64_t ntiles) {
  char *ws = (char *)state_ws;
  WsBuffers B;
  B.a = WsState{(double *)ws, (int32_t *)(ws + 8 * n), (int32_t *)(ws + 12 * n)};
  B.b = WsState{(double *)(ws + 16 * n), (int32_t *)(ws + 24 * n), (int32_t *)(ws + 28 * n)};
  B.ptr = (int32_t *)(ws + 32 * n);
  B.list = (int32_t *)(ws + 36 * n);
  B.retry = (int32_t *)(ws + 40 * n);
  B.tf = (int32_t *)(ws + 44 * n);
  (void)ntiles;
  return B;
}

}  // namespace

extern "C" {

int64_t hrf_watershed_workspace_bytes(int64_t H, int64_t W) {
  if (H < 0 || W < 0) return -1;
  const int64_t ntiles = hrf::cdiv(W, WT) * hrf::cdiv(H, WT);
  return 44 * H * W + 12 * ntiles + 256;
}

// flag_ws (>= 8 int32): [0] change flag of a batch's last pass, [1] the other passes',
// [2] contest count, [3] retry count, [4] heap-layout decisions
hrf_status hrf_watershed_ex(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask, int64_t H,
                            int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws, int32_t max_passes,
                            int32_t *passes_host, int32_t *ties_host, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = H * W;
  HRF_REQUIRE(H >= 0 && W >= 0 && H <= 65535 * (int64_t)WT && W <= 65535 * (int64_t)WT && n < ((int64_t)1 << 31),
              "watershed: bad shape");
  if (ties_host) ties_host[0] = ties_host[1] = ties_host[2] = 0;
  if (passes_host) *passes_host = 0;
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(image && markers && out_labels && state_ws && flag_ws, "watershed: null buffer");
  dim3 grid((unsigned)hrf::cdiv(W, WT), (unsigned)hrf::cdiv(H, WT));
  const int64_t ntiles = (int64_t)grid.x * grid.y;
  WsBuffers B = carve(state_ws, n, ntiles);
  WsState a = B.a, b = B.b;
  ws_init_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(image, negate, markers, mask, n, a.lam, a.hop, a.lab, B.ptr);
  HRF_LAUNCHED();
  int32_t *tf = B.tf;  // per-tile change flags, three rotating generations
  int32_t hflag[4] = {0, 0, 0, 0};  // host copies of flag_ws[0..3]
  HRF_HIP(hipMemsetAsync(flag_ws, 0, sizeof(int32_t) * 8, s));
  int passes = 0;

  // Passes run in batches with one host read per batch (change flag + contest count): the
  // first batch of 8 covers the typical tile (~7 passes) with a single synchronisation, later
  // batches 4.  Passes after convergence skip every tile (no tile changed).
  auto run = [&](bool relabel, int32_t *count_out) -> hrf_status {
    HRF_HIP(hipMemsetAsync(tf, 0, sizeof(int32_t) * 2 * ntiles, s));  // generations of passes 0 and 1
    int local = 0;
    for (int batch = 8;; batch = 4) {
      HRF_HIP(hipMemsetAsync(flag_ws, 0, sizeof(int32_t) * 3, s));
      for (int k = 0; k < batch; ++k) {
        int32_t *cur = tf + (local % 3) * ntiles;
        const int32_t *prev = local == 0 ? nullptr : tf + ((local + 2) % 3) * ntiles;
        int32_t *next = tf + ((local + 1) % 3) * ntiles;
        int32_t *chg = flag_ws + (k == batch - 1 ? 0 : 1);
        if (relabel)
          ws_pass_kernel<true><<<grid, 256, 0, s>>>(image, negate, markers, mask, H, W, a, b, B.ptr, chg, prev, cur,
                                                    next);
        else
          ws_pass_kernel<false><<<grid, 256, 0, s>>>(image, negate, markers, mask, H, W, a, b, B.ptr, chg, prev, cur,
                                                     next);
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
      HRF_HIP(hipMemcpyAsync(hflag, flag_ws, sizeof(int32_t) * 3, hipMemcpyDeviceToHost, s));
      HRF_HIP(hipStreamSynchronize(s));
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
  struct Scratch {
    char **p;
    ~Scratch() {
      if (*p) hipFree(*p);
    }
  } sguard{&scratch};
  while (ncontest > 0) {
    total += ncontest;
    ++rounds;
    WsGeom g{image, negate, markers, mask, H, W, a.lam, a.hop};
    const int32_t *todo = B.list;
    int32_t ntodo = ncontest;
    for (int32_t cap = 4096, threads = 256;; cap *= 16, threads = threads > 16 ? threads / 16 : 1) {
      const int32_t hcap = 2 * cap, gcap = cap;
      const int64_t stride = walker_bytes(cap, hcap, gcap);
      const int64_t nth = ntodo < threads ? ntodo : threads;
      if (nth * stride > scratch_bytes) {
        if (scratch) HRF_HIP(hipFree(scratch));
        scratch = nullptr;
        scratch_bytes = 0;
        HRF_HIP(hipMalloc((void **)&scratch, (size_t)(nth * stride)));
        scratch_bytes = nth * stride;
      }
      HRF_HIP(hipMemsetAsync(flag_ws + 3, 0, sizeof(int32_t), s));
      ws_resolve_kernel<<<(unsigned)hrf::cdiv(nth, 64), 64, 0, s>>>(g, todo, ntodo, B.ptr, scratch, stride, cap,
                                                                     hcap, gcap, B.retry, flag_ws + 3, flag_ws + 4);
      HRF_LAUNCHED();
      HRF_HIP(hipMemcpyAsync(hflag + 3, flag_ws + 3, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      HRF_HIP(hipStreamSynchronize(s));
      if (!hflag[3]) break;
      HRF_REQUIRE((int64_t)cap * 16 <= 4 * n + 64, "watershed: tie resolution exceeded its scratch (%d pixels)", cap);
      // retry list -> list (the retry buffer is rewritten by the next launch)
      HRF_HIP(hipMemcpyAsync(B.list, B.retry, sizeof(int32_t) * hflag[3], hipMemcpyDeviceToDevice, s));
      todo = B.list;
      ntodo = hflag[3];
    }
    ws_reset_labels_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(markers, mask, n, a.lab, b.lab);
    HRF_LAUNCHED();
    if (hrf_status r = run(true, &ncontest)) return r;
    HRF_REQUIRE(rounds < 100000, "watershed: tie resolution does not terminate");
  }
  if (ties_host) {
    ties_host[0] = total;
    ties_host[1] = rounds;
    if (rounds) {
      HRF_HIP(hipMemcpyAsync(hflag + 3, flag_ws + 4, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      HRF_HIP(hipStreamSynchronize(s));
      ties_host[2] = hflag[3];
    }
  }
  HRF_HIP(hipMemcpyAsync(out_labels, a.lab, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
  if (passes_host) *passes_host = passes;
  return HRF_OK;
}

hrf_status hrf_watershed(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask, int64_t H,
                         int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws, int32_t max_passes,
                         int32_t *passes_host, hrf_stream_t stream) {
  return hrf_watershed_ex(image, negate, markers, mask, H, W, out_labels, state_ws, flag_ws, max_passes, passes_host,
                          nullptr, stream);
}

}  // extern "C"
