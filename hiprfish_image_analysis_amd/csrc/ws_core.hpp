// ws_core.hpp -- the exact tie resolution of the watershed (watershed.hip), written once for
// the device and for the host (tools/ws_emul.cpp replays the whole flow on the CPU to test it).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#define HRF_HD __host__ __device__

namespace hrf_ws {

constexpr int32_t HOP_INF = 0x7fffffff;

struct WsGeom {
  const double *f;
  int negate;
  const int32_t *mk;
  const uint8_t *mask;
  int64_t H, W;
  const double *lam;
  const int32_t *hop;
};

HRF_HD inline bool g_in(const WsGeom &g, int64_t i) { return !g.mask || g.mask[i]; }
HRF_HD inline bool g_marker(const WsGeom &g, int64_t i) { return g_in(g, i) && g.mk[i] != 0; }
HRF_HD inline double g_f(const WsGeom &g, int64_t i) { return g.negate ? -g.f[i] : g.f[i]; }
HRF_HD inline bool g_basin(const WsGeom &g, int64_t i) { return !g_marker(g, i) && g_f(g, i) < g.lam[i]; }
HRF_HD inline bool kless(double l1, int32_t h1, double l2, int32_t h2) {
  return l1 < l2 || (l1 == l2 && h1 < h2);
}

// candidates of x: in-mask reached neighbours with the least key
HRF_HD inline int g_cands(const WsGeom &g, int64_t x, int32_t *out) {
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

  HRF_HD void new_gen() {
    ++gen;
    hcount = 0;
  }
  HRF_HD bool contains(int32_t p, int32_t grp) const {
    const uint64_t key = ((uint64_t)(uint32_t)p << 32) | (uint32_t)grp;
    uint64_t h = key * 0x9E3779B97F4A7C15ull;
    uint32_t s = (uint32_t)(h >> 33) & (uint32_t)(hcap - 1);
    for (;;) {
      if (hgen[s] != gen) return false;
      if (hkey[s] == key) return true;
      s = (s + 1) & (uint32_t)(hcap - 1);
    }
  }
  // true if (p, grp) was not yet in this generation's set (then inserted); false if present
  // or the table is full (*ovf set)
  HRF_HD bool insert(int32_t p, int32_t grp, bool *ovf) {
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
HRF_HD inline int ws_walk(const WsGeom &g, const int32_t *cand, int k, Walker &w, int32_t *layout) {
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
  // every step consumes one key of a finite string; the bound only guards against a
  // corrupted state (then the pixel is retried and the call fails loudly)
  for (int64_t step = 0;; ++step) {
    if (step > 4 * g.H * g.W + 16) return -1;
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
      int32_t l0 = 0, bmr = 0, bc = 0;
      bool multi = false;
      for (int j = 0; j < k; ++j) {
        const int32_t mrj = w.mr[j];
        if (!w.alive[j] || mrj < 0) continue;
        ++nm;
        if (nm == 1) l0 = g.mk[mrj];
        else if (g.mk[mrj] != l0) multi = true;
        // equal strings end at the same marker: the smaller candidate pixel wins, so the
        // decision does not depend on the order the candidates were listed in (threads that
        // resolve one basin component from different pixels must agree on its root).  Kept
        // as a running best in registers: the indexed form (mr[j] == mr[win] && cand[j] <
        // cand[win]) was compiled to a wrong choice for gfx950 (ROCm 7.2), see DESIGN.md.
        const int32_t cj = cand[j];
        if (win < 0 || mrj < bmr || (mrj == bmr && cj < bc)) {
          win = j;
          bmr = mrj;
          bc = cj;
        }
      }
      if (nm > 1 && multi) *layout += 1;  // per-thread count, summed by the caller
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


// Decide listed pixel x: a plateau/entry pixel gets the winning candidate as parent; a basin
// pixel decides its whole basin component (a BFS tree over the component rooted at the
// winning slot: every pixel points at a NEIGHBOUR, no cycles).  false on scratch overflow.
HRF_HD inline bool ws_resolve_one(const WsGeom &g, int32_t x, int32_t *ptr, Walker &w, int32_t *layout,
                                   int32_t *root = nullptr) {
  const int32_t cap = w.cap;
  bool fail = false;
  if (!g_basin(g, x)) {
    int32_t cc[4];
    const int m = g_cands(g, x, cc);
    const int win = ws_walk(g, cc, m, w, layout);
    if (win < 0) fail = true;
    else ptr[x] = cc[win];
    if (root && win >= 0) *root = cc[win];
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
      // the component again as the set (p, 0), then a BFS tree over it rooted at the
      // winning slot, visited as (p, 1): every pixel points at a NEIGHBOUR, so the relabel
      // passes' tile activity (a tile reruns when a neighbouring tile changed) stays valid
      const int32_t wp = w.slots[win];
      if (root) *root = wp;
      w.new_gen();
      nq = 0;
      w.insert(x, 0, &ovf);
      w.pa[nq++] = x;
      for (int32_t qi = 0; qi < nq; ++qi) {
        int32_t cc[4];
        const int m = g_cands(g, w.pa[qi], cc);
        for (int j = 0; j < m; ++j)
          if (g_basin(g, cc[j]) && w.insert(cc[j], 0, &ovf)) w.pa[nq++] = cc[j];
      }
      int32_t nt2 = 0;
      w.pb[nt2++] = wp;
      for (int32_t qi = 0; qi < nt2 && !fail; ++qi) {
        const int32_t q = w.pb[qi];
        const int64_t r = q / g.W, c = q - r * g.W;
        const int32_t nb[4] = {r > 0 ? q - (int32_t)g.W : -1, c > 0 ? q - 1 : -1, c + 1 < g.W ? q + 1 : -1,
                               r + 1 < g.H ? q + (int32_t)g.W : -1};
        for (int j = 0; j < 4; ++j) {
          const int32_t y = nb[j];
          if (y < 0 || !w.contains(y, 0) || !w.insert(y, 1, &ovf)) continue;
          if (nt2 >= cap) {  // the slot plus the whole component: cap + 1 entries at most
            fail = true;
            break;
          }
          ptr[y] = q;
          w.pb[nt2++] = y;
        }
      }
      if (ovf) fail = true;  // retried with more scratch: the same BFS order, so the same tree
    }
  }
  return !fail;
}

}  // namespace hrf_ws
