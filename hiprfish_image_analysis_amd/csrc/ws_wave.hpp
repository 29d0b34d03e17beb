// ws_wave.hpp -- the watershed tie walk (ws_core.hpp ws_walk / ws_resolve_one) with one 64-lane
// workgroup per walker: the frontier sets are processed 64 members at a time, the (pixel, group)
// set is a lock-free hash (compare-and-swap on one 64-bit word holding generation, group and
// pixel), per-group flags and marker minima are plain stores / atomicMin.  The walk is set
// logic -- which members are in a frontier, never the order they were found in -- so every
// decision equals the serial walk's (tests/test_watershed_gpu.py checks the result against the
// restated heap); only the scratch-overflow points differ, and an overflow is retried with more
// scratch as before.  Device only; the serial form stays the host emulator's.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "wave.hpp"
#include "ws_core.hpp"

namespace hrf_ws {

#ifndef WSW_DBG
#define WSW_DBG(...)
#endif

struct WalkerW {
  int32_t *pa, *ga, *pb, *gb, *slots;
  unsigned long long *hs;  // hcap slots: [gen : genb][group : gb][pixel : pbits]
  int32_t *hit, *mr;       // per group
  uint8_t *alive;
  int32_t cap, hcap, gcap;
  int pbits, gbits, genb;
  unsigned long long gen;  // current generation (1 .. 2^genb - 1), uniform
};

__device__ __forceinline__ int wv_excl(int v) { return hrf::wave_inclusive_scan(v) - v; }
__device__ __forceinline__ int wv_sum(int v) { return hrf::wave_sum(v); }

// a new generation: every slot of an older one reads as empty; on wrap the table is cleared
__device__ __forceinline__ void wv_new_gen(WalkerW &w) {
  ++w.gen;
  if (w.gen >= (1ull << w.genb)) {
    for (int32_t i = threadIdx.x; i < w.hcap; i += 64) w.hs[i] = 0ull;
    __syncthreads();
    w.gen = 1;
  }
}

__device__ __forceinline__ unsigned long long wv_key(const WalkerW &w, int32_t p, int32_t grp) {
  return (w.gen << (w.pbits + w.gbits)) | ((unsigned long long)(uint32_t)grp << w.pbits) | (uint32_t)p;
}

__device__ __forceinline__ uint32_t wv_slot0(const WalkerW &w, int32_t p, int32_t grp) {
  const uint64_t h = (((uint64_t)(uint32_t)p << 32) | (uint32_t)grp) * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(h >> 33) & (uint32_t)(w.hcap - 1);
}

// insert (p, grp) into this generation's set: true if it was not there; *ovf on a full probe
__device__ __forceinline__ bool wv_insert(WalkerW &w, int32_t p, int32_t grp, bool *ovf) {
  const unsigned long long key = wv_key(w, p, grp);
  const int sh = w.pbits + w.gbits;
  uint32_t s = wv_slot0(w, p, grp);
  for (int32_t probe = 0; probe < w.hcap;) {
    unsigned long long cur = __hip_atomic_load(w.hs + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if ((cur >> sh) != w.gen) {  // empty for this generation: claim it
      const unsigned long long prev = atomicCAS(w.hs + s, cur, key);
      if (prev == cur) return true;
      continue;  // another lane wrote this slot: look at it again
    }
    if (cur == key) return false;
    s = (s + 1) & (uint32_t)(w.hcap - 1);
    ++probe;
  }
  *ovf = true;
  return false;
}

__device__ __forceinline__ bool wv_contains(const WalkerW &w, int32_t p, int32_t grp) {
  const unsigned long long key = wv_key(w, p, grp);
  const int sh = w.pbits + w.gbits;
  uint32_t s = wv_slot0(w, p, grp);
  for (int32_t probe = 0; probe < w.hcap; ++probe) {
    const unsigned long long cur = __hip_atomic_load(w.hs + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if ((cur >> sh) != w.gen) return false;
    if (cur == key) return true;
    s = (s + 1) & (uint32_t)(w.hcap - 1);
  }
  return false;
}

// lexicographic (lambda, hop) minimum across the wave
__device__ __forceinline__ void wv_min_key(double &l, int32_t &h) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double l2 = __shfl_xor(l, o, 64);
    const int32_t h2 = __shfl_xor(h, o, 64);
    if (kless(l2, h2, l, h)) {
      l = l2;
      h = h2;
    }
  }
}

// ws_walk with the whole workgroup (64 lanes, uniform arguments); the same value in every lane.
// -1 on scratch overflow (retried larger), -2 when the groups do not fit the key's group field.
__device__ int ws_walk_wave(const WsGeom &g, const int32_t *cand, int k, WalkerW &w, int32_t *layout) {
  const int lane = threadIdx.x;
  WSW_DBG("walk k=%d cap=%d hcap=%d gbits=%d pbits=%d genb=%d gen=%llu\n", k, w.cap, w.hcap, w.gbits, w.pbits, w.genb, w.gen);
  if (k <= 0 || k > w.gcap || k > w.cap) return -1;
  if (k >= (1 << w.gbits)) return -2;
  if (k == 1) return 0;
  int32_t *cp = w.pa, *cg = w.ga, *op = w.pb, *og = w.gb;
  for (int j = lane; j < k; j += 64) {
    cp[j] = cand[j];
    cg[j] = j;
    w.alive[j] = 1;
  }
  __syncthreads();
  int32_t ncur = k;
  for (int64_t step = 0;; ++step) {
    if (step > 4 * g.H * g.W + 16) return -1;
    // 1. basin members -> the non-basin pixels of equal key reachable through the basin
    wv_new_gen(w);
    int32_t nout = 0, hcount = 0;
    for (int32_t base = 0; base < ncur;) {  // ncur grows as basin members append
      const int32_t i = base + lane, lim = ncur;  // this batch: [base, min(base + 64, lim))
      int32_t x = -1, gr = 0, cc[4];
      int m = 0, isout = 0, isnew = 0;
      bool ovf = false;
      if (i < lim) {
        x = cp[i];
        gr = cg[i];
        if (wv_insert(w, x, gr, &ovf)) {
          isnew = 1;
          if (g_basin(g, x)) m = g_cands(g, x, cc);
          else isout = 1;
        }
      }
      if (__ballot(ovf)) { WSW_DBG("s1 ovf step %lld\n", (long long)step); return -1; }
      hcount += wv_sum(isnew);
      const int32_t ax = wv_excl(m), at = wv_sum(m), ox = wv_excl(isout), ot = wv_sum(isout);
      if (2 * hcount > w.hcap || ncur + at > w.cap || nout + ot > w.cap) { WSW_DBG("s1 cap step %lld hc %d ncur %d at %d nout %d ot %d\n", (long long)step, hcount, ncur, at, nout, ot); return -1; }
      for (int t = 0; t < m; ++t) {
        cp[ncur + ax + t] = cc[t];
        cg[ncur + ax + t] = gr;
      }
      if (isout) {
        op[nout + ox] = x;
        og[nout + ox] = gr;
      }
      __syncthreads();
      base = base + 64 < lim ? base + 64 : lim;  // the appended members come in later batches
      ncur += at;
      nout += ot;
    }
    WSW_DBG("step %lld ncur %d nout %d\n", (long long)step, ncur, nout);
    if (nout == 0) return -1;  // cannot happen (every string ends at a marker)
    // 2. the overall least key; groups without a member at it drop out
    double bl = __builtin_inf();
    int32_t bh = HOP_INF;
    for (int32_t i = lane; i < nout; i += 64) {
      const int32_t x = op[i];
      if (kless(g.lam[x], g.hop[x], bl, bh)) {
        bl = g.lam[x];
        bh = g.hop[x];
      }
    }
    wv_min_key(bl, bh);
    for (int j = lane; j < k; j += 64) w.hit[j] = 0;
    __syncthreads();
    for (int32_t i = lane; i < nout; i += 64) {
      const int32_t x = op[i];
      if (g.lam[x] == bl && g.hop[x] == bh) w.hit[og[i]] = 1;
    }
    __syncthreads();
    int nal = 0, last = -1;
    for (int j = lane; j < k; j += 64) {
      if (w.alive[j] && !w.hit[j]) w.alive[j] = 0;
      if (w.alive[j]) {
        ++nal;
        last = j > last ? j : last;
      }
    }
    nal = wv_sum(nal);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int l2 = __shfl_xor(last, o, 64);
      last = l2 > last ? l2 : last;
    }
    __syncthreads();
    WSW_DBG("  least %g %d nal %d last %d\n", bl, bh, nal, last);
    if (nal == 1) return last;
    // 3. members at the least key; markers among them end their string (BOTTOM . rank)
    for (int j = lane; j < k; j += 64) w.mr[j] = 0x7fffffff;
    __syncthreads();
    int32_t nkeep = 0;
    bool anym = false;
    for (int32_t base = 0; base < nout; base += 64) {
      const int32_t i = base + lane;
      int keep = 0;
      int32_t x = -1, gr = 0;
      if (i < nout) {
        x = op[i];
        gr = og[i];
        if (w.alive[gr] && g.lam[x] == bl && g.hop[x] == bh) {
          keep = 1;
          if (g_marker(g, x)) {
            atomicMin(w.mr + gr, x);
            anym = true;
          }
        }
      }
      const int32_t kx = wv_excl(keep), kt = wv_sum(keep);
      if (keep) {
        cp[nkeep + kx] = x;
        cg[nkeep + kx] = gr;
      }
      nkeep += kt;
    }
    const bool anyw = __ballot(anym) != 0ull;
    __syncthreads();
    if (anyw) {
      int win = -1;
      if (lane == 0) {  // ws_walk's marker decision, serially over the groups
        int nm = 0;
        int32_t l0 = 0, bmr = 0, bc = 0;
        bool multi = false;
        for (int j = 0; j < k; ++j) {
          const int32_t mrj = w.mr[j];
          if (!w.alive[j] || mrj == 0x7fffffff) continue;
          ++nm;
          if (nm == 1) l0 = g.mk[mrj];
          else if (g.mk[mrj] != l0) multi = true;
          const int32_t cj = cand[j];
          if (win < 0 || mrj < bmr || (mrj == bmr && cj < bc)) {
            win = j;
            bmr = mrj;
            bc = cj;
          }
        }
        if (nm > 1 && multi) *layout += 1;
      }
      return __shfl(win, 0, 64);
    }
    // 4. one symbol further: the union of the kept members' candidates, per group
    wv_new_gen(w);
    int32_t nn = 0;
    hcount = 0;
    for (int32_t base = 0; base < nkeep; base += 64) {
      const int32_t i = base + lane;
      int32_t cc[4], gr = 0;
      int m = 0, nnew = 0;
      bool ovf = false, isn[4] = {false, false, false, false};
      if (i < nkeep) {
        gr = cg[i];
        m = g_cands(g, cp[i], cc);
        for (int t = 0; t < m; ++t) {
          isn[t] = wv_insert(w, cc[t], gr, &ovf);
          nnew += isn[t];
        }
      }
      if (__ballot(ovf)) { WSW_DBG("s4 ovf\n"); return -1; }
      const int32_t nx = wv_excl(nnew), nt = wv_sum(nnew);
      hcount += nt;
      if (2 * hcount > w.hcap || nn + nt > w.cap) { WSW_DBG("s4 cap\n"); return -1; }
      int32_t o = nn + nx;
      for (int t = 0; t < m; ++t)
        if (isn[t]) {
          op[o] = cc[t];
          og[o] = gr;
          ++o;
        }
      nn += nt;
    }
    __syncthreads();
    int32_t *t0 = cp, *t1 = cg;
    cp = op;
    cg = og;
    op = t0;
    og = t1;
    ncur = nn;
    WSW_DBG("  keep %d next %d\n", nkeep, nn);
  }
}

// ws_resolve_one with the workgroup: the walk runs on all lanes, the basin component's BFS
// passes on lane 0 (their sets in the same hash).  Uniform result: false on scratch overflow or
// a group count the key cannot hold (then the pixel is retried with more scratch / fails loudly).
__device__ bool ws_resolve_one_wave(const WsGeom &g, int32_t x, int32_t *ptr, WalkerW &w, int32_t *layout) {
  const int lane = threadIdx.x;
  if (!g_basin(g, x)) {
    int32_t cc[4];
    const int m = g_cands(g, x, cc);
    const int win = ws_walk_wave(g, cc, m, w, layout);
    if (win < 0) return false;
    if (lane == 0) ptr[x] = cc[win];
    return true;
  }
  // component of equal-key basin pixels and its slots (lane 0), then the walk over the slots
  __shared__ int32_t s_ns, s_fail;
  wv_new_gen(w);
  if (lane == 0) {
    bool ovf = false, fail = false;
    int32_t nq = 0, ns = 0;
    wv_insert(w, x, 0, &ovf);
    w.pa[nq++] = x;
    for (int32_t qi = 0; qi < nq && !fail; ++qi) {
      int32_t cc[4];
      const int m = g_cands(g, w.pa[qi], cc);
      for (int j = 0; j < m; ++j) {
        if (!wv_insert(w, cc[j], 0, &ovf)) {
          if (ovf) fail = true;
          continue;
        }
        if (g_basin(g, cc[j])) {
          if (nq >= w.cap) fail = true;
          else w.pa[nq++] = cc[j];
        } else {
          if (ns >= w.cap) fail = true;
          else w.slots[ns++] = cc[j];
        }
      }
    }
    s_ns = ns;
    s_fail = fail;
  }
  __syncthreads();
  if (s_fail) return false;
  const int32_t ns = s_ns;
  const int win = ws_walk_wave(g, w.slots, ns, w, layout);
  if (win < 0) return false;
  // the component again as (p, 0), then a BFS tree over it rooted at the winning slot (p, 1):
  // every pixel points at a NEIGHBOUR, as ws_resolve_one builds it
  wv_new_gen(w);
  if (lane == 0) {
    bool ovf = false, fail = false;
    const int32_t wp = w.slots[win];
    int32_t nq = 0;
    wv_insert(w, x, 0, &ovf);
    w.pa[nq++] = x;
    for (int32_t qi = 0; qi < nq; ++qi) {
      int32_t cc[4];
      const int m = g_cands(g, w.pa[qi], cc);
      for (int j = 0; j < m; ++j)
        if (g_basin(g, cc[j]) && wv_insert(w, cc[j], 0, &ovf)) w.pa[nq++] = cc[j];
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
        if (y < 0 || !wv_contains(w, y, 0) || !wv_insert(w, y, 1, &ovf)) continue;
        if (nt2 >= w.cap) {
          fail = true;
          break;
        }
        ptr[y] = q;
        w.pb[nt2++] = y;
      }
    }
    s_fail = fail || ovf;
  }
  __syncthreads();
  return !s_fail;
}

}  // namespace hrf_ws
