// ws_emul.cpp -- development tool: replays hrf_watershed_ex's flow on the CPU with the SAME
// resolution code (csrc/ws_core.hpp), serially, so the tie logic can be checked against the
// heap flood (oracle_watershed) without a GPU.  Not part of libhrf.so.
//   hipcc -O2 -fPIC -shared -o tools/libws_emul.so tools/ws_emul.cpp
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../hiprfish_image_analysis_amd/csrc/ws_core.hpp"

using namespace hrf_ws;

static bool better(double l1, int32_t h1, int32_t d1, int32_t b1, double l2, int32_t h2, int32_t d2, int32_t b2) {
  if (l1 != l2) return l1 < l2;
  if (h1 != h2) return h1 < h2;
  if (d1 != d2) return d1 < d2;
  return b1 < b2;
}

extern "C" int ws_emul(const double *f, int negate, const int32_t *mk, const uint8_t *mask, int64_t H, int64_t W,
                       int32_t *out, int32_t *ties, int32_t *ptr_out = nullptr, double *lam_out = nullptr,
                       int32_t *hop_out = nullptr) {
  const int64_t n = H * W;
  std::vector<double> lam(n);
  std::vector<int32_t> hop(n), lab(n), ptr(n, -1), dst(n);
  auto in = [&](int64_t i) { return !mask || mask[i]; };
  for (int64_t i = 0; i < n; ++i) {
    const int32_t m = in(i) ? mk[i] : 0;
    lam[i] = m ? (negate ? -f[i] : f[i]) : INFINITY;
    hop[i] = m ? 0 : HOP_INF;
    dst[i] = m ? 0 : HOP_INF;
    lab[i] = m;
  }
  auto nbrs = [&](int64_t x, int64_t *nb) {
    const int64_t r = x / W, c = x % W;
    int k = 0;
    if (r > 0) nb[k++] = x - W;
    if (c > 0) nb[k++] = x - 1;
    if (c + 1 < W) nb[k++] = x + 1;
    if (r + 1 < H) nb[k++] = x + W;
    return k;
  };
  for (bool ch = true; ch;) {  // relaxation, the pass kernel's rule
    ch = false;
    for (int64_t x = 0; x < n; ++x) {
      if (!in(x) || (in(x) && mk[x])) continue;
      int64_t nb[4];
      const int k = nbrs(x, nb);
      double bl = INFINITY;
      int32_t bh = HOP_INF, bd = HOP_INF, bb = 0;
      for (int j = 0; j < k; ++j) {
        const int64_t y = nb[j];
        if (!lab[y] || !in(y)) continue;
        if (better(lam[y], hop[y], dst[y], lab[y], bl, bh, bd, bb)) bl = lam[y], bh = hop[y], bd = dst[y], bb = lab[y];
      }
      if (!bb) continue;
      const double fv = negate ? -f[x] : f[x];
      double nl;
      int32_t nh, nd;
      if (bl < fv) nl = fv, nh = 0, nd = 0;
      else if (bl == fv) nl = bl, nh = bh + 1, nd = 0;
      else nl = bl, nh = bh, nd = bd + 1;
      if (nl != lam[x] || nh != hop[x] || nd != dst[x] || bb != lab[x]) {
        lam[x] = nl;
        hop[x] = nh;
        dst[x] = nd;
        lab[x] = bb;
        ch = true;
      }
    }
  }
  WsGeom g{f, negate, mk, mask, H, W, lam.data(), hop.data()};
  const int32_t capx = getenv("WS_EMUL_CAPX") ? atoi(getenv("WS_EMUL_CAPX")) : 16;
  const int32_t cap = getenv("WS_EMUL_SMALL") ? 4096 : (int32_t)(capx * n + 64),
                hcap = getenv("WS_EMUL_SMALL") ? 8192 : 1 << (int)std::ceil(std::log2(2.0 * (capx * n + 64))), gcap = cap;
  std::vector<int32_t> pa(cap), ga(cap), pb(cap), gb(cap), slots(cap), mh(gcap), mr(gcap);
  std::vector<uint64_t> hkey(hcap);
  std::vector<uint32_t> hgen(hcap, 0);
  std::vector<double> ml(gcap);
  std::vector<uint8_t> alive(gcap);
  Walker w{pa.data(), ga.data(), pb.data(), gb.data(), slots.data(), hkey.data(), hgen.data(), ml.data(),
           mh.data(), mr.data(), alive.data(), cap, hcap, gcap, 0, 0};
  int32_t total = 0, rounds = 0, layout = 0;
  for (;;) {
    std::vector<int32_t> list;
    for (int64_t x = 0; x < n; ++x) {
      if (!in(x) || mk[x] || lam[x] == INFINITY || ptr[x] >= 0) continue;
      int32_t cc[4];
      const int m = g_cands(g, x, cc);
      bool diff = false;
      for (int j = 1; j < m; ++j) diff |= lab[cc[j]] != lab[cc[0]];
      if (diff) list.push_back((int32_t)x);
    }
    if (list.empty()) break;
    total += (int32_t)list.size();
    ++rounds;
    if (getenv("WS_EMUL_CHECK")) {  // every listed basin pixel resolves its component alone
      std::vector<int32_t> ref(n, -1), tmp(n, -1);
      for (int32_t x : list) {
        if (!(!in(x) || mk[x]) && (negate ? -f[x] : f[x]) < lam[x]) {
          std::fill(tmp.begin(), tmp.end(), -1);
          int32_t lay = 0;
          if (!ws_resolve_one(g, x, tmp.data(), w, &lay)) return 3;
          for (int64_t i = 0; i < n; ++i)
            if (tmp[i] >= 0) {
              if (ref[i] >= 0 && ref[i] != tmp[i]) {
                fprintf(stderr, "inconsistent tree at %lld (from %d): %d vs %d\n", (long long)i, x, ref[i], tmp[i]);
              }
              ref[i] = tmp[i];
            }
        }
      }
    }
    if (getenv("WS_EMUL_ROOTS")) {
      std::vector<int32_t> tmp(n, -1);
      for (int32_t x : list) {
        int32_t lay = 0, rt = -1;
        ws_resolve_one(g, x, tmp.data(), w, &lay, &rt);
        fprintf(stderr, "emul: round %d resolve %d -> %d\n", rounds, x, rt);
      }
    }
    for (int32_t x : list) {
      if (ptr[x] >= 0) continue;
      if (!ws_resolve_one(g, x, ptr.data(), w, &layout)) return 1;
    }
    for (int64_t i = 0; i < n; ++i) lab[i] = in(i) ? mk[i] : 0;
    const bool jacobi = getenv("WS_EMUL_JACOBI") != nullptr;
    for (bool ch = true; ch;) {  // relabel, the RELABEL pass rule
      ch = false;
      std::vector<int32_t> old(lab);
      for (int64_t x = 0; x < n; ++x) {
        if (!in(x) || mk[x] || lam[x] == INFINITY) continue;
        int32_t lb = 0;
        const int32_t *src = jacobi ? old.data() : lab.data();
        if (ptr[x] >= 0) lb = src[ptr[x]];
        else {
          int32_t cc[4];
          const int m = g_cands(g, x, cc);
          for (int j = 0; j < m; ++j)
            if (src[cc[j]] && (!lb || src[cc[j]] < lb)) lb = src[cc[j]];
        }
        if (lb != lab[x]) {
          lab[x] = lb;
          ch = true;
        }
      }
    }
    if (rounds > 10000) return 2;
  }
  std::memcpy(out, lab.data(), sizeof(int32_t) * n);
  if (ptr_out) std::memcpy(ptr_out, ptr.data(), sizeof(int32_t) * n);
  if (lam_out) std::memcpy(lam_out, lam.data(), sizeof(double) * n);
  if (hop_out) std::memcpy(hop_out, hop.data(), sizeof(int32_t) * n);
  ties[0] = total;
  ties[1] = rounds;
  ties[2] = layout;
  return 0;
}
