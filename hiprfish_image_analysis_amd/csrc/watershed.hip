// watershed.hip -- marker-controlled watershed (a12) as a parallel minimax relaxation.
//
// Reference: skimage.morphology.watershed(image, markers, mask) (ecoli measurement.py:113,
// multispecies :154): a sequential heap flood, (value, age) ordered, labels on push.
// Pop order of that flood is non-decreasing in the flood level
//   lambda(q) = min over marker paths of max value on the path    (lambda(marker) = value),
// and a pixel takes the label of its first-popped neighbour, i.e. the neighbour with the
// least lambda.  Within one flood level the pixels of a basin are entered through a single
// pass pixel, so ties there carry one label.  We therefore relax, per pixel, the key
//   (lambda, hops) with hops = plateau distance from where lambda was last raised:
// from the least-key labelled neighbour p, lambda(q) = max(f(q), lambda(p)) and
// hops(q) = lambda(p) >= f(q) ? hops(p) + 1 : 0, and q takes p's label.  Keys strictly
// increase along these pointers, so the fixed point is unique (ties -> smaller label).  On inputs without equal competing
// values this reproduces the heap flood exactly (tests/test_watershed_gpu.py checks it
// against the restated heap flood, oracle_watershed).
//
// Execution: 32x32 tiles with a 1-pixel halo in LDS, Jacobi sweeps inside the tile until it
// is locally stable, ping-pong state between global passes until no tile changes.
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
                               int32_t *__restrict__ hop, int32_t *__restrict__ lab) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool in = !mask || mask[i];
    const int32_t m = in ? markers[i] : 0;
    lam[i] = m ? (negate ? -f[i] : f[i]) : __builtin_inf();
    hop[i] = m ? 0 : HOP_INF;
    lab[i] = m;
  }
}

__device__ __forceinline__ bool better(double l1, int32_t h1, int32_t b1, double l2, int32_t h2, int32_t b2) {
  if (l1 != l2) return l1 < l2;
  if (h1 != h2) return h1 < h2;
  return b1 < b2;
}

// flags: bit0 = in mask, bit1 = marker (fixed)
__global__ __launch_bounds__(256) void ws_pass_kernel(const double *__restrict__ f, int negate,
                                                      const int32_t *__restrict__ markers,
                                                      const uint8_t *__restrict__ mask, int64_t H, int64_t W,
                                                      WsState in, WsState out, int32_t *__restrict__ changed,
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
#pragma unroll
  for (int k = 0; k < 4; ++k) own[k] = ((tid >> 5) + 8 * k + 1) * WL + (tid & 31) + 1;
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
      // first-popped neighbour = least (lambda, hops) among labelled in-mask neighbours
      double bl = __builtin_inf();
      int32_t bh = HOP_INF, bb = 0;
      const int nbr[4] = {i - WL, i - 1, i + 1, i + WL};
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
        nl[k] = bl >= fv ? bl : fv;
        nh[k] = bl >= fv ? bh + 1 : 0;
        nb[k] = bb;
      }
      ch |= (nb[k] != sb[i]) || (nl[k] != sl[i]) || (nh[k] != sh[i]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sl[own[k]] = nl[k];
      sh[own[k]] = nh[k];
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
      out.lam[g] = sl[i];
      out.hop[g] = sh[i];
      out.lab[g] = sb[i];
    }
  }
  if (__syncthreads_or(any_change) && tid == 0) {
    *changed = 1;
    cur_tile[blockIdx.y * gridDim.x + blockIdx.x] = 1;
  }
}

}  // namespace

extern "C" {

// state_ws: 2 * n * (8 + 4 + 4) bytes; flags_ws: >= 1 int32
hrf_status hrf_watershed(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask, int64_t H, int64_t W,
                         int32_t *out_labels, void *state_ws, int32_t *flag_ws, int32_t max_passes,
                         int32_t *passes_host, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = H * W;
  HRF_REQUIRE(H >= 0 && W >= 0 && H <= 65535 * (int64_t)WT && W <= 65535 * (int64_t)WT, "watershed: bad shape");
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(image && markers && out_labels && state_ws && flag_ws, "watershed: null buffer");
  char *ws = (char *)state_ws;
  WsState a{(double *)ws, (int32_t *)(ws + 8 * n), (int32_t *)(ws + 12 * n)};
  WsState b{(double *)(ws + 16 * n), (int32_t *)(ws + 24 * n), (int32_t *)(ws + 28 * n)};
  ws_init_kernel<<<hrf::stream_grid(n), 256, 0, s>>>(image, negate, markers, mask, n, a.lam, a.hop, a.lab);
  HRF_LAUNCHED();
  dim3 grid((unsigned)hrf::cdiv(W, WT), (unsigned)hrf::cdiv(H, WT));
  const int64_t ntiles = (int64_t)grid.x * grid.y;
  int32_t *tf = nullptr;  // per-tile change flags, three rotating generations
  HRF_HIP(hipMallocAsync((void **)&tf, sizeof(int32_t) * 3 * ntiles, s));
  HRF_HIP(hipMemsetAsync(tf, 0, sizeof(int32_t) * 2 * ntiles, s));  // generations of passes 0 and 1
  int passes = 0;
  // Passes run in batches with one host read per batch: the first batch of 8 covers the
  // typical tile (~7 passes) with a single synchronisation, later batches 4.  Passes after
  // convergence change nothing (unique fixed point) and skip every tile (no tile changed).
  // flag_ws[0] = change flag of the batch's last pass, flag_ws[1] = scratch for the others.
  for (int batch = 8;; batch = 4) {
    HRF_HIP(hipMemsetAsync(flag_ws, 0, sizeof(int32_t) * 2, s));
    for (int k = 0; k < batch; ++k) {
      int32_t *cur = tf + (passes % 3) * ntiles;
      const int32_t *prev = passes == 0 ? nullptr : tf + ((passes + 2) % 3) * ntiles;
      int32_t *next = tf + ((passes + 1) % 3) * ntiles;
      ws_pass_kernel<<<grid, 256, 0, s>>>(image, negate, markers, mask, H, W, a, b, flag_ws + (k == batch - 1 ? 0 : 1),
                                          prev, cur, next);
      WsState t = a;
      a = b;
      b = t;
      ++passes;
    }
    HRF_LAUNCHED();
    int32_t fl = 0;
    HRF_HIP(hipMemcpyAsync(&fl, flag_ws, sizeof(fl), hipMemcpyDeviceToHost, s));
    HRF_HIP(hipStreamSynchronize(s));
    if (!fl || passes >= max_passes) break;
  }
  HRF_HIP(hipFreeAsync(tf, s));
  HRF_HIP(hipMemcpyAsync(out_labels, a.lab, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
  if (passes_host) *passes_host = passes;
  return HRF_OK;
}

}  // extern "C"
