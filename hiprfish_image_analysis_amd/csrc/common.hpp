// common.hpp -- shared plumbing for libhrf.so (MI355X / gfx950 only).
//
// Every C-ABI entry point returns an hrf_status (0 = OK) and records a thread-local
// message retrievable with hrf_last_error().  All device work is stream-ordered on the
// caller's hipStream_t; nothing here synchronises unless an entry point says so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/hrf.h"

namespace hrf {

void set_error(const char *fmt, ...);

struct Err {
  hrf_status code;
};

#define HRF_REQUIRE(cond, ...)                    \
  do {                                            \
    if (!(cond)) {                                \
      ::hrf::set_error(__VA_ARGS__);              \
      return HRF_EINVAL;                          \
    }                                             \
  } while (0)

#define HRF_HIP(expr)                                                               \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ::hrf::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                       __FILE__, __LINE__);                                         \
      return HRF_EHIP;                                                              \
    }                                                                               \
  } while (0)

#define HRF_LAUNCHED()                                                              \
  do {                                                                              \
    hipError_t e_ = hipGetLastError();                                              \
    if (e_ != hipSuccess) {                                                         \
      ::hrf::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(e_),  \
                       __FILE__, __LINE__);                                         \
      return HRF_EHIP;                                                              \
    }                                                                               \
  } while (0)

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Grid for a grid-stride elementwise kernel: at most 512 blocks (two per CU).  Beside the
// concurrent classifier every dispatched block waits for a CU slot, so fewer, longer blocks win:
// 1037-1050 vs 1027-1042 Mpix/s against 2048 (means of 3; 4 of 6 interleaved pairs; 256: 1032,
// 1024: 1030).
constexpr int64_t STREAM_GRID_MAX = 512;
inline unsigned stream_grid(int64_t n, int block = 256) {
  int64_t g = cdiv(n, block);
  if (g > STREAM_GRID_MAX) g = STREAM_GRID_MAX;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Grid for a persistent chunk loop: exactly the blocks that are resident at once (occupancy
// x CUs), so every CU runs the same number of chunk iterations and no partial second wave of
// blocks trails the launch.  The CU count is cached per device.
inline int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}
template <class Kern>
inline unsigned resident_grid(Kern kernel, int block, size_t shm, int64_t nwork) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, shm) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  int64_t g = (int64_t)per_cu * cu_count();
  if (g > nwork) g = nwork;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Line-profile sampling tables (neighbor2d.pyx:32-55, neighbor.pyx:209-243), computed on
// the host and uploaded per call.  tables.cpp.
int lp_table_2d(int patch, int nphi, int32_t *off /*[nphi][patch][2]*/);
int lp_table_3d(int patch, int ntheta, int nphi, int32_t *off /*[ndir][patch][3]*/);

// hrf_erosion_seeds with the component boxes already read back to the host (seeds.hip)
hrf_status erosion_seeds_hostbox(const int32_t *labels, int64_t H, int64_t W, int32_t ncomp, const int32_t *box,
                                 const int32_t *hb, int32_t area_max, int32_t min_obj, uint8_t *be_out,
                                 hipStream_t s, int32_t *ovf_dev, char *px_scratch);
int64_t seed_px_scratch_bytes();  // px_scratch size for erosion_seeds_hostbox

hrf_status kmeans_1d_sorted_pair_deferred(const double *x, int64_t n, int32_t k1, int32_t k2, int32_t max_iter,
                                          int32_t n_init, int32_t rule1, int32_t rule2, uint8_t *top1, uint8_t *top2,
                                          void *work, int64_t work_bytes, hipStream_t s, int32_t *err_pinned);
const int32_t *kmeans_error_flag(void *work, int64_t n);

// the per-cell tail with device-held row counts (classify.hip, stats.hip; used by tile.hip)
hrf_status cells_lib_prep(const double *a, int32_t R, int32_t C, const int32_t *bounds_host, int32_t nseg, double *t,
                          double *ny, hipStream_t s);
hrf_status segment_flags_devn(const double *x, int64_t nmax, const int32_t *nrows_dev, int32_t C,
                              const int32_t *bounds_host, int32_t nseg, double thr, double *out, hipStream_t s);
hrf_status classify_cells_devn(const double *x, int64_t nmax, const int32_t *nrows_dev, const double *refT,
                               const double *ny, int32_t R, int32_t C, const int32_t *bounds_host, int32_t nseg,
                               int32_t variant, const double *fx, const double *fr, int32_t *arg, double *dmin,
                               hipStream_t s);
hrf_status barcode_counts_devn(const int32_t *bc, int64_t nmax, const int32_t *n_dev, int32_t R, int64_t *counts,
                               hipStream_t s, bool zeroed = false);
hrf_status paint_ids_devn(const int32_t *labels, int64_t n, const int32_t *code, int32_t nmax, const int32_t *ncell_dev,
                          int32_t add, int32_t *out, hipStream_t s);
// One kernel that clears device buffers and copies device words into pinned host memory the
// caller reads after its next synchronisation (chainops.hip).  The native chains use it in
// place of hipMemsetAsync / hipMemcpyAsync(DeviceToHost), whose rocclr fill and copy kernels
// are each a dispatch of their own between the chain's kernels.
struct ZeroPub {
  static constexpr int N = 10;
  int nz = 0, np = 0;
  void *zp[N];
  int64_t zw[N];  // 4-byte words to clear
  const int32_t *ps[N];
  int32_t *pd[N];  // device address of pinned host memory (hrf::mapped)
  int32_t pn[N];
  bool zero(void *p, int64_t bytes) {
    if (!p || bytes <= 0) return true;
    if (nz == N || bytes % 4 != 0) return false;
    zp[nz] = p;
    zw[nz++] = bytes / 4;
    return true;
  }
  bool pub(const int32_t *src, int32_t *dst_dev, int32_t words) {
    if (words <= 0) return true;
    if (np == N || !src || !dst_dev) return false;
    ps[np] = src;
    pd[np] = dst_dev;
    pn[np++] = words;
    return true;
  }
};
hrf_status zero_publish(const ZeroPub &z, hipStream_t s);
// hrf_label(mask, u8, conn) with the component count left in device memory (label.hip)
int64_t label_dev_ws_words(int64_t n);
hrf_status label_dev(const uint8_t *mask, int64_t H, int64_t W, int32_t conn, int32_t *labels,
                          int32_t *parent_ws, int32_t *blk_ws, int32_t *nlab_dev, hipStream_t s);
// hrf_binary_erosion(border_value) followed by hrf_binary_dilation, fused (label.hip)
hrf_status binary_opening(const uint8_t *mask, int64_t H, int64_t W, int32_t border_value, uint8_t *out,
                          hipStream_t s);
// hrf_remove_small_objects_labels / hrf_region_moments on count buffers the caller has cleared
hrf_status remove_small_objects_labels_zeroed(const int32_t *labels, int64_t n, int32_t maxlab, int64_t min_size,
                                              int32_t *out, int32_t *cnt_ws, hipStream_t s);
hrf_status region_moments_zeroed(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, int64_t *mom,
                                 hipStream_t s);
// hrf_label_sums_lasers on sums / counts the caller has cleared
hrf_status label_sums_lasers_zeroed(const float *const *src_host, const int32_t *channels_host,
                                    const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                    int32_t apply_mask, const int32_t *labels, int32_t maxlab, const float *cal,
                                    int32_t cal_c0, int32_t cal_c1, double *sums, int64_t *counts, hipStream_t s);
hrf_status segment_ecoli_cn_extra(hrf_seg_ctx *c, const double *image_cn, int32_t *seg_out, int32_t *maxlab_host,
                                  hipStream_t s, const ZeroPub *extra);
hrf_status watershed_ex_extra(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask,
                              int64_t H, int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws,
                              int32_t max_passes, int32_t *passes_host, int32_t *ties_host, hipStream_t s,
                              const ZeroPub *extra);
// device address of pinned host memory from hipHostMalloc (nullptr when it has none)
int32_t *mapped(int32_t *host);
// hipHostMalloc with the flags zero_publish's host slots need (mapped, coherent)
hipError_t host_alloc_mapped(void **p, size_t bytes);

}  // namespace hrf
