// common.hpp -- shared plumbing for libhrf.so (MI355X / gfx950 only).
//
// Every C-ABI entry point returns an hrf_status (0 = OK) and records a thread-local
// message retrievable with hrf_last_error().  All device work is stream-ordered on the
// caller's hipStream_t; nothing here synchronises unless an entry point says so.
#pragma once
#include <hip/hip_runtime.h>

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

// Grid for a grid-stride elementwise kernel: enough blocks to fill 256 CUs x 8.
inline unsigned stream_grid(int64_t n, int block = 256) {
  int64_t g = cdiv(n, block);
  if (g > 2048) g = 2048;
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
                               hipStream_t s);
hrf_status paint_ids_devn(const int32_t *labels, int64_t n, const int32_t *code, int32_t nmax, const int32_t *ncell_dev,
                          int32_t add, int32_t *out, hipStream_t s);
}  // namespace hrf
