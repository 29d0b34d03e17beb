// core.hip -- error plumbing, version, device probe and the line-profile sampling tables.
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>

#include "common.hpp"

namespace hrf {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

// One sampled line of `patch` taps (neighbor2d.pyx:35-55 / neighbor.pyx:213-243): the
// 2*|max interval|+1 samples of the direction `iv` (round-half-even of increment *
// direction cosines) are laid along the patch with truncating division; when the line is
// shorter than the patch its first/last sample repeats at both ends.
static void sample_line(int patch, int ndim, const long long *iv, int32_t *off) {
  const int inc = (patch - 1) / 2;
  int arg = 0;
  for (int k = 1; k < ndim; ++k)
    if (std::llabs(iv[k]) > std::llabs(iv[arg])) arg = k;
  const int line_n = (int)(2 * std::llabs(iv[arg]) + 1);
  const int base = line_n < patch ? (patch - line_n) / 2 : 0;
  std::memset(off, 0, sizeof(int32_t) * patch * ndim);
  for (int li = 0; li < line_n; ++li)
    for (int k = 0; k < ndim; ++k) {
      const long long s = (iv[k] > 0) - (iv[k] < 0);
      const double h = (double)(s * li) * (double)(2 * std::llabs(iv[k]) + 1) / (double)line_n;
      const double tr = (h > 0 ? 1.0 : (h < 0 ? -1.0 : 0.0)) * std::floor(std::fabs(h));
      off[(li + base) * ndim + k] = (int32_t)(tr + (double)inc - (double)iv[k]);
    }
  if (line_n < patch) {
    for (int li = 0; li < base; ++li)
      for (int k = 0; k < ndim; ++k) {
        off[li * ndim + k] = off[base * ndim + k];
        off[(li + line_n + base) * ndim + k] = off[(line_n + base - 1) * ndim + k];
      }
  }
}

int lp_table_2d(int patch, int nphi, int32_t *off) {
  const int inc = (patch - 1) / 2;
  for (int phi = 0; phi < nphi; ++phi) {
    const double a = (double)phi * M_PI / (double)nphi;
    long long iv[2] = {(long long)std::nearbyint((double)inc * std::cos(a)),
                       (long long)std::nearbyint((double)inc * std::sin(a))};
    sample_line(patch, 2, iv, off + (size_t)phi * patch * 2);
  }
  return 0;
}

int lp_table_3d(int patch, int ntheta, int nphi, int32_t *off) {
  const int inc = (patch - 1) / 2;
  for (int th = 1; th < ntheta; ++th)
    for (int phi = 0; phi < nphi; ++phi) {
      const double ap = (double)phi * M_PI / (double)nphi;
      const double at = (double)th * M_PI / (double)ntheta;
      long long iv[3] = {(long long)std::nearbyint((double)inc * std::cos(ap) * std::sin(at)),
                         (long long)std::nearbyint((double)inc * std::sin(ap) * std::sin(at)),
                         (long long)std::nearbyint((double)inc * std::cos(at))};
      sample_line(patch, 3, iv, off + (size_t)((th - 1) * nphi + phi) * patch * 3);
    }
  return 0;
}

}  // namespace hrf

extern "C" {

const char *hrf_last_error(void) { return hrf::g_err.c_str(); }

int32_t hrf_version(void) { return 0x000100; }

int32_t hrf_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 0;
  hipDeviceProp_t p;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return std::strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

hrf_status hrf_lp_table_2d(int32_t patch, int32_t nphi, int32_t *off_host) {
  HRF_REQUIRE(patch >= 1 && patch <= 64 && nphi >= 1 && nphi <= 64 && off_host,
              "hrf_lp_table_2d: bad arguments");
  hrf::lp_table_2d(patch, nphi, off_host);
  return HRF_OK;
}

hrf_status hrf_lp_table_3d(int32_t patch, int32_t ntheta, int32_t nphi, int32_t *off_host) {
  HRF_REQUIRE(patch >= 1 && patch <= 64 && ntheta >= 2 && nphi >= 1 && (ntheta - 1) * nphi <= 512 && off_host,
              "hrf_lp_table_3d: bad arguments");
  hrf::lp_table_3d(patch, ntheta, nphi, off_host);
  return HRF_OK;
}

}  // extern "C"
