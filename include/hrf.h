/*
 * hrf.h -- C ABI of libhrf.so, the MI355X (gfx950) HiPR-FISH measurement/classification
 * hot path.  Plain C: pointers, sizes, status codes.  No torch or HIP C++ types.
 *
 * Conventions
 *   - Every function returns hrf_status; on failure hrf_last_error() holds a message
 *     (thread-local, valid until the next failing call on the same thread).
 *   - Buffers are caller-owned DEVICE pointers (e.g. torch tensor data_ptr()), row-major,
 *     unless a parameter says "host".  The library never frees caller memory.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  Work is
 *     stream-ordered and asynchronous; functions that return a host-visible count say so
 *     and synchronise the stream.
 *   - Scratch: functions needing temporary device memory take a `work` pointer and its
 *     size in bytes; hrf_*_workspace() reports the size needed.
 *
 * Each entry point names the reference interface it replaces (file:line, relative to the
 * reference repository root).
 */
#ifndef HRF_H
#define HRF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t hrf_status;
#define HRF_OK 0
#define HRF_EINVAL 1   /* bad argument (shape, size, unsupported parameter) */
#define HRF_EHIP 2     /* HIP runtime error */
#define HRF_ENOMEM 3   /* workspace too small */

typedef void *hrf_stream_t;

#if defined(__GNUC__)
#define HRF_API __attribute__((visibility("default")))
#else
#define HRF_API
#endif

HRF_API const char *hrf_last_error(void);
/* library version as 0xMMmmpp */
HRF_API int32_t hrf_version(void);
/* 1 when a gfx950 device is visible, else 0 (no error) */
HRF_API int32_t hrf_device_ok(void);

/* ---- line-profile tables (host) ----------------------------------------------------
 * neighbor2d.pyx:32-55 and neighbor.pyx:209-243: sampling offsets inside a patch. */
HRF_API hrf_status hrf_lp_table_2d(int32_t patch, int32_t nphi, int32_t *off_host /*[nphi][patch][2]*/);
HRF_API hrf_status hrf_lp_table_3d(int32_t patch, int32_t ntheta, int32_t nphi,
                           int32_t *off_host /*[(ntheta-1)*nphi][patch][3]*/);

/* ---- a5: neighbor2d.line_profile_2d_v2(image_padded, patch_size, phi_range) ----------
 * neighbor2d.pyx:8-64.  pad (hp, wp) f64, row stride ld (elements).
 * out (hp-patch+1, wp-patch+1, nphi, patch) f64, contiguous. */
HRF_API hrf_status hrf_line_profile_2d(const double *pad, int64_t hp, int64_t wp, int64_t ld, int32_t patch,
                               int32_t nphi, double *out, hrf_stream_t stream);

/* ---- a5+a6 fused: line profile + 2-D enhancement chain ----------------------------
 * multispecies_spectral_image_measurement.py:110-124 (biofilm :352-366).
 * final (hp-patch+1, wp-patch+1) f64.  Bit-exact with the numpy chain (NaN on flat lines). */
HRF_API hrf_status hrf_enhance_2d(const double *pad, int64_t hp, int64_t wp, int64_t ld, int32_t patch,
                          int32_t nphi, double *final_, hrf_stream_t stream);

/* ---- a7: neighbor.line_profile_v2 (neighbor.pyx:115-181) ------------------------------
 * pad (xp, yp, zp) f64 contiguous -> out (X, Y, Z, (ntheta-1)*nphi, patch) f64. */
HRF_API hrf_status hrf_line_profile_3d(const double *pad, int64_t xp, int64_t yp, int64_t zp, int32_t patch,
                               int32_t ntheta, int32_t nphi, double *out, hrf_stream_t stream);

/* ---- a7: neighbor.line_profile_memory_efficient_v2 (neighbor.pyx:186-263) -------------
 * out (X, Y, Z, (ntheta-1)*nphi) f64: (centre-min)/max(max-min, 1e-8) per direction. */
HRF_API hrf_status hrf_line_profile_3d_norm(const double *pad, int64_t xp, int64_t yp, int64_t zp,
                                    int32_t patch, int32_t ntheta, int32_t nphi, double *out,
                                    hrf_stream_t stream);

/* ---- a7 fused: 3-D enhancement (biofilm_analysis.py:811-817) -------------------------
 * final (X, Y, Z) f64 = mean_dir * (1 - nan_to_num((q75-q25)/(q75+q25))); never
 * materialises the (X,Y,Z,72) intermediate.  patch 11, ntheta 9, nphi 9 only. */
HRF_API hrf_status hrf_enhance_3d(const double *pad, int64_t xp, int64_t yp, int64_t zp, int32_t patch,
                          int32_t ntheta, int32_t nphi, double *final_, hrf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HRF_H */
