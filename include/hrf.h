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
typedef void *hrf_event_t; /* hipEvent_t */

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
/* neighbor.line_profile_memory_efficient_v3(pad, 11, 9, 9) (neighbor.pyx:268-349; imported
 * by biofilm :40): its own table, flat-address reads as the reference's unchecked memoryview
 * makes them (0 past the array's end, where the reference is undefined),
 * out (X,Y,Z) = mean * (p25 - p75) / (p25 + p75 + 1e-8). */
HRF_API hrf_status hrf_enhance_3d_v3(const double *pad, int64_t xp, int64_t yp, int64_t zp, int32_t patch,
                                     int32_t ntheta, int32_t nphi, double *out, hrf_stream_t stream);


/* ==== a1-a3: stack assembly and channel reductions (stack.hip) ======================== */
/* ecoli measurement.py:51-70 / multispecies :88-102: per-laser (H,W,C_l) f32 stacks
 * (src_host = HOST array of DEVICE pointers) shifted by integer (dr, dc) each
 * (shifts_host[2*i], [2*i+1]) and concatenated into dst (H,W,sum C_l); zero outside each
 * laser's coverage; apply_mask=1 also zeroes pixels outside the coverage intersection
 * (ecoli :69-70). */
HRF_API hrf_status hrf_register_assemble(const float *const *src_host, const int32_t *channels_host,
                                         const int32_t *shifts_host, int32_t nlaser, int64_t H, int64_t W,
                                         int32_t apply_mask, float *dst, hrf_stream_t stream);
/* the same with the shifts read from DEVICE memory (shifts_dev: nlaser (dr, dc) int32 pairs,
 * e.g. written by hrf_register_translation_dev): no host round trip between estimate and apply */
HRF_API hrf_status hrf_register_assemble_dev(const float *const *src_host, const int32_t *channels_host,
                                             const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                             int32_t apply_mask, float *dst, hrf_stream_t stream);
/* the same, also writing the channel sum of the assembled stack (numpy pairwise order, f64;
 * cn_mode 0 sum, 1 log(sum + 1e-2) = ecoli :71-72 image_cn, 2 log10(sum + 1)) from the tile
 * the assembly already holds -- no second pass over the stack.  cn_out (H x W) f64 */
HRF_API hrf_status hrf_register_assemble_cn_dev(const float *const *src_host, const int32_t *channels_host,
                                                const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                                int32_t apply_mask, float *dst, double *cn_out, int32_t cn_mode,
                                                hrf_stream_t stream);
/* the E. coli registered assembly (five lasers, W a multiple of 16) writing image_cn (cn_mode as
 * above) and the per-pixel classifier's prepared operands (table: hrf_pixtable_bytes(H * W, ...)
 * bytes, flags: H * W bytes; see hrf_pixtable_prepare) from the same LDS strip; dst (nullable)
 * also receives the registered stack -- without it the stack never exists (the per-cell spectra
 * then come from hrf_label_sums_lasers).  table and flags both NULL: image_cn only */
HRF_API hrf_status hrf_register_assemble_pixtable(const float *const *src_host, const int32_t *channels_host,
                                                  const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                                  int32_t apply_mask, float *dst, double *cn_out, int32_t cn_mode,
                                                  void *table, uint8_t *flags, hrf_stream_t stream);
/* hrf_label_sums of the registered stack hrf_register_assemble_dev would build (shifts on the
 * device, apply_mask), read from the per-laser acquisitions; cal (nullable): a per-pixel (H, W)
 * flat field dividing channels [cal_c0, cal_c1) */
HRF_API hrf_status hrf_label_sums_lasers(const float *const *src_host, const int32_t *channels_host,
                                         const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                         int32_t apply_mask, const int32_t *labels, int32_t maxlab, const float *cal,
                                         int32_t cal_c0, int32_t cal_c1, double *sums, int64_t *counts,
                                         hrf_stream_t stream);
/* per-pixel sum over C in numpy pairwise order (== np.sum(stack, axis=2) in f64);
 * mode 0: sum, 1: log(sum + 1e-2) (ecoli :72), 2: log10(sum + 1) (biofilm :831);
 * mask (nullable) zeroes the sum; negate flips the sign (watershed input). */
HRF_API hrf_status hrf_channel_sum(const float *stack, int64_t npix, int32_t C, const uint8_t *mask, int32_t mode,
                                   int32_t negate, double *out, hrf_stream_t stream);
/* the same sum over the flat-field corrected stack (multispecies :103-105): channels
 * [cal_c0, cal_c1) of pixel p divided by cal[p*cal_sp + c*cal_sc] in f64 first -- numpy's
 * stack / calibration broadcasting for an (H,W) plane (sp 1, sc 0), a (C,) vector (sp 0,
 * sc 1) or a full (H,W,C) array (sp C, sc 1).  C <= 128.  cal NULL: plain sum. */
HRF_API hrf_status hrf_channel_sum_cal(const float *stack, int64_t npix, int32_t C, const float *cal, int64_t cal_sp,
                                       int32_t cal_sc, int32_t cal_c0, int32_t cal_c1, int32_t mode, double *out,
                                       hrf_stream_t stream);
/* np.max(stack, axis=2) as f64 (ecoli :45, the per-laser registration images) */
HRF_API hrf_status hrf_channel_max(const float *stack, int64_t npix, int32_t C, double *out, hrf_stream_t stream);
/* every laser's np.max(stack, axis=2) projection (ecoli :45) in one launch: src / out per laser
 * ((npix x C_l) f32 -> npix f64) */
HRF_API hrf_status hrf_channel_max_multi(const float *const *src_host, const int32_t *channels_host, int32_t nlaser,
                                         int64_t npix, double *const *out_host, hrf_stream_t stream);
/* the same with a workgroup budget (0 = the default 4096): the tile path (hrf_tile_ecoli) runs the
 * projections on 512 workgroups, which leaves room on every CU for concurrent tiles' work */
HRF_API hrf_status hrf_channel_max_multi_grid(const float *const *src_host, const int32_t *channels_host,
                                              int32_t nlaser, int64_t npix, double *const *out_host,
                                              int32_t max_workgroups, hrf_stream_t stream);
/* the calibrated stack as f64, out (npix, C) (multispecies :104 image_channel / :166 _registered.npy) */
HRF_API hrf_status hrf_calibrate_f64(const float *stack, int64_t npix, int32_t C, const float *cal, int64_t cal_sp,
                                     int32_t cal_sc, int32_t cal_c0, int32_t cal_c1, double *out,
                                     hrf_stream_t stream);
/* out = a AND b on u8 masks (multispecies :140, :153) */
HRF_API hrf_status hrf_and_u8(const uint8_t *a, const uint8_t *b, int64_t n, uint8_t *out, hrf_stream_t stream);
/* out = labels where mask, else 0 (multispecies :152 seeds * bkg) */
HRF_API hrf_status hrf_mask_labels(const int32_t *labels, const uint8_t *mask, int64_t n, int32_t *out,
                                   hrf_stream_t stream);
HRF_API hrf_status hrf_max_f64(const double *a, int64_t n, double *max_dev, hrf_stream_t stream);
HRF_API hrf_status hrf_div_scalar_f64(const double *a, int64_t n, const double *divisor_dev, double *out,
                                      hrf_stream_t stream);
/* skimage.util.pad(img, width, mode='edge') (multispecies :109) */
HRF_API hrf_status hrf_pad_edge_f64(const double *a, int64_t H, int64_t W, int32_t width, double *out,
                                    hrf_stream_t stream);
/* skimage.util.pad(a, width, mode='edge') of an (X, Y, Z) volume (biofilm :810) */
HRF_API hrf_status hrf_pad_edge3_f64(const double *a, int64_t X, int64_t Y, int64_t Z, int32_t width, double *out,
                                     hrf_stream_t stream);
HRF_API hrf_status hrf_mask_mul_f64(const double *a, const uint8_t *mask, int64_t n, double *out,
                                    hrf_stream_t stream);

/* ==== f1: registration shifts of a laser set, hand-written f64 FFT pipeline (xcorr.hip) ======
 * register_translation(imgs[0], imgs[t]) for t = 1..nimg-1 (ecoli :45-57, multispecies :82-84)
 * in six launches: rows, column four-step pass A, pass B fused with the conjugate product and its
 * inverse, inverse pass A, inverse rows with the per-row first |cc| maximum, per-target shift.
 * imgs: nimg x H x W f64 (reference first); H a power of two 16..4096, W 4..4096; nimg 2..16.
 * work: hrf_xcorr_workspace_bytes(nimg, H, W) device bytes (-1: size unsupported -- use
 * hrf_register_translations_batch_dev); shifts_dev: nimg x 2 int32, row 0 = (0, 0); clamp >= 0:
 * |component| > clamp -> 0.  Stream-ordered, no synchronisation. */
HRF_API int64_t hrf_xcorr_workspace_bytes(int32_t nimg, int64_t H, int64_t W);
HRF_API hrf_status hrf_xcorr_shifts_dev(const double *imgs, int32_t nimg, int64_t H, int64_t W, void *work,
                                        int32_t clamp, int32_t *shifts_dev, hrf_stream_t stream);
/* the same pipeline writing the correlation surfaces instead of the shifts (tests): cc_out
 * (nimg - 1) x H x W f64 = H * W / 2 * numpy.fft.ifft2(F(ref) conj(F(img_t))).real */
HRF_API hrf_status hrf_xcorr_surfaces_dev(const double *imgs, int32_t nimg, int64_t H, int64_t W, void *work,
                                          double *cc_out, hrf_stream_t stream);

/* ==== f1: registration shift estimate (register.hip) ====================================
 * skimage.feature.register_translation(src, target)[0] (upsample_factor 1; ecoli :45-46,
 * multispecies :82-83): argmax |ifft(F(src) conj(F(target)))| wrapped to (-n/2, n/2] per
 * axis, via hipFFT (f64).  src/target (H, W) f64; work: hrf_register_workspace_bytes(H, W)
 * device bytes; shift_host[2] = (row, col) integer shift.  Synchronises the stream. */
HRF_API int64_t hrf_register_workspace_bytes(int64_t H, int64_t W);
HRF_API hrf_status hrf_register_translation(const double *src, const double *target, int64_t H, int64_t W,
                                            void *work, int32_t *shift_host, hrf_stream_t stream);
/* the same, the (row, col) shift written to DEVICE memory (no synchronisation); clamp >= 0 zeroes
 * a component whose magnitude exceeds it (ecoli :47-57), -1 keeps it.  src == NULL reuses the
 * reference image's transform already in `work` from the previous call on that workspace. */
HRF_API hrf_status hrf_register_translation_dev(const double *src, const double *target, int64_t H, int64_t W,
                                                void *work, int32_t clamp, int32_t *shift_dev, hrf_stream_t stream);
/* every target against the reference in one batch: imgs = nimg contiguous H x W f64 images
 * (reference first, 2 <= nimg <= 64), shifts_dev = nimg x 2 int32 (row 0 = (0, 0)); clamp as
 * hrf_register_translation_dev; work: hrf_register_batch_workspace_bytes(nimg, H, W) bytes */
HRF_API int64_t hrf_register_batch_workspace_bytes(int32_t nimg, int64_t H, int64_t W);
HRF_API hrf_status hrf_register_translations_batch_dev(const double *imgs, int32_t nimg, int64_t H, int64_t W,
                                                       void *work, int32_t clamp, int32_t *shifts_dev,
                                                       hrf_stream_t stream);

/* ==== a4: non-local means (nlmeans.hip) ==================================================
 * skimage.restoration.denoise_nl_means(img, patch_size, patch_distance, h, fast_mode=True,
 * sigma) on a 2-D f64 image (multispecies :108 h=0.02, biofilm :350): reflect padding,
 * out (H, W) f64.  Built for the reference's defaults patch_size 7, patch_distance 11
 * (others -> HRF_EINVAL). */
HRF_API hrf_status hrf_nl_means_2d(const double *img, int64_t H, int64_t W, int32_t patch_size, int32_t patch_distance,
                                   double h, double sigma, double *out, hrf_stream_t stream);

/* ==== a8: 1-D KMeans (kmeans.hip) ======================================================
 * sklearn KMeans(n_clusters=k, random_state=0, n_init).fit_predict(x.reshape(-1, 1)) (ecoli
 * measurement.py:73, :85; multispecies :125, :141; the reference era's n_init = 10), restated
 * from sklearn 1.7.2 with its random stream (numpy RandomState(0)) replayed: k-means++ init,
 * Lloyd with sklearn's stopping rule and empty-cluster relocation, best of n_init by inertia
 * (see oracle/kmeans_sk.c).  Only entries with valid[i] (valid NULL: all) take part, in raster
 * order.  labels (nullable) int32 = sklearn's cluster ids (-1 where not valid); top_mask
 * (nullable) u8 = the cluster chosen by top_rule: 0 the largest centre; 1 (k = 2, multispecies
 * :126-135/:142-149) the larger cluster when both hold a positive value, else cluster 0; 2
 * (k = 2, ecoli :75-84) the larger cluster when both are non-empty, else cluster 0.
 * centers_host[k] / iters_host (nullable) receive sklearn's cluster_centers_ / n_iter_.  NaN
 * input -> HRF_EINVAL (sklearn raises).  work: hrf_kmeans_sorted_workspace_bytes(n) device
 * bytes; reuse_sort != 0: `work` already holds the sort of this very x / valid from a
 * previous call (e.g. k = 2 then k = 3 on ecoli image_cn).  Synchronises the stream once. */
HRF_API int64_t hrf_kmeans_sorted_workspace_bytes(int64_t n);
/* diagnostics: per-run Lloyd iterations, empty-cluster relocations and strict convergence of
 * this thread's last hrf_kmeans_1d_sorted call (n = its n_init) */
HRF_API hrf_status hrf_kmeans_last_runs(int32_t *iters, int32_t *relocations, int32_t *strict, int32_t n);
HRF_API hrf_status hrf_kmeans_1d_sorted(const double *x, const uint8_t *valid, int64_t n, int32_t k, int32_t max_iter,
                                        int32_t n_init, int32_t top_rule, int32_t *labels, uint8_t *top_mask,
                                        double *centers_host, int32_t *iters_host, void *work, int64_t work_bytes,
                                        int32_t reuse_sort, hrf_stream_t stream);
/* Two fits (k1, then k2 reusing the sort) on the same x with ONE host synchronisation: ecoli
 * measurement.py:73-84 (k = 2, rule 2 -> top1) and :85-94 (k = 3, rule 0 -> top2). */
HRF_API hrf_status hrf_kmeans_1d_sorted_pair(const double *x, const uint8_t *valid, int64_t n, int32_t k1, int32_t k2,
                                             int32_t max_iter, int32_t n_init, int32_t rule1, int32_t rule2,
                                             uint8_t *top1, uint8_t *top2, void *work, int64_t work_bytes,
                                             hrf_stream_t stream);
/* the random stream of the fit (host): per run the first centre's rank among the valid samples
 * (numpy RandomState.choice(nv, p=1/nv)) and the k-means++ trial draws, for tests against
 * numpy; draws_host holds n_init * (k - 1) * (2 + int(log k)) doubles */
HRF_API hrf_status hrf_kmeans_draws(int64_t nv, int32_t k, int32_t n_init, int64_t *first_host, double *draws_host);

/* ==== a9/a10/a13: components, morphology, label cleanup (label.hip) ====================
 * img dtype: 0 = uint8 mask, 1 = int32 label image (equal values connect), 2 = uint8 mask
 * inverted.  conn 1 = 4-, 2 = 8-connectivity (skimage label default for 2-D).
 * parent[p] = minimum raster index of p's component, -1 for background. */
HRF_API hrf_status hrf_cc_roots(const void *img, int32_t dtype, int64_t H, int64_t W, int32_t conn, int32_t *parent,
                                hrf_stream_t stream);
/* raster-first numbering 1..N (skimage.measure.label / ndi.label order); blk_ws holds
 * ceil(n/1024)+1 int32; *nlab_dev (device) = N. */
HRF_API hrf_status hrf_cc_number(const int32_t *parent, int64_t n, int32_t *labels, int32_t *blk_ws,
                                 int32_t *nlab_dev, hrf_stream_t stream);
/* skimage.measure.label(img, connectivity=conn) (ecoli :97-98,109,111-112; multispecies :140) */
HRF_API hrf_status hrf_label(const void *img, int32_t dtype, int64_t H, int64_t W, int32_t conn, int32_t *labels,
                             int32_t *parent_ws, int32_t *blk_ws, int32_t *nlab_dev, hrf_stream_t stream);
/* size[root] = component size (size zeroed here; n int32) */
HRF_API hrf_status hrf_cc_sizes(const int32_t *parent, int64_t n, int32_t *size, hrf_stream_t stream);
/* skimage.morphology.remove_small_objects on a bool image (ecoli :96,108; multispecies :137) */
HRF_API hrf_status hrf_remove_small_objects_mask(const uint8_t *mask, int64_t H, int64_t W, int64_t min_size,
                                                 int32_t conn, uint8_t *out, int32_t *parent_ws, int32_t *size_ws,
                                                 hrf_stream_t stream);
/* skimage.morphology.remove_small_holes(ar, area_threshold) (ecoli :95) */
HRF_API hrf_status hrf_remove_small_holes(const uint8_t *mask, int64_t H, int64_t W, int64_t area_threshold,
                                          int32_t conn, uint8_t *out, int32_t *parent_ws, int32_t *size_ws,
                                          hrf_stream_t stream);
/* erosion-seed freeze step (ecoli :102-106): components (conn) of mask with size < thr are
 * OR-ed into small_or, the rest written to large (mask and large may not alias). */
HRF_API hrf_status hrf_split_by_size(const uint8_t *mask, int64_t H, int64_t W, int32_t conn, int64_t thr,
                                     uint8_t *small_or, uint8_t *large, int32_t *parent_ws, int32_t *size_ws,
                                     hrf_stream_t stream);
/* per-label bounding boxes box[(maxlab+1)*4] = {r0, c0, r1, c1} (inclusive; empty: r1 < r0) */
HRF_API hrf_status hrf_label_boxes(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, int32_t *box,
                                   hrf_stream_t stream);
/* the whole erosion-seeding loop (ecoli :97-110) in one launch, one workgroup per
 * 8-connected component (labels 1..ncomp from hrf_label, box from hrf_label_boxes);
 * be_out (H*W u8) = dist_be.  Synchronises once (sizes a scratch slab for big boxes). */
HRF_API hrf_status hrf_erosion_seeds(const int32_t *labels, int64_t H, int64_t W, int32_t ncomp, const int32_t *box,
                                     int32_t area_max, int32_t min_obj, uint8_t *be_out, hrf_stream_t stream);
/* scipy.ndimage.binary_fill_holes (multispecies :138-139); flag_ws n int32 */
HRF_API hrf_status hrf_fill_holes(const uint8_t *mask, int64_t H, int64_t W, uint8_t *out, int32_t *parent_ws,
                                  int32_t *flag_ws, hrf_stream_t stream);
/* skimage.segmentation.clear_border(labels) (ecoli :115, multispecies :156) */
HRF_API hrf_status hrf_clear_border(const int32_t *labels, int64_t H, int64_t W, int32_t *out, int32_t *parent_ws,
                                    int32_t *flag_ws, hrf_stream_t stream);
/* remove_small_objects on an int label image (ecoli :114, multispecies :155); cnt_ws maxlab+1 */
HRF_API hrf_status hrf_remove_small_objects_labels(const int32_t *labels, int64_t n, int32_t maxlab,
                                                   int64_t min_size, int32_t *out, int32_t *cnt_ws,
                                                   hrf_stream_t stream);
/* skimage.segmentation.relabel_sequential(labels)[0] (multispecies :157); map_ws maxlab+1 */
HRF_API hrf_status hrf_relabel_sequential(const int32_t *labels, int64_t n, int32_t maxlab, int32_t *out,
                                          int32_t *map_ws, int32_t *nlab_dev, hrf_stream_t stream);
/* skimage.morphology.binary_erosion / binary_dilation, cross footprint (ecoli :107,:122) */
HRF_API hrf_status hrf_binary_erosion(const uint8_t *mask, int64_t H, int64_t W, int32_t border_value, uint8_t *out,
                                      hrf_stream_t stream);
HRF_API hrf_status hrf_binary_dilation(const uint8_t *mask, int64_t H, int64_t W, uint8_t *out, hrf_stream_t stream);
HRF_API hrf_status hrf_count_nonzero_u8(const uint8_t *mask, int64_t n, int64_t *count_dev, hrf_stream_t stream);
HRF_API hrf_status hrf_max_i32(const int32_t *a, int64_t n, int32_t *max_dev, hrf_stream_t stream);

/* ==== a12: watershed (watershed.hip) =====================================================
 * skimage.morphology.watershed(+/-image, markers, mask) (ecoli :113, multispecies :154),
 * 4-connectivity, including the heap's (value, age) order on equal values.  state_ws:
 * hrf_watershed_workspace_bytes(H, W) device bytes; flag_ws: >= 8 int32.  Synchronises after
 * 8 relaxation passes, then per 4; HRF_EINVAL if not converged within max_passes.
 * ties_host (nullable, 3 int32): pixels whose label needed the exact order, resolution
 * rounds, and decisions between equal-valued markers of different labels (skimage decides
 * those by its binary heap's layout: when there is one, the tile is flooded again by
 * hrf_watershed_heap's kernel and its labels are returned) -- see DESIGN.md "Watershed".
 * hrf_watershed_heap: skimage's heap flood itself, run by one workgroup (serial; exact on any
 * input, slow on large images -- the tie path of hrf_watershed_ex, exported for tests). */
HRF_API int64_t hrf_watershed_workspace_bytes(int64_t H, int64_t W);
HRF_API hrf_status hrf_watershed(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask,
                                 int64_t H, int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws,
                                 int32_t max_passes, int32_t *passes_host, hrf_stream_t stream);
HRF_API hrf_status hrf_watershed_ex(const double *image, int32_t negate, const int32_t *markers, const uint8_t *mask,
                                    int64_t H, int64_t W, int32_t *out_labels, void *state_ws, int32_t *flag_ws,
                                    int32_t max_passes, int32_t *passes_host, int32_t *ties_host,
                                    hrf_stream_t stream);
HRF_API hrf_status hrf_watershed_heap(const double *image, int32_t negate, const int32_t *markers,
                                      const uint8_t *mask, int64_t H, int64_t W, int32_t *out_labels,
                                      hrf_stream_t stream);

/* ==== native segmentation drivers (segment.hip) ==========================================
 * One call runs a whole segmentation chain -- the same library calls, in the same order, as
 * pipeline.segment_ecoli / segment_multispecies -- with device buffers owned by a context
 * sized for one H x W tile (create once per tile size and per concurrently used stream; a
 * context serves one call at a time).  Outputs are caller-owned device buffers. */
typedef struct hrf_seg_ctx hrf_seg_ctx;
HRF_API hrf_status hrf_seg_ctx_create(int64_t H, int64_t W, hrf_seg_ctx **out);
HRF_API hrf_status hrf_seg_ctx_destroy(hrf_seg_ctx *ctx);
/* the context's last chain, its watershed: out[4] = passes, contested pixels, resolution
 * rounds, equal-valued-marker decisions (hrf_watershed_ex ties_host) */
HRF_API hrf_status hrf_seg_ctx_stats(const hrf_seg_ctx *ctx, int32_t *out);
/* ecoli measurement.py:44-127: seg_out (H*W int32, labels not re-sequenced), *maxlab_host */
HRF_API hrf_status hrf_segment_ecoli(hrf_seg_ctx *ctx, const float *stack, int32_t C, int32_t *seg_out,
                                     int32_t *maxlab_host, hrf_stream_t stream);
/* the same chain from a precomputed image_cn = log(sum + 1e-2) (H x W f64, e.g. written by
 * hrf_register_assemble_cn_dev) */
HRF_API hrf_status hrf_segment_ecoli_cn(hrf_seg_ctx *ctx, const double *image_cn, int32_t *seg_out,
                                        int32_t *maxlab_host, hrf_stream_t stream);
/* multispecies measurement.py:102-157 (calibration as hrf_channel_sum_cal, cal may be NULL):
 * seg_out relabelled 1..*nlab_host; image_sum_out / final_bkg_out (nullable, H*W f64) receive
 * the calibrated channel sum (:105) and the background-filtered enhanced image (:150). */
HRF_API hrf_status hrf_segment_multispecies(hrf_seg_ctx *ctx, const float *stack, int32_t C, const float *cal,
                                            int64_t cal_sp, int32_t cal_sc, int32_t cal_c0, int32_t cal_c1,
                                            int32_t *seg_out, int32_t *nlab_host, double *image_sum_out,
                                            double *final_bkg_out, hrf_stream_t stream);

/* ==== one E. coli tile in one call (tile.hip) ============================================
 * ecoli measurement.py:44-162 (-c T) + image_classification.py:43-71 + collect :92-98:
 * registration (channel-max projections, xcorr shifts, assembly writing image_cn and the pixel
 * table), the per-pixel classifier on side_stream (nullable: the same stream; pix_start/pix_end,
 * nullable, recorded around it there), the segmentation chain, flat-fielded label sums read from
 * the lasers (cal: H x W f32 on channels 0-31, nullable), cell table, presence flags (variant 1/2:
 * lib_flags R x 5 f64 = the library's), per-cell classification, counts (R int64), identification
 * map.  Caller buffers: seg, ident (H*W int32), pixel_idx/pixel_dist (H*W, per_pixel only), the
 * per-cell rows labels (cell_cap int32), avgint / avgint_norm (cell_cap x 95 f64), cell_idx
 * (int32) / cell_dist (f64); ncells_dev (device int32) receives the row count, *maxlab_host the
 * segmentation's maximum label.  When *maxlab_host > cell_cap the per-cell part is not run:
 * call hrf_tile_ecoli_cells with buffers of at least *maxlab_host rows.  lasers_host: the five
 * (H, W, 32/23/20/14/6) f32 acquisitions; H, W powers of two.  Stream-ordered after the
 * segmentation's two synchronisations; side_stream is joined before return. */
typedef struct hrf_tile_ctx hrf_tile_ctx;
HRF_API hrf_status hrf_tile_ctx_create(int64_t H, int64_t W, hrf_tile_ctx **out);
HRF_API hrf_status hrf_tile_ctx_destroy(hrf_tile_ctx *ctx);
/* the segmentation context the tile context runs (hrf_seg_ctx_stats of the last tile) */
HRF_API hrf_status hrf_tile_ctx_seg(hrf_tile_ctx *ctx, hrf_seg_ctx **seg);
/* pixels of the last tile the per-pixel certificate did not settle (scored in full by the refine's
 * list pass); synchronises with the device */
HRF_API hrf_status hrf_tile_ctx_pixel_listed(hrf_tile_ctx *ctx, int32_t *n_host);
HRF_API hrf_status hrf_tile_ecoli(hrf_tile_ctx *ctx, const float *const *lasers_host, const float *cal,
                                  const void *refx, const double *lib, const double *lib_flags, int32_t R,
                                  int32_t variant, double flag_thr, int32_t per_pixel, int32_t *seg,
                                  int32_t *pixel_idx, float *pixel_dist, int32_t cell_cap, int32_t *labels,
                                  double *avgint, double *avgint_norm, int32_t *cell_idx, double *cell_dist,
                                  int32_t *ident, int64_t *counts, int32_t *ncells_dev, int32_t *maxlab_host,
                                  hrf_stream_t stream, hrf_stream_t side_stream, hrf_event_t pix_start,
                                  hrf_event_t pix_end);
HRF_API hrf_status hrf_tile_ecoli_cells(hrf_tile_ctx *ctx, const int32_t *seg, const double *lib,
                                        const double *lib_flags, int32_t R, int32_t variant, double flag_thr,
                                        int32_t cell_cap, int32_t *labels, double *avgint, double *avgint_norm,
                                        int32_t *cell_idx, double *cell_dist, int32_t *ident, int64_t *counts,
                                        int32_t *ncells_dev, hrf_stream_t stream);

/* ==== a14-a16, a20, a21, a23: per-label reductions (stats.hip) ==========================
 * regionprops(seg, intensity_image=stack[:,:,k]).mean_intensity for all k in ONE pass
 * (ecoli :151-155, multispecies :167-171): sums[(maxlab+1)*C] f64, counts[maxlab+1];
 * cal (nullable, (H*W) f32) divides channels [cal_c0, cal_c1) (flat field, ecoli :147-150). */
HRF_API hrf_status hrf_label_sums(const float *stack, const int32_t *labels, int64_t npix, int32_t C, int32_t maxlab,
                                  const float *cal, int32_t cal_c0, int32_t cal_c1, double *sums, int64_t *counts,
                                  hrf_stream_t stream);
/* the same with a strided calibration: channels [c0, c1) of pixel p divided by
 * cal[p*cal_sp + c*cal_sc] (plane: sp 1, sc 0; per channel: sp 0, sc 1; full: sp C, sc 1) */
HRF_API hrf_status hrf_label_sums_cal(const float *stack, const int32_t *labels, int64_t npix, int32_t C,
                                      int32_t maxlab, const float *cal, int64_t cal_sp, int32_t cal_sc, int32_t cal_c0,
                                      int32_t cal_c1, double *sums, int64_t *counts, hrf_stream_t stream);
/* rows = present labels ascending (regionprops order); avgint = sums/counts,
 * avgint_norm = avgint / rowmax (ecoli :157, classify_spectra.py:27). */
HRF_API hrf_status hrf_cell_table(const double *sums, const int64_t *counts, int32_t maxlab, int32_t C,
                                  int32_t max_rows, int32_t *row_of_label, int32_t *label_of_row, double *avgint,
                                  double *avgint_norm, int32_t *nrows_dev, hrf_stream_t stream);
/* exact raw moments mom[(maxlab+1)*6] = {area, sum r, sum c, sum r^2, sum c^2, sum rc} */
HRF_API hrf_status hrf_region_moments(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, int64_t *mom,
                                      hrf_stream_t stream);
/* regionprops area, centroid, major/minor axis, eccentricity, orientation
 * (classify_spectra.py:38-46): props[(maxlab+1)*8] */
HRF_API hrf_status hrf_region_props(const int64_t *mom, int32_t maxlab, double *props, hrf_stream_t stream);
/* E. coli per-cell filter (ecoli measurement.py:116-126): cells with minor axis in
 * [minor_lo, minor_hi] keep their 2x-cross-eroded interior, others vanish. */
HRF_API hrf_status hrf_shape_filter(const int32_t *labels, int64_t H, int64_t W, const double *props, int32_t maxlab,
                                    double minor_lo, double minor_hi, int32_t *out, hrf_stream_t stream);
/* per-barcode counts (collect_measurement_results.py:92-98) */
HRF_API hrf_status hrf_barcode_counts(const int32_t *bc, int64_t n, int32_t R, int64_t *counts, hrf_stream_t stream);
/* identification image (image_classification.py:65-71): label L in 1..ncell -> code[L-1] */
HRF_API hrf_status hrf_paint_ids(const int32_t *labels, int64_t n, const int32_t *code, int32_t ncell, int32_t *out,
                                 hrf_stream_t stream);

/* ==== a19: segmented-cosine classification (classify.hip) ===============================
 * train_reference.py:223-386 (channel_cosine_intensity), :993-1072 (_7b_v2).
 * bounds_host: nseg+1 channel offsets on the HOST (e.g. 0,32,55,75,89,95). */
/* mode 0: f32 MFMA (v_mfma_f32_32x32x2_f32); mode 1: split-fp16 MFMA (hi/lo' fp16 operands,
 * ~2^-22 relative per product, 16x-rate v_mfma_f32_32x32x16_f16).  kp/rpad: prepared-table
 * geometry (mode 0: rpad x kp f32; mode 1: rpad x 2*kp fp16). */
HRF_API hrf_status hrf_classify_geometry(int32_t C, int32_t nseg, int32_t R, int32_t mode, int32_t *kp_host,
                                         int32_t *rpad_host);
/* segment-normalised references + zero-segment indicator columns, padded */
/* bytes per row of the prepared table of `mode` (mode 0: f32 [kp]; 1/2: fp16 hi | lo | pad, the
 * pad 16 B, or 32 B for mode 2 on the E. coli layout) */
HRF_API hrf_status hrf_classify_table_row_bytes(int32_t C, const int32_t *bounds_host, int32_t nseg, int32_t mode,
                                                int32_t *row_bytes_host);
HRF_API hrf_status hrf_classify_prepare_refs(const float *ref, int32_t R, int32_t C, const int32_t *bounds_host,
                                             int32_t nseg, int32_t mode, void *refx, hrf_stream_t stream);
/* bytes of the prepared library of `mode` for R rows: the MFMA table (rpad rows of
 * hrf_classify_table_row_bytes) followed by the exact section the refine reads (the f32 library
 * row- and channel-major, its f64 segment sums of squares, the all-zero pixel's answer) */
HRF_API int64_t hrf_classify_refx_bytes(int32_t C, const int32_t *bounds_host, int32_t nseg, int32_t R, int32_t mode);
/* per pixel (north_star mode), exact: best_idx[p] = the restatement's argmin_r of the ungated
 * segmented-cosine distance (oracle_segcos variant 0 in f64 on the f32 values; lowest r on ties),
 * best_dist[p] = that distance rounded to f32.  = hrf_classify_pixels_screen + hrf_classify_pixels_refine
 * on the stack (workspace allocated stream-ordered). */
HRF_API hrf_status hrf_classify_pixels(const float *stack, int64_t P, int32_t C, const void *refx, int32_t R,
                                       const int32_t *bounds_host, int32_t nseg, int32_t mode, int32_t *best_idx,
                                       float *best_dist, hrf_stream_t stream);
/* the MFMA screen alone: best_idx = the device argmax of the split-fp16 (mode 1/2) or f32 (mode 0)
 * scores (lowest row on equal device scores), best_dist = its device distance, second[p]
 * (nullable) = an upper bound on the device score of every other library row */
HRF_API hrf_status hrf_classify_pixels_screen(const float *stack, int64_t P, int32_t C, const void *refx, int32_t R,
                                              const int32_t *bounds_host, int32_t nseg, int32_t mode,
                                              int32_t *best_idx, float *best_dist, float *second,
                                              hrf_stream_t stream);
/* the f64 refine of a screen's output, in place: certify the screen's row by its exact distance
 * against the screen's proven error bound, else score every row (f32 with its own bound, f64 on the
 * survivors).  The pixels' f32 values come from nlaser acquisitions (a plain (P, C) stack: nlaser 1,
 * channels {C}, shifts NULL, H*W = P): pixel p = (p / W, p % W) reads laser q at its device shift
 * (shifts_dev: nlaser (dr, dc) pairs, or NULL), 0 outside its frame and, with apply_mask, outside
 * any laser's frame (hrf_register_assemble's stack).  screen: the sweep that produced second
 * (0/1/2: hrf_classify_pixels_screen mode 0/1/2, 3: hrf_classify_pixels_table); refx prepared for
 * that mode (3: mode 2).  work: hrf_classify_refine_work_bytes(H*W) device bytes; its first int32
 * is the number of pixels the certificate did not settle (readable after the stream syncs). */
HRF_API int64_t hrf_classify_refine_work_bytes(int64_t P);
/* the refine's error bounds for `screen`, in score units (score = nseg (1 - distance)):
 * eps_host[0] = the screen's bound for a pixel with no all-zero segment, [1] = the increment per
 * all-zero segment of the pixel, [2] = the list pass's f32 bound */
HRF_API hrf_status hrf_classify_screen_eps(int32_t C, const int32_t *bounds_host, int32_t nseg, int32_t R,
                                           int32_t screen, double *eps_host);
HRF_API hrf_status hrf_classify_pixels_refine(const float *const *src_host, const int32_t *channels_host,
                                              const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                              int32_t apply_mask, const void *refx, int32_t R,
                                              const int32_t *bounds_host, int32_t nseg, int32_t screen,
                                              const float *second, int32_t *best_idx, float *best_dist, void *work,
                                              int64_t work_bytes, hrf_stream_t stream);
/* the per-pixel classifier's operands prepared once (pixtable.hpp): the split-fp16,
 * segment-normalised pixels in the MFMA register layout (table: hrf_pixtable_bytes(P, ...) device
 * bytes) and a flag byte per pixel (flags: P bytes).  Mode-2 layouts (E. coli, multispecies). */
HRF_API int64_t hrf_pixtable_bytes(int64_t P, int32_t C, const int32_t *bounds_host, int32_t nseg);
HRF_API hrf_status hrf_pixtable_prepare(const float *stack, int64_t P, int32_t C, const int32_t *bounds_host,
                                        int32_t nseg, void *table, uint8_t *flags, hrf_stream_t stream);
/* the mode-2 screen (hrf_classify_pixels_screen) from a prepared pixel table: the same device
 * scores bit for bit; second nullable.  Exact results: hrf_classify_pixels_refine (screen 3). */
HRF_API hrf_status hrf_classify_pixels_table(const void *table, const uint8_t *flags, int64_t P, int32_t C,
                                             const void *refx, int32_t R, const int32_t *bounds_host, int32_t nseg,
                                             int32_t *best_idx, float *best_dist, float *second,
                                             hrf_stream_t stream);
/* hrf_classify_pixels_table + hrf_classify_pixels_refine (screen 3): the table sweep with its
 * runner-up bounds (held in `work`), the certificate pass, the list pass.  Pixel source and work as
 * hrf_classify_pixels_refine; exact results.  _fused: the sweep certifies its own rows (the f64
 * refine in the sweep's workgroups), then the list pass -- the same results bit for bit (slower
 * beside concurrent tiles: DESIGN.md). */
HRF_API hrf_status hrf_classify_pixels_table_exact(const void *table, const uint8_t *flags,
                                                   const float *const *src_host, const int32_t *channels_host,
                                                   const int32_t *shifts_dev, int32_t nlaser, int64_t H, int64_t W,
                                                   int32_t apply_mask, const void *refx, int32_t R,
                                                   const int32_t *bounds_host, int32_t nseg, int32_t *best_idx,
                                                   float *best_dist, void *work, int64_t work_bytes,
                                                   hrf_stream_t stream);
HRF_API hrf_status hrf_classify_pixels_table_exact_fused(const void *table, const uint8_t *flags,
                                                         const float *const *src_host, const int32_t *channels_host,
                                                         const int32_t *shifts_dev, int32_t nlaser, int64_t H,
                                                         int64_t W, int32_t apply_mask, const void *refx, int32_t R,
                                                         const int32_t *bounds_host, int32_t nseg, int32_t *best_idx,
                                                         float *best_dist, void *work, int64_t work_bytes,
                                                         hrf_stream_t stream);
/* one v_mfma_f32_16x16x32_f16 (shape 0: A 16x32, B 32x16, C/D 16x16 per tile) or
 * v_mfma_f32_32x32x16_f16 (shape 1: A 32x16, B 16x32, C/D 32x32) per tile, all row-major (A, B
 * fp16; C, D f32): pins the accumulation model the per-pixel screen's error bound assumes */
HRF_API hrf_status hrf_probe_mfma_f16(int32_t shape, const void *a, const void *b, const float *c, float *d,
                                      int32_t ntiles, hrf_stream_t stream);
/* presence flags of the gated variants on the library path (no classifier bundle): out (N x nseg)
 * f64, 1.0 where max(x[n, bounds[s]:bounds[s+1]]) > thr, else 0.0 (a NaN in the segment: 0.0) */
HRF_API hrf_status hrf_segment_flags(const double *x, int64_t N, int32_t C, const int32_t *bounds_host, int32_t nseg,
                                     double thr, double *out, hrf_stream_t stream);
/* per cell (f64): variant 0 ungated, 1 channel_cosine_intensity, 2 _7b_v2; fx (N x nseg),
 * fr (R x nseg) presence flags (needed for variants 1, 2) */
HRF_API hrf_status hrf_classify_cells(const double *x, int64_t N, const double *ref, int32_t R, int32_t C,
                                      const int32_t *bounds_host, int32_t nseg, int32_t variant, const double *fx,
                                      const double *fr, int32_t *arg, double *dmin, hrf_stream_t stream);

/* ==== a17, a18, f2: classifier back-end (backend.hip) ======================================
 * ecoli image_classification.py:43-56, synthetic-community classify_spectra.py:27-35.  Models
 * arrive as arrays (never pickles).  All f64. */
/* E. coli features out (n x 132) = avgint_norm (n x 95) | np.diff(avgint_norm[:, 0:32]) | 0 x 6
 * (the six check-SVC flag columns, filled by hrf_svc_predict) (:47-48) */
HRF_API hrf_status hrf_features_ecoli(const double *avgint_norm, int64_t n, double *out, hrf_stream_t stream);
/* community features out (n x 67) = avgint_norm (n x 63) | 0 x 4 (classify_spectra.py:27-28) */
HRF_API hrf_status hrf_features_multi(const double *avgint_norm, int64_t n, double *out, hrf_stream_t stream);
/* sklearn StandardScaler.transform: out (n x f) = (x - mean) / scale (either may be NULL) */
HRF_API hrf_status hrf_standard_scale(const double *x, int64_t n, int32_t f, int64_t ldx, const double *mean,
                                      const double *scale, double *out, hrf_stream_t stream);
/* sklearn SVC.predict (libsvm one-vs-one voting; kernel 0 linear, 1 poly, 2 rbf, 3 sigmoid).
 * sv (nsv x f); coef (n_class-1 x nsv) and intercept (n_class(n_class-1)/2) in libsvm's sign
 * convention (pair (a, b) votes a when its sum > 0: sklearn's dual_coef_ / intercept_ for
 * multi-class, both negated for two classes); start (n_class+1) first support vector per class.
 * pred[i] = class index; dec (n x pairs) optional; val_out[i*val_stride] = class_values[pred]
 * (or the index) when val_out is given -- e.g. a flag column of the feature table. */
HRF_API hrf_status hrf_svc_predict(const double *x, int64_t n, int64_t ldx, int32_t f, const double *sv, int32_t nsv,
                                   const double *coef, const double *intercept, const int32_t *start,
                                   int32_t n_class, int32_t kernel, double gamma, double coef0, int32_t degree,
                                   int32_t *pred, double *dec, double *val_out, int64_t val_stride,
                                   const double *class_values, hrf_stream_t stream);
/* sklearn SVC.predict_proba (probability=True; libsvm svm_predict_probability): Platt sigmoids
 * of the pair decision values with probA / probB (sklearn probA_ / probB_, n_pairs each), then
 * libsvm's multiclass_probability coupling.  prob (n x n_class) in class order; n_class <= 128
 * (biofilm_analysis.py:1229) */
HRF_API hrf_status hrf_svc_predict_proba(const double *x, int64_t n, int64_t ldx, int32_t f, const double *sv,
                                         int32_t nsv, const double *coef, const double *intercept,
                                         const int32_t *start, int32_t n_class, int32_t kernel, double gamma,
                                         double coef0, int32_t degree, const double *probA, const double *probB,
                                         double *prob, hrf_stream_t stream);
/* exact k nearest training rows (trainT: f x nt, feature-major) under metric 0 euclidean, 1
 * channel_cosine_intensity_7b_v2 (train_reference.py:993-1072), 2 the scalar of
 * channel_cosine_intensity_violet_derivative_v2 (:569-731); ascending distance, ties to the
 * lower row.  idx/dist (nq x k) */
HRF_API hrf_status hrf_knn(const double *q, int64_t nq, int64_t ldq, const double *trainT, int64_t nt, int32_t f,
                           int32_t metric, int32_t k, int32_t *idx_out, double *dist_out, hrf_stream_t stream);
/* umap-learn transform's initial embedding from the kNN (umap_.py transform, 0.4 era):
 * smooth_knn_dist, membership strengths (float32), l1 rows, init_transform (float32).
 * mean_dist_dev: the mean of all knn distances (device scalar); embedding (ntrain x d) float32;
 * memb_out (nq x k, optional): the membership strengths in knn order (0 for missing rows), the
 * graph hrf_umap_refine optimises; out (nq x d) float32 */
HRF_API hrf_status hrf_umap_init_transform(const int32_t *knn_idx, const double *knn_dist, int64_t nq, int32_t k,
                                           double n_neighbors, double local_connectivity,
                                           const double *mean_dist_dev, const float *embedding, int32_t d,
                                           float *memb_out, float *out, hrf_stream_t stream);
/* transform()'s layout refinement (optimize_layout_euclidean, training embedding fixed): edges
 * below wmax/n_epochs dropped (wmax = max of memb, device scalar), alpha initial_alpha (pass
 * umap's _initial_alpha / 4), negative samples from per-query Tausworthe streams seeded by
 * (seed, query) -- deterministic, unlike the reference's unseeded shared stream.  embedding
 * (nq x d, float32) in/out, d <= 8 */
HRF_API hrf_status hrf_umap_refine(const int32_t *knn_idx, const float *memb, int64_t nq, int32_t k,
                                   const float *wmax_dev, int32_t n_epochs, const float *tail_embedding, int64_t ntrain,
                                   int32_t d, double a, double b, double repulsion_strength, double initial_alpha,
                                   double negative_sample_rate, uint64_t seed, float *embedding, hrf_stream_t stream);

/* ==== a22: label adjacency (rag.hip) ====================================================
 * skimage.future.graph.rag_boundary edge set (biofilm :1277-1278): edge[(maxlab+1)^2] u8,
 * edge[a*(maxlab+1)+b] = 1 for a < b. */
HRF_API hrf_status hrf_rag_edges(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, uint8_t *edge,
                                 hrf_stream_t stream);
/* barcode x barcode adjacency counts (biofilm :1283-1292): adj[R*R] int64 */
HRF_API hrf_status hrf_barcode_adjacency(const uint8_t *edge, int32_t maxlab, const int32_t *bc_of_label, int32_t R,
                                         int64_t *adj, hrf_stream_t stream);

/* raw and cell-filtered barcode adjacency in one pass (biofilm :1283-1295): adj_filtered counts
 * an edge only when keep_of_label[a] and keep_of_label[b] (the rows typed 'cell') */
HRF_API hrf_status hrf_barcode_adjacency_filtered(const uint8_t *edge, int32_t maxlab, const int32_t *bc_of_label,
                                                  const uint8_t *keep_of_label, int32_t R, int64_t *adj,
                                                  int64_t *adj_filtered, hrf_stream_t stream);
/* out[l] = 1 when label l has a pixel inside mask (debris labels, biofilm :1259-1262);
 * out[maxlab+1] u8 */
HRF_API hrf_status hrf_label_overlap(const int32_t *labels, const uint8_t *mask, int64_t H, int64_t W, int32_t maxlab,
                                     uint8_t *out, hrf_stream_t stream);
/* per cell row: is_cell = !(area > area_max || overlap[label] || maxprob <= prob_min)
 * (biofilm :1263-1269; overlap / maxprob may be NULL) */
HRF_API hrf_status hrf_cell_typing(const int32_t *label, const double *area, const double *maxprob,
                                   const uint8_t *overlap, int32_t maxlab, int64_t n, double area_max, double prob_min,
                                   uint8_t *is_cell, hrf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HRF_H */
