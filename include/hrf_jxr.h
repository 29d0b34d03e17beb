/* hrf_jxr.h -- libhrfjxr.so: JPEG-XR subblock decoding for the native CZI reader (row f3).
 *
 * Replaces the JPEG-XR codec path of bioformats.load_image(filename)
 * (…ecoli/hiprfish_imaging_spectral_image_measurement.py:145, …synthetic-community/
 * hiprfish_imaging_multispecies_spectral_image_measurement.py:81, the biofilm loaders
 * hiprfish_imaging_biofilm_analysis.py:55-120), which hands ZEN's "JpegXrFile" subblocks to a
 * JPEG XR decoder.  Host-side: a shim (csrc/jxr.c) over jxrlib 1.1, the reference implementation
 * of ITU-T T.832, linked from the image's /opt/conda/lib.  Plain pointers and sizes; no device
 * memory.  Returns 0 on success, < 0 on a codec error, -100 for a pixel format that is not grey
 * 8 / 16-bit or 32-bit float. */
#ifndef HRF_JXR_H
#define HRF_JXR_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* size and bytes per pixel of one JPEG XR file held in memory (data, n bytes) */
int hrf_jxr_info(const uint8_t *data, int64_t n, int32_t *width, int32_t *height, int32_t *bytes_per_pixel);
/* decode it into out: height rows of `stride` bytes, samples little endian */
int hrf_jxr_decode(const uint8_t *data, int64_t n, uint8_t *out, int64_t stride);

#ifdef __cplusplus
}
#endif
#endif
