/* jxr.c -- JPEG-XR subblock decoding for the native CZI reader (czi.py; row f3).
 *
 * The reference reads CZI acquisitions through bioformats.load_image
 * (…ecoli/hiprfish_imaging_spectral_image_measurement.py:145, the biofilm z/t/tile loaders
 * :55-120), whose ZeissCZIReader hands JPEG-XR ("JpgXr", compression 4) subblocks to a JPEG-XR
 * codec.  Here the codestream (the JPEG XR file container Zeiss stores per subblock) is decoded
 * by jxrlib 1.1 -- Microsoft's reference implementation of ITU-T T.832, the libjxrglue /
 * libjpegxr shipped in this image under /opt/conda/lib -- through this host-side shim, built
 * into libhrfjxr.so by _build.py when the jxrlib headers are present.  Grey 8- and 16-bit and
 * 32-bit float pixel formats (the Gray8 / Gray16 / Gray32Float CZI pixel types).
 *
 * hrf_jxr_info(data, n, &w, &h, &bytes_per_pixel) and hrf_jxr_decode(data, n, out, stride):
 * 0 on success, < 0 on a codec error, -100 for a pixel format that is not grey. */
#include <stdint.h>
#include <string.h>

#include "JXRGlue.h"
#include "../../include/hrf_jxr.h"

#define EXPORT __attribute__((visibility("default")))

static int bytes_of(const PKPixelFormatGUID *pf) {
  if (IsEqualGUID(pf, &GUID_PKPixelFormat8bppGray)) return 1;
  if (IsEqualGUID(pf, &GUID_PKPixelFormat16bppGray)) return 2;
  if (IsEqualGUID(pf, &GUID_PKPixelFormat32bppGrayFloat)) return 4;
  return -100;
}

/* decoder over an in-memory codestream; the caller releases stream and decoder */
static int open_decoder(const uint8_t *data, size_t n, PKFactory **fac, struct WMPStream **st, PKImageDecode **dec) {
  *fac = NULL;
  *st = NULL;
  *dec = NULL;
  if (PKCreateFactory(fac, PK_SDK_VERSION) < 0) return -1;
  if ((*fac)->CreateStreamFromMemory(st, (void *)data, n) < 0) return -2;
  if (PKImageDecode_Create_WMP(dec) < 0) return -3;
  if ((*dec)->Initialize(*dec, *st) < 0) return -4;
  (*dec)->fStreamOwner = 0;
  return 0;
}

static void close_decoder(PKFactory *fac, struct WMPStream *st, PKImageDecode *dec) {
  if (dec) dec->Release(&dec);
  if (st) st->Close(&st);
  if (fac) fac->Release(&fac);
}

EXPORT int hrf_jxr_info(const uint8_t *data, int64_t n, int32_t *w, int32_t *h, int32_t *bpp) {
  PKFactory *fac;
  struct WMPStream *st;
  PKImageDecode *dec;
  int r = open_decoder(data, (size_t)n, &fac, &st, &dec);
  if (r == 0) {
    PKPixelFormatGUID pf;
    I32 iw = 0, ih = 0;
    if (dec->GetPixelFormat(dec, &pf) < 0 || dec->GetSize(dec, &iw, &ih) < 0) r = -5;
    else {
      *w = iw;
      *h = ih;
      *bpp = bytes_of(&pf);
      if (*bpp < 0) r = *bpp;
    }
  }
  close_decoder(fac, st, dec);
  return r;
}

EXPORT int hrf_jxr_decode(const uint8_t *data, int64_t n, uint8_t *out, int64_t stride) {
  PKFactory *fac;
  struct WMPStream *st;
  PKImageDecode *dec;
  int r = open_decoder(data, (size_t)n, &fac, &st, &dec);
  if (r == 0) {
    PKPixelFormatGUID pf;
    I32 iw = 0, ih = 0;
    if (dec->GetPixelFormat(dec, &pf) < 0 || dec->GetSize(dec, &iw, &ih) < 0) r = -5;
    else if (bytes_of(&pf) < 0) r = -100;
    else {
      PKRect rc = {0, 0, iw, ih};
      if (dec->Copy(dec, &rc, out, (U32)stride) < 0) r = -6;
    }
  }
  close_decoder(fac, st, dec);
  return r;
}
