// segment.hip -- native drivers for the two segmentation chains.
//
// The E. coli chain (ecoli measurement.py:44-127) and the synthetic-community chain
// (multispecies measurement.py:102-157) are ~25-30 library calls each, a few of which
// synchronise (KMeans centres, component counts, watershed convergence).  Composed from
// Python, every call pays the interpreter and allocator, and two host threads driving
// concurrent tiles serialise on the GIL.  These drivers run the same calls from C++ with a
// per-context set of device buffers allocated once for the tile size, so one foreign call
// (ctypes drops the GIL for it) does a whole chain.  The composition is the one in
// pipeline.py, step for step; tests check the two give identical label maps.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"

struct hrf_seg_ctx {
  int64_t H = 0, W = 0, n = 0;
  int device = 0;
  // f64 images
  double *cn = nullptr, *f1 = nullptr, *f2 = nullptr, *f3 = nullptr, *pad = nullptr;
  double *scal = nullptr;  // device scalar (max)
  // u8 masks
  uint8_t *m[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  // int32 images / scratch
  int32_t *l[4] = {nullptr, nullptr, nullptr, nullptr};
  int32_t *parent = nullptr, *size = nullptr, *blk = nullptr, *dint = nullptr;
  void *ws_state = nullptr;
  int32_t *ws_flag = nullptr;
  int32_t *hpin = nullptr;  // pinned host slots for counts read back at a later synchronisation
  int32_t *hpin_dev = nullptr, *hbox_dev = nullptr;  // their device addresses (hrf::zero_publish)
  void *km = nullptr;
  int64_t km_bytes = 0;
  char *seed_px = nullptr;  // erosion seeding's pixel-kernel scratch
  // the last chain's watershed: passes, contested pixels, resolution rounds, decisions between
  // equal-valued markers of different labels (hrf_watershed_ex ties_host) -- hrf_seg_ctx_stats
  int32_t ws_stats[4] = {0, 0, 0, 0};
  // per-label scratch, grown on demand
  int64_t lab_cap = 0;
  int32_t *box = nullptr, *cnt = nullptr;
  int32_t *hbox = nullptr;  // pinned host copy of box (4 * lab_cap)
  int64_t *mom = nullptr;
  double *props = nullptr;
};

namespace {

template <class T>
hrf_status dalloc(T **p, size_t count) {
  HRF_HIP(hipMalloc((void **)p, sizeof(T) * (count ? count : 1)));
  return HRF_OK;
}

hrf_status ensure_labels(hrf_seg_ctx *c, int64_t maxlab, hipStream_t s) {
  if (maxlab + 1 <= c->lab_cap) return HRF_OK;
  HRF_HIP(hipStreamSynchronize(s));  // buffers of the previous size may still be in use
  hipFree(c->box);
  hipFree(c->cnt);
  hipFree(c->mom);
  hipFree(c->props);
  if (c->hbox) hipHostFree(c->hbox);
  c->hbox = nullptr;
  c->hbox_dev = nullptr;
  int64_t cap = 1024;
  while (cap < maxlab + 1) cap *= 2;
  if (hrf_status r = dalloc(&c->box, 4 * cap)) return r;
  if (hrf_status r = dalloc(&c->cnt, cap)) return r;
  if (hrf_status r = dalloc(&c->mom, 6 * cap)) return r;
  if (hrf_status r = dalloc(&c->props, 8 * cap)) return r;
  if (::hrf::host_alloc_mapped((void **)&c->hbox, sizeof(int32_t) * 4 * cap) != hipSuccess ||
      !(c->hbox_dev = ::hrf::mapped(c->hbox))) {
    if (c->hbox) hipHostFree(c->hbox);
    c->hbox = nullptr;
    c->lab_cap = 0;
    ::hrf::set_error("seg_ctx: pinned host allocation failed");
    return HRF_EHIP;
  }
  // the chain clears cnt and mom at the watershed's synchronisation (capacity-wide); buffers
  // allocated after it are cleared here
  HRF_HIP(hipMemsetAsync(c->cnt, 0, sizeof(int32_t) * cap, s));
  HRF_HIP(hipMemsetAsync(c->mom, 0, sizeof(int64_t) * 6 * cap, s));
  c->lab_cap = cap;
  return HRF_OK;
}

hrf_status read_i32(const int32_t *dev, int32_t *host, hipStream_t s) {
  HRF_HIP(hipMemcpyAsync(host, dev, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HRF_HIP(hipStreamSynchronize(s));
  return HRF_OK;
}

#define HRF_TRY(expr)                   \
  do {                                  \
    if (hrf_status r_ = (expr)) return r_; \
  } while (0)

// skimage.measure.label(mask, connectivity=2) -> labels, count (host)
hrf_status label_conn2(hrf_seg_ctx *c, const uint8_t *mask, int32_t *labels, int32_t *nlab, hipStream_t s) {
  HRF_TRY(hrf_label(mask, 0, c->H, c->W, 2, labels, c->parent, c->blk, c->dint, s));
  return read_i32(c->dint, nlab, s);
}

// skimage.measure.label(mask, connectivity=2) with the count's read-back only enqueued: it
// lands in c->hpin[0] at the caller's next synchronisation (saves one host round trip)
hrf_status label_conn2_deferred(hrf_seg_ctx *c, const uint8_t *mask, int32_t *labels, hipStream_t s) {
  HRF_TRY(hrf_label(mask, 0, c->H, c->W, 2, labels, c->parent, c->blk, c->dint, s));
  HRF_HIP(hipMemcpyAsync(c->hpin, c->dint, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  return HRF_OK;
}

// KMeans(k) top-cluster mask (rule: see hrf.h); `reuse` when the previous call sorted the same x
hrf_status kmeans_top(hrf_seg_ctx *c, const double *x, int k, int rule, int reuse, uint8_t *top, hipStream_t s) {
  return hrf_kmeans_1d_sorted(x, nullptr, c->n, k, 300, 10, rule, nullptr, top, nullptr, nullptr, c->km, c->km_bytes,
                              reuse, s);
}

}  // namespace

extern "C" {

hrf_status hrf_seg_ctx_create(int64_t H, int64_t W, hrf_seg_ctx **out) {
  HRF_REQUIRE(out && H >= 1 && W >= 1 && H * W < ((int64_t)1 << 31), "seg_ctx: bad size");
  hrf_seg_ctx *c = new hrf_seg_ctx();
  c->H = H;
  c->W = W;
  c->n = H * W;
  const size_t n = (size_t)c->n;
  hrf_status r = HRF_OK;
  auto fail = [&](hrf_status st) {
    hrf_seg_ctx_destroy(c);
    return st;
  };
  HRF_HIP(hipGetDevice(&c->device));
  if ((r = dalloc(&c->cn, n)) || (r = dalloc(&c->f1, n)) || (r = dalloc(&c->f2, n)) || (r = dalloc(&c->f3, n)) ||
      (r = dalloc(&c->pad, (size_t)(H + 10) * (W + 10))) || (r = dalloc(&c->scal, 8)))
    return fail(r);
  for (auto &p : c->m)
    if ((r = dalloc(&p, n))) return fail(r);
  for (auto &p : c->l)
    if ((r = dalloc(&p, n))) return fail(r);
  if ((r = dalloc(&c->parent, n)) || (r = dalloc(&c->size, n)) || (r = dalloc(&c->blk, (size_t)::hrf::label_dev_ws_words(c->n))) ||
      (r = dalloc(&c->dint, 16)) || (r = dalloc(&c->ws_flag, 8)))
    return fail(r);
  if ((r = dalloc((char **)&c->ws_state, (size_t)hrf_watershed_workspace_bytes(H, W)))) return fail(r);
  if (::hrf::host_alloc_mapped((void **)&c->hpin, 16 * sizeof(int32_t)) != hipSuccess ||
      !(c->hpin_dev = ::hrf::mapped(c->hpin))) {
    ::hrf::set_error("seg_ctx: pinned host allocation failed");
    return fail(HRF_EHIP);
  }
  c->km_bytes = hrf_kmeans_sorted_workspace_bytes(c->n);
  if (c->km_bytes <= 0) return fail(HRF_EHIP);
  if ((r = dalloc((char **)&c->km, (size_t)c->km_bytes))) return fail(r);
  if ((r = dalloc(&c->seed_px, (size_t)::hrf::seed_px_scratch_bytes()))) return fail(r);

  *out = c;
  return HRF_OK;
}

hrf_status hrf_seg_ctx_destroy(hrf_seg_ctx *c) {
  if (!c) return HRF_OK;
  hipFree(c->cn);
  hipFree(c->f1);
  hipFree(c->f2);
  hipFree(c->f3);
  hipFree(c->pad);
  hipFree(c->scal);
  for (auto p : c->m) hipFree(p);
  for (auto p : c->l) hipFree(p);
  hipFree(c->parent);
  hipFree(c->size);
  hipFree(c->blk);
  hipFree(c->dint);
  hipFree(c->ws_state);
  hipFree(c->ws_flag);
  if (c->hpin) hipHostFree(c->hpin);
  if (c->hbox) hipHostFree(c->hbox);
  hipFree(c->km);
  hipFree(c->seed_px);
  hipFree(c->box);
  hipFree(c->cnt);
  hipFree(c->mom);
  hipFree(c->props);
  delete c;
  return HRF_OK;
}

// ecoli :73-127 from image_cn (f64, H x W).  Clears and host read-backs ride on the chain's two
// synchronisations (components + boxes, watershed batch) as ZeroPub launches; `extra` (the
// native tile's per-label buffers) is cleared at the watershed's.
static hrf_status segment_ecoli_from_cn(hrf_seg_ctx *c, const double *cn, int32_t *seg_out, int32_t *maxlab_host,
                                        hipStream_t s, const ::hrf::ZeroPub *extra) {
  const int64_t H = c->H, W = c->W, n = c->n;
  uint8_t *rough = c->m[0], *interior = c->m[1], *a = c->m[2], *b = c->m[3], *d = c->m[4];
  int32_t *lab1 = c->l[0], *seeds = c->l[1], *ws = c->l[2], *lab3 = c->l[3];
  // :73-94; the NaN check (sklearn raises) is read at the component-count synchronisation below
  HRF_TRY(::hrf::kmeans_1d_sorted_pair_deferred(cn, c->n, 2, 3, 300, 10, 2, 0, rough, interior, c->km, c->km_bytes, s,
                                                nullptr));
  const int32_t *km_err = ::hrf::kmeans_error_flag(c->km, c->n);
  HRF_REQUIRE(km_err, "segment_ecoli: kmeans workspace");
  HRF_TRY(hrf_remove_small_holes(interior, H, W, 64, 1, a, c->parent, c->size, s));   // :95
  HRF_TRY(::hrf::binary_opening(a, H, W, 1, d, s));                                 // erosion, dilation
  HRF_TRY(hrf_remove_small_objects_mask(d, H, W, 50, 1, a, c->parent, c->size, s));  // :96 cell_sm = a
  // :97-110.  Components, their count and their boxes come back in ONE synchronisation: the
  // boxes are computed for every label the current capacity holds (labels above it are
  // ignored by the box kernel) and redone in the rare case the count exceeds it.
  HRF_TRY(::hrf::label_dev(a, H, W, 2, lab1, c->parent, c->blk, c->dint, s));
  HRF_TRY(ensure_labels(c, 1, s));
  int32_t guess = (int32_t)(c->lab_cap - 1);
  HRF_TRY(hrf_label_boxes(lab1, H, W, guess, c->box, s));
  {
    ::hrf::ZeroPub zp;
    HRF_REQUIRE(zp.pub(c->dint, c->hpin_dev + 1, 1) && zp.pub(km_err, c->hpin_dev + 3, 1) &&
                    zp.pub(c->box, c->hbox_dev, 4 * (guess + 1)),
                "segment_ecoli: too many read-backs");
    HRF_TRY(::hrf::zero_publish(zp, s));
  }
  HRF_HIP(hipStreamSynchronize(s));
  HRF_REQUIRE(!c->hpin[3], "kmeans_1d_pair: input contains NaN (sklearn KMeans raises ValueError)");
  const int32_t ncomp = c->hpin[1];
  HRF_REQUIRE(ncomp >= 0, "segment_ecoli: component numbering failed");
  if (ncomp > guess) {
    HRF_TRY(ensure_labels(c, ncomp, s));
    HRF_TRY(hrf_label_boxes(lab1, H, W, ncomp, c->box, s));
    ::hrf::ZeroPub zp;
    HRF_REQUIRE(zp.pub(c->box, c->hbox_dev, 4 * (ncomp + 1)), "segment_ecoli: too many read-backs");
    HRF_TRY(::hrf::zero_publish(zp, s));
    HRF_HIP(hipStreamSynchronize(s));
  }
  // Large-box components go to the run kernel too; how many overflowed it lands in hpin[2]
  // at the watershed's synchronisation, and in that (rare) case the seeds and everything
  // after them are redone with those components in the whole-image loop.
  for (int attempt = 0;; ++attempt) {
    HRF_TRY(::hrf::erosion_seeds_hostbox(lab1, H, W, ncomp, c->box, c->hbox, 600, 10, b, s,
                                         attempt == 0 ? c->dint + 8 : nullptr, c->seed_px));
    HRF_TRY(hrf_remove_small_objects_mask(b, H, W, 10, 2, d, c->parent, c->size, s));  // :111
    HRF_TRY(::hrf::label_dev(d, H, W, 2, seeds, c->parent, c->blk, c->dint, s));  // :111-112
    // read back at the watershed's synchronisation: the seed count, the run kernel's overflow
    // count; cleared there: the per-label counts and moments (capacity-wide) and `extra`
    ::hrf::ZeroPub zp = extra ? *extra : ::hrf::ZeroPub();
    HRF_REQUIRE(zp.pub(c->dint, c->hpin_dev + 0, 1) && (attempt > 0 || zp.pub(c->dint + 8, c->hpin_dev + 2, 1)) &&
                    zp.zero(c->cnt, sizeof(int32_t) * c->lab_cap) && zp.zero(c->mom, sizeof(int64_t) * 6 * c->lab_cap),
                "segment_ecoli: too many read-backs");
    HRF_TRY(::hrf::watershed_ex_extra(cn, 1, seeds, rough, H, W, ws, c->ws_state, c->ws_flag, 100000, c->ws_stats,
                                      c->ws_stats + 1, s, &zp));  // :113
    if (attempt > 0 || c->hpin[2] == 0) break;
  }
  const int32_t nseeds = c->hpin[0];  // read back by the watershed's synchronisation
  HRF_REQUIRE(nseeds >= 0, "segment_ecoli: seed numbering failed");
  HRF_TRY(ensure_labels(c, nseeds, s));
  HRF_TRY(::hrf::remove_small_objects_labels_zeroed(ws, n, nseeds, 100, lab1, c->cnt, s));    // :114
  HRF_TRY(hrf_clear_border(lab1, H, W, lab3, c->parent, c->size, s));          // :115
  HRF_TRY(::hrf::region_moments_zeroed(lab3, H, W, nseeds, c->mom, s));         // :116
  // the props pass + shape filter (:116-126; the filter straight from the moments -- one launch
  // less, every labelled pixel recomputing its label's eigenvalues -- lost, removed in round 5)
  HRF_TRY(hrf_region_props(c->mom, nseeds, c->props, s));
  HRF_TRY(hrf_shape_filter(lab3, H, W, c->props, nseeds, 15.0, 35.0, seg_out, s));
  *maxlab_host = nseeds;
  return HRF_OK;
}

hrf_status hrf_seg_ctx_stats(const hrf_seg_ctx *c, int32_t *out) {
  HRF_REQUIRE(c && out, "seg_ctx_stats: bad arguments");
  for (int i = 0; i < 4; ++i) out[i] = c->ws_stats[i];
  return HRF_OK;
}

hrf_status hrf_segment_ecoli(hrf_seg_ctx *c, const float *stack, int32_t C, int32_t *seg_out, int32_t *maxlab_host,
                             hrf_stream_t stream) {
  HRF_REQUIRE(c && stack && seg_out && maxlab_host && C >= 1, "segment_ecoli: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  HRF_TRY(hrf_channel_sum(stack, c->n, C, nullptr, 1, 0, c->cn, s));            // :71-72
  return segment_ecoli_from_cn(c, c->cn, seg_out, maxlab_host, s, nullptr);
}

hrf_status hrf_segment_ecoli_cn(hrf_seg_ctx *c, const double *image_cn, int32_t *seg_out, int32_t *maxlab_host,
                                hrf_stream_t stream) {
  HRF_REQUIRE(c && image_cn && seg_out && maxlab_host, "segment_ecoli_cn: bad arguments");
  return segment_ecoli_from_cn(c, image_cn, seg_out, maxlab_host, (hipStream_t)stream, nullptr);
}

}  // extern "C"

// the native tile's entry: hrf_segment_ecoli_cn with the tile's per-label buffers cleared at the
// watershed's synchronisation
hrf_status hrf::segment_ecoli_cn_extra(hrf_seg_ctx *c, const double *image_cn, int32_t *seg_out,
                                       int32_t *maxlab_host, hipStream_t s, const ZeroPub *extra) {
  HRF_REQUIRE(c && image_cn && seg_out && maxlab_host, "segment_ecoli_cn: bad arguments");
  return segment_ecoli_from_cn(c, image_cn, seg_out, maxlab_host, s, extra);
}

extern "C" {

hrf_status hrf_segment_multispecies(hrf_seg_ctx *c, const float *stack, int32_t C, const float *cal, int64_t cal_sp,
                                    int32_t cal_sc, int32_t cal_c0, int32_t cal_c1, int32_t *seg_out,
                                    int32_t *nlab_host, double *image_sum_out, double *final_bkg_out,
                                    hrf_stream_t stream) {
  HRF_REQUIRE(c && stack && seg_out && nlab_host && C >= 1, "segment_multispecies: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const int64_t H = c->H, W = c->W, n = c->n;
  uint8_t *rough = c->m[0], *bkg = c->m[1], *a = c->m[2], *b = c->m[3], *d = c->m[4], *e = c->m[5];
  int32_t *seeds = c->l[0], *seeds_b = c->l[1], *ws = c->l[2], *lab3 = c->l[3];
  // sum: out or cn; norm: f3; nl: f1; final: f2; final_bkg: out or cn (sum is dead by then)
  double *sum = image_sum_out ? image_sum_out : c->cn;
  double *norm = c->f3, *nl = c->f1, *fin = c->f2;
  HRF_TRY(hrf_channel_sum_cal(stack, n, C, cal, cal_sp, cal_sc, cal_c0, cal_c1, 0, sum, s));   // :104-105
  HRF_TRY(hrf_max_f64(sum, n, c->scal, s));                                     // :106
  HRF_TRY(hrf_div_scalar_f64(sum, n, c->scal, norm, s));
  HRF_TRY(hrf_nl_means_2d(norm, H, W, 7, 11, 0.02, 0.0, nl, s));               // :108
  HRF_TRY(hrf_pad_edge_f64(nl, H, W, 5, c->pad, s));                            // :109
  HRF_TRY(hrf_enhance_2d(c->pad, H + 10, W + 10, W + 10, 11, 9, fin, s));      // :110-124
  HRF_TRY(kmeans_top(c, fin, 2, 1, 0, rough, s));                               // :125-135
  HRF_TRY(::hrf::binary_opening(rough, H, W, 1, b, s));                          // :136 erosion, dilation
  HRF_TRY(hrf_remove_small_objects_mask(b, H, W, 10, 1, a, c->parent, c->size, s));  // :137
  HRF_TRY(hrf_fill_holes(a, H, W, b, c->parent, c->size, s));                  // :138
  HRF_TRY(hrf_fill_holes(rough, H, W, d, c->parent, c->size, s));              // :139
  HRF_TRY(hrf_and_u8(b, d, n, e, s));                                          // :140
  HRF_TRY(label_conn2_deferred(c, e, seeds, s));
  HRF_TRY(kmeans_top(c, nl, 2, 1, 0, bkg, s));                                  // :141-149
  const int32_t nseeds = c->hpin[0];  // read back by the KMeans synchronisation
  double *final_bkg = final_bkg_out ? final_bkg_out : c->cn;
  HRF_TRY(hrf_mask_mul_f64(fin, bkg, n, final_bkg, s));                         // :150
  HRF_TRY(hrf_mask_labels(seeds, bkg, n, seeds_b, s));                          // :152
  HRF_TRY(hrf_and_u8(rough, bkg, n, a, s));                                     // :153
  HRF_TRY(hrf_watershed_ex(final_bkg, 1, seeds_b, a, H, W, ws, c->ws_state, c->ws_flag, 100000, c->ws_stats,
                           c->ws_stats + 1, s));  // :154
  HRF_TRY(ensure_labels(c, nseeds, s));
  HRF_TRY(hrf_remove_small_objects_labels(ws, n, nseeds, 60, seeds, c->cnt, s));     // :155
  HRF_TRY(hrf_clear_border(seeds, H, W, lab3, c->parent, c->size, s));         // :156
  HRF_TRY(hrf_relabel_sequential(lab3, n, nseeds, seg_out, c->cnt, c->dint, s));     // :157
  return read_i32(c->dint, nlab_host, s);
}

}  // extern "C"
