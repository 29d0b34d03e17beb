// tile.hip -- one E. coli tile of the hot path as one native call (hrf_tile_ecoli).
//
// Reference: ecoli hiprfish_imaging_spectral_image_measurement.py measure_reference_images
// (:142-162 with -c T: segment_images :44-127, flat field :33-38, :147-157 per-cell means) and
// image_classification.py :43-71 (classification, identification map), collect :92-98 (counts).
// pipeline.register_tile + pipeline.process_tile compose the same steps from Python (~15
// foreign calls, ~30 tensor allocations and a host synchronisation for the cell count per
// tile); here they run from C++ on buffers a context owns for the tile size, so a tile is one
// foreign call (ctypes releases the GIL for its whole duration) and the per-cell tail runs on
// device-held row counts:
//   channel-max projections -> xcorr shifts (device) -> registered assembly writing image_cn and
//   the classifier's pixel table -> [side stream: per-pixel classification from the table] ->
//   segmentation chain (hrf_segment_ecoli_cn: its two synchronisations are the tile's only ones)
//   -> flat-fielded label sums read from the lasers -> cell table -> presence flags -> per-cell
//   classification -> barcode counts -> identification map -> join of the side stream.
// The calls are the library's own entry points (or their device-count twins), in pipeline.py's
// order, so the results equal the composed path bit for bit (tests/test_tile_gpu.py).
#include <algorithm>

#include "common.hpp"

namespace {

constexpr int NL = 5;                                    // E. coli lasers 405, 488, 514, 561, 633
constexpr int32_t CH[NL] = {32, 23, 20, 14, 6};          // channels per laser (ecoli :51-70)
constexpr int32_t BOUNDS[NL + 1] = {0, 32, 55, 75, 89, 95};
constexpr int32_t C = 95;
constexpr int32_t TILE_CHANMAX_WG = 512;  // the projections' workgroup budget in the tile path

template <class T>
hrf_status dalloc(T **p, size_t count) {
  HRF_HIP(hipMalloc((void **)p, sizeof(T) * (count ? count : 1)));
  return HRF_OK;
}

#define HRF_TRY(expr)                      \
  do {                                     \
    if (hrf_status r_ = (expr)) return r_; \
  } while (0)

}  // namespace

struct hrf_tile_ctx {
  int64_t H = 0, W = 0;
  hrf_seg_ctx *seg = nullptr;
  double *proj = nullptr;       // NL x H x W channel-max projections
  void *xwork = nullptr;        // xcorr workspace (power-of-two tiles) or the hipFFT one (others)
  bool pow2 = true;
  int32_t *shifts = nullptr;    // NL x 2
  double *cn = nullptr;         // image_cn
  void *table = nullptr;        // pixel table
  uint8_t *flags = nullptr;
  void *rwork = nullptr;        // the refine's list (hrf_classify_refine_work_bytes)
  int64_t rwork_bytes = 0;
  // per-label buffers, grown on demand (capacity cap labels + 1)
  int64_t cap = 0;
  double *sums = nullptr;
  int64_t *counts = nullptr;
  int32_t *rol = nullptr;
  double *fx = nullptr;         // cell presence flags (cap x NL)
  int32_t *nrows = nullptr;     // device row count
  double *refT = nullptr;       // library, channel-major, then its segment norms (R x 5)
  int64_t refT_cap = 0;
  hipEvent_t ev_reg = nullptr, ev_pix = nullptr;
  int32_t maxlab = 0;           // the last tile's, for hrf_tile_ecoli_cells
};

namespace {

hrf_status ensure_cap(hrf_tile_ctx *t, int64_t maxlab, hipStream_t s) {
  if (maxlab + 1 <= t->cap) return HRF_OK;
  HRF_HIP(hipStreamSynchronize(s));  // the previous tile's per-label work is done with them
  hipFree(t->sums);
  hipFree(t->counts);
  hipFree(t->rol);
  hipFree(t->fx);
  t->sums = nullptr;
  t->counts = nullptr;
  t->rol = nullptr;
  t->fx = nullptr;
  t->cap = 0;
  int64_t cap = 2048;
  while (cap < maxlab + 1) cap *= 2;
  HRF_TRY(dalloc(&t->sums, (size_t)cap * C));
  HRF_TRY(dalloc(&t->counts, (size_t)cap));
  HRF_TRY(dalloc(&t->rol, (size_t)cap));
  HRF_TRY(dalloc(&t->fx, (size_t)cap * NL));
  // later tiles clear sums and counts at the chain's watershed synchronisation
  HRF_HIP(hipMemsetAsync(t->sums, 0, sizeof(double) * (size_t)cap * C, s));
  HRF_HIP(hipMemsetAsync(t->counts, 0, sizeof(int64_t) * (size_t)cap, s));
  t->cap = cap;
  return HRF_OK;
}

// cell table onward (image_classification.py :43-71, collect :92-98) for the tile held in t
hrf_status tile_cells(hrf_tile_ctx *t, const int32_t *seg, const double *lib, const double *lib_flags, int32_t R,
                      int32_t variant, double flag_thr, int32_t cell_cap, int32_t *labels, double *avgint,
                      double *avgint_norm, int32_t *cell_idx, double *cell_dist, int32_t *ident, int64_t *counts,
                      int32_t *ncells_dev, hipStream_t s, bool counts_zeroed) {
  const int32_t maxlab = t->maxlab;
  HRF_REQUIRE(cell_cap >= maxlab, "tile_ecoli: cell buffers hold %d rows, the tile needs %d", cell_cap, maxlab);
  HRF_REQUIRE(variant == 0 || lib_flags, "tile_ecoli: the gated variants need the library's presence flags");
  HRF_TRY(hrf_cell_table(t->sums, t->counts, maxlab, C, maxlab, t->rol, labels, avgint, avgint_norm, ncells_dev, s));
  if (variant) HRF_TRY(hrf::segment_flags_devn(avgint_norm, maxlab, ncells_dev, C, BOUNDS, NL, flag_thr, t->fx, s));
  if ((int64_t)R * (C + NL) > t->refT_cap) {
    HRF_HIP(hipStreamSynchronize(s));
    hipFree(t->refT);
    t->refT = nullptr;
    t->refT_cap = 0;
    HRF_TRY(dalloc(&t->refT, (size_t)R * (C + NL)));
    t->refT_cap = (int64_t)R * (C + NL);
  }
  double *ny = t->refT + (size_t)R * C;
  HRF_TRY(hrf::cells_lib_prep(lib, R, C, BOUNDS, NL, t->refT, ny, s));
  HRF_TRY(hrf::classify_cells_devn(avgint_norm, maxlab, ncells_dev, t->refT, ny, R, C, BOUNDS, NL, variant,
                                   variant ? t->fx : nullptr, variant ? lib_flags : nullptr, cell_idx, cell_dist, s));
  // per-barcode counts (collect :92-98) and the identification map (:65-71); one fused launch
  // lost (1013 vs 1019 Mpix/s, profiles/r4i_fusion_ab.txt) and was removed in round 5
  HRF_TRY(hrf::barcode_counts_devn(cell_idx, maxlab, ncells_dev, R, counts, s, counts_zeroed));
  HRF_TRY(hrf::paint_ids_devn(seg, t->H * t->W, cell_idx, maxlab, ncells_dev, 1, ident, s));
  return HRF_OK;
}

}  // namespace

extern "C" {

hrf_status hrf_tile_ctx_create(int64_t H, int64_t W, hrf_tile_ctx **out) {
  HRF_REQUIRE(out && H >= 1 && W >= 16 && W % 16 == 0 && H * W < ((int64_t)1 << 31),
              "tile_ctx: bad size (W a multiple of 16)");
  // power-of-two tiles: the hand-written FFT pipeline (xcorr.hip); other sizes: hipFFT per target
  // (register.hip), the same shifts (tests/test_registration_gpu.py)
  const int64_t xw = hrf_xcorr_workspace_bytes(NL, H, W);
  const int64_t xb = xw > 0 ? xw : hrf_register_workspace_bytes(H, W);
  HRF_REQUIRE(xb > 0, "tile_ctx: registration workspace size");
  const int64_t tb = hrf_pixtable_bytes(H * W, C, BOUNDS, NL);
  HRF_REQUIRE(tb > 0, "tile_ctx: pixel table size");
  hrf_tile_ctx *t = new hrf_tile_ctx();
  t->H = H;
  t->W = W;
  t->pow2 = xw > 0;
  auto fail = [&](hrf_status st) {
    hrf_tile_ctx_destroy(t);
    return st;
  };
  const size_t n = (size_t)(H * W);
  hrf_status r;
  if ((r = hrf_seg_ctx_create(H, W, &t->seg))) return fail(r);
  if ((r = dalloc(&t->proj, NL * n)) || (r = dalloc((char **)&t->xwork, (size_t)xb)) ||
      (r = dalloc(&t->shifts, 2 * NL)) || (r = dalloc(&t->cn, n)) || (r = dalloc((char **)&t->table, (size_t)tb)) ||
      (r = dalloc(&t->flags, n)) || (r = dalloc(&t->nrows, 4)) ||
      (r = dalloc((char **)&t->rwork, (size_t)hrf_classify_refine_work_bytes((int64_t)n))))
    return fail(r);
  t->rwork_bytes = hrf_classify_refine_work_bytes((int64_t)n);
  if (hipEventCreateWithFlags(&t->ev_reg, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&t->ev_pix, hipEventDisableTiming) != hipSuccess) {
    ::hrf::set_error("tile_ctx: event creation failed");
    return fail(HRF_EHIP);
  }
  *out = t;
  return HRF_OK;
}

hrf_status hrf_tile_ctx_destroy(hrf_tile_ctx *t) {
  if (!t) return HRF_OK;
  if (t->seg) hrf_seg_ctx_destroy(t->seg);
  hipFree(t->proj);
  hipFree(t->xwork);
  hipFree(t->shifts);
  hipFree(t->cn);
  hipFree(t->table);
  hipFree(t->flags);
  hipFree(t->rwork);
  hipFree(t->nrows);
  hipFree(t->sums);
  hipFree(t->counts);
  hipFree(t->rol);
  hipFree(t->fx);
  hipFree(t->refT);
  if (t->ev_reg) hipEventDestroy(t->ev_reg);
  if (t->ev_pix) hipEventDestroy(t->ev_pix);
  delete t;
  return HRF_OK;
}

hrf_status hrf_tile_ctx_pixel_listed(hrf_tile_ctx *t, int32_t *n_host) {
  HRF_REQUIRE(t && n_host, "tile_ctx_pixel_listed: bad arguments");
  HRF_HIP(hipMemcpy(n_host, t->rwork, sizeof(int32_t), hipMemcpyDeviceToHost));
  return HRF_OK;
}

hrf_status hrf_tile_ctx_seg(hrf_tile_ctx *t, hrf_seg_ctx **seg) {
  HRF_REQUIRE(t && seg, "tile_ctx_seg: bad arguments");
  *seg = t->seg;
  return HRF_OK;
}

hrf_status hrf_tile_ecoli(hrf_tile_ctx *t, const float *const *lasers_host, const float *cal, const void *refx,
                          const double *lib, const double *lib_flags, int32_t R, int32_t variant, double flag_thr,
                          int32_t per_pixel, int32_t *seg, int32_t *pixel_idx, float *pixel_dist, int32_t cell_cap,
                          int32_t *labels, double *avgint, double *avgint_norm, int32_t *cell_idx, double *cell_dist,
                          int32_t *ident, int64_t *counts, int32_t *ncells_dev, int32_t *maxlab_host,
                          hrf_stream_t stream, hrf_stream_t side_stream, hrf_event_t pix_start, hrf_event_t pix_end) {
  HRF_REQUIRE(t && lasers_host && lib && R >= 1 && seg && ident && counts && ncells_dev && maxlab_host,
              "tile_ecoli: bad arguments");
  HRF_REQUIRE(!per_pixel || (refx && pixel_idx && pixel_dist), "tile_ecoli: per-pixel outputs missing");
  for (int l = 0; l < NL; ++l) HRF_REQUIRE(lasers_host[l], "tile_ecoli: laser %d missing", l);
  hipStream_t s = (hipStream_t)stream;
  hipStream_t side = side_stream ? (hipStream_t)side_stream : s;
  const int64_t H = t->H, W = t->W, n = H * W;
  // ecoli :45-57 shifts of the channel-max projections, on the device
  double *proj[NL];
  for (int l = 0; l < NL; ++l) proj[l] = t->proj + l * n;
  // on 512 workgroups (two per CU): slower alone (0.77 vs 0.39 ms) but it leaves room on every CU
  // for the concurrent tiles' classifier workgroups -- +1.4 % end to end, 5 of 5 interleaved runs
  // (profiles/r5_chanmax_grid_ab.txt)
  HRF_TRY(hrf_channel_max_multi_grid(lasers_host, CH, NL, n, proj, TILE_CHANMAX_WG, s));
  if (t->pow2) {
    HRF_TRY(hrf_xcorr_shifts_dev(t->proj, NL, H, W, t->xwork, 15, t->shifts, s));
  } else {  // row 0 = (0, 0); the reference's transform is taken once (src == NULL reuses it)
    HRF_HIP(hipMemsetAsync(t->shifts, 0, 2 * sizeof(int32_t), s));
    for (int l = 1; l < NL; ++l)
      HRF_TRY(hrf_register_translation_dev(l == 1 ? proj[0] : nullptr, proj[l], H, W, t->xwork, 15, t->shifts + 2 * l,
                                           s));
  }
  // ecoli :58-72 registered assembly (coverage mask) -> image_cn + the pixel table (image_cn only
  // without the per-pixel classifier: 0.78 vs 0.94 ms)
  HRF_TRY(hrf_register_assemble_pixtable(lasers_host, CH, t->shifts, NL, H, W, 1, nullptr, t->cn, 1,
                                         per_pixel ? t->table : nullptr, per_pixel ? t->flags : nullptr, s));
  if (per_pixel) {  // north_star per-pixel mode, beside the segmentation chain
    if (side != s) {
      HRF_HIP(hipEventRecord(t->ev_reg, s));
      HRF_HIP(hipStreamWaitEvent(side, t->ev_reg, 0));
    }
    if (pix_start) HRF_HIP(hipEventRecord((hipEvent_t)pix_start, side));
    // the split-fp16 screen from the assembly's table with its exact f64 refine fused in, reading
    // the pixels from the five shifted acquisitions, then the list pass
    // (hrf_classify_pixels_table_exact)
    HRF_TRY(hrf_classify_pixels_table_exact(t->table, t->flags, lasers_host, CH, t->shifts, NL, H, W, 1, refx, R,
                                            BOUNDS, NL, pixel_idx, pixel_dist, t->rwork, t->rwork_bytes, side));
    if (pix_end) HRF_HIP(hipEventRecord((hipEvent_t)pix_end, side));
    if (side != s) HRF_HIP(hipEventRecord(t->ev_pix, side));
  }
  auto join = [&]() -> hrf_status {
    if (per_pixel && side != s) HRF_HIP(hipStreamWaitEvent(s, t->ev_pix, 0));
    return HRF_OK;
  };
  int32_t maxlab = 0;
  // the per-label sums and counts (their current capacity) and the barcode counts are cleared
  // inside the chain's watershed read-back launch (no fill kernels of their own)
  // Entry budget: these 3 clears + the segmentation's 2 clears and 3 read-backs at the watershed
  // batch (segment.hip) must fit ZeroPub::N per kind; every add is checked, since a dropped clear
  // would add the previous tile's sums into this one.
  static_assert(::hrf::ZeroPub::N >= 5, "ZeroPub: the tile's and the segmentation's clears share one launch");
  ::hrf::ZeroPub zp;
  if (!(zp.zero(t->sums, sizeof(double) * (size_t)t->cap * C) && zp.zero(t->counts, sizeof(int64_t) * (size_t)t->cap) &&
        zp.zero(counts, sizeof(int64_t) * (size_t)R))) {
    join();
    ::hrf::set_error("tile_ecoli: per-label clears do not fit the read-back launch");
    return HRF_EINVAL;
  }
  hrf_status st = ::hrf::segment_ecoli_cn_extra(t->seg, t->cn, seg, &maxlab, s, &zp);   // :73-127
  if (st) {
    join();
    return st;
  }
  t->maxlab = maxlab;
  *maxlab_host = maxlab;
  if ((st = ensure_cap(t, maxlab, s)) ||
      (st = ::hrf::label_sums_lasers_zeroed(lasers_host, CH, t->shifts, NL, H, W, 1, seg, maxlab, cal, 0, 32,
                                            t->sums, t->counts, s))) {                   // :147-155
    join();
    return st;
  }
  if (maxlab <= cell_cap)
    st = tile_cells(t, seg, lib, lib_flags, R, variant, flag_thr, cell_cap, labels, avgint, avgint_norm, cell_idx,
                    cell_dist, ident, counts, ncells_dev, s, true);
  if (hrf_status j = join()) return st ? st : j;
  return st;
}

hrf_status hrf_tile_ecoli_cells(hrf_tile_ctx *t, const int32_t *seg, const double *lib, const double *lib_flags,
                                int32_t R, int32_t variant, double flag_thr, int32_t cell_cap, int32_t *labels,
                                double *avgint, double *avgint_norm, int32_t *cell_idx, double *cell_dist,
                                int32_t *ident, int64_t *counts, int32_t *ncells_dev, hrf_stream_t stream) {
  HRF_REQUIRE(t && seg && lib && R >= 1 && ident && counts && ncells_dev, "tile_ecoli_cells: bad arguments");
  return tile_cells(t, seg, lib, lib_flags, R, variant, flag_thr, cell_cap, labels, avgint, avgint_norm, cell_idx,
                    cell_dist, ident, counts, ncells_dev, (hipStream_t)stream, false);
}

}  // extern "C"
