"""Device pipelines: the reference's measurement and classification stages, every compute
step a libhrf.so kernel (kernels.py).  Tensors stay resident in HBM from the (H, W, C) stack
to the label map, per-cell spectra, barcode ids and counts.

Each function cites the reference lines it stands in for.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from dataclasses import dataclass, field

import torch

from . import kernels as K

ECOLI_BOUNDS = (0, 32, 55, 75, 89, 95)
MULTI_BOUNDS = (0, 23, 43, 57, 63)


# --------------------------------------------------------------------------------------------
# E. coli / reference-library measurement (hiprfish_imaging_spectral_image_measurement.py)
# --------------------------------------------------------------------------------------------
def erosion_seeds(cell_sm: torch.Tensor, area_max: int = 600, min_obj: int = 10) -> torch.Tensor:
    """ecoli measurement.py:97-110: freeze regions below `area_max` as seeds, erode the rest,
    drop fragments < `min_obj` (4-connected), repeat until nothing is left.  -> seed mask u8
    One launch, one workgroup per 8-connected component (seeds.hip)."""
    return K.erosion_seeds(cell_sm, area_max, min_obj)


def erosion_seeds_global(cell_sm: torch.Tensor, area_max: int = 600, min_obj: int = 10) -> torch.Tensor:
    """The same loop as whole-image passes (one CC / erosion / sieve launch set per iteration);
    kept as a cross-check of the per-component kernel."""
    be = torch.zeros_like(K._u8(cell_sm, "cell_sm"))
    m = K._u8(cell_sm, "cell_sm")
    while K.count_nonzero(m) > 0:                      # markers = regionprops(dist_lab) non-empty
        m = K.split_by_size(m, area_max, be, conn=2)   # :102-106 (dist_lab is 8-connected)
        m = K.binary_erosion(m, 1)                     # :107
        m = K.remove_small_objects(m, min_obj, conn=1)  # :108
    return be


# The segmentation chains run as one native call (segment.hip, same calls in the same order)
# unless intermediates are requested (`keep`) or HRF_NATIVE_SEG=0.
NATIVE_SEG = os.environ.get("HRF_NATIVE_SEG", "1") != "0"
# power-of-two tiles: the registration cross-correlations through xcorr.hip (six launches for all
# lasers) instead of hipFFT; HRF_XCORR=0 keeps hipFFT
XCORR = os.environ.get("HRF_XCORR", "1") != "0"


def segment_ecoli(stack: torch.Tensor, keep: dict | None = None, image_cn: torch.Tensor | None = None):
    """ecoli measurement.py:44-127 on the registered stack.  -> (segmentation int32, max label)
    image_cn: the stack's log(sum + 1e-2) when already computed (register_stack(want_cn=True))"""
    if keep is None and NATIVE_SEG:
        return K.segment_ecoli_native(stack, image_cn)
    if image_cn is None:
        image_cn = K.channel_sum(stack, mode=1)                          # :71-72 log(sum + 1e-2)
    share = {}                                                           # one sort for both fits
    _, rough_mask, _, _ = K.kmeans_1d(image_cn, 2, want_labels=False, share=share, rule=2)  # :73-84 brighter
    _, interior, _, _ = K.kmeans_1d(image_cn, 3, want_labels=False, share=share, rule=0)    # :85-94 brightest
    opened = K.binary_opening(K.remove_small_holes(interior, 64, 1))      # :95
    cell_sm = K.remove_small_objects(opened, 50, conn=1)                 # :96
    be = erosion_seeds(cell_sm)                                          # :97-110
    seeds_mask = K.remove_small_objects(be, 10, conn=2)                  # :111 rso(label(dist_be), 10)
    seeds, nseeds = K.label(seeds_mask, conn=2)                          # :111-112
    seg = K.watershed(image_cn, seeds, rough_mask, negate=True)          # :113 watershed(-image_cn)
    seg = K.remove_small_objects(seg, 100, maxlab=nseeds)                # :114
    seg = K.clear_border(seg)                                            # :115
    props = K.region_props(seg, nseeds)                                  # :116 regionprops
    final = K.shape_filter(seg, props, nseeds, 15.0, 35.0)               # :117-126
    if keep is not None:
        keep.update(image_cn=image_cn, rough_mask=rough_mask, interior=interior, cell_sm=cell_sm, seeds=seeds,
                    watershed=seg)
    return final, nseeds


@dataclass
class Measurement:
    segmentation: torch.Tensor      # (H, W) int32 (labels not re-sequenced, as the reference)
    maxlab: int
    labels: torch.Tensor            # (N,) int32 label of each row (ascending, regionprops order)
    avgint: torch.Tensor            # (N, C) f64 per-cell mean spectrum
    avgint_norm: torch.Tensor       # (N, C) f64 max-normalised
    extras: dict = field(default_factory=dict)


def measure_ecoli(stack: torch.Tensor, calibration: torch.Tensor | None = None, keep: dict | None = None,
                  image_cn: torch.Tensor | None = None):
    """ecoli measurement.py:142-162: segment, flat-field channels 0..31 (load_calibration_images
    :33-38 puts the calibration image on channels 0-31 and 1.0 elsewhere), per-cell means."""
    if isinstance(stack, RegisteredTile):
        seg, maxlab = segment_ecoli(stack, keep, stack.image_cn)
        sums, counts = K.label_sums_lasers(stack.lasers, stack.shifts, seg, maxlab, stack.apply_mask,
                                           cal=calibration, cal_range=(0, 32))                   # :147-155
        _, lor, avgint, avgint_norm = K.cell_table(sums, counts, maxlab)                          # :151-157
        return Measurement(seg, maxlab, lor, avgint, avgint_norm)
    seg, maxlab = segment_ecoli(stack, keep, image_cn)
    sums, counts = K.label_sums(stack, seg, maxlab, cal=calibration,
                                cal_range=(0, 32) if calibration is not None else None)   # :147-155
    _, lor, avgint, avgint_norm = K.cell_table(sums, counts, maxlab)                      # :151-157
    return Measurement(seg, maxlab, lor, avgint, avgint_norm)


# --------------------------------------------------------------------------------------------
# Registration shift estimate
# --------------------------------------------------------------------------------------------
def estimate_shifts(lasers, reduce: str = "max", clamp: int | None = 15, device: bool = False):
    """Integer shift of every laser stack against the first, skimage register_translation
    (upsample 1) on a per-laser projection:
    * reduce "max": np.max(image, axis=2), |shift| > clamp -> 0 (ecoli measurement.py:45-57);
    * reduce "sum": np.sum(image, axis=2), no clamp (multispecies measurement.py:82-84).
    -> [(0, 0), (dr_1, dc_1), ...] ready for kernels.register_assemble; with `device` an
    (nlaser, 2) int32 device tensor instead (no host synchronisation; register_assemble reads
    it on the device)."""
    H, W = lasers[0].shape[:2]
    if reduce == "max" and len(lasers) <= 8:
        proj = K.channel_max_multi(lasers, stacked=True)                 # one launch for all lasers
        if device and len(lasers) >= 2 and XCORR and K.xcorr_supported(*proj.shape):
            return K.xcorr_shifts_dev(proj, clamp)                      # hand-written FFT pipeline
        proj = list(proj.unbind(0))
    elif reduce == "sum" and device and len(lasers) >= 2 and XCORR and K.xcorr_supported(len(lasers), H, W):
        proj = torch.empty((len(lasers), H, W), dtype=torch.float64, device=lasers[0].device)
        for i, s in enumerate(lasers):
            K.channel_sum(s, out=proj[i])                               # numpy's pairwise order
        return K.xcorr_shifts_dev(proj, clamp)
    else:
        proj = [K.channel_max(s) if reduce == "max" else K.channel_sum(s) for s in lasers]
    if device:
        return K.register_translations_dev(proj[0], proj[1:], clamp)
    shifts = [(0, 0)]
    for img in proj[1:]:
        r, c = K.register_translation(proj[0], img)
        if clamp is not None:
            r = 0 if abs(r) > clamp else r
            c = 0 if abs(c) > clamp else c
        shifts.append((r, c))
    return shifts


def register_stack(lasers, reduce: str = "max", clamp: int | None = 15, apply_mask: bool = True,
                   want_cn: bool = False):
    """ecoli measurement.py:44-70 (-c T: plus load_calibration_images :33-38, applied to the
    per-cell spectra by measure_ecoli): shift estimate on the per-laser projections, then the
    registered, concatenated (H, W, C) stack -- one stream, no synchronisation.  want_cn: also
    image_cn = log(sum + 1e-2) of the registered stack (:71-72) from the assembly pass
    -> (stack, image_cn)."""
    return K.register_assemble(lasers, estimate_shifts(lasers, reduce, clamp, device=True), apply_mask,
                               cn_mode=1 if want_cn else None)


def register_multispecies(lasers, shifts=None):
    """multispecies measurement.py:79-102: the four acquisitions (488, 514, 561, 633) registered on
    their channel sums -- skimage register_translation(sum_0, sum_i), no clamp (:82-84) -- and
    concatenated with zeros outside each shifted frame and NO coverage-mask multiply (:85-102;
    the mask is built but never applied).  shifts: (n, 2) device tensor or host pairs to use
    instead of the estimate.  -> (H, W, C) f32 registered stack (one stream, no synchronisation)"""
    if shifts is None:
        shifts = estimate_shifts(lasers, reduce="sum", clamp=None, device=True)
    return K.register_assemble(lasers, shifts, apply_mask=False)


@dataclass
class RegisteredTile:
    """A registered E. coli tile that is never materialised as an (H, W, C) stack: the per-laser
    acquisitions with their device shifts, image_cn (:71-72) and the per-pixel classifier's
    prepared operands, all written by one assembly pass (register_tile).  process_tile classifies
    its pixels from the table and takes the per-cell spectra from the lasers
    (kernels.label_sums_lasers) -- the same results as register_stack + process_tile."""
    lasers: list
    shifts: torch.Tensor
    image_cn: torch.Tensor
    pixtable: object
    apply_mask: bool = True

    @property
    def shape(self):
        H, W = self.image_cn.shape
        return (H, W, self.pixtable.C)

    @property
    def device(self):
        return self.image_cn.device


def register_tile(lasers, reduce: str = "max", clamp: int | None = 15, apply_mask: bool = True):
    """register_stack(lasers, want_cn=True) without the stack (ecoli measurement.py:44-72): shift
    estimate on the device, then ONE pass over the lasers writing image_cn and the classifier's
    pixel table.  Needs the five E. coli lasers and W a multiple of 16; otherwise returns
    register_stack's (stack, image_cn)."""
    H, W = lasers[0].shape[:2]
    if len(lasers) != 5 or W % 16 or [int(l.shape[2]) for l in lasers] != [32, 23, 20, 14, 6]:
        return register_stack(lasers, reduce, clamp, apply_mask, want_cn=True)
    shifts = estimate_shifts(lasers, reduce, clamp, device=True)
    cn, pt, _ = K.register_assemble_pixtable(lasers, shifts, apply_mask, cn_mode=1, bounds=ECOLI_BOUNDS)
    return RegisteredTile(list(lasers), shifts, cn, pt, apply_mask)


# --------------------------------------------------------------------------------------------
# Biofilm 3-D enhancement input (hiprfish_imaging_biofilm_analysis.py:808-817)
# --------------------------------------------------------------------------------------------
def enhance_volume(stack: torch.Tensor, v3: bool = False) -> torch.Tensor:
    """biofilm :808-817 on the registered (X, Y, Z, C) volume: channel sum (numpy order),
    / max, edge pad 5, line_profile_memory_efficient_v2 (v3 with `v3`) and the
    average * (1 - quartile coefficient) post-chain -> image_final (X+10, Y+10, Z+10) f64"""
    X, Y, Z, C = stack.shape
    s = K.channel_sum(stack.reshape(X * Y, Z, C)).reshape(X, Y, Z)     # :808
    s = K.div_scalar(s, K.max_f64(s))                                   # :809
    pad = K.pad_edge_3d(s, 5)                                           # :810
    return K.enhance_3d_v3(pad) if v3 else K.enhance_3d(pad)            # :811-817


# --------------------------------------------------------------------------------------------
# Synthetic-community measurement (hiprfish_imaging_multispecies_spectral_image_measurement.py)
# --------------------------------------------------------------------------------------------
def segment_multispecies(stack: torch.Tensor, calibration: torch.Tensor | None = None, keep: dict | None = None):
    """multispecies measurement.py:102-157 on the registered (H, W, C) stack.
    -> (segmentation int32 relabelled 1..n, n, registered sum f64, final_bkg_filtered f64)

    The two KMeans(2) cluster choices (:125-135, :141-149) take the cluster whose positive
    values have the larger mean -- for a 1-D partition into intervals the upper one -- and
    sklearn's cluster 0 when one of them holds no positive value (the reference compares a NaN
    mean then): kernels.kmeans_1d rule 1."""
    if keep is None and NATIVE_SEG:
        return K.segment_multispecies_native(stack, calibration)
    s = K.channel_sum(stack, cal=calibration)                    # :104-105 sum(stack / cal)
    norm = K.div_scalar(s, K.max_f64(s))                         # :106
    nl = K.nl_means_2d(norm, 7, 11, 0.02, 0.0)                   # :108 (estimate_sigma :107 unused)
    final = K.enhance_2d(K.pad_edge(nl, 5))                      # :109-124
    _, rough, _, _ = K.kmeans_1d(final, 2, want_labels=False, rule=1)    # :125-135
    opened = K.remove_small_objects(K.binary_opening(rough), 10, conn=1)   # :136-137
    seeds_mask = K.and_mask(K.fill_holes(opened), K.fill_holes(rough))     # :138-140
    seeds, nseeds = K.label(seeds_mask, conn=2)                  # :140 measure.label (8-conn)
    _, bkg, _, _ = K.kmeans_1d(nl, 2, want_labels=False, rule=1)         # :141-149
    final_bkg = K.mask_mul(final, bkg)                           # :150
    seeds_bkg = K.mask_labels(seeds, bkg)                        # :152
    wmask = K.and_mask(rough, bkg)                               # :153
    seg = K.watershed(final_bkg, seeds_bkg, wmask, negate=True)  # :154 watershed(-final_bkg)
    seg = K.remove_small_objects(seg, 60, maxlab=nseeds)         # :155
    seg = K.clear_border(seg)                                    # :156
    seg, n = K.relabel_sequential(seg, nseeds)                   # :157
    if keep is not None:
        keep.update(image_sum=s, nl=nl, final=final, rough_mask=rough, seeds=seeds, bkg_mask=bkg,
                    watershed=seg)
    return seg, n, s, final_bkg


def measure_multispecies(stack: torch.Tensor, calibration: torch.Tensor | None = None, keep: dict | None = None):
    """multispecies measurement.py:161-174: segment, per-cell mean of the calibrated stack
    (regionprops mean_intensity per channel, :167-171), row-max normalisation (:172)."""
    seg, n, s, final_bkg = segment_multispecies(stack, calibration, keep)
    sums, counts = K.label_sums(stack, seg, n, cal=calibration)
    _, lor, avgint, avgint_norm = K.cell_table(sums, counts, n)
    return Measurement(seg, n, lor, avgint, avgint_norm, extras=dict(image_sum=s, final_bkg=final_bkg))


# --------------------------------------------------------------------------------------------
# Classification (segmented cosine against a reference library)
# --------------------------------------------------------------------------------------------
@dataclass
class Library:
    """Reference barcode library: row r is barcode r + 1 (mean spectrum of enc_{r+1},
    train_reference.py:1397), max-normalised."""
    spectra: torch.Tensor        # (R, C) f64
    bounds: tuple
    nbit: int
    _refx: torch.Tensor | None = None
    _refx2: torch.Tensor | None = None
    _flags: dict = field(default_factory=dict)

    @property
    def R(self):
        return self.spectra.shape[0]

    def refx(self):
        if self._refx is None:
            self._refx = K.classify_prepare(self.spectra.to(torch.float32), self.bounds)
        return self._refx

    def refx_table(self):
        """the mode-2 table the pixel-table classifier (register_tile, process_tile_native) reads,
        whatever mode refx() was prepared in"""
        r = self.refx()
        if K.refx_mode(r, self.spectra.shape[1], self.bounds) == 2:
            return r
        if self._refx2 is None:
            self._refx2 = K.classify_prepare(self.spectra.to(torch.float32), self.bounds, mode=2)
        return self._refx2

    def presence_flags(self, thr: float = 0.1) -> torch.Tensor:
        """per-segment presence of the library rows (max over the segment > thr), computed once
        per threshold"""
        f = self._flags.get(thr)
        if f is None:
            f = self._flags[thr] = segment_flags(self.spectra, self.bounds, thr)
        return f


def segment_flags(x: torch.Tensor, bounds, thr: float = 0.1) -> torch.Tensor:
    """the gated metrics' presence flags on the library path: max over each segment > thr
    (hrf_segment_flags)"""
    return K.segment_flags(x, bounds, thr)


def classify_cells(avgint_norm: torch.Tensor, lib: Library, variant: int = 0, flag_thr: float = 0.1):
    """image_classification.py:43-56 / classify_spectra.py:27-35 restated on the max-normalised
    cell spectra (hrf_cell_table computes avgint / rowmax, :43): argmin of the segmented-cosine
    distance over the library.  variant 0: ungated mean of segment distances; 1:
    channel_cosine_intensity gating (train_reference.py:223-386); 2: _7b_v2 gating
    (:993-1072).  -> (index, distance)"""
    x = avgint_norm
    fx = fr = None
    if variant:
        fx = segment_flags(x, lib.bounds, flag_thr)
        fr = lib.presence_flags(flag_thr)
    return K.classify_cells(x, lib.spectra, lib.bounds, variant, fx, fr)


def classify_pixels(stack: torch.Tensor, lib: Library):
    """north_star per-pixel mode: argmin over the library of the ungated segmented-cosine
    distance for every pixel spectrum (one fused f32-MFMA GEMM + argmax)."""
    return K.classify_pixels(stack, lib.refx(), lib.R, lib.bounds)


def barcode_strings(idx, nbit: int):
    """barcode number = library row + 1, written as the reference's binary code string"""
    return [format(int(i) + 1, "0%db" % nbit) for i in idx]


@dataclass
class TileResult:
    meas: Measurement
    cell_idx: torch.Tensor
    cell_dist: torch.Tensor
    counts: torch.Tensor
    identification: torch.Tensor
    pixel_idx: torch.Tensor | None = None
    pixel_dist: torch.Tensor | None = None


_SIDE_STREAMS: "OrderedDict" = OrderedDict()
SIDE_PRIORITY = 0   # stream priority of the classifier side streams (torch convention: lower = higher)
SIDE_STREAMS_MAX = 64


def _side_stream(main: torch.cuda.Stream) -> torch.cuda.Stream:
    """the side stream paired with `main` (one per caller stream, so concurrent tiles on
    different streams do not serialise on a shared one); the least recently used beyond
    SIDE_STREAMS_MAX are dropped (work queued on them is held by the events their callers joined)"""
    key = (main.device, main.cuda_stream, SIDE_PRIORITY)
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=main.device, priority=SIDE_PRIORITY)
        while len(_SIDE_STREAMS) > SIDE_STREAMS_MAX:
            _SIDE_STREAMS.popitem(last=False)
    else:
        _SIDE_STREAMS.move_to_end(key)
    return s


@dataclass
class PendingTile:
    """A tile whose per-pixel classification is enqueued (start_tile) and whose measurement is
    not yet (finish_tile)."""
    stack: object
    lib: Library
    main: torch.cuda.Stream
    side: torch.cuda.Stream | None
    pix: tuple | None
    overlap: bool


def process_tile(stack: torch.Tensor, lib: Library, calibration=None, per_pixel: bool = True, variant: int = 0,
                 overlap: bool = True, pixel_events: list | None = None, measure=None, image_cn=None):
    """One tile of the hot path: measure (segment + per-cell spectra) + classify + count.

    The per-pixel classification does not depend on the segmentation, so with `overlap` it
    runs on a side stream concurrently with the segmentation chain (many small, latency-bound
    launches and a few host synchronisations) and fills the compute units that chain leaves
    idle; the caller's stream joins it before returning.  `pixel_events`, if given, receives
    the (start, end) events recorded around the classification on the stream it ran on.
    `measure` selects the measurement chain (default measure_ecoli; measure_multispecies for
    the synthetic-community pipeline); `image_cn` hands measure_ecoli the log-sum image the
    registration pass already produced.  `stack` may be a RegisteredTile (register_tile): the
    pixels are then classified from its prepared table and the per-cell spectra read from its
    lasers.  process_tile = finish_tile(start_tile(...)); a caller driving a sequence of tiles
    may start tile i+1 before finishing tile i, so that tile's classifier is queued while tile
    i's segmentation chain runs."""
    p = start_tile(stack, lib, per_pixel, overlap, pixel_events)
    return finish_tile(p, calibration, variant, measure, image_cn)


def start_tile(stack, lib: Library, per_pixel: bool = True, overlap: bool = True,
               pixel_events: list | None = None) -> PendingTile:
    """first half of process_tile: enqueue the per-pixel classification (side stream with
    `overlap`, after everything the caller's stream holds so far, i.e. the stack / table)"""
    main = torch.cuda.current_stream(stack.device)
    reg = isinstance(stack, RegisteredTile)
    pix = None
    side = None
    if per_pixel:
        refx = lib.refx_table() if reg else lib.refx()        # prepared on the caller's stream
        side = _side_stream(main) if overlap else main
        if overlap:
            side.wait_stream(main)                            # stack (and refx) ready
        with torch.cuda.stream(side):
            e0 = e1 = None
            if pixel_events is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(side)
            if reg:                                           # from the assembly's pixel table
                pix = K.classify_pixels_table(stack.pixtable, refx, lib.R)
            else:
                pix = K.classify_pixels(stack, refx, lib.R, lib.bounds)
            if pixel_events is not None:
                e1.record(side)
                pixel_events.append((e0, e1))
        if overlap:
            if reg:
                stack.pixtable.table.record_stream(side)
                stack.pixtable.flags.record_stream(side)
            else:
                stack.record_stream(side)
            refx.record_stream(side)
    return PendingTile(stack, lib, main, side, pix, overlap)


def finish_tile(p: PendingTile, calibration=None, variant: int = 0, measure=None, image_cn=None) -> TileResult:
    """second half of process_tile, on the stream start_tile was called on: measurement,
    per-cell classification, counts, identification map, then the join with the per-pixel
    classification"""
    stack, lib, main, side, pix, overlap = p.stack, p.lib, p.main, p.side, p.pix, p.overlap
    per_pixel = pix is not None
    reg = isinstance(stack, RegisteredTile)
    if reg:
        meas = measure_ecoli(stack, calibration)
    elif image_cn is not None:
        meas = (measure or measure_ecoli)(stack, calibration, image_cn=image_cn)
    else:
        meas = (measure or measure_ecoli)(stack, calibration)
    idx, dist = classify_cells(meas.avgint_norm, lib, variant)
    counts = K.barcode_counts(idx, lib.R)                       # collect_measurement_results.py:92-98
    ident = K.paint_ids(meas.segmentation, idx + 1)             # image_classification.py:65-71
    res = TileResult(meas, idx, dist, counts, ident)
    if per_pixel:
        if overlap:
            main.wait_stream(side)
            for t in pix:
                t.record_stream(main)
        res.pixel_idx, res.pixel_dist = pix
    return res


class NativeTileResult:
    """TileResult of process_tile_native: the per-cell rows are narrowed to the tile's cell count
    on first access (one read of the device-held count); counts, the identification map and
    the per-pixel outputs need no host round trip."""

    def __init__(self, d):
        self._d = d
        self._n = None
        self.counts = d["counts"]
        self.identification = d["ident"]
        self.pixel_idx = d["pixel_idx"]
        self.pixel_dist = d["pixel_dist"]

    @property
    def ncells(self) -> int:
        if self._n is None:
            self._n = int(self._d["ncells"].item())
        return self._n

    @property
    def cell_idx(self):
        return self._d["cell_idx"][:self.ncells]

    @property
    def cell_dist(self):
        return self._d["cell_dist"][:self.ncells]

    @property
    def meas(self) -> Measurement:
        d, n = self._d, self.ncells
        return Measurement(d["seg"], d["maxlab"], d["labels"][:n], d["avgint"][:n], d["avgint_norm"][:n])


def process_tile_native(lasers, lib: Library, calibration=None, per_pixel: bool = True, variant: int = 1,
                        overlap: bool = True, pixel_events: list | None = None) -> NativeTileResult:
    """register_tile(lasers) + process_tile(..., variant) as ONE native call (hrf_tile_ecoli,
    tile.hip): ecoli measurement.py:44-162 (-c T) + image_classification.py:43-71 + collect
    :92-98, the per-pixel classifier on the side stream with `overlap`.  The same results as the
    composed path bit for bit (tests/test_tile_gpu.py).  lasers: the five E. coli acquisitions
    (W a multiple of 16; the registration FFT is xcorr.hip for power-of-two H and W, hipFFT
    otherwise)."""
    main = torch.cuda.current_stream(lasers[0].device)
    side = _side_stream(main) if (per_pixel and overlap) else None
    refx = lib.refx_table() if per_pixel else None
    flags = lib.presence_flags() if variant else None
    d = K.tile_ecoli(lasers, calibration, refx, lib.spectra, flags, variant=variant, per_pixel=per_pixel, side=side,
                     pix_events=pixel_events)
    return NativeTileResult(d)


# --------------------------------------------------------------------------------------------
# Multi-GPU: tiles shard round-robin; the only exchange is the per-barcode count vector
# --------------------------------------------------------------------------------------------
def shard(n_tiles: int, rank: int, world: int):
    """tile indices owned by `rank` (tile_idx % world)"""
    return list(range(rank, n_tiles, world))


def allreduce_counts(counts: torch.Tensor, group=None) -> torch.Tensor:
    """global per-barcode counts = SUM over ranks (collect_measurement_results.py:92-98 across
    FOVs).  RCCL on device tensors; any torch.distributed backend works."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    return counts


def allreduce_adjacency(adj: torch.Tensor, group=None) -> torch.Tensor:
    """the optional second exchange: the int64 (R, R) barcode adjacency summed over
    ranks, one all-reduce of R*R*8 bytes per job"""
    return allreduce_counts(adj, group)


# --------------------------------------------------------------------------------------------
# Biofilm cell typing and the filtered adjacency (biofilm_analysis.py:1259-1295, row f4)
# --------------------------------------------------------------------------------------------
@dataclass
class CellTyping:
    is_cell: torch.Tensor          # (N,) u8 per cell row: 1 'cell', 0 'debris'
    debris_labels: torch.Tensor    # (maxlab + 1,) u8: labels overlapping the epithelial area
    adjacency: torch.Tensor        # (R, R) int64
    adjacency_filtered: torch.Tensor


def biofilm_typing_and_adjacency(segmentation: torch.Tensor, adjacency_seg: torch.Tensor, bc_idx: torch.Tensor,
                                 R: int, max_probability: torch.Tensor | None = None,
                                 epithelial_area: torch.Tensor | None = None, area_max: float = 10000.0,
                                 prob_min: float = 0.95) -> CellTyping:
    """cell rows = the labels of `segmentation` in ascending order (regionprops), bc_idx their
    barcode index in the (R, R) matrices (-1: not counted).  As the reference, row i stands for
    node i + 1 of the adjacency graph of `adjacency_seg` (:1285-1290 index cell_info by
    node - 1), so the labels are expected to be sequential."""
    seg = segmentation.to(torch.int32).contiguous()
    maxlab = int(seg.max().item()) if seg.numel() else 0
    props = K.region_props(seg, maxlab)
    present = props[1:, 7] > 0
    labels = (torch.nonzero(present).flatten() + 1).to(torch.int32)
    area = props[1:, 0][present].contiguous()
    overlap = None
    if epithelial_area is not None:
        overlap = K.label_overlap(seg, epithelial_area, maxlab)                       # :1259-1262
    is_cell = K.cell_typing(labels, area, max_probability, overlap, maxlab, area_max, prob_min)   # :1263-1269
    aseg = adjacency_seg.to(torch.int32).contiguous()
    amax = int(aseg.max().item()) if aseg.numel() else 0
    edge = K.rag_edges(aseg, amax)                                                    # :1277-1278
    n = labels.numel()
    bc = torch.full((amax + 1,), -1, dtype=torch.int32, device=seg.device)
    keep = torch.zeros(amax + 1, dtype=torch.uint8, device=seg.device)
    m = min(n, amax)
    bc[1:m + 1] = bc_idx[:m].to(torch.int32)
    keep[1:m + 1] = is_cell[:m]
    adj, adjf = K.barcode_adjacency_filtered(edge, bc, keep, R)                       # :1283-1295
    return CellTyping(is_cell, overlap if overlap is not None else torch.zeros(maxlab + 1, dtype=torch.uint8,
                                                                              device=seg.device), adj, adjf)
