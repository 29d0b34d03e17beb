"""Synthetic HiPR-FISH tiles for tests and bench.py.

The reference ships no images or classifier pickles, so every measurement uses synthetic
(H, W, C) stacks of the shape the reference pipelines consume:

* a barcode reference library: nbit fluorophores with Gaussian emission bands, each excited
  by its own laser and weakly by the next one (the structure of the excitation matrix in
  train_reference.py:1901-1904), summed over the barcode's set bits, max-normalised;
* rod-shaped elliptical cells (minor axis 18-30 px, major 40-80 px), each carrying a random
  barcode; pixel spectrum = a * dome * ref_r / mean(ref_r) * 0.3 + N(0, 0.02), a ~ U(0.5, 1),
  clipped at 0 -- the cell's total brightness does not depend on how many bits its barcode
  has, and the dome (1 at the centre, 0.6 at the rim) gives touching rods the intensity
  valley the reference's watershed on -log(sum) separates them by;
* background 0.01 + N(0, 0.005) so no line-profile window is flat.

Geometry comes from numpy (seeded); the stack is rendered on the device with torch.
"""
from __future__ import annotations

import numpy as np

ECOLI_BOUNDS = (0, 32, 55, 75, 89, 95)        # 405/488/514/561/633 nm (train_reference.py:1401)
MULTI_BOUNDS = (0, 23, 43, 57, 63)            # 488/514/561/633 nm (train_reference.py:1488)


def reference_library(nbit: int = 10, bounds=ECOLI_BOUNDS, sigma: float = 0.12) -> np.ndarray:
    """-> (2**nbit - 1, C) float32; row r is barcode r + 1 (binary code format(r+1, '0{nbit}b'))."""
    bounds = list(bounds)
    nl = len(bounds) - 1
    C = bounds[-1]
    # emission of fluorophore f in each channel, per laser segment
    u = np.zeros(C)
    seg = np.zeros(C, int)
    for l in range(nl):
        n = bounds[l + 1] - bounds[l]
        u[bounds[l]:bounds[l + 1]] = (np.arange(n) + 0.5) / n
        seg[bounds[l]:bounds[l + 1]] = l
    peaks = (np.arange(nbit) + 0.5) / nbit
    primary = (np.arange(nbit) * nl) // nbit
    exc = np.zeros((nl, nbit))
    exc[primary, np.arange(nbit)] = 1.0
    nxt = np.minimum(primary + 1, nl - 1)
    exc[nxt, np.arange(nbit)] = np.maximum(exc[nxt, np.arange(nbit)], 0.3)
    emis = np.exp(-((u[None, :] - peaks[:, None]) ** 2) / (2 * sigma ** 2)) * exc.T[:, seg]
    R = 2 ** nbit - 1
    codes = ((np.arange(1, R + 1)[:, None] >> np.arange(nbit - 1, -1, -1)[None, :]) & 1).astype(np.float64)
    spec = codes @ emis
    spec /= spec.max(axis=1, keepdims=True)
    return spec.astype(np.float32)


def cell_layout(H: int, W: int, ncells: int, R: int, seed: int = 20190101):
    """Random rod-shaped cells: arrays (cy, cx, a_major, b_minor, theta, barcode_index)."""
    rng = np.random.default_rng(seed)
    cy = rng.uniform(0, H, ncells)
    cx = rng.uniform(0, W, ncells)
    maj = rng.uniform(40, 80, ncells) / 2
    mnr = rng.uniform(18, 30, ncells) / 2
    th = rng.uniform(0, np.pi, ncells)
    bc = rng.integers(0, R, ncells)
    amp = rng.uniform(0.5, 1.0, ncells)
    return cy, cx, maj, mnr, th, bc, amp


def default_ncells(H: int, W: int) -> int:
    return max(1, int(round(1500 * H * W / (2048 * 2048))))


def render_truth(H: int, W: int, layout, with_profile: bool = False, max_overlap: float = 0.05):
    """Ground-truth cell index map (int32, 0 = background, i+1 = cell i), optionally with the
    per-pixel dome intensity profile (float32).  Cells are placed in order and a cell that
    would cover more than `max_overlap` of its area with earlier cells is dropped: cells in a
    FOV touch but do not stack, so clumps stay a few cells large."""
    cy, cx, maj, mnr, th, _, _ = layout
    lab = np.zeros((H, W), np.int32)
    prof = np.zeros((H, W), np.float32)
    for i in range(len(cy)):
        r = int(np.ceil(maj[i])) + 1
        r0, r1 = max(0, int(cy[i]) - r), min(H, int(cy[i]) + r + 1)
        c0, c1 = max(0, int(cx[i]) - r), min(W, int(cx[i]) + r + 1)
        if r0 >= r1 or c0 >= c1:
            continue
        yy, xx = np.mgrid[r0:r1, c0:c1]
        dy, dx = yy - cy[i], xx - cx[i]
        ct, st = np.cos(th[i]), np.sin(th[i])
        u = dx * ct + dy * st
        v = -dx * st + dy * ct
        rr = (u / maj[i]) ** 2 + (v / mnr[i]) ** 2
        inside = rr <= 1.0
        if np.count_nonzero(lab[r0:r1, c0:c1][inside]) > max_overlap * np.count_nonzero(inside):
            continue
        lab[r0:r1, c0:c1][inside] = i + 1
        prof[r0:r1, c0:c1][inside] = (1.0 - 0.4 * rr[inside]).astype(np.float32)
    return (lab, prof) if with_profile else lab


def render_stack(truth, layout, ref, seed: int = 0, device="cuda", noise=0.02, bg=0.01, bg_noise=0.005,
                 profile=None, level=0.3):
    """(H, W, C) float32 device stack: cell pixels a*dome*ref_r/mean(ref_r)*level + N(0, noise)
    clipped at 0, background bg + N(0, bg_noise) (clipped at 0)."""
    import torch
    _, _, _, _, _, bc, amp = layout
    H, W = truth.shape
    C = ref.shape[1]
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    t = torch.from_numpy(truth).to(device)
    refn = ref / ref.mean(axis=1, keepdims=True) * level
    refs = torch.from_numpy(refn.astype(np.float32)).to(device)
    cell_spec = torch.cat([torch.zeros(1, C, device=device),
                           torch.from_numpy(amp.astype(np.float32)).to(device)[:, None] *
                           refs[torch.from_numpy(bc).to(device).long()]], 0)
    stack = cell_spec[t.long()]
    if profile is not None:
        stack = stack * torch.from_numpy(profile).to(device)[..., None]
    fg = (t > 0)[..., None]
    n = torch.randn((H, W, C), generator=g, device=device, dtype=torch.float32)
    stack = torch.where(fg, stack + noise * n, bg + bg_noise * n)
    return stack.clamp_(min=0.0).contiguous()


def tile(H: int = 2048, W: int = 2048, nbit: int = 10, bounds=ECOLI_BOUNDS, seed: int = 20190101, device="cuda",
         ncells: int | None = None):
    """Convenience: (stack, truth, layout, ref) for one synthetic tile."""
    ref = reference_library(nbit, bounds)
    lay = cell_layout(H, W, ncells or default_ncells(H, W), ref.shape[0], seed)
    truth, prof = render_truth(H, W, lay, with_profile=True)
    stack = render_stack(truth, lay, ref, seed=seed, device=device, profile=prof)
    return stack, truth, lay, ref


def tie_tile(H: int = 256, W: int = 256, gap: int = 1, cell: int = 14, bright: float = 1.0, mid: float = 0.3,
             device="cuda"):
    """A registered (H, W, 95) stack whose E. coli watershed (ecoli measurement.py:113) makes
    decisions between equal-valued markers of different labels: pairs of equal, uniform cells
    (cell x cell, brightness `bright`, one spectrum) `gap` pixels apart inside a uniform halo of
    brightness `mid` (the rough mask, not the interior), so the seeds are whole cells of one value
    and the corridor pixels between a pair are reached in the same FIFO layer from both -- which
    cell's label they take is the heap layout's (skimage pops equal-valued age-0 markers in
    whatever order its binary heap holds them).  An odd gap makes such decisions."""
    import torch
    img = np.zeros((H, W), np.float64)
    y0 = 20
    while y0 + cell + 3 < H - 10:
        x0 = 20
        while x0 + 2 * cell + gap + 3 < W - 10:
            img[y0 - 3:y0 + cell + 3, x0 - 3:x0 + 2 * cell + gap + 3] = mid
            img[y0:y0 + cell, x0:x0 + cell] = bright
            img[y0:y0 + cell, x0 + cell + gap:x0 + 2 * cell + gap] = bright
            x0 += 2 * cell + gap + 20
        y0 += cell + 26
    spec = np.linspace(0.5, 1.5, 95)
    st = (img[:, :, None] * spec[None, None, :]).astype(np.float32)
    return torch.from_numpy(st).to(device).contiguous()


# the misregistration applied to each laser's channels by laser_split (E. coli lasers
# 405/488/514/561/633, ecoli measurement.py:45-70 estimates and undoes it)
LASER_SHIFTS = ((0, 0), (2, -1), (0, 3), (-1, 0), (1, 1))


def laser_split(stack, bounds=ECOLI_BOUNDS, shifts=LASER_SHIFTS):
    """The per-laser (H, W, C_l) acquisitions of a registered stack, laser l displaced by
    -shifts[l] (so registration recovers shifts[l]; the wrapped rows/columns fall outside the
    coverage mask)."""
    import torch
    out = []
    for k in range(len(bounds) - 1):
        dr, dc = shifts[k]
        out.append(torch.roll(stack[:, :, bounds[k]:bounds[k + 1]], shifts=(-dr, -dc), dims=(0, 1)).contiguous())
    return out


def flat_field(H: int, W: int, device="cuda"):
    """A smooth flat-field calibration image (H, W) f32 in [0.7, 1.0] (the reference divides
    channels 0..31 by its calibration image, ecoli measurement.py:33-38, :147-150)."""
    import torch
    y = torch.linspace(-1.0, 1.0, H, device=device)[:, None]
    x = torch.linspace(-1.0, 1.0, W, device=device)[None, :]
    return (1.0 - 0.3 * (0.6 * y * y + 0.4 * x * x)).to(torch.float32).contiguous()


COMMUNITY_SHIFTS = ((0, 0), (3, -2), (-1, 4), (2, 1))   # 488, 514, 561, 633 (multispecies :79-84)


def calibration_stack(H: int, W: int, C: int, device="cuda"):
    """A (H, W, C) f32 calibration array for the community stage (multispecies :103-104 divides the
    registered stack by the loaded calibration image with numpy broadcasting): the flat field
    times a smooth per-channel gain in [0.8, 1.2]."""
    import torch
    g = 1.0 + 0.2 * torch.sin(torch.arange(C, device=device, dtype=torch.float32) * 0.37)
    return (flat_field(H, W, device)[:, :, None] * g[None, None, :]).to(torch.float32).contiguous()
