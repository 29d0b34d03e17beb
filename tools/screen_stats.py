"""How sparse would a screened per-pixel classifier's correction work be?  On one bench tile's
rows 1000-1015 (CPU, f64): per pixel, the library rows whose exact segmented-cosine score lies
within 2 delta of the best (the rows a screen with margin delta must finish), and the fraction of
(16-pixel group, 16-row block) and (64-pixel wave, 16-row block) tiles holding one -- the blocks
that would need the hi x lo / lo x hi products even with the final best known in advance
(DESIGN.md "Tried and not kept (round 5)").  usage: python tools/screen_stats.py"""
import sys, numpy as np, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench as B
from hiprfish_image_analysis_amd import synthetic as S
ref = S.reference_library(B.NBIT, S.ECOLI_BOUNDS).astype(np.float64)
H = W = 2048
lay = S.cell_layout(H, W, S.default_ncells(H, W), ref.shape[0], 20190101)
truth, prof = S.render_truth(H, W, lay, with_profile=True)
stack = S.render_stack(truth, lay, ref.astype(np.float32), seed=20190101, device="cpu", profile=prof)
x = stack[1000:1016].reshape(-1, 95).numpy().astype(np.float64)   # 16 rows x 2048
b = S.ECOLI_BOUNDS
def segnorm(a):
    a = a.copy()
    for s in range(5):
        n = np.sqrt((a[:, b[s]:b[s+1]]**2).sum(1, keepdims=True)); n[n == 0] = 1
        a[:, b[s]:b[s+1]] /= n
    return a
xn, yn = segnorm(x), segnorm(ref)
Sx = xn @ yn.T                         # exact scores (pixels x refs)
xh = xn.astype(np.float16).astype(np.float64); yh = yn.astype(np.float16).astype(np.float64)
St = xh @ yh.T
print("max |St - S|", np.abs(St - Sx).max())
best = Sx.max(1)
for d in (0.0078125, 0.004, 0.002):
    cand = Sx >= best[:, None] - 2 * d
    print("delta %.4f: candidates per pixel mean %.2f  p99 %d" % (d, cand.sum(1).mean(), np.percentile(cand.sum(1), 99)))
    R = cand.shape[1]; Rp = 1024
    c = np.zeros((cand.shape[0], Rp), bool); c[:, :R] = cand
    # group = 16 consecutive pixels, block = 16 refs
    g = c.reshape(-1, 16, Rp // 16, 16).any(axis=(1, 3))
    print("   group-block hot frac (ideal floor): %.3f" % g.mean())
    w = c.reshape(-1, 64, Rp // 16, 16).any(axis=(1, 3))
    print("   wave-block hot frac (ideal floor): %.3f" % w.mean())
