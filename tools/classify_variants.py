"""Per-pixel classifier variants on one resident 2048x2048x95 synthetic tile (R = 1023): mean
launch time (HIP events) and agreement with the lay16 kernel's output.  One process per
variant (the kernel choice is read from HRF_CLASSIFY_W16 once per process).

python tools/classify_variants.py [cfg ...]      cfg: "0" (lay16) or "NW,NBUF,CR"
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg, out):
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    from hiprfish_image_analysis_amd import kernels as K, synthetic as S
    st, _, _, ref = S.tile(2048, 2048, seed=20190101)
    refx = K.classify_prepare(torch.from_numpy(ref).cuda(), S.ECOLI_BOUNDS)
    R = ref.shape[0]
    for _ in range(2):
        idx, dist = K.classify_pixels(st, refx, R, S.ECOLI_BOUNDS)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        K.classify_pixels(st, refx, R, S.ECOLI_BOUNDS)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    np.save(out, np.stack([idx.cpu().numpy().astype(np.float64).ravel(), dist.cpu().numpy().astype(np.float64).ravel()]))
    print(json.dumps({"cfg": cfg, "ms": round(ms, 4), "tflops_alg": round(2.0 * 2048 * 2048 * R * 95 / ms / 1e9, 1)}))


def main():
    import numpy as np
    cfgs = sys.argv[1:] or ["0", "4,2,64"]
    base = None
    for cfg in cfgs:
        out = "/tmp/cv_%s.npy" % cfg.replace(",", "_")
        env = dict(os.environ, HRF_CLASSIFY_W16=cfg)
        r = subprocess.run([sys.executable, __file__, "--child", cfg, out], env=env, capture_output=True, text=True,
                           timeout=300)
        if r.returncode != 0:
            print(cfg, "FAILED", r.stderr[-2000:])
            sys.exit(1)
        rec = json.loads(r.stdout.strip().splitlines()[-1])
        a = np.load(out)
        if base is None:
            base = a
        rec["idx_agree"] = float((a[0] == base[0]).mean())
        rec["dist_maxdiff"] = float(np.abs(a[1] - base[1]).max())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
    else:
        main()
