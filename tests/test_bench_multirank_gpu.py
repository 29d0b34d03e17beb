"""bench.py's world > 1 path, run once on hardware: two ranks on the one leased GPU (gloo for the
collectives -- HRF_DIST_BACKEND), started as `bench.py --gpus 2` (bench.py launches
torch.distributed.run itself when WORLD_SIZE is unset; the driver's torchrun form runs the
same rank code).  Every rank processes its own tile (registration + calibration +
process_tile); the all-reduced per-barcode counts must equal one process's sum over the same
two tiles (collect_measurement_results.py:92-98).  No scaling figure comes from this test."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_two_ranks_counts(tmp_path):
    out = tmp_path / "counts.npy"
    env = dict(os.environ, HRF_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0", "--concurrent", "1", "--tiles", "1", "--no-extras",
           "--no-cpu-baseline", "--dump-counts", str(out)]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    import json
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 2
    got = np.load(out)

    # one process over the same two tiles (bench.py's tile generation for ranks 0 and 1)
    sys.path.insert(0, REPO)
    import bench
    from hiprfish_image_analysis_amd import pipeline as P
    from hiprfish_image_analysis_amd import synthetic as S
    ref = S.reference_library(bench.NBIT, S.ECOLI_BOUNDS)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, bench.NBIT)
    cal = S.flat_field(bench.H, bench.W)
    want = None
    for rank in (0, 1):
        seed = 20190101 + rank * 1000
        lay = S.cell_layout(bench.H, bench.W, S.default_ncells(bench.H, bench.W), lib.R, seed)
        truth, prof = S.render_truth(bench.H, bench.W, lay, with_profile=True)
        stack = S.render_stack(truth, lay, ref, seed=seed, profile=prof)
        # bench.py's per-cell metric: the gated channel_cosine_intensity (variant 1)
        res = P.process_tile(P.register_stack(S.laser_split(stack)), lib, calibration=cal, variant=1)
        c = res.counts.cpu().numpy()
        want = c if want is None else want + c
    assert got.sum() > 1000
    assert np.array_equal(got, want)
    assert rec["config"]["cells_counted"] == int(want.sum())
