import sys, ctypes
sys.path.insert(0, ".")
import numpy as np
import torch
from hiprfish_image_analysis_amd import _lib, kernels as K, pipeline as P, synthetic as S

def free():
    torch.cuda.synchronize(); torch.cuda.empty_cache()
    return torch.cuda.mem_get_info()[0] / 2**20
H = W = 512
print("start", free())
for i in range(6):
    h = ctypes.c_void_p()
    _lib.call("hrf_tile_ctx_create", H, W, ctypes.addressof(h))
    a = free()
    _lib.call("hrf_tile_ctx_destroy", h)
    print("raw ctx create/destroy", i, a, free())
ref = S.reference_library(10, S.ECOLI_BOUNDS)
lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
lay = S.cell_layout(H, W, S.default_ncells(H, W), ref.shape[0], 5)
truth, prof = S.render_truth(H, W, lay, with_profile=True)
lasers = S.laser_split(S.render_stack(truth, lay, ref, seed=5, device="cuda", profile=prof))
cal = S.flat_field(H, W)
P.process_tile_native(lasers, lib, calibration=cal, variant=1)
print("after first tile", free())
for i in range(40):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        P.process_tile_native(lasers, lib, calibration=cal, variant=1)
    s.synchronize()
    print("stream", i, hex(s.cuda_stream), "ctx", len(K._TILE_CTX), "free MiB %.0f" % free(),
          "torch reserved %.0f" % (torch.cuda.memory_reserved() / 2**20))
# the test's sequence: segment_ecoli_native on each fresh stream too, after release_contexts
cn = P.register_tile(lasers).image_cn
K.release_contexts()
print("released", free(), len(K._TILE_CTX), len(K._SEG_CTX))
for i in range(30):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        P.process_tile_native(lasers, lib, calibration=cal, variant=1)
        K.segment_ecoli_native(None, image_cn=cn)
    s.synchronize()
    print("B stream", i, hex(s.cuda_stream), "ctx", len(K._TILE_CTX), len(K._SEG_CTX), "free MiB %.0f" % free())
