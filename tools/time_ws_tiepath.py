import sys, time
sys.path.insert(0, ".")
import torch, bench
from hiprfish_image_analysis_amd import _lib
_lib.lib()
t = time.time()
print(bench._watershed_ties(torch.device("cuda", 0)))
print("total s", time.time() - t)
