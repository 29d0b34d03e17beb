"""hiprfish_image_analysis_amd -- MI355X-native HiPR-FISH spectral measurement + barcode
classification hot path.  Device kernels live in libhrf.so (csrc/, C ABI in
include/hrf.h); this package is the host side mirroring the reference's scripts."""
__version__ = "0.1.0"
