// chainops.hip -- clears and host read-backs of the native chains as one kernel (common.hpp
// ZeroPub).  A hipMemsetAsync or a small hipMemcpyAsync to pinned memory is a rocclr fill or copy
// kernel of its own; the chains instead fold them into one launch at the points where they
// synchronise anyway (component boxes, watershed batches, erosion seeding).
#include "common.hpp"

namespace {

struct ZeroPubArgs {
  int nz, np;
  uint32_t *zp[hrf::ZeroPub::N];
  int64_t zoff[hrf::ZeroPub::N + 1];  // prefix sums of the word counts
  const int32_t *ps[hrf::ZeroPub::N];
  int32_t *pd[hrf::ZeroPub::N];
  int32_t poff[hrf::ZeroPub::N + 1];
};

__global__ __launch_bounds__(256) void zero_publish_kernel(ZeroPubArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = i0; i < a.zoff[a.nz]; i += stride) {
    int k = 0;
    while (i >= a.zoff[k + 1]) ++k;
    a.zp[k][i - a.zoff[k]] = 0u;
  }
  for (int64_t i = i0; i < a.poff[a.np]; i += stride) {
    int k = 0;
    while (i >= a.poff[k + 1]) ++k;
    const int64_t j = i - a.poff[k];
    // pinned, coherent host memory: a plain vector store, visible once the stream completes
    a.pd[k][j] = a.ps[k][j];
  }
}

}  // namespace

namespace hrf {

hrf_status zero_publish(const ZeroPub &z, hipStream_t s) {
  if (z.nz == 0 && z.np == 0) return HRF_OK;
  ZeroPubArgs a{};
  a.nz = z.nz;
  a.np = z.np;
  a.zoff[0] = 0;
  for (int k = 0; k < z.nz; ++k) {
    a.zp[k] = (uint32_t *)z.zp[k];
    a.zoff[k + 1] = a.zoff[k] + z.zw[k];
  }
  a.poff[0] = 0;
  for (int k = 0; k < z.np; ++k) {
    a.ps[k] = z.ps[k];
    a.pd[k] = z.pd[k];
    a.poff[k + 1] = a.poff[k] + z.pn[k];
  }
  const int64_t work = a.zoff[a.nz] > a.poff[a.np] ? a.zoff[a.nz] : (int64_t)a.poff[a.np];
  zero_publish_kernel<<<stream_grid(work), 256, 0, s>>>(a);
  HRF_LAUNCHED();
  return HRF_OK;
}

int32_t *mapped(int32_t *host) {
  if (!host) return nullptr;
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return nullptr;
  return (int32_t *)d;
}

hipError_t host_alloc_mapped(void **p, size_t bytes) {
  return hipHostMalloc(p, bytes, hipHostMallocMapped | hipHostMallocCoherent);
}

}  // namespace hrf
