// bw_probe.hip -- achievable HBM rates on this box for the shapes the path uses (dev tool):
// a float4 read-reduce and a float4 copy over 1.6 GB (one 2048x2048x95 f32 stack), grid-stride,
// several grid sizes.  hipcc --offload-arch=gfx950 -O3 -o /tmp/bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int U>
__global__ __launch_bounds__(256) void read_kernel(const float4 *__restrict__ a, long n, float *__restrict__ out) {
  float s = 0.f;
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * 256 < n ? a[i + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int U>
__global__ __launch_bounds__(256) void copy_kernel(const float4 *__restrict__ a, long n, float4 *__restrict__ b) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < n) v[u] = a[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < n) b[i + u * 256] = v[u];
  }
}

int main() {
  const long bytes = 2048L * 2048 * 95 * 4;
  const long n = bytes / 16;
  float4 *a, *b;
  float *o;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&o, 4096));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (int g : grids) {
    for (int k = 0; k < 2; ++k) {
      auto run = [&](int which) {
        if (which == 0) read_kernel<4><<<g, 256>>>(a, n, o);
        else if (which == 1) read_kernel<8><<<g, 256>>>(a, n, o);
        else copy_kernel<4><<<g, 256>>>(a, n, b);
      };
      for (int which = 0; which < 3; ++which) {
        run(which);
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) run(which);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 10;
        const double moved = which == 2 ? 2.0 * bytes : (double)bytes;
        if (k == 1)
          printf("%-8s grid %5d  %.4f ms  %.2f TB/s\n", which == 0 ? "read4" : which == 1 ? "read8" : "copy4", g, ms,
                 moved / ms / 1e9);
      }
    }
  }
  return 0;
}
