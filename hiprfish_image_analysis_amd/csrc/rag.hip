// rag.hip -- label adjacency (a22).
//
// Reference: skimage.future.graph.rag_boundary(adjacency_seg, edge_map) followed by the
// barcode x barcode count loop (biofilm_analysis.py:1277-1295).  The RAG's edge set is, per
// pixel, (3x3 grey-erosion value, label) and (label, 3x3 grey-dilation value) where they
// differ (ndi reflect border == the in-image window for 3x3).  One pass marks those pairs
// in a dense (L x L) byte matrix (L = max label + 1); a second pass turns every marked
// undirected edge (a, b), a, b >= 1 into +1 at adj[bc[a]][bc[b]] and adj[bc[b]][bc[a]]
// (the reference visits each edge from both endpoints).
#include "common.hpp"

namespace {

__global__ void rag_mark_kernel(const int32_t *__restrict__ lab, int64_t H, int64_t W, int64_t L,
                                uint8_t *__restrict__ edge) {
  const int64_t n = H * W;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = p / W, c = p - r * W;
    const int32_t v = lab[p];
    int32_t mn = v, mx = v;
#pragma unroll
    for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
      for (int dc = -1; dc <= 1; ++dc) {
        const int64_t rr = r + dr, cc = c + dc;
        if (rr < 0 || rr >= H || cc < 0 || cc >= W) continue;
        const int32_t u = lab[rr * W + cc];
        mn = u < mn ? u : mn;
        mx = u > mx ? u : mx;
      }
    if (mn != v && mn >= 0 && mn < L && v < L) edge[(int64_t)mn * L + v] = 1;
    if (mx != v && v >= 0 && mx < L) edge[(int64_t)v * L + mx] = 1;
  }
}

__global__ void rag_count_kernel(const uint8_t *__restrict__ edge, int64_t L, const int32_t *__restrict__ bc,
                                 int32_t R, unsigned long long *__restrict__ adj) {
  const int64_t n = L * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    if (!edge[e]) continue;
    const int64_t a = e / L, b = e - a * L;
    if (a < 1 || b <= a) continue;
    const int32_t ba = bc[a], bb = bc[b];
    if (ba < 0 || ba >= R || bb < 0 || bb >= R) continue;
    atomicAdd(&adj[(int64_t)ba * R + bb], 1ull);
    atomicAdd(&adj[(int64_t)bb * R + ba], 1ull);
  }
}

}  // namespace

extern "C" {

hrf_status hrf_rag_edges(const int32_t *labels, int64_t H, int64_t W, int32_t maxlab, uint8_t *edge,
                         hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && maxlab < 65536 && edge, "rag_edges: max label must be < 65536");
  const int64_t L = (int64_t)maxlab + 1;
  HRF_HIP(hipMemsetAsync(edge, 0, (size_t)(L * L), s));
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(labels, "rag_edges: null labels");
  rag_mark_kernel<<<hrf::stream_grid(H * W), 256, 0, s>>>(labels, H, W, L, edge);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_barcode_adjacency(const uint8_t *edge, int32_t maxlab, const int32_t *bc_of_label, int32_t R,
                                 int64_t *adj, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && R >= 1 && edge && bc_of_label && adj, "barcode_adjacency: bad arguments");
  const int64_t L = (int64_t)maxlab + 1;
  HRF_HIP(hipMemsetAsync(adj, 0, sizeof(int64_t) * (size_t)R * R, s));
  rag_count_kernel<<<hrf::stream_grid(L * L), 256, 0, s>>>(edge, L, bc_of_label, R, (unsigned long long *)adj);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
