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

// raw and "cell"-filtered counts in one pass (biofilm :1290-1291: the filtered matrix counts an
// edge only when both endpoint rows are typed 'cell')
__global__ void rag_count2_kernel(const uint8_t *__restrict__ edge, int64_t L, const int32_t *__restrict__ bc,
                                  const uint8_t *__restrict__ keep, int32_t R, unsigned long long *__restrict__ adj,
                                  unsigned long long *__restrict__ adjf) {
  const int64_t n = L * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    if (!edge[e]) continue;
    const int64_t a = e / L, b = e - a * L;
    if (a < 1 || b <= a) continue;
    const int32_t ba = bc[a], bb = bc[b];
    if (ba < 0 || ba >= R || bb < 0 || bb >= R) continue;
    atomicAdd(&adj[(int64_t)ba * R + bb], 1ull);
    atomicAdd(&adj[(int64_t)bb * R + ba], 1ull);
    if (keep[a] && keep[b]) {
      atomicAdd(&adjf[(int64_t)ba * R + bb], 1ull);
      atomicAdd(&adjf[(int64_t)bb * R + ba], 1ull);
    }
  }
}

// labels with any pixel inside the mask (biofilm :1259-1262: debris = segmentation *
// image_epithelial_area; debris_labels = its non-zero values)
__global__ void label_overlap_kernel(const int32_t *__restrict__ lab, const uint8_t *__restrict__ mask, int64_t n,
                                     int32_t maxlab, uint8_t *__restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t v = lab[p];
    if (v > 0 && v <= maxlab && mask[p]) out[v] = 1;
  }
}

// biofilm :1263-1269: a row is debris when area > area_max, its label overlaps the epithelial
// area, or max_probability <= prob_min (a NaN probability compares false: stays a cell)
__global__ void cell_typing_kernel(const int32_t *__restrict__ label, const double *__restrict__ area,
                                   const double *__restrict__ maxprob, const uint8_t *__restrict__ overlap,
                                   int32_t maxlab, int64_t n, double area_max, double prob_min,
                                   uint8_t *__restrict__ is_cell) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t l = label[i];
  const bool over = overlap && l > 0 && l <= maxlab && overlap[l];
  is_cell[i] = !((area[i] > area_max) || over || (maxprob && maxprob[i] <= prob_min));
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

hrf_status hrf_barcode_adjacency_filtered(const uint8_t *edge, int32_t maxlab, const int32_t *bc_of_label,
                                          const uint8_t *keep_of_label, int32_t R, int64_t *adj, int64_t *adj_filtered,
                                          hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && R >= 1 && edge && bc_of_label && keep_of_label && adj && adj_filtered,
              "barcode_adjacency_filtered: bad arguments");
  const int64_t L = (int64_t)maxlab + 1;
  HRF_HIP(hipMemsetAsync(adj, 0, sizeof(int64_t) * (size_t)R * R, s));
  HRF_HIP(hipMemsetAsync(adj_filtered, 0, sizeof(int64_t) * (size_t)R * R, s));
  rag_count2_kernel<<<hrf::stream_grid(L * L), 256, 0, s>>>(edge, L, bc_of_label, keep_of_label, R,
                                                             (unsigned long long *)adj,
                                                             (unsigned long long *)adj_filtered);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_label_overlap(const int32_t *labels, const uint8_t *mask, int64_t H, int64_t W, int32_t maxlab,
                             uint8_t *out, hrf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  HRF_REQUIRE(maxlab >= 0 && out, "label_overlap: bad arguments");
  HRF_HIP(hipMemsetAsync(out, 0, (size_t)maxlab + 1, s));
  if (H * W == 0) return HRF_OK;
  HRF_REQUIRE(labels && mask, "label_overlap: null buffer");
  label_overlap_kernel<<<hrf::stream_grid(H * W), 256, 0, s>>>(labels, mask, H * W, maxlab, out);
  HRF_LAUNCHED();
  return HRF_OK;
}

hrf_status hrf_cell_typing(const int32_t *label, const double *area, const double *maxprob, const uint8_t *overlap,
                           int32_t maxlab, int64_t n, double area_max, double prob_min, uint8_t *is_cell,
                           hrf_stream_t stream) {
  if (n == 0) return HRF_OK;
  HRF_REQUIRE(label && area && is_cell, "cell_typing: null buffer");
  cell_typing_kernel<<<(unsigned)hrf::cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(
      label, area, maxprob, overlap, maxlab, n, area_max, prob_min, is_cell);
  HRF_LAUNCHED();
  return HRF_OK;
}

}  // extern "C"
