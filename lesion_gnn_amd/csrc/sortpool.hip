// SortAggregation (PyG 2.5.1, DGCNN sort pooling) forward and backward for gfx950.
// Reference: src/lesion_gnn/models/drgnet.py:37 (SortAggregation(sortpool_k)), called at :59 on
// the concatenated GraphConv outputs. Semantics restated in oracle/pyg_ref.py:sort_aggregation:
//   fill = min(x) - 1; per graph, rows sorted by the LAST channel descending (ties: node order),
//   first k rows kept, missing rows = fill; every element equal to fill -> 0; out [B, k * D].
//
// Forward: k_min_partials (grid-stride min over x, one partial per block) + k_sort_pool (one
// workgroup per graph): each workgroup folds the partials into `fill`, ranks its graph's keys by
// counting (rank_i = #{j : key_j > key_i or (key_j == key_i and j < i)} — a stable descending
// order, deterministic, no sort network), records the node of every rank < k in LDS and writes
// the k output rows (coalesced over the D channels). It also stores rank[i] (or -1) per node for
// the backward, which is then a pure per-element map: dx[i, d] = dout[g(i), rank[i], d] unless
// rank[i] < 0 or x[i, d] == fill (the masked_fill of the forward).
//
// Bound: HBM (reads x once for the min, k rows per graph + its keys; writes B*k*D + M ints).
// The key ranking is O(n_g^2) LDS compares per graph (n_g <= 512 for lesion graphs: 1k compares
// per thread), not on the critical path at these sizes.
#include "common.h"

namespace lgnn_sortpool {

constexpr int kThreads = 256;
constexpr int kMinBlocks = 256;
constexpr int kKeyChunk = 2048;
constexpr int kMaxK = 4096;

__device__ __forceinline__ float wave_min(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ void __launch_bounds__(kThreads) k_min_partials(const float* __restrict__ x,
                                                           int64_t n, float* __restrict__ part) {
  __shared__ float red[kThreads / 64];
  float m = __builtin_inff();
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads)
    m = fminf(m, x[i]);
  m = wave_min(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int w = 1; w < kThreads / 64; ++w) r = fminf(r, red[w]);
    part[blockIdx.x] = r;
  }
}

__global__ void __launch_bounds__(kThreads)
    k_sort_pool(const float* __restrict__ x, int D, const int32_t* __restrict__ gptr, int k,
                const float* __restrict__ part, int nparts, float* __restrict__ out,
                int32_t* __restrict__ rank, float* __restrict__ fill_out) {
  __shared__ float keys[kKeyChunk];
  __shared__ int32_t slot[kMaxK];
  __shared__ float red[kThreads / 64];
  const int g = blockIdx.x;
  const int tid = threadIdx.x;

  // fill = min(x) - 1 from the per-block partials (every workgroup folds the same values in the
  // same order, so all agree bit for bit)
  float m = tid < nparts ? part[tid] : __builtin_inff();
  m = wave_min(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  for (int i = tid; i < k; i += kThreads) slot[i] = -1;
  __syncthreads();
  float mn = red[0];
  for (int w = 1; w < kThreads / 64; ++w) mn = fminf(mn, red[w]);
  const float fill = mn - 1.f;
  if (g == 0 && tid == 0 && fill_out) fill_out[0] = fill;

  const int start = gptr[g];
  const int n = gptr[g + 1] - start;
  const float* xg = x + (int64_t)start * D;
  for (int i0 = 0; i0 < n; i0 += kThreads) {
    const int i = i0 + tid;
    const float ki = i < n ? xg[(int64_t)i * D + (D - 1)] : 0.f;
    int r = 0;
    for (int j0 = 0; j0 < n; j0 += kKeyChunk) {
      const int cnt = min(kKeyChunk, n - j0);
      __syncthreads();
      for (int j = tid; j < cnt; j += kThreads) keys[j] = xg[(int64_t)(j0 + j) * D + (D - 1)];
      __syncthreads();
      if (i < n) {
        for (int j = 0; j < cnt; ++j) {
          const float kj = keys[j];
          r += (kj > ki) | ((kj == ki) & (j0 + j < i));
        }
      }
    }
    if (i < n) {
      rank[start + i] = r < k ? r : -1;
      if (r < k) slot[r] = i;
    }
  }
  __syncthreads();

  float* og = out + (int64_t)g * k * D;
  const int64_t total = (int64_t)k * D;
  for (int64_t e = tid; e < total; e += kThreads) {
    const int r = (int)(e / D);
    const int d = (int)(e - (int64_t)r * D);
    const int node = slot[r];
    float v = node >= 0 ? xg[(int64_t)node * D + d] : 0.f;
    og[e] = (v == fill) ? 0.f : v;
  }
}

__global__ void __launch_bounds__(kThreads)
    k_sort_pool_bwd(const float* __restrict__ dout, const float* __restrict__ x,
                    const int32_t* __restrict__ rank, const int64_t* __restrict__ batch,
                    const float* __restrict__ fill, int64_t M, int D, int k,
                    float* __restrict__ dx) {
  const float f = fill[0];
  const int64_t total = M * D;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * kThreads) {
    const int64_t i = e / D;
    const int d = (int)(e - i * D);
    const int r = rank[i];
    float v = 0.f;
    if (r >= 0 && x[e] != f) v = dout[(batch[i] * k + r) * D + d];
    dx[e] = v;
  }
}

}  // namespace lgnn_sortpool

using namespace lgnn_sortpool;

extern "C" size_t lgnn_sort_pool_workspace_bytes(void) { return kMinBlocks * sizeof(float); }

extern "C" int lgnn_sort_pool_fwd(const float* x, int64_t num_nodes, int dims,
                                  const int32_t* gptr, int64_t num_graphs, int k, float* out,
                                  int32_t* rank, float* fill, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (num_nodes < 0 || dims <= 0 || num_graphs < 0 || k <= 0 || k > kMaxK)
    return LGNN_EINVAL;
  if (workspace_bytes < lgnn_sort_pool_workspace_bytes() || !x || !gptr || !out || !rank ||
      !fill || !workspace)
    return LGNN_EINVAL;
  if (num_graphs == 0) return LGNN_OK;
  hipStream_t s = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  const int64_t n = num_nodes * dims;
  const int blocks = (int)std::min<int64_t>(kMinBlocks, std::max<int64_t>(1, (n + kThreads - 1) / kThreads));
  hipLaunchKernelGGL(k_min_partials, dim3(blocks), dim3(kThreads), 0, s, x, n, part);
  LGNN_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sort_pool, dim3((unsigned)num_graphs), dim3(kThreads), 0, s, x, dims, gptr,
                     k, part, blocks, out, rank, fill);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_sort_pool_bwd(const float* dout, const float* x, const int32_t* rank,
                                  const int64_t* batch, const float* fill, int64_t num_nodes,
                                  int dims, int k, float* dx, void* stream) {
  if (num_nodes < 0 || dims <= 0 || k <= 0 || k > kMaxK) return LGNN_EINVAL;
  if (num_nodes == 0) return LGNN_OK;
  if (!dout || !x || !rank || !batch || !fill || !dx) return LGNN_EINVAL;
  const int64_t total = num_nodes * dims;
  const int blocks = (int)std::min<int64_t>(4096, (total + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(k_sort_pool_bwd, dim3(blocks), dim3(kThreads), 0, as_stream(stream), dout,
                     x, rank, batch, fill, num_nodes, dims, k, dx);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
