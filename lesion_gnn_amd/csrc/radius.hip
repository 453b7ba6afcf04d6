// Radius graph construction on the GPU for a batch of graphs: torch_cluster.radius_graph(pos, r,
// batch, loop, max_num_neighbors, flow='source_to_target') as PyG 2.5.1's RadiusGraph transform
// calls it — the connectivity the reference's sweep offers beside KNNGraph
// (src/lesion_gnn/scripts/sweep.py:113-118: RadiusGraph(r), r in [1, 1536] pixels; transforms.py:19-23
// resolves it by name). torch_cluster is not under /root/reference; its published algorithm
// (1.6.3, radius_cuda.cu + radius.py) is restated here:
//   radius_graph: limit = loop ? max_num_neighbors : max_num_neighbors + 1; radius(x, x, r, ...)
//   radius:       for every query q of graph g, walk the candidates c of g in INDEX order and take
//                 c when |p_q - p_c|^2 < r * r (strict), stopping once `limit` are taken
//   radius_graph: edge_index = [c, q] (source_to_target), and without `loop` the self pair is
//                 removed afterwards — so a query whose first `limit` in-range candidates do not
//                 include itself keeps max_num_neighbors + 1 neighbours, as torch_cluster does.
// The neighbour choice when more than `limit` candidates are in range is torch_cluster's CUDA
// one (the first `limit` in index order); its CPU path (nanoflann, unsorted radius search) keeps
// a traversal-dependent subset — documented, parity unpinned there (oracle/pyg_ref.py).
// Squared distances: fp64 dx*dx + dy*dy (+ dz*dz) with each operation rounded on its own, the
// arithmetic of the oracle's restatement ((p_q - p_c)**2).sum(-1), so edge lists are bit-exact.
//
// Two passes with one host read between them (the edge count sizes the output):
//   lgnn_radius_count:  per-query neighbour counts, then their exclusive scan (int64 offsets in
//                       the workspace; offsets[N] = the edge count);
//   lgnn_radius_graph:  the same walk again, each query writing its edges at offsets[q].
// Layout: pos [N][D] fp64 (D = 2 or 3), ptr [B+1] int32 graph offsets (Batch.ptr), batch [N]
// int64 sorted. One thread per query; a block's queries are consecutive nodes, so the candidates
// of its graphs are one contiguous node range, staged through LDS in chunks (as k_knn).
#include "common.h"

namespace {

constexpr int QT = 256;      // queries (threads) per block
constexpr int CHUNK = 1024;  // candidates staged per round
constexpr int ST = 1024;     // scan threads

__device__ __forceinline__ double sqd(const double* a, const double* b, int D) {
#pragma clang fp contract(off)
  const double dx = a[0] - b[0], dy = a[1] - b[1];
  double s = dx * dx + dy * dy;
  if (D == 3) {
    const double dz = a[2] - b[2];
    s = s + dz * dz;
  }
  return s;
}

// WRITE = false: cnt[q] = the query's edge count; WRITE = true: its edges at off[q]
template <int D, bool WRITE>
__global__ __launch_bounds__(QT) void k_radius(const double* __restrict__ pos, int64_t N,
                                               const int64_t* __restrict__ batch,
                                               const int32_t* __restrict__ ptr, double r2,
                                               int limit, int loop, int32_t* __restrict__ cnt,
                                               const int64_t* __restrict__ off, int64_t E,
                                               int64_t* __restrict__ ei) {
  __shared__ double cp[CHUNK * D];
  const int64_t q0 = (int64_t)blockIdx.x * QT;
  const int64_t q = q0 + threadIdx.x;
  const int64_t qlast = q0 + QT - 1 < N - 1 ? q0 + QT - 1 : N - 1;
  const int64_t cbeg = ptr[batch[q0]], cend = ptr[batch[qlast] + 1];
  const bool active = q < N;
  int64_t gs = 0, ge = 0;
  double pq[D];
  if (active) {
    const int64_t g = batch[q];
    gs = ptr[g];
    ge = ptr[g + 1];
#pragma unroll
    for (int d = 0; d < D; ++d) pq[d] = pos[q * D + d];
  }
  int taken = 0;    // candidates taken by the walk (self included), <= limit
  int64_t w = 0;    // edges written (WRITE)
  const int64_t base = WRITE && active ? off[q] : 0;
  for (int64_t c0 = cbeg; c0 < cend; c0 += CHUNK) {
    const int64_t c1 = c0 + CHUNK < cend ? c0 + CHUNK : cend;
    // every query of the block has taken `limit` candidates, or its graph ends before this
    // chunk: the rest of the range cannot add an edge (block-uniform, so the barriers stay so)
    if (!__syncthreads_or(active && taken < limit && ge > c0)) break;
    for (int64_t i = c0 * D + threadIdx.x; i < c1 * D; i += QT) cp[i - c0 * D] = pos[i];
    __syncthreads();
    if (!active || taken >= limit) continue;
    const int64_t lo = gs > c0 ? gs : c0, hi = ge < c1 ? ge : c1;
    for (int64_t c = lo; c < hi && taken < limit; ++c) {
      if (sqd(pq, cp + (c - c0) * D, D) < r2) {
        ++taken;
        if (!loop && c == q) continue;  // removed by radius_graph after the walk
        if constexpr (WRITE) {
          if (base + w < E) {  // E = offsets[N] (lgnn_radius_count); a short buffer is not overrun
            ei[base + w] = c;
            ei[E + base + w] = q;
          }
        }
        ++w;
      }
    }
  }
  if constexpr (!WRITE) {
    if (active) cnt[q] = (int32_t)w;
  }
}

// off[i] = sum_{j < i} cnt[j], off[N] = total: one block, each thread a contiguous range
__global__ __launch_bounds__(ST) void k_radius_scan(const int32_t* __restrict__ cnt, int64_t N,
                                                    int64_t* __restrict__ off) {
  __shared__ int64_t part[ST];
  const int t = threadIdx.x;
  const int64_t per = (N + ST - 1) / ST;
  const int64_t i0 = t * per < N ? t * per : N, i1 = i0 + per < N ? i0 + per : N;
  int64_t s = 0;
  for (int64_t i = i0; i < i1; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    int64_t run = 0;
    for (int i = 0; i < ST; ++i) {
      const int64_t v = part[i];
      part[i] = run;
      run += v;
    }
    off[N] = run;
  }
  __syncthreads();
  int64_t run = part[t];
  for (int64_t i = i0; i < i1; ++i) {
    off[i] = run;
    run += cnt[i];
  }
}

struct RadiusWs {
  int64_t* off;  // [N + 1]
  int32_t* cnt;  // [N]
};

RadiusWs radius_ws(void* ws, int64_t N) {
  RadiusWs r;
  r.off = static_cast<int64_t*>(ws);
  r.cnt = reinterpret_cast<int32_t*>(r.off + N + 1);
  return r;
}

int radius_args_ok(const double* pos, int64_t N, int dims, const int64_t* batch,
                   const int32_t* ptr, int64_t B, double r, int max_num_neighbors) {
  if (N < 0 || B < 0 || (dims != 2 && dims != 3) || !(r >= 0.0) || max_num_neighbors < 1)
    return 0;
  if (N > 0 && (!pos || !batch || !ptr)) return 0;
  if (N > 0 && B == 0) return 0;  // nodes but no graphs: batch cannot index ptr
  if (N > INT32_MAX) return 0;
  return 1;
}

}  // namespace

extern "C" size_t lgnn_radius_workspace_bytes(int64_t num_nodes) {
  if (num_nodes < 0) return 0;
  return (size_t)(num_nodes + 1) * sizeof(int64_t) + (size_t)num_nodes * sizeof(int32_t);
}

extern "C" int lgnn_radius_count(const double* pos, int64_t N, int dims, const int64_t* batch,
                                 const int32_t* ptr, int64_t B, double r, int max_num_neighbors,
                                 int loop, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  if (!radius_args_ok(pos, N, dims, batch, ptr, B, r, max_num_neighbors)) return LGNN_EINVAL;
  if (!workspace || workspace_bytes < lgnn_radius_workspace_bytes(N)) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const RadiusWs w = radius_ws(workspace, N);
  if (N == 0) {
    if (hipMemsetAsync(w.off, 0, sizeof(int64_t), s) != hipSuccess) return (int)hipGetLastError();
    return LGNN_OK;
  }
  const double r2 = r * r;  // torch_cluster squares r on the host, in double
  const int limit = loop ? max_num_neighbors : max_num_neighbors + 1;
  const dim3 grid((unsigned)((N + QT - 1) / QT));
  if (dims == 2)
    hipLaunchKernelGGL((k_radius<2, false>), grid, dim3(QT), 0, s, pos, N, batch, ptr, r2, limit,
                       loop, w.cnt, nullptr, 0, nullptr);
  else
    hipLaunchKernelGGL((k_radius<3, false>), grid, dim3(QT), 0, s, pos, N, batch, ptr, r2, limit,
                       loop, w.cnt, nullptr, 0, nullptr);
  LGNN_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_radius_scan, dim3(1), dim3(ST), 0, s, w.cnt, N, w.off);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_radius_graph(const double* pos, int64_t N, int dims, const int64_t* batch,
                                 const int32_t* ptr, int64_t B, double r, int max_num_neighbors,
                                 int loop, int64_t* edge_index, int64_t num_edges,
                                 const void* workspace, size_t workspace_bytes, void* stream) {
  if (!radius_args_ok(pos, N, dims, batch, ptr, B, r, max_num_neighbors)) return LGNN_EINVAL;
  if (num_edges < 0 || (num_edges > 0 && !edge_index)) return LGNN_EINVAL;
  if (!workspace || workspace_bytes < lgnn_radius_workspace_bytes(N)) return LGNN_ENOSPC;
  if (N == 0 || num_edges == 0) return LGNN_OK;
  hipStream_t s = as_stream(stream);
  const RadiusWs w = radius_ws(const_cast<void*>(workspace), N);
  const double r2 = r * r;
  const int limit = loop ? max_num_neighbors : max_num_neighbors + 1;
  const dim3 grid((unsigned)((N + QT - 1) / QT));
  if (dims == 2)
    hipLaunchKernelGGL((k_radius<2, true>), grid, dim3(QT), 0, s, pos, N, batch, ptr, r2, limit,
                       loop, nullptr, w.off, num_edges, edge_index);
  else
    hipLaunchKernelGGL((k_radius<3, true>), grid, dim3(QT), 0, s, pos, N, batch, ptr, r2, limit,
                       loop, nullptr, w.off, num_edges, edge_index);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
