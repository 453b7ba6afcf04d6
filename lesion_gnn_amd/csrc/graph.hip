// Graph-structure kernels: edge_index (int64 COO, any order) -> CSR by target + CSR by source,
// with PyG 2.5.1 self-loop semantics and GCN normalisation; Batch.ptr from `batch`.
//
// Replaces (reference call sites): gcn_norm inside GCNConv, GATConv's
// remove_self_loops/add_self_loops (gat.py:31), ToSparseTensor (datasets/datamodule.py:44-45).
//
// Determinism: slots are claimed with integer atomics (order varies), then every row is sorted by
// original edge id, so the final CSR is identical run to run and keeps edge_index order inside a
// row — the order PyG's scatter_add_ visits a target's messages in.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

constexpr int kThreads = 256;

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

struct GraphWs {
  int32_t* cnt;    // [N+1] non-loop in-degree, then scanned in place -> rowptr source
  int32_t* tcnt;   // [N+1]
  int32_t* fill;   // [N]
  int32_t* tfill;  // [N]
  int32_t* loopc;  // [N] number of self pairs seen per node (LOOPS_KEEP ignores)
  int32_t* eid;    // [E+N]
  int32_t* teid;   // [E+N]
  void* scan_tmp;
  size_t scan_bytes;
};

size_t scan_temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  return bytes;
}

GraphWs carve(void* base, int64_t N, int64_t E) {
  GraphWs ws;
  char* p = static_cast<char*>(base);
  auto take = [&](size_t bytes) {
    char* q = p;
    p += align_up(bytes);
    return q;
  };
  ws.cnt = (int32_t*)take((N + 1) * 4);
  ws.tcnt = (int32_t*)take((N + 1) * 4);
  ws.fill = (int32_t*)take(N * 4);
  ws.tfill = (int32_t*)take(N * 4);
  ws.loopc = (int32_t*)take(N * 4);
  ws.eid = (int32_t*)take((E + N) * 4);
  ws.teid = (int32_t*)take((E + N) * 4);
  ws.scan_bytes = scan_temp_bytes(N + 1);
  ws.scan_tmp = take(ws.scan_bytes);
  return ws;
}

size_t ws_total(int64_t N, int64_t E) {
  return 2 * align_up((N + 1) * 4) + 3 * align_up(N * 4) + 2 * align_up((E + N) * 4) +
         align_up(scan_temp_bytes(N + 1)) + 256;
}

__global__ void k_count(const int64_t* __restrict__ ei, int64_t E, int64_t N, int loops,
                        int32_t* cnt, int32_t* tcnt, int32_t* loopc, int32_t* err) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = ei[e], d = ei[E + e];
    if (s < 0 || s >= N || d < 0 || d >= N) {
      if (err) atomicAdd(err, 1);
      continue;
    }
    if (loops != LGNN_LOOPS_KEEP && s == d) {
      atomicAdd(&loopc[d], 1);
      continue;
    }
    atomicAdd(&cnt[d], 1);
    if (tcnt) atomicAdd(&tcnt[s], 1);
  }
}

// cnt[i] += add_loop (one appended loop per node); cnt[N] = 0 so the exclusive scan of N+1
// entries ends with the total.
__global__ void k_add_loops(int32_t* cnt, int32_t* tcnt, int64_t N, int add_loop) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= N;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i == N) {
      cnt[i] = 0;
      if (tcnt) tcnt[i] = 0;
    } else {
      cnt[i] += add_loop;
      if (tcnt) tcnt[i] += add_loop;
    }
  }
}

__global__ void k_fill(const int64_t* __restrict__ ei, int64_t E, int64_t N, int loops,
                       const int32_t* __restrict__ rowptr, int32_t* fill, int32_t* col,
                       int32_t* eid, const int32_t* __restrict__ tptr, int32_t* tfill,
                       int32_t* tidx, int32_t* teid) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = ei[e], d = ei[E + e];
    if (s < 0 || s >= N || d < 0 || d >= N) continue;
    if (loops != LGNN_LOOPS_KEEP && s == d) continue;
    const int slot = atomicAdd(&fill[d], 1);
    col[rowptr[d] + slot] = (int32_t)s;
    eid[rowptr[d] + slot] = (int32_t)e;
    if (tptr) {
      const int ts = atomicAdd(&tfill[s], 1);
      tidx[tptr[s] + ts] = (int32_t)d;
      teid[tptr[s] + ts] = (int32_t)e;
    }
  }
}

// Per node: append the self loop (if the mode appends one), sort the row by edge id, write
// weights. Rows are short (k-NN in-degree = k); insertion sort per thread.
__device__ void sort_row(int32_t* idx, int32_t* key, int n) {
  for (int a = 1; a < n; ++a) {
    const int32_t kk = key[a], vv = idx[a];
    int b = a - 1;
    while (b >= 0 && key[b] > kk) {
      key[b + 1] = key[b];
      idx[b + 1] = idx[b];
      --b;
    }
    key[b + 1] = kk;
    idx[b + 1] = vv;
  }
}

__global__ void k_finish(int64_t N, int64_t E, int add_loop, int norm,
                         const int32_t* __restrict__ rowptr, int32_t* col, int32_t* eid, float* w,
                         const int32_t* __restrict__ tptr, int32_t* tidx, int32_t* teid,
                         float* tw) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r0 = rowptr[i], r1 = rowptr[i + 1];
    if (add_loop) {
      col[r1 - 1] = (int32_t)i;
      eid[r1 - 1] = (int32_t)(E + i);
    }
    sort_row(col + r0, eid + r0, r1 - r0);
    if (tptr) {
      const int t0 = tptr[i], t1 = tptr[i + 1];
      if (add_loop) {
        tidx[t1 - 1] = (int32_t)i;
        teid[t1 - 1] = (int32_t)(E + i);
      }
      sort_row(tidx + t0, teid + t0, t1 - t0);
    }
  }
}

// GCN weights: deg_i = row length of target i (all weights 1, loops included);
// dis = deg^-1/2 (inf -> 0); w_e = dis[src] * dis[dst]  (PyG: dis[row] * 1 * dis[col]).
__device__ __forceinline__ float gcn_dis(const int32_t* rowptr, int64_t j) {
  const int deg = rowptr[j + 1] - rowptr[j];
  return deg > 0 ? 1.0f / sqrtf((float)deg) : 0.0f;
}

__global__ void k_weights(int64_t N, int norm, const int32_t* __restrict__ rowptr,
                          const int32_t* __restrict__ col, float* w,
                          const int32_t* __restrict__ tptr, const int32_t* __restrict__ tidx,
                          float* tw) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float di = norm == LGNN_NORM_GCN ? gcn_dis(rowptr, i) : 1.f;
    if (w) {
      for (int e = rowptr[i]; e < rowptr[i + 1]; ++e)
        w[e] = norm == LGNN_NORM_GCN ? gcn_dis(rowptr, col[e]) * 1.0f * di : 1.0f;
    }
    if (tptr && tw) {
      // transposed entry (source i -> target t): weight dis[i] * dis[t]
      for (int e = tptr[i]; e < tptr[i + 1]; ++e)
        tw[e] = norm == LGNN_NORM_GCN ? di * 1.0f * gcn_dis(rowptr, tidx[e]) : 1.0f;
    }
  }
}

__global__ void k_batch_ptr(const int64_t* __restrict__ batch, int64_t M, int64_t B,
                            int32_t* ptr) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= M;
       i += (int64_t)gridDim.x * blockDim.x) {
    // graphs q with prev < q <= cur start at node i (prev = batch[i-1] or -1; cur = batch[i] or B)
    int64_t prev = i == 0 ? -1 : batch[i - 1];
    int64_t cur = i == M ? B : batch[i];
    if (prev < -1) prev = -1;
    if (cur > B) cur = B;
    for (int64_t q = prev + 1; q <= cur; ++q) ptr[q] = (int32_t)i;
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

}  // namespace

extern "C" int lgnn_abi_version(void) { return LGNN_ABI_VERSION; }

extern "C" const char* lgnn_status_string(int status) {
  switch (status) {
    case LGNN_OK: return "ok";
    case LGNN_EINVAL: return "invalid argument";
    case LGNN_ENOSPC: return "workspace too small";
    default: return status > 0 ? hipGetErrorString((hipError_t)status) : "unknown error";
  }
}

extern "C" size_t lgnn_graph_workspace_bytes(int64_t num_nodes, int64_t num_edges) {
  return ws_total(num_nodes, num_edges);
}

extern "C" int lgnn_graph_build(const int64_t* edge_index, int64_t E, int64_t N, int loops,
                                int norm, int32_t* rowptr, int32_t* col, float* w, int32_t* tptr,
                                int32_t* tidx, float* tw, int32_t* err_count, void* workspace,
                                size_t workspace_bytes, void* stream) {
  if (N < 0 || E < 0 || loops < 0 || loops > 2 || norm < 0 || norm > 1) return LGNN_EINVAL;
  if (!rowptr || !col || (E > 0 && !edge_index)) return LGNN_EINVAL;
  if (N + E > INT32_MAX) return LGNN_EINVAL;
  if ((tptr == nullptr) != (tidx == nullptr)) return LGNN_EINVAL;
  if (workspace_bytes < ws_total(N, E) || !workspace) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const int add_loop = loops == LGNN_LOOPS_KEEP ? 0 : 1;
  GraphWs ws = carve(workspace, N, E);
  // zero the counters (one contiguous region: cnt .. loopc)
  const size_t zero_bytes = (char*)ws.eid - (char*)ws.cnt;
  if (hipMemsetAsync(ws.cnt, 0, zero_bytes, s) != hipSuccess) return (int)hipGetLastError();
  if (N == 0) {
    if (hipMemsetAsync(rowptr, 0, 4, s) != hipSuccess) return (int)hipGetLastError();
    if (tptr && hipMemsetAsync(tptr, 0, 4, s) != hipSuccess) return (int)hipGetLastError();
    return LGNN_OK;
  }
  if (E > 0) {
    hipLaunchKernelGGL(k_count, dim3(grid_for(E)), dim3(kThreads), 0, s, edge_index, E, N, loops,
                       ws.cnt, tptr ? ws.tcnt : nullptr, ws.loopc, err_count);
    LGNN_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_add_loops, dim3(grid_for(N + 1)), dim3(kThreads), 0, s, ws.cnt,
                     tptr ? ws.tcnt : nullptr, N, add_loop);
  LGNN_LAUNCH_CHECK();
  size_t tb = ws.scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, tb, ws.cnt, rowptr, (int)(N + 1), s) !=
      hipSuccess)
    return (int)hipGetLastError();
  if (tptr) {
    tb = ws.scan_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, tb, ws.tcnt, tptr, (int)(N + 1), s) !=
        hipSuccess)
      return (int)hipGetLastError();
  }
  if (E > 0) {
    hipLaunchKernelGGL(k_fill, dim3(grid_for(E)), dim3(kThreads), 0, s, edge_index, E, N, loops,
                       rowptr, ws.fill, col, ws.eid, tptr, ws.tfill, tidx, ws.teid);
    LGNN_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_finish, dim3(grid_for(N)), dim3(kThreads), 0, s, N, E, add_loop, norm,
                     rowptr, col, ws.eid, w, tptr, tidx, ws.teid, tw);
  LGNN_LAUNCH_CHECK();
  if (w || tw) {
    hipLaunchKernelGGL(k_weights, dim3(grid_for(N)), dim3(kThreads), 0, s, N, norm, rowptr, col, w,
                       tptr, tidx, tw);
    LGNN_LAUNCH_CHECK();
  }
  return LGNN_OK;
}

extern "C" int lgnn_batch_ptr(const int64_t* batch, int64_t M, int64_t B, int32_t* ptr,
                              void* stream) {
  if (M < 0 || B < 0 || !ptr || (M > 0 && !batch) || M > INT32_MAX) return LGNN_EINVAL;
  hipLaunchKernelGGL(k_batch_ptr, dim3(grid_for(M + 1)), dim3(kThreads), 0, as_stream(stream),
                     batch, M, B, ptr);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
