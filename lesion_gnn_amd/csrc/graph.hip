// Graph-structure kernels: edge_index (int64 COO, any order) -> CSR by target + CSR by source,
// with PyG 2.5.1 self-loop semantics and GCN normalisation; Batch.ptr from `batch`.
//
// Replaces (reference call sites): gcn_norm inside GCNConv, GATConv's
// remove_self_loops/add_self_loops (gat.py:31), ToSparseTensor (datasets/datamodule.py:44-45).
//
// Pipeline (one memset + 4 kernels + 2 scans, no host sync):
//   k_count   per-edge in/out degree; runs of equal targets inside a wave (k-NN input is grouped by
//             target) are folded into one atomic
//   scan      rowptr / tptr = exclusive scan of (degree + appended loop)
//   k_fill    claim slots (same run folding), write (source, edge id)
//   k_finish  per 256-row block: stage the rows in LDS, append the self loop, sort each row by
//             edge id (restores edge_index order: the order PyG's scatter_add_ visits a target's
//             messages in), compute GCN weights, write back coalesced. Run for both CSRs.
// The result is identical run to run.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kFinishCap = 6144;  // staged CSR entries per 256-row block

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

struct AddLoop {
  int add;
  __host__ __device__ int operator()(int v) const { return v + add; }
};

using CntIter = hipcub::TransformInputIterator<int, AddLoop, const int32_t*>;

size_t scan_temp_bytes(int64_t n) {
  size_t bytes = 0;
  CntIter it(nullptr, AddLoop{0});
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, it, (int32_t*)nullptr, (int)n);
  return bytes;
}

struct GraphWs {
  int32_t* cnt;    // [N+1] in-degree without loops
  int32_t* tcnt;   // [N+1]
  int32_t* fill;   // [N]
  int32_t* tfill;  // [N]
  int32_t* eid;    // [E+N]
  int32_t* teid;   // [E+N]
  int32_t* inv;    // [E+N] edge id -> target-CSR position (for tmap)
  float* dis;      // [N] deg^-1/2 (GCN normalisation), inf -> 0
  void* scan_tmp;
  size_t scan_bytes;
  size_t zero_bytes;
};

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
  ws.zero_bytes = (size_t)(p - static_cast<char*>(base));
  ws.eid = (int32_t*)take((E + N) * 4);
  ws.teid = (int32_t*)take((E + N) * 4);
  ws.inv = (int32_t*)take((E + N) * 4);
  ws.dis = (float*)take(N * 4);
  ws.scan_bytes = scan_temp_bytes(N + 1);
  ws.scan_tmp = take(ws.scan_bytes);
  return ws;
}

size_t ws_total(int64_t N, int64_t E) {
  return 2 * align_up((N + 1) * 4) + 3 * align_up(N * 4) + 3 * align_up((E + N) * 4) +
         align_up(scan_temp_bytes(N + 1)) + 256;
}

// Wave-level run detection over consecutive edges: lanes whose target equals the previous
// lane's form a run; the head lane acts for the run. Invalid/skipped lanes get unique keys.
struct Run {
  bool head;
  int head_lane;
  int len;  // valid on head lanes
};

__device__ __forceinline__ Run wave_run(int64_t key) {
  const int lane = threadIdx.x & 63;
  const int64_t prev = __shfl_up(key, 1, 64);
  const bool head = lane == 0 || key != prev;
  const unsigned long long hm = __ballot(head);
  const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  Run r;
  r.head = head;
  r.head_lane = 63 - __clzll(hm & upto);
  const unsigned long long after = hm & ~upto;
  const int next = after ? __ffsll((long long)after) - 1 : 64;
  r.len = next - lane;
  return r;
}

__device__ __forceinline__ bool edge_ok(int64_t s, int64_t d, int64_t N) {
  return s >= 0 && s < N && d >= 0 && d < N;
}

// grid-stride over wave-aligned chunks so every wave sees 64 consecutive edges
__global__ __launch_bounds__(kThreads) void k_count(const int64_t* __restrict__ ei, int64_t E,
                                                    int64_t N, int loops, int32_t* cnt,
                                                    int32_t* tcnt, int32_t* err) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t base = wave0 * 64; base < E; base += nwaves * 64) {
    const int64_t e = base + lane;
    int64_t s = -1, d = -1;
    if (e < E) {
      s = ei[e];
      d = ei[E + e];
    }
    const bool valid = e < E && edge_ok(s, d, N);
    if (e < E && !valid && err) atomicAdd(err, 1);
    const bool use = valid && !(loops != LGNN_LOOPS_KEEP && s == d);
    const Run r = wave_run(use ? d : -2 - lane);
    if (use && r.head) atomicAdd(&cnt[d], r.len);
    if (use && tcnt) atomicAdd(&tcnt[s], 1);
  }
}

__global__ __launch_bounds__(kThreads) void k_fill(const int64_t* __restrict__ ei, int64_t E,
                                                   int64_t N, int loops,
                                                   const int32_t* __restrict__ rowptr,
                                                   int32_t* fill, int32_t* col, int32_t* eid,
                                                   const int32_t* __restrict__ tptr,
                                                   int32_t* tfill, int32_t* tidx, int32_t* teid) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t base = wave0 * 64; base < E; base += nwaves * 64) {
    const int64_t e = base + lane;
    int64_t s = -1, d = -1;
    if (e < E) {
      s = ei[e];
      d = ei[E + e];
    }
    const bool use = e < E && edge_ok(s, d, N) && !(loops != LGNN_LOOPS_KEEP && s == d);
    const Run r = wave_run(use ? d : -2 - lane);
    int slot0 = 0;
    if (use && r.head) slot0 = atomicAdd(&fill[d], r.len);
    slot0 = __shfl(slot0, r.head_lane, 64);
    if (use) {
      const int pos = rowptr[d] + slot0 + (lane - r.head_lane);
      col[pos] = (int32_t)s;
      eid[pos] = (int32_t)e;
      if (tptr) {
        const int ts = atomicAdd(&tfill[s], 1);
        tidx[tptr[s] + ts] = (int32_t)d;
        teid[tptr[s] + ts] = (int32_t)e;
      }
    }
  }
}

// Both degree scans in one launch (block 0: rowptr from cnt, block 1: tptr from tcnt), for
// N + 1 <= kScanSmall: thread t scans a contiguous chunk, chunk totals are scanned across the
// block. Block 0 also writes dis[i] = deg_i^-1/2 (GCN normalisation; deg 0 -> 0).
constexpr int kScanThreads = 1024;
constexpr int64_t kScanSmall = 1 << 18;

__global__ __launch_bounds__(kScanThreads) void k_scan2(const int32_t* __restrict__ cnt,
                                                        const int32_t* __restrict__ tcnt,
                                                        int64_t N, int add,
                                                        int32_t* __restrict__ rowptr,
                                                        int32_t* __restrict__ tptr,
                                                        float* __restrict__ dis) {
  __shared__ int wsum[kScanThreads / 64];
  const bool tr = blockIdx.x == 1;
  const int32_t* __restrict__ c = tr ? tcnt : cnt;
  int32_t* __restrict__ out = tr ? tptr : rowptr;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t n = N + 1;
  const int64_t chunk = (n + kScanThreads - 1) / kScanThreads;
  const int64_t b0 = tid * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
  int sum = 0;
  for (int64_t i = b0; i < b1; ++i) sum += i < N ? c[i] + add : 0;
  // inclusive scan of the chunk sums: wave, then across waves
  int x = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int v = lane < kScanThreads / 64 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    if (lane < kScanThreads / 64) wsum[lane] = v;
  }
  __syncthreads();
  int run = x - sum + (wave > 0 ? wsum[wave - 1] : 0);  // exclusive prefix of this chunk
  for (int64_t i = b0; i < b1; ++i) {
    out[i] = run;
    if (i < N) {
      const int deg = c[i] + add;
      if (!tr && dis) dis[i] = deg > 0 ? 1.0f / sqrtf((float)deg) : 0.0f;
      run += deg;
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_dis(const int32_t* __restrict__ rowptr, int64_t N,
                                                  float* __restrict__ dis) {
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * kThreads) {
    const int deg = rowptr[i + 1] - rowptr[i];
    dis[i] = deg > 0 ? 1.0f / sqrtf((float)deg) : 0.0f;
  }
}

__device__ __forceinline__ float gcn_dis(const int32_t* __restrict__ rowptr, int64_t j) {
  const int deg = rowptr[j + 1] - rowptr[j];
  return deg > 0 ? 1.0f / sqrtf((float)deg) : 0.0f;
}

// insertion sort of n (key, val) pairs by key (keys distinct)
template <typename KP, typename VP>
__device__ __forceinline__ void sort_row(KP key, VP val, int n) {
  for (int a = 1; a < n; ++a) {
    const int32_t kk = key[a], vv = val[a];
    int b = a - 1;
    while (b >= 0 && key[b] > kk) {
      key[b + 1] = key[b];
      val[b + 1] = val[b];
      --b;
    }
    key[b + 1] = kk;
    val[b + 1] = vv;
  }
}

// blockIdx.y = 0: target CSR (rowptr/col/eid/w); 1: source CSR (tptr/tidx/teid/tw).
// Weight of entry (row i, neighbour j): GCN (dis(src) * 1) * dis(dst) = dis(j) * dis(i).
__global__ __launch_bounds__(kThreads) void k_finish(int64_t N, int64_t E, int add_loop, int norm,
                                                     const int32_t* __restrict__ rowptr,
                                                     int32_t* col, int32_t* eid, float* w,
                                                     const int32_t* __restrict__ tptr,
                                                     int32_t* tidx, int32_t* teid, float* tw,
                                                     const float* __restrict__ dis) {
  __shared__ int32_t s_key[kFinishCap];
  __shared__ int32_t s_val[kFinishCap];
  const bool tr = blockIdx.y == 1;
  const int32_t* __restrict__ ptr = tr ? tptr : rowptr;
  int32_t* idx = tr ? tidx : col;
  int32_t* key = tr ? teid : eid;
  float* wt = tr ? tw : w;
  const int64_t i0 = (int64_t)blockIdx.x * kThreads;
  const int64_t i = i0 + threadIdx.x;
  const int64_t iend = i0 + kThreads < N ? i0 + kThreads : N;
  const int eb = ptr[i0], ee = ptr[iend];
  const bool staged = ee - eb <= kFinishCap;
  if (staged) {
    for (int j = eb + threadIdx.x; j < ee; j += kThreads) {
      s_key[j - eb] = key[j];
      s_val[j - eb] = idx[j];
    }
  }
  __syncthreads();
  if (i < N) {
    const int r0 = ptr[i], r1 = ptr[i + 1];
    if (staged) {
      if (add_loop) {
        s_val[r1 - 1 - eb] = (int32_t)i;
        s_key[r1 - 1 - eb] = (int32_t)(E + i);
      }
      sort_row(s_key + (r0 - eb), s_val + (r0 - eb), r1 - r0);
    } else {
      if (add_loop) {
        idx[r1 - 1] = (int32_t)i;
        key[r1 - 1] = (int32_t)(E + i);
      }
      sort_row(key + r0, idx + r0, r1 - r0);
    }
  }
  __syncthreads();
  if (staged) {
    for (int j = eb + threadIdx.x; j < ee; j += kThreads) {
      idx[j] = s_val[j - eb];
      key[j] = s_key[j - eb];
    }
  }
  if (wt) {
    // row of each entry: binary search is avoided by a per-thread row walk (rows are short)
    if (i < N) {
      const int r0 = ptr[i], r1 = ptr[i + 1];
      const float di = norm == LGNN_NORM_GCN ? dis[i] : 1.f;
      for (int j = r0; j < r1; ++j) {
        const int nb = staged ? s_val[j - eb] : idx[j];
        wt[j] = norm == LGNN_NORM_GCN ? (dis[nb] * 1.0f) * di : 1.0f;
      }
    }
  }
}

// tmap[q] = position in the target CSR of the edge at source-CSR position q (both CSRs hold the
// same entries; edge ids are unique: e for edges, E + i for appended loops).
__global__ __launch_bounds__(kThreads) void k_tmap_inv(const int32_t* __restrict__ rowptr,
                                                       int64_t N, const int32_t* __restrict__ eid,
                                                       int32_t* __restrict__ inv) {
  const int nnz = rowptr[N];
  for (int p = blockIdx.x * kThreads + threadIdx.x; p < nnz; p += gridDim.x * kThreads)
    inv[eid[p]] = p;
}

__global__ __launch_bounds__(kThreads) void k_tmap(const int32_t* __restrict__ tptr, int64_t N,
                                                   const int32_t* __restrict__ teid,
                                                   const int32_t* __restrict__ inv,
                                                   int32_t* __restrict__ tmap) {
  const int nnz = tptr[N];
  for (int q = blockIdx.x * kThreads + threadIdx.x; q < nnz; q += gridDim.x * kThreads)
    tmap[q] = inv[teid[q]];
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

inline int grid_for(int64_t n, int64_t cap = 4096) {
  int64_t g = (n + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
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
                                int32_t* tidx, float* tw, int32_t* tmap, int32_t* err_count,
                                void* workspace,
                                size_t workspace_bytes, void* stream) {
  if (N < 0 || E < 0 || loops < 0 || loops > 2 || norm < 0 || norm > 1) return LGNN_EINVAL;
  if (!rowptr || !col || (E > 0 && !edge_index)) return LGNN_EINVAL;
  if (N + E > INT32_MAX) return LGNN_EINVAL;
  if ((tptr == nullptr) != (tidx == nullptr)) return LGNN_EINVAL;
  if (tmap && !tptr) return LGNN_EINVAL;
  if (workspace_bytes < ws_total(N, E) || !workspace) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const int add_loop = loops == LGNN_LOOPS_KEEP ? 0 : 1;
  GraphWs ws = carve(workspace, N, E);
  if (hipMemsetAsync(ws.cnt, 0, ws.zero_bytes, s) != hipSuccess) return (int)hipGetLastError();
  if (N == 0) {
    if (hipMemsetAsync(rowptr, 0, 4, s) != hipSuccess) return (int)hipGetLastError();
    if (tptr && hipMemsetAsync(tptr, 0, 4, s) != hipSuccess) return (int)hipGetLastError();
    return LGNN_OK;
  }
  if (E > 0) {
    hipLaunchKernelGGL(k_count, dim3(grid_for(E, 2048)), dim3(kThreads), 0, s, edge_index, E, N,
                       loops, ws.cnt, tptr ? ws.tcnt : nullptr, err_count);
    LGNN_LAUNCH_CHECK();
  }
  if (N + 1 <= kScanSmall) {
    hipLaunchKernelGGL(k_scan2, dim3(tptr ? 2 : 1), dim3(kScanThreads), 0, s, ws.cnt, ws.tcnt, N,
                       add_loop, rowptr, tptr, ws.dis);
    LGNN_LAUNCH_CHECK();
  } else {
    size_t tb = ws.scan_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, tb, CntIter(ws.cnt, AddLoop{add_loop}),
                                         rowptr, (int)(N + 1), s) != hipSuccess)
      return (int)hipGetLastError();
    if (tptr) {
      tb = ws.scan_bytes;
      if (hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, tb, CntIter(ws.tcnt, AddLoop{add_loop}),
                                           tptr, (int)(N + 1), s) != hipSuccess)
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(k_dis, dim3(grid_for(N)), dim3(kThreads), 0, s, rowptr, N, ws.dis);
    LGNN_LAUNCH_CHECK();
  }
  if (E > 0) {
    hipLaunchKernelGGL(k_fill, dim3(grid_for(E, 2048)), dim3(kThreads), 0, s, edge_index, E, N,
                       loops, rowptr, ws.fill, col, ws.eid, tptr, ws.tfill, tidx, ws.teid);
    LGNN_LAUNCH_CHECK();
  }
  dim3 fg((unsigned)((N + kThreads - 1) / kThreads), tptr ? 2u : 1u);
  hipLaunchKernelGGL(k_finish, fg, dim3(kThreads), 0, s, N, E, add_loop, norm, rowptr, col,
                     ws.eid, w, tptr, tidx, ws.teid, tw, ws.dis);
  LGNN_LAUNCH_CHECK();
  if (tmap) {
    const int g = grid_for(E + N, 2048);
    hipLaunchKernelGGL(k_tmap_inv, dim3(g), dim3(kThreads), 0, s, rowptr, N, ws.eid, ws.inv);
    LGNN_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_tmap, dim3(g), dim3(kThreads), 0, s, tptr, N, ws.teid, ws.inv, tmap);
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
