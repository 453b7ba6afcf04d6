/*
 * lgnn.h — C ABI of the MI355X (gfx950) lesion-graph message-passing library (liblgnn.so).
 *
 * This is the drop-in boundary for the reference's hot path: everything beneath
 * `self.model(data.x, edge_index, data.batch)` (reference src/lesion_gnn/models/gin.py:64,
 * src/lesion_gnn/models/gat.py:92), i.e. the work PyG 2.5.1 + torch_scatter + torch_sparse do for
 * GINConv / GATConv / GCNConv / global_mean_pool (reference call sites gin.py:9,23,31,33 and
 * gat.py:9,31,51,56). Each entry point names the reference interface it replaces.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer (hipMalloc / torch caching allocator) unless marked host;
 *   - `stream` is a hipStream_t passed as void*; work is enqueued asynchronously on it;
 *   - nothing is allocated inside; scratch comes from caller-provided workspaces;
 *   - return 0 (LGNN_OK) or a negative LGNN_E* code / positive hipError_t; never throws;
 *   - no host synchronisation inside any call, so every call is hipGraph-capturable;
 *   - fp32 storage, fp32 accumulate; index arrays int32 (CSR) or int64 (edge_index / batch, as
 *     PyG hands them over).
 */
#ifndef LGNN_H
#define LGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LGNN_ABI_VERSION 39

#define LGNN_OK 0
#define LGNN_EINVAL (-22)
#define LGNN_ENOSPC (-28)
#define LGNN_EBUSY (-16) /* a grid-barrier launch cannot have all its workgroups resident */

/* tile flag arrays (tile_open) hold ceil(N/64) + LGNN_TILE_OPEN_EXTRA int32: one flag per 64-node
 * tile, the number of flagged tiles, six words the fused GCN stack kernels use as grid-barrier
 * counters for their open-tile phase (zeroed by whoever writes the flags, re-armed by the kernels),
 * then LGNN_SLOT_FLAGS partial-slot skip words at [ceil(N/64) + LGNN_SLOT_FLAG0 + b]: set by
 * lgnn_gcn_stack_bwd_s3f for a workgroup b that processed no closed tile and so wrote no partial
 * slot, read by lgnn_node_linear_bwd_tiles(..., accumulate = 2) (see there) */
#define LGNN_SLOT_FLAG0 7
#define LGNN_SLOT_FLAGS 256
#define LGNN_TILE_OPEN_EXTRA (LGNN_SLOT_FLAG0 + LGNN_SLOT_FLAGS)

/* self-loop handling of the graph build (which PyG utility the conv applies to edge_index) */
#define LGNN_LOOPS_KEEP 0      /* GINConv: edges used as given (KNN loop=True self pairs kept) */
#define LGNN_LOOPS_REMAINING 1 /* GCNConv gcn_norm: add_remaining_self_loops (one loop/node, last) */
#define LGNN_LOOPS_READD 2     /* GATConv: remove_self_loops + add_self_loops (one loop/node, last) */

/* edge weights written by the graph build */
#define LGNN_NORM_NONE 0 /* w = 1 */
#define LGNN_NORM_GCN 1  /* w_ij = deg_j^-1/2 * deg_i^-1/2, deg = in-degree incl. loop, inf -> 0 */

/* activation fused into the node-tile kernels */
#define LGNN_ACT_NONE 0
#define LGNN_ACT_ELU 1

/* upstream-gradient source of lgnn_node_linear_bwd */
#define LGNN_GRAD_DIRECT 0   /* dY[M,N] as given */
#define LGNN_GRAD_POOL 1     /* dY[i] = dP[batch[i]] (/ count for mean pooling) */
#define LGNN_GRAD_TRANSPOSE 2 /* dY[i] = tself*dS[i] + sum_{e in T(i)} tw_e dS[tidx_e] */

int lgnn_abi_version(void);
const char* lgnn_status_string(int status);

/* Process-wide path options (ABI v38; they replace round-5's LGNN_* environment reads): the
 * alternative kernels the default path was measured against, kept selectable for the tests that
 * check the pair bit for bit. lgnn_set_option returns the previous value (LGNN_EINVAL for an
 * unknown option); lgnn_get_option the current one. Not meant to change while launches that read
 * them are being recorded into a graph.
 *   LGNN_OPT_GAT_PIPE      1 (default): the row-pipelined GATConv kernels where the shape allows;
 *                          0: the per-row kernels
 *   LGNN_OPT_GAT_BPC       0 (default): the pipelined grids are occupancy-sized; n > 0: n
 *                          workgroups per CU
 *   LGNN_OPT_GRAPH_SORTED  1 (default): the graph build tries its target-sorted path; 0: the
 *                          general counting sort always */
#define LGNN_OPT_GAT_PIPE 0
#define LGNN_OPT_GAT_BPC 1
#define LGNN_OPT_GRAPH_SORTED 2
#define LGNN_OPT_COUNT 3
int lgnn_set_option(int option, int value);
int lgnn_get_option(int option);

/* ---------------------------------------------------------------------------------------------
 * Graph structure.
 * Replaces: PyG gcn_norm / add_remaining_self_loops (GCNConv), remove_self_loops+add_self_loops
 * (GATConv, reference gat.py:31), torch_sparse ToSparseTensor CSR (reference
 * datasets/datamodule.py:44-45) — i.e. the per-forward edge_index preprocessing.
 *
 * Builds, from edge_index int64 [2, E] (row 0 = source j, row 1 = target i, any order), a CSR
 * grouped by TARGET (rowptr[N+1], col[cap] = source, w[cap]) and optionally its transpose grouped
 * by SOURCE (tptr[N+1], tidx[cap] = target, tw[cap]), cap = E + N. Within a row entries keep
 * edge_index order; with LOOPS_REMAINING / LOOPS_READD the node's single self loop is last (as
 * PyG appends loops after the edge list). Invalid indices (<0 or >= N) are dropped and counted in
 * *err_count (device int, may be NULL). tmap (nullable, needs the transpose) [cap]: for each
 * transpose entry, the position of the same edge in the target CSR (GAT backward reads per-edge
 * attention saved in target order). tile_open (nullable) [ceil(N/64) + LGNN_TILE_OPEN_EXTRA]: as lgnn_tile_open,
 * in the same launches. gptr (nullable) [num_graphs + 1]: as lgnn_batch_ptr from batch [N],
 * in the same launches. *err_count is written (not accumulated). Workspace size:
 * lgnn_graph_workspace_bytes. N + E < 2^30. Five launches, no host synchronisation.
 *
 * Target-sorted fast path (builds without the source CSR, or lazy ones; no tmap): the first
 * launch checks edge_index on the device — targets non-decreasing, indices valid, at most one
 * self loop per row, at most 16 CSR entries per row, runs of at most 64 rows without entries and
 * (lazy) no edge leaving its 64-node tile. When every check passes (k-NN input collated in graph
 * order: PyG knn_graph groups the edges by target) the third launch writes the CSR by a scan of
 * the row lengths and a coalesced copy, and the count / fill / finish launches return at once;
 * otherwise the general counting-sort launches run. Same outputs either way (bit-identical).
 * LGNN_GRAPH_SORTED=0 in the environment disables the fast path (A/B, tests).
 * ------------------------------------------------------------------------------------------- */
size_t lgnn_graph_workspace_bytes(int64_t num_nodes, int64_t num_edges);
int lgnn_graph_build(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes, int loops,
                     int norm, int32_t* rowptr, int32_t* col, float* w, int32_t* tptr,
                     int32_t* tidx, float* tw, int32_t* tmap, int32_t* tile_open,
                     const int64_t* batch, int64_t num_graphs, int32_t* gptr, int32_t* err_count,
                     void* workspace, size_t workspace_bytes, void* stream);
/* lgnn_graph_build for a consumer that reads the source (transpose) CSR only for open tiles
 * (the fused GCN stack): tile_open and tptr required, tmap NULL; the tiles' open flags are set
 * by the count and scan passes, and tptr / tidx / tw are meaningful only when some tile is open
 * (the sorted fast path leaves them unwritten: it is taken only when no tile is open). Same target
 * CSR, flags and weights as lgnn_graph_build. */
int lgnn_graph_build_lazy(const int64_t* edge_index, int64_t E, int64_t N, int loops, int norm,
                          int32_t* rowptr, int32_t* col, float* w, int32_t* tptr, int32_t* tidx,
                          float* tw, int32_t* tmap, int32_t* tile_open, const int64_t* batch,
                          int64_t num_graphs, int32_t* gptr, int32_t* err_count, void* workspace,
                          size_t workspace_bytes, void* stream);
/* lgnn_graph_build[_lazy] (lazy != 0: the lazy variant) whose first launch also writes the split-3
 * weight planes of `job` (what lgnn_weight_planes(job->nl, job->W, job->widths, job->planes,
 * job->planes_t) writes, bitwise) as extra workgroups: the planes a fused GCN stack forward reads
 * are made from the live weights by every forward that builds its graph, with no launch of their
 * own (a captured step replays the split, so weights written between replays are seen). */
#define LGNN_PLANE_JOB_MAX 8
typedef struct lgnn_plane_job {
  int nl;                                /* layers, 1..LGNN_PLANE_JOB_MAX */
  int widths[LGNN_PLANE_JOB_MAX + 1];    /* W[l] is [widths[l+1]][widths[l]] */
  const float* W[LGNN_PLANE_JOB_MAX];
  uint16_t* planes;                      /* lgnn_weight_planes_bytes(nl) */
  uint16_t* planes_t;                    /* nullable: the transposed planes */
} lgnn_plane_job;
int lgnn_graph_build_planes(const int64_t* edge_index, int64_t E, int64_t N, int loops, int norm,
                            int32_t* rowptr, int32_t* col, float* w, int32_t* tptr,
                            int32_t* tidx, float* tw, int32_t* tmap, int32_t* tile_open,
                            const int64_t* batch, int64_t num_graphs, int32_t* gptr,
                            int32_t* err_count, void* workspace, size_t workspace_bytes, int lazy,
                            const lgnn_plane_job* job, void* stream);

/* Diagnostic (synchronises `stream`): 1 when the last lgnn_graph_build[_lazy] on `workspace`
 * took the target-sorted fast path, 0 when it ran the general launches. Meaningful only after a
 * build that tried the fast path (see above). */
int lgnn_graph_build_path(const void* workspace, int64_t num_nodes, int64_t num_edges,
                          void* stream);

/* Graph offsets from a sorted PyG `batch` vector (Batch.ptr): ptr[g] = first node of graph g,
 * ptr[B] = M. Replaces the count/offset half of PyG scatter(reduce='mean') over `batch`. */
int lgnn_batch_ptr(const int64_t* batch, int64_t num_nodes, int64_t num_graphs, int32_t* ptr,
                   void* stream);

/* ---------------------------------------------------------------------------------------------
 * k-NN graph of a batch of point sets. Replaces: torch_cluster.knn_graph(pos, k, batch, loop,
 * flow='source_to_target') behind PyG's KNNGraph transform (reference configs/config.py:47
 * KNNGraph(k=6, loop=True); per graph in datasets/datamodule.py:43-48; sweep.py:105-120 k in
 * [2, 32]). pos [N][dims] fp64 (dims 2 or 3); batch [N] int64 sorted graph ids; ptr [B+1] int32
 * graph offsets (lgnn_batch_ptr). For every node q: its kk = min(k, n_g) (loop) or
 * min(k + 1, n_g) - 1 (!loop, q itself excluded) nearest nodes of its graph, ordered by (fp64
 * squared distance, index); edge_index [2][num_edges] int64 = (neighbour, q), grouped by q in node
 * order. num_edges = sum_g n_g * kk_g (the caller computes it to size edge_index). 1 <= k <= 32.
 * workspace: lgnn_knn_workspace_bytes(B) bytes. Deterministic, bit-exact vs the fp64 restatement.
 * ------------------------------------------------------------------------------------------- */
size_t lgnn_knn_workspace_bytes(int64_t num_graphs);
int lgnn_knn_graph(const double* pos, int64_t num_nodes, int dims, const int64_t* batch,
                   const int32_t* ptr, int64_t num_graphs, int k, int loop, int64_t* edge_index,
                   int64_t num_edges, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Radius graph of a batch of point sets (ABI v32). Replaces: torch_cluster.radius_graph(pos, r,
 * batch, loop, max_num_neighbors, flow='source_to_target') behind PyG's RadiusGraph transform,
 * the reference sweep's alternative to KNNGraph (src/lesion_gnn/scripts/sweep.py:113-118,
 * RadiusGraph(r=...) with PyG's defaults loop=False, max_num_neighbors=32; resolved by name in
 * transforms.py:19-23). For every node q of graph g: walk the nodes c of g in index order, taking
 * c when the fp64 squared distance |p_q - p_c|^2 < r * r, until limit = max_num_neighbors (loop)
 * or max_num_neighbors + 1 (!loop) are taken; without loop the pair (q, q) is then dropped
 * (torch_cluster 1.6.3's CUDA selection; its CPU kd-tree keeps a traversal-order subset when more
 * than `limit` are in range). edge_index [2][E] int64 = (c, q), grouped by q in node order, c
 * ascending. pos / batch / ptr as lgnn_knn_graph; workspace lgnn_radius_workspace_bytes(N).
 *   lgnn_radius_count: per-node counts and their scan into the workspace; the edge count E is the
 *                      int64 at byte offset N * 8 of the workspace (the caller reads it to size
 *                      edge_index: the one host synchronisation).
 *   lgnn_radius_graph: writes the edges (same workspace, untouched in between; num_edges = E).
 * Deterministic, bit-exact vs the fp64 restatement (oracle/pyg_ref.py radius_graph).
 * ------------------------------------------------------------------------------------------- */
size_t lgnn_radius_workspace_bytes(int64_t num_nodes);
int lgnn_radius_count(const double* pos, int64_t num_nodes, int dims, const int64_t* batch,
                      const int32_t* ptr, int64_t num_graphs, double r, int max_num_neighbors,
                      int loop, void* workspace, size_t workspace_bytes, void* stream);
int lgnn_radius_graph(const double* pos, int64_t num_nodes, int dims, const int64_t* batch,
                      const int32_t* ptr, int64_t num_graphs, double r, int max_num_neighbors,
                      int loop, int64_t* edge_index, int64_t num_edges, const void* workspace,
                      size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Gaussian edge weights. Replaces lesion_gnn.transforms.GaussianDistance.__call__ (reference
 * src/lesion_gnn/transforms.py:49-58; known answers test/test_transforms.py:8-77), the
 * edge_weight producer of DRGNet's GraphConv stack (models/drgnet.py:55, :103):
 *   out[e] = exp(-|pos[row_e] - pos[col_e]|^2 / (2 sigma^2)) / sqrt(2 pi sigma^2)
 * evaluated in pos's precision (pos_f64: 0 = fp32, 1 = fp64; pos [num_nodes][dims], dims <= 16),
 * stored as fp32 (out_f64 = 0, the reference's default dtype) or fp64. edge_index [2][num_edges]
 * int64 (row, col). err [1] (device) = number of edges with an out-of-range index (their weight
 * is 0). num_edges == 0 is a no-op (the reference warns and leaves the graph unchanged).
 * ------------------------------------------------------------------------------------------- */
int lgnn_gaussian_distance(const void* pos, int pos_f64, int64_t num_nodes, int dims,
                           const int64_t* edge_index, int64_t num_edges, double sigma, void* out,
                           int out_f64, int32_t* err, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Node-tile fused aggregate + linear (+bias, +activation), forward.
 * Replaces: nn.Linear (reference gin.py:21 in_proj), GCNConv.lin + propagate + bias
 * (A_hat (X W^T) == (A_hat X) W^T), GINConv aggregate + first MLP Linear (reference gin.py:23),
 * with F.elu (gin.py:31) fused.
 *
 *   Y[M,N] = act( P(X) W^T + b ),  W [N,K] row-major (torch Linear layout), b [N] or NULL,
 *   P(X) = X                                   if rowptr == NULL,
 *   P(X)_i = sum_{e in row i} w_e X[col_e] + self_scale * X_i   otherwise (w == NULL: w_e = 1).
 *   S_out [M,K] (may be NULL): also store P(X) — the backward then streams it instead of
 *   re-aggregating (supported when K <= 128 and N <= 128, multiples of 4; else LGNN_EINVAL).
 * ------------------------------------------------------------------------------------------- */
int lgnn_node_linear_fwd(const float* X, int64_t M, int K, const int32_t* rowptr,
                         const int32_t* col, const float* w, float self_scale, const float* W,
                         const float* b, int N, int act, float* Y, float* S_out, void* stream);
/* Same, restricted to the 64-node tiles t with (tile_open[t] != 0) == want_open (tile_open from
 * lgnn_tile_open; NULL = every tile). Fast-path shapes only. Used to pair the layer-by-layer
 * kernels with lgnn_gcn_stack_fwd, which takes the tiles no edge leaves. */
int lgnn_node_linear_fwd_tiles(const float* X, int64_t M, int K, const int32_t* rowptr,
                               const int32_t* col, const float* w, float self_scale,
                               const float* W, const float* b, int N, int act, float* Y,
                               float* S_out, const int32_t* tile_open, int want_open,
                               void* stream);

/* ---------------------------------------------------------------------------------------------
 * Node-tile fused backward of lgnn_node_linear_fwd.
 * Replaces: autograd of nn.Linear / GCNConv / GINConv-first-Linear + F.elu + the scatter-add
 * backward (index_select / index_add_) and the global_mean_pool backward (reference gin.py:33).
 *
 *   G   = upstream gradient by grad_mode (LGNN_GRAD_*):
 *           DIRECT: dY[M,N];  POOL: dY[batch_i] (dY is [B,N]; mean: / (ptr[g+1]-ptr[g]));
 *           TRANSPOSE: tself*dY[i] + sum_{e in tptr row i} tw_e dY[tidx_e] (tw NULL: 1)
 *   dZ  = G ⊙ act'(H),  H = this layer's saved forward output [M,N] (ELU: H>0 ? 1 : H+1)
 *   dW_partial[g] (+)= dZ^T P(X) over the row tiles owned by partial slot g  ([P][N][K])
 *   db_partial[g] (+)= colsum(dZ)                                          ([P][N], may be NULL)
 *   dXpre = dZ W  [M,K]  (may be NULL)
 * The P partial slots are summed by lgnn_reduce_partials (deterministic order).
 * num_partials: lgnn_bwd_num_partials(M, N, K, rowptr != NULL) — pass that value and size the
 * slabs with it.
 * ------------------------------------------------------------------------------------------- */
int lgnn_bwd_num_partials(int64_t M, int N, int K, int gather);
int lgnn_node_linear_bwd(int grad_mode, const float* dY, const int64_t* batch, const int32_t* gptr,
                         int pool_mean, const int32_t* tptr, const int32_t* tidx, const float* tw,
                         float tself, const float* H, int act, const float* X, int64_t M, int K,
                         const int32_t* rowptr, const int32_t* col, const float* w,
                         float self_scale, const float* W, int N, float* dXpre,
                         float* dW_partial, float* db_partial, int num_partials, void* stream);

/* Same, restricted to the 64-node tiles t with (tile_open[t] != 0) == want_open; with
 * accumulate = 1 a workgroup that processed a tile adds its dW/db into partial slot blockIdx.x
 * (num_partials = lgnn_gcn_stack_bwd_partials, slots written by lgnn_gcn_stack_bwd) instead of
 * overwriting it, and a workgroup that processed none leaves its slot alone. accumulate = 2 (after
 * lgnn_gcn_stack_bwd_s3f, num_partials <= LGNN_SLOT_FLAGS): the same, except for slots whose skip
 * word in tile_open is set (the fused kernel wrote nothing there): those are written, with zeros
 * by a workgroup that processed no tile. Fast path only. */
int lgnn_node_linear_bwd_tiles(int grad_mode, const float* dY, const int64_t* batch,
                               const int32_t* gptr, int pool_mean, const int32_t* tptr,
                               const int32_t* tidx, const float* tw, float tself, const float* H,
                               int act, const float* X, int64_t M, int K, const int32_t* rowptr,
                               const int32_t* col, const float* w, float self_scale,
                               const float* W, int N, float* dXpre, float* dW_partial,
                               float* db_partial, int num_partials, const int32_t* tile_open,
                               int want_open, int accumulate, void* stream);

/* out[i] = sum_{p < P} partial[p*len + i], fixed order (bitwise reproducible). */
int lgnn_reduce_partials(const float* partial, int num_partials, int64_t len, float* out,
                         void* stream);
/* The same for n <= 16 independent slabs in one launch (host arrays of n entries). */
int lgnn_reduce_partials_multi(int n, const float* const* partials, const int* num_partials,
                               const int64_t* len, float* const* out, void* stream);
/* lgnn_reduce_partials_multi + outer-product jobs: where factor[j] is set (factor / width may be
 * NULL for none), out_j[c * width_j + d] = sum_{p < P_j} partials_j[p * (len_j / width_j) + c] *
 * factor_j[p * width_j + d] (fixed order). One such job is out_proj's weight gradient
 * dW_out = dlogits^T pooled, queued with the stack's slab reductions. */
int lgnn_reduce_jobs(int n, const float* const* partials, const float* const* factor,
                     const int* width, const int* num_partials, const int64_t* len,
                     float* const* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Sparse aggregation alone (no linear): Y_i = self_scale*X_i + sum_{e in row i} w_e X[col_e].
 * Replaces: torch_sparse spmm(adj_t, x, 'sum') / PyG propagate(aggr='add') (GINConv, and the
 * transposed pass of every conv backward when called with the transpose CSR).
 * ------------------------------------------------------------------------------------------- */
int lgnn_spmm(const int32_t* rowptr, const int32_t* col, const float* w, float self_scale,
              const float* X, int64_t M, int D, float* Y, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Readout: per-graph segmented pool fused with the out_proj Linear.
 * Replaces: global_mean_pool / global_add_pool (reference gin.py:33, gat.py:56) + out_proj
 * (gin.py:25, gat.py:46).
 *   pooled[B,D] = sum_{i in graph g} H_i (/ count if mean; empty graph -> 0)
 *   logits[B,C] = pooled Wout^T + bout        (Wout may be NULL: pool only, logits unused)
 * ------------------------------------------------------------------------------------------- */
int lgnn_pool_head_fwd(const float* H, const int32_t* gptr, int64_t B, int D, int pool_mean,
                       const float* Wout, const float* bout, int C, float* pooled,
                       float* logits, void* stream);

/* Backward of lgnn_pool_head_fwd's Linear part:
 *   dpooled = dlogits Wout;  dWout = dlogits^T pooled;  dbout = colsum(dlogits). */
int lgnn_pool_head_bwd(const float* dlogits, const float* pooled, int64_t B, int D,
                       const float* Wout, int C, float* dpooled, float* dWout, float* dbout,
                       void* stream);

/* Backward of a bare segmented pool: dH_i = dpooled[batch_i] (/ count if mean). */
int lgnn_pool_bwd(const float* dpooled, const int64_t* batch, const int32_t* gptr, int64_t M,
                  int D, int pool_mean, float* dH, void* stream);

/* ---------------------------------------------------------------------------------------------
 * BatchNorm1d + ELU (+ dropout mask) of the GIN MLP.
 * Replaces: PyG MLP([d1,d2,d2], act="ELU", norm="batch_norm") internals (reference gin.py:23):
 * torch.nn.BatchNorm1d forward/backward (training: batch statistics, running stats updated with
 * momentum and the unbiased variance; eval: running statistics), F.elu, F.dropout.
 * Statistics in fp64, deterministic. `sums` is [2N] fp64: forward (sum z, sum z^2); backward
 * (sum g, sum g*xhat) — caller-visible so a SyncBN all-reduce can run in between.
 * mask (nullable): dropout keep-mask already scaled by 1/(1-p), [M,N].
 * ------------------------------------------------------------------------------------------- */
size_t lgnn_bn_workspace_bytes(int64_t num_rows, int N);
int lgnn_bn_stats(const float* Z, int64_t M, int N, double* sums, void* workspace,
                  size_t workspace_bytes, void* stream);
/* mean/invstd/scale/shift [N] out; scale = gamma*invstd, shift = beta - mean*scale. training=0
 * reads running_mean/var; training=1 updates them (if non-NULL) and num_batches_tracked. */
int lgnn_bn_finalize(const double* sums, double count, const float* gamma, const float* beta,
                     float eps, float momentum, int training, int N, float* running_mean,
                     float* running_var, int64_t* num_batches_tracked, float* mean,
                     float* invstd, float* scale, float* shift, void* stream);
/* A = ELU(Z*scale + shift) [* mask] */
int lgnn_bn_act(const float* Z, int64_t M, int N, const float* scale, const float* shift,
                const float* mask, float* A, void* stream);
/* sums = (sum g, sum g*xhat), g = dA * mask * ELU'(Z*scale+shift), xhat = (Z-mean)*invstd */
int lgnn_bn_bwd_stats(const float* dA, const float* Z, const float* mask, int64_t M, int N,
                      const float* scale, const float* shift, const float* mean,
                      const float* invstd, double* sums, void* workspace, size_t workspace_bytes,
                      void* stream);
/* dZ = scale*(g - sum g/count - xhat * sum(g xhat)/count) (training) | scale*g (eval);
 * dgamma = sum g*xhat, dbeta = sum g (each nullable) */
int lgnn_bn_bwd_apply(const float* dA, const float* Z, const float* mask, int64_t M, int N,
                      const float* scale, const float* shift, const float* mean,
                      const float* invstd, const double* sums, double count, int training,
                      float* dZ, float* dgamma, float* dbeta, void* stream);
/* sums[2N] = the fixed-order sum of num_partials fp64 partial rows part[p][2N] (the BN-fused
 * linear kernels below write one row per workgroup); dgamma = sums[N..2N), dbeta = sums[0..N)
 * (each nullable: the backward's affine gradients, as lgnn_bn_bwd_apply's). */
int lgnn_bn_partials_reduce(const double* part, int num_partials, int N, double* sums,
                            float* dgamma, float* dbeta, void* stream);
/* lgnn_bn_partials_reduce + lgnn_bn_finalize (training) in one launch (no SyncBN all-reduce
 * between them). */
int lgnn_bn_partials_finalize(const double* part, int num_partials, int N, double* sums,
                              double count, const float* gamma, const float* beta, float eps,
                              float momentum, float* running_mean, float* running_var,
                              int64_t* num_batches_tracked, float* mean, float* invstd,
                              float* scale, float* shift, void* stream);

/* ---------------------------------------------------------------------------------------------
 * The GIN MLP's linear layers with BatchNorm folded into them (the same arithmetic as the
 * lgnn_bn_* kernels above, without their passes over HBM). Fast-path shapes only (K, N <= 128,
 * multiples of 4); one partial row per workgroup, lgnn_bn_fused_partials(M) rows.
 * lgnn_node_linear_fwd_bn = lgnn_node_linear_fwd (no tile selection) with exactly one of
 *   stats_part: [P][2N] fp64 per-workgroup (sum y, sum y^2) of the output Y (then
 *     lgnn_bn_partials_reduce -> lgnn_bn_finalize), or
 *   bn_scale / bn_shift [K] (+ bn_mask [M,K], nullable): the input rows are first mapped to
 *     ELU(X*scale + shift) [* mask] — lgnn_bn_act fused into the load — and that activation is
 *     also written to bn_out [M,K] (the backward's dW input); no gather.
 * lgnn_node_linear_bwd_bn = lgnn_node_linear_bwd in LGNN_GRAD_DIRECT mode (no gather) with
 *   bn_mode LGNN_BN_GSTATS: the dX output is the gradient dA of a BN + ELU (+ mask) output whose
 *     input is bn_Z [M,K]; gstats_part [P][2K] receives per-workgroup (sum g, sum g*xhat)
 *     (lgnn_bn_bwd_stats fused into the dX epilogue), or
 *   bn_mode LGNN_BN_GIN (act NONE): dY is such a dA [M,N] of BN input bn_Z [M,N]; the kernel
 *     applies the BN backward (lgnn_bn_bwd_apply's dZ, with bn_sums / count / training) before
 *     using it, so dZ never goes to HBM.
 * ------------------------------------------------------------------------------------------- */
#define LGNN_BN_GSTATS 3
#define LGNN_BN_GIN 4
/* lgnn_node_linear_bwd_bn with the layer's output gradient taken from the pooled readout
 * (LGNN_GRAD_POOL, bn_mode LGNN_BN_GSTATS only): row i's gradient is
 *   (dlogits[batch[i]] . Wout)[n] (/ |graph| when pool_mean),
 * i.e. the global pool + out_proj backward (lgnn_pool_head_bwd's dpooled and lgnn_pool_bwd)
 * folded into the load, in the same arithmetic; dY is unused (NULL). The GIN model's last conv. */
int lgnn_node_linear_bwd_bn_pool(int bn_mode, const float* dY, const float* H, int act,
                                 const float* X, int64_t M, int K, const float* W, int N,
                                 float* dXpre, float* dW_partial, float* db_partial,
                                 int num_partials, const float* bn_Z, const float* bn_mask,
                                 const float* bn_scale, const float* bn_shift,
                                 const float* bn_mean, const float* bn_invstd,
                                 double* gstats_part, const double* bn_sums, double count,
                                 int training, const int64_t* batch, const int32_t* gptr,
                                 int pool_mean, const float* dlogits, const float* Wout,
                                 int num_classes, void* stream);
/* lgnn_node_linear_bwd_bn (bn_mode LGNN_BN_GSTATS) with the output gradient gathered through the
 * transpose CSR as it is loaded (ABI v21): row i's gradient is
 *   tself * dS[i] + sum_{e in T(i)} tw_e dS[tidx_e]   (LGNN_GRAD_TRANSPOSE),
 * dS [M,N] being the NEXT GINConv's pre-aggregation input gradient (its Lin1 dX). This is the
 * backward of that conv's aggregation (PyG GINConv propagate + (1 + eps) x, reference gin.py:23)
 * folded into this conv's Lin2 backward, so the aggregated gradient never goes to HBM. */
int lgnn_node_linear_bwd_bn_gather(const float* dS, const int32_t* tptr, const int32_t* tidx,
                                   const float* tw, float tself, const float* H, int act,
                                   const float* X, int64_t M, int K, const float* W, int N,
                                   float* dXpre, float* dW_partial, float* db_partial,
                                   int num_partials, const float* bn_Z, const float* bn_mask,
                                   const float* bn_scale, const float* bn_shift,
                                   const float* bn_mean, const float* bn_invstd,
                                   double* gstats_part, void* stream);
int lgnn_bn_fused_partials(int64_t num_rows);
int lgnn_node_linear_fwd_bn(const float* X, int64_t M, int K, const int32_t* rowptr,
                            const int32_t* col, const float* w, float self_scale, const float* W,
                            const float* b, int N, int act, float* Y, float* S_out,
                            double* stats_part, const float* bn_scale, const float* bn_shift,
                            const float* bn_mask, float* bn_out, void* stream);
int lgnn_node_linear_bwd_bn(int bn_mode, const float* dY, const float* H, int act,
                            const float* X, int64_t M, int K, const float* W, int N,
                            float* dXpre, float* dW_partial, float* db_partial, int num_partials,
                            const float* bn_Z, const float* bn_mask, const float* bn_scale,
                            const float* bn_shift, const float* bn_mean, const float* bn_invstd,
                            double* gstats_part, const double* bn_sums, double count,
                            int training, void* stream);

/* ---------------------------------------------------------------------------------------------
 * GATConv attention (PyG 2.5.1 GATConv(d1, d2//H, heads=H, dropout=p), reference gat.py:31:
 * concat=True, negative_slope, add_self_loops=True, bias=True) + the model's F.elu (gat.py:51).
 * XP = lin(x) [M, H*C] (lgnn_node_linear_fwd without bias). Graph: the LGNN_LOOPS_READD CSR
 * (remove_self_loops + add_self_loops). Per-edge arrays are [cap, H] in target-CSR order.
 * Shapes: C a power of two in [4, 512], H*C <= 512. edge_mask (nullable): attention dropout keep-mask
 * already scaled by 1/(1-p).
 * ------------------------------------------------------------------------------------------- */
/* a_s[i,h] = <XP[i,h,:], att_src[h,:]>, a_d likewise with att_dst (the alpha_src/alpha_dst sums) */
int lgnn_gat_att(const float* XP, int64_t M, int H, int C, const float* att_src,
                 const float* att_dst, float* a_s, float* a_d, void* stream);
/* alpha = softmax_i(leaky_relu(a_s[j] + a_d[i])) (PyG utils.softmax, +1e-16; written if
 * non-NULL), Y_i = act(sum_j alpha_ij mask_ij XP_j + bias); Y_bf16 (nullable) also receives Y
 * rounded to bf16 (RNE, torch's .to(bfloat16)): the next layer's bf16 GEMM operand */
int lgnn_gat_fwd(const int32_t* rowptr, const int32_t* col, const float* XP, const float* a_s,
                 const float* a_d, int64_t M, int H, int C, float negative_slope,
                 const float* edge_mask, const float* bias, int act, float* alpha, float* Y,
                 uint16_t* Y_bf16, void* stream);
/* Backward, target rows: dZ = dY * act'(Y); da_e = d(logit) per edge; da_d = row sums. */
int lgnn_gat_bwd_edge(const int32_t* rowptr, const int32_t* col, const float* XP,
                      const float* a_s, const float* a_d, const float* alpha,
                      const float* edge_mask, const float* dY, const float* Y, int act, int64_t M,
                      int H, int C, float negative_slope, float* dZ, float* da_e, float* da_d,
                      void* stream);
/* lgnn_gat_bwd_edge with the output gradient formed from the readout's gradient (ABI v22):
 * dY[i] = (dlogits[batch[i]] . Wout) (/ |graph| when pool_mean), with lgnn_pool_head_bwd's and
 * lgnn_pool_bwd's arithmetic (bitwise), so the GAT model's last conv needs no dH tensor: the
 * global_mean_pool / global_add_pool + out_proj backward (reference gat.py:56-58) folded into
 * this kernel's load. Wout [num_classes][H*C]; dY is not an argument. */
int lgnn_gat_bwd_edge_pool(const int32_t* rowptr, const int32_t* col, const float* XP,
                           const float* a_s, const float* a_d, const float* alpha,
                           const float* edge_mask, const float* Y, int act, int64_t M, int H,
                           int C, float negative_slope, const int64_t* batch,
                           const int32_t* gptr, int pool_mean, const float* dlogits,
                           const float* Wout, int num_classes, float* dZ, float* da_e,
                           float* da_d, void* stream);
/* Backward, source rows (transpose CSR + tmap from lgnn_graph_build): dXP, and per-block column
 * partials [P][3][H*C] = (d att_src, d att_dst, d bias) for lgnn_reduce_partials. */
int lgnn_gat_bwd_num_partials(int64_t M);
int lgnn_gat_bwd_node(const int32_t* tptr, const int32_t* tidx, const int32_t* tmap,
                      const float* alpha, const float* edge_mask, const float* da_e,
                      const float* da_d, const float* dZ, const float* XP, const float* att_src,
                      const float* att_dst, int64_t M, int H, int C, float* dXP,
                      float* partials, int num_partials, uint16_t* dXP_bf16, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused GCN layer stack, forward (one launch for the whole model body below the readout).
 * Replaces: in_proj nn.Linear (reference gin.py:21 skeleton) + L x (GCNConv + F.elu) — the
 * layer-by-layer lgnn_node_linear_fwd chain — keeping each 64-node tile on chip across layers.
 *   has_in_proj=1: H[0] = X W[0]^T + b[0] (X [M, d_in]); else layer 1 reads X (widths[0]=d_in)
 *   for l = 1..L: H[l] = ELU(Â (H[l-1] W[l]^T) + b[l]) (CSR rowptr/col/w, self loops in the
 *   CSR; PyG 2.5.1 GCNConv order: lin, then propagate, then bias).  W, b, H: host arrays of
 *   L+1 device pointers; widths[l] = output width of layer l. All widths and d_in <= 128,
 *   multiples of 4; L + 1 <= 8.
 *   tile_open (required when L >= 1): only tiles with tile_open[t] == 0 are computed — their
 *   CSR entries stay inside the tile and number at most 2048 (lgnn_graph_build /
 *   lgnn_tile_open flags); run the others with lgnn_node_linear_fwd_tiles(..., tile_open, 1).
 * ------------------------------------------------------------------------------------------- */
int lgnn_gcn_stack_fwd(const float* X, int64_t M, int d_in, int has_in_proj,
                       const int32_t* rowptr, const int32_t* col, const float* w, int L,
                       const float* const* W, const float* const* b, const int* widths,
                       float* const* H, const int32_t* tile_open, void* stream);
/* Split-3 variant of lgnn_gcn_stack_fwd: the same math and arguments, the GEMMs on bf16 MFMA at
 * fp32 accuracy — every operand held as three bf16 planes (x = hi + mid + lo to 2^-24) and each
 * product taken as the six plane products that matter (liblgnn stack3.hip). `planes` holds the
 * weights of layers 0..L as written by lgnn_weight_planes (in place of W). L >= 1.
 * adjt (nullable): ceil(M/64) * LGNN_S3_ADJT_TILE_BYTES bytes; receives, for every closed tile,
 * the tile's dense fp32 Â (64 x 64, as summed from the CSR block), which
 * lgnn_gcn_stack_bwd_s3f(_all) then loads instead of rebuilding it (same graph, same tile_open). */
#define LGNN_S3_ADJT_TILE_BYTES 16384
int lgnn_gcn_stack_fwd_s3(const float* X, int64_t M, int d_in, int has_in_proj,
                          const int32_t* rowptr, const int32_t* col, const float* w, int L,
                          const uint16_t* planes, const float* const* b, const int* widths,
                          float* const* H, const int32_t* tile_open, void* adjt, void* stream);
/* Weight planes for the split-3 kernels: nl layers, W[l] [widths[l+1], widths[l]] fp32
 * (torch Linear layout; widths <= 128, multiples of 4) -> planes[l][3][128][128] bf16 (zero
 * padded, feature order perm16), lgnn_weight_planes_bytes(nl) bytes; planes_t (nullable, same
 * size) also gets the transposed planes. One launch; rerun whenever the weights change. */
size_t lgnn_weight_planes_bytes(int nl);
int lgnn_weight_planes(int nl, const float* const* W, const int* widths, uint16_t* planes,
                       uint16_t* planes_t, void* stream);

/* Split-3 backward of the fused GCN stack for the closed tiles (tile_open[t] == 0), one launch per
 * layer (stack3_bwd.hip), the same math and outputs as lgnn_gcn_stack_bwd with any L >= 1 (L + 1 <=
 * 8): the GEMMs on bf16 MFMA at fp32 accuracy. planes_t: the transposed weight planes of layers
 * 0..L (lgnn_weight_planes(..., planes_t)); dP [num_graphs][widths[L+1]] the pooled-output
 * gradient; dz_ws: 2 * M * 128 floats of scratch (dZ between the layer launches); dWp/dbp slabs
 * with num_partials = lgnn_gcn_stack_bwd_s3_partials(M) slots, every slot written. */
int lgnn_gcn_stack_bwd_s3_partials(int64_t num_nodes);
int lgnn_gcn_stack_bwd_s3(const float* dP, const int64_t* batch, const int32_t* gptr,
                          int pool_mean, int64_t num_graphs, const int32_t* rowptr,
                          const int32_t* col, const float* w, const float* X, int64_t M, int L,
                          const uint16_t* planes_t, const float* const* H, const int* widths,
                          float* const* dWp, float* const* dbp, int num_partials, float* dz_ws,
                          const int32_t* tile_open, void* stream);
/* Tiles: 64 consecutive node rows. open[t] = 1 when an edge joins tile t to another tile (its
 * layers then depend on other tiles) or when the tile holds more than 2048 CSR entries; the
 * fused stacks skip open tiles. open has lgnn_tile_count(N) + 1 entries: the last one counts the
 * open tiles (the *_tiles kernels with want_open = 1 return at once when it is 0). */
int lgnn_tile_count(int64_t num_nodes);
int lgnn_tile_open(const int32_t* rowptr, const int32_t* col, int64_t num_nodes, int32_t* open,
                   void* stream);

/* ---------------------------------------------------------------------------------------------
 * Criterion. Replaces: nn.CrossEntropyLoss(weight=class_weights) of BaseLightningModule
 * (reference models/base.py:93-94, training_step :196-201), mean reduction.
 *   fwd: lse[B] = logsumexp(logits_i); loss[0] = sum w[y] (lse - z[y]) / sum w[y]; wsum[0] =
 *        sum w[y] (weight NULL = 1); *bad = 1 if a target is outside [0, C) (such rows skipped).
 *   bwd: dlogits = grad_loss[0] * w[y_i] / wsum * (softmax(z_i) - onehot(y_i)).
 * Deterministic (one workgroup, fixed reduction order). All pointers device pointers.
 * ------------------------------------------------------------------------------------------- */
int lgnn_ce_fwd(const float* logits, const int64_t* target, const float* weight, int64_t B, int C,
                float* lse, float* loss, float* wsum, int* bad, void* stream);
int lgnn_ce_bwd(const float* logits, const int64_t* target, const float* weight, int64_t B, int C,
                const float* lse, const float* wsum, const float* grad_loss, float* dlogits,
                void* stream);
/* lgnn_ce_fwd that also writes the logits gradient's per-row factors (ABI v35):
 * pm [B][C] = exp(z - lse) - [c == y], wt [B] = weight[y] (1 unweighted, 0 for a target outside
 * [0, C)) — lgnn_ce_src's inputs, so a consumer forms lgnn_ce_bwd's dlogits from plain loads. */
int lgnn_ce_fwd_factors(const float* logits, const int64_t* target, const float* weight,
                        int64_t B, int C, float* lse, float* loss, float* wsum, int* bad,
                        float* pm, float* wt, void* stream);
/* The CE logits gradient without materialising it (ABI v33; v35: from the readout's pm / wt): the
 * consumers form lgnn_ce_bwd's dlogits[i][c] = gloss * wt[i] / wsum * pm[i][c] themselves, bit
 * for bit (lgnn_ce_fwd_factors writes pm and wt with lgnn_ce_bwd's expressions).
 * lgnn_reduce_jobs_ce = lgnn_reduce_jobs where jobs with ce_job[j] != 0 take the [P][C] logits
 * gradient (P = B) in place of partials[j] (which may be NULL): out_proj's db (len C) and
 * dW = dlogits^T pooled (factor = pooled, len C * width). The same sums as lgnn_reduce_jobs on
 * lgnn_ce_bwd's output, bitwise. */
typedef struct lgnn_ce_src {
  const float* pm;     /* [B][C] exp(z - lse) - [c == y] (lgnn_ce_fwd_factors) */
  const float* wt;     /* [B] weight[y] (lgnn_ce_fwd_factors) */
  const float* wsum;   /* [1] */
  const float* gloss;  /* [1] gradient of the loss */
} lgnn_ce_src;
int lgnn_reduce_jobs_ce(int n, const float* const* partials, const float* const* factor,
                        const int* width, const int* num_partials, const int64_t* len,
                        float* const* out, const int* ce_job, const lgnn_ce_src* ce,
                        int num_classes, void* stream);
/* Regression head + criterion (ABI v23): pred = clamp(z, lo, hi) (reference gat.py:94-95,
 * gin.py:66-67: logits.squeeze(1).clamp(0, C - 1)) and loss = mean l(pred - y) with
 * l = nn.MSELoss (smooth_l1 = 0) or nn.SmoothL1Loss(beta = 1) (models/base.py:95-96), one
 * workgroup, fixed-order sum. target: int64 class labels (target_is_i64; the reference's
 * y.float()) or fp32 [B]. Backward: dz = [lo <= z <= hi] (grad_pred + grad_loss / B l'(pred - y));
 * grad_loss / grad_pred nullable (not both). */
int lgnn_regression_fwd(const float* z, const void* target, int target_is_i64, int64_t B,
                        float lo, float hi, int smooth_l1, float* pred, float* loss,
                        void* stream);
int lgnn_regression_bwd(const float* z, const void* target, int target_is_i64, int64_t B,
                        float lo, float hi, int smooth_l1, const float* grad_loss,
                        const float* grad_pred, float* dz, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused GCN layer stack, backward, for the tiles with tile_open[t] == 0 (L = 1 or 2 convs).
 * Replaces: the autograd chain below the readout of in_proj -> L x ELU(GCNConv) — pool broadcast
 * of dP (global_mean/add_pool backward), per conv G = Â^T dZ, dW += G^T H_{l-1}, dH = G W,
 * dZ = dH * ELU'(H) (PyG 2.5.1 GCNConv: out = propagate(lin(x)) + bias,
 * torch_geometric/nn/conv/gcn_conv.py) and dW_0 += dZ_0^T X for in_proj — with every
 * intermediate on chip.
 *   rowptr/col/w: the forward (target-row) CSR of lgnn_graph_build;
 *   W, H: host arrays of L+1 device pointers (H[l] = output of layer l, H[0] = in_proj output);
 *   widths[0..L+1] = d_in, h_0, ..., h_L; dWp/dbp: per-layer partial slabs with num_partials =
 *   lgnn_gcn_stack_bwd_partials(M) slots (reduce with lgnn_reduce_partials[_multi]).
 * Tiles with tile_open[t] != 0 are left to lgnn_node_linear_bwd_tiles(..., want_open = 1,
 * accumulate = 1) on the same slabs. No input gradient (the model input needs none).
 * ------------------------------------------------------------------------------------------- */
int lgnn_gcn_stack_bwd_partials(int64_t num_nodes);

int lgnn_gcn_stack_bwd(const float* dP, const int64_t* batch, const int32_t* gptr, int pool_mean,
                       const int32_t* rowptr, const int32_t* col, const float* w, const float* X,
                       int64_t M, int L, const float* const* W, const float* const* H,
                       const int* widths, float* const* dWp, float* const* dbp, int num_partials,
                       const int32_t* tile_open, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Optimizer step. Replaces: torch.optim.Adam / AdamW (amsgrad = False) as configured by the
 * reference (models/base.py:162-188), in one launch over up to 16 fp32 tensors.
 *   decoupled = 0: Adam (L2: g += weight_decay * p); 1: AdamW (p *= 1 - lr * weight_decay).
 *   step: device float, the number of steps taken (read by every workgroup; with advance = 1
 *   incremented once, by the last one); ticket: device uint32[9], zero before the first call
 *   (re-armed by the call). Split a longer list over several calls with advance = 0 on all but
 *   the last (every call of one step then uses the same step count).
 *   Graph-capturable (lr and the betas are launch arguments: fixed in a captured graph).
 * ------------------------------------------------------------------------------------------- */
int lgnn_adam_step(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, const int64_t* numels, float* step,
                   unsigned int* ticket, float lr, float beta1, float beta2, float eps,
                   float weight_decay, int decoupled, int maximize, int advance,
                   void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused GCN stack backward on split-3 bf16 MFMA (fp32 accuracy), every layer of a tile in one
 * pass, one launch. Replaces the same autograd chain as lgnn_gcn_stack_bwd (reference path:
 * global_mean/add_pool backward, per conv G = Â^T dZ, dW += G^T H, dH = G W, ELU', and in_proj
 * dW) for tiles with tile_open[t] == 0, L = 1 or 2 convs (3 through the _all / _ce entries
 * below), every width <= 128 and % 4 == 0.
 *   planes_t: the transposed weight planes of lgnn_weight_planes (all L + 1 layers);
 *   H[0..L]: layer outputs (H[0] = in_proj output); X: model input; widths[0..L+1];
 *   dWp / dbp: per-layer partial slabs with num_partials = lgnn_gcn_stack_bwd_partials(M)
 *   slots. A workgroup that processed no closed tile writes NO slot: it sets its skip word
 *   tile_open[ceil(M/64) + LGNN_SLOT_FLAG0 + b] instead (so tile_open is written by this call,
 *   beside the barrier words), and the open tiles must then be accumulated by
 *   lgnn_node_linear_bwd_tiles(..., accumulate = 2), which writes the skipped slots (zeros where
 *   it has no tile either). accumulate = 1 after this call would add to uninitialised slots.
 *   adjt (nullable): the tile adjacencies the split-3 forward wrote for this graph (its adjt);
 *   each tile's goes straight into LDS (prefetched during the previous tile) instead of being
 *   rebuilt from the CSR.
 * ------------------------------------------------------------------------------------------- */
int lgnn_gcn_stack_bwd_s3f(const float* dP, const int64_t* batch, const int32_t* gptr,
                           int pool_mean, int64_t num_graphs, const int32_t* rowptr,
                           const int32_t* col, const float* w, const float* X, int64_t M, int L,
                           const uint16_t* planes_t, const float* const* H, const int* widths,
                           float* const* dWp, float* const* dbp, int num_partials,
                           const int32_t* tile_open, const void* adjt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * The fused GCN stack with its open-tile phase in the same launch (no separate layer-by-layer
 * launches). Tiles flagged open (an edge leaves them, or > 2048 CSR entries) share no edge with
 * closed tiles, so after the closed tiles the kernel runs them layer by layer in fp32 (the bodies
 * of lgnn_node_linear_fwd_tiles / _bwd_tiles) with a grid barrier between layers; with no open
 * tile (the count word of tile_open is 0) that phase is skipped. tile_open: the graph build's
 * [ceil(M/64) + LGNN_TILE_OPEN_EXTRA] array (its barrier words are used and re-armed).
 * lgnn_gcn_stack_fwd_s3_all = lgnn_gcn_stack_fwd_s3 + W (fp32 weights, host array of L + 1
 *   device pointers) + S (host array of L pointers: S[l - 1] [M][K_l] receives Â H_{l-1} of the
 *   open tiles, read by the backward's open phase).
 * lgnn_gcn_stack_bwd_s3f_all = lgnn_gcn_stack_bwd_s3f + the transpose CSR (tptr / tidx / tw),
 *   W, S (as above) and dS_ws (2 * M * 128 floats of workspace). L = 3 (ABI v39; this entry and
 *   _ce only): dS_ws holds 3 * M * 128 floats, its last block receives dZ_0 [M][widths[1]] (the
 *   in_proj output gradient, every row) and dWp[0] / dbp[0] are not written — the caller forms
 *   dW_0 = dZ_0^T X and db_0 = colsum dZ_0 (lgnn_s3_wgrad). With dlogits [B][C] and Wout
 *   [C][N_L] (C <= 8) the pooled-output gradient dP = dlogits Wout (out_proj backward) is formed
 *   inside the kernel and dP may be NULL (lgnn_pool_head_bwd then only needs dWout / dbout, and
 *   can run concurrently).
 * Both _all entries return LGNN_EBUSY (nothing launched) when the device cannot hold every
 * workgroup of the launch at once (its grid barriers need co-residency): the caller then runs the
 * open tiles in separate launches. lgnn_fused_grid_capacity(which) = workgroups resident at once
 * (occupancy per CU x CUs; which 0 = forward, 1 = backward), or an error code (< 0). A barrier
 * that still times out (~0.5 s) counts itself in the third barrier word (tile_open[ntiles + 3]
 * forward, [ntiles + 6] backward), which stays set until the next graph build zeroes it.
 * ------------------------------------------------------------------------------------------- */
int lgnn_fused_grid_capacity(int which);
int lgnn_gcn_stack_fwd_s3_all(const float* X, int64_t M, int d_in, int has_in_proj,
                              const int32_t* rowptr, const int32_t* col, const float* w, int L,
                              const uint16_t* planes, const float* const* W,
                              const float* const* b, const int* widths, float* const* H,
                              float* const* S, int32_t* tile_open, void* adjt, void* stream);
int lgnn_gcn_stack_bwd_s3f_all(const float* dP, const int64_t* batch, const int32_t* gptr,
                               int pool_mean, int64_t num_graphs, const int32_t* rowptr,
                               const int32_t* col, const float* w, const int32_t* tptr,
                               const int32_t* tidx, const float* tw, const float* X, int64_t M,
                               int L, const uint16_t* planes_t, const float* const* W,
                               const float* const* H, const float* const* S, const int* widths,
                               float* const* dWp, float* const* dbp, int num_partials,
                               float* dS_ws, int32_t* tile_open, const float* dlogits,
                               const float* Wout, int num_classes, const void* adjt,
                               void* stream);
/* lgnn_gcn_stack_bwd_s3f_all with the logits gradient formed in the kernel from the CE forward
 * (ABI v33: lgnn_ce_src, declared with lgnn_ce_fwd below): the model + criterion backward without
 * a dlogits tensor or the lgnn_ce_bwd launch (reference models/base.py:93-94 + :196-201). The
 * same arithmetic as lgnn_ce_bwd followed by lgnn_gcn_stack_bwd_s3f_all, bitwise. */
struct lgnn_ce_src;
int lgnn_gcn_stack_bwd_s3f_ce(const int64_t* batch, const int32_t* gptr, int pool_mean,
                              int64_t num_graphs, const int32_t* rowptr, const int32_t* col,
                              const float* w, const int32_t* tptr, const int32_t* tidx,
                              const float* tw, const float* X, int64_t M, int L,
                              const uint16_t* planes_t, const float* const* W,
                              const float* const* H, const float* const* S, const int* widths,
                              float* const* dWp, float* const* dbp, int num_partials,
                              float* dS_ws, int32_t* tile_open, const struct lgnn_ce_src* ce,
                              const float* Wout, int num_classes, const void* adjt,
                              void* stream);

/* ---------------------------------------------------------------------------------------------
 * Dense GEMMs at fp32 accuracy on bf16 MFMA ("split-3"), any width. Replace: the plain
 * nn.Linear shapes outside the 128-feature tile kernels — the reference's fp32 in_proj
 * nn.Linear(1025, 128) (src/lesion_gnn/models/gat.py:29; configs/config.py:52-65) and every
 * GATConv.lin / GraphConv / in_proj wider than 128 (scripts/sweep.py:126) — forward and backward,
 * i.e. the cuBLAS addmm / mm torch runs for them.
 * Every fp32 operand is held as three bf16 planes x = hi + mid + lo (each the RNE bf16 of what the
 * planes above left) and a product as the six plane products reaching 2^-24: fp32-class results
 * (error comparable to an fp32 GEMM's). planes = 1 instead rounds each operand once to bf16 (RNE)
 * and accumulates in fp32 (the bf16 GEMM mode of BASELINE config C3, any width).
 * lgnn_s3_weight_planes: the weight operand of lgnn_s3_gemm for B = W [rows][cols] (transposed 0:
 *   Y = A W^T) or B = W^T (transposed 1: Y = A W), i.e. [ceil(out/128)][planes][128][kpad(in)]
 *   bf16 in MFMA fragment order, zero-padded; lgnn_s3_weight_planes_numel(out, in, planes) its
 *   size in elements (out = B's rows, in = B's columns).
 * lgnn_s3_weight_planes_multi: n (<= LGNN_MAX_WPREP) such operands in ONE launch (job j: W[j],
 *   rows[j], cols[j], transposed[j] -> Wp[j]; planes shared) — a model's every weight operand of a
 *   step (forward B = W and backward B = W^T) at once instead of one small launch per GEMM.
 * lgnn_s3_gemm_att: lgnn_s3_gemm (planes = 3) for a GATConv.lin (N = heads * C <= 128, no bias) that also
 *   writes the attention scores a_s[m][h] = <Y[m][hC ..), att_src[h]>, a_d likewise ([M][heads],
 *   one fmaf chain over the head's C features in feature order) — replaces lgnn_gat_att's pass.
 * lgnn_s3_gemm: Y[M][N] = A[M][K] B[N][K]^T (+ bias[N]), A fp32 (split or rounded as loaded).
 *   colsum_part (nullable): [ceil(M/64)][N] per-64-row-tile column sums of Y (fixed order).
 * lgnn_s3_wgrad: partial slabs of dW[N][K] = dY^T X (dY [M][N], X [M][K] fp32, N even):
 *   partials [num_partials][N][K], num_partials = lgnn_s3_wgrad_partials(M, K, N), summed in fixed
 *   order by lgnn_reduce_partials(_multi); db_partials (nullable) [num_partials][N] the matching
 *   column sums of dY (the bias gradient).
 * ------------------------------------------------------------------------------------------- */
size_t lgnn_s3_weight_planes_numel(int out_features, int in_features, int planes);
int lgnn_s3_weight_planes(const float* W, int rows, int cols, int transposed, int planes,
                          uint16_t* Wp, void* stream);
#define LGNN_MAX_WPREP 16
int lgnn_s3_weight_planes_multi(int n, const float* const* W, const int* rows, const int* cols,
                                const int* transposed, int planes, uint16_t* const* Wp,
                                void* stream);
int lgnn_s3_gemm(const float* A, int64_t M, int K, const uint16_t* Wp, int N, int planes,
                 const float* bias, float* Y, float* colsum_part, void* stream);
int lgnn_s3_gemm_att(const float* A, int64_t M, int K, const uint16_t* Wp, int N, int planes,
                     float* Y, const float* att_src, const float* att_dst, int heads, int C,
                     float* a_s, float* a_d, void* stream);
int lgnn_s3_wgrad_partials(int64_t M, int K, int N);
int lgnn_s3_wgrad(const float* dY, int N, const float* X, int64_t M, int K, int planes,
                  float* partials, int num_partials, float* db_partials, void* stream);
/* lgnn_s3_gemm_act (ABI v37): lgnn_s3_gemm (planes = 3, no column sums) with the activation in
 * the epilogue, Y = act(A B^T + b) (LGNN_ACT_ELU = torch's F.elu, reference gin.py:31) — the wide
 * (K or N > 128) GIN / GCN linears of the reference sweep (scripts/sweep.py:126) */
int lgnn_s3_gemm_act(const float* A, int64_t M, int K, const uint16_t* Wp, int N,
                     const float* bias, int act, float* Y, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Dropout. Replaces: the Bernoulli draws of torch's dropout on the hot path — nn.Dropout between
 * GIN convs (reference src/lesion_gnn/models/gin.py:27,32), the Dropout of PyG's MLP after each
 * BatchNorm + ELU (gin.py:23) and GATConv's attention dropout (gat.py:31; PyG 2.5.1
 * F.dropout(alpha, p) before the aggregation).
 * lgnn_dropout_masks: num_masks (<= LGNN_MAX_MASKS) fp32 masks in ONE launch; mask j (host arrays:
 *   out[j] device pointer, 16-B aligned, numel[j] elements, thr[j], scale[j]) holds
 *     out[j][i] = u(j, i) >= thr[j] ? scale[j] : 0,
 *     u(j, i) = mix(key + j * 0xD1B54A32D192ED03 + i * G) >> 40,  key = mix(seed ^ counter * G),
 *   mix = the splitmix64 finalizer, G = 0x9E3779B97F4A7C15, thr = (uint32)(p * 2^24) (<= 2^24),
 *   scale = fp32(1 / (1 - p)). state: device uint64[8] = [seed, counter, ticket words (zero)]; with
 *   advance != 0 the launch increments the counter when done (a captured graph draws fresh masks
 *   per replay). The masks are a pure function of (seed, counter, j, i): the CPU oracle
 *   regenerates them bit for bit (parity with dropout on).
 * lgnn_mask_mul: y = x * mask elementwise (n floats, 16-B aligned; y may alias x) — the dropout
 *   product and its backward dx = dy * mask.
 * ------------------------------------------------------------------------------------------- */
#define LGNN_MAX_MASKS 16
int lgnn_dropout_masks(int num_masks, float* const* out, const int64_t* numel,
                       const uint32_t* thr, const float* scale, uint64_t* state, int advance,
                       void* stream);
int lgnn_mask_mul(const float* x, const float* mask, float* y, int64_t n, void* stream);
/* lgnn_act_bwd (ABI v37): dZ = dY * act'(H) elementwise from the activation's saved output H
 * (act = LGNN_ACT_ELU: 1 where H > 0, H + 1 elsewhere — F.elu's autograd, reference gin.py:31);
 * n floats, 16-B aligned; dZ may alias dY */
int lgnn_act_bwd(const float* dY, const float* H, float* dZ, int64_t n, int act, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Sort pooling (DGCNN). Replaces: PyG 2.5.1 SortAggregation(k) as DRGNet applies it to the
 * concatenated GraphConv outputs (reference src/lesion_gnn/models/drgnet.py:37, called at :59).
 *   x [M, D] fp32 (rows of one graph contiguous, PyG Batch order), gptr [B+1] int32 (Batch.ptr);
 *   out [B, k*D]: per graph the rows sorted by the LAST channel descending (ties: node order,
 *   i.e. a stable sort), the first k kept, missing rows 0; fill = min(x) - 1 and every element
 *   equal to fill is 0 (PyG's masked_fill). rank [M] int32: each node's output row, or -1;
 *   fill [1]: device float, written (read by the backward). Workspace:
 *   lgnn_sort_pool_workspace_bytes(). 1 <= k <= 4096. Two launches.
 * lgnn_sort_pool_bwd: dx [M, D] = dout[batch[i], rank[i], :] where rank[i] >= 0 and
 *   x[i, d] != fill, else 0. One launch.
 * ------------------------------------------------------------------------------------------- */
size_t lgnn_sort_pool_workspace_bytes(void);
int lgnn_sort_pool_fwd(const float* x, int64_t num_nodes, int dims, const int32_t* gptr,
                       int64_t num_graphs, int k, float* out, int32_t* rank, float* fill,
                       void* workspace, size_t workspace_bytes, void* stream);
int lgnn_sort_pool_bwd(const float* dout, const float* x, const int32_t* rank,
                       const int64_t* batch, const float* fill, int64_t num_nodes, int dims,
                       int k, float* dx, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Lesion-node feature pooling. Replaces: extract_features_by_cc (reference
 * src/lesion_gnn/datasets/nodes/lesions.py:88-93, called at :172) — torch_scatter
 * scatter(features.view(C, H*W).T, cc.flatten(), 0, reduce) with reduce "mean" or "max"
 * (FeaturesReduction, lesions.py:62-64).
 *   features [C, num_pixels] fp32 channel-major (the encoder's (1, C, H, W), contiguous);
 *   cc [num_pixels] int64 component labels; out [num_segments, C] fp32 (num_segments =
 *   max(cc) + 1 as PyG sizes it): mean = sum / max(count, 1); max of an empty segment = 0.
 *   Labels outside [0, num_segments) are skipped and counted in *err (written). counts_out
 *   [num_segments] int32 (nullable): pixels per label. 1 <= num_segments <= 4032. Workspace:
 *   lgnn_cc_pool_workspace_bytes. Two launches + two memsets, no host synchronisation.
 * ------------------------------------------------------------------------------------------- */
size_t lgnn_cc_pool_workspace_bytes(int64_t num_pixels, int channels, int num_segments);
int lgnn_cc_pool(const float* features, int channels, int64_t num_pixels, const int64_t* cc,
                 int num_segments, int reduce_max, float* out, int32_t* counts_out, int32_t* err,
                 void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * bf16 dense GEMMs (bf16 GEMM operands rounded round-to-nearest-even as torch's
 * .to(torch.bfloat16), fp32 accumulation and output). Replace the bf16 nn.Linear / GATConv.lin
 * GEMMs of the bf16 configuration — in_proj (reference src/lesion_gnn/models/gat.py:29,
 * nn.Linear(1025, 128)) and GATConv.lin (gat.py:31, PyG Linear(bias=False)) — forward and
 * backward. Weight operands: lgnn_bf16_weight_prep writes Wb = bf16 W as a zero-padded
 * [128][lgnn_bf16_kpad(K)] matrix and, when WTb != NULL (requires K <= 128), WTb = bf16 W^T as
 * [128][lgnn_bf16_kpad(N)], both in MFMA fragment order: element (r, q) at
 * ((((q / 16) * 4 + r / 32) * 64 + 32 ((q / 8) & 1) + r % 32) * 8 + q % 8.
 *   lgnn_bf16_gemm: Y[M][N] = A[M][K] W^T (+ bias), N <= 128; A fp32 (a_is_f32 = 1, rounded
 *     as loaded, any K) or bf16 (K % 4 == 0); writes Y fp32 and/or Yb bf16 (either nullable);
 *     colsum_part (nullable) [ceil(M / 64)][N]: each 64-row tile's column sums of Y (sum them
 *     with lgnn_reduce_partials: the bias gradient of a following Linear, fixed order).
 *     For dX: A = dY (bf16, K = N), Wb = WTb, N = K.
 *   lgnn_bf16_wgrad: partials [num_partials][N][K] of dW = dY^T X (dYb bf16 [M][N], N even;
 *     X fp32 or bf16 [M][K]); num_partials from lgnn_bf16_wgrad_partials(M, K); sum them with
 *     lgnn_reduce_partials (fixed order). M * K * 4 < 2^31 for both entries.
 * ------------------------------------------------------------------------------------------- */
int lgnn_bf16_kpad(int K);
int lgnn_bf16_weight_prep(const float* W, int N, int K, uint16_t* Wb, uint16_t* WTb,
                          void* stream);
/* lgnn_bf16_weight_prep for n <= 8 weights in one launch (ABI v20): W[j] [N[j]][K[j]] fp32 ->
 * Wb[j] (and WTb[j], nullable, when K[j] <= 128), the same operands as n separate calls. The
 * bf16 GAT forward prepares in_proj's and every GATConv.lin's operands this way once per step. */
int lgnn_bf16_weight_prep_multi(int n, const float* const* W, const int* N, const int* K,
                                uint16_t* const* Wb, uint16_t* const* WTb, void* stream);
int lgnn_bf16_gemm(const void* A, int a_is_f32, int64_t M, int K, const uint16_t* Wb,
                   const float* bias, int N, float* Y, uint16_t* Yb, float* colsum_part,
                   void* stream);
/* lgnn_bf16_gemm for GATConv.lin's forward with the attention scores in its epilogue (ABI v24):
 * Y = bf16(A) bf16(W)^T (A bf16, or fp32 rounded as loaded; 64 < K <= 128; no bias;
 * N = H * C <= 128) and
 * a_s[m][h] = <Y[m][hC .. hC + C), att_src[h]>, a_d likewise with att_dst (PyG GATConv
 * alpha_src / alpha_dst, reference gat.py:31), so lgnn_gat_att does not run. */
int lgnn_bf16_gemm_att(const void* A, int a_is_f32, int64_t M, int K, const uint16_t* Wb, int N,
                       float* Y, uint16_t* Yb, const float* att_src, const float* att_dst, int H,
                       int C, float* a_s, float* a_d, void* stream);
int lgnn_bf16_wgrad_partials(int64_t M, int K);
int lgnn_bf16_wgrad(const uint16_t* dYb, int N, const void* X, int x_is_f32, int64_t M, int K,
                    float* partials, int num_partials, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LGNN_H */
