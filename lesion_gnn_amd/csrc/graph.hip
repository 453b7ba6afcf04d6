// Graph-structure kernels: edge_index (int64 COO, any order) -> CSR by target + CSR by source,
// with PyG 2.5.1 self-loop semantics and GCN normalisation; Batch.ptr from `batch`.
//
// Replaces (reference call sites): gcn_norm inside GCNConv, GATConv's
// remove_self_loops/add_self_loops (gat.py:31), ToSparseTensor (datasets/datamodule.py:44-45).
//
// Pipeline (one memset + 5 kernels, no host sync):
//   k_count   per-edge in/out degree; runs of equal targets inside a wave (k-NN input is grouped by
//             target) are folded into one atomic
//   k_scan_*  rowptr / tptr = exclusive scans of (degree + appended loop), both arrays per
//             launch; dis = deg^-1/2 for the GCN weights
//   k_fill    claim slots (same run folding), write (source, edge id)
//   k_finish  per 16-row block (one wave): stage the entries in LDS, append the self loop, place
//             each entry at its rank by edge id within its row (restores edge_index order: the
//             order PyG's scatter_add_ visits a target's messages in), compute GCN weights,
//             write back. Run for both CSRs.
// The result is identical run to run.
#include "common.h"
#include "tile_util.h"
#include "s3_util.h"

namespace {

constexpr int kThreads = 256;
constexpr int kFinR = 16;          // k_finish: rows per wave (virtual block)
constexpr int kFinishCap = 1024;   // staged CSR entries per k_finish virtual block
constexpr int kFinGrid = 1024;     // k_finish: workgroup cap (grid-stride over virtual blocks)
// Target-sorted fast path (k_prep_sorted + the sorted body of k_scan): rows of at most
// kSortedRowCap CSR entries (a 64-row tile then stays within the fused kernels' CAPE_TILE
// entries: k <= 32, the reference sweep's range), runs of at most kGapCap rows without entries,
// at most one self loop per row
constexpr int kSortedRowCap = 32;
static_assert(kSortedRowCap * 64 <= lgnn_tile::CAPE_TILE, "a sorted tile fits the closed cap");
constexpr int kGapCap = 64;
constexpr int kVerdictMax = 1024;  // k_prep_sorted workgroups (one verdict word each)
constexpr int kSortedChunks = 2;   // k_prep_sorted: 64-edge chunks per wave pass (more waves in flight)
constexpr int kSortedRows = 256;   // k_scan's sorted body: rows per workgroup (one per thread)

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

inline size_t scan_bsum_bytes(int64_t N) {
  // 2 arrays x blocks of 1024 elements; the sorted path's scan: one word per 256 rows (4 per
  // 1024), then the sorted-open mode's source scan (one per 1024 rows) after them
  return (size_t)4 * 5 * ((N + 1 + 1023) / 1024);
}

struct GraphWs {
  int32_t* err;    // [1] dropped edges (zeroed with the counters, copied to err_count)
  int32_t* cnt;    // [N+1] in-degree without loops
  int32_t* tcnt;   // [N+1]
  int32_t* stat;   // [2 * scan blocks] chained-scan block prefixes, flagged (zeroed)
  int32_t* fill;   // [N] next free slot of each row (set by the scan)
  int32_t* tfill;  // [N]
  int32_t* eid;    // [E+N]
  int32_t* teid;   // [E+N]
  int32_t* inv;    // [E+N] edge id -> target-CSR position (for tmap)
  float* dis;      // [N] deg^-1/2 (GCN normalisation), inf -> 0
  int32_t* rs;     // [N+1] sorted path: first input edge of each row (rs[N] = E)
  int32_t* scnt;   // [N] sorted path: entries of each row without its self loop
  int32_t* lp;     // [N] sorted path: offset of the row's self loop in its input run, or -1
  int32_t* verdict;  // [kVerdictMax + 1] sorted path: one word per k_prep_sorted workgroup, then
                     // the summary k_scan writes for k_fill / k_finish
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
  ws.err = (int32_t*)take(4);
  ws.cnt = (int32_t*)take((N + 1) * 4);
  ws.tcnt = (int32_t*)take((N + 1) * 4);
  ws.stat = (int32_t*)take(scan_bsum_bytes(N));
  ws.zero_bytes = (size_t)(p - static_cast<char*>(base));
  ws.fill = (int32_t*)take(N * 4);
  ws.tfill = (int32_t*)take(N * 4);
  ws.eid = (int32_t*)take((E + N) * 4);
  ws.teid = (int32_t*)take((E + N) * 4);
  ws.inv = (int32_t*)take((E + N) * 4);
  ws.dis = (float*)take(N * 4);
  ws.rs = (int32_t*)take((N + 1) * 4);
  ws.scnt = (int32_t*)take(N * 4);
  ws.lp = (int32_t*)take(N * 4);
  ws.verdict = (int32_t*)take((kVerdictMax + 1) * 4);
  return ws;
}

size_t ws_total(int64_t N, int64_t E) {
  return align_up(4) + 3 * align_up((N + 1) * 4) + 5 * align_up(N * 4) + 3 * align_up((E + N) * 4) +
         2 * align_up(scan_bsum_bytes(N)) + align_up((kVerdictMax + 1) * 4) + 256;
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

// First launch of a build: zero the counters, scan flags and tile flags (ntiles + the count),
// and, when a batch vector is given, the graph offsets (as lgnn_batch_ptr).
__device__ __forceinline__ void prep_body(int32_t* __restrict__ zero, int64_t nzero,
                                          int32_t* __restrict__ tile_open, int64_t ntiles,
                                          const int64_t* __restrict__ batch, int64_t M, int64_t B,
                                          int32_t* __restrict__ gptr, int bx, int gx) {
  const int64_t i0 = (int64_t)bx * kThreads + threadIdx.x;
  const int64_t step = (int64_t)gx * kThreads;
  for (int64_t i = i0; i < nzero; i += step) zero[i] = 0;
  if (tile_open)  // flags, their count, and the fused kernels' grid-barrier words
    for (int64_t t = i0; t < ntiles + LGNN_TILE_OPEN_EXTRA; t += step) tile_open[t] = 0;
  if (gptr) {
    for (int64_t i = i0; i <= M; i += step) {
      // graphs q with prev < q <= cur start at node i (prev = batch[i-1] or -1; cur = batch[i]
      // or B)
      int64_t prev = i == 0 ? -1 : batch[i - 1];
      int64_t cur = i == M ? B : batch[i];
      if (prev < -1) prev = -1;
      if (cur > B) cur = B;
      for (int64_t q = prev + 1; q <= cur; ++q) gptr[q] = (int32_t)i;
    }
  }
}

// workgroups past the build's own grid (gx) run the weight-plane side job (lgnn_graph_build_planes)
__device__ __forceinline__ bool plane_side_job(const lgnn_s3::PlaneArgs& pj, int gx) {
  if ((int)blockIdx.x < gx) return false;
  lgnn_s3::wplanes_item(pj, ((int)blockIdx.x - gx) * kThreads + threadIdx.x);
  return true;
}

__global__ __launch_bounds__(kThreads) void k_prep(int32_t* __restrict__ zero, int64_t nzero,
                                                   int32_t* __restrict__ tile_open,
                                                   int64_t ntiles,
                                                   const int64_t* __restrict__ batch, int64_t M,
                                                   int64_t B, int32_t* __restrict__ gptr,
                                                   lgnn_s3::PlaneArgs pj, int gx) {
  if (plane_side_job(pj, gx)) return;
  prep_body(zero, nzero, tile_open, ntiles, batch, M, B, gptr, blockIdx.x, gx);
}

// ---------------------------------------------------------------------------------------------
// Target-sorted fast path. k-NN input (PyG knn_graph per graph, collated in graph order) arrives
// grouped by target with rows in ascending order: each row's messages are one contiguous run of
// edge_index, already in edge-id order, so the counting sort (count / fill / finish) reduces to a
// scan of the row lengths and a coalesced copy. The first launch (k_prep_sorted, in place of
// k_prep) does k_prep's zeroing and, per edge, checks the input: targets non-decreasing, indices
// in range, at most one self loop per row, rows of at most kSortedRowCap entries, empty-row runs
// of at most kGapCap, and (lazy build) no edge leaving its 64-row tile — any failure sends the
// build down the general launches. The head edge of each row records the row's run (rs, scnt,
// lp) and dis. Every workgroup writes its verdict word (no zeroing needed); the later launches
// OR the words: all clear -> k_scan writes the CSR (sorted body) and k_count / k_fill / k_finish
// return at once; else they run as before and k_scan runs its scan. The CSR is bit-identical to
// the general path's: same entry order (the row's edges in edge-id order, its self loop last),
// the same weight expression.
struct SortedArgs {
  const int64_t* ei;
  int64_t E;
  int loops, add_loop, norm, need_closed;
  int32_t *rs, *scnt, *lp;
  float* dis;
  int32_t* verdict;
  int nverdict;
  int summary_ready;  // k_count ran: verdict[kVerdictMax] already holds the OR of the words
};

__device__ __forceinline__ void sorted_empty_row(const SortedArgs& a, int64_t r, int64_t start) {
  a.rs[r] = (int32_t)start;
  a.scnt[r] = 0;
  a.lp[r] = -1;
  a.dis[r] = a.add_loop ? 1.0f / sqrtf(1.0f) : 0.0f;
}

__global__ __launch_bounds__(kThreads) void k_prep_sorted(int32_t* __restrict__ zero,
                                                          int64_t nzero,
                                                          int32_t* __restrict__ tile_open,
                                                          int64_t ntiles,
                                                          const int64_t* __restrict__ batch,
                                                          int64_t M, int64_t B,
                                                          int32_t* __restrict__ gptr,
                                                          SortedArgs a, lgnn_s3::PlaneArgs pj,
                                                          int gx) {
  if (plane_side_job(pj, gx)) return;  // (block-uniform: before any barrier)
  constexpr int CH = kSortedChunks;
  const int64_t E = a.E, N = M;
  const int64_t* __restrict__ src = a.ei;
  const int64_t* __restrict__ dst = a.ei + E;
  const bool drop_loops = a.loops != LGNN_LOOPS_KEEP;
  const int lane = threadIdx.x & 63;
  const int64_t wv = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int64_t nwv = ((int64_t)gx * kThreads) >> 6;
  int bad = 0;
  bool prepped = false;
  // a wave takes CH chunks of 64 consecutive edges (+ one chunk of look-ahead for the row that
  // runs past the last one), every load issued up front; rows are found by wave run detection.
  // k_prep's zeroing runs behind the first pass's loads.
  for (int64_t base = wv * 64 * CH; base < E; base += nwv * 64 * CH) {
    int64_t s[CH + 1], d[CH + 1];
#pragma unroll
    for (int c = 0; c <= CH; ++c) {
      const int64_t e = base + 64 * c + lane;
      s[c] = e < E ? src[e] : -1;
      d[c] = e < E ? dst[e] : -1;
    }
    const int64_t before = base > 0 ? dst[base - 1] : -1;
    if (!prepped) {
      prep_body(zero, nzero, tile_open, ntiles, batch, M, B, gptr, blockIdx.x, gx);
      prepped = true;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t e = base + 64 * c + lane;
      const bool in = e < E;
      const int64_t last_prev = c == 0 ? before : __shfl(d[c - 1], 63, 64);
      int64_t dp = __shfl_up(d[c], 1, 64);
      if (lane == 0) dp = last_prev;
      const Run r = wave_run(in ? d[c] : -2 - lane);
      const unsigned long long lm = __ballot(in && drop_loops && s[c] == d[c]);
      // the chunk's last row continuing into the next chunk: its leading lanes with the same
      // target (sorted input), and the self loops among them
      const int64_t dl = __shfl(d[c], 63, 64);
      const unsigned long long cm = __ballot(dl >= 0 && d[c + 1] == dl);
      const unsigned long long clm = __ballot(drop_loops && d[c + 1] >= 0 && s[c + 1] == d[c + 1]);
      const int clen = ~cm == 0 ? 64 : __ffsll((long long)~cm) - 1;
      const unsigned long long cmask = clen >= 64 ? ~0ull : (1ull << clen) - 1;
      if (!in) continue;
      const int64_t sv = s[c], dv = d[c];
      if (drop_loops && sv == dv) bad |= 4;  // a dropped input self loop (k_scan: scan needed)
      if (!edge_ok(sv, dv, N) || dp > dv) {
        bad |= 1;
        continue;
      }
      // an edge leaving its tile: the lazy build needs the source CSR (sorted-open mode)
      if (a.need_closed && (sv >> 6) != (dv >> 6)) bad |= 2;
      if (dv != dp) {  // head of row dv: the rows since the previous target have no entries
        const int64_t r0 = dp < 0 ? 0 : dp + 1;
        if (dv - r0 > kGapCap) {
          bad |= 1;
        } else {
          for (int64_t q = r0; q < dv; ++q) sorted_empty_row(a, q, e);
          if (r0 < dv) bad |= 8;  // a row without a (dropped) self loop
        }
        const unsigned long long run = (r.len >= 64 ? ~0ull : ((1ull << r.len) - 1)) << lane;
        int n = r.len, nl = __popcll(lm & run);
        int lpos = nl ? __ffsll((long long)(lm & run)) - 1 - lane : -1;
        if (lane + r.len == 64) {
          const int cl = __popcll(clm & cmask);
          if (nl == 0 && cl) lpos = r.len + __ffsll((long long)(clm & cmask)) - 1;
          nl += cl;
          n += clen;
          if (clen == 64) bad |= 1;  // longer than any row the fast path takes
        }
        const int deg = n - nl;
        if (nl == 0) bad |= 8;
        if (n > kSortedRowCap + 1 || nl > 1 || deg + a.add_loop > kSortedRowCap) bad |= 1;
        a.rs[dv] = (int32_t)e;
        a.scnt[dv] = deg;
        a.lp[dv] = nl ? lpos : -1;
        const int dg = deg + a.add_loop;
        a.dis[dv] = dg > 0 ? 1.0f / sqrtf((float)dg) : 0.0f;
      }
      if (e == E - 1) {  // rows after the last target
        if (N - 1 - dv > kGapCap) {
          bad |= 1;
        } else {
          for (int64_t q = dv + 1; q < N; ++q) sorted_empty_row(a, q, E);
          if (dv + 1 < N) bad |= 8;
        }
        a.rs[N] = (int32_t)E;
      }
    }
  }
  if (!prepped) prep_body(zero, nzero, tile_open, ntiles, batch, M, B, gptr, blockIdx.x, gx);
  const int b1 = __syncthreads_or(bad & 1), b2 = __syncthreads_or(bad & 2);
  const int b4 = __syncthreads_or(bad & 4), b8 = __syncthreads_or(bad & 8);
  if (threadIdx.x == 0)
    a.verdict[blockIdx.x] = (b1 ? 1 : 0) | (b2 ? 2 : 0) | (b4 ? 4 : 0) | (b8 ? 8 : 0);
}

// The build mode from k_prep_sorted's verdict words (block-uniform, every thread must call it):
//   kModeSorted: target-sorted, every tile closed -> k_scan's sorted body writes the CSR, the
//                general launches return at once (no source CSR is needed);
//   kModeSortedOpen: target-sorted but some edge leaves its tile (lazy build) -> the sorted body
//                writes the target CSR, the general launches build only the source CSR;
//   kModeGeneral: the counting sort for both.
// The summary word (verdict[kVerdictMax]) is the mode | kNoDrop when no input self loop is dropped
// (graphs built with loop = False, or loops kept) | kAllDrop when every row drops exactly one
// (k-NN with loop = True: each node is its own nearest neighbour, configs/config.py:47): the
// sorted body's rowptr is then rs[d] + d * add_loop (- d) directly, with no scan across
// workgroups. Readers mask with kModeMask.
constexpr int kModeGeneral = 0, kModeSorted = 1, kModeSortedOpen = 2;
constexpr int kModeMask = 3, kNoDrop = 4, kAllDrop = 8;
__device__ __forceinline__ int sorted_mode(const int32_t* verdict, int nverdict) {
  if (!verdict) return kModeGeneral;
  int v = 0;
  for (int i = threadIdx.x; i < nverdict; i += blockDim.x) v |= verdict[i];
  const int b1 = __syncthreads_or(v & 1), b2 = __syncthreads_or(v & 2);
  const int b4 = __syncthreads_or(v & 4), b8 = __syncthreads_or(v & 8);
  const int flags = !b4 ? kNoDrop : (!b8 ? kAllDrop : 0);
  return b1 ? kModeGeneral : ((b2 ? kModeSortedOpen : kModeSorted) | flags);
}

// Edge passes. A block takes a chunk of kChunk consecutive edges, kPer per thread, so every
// wave sees 64 consecutive edges per step (run detection on targets: one atomic per run of equal
// targets). Sources are binned in LDS when the chunk's sources span fewer than kBins nodes (the
// k-NN case: a chunk covers a few graphs), so the transpose needs one global atomic per distinct
// source per chunk instead of one per edge; otherwise per-edge global atomics.
// kPer edges per thread (8; 4 when the 8-edge chunks would not give every CU a workgroup: the
// reference config's 254 k edges took 124 workgroups, count + fill 21 -> 16 us; at C5 k = 16's
// 933 k edges 4 was slower — more global atomics per edge)
constexpr int kPer = 8;
constexpr int kChunk = kThreads * kPer;
__host__ __device__ constexpr int chunk_of(int per) { return kThreads * per; }
// fewer 8-edge chunks than CUs: the edge passes take 4 edges per thread instead
static bool small_edges(int64_t E) { return (E + kChunk - 1) / kChunk < 256; }
constexpr int kBins = 4096;

template <int PER = kPer>
struct EdgeChunk {
  int64_t s[PER], d[PER];
  bool use[PER];
};

template <int PER>
__device__ __forceinline__ void load_chunk(EdgeChunk<PER>& c, const int64_t* __restrict__ ei,
                                           int64_t E, int64_t N, int loops, int64_t c0,
                                           int32_t* err) {
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int64_t e = c0 + (int64_t)it * kThreads + threadIdx.x;
    int64_t s = -1, d = -1;
    if (e < E) {
      s = ei[e];
      d = ei[E + e];
    }
    const bool valid = e < E && edge_ok(s, d, N);
    if (e < E && !valid && err) atomicAdd(err, 1);
    c.s[it] = s;
    c.d[it] = d;
    c.use[it] = valid && !(loops != LGNN_LOOPS_KEEP && s == d);
  }
}

// block-uniform: the chunk's smallest used source and whether all used sources fit the bins
template <int PER>
__device__ __forceinline__ bool chunk_binned(const EdgeChunk<PER>& c, int64_t& smin, int* red) {
  int64_t lo = INT64_MAX, hi = -1;
#pragma unroll
  for (int it = 0; it < PER; ++it)
    if (c.use[it]) {
      lo = c.s[it] < lo ? c.s[it] : lo;
      hi = c.s[it] > hi ? c.s[it] : hi;
    }
  int lo32 = lo == INT64_MAX ? INT32_MAX : (int)lo, hi32 = (int)hi;
  for (int o = 32; o > 0; o >>= 1) {
    const int a = __shfl_xor(lo32, o, 64), b = __shfl_xor(hi32, o, 64);
    lo32 = a < lo32 ? a : lo32;
    hi32 = b > hi32 ? b : hi32;
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * wave] = lo32;
    red[2 * wave + 1] = hi32;
  }
  __syncthreads();
  int L = INT32_MAX, H = -1;
  for (int w = 0; w < kThreads / 64; ++w) {
    L = red[2 * w] < L ? red[2 * w] : L;
    H = red[2 * w + 1] > H ? red[2 * w + 1] : H;
  }
  smin = L;
  return H < 0 || H - L < kBins;
}

// open-tile flag setter: the first writer of a tile also counts it (tile_open[ntiles])
__device__ __forceinline__ void mark_open(int32_t* tile_open, int64_t t, int64_t ntiles) {
  if (atomicCAS(&tile_open[t], 0, 1) == 0) atomicAdd(&tile_open[ntiles], 1);
}

// count_body's tile marks are first collected per workgroup in LDS (kMarkWin tiles around the
// chunk's first target): many edges of a chunk leave the same few tiles (C5: graphs straddling
// tiles), and their racing first-marker atomics on one word serialised (~50 us at k = 16)
constexpr int kMarkWin = 64;

template <int PER = kPer>
__device__ __forceinline__ void count_body(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                                           int loops, int32_t* cnt, int32_t* tcnt, int32_t* err,
                                           int32_t* tile_open, int* hist, int* red, int64_t bx,
                                           int* tmk = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t c0 = bx * chunk_of(PER);
  EdgeChunk<PER> c;
  load_chunk(c, ei, E, N, loops, c0, err);
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const Run r = wave_run(c.use[it] ? c.d[it] : -2 - lane);
    if (cnt && c.use[it] && r.head) atomicAdd(&cnt[c.d[it]], r.len);
  }
  if (tile_open) {  // lazy transpose: the tiles an edge leaves are known before the fill
    const int64_t ntiles = (N + 63) >> 6;
    int64_t tb = 0;
    if (tmk) {
      const int64_t d0 = E > 0 ? ei[E + (c0 < E ? c0 : E - 1)] : 0;
      tb = (d0 >> 6) - kMarkWin / 2;
      for (int q = threadIdx.x; q < kMarkWin; q += kThreads) tmk[q] = 0;
      __syncthreads();
    }
    auto mk = [&](int64_t t) {
      const int64_t rel = t - tb;
      if (tmk && rel >= 0 && rel < kMarkWin) tmk[rel] = 1;  // idempotent plain store
      else if (tile_open[t] == 0) mark_open(tile_open, t, ntiles);
    };
#pragma unroll
    for (int it = 0; it < PER; ++it)
      if (c.use[it] && (c.s[it] >> 6) != (c.d[it] >> 6)) {
        mk(c.d[it] >> 6);
        mk(c.s[it] >> 6);
      }
    if (tmk) {
      __syncthreads();
      for (int q = threadIdx.x; q < kMarkWin; q += kThreads)
        if (tmk[q] && tile_open[tb + q] == 0) mark_open(tile_open, tb + q, ntiles);
    }
  }
  if (!tcnt) return;
  int64_t smin;
  if (chunk_binned(c, smin, red)) {
    for (int b = threadIdx.x; b < kBins; b += kThreads) hist[b] = 0;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it)
      if (c.use[it]) atomicAdd(&hist[c.s[it] - smin], 1);
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += kThreads)
      if (hist[b]) atomicAdd(&tcnt[smin + b], hist[b]);
  } else {
#pragma unroll
    for (int it = 0; it < PER; ++it)
      if (c.use[it]) atomicAdd(&tcnt[c.s[it]], 1);
  }
}

template <int PER>
__global__ __launch_bounds__(kThreads) void k_count(const int64_t* __restrict__ ei, int64_t E,
                                                    int64_t N, int loops, int32_t* cnt,
                                                    int32_t* tcnt, int32_t* err,
                                                    int32_t* tile_open,
                                                    int32_t* verdict, int nverdict) {
  __shared__ int hist[kBins];
  __shared__ int red[2 * kThreads / 64];
  __shared__ int tmk[kMarkWin];
  const int summary = sorted_mode(verdict, nverdict), mode = summary & kModeMask;
  // the summary word for k_scan / k_fill / k_finish (one word to read instead of all of them)
  if (verdict && blockIdx.x == 0 && threadIdx.x == 0) verdict[kVerdictMax] = summary;
  if (mode == kModeSorted) return;
  count_body<PER>(ei, E, N, loops, mode == kModeSortedOpen ? nullptr : cnt, tcnt, err, tile_open,
                  hist, red, blockIdx.x, tmk);
}

// fill[d] / tfill[s] start at the row offsets (set by k_scan); slots come from atomics on them,
// so the order inside a row is arbitrary here and restored by k_finish (sort by edge id).
template <int PER = kPer>
__device__ __forceinline__ void fill_body(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                                          int loops, const int32_t* __restrict__ rowptr,
                                          int32_t* fill, int32_t* col, int32_t* eid,
                                          const int32_t* __restrict__ tptr, int32_t* tfill,
                                          int32_t* tidx, int32_t* teid, const int32_t* lazy_open,
                                          int* hist, int* red, int64_t bx) {
  const int lane = threadIdx.x & 63;
  const int64_t c0 = bx * chunk_of(PER);
  EdgeChunk<PER> c;
  load_chunk(c, ei, E, N, loops, c0, nullptr);
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    if (!fill) break;  // sorted-open mode: the target CSR comes from k_scan's sorted body
    const int64_t e = c0 + (int64_t)it * kThreads + threadIdx.x;
    const Run r = wave_run(c.use[it] ? c.d[it] : -2 - lane);
    int slot0 = 0;
    if (c.use[it] && r.head) slot0 = atomicAdd(&fill[c.d[it]], r.len);
    slot0 = __shfl(slot0, r.head_lane, 64);
    if (c.use[it]) {
      const int pos = slot0 + (lane - r.head_lane);
      col[pos] = (int32_t)c.s[it];
      eid[pos] = (int32_t)e;
    }
  }
  if (!tptr) return;
  if (lazy_open && __hip_atomic_load(lazy_open, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    return;  // lazy transpose, no open tile: the source CSR is not needed
  int64_t smin;
  if (chunk_binned(c, smin, red)) {
    for (int b = threadIdx.x; b < kBins; b += kThreads) hist[b] = 0;
    __syncthreads();
    int rank[PER];
#pragma unroll
    for (int it = 0; it < PER; ++it)
      rank[it] = c.use[it] ? atomicAdd(&hist[c.s[it] - smin], 1) : 0;
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += kThreads) {
      const int n = hist[b];
      if (n) hist[b] = atomicAdd(&tfill[smin + b], n);  // the chunk's base slot for source b
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it)
      if (c.use[it]) {
        const int pos = hist[c.s[it] - smin] + rank[it];
        tidx[pos] = (int32_t)c.d[it];
        teid[pos] = (int32_t)(c0 + (int64_t)it * kThreads + threadIdx.x);
      }
  } else {
#pragma unroll
    for (int it = 0; it < PER; ++it)
      if (c.use[it]) {
        const int pos = atomicAdd(&tfill[c.s[it]], 1);
        tidx[pos] = (int32_t)c.d[it];
        teid[pos] = (int32_t)(c0 + (int64_t)it * kThreads + threadIdx.x);
      }
  }
}

template <int PER>
__global__ __launch_bounds__(kThreads) void k_fill(const int64_t* __restrict__ ei, int64_t E,
                                                   int64_t N, int loops,
                                                   const int32_t* __restrict__ rowptr,
                                                   int32_t* fill, int32_t* col, int32_t* eid,
                                                   const int32_t* __restrict__ tptr,
                                                   int32_t* tfill, int32_t* tidx, int32_t* teid,
                                                   const int32_t* lazy_open,
                                                   const int32_t* summary) {
  __shared__ int hist[kBins];
  __shared__ int red[2 * kThreads / 64];
  const int mode = summary ? __builtin_amdgcn_readfirstlane(*summary) & kModeMask : kModeGeneral;
  if (mode == kModeSorted) return;  // the sorted path took it
  fill_body<PER>(ei, E, N, loops, rowptr, mode == kModeSortedOpen ? nullptr : fill, col, eid, tptr,
                 tfill, tidx, teid, lazy_open, hist, red, blockIdx.x);
}

// Both degree scans (blockIdx.y = 0: rowptr from cnt, 1: tptr from tcnt) in ONE launch over
// 1024-element blocks: block b sums its elements and publishes the sum (flagged) in stat[b] at
// once; its 256 threads then read the sums of blocks 0..b-1 in parallel (each spinning until its
// entry is flagged — a block publishes before it waits, so the spin always ends) and add them
// in a fixed order; then the block writes the exclusive prefix of its elements (4 per thread,
// coalesced), the first free slot of each row (fill = rowptr) and, for rowptr,
// dis[i] = deg_i^-1/2 (GCN normalisation; deg 0 -> 0). One round of cross-block latency instead
// of a chain of them.
constexpr int kScanT = 256;
constexpr int kScanPer = 4;
constexpr int kScanBlk = kScanT * kScanPer;
constexpr int32_t kScanFlag = 0x40000000;  // prefix values stay below 2^30 (N + E <= INT32_MAX / 2)

__device__ __forceinline__ int scan_val(const int32_t* __restrict__ c, int64_t i, int64_t N,
                                        int add) {
  return i < N ? c[i] + add : 0;
}

struct ScanSmem {
  int wsc[kScanT / 64];
  int wpre[kScanT / 64];
  int s_pre;
};

__device__ __forceinline__ void scan_body(const int32_t* __restrict__ cnt,
                                          const int32_t* __restrict__ tcnt, int64_t N, int add,
                                          int32_t* stat, int32_t* __restrict__ rowptr,
                                          int32_t* __restrict__ tptr, int32_t* __restrict__ fill,
                                          int32_t* __restrict__ tfill, float* __restrict__ dis,
                                          int32_t* tile_open, ScanSmem& sm, int bx, int by,
                                          int nblk) {
  int* wsc = sm.wsc;
  const bool tr = by == 1;
  const int32_t* __restrict__ c = tr ? tcnt : cnt;
  int32_t* __restrict__ out = tr ? tptr : rowptr;
  int32_t* __restrict__ fl = tr ? tfill : fill;
  int32_t* st = stat + (int64_t)by * nblk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i0 = (int64_t)bx * kScanBlk + (int64_t)tid * kScanPer;
  int v[kScanPer];
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    v[j] = scan_val(c, i0 + j, N, add);
    s += v[j];
  }
  int x = s;  // inclusive scan of the thread sums
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsc[wave] = x;
  __syncthreads();
  if (tid == 0)  // relaxed: the flag word is its own payload (as in sorted_body)
    __hip_atomic_store(&st[bx], (wsc[0] + wsc[1] + wsc[2] + wsc[3]) | kScanFlag,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int pre = 0;  // sums of the preceding blocks, thread-strided, then combined in wave order
  for (int j = tid; j < bx; j += kScanT) {
    int f;
    while (((f = __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) &
            kScanFlag) == 0)
      __builtin_amdgcn_s_sleep(1);
    pre += f & (kScanFlag - 1);
  }
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (lane == 0) sm.wpre[wave] = pre;
  __syncthreads();
  if (tid == 0) sm.s_pre = sm.wpre[0] + sm.wpre[1] + sm.wpre[2] + sm.wpre[3];
  __syncthreads();
  int run = sm.s_pre + x - s;
  for (int w = 0; w < wave; ++w) run += wsc[w];
  if (!tr && tile_open) {  // lazy transpose: tiles with more CSR entries than a tile stages
    int ts = s;            // (a 64-row tile = 16 threads' elements; tiles never straddle blocks)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) ts += __shfl_xor(ts, o, 64);
    if ((tid & 15) == 0 && i0 < N && ts > lgnn_tile::CAPE_TILE) {
      const int64_t t = i0 >> 6;
      if (tile_open[t] == 0) mark_open(tile_open, t, (N + 63) >> 6);
    }
  }
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    const int64_t i = i0 + j;
    if (i <= N) out[i] = run;
    if (i < N) fl[i] = run;
    if (!tr && dis && i < N) {
      const int deg = v[j];
      dis[i] = deg > 0 ? 1.0f / sqrtf((float)deg) : 0.0f;
    }
    run += v[j];
  }
}

// Sorted body of k_scan (kSortedRows rows per workgroup, one per thread): rowptr = exclusive
// scan of (entries without the self loop + the appended loop), chained across workgroups as the
// general scan; then the workgroup copies its rows' input run — one contiguous range of
// edge_index — into the CSR, coalesced, all loads of a pass issued up front: entry e of row d goes
// to rowptr[d] + (e - rs[d]), one slot less past the row's self loop (which is skipped); the
// appended loops take the last slot of each row.
struct SortedSmem {
  int32_t rp[kSortedRows + 1];
  int32_t rs[kSortedRows + 1];
  int32_t lp[kSortedRows];
  float dis[kSortedRows];
  int wsum[kSortedRows / 64];
  int wpre[kSortedRows / 64];
};

__device__ __forceinline__ void sorted_body(const SortedArgs& a, int64_t N, int32_t* stat,
                                            int32_t* __restrict__ rowptr,
                                            int32_t* __restrict__ col, float* __restrict__ w,
                                            int32_t* tile_open, int32_t* err_out, SortedSmem& ss,
                                            int bx, int scanless) {
  constexpr int PASS = 8;  // entries per thread per copy pass
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)bx * kSortedRows;
  const int nrow = (int)(N - r0 < kSortedRows ? N - r0 : kSortedRows);
  const int64_t row = r0 + tid;
  const int64_t E = a.E;
  const int64_t* __restrict__ src = a.ei;
  const int64_t* __restrict__ dst = a.ei + E;
  const bool gcn = a.norm == LGNN_NORM_GCN;
  // the copy's first pass (edge_index rows and the sources' dis) does not depend on the scan:
  // issued first, its latency overlaps the scan and the look-back
  const int in0 = a.rs[r0], in1 = a.rs[r0 + nrow];
  int64_t sv[PASS], dv[PASS];
  float ds[PASS];
  auto load_pass = [&](int e0) {
#pragma unroll
    for (int it = 0; it < PASS; ++it) {
      const int e = e0 + it * kSortedRows + tid;
      sv[it] = e < in1 ? src[e] : 0;
      dv[it] = e < in1 ? dst[e] : r0;
    }
#pragma unroll
    for (int it = 0; it < PASS; ++it) ds[it] = gcn && w ? a.dis[sv[it]] : 1.0f;
  };
  load_pass(in0);
  int v = 0;
  if (tid < nrow) {
    v = a.scnt[row] + a.add_loop;
    ss.rs[tid] = a.rs[row];
    ss.lp[tid] = a.lp[row];
    ss.dis[tid] = a.dis[row];
  }
  if (tid == 0) ss.rs[nrow] = in1;
  int excl;
  if (scanless) {
    // no input self loop dropped (kNoDrop) or exactly one per row (kAllDrop), by every
    // workgroup's verdict: the entries before row d are the input edges before its head, rs[d],
    // less d dropped loops (kAllDrop), plus one appended loop per earlier row — the integers the
    // scan would yield, without the scan's look-back across workgroups
    excl = (tid < nrow ? ss.rs[tid] : 0) + (int)row * (a.add_loop - (scanless == kAllDrop));
  } else {
    int x = v;  // inclusive scan in the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) ss.wsum[wave] = x;
    __syncthreads();
    int tot = 0, before = 0;
#pragma unroll
    for (int q = 0; q < kSortedRows / 64; ++q) {
      tot += ss.wsum[q];
      before += q < wave ? ss.wsum[q] : 0;
    }
    // the flag word carries its own payload (the sum), so relaxed agent-scope atomics suffice: no
    // release / acquire fence (an agent-scope release writes back the XCD's whole L2)
    if (tid == 0)
      __hip_atomic_store(&stat[bx], tot | kScanFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int pre = 0;  // the preceding workgroups' sums, thread-strided, combined in a fixed order
    for (int j = tid; j < bx; j += kSortedRows) {
      int f;
      while (((f = __hip_atomic_load(&stat[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) &
              kScanFlag) == 0)
        __builtin_amdgcn_s_sleep(1);
      pre += f & (kScanFlag - 1);
    }
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
    if (lane == 0) ss.wpre[wave] = pre;
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int q = 0; q < kSortedRows / 64; ++q) base += ss.wpre[q];
    excl = base + before + x - v;
  }
  if (tid < nrow) {
    rowptr[row] = excl;
    ss.rp[tid] = excl;
  }
  if (tid == nrow - 1) {
    ss.rp[nrow] = excl + v;
    if (r0 + nrow == N) rowptr[N] = excl + v;
  }
  if (err_out && bx == 0 && tid == 0) *err_out = 0;
  __syncthreads();
  const int64_t ntiles = (N + 63) >> 6;
  for (int e0 = in0; e0 < in1; e0 += PASS * kSortedRows) {
    if (e0 != in0) load_pass(e0);
#pragma unroll
    for (int it = 0; it < PASS; ++it) {
      const int e = e0 + it * kSortedRows + tid;
      if (e >= in1) break;
      const int dl = (int)(dv[it] - r0);
      const int off = e - ss.rs[dl], lpd = ss.lp[dl];
      if (off == lpd) continue;  // the row's self loop: appended at the end instead
      const int pos = ss.rp[dl] + off - (lpd >= 0 && off > lpd ? 1 : 0);
      col[pos] = (int32_t)sv[it];
      if (w) w[pos] = gcn ? (ds[it] * 1.0f) * ss.dis[dl] : 1.0f;
      if (tile_open && (sv[it] >> 6) != (dv[it] >> 6)) {
        if (tile_open[dv[it] >> 6] == 0) mark_open(tile_open, dv[it] >> 6, ntiles);
        if (tile_open[sv[it] >> 6] == 0) mark_open(tile_open, sv[it] >> 6, ntiles);
      }
    }
  }
  if (a.add_loop && tid < nrow) {
    const int pos = ss.rp[tid + 1] - 1;
    col[pos] = (int32_t)row;
    if (w) {
      const float di = ss.dis[tid];
      w[pos] = gcn ? (di * 1.0f) * di : 1.0f;
    }
  }
}

__global__ __launch_bounds__(kScanT) void k_scan(const int32_t* __restrict__ cnt,
                                                 const int32_t* __restrict__ tcnt, int64_t N,
                                                 int add, int32_t* stat,
                                                 int32_t* __restrict__ rowptr,
                                                 int32_t* __restrict__ tptr,
                                                 int32_t* __restrict__ fill,
                                                 int32_t* __restrict__ tfill,
                                                 float* __restrict__ dis,
                                                 int32_t* tile_open, SortedArgs sa,
                                                 int32_t* __restrict__ col, float* __restrict__ w,
                                                 int32_t* err_out, int nblk) {
  __shared__ ScanSmem sm;
  __shared__ SortedSmem ss;
  const int summary = sa.summary_ready
                          ? (sa.verdict ? __builtin_amdgcn_readfirstlane(sa.verdict[kVerdictMax])
                                        : kModeGeneral)
                          : sorted_mode(sa.verdict, sa.nverdict);
  const int mode = summary & kModeMask;
  if (!sa.summary_ready && sa.verdict && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    sa.verdict[kVerdictMax] = summary;  // the summary word k_fill / k_finish read
  if (mode != kModeGeneral) {
    if (blockIdx.y == 0) {
      if ((int64_t)blockIdx.x * kSortedRows < N)
        sorted_body(sa, N, stat, rowptr, col, w, tile_open, err_out, ss, blockIdx.x,
                    summary & (kNoDrop | kAllDrop));
      return;
    }
    // sorted-open: the source scan (y = 1), its flags past the sorted body's (stat + 4 nblk)
    if (mode == kModeSorted || (int)blockIdx.x >= nblk) return;
    scan_body(cnt, tcnt, N, add, stat + 3 * (int64_t)nblk, rowptr, tptr, fill, tfill, dis,
              tile_open, sm, blockIdx.x, 1, nblk);
    return;
  }
  if ((int)blockIdx.x >= nblk) return;
  scan_body(cnt, tcnt, N, add, stat, rowptr, tptr, fill, tfill, dis, tile_open, sm, blockIdx.x,
            blockIdx.y, nblk);
}

// insertion sort of n (key, val) pairs by key (keys distinct): k_finish's unstaged blocks
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

// by = 0: target CSR (rowptr/col/eid/w); 1: source CSR (tptr/tidx/teid/tw). One virtual block
// = kFinR rows, run by one wave (tid = lane 0..63) with its own staging arrays and `sync` its
// wave-scope ordering. Weight of entry (row i, neighbour j): GCN (dis(src) * 1) * dis(dst) =
// dis(j) * dis(i).
// Staged blocks (<= kFinishCap entries) are finished entry-parallel: every lane takes entries
// eb + t, + 64, ...; an entry's place in its row is its rank among the row's (distinct) edge
// ids, counted over the staged row (lanes of one row read the same LDS words), and the entry,
// its weight, the inverse map and the tile marks are written from there in one pass. Round 5
// sorted each row by one lane (insertion sort, 64 rows per wave, 1536 entries): C5 k = 16's
// source CSR finish took 40 us at under one wave per SIMD. Blocks past the cap (hub rows of
// general graphs) sort each row in place in global memory, one lane per row.
template <typename Sync>
__device__ __forceinline__ void finish_body(int64_t N, int64_t E, int add_loop, int norm,
                                            const int32_t* __restrict__ rowptr, int32_t* col,
                                            int32_t* eid, float* w,
                                            const int32_t* __restrict__ tptr, int32_t* tidx,
                                            int32_t* teid, float* tw,
                                            const float* __restrict__ dis,
                                            int32_t* tile_open, int lazy,
                                            int32_t* __restrict__ inv, int32_t* s_key,
                                            int32_t* s_val, uint8_t* s_row, int32_t* s_ptr,
                                            int64_t bx, int by, int tid, Sync sync) {
  const bool tr = by == 1;
  const int32_t* __restrict__ ptr = tr ? tptr : rowptr;
  int32_t* idx = tr ? tidx : col;
  int32_t* key = tr ? teid : eid;
  float* wt = tr ? tw : w;
  const int64_t i0 = bx * kFinR;
  const int64_t i = i0 + tid;
  const int64_t iend = i0 + kFinR < N ? i0 + kFinR : N;
  const bool own = tid < kFinR && i < N;  // lane tid < kFinR: row i of the block
  const int eb = ptr[i0], ee = ptr[iend];
  const int n = ee - eb;
  // lazy builds took the tile marks in k_count (cross edges) and k_scan (capacity)
  const bool marks = tile_open && !tr && !lazy;
  const int64_t ntiles = (N + 63) >> 6;
  if (marks && own && (i & 63) == 0) {  // more CSR entries than a closed tile takes
    const int64_t iend64 = i + 64 < N ? i + 64 : N;
    if (ptr[iend64] - ptr[i] > lgnn_tile::CAPE_TILE) mark_open(tile_open, i >> 6, ntiles);
  }
  if (n <= kFinishCap) {
    for (int j = tid; j < n; j += 64) {
      s_key[j] = key[eb + j];
      s_val[j] = idx[eb + j];
    }
    if (tid <= kFinR) s_ptr[tid] = ptr[i0 + tid < iend ? i0 + tid : iend] - eb;
    sync();
    if (own) {  // the row table, and the appended self loop (the row's last slot)
      const int r0 = s_ptr[tid], r1 = s_ptr[tid + 1];
      for (int j = r0; j < r1; ++j) s_row[j] = (uint8_t)tid;
      if (add_loop) {
        s_val[r1 - 1] = (int32_t)i;
        s_key[r1 - 1] = (int32_t)(E + i);
      }
    }
    sync();
    for (int j = tid; j < n; j += 64) {
      const int r = s_row[j];
      const int r0 = s_ptr[r], r1 = s_ptr[r + 1];
      const int kj = s_key[j], nb = s_val[j];
      int rank = 0;
      for (int m = r0; m < r1; ++m) rank += s_key[m] < kj;
      const int dst = eb + r0 + rank;
      const int64_t row = i0 + r;
      idx[dst] = nb;
      key[dst] = kj;
      if (wt) wt[dst] = norm == LGNN_NORM_GCN ? (dis[nb] * 1.0f) * dis[row] : 1.0f;
      if (inv && !tr) inv[kj] = dst;  // k_tmap's map, while the keys are at hand
      // 64-node tiles an edge leaves are open: the fused layer stacks skip them
      if (marks && (nb >> 6) != (row >> 6)) {
        if (tile_open[row >> 6] == 0) mark_open(tile_open, row >> 6, ntiles);
        if (tile_open[nb >> 6] == 0) mark_open(tile_open, nb >> 6, ntiles);
      }
    }
    sync();  // the staging arrays are free for the wave's next virtual block
    return;
  }
  if (!own) return;
  const int r0 = ptr[i], r1 = ptr[i + 1];
  if (add_loop) {
    idx[r1 - 1] = (int32_t)i;
    key[r1 - 1] = (int32_t)(E + i);
  }
  sort_row(key + r0, idx + r0, r1 - r0);
  if (inv && !tr)
    for (int j = r0; j < r1; ++j) inv[key[j]] = j;
  if (wt) {
    const float di = norm == LGNN_NORM_GCN ? dis[i] : 1.f;
    for (int j = r0; j < r1; ++j) wt[j] = norm == LGNN_NORM_GCN ? (dis[idx[j]] * 1.0f) * di : 1.0f;
  }
  if (marks) {
    // a row's neighbours sit in one or two tiles: each tile is looked up (and marked) once per
    // run of equal neighbour tiles, this row's own tile once per row (marks are idempotent)
    const int64_t ti = i >> 6;
    bool self_done = false;
    int64_t last = -1;
    for (int j = r0; j < r1; ++j) {
      const int64_t nt = idx[j] >> 6;
      if (nt != ti) {
        if (!self_done) {
          if (tile_open[ti] == 0) mark_open(tile_open, ti, ntiles);
          self_done = true;
        }
        if (nt != last) {
          if (tile_open[nt] == 0) mark_open(tile_open, nt, ntiles);
          last = nt;
        }
      }
    }
  }
}

// one wave: its LDS accesses are ordered by a wave-scope fence (no cross-wave barrier)
struct WaveSync {
  __device__ void operator()() const {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
};

// one wave per virtual block, four per workgroup (each wave its own staging arrays and
// wave-scope ordering), grid-stride over the blocks past kFinGrid workgroups
constexpr int kFinWaves = kThreads / 64;
__global__ __launch_bounds__(kThreads) void k_finish(int64_t N, int64_t E, int add_loop, int norm,
                                                     const int32_t* __restrict__ rowptr,
                                                     int32_t* col, int32_t* eid, float* w,
                                                     const int32_t* __restrict__ tptr,
                                                     int32_t* tidx, int32_t* teid, float* tw,
                                                     const float* __restrict__ dis,
                                                     const int32_t* __restrict__ ws_err,
                                                     int32_t* err_out, int32_t* tile_open,
                                                     int lazy, int32_t* __restrict__ inv,
                                                     const int32_t* summary) {
  __shared__ int32_t s_key[kFinWaves][kFinishCap];
  __shared__ int32_t s_val[kFinWaves][kFinishCap];
  __shared__ uint8_t s_row[kFinWaves][kFinishCap];
  __shared__ int32_t s_ptr[kFinWaves][kFinR + 1];
  const int mode = summary ? __builtin_amdgcn_readfirstlane(*summary) & kModeMask : kModeGeneral;
  if (mode == kModeSorted) return;  // the sorted path took it
  if (mode == kModeSortedOpen && blockIdx.y == 0) return;  // target CSR: k_scan's sorted body
  const int by = blockIdx.y;
  if (err_out && blockIdx.x == 0 && by == 0 && threadIdx.x == 0) *err_out = *ws_err;
  if (lazy && by == 1 && tile_open[(N + 63) >> 6] == 0) return;  // no source CSR needed
  const int wave = threadIdx.x >> 6;
  const int64_t nblk = (N + kFinR - 1) / kFinR;
  for (int64_t v = (int64_t)blockIdx.x * kFinWaves + wave; v < nblk;
       v += (int64_t)gridDim.x * kFinWaves)
    finish_body(N, E, add_loop, norm, rowptr, col, eid, w, tptr, tidx, teid, tw, dis, tile_open,
                lazy, inv, s_key[wave], s_val[wave], s_row[wave], s_ptr[wave], v, by,
                threadIdx.x & 63, WaveSync{});
}

// tmap[q] = position in the target CSR of the edge at source-CSR position q (both CSRs hold the
// same entries; edge ids are unique: e for edges, E + i for appended loops); inv (edge id ->
// target-CSR position) is written by k_finish's target side.
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

// path options (lgnn_set_option): plain ints read on the host when a launch is configured
static int g_options[LGNN_OPT_COUNT] = {1, 0, 1};

int lgnn_option(int option) {
  return option >= 0 && option < LGNN_OPT_COUNT ? __atomic_load_n(&g_options[option], __ATOMIC_RELAXED)
                                                : 0;
}

extern "C" int lgnn_set_option(int option, int value) {
  if (option < 0 || option >= LGNN_OPT_COUNT || value < 0) return LGNN_EINVAL;
  return __atomic_exchange_n(&g_options[option], value, __ATOMIC_RELAXED);
}

extern "C" int lgnn_get_option(int option) {
  if (option < 0 || option >= LGNN_OPT_COUNT) return LGNN_EINVAL;
  return lgnn_option(option);
}

extern "C" const char* lgnn_status_string(int status) {
  switch (status) {
    case LGNN_OK: return "ok";
    case LGNN_EINVAL: return "invalid argument";
    case LGNN_ENOSPC: return "workspace too small";
    case LGNN_EBUSY: return "grid-barrier launch cannot be co-resident";
    default: return status > 0 ? hipGetErrorString((hipError_t)status) : "unknown error";
  }
}

extern "C" size_t lgnn_graph_workspace_bytes(int64_t num_nodes, int64_t num_edges) {
  return ws_total(num_nodes, num_edges);
}

// Ablation knob (timing only, never a product setting): LGNN_ABL_SKIP_GENERAL=1 drops the three
// general-path launches of a target-sorted-path build (k_count / k_fill / k_finish), which is
// correct only for input the sorted path accepts — it measures what those no-op launches cost.
static bool abl_skip_general() {
#ifdef LGNN_ABLATION_BUILD  // timing-only libraries (never the product): the knob is compiled out
  const char* e = getenv("LGNN_ABL_SKIP_GENERAL");
  return e && e[0] == '1';
#else
  return false;
#endif
}

static int graph_build(const int64_t* edge_index, int64_t E, int64_t N, int loops, int norm,
                       int32_t* rowptr, int32_t* col, float* w, int32_t* tptr, int32_t* tidx,
                       float* tw, int32_t* tmap, int32_t* tile_open, const int64_t* batch,
                       int64_t num_graphs, int32_t* gptr, int32_t* err_count, void* workspace,
                       size_t workspace_bytes, void* stream, int lazy,
                       const lgnn_s3::PlaneArgs* planes = nullptr);

extern "C" int lgnn_graph_build(const int64_t* edge_index, int64_t E, int64_t N, int loops,
                                int norm, int32_t* rowptr, int32_t* col, float* w, int32_t* tptr,
                                int32_t* tidx, float* tw, int32_t* tmap, int32_t* tile_open,
                                const int64_t* batch, int64_t num_graphs, int32_t* gptr,
                                int32_t* err_count, void* workspace,
                                size_t workspace_bytes, void* stream) {
  return graph_build(edge_index, E, N, loops, norm, rowptr, col, w, tptr, tidx, tw, tmap,
                     tile_open, batch, num_graphs, gptr, err_count, workspace, workspace_bytes,
                     stream, 0);
}

extern "C" int lgnn_graph_build_planes(const int64_t* edge_index, int64_t E, int64_t N,
                                       int loops, int norm, int32_t* rowptr, int32_t* col,
                                       float* w, int32_t* tptr, int32_t* tidx, float* tw,
                                       int32_t* tmap, int32_t* tile_open, const int64_t* batch,
                                       int64_t num_graphs, int32_t* gptr, int32_t* err_count,
                                       void* workspace, size_t workspace_bytes, int lazy,
                                       const lgnn_plane_job* job, void* stream) {
  if (lazy && (!tile_open || !tptr || tmap)) return LGNN_EINVAL;
  if (!job || job->nl > LGNN_PLANE_JOB_MAX) return LGNN_EINVAL;
  lgnn_s3::PlaneArgs pj;
  const int r = lgnn_s3::plane_args(job->nl, job->W, job->widths, job->planes, job->planes_t, pj);
  if (r != LGNN_OK) return r;
  return graph_build(edge_index, E, N, loops, norm, rowptr, col, w, tptr, tidx, tw, tmap,
                     tile_open, batch, num_graphs, gptr, err_count, workspace, workspace_bytes,
                     stream, lazy ? 1 : 0, &pj);
}

extern "C" int lgnn_graph_build_lazy(const int64_t* edge_index, int64_t E, int64_t N, int loops,
                                     int norm, int32_t* rowptr, int32_t* col, float* w,
                                     int32_t* tptr, int32_t* tidx, float* tw, int32_t* tmap,
                                     int32_t* tile_open, const int64_t* batch,
                                     int64_t num_graphs, int32_t* gptr, int32_t* err_count,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  if (!tile_open || !tptr || tmap) return LGNN_EINVAL;
  return graph_build(edge_index, E, N, loops, norm, rowptr, col, w, tptr, tidx, tw, tmap,
                     tile_open, batch, num_graphs, gptr, err_count, workspace, workspace_bytes,
                     stream, 1);
}

// k_prep_sorted's workgroups (= verdict words)
static int sorted_grid(int64_t N, int64_t E) {
  (void)N;
  const int64_t per = (int64_t)kThreads * kSortedChunks;  // edges per workgroup pass
  int64_t g = (E + per - 1) / per;
  return (int)(g < 1 ? 1 : g > kVerdictMax ? kVerdictMax : g);
}

extern "C" int lgnn_graph_build_path(const void* workspace, int64_t num_nodes, int64_t num_edges,
                                     void* stream) {
  if (!workspace || num_nodes <= 0 || num_edges <= 0) return 0;
  const GraphWs ws = carve(const_cast<void*>(workspace), num_nodes, num_edges);
  int32_t v = 0;
  if (hipMemcpyAsync(&v, ws.verdict + kVerdictMax, 4, hipMemcpyDeviceToHost,
                     as_stream(stream)) != hipSuccess ||
      hipStreamSynchronize(as_stream(stream)) != hipSuccess)
    return LGNN_EINVAL;
  return v & kModeMask;  // kModeGeneral 0, kModeSorted 1, kModeSortedOpen 2
}

// the target-sorted fast path is tried unless LGNN_OPT_GRAPH_SORTED is 0 (a test / A-B option)
static bool sorted_path_enabled() { return lgnn_option(LGNN_OPT_GRAPH_SORTED) != 0; }

static int graph_build(const int64_t* edge_index, int64_t E, int64_t N, int loops, int norm,
                       int32_t* rowptr, int32_t* col, float* w, int32_t* tptr, int32_t* tidx,
                       float* tw, int32_t* tmap, int32_t* tile_open, const int64_t* batch,
                       int64_t num_graphs, int32_t* gptr, int32_t* err_count, void* workspace,
                       size_t workspace_bytes, void* stream, int lazy,
                       const lgnn_s3::PlaneArgs* planes) {
  if (N < 0 || E < 0 || loops < 0 || loops > 2 || norm < 0 || norm > 1) return LGNN_EINVAL;
  if (!rowptr || !col || (E > 0 && !edge_index)) return LGNN_EINVAL;
  if (N + E >= (int64_t)1 << 30) return LGNN_EINVAL;
  if (gptr && (num_graphs < 0 || (N > 0 && !batch))) return LGNN_EINVAL;
  if ((tptr == nullptr) != (tidx == nullptr)) return LGNN_EINVAL;
  if (tmap && !tptr) return LGNN_EINVAL;
  if (workspace_bytes < ws_total(N, E) || !workspace) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const int add_loop = loops == LGNN_LOOPS_KEEP ? 0 : 1;
  GraphWs ws = carve(workspace, N, E);
  // the weight-plane side job rides the first launch as extra workgroups
  lgnn_s3::PlaneArgs pj{};
  if (planes) pj = *planes;
  const int pblocks = planes ? (pj.nl * lgnn_s3::PLANE_ITEMS + kThreads - 1) / kThreads : 0;
  // target-sorted fast path: only for builds without the source CSR (or lazily with it) and
  // without tmap
  SortedArgs sa{};
  const bool try_sorted = sorted_path_enabled() && N > 0 && E > 0 && !tmap && (!tptr || lazy);
  {
    const int64_t nzero = (int64_t)(ws.zero_bytes / 4);
    const int64_t ntiles = (N + 63) / 64;
    if (try_sorted) {
      sa.ei = edge_index;
      sa.E = E;
      sa.loops = loops;
      sa.add_loop = add_loop;
      sa.norm = norm;
      sa.need_closed = tptr != nullptr;  // lazy: an edge leaving its tile needs the source CSR
      sa.rs = ws.rs;
      sa.scnt = ws.scnt;
      sa.lp = ws.lp;
      sa.dis = ws.dis;
      sa.verdict = ws.verdict;
      sa.nverdict = sorted_grid(N, E);
      hipLaunchKernelGGL(k_prep_sorted, dim3(sa.nverdict + pblocks), dim3(kThreads), 0, s,
                         ws.err, nzero, tile_open, ntiles, batch, N, num_graphs, gptr, sa, pj,
                         sa.nverdict);
    } else {
      const int g = grid_for(nzero > N + 1 ? nzero : N + 1, 1024);
      hipLaunchKernelGGL(k_prep, dim3(g + pblocks), dim3(kThreads), 0, s, ws.err, nzero,
                         tile_open, ntiles, batch, N, num_graphs, gptr, pj, g);
    }
    LGNN_LAUNCH_CHECK();
  }
  if (N == 0) {
    if (hipMemsetAsync(rowptr, 0, 4, s) != hipSuccess) return (int)hipGetLastError();
    if (tptr && hipMemsetAsync(tptr, 0, 4, s) != hipSuccess) return (int)hipGetLastError();
    if (err_count && hipMemsetAsync(err_count, 0, 4, s) != hipSuccess)
      return (int)hipGetLastError();
    return LGNN_OK;
  }
  const bool skip_general = try_sorted && abl_skip_general();
  if (E > 0 && !skip_general) {
    if (small_edges(E))
      hipLaunchKernelGGL(k_count<4>, dim3((unsigned)((E + chunk_of(4) - 1) / chunk_of(4))),
                         dim3(kThreads), 0, s, edge_index, E, N, loops, ws.cnt,
                         tptr ? ws.tcnt : nullptr, ws.err, lazy ? tile_open : nullptr, sa.verdict,
                         sa.nverdict);
    else
      hipLaunchKernelGGL(k_count<kPer>, dim3((unsigned)((E + kChunk - 1) / kChunk)),
                         dim3(kThreads), 0, s, edge_index, E, N, loops, ws.cnt,
                         tptr ? ws.tcnt : nullptr, ws.err, lazy ? tile_open : nullptr, sa.verdict,
                         sa.nverdict);
    LGNN_LAUNCH_CHECK();
    sa.summary_ready = sa.verdict != nullptr;
  }
  {
    const int64_t nblk = (N + 1 + kScanBlk - 1) / kScanBlk;
    const int64_t nsb = try_sorted ? (N + kSortedRows - 1) / kSortedRows : 0;
    dim3 sg((unsigned)(nsb > nblk ? nsb : nblk), tptr ? 2u : 1u);
    hipLaunchKernelGGL(k_scan, sg, dim3(kScanT), 0, s, ws.cnt, ws.tcnt, N, add_loop, ws.stat,
                       rowptr, tptr, ws.fill, ws.tfill, ws.dis, lazy ? tile_open : nullptr, sa,
                       col, w, err_count, (int)nblk);
    LGNN_LAUNCH_CHECK();
  }
  if (E > 0 && !skip_general) {
    if (small_edges(E))
      hipLaunchKernelGGL(k_fill<4>, dim3((unsigned)((E + chunk_of(4) - 1) / chunk_of(4))),
                         dim3(kThreads), 0, s, edge_index, E, N, loops, rowptr, ws.fill, col,
                         ws.eid, tptr, ws.tfill, tidx, ws.teid,
                         lazy ? tile_open + (N + 63) / 64 : nullptr,
                         try_sorted ? ws.verdict + kVerdictMax : nullptr);
    else
      hipLaunchKernelGGL(k_fill<kPer>, dim3((unsigned)((E + kChunk - 1) / kChunk)),
                         dim3(kThreads), 0, s, edge_index, E, N, loops, rowptr, ws.fill, col,
                         ws.eid, tptr, ws.tfill, tidx, ws.teid,
                         lazy ? tile_open + (N + 63) / 64 : nullptr,
                         try_sorted ? ws.verdict + kVerdictMax : nullptr);
    LGNN_LAUNCH_CHECK();
  }
  const int64_t nfin = (N + kFinR - 1) / kFinR;
  const int64_t fgx = (nfin + kFinWaves - 1) / kFinWaves;
  dim3 fg((unsigned)(fgx < kFinGrid ? fgx : kFinGrid), tptr ? 2u : 1u);
  // with tmap, the target side of k_finish also writes inv (edge id -> target-CSR position)
  if (!skip_general) {
    hipLaunchKernelGGL(k_finish, fg, dim3(kThreads), 0, s, N, E, add_loop, norm, rowptr, col,
                       ws.eid, w, tptr, tidx, ws.teid, tw, ws.dis, ws.err, err_count, tile_open,
                       lazy, tmap ? ws.inv : nullptr,
                       try_sorted ? ws.verdict + kVerdictMax : nullptr);
    LGNN_LAUNCH_CHECK();
  }
  if (tmap) {
    const int g = grid_for(E + N, 2048);
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
