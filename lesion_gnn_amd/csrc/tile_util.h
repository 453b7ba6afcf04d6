// Shared by the tile kernels (tile.hip, stack3.hip): tile constants, tile selection, raw
// buffer access, coalesced row loads and the per-tile CSR block (registers, LDS, dense Â).
#pragma once
#include "common.h"

// Timing-only ablation builds (tools/ablate.py, tools/stamps.py): -DLGNN_ABLATE=<mask> removes
// phases of the tile kernels (1 MFMA, 2 aggregation, 4 global stores, 8 ELU, 16 global row loads,
// 64 dense-adjacency build). The product build is mask 0; ablated libraries are built outside
// the package and never loaded by it.
#ifndef LGNN_ABLATE
#define LGNN_ABLATE 0
#endif

// Diagnostic build only (-DLGNN_STAMPS, tools/stamps.py): thread 0 of each block records
// s_memtime at phase boundaries of k_stack_fwd; never compiled into the product library.
#ifdef LGNN_STAMPS
__device__ unsigned long long lgnn_stamp_buf[1024 * 64];
#define STAMP(k)                                                                   \
  do {                                                                             \
    const int _k = (k);                                                            \
    if (threadIdx.x == 0 && _k < 62)                                               \
      lgnn_stamp_buf[blockIdx.x * 64 + _k] = __builtin_amdgcn_s_memtime();         \
    if (threadIdx.x == 0 && _k == 0) {  /* placement: HW_ID, XCC_ID */             \
      lgnn_stamp_buf[blockIdx.x * 64 + 62] = __builtin_amdgcn_s_getreg(4 | (31 << 11));  \
      lgnn_stamp_buf[blockIdx.x * 64 + 63] = __builtin_amdgcn_s_getreg(20 | (31 << 11)); \
    }                                                                              \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif

namespace lgnn_tile {

constexpr int ABL = LGNN_ABLATE;
#ifndef LGNN_AGG_UNROLL
#define LGNN_AGG_UNROLL 2
#endif
constexpr int TM = 64;
constexpr int KC = 128;
constexpr int LDS = KC + 4;
constexpr int NT = 256;
constexpr int CAPE = 1024;     // CSR entries of a closed tile staged in registers (the fused
                               // stack kernels; a closed tile's entries past them are read from
                               // global memory as its Â is built: adj_scatter)
constexpr int CAPE_TILE = 2048;  // CSR entries of a closed tile (64 x 32: the reference sweep's
                                 // largest k, scripts/sweep.py:110); more -> the tile is open
constexpr int CAPE_LW = 1280;  // CSR entries staged by the layer-wise tile bodies (64 x (16 + 1)
                               // at k = 16 fits; 5 per thread)
constexpr int EB = 8;

// How a tile's rows are aggregated (idx_store):
enum { AGG_GLOBAL = 0,   // index block too large: CSR entries and source rows from global memory
       AGG_LOCAL = 1,    // every source row is in this tile: ow[j] = (float offset of the source
                         // row in the A image, weight bits), rows read from LDS
       AGG_GROWS = 2 };  // sources leave the tile: ow[j] = (global source row, weight bits),
                         // rows gathered from global memory, no index round trip
// A tile's CSR block in LDS, padded with EB zero-weight entries (source offset / row 0) so a
// row's batch reads need no bounds logic.
struct TileIdx {
  int rp[TM + 1];
  int2 ow[CAPE_LW + EB];
};

// Tile selection by a per-tile mask (nullable = every tile): with `want` = 1 only tiles whose
// mask is non-zero, with 0 only tiles whose mask is zero. Block-uniform scalar reads.
// mask[ntiles] counts the non-zero flags: a want = 1 launch with none returns after one load.
__device__ __forceinline__ int64_t seek_tile(int64_t t, int64_t ntiles,
                                             const int32_t* __restrict__ mask, int want) {
  if (mask) {
    if (want && mask[ntiles] == 0) return ntiles;
    while (t < ntiles && ((mask[t] != 0) != (want != 0))) t += gridDim.x;
  }
  return t;
}

// Raw buffer access (SGPR descriptor + 32-bit byte offset): out-of-range loads return 0 and
// out-of-range stores are dropped by the hardware range check, so row tails need no clamping
// and addresses cost one VGPR. Tensors addressed this way are < 4 GiB (checked on the host).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t Buf;
__device__ __forceinline__ Buf mkbuf(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(uint32_t)bytes,
                                           0x00020000);
}
__device__ __forceinline__ f32x4 bld4(Buf r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void bst4(Buf r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

// A wave's weight fragment for the fp32 MFMA (lane (h, li) of wave w: row n = 32 w + li of W
// [N][K], columns 64 h .. + 63): rows past N and columns past K read 0 through an out-of-range
// buffer offset (K % 4 == 0), so no select consumes the loaded values here — a select right after
// the loads made the compiler wait for them on the spot instead of at the first MFMA
__device__ __forceinline__ void load_wfrag(float (&bf)[64], const float* __restrict__ W, int N,
                                           int K, int n, int h) {
  const Buf bW = mkbuf(W, (int64_t)N * K * 4);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = 64 * h + 4 * q;
    const f32x4 v = bld4(bW, (n < N && k < K) ? (n * K + k) * 4 : 0x7ff00000);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[4 * q + j] = v[j];
  }
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ f32x4 sel4(bool c, f32x4 v) { return c ? v : zero4(); }

// Coalesced raw tile load: half-wave hw = tid / 32 owns rows hw + (64 / RPT) * it (it < RPT;
// RPT = 8 for 256-thread blocks, 4 for 512), columns 4li..4li+3 — the same (row, column) mapping
// as the half-wave-per-row aggregation, so register values can be reused.
template <int RPT>
__device__ __forceinline__ void load_rows(f32x4 (&v)[RPT], Buf X, int K, int r0) {
  const int hw = threadIdx.x >> 5, li = threadIdx.x & 31;
  const int k = 4 * li;
  const int kc = k < K ? k : K - 4;
#pragma unroll
  for (int it = 0; it < RPT; ++it) v[it] = bld4(X, ((r0 + hw + (TM / RPT) * it) * K + kc) * 4);
}

template <int RPT>
__device__ __forceinline__ void store_rows_lds(float* A, const f32x4 (&v)[RPT], int64_t M, int K,
                                               int64_t r0) {
  const int hw = threadIdx.x >> 5, li = threadIdx.x & 31;
  const bool kin = 4 * li < K;
#pragma unroll
  for (int it = 0; it < RPT; ++it) {
    const int rr = hw + (TM / RPT) * it;
    st4(A + rr * LDS + 4 * li, sel4(kin && r0 + rr < M, v[it]));
  }
}

// One tile's CSR index block, loaded into registers ahead of use (software pipelining: the next
// tile's block is in flight while the current tile aggregates and runs its MFMAs).
//   head: rowptr[r0 .. r0+64] (one per thread, tid <= 64) + the uniform entry range (eb, ne)
//   body: the ne <= CAPE entries (col, w), CAPE/NT per thread; issued once the head has landed
template <int NTH, int CAP = CAPE>
struct IdxRegsT {
  static constexpr int cap = CAP;
  int rp;
  int eb, ne;
  int c[CAP / NTH];
  float w[CAP / NTH];
};
using IdxRegs = IdxRegsT<NT>;
using IdxRegsLw = IdxRegsT<NT, CAPE_LW>;  // the layer-wise tile bodies (tile_lw.h)

template <int NTH, int CAP>
__device__ __forceinline__ void idx_load_head(IdxRegsT<NTH, CAP>& R, const int32_t* __restrict__ rowptr,
                                              int64_t M, int64_t r0, int tid_ = -1) {
  const int tid = tid_ < 0 ? (int)threadIdx.x : tid_;
  const int64_t r = r0 + (tid <= TM ? tid : 0);
  R.rp = rowptr[r < M ? r : M];
  const int64_t rl = r0 + TM < M ? r0 + TM : M;
  R.eb = rowptr[r0];
  R.ne = rowptr[rl] - R.eb;
}

template <int NTH, int CAP>
__device__ __forceinline__ void idx_load_body(IdxRegsT<NTH, CAP>& R, const int32_t* __restrict__ col,
                                              const float* __restrict__ w, int tid_ = -1) {
  // (a closed tile of up to CAPE_TILE entries stages its first CAPE; adj_scatter reads the rest)
  if (R.ne > CAP && !(CAP == CAPE && R.ne <= CAPE_TILE)) return;
  const int tid = tid_ < 0 ? (int)threadIdx.x : tid_;
#pragma unroll
  for (int u = 0; u < CAP / NTH; ++u) {
    const int j = tid + u * NTH;
    const int jc = j < R.ne ? j : 0;
    R.c[u] = col[R.eb + jc];
    R.w[u] = w ? w[R.eb + jc] : 1.f;
  }
}

// Writes the prefetched block to LDS and returns how the tile aggregates (AGG_*, block-uniform).
// Ends with a barrier (block-wide OR of "an entry leaves the tile").
template <int NTH, int CAP>
__device__ __forceinline__ int idx_store(TileIdx& ti, const IdxRegsT<NTH, CAP>& R, int64_t r0) {
  static_assert(CAP <= CAPE_LW, "TileIdx holds CAPE_LW entries");
  const int tid = threadIdx.x;
  if (tid <= TM) ti.rp[tid] = R.rp;
  const bool fits = R.ne <= CAP;
  int out = 0;
  if (fits) {
#pragma unroll
    for (int u = 0; u < CAP / NTH; ++u) {
      const int j = tid + u * NTH;
      const int rel = R.c[u] - (int)r0;
      if (j < R.ne && (unsigned)rel >= (unsigned)TM) out = 1;
    }
  }
  const bool any_out = __syncthreads_or(out);
  if (!fits) return AGG_GLOBAL;
#pragma unroll
  for (int u = 0; u < CAP / NTH; ++u) {
    const int j = tid + u * NTH;
    if (j < R.ne)
      ti.ow[j] = make_int2(any_out ? R.c[u] : (R.c[u] - (int)r0) * LDS, __float_as_int(R.w[u]));
  }
  if (tid < EB) ti.ow[R.ne + tid] = make_int2(0, 0);
  return any_out ? AGG_GROWS : AGG_LOCAL;
}

// Dense Â_tile from the tile's row-CSR block (entry j of R: source R.c, weight R.w; its target
// row found by binary search over rp): Adj[target][source] (TRANS = false) or Adj[source][target]
// (TRANS = true), row stride TM. Adj must be zero and rp visible. Duplicate (target, source)
// pairs carry equal weights, so the LDS float adds are order independent. A closed tile with
// more than CAPE entries (k > 16 neighbours at 64 nodes, up to CAPE_TILE) adds the rest straight
// from the CSR (col / w, the tile's entries past the staged ones) — before R is reloaded for the
// next tile.
__device__ __forceinline__ int adj_row(const int* rp, int e) {
  int lo = 0, hi = TM;
#pragma unroll
  for (int it = 0; it < 6; ++it) {
    const int mid = (lo + hi) >> 1;
    if (rp[mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}
template <bool TRANS, int NTH>
__device__ __forceinline__ void adj_scatter(float* Adj, const int* rp, const IdxRegsT<NTH>& R,
                                            int64_t r0, const int32_t* __restrict__ col,
                                            const float* __restrict__ w, int tid_ = -1) {
  const int tid = tid_ < 0 ? (int)threadIdx.x : tid_;
#pragma unroll
  for (int u = 0; u < CAPE / NTH; ++u) {
    const int j = tid + u * NTH;
    if (j < R.ne) {
      const int lo = adj_row(rp, R.eb + j);
      const int c = R.c[u] - (int)r0;
      atomicAdd(&Adj[TRANS ? c * TM + lo : lo * TM + c], R.w[u]);
    }
  }
  if (R.ne > CAPE) {  // block-uniform
    for (int j = CAPE + tid; j < R.ne; j += NTH) {
      const int e = R.eb + j;
      const int lo = adj_row(rp, e);
      const int c = col[e] - (int)r0;
      atomicAdd(&Adj[TRANS ? c * TM + lo : lo * TM + c], w ? w[e] : 1.f);
    }
  }
}

// Workgroup barrier ordering LDS only: unlike __syncthreads it does not wait for outstanding
// global loads and stores (s_waitcnt vmcnt(0)), so loads issued a phase ahead stay in flight
// across it. For kernels whose threads exchange data through LDS only.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Grid-wide barrier of a persistent launch whose workgroups are all co-resident (the fused
// stack kernels: 2 per CU forward, 1 per CU backward, grid <= that). sync[0] counts arrivals
// (barrier `gen` = 1, 2, ... waits for gen * gridDim.x), sync[1] counts exits; both start at 0
// (zeroed by the graph build) and grid_exit() re-arms them for the next launch: the workgroup
// that completes the exit count resets both, when no other workgroup reads them any more.
// Producer side: __syncthreads drains every wave's stores (vmcnt(0)), then one lane releases at
// agent scope (L2 write-back for the other XCDs); consumer: agent-scope acquire (L1/L2
// invalidate), then __syncthreads before any wave reads (MI355X_MICROARCH.md, correctness
// boundaries). The spin is bounded (~0.5 s): a barrier that cannot complete yields wrong
// results, never a hang; it counts itself in sync[2].
// max_spins x s_sleep(8) (512 clocks): 2^20 ~ 0.25 s — a safety net, not a schedule; a phase
// with a legitimately long straggler (the graph build's single-thread sort of a row too long for
// LDS) passes a larger bound
__device__ __forceinline__ void grid_sync(int32_t* sync, int gen, int max_spins = 1 << 20) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(sync, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const int target = gen * (int)gridDim.x;
    int spins = 0;
    while (__hip_atomic_load(sync, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(8);
      if (++spins > max_spins) {
        __hip_atomic_fetch_add(sync + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void grid_exit(int32_t* sync) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int n = __hip_atomic_fetch_add(sync + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (n == (int)gridDim.x - 1) {
      __hip_atomic_store(sync, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sync + 1, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Layer-wise (open-tile) LDS of tile_lw.h's bodies, aliased onto a fused kernel's LDS.
// BatchNorm1d (+ ELU + dropout mask) folded into the layer-wise kernels (the GIN MLP,
// Lin -> BN -> ELU -> Lin; norm.hip holds the standalone kernels with the same arithmetic).
// Template mode BNM of fwd_tiles / bwd_tiles:
//   BN_STATS   forward epilogue: per-workgroup fp64 sums of Y and Y^2 per column -> part
//   BN_IN      forward prologue: X := ELU(X * scale + shift) * mask, also written to act_out
//   BN_GSTATS  backward dX epilogue: sums of g and g * xhat, g = dX * mask * ELU'(Z*sc+sh),
//              xhat = (Z - mean) * invstd (the BN backward's batch sums) -> part
//   BN_GIN     backward prologue (DIRECT): dY := scale * (g - sums0/count - xhat * sums1/count)
//              (training) or scale * g (eval), g as above from the given dY
// part: [gridDim.x][2 * width] (sum kind, column), every workgroup writes its row.
enum { BN_NONE = 0, BN_STATS = 1, BN_IN = 2, BN_GSTATS = LGNN_BN_GSTATS, BN_GIN = LGNN_BN_GIN };
struct BnFuse {
  double* part;
  const float* scale;
  const float* shift;
  const float* mean;
  const float* invstd;
  const float* Z;
  const float* mask;
  const double* sums;
  double count;
  int training;
  float* act_out;
};

// Fold the 8 row groups' fp64 column sums (s0, s1: 4 columns 4 li.. per lane) in a fixed order
// and write this workgroup's partial row; `red` = 16 KiB of free LDS. Every thread calls it.
__device__ __forceinline__ void bn_part_write(double* red, const double (&s0)[4],
                                              const double (&s1)[4], double* part, int N) {
  const int tid = threadIdx.x, li = tid & 31, hw = tid >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[(hw * 2 + 0) * 128 + 4 * li + j] = s0[j];
    red[(hw * 2 + 1) * 128 + 4 * li + j] = s1[j];
  }
  __syncthreads();
  if (tid < 256) {
    const int k = tid >> 7, c = tid & 127;
    double t = red[k * 128 + c];
#pragma unroll
    for (int g = 1; g < 8; ++g) t += red[(g * 2 + k) * 128 + c];
    if (c < N) part[(int64_t)blockIdx.x * 2 * N + k * N + c] = t;
  }
}

struct LwSmem {
  float A[TM * LDS];
  float C[TM * LDS];
  TileIdx ti;
};

// Arguments of the fused GCN stack forward kernels (tile.hip, stack3.hip).
struct StackArgs {
  const float* W[LGNN_MAX_STACK];
  const float* b[LGNN_MAX_STACK];
  float* H[LGNN_MAX_STACK];
  int width[LGNN_MAX_STACK + 1];  // width[0] = input width, width[l+1] = output of layer l
};

}  // namespace lgnn_tile
