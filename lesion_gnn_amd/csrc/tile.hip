// Fast-path node-tile kernels (K <= 128, N <= 128, K % 4 == N % 4 == 0 — every hidden layer of
// the reference configs). Same math and C ABI as node.hip; lgnn_node_linear_fwd/bwd dispatch
// here when the shape allows.
//
// What differs from the generic kernels:
//  * in-tile aggregation from LDS: the tile's own rows [r0, r0+64) are loaded once, coalesced, and
//    the neighbour sum reads them from LDS. k-NN edges never leave their graph, so with N = 64
//    graphs every neighbour is in the tile; neighbours outside the tile (graphs crossing a tile
//    boundary) are read from global memory in a wave-uniform fallback branch.
//  * the forward can save the aggregated tile S = P(X) (S_out), so the backward's dW = dZ^T S
//    streams S instead of re-gathering;
//  * outputs are staged through LDS and written as whole 512-B rows;
//  * persistent grid (2 workgroups per CU) with the weight fragment loaded once per workgroup.
#include "common.h"
#include "tile.h"
#include "tile_util.h"
#include "tile_lw.h"

#include <cstdlib>
#include <type_traits>

namespace lgnn_tile {


// The layer-wise kernels: the bodies in tile_lw.h on their own LDS.
template <bool GATHER, int ACT, int BNM = BN_NONE>
__global__ __launch_bounds__(NT, 2) void k_fwd(const float* __restrict__ X, int64_t M, int K,
                                               const int32_t* __restrict__ rowptr,
                                               const int32_t* __restrict__ col,
                                               const float* __restrict__ w, float self_scale,
                                               const float* __restrict__ W,
                                               const float* __restrict__ b, int N,
                                               float* __restrict__ Y, float* __restrict__ S_out,
                                               const int32_t* __restrict__ tmask, int want,
                                               BnFuse bn) {
  __shared__ __attribute__((aligned(16))) float A[TM * LDS];
  __shared__ __attribute__((aligned(16))) float S[GATHER ? TM * LDS : 4];
  __shared__ TileIdx ti;
  fwd_tiles<GATHER, ACT, BNM>(A, S, ti, X, M, K, rowptr, col, w, self_scale, W, b, N, Y, S_out,
                              tmask, want, bn);
}

template <int GMODE, int ACT, bool DX, int BNM = BN_NONE>
__global__ __launch_bounds__(NT, 2) void k_bwd(
    const float* __restrict__ dY, const int64_t* __restrict__ batch,
    const int32_t* __restrict__ gptr, int pool_mean, const int32_t* __restrict__ tptr,
    const int32_t* __restrict__ tidx, const float* __restrict__ tw, float tself,
    const float* __restrict__ H, const float* __restrict__ X, int64_t M, int K,
    const float* __restrict__ W, int N, float* __restrict__ dXpre, float* __restrict__ dWp,
    float* __restrict__ dbp, const int32_t* __restrict__ tmask, int want, int accumulate,
    BnFuse bn, const float* __restrict__ dlog = nullptr, const float* __restrict__ Wout = nullptr,
    int nclass = 0) {
  __shared__ __attribute__((aligned(16))) float A[TM * LDS];
  __shared__ __attribute__((aligned(16))) float C[TM * LDS];
  __shared__ TileIdx ti;
  bwd_tiles<GMODE, ACT, DX, BNM>(A, C, ti, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H,
                                 X, M, K, W, N, dXpre, dWp, dbp, tmask, want, accumulate, dlog,
                                 Wout, nclass, bn);
}


// ------------------------------------------------------------------------------------------
// Fused layer stack, forward: a workgroup keeps one 64-node tile on chip through every layer
//   H_0 = X W_0^T + b_0                      (in_proj; skipped when FIRST = false: X is H_0)
//   S_l = Â H_{l-1},  H_l = ELU(S_l W_l^T + b_l),  l = 1..L   (GCNConv + the model's F.elu)
// storing H_l and S_l for the backward. The tile's CSR block is staged once for all layers;
// the next tile's rows and CSR block are prefetched into registers while this tile computes,
// and each layer's weight fragment is fetched (L2) while the previous layer finishes its
// epilogue and aggregation. Every k-NN neighbour of a graph aligned to the tile is in LDS.
// All widths <= 128 (fast-path shapes).
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ void load_bfrag(float (&bf)[64], const float* __restrict__ W, int N,
                                           int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  load_wfrag(bf, W, N, K, wave * 32 + (lane & 31), lane >> 5);
}

// ------------------------------------------------------------------------------------------
// Fused GCN stack forward, for the tiles no edge leaves: in_proj + L x ELU(GCNConv) in one
// launch, the tile on chip between layers. PyG's association (GCNConv: lin, then propagate):
//   H_0 = X W_0^T + b_0;   H_l = ELU(Â_tile (H_{l-1} W_l^T) + b_l)
// Â_tile is staged dense in LDS (transposed, 64 x 64, from the tile's CSR block), so the
// aggregation is an MFMA product. 4 waves, 2 workgroups per CU (one's MFMAs overlap the
// other's stores and barriers); wave w owns output columns [32w, 32w + 32) of all 64 rows (two
// 32x32 accumulators). Per layer: P = A W^T (A = H_{l-1} image, W fragment in registers,
// loaded a layer ahead) -> A; Z = Â P -> epilogue -> A (next layer's input) and HBM (H_l, rows
// staged through LDS and written as whole rows). Only the H_l are written: the backward uses
// G = Â^T dZ, dW = G^T H_{l-1} (k_stack_bwd), so no aggregated input is saved.
// ------------------------------------------------------------------------------------------
struct FwdSmem {
  float A[TM * LDS];
  float AdjT[TM * TM];  // Â_tile[source][target]
  int rp[TM + 1];
};

template <bool FIRST>
__global__ __launch_bounds__(NT, 2) void k_stack_fwd(const float* __restrict__ X, int64_t M,
                                                     const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     const float* __restrict__ w, int L,
                                                     StackArgs args,
                                                     const int32_t* __restrict__ tmask) {
  __shared__ __attribute__((aligned(16))) FwdSmem sm;
  float* const A = sm.A;
  float* const AdjT = sm.AdjT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31, hw = tid >> 5;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int n = wave * 32 + li;
  const int l0 = FIRST ? 0 : 1;
  const int K0 = args.width[l0];

  [[maybe_unused]] int stamp = 0;
  STAMP(stamp++);
  int64_t t = seek_tile(blockIdx.x, ntiles, tmask, 0);
  if (t >= ntiles) return;
#ifdef LGNN_DESYNC
#ifndef LGNN_DESYNC_PRED
#define LGNN_DESYNC_PRED (blockIdx.x & 1)
#endif
  // diagnostic: one workgroup of each CU pair starts late
  if (LGNN_DESYNC_PRED)
    for (int i = 0; i < LGNN_DESYNC; ++i) __builtin_amdgcn_s_sleep(1);
#endif
  f32x4 xr[8];
  IdxRegs R;
  float bf[64];
  const Buf bX = mkbuf(X, M * K0 * 4);
  const bool any_conv = L >= 1;
  load_rows(xr, bX, K0, (int)(t * TM));
  if (any_conv) idx_load_head(R, rowptr, M, t * TM);
  load_bfrag(bf, args.W[l0], args.width[l0 + 1], args.width[l0]);
  // bias of the layer whose fragment is in bf (loaded with it, a layer ahead of its use)
  float bias = n < args.width[l0 + 1] ? args.b[l0][n] : 0.f;
  if (any_conv) idx_load_body(R, col, w);
  for (; t < ntiles;) {
    const int64_t r0 = t * TM;
    const int64_t tn = seek_tile(t + gridDim.x, ntiles, tmask, 0);
    const bool has_next = tn < ntiles;
    store_rows_lds(A, xr, M, K0, r0);
    if (any_conv) {
      for (int i = tid; i < TM * TM / 4; i += NT) st4(AdjT + 4 * i, zero4());
      if (tid <= TM) sm.rp[tid] = R.rp;
    }
    __syncthreads();
    STAMP(stamp++);
    if (any_conv && !(ABL & 64)) adj_scatter<true>(AdjT, sm.rp, R, r0, col, w);
    if (has_next) {
      load_rows(xr, bX, K0, (int)(tn * TM));
      if (any_conv) idx_load_head(R, rowptr, M, tn * TM);
    }
    for (int l = l0; l <= L; ++l) {
      const int N = args.width[l + 1];
      const bool conv = l > 0;
      // P = A W_l^T (A = X or H_{l-1} image); wave: columns n, rows li (acc0) and 32 + li (acc1)
      f32x16 acc0 = {}, acc1 = {};
      if (wave * 32 < N && !(ABL & 1)) {
        const float* ap = A + li * LDS + 64 * h;
        f32x4 a0 = ld4(ap), a1 = ld4(ap + 32 * LDS);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int nx = q + 1 < 16 ? q + 1 : q;
          const f32x4 b0 = ld4(ap + 4 * nx), b1 = ld4(ap + 32 * LDS + 4 * nx);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc0 = mfma32(a0[j], bf[4 * q + j], acc0);
            acc1 = mfma32(a1[j], bf[4 * q + j], acc1);
          }
          a0 = b0;
          a1 = b1;
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        }
      }
      // next layer's weight fragment (or the first layer's, for the next tile)
      const int lnext = l < L ? l + 1 : l0;
      const float bias_l = bias;
      if (l < L || has_next) {
        load_bfrag(bf, args.W[lnext], args.width[lnext + 1], args.width[lnext]);
        bias = n < args.width[lnext + 1] ? args.b[lnext][n] : 0.f;
      }
      if (l == l0 && any_conv && has_next) idx_load_body(R, col, w);  // head has landed
      __syncthreads();  // every wave is done reading A
      STAMP(stamp++);
      if (conv) {
        // P -> A, then Z = Â P: Z[m][n] = sum_j AdjT[j][m] P[j][n]
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          A[rl * LDS + n] = n < N ? acc0[r] : 0.f;
          A[(32 + rl) * LDS + n] = n < N ? acc1[r] : 0.f;
        }
        __syncthreads();
        if (!(ABL & 2)) {
          acc0 = f32x16{};
          acc1 = f32x16{};
        }
        if (wave * 32 < N && !(ABL & 2)) {
          const float* jp = AdjT + h * TM + li;
          const float* pp = A + h * LDS + n;
          float m0 = jp[0], m1 = jp[32], pv = pp[0];
          __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
          for (int s2 = 0; s2 < TM / 2; ++s2) {
            const int nx = s2 + 1 < TM / 2 ? s2 + 1 : s2;
            const float n0 = jp[2 * nx * TM], n1 = jp[2 * nx * TM + 32], pn = pp[2 * nx * LDS];
            acc0 = mfma32(m0, pv, acc0);
            acc1 = mfma32(m1, pv, acc1);
            m0 = n0;
            m1 = n1;
            pv = pn;
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          }
        }
        __syncthreads();  // every wave is done reading P
        STAMP(stamp++);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        float v0 = acc0[r] + bias_l, v1 = acc1[r] + bias_l;
        if (conv && !(ABL & 8)) {
          v0 = elu_f(v0);
          v1 = elu_f(v1);
        }
        A[rl * LDS + n] = n < N ? v0 : 0.f;
        A[(32 + rl) * LDS + n] = n < N ? v1 : 0.f;
      }
      STAMP(stamp++);
      __syncthreads();
      STAMP(stamp++);
      if (4 * li < N && !(ABL & 4)) {
        const Buf hb = mkbuf(args.H[l], M * N * 4);
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int rr = hw + 8 * it;
          bst4(hb, (int)((r0 + rr) * N + 4 * li) * 4, ld4(A + rr * LDS + 4 * li));
        }
      }
      STAMP(stamp++);
      // A now holds H_l (zero beyond N) for the next layer; its next writer comes after a
      // barrier (the next layer's MFMA) or the tile-end barrier below
    }
    __syncthreads();
    t = tn;
  }
}
// ------------------------------------------------------------------------------------------
// Fused GCN stack backward, for the tiles no edge leaves (the forward's k_stack_fwd tiles): from
// the pooled-output gradient dP down to the in_proj weights in one launch, the tile on chip.
// Autograd's own association for GCNConv (out = Â (H W^T) + b, PyG order):
//   dZ_L = dP[g(i)] (/ count) * ELU'(H_L)
//   for l = L..1:  db_l += colsum dZ_l;  G = Â^T dZ_l;  dW_l += G^T H_{l-1};
//                  dZ_{l-1} = (G W_l) * ELU'(H_{l-1})   (no ELU' below the first conv)
//   dW_0 += dZ_0^T X, db_0 += colsum dZ_0
// 512 threads = 8 waves, one workgroup per CU (two waves per SIMD hide each other's latency).
// Â of the tile is staged dense in LDS (64 x 64, built from the tile's CSR block by scattered
// LDS adds), so the aggregation is an MFMA product instead of a latency-bound gather.
// LDS: C = dZ_l / G, A = the H_{l-1} (or X) image, Wl = W_l (unpadded [o][k], filled by
// direct-to-LDS buffer loads a phase ahead, so the weight costs no registers), Adj = Â_tile.
// Work split per wave w (q = w & 3, r2 = w >> 2): dW_l block dW[32q..+32][64r2..+64] (two 32x32
// accumulators per layer, resident over all the workgroup's tiles, written once as partial slot
// blockIdx.x); G block rows 32r2.., columns 32q..; (G W_l)^T block k in [32q, +32), m in
// [32r2, +32). db: per-wave column partials in LDS, reduced in a fixed order at the end.
// ------------------------------------------------------------------------------------------
struct StackBwdArgs {
  const float* W[LGNN_MAX_STACK];
  const float* H[LGNN_MAX_STACK];  // H[l]: output of layer l (H[0] = in_proj output)
  const float* X;                  // model input (in_proj dW operand)
  float* dWp[LGNN_MAX_STACK];      // [P][N_l][K_l]
  float* dbp[LGNN_MAX_STACK];      // [P][N_l]
  int width[LGNN_MAX_STACK + 1];   // width[l] = input width of layer l, width[l+1] = output
};

// dH_L rows of a tile from the pooled-output gradient (global_mean/add_pool backward):
// dH[m] = dP[batch[m]] (/ |graph|), in two steps so neither waits on the other: the graph ids
// (pool_ids), then the dP rows and graph sizes (pool_rows); the division happens at use
// (pool_scale). Same row mapping as load_rows.
template <int RPT>
__device__ __forceinline__ void pool_ids(int (&gi)[RPT], const int64_t* __restrict__ batch,
                                         int64_t M, int64_t r0) {
  const int hw = threadIdx.x >> 5;
#pragma unroll
  for (int it = 0; it < RPT; ++it) {
    const int64_t row = r0 + hw + (TM / RPT) * it;
    gi[it] = (int)batch[row < M ? row : M - 1];
  }
}

template <int RPT>
__device__ __forceinline__ void pool_rows(f32x4 (&gv)[RPT], int (&cnt)[RPT], const int (&gi)[RPT],
                                          const float* __restrict__ dP,
                                          const int32_t* __restrict__ gptr, int pool_mean, int N) {
  const int li = threadIdx.x & 31;
  const int oc = 4 * li < N ? 4 * li : N - 4;
#pragma unroll
  for (int it = 0; it < RPT; ++it) {
    gv[it] = ld4(dP + (int64_t)gi[it] * N + oc);
    cnt[it] = pool_mean ? gptr[gi[it] + 1] - gptr[gi[it]] : 1;
  }
}

__device__ __forceinline__ f32x4 pool_scale(f32x4 v, int cnt) {
  return cnt > 1 ? v / (float)cnt : v;
}

constexpr int NTB = 512;
constexpr int RPB = TM / (NTB / 32);  // rows per thread (4)

// Register-lean row access for the 512-thread kernel: one buffer descriptor (SGPRs) per row
// group, so the per-lane offset is a single VGPR per width instead of one per row (row offsets
// held in VGPRs across the persistent tile loop would spill). Rows past M read as zeros.
__device__ __forceinline__ Buf rows_buf(const float* X, int64_t M, int K, int64_t rb) {
  const int64_t rem = M - rb;
  return mkbuf(X + rb * K, rem > 0 ? rem * K * 4 : 0);
}

template <int RPT>
__device__ __forceinline__ void load_rows_d(f32x4 (&v)[RPT], const float* X, int64_t M, int K,
                                            int64_t r0) {
  const int hw = threadIdx.x >> 5, li = threadIdx.x & 31;
  const int kc = 4 * li < K ? 4 * li : K - 4;
  const int off = (hw * K + kc) * 4;
#pragma unroll
  for (int it = 0; it < RPT; ++it) v[it] = bld4(rows_buf(X, M, K, r0 + (TM / RPT) * it), off);
}

// W [N][K] (row-major, global) -> Wl [N][KC] in LDS, zero-filled past N and K. 16 B per lane,
// two 128-float rows per wave instruction; no registers, completion by vmcnt.
__device__ __forceinline__ void stage_w_lds(float* Wl, const float* W, int N, int K) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = 4 * (lane & 31);
  const int off = c < K ? ((lane >> 5) * K + c) * 4 : 0x7ffffff0;  // OOB -> zeros
#pragma unroll
  for (int u = 0; u < KC / (2 * (NTB / 64)); ++u) {  // 8 instructions per wave
    const int o0 = 2 * (wave + (NTB / 64) * u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rows_buf(W, N, K, o0), (__attribute__((address_space(3))) void*)(Wl + o0 * KC), 16, off,
        0, 0, 0);
  }
}

// LDS image of k_stack_bwd (162 KB for three layers). A and C first: every row access then
// fits the 16-bit immediate offset of ds_read/ds_write (no per-access address VALU).
template <int NL>
struct BwdSmem {
  float A[TM * LDS];
  float C[TM * LDS];
  float Wl[KC * KC];
  float Adj[TM * TM];          // Â_tile[target][source]
  float Db[NL][NTB / 64][KC];  // db partials per wave, column
  int rp[TM + 1];
};

template <int NL>
__global__ __launch_bounds__(NTB, 1) void k_stack_bwd(const float* __restrict__ dP,
                                                      const int64_t* __restrict__ batch,
                                                      const int32_t* __restrict__ gptr,
                                                      int pool_mean,
                                                      const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col,
                                                      const float* __restrict__ w, int64_t M,
                                                      StackBwdArgs a,
                                                      const int32_t* __restrict__ tmask) {
  constexpr int L = NL - 1;
  __shared__ __attribute__((aligned(16))) BwdSmem<NL> sm;
  float* const A = sm.A;
  float* const C = sm.C;
  float* const Wl = sm.Wl;
  float* const Adj = sm.Adj;
  auto& Db = sm.Db;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31, hw = tid >> 5;
  const int wq = wave & 3, wr2 = wave >> 2;
  const int64_t ntiles = (M + TM - 1) / TM;

  f32x16 dw[NL][2];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    dw[l][0] = f32x16{};
    dw[l][1] = f32x16{};
  }
  for (int i = tid; i < NL * (NTB / 64) * KC; i += NTB) (&Db[0][0][0])[i] = 0.f;
  for (int i = tid; i < TM * TM / 4; i += NTB) st4(Adj + 4 * i, zero4());
  // db partials: the two half-waves' column sums combined, added into the wave's LDS row by
  // the lane that owns those 4 columns (no other thread touches them until the end)
  auto db_flush = [&](int l, f32x4 v) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += __shfl_xor(v[j], 32);
    if (h == 0) {
      float* d = &Db[l][wave][4 * li];
      st4(d, ld4(d) + v);
    }
  };
  // column sums of this thread's rows of C = dZ_l (row mapping of load_rows)
  auto db_from_c = [&](int l) {
    f32x4 v = zero4();
#pragma unroll
    for (int it = 0; it < RPB; ++it) v += ld4(C + (hw + (TM / RPB) * it) * LDS + 4 * li);
    db_flush(l, v);
  };
  // image rows of layer l's dW operand: H_{l-1}, or X for in_proj
  auto img_ptr = [&](int l) { return l >= 1 ? a.H[l - 1] : a.X; };

  f32x4 hv[RPB], sr[RPB], gv[RPB];
  int gi[RPB], cnt[RPB];
  IdxRegsT<NTB> R;
  int64_t t = seek_tile(blockIdx.x, ntiles, tmask, 0);
  if (t < ntiles) {
    pool_ids(gi, batch, M, t * TM);
    pool_rows(gv, cnt, gi, dP, gptr, pool_mean, a.width[L + 1]);
    load_rows_d(hv, a.H[L], M, a.width[L + 1], t * TM);
    load_rows_d(sr, img_ptr(L), M, a.width[L], t * TM);
    idx_load_head(R, rowptr, M, t * TM);
    idx_load_body(R, col, w);
    stage_w_lds(Wl, a.W[L], a.width[L + 1], a.width[L]);
  }
  [[maybe_unused]] int stamp = 0;
  STAMP(stamp++);
  for (; t < ntiles;) {
    const int64_t r0 = t * TM;
    const int64_t tn = seek_tile(t + gridDim.x, ntiles, tmask, 0);
    const bool has_next = tn < ntiles;
    if (tid <= TM) sm.rp[tid] = R.rp;
    __syncthreads();  // rp visible, Adj zero
    adj_scatter<false>(Adj, sm.rp, R, r0, col, w);
    {
      const int N = a.width[L + 1];
      f32x4 dsum = zero4();
#pragma unroll
      for (int it = 0; it < RPB; ++it) {
        const int rr = hw + (TM / RPB) * it;
        f32x4 v = pool_scale(gv[it], cnt[it]);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= elu_grad_from_out(hv[it][j]);
        v = sel4(4 * li < N && r0 + rr < M, v);
        dsum += v;
        st4(C + rr * LDS + 4 * li, v);
      }
      db_flush(L, dsum);
    }
    store_rows_lds(A, sr, M, a.width[L], r0);
    __builtin_amdgcn_s_waitcnt(0);  // W_L staged a phase ago
    __syncthreads();
    STAMP(stamp++);
#pragma unroll
    for (int l = L; l >= 1; --l) {
      const int N = a.width[l + 1], K = a.width[l];
      if (l < L) db_from_c(l);
      // prefetch: the next image (H_{l-2} or X); at l = 1 also the next tile's graph ids and
      // CSR head (no load waits on another in front of the MFMAs)
      load_rows_d(sr, img_ptr(l - 1), M, a.width[l - 1], r0);
      if (l == 1 && has_next) {
        pool_ids(gi, batch, M, tn * TM);
        idx_load_head(R, rowptr, M, tn * TM);
      }
      // G[m][n] = sum_i Â[i][m] dZ[i][n]; wave block m in [32 r2, +32), n in [32q, +32)
      f32x16 g = {};
      {
        const float* ap = Adj + h * TM + 32 * wr2 + li;
        const float* cp = C + h * LDS + 32 * wq + li;
        float av = ap[0], cv = cp[0];
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int s2 = 0; s2 < TM / 2; ++s2) {
          const int nx = s2 + 1 < TM / 2 ? s2 + 1 : s2;
          const float an = ap[2 * nx * TM], cn = cp[2 * nx * LDS];
          g = mfma32(av, cv, g);
          av = an;
          cv = cn;
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      }
      __syncthreads();  // every wave is done reading dZ_l
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 32 * wr2 + (r & 3) + 8 * (r >> 2) + 4 * h;
        C[m * LDS + 32 * wq + li] = 32 * wq + li < N ? g[r] : 0.f;
      }
      __builtin_amdgcn_s_waitcnt(0);  // W_l (staged a phase ago) has landed
      __syncthreads();
      STAMP(stamp++);
      // dW_l[o][k] += sum_m G[m][o] H_{l-1}[m][k], m = 2 s2 + h. Accumulator j holds the
      // columns k = 64 wk + 2 li + j, so a lane's two B operands are one ds_read_b64.
      {
        const float* cp = C + h * LDS + 32 * wq + li;
        const float* ap = A + h * LDS + 64 * wr2 + 2 * li;
        float a0 = cp[0];
        float2 b = *reinterpret_cast<const float2*>(ap);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int s2 = 0; s2 < TM / 2; ++s2) {
          const int nx = (s2 + 1 < TM / 2 ? s2 + 1 : s2) * 2 * LDS;
          const float a1 = cp[nx];
          const float2 bn = *reinterpret_cast<const float2*>(ap + nx);
          dw[l][0] = mfma32(a0, b.x, dw[l][0]);
          dw[l][1] = mfma32(a0, b.y, dw[l][1]);
          a0 = a1;
          b = bn;
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
      }
      // (G W_l)^T[k][m] = sum_o W_l[o][k] G[m][o]; half h contracts o in [64h, 64h + 64)
      f32x16 x = {};
      {
        const float* wp = Wl + 64 * h * KC + 32 * wq + li;
        const float* cp = C + (32 * wr2 + li) * LDS + 64 * h;
        f32x4 cv = ld4(cp);
        float wv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) wv[j] = wp[j * KC];
        __builtin_amdgcn_sched_group_barrier(0x100, 5, 0);
#pragma unroll
        for (int p4 = 0; p4 < 16; ++p4) {  // operands of group p4 + 1 read ahead
          const int nx = p4 + 1 < 16 ? p4 + 1 : p4;
          const f32x4 cn = ld4(cp + 4 * nx);
          float wn[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) wn[j] = wp[(4 * nx + j) * KC];
#pragma unroll
          for (int j = 0; j < 4; ++j) x = mfma32(wv[j], cv[j], x);
          cv = cn;
#pragma unroll
          for (int j = 0; j < 4; ++j) wv[j] = wn[j];
          __builtin_amdgcn_sched_group_barrier(0x100, 5, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
      }
      STAMP(stamp++);
      // dZ_{l-1} = (G W_l) * ELU'(H_{l-1}) at (m = 32 r2 + li, k = 32q + 8g + 4h + 0..3); the
      // H_{l-1} values come from the A image
      f32x4 dz[4];
      {
        const float* hp = A + (32 * wr2 + li) * LDS + 32 * wq + 4 * h;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          f32x4 v = f32x4{x[4 * g4], x[4 * g4 + 1], x[4 * g4 + 2], x[4 * g4 + 3]};
          if (l >= 2) {
            const f32x4 hh = ld4(hp + 8 * g4);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] *= elu_grad_from_out(hh[j]);
          }
          dz[g4] = sel4(32 * wq + 8 * g4 + 4 * h < K && r0 + 32 * wr2 + li < M, v);
        }
      }
      __syncthreads();  // every wave is done reading A (H_{l-1}), C (G) and Wl
      {
        float* cp = C + (32 * wr2 + li) * LDS + 32 * wq + 4 * h;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) st4(cp + 8 * g4, dz[g4]);
      }
      store_rows_lds(A, sr, M, a.width[l - 1], r0);
      if (l >= 2) stage_w_lds(Wl, a.W[l - 1], a.width[l], a.width[l - 1]);
      __syncthreads();
      STAMP(stamp++);
    }
    // in_proj: dW_0 += dZ_0^T X; the next tile's loads go out first
    db_from_c(0);
    if (has_next) {
      pool_rows(gv, cnt, gi, dP, gptr, pool_mean, a.width[L + 1]);
      load_rows_d(hv, a.H[L], M, a.width[L + 1], tn * TM);
      load_rows_d(sr, img_ptr(L), M, a.width[L], tn * TM);
      idx_load_body(R, col, w);
      stage_w_lds(Wl, a.W[L], a.width[L + 1], a.width[L]);  // Wl is free since l = 1's DX
    }
    for (int i = tid; i < TM * TM / 4; i += NTB) st4(Adj + 4 * i, zero4());  // read at l = 1
    {
      const float* cp = C + h * LDS + 32 * wq + li;
      const float* ap = A + h * LDS + 64 * wr2 + 2 * li;
      float a0 = cp[0];
      float2 b = *reinterpret_cast<const float2*>(ap);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int s2 = 0; s2 < TM / 2; ++s2) {
        const int nx = (s2 + 1 < TM / 2 ? s2 + 1 : s2) * 2 * LDS;
        const float a1 = cp[nx];
        const float2 bn = *reinterpret_cast<const float2*>(ap + nx);
        dw[0][0] = mfma32(a0, b.x, dw[0][0]);
        dw[0][1] = mfma32(a0, b.y, dw[0][1]);
        a0 = a1;
        b = bn;
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
    }
    __syncthreads();  // A / C free for the next tile
    STAMP(stamp++);
    t = tn;
  }
  __syncthreads();  // db: the 8 wave partials of each column, summed in a fixed order
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const int N = a.width[l + 1], K = a.width[l];
    if (tid < N) {
      float acc = 0.f;
#pragma unroll
      for (int g = 0; g < NTB / 64; ++g) acc += Db[l][g][tid];
      a.dbp[l][(int64_t)blockIdx.x * N + tid] = acc;
    }
    float* slab = a.dWp[l] + (int64_t)blockIdx.x * N * K;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = 64 * wr2 + 2 * li + j;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = 32 * wq + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o < N && k < K) slab[(int64_t)o * K + k] = dw[l][j][r];
      }
    }
  }
}

// open[t] = 1 if an edge joins a node of tile t with a node of another tile (target CSR), or
// if the tile holds more than CAPE_TILE CSR entries.
__global__ __launch_bounds__(NT) void k_tile_open(const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col, int64_t M,
                                                  int32_t* __restrict__ open) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < M; i += (int64_t)gridDim.x * NT) {
    const int ti = (int)(i / TM);
    const int64_t ntiles = (M + TM - 1) / TM;
    auto mark = [&](int64_t t) {  // the first writer of a tile also counts it
      if (atomicCAS(&open[t], 0, 1) == 0) atomicAdd(&open[ntiles], 1);
    };
    if (i % TM == 0) {
      const int64_t ie = i + TM < M ? i + TM : M;
      if (rowptr[ie] - rowptr[i] > CAPE_TILE) mark(ti);
    }
    const int e0 = rowptr[i], e1 = rowptr[i + 1];
    for (int e = e0; e < e1; ++e) {
      const int tj = col[e] / TM;
      if (tj != ti) {
        if (open[ti] == 0) mark(ti);
        if (open[tj] == 0) mark(tj);
      }
    }
  }
}

}  // namespace lgnn_tile

using namespace lgnn_tile;

// Fast-path shapes; buffer offsets are 32-bit signed byte offsets, so tensors stay < 2 GiB.
bool lgnn_tile_fits(int64_t M, int K, int N) {
  return K <= KC && N <= KC && K % 4 == 0 && N % 4 == 0 && K > 0 && N > 0 &&
         (M + TM) * (int64_t)(K > N ? K : N) * 4 < (int64_t)INT32_MAX;
}

// Workgroups of the backward kernels = dW partial slots (persistent over the tiles): 512 = 2 per CU.
int lgnn_tile_partials(int64_t M) {
  const int64_t cap = 512;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int64_t p = ntiles < cap ? ntiles : cap;
  return (int)(p < 1 ? 1 : p);
}

hipError_t lgnn_tile_fwd(hipStream_t s, const float* X, int64_t M, int K, const int32_t* rowptr,
                         const int32_t* col, const float* w, float self_scale, const float* W,
                         const float* b, int N, int act, float* Y, float* S_out,
                         const int32_t* tile_mask, int want) {
  const int64_t ntiles = (M + TM - 1) / TM;
  dim3 grid((unsigned)(ntiles < 512 ? ntiles : 512));
#define LGNN_TF(G, A)                                                                         \
  hipLaunchKernelGGL((k_fwd<G, A>), grid, dim3(NT), 0, s, X, M, K, rowptr, col, w, self_scale, \
                     W, b, N, Y, S_out, tile_mask, want, BnFuse{})
  if (rowptr) {
    if (act == LGNN_ACT_ELU) LGNN_TF(true, LGNN_ACT_ELU);
    else LGNN_TF(true, LGNN_ACT_NONE);
  } else {
    if (act == LGNN_ACT_ELU) LGNN_TF(false, LGNN_ACT_ELU);
    else LGNN_TF(false, LGNN_ACT_NONE);
  }
#undef LGNN_TF
  return hipGetLastError();
}

hipError_t lgnn_tile_bwd(hipStream_t s, int grad_mode, const float* dY, const int64_t* batch,
                         const int32_t* gptr, int pool_mean, const int32_t* tptr,
                         const int32_t* tidx, const float* tw, float tself, const float* H,
                         int act, const float* X, int64_t M, int K, const float* W, int N,
                         float* dXpre, float* dWp, float* dbp, int P, const int32_t* tile_mask,
                         int want, int accumulate) {
  dim3 grid((unsigned)P);
#define LGNN_TB(GM, AC, D)                                                                     \
  hipLaunchKernelGGL((k_bwd<GM, AC, D>), grid, dim3(NT), 0, s, dY, batch, gptr, pool_mean, tptr, \
                     tidx, tw, tself, H, X, M, K, W, N, dXpre, dWp, dbp, tile_mask, want,        \
                     accumulate, BnFuse{})
#define LGNN_TB_D(GM, AC) \
  if (dXpre) LGNN_TB(GM, AC, true); else LGNN_TB(GM, AC, false);
  if (act == LGNN_ACT_ELU) {
    if (grad_mode == LGNN_GRAD_DIRECT) { LGNN_TB_D(LGNN_GRAD_DIRECT, LGNN_ACT_ELU) }
    else if (grad_mode == LGNN_GRAD_POOL) { LGNN_TB_D(LGNN_GRAD_POOL, LGNN_ACT_ELU) }
    else { LGNN_TB_D(LGNN_GRAD_TRANSPOSE, LGNN_ACT_ELU) }
  } else {
    if (grad_mode == LGNN_GRAD_DIRECT) { LGNN_TB_D(LGNN_GRAD_DIRECT, LGNN_ACT_NONE) }
    else if (grad_mode == LGNN_GRAD_POOL) { LGNN_TB_D(LGNN_GRAD_POOL, LGNN_ACT_NONE) }
    else { LGNN_TB_D(LGNN_GRAD_TRANSPOSE, LGNN_ACT_NONE) }
  }
#undef LGNN_TB_D
#undef LGNN_TB
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// C ABI: fused GCN stack forward
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// C ABI: layer-wise linear kernels with BatchNorm folded in (the GIN MLP)
// ------------------------------------------------------------------------------------------
extern "C" int lgnn_bn_fused_partials(int64_t M) {
  if (M < 0) return LGNN_EINVAL;
  return lgnn_tile_partials(M);
}

extern "C" int lgnn_node_linear_fwd_bn(const float* X, int64_t M, int K, const int32_t* rowptr,
                                       const int32_t* col, const float* w, float self_scale,
                                       const float* W, const float* b, int N, int act, float* Y,
                                       float* S_out, double* stats_part, const float* bn_scale,
                                       const float* bn_shift, const float* bn_mask,
                                       float* bn_out, void* stream) {
  if (M < 0 || !W || !Y || (M > 0 && !X) || !lgnn_tile_fits(M, K, N)) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  const bool stats = stats_part != nullptr, bnin = bn_scale != nullptr;
  if (stats == bnin) return LGNN_EINVAL;  // exactly one of the two
  if (bnin && (rowptr || !bn_shift || !bn_out)) return LGNN_EINVAL;
  if (rowptr && !col) return LGNN_EINVAL;
  const int P = lgnn_tile_partials(M);
  BnFuse bn = {};
  bn.part = stats_part;
  bn.scale = bn_scale;
  bn.shift = bn_shift;
  bn.mask = bn_mask;
  bn.act_out = bn_out;
  hipStream_t s = as_stream(stream);
  if (M == 0) {  // the partial rows still hold zeros
    if (stats && hipMemsetAsync(stats_part, 0, (size_t)P * 2 * N * sizeof(double), s) != hipSuccess)
      return (int)hipGetLastError();
    return LGNN_OK;
  }
  const dim3 grid((unsigned)P);  // the stats need one partial row per workgroup
  float* So = rowptr ? S_out : nullptr;
#define LGNN_TFB(G, A, BM)                                                                      \
  hipLaunchKernelGGL((k_fwd<G, A, BM>), grid, dim3(NT), 0, s, X, M, K, rowptr, col, w,        \
                     self_scale, W, b, N, Y, So, nullptr, 0, bn)
  if (stats) {
    if (rowptr) {
      if (act == LGNN_ACT_ELU) LGNN_TFB(true, LGNN_ACT_ELU, BN_STATS);
      else LGNN_TFB(true, LGNN_ACT_NONE, BN_STATS);
    } else {
      if (act == LGNN_ACT_ELU) LGNN_TFB(false, LGNN_ACT_ELU, BN_STATS);
      else LGNN_TFB(false, LGNN_ACT_NONE, BN_STATS);
    }
  } else {
    if (act == LGNN_ACT_ELU) LGNN_TFB(false, LGNN_ACT_ELU, BN_IN);
    else LGNN_TFB(false, LGNN_ACT_NONE, BN_IN);
  }
#undef LGNN_TFB
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_node_linear_bwd_bn(int bn_mode, const float* dY, const float* H, int act,
                                       const float* X, int64_t M, int K, const float* W, int N,
                                       float* dXpre, float* dW_partial, float* db_partial,
                                       int num_partials, const float* bn_Z, const float* bn_mask,
                                       const float* bn_scale, const float* bn_shift,
                                       const float* bn_mean, const float* bn_invstd,
                                       double* gstats_part, const double* bn_sums, double count,
                                       int training, void* stream) {
  return lgnn_node_linear_bwd_bn_pool(bn_mode, dY, H, act, X, M, K, W, N, dXpre, dW_partial,
                                      db_partial, num_partials, bn_Z, bn_mask, bn_scale, bn_shift,
                                      bn_mean, bn_invstd, gstats_part, bn_sums, count, training,
                                      nullptr, nullptr, 0, nullptr, nullptr, 0, stream);
}

static int node_linear_bwd_bn_impl(
    int bn_mode, const float* dY, const float* H, int act, const float* X, int64_t M, int K,
    const float* W, int N, float* dXpre, float* dW_partial, float* db_partial, int num_partials,
    const float* bn_Z, const float* bn_mask, const float* bn_scale, const float* bn_shift,
    const float* bn_mean, const float* bn_invstd, double* gstats_part, const double* bn_sums,
    double count, int training, const int64_t* batch, const int32_t* gptr, int pool_mean,
    const float* dlogits, const float* Wout, int num_classes, const int32_t* tptr,
    const int32_t* tidx, const float* tw, float tself, void* stream) {
  const bool pool = batch != nullptr;
  if (pool && (!gptr || bn_mode != BN_GSTATS || !dlogits || !Wout || num_classes < 1))
    return LGNN_EINVAL;
  if (tptr && (pool || bn_mode != BN_GSTATS || !tidx || !tw)) return LGNN_EINVAL;
  if (M < 0 || !W || !dW_partial || !lgnn_tile_fits(M, K, N)) return LGNN_EINVAL;
  if (num_partials != lgnn_tile_partials(M)) return LGNN_EINVAL;
  if (M > 0 && ((!dY && !pool) || !X)) return LGNN_EINVAL;
  if (!bn_Z || !bn_scale || !bn_shift || !bn_mean || !bn_invstd) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  if (act == LGNN_ACT_ELU && !H) return LGNN_EINVAL;
  if (bn_mode == BN_GSTATS && (!dXpre || !gstats_part)) return LGNN_EINVAL;
  if (bn_mode == BN_GIN && (act != LGNN_ACT_NONE || (training && (!bn_sums || count <= 0.0))))
    return LGNN_EINVAL;
  if (bn_mode != BN_GSTATS && bn_mode != BN_GIN) return LGNN_EINVAL;
  BnFuse bn = {};
  bn.part = gstats_part;
  bn.scale = bn_scale;
  bn.shift = bn_shift;
  bn.mean = bn_mean;
  bn.invstd = bn_invstd;
  bn.Z = bn_Z;
  bn.mask = bn_mask;
  bn.sums = bn_sums;
  bn.count = count;
  bn.training = training;
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    if (hipMemsetAsync(dW_partial, 0, (size_t)num_partials * N * K * 4, s) != hipSuccess ||
        (db_partial && hipMemsetAsync(db_partial, 0, (size_t)num_partials * N * 4, s)) ||
        (gstats_part &&
         hipMemsetAsync(gstats_part, 0, (size_t)num_partials * 2 * K * sizeof(double), s)))
      return (int)hipGetLastError();
    return LGNN_OK;
  }
  const dim3 grid((unsigned)num_partials);
#define LGNN_TBB(AC, D, BM)                                                                     \
  hipLaunchKernelGGL((k_bwd<LGNN_GRAD_DIRECT, AC, D, BM>), grid, dim3(NT), 0, s, dY, nullptr,  \
                     nullptr, 0, nullptr, nullptr, nullptr, 0.f, H, X, M, K, W, N, dXpre,      \
                     dW_partial, db_partial, nullptr, 0, 0, bn)
#define LGNN_TBP(AC)                                                                            \
  hipLaunchKernelGGL((k_bwd<LGNN_GRAD_POOL, AC, true, BN_GSTATS>), grid, dim3(NT), 0, s, nullptr, \
                     batch, gptr, pool_mean, nullptr, nullptr, nullptr, 0.f, H, X, M, K, W, N,    \
                     dXpre, dW_partial, db_partial, nullptr, 0, 0, bn, dlogits, Wout,           \
                     num_classes)
#define LGNN_TBT(AC)                                                                            \
  hipLaunchKernelGGL((k_bwd<LGNN_GRAD_TRANSPOSE, AC, true, BN_GSTATS>), grid, dim3(NT), 0, s, dY, \
                     nullptr, nullptr, 0, tptr, tidx, tw, tself, H, X, M, K, W, N, dXpre,        \
                     dW_partial, db_partial, nullptr, 0, 0, bn)
  if (pool) {  // the pooled-output gradient formed from dlogits and out_proj's W (no dH tensor)
    if (act == LGNN_ACT_ELU) LGNN_TBP(LGNN_ACT_ELU);
    else LGNN_TBP(LGNN_ACT_NONE);
  } else if (tptr) {  // dY = tself dS + A^T dS gathered through the transpose CSR as loaded
    if (act == LGNN_ACT_ELU) LGNN_TBT(LGNN_ACT_ELU);
    else LGNN_TBT(LGNN_ACT_NONE);
  } else if (bn_mode == BN_GSTATS) {
    if (act == LGNN_ACT_ELU) LGNN_TBB(LGNN_ACT_ELU, true, BN_GSTATS);
    else LGNN_TBB(LGNN_ACT_NONE, true, BN_GSTATS);
  } else {
    if (dXpre) LGNN_TBB(LGNN_ACT_NONE, true, BN_GIN);
    else LGNN_TBB(LGNN_ACT_NONE, false, BN_GIN);
  }
#undef LGNN_TBB
#undef LGNN_TBP
#undef LGNN_TBT
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_node_linear_bwd_bn_pool(
    int bn_mode, const float* dY, const float* H, int act, const float* X, int64_t M, int K,
    const float* W, int N, float* dXpre, float* dW_partial, float* db_partial, int num_partials,
    const float* bn_Z, const float* bn_mask, const float* bn_scale, const float* bn_shift,
    const float* bn_mean, const float* bn_invstd, double* gstats_part, const double* bn_sums,
    double count, int training, const int64_t* batch, const int32_t* gptr, int pool_mean,
    const float* dlogits, const float* Wout, int num_classes, void* stream) {
  return node_linear_bwd_bn_impl(bn_mode, dY, H, act, X, M, K, W, N, dXpre, dW_partial,
                                 db_partial, num_partials, bn_Z, bn_mask, bn_scale, bn_shift,
                                 bn_mean, bn_invstd, gstats_part, bn_sums, count, training, batch,
                                 gptr, pool_mean, dlogits, Wout, num_classes, nullptr, nullptr,
                                 nullptr, 0.f, stream);
}

extern "C" int lgnn_node_linear_bwd_bn_gather(
    const float* dS, const int32_t* tptr, const int32_t* tidx, const float* tw, float tself,
    const float* H, int act, const float* X, int64_t M, int K, const float* W, int N,
    float* dXpre, float* dW_partial, float* db_partial, int num_partials, const float* bn_Z,
    const float* bn_mask, const float* bn_scale, const float* bn_shift, const float* bn_mean,
    const float* bn_invstd, double* gstats_part, void* stream) {
  if (!tptr) return LGNN_EINVAL;
  return node_linear_bwd_bn_impl(BN_GSTATS, dS, H, act, X, M, K, W, N, dXpre, dW_partial,
                                 db_partial, num_partials, bn_Z, bn_mask, bn_scale, bn_shift,
                                 bn_mean, bn_invstd, gstats_part, nullptr, 0.0, 0, nullptr,
                                 nullptr, 0, nullptr, nullptr, 0, tptr, tidx, tw, tself, stream);
}

extern "C" int lgnn_tile_count(int64_t M) {
  if (M < 0) return LGNN_EINVAL;
  return (int)((M + lgnn_tile::TM - 1) / lgnn_tile::TM);
}

extern "C" int lgnn_tile_open(const int32_t* rowptr, const int32_t* col, int64_t M,
                              int32_t* open, void* stream) {
  if (M < 0 || !open || (M > 0 && (!rowptr || !col))) return LGNN_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t ntiles = (M + lgnn_tile::TM - 1) / lgnn_tile::TM;
  if (hipMemsetAsync(open, 0, (ntiles + LGNN_TILE_OPEN_EXTRA) * sizeof(int32_t), s) != hipSuccess)
    return (int)hipGetLastError();
  if (ntiles == 0) return LGNN_OK;
  int64_t g = (M + lgnn_tile::NT - 1) / lgnn_tile::NT;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(lgnn_tile::k_tile_open, dim3((unsigned)g), dim3(lgnn_tile::NT), 0, s, rowptr,
                     col, M, open);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_gcn_stack_fwd(const float* X, int64_t M, int d_in, int has_in_proj,
                                  const int32_t* rowptr, const int32_t* col, const float* w,
                                  int L, const float* const* W, const float* const* b,
                                  const int* widths, float* const* H, const int32_t* tile_open,
                                  void* stream) {
  if (M < 0 || L < 0 || L + 1 > LGNN_MAX_STACK || !W || !b || !widths || !H) return LGNN_EINVAL;
  if (L > 0 && (!rowptr || !col || !tile_open)) return LGNN_EINVAL;
  lgnn_tile::StackArgs a = {};
  const int l0 = has_in_proj ? 0 : 1;
  if (l0 > L) return LGNN_EINVAL;
  if (!has_in_proj && widths[0] != d_in) return LGNN_EINVAL;
  a.width[0] = d_in;
  for (int l = 0; l <= L; ++l) {
    a.width[l + 1] = widths[l];
    if (l < l0) continue;
    const int K = a.width[l], N = a.width[l + 1];
    if (!lgnn_tile_fits(M, K, N) || !W[l] || !b[l] || !H[l]) return LGNN_EINVAL;
    a.W[l] = W[l];
    a.b[l] = b[l];
    a.H[l] = H[l];
  }
  if (M == 0) return LGNN_OK;
  if (!X) return LGNN_EINVAL;
  const int64_t ntiles = (M + lgnn_tile::TM - 1) / lgnn_tile::TM;
  dim3 grid((unsigned)(ntiles < 512 ? ntiles : 512));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (has_in_proj)
    hipLaunchKernelGGL(lgnn_tile::k_stack_fwd<true>, grid, dim3(lgnn_tile::NT), 0, s, X, M,
                       rowptr, col, w, L, a, tile_open);
  else
    hipLaunchKernelGGL(lgnn_tile::k_stack_fwd<false>, grid, dim3(lgnn_tile::NT), 0, s, X, M,
                       rowptr, col, w, L, a, tile_open);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

#ifdef LGNN_STAMPS
extern "C" int lgnn_debug_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(lgnn_stamp_buf), sizeof(lgnn_stamp_buf));
}
#endif

// ------------------------------------------------------------------------------------------
// C ABI: fused GCN stack backward (closed tiles)
// ------------------------------------------------------------------------------------------
extern "C" int lgnn_gcn_stack_bwd_partials(int64_t M) {
  if (M < 0) return LGNN_EINVAL;
  const int64_t ntiles = (M + lgnn_tile::TM - 1) / lgnn_tile::TM;
  const int64_t p = ntiles < 256 ? ntiles : 256;
  return (int)(p < 1 ? 1 : p);
}

extern "C" int lgnn_gcn_stack_bwd(const float* dP, const int64_t* batch, const int32_t* gptr,
                                  int pool_mean, const int32_t* rowptr, const int32_t* col,
                                  const float* w, const float* X, int64_t M, int L,
                                  const float* const* W, const float* const* H, const int* widths,
                                  float* const* dWp, float* const* dbp, int num_partials,
                                  const int32_t* tile_open, void* stream) {
  if (M < 0 || L < 1 || L > 2 || !dP || !batch || !gptr || !rowptr || !col || !X || !W || !H ||
      !widths || !dWp || !dbp || !tile_open)
    return LGNN_EINVAL;
  if (num_partials != lgnn_gcn_stack_bwd_partials(M)) return LGNN_EINVAL;
  lgnn_tile::StackBwdArgs a = {};
  for (int l = 0; l <= L + 1; ++l) a.width[l] = widths[l];
  a.X = X;
  for (int l = 0; l <= L; ++l) {
    const int K = a.width[l], N = a.width[l + 1];
    if (!lgnn_tile_fits(M, K, N) || !W[l] || !H[l] || !dWp[l] || !dbp[l]) return LGNN_EINVAL;
    a.W[l] = W[l];
    a.H[l] = H[l];
    a.dWp[l] = dWp[l];
    a.dbp[l] = dbp[l];
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (M == 0) {  // one all-zero slot per layer
    for (int l = 0; l <= L; ++l) {
      if (hipMemsetAsync(a.dWp[l], 0, (size_t)a.width[l] * a.width[l + 1] * 4, s) != hipSuccess ||
          hipMemsetAsync(a.dbp[l], 0, (size_t)a.width[l + 1] * 4, s) != hipSuccess)
        return (int)hipGetLastError();
    }
    return LGNN_OK;
  }
  dim3 grid((unsigned)num_partials);
  if (L == 1)
    hipLaunchKernelGGL(lgnn_tile::k_stack_bwd<2>, grid, dim3(lgnn_tile::NTB), 0, s, dP, batch, gptr,
                       pool_mean, rowptr, col, w, M, a, tile_open);
  else
    hipLaunchKernelGGL(lgnn_tile::k_stack_bwd<3>, grid, dim3(lgnn_tile::NTB), 0, s, dP, batch, gptr,
                       pool_mean, rowptr, col, w, M, a, tile_open);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}
