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

namespace lgnn_tile {

constexpr int TM = 64;
constexpr int KC = 128;
constexpr int LDS = KC + 4;
constexpr int NT = 256;
constexpr int CAPE = 1024;
constexpr int EB = 8;

struct TileIdx {
  int rp[TM + 1];
  int col[CAPE];
  float w[CAPE];
};

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ f32x4 sel4(bool c, f32x4 v) { return c ? v : zero4(); }

// Coalesced raw tile load: thread owns rows hw + 8*it (it < 8), columns 4li..4li+3 — the same
// (row, column) mapping as the half-wave-per-row aggregation, so register values can be reused.
__device__ __forceinline__ void load_rows(f32x4 (&v)[8], const float* __restrict__ X, int64_t M,
                                          int K, int64_t r0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hw = wave * 2 + (lane >> 5), li = lane & 31;
  const int k = 4 * li;
  const int kc = k < K ? k : K - 4;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int64_t row = r0 + hw + 8 * it;
    const int64_t rc = row < M ? row : M - 1;
    v[it] = ld4(X + rc * K + kc);
  }
}

__device__ __forceinline__ void store_rows_lds(float* A, const f32x4 (&v)[8], int64_t M, int K,
                                               int64_t r0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hw = wave * 2 + (lane >> 5), li = lane & 31;
  const bool kin = 4 * li < K;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int rr = hw + 8 * it;
    st4(A + rr * LDS + 4 * li, sel4(kin && r0 + rr < M, v[it]));
  }
}

__device__ __forceinline__ void stage_idx(TileIdx& ti, bool& staged,
                                          const int32_t* __restrict__ rowptr,
                                          const int32_t* __restrict__ col,
                                          const float* __restrict__ w, int64_t M, int64_t r0) {
  const int tid = threadIdx.x;
  if (tid <= TM) {
    const int64_t r = r0 + tid;
    ti.rp[tid] = rowptr[r < M ? r : M];
  }
  __syncthreads();
  const int eb = ti.rp[0], ne = ti.rp[TM] - eb;
  staged = ne <= CAPE;
  if (staged) {
    for (int j = tid; j < ne; j += NT) {
      ti.col[j] = col[eb + j];
      ti.w[j] = w ? w[eb + j] : 1.f;
    }
  }
  __syncthreads();
}

// sum_{e in row rr} w_e * X[c_e][4li..], in CSR order; X rows of the tile come from the LDS image
// A, others from global X (wave-uniform fallback).
__device__ __forceinline__ f32x4 agg_row(const TileIdx& ti, bool staged, int rr, const float* A,
                                         int64_t r0, const float* __restrict__ X, int K, int kc,
                                         const int32_t* __restrict__ col,
                                         const float* __restrict__ w) {
  const int li = threadIdx.x & 31;
  const int eb = ti.rp[0];
  const int e0 = ti.rp[rr], e1 = ti.rp[rr + 1];
  f32x4 acc = zero4();
  for (int e = e0; e < e1; e += EB) {
    int c[EB];
    float ww[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const bool ok = e + u < e1;
      const int ee = ok ? e + u : e0;
      c[u] = staged ? ti.col[ee - eb] : col[ee];
      const float wv = staged ? ti.w[ee - eb] : (w ? w[ee] : 1.f);
      ww[u] = ok ? wv : 0.f;
    }
    f32x4 v[EB];
    bool out = false;
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int64_t rel = (int64_t)c[u] - r0;
      const bool in = rel >= 0 && rel < TM;
      out |= (e + u < e1) && !in;
      v[u] = ld4(A + (in ? (int)rel : 0) * LDS + 4 * li);
    }
    if (__any(out)) {
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int64_t rel = (int64_t)c[u] - r0;
        const bool in = rel >= 0 && rel < TM;
        const f32x4 g = ld4(X + (int64_t)c[u] * K + kc);
        v[u] = in ? v[u] : g;
      }
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const f32x4 t = ww[u] * v[u];
      acc += (e + u < e1) ? t : zero4();
    }
  }
  return acc;
}

// ------------------------------------------------------------------------------------------
// forward: Y = act(P(X) W^T + b); optional S_out = P(X)
// ------------------------------------------------------------------------------------------
template <bool GATHER, int ACT>
__global__ __launch_bounds__(NT, 2) void k_fwd(const float* __restrict__ X, int64_t M, int K,
                                               const int32_t* __restrict__ rowptr,
                                               const int32_t* __restrict__ col,
                                               const float* __restrict__ w, float self_scale,
                                               const float* __restrict__ W,
                                               const float* __restrict__ b, int N,
                                               float* __restrict__ Y, float* __restrict__ S_out) {
  __shared__ __attribute__((aligned(16))) float A[TM * LDS];
  __shared__ __attribute__((aligned(16))) float S[GATHER ? TM * LDS : 4];
  __shared__ TileIdx ti;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31, hw = wave * 2 + h;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int n = wave * 32 + li;
  const int ncl = n < N ? n : N - 1;
  const bool wave_active = wave * 32 < N;
  float bf[64];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = 64 * h + 4 * q;
    const f32x4 v = ld4(W + (int64_t)ncl * K + (k < K ? k : K - 4));
    const bool ok = n < N && k < K;
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[4 * q + j] = ok ? v[j] : 0.f;
  }
  const float bias = b ? b[ncl] : 0.f;
  const int kc = 4 * li < K ? 4 * li : K - 4;
  float* Ain = GATHER ? S : A;  // MFMA A-operand image

  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * TM;
    f32x4 xr[8];
    load_rows(xr, X, M, K, r0);
    bool staged = true;
    if constexpr (GATHER) stage_idx(ti, staged, rowptr, col, w, M, r0);
    store_rows_lds(A, xr, M, K, r0);
    __syncthreads();
    if constexpr (GATHER) {
#pragma unroll 2
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        f32x4 a = agg_row(ti, staged, rr, A, r0, X, K, kc, col, w);
        if (self_scale != 0.f) a += self_scale * xr[it];
        a = sel4(4 * li < K && r0 + rr < M, a);
        st4(S + rr * LDS + 4 * li, a);
        if (S_out && r0 + rr < M && 4 * li < K) st4(S_out + (r0 + rr) * K + 4 * li, a);
      }
      __syncthreads();
    }
    f32x16 acc0 = {}, acc1 = {};
    if (wave_active) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const f32x4 a0 = ld4(Ain + li * LDS + 64 * h + 4 * q);
        const f32x4 a1 = ld4(Ain + (32 + li) * LDS + 64 * h + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc0 = mfma32(a0[j], bf[4 * q + j], acc0);
          acc1 = mfma32(a1[j], bf[4 * q + j], acc1);
        }
      }
    }
    __syncthreads();  // every wave is done reading A / S
    // epilogue staged in A as [row][col], then whole-row stores
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
      float v0 = acc0[r] + bias, v1 = acc1[r] + bias;
      if (ACT == LGNN_ACT_ELU) {
        v0 = elu_f(v0);
        v1 = elu_f(v1);
      }
      A[rl * LDS + n] = v0;
      A[(32 + rl) * LDS + n] = v1;
    }
    __syncthreads();
    if (4 * li < N) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        if (r0 + rr < M) st4(Y + (r0 + rr) * N + 4 * li, ld4(A + rr * LDS + 4 * li));
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// backward: dZ = G ⊙ act'(H); dW += dZ^T S (S = X, direct); db += colsum dZ; dXpre = dZ W
// ------------------------------------------------------------------------------------------
template <int GMODE, int ACT, bool DX>
__global__ __launch_bounds__(NT, 2) void k_bwd(
    const float* __restrict__ dY, const int64_t* __restrict__ batch,
    const int32_t* __restrict__ gptr, int pool_mean, const int32_t* __restrict__ tptr,
    const int32_t* __restrict__ tidx, const float* __restrict__ tw, float tself,
    const float* __restrict__ H, const float* __restrict__ X, int64_t M, int K,
    const float* __restrict__ W, int N, float* __restrict__ dXpre, float* __restrict__ dWp,
    float* __restrict__ dbp) {
  __shared__ __attribute__((aligned(16))) float A[TM * LDS];
  __shared__ __attribute__((aligned(16))) float C[TM * LDS];
  __shared__ TileIdx ti;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31, hw = wave * 2 + h;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int oc = 4 * li < N ? 4 * li : N - 4;
  const bool oin = 4 * li < N;

  f32x16 dw[4] = {{}, {}, {}, {}};
  float dbacc = 0.f;
  const int kx = 32 * wave + li;
  const int kxc = kx < K ? kx : K - 1;

  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * TM;
    // ---- dZ tile -> C
    if constexpr (GMODE == LGNN_GRAD_TRANSPOSE) {
      bool staged;
      {
        f32x4 dr[8];
        load_rows(dr, dY, M, N, r0);
        stage_idx(ti, staged, tptr, tidx, tw, M, r0);
        store_rows_lds(A, dr, M, N, r0);
      }
      __syncthreads();
#pragma unroll 1
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        const int64_t row = r0 + rr, rc = row < M ? row : M - 1;
        f32x4 hv = zero4();
        if constexpr (ACT == LGNN_ACT_ELU) hv = ld4(H + rc * N + oc);
        f32x4 g = agg_row(ti, staged, rr, A, r0, dY, N, oc, tidx, tw);
        if (tself != 0.f) g += tself * ld4(A + rr * LDS + 4 * li);
        if constexpr (ACT == LGNN_ACT_ELU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) g[j] *= elu_grad_from_out(hv[j]);
        }
        st4(C + rr * LDS + 4 * li, sel4(oin && row < M, g));
      }
    } else {
      f32x4 g[8], hv[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int64_t row = r0 + hw + 8 * it;
        const int64_t rc = row < M ? row : M - 1;
        if constexpr (GMODE == LGNN_GRAD_DIRECT) {
          g[it] = ld4(dY + rc * N + oc);
        } else {
          const int64_t gi = batch[rc];
          g[it] = ld4(dY + gi * N + oc);
          if (pool_mean) {
            const int cnt = gptr[gi + 1] - gptr[gi];
            g[it] = g[it] / (float)(cnt > 0 ? cnt : 1);
          }
        }
        if constexpr (ACT == LGNN_ACT_ELU) hv[it] = ld4(H + rc * N + oc);
      }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        f32x4 v = g[it];
        if constexpr (ACT == LGNN_ACT_ELU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] *= elu_grad_from_out(hv[it][j]);
        }
        st4(C + rr * LDS + 4 * li, sel4(oin && r0 + rr < M, v));
      }
    }
    // ---- S tile -> A (A's raw dY image is dead once every wave has passed this barrier)
    f32x4 sr[8];
    load_rows(sr, X, M, K, r0);
    __syncthreads();
    store_rows_lds(A, sr, M, K, r0);
    __syncthreads();
    if (tid < 128) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll 8
      for (int r = 0; r < TM; r += 2) {
        s0 += C[r * LDS + tid];
        s1 += C[(r + 1) * LDS + tid];
      }
      dbacc += s0 + s1;
    }
    // DX B-fragment W[o = 64h + s][kx], re-read per tile (L2) so it is not live during the
    // aggregation phase; its latency hides under the dW MFMAs.
    // Buffer loads: per-lane voffset (column kx, half-wave row block 64h) + uniform soffset
    // (row s); rows o >= N fall outside the descriptor's range and read 0.
    float wt[64];
    if constexpr (DX) {
      const __amdgpu_buffer_rsrc_t wr =
          __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, N * K * 4, 0x00020000);
      const int voff = (64 * h * K + kxc) * 4;
#pragma unroll
      for (int s = 0; s < 64; ++s) {
        const float v = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(wr, voff, s * K * 4, 0));
        wt[s] = kx < K ? v : 0.f;
      }
    }
    // dW[o][k] += sum_m dZ[m][o] S[m][k]; wave owns o in [32w, 32w+32)
#pragma unroll 4
    for (int s = 0; s < TM / 2; ++s) {
      const int m = 2 * s + h;
      const float a = C[m * LDS + 32 * wave + li];
#pragma unroll
      for (int j = 0; j < 4; ++j) dw[j] = mfma32(a, A[m * LDS + 32 * j + li], dw[j]);
    }
    if constexpr (DX) {
      f32x16 x0 = {}, x1 = {};
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const f32x4 a0 = ld4(C + li * LDS + 64 * h + 4 * q);
        const f32x4 a1 = ld4(C + (32 + li) * LDS + 64 * h + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x0 = mfma32(a0[j], wt[4 * q + j], x0);
          x1 = mfma32(a1[j], wt[4 * q + j], x1);
        }
      }
      __syncthreads();  // dW reads of A are done
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        A[rl * LDS + kx] = x0[r];
        A[(32 + rl) * LDS + kx] = x1[r];
      }
      __syncthreads();
      if (4 * li < K) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int rr = hw + 8 * it;
          if (r0 + rr < M) st4(dXpre + (r0 + rr) * K + 4 * li, ld4(A + rr * LDS + 4 * li));
        }
      }
    }
    __syncthreads();
  }
  float* slab = dWp + (int64_t)blockIdx.x * N * K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 32 * j + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (o < N && k < K) slab[(int64_t)o * K + k] = dw[j][r];
    }
  }
  if (dbp && tid < N) dbp[(int64_t)blockIdx.x * N + tid] = dbacc;
}

}  // namespace lgnn_tile

using namespace lgnn_tile;

bool lgnn_tile_fits(int K, int N) { return K <= KC && N <= KC && K % 4 == 0 && N % 4 == 0; }

int lgnn_tile_partials(int64_t M) {
  const int64_t ntiles = (M + TM - 1) / TM;
  const int64_t p = ntiles < 512 ? ntiles : 512;
  return (int)(p < 1 ? 1 : p);
}

hipError_t lgnn_tile_fwd(hipStream_t s, const float* X, int64_t M, int K, const int32_t* rowptr,
                         const int32_t* col, const float* w, float self_scale, const float* W,
                         const float* b, int N, int act, float* Y, float* S_out) {
  const int64_t ntiles = (M + TM - 1) / TM;
  dim3 grid((unsigned)(ntiles < 512 ? ntiles : 512));
#define LGNN_TF(G, A)                                                                         \
  hipLaunchKernelGGL((k_fwd<G, A>), grid, dim3(NT), 0, s, X, M, K, rowptr, col, w, self_scale, \
                     W, b, N, Y, S_out)
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
                         float* dXpre, float* dWp, float* dbp, int P) {
  dim3 grid((unsigned)P);
#define LGNN_TB(GM, AC, D)                                                                     \
  hipLaunchKernelGGL((k_bwd<GM, AC, D>), grid, dim3(NT), 0, s, dY, batch, gptr, pool_mean, tptr, \
                     tidx, tw, tself, H, X, M, K, W, N, dXpre, dWp, dbp)
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
