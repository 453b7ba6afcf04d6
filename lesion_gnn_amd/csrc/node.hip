// Node-tile kernels: fused (aggregate ->) Linear (-> bias -> ELU) forward and the matching fused
// backward, on fp32 MFMA (v_mfma_f32_32x32x2_f32 — exact fp32, gfx950 has no xf32).
//
// Tiling (both kernels): a workgroup = 4 waves = 256 threads owns a 64-node row tile; the tile's
// (aggregated) features are staged in LDS as [64][132] fp32 (row pad 4 floats: conflict-free
// ds_read_b128 A-fragments); wave w owns 32 output columns, so one WG covers 128
// output features. K is streamed in chunks of 128.
//
// K permutation: in a 32x32x2 MFMA, lane-half h supplies k-slot h. Slot h of step s is bound to
// feature k = 64h + s, so a lane's A values for consecutive steps are contiguous in LDS (one
// ds_read_b128 feeds 4 steps) and its B values are 64 contiguous floats of one weight row.
//
// Loads are never predicated: out-of-range rows/columns load a clamped (valid) address and are
// zeroed by a select afterwards — a predicated load makes hipcc branch and drain vmcnt per load.
// CSR indices of a tile are staged in LDS once, so each row's neighbour loads are one round trip
// with all of them in flight.
//
// Replaces (reference): nn.Linear in_proj/out_proj (gin.py:21,25), GCNConv/GINConv propagate +
// lin (gin.py:23), F.elu (gin.py:31) and their autograd backward.
#include "common.h"
#include "tile.h"

namespace {

constexpr int TM = 64;        // node rows per tile
constexpr int TN = 128;       // output features per workgroup (4 waves x 32)
constexpr int KC = 128;       // K chunk staged in LDS
constexpr int LDS = KC + 4;   // padded LDS row stride (floats)
constexpr int NT = 256;
constexpr int CAPE = 1024;    // CSR entries of one tile staged in LDS (else read from global)
constexpr int EB = 8;         // neighbour rows in flight per row

struct TileIdx {
  int rp[TM + 1];
  int col[CAPE];
  float w[CAPE];
};

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ f32x4 sel4(bool c, f32x4 v) { return c ? v : zero4(); }

// ------------------------------------------------------------------------------------------
// Direct tile fill: Xs[r][c] = X[r0 + r][k0 + c], zero outside [M) x [K).
// ------------------------------------------------------------------------------------------
template <bool VEC>
__device__ __forceinline__ void fill_direct(float* Xs, const float* __restrict__ X, int64_t M,
                                            int K, int k0, int64_t r0) {
  const int tid = threadIdx.x;
  if constexpr (VEC) {
    f32x4 v[(TM * KC / 4) / NT];
#pragma unroll
    for (int it = 0; it < (TM * KC / 4) / NT; ++it) {
      const int idx = it * NT + tid;
      const int64_t row = r0 + (idx >> 5);
      const int k = k0 + 4 * (idx & 31);
      const int64_t rc = row < M ? row : M - 1;
      const int kc = k < K ? k : K - 4;
      v[it] = sel4(row < M && k < K, ld4(X + rc * K + kc));
    }
#pragma unroll
    for (int it = 0; it < (TM * KC / 4) / NT; ++it) {
      const int idx = it * NT + tid;
      st4(Xs + (idx >> 5) * LDS + 4 * (idx & 31), v[it]);
    }
  } else {
#pragma unroll 8
    for (int it = 0; it < (TM * KC) / NT; ++it) {
      const int idx = it * NT + tid;
      const int64_t row = r0 + (idx >> 7);
      const int k = k0 + (idx & 127);
      const int64_t rc = row < M ? row : M - 1;
      const int kc = k < K ? k : K - 1;
      const float v = X[rc * K + kc];
      Xs[(idx >> 7) * LDS + (idx & 127)] = (row < M && k < K) ? v : 0.f;
    }
  }
}

// Stage rowptr[r0 .. r0+64] and (if they fit) the tile's CSR entries in LDS. Returns whether
// the entries were staged. Ends with a barrier.
__device__ __forceinline__ bool stage_idx(TileIdx& ti, const int32_t* __restrict__ rowptr,
                                          const int32_t* __restrict__ col,
                                          const float* __restrict__ w, int64_t M, int64_t r0) {
  const int tid = threadIdx.x;
  if (tid <= TM) {
    const int64_t r = r0 + tid;
    ti.rp[tid] = rowptr[r < M ? r : M];
  }
  __syncthreads();
  const int eb = ti.rp[0], ne = ti.rp[TM] - eb;
  const bool staged = ne <= CAPE;
  if (staged) {
    for (int j = tid; j < ne; j += NT) {
      ti.col[j] = col[eb + j];
      ti.w[j] = w ? w[eb + j] : 1.f;
    }
  }
  __syncthreads();
  return staged;
}

// Aggregation of one row strip (4 features at k) for a half wave: returns
//   sum_{e in row} w_e * X[col_e][k..k+3]  (CSR order)  [+ self_scale * X[row]]
// All EB neighbour loads of a batch are issued before any is consumed.
template <bool STAGED>
__device__ __forceinline__ f32x4 agg_row(const TileIdx& ti, int rr, const float* __restrict__ X,
                                         int K, int kc, const int32_t* __restrict__ col,
                                         const float* __restrict__ w, int64_t rowc) {
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
      if constexpr (STAGED) {
        c[u] = ti.col[ee - eb];
        ww[u] = ok ? ti.w[ee - eb] : 0.f;
      } else {
        c[u] = col[ee];
        ww[u] = ok ? (w ? w[ee] : 1.f) : 0.f;
      }
    }
    f32x4 v[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) v[u] = ld4(X + (int64_t)c[u] * K + kc);
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const f32x4 t = ww[u] * v[u];
      acc += (e + u < e1) ? t : zero4();
    }
  }
  (void)rowc;
  return acc;
}

// Aggregated tile fill (K % 4 == 0): Xs[r][c] = P(X)[r0 + r][k0 + c]. Half wave per row, float4
// per lane, two rows per half wave in flight. Order: CSR sum, then + self term (GINConv:
// scatter-sum + (1 + eps) x).
template <bool STAGED>
__device__ __forceinline__ void fill_gather_t(float* Xs, const TileIdx& ti,
                                              const float* __restrict__ X, int64_t M, int K,
                                              int k0, int64_t r0, const int32_t* __restrict__ col,
                                              const float* __restrict__ w, float self_scale) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int k = k0 + 4 * li;
  const bool kin = k < K;
  const int kc = kin ? k : K - 4;
  const int hw = wave * 2 + h;  // 0..7
#pragma unroll 1
  for (int it = 0; it < TM / 16; ++it) {
    const int ra = hw + 16 * it, rb = ra + 8;
    const int64_t rowa = r0 + ra, rowb = r0 + rb;
    const int64_t rca = rowa < M ? rowa : M - 1, rcb = rowb < M ? rowb : M - 1;
    f32x4 sa = zero4(), sb = zero4();
    if (self_scale != 0.f) {
      sa = ld4(X + rca * K + kc);
      sb = ld4(X + rcb * K + kc);
    }
    f32x4 a = agg_row<STAGED>(ti, ra, X, K, kc, col, w, rca);
    f32x4 b = agg_row<STAGED>(ti, rb, X, K, kc, col, w, rcb);
    if (self_scale != 0.f) {
      a += self_scale * sa;
      b += self_scale * sb;
    }
    st4(Xs + ra * LDS + 4 * li, sel4(kin && rowa < M, a));
    st4(Xs + rb * LDS + 4 * li, sel4(kin && rowb < M, b));
  }
}

__device__ __forceinline__ void fill_gather(float* Xs, TileIdx& ti, const float* __restrict__ X,
                                            int64_t M, int K, int k0, int64_t r0,
                                            const int32_t* __restrict__ rowptr,
                                            const int32_t* __restrict__ col,
                                            const float* __restrict__ w, float self_scale) {
  if (stage_idx(ti, rowptr, col, w, M, r0))
    fill_gather_t<true>(Xs, ti, X, M, K, k0, r0, col, w, self_scale);
  else
    fill_gather_t<false>(Xs, ti, X, M, K, k0, r0, col, w, self_scale);
}

// ------------------------------------------------------------------------------------------
// Forward: Y = act(P(X) W^T + b)
// ------------------------------------------------------------------------------------------
template <bool GATHER, bool VEC, int ACT>
__global__ __launch_bounds__(NT) void k_linear_fwd(const float* __restrict__ X, int64_t M, int K,
                                                   const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ col,
                                                   const float* __restrict__ w, float self_scale,
                                                   const float* __restrict__ W,
                                                   const float* __restrict__ b, int N,
                                                   float* __restrict__ Y) {
  __shared__ __attribute__((aligned(16))) float Xs[TM * LDS];
  __shared__ TileIdx ti;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t r0 = (int64_t)blockIdx.x * TM;
  const int nw = blockIdx.y * TN + wave * 32;  // first output column of this wave
  const int n = nw + li;                        // this lane's B / output column
  const int ncl = n < N ? n : N - 1;
  const bool wave_active = nw < N;
  f32x16 acc0 = {}, acc1 = {};

  for (int k0 = 0; k0 < K; k0 += KC) {
    // B fragment: W[n][k0 + 64h + s], s = 0..63 (issued before the tile fill)
    float bf[64];
    if constexpr (VEC) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = k0 + 64 * h + 4 * q;
        const f32x4 v = ld4(W + (int64_t)ncl * K + (k < K ? k : K - 4));
        const bool ok = n < N && k < K;
        bf[4 * q + 0] = ok ? v[0] : 0.f;
        bf[4 * q + 1] = ok ? v[1] : 0.f;
        bf[4 * q + 2] = ok ? v[2] : 0.f;
        bf[4 * q + 3] = ok ? v[3] : 0.f;
      }
    } else {
#pragma unroll
      for (int s = 0; s < 64; ++s) {
        const int k = k0 + 64 * h + s;
        const float v = W[(int64_t)ncl * K + (k < K ? k : K - 1)];
        bf[s] = (n < N && k < K) ? v : 0.f;
      }
    }
    if constexpr (GATHER)
      fill_gather(Xs, ti, X, M, K, k0, r0, rowptr, col, w, self_scale);
    else
      fill_direct<VEC>(Xs, X, M, K, k0, r0);
    __syncthreads();
    if (wave_active) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const f32x4 a0 = ld4(Xs + li * LDS + 64 * h + 4 * q);
        const f32x4 a1 = ld4(Xs + (32 + li) * LDS + 64 * h + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc0 = mfma32(a0[j], bf[4 * q + j], acc0);
          acc1 = mfma32(a1[j], bf[4 * q + j], acc1);
        }
      }
    }
    __syncthreads();
  }
  if (!wave_active || n >= N) return;
  const float bias = b ? b[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
    const int64_t row0 = r0 + rl, row1 = r0 + 32 + rl;
    float v0 = acc0[r] + bias, v1 = acc1[r] + bias;
    if (ACT == LGNN_ACT_ELU) {
      v0 = elu_f(v0);
      v1 = elu_f(v1);
    }
    if (row0 < M) Y[row0 * N + n] = v0;
    if (row1 < M) Y[row1 * N + n] = v1;
  }
}

// ------------------------------------------------------------------------------------------
// Backward
// ------------------------------------------------------------------------------------------
// dZ tile: dZs[r][c] = G[r0 + r][o0 + c] * act'(H[r0 + r][o0 + c]); requires N % 4 == 0.
// TRANSPOSE mode stages the tile's transpose-CSR (tptr/tidx/tw) like the forward gather.
template <int GMODE, int ACT>
__device__ __forceinline__ void fill_dz(float* dZs, TileIdx& ti, const float* __restrict__ dY,
                                        const int64_t* __restrict__ batch,
                                        const int32_t* __restrict__ gptr, int pool_mean,
                                        const int32_t* __restrict__ tptr,
                                        const int32_t* __restrict__ tidx,
                                        const float* __restrict__ tw, float tself,
                                        const float* __restrict__ H, int64_t M, int N, int o0,
                                        int64_t r0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int o = o0 + 4 * li;
  const bool oin = o < N;
  const int oc = oin ? o : N - 4;
  const int hw = wave * 2 + h;
  if constexpr (GMODE == LGNN_GRAD_TRANSPOSE) {
    const bool staged = stage_idx(ti, tptr, tidx, tw, M, r0);
#pragma unroll 1
    for (int it = 0; it < TM / 16; ++it) {
      const int ra = hw + 16 * it, rb = ra + 8;
      const int64_t rowa = r0 + ra, rowb = r0 + rb;
      const int64_t rca = rowa < M ? rowa : M - 1, rcb = rowb < M ? rowb : M - 1;
      f32x4 sa = zero4(), sb = zero4(), ha = zero4(), hb = zero4();
      if (tself != 0.f) {
        sa = ld4(dY + rca * N + oc);
        sb = ld4(dY + rcb * N + oc);
      }
      if constexpr (ACT == LGNN_ACT_ELU) {
        ha = ld4(H + rca * N + oc);
        hb = ld4(H + rcb * N + oc);
      }
      f32x4 a, b;
      if (staged) {
        a = agg_row<true>(ti, ra, dY, N, oc, tidx, tw, rca);
        b = agg_row<true>(ti, rb, dY, N, oc, tidx, tw, rcb);
      } else {
        a = agg_row<false>(ti, ra, dY, N, oc, tidx, tw, rca);
        b = agg_row<false>(ti, rb, dY, N, oc, tidx, tw, rcb);
      }
      if (tself != 0.f) {
        a += tself * sa;
        b += tself * sb;
      }
      if constexpr (ACT == LGNN_ACT_ELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] *= elu_grad_from_out(ha[j]);
          b[j] *= elu_grad_from_out(hb[j]);
        }
      }
      st4(dZs + ra * LDS + 4 * li, sel4(oin && rowa < M, a));
      st4(dZs + rb * LDS + 4 * li, sel4(oin && rowb < M, b));
    }
  } else {
    f32x4 g[TM / 8], hv[TM / 8];
#pragma unroll
    for (int it = 0; it < TM / 8; ++it) {
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
    for (int it = 0; it < TM / 8; ++it) {
      const int rr = hw + 8 * it;
      f32x4 v = g[it];
      if constexpr (ACT == LGNN_ACT_ELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= elu_grad_from_out(hv[it][j]);
      }
      st4(dZs + rr * LDS + 4 * li, sel4(oin && r0 + rr < M, v));
    }
  }
}

// grid: x = partial slots (persistent over row tiles), y = output block (o0 = 128*y),
// z = input block (k0 = 128*z). With DX, gridDim.y must be 1 (N <= 128).
template <int GMODE, int ACT, bool GATHER, bool DX>
__global__ __launch_bounds__(NT) void k_linear_bwd(
    const float* __restrict__ dY, const int64_t* __restrict__ batch,
    const int32_t* __restrict__ gptr, int pool_mean, const int32_t* __restrict__ tptr,
    const int32_t* __restrict__ tidx, const float* __restrict__ tw, float tself,
    const float* __restrict__ H, const float* __restrict__ X, int64_t M, int K,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ w, float self_scale, const float* __restrict__ W, int N,
    float* __restrict__ dXpre, float* __restrict__ dWp, float* __restrict__ dbp) {
  __shared__ __attribute__((aligned(16))) float dZs[TM * LDS];
  __shared__ __attribute__((aligned(16))) float Ss[TM * LDS];
  __shared__ TileIdx ti;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int o0 = blockIdx.y * TN, k0 = blockIdx.z * KC;
  const int64_t ntiles = (M + TM - 1) / TM;

  f32x16 dw[4] = {{}, {}, {}, {}};
  float dbacc = 0.f;
  // DX B-fragment: W[o = 64h + s][k0 + 32*wave + li]
  float wt[64];
  const int kx = k0 + 32 * wave + li;
  if constexpr (DX) {
    const int kxc = kx < K ? kx : K - 1;
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int o = 64 * h + s;
      const float v = W[(int64_t)(o < N ? o : N - 1) * K + kxc];
      wt[s] = (o < N && kx < K) ? v : 0.f;
    }
  }

  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * TM;
    fill_dz<GMODE, ACT>(dZs, ti, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H, M, N, o0,
                        r0);
    if constexpr (GATHER) {
      __syncthreads();  // ti reuse
      fill_gather(Ss, ti, X, M, K, k0, r0, rowptr, col, w, self_scale);
    } else if ((K & 3) == 0) {
      fill_direct<true>(Ss, X, M, K, k0, r0);
    } else {
      fill_direct<false>(Ss, X, M, K, k0, r0);
    }
    __syncthreads();
    if (tid < TN) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll 8
      for (int r = 0; r < TM; r += 2) {
        s0 += dZs[r * LDS + tid];
        s1 += dZs[(r + 1) * LDS + tid];
      }
      dbacc += s0 + s1;
    }
    // dW[o][k] += sum_m dZ[m][o] S[m][k]; wave owns o in [32w, 32w+32), 4 k-tiles.
#pragma unroll 4
    for (int s = 0; s < TM / 2; ++s) {
      const int m = 2 * s + h;
      const float a = dZs[m * LDS + 32 * wave + li];
#pragma unroll
      for (int j = 0; j < 4; ++j) dw[j] = mfma32(a, Ss[m * LDS + 32 * j + li], dw[j]);
    }
    if constexpr (DX) {
      // dXpre[m][k] = sum_o dZ[m][o] W[o][k]; wave owns k in [k0 + 32w, +32)
      f32x16 x0 = {}, x1 = {};
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const f32x4 a0 = ld4(dZs + li * LDS + 64 * h + 4 * q);
        const f32x4 a1 = ld4(dZs + (32 + li) * LDS + 64 * h + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x0 = mfma32(a0[j], wt[4 * q + j], x0);
          x1 = mfma32(a1[j], wt[4 * q + j], x1);
        }
      }
      if (kx < K) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int64_t row0 = r0 + rl, row1 = r0 + 32 + rl;
          if (row0 < M) dXpre[row0 * K + kx] = x0[r];
          if (row1 < M) dXpre[row1 * K + kx] = x1[r];
        }
      }
    }
    __syncthreads();
  }
  // partial slot blockIdx.x: dW [N][K], db [N]
  float* slab = dWp + (int64_t)blockIdx.x * N * K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + 32 * j + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (o < N && k < K) slab[(int64_t)o * K + k] = dw[j][r];
    }
  }
  if (dbp && blockIdx.z == 0 && tid < TN && o0 + tid < N)
    dbp[(int64_t)blockIdx.x * N + o0 + tid] = dbacc;
}

// dXpre = dZ W for N > 128: one WG per (row tile, 128-wide k block), looping over 128-wide
// output blocks (dZ re-derived per block from the upstream gradient, W fragment per block).
template <int GMODE, int ACT>
__global__ __launch_bounds__(NT) void k_linear_dx(
    const float* __restrict__ dY, const int64_t* __restrict__ batch,
    const int32_t* __restrict__ gptr, int pool_mean, const int32_t* __restrict__ tptr,
    const int32_t* __restrict__ tidx, const float* __restrict__ tw, float tself,
    const float* __restrict__ H, int64_t M, int K, const float* __restrict__ W, int N,
    float* __restrict__ dXpre) {
  __shared__ __attribute__((aligned(16))) float dZs[TM * LDS];
  __shared__ TileIdx ti;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t r0 = (int64_t)blockIdx.x * TM;
  const int kx = blockIdx.y * KC + 32 * wave + li;
  const int kxc = kx < K ? kx : K - 1;
  f32x16 x0 = {}, x1 = {};
  for (int o0 = 0; o0 < N; o0 += TN) {
    float wt[64];
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int o = o0 + 64 * h + s;
      const float v = W[(int64_t)(o < N ? o : N - 1) * K + kxc];
      wt[s] = (o < N && kx < K) ? v : 0.f;
    }
    fill_dz<GMODE, ACT>(dZs, ti, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H, M, N, o0,
                        r0);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const f32x4 a0 = ld4(dZs + li * LDS + 64 * h + 4 * q);
      const f32x4 a1 = ld4(dZs + (32 + li) * LDS + 64 * h + 4 * q);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x0 = mfma32(a0[j], wt[4 * q + j], x0);
        x1 = mfma32(a1[j], wt[4 * q + j], x1);
      }
    }
    __syncthreads();
  }
  if (kx >= K) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
    const int64_t row0 = r0 + rl, row1 = r0 + 32 + rl;
    if (row0 < M) dXpre[row0 * K + kx] = x0[r];
    if (row1 < M) dXpre[row1 * K + kx] = x1[r];
  }
}

template <int GMODE, int ACT>
hipError_t launch_dx(hipStream_t s, const float* dY, const int64_t* batch, const int32_t* gptr,
                     int pool_mean, const int32_t* tptr, const int32_t* tidx, const float* tw,
                     float tself, const float* H, int64_t M, int K, const float* W, int N,
                     float* dXpre) {
  dim3 grid((unsigned)((M + TM - 1) / TM), (unsigned)((K + KC - 1) / KC));
  hipLaunchKernelGGL((k_linear_dx<GMODE, ACT>), grid, dim3(NT), 0, s, dY, batch, gptr, pool_mean,
                     tptr, tidx, tw, tself, H, M, K, W, N, dXpre);
  return hipGetLastError();
}

// out[i] = sum_p partial[p*len + i]: block = 16 waves x 64 columns; wave w sums p = w, w+16, ...
// (all of its loads in flight), then the 16 wave sums are combined in fixed order.
constexpr int RT = 1024;
__global__ __launch_bounds__(RT) void k_reduce(const float* __restrict__ part, int P, int64_t len,
                                               float* __restrict__ out) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  const int64_t ic = i < len ? i : len - 1;
  float s = 0.f;
  int p = wave;
  for (; p + 48 < P; p += 64) {
    const float v0 = part[(int64_t)p * len + ic], v1 = part[(int64_t)(p + 16) * len + ic];
    const float v2 = part[(int64_t)(p + 32) * len + ic], v3 = part[(int64_t)(p + 48) * len + ic];
    s += v0;
    s += v1;
    s += v2;
    s += v3;
  }
  for (; p < P; p += 16) s += part[(int64_t)p * len + ic];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && i < len) {
    float t = red[0][lane];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += red[q][lane];
    out[i] = t;
  }
}

// lgnn_spmm, Y_i = sum_e w_e X[col_e] + self_scale X_i (D % 4 == 0), by 64-row tiles and
// 128-feature chunks: a tile none of whose CSR entries leaves it (k-NN graphs aligned to tiles)
// stages its 64 rows x 128 features in LDS (32 KiB, one coalesced read per row) and gathers
// from there; other tiles gather from global memory. A half wave per row, float4 per lane, EB
// neighbour loads in flight; each row sums its entries in CSR order. Against round 5's
// one-half-wave-per-row kernel (global gathers only, the same sums bit for bit): the sweep's
// width-512 GIN aggregation 116.4 -> 113.9 us per launch, the step -1.0 % (same-box A/B);
// staging the tile's CSR block in LDS as well cost occupancy (145 us).
constexpr int kSpC = 128;  // features per chunk
__global__ __launch_bounds__(NT) void k_spmm_tile(const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col,
                                                  const float* __restrict__ w, float self_scale,
                                                  const float* __restrict__ X, int64_t M, int D,
                                                  float* __restrict__ Y) {
  __shared__ __attribute__((aligned(16))) float S[TM * kSpC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t t = xcd_block();
  const int64_t r0 = t * TM, r1 = r0 + TM < M ? r0 + TM : M;
  const int f0 = blockIdx.y * kSpC;
  const int nf = D - f0 < kSpC ? D - f0 : kSpC;
  const int eb = rowptr[r0], ee = rowptr[r1];
  int out = 0;
  for (int e = eb + (int)threadIdx.x; e < ee; e += NT) {
    const int c = col[e];
    out |= c < r0 || c >= r1;
  }
  const bool closed = !__syncthreads_or(out);
  if (closed) {  // the tile's rows, this chunk's features, into LDS
    for (int q = threadIdx.x; q < (int)(r1 - r0) * (kSpC / 4); q += NT) {
      const int rr = q / (kSpC / 4), k = 4 * (q % (kSpC / 4));
      if (k < nf) st4(S + rr * kSpC + k, ld4(X + (r0 + rr) * D + f0 + k));
    }
    __syncthreads();
  }
  const int k = 4 * li;
  if (k >= nf) return;
  for (int rr = 2 * wave + h; rr < (int)(r1 - r0); rr += NT / 32) {
    const int64_t row = r0 + rr;
    const int e0 = rowptr[row], e1 = rowptr[row + 1];
    f32x4 acc = zero4();
    for (int e = e0; e < e1; e += EB) {
      int c[EB];
      float ww[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const bool ok = e + u < e1;
        const int ee2 = ok ? e + u : e0;
        c[u] = col[ee2];
        ww[u] = ok ? (w ? w[ee2] : 1.f) : 0.f;
      }
      f32x4 v[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u)
        v[u] = closed ? ld4(S + (c[u] - r0) * kSpC + k) : ld4(X + (int64_t)c[u] * D + f0 + k);
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const f32x4 tt = ww[u] * v[u];
        acc += (e + u < e1) ? tt : zero4();
      }
    }
    if (self_scale != 0.f)
      acc += self_scale * (closed ? ld4(S + rr * kSpC + k) : ld4(X + row * D + f0 + k));
    st4(Y + row * D + f0 + k, acc);
  }
}

int grid_partials(int64_t M, int N, int K) {
  const int64_t ntiles = (M + TM - 1) / TM;
  const int gy = (N + TN - 1) / TN, gz = (K + KC - 1) / KC;
  int64_t target = 512 / (gy * gz);
  if (target < 64) target = 64;
  int64_t p = ntiles < target ? ntiles : target;
  return (int)(p < 1 ? 1 : p);
}

template <int GMODE, int ACT, bool GATHER, bool DX>
hipError_t launch_bwd(dim3 grid, hipStream_t s, const float* dY, const int64_t* batch,
                      const int32_t* gptr, int pool_mean, const int32_t* tptr,
                      const int32_t* tidx, const float* tw, float tself, const float* H,
                      const float* X, int64_t M, int K, const int32_t* rowptr, const int32_t* col,
                      const float* w, float self_scale, const float* W, int N, float* dXpre,
                      float* dWp, float* dbp) {
  hipLaunchKernelGGL((k_linear_bwd<GMODE, ACT, GATHER, DX>), grid, dim3(NT), 0, s, dY, batch, gptr,
                     pool_mean, tptr, tidx, tw, tself, H, X, M, K, rowptr, col, w, self_scale, W,
                     N, dXpre, dWp, dbp);
  return hipGetLastError();
}

template <int GMODE, int ACT>
hipError_t dispatch_bwd2(bool gather, bool dx, dim3 grid, hipStream_t s, const float* dY,
                         const int64_t* batch, const int32_t* gptr, int pool_mean,
                         const int32_t* tptr, const int32_t* tidx, const float* tw, float tself,
                         const float* H, const float* X, int64_t M, int K, const int32_t* rowptr,
                         const int32_t* col, const float* w, float self_scale, const float* W,
                         int N, float* dXpre, float* dWp, float* dbp) {
#define LGNN_BWD_ARGS                                                                          \
  grid, s, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H, X, M, K, rowptr, col, w,      \
      self_scale, W, N, dXpre, dWp, dbp
  if (gather) {
    if (dx) return launch_bwd<GMODE, ACT, true, true>(LGNN_BWD_ARGS);
    return launch_bwd<GMODE, ACT, true, false>(LGNN_BWD_ARGS);
  }
  if (dx) return launch_bwd<GMODE, ACT, false, true>(LGNN_BWD_ARGS);
  return launch_bwd<GMODE, ACT, false, false>(LGNN_BWD_ARGS);
#undef LGNN_BWD_ARGS
}

}  // namespace

extern "C" int lgnn_node_linear_fwd(const float* X, int64_t M, int K, const int32_t* rowptr,
                                    const int32_t* col, const float* w, float self_scale,
                                    const float* W, const float* b, int N, int act, float* Y,
                                    float* S_out, void* stream) {
  return lgnn_node_linear_fwd_tiles(X, M, K, rowptr, col, w, self_scale, W, b, N, act, Y, S_out,
                                    nullptr, 0, stream);
}

extern "C" int lgnn_node_linear_fwd_tiles(const float* X, int64_t M, int K,
                                          const int32_t* rowptr, const int32_t* col,
                                          const float* w, float self_scale, const float* W,
                                          const float* b, int N, int act, float* Y, float* S_out,
                                          const int32_t* tile_open, int want_open,
                                          void* stream) {
  if (M < 0 || K <= 0 || N <= 0 || !W || !Y || (M > 0 && !X)) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  const bool gather = rowptr != nullptr;
  if (gather && (!col || (K & 3))) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  const int64_t gx = (M + TM - 1) / TM;
  if (gx > INT32_MAX) return LGNN_EINVAL;
  hipStream_t s = as_stream(stream);
  if (lgnn_tile_fits(M, K, N)) {
    const hipError_t e = lgnn_tile_fwd(s, X, M, K, rowptr, col, w, self_scale, W, b, N, act, Y,
                                       gather ? S_out : nullptr, tile_open, want_open);
    return e == hipSuccess ? LGNN_OK : (int)e;
  }
  if (tile_open) return LGNN_EINVAL;  // tile selection only on the fast path
  if (S_out) return LGNN_EINVAL;  // S_out only on the fast path (K, N <= 128)
  dim3 grid((unsigned)gx, (unsigned)((N + TN - 1) / TN));
  const bool vec = (K & 3) == 0;
#define LGNN_FWD(G, V, A)                                                                         \
  hipLaunchKernelGGL((k_linear_fwd<G, V, A>), grid, dim3(NT), 0, s, X, M, K, rowptr, col, w,      \
                     self_scale, W, b, N, Y)
  if (gather) {
    if (act == LGNN_ACT_ELU) LGNN_FWD(true, true, LGNN_ACT_ELU);
    else LGNN_FWD(true, true, LGNN_ACT_NONE);
  } else if (vec) {
    if (act == LGNN_ACT_ELU) LGNN_FWD(false, true, LGNN_ACT_ELU);
    else LGNN_FWD(false, true, LGNN_ACT_NONE);
  } else {
    if (act == LGNN_ACT_ELU) LGNN_FWD(false, false, LGNN_ACT_ELU);
    else LGNN_FWD(false, false, LGNN_ACT_NONE);
  }
#undef LGNN_FWD
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

// The fast path applies when the prologue is direct (S streamed, not re-gathered).
static hipStream_t s_(void* p) { return as_stream(p); }
static bool bwd_fast(int64_t M, int N, int K, bool gather) {
  return !gather && lgnn_tile_fits(M, K, N);
}

extern "C" int lgnn_bwd_num_partials(int64_t M, int N, int K, int gather) {
  if (M < 0 || N <= 0 || K <= 0) return LGNN_EINVAL;
  return bwd_fast(M, N, K, gather != 0) ? lgnn_tile_partials(M) : grid_partials(M, N, K);
}

extern "C" int lgnn_node_linear_bwd(int grad_mode, const float* dY, const int64_t* batch,
                                    const int32_t* gptr, int pool_mean, const int32_t* tptr,
                                    const int32_t* tidx, const float* tw, float tself,
                                    const float* H, int act, const float* X, int64_t M, int K,
                                    const int32_t* rowptr, const int32_t* col, const float* w,
                                    float self_scale, const float* W, int N, float* dXpre,
                                    float* dW_partial, float* db_partial, int num_partials,
                                    void* stream) {
  return lgnn_node_linear_bwd_tiles(grad_mode, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself,
                                    H, act, X, M, K, rowptr, col, w, self_scale, W, N, dXpre,
                                    dW_partial, db_partial, num_partials, nullptr, 0, 0, stream);
}

extern "C" int lgnn_node_linear_bwd_tiles(int grad_mode, const float* dY, const int64_t* batch,
                                          const int32_t* gptr, int pool_mean,
                                          const int32_t* tptr, const int32_t* tidx,
                                          const float* tw, float tself, const float* H, int act,
                                          const float* X, int64_t M, int K,
                                          const int32_t* rowptr, const int32_t* col,
                                          const float* w, float self_scale, const float* W, int N,
                                          float* dXpre, float* dW_partial, float* db_partial,
                                          int num_partials, const int32_t* tile_open,
                                          int want_open, int accumulate, void* stream) {
  if (M < 0 || K <= 0 || N <= 0 || (N & 3) || !W || !dW_partial) return LGNN_EINVAL;
  if (accumulate < 0 || accumulate > 2 ||
      (accumulate == 2 && (!tile_open || num_partials > LGNN_SLOT_FLAGS)))
    return LGNN_EINVAL;
  const bool fast = bwd_fast(M, N, K, rowptr != nullptr);
  if (tile_open && !fast) return LGNN_EINVAL;  // tile selection only on the fast path
  if (!tile_open && num_partials != (fast ? lgnn_tile_partials(M) : grid_partials(M, N, K)))
    return LGNN_EINVAL;
  if (num_partials <= 0) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  if (act == LGNN_ACT_ELU && !H) return LGNN_EINVAL;
  if (grad_mode == LGNN_GRAD_POOL && (!batch || !gptr)) return LGNN_EINVAL;
  if (grad_mode == LGNN_GRAD_TRANSPOSE && (!tptr || !tidx)) return LGNN_EINVAL;
  if (grad_mode < 0 || grad_mode > 2 || (M > 0 && (!dY || !X))) return LGNN_EINVAL;
  const bool gather = rowptr != nullptr;
  if (gather && (!col || (K & 3))) return LGNN_EINVAL;
  if (fast && M > 0) {
    const hipError_t ef = lgnn_tile_bwd(s_(stream), grad_mode, dY, batch, gptr, pool_mean, tptr,
                                        tidx, tw, tself, H, act, X, M, K, W, N, dXpre, dW_partial,
                                        db_partial, num_partials, tile_open, want_open,
                                        accumulate);
    return ef == hipSuccess ? LGNN_OK : (int)ef;
  }
  const bool dx_sep = dXpre != nullptr && N > TN;  // dZ W needs every output block: own kernel
  const bool dx = dXpre != nullptr && !dx_sep;
  hipStream_t s = as_stream(stream);
  if (dx_sep && M > 0) {
    hipError_t e2;
#define LGNN_DX_CALL(GM, AC) \
  launch_dx<GM, AC>(s, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H, M, K, W, N, dXpre)
    if (act == LGNN_ACT_ELU) {
      if (grad_mode == LGNN_GRAD_DIRECT) e2 = LGNN_DX_CALL(LGNN_GRAD_DIRECT, LGNN_ACT_ELU);
      else if (grad_mode == LGNN_GRAD_POOL) e2 = LGNN_DX_CALL(LGNN_GRAD_POOL, LGNN_ACT_ELU);
      else e2 = LGNN_DX_CALL(LGNN_GRAD_TRANSPOSE, LGNN_ACT_ELU);
    } else {
      if (grad_mode == LGNN_GRAD_DIRECT) e2 = LGNN_DX_CALL(LGNN_GRAD_DIRECT, LGNN_ACT_NONE);
      else if (grad_mode == LGNN_GRAD_POOL) e2 = LGNN_DX_CALL(LGNN_GRAD_POOL, LGNN_ACT_NONE);
      else e2 = LGNN_DX_CALL(LGNN_GRAD_TRANSPOSE, LGNN_ACT_NONE);
    }
#undef LGNN_DX_CALL
    if (e2 != hipSuccess) return (int)e2;
  }
  dim3 grid((unsigned)num_partials, (unsigned)((N + TN - 1) / TN), (unsigned)((K + KC - 1) / KC));
  hipError_t e;
#define LGNN_BWD_CALL(GM, AC)                                                                    \
  dispatch_bwd2<GM, AC>(gather, dx, grid, s, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H, \
                        X, M, K, rowptr, col, w, self_scale, W, N, dXpre, dW_partial, db_partial)
  if (act == LGNN_ACT_ELU) {
    if (grad_mode == LGNN_GRAD_DIRECT) e = LGNN_BWD_CALL(LGNN_GRAD_DIRECT, LGNN_ACT_ELU);
    else if (grad_mode == LGNN_GRAD_POOL) e = LGNN_BWD_CALL(LGNN_GRAD_POOL, LGNN_ACT_ELU);
    else e = LGNN_BWD_CALL(LGNN_GRAD_TRANSPOSE, LGNN_ACT_ELU);
  } else {
    if (grad_mode == LGNN_GRAD_DIRECT) e = LGNN_BWD_CALL(LGNN_GRAD_DIRECT, LGNN_ACT_NONE);
    else if (grad_mode == LGNN_GRAD_POOL) e = LGNN_BWD_CALL(LGNN_GRAD_POOL, LGNN_ACT_NONE);
    else e = LGNN_BWD_CALL(LGNN_GRAD_TRANSPOSE, LGNN_ACT_NONE);
  }
#undef LGNN_BWD_CALL
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_reduce_partials(const float* partial, int P, int64_t len, float* out,
                                    void* stream) {
  if (P <= 0 || len < 0 || !partial || !out) return LGNN_EINVAL;
  if (len == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_reduce, dim3((unsigned)((len + 63) / 64)), dim3(RT), 0, as_stream(stream),
                     partial, P, len, out);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_spmm(const int32_t* rowptr, const int32_t* col, const float* w,
                         float self_scale, const float* X, int64_t M, int D, float* Y,
                         void* stream) {
  if (M < 0 || D <= 0 || (D & 3) || !rowptr || !col || (M > 0 && (!X || !Y))) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_spmm_tile,
                     dim3((unsigned)((M + TM - 1) / TM), (unsigned)((D + kSpC - 1) / kSpC)),
                     dim3(NT), 0, as_stream(stream), rowptr, col, w, self_scale, X, M, D, Y);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
