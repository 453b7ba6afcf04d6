// Node-tile kernels: fused (aggregate ->) Linear (-> bias -> ELU) forward and the matching fused
// backward, on fp32 MFMA (v_mfma_f32_32x32x2_f32 — exact fp32, gfx950 has no xf32).
//
// Tiling (both kernels): a workgroup = 4 waves = 256 threads owns a 64-node row tile; the tile's
// (aggregated) features are staged in LDS as [64][132] fp32 (row pad 4 floats: conflict-free
// ds_read_b128 A-fragments); wave w owns 32 output columns, so one WG
// covers 128 output features. The K dimension is streamed in chunks of 128.
//
// K permutation: in a 32x32x2 MFMA, lane-half h supplies the k-slot h. We bind slot h of step s
// to feature k = 64h + s, so each lane's A values for consecutive steps are contiguous in LDS
// (one ds_read_b128 feeds 4 steps) and its B values are 64 contiguous floats of one weight row.
//
// Replaces (reference): nn.Linear in_proj/out_proj (gin.py:21,25), GCNConv/GINConv propagate +
// lin (gin.py:23), F.elu (gin.py:31) and their autograd backward.
#include "common.h"

namespace {

constexpr int TM = 64;        // node rows per tile
constexpr int TN = 128;       // output features per workgroup (4 waves x 32)
constexpr int KC = 128;       // K chunk staged in LDS
constexpr int LDS = KC + 4;   // padded LDS row stride (floats)
constexpr int NT = 256;

// ------------------------------------------------------------------------------------------
// Tile fill: Xs[r][c] = P(X)[r0 + r][k0 + c], r < 64, c < 128, zero outside [M) x [K).
// ------------------------------------------------------------------------------------------
template <bool VEC>
__device__ __forceinline__ void fill_direct(float* Xs, const float* __restrict__ X, int64_t M,
                                            int K, int k0, int64_t r0) {
  const int tid = threadIdx.x;
  if constexpr (VEC) {
#pragma unroll
    for (int it = 0; it < (TM * KC / 4) / NT; ++it) {
      const int idx = it * NT + tid;
      const int r = idx >> 5, c4 = idx & 31;
      const int64_t row = r0 + r;
      const int k = k0 + 4 * c4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (row < M && k < K) v = ld4(X + row * K + k);
      st4(Xs + r * LDS + 4 * c4, v);
    }
  } else {
    for (int it = 0; it < (TM * KC) / NT; ++it) {
      const int idx = it * NT + tid;
      const int r = idx >> 7, c = idx & 127;
      const int64_t row = r0 + r;
      const int k = k0 + c;
      Xs[r * LDS + c] = (row < M && k < K) ? X[row * K + k] : 0.f;
    }
  }
}

// Aggregation tile (K % 4 == 0): half-wave per row, float4 per lane. Sum in CSR order (PyG's
// scatter_add_ order), then the self term (GINConv: out + (1 + eps) x).
__device__ __forceinline__ void fill_gather(float* Xs, const float* __restrict__ X, int64_t M,
                                            int K, int k0, int64_t r0,
                                            const int32_t* __restrict__ rowptr,
                                            const int32_t* __restrict__ col,
                                            const float* __restrict__ w, float self_scale) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int k = k0 + 4 * li;
  const bool kin = k < K;
  for (int rr = wave * 2 + h; rr < TM; rr += 8) {
    const int64_t row = r0 + rr;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (row < M) {
      const int e0 = rowptr[row], e1 = rowptr[row + 1];
      int e = e0;
      for (; e + 4 <= e1; e += 4) {
        int c[4];
        float ww[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          c[u] = col[e + u];
          ww[u] = w ? w[e + u] : 1.f;
        }
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[u] = kin ? ld4(X + (int64_t)c[u] * K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += ww[u] * v[u];
      }
      for (; e < e1; ++e) {
        const int c = col[e];
        const float ww = w ? w[e] : 1.f;
        if (kin) acc += ww * ld4(X + (int64_t)c * K + k);
      }
      if (self_scale != 0.f && kin) acc += self_scale * ld4(X + row * K + k);
    }
    if (li < KC / 4) st4(Xs + rr * LDS + 4 * li, acc);
  }
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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t r0 = (int64_t)blockIdx.x * TM;
  const int nw = blockIdx.y * TN + wave * 32;  // first output column of this wave
  const int n = nw + li;                        // this lane's B / output column
  const bool wave_active = nw < N;
  f32x16 acc0 = {}, acc1 = {};

  for (int k0 = 0; k0 < K; k0 += KC) {
    if constexpr (GATHER)
      fill_gather(Xs, X, M, K, k0, r0, rowptr, col, w, self_scale);
    else
      fill_direct<VEC>(Xs, X, M, K, k0, r0);
    // B fragment: W[n][k0 + 64h + s], s = 0..63
    float bf[64];
    if constexpr (VEC) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = k0 + 64 * h + 4 * q;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (n < N && k < K) v = ld4(W + (int64_t)n * K + k);
        bf[4 * q + 0] = v[0];
        bf[4 * q + 1] = v[1];
        bf[4 * q + 2] = v[2];
        bf[4 * q + 3] = v[3];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 64; ++s) {
        const int k = k0 + 64 * h + s;
        bf[s] = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.f;
      }
    }
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
template <int GMODE, int ACT>
__device__ __forceinline__ void fill_dz(float* dZs, const float* __restrict__ dY,
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
  for (int rr = wave * 2 + h; rr < TM; rr += 8) {
    const int64_t row = r0 + rr;
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
    if (row < M && oin) {
      if constexpr (GMODE == LGNN_GRAD_DIRECT) {
        g = ld4(dY + row * N + o);
      } else if constexpr (GMODE == LGNN_GRAD_POOL) {
        const int64_t gi = batch[row];
        g = ld4(dY + gi * N + o);
        if (pool_mean) {
          const int cnt = gptr[gi + 1] - gptr[gi];
          g = g / (float)(cnt > 0 ? cnt : 1);
        }
      } else {
        const int e0 = tptr[row], e1 = tptr[row + 1];
        int e = e0;
        for (; e + 4 <= e1; e += 4) {
          int c[4];
          float ww[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            c[u] = tidx[e + u];
            ww[u] = tw ? tw[e + u] : 1.f;
          }
          f32x4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = ld4(dY + (int64_t)c[u] * N + o);
#pragma unroll
          for (int u = 0; u < 4; ++u) g += ww[u] * v[u];
        }
        for (; e < e1; ++e) g += (tw ? tw[e] : 1.f) * ld4(dY + (int64_t)tidx[e] * N + o);
        if (tself != 0.f) g += tself * ld4(dY + row * N + o);
      }
      if constexpr (ACT == LGNN_ACT_ELU) {
        const f32x4 hv = ld4(H + row * N + o);
        g[0] *= elu_grad_from_out(hv[0]);
        g[1] *= elu_grad_from_out(hv[1]);
        g[2] *= elu_grad_from_out(hv[2]);
        g[3] *= elu_grad_from_out(hv[3]);
      }
    }
    st4(dZs + rr * LDS + 4 * li, g);
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
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int o = 64 * h + s;
      wt[s] = (o < N && kx < K) ? W[(int64_t)o * K + kx] : 0.f;
    }
  }

  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * TM;
    fill_dz<GMODE, ACT>(dZs, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H, M, N, o0, r0);
    if constexpr (GATHER)
      fill_gather(Ss, X, M, K, k0, r0, rowptr, col, w, self_scale);
    else if ((K & 3) == 0)
      fill_direct<true>(Ss, X, M, K, k0, r0);
    else
      fill_direct<false>(Ss, X, M, K, k0, r0);
    __syncthreads();
    if (tid < TN) {
#pragma unroll 8
      for (int r = 0; r < TM; ++r) dbacc += dZs[r * LDS + tid];
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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t r0 = (int64_t)blockIdx.x * TM;
  const int kx = blockIdx.y * KC + 32 * wave + li;
  f32x16 x0 = {}, x1 = {};
  for (int o0 = 0; o0 < N; o0 += TN) {
    fill_dz<GMODE, ACT>(dZs, dY, batch, gptr, pool_mean, tptr, tidx, tw, tself, H, M, N, o0, r0);
    float wt[64];
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int o = o0 + 64 * h + s;
      wt[s] = (o < N && kx < K) ? W[(int64_t)o * K + kx] : 0.f;
    }
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

// out[i] = sum_p partial[p*len + i]: block = 4 waves x 64 columns; wave w sums p = w, w+4, ...;
// the four wave sums are combined in fixed order.
__global__ __launch_bounds__(NT) void k_reduce(const float* __restrict__ part, int P, int64_t len,
                                               float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  float s = 0.f;
  if (i < len) {
    int p = wave;
    for (; p + 12 < P; p += 16) {
      const float v0 = part[(int64_t)p * len + i], v1 = part[(int64_t)(p + 4) * len + i];
      const float v2 = part[(int64_t)(p + 8) * len + i], v3 = part[(int64_t)(p + 12) * len + i];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; p < P; p += 4) s += part[(int64_t)p * len + i];
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && i < len) out[i] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// Y_i = sum_e w_e X[col_e] + self_scale X_i; D % 4 == 0; a half wave per row, float4 per lane,
// looping over D in 128-float strips.
__global__ __launch_bounds__(NT) void k_spmm(const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ col,
                                             const float* __restrict__ w, float self_scale,
                                             const float* __restrict__ X, int64_t M, int D,
                                             float* __restrict__ Y) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t row = ((int64_t)blockIdx.x * 4 + wave) * 2 + h;
  if (row >= M) return;
  const int e0 = rowptr[row], e1 = rowptr[row + 1];
  for (int k = 4 * li; k < D; k += 128) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int e = e0; e < e1; ++e) acc += (w ? w[e] : 1.f) * ld4(X + (int64_t)col[e] * D + k);
    if (self_scale != 0.f) acc += self_scale * ld4(X + row * D + k);
    st4(Y + row * D + k, acc);
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
                                    void* stream) {
  if (M < 0 || K <= 0 || N <= 0 || !W || !Y || (M > 0 && !X)) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  const bool gather = rowptr != nullptr;
  if (gather && (!col || (K & 3))) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  const int64_t gx = (M + TM - 1) / TM;
  if (gx > INT32_MAX) return LGNN_EINVAL;
  dim3 grid((unsigned)gx, (unsigned)((N + TN - 1) / TN));
  hipStream_t s = as_stream(stream);
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

extern "C" int lgnn_bwd_num_partials(int64_t M, int N, int K) {
  if (M < 0 || N <= 0 || K <= 0) return LGNN_EINVAL;
  return grid_partials(M, N, K);
}

extern "C" int lgnn_node_linear_bwd(int grad_mode, const float* dY, const int64_t* batch,
                                    const int32_t* gptr, int pool_mean, const int32_t* tptr,
                                    const int32_t* tidx, const float* tw, float tself,
                                    const float* H, int act, const float* X, int64_t M, int K,
                                    const int32_t* rowptr, const int32_t* col, const float* w,
                                    float self_scale, const float* W, int N, float* dXpre,
                                    float* dW_partial, float* db_partial, int num_partials,
                                    void* stream) {
  if (M < 0 || K <= 0 || N <= 0 || (N & 3) || !W || !dW_partial) return LGNN_EINVAL;
  if (num_partials != grid_partials(M, N, K)) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  if (act == LGNN_ACT_ELU && !H) return LGNN_EINVAL;
  if (grad_mode == LGNN_GRAD_POOL && (!batch || !gptr)) return LGNN_EINVAL;
  if (grad_mode == LGNN_GRAD_TRANSPOSE && (!tptr || !tidx)) return LGNN_EINVAL;
  if (grad_mode < 0 || grad_mode > 2 || (M > 0 && (!dY || !X))) return LGNN_EINVAL;
  const bool gather = rowptr != nullptr;
  if (gather && (!col || (K & 3))) return LGNN_EINVAL;
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
  hipLaunchKernelGGL(k_reduce, dim3((unsigned)((len + 63) / 64)), dim3(NT), 0, as_stream(stream),
                     partial, P, len, out);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_spmm(const int32_t* rowptr, const int32_t* col, const float* w,
                         float self_scale, const float* X, int64_t M, int D, float* Y,
                         void* stream) {
  if (M < 0 || D <= 0 || (D & 3) || !rowptr || !col || (M > 0 && (!X || !Y))) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_spmm, dim3((unsigned)((M + 7) / 8)), dim3(NT), 0, as_stream(stream), rowptr,
                     col, w, self_scale, X, M, D, Y);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
