// Readout kernels: per-graph segmented pool (global_mean_pool / global_add_pool) fused with the
// out_proj Linear, and their backward.
//
// Replaces (reference): global_mean_pool(x, batch) gin.py:33 / gat.py:56 (PyG scatter mean =
// sum / clamp(count, 1)), global_add_pool (NEW), out_proj nn.Linear gin.py:25.
#include "common.h"

namespace {

constexpr int NT = 256;

// One wave per graph. Node rows of graph g are contiguous ([ptr[g], ptr[g+1])); lanes stride the
// feature dimension; rows are summed in node order (PyG scatter_add_ order). Then each class logit
// is a wave dot product.
__global__ __launch_bounds__(NT) void k_pool_head_fwd(const float* __restrict__ H,
                                                      const int32_t* __restrict__ gptr, int64_t B,
                                                      int D, int pool_mean,
                                                      const float* __restrict__ Wout,
                                                      const float* __restrict__ bout, int C,
                                                      float* __restrict__ pooled,
                                                      float* __restrict__ logits) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t g = (int64_t)blockIdx.x * 4 + wave;
  if (g >= B) return;
  const int n0 = gptr[g], n1 = gptr[g + 1];
  const int cnt = n1 - n0;
  const float denom = (float)(cnt > 0 ? cnt : 1);
  // up to 8 feature strips of 64 lanes in registers (D <= 512)
  float p[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int d = q * 64 + lane;
    float s = 0.f;
    if (d < D) {
      int i = n0;
      for (; i + 4 <= n1; i += 4) {
        const float v0 = H[(int64_t)i * D + d], v1 = H[(int64_t)(i + 1) * D + d];
        const float v2 = H[(int64_t)(i + 2) * D + d], v3 = H[(int64_t)(i + 3) * D + d];
        s += v0;
        s += v1;
        s += v2;
        s += v3;
      }
      for (; i < n1; ++i) s += H[(int64_t)i * D + d];
      if (pool_mean) s = s / denom;
      pooled[g * D + d] = s;
    }
    p[q] = s;
  }
  if (!Wout) return;
  for (int c = 0; c < C; ++c) {
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int d = q * 64 + lane;
      if (d < D) acc = fmaf(p[q], Wout[(int64_t)c * D + d], acc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) logits[g * C + c] = acc + (bout ? bout[c] : 0.f);
  }
}

__global__ __launch_bounds__(NT) void k_pool_head_fwd4(const float* __restrict__ H,
                                                       const int32_t* __restrict__ gptr, int D,
                                                       int pool_mean,
                                                       const float* __restrict__ Wout,
                                                       const float* __restrict__ bout, int C,
                                                       float* __restrict__ pooled,
                                                       float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) float red[8][512];
  __shared__ float pl[512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, hw = wave * 2 + (lane >> 5);
  const int64_t g = blockIdx.x;
  const int n0 = gptr[g], n1 = gptr[g + 1];
  for (int s0 = 0; s0 < D; s0 += 128) {
    const int f = s0 + 4 * li;
    const int fc = f < D ? f : D - 4;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    int i = n0 + hw;
    for (; i + 56 < n1; i += 64) {  // eight rows in flight, the two-row loop's addition order
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld4(H + (int64_t)(i + 8 * u) * D + fc);
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        a0 += v[u];
        a1 += v[u + 1];
      }
    }
    for (; i + 24 < n1; i += 32) {  // four rows in flight, the two-row loop's addition order
      const f32x4 v0 = ld4(H + (int64_t)i * D + fc);
      const f32x4 v1 = ld4(H + (int64_t)(i + 8) * D + fc);
      const f32x4 v2 = ld4(H + (int64_t)(i + 16) * D + fc);
      const f32x4 v3 = ld4(H + (int64_t)(i + 24) * D + fc);
      a0 += v0;
      a1 += v1;
      a0 += v2;
      a1 += v3;
    }
    for (; i + 8 < n1; i += 16) {
      const f32x4 v0 = ld4(H + (int64_t)i * D + fc);
      const f32x4 v1 = ld4(H + (int64_t)(i + 8) * D + fc);
      a0 += v0;
      a1 += v1;
    }
    if (i < n1) a0 += ld4(H + (int64_t)i * D + fc);
    if (f < D) st4(&red[hw][f], a0 + a1);
  }
  __syncthreads();
  const int cnt = n1 - n0;
  const float denom = (float)(cnt > 0 ? cnt : 1);
  for (int d = threadIdx.x; d < D; d += NT) {
    float t = red[0][d];
#pragma unroll
    for (int r = 1; r < 8; ++r) t += red[r][d];
    if (pool_mean) t = t / denom;
    pooled[g * D + d] = t;
    pl[d] = t;
  }
  if (!Wout) return;
  __syncthreads();
  for (int c = wave; c < C; c += NT / 64) {
    float acc = 0.f;
    for (int d = lane; d < D; d += 64) acc = fmaf(pl[d], Wout[(int64_t)c * D + d], acc);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) logits[g * C + c] = acc + (bout ? bout[c] : 0.f);
  }
}

// One launch for the out_proj backward: blocks [0, nb_dp) compute dpooled[g][d] = sum_c
// dlogits[g][c] Wout[c][d] (one element per thread); the rest compute dWout[c][d] = sum_g
// dlogits[g][c] pooled[g][d] and dbout[c] (block = (class c, 64-wide feature strip), 16 waves
// split g, fixed-order combine).
constexpr int HT = 1024;
__global__ __launch_bounds__(HT) void k_head_bwd(const float* __restrict__ dlogits,
                                                 const float* __restrict__ pooled, int64_t B,
                                                 int D, const float* __restrict__ Wout, int C,
                                                 float* __restrict__ dpooled,
                                                 float* __restrict__ dWout,
                                                 float* __restrict__ dbout, int nb_dp) {
  __shared__ float red[16][65];
  if ((int)blockIdx.x < nb_dp) {
    const int64_t idx = (int64_t)blockIdx.x * HT + threadIdx.x;
    if (idx >= B * D) return;
    const int64_t g = idx / D;
    const int d = (int)(idx % D);
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc = fmaf(dlogits[g * C + c], Wout[(int64_t)c * D + d], acc);
    dpooled[idx] = acc;
    return;
  }
  const int b = (int)blockIdx.x - nb_dp;
  const int nstrip = (D + 63) / 64;
  const int c = b / nstrip, strip = b % nstrip;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int d = strip * 64 + lane;
  const int dc = d < D ? d : D - 1;
  float s = 0.f, sb = 0.f;
#pragma unroll 4
  for (int64_t g = wave; g < B; g += 16) {
    const float dl = dlogits[g * C + c];
    s = fmaf(dl, pooled[g * D + dc], s);
    sb += dl;
  }
  red[wave][lane] = s;
  if (lane == 0) red[wave][64] = sb;
  __syncthreads();
  if (wave == 0) {
    float t = red[0][lane], tb = red[0][64];
#pragma unroll
    for (int q = 1; q < 16; ++q) {
      t += red[q][lane];
      tb += red[q][64];
    }
    if (d < D) dWout[(int64_t)c * D + d] = t;
    if (lane == 0 && strip == 0 && dbout) dbout[c] = tb;
  }
}

__global__ __launch_bounds__(NT) void k_pool_bwd(const float* __restrict__ dp,
                                                 const int64_t* __restrict__ batch,
                                                 const int32_t* __restrict__ gptr, int64_t M,
                                                 int D, int pool_mean, float* __restrict__ dH) {
  const int64_t idx = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (idx >= M * D) return;
  const int64_t i = idx / D;
  const int d = (int)(idx % D);
  const int64_t g = batch[i];
  float v = dp[g * D + d];
  if (pool_mean) {
    const int cnt = gptr[g + 1] - gptr[g];
    v = v / (float)(cnt > 0 ? cnt : 1);
  }
  dH[idx] = v;
}

}  // namespace

extern "C" int lgnn_pool_head_fwd(const float* H, const int32_t* gptr, int64_t B, int D,
                                  int pool_mean, const float* Wout, const float* bout, int C,
                                  float* pooled, float* logits, void* stream) {
  if (B < 0 || D <= 0 || D > 512 || !gptr || !pooled) return LGNN_EINVAL;
  if (Wout && (C <= 0 || !logits)) return LGNN_EINVAL;
  if (B == 0) return LGNN_OK;
  if ((D & 3) == 0)
    hipLaunchKernelGGL(k_pool_head_fwd4, dim3((unsigned)B), dim3(NT), 0, as_stream(stream), H,
                       gptr, D, pool_mean, Wout, bout, C, pooled, logits);
  else
    hipLaunchKernelGGL(k_pool_head_fwd, dim3((unsigned)((B + 3) / 4)), dim3(NT), 0,
                       as_stream(stream), H, gptr, B, D, pool_mean, Wout, bout, C, pooled,
                       logits);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_pool_head_bwd(const float* dlogits, const float* pooled, int64_t B, int D,
                                  const float* Wout, int C, float* dpooled, float* dWout,
                                  float* dbout, void* stream) {
  if (B < 0 || D <= 0 || C <= 0 || !dlogits || !pooled || !Wout) return LGNN_EINVAL;
  const int nb_dp = (dpooled && B > 0) ? (int)((B * D + HT - 1) / HT) : 0;
  const int nb_dw = dWout ? C * ((D + 63) / 64) : 0;
  if (nb_dp + nb_dw == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_head_bwd, dim3((unsigned)(nb_dp + nb_dw)), dim3(HT), 0, as_stream(stream),
                     dlogits, pooled, B, D, Wout, C, dpooled, dWout, dbout, nb_dp);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_pool_bwd(const float* dpooled, const int64_t* batch, const int32_t* gptr,
                             int64_t M, int D, int pool_mean, float* dH, void* stream) {
  if (M < 0 || D <= 0 || !dpooled || !batch || !gptr || !dH) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_pool_bwd, dim3((unsigned)((M * D + NT - 1) / NT)), dim3(NT), 0,
                     as_stream(stream), dpooled, batch, gptr, M, D, pool_mean, dH);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
