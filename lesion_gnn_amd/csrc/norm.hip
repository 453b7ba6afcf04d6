// BatchNorm1d (training and eval) + ELU (+ dropout mask) kernels for the GIN MLP
// (PyG MLP([d1, d2, d2], act="ELU", norm="batch_norm"), reference gin.py:23:
//  Lin -> BatchNorm -> ELU -> Dropout -> Lin).
//
// Statistics are accumulated in fp64 (as ATen's CPU batch_norm does: acc_type<float> = double),
// deterministically: fixed row ranges per block, fixed-order combination. The per-column sums are
// left in a caller-visible fp64 buffer so a SyncBN all-reduce (RCCL) can run between
// lgnn_bn_stats and lgnn_bn_finalize.
//
// Thread mapping (all kernels): a row of up to 128 columns is covered by 32 lanes holding 4
// consecutive columns each (blockIdx.y = 128-column chunk); the block's 8 half-wave row groups
// stride rows, so per-column constants stay in registers and every row access is one 16-B load
// per lane (512 contiguous bytes per half-wave). Sums: four rows in flight per thread.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int RG = NT / 32;           // row groups per block
constexpr int ROWS_PER_BLOCK = 256;   // rows summed by one block into one partial
constexpr int RED_SPLIT = 8;          // k_colsum_reduce: partial groups per output

inline int row_blocks(int64_t M) {
  const int64_t b = (M + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  return (int)(b < 1 ? 1 : b);
}

__device__ __forceinline__ f32x4 ld4c(const float* p, int c, int N) {
  return c < N ? ld4(p + c) : f32x4{0.f, 0.f, 0.f, 0.f};
}

// MODE 0: sums of z and z^2                        (forward statistics)
// MODE 1: sums of g and g * xhat, g = dA * mask * ELU'(z*scale+shift), xhat = (z-mean)*invstd
template <int MODE>
__global__ __launch_bounds__(NT) void k_colsum(const float* __restrict__ Z,
                                               const float* __restrict__ dA,
                                               const float* __restrict__ mask, int64_t M, int N,
                                               const float* __restrict__ scale,
                                               const float* __restrict__ shift,
                                               const float* __restrict__ mean,
                                               const float* __restrict__ invstd,
                                               double* __restrict__ part) {
  __shared__ double red[2][RG][128];
  const int li = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.y * 128 + 4 * li;
  const bool cin = c < N;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS_PER_BLOCK;
  const int64_t r1 = r0 + ROWS_PER_BLOCK < M ? r0 + ROWS_PER_BLOCK : M;
  f32x4 sc = {}, sh = {}, mu = {}, is = {};
  if constexpr (MODE == 1) {
    sc = ld4c(scale, c, N);
    sh = ld4c(shift, c, N);
    mu = ld4c(mean, c, N);
    is = ld4c(invstd, c, N);
  }
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};
  auto term = [&](int64_t r) {
    const f32x4 z = ld4(Z + r * N + c);
    if constexpr (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s0[j] += (double)z[j];
        s1[j] += (double)z[j] * (double)z[j];
      }
    } else {
      const f32x4 da = ld4(dA + r * N + c);
      const f32x4 m = mask ? ld4(mask + r * N + c) : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g = da[j] * bn_elu_grad(z[j], sc[j], sh[j]) * m[j];
        const float xh = (z[j] - mu[j]) * is[j];
        s0[j] += (double)g;
        s1[j] += (double)g * (double)xh;
      }
    }
  };
  if (cin) {
    int64_t r = r0 + rg;
    for (; r + 3 * RG < r1; r += 4 * RG) {
      term(r);
      term(r + RG);
      term(r + 2 * RG);
      term(r + 3 * RG);
    }
    for (; r < r1; r += RG) term(r);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[0][rg][4 * li + j] = s0[j];
    red[1][rg][4 * li + j] = s1[j];
  }
  __syncthreads();
  if (threadIdx.x < 256) {  // 2 x 128 outputs: (sum kind, column), row groups in fixed order
    const int k = threadIdx.x >> 7, cl = threadIdx.x & 127;
    const int cc = blockIdx.y * 128 + cl;
    double t = red[k][0][cl];
#pragma unroll
    for (int g = 1; g < RG; ++g) t += red[k][g][cl];
    if (cc < N) part[(int64_t)blockIdx.x * 2 * N + k * N + cc] = t;
  }
}

// sums[2N] = sum over P partials: RED_SPLIT strided groups per output (four loads in flight
// each), combined in group order
__global__ __launch_bounds__(NT) void k_colsum_reduce(const double* __restrict__ part, int P,
                                                      int N2, double* __restrict__ sums) {
  __shared__ double red[RED_SPLIT][NT / RED_SPLIT];
  const int o = blockIdx.x * (NT / RED_SPLIT) + (threadIdx.x % (NT / RED_SPLIT));
  const int g = threadIdx.x / (NT / RED_SPLIT);
  double s = 0.0;
  if (o < N2) {
    int p = g;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (; p + 3 * RED_SPLIT < P; p += 4 * RED_SPLIT) {
      a0 += part[(int64_t)p * N2 + o];
      a1 += part[(int64_t)(p + RED_SPLIT) * N2 + o];
      a2 += part[(int64_t)(p + 2 * RED_SPLIT) * N2 + o];
      a3 += part[(int64_t)(p + 3 * RED_SPLIT) * N2 + o];
    }
    for (; p < P; p += RED_SPLIT) a0 += part[(int64_t)p * N2 + o];
    s = (a0 + a1) + (a2 + a3);
  }
  red[g][threadIdx.x % (NT / RED_SPLIT)] = s;
  __syncthreads();
  if (g == 0 && o < N2) {
    double t = red[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < RED_SPLIT; ++k) t += red[k][threadIdx.x];
    sums[o] = t;
  }
}

// Per-column constants. training: batch mean / biased var from the sums s0 = sum z, s1 = sum z^2
// (count rows), running stats updated with the unbiased var (torch.nn.BatchNorm1d, momentum m):
//   running = (1 - m) * running + m * stat.  eval: running stats used as is.
// scale = gamma * invstd, shift = beta - mean * scale (gamma/beta NULL: 1 / 0).
__device__ __forceinline__ void bn_finalize_col(int c, double s0, double s1, double count,
                                                const float* __restrict__ gamma,
                                                const float* __restrict__ beta, float eps,
                                                float momentum, int training,
                                                float* __restrict__ running_mean,
                                                float* __restrict__ running_var,
                                                float* __restrict__ mean_out,
                                                float* __restrict__ invstd_out,
                                                float* __restrict__ scale,
                                                float* __restrict__ shift) {
  double mean, var;
  if (training) {
    mean = s0 / count;
    var = s1 / count - mean * mean;
    if (var < 0.0) var = 0.0;
    if (running_mean) {
      const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
      running_mean[c] = (float)((1.0 - momentum) * (double)running_mean[c] + momentum * mean);
      running_var[c] = (float)((1.0 - momentum) * (double)running_var[c] + momentum * unbiased);
    }
  } else {
    mean = running_mean[c];
    var = running_var[c];
  }
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float m = (float)mean;
  const float g = gamma ? gamma[c] : 1.f;
  const float sc = g * is;
  mean_out[c] = m;
  invstd_out[c] = is;
  scale[c] = sc;
  shift[c] = (beta ? beta[c] : 0.f) - m * sc;
}

__global__ __launch_bounds__(NT) void k_bn_finalize(const double* __restrict__ sums, double count,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float eps,
                                                    float momentum, int training, int N,
                                                    float* __restrict__ running_mean,
                                                    float* __restrict__ running_var,
                                                    int64_t* __restrict__ num_batches_tracked,
                                                    float* __restrict__ mean_out,
                                                    float* __restrict__ invstd_out,
                                                    float* __restrict__ scale,
                                                    float* __restrict__ shift) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c == 0 && training && num_batches_tracked) *num_batches_tracked += 1;
  if (c >= N) return;
  bn_finalize_col(c, training ? sums[c] : 0.0, training ? sums[N + c] : 0.0, count, gamma, beta,
                  eps, momentum, training, running_mean, running_var, mean_out, invstd_out,
                  scale, shift);
}

// The BN-fused linear kernels' partial rows [P][2N] -> sums (fixed order: 8 strided groups per
// column, folded in group order); then (FIN) the per-column constants as k_bn_finalize, and/or
// (PG) the affine parameters' gradients as k_bn_param_grads: one launch instead of two.
template <bool FIN, bool PG>
__global__ __launch_bounds__(NT) void k_bn_reduce_tail(
    const double* __restrict__ part, int P, int N, double* __restrict__ sums, double count,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    int training, float* __restrict__ running_mean, float* __restrict__ running_var,
    int64_t* __restrict__ num_batches_tracked, float* __restrict__ mean_out,
    float* __restrict__ invstd_out, float* __restrict__ scale, float* __restrict__ shift,
    float* __restrict__ dg, float* __restrict__ db) {
  // 8 columns per block, 32 strided groups of partial rows per column (latency: ~P/32 loads
  // per thread, 4 in flight)
  constexpr int RCOL = 8, RGRP = NT / RCOL;
  __shared__ double red[RGRP][2][RCOL];
  const int cl = threadIdx.x % RCOL, g = threadIdx.x / RCOL;
  const int c = blockIdx.x * RCOL + cl;
  double s0 = 0.0, s1 = 0.0;
  if (c < N) {
#pragma unroll 4
    for (int p = g; p < P; p += RGRP) {
      s0 += part[(int64_t)p * 2 * N + c];
      s1 += part[(int64_t)p * 2 * N + N + c];
    }
  }
  red[g][0][cl] = s0;
  red[g][1][cl] = s1;
  __syncthreads();
  if (g != 0 || c >= N) return;
  double t0 = red[0][0][cl], t1 = red[0][1][cl];
#pragma unroll 8
  for (int k = 1; k < RGRP; ++k) {
    t0 += red[k][0][cl];
    t1 += red[k][1][cl];
  }
  sums[c] = t0;
  sums[N + c] = t1;
  if constexpr (PG) {
    if (dg) dg[c] = (float)t1;
    if (db) db[c] = (float)t0;
  }
  if constexpr (FIN) {
    if (c == 0 && training && num_batches_tracked) *num_batches_tracked += 1;
    bn_finalize_col(c, t0, t1, count, gamma, beta, eps, momentum, training, running_mean,
                    running_var, mean_out, invstd_out, scale, shift);
  }
}

// A = ELU(Z * scale + shift) [* mask]; per-column constants in registers (thread mapping above)
__global__ __launch_bounds__(NT) void k_bn_act(const float* __restrict__ Z, int64_t M, int N,
                                               const float* __restrict__ scale,
                                               const float* __restrict__ shift,
                                               const float* __restrict__ mask,
                                               float* __restrict__ A) {
  const int li = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.y * 128 + 4 * li;
  if (c >= N) return;
  const f32x4 sc = ld4(scale + c), sh = ld4(shift + c);
  for (int64_t r = (int64_t)blockIdx.x * RG + rg; r < M; r += (int64_t)gridDim.x * RG) {
    const f32x4 z = ld4(Z + r * N + c);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = elu_f(fmaf(z[j], sc[j], sh[j]));
    if (mask) o *= ld4(mask + r * N + c);
    st4(A + r * N + c, o);
  }
}

// dZ = scale * (g - sums0/count - xhat * sums1/count)   (training; torch batch_norm backward)
// dZ = scale * g                                         (eval)
// g = dA * mask * ELU'(Z*scale+shift), xhat = (Z - mean) * invstd.
__global__ __launch_bounds__(NT) void k_bn_bwd_apply(const float* __restrict__ dA,
                                                     const float* __restrict__ Z,
                                                     const float* __restrict__ mask, int64_t M,
                                                     int N, const float* __restrict__ scale,
                                                     const float* __restrict__ shift,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ invstd,
                                                     const double* __restrict__ sums,
                                                     double count, int training,
                                                     float* __restrict__ dZ) {
  const int li = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.y * 128 + 4 * li;
  if (c >= N) return;
  const f32x4 sc = ld4(scale + c), sh = ld4(shift + c), mu = ld4(mean + c), is = ld4(invstd + c);
  f32x4 mg = {}, mgx = {};
  if (training) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mg[j] = (float)(sums[c + j] / count);
      mgx[j] = (float)(sums[N + c + j] / count);
    }
  }
  for (int64_t r = (int64_t)blockIdx.x * RG + rg; r < M; r += (int64_t)gridDim.x * RG) {
    const f32x4 z = ld4(Z + r * N + c);
    const f32x4 da = ld4(dA + r * N + c);
    const f32x4 m = mask ? ld4(mask + r * N + c) : f32x4{1.f, 1.f, 1.f, 1.f};
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float g = da[j] * bn_elu_grad(z[j], sc[j], sh[j]) * m[j];
      if (training) {
        const float xh = (z[j] - mu[j]) * is[j];
        o[j] = sc[j] * (g - mg[j] - xh * mgx[j]);
      } else {
        o[j] = sc[j] * g;
      }
    }
    st4(dZ + r * N + c, o);
  }
}

// dgamma = sums1, dbeta = sums0 (fp64 -> fp32)
__global__ void k_bn_param_grads(const double* __restrict__ sums, int N, float* __restrict__ dg,
                                 float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  if (dg) dg[c] = (float)sums[N + c];
  if (db) db[c] = (float)sums[c];
}

// elementwise grid: row blocks of RG rows (capped), x 128-column chunks
inline dim3 ew_grid(int64_t M, int N) {
  int64_t g = (M + RG - 1) / RG;
  if (g > 2048) g = 2048;
  return dim3((unsigned)(g < 1 ? 1 : g), (unsigned)((N + 127) / 128));
}

}  // namespace

extern "C" size_t lgnn_bn_workspace_bytes(int64_t M, int N) {
  return (size_t)row_blocks(M) * 2 * (size_t)N * sizeof(double);
}

extern "C" int lgnn_bn_stats(const float* Z, int64_t M, int N, double* sums, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (M < 0 || N <= 0 || (N & 3) || !sums || (M > 0 && !Z)) return LGNN_EINVAL;
  if (!workspace || workspace_bytes < lgnn_bn_workspace_bytes(M, N)) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const int P = row_blocks(M);
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(k_colsum<0>, dim3(P, (N + 127) / 128), dim3(NT), 0, s, Z, nullptr, nullptr,
                     M, N, nullptr, nullptr, nullptr, nullptr, part);
  LGNN_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_colsum_reduce, dim3((2 * N + NT / RED_SPLIT - 1) / (NT / RED_SPLIT)),
                     dim3(NT), 0, s, part, P, 2 * N, sums);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_bn_finalize(const double* sums, double count, const float* gamma,
                                const float* beta, float eps, float momentum, int training, int N,
                                float* running_mean, float* running_var,
                                int64_t* num_batches_tracked, float* mean, float* invstd,
                                float* scale, float* shift, void* stream) {
  if (N <= 0 || !mean || !invstd || !scale || !shift) return LGNN_EINVAL;
  if (training && (!sums || count <= 0.0)) return LGNN_EINVAL;
  if (!training && (!running_mean || !running_var)) return LGNN_EINVAL;
  if ((running_mean == nullptr) != (running_var == nullptr)) return LGNN_EINVAL;
  hipLaunchKernelGGL(k_bn_finalize, dim3((N + NT - 1) / NT), dim3(NT), 0, as_stream(stream), sums,
                     count, gamma, beta, eps, momentum, training, N, running_mean, running_var,
                     num_batches_tracked, mean, invstd, scale, shift);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_bn_act(const float* Z, int64_t M, int N, const float* scale,
                           const float* shift, const float* mask, float* A, void* stream) {
  if (M < 0 || N <= 0 || (N & 3) || !scale || !shift || (M > 0 && (!Z || !A)))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_bn_act, ew_grid(M, N), dim3(NT), 0, as_stream(stream), Z, M, N, scale,
                     shift, mask, A);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_bn_bwd_stats(const float* dA, const float* Z, const float* mask, int64_t M,
                                 int N, const float* scale, const float* shift, const float* mean,
                                 const float* invstd, double* sums, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  if (M < 0 || N <= 0 || (N & 3) || !sums || !scale || !shift || !mean || !invstd)
    return LGNN_EINVAL;
  if (M > 0 && (!dA || !Z)) return LGNN_EINVAL;
  if (!workspace || workspace_bytes < lgnn_bn_workspace_bytes(M, N)) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const int P = row_blocks(M);
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(k_colsum<1>, dim3(P, (N + 127) / 128), dim3(NT), 0, s, Z, dA, mask, M, N,
                     scale, shift, mean, invstd, part);
  LGNN_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_colsum_reduce, dim3((2 * N + NT / RED_SPLIT - 1) / (NT / RED_SPLIT)),
                     dim3(NT), 0, s, part, P, 2 * N, sums);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_bn_partials_reduce(const double* part, int num_partials, int N,
                                       double* sums, float* dgamma, float* dbeta, void* stream) {
  if (num_partials <= 0 || N <= 0 || !part || !sums) return LGNN_EINVAL;
  const dim3 grid((unsigned)((N + 7) / 8));
  if (dgamma || dbeta)
    hipLaunchKernelGGL((k_bn_reduce_tail<false, true>), grid, dim3(NT), 0, as_stream(stream),
                       part, num_partials, N, sums, 0.0, nullptr, nullptr, 0.f, 0.f, 0, nullptr,
                       nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, dgamma, dbeta);
  else
    hipLaunchKernelGGL((k_bn_reduce_tail<false, false>), grid, dim3(NT), 0, as_stream(stream),
                       part, num_partials, N, sums, 0.0, nullptr, nullptr, 0.f, 0.f, 0, nullptr,
                       nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_bn_partials_finalize(const double* part, int num_partials, int N,
                                         double* sums, double count, const float* gamma,
                                         const float* beta, float eps, float momentum,
                                         float* running_mean, float* running_var,
                                         int64_t* num_batches_tracked, float* mean,
                                         float* invstd, float* scale, float* shift,
                                         void* stream) {
  if (num_partials <= 0 || N <= 0 || !part || !sums || count <= 0.0) return LGNN_EINVAL;
  if (!mean || !invstd || !scale || !shift) return LGNN_EINVAL;
  if ((running_mean == nullptr) != (running_var == nullptr)) return LGNN_EINVAL;
  hipLaunchKernelGGL((k_bn_reduce_tail<true, false>), dim3((unsigned)((N + 7) / 8)), dim3(NT),
                     0, as_stream(stream), part, num_partials, N, sums, count, gamma, beta, eps,
                     momentum, 1, running_mean, running_var, num_batches_tracked, mean, invstd,
                     scale, shift, nullptr, nullptr);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_bn_bwd_apply(const float* dA, const float* Z, const float* mask, int64_t M,
                                 int N, const float* scale, const float* shift, const float* mean,
                                 const float* invstd, const double* sums, double count,
                                 int training, float* dZ, float* dgamma, float* dbeta,
                                 void* stream) {
  if (M < 0 || N <= 0 || (N & 3) || !scale || !shift || !mean || !invstd || !sums)
    return LGNN_EINVAL;
  if (training && count <= 0.0) return LGNN_EINVAL;
  hipStream_t s = as_stream(stream);
  if (M > 0) {
    if (!dA || !Z || !dZ) return LGNN_EINVAL;
    hipLaunchKernelGGL(k_bn_bwd_apply, ew_grid(M, N), dim3(NT), 0, s, dA, Z, mask, M, N, scale,
                       shift, mean, invstd, sums, count, training, dZ);
    LGNN_LAUNCH_CHECK();
  }
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(k_bn_param_grads, dim3((N + NT - 1) / NT), dim3(NT), 0, s, sums, N, dgamma,
                       dbeta);
    LGNN_LAUNCH_CHECK();
  }
  return LGNN_OK;
}
