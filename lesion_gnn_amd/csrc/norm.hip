// BatchNorm1d (training and eval) + ELU (+ dropout mask) kernels for the GIN MLP
// (PyG MLP([d1, d2, d2], act="ELU", norm="batch_norm"), reference gin.py:23:
//  Lin -> BatchNorm -> ELU -> Dropout -> Lin).
//
// Statistics are accumulated in fp64 (as ATen's CPU batch_norm does: acc_type<float> = double),
// deterministically: fixed row ranges per block, fixed-order combination. The per-column sums are
// left in a caller-visible fp64 buffer so a SyncBN all-reduce (RCCL) can run between
// lgnn_bn_stats and lgnn_bn_finalize.
//
// Column mapping (all kernels): blockIdx.y = 64-column chunk, lane = column, the block's 4 waves
// stride rows. One fp32 load per lane and row = 256 contiguous bytes per wave instruction.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int ROWS_PER_BLOCK = 512;  // rows summed by one block into one partial

inline int row_blocks(int64_t M) {
  const int64_t b = (M + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  return (int)(b < 1 ? 1 : b);
}

// xhat-side helpers -------------------------------------------------------------------------
__device__ __forceinline__ float bn_elu_grad(float z, float sc, float sh) {
  const float zn = fmaf(z, sc, sh);
  return zn > 0.f ? 1.f : expf(zn);
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
  __shared__ double red[2][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const int cc = c < N ? c : N - 1;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS_PER_BLOCK;
  const int64_t r1 = r0 + ROWS_PER_BLOCK < M ? r0 + ROWS_PER_BLOCK : M;
  float sc = 0.f, sh = 0.f, mu = 0.f, is = 0.f;
  if constexpr (MODE == 1) {
    sc = scale[cc];
    sh = shift[cc];
    mu = mean[cc];
    is = invstd[cc];
  }
  double s0 = 0.0, s1 = 0.0;
  for (int64_t r = r0 + wave; r < r1; r += 4) {
    const float z = Z[r * N + cc];
    if constexpr (MODE == 0) {
      s0 += (double)z;
      s1 += (double)z * (double)z;
    } else {
      float g = dA[r * N + cc] * bn_elu_grad(z, sc, sh);
      if (mask) g *= mask[r * N + cc];
      const float xh = (z - mu) * is;
      s0 += (double)g;
      s1 += (double)g * (double)xh;
    }
  }
  red[0][wave][lane] = s0;
  red[1][wave][lane] = s1;
  __syncthreads();
  if (wave == 0 && c < N) {
    const double t0 = ((red[0][0][lane] + red[0][1][lane]) + red[0][2][lane]) + red[0][3][lane];
    const double t1 = ((red[1][0][lane] + red[1][1][lane]) + red[1][2][lane]) + red[1][3][lane];
    part[(int64_t)blockIdx.x * 2 * N + c] = t0;
    part[(int64_t)blockIdx.x * 2 * N + N + c] = t1;
  }
}

// sums[2N] = sum over P partials in block order
__global__ __launch_bounds__(NT) void k_colsum_reduce(const double* __restrict__ part, int P,
                                                      int N2, double* __restrict__ sums) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= N2) return;
  double s = 0.0;
  for (int p = 0; p < P; ++p) s += part[(int64_t)p * N2 + i];
  sums[i] = s;
}

// Per-column constants. training: batch mean / biased var from sums (count rows), running stats
// updated with the unbiased var (torch.nn.BatchNorm1d, momentum m):
//   running = (1 - m) * running + m * stat.  eval: running stats used as is.
// scale = gamma * invstd, shift = beta - mean * scale (gamma/beta NULL: 1 / 0).
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
  double mean, var;
  if (training) {
    mean = sums[c] / count;
    var = sums[N + c] / count - mean * mean;
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

// A = ELU(Z * scale + shift) [* mask]
__global__ __launch_bounds__(NT) void k_bn_act(const float* __restrict__ Z, int64_t M, int N,
                                               const float* __restrict__ scale,
                                               const float* __restrict__ shift,
                                               const float* __restrict__ mask,
                                               float* __restrict__ A) {
  const int64_t n4 = M * N / 4;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * NT) {
    const int c = (int)((i * 4) % N);
    f32x4 z = ld4(Z + 4 * i);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = elu_f(fmaf(z[j], scale[c + j], shift[c + j]));
    if (mask) o *= ld4(mask + 4 * i);
    st4(A + 4 * i, o);
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
  const int64_t n4 = M * N / 4;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * NT) {
    const int c = (int)((i * 4) % N);
    const f32x4 z = ld4(Z + 4 * i);
    const f32x4 da = ld4(dA + 4 * i);
    f32x4 m = {1.f, 1.f, 1.f, 1.f};
    if (mask) m = ld4(mask + 4 * i);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cj = c + j;
      const float g = da[j] * bn_elu_grad(z[j], scale[cj], shift[cj]) * m[j];
      if (training) {
        const float mg = (float)(sums[cj] / count);
        const float mgx = (float)(sums[N + cj] / count);
        const float xh = (z[j] - mean[cj]) * invstd[cj];
        o[j] = scale[cj] * (g - mg - xh * mgx);
      } else {
        o[j] = scale[cj] * g;
      }
    }
    st4(dZ + 4 * i, o);
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

inline unsigned ew_grid(int64_t n4) {
  int64_t g = (n4 + NT - 1) / NT;
  if (g > 4096) g = 4096;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" size_t lgnn_bn_workspace_bytes(int64_t M, int N) {
  return (size_t)row_blocks(M) * 2 * (size_t)N * sizeof(double);
}

extern "C" int lgnn_bn_stats(const float* Z, int64_t M, int N, double* sums, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (M < 0 || N <= 0 || !sums || (M > 0 && !Z)) return LGNN_EINVAL;
  if (!workspace || workspace_bytes < lgnn_bn_workspace_bytes(M, N)) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const int P = row_blocks(M);
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(k_colsum<0>, dim3(P, (N + 63) / 64), dim3(NT), 0, s, Z, nullptr, nullptr, M,
                     N, nullptr, nullptr, nullptr, nullptr, part);
  LGNN_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_colsum_reduce, dim3((2 * N + NT - 1) / NT), dim3(NT), 0, s, part, P, 2 * N,
                     sums);
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
  hipLaunchKernelGGL(k_bn_act, dim3(ew_grid(M * N / 4)), dim3(NT), 0, as_stream(stream), Z, M, N,
                     scale, shift, mask, A);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_bn_bwd_stats(const float* dA, const float* Z, const float* mask, int64_t M,
                                 int N, const float* scale, const float* shift, const float* mean,
                                 const float* invstd, double* sums, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  if (M < 0 || N <= 0 || !sums || !scale || !shift || !mean || !invstd) return LGNN_EINVAL;
  if (M > 0 && (!dA || !Z)) return LGNN_EINVAL;
  if (!workspace || workspace_bytes < lgnn_bn_workspace_bytes(M, N)) return LGNN_ENOSPC;
  hipStream_t s = as_stream(stream);
  const int P = row_blocks(M);
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(k_colsum<1>, dim3(P, (N + 63) / 64), dim3(NT), 0, s, Z, dA, mask, M, N,
                     scale, shift, mean, invstd, part);
  LGNN_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_colsum_reduce, dim3((2 * N + NT - 1) / NT), dim3(NT), 0, s, part, P, 2 * N,
                     sums);
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
    hipLaunchKernelGGL(k_bn_bwd_apply, dim3(ew_grid(M * N / 4)), dim3(NT), 0, s, dA, Z, mask, M,
                       N, scale, shift, mean, invstd, sums, count, training, dZ);
    LGNN_LAUNCH_CHECK();
  }
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(k_bn_param_grads, dim3((N + NT - 1) / NT), dim3(NT), 0, s, sums, N, dgamma,
                       dbeta);
    LGNN_LAUNCH_CHECK();
  }
  return LGNN_OK;
}
