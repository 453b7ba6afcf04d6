// Cross-entropy criterion (reference models/base.py:93-94: nn.CrossEntropyLoss(weight=class
// weights), mean reduction) and the batched deterministic reduction of per-workgroup partial
// slabs, each in one launch.
//
//   loss = sum_i w[y_i] * (lse_i - z_i[y_i]) / sum_i w[y_i]       (w = 1 when weight == NULL)
//   dz_i = g * w[y_i] / sum_j w[y_j] * (softmax(z_i) - onehot(y_i))
// One workgroup; rows are summed in fixed order (per-thread strided partials, then a fixed
// tree), so the loss is bitwise reproducible.
#include "common.h"

namespace {

constexpr int CT = 1024;

__device__ __forceinline__ float block_sum_fixed(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
    for (int w = 0; w < CT / 64; ++w) t += red[w];
    red[CT / 64] = t;
  }
  __syncthreads();
  return red[CT / 64];
}

// lse[i] = logsumexp(z_i) (saved for the backward); loss[0] = weighted mean NLL; wsum[0];
// FACTORS: also the logits gradient's per-row factors pm [B][C], wt [B] (lgnn_ce_src)
template <bool FACTORS>
__global__ __launch_bounds__(CT) void k_ce_fwd(const float* __restrict__ z,
                                               const int64_t* __restrict__ y,
                                               const float* __restrict__ weight, int64_t B, int C,
                                               float* __restrict__ lse, float* __restrict__ loss,
                                               float* __restrict__ wsum, int* __restrict__ bad,
                                               float* __restrict__ pm, float* __restrict__ wtf) {
  __shared__ float red[CT / 64 + 1];
  if (threadIdx.x == 0) *bad = 0;
  __syncthreads();
  float num = 0.f, den = 0.f;
  for (int64_t i = threadIdx.x; i < B; i += CT) {
    const float* zi = z + i * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, zi[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(zi[c] - m);
    const float l = m + logf(s);
    lse[i] = l;
    const int64_t t = y[i];
    if constexpr (FACTORS) {
      for (int c = 0; c < C; ++c) pm[i * C + c] = ce_pm(zi[c], l, t, c);
      wtf[i] = ce_wt(y, weight, C, i);
    }
    if (t < 0 || t >= C) {
      atomicOr(bad, 1);
      continue;
    }
    const float wt = weight ? weight[t] : 1.f;
    num += wt * (l - zi[t]);
    den += wt;
  }
  const float n = block_sum_fixed(num, red);
  __syncthreads();
  const float d = block_sum_fixed(den, red);
  if (threadIdx.x == 0) {
    loss[0] = n / d;
    wsum[0] = d;
  }
}

__global__ __launch_bounds__(256) void k_ce_bwd(const float* __restrict__ z,
                                                const int64_t* __restrict__ y,
                                                const float* __restrict__ weight, int64_t B,
                                                int C, const float* __restrict__ lse,
                                                const float* __restrict__ wsum,
                                                const float* __restrict__ gloss,
                                                float* __restrict__ dz) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * C) return;
  const int64_t i = idx / C;
  const int c = (int)(idx % C);
  dz[idx] = ce_grad(gloss[0], ce_wt(y, weight, C, i), wsum[0], ce_pm(z[idx], lse[i], y[i], c));
}

// Regression head + criterion (reference gat.py:94-95 / gin.py:66-67: logits.squeeze(1).clamp(0,
// C - 1), then models/base.py:95-96 nn.MSELoss() / nn.SmoothL1Loss(), mean reduction):
//   p_i = clamp(z_i, lo, hi);  loss = (1/B) sum_i l(p_i - y_i)
//   l(d) = d^2 (MSE) | (|d| < 1 ? d^2 / 2 : |d| - 1/2) (SmoothL1, beta = 1)
//   dz_i = [lo <= z_i <= hi] (g_p[i] + g_loss / B * l'(p_i - y_i))   (torch's clamp backward
//   passes the gradient where lo <= z <= hi; l'(d) = 2d | clamp(d, -1, 1))
// Targets are read as int64 class labels (y.float() in the reference) or fp32.
template <typename T>
__device__ __forceinline__ float target_at(const T* y, int64_t i) { return (float)y[i]; }

__device__ __forceinline__ float reg_term(float d, int smooth) {
  if (!smooth) return d * d;
  const float a = fabsf(d);
  return a < 1.f ? 0.5f * d * d : a - 0.5f;
}

template <typename T>
__global__ __launch_bounds__(CT) void k_reg_fwd(const float* __restrict__ z,
                                                const T* __restrict__ y, int64_t B, float lo,
                                                float hi, int smooth, float* __restrict__ pred,
                                                float* __restrict__ loss) {
  __shared__ float red[CT / 64 + 1];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < B; i += CT) {
    const float p = fminf(fmaxf(z[i], lo), hi);
    pred[i] = p;
    acc += reg_term(p - target_at(y, i), smooth);
  }
  const float t = block_sum_fixed(acc, red);
  if (threadIdx.x == 0) loss[0] = t / (float)B;
}

template <typename T>
__global__ __launch_bounds__(256) void k_reg_bwd(const float* __restrict__ z,
                                                 const T* __restrict__ y, int64_t B, float lo,
                                                 float hi, int smooth,
                                                 const float* __restrict__ gloss,
                                                 const float* __restrict__ gpred,
                                                 float* __restrict__ dz) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const float zi = z[i];
  const float p = fminf(fmaxf(zi, lo), hi);
  const float d = p - target_at(y, i);
  const float dl = smooth ? fminf(fmaxf(d, -1.f), 1.f) : 2.f * d;
  float g = gloss ? gloss[0] / (float)B * dl : 0.f;
  if (gpred) g += gpred[i];
  dz[i] = (zi >= lo && zi <= hi) ? g : 0.f;
}

// job j: out_j[i] = sum_{p < P_j} part_j[p * len_j + i] in slot order (as lgnn_reduce_partials);
// with a factor (outer-product job): out_j[c * width_j + d] =
//   sum_p part_j[p * (len_j / width_j) + c] * factor_j[p * width_j + d]
struct ReduceJobs {
  CeSrc ce;                    // ce_part jobs: part[p][c] = the CE logits gradient (ce_dlogit)
  int ce_part[LGNN_MAX_REDUCE];
  const float* part[LGNN_MAX_REDUCE];
  const float* factor[LGNN_MAX_REDUCE];
  float* out[LGNN_MAX_REDUCE];
  int64_t len[LGNN_MAX_REDUCE];
  int P[LGNN_MAX_REDUCE];
  int width[LGNN_MAX_REDUCE];
};

constexpr int RT = 1024;
__global__ __launch_bounds__(RT) void k_reduce_multi(ReduceJobs jobs) {
  __shared__ f32x4 red4[16][64];
  float(*red)[64] = reinterpret_cast<float(*)[64]>(red4);
  const int j = blockIdx.y;
  const int64_t len = jobs.len[j];
  // long plain jobs (the dW slabs) take 16-B loads: 4 columns per lane, 256 per block, the same
  // slot order per column (bitwise the scalar path's sums)
  const bool vec = !jobs.factor[j] && !jobs.ce_part[j] && (len & 3) == 0 && len >= 4096;
  if ((int64_t)blockIdx.x * (vec ? 256 : 64) >= len) return;
  const float* __restrict__ part = jobs.part[j];
  int P = jobs.P[j];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (vec) {
    const int64_t i4 = (int64_t)blockIdx.x * 256 + 4 * lane;
    const int64_t ic4 = i4 < len ? i4 : len - 4;
    f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
    int p = wave;
    for (; p + 16 * 15 < P; p += 16 * 16) {
      f32x4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = ld4(part + (int64_t)(p + 16 * u) * len + ic4);
#pragma unroll
      for (int u = 0; u < 16; ++u) s4 += v[u];
    }
    for (; p < P; p += 16) s4 += ld4(part + (int64_t)p * len + ic4);
    red4[wave][lane] = s4;
    __syncthreads();
    if (wave == 0 && i4 < len) {
      f32x4 t = red4[0][lane];
#pragma unroll
      for (int q = 1; q < 16; ++q) t += red4[q][lane];
      st4(jobs.out[j] + i4, t);
    }
    return;
  }
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  const int64_t ic = i < len ? i : len - 1;
  float s = 0.f;
  int p = wave;
  if (jobs.ce_part[j]) {  // part = the CE logits gradient [P][C], formed here (no dlogits)
    const CeSrc& ce = jobs.ce;
    // the slot order of the materialised-part paths (p = wave, wave + 16, ...), 16 slots'
    // gradients formed (their loads in flight) before they are summed in order
    if (const float* __restrict__ f = jobs.factor[j]) {  // sum_p dz[p][c] * f[p][d]
      const int width = jobs.width[j];
      const int64_t c = ic / width, d = ic % width;
      for (; p + 16 * 15 < P; p += 16 * 16) {
        float av[16], fv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          av[u] = ce_dlogit(ce, p + 16 * u, (int)c);
          fv[u] = f[(int64_t)(p + 16 * u) * width + d];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) s = fmaf(av[u], fv[u], s);
      }
      for (; p < P; p += 16) s = fmaf(ce_dlogit(ce, p, (int)c), f[(int64_t)p * width + d], s);
    } else {
      for (; p + 16 * 15 < P; p += 16 * 16) {
        float av[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) av[u] = ce_dlogit(ce, p + 16 * u, (int)ic);
#pragma unroll
        for (int u = 0; u < 16; ++u) s += av[u];
      }
      for (; p < P; p += 16) s += ce_dlogit(ce, p, (int)ic);
    }
    P = 0;  // fall through to the fixed-order wave fold
  } else if (const float* __restrict__ f = jobs.factor[j]) {  // sum_p part[p][c] * f[p][d]
    const int width = jobs.width[j];
    const int64_t rows = len / width, c = ic / width, d = ic % width;
    for (; p + 16 * 31 < P; p += 16 * 32) {  // 64 loads in flight per lane (latency bound:
      float av[32], fv[32];                   // out_proj's dW over 1024 graphs is 2 rounds)
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        av[u] = part[(int64_t)(p + 16 * u) * rows + c];
        fv[u] = f[(int64_t)(p + 16 * u) * width + d];
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) s = fmaf(av[u], fv[u], s);
    }
    for (; p + 16 * 15 < P; p += 16 * 16) {  // then 32 in flight
      float av[16], fv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        av[u] = part[(int64_t)(p + 16 * u) * rows + c];
        fv[u] = f[(int64_t)(p + 16 * u) * width + d];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) s = fmaf(av[u], fv[u], s);
    }
    for (; p < P; p += 16) s = fmaf(part[(int64_t)p * rows + c], f[(int64_t)p * width + d], s);
    P = 0;  // fall through to the fixed-order wave fold
  }
  // slot order p = wave, wave + 16, ... in every lane; 16 loads in flight (many-slot jobs such
  // as the GAT attention partials, 2048 slots of 384 columns, are latency bound)
  for (; p + 16 * 15 < P; p += 16 * 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = part[(int64_t)(p + 16 * u) * len + ic];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
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
    jobs.out[j][i] = t;
  }
}

}  // namespace

extern "C" int lgnn_ce_fwd(const float* logits, const int64_t* target, const float* weight,
                           int64_t B, int C, float* lse, float* loss, float* wsum, int* bad,
                           void* stream) {
  if (B <= 0 || C <= 0 || !logits || !target || !lse || !loss || !wsum || !bad)
    return LGNN_EINVAL;
  hipLaunchKernelGGL(k_ce_fwd<false>, dim3(1), dim3(CT), 0, as_stream(stream), logits, target,
                     weight, B, C, lse, loss, wsum, bad, nullptr, nullptr);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_ce_fwd_factors(const float* logits, const int64_t* target,
                                   const float* weight, int64_t B, int C, float* lse, float* loss,
                                   float* wsum, int* bad, float* pm, float* wt, void* stream) {
  if (B <= 0 || C <= 0 || !logits || !target || !lse || !loss || !wsum || !bad || !pm || !wt)
    return LGNN_EINVAL;
  hipLaunchKernelGGL(k_ce_fwd<true>, dim3(1), dim3(CT), 0, as_stream(stream), logits, target,
                     weight, B, C, lse, loss, wsum, bad, pm, wt);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_ce_bwd(const float* logits, const int64_t* target, const float* weight,
                           int64_t B, int C, const float* lse, const float* wsum,
                           const float* grad_loss, float* dlogits, void* stream) {
  if (B <= 0 || C <= 0 || !logits || !target || !lse || !wsum || !grad_loss || !dlogits)
    return LGNN_EINVAL;
  hipLaunchKernelGGL(k_ce_bwd, dim3((unsigned)((B * C + 255) / 256)), dim3(256), 0,
                     as_stream(stream), logits, target, weight, B, C, lse, wsum, grad_loss,
                     dlogits);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_regression_fwd(const float* z, const void* target, int target_is_i64,
                                   int64_t B, float lo, float hi, int smooth_l1, float* pred,
                                   float* loss, void* stream) {
  if (B <= 0 || !z || !target || !pred || !loss || !(lo <= hi)) return LGNN_EINVAL;
  if (target_is_i64)
    hipLaunchKernelGGL(k_reg_fwd<int64_t>, dim3(1), dim3(CT), 0, as_stream(stream), z,
                       static_cast<const int64_t*>(target), B, lo, hi, smooth_l1, pred, loss);
  else
    hipLaunchKernelGGL(k_reg_fwd<float>, dim3(1), dim3(CT), 0, as_stream(stream), z,
                       static_cast<const float*>(target), B, lo, hi, smooth_l1, pred, loss);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_regression_bwd(const float* z, const void* target, int target_is_i64,
                                   int64_t B, float lo, float hi, int smooth_l1,
                                   const float* grad_loss, const float* grad_pred, float* dz,
                                   void* stream) {
  if (B <= 0 || !z || !target || !dz || (!grad_loss && !grad_pred)) return LGNN_EINVAL;
  const dim3 grid((unsigned)((B + 255) / 256));
  if (target_is_i64)
    hipLaunchKernelGGL(k_reg_bwd<int64_t>, grid, dim3(256), 0, as_stream(stream), z,
                       static_cast<const int64_t*>(target), B, lo, hi, smooth_l1, grad_loss,
                       grad_pred, dz);
  else
    hipLaunchKernelGGL(k_reg_bwd<float>, grid, dim3(256), 0, as_stream(stream), z,
                       static_cast<const float*>(target), B, lo, hi, smooth_l1, grad_loss,
                       grad_pred, dz);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_reduce_partials_multi(int n, const float* const* partials,
                                          const int* num_partials, const int64_t* len,
                                          float* const* out, void* stream) {
  return lgnn_reduce_jobs(n, partials, nullptr, nullptr, num_partials, len, out, stream);
}

static int reduce_jobs(int n, const float* const* partials, const float* const* factor,
                       const int* width, const int* num_partials, const int64_t* len,
                       float* const* out, const int* ce_job, const lgnn_ce_src* ce, int C,
                       void* stream) {
  if (n <= 0 || n > LGNN_MAX_REDUCE || !partials || !num_partials || !len || !out)
    return LGNN_EINVAL;
  ReduceJobs jobs = {};
  if (ce_job) {
    if (!ce || !ce->pm || !ce->wt || !ce->wsum || !ce->gloss || C < 1)
      return LGNN_EINVAL;
    jobs.ce = CeSrc{ce->pm, ce->wt, ce->wsum, ce->gloss, C};
  }
  int64_t maxlen = 0;
  for (int j = 0; j < n; ++j) {
    const bool cj = ce_job && ce_job[j];
    if ((!partials[j] && !cj) || !out[j] || num_partials[j] <= 0 || len[j] < 0)
      return LGNN_EINVAL;
    if (cj) {  // the [P][C] logits gradient: len = C (db) or C * width (outer product)
      const int64_t rows = factor && factor[j] && width ? len[j] / width[j] : len[j];
      if (rows != C) return LGNN_EINVAL;
      jobs.ce_part[j] = 1;
    }
    if (factor && factor[j]) {
      if (!width || width[j] <= 0 || len[j] % width[j] != 0) return LGNN_EINVAL;
      jobs.factor[j] = factor[j];
      jobs.width[j] = width[j];
    }
    jobs.part[j] = partials[j];
    jobs.out[j] = out[j];
    jobs.len[j] = len[j];
    jobs.P[j] = num_partials[j];
    if (len[j] > maxlen) maxlen = len[j];
  }
  if (maxlen == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_reduce_multi, dim3((unsigned)((maxlen + 63) / 64), (unsigned)n), dim3(RT),
                     0, as_stream(stream), jobs);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_reduce_jobs(int n, const float* const* partials, const float* const* factor,
                                const int* width, const int* num_partials, const int64_t* len,
                                float* const* out, void* stream) {
  return reduce_jobs(n, partials, factor, width, num_partials, len, out, nullptr, nullptr, 0,
                     stream);
}

extern "C" int lgnn_reduce_jobs_ce(int n, const float* const* partials,
                                   const float* const* factor, const int* width,
                                   const int* num_partials, const int64_t* len,
                                   float* const* out, const int* ce_job, const lgnn_ce_src* ce,
                                   int num_classes, void* stream) {
  if (!ce_job) return LGNN_EINVAL;
  return reduce_jobs(n, partials, factor, width, num_partials, len, out, ce_job, ce, num_classes,
                     stream);
}
