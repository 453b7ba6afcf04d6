// Dropout masks from a counter-based generator, and the elementwise mask product.
//
// Replaces the Bernoulli draws of torch's dropout on the hot path: nn.Dropout between GIN convs
// (reference src/lesion_gnn/models/gin.py:27,32), the dropout inside PyG's MLP after each
// BatchNorm + ELU (gin.py:23) and GATConv's attention dropout (gat.py:31, PyG 2.5.1
// `F.dropout(alpha, p)`). torch draws them from its Philox generator inside each dropout kernel;
// here every mask of a model's forward comes out of ONE launch, as fp32 multipliers
// (0 or 1 / (1 - p), the value the consuming kernels multiply by), from a generator whose output
// is a pure function of (seed, counter, stream, element) — so the CPU oracle regenerates the
// exact same masks (oracle/pyg_ref.py DropoutMasks) and parity holds with dropout ON.
//
// Generator (splitmix64 finalizer as the mixing function, G = 0x9E3779B97F4A7C15):
//   key      = mix(seed ^ (counter * G))
//   u(s, i)  = mix(key + s * 0xD1B54A32D192ED03 + i * G) >> 40      (24 uniform bits)
//   mask[i]  = u >= thr ? scale : 0,   thr = (uint32)(p * 2^24),  scale = fp32(1 / (1 - p))
// s = the job's stream id, i = the element index within the job's mask.
//
// State (device, uint64[8]): [seed, counter, 9 ticket words (32-bit), 0...]. Every workgroup reads
// the seed and counter; with `advance` the last workgroup to finish (last_workgroup: a two-level
// ticket) increments the counter, so a captured HIP graph draws fresh masks on every replay
// (torch's generator does the same for captured dropout).
#include "common.h"

namespace {

constexpr int kT = 256;
constexpr int64_t kMaxBlocks = 512;
constexpr uint64_t kGold = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kStream = 0xD1B54A32D192ED03ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct MaskJobs {
  float* out[LGNN_MAX_MASKS];
  int64_t n[LGNN_MAX_MASKS];
  uint32_t thr[LGNN_MAX_MASKS];
  float scale[LGNN_MAX_MASKS];
  int boff[LGNN_MAX_MASKS + 1];  // prefix of the workgroups per job
  int nj;
};

// 4 consecutive elements per thread, one 16-B store (each job's mask is a separate allocation,
// 16-B aligned); workgroups in proportion to each job's size.
__global__ __launch_bounds__(kT) void k_masks(MaskJobs J, uint64_t* __restrict__ state,
                                              int advance) {
  const uint64_t seed = state[0], ctr = state[1];
  const uint64_t key = mix64(seed ^ (ctr * kGold));
  int j = 0;
  while (j + 1 < J.nj && J.boff[j + 1] <= (int)blockIdx.x) ++j;
  const int lb = (int)blockIdx.x - J.boff[j], nb = J.boff[j + 1] - J.boff[j];
  const int64_t n = J.n[j];
  float* __restrict__ out = J.out[j];
  const uint32_t thr = J.thr[j];
  const float scale = J.scale[j];
  const uint64_t base = key + (uint64_t)j * kStream;
  for (int64_t i0 = ((int64_t)lb * kT + threadIdx.x) * 4; i0 < n; i0 += (int64_t)nb * kT * 4) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t u = (uint32_t)(mix64(base + (uint64_t)(i0 + e) * kGold) >> 40);
      v[e] = u >= thr ? scale : 0.f;
    }
    if (i0 + 4 <= n) {
      f32x4 q = {v[0], v[1], v[2], v[3]};
      st4(out + i0, q);
    } else {
      for (int e = 0; i0 + e < n; ++e) out[i0 + e] = v[e];
    }
  }
  if (!advance) return;
  __syncthreads();
  // the ticket's operand depends on the counter read, so that read has returned before this
  // workgroup's ticket is taken (the last arrival then overwrites the counter safely)
  const unsigned int inc = ticket_after((unsigned int)ctr ^ (unsigned int)(ctr >> 32));
  if (threadIdx.x == 0 && last_workgroup(reinterpret_cast<unsigned int*>(state + 2), inc)) {
    state[1] = ctr + 1;
    __threadfence();
  }
}

__global__ __launch_bounds__(kT) void k_mask_mul(const float* __restrict__ x,
                                                 const float* __restrict__ m,
                                                 float* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kT * 4;
  for (int64_t i = ((int64_t)blockIdx.x * kT + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      st4(y + i, ld4(x + i) * ld4(m + i));
    } else {
      for (int64_t k = i; k < n; ++k) y[k] = x[k] * m[k];
    }
  }
}

// dZ = dY * act'(H) from the activation's saved output (ELU: 1 above 0, H + 1 below)
__global__ __launch_bounds__(kT) void k_act_bwd(const float* __restrict__ dy,
                                                const float* __restrict__ h,
                                                float* __restrict__ dz, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kT * 4;
  for (int64_t i = ((int64_t)blockIdx.x * kT + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      const f32x4 g = ld4(dy + i), hv = ld4(h + i);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = g[j] * elu_grad_from_out(hv[j]);
      st4(dz + i, o);
    } else {
      for (int64_t k = i; k < n; ++k) dz[k] = dy[k] * elu_grad_from_out(h[k]);
    }
  }
}

}  // namespace

extern "C" int lgnn_act_bwd(const float* dy, const float* h, float* dz, int64_t n, int act,
                            void* stream) {
  if (n < 0 || act != LGNN_ACT_ELU || (n > 0 && (!dy || !h || !dz))) return LGNN_EINVAL;
  if (((uintptr_t)dy | (uintptr_t)h | (uintptr_t)dz) % 16) return LGNN_EINVAL;
  if (n == 0) return LGNN_OK;
  int64_t nb = (n + 4 * kT - 1) / (4 * kT);
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(k_act_bwd, dim3((unsigned)nb), dim3(kT), 0, as_stream(stream), dy, h, dz, n);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_dropout_masks(int num_masks, float* const* out, const int64_t* numel,
                                  const uint32_t* thr, const float* scale, uint64_t* state,
                                  int advance, void* stream) {
  if (num_masks < 1 || num_masks > LGNN_MAX_MASKS || !out || !numel || !thr || !scale || !state)
    return LGNN_EINVAL;
  MaskJobs J = {};
  J.nj = num_masks;
  J.boff[0] = 0;
  int64_t total = 0;
  for (int i = 0; i < num_masks; ++i) total += numel[i] > 0 ? numel[i] : 0;
  // elements per workgroup: at least 4 per thread, and few enough workgroups (<= ~512 + jobs)
  // that the ticket atomics (last_workgroup: ~64 per word) stay cheap (they serialise in L2)
  int64_t per = (total + kMaxBlocks - 1) / kMaxBlocks;
  per = (per + 4 * kT - 1) / (4 * kT) * (4 * kT);
  if (per < 4 * kT) per = 4 * kT;
  for (int i = 0; i < num_masks; ++i) {
    if (numel[i] < 0 || (numel[i] > 0 && !out[i]) || thr[i] > (1u << 24)) return LGNN_EINVAL;
    if (reinterpret_cast<uintptr_t>(out[i]) % 16) return LGNN_EINVAL;
    J.out[i] = out[i];
    J.n[i] = numel[i];
    J.thr[i] = thr[i];
    J.scale[i] = scale[i];
    const int64_t nb = (numel[i] + per - 1) / per;
    J.boff[i + 1] = J.boff[i] + (int)(nb > 0 ? nb : 1);
  }
  hipLaunchKernelGGL(k_masks, dim3((unsigned)J.boff[num_masks]), dim3(kT), 0, as_stream(stream), J,
                     state, advance);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_mask_mul(const float* x, const float* mask, float* y, int64_t n,
                             void* stream) {
  if (n < 0 || (n > 0 && (!x || !mask || !y))) return LGNN_EINVAL;
  if (((uintptr_t)x | (uintptr_t)mask | (uintptr_t)y) % 16) return LGNN_EINVAL;
  if (n == 0) return LGNN_OK;
  int64_t nb = (n + 4 * kT - 1) / (4 * kT);
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(k_mask_mul, dim3((unsigned)nb), dim3(kT), 0, as_stream(stream), x, mask, y,
                     n);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
