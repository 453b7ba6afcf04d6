// Fused Adam / AdamW step over a list of fp32 tensors in ONE launch (torch.optim.Adam /
// AdamW semantics, amsgrad = False). Replaces the optimizer step of the reference's training
// loop (models/base.py:162-188 configure_optimizers -> torch.optim.Adam/AdamW), which torch
// runs as multi_tensor_apply launches plus a separate step-count update.
//
// Per element (t = step + 1, bc1 = 1 - beta1^t, bc2 = 1 - beta2^t):
//   g = grad (negated if maximize); Adam: g += wd * p;  AdamW: p *= 1 - lr * wd
//   m = beta1 m + (1 - beta1) g;  v = beta2 v + (1 - beta2) g^2
//   p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
// The step count lives on the device (graph-capturable): every workgroup reads it, the last one
// to finish (ticket counter) increments it and re-arms the ticket (advance = 1; a group of
// more than LGNN_MAX_ADAM (16) tensors is stepped in several launches, the last one advancing).
#include "common.h"

namespace {

constexpr int kT = 256;

struct AdamJobs {
  float* p[LGNN_MAX_ADAM];
  const float* g[LGNN_MAX_ADAM];
  float* m[LGNN_MAX_ADAM];
  float* v[LGNN_MAX_ADAM];
  int64_t off[LGNN_MAX_ADAM + 1];  // prefix of the element counts
  int boff[LGNN_MAX_ADAM + 1];     // prefix of the workgroups per tensor
  int n;
};

constexpr int kE = 2;  // elements per thread: workgroups in proportion to each tensor's size

// 1-D grid: workgroup b takes tensor j with boff[j] <= b < boff[j + 1] (uniform: its pointers are
// scalar loads) and strides that tensor's elements with the tensor's other workgroups
__global__ __launch_bounds__(kT) void k_adam(AdamJobs J, float* __restrict__ step,
                                             unsigned int* __restrict__ ticket, float lr,
                                             float beta1, float beta2, float eps, float wd,
                                             int decoupled, int maximize, int advance) {
  const float t = step[0] + 1.f;
  const float bc1 = 1.f - powf(beta1, t);
  const float bc2s = sqrtf(1.f - powf(beta2, t));
  const float step_size = lr / bc1;
  int j = 0;
  while (j + 1 < J.n && J.boff[j + 1] <= (int)blockIdx.x) ++j;
  const int lb = (int)blockIdx.x - J.boff[j], nb = J.boff[j + 1] - J.boff[j];
  const int64_t n = J.off[j + 1] - J.off[j];
  float* __restrict__ P = J.p[j];
  const float* __restrict__ G = J.g[j];
  float* __restrict__ Mv = J.m[j];
  float* __restrict__ Vv = J.v[j];
#pragma unroll 2
  for (int64_t k = (int64_t)lb * kT + threadIdx.x; k < n; k += (int64_t)nb * kT) {
    float p = P[k];
    float g = G[k];
    if (maximize) g = -g;
    if (decoupled) p *= 1.f - lr * wd;
    else g = fmaf(wd, p, g);
    const float m = fmaf(beta1, Mv[k], (1.f - beta1) * g);
    const float v = fmaf(beta2, Vv[k], (1.f - beta2) * g * g);
    Mv[k] = m;
    Vv[k] = v;
    p -= step_size * m / (sqrtf(v) / bc2s + eps);
    P[k] = p;
  }
  if (!advance) return;
  __syncthreads();
  // The last workgroup to arrive advances the step. No release fence before the ticket: the only
  // cross-workgroup hazard is step[0] (read at the top, written by the last arrival), and every
  // workgroup's read of it has returned before its ticket is taken (see `inc` below). A
  // device-scope fence here wrote back each XCD's dirty L2 (the parameters and moments this
  // kernel just updated) once per workgroup.
  // The ticket's operand depends on t, so this workgroup's read of step[0] has returned before
  // its ticket is taken even when its loop ran no iteration (a numel-0 tensor).
  const unsigned int inc = ticket_after(__float_as_uint(t));
  if (threadIdx.x == 0 && last_workgroup(ticket, inc)) {
    step[0] = t;
    __threadfence();
  }
}

}  // namespace

static int adam_step(int n, float* const* params, const float* const* grads,
                     float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numels,
                     float* step, unsigned int* ticket, float lr, float beta1, float beta2,
                     float eps, float weight_decay, int decoupled, int maximize, int advance,
                     void* stream) {
  if (n < 0 || n > LGNN_MAX_ADAM || !step || !ticket || (n > 0 && (!params || !grads ||
      !exp_avg || !exp_avg_sq || !numels)))
    return LGNN_EINVAL;
  AdamJobs J = {};
  J.n = n;
  J.off[0] = 0;
  J.boff[0] = 0;
  // elements per workgroup: kE per thread, more when the tensors are large, so the grid stays
  // within ~512 workgroups (+ one per tensor): the step ticket (last_workgroup, two levels) is
  // one same-address atomic per workgroup on its group's word, and those serialise in L2 (C3:
  // 1.8k workgroups on one word cost ~8 us of tickets)
  int64_t total = 0;
  for (int i = 0; i < n; ++i) total += numels[i] > 0 ? numels[i] : 0;
  int64_t per = (total + 511) / 512;
  per = (per + kE * kT - 1) / (kE * kT) * (kE * kT);
  if (per < kE * kT) per = kE * kT;
  for (int i = 0; i < n; ++i) {
    if (numels[i] < 0 || (numels[i] > 0 && (!params[i] || !grads[i] || !exp_avg[i] ||
        !exp_avg_sq[i])))
      return LGNN_EINVAL;
    J.p[i] = params[i];
    J.g[i] = grads[i];
    J.m[i] = exp_avg[i];
    J.v[i] = exp_avg_sq[i];
    J.off[i + 1] = J.off[i] + numels[i];
    const int64_t nb = (numels[i] + per - 1) / per;
    J.boff[i + 1] = J.boff[i] + (int)(nb > 0 ? nb : 1);
  }
  if (n == 0) J.boff[1] = 1;
  hipLaunchKernelGGL(k_adam, dim3((unsigned)J.boff[n > 0 ? n : 1]), dim3(kT), 0,
                     as_stream(stream), J, step, ticket, lr, beta1, beta2, eps, weight_decay,
                     decoupled, maximize, advance);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_adam_step(int n, float* const* params, const float* const* grads,
                              float* const* exp_avg, float* const* exp_avg_sq,
                              const int64_t* numels, float* step, unsigned int* ticket, float lr,
                              float beta1, float beta2, float eps, float weight_decay,
                              int decoupled, int maximize, int advance, void* stream) {
  return adam_step(n, params, grads, exp_avg, exp_avg_sq, numels, step, ticket, lr, beta1, beta2,
                   eps, weight_decay, decoupled, maximize, advance, stream);
}
