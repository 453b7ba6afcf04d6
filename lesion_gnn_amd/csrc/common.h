// Shared helpers for the gfx950 kernels of liblgnn.so. CDNA4 only: wave64, MFMA f32 32x32x2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lgnn.h"

#define LGNN_MAX_STACK 8  // layers of one fused stack launch (in_proj + 7 convs)
#define LGNN_MAX_REDUCE 16  // slabs of one lgnn_reduce_partials_multi launch
#define LGNN_MAX_ADAM 16    // tensors of one lgnn_adam_step launch

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define LGNN_LAUNCH_CHECK()                         \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return (int)_e;           \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// the process-wide path options of lgnn_set_option (include/lgnn.h; defined in graph.hip)
int lgnn_option(int option);

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// PyTorch ELU(alpha=1): x > 0 ? x : expm1(x). Branch-free: expm1 is evaluated unconditionally
// on min(x, 0), so a run of them interleaves instead of each sitting behind an exec-mask branch.
#ifdef LGNN_FAST_ELU
// expm1 on x <= 0 in ~14 instructions: Taylor to x^8 on [-0.5, 0] (truncation < 1e-8 relative),
// exp2 (v_exp_f32) - 1 below (no cancellation there: the result is <= -0.39).
__device__ __forceinline__ float expm1_neg(float x) {
  float q = 1.f / 40320.f;
  q = fmaf(q, x, 1.f / 5040.f);
  q = fmaf(q, x, 1.f / 720.f);
  q = fmaf(q, x, 1.f / 120.f);
  q = fmaf(q, x, 1.f / 24.f);
  q = fmaf(q, x, 1.f / 6.f);
  q = fmaf(q, x, 0.5f);
  const float p = fmaf(q, x * x, x);
  const float e = __builtin_amdgcn_exp2f(x * 1.44269504088896341f) - 1.f;
  return x > -0.5f ? p : e;
}
__device__ __forceinline__ float elu_f(float x) {
  const float e = expm1_neg(fminf(x, 0.f));
  return x > 0.f ? x : e;
}
#else
__device__ __forceinline__ float elu_f(float x) {
  const float e = expm1f(fminf(x, 0.f));
  return x > 0.f ? x : e;
}
#endif
// ELU derivative from the saved OUTPUT h = elu(z): z > 0 <=> h > 0; exp(z) = h + 1.
__device__ __forceinline__ float elu_grad_from_out(float h) { return h > 0.f ? 1.f : h + 1.f; }
// Blocks are dealt round-robin over the 8 XCDs (observed placement, speed only): block b's
// position in a contiguous per-XCD run of the grid (bijective for any grid size), so the rows an
// XCD's blocks visit are one contiguous range and the neighbour rows they gather (same graph:
// adjacent rows) stay in that XCD's L2.
__device__ __forceinline__ int64_t xcd_block() {
  const int64_t nwg = gridDim.x, b = blockIdx.x;
  const int64_t q = nwg / 8, r = nwg % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// ELU'(zn) for zn = z * scale + shift (BatchNorm then ELU): 1 above 0, exp(zn) below (exp2 form)
__device__ __forceinline__ float bn_elu_grad(float z, float sc, float sh) {
  const float zn = fmaf(z, sc, sh);
  return zn > 0.f ? 1.f : __builtin_amdgcn_exp2f(zn * 1.44269504088896341f);
}

// Is this workgroup the last of the grid to get here? (thread 0 asks, after the workgroup's work.)
// A two-level ticket: workgroup b first takes a ticket on word b % 8 — its group's own word, so a
// group's same-address atomics serialise in one XCD's L2 in parallel with the others' (blocks are
// dealt round-robin over the XCDs: speed only, correct for any placement) — then each group's
// last arrival on word 8. At most ~gridDim/8 + 8 atomics meet on one word instead of gridDim.
// tk: 9 zeroed words, left zero (re-armed). inc: 1, computed by ticket_after(x) from data the
// caller read first (a dependency that orders those reads before the ticket). Returns true for
// exactly one workgroup.
__device__ __forceinline__ bool last_workgroup(unsigned int* tk, unsigned int inc) {
  const unsigned int G = gridDim.x, g = blockIdx.x & 7u;
  const unsigned int ng = (G - g + 7u) >> 3, groups = G < 8u ? G : 8u;
  if (atomicAdd(tk + g, inc) != ng - 1u) return false;
  tk[g] = 0u;
  if (atomicAdd(tk + 8, 1u) != groups - 1u) return false;
  tk[8] = 0u;
  return true;
}

// The ticket increment 1, as a value the compiler must compute after `dep` has arrived: the empty
// asm takes dep as an input and may (as far as the compiler knows) rewrite the 1, so the load
// behind dep completes before the ticket atomic that consumes the result is issued. The value is
// always 1 (round 3 used `dep-condition ? 2 : 1`, whose 2 would wedge the ticket words).
__device__ __forceinline__ unsigned int ticket_after(unsigned int dep) {
  unsigned int one = 1u;
  asm volatile("" : "+v"(one) : "v"(dep));
  return one;
}

// nn.CrossEntropyLoss(weight) (mean reduction) logits gradient, k_ce_bwd's expression:
//   dz[i][c] = gloss * wt_i / wsum * pm_ic,  wt_i = w[y_i] (0 if y_i is outside [0, C)),
//   pm_ic = exp(z[i][c] - lse[i]) - [c == y_i]
// ce_pm / ce_wt are the per-graph factors (the readout's CE forward stores them); ce_dlogit forms
// the gradient where it is consumed from plain loads of them, bit for bit k_ce_bwd's value.
__device__ __forceinline__ float ce_wt(const int64_t* y, const float* w, int C, int64_t i) {
  const int64_t t = y[i];
  return (t >= 0 && t < C) ? (w ? w[t] : 1.f) : 0.f;
}
__device__ __forceinline__ float ce_pm(float z, float lse, int64_t t, int c) {
  return expf(z - lse) - (c == t ? 1.f : 0.f);
}
__device__ __forceinline__ float ce_grad(float gloss, float wt, float wsum, float pm) {
  // rounded as a stored dlogits value is: no FMA contraction into the consumer's sum
#pragma clang fp contract(off)
  return gloss * wt / wsum * pm;
}
struct CeSrc {
  const float* pm;     // [B][C]
  const float* wt;     // [B]
  const float* wsum;   // [1]
  const float* gloss;  // [1]
  int C;
};
__device__ __forceinline__ float ce_dlogit(const CeSrc& s, int64_t i, int c) {
  return ce_grad(s.gloss[0], s.wt[i], s.wsum[0], s.pm[i * s.C + c]);
}

// Write-through (sc1) store: the line leaves the XCD's L2 as it is written (MI355X_MICROARCH.md:
// sc1 stores drop the line from L2; 16-B sc1 stores cost about what plain ones do)
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
