// Shared helpers for the gfx950 kernels of liblgnn.so. CDNA4 only: wave64, MFMA f32 32x32x2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lgnn.h"

#define LGNN_MAX_STACK 8  // layers of one fused stack launch (in_proj + 7 convs)
#define LGNN_MAX_REDUCE 16  // slabs of one lgnn_reduce_partials_multi launch

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define LGNN_LAUNCH_CHECK()                         \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return (int)_e;           \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// PyTorch ELU(alpha=1): x > 0 ? x : expm1(x)
__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }
// ELU derivative from the saved OUTPUT h = elu(z): z > 0 <=> h > 0; exp(z) = h + 1.
__device__ __forceinline__ float elu_grad_from_out(float h) { return h > 0.f ? 1.f : h + 1.f; }

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
