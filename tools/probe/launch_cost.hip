// Probe: what a graph-build launch that only reads a verdict and exits costs inside a replayed
// HIP graph, by variant (tools/launch_cost.py drives it). Not part of liblgnn.so.
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ int g_flag_word;

// v0: empty
__global__ __launch_bounds__(256) void k_empty() {}

// v1: one word through a kernarg pointer, exit when set
__global__ __launch_bounds__(256) void k_flag(const int* __restrict__ flag, int* __restrict__ out) {
  if (*flag == 1) return;
  out[blockIdx.x * 256 + threadIdx.x] = 1;
}

// v2: k_count's verdict OR: n words per workgroup, four block-wide ORs
__global__ __launch_bounds__(256) void k_or(const int* __restrict__ words, int n, int* __restrict__ out) {
  int v = 0;
  for (int i = threadIdx.x; i < n; i += 256) v |= words[i];
  const int b1 = __syncthreads_or(v & 1), b2 = __syncthreads_or(v & 2);
  const int b4 = __syncthreads_or(v & 4), b8 = __syncthreads_or(v & 8);
  if ((b1 | b2 | b4 | b8) == 0) return;
  out[blockIdx.x * 256 + threadIdx.x] = 1;
}

// v3: v1 with a large static LDS allocation
__global__ __launch_bounds__(256) void k_flag_lds(const int* __restrict__ flag, int* __restrict__ out) {
  __shared__ int big[15000];
  if (*flag == 1) return;
  big[threadIdx.x] = threadIdx.x;
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = big[255 - threadIdx.x];
}

// v4: the word from a device global (no kernarg load before it)
__global__ __launch_bounds__(256) void k_flag_global(int* __restrict__ out) {
  if (__atomic_load_n(&g_flag_word, __ATOMIC_RELAXED) == 1) return;
  out[blockIdx.x * 256 + threadIdx.x] = 1;
}

// writer: sets the flag words (kernarg target and the global)
__global__ void k_set(int* flag, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *flag = v;
    g_flag_word = v;
  }
}

extern "C" int probe_launch(int variant, int grid, const int* flag, int* out, int n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s); break;
    case 1: hipLaunchKernelGGL(k_flag, dim3(grid), dim3(256), 0, s, flag, out); break;
    case 2: hipLaunchKernelGGL(k_or, dim3(grid), dim3(256), 0, s, flag, n, out); break;
    case 3: hipLaunchKernelGGL(k_flag_lds, dim3(grid), dim3(256), 0, s, flag, out); break;
    case 4: hipLaunchKernelGGL(k_flag_global, dim3(grid), dim3(256), 0, s, out); break;
    case 9: hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, s, (int*)flag, n); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}
