// MFMA issue / dependency probe (tuning aid, not part of the library): cycles per
// v_mfma_f32_32x32x16_bf16 for 1, 2, 4 independent accumulator chains, one wave per SIMD and
// two waves per SIMD. Build: hipcc --offload-arch=gfx950 -O3 mfma_probe.hip -o mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// per block: start / end (s_memrealtime, 100 MHz) and HW_ID (CU, SE, XCC) of wave 0
__device__ long long* g_rec;

template <int CH>
__global__ void k_probe(float* out, long long* cyc, int iters) {
  const long long rt0 = __builtin_amdgcn_s_memrealtime();
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(threadIdx.x * 0.001f + i);
    b[i] = (__bf16)(i * 0.5f);
  }
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x16{};
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < CH; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int c = 0; c < CH; ++c)
    for (int i = 0; i < 16; ++i) s += acc[c][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    cyc[blockIdx.x] = t1 - t0;
    const long long rt1 = __builtin_amdgcn_s_memrealtime();
    unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID all bits
    unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); // XCC_ID
    if (g_rec) {
      g_rec[blockIdx.x * 3 + 0] = rt0;
      g_rec[blockIdx.x * 3 + 1] = rt1;
      g_rec[blockIdx.x * 3 + 2] = ((long long)xcc << 32) | hw;
    }
  }
}

template <int CH>
void run(int blocks, int threads, int iters) {
  float* out;
  long long* cyc;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL(k_probe<CH>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_probe<CH>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  {
    long long* rec;
    hipMalloc(&rec, sizeof(long long) * 3 * blocks);
    hipMemcpyToSymbol(HIP_SYMBOL(g_rec), &rec, sizeof(rec));
    hipLaunchKernelGGL(k_probe<CH>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    long long* h = (long long*)malloc(sizeof(long long) * 3 * blocks);
    hipMemcpy(h, rec, sizeof(long long) * 3 * blocks, hipMemcpyDeviceToHost);
    // max number of blocks overlapping in time on one (xcc, se, cu)
    int best = 0;
    for (int i = 0; i < blocks; ++i) {
      int n = 0;
      const long long key = h[3 * i + 2] & 0xFFFFFFFF0000FF00ll;  // xcc | SE/SH/CU fields
      for (int j = 0; j < blocks; ++j)
        if ((h[3 * j + 2] & 0xFFFFFFFF0000FF00ll) == key && h[3 * j] < h[3 * i + 1] &&
            h[3 * j + 1] > h[3 * i])
          ++n;
      if (n > best) best = n;
    }
    printf("  max co-resident blocks per CU: %d\n", best);
    free(h);
    void* z = nullptr;
    hipMemcpyToSymbol(HIP_SYMBOL(g_rec), &z, sizeof(z));
    hipFree(rec);
  }
  long long c = 0;
  hipMemcpy(&c, cyc, sizeof(long long), hipMemcpyDeviceToHost);
  const double n = (double)iters * 8 * CH;  // MFMAs per wave
  const double waves = (double)blocks * threads / 64;
  const double tflops = waves * n * 32768.0 / (ms * 1e-3) / 1e12;
  printf("chains=%d blocks=%d threads=%d: %.1f clk/MFMA (wave clock), %.1f TFLOP/s, %.3f ms\n",
         CH, blocks, threads, (double)c / n, tflops, ms);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  const int it = 2000;
  run<1>(256, 256, it);
  run<2>(256, 256, it);
  run<4>(256, 256, it);
  run<1>(512, 256, it);
  run<2>(512, 256, it);
  run<4>(512, 256, it);
  run<2>(1024, 256, it);
  return 0;
}
