// Lesion-node feature pooling: per-connected-component mean / max of a channel-major feature map.
// Reference: src/lesion_gnn/datasets/nodes/lesions.py:88-93 (extract_features_by_cc, called at
// :172 with reduce = FeaturesReduction, :62-64): features (1, C, H, W) -> (H*W, C) view ->
// torch_scatter scatter(features, cc.flatten(), 0, reduce) -> [max(cc) + 1, C]. With the reference
// config (configs/config.py:15, reinterpolation=(512, 512)) one image is C = 1025 channels x 262,144
// pixels = 1.07 GB of fp32, read once: HBM-bound.
//
// Layout: the feature map stays channel-major as the encoder leaves it (no transpose pass).
// k_cc_count — label histogram (LDS per workgroup, then one global atomic per touched bin;
//              integer, so order-free) and the out-of-range count.
// k_cc_pool  — one workgroup per (channel, pixel slice): lanes read consecutive pixels of the
//              channel (coalesced 256-B wave loads), each lane keeps a (label, partial) run in
//              registers and flushes it to its wave's private LDS bins only when the label changes
//              (component pixels form long runs along the raster), so LDS traffic is per run, not
//              per pixel; the wave bins are folded in fixed wave order and written as one partial
//              per slice; the last-arriving slice of a channel folds the slices in slice order and
//              divides by the count (mean). Deterministic: every float sum is in a fixed order
//              except within one wave's LDS add instruction, whose lane order the hardware fixes.
#include "common.h"

namespace lgnn_ccpool {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxSeg = 4032;        // 4 wave-private bin arrays (< 64 KB of LDS)
constexpr int64_t kSlicePix = 65536; // pixels per workgroup slice

__device__ __forceinline__ int32_t f2ord(float f) {
  const int32_t i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int32_t i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

__global__ void __launch_bounds__(kThreads)
    k_cc_count(const int64_t* __restrict__ cc, int64_t npix, int nseg, int32_t* __restrict__ count,
               int16_t* __restrict__ lab, int32_t* __restrict__ err) {
  extern __shared__ int32_t hist[];
  for (int i = threadIdx.x; i < nseg; i += kThreads) hist[i] = 0;
  __syncthreads();
  int bad = 0;
  const int64_t per = (npix + gridDim.x - 1) / gridDim.x;
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = min(npix, p0 + per);
  for (int64_t p = p0 + threadIdx.x; p < p1; p += kThreads) {
    const int64_t l = cc[p];
    if (l < 0 || l >= nseg) {
      ++bad;
      lab[p] = -1;
      continue;
    }
    lab[p] = (int16_t)l;
    atomicAdd(&hist[l], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nseg; i += kThreads)
    if (hist[i]) atomicAdd(&count[i], hist[i]);
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(err, bad);
}

template <bool kMax>
__global__ void __launch_bounds__(kThreads)
    k_cc_pool(const float* __restrict__ feat, const int16_t* __restrict__ lab, int64_t npix,
              int C, int nseg, int nslice, const int32_t* __restrict__ count,
              float* __restrict__ part, int32_t* __restrict__ arrive, float* __restrict__ out) {
  extern __shared__ float bins[];  // [kWaves][nseg]
  __shared__ int last;
  const int c = blockIdx.x / nslice;
  const int s = blockIdx.x - c * nslice;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float init = kMax ? -__builtin_inff() : 0.f;
  for (int i = threadIdx.x; i < kWaves * nseg; i += kThreads) {
    if (kMax)  // order-preserving ints for the integer LDS max
      reinterpret_cast<int32_t*>(bins)[i] = f2ord(init);
    else
      bins[i] = 0.f;
  }
  __syncthreads();

  float* wb = bins + wave * nseg;
  const float* f = feat + (int64_t)c * npix;
  const int64_t p0 = (int64_t)s * kSlicePix;
  const int64_t p1 = min(npix, p0 + kSlicePix);
  int cur = -1;
  float acc = init;
  auto flush = [&]() {
    if (cur < 0) return;
    if (kMax)
      atomicMax(reinterpret_cast<int32_t*>(&wb[cur]), f2ord(acc));
    else
      atomicAdd(&wb[cur], acc);
  };
  for (int64_t p = p0 + wave * 64 + lane; p < p1; p += kThreads) {
    const int l = lab[p];
    if (l < 0) continue;
    const float v = f[p];
    if (l != cur) {
      flush();
      cur = l;
      acc = v;
    } else {
      acc = kMax ? fmaxf(acc, v) : acc + v;
    }
  }
  flush();
  __syncthreads();

  // fold the wave bins in wave order -> this slice's partial [nseg] for channel c
  float* pc = part + ((int64_t)c * nslice + s) * nseg;
  for (int i = threadIdx.x; i < nseg; i += kThreads) {
    float r;
    if (kMax) {
      int32_t m = reinterpret_cast<int32_t*>(bins)[i];
      for (int w = 1; w < kWaves; ++w) m = max(m, reinterpret_cast<int32_t*>(bins)[w * nseg + i]);
      r = ord2f(m);
    } else {
      r = bins[i];
      for (int w = 1; w < kWaves; ++w) r += bins[w * nseg + i];
    }
    if (nslice == 1) {
      if (kMax)
        r = count[i] > 0 ? r : 0.f;
      else
        r = r / (float)max(count[i], 1);
      out[(int64_t)i * C + c] = r;
    } else {
      pc[i] = r;
    }
  }
  if (nslice == 1) return;

  // last slice of channel c to arrive folds the slices in slice order
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&arrive[c], 1) == nslice - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  const float* pcs = part + (int64_t)c * nslice * nseg;
  for (int i = threadIdx.x; i < nseg; i += kThreads) {
    float r = __builtin_nontemporal_load(&pcs[i]);
    for (int t = 1; t < nslice; ++t) {
      const float v = __builtin_nontemporal_load(&pcs[(int64_t)t * nseg + i]);
      r = kMax ? fmaxf(r, v) : r + v;
    }
    if (kMax)
      r = count[i] > 0 ? r : 0.f;
    else
      r = r / (float)max(count[i], 1);
    out[(int64_t)i * C + c] = r;
  }
  if (threadIdx.x == 0) arrive[c] = 0;  // re-armed for the next call (graph replay)
}

}  // namespace lgnn_ccpool

using namespace lgnn_ccpool;

static int cc_nslice(int64_t npix) { return (int)std::max<int64_t>(1, (npix + kSlicePix - 1) / kSlicePix); }

extern "C" size_t lgnn_cc_pool_workspace_bytes(int64_t num_pixels, int channels, int num_segments) {
  const int ns = cc_nslice(num_pixels);
  size_t b = (size_t)num_segments * sizeof(int32_t) + 64;              // counts
  b += (size_t)num_pixels * sizeof(int16_t) + 64;                        // compact labels
  b += (size_t)channels * sizeof(int32_t) + 64;                          // arrival counters
  if (ns > 1) b += (size_t)channels * ns * num_segments * sizeof(float);  // slice partials
  return b;
}

extern "C" int lgnn_cc_pool(const float* features, int channels, int64_t num_pixels,
                            const int64_t* cc, int num_segments, int reduce_max, float* out,
                            int32_t* counts_out, int32_t* err, void* workspace,
                            size_t workspace_bytes, void* stream) {
  if (channels <= 0 || num_pixels < 0 || num_segments <= 0 || num_segments > kMaxSeg)
    return LGNN_EINVAL;
  if (!features || !cc || !out || !err || !workspace ||
      workspace_bytes < lgnn_cc_pool_workspace_bytes(num_pixels, channels, num_segments))
    return LGNN_EINVAL;
  hipStream_t s = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  int32_t* count = counts_out ? counts_out : reinterpret_cast<int32_t*>(ws);
  ws += (size_t)num_segments * sizeof(int32_t) + 64;
  int16_t* lab = reinterpret_cast<int16_t*>(ws);
  ws += ((size_t)num_pixels * sizeof(int16_t) + 64) & ~(size_t)63;
  int32_t* arrive = reinterpret_cast<int32_t*>(ws);
  ws += (size_t)channels * sizeof(int32_t) + 64;
  float* part = reinterpret_cast<float*>(ws);
  const int ns = cc_nslice(num_pixels);
  hipError_t e = hipMemsetAsync(count, 0, (size_t)num_segments * sizeof(int32_t), s);
  if (e == hipSuccess) e = hipMemsetAsync(err, 0, sizeof(int32_t), s);
  if (e == hipSuccess && ns > 1) e = hipMemsetAsync(arrive, 0, (size_t)channels * sizeof(int32_t), s);
  if (e != hipSuccess) return (int)e;
  const int cblocks = (int)std::min<int64_t>(1024, std::max<int64_t>(1, num_pixels / 4096));
  hipLaunchKernelGGL(k_cc_count, dim3(cblocks), dim3(kThreads), num_segments * sizeof(int32_t), s,
                     cc, num_pixels, num_segments, count, lab, err);
  LGNN_LAUNCH_CHECK();
  const size_t lds = (size_t)kWaves * num_segments * sizeof(float);
  const dim3 grid((unsigned)((int64_t)channels * ns));
  if (reduce_max)
    hipLaunchKernelGGL(k_cc_pool<true>, grid, dim3(kThreads), lds, s, features, lab, num_pixels,
                       channels, num_segments, ns, count, part, arrive, out);
  else
    hipLaunchKernelGGL(k_cc_pool<false>, grid, dim3(kThreads), lds, s, features, lab, num_pixels,
                       channels, num_segments, ns, count, part, arrive, out);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
