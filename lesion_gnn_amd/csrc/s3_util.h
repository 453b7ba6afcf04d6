// Split-3 helpers shared by the fused GCN stack kernels (stack3.hip forward, stack3_bwd.hip
// backward): bf16 plane splitting, the six-product MFMA, the perm16 feature order, LDS image
// addressing, weight-plane fragment order.
#pragma once
#include "common.h"
#include "tile_util.h"

namespace lgnn_s3 {
using namespace lgnn_tile;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int WP = 128;           // padded width of the weight planes and the H image
constexpr int PLANE = WP * WP;    // bf16 elements per weight plane
constexpr int AROW = WP * 2;      // bytes per H-image row (chunk-swizzled, no padding)
constexpr int ADJ_LD = 72;        // Â plane row stride in bf16 (144 B: conflict-free b128 rows)
constexpr int ADJ_PLANE = TM * ADJ_LD * 2;  // bytes per Â plane
// one tile's fp32 Â [target][source] as the split-3 forward hands it to the fused backward (the
// forward's LDS sum, row-major: 16 chunks of 1 KiB, one direct-to-LDS wave load each)
constexpr int ADJT_TILE_BYTES = TM * TM * 4;
static_assert(ADJT_TILE_BYTES == LGNN_S3_ADJT_TILE_BYTES && ADJT_TILE_BYTES % 1024 == 0, "");

__device__ __forceinline__ constexpr int perm16(int k) {
  return (k & ~12) | ((k & 4) << 1) | ((k & 8) >> 1);
}

// (a, b) -> three packed bf16 pairs (a in the low half), x = hi + mid + lo to 2^-24.
struct Split2 {
  uint32_t p[3];
};
__device__ __forceinline__ Split2 split2(float a, float b) {
  Split2 s;
  f32x2 v = {a, b};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint32_t q = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
    s.p[i] = q;
    if (i < 2) {
      const f32x2 back = {__uint_as_float(q << 16), __uint_as_float(q & 0xffff0000u)};
      v -= back;
    }
  }
  return s;
}

// four consecutive fp32 -> three planes of four bf16 (8 bytes each)
__device__ __forceinline__ void split4(f32x4 v, u32x2 (&o)[3]) {
  const Split2 a = split2(v[0], v[1]), b = split2(v[2], v[3]);
#pragma unroll
  for (int p = 0; p < 3; ++p) o[p] = u32x2{a.p[p], b.p[p]};
}

__device__ __forceinline__ f32x16 mfma16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// c += a.b at fp32 accuracy: the six plane products, smallest first.
__device__ __forceinline__ f32x16 mfma_s3(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
  c = mfma16(a[2], b[0], c);
  c = mfma16(a[1], b[1], c);
  c = mfma16(a[0], b[2], c);
  c = mfma16(a[1], b[0], c);
  c = mfma16(a[0], b[1], c);
  return mfma16(a[0], b[0], c);
}
// b exact in bf16 (b_mid = b_lo = 0): three products.
__device__ __forceinline__ f32x16 mfma_s3_bexact(const u32x4 (&a)[3], u32x4 b0, f32x16 c) {
  c = mfma16(a[2], b0, c);
  c = mfma16(a[1], b0, c);
  return mfma16(a[0], b0, c);
}

// a exact in bf16 (a_mid = a_lo = 0): three products.
__device__ __forceinline__ f32x16 mfma_s3_aexact(u32x4 a0, const u32x4 (&b)[3], f32x16 c) {
  c = mfma16(a0, b[2], c);
  c = mfma16(a0, b[1], c);
  return mfma16(a0, b[0], c);
}

// Byte offset of (row, 4-aligned feature k) in an H-image plane: position perm16(k), 16-B chunk
// XOR-swizzled by row & 15 so a b128 read of one chunk by 16 rows is conflict-free.
__device__ __forceinline__ int ap_off(int row, int k) {
  const int p = perm16(k);
  return row * AROW + ((((p >> 3) ^ (row & 15))) << 4) + ((p & 7) << 1);
}
__device__ __forceinline__ int ap_chunk(int row, int c) {
  return row * AROW + ((c ^ (row & 15)) << 4);
}

__device__ __forceinline__ u32x4 lds16(const unsigned char* p) {
  return *reinterpret_cast<const u32x4*>(p);
}
__device__ __forceinline__ void sts8(unsigned char* p, u32x2 v) {
  *reinterpret_cast<u32x2*>(p) = v;
}

// element index of (row, phys position) within one fragment-ordered 128 x 128 plane
__device__ __forceinline__ int frag_index(int row, int phys) {
  return ((((row >> 5) * 8 + (phys >> 4)) * 2 + ((phys >> 3) & 1)) * 32 + (row & 31)) * 8 +
         (phys & 7);
}

// Weight planes: W_l [N][K] fp32 -> bf16 planes of W_l[n][perm16(k)], zero-padded to 128 x 128,
// stored in MFMA fragment order so that one wave's load of a k-step fragment is 1 KiB contiguous:
//   Wp[l][plane][n / 32][s][h][n % 32][8]  holds  phys positions 16 s + 8 h .. + 7 of row n
// (lane h * 32 + n % 32 of wave n / 32 loads k-step s with one 16-B load). With WpT also the
// transposed planes (rows k, positions perm16(n)) in the same order: the backward's dH = G W_l
// operand. Item i = one (layer, n, 4 consecutive k); nl * PLANE_ITEMS items in all. Run by
// k_wplanes (stack3.hip) or as side work of the graph build's first launch (graph.hip).
struct PlaneArgs {
  const float* W[LGNN_MAX_STACK];
  int N[LGNN_MAX_STACK];
  int K[LGNN_MAX_STACK];
  int nl;
  uint16_t* Wp;
  uint16_t* WpT;  // nullable
};
constexpr int PLANE_ITEMS = WP * WP / 4;  // items per layer
static_assert(LGNN_PLANE_JOB_MAX == LGNN_MAX_STACK, "plane job layers");

__device__ __forceinline__ void wplanes_item(const PlaneArgs& a, int i) {
  const int l = i / PLANE_ITEMS;
  if (l >= a.nl) return;
  const int n = (i / (WP / 4)) % WP, k = 4 * (i % (WP / 4));
  const int N = a.N[l], K = a.K[l];
  const f32x4 v = (n < N && k < K) ? ld4(a.W[l] + (int64_t)n * K + k) : zero4();
  u32x2 o[3];
  split4(v, o);
  uint16_t* base = a.Wp + (size_t)l * 3 * PLANE;
#pragma unroll
  for (int p = 0; p < 3; ++p)
    *reinterpret_cast<u32x2*>(base + p * PLANE + frag_index(n, perm16(k))) = o[p];
  if (a.WpT) {
    uint16_t* bt = a.WpT + (size_t)l * 3 * PLANE;
    const int pn = perm16(n);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      bt[p * PLANE + frag_index(k + 0, pn)] = (uint16_t)(o[p][0] & 0xffffu);
      bt[p * PLANE + frag_index(k + 1, pn)] = (uint16_t)(o[p][0] >> 16);
      bt[p * PLANE + frag_index(k + 2, pn)] = (uint16_t)(o[p][1] & 0xffffu);
      bt[p * PLANE + frag_index(k + 3, pn)] = (uint16_t)(o[p][1] >> 16);
    }
  }
}

// host: the plane job of lgnn_weight_planes' arguments (LGNN_EINVAL on a bad shape)
inline int plane_args(int nl, const float* const* W, const int* widths, uint16_t* planes,
                      uint16_t* planes_t, PlaneArgs& a) {
  if (nl < 1 || nl > LGNN_MAX_STACK || !W || !widths || !planes) return LGNN_EINVAL;
  a = PlaneArgs{};
  for (int l = 0; l < nl; ++l) {
    const int K = widths[l], N = widths[l + 1];
    if (!W[l] || K < 4 || N < 4 || K > WP || N > WP || K % 4 || N % 4) return LGNN_EINVAL;
    a.W[l] = W[l];
    a.N[l] = N;
    a.K[l] = K;
  }
  a.nl = nl;
  a.Wp = planes;
  a.WpT = planes_t;
  return LGNN_OK;
}

// threadIdx.x through an empty asm: addresses derived from it cannot be hoisted out of the tile
// loop or merged across phases (held over the whole loop they cost ~60 registers); each phase
// recomputes its own in a few VALU ops.
__device__ __forceinline__ int fresh_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// ELU(alpha = 1) as exp2-based exp(min(x, 0)) - 1: five VALU ops. Against PyTorch's expm1 form
// the absolute difference is below 1e-7 (v_exp_f32 is ~1 ulp; the argument's rounding moves
// exp(x) by at most |x| e^x 2^-24 ln 2 <= 2.3e-8), i.e. fp32 rounding level for |ELU| <= 1.
__device__ __forceinline__ float elu_s3(float x) {
  const float e = __builtin_amdgcn_exp2f(fminf(x, 0.f) * 1.44269504088896341f) - 1.f;
  return x > 0.f ? x : e;
}

}  // namespace lgnn_s3
