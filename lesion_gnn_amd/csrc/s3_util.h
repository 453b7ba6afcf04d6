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
