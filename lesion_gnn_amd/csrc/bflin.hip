// bf16 dense GEMMs of the bf16 configuration (BASELINE C3: GAT with bf16 GEMM operands, fp32
// accumulation and fp32 activations) on hand-written gfx950 MFMA (v_mfma_f32_32x32x16_bf16):
//   lgnn_bf16_gemm   Y[M][N] = A[M][K] W[N][K]^T (+ b), N <= 128: the reference's in_proj
//                    (nn.Linear(1025, 128), gat.py:29) and every GATConv.lin (gat.py:31) forward,
//                    and dX = dY W of the lin backward (A = dY, W^T as the weight operand)
//   lgnn_bf16_wgrad  dW[N][K] = dY^T X as fixed-order partial slabs over row splits
//   lgnn_bf16_weight_prep  W fp32 -> the kernels' bf16 weight operands (W and W^T, zero-padded)
// Operands are rounded to bf16 round-to-nearest-even exactly as torch's .to(torch.bfloat16)
// (v_cvt_pk_bf16_f32): an fp32 A (the 1025-wide node features) is rounded as it is loaded, so
// the model needs no bf16 copy of it; a bf16 A is the copy the producing kernel wrote.
//
// Layouts (256 threads = 4 waves; 64-row tiles TM; k in chunks of 64 = four MFMA k-steps):
//   LDS images  bf16 [row][64], 128-B rows, 16-B chunk c at position c ^ (row & 7)
//   gemm        wave w owns output features 32 w .. 32 w + 31; A rows from the image, W
//               fragments straight from L2 (16 B per lane per k-step); fp32 accumulators in P
//               layout (feature on the lane, rows m = 32 q + (r & 3) + 8 (r >> 2) + 4 h)
//   wgrad       dY^T [n][m] and X^T [k][m] images (transposed in registers: each lane packs 8
//               consecutive rows of one column into one 16-B LDS write); wave w owns dW rows
//               32 w .. + 31, the 64 k of its k-block on the lane
// Both kernels double-buffer the image: chunk c + 1's global loads are in flight while chunk c's
// MFMAs run. Blocks map to tiles XCD-contiguously (xcd_block).
#include <algorithm>

#include "common.h"
#include "tile_util.h"

namespace lgnn_bf {
using namespace lgnn_tile;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int BK = 64;          // k per chunk
constexpr int ROWB = BK * 2;    // bytes per image row
constexpr int OOB = 0x7ff00000;  // buffer offset past every range: the load returns 0

__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}
__device__ __forceinline__ int swz(int row, int chunk) {
  return row * ROWB + ((chunk ^ (row & 7)) << 4);
}
__device__ __forceinline__ u32x4 lds16(const unsigned char* p) {
  return *reinterpret_cast<const u32x4*>(p);
}
__device__ __forceinline__ f32x16 mfma_bf(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ uint32_t ldb32(Buf b, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(b, off, 0, 0);
}

// ------------------------------------------------------------------------------------------
// Y = A W^T (+ b)
// ------------------------------------------------------------------------------------------
// A-chunk registers: rows 16 wave + 4 i + (lane >> 4) (i < 4), k = 4 (lane & 15) + 0..3
template <bool AF32>
struct ARegs {
  uint32_t v[AF32 ? 16 : 8];
};

// AF32 && VEC: K % 4 == 0 (one 16-B load per row); AF32 && !VEC: any K (four 4-B loads);
// bf16 A: K % 4 == 0 (one 8-B load per row)
template <bool AF32, bool VEC>
__device__ __forceinline__ void gemm_load_a(ARegs<AF32>& R, Buf bA, int K, int c, int rq, int kq) {
  const int k = c * BK + kq;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = rq + 4 * i;
    if constexpr (AF32 && VEC) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(bA, k < K ? (row * K + k) * 4 : OOB,
                                                            0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) R.v[4 * i + j] = v[j];
    } else if constexpr (AF32) {
#pragma unroll
      for (int j = 0; j < 4; ++j) R.v[4 * i + j] = ldb32(bA, k + j < K ? (row * K + k + j) * 4 : OOB);
    } else {
      const u32x2 v = __builtin_bit_cast(
          u32x2, __builtin_amdgcn_raw_buffer_load_b64(bA, k < K ? (row * K + k) * 2 : OOB, 0, 0));
      R.v[2 * i] = v[0];
      R.v[2 * i + 1] = v[1];
    }
  }
}

template <bool AF32>
__device__ __forceinline__ void gemm_store_a(unsigned char* img, const ARegs<AF32>& R, int rq,
                                             int kq) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = rq + 4 * i;
    u32x2 p;
    if constexpr (AF32) {
      p[0] = pk2(__uint_as_float(R.v[4 * i]), __uint_as_float(R.v[4 * i + 1]));
      p[1] = pk2(__uint_as_float(R.v[4 * i + 2]), __uint_as_float(R.v[4 * i + 3]));
    } else {
      p[0] = R.v[2 * i];
      p[1] = R.v[2 * i + 1];
    }
    *reinterpret_cast<u32x2*>(img + swz(row, kq >> 3) + ((kq & 7) << 1)) = p;
  }
}

// W fragments of chunk c: row 32 wave + li of the [128][Kp] bf16 operand, k 16 s + 8 h .. + 7
__device__ __forceinline__ void gemm_load_b(u32x4 (&b)[4], const uint16_t* __restrict__ Wrow,
                                            int c, int h) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
    b[s] = *reinterpret_cast<const u32x4*>(Wrow + c * BK + 16 * s + 8 * h);
}

template <bool AF32, bool VEC>
__global__ __launch_bounds__(NT) void k_bf_gemm(const void* __restrict__ A, int64_t M, int K,
                                                const uint16_t* __restrict__ Wb, int Kp,
                                                const float* __restrict__ bias, int N,
                                                float* __restrict__ Y, uint16_t* __restrict__ Yb) {
  __shared__ __attribute__((aligned(16))) unsigned char img[2][TM * ROWB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t r0 = xcd_block() * TM;
  constexpr int ESZ = AF32 ? 4 : 2;
  const Buf bA = mkbuf(static_cast<const char*>(A) + r0 * K * ESZ, (M - r0) * K * ESZ);
  const int rq = 16 * wave + (lane >> 4), kq = 4 * (lane & 15);
  const int nck = Kp / BK;
  const uint16_t* Wrow = Wb + (int64_t)(32 * wave + li) * Kp;
  f32x16 acc0 = {}, acc1 = {};
  ARegs<AF32> R;
  u32x4 b0[4], b1[4];
  gemm_load_a<AF32, VEC>(R, bA, K, 0, rq, kq);
  gemm_load_b(b0, Wrow, 0, h);
  auto step = [&](int c, const u32x4(&bc)[4], u32x4(&bn)[4]) {
    unsigned char* im = img[c & 1];
    gemm_store_a<AF32>(im, R, rq, kq);
    if (c + 1 < nck) {
      gemm_load_a<AF32, VEC>(R, bA, K, c + 1, rq, kq);
      gemm_load_b(bn, Wrow, c + 1, h);
    }
    __syncthreads();  // image c complete (and image c - 1's reads done two chunks ago)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u32x4 a0 = lds16(im + swz(li, 2 * s + h));
      const u32x4 a1 = lds16(im + swz(32 + li, 2 * s + h));
      acc0 = mfma_bf(a0, bc[s], acc0);
      acc1 = mfma_bf(a1, bc[s], acc1);
    }
  };
  for (int c = 0; c < nck; c += 2) {
    step(c, b0, b1);
    if (c + 1 < nck) step(c + 1, b1, b0);
  }
  // epilogue (P layout): + b; fp32 rows and their bf16 copy as 128-B / 64-B row segments
  const int n = 32 * wave + li;
  const bool nok = n < N;
  const float bv = (bias && nok) ? bias[n] : 0.f;
  const Buf bY = mkbuf(Y ? Y + r0 * N : nullptr, Y ? (M - r0) * N * 4 : 0);
  const Buf bYb = mkbuf(Yb ? Yb + r0 * N : nullptr, Yb ? (M - r0) * N * 2 : 0);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = (q ? acc1[r] : acc0[r]) + bv;
      const int e = m * N + n;
      if (Y) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), bY, nok ? e * 4 : OOB, 0, 0);
      if (Yb)
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(pk2(v, 0.f) & 0xffffu), bYb,
                                              nok ? e * 2 : OOB, 0, 0);
    }
}

// ------------------------------------------------------------------------------------------
// dW partial slabs: part[s][n][k] = sum over split s's row chunks of dY[m][n] X[m][k]
// ------------------------------------------------------------------------------------------
template <bool XF32>
struct WRegs {
  uint32_t x[XF32 ? 16 : 8];  // X: XF32 k = lane, rows 16 w + 8 g + j; bf16 k pair, 8 rows
  uint32_t y[16];             // dY: n pair 2 lane, rows 16 w + 8 g + j (g < 2, j < 8)
};

template <bool XF32>
__device__ __forceinline__ void wg_load(WRegs<XF32>& R, Buf bX, Buf bY, int64_t M, int K, int N,
                                        int64_t m0, int k0, int lane, int wave) {
  // every row offset below is < M * K * size (checked on the host: < 2^31)
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t m = m0 + 16 * wave + 8 * g + j;
      const bool mok = m < M;
      const int n = 2 * lane;
      R.y[8 * g + j] = ldb32(bY, mok && n < N ? (int)((m * N + n) * 2) : OOB);
      if constexpr (XF32) {
        const int k = k0 + lane;
        R.x[8 * g + j] = ldb32(bX, mok && k < K ? (int)((m * K + k) * 4) : OOB);
      }
    }
  if constexpr (!XF32) {  // lanes 0-31 rows 16 w + j, lanes 32-63 rows 16 w + 8 + j
    const int k = k0 + 2 * (lane & 31);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t m = m0 + 16 * wave + 8 * (lane >> 5) + j;
      R.x[j] = ldb32(bX, m < M && k < K ? (int)((m * K + k) * 2) : OOB);
    }
  }
}

// pack the low (HI = false) or high bf16 halves of eight u32 into one 16-B vector
template <bool HI>
__device__ __forceinline__ u32x4 pack_halves(const uint32_t* v) {
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t a = v[2 * i], b = v[2 * i + 1];
    o[i] = HI ? ((a >> 16) | (b & 0xffff0000u)) : ((a & 0xffffu) | (b << 16));
  }
  return o;
}

template <bool XF32>
__device__ __forceinline__ void wg_store(unsigned char* iy, unsigned char* ix, const WRegs<XF32>& R,
                                         int lane, int wave) {
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int ch = 2 * wave + g;  // rows 8 ch .. 8 ch + 7 of the chunk
    *reinterpret_cast<u32x4*>(iy + swz(2 * lane, ch)) = pack_halves<false>(R.y + 8 * g);
    *reinterpret_cast<u32x4*>(iy + swz(2 * lane + 1, ch)) = pack_halves<true>(R.y + 8 * g);
    if constexpr (XF32) {
      u32x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        o[i] = pk2(__uint_as_float(R.x[8 * g + 2 * i]), __uint_as_float(R.x[8 * g + 2 * i + 1]));
      *reinterpret_cast<u32x4*>(ix + swz(lane, ch)) = o;
    }
  }
  if constexpr (!XF32) {
    const int ch = 2 * wave + (lane >> 5), k = 2 * (lane & 31);
    *reinterpret_cast<u32x4*>(ix + swz(k, ch)) = pack_halves<false>(R.x);
    *reinterpret_cast<u32x4*>(ix + swz(k + 1, ch)) = pack_halves<true>(R.x);
  }
}

template <bool XF32>
__global__ __launch_bounds__(NT) void k_bf_wgrad(const uint16_t* __restrict__ dYb, int N,
                                                 const void* __restrict__ X, int64_t M, int K,
                                                 int nkb, int S, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) unsigned char iy[2][128 * ROWB];  // dY^T [n][m]
  __shared__ __attribute__((aligned(16))) unsigned char ix[2][64 * ROWB];   // X^T [k][m]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t L = xcd_block();  // blocks of one row split (adjacent k-blocks) share an XCD
  const int kb = (int)(L % nkb), s = (int)(L / nkb);
  const int k0 = kb * BK;
  const int64_t nch = (M + TM - 1) / TM;
  constexpr int ESZ = XF32 ? 4 : 2;
  const Buf bX = mkbuf(X, M * K * ESZ), bY = mkbuf(dYb, M * N * 2);
  f32x16 acc0 = {}, acc1 = {};
  WRegs<XF32> R;
  int64_t c = s;
  if (c < nch) wg_load<XF32>(R, bX, bY, M, K, N, c * TM, k0, lane, wave);
  for (int it = 0; c < nch; c += S, ++it) {
    unsigned char* py = iy[it & 1];
    unsigned char* px = ix[it & 1];
    wg_store<XF32>(py, px, R, lane, wave);
    if (c + S < nch) wg_load<XF32>(R, bX, bY, M, K, N, (c + S) * TM, k0, lane, wave);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const u32x4 a = lds16(py + swz(32 * wave + li, 2 * st + h));
      const u32x4 x0 = lds16(px + swz(li, 2 * st + h));
      const u32x4 x1 = lds16(px + swz(32 + li, 2 * st + h));
      acc0 = mfma_bf(a, x0, acc0);
      acc1 = mfma_bf(a, x1, acc1);
    }
  }
  // slab s: rows n = 32 w + (r & 3) + 8 (r >> 2) + 4 h, columns k0 + 32 kk + li
  float* slab = part + (int64_t)s * N * K;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int k = k0 + 32 * kk + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (n < N && k < K) slab[(int64_t)n * K + k] = kk ? acc1[r] : acc0[r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// weight operands: Wb [128][Kp] = bf16(W), WTb [128][Np] = bf16(W^T), zero-padded
// ------------------------------------------------------------------------------------------
__global__ void k_bf_wprep(const float* __restrict__ W, int N, int K, int Kp, int Np,
                           uint16_t* __restrict__ Wb, uint16_t* __restrict__ WTb) {
  const int64_t n1 = (int64_t)128 * Kp, n2 = WTb ? (int64_t)128 * Np : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + n2;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n1) {
      const int n = (int)(i / Kp), k = (int)(i % Kp);
      const float v = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.f;
      Wb[i] = (uint16_t)(pk2(v, 0.f) & 0xffffu);
    } else {
      const int64_t j = i - n1;
      const int k = (int)(j / Np), n = (int)(j % Np);
      const float v = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.f;
      WTb[j] = (uint16_t)(pk2(v, 0.f) & 0xffffu);
    }
  }
}

}  // namespace lgnn_bf

using namespace lgnn_bf;

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" int lgnn_bf16_kpad(int K) { return K <= 0 ? 0 : (K + BK - 1) / BK * BK; }

extern "C" int lgnn_bf16_weight_prep(const float* W, int N, int K, uint16_t* Wb, uint16_t* WTb,
                                     void* stream) {
  if (!W || !Wb || N < 1 || N > 128 || K < 1) return LGNN_EINVAL;
  if (WTb && K > 128) return LGNN_EINVAL;
  const int Kp = lgnn_bf16_kpad(K), Np = lgnn_bf16_kpad(N);
  const int64_t total = (int64_t)128 * Kp + (WTb ? (int64_t)128 * Np : 0);
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 1024);
  hipLaunchKernelGGL(k_bf_wprep, dim3(grid), dim3(256), 0, as_stream(stream), W, N, K, Kp, Np, Wb,
                     WTb);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_bf16_gemm(const void* A, int a_is_f32, int64_t M, int K, const uint16_t* Wb,
                              const float* bias, int N, float* Y, uint16_t* Yb, void* stream) {
  if (M < 0 || K < 1 || N < 1 || N > 128 || !Wb || (!Y && !Yb)) return LGNN_EINVAL;
  if (M > 0 && !A) return LGNN_EINVAL;
  if (!a_is_f32 && K % 4 != 0) return LGNN_EINVAL;
  if (M * (int64_t)K * 4 >= ((int64_t)1 << 31) || M * (int64_t)N * 4 >= ((int64_t)1 << 31))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  const int Kp = lgnn_bf16_kpad(K);
  const dim3 grid((unsigned)((M + TM - 1) / TM)), block(NT);
  hipStream_t s = as_stream(stream);
  if (!a_is_f32)
    hipLaunchKernelGGL((k_bf_gemm<false, true>), grid, block, 0, s, A, M, K, Wb, Kp, bias, N, Y,
                       Yb);
  else if (K % 4 == 0)
    hipLaunchKernelGGL((k_bf_gemm<true, true>), grid, block, 0, s, A, M, K, Wb, Kp, bias, N, Y, Yb);
  else
    hipLaunchKernelGGL((k_bf_gemm<true, false>), grid, block, 0, s, A, M, K, Wb, Kp, bias, N, Y,
                       Yb);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_bf16_wgrad_partials(int64_t M, int K) {
  // about 512 workgroups (two per CU) over (k-block, row split), at most one split per chunk
  const int64_t nch = (M + TM - 1) / TM;
  const int nkb = lgnn_bf16_kpad(K) / BK;
  int64_t S = (512 + nkb - 1) / std::max(nkb, 1);
  S = std::min<int64_t>(std::max<int64_t>(S, 1), std::max<int64_t>(nch, 1));
  return (int)S;
}

extern "C" int lgnn_bf16_wgrad(const uint16_t* dYb, int N, const void* X, int x_is_f32, int64_t M,
                               int K, float* partials, int num_partials, void* stream) {
  if (M < 0 || K < 1 || N < 1 || N > 128 || N % 2 != 0 || !partials || num_partials < 1)
    return LGNN_EINVAL;
  if (M > 0 && (!dYb || !X)) return LGNN_EINVAL;
  if (!x_is_f32 && K % 2 != 0) return LGNN_EINVAL;
  if (M * (int64_t)K * 4 >= ((int64_t)1 << 31)) return LGNN_EINVAL;
  const int nkb = lgnn_bf16_kpad(K) / BK;
  const dim3 grid((unsigned)(nkb * num_partials)), block(NT);
  hipStream_t s = as_stream(stream);
  if (x_is_f32)
    hipLaunchKernelGGL((k_bf_wgrad<true>), grid, block, 0, s, dYb, N, X, M, K, nkb, num_partials,
                       partials);
  else
    hipLaunchKernelGGL((k_bf_wgrad<false>), grid, block, 0, s, dYb, N, X, M, K, nkb, num_partials,
                       partials);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}
