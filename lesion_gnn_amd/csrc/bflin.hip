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
// 16-B chunk XOR-swizzled by (row >> 1) & 7: the 16 rows of a ds_read_b128 lane group land in
// 16 distinct 16-B bank slots (s3gemm.hip swz)
__device__ __forceinline__ int swz(int row, int chunk) {
  return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ u32x4 lds16(const unsigned char* p) {
  return *reinterpret_cast<const u32x4*>(p);
}
__device__ __forceinline__ f32x16 mfma_bf(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// a value through an empty asm: a select feeding a buffer offset stays a v_cndmask instead of being
// sunk into two branch-guarded loads (whose join makes the wait-count pass drain to vmcnt(0))
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
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

// One 16-B (fp32) or 8-B (bf16) load per row and lane. FULL: the chunk lies inside K, so no
// column test; else every group past K reads 0 and (fp32, K % 4 != 0: !VEC) the one group that
// straddles K loads dword by dword. Rows past M read 0 through the buffer range. Buffer loads
// need dword alignment only, so fp32 rows of any K take the 16-B form. Branch-free, so the
// compiler's wait counts stay exact across the unrolled chunk sequence.
template <bool AF32, bool VEC, bool FULL>
__device__ __forceinline__ void gemm_load_a(ARegs<AF32>& R, Buf bA, int K, int c, int rq, int kq) {
  const int k = c * BK + kq;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = rq + 4 * i;
    const int off = row * K + k;
    if constexpr (AF32 && (FULL || VEC)) {
      const u32x4 v =
          __builtin_amdgcn_raw_buffer_load_b128(bA, FULL ? off * 4 : opaque(k < K ? off * 4 : OOB), 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) R.v[4 * i + j] = v[j];
    } else if constexpr (AF32) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        R.v[4 * i + j] = ldb32(bA, opaque(k + j < K ? (off + j) * 4 : OOB));
    } else {
      const u32x2 v = __builtin_bit_cast(
          u32x2, __builtin_amdgcn_raw_buffer_load_b64(bA, FULL ? off * 2 : opaque(k < K ? off * 2 : OOB),
                                                      0, 0));
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

// Weight operand in fragment order: for chunk c, k-step s and wave w, the 64 lanes' 16-B MFMA
// fragments (row 32 w + li, columns 64 c + 16 s + 8 h .. + 7) are 1 KiB contiguous, so each wave
// load reads whole cache lines. Element (row r, column q) sits at
//   ((((q / 16) * 4 + r / 32) * 64 + 32 ((q / 8) & 1) + r % 32) * 8 + q % 8.
__device__ __forceinline__ void gemm_load_b(u32x4 (&b)[4], Buf bW, int wlane, int c, int h) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
    b[s] = __builtin_amdgcn_raw_buffer_load_b128(bW, ((c * 4 + s) * 4 * 512 + wlane) * 2, 0, 0);
}

// NCK > 0: exactly NCK chunks (Kp = 64 NCK), the loop fully unrolled — chunks 0 .. NCK - 2 are
// inside K, only the last tests columns; NCK = 0: any Kp, every chunk tests its columns.
// GATConv attention scores of the output (ATT): a_s[m][h] = <Y[m][hC .. hC + C), att_src[h]>,
// a_d likewise (PyG GATConv alpha_src / alpha_dst, reference gat.py:31): the tile's Y values go
// to LDS and each thread takes (row, head) pairs, so lgnn_gat_att's pass over XP disappears.
struct AttOut {
  const float* src;  // [H*C]
  const float* dst;
  float* a_s;        // [M][H]
  float* a_d;
  int H, C;
};
constexpr int YLD = 128 + 4;  // LDS row stride of the staged Y tile (floats)

template <bool AF32, bool VEC, int NCK, bool ATT = false>
__global__ __launch_bounds__(NT) void k_bf_gemm(const void* __restrict__ A, int64_t M, int K,
                                                const uint16_t* __restrict__ Wb, int Kp,
                                                const float* __restrict__ bias, int N,
                                                float* __restrict__ Y, uint16_t* __restrict__ Yb,
                                                float* __restrict__ colsum,
                                                AttOut att = AttOut{}) {
  __shared__ __attribute__((aligned(16))) unsigned char img[2][TM * ROWB];
  __shared__ __attribute__((aligned(16))) float ytile[ATT ? TM * YLD : 1];
  __shared__ float attv[ATT ? 256 : 1];  // att_src / att_dst (the chains read LDS only)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t r0 = xcd_block() * TM;
  constexpr int ESZ = AF32 ? 4 : 2;
  const Buf bA = mkbuf(static_cast<const char*>(A) + r0 * K * ESZ, (M - r0) * K * ESZ);
  const Buf bW = mkbuf(Wb, (int64_t)128 * Kp * 2);
  const int rq = 16 * wave + (lane >> 4), kq = 4 * (lane & 15);
  const int nck = NCK > 0 ? NCK : Kp / BK;
  const int wrow = wave * 512 + lane * 8;  // this lane's fragment within a (chunk, k-step)
  f32x16 acc0 = {}, acc1 = {};
  auto load_a = [&](ARegs<AF32>& R, int c) {
    if (NCK > 0 && c < NCK - 1) gemm_load_a<AF32, VEC, true>(R, bA, K, c, rq, kq);
    else gemm_load_a<AF32, VEC, false>(R, bA, K, c, rq, kq);
  };
  auto mfma_chunk = [&](const unsigned char* im, const u32x4(&bc)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u32x4 a0 = lds16(im + swz(li, 2 * s + h));
      const u32x4 a1 = lds16(im + swz(32 + li, 2 * s + h));
      acc0 = mfma_bf(a0, bc[s], acc0);
      acc1 = mfma_bf(a1, bc[s], acc1);
    }
  };
  if constexpr (NCK > 0) {
    // D register sets, the chunk sequence unrolled: chunks c + 1 .. c + D are in flight while
    // chunk c is stored and used (D = 3 for the 17-chunk in_proj: 48 KiB per workgroup)
    constexpr int D = NCK >= 8 ? 3 : 2;
    ARegs<AF32> R[D];
    u32x4 Bq[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d < NCK) {
        load_a(R[d], d);
        gemm_load_b(Bq[d], bW, wrow, d, h);
      }
#pragma unroll
    for (int c = 0; c < NCK; ++c) {
      unsigned char* im = img[c & 1];
      gemm_store_a<AF32>(im, R[c % D], rq, kq);
      if (c + D < NCK) load_a(R[c % D], c + D);
      __syncthreads();  // image c complete (and image c - 2's reads done before barrier c - 1)
      mfma_chunk(im, Bq[c % D]);
      if (c + D < NCK) gemm_load_b(Bq[c % D], bW, wrow, c + D, h);
    }
  } else {
    // any Kp: two register sets, ping-pong
    ARegs<AF32> R0, R1;
    u32x4 b0[4], b1[4];
    load_a(R0, 0);
    gemm_load_b(b0, bW, wrow, 0, h);
    if (nck > 1) {
      load_a(R1, 1);
      gemm_load_b(b1, bW, wrow, 1, h);
    }
    auto step = [&](int c, ARegs<AF32>& R, u32x4(&bc)[4]) {
      unsigned char* im = img[c & 1];
      gemm_store_a<AF32>(im, R, rq, kq);
      if (c + 2 < nck) load_a(R, c + 2);
      __syncthreads();
      mfma_chunk(im, bc);
      if (c + 2 < nck) gemm_load_b(bc, bW, wrow, c + 2, h);
    };
    for (int c = 0; c < nck; c += 2) {
      step(c, R0, b0);
      if (c + 1 < nck) step(c + 1, R1, b1);
    }
  }
  // epilogue (P layout): + b; fp32 rows and their bf16 copy as 128-B / 64-B row segments
  const int n = 32 * wave + li;
  const bool nok = n < N;
  const float bv = (bias && nok) ? bias[n] : 0.f;
  const Buf bY = mkbuf(Y ? Y + r0 * N : nullptr, Y ? (M - r0) * N * 4 : 0);
  const Buf bYb = mkbuf(Yb ? Yb + r0 * N : nullptr, Yb ? (M - r0) * N * 2 : 0);
  const int ncol = nok ? n : OOB / 4;  // out-of-range column: every store lands past the range
  if (colsum) {  // this tile's column sums of Y (rows past M hold 0): 32 rows per lane half
    float cs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) cs += acc0[r];
#pragma unroll
    for (int r = 0; r < 16; ++r) cs += acc1[r];
    cs += __shfl_xor(cs, 32, 64);
    const int64_t rows = M - r0 < TM ? M - r0 : TM;
    if (h == 0 && nok) colsum[(r0 / TM) * N + n] = cs + (float)rows * bv;
  }
  if (Y) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = (q ? acc1[r] : acc0[r]) + bv;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), bY, (m * N + ncol) * 4, 0, 0);
      }
  }
  if (Yb) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = (q ? acc1[r] : acc0[r]) + bv;
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(pk2(v, 0.f) & 0xffffu), bYb,
                                              (m * N + ncol) * 2, 0, 0);
      }
  }
  if constexpr (ATT) {
    if (nok) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
          ytile[m * YLD + n] = (q ? acc1[r] : acc0[r]) + bv;
        }
    }
    if (tid < N) {  // N = H C <= 128 (lgnn_bf16_gemm_att)
      attv[tid] = att.src[tid];
      attv[128 + tid] = att.dst[tid];
    }
    __syncthreads();
    const int H = att.H, C = att.C;
    const int64_t rows = M - r0 < TM ? M - r0 : TM;
    for (int p = tid; p < TM * H; p += NT) {
      const int m = p / H, hd = p % H;
      if (m >= rows) continue;
      const float* yr = ytile + m * YLD + hd * C;
      const float* ws = attv + hd * C;
      const float* wd = attv + 128 + hd * C;
      float ps = 0.f, pd = 0.f;
#pragma unroll 8
      for (int c = 0; c < C; ++c) {
        ps = fmaf(yr[c], ws[c], ps);
        pd = fmaf(yr[c], wd[c], pd);
      }
      att.a_s[(r0 + m) * H + hd] = ps;
      att.a_d[(r0 + m) * H + hd] = pd;
    }
  }
}

// ------------------------------------------------------------------------------------------
// dW partial slabs: part[s][n][k] = sum over split s's CPB row chunks of dY[m][n] X[m][k]
// ------------------------------------------------------------------------------------------
template <bool XF32>
struct WRegs {
  // X: XF32 k = k0 + 4 (lane & 15) + 0..3 of rows 16 w + 4 (lane >> 4) + i (i < 4); bf16 the k
  // pair 2 (lane & 31) of rows 16 w + 8 (lane >> 5) + j (j < 8)
  uint32_t x[XF32 ? 16 : 8];
  uint32_t y[16];  // dY: n pair 2 lane, rows 16 w + 8 g + j (g < 2, j < 8)
};

// Rows past M read 0 through the buffer ranges (offsets computed in 32 bits: M K size < 2^31 is
// checked on the host, and a row past M lands past the range or wraps negative, i.e. past it
// too). Columns n >= N of dY and k >= K of X are not masked: they only feed dW entries the slab
// store drops. No selects, so no branches: the compiler's wait counts stay exact. FULL: the
// k-block lies inside K (16-B loads); else dword loads, each range-checked on its own.
template <bool XF32, bool FULL>
__device__ __forceinline__ void wg_load(WRegs<XF32>& R, Buf bX, Buf bY, int K, int N, int m0,
                                        int k0, int lane, int wave) {
  const int n = 2 * lane;
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + 16 * wave + 8 * g + j;
      R.y[8 * g + j] = ldb32(bY, (m * N + n) * 2);
    }
  if constexpr (XF32) {
    const int k = k0 + 4 * (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = (m0 + 16 * wave + 4 * (lane >> 4) + i) * K + k;
      if constexpr (FULL) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(bX, off * 4, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) R.x[4 * i + j] = v[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) R.x[4 * i + j] = ldb32(bX, (off + j) * 4);
      }
    }
  } else {  // lanes 0-31 rows 16 w + j, lanes 32-63 rows 16 w + 8 + j
    const int k = k0 + 2 * (lane & 31);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + 16 * wave + 8 * (lane >> 5) + j;
      R.x[j] = ldb32(bX, (m * K + k) * 2);
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
  }
  if constexpr (XF32) {  // column k + j: rows 16 w + 4 q .. + 3 as one 8-B write
    const int q = lane >> 4, kq = 4 * (lane & 15);
    const int ch = 2 * wave + (q >> 1), off = (q & 1) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      u32x2 o;
      o[0] = pk2(__uint_as_float(R.x[j]), __uint_as_float(R.x[4 + j]));
      o[1] = pk2(__uint_as_float(R.x[8 + j]), __uint_as_float(R.x[12 + j]));
      *reinterpret_cast<u32x2*>(ix + swz(kq + j, ch) + off) = o;
    }
  } else {
    const int ch = 2 * wave + (lane >> 5), k = 2 * (lane & 31);
    *reinterpret_cast<u32x4*>(ix + swz(k, ch)) = pack_halves<false>(R.x);
    *reinterpret_cast<u32x4*>(ix + swz(k + 1, ch)) = pack_halves<true>(R.x);
  }
}

struct WgSmem {
  unsigned char y[2][128 * ROWB];  // dY^T [n][m]
  unsigned char x[2][64 * ROWB];   // X^T [k][m]
};

// the split's CPB chunks, fully unrolled with two register sets in flight
template <bool XF32, bool FULL, int CPB>
__device__ __forceinline__ void wg_run(WgSmem& sm, f32x16& acc0, f32x16& acc1, Buf bX, Buf bY,
                                       int K, int N, int c0, int k0, int lane, int wave) {
  const int h = lane >> 5, li = lane & 31;
  WRegs<XF32> R0, R1;
  wg_load<XF32, FULL>(R0, bX, bY, K, N, c0 * TM, k0, lane, wave);
  if (CPB > 1) wg_load<XF32, FULL>(R1, bX, bY, K, N, (c0 + 1) * TM, k0, lane, wave);
#pragma unroll
  for (int i = 0; i < CPB; ++i) {
    WRegs<XF32>& R = (i & 1) ? R1 : R0;
    unsigned char* py = sm.y[i & 1];
    unsigned char* px = sm.x[i & 1];
    wg_store<XF32>(py, px, R, lane, wave);
    if (i + 2 < CPB) wg_load<XF32, FULL>(R, bX, bY, K, N, (c0 + i + 2) * TM, k0, lane, wave);
    __syncthreads();  // images i complete (images i - 2's reads done before barrier i - 1)
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const u32x4 a = lds16(py + swz(32 * wave + li, 2 * st + h));
      const u32x4 x0 = lds16(px + swz(li, 2 * st + h));
      const u32x4 x1 = lds16(px + swz(32 + li, 2 * st + h));
      acc0 = mfma_bf(a, x0, acc0);
      acc1 = mfma_bf(a, x1, acc1);
    }
  }
}

template <bool XF32, int CPB>
__global__ __launch_bounds__(NT) void k_bf_wgrad(const uint16_t* __restrict__ dYb, int N,
                                                 const void* __restrict__ X, int64_t M, int K,
                                                 int nkb, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) WgSmem sm;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t L = xcd_block();  // the k-blocks of one row split are adjacent: one XCD's L2
  const int kb = (int)(L % nkb), s = (int)(L / nkb);
  const int k0 = kb * BK;
  constexpr int ESZ = XF32 ? 4 : 2;
  const Buf bX = mkbuf(X, M * K * ESZ), bY = mkbuf(dYb, M * N * 2);
  f32x16 acc0 = {}, acc1 = {};
  if (k0 + BK <= K)  // uniform: one unrolled body per block
    wg_run<XF32, true, CPB>(sm, acc0, acc1, bX, bY, K, N, s * CPB, k0, lane, wave);
  else
    wg_run<XF32, false, CPB>(sm, acc0, acc1, bX, bY, K, N, s * CPB, k0, lane, wave);
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
// weight operands: Wb [128][Kp] = bf16(W), WTb [128][Np] = bf16(W^T), zero-padded, in the
// fragment order of gemm_load_b
// ------------------------------------------------------------------------------------------
__global__ void k_bf_wprep(const float* __restrict__ W, int N, int K, int Kp, int Np,
                           uint16_t* __restrict__ Wb, uint16_t* __restrict__ WTb) {
  const int64_t n1 = (int64_t)128 * Kp, n2 = WTb ? (int64_t)128 * Np : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + n2;
       i += (int64_t)gridDim.x * blockDim.x) {
    // element i of the fragment order: (row r, column q) of the [128][width] operand
    const bool t = i >= n1;
    const int64_t j = t ? i - n1 : i;
    const int e = (int)(j & 7), lane = (int)((j >> 3) & 63), wave = (int)((j >> 9) & 3);
    const int64_t cs = j >> 11;  // 4 chunk + k-step
    const int r = 32 * wave + (lane & 31), q = (int)(cs * 16) + 8 * (lane >> 5) + e;
    const int n = t ? q : r, k = t ? r : q;  // W^T: row k, column n
    const float v = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.f;
    (t ? WTb : Wb)[j] = (uint16_t)(pk2(v, 0.f) & 0xffffu);
  }
}

// several weights' operands in one launch: job j owns blocks [first[j], first[j + 1])
constexpr int kMaxPrep = 8;
struct PrepJobs {
  const float* W[kMaxPrep];
  uint16_t* Wb[kMaxPrep];
  uint16_t* WTb[kMaxPrep];
  int N[kMaxPrep], K[kMaxPrep], Kp[kMaxPrep], Np[kMaxPrep];
  int first[kMaxPrep + 1];
  int n;
};

__global__ void k_bf_wprep_multi(PrepJobs jobs) {
  int j = 0;
  while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.first[j + 1]) ++j;
  const int nb = jobs.first[j + 1] - jobs.first[j];
  const int N = jobs.N[j], K = jobs.K[j], Kp = jobs.Kp[j], Np = jobs.Np[j];
  const float* __restrict__ W = jobs.W[j];
  uint16_t* __restrict__ Wb = jobs.Wb[j];
  uint16_t* __restrict__ WTb = jobs.WTb[j];
  const int64_t n1 = (int64_t)128 * Kp, n2 = WTb ? (int64_t)128 * Np : 0;
  for (int64_t i = (int64_t)(blockIdx.x - jobs.first[j]) * blockDim.x + threadIdx.x; i < n1 + n2;
       i += (int64_t)nb * blockDim.x) {
    const bool t = i >= n1;  // the same element map as k_bf_wprep
    const int64_t q0 = t ? i - n1 : i;
    const int e = (int)(q0 & 7), lane = (int)((q0 >> 3) & 63), wave = (int)((q0 >> 9) & 3);
    const int64_t cs = q0 >> 11;
    const int r = 32 * wave + (lane & 31), q = (int)(cs * 16) + 8 * (lane >> 5) + e;
    const int n = t ? q : r, k = t ? r : q;
    const float v = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.f;
    (t ? WTb : Wb)[q0] = (uint16_t)(pk2(v, 0.f) & 0xffffu);
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

extern "C" int lgnn_bf16_weight_prep_multi(int n, const float* const* W, const int* N,
                                           const int* K, uint16_t* const* Wb,
                                           uint16_t* const* WTb, void* stream) {
  if (n < 1 || n > kMaxPrep || !W || !N || !K || !Wb || !WTb) return LGNN_EINVAL;
  PrepJobs jobs{};
  jobs.n = n;
  jobs.first[0] = 0;
  for (int j = 0; j < n; ++j) {
    if (!W[j] || !Wb[j] || N[j] < 1 || N[j] > 128 || K[j] < 1) return LGNN_EINVAL;
    if (WTb[j] && K[j] > 128) return LGNN_EINVAL;
    jobs.W[j] = W[j];
    jobs.Wb[j] = Wb[j];
    jobs.WTb[j] = WTb[j];
    jobs.N[j] = N[j];
    jobs.K[j] = K[j];
    jobs.Kp[j] = lgnn_bf16_kpad(K[j]);
    jobs.Np[j] = lgnn_bf16_kpad(N[j]);
    const int64_t total = (int64_t)128 * jobs.Kp[j] + (WTb[j] ? (int64_t)128 * jobs.Np[j] : 0);
    jobs.first[j + 1] = jobs.first[j] + (int)std::min<int64_t>((total + 255) / 256, 512);
  }
  hipLaunchKernelGGL(k_bf_wprep_multi, dim3(jobs.first[n]), dim3(256), 0, as_stream(stream), jobs);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_bf16_gemm_att(const void* A, int a_is_f32, int64_t M, int K,
                                  const uint16_t* Wb, int N,
                                  float* Y, uint16_t* Yb, const float* att_src,
                                  const float* att_dst, int H, int C, float* a_s, float* a_d,
                                  void* stream) {
  // the GATConv.lin forward, 64 < K <= 128 (two chunks), with the scores
  if (M < 0 || K <= BK || K > 2 * BK || K % 4 != 0 || N < 1 || N > 128 || !Wb || !Y)
    return LGNN_EINVAL;
  if (H < 1 || C < 1 || H * C != N || !att_src || !att_dst || !a_s || !a_d) return LGNN_EINVAL;
  if (M > 0 && !A) return LGNN_EINVAL;
  if ((M + TM) * (int64_t)K * 4 >= ((int64_t)1 << 31) || M * (int64_t)N * 4 >= ((int64_t)1 << 30))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  const int Kp = lgnn_bf16_kpad(K);
  const AttOut att{att_src, att_dst, a_s, a_d, H, C};
  const dim3 grid((unsigned)((M + TM - 1) / TM));
  if (a_is_f32)  // rounded to bf16 as loaded, as lgnn_bf16_gemm does
    hipLaunchKernelGGL((k_bf_gemm<true, true, 2, true>), grid, dim3(NT), 0, as_stream(stream), A,
                       M, K, Wb, Kp, nullptr, N, Y, Yb, nullptr, att);
  else
    hipLaunchKernelGGL((k_bf_gemm<false, true, 2, true>), grid, dim3(NT), 0, as_stream(stream), A,
                       M, K, Wb, Kp, nullptr, N, Y, Yb, nullptr, att);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_bf16_gemm(const void* A, int a_is_f32, int64_t M, int K, const uint16_t* Wb,
                              const float* bias, int N, float* Y, uint16_t* Yb, float* colsum_part,
                              void* stream) {
  if (M < 0 || K < 1 || N < 1 || N > 128 || !Wb || (!Y && !Yb)) return LGNN_EINVAL;
  if (M > 0 && !A) return LGNN_EINVAL;
  if (!a_is_f32 && K % 4 != 0) return LGNN_EINVAL;
  // 32-bit buffer offsets; a masked column's stores land at >= 2^30 bytes, past Yb's range too
  if ((M + TM) * (int64_t)K * 4 >= ((int64_t)1 << 31) || M * (int64_t)N * 4 >= ((int64_t)1 << 30))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  const int Kp = lgnn_bf16_kpad(K), nck = Kp / BK;
  const dim3 grid((unsigned)((M + TM - 1) / TM)), block(NT);
  hipStream_t s = as_stream(stream);
#define LGNN_BFG(AF, V, NC) \
  hipLaunchKernelGGL((k_bf_gemm<AF, V, NC>), grid, block, 0, s, A, M, K, Wb, Kp, bias, N, Y, Yb, \
                     colsum_part)
  // the unrolled bodies: K <= 128 (the GAT layers, dX) and K <= 1088 (the reference in_proj,
  // 1025 input channels); other widths run the generic loop
  const bool v = K % 4 == 0;
  if (!a_is_f32) {
    if (nck == 2) LGNN_BFG(false, true, 2);
    else LGNN_BFG(false, true, 0);
  } else if (nck == 2) {
    if (v) LGNN_BFG(true, true, 2);
    else LGNN_BFG(true, false, 2);
  } else if (nck == 17) {
    if (v) LGNN_BFG(true, true, 17);
    else LGNN_BFG(true, false, 17);
  } else {
    if (v) LGNN_BFG(true, true, 0);
    else LGNN_BFG(true, false, 0);
  }
#undef LGNN_BFG
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

// chunks per split: the smallest of 3, 6, 12, 24 that keeps the grid within about 480
// workgroups (two per CU fit at once)
static int wg_cpb(int64_t M, int K) {
  const int64_t nch = std::max<int64_t>((M + TM - 1) / TM, 1);
  const int nkb = lgnn_bf16_kpad(K) / BK;
  for (int cpb = 3; cpb < 24; cpb *= 2)
    if (nkb * ((nch + cpb - 1) / cpb) <= 480) return cpb;
  return 24;
}

extern "C" int lgnn_bf16_wgrad_partials(int64_t M, int K) {
  if (M < 0 || K < 1) return 0;
  const int64_t nch = std::max<int64_t>((M + TM - 1) / TM, 1);
  const int cpb = wg_cpb(M, K);
  return (int)((nch + cpb - 1) / cpb);
}

extern "C" int lgnn_bf16_wgrad(const uint16_t* dYb, int N, const void* X, int x_is_f32, int64_t M,
                               int K, float* partials, int num_partials, void* stream) {
  if (M < 0 || K < 1 || N < 1 || N > 128 || N % 2 != 0 || !partials) return LGNN_EINVAL;
  if (num_partials != lgnn_bf16_wgrad_partials(M, K)) return LGNN_EINVAL;
  if (M > 0 && (!dYb || !X)) return LGNN_EINVAL;
  if (!x_is_f32 && K % 2 != 0) return LGNN_EINVAL;
  if ((M + 32 * TM) * (int64_t)K * 4 >= ((int64_t)1 << 31)) return LGNN_EINVAL;
  const int nkb = lgnn_bf16_kpad(K) / BK, cpb = wg_cpb(M, K);
  const dim3 grid((unsigned)(nkb * num_partials)), block(NT);
  hipStream_t s = as_stream(stream);
#define LGNN_BFW(XF, C) \
  hipLaunchKernelGGL((k_bf_wgrad<XF, C>), grid, block, 0, s, dYb, N, X, M, K, nkb, partials)
#define LGNN_BFW_C(XF)              \
  switch (cpb) {                    \
    case 3: LGNN_BFW(XF, 3); break;   \
    case 6: LGNN_BFW(XF, 6); break;   \
    case 12: LGNN_BFW(XF, 12); break; \
    default: LGNN_BFW(XF, 24); break; \
  }
  if (x_is_f32) {
    LGNN_BFW_C(true)
  } else {
    LGNN_BFW_C(false)
  }
#undef LGNN_BFW_C
#undef LGNN_BFW
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}
