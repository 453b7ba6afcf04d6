// Dense GEMMs at fp32 accuracy on bf16 MFMA ("split-3"), any N, any K — the plain nn.Linear
// shapes outside the fused tile kernels, which the previous rounds sent to the vendor library:
//   * the reference's own in_proj, nn.Linear(1025, 128) in fp32 (gat.py:29; configs/config.py:
//     52-65 trains the GAT in fp32 on 1024 encoder channels + the lesion class, lesions.py:142,169)
//     forward Y = X W^T + b and weight gradient dW = dY^T X,
//   * every GATConv.lin / GraphConv / in_proj wider than the 128-feature tiles (the sweep's
//     widths 256 / 512, scripts/sweep.py:126) and its input gradient dX = dY W,
//   * with PLANES = 1 the same kernels are the bf16-operand GEMMs of the bf16 mode for N > 128.
//
// Split-3 (as stack3.hip): every fp32 operand x is three bf16 planes hi + mid + lo (each the RNE
// bf16 of what the planes above left; residual <= 2^-24 |x|), a product is the six plane
// products that reach 2^-24 (s3_util.h mfma_s3); bf16 x bf16 products are exact in fp32 and the
// MFMA accumulates in fp32, so the result has fp32-class error at 16/6 = 2.7x the fp32 MFMA rate.
// The fp32 A operand (node features / output gradient) is split as it is loaded; the weight
// operand's planes are written once per step (lgnn_s3_weight_planes) in the MFMA fragment order.
//
//   k_s3_gemm   Y[M][N] = A[M][K] B[N][K]^T (+ bias): grid (64-row tiles, 128-column blocks);
//               4 waves, wave w owns columns 32 w .. + 31 of the block; the A chunk (64 rows x 64
//               k) goes through three XOR-swizzled LDS planes, double-buffered; the B fragments
//               come straight from L2 (whole 1-KiB lines per wave load), one chunk ahead.
//   k_s3_wgrad2 dW partial slabs part[s][n][k] = sum over row split s of dY[m][n] X[m][k]: a
//               128 n x 128 k tile per workgroup (64 x 64 per wave), the transposed 32-row images
//               dY^T and X^T per plane in one 48-KiB buffer, the next chunk's rows in registers
//               during the MFMAs; the slabs are summed in fixed order by
//               lgnn_reduce_partials(_multi) (deterministic).
#include <algorithm>

#include "common.h"
#include "s3_util.h"

namespace lgnn_s3g {
using namespace lgnn_tile;
using lgnn_s3::bf16x2;
using lgnn_s3::f32x2;
using lgnn_s3::lds16;
using lgnn_s3::mfma16;
using lgnn_s3::mfma_s3;
using lgnn_s3::split2;
using lgnn_s3::Split2;
using lgnn_s3::u32x2;

constexpr int BK = 64;          // k per chunk
constexpr int ROWB = BK * 2;    // bytes per image row (bf16)
constexpr int IMG = TM * ROWB;  // bytes per 64-row image plane
constexpr int OOB = 0x7ff00000;  // buffer offset past every range: loads return 0

// 128-B image rows, 16-B chunk XOR-swizzled by (row >> 1) & 7: the 16 rows of a ds_read_b128
// lane group ({0-3, 12-15, 20-27} / {4-11, 16-19, 28-31}, MI355X_MICROARCH.md §LDS) land in 16
// distinct 16-B bank slots (an (row & 7) key pairs rows 8 apart on one slot: 2-way conflicts,
// measured 40 % extra LDS cycles)
__device__ __forceinline__ int swz(int row, int chunk) {
  return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ uint32_t ldb32(Buf b, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(b, off, 0, 0);
}
__device__ __forceinline__ uint32_t rne16(float v) {  // bf16 bits of v (RNE), low half
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{v, 0.f}), bf16x2)) & 0xffffu;
}

// products of one k-step: PLANES = 3 -> the six split-3 products, 1 -> the single bf16 product
template <int PLANES>
__device__ __forceinline__ f32x16 mma(const u32x4 (&a)[PLANES], const u32x4 (&b)[PLANES],
                                      f32x16 c) {
  if constexpr (PLANES == 3) return mfma_s3(a, b, c);
  else return mfma16(a[0], b[0], c);
}

// ------------------------------------------------------------------------------------------
// Y = A B^T (+ bias)
// ------------------------------------------------------------------------------------------
// A registers of a 32 MT-row tile: rows 8 MT wave + 4 i + (lane >> 4) (i < 2 MT),
// k = 4 (lane & 15) + 0..3, fp32.
template <int MT>
struct ARegs {
  uint32_t v[8 * MT];
};

// One 16-B load per row and lane, branch-free (a join of guarded loads would make the wait-count
// pass drain every load in flight): a group at or past K reads 0 through an out-of-range offset,
// and with K % 4 != 0 (!VEC) the group straddling K zeroes its columns >= K after the load (it
// reads the next row's head, or 0 past the buffer). Rows past M read 0 through the buffer range.
template <bool VEC, int MT>
__device__ __forceinline__ void load_a(ARegs<MT>& R, Buf bA, int K, int c, int rq, int kq) {
  const int k = c * BK + kq;
#pragma unroll
  for (int i = 0; i < 2 * MT; ++i) {
    const int off = (rq + 4 * i) * K + k;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(bA, opaque(k < K ? off * 4 : OOB), 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) R.v[4 * i + j] = (VEC || k + j < K) ? v[j] : 0u;
  }
}

// the chunk's four fp32 of row rq + 4 i -> PLANES bf16 planes (8 B per row and plane)
template <int PLANES, int MT>
__device__ __forceinline__ void store_a_row(unsigned char* img, const ARegs<MT>& R, int rq, int kq,
                                            int i) {
  {
    const int pos = swz(rq + 4 * i, kq >> 3) + ((kq & 7) << 1);
    const float f0 = __uint_as_float(R.v[4 * i]), f1 = __uint_as_float(R.v[4 * i + 1]);
    const float f2 = __uint_as_float(R.v[4 * i + 2]), f3 = __uint_as_float(R.v[4 * i + 3]);
    if constexpr (PLANES == 3) {
      const Split2 a = split2(f0, f1), b = split2(f2, f3);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        *reinterpret_cast<u32x2*>(img + p * IMG + pos) = u32x2{a.p[p], b.p[p]};
    } else {
      *reinterpret_cast<u32x2*>(img + pos) =
          u32x2{rne16(f0) | (rne16(f1) << 16), rne16(f2) | (rne16(f3) << 16)};
    }
  }
}
template <int PLANES, int MT>
__device__ __forceinline__ void store_a(unsigned char* img, const ARegs<MT>& R, int rq, int kq) {
#pragma unroll
  for (int i = 0; i < 2 * MT; ++i) store_a_row<PLANES>(img, R, rq, kq, i);
}

// Weight planes in fragment order (as bflin.hip's weight operand): for 128-column block nb,
// plane p, chunk c, k-step s and wave w, the 64 lanes' 16-B fragments (row 32 w + li, columns
// 64 c + 16 s + 8 h .. + 7) are 1 KiB contiguous. Plane (nb, p) starts at (nb PLANES + p) 128 Kp.
template <int PLANES>
__device__ __forceinline__ void load_b(u32x4 (&b)[4][PLANES], Buf bW, int64_t pstride, int wlane,
                                       int c) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int p = 0; p < PLANES; ++p)
      b[s][p] = __builtin_amdgcn_raw_buffer_load_b128(
          bW, (int)(p * pstride * 2) + ((c * 4 + s) * 4 * 512 + wlane) * 2, 0, 0);
}

// NCK > 0: exactly NCK chunks, the chunk sequence fully unrolled (straight-line code: the
// compiler's wait counts stay exact, every load stays in flight across the LDS-only barriers);
// NCK = 0: any K, a loop over chunk pairs whose body is the same branch-free sequence (an odd
// chunk count runs one all-zero chunk). Prefetches past the last chunk read zeros (offsets past
// the buffers' ranges), so no load is guarded by a branch.
// GATConv attention scores of the output (ATT, N <= 128): a_s[m][h] = <Y[m][hC .. hC + C),
// att_src[h]>, a_d likewise (PyG GATConv alpha_src / alpha_dst, reference gat.py:31), one fmaf
// chain per (row, head) over the tile's Y staged in the (then free) A images — the fp32 twin of
// bflin.hip's epilogue, so lgnn_gat_att's pass over XP disappears from the fp32 GAT too.
struct AttOut {
  const float* src;  // [H*C]
  const float* dst;
  float* a_s;        // [M][H]
  float* a_d;
  int H, C;
};
constexpr int YLD = 128 + 4;  // LDS row stride of the staged Y tile (floats)

// One tile of 32 MT rows (MT = 2: the 64-row tile; MT = 1: the 32-row tiles that finish a grid
// whose 64-row tiles would leave a mostly idle last round)
template <int PLANES, bool VEC, int NCK, bool ATT, int MT, int ACT = LGNN_ACT_NONE>
__device__ __forceinline__ void gemm_tile(unsigned char (&img)[2][PLANES * IMG], int64_t r0,
                                          const float* __restrict__ A, int64_t M, int K,
                                          const uint16_t* __restrict__ Wp, int Kp,
                                          const float* __restrict__ bias, int N,
                                          float* __restrict__ Y, float* __restrict__ colsum,
                                          const AttOut& att) {
  constexpr int RA = 2 * MT;  // A row groups per lane
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int nb = blockIdx.y;
  const Buf bA = mkbuf(A + r0 * K, (M - r0) * K * 4);
  const int64_t pstride = (int64_t)128 * Kp;  // bf16 elements per plane
  const Buf bW = mkbuf(Wp + nb * PLANES * pstride, PLANES * pstride * 2);
  const int rq = 8 * MT * wave + (lane >> 4), kq = 4 * (lane & 15);
  const int wlane = wave * 512 + lane * 8;
  f32x16 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x16{};
  // Software pipeline. Chunk c's products run while (a) the A fragments of k-step s + 1 are
  // read from LDS (two fragment sets: an LDS read's latency is not paid in front of each step)
  // and (b) chunk c + 1's rows are split into planes and written to the other image (one row per
  // k-step: the split's VALU work issues in the MFMAs' shadow). sched_barrier fences keep the
  // compiler from sinking the reads back to their uses. The other image was last read by chunk
  // c - 1, which every wave finished before the barrier in front of chunk c.
  auto chunk = [&](const unsigned char* im, const u32x4 (&bc)[4][PLANES], unsigned char* imn,
                   const ARegs<MT>& Rn, bool store_next) {
    u32x4 a[2][MT][PLANES];
#pragma unroll
    for (int p = 0; p < PLANES; ++p)
#pragma unroll
      for (int t = 0; t < MT; ++t) a[0][t][p] = lds16(im + p * IMG + swz(32 * t + li, h));
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s + 1 < 4) {
#pragma unroll
        for (int p = 0; p < PLANES; ++p)
#pragma unroll
          for (int t = 0; t < MT; ++t)
            a[(s + 1) & 1][t][p] = lds16(im + p * IMG + swz(32 * t + li, 2 * (s + 1) + h));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
#if defined(LGNN_ABL_S3G) && (LGNN_ABL_S3G & 1)  // timing ablation: no MFMA (operands kept live)
        acc[t][0] += __uint_as_float(a[s & 1][t][0][0] ^ bc[s][0][0]);
#else
        acc[t] = mma<PLANES>(a[s & 1][t], bc[s], acc[t]);
#endif
      }
      if (store_next && s < RA) store_a_row<PLANES>(imn, Rn, rq, kq, s);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // two register sets ping-pong: R[c & 1] holds chunk c's rows until chunk c - 1's products
  // have stored them, then takes chunk c + 2's
  ARegs<MT> R0, R1;
  u32x4 b0[4][PLANES], b1[4][PLANES];
  load_a<VEC>(R0, bA, K, 0, rq, kq);
  load_b<PLANES>(b0, bW, pstride, wlane, 0);
  load_a<VEC>(R1, bA, K, 1, rq, kq);
  load_b<PLANES>(b1, bW, pstride, wlane, 1);
  store_a<PLANES>(img[0], R0, rq, kq);
  load_a<VEC>(R0, bA, K, 2, rq, kq);
  lds_barrier();
  auto step = [&](int c, ARegs<MT>& Rn, u32x4 (&bc)[4][PLANES], bool store_next) {
    chunk(img[c & 1], bc, img[(c + 1) & 1], Rn, store_next);
    load_a<VEC>(Rn, bA, K, c + 3, rq, kq);
#if !(defined(LGNN_ABL_S3G) && (LGNN_ABL_S3G & 2))  // timing ablation: no B loads in the loop
    load_b<PLANES>(bc, bW, pstride, wlane, c + 2);
#endif
    lds_barrier();  // image c + 1 complete, image c's reads done
  };
  if constexpr (NCK > 0) {
#pragma unroll
    for (int c = 0; c < NCK; ++c) {
      if (c & 1) step(c, R0, b1, c + 1 < NCK);
      else step(c, R1, b0, c + 1 < NCK);
    }
  } else {
    const int npair = (Kp / BK + 1) / 2;
    for (int cp = 0; cp < npair; ++cp) {
      step(2 * cp, R1, b0, true);
      step(2 * cp + 1, R0, b1, true);
    }
  }
  // epilogue: + bias; fp32 rows as 128-B segments per (row, wave); optional column sums
  const int n = nb * 128 + 32 * wave + li;
  const bool nok = n < N;
  const float bv = (bias && nok) ? bias[n] : 0.f;
  const Buf bY = mkbuf(Y + r0 * N, (M - r0) * N * 4);
  const int ncol = nok ? n : OOB / 4;
  if (MT == 2 && colsum) {  // this tile's column sums of Y (rows past M hold 0; 64-row grids)
    float cs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) cs += acc[0][r] + acc[MT - 1][r];
    cs += __shfl_xor(cs, 32, 64);
    const int64_t rows = M - r0 < TM ? M - r0 : TM;
    if (h == 0 && nok) colsum[(r0 / TM) * N + n] = cs + (float)rows * bv;
  }
#pragma unroll
  for (int q = 0; q < MT; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
      float v = acc[q][r] + bv;
      if constexpr (ACT == LGNN_ACT_ELU) v = elu_f(v);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), bY, (m * N + ncol) * 4, 0, 0);
    }
  if constexpr (ATT) {
    static_assert((TM * YLD + 256) * 4 <= 2 * PLANES * IMG, "the Y tile fits in the A images");
    float* ytile = reinterpret_cast<float*>(&img[0][0]);
    // att_src / att_dst staged beside the tile: the chains below then read LDS only (from global
    // memory every step of a chain waited on an L1/L2 round trip: 19.2 vs 14.4 us per launch at
    // the reference lins, K = 128)
    float* attv = ytile + TM * YLD;
    lds_barrier();  // every wave's last image reads are done
    if (nok) {
#pragma unroll
      for (int q = 0; q < MT; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
          ytile[m * YLD + n] = acc[q][r] + bv;
        }
    }
    if (tid < N) {  // N = H C <= 128 (lgnn_s3_gemm_att)
      attv[tid] = att.src[tid];
      attv[128 + tid] = att.dst[tid];
    }
    lds_barrier();
    const int H = att.H, C = att.C;
    const int64_t rows = M - r0 < 32 * MT ? M - r0 : 32 * MT;
    for (int p = tid; p < 32 * MT * H; p += NT) {
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

// Grid: n64 tiles of 64 rows (blocks 0 .. n64 - 1, dealt to the XCDs in contiguous ranges), then
// 32-row tiles for the remaining rows. With more 64-row tiles than resident workgroups the
// launch's last round would hold a few of them on an otherwise idle chip; the host keeps whole
// rounds of 64-row tiles and cuts the rest in halves (lgnn_s3_gemm: the reference in_proj at
// 42,279 rows is 661 tiles over 512 slots).
template <int PLANES, bool VEC, int NCK, bool ATT = false, int ACT = LGNN_ACT_NONE>
__global__ __launch_bounds__(NT, 2) void k_s3_gemm(const float* __restrict__ A, int64_t M, int K,
                                                   const uint16_t* __restrict__ Wp, int Kp,
                                                   const float* __restrict__ bias, int N,
                                                   float* __restrict__ Y,
                                                   float* __restrict__ colsum, int n64,
                                                   AttOut att = AttOut{}) {
  __shared__ __attribute__((aligned(16))) unsigned char img[2][PLANES * IMG];
  const int64_t b = blockIdx.x;
  if (b < n64) {
    const int64_t q = n64 / 8, r = n64 % 8, xcd = b % 8;
    const int64_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    gemm_tile<PLANES, VEC, NCK, ATT, 2, ACT>(img, t * TM, A, M, K, Wp, Kp, bias, N, Y, colsum,
                                             att);
  } else {
    gemm_tile<PLANES, VEC, NCK, ATT, 1, ACT>(img, (int64_t)n64 * TM + (b - n64) * 32, A, M, K, Wp,
                                             Kp, bias, N, Y, nullptr, att);
  }
}

// ------------------------------------------------------------------------------------------
// dW partial slabs (k_s3_wgrad2): a workgroup owns a 128 (n) x 128 (k) tile of dW and a row
// split; 4 waves each own 64 n x 64 k (four 32 x 32 accumulators), so every operand fragment a
// wave reads from LDS feeds two column (row) blocks: 0.5 KiB of LDS per MFMA (a 32-n wave tile
// took 0.75 KiB and ran LDS-bound: 155 us for the C3 in_proj, 67 % bank-conflict cycles). Chunks of 32
// rows: the transposed images dY^T [128 n][32 m] and X^T [128 k][32 m] x 3 planes are 48 KiB
// (single buffer, two workgroups per CU), the next chunk's rows in registers during the MFMAs.
// Image rows are 64 B (4 chunks of 16 B), chunk-swizzled by (row >> 2) & 3: a 16-lane b128 read
// group of consecutive rows touches 64 distinct banks. (The transposed ds_write_b64 groups are
// 2-way: rows j and j + 4 share a 16-bank quarter. 64 B of padding per 4 rows removes that, and
// measured no faster: 229 vs 232 us at 65,536 x 512 x 512, equal at the in_proj.)
// ------------------------------------------------------------------------------------------
constexpr int W2M = 32;               // rows per chunk
constexpr int W2ROW = W2M * 2;        // bytes per image row (bf16)
constexpr int W2IMG = 128 * W2ROW;    // bytes per 128-row image plane

__device__ __forceinline__ int w2off(int row, int c16) {  // byte offset of 16-B chunk c16
  return row * W2ROW + ((c16 ^ ((row >> 2) & 3)) << 4);
}

// per lane: rows 4 rq .. 4 rq + 3 of the chunk (rq = tid % 8), columns 4 cq .. 4 cq + 3
// (cq = tid / 8) of the 128-wide block, one 16-B load per row, for dY and for X (rq fast: a
// 16-lane write group then covers two image rows whole — 2-way bank overlap instead of 4)
struct W2Regs {
  u32x4 y[4];
  u32x4 x[4];
};

__device__ __forceinline__ u32x4 ld16(Buf b, int off, int col, int ncol) {
  // a 4-column group inside the columns [0, ncol): one 16-B load; at or past it: 0 (OOB offset).
  // Straddling it (ncol % 4 != 0) the columns past it are zeroed by w2_mask when the registers
  // are consumed, not here: a select right after the load makes the compiler wait for the load
  // in the middle of the MFMA phase it is meant to overlap
  return __builtin_amdgcn_raw_buffer_load_b128(b, opaque(col < ncol ? off : OOB), 0, 0);
}

__device__ __forceinline__ void w2_load(W2Regs& R, Buf bY, Buf bX, int N, int K, int m0, int n0,
                                        int k0, int tid) {
  const int rq = tid & 7, cq = tid >> 3;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 4 * rq + i;
    const int n = n0 + 4 * cq, k = k0 + 4 * cq;
    R.y[i] = ld16(bY, (m * N + n) * 4, n, N);
    R.x[i] = ld16(bX, (m * K + k) * 4, k, K);
  }
}

// the straddling group's columns >= N (dY) / >= K (X) -> 0 (no-op unless N or K % 4 != 0)
__device__ __forceinline__ void w2_mask(W2Regs& R, int N, int K, int n0, int k0, int tid) {
  const int cq = tid >> 3, n = n0 + 4 * cq, k = k0 + 4 * cq;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      R.y[i][j] = n + j < N ? R.y[i][j] : 0u;
      R.x[i][j] = k + j < K ? R.x[i][j] : 0u;
    }
}

// transposed write of one operand: column c (4 cq + j) gets rows 4 rq .. + 3 as 8 B per plane
template <int PLANES>
__device__ __forceinline__ void w2_store1(unsigned char* img, const u32x4 (&v)[4], int tid) {
  const int rq = tid & 7, cq = tid >> 3;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 4 * cq + j;
    const int pos = w2off(row, rq >> 1) + (rq & 1) * 8;  // rows 4 rq .. of 32: chunk rq / 2
    const float f0 = __uint_as_float(v[0][j]), f1 = __uint_as_float(v[1][j]);
    const float f2 = __uint_as_float(v[2][j]), f3 = __uint_as_float(v[3][j]);
    if constexpr (PLANES == 3) {
      const Split2 a = split2(f0, f1), b = split2(f2, f3);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        *reinterpret_cast<u32x2*>(img + p * W2IMG + pos) = u32x2{a.p[p], b.p[p]};
    } else {
      *reinterpret_cast<u32x2*>(img + pos) =
          u32x2{rne16(f0) | (rne16(f1) << 16), rne16(f2) | (rne16(f3) << 16)};
    }
  }
}

template <int PLANES>
__global__ __launch_bounds__(NT, 2) void k_s3_wgrad2(const float* __restrict__ dY, int N,
                                                     const float* __restrict__ X, int64_t M,
                                                     int K, int nkb, int cps,
                                                     float* __restrict__ part,
                                                     float* __restrict__ dbpart) {
  __shared__ __attribute__((aligned(16))) unsigned char sm[2 * PLANES * W2IMG];
  unsigned char* iy = sm;
  unsigned char* ix = sm + PLANES * W2IMG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wn = wave & 1, wk = wave >> 1;  // this wave's 64 n x 64 k quarter of the tile
  const int64_t L = xcd_block();  // the k-blocks of one row split are adjacent: one XCD's L2
  const int kb = (int)(L % nkb), s = (int)(L / nkb);
  const int k0 = kb * 128, n0 = blockIdx.y * 128;
  const Buf bX = mkbuf(X, M * K * 4), bY = mkbuf(dY, M * N * 4);
  const int64_t nch = (M + W2M - 1) / W2M;
  const int64_t c0 = (int64_t)s * cps;
  const int64_t cend = c0 + cps < nch ? c0 + cps : nch;
  f32x16 acc[2][2] = {{{}, {}}, {{}, {}}};
  float cs[4] = {0.f, 0.f, 0.f, 0.f};  // column sums of dY (the bias gradient), this lane's 4 n
  W2Regs R;
  // branch-free: the prefetch after the split's last chunk reads the next split's rows (or zeros
  // past M) and is dropped
  w2_load(R, bY, bX, N, K, (int)(c0 * W2M), n0, k0, tid);
  for (int64_t c = c0; c < cend; ++c) {
    lds_barrier();  // the previous chunk's image reads are done
    if ((N | K) & 3) w2_mask(R, N, K, n0, k0, tid);  // uniform: only a width % 4 != 0 straddles
    w2_store1<PLANES>(iy, R.y, tid);
    w2_store1<PLANES>(ix, R.x, tid);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) cs[j] += __uint_as_float(R.y[i][j]);
#if !(defined(LGNN_ABL_S3G) && (LGNN_ABL_S3G & 2))  // timing ablation: no global loads in the loop
    w2_load(R, bY, bX, N, K, (int)((c + 1) * W2M), n0, k0, tid);
#endif
    lds_barrier();  // images complete (the next chunk's loads stay in flight)
#pragma unroll
    for (int st = 0; st < 2; ++st) {  // two k-steps of 16 rows
      u32x4 a[2][PLANES], b[2][PLANES];
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int p = 0; p < PLANES; ++p) {
          a[q][p] = lds16(iy + p * W2IMG + w2off(64 * wn + 32 * q + li, 2 * st + h));
          b[q][p] = lds16(ix + p * W2IMG + w2off(64 * wk + 32 * q + li, 2 * st + h));
        }
#pragma unroll
      for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
#if defined(LGNN_ABL_S3G) && (LGNN_ABL_S3G & 1)
          acc[qa][qb][0] += __uint_as_float(a[qa][0][0] ^ b[qb][0][0]);
#else
          acc[qa][qb] = mma<PLANES>(a[qa], b[qb], acc[qa][qb]);
#endif
        }
    }
  }
  // slab s: rows n = n0 + 64 wn + 32 qa + (r & 3) + 8 (r >> 2) + 4 h, columns k0 + 64 wk + 32 qb + li
  float* slab = part + (int64_t)s * N * K;
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int k = k0 + 64 * wk + 32 * qb + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + 64 * wn + 32 * qa + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (n < N && k < K) slab[(int64_t)n * K + k] = acc[qa][qb][r];
      }
    }
  if (dbpart && kb == 0) {  // db partial row s: the 8 row groups' sums folded in group order
    float* red = reinterpret_cast<float*>(sm);
    __syncthreads();
    const int rq = tid & 7, cq = tid >> 3;
#pragma unroll
    for (int j = 0; j < 4; ++j) red[rq * 128 + 4 * cq + j] = cs[j];
    __syncthreads();
    if (tid < 128 && n0 + tid < N) {
      float t = red[tid];
#pragma unroll
      for (int g = 1; g < 8; ++g) t += red[g * 128 + tid];
      dbpart[(int64_t)s * N + n0 + tid] = t;
    }
  }
}

// ------------------------------------------------------------------------------------------
// weight planes: Wp[nb][p][128][Kp] of W [N][K] (or of W^T [K][N] with transposed = 1: the
// operand of dX = dY W), fragment order, zero-padded, PLANES = 3 (split) or 1 (bf16 RNE)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void wprep_range(const float* __restrict__ W, int rows, int cols,
                                            int transposed, int planes, int Kp, int nnb,
                                            uint16_t* __restrict__ Wp, int64_t i0, int64_t stride) {
  const int64_t per = (int64_t)128 * Kp;  // elements of one plane of one block
  const int64_t total = per * nnb;
  for (int64_t i = i0; i < total; i += stride) {
    const int nb = (int)(i / per);
    const int64_t j = i % per;
    const int e = (int)(j & 7), lane = (int)((j >> 3) & 63), wave = (int)((j >> 9) & 3);
    const int64_t cs = j >> 11;  // 4 chunk + k-step
    const int r = nb * 128 + 32 * wave + (lane & 31);       // output column (operand row)
    const int q = (int)(cs * 16) + 8 * (lane >> 5) + e;     // reduction index
    // operand element (r, q) of B [R][Q]: W[r][q], or W^T: W[q][r]
    float v = 0.f;
    if (!transposed) {
      if (r < rows && q < cols) v = W[(int64_t)r * cols + q];
    } else {
      if (r < cols && q < rows) v = W[(int64_t)q * cols + r];
    }
    uint16_t* base = Wp + (int64_t)nb * planes * per + j;
    for (int p = 0; p < planes; ++p) {
      const uint32_t b = rne16(v);
      base[p * per] = (uint16_t)b;
      v -= __uint_as_float(b << 16);
    }
  }
}

__global__ void k_s3_wprep(const float* __restrict__ W, int rows, int cols, int transposed,
                           int planes, int Kp, int nnb, uint16_t* __restrict__ Wp) {
  wprep_range(W, rows, cols, transposed, planes, Kp, nnb, Wp,
              (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

struct WprepJobs {
  const float* W[LGNN_MAX_WPREP];
  uint16_t* Wp[LGNN_MAX_WPREP];
  int rows[LGNN_MAX_WPREP], cols[LGNN_MAX_WPREP], tr[LGNN_MAX_WPREP];
  int Kp[LGNN_MAX_WPREP], nnb[LGNN_MAX_WPREP];
  int boff[LGNN_MAX_WPREP + 1];  // prefix of the workgroups per job
  int n, planes;
};

__global__ void k_s3_wprep_multi(WprepJobs J) {
  int j = 0;
  while (j + 1 < J.n && J.boff[j + 1] <= (int)blockIdx.x) ++j;
  const int lb = (int)blockIdx.x - J.boff[j], nb = J.boff[j + 1] - J.boff[j];
  wprep_range(J.W[j], J.rows[j], J.cols[j], J.tr[j], J.planes, J.Kp[j], J.nnb[j], J.Wp[j],
              (int64_t)lb * blockDim.x + threadIdx.x, (int64_t)nb * blockDim.x);
}

}  // namespace lgnn_s3g

using namespace lgnn_s3g;

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" int lgnn_s3_weight_planes_multi(int n, const float* const* W, const int* rows,
                                           const int* cols, const int* transposed, int planes,
                                           uint16_t* const* Wp, void* stream) {
  if (n < 1 || n > LGNN_MAX_WPREP || !W || !rows || !cols || !transposed || !Wp ||
      (planes != 1 && planes != 3))
    return LGNN_EINVAL;
  WprepJobs J = {};
  J.n = n;
  J.planes = planes;
  for (int j = 0; j < n; ++j) {
    if (!W[j] || !Wp[j] || rows[j] < 1 || cols[j] < 1) return LGNN_EINVAL;
    const int out = transposed[j] ? cols[j] : rows[j], in = transposed[j] ? rows[j] : cols[j];
    J.W[j] = W[j];
    J.Wp[j] = Wp[j];
    J.rows[j] = rows[j];
    J.cols[j] = cols[j];
    J.tr[j] = transposed[j] ? 1 : 0;
    J.Kp[j] = (in + BK - 1) / BK * BK;
    J.nnb[j] = (out + 127) / 128;
    const int64_t total = (int64_t)128 * J.Kp[j] * J.nnb[j];
    J.boff[j + 1] = J.boff[j] + (int)std::min<int64_t>((total + 255) / 256, 512);
  }
  hipLaunchKernelGGL(k_s3_wprep_multi, dim3((unsigned)J.boff[n]), dim3(256), 0, as_stream(stream),
                     J);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" size_t lgnn_s3_weight_planes_numel(int out_features, int in_features, int planes) {
  if (out_features < 1 || in_features < 1 || (planes != 1 && planes != 3)) return 0;
  const int Kp = (in_features + BK - 1) / BK * BK, nnb = (out_features + 127) / 128;
  return (size_t)nnb * planes * 128 * Kp;
}

extern "C" int lgnn_s3_weight_planes(const float* W, int rows, int cols, int transposed,
                                     int planes, uint16_t* Wp, void* stream) {
  if (!W || !Wp || rows < 1 || cols < 1 || (planes != 1 && planes != 3)) return LGNN_EINVAL;
  const int out = transposed ? cols : rows, in = transposed ? rows : cols;
  const int Kp = (in + BK - 1) / BK * BK, nnb = (out + 127) / 128;
  const int64_t total = (int64_t)128 * Kp * nnb;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(k_s3_wprep, dim3(grid), dim3(256), 0, as_stream(stream), W, rows, cols,
                     transposed, planes, Kp, nnb, Wp);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

// Row tiling of k_s3_gemm: whole rounds of 64-row tiles over the resident slots (2 workgroups per
// CU, divided among the column blocks), the rest as 32-row tiles — for long K only (the in_proj,
// K = 1025: 75.3 -> 73.5 us; at K = 128 the halves lost more per tile than the round saved);
// only 64-row tiles when the caller wants per-64-row column sums. Returns grid.x, sets *n64.
static unsigned s3g_grid(int64_t M, int K, int nblk, bool colsum, int* n64) {
  const int64_t t64 = (M + TM - 1) / TM;
  static int slots = -1;
  if (slots < 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      slots = 2 * cus;
    else slots = 0;
  }
  const int64_t per = nblk > 0 ? slots / nblk : 0;
  if (colsum || K < 512 || per < 8 || t64 <= per) {
    *n64 = (int)t64;
    return (unsigned)t64;
  }
  const int64_t full = t64 / per * per;  // whole rounds of 64-row tiles
  *n64 = (int)full;
  return (unsigned)(full + (M - full * TM + 31) / 32);
}

extern "C" int lgnn_s3_gemm(const float* A, int64_t M, int K, const uint16_t* Wp, int N,
                            int planes, const float* bias, float* Y, float* colsum_part,
                            void* stream) {
  if (M < 0 || K < 1 || N < 1 || !Wp || !Y || (planes != 1 && planes != 3)) return LGNN_EINVAL;
  if (M > 0 && !A) return LGNN_EINVAL;
  const int Kp = (K + BK - 1) / BK * BK;
  // 32-bit buffer offsets: A's tile range, Y's range (a masked column stores at >= 2^31 - 2^20
  // bytes, past it), and one weight block's planes
  if ((M + TM) * (int64_t)K * 4 >= ((int64_t)1 << 31) || M * (int64_t)N * 4 >= ((int64_t)1 << 30) ||
      (int64_t)3 * 128 * Kp * 2 >= ((int64_t)1 << 31))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  int n64 = 0;
  const unsigned gx = s3g_grid(M, K, (N + 127) / 128, colsum_part != nullptr, &n64);
  const dim3 grid(gx, (unsigned)((N + 127) / 128)), block(NT);
  hipStream_t s = as_stream(stream);
  const bool v = K % 4 == 0;
  const int nck = Kp / BK;
#define LGNN_S3G(P, V, NC) \
  hipLaunchKernelGGL((k_s3_gemm<P, V, NC>), grid, block, 0, s, A, M, K, Wp, Kp, bias, N, Y, \
                     colsum_part, n64)
#define LGNN_S3G_N(P, V)                 \
  switch (nck) {                         \
    case 2: LGNN_S3G(P, V, 2); break;    \
    case 4: LGNN_S3G(P, V, 4); break;    \
    case 8: LGNN_S3G(P, V, 8); break;    \
    case 17: LGNN_S3G(P, V, 17); break;  \
    default: LGNN_S3G(P, V, 0); break;   \
  }
  // the unrolled bodies: K <= 128 / 256 / 512 (lins and their dX) and 1025..1088 (the
  // reference in_proj); other widths run the pair loop
  if (planes == 3) {
    if (v) { LGNN_S3G_N(3, true) } else { LGNN_S3G_N(3, false) }
  } else {
    if (v) { LGNN_S3G_N(1, true) } else { LGNN_S3G_N(1, false) }
  }
#undef LGNN_S3G_N
#undef LGNN_S3G
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

// Y = act(A B^T + b) (act = LGNN_ACT_ELU: torch's ELU in the epilogue, as the tile kernels)
extern "C" int lgnn_s3_gemm_act(const float* A, int64_t M, int K, const uint16_t* Wp, int N,
                                const float* bias, int act, float* Y, void* stream) {
  if (act == LGNN_ACT_NONE) return lgnn_s3_gemm(A, M, K, Wp, N, 3, bias, Y, nullptr, stream);
  if (act != LGNN_ACT_ELU || M < 0 || K < 1 || N < 1 || !Wp || !Y) return LGNN_EINVAL;
  if (M > 0 && !A) return LGNN_EINVAL;
  const int Kp = (K + BK - 1) / BK * BK;
  if ((M + TM) * (int64_t)K * 4 >= ((int64_t)1 << 31) || M * (int64_t)N * 4 >= ((int64_t)1 << 30) ||
      (int64_t)3 * 128 * Kp * 2 >= ((int64_t)1 << 31))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  int n64 = 0;
  const unsigned gx = s3g_grid(M, K, (N + 127) / 128, false, &n64);
  const dim3 grid(gx, (unsigned)((N + 127) / 128)), block(NT);
  hipStream_t s = as_stream(stream);
  const bool v = K % 4 == 0;
  const int nck = Kp / BK;
#define LGNN_S3E(V, NC)                                                                          \
  hipLaunchKernelGGL((k_s3_gemm<3, V, NC, false, LGNN_ACT_ELU>), grid, block, 0, s, A, M, K, Wp, \
                     Kp, bias, N, Y, nullptr, n64)
#define LGNN_S3E_N(V)                  \
  switch (nck) {                       \
    case 2: LGNN_S3E(V, 2); break;     \
    case 8: LGNN_S3E(V, 8); break;     \
    default: LGNN_S3E(V, 0); break;    \
  }
  if (v) { LGNN_S3E_N(true) } else { LGNN_S3E_N(false) }
#undef LGNN_S3E_N
#undef LGNN_S3E
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_s3_gemm_att(const float* A, int64_t M, int K, const uint16_t* Wp, int N,
                                int planes, float* Y, const float* att_src, const float* att_dst,
                                int heads, int C, float* a_s, float* a_d, void* stream) {
  if (M < 0 || K < 1 || N < 1 || N > 128 || !Wp || !Y || planes != 3 || heads < 1 || C < 1 || heads * C != N || !att_src || !att_dst || !a_s || !a_d)
    return LGNN_EINVAL;
  if (M > 0 && !A) return LGNN_EINVAL;
  const int Kp = (K + BK - 1) / BK * BK;
  if ((M + TM) * (int64_t)K * 4 >= ((int64_t)1 << 31) || M * (int64_t)N * 4 >= ((int64_t)1 << 30) ||
      (int64_t)3 * 128 * Kp * 2 >= ((int64_t)1 << 31))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  int n64 = 0;
  const dim3 grid(s3g_grid(M, K, 1, false, &n64), 1), block(NT);
  hipStream_t s = as_stream(stream);
  const AttOut at{att_src, att_dst, a_s, a_d, heads, C};
  const bool v = K % 4 == 0;
  const int nck = Kp / BK;
#define LGNN_S3A(P, V, NC)                                                                      \
  hipLaunchKernelGGL((k_s3_gemm<P, V, NC, true>), grid, block, 0, s, A, M, K, Wp, Kp, nullptr, N, \
                     Y, nullptr, n64, at)
#define LGNN_S3A_N(P, V)                 \
  switch (nck) {                         \
    case 2: LGNN_S3A(P, V, 2); break;    \
    case 17: LGNN_S3A(P, V, 17); break;  \
    default: LGNN_S3A(P, V, 0); break;   \
  }
  if (v) { LGNN_S3A_N(3, true) } else { LGNN_S3A_N(3, false) }
#undef LGNN_S3A_N
#undef LGNN_S3A
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

// k_s3_wgrad2: 32-row chunks per split, so that the grid (128-wide k-blocks x splits x n-blocks)
// holds about two workgroups per CU (512), at least 4 chunks per split
static int s3_wg_cps(int64_t M, int K, int N) {
  const int64_t nch = std::max<int64_t>((M + W2M - 1) / W2M, 1);
  const int64_t work = (int64_t)((K + 127) / 128) * ((N + 127) / 128);
  int64_t splits = std::max<int64_t>(512 / work, 1);
  int64_t cps = (nch + splits - 1) / splits;
  const int mincps = 4;
  if (cps < mincps) cps = mincps;
  return (int)cps;
}

extern "C" int lgnn_s3_wgrad_partials(int64_t M, int K, int N) {
  if (M < 0 || K < 1 || N < 1) return 0;
  const int64_t nch = std::max<int64_t>((M + W2M - 1) / W2M, 1);
  const int cps = s3_wg_cps(M, K, N);
  return (int)((nch + cps - 1) / cps);
}

extern "C" int lgnn_s3_wgrad(const float* dY, int N, const float* X, int64_t M, int K, int planes,
                             float* partials, int num_partials, float* db_partials,
                             void* stream) {
  if (M < 0 || K < 1 || N < 1 || !partials || (planes != 1 && planes != 3)) return LGNN_EINVAL;
  if (num_partials != lgnn_s3_wgrad_partials(M, K, N)) return LGNN_EINVAL;
  if (M > 0 && (!dY || !X)) return LGNN_EINVAL;
  if ((M + 2 * W2M) * (int64_t)std::max(K, N) * 4 >= ((int64_t)1 << 31)) return LGNN_EINVAL;
  const int nkb = (K + 127) / 128, cps = s3_wg_cps(M, K, N);
  const dim3 grid((unsigned)(nkb * num_partials), (unsigned)((N + 127) / 128)), block(NT);
  hipStream_t s = as_stream(stream);
  if (planes == 3)
    hipLaunchKernelGGL((k_s3_wgrad2<3>), grid, block, 0, s, dY, N, X, M, K, nkb, cps, partials,
                       db_partials);
  else
    hipLaunchKernelGGL((k_s3_wgrad2<1>), grid, block, 0, s, dY, N, X, M, K, nkb, cps, partials,
                       db_partials);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
