// Split-3 layer-wise linear kernels: Y = act(P(X) W^T + b) and its backward on bf16 MFMA at fp32
// accuracy (the three-plane operands and six products of stack3.hip), for the layers the fused GCN
// stack does not cover — the GIN MLP's two Linears around BatchNorm (reference gin.py:23,
// GINConv(MLP([d1, d2, d2]))) — with the same BatchNorm folding as the fp32 bodies in tile_lw.h
// (BnFuse modes). Fast-path shapes (K, N <= 128, multiples of 4), every tile (no tile mask).
//
// Unlike stack3.hip the LDS images hold fp32 rows and the MFMA operands are split into planes as
// they are read (two ds_read_b128 + four split2 per k-step fragment): the images stay 32 KiB each,
// so two workgroups share a CU, and no plane image has to be rebuilt per layer. Weights come as
// the fragment-ordered planes of lgnn_weight_planes (W for the forward, W^T for dX).
//
// Layouts (4 waves, wave w owns features [32w, 32w + 32)):
//   P layout   MFMA accumulator: feature on the lane, rows m = 32 q + (r & 3) + 8 (r >> 2) + 4 h
//   images     fp32 [row][128], 16-B chunks XOR-swizzled by row & 15 (conflict-free b128 reads of
//              one chunk by 16 rows, and of 16 chunks of one row)
// forward : image = X (or S = (1 + eps) X + sum of neighbours, aggregated from a raw-row copy as
//           tile_lw.h does) -> P = image W^T -> + b, act -> Y (P layout stores: 128-B row
//           segments per wave), BN statistics per lane's column.
// backward: dZ (P layout, loaded straight from dY with act' / BN backward applied) -> node-major
//           image; X (P layout) -> feature-major image; dW += dZ^T X (dZ split in registers),
//           dX = dZ W (image rows x W^T planes) -> HBM, BN backward sums per lane's column.
#include "common.h"
#include "tile.h"
#include "tile_util.h"
#include "s3_util.h"
#include "tile_lw.h"

namespace lgnn_s3 {

// float index of (row, col) in a [rows][W] fp32 image (W = 128 or 64)
template <int W = 128>
__device__ __forceinline__ int img_off(int row, int col) {
  return row * W + (((col >> 2) ^ (row & 15)) << 2) + (col & 3);
}

// operand fragment of image row `row`, k-step s, lane half h: the eight values at perm16 positions
// 16 s + 8 h .. + 7 (columns 16 s + 4 h + 0..3 and 16 s + 8 + 4 h + 0..3), as three planes
template <int W = 128>
__device__ __forceinline__ void frag_split(const float* img, int row, int s, int h,
                                           u32x4 (&f)[3]) {
  const f32x4 a = ld4(img + img_off<W>(row, 16 * s + 4 * h));
  const f32x4 b = ld4(img + img_off<W>(row, 16 * s + 8 + 4 * h));
  u32x2 oa[3], ob[3];
  split4(a, oa);
  split4(b, ob);
#pragma unroll
  for (int p = 0; p < 3; ++p) f[p] = u32x4{oa[p][0], oa[p][1], ob[p][0], ob[p][1]};
}

// A tile of a [rows][ld] fp32 matrix in P layout (lane column colv < ncols, else 0; rows past M
// read 0)
__device__ __forceinline__ void ld_pt(f32x16 (&v)[2], const float* base, int64_t M, int64_t r0,
                                      int ld, int colv, int ncols, int h) {
  const int64_t rem = M - r0;
  const Buf b = mkbuf(base + r0 * ld, rem > 0 ? rem * ld * 4 : 0);
  const int vb = colv < ncols ? (4 * h * ld + colv) * 4 : 0x7fff0000;
  const int rs = __builtin_amdgcn_readfirstlane(ld * 4);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mc = 32 * a + (r & 3) + 8 * (r >> 2);
      v[a][r] = __builtin_bit_cast(float,
                                   __builtin_amdgcn_raw_buffer_load_b32(b, vb + mc * rs, 0, 0));
    }
}

// P-layout pair -> node-step operand fragments (s = 0, 1 from v[0], 2, 3 from v[1])
__device__ __forceinline__ void split_pl(const f32x16 (&v)[2], u32x4 (&o)[4][3]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const f32x16& pa = v[s >> 1];
    const int rb = 8 * (s & 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const Split2 s2 = split2(pa[rb + 2 * i], pa[rb + 2 * i + 1]);
#pragma unroll
      for (int p = 0; p < 3; ++p) o[s][p][i] = s2.p[p];
    }
  }
}

// this lane's fragments of a fragment-ordered weight plane set (row 32 w + li)
__device__ __forceinline__ void load_wfrag(u32x4 (&wf)[3][8], const uint16_t* __restrict__ Wp) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint16_t* base = Wp + wave * 8 * 512 + lane * 8;
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      wf[p][s] = *reinterpret_cast<const u32x4*>(base + p * PLANE + 512 * s);
}

// fold the lane halves' fp64 column sums and write this workgroup's partial row (lanes h = 0)
__device__ __forceinline__ void part_write_pl(double s0, double s1, double* part, int N) {
  s0 += __shfl_xor(s0, 32, 64);
  s1 += __shfl_xor(s1, 32, 64);
  const int lane = threadIdx.x & 63, n = 32 * (threadIdx.x >> 6) + (lane & 31);
  if (lane < 32 && n < N) {
    part[(int64_t)blockIdx.x * 2 * N + n] = s0;
    part[(int64_t)blockIdx.x * 2 * N + N + n] = s1;
  }
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
template <bool GATHER>
struct LinFwdSmem {
  float img[TM * 128];                   // the A image (X, BN(X) or S), split as it is read
  float xa[GATHER ? TM * LDS : 4];       // GATHER: the raw rows the aggregation reads
  TileIdx ti;
};

template <bool GATHER, int ACT, int BNM>
__global__ __launch_bounds__(NT, 1) void k_s3_lin_fwd(
    const float* __restrict__ X, int64_t M, int K, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const float* __restrict__ w, float self_scale,
    const uint16_t* __restrict__ Wp, const float* __restrict__ b, int N, float* __restrict__ Y,
    float* __restrict__ S_out, BnFuse bn) {
  static_assert(BNM == BN_NONE || BNM == BN_STATS || (BNM == BN_IN && !GATHER), "");
  __shared__ __attribute__((aligned(16))) LinFwdSmem<GATHER> sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31, hw = tid >> 5;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int n = 32 * wave + li;
  double s0 = 0.0, s1 = 0.0;  // BN_STATS: this lane's column
  int64_t t = blockIdx.x;
  if (t >= ntiles) {
    if constexpr (BNM == BN_STATS) part_write_pl(s0, s1, bn.part, N);
    return;
  }
  u32x4 wf[3][8];
  load_wfrag(wf, Wp);
  const float bias = (b && n < N) ? b[n] : 0.f;
  const bool kin = 4 * li < K;
  const int kq = kin ? 4 * li : K - 4;
  f32x4 bsc = {}, bsh = {};
  if constexpr (BNM == BN_IN) {
    bsc = ld4(bn.scale + kq);
    bsh = ld4(bn.shift + kq);
  }
  const Buf bX = mkbuf(X, M * K * 4);
  const Buf bS = mkbuf(S_out, S_out ? M * K * 4 : 0);
  f32x4 xr[8];
  IdxRegs R;
  load_rows(xr, bX, K, (int)(t * TM));
  if constexpr (GATHER) {
    idx_load_head(R, rowptr, M, t * TM);
    idx_load_body(R, col, w);
  }
  for (; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * TM;
    const int64_t tn = t + gridDim.x;
    const bool has_next = tn < ntiles;
    if constexpr (GATHER) {
      bool staged = true;
      store_rows_lds(sm.xa, xr, M, K, r0);
      idx_store(sm.ti, staged, R, r0);
      __syncthreads();
      if (has_next) {
        load_rows(xr, bX, K, (int)(tn * TM));
        idx_load_head(R, rowptr, M, tn * TM);
      }
      auto agg_tile = [&](auto staged_tag) {
        constexpr bool STG = decltype(staged_tag)::value;
#pragma unroll 1
        for (int it = 0; it < 8; ++it) {
          const int rr = hw + 8 * it;
          f32x4 a;
          if constexpr (STG) a = agg_row_local(sm.ti, rr, sm.xa);
          else a = agg_row_global(sm.ti, rr, X, K, kq, col, w);
          if (self_scale != 0.f) a += self_scale * ld4(sm.xa + rr * LDS + 4 * li);
          a = sel4(kin && r0 + rr < M, a);
          st4(sm.img + img_off(rr, 4 * li), a);
          if (S_out && kin) bst4(bS, (int)((r0 + rr) * K + 4 * li) * 4, a);
        }
      };
      if (staged) agg_tile(std::true_type{});
      else agg_tile(std::false_type{});
      if (has_next) idx_load_body(R, col, w);
    } else {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        const int64_t row = r0 + rr;
        const bool ok = kin && row < M;
        f32x4 v = xr[it];
        if constexpr (BNM == BN_IN) {  // A = ELU(X * scale + shift) * mask, also to act_out
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = elu_f(fmaf(v[j], bsc[j], bsh[j]));
          if (bn.mask && ok) v *= ld4(bn.mask + row * K + 4 * li);
          if (ok) st4(bn.act_out + row * K + 4 * li, v);
        }
        st4(sm.img + img_off(rr, 4 * li), sel4(ok, v));
      }
      if (has_next) load_rows(xr, bX, K, (int)(tn * TM));
    }
    __syncthreads();  // image complete
    // P = image W^T: A = image rows (split as read), B = W planes (registers)
    f32x16 p0 = {}, p1 = {};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u32x4 f0[3], f1[3], w3[3];
      frag_split(sm.img, li, s, h, f0);
      frag_split(sm.img, 32 + li, s, h, f1);
#pragma unroll
      for (int p = 0; p < 3; ++p) w3[p] = wf[p][s];
      p0 = mfma_s3(f0, w3, p0);
      p1 = mfma_s3(f1, w3, p1);
    }
    // epilogue (P layout): + b, act, Y rows as 128-B segments per wave; BN statistics
    const Buf bY = mkbuf(Y + r0 * N, (M - r0) * N * 4);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
        float v = (q ? p1[r] : p0[r]) + bias;
        if constexpr (ACT == LGNN_ACT_ELU) v = elu_f(v);
        const bool ok = n < N && r0 + m < M;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), bY,
                                              ok ? (m * N + n) * 4 : INT32_MAX - 3, 0, 0);
        if constexpr (BNM == BN_STATS) {
          if (ok) {
            s0 += (double)v;
            s1 += (double)v * (double)v;
          }
        }
      }
    __syncthreads();  // image reads done before the next tile writes it
  }
  if constexpr (BNM == BN_STATS) part_write_pl(s0, s1, bn.part, N);
}

// ------------------------------------------------------------------------------------------
// backward (DIRECT gradient): dZ = dY act'(H) [BN_GIN: BN backward of dY]; dW += dZ^T X;
// db += colsum dZ; dX = dZ W [BN_GSTATS: BN backward sums over dX]
// ------------------------------------------------------------------------------------------
struct LinBwdSmem {
  float z[TM * 128];  // dZ, node-major [m][n]: the A image of dX = dZ W
  float x[128 * TM];  // X^T, feature-major [k][m]: the B image of dW = dZ^T X
};

template <int ACT, bool DX, int BNM>
__global__ __launch_bounds__(NT, 1) void k_s3_lin_bwd(
    const float* __restrict__ dY, const float* __restrict__ H, const float* __restrict__ X,
    int64_t M, int K, const uint16_t* __restrict__ WpT, int N, float* __restrict__ dX,
    float* __restrict__ dWp, float* __restrict__ dbp, BnFuse bn) {
  static_assert(BNM == BN_NONE || (BNM == BN_GSTATS && DX) ||
                    (BNM == BN_GIN && ACT == LGNN_ACT_NONE), "");
  __shared__ __attribute__((aligned(16))) LinBwdSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int n = 32 * wave + li;  // dZ column (P layout) and dX column k
  // BatchNorm constants of this lane's column: of dY (BN_GIN) or of dX (BN_GSTATS)
  float bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f, bmg = 0.f, bmgx = 0.f;
  if constexpr (BNM != BN_NONE) {
    const int W1 = BNM == BN_GIN ? N : K;
    const int c = n < W1 ? n : W1 - 1;
    bsc = bn.scale[c];
    bsh = bn.shift[c];
    bmu = bn.mean[c];
    bis = bn.invstd[c];
    if (BNM == BN_GIN && bn.training) {
      bmg = (float)(bn.sums[c] / bn.count);
      bmgx = (float)(bn.sums[N + c] / bn.count);
    }
  }
  f32x16 dw[4] = {{}, {}, {}, {}};
  float dbacc = 0.f;
  double s0 = 0.0, s1 = 0.0;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * TM;
    // dZ (P layout)
    f32x16 dz[2];
    ld_pt(dz, dY, M, r0, N, n, N, h);
    if constexpr (ACT == LGNN_ACT_ELU) {
      f32x16 hv[2];
      ld_pt(hv, H, M, r0, N, n, N, h);
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) dz[q][r] *= elu_grad_from_out(hv[q][r]);
    }
    if constexpr (BNM == BN_GIN) {  // dZ = BN backward of the ELU(BN(Z)) * mask output
      f32x16 zv[2], mk[2];
      ld_pt(zv, bn.Z, M, r0, N, n, N, h);
      if (bn.mask) ld_pt(mk, bn.mask, M, r0, N, n, N, h);
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float z = zv[q][r];
          const float gg =
              dz[q][r] * bn_elu_grad(z, bsc, bsh) * (bn.mask ? mk[q][r] : 1.f);
          const float v = bn.training ? bsc * (gg - bmg - (z - bmu) * bis * bmgx) : bsc * gg;
          dz[q][r] = (n < N && r0 + m < M) ? v : 0.f;
        }
    }
    {  // db: this lane's 32 rows, then the partner half's
      float sacc = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc += dz[q][r];
      sacc += __shfl_xor(sacc, 32, 64);
      dbacc += sacc;
    }
    // X (P layout: feature k = n on the lane) -> feature-major image; dZ -> node-major image
    {
      f32x16 xp[2];
      ld_pt(xp, X, M, r0, K, n, K, h);
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m0 = 32 * q + 8 * g + 4 * h;
          st4(sm.x + img_off<TM>(n, m0),
              f32x4{xp[q][4 * g], xp[q][4 * g + 1], xp[q][4 * g + 2], xp[q][4 * g + 3]});
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
        sm.z[img_off(m, n)] = dz[q][r];
      }
    __syncthreads();
    // dW[n][k] += sum_m dZ[m][n] X[m][k]: A = dZ (split from registers, node steps), B = X^T
    // image rows k = 32 kb + li
    {
      u32x4 gp[4][3];
      split_pl(dz, gp);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          u32x4 xb[3];
          frag_split<TM>(sm.x, 32 * kb + li, s, h, xb);
          dw[kb] = mfma_s3(gp[s], xb, dw[kb]);
        }
    }
    if constexpr (DX) {
      // dX[m][k] = sum_n dZ[m][n] W[n][k]: A = dZ image rows m, B = W^T planes (L2, two halves)
      const uint16_t* wbase = WpT + wave * 8 * 512 + lane * 8;
      f32x16 dh[2] = {f32x16{}, f32x16{}};
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        u32x4 wf[3][4];
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            wf[p][s4] = *reinterpret_cast<const u32x4*>(wbase + p * PLANE + 512 * (4 * half + s4));
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            u32x4 f[3], bw[3];
            frag_split(sm.z, 32 * q + li, 4 * half + s4, h, f);
#pragma unroll
            for (int p = 0; p < 3; ++p) bw[p] = wf[p][s4];
            dh[q] = mfma_s3(f, bw, dh[q]);
          }
      }
      // dX rows (P layout: feature k = n on the lane); BN backward sums of dX = dA
      const Buf bdX = mkbuf(dX + r0 * K, (M - r0) * K * 4);
      f32x16 zv[2], mk[2];
      if constexpr (BNM == BN_GSTATS) {
        ld_pt(zv, bn.Z, M, r0, K, n, K, h);
        if (bn.mask) ld_pt(mk, bn.mask, M, r0, K, n, K, h);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float v = dh[q][r];
          const bool ok = n < K && r0 + m < M;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), bdX,
                                                ok ? (m * K + n) * 4 : INT32_MAX - 3, 0, 0);
          if constexpr (BNM == BN_GSTATS) {
            if (ok) {
              const float z = zv[q][r];
              const float gg = v * bn_elu_grad(z, bsc, bsh) * (bn.mask ? mk[q][r] : 1.f);
              s0 += (double)gg;
              s1 += (double)gg * (double)((z - bmu) * bis);
            }
          }
        }
    }
    __syncthreads();  // image reads done before the next tile writes them
  }
  if constexpr (BNM == BN_GSTATS) part_write_pl(s0, s1, bn.part, K);
  // partial slot blockIdx.x: dW rows n = 32 wave + (r & 3) + 8 (r >> 2) + 4h, columns
  // k = 32 kb + li; db from the h = 0 lanes
  float* slab = dWp + (int64_t)blockIdx.x * N * K;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const int k = 32 * kb + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (o < N && k < K) slab[(int64_t)o * K + k] = dw[kb][r];
    }
  }
  if (dbp && h == 0 && n < N) dbp[(int64_t)blockIdx.x * N + n] = dbacc;
}

}  // namespace lgnn_s3

using namespace lgnn_s3;

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" int lgnn_node_linear_fwd_s3(const float* X, int64_t M, int K, const int32_t* rowptr,
                                       const int32_t* col, const float* w, float self_scale,
                                       const uint16_t* planes, const float* b, int N, int act,
                                       float* Y, float* S_out, double* stats_part,
                                       const float* bn_scale, const float* bn_shift,
                                       const float* bn_mask, float* bn_out, void* stream) {
  if (M < 0 || !planes || !Y || (M > 0 && !X) || !lgnn_tile_fits(M, K, N)) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  const bool stats = stats_part != nullptr, bnin = bn_scale != nullptr;
  if (stats && bnin) return LGNN_EINVAL;
  if (bnin && (rowptr || !bn_shift || !bn_out)) return LGNN_EINVAL;
  if (rowptr && !col) return LGNN_EINVAL;
  const int P = lgnn_tile_partials(M);
  BnFuse bn = {};
  bn.part = stats_part;
  bn.scale = bn_scale;
  bn.shift = bn_shift;
  bn.mask = bn_mask;
  bn.act_out = bn_out;
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    if (stats && hipMemsetAsync(stats_part, 0, (size_t)P * 2 * N * sizeof(double), s) != hipSuccess)
      return (int)hipGetLastError();
    return LGNN_OK;
  }
  const dim3 grid((unsigned)P);
  float* So = rowptr ? S_out : nullptr;
#define LGNN_S3L(G, A, BM)                                                                   \
  hipLaunchKernelGGL((k_s3_lin_fwd<G, A, BM>), grid, dim3(NT), 0, s, X, M, K, rowptr, col, w, \
                     self_scale, planes, b, N, Y, So, bn)
  const int bm = stats ? BN_STATS : (bnin ? BN_IN : BN_NONE);
  if (rowptr) {
    if (bm == BN_STATS) {
      if (act == LGNN_ACT_ELU) LGNN_S3L(true, LGNN_ACT_ELU, BN_STATS);
      else LGNN_S3L(true, LGNN_ACT_NONE, BN_STATS);
    } else {
      if (act == LGNN_ACT_ELU) LGNN_S3L(true, LGNN_ACT_ELU, BN_NONE);
      else LGNN_S3L(true, LGNN_ACT_NONE, BN_NONE);
    }
  } else if (bm == BN_IN) {
    if (act == LGNN_ACT_ELU) LGNN_S3L(false, LGNN_ACT_ELU, BN_IN);
    else LGNN_S3L(false, LGNN_ACT_NONE, BN_IN);
  } else if (bm == BN_STATS) {
    if (act == LGNN_ACT_ELU) LGNN_S3L(false, LGNN_ACT_ELU, BN_STATS);
    else LGNN_S3L(false, LGNN_ACT_NONE, BN_STATS);
  } else {
    if (act == LGNN_ACT_ELU) LGNN_S3L(false, LGNN_ACT_ELU, BN_NONE);
    else LGNN_S3L(false, LGNN_ACT_NONE, BN_NONE);
  }
#undef LGNN_S3L
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

extern "C" int lgnn_node_linear_bwd_s3(int bn_mode, const float* dY, const float* H, int act,
                                       const float* X, int64_t M, int K,
                                       const uint16_t* planes_t, int N, float* dXpre,
                                       float* dW_partial, float* db_partial, int num_partials,
                                       const float* bn_Z, const float* bn_mask,
                                       const float* bn_scale, const float* bn_shift,
                                       const float* bn_mean, const float* bn_invstd,
                                       double* gstats_part, const double* bn_sums, double count,
                                       int training, void* stream) {
  if (M < 0 || !dW_partial || !lgnn_tile_fits(M, K, N)) return LGNN_EINVAL;
  if (num_partials != lgnn_tile_partials(M)) return LGNN_EINVAL;
  if (M > 0 && (!dY || !X)) return LGNN_EINVAL;
  if (dXpre && !planes_t) return LGNN_EINVAL;
  if (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU) return LGNN_EINVAL;
  if (act == LGNN_ACT_ELU && !H) return LGNN_EINVAL;
  if (bn_mode != BN_NONE && bn_mode != BN_GSTATS && bn_mode != BN_GIN) return LGNN_EINVAL;
  if (bn_mode != BN_NONE && (!bn_Z || !bn_scale || !bn_shift || !bn_mean || !bn_invstd))
    return LGNN_EINVAL;
  if (bn_mode == BN_GSTATS && (!dXpre || !gstats_part)) return LGNN_EINVAL;
  if (bn_mode == BN_GIN && (act != LGNN_ACT_NONE || (training && (!bn_sums || count <= 0.0))))
    return LGNN_EINVAL;
  BnFuse bn = {};
  bn.part = gstats_part;
  bn.scale = bn_scale;
  bn.shift = bn_shift;
  bn.mean = bn_mean;
  bn.invstd = bn_invstd;
  bn.Z = bn_Z;
  bn.mask = bn_mask;
  bn.sums = bn_sums;
  bn.count = count;
  bn.training = training;
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    if (hipMemsetAsync(dW_partial, 0, (size_t)num_partials * N * K * 4, s) != hipSuccess ||
        (db_partial && hipMemsetAsync(db_partial, 0, (size_t)num_partials * N * 4, s)) ||
        (gstats_part &&
         hipMemsetAsync(gstats_part, 0, (size_t)num_partials * 2 * K * sizeof(double), s)))
      return (int)hipGetLastError();
    return LGNN_OK;
  }
  const dim3 grid((unsigned)num_partials);
#define LGNN_S3B(AC, D, BM)                                                                   \
  hipLaunchKernelGGL((k_s3_lin_bwd<AC, D, BM>), grid, dim3(NT), 0, s, dY, H, X, M, K,        \
                     planes_t, N, dXpre, dW_partial, db_partial, bn)
  if (bn_mode == BN_GSTATS) {
    if (act == LGNN_ACT_ELU) LGNN_S3B(LGNN_ACT_ELU, true, BN_GSTATS);
    else LGNN_S3B(LGNN_ACT_NONE, true, BN_GSTATS);
  } else if (bn_mode == BN_GIN) {
    if (dXpre) LGNN_S3B(LGNN_ACT_NONE, true, BN_GIN);
    else LGNN_S3B(LGNN_ACT_NONE, false, BN_GIN);
  } else if (act == LGNN_ACT_ELU) {
    if (dXpre) LGNN_S3B(LGNN_ACT_ELU, true, BN_NONE);
    else LGNN_S3B(LGNN_ACT_ELU, false, BN_NONE);
  } else {
    if (dXpre) LGNN_S3B(LGNN_ACT_NONE, true, BN_NONE);
    else LGNN_S3B(LGNN_ACT_NONE, false, BN_NONE);
  }
#undef LGNN_S3B
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}
