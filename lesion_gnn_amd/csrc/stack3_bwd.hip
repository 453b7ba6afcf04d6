// Split-3 backward of the fused GCN stack (closed tiles), one launch per layer ("layer-major"):
// the GEMMs on bf16 MFMA at fp32 accuracy exactly as the forward (stack3.hip: three-plane
// operands, six products, three when Â is exact in bf16). Autograd of PyG's GCNConv
// (out = Â (H W^T) + b, torch_geometric/nn/conv/gcn_conv.py) + the model's F.elu, per layer l:
//   G = Â^T dZ_l,   dW_l += G^T H_{l-1},   db_l += colsum dZ_l,
//   dZ_{l-1} = (G W_l) ⊙ ELU'(H_{l-1})        (no ELU' below the first conv: in_proj has none)
// and for in_proj (mode LIN) dW_0 += dZ_0^T X, db_0 += colsum dZ_0.
//
// Layouts (4 waves; wave w owns features [32w, 32w + 32) of dZ / G / dW rows and of dH columns):
//   P layout   accumulator with the feature on the lane and 32 nodes in its 16 registers (two
//              accumulators per 64-node tile): dZ_l is loaded straight into it; as an MFMA operand
//              it contracts over nodes with no LDS round trip (perm16 node order)
//   Z^T layout the node on the lane, four consecutive features per register group
// Per tile: G (P layout) = Â^T dZ and G^T (Z^T layout) = dZ^T Â both from the dZ registers and the
// tile's Â^T planes (LDS); H_{l-1} is staged feature-major in LDS ([k][perm16 m]) so that dW_l =
// G^T H_{l-1} takes G from registers and H from the image, for all 128 k, into dW accumulators that
// stay in registers over the workgroup's tiles (64 VGPRs) and are written once as partial slot
// blockIdx.x; G^T is then written node-major ([m][perm16 n]) and dH = G W_l runs like the
// forward's GEMM1 with the transposed weight planes (k_wplanes WpT). dZ_{l-1} goes to HBM in P
// layout (feature on the lane: 128-B row segments) for the next launch.
#include <cstdlib>
#include "common.h"
#include "tile.h"
#include "tile_util.h"
#include "s3_util.h"
#include "tile_lw.h"

namespace lgnn_s3 {

constexpr int BM_POOL = 0;  // top conv: dZ_L = pool broadcast of dP (/ |graph|), times ELU'(H_L)
constexpr int BM_CONV = 1;  // lower conv: dZ_l from HBM (the previous launch applied ELU')
constexpr int BM_LIN = 2;   // in_proj: dW_0 = dZ_0^T X, db_0 only

struct BwdLayerArgs {
  const float* dZin;      // dZ_l [M][N] (CONV, LIN) or dP [B][N] (POOL)
  const int64_t* batch;   // POOL
  const int32_t* gptr;    // POOL
  int pool_mean;          // POOL
  int64_t num_graphs;     // POOL
  const float* Hout;      // H_l [M][N] (POOL: ELU'(H_L))
  const float* Hin;       // H_{l-1} [M][K], or X for LIN
  const uint16_t* WpT;    // transposed planes of W_l, fragment order (POOL, CONV)
  float* dZout;           // dZ_{l-1} [M][K] (POOL, CONV)
  float* dWp;             // [P][N][K]
  float* dbp;             // [P][N]
  int N, K;               // out / in width of layer l (<= 128)
  int elu_prev;           // dZ_{l-1} = dH * ELU'(H_{l-1})
};

struct BwdSmem {
  unsigned char Img[3][TM * AROW];  // 48 KiB: H_{l-1} feature-major [k][perm16 m] (128 rows of
                                    // 128 B), then G node-major [m][perm16 n] (64 rows of 256 B)
  unsigned char Adj[3][ADJ_PLANE];  // 27 KiB: Â^T planes [source m][perm16 target]; the first
                                    // 16 KiB hold it in fp32 while it is summed
  float pscale[TM];                 // POOL: 1 / |graph| (mean) or 1, per tile row (0 past M)
  int pg[TM];                       // POOL: graph id per tile row
  int rp[TM + 1];
  int flag;
};

// Feature-major image: row k (128 B = 64 nodes), 16-B chunk XOR-swizzled by (k >> 1) & 7 (a b128
// read of one chunk by 16 consecutive rows is conflict-free).
__device__ __forceinline__ int hf_chunk(int k, int c) { return k * 128 + ((c ^ ((k >> 1) & 7)) << 4); }
__device__ __forceinline__ int hf_off(int k, int m4) {
  const int p = perm16(m4 & 15) + (m4 & ~15);
  return hf_chunk(k, p >> 3) + ((p & 7) << 1);
}

// A tile of a [rows][ld] fp32 matrix in P layout: lane column `colv` (< ncols, else 0), node rows
// m = 32 a + (r & 3) + 8 (r >> 2) + 4h of the tile (rows past the buffer read 0).
__device__ __forceinline__ void load_p(f32x16 (&v)[2], Buf b, int64_t r0, int ld, int colv,
                                       int ncols, int h) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int off = colv < ncols ? (int)(((r0 + m) * ld + colv) * 4) : INT32_MAX - 3;
      v[a][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b, off, 0, 0));
    }
}

// load_p with the descriptor based at the tile's first row: one lane-base VGPR, and each of the
// 32 loads adds a wave-uniform row offset (one VALU add instead of 64-bit address arithmetic).
// Rows past M fall outside the descriptor's range and read 0.
__device__ __forceinline__ void load_pt(f32x16 (&v)[2], const float* base, int64_t M, int64_t r0,
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
      v[a][r] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(b, vb + mc * rs, 0, 0));
    }
}

// P-layout pair -> node-step operand fragments (s = 0, 1 from v[0], 2, 3 from v[1])
__device__ __forceinline__ void split_p(const f32x16 (&v)[2], u32x4 (&o)[4][3]) {
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

// Two workgroups per CU (77 KB LDS, 256 VGPRs each). Tried: one 512-thread workgroup whose
// two 4-wave halves take a tile each and combine their dW at the end (half the partial slots):
// the halves' lockstep barriers cost more (+30 %) than the slab traffic saved.
template <int MODE>
__global__ __launch_bounds__(NT, 2) void k_s3_bwd(const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col,
                                                  const float* __restrict__ w, int64_t M,
                                                  BwdLayerArgs a, const int32_t* __restrict__ tmask) {
  constexpr bool AGG = MODE != BM_LIN;
  __shared__ __attribute__((aligned(16))) BwdSmem sm;
  const int64_t ntiles = (M + TM - 1) / TM;
  float* const scr = reinterpret_cast<float*>(sm.Adj[0]);  // fp32 Â^T [source][target]
  const int N = a.N, K = a.K;
  const Buf bZ = mkbuf(a.dZin, MODE == BM_POOL ? a.num_graphs * N * 4 : M * N * 4);
  const Buf bHo = mkbuf(a.Hout, MODE == BM_POOL ? M * N * 4 : 0);
  const Buf bHi = mkbuf(a.Hin, M * K * 4);
  const Buf bZo = mkbuf(a.dZout, AGG ? M * K * 4 : 0);

  f32x16 dw[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) dw[kb] = f32x16{};
  float dbacc = 0.f;
  IdxRegs R;
  int64_t t = seek_tile(blockIdx.x, ntiles, tmask, 0);
  if (AGG && t < ntiles) {
    idx_load_head(R, rowptr, M, t * TM);
    idx_load_body(R, col, w);
  }
  for (; t < ntiles;) {
    const int64_t r0 = t * TM;
    const int64_t tn = seek_tile(t + gridDim.x, ntiles, tmask, 0);
    const bool has_next = tn < ntiles;
    {
      const int tq = fresh_tid();
      if (AGG) {
#pragma unroll
        for (int i = 0; i < TM * TM / 4 / NT; ++i) st4(scr + 4 * (tq + i * NT), zero4());
        if (tq <= TM) sm.rp[tq] = R.rp;
        if (tq == 0) sm.flag = 0;
      }
      if (MODE == BM_POOL && tq < TM) {
        const int64_t row = r0 + tq;
        const int64_t g = row < M ? a.batch[row] : 0;
        const int cnt = a.gptr[g + 1] - a.gptr[g];
        sm.pg[tq] = (int)g;
        sm.pscale[tq] = row >= M ? 0.f : (a.pool_mean && cnt > 1 ? 1.f / (float)cnt : 1.f);
      }
    }
    lds_barrier();
    if (AGG) {
      adj_scatter<true>(scr, sm.rp, R, r0, col, w);
      if (has_next) idx_load_head(R, rowptr, M, tn * TM);
    }
    // dZ_l in P layout (feature n = 32 wave + li on the lane)
    f32x16 dz[2];
    {
      const int tq = fresh_tid();
      const int h = (tq >> 5) & 1, n = 32 * (tq >> 6) + (tq & 31);
      if (MODE == BM_POOL) {
        f32x16 hv[2];
        load_p(hv, bHo, r0, N, n, N, h);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int off = n < N ? (sm.pg[m] * N + n) * 4 : INT32_MAX - 3;
            const float gv =
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(bZ, off, 0, 0));
            dz[q][r] = gv * sm.pscale[m] * elu_grad_from_out(hv[q][r]);
          }
      } else {
        load_p(dz, bZ, r0, N, n, N, h);
      }
      // db_l: this lane's 32 nodes, then the partner half's
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += dz[q][r];
      s += __shfl_xor(s, 32, 64);
      dbacc += s;
    }
    u32x4 dzp[4][3];
    split_p(dz, dzp);
    f32x16 g[2], gt[2];
    if (AGG) {
      lds_barrier();  // Â^T summed
      f32x4 av[4];
      {
        const int tq = fresh_tid();
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = ld4(scr + (tq >> 2) * TM + 16 * (tq & 3) + 4 * i);
      }
      lds_barrier();  // every scratch read done
      int inexact = 0;
      {
        const int tq = fresh_tid();
        const int am = tq >> 2, aq = tq & 3;
        float f[16];
#pragma unroll
        for (int y = 0; y < 16; ++y) {
          const int src = perm16(y);
          f[y] = av[src >> 2][src & 3];
        }
        uint32_t q[3][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const Split2 s2 = split2(f[2 * i], f[2 * i + 1]);
#pragma unroll
          for (int p = 0; p < 3; ++p) q[p][i] = s2.p[p];
          inexact |= (s2.p[1] | s2.p[2]) != 0;
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          unsigned char* dst = sm.Adj[p] + am * ADJ_LD * 2 + 32 * aq;
          *reinterpret_cast<u32x4*>(dst) = u32x4{q[p][0], q[p][1], q[p][2], q[p][3]};
          *reinterpret_cast<u32x4*>(dst + 16) = u32x4{q[p][4], q[p][5], q[p][6], q[p][7]};
        }
      }
      if (inexact) sm.flag = 1;
      lds_barrier();
      const bool exact = sm.flag == 0;
      if (has_next) idx_load_body(R, col, w);
      // G = Â^T dZ (P layout: A = Â^T rows m, B = dZ) and G^T = dZ^T Â (Z^T layout: A = dZ,
      // B = Â^T rows m as columns), both over the 64 target nodes i (four k-steps)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        g[q] = f32x16{};
        gt[q] = f32x16{};
      }
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int off = (32 * q + li) * ADJ_LD * 2 + 16 * (2 * s + h);
            if (exact) {
              const u32x4 at0 = lds16(sm.Adj[0] + off);
              g[q] = mfma_s3_aexact(at0, dzp[s], g[q]);
              gt[q] = mfma_s3_bexact(dzp[s], at0, gt[q]);
            } else {
              u32x4 at[3];
#pragma unroll
              for (int p = 0; p < 3; ++p) at[p] = lds16(sm.Adj[p] + off);
              g[q] = mfma_s3(at, dzp[s], g[q]);
              gt[q] = mfma_s3(dzp[s], at, gt[q]);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
      g[0] = dz[0];
      g[1] = dz[1];
    }
    // H_{l-1} (X for in_proj) in P layout, feature k = 32 wave + li: -> feature-major image
    f32x16 hp[2];
    {
      const int tq = fresh_tid();
      const int h = (tq >> 5) & 1, li = tq & 31, k = 32 * (tq >> 6) + li;
      load_p(hp, bHi, r0, K, k, K, h);
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          u32x2 o[3];
          split4(f32x4{hp[q][4 * gq], hp[q][4 * gq + 1], hp[q][4 * gq + 2], hp[q][4 * gq + 3]}, o);
          const int off = hf_off(k, 32 * q + 8 * gq + 4 * h);
#pragma unroll
          for (int p = 0; p < 3; ++p) sts8(sm.Img[p] + off, o[p]);
        }
    }
    lds_barrier();  // H image complete (and, LIN, nothing else)
    // dW_l += G^T H: A = G (P layout, node steps), B = H image rows k = 32 kb + li
    {
      u32x4 gp[4][3];
      split_p(g, gp);
      const int tq = fresh_tid();
      const int h = (tq >> 5) & 1, li = tq & 31;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          u32x4 hb[3];
          const int off = hf_chunk(32 * kb + li, 2 * s + h);
#pragma unroll
          for (int p = 0; p < 3; ++p) hb[p] = lds16(sm.Img[p] + off);
          dw[kb] = mfma_s3(gp[s], hb, dw[kb]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (AGG) {
      lds_barrier();  // every read of the H image done
      // G^T (Z^T layout: node m on the lane, features 32 wave + 8 gq + 4h + 0..3) -> node-major
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31, wv = tq >> 6;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            u32x2 o[3];
            split4(f32x4{gt[q][4 * gq], gt[q][4 * gq + 1], gt[q][4 * gq + 2], gt[q][4 * gq + 3]},
                   o);
            const int off = ap_off(32 * q + li, 32 * wv + 8 * gq + 4 * h);
#pragma unroll
            for (int p = 0; p < 3; ++p) sts8(sm.Img[p] + off, o[p]);
          }
      }
      lds_barrier();
      // dH = G W_l (P layout: feature k on the lane): A = G image rows m, B = W_l^T planes
      f32x16 dh[2] = {f32x16{}, f32x16{}};
      {
        u32x4 wf[3][8];
        const int tq = fresh_tid();
        const int lane = tq & 63, wv = tq >> 6, h = lane >> 5, li = lane & 31;
        const uint16_t* base = a.WpT + wv * 8 * 512 + lane * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int s = 0; s < 8; ++s)
            wf[p][s] = *reinterpret_cast<const u32x4*>(base + p * PLANE + 512 * s);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            u32x4 f[3];
            const int off = ap_chunk(32 * q + li, 2 * s + h);
#pragma unroll
            for (int p = 0; p < 3; ++p) f[p] = lds16(sm.Img[p] + off);
            u32x4 b[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) b[p] = wf[p][s];
            dh[q] = mfma_s3(f, b, dh[q]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // dZ_{l-1} = dH * ELU'(H_{l-1}) -> HBM (P layout: feature k on the lane)
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, k = 32 * (tq >> 6) + (tq & 31);
        if (a.elu_prev) load_p(hp, bHi, r0, K, k, K, h);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float v = a.elu_prev ? dh[q][r] * elu_grad_from_out(hp[q][r]) : dh[q][r];
            const int off = k < K ? (int)(((r0 + m) * K + k) * 4) : INT32_MAX - 3;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), bZo, off, 0, 0);
          }
      }
    }
    t = tn;
  }
  // partial slot blockIdx.x: dW rows n = 32 wave + (r & 3) + 8 (r >> 2) + 4h, columns
  // k = 32 kb + li; db from the h = 0 lanes (both halves' sums)
  {
    const int tq = threadIdx.x;
    const int h = (tq >> 5) & 1, li = tq & 31, wv = tq >> 6;
    float* slab = a.dWp + (int64_t)blockIdx.x * N * K;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int k = 32 * kb + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = 32 * wv + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (n < N && k < K) slab[(int64_t)n * K + k] = dw[kb][r];
      }
    }
    const int n = 32 * wv + li;
    if (h == 0 && n < N) a.dbp[(int64_t)blockIdx.x * N + n] = dbacc;
  }
}

}  // namespace lgnn_s3

extern "C" int lgnn_gcn_stack_bwd_s3_partials(int64_t M) {
  if (M < 0) return LGNN_EINVAL;
  const int64_t ntiles = (M + lgnn_tile::TM - 1) / lgnn_tile::TM;
  const int64_t p = ntiles < 512 ? ntiles : 512;
  return (int)(p < 1 ? 1 : p);
}

extern "C" int lgnn_gcn_stack_bwd_s3(const float* dP, const int64_t* batch, const int32_t* gptr,
                                     int pool_mean, int64_t num_graphs, const int32_t* rowptr,
                                     const int32_t* col, const float* w, const float* X,
                                     int64_t M, int L, const uint16_t* planes_t,
                                     const float* const* H, const int* widths,
                                     float* const* dWp, float* const* dbp, int num_partials,
                                     float* dz_ws, const int32_t* tile_open, void* stream) {
  if (M < 0 || L < 1 || L + 1 > LGNN_MAX_STACK || !dP || !batch || !gptr || !rowptr || !col ||
      !X || !planes_t || !H || !widths || !dWp || !dbp || !dz_ws || !tile_open || num_graphs < 0)
    return LGNN_EINVAL;
  if (num_partials != lgnn_gcn_stack_bwd_s3_partials(M)) return LGNN_EINVAL;
  for (int l = 0; l <= L; ++l) {
    if (!lgnn_tile_fits(M, widths[l], widths[l + 1]) || !H[l] || !dWp[l] || !dbp[l])
      return LGNN_EINVAL;
  }
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    for (int l = 0; l <= L; ++l)
      if (hipMemsetAsync(dWp[l], 0, (size_t)widths[l] * widths[l + 1] * 4, s) != hipSuccess ||
          hipMemsetAsync(dbp[l], 0, (size_t)widths[l + 1] * 4, s) != hipSuccess)
        return (int)hipGetLastError();
    return LGNN_OK;
  }
  float* dz[2] = {dz_ws, dz_ws + M * lgnn_s3::WP};
  const dim3 grid((unsigned)num_partials), blk(lgnn_tile::NT);
  for (int l = L; l >= 0; --l) {
    lgnn_s3::BwdLayerArgs a = {};
    a.N = widths[l + 1];
    a.K = widths[l];
    a.dWp = dWp[l];
    a.dbp = dbp[l];
    a.Hin = l >= 1 ? H[l - 1] : X;
    if (l == L) {
      a.dZin = dP;
      a.batch = batch;
      a.gptr = gptr;
      a.pool_mean = pool_mean;
      a.num_graphs = num_graphs;
      a.Hout = H[L];
    } else {
      a.dZin = dz[(L - 1 - l) & 1];
    }
    if (l >= 1) {
      a.WpT = planes_t + (size_t)l * 3 * lgnn_s3::PLANE;
      a.dZout = dz[(L - l) & 1];
      a.elu_prev = l >= 2;
    }
    if (l == L)
      hipLaunchKernelGGL(lgnn_s3::k_s3_bwd<lgnn_s3::BM_POOL>, grid, blk, 0, s, rowptr, col, w, M,
                         a, tile_open);
    else if (l >= 1)
      hipLaunchKernelGGL(lgnn_s3::k_s3_bwd<lgnn_s3::BM_CONV>, grid, blk, 0, s, rowptr, col, w, M,
                         a, tile_open);
    else
      hipLaunchKernelGGL(lgnn_s3::k_s3_bwd<lgnn_s3::BM_LIN>, grid, blk, 0, s, rowptr, col, w, M,
                         a, tile_open);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return LGNN_OK;
}

namespace lgnn_s3 {

// ==============================================================================================
// Fused split-3 backward: every layer of a tile in one pass (tile-major), one launch.
//
// Same arithmetic and layouts as k_s3_bwd above, with the layer loop inside the tile loop:
//   * the tile's Â^T planes are built once and serve every conv layer;
//   * dZ stays in registers (P layout) from one layer to the next: dH = G W_l comes out of its
//     MFMAs in exactly the layout the next layer's dZ is consumed in, so no HBM round trip;
//   * the dW accumulators of ALL layers stay in registers over the workgroup's tiles (64 per
//     layer per lane; the MFMA accumulators live in AGPRs at one wave per SIMD) and are written
//     once as partial slot blockIdx.x — one workgroup per CU, the fp32 kernel's 256 slots;
//   * G^T has its own LDS image, so the H image of the dW product and the G^T image of the dH
//     product coexist (two barriers per conv layer);
//   * the next tile's CSR block is prefetched during the current tile (idx head/body), and the
//     next layer's H_{l-1} rows are issued before the current layer's G products.
// Per tile HBM traffic: H_L, H_{L-1}, ..., H_0, X read once (the algorithmic bytes).
// ==============================================================================================

// scheduling fence between MFMA groups: none by default (the compiler interleaves the groups'
// LDS reads and MFMAs freely: 122 -> 113 us at C2, tools/stamps_s3f.py); -DLGNN_S3F_SB restores
// a sched_barrier after each group
#ifdef LGNN_S3F_SB
#define S3F_SB() __builtin_amdgcn_sched_barrier(0)
#else
#define S3F_SB() \
  do {           \
  } while (0)
#endif

struct FBwdArgs {
  const float* dP;                // [B][N_L] pooled-output gradient (or formed from dlog / Wout)
  const float* dlog;              // [B][C] logits gradient (nullable): dP = dlog Wout on the fly
  CeSrc ce;                       // or (ce.pm set) the CE logits gradient, formed on the fly
  const float* Wout;              // [C][N_L]
  int C;
  const unsigned char* adjt;      // Â^T planes per tile from the forward (AG), or nullptr
  const int64_t* batch;
  const int32_t* gptr;
  int pool_mean;
  int64_t num_graphs;
  const float* X;                 // model input (in_proj dW operand)
  const float* H[LGNN_MAX_STACK];  // H[l] = output of layer l
  const uint16_t* WpT;            // transposed weight planes, [l][3][PLANE] fragment order
  float* dWp[LGNN_MAX_STACK];     // [P][N_l][K_l]
  float* dbp[LGNN_MAX_STACK];     // [P][N_l]
  int width[LGNN_MAX_STACK + 1];
  float* dZ0;                     // XIN: [M][N_0] in_proj output gradient (dWp[0] / dbp[0] unused)
};

// Open-tile phase of the fused backward (optional): after this workgroup wrote its partial
// slots, the open tiles run layer by layer on the fp32 layer-wise bodies (tile_lw.h), adding into
// the same slots (program order: no race), a grid barrier between layers (layer l - 1 gathers
// layer l's pre-aggregation gradient dS through the transposed CSR).
struct OpenBwdArgs {
  const float* W[LGNN_MAX_STACK];  // fp32 weights
  const float* S[LGNN_MAX_STACK];  // S[l - 1]: the forward's saved aggregated inputs (open tiles)
  float* dS[2];                    // ping-pong [M][128] pre-aggregation gradients
  const int32_t* tptr;             // transpose CSR
  const int32_t* tidx;
  const float* tw;
  int32_t* sync;                   // grid-barrier words (nullptr: no open phase)
};

constexpr int kMaxHeadC = 8;  // classes for which dP is formed in the kernel

// the logits gradient row of graph g: given (dlog) or formed from the CE forward (ce)
__device__ __forceinline__ bool has_head(const FBwdArgs& a) { return a.dlog || a.ce.pm; }
// the raw per-graph value loaded a tile ahead: dlog, or CE's pm (the factor gloss * wt / wsum is
// applied where the row is used, so that the prefetch stays a plain load nothing waits on)
__device__ __forceinline__ float head_raw(const FBwdArgs& a, int64_t g, int c) {
  return a.ce.pm ? a.ce.pm[g * a.C + c] : a.dlog[g * a.C + c];
}
// the logits gradient from the raw value: ce_dlogit's expression, bit for bit
__device__ __forceinline__ float head_dl(const FBwdArgs& a, float raw, float wt, float gl,
                                         float ws) {
  return a.ce.pm ? ce_grad(gl, wt, ws, raw) : raw;
}

struct FBwdSmem {
  unsigned char Img[3][TM * AROW];  // 48 KiB: H_{l-1} (or X) feature-major [k][perm16 m]
  unsigned char Gt[3][TM * AROW];   // 48 KiB: G node-major [m][perm16 n]
  unsigned char Adj[3][ADJ_PLANE];  // 27 KiB: Â^T planes; first 16 KiB fp32 while summed
  float pscale[TM];
  int pg[TM];
  int rp[TM + 1];
  int flag;
  __attribute__((aligned(16))) float dl[TM][kMaxHeadC];  // dlog rows of the tile's graphs, pre-scaled by pscale
  // 32 KiB: the tile's H_L rows ([row][N_L] fp32, contiguous as in HBM), loaded direct-to-LDS
  // during the previous tile so the prologue's dZ_L needs no global round trip
  __attribute__((aligned(16))) float hl[TM * WP];
};
static_assert(sizeof(FBwdSmem) <= 160 * 1024, "fused backward LDS exceeds the CU's 160 KiB");

// the tile's fp32 Â [target][source] (the forward's sum) straight into the scratch: 16 wave loads
// of 1 KiB, no registers, completion by vmcnt
__device__ __forceinline__ void adj_issue(FBwdSmem& sm, const unsigned char* adjt, int64_t t) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Buf rs = mkbuf(adjt + t * ADJT_TILE_BYTES, ADJT_TILE_BYTES);
  for (int c = wave; c < ADJT_TILE_BYTES / 1024; c += NT / 64)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(&sm.Adj[0][0] + c * 1024), 16,
        c * 1024 + lane * 16, 0, 0, 0);
}

// tile t's H_L rows (ld floats each, contiguous) straight into sm.hl: 1 KiB wave loads, no
// registers, completion by vmcnt; rows past M are not read (the prologue masks them)
__device__ __forceinline__ void hl_issue(FBwdSmem& sm, const float* H, int64_t M, int64_t t,
                                         int ld) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r0 = t * TM;
  const int64_t rows = M - r0 < TM ? M - r0 : TM;
  const Buf rs = mkbuf(H + r0 * ld, rows * ld * 4);
  const int nch = (TM * ld * 4 + 1023) >> 10;  // <= 32: sm.hl holds TM * WP floats
  for (int c = wave; c < nch; c += NT / 64)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(reinterpret_cast<unsigned char*>(sm.hl) +
                                                      c * 1024),
        16, c * 1024 + lane * 16, 0, 0, 0);
}

// 4 x 4 transpose inside each quad of lanes (DPP): lane i's v[k] -> lane k's v[i]
__device__ __forceinline__ float dpp_quad(float x, int ctrl_xor) {
  const int xi = __builtin_bit_cast(int, x);
  return __builtin_bit_cast(float, ctrl_xor == 1 ? __builtin_amdgcn_mov_dpp(xi, 0xB1, 0xF, 0xF, false)
                                                 : __builtin_amdgcn_mov_dpp(xi, 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ void quad_transpose(float (&v)[4], int qi) {
  const bool b0 = qi & 1, b1 = qi & 2;
#pragma unroll
  for (int k = 0; k < 4; k += 2) {  // exchange at distance 1
    const float r = dpp_quad(b0 ? v[k] : v[k + 1], 1);
    if (b0) v[k] = r; else v[k + 1] = r;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // exchange at distance 2
    const float r = dpp_quad(b1 ? v[k] : v[k + 2], 2);
    if (b1) v[k] = r; else v[k + 2] = r;
  }
}

// The same 4 x 4 transpose on bf16 planes: lane qi holds feature qi of nodes 0, 1 (w0) and
// 2, 3 (w1) as packed pairs; returns node qi's features 0, 1 and 2, 3 as packed pairs (one
// exchange of 2 x 2 bf16 blocks with lane qi ^ 1 by v_perm, then of words with lane qi ^ 2)
__device__ __forceinline__ u32x2 quad_transpose_bf16(uint32_t w0, uint32_t w1, int qi) {
  const uint32_t sel = (qi & 1) ? 0x03020706u : 0x05040100u;
  const uint32_t p0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)w0, 0xB1, 0xF, 0xF, false);
  const uint32_t p1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)w1, 0xB1, 0xF, 0xF, false);
  const uint32_t a = __builtin_amdgcn_perm(p0, w0, sel);
  const uint32_t b = __builtin_amdgcn_perm(p1, w1, sel);
  const bool b1 = qi & 2;
  const uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)(b1 ? a : b), 0x4E, 0xF, 0xF, false);
  return u32x2{b1 ? r : a, b1 ? b : r};
}

// Â^T planes of a tile from the fp32 scratch the forward handed over (AG): each thread reads its
// 16 targets of one source row (a wave reads 64 different banks) and splits them into the three
// planes; adj_write (after a barrier: the planes overwrite the scratch) stores them
struct AdjPlanes {
  uint32_t q[3][8];
};
__device__ __forceinline__ AdjPlanes adj_split(FBwdSmem& sm) {
  const float* scr = reinterpret_cast<const float*>(sm.Adj[0]);
  const int tq = fresh_tid();
  const int am = tq & 63, aq = tq >> 6;
  float f[16];
#pragma unroll
  for (int y = 0; y < 16; ++y) f[y] = scr[(16 * aq + perm16(y)) * TM + am];
  AdjPlanes o;
  uint32_t inexact = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const Split2 s2 = split2(f[2 * i], f[2 * i + 1]);
#pragma unroll
    for (int p = 0; p < 3; ++p) o.q[p][i] = s2.p[p];
    inexact |= s2.p[1] | s2.p[2];
  }
  // sm.flag: set when some Â weight of the tile is inexact in bf16 (cleared before)
  if (__any(inexact != 0) && (tq & 63) == 0) sm.flag = 1;
  return o;
}
__device__ __forceinline__ void adj_write(FBwdSmem& sm, const AdjPlanes& o) {
  const int tq = fresh_tid();
  const int am = tq & 63, aq = tq >> 6;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    unsigned char* dst = sm.Adj[p] + am * ADJ_LD * 2 + 32 * aq;
    *reinterpret_cast<u32x4*>(dst) = u32x4{o.q[p][0], o.q[p][1], o.q[p][2], o.q[p][3]};
    *reinterpret_cast<u32x4*>(dst + 16) = u32x4{o.q[p][4], o.q[p][5], o.q[p][6], o.q[p][7]};
  }
}

// AG: the next tile's Â^T planes are split during this tile's in_proj phase (VALU and LDS work
// beside the dW_0 MFMAs) instead of in the next tile's prologue; -DLGNN_S3F_NOPIPE: in the
// prologue (the round-3 order; A/B builds only)
#ifdef LGNN_S3F_NOPIPE
constexpr bool kAdjPipe = false;
#else
constexpr bool kAdjPipe = true;
#endif

// The open-tile gather of the in_proj gradient for XIN launches: dZ_0 rows of the open tiles
// = Â^T dS_1 through the transposed CSR (one wave per row, two features per lane)
__device__ __forceinline__ void open_dz0(float* __restrict__ dZ0, const float* __restrict__ dS,
                                         const int32_t* __restrict__ tptr,
                                         const int32_t* __restrict__ tidx,
                                         const float* __restrict__ tw, int64_t M, int N,
                                         const int32_t* __restrict__ tmask) {
  const int64_t ntiles = (M + TM - 1) / TM;
  const int c = 2 * (threadIdx.x & 63), wave = threadIdx.x >> 6;
  for (int64_t t = seek_tile(xcd_block(), ntiles, tmask, 1); t < ntiles;
       t = seek_tile(t + gridDim.x, ntiles, tmask, 1)) {
    for (int rr = wave; rr < TM; rr += NT / 64) {
      const int64_t row = t * TM + rr;
      if (row >= M) break;
      float a0 = 0.f, a1 = 0.f;
      const int j1 = tptr[row + 1];
      for (int j = tptr[row]; j < j1; ++j) {
        const float wgt = tw[j];
        const int64_t src = tidx[j];
        if (c < N) {
          a0 += wgt * dS[src * N + c];
          a1 += wgt * dS[src * N + c + 1];
        }
      }
      if (c < N) {
        dZ0[row * N + c] = a0;
        dZ0[row * N + c + 1] = a1;
      }
    }
  }
}

// XIN (NL = 4: in_proj + 3 convs): the in_proj weight gradient is not accumulated here — three
// layers of dW fill the accumulator registers (192 of 512 per lane at one wave per SIMD), a fourth
// would spill — the kernel writes dZ_0 (the in_proj output gradient) instead and the caller forms
// dW_0 = dZ_0^T X, db_0 = colsum dZ_0 with one split-3 weight-gradient GEMM (lgnn_s3_wgrad)
template <int NL, bool AG, bool XIN = false>
__global__ __launch_bounds__(NT, 1) void k_s3_fbwd(const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ col,
                                                   const float* __restrict__ w, int64_t M,
                                                   FBwdArgs a, const int32_t* __restrict__ tmask,
                                                   OpenBwdArgs o) {
  constexpr int L = NL - 1;
  constexpr int ND = XIN ? NL - 1 : NL;  // layers whose dW is accumulated here
  __shared__ __attribute__((aligned(16))) FBwdSmem sm;
  const int64_t ntiles = (M + TM - 1) / TM;
  float* const scr = reinterpret_cast<float*>(sm.Adj[0]);  // fp32 Â^T [source][target]
  const int NLast = a.width[L + 1];
  const Buf bP = mkbuf(a.dP, a.num_graphs * NLast * 4);

  f32x16 dw[ND][4];
#pragma unroll
  for (int l = 0; l < ND; ++l)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) dw[l][kb] = f32x16{};
  float dbacc[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) dbacc[l] = 0.f;

  IdxRegs R;
  [[maybe_unused]] int stamp = 0;
  int64_t t = seek_tile(blockIdx.x, ntiles, tmask, 0);
  // a workgroup with no closed tile writes no partial slot when separate open-tile launches
  // follow (no o.sync): it sets its skip word instead, and those launches write the slot (C5:
  // nearly every tile open, 49.5 MB of zero slabs no longer written)
  const bool write_slots = t < ntiles || o.sync != nullptr || blockIdx.x >= LGNN_SLOT_FLAGS;
  if (!o.sync && blockIdx.x < LGNN_SLOT_FLAGS && threadIdx.x == 0)
    const_cast<int32_t*>(tmask)[ntiles + LGNN_SLOT_FLAG0 + blockIdx.x] = write_slots ? 0 : 1;
  // graph of row tq of the tile and its size (tq < TM), loaded a tile ahead
  int64_t pre_g = 0;
  int pre_cnt = 0;
  float pre_dl[kMaxHeadC];  // dlog (or CE pm) row of pre_g (tq < TM), loaded a tile ahead
  float pre_wt = 0.f;       // CE: wt[pre_g]
  const float ce_gl = a.ce.pm ? a.ce.gloss[0] : 0.f, ce_ws = a.ce.pm ? a.ce.wsum[0] : 1.f;
#pragma unroll
  for (int c = 0; c < kMaxHeadC; ++c) pre_dl[c] = 0.f;
  // out_proj's W as the B operand of the dZ_L product (lane: feature n; K: class 8h + e; classes
  // past C, features past N_L and the h = 1 half read 0 through the buffer range), split once
  u32x4 wob[3] = {};
  if (has_head(a)) {
    const int tq = fresh_tid();
    const int h = (tq >> 5) & 1, n = 32 * (tq >> 6) + (tq & 31);
    const Buf bW = mkbuf(a.Wout, (int64_t)a.C * NLast * 4);
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      f[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           bW, (h == 0 && n < NLast) ? (e * NLast + n) * 4
                                                                     : INT32_MAX - 3, 0, 0));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const Split2 s2 = split2(f[2 * i], f[2 * i + 1]);
#pragma unroll
      for (int p = 0; p < 3; ++p) wob[p][i] = s2.p[p];
    }
  }
  if (t < ntiles) {
    hl_issue(sm, a.H[L], M, t, NLast);
    {
      const int tq = fresh_tid();
      const int64_t row = t * TM + tq;
      if (tq < TM && row < M) {
        pre_g = a.batch[row];
        pre_cnt = a.gptr[pre_g + 1] - a.gptr[pre_g];
        if (has_head(a)) {
#pragma unroll
          for (int c = 0; c < kMaxHeadC; ++c) pre_dl[c] = c < a.C ? head_raw(a, pre_g, c) : 0.f;
          if (a.ce.pm) pre_wt = a.ce.wt[pre_g];
        }
      }
    }
    if constexpr (AG) {
      adj_issue(sm, a.adjt, t);
    } else {
      idx_load_head(R, rowptr, M, t * TM);
      idx_load_body(R, col, w);
    }
  }
  if constexpr (AG && kAdjPipe) {  // the first tile's Â^T planes (later tiles': in_proj phase)
    if (t < ntiles) {
      if (fresh_tid() == 0) sm.flag = 0;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      const AdjPlanes ap = adj_split(sm);
      lds_barrier();
      adj_write(sm, ap);
    }
  }
  for (; t < ntiles;) {
    STAMP(stamp++);
    const int64_t r0 = t * TM;
    const int64_t tn = seek_tile(t + gridDim.x, ntiles, tmask, 0);
    const bool has_next = tn < ntiles;
    {
      const int tq = fresh_tid();
      if constexpr (!AG) {
#pragma unroll
        for (int i = 0; i < TM * TM / 4 / NT; ++i) st4(scr + 4 * (tq + i * NT), zero4());
        if (tq <= TM) sm.rp[tq] = R.rp;
      }
      // set below when some Â weight of the tile is inexact in bf16 (pipelined: set while the
      // previous tile split this one's planes)
      if (!(AG && kAdjPipe) && tq == 0) sm.flag = 0;
      if (tq < TM) {
        const int64_t row = r0 + tq;
        const int64_t g = pre_g;
        const int cnt = pre_cnt;
        const float ps = row >= M ? 0.f : (a.pool_mean && cnt > 1 ? 1.f / (float)cnt : 1.f);
        sm.pg[tq] = (int)g;
        sm.pscale[tq] = ps;
        if (has_head(a)) {  // zero-padded to kMaxHeadC: the dZ_L loop below runs without branches
          float v[kMaxHeadC];
#pragma unroll
          for (int c = 0; c < kMaxHeadC; ++c) v[c] = head_dl(a, pre_dl[c], pre_wt, ce_gl, ce_ws) * ps;
          st4(&sm.dl[tq][0], f32x4{v[0], v[1], v[2], v[3]});
          st4(&sm.dl[tq][4], f32x4{v[4], v[5], v[6], v[7]});
        }
      }
    }
    // this tile's H_L rows (and, AG, its Â) were issued during the previous tile: landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();  // ... in every wave; the staging above is visible
    STAMP(stamp++);
    if constexpr (!AG) {
      adj_scatter<true>(scr, sm.rp, R, r0, col, w);
      if (has_next) idx_load_head(R, rowptr, M, tn * TM);
    }
    // dZ_L = pool broadcast of dP (/ |graph|) * ELU'(H_L), P layout (feature n on the lane)
    f32x16 dz[2];
    {
      const int tq = fresh_tid();
      const int h = (tq >> 5) & 1, n = 32 * (tq >> 6) + (tq & 31);
      f32x16 hv[2];  // H_L from the LDS copy
      {
        // unconditional reads, no masks: rows past M hold zeros (hl_issue's out-of-range DMA
        // lanes write 0), and lanes past N_L read column 0 (finite), which every use below
        // multiplies by an exact 0 (W_out / dP columns past N_L read 0); conditional reads
        // compiled to exec-masked blocks with a v_mul_lo each (the phase took 6.8 k ticks)
        const int nl = __builtin_amdgcn_readfirstlane(NLast);
        const float* hb = sm.hl + 4 * h * nl + (n < nl ? n : 0);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) hv[q][r] = hb[(32 * q + (r & 3) + 8 * (r >> 2)) * nl];
      }
      if (has_head(a)) {
        // dP[g(m)][n] / |g(m)| = sum_c dl[m][c] Wout[c][n] as ONE split-3 product per node half
        // (K = the <= 8 classes, zero-padded to 16): A = the staged dl rows (node on the lane:
        // two 16-B LDS reads per half instead of 32 rows x 8 classes per lane), B = out_proj's
        // W planes (wob, split once per launch); the output is in P layout, as dZ_L is consumed
        const int li = tq & 31;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 d0 = ld4(&sm.dl[32 * q + li][0]), d1 = ld4(&sm.dl[32 * q + li][4]);
          u32x4 ad[3];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float x0 = h ? 0.f : (i < 2 ? d0[2 * i] : d1[2 * i - 4]);
            const float x1 = h ? 0.f : (i < 2 ? d0[2 * i + 1] : d1[2 * i - 3]);
            const Split2 s2 = split2(x0, x1);
#pragma unroll
            for (int p = 0; p < 3; ++p) ad[p][i] = s2.p[p];
          }
          const f32x16 gv = mfma_s3(ad, wob, f32x16{});
#pragma unroll
          for (int r = 0; r < 16; ++r) dz[q][r] = gv[r] * elu_grad_from_out(hv[q][r]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int off = n < NLast ? (sm.pg[m] * NLast + n) * 4 : INT32_MAX - 3;
            const float gv =
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(bP, off, 0, 0));
            dz[q][r] = gv * sm.pscale[m] * elu_grad_from_out(hv[q][r]);
          }
      }
    }
    STAMP(stamp++);
    if constexpr (AG) {
      // (every wave's Â loads landed before the barrier above)
      if constexpr (!kAdjPipe) {
        const AdjPlanes ap = adj_split(sm);
        lds_barrier();  // every scratch read done (the planes overwrite it)
        adj_write(sm, ap);
        lds_barrier();
      }
    } else {
    lds_barrier();  // Â^T summed
    {
      f32x4 av[4];
      {
        const int tq = fresh_tid();
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = ld4(scr + (tq >> 2) * TM + 16 * (tq & 3) + 4 * i);
      }
      lds_barrier();  // every scratch read done
      int inexact = 0;
      {
        const int tq = fresh_tid();
        const int am = tq >> 2, aq = tq & 3;
        float f[16];
#pragma unroll
        for (int y = 0; y < 16; ++y) {
          const int src = perm16(y);
          f[y] = av[src >> 2][src & 3];
        }
        uint32_t q[3][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const Split2 s2 = split2(f[2 * i], f[2 * i + 1]);
#pragma unroll
          for (int p = 0; p < 3; ++p) q[p][i] = s2.p[p];
          inexact |= (s2.p[1] | s2.p[2]) != 0;
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          unsigned char* dst = sm.Adj[p] + am * ADJ_LD * 2 + 32 * aq;
          *reinterpret_cast<u32x4*>(dst) = u32x4{q[p][0], q[p][1], q[p][2], q[p][3]};
          *reinterpret_cast<u32x4*>(dst + 16) = u32x4{q[p][4], q[p][5], q[p][6], q[p][7]};
        }
        if (__any(inexact) && (tq & 63) == 0) sm.flag = 1;
      }
      lds_barrier();
    }
    if (has_next) idx_load_body(R, col, w);
    }
    // every Â weight exact in bf16 (k-regular kNN graphs with k a power of two: 1/k): the
    // aggregation products take three plane products instead of six and read one Â plane
    const bool aexact = __builtin_amdgcn_readfirstlane(sm.flag) == 0;
    STAMP(stamp++);

    f32x16 xp[2];  // X rows of the in_proj phase (issued during the last conv's dH)
#pragma unroll
    for (int l = L; l >= 1; --l) {
      const int K = a.width[l];
      const bool elu_prev = l >= 2;
      // H_{l-1} rows (P layout, feature k on the lane): issued first, consumed by the image
      // write after the G products and by ELU' at the end of the layer
      f32x16 hp[2];
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, k = 32 * (tq >> 6) + (tq & 31);
        load_pt(hp, a.H[l - 1], (ABL & 16) ? 0 : M, r0, K, k, K, h);
      }
      // db_l: this lane's 32 nodes, then the partner half's
      {
        float sacc = 0.f;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc += dz[q][r];
        sacc += __shfl_xor(sacc, 32, 64);
        dbacc[l] += sacc;
      }
      u32x4 dzp[4][3];
      split_p(dz, dzp);
      // G = Â^T dZ (P layout)
      f32x16 g[2] = {f32x16{}, f32x16{}};
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31;
        if (aexact) {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int off = (32 * q + li) * ADJ_LD * 2 + 16 * (2 * s + h);
              const u32x4 a0 = lds16(sm.Adj[0] + off);
              if constexpr (!(ABL & 1)) g[q] = mfma_s3_aexact(a0, dzp[s], g[q]);
            }
          }
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int off = (32 * q + li) * ADJ_LD * 2 + 16 * (2 * s + h);
              u32x4 at[3];
#pragma unroll
              for (int p = 0; p < 3; ++p) at[p] = lds16(sm.Adj[p] + off);
              if constexpr (!(ABL & 1)) g[q] = mfma_s3(at, dzp[s], g[q]);
            }
            S3F_SB();
          }
        }
      }
      // G's operand planes, split once: dW's A operand below, and (transposed) the G image
      u32x4 gp[4][3];
      split_p(g, gp);
      // G -> node-major image [m][perm16 n] for dH = G W_l: each quad of lanes (4 features,
      // 4 nodes per packed pair of planes) transposes its 4 x 4 blocks of bf16 by DPP + v_perm,
      // so a lane holds four consecutive features of one node (no G^T = dZ^T Â products)
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31, wv = tq >> 6, qi = li & 3;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            // nodes 32 q + 8 j + 4 h + 0..3: node step 2 q + (j >> 1), pairs 2 (j & 1) and + 1
            const int st = 2 * q + (j >> 1), i0 = 2 * (j & 1);
            const int off = ap_off(32 * q + 8 * j + 4 * h + qi, 32 * wv + (li & ~3));
#pragma unroll
            for (int p = 0; p < 3; ++p)
              sts8(sm.Gt[p] + off, quad_transpose_bf16(gp[st][p][i0], gp[st][p][i0 + 1], qi));
          }
      }
      STAMP(stamp++);
      // H_{l-1} -> feature-major image (the previous layer's dW readers passed its barrier)
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31, k = 32 * (tq >> 6) + li;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            u32x2 o[3];
            split4(f32x4{hp[q][4 * gq], hp[q][4 * gq + 1], hp[q][4 * gq + 2], hp[q][4 * gq + 3]},
                   o);
            const int off = hf_off(k, 32 * q + 8 * gq + 4 * h);
#pragma unroll
            for (int p = 0; p < 3; ++p) sts8(sm.Img[p] + off, o[p]);
          }
      }
      // W_l^T planes for dH (L2-resident, 1 KiB per wave-load), two k-steps at a time: the first
      // pair flies during the dW products, the second from their middle on, each later pair
      // during the two before it
      const uint16_t* wbase;
      {
        const int tq = fresh_tid();
        const int lane = tq & 63, wv = tq >> 6;
        wbase = a.WpT + (size_t)l * 3 * PLANE + wv * 8 * 512 + lane * 8;
      }
      auto load_w2 = [&](u32x4 (&wf)[3][2], int pair) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
            wf[p][s2] = (ABL & 16) ? u32x4{}
                                   : *reinterpret_cast<const u32x4*>(wbase + p * PLANE +
                                                                     512 * (2 * pair + s2));
      };
      u32x4 wa[3][2], wb[3][2];
      load_w2(wa, 0);
      lds_barrier();  // both images complete
      // the last conv's Â^T reads are done: the next tile's planes load into LDS behind the
      // remaining phases of this tile
      if constexpr (AG) {
        if (l == 1 && has_next) adj_issue(sm, a.adjt, tn);
      }
      // ... and the next tile's H_L rows (the prologue's reads of sm.hl passed many barriers)
      if (l == 1 && has_next) hl_issue(sm, a.H[L], M, tn, NLast);
      if (l == 1) {  // the next tile's graph ids (their sizes follow in the in_proj phase)
        const int tq = fresh_tid();
        const int64_t row = tn * TM + tq;
        pre_g = (has_next && tq < TM && row < M) ? a.batch[row] : 0;
      }
      // this tile's X rows for the in_proj phase, in flight from the first conv's dW on (issued
      // at the last conv they crowded that phase's load queue: in-step 107.6 -> 106.0 us)
      if (!XIN && l == L) {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, k = 32 * (tq >> 6) + (tq & 31);
        load_pt(xp, a.X, (ABL & 16) ? 0 : M, r0, a.width[0], k, a.width[0], h);
      }
      STAMP(stamp++);
      // dW_l += G^T H: A = G (P layout, node steps: the planes split above), B = H image rows
      // k = 32 kb + li. Node steps outer: consecutive products go to different accumulators,
      // each accumulator still takes s = 0..3 in order, and gp[s] is dead after its step — the
      // second pair of W^T planes loads into the registers the first two steps freed
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) {
            u32x4 hb[3];
            const int off = hf_chunk(32 * kb + li, 2 * s + h);
#pragma unroll
            for (int p = 0; p < 3; ++p) hb[p] = lds16(sm.Img[p] + off);
            if constexpr (!(ABL & 1))
              dw[XIN ? l - 1 : l][kb] = mfma_s3(gp[s], hb, dw[XIN ? l - 1 : l][kb]);
          }
          if (s == 1) load_w2(wb, 1);
          S3F_SB();
        }
      }
      STAMP(stamp++);
      // dH = G W_l (P layout: feature k on the lane): A = G^T image rows m, B = W_l^T planes
      f32x16 dh[2] = {f32x16{}, f32x16{}};
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31;
        auto dh_pair = [&](const u32x4 (&wf)[3][2], int pair) {
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              u32x4 f[3];
              const int off = ap_chunk(32 * q + li, 2 * (2 * pair + s2) + h);
#pragma unroll
              for (int p = 0; p < 3; ++p) f[p] = lds16(sm.Gt[p] + off);
              u32x4 bw[3];
#pragma unroll
              for (int p = 0; p < 3; ++p) bw[p] = wf[p][s2];
              if constexpr (!(ABL & 1)) dh[q] = mfma_s3(f, bw, dh[q]);
            }
            S3F_SB();
          }
        };
        dh_pair(wa, 0);
        load_w2(wa, 2);
        dh_pair(wb, 1);
        load_w2(wb, 3);
        dh_pair(wa, 2);
        dh_pair(wb, 3);
      }
      // dZ_{l-1} = dH * ELU'(H_{l-1}) (no ELU below the first conv: in_proj has none); rows past
      // M and features past K are zero
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, k = 32 * (tq >> 6) + (tq & 31);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float v = elu_prev ? dh[q][r] * elu_grad_from_out(hp[q][r]) : dh[q][r];
            dz[q][r] = (k < K && r0 + m < M) ? v : 0.f;
          }
      }
      lds_barrier();  // every read of both images done
      STAMP(stamp++);
    }
    if constexpr (XIN) {
      // in_proj outside: this tile's dZ_0 rows to HBM (feature k on the lane: 128-B row pieces)
      if constexpr (AG && kAdjPipe) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (fresh_tid() == 0) sm.flag = 0;
      }
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, k = 32 * (tq >> 6) + (tq & 31);
        const int N0 = a.width[1];
        if (k < N0) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int64_t row = r0 + 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
              if (row < M) a.dZ0[row * N0 + k] = dz[q][r];
            }
        }
        pre_cnt = (has_next && tq < TM) ? a.gptr[pre_g + 1] - a.gptr[pre_g] : 0;
        if (has_head(a)) {
#pragma unroll
          for (int c = 0; c < kMaxHeadC; ++c)
            pre_dl[c] = (has_next && tq < TM && c < a.C) ? head_raw(a, pre_g, c) : 0.f;
          if (a.ce.pm) pre_wt = (has_next && tq < TM) ? a.ce.wt[pre_g] : 0.f;
        }
      }
      lds_barrier();  // every wave's next-tile Â landed
      if constexpr (AG && kAdjPipe) {
        const AdjPlanes nap = adj_split(sm);
        lds_barrier();  // every scratch read done (the planes overwrite it)
        adj_write(sm, nap);
        lds_barrier();  // the next tile's Â^T planes are in place
      }
      STAMP(stamp++);
    } else {
    // in_proj: db_0, dW_0 += dZ_0^T X
    {
      const int K = a.width[0];
      // (pipelined Â: unconditional — a branch around these barriers and stores made the
      // register allocator spill ~116 VGPRs; past the last tile the planes written are unused)
      if constexpr (AG && kAdjPipe) {
        // the next tile's Â (issued at the last conv, long landed) and H_L rows: complete before
        // the barrier below, so every wave can split the Â planes beside the dW_0 products
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (fresh_tid() == 0) sm.flag = 0;
      }
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31, k = 32 * (tq >> 6) + li;
        float sacc = 0.f;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc += dz[q][r];
        sacc += __shfl_xor(sacc, 32, 64);
        dbacc[0] += sacc;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            u32x2 o[3];
            split4(f32x4{xp[q][4 * gq], xp[q][4 * gq + 1], xp[q][4 * gq + 2], xp[q][4 * gq + 3]},
                   o);
            const int off = hf_off(k, 32 * q + 8 * gq + 4 * h);
#pragma unroll
            for (int p = 0; p < 3; ++p) sts8(sm.Img[p] + off, o[p]);
          }
        (void)K;
        pre_cnt = (has_next && tq < TM) ? a.gptr[pre_g + 1] - a.gptr[pre_g] : 0;
        if (has_head(a)) {
#pragma unroll
          for (int c = 0; c < kMaxHeadC; ++c)
            pre_dl[c] = (has_next && tq < TM && c < a.C) ? head_raw(a, pre_g, c) : 0.f;
          if (a.ce.pm) pre_wt = (has_next && tq < TM) ? a.ce.wt[pre_g] : 0.f;
        }
      }
      lds_barrier();
      AdjPlanes nap;  // the next tile's Â^T planes (pipe)
      {
        u32x4 gp[4][3];
        split_p(dz, gp);
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31;
#pragma unroll
        for (int s = 0; s < 4; ++s) {  // node steps outer, as the conv layers' dW
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) {
            u32x4 hb[3];
            const int off = hf_chunk(32 * kb + li, 2 * s + h);
#pragma unroll
            for (int p = 0; p < 3; ++p) hb[p] = lds16(sm.Img[p] + off);
            if constexpr (!(ABL & 1) && !XIN) dw[0][kb] = mfma_s3(gp[s], hb, dw[0][kb]);
          }
          // the next tile's Â split beside the products (independent VALU / LDS work)
          if constexpr (AG && kAdjPipe) {
            // (unconditional: without a next tile the planes are not written, and its flag
            // word is never read)
            if (s == 1) nap = adj_split(sm);
          }
          S3F_SB();
        }
      }
      lds_barrier();  // X image read (and the Â scratch); the next tile may overwrite LDS
      if constexpr (AG && kAdjPipe) {
        adj_write(sm, nap);
        lds_barrier();  // the next tile's Â^T planes are in place
      }
      STAMP(stamp++);
    }
    }
    t = tn;
  }
  // partial slot blockIdx.x of every layer: dW rows n = 32 wave + (r & 3) + 8 (r >> 2) + 4h,
  // columns k = 32 kb + li; db from the h = 0 lanes
  if (write_slots) {
    const int tq = threadIdx.x;
    const int h = (tq >> 5) & 1, li = tq & 31, wv = tq >> 6;
#pragma unroll
    for (int l = XIN ? 1 : 0; l < NL; ++l) {
      const int N = a.width[l + 1], K = a.width[l];
      float* slab = a.dWp[l] + (int64_t)blockIdx.x * N * K;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int k = 32 * kb + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int n = 32 * wv + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (n < N && k < K) {
            // write-through (sc1): the slab lines leave this XCD's L2 as they are written
            // instead of at the kernel-end write-back (one-box A/B: step 0.2306 -> 0.2294 ms)
            st_wt(slab + (int64_t)n * K + k, dw[XIN ? l - 1 : l][kb][r]);
          }
        }
      }
      const int n = 32 * wv + li;
      if (h == 0 && n < N) a.dbp[l][(int64_t)blockIdx.x * N + n] = dbacc[l];
    }
  }
  if (o.sync && tmask[ntiles] > 0) {
    static_assert(sizeof(LwSmem) <= sizeof(FBwdSmem), "open-tile LDS aliases the fused LDS");
    __syncthreads();  // the closed phase's LDS is free; this workgroup's slots are written
    LwSmem& lw = *reinterpret_cast<LwSmem*>(&sm);
    for (int l = L; l >= 0; --l) {
      if (l < L) grid_sync(o.sync, L - l);  // dS of layer l + 1 complete for every open tile
      const int K = a.width[l], N = a.width[l + 1];
      const float* Sx = l == 0 ? a.X : o.S[l - 1];
      if (l == L)
        bwd_tiles<LGNN_GRAD_POOL, LGNN_ACT_ELU, true>(
            lw.A, lw.C, lw.ti, a.dP, a.batch, a.gptr, a.pool_mean, nullptr, nullptr, nullptr, 0.f,
            a.H[l], Sx, M, K, o.W[l], N, o.dS[l & 1], a.dWp[l], a.dbp[l], tmask, 1, 1, a.dlog,
            a.Wout, a.C, BnFuse{}, a.ce);
      else if (l >= 1)
        bwd_tiles<LGNN_GRAD_TRANSPOSE, LGNN_ACT_ELU, true>(
            lw.A, lw.C, lw.ti, o.dS[(l + 1) & 1], a.batch, a.gptr, a.pool_mean, o.tptr, o.tidx,
            o.tw, 0.f, a.H[l], Sx, M, K, o.W[l], N, o.dS[l & 1], a.dWp[l], a.dbp[l], tmask, 1,
            1);
      else if constexpr (XIN)
        open_dz0(a.dZ0, o.dS[1], o.tptr, o.tidx, o.tw, M, N, tmask);
      else
        bwd_tiles<LGNN_GRAD_TRANSPOSE, LGNN_ACT_NONE, false>(
            lw.A, lw.C, lw.ti, o.dS[1], a.batch, a.gptr, a.pool_mean, o.tptr, o.tidx, o.tw, 0.f,
            nullptr, Sx, M, K, o.W[0], N, nullptr, a.dWp[0], a.dbp[0], tmask, 1, 1);
    }
    grid_exit(o.sync);
  }
}

}  // namespace lgnn_s3

static int stack_bwd_s3f(const float* dP, const int64_t* batch, const int32_t* gptr,
                         int pool_mean, int64_t num_graphs, const int32_t* rowptr,
                         const int32_t* col, const float* w, const float* X, int64_t M, int L,
                         const uint16_t* planes_t, const float* const* H, const int* widths,
                         float* const* dWp, float* const* dbp, int num_partials,
                         const int32_t* tile_open, const lgnn_s3::OpenBwdArgs& o, void* stream,
                         const float* dlogits = nullptr, const float* Wout = nullptr,
                         int num_classes = 0, const void* adjt = nullptr,
                         const lgnn_ce_src* ce = nullptr, float* dz0 = nullptr);

extern "C" int lgnn_gcn_stack_bwd_s3f(const float* dP, const int64_t* batch, const int32_t* gptr,
                                      int pool_mean, int64_t num_graphs, const int32_t* rowptr,
                                      const int32_t* col, const float* w, const float* X,
                                      int64_t M, int L, const uint16_t* planes_t,
                                      const float* const* H, const int* widths,
                                      float* const* dWp, float* const* dbp, int num_partials,
                                      const int32_t* tile_open, const void* adjt, void* stream) {
  const lgnn_s3::OpenBwdArgs o = {};
  return stack_bwd_s3f(dP, batch, gptr, pool_mean, num_graphs, rowptr, col, w, X, M, L, planes_t,
                       H, widths, dWp, dbp, num_partials, tile_open, o, stream, nullptr, nullptr,
                       0, adjt);
}

static int stack_bwd_s3f_all(
    const float* dP, const int64_t* batch, const int32_t* gptr, int pool_mean,
    int64_t num_graphs, const int32_t* rowptr, const int32_t* col, const float* w,
    const int32_t* tptr, const int32_t* tidx, const float* tw, const float* X, int64_t M, int L,
    const uint16_t* planes_t, const float* const* W, const float* const* H,
    const float* const* S, const int* widths, float* const* dWp, float* const* dbp,
    int num_partials, float* dS_ws, int32_t* tile_open, const float* dlogits,
    const lgnn_ce_src* ce, const float* Wout, int num_classes, const void* adjt, void* stream) {
  if (M < 0 || L < 1 || L > 3 || !W || !S || !tptr || !tidx || !tw || !dS_ws || !tile_open)
    return LGNN_EINVAL;
  if ((dlogits || ce) && (!Wout || num_classes < 1 || num_classes > lgnn_s3::kMaxHeadC))
    return LGNN_EINVAL;
  lgnn_s3::OpenBwdArgs o = {};
  for (int l = 0; l <= L; ++l) {
    if (!W[l] || (l >= 1 && !S[l - 1])) return LGNN_EINVAL;
    o.W[l] = W[l];
    if (l >= 1) o.S[l - 1] = S[l - 1];
  }
  o.dS[0] = dS_ws;
  o.dS[1] = dS_ws + M * lgnn_s3::WP;
  o.tptr = tptr;
  o.tidx = tidx;
  o.tw = tw;
  const int64_t ntiles = (M + lgnn_tile::TM - 1) / lgnn_tile::TM;
  o.sync = tile_open + ntiles + 4;
  // L = 3: the third [M][128] block of dS_ws receives dZ_0 (the in_proj gradient is the caller's)
  return stack_bwd_s3f(dP, batch, gptr, pool_mean, num_graphs, rowptr, col, w, X, M, L, planes_t,
                       H, widths, dWp, dbp, num_partials, tile_open, o, stream, dlogits, Wout,
                       num_classes, adjt, ce, L == 3 ? dS_ws + 2 * M * lgnn_s3::WP : nullptr);
}

extern "C" int lgnn_gcn_stack_bwd_s3f_all(
    const float* dP, const int64_t* batch, const int32_t* gptr, int pool_mean,
    int64_t num_graphs, const int32_t* rowptr, const int32_t* col, const float* w,
    const int32_t* tptr, const int32_t* tidx, const float* tw, const float* X, int64_t M, int L,
    const uint16_t* planes_t, const float* const* W, const float* const* H,
    const float* const* S, const int* widths, float* const* dWp, float* const* dbp,
    int num_partials, float* dS_ws, int32_t* tile_open, const float* dlogits, const float* Wout,
    int num_classes, const void* adjt, void* stream) {
  return stack_bwd_s3f_all(dP, batch, gptr, pool_mean, num_graphs, rowptr, col, w, tptr, tidx, tw,
                           X, M, L, planes_t, W, H, S, widths, dWp, dbp, num_partials, dS_ws,
                           tile_open, dlogits, nullptr, Wout, num_classes, adjt, stream);
}

extern "C" int lgnn_gcn_stack_bwd_s3f_ce(
    const int64_t* batch, const int32_t* gptr, int pool_mean, int64_t num_graphs,
    const int32_t* rowptr, const int32_t* col, const float* w, const int32_t* tptr,
    const int32_t* tidx, const float* tw, const float* X, int64_t M, int L,
    const uint16_t* planes_t, const float* const* W, const float* const* H,
    const float* const* S, const int* widths, float* const* dWp, float* const* dbp,
    int num_partials, float* dS_ws, int32_t* tile_open, const struct lgnn_ce_src* ce,
    const float* Wout, int num_classes, const void* adjt, void* stream) {
  if (!ce) return LGNN_EINVAL;
  return stack_bwd_s3f_all(nullptr, batch, gptr, pool_mean, num_graphs, rowptr, col, w, tptr, tidx,
                           tw, X, M, L, planes_t, W, H, S, widths, dWp, dbp, num_partials, dS_ws,
                           tile_open, nullptr, ce, Wout, num_classes, adjt, stream);
}

static int stack_bwd_s3f(const float* dP, const int64_t* batch, const int32_t* gptr,
                         int pool_mean, int64_t num_graphs, const int32_t* rowptr,
                         const int32_t* col, const float* w, const float* X, int64_t M, int L,
                         const uint16_t* planes_t, const float* const* H, const int* widths,
                         float* const* dWp, float* const* dbp, int num_partials,
                         const int32_t* tile_open, const lgnn_s3::OpenBwdArgs& o, void* stream,
                         const float* dlogits, const float* Wout, int num_classes,
                         const void* adjt, const lgnn_ce_src* ce, float* dz0) {
  // L = 3 (XIN) only with the open-tile phase in the launch: it gathers the open tiles' dZ_0 rows
  if (M < 0 || L < 1 || L > 3 || (L == 3 && (!dz0 || !o.sync)) || !(dP || dlogits || ce) || !batch || !gptr || !rowptr || !col ||
      !X ||
      !planes_t || !H || !widths || !dWp || !dbp || !tile_open || num_graphs < 0)
    return LGNN_EINVAL;
  if (num_partials != lgnn_gcn_stack_bwd_partials(M)) return LGNN_EINVAL;
  lgnn_s3::FBwdArgs a = {};
  a.dP = dP;
  a.dlog = dlogits;
  if (ce) {
    if (dlogits || !ce->pm || !ce->wt || !ce->wsum || !ce->gloss)
      return LGNN_EINVAL;
    a.ce = CeSrc{ce->pm, ce->wt, ce->wsum, ce->gloss, num_classes};
  }
  a.Wout = Wout;
  a.C = num_classes;
  a.adjt = static_cast<const unsigned char*>(adjt);
  a.batch = batch;
  a.gptr = gptr;
  a.pool_mean = pool_mean;
  a.num_graphs = num_graphs;
  a.X = X;
  a.WpT = planes_t;
  a.dZ0 = dz0;
  for (int l = 0; l <= L + 1; ++l) a.width[l] = widths[l];
  for (int l = 0; l <= L; ++l) {
    if (!lgnn_tile_fits(M, widths[l], widths[l + 1]) || !H[l] || !dWp[l] || !dbp[l])
      return LGNN_EINVAL;
    a.H[l] = H[l];
    a.dWp[l] = dWp[l];
    a.dbp[l] = dbp[l];
  }
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    for (int l = 0; l <= L; ++l)
      if (hipMemsetAsync(dWp[l], 0, (size_t)widths[l] * widths[l + 1] * 4, s) != hipSuccess ||
          hipMemsetAsync(dbp[l], 0, (size_t)widths[l + 1] * 4, s) != hipSuccess)
        return (int)hipGetLastError();
    return LGNN_OK;
  }
  const dim3 grid((unsigned)num_partials), blk(lgnn_tile::NT);
  if (o.sync) {  // open tiles behind grid barriers: every workgroup must be resident at once
    const int cap = lgnn_fused_grid_capacity(1);
    if (cap < (int)grid.x) return cap == LGNN_EINVAL ? cap : cap < 0 ? -cap : LGNN_EBUSY;
  }
  if (L == 3 && adjt)
    hipLaunchKernelGGL((lgnn_s3::k_s3_fbwd<4, true, true>), grid, blk, 0, s, rowptr, col, w, M, a,
                       tile_open, o);
  else if (L == 3)
    hipLaunchKernelGGL((lgnn_s3::k_s3_fbwd<4, false, true>), grid, blk, 0, s, rowptr, col, w, M,
                       a, tile_open, o);
  else if (L == 1 && adjt)
    hipLaunchKernelGGL((lgnn_s3::k_s3_fbwd<2, true>), grid, blk, 0, s, rowptr, col, w, M, a,
                       tile_open, o);
  else if (L == 1)
    hipLaunchKernelGGL((lgnn_s3::k_s3_fbwd<2, false>), grid, blk, 0, s, rowptr, col, w, M, a,
                       tile_open, o);
  else if (adjt)
    hipLaunchKernelGGL((lgnn_s3::k_s3_fbwd<3, true>), grid, blk, 0, s, rowptr, col, w, M, a,
                       tile_open, o);
  else
    hipLaunchKernelGGL((lgnn_s3::k_s3_fbwd<3, false>), grid, blk, 0, s, rowptr, col, w, M, a,
                       tile_open, o);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

// workgroups per CU of the fused backward (the open-tile phase's grid barrier needs them all
// resident)
hipError_t lgnn_s3_fbwd_occupancy(int* per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, lgnn_s3::k_s3_fbwd<3, true>,
                                                      lgnn_tile::NT, 0);
}

#ifdef LGNN_STAMPS
extern "C" int lgnn_debug_stamps_s3b(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(lgnn_stamp_buf), sizeof(lgnn_stamp_buf));
}
#endif
