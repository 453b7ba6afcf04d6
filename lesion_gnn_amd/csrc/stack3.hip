// Fused GCN stack on bf16 MFMA at fp32 accuracy ("split-3"): every fp32 GEMM operand x is held as
// three bf16 planes x = x_hi + x_mid + x_lo (+ r, |r| <= 2^-24 |x|; each plane is the RNE bf16 of
// what the planes above it left over), and a product a.b is taken as the six plane products
//   a_lo b_hi + a_mid b_mid + a_hi b_lo + a_mid b_hi + a_hi b_mid + a_hi b_hi
// (the three dropped ones are below 2^-24 relative). Each bf16 x bf16 product is exact in fp32 and
// the MFMA accumulates in fp32, so the result carries fp32-class error (a few ulp of the sum of
// |a.b|), like the fp32 MFMA chain — at 16 / 6 = 2.7x its rate: gfx950 runs
// v_mfma_f32_32x32x16_bf16 at 16x the FLOP rate of v_mfma_f32_32x32x2_f32 and has no xf32.
//
// k_s3_fwd is the split-3 twin of k_stack_fwd (tile.hip): in_proj + L x ELU(GCNConv) for the
// tiles no edge leaves, PyG's association H_l = ELU(Â (H_{l-1} W_l^T) + b_l). Per layer:
//   GEMM1  P = H W_l^T          A operand = H planes (LDS image), B operand = W_l planes
//                               (registers, loaded a layer ahead, pre-split by k_wplanes)
//   GEMM2  Z^T = P^T Â^T        A operand = P straight from GEMM1's accumulators (split in
//                               registers; the accumulator's row order is the operand's k order),
//                               B operand = Â_tile planes (LDS, built once per tile)
//   epilogue  +b, ELU; H_l -> HBM (fp32, 16-B stores) and -> the LDS planes of the next layer
// GEMM2's output has the node on the lane and four consecutive features per register group, so
// the next layer's H planes are written with 8-byte stores and read back as whole MFMA fragments:
// one LDS round trip per layer. When every weight of a tile's Â is exact in bf16 (k-regular
// k-NN graphs: 1/k with k a power of two) GEMM2 takes three plane products instead of six.
//
// Feature index order: the planes store feature k at position perm16(k) (bits 2 and 3 of k
// swapped), which is the k order an MFMA accumulator hands to the next MFMA; weights, images and
// accumulators all use it, so every product pairs equal k.
#include "common.h"
#include "tile.h"
#include "tile_util.h"
#include "s3_util.h"
#include "tile_lw.h"

// Timing-only ablation builds (tools/s3_probe.py): -DLGNN_S3_ABLATE=<mask> removes phases of
// k_s3_fwd (1 GEMM1 MFMAs, 2 GEMM2 MFMAs, 4 H stores, 8 ELU, 16 epilogue plane split, 32 weight
// reloads, 64 next-tile X loads). The product build is mask 0; ablated libraries are built
// outside the package and never loaded by it.
#ifndef LGNN_S3_ABLATE
#define LGNN_S3_ABLATE 0
#endif

// Diagnostic build only (-DLGNN_S3_STAMPS, tools/s3_probe.py stamps): thread 0 of each block
// records s_memtime at phase boundaries of k_s3_fwd; never compiled into the product library.
#ifdef LGNN_S3_STAMPS
__device__ unsigned long long lgnn_s3_stamp_buf[1024 * 64];
#define S3STAMP()                                                                  \
  do {                                                                             \
    if (threadIdx.x == 0 && stamp_i < 64)                                          \
      lgnn_s3_stamp_buf[blockIdx.x * 64 + stamp_i] = __builtin_amdgcn_s_memtime(); \
    ++stamp_i;                                                                     \
  } while (0)
#else
#define S3STAMP() \
  do {            \
  } while (0)
#endif

namespace lgnn_s3 {
using namespace lgnn_tile;
constexpr int S3ABL = LGNN_S3_ABLATE;

// Weight planes (s3_util.h wplanes_item): one thread per (layer, n, 4 consecutive k).
__global__ __launch_bounds__(256) void k_wplanes(PlaneArgs a) {
  wplanes_item(a, blockIdx.x * 256 + threadIdx.x);
}

// ------------------------------------------------------------------------------------------
// Fused forward
// ------------------------------------------------------------------------------------------
struct FwdSmem {
  unsigned char Ap[3][TM * AROW];     // H_{l-1} (or X) planes, 48 KiB
  unsigned char Adj[3][ADJ_PLANE];    // Â_tile planes [target][perm16(source)], 27 KiB; the first
                                      // 16 KiB first hold Â in fp32 while it is summed
  float bias[LGNN_MAX_STACK][WP];     // zero past each layer's width
  int rp[TM + 1];
  int flag;                           // some Â weight of the tile is not exact in bf16
};

// W_l planes fragment of this lane: row n = 32 * wave + li, chunk 2s + h of each plane.
__device__ __forceinline__ void load_wf(u32x4 (&wf)[3][8], const uint16_t* __restrict__ Wp,
                                        int l) {
  const int t = fresh_tid(), lane = t & 63, wave = t >> 6;
  // fragment order (k_wplanes): one contiguous 1-KiB wave load per plane and k-step
  const uint16_t* base = Wp + (size_t)l * 3 * PLANE + wave * 8 * 512 + lane * 8;
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      wf[p][s] = *reinterpret_cast<const u32x4*>(base + p * PLANE + 512 * s);
}

// Epilogue of one layer from the Z^T accumulators (z0: node li, z1: node 32 + li; register r:
// feature 32 * wave + (r & 3) + 8 * (r >> 2) + 4h): + bias, ELU, H_l -> HBM, planes -> Ap.
template <bool ELU, bool PLANES>
__device__ __forceinline__ void epilogue(FwdSmem& sm, const f32x16& z0, const f32x16& z1,
                                         const float* bias, Buf hb, int N, int64_t r0) {
  const int t = fresh_tid(), lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  f32x4 bv[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bv[g] = ld4(bias + 32 * wave + 8 * g + 4 * h);
  const int rowb = (int)(r0 * N * 4);  // byte offset of the tile's first row (< 2 GiB: host)
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int m = 32 * a + li;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n0 = 32 * wave + 8 * g + 4 * h;
      const f32x16& z = a ? z1 : z0;
      f32x4 v = f32x4{z[4 * g], z[4 * g + 1], z[4 * g + 2], z[4 * g + 3]} + bv[g];
      if (ELU && !(S3ABL & 8)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = elu_s3(v[j]);
      }
      // columns past N: an offset past the buffer's range, so the store is dropped (no branch)
      if (!(S3ABL & 4)) bst4(hb, n0 < N ? rowb + (m * N + n0) * 4 : INT32_MAX - 15, v);
      if (PLANES) {
        u32x2 o[3];
        if (S3ABL & 16)
          o[0] = o[1] = o[2] = u32x2{__float_as_uint(v[0]), __float_as_uint(v[1])};
        else
          split4(v, o);
        const int off = ap_off(m, n0);
#pragma unroll
        for (int p = 0; p < 3; ++p) sts8(sm.Ap[p] + off, o[p]);
      }
      __builtin_amdgcn_sched_barrier(0);  // one (row block, group) at a time
    }
  }
}

// k-step s fragment (three planes) of image row `row` (chunk 2s + h of an H-image plane, or of
// an Â plane when ADJ)
template <bool ADJ = false>
__device__ __forceinline__ void rd_half(u32x4 (&f)[3], const FwdSmem& sm, int h, int row, int s) {
  const int off = ADJ ? row * ADJ_LD * 2 + 16 * (2 * s + h) : ap_chunk(row, 2 * s + h);
#pragma unroll
  for (int p = 0; p < 3; ++p) f[p] = lds16((ADJ ? sm.Adj[p] : sm.Ap[p]) + off);
}

// one k-step: six MFMAs on the first accumulator, then the first operand's next reads, six on
// the second, its next reads (single-buffered operands: a read is issued once its last MFMA is)
__device__ __forceinline__ void gemm_sched(bool reads) {
  __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
  if (reads) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
  __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
  if (reads) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
  __builtin_amdgcn_sched_barrier(0);
}

// GEMM over the 128 features of the H image with the W fragment: for the node blocks li and
// 32 + li of the image, c0/c1 += (W-side) x (image-side). TRANS = false: the image is the A
// operand (P = H W^T: feature on the lane); true: the B operand (H^T = W X^T: node on the lane).
template <bool TRANS>
__device__ __forceinline__ void gemm_feat(f32x16& c0, f32x16& c1, const u32x4 (&wf)[3][8],
                                          const FwdSmem& sm) {
  const int t = fresh_tid();
  const int h = (t >> 5) & 1, li = t & 31;
  u32x4 f0[3], f1[3];
  rd_half(f0, sm, h, li, 0);
  rd_half(f1, sm, h, 32 + li, 0);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    u32x4 w3[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) w3[p] = wf[p][s];
    if (!(S3ABL & 1)) c0 = TRANS ? mfma_s3(w3, f0, c0) : mfma_s3(f0, w3, c0);
    if (s + 1 < 8) rd_half(f0, sm, h, li, s + 1);
    if (!(S3ABL & 1)) c1 = TRANS ? mfma_s3(w3, f1, c1) : mfma_s3(f1, w3, c1);
    if (s + 1 < 8) rd_half(f1, sm, h, 32 + li, s + 1);
    gemm_sched(s + 1 < 8);
  }
}

// Open-tile phase of the fused forward (optional): after the closed tiles, the tiles an edge
// leaves run layer by layer on the fp32 layer-wise bodies (tile_lw.h, fp32 weights W, aggregated
// inputs saved to S[l - 1] for the backward), a grid barrier between layers. Closed and open tiles
// share no edge (the graph build flags both ends of a crossing edge), so the two phases are
// independent; with no open tile (k-NN graphs aligned to tiles) the phase is skipped.
struct OpenFwdArgs {
  const float* W[LGNN_MAX_STACK];  // fp32 weights [N_l][K_l]
  float* S[LGNN_MAX_STACK];        // S[l - 1] = Â H_{l-1} of the open tiles (conv l)
  int32_t* sync;                   // grid-barrier words (nullptr: no open phase)
  unsigned char* adjt;             // nullable: fp32 Â of every closed tile for the fused backward,
                                   // ADJT_TILE_BYTES per tile
};

template <bool FIRST>
__global__ __launch_bounds__(NT, 2) void k_s3_fwd(const float* __restrict__ X, int64_t M,
                                                  const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col,
                                                  const float* __restrict__ w, int L,
                                                  StackArgs args, const uint16_t* __restrict__ Wp,
                                                  const int32_t* __restrict__ tmask,
                                                  OpenFwdArgs o) {
  __shared__ __attribute__((aligned(16))) FwdSmem sm;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int l0 = FIRST ? 0 : 1;
  const int K0 = args.width[l0];
  float* const scr = reinterpret_cast<float*>(sm.Adj[0]);  // fp32 Â [target][source], 16 KiB

  for (int i = threadIdx.x; i < (L + 1) * WP; i += NT) {
    const int l = i / WP, n = i % WP;
    sm.bias[l][n] = (l >= l0 && n < args.width[l + 1]) ? args.b[l][n] : 0.f;
  }
  int64_t t = seek_tile(blockIdx.x, ntiles, tmask, 0);
  if (t < ntiles) {
  [[maybe_unused]] int stamp_i = 0;
  S3STAMP();

  f32x4 xr[8];
  IdxRegs R;
  u32x4 wf[3][8];
  const Buf bX = mkbuf(X, M * K0 * 4);
  load_rows(xr, bX, K0, (int)(t * TM));
  load_wf(wf, Wp, l0);
  idx_load_head(R, rowptr, M, t * TM);
  idx_load_body(R, col, w);
  for (; t < ntiles;) {
    const int64_t r0 = t * TM;
    const int64_t tn = seek_tile(t + gridDim.x, ntiles, tmask, 0);
    const bool has_next = tn < ntiles;
    // X planes (zero past K0 and M), fp32 Â scratch zeroed, the tile's rowptr
    {
      const int tq = fresh_tid();
      const int li = tq & 31, hw = tq >> 5;
      const bool kin = 4 * li < K0;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        u32x2 o[3];
        split4(sel4(kin && r0 + rr < M, xr[it]), o);
        const int off = ap_off(rr, 4 * li);
#pragma unroll
        for (int p = 0; p < 3; ++p) sts8(sm.Ap[p] + off, o[p]);
      }
#pragma unroll
      for (int i = 0; i < TM * TM / 4 / NT; ++i) st4(scr + 4 * (tq + i * NT), zero4());
      if (tq <= TM) sm.rp[tq] = R.rp;
      if (tq == 0) sm.flag = 0;
    }
    lds_barrier();
    S3STAMP();  // 1: prologue (X planes) + B1
    adj_scatter<false>(scr, sm.rp, R, r0, col, w);
    if (has_next) idx_load_head(R, rowptr, M, tn * TM);
    f32x16 z0 = {}, z1 = {};
    if (FIRST) {
      // H_0^T = W_0 X^T: A = W_0 planes (registers), B = X planes; node on the lane
      gemm_feat<true>(z0, z1, wf, sm);
      if (!(S3ABL & 32)) load_wf(wf, Wp, 1);
    }
    S3STAMP();  // 2: scatter + in_proj GEMM
    if (has_next) idx_load_body(R, col, w);
    lds_barrier();  // Â summed; every read of the X planes done
    S3STAMP();  // 3: B2
    // this thread's 16 Â weights: target row tid / 4, sources 16 (tid & 3) ..
    f32x4 av[4];
    {
      const int tq = fresh_tid();
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = ld4(scr + (tq >> 2) * TM + 16 * (tq & 3) + 4 * i);
    }
    if (o.adjt) {  // the summed fp32 Â for the backward: this thread's 64 B, the tile coalesced
      const Buf ba = mkbuf(o.adjt + t * ADJT_TILE_BYTES, ADJT_TILE_BYTES);
      const int tq = fresh_tid();
#pragma unroll
      for (int i = 0; i < 4; ++i) bst4(ba, 64 * tq + 16 * i, av[i]);
    }
    if (FIRST)
      epilogue<false, true>(sm, z0, z1, sm.bias[0], mkbuf(args.H[0], M * args.width[1] * 4),
                            args.width[1], r0);
    S3STAMP();  // 4: in_proj epilogue
    lds_barrier();  // every scratch read done
    int inexact = 0;
    {
      const int tq = fresh_tid();
      const int am = tq >> 2, aq = tq & 3;
      // phys position y of the 16-block holds source 16 aq + perm16(y)
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
    S3STAMP();  // 5: Â planes + B4
    for (int l = 1; l <= L; ++l) {
      const int N = args.width[l + 1];
      // GEMM1: P = H W_l^T (A = H planes, B = W_l planes; feature on the lane)
      f32x16 p0 = {}, p1 = {};
      gemm_feat<false>(p0, p1, wf, sm);
      S3STAMP();  // l: W load + GEMM1
      // the next tile's rows, a GEMM2 and an epilogue ahead of their use (vmcnt is in order:
      // they are issued after this layer's weight loads, before the next ones)
      if (l == L && has_next && !(S3ABL & 64)) load_rows(xr, bX, K0, (int)(tn * TM));
      // P (feature on the lane, node in the registers) -> A-operand fragments over nodes:
      // k-step s uses registers 8 (s & 1) .. + 7 of p0 (s < 2) or p1
      u32x4 pp[4][3];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const f32x16& pa = s < 2 ? p0 : p1;
        const int rb = 8 * (s & 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const Split2 s2 = split2(pa[rb + 2 * i], pa[rb + 2 * i + 1]);
#pragma unroll
          for (int p = 0; p < 3; ++p) pp[s][p][i] = s2.p[p];
        }
      }
      S3STAMP();  // l: P split
      // GEMM2: Z^T = P^T Â^T (B = Â planes, target node li / 32 + li)
      z0 = f32x16{};
      z1 = f32x16{};
      {
        const int tq = fresh_tid();
        const int h = (tq >> 5) & 1, li = tq & 31;
        if (exact) {
          // Â_hi only: all eight operand reads up front, then 24 MFMAs
          u32x4 b0[4], b1[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            b0[s] = lds16(sm.Adj[0] + li * ADJ_LD * 2 + 16 * (2 * s + h));
            b1[s] = lds16(sm.Adj[0] + (32 + li) * ADJ_LD * 2 + 16 * (2 * s + h));
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            if (!(S3ABL & 2)) {
              z0 = mfma_s3_bexact(pp[s], b0[s], z0);
              z1 = mfma_s3_bexact(pp[s], b1[s], z1);
            }
          }
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            u32x4 b0[3], b1[3];
            rd_half<true>(b0, sm, h, li, s);
            rd_half<true>(b1, sm, h, 32 + li, s);
            if (!(S3ABL & 2)) {
              z0 = mfma_s3(pp[s], b0, z0);
              z1 = mfma_s3(pp[s], b1, z1);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      S3STAMP();  // l: GEMM2
      // the next layer's weights (or the first layer's, for the next tile): issued before the
      // epilogue's stores so that waiting for them never waits for the stores
      if (!(S3ABL & 32)) load_wf(wf, Wp, l < L ? l + 1 : l0);
      lds_barrier();  // every read of the H planes and Â done
      S3STAMP();  // l: B5
      const Buf hb = mkbuf(args.H[l], M * N * 4);
      if (l < L) {
        epilogue<true, true>(sm, z0, z1, sm.bias[l], hb, N, r0);
        S3STAMP();  // l: epilogue
        lds_barrier();
        S3STAMP();  // l: B6
      } else {
        epilogue<true, false>(sm, z0, z1, sm.bias[l], hb, N, r0);
        S3STAMP();  // L: epilogue
      }
    }
    t = tn;
  }
  }
  if (o.sync && tmask[ntiles] > 0) {
    static_assert(sizeof(LwSmem) <= sizeof(FwdSmem), "open-tile LDS aliases the fused LDS");
    __syncthreads();  // the closed phase's LDS is free
    LwSmem& lw = *reinterpret_cast<LwSmem*>(&sm);
    for (int l = l0; l <= L; ++l) {
      if (l > l0) grid_sync(o.sync, l - l0);  // layer l reads other open tiles' H_{l-1}
      const int K = args.width[l], N = args.width[l + 1];
      if (l == 0)
        fwd_tiles<false, LGNN_ACT_NONE>(lw.A, lw.C, lw.ti, X, M, K, nullptr, nullptr, nullptr,
                                        0.f, o.W[0], args.b[0], N, args.H[0], nullptr, tmask, 1);
      else
        fwd_tiles<true, LGNN_ACT_ELU>(lw.A, lw.C, lw.ti, l == 1 && !FIRST ? X : args.H[l - 1], M,
                                      K, rowptr, col, w, 0.f, o.W[l], args.b[l], N, args.H[l],
                                      o.S[l - 1], tmask, 1);
    }
    grid_exit(o.sync);
  }
}

}  // namespace lgnn_s3

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
#ifdef LGNN_S3_STAMPS
extern "C" int lgnn_s3_debug_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(lgnn_s3_stamp_buf),
                                  sizeof(lgnn_s3_stamp_buf));
}
#endif

hipError_t lgnn_s3_fbwd_occupancy(int* per_cu);  // stack3_bwd.hip

// Workgroups of a fused stack kernel that can be resident on this device at once (occupancy
// per CU x CU count), cached per device: which = 0 forward (k_s3_fwd<true>), 1 backward
// (k_s3_fbwd<3, true>). A negative value is a HIP error code.
extern "C" int lgnn_fused_grid_capacity(int which) {
  static int cache[2][16];
  static bool have[2][16];
  int dev = 0;
  if (which < 0 || which > 1) return LGNN_EINVAL;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return -(int)hipErrorInvalidDevice;
  if (have[which][dev]) return cache[which][dev];
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -(int)hipGetLastError();
  const hipError_t e = which == 0
      ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lgnn_s3::k_s3_fwd<true>,
                                                     lgnn_tile::NT, 0)
      : lgnn_s3_fbwd_occupancy(&per_cu);
  if (e != hipSuccess) return -(int)e;
  cache[which][dev] = cus * per_cu;
  have[which][dev] = true;
  return cache[which][dev];
}

extern "C" size_t lgnn_weight_planes_bytes(int nl) {
  if (nl < 1 || nl > LGNN_MAX_STACK) return 0;
  return (size_t)nl * 3 * lgnn_s3::PLANE * sizeof(uint16_t);
}

extern "C" int lgnn_weight_planes(int nl, const float* const* W, const int* widths,
                                  uint16_t* planes, uint16_t* planes_t, void* stream) {
  lgnn_s3::PlaneArgs a;
  const int r = lgnn_s3::plane_args(nl, W, widths, planes, planes_t, a);
  if (r != LGNN_OK) return r;
  const int threads = nl * lgnn_s3::PLANE_ITEMS;
  hipLaunchKernelGGL(lgnn_s3::k_wplanes, dim3((threads + 255) / 256), dim3(256), 0,
                     as_stream(stream), a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}

static int stack_fwd_s3(const float* X, int64_t M, int d_in, int has_in_proj,
                        const int32_t* rowptr, const int32_t* col, const float* w, int L,
                        const uint16_t* planes, const float* const* b, const int* widths,
                        float* const* H, const int32_t* tile_open, const float* const* Wf,
                        float* const* S, int32_t* sync, void* adjt, void* stream);

extern "C" int lgnn_gcn_stack_fwd_s3(const float* X, int64_t M, int d_in, int has_in_proj,
                                     const int32_t* rowptr, const int32_t* col, const float* w,
                                     int L, const uint16_t* planes, const float* const* b,
                                     const int* widths, float* const* H,
                                     const int32_t* tile_open, void* adjt, void* stream) {
  return stack_fwd_s3(X, M, d_in, has_in_proj, rowptr, col, w, L, planes, b, widths, H, tile_open,
                      nullptr, nullptr, nullptr, adjt, stream);
}

extern "C" int lgnn_gcn_stack_fwd_s3_all(const float* X, int64_t M, int d_in, int has_in_proj,
                                         const int32_t* rowptr, const int32_t* col,
                                         const float* w, int L, const uint16_t* planes,
                                         const float* const* W, const float* const* b,
                                         const int* widths, float* const* H, float* const* S,
                                         int32_t* tile_open, void* adjt, void* stream) {
  if (!W || !S || !tile_open || M < 0) return LGNN_EINVAL;
  const int64_t ntiles = (M + lgnn_tile::TM - 1) / lgnn_tile::TM;
  return stack_fwd_s3(X, M, d_in, has_in_proj, rowptr, col, w, L, planes, b, widths, H, tile_open,
                      W, S, tile_open + ntiles + 1, adjt, stream);
}

static int stack_fwd_s3(const float* X, int64_t M, int d_in, int has_in_proj,
                        const int32_t* rowptr, const int32_t* col, const float* w, int L,
                        const uint16_t* planes, const float* const* b, const int* widths,
                        float* const* H, const int32_t* tile_open, const float* const* Wf,
                        float* const* S, int32_t* sync, void* adjt, void* stream) {
  if (M < 0 || L < 1 || L + 1 > LGNN_MAX_STACK || !planes || !b || !widths || !H || !rowptr ||
      !col || !tile_open)
    return LGNN_EINVAL;
  lgnn_tile::StackArgs a = {};
  const int l0 = has_in_proj ? 0 : 1;
  if (!has_in_proj && widths[0] != d_in) return LGNN_EINVAL;
  a.width[0] = d_in;
  for (int l = 0; l <= L; ++l) {
    a.width[l + 1] = widths[l];
    if (l < l0) continue;
    const int K = a.width[l], N = a.width[l + 1];
    if (!lgnn_tile_fits(M, K, N) || !b[l] || !H[l]) return LGNN_EINVAL;
    a.b[l] = b[l];
    a.H[l] = H[l];
  }
  lgnn_s3::OpenFwdArgs o = {};
  if (sync) {
    for (int l = l0; l <= L; ++l) {
      if (!Wf[l] || (l >= 1 && !S[l - 1])) return LGNN_EINVAL;
      o.W[l] = Wf[l];
      if (l >= 1) o.S[l - 1] = S[l - 1];
    }
    o.sync = sync;
  }
  o.adjt = static_cast<unsigned char*>(adjt);
  if (M == 0) return LGNN_OK;
  if (!X) return LGNN_EINVAL;
  const int64_t ntiles = (M + lgnn_tile::TM - 1) / lgnn_tile::TM;
  dim3 grid((unsigned)(ntiles < 512 ? ntiles : 512));
  // open tiles behind grid barriers need every workgroup resident at once: refuse (the caller
  // then runs them in separate launches) rather than let a barrier time out
  if (sync) {
    const int cap = lgnn_fused_grid_capacity(0);
    if (cap < (int)grid.x) return cap == LGNN_EINVAL ? cap : cap < 0 ? -cap : LGNN_EBUSY;
  }
  hipStream_t s = as_stream(stream);
  if (has_in_proj)
    hipLaunchKernelGGL(lgnn_s3::k_s3_fwd<true>, grid, dim3(lgnn_tile::NT), 0, s, X, M, rowptr,
                       col, w, L, a, planes, tile_open, o);
  else
    hipLaunchKernelGGL(lgnn_s3::k_s3_fwd<false>, grid, dim3(lgnn_tile::NT), 0, s, X, M, rowptr,
                       col, w, L, a, planes, tile_open, o);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LGNN_OK : (int)e;
}
