// Windowed dense aggregation for the layer-wise GCN path's open tiles (graphs that straddle the
// 64-row tiles: C5's power-law batches).
//
//   Out[r][:] = sum_{e in row r} w_e In[col_e][:]      rows r of the tiles t with mask[t] == want
//
// The row-gather form (tile_lw.h agg_row_global) reads a 512-B source row per CSR entry: at C5
// k = 16, 0.93 M gathers = 479 MB of L2 traffic per layer. Here a 64-row tile instead walks the
// 64-row source chunks its entries reach (the window: the graphs it overlaps) and multiplies the
// dense 64 x 64 block Â_tc, built in LDS from the tile's entries with a source in chunk c, by the
// chunk's rows on split-3 bf16 MFMA (fp32 accuracy, stack3.hip's plane arithmetic): each source
// row is read once per tile that reaches it, not once per entry.
//
// The MFMA operands need no LDS image for the rows: In_c is loaded straight into the P layout
// (lane = feature, registers = rows in accumulator order) and split in registers — the B operand
// over the chunk's 64 rows — while Â_tc is the A operand with its sources in the matching perm16
// order (the fused backward's G = Â^T dZ product, stack3_bwd.hip). The sum over a row's entries
// is therefore not in CSR order: fp32-accurate, not bitwise the gather's (tests: oracle bar).
//
// Chunks are the natural 64-row tiles; a chunk whose tile is masked out holds no source of a
// selected tile (an edge between two tiles marks both open) and is skipped, so rows no launch of
// this layer wrote are never read. A tile whose window spans more than max_chunks chunks or that
// holds more than kWinCap entries falls back to the per-row gather (CSR order).
#include "s3_util.h"

namespace {
using namespace lgnn_s3;

constexpr int kWinCap = 2048;           // entries of a tile held in registers (8 per thread)
constexpr int kWinPer = kWinCap / NT;

struct WinSmem {
  float scr[TM * TM];                 // fp32 Â_tc [target][source] while it is summed
  unsigned char Adj[3][ADJ_PLANE];    // its planes [target][perm16 source]
  int rp[TM + 1];
  int red[2][NT / 64];
  int any;
};

// rows of chunk c (c0 = first row) in P layout for feature column n: v[a][r] = In[c0 + m][n],
// m = 32 a + (r & 3) + 8 (r >> 2) + 4 h; rows past M read 0 (descriptor range)
__device__ __forceinline__ void load_chunk_p(f32x16 (&v)[2], const float* In, int64_t M,
                                             int64_t c0, int n, int h) {
  const int64_t rem = M - c0;
  const Buf b = mkbuf(In + c0 * WP, rem > 0 ? rem * WP * 4 : 0);
  const int vb = (4 * h * WP + n) * 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mc = 32 * a + (r & 3) + 8 * (r >> 2);
      v[a][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b, vb + mc * WP * 4,
                                                                               0, 0));
    }
}

__global__ __launch_bounds__(NT, 2) void k_win_agg(const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ col,
                                                   const float* __restrict__ w, int64_t M,
                                                   const float* __restrict__ In,
                                                   float* __restrict__ Out,
                                                   const int32_t* __restrict__ tmask, int want,
                                                   int max_chunks) {
  __shared__ __attribute__((aligned(16))) WinSmem sm;
  const int64_t ntiles = (M + TM - 1) / TM;
  const Buf bO = mkbuf(Out, M * WP * 4);
  for (int64_t t = seek_tile(xcd_block(), ntiles, tmask, want); t < ntiles;
       t = seek_tile(t + gridDim.x, ntiles, tmask, want)) {
    const int64_t r0 = t * TM;
    const int tq = threadIdx.x;
    const int lane = tq & 63, wv = tq >> 6, h = lane >> 5, li = lane & 31;
    const int n = 32 * wv + li;
    if (tq <= TM) sm.rp[tq] = rowptr[r0 + tq < M ? r0 + tq : M];
    __syncthreads();
    const int E0 = sm.rp[0], ne = sm.rp[TM] - E0;
    // the tile's entries in registers: source, weight and target row (binary search of rp)
    int ec[kWinPer], et[kWinPer];
    float ew[kWinPer];
    int lo = INT32_MAX, hi = -1;
    const bool fits = ne <= kWinCap;
    if (fits) {
#pragma unroll
      for (int u = 0; u < kWinPer; ++u) {
        const int j = tq + u * NT;
        ec[u] = -1;
        et[u] = 0;
        ew[u] = 0.f;
        if (j < ne) {
          const int e = E0 + j;
          ec[u] = col[e];
          ew[u] = w ? w[e] : 1.f;
          int a = 0, b = TM;
#pragma unroll
          for (int it = 0; it < 6; ++it) {
            const int mid = (a + b) >> 1;
            if (sm.rp[mid] <= e) a = mid;
            else b = mid;
          }
          et[u] = a;
          lo = ec[u] < lo ? ec[u] : lo;
          hi = ec[u] > hi ? ec[u] : hi;
        }
      }
    }
    // the window: chunks lo >> 6 .. hi >> 6 (block min / max)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    if (lane == 0) {
      sm.red[0][wv] = lo;
      sm.red[1][wv] = hi;
    }
    __syncthreads();
    lo = sm.red[0][0];
    hi = sm.red[1][0];
#pragma unroll
    for (int q = 1; q < NT / 64; ++q) {
      lo = sm.red[0][q] < lo ? sm.red[0][q] : lo;
      hi = sm.red[1][q] > hi ? sm.red[1][q] : hi;
    }
    const int c_lo = hi < 0 ? 0 : lo >> 6, c_hi = hi < 0 ? -1 : hi >> 6;
    if (!fits || c_hi - c_lo + 1 > max_chunks) {
      // fallback: half wave per row, CSR order, source rows from global memory
      const int hw = tq >> 5;
      for (int rr = hw; rr < TM; rr += NT / 32) {
        const int e0 = sm.rp[rr], e1 = sm.rp[rr + 1];
        f32x4 acc = zero4();
        for (int e = e0; e < e1; ++e) {
          const float wv2 = w ? w[e] : 1.f;
          acc += wv2 * ld4(In + (int64_t)col[e] * WP + 4 * li);
        }
        if (r0 + rr < M) st4(Out + (r0 + rr) * WP + 4 * li, acc);
      }
      __syncthreads();
      continue;
    }
    f32x16 s[2] = {f32x16{}, f32x16{}};
    f32x16 hraw[2];
    int c = c_lo;
    auto selected = [&](int ch) { return !tmask || ((tmask[ch] != 0) == (want != 0)); };
    while (c <= c_hi && !selected(c)) ++c;
    if (c <= c_hi) load_chunk_p(hraw, In, M, (int64_t)c * TM, n, h);
    while (c <= c_hi) {
      int cn = c + 1;
      while (cn <= c_hi && !selected(cn)) ++cn;
      // Â_tc: zero, scatter the entries with a source in chunk c (equal duplicates carry equal
      // weights: the LDS float adds are order independent), split into planes
#pragma unroll
      for (int i = 0; i < TM * TM / 4 / NT; ++i) st4(sm.scr + 4 * (tq + i * NT), zero4());
      __syncthreads();
      int mine = 0;
#pragma unroll
      for (int u = 0; u < kWinPer; ++u)
        if ((ec[u] >> 6) == c) {
          atomicAdd(&sm.scr[et[u] * TM + (ec[u] & 63)], ew[u]);
          mine = 1;
        }
      const int any = __syncthreads_or(mine);
      if (any) {
        const int am = tq >> 2, aq = tq & 3;
        f32x4 av[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = ld4(sm.scr + am * TM + 16 * aq + 4 * i);
        float f[16];
#pragma unroll
        for (int y = 0; y < 16; ++y) {
          const int src = perm16(y);
          f[y] = av[src >> 2][src & 3];
        }
        uint32_t q3[3][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const Split2 s2 = split2(f[2 * i], f[2 * i + 1]);
#pragma unroll
          for (int p = 0; p < 3; ++p) q3[p][i] = s2.p[p];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          unsigned char* dst = sm.Adj[p] + am * ADJ_LD * 2 + 32 * aq;
          *reinterpret_cast<u32x4*>(dst) = u32x4{q3[p][0], q3[p][1], q3[p][2], q3[p][3]};
          *reinterpret_cast<u32x4*>(dst + 16) = u32x4{q3[p][4], q3[p][5], q3[p][6], q3[p][7]};
        }
      }
      // this chunk's rows -> operand fragments; the next chunk's rows are issued now
      u32x4 hf[4][3];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const f32x16& pa = hraw[st >> 1];
        const int rb = 8 * (st & 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const Split2 s2 = split2(pa[rb + 2 * i], pa[rb + 2 * i + 1]);
#pragma unroll
          for (int p = 0; p < 3; ++p) hf[st][p][i] = s2.p[p];
        }
      }
      if (cn <= c_hi) load_chunk_p(hraw, In, M, (int64_t)cn * TM, n, h);
      __syncthreads();  // planes written
      if (any) {
#pragma unroll
        for (int st = 0; st < 4; ++st) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int off = (32 * q + li) * ADJ_LD * 2 + 16 * (2 * st + h);
            u32x4 at[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) at[p] = lds16(sm.Adj[p] + off);
            s[q] = mfma_s3(at, hf[st], s[q]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      c = cn;
    }
    // S (P layout: feature n on the lane, target rows in the registers) -> Out; rows past M are
    // dropped by the descriptor range
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 32 * q + (r & 3) + 8 * (r >> 2) + 4 * h;
        // (__float_as_uint, not __builtin_bit_cast on the vector-element lvalue: this clang
        // bit-casts from the vector's first element there)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s[q][r]), bO,
                                              (int)(((r0 + m) * WP + n) * 4), 0, 0);
      }
    __syncthreads();  // sm.rp / scr / Adj are rewritten by the next tile
  }
}

}  // namespace

extern "C" int lgnn_window_aggregate(const int32_t* rowptr, const int32_t* col, const float* w,
                                     int64_t M, const float* in, int width, float* out,
                                     const int32_t* tile_mask, int want, int max_chunks,
                                     void* stream) {
  if (M < 0 || !rowptr || !col || !in || !out || width != WP || max_chunks < 1) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  if (M * WP * 4 >= ((int64_t)1 << 32)) return LGNN_EINVAL;  // 32-bit buffer offsets
  const int64_t ntiles = (M + TM - 1) / TM;
  const unsigned grid = (unsigned)(ntiles < 512 ? ntiles : 512);
  hipLaunchKernelGGL(k_win_agg, dim3(grid), dim3(NT), 0, as_stream(stream), rowptr, col, w, M, in,
                     out, tile_mask, want, max_chunks);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
