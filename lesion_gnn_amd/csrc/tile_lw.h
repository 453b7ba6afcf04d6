// Layer-wise node-tile bodies (the open-tile path): forward Y = act(P(X) W^T + b) with optional
// S_out = P(X), and its backward, for every tile selected by a tile mask, persistent over the
// grid. Shared by the layer-wise kernels (tile.hip k_fwd / k_bwd) and by the fused GCN stack
// kernels' open-tile phase (stack3.hip, stack3_bwd.hip), which call them with their own LDS.
#pragma once
#include <type_traits>

#include "tile_util.h"

namespace lgnn_tile {

// sum_{e in row rr} w_e * X[c_e][4li..], in CSR order.
// Local path: every source row is in the LDS image A; per entry one ds_read_b64 (offset,
// weight), one ds_read_b128 and two packed FMAs, no bounds logic and no global access (so no
// vmcnt wait that would drain the prefetch loads and row stores in flight).
template <int UB = EB>
__device__ __forceinline__ f32x4 agg_row_local(const TileIdx& ti, int rr, const float* A) {
  static_assert(UB <= EB, "row batches read at most EB padding entries");
  const int li = threadIdx.x & 31;
  const int eb = ti.rp[0];
  const int e0 = ti.rp[rr] - eb, e1 = ti.rp[rr + 1] - eb;
  f32x4 acc = zero4();
  for (int e = e0; e < e1; e += UB) {
    int2 p[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) p[u] = ti.ow[e + u];
    f32x4 v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) v[u] = ld4(A + p[u].x + 4 * li);
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const float wv = e + u < e1 ? __int_as_float(p[u].y) : 0.f;
      acc += wv * v[u];
    }
  }
  return acc;
}

// Staged-index global path (AGG_GROWS: sources outside the tile, the block within CAPE_LW): the
// entries from LDS as the local path reads them, the source rows gathered from global memory —
// one dependent round trip per EB batch instead of two; same order and arithmetic.
template <int UB = EB>
__device__ __forceinline__ f32x4 agg_row_grows(const TileIdx& ti, int rr,
                                               const float* __restrict__ X, int K, int kc) {
  static_assert(UB <= EB, "row batches read at most EB padding entries");
  const int eb = ti.rp[0];
  const int e0 = ti.rp[rr] - eb, e1 = ti.rp[rr + 1] - eb;
  f32x4 acc = zero4();
  for (int e = e0; e < e1; e += UB) {
    int2 p[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) p[u] = ti.ow[e + u];
    f32x4 v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) v[u] = ld4(X + (int64_t)p[u].x * K + kc);
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const float wv = e + u < e1 ? __int_as_float(p[u].y) : 0.f;
      acc += wv * v[u];
    }
  }
  return acc;
}

// Global path (graphs straddling tiles with more than CAPE_LW entries): CSR and source rows read
// from global memory, same order and arithmetic as the local path (bitwise-identical sums).
__device__ __forceinline__ f32x4 agg_row_global(const TileIdx& ti, int rr,
                                                const float* __restrict__ X, int K, int kc,
                                                const int32_t* __restrict__ col,
                                                const float* __restrict__ w) {
  const int e0 = ti.rp[rr], e1 = ti.rp[rr + 1];
  f32x4 acc = zero4();
  for (int e = e0; e < e1; e += EB) {
    int c[EB];
    float ww[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const bool ok = e + u < e1;
      const int ee = ok ? e + u : e0;
      c[u] = col[ee];
      ww[u] = ok ? (w ? w[ee] : 1.f) : 0.f;
    }
    f32x4 v[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) v[u] = ld4(X + (int64_t)c[u] * K + kc);
#pragma unroll
    for (int u = 0; u < EB; ++u) acc += ww[u] * v[u];
  }
  return acc;
}

// ------------------------------------------------------------------------------------------
// forward: Y = act(P(X) W^T + b); optional S_out = P(X)
// ------------------------------------------------------------------------------------------
template <bool GATHER, int ACT, int BNM = BN_NONE>
__device__ __forceinline__ void fwd_tiles(float* A, float* S, TileIdx& ti,
                                          const float* __restrict__ X, int64_t M, int K,
                                          const int32_t* __restrict__ rowptr,
                                          const int32_t* __restrict__ col,
                                          const float* __restrict__ w, float self_scale,
                                          const float* __restrict__ W,
                                          const float* __restrict__ b, int N,
                                          float* __restrict__ Y, float* __restrict__ S_out,
                                          const int32_t* __restrict__ tmask, int want,
                                          const BnFuse& bn = BnFuse{}) {
  static_assert(BNM == BN_NONE || BNM == BN_STATS || (BNM == BN_IN && !GATHER), "");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31, hw = wave * 2 + h;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int n = wave * 32 + li;
  const int ncl = n < N ? n : N - 1;
  const bool wave_active = wave * 32 < N;
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};  // BN_STATS
  int64_t t = seek_tile(xcd_block(), ntiles, tmask, want);  // XCD-contiguous tiles
  if (t >= ntiles) {
    if constexpr (BNM == BN_STATS) bn_part_write(reinterpret_cast<double*>(A), s0, s1, bn.part, N);
    return;
  }
  // BN_IN: the input columns' constants (k = 4 li ..)
  f32x4 bsc = {}, bsh = {};
  if constexpr (BNM == BN_IN) {
    const int kq = 4 * li < K ? 4 * li : K - 4;
    bsc = ld4(bn.scale + kq);
    bsh = ld4(bn.shift + kq);
  }
  float bf[64];
  load_wfrag(bf, W, N, K, n, h);
  const float bias = b ? b[ncl] : 0.f;
  const int kc = 4 * li < K ? 4 * li : K - 4;
  const Buf bX = mkbuf(X, M * K * 4), bY = mkbuf(Y, M * N * 4);
  const Buf bS = mkbuf(S_out, S_out ? M * K * 4 : 0);
  float* Ain = GATHER ? S : A;  // MFMA A-operand image

  if constexpr (ABL & 32) {  // desync experiment: odd blocks start half a tile late
    if (blockIdx.x & 1) {
      for (int i = 0; i < 4; ++i) __builtin_amdgcn_s_sleep(127);
    }
  }
  // pipeline prologue: the first tile's rows and index block
  f32x4 xr[8];
  IdxRegsLw R;
  if constexpr (!(ABL & 16)) load_rows(xr, bX, K, (int)(t * TM));
  if constexpr (GATHER && !(ABL & 2)) {
    idx_load_head(R, rowptr, M, t * TM);
    idx_load_body(R, col, w);
  }
  for (; t < ntiles; t = seek_tile(t + gridDim.x, ntiles, tmask, want)) {
    const int64_t r0 = t * TM;
    const int64_t tn = seek_tile(t + gridDim.x, ntiles, tmask, want);
    const bool has_next = tn < ntiles;
    int agg = AGG_LOCAL;
    if constexpr (ABL & 16) {
#pragma unroll
      for (int it = 0; it < 8; ++it) xr[it] = zero4();
    }
    if constexpr (BNM == BN_IN) {  // A = ELU(X * scale + shift) * mask, also to act_out
      const bool kin = 4 * li < K;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        const int64_t row = r0 + rr;
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = elu_f(fmaf(xr[it][j], bsc[j], bsh[j]));
        const bool ok = kin && row < M;
        if (bn.mask && ok) v *= ld4(bn.mask + row * K + 4 * li);
        if (ok) st4(bn.act_out + row * K + 4 * li, v);
        st4(A + rr * LDS + 4 * li, sel4(ok, v));
      }
    } else {
      store_rows_lds(A, xr, M, K, r0);
    }
    if constexpr (GATHER && !(ABL & 2)) agg = idx_store(ti, R, r0);
    __syncthreads();
    // prefetch: next tile's rows and index head fly during this tile's aggregation and MFMAs
    if (has_next) {
      if constexpr (!(ABL & 16)) load_rows(xr, bX, K, (int)(tn * TM));
      if constexpr (GATHER && !(ABL & 2)) idx_load_head(R, rowptr, M, tn * TM);
    }
    if constexpr (GATHER) {
      auto agg_tile = [&](auto mode_tag) {
        constexpr int MODE = decltype(mode_tag)::value;
#pragma unroll 1
        for (int it = 0; it < 8; ++it) {
          const int rr = hw + 8 * it;
          f32x4 a;
          if constexpr (ABL & 2) a = ld4(A + rr * LDS + 4 * li);
          else if constexpr (MODE == AGG_LOCAL) a = agg_row_local(ti, rr, A);
          else if constexpr (MODE == AGG_GROWS) a = agg_row_grows(ti, rr, X, K, kc);
          else a = agg_row_global(ti, rr, X, K, kc, col, w);
          if (self_scale != 0.f) a += self_scale * ld4(A + rr * LDS + 4 * li);
          a = sel4(4 * li < K && r0 + rr < M, a);
          st4(S + rr * LDS + 4 * li, a);
          if (!(ABL & 4) && S_out && 4 * li < K)
            bst4(bS, (int)((r0 + rr) * K + 4 * li) * 4, a);
        }
      };
      if (agg == AGG_LOCAL) agg_tile(std::integral_constant<int, AGG_LOCAL>{});
      else if (agg == AGG_GROWS) agg_tile(std::integral_constant<int, AGG_GROWS>{});
      else agg_tile(std::integral_constant<int, AGG_GLOBAL>{});
      if constexpr (!(ABL & 2)) {
        if (has_next) idx_load_body(R, col, w);
      }
      __syncthreads();
    }
    f32x16 acc0 = {}, acc1 = {};
    if (wave_active && !(ABL & 1)) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const f32x4 a0 = ld4(Ain + li * LDS + 64 * h + 4 * q);
        const f32x4 a1 = ld4(Ain + (32 + li) * LDS + 64 * h + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc0 = mfma32(a0[j], bf[4 * q + j], acc0);
          acc1 = mfma32(a1[j], bf[4 * q + j], acc1);
        }
      }
    }
    __syncthreads();  // every wave is done reading A / S
    // epilogue staged in A as [row][col], then whole-row stores
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
      float v0 = acc0[r] + bias, v1 = acc1[r] + bias;
      if (ACT == LGNN_ACT_ELU) {
        v0 = elu_f(v0);
        v1 = elu_f(v1);
      }
      A[rl * LDS + n] = v0;
      A[(32 + rl) * LDS + n] = v1;
    }
    __syncthreads();
    if (4 * li < N && !(ABL & 4)) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        const f32x4 v = ld4(A + rr * LDS + 4 * li);
        bst4(bY, (int)((r0 + rr) * N + 4 * li) * 4, v);
        if constexpr (BNM == BN_STATS) {
          if (r0 + rr < M) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              s0[j] += (double)v[j];
              s1[j] += (double)v[j] * (double)v[j];
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if constexpr (BNM == BN_STATS) bn_part_write(reinterpret_cast<double*>(A), s0, s1, bn.part, N);
}

// ------------------------------------------------------------------------------------------
// backward: dZ = G ⊙ act'(H); dW += dZ^T S (S = X, direct); db += colsum dZ; dXpre = dZ W
// ------------------------------------------------------------------------------------------
template <int GMODE, int ACT, bool DX, int BNM = BN_NONE>
__device__ __forceinline__ void bwd_tiles(
    float* A, float* C, TileIdx& ti,
    const float* __restrict__ dY, const int64_t* __restrict__ batch,
    const int32_t* __restrict__ gptr, int pool_mean, const int32_t* __restrict__ tptr,
    const int32_t* __restrict__ tidx, const float* __restrict__ tw, float tself,
    const float* __restrict__ H, const float* __restrict__ X, int64_t M, int K,
    const float* __restrict__ W, int N, float* __restrict__ dXpre, float* __restrict__ dWp,
    float* __restrict__ dbp, const int32_t* __restrict__ tmask, int want, int accumulate,
    const float* __restrict__ dlog = nullptr, const float* __restrict__ Wout = nullptr,
    int nclass = 0, const BnFuse& bn = BnFuse{}, const CeSrc ce = CeSrc{}) {
  static_assert(BNM == BN_NONE || (BNM == BN_GSTATS && DX) ||
                    (BNM == BN_GIN && GMODE == LGNN_GRAD_DIRECT && ACT == LGNN_ACT_NONE), "");
  // GRAD_POOL with dlog: the pooled-output gradient is formed on the fly from the logits'
  // gradient, dP[g][n] = sum_c dlog[g][c] Wout[c][n] (out_proj backward, nclass classes)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, li = lane & 31, hw = wave * 2 + h;
  const int64_t ntiles = (M + TM - 1) / TM;
  const int oc = 4 * li < N ? 4 * li : N - 4;
  const bool oin = 4 * li < N;

  const Buf bdY = mkbuf(dY, M * N * 4), bH = mkbuf(H, H ? M * N * 4 : 0);
  const Buf bX = mkbuf(X, M * K * 4), bdX = mkbuf(dXpre, dXpre ? M * K * 4 : 0);
  f32x16 dw[4] = {{}, {}, {}, {}};
  float dbacc = 0.f;
  const int kx = 32 * wave + li;
  const int kxc = kx < K ? kx : K - 1;
  // BatchNorm constants of this lane's 4 columns: the dY columns (BN_GIN) or the dX columns
  // (BN_GSTATS)
  f32x4 bsc = {}, bsh = {}, bmu = {}, bis = {}, bmg = {}, bmgx = {};
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};
  if constexpr (BNM != BN_NONE) {
    const int W4 = BNM == BN_GIN ? N : K;
    const int cq = 4 * li < W4 ? 4 * li : W4 - 4;
    bsc = ld4(bn.scale + cq);
    bsh = ld4(bn.shift + cq);
    bmu = ld4(bn.mean + cq);
    bis = ld4(bn.invstd + cq);
    if (BNM == BN_GIN && bn.training) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bmg[j] = (float)(bn.sums[cq + j] / bn.count);
        bmgx[j] = (float)(bn.sums[N + cq + j] / bn.count);
      }
    }
  }

  // pipeline prologue (TRANSPOSE): the first tile's dY rows and transpose-CSR index block.
  // With the BN_GSTATS epilogue the next tile's rows are NOT prefetched into registers (PREF):
  // their 32 VGPRs live across the MFMAs pushed that variant past 256 and spilled ~96 (GIN
  // Lin2 backward under the model-wide node); its rows are loaded at the tile's start instead.
#ifndef LGNN_TPREF_ALL
#define LGNN_TPREF_ALL 0
#endif
  constexpr bool PREF =
      !(GMODE == LGNN_GRAD_TRANSPOSE && (BNM == BN_GSTATS || LGNN_TPREF_ALL));
  f32x4 dr[8];
  IdxRegsLw R;
  const int64_t tfirst = seek_tile(xcd_block(), ntiles, tmask, want);  // XCD-contiguous tiles
  if constexpr (GMODE == LGNN_GRAD_TRANSPOSE) {
    const int64_t t0 = tfirst;
    if (t0 < ntiles) {
      if constexpr (!(ABL & 16) && PREF) load_rows(dr, bdY, N, (int)(t0 * TM));
      if constexpr (!(ABL & 2)) {
        idx_load_head(R, tptr, M, t0 * TM);
        idx_load_body(R, tidx, tw);
      }
    }
  }

  for (int64_t t = tfirst; t < ntiles; t = seek_tile(t + gridDim.x, ntiles, tmask, want)) {
    const int64_t r0 = t * TM;
    const int64_t tn = seek_tile(t + gridDim.x, ntiles, tmask, want);
    const bool has_next = tn < ntiles;
    // ---- dZ tile -> C
    if constexpr (GMODE == LGNN_GRAD_TRANSPOSE) {
      int agg = AGG_LOCAL;
      if constexpr (ABL & 16) {
#pragma unroll
        for (int it = 0; it < 8; ++it) dr[it] = zero4();
      } else if constexpr (!PREF) {
        load_rows(dr, bdY, N, (int)r0);
      }
      store_rows_lds(A, dr, M, N, r0);
      if constexpr (!(ABL & 2)) agg = idx_store(ti, R, r0);
      // this tile's H rows (ELU') are issued before the barrier so they land during it
      f32x4 hv[8];
      if constexpr (ACT == LGNN_ACT_ELU) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int64_t row = r0 + hw + 8 * it;
          hv[it] = (ABL & 16) ? zero4() : bld4(bH, (int)(row * N + oc) * 4);
        }
      }
      __syncthreads();
      // prefetch: next tile's dY rows and index head
      if (has_next) {
        if constexpr (!(ABL & 16) && PREF) load_rows(dr, bdY, N, (int)(tn * TM));
        if constexpr (!(ABL & 2)) idx_load_head(R, tptr, M, tn * TM);
      }
      auto agg_tile = [&](auto mode_tag) {
        constexpr int MODE = decltype(mode_tag)::value;
#pragma unroll 1
        for (int it = 0; it < 8; ++it) {
          const int rr = hw + 8 * it;
          const int64_t row = r0 + rr;
          f32x4 g;
          if constexpr (ABL & 2) g = ld4(A + rr * LDS + 4 * li);
          else if constexpr (MODE == AGG_LOCAL) g = agg_row_local(ti, rr, A);
          else if constexpr (MODE == AGG_GROWS) g = agg_row_grows(ti, rr, dY, N, oc);
          else g = agg_row_global(ti, rr, dY, N, oc, tidx, tw);
          if (tself != 0.f) g += tself * ld4(A + rr * LDS + 4 * li);
          if constexpr (ACT == LGNN_ACT_ELU) {
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] *= elu_grad_from_out(hv[it][j]);
          }
          st4(C + rr * LDS + 4 * li, sel4(oin && row < M, g));
        }
      };
      if (agg == AGG_LOCAL) agg_tile(std::integral_constant<int, AGG_LOCAL>{});
      else if (agg == AGG_GROWS) agg_tile(std::integral_constant<int, AGG_GROWS>{});
      else agg_tile(std::integral_constant<int, AGG_GLOBAL>{});
      if constexpr (!(ABL & 2)) {
        if (has_next) idx_load_body(R, tidx, tw);
      }
    } else {
      f32x4 g[8], hv[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int64_t row = r0 + hw + 8 * it;
        const int64_t rc = row < M ? row : M - 1;
        if constexpr (GMODE == LGNN_GRAD_DIRECT) {
          g[it] = ld4(dY + rc * N + oc);
          if constexpr (BNM == BN_GIN) hv[it] = ld4(bn.Z + rc * N + oc);  // BN input rows
        } else {
          const int64_t gi = batch[rc];
          if (dlog || ce.pm) {  // k_head_bwd's arithmetic: an fmaf chain over the classes in order
            f32x4 acc = zero4();
            for (int c = 0; c < nclass; ++c) {
              // the logits gradient as given, or formed from the CE forward (bitwise the same)
              const float d = ce.pm ? ce_dlogit(ce, gi, c) : dlog[gi * nclass + c];
              const f32x4 wv = ld4(Wout + (int64_t)c * N + oc);
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[j] = fmaf(d, wv[j], acc[j]);
            }
            g[it] = acc;
          } else {
            g[it] = ld4(dY + gi * N + oc);
          }
          if (pool_mean) {
            const int cnt = gptr[gi + 1] - gptr[gi];
            g[it] = g[it] / (float)(cnt > 0 ? cnt : 1);
          }
        }
        if constexpr (ACT == LGNN_ACT_ELU) hv[it] = ld4(H + rc * N + oc);
      }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = hw + 8 * it;
        f32x4 v = g[it];
        if constexpr (ACT == LGNN_ACT_ELU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] *= elu_grad_from_out(hv[it][j]);
        }
        if constexpr (BNM == BN_GIN) {  // dZ = BN backward of the ELU(BN(Z)) * mask output
          const int64_t row = r0 + rr;
          const int64_t rc = row < M ? row : M - 1;
          const f32x4 m = bn.mask ? ld4(bn.mask + rc * N + oc) : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float z = hv[it][j];
            const float gg = v[j] * bn_elu_grad(z, bsc[j], bsh[j]) * m[j];
            if (bn.training) {
              const float xh = (z - bmu[j]) * bis[j];
              v[j] = bsc[j] * (gg - bmg[j] - xh * bmgx[j]);
            } else {
              v[j] = bsc[j] * gg;
            }
          }
        }
        st4(C + rr * LDS + 4 * li, sel4(oin && r0 + rr < M, v));
      }
    }
    // ---- S tile -> A (A's raw dY image is dead once every wave has passed this barrier)
    f32x4 sr[8];
    if constexpr (ABL & 16) {
#pragma unroll
      for (int it = 0; it < 8; ++it) sr[it] = zero4();
    } else {
      load_rows(sr, bX, K, (int)r0);
    }
    __syncthreads();
    store_rows_lds(A, sr, M, K, r0);
    __syncthreads();
    if (tid < 128) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll 8
      for (int r = 0; r < TM; r += 2) {
        s0 += C[r * LDS + tid];
        s1 += C[(r + 1) * LDS + tid];
      }
      dbacc += s0 + s1;
    }
    // DX B-fragment W[o = 64h + s][kx], re-read per tile (L2) so it is not live during the
    // aggregation phase; its latency hides under the dW MFMAs.
    // Buffer loads: per-lane voffset (column kx, half-wave row block 64h) + uniform soffset
    // (row s); rows o >= N fall outside the descriptor's range and read 0.
    float wt[64];
    if constexpr (DX) {
      const __amdgpu_buffer_rsrc_t wr =
          __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, N * K * 4, 0x00020000);
      const int voff = (64 * h * K + kxc) * 4;
#pragma unroll
      for (int s = 0; s < 64; ++s) {
        const float v = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(wr, voff, s * K * 4, 0));
        wt[s] = kx < K ? v : 0.f;
      }
    }
    // dW[o][k] += sum_m dZ[m][o] S[m][k]; wave owns o in [32w, 32w+32)
#pragma unroll 4
    for (int s = 0; s < (ABL & 1 ? 0 : TM / 2); ++s) {
      const int m = 2 * s + h;
      const float a = C[m * LDS + 32 * wave + li];
#pragma unroll
      for (int j = 0; j < 4; ++j) dw[j] = mfma32(a, A[m * LDS + 32 * j + li], dw[j]);
    }
    if constexpr (DX) {
      f32x16 x0 = {}, x1 = {};
#pragma unroll
      for (int q = 0; q < (ABL & 1 ? 0 : 16); ++q) {
        const f32x4 a0 = ld4(C + li * LDS + 64 * h + 4 * q);
        const f32x4 a1 = ld4(C + (32 + li) * LDS + 64 * h + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x0 = mfma32(a0[j], wt[4 * q + j], x0);
          x1 = mfma32(a1[j], wt[4 * q + j], x1);
        }
      }
      __syncthreads();  // dW reads of A are done
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        A[rl * LDS + kx] = x0[r];
        A[(32 + rl) * LDS + kx] = x1[r];
      }
      __syncthreads();
      if (4 * li < K && !(ABL & 4)) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int rr = hw + 8 * it;
          const f32x4 v = ld4(A + rr * LDS + 4 * li);
          bst4(bdX, (int)((r0 + rr) * K + 4 * li) * 4, v);
          if constexpr (BNM == BN_GSTATS) {  // the BN backward's batch sums over dX = dA
            const int64_t row = r0 + rr;
            if (row < M) {
              const f32x4 z = ld4(bn.Z + row * K + 4 * li);
              const f32x4 m = bn.mask ? ld4(bn.mask + row * K + 4 * li)
                                      : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const float gg = v[j] * bn_elu_grad(z[j], bsc[j], bsh[j]) * m[j];
                const float xh = (z[j] - bmu[j]) * bis[j];
                s0[j] += (double)gg;
                s1[j] += (double)gg * (double)xh;
              }
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if constexpr (BNM == BN_GSTATS) bn_part_write(reinterpret_cast<double*>(A), s0, s1, bn.part, K);
  // accumulate: add into slot blockIdx.x (written by the fused stack backward) if this
  // workgroup processed any tile; otherwise leave the slot untouched. accumulate = 2: a slot
  // whose skip word is set was not written by the fused kernel: write it (zeros when this
  // workgroup processed no tile)
  const bool skipped = accumulate == 2 && blockIdx.x < LGNN_SLOT_FLAGS &&
                       tmask[ntiles + LGNN_SLOT_FLAG0 + blockIdx.x] != 0;
  if (accumulate && tfirst >= ntiles && !skipped) return;
  const bool add = accumulate && !skipped;
  float* slab = dWp + (int64_t)blockIdx.x * N * K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 32 * j + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (o < N && k < K) {
        float* p = slab + (int64_t)o * K + k;
        *p = add ? *p + dw[j][r] : dw[j][r];
      }
    }
  }
  if (dbp && tid < N) {
    float* p = dbp + (int64_t)blockIdx.x * N + tid;
    *p = add ? *p + dbacc : dbacc;
  }
}

}  // namespace lgnn_tile
