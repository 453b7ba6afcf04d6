// GATConv attention kernels (PyG 2.5.1 GATConv(d1, d2 // H, heads=H, dropout=p), reference
// gat.py:31; concat=True, negative_slope=0.2, add_self_loops=True, bias=True), forward and
// backward, fp32.
//
//   a_s[j,h] = <xp_j[h], att_src[h]>,  a_d[i,h] = <xp_i[h], att_dst[h]>
//   e_ij = leaky_relu(a_s[j,h] + a_d[i,h]);  alpha_ij = exp(e_ij - max_i e) / (sum_i exp(.) + 1e-16)
//   out_i[h] = sum_j alpha_ij * mask_ij * xp_j[h]  (+ bias, + ELU of the model, gat.py:51)
//
// Layout: XP [M, H*C] row-major (the lin output viewed [M, H, C]); per-edge arrays [cap, H] in
// target-CSR order. Work mapping: one half wave (32 lanes) per node row, a lane owns 4
// consecutive features (float4) of a 128-feature strip, so a head (C features, C | 128) is C/4
// adjacent lanes and per-head dot products are xor-butterflies inside the half wave. Rows are
// visited in CSR order (= PyG's edge order; the self loop is last), so sums follow PyG's
// scatter_add_ order.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int RB = 8;       // rows per block (8 half waves)
constexpr int EB = 8;       // edges in flight per batch
constexpr int MAXS = 4;     // feature strips of 128 (H*C <= 512)
constexpr float EPS16 = 1e-16f;

// optional occupancy floor of the row kernels (waves per SIMD; 0 = the compiler's choice). Forcing
// one below their register demand spills, which costs far more than the waves gain (C3 step
// 0.73 -> 1.32 ms at 6 waves); the 32-bit buffer offsets are what lowered the demand
#ifndef LGNN_GAT_WPE
#define LGNN_GAT_WPE 0
#endif
#ifndef LGNN_GAT_NODE_XCD
#define LGNN_GAT_NODE_XCD 1
#endif
#if LGNN_GAT_WPE > 0
#define GAT_OCC __attribute__((amdgpu_waves_per_eu(LGNN_GAT_WPE)))
#else
#define GAT_OCC
#endif

__device__ __forceinline__ float leaky(float v, float slope) { return v > 0.f ? v : v * slope; }
// a value the compiler cannot see into: a sum of such terms is never fused with their products,
// so kernels whose instruction selection differs still round it alike (the bitwise pairs)
__device__ __forceinline__ float opaque(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Raw buffer access (SGPR descriptor + 32-bit byte offset): one VGPR per gathered address instead
// of two, which is what bounds these gather kernels' registers (8 source rows in flight). Every
// array addressed this way is < 4 GiB (checked on the host, bytes_ok).
typedef __amdgpu_buffer_rsrc_t Buf;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Buf mkbuf(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(uint32_t)bytes,
                                           0x00020000);
}
__device__ __forceinline__ f32x4 bld4(Buf r, uint32_t off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ float bld1(Buf r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ int bldi(Buf r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ void bst1(Buf r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, off, 0, 0);
}
__device__ __forceinline__ void bst4(Buf r, uint32_t off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

// sum over the G = C/4 lanes of a head group (all lanes receive the sum). Within a 16-lane DPP
// row the butterfly runs on DPP moves instead of LDS permutes: xor 1 / xor 2 are quad
// permutations; at the xor-4 (xor-8) stage every lane of a 4 (8)-lane block already holds that
// block's sum, so the half-row (row) mirror reads a lane of the partner block with the same
// value the xor partner holds — the same additions in the same order, bitwise.
#ifndef LGNN_GAT_DPP
#define LGNN_GAT_DPP 1
#endif
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float group_sum(float v, int G) {
#if LGNN_GAT_DPP
  if (G >= 2) v += dppf<0xB1>(v);   // quad_perm [1, 0, 3, 2]: lane ^ 1
  if (G >= 4) v += dppf<0x4E>(v);   // quad_perm [2, 3, 0, 1]: lane ^ 2
  if (G >= 8) v += dppf<0x141>(v);  // row_half_mirror
  if (G >= 16) v += dppf<0x140>(v); // row_mirror
  if (G >= 32) v += __shfl_xor(v, 16, 64);
  return v;
#else
  for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
#endif
}

__device__ __forceinline__ float dot4(f32x4 a, f32x4 b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}

struct Lane {
  int li, hw;
  int64_t row;
};

__device__ __forceinline__ Lane lane_row() {
  Lane l;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  l.li = lane & 31;
  l.hw = wave * 2 + (lane >> 5);
  l.row = xcd_block() * RB + l.hw;
  return l;
}

// Feature passes. A half wave covers NS strips of 128 features per pass: NS = 1 when C <= 128
// (a pass holds 128/C whole heads; head group = C/4 adjacent lanes), NS = C/128 when C > 128
// (a pass is one head; its dot products add the NS strip partials, then all 32 lanes).
template <int NS>
struct Pass {
  int f[NS];     // feature of sub-strip s for this lane
  bool act[NS];  // f < HC
  int fc[NS];    // clamped feature (loads stay in bounds)
  int head, G;
  bool leader;
  Pass() = default;
  __device__ __forceinline__ Pass(int p, int li, int HC, int C) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      f[s] = p * 128 * NS + s * 128 + 4 * li;
      act[s] = f[s] < HC;
      fc[s] = act[s] ? f[s] : HC - 4;
    }
    head = fc[0] / C;
    G = NS == 1 ? C / 4 : 32;
    leader = act[0] && (li % G) == 0;
  }
};

__device__ __forceinline__ int num_passes(int HC, int NS) { return (HC + 128 * NS - 1) / (128 * NS); }

// ------------------------------------------------------------------------------------------
// a_s / a_d
// ------------------------------------------------------------------------------------------
template <int NS>
__global__ __launch_bounds__(NT) void k_gat_att(const float* __restrict__ XP, int64_t M, int H,
                                                int C, const float* __restrict__ att_src,
                                                const float* __restrict__ att_dst,
                                                float* __restrict__ a_s, float* __restrict__ a_d) {
  const Lane L = lane_row();
  if (L.row >= M) return;
  const int HC = H * C;
  for (int p = 0; p < num_passes(HC, NS); ++p) {
    const Pass<NS> P(p, L.li, HC, C);
    float ps = 0.f, pd = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const f32x4 v = ld4(XP + L.row * HC + P.fc[s]);
      ps += P.act[s] ? dot4(v, ld4(att_src + P.fc[s])) : 0.f;
      pd += P.act[s] ? dot4(v, ld4(att_dst + P.fc[s])) : 0.f;
    }
    ps = group_sum(ps, P.G);
    pd = group_sum(pd, P.G);
    if (P.leader) {
      a_s[L.row * H + P.head] = ps;
      a_d[L.row * H + P.head] = pd;
    }
  }
}

// ------------------------------------------------------------------------------------------
// forward: softmax over each target row + weighted sum of source rows (+ bias, ELU)
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
// four fp32 -> bf16 (round to nearest even, as torch's .to(torch.bfloat16)), one 8-B store
__device__ __forceinline__ void st4_bf16(uint16_t* p, f32x4 v) {
  *reinterpret_cast<unsigned long long*>(p) =
      __builtin_bit_cast(unsigned long long, __builtin_convertvector(v, bf16x4_t));
}

// + bias, activation; fp32 row and (Yb) its bf16 copy, the next bf16 GEMM's operand
template <int ACT, int NS>
__device__ __forceinline__ void gat_out(const Pass<NS>& P, const f32x4 (&acc)[NS],
                                        const float* __restrict__ bias, float* __restrict__ Y,
                                        uint16_t* __restrict__ Yb, int64_t base) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (P.act[s]) {
      const f32x4 bv = bias ? ld4(bias + P.fc[s]) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 o = acc[s] + bv;
      if (ACT == LGNN_ACT_ELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = elu_f(o[j]);
      }
      st4(Y + base + P.f[s], o);
      if (Yb) st4_bf16(Yb + base + P.f[s], o);
    }
  }
}

template <int ACT, int NS>
__global__ __launch_bounds__(NT) GAT_OCC void k_gat_fwd(const int32_t* __restrict__ rowptr,
                                                const int32_t* __restrict__ col,
                                                const float* __restrict__ XP,
                                                const float* __restrict__ a_s,
                                                const float* __restrict__ a_d, int64_t M, int H,
                                                int C, float slope, const float* __restrict__ mask,
                                                const float* __restrict__ bias,
                                                float* __restrict__ alpha, float* __restrict__ Y,
                                                uint16_t* __restrict__ Yb) {
  constexpr int EBN = EB / NS;
  const Lane L = lane_row();
  if (L.row >= M) return;
  const int HC = H * C;
  const int64_t cap = rowptr[M];  // CSR entries: the extent of col and the per-edge arrays
  const Buf bX = mkbuf(XP, M * HC * 4), bA = mkbuf(a_s, M * H * 4), bC = mkbuf(col, cap * 4);
  const Buf bAl = mkbuf(alpha, alpha ? cap * H * 4 : 0), bM = mkbuf(mask, mask ? cap * H * 4 : 0);
  const int e0 = rowptr[L.row], e1 = rowptr[L.row + 1];
  for (int p = 0; p < num_passes(HC, NS); ++p) {
    const Pass<NS> P(p, L.li, HC, C);
    const int head = P.head;
    const float ad = a_d[L.row * H + head];
    if (e1 - e0 <= EBN) {  // short row (k-NN graphs: k + 1 entries): one gather of everything,
      // the same operations in the same order as the three passes below
      int c[EBN];
      float a[EBN];
#pragma unroll
      for (int u = 0; u < EBN; ++u) {
        c[u] = bldi(bC, (uint32_t)(e0 + u < e1 ? e0 + u : e0) * 4u);
        a[u] = bld1(bA, (uint32_t)(c[u] * H + head) * 4u);
      }
      f32x4 xv[EBN][NS];
#pragma unroll
      for (int u = 0; u < EBN; ++u)
#pragma unroll
        for (int s = 0; s < NS; ++s) xv[u][s] = bld4(bX, ((uint32_t)c[u] * HC + P.fc[s]) * 4u);
      float m = -INFINITY;
#pragma unroll
      for (int u = 0; u < EBN; ++u)
        if (e0 + u < e1) m = fmaxf(m, leaky(a[u] + ad, slope));
      float sum = 0.f;
#pragma unroll
      for (int u = 0; u < EBN; ++u)
        if (e0 + u < e1) sum += expf(leaky(a[u] + ad, slope) - m);
      sum += EPS16;
      f32x4 acc[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < EBN; ++u) {
        if (e0 + u < e1) {
          const uint32_t eo = (uint32_t)((e0 + u) * H + head) * 4u;
          float al = expf(leaky(a[u] + ad, slope) - m) / sum;
          if (P.leader && alpha) bst1(bAl, eo, al);
          if (mask) al *= bld1(bM, eo);
#pragma unroll
          for (int s = 0; s < NS; ++s) acc[s] += al * xv[u][s];
        }
      }
      gat_out<ACT, NS>(P, acc, bias, Y, Yb, L.row * HC);
      continue;
    }
    // pass 1: row max of the logits (PyG: scatter max of the detached logits)
    float m = -INFINITY;
    for (int e = e0; e < e1; e += EB) {
      float v[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int ee = e + u < e1 ? e + u : e0;
        v[u] = bld1(bA, (uint32_t)(bldi(bC, (uint32_t)ee * 4u) * H + head) * 4u);
      }
#pragma unroll
      for (int u = 0; u < EB; ++u)
        if (e + u < e1) m = fmaxf(m, leaky(v[u] + ad, slope));
    }
    // pass 2: denominator, in CSR order
    float sum = 0.f;
    for (int e = e0; e < e1; e += EB) {
      float v[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int ee = e + u < e1 ? e + u : e0;
        v[u] = bld1(bA, (uint32_t)(bldi(bC, (uint32_t)ee * 4u) * H + head) * 4u);
      }
#pragma unroll
      for (int u = 0; u < EB; ++u)
        if (e + u < e1) sum += expf(leaky(v[u] + ad, slope) - m);
    }
    sum += EPS16;
    // pass 3: alpha, message sum
    f32x4 acc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int e = e0; e < e1; e += EBN) {
      int c[EBN];
      float a[EBN];
#pragma unroll
      for (int u = 0; u < EBN; ++u) {
        const int ee = e + u < e1 ? e + u : e0;
        c[u] = bldi(bC, (uint32_t)ee * 4u);
        a[u] = bld1(bA, (uint32_t)(c[u] * H + head) * 4u);
      }
      f32x4 xv[EBN][NS];
#pragma unroll
      for (int u = 0; u < EBN; ++u)
#pragma unroll
        for (int s = 0; s < NS; ++s) xv[u][s] = bld4(bX, ((uint32_t)c[u] * HC + P.fc[s]) * 4u);
#pragma unroll
      for (int u = 0; u < EBN; ++u) {
        if (e + u < e1) {
          const uint32_t eo = (uint32_t)((e + u) * H + head) * 4u;
          float al = expf(leaky(a[u] + ad, slope) - m) / sum;
          if (P.leader && alpha) bst1(bAl, eo, al);
          if (mask) al *= bld1(bM, eo);
#pragma unroll
          for (int s = 0; s < NS; ++s) acc[s] += al * xv[u][s];
        }
      }
    }
    gat_out<ACT, NS>(P, acc, bias, Y, Yb, L.row * HC);
  }
}

// ------------------------------------------------------------------------------------------
// backward, pass over target rows i:
//   dZ_i = dY_i * act'(Y_i)                                   (written: gathered by the next pass)
//   dal_ij = <dZ_i[h], xp_j[h]> * mask_ij;  s_i = sum_j alpha_ij dal_ij
//   de_ij = alpha_ij (dal_ij - s_i);  da_ij = de_ij * leaky'(a_s[j] + a_d[i])
//   da_e[ij] = da_ij (per edge),  da_d[i] = sum_j da_ij
// ------------------------------------------------------------------------------------------
// Readout gradient (POOL): the layer's output gradient is not a tensor but formed per row from
// the logits' gradient, dY[i] = (dlog[g] . Wout) / |g| (g = batch[i]; mean pooling), with
// k_head_bwd's fmaf chain over the classes and k_pool_bwd's division: the global pool + out_proj
// backward folded into this load, bitwise what those two kernels would have written.
struct PoolGrad {
  const int64_t* batch;
  const int32_t* gptr;
  const float* dlog;  // [B][nclass]
  const float* Wout;  // [nclass][H*C]
  int nclass;
  int mean;
};

template <int ACT, int NS, bool POOL = false>
__global__ __launch_bounds__(NT) GAT_OCC void k_gat_bwd_edge(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ XP, const float* __restrict__ a_s, const float* __restrict__ a_d,
    const float* __restrict__ alpha, const float* __restrict__ mask, const float* __restrict__ dY,
    const float* __restrict__ Y, int64_t M, int H, int C, float slope, float* __restrict__ dZ,
    float* __restrict__ da_e, float* __restrict__ da_d, PoolGrad pg = PoolGrad{}) {
  constexpr int EBN = EB / NS;
  const Lane L = lane_row();
  if (L.row >= M) return;
  const int HC = H * C;
  const int64_t cap = rowptr[M];  // CSR entries: the extent of col and the per-edge arrays
  const Buf bX = mkbuf(XP, M * HC * 4), bA = mkbuf(a_s, M * H * 4), bC = mkbuf(col, cap * 4);
  const Buf bAl = mkbuf(alpha, cap * H * 4), bM = mkbuf(mask, mask ? cap * H * 4 : 0);
  const Buf bDa = mkbuf(da_e, cap * H * 4);
  const int e0 = rowptr[L.row], e1 = rowptr[L.row + 1];
  for (int p = 0; p < num_passes(HC, NS); ++p) {
    const Pass<NS> P(p, L.li, HC, C);
    const int head = P.head;
    f32x4 dz[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if constexpr (POOL) {
        const int64_t g = pg.batch[L.row];
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < pg.nclass; ++c) {
          const float d = pg.dlog[g * pg.nclass + c];
          const f32x4 wv = ld4(pg.Wout + (int64_t)c * HC + P.fc[s]);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fmaf(d, wv[j], acc[j]);
        }
        if (pg.mean) {
          const int cnt = pg.gptr[g + 1] - pg.gptr[g];
          acc = acc / (float)(cnt > 0 ? cnt : 1);
        }
        dz[s] = acc;
      } else {
        dz[s] = ld4(dY + L.row * HC + P.fc[s]);
      }
      if (ACT == LGNN_ACT_ELU) {
        const f32x4 y = ld4(Y + L.row * HC + P.fc[s]);
#pragma unroll
        for (int j = 0; j < 4; ++j) dz[s][j] *= elu_grad_from_out(y[j]);
      }
      if (!P.act[s]) dz[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (P.act[s]) st4(dZ + L.row * HC + P.f[s], dz[s]);
    }
    const float ad = a_d[L.row * H + head];
    float s_i = 0.f, dad = 0.f;
    if (e1 - e0 <= EBN) {  // short row: one gather of the source rows, the dot products kept
      // (the same operations in the same order as the two sweeps below)
      int c[EBN];
#pragma unroll
      for (int u = 0; u < EBN; ++u) c[u] = bldi(bC, (uint32_t)(e0 + u < e1 ? e0 + u : e0) * 4u);
      f32x4 xv[EBN][NS];
#pragma unroll
      for (int u = 0; u < EBN; ++u)
#pragma unroll
        for (int s = 0; s < NS; ++s) xv[u][s] = bld4(bX, ((uint32_t)c[u] * HC + P.fc[s]) * 4u);
      float d[EBN], al[EBN];
#pragma unroll
      for (int u = 0; u < EBN; ++u) {
        const uint32_t eo = (uint32_t)((e0 + u < e1 ? e0 + u : e0) * H + head) * 4u;
        float part = 0.f;
#pragma unroll
        for (int s = 0; s < NS; ++s) part += dot4(dz[s], xv[u][s]);
        d[u] = group_sum(part, P.G);
        if (mask) d[u] *= bld1(bM, eo);
        al[u] = bld1(bAl, eo);
      }
#pragma unroll
      for (int u = 0; u < EBN; ++u)
        if (e0 + u < e1) s_i += al[u] * d[u];
#pragma unroll
      for (int u = 0; u < EBN; ++u) {
        if (e0 + u < e1) {
          const float pre = bld1(bA, (uint32_t)(c[u] * H + head) * 4u) + ad;
          const float da = al[u] * (d[u] - s_i) * (pre > 0.f ? 1.f : slope);
          dad += opaque(da);  // (never contracted with da's product: every form alike)
          if (P.leader) bst1(bDa, (uint32_t)((e0 + u) * H + head) * 4u, da);
        }
      }
      if (P.leader) da_d[L.row * H + head] = dad;
      continue;
    }
    // two sweeps over the row: sweep 0 accumulates s_i, sweep 1 emits the logit gradients
#pragma unroll 1
    for (int sweep = 0; sweep < 2; ++sweep) {
      for (int e = e0; e < e1; e += EBN) {
        int c[EBN];
#pragma unroll
        for (int u = 0; u < EBN; ++u) c[u] = bldi(bC, (uint32_t)(e + u < e1 ? e + u : e0) * 4u);
        f32x4 xv[EBN][NS];
#pragma unroll
        for (int u = 0; u < EBN; ++u)
#pragma unroll
          for (int s = 0; s < NS; ++s) xv[u][s] = bld4(bX, ((uint32_t)c[u] * HC + P.fc[s]) * 4u);
#pragma unroll
        for (int u = 0; u < EBN; ++u) {
          const int ee = e + u < e1 ? e + u : e0;
          const uint32_t eo = (uint32_t)(ee * H + head) * 4u;
          float part = 0.f;
#pragma unroll
          for (int s = 0; s < NS; ++s) part += dot4(dz[s], xv[u][s]);
          float d = group_sum(part, P.G);
          if (mask) d *= bld1(bM, eo);
          const float al = bld1(bAl, eo);
          if (sweep == 0) {
            if (e + u < e1) s_i += al * d;
          } else {
            const float pre = bld1(bA, (uint32_t)(c[u] * H + head) * 4u) + ad;
            const float da = al * (d - s_i) * (pre > 0.f ? 1.f : slope);
            if (e + u < e1) {
              dad += opaque(da);  // (never contracted with da's product: every form alike)
              if (P.leader) bst1(bDa, eo, da);
            }
          }
        }
      }
    }
    if (P.leader) da_d[L.row * H + head] = dad;
  }
}

// ------------------------------------------------------------------------------------------
// backward, pass over source rows j (transpose CSR; tmap[q] = target-CSR position of entry q):
//   dXP_j[h] = sum_{j->i} alpha_ij mask_ij dZ_i[h] + (sum_i da_ij) att_src[h] + da_d[j,h] att_dst[h]
// plus per-block column partials: [0] datt_src = sum_j (sum_i da_ij) xp_j,
//                                 [1] datt_dst = sum_j da_d[j] xp_j,  [2] dbias = sum_j dZ_j.
// Persistent over rows (block b owns rows b*8 + hw + 8*P*t), fixed-order in-block combine.
// Features are walked in strips of 128 (strip st = features [128 st, 128 st + 128)).
// ------------------------------------------------------------------------------------------
template <int NST>  // 128-feature strips: ceil(H*C / 128)
__global__ __launch_bounds__(NT) GAT_OCC void k_gat_bwd_node(
    const int32_t* __restrict__ tptr, const int32_t* __restrict__ tidx,
    const int32_t* __restrict__ tmap, const float* __restrict__ alpha,
    const float* __restrict__ mask, const float* __restrict__ da_e,
    const float* __restrict__ da_d, const float* __restrict__ dZ, const float* __restrict__ XP,
    const float* __restrict__ att_src, const float* __restrict__ att_dst, int64_t M, int H,
    int C, float* __restrict__ dXP, float* __restrict__ part, uint16_t* __restrict__ dXPb) {
  __shared__ __attribute__((aligned(16))) float red[RB][3 * NST * 128];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, hw = wave * 2 + (lane >> 5);
  const int HC = H * C;
  f32x4 ps[NST], pd[NST], pb[NST];
#pragma unroll
  for (int q = 0; q < NST; ++q) ps[q] = pd[q] = pb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t cap = M > 0 ? tptr[M] : 0;  // transpose-CSR entries
  const Buf bT = mkbuf(tidx, cap * 4), bP = mkbuf(tmap, cap * 4), bZ = mkbuf(dZ, M * HC * 4);
  const Buf bAl = mkbuf(alpha, cap * H * 4), bM = mkbuf(mask, mask ? cap * H * 4 : 0);
  const Buf bDa = mkbuf(da_e, cap * H * 4);
#if LGNN_GAT_NODE_XCD
  // rows in 8 contiguous ranges, range x walked by the workgroups on XCD x (blocks are dealt
  // round-robin over the XCDs): the alpha / da_e entries a source row gathers through tmap, and
  // the dZ rows, belong to its own graph, so they stay in that XCD's L2
  const int64_t xcd = blockIdx.x % 8, nb = ((int64_t)gridDim.x - xcd + 7) / 8;
  const int64_t span = ((M + 7) / 8 + RB - 1) / RB * RB;
  const int64_t rbeg = xcd * span, rend = rbeg + span < M ? rbeg + span : M;
  for (int64_t row = rbeg + (int64_t)(blockIdx.x / 8) * RB + hw; row < rend; row += nb * RB) {
#else
  // (plain block order: the XCD-contiguous mapping of lane_row measured 3 us slower here)
  for (int64_t row = (int64_t)blockIdx.x * RB + hw; row < M; row += (int64_t)gridDim.x * RB) {
#endif
    const int q0 = tptr[row], q1 = tptr[row + 1];
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      const int s0 = st * 128;
      if (s0 >= HC) break;
      const int f = s0 + 4 * li;
      const bool act = f < HC;
      const int fc = act ? f : HC - 4;
      const int head = fc / C;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      float sda = 0.f;
      for (int q = q0; q < q1; q += EB) {
        int ti[EB], pp[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          const uint32_t qo = (uint32_t)(q + u < q1 ? q + u : q0) * 4u;
          ti[u] = bldi(bT, qo);
          pp[u] = bldi(bP, qo);
        }
        f32x4 dv[EB];
        float al[EB], da[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          const uint32_t eo = (uint32_t)(pp[u] * H + head) * 4u;
          dv[u] = bld4(bZ, ((uint32_t)ti[u] * HC + fc) * 4u);
          al[u] = bld1(bAl, eo);
          if (mask) al[u] *= bld1(bM, eo);
          da[u] = bld1(bDa, eo);
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          if (q + u < q1) {
            acc += al[u] * dv[u];
            sda += da[u];
          }
        }
      }
      const float dd = da_d[row * H + head];
      const f32x4 xp = ld4(XP + row * HC + fc);
      const f32x4 o = acc + sda * ld4(att_src + fc) + dd * ld4(att_dst + fc);
      if (act) {
        st4(dXP + row * HC + f, o);
        if (dXPb) st4_bf16(dXPb + row * HC + f, o);  // the lin backward's bf16 operand
        ps[st] += sda * xp;
        pd[st] += dd * xp;
        pb[st] += ld4(dZ + row * HC + f);
      }
    }
  }
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    st4(&red[hw][(0 * NST + st) * 128 + 4 * li], ps[st]);
    st4(&red[hw][(1 * NST + st) * 128 + 4 * li], pd[st]);
    st4(&red[hw][(2 * NST + st) * 128 + 4 * li], pb[st]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * HC; i += NT) {
    const int kind = i / HC, f = i % HC;
    const int idx = (kind * NST + f / 128) * 128 + f % 128;
    float t = red[0][idx];
#pragma unroll
    for (int r = 1; r < RB; ++r) t += red[r][idx];
    part[(int64_t)blockIdx.x * 3 * HC + i] = t;
  }
}

// ------------------------------------------------------------------------------------------
// Row-pipelined variants (one 128-feature pass: H*C <= 128, H <= 4 — every GAT of the reference
// config and of C3). The kernels above spend a row's life in a chain of dependent round trips
// (row extent -> column indices -> logit inputs / source rows -> stores) with only the source
// rows carrying bandwidth, and each wave sees two rows. Here a half wave walks many rows and
// keeps the chain off the critical path: while row r's source rows are gathered, the column
// indices of row r + step and the extent of row r + 2 step are already in flight. And the
// per-edge scalars are loaded edge-parallel, one instruction for 8 edges x 4 heads (lane
// u + 8 h of a half wave: edge u, head h), then handed to the feature lanes with ds_bpermute
// instead of 8-24 same-address loads per row. Every quantity is formed with the same
// operations in the same order as in the kernels above (bitwise the same results; tested).
// Rows longer than EB entries take an in-place batched walk (not pipelined).
// ------------------------------------------------------------------------------------------
constexpr uint32_t OOB = 0x7ff00000u;  // buffer offset past every range: the load returns 0

__device__ __forceinline__ int bperm_i(int v, int src) {
  return __builtin_amdgcn_ds_bpermute(src << 2, v);
}
__device__ __forceinline__ float bperm_f(float v, int src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src << 2, __builtin_bit_cast(int, v)));
}
// max over the 8-lane group of an edge lane (order-free, so any butterfly)
__device__ __forceinline__ float max8(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  return fmaxf(v, dppf<0x141>(v));
}

// the rows of a half wave: 8 contiguous ranges of rows, range x walked by the workgroups on XCD x
// (dealt round-robin over the XCDs; a launch has >= 8 workgroups), consecutive half waves on
// consecutive rows — a graph's rows, and the source rows they gather, stay in one XCD's L2
struct RowWalk {
  int64_t r, rend, step;
};
__device__ __forceinline__ RowWalk row_walk(int64_t M) {
  const int lane = threadIdx.x & 63, hw = (threadIdx.x >> 6) * 2 + (lane >> 5);
  const int64_t xcd = blockIdx.x & 7, nb = ((int64_t)gridDim.x - xcd + 7) >> 3;
  const int64_t span = ((M + 7) / 8 + RB - 1) / RB * RB;  // (k_gat_bwd_node's row sets)
  RowWalk w;
  const int64_t rbeg = xcd * span;
  w.rend = rbeg + span < M ? rbeg + span : M;
  w.r = rbeg + (int64_t)(blockIdx.x >> 3) * RB + hw;
  w.step = nb * RB;
  return w;
}

struct EdgeLane {
  int li, hwb, u, hh, hq;  // lane in the half wave, half-wave base lane, edge slot, head slot
  bool hv;                  // hh < H
  int hh2, hq2;             // 8 heads (HS = 2): the lane's second head, hh + 4
  bool hv2;
  __device__ __forceinline__ EdgeLane(int H) {
    const int lane = threadIdx.x & 63;
    li = lane & 31;
    hwb = lane & 32;
    u = li & 7;
    hh = li >> 3;
    hv = hh < H;
    hq = hv ? hh : 0;
    hh2 = hh + 4;
    hv2 = hh2 < H;
    hq2 = hv2 ? hh2 : 0;
  }
  // CSR position of edge slot u of the batch starting at b (clamped into the row)
  __device__ __forceinline__ int pos(int b, int e1) const { return b + (b + u < e1 ? u : 0); }
};

// Head slots per edge lane: HS = 1 for H <= 4 (lane u + 8 h: edge u, head h), HS = 2 for
// 5..8 heads (the same lane also holds head h + 4 in a second register: 8 heads of C <= 16, the
// sweep's heads 8 at widths <= 128). A feature lane of head h reads its head's per-edge value
// from lane 8 (h & 3) + k of its half wave, in register (h >> 2).
template <int HS>
__device__ __forceinline__ float head_perm(float v1, float v2, int base, int k, int head) {
  const float x1 = bperm_f(v1, base + k);
  if constexpr (HS == 1) {
    (void)v2;
    (void)head;
    return x1;
  } else {
    const float x2 = bperm_f(v2, base + k);
    return head >= 4 ? x2 : x1;
  }
}

template <int ACT, int HS>
__global__ __launch_bounds__(NT) void k_gat_fwd_p(const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col,
                                                  const float* __restrict__ XP,
                                                  const float* __restrict__ a_s,
                                                  const float* __restrict__ a_d, int64_t M, int H,
                                                  int C, float slope,
                                                  const float* __restrict__ mask,
                                                  const float* __restrict__ bias,
                                                  float* __restrict__ alpha, float* __restrict__ Y,
                                                  uint16_t* __restrict__ Yb) {
  const EdgeLane L(H);
  const int HC = H * C;
  const Pass<1> P(0, L.li, HC, C);
  const int hbase = L.hwb + 8 * (P.head & 3);  // this feature lane's head: its edge lanes
  RowWalk W = row_walk(M);
  if (W.r >= W.rend) return;
  const int64_t cap = rowptr[M];
  const Buf bR = mkbuf(rowptr, (M + 1) * 4), bC = mkbuf(col, cap * 4);
  const Buf bX = mkbuf(XP, M * HC * 4), bA = mkbuf(a_s, M * H * 4), bD = mkbuf(a_d, M * H * 4);
  const Buf bAl = mkbuf(alpha, alpha ? cap * H * 4 : 0), bM = mkbuf(mask, mask ? cap * H * 4 : 0);
  const bool two = HS == 2;
  int64_t r = W.r;
  int e0 = bldi(bR, (uint32_t)r * 4u), e1 = bldi(bR, (uint32_t)r * 4u + 4u);
  int cu = bldi(bC, (uint32_t)L.pos(e0, e1) * 4u);
  int64_t rn = r + W.step;
  uint32_t ro = rn < W.rend ? (uint32_t)rn * 4u : OOB;
  int e0n = bldi(bR, ro), e1n = bldi(bR, ro + 4u);
  for (;;) {
    const int deg = e1 - e0;
    // row r: edge lanes load the logit inputs, feature lanes gather the first batch's rows
    const int eu = L.pos(e0, e1);
    const float a = bld1(bA, (uint32_t)(cu * H + L.hq) * 4u);
    const float ad = bld1(bD, (uint32_t)(r * H + L.hq) * 4u);
    const float mk = mask ? bld1(bM, (uint32_t)(eu * H + L.hq) * 4u) : 1.f;
    float a2 = 0.f, ad2 = 0.f, mk2 = 1.f;
    if (two) {
      a2 = bld1(bA, (uint32_t)(cu * H + L.hq2) * 4u);
      ad2 = bld1(bD, (uint32_t)(r * H + L.hq2) * 4u);
      mk2 = mask ? bld1(bM, (uint32_t)(eu * H + L.hq2) * 4u) : 1.f;
    }
    f32x4 xv[EB];
#pragma unroll
    for (int k = 0; k < EB; ++k)
      xv[k] = bld4(bX, ((uint32_t)bperm_i(cu, L.hwb + k) * HC + P.fc[0]) * 4u);
    // row r + step: its first batch's columns; row r + 2 step: its extent
    const int64_t rnn = rn + W.step;
    const int cun = bldi(bC, rn < W.rend ? (uint32_t)L.pos(e0n, e1n) * 4u : OOB);
    const uint32_t ron = rnn < W.rend ? (uint32_t)rnn * 4u : OOB;
    const int e0nn = bldi(bR, ron), e1nn = bldi(bR, ron + 4u);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (deg <= EB) {
      const bool ev = L.u < deg && L.hv, ev2 = L.u < deg && L.hv2;
      const float lg = leaky(a + ad, slope);
      const float m = max8(ev ? lg : -INFINITY);
      const float ex = ev ? expf(lg - m) : 0.f;
      float sum = 0.f;  // in CSR order (the zeros of absent edges add exactly nothing)
#pragma unroll
      for (int k = 0; k < EB; ++k) sum += bperm_f(ex, L.hwb + 8 * L.hh + k);
      sum += EPS16;
      const float al = ex / sum;
      if (alpha && ev) bst1(bAl, (uint32_t)(eu * H + L.hh) * 4u, al);
      const float alm = mask ? al * mk : al;
      float alm2 = 0.f;
      if (two) {  // the second head slot: the same operations
        const float lg2 = leaky(a2 + ad2, slope);
        const float m2 = max8(ev2 ? lg2 : -INFINITY);
        const float ex2 = ev2 ? expf(lg2 - m2) : 0.f;
        float sum2 = 0.f;
#pragma unroll
        for (int k = 0; k < EB; ++k) sum2 += bperm_f(ex2, L.hwb + 8 * L.hh + k);
        sum2 += EPS16;
        const float al2 = ex2 / sum2;
        if (alpha && ev2) bst1(bAl, (uint32_t)(eu * H + L.hh2) * 4u, al2);
        alm2 = mask ? al2 * mk2 : al2;
      }
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const float w = head_perm<HS>(alm, alm2, hbase, k, P.head);
        if (k < deg) acc += w * xv[k];
      }
    } else {  // long row: max, denominator, messages, each a walk over batches of EB entries
      float m = -INFINITY, m2 = -INFINITY;
      for (int b = e0; b < e1; b += EB) {
        const int c = bldi(bC, (uint32_t)L.pos(b, e1) * 4u);
        const float lg = leaky(bld1(bA, (uint32_t)(c * H + L.hq) * 4u) + ad, slope);
        if (b + L.u < e1 && L.hv) m = fmaxf(m, lg);
        if (two) {
          const float lg2 = leaky(bld1(bA, (uint32_t)(c * H + L.hq2) * 4u) + ad2, slope);
          if (b + L.u < e1 && L.hv2) m2 = fmaxf(m2, lg2);
        }
      }
      m = max8(m);
      if (two) m2 = max8(m2);
      float sum = 0.f, sum2 = 0.f;
      for (int b = e0; b < e1; b += EB) {
        const int c = bldi(bC, (uint32_t)L.pos(b, e1) * 4u);
        const float lg = leaky(bld1(bA, (uint32_t)(c * H + L.hq) * 4u) + ad, slope);
        const float ex = b + L.u < e1 && L.hv ? expf(lg - m) : 0.f;
#pragma unroll
        for (int k = 0; k < EB; ++k) sum += bperm_f(ex, L.hwb + 8 * L.hh + k);
        if (two) {
          const float lg2 = leaky(bld1(bA, (uint32_t)(c * H + L.hq2) * 4u) + ad2, slope);
          const float ex2 = b + L.u < e1 && L.hv2 ? expf(lg2 - m2) : 0.f;
#pragma unroll
          for (int k = 0; k < EB; ++k) sum2 += bperm_f(ex2, L.hwb + 8 * L.hh + k);
        }
      }
      sum += EPS16;
      sum2 += EPS16;
      for (int b = e0; b < e1; b += EB) {
        const int eb = L.pos(b, e1);
        const bool ev = b + L.u < e1 && L.hv;
        const int c = bldi(bC, (uint32_t)eb * 4u);
        const float lg = leaky(bld1(bA, (uint32_t)(c * H + L.hq) * 4u) + ad, slope);
        const float mb = mask ? bld1(bM, (uint32_t)(eb * H + L.hq) * 4u) : 1.f;
        f32x4 xb[EB];
#pragma unroll
        for (int k = 0; k < EB; ++k)
          xb[k] = bld4(bX, ((uint32_t)bperm_i(c, L.hwb + k) * HC + P.fc[0]) * 4u);
        const float al = (ev ? expf(lg - m) : 0.f) / sum;
        if (alpha && ev) bst1(bAl, (uint32_t)(eb * H + L.hh) * 4u, al);
        const float alm = mask ? al * mb : al;
        float alm2 = 0.f;
        if (two) {
          const bool ev2 = b + L.u < e1 && L.hv2;
          const float lg2 = leaky(bld1(bA, (uint32_t)(c * H + L.hq2) * 4u) + ad2, slope);
          const float mb2 = mask ? bld1(bM, (uint32_t)(eb * H + L.hq2) * 4u) : 1.f;
          const float al2 = (ev2 ? expf(lg2 - m2) : 0.f) / sum2;
          if (alpha && ev2) bst1(bAl, (uint32_t)(eb * H + L.hh2) * 4u, al2);
          alm2 = mask ? al2 * mb2 : al2;
        }
#pragma unroll
        for (int k = 0; k < EB; ++k) {
          const float w = head_perm<HS>(alm, alm2, hbase, k, P.head);
          if (b + k < e1) acc += w * xb[k];
        }
      }
    }
    const f32x4 out[1] = {acc};
    gat_out<ACT, 1>(P, out, bias, Y, Yb, r * HC);
    if (rn >= W.rend) break;
    r = rn;
    rn = rnn;
    e0 = e0n;
    e1 = e1n;
    cu = cun;
    e0n = e0nn;
    e1n = e1nn;
  }
}

// the output gradient of row r for this feature lane (dY, or the readout's, see PoolGrad), times
// the activation's derivative
template <int ACT, bool POOL>
__device__ __forceinline__ f32x4 dz_row(int64_t r, int HC, int fc, const float* __restrict__ dY,
                                        const float* __restrict__ Y, const PoolGrad& pg) {
  f32x4 dz;
  if constexpr (POOL) {
    const int64_t g = pg.batch[r];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < pg.nclass; ++c) {
      const float d = pg.dlog[g * pg.nclass + c];
      const f32x4 wv = ld4(pg.Wout + (int64_t)c * HC + fc);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = fmaf(d, wv[j], acc[j]);
    }
    if (pg.mean) {
      const int cnt = pg.gptr[g + 1] - pg.gptr[g];
      acc = acc / (float)(cnt > 0 ? cnt : 1);
    }
    dz = acc;
  } else {
    dz = ld4(dY + r * HC + fc);
  }
  if (ACT == LGNN_ACT_ELU) {
    const f32x4 y = ld4(Y + r * HC + fc);
#pragma unroll
    for (int j = 0; j < 4; ++j) dz[j] *= elu_grad_from_out(y[j]);
  }
  return dz;
}

template <int ACT, bool POOL, int HS>
__global__ __launch_bounds__(NT) void k_gat_bwd_edge_p(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ XP, const float* __restrict__ a_s, const float* __restrict__ a_d,
    const float* __restrict__ alpha, const float* __restrict__ mask, const float* __restrict__ dY,
    const float* __restrict__ Y, int64_t M, int H, int C, float slope, float* __restrict__ dZ,
    float* __restrict__ da_e, float* __restrict__ da_d, PoolGrad pg) {
  const EdgeLane L(H);
  const int HC = H * C;
  const Pass<1> P(0, L.li, HC, C);
  const int hbase = L.hwb + 8 * (P.head & 3);
  const int hlead = L.hwb + L.hq * P.G;    // the first feature lane of edge lane's head
  const int hlead2 = L.hwb + L.hq2 * P.G;  // ... of its second head (HS = 2)
  const bool two = HS == 2;
  RowWalk W = row_walk(M);
  if (W.r >= W.rend) return;
  const int64_t cap = rowptr[M];
  const Buf bR = mkbuf(rowptr, (M + 1) * 4), bC = mkbuf(col, cap * 4);
  const Buf bX = mkbuf(XP, M * HC * 4), bA = mkbuf(a_s, M * H * 4), bD = mkbuf(a_d, M * H * 4);
  const Buf bAl = mkbuf(alpha, cap * H * 4), bM = mkbuf(mask, mask ? cap * H * 4 : 0);
  const Buf bDa = mkbuf(da_e, cap * H * 4);
  int64_t r = W.r;
  int e0 = bldi(bR, (uint32_t)r * 4u), e1 = bldi(bR, (uint32_t)r * 4u + 4u);
  int cu = bldi(bC, (uint32_t)L.pos(e0, e1) * 4u);
  int64_t rn = r + W.step;
  uint32_t ro = rn < W.rend ? (uint32_t)rn * 4u : OOB;
  int e0n = bldi(bR, ro), e1n = bldi(bR, ro + 4u);
  for (;;) {
    const int deg = e1 - e0;
    const int eu = L.pos(e0, e1);
    const float al = bld1(bAl, (uint32_t)(eu * H + L.hq) * 4u);
    const float mk = mask ? bld1(bM, (uint32_t)(eu * H + L.hq) * 4u) : 1.f;
    const float pre = bld1(bA, (uint32_t)(cu * H + L.hq) * 4u) +
                      bld1(bD, (uint32_t)(r * H + L.hq) * 4u);
    float al2 = 0.f, mk2 = 1.f, pre2 = 0.f;
    if (two) {
      al2 = bld1(bAl, (uint32_t)(eu * H + L.hq2) * 4u);
      mk2 = mask ? bld1(bM, (uint32_t)(eu * H + L.hq2) * 4u) : 1.f;
      pre2 = bld1(bA, (uint32_t)(cu * H + L.hq2) * 4u) + bld1(bD, (uint32_t)(r * H + L.hq2) * 4u);
    }
    f32x4 xv[EB];
#pragma unroll
    for (int k = 0; k < EB; ++k)
      xv[k] = bld4(bX, ((uint32_t)bperm_i(cu, L.hwb + k) * HC + P.fc[0]) * 4u);
    f32x4 dz = dz_row<ACT, POOL>(r, HC, P.fc[0], dY, Y, pg);
    const int64_t rnn = rn + W.step;
    const int cun = bldi(bC, rn < W.rend ? (uint32_t)L.pos(e0n, e1n) * 4u : OOB);
    const uint32_t ron = rnn < W.rend ? (uint32_t)rnn * 4u : OOB;
    const int e0nn = bldi(bR, ron), e1nn = bldi(bR, ron + 4u);
    if (!P.act[0]) dz = f32x4{0.f, 0.f, 0.f, 0.f};
    if (P.act[0]) st4(dZ + r * HC + P.f[0], dz);
    float dad = 0.f;
    if (deg <= EB) {
      float d[EB], alk[EB];
      float s_i = 0.f;
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        d[k] = group_sum(dot4(dz, xv[k]), P.G);
        if (mask) d[k] *= head_perm<HS>(mk, mk2, hbase, k, P.head);
        alk[k] = head_perm<HS>(al, al2, hbase, k, P.head);
        if (k < deg) s_i += alk[k] * d[k];
      }
      float mine = 0.f, mine2 = 0.f;  // edge lane (u, h): the logit gradient of its edge and head
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const float fk = head_perm<HS>(pre > 0.f ? 1.f : slope, pre2 > 0.f ? 1.f : slope, hbase,
                                       k, P.head);
        const float da = alk[k] * (d[k] - s_i) * fk;
        if (k < deg) dad += opaque(da);  // (never contracted with da's product: every form alike)
        const float t = bperm_f(da, hlead);
        mine = L.u == k ? t : mine;
        if (two) {
          const float t2 = bperm_f(da, hlead2);
          mine2 = L.u == k ? t2 : mine2;
        }
      }
      if (L.u < deg && L.hv) bst1(bDa, (uint32_t)(eu * H + L.hh) * 4u, mine);
      if (two && L.u < deg && L.hv2) bst1(bDa, (uint32_t)(eu * H + L.hh2) * 4u, mine2);
    } else {  // long row: two walks over batches of EB entries (s_i, then the gradients)
      float s_i = 0.f;
#pragma unroll 1
      for (int sweep = 0; sweep < 2; ++sweep) {
        for (int b = e0; b < e1; b += EB) {
          const int eb = L.pos(b, e1);
          const int c = bldi(bC, (uint32_t)eb * 4u);
          const float alb = bld1(bAl, (uint32_t)(eb * H + L.hq) * 4u);
          const float mb = mask ? bld1(bM, (uint32_t)(eb * H + L.hq) * 4u) : 1.f;
          const float preb = bld1(bA, (uint32_t)(c * H + L.hq) * 4u) +
                             bld1(bD, (uint32_t)(r * H + L.hq) * 4u);
          float alb2 = 0.f, mb2 = 1.f, preb2 = 0.f;
          if (two) {
            alb2 = bld1(bAl, (uint32_t)(eb * H + L.hq2) * 4u);
            mb2 = mask ? bld1(bM, (uint32_t)(eb * H + L.hq2) * 4u) : 1.f;
            preb2 = bld1(bA, (uint32_t)(c * H + L.hq2) * 4u) +
                    bld1(bD, (uint32_t)(r * H + L.hq2) * 4u);
          }
          f32x4 xb[EB];
#pragma unroll
          for (int k = 0; k < EB; ++k)
            xb[k] = bld4(bX, ((uint32_t)bperm_i(c, L.hwb + k) * HC + P.fc[0]) * 4u);
          float mine = 0.f, mine2 = 0.f;
#pragma unroll
          for (int k = 0; k < EB; ++k) {
            float dk = group_sum(dot4(dz, xb[k]), P.G);
            if (mask) dk *= head_perm<HS>(mb, mb2, hbase, k, P.head);
            const float ak = head_perm<HS>(alb, alb2, hbase, k, P.head);
            const float fk = head_perm<HS>(preb > 0.f ? 1.f : slope, preb2 > 0.f ? 1.f : slope,
                                           hbase, k, P.head);
            if (sweep == 0) {
              if (b + k < e1) s_i += ak * dk;
            } else {
              const float da = ak * (dk - s_i) * fk;
              if (b + k < e1) dad += opaque(da);  // (never contracted with da's product: every form alike)
              const float t = bperm_f(da, hlead);
              mine = L.u == k ? t : mine;
              if (two) {
                const float t2 = bperm_f(da, hlead2);
                mine2 = L.u == k ? t2 : mine2;
              }
            }
          }
          if (sweep == 1 && b + L.u < e1 && L.hv)
            bst1(bDa, (uint32_t)(eb * H + L.hh) * 4u, mine);
          if (two && sweep == 1 && b + L.u < e1 && L.hv2)
            bst1(bDa, (uint32_t)(eb * H + L.hh2) * 4u, mine2);
        }
      }
    }
    if (P.leader) da_d[r * H + P.head] = dad;
    if (rn >= W.rend) break;
    r = rn;
    rn = rnn;
    e0 = e0n;
    e1 = e1n;
    cu = cun;
    e0n = e0nn;
    e1n = e1nn;
  }
}

// source-row pass (see k_gat_bwd_node), one 128-feature strip, pipelined: the next row's first
// batch of transpose entries (target row, target-CSR position) is in flight during this row's
// gathers. Same per-workgroup partials (grid = lgnn_gat_bwd_num_partials).
template <int HS>
__global__ __launch_bounds__(NT) void k_gat_bwd_node_p(
    const int32_t* __restrict__ tptr, const int32_t* __restrict__ tidx,
    const int32_t* __restrict__ tmap, const float* __restrict__ alpha,
    const float* __restrict__ mask, const float* __restrict__ da_e,
    const float* __restrict__ da_d, const float* __restrict__ dZ, const float* __restrict__ XP,
    const float* __restrict__ att_src, const float* __restrict__ att_dst, int64_t M, int H,
    int C, float* __restrict__ dXP, float* __restrict__ part, uint16_t* __restrict__ dXPb) {
  __shared__ __attribute__((aligned(16))) float red[RB][3 * 128];
  const EdgeLane L(H);
  const int HC = H * C;
  const Pass<1> P(0, L.li, HC, C);
  const int hbase = L.hwb + 8 * (P.head & 3);
  const bool two = HS == 2;
  const int hw = (threadIdx.x >> 6) * 2 + ((threadIdx.x & 63) >> 5);
  f32x4 ps = {0.f, 0.f, 0.f, 0.f}, pd = ps, pb = ps;
  RowWalk W = row_walk(M);
  if (W.r < W.rend) {
    const int64_t cap = tptr[M];
    const Buf bR = mkbuf(tptr, (M + 1) * 4), bT = mkbuf(tidx, cap * 4), bP = mkbuf(tmap, cap * 4);
    const Buf bZ = mkbuf(dZ, M * HC * 4), bAl = mkbuf(alpha, cap * H * 4);
    const Buf bM = mkbuf(mask, mask ? cap * H * 4 : 0), bDa = mkbuf(da_e, cap * H * 4);
    const f32x4 as = ld4(att_src + P.fc[0]), adv = ld4(att_dst + P.fc[0]);
    int64_t r = W.r;
    int q0 = bldi(bR, (uint32_t)r * 4u), q1 = bldi(bR, (uint32_t)r * 4u + 4u);
    int tu = bldi(bT, (uint32_t)L.pos(q0, q1) * 4u), pu = bldi(bP, (uint32_t)L.pos(q0, q1) * 4u);
    int64_t rn = r + W.step;
    uint32_t ro = rn < W.rend ? (uint32_t)rn * 4u : OOB;
    int q0n = bldi(bR, ro), q1n = bldi(bR, ro + 4u);
    for (;;) {
      const int deg = q1 - q0;
      float alu = bld1(bAl, (uint32_t)(pu * H + L.hq) * 4u);
      const float mk = mask ? bld1(bM, (uint32_t)(pu * H + L.hq) * 4u) : 1.f;
      const float dau = bld1(bDa, (uint32_t)(pu * H + L.hq) * 4u);
      float alu2 = 0.f, mk2 = 1.f, dau2 = 0.f;
      if (two) {
        alu2 = bld1(bAl, (uint32_t)(pu * H + L.hq2) * 4u);
        mk2 = mask ? bld1(bM, (uint32_t)(pu * H + L.hq2) * 4u) : 1.f;
        dau2 = bld1(bDa, (uint32_t)(pu * H + L.hq2) * 4u);
      }
      f32x4 dv[EB];
#pragma unroll
      for (int k = 0; k < EB; ++k)
        dv[k] = bld4(bZ, ((uint32_t)bperm_i(tu, L.hwb + k) * HC + P.fc[0]) * 4u);
      const float dd = da_d[r * H + P.head];
      const f32x4 xp = ld4(XP + r * HC + P.fc[0]);
      const f32x4 zr = ld4(dZ + r * HC + P.fc[0]);
      const int64_t rnn = rn + W.step;
      const uint32_t qn = rn < W.rend ? (uint32_t)L.pos(q0n, q1n) * 4u : OOB;
      const int tun = bldi(bT, qn), pun = bldi(bP, qn);
      const uint32_t ron = rnn < W.rend ? (uint32_t)rnn * 4u : OOB;
      const int q0nn = bldi(bR, ron), q1nn = bldi(bR, ron + 4u);
      if (mask) alu *= mk;
      if (mask) alu2 *= mk2;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      float sda = 0.f;
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const float ak = head_perm<HS>(alu, alu2, hbase, k, P.head);
        const float dk = head_perm<HS>(dau, dau2, hbase, k, P.head);
        if (k < deg) {
          acc += ak * dv[k];
          sda += dk;
        }
      }
      for (int b = q0 + EB; b < q1; b += EB) {  // entries past the first batch
        const int qb = L.pos(b, q1);
        const int tb = bldi(bT, (uint32_t)qb * 4u), pb_ = bldi(bP, (uint32_t)qb * 4u);
        float alb = bld1(bAl, (uint32_t)(pb_ * H + L.hq) * 4u);
        if (mask) alb *= bld1(bM, (uint32_t)(pb_ * H + L.hq) * 4u);
        const float dab = bld1(bDa, (uint32_t)(pb_ * H + L.hq) * 4u);
        float alb2 = 0.f, dab2 = 0.f;
        if (two) {
          alb2 = bld1(bAl, (uint32_t)(pb_ * H + L.hq2) * 4u);
          if (mask) alb2 *= bld1(bM, (uint32_t)(pb_ * H + L.hq2) * 4u);
          dab2 = bld1(bDa, (uint32_t)(pb_ * H + L.hq2) * 4u);
        }
        f32x4 db[EB];
#pragma unroll
        for (int k = 0; k < EB; ++k)
          db[k] = bld4(bZ, ((uint32_t)bperm_i(tb, L.hwb + k) * HC + P.fc[0]) * 4u);
#pragma unroll
        for (int k = 0; k < EB; ++k) {
          const float ak = head_perm<HS>(alb, alb2, hbase, k, P.head);
          const float dk = head_perm<HS>(dab, dab2, hbase, k, P.head);
          if (b + k < q1) {
            acc += ak * db[k];
            sda += dk;
          }
        }
      }
      const f32x4 o = acc + sda * as + dd * adv;
      if (P.act[0]) {
        st4(dXP + r * HC + P.f[0], o);
        if (dXPb) st4_bf16(dXPb + r * HC + P.f[0], o);
        ps += sda * xp;
        pd += dd * xp;
        pb += zr;
      }
      if (rn >= W.rend) break;
      r = rn;
      rn = rnn;
      q0 = q0n;
      q1 = q1n;
      tu = tun;
      pu = pun;
      q0n = q0nn;
      q1n = q1nn;
    }
  }
  st4(&red[hw][0 * 128 + 4 * L.li], ps);
  st4(&red[hw][1 * 128 + 4 * L.li], pd);
  st4(&red[hw][2 * 128 + 4 * L.li], pb);
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * HC; i += NT) {
    const int kind = i / HC, f = i % HC;
    const int idx = kind * 128 + f;
    float t = red[0][idx];
#pragma unroll
    for (int q = 1; q < RB; ++q) t += red[q][idx];
    part[(int64_t)blockIdx.x * 3 * HC + i] = t;
  }
}

// Two-strip form (k_gat_fwd_ps<…, 2>, 128 < H*C <= 256): NST strips of 128 features per row
// (H*C <= 128 NST, C <= 128; with NST > 1, C >= 32, so a
// strip's heads, 128 / C of them, fit the 4 head slots of the edge lanes). Every row's loads of
// all strips are issued together; each strip's softmax and messages are then those of the
// single-strip kernel for the strip's heads (bitwise k_gat_fwd's per-head values). The
// one-strip shapes keep k_gat_fwd_p: this form at NST = 1 compiled 1.5 us slower per launch.
template <int ACT, int NST>
__global__ __launch_bounds__(NT) void k_gat_fwd_ps(const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col,
                                                  const float* __restrict__ XP,
                                                  const float* __restrict__ a_s,
                                                  const float* __restrict__ a_d, int64_t M, int H,
                                                  int C, int s0, float slope,
                                                  const float* __restrict__ mask,
                                                  const float* __restrict__ bias,
                                                  float* __restrict__ alpha, float* __restrict__ Y,
                                                  uint16_t* __restrict__ Yb) {
  const EdgeLane L(H);
  const int HC = H * C;
  const int hps = 128 / C < H ? 128 / C : H;  // heads per strip
  RowWalk W = row_walk(M);
  if (W.r >= W.rend) return;
  // per strip: the feature lane's pass, its head's edge lanes, and this edge lane's head
  Pass<1> P[NST];
  int hbase[NST], hq[NST];
  bool hv[NST];
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    P[st] = Pass<1>(s0 + st, L.li, HC, C);
    hbase[st] = L.hwb + 8 * (P[st].head - (s0 + st) * hps);
    const int he = (s0 + st) * hps + L.hh;
    hv[st] = L.hh < hps && he < H;
    hq[st] = hv[st] ? he : 0;
  }
  const int64_t cap = rowptr[M];
  const Buf bR = mkbuf(rowptr, (M + 1) * 4), bC = mkbuf(col, cap * 4);
  const Buf bX = mkbuf(XP, M * HC * 4), bA = mkbuf(a_s, M * H * 4), bD = mkbuf(a_d, M * H * 4);
  const Buf bAl = mkbuf(alpha, alpha ? cap * H * 4 : 0), bM = mkbuf(mask, mask ? cap * H * 4 : 0);
  int64_t r = W.r;
  int e0 = bldi(bR, (uint32_t)r * 4u), e1 = bldi(bR, (uint32_t)r * 4u + 4u);
  int cu = bldi(bC, (uint32_t)L.pos(e0, e1) * 4u);
  int64_t rn = r + W.step;
  uint32_t ro = rn < W.rend ? (uint32_t)rn * 4u : OOB;
  int e0n = bldi(bR, ro), e1n = bldi(bR, ro + 4u);
  for (;;) {
    const int deg = e1 - e0;
    // row r: edge lanes load the logit inputs, feature lanes gather the first batch's rows
    const int eu = L.pos(e0, e1);
    float a[NST], ad[NST], mk[NST];
    f32x4 xv[NST][EB];
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      a[st] = bld1(bA, (uint32_t)(cu * H + hq[st]) * 4u);
      ad[st] = bld1(bD, (uint32_t)(r * H + hq[st]) * 4u);
      mk[st] = mask ? bld1(bM, (uint32_t)(eu * H + hq[st]) * 4u) : 1.f;
#pragma unroll
      for (int k = 0; k < EB; ++k)
        xv[st][k] = bld4(bX, ((uint32_t)bperm_i(cu, L.hwb + k) * HC + P[st].fc[0]) * 4u);
    }
    // row r + step: its first batch's columns; row r + 2 step: its extent
    const int64_t rnn = rn + W.step;
    const int cun = bldi(bC, rn < W.rend ? (uint32_t)L.pos(e0n, e1n) * 4u : OOB);
    const uint32_t ron = rnn < W.rend ? (uint32_t)rnn * 4u : OOB;
    const int e0nn = bldi(bR, ron), e1nn = bldi(bR, ron + 4u);
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (deg <= EB) {
        const bool ev = L.u < deg && hv[st];
        const float lg = leaky(a[st] + ad[st], slope);
        const float m = max8(ev ? lg : -INFINITY);
        const float ex = ev ? expf(lg - m) : 0.f;
        float sum = 0.f;  // in CSR order (the zeros of absent edges add exactly nothing)
#pragma unroll
        for (int k = 0; k < EB; ++k) sum += bperm_f(ex, L.hwb + 8 * L.hh + k);
        sum += EPS16;
        const float al = ex / sum;
        if (alpha && ev) bst1(bAl, (uint32_t)(eu * H + hq[st]) * 4u, al);
        const float alm = mask ? al * mk[st] : al;
#pragma unroll
        for (int k = 0; k < EB; ++k) {
          const float w = bperm_f(alm, hbase[st] + k);
          if (k < deg) acc += w * xv[st][k];
        }
      } else {  // long row: max, denominator, messages, each a walk over batches of EB entries
        float m = -INFINITY;
        for (int b = e0; b < e1; b += EB) {
          const int c = bldi(bC, (uint32_t)L.pos(b, e1) * 4u);
          const float lg = leaky(bld1(bA, (uint32_t)(c * H + hq[st]) * 4u) + ad[st], slope);
          if (b + L.u < e1 && hv[st]) m = fmaxf(m, lg);
        }
        m = max8(m);
        float sum = 0.f;
        for (int b = e0; b < e1; b += EB) {
          const int c = bldi(bC, (uint32_t)L.pos(b, e1) * 4u);
          const float lg = leaky(bld1(bA, (uint32_t)(c * H + hq[st]) * 4u) + ad[st], slope);
          const float ex = b + L.u < e1 && hv[st] ? expf(lg - m) : 0.f;
#pragma unroll
          for (int k = 0; k < EB; ++k) sum += bperm_f(ex, L.hwb + 8 * L.hh + k);
        }
        sum += EPS16;
        for (int b = e0; b < e1; b += EB) {
          const int eb = L.pos(b, e1);
          const bool ev = b + L.u < e1 && hv[st];
          const int c = bldi(bC, (uint32_t)eb * 4u);
          const float lg = leaky(bld1(bA, (uint32_t)(c * H + hq[st]) * 4u) + ad[st], slope);
          const float mb = mask ? bld1(bM, (uint32_t)(eb * H + hq[st]) * 4u) : 1.f;
          f32x4 xb[EB];
#pragma unroll
          for (int k = 0; k < EB; ++k)
            xb[k] = bld4(bX, ((uint32_t)bperm_i(c, L.hwb + k) * HC + P[st].fc[0]) * 4u);
          const float al = (ev ? expf(lg - m) : 0.f) / sum;
          if (alpha && ev) bst1(bAl, (uint32_t)(eb * H + hq[st]) * 4u, al);
          const float alm = mask ? al * mb : al;
#pragma unroll
          for (int k = 0; k < EB; ++k) {
            const float w = bperm_f(alm, hbase[st] + k);
            if (b + k < e1) acc += w * xb[k];
          }
        }
      }
      const f32x4 out[1] = {acc};
      gat_out<ACT, 1>(P[st], out, bias, Y, Yb, r * HC);
    }
    if (rn >= W.rend) break;
    r = rn;
    rn = rnn;
    e0 = e0n;
    e1 = e1n;
    cu = cun;
    e0n = e0nn;
    e1n = e1nn;
  }
}

// NST strips as in k_gat_fwd_ps (two-strip shapes only, as there): the row's loads of every strip issued together, then each
// strip's logit gradients for its heads.
template <int ACT, bool POOL, int NST>
__global__ __launch_bounds__(NT) void k_gat_bwd_edge_ps(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ XP, const float* __restrict__ a_s, const float* __restrict__ a_d,
    const float* __restrict__ alpha, const float* __restrict__ mask, const float* __restrict__ dY,
    const float* __restrict__ Y, int64_t M, int H, int C, int s0, float slope,
    float* __restrict__ dZ, float* __restrict__ da_e, float* __restrict__ da_d, PoolGrad pg) {
  const EdgeLane L(H);
  const int HC = H * C;
  const int hps = 128 / C < H ? 128 / C : H;  // heads per strip
  Pass<1> P[NST];
  int hbase[NST], hlead[NST], hq[NST];
  bool hv[NST];
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    P[st] = Pass<1>(s0 + st, L.li, HC, C);
    hbase[st] = L.hwb + 8 * (P[st].head - (s0 + st) * hps);
    const int he = (s0 + st) * hps + L.hh;
    hv[st] = L.hh < hps && he < H;
    hq[st] = hv[st] ? he : (s0 + st) * hps;
    hlead[st] = L.hwb + (hq[st] - (s0 + st) * hps) * P[st].G;  // the first feature lane of that head
  }
  RowWalk W = row_walk(M);
  if (W.r >= W.rend) return;
  const int64_t cap = rowptr[M];
  const Buf bR = mkbuf(rowptr, (M + 1) * 4), bC = mkbuf(col, cap * 4);
  const Buf bX = mkbuf(XP, M * HC * 4), bA = mkbuf(a_s, M * H * 4), bD = mkbuf(a_d, M * H * 4);
  const Buf bAl = mkbuf(alpha, cap * H * 4), bM = mkbuf(mask, mask ? cap * H * 4 : 0);
  const Buf bDa = mkbuf(da_e, cap * H * 4);
  int64_t r = W.r;
  int e0 = bldi(bR, (uint32_t)r * 4u), e1 = bldi(bR, (uint32_t)r * 4u + 4u);
  int cu = bldi(bC, (uint32_t)L.pos(e0, e1) * 4u);
  int64_t rn = r + W.step;
  uint32_t ro = rn < W.rend ? (uint32_t)rn * 4u : OOB;
  int e0n = bldi(bR, ro), e1n = bldi(bR, ro + 4u);
  for (;;) {
    const int deg = e1 - e0;
    const int eu = L.pos(e0, e1);
    float al[NST], mk[NST], pre[NST];
    f32x4 xv[NST][EB], dz[NST];
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      al[st] = bld1(bAl, (uint32_t)(eu * H + hq[st]) * 4u);
      mk[st] = mask ? bld1(bM, (uint32_t)(eu * H + hq[st]) * 4u) : 1.f;
      pre[st] = bld1(bA, (uint32_t)(cu * H + hq[st]) * 4u) +
                bld1(bD, (uint32_t)(r * H + hq[st]) * 4u);
#pragma unroll
      for (int k = 0; k < EB; ++k)
        xv[st][k] = bld4(bX, ((uint32_t)bperm_i(cu, L.hwb + k) * HC + P[st].fc[0]) * 4u);
      dz[st] = dz_row<ACT, POOL>(r, HC, P[st].fc[0], dY, Y, pg);
    }
    const int64_t rnn = rn + W.step;
    const int cun = bldi(bC, rn < W.rend ? (uint32_t)L.pos(e0n, e1n) * 4u : OOB);
    const uint32_t ron = rnn < W.rend ? (uint32_t)rnn * 4u : OOB;
    const int e0nn = bldi(bR, ron), e1nn = bldi(bR, ron + 4u);
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      const Pass<1>& Ps = P[st];
      if (!Ps.act[0]) dz[st] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (Ps.act[0]) st4(dZ + r * HC + Ps.f[0], dz[st]);
      float dad = 0.f;
      if (deg <= EB) {
        float d[EB], alk[EB];
        float s_i = 0.f;
#pragma unroll
        for (int k = 0; k < EB; ++k) {
          d[k] = group_sum(dot4(dz[st], xv[st][k]), Ps.G);
          if (mask) d[k] *= bperm_f(mk[st], hbase[st] + k);
          alk[k] = bperm_f(al[st], hbase[st] + k);
          if (k < deg) s_i += alk[k] * d[k];
        }
        float mine = 0.f;  // edge lane (u, h): the logit gradient of its edge and head
#pragma unroll
        for (int k = 0; k < EB; ++k) {
          const float fk = bperm_f(pre[st] > 0.f ? 1.f : slope, hbase[st] + k);
          const float da = alk[k] * (d[k] - s_i) * fk;
          if (k < deg) dad += opaque(da);  // (never contracted with da's product: every form alike)
          const float t = bperm_f(da, hlead[st]);
          mine = L.u == k ? t : mine;
        }
        if (L.u < deg && hv[st]) bst1(bDa, (uint32_t)(eu * H + hq[st]) * 4u, mine);
      } else {  // long row: two walks over batches of EB entries (s_i, then the gradients)
        float s_i = 0.f;
#pragma unroll 1
        for (int sweep = 0; sweep < 2; ++sweep) {
          for (int b = e0; b < e1; b += EB) {
            const int eb = L.pos(b, e1);
            const int c = bldi(bC, (uint32_t)eb * 4u);
            const float alb = bld1(bAl, (uint32_t)(eb * H + hq[st]) * 4u);
            const float mb = mask ? bld1(bM, (uint32_t)(eb * H + hq[st]) * 4u) : 1.f;
            const float preb = bld1(bA, (uint32_t)(c * H + hq[st]) * 4u) +
                               bld1(bD, (uint32_t)(r * H + hq[st]) * 4u);
            f32x4 xb[EB];
#pragma unroll
            for (int k = 0; k < EB; ++k)
              xb[k] = bld4(bX, ((uint32_t)bperm_i(c, L.hwb + k) * HC + Ps.fc[0]) * 4u);
            float mine = 0.f;
#pragma unroll
            for (int k = 0; k < EB; ++k) {
              float dk = group_sum(dot4(dz[st], xb[k]), Ps.G);
              if (mask) dk *= bperm_f(mb, hbase[st] + k);
              const float ak = bperm_f(alb, hbase[st] + k);
              const float fk = bperm_f(preb > 0.f ? 1.f : slope, hbase[st] + k);
              if (sweep == 0) {
                if (b + k < e1) s_i += ak * dk;
              } else {
                const float da = ak * (dk - s_i) * fk;
                if (b + k < e1) dad += opaque(da);  // (never contracted with da's product: every form alike)
                const float t = bperm_f(da, hlead[st]);
                mine = L.u == k ? t : mine;
              }
            }
            if (sweep == 1 && b + L.u < e1 && hv[st])
              bst1(bDa, (uint32_t)(eb * H + hq[st]) * 4u, mine);
          }
        }
      }
      if (Ps.leader) da_d[r * H + Ps.head] = dad;
    }
    if (rn >= W.rend) break;
    r = rn;
    rn = rnn;
    e0 = e0n;
    e1 = e1n;
    cu = cun;
    e0n = e0nn;
    e1n = e1nn;
  }
}

// source-row pass, NST strips (two-strip shapes only, as k_gat_fwd_ps)
template <int NST>
__global__ __launch_bounds__(NT) void k_gat_bwd_node_ps(
    const int32_t* __restrict__ tptr, const int32_t* __restrict__ tidx,
    const int32_t* __restrict__ tmap, const float* __restrict__ alpha,
    const float* __restrict__ mask, const float* __restrict__ da_e,
    const float* __restrict__ da_d, const float* __restrict__ dZ, const float* __restrict__ XP,
    const float* __restrict__ att_src, const float* __restrict__ att_dst, int64_t M, int H,
    int C, int s0, float* __restrict__ dXP, float* __restrict__ part,
    uint16_t* __restrict__ dXPb) {
  constexpr int SW = 128 * NST;  // features of the partial rows in LDS
  __shared__ __attribute__((aligned(16))) float red[RB][3 * SW];
  const EdgeLane L(H);
  const int HC = H * C;
  const int hps = 128 / C < H ? 128 / C : H;  // heads per strip
  Pass<1> P[NST];
  int hbase[NST], hq[NST];
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    P[st] = Pass<1>(s0 + st, L.li, HC, C);
    hbase[st] = L.hwb + 8 * (P[st].head - (s0 + st) * hps);
    const int he = (s0 + st) * hps + L.hh;
    hq[st] = L.hh < hps && he < H ? he : (s0 + st) * hps;
  }
  const int hw = (threadIdx.x >> 6) * 2 + ((threadIdx.x & 63) >> 5);
  f32x4 ps[NST], pd[NST], pb[NST];
#pragma unroll
  for (int st = 0; st < NST; ++st) ps[st] = pd[st] = pb[st] = f32x4{0.f, 0.f, 0.f, 0.f};
  RowWalk W = row_walk(M);
  if (W.r < W.rend) {
    const int64_t cap = tptr[M];
    const Buf bR = mkbuf(tptr, (M + 1) * 4), bT = mkbuf(tidx, cap * 4), bP = mkbuf(tmap, cap * 4);
    const Buf bZ = mkbuf(dZ, M * HC * 4), bAl = mkbuf(alpha, cap * H * 4);
    const Buf bM = mkbuf(mask, mask ? cap * H * 4 : 0), bDa = mkbuf(da_e, cap * H * 4);
    f32x4 as[NST], adv[NST];
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      as[st] = ld4(att_src + P[st].fc[0]);
      adv[st] = ld4(att_dst + P[st].fc[0]);
    }
    int64_t r = W.r;
    int q0 = bldi(bR, (uint32_t)r * 4u), q1 = bldi(bR, (uint32_t)r * 4u + 4u);
    int tu = bldi(bT, (uint32_t)L.pos(q0, q1) * 4u), pu = bldi(bP, (uint32_t)L.pos(q0, q1) * 4u);
    int64_t rn = r + W.step;
    uint32_t ro = rn < W.rend ? (uint32_t)rn * 4u : OOB;
    int q0n = bldi(bR, ro), q1n = bldi(bR, ro + 4u);
    for (;;) {
      const int deg = q1 - q0;
      float alu[NST], mk[NST], dau[NST], dd[NST];
      f32x4 dv[NST][EB], xp[NST], zr[NST];
#pragma unroll
      for (int st = 0; st < NST; ++st) {
        alu[st] = bld1(bAl, (uint32_t)(pu * H + hq[st]) * 4u);
        mk[st] = mask ? bld1(bM, (uint32_t)(pu * H + hq[st]) * 4u) : 1.f;
        dau[st] = bld1(bDa, (uint32_t)(pu * H + hq[st]) * 4u);
#pragma unroll
        for (int k = 0; k < EB; ++k)
          dv[st][k] = bld4(bZ, ((uint32_t)bperm_i(tu, L.hwb + k) * HC + P[st].fc[0]) * 4u);
        dd[st] = da_d[r * H + P[st].head];
        xp[st] = ld4(XP + r * HC + P[st].fc[0]);
        zr[st] = ld4(dZ + r * HC + P[st].fc[0]);
      }
      const int64_t rnn = rn + W.step;
      const uint32_t qn = rn < W.rend ? (uint32_t)L.pos(q0n, q1n) * 4u : OOB;
      const int tun = bldi(bT, qn), pun = bldi(bP, qn);
      const uint32_t ron = rnn < W.rend ? (uint32_t)rnn * 4u : OOB;
      const int q0nn = bldi(bR, ron), q1nn = bldi(bR, ron + 4u);
#pragma unroll
      for (int st = 0; st < NST; ++st) {
        if (mask) alu[st] *= mk[st];
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        float sda = 0.f;
#pragma unroll
        for (int k = 0; k < EB; ++k) {
          const float ak = bperm_f(alu[st], hbase[st] + k), dk = bperm_f(dau[st], hbase[st] + k);
          if (k < deg) {
            acc += ak * dv[st][k];
            sda += dk;
          }
        }
        for (int b = q0 + EB; b < q1; b += EB) {  // entries past the first batch
          const int qb = L.pos(b, q1);
          const int tb = bldi(bT, (uint32_t)qb * 4u), pb_ = bldi(bP, (uint32_t)qb * 4u);
          float alb = bld1(bAl, (uint32_t)(pb_ * H + hq[st]) * 4u);
          if (mask) alb *= bld1(bM, (uint32_t)(pb_ * H + hq[st]) * 4u);
          const float dab = bld1(bDa, (uint32_t)(pb_ * H + hq[st]) * 4u);
          f32x4 db[EB];
#pragma unroll
          for (int k = 0; k < EB; ++k)
            db[k] = bld4(bZ, ((uint32_t)bperm_i(tb, L.hwb + k) * HC + P[st].fc[0]) * 4u);
#pragma unroll
          for (int k = 0; k < EB; ++k) {
            const float ak = bperm_f(alb, hbase[st] + k), dk = bperm_f(dab, hbase[st] + k);
            if (b + k < q1) {
              acc += ak * db[k];
              sda += dk;
            }
          }
        }
        const f32x4 o = acc + sda * as[st] + dd[st] * adv[st];
        if (P[st].act[0]) {
          st4(dXP + r * HC + P[st].f[0], o);
          if (dXPb) st4_bf16(dXPb + r * HC + P[st].f[0], o);
          ps[st] += sda * xp[st];
          pd[st] += dd[st] * xp[st];
          pb[st] += zr[st];
        }
      }
      if (rn >= W.rend) break;
      r = rn;
      rn = rnn;
      q0 = q0n;
      q1 = q1n;
      tu = tun;
      pu = pun;
      q0n = q0nn;
      q1n = q1nn;
    }
  }
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    st4(&red[hw][0 * SW + 128 * st + 4 * L.li], ps[st]);
    st4(&red[hw][1 * SW + 128 * st + 4 * L.li], pd[st]);
    st4(&red[hw][2 * SW + 128 * st + 4 * L.li], pb[st]);
  }
  __syncthreads();
  // this launch's features [128 s0, 128 s0 + SW) of each partial row
  for (int i = threadIdx.x; i < 3 * SW; i += NT) {
    const int kind = i / SW, fl = i % SW, f = 128 * s0 + fl;
    if (f >= HC) continue;
    float t = red[0][i];
#pragma unroll
    for (int q = 1; q < RB; ++q) t += red[q][i];
    part[(int64_t)blockIdx.x * 3 * HC + kind * HC + f] = t;
  }
}

// the pipelined kernels' shapes, and whether they are enabled (LGNN_OPT_GAT_PIPE = 0: the
// kernels above)
inline bool pipe_ok(int H, int C) {
  return H <= 8 && H * C <= 128 && lgnn_option(LGNN_OPT_GAT_PIPE) != 0;
}
// the two-strip forms: 128 < H*C <= 512, 32 <= C <= 128 (the sweep's GAT widths 256 and 512 at
// 2..8 heads), one launch per 256 features (a pass's heads are independent of the others')
inline bool pipe2_ok(int H, int C) {
  return H * C > 128 && H * C <= 512 && C >= 32 && C <= 128 &&
         lgnn_option(LGNN_OPT_GAT_PIPE) != 0;
}

// persistent grid of a row-pipelined kernel: the workgroups one launch keeps resident (occupancy
// API, cached per device and kernel), LGNN_OPT_GAT_BPC per CU if set
template <typename K>
inline unsigned pipe_grid(K kernel, int slot, int64_t M) {
  static int cap[16][24];  // [device][kernel slot]
  int dev = 0;
  (void)hipGetDevice(&dev);
  dev &= 15;
  if (cap[dev][slot] <= 0) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, NT, 0) != hipSuccess || per < 1)
      per = 4;
    cap[dev][slot] = cus * per;
  }
  int64_t c = cap[dev][slot];
  if (const int bpc = lgnn_option(LGNN_OPT_GAT_BPC)) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      c = (int64_t)cus * bpc;
  }
  int64_t g = (M + RB - 1) / RB;
  if (g > c) g = c;
  return (unsigned)(g < 8 ? 8 : g);
}

// C a power of two in [4, 512] (the reference sweep: widths 32..512, heads 1/2/4/8), H*C <= 512
inline bool shape_ok(int H, int C) {
  return H > 0 && C >= 4 && C <= 512 && (C & (C - 1)) == 0 && H * C <= MAXS * 128;
}

inline int ns_of(int C) { return C <= 128 ? 1 : C / 128; }

inline unsigned row_grid(int64_t M) { return (unsigned)((M + RB - 1) / RB); }

// node arrays addressed by 32-bit byte offsets (the per-edge arrays: documented in lgnn.h)
inline bool bytes_ok(int64_t M, int H, int C) { return M * H * C * 4 < ((int64_t)1 << 32); }

}  // namespace

extern "C" int lgnn_gat_att(const float* XP, int64_t M, int H, int C, const float* att_src,
                            const float* att_dst, float* a_s, float* a_d, void* stream) {
  if (M < 0 || !shape_ok(H, C) || !att_src || !att_dst || (M > 0 && (!XP || !a_s || !a_d)))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
#define LGNN_ATT(NS_)                                                                       \
  hipLaunchKernelGGL(k_gat_att<NS_>, dim3(row_grid(M)), dim3(NT), 0, as_stream(stream), XP, M, H, \
                     C, att_src, att_dst, a_s, a_d)
  switch (ns_of(C)) {
    case 1: LGNN_ATT(1); break;
    case 2: LGNN_ATT(2); break;
    default: LGNN_ATT(4); break;
  }
#undef LGNN_ATT
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_gat_fwd(const int32_t* rowptr, const int32_t* col, const float* XP,
                            const float* a_s, const float* a_d, int64_t M, int H, int C,
                            float negative_slope, const float* edge_mask, const float* bias,
                            int act, float* alpha, float* Y, uint16_t* Y_bf16, void* stream) {
  if (M < 0 || !shape_ok(H, C) || (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU))
    return LGNN_EINVAL;
  if (M > 0 && (!rowptr || !col || !XP || !a_s || !a_d || !Y)) return LGNN_EINVAL;
  if (!bytes_ok(M, H, C)) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  if (pipe2_ok(H, C)) {
#define LGNN_GFS(A_, SLOT_)                                                                     \
  hipLaunchKernelGGL((k_gat_fwd_ps<A_, 2>), dim3(pipe_grid(k_gat_fwd_ps<A_, 2>, SLOT_, M)),        \
                     dim3(NT), 0, as_stream(stream), rowptr, col, XP, a_s, a_d, M, H, C, s0,       \
                     negative_slope, edge_mask, bias, alpha, Y, Y_bf16)
    for (int s0 = 0; 128 * s0 < H * C; s0 += 2) {
      if (act == LGNN_ACT_ELU) LGNN_GFS(LGNN_ACT_ELU, 6);
      else LGNN_GFS(LGNN_ACT_NONE, 7);
    }
#undef LGNN_GFS
    LGNN_LAUNCH_CHECK();
    return LGNN_OK;
  }
  if (pipe_ok(H, C)) {
#define LGNN_GFP(A_, HS_, SLOT_)                                                                \
  hipLaunchKernelGGL((k_gat_fwd_p<A_, HS_>), dim3(pipe_grid(k_gat_fwd_p<A_, HS_>, SLOT_, M)),      \
                     dim3(NT), 0, as_stream(stream), rowptr, col, XP, a_s, a_d, M, H, C,            \
                     negative_slope, edge_mask, bias, alpha, Y, Y_bf16)
    if (H <= 4) {
      if (act == LGNN_ACT_ELU) LGNN_GFP(LGNN_ACT_ELU, 1, 0); else LGNN_GFP(LGNN_ACT_NONE, 1, 1);
    } else {
      if (act == LGNN_ACT_ELU) LGNN_GFP(LGNN_ACT_ELU, 2, 12); else LGNN_GFP(LGNN_ACT_NONE, 2, 13);
    }
#undef LGNN_GFP
    LGNN_LAUNCH_CHECK();
    return LGNN_OK;
  }
#define LGNN_GF(A_, NS_)                                                                     \
  hipLaunchKernelGGL((k_gat_fwd<A_, NS_>), dim3(row_grid(M)), dim3(NT), 0, as_stream(stream),    \
                     rowptr, col, XP, a_s, a_d, M, H, C, negative_slope, edge_mask, bias, alpha, Y, \
                     Y_bf16)
#define LGNN_GF_NS(A_)                    \
  switch (ns_of(C)) {                     \
    case 1: LGNN_GF(A_, 1); break;        \
    case 2: LGNN_GF(A_, 2); break;        \
    default: LGNN_GF(A_, 4); break;       \
  }
  if (act == LGNN_ACT_ELU) {
    LGNN_GF_NS(LGNN_ACT_ELU)
  } else {
    LGNN_GF_NS(LGNN_ACT_NONE)
  }
#undef LGNN_GF_NS
#undef LGNN_GF
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

namespace {
int gat_bwd_edge_launch(const int32_t* rowptr, const int32_t* col, const float* XP,
                        const float* a_s, const float* a_d, const float* alpha,
                        const float* edge_mask, const float* dY, const float* Y, int act,
                        int64_t M, int H, int C, float slope, float* dZ, float* da_e, float* da_d,
                        const PoolGrad* pg, void* stream) {
  if (M < 0 || !shape_ok(H, C) || (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU))
    return LGNN_EINVAL;
  if (M > 0 && (!rowptr || !col || !XP || !a_s || !a_d || !alpha || (!dY && !pg) || !dZ ||
                !da_e || !da_d))
    return LGNN_EINVAL;
  if (act == LGNN_ACT_ELU && M > 0 && !Y) return LGNN_EINVAL;
  if (!bytes_ok(M, H, C)) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  const PoolGrad p = pg ? *pg : PoolGrad{};
  if (pipe2_ok(H, C)) {
#define LGNN_GBS(A_, POOL_, SLOT_)                                                             \
  hipLaunchKernelGGL((k_gat_bwd_edge_ps<A_, POOL_, 2>),                                         \
                     dim3(pipe_grid(k_gat_bwd_edge_ps<A_, POOL_, 2>, SLOT_, M)), dim3(NT), 0,    \
                     as_stream(stream), rowptr, col, XP, a_s, a_d, alpha, edge_mask, dY, Y, M, H, \
                     C, s0, slope, dZ, da_e, da_d, p)
    for (int s0 = 0; 128 * s0 < H * C; s0 += 2) {
      if (act == LGNN_ACT_ELU) {
        if (pg) LGNN_GBS(LGNN_ACT_ELU, true, 8); else LGNN_GBS(LGNN_ACT_ELU, false, 9);
      } else {
        if (pg) LGNN_GBS(LGNN_ACT_NONE, true, 10); else LGNN_GBS(LGNN_ACT_NONE, false, 11);
      }
    }
#undef LGNN_GBS
    LGNN_LAUNCH_CHECK();
    return LGNN_OK;
  }
  if (pipe_ok(H, C)) {
#define LGNN_GBP(A_, POOL_, HS_, SLOT_)                                                        \
  hipLaunchKernelGGL((k_gat_bwd_edge_p<A_, POOL_, HS_>),                                        \
                     dim3(pipe_grid(k_gat_bwd_edge_p<A_, POOL_, HS_>, SLOT_, M)), dim3(NT), 0,   \
                     as_stream(stream), rowptr, col, XP, a_s, a_d, alpha, edge_mask, dY, Y, M, H, \
                     C, slope, dZ, da_e, da_d, p)
    if (H <= 4) {
      if (act == LGNN_ACT_ELU) {
        if (pg) LGNN_GBP(LGNN_ACT_ELU, true, 1, 2); else LGNN_GBP(LGNN_ACT_ELU, false, 1, 3);
      } else {
        if (pg) LGNN_GBP(LGNN_ACT_NONE, true, 1, 4); else LGNN_GBP(LGNN_ACT_NONE, false, 1, 5);
      }
    } else {
      if (act == LGNN_ACT_ELU) {
        if (pg) LGNN_GBP(LGNN_ACT_ELU, true, 2, 14); else LGNN_GBP(LGNN_ACT_ELU, false, 2, 15);
      } else {
        if (pg) LGNN_GBP(LGNN_ACT_NONE, true, 2, 16); else LGNN_GBP(LGNN_ACT_NONE, false, 2, 17);
      }
    }
#undef LGNN_GBP
    LGNN_LAUNCH_CHECK();
    return LGNN_OK;
  }
#define LGNN_GB(A_, NS_)                                                                        \
  do {                                                                                          \
    if (pg)                                                                                     \
      hipLaunchKernelGGL((k_gat_bwd_edge<A_, NS_, true>), dim3(row_grid(M)), dim3(NT), 0,        \
                         as_stream(stream), rowptr, col, XP, a_s, a_d, alpha, edge_mask, dY, Y, \
                         M, H, C, slope, dZ, da_e, da_d, p);                                    \
    else                                                                                        \
      hipLaunchKernelGGL((k_gat_bwd_edge<A_, NS_, false>), dim3(row_grid(M)), dim3(NT), 0,       \
                         as_stream(stream), rowptr, col, XP, a_s, a_d, alpha, edge_mask, dY, Y, \
                         M, H, C, slope, dZ, da_e, da_d, p);                                    \
  } while (0)
#define LGNN_GB_NS(A_)                    \
  switch (ns_of(C)) {                     \
    case 1: LGNN_GB(A_, 1); break;        \
    case 2: LGNN_GB(A_, 2); break;        \
    default: LGNN_GB(A_, 4); break;       \
  }
  if (act == LGNN_ACT_ELU) {
    LGNN_GB_NS(LGNN_ACT_ELU)
  } else {
    LGNN_GB_NS(LGNN_ACT_NONE)
  }
#undef LGNN_GB_NS
#undef LGNN_GB
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
}  // namespace

extern "C" int lgnn_gat_bwd_edge(const int32_t* rowptr, const int32_t* col, const float* XP,
                                 const float* a_s, const float* a_d, const float* alpha,
                                 const float* edge_mask, const float* dY, const float* Y,
                                 int act, int64_t M, int H, int C, float negative_slope,
                                 float* dZ, float* da_e, float* da_d, void* stream) {
  if (M > 0 && !dY) return LGNN_EINVAL;
  return gat_bwd_edge_launch(rowptr, col, XP, a_s, a_d, alpha, edge_mask, dY, Y, act, M, H, C,
                             negative_slope, dZ, da_e, da_d, nullptr, stream);
}

extern "C" int lgnn_gat_bwd_edge_pool(const int32_t* rowptr, const int32_t* col, const float* XP,
                                      const float* a_s, const float* a_d, const float* alpha,
                                      const float* edge_mask, const float* Y, int act, int64_t M,
                                      int H, int C, float negative_slope, const int64_t* batch,
                                      const int32_t* gptr, int pool_mean, const float* dlogits,
                                      const float* Wout, int num_classes, float* dZ, float* da_e,
                                      float* da_d, void* stream) {
  if (M > 0 && (!batch || !gptr || !dlogits || !Wout || num_classes < 1)) return LGNN_EINVAL;
  const PoolGrad pg{batch, gptr, dlogits, Wout, num_classes, pool_mean ? 1 : 0};
  return gat_bwd_edge_launch(rowptr, col, XP, a_s, a_d, alpha, edge_mask, nullptr, Y, act, M, H,
                             C, negative_slope, dZ, da_e, da_d, &pg, stream);
}

extern "C" int lgnn_gat_bwd_num_partials(int64_t M) {
  if (M < 0) return LGNN_EINVAL;
  // persistent rows; enough workgroups to keep LGNN_GAT_WPE waves per SIMD resident
  const int64_t b = (M + RB - 1) / RB;
  // (>= 8: the row-pipelined kernel deals rows to the 8 XCDs' workgroups; <= 1024: 4 per CU,
  // what its registers keep resident — a second round of workgroups would not be pipelined)
  return (int)(b < 8 ? 8 : (b > 1024 ? 1024 : b));
}

extern "C" int lgnn_gat_bwd_node(const int32_t* tptr, const int32_t* tidx, const int32_t* tmap,
                                 const float* alpha, const float* edge_mask, const float* da_e,
                                 const float* da_d, const float* dZ, const float* XP,
                                 const float* att_src, const float* att_dst, int64_t M, int H,
                                 int C, float* dXP, float* partials, int num_partials,
                                 uint16_t* dXP_bf16, void* stream) {
  if (M < 0 || !shape_ok(H, C) || !att_src || !att_dst || !partials) return LGNN_EINVAL;
  if (num_partials != lgnn_gat_bwd_num_partials(M)) return LGNN_EINVAL;
  if (M > 0 && (!tptr || !tidx || !tmap || !alpha || !da_e || !da_d || !dZ || !XP || !dXP))
    return LGNN_EINVAL;
  if (!bytes_ok(M, H, C)) return LGNN_EINVAL;
  if (pipe2_ok(H, C) && M > 0) {
    for (int s0 = 0; 128 * s0 < H * C; s0 += 2)
      hipLaunchKernelGGL(k_gat_bwd_node_ps<2>, dim3(num_partials), dim3(NT), 0,
                         as_stream(stream), tptr, tidx, tmap, alpha, edge_mask, da_e, da_d, dZ, XP,
                         att_src, att_dst, M, H, C, s0, dXP, partials, dXP_bf16);
    LGNN_LAUNCH_CHECK();
    return LGNN_OK;
  }
  if (pipe_ok(H, C) && M > 0) {
    if (H <= 4)
      hipLaunchKernelGGL(k_gat_bwd_node_p<1>, dim3(num_partials), dim3(NT), 0, as_stream(stream),
                         tptr, tidx, tmap, alpha, edge_mask, da_e, da_d, dZ, XP, att_src, att_dst,
                         M, H, C, dXP, partials, dXP_bf16);
    else
      hipLaunchKernelGGL(k_gat_bwd_node_p<2>, dim3(num_partials), dim3(NT), 0, as_stream(stream),
                         tptr, tidx, tmap, alpha, edge_mask, da_e, da_d, dZ, XP, att_src, att_dst,
                         M, H, C, dXP, partials, dXP_bf16);
    LGNN_LAUNCH_CHECK();
    return LGNN_OK;
  }
#define LGNN_GN(NST_)                                                                        \
  hipLaunchKernelGGL(k_gat_bwd_node<NST_>, dim3(num_partials), dim3(NT), 0, as_stream(stream),  \
                     tptr, tidx, tmap, alpha, edge_mask, da_e, da_d, dZ, XP, att_src, att_dst, M, \
                     H, C, dXP, partials, dXP_bf16)
  switch ((H * C + 127) / 128) {
    case 1: LGNN_GN(1); break;
    case 2: LGNN_GN(2); break;
    default: LGNN_GN(4); break;
  }
#undef LGNN_GN
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
