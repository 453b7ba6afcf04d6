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

__device__ __forceinline__ float leaky(float v, float slope) { return v > 0.f ? v : v * slope; }

// sum over the G = C/4 lanes of a head group (all lanes receive the sum)
__device__ __forceinline__ float group_sum(float v, int G) {
  for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
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
  l.row = (int64_t)blockIdx.x * RB + l.hw;
  return l;
}

// ------------------------------------------------------------------------------------------
// a_s / a_d
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_gat_att(const float* __restrict__ XP, int64_t M, int H,
                                                int C, const float* __restrict__ att_src,
                                                const float* __restrict__ att_dst,
                                                float* __restrict__ a_s, float* __restrict__ a_d) {
  const Lane L = lane_row();
  if (L.row >= M) return;
  const int HC = H * C, G = C / 4;
  for (int s0 = 0; s0 < HC; s0 += 128) {
    const int f = s0 + 4 * L.li;
    const bool act = f < HC;
    const int fc = act ? f : HC - 4;
    const f32x4 v = ld4(XP + L.row * HC + fc);
    float ps = act ? dot4(v, ld4(att_src + fc)) : 0.f;
    float pd = act ? dot4(v, ld4(att_dst + fc)) : 0.f;
    ps = group_sum(ps, G);
    pd = group_sum(pd, G);
    if (act && (L.li % G) == 0) {
      a_s[L.row * H + f / C] = ps;
      a_d[L.row * H + f / C] = pd;
    }
  }
}

// ------------------------------------------------------------------------------------------
// forward: softmax over each target row + weighted sum of source rows (+ bias, ELU)
// ------------------------------------------------------------------------------------------
template <int ACT>
__global__ __launch_bounds__(NT) void k_gat_fwd(const int32_t* __restrict__ rowptr,
                                                const int32_t* __restrict__ col,
                                                const float* __restrict__ XP,
                                                const float* __restrict__ a_s,
                                                const float* __restrict__ a_d, int64_t M, int H,
                                                int C, float slope, const float* __restrict__ mask,
                                                const float* __restrict__ bias,
                                                float* __restrict__ alpha, float* __restrict__ Y) {
  const Lane L = lane_row();
  if (L.row >= M) return;
  const int HC = H * C, G = C / 4;
  const int e0 = rowptr[L.row], e1 = rowptr[L.row + 1];
  for (int s0 = 0; s0 < HC; s0 += 128) {
    const int f = s0 + 4 * L.li;
    const bool act = f < HC;
    const int fc = act ? f : HC - 4;
    const int head = fc / C;
    const float ad = a_d[L.row * H + head];
    // pass 1: row max of the logits (PyG: scatter max of the detached logits)
    float m = -INFINITY;
    for (int e = e0; e < e1; e += EB) {
      float v[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int ee = e + u < e1 ? e + u : e0;
        v[u] = a_s[(int64_t)col[ee] * H + head];
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
        v[u] = a_s[(int64_t)col[ee] * H + head];
      }
#pragma unroll
      for (int u = 0; u < EB; ++u)
        if (e + u < e1) sum += expf(leaky(v[u] + ad, slope) - m);
    }
    sum += EPS16;
    // pass 3: alpha, message sum
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const bool leader = act && (L.li % G) == 0;
    for (int e = e0; e < e1; e += EB) {
      int c[EB];
      float a[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int ee = e + u < e1 ? e + u : e0;
        c[u] = col[ee];
        a[u] = a_s[(int64_t)c[u] * H + head];
      }
      f32x4 xv[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) xv[u] = ld4(XP + (int64_t)c[u] * HC + fc);
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        if (e + u < e1) {
          float al = expf(leaky(a[u] + ad, slope) - m) / sum;
          if (leader && alpha) alpha[(int64_t)(e + u) * H + head] = al;
          if (mask) al *= mask[(int64_t)(e + u) * H + head];
          acc += al * xv[u];
        }
      }
    }
    if (act) {
      const f32x4 bv = bias ? ld4(bias + fc) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 o = acc + bv;
      if (ACT == LGNN_ACT_ELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = elu_f(o[j]);
      }
      st4(Y + L.row * HC + f, o);
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward, pass over target rows i:
//   dZ_i = dY_i * act'(Y_i)                                   (written: gathered by the next pass)
//   dal_ij = <dZ_i[h], xp_j[h]> * mask_ij;  s_i = sum_j alpha_ij dal_ij
//   de_ij = alpha_ij (dal_ij - s_i);  da_ij = de_ij * leaky'(a_s[j] + a_d[i])
//   da_e[ij] = da_ij (per edge),  da_d[i] = sum_j da_ij
// ------------------------------------------------------------------------------------------
template <int ACT>
__global__ __launch_bounds__(NT) void k_gat_bwd_edge(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ XP, const float* __restrict__ a_s, const float* __restrict__ a_d,
    const float* __restrict__ alpha, const float* __restrict__ mask, const float* __restrict__ dY,
    const float* __restrict__ Y, int64_t M, int H, int C, float slope, float* __restrict__ dZ,
    float* __restrict__ da_e, float* __restrict__ da_d) {
  const Lane L = lane_row();
  if (L.row >= M) return;
  const int HC = H * C, G = C / 4;
  const int e0 = rowptr[L.row], e1 = rowptr[L.row + 1];
  for (int s0 = 0; s0 < HC; s0 += 128) {
    const int f = s0 + 4 * L.li;
    const bool act = f < HC;
    const int fc = act ? f : HC - 4;
    const int head = fc / C;
    const bool leader = act && (L.li % G) == 0;
    f32x4 dz = ld4(dY + L.row * HC + fc);
    if (ACT == LGNN_ACT_ELU) {
      const f32x4 y = ld4(Y + L.row * HC + fc);
#pragma unroll
      for (int j = 0; j < 4; ++j) dz[j] *= elu_grad_from_out(y[j]);
    }
    if (!act) dz = f32x4{0.f, 0.f, 0.f, 0.f};
    if (act) st4(dZ + L.row * HC + f, dz);
    const float ad = a_d[L.row * H + head];
    // pass 1: s_i
    float s = 0.f;
    for (int e = e0; e < e1; e += EB) {
      int c[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) c[u] = col[e + u < e1 ? e + u : e0];
      f32x4 xv[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) xv[u] = ld4(XP + (int64_t)c[u] * HC + fc);
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int ee = e + u < e1 ? e + u : e0;
        float d = group_sum(dot4(dz, xv[u]), G);
        if (mask) d *= mask[(int64_t)ee * H + head];
        const float al = alpha[(int64_t)ee * H + head];
        if (e + u < e1) s += al * d;
      }
    }
    // pass 2: per-edge logit gradients
    float dad = 0.f;
    for (int e = e0; e < e1; e += EB) {
      int c[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) c[u] = col[e + u < e1 ? e + u : e0];
      f32x4 xv[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) xv[u] = ld4(XP + (int64_t)c[u] * HC + fc);
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int ee = e + u < e1 ? e + u : e0;
        float d = group_sum(dot4(dz, xv[u]), G);
        if (mask) d *= mask[(int64_t)ee * H + head];
        const float al = alpha[(int64_t)ee * H + head];
        const float pre = a_s[(int64_t)c[u] * H + head] + ad;
        const float da = al * (d - s) * (pre > 0.f ? 1.f : slope);
        if (e + u < e1) {
          dad += da;
          if (leader) da_e[(int64_t)ee * H + head] = da;
        }
      }
    }
    if (leader) da_d[L.row * H + head] = dad;
  }
}

// ------------------------------------------------------------------------------------------
// backward, pass over source rows j (transpose CSR; tmap[q] = target-CSR position of entry q):
//   dXP_j[h] = sum_{j->i} alpha_ij mask_ij dZ_i[h] + (sum_i da_ij) att_src[h] + da_d[j,h] att_dst[h]
// plus per-block column partials: [0] datt_src = sum_j (sum_i da_ij) xp_j,
//                                 [1] datt_dst = sum_j da_d[j] xp_j,  [2] dbias = sum_j dZ_j.
// Persistent over rows (block b owns rows b*8 + hw + 8*P*t), fixed-order in-block combine.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_gat_bwd_node(
    const int32_t* __restrict__ tptr, const int32_t* __restrict__ tidx,
    const int32_t* __restrict__ tmap, const float* __restrict__ alpha,
    const float* __restrict__ mask, const float* __restrict__ da_e,
    const float* __restrict__ da_d, const float* __restrict__ dZ, const float* __restrict__ XP,
    const float* __restrict__ att_src, const float* __restrict__ att_dst, int64_t M, int H,
    int C, float* __restrict__ dXP, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float red[RB][3 * MAXS * 128];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, hw = wave * 2 + (lane >> 5);
  const int HC = H * C;
  f32x4 ps[MAXS], pd[MAXS], pb[MAXS];
#pragma unroll
  for (int q = 0; q < MAXS; ++q) ps[q] = pd[q] = pb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t row = (int64_t)blockIdx.x * RB + hw; row < M; row += (int64_t)gridDim.x * RB) {
    const int q0 = tptr[row], q1 = tptr[row + 1];
#pragma unroll
    for (int st = 0; st < MAXS; ++st) {
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
          const int qq = q + u < q1 ? q + u : q0;
          ti[u] = tidx[qq];
          pp[u] = tmap[qq];
        }
        f32x4 dv[EB];
        float al[EB], da[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          dv[u] = ld4(dZ + (int64_t)ti[u] * HC + fc);
          al[u] = alpha[(int64_t)pp[u] * H + head];
          if (mask) al[u] *= mask[(int64_t)pp[u] * H + head];
          da[u] = da_e[(int64_t)pp[u] * H + head];
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
        ps[st] += sda * xp;
        pd[st] += dd * xp;
        pb[st] += ld4(dZ + row * HC + f);
      }
    }
  }
#pragma unroll
  for (int st = 0; st < MAXS; ++st) {
    st4(&red[hw][(0 * MAXS + st) * 128 + 4 * li], ps[st]);
    st4(&red[hw][(1 * MAXS + st) * 128 + 4 * li], pd[st]);
    st4(&red[hw][(2 * MAXS + st) * 128 + 4 * li], pb[st]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * HC; i += NT) {
    const int kind = i / HC, f = i % HC;
    const int idx = (kind * MAXS + f / 128) * 128 + f % 128;
    float t = red[0][idx];
#pragma unroll
    for (int r = 1; r < RB; ++r) t += red[r][idx];
    part[(int64_t)blockIdx.x * 3 * HC + i] = t;
  }
}

inline bool shape_ok(int H, int C) {
  return H > 0 && C >= 4 && C <= 128 && (128 % C) == 0 && H * C <= MAXS * 128;
}

inline unsigned row_grid(int64_t M) { return (unsigned)((M + RB - 1) / RB); }

}  // namespace

extern "C" int lgnn_gat_att(const float* XP, int64_t M, int H, int C, const float* att_src,
                            const float* att_dst, float* a_s, float* a_d, void* stream) {
  if (M < 0 || !shape_ok(H, C) || !att_src || !att_dst || (M > 0 && (!XP || !a_s || !a_d)))
    return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  hipLaunchKernelGGL(k_gat_att, dim3(row_grid(M)), dim3(NT), 0, as_stream(stream), XP, M, H, C,
                     att_src, att_dst, a_s, a_d);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_gat_fwd(const int32_t* rowptr, const int32_t* col, const float* XP,
                            const float* a_s, const float* a_d, int64_t M, int H, int C,
                            float negative_slope, const float* edge_mask, const float* bias,
                            int act, float* alpha, float* Y, void* stream) {
  if (M < 0 || !shape_ok(H, C) || (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU))
    return LGNN_EINVAL;
  if (M > 0 && (!rowptr || !col || !XP || !a_s || !a_d || !Y)) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  if (act == LGNN_ACT_ELU)
    hipLaunchKernelGGL(k_gat_fwd<LGNN_ACT_ELU>, dim3(row_grid(M)), dim3(NT), 0, as_stream(stream),
                       rowptr, col, XP, a_s, a_d, M, H, C, negative_slope, edge_mask, bias, alpha,
                       Y);
  else
    hipLaunchKernelGGL(k_gat_fwd<LGNN_ACT_NONE>, dim3(row_grid(M)), dim3(NT), 0,
                       as_stream(stream), rowptr, col, XP, a_s, a_d, M, H, C, negative_slope,
                       edge_mask, bias, alpha, Y);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_gat_bwd_edge(const int32_t* rowptr, const int32_t* col, const float* XP,
                                 const float* a_s, const float* a_d, const float* alpha,
                                 const float* edge_mask, const float* dY, const float* Y,
                                 int act, int64_t M, int H, int C, float negative_slope,
                                 float* dZ, float* da_e, float* da_d, void* stream) {
  if (M < 0 || !shape_ok(H, C) || (act != LGNN_ACT_NONE && act != LGNN_ACT_ELU))
    return LGNN_EINVAL;
  if (M > 0 && (!rowptr || !col || !XP || !a_s || !a_d || !alpha || !dY || !dZ || !da_e || !da_d))
    return LGNN_EINVAL;
  if (act == LGNN_ACT_ELU && M > 0 && !Y) return LGNN_EINVAL;
  if (M == 0) return LGNN_OK;
  if (act == LGNN_ACT_ELU)
    hipLaunchKernelGGL(k_gat_bwd_edge<LGNN_ACT_ELU>, dim3(row_grid(M)), dim3(NT), 0,
                       as_stream(stream), rowptr, col, XP, a_s, a_d, alpha, edge_mask, dY, Y, M,
                       H, C, negative_slope, dZ, da_e, da_d);
  else
    hipLaunchKernelGGL(k_gat_bwd_edge<LGNN_ACT_NONE>, dim3(row_grid(M)), dim3(NT), 0,
                       as_stream(stream), rowptr, col, XP, a_s, a_d, alpha, edge_mask, dY, Y, M,
                       H, C, negative_slope, dZ, da_e, da_d);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

extern "C" int lgnn_gat_bwd_num_partials(int64_t M) {
  if (M < 0) return LGNN_EINVAL;
  const int64_t b = (M + RB - 1) / RB;
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

extern "C" int lgnn_gat_bwd_node(const int32_t* tptr, const int32_t* tidx, const int32_t* tmap,
                                 const float* alpha, const float* edge_mask, const float* da_e,
                                 const float* da_d, const float* dZ, const float* XP,
                                 const float* att_src, const float* att_dst, int64_t M, int H,
                                 int C, float* dXP, float* partials, int num_partials,
                                 void* stream) {
  if (M < 0 || !shape_ok(H, C) || !att_src || !att_dst || !partials) return LGNN_EINVAL;
  if (num_partials != lgnn_gat_bwd_num_partials(M)) return LGNN_EINVAL;
  if (M > 0 && (!tptr || !tidx || !tmap || !alpha || !da_e || !da_d || !dZ || !XP || !dXP))
    return LGNN_EINVAL;
  hipLaunchKernelGGL(k_gat_bwd_node, dim3(num_partials), dim3(NT), 0, as_stream(stream), tptr,
                     tidx, tmap, alpha, edge_mask, da_e, da_d, dZ, XP, att_src, att_dst, M, H, C,
                     dXP, partials);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}
