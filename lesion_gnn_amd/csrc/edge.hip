// Gaussian edge weights of lesion graphs: lesion_gnn.transforms.GaussianDistance
// (reference src/lesion_gnn/transforms.py:32-79; its known-answer tests are
// test/test_transforms.py:8-77). For edge e = (row_e, col_e):
//   w_e = exp(-|pos[row_e] - pos[col_e]|^2 / (2 sigma^2)) / sqrt(2 pi sigma^2)
// in the precision of `pos` (fp32 or fp64, as torch evaluates the reference's expression on a
// tensor of that dtype), then cast to the output dtype (GaussianDistance(dtype=...), :44).
//
// Squared distances are summed over the coordinates in index order with explicit
// round-to-nearest operations (no FMA contraction), like (pos[row] - pos[col]).pow(2).sum(-1);
// the scale constants are rounded to the pos dtype first, as torch rounds a Python scalar
// operand to the tensor's dtype.
//
// HBM-bound gather: per edge 16 B of indices + 2 * dims * sizeof(pos) of (L2-resident) positions
// in, 4 or 8 B out. One thread per edge, grid-stride; edge_index rows are read coalesced.
#include "common.h"

namespace {

// Each operation rounds on its own, as torch's CPU ops do. HIP's __fmul_rn / __dadd_rn are
// plain operators carrying the `contract` flag of the header they come from, so under the
// default -ffp-contract=fast a product feeding a sum still fuses into an FMA (an ulp of the
// squared distance is |arg| ulps of the weight: up to ~350 at sigma = 0.05). Plain operators in
// a contract(off) scope carry no flag and stay separate instructions.
template <typename T>
struct Ops {
  static __device__ __forceinline__ T sub(T a, T b) {
#pragma clang fp contract(off)
    return a - b;
  }
  static __device__ __forceinline__ T mul(T a, T b) {
#pragma clang fp contract(off)
    return a * b;
  }
  static __device__ __forceinline__ T add(T a, T b) {
#pragma clang fp contract(off)
    return a + b;
  }
  static __device__ __forceinline__ T div(T a, T b) {
#pragma clang fp contract(off)
    return a / b;  // IEEE division (div_scale / div_fmas / div_fixup), correctly rounded
  }
  // fp32: exp evaluated in fp64 and rounded once — the correctly rounded fp32 exp (double
  // rounding needs a tie within 2^-29 relative), graceful in the subnormal band (exp(x) for
  // x in [-103.9, -87.3] is subnormal in fp32 and feeds the division by the norm constant,
  // which can bring it back into the normal range). torch's CPU expf is a <= 1-ulp
  // approximation of the same value, so the two agree to within 2 ulp after the division in
  // the normal range (tests/test_gpu_edge.py); in the subnormal band the CPU result itself
  // depends on the host ISA (some vectorised expf flush it), so the test bounds it absolutely.
  static __device__ __forceinline__ T ex(T a) { return (T)exp((double)a); }
};

template <typename T, typename O>
__global__ __launch_bounds__(256) void k_gauss(const T* __restrict__ pos, int64_t n, int dims,
                                               const int64_t* __restrict__ ei, int64_t E,
                                               T two_s2, T norm, O* __restrict__ out,
                                               int32_t* __restrict__ err) {
  using X = Ops<T>;
  int bad = 0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = ei[e], c = ei[E + e];
    if (r < 0 || r >= n || c < 0 || c >= n) {
      out[e] = O(0);
      ++bad;
      continue;
    }
    const T* a = pos + r * dims;
    const T* b = pos + c * dims;
    T s = T(0);
    for (int d = 0; d < dims; ++d) {
      const T df = X::sub(a[d], b[d]);
      s = d == 0 ? X::mul(df, df) : X::add(s, X::mul(df, df));
    }
    out[e] = O(X::div(X::ex(X::div(-s, two_s2)), norm));
  }
  if (bad) atomicAdd(err, bad);
}

template <typename T>
int launch(const T* pos, int64_t n, int dims, const int64_t* ei, int64_t E, double sigma,
           void* out, int out_f64, int32_t* err, hipStream_t s) {
  // The two constants are rounded exactly as Python evaluates the reference's expressions in
  // double and torch then rounds the scalar operand to T: `2 * self.sigma**2` (:57) is
  // 2 * (sigma * sigma), and `math.sqrt(2 * math.pi * sigma**2)` (:45) is
  // sqrt((2 * pi) * (sigma * sigma)). A different association moves the constant by an ulp,
  // which the exponent turns into |arg| ulps of the result (up to ~350 at sigma = 0.05).
  const double s2 = sigma * sigma;
  const T two_s2 = T(2.0 * s2);
  const T norm = T(std::sqrt((2.0 * M_PI) * s2));
  const int64_t want = (E + 255) / 256;
  const int grid = (int)(want < 8192 ? want : 8192);
  if (out_f64)
    k_gauss<T, double><<<grid, 256, 0, s>>>(pos, n, dims, ei, E, two_s2, norm,
                                            static_cast<double*>(out), err);
  else
    k_gauss<T, float><<<grid, 256, 0, s>>>(pos, n, dims, ei, E, two_s2, norm,
                                           static_cast<float*>(out), err);
  LGNN_LAUNCH_CHECK();
  return LGNN_OK;
}

}  // namespace

extern "C" int lgnn_gaussian_distance(const void* pos, int pos_f64, int64_t num_nodes, int dims,
                                      const int64_t* edge_index, int64_t num_edges, double sigma,
                                      void* out, int out_f64, int32_t* err, void* stream) {
  if (num_edges < 0 || num_nodes < 0 || dims < 1 || dims > 16 || !(sigma > 0.0) || !err)
    return LGNN_EINVAL;
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(err, 0, sizeof(int32_t), s) != hipSuccess) return LGNN_EINVAL;
  if (num_edges == 0) return LGNN_OK;
  if (!pos || !edge_index || !out) return LGNN_EINVAL;
  return pos_f64 ? launch(static_cast<const double*>(pos), num_nodes, dims, edge_index,
                          num_edges, sigma, out, out_f64, err, s)
                 : launch(static_cast<const float*>(pos), num_nodes, dims, edge_index, num_edges,
                          sigma, out, out_f64, err, s);
}
