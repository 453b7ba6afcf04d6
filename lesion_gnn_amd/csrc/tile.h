// Internal interface between the C-ABI dispatch (node.hip) and the fast-path tile kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

bool lgnn_tile_fits(int64_t M, int K, int N);
int lgnn_tile_partials(int64_t M);
hipError_t lgnn_tile_fwd(hipStream_t s, const float* X, int64_t M, int K, const int32_t* rowptr,
                         const int32_t* col, const float* w, float self_scale, const float* W,
                         const float* b, int N, int act, float* Y, float* S_out,
                         const int32_t* tile_mask, int want);
hipError_t lgnn_tile_bwd(hipStream_t s, int grad_mode, const float* dY, const int64_t* batch,
                         const int32_t* gptr, int pool_mean, const int32_t* tptr,
                         const int32_t* tidx, const float* tw, float tself, const float* H,
                         int act, const float* X, int64_t M, int K, const float* W, int N,
                         float* dXpre, float* dWp, float* dbp, int P, const int32_t* tile_mask,
                         int want, int accumulate);
