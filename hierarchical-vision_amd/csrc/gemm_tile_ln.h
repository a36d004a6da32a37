// The 128 x 192 tile with the post-norm LayerNorm + residual of a C = 192 row in its epilogue
// (gemm_tile.hip EPI 5; N must be 192): a = X W^T stored, then x / xb / mean / rstd as
// ln_fwd_kernel<8, 32> computes them from a.  An HVK status.  (gemm.hip routes hvk_linear_ln_fwd
// here for C = 192.)
#pragma once
#include <hip/hip_runtime.h>

typedef unsigned short hvk_bf16;

struct LnEpi;
namespace hvk_tile_ln {
bool supported(int M, int N, int K);
int launch(const hvk_bf16* X, const hvk_bf16* W, hvk_bf16* Y, int M, int N, int K, const LnEpi& ln, hipStream_t st);
}  // namespace hvk_tile_ln
