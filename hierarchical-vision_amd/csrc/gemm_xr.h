// Persistent row-range GEMM (gemm_xr.hip): host entry used by the tiled-GEMM launchers.
#pragma once
#include <hip/hip_runtime.h>
// (also declares hvk_wide below)

typedef unsigned short hvk_bf16;

namespace hvk_xr {
struct Args {
  const hvk_bf16* X;
  const hvk_bf16* W;
  const float* bias;
  hvk_bf16* Y;
  hvk_bf16* Y2;
  int M, N, K;
  int NG, G, NT, ipw;  // granules, row groups, 384-column tiles, items per workgroup
};
// Y = X W^T (+ bias) (epi 0) or h = X W^T + bias, GELU(h) (epi 1) when a balanced plan exists;
// returns -1 (nothing launched) otherwise, else an HVK status.
int launch(int epi, const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2, int M,
           int N, int K, hipStream_t st);
bool plan(int M, int N, int K, Args& a, int& mg);
}  // namespace hvk_xr

// Whole-row 208 x 384 tile GEMM (gemm_wide.hip): epi 0 / 1 / 2 / 4 as the tiled kernels; returns -1
// (nothing launched) where it is not built, else an HVK status.
namespace hvk_wide {
bool supported(int M, int N, int K);
int launch(int epi, const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2, int M,
           int N, int K, hipStream_t st, float* rn, const float* qscale);
}  // namespace hvk_wide

// The 128 x 192 tile with the post-norm LayerNorm + residual of a C = 192 row in its epilogue
// (gemm_tile.hip EPI 5; N must be 192): a = X W^T stored, then x / xb / mean / rstd as
// ln_fwd_kernel<8, 32> computes them from a.  An HVK status.
struct LnEpi;
namespace hvk_tile_ln {
bool supported(int M, int N, int K);
int launch(const hvk_bf16* X, const hvk_bf16* W, hvk_bf16* Y, int M, int N, int K, const LnEpi& ln, hipStream_t st);
}  // namespace hvk_tile_ln
