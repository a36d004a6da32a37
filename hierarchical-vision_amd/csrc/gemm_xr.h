// Persistent row-range GEMM (gemm_xr.hip): host entry used by the tiled-GEMM launchers.
#pragma once
#include <hip/hip_runtime.h>

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
