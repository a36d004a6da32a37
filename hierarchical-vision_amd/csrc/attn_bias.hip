// The two bias vectors of a W-MSA block's GEMMs, one launch each way (swinv2.py:218-220,
// 262): the reference adds cat(q_bias, 0, v_bias) in the qkv Linear and proj.bias in proj.
// Here the qkv GEMM gets (q_bias, 0, 0) (q_bias's gradient comes out of the W-MSA backward)
// and v_bias passes through attention unchanged (softmax rows sum to 1) into proj's bias:
//   eff = proj.bias + W_proj v_bias      (f32, [C])
// backward: d proj.bias = g, d v_bias = W_proj^T g, d W_proj = g v_bias^T (this term only;
// autograd adds the proj GEMM's own weight gradient).
#include "hvk_common.h"

namespace {

__global__ __launch_bounds__(256) void attn_bias_fwd_kernel(const float* __restrict__ qb,
                                                            const float* __restrict__ vb,
                                                            const float* __restrict__ pb,
                                                            const float* __restrict__ w, int C,
                                                            float* __restrict__ qkv_bias,
                                                            float* __restrict__ eff,
                                                            float* __restrict__ dv_zero) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < 3 * C; i += gridDim.x * 256) {
    qkv_bias[i] = (i < C && qb) ? qb[i] : 0.f;
    if (dv_zero && i < C) dv_zero[i] = 0.f;  // the backward's d v_bias accumulator
  }
  // one wave per output row n: lanes stride over k, wave reduction
  const int lane = threadIdx.x & 63;
  for (int n = blockIdx.x * 4 + (threadIdx.x >> 6); n < C; n += gridDim.x * 4) {
    float s = 0.f;
    for (int k = lane; k < C; k += 64) s = fmaf(w[(size_t)n * C + k], vb[k], s);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) eff[n] = (pb ? pb[n] : 0.f) + s;
  }
}

// 8 rows n of W per workgroup: d W[n, :] = g[n] v^T and the rows' share of d v = W^T g
// (column partial sums, one f32 atomic per column per workgroup into d v, which the
// forward launch zeroed)
constexpr int kRows = 8;
__global__ __launch_bounds__(256) void attn_bias_bwd_kernel(const float* __restrict__ g,
                                                            const float* __restrict__ vb,
                                                            const float* __restrict__ w, int C,
                                                            float* __restrict__ dpb,
                                                            float* __restrict__ dvb,
                                                            float* __restrict__ dw) {
  const int n0 = blockIdx.x * kRows;
  for (int k = threadIdx.x; k < C; k += 256) {
    const float vk = vb[k];
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int n = n0 + r;
      if (n < C) {
        const float gn = g[n];
        dw[(size_t)n * C + k] = gn * vk;
        acc = fmaf(w[(size_t)n * C + k], gn, acc);
      }
    }
    atomicAdd(dvb + k, acc);
  }
  if (dpb)
    for (int i = threadIdx.x; i < kRows && n0 + i < C; i += 256) dpb[n0 + i] = g[n0 + i];
}

}  // namespace

extern "C" {

int hvk_attn_bias_fwd(const float* q_bias, const float* v_bias, const float* proj_bias,
                      const float* proj_w, int C, float* qkv_bias, float* eff, float* dv_zero,
                      void* stream) {
  if (!v_bias || !proj_w || !qkv_bias || !eff || C <= 0)
    return hvk_set_error(HVK_EINVAL, "hvk_attn_bias_fwd: null pointer or C=%d", C);
  hipLaunchKernelGGL(attn_bias_fwd_kernel, dim3((C + 3) / 4), dim3(256), 0,
                     static_cast<hipStream_t>(stream), q_bias, v_bias, proj_bias, proj_w, C, qkv_bias,
                     eff, dv_zero);
  HVK_CHECK_LAUNCH("hvk_attn_bias_fwd");
  return HVK_OK;
}

int hvk_attn_bias_bwd(const float* g, const float* v_bias, const float* proj_w, int C,
                      float* d_proj_bias, float* d_v_bias, float* d_proj_w, void* stream) {
  if (!g || !v_bias || !proj_w || !d_v_bias || !d_proj_w || C <= 0)
    return hvk_set_error(HVK_EINVAL, "hvk_attn_bias_bwd: null pointer or C=%d", C);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(attn_bias_bwd_kernel, dim3((C + kRows - 1) / kRows), dim3(256), 0, st, g, v_bias,
                     proj_w, C, d_proj_bias, d_v_bias, d_proj_w);
  HVK_CHECK_LAUNCH("hvk_attn_bias_bwd");
  return HVK_OK;
}

}  // extern "C"
