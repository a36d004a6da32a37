// The two bias vectors of a W-MSA block's GEMMs, one launch each way (swinv2.py:218-220,
// 262): the reference adds cat(q_bias, 0, v_bias) in the qkv Linear and proj.bias in proj.
// Here the qkv GEMM gets (q_bias, 0, 0) (q_bias's gradient comes out of the W-MSA backward)
// and v_bias passes through attention unchanged (softmax rows sum to 1) into proj's bias:
//   eff = proj.bias + W_proj v_bias      (f32, [C])
// backward: d proj.bias = g, d v_bias = W_proj^T g, d W_proj = g v_bias^T (this term only;
// autograd adds the proj GEMM's own weight gradient).
#include "block_bias.h"

namespace {

__global__ __launch_bounds__(256) void attn_bias_fwd_kernel(const float* __restrict__ qb, const float* __restrict__ vb,
                                                            const float* __restrict__ pb, const float* __restrict__ w,
                                                            int C, float* __restrict__ qkv_bias, float* __restrict__ eff,
                                                            float* __restrict__ dv_zero) {
  hvk_bias::attn_bias_fwd_body(blockIdx.x, gridDim.x, qb, vb, pb, w, C, qkv_bias, eff, dv_zero);
}

constexpr int kRows = hvk_bias::kAbRows;
__global__ __launch_bounds__(256) void attn_bias_bwd_kernel(const float* __restrict__ g, const float* __restrict__ vb,
                                                            const float* __restrict__ w, int C, float* __restrict__ dpb,
                                                            float* __restrict__ dvb, float* __restrict__ dw) {
  hvk_bias::attn_bias_bwd_body(blockIdx.x, g, vb, w, C, dpb, dvb, dw);
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
