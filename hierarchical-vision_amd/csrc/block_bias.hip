// Every per-block small table of a SwinV2 W-MSA block in ONE launch forward and two backward
// (instead of two and three): the GEMM bias vectors (attn_bias.hip: qkv bias (q_bias, 0, 0),
// proj bias + W_proj v_bias; swinv2.py:218-220, 262) and the continuous relative-position
// bias table + logit scale (cpb.hip; swinv2.py:130-145, 230-247).  The grid is split by role;
// the bodies are the per-op kernels' (block_bias.h), so results are identical to them.
#include "block_bias.h"

namespace {

using hvk_bias::kAbRows;
using hvk_bias::kHid;
using hvk_bias::kRowsPerBlock;

struct BiasFwd {
  const float *qb, *vb, *pb, *pw;
  int C, nab;
  const float *coords, *w1, *b1, *w2, *logit;
  float clamp_max;
  int RR, nH;
  float *qkv_bias, *eff, *dv_zero, *table, *scale;
};

__global__ __launch_bounds__(256) void block_bias_fwd_kernel(BiasFwd a) {
  if ((int)blockIdx.x < a.nab)
    hvk_bias::attn_bias_fwd_body(blockIdx.x, a.nab, a.qb, a.vb, a.pb, a.pw, a.C, a.qkv_bias, a.eff, a.dv_zero);
  else
    hvk_bias::cpb_fwd_body(blockIdx.x - a.nab, a.coords, a.w1, a.b1, a.w2, a.logit, a.clamp_max, a.RR, a.nH,
                           a.table, a.scale);
}

struct BiasBwd {
  const float *g_eff, *vb, *pw;
  int C, nab;
  float *dpb, *dvb, *dpw;
  const float *coords, *w1, *b1, *w2, *table, *dtable;
  int RR, nH;
  float* part;
};

// stage 1: [0, nab) attention-bias gradients, then the CPB partials (512 threads each)
__global__ __launch_bounds__(kHid) void block_bias_bwd_kernel(BiasBwd a) {
  if ((int)blockIdx.x < a.nab)
    hvk_bias::attn_bias_bwd_body(blockIdx.x, a.g_eff, a.vb, a.pw, a.C, a.dpb, a.dvb, a.dpw);
  else
    hvk_bias::cpb_bwd_partial_body(blockIdx.x - a.nab, a.coords, a.w1, a.b1, a.w2, a.table, a.dtable, a.RR,
                                   a.nH, a.part);
}

__global__ __launch_bounds__(256) void block_bias_reduce_kernel(const float* __restrict__ part, int nblk, int nH,
                                                                const float* __restrict__ logit, float clamp_max,
                                                                const float* __restrict__ dscale,
                                                                float* __restrict__ dw1, float* __restrict__ db1,
                                                                float* __restrict__ dw2, float* __restrict__ dlogit) {
  hvk_bias::cpb_bwd_reduce_body(blockIdx.x, part, nblk, nH, logit, clamp_max, dscale, dw1, db1, dw2, dlogit);
}

}  // namespace

extern "C" {

int hvk_block_bias_fwd(const float* q_bias, const float* v_bias, const float* proj_bias, const float* proj_w,
                       int C, const float* coords, const float* w1, const float* b1, const float* w2,
                       const float* logit_scale, float clamp_max, int RR, int nH, int hidden, float* qkv_bias,
                       float* eff, float* dv_zero, float* table, float* scale, void* stream) {
  if (!v_bias || !proj_w || !qkv_bias || !eff || !coords || !w1 || !b1 || !w2 || !logit_scale || !table ||
      !scale || C <= 0)
    return hvk_set_error(HVK_EINVAL, "hvk_block_bias_fwd: null pointer or C=%d", C);
  if (hidden != kHid || nH <= 0 || nH > 32 || RR <= 0)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_block_bias_fwd: hidden=%d (512) nH=%d (<= 32) RR=%d", hidden,
                         nH, RR);
  BiasFwd a{q_bias, v_bias, proj_bias, proj_w, C, (C + 3) / 4, coords, w1, b1, w2, logit_scale, clamp_max,
            RR, nH, qkv_bias, eff, dv_zero, table, scale};
  const int ncpb = (nH * RR + 3) / 4;
  hipLaunchKernelGGL(block_bias_fwd_kernel, dim3(a.nab + ncpb), dim3(256), 0, static_cast<hipStream_t>(stream),
                     a);
  HVK_CHECK_LAUNCH("block_bias_fwd");
  return HVK_OK;
}

int hvk_block_bias_bwd(const float* g_eff, const float* v_bias, const float* proj_w, int C, float* d_proj_bias,
                       float* d_v_bias, float* d_proj_w, const float* coords, const float* w1, const float* b1,
                       const float* w2, const float* logit_scale, float clamp_max, int RR, int nH, int hidden,
                       const float* table, const float* dtable, const float* dscale, float* dw1, float* db1,
                       float* dw2, float* dlogit, float* workspace, size_t workspace_bytes, void* stream) {
  if (!v_bias || !proj_w || !coords || !w1 || !b1 || !w2 || !logit_scale || !table || !dtable || !dscale ||
      !dw1 || !db1 || !dw2 || !dlogit || !workspace || C <= 0)
    return hvk_set_error(HVK_EINVAL, "hvk_block_bias_bwd: null pointer or C=%d", C);
  if (g_eff && !d_v_bias)
    return hvk_set_error(HVK_EINVAL, "hvk_block_bias_bwd: null d v_bias");
  if (hidden != kHid || nH <= 0 || nH > 32 || RR <= 0)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_block_bias_bwd: hidden=%d (512) nH=%d (<= 32)", hidden, nH);
  const int nblk = (RR + kRowsPerBlock - 1) / kRowsPerBlock;
  if (workspace_bytes < (size_t)nblk * (nH + 3) * kHid * sizeof(float))
    return hvk_set_error(HVK_EINVAL, "hvk_block_bias_bwd: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  // no eff gradient (eff unused downstream): the CPB part only
  BiasBwd a{g_eff, v_bias, proj_w, C, g_eff ? (C + kAbRows - 1) / kAbRows : 0, d_proj_bias, d_v_bias, d_proj_w,
            coords, w1, b1, w2, table, dtable, RR, nH, workspace};
  hipLaunchKernelGGL(block_bias_bwd_kernel, dim3(a.nab + nblk), dim3(kHid), 0, st, a);
  HVK_CHECK_LAUNCH("block_bias_bwd");
  const int n = (nH + 3) * kHid;
  hipLaunchKernelGGL(block_bias_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, st, workspace, nblk, nH,
                     logit_scale, clamp_max, dscale, dw1, db1, dw2, dlogit);
  HVK_CHECK_LAUNCH("block_bias_reduce");
  return HVK_OK;
}

}  // extern "C"
