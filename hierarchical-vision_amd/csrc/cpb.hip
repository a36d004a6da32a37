// Continuous relative-position bias (CPB) table and logit scale of one SwinV2 block
// (swinv2.py:130-145, 230-247), fused on gfx950:
//   table[h, r] = 16 * sigmoid( sum_j W2[h, j] * relu(W1[j, :] . coords[r, :] + b1[j]) )
//   scale[h]    = exp(min(logit_scale[h], clamp_max))
// coords = relative_coords_table [(2w-1)^2, 2] (log-spaced, swinv2.py:147-164), hidden 512.
// The reference runs this as ~10 eager ops per block per forward (two Linear, ReLU, sigmoid,
// scale, permute, clamp, exp) and ~15 in the backward; here it is one launch forward and two
// backward (partials, then their reduction).  Computed in f32 (the reference's autocast runs
// the two Linears in bf16; f32 is the tighter of the two, parity-tested).
#include "block_bias.h"

namespace {

using hvk_bias::kHid;
using hvk_bias::kRowsPerBlock;

__global__ __launch_bounds__(256) void cpb_fwd_kernel(const float* __restrict__ coords, const float* __restrict__ w1,
                                                      const float* __restrict__ b1, const float* __restrict__ w2,
                                                      const float* __restrict__ logit, float clamp_max, int RR,
                                                      int nH, float* __restrict__ table, float* __restrict__ scale) {
  hvk_bias::cpb_fwd_body(blockIdx.x, coords, w1, b1, w2, logit, clamp_max, RR, nH, table, scale);
}

__global__ __launch_bounds__(kHid) void cpb_bwd_partial_kernel(
    const float* __restrict__ coords, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ table, const float* __restrict__ dtable,
    int RR, int nH, float* __restrict__ part) {
  hvk_bias::cpb_bwd_partial_body(blockIdx.x, coords, w1, b1, w2, table, dtable, RR, nH, part);
}

__global__ __launch_bounds__(256) void cpb_bwd_reduce_kernel(
    const float* __restrict__ part, int nblk, int nH, const float* __restrict__ logit,
    float clamp_max, const float* __restrict__ dscale, float* __restrict__ dw1,
    float* __restrict__ db1, float* __restrict__ dw2, float* __restrict__ dlogit) {
  hvk_bias::cpb_bwd_reduce_body(blockIdx.x, part, nblk, nH, logit, clamp_max, dscale, dw1, db1, dw2, dlogit);
}

}  // namespace

extern "C" {

int hvk_cpb_fwd(const float* coords, const float* w1, const float* b1, const float* w2,
                const float* logit_scale, float clamp_max, int RR, int nH, int hidden,
                float* table, float* scale, void* stream) {
  if (!coords || !w1 || !b1 || !w2 || !logit_scale || !table || !scale)
    return hvk_set_error(HVK_EINVAL, "hvk_cpb_fwd: null pointer");
  if (hidden != kHid || nH <= 0 || nH > 32 || RR <= 0)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_cpb_fwd: hidden=%d (512) nH=%d (<= 32) RR=%d",
                         hidden, nH, RR);
  const int n = nH * RR;  // outputs, one wave each
  hipLaunchKernelGGL(cpb_fwd_kernel, dim3((n + 3) / 4), dim3(256), 0,
                     static_cast<hipStream_t>(stream), coords, w1, b1, w2, logit_scale, clamp_max,
                     RR, nH, table, scale);
  HVK_CHECK_LAUNCH("cpb_fwd");
  return HVK_OK;
}

size_t hvk_cpb_bwd_workspace_bytes(int RR, int nH) {
  const size_t nblk = (RR + kRowsPerBlock - 1) / kRowsPerBlock;
  return nblk * (size_t)(nH + 3) * kHid * sizeof(float);
}

int hvk_cpb_bwd(const float* coords, const float* w1, const float* b1, const float* w2,
                const float* logit_scale, float clamp_max, int RR, int nH, int hidden,
                const float* table, const float* dtable, const float* dscale, float* dw1,
                float* db1, float* dw2, float* dlogit, float* workspace, size_t workspace_bytes,
                void* stream) {
  if (!coords || !w1 || !b1 || !w2 || !logit_scale || !table || !dtable || !dscale || !dw1 ||
      !db1 || !dw2 || !dlogit || !workspace)
    return hvk_set_error(HVK_EINVAL, "hvk_cpb_bwd: null pointer");
  if (hidden != kHid || nH <= 0 || nH > 32 || RR <= 0)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_cpb_bwd: hidden=%d (512) nH=%d (<= 32)", hidden, nH);
  if (workspace_bytes < hvk_cpb_bwd_workspace_bytes(RR, nH))
    return hvk_set_error(HVK_EINVAL, "hvk_cpb_bwd: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nblk = (RR + kRowsPerBlock - 1) / kRowsPerBlock;
  hipLaunchKernelGGL(cpb_bwd_partial_kernel, dim3(nblk), dim3(kHid), 0, st, coords, w1, b1, w2,
                     table, dtable, RR, nH, workspace);
  HVK_CHECK_LAUNCH("cpb_bwd_partial");
  const int n = (nH + 3) * kHid;
  hipLaunchKernelGGL(cpb_bwd_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, st, workspace,
                     nblk, nH, logit_scale, clamp_max, dscale, dw1, db1, dw2, dlogit);
  HVK_CHECK_LAUNCH("cpb_bwd_reduce");
  return HVK_OK;
}

}  // extern "C"
