// Continuous relative-position bias (CPB) table and logit scale of one SwinV2 block
// (swinv2.py:130-145, 230-247), fused on gfx950:
//   table[h, r] = 16 * sigmoid( sum_j W2[h, j] * relu(W1[j, :] . coords[r, :] + b1[j]) )
//   scale[h]    = exp(min(logit_scale[h], clamp_max))
// coords = relative_coords_table [(2w-1)^2, 2] (log-spaced, swinv2.py:147-164), hidden 512.
// The reference runs this as ~10 eager ops per block per forward (two Linear, ReLU, sigmoid,
// scale, permute, clamp, exp) and ~15 in the backward; here it is one launch forward and two
// backward (partials, then their reduction).  Computed in f32 (the reference's autocast runs
// the two Linears in bf16; f32 is the tighter of the two, parity-tested).
#include "hvk_common.h"

namespace {

constexpr int kHid = 512;  // cpb_mlp hidden width (swinv2.py:141)
constexpr int kRowsPerBlock = 8;  // 22 workgroups for the (2w-1)^2 = 169 rows of w7

// one wave per (h, r) output: lane l owns hidden units l, l+64, ... (8 of 512), the dot
// product is a wave reduction; the hidden layer is recomputed per head (<= 32 heads, tiny)
__global__ __launch_bounds__(256) void cpb_fwd_kernel(const float* __restrict__ coords,
                                                      const float* __restrict__ w1,
                                                      const float* __restrict__ b1,
                                                      const float* __restrict__ w2,
                                                      const float* __restrict__ logit,
                                                      float clamp_max, int RR, int nH,
                                                      float* __restrict__ table,
                                                      float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int out = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x < nH)
    scale[threadIdx.x] = __expf(fminf(logit[threadIdx.x], clamp_max));
  if (out >= nH * RR) return;
  const int h = out / RR, r = out % RR;
  const float c0 = coords[2 * r], c1 = coords[2 * r + 1];
  const float* w2h = w2 + (size_t)h * kHid;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < kHid / 64; ++k) {
    const int jj = lane + 64 * k;
    const float a = fmaxf(fmaf(w1[2 * jj], c0, fmaf(w1[2 * jj + 1], c1, b1[jj])), 0.f);
    acc = fmaf(w2h[jj], a, acc);
  }
  acc = hvk_wave_sum(acc);
  if (lane == 0) table[(size_t)h * RR + r] = 16.f / (1.f + __expf(-acc));
}

// backward, stage 1: a block = 16 rows r, thread j = hidden unit.  d_pre from the forward
// table (16 s, s = sigmoid: d table / d pre = table * (1 - table / 16)); per thread the
// partial dW2[:, j], dW1[j, :], db1[j] over its rows -> part[blk][nH + 3][512]
__global__ __launch_bounds__(kHid) void cpb_bwd_partial_kernel(
    const float* __restrict__ coords, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ table, const float* __restrict__ dtable,
    int RR, int nH, float* __restrict__ part) {
  __shared__ float dpre[kRowsPerBlock][32];
  const int j = threadIdx.x;
  const int r0 = blockIdx.x * kRowsPerBlock;
  for (int e = j; e < kRowsPerBlock * nH; e += kHid) {
    const int rr = e / nH, h = e % nH, r = r0 + rr;
    float v = 0.f;
    if (r < RR) {
      const float t = table[(size_t)h * RR + r];
      v = dtable[(size_t)h * RR + r] * t * (1.f - t * (1.f / 16.f));
    }
    dpre[rr][h] = v;
  }
  __syncthreads();
  const float w10 = w1[2 * j], w11 = w1[2 * j + 1], bj = b1[j];
  float dw2[32], w2j[32];  // this hidden unit's W2 column, loaded once (all loads in flight)
#pragma unroll
  for (int h = 0; h < 32; ++h) {
    dw2[h] = 0.f;
    w2j[h] = h < nH ? w2[(size_t)h * kHid + j] : 0.f;
  }
  float dw10 = 0.f, dw11 = 0.f, db = 0.f;
  for (int rr = 0; rr < kRowsPerBlock; ++rr) {
    const int r = r0 + rr;
    if (r >= RR) break;
    const float c0 = coords[2 * r], c1 = coords[2 * r + 1];
    const float hid = fmaf(w10, c0, fmaf(w11, c1, bj));
    const float a = fmaxf(hid, 0.f);
    float dh = 0.f;
#pragma unroll
    for (int h = 0; h < 32; ++h) {
      if (h < nH) {
        const float d = dpre[rr][h];
        dw2[h] = fmaf(d, a, dw2[h]);
        dh = fmaf(d, w2j[h], dh);
      }
    }
    dh = hid > 0.f ? dh : 0.f;
    dw10 = fmaf(dh, c0, dw10);
    dw11 = fmaf(dh, c1, dw11);
    db += dh;
  }
  float* p = part + (size_t)blockIdx.x * (nH + 3) * kHid;
#pragma unroll
  for (int h = 0; h < 32; ++h)
    if (h < nH) p[(size_t)h * kHid + j] = dw2[h];
  p[(size_t)nH * kHid + j] = dw10;
  p[(size_t)(nH + 1) * kHid + j] = dw11;
  p[(size_t)(nH + 2) * kHid + j] = db;
}

// backward, stage 2: sum the partials; write dW2 [nH, 512], dW1 [512, 2], db1 [512], and
// d logit_scale = d scale * scale * [logit < clamp_max]
__global__ __launch_bounds__(256) void cpb_bwd_reduce_kernel(
    const float* __restrict__ part, int nblk, int nH, const float* __restrict__ logit,
    float clamp_max, const float* __restrict__ dscale, float* __restrict__ dw1,
    float* __restrict__ db1, float* __restrict__ dw2, float* __restrict__ dlogit) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < nH && dlogit) {
    const float l = logit[idx];
    dlogit[idx] = l <= clamp_max ? dscale[idx] * __expf(l) : 0.f;  // clamp passes x == max
  }
  const int n = (nH + 3) * kHid;
  if (idx >= n) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = 0;
  for (; b + 3 < nblk; b += 4) {
    s0 += part[(size_t)b * n + idx];
    s1 += part[(size_t)(b + 1) * n + idx];
    s2 += part[(size_t)(b + 2) * n + idx];
    s3 += part[(size_t)(b + 3) * n + idx];
  }
  for (; b < nblk; ++b) s0 += part[(size_t)b * n + idx];
  const float v = (s0 + s1) + (s2 + s3);
  const int row = idx / kHid, j = idx % kHid;
  if (row < nH) dw2[(size_t)row * kHid + j] = v;
  else if (row == nH) dw1[2 * j] = v;
  else if (row == nH + 1) dw1[2 * j + 1] = v;
  else db1[j] = v;
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
