// PatchMerging 2x2 strided gather (gfx950): swinv2.py:484-491, and the PatchEmbed patchify
// + bf16 cast (below)
//   x0 = x[:, 0::2, 0::2]; x1 = x[:, 1::2, 0::2]; x2 = x[:, 0::2, 1::2]; x3 = x[:, 1::2, 1::2]
//   cat([x0, x1, x2, x3], -1)
// Each merged token's 4C output row is assembled from four C-wide source rows; one
// 16-byte chunk per lane, so both the reads (contiguous C-wide rows) and the writes
// (contiguous 4C-wide rows) are coalesced.  The backward is the inverse permutation.
#include "hvk_common.h"

namespace {

template <bool kScatter>
__global__ __launch_bounds__(256) void merge_kernel(const uint4* __restrict__ src,
                                                    uint4* __restrict__ dst, int B, int H, int W,
                                                    int C8) {
  // one thread per 16-byte chunk of the merged tensor [B, H/2*W/2, 4*C]
  const int Ho = H >> 1, Wo = W >> 1;
  const long long total = (long long)B * Ho * Wo * 4 * C8;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C8);
    long long t = e / C8;
    const int k = (int)(t & 3);
    t >>= 2;
    const int j = (int)(t % Wo);
    t /= Wo;
    const int i = (int)(t % Ho);
    const int b = (int)(t / Ho);
    const int hs = 2 * i + (k & 1), ws = 2 * j + (k >> 1);
    const long long s = ((long long)(b * H + hs) * W + ws) * C8 + c;
    if (kScatter) dst[s] = src[e];
    else dst[e] = src[s];
  }
}

int launch(bool scatter, const void* in, void* out, int B, int H, int W, int C, void* stream) {
  if (!in || !out) return hvk_set_error(HVK_EINVAL, "patch_merge: null pointer");
  if (B <= 0 || H <= 0 || W <= 0 || H % 2 || W % 2)
    return hvk_set_error(HVK_EINVAL, "patch_merge: bad shape B=%d H=%d W=%d", B, H, W);
  if (C % 8) return hvk_set_error(HVK_EUNSUPPORTED, "patch_merge: C=%d not a multiple of 8", C);
  const long long total = (long long)B * H * W * C / 8;
  long long grid = (total + 255) / 256;
  if (grid > 256 * 64) grid = 256 * 64;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (scatter)
    hipLaunchKernelGGL(merge_kernel<true>, dim3((unsigned)grid), dim3(256), 0, st,
                       static_cast<const uint4*>(in), static_cast<uint4*>(out), B, H, W, C / 8);
  else
    hipLaunchKernelGGL(merge_kernel<false>, dim3((unsigned)grid), dim3(256), 0, st,
                       static_cast<const uint4*>(in), static_cast<uint4*>(out), B, H, W, C / 8);
  HVK_CHECK_LAUNCH("patch_merge");
  return HVK_OK;
}

// PatchEmbed input (swinv2.py:652-660): the 4x4/s4 Conv2d as a GEMM wants token-major
// patches [B, (H/4)(W/4), C*16] in the conv weight's (c, py, px) order, in bf16.  One
// thread per patch: 4C float4 row loads (neighbouring threads read neighbouring 16 B of one
// image row) and 2C contiguous 16-B stores of its 32C-byte patch row; the bf16 rounding is
// round-to-nearest-even, as x.to(torch.bfloat16).
template <int C>
__global__ __launch_bounds__(256) void patchify_kernel(const float4* __restrict__ x, uint4* __restrict__ out,
                                                       int B, int H, int W) {
  const int GH = H >> 2, GW = W >> 2, W4 = W >> 2;
  const long long total = (long long)B * GH * GW;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < total;
       p += (long long)gridDim.x * blockDim.x) {
    const int gx = (int)(p % GW);
    const long long t = p / GW;
    const int gy = (int)(t % GH);
    const int b = (int)(t / GH);
    float v[C * 16];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int py = 0; py < 4; ++py) {
        const float4 f = x[(((long long)b * C + c) * H + 4 * gy + py) * W4 + gx];
        v[16 * c + 4 * py] = f.x; v[16 * c + 4 * py + 1] = f.y;
        v[16 * c + 4 * py + 2] = f.z; v[16 * c + 4 * py + 3] = f.w;
      }
    uint4* o = out + p * (2 * C);
#pragma unroll
    for (int i = 0; i < 2 * C; ++i) o[i] = hvk_pack8(v + 8 * i);
  }
}

}  // namespace

extern "C" {

int hvk_patchify_bf16(const float* x, void* out, int B, int C, int H, int W, void* stream) {
  if (!x || !out) return hvk_set_error(HVK_EINVAL, "hvk_patchify_bf16: null pointer");
  if (B <= 0 || H <= 0 || W <= 0 || H % 4 || W % 4)
    return hvk_set_error(HVK_EINVAL, "hvk_patchify_bf16: bad shape B=%d H=%d W=%d", B, H, W);
  if (C != 3) return hvk_set_error(HVK_EUNSUPPORTED, "hvk_patchify_bf16: C=%d (built for 3)", C);
  const long long total = (long long)B * (H / 4) * (W / 4);
  long long grid = (total + 255) / 256;
  if (grid > 256 * 64) grid = 256 * 64;
  hipLaunchKernelGGL(patchify_kernel<3>, dim3((unsigned)grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const float4*>(x), static_cast<uint4*>(out), B, H, W);
  HVK_CHECK_LAUNCH("patchify");
  return HVK_OK;
}


int hvk_patch_merge_gather(const void* x, void* out, int B, int H, int W, int C, void* stream) {
  return launch(false, x, out, B, H, W, C, stream);
}

int hvk_patch_merge_scatter(const void* gout, void* gx, int B, int H, int W, int C,
                            void* stream) {
  return launch(true, gout, gx, B, H, W, C, stream);
}

}  // extern "C"
