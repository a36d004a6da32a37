// PatchMerging 2x2 strided gather (gfx950): swinv2.py:484-491
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

}  // namespace

extern "C" {

int hvk_patch_merge_gather(const void* x, void* out, int B, int H, int W, int C, void* stream) {
  return launch(false, x, out, B, H, W, C, stream);
}

int hvk_patch_merge_scatter(const void* gout, void* gx, int B, int H, int W, int C,
                            void* stream) {
  return launch(true, gout, gx, B, H, W, C, stream);
}

}  // extern "C"
