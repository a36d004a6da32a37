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
// thread per patch: 4C row loads (neighbouring threads read neighbouring bytes of one image
// row) and 2C contiguous 16-B stores of its 32C-byte patch row; the bf16 rounding is
// round-to-nearest-even, as x.to(torch.bfloat16).
//   U8 = false: f32 images (already normalised), 16-B float4 row loads;
//   U8 = true: the uint8 [B, C, H, W] batch of pil_image_collate (data.py:36-76) with the
//   device-side NormalizationFn of data.py:130-136 fused in: (x - mean[c]) / std[c] in f32
//   (correctly rounded division, as torch's sub_ + div_), one 4-B row load per (c, py).
template <int C, bool U8>
__global__ __launch_bounds__(256) void patchify_kernel(const void* __restrict__ xv, uint4* __restrict__ out,
                                                       int B, int H, int W, const float* __restrict__ mean,
                                                       const float* __restrict__ std) {
  const int GH = H >> 2, GW = W >> 2, W4 = W >> 2;
  const long long total = (long long)B * GH * GW;
  float mu[C], sd[C];
  if constexpr (U8) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      mu[c] = mean[c];
      sd[c] = std[c];
    }
  }
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
        const long long rowq = (((long long)b * C + c) * H + 4 * gy + py) * W4 + gx;
        if constexpr (U8) {
          const uint32_t u = reinterpret_cast<const uint32_t*>(xv)[rowq];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[16 * c + 4 * py + j] = __fdiv_rn((float)((u >> (8 * j)) & 0xFFu) - mu[c], sd[c]);
        } else {
          const float4 f = reinterpret_cast<const float4*>(xv)[rowq];
          v[16 * c + 4 * py] = f.x; v[16 * c + 4 * py + 1] = f.y;
          v[16 * c + 4 * py + 2] = f.z; v[16 * c + 4 * py + 3] = f.w;
        }
      }
    uint4* o = out + p * (2 * C);
#pragma unroll
    for (int i = 0; i < 2 * C; ++i) o[i] = hvk_pack8(v + 8 * i);
  }
}

// composer NormalizationFn on its own (data.py:130-136 as the device transform, for callers
// that want the f32 images): out = (x - mean[c]) / std[c], x uint8 [B, C, HW]; 4 pixels per
// thread (one 4-B load, one 16-B store)
__global__ __launch_bounds__(256) void normalize_u8_kernel(const uint32_t* __restrict__ x, float4* __restrict__ out,
                                                           long long quads, int C, int hw4,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ std) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < quads;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)((i / hw4) % C);
    const float m = mean[c], s = std[c];
    const uint32_t u = x[i];
    out[i] = make_float4(__fdiv_rn((float)(u & 0xFFu) - m, s), __fdiv_rn((float)((u >> 8) & 0xFFu) - m, s),
                         __fdiv_rn((float)((u >> 16) & 0xFFu) - m, s), __fdiv_rn((float)(u >> 24) - m, s));
  }
}

}  // namespace

extern "C" {

static int patchify(const void* x, void* out, int B, int C, int H, int W, const float* mean, const float* std,
                    void* stream, const char* who) {
  if (!x || !out) return hvk_set_error(HVK_EINVAL, "%s: null pointer", who);
  if (B <= 0 || H <= 0 || W <= 0 || H % 4 || W % 4)
    return hvk_set_error(HVK_EINVAL, "%s: bad shape B=%d H=%d W=%d", who, B, H, W);
  if (C != 3) return hvk_set_error(HVK_EUNSUPPORTED, "%s: C=%d (built for 3)", who, C);
  const long long total = (long long)B * (H / 4) * (W / 4);
  long long grid = (total + 255) / 256;
  if (grid > 256 * 64) grid = 256 * 64;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (mean)
    hipLaunchKernelGGL((patchify_kernel<3, true>), dim3((unsigned)grid), dim3(256), 0, st, x,
                       static_cast<uint4*>(out), B, H, W, mean, std);
  else
    hipLaunchKernelGGL((patchify_kernel<3, false>), dim3((unsigned)grid), dim3(256), 0, st, x,
                       static_cast<uint4*>(out), B, H, W, nullptr, nullptr);
  HVK_CHECK_LAUNCH("patchify");
  return HVK_OK;
}

int hvk_patchify_bf16(const float* x, void* out, int B, int C, int H, int W, void* stream) {
  return patchify(x, out, B, C, H, W, nullptr, nullptr, stream, "hvk_patchify_bf16");
}

int hvk_patchify_u8_bf16(const uint8_t* x, void* out, const float* mean, const float* std, int B, int C, int H,
                         int W, void* stream) {
  if (!mean || !std) return hvk_set_error(HVK_EINVAL, "hvk_patchify_u8_bf16: null mean / std");
  return patchify(x, out, B, C, H, W, mean, std, stream, "hvk_patchify_u8_bf16");
}

int hvk_normalize_u8(const uint8_t* x, float* out, const float* mean, const float* std, int B, int C, int HW,
                     void* stream) {
  if (!x || !out || !mean || !std) return hvk_set_error(HVK_EINVAL, "hvk_normalize_u8: null pointer");
  if (B <= 0 || C <= 0 || HW <= 0 || HW % 4)
    return hvk_set_error(HVK_EINVAL, "hvk_normalize_u8: bad shape B=%d C=%d HW=%d", B, C, HW);
  const long long quads = (long long)B * C * HW / 4;
  long long grid = (quads + 255) / 256;
  if (grid > 256 * 64) grid = 256 * 64;
  hipLaunchKernelGGL(normalize_u8_kernel, dim3((unsigned)grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const uint32_t*>(x), reinterpret_cast<float4*>(out), quads, C, HW / 4,
                     mean, std);
  HVK_CHECK_LAUNCH("normalize_u8");
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
