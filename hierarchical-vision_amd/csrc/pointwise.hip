// Fused bias + exact GELU of the SwinV2 MLP (swinv2.py:60-62: fc1 -> GELU) on gfx950.
//
// fc1 runs as a plain GEMM without its bias; this kernel applies `u = h + b`,
// `y = 0.5 u (1 + erf(u / sqrt 2))` and writes bf16.  The backward recomputes u from the
// saved GEMM output and, in the same pass, column-sums the pre-activation gradient --
// that sum is the fc1 bias gradient, so no separate reduction reads it again.
//
// Layout: a wave owns 64 consecutive 8-channel chunks (512 channels) of a row tile and
// walks rows; each lane keeps its 8 column sums in registers.
#include "hvk_common.h"

namespace {

constexpr int kWaves = 4;


__global__ __launch_bounds__(64 * kWaves) void bias_gelu_fwd_kernel(const hvk_bf16* __restrict__ h,
                                                                    const float* __restrict__ b,
                                                                    hvk_bf16* __restrict__ y,
                                                                    int rows, int N) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = (blockIdx.y * 64 + lane) * 8;
  if (c >= N) return;
  float bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bb[j] = b ? b[c + j] : 0.f;
  for (int r = blockIdx.x * kWaves + wave; r < rows; r += gridDim.x * kWaves) {
    const size_t off = (size_t)r * N + c;
    float f[8];
    hvk_unpack8(*reinterpret_cast<const uint4*>(h + off), f);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const hvk_gelu::f32x2 v = hvk_gelu::gelu2(hvk_gelu::f32x2{f[j] + bb[j], f[j + 1] + bb[j + 1]});
      f[j] = v.x;
      f[j + 1] = v.y;
    }
    *reinterpret_cast<uint4*>(y + off) = hvk_pack8(f);
  }
}

__global__ __launch_bounds__(64 * kWaves) void bias_gelu_bwd_kernel(const hvk_bf16* __restrict__ h,
                                                                    const float* __restrict__ b,
                                                                    const hvk_bf16* __restrict__ gy,
                                                                    hvk_bf16* __restrict__ gh,
                                                                    float* __restrict__ part,
                                                                    float* __restrict__ dbias,
                                                                    int rows, int N) {
  __shared__ float red[kWaves][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // dbias is accumulated by the colsum kernel that follows in the stream: zero it here
  if (dbias && blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = threadIdx.x; i < N; i += blockDim.x) dbias[i] = 0.f;
  const int c = (blockIdx.y * 64 + lane) * 8;
  const bool act = c < N;
  float bb[8], acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bb[j] = (act && b) ? b[c + j] : 0.f; acc[j] = 0.f; }
  if (act) {
    for (int r = blockIdx.x * kWaves + wave; r < rows; r += gridDim.x * kWaves) {
      const size_t off = (size_t)r * N + c;
      float u[8], g[8];
      hvk_unpack8(*reinterpret_cast<const uint4*>(h + off), u);
      hvk_unpack8(*reinterpret_cast<const uint4*>(gy + off), g);
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const hvk_gelu::f32x2 d = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{u[j] + bb[j], u[j + 1] + bb[j + 1]});
        g[j] *= d.x;
        g[j + 1] *= d.y;
        acc[j] += g[j];
        acc[j + 1] += g[j + 1];
      }
      *reinterpret_cast<uint4*>(gh + off) = hvk_pack8(g);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += blockDim.x) {
    const int cc = blockIdx.y * 512 + i;
    if (cc < N) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) s += red[w][i];
      part[(size_t)blockIdx.x * N + cc] = s;
    }
  }
}

__global__ __launch_bounds__(64) void colsum_rows_kernel(const float* part, int nblk, int N,
                                                         float* out) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= N) return;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int b = blockIdx.y;
  const int G = gridDim.y;
  for (; b + 7 * G < nblk; b += 8 * G)
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += part[(size_t)(b + u * G) * N + c];
  for (; b < nblk; b += G) s[0] += part[(size_t)b * N + c];
  atomicAdd(out + c, ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7])));
}

constexpr int kBwdRowBlocks = 512;

}  // namespace

namespace {

// q / k head normalisation of a qkv tensor in place (hvk_qk_normalize): a wave owns 16 rows x one
// head (lane = row li, 8-channel chunk g), the layout of the fused GEMM epilogues, so the sums
// of squares reduce in the same order and the results are bit-identical to theirs
__global__ __launch_bounds__(256) void qk_normalize_kernel(hvk_bf16* __restrict__ qkv, float* __restrict__ rn,
                                                           const float* __restrict__ qscale, int T, int C) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int heads2 = 2 * C / 32;
  const long long item = (long long)blockIdx.x * 4 + wave;  // (16-row tile, head)
  const int hd = (int)(item % heads2);
  const long long row = (item / heads2) * 16 + li;
  if (item / heads2 * 16 >= T) return;
  const bool ok = row < T;
  const size_t off = (size_t)(ok ? row : 0) * 3 * C + hd * 32 + 8 * g;
  uint4 v = *reinterpret_cast<const uint4*>(qkv + off);
  float r;
  const float post = (qscale && hd < C / 32) ? qscale[hd] * HVK_LOG2E : 1.f;  // q: q^ * scale * log2e
  v = hvk_head_normalize8(v, r, post);  // all 64 lanes take part in the group sums
  if (ok) {
    *reinterpret_cast<uint4*>(qkv + off) = v;
    if (g == 0) rn[(size_t)row * heads2 + hd] = r;
  }
}

}  // namespace

extern "C" {

int hvk_qk_normalize(void* qkv, float* rn, const float* qscale, int T, int C, void* stream) {
  if (!qkv || !rn) return hvk_set_error(HVK_EINVAL, "hvk_qk_normalize: null pointer");
  if (T <= 0 || C <= 0 || C % 32) return hvk_set_error(HVK_EINVAL, "hvk_qk_normalize: T=%d C=%d (C %% 32)", T, C);
  const long long items = (long long)((T + 15) / 16) * (2 * C / 32);
  const long long grid = (items + 3) / 4;
  if (grid > 0x7fffffffLL) return hvk_set_error(HVK_EINVAL, "hvk_qk_normalize: too many rows");
  hipLaunchKernelGGL(qk_normalize_kernel, dim3((unsigned)grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<hvk_bf16*>(qkv), rn, qscale, T, C);
  HVK_CHECK_LAUNCH("hvk_qk_normalize");
  return HVK_OK;
}

size_t hvk_bias_gelu_bwd_workspace_bytes(int N) {
  return (size_t)kBwdRowBlocks * N * sizeof(float);
}

int hvk_bias_gelu_fwd(const void* h, const float* bias, void* y, int rows, int N, void* stream) {
  if (!h || !y) return hvk_set_error(HVK_EINVAL, "hvk_bias_gelu_fwd: null pointer");
  if (rows <= 0 || N <= 0 || N % 8)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_bias_gelu_fwd: rows=%d N=%d (N %% 8 == 0)", rows, N);
  int gx = (rows + kWaves - 1) / kWaves;
  if (gx > 2048) gx = 2048;
  dim3 grid(gx, (N + 511) / 512);
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, grid, dim3(64 * kWaves), 0,
                     static_cast<hipStream_t>(stream), static_cast<const hvk_bf16*>(h), bias,
                     static_cast<hvk_bf16*>(y), rows, N);
  HVK_CHECK_LAUNCH("bias_gelu_fwd");
  return HVK_OK;
}

int hvk_bias_gelu_bwd(const void* h, const float* bias, const void* gy, void* gh, float* dbias,
                      float* workspace, size_t workspace_bytes, int rows, int N, void* stream) {
  if (!h || !gy || !gh) return hvk_set_error(HVK_EINVAL, "hvk_bias_gelu_bwd: null pointer");
  if (rows <= 0 || N <= 0 || N % 8)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_bias_gelu_bwd: rows=%d N=%d", rows, N);
  if (dbias && (!workspace || workspace_bytes < hvk_bias_gelu_bwd_workspace_bytes(N)))
    return hvk_set_error(HVK_EINVAL, "hvk_bias_gelu_bwd: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  int gx = (rows + kWaves - 1) / kWaves;
  if (gx > kBwdRowBlocks) gx = kBwdRowBlocks;
  dim3 grid(gx, (N + 511) / 512);
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, grid, dim3(64 * kWaves), 0, st,
                     static_cast<const hvk_bf16*>(h), bias, static_cast<const hvk_bf16*>(gy),
                     static_cast<hvk_bf16*>(gh), workspace, dbias, rows, N);
  HVK_CHECK_LAUNCH("bias_gelu_bwd");
  if (dbias) {
    hipLaunchKernelGGL(colsum_rows_kernel, dim3((N + 63) / 64, 16), dim3(64), 0, st, workspace,
                       gx, N, dbias);
    HVK_CHECK_LAUNCH("bias_gelu_colsum");
  }
  return HVK_OK;
}

}  // extern "C"
