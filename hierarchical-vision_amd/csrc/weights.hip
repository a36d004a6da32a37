// bf16 operand copies of the f32 master weights, all Linears of a step in ONE launch: for
// each weight W [rows, cols] f32, Wb = bf16(W) and (optionally) Wt = bf16(W)^T [cols, rows]
// -- the `weight.to(bfloat16)` of every autocast F.linear (swinv2.py:58-62, 220, 262, 296,
// 492, 653) and the transposed copy its input gradient runs on.  One workgroup per 32 x 32
// tile; the transpose goes through LDS.
#include "hvk_common.h"

namespace {

constexpr int kMaxT = 64;

struct CastBatch {
  const float* src[kMaxT];
  hvk_bf16* dst[kMaxT];
  hvk_bf16* dst_t[kMaxT];
  int rows[kMaxT];
  int cols[kMaxT];
  int tile0[kMaxT + 1];  // first tile of each weight (prefix sums)
  int n;
};

__global__ __launch_bounds__(256) void cast_weights_kernel(CastBatch b) {
  __shared__ float tile[32][33];
  const int bid = blockIdx.x;
  int t = 0;
  while (t + 1 < b.n && b.tile0[t + 1] <= bid) ++t;  // uniform scalar search, n <= 64
  const int local = bid - b.tile0[t];
  const int R = b.rows[t], C = b.cols[t];
  const int tc = (C + 31) >> 5;
  const int r0 = (local / tc) * 32, c0 = (local % tc) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* src = b.src[t];
  hvk_bf16* dst = b.dst[t];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + ty + 8 * i, c = c0 + tx;
    float v = 0.f;
    if (r < R && c < C) {
      v = src[(size_t)r * C + c];
      dst[(size_t)r * C + c] = (hvk_bf16)hvk_f2bf(v);
    }
    tile[ty + 8 * i][tx] = v;
  }
  hvk_bf16* dt = b.dst_t[t];
  if (!dt) return;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = c0 + ty + 8 * i, c = r0 + tx;  // row of W^T = column of W
    if (r < C && c < R) dt[(size_t)r * R + c] = (hvk_bf16)hvk_f2bf(tile[tx][ty + 8 * i]);
  }
}

// 64 x 64 tiles with 16-B loads and 8-B stores (rows and cols multiples of 4, every weight of
// SwinV2): lane (ty, tx) of 16 x 16 handles rows ty + 16 i, columns 4 tx .. 4 tx + 3; the
// transpose reads the LDS tile column-wise (stride 65 floats: conflict-free)
__global__ __launch_bounds__(256) void cast_weights_v4_kernel(CastBatch b) {
  __shared__ float tile[64][65];
  const int bid = blockIdx.x;
  int t = 0;
  while (t + 1 < b.n && b.tile0[t + 1] <= bid) ++t;
  const int local = bid - b.tile0[t];
  const int R = b.rows[t], C = b.cols[t];
  const int tc = (C + 63) >> 6;
  const int r0 = (local / tc) * 64, c0 = (local % tc) * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const float* src = b.src[t];
  hvk_bf16* dst = b.dst[t];
  const int c = c0 + 4 * tx;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + ty + 16 * i;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < R && c < C) {
      v = *reinterpret_cast<const float4*>(src + (size_t)r * C + c);
      *reinterpret_cast<uint2*>(dst + (size_t)r * C + c) = make_uint2(hvk_pack2(v.x, v.y), hvk_pack2(v.z, v.w));
    }
    tile[ty + 16 * i][4 * tx] = v.x;
    tile[ty + 16 * i][4 * tx + 1] = v.y;
    tile[ty + 16 * i][4 * tx + 2] = v.z;
    tile[ty + 16 * i][4 * tx + 3] = v.w;
  }
  hvk_bf16* dt = b.dst_t[t];
  if (!dt) return;
  __syncthreads();
  const int rr = r0 + 4 * tx;  // 4 consecutive rows of W = 4 consecutive columns of W^T
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cc = c0 + ty + 16 * i;  // column of W = row of W^T
    if (cc < C && rr < R) {
      const int lr = ty + 16 * i;
      *reinterpret_cast<uint2*>(dt + (size_t)cc * R + rr) =
          make_uint2(hvk_pack2(tile[4 * tx][lr], tile[4 * tx + 1][lr]),
                     hvk_pack2(tile[4 * tx + 2][lr], tile[4 * tx + 3][lr]));
    }
  }
}

}  // namespace

extern "C" {

int hvk_cast_weights(int n, const float* const* src, void* const* dst, void* const* dst_t,
                     const int* rows, const int* cols, void* stream) {
  if (n < 0 || (n > 0 && (!src || !dst || !rows || !cols)))
    return hvk_set_error(HVK_EINVAL, "hvk_cast_weights: null argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  for (int base = 0; base < n; base += kMaxT) {
    CastBatch b;
    b.n = n - base < kMaxT ? n - base : kMaxT;
    // the 16-B-load kernel: every weight of the batch with rows and cols multiples of 4, the f32
    // source 16-B aligned and the bf16 copies 8-B aligned (a view into a flat buffer may not be)
    bool v4 = true;
    for (int i = 0; i < b.n; ++i) {
      const int k = base + i;
      v4 = v4 && rows[k] % 4 == 0 && cols[k] % 4 == 0 && (uintptr_t)src[k] % 16 == 0 &&
           (uintptr_t)dst[k] % 8 == 0 && (!dst_t || (uintptr_t)dst_t[k] % 8 == 0);
    }
    const int T = v4 ? 64 : 32;
    int tiles = 0;
    for (int i = 0; i < b.n; ++i) {
      const int k = base + i;
      if (!src[k] || !dst[k] || rows[k] <= 0 || cols[k] <= 0)
        return hvk_set_error(HVK_EINVAL, "hvk_cast_weights: weight %d: null pointer or empty shape", k);
      b.src[i] = src[k];
      b.dst[i] = static_cast<hvk_bf16*>(dst[k]);
      b.dst_t[i] = dst_t ? static_cast<hvk_bf16*>(dst_t[k]) : nullptr;
      b.rows[i] = rows[k];
      b.cols[i] = cols[k];
      b.tile0[i] = tiles;
      tiles += ((rows[k] + T - 1) / T) * ((cols[k] + T - 1) / T);
    }
    b.tile0[b.n] = tiles;
    if (v4)
      hipLaunchKernelGGL(cast_weights_v4_kernel, dim3(tiles), dim3(256), 0, st, b);
    else
      hipLaunchKernelGGL(cast_weights_kernel, dim3(tiles), dim3(256), 0, st, b);
    HVK_CHECK_LAUNCH("hvk_cast_weights");
  }
  return HVK_OK;
}

}  // extern "C"
