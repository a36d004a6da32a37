// Post-norm residual LayerNorm for SwinV2's res-post-norm blocks (gfx950).
//
//   x = x0 + s[b] * (gamma * (a - mean) * rstd + beta)
//
// replaces `shortcut + drop_path(norm1(x))` / `x + drop_path(norm2(mlp(x)))`
// (swinv2.py:431, 434) -- a is the bf16 output of the proj / fc2 GEMM, x0 the f32
// residual stream, s the per-sample DropPath factor -- and, with no x0, the plain
// norms of PatchMerging (swinv2.py:494), PatchEmbed (656) and the final norm (833).
// It writes the f32 residual stream and its bf16 copy (the next GEMM's operand) in
// one pass.  One wave per row; each lane owns bf16 pairs (4-byte loads) strided by 64.
#include "hvk_common.h"

namespace {

constexpr int kRowsPerBlock = 4;  // one wave per row
constexpr int kMaxPairs = 8;      // C <= 1024

struct LnFwd {
  const hvk_bf16* a; const float* x0; const float* gamma; const float* beta; const float* sscale;
  int rows, C, rows_per_sample; float eps;
  float* x; hvk_bf16* xb; float* mean; float* rstd;
};

__global__ __launch_bounds__(256) void ln_fwd_kernel(LnFwd p) {
  const int lane = threadIdx.x & 63;
  const int npair = p.C >> 1;
  for (int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6); row < p.rows;
       row += gridDim.x * kRowsPerBlock) {
    const uint32_t* ar = reinterpret_cast<const uint32_t*>(p.a + (size_t)row * p.C);
    float v[kMaxPairs][2];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxPairs; ++k) {
      const int j = lane + 64 * k;
      if (j < npair) {
        const uint32_t w = ar[j];
        v[k][0] = hvk_lo(w); v[k][1] = hvk_hi(w);
        s += v[k][0] + v[k][1];
      } else {
        v[k][0] = v[k][1] = 0.f;
      }
    }
    const float mu = hvk_wave_sum(s) / p.C;
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxPairs; ++k) {
      const int j = lane + 64 * k;
      if (j < npair) {
        const float d0 = v[k][0] - mu, d1 = v[k][1] - mu;
        ss += d0 * d0 + d1 * d1;
      }
    }
    const float var = hvk_wave_sum(ss) / p.C;
    const float rs = rsqrtf(var + p.eps);
    const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
    const float2* x0r = p.x0 ? reinterpret_cast<const float2*>(p.x0 + (size_t)row * p.C) : nullptr;
    float2* xr = reinterpret_cast<float2*>(p.x + (size_t)row * p.C);
    uint32_t* xbr = p.xb ? reinterpret_cast<uint32_t*>(p.xb + (size_t)row * p.C) : nullptr;
    const float2* g2 = reinterpret_cast<const float2*>(p.gamma);
    const float2* b2 = reinterpret_cast<const float2*>(p.beta);
#pragma unroll
    for (int k = 0; k < kMaxPairs; ++k) {
      const int j = lane + 64 * k;
      if (j < npair) {
        const float2 gg = g2[j], bb = b2[j];
        float y0 = ((v[k][0] - mu) * rs * gg.x + bb.x) * sc;
        float y1 = ((v[k][1] - mu) * rs * gg.y + bb.y) * sc;
        if (x0r) {
          const float2 r = x0r[j];
          y0 += r.x; y1 += r.y;
        }
        xr[j] = make_float2(y0, y1);
        if (xbr) xbr[j] = hvk_pack2(y0, y1);
      }
    }
    if (lane == 0) { p.mean[row] = mu; p.rstd[row] = rs; }
  }
}

struct LnBwd {
  const hvk_bf16* a; const float* gamma; const float* sscale; const float* mean; const float* rstd;
  const float* gx; const hvk_bf16* gxb; int rows, C, rows_per_sample;
  float* gx0; hvk_bf16* ga; float* part;  // part: [gridDim.x][2][C] per-block dgamma/dbeta
};

__global__ __launch_bounds__(256) void ln_bwd_kernel(LnBwd p) {
  __shared__ float red[2][kRowsPerBlock][2 * 64 * kMaxPairs];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int npair = p.C >> 1;
  float dg[kMaxPairs][2], db[kMaxPairs][2];
#pragma unroll
  for (int k = 0; k < kMaxPairs; ++k) dg[k][0] = dg[k][1] = db[k][0] = db[k][1] = 0.f;
  const float2* g2 = reinterpret_cast<const float2*>(p.gamma);
  for (int row = blockIdx.x * kRowsPerBlock + wv; row < p.rows; row += gridDim.x * kRowsPerBlock) {
    const float mu = p.mean[row], rs = p.rstd[row];
    const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
    const uint32_t* ar = reinterpret_cast<const uint32_t*>(p.a + (size_t)row * p.C);
    const float2* gxr = p.gx ? reinterpret_cast<const float2*>(p.gx + (size_t)row * p.C) : nullptr;
    const uint32_t* gxbr = p.gxb ? reinterpret_cast<const uint32_t*>(p.gxb + (size_t)row * p.C) : nullptr;
    float y[kMaxPairs][2], gy[kMaxPairs][2], go[kMaxPairs][2];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxPairs; ++k) {
      const int j = lane + 64 * k;
      y[k][0] = y[k][1] = gy[k][0] = gy[k][1] = go[k][0] = go[k][1] = 0.f;
      if (j < npair) {
        const uint32_t w = ar[j];
        y[k][0] = (hvk_lo(w) - mu) * rs;
        y[k][1] = (hvk_hi(w) - mu) * rs;
        float t0 = 0.f, t1 = 0.f;
        if (gxr) { const float2 q = gxr[j]; t0 += q.x; t1 += q.y; }
        if (gxbr) { const uint32_t q = gxbr[j]; t0 += hvk_lo(q); t1 += hvk_hi(q); }
        go[k][0] = t0; go[k][1] = t1;       // gradient of the block output (and of x0)
        const float o0 = t0 * sc, o1 = t1 * sc;  // gradient of the LN output
        dg[k][0] += o0 * y[k][0]; dg[k][1] += o1 * y[k][1];
        db[k][0] += o0; db[k][1] += o1;
        const float2 gg = g2[j];
        gy[k][0] = o0 * gg.x; gy[k][1] = o1 * gg.y;
        s1 += gy[k][0] + gy[k][1];
        s2 += gy[k][0] * y[k][0] + gy[k][1] * y[k][1];
      }
    }
    s1 = hvk_wave_sum(s1) / p.C;
    s2 = hvk_wave_sum(s2) / p.C;
    uint32_t* gar = reinterpret_cast<uint32_t*>(p.ga + (size_t)row * p.C);
    float2* gx0r = p.gx0 ? reinterpret_cast<float2*>(p.gx0 + (size_t)row * p.C) : nullptr;
#pragma unroll
    for (int k = 0; k < kMaxPairs; ++k) {
      const int j = lane + 64 * k;
      if (j < npair) {
        const float d0 = rs * (gy[k][0] - s1 - y[k][0] * s2);
        const float d1 = rs * (gy[k][1] - s1 - y[k][1] * s2);
        gar[j] = hvk_pack2(d0, d1);
        if (gx0r) gx0r[j] = make_float2(go[k][0], go[k][1]);
      }
    }
  }
  // block partials of dgamma / dbeta (deterministic: no atomics)
#pragma unroll
  for (int k = 0; k < kMaxPairs; ++k) {
    const int j = lane + 64 * k;
    red[0][wv][2 * j] = dg[k][0]; red[0][wv][2 * j + 1] = dg[k][1];
    red[1][wv][2 * j] = db[k][0]; red[1][wv][2 * j + 1] = db[k][1];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < p.C; c += blockDim.x) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int w = 0; w < kRowsPerBlock; ++w) { a0 += red[0][w][c]; a1 += red[1][w][c]; }
    p.part[(size_t)blockIdx.x * 2 * p.C + c] = a0;
    p.part[(size_t)blockIdx.x * 2 * p.C + p.C + c] = a1;
  }
}

// dgamma/dbeta = column sums of the per-block partials [nblk][2C]: one wave per
// (64-column group, row group), 8 independent loads in flight, one atomic per column.
constexpr int kRedRowGroups = 32;
__global__ __launch_bounds__(64) void ln_bwd_reduce_kernel(const float* part, int nblk, int C,
                                                           float* dgamma, float* dbeta) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= 2 * C) return;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int b = blockIdx.y;
  for (; b + 7 * kRedRowGroups < nblk; b += 8 * kRedRowGroups)
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += part[(size_t)(b + u * kRedRowGroups) * 2 * C + c];
  for (; b < nblk; b += kRedRowGroups) s[0] += part[(size_t)b * 2 * C + c];
  const float t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  atomicAdd(c < C ? dgamma + c : dbeta + (c - C), t);
}

constexpr int kBwdBlocks = 1024;

int check_shape(const char* who, int rows, int C, int rps) {
  if (rows <= 0 || C <= 0 || rps <= 0)
    return hvk_set_error(HVK_EINVAL, "%s: bad shape rows=%d C=%d rows_per_sample=%d", who, rows, C, rps);
  if (C % 2 || C > 2 * 64 * kMaxPairs)
    return hvk_set_error(HVK_EUNSUPPORTED, "%s: C=%d must be even and <= %d", who, C, 2 * 64 * kMaxPairs);
  return HVK_OK;
}

}  // namespace

extern "C" {

int hvk_ln_residual_fwd(const void* a, const float* x0, const float* gamma, const float* beta,
                        const float* sample_scale, int rows, int C, int rows_per_sample,
                        float eps, float* x_out, void* xb_out, float* mean, float* rstd,
                        void* stream) {
  int rc = check_shape("hvk_ln_residual_fwd", rows, C, rows_per_sample);
  if (rc) return rc;
  if (!a || !gamma || !beta || !x_out || !mean || !rstd)
    return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_fwd: null pointer");
  LnFwd p{static_cast<const hvk_bf16*>(a), x0, gamma, beta, sample_scale, rows, C,
          rows_per_sample, eps, x_out, static_cast<hvk_bf16*>(xb_out), mean, rstd};
  int grid = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  if (grid > 256 * 32) grid = 256 * 32;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), p);
  HVK_CHECK_LAUNCH("ln_fwd");
  return HVK_OK;
}

size_t hvk_ln_bwd_workspace_bytes(int C) { return (size_t)kBwdBlocks * 2 * C * sizeof(float); }

int hvk_ln_residual_bwd(const void* a, const float* gamma, const float* sample_scale,
                        const float* mean, const float* rstd, const float* gx, const void* gxb,
                        int rows, int C, int rows_per_sample, float* gx0, void* ga,
                        float* dgamma, float* dbeta, float* workspace, size_t workspace_bytes,
                        void* stream) {
  int rc = check_shape("hvk_ln_residual_bwd", rows, C, rows_per_sample);
  if (rc) return rc;
  if (!a || !gamma || !mean || !rstd || !ga || !dgamma || !dbeta || !workspace || (!gx && !gxb))
    return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_bwd: null pointer");
  if (workspace_bytes < hvk_ln_bwd_workspace_bytes(C))
    return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_bwd: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  int grid = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  if (grid > kBwdBlocks) grid = kBwdBlocks;
  LnBwd p{static_cast<const hvk_bf16*>(a), gamma, sample_scale, mean, rstd, gx,
          static_cast<const hvk_bf16*>(gxb), rows, C, rows_per_sample, gx0,
          static_cast<hvk_bf16*>(ga), workspace};
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(grid), dim3(256), 0, st, p);
  HVK_CHECK_LAUNCH("ln_bwd");
  if (hipMemsetAsync(dgamma, 0, sizeof(float) * C, st) != hipSuccess ||
      hipMemsetAsync(dbeta, 0, sizeof(float) * C, st) != hipSuccess)
    return hvk_set_error(HVK_EHIP, "hvk_ln_residual_bwd: memset failed");
  hipLaunchKernelGGL(ln_bwd_reduce_kernel, dim3((2 * C + 63) / 64, kRedRowGroups), dim3(64), 0,
                     st, workspace, grid, C, dgamma, dbeta);
  HVK_CHECK_LAUNCH("ln_bwd_reduce");
  return HVK_OK;
}

}  // extern "C"
