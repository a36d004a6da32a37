// Post-norm residual LayerNorm for SwinV2's res-post-norm blocks (gfx950).
//
//   a' = a + abias                       (bias of the Linear that produced a, folded in)
//   x  = x0 + s[b] * (gamma * (a' - mean) * rstd + beta)
//
// replaces `shortcut + drop_path(norm1(x))` / `x + drop_path(norm2(mlp(x)))`
// (swinv2.py:431, 434) -- a is the bf16 output of the proj / fc2 GEMM (run without its
// bias), x0 the f32 residual stream, s the per-sample DropPath factor -- and, with no x0,
// the plain norms of PatchMerging (swinv2.py:494), PatchEmbed (656) and the final norm
// (833).  One pass writes the f32 residual stream and its bf16 copy (next GEMM operand).
// The backward also column-sums the branch gradient, which IS the folded bias's gradient,
// so no separate bias-reduction pass exists.
//
// Layout: a row of C channels is owned by TPR lanes (power of two) holding EPT contiguous
// channels each (16/32-byte bf16 loads, 32/64-byte f32 loads); a wave works on 64/TPR
// rows at once, grid-strided.  Row statistics are TPR-lane xor-shuffle reductions.
#include "hvk_common.h"

namespace {

constexpr int kWaves = 4;

template <int EPT>
__device__ __forceinline__ void load_bf16(const hvk_bf16* p, float v[EPT]) {
#pragma unroll
  for (int i = 0; i < EPT / 8; ++i) {
    const uint4 w = reinterpret_cast<const uint4*>(p)[i];
    float f[8];
    hvk_unpack8(w, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[8 * i + j] = f[j];
  }
}
template <int EPT>
__device__ __forceinline__ void store_bf16(hvk_bf16* p, const float v[EPT]) {
#pragma unroll
  for (int i = 0; i < EPT / 8; ++i) reinterpret_cast<uint4*>(p)[i] = hvk_pack8(v + 8 * i);
}
template <int EPT>
__device__ __forceinline__ void load_f32(const float* p, float v[EPT]) {
#pragma unroll
  for (int i = 0; i < EPT / 4; ++i) {
    const float4 w = reinterpret_cast<const float4*>(p)[i];
    v[4 * i] = w.x; v[4 * i + 1] = w.y; v[4 * i + 2] = w.z; v[4 * i + 3] = w.w;
  }
}
template <int EPT>
__device__ __forceinline__ void store_f32(float* p, const float v[EPT]) {
#pragma unroll
  for (int i = 0; i < EPT / 4; ++i)
    reinterpret_cast<float4*>(p)[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}
template <int TPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = TPR / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

struct LnFwd {
  const hvk_bf16* a; const float* abias; const float* x0; const float* gamma; const float* beta;
  const float* sscale; int rows, C, rows_per_sample; float eps;
  float* x; hvk_bf16* xb; float* mean; float* rstd;
};

template <int EPT, int TPR>
__global__ __launch_bounds__(64 * kWaves) void ln_fwd_kernel(LnFwd p) {
  constexpr int RPW = 64 / TPR;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / TPR, t = lane % TPR;
  const int c0 = t * EPT;
  const bool act = c0 < p.C;
  float gm[EPT], bt[EPT], ab[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) { gm[j] = 0.f; bt[j] = 0.f; ab[j] = 0.f; }
  if (act) {
    load_f32<EPT>(p.gamma + c0, gm);
    load_f32<EPT>(p.beta + c0, bt);
    if (p.abias) load_f32<EPT>(p.abias + c0, ab);
  }
  const float invC = 1.f / p.C;
  for (int row = (blockIdx.x * kWaves + wave) * RPW + sub; row < p.rows;
       row += gridDim.x * kWaves * RPW) {
    float v[EPT];
    float s = 0.f;
    if (act) {
      load_bf16<EPT>(p.a + (size_t)row * p.C + c0, v);
#pragma unroll
      for (int j = 0; j < EPT; ++j) { v[j] += ab[j]; s += v[j]; }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) v[j] = 0.f;
    }
    const float mu = group_sum<TPR>(s) * invC;
    float ss = 0.f;
    if (act) {
#pragma unroll
      for (int j = 0; j < EPT; ++j) { const float d = v[j] - mu; ss += d * d; }
    }
    const float rs = rsqrtf(group_sum<TPR>(ss) * invC + p.eps);
    if (act) {
      const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
      float r[EPT];
      if (p.x0) load_f32<EPT>(p.x0 + (size_t)row * p.C + c0, r);
      else {
#pragma unroll
        for (int j = 0; j < EPT; ++j) r[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < EPT; ++j) r[j] += ((v[j] - mu) * rs * gm[j] + bt[j]) * sc;
      store_f32<EPT>(p.x + (size_t)row * p.C + c0, r);
      if (p.xb) store_bf16<EPT>(p.xb + (size_t)row * p.C + c0, r);
      if (t == 0) { p.mean[row] = mu; p.rstd[row] = rs; }
    }
  }
}

struct LnBwd {
  const hvk_bf16* a; const float* abias; const float* gamma; const float* sscale;
  const float* mean; const float* rstd; const float* gx; const hvk_bf16* gxb;
  int rows, C, rows_per_sample;
  float* gx0; hvk_bf16* ga; float* part;  // part: [gridDim.x][3][C] dgamma / dbeta / dabias
  float* zero0; float* zero1; float* zero2;  // [C] outputs of the colsum kernel that follows:
                                             // zeroed here (stream order) instead of memsets
};

template <int EPT, int TPR>
__global__ __launch_bounds__(64 * kWaves) void ln_bwd_kernel(LnBwd p) {
  constexpr int RPW = 64 / TPR;
  __shared__ float red[kWaves][3][TPR * EPT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / TPR, t = lane % TPR;
  const int c0 = t * EPT;
  const bool act = c0 < p.C;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < p.C; i += blockDim.x) {
      p.zero0[i] = 0.f;
      p.zero1[i] = 0.f;
      if (p.zero2) p.zero2[i] = 0.f;
    }
  float gm[EPT], ab[EPT], dg[EPT], db[EPT], dab[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) { gm[j] = ab[j] = dg[j] = db[j] = dab[j] = 0.f; }
  if (act) {
    load_f32<EPT>(p.gamma + c0, gm);
    if (p.abias) load_f32<EPT>(p.abias + c0, ab);
  }
  const float invC = 1.f / p.C;
  for (int row = (blockIdx.x * kWaves + wave) * RPW + sub; row < p.rows;
       row += gridDim.x * kWaves * RPW) {
    float y[EPT], go[EPT], gy[EPT];
    float s1 = 0.f, s2 = 0.f;
    const float mu = p.mean[row], rs = p.rstd[row];
    const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
    if (act) {
      load_bf16<EPT>(p.a + (size_t)row * p.C + c0, y);
      if (p.gx) load_f32<EPT>(p.gx + (size_t)row * p.C + c0, go);
      else {
#pragma unroll
        for (int j = 0; j < EPT; ++j) go[j] = 0.f;
      }
      if (p.gxb) {
        float q[EPT];
        load_bf16<EPT>(p.gxb + (size_t)row * p.C + c0, q);
#pragma unroll
        for (int j = 0; j < EPT; ++j) go[j] += q[j];
      }
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        y[j] = (y[j] + ab[j] - mu) * rs;
        const float o = go[j] * sc;  // gradient of the LN output
        dg[j] += o * y[j];
        db[j] += o;
        gy[j] = o * gm[j];
        s1 += gy[j];
        s2 += gy[j] * y[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) y[j] = go[j] = gy[j] = 0.f;
    }
    s1 = group_sum<TPR>(s1) * invC;
    s2 = group_sum<TPR>(s2) * invC;
    if (act) {
      float d[EPT];
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        d[j] = rs * (gy[j] - s1 - y[j] * s2);
        dab[j] += d[j];
      }
      store_bf16<EPT>(p.ga + (size_t)row * p.C + c0, d);
      if (p.gx0) store_f32<EPT>(p.gx0 + (size_t)row * p.C + c0, go);
    }
  }
  // fold the RPW row slots of the wave (lanes t, t+TPR, ...), then the waves via LDS
#pragma unroll
  for (int m = TPR; m < 64; m <<= 1)
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      dg[j] += __shfl_xor(dg[j], m);
      db[j] += __shfl_xor(db[j], m);
      dab[j] += __shfl_xor(dab[j], m);
    }
  if (sub == 0) {
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      red[wave][0][c0 + j] = dg[j];
      red[wave][1][c0 + j] = db[j];
      red[wave][2][c0 + j] = dab[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 3 * p.C; c += blockDim.x) {
    const int k = c / p.C, cc = c % p.C;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) acc += red[w][k][cc];
    p.part[(size_t)blockIdx.x * 3 * p.C + c] = acc;
  }
}

// column sums of the per-block partials [nblk][ncol]: one wave per (64-column group,
// row group), 8 independent loads in flight, one atomic per column and row group.
constexpr int kRedRowGroups = 32;
__global__ __launch_bounds__(64) void colsum_kernel(const float* part, int nblk, int ncol,
                                                    float* out0, float* out1, float* out2, int C) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= ncol) return;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int b = blockIdx.y;
  for (; b + 7 * kRedRowGroups < nblk; b += 8 * kRedRowGroups)
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += part[(size_t)(b + u * kRedRowGroups) * ncol + c];
  for (; b < nblk; b += kRedRowGroups) s[0] += part[(size_t)b * ncol + c];
  const float v = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  float* base = c < C ? out0 : (c < 2 * C ? out1 : out2);
  if (base) atomicAdd(base + (c % C), v);  // NULL output (e.g. no folded bias): skip
}

constexpr int kBwdBlocks = 1024;

// (EPT, TPR) for a channel count: TPR * EPT >= C, TPR a power of two <= 64
int pick_layout(int C, int& ept, int& tpr) {
  if (C % 8) return 1;
  ept = C > 512 ? 16 : 8;
  tpr = 1;
  while (tpr * ept < C) tpr <<= 1;
  return tpr > 64 ? 1 : 0;
}

#define HVK_LN_DISPATCH(KERNEL, GRID, ST, ARGS)                                               \
  switch (ept * 1000 + tpr) {                                                                 \
    case 8001: hipLaunchKernelGGL((KERNEL<8, 1>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break;   \
    case 8002: hipLaunchKernelGGL((KERNEL<8, 2>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break;   \
    case 8004: hipLaunchKernelGGL((KERNEL<8, 4>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break;   \
    case 8008: hipLaunchKernelGGL((KERNEL<8, 8>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break;   \
    case 8016: hipLaunchKernelGGL((KERNEL<8, 16>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break;  \
    case 8032: hipLaunchKernelGGL((KERNEL<8, 32>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break;  \
    case 8064: hipLaunchKernelGGL((KERNEL<8, 64>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break;  \
    case 16064: hipLaunchKernelGGL((KERNEL<16, 64>), GRID, dim3(64 * kWaves), 0, ST, ARGS); break; \
    default: return hvk_set_error(HVK_EUNSUPPORTED, "layernorm: no layout for C=%d", C);      \
  }

int check_shape(const char* who, int rows, int C, int rps, int& ept, int& tpr) {
  if (rows <= 0 || C <= 0 || rps <= 0)
    return hvk_set_error(HVK_EINVAL, "%s: bad shape rows=%d C=%d rows_per_sample=%d", who, rows, C, rps);
  if (pick_layout(C, ept, tpr))
    return hvk_set_error(HVK_EUNSUPPORTED, "%s: C=%d must be a multiple of 8 and <= 1024", who, C);
  return HVK_OK;
}

}  // namespace

extern "C" {

int hvk_ln_residual_fwd(const void* a, const float* abias, const float* x0, const float* gamma,
                        const float* beta, const float* sample_scale, int rows, int C,
                        int rows_per_sample, float eps, float* x_out, void* xb_out, float* mean,
                        float* rstd, void* stream) {
  int ept, tpr;
  int rc = check_shape("hvk_ln_residual_fwd", rows, C, rows_per_sample, ept, tpr);
  if (rc) return rc;
  if (!a || !gamma || !beta || !x_out || !mean || !rstd)
    return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_fwd: null pointer");
  LnFwd p{static_cast<const hvk_bf16*>(a), abias, x0, gamma, beta, sample_scale, rows, C,
          rows_per_sample, eps, x_out, static_cast<hvk_bf16*>(xb_out), mean, rstd};
  const int rows_per_block = kWaves * (64 / tpr);
  int grid = (rows + rows_per_block - 1) / rows_per_block;
  if (grid > 256 * 8) grid = 256 * 8;
  hipStream_t st = static_cast<hipStream_t>(stream);
  HVK_LN_DISPATCH(ln_fwd_kernel, dim3(grid), st, p);
  HVK_CHECK_LAUNCH("ln_fwd");
  return HVK_OK;
}

size_t hvk_ln_bwd_workspace_bytes(int C) { return (size_t)kBwdBlocks * 3 * C * sizeof(float); }

int hvk_ln_residual_bwd(const void* a, const float* abias, const float* gamma,
                        const float* sample_scale, const float* mean, const float* rstd,
                        const float* gx, const void* gxb, int rows, int C, int rows_per_sample,
                        float* gx0, void* ga, float* dgamma, float* dbeta, float* dabias,
                        float* workspace, size_t workspace_bytes, void* stream) {
  int ept, tpr;
  int rc = check_shape("hvk_ln_residual_bwd", rows, C, rows_per_sample, ept, tpr);
  if (rc) return rc;
  if (!a || !gamma || !mean || !rstd || !ga || !dgamma || !dbeta || !workspace || (!gx && !gxb))
    return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_bwd: null pointer");
  if (workspace_bytes < hvk_ln_bwd_workspace_bytes(C))
    return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_bwd: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int rows_per_block = kWaves * (64 / tpr);
  int grid = (rows + rows_per_block - 1) / rows_per_block;
  if (grid > kBwdBlocks) grid = kBwdBlocks;
  LnBwd p{static_cast<const hvk_bf16*>(a), abias, gamma, sample_scale, mean, rstd, gx,
          static_cast<const hvk_bf16*>(gxb), rows, C, rows_per_sample, gx0,
          static_cast<hvk_bf16*>(ga), workspace, dgamma, dbeta, dabias};
  HVK_LN_DISPATCH(ln_bwd_kernel, dim3(grid), st, p);
  HVK_CHECK_LAUNCH("ln_bwd");
  hipLaunchKernelGGL(colsum_kernel, dim3((3 * C + 63) / 64, kRedRowGroups), dim3(64), 0, st,
                     workspace, grid, 3 * C, dgamma, dbeta, dabias, C);
  HVK_CHECK_LAUNCH("ln_bwd_colsum");
  return HVK_OK;
}

}  // extern "C"
