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
// Layout: a row of C channels is owned by TPR lanes (power of two); lane t holds EPT channels
// as groups of 4 at channel 4 (i TPR + t), i < EPT / 4, so every wave-instruction reads or writes
// whole lines: lanes t, t+1, ... cover adjacent 16-B f32 (8-B bf16) pieces of the row.  (The
// round-1..3 layout gave a lane 8 contiguous channels: its two float4 accesses then sat 32 B
// apart, each f32 instruction touching every line it read or wrote by halves -- 1.8x slower
// at stage 0, tools/probe/ln_probe.hip, profiles/round4/ln_probe.txt.)  A wave works on 64/TPR
// rows at once, grid-strided.  Row statistics are TPR-lane xor-shuffle reductions.
#include <mutex>
#include "hvk_common.h"

#ifndef HVK_LN_X0_EARLY  // A/B build switch: residual loads issued with the branch-output loads
#define HVK_LN_X0_EARLY 1  // (up to TPR = 16, i.e. C <= 128: tools/bench_ln.py, profiles/round4/ln_ab)
#endif

namespace {

constexpr int kWaves = 4;

// group i of lane t: channels 4 (i TPR + t) .. +3
template <int TPR>
__device__ __forceinline__ int grp_c(int t, int i) { return 4 * (i * TPR + t); }
// HVK_NT_SAVED bit 4: the LayerNorm kernels' streamed inputs (the GEMM output a, the f32
// residual stream / its gradient, the bf16 gradient) are read for the last time in the pass
// (a again only by the backward), so they are loaded nontemporally
__device__ __forceinline__ void ld4_bf16(const hvk_bf16* p, float* v) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = hvk_lo(u.x); v[1] = hvk_hi(u.x); v[2] = hvk_lo(u.y); v[3] = hvk_hi(u.y);
}
__device__ __forceinline__ void st4_bf16(hvk_bf16* p, const float* v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
}
__device__ __forceinline__ void ld4_f32(const float* p, float* v) {
  const float4 w = *reinterpret_cast<const float4*>(p);
  v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
}
__device__ __forceinline__ void ld4_f32_stream(const float* p, float* v) {
  if (HVK_NT_SAVED & 16) {
    const uint4 u = hvk_ld16_nt(p);
    v[0] = __uint_as_float(u.x); v[1] = __uint_as_float(u.y); v[2] = __uint_as_float(u.z); v[3] = __uint_as_float(u.w);
  } else {
    ld4_f32(p, v);
  }
}
__device__ __forceinline__ void st4_f32(float* p, const float* v, bool nt) {
  const uint4 u = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
  if (nt) hvk_st16_nt(p, u);
  else *reinterpret_cast<uint4*>(p) = u;
}
template <int TPR>
__device__ __forceinline__ float group_sum(float v) {
  return hvk_xor_sum<TPR>(v);  // the xor butterfly m = TPR/2 .. 1, by DPP / permlane swaps
}

struct LnFwd {
  const hvk_bf16* a; const float* abias; const float* x0; const float* gamma; const float* beta;
  const float* sscale; int rows, C, rows_per_sample; float eps;
  float* x; hvk_bf16* xb; float* mean; float* rstd;
};

template <int EPT, int TPR>
__global__ __launch_bounds__(64 * kWaves) void ln_fwd_kernel(LnFwd p) {
  constexpr int RPW = 64 / TPR, NG = EPT / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / TPR, t = lane % TPR;
  float gm[EPT], bt[EPT], ab[EPT];
  bool ok[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int c = grp_c<TPR>(t, i);
    ok[i] = c < p.C;
#pragma unroll
    for (int j = 0; j < 4; ++j) gm[4 * i + j] = bt[4 * i + j] = ab[4 * i + j] = 0.f;
    if (ok[i]) {
      ld4_f32(p.gamma + c, gm + 4 * i);
      ld4_f32(p.beta + c, bt + 4 * i);
      if (p.abias) ld4_f32(p.abias + c, ab + 4 * i);
    }
  }
  const float invC = 1.f / p.C;
  for (int row = (blockIdx.x * kWaves + wave) * RPW + sub; row < p.rows;
       row += gridDim.x * kWaves * RPW) {
    const size_t rb = (size_t)row * p.C;
    float v[EPT], x0v[EPT];
    float s = 0.f;
    // the residual row loaded with the branch output, before the statistics: one memory round
    // trip per row instead of two (+EPT VGPRs).  Stage 0 (C = 96, 4 rows per wave) -1.4 %, the
    // 1-2-row-per-wave layouts of C >= 192 +6-12 % (tools/bench_ln.py): there it stays after
    constexpr bool early = HVK_LN_X0_EARLY && TPR <= 16;
    if constexpr (early) {
#pragma unroll
      for (int i = 0; i < NG; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) x0v[4 * i + j] = 0.f;
        if (ok[i] && p.x0) ld4_f32_stream(p.x0 + rb + grp_c<TPR>(t, i), x0v + 4 * i);
      }
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      if (ok[i]) {
        ld4_bf16(p.a + rb + grp_c<TPR>(t, i), v + 4 * i);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[4 * i + j] += ab[4 * i + j]; s += v[4 * i + j]; }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * i + j] = 0.f;
      }
    }
    const float mu = group_sum<TPR>(s) * invC;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NG; ++i)
      if (ok[i]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) ss = hvk_ln_sq(ss, v[4 * i + j] - mu);
      }
    const float rs = hvk_ln_rstd(group_sum<TPR>(ss), invC, p.eps);
    const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      if (!ok[i]) continue;
      const int c = grp_c<TPR>(t, i);
      float r[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (early) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = x0v[4 * i + j];
      } else if (p.x0) {
        ld4_f32_stream(p.x0 + rb + c, r);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = hvk_ln_out(r[j], v[4 * i + j], mu, rs, gm[4 * i + j], bt[4 * i + j], sc);
      st4_f32(p.x + rb + c, r, HVK_NT_SAVED & 2);  // the f32 stream is read again only at the next LayerNorm
      if (p.xb) st4_bf16(p.xb + rb + c, r);
    }
    if (t == 0) { p.mean[row] = mu; p.rstd[row] = rs; }
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
  constexpr int RPW = 64 / TPR, NG = EPT / 4;
  __shared__ float red[kWaves][3][TPR * EPT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / TPR, t = lane % TPR;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < p.C; i += blockDim.x) {
      p.zero0[i] = 0.f;
      p.zero1[i] = 0.f;
      if (p.zero2) p.zero2[i] = 0.f;
    }
  float gm[EPT], ab[EPT], dg[EPT], db[EPT], dab[EPT];
  bool ok[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int c = grp_c<TPR>(t, i);
    ok[i] = c < p.C;
#pragma unroll
    for (int j = 0; j < 4; ++j) gm[4 * i + j] = ab[4 * i + j] = dg[4 * i + j] = db[4 * i + j] = dab[4 * i + j] = 0.f;
    if (ok[i]) {
      ld4_f32(p.gamma + c, gm + 4 * i);
      if (p.abias) ld4_f32(p.abias + c, ab + 4 * i);
    }
  }
  const float invC = 1.f / p.C;
  for (int row = (blockIdx.x * kWaves + wave) * RPW + sub; row < p.rows;
       row += gridDim.x * kWaves * RPW) {
    const size_t rb = (size_t)row * p.C;
    float y[EPT], go[EPT], gy[EPT];
    float s1 = 0.f, s2 = 0.f;
    const float mu = p.mean[row], rs = p.rstd[row];
    const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      float* yi = y + 4 * i;
      float* gi = go + 4 * i;
      if (ok[i]) {
        const int c = grp_c<TPR>(t, i);
        ld4_bf16(p.a + rb + c, yi);
        if (p.gx) ld4_f32_stream(p.gx + rb + c, gi);
        else gi[0] = gi[1] = gi[2] = gi[3] = 0.f;
        if (p.gxb) {
          float q[4];
          ld4_bf16(p.gxb + rb + c, q);
#pragma unroll
          for (int j = 0; j < 4; ++j) gi[j] += q[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int e = 4 * i + j;
          y[e] = (y[e] + ab[e] - mu) * rs;
          const float o = go[e] * sc;  // gradient of the LN output
          dg[e] += o * y[e];
          db[e] += o;
          gy[e] = o * gm[e];
          s1 += gy[e];
          s2 += gy[e] * y[e];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) yi[j] = gi[j] = gy[4 * i + j] = 0.f;
      }
    }
    s1 = group_sum<TPR>(s1) * invC;
    s2 = group_sum<TPR>(s2) * invC;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      if (!ok[i]) continue;
      const int c = grp_c<TPR>(t, i);
      float d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = 4 * i + j;
        d[j] = rs * (gy[e] - s1 - y[e] * s2);
        dab[e] += d[j];
      }
      st4_bf16(p.ga + rb + c, d);
      if (p.gx0) st4_f32(p.gx0 + rb + c, go + 4 * i, HVK_NT_SAVED & 4);
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
      const int c = grp_c<TPR>(t, j / 4) + (j & 3);  // < TPR * EPT
      red[wave][0][c] = dg[j];
      red[wave][1][c] = db[j];
      red[wave][2][c] = dab[j];
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

// (EPT, TPR) for a channel count: TPR * EPT >= C, TPR a power of two <= 64 (tools/probe/
// ln_probe.hip: 8 channels per lane up to C = 512, the fastest at C = 96 / 192 / 384, 16 above)
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

// Final LayerNorm + token average pool (swinv2.py:833-835): y[b] = mean_t LN(x[b, t, :]) for
// the f32 stream x [B, T, C].  One 256-thread workgroup per sample; a wave normalizes rows
// t = wave, wave + 4, ... with its lanes holding V float4 columns each (C = 256 V); the
// per-sample sums of x-hat are kept (xsum) -- they are all the backward needs besides the
// row statistics: y = gamma * xsum / T + beta, d gamma = sum_b (dy_b / T) xsum_b, d beta =
// sum_b dy_b.  Workgroup 0 also zeroes the backward's d gamma / d beta accumulators.
template <int V>
__global__ __launch_bounds__(256) void ln_pool_fwd_kernel(const float4* __restrict__ x, const float4* __restrict__ gamma,
                                                          const float4* __restrict__ beta, int T, float eps,
                                                          float4* __restrict__ y, float4* __restrict__ xsum,
                                                          float* __restrict__ mean, float* __restrict__ rstd,
                                                          float4* __restrict__ zero_g, float4* __restrict__ zero_b) {
  constexpr int C4 = 64 * V;
  __shared__ float4 red[4][C4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (b == 0)
    for (int i = threadIdx.x; i < C4; i += 256) zero_g[i] = zero_b[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float invC = 1.f / (4 * C4);
  float4 acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int t = wave; t < T; t += 4) {
    const float4* xr = x + ((size_t)b * T + t) * C4;
    float4 v[V];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      v[j] = xr[lane + 64 * j];
      s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    }
    s = hvk_xor_sum<64>(s);
    const float mu = s * invC;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      v[j].x -= mu; v[j].y -= mu; v[j].z -= mu; v[j].w -= mu;
      q += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
    }
    q = hvk_xor_sum<64>(q);
    const float rs = rsqrtf(q * invC + eps);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      acc[j].x += v[j].x * rs; acc[j].y += v[j].y * rs; acc[j].z += v[j].z * rs; acc[j].w += v[j].w * rs;
    }
    if (lane == 0) {
      mean[(size_t)b * T + t] = mu;
      rstd[(size_t)b * T + t] = rs;
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) red[wave][lane + 64 * j] = acc[j];
  __syncthreads();
  const float invT = 1.f / T;
  for (int i = threadIdx.x; i < C4; i += 256) {
    float4 a = red[0][i];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 r = red[w][i];
      a.x += r.x; a.y += r.y; a.z += r.z; a.w += r.w;
    }
    xsum[(size_t)b * C4 + i] = a;
    const float4 g = gamma[i], be = beta[i];
    y[(size_t)b * C4 + i] = make_float4(g.x * a.x * invT + be.x, g.y * a.y * invT + be.y,
                                        g.z * a.z * invT + be.z, g.w * a.w * invT + be.w);
  }
}

// backward: every row of sample b receives g = dy_b / T; dx = rstd (g gamma - mean_c(g gamma)
// - xhat mean_c(g gamma xhat)); d gamma, d beta by one float atomic per column and sample
template <int V>
__global__ __launch_bounds__(256) void ln_pool_bwd_kernel(const float4* __restrict__ x, const float4* __restrict__ gamma,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          const float4* __restrict__ xsum, const float4* __restrict__ dy,
                                                          int T, float4* __restrict__ dx, float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta) {
  constexpr int C4 = 64 * V;
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float invT = 1.f / T, invC = 1.f / (4 * C4);
  float4 gg[V];
  float s1 = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const float4 d = dy[(size_t)b * C4 + lane + 64 * j], g = gamma[lane + 64 * j];
    gg[j] = make_float4(d.x * invT * g.x, d.y * invT * g.y, d.z * invT * g.z, d.w * invT * g.w);
    s1 += (gg[j].x + gg[j].y) + (gg[j].z + gg[j].w);
  }
  s1 = hvk_xor_sum<64>(s1);
  s1 *= invC;
  for (int t = wave; t < T; t += 4) {
    const size_t r = (size_t)b * T + t;
    const float mu = mean[r], rs = rstd[r];
    const float4* xr = x + r * C4;
    float4 h[V];
    float s2 = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float4 v = xr[lane + 64 * j];
      h[j] = make_float4((v.x - mu) * rs, (v.y - mu) * rs, (v.z - mu) * rs, (v.w - mu) * rs);
      s2 += (gg[j].x * h[j].x + gg[j].y * h[j].y) + (gg[j].z * h[j].z + gg[j].w * h[j].w);
    }
    s2 = hvk_xor_sum<64>(s2);
    s2 *= invC;
#pragma unroll
    for (int j = 0; j < V; ++j)
      dx[r * C4 + lane + 64 * j] =
          make_float4(rs * (gg[j].x - s1 - h[j].x * s2), rs * (gg[j].y - s1 - h[j].y * s2),
                      rs * (gg[j].z - s1 - h[j].z * s2), rs * (gg[j].w - s1 - h[j].w * s2));
  }
  for (int i = threadIdx.x; i < C4; i += 256) {
    const float4 d = dy[(size_t)b * C4 + i], xs = xsum[(size_t)b * C4 + i];
    atomicAdd(dgamma + 4 * i, d.x * invT * xs.x);
    atomicAdd(dgamma + 4 * i + 1, d.y * invT * xs.y);
    atomicAdd(dgamma + 4 * i + 2, d.z * invT * xs.z);
    atomicAdd(dgamma + 4 * i + 3, d.w * invT * xs.w);
    atomicAdd(dbeta + 4 * i, d.x);
    atomicAdd(dbeta + 4 * i + 1, d.y);
    atomicAdd(dbeta + 4 * i + 2, d.z);
    atomicAdd(dbeta + 4 * i + 3, d.w);
  }
}

#define HVK_POOL_DISPATCH(KERNEL, ...)                                                          \
  switch (C / 256) {                                                                           \
    case 1: hipLaunchKernelGGL((KERNEL<1>), dim3(B), dim3(256), 0, st, __VA_ARGS__); break;   \
    case 2: hipLaunchKernelGGL((KERNEL<2>), dim3(B), dim3(256), 0, st, __VA_ARGS__); break;   \
    case 3: hipLaunchKernelGGL((KERNEL<3>), dim3(B), dim3(256), 0, st, __VA_ARGS__); break;   \
    case 4: hipLaunchKernelGGL((KERNEL<4>), dim3(B), dim3(256), 0, st, __VA_ARGS__); break;   \
    case 6: hipLaunchKernelGGL((KERNEL<6>), dim3(B), dim3(256), 0, st, __VA_ARGS__); break;   \
    default: return hvk_set_error(HVK_EUNSUPPORTED, "ln_pool: C=%d", C);                      \
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

static int ln_residual_bwd(const void* a, const float* abias, const float* gamma, const float* sample_scale,
                           const float* mean, const float* rstd, const float* gx, const void* gxb, int rows, int C,
                           int rows_per_sample, float* gx0, void* ga, float* dgamma, float* dbeta, float* dabias,
                           float* workspace, size_t workspace_bytes, void* stream, void* param_stream);

int hvk_ln_residual_bwd(const void* a, const float* abias, const float* gamma,
                        const float* sample_scale, const float* mean, const float* rstd,
                        const float* gx, const void* gxb, int rows, int C, int rows_per_sample,
                        float* gx0, void* ga, float* dgamma, float* dbeta, float* dabias,
                        float* workspace, size_t workspace_bytes, void* stream) {
  return ln_residual_bwd(a, abias, gamma, sample_scale, mean, rstd, gx, gxb, rows, C, rows_per_sample, gx0, ga,
                         dgamma, dbeta, dabias, workspace, workspace_bytes, stream, nullptr);
}

int hvk_ln_residual_bwd_split(const void* a, const float* abias, const float* gamma, const float* sample_scale,
                              const float* mean, const float* rstd, const float* gx, const void* gxb, int rows,
                              int C, int rows_per_sample, float* gx0, void* ga, float* dgamma, float* dbeta,
                              float* dabias, float* workspace, size_t workspace_bytes, void* stream,
                              void* param_stream) {
  return ln_residual_bwd(a, abias, gamma, sample_scale, mean, rstd, gx, gxb, rows, C, rows_per_sample, gx0, ga,
                         dgamma, dbeta, dabias, workspace, workspace_bytes, stream, param_stream);
}

// The ordering event of hvk_ln_residual_bwd_split, one per device (an event recorded on another
// device's stream is invalid), created once under a lock (callers may be several host threads).
static hipEvent_t split_event() {
  static std::mutex mu;
  static hipEvent_t ev[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!ev[dev] && hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming) != hipSuccess) ev[dev] = nullptr;
  return ev[dev];
}

static int ln_residual_bwd(const void* a, const float* abias, const float* gamma, const float* sample_scale,
                           const float* mean, const float* rstd, const float* gx, const void* gxb, int rows, int C,
                           int rows_per_sample, float* gx0, void* ga, float* dgamma, float* dbeta, float* dabias,
                           float* workspace, size_t workspace_bytes, void* stream, void* param_stream) {
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
  hipStream_t cs = st;
  if (param_stream && param_stream != stream) {
    // the column sums (parameter gradients only) on the caller's parameter-gradient stream,
    // ordered after the row kernel by an event: they overlap the next input-gradient launches
    hipEvent_t ev = split_event();
    if (!ev) return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_bwd_split: event create failed");
    cs = static_cast<hipStream_t>(param_stream);
    if (hipEventRecord(ev, st) != hipSuccess || hipStreamWaitEvent(cs, ev, 0) != hipSuccess)
      return hvk_set_error(HVK_EINVAL, "hvk_ln_residual_bwd_split: stream ordering failed");
  }
  hipLaunchKernelGGL(colsum_kernel, dim3((3 * C + 63) / 64, kRedRowGroups), dim3(64), 0, cs,
                     workspace, grid, 3 * C, dgamma, dbeta, dabias, C);
  HVK_CHECK_LAUNCH("ln_bwd_colsum");
  return HVK_OK;
}

int hvk_ln_pool_supported(int C) { return C > 0 && C % 256 == 0 && (C / 256 <= 4 || C / 256 == 6); }

int hvk_ln_pool_fwd(const float* x, const float* gamma, const float* beta, int B, int T, int C, float eps,
                    float* y, float* xsum, float* mean, float* rstd, float* dgamma_zero, float* dbeta_zero,
                    void* stream) {
  if (!x || !gamma || !beta || !y || !xsum || !mean || !rstd || !dgamma_zero || !dbeta_zero)
    return hvk_set_error(HVK_EINVAL, "hvk_ln_pool_fwd: null pointer");
  if (B <= 0 || T <= 0 || !hvk_ln_pool_supported(C))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_ln_pool_fwd: B=%d T=%d C=%d", B, T, C);
  hipStream_t st = static_cast<hipStream_t>(stream);
  HVK_POOL_DISPATCH(ln_pool_fwd_kernel, reinterpret_cast<const float4*>(x), reinterpret_cast<const float4*>(gamma),
                    reinterpret_cast<const float4*>(beta), T, eps, reinterpret_cast<float4*>(y),
                    reinterpret_cast<float4*>(xsum), mean, rstd, reinterpret_cast<float4*>(dgamma_zero),
                    reinterpret_cast<float4*>(dbeta_zero));
  HVK_CHECK_LAUNCH("ln_pool_fwd");
  return HVK_OK;
}

int hvk_ln_pool_bwd(const float* x, const float* gamma, const float* mean, const float* rstd, const float* xsum,
                    const float* dy, int B, int T, int C, float* dx, float* dgamma, float* dbeta, void* stream) {
  if (!x || !gamma || !mean || !rstd || !xsum || !dy || !dx || !dgamma || !dbeta)
    return hvk_set_error(HVK_EINVAL, "hvk_ln_pool_bwd: null pointer");
  if (B <= 0 || T <= 0 || !hvk_ln_pool_supported(C))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_ln_pool_bwd: B=%d T=%d C=%d", B, T, C);
  hipStream_t st = static_cast<hipStream_t>(stream);
  HVK_POOL_DISPATCH(ln_pool_bwd_kernel, reinterpret_cast<const float4*>(x), reinterpret_cast<const float4*>(gamma),
                    mean, rstd, reinterpret_cast<const float4*>(xsum), reinterpret_cast<const float4*>(dy), T,
                    reinterpret_cast<float4*>(dx), dgamma, dbeta);
  HVK_CHECK_LAUNCH("ln_pool_bwd");
  return HVK_OK;
}

}  // extern "C"
