// LayerNorm forward / backward memory-shape probe (NOT product code): the product kernels'
// arithmetic (csrc/layernorm.hip: LN + DropPath + residual + folded bias, 12 B per element
// forward, 14 B backward) in several access layouts and grid forms, timed with hip events on the
// SwinV2-T bs256 stage shapes.  Variants:
//   L (layout) 0: lane holds 8 contiguous channels (the product form: 16-B bf16 loads, two
//                 float4 loads 32 B apart per lane -- each f32 instruction touches half of every
//                 line it reads);
//              1: lane holds channel groups of 4 at g = t, t + TPR, ... (8-B bf16 loads, f32
//                 float4 loads lane-contiguous: every instruction reads whole lines)
//   PF 1: the next row group's inputs are loaded before the current one is reduced
//   grid: "cap" = min(rows / rows-per-block, 2048) persistent blocks, "full" = one row group
//         per wave (non-persistent)
//   hipcc -O3 --offload-arch=gfx950 -I../../hierarchical-vision_amd/csrc ln_probe.hip -o ln_probe
#include <stdio.h>
#include <stdlib.h>

#include "hvk_common.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

namespace {
constexpr int kWaves = 4;

template <int TPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = TPR / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

struct Fwd {
  const hvk_bf16* a; const float* x0; const float* gamma; const float* beta;
  int rows, C; float eps;
  float* x; hvk_bf16* xb; float* mean; float* rstd;
};

// channel of element j (0..EPT-1) held by lane t
template <int L, int EPT, int TPR>
__device__ __forceinline__ int chan(int t, int j) {
  if constexpr (L == 0) return t * EPT + j;
  else return 4 * ((j / 4) * TPR + t) + (j % 4);
}

template <int L, int EPT, int TPR>
__device__ __forceinline__ void ld_row(const Fwd& p, int row, int t, float v[EPT], float r[EPT]) {
  const hvk_bf16* ar = p.a + (size_t)row * p.C;
  const float* xr = p.x0 + (size_t)row * p.C;
  if constexpr (L == 0) {
    const int c0 = t * EPT;
    if (c0 < p.C) {
#pragma unroll
      for (int i = 0; i < EPT / 8; ++i) {
        float f[8];
        hvk_unpack8(reinterpret_cast<const uint4*>(ar + c0)[i], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[8 * i + k] = f[k];
      }
#pragma unroll
      for (int i = 0; i < EPT / 4; ++i) {
        const float4 w = reinterpret_cast<const float4*>(xr + c0)[i];
        r[4 * i] = w.x; r[4 * i + 1] = w.y; r[4 * i + 2] = w.z; r[4 * i + 3] = w.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) v[j] = r[j] = 0.f;
    }
  } else {
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i) {
      const int c = 4 * (i * TPR + t);
      if (c < p.C) {
        const uint2 u = *reinterpret_cast<const uint2*>(ar + c);
        v[4 * i] = hvk_lo(u.x); v[4 * i + 1] = hvk_hi(u.x); v[4 * i + 2] = hvk_lo(u.y); v[4 * i + 3] = hvk_hi(u.y);
        const float4 w = *reinterpret_cast<const float4*>(xr + c);
        r[4 * i] = w.x; r[4 * i + 1] = w.y; r[4 * i + 2] = w.z; r[4 * i + 3] = w.w;
      } else {
        v[4 * i] = v[4 * i + 1] = v[4 * i + 2] = v[4 * i + 3] = 0.f;
        r[4 * i] = r[4 * i + 1] = r[4 * i + 2] = r[4 * i + 3] = 0.f;
      }
    }
  }
}

template <int L, int EPT, int TPR>
__device__ __forceinline__ void finish_row(const Fwd& p, int row, int t, const float gm[EPT], const float bt[EPT],
                                           float v[EPT], float r[EPT]) {
  const float invC = 1.f / p.C;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < EPT; ++j) s += v[j];
  const float mu = group_sum<TPR>(s) * invC;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const bool ok = chan<L, EPT, TPR>(t, j) < p.C;
    const float d = ok ? v[j] - mu : 0.f;
    ss += d * d;
  }
  const float rs = rsqrtf(group_sum<TPR>(ss) * invC + p.eps);
#pragma unroll
  for (int j = 0; j < EPT; ++j) r[j] += (v[j] - mu) * rs * gm[j] + bt[j];
  float* xr = p.x + (size_t)row * p.C;
  hvk_bf16* br = p.xb + (size_t)row * p.C;
  if constexpr (L == 0) {
    const int c0 = t * EPT;
    if (c0 < p.C) {
#pragma unroll
      for (int i = 0; i < EPT / 4; ++i)
        hvk_st16_nt(xr + c0 + 4 * i, make_uint4(__float_as_uint(r[4 * i]), __float_as_uint(r[4 * i + 1]),
                                                __float_as_uint(r[4 * i + 2]), __float_as_uint(r[4 * i + 3])));
#pragma unroll
      for (int i = 0; i < EPT / 8; ++i) reinterpret_cast<uint4*>(br + c0)[i] = hvk_pack8(r + 8 * i);
    }
  } else {
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i) {
      const int c = 4 * (i * TPR + t);
      if (c < p.C) {
        hvk_st16_nt(xr + c, make_uint4(__float_as_uint(r[4 * i]), __float_as_uint(r[4 * i + 1]),
                                       __float_as_uint(r[4 * i + 2]), __float_as_uint(r[4 * i + 3])));
        *reinterpret_cast<uint2*>(br + c) = make_uint2(hvk_pack2(r[4 * i], r[4 * i + 1]), hvk_pack2(r[4 * i + 2], r[4 * i + 3]));
      }
    }
  }
  if (t == 0) { p.mean[row] = mu; p.rstd[row] = rs; }
}

template <int L, int EPT, int TPR, int PF>
__global__ __launch_bounds__(64 * kWaves) void fwd_kernel(Fwd p) {
  constexpr int RPW = 64 / TPR;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / TPR, t = lane % TPR;
  float gm[EPT], bt[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int c = chan<L, EPT, TPR>(t, j);
    gm[j] = c < p.C ? p.gamma[c] : 0.f;
    bt[j] = c < p.C ? p.beta[c] : 0.f;
  }
  const int stride = gridDim.x * kWaves * RPW;
  int row = (blockIdx.x * kWaves + wave) * RPW + sub;
  if constexpr (PF == 0) {
    for (; row < p.rows; row += stride) {
      float v[EPT], r[EPT];
      ld_row<L, EPT, TPR>(p, row, t, v, r);
      finish_row<L, EPT, TPR>(p, row, t, gm, bt, v, r);
    }
  } else {
    if (row >= p.rows) return;
    float v[EPT], r[EPT];
    ld_row<L, EPT, TPR>(p, row, t, v, r);
    for (;;) {
      const int nxt = row + stride;
      float v2[EPT], r2[EPT];
      const bool more = nxt < p.rows;
      if (more) ld_row<L, EPT, TPR>(p, nxt, t, v2, r2);
      finish_row<L, EPT, TPR>(p, row, t, gm, bt, v, r);
      if (!more) break;
#pragma unroll
      for (int j = 0; j < EPT; ++j) { v[j] = v2[j]; r[j] = r2[j]; }
      row = nxt;
    }
  }
}

template <int L, int EPT, int TPR, int PF>
float run_fwd(const Fwd& p, int grid, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((fwd_kernel<L, EPT, TPR, PF>), dim3(grid), dim3(256), 0, 0, p);
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((fwd_kernel<L, EPT, TPR, PF>), dim3(grid), dim3(256), 0, 0, p);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int L, int EPT, int TPR>
void stage(const char* nm, Fwd p) {
  constexpr int rpb = kWaves * (64 / TPR);
  const int full = (p.rows + rpb - 1) / rpb;
  const int cap = full < 2048 ? full : 2048;
  const double bytes = 12.0 * p.rows * p.C;
  const int reps = 20;
  struct { const char* what; float us; } res[6];
  res[0] = {"cap", 1e3f * run_fwd<L, EPT, TPR, 0>(p, cap, reps)};
  res[1] = {"full", 1e3f * run_fwd<L, EPT, TPR, 0>(p, full, reps)};
  res[2] = {"cap pf", 1e3f * run_fwd<L, EPT, TPR, 1>(p, cap, reps)};
  res[3] = {"1024 pf", 1e3f * run_fwd<L, EPT, TPR, 1>(p, cap < 1024 ? cap : 1024, reps)};
  res[4] = {"512 pf", 1e3f * run_fwd<L, EPT, TPR, 1>(p, cap < 512 ? cap : 512, reps)};
  res[5] = {"full (again)", 1e3f * run_fwd<L, EPT, TPR, 0>(p, full, reps)};
  for (auto& r : res)
    printf("%-8s C=%4d L=%d EPT=%2d TPR=%2d %-12s %8.1f us  %6.0f GB/s  %.3f of 8 TB/s\n", nm, p.C, L, EPT, TPR,
           r.what, r.us, bytes / r.us * 1e-3, bytes / r.us * 1e-3 / 8000.0);
}
}  // namespace

int main() {
  const long long maxel = 802816ll * 96;
  hvk_bf16 *a, *xb;
  float *x0, *x, *gamma, *beta, *mean, *rstd;
  CK(hipMalloc(&a, maxel * 2));
  CK(hipMalloc(&xb, maxel * 2));
  CK(hipMalloc(&x0, maxel * 4));
  CK(hipMalloc(&x, maxel * 4));
  CK(hipMalloc(&gamma, 4096 * 4));
  CK(hipMalloc(&beta, 4096 * 4));
  CK(hipMalloc(&mean, 802816 * 4));
  CK(hipMalloc(&rstd, 802816 * 4));
  CK(hipMemset(a, 0x3c, maxel * 2));
  CK(hipMemset(x0, 0x3c, maxel * 4));
  CK(hipMemset(gamma, 0x3c, 4096 * 4));
  CK(hipMemset(beta, 0, 4096 * 4));
  struct { const char* nm; int rows, C; } st[] = {{"stage0", 802816, 96}, {"stage1", 200704, 192},
                                                  {"stage2", 50176, 384}, {"stage3", 12544, 768}};
  for (auto& s : st) {
    Fwd p{a, x0, gamma, beta, s.rows, s.C, 1e-5f, x, xb, mean, rstd};
    if (s.C == 96) { stage<0, 8, 16>(s.nm, p); stage<1, 8, 16>(s.nm, p); stage<1, 4, 32>(s.nm, p); }
    if (s.C == 192) { stage<0, 8, 32>(s.nm, p); stage<1, 8, 32>(s.nm, p); stage<1, 4, 64>(s.nm, p); }
    if (s.C == 384) { stage<0, 8, 64>(s.nm, p); stage<1, 8, 64>(s.nm, p); }
    if (s.C == 768) { stage<0, 16, 64>(s.nm, p); stage<1, 16, 64>(s.nm, p); }
  }
  return 0;
}
