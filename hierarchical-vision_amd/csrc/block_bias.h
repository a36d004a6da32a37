// Device bodies of the per-block bias kernels (attn_bias.hip, cpb.hip), shared with the
// combined one-launch-per-direction block kernels (block_bias.hip).  `bid` / `nblk` are the
// workgroup's index / count within its role (a combined launch splits its grid by role).
#pragma once
#include "hvk_common.h"

namespace hvk_bias {

constexpr int kHid = 512;        // cpb_mlp hidden width (swinv2.py:141)
constexpr int kRowsPerBlock = 8;  // CPB backward rows per workgroup (22 for the 169 rows of w7)
constexpr int kAbRows = 8;        // attention-bias backward: rows of W_proj per workgroup

// qkv_bias = (q_bias, 0, 0), dv_zero = 0, eff[n] = pb[n] + W[n, :] . v (one wave per row)
__device__ __forceinline__ void attn_bias_fwd_body(int bid, int nblk, const float* __restrict__ qb,
                                                   const float* __restrict__ vb, const float* __restrict__ pb,
                                                   const float* __restrict__ w, int C, float* __restrict__ qkv_bias,
                                                   float* __restrict__ eff, float* __restrict__ dv_zero) {
  const int nt = blockDim.x;
  for (int i = bid * nt + threadIdx.x; i < 3 * C; i += nblk * nt) {
    qkv_bias[i] = (i < C && qb) ? qb[i] : 0.f;
    if (dv_zero && i < C) dv_zero[i] = 0.f;  // the backward's d v_bias accumulator
  }
  const int lane = threadIdx.x & 63, waves = nt >> 6;
  for (int n = bid * waves + (threadIdx.x >> 6); n < C; n += nblk * waves) {
    float s = 0.f;
    for (int k = lane; k < C; k += 64) s = fmaf(w[(size_t)n * C + k], vb[k], s);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) eff[n] = (pb ? pb[n] : 0.f) + s;
  }
}

// kAbRows rows n of W per workgroup: d W[n, :] = g[n] v^T (dw not null) and the rows' share of
// d v = W^T g (column partial sums, one f32 atomic per column per workgroup into d v, zeroed forward)
__device__ __forceinline__ void attn_bias_bwd_body(int bid, const float* __restrict__ g,
                                                   const float* __restrict__ vb, const float* __restrict__ w,
                                                   int C, float* __restrict__ dpb, float* __restrict__ dvb,
                                                   float* __restrict__ dw) {
  const int n0 = bid * kAbRows;
  for (int k = threadIdx.x; k < C; k += blockDim.x) {
    const float vk = vb[k];
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < kAbRows; ++r) {
      const int n = n0 + r;
      if (n < C) {
        const float gn = g[n];
        if (dw) dw[(size_t)n * C + k] = gn * vk;  // null: the proj weight-gradient kernel adds it
        acc = fmaf(w[(size_t)n * C + k], gn, acc);
      }
    }
    atomicAdd(dvb + k, acc);
  }
  if (dpb)
    for (int i = threadIdx.x; i < kAbRows && n0 + i < C; i += blockDim.x) dpb[n0 + i] = g[n0 + i];
}

// CPB table: one wave per (h, r) output (lane l owns hidden units l, l+64, ...), 4 per
// workgroup of 256; workgroup 0 also writes scale = exp(min(logit, clamp_max))
__device__ __forceinline__ void cpb_fwd_body(int bid, const float* __restrict__ coords, const float* __restrict__ w1,
                                             const float* __restrict__ b1, const float* __restrict__ w2,
                                             const float* __restrict__ logit, float clamp_max, int RR, int nH,
                                             float* __restrict__ table, float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int out = bid * 4 + (threadIdx.x >> 6);
  if (bid == 0 && threadIdx.x < nH)
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

// CPB backward, stage 1 (512 threads: thread j = hidden unit; kRowsPerBlock rows r per
// workgroup): partial dW2[:, j], dW1[j, :], db1[j] -> part[bid][nH + 3][512]
__device__ __forceinline__ void cpb_bwd_partial_body(int bid, const float* __restrict__ coords,
                                                     const float* __restrict__ w1, const float* __restrict__ b1,
                                                     const float* __restrict__ w2, const float* __restrict__ table,
                                                     const float* __restrict__ dtable, int RR, int nH,
                                                     float* __restrict__ part) {
  __shared__ float dpre[kRowsPerBlock][32];
  const int j = threadIdx.x;
  const int r0 = bid * kRowsPerBlock;
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
  float* p = part + (size_t)bid * (nH + 3) * kHid;
#pragma unroll
  for (int h = 0; h < 32; ++h)
    if (h < nH) p[(size_t)h * kHid + j] = dw2[h];
  p[(size_t)nH * kHid + j] = dw10;
  p[(size_t)(nH + 1) * kHid + j] = dw11;
  p[(size_t)(nH + 2) * kHid + j] = db;
}

// CPB backward, stage 2: sum the partials into dW2 [nH, 512], dW1 [512, 2], db1 [512] and
// d logit_scale = d scale * scale * [logit <= clamp_max]
__device__ __forceinline__ void cpb_bwd_reduce_body(int bid, const float* __restrict__ part, int nblk, int nH,
                                                    const float* __restrict__ logit, float clamp_max,
                                                    const float* __restrict__ dscale, float* __restrict__ dw1,
                                                    float* __restrict__ db1, float* __restrict__ dw2,
                                                    float* __restrict__ dlogit) {
  const int idx = bid * blockDim.x + threadIdx.x;
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

}  // namespace hvk_bias
