// Taxonomy losses on gfx950.
//
// * Multitask CE (hierarchy.py:65-94) -- all tiers' heads in ONE launch over a
//   concatenated logit matrix; one wave per (tier, sample) row; hard int targets or
//   dense soft targets (LabelSmoothing, algorithmic.py:91-116).  Also the flat CE of
//   models.py:112 (n_heads = 1).
// * HXE (hierarchical cross-entropy; not implemented by the reference,
//   hierarchy.py:183-185): per sample, a segmented log-sum-exp over the nested
//   leaf ranges of the target's ancestors, each range contiguous in `perm` order.
//   One workgroup per sample; every range is a strided wavefront scan with an
//   online (max, sum) pair and a cross-wave merge.
#include "hvk_common.h"

namespace {

constexpr int kTiers = 7;
constexpr int kLevels = 8;  // 7 tiers + root

struct Lse {
  float m, s;
};
__device__ __forceinline__ Lse lse_push(Lse a, float x) {
  if (x > a.m) {
    a.s = a.s * __expf(a.m - x) + 1.f;
    a.m = x;
  } else {
    a.s += __expf(x - a.m);
  }
  return a;
}
__device__ __forceinline__ Lse lse_merge(Lse a, Lse b) {
  if (b.m == -INFINITY) return a;
  if (a.m == -INFINITY) return b;
  const float m = fmaxf(a.m, b.m);
  return Lse{m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}
__device__ __forceinline__ Lse wave_lse(Lse v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    Lse w{__shfl_xor(v.m, o), __shfl_xor(v.s, o)};
    v = lse_merge(v, w);
  }
  return v;
}

// ----------------------------------------------------------------- multitask CE
__global__ __launch_bounds__(256) void mt_ce_fwd_kernel(const float* __restrict__ logits, int ld,
                                                        int B, int n_heads,
                                                        const int* __restrict__ off,
                                                        const int64_t* __restrict__ tgt,
                                                        const float* __restrict__ soft,
                                                        float* row_loss, float* lse_out) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid >= B * n_heads) return;
  const int h = wid / B, b = wid % B;
  const int c0 = off[h], c1 = off[h + 1];
  const float* z = logits + (size_t)b * ld;
  Lse acc{-INFINITY, 0.f};
  float tz = 0.f, tsum = 0.f;
  for (int c = c0 + lane; c < c1; c += 64) {
    const float x = z[c];
    acc = lse_push(acc, x);
    if (soft) {
      const float t = soft[(size_t)b * ld + c];
      tz += t * x;
      tsum += t;
    }
  }
  acc = wave_lse(acc);
  const float lse = acc.m + __logf(acc.s);
  float loss;
  if (soft) {
    tz = hvk_wave_sum(tz);
    tsum = hvk_wave_sum(tsum);
    loss = lse * tsum - tz;
  } else {
    const int64_t t = tgt[(size_t)b * n_heads + h];
    // a target outside [0, classes) (torch's CE raises "Target out of bounds"): NaN loss, no
    // out-of-range read
    loss = (t >= 0 && t < c1 - c0) ? lse - z[c0 + (int)t] : __builtin_nanf("");
  }
  if (lane == 0) {
    row_loss[wid] = loss;
    lse_out[wid] = lse;
  }
}

__global__ __launch_bounds__(256) void mt_ce_bwd_kernel(const float* __restrict__ logits, int ld,
                                                        int B, int n_heads,
                                                        const int* __restrict__ off,
                                                        const int64_t* __restrict__ tgt,
                                                        const float* __restrict__ soft,
                                                        const float* __restrict__ lse,
                                                        const float* __restrict__ coeff,
                                                        const float* __restrict__ gout,
                                                        float* dlogits) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid >= B * n_heads) return;
  const int h = wid / B, b = wid % B;
  const int c0 = off[h], c1 = off[h + 1];
  const float g = gout[0] * coeff[h] / B;
  const float l = lse[wid];
  const float* z = logits + (size_t)b * ld;
  float* dz = dlogits + (size_t)b * ld;
  float tsum = 1.f;
  if (soft) {
    float s = 0.f;
    for (int c = c0 + lane; c < c1; c += 64) s += soft[(size_t)b * ld + c];
    tsum = hvk_wave_sum(s);
  }
  const int t = soft ? -1 : (int)tgt[(size_t)b * n_heads + h];
  for (int c = c0 + lane; c < c1; c += 64) {
    const float p = __expf(z[c] - l);
    const float tv = soft ? soft[(size_t)b * ld + c] : (c - c0 == t ? 1.f : 0.f);
    dz[c] = g * (p * tsum - tv);
  }
}

// ----------------------------------------------------------------- HXE
struct HxeArgs {
  const float* logits; int B, L; const int* perm; const int64_t* tgt;
  const int* nstart; const int* nend; const int* tbase; const float* coeff;
  float* row_loss; float* lse; const float* gout; float* dlogits;
};

// segment [lo, hi) in permuted positions of the target's node at level l (l = 7: all)
__device__ __forceinline__ void level_range(const HxeArgs& a, int b, int l, int& lo, int& hi) {
  if (l == kLevels - 1) { lo = 0; hi = a.L; return; }
  const int tier = kTiers - 1 - l;
  const int64_t node = a.tgt[(size_t)b * kTiers + tier];
  const int n_nodes = tier + 1 < kTiers ? a.tbase[tier + 1] - a.tbase[tier] : a.L;
  if (node < 0 || node >= n_nodes) {  // out-of-range target: an empty segment (NaN loss), no OOB read
    lo = 0;
    hi = -1;
    return;
  }
  lo = a.nstart[a.tbase[tier] + (int)node];
  hi = a.nend[a.tbase[tier] + (int)node];
}

__global__ __launch_bounds__(256) void hxe_fwd_kernel(HxeArgs a) {
  __shared__ float sm[4], ss[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* z = a.logits + (size_t)b * a.L;
  float loss = 0.f;
  for (int l = 0; l < kLevels; ++l) {
    int lo, hi;
    level_range(a, b, l, lo, hi);
    Lse acc{-INFINITY, 0.f};
    for (int pos = lo + threadIdx.x; pos < hi; pos += blockDim.x)
      acc = lse_push(acc, z[a.perm ? a.perm[pos] : pos]);
    acc = wave_lse(acc);
    if (lane == 0) { sm[wv] = acc.m; ss[wv] = acc.s; }
    __syncthreads();
    Lse tot{sm[0], ss[0]};
    for (int w = 1; w < 4; ++w) tot = lse_merge(tot, Lse{sm[w], ss[w]});
    __syncthreads();
    const float v = hi < lo ? __builtin_nanf("") : tot.m + __logf(tot.s);  // NaN: target out of range
    loss += a.coeff[l] * v;
    if (threadIdx.x == 0) a.lse[(size_t)b * kLevels + l] = v;
  }
  if (threadIdx.x == 0) a.row_loss[b] = loss;
}

__global__ __launch_bounds__(256) void hxe_bwd_kernel(HxeArgs a) {
  const int b = blockIdx.x;
  __shared__ int lo[kLevels], hi[kLevels];
  __shared__ float lv[kLevels];
  if (threadIdx.x < kLevels) {
    level_range(a, b, threadIdx.x, lo[threadIdx.x], hi[threadIdx.x]);
    lv[threadIdx.x] = a.lse[(size_t)b * kLevels + threadIdx.x];
  }
  __syncthreads();
  const float g = a.gout[0] / a.B;
  const float* z = a.logits + (size_t)b * a.L;
  float* dz = a.dlogits + (size_t)b * a.L;
  for (int pos = threadIdx.x; pos < a.L; pos += blockDim.x) {
    const int k = a.perm ? a.perm[pos] : pos;
    const float x = z[k];
    float d = 0.f;
#pragma unroll
    for (int l = 0; l < kLevels; ++l)
      if (pos >= lo[l] && pos < hi[l]) d += a.coeff[l] * __expf(x - lv[l]);
    dz[k] = g * d;
  }
}

}  // namespace

extern "C" {

int hvk_multitask_ce_fwd(const float* logits, int ld, int B, int n_heads, const int* head_off,
                         const int64_t* targets, const float* soft, float* row_loss, float* lse,
                         void* stream) {
  if (!logits || !head_off || !row_loss || !lse || (!targets && !soft))
    return hvk_set_error(HVK_EINVAL, "hvk_multitask_ce_fwd: null pointer");
  if (B <= 0 || n_heads <= 0 || ld <= 0)
    return hvk_set_error(HVK_EINVAL, "hvk_multitask_ce_fwd: bad shape");
  const int rows = B * n_heads;
  hipLaunchKernelGGL(mt_ce_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0,
                     static_cast<hipStream_t>(stream), logits, ld, B, n_heads, head_off, targets,
                     soft, row_loss, lse);
  HVK_CHECK_LAUNCH("multitask_ce_fwd");
  return HVK_OK;
}

int hvk_multitask_ce_bwd(const float* logits, int ld, int B, int n_heads, const int* head_off,
                         const int64_t* targets, const float* soft, const float* lse,
                         const float* coeff, const float* grad_out, float* dlogits,
                         void* stream) {
  if (!logits || !head_off || !lse || !coeff || !grad_out || !dlogits || (!targets && !soft))
    return hvk_set_error(HVK_EINVAL, "hvk_multitask_ce_bwd: null pointer");
  const int rows = B * n_heads;
  hipLaunchKernelGGL(mt_ce_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0,
                     static_cast<hipStream_t>(stream), logits, ld, B, n_heads, head_off, targets,
                     soft, lse, coeff, grad_out, dlogits);
  HVK_CHECK_LAUNCH("multitask_ce_bwd");
  return HVK_OK;
}

int hvk_hxe_fwd(const float* logits, int B, int L, const int* perm, const int64_t* targets,
                const int* node_start, const int* node_end, const int* tier_base,
                const float* level_coeff, float* row_loss, float* lse, void* stream) {
  if (!logits || !targets || !node_start || !node_end || !tier_base || !level_coeff ||
      !row_loss || !lse)
    return hvk_set_error(HVK_EINVAL, "hvk_hxe_fwd: null pointer");
  if (B <= 0 || L <= 0) return hvk_set_error(HVK_EINVAL, "hvk_hxe_fwd: bad shape");
  HxeArgs a{logits, B, L, perm, targets, node_start, node_end, tier_base, level_coeff,
            row_loss, lse, nullptr, nullptr};
  hipLaunchKernelGGL(hxe_fwd_kernel, dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  HVK_CHECK_LAUNCH("hxe_fwd");
  return HVK_OK;
}

int hvk_hxe_bwd(const float* logits, int B, int L, const int* perm, const int64_t* targets,
                const int* node_start, const int* node_end, const int* tier_base,
                const float* level_coeff, const float* lse, const float* grad_out,
                float* dlogits, void* stream) {
  if (!logits || !targets || !node_start || !node_end || !tier_base || !level_coeff || !lse ||
      !grad_out || !dlogits)
    return hvk_set_error(HVK_EINVAL, "hvk_hxe_bwd: null pointer");
  HxeArgs a{logits, B, L, perm, targets, node_start, node_end, tier_base, level_coeff,
            nullptr, const_cast<float*>(lse), grad_out, dlogits};
  hipLaunchKernelGGL(hxe_bwd_kernel, dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  HVK_CHECK_LAUNCH("hxe_bwd");
  return HVK_OK;
}

}  // extern "C"
