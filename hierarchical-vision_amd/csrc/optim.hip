// Fused optimizer step for the training loop: the data-parallel gradient mean, global-norm
// gradient clipping (torch.nn.utils.clip_grad_norm_, algorithmic.py GradientClipping ->
// composer), DecoupledSGDW (composer.optim.DecoupledSGDW: momentum SGD with weight decay
// decoupled from the gradient, scaled by lr / initial_lr) and, on the batches the recipe asks
// for it, the weight EMA (configs/pretrain/inat21.yaml:31-34) over every parameter tensor in
// three launches, instead of one foreach pass per operation:
//   1. sumsq: each workgroup writes the sum of squares of its gradient chunk to its slot of
//      the workspace (no atomics, no memset);
//   2. coef: one workgroup sums the slots (fixed order: deterministic) and stores
//      coef = s min(1, max_norm / (s ||g|| + 1e-6)) with s = grad_scale (1 / world for the
//      summed all-reduce buckets: the mean is never materialised as a separate pass);
//   3. update, per chunk:
//        g' = coef g;  m = first ? g' : mom m + (1 - damp) g';  u = nesterov ? g' + mom m : m
//        p = p * decay - lr u      (decay = 1 - wd lr / initial_lr, 1 for the no-decay group)
//        ema = a ema + (1 - a) p   (only with an EMA table: the new p is in registers already)
//      with the products rounded in the same order as the torch foreach sequence.
// lr / decay come from the kernel arguments or, for HIP-graph replays (trainer.py), from a
// device array the host refreshes before each replay.
// The tensor table (pointers, sizes, parameter group) travels in the kernel arguments, up to
// kBatch tensors per launch (no device-side table to keep in sync with the autograd-owned
// gradient buffers, and graph capture sees plain kernel nodes).
#include <vector>

#include "hvk_common.h"

namespace {

constexpr int kChunk = 16384;  // elements per workgroup
constexpr int kThreads = 256;
constexpr int kMaxGroups = 4;
constexpr int kBatch = 64;  // 48-B entries: the table stays well inside the kernel-argument limit

struct Entry {  // one parameter tensor
  float* p;
  const float* g;
  float* m;
  float* ema;  // nullptr: no EMA this step
  int n;
  int chunk0;  // first chunk of the tensor (within its batch)
  int group;   // parameter group; bit 8: pointers 16-B aligned and n % 4 == 0
};

struct Batch {
  Entry e[kBatch];
  int nt;
  int part0;  // first workspace slot of the batch
};

struct Groups {
  float lr[kMaxGroups];
  float decay[kMaxGroups];
};

__device__ __forceinline__ int find_entry(const Entry* t, int n, int chunk) {
  int lo = 0, hi = n - 1;  // last entry with chunk0 <= chunk
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].chunk0 <= chunk)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) s += red[i];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(kThreads) void sumsq_kernel(Batch b, float* __restrict__ part) {
  __shared__ float red[kThreads / 64];
  const Entry e = b.e[find_entry(b.e, b.nt, blockIdx.x)];
  const long long c0 = (long long)(blockIdx.x - e.chunk0) * kChunk;
  const long long c1 = c0 + kChunk < e.n ? c0 + kChunk : e.n;
  float s = 0.f;
  if (e.group & 256) {
    const float4* g4 = reinterpret_cast<const float4*>(e.g);
#pragma unroll 4
    for (long long i = c0 / 4 + threadIdx.x; i < c1 / 4; i += kThreads) {
      const float4 v = g4[i];
      s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
    }
  } else {
    for (long long i = c0 + threadIdx.x; i < c1; i += kThreads) s = fmaf(e.g[i], e.g[i], s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[b.part0 + blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void coef_kernel(float* __restrict__ part, int nparts,
                                                       float max_norm, float gscale) {
  __shared__ float red[kThreads / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += kThreads) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[nparts] = gscale * fminf(1.f, max_norm / (gscale * sqrtf(s) + 1e-6f));
}

__device__ __forceinline__ void sgdw1(float& p, float& m, float g, float coef, float mom, float damp,
                                      bool nesterov, bool first, float decay, float lr) {
  const float gc = g * coef;
  const float mv = first ? gc : fmaf(1.f - damp, gc, __fmul_rn(m, mom));
  m = mv;
  const float u = nesterov ? fmaf(mom, mv, gc) : mv;
  p = fmaf(-lr, u, __fmul_rn(p, decay));
}

__device__ __forceinline__ void ema1(float& e, float p, float a) {
  e = fmaf(1.f - a, p, __fmul_rn(e, a));
}

__global__ __launch_bounds__(kThreads) void sgdw_kernel(Batch b, const float* __restrict__ coefp,
                                                       float coef_host, Groups grp,
                                                       const float* __restrict__ hyper, float mom,
                                                       float damp, int nesterov, int first,
                                                       float ema_a) {
  const Entry e = b.e[find_entry(b.e, b.nt, blockIdx.x)];
  const float coef = coefp ? *coefp : coef_host;
  const int gi = e.group & 255;
  const float decay = hyper ? hyper[kMaxGroups + gi] : grp.decay[gi];
  const float lr = hyper ? hyper[gi] : grp.lr[gi];
  const long long c0 = (long long)(blockIdx.x - e.chunk0) * kChunk;
  const long long c1 = c0 + kChunk < e.n ? c0 + kChunk : e.n;
  const bool nes = nesterov != 0, fst = first != 0;
  if (e.group & 256) {
    float4* p4 = reinterpret_cast<float4*>(e.p);
    float4* m4 = reinterpret_cast<float4*>(e.m);
    const float4* g4 = reinterpret_cast<const float4*>(e.g);
#pragma unroll 2
    for (long long i = c0 / 4 + threadIdx.x; i < c1 / 4; i += kThreads) {
      float4 p = p4[i], m = fst ? make_float4(0.f, 0.f, 0.f, 0.f) : m4[i];
      const float4 g = g4[i];
      sgdw1(p.x, m.x, g.x, coef, mom, damp, nes, fst, decay, lr);
      sgdw1(p.y, m.y, g.y, coef, mom, damp, nes, fst, decay, lr);
      sgdw1(p.z, m.z, g.z, coef, mom, damp, nes, fst, decay, lr);
      sgdw1(p.w, m.w, g.w, coef, mom, damp, nes, fst, decay, lr);
      p4[i] = p;
      m4[i] = m;
      if (e.ema) {
        float4* e4 = reinterpret_cast<float4*>(e.ema);
        float4 q = e4[i];
        ema1(q.x, p.x, ema_a); ema1(q.y, p.y, ema_a); ema1(q.z, p.z, ema_a); ema1(q.w, p.w, ema_a);
        e4[i] = q;
      }
    }
  } else {
    for (long long i = c0 + threadIdx.x; i < c1; i += kThreads) {
      float p = e.p[i], m = fst ? 0.f : e.m[i];
      sgdw1(p, m, e.g[i], coef, mom, damp, nes, fst, decay, lr);
      e.p[i] = p;
      e.m[i] = m;
      if (e.ema) ema1(e.ema[i], p, ema_a);
    }
  }
}

int chunks_of(long long n) { return (int)((n + kChunk - 1) / kChunk); }

}  // namespace

extern "C" {

size_t hvk_sgdw_workspace_bytes(int n, const long long* numel) {
  size_t parts = 0;
  for (int i = 0; i < n; ++i) parts += (size_t)chunks_of(numel[i]);
  return (parts + 1) * sizeof(float);  // chunk slots + the clip coefficient
}

int hvk_sgdw_step(int n, float* const* p, const float* const* g, float* const* m,
                  float* const* ema, const long long* numel, const int* group, const float* lr,
                  const float* decay, int ngroups, const float* hyper, float grad_scale,
                  float max_norm, float momentum, float dampening, int nesterov, int first,
                  float ema_smoothing, float* workspace, size_t ws_bytes, void* stream) {
  if (n <= 0) return HVK_OK;
  if (!p || !g || !m || !numel || !group || !lr || !decay || !workspace)
    return hvk_set_error(HVK_EINVAL, "hvk_sgdw_step: null argument");
  if (!(grad_scale > 0.f))
    return hvk_set_error(HVK_EINVAL, "hvk_sgdw_step: grad_scale %g", (double)grad_scale);
  if (ngroups < 1 || ngroups > kMaxGroups)
    return hvk_set_error(HVK_EINVAL, "hvk_sgdw_step: %d parameter groups (max %d)", ngroups, kMaxGroups);
  if (ws_bytes < hvk_sgdw_workspace_bytes(n, numel))
    return hvk_set_error(HVK_EINVAL, "hvk_sgdw_step: workspace %zu B too small", ws_bytes);
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<Batch> batches((n + kBatch - 1) / kBatch);
  int part = 0;
  for (size_t bi = 0; bi < batches.size(); ++bi) {
    Batch& b = batches[bi];
    b.nt = n - (int)bi * kBatch < kBatch ? n - (int)bi * kBatch : kBatch;
    b.part0 = part;
    int ch = 0;
    for (int i = 0; i < b.nt; ++i) {
      const int k = (int)bi * kBatch + i;
      float* ek = ema ? ema[k] : nullptr;
      if (!p[k] || !g[k] || !m[k] || (ema && !ek) || numel[k] <= 0 || numel[k] > (1ll << 30) ||
          group[k] < 0 || group[k] >= ngroups)
        return hvk_set_error(HVK_EINVAL, "hvk_sgdw_step: tensor %d invalid", k);
      const bool v4 = ((reinterpret_cast<size_t>(p[k]) | reinterpret_cast<size_t>(g[k]) |
                        reinterpret_cast<size_t>(m[k]) | reinterpret_cast<size_t>(ek)) % 16 == 0) &&
                      numel[k] % 4 == 0;
      b.e[i] = Entry{p[k], g[k], m[k], ek, (int)numel[k], ch, group[k] | (v4 ? 256 : 0)};
      ch += chunks_of(numel[k]);
    }
    part += ch;
  }
  Groups gp;
  for (int i = 0; i < kMaxGroups; ++i) {
    gp.lr[i] = i < ngroups ? lr[i] : 0.f;
    gp.decay[i] = i < ngroups ? decay[i] : 1.f;
  }
  auto nch = [](const Batch& b) { return b.e[b.nt - 1].chunk0 + chunks_of(b.e[b.nt - 1].n); };
  const float* coefp = nullptr;
  if (max_norm > 0.f) {
    for (const Batch& b : batches) {
      hipLaunchKernelGGL(sumsq_kernel, dim3(nch(b)), dim3(kThreads), 0, st, b, workspace);
      HVK_CHECK_LAUNCH("hvk_sgdw_step (norm)");
    }
    hipLaunchKernelGGL(coef_kernel, dim3(1), dim3(kThreads), 0, st, workspace, part, max_norm,
                       grad_scale);
    HVK_CHECK_LAUNCH("hvk_sgdw_step (coef)");
    coefp = workspace + part;
  }
  for (const Batch& b : batches) {
    hipLaunchKernelGGL(sgdw_kernel, dim3(nch(b)), dim3(kThreads), 0, st, b, coefp, grad_scale, gp,
                       hyper, momentum, dampening, nesterov, first, ema_smoothing);
    HVK_CHECK_LAUNCH("hvk_sgdw_step");
  }
  return HVK_OK;
}

}  // extern "C"
