// The classifier head's GEMMs (swinv2.py:786-794 `self.head`, the multitask tiers of
// hierarchy.py:19-47): M = the batch (hundreds of rows), K = the feature width, N = the class
// count (10 000 leaves for iNat21 HXE) -- a shape none of the token GEMMs has: M is too short
// for the 128-row tiles and the class count is not a tile multiple.
//
//   forward        y[M, N]  = bf16(x[M, K] w[N, K]^T + bias)             (F.linear)
//   input grad     gx[M, K] = g[M, N] w[N, K]            (f32; split over N, then summed)
//   weight grad    dw[N, K] = g^T x, db[N] = sum_m g[m, :] (f32)
//
// One kernel form: C[i][j] = sum_c A(i, c) B(j, c) on 64 x 64 output tiles (four waves, 32 x 32
// each, 16x16x32 bf16 MFMA), the contraction staged through registers and LDS 64 at a time (the
// next block's global reads in flight under the current block's MFMAs).  An operand whose
// contraction index is not the contiguous one (w in the input gradient, both in the weight
// gradient) is transposed on its way into LDS (8 two-byte LDS writes per 16-B global read), so
// every fragment read is one ds_read_b128.  Ragged edges: 8-element chunks past a bound load as
// zero, stores past M / N are dropped -- N and K must be multiples of 8 (hvk_head_supported).
#include "hvk_common.h"

namespace {

constexpr int HB = 64;       // output tile rows / columns and contraction chunk
constexpr int HLD = HB + 8;  // LDS row stride (bf16): rows 16 B apart in bank space

// One [HB x HB] block (rows r0.., contraction c0..) of a logical operand L, staged through
// registers into LDS as lds[r][c] (stride HLD).  T = false: L(r, c) = g[r * ld + c]; T = true:
// L(r, c) = g[c * ld + r].  R / CE bound r / c; the contiguous index of g comes in whole
// 8-element chunks.  load() issues the thread's two 16-B global reads, store() writes them
// (transposed: 8 two-byte LDS writes per read) -- split so the next block's reads are in flight
// while the current block's MFMAs run.
template <bool T>
struct Stager {
  uint4 v[2];
  __device__ __forceinline__ void load(const hvk_bf16* __restrict__ g, int ld, int r0, int c0, int R, int CE) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = threadIdx.x + 256 * k;
      const int a = e >> 3, b = (e & 7) * 8;  // a: the strided index, b: 8 contiguous ones
      v[k] = make_uint4(0, 0, 0, 0);
      if constexpr (!T) {
        const int r = r0 + a, c = c0 + b;
        if (r < R && c < CE) v[k] = hvk_ld16(g + (size_t)r * ld + c);
      } else {
        const int c = c0 + a, r = r0 + b;
        if (c < CE && r < R) v[k] = hvk_ld16(g + (size_t)c * ld + r);
      }
    }
  }
  __device__ __forceinline__ void store(hvk_bf16* lds) const {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = threadIdx.x + 256 * k;
      const int a = e >> 3, b = (e & 7) * 8;
      if constexpr (!T) {
        *reinterpret_cast<uint4*>(lds + a * HLD + b) = v[k];
      } else {
        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          lds[(b + 2 * q) * HLD + a] = (hvk_bf16)(w[q] & 0xffff);
          lds[(b + 2 * q + 1) * HLD + a] = (hvk_bf16)(w[q] >> 16);
        }
      }
    }
  }
};

// EPI 0: bf16 out[j][i] = C + bias[i] (the forward, i = class, j = row of the batch);
// EPI 1: f32 out[z][j][i] = C over contraction slice z (input-gradient partials, weight gradient);
// DB: also db[j] = sum_c B(j, c) (the weight gradient's bias gradient, from the staged g^T).
template <bool AT, bool BT, int EPI, bool DB>
__global__ __launch_bounds__(256) void head_kernel(const hvk_bf16* __restrict__ A, int lda,
                                                   const hvk_bf16* __restrict__ B, int ldb, int I, int J,
                                                   int CT, int cslice, void* __restrict__ out, int ldo,
                                                   const float* __restrict__ bias, float* __restrict__ db) {
  __shared__ __attribute__((aligned(16))) hvk_bf16 As[HB * HLD];
  __shared__ __attribute__((aligned(16))) hvk_bf16 Bs[HB * HLD];
  const int i0 = blockIdx.x * HB, j0 = blockIdx.y * HB;
  const int cb = blockIdx.z * cslice;
  const int ce = cb + cslice < CT ? cb + cslice : CT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int wi = wave & 1, wj = wave >> 1;
  hvk_f32x4 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[t][u] = hvk_f32x4{0, 0, 0, 0};
  float dbs = 0.f;
  Stager<AT> sa;
  Stager<BT> sb;
  if (cb < ce) {
    sa.load(A, lda, i0, cb, I, ce);
    sb.load(B, ldb, j0, cb, J, ce);
  }
  for (int c0 = cb; c0 < ce; c0 += HB) {
    sa.store(As);
    sb.store(Bs);
    __syncthreads();
    if (c0 + HB < ce) {  // the next block's reads, in flight under this block's MFMAs
      sa.load(A, lda, i0, c0 + HB, I, ce);
      sb.load(B, ldb, j0, c0 + HB, J, ce);
    }
    if (DB && blockIdx.x == 0 && threadIdx.x < HB) {
#pragma unroll 8
      for (int c = 0; c < HB; ++c) dbs += __uint_as_float((uint32_t)Bs[threadIdx.x * HLD + c] << 16);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = *reinterpret_cast<const uint4*>(As + (32 * wi + 16 * t + li) * HLD + 32 * ks + 8 * gq);
        b[t] = *reinterpret_cast<const uint4*>(Bs + (32 * wj + 16 * t + li) * HLD + 32 * ks + 8 * gq);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[t][u] = hvk_mfma16(a[t], b[u], acc[t][u]);
    }
    __syncthreads();
  }
  if (DB && blockIdx.x == 0 && threadIdx.x < HB && j0 + threadIdx.x < J) db[j0 + threadIdx.x] = dbs;
  // lane (li, gq), element r of acc[t][u] = C[i0 + 32 wi + 16 t + 4 gq + r][j0 + 32 wj + 16 u + li]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + 32 * wi + 16 * t + 4 * gq, j = j0 + 32 * wj + 16 * u + li;
      if (i >= I || j >= J) continue;  // I % 8 == 0: i .. i + 3 all inside or all outside
      if constexpr (EPI == 0) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[t][u][r] + (bias ? bias[i + r] : 0.f);
        *reinterpret_cast<uint2*>(static_cast<hvk_bf16*>(out) + (size_t)j * ldo + i) =
            make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
      } else {
        float* o = static_cast<float*>(out) + ((size_t)blockIdx.z * J + j) * ldo + i;
        *reinterpret_cast<float4*>(o) = make_float4(acc[t][u][0], acc[t][u][1], acc[t][u][2], acc[t][u][3]);
      }
    }
}

// gx[e] = sum_z part[z][e]
__global__ __launch_bounds__(256) void head_sum_kernel(const float4* __restrict__ part, float4* __restrict__ gx,
                                                       int n4, int Z) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n4; e += gridDim.x * 256) {
    float4 s = part[e];
    for (int z = 1; z < Z; ++z) {
      const float4 p = part[(size_t)z * n4 + e];
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
    gx[e] = s;
  }
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// the input gradient's split of the class dimension: about 768 workgroups, slices of whole chunks
inline void dgrad_split(int M, int K, int N, int& Z, int& slice) {
  const int tiles = cdiv(K, HB) * cdiv(M, HB);
  const int chunks = cdiv(N, HB);
  Z = cdiv(768, tiles);
  if (Z > chunks) Z = chunks;
  if (Z < 1) Z = 1;
  slice = cdiv(chunks, Z) * HB;
  Z = cdiv(N, slice);
}

}  // namespace

extern "C" {

int hvk_head_supported(int M, int K, int N) {
  return M > 0 && K > 0 && N > 0 && K % 8 == 0 && N % 8 == 0 && (long long)M * N < (1ll << 31) &&
         (long long)N * K < (1ll << 31);
}

size_t hvk_head_bwd_workspace_bytes(int M, int K, int N) {
  if (!hvk_head_supported(M, K, N)) return 0;
  int Z, slice;
  dgrad_split(M, K, N, Z, slice);
  return Z > 1 ? (size_t)Z * M * K * sizeof(float) : 0;
}

int hvk_head_fwd(const void* x, const void* w, const float* bias, void* y, int M, int K, int N, void* stream) {
  if (!x || !w || !y) return hvk_set_error(HVK_EINVAL, "hvk_head_fwd: null pointer");
  if (!hvk_head_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_head_fwd: M=%d K=%d N=%d (K, N multiples of 8)", M, K, N);
  hipLaunchKernelGGL((head_kernel<false, false, 0, false>), dim3(cdiv(N, HB), cdiv(M, HB), 1), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const hvk_bf16*>(w), K,
                     static_cast<const hvk_bf16*>(x), K, N, M, K, K, y, N, bias, nullptr);
  HVK_CHECK_LAUNCH("head_fwd");
  return HVK_OK;
}

int hvk_head_bwd(const void* g, const void* x, const void* w, float* gx, float* dw, float* db, int M, int K,
                 int N, float* workspace, size_t workspace_bytes, void* stream) {
  if (!g || (gx && !w) || (dw && !x) || (db && !dw))
    return hvk_set_error(HVK_EINVAL, "hvk_head_bwd: null pointer");
  if (!hvk_head_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_head_bwd: M=%d K=%d N=%d (K, N multiples of 8)", M, K, N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hvk_bf16* G = static_cast<const hvk_bf16*>(g);
  if (gx) {
    int Z, slice;
    dgrad_split(M, K, N, Z, slice);
    if (Z > 1 && (!workspace || workspace_bytes < (size_t)Z * M * K * sizeof(float)))
      return hvk_set_error(HVK_EINVAL, "hvk_head_bwd: workspace too small");
    // C[k][m] = sum_n w[n][k] g[m][n]: A = w^T (staged transposed), B = g
    hipLaunchKernelGGL((head_kernel<true, false, 1, false>), dim3(cdiv(K, HB), cdiv(M, HB), Z), dim3(256), 0, st,
                       static_cast<const hvk_bf16*>(w), K, G, N, K, M, N, slice, Z > 1 ? (void*)workspace : (void*)gx,
                       K, nullptr, nullptr);
    HVK_CHECK_LAUNCH("head_dgrad");
    if (Z > 1) {
      const int n4 = M * K / 4;
      int blocks = cdiv(n4, 256);
      if (blocks > 1024) blocks = 1024;
      hipLaunchKernelGGL(head_sum_kernel, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const float4*>(workspace),
                         reinterpret_cast<float4*>(gx), n4, Z);
      HVK_CHECK_LAUNCH("head_dgrad_sum");
    }
  }
  if (dw) {
    // C[k][n] = sum_m x[m][k] g[m][n]: A = x^T, B = g^T (both staged transposed)
    const hvk_bf16* X = static_cast<const hvk_bf16*>(x);
    if (db)
      hipLaunchKernelGGL((head_kernel<true, true, 1, true>), dim3(cdiv(K, HB), cdiv(N, HB), 1), dim3(256), 0, st, X, K,
                         G, N, K, N, M, M, dw, K, nullptr, db);
    else
      hipLaunchKernelGGL((head_kernel<true, true, 1, false>), dim3(cdiv(K, HB), cdiv(N, HB), 1), dim3(256), 0, st, X,
                         K, G, N, K, N, M, M, dw, K, nullptr, nullptr);
    HVK_CHECK_LAUNCH("head_wgrad");
  }
  return HVK_OK;
}

}  // extern "C"
