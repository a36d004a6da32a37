// Skinny MFMA GEMM for the memory-bound SwinV2 Linear layers on gfx950:
//   Y[M, N] = X[M, K] W[N, K]^T (+ bias[N])      (nn.Linear / F.linear layout)
// used for the forward (W = weight) and the input gradient (W = weight^T) of qkv / proj /
// fc1 / fc2 / PatchMerging.reduction / PatchEmbed at the stages where K and N are small
// (SwinV2-T stage 0-1: M = 200k-800k tokens, K, N <= 384).  Replaces F.linear of
// swinv2.py:58-62, 220, 262, 492, 652 (as GEMM) for those shapes.
//
// These GEMMs are HBM-bound (arithmetic intensity K N / (K + N) <= 100 flop/B against a
// machine balance of ~400), so the design streams X once and keeps W on chip:
//  * a workgroup stages a BN x K block of W in LDS once and keeps it for its whole
//    (persistent) life; the A operand of every MFMA is a W fragment read from LDS in a
//    fragment-contiguous layout (one 1-KB conflict-free ds_read_b128 per MFMA);
//  * Y^T = W X^T: the B operand is a 16-row tile of X read straight from HBM (16 B per
//    lane), so X bytes are touched exactly once and no X staging is needed; the next
//    tile's loads are issued before the current tile's MFMAs (software prefetch);
//  * W rows are stored in LDS in a permuted order so that every lane ends up holding 8
//    consecutive output columns of one row: each output row segment leaves as one 16-B
//    store, bias added on the way (f32, from LDS).
// v_mfma_f32_16x16x32_bf16, f32 accumulation, bf16 output (as F.linear under autocast).
#include <stdlib.h>

#include "hvk_common.h"
#include "gemm_tile_ln.h"

namespace {

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}

template <int K, int BN>
struct GCfg {
  static_assert(K % 16 == 0 && BN % 32 == 0, "K multiple of 16, BN multiple of 32");
  static constexpr int KS = (K + 31) / 32;   // MFMA k-steps (last one half-empty if K%32 == 16)
  static constexpr int U4 = KS * 4;          // 16-B units per staged W row (zero padded)
  static constexpr int NT = BN / 16;         // output-column tiles per workgroup
  static constexpr size_t LDS = (size_t)BN * U4 * 16 + (size_t)BN * 4;  // W block + bias
};

// LDS row p (= MFMA A row m = p%16 of tile t = p/16) holds W row n = perm(p): for the tile
// pair (2j, 2j+1), A rows 4g + r of tile 2j + e hold n = 32j + 8g + 4e + r.  The MFMA
// result D[4g + r][li] of tiles 2j, 2j+1 then gives lane (li, g) columns 32j + 8g .. +7.
__device__ __forceinline__ int perm_row(int p) {
  const int t = p >> 4, m = p & 15;
  return 32 * (t >> 1) + 8 * (m >> 2) + 4 * (t & 1) + (m & 3);
}

#ifndef HVK_LIN_PAIRSTORE  // 1: output slices stored in row pairs as whole 128-B lines (A/B switch)
#define HVK_LIN_PAIRSTORE 1
#endif
// Full-line output stores: lane (li, g) holds columns 32j + 8g .. +7 of row li for every slice j,
// so a plain store writes 16 rows x 64 B (16 half lines).  For a slice pair (j, j+1), rows li and
// li ^ 8 swap halves (one DPP row_ror:8 per dword): lanes li < 8 then hold (row li, j) and
// (row li + 8, j), lanes li >= 8 (row li - 8, j+1) and (row li, j+1) -- two stores of 8 rows x
// 128 B each, every line written whole by one instruction.

// ---- post-norm LayerNorm + residual epilogue (EPI 5 of linear_kernel, mlp_fwd_kernel<LN>) --------
// The res-post-norm `x = x0 + drop_path(norm(a))` of swinv2.py:431 / 434 (and the plain norm of
// PatchEmbed, 656, with no x0) applied to the GEMM's bf16 output a where ONE workgroup holds whole
// C = 96 rows (stage 0): a is still stored (the LayerNorm backward reads it), but the separate
// LayerNorm launch -- its re-read of a and its own pass over the rows -- disappears.  Per 16-row
// tile a wave hands its rows through a 768-B LDS staging buffer, four rows at a time, into
// ln_fwd_kernel<8, 16>'s lane layout (layernorm.hip: 16 lanes per row, channel groups of 4 at
// 4 (16 i + t)) and runs that kernel's arithmetic on it, so x, xb, mean and rstd are bit-identical
// to the two-launch path (tests/test_gpu_linear_ln.py).
// LnEpi (hvk_common.h): the norm's parameters and outputs
#ifndef HVK_LN96_U  // norm passes (4 rows each) staged and reduced together (A/B build switch: 1, 2)
#define HVK_LN96_U 2
#endif
namespace ln96 {
// U passes of 4 rows share one staging write / wait / read round and run their row reductions as
// independent chains (one pass at a time serialised each pass's LDS round trip and shuffles);
// U = 2 keeps the fused MLP kernel inside one CU's LDS (162 816 of 163 840 B)
constexpr int U = HVK_LN96_U;
constexpr int C = 96, TPR = 16, NG = 2, EPT = 8, STAGE_BYTES = U * 4 * C * 2;
constexpr int PARAM_BYTES = 3 * C * 4;
// gamma, beta, abias as a [3][96] f32 table in LDS (one copy per workgroup, written before the
// workgroup's first barrier), read per pass instead of pinning 24 VGPRs per lane
struct Params {
  uint32_t lds;  // LDS byte address of the table
};
__device__ __forceinline__ bool grp_ok(int t, int i) { return 4 * (i * TPR + t) < C; }
__device__ __forceinline__ void load_params(const LnEpi& p, float* tab) {
  for (int e = threadIdx.x; e < 3 * C; e += blockDim.x) {
    const int k = e / C, c = e - k * C;
    tab[e] = k == 0 ? p.gamma[c] : (k == 1 ? p.beta[c] : (p.abias ? p.abias[c] : 0.f));
  }
}
__device__ __forceinline__ float4 param4(const Params& q, int k, int c) {
  const hvk_f32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) hvk_f32x4*>(
      (const __attribute__((address_space(3))) char*)(size_t)(q.lds + (k * C + c) * 4));
  return make_float4(v[0], v[1], v[2], v[3]);
}
// the residual rows of a 16-row tile in the norm's layout (pass pp: rows 4 pp + lane / 16), one
// tile ahead of their use; rows past M and absent x0 read 0 (buffer view, no branch)
__device__ __forceinline__ void load_x0(const LnEpi& p, int row0, int M, uint4 (&x0v)[4][NG]) {
  const int t = threadIdx.x & (TPR - 1), sub = (threadIdx.x & 63) / TPR;
  const auto r = hvk_tile_rsrc(p.x0, row0, p.x0 ? M : 0, C * 4);
#pragma unroll
  for (int pp = 0; pp < 4; ++pp)
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int c = 4 * (i * TPR + t);
      x0v[pp][i] = hvk_bld16(r, grp_ok(t, i) ? (uint32_t)((4 * pp + sub) * C + c) * 4 : HVK_OOB);
    }
}
// av[j]: this lane's packed a of row li, columns 32 j + 8 g .. +7 (the skinny kernels' layout)
__device__ __forceinline__ void tile(const LnEpi& p, const Params& q, uint32_t stage, const uint4 (&av)[3],
                                     const uint4 (&x0v)[4][NG], int row0, int M) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int t = lane & (TPR - 1), sub = lane / TPR;
  const float invC = 1.f / C;
#pragma unroll
  for (int p0 = 0; p0 < 4; p0 += U) {
    // rows 4 p0 .. 4 (p0 + U) - 1 of the tile into the staging buffer (row 4 u + k at u * 768 + k * 192)
    if ((li >> 2) >= p0 && (li >> 2) < p0 + U) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
        *reinterpret_cast<__attribute__((address_space(3))) hvk_u32x4*>((__attribute__((address_space(3))) char*)(size_t)(stage + (li - 4 * p0) * C * 2 + (32 * j + 8 * g) * 2)) =
            __builtin_bit_cast(hvk_u32x4, av[j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float v[U][EPT], s[U], mu[U], ss[U], rs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s[u] = 0.f;
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        if (grp_ok(t, i)) {
          const int c = 4 * (i * TPR + t);
          const hvk_u32x2 w = *reinterpret_cast<const __attribute__((address_space(3))) hvk_u32x2*>(
              (const __attribute__((address_space(3))) char*)(size_t)(stage + (4 * u + sub) * C * 2 + c * 2));
          v[u][4 * i] = hvk_lo(w[0]); v[u][4 * i + 1] = hvk_hi(w[0]); v[u][4 * i + 2] = hvk_lo(w[1]); v[u][4 * i + 3] = hvk_hi(w[1]);
          const float4 ab = param4(q, 2, c);
          const float abv[4] = {ab.x, ab.y, ab.z, ab.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[u][4 * i + j] += abv[j]; s[u] += v[u][4 * i + j]; }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[u][4 * i + j] = 0.f;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the staging reads are back before the next round's writes
#pragma unroll
    for (int u = 0; u < U; ++u) mu[u] = hvk_xor_sum<TPR>(s[u]) * invC;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ss[u] = 0.f;
#pragma unroll
      for (int i = 0; i < NG; ++i)
        if (grp_ok(t, i)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) ss[u] = hvk_ln_sq(ss[u], v[u][4 * i + j] - mu[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) rs[u] = hvk_ln_rstd(hvk_xor_sum<TPR>(ss[u]), invC, p.eps);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pp = p0 + u;
      const int row = row0 + 4 * pp + sub;
      if (row >= M) continue;
      const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
      const size_t rb = (size_t)row * C;
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        if (!grp_ok(t, i)) continue;
        const int c = 4 * (i * TPR + t);
        float r[4] = {__uint_as_float(x0v[pp][i].x), __uint_as_float(x0v[pp][i].y), __uint_as_float(x0v[pp][i].z),
                      __uint_as_float(x0v[pp][i].w)};
        const float4 g4 = param4(q, 0, c), b4 = param4(q, 1, c);
        const float gm[4] = {g4.x, g4.y, g4.z, g4.w}, bt[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = hvk_ln_out(r[j], v[u][4 * i + j], mu[u], rs[u], gm[j], bt[j], sc);
        const uint4 xr = make_uint4(__float_as_uint(r[0]), __float_as_uint(r[1]), __float_as_uint(r[2]), __float_as_uint(r[3]));
        if (HVK_NT_SAVED & 2) hvk_st16_nt(p.x + rb + c, xr);  // read again only at the next LayerNorm
        else *reinterpret_cast<uint4*>(p.x + rb + c) = xr;
        if (p.xb) *reinterpret_cast<uint2*>(p.xb + rb + c) = make_uint2(hvk_pack2(r[0], r[1]), hvk_pack2(r[2], r[3]));
      }
      if (t == 0) {
        p.mean[row] = mu[u];
        p.rstd[row] = rs[u];
      }
    }
  }
}
}  // namespace ln96

// EPI 0: Y = acc (+ bias).  EPI 1 (fc1): Y = h = bf16(acc + bias) and Y2 = GELU(h), the
// bf16 pre-activation kept for the backward and the activation for fc2 (the reference's
// F.linear(+bias) -> nn.GELU on the bf16 tensor, swinv2.py:58-62).
// EPI 3 (fc2 forward on the saved pre-activation): Y = GELU(X) W^T (+ bias), the GELU of
// each loaded X fragment recomputed and rounded to bf16 exactly as EPI 1 stores it.
// EPI 2 (fc2 input gradient through the activation): Y = gh = bf16(acc * GELU'(h)) with h
// read from Y2 (the saved fc1 pre-activation), and csum[n] += sum over rows of gh (the fc1
// bias gradient): per-lane register sums over the workgroup's row tiles, one 16-lane
// shuffle reduction and one atomic per column and wave at the end.
// EPI 4 (the qkv Linear of a w <= 8 W-MSA block): EPI 0 with every q and k head slice (columns
// < 2N/3) normalised (hvk_head_normalize8, F.normalize of swinv2.py:229) and its
// 1 / max(||x||, eps) stored to rn [M, 2N/96] (passed in csum).
// EPI 5 (C = 96, one column block): Y = a = bf16(acc) and the post-norm LayerNorm + residual of
// a (LnEpi, above) in the same pass.
template <int K, int BN, int WAVES, bool PREF, bool BIAS, int EPI = 0>
__global__ __launch_bounds__(64 * WAVES) void linear_kernel(const hvk_bf16* __restrict__ X,
                                                          const hvk_bf16* __restrict__ W,
                                                          const float* __restrict__ bias,
                                                          hvk_bf16* __restrict__ Y,
                                                          hvk_bf16* __restrict__ Y2, int M, int N,
                                                          int ncb, int row_groups,
                                                          float* __restrict__ csum = nullptr,
                                                          const float* __restrict__ qscale = nullptr,
                                                          LnEpi ln = LnEpi{}) {
  using G = GCfg<K, BN>;
  static_assert(EPI != 5 || BN == 96, "the LayerNorm epilogue holds whole C = 96 rows");
  constexpr int kThreads = 64 * WAVES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* wl = reinterpret_cast<uint4*>(smem);                                // [NT][U4][16]
  float* bl = reinterpret_cast<float*>(smem + (size_t)BN * G::U4 * 16);     // [BN]
  // XCD-aware decode: the ncb column blocks of one row group share an XCD (L2) and walk
  // the same row tiles in the same order
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int cb = loc % ncb, rg = (loc / ncb) * 8 + xcd;
  if (rg >= row_groups) return;
  const int n0 = cb * BN;

  // stage W[n0 .. n0+BN) in the permuted, fragment-contiguous layout
  for (int e = threadIdx.x; e < BN * G::U4; e += kThreads) {
    const int p = e / G::U4, u = e % G::U4;
    const int n = n0 + perm_row(p);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (8 * u < K) v = *reinterpret_cast<const uint4*>(W + (size_t)n * K + 8 * u);
    wl[((p >> 4) * G::U4 + u) * 16 + (p & 15)] = v;
  }
  if (BIAS)
    for (int e = threadIdx.x; e < BN; e += kThreads) bl[e] = bias[n0 + e];
  if constexpr (EPI == 5)
    ln96::load_params(ln, reinterpret_cast<float*>(smem + G::LDS + WAVES * ln96::STAGE_BYTES));
  __syncthreads();

  // wave-uniform tile index: every global access goes through a buffer view of its 16-row
  // tile clipped at M (hvk_tile_rsrc), so rows past M need no exec branch -- a load or store
  // under a branch made the compiler's vmcnt accounting conservative: it waited vmcnt(0) at
  // every tile's MFMAs, for the tile-ahead prefetch and every store in flight
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int tiles = (M + 15) >> 4;
  const int stride = row_groups * WAVES;
  int tile = rg * WAVES + wave;

  auto load_x = [&](int t, uint4 (&xf)[G::KS]) {
    const auto rx = hvk_tile_rsrc(X, 16 * t, M, K * 2);
    const uint32_t o = (uint32_t)(li * K + 8 * g) * 2;
#pragma unroll
    for (int s = 0; s < G::KS; ++s) {
      const bool in_k = (K % 32 == 0) || s + 1 < G::KS || g < 2;
      xf[s] = hvk_bld16(rx, in_k ? o + 64 * s : HVK_OOB);
    }
  };

  // EPI 2: the saved pre-activation of the row tile, prefetched one tile ahead like X
  auto load_h = [&](int t, uint4 (&hf)[EPI == 2 ? G::NT / 2 : 1]) {
    if (EPI != 2) return;
    const auto rh = hvk_tile_rsrc(Y2, 16 * t, M, N * 2);
    const uint32_t o = (uint32_t)(li * N + n0 + 8 * g) * 2;
#pragma unroll
    for (int j = 0; j < G::NT / 2; ++j)
      hf[j] = (HVK_NT_SAVED & 8) ? hvk_bld16_nt(rh, o + 64 * j) : hvk_bld16(rh, o + 64 * j);
  };
  uint4 xf[G::KS];
  load_x(tile, xf);
  uint4 hf[EPI == 2 ? G::NT / 2 : 1];
  load_h(tile, hf);
  // EPI 5: the norm's parameters (its lane layout), and the residual rows one tile ahead like X
  const uint32_t lstage = lds_addr(smem) + (uint32_t)G::LDS + (uint32_t)wave * ln96::STAGE_BYTES;
  const ln96::Params lnq{lds_addr(smem) + (uint32_t)G::LDS + (uint32_t)WAVES * ln96::STAGE_BYTES};
  // the first tile's operands land before the loop (the loop header's wait then serves only
  // the back edge, counted, instead of vmcnt(0) on every iteration)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < G::KS; ++s) hvk_launder(xf[s]);
  if (EPI == 2)
#pragma unroll
    for (int j = 0; j < (EPI == 2 ? G::NT / 2 : 1); ++j) hvk_launder(hf[j]);
  float cs[EPI == 2 ? G::NT / 2 : 1][8];
  if (EPI == 2)
#pragma unroll
    for (int j = 0; j < G::NT / 2; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[j][e] = 0.f;
  for (; tile < tiles; tile += stride) {
    // W never changes, but re-read its fragments from LDS every tile: hoisting them out of
    // the loop would pin KS x NT x 4 VGPRs (and spill)
    asm volatile("" ::: "memory");
    uint4 xn[G::KS];
    if (PREF) load_x(tile + stride, xn);
    uint4 hn[EPI == 2 ? G::NT / 2 : 1];
    load_h(tile + stride, hn);
    // EPI 5: this tile's residual rows (issued here, used by the norm after the MFMAs and the a
    // stores; a tile ahead they held 32 more VGPRs: 164, 3 waves per SIMD)
    uint4 x0f[EPI == 5 ? 4 : 1][ln96::NG];
    if constexpr (EPI == 5) ln96::load_x0(ln, 16 * tile, M, x0f);
    __builtin_amdgcn_sched_barrier(0);  // the next tile's loads issue here, not after the MFMAs
    hvk_f32x4 acc[G::NT];
#pragma unroll
    for (int t = 0; t < G::NT; ++t) acc[t] = hvk_f32x4{0, 0, 0, 0};
    uint4 xg[G::KS];  // EPI 3: the operand is GELU(X) (X = the saved fc1 pre-activation h)
#pragma unroll
    for (int s = 0; s < G::KS; ++s) xg[s] = EPI == 3 ? hvk_gelu8_bf16(xf[s]) : xf[s];
#pragma unroll
    for (int s = 0; s < G::KS; ++s)
#pragma unroll
      for (int t = 0; t < G::NT; ++t)
        acc[t] = hvk_mfma16(wl[(t * G::U4 + 4 * s + g) * 16 + li], xg[s], acc[t]);
    {
      const auto ry = hvk_tile_rsrc(Y, 16 * tile, M, N * 2);
      const auto ry2 = hvk_tile_rsrc(Y2, 16 * tile, M, N * 2);
      const uint32_t yo = (uint32_t)(li * N + n0 + 8 * g) * 2;
      // pair stores: rows li & 7 (+8), the j+1 half for lanes li >= 8
      const bool lo8 = li < 8;
      const uint32_t yp = (uint32_t)((li & 7) * N + n0 + 8 * g + (lo8 ? 0 : 32)) * 2;
      uint4 pend = make_uint4(0, 0, 0, 0), pend2 = make_uint4(0, 0, 0, 0);  // slice j-1 (j odd)
      // store slice j (value v, second output v2 for EPI 1) now or as the second of a pair
      auto put = [&](int j, const uint4& v, const uint4& v2, bool nt) {
        if (!HVK_LIN_PAIRSTORE || (j % 2 == 0 && j + 1 >= G::NT / 2)) {  // unpaired last slice
          if (nt) hvk_bst16_nt(ry, yo + 64 * j, v);
          else hvk_bst16(ry, yo + 64 * j, v);
          if (EPI == 1) hvk_bst16(ry2, yo + 64 * j, v2);
          return;
        }
        if (j % 2 == 0) {
          pend = v;
          pend2 = v2;
          return;
        }
        uint4 a0, b0;
        pair_rows(pend, v, lo8, a0, b0);
        const uint32_t o = yp + 64 * (j - 1);
        if (nt) {
          hvk_bst16_nt(ry, o, a0);
          hvk_bst16_nt(ry, o + 16 * N, b0);
        } else {
          hvk_bst16(ry, o, a0);
          hvk_bst16(ry, o + 16 * N, b0);
        }
        if (EPI == 1) {
          pair_rows(pend2, v2, lo8, a0, b0);
          hvk_bst16(ry2, o, a0);
          hvk_bst16(ry2, o + 16 * N, b0);
        }
      };
      uint4 av[EPI == 5 ? G::NT / 2 : 1];   // EPI 5: the row's packed a, for the norm
      float rq[EPI == 4 ? G::NT / 2 : 1];  // EPI 4: the row's 1/||x|| per head slice
#pragma unroll
      for (int j = 0; j < (EPI == 4 ? G::NT / 2 : 1); ++j) rq[j] = 0.f;
#pragma unroll
      for (int j = 0; j < G::NT / 2; ++j) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[2 * j][r];
          v[4 + r] = acc[2 * j + 1][r];
        }
        if (EPI == 2) {
          float hv[8];
          hvk_unpack8(hf[EPI == 2 ? j : 0], hv);
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const hvk_gelu::f32x2 d = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{hv[e], hv[e + 1]});
            v[e] *= d.x;
            v[e + 1] *= d.y;
          }
          const uint4 gv = hvk_pack8(v);
          put(j, gv, gv, false);
          float r[8];
          hvk_unpack8(gv, r);  // the bias gradient sums the stored (rounded) gradient (0 past M)
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[j][e] += r[e];
          continue;
        }
        if (BIAS) {
          const float4 b0 = *reinterpret_cast<const float4*>(bl + 32 * j + 8 * g);
          const float4 b1 = *reinterpret_cast<const float4*>(bl + 32 * j + 8 * g + 4);
          v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
          v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        uint4 hv = hvk_pack8(v);
        if constexpr (EPI == 4) {
          const int qk_cols = 2 * (N / 3), col = n0 + 32 * j;
          if (col < qk_cols) {  // wave-uniform: the v column blocks skip it
            // q slices (col < N/3) as q^ * scale_h * log2e (tile_epilogue, gemm_tile.hip)
            const float post = (qscale && col < N / 3) ? qscale[col / 32] * HVK_LOG2E : 1.f;
            float r;
            hv = hvk_head_normalize8(hv, r, post);  // all 64 lanes take part in the group sums
            rq[j] = r;
          }
        }
        uint4 gl = hv;
        if (EPI == 1) {
          float u[8];
          hvk_unpack8(hv, u);  // GELU of the rounded pre-activation, as the reference
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const hvk_gelu::f32x2 y = hvk_gelu::gelu2(hvk_gelu::f32x2{u[e], u[e + 1]});
            u[e] = y.x;
            u[e + 1] = y.y;
          }
          gl = hvk_pack8(u);
        }
        if constexpr (EPI == 5) av[j] = hv;
        put(j, hv, gl, EPI == 1 && (HVK_NT_SAVED & 1));
      }
      if constexpr (EPI == 5) ln96::tile(ln, lnq, lstage, av, x0f, 16 * tile, M);
      if constexpr (EPI == 4) {
        // the row's 1/||x|| per q / k head slice j (all 4 lanes of a row hold every one): lane g
        // stores slices g, g + 4, ..., a buffer store dropped past M and past the q / k columns
        const int hc = 2 * (N / 3) / 32, row = 16 * tile + li;
        const int nqk = (2 * (N / 3) - n0) / 32;  // q / k slices of this column block (prefix)
        const auto rr = hvk_rsrc(csum, (size_t)M * hc * 4);
#pragma unroll
        for (int j0 = 0; j0 < G::NT / 2; j0 += 4) {
          float r = rq[j0];
#pragma unroll
          for (int k = 1; k < 4; ++k)
            if (j0 + k < G::NT / 2) r = g == k ? rq[j0 + k] : r;
          const int j = j0 + g;
          hvk_bst4f(rr, row < M && j < nqk && j < G::NT / 2 ? (uint32_t)(row * hc + n0 / 32 + j) * 4 : HVK_OOB, r);
        }
      }
    }
    if (EPI == 2)
#pragma unroll
      for (int j = 0; j < G::NT / 2; ++j) hf[j] = hn[j];
    if (PREF) {
#pragma unroll
      for (int s = 0; s < G::KS; ++s) xf[s] = xn[s];
    } else {
      load_x(tile + stride, xf);
    }
  }
  if (EPI == 2) {
#pragma unroll
    for (int j = 0; j < G::NT / 2; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = cs[j][e];
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m);
        if (li == 0 && csum) atomicAdd(csum + n0 + 32 * j + 8 * g + e, v);
      }
  }
}

// Fused MLP forward for the stage-0 width (swinv2.py:58-65, C = 96, hidden 384): fc1 + bias +
// GELU and fc2 in one persistent kernel.  W1 [384 x 96] and W2 [96 x 384] both stay in LDS
// (2 x 72 KB, one 8-wave workgroup per CU); per 16-token tile a wave computes h^T = W1 x^T
// (24 tiles), writes h (nontemporal: read again only by the backward) and GELU(h) (saved for
// fc2's weight gradient) exactly as linear_kernel<96, 384, EPI 1> does, and feeds GELU(h)
// straight from registers into y^T = W2 GELU(h)^T: with W1's rows permuted (perm_row) a lane
// holds hidden units 32j + 8g .. +7 of its token, which IS the B fragment of fc2's k-chunk j,
// so the chain needs no data movement and fc2 accumulates its 12 chunks in the same order as
// linear_kernel<384, 96> (bit-identical y).  Saves fc2's re-read of GELU(h) (616 MB per block
// at bs256).
// LN: the block's post-norm LayerNorm + residual of y in the same pass (ln96, above; y = a is
// still stored for the LayerNorm backward).
template <int WAVES, bool LN = false>
__global__ __launch_bounds__(64 * WAVES) void mlp_fwd_kernel(const hvk_bf16* __restrict__ X,
                                                           const hvk_bf16* __restrict__ W1,
                                                           const float* __restrict__ b1,
                                                           const hvk_bf16* __restrict__ W2,
                                                           const float* __restrict__ b2,
                                                           hvk_bf16* __restrict__ H,
                                                           hvk_bf16* __restrict__ Gh,
                                                           hvk_bf16* __restrict__ Y, int M,
                                                           int row_groups, LnEpi ln = LnEpi{}) {
  using G1 = GCfg<96, 384>;   // fc1: K 96, 384 outputs
  using G2 = GCfg<384, 96>;   // fc2: K 384, 96 outputs
  constexpr int K = 96, N1 = 384, N2 = 96, kThreads = 64 * WAVES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* w1l = reinterpret_cast<uint4*>(smem);                                      // [24][12][16]
  uint4* w2l = reinterpret_cast<uint4*>(smem + (size_t)N1 * G1::U4 * 16);            // [6][48][16]
  float* b1l = reinterpret_cast<float*>(smem + (size_t)N1 * G1::U4 * 16 + (size_t)N2 * G2::U4 * 16);
  float* b2l = b1l + N1;
  for (int e = threadIdx.x; e < N1 * G1::U4; e += kThreads) {
    const int p = e / G1::U4, u = e % G1::U4;
    w1l[((p >> 4) * G1::U4 + u) * 16 + (p & 15)] =
        *reinterpret_cast<const uint4*>(W1 + (size_t)perm_row(p) * K + 8 * u);
  }
  for (int e = threadIdx.x; e < N2 * G2::U4; e += kThreads) {
    const int p = e / G2::U4, u = e % G2::U4;
    w2l[((p >> 4) * G2::U4 + u) * 16 + (p & 15)] =
        *reinterpret_cast<const uint4*>(W2 + (size_t)perm_row(p) * N1 + 8 * u);
  }
  for (int e = threadIdx.x; e < N1; e += kThreads) b1l[e] = b1[e];
  for (int e = threadIdx.x; e < N2; e += kThreads) b2l[e] = b2 ? b2[e] : 0.f;
  if constexpr (LN) ln96::load_params(ln, b2l + N2 + WAVES * ln96::STAGE_BYTES / 4);
  __syncthreads();

  // branch-free global accesses through 16-row tile buffer views (see linear_kernel)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int tiles = (M + 15) >> 4;
  const int stride = row_groups * WAVES;
  int tile = blockIdx.x * WAVES + wave;
  auto load_x = [&](int t, uint4 (&xf)[G1::KS]) {
    const auto rx = hvk_tile_rsrc(X, 16 * t, M, K * 2);
    const uint32_t o = (uint32_t)(li * K + 8 * g) * 2;
#pragma unroll
    for (int s = 0; s < G1::KS; ++s) xf[s] = hvk_bld16(rx, o + 64 * s);
  };
  uint4 xf[G1::KS];
  load_x(tile, xf);
  const uint32_t lstage = lds_addr(smem) + (uint32_t)(b2l + N2 - reinterpret_cast<float*>(smem)) * 4 +
                          (uint32_t)wave * ln96::STAGE_BYTES;
  const ln96::Params lnq{lds_addr(smem) + (uint32_t)(b2l + N2 - reinterpret_cast<float*>(smem)) * 4 +
                         (uint32_t)WAVES * ln96::STAGE_BYTES};
  // the first tile's operands land before the loop: otherwise the loop header's wait serves
  // both entries and becomes vmcnt(0) on every iteration (draining the stores in flight)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < G1::KS; ++s) hvk_launder(xf[s]);
  for (; tile < tiles; tile += stride) {
    asm volatile("" ::: "memory");
    uint4 xn[G1::KS];
    load_x(tile + stride, xn);
    // LN: this tile's residual rows, issued here: they land under the tile's 144 MFMAs (a tile
    // ahead they would hold 32 more VGPRs in a kernel at the 256 limit)
    uint4 x0f[LN ? 4 : 1][ln96::NG];
    if constexpr (LN) ln96::load_x0(ln, 16 * tile, M, x0f);
    __builtin_amdgcn_sched_barrier(0);  // the next tile's loads issue here, not after the MFMAs
    const auto rh = hvk_tile_rsrc(H, 16 * tile, M, N1 * 2), rg2 = hvk_tile_rsrc(Gh, 16 * tile, M, N1 * 2);
    const auto ry = hvk_tile_rsrc(Y, 16 * tile, M, N2 * 2);
    const uint32_t ho = (uint32_t)(li * N1 + 8 * g) * 2, yo = (uint32_t)(li * N2 + 8 * g) * 2;
    const bool lo8 = li < 8;
    const uint32_t hp = (uint32_t)((li & 7) * N1 + 8 * g + (lo8 ? 0 : 32)) * 2;
    const uint32_t yp = (uint32_t)((li & 7) * N2 + 8 * g + (lo8 ? 0 : 32)) * 2;
    uint4 ph = make_uint4(0, 0, 0, 0), pg = ph;
    hvk_f32x4 acc[G1::NT];
#pragma unroll
    for (int t = 0; t < G1::NT; ++t) acc[t] = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < G1::KS; ++s)
#pragma unroll
      for (int t = 0; t < G1::NT; ++t) acc[t] = hvk_mfma16(w1l[(t * G1::U4 + 4 * s + g) * 16 + li], xf[s], acc[t]);
    hvk_f32x4 acc2[G2::NT];
#pragma unroll
    for (int t = 0; t < G2::NT; ++t) acc2[t] = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < G1::NT / 2; ++j) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[2 * j][r] + b1l[32 * j + 8 * g + r];
        v[4 + r] = acc[2 * j + 1][r] + b1l[32 * j + 8 * g + 4 + r];
      }
      const uint4 hv = hvk_pack8(v);
      const uint4 gv = hvk_gelu8_bf16(hv);  // GELU of the rounded pre-activation, as the reference
      if (!HVK_LIN_PAIRSTORE) {
        if (HVK_NT_SAVED & 1)
          hvk_bst16_nt(rh, ho + 64 * j, hv);
        else
          hvk_bst16(rh, ho + 64 * j, hv);
        hvk_bst16(rg2, ho + 64 * j, gv);
      } else if (j % 2 == 0) {  // whole-line row-pair stores (see pair_rows)
        ph = hv;
        pg = gv;
      } else {
        uint4 a0, b0;
        const uint32_t o = hp + 64 * (j - 1);
        pair_rows(ph, hv, lo8, a0, b0);
        if (HVK_NT_SAVED & 1) {
          hvk_bst16_nt(rh, o, a0);
          hvk_bst16_nt(rh, o + 16 * N1, b0);
        } else {
          hvk_bst16(rh, o, a0);
          hvk_bst16(rh, o + 16 * N1, b0);
        }
        pair_rows(pg, gv, lo8, a0, b0);
        hvk_bst16(rg2, o, a0);
        hvk_bst16(rg2, o + 16 * N1, b0);
      }
      // fc2 k-chunk j: this lane's GELU(h) of hidden units 32j + 8g .. +7 is the B fragment
#pragma unroll
      for (int t = 0; t < G2::NT; ++t) acc2[t] = hvk_mfma16(w2l[(t * G2::U4 + 4 * j + g) * 16 + li], gv, acc2[t]);
    }
    uint4 av[3];  // LN: the row's packed y
#pragma unroll
    for (int j = 0; j < G2::NT / 2; ++j) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc2[2 * j][r];
        v[4 + r] = acc2[2 * j + 1][r];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += b2l[32 * j + 8 * g + e];  // 0 without a bias
      const uint4 yv = hvk_pack8(v);
      av[j] = yv;
      if (!HVK_LIN_PAIRSTORE || j == G2::NT / 2 - 1) {  // the third slice stores alone
        hvk_bst16(ry, yo + 64 * j, yv);
      } else if (j % 2 == 0) {
        ph = yv;
      } else {
        uint4 a0, b0;
        pair_rows(ph, yv, lo8, a0, b0);
        hvk_bst16(ry, yp + 64 * (j - 1), a0);
        hvk_bst16(ry, yp + 64 * (j - 1) + 16 * N2, b0);
      }
    }
    if constexpr (LN) ln96::tile(ln, lnq, lstage, av, x0f, 16 * tile, M);
#pragma unroll
    for (int s = 0; s < G1::KS; ++s) xf[s] = xn[s];
  }
}

// Fused MLP input-gradient chain for the stage-0 width (the backward of swinv2.py:58-65 at
// C = 96): gh = bf16((gy w2t^T) * GELU'(h)) (linear_kernel<96, 128, EPI 2>'s math) and
// gx = gh w1t^T (linear_kernel<384, 96>'s), one persistent kernel with w2t [384 x 96] and
// w1t [96 x 384] in LDS.  Per 16-token tile a wave produces gh in three 128-column chunks; each
// chunk is stored (fc1's weight gradient reads it) and fed from registers into gx's k-chunks
// 4q .. 4q+3 (same layout argument as mlp_fwd_kernel), so fc1's input gradient does not
// re-read gh (616 MB per block at bs256).  Bit-identical to the two launches it replaces.
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void mlp_bwd_kernel(const hvk_bf16* __restrict__ GY,
                                                           const hvk_bf16* __restrict__ W2t,
                                                           const hvk_bf16* __restrict__ Hs,
                                                           const hvk_bf16* __restrict__ W1t,
                                                           hvk_bf16* __restrict__ GH,
                                                           hvk_bf16* __restrict__ GX, int M,
                                                           int row_groups) {
  using G1 = GCfg<96, 384>;   // gh: K 96, 384 outputs
  using G2 = GCfg<384, 96>;   // gx: K 384, 96 outputs
  constexpr int K = 96, N1 = 384, N2 = 96, kThreads = 64 * WAVES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* w1l = reinterpret_cast<uint4*>(smem);                                   // w2t [24][12][16]
  uint4* w2l = reinterpret_cast<uint4*>(smem + (size_t)N1 * G1::U4 * 16);         // w1t [6][48][16]
  for (int e = threadIdx.x; e < N1 * G1::U4; e += kThreads) {
    const int p = e / G1::U4, u = e % G1::U4;
    w1l[((p >> 4) * G1::U4 + u) * 16 + (p & 15)] =
        *reinterpret_cast<const uint4*>(W2t + (size_t)perm_row(p) * K + 8 * u);
  }
  for (int e = threadIdx.x; e < N2 * G2::U4; e += kThreads) {
    const int p = e / G2::U4, u = e % G2::U4;
    w2l[((p >> 4) * G2::U4 + u) * 16 + (p & 15)] =
        *reinterpret_cast<const uint4*>(W1t + (size_t)perm_row(p) * N1 + 8 * u);
  }
  __syncthreads();

  // branch-free global accesses through 16-row tile buffer views (see linear_kernel)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int tiles = (M + 15) >> 4;
  const int stride = row_groups * WAVES;
  int tile = blockIdx.x * WAVES + wave;
  auto load_x = [&](int t, uint4 (&xf)[G1::KS]) {
    const auto rx = hvk_tile_rsrc(GY, 16 * t, M, K * 2);
    const uint32_t o = (uint32_t)(li * K + 8 * g) * 2;
#pragma unroll
    for (int s = 0; s < G1::KS; ++s) xf[s] = hvk_bld16(rx, o + 64 * s);
  };
  auto load_h = [&](int t, uint4 (&hf)[G1::NT / 2]) {
    const auto rh = hvk_tile_rsrc(Hs, 16 * t, M, N1 * 2);
    const uint32_t o = (uint32_t)(li * N1 + 8 * g) * 2;
#pragma unroll
    for (int j = 0; j < G1::NT / 2; ++j) hf[j] = hvk_bld16(rh, o + 64 * j);
  };
  uint4 xf[G1::KS], hf[G1::NT / 2];
  load_x(tile, xf);
  load_h(tile, hf);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // see mlp_fwd_kernel
#pragma unroll
  for (int s = 0; s < G1::KS; ++s) hvk_launder(xf[s]);
#pragma unroll
  for (int j = 0; j < G1::NT / 2; ++j) hvk_launder(hf[j]);
  for (; tile < tiles; tile += stride) {
    asm volatile("" ::: "memory");
    uint4 xn[G1::KS], hn[G1::NT / 2];
    load_x(tile + stride, xn);
    load_h(tile + stride, hn);
    __builtin_amdgcn_sched_barrier(0);
    const auto rgh = hvk_tile_rsrc(GH, 16 * tile, M, N1 * 2), rgx = hvk_tile_rsrc(GX, 16 * tile, M, N2 * 2);
    const uint32_t ho = (uint32_t)(li * N1 + 8 * g) * 2, xo = (uint32_t)(li * N2 + 8 * g) * 2;
    const bool lo8 = li < 8;
    const uint32_t hp = (uint32_t)((li & 7) * N1 + 8 * g + (lo8 ? 0 : 32)) * 2;
    const uint32_t xp = (uint32_t)((li & 7) * N2 + 8 * g + (lo8 ? 0 : 32)) * 2;
    uint4 ph = make_uint4(0, 0, 0, 0);
    hvk_f32x4 acc2[G2::NT];
#pragma unroll
    for (int t = 0; t < G2::NT; ++t) acc2[t] = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 3; ++q) {  // gh columns 128q .. 128q + 127 (W tiles 8q .. 8q + 7)
      hvk_f32x4 acc[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < G1::KS; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t)
          acc[t] = hvk_mfma16(w1l[((8 * q + t) * G1::U4 + 4 * s + g) * 16 + li], xf[s], acc[t]);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int j = 4 * q + jj;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[2 * jj][r];
          v[4 + r] = acc[2 * jj + 1][r];
        }
        float hv[8];
        hvk_unpack8(hf[j], hv);
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const hvk_gelu::f32x2 d = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{hv[e], hv[e + 1]});
          v[e] *= d.x;
          v[e + 1] *= d.y;
        }
        const uint4 gv = hvk_pack8(v);
        if (!HVK_LIN_PAIRSTORE) {
          hvk_bst16(rgh, ho + 64 * j, gv);
        } else if (jj % 2 == 0) {  // whole-line row-pair stores (see pair_rows)
          ph = gv;
        } else {
          uint4 a0, b0;
          pair_rows(ph, gv, lo8, a0, b0);
          hvk_bst16(rgh, hp + 64 * (j - 1), a0);
          hvk_bst16(rgh, hp + 64 * (j - 1) + 16 * N1, b0);
        }
#pragma unroll
        for (int t = 0; t < G2::NT; ++t) acc2[t] = hvk_mfma16(w2l[(t * G2::U4 + 4 * j + g) * 16 + li], gv, acc2[t]);
      }
    }
#pragma unroll
    for (int j = 0; j < G2::NT / 2; ++j) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc2[2 * j][r];
        v[4 + r] = acc2[2 * j + 1][r];
      }
      const uint4 xv = hvk_pack8(v);
      if (!HVK_LIN_PAIRSTORE || j == G2::NT / 2 - 1) {
        hvk_bst16(rgx, xo + 64 * j, xv);
      } else if (j % 2 == 0) {
        ph = xv;
      } else {
        uint4 a0, b0;
        pair_rows(ph, xv, lo8, a0, b0);
        hvk_bst16(rgx, xp + 64 * (j - 1), a0);
        hvk_bst16(rgx, xp + 64 * (j - 1) + 16 * N2, b0);
      }
    }
#pragma unroll
    for (int s = 0; s < G1::KS; ++s) xf[s] = xn[s];
#pragma unroll
    for (int j = 0; j < G1::NT / 2; ++j) hf[j] = hn[j];
  }
}

int g_cu_count = 0;

template <int K, int BN, int WAVES, bool PREF, int EPI = 0>
int launch_linear(const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, int M,
                  int N, hipStream_t st, hvk_bf16* Y2 = nullptr, float* csum = nullptr,
                  const float* qscale = nullptr, const LnEpi& ln = LnEpi{}) {
  using G0 = GCfg<K, BN>;
  struct G {  // EPI 5: + one 768-B norm staging buffer per wave
    enum : size_t { LDS = G0::LDS + (EPI == 5 ? (size_t)WAVES * ln96::STAGE_BYTES + ln96::PARAM_BYTES : 0) };
  };
  constexpr int kThreads = 64 * WAVES;
  auto kb = &linear_kernel<K, BN, WAVES, PREF, true, EPI>;
  auto kn = &linear_kernel<K, BN, WAVES, PREF, false, EPI>;
  static int per_cu = 0;  // resident workgroups per CU (LDS + VGPR limits), queried once
  if (!per_cu) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kb),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kn),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kb),
                                                     kThreads, G::LDS) != hipSuccess || nb < 1)
      nb = 1;
    per_cu = nb;
  }
  if (!g_cu_count) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return hvk_set_error(HVK_EHIP, "hvk_linear: device query failed");
    g_cu_count = prop.multiProcessorCount;
  }
  const int ncb = N / BN;
  // persistent grid: every workgroup resident (it loops over row tiles)
  const int tiles = (M + 15) / 16;
  int row_groups = g_cu_count * per_cu / ncb / 8 * 8;
  const int need = (tiles + WAVES - 1) / WAVES;
  if (row_groups > need) row_groups = (need + 7) / 8 * 8;
  if (row_groups < 8) row_groups = 8;
  const dim3 grid(row_groups * ncb);
  const double flops = 2.0 * M * N * K;
  // algorithmic bytes: X, W read once, Y written once; EPI 1 also writes GELU(h), EPI 2 reads h,
  // EPI 4 writes 1/||.|| per token and q / k head (f32)
  hvk_timer_shape("linear", EPI, BN, M, N, K,
                  2.0 * ((double)M * K + (double)N * K + (double)M * N) +
                      (EPI == 1 || EPI == 2 ? 2.0 * M * N : 0.0) + (EPI == 4 ? 4.0 * M * (2.0 * N / 96.0) : 0.0) +
                      (EPI == 5 ? (ln.x0 ? 4.0 : 0.0) * M * N + (ln.xb ? 6.0 : 4.0) * M * N + 8.0 * M : 0.0));
  if (bias)
    HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, flops, kb, grid, dim3(kThreads), G::LDS, st, X, W, bias, Y, Y2, M, N,
                       ncb, row_groups, csum, qscale, ln);
  else
    HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, flops, kn, grid, dim3(kThreads), G::LDS, st, X, W, bias, Y, Y2, M, N,
                       ncb, row_groups, csum, qscale, ln);
  HVK_CHECK_LAUNCH("hvk_linear");
  return HVK_OK;
}

struct LinCfg {
  int K, N, BN, waves, pref;
};
// built configurations; variant 0 is the default, HVK_LINEAR_VARIANT picks another row
// of the same (K, N) for experiments (tools/bench_gemm.py)
const LinCfg kLin[][4] = {
    //  default               16 waves               16 waves, no pref       half BN
    {{48, 96, 96, 8, 1}, {48, 96, 96, 16, 1}, {48, 96, 96, 16, 0}, {48, 96, 96, 8, 1}},
    {{96, 96, 96, 8, 1}, {96, 96, 96, 16, 1}, {96, 96, 96, 16, 0}, {96, 96, 96, 8, 1}},
    {{96, 288, 288, 8, 1}, {96, 288, 288, 16, 1}, {96, 288, 288, 16, 0}, {96, 288, 96, 16, 1}},
    {{96, 384, 384, 8, 1}, {96, 384, 384, 16, 1}, {96, 384, 384, 16, 0}, {96, 384, 192, 16, 1}},
    {{384, 96, 96, 8, 1}, {384, 96, 96, 16, 1}, {384, 96, 96, 16, 0}, {384, 96, 96, 8, 0}},
    {{288, 96, 96, 8, 1}, {288, 96, 96, 16, 1}, {288, 96, 96, 16, 0}, {288, 96, 96, 8, 0}},
    {{192, 192, 192, 8, 1}, {192, 192, 192, 16, 1}, {192, 192, 192, 16, 0}, {192, 192, 96, 16, 1}},
    {{192, 576, 288, 8, 1}, {192, 576, 288, 16, 1}, {192, 576, 288, 16, 0}, {192, 576, 192, 16, 1}},
    {{192, 768, 256, 8, 1}, {192, 768, 256, 16, 1}, {192, 768, 256, 16, 0}, {192, 768, 192, 16, 1}},
    {{384, 192, 192, 8, 1}, {384, 192, 192, 16, 1}, {384, 192, 192, 16, 0}, {384, 192, 96, 16, 1}},
    // stage 2 fc2 input gradient with the GELU backward (EPI 2); plain stage-2 GEMMs run on the
    // tiled kernel (gemm_tile.hip)
    {{384, 1536, 128, 8, 1}, {384, 1536, 64, 8, 1}, {384, 1536, 128, 8, 1}, {384, 1536, 64, 4, 1}},
    // SwinV2-B stages 0-1 (C = 128, 256) and its patch embedding; fc1 (N = 4C) also as the
    // fused GELU epilogues (hvk_linear_gelu_fwd / _bwd)
    {{48, 128, 128, 8, 1}, {48, 128, 128, 16, 1}, {48, 128, 128, 16, 0}, {48, 128, 128, 8, 1}},
    {{128, 128, 128, 8, 1}, {128, 128, 128, 16, 1}, {128, 128, 128, 16, 0}, {128, 128, 128, 8, 1}},
    {{128, 384, 192, 8, 1}, {128, 384, 192, 16, 1}, {128, 384, 192, 16, 0}, {128, 384, 128, 8, 1}},
    {{128, 512, 256, 8, 1}, {128, 512, 256, 16, 1}, {128, 512, 256, 16, 0}, {128, 512, 128, 8, 1}},
    {{256, 256, 128, 8, 1}, {256, 256, 128, 16, 1}, {256, 256, 128, 16, 0}, {256, 256, 128, 8, 1}},
    {{256, 768, 128, 8, 1}, {256, 768, 128, 16, 1}, {256, 768, 128, 16, 0}, {256, 768, 128, 8, 1}},
    {{256, 1024, 128, 8, 1}, {256, 1024, 128, 16, 1}, {256, 1024, 128, 16, 0}, {256, 1024, 128, 8, 1}},
};

const LinCfg* pick(int K, int N) {
  for (const auto& row : kLin)
    if (row[0].K == K && row[0].N == N) return &row[0];
  return nullptr;
}

}  // namespace

extern "C" {

int hvk_linear_supported(int M, int K, int N) { return M > 0 && pick(K, N) != nullptr; }

int hvk_linear_fwd(const void* x, const void* w, const float* bias, void* y, int M, int K, int N,
                   void* stream) {
  if (!x || !w || !y) return hvk_set_error(HVK_EINVAL, "hvk_linear_fwd: null pointer");
  if (M <= 0) return hvk_set_error(HVK_EINVAL, "hvk_linear_fwd: M=%d", M);
  const LinCfg* c = pick(K, N);
  if (!c) return hvk_set_error(HVK_EUNSUPPORTED, "hvk_linear_fwd: shape K=%d N=%d not built", K, N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hvk_bf16* X = static_cast<const hvk_bf16*>(x);
  const hvk_bf16* W = static_cast<const hvk_bf16*>(w);
  hvk_bf16* Y = static_cast<hvk_bf16*>(y);
#define HVK_LIN(k, bn, wv, pf)                                         \
  if (c->K == k && c->BN == bn && c->waves == wv && c->pref == pf)     \
    return launch_linear<k, bn, wv, pf>(X, W, bias, Y, M, N, st);
#define HVK_LIN3(k, bn) HVK_LIN(k, bn, 8, 1) HVK_LIN(k, bn, 16, 1) HVK_LIN(k, bn, 16, 0)
  HVK_LIN3(48, 96) HVK_LIN3(96, 96) HVK_LIN3(96, 288) HVK_LIN3(96, 384) HVK_LIN3(384, 96)
  HVK_LIN3(288, 96) HVK_LIN3(192, 192) HVK_LIN3(192, 288) HVK_LIN3(192, 256) HVK_LIN3(384, 192)
  HVK_LIN(96, 192, 16, 1) HVK_LIN(384, 96, 8, 0) HVK_LIN(288, 96, 8, 0) HVK_LIN(192, 96, 16, 1)
  HVK_LIN(384, 96, 16, 1) HVK_LIN(384, 128, 8, 1) HVK_LIN(384, 64, 8, 1) HVK_LIN(384, 64, 4, 1)
  HVK_LIN3(48, 128) HVK_LIN3(128, 128) HVK_LIN3(128, 192) HVK_LIN3(128, 256) HVK_LIN3(256, 128)
#undef HVK_LIN3
#undef HVK_LIN
  return hvk_set_error(HVK_EUNSUPPORTED, "hvk_linear_fwd: config K=%d BN=%d not built", K, c->BN);
}

int hvk_linear_qkv_supported(int M, int K, int N) {
  const LinCfg* c = pick(K, N);
  return M > 0 && c && N == 3 * K && K % 32 == 0 &&
         ((K == 96 && c->BN == 288) || (K == 192 && c->BN == 288) || (K == 128 && c->BN == 192) ||
          (K == 256 && c->BN == 128)) && c->waves == 8 && c->pref == 1;
}

int hvk_linear_qkv_fwd(const void* x, const void* w, const float* bias, void* y, float* rn, const float* qscale,
                       int M, int K, int N, void* stream) {
  if (!x || !w || !y || !rn) return hvk_set_error(HVK_EINVAL, "hvk_linear_qkv_fwd: null pointer");
  if (!hvk_linear_qkv_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_linear_qkv_fwd: shape M=%d K=%d N=%d not built", M, K, N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hvk_bf16* X = static_cast<const hvk_bf16*>(x);
  const hvk_bf16* W = static_cast<const hvk_bf16*>(w);
  hvk_bf16* Y = static_cast<hvk_bf16*>(y);
  if (K == 96) return launch_linear<96, 288, 8, true, 4>(X, W, bias, Y, M, N, st, nullptr, rn, qscale);
  if (K == 192) return launch_linear<192, 288, 8, true, 4>(X, W, bias, Y, M, N, st, nullptr, rn, qscale);
  if (K == 128) return launch_linear<128, 192, 8, true, 4>(X, W, bias, Y, M, N, st, nullptr, rn, qscale);
  return launch_linear<256, 128, 8, true, 4>(X, W, bias, Y, M, N, st, nullptr, rn, qscale);
}

int hvk_linear_gelu_supported(int M, int K, int N) {
  const LinCfg* c = pick(K, N);
  return M > 0 && c &&
         ((c->K == 96 && c->BN == 384) || (c->K == 192 && c->BN == 256) || (c->K == 384 && c->BN == 128) ||
          (c->K == 128 && c->BN == 256) || (c->K == 256 && c->BN == 128)) &&
         c->N == 4 * c->K && c->waves == 8 && c->pref == 1;
}

int hvk_linear_gelu_fwd(const void* x, const void* w, const float* bias, void* h, void* y, int M,
                        int K, int N, void* stream) {
  if (!x || !w || !h || !y) return hvk_set_error(HVK_EINVAL, "hvk_linear_gelu_fwd: null pointer");
  if (!hvk_linear_gelu_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_linear_gelu_fwd: shape M=%d K=%d N=%d not built", M, K, N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hvk_bf16* X = static_cast<const hvk_bf16*>(x);
  const hvk_bf16* W = static_cast<const hvk_bf16*>(w);
  hvk_bf16* H = static_cast<hvk_bf16*>(h);
  hvk_bf16* Yg = static_cast<hvk_bf16*>(y);
  if (K == 96) return launch_linear<96, 384, 8, true, 1>(X, W, bias, H, M, N, st, Yg);
  if (K == 384) return launch_linear<384, 128, 8, true, 1>(X, W, bias, H, M, N, st, Yg);
  if (K == 128) return launch_linear<128, 256, 8, true, 1>(X, W, bias, H, M, N, st, Yg);
  if (K == 256) return launch_linear<256, 128, 8, true, 1>(X, W, bias, H, M, N, st, Yg);
  return launch_linear<192, 256, 8, true, 1>(X, W, bias, H, M, N, st, Yg);
}

namespace {
constexpr size_t kMlpFwdLds = (size_t)384 * GCfg<96, 384>::U4 * 16 + (size_t)96 * GCfg<384, 96>::U4 * 16 + (384 + 96) * 4;
constexpr size_t kMlpBwdLds = (size_t)384 * GCfg<96, 384>::U4 * 16 + (size_t)96 * GCfg<384, 96>::U4 * 16;
// grant the fused MLP kernels their dynamic LDS (~149 KB) once; false when the device refuses
// it (or there is no device), so the supported() predicates send the caller to the two-launch path
bool mlp_lds_granted(const void* fn, size_t bytes, int& state) {
  if (state == 0)
    state = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess ? 1 : -1;
  return state > 0;
}
int g_mlp_fwd_lds = 0, g_mlp_bwd_lds = 0;
}  // namespace

int hvk_mlp_fwd_supported(int M, int K, int N1, int N2) {
  return M > 0 && K == 96 && N1 == 384 && N2 == 96 &&
         mlp_lds_granted(reinterpret_cast<const void*>(&mlp_fwd_kernel<8>), kMlpFwdLds, g_mlp_fwd_lds);
}

}  // extern "C"
namespace {
template <bool LN>
int launch_mlp_fwd(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* h,
                   void* g, void* y, int M, int K, int N1, int N2, const LnEpi& ln, void* stream) {
  constexpr int WAVES = 8;
  constexpr size_t LDS = kMlpFwdLds + (LN ? (size_t)WAVES * ln96::STAGE_BYTES + ln96::PARAM_BYTES : 0);
  if (!g_cu_count) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return hvk_set_error(HVK_EHIP, "hvk_mlp_fwd: device query failed");
    g_cu_count = prop.multiProcessorCount;
  }
  const int tiles = (M + 15) / 16;
  int groups = g_cu_count;  // one resident workgroup per CU (LDS)
  const int need = (tiles + WAVES - 1) / WAVES;
  if (groups > need) groups = need;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // x in; h, GELU(h), y out (the hidden tensors are written for the backward, never re-read here);
  // LN: + x0 in, x (f32), xb out
  hvk_timer_shape("mlp_fwd", LN ? 5 : 1, WAVES, M, N1, K,
                  2.0 * M * (K + 2.0 * N1 + N2) + 4.0 * N1 * K +
                      (LN ? (ln.x0 ? 4.0 : 0.0) * M * N2 + (ln.xb ? 6.0 : 4.0) * M * N2 + 8.0 * M : 0.0));
  HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, 2.0 * M * (double)N1 * K * 2, (mlp_fwd_kernel<WAVES, LN>), dim3(groups),
                     dim3(64 * WAVES), LDS, st, static_cast<const hvk_bf16*>(x), static_cast<const hvk_bf16*>(w1),
                     b1, static_cast<const hvk_bf16*>(w2), b2, static_cast<hvk_bf16*>(h),
                     static_cast<hvk_bf16*>(g), static_cast<hvk_bf16*>(y), M, groups, ln);
  HVK_CHECK_LAUNCH("hvk_mlp_fwd");
  return HVK_OK;
}
int g_mlp_ln_lds = 0;
int check_ln(const char* who, const float* gamma, const float* beta, int rows_per_sample, const float* sscale,
             float* x_out, float* mean, float* rstd) {
  if (!gamma || !beta || !x_out || !mean || !rstd) return hvk_set_error(HVK_EINVAL, "%s: null pointer", who);
  if (sscale && rows_per_sample <= 0) return hvk_set_error(HVK_EINVAL, "%s: rows_per_sample %d", who, rows_per_sample);
  return HVK_OK;
}
}  // namespace
extern "C" {

int hvk_mlp_fwd(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* h,
                void* g, void* y, int M, int K, int N1, int N2, void* stream) {
  if (!x || !w1 || !b1 || !w2 || !h || !g || !y) return hvk_set_error(HVK_EINVAL, "hvk_mlp_fwd: null pointer");
  if (!hvk_mlp_fwd_supported(M, K, N1, N2))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_mlp_fwd: shape M=%d K=%d N1=%d N2=%d not built", M, K, N1, N2);
  return launch_mlp_fwd<false>(x, w1, b1, w2, b2, h, g, y, M, K, N1, N2, LnEpi{}, stream);
}

int hvk_mlp_ln_supported(int M, int K, int N1, int N2) {
  return M > 0 && K == 96 && N1 == 384 && N2 == 96 &&
         mlp_lds_granted(reinterpret_cast<const void*>(&mlp_fwd_kernel<8, true>),
                         kMlpFwdLds + 8 * ln96::STAGE_BYTES + ln96::PARAM_BYTES, g_mlp_ln_lds);
}

int hvk_mlp_ln_fwd(const void* x, const void* w1, const float* b1, const void* w2, void* h, void* g, void* a_out,
                   int M, int K, int N1, int N2, const float* abias, const float* x0, const float* gamma,
                   const float* beta, const float* sample_scale, int rows_per_sample, float eps, float* x_out,
                   void* xb_out, float* mean, float* rstd, void* stream) {
  if (!x || !w1 || !b1 || !w2 || !h || !g || !a_out) return hvk_set_error(HVK_EINVAL, "hvk_mlp_ln_fwd: null pointer");
  int rc = check_ln("hvk_mlp_ln_fwd", gamma, beta, rows_per_sample, sample_scale, x_out, mean, rstd);
  if (rc) return rc;
  if (!hvk_mlp_ln_supported(M, K, N1, N2))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_mlp_ln_fwd: shape M=%d K=%d N1=%d N2=%d not built", M, K, N1, N2);
  const LnEpi ln{abias, x0, gamma, beta, sample_scale, rows_per_sample, eps, x_out, static_cast<hvk_bf16*>(xb_out),
                 mean, rstd};
  return launch_mlp_fwd<true>(x, w1, b1, w2, nullptr, h, g, a_out, M, K, N1, N2, ln, stream);
}

// C = 96: the skinny kernel (K 96 / 48); C = 192: the 128 x 192 tile kernel (K % 64 == 0)
int hvk_linear_ln_supported(int M, int K, int N) {
  return M > 0 && ((N == 96 && (K == 96 || K == 48)) || hvk_tile_ln::supported(M, N, K));
}

int hvk_linear_ln_fwd(const void* x, const void* w, int M, int K, int N, const float* abias, const float* x0,
                      const float* gamma, const float* beta, const float* sample_scale, int rows_per_sample,
                      float eps, void* a_out, float* x_out, void* xb_out, float* mean, float* rstd, void* stream) {
  if (!x || !w || !a_out) return hvk_set_error(HVK_EINVAL, "hvk_linear_ln_fwd: null pointer");
  int rc = check_ln("hvk_linear_ln_fwd", gamma, beta, rows_per_sample, sample_scale, x_out, mean, rstd);
  if (rc) return rc;
  if (!hvk_linear_ln_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_linear_ln_fwd: shape M=%d K=%d N=%d not built", M, K, N);
  const LnEpi ln{abias, x0, gamma, beta, sample_scale, rows_per_sample, eps, x_out, static_cast<hvk_bf16*>(xb_out),
                 mean, rstd};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hvk_bf16* X = static_cast<const hvk_bf16*>(x);
  const hvk_bf16* W = static_cast<const hvk_bf16*>(w);
  hvk_bf16* A = static_cast<hvk_bf16*>(a_out);
  if (N != 96) return hvk_tile_ln::launch(X, W, A, M, N, K, ln, st);
  if (K == 96) return launch_linear<96, 96, 8, true, 5>(X, W, nullptr, A, M, N, st, nullptr, nullptr, nullptr, ln);
  return launch_linear<48, 96, 8, true, 5>(X, W, nullptr, A, M, N, st, nullptr, nullptr, nullptr, ln);
}

int hvk_mlp_bwd_supported(int M, int K, int N1, int N2) {
  return M > 0 && K == 96 && N1 == 384 && N2 == 96 &&
         mlp_lds_granted(reinterpret_cast<const void*>(&mlp_bwd_kernel<8>), kMlpBwdLds, g_mlp_bwd_lds);
}

int hvk_mlp_bwd(const void* gy, const void* w2t, const void* h, const void* w1t, void* gh, void* gx, int M,
                int K, int N1, int N2, void* stream) {
  if (!gy || !w2t || !h || !w1t || !gh || !gx) return hvk_set_error(HVK_EINVAL, "hvk_mlp_bwd: null pointer");
  if (!hvk_mlp_bwd_supported(M, K, N1, N2))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_mlp_bwd: shape M=%d K=%d N1=%d N2=%d not built", M, K, N1, N2);
  constexpr int WAVES = 8;
  constexpr size_t LDS = kMlpBwdLds;
  if (!g_cu_count) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return hvk_set_error(HVK_EHIP, "hvk_mlp_bwd: device query failed");
    g_cu_count = prop.multiProcessorCount;
  }
  const int tiles = (M + 15) / 16;
  int groups = g_cu_count;
  const int need = (tiles + WAVES - 1) / WAVES;
  if (groups > need) groups = need;
  // gy, h in; gh (for fc1's weight gradient), gx out
  hvk_timer_shape("mlp_bwd", 2, WAVES, M, N1, K, 2.0 * M * (K + 2.0 * N1 + N2) + 4.0 * N1 * K);
  HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, 2.0 * M * (double)N1 * K * 2, (mlp_bwd_kernel<WAVES>), dim3(groups),
                     dim3(64 * WAVES), LDS, static_cast<hipStream_t>(stream), static_cast<const hvk_bf16*>(gy),
                     static_cast<const hvk_bf16*>(w2t), static_cast<const hvk_bf16*>(h),
                     static_cast<const hvk_bf16*>(w1t), static_cast<hvk_bf16*>(gh), static_cast<hvk_bf16*>(gx),
                     M, groups);
  HVK_CHECK_LAUNCH("hvk_mlp_bwd");
  return HVK_OK;
}

int hvk_linear_gelu_in_supported(int M, int K, int N) { return M > 0 && K == 384 && N == 96; }

int hvk_linear_gelu_in_fwd(const void* h, const void* w, const float* bias, void* y, int M, int K, int N,
                           void* stream) {
  if (!h || !w || !y) return hvk_set_error(HVK_EINVAL, "hvk_linear_gelu_in_fwd: null pointer");
  if (!hvk_linear_gelu_in_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_linear_gelu_in_fwd: shape M=%d K=%d N=%d not built", M, K, N);
  return launch_linear<384, 96, 8, true, 3>(static_cast<const hvk_bf16*>(h), static_cast<const hvk_bf16*>(w),
                                            bias, static_cast<hvk_bf16*>(y), M, N,
                                            static_cast<hipStream_t>(stream));
}

int hvk_linear_gelu_bwd_supported(int M, int K, int N) {
  return M > 0 && ((K == 96 && N == 384) || (K == 192 && N == 768) || (K == 384 && N == 1536) ||
                   (K == 128 && N == 512) || (K == 256 && N == 1024));
}

int hvk_linear_gelu_bwd(const void* gy, const void* w, const void* h, void* gh, float* dbias,
                        int M, int K, int N, void* stream) {
  if (!gy || !w || !h || !gh)
    return hvk_set_error(HVK_EINVAL, "hvk_linear_gelu_bwd: null pointer");
  if (!hvk_linear_gelu_bwd_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_linear_gelu_bwd: shape M=%d K=%d N=%d not built", M, K, N);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hvk_bf16* X = static_cast<const hvk_bf16*>(gy);
  const hvk_bf16* W = static_cast<const hvk_bf16*>(w);
  hvk_bf16* H = const_cast<hvk_bf16*>(static_cast<const hvk_bf16*>(h));
  hvk_bf16* G = static_cast<hvk_bf16*>(gh);
  if (K == 96) return launch_linear<96, 128, 8, true, 2>(X, W, nullptr, G, M, N, st, H, dbias);
  if (K == 384) return launch_linear<384, 128, 8, true, 2>(X, W, nullptr, G, M, N, st, H, dbias);
  if (K == 128) return launch_linear<128, 128, 8, true, 2>(X, W, nullptr, G, M, N, st, H, dbias);
  if (K == 256) return launch_linear<256, 128, 8, true, 2>(X, W, nullptr, G, M, N, st, H, dbias);
  return launch_linear<192, 128, 8, true, 2>(X, W, nullptr, G, M, N, st, H, dbias);
}

}  // extern "C"
