// Tiled MFMA GEMM for the compute-heavier SwinV2 Linears on gfx950 (stage 2-3 of SwinV2-T:
// M = 12544-50176 tokens, K = 384-3072, N = 384-3072, and the stage-1 N = 192 GEMMs with
// K = 576-768), where the weight block no longer fits the skinny kernel's LDS (gemm.hip):
//   Y[M, N] = X[M, K] W[N, K]^T (+ bias[N]) (EPI 0), or the fc1 form h = Y + bias, GELU(h)
//   (EPI 1) -- F.linear of swinv2.py:58-62, 220, 262 and the input gradients (W = weight^T).
// 128 x 128 output tile per 256-thread workgroup (2 x 2 waves of 64 x 64), K in steps of 64:
//  * both operand tiles are staged by LDS-DMA (global_load_lds_dwordx4, nontemporal off),
//    each wave-instruction moving 8 whole 128-B row segments; two buffers, the next k-step's
//    DMA in flight during the current MFMAs (counted vmcnt, raw s_barrier);
//  * LDS rows are 128 B with the 16-B chunk index XOR-swizzled by (row & 7): the fragment
//    reads (ds_read_b128, 16 rows x 16 B per lane group) are bank-conflict free; the swizzle
//    is applied on the DMA's global source address (the LDS side of a DMA is lane-linear);
//  * Y^T = W X^T on v_mfma_f32_16x16x32_bf16 with the W rows of each 32-row pair permuted
//    (as gemm.hip), so a lane ends with 8 consecutive output columns of one row: 16-B stores.
#include <stdlib.h>

#include "gemm_tile_ln.h"
#include "hvk_common.h"

// experiment builds (tools/probe/Makefile, NOT the product): 1 no MFMA, 2 no stores, 3 no DMA,
// 4 per-workgroup phase timestamps (hvk_gemm_probe_read, tools/gemm_timeline.py)
#ifndef HVK_GEMM_PROBE
#define HVK_GEMM_PROBE 0
#endif
#ifndef HVK_TILE_HPRE  // 1: EPI 2's h loads issued two k-steps before the epilogue
#define HVK_TILE_HPRE 1
#endif
#ifndef HVK_TILE_PRIO  // A/B build: s_setprio 1 over each k-step's MFMAs
#define HVK_TILE_PRIO 0
#endif
#ifndef HVK_TILE_STAGED  // 1: the 128-row tiles store their outputs through LDS as whole row runs
#define HVK_TILE_STAGED 1
#endif
#if HVK_GEMM_PROBE == 4
__device__ unsigned long long g_gemm_probe[32768 * 6];
#endif

namespace {

typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef __attribute__((address_space(1))) void* gbl_vptr_t;

// 2 x 2 waves per 256-thread workgroup; a wave owns 64 rows (4 x-tiles of 16 tokens) and
// 16 TN columns (TN W-tiles): TN = 4 -> 128 x 128 output tiles (64 KB LDS, double buffered),
// TN = 6 -> 128 x 192 for N = 192 (80 KB: still two workgroups per CU)
constexpr int BM = 128, BK = 64;
constexpr int XTILE_BYTES = BM * BK * 2;  // 16 KB
template <int TN>
struct TileCfg {
  static constexpr int BN = 32 * TN, WTILE = BN * BK * 2, STAGE = WTILE + XTILE_BYTES, LDS = 2 * STAGE;
};

// LDS row p of a W tile holds W row perm(p) of the tile (see gemm.hip: the accumulator rows
// 4g + r of tiles 2j, 2j+1 then map to output columns 32j + 8g .. 32j + 8g + 7)
__device__ __forceinline__ int perm_row(int p) {
  const int t = p >> 4, m = p & 15;
  return 32 * (t >> 1) + 8 * (m >> 2) + 4 * (t & 1) + (m & 3);
}

// workgroup barrier that waits only for this wave's LDS operations (stores in flight stay)
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
// fragment reads from inline asm: hipcc would otherwise wait vmcnt(0) before every LDS read
// while the next k-step's DMA is in flight (cdna_hip_programming.md, glds pipelining)
template <int OFF>
__device__ __forceinline__ hvk_u32x4 rd128(uint32_t a) {
  hvk_u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
__device__ __forceinline__ uint4 tie(hvk_u32x4 v) {
  asm volatile("" : "+v"(v));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// Epilogue shared by both tiled kernels: acc[t][b] of a lane (li, gq) holds W-tile t x token
// tile b of a wave whose tokens start at row0 and columns at col0; tiles 2j, 2j+1 give the 8
// consecutive columns col0 + 32j + 8gq .. +7 of token row0 + 16b + li (perm_row).  Bias / h
// loads first, every output packed, then all 16-B stores back to back: a register still read
// by an outstanding store cannot be rewritten before vmcnt says so, and a load waited for
// between stores would wait for every store before it (vmcnt counts in order).
// EPI 2's saved pre-activation h of a lane's outputs, in the output layout
template <int EPI, int NT, int MT, int B0 = 0, int B1 = MT, int HM = MT>
__device__ __forceinline__ void load_h_tile(uint4 (&hp)[EPI == 2 ? HM : 1][NT / 2], const hvk_bf16* __restrict__ Y2,
                                            int M, int N, int row0, int col0) {
  if (EPI != 2) return;
  const int lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
#pragma unroll
  for (int b = B0; b < B1; ++b) {
    int row = row0 + 16 * b + li;
    if (row >= M) row = M - 1;
#pragma unroll
    for (int j = 0; j < NT / 2; ++j)
      hp[b][j] = (HVK_NT_SAVED & 8) ? hvk_ld16_nt(Y2 + (size_t)row * N + col0 + 32 * j + 8 * gq)
                                    : *reinterpret_cast<const uint4*>(Y2 + (size_t)row * N + col0 + 32 * j + 8 * gq);
  }
}

// LDS-staged output (128-row tiles): a fragment store from registers writes 16 rows x 64 B per
// wave-instruction (16 half lines); staged through the tile's LDS, which the k-loop no longer
// uses, each 256-thread store round writes 4 KB of whole row runs (cdna_hip_programming.md:
// "O staged through LDS and stored as whole rows").  Image [BM rows][BN bf16], the 16-B chunk
// cc of row r at cc ^ (r & 7): the fragment writes (8-lane groups = 8 rows, one chunk) and the
// row-run reads are bank-conflict free under the §LDS model of MI355X_MICROARCH.md.
template <int BN>
__device__ __forceinline__ uint32_t stage_off(int row, int cc) {
  return (uint32_t)(row * BN * 2 + 16 * (cc ^ (row & 7)));
}
template <int NT, int MT, int BN>
__device__ __forceinline__ void stage_write(char* smem, const hvk_u32x4 (&v)[MT][NT / 2], int r0, int c0) {
  const int lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
#pragma unroll
  for (int b = 0; b < MT; ++b)
#pragma unroll
    for (int j = 0; j < NT / 2; ++j)
      *reinterpret_cast<hvk_u32x4*>(smem + stage_off<BN>(r0 + 16 * b + li, c0 + 4 * j + gq)) = v[b][j];
}
// every 16-B chunk of the 128 x BN image -> Y rows m0 .., columns n0 ..: all LDS reads first,
// then the stores back to back.  SC: Y is PatchMerging's token tensor and the image rows are
// merged rows, each chunk scattered to its source token (hvk_merge_tok / hvk_merge_col)
template <int BN, bool NTS, int BM_ = 128, int THREADS = 256, bool SC = false>
__device__ __forceinline__ void stage_store(const char* smem, hvk_bf16* __restrict__ Y, int M, int N, int m0, int n0,
                                            const MergeGeo& mg = MergeGeo{}) {
  constexpr int CPR = BN / 8, PER = BM_ * CPR / THREADS;
  static_assert(BM_ * CPR % THREADS == 0, "whole store rounds");
  hvk_u32x4 v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + THREADS * i, row = c / CPR, cc = c - row * CPR;
    v[i] = *reinterpret_cast<const hvk_u32x4*>(smem + stage_off<BN>(row, cc));
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + THREADS * i, row = c / CPR, cc = c - row * CPR;
    if (m0 + row < M) {
      hvk_u32x4* dst = reinterpret_cast<hvk_u32x4*>(
          SC ? Y + (size_t)hvk_merge_tok(m0 + row, mg) * mg.C + hvk_merge_col(n0 + 8 * cc, mg)
             : Y + (size_t)(m0 + row) * N + n0 + 8 * cc);
      if (NTS) __builtin_nontemporal_store(v[i], dst);
      else *dst = v[i];
    }
  }
}

// EPI 4 (the qkv Linear of a w <= 8 W-MSA block): Y = acc + bias with every q and k head slice
// (columns < 2N/3) normalised (hvk_head_normalize8, F.normalize of swinv2.py:229) and its
// 1 / max(||x||, eps) stored to rn [M, 2N/96]; the v columns as EPI 0.
template <int EPI, int NT, int MT, int HPRE = 0, int SBN = 0, int SBM = 128, int STHREADS = 256, bool SC = false>
__device__ __forceinline__ void tile_epilogue(const hvk_f32x4 (&acc)[NT][MT], const float* __restrict__ bias,
                                              hvk_bf16* __restrict__ Y, hvk_bf16* __restrict__ Y2, int M,
                                              int N, int row0, int col0,
                                              const uint4 (*hpre)[NT / 2] = nullptr, float* __restrict__ rn = nullptr,
                                              const float* __restrict__ qscale = nullptr, char* smem = nullptr,
                                              int m0 = 0, int n0 = 0, const MergeGeo& mg = MergeGeo{}) {
  // SC: Y is PatchMerging's token tensor (EPI 0, staged; stage_store)
  static_assert(!SC || (EPI == 0 && SBN > 0), "the scattered store is the staged EPI 0 form");
  // SBN > 0: outputs staged through the LDS image of a 128 x SBN tile whose origin is (m0, n0)
  // (every wave of the workgroup calls this; the k-loop's LDS reads are all complete)
  // HPRE: h of token tiles 0 .. HPRE-1 was loaded early by the caller (hpre)
  const int lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  float bv[NT / 2][8];
  if (EPI != 2 && bias) {
#pragma unroll
    for (int j = 0; j < NT / 2; ++j) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + col0 + 32 * j + 8 * gq);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + col0 + 32 * j + 8 * gq + 4);
      bv[j][0] = b0.x; bv[j][1] = b0.y; bv[j][2] = b0.z; bv[j][3] = b0.w;
      bv[j][4] = b1.x; bv[j][5] = b1.y; bv[j][6] = b1.z; bv[j][7] = b1.w;
    }
  }
  uint4 hp[EPI == 2 ? MT : 1][NT / 2];  // gh = (gy w) * GELU'(h): h (Y2) in the output layout
  if (EPI == 2) {
#pragma unroll
    for (int b = 0; b < HPRE; ++b)
#pragma unroll
      for (int j = 0; j < NT / 2; ++j) hp[b][j] = hpre[b][j];
    load_h_tile<EPI, NT, MT, HPRE, MT>(hp, Y2, M, N, row0, col0);
  }
  hvk_u32x4 pk[MT][NT / 2], pg[EPI == 1 ? MT : 1][NT / 2];
  float rv[EPI == 4 ? MT : 1][NT / 2];
  const int qk_cols = 2 * (N / 3);
  // EPI 4: q slices (columns < N/3) come out as q^ * scale_h * log2e (qscale = the head's
  // exp(clamp(logit_scale)), the W-MSA forward's logit scale), k slices as k^
  float qpost[EPI == 4 ? NT / 2 : 1];
  if constexpr (EPI == 4) {
#pragma unroll
    for (int j = 0; j < NT / 2; ++j) {
      const int c = col0 + 32 * j;
      qpost[j] = (qscale && c < N / 3) ? qscale[c / 32] * HVK_LOG2E : 1.f;
    }
  }
#pragma unroll
  for (int b = 0; b < MT; ++b)
#pragma unroll
    for (int j = 0; j < NT / 2; ++j) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[2 * j][b][r];
        v[4 + r] = acc[2 * j + 1][b][r];
      }
      if (EPI != 2 && bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bv[j][e];
      }
      if (EPI == 2) {
        float hf[8];
        hvk_unpack8(hp[b][j], hf);
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const hvk_gelu::f32x2 d = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{hf[e], hf[e + 1]});
          v[e] *= d.x;
          v[e + 1] *= d.y;
        }
      }
      const uint4 hv = hvk_pack8(v);
      pk[b][j] = __builtin_bit_cast(hvk_u32x4, hv);
      if (EPI == 1) pg[b][j] = __builtin_bit_cast(hvk_u32x4, hvk_gelu8_bf16(hv));  // GELU of the rounded h
      if constexpr (EPI == 4) {
        rv[b][j] = 0.f;
        if (col0 + 32 * j < qk_cols) {  // wave-uniform: the v column blocks skip it
          float r;
          pk[b][j] = __builtin_bit_cast(hvk_u32x4, hvk_head_normalize8(hv, r, qpost[j]));  // all 64 lanes
          rv[b][j] = r;
        }
      }
    }
  // pin the packing here (else hipcc sinks it into each row's store branch and reuses the
  // registers of the previous row's stores)
#pragma unroll
  for (int b = 0; b < MT; ++b)
#pragma unroll
    for (int j = 0; j < NT / 2; ++j) {
      asm volatile("" : "+v"(pk[b][j]));
      if (EPI == 1) asm volatile("" : "+v"(pg[b][j]));
    }
  if constexpr (SBN > 0) {
    const int r0 = row0 - m0, c0 = (col0 - n0) / 8;
    stage_write<NT, MT, SBN>(smem, pk, r0, c0);
    lds_sync();
    stage_store<SBN, EPI == 1 && (HVK_NT_SAVED & 1), SBM, STHREADS, SC>(smem, Y, M, N, m0, n0, mg);  // h: read again only by the backward
    if constexpr (EPI == 1) {
      lds_sync();  // every thread's image reads are back before the GELU outputs overwrite it
      stage_write<NT, MT, SBN>(smem, pg, r0, c0);
      lds_sync();
      stage_store<SBN, false, SBM, STHREADS>(smem, Y2, M, N, m0, n0);
    }
  }
#pragma unroll
  for (int b = 0; b < MT; ++b) {
    const int row = row0 + 16 * b + li;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < NT / 2; ++j) {
      if constexpr (SBN > 0) break;
      const size_t o = (size_t)row * N + col0 + 32 * j + 8 * gq;
      if (EPI == 1 && (HVK_NT_SAVED & 1))  // h: read again only by the backward
        __builtin_nontemporal_store(pk[b][j], reinterpret_cast<hvk_u32x4*>(Y + o));
      else
        *reinterpret_cast<hvk_u32x4*>(Y + o) = pk[b][j];
      if (EPI == 1) *reinterpret_cast<hvk_u32x4*>(Y2 + o) = pg[b][j];
    }
    if constexpr (EPI == 4) {
      // the row's 1/||x|| of head slices j = 0 .. NT/2-1 (every lane of the row holds all of them):
      // lane gq stores slice gq, one store instruction per row instead of one per slice
      float r = rv[b][0];
#pragma unroll
      for (int j = 1; j < NT / 2; ++j) r = gq == j ? rv[b][j] : r;
      const int c = col0 + 32 * gq;
      if (gq < NT / 2 && c < qk_cols) rn[(size_t)row * (qk_cols / 32) + c / 32] = r;
    }
  }
}

// EPI 5 (N = C = 192: a 128 x 192 tile is whole rows, stage 1): the res-post-norm LayerNorm +
// residual of swinv2.py:431 / 434 on the staged output image (the tile's `a`, already stored for
// the norm's backward), in ln_fwd_kernel<8, 32>'s lane layout (32 lanes per row, channel groups
// of 4 at 4 (32 i + t); layernorm.hip) with its arithmetic (hvk_ln_*), so x, xb, mean and rstd
// are bit-identical to the two-launch path (tests/test_gpu_linear_ln.py).  A wave takes 2 rows a
// pass, 16 passes per tile; the next pass's residual rows are loaded under this pass's math.
#ifndef HVK_LN192_U  // norm passes interleaved per iteration (A/B build switch: 1, 2, 4)
#define HVK_LN192_U 2
#endif
namespace ln192 {
constexpr int C = 192, PASSES = BM / 8;
__device__ __forceinline__ void rows(const char* img, const LnEpi& p, int M, int m0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 31, sub = lane >> 5;
  const bool ok1 = t < 16;  // group 1 (channels 128 + 4t ..) exists for t < 16
  float gm[8], bt[8], ab[8];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = 4 * (32 * i + t);
    float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f), b4 = g4, a4 = g4;
    if (i == 0 || ok1) {
      g4 = *reinterpret_cast<const float4*>(p.gamma + c);
      b4 = *reinterpret_cast<const float4*>(p.beta + c);
      if (p.abias) a4 = *reinterpret_cast<const float4*>(p.abias + c);
    }
    gm[4 * i] = g4.x; gm[4 * i + 1] = g4.y; gm[4 * i + 2] = g4.z; gm[4 * i + 3] = g4.w;
    bt[4 * i] = b4.x; bt[4 * i + 1] = b4.y; bt[4 * i + 2] = b4.z; bt[4 * i + 3] = b4.w;
    ab[4 * i] = a4.x; ab[4 * i + 1] = a4.y; ab[4 * i + 2] = a4.z; ab[4 * i + 3] = a4.w;
  }
  const float invC = 1.f / C;
  auto ld_x0 = [&](int pass, float4 (&d)[2]) {
    const int row = m0 + 8 * pass + 2 * wave + sub;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      d[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.x0 && row < M && (i == 0 || ok1))
        d[i] = *reinterpret_cast<const float4*>(p.x0 + (size_t)row * C + 4 * (32 * i + t));
    }
  };
  // U passes (rows r, r + 8, ...) per iteration, their reductions independent chains the compiler
  // interleaves (one pass at a time left each shuffle's latency exposed at 2 waves per SIMD)
  constexpr int U = HVK_LN192_U;
  float4 xn[U][2];
#pragma unroll
  for (int u = 0; u < U; ++u) ld_x0(u, xn[u]);
  for (int pp = 0; pp < PASSES; pp += U) {
    float4 xc[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xc[u][0] = xn[u][0];
      xc[u][1] = xn[u][1];
    }
    if (pp + U < PASSES)
#pragma unroll
      for (int u = 0; u < U; ++u) ld_x0(pp + U + u, xn[u]);
    float v[U][8], s[U], mu[U], ss[U], rs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = 8 * (pp + u) + 2 * wave + sub;
      s[u] = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i == 0 || ok1) {
          const int c = 4 * (32 * i + t);
          const uint2 w = *reinterpret_cast<const uint2*>(img + stage_off<C>(r, c >> 3) + ((c & 7) << 1));
          v[u][4 * i] = hvk_lo(w.x); v[u][4 * i + 1] = hvk_hi(w.x); v[u][4 * i + 2] = hvk_lo(w.y); v[u][4 * i + 3] = hvk_hi(w.y);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[u][4 * i + j] += ab[4 * i + j]; s[u] += v[u][4 * i + j]; }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[u][4 * i + j] = 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) mu[u] = hvk_xor_sum<32>(s[u]) * invC;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ss[u] = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (i == 0 || ok1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) ss[u] = hvk_ln_sq(ss[u], v[u][4 * i + j] - mu[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) rs[u] = hvk_ln_rstd(hvk_xor_sum<32>(ss[u]), invC, p.eps);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = m0 + 8 * (pp + u) + 2 * wave + sub;
      if (row >= M) continue;
      const float sc = p.sscale ? p.sscale[row / p.rows_per_sample] : 1.f;
      const size_t rb = (size_t)row * C;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (!(i == 0 || ok1)) continue;
        const int c = 4 * (32 * i + t);
        float o[4] = {xc[u][i].x, xc[u][i].y, xc[u][i].z, xc[u][i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = hvk_ln_out(o[j], v[u][4 * i + j], mu[u], rs[u], gm[4 * i + j], bt[4 * i + j], sc);
        const uint4 xr = make_uint4(__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3]));
        if (HVK_NT_SAVED & 2) hvk_st16_nt(p.x + rb + c, xr);  // read again only at the next LayerNorm
        else *reinterpret_cast<uint4*>(p.x + rb + c) = xr;
        if (p.xb) *reinterpret_cast<uint2*>(p.xb + rb + c) = make_uint2(hvk_pack2(o[0], o[1]), hvk_pack2(o[2], o[3]));
      }
      if (t == 0) {
        p.mean[row] = mu[u];
        p.rstd[row] = rs[u];
      }
    }
  }
}
}  // namespace ln192

// MG 1: X is PatchMerging's token tensor [B, H W, C], gathered into the merged rows on the DMA
// (K = 4C); MG 2: Y is, the merged output rows scattered to it (N = 4C; hvk_common.h MergeGeo)
template <int EPI, bool PIPE, int TN, int MG = 0>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const hvk_bf16* __restrict__ X,
                                                        const hvk_bf16* __restrict__ Wt,
                                                        const float* __restrict__ bias,
                                                        hvk_bf16* __restrict__ Y,
                                                        hvk_bf16* __restrict__ Y2, int M, int N,
                                                        int K, int mtiles, float* __restrict__ rn,
                                                        const float* __restrict__ qscale, LnEpi ln,
                                                        MergeGeo mg) {
  using T = TileCfg<TN>;
  constexpr int BN = T::BN, STAGE_BYTES = T::STAGE, TILE_BYTES = T::WTILE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntiles = N / BN;
  // XCD-aware decode: the n-tiles of one m-tile share blockIdx % 8 (one L2): the X row block
  // is fetched from HBM once and re-read from L2
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int nt = loc % ntiles, mt = (loc / ntiles) * 8 + xcd;
  if (mt >= mtiles) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  const int wn = wave & 1, wm = wave >> 1;  // this wave's 64 x 16TN sub-tile (n half, m half)
  const int KT = K / BK;

  // DMA: operand instruction j fills LDS rows 8j .. 8j+7 of its tile; lane L -> row
  // 8j + L/8, LDS chunk L%8 <- global chunk (L%8) ^ (row & 7).  Wave w issues j = w + 4i
  // (4 x-tile and TN W-tile instructions per wave and stage).
  const int lr = lane >> 3, lc = lane & 7;
  size_t xsrc[4], wsrc[TN];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (wave + 4 * i) + lr;
    int xr = m0 + row;
    if (xr >= M) xr = M - 1;  // rows past M: any valid row (never stored)
    xsrc[i] = MG == 1 ? (size_t)hvk_merge_tok(xr, mg) * mg.C : (size_t)xr * K + 8 * (lc ^ (row & 7));
  }
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int row = 8 * (wave + 4 * i) + lr;
    wsrc[i] = (size_t)(n0 + perm_row(row)) * K + 8 * (lc ^ (row & 7));
  }
  auto issue = [&](int kt, int buf) {
    if (HVK_GEMM_PROBE == 3) return;
    char* base = smem + buf * STAGE_BYTES;
    const int k0 = kt * BK;
    // MG 1: a lane's chunk column k0 + 8 (lc ^ lr) is the same in its 4 rows (row & 7 == lr)
    const int xk = MG == 1 ? hvk_merge_col(k0 + 8 * (lc ^ lr), mg) : k0;
#pragma unroll
    for (int i = 0; i < TN; ++i)
      __builtin_amdgcn_global_load_lds((gbl_vptr_t)(Wt + wsrc[i] + k0),
                                       (lds_vptr_t)(base + (wave + 4 * i) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((gbl_vptr_t)(X + xsrc[i] + xk),
                                       (lds_vptr_t)(base + TILE_BYTES + (wave + 4 * i) * 1024), 16, 0, 0);
  };

  hvk_f32x4 acc[TN][4];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = hvk_f32x4{0, 0, 0, 0};

#if HVK_GEMM_PROBE == 4
  const unsigned long long t0 = wall_clock64();
  unsigned long long t1 = 0;
#endif
  // EPI 2: the epilogue's h vectors are loaded at the top of k-step KT-2 (after its DMA wait;
  // the last two k-steps issue no DMA, and the vmcnt(0) at the top of k-step KT-1 covers them),
  // so their latency hides under the last k-steps instead of opening the epilogue
  constexpr int HPB = (EPI == 2 && HVK_TILE_HPRE) ? 2 : 0;  // token tiles prefetched (VGPR budget)
  uint4 hpre[HPB ? HPB : 1][TN / 2];
  const int hk = KT >= 2 ? KT - 2 : 0;
  issue(0, 0);
  if (KT > 1) issue(1, 1);
  for (int kt = 0; kt < KT; ++kt) {
    // this k-step's tile has landed (the next one's TN + 4 DMAs per wave may stay in flight)
    if (kt + 1 < KT)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(TN + 4) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (HPB && kt == hk)
      load_h_tile<EPI, TN, 4, 0, HPB, HPB ? HPB : 1>(hpre, Y2, M, N, m0 + 64 * wm, n0 + 16 * TN * wn);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#if HVK_GEMM_PROBE == 4
    if (kt == 0) t1 = wall_clock64();
#endif
    const uint32_t base = lds_u32(smem) + (kt & 1) * STAGE_BYTES;
    // PIPE: all 2 (TN + 4) fragments of the k-step in flight at once, the first half's MFMAs
    // start as soon as their reads are back (lgkmcnt counts in issue order); else
    // read-wait-compute per half
    hvk_u32x4 ra[2][TN], rb[2][4];
    auto read_half = [&](int ks) {
      // rows 16 TN wn + 16t + li (row & 7 = li & 7), chunk 4ks + g swizzled; t in immediates
      const uint32_t aw = base + (16 * TN * wn + li) * 128 + (((4 * ks + g) ^ (li & 7)) << 4);
      const uint32_t ax = base + TILE_BYTES + (64 * wm + li) * 128 + (((4 * ks + g) ^ (li & 7)) << 4);
      ra[ks][0] = rd128<0>(aw);
      ra[ks][1] = rd128<2048>(aw);
      ra[ks][2] = rd128<4096>(aw);
      ra[ks][3] = rd128<6144>(aw);
      if constexpr (TN > 4) {
        ra[ks][4 % TN] = rd128<8192>(aw);
        ra[ks][5 % TN] = rd128<10240>(aw);
      }
      rb[ks][0] = rd128<0>(ax);
      rb[ks][1] = rd128<2048>(ax);
      rb[ks][2] = rd128<4096>(ax);
      rb[ks][3] = rd128<6144>(ax);
    };
    auto mfma_half = [&](int ks) {
      uint4 af[TN], bf[4];
#pragma unroll
      for (int t = 0; t < TN; ++t) af[t] = tie(ra[ks][t]);
#pragma unroll
      for (int t = 0; t < 4; ++t) bf[t] = tie(rb[ks][t]);
      if (HVK_GEMM_PROBE == 1) {
        acc[0][0][0] += __uint_as_float(af[0].x ^ bf[0].x ^ af[3].y ^ bf[3].y);
        return;
      }
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = hvk_mfma16(af[a], bf[b], acc[a][b]);
    };
    if (PIPE) {
      read_half(0);
      read_half(1);
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(TN + 4) : "memory");
      if (HVK_TILE_PRIO) __builtin_amdgcn_s_setprio(1);
      mfma_half(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_half(1);
      if (HVK_TILE_PRIO) __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        read_half(ks);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        mfma_half(ks);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done with this buffer
    asm volatile("" ::: "memory");
    if (kt + 2 < KT) issue(kt + 2, kt & 1);
  }

#if HVK_GEMM_PROBE == 4
  const unsigned long long t2 = wall_clock64();
#endif
  if (HVK_GEMM_PROBE == 2 && acc[0][0][0] != 1234.5f) return;
  // EPI 5: `a` leaves as EPI 0 (no bias: it is the norm's abias), then the norm of the image
  static_assert(EPI != 5 || (HVK_TILE_STAGED && TN == 6), "EPI 5 runs on the staged 128 x 192 image");
  static_assert(MG != 2 || (HVK_TILE_STAGED && EPI == 0), "MG 2 scatters the staged EPI 0 image");
  tile_epilogue<EPI == 5 ? 0 : EPI, TN, 4, HPB, HVK_TILE_STAGED ? BN : 0, 128, 256, MG == 2>(
      acc, EPI == 5 ? nullptr : bias, Y, Y2, M, N, m0 + 64 * wm, n0 + 16 * TN * wn, hpre, rn, qscale, smem, m0, n0, mg);
  if constexpr (EPI == 5) ln192::rows(smem, ln, M, m0);
#if HVK_GEMM_PROBE == 4
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t3 = wall_clock64();
  if (threadIdx.x == 0 && blockIdx.x < 32768) {
    unsigned long long* q = g_gemm_probe + 6 * blockIdx.x;
    q[0] = t0; q[1] = t1; q[2] = t2; q[3] = t3;
    q[4] = __builtin_amdgcn_s_getreg(63492);  // HW_ID
    q[5] = __builtin_amdgcn_s_getreg(63508);  // XCC_ID
  }
#endif
}

// algorithmic HBM bytes of one Y = X W^T launch: X, W read once, Y written once; EPI 1 also
// writes GELU(h), EPI 2 reads h, EPI 4 writes 1/||.|| per token and q / k head (f32)
double tile_bytes(int epi, double M, double N, double K) {
  return 2.0 * (M * K + N * K + M * N) + (epi == 1 || epi == 2 ? 2.0 * M * N : 0.0) +
         (epi == 4 ? 4.0 * M * (2.0 * N / 96.0) : 0.0) +
         (epi == 5 ? 10.0 * M * N + 8.0 * M : 0.0);  // EPI 5: x0 in, x + xb out, mean / rstd (x0 counted)
}

template <int EPI, bool PIPE, int TN, int MG = 0>
int launch_tile_(const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2,
                 int M, int N, int K, hipStream_t st, float* rn = nullptr, const float* qscale = nullptr,
                 const LnEpi& ln = LnEpi{}, const MergeGeo& mg = MergeGeo{}) {
  using T = TileCfg<TN>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<EPI, PIPE, TN, MG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
    attr = true;
  }
  const int mtiles = (M + BM - 1) / BM;
  const int mpad = (mtiles + 7) / 8 * 8;
  const dim3 grid(mpad * (N / T::BN));
  hvk_timer_shape(MG ? "gemm_nt_merge" : "gemm_nt", EPI, T::BN, M, N, K, tile_bytes(EPI, M, N, K));
  HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, 2.0 * M * N * K, (gemm_nt_kernel<EPI, PIPE, TN, MG>), grid, dim3(256),
                     T::LDS, st, X, W, bias, Y, Y2, M, N, K, mtiles, rn, qscale, ln, mg);
  HVK_CHECK_LAUNCH("hvk_gemm_tile");
  return HVK_OK;
}

// 128 x 128 or 128 x 192 tiles
template <int EPI>
int launch_tile(const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2,
                int M, int N, int K, hipStream_t st, float* rn = nullptr, const float* qscale = nullptr) {
  // 128 x 192 also where 192 | N and the tile is not the narrow N = 384, K < 1152 case
  // (tools/bench_gemm.py, interleaved: 3-25 % faster on the stage-2/3 shapes, 6 % slower on
  // the stage-2 projection; with the LDS-staged epilogue also 5 % faster for the stage-2 qkv
  // input gradient, K = 1152: profiles/round4/tile_width_staged/); option "tile_wide" 0 / 1
  // forces 128 / 192 columns where both divide N
  const int force = (int)hvk_opt(HVK_OPT_TILE_WIDE);
  if constexpr (EPI == 4) {  // the qkv form: the 128-row tile kernel only
    // 192 columns where 192 | N and either 128 does not divide N (N = 192, 576, ...) or the rule
    // / option asks for them
    if (N % TileCfg<6>::BN == 0 &&
        (N % TileCfg<4>::BN != 0 || (force >= 0 ? force == 1 : (N > 384 || K >= 1152))))
      return launch_tile_<EPI, true, 6>(X, W, bias, Y, Y2, M, N, K, st, rn, qscale);
    return launch_tile_<EPI, true, 4>(X, W, bias, Y, Y2, M, N, K, st, rn, qscale);
  } else {
  // the fused fc1 + GELU epilogue (EPI 1) at K >= 384 (stages 2-3) prefers 128-column tiles:
  // half the per-tile epilogue, which the co-resident workgroup then hides better
  // (tools/gpu_tilew.sh: 2-7 % on s2/s3 fc1; 192 stays faster for stage-1 fc1 and for EPI 2)
  const bool epi1_narrow = EPI == 1 && K >= 384 && N % TileCfg<4>::BN == 0;
  const bool wide = N % TileCfg<6>::BN == 0 &&
                    (force >= 0 ? force == 1 : ((N > 384 || K >= 1152) && !epi1_narrow));
  if (N % TileCfg<4>::BN == 0 && !wide)
    return launch_tile_<EPI, true, 4>(X, W, bias, Y, Y2, M, N, K, st);
  return launch_tile_<EPI, true, 6>(X, W, bias, Y, Y2, M, N, K, st);
  }
}

// PatchMerging's reduction GEMM with the 2x2 gather on its X operand (MG 1: EPI 0, or EPI 5 with
// the norm) or its input gradient with the scatter in its store (MG 2): the tile launch_tile<0>
// picks for the same shape with default options, so the bits equal gather + GEMM / GEMM + scatter
template <int EPI, int MG>
int launch_merge(const hvk_bf16* X, const hvk_bf16* W, hvk_bf16* Y, int M, int N, int K, const MergeGeo& mg,
                 hipStream_t st, const LnEpi& ln = LnEpi{}) {
  if constexpr (EPI == 5) {
    return launch_tile_<5, true, 6, MG>(X, W, nullptr, Y, nullptr, M, N, K, st, nullptr, nullptr, ln, mg);
  } else {
    const int force = (int)hvk_opt(HVK_OPT_TILE_WIDE);
    const bool wide = N % TileCfg<6>::BN == 0 && (force >= 0 ? force == 1 : (N > 384 || K >= 1152));
    if (N % TileCfg<4>::BN == 0 && !wide)
      return launch_tile_<EPI, true, 4, MG>(X, W, nullptr, Y, nullptr, M, N, K, st, nullptr, nullptr, ln, mg);
    return launch_tile_<EPI, true, 6, MG>(X, W, nullptr, Y, nullptr, M, N, K, st, nullptr, nullptr, ln, mg);
  }
}

}  // namespace

extern "C" int hvk_gemm_supported(int M, int K, int N);
namespace hvk_tile_ln {
bool supported(int M, int N, int K) { return N == ln192::C && hvk_gemm_supported(M, K, N); }
int launch(const hvk_bf16* X, const hvk_bf16* W, hvk_bf16* Y, int M, int N, int K, const LnEpi& ln, hipStream_t st) {
  if (!supported(M, N, K)) return hvk_set_error(HVK_EUNSUPPORTED, "tile LN epilogue: M=%d K=%d N=%d", M, K, N);
  return launch_tile_<5, true, 6>(X, W, nullptr, Y, nullptr, M, N, K, st, nullptr, nullptr, ln);
}
}  // namespace hvk_tile_ln

extern "C" {

#if HVK_GEMM_PROBE == 4
int hvk_gemm_probe_read(void* dst, int nblocks) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_gemm_probe), sizeof(unsigned long long) * 6 * nblocks, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

int hvk_gemm_supported(int M, int K, int N) {
  return M > 0 && K >= BK && K % BK == 0 && (N % TileCfg<4>::BN == 0 || N % TileCfg<6>::BN == 0) &&
         K <= 8192 && N <= 16384;
}

int hvk_gemm_fwd(const void* x, const void* w, const float* bias, void* y, int M, int K, int N,
                 void* stream) {
  if (!x || !w || !y) return hvk_set_error(HVK_EINVAL, "hvk_gemm_fwd: null pointer");
  if (!hvk_gemm_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_gemm_fwd: M=%d K=%d N=%d (K %% 64, N %% 128)", M, K, N);
  return launch_tile<0>(static_cast<const hvk_bf16*>(x), static_cast<const hvk_bf16*>(w), bias,
                        static_cast<hvk_bf16*>(y), nullptr, M, N, K, static_cast<hipStream_t>(stream));
}

int hvk_gemm_gelu_bwd(const void* gy, const void* w, const void* h, void* gh, int M, int K, int N,
                      void* stream) {
  if (!gy || !w || !h || !gh) return hvk_set_error(HVK_EINVAL, "hvk_gemm_gelu_bwd: null pointer");
  if (!hvk_gemm_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_gemm_gelu_bwd: M=%d K=%d N=%d", M, K, N);
  return launch_tile<2>(static_cast<const hvk_bf16*>(gy), static_cast<const hvk_bf16*>(w), nullptr,
                        static_cast<hvk_bf16*>(gh),
                        const_cast<hvk_bf16*>(static_cast<const hvk_bf16*>(h)), M, N, K,
                        static_cast<hipStream_t>(stream));
}

int hvk_gemm_qkv_fwd(const void* x, const void* w, const float* bias, void* y, float* rn, const float* qscale, int M, int K,
                     int N, void* stream) {
  if (!x || !w || !y || !rn) return hvk_set_error(HVK_EINVAL, "hvk_gemm_qkv_fwd: null pointer");
  if (!hvk_gemm_supported(M, K, N) || N % 96)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_gemm_qkv_fwd: M=%d K=%d N=%d (N = 3C, 32 | C)", M, K, N);
  return launch_tile<4>(static_cast<const hvk_bf16*>(x), static_cast<const hvk_bf16*>(w), bias,
                        static_cast<hvk_bf16*>(y), nullptr, M, N, K, static_cast<hipStream_t>(stream), rn, qscale);
}

// ---- PatchMerging (swinv2.py:484-494): gather / scatter folded into the reduction GEMM ----------
static bool merge_geo(int B, int H, int W, int C, int& M, MergeGeo& g) {
  if (B <= 0 || H <= 0 || W <= 0 || H % 2 || W % 2 || C <= 0 || C % 8) return false;
  const long long m = (long long)B * (H / 2) * (W / 2);
  if (m >= (1ll << 21) || (long long)B * H * W * C >= (1ll << 31)) return false;  // hvk_merge_tok exactness
  M = (int)m;
  g.W = W;
  g.C = C;
  g.inv_wo = 1.0f / (float)(W / 2);
  return true;
}

int hvk_merge_gemm_supported(int B, int H, int W, int C, int N) {
  int M;
  MergeGeo g;
  return merge_geo(B, H, W, C, M, g) && hvk_gemm_supported(M, 4 * C, N) && hvk_gemm_supported(M, N, 4 * C);
}

int hvk_merge_gemm_fwd(const void* x, const void* w, void* y, int B, int H, int W, int C, int N, void* stream) {
  if (!x || !w || !y) return hvk_set_error(HVK_EINVAL, "hvk_merge_gemm_fwd: null pointer");
  int M;
  MergeGeo g;
  if (!merge_geo(B, H, W, C, M, g) || !hvk_merge_gemm_supported(B, H, W, C, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_merge_gemm_fwd: B=%d H=%d W=%d C=%d N=%d", B, H, W, C, N);
  return launch_merge<0, 1>(static_cast<const hvk_bf16*>(x), static_cast<const hvk_bf16*>(w), static_cast<hvk_bf16*>(y),
                            M, N, 4 * C, g, static_cast<hipStream_t>(stream));
}

int hvk_merge_linear_ln_supported(int B, int H, int W, int C, int N) {
  int M;
  MergeGeo g;
  return merge_geo(B, H, W, C, M, g) && hvk_merge_gemm_supported(B, H, W, C, N) && hvk_tile_ln::supported(M, N, 4 * C);
}

int hvk_merge_linear_ln_fwd(const void* x, const void* w, int B, int H, int W, int C, int N, const float* gamma,
                            const float* beta, float eps, void* a_out, float* x_out, void* xb_out, float* mean,
                            float* rstd, void* stream) {
  if (!x || !w || !a_out || !gamma || !beta || !x_out || !mean || !rstd)
    return hvk_set_error(HVK_EINVAL, "hvk_merge_linear_ln_fwd: null pointer");
  int M;
  MergeGeo g;
  if (!merge_geo(B, H, W, C, M, g) || !hvk_merge_linear_ln_supported(B, H, W, C, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_merge_linear_ln_fwd: B=%d H=%d W=%d C=%d N=%d", B, H, W, C, N);
  const LnEpi ln{nullptr, nullptr, gamma, beta, nullptr, 1, eps, x_out, static_cast<hvk_bf16*>(xb_out), mean, rstd};
  return launch_merge<5, 1>(static_cast<const hvk_bf16*>(x), static_cast<const hvk_bf16*>(w),
                            static_cast<hvk_bf16*>(a_out), M, N, 4 * C, g, static_cast<hipStream_t>(stream), ln);
}

int hvk_merge_gemm_dgrad(const void* gy, const void* wt, void* gx, int B, int H, int W, int C, int N, void* stream) {
  if (!gy || !wt || !gx) return hvk_set_error(HVK_EINVAL, "hvk_merge_gemm_dgrad: null pointer");
  int M;
  MergeGeo g;
  if (!merge_geo(B, H, W, C, M, g) || !hvk_merge_gemm_supported(B, H, W, C, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_merge_gemm_dgrad: B=%d H=%d W=%d C=%d N=%d", B, H, W, C, N);
  return launch_merge<0, 2>(static_cast<const hvk_bf16*>(gy), static_cast<const hvk_bf16*>(wt),
                            static_cast<hvk_bf16*>(gx), M, 4 * C, N, g, static_cast<hipStream_t>(stream));
}

int hvk_gemm_gelu_fwd(const void* x, const void* w, const float* bias, void* h, void* y, int M, int K,
                      int N, void* stream) {
  if (!x || !w || !h || !y || !bias) return hvk_set_error(HVK_EINVAL, "hvk_gemm_gelu_fwd: null pointer");
  if (!hvk_gemm_supported(M, K, N))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_gemm_gelu_fwd: M=%d K=%d N=%d", M, K, N);
  return launch_tile<1>(static_cast<const hvk_bf16*>(x), static_cast<const hvk_bf16*>(w), bias,
                        static_cast<hvk_bf16*>(h), static_cast<hvk_bf16*>(y), M, N, K,
                        static_cast<hipStream_t>(stream));
}

}  // extern "C"
