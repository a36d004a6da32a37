// Weight-gradient GEMM of the SwinV2 Linears on gfx950 (the backward of F.linear,
// swinv2.py:58-62 / 220 / 262 / 296): dW[N, K] = g[M, N]^T x[M, K] in f32 and, fused,
// db[N] = sum_m g[m, n], for M = tokens (12544 .. 802816) and N, K = 96 .. 3072.
//
// Both operands are token-major (rows = tokens), the contraction runs over the tokens:
//  * the tokens are cut into chunks, one workgroup per (output tile, chunk), ~one per CU;
//    each streams its chunk through a 4-8 deep ring of LDS stages of 32 tokens, filled by
//    LDS-DMA (global_load_lds_dwordx4) with counted vmcnt waits and raw s_barriers;
//  * a stage holds the g and x rows as 4-token x 16-column subtiles of 128 B (row blocks
//    padded to an odd number of subtiles), so the MFMA operands come out of
//    ds_read_b64_tr_b16 (4 tokens of one column per lane) without bank conflicts;
//  * v_mfma_f32_16x16x32_bf16 with A = x^T, B = g^T: a lane ends with 4 consecutive k of one
//    n, a 16-B store of dW[n][k..k+3]; db rides along as one MFMA per g fragment with an
//    all-ones A operand;
//  * each workgroup writes its f32 partial tile to a workspace slab; a second kernel sums
//    the slabs over the chunks into dW and db (deterministic, no atomics).
#include <stdlib.h>

#include <type_traits>

#include "hvk_common.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef __attribute__((address_space(1))) void* gbl_vptr_t;

constexpr int LDS_CAP = 150 * 1024;
constexpr int TOK = 32;  // tokens per stage = the MFMA contraction depth

// FK x FN 16x16 fragments per wave, WK x WN waves: workgroup tile TK x TN
template <int FK, int FN, int WK, int WN>
struct TnCfg {
  static constexpr int THREADS = 64 * WK * WN;
  static constexpr int TK = 16 * FK * WK, TN = 16 * FN * WN;
  static constexpr int NCBG = TN / 16, NCBX = TK / 16;       // 16-column blocks per operand
  static constexpr int RBSG = (NCBG | 1) * 128;              // bytes per 4-token row block:
  static constexpr int RBSX = (NCBX | 1) * 128;              //   odd subtile count, no conflicts
  static constexpr int REGG = 8 * RBSG, REGX = 8 * RBSX;
  static constexpr int CHUNKS = (REGG + REGX) / 16;          // 16-B DMA chunks per stage
  static constexpr int D = (CHUNKS + THREADS - 1) / THREADS;  // DMA instructions per lane per stage
  static constexpr int STAGE = D * THREADS * 16;
  // the 128 x <=192 tiles run two workgroups per CU (half the LDS each, <= 128 VGPRs)
  static constexpr int PER_CU = (TK == 128 && TN <= 192) ? 2 : 1, CAP = LDS_CAP / PER_CU;
  static constexpr int NST = (CAP / STAGE) > 8 ? 8 : (CAP / STAGE);
  static constexpr int LDS = NST * STAGE;
  static_assert(NST >= 3, "LDS ring too shallow");
  static_assert((NST - 1) * D <= 63, "vmcnt range");
};

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
template <int OFF>
__device__ __forceinline__ hvk_u32x2 rd_tr(uint32_t a) {
  hvk_u32x2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
__device__ __forceinline__ uint4 tie2(hvk_u32x2 lo, hvk_u32x2 hi) {
  asm volatile("" : "+v"(lo), "+v"(hi));
  return make_uint4(lo[0], lo[1], hi[0], hi[1]);
}
template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most min(r, R) later stages (D instructions each) are outstanding
template <int D, int R>
__device__ __forceinline__ void wait_stages(int r) {
  if constexpr (R <= 0) {
    wait_vm<0>();
  } else {
    if (r >= R)
      wait_vm<R * D>();
    else
      wait_stages<D, R - 1>(r);
  }
}

// MG: X is PatchMerging's token tensor [B, H W, C] (K = 4C), its merged rows gathered on the DMA
// (hvk_common.h MergeGeo): the reduction Linear's weight gradient without the materialised gather
template <int FK, int FN, int WK, int WN, bool DB, bool GX = false, bool MG = false>
__global__ __launch_bounds__(64 * WK * WN, (16 * FK * WK == 128 && 16 * FN * WN <= 192) ? 2 : 1) void dw_kernel(const hvk_bf16* __restrict__ G,
                                                           const hvk_bf16* __restrict__ X,
                                                           float* __restrict__ P, int N, int K,
                                                           int ntk, int ntiles, int nslices,
                                                           int nchunk, long pstride, MergeGeo mg) {
  using C = TnCfg<FK, FN, WK, WN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // XCD-aware decode: work items (chunk-major: item = c * ntiles + tile) are dealt to the 8
  // XCDs (blockIdx % 8) in contiguous runs, so the workgroups of one L2 share their chunk's
  // token rows and those come from HBM about once
  const int items = ntiles * nchunk, per = (items + 7) >> 3;
  const int item = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if ((blockIdx.x >> 3) >= per || item >= items) return;
  const int tile = item % ntiles, c = item / ntiles;
  const int k0 = (tile % ntk) * C::TK, n0 = (tile / ntk) * C::TN;
  const int sb = (int)((long)c * nslices / nchunk);
  const int ns = (int)((long)(c + 1) * nslices / nchunk) - sb;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;

  // DMA: LDS chunk ci = THREADS i + tid of a stage (lane-linear) <- global 16 B of
  // (operand, token row 4 rb + q, column 16 cb + 8 hf); pad subtiles / tail chunks re-read
  // the operand's first row of the stage and land in LDS nobody reads
  // MG: an x chunk's address is rebuilt per stage from its merged row mrow (-1: a g chunk) and its
  // column's offset mcol
  const char* src[C::D];
  uint32_t inc[C::D];
  int mrow[MG ? C::D : 1], mcol[MG ? C::D : 1];
#pragma unroll
  for (int i = 0; i < C::D; ++i) {
    const int ci = i * C::THREADS + tid;
    const hvk_bf16* base = G + (size_t)sb * TOK * N + n0;
    size_t off = 0;
    uint32_t step = 2u * TOK * N;
    if (MG) mrow[i] = -1, mcol[i] = 0;
    if (ci < C::REGG / 16) {
      const int rb = ci / (C::RBSG / 16), w = ci % (C::RBSG / 16);
      if (w < 8 * C::NCBG) off = (size_t)(4 * rb + ((w & 7) >> 1)) * N + 16 * (w >> 3) + 8 * (w & 1);
    } else if (ci < C::CHUNKS) {
      const int lc = ci - C::REGG / 16;
      const int rb = lc / (C::RBSX / 16), w = lc % (C::RBSX / 16);
      base = X + (size_t)sb * TOK * K + k0;
      step = 2u * TOK * K;
      const bool real = w < 8 * C::NCBX;
      if (real) off = (size_t)(4 * rb + ((w & 7) >> 1)) * K + 16 * (w >> 3) + 8 * (w & 1);
      if (MG) {
        mrow[i] = sb * TOK + (real ? 4 * rb + ((w & 7) >> 1) : 0);
        mcol[i] = hvk_merge_col(k0 + (real ? 16 * (w >> 3) + 8 * (w & 1) : 0), mg);
      }
    }
    src[i] = reinterpret_cast<const char*>(base + off);
    inc[i] = step;
  }
  auto issue = [&](int buf) {
    char* b = smem + buf * C::STAGE + wave * 1024;
#pragma unroll
    for (int i = 0; i < C::D; ++i) {
      const char* p = src[i];
      if constexpr (MG) {
        if (mrow[i] >= 0) {
          p = reinterpret_cast<const char*>(X + (size_t)hvk_merge_tok(mrow[i], mg) * mg.C + mcol[i]);
          mrow[i] += TOK;
        }
      }
      __builtin_amdgcn_global_load_lds((gbl_vptr_t)p, (lds_vptr_t)(b + i * C::THREADS * 16), 16, 0, 0);
      src[i] += inc[i];
    }
  };

  // fragment reads: group gq of 16 lanes, lane 4q + p: token rows 4 (4h + gq) + q,
  // columns 4p .. 4p+3 of 16-column block cb -> kk = 8 gq + 4 h + q of the MFMA
  const int l16 = lane & 15, gq = lane >> 4;
  const int wk = wave % WK, wn = wave / WK;
  const uint32_t la = C::REGG + gq * C::RBSX + (l16 >> 2) * 32 + (l16 & 3) * 8 + wk * FK * 128;
  const uint32_t lb = gq * C::RBSG + (l16 >> 2) * 32 + (l16 & 3) * 8 + wn * FN * 128;

  hvk_f32x4 acc[FK][FN], adb[FN];
#pragma unroll
  for (int a = 0; a < FK; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
  for (int b = 0; b < FN; ++b) adb[b] = hvk_f32x4{0, 0, 0, 0};
  const uint4 ones = make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u);

  for (int s = 0; s < C::NST - 1 && s < ns; ++s) issue(s);
  for (int s = 0; s < ns; ++s) {
    wait_stages<C::D, C::NST - 2>(ns - 1 - s);  // this stage's DMA (per wave) has landed
    __builtin_amdgcn_s_barrier();               // ... for every wave; stage s-1 is free
    asm volatile("" ::: "memory");
    if (s + C::NST - 1 < ns) issue((s + C::NST - 1) % C::NST);
    const uint32_t base = lds_u32(smem) + (s % C::NST) * C::STAGE;
    const uint32_t ax = base + la, bx = base + lb;
    hvk_u32x2 ra[FK][2], rb[FN][2];
    sfor<0, FN>([&](auto ic) {
      constexpr int b = decltype(ic)::value;
      rb[b][0] = rd_tr<b * 128>(bx);
      rb[b][1] = rd_tr<4 * C::RBSG + b * 128>(bx);
    });
    sfor<0, FK>([&](auto ic) {
      constexpr int a = decltype(ic)::value;
      ra[a][0] = rd_tr<a * 128>(ax);
      ra[a][1] = rd_tr<4 * C::RBSX + a * 128>(ax);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint4 fa[FK], fb[FN];
#pragma unroll
    for (int b = 0; b < FN; ++b) fb[b] = tie2(rb[b][0], rb[b][1]);
#pragma unroll
    for (int a = 0; a < FK; ++a) {
      fa[a] = tie2(ra[a][0], ra[a][1]);
      if (GX) fa[a] = hvk_gelu8_bf16(fa[a]);  // x = GELU(h) of the saved pre-activation
    }
#pragma unroll
    for (int a = 0; a < FK; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b) acc[a][b] = hvk_mfma16(fa[a], fb[b], acc[a][b]);
    if (DB) {  // the bias gradient: the n-fragments dealt over the WK waves that share them
#pragma unroll
      for (int b = 0; b < FN; ++b)
        if (b % WK == wk) adb[b] = hvk_mfma16(ones, fb[b], adb[b]);
    }
  }

  // lane (l16, gq) holds dW[n0 + 16 FN wn + 16 b + l16][k0 + 16 FK wk + 16 a + 4 gq + r]
  float* Pc = P + (size_t)c * pstride;
#pragma unroll
  for (int b = 0; b < FN; ++b) {
    const int n = n0 + wn * 16 * FN + 16 * b + l16;
#pragma unroll
    for (int a = 0; a < FK; ++a) {
      const int k = k0 + wk * 16 * FK + 16 * a + 4 * gq;
      *reinterpret_cast<float4*>(Pc + (size_t)n * K + k) =
          make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
    }
    if (DB && b % WK == wk && gq == 0) Pc[(size_t)N * K + n] = adb[b][0];
  }
}

// dW / db = sum over the chunks' slabs; 32 float4 columns x 8 chunk phases per workgroup.
// xshift (K floats) or null: dW += db (x) xshift, i.e. dW = g^T (x + 1 xshift^T) -- the proj
// Linear's input is o + v_bias in the reference (swinv2.py:255-262) while the GEMM ran on o, its
// v_bias share folded into the bias (hvk_block_bias_fwd); db[n] is re-summed from the slabs here
// (K / 4 threads share each row's partials through L2).  db null: not stored.
template <int NPH>  // chunk phases (warps of 32 threads) per workgroup
__global__ __launch_bounds__(32 * NPH) void dw_reduce_kernel(const float4* __restrict__ P, int e4,
                                                        int ndw4, int nchunk, long pstride4,
                                                        float4* __restrict__ dw,
                                                        float4* __restrict__ db,
                                                        const float* __restrict__ xshift, int K) {
  __shared__ float4 red[NPH][32];
  __shared__ float redd[NPH][32];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int e = blockIdx.x * 32 + tx;
  const int n = (4 * e) / K;  // the dW row of this float4 (e < ndw4)
  const float* Pdb = reinterpret_cast<const float*>(P) + 4 * (size_t)ndw4 + n;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  float sd = 0.f;
  if (e < e4) {
#pragma unroll 4
    for (int c = ty; c < nchunk; c += NPH) {
      const float4 v = P[(size_t)c * pstride4 + e];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      if (xshift && e < ndw4) sd += Pdb[(size_t)c * pstride4 * 4];
    }
  }
  red[ty][tx] = s;
  redd[ty][tx] = sd;
  __syncthreads();
  if (ty == 0 && e < e4) {
#pragma unroll
    for (int j = 1; j < NPH; ++j) {
      const float4 v = red[j][tx];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      sd += redd[j][tx];
    }
    if (xshift && e < ndw4) {
      const float4 xs = *reinterpret_cast<const float4*>(xshift + (4 * e) % K);
      s.x = fmaf(sd, xs.x, s.x); s.y = fmaf(sd, xs.y, s.y); s.z = fmaf(sd, xs.z, s.z); s.w = fmaf(sd, xs.w, s.w);
    }
    if (e >= ndw4 && !db) return;
    float4* dst = e < ndw4 ? dw + e : db + (e - ndw4);
    if (HVK_NT_SAVED & 64)  // read only by the optimizer at the end of the step
      hvk_st16_nt(dst, make_uint4(__float_as_uint(s.x), __float_as_uint(s.y), __float_as_uint(s.z),
                                  __float_as_uint(s.w)));
    else
      *dst = s;
  }
}

// workgroup shapes: 0-3 the stage-0 Linears (whole output per workgroup), 4-7 a 192 x 192
// or 192 x 384 tile for the rest; default 192 x 192 on 8 waves (tools/bench_dw.py: fastest
// with the fused bias gradient on every stage 1-3 shape); B256 / B128: 128 x 256 and 128 x 128
// tiles for the widths 192 does not divide (SwinV2-B: C = 128 ... 1024)
// V_T4 .. V_T8C are the option "dw_tile" values 4 .. 8 (tile_variant): keep their numbers
enum { V_288x96, V_96x96, V_384x96, V_96x384, V_T4, V_T8A, V_T8B, V_T8W, V_T8C, V_B256, V_B128, V_96x48, V_128x48 };
static_assert(V_T4 == 4 && V_T8C == 8, "dw_tile option values");

struct Plan {
  int var = -1, tk = 0, tn = 0, ntk = 0, ntiles = 0, nslices = 0, nchunk = 0;
  long pstride = 0;
};

int tile_variant() {
  return (int)hvk_opt(HVK_OPT_DW_TILE);
}

bool plan(int M, int N, int K, Plan& p) {
  if (M <= 0 || M % TOK) return false;
  if (N == 288 && K == 96) p.var = V_288x96, p.tk = 96, p.tn = 288;
  else if (N == 96 && K == 96) p.var = V_96x96, p.tk = 96, p.tn = 96;
  else if (N == 384 && K == 96) p.var = V_384x96, p.tk = 96, p.tn = 384;
  else if (N == 96 && K == 384) p.var = V_96x384, p.tk = 384, p.tn = 96;
  else if (N == 96 && K == 48) p.var = V_96x48, p.tk = 48, p.tn = 96;  // the patch embedding (4x4x3 -> 96)
  else if (N == 128 && K == 48) p.var = V_128x48, p.tk = 48, p.tn = 128;  // SwinV2-B's (4x4x3 -> 128)
  else if (N % 192 == 0 && K % 192 == 0 && N <= 8192 && K <= 8192) {
    p.var = tile_variant();
    if (p.var < V_T4 || p.var > V_T8C || (p.var == V_T8W && N % 384)) p.var = V_T4;
    if (p.var == V_T8C && K % 128) p.var = V_T8A;
    p.tk = p.var == V_T8C ? 128 : 192, p.tn = p.var == V_T8W ? 384 : 192;
  } else if (N % 128 == 0 && K % 128 == 0 && N <= 8192 && K <= 8192) {
    p.var = N % 256 == 0 ? V_B256 : V_B128;
    p.tk = 128, p.tn = p.var == V_B256 ? 256 : 128;
  } else {
    return false;
  }
  p.ntk = K / p.tk;
  p.ntiles = p.ntk * (N / p.tn);
  p.nslices = M / TOK;
  const int target = (int)hvk_opt(HVK_OPT_DW_CHUNKS);  // default 256: about one workgroup per CU
  int nc = (p.var == V_T8C || p.var == V_B128 ? 2 * target : target) / p.ntiles;
  if (nc < 1) nc = 1;
  if (nc > p.nslices) nc = p.nslices;
  p.nchunk = nc;
  p.pstride = (long)N * K + N;
  return true;
}

template <int FK, int FN, int WK, int WN, bool GX = false, bool MG = false>
int launch(const hvk_bf16* g, const hvk_bf16* x, float* P, bool with_db, int N, int K, const Plan& p,
           hipStream_t st, const MergeGeo& mg = MergeGeo{}) {
  using C = TnCfg<FK, FN, WK, WN>;
  static_assert(C::TK > 0 && C::TN > 0, "tile");
  if (C::TK != p.tk || C::TN != p.tn) return hvk_set_error(HVK_EINVAL, "hvk_weight_grad: plan/tile mismatch");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_kernel<FK, FN, WK, WN, true, GX, MG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_kernel<FK, FN, WK, WN, false, GX, MG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  const dim3 grid((unsigned)((p.ntiles * p.nchunk + 7) / 8 * 8));
  const double flops = 2.0 * p.nslices * TOK * N * K;  // g^T x (the fused db adds 2 M N)
  {  // algorithmic bytes: g and x read once, dW (+ db) written once in f32 (partial slabs excluded)
    const double M = (double)p.nslices * TOK;
    hvk_timer_shape(GX ? "dw_gelu_x" : MG ? "dw_merge" : "dw", with_db ? 1 : 0, C::TN, M, N, K,
                    2.0 * M * (N + K) + 4.0 * N * K + (with_db ? 4.0 * N : 0.0));
  }
  if (with_db)
    HVK_LAUNCH_TIMED_W(HVK_TIMER_WGRAD, flops, (dw_kernel<FK, FN, WK, WN, true, GX, MG>), grid, dim3(C::THREADS),
                       C::LDS, st, g, x, P, N, K, p.ntk, p.ntiles, p.nslices, p.nchunk, p.pstride, mg);
  else
    HVK_LAUNCH_TIMED_W(HVK_TIMER_WGRAD, flops, (dw_kernel<FK, FN, WK, WN, false, GX, MG>), grid, dim3(C::THREADS),
                       C::LDS, st, g, x, P, N, K, p.ntk, p.ntiles, p.nslices, p.nchunk, p.pstride, mg);
  HVK_CHECK_LAUNCH("hvk_weight_grad");
  return HVK_OK;
}

}  // namespace

extern "C" {

int hvk_weight_grad_supported(int M, int N, int K) {
  Plan p;
  return plan(M, N, K, p) ? 1 : 0;
}

size_t hvk_weight_grad_workspace(int M, int N, int K) {
  Plan p;
  if (!plan(M, N, K, p)) return 0;
  return (size_t)p.nchunk * (size_t)p.pstride * sizeof(float);
}

static int weight_grad(const void* g, const void* x, float* dw, float* db, int M, int N, int K, void* ws,
                       size_t ws_bytes, void* stream, bool gx, const float* xshift = nullptr,
                       const MergeGeo* mg = nullptr) {
  if (!g || !x || !dw || !ws) return hvk_set_error(HVK_EINVAL, "hvk_weight_grad: null pointer");
  Plan p;
  if (!plan(M, N, K, p))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_weight_grad: M=%d N=%d K=%d", M, N, K);
  if (ws_bytes < (size_t)p.nchunk * (size_t)p.pstride * sizeof(float))
    return hvk_set_error(HVK_EINVAL, "hvk_weight_grad: workspace %zu B too small", ws_bytes);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hvk_bf16* gb = static_cast<const hvk_bf16*>(g);
  const hvk_bf16* xb = static_cast<const hvk_bf16*>(x);
  float* P = static_cast<float*>(ws);
  const bool wd = db != nullptr || xshift != nullptr;  // the shift needs the bias partials
  int rc;
  if (gx && p.var != V_96x384)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_weight_grad_gelu_x: M=%d N=%d K=%d", M, N, K);
  if (mg) {  // PatchMerging's reduction: the tile variants of its shapes (merge_plan_ok)
    switch (p.var) {
      case V_T4: rc = launch<6, 6, 2, 2, false, true>(gb, xb, P, wd, N, K, p, st, *mg); break;
      case V_T8A: rc = launch<6, 3, 2, 4, false, true>(gb, xb, P, wd, N, K, p, st, *mg); break;
      case V_B256: rc = launch<4, 4, 2, 4, false, true>(gb, xb, P, wd, N, K, p, st, *mg); break;
      case V_B128: rc = launch<4, 2, 2, 4, false, true>(gb, xb, P, wd, N, K, p, st, *mg); break;
      default: return hvk_set_error(HVK_EUNSUPPORTED, "hvk_merge_weight_grad: tile variant %d", p.var);
    }
  } else
  switch (gx ? -1 : p.var) {
    case -1: rc = launch<12, 3, 2, 2, true>(gb, xb, P, wd, N, K, p, st); break;
    case V_288x96: rc = launch<3, 9, 2, 2>(gb, xb, P, wd, N, K, p, st); break;
    case V_96x96: rc = launch<3, 3, 2, 2>(gb, xb, P, wd, N, K, p, st); break;
    case V_96x48: rc = launch<3, 3, 1, 2>(gb, xb, P, wd, N, K, p, st); break;
    case V_128x48: rc = launch<3, 4, 1, 2>(gb, xb, P, wd, N, K, p, st); break;
    case V_384x96: rc = launch<3, 12, 2, 2>(gb, xb, P, wd, N, K, p, st); break;
    case V_96x384: rc = launch<12, 3, 2, 2>(gb, xb, P, wd, N, K, p, st); break;
    case V_T8A: rc = launch<6, 3, 2, 4>(gb, xb, P, wd, N, K, p, st); break;
    case V_T8B: rc = launch<3, 6, 4, 2>(gb, xb, P, wd, N, K, p, st); break;
    case V_T8W: rc = launch<6, 6, 2, 4>(gb, xb, P, wd, N, K, p, st); break;
    case V_T8C: rc = launch<4, 3, 2, 4>(gb, xb, P, wd, N, K, p, st); break;
    case V_B256: rc = launch<4, 4, 2, 4>(gb, xb, P, wd, N, K, p, st); break;
    case V_B128: rc = launch<4, 2, 2, 4>(gb, xb, P, wd, N, K, p, st); break;
    default: rc = launch<6, 6, 2, 2>(gb, xb, P, wd, N, K, p, st); break;
  }
  if (rc != HVK_OK) return rc;
  const int ndw4 = N * K / 4;
  const int e4 = wd ? (int)(p.pstride / 4) : ndw4;
  // deep slab stacks (the stage-0 shapes: 256 chunks over few columns) get 32 chunk phases per
  // workgroup instead of 8, so each thread's dependent chain of slab reads is 4x shorter
  // (profiles/round4/dw_reduce_phases/: stage-0 proj / embed -1.3-2 us, 128-chunk merge +3 us)
  if (p.nchunk >= 256)
    hipLaunchKernelGGL(dw_reduce_kernel<32>, dim3((unsigned)((e4 + 31) / 32)), dim3(1024), 0, st,
                       reinterpret_cast<const float4*>(P), e4, ndw4, p.nchunk, p.pstride / 4,
                       reinterpret_cast<float4*>(dw), reinterpret_cast<float4*>(db), xshift, K);
  else
    hipLaunchKernelGGL(dw_reduce_kernel<8>, dim3((unsigned)((e4 + 31) / 32)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(P), e4, ndw4, p.nchunk, p.pstride / 4,
                       reinterpret_cast<float4*>(dw), reinterpret_cast<float4*>(db), xshift, K);
  HVK_CHECK_LAUNCH("hvk_weight_grad_reduce");
  return HVK_OK;
}

int hvk_weight_grad(const void* g, const void* x, float* dw, float* db, int M, int N, int K, void* ws,
                    size_t ws_bytes, void* stream) {
  return weight_grad(g, x, dw, db, M, N, K, ws, ws_bytes, stream, false);
}

int hvk_weight_grad_shift(const void* g, const void* x, const float* xshift, float* dw, float* db, int M, int N,
                          int K, void* ws, size_t ws_bytes, void* stream) {
  if (!xshift) return hvk_set_error(HVK_EINVAL, "hvk_weight_grad_shift: null xshift");
  return weight_grad(g, x, dw, db, M, N, K, ws, ws_bytes, stream, false, xshift);
}

static bool merge_plan_ok(int B, int H, int W, int C, int N, int& M, MergeGeo& g) {
  if (B <= 0 || H <= 0 || W <= 0 || H % 2 || W % 2 || C <= 0 || C % 8) return false;
  const long long m = (long long)B * (H / 2) * (W / 2);
  if (m >= (1ll << 21) || (long long)B * H * W * C >= (1ll << 31)) return false;  // hvk_merge_tok exactness
  M = (int)m;
  g.W = W;
  g.C = C;
  g.inv_wo = 1.0f / (float)(W / 2);
  Plan p;
  if (!plan(M, N, 4 * C, p)) return false;
  return p.var == V_T4 || p.var == V_T8A || p.var == V_B256 || p.var == V_B128;
}

int hvk_merge_weight_grad_supported(int B, int H, int W, int C, int N) {
  int M;
  MergeGeo g;
  return merge_plan_ok(B, H, W, C, N, M, g) ? 1 : 0;
}

// dW [N, 4C] of PatchMerging's reduction = gy [M, N]^T gather(x) with x [B, H W, C] the token rows
// (no bias); workspace hvk_weight_grad_workspace(M, N, 4C), M = B H W / 4
int hvk_merge_weight_grad(const void* gy, const void* x, float* dw, int B, int H, int W, int C, int N, void* ws,
                          size_t ws_bytes, void* stream) {
  int M;
  MergeGeo g;
  if (!merge_plan_ok(B, H, W, C, N, M, g))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_merge_weight_grad: B=%d H=%d W=%d C=%d N=%d", B, H, W, C, N);
  return weight_grad(gy, x, dw, nullptr, M, N, 4 * C, ws, ws_bytes, stream, false, nullptr, &g);
}

int hvk_weight_grad_gelu_x_supported(int M, int N, int K) {
  Plan p;
  return plan(M, N, K, p) && p.var == V_96x384 ? 1 : 0;
}

int hvk_weight_grad_gelu_x(const void* g, const void* h, float* dw, float* db, int M, int N, int K, void* ws,
                           size_t ws_bytes, void* stream) {
  return weight_grad(g, h, dw, db, M, N, K, ws, ws_bytes, stream, true);
}

}  // extern "C"
