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

#include "hvk_common.h"

// experiment builds (tools/probe/Makefile, NOT the product): 1 no MFMA, 2 no stores, 3 no DMA,
// 4 per-workgroup phase timestamps (hvk_gemm_probe_read, tools/gemm_timeline.py)
#ifndef HVK_GEMM_PROBE
#define HVK_GEMM_PROBE 0
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

template <int EPI, bool PIPE, int TN>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const hvk_bf16* __restrict__ X,
                                                        const hvk_bf16* __restrict__ Wt,
                                                        const float* __restrict__ bias,
                                                        hvk_bf16* __restrict__ Y,
                                                        hvk_bf16* __restrict__ Y2, int M, int N,
                                                        int K, int mtiles) {
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
    xsrc[i] = (size_t)xr * K + 8 * (lc ^ (row & 7));
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
#pragma unroll
    for (int i = 0; i < TN; ++i)
      __builtin_amdgcn_global_load_lds((gbl_vptr_t)(Wt + wsrc[i] + k0),
                                       (lds_vptr_t)(base + (wave + 4 * i) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((gbl_vptr_t)(X + xsrc[i] + k0),
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
  issue(0, 0);
  if (KT > 1) issue(1, 1);
  for (int kt = 0; kt < KT; ++kt) {
    // this k-step's tile has landed (the next one's TN + 4 DMAs per wave may stay in flight)
    if (kt + 1 < KT)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(TN + 4) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
      mfma_half(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_half(1);
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
  // EPI 2: the 8 h vectors of this lane, loaded as one batch before the epilogue math
  uint4 hp[EPI == 2 ? 4 : 1][TN / 2];
  if (EPI == 2) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      int row = m0 + 64 * wm + 16 * b + li;
      if (row >= M) row = M - 1;
#pragma unroll
      for (int j = 0; j < TN / 2; ++j)
        hp[b][j] = *reinterpret_cast<const uint4*>(Y2 + (size_t)row * N + n0 + 16 * TN * wn + 32 * j + 8 * g);
    }
  }
  // epilogue: lane (li, g) holds, for m-tile b and n-tile pair (2j, 2j+1), row
  // m0 + 64wm + 16b + li and columns n0 + 16 TN wn + 32j + 8g .. +7
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int row = m0 + 64 * wm + 16 * b + li;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < TN / 2; ++j) {
      const int col = n0 + 16 * TN * wn + 32 * j + 8 * g;
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[2 * j][b][r];
        v[4 + r] = acc[2 * j + 1][b][r];
      }
      if (EPI != 2 && bias) {
        const float4 b0 = *reinterpret_cast<const float4*>(bias + col);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + col + 4);
        v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
        v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
      }
      if (EPI == 2) {  // gh = (gy w) * GELU'(h): h (Y2) read in the output layout
        float hf[8];
        hvk_unpack8(hp[b][j], hf);
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const hvk_gelu::f32x2 d = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{hf[e], hf[e + 1]});
          v[e] *= d.x;
          v[e + 1] *= d.y;
        }
        *reinterpret_cast<uint4*>(Y + (size_t)row * N + col) = hvk_pack8(v);
        continue;
      }
      const uint4 hv = hvk_pack8(v);
      *reinterpret_cast<uint4*>(Y + (size_t)row * N + col) = hv;
      if (EPI == 1) {
        float u[8];
        hvk_unpack8(hv, u);  // GELU of the rounded pre-activation, as the reference
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            const hvk_gelu::f32x2 y = hvk_gelu::gelu2(hvk_gelu::f32x2{u[e], u[e + 1]});
            u[e] = y.x;
            u[e + 1] = y.y;
          }
        *reinterpret_cast<uint4*>(Y2 + (size_t)row * N + col) = hvk_pack8(u);
      }
    }
  }
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

static bool tile_pipe() {
  static const int v = [] {
    const char* e = getenv("HVK_TILE_PIPE");
    return e ? atoi(e) : 1;
  }();
  return v != 0;
}

template <int EPI, bool PIPE, int TN>
int launch_tile_(const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2,
                 int M, int N, int K, hipStream_t st) {
  using T = TileCfg<TN>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<EPI, PIPE, TN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
    attr = true;
  }
  const int mtiles = (M + BM - 1) / BM;
  const int mpad = (mtiles + 7) / 8 * 8;
  const dim3 grid(mpad * (N / T::BN));
  HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, 2.0 * M * N * K, (gemm_nt_kernel<EPI, PIPE, TN>), grid, dim3(256),
                     T::LDS, st, X, W, bias, Y, Y2, M, N, K, mtiles);
  HVK_CHECK_LAUNCH("hvk_gemm_tile");
  return HVK_OK;
}

// 128 x 128 or 128 x 192 tiles
template <int EPI>
int launch_tile(const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2,
                int M, int N, int K, hipStream_t st) {
  // 128 x 192 also where 192 | N and the tile is not the narrow N = 384, K < 1536 case
  // (tools/bench_gemm.py, interleaved: 3-25 % faster on the stage-2/3 shapes, 6 % slower on
  // the stage-2 projection); HVK_TILE_WIDE=0 / 1 forces 128 / 192 columns where both divide N
  static const int force = [] {
    const char* e = getenv("HVK_TILE_WIDE");
    return e ? atoi(e) : -1;
  }();
  const bool wide = N % TileCfg<6>::BN == 0 && (force >= 0 ? force == 1 : (N > 384 || K >= 1536));
  if (N % TileCfg<4>::BN == 0 && !wide)
    return tile_pipe() ? launch_tile_<EPI, true, 4>(X, W, bias, Y, Y2, M, N, K, st)
                       : launch_tile_<EPI, false, 4>(X, W, bias, Y, Y2, M, N, K, st);
  return tile_pipe() ? launch_tile_<EPI, true, 6>(X, W, bias, Y, Y2, M, N, K, st)
                     : launch_tile_<EPI, false, 6>(X, W, bias, Y, Y2, M, N, K, st);
}

}  // namespace

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
