// Whole-row MFMA GEMM for the stage-2 SwinV2 Linears (M = 50 176 tokens at bs256):
//   Y[M, N] = X[M, K] W[N, K]^T (+ bias)  -- F.linear of swinv2.py:58-62, 220, 262, 492 and the
//   input gradients (W = weight^T), epilogues EPI 0 (plain), 1 (fc1: h and GELU(h)), 2 (fc2's
//   input gradient through the activation: gh = (gy W) * GELU'(h), h read from Y2), 4 (qkv: q / k
//   head slices L2-normalised, q times the logit scale, swinv2.py:229-231).
//
// Why another tile: the 128-row tiles (gemm_tile.hip) run two workgroups per CU and stream
// (128 + 192) x 64 x 2 B from L2 per 1.57 M MACs, 0.026 B/MAC, while a CU's L2->LDS DMA path
// moves ~35 B/clk against 2 048 MAC/clk of MFMA: the k-loop is DMA-bound at <= 66 % of the MFMA
// rate, and on the N = 384 shapes 784 tiles fill 512 slots in 1.53 rounds.  Here ONE 512-thread
// workgroup per CU owns 13 row tiles x 384 columns (208 x 384):
//  * 2 (208 + 384) / (208 x 384) = 0.0148 B/MAC: the DMA stream (~30 B/clk at the MFMA rate) no
//    longer caps the loop;
//  * M = 50 176 = 3 136 row tiles -> 242 workgroups <= 256 CUs: an N = 384 product is ONE round
//    (the stage-2 fc2 / fc1-dgrad / qkv-dgrad / proj GEMMs), N = 1152 / 1536 three / four;
//  * K in steps of 32 through a 4-stage LDS ring filled by LDS-DMA (global_load_lds_dwordx4,
//    37 KB per stage, three stages in flight), one raw s_barrier per step, counted vmcnt;
//    64-B rows, 16-B chunk c of in-block row r at c ^ (r & 8 ? 2 : 0) (applied on the DMA's
//    global source; the fragment reads are bank-conflict free under the ds_read_b128 lane groups
//    of MI355X_MICROARCH.md §LDS);
//  * wave w (of 8) owns columns 48w .. 48w + 47 (3 MFMA tiles) of all 13 row tiles (156 f32
//    accumulators); W rows are permuted so a lane ends with 12 consecutive output columns;
//  * the output leaves through LDS: the 208 x 384 bf16 image (156 KB, the ring's space) is
//    written from the accumulators (+ bias, rounded), then stored as whole 768-B rows; the
//    EPI 1 / 4 math runs on the rounded values in that store pass (as the reference applies
//    GELU / F.normalize to the bf16 linear output).
// v_mfma_f32_16x16x32_bf16, f32 accumulation; results equal gemm_nt_kernel's bit for bit (same
// k order: sequential 32-deep steps; tests/test_gpu_wide.py).
#include "hvk_common.h"
#include "gemm_xr.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef __attribute__((address_space(1))) void* gbl_vptr_t;

constexpr int WMT = 13;                  // row tiles (16 tokens) per workgroup
constexpr int WBM = 16 * WMT;            // 208 rows
constexpr int WBN = 384;                 // columns per workgroup
constexpr int WAVES = 8, THREADS = 64 * WAVES;
constexpr int TW = WBN / 16 / WAVES;     // 3 column tiles per wave
constexpr int WCOLS = 16 * TW;           // 48 columns per wave
constexpr int BKW = 32;                  // k per ring stage
constexpr int NST = 4;                   // ring stages (three in flight)
constexpr int XBLK = WMT;                // X DMA blocks (16 rows x 64 B = 1 KB) per stage
constexpr int WBLK = WBN / 16;           // W DMA blocks per stage
constexpr int NBLK = XBLK + WBLK;        // 37
constexpr int NI = (NBLK + WAVES - 1) / WAVES;  // DMA instructions per wave and stage (5; 4 for waves >= 5)
constexpr int STAGE = NBLK * 1024;
constexpr int RING = NST * STAGE;        // 151 552 B
constexpr int IMG_ROW = WBN * 2;         // 768 B
constexpr int IMG = WBM * IMG_ROW;       // 159 744 B
constexpr int LDS = IMG > RING ? IMG : RING;
constexpr int CPR = WBN / 8;             // 16-B chunks per image row (48)
constexpr int STORE_ROUNDS = (WBM * CPR + THREADS - 1) / THREADS;  // 20
static_assert(LDS <= 163840, "one workgroup per CU");
static_assert(WBM * CPR % 4 == 0 && THREADS % 4 == 0 && CPR % 4 == 0, "quads hold one 32-column head");

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
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
// ring swizzle: 16-B chunk of in-block row r (0..15) -> chunk ^ rsw(r)
__device__ __forceinline__ int rsw(int r) { return (r & 8) ? 2 : 0; }
// W row permutation within a stage: LDS row p -> W row (column of Y) of the tile
__device__ __forceinline__ int wperm(int p) {
  const int w = p / WCOLS, q = p % WCOLS, t = q >> 4, m = q & 15;
  return WCOLS * w + 12 * (m >> 2) + 4 * t + (m & 3);
}
// output image: 16-B chunk c of row r at r * 768 + 16 (c ^ (r & 15))
__device__ __forceinline__ uint32_t img_off(int r, int byte) {
  const int c = byte >> 4;
  return (uint32_t)(r * IMG_ROW + 16 * (c ^ (r & 15)) + (byte & 15));
}
// quad (4 consecutive lanes) sums in the order (l0 + l1) + (l2 + l3): the group-of-4 sum of
// hvk_head_normalize8, whose lanes l, l^16 / l^32 hold the same chunks of a head
__device__ __forceinline__ float quad_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  return v;
}

template <int EPI>
__global__ __launch_bounds__(THREADS, 1) void gemm_wide_kernel(const hvk_bf16* __restrict__ X,
                                                              const hvk_bf16* __restrict__ Wt,
                                                              const float* __restrict__ bias,
                                                              hvk_bf16* __restrict__ Y,
                                                              hvk_bf16* __restrict__ Y2, int M, int N, int K,
                                                              int mtiles, float* __restrict__ rn,
                                                              const float* __restrict__ qscale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntiles = N / WBN;
  // XCD-aware decode: the column blocks of one row block share blockIdx % 8 (one L2)
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int nt = loc % ntiles, mt = (loc / ntiles) * 8 + xcd;
  if (mt >= mtiles) return;
  const int m0 = mt * WBM, n0 = nt * WBN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  const int KT = K / BKW;

  // DMA: wave w issues blocks j = w + 8i (i < NI, j < 37): j < 13 the X rows m0 + 16j .., else
  // W block j - 13.  Lane L -> in-block row L >> 2, LDS chunk L & 3 <- global chunk (L & 3) ^ rsw.
  const int lr = lane >> 2, lc = lane & 3;
  uint32_t src[NI];
  bool isx[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int j = wave + WAVES * i;
    isx[i] = j < XBLK;
    const int chunk = lc ^ rsw(lr);
    if (isx[i]) {
      int r = m0 + 16 * j + lr;
      if (r >= M) r = M - 1;  // rows past M: any valid row (never stored)
      src[i] = (uint32_t)r * K + 8 * chunk;
    } else {
      const int jj = j < NBLK ? j - XBLK : 0;
      src[i] = (uint32_t)(n0 + wperm(16 * jj + lr)) * K + 8 * chunk;
    }
  }
  const bool five = wave + WAVES * (NI - 1) < NBLK;  // this wave issues NI (else NI - 1) per stage
  auto issue = [&](int kt) {
    char* base = smem + (kt % NST) * STAGE;
    const int k0 = kt * BKW;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (i == NI - 1 && !five) break;
      const hvk_bf16* s = (isx[i] ? X : Wt) + src[i] + k0;
      __builtin_amdgcn_global_load_lds((gbl_vptr_t)s, (lds_vptr_t)(base + (wave + WAVES * i) * 1024), 16, 0, 0);
    }
  };

  hvk_f32x4 acc[WMT][TW];
#pragma unroll
  for (int a = 0; a < WMT; ++a)
#pragma unroll
    for (int t = 0; t < TW; ++t) acc[a][t] = hvk_f32x4{0, 0, 0, 0};

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < KT) issue(s);
  const uint32_t sw = 16 * (g ^ rsw(li));
  for (int kt = 0; kt < KT; ++kt) {
    // stage kt landed: the younger stages (up to two) may stay in flight
    const int younger = (kt + NST - 2 < KT - 1 ? kt + NST - 2 : KT - 1) - kt;
    if (younger >= 2) {
      if (five) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (younger == 1) {
      if (five) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // every wave's stage-kt DMA landed, and every wave is done reading stage kt - 1, whose
    // buffer the DMA below refills
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < KT) issue(kt + NST - 1);
    const uint32_t base = lds_u32(smem) + (kt % NST) * STAGE;
    const uint32_t aw = base + XBLK * 1024 + (WCOLS * wave + li) * 64 + sw;
    const uint32_t ax = base + li * 64 + sw;
    hvk_u32x4 ra[TW], rb[WMT];
    ra[0] = rd128<0>(aw);
    ra[1] = rd128<1024>(aw);
    ra[2] = rd128<2048>(aw);
    rb[0] = rd128<0>(ax);
    rb[1] = rd128<1024>(ax);
    rb[2] = rd128<2048>(ax);
    rb[3] = rd128<3072>(ax);
    rb[4] = rd128<4096>(ax);
    rb[5] = rd128<5120>(ax);
    rb[6] = rd128<6144>(ax);
    rb[7] = rd128<7168>(ax);
    rb[8] = rd128<8192>(ax);
    rb[9] = rd128<9216>(ax);
    rb[10] = rd128<10240>(ax);
    rb[11] = rd128<11264>(ax);
    rb[12] = rd128<12288>(ax);
    uint4 af[TW];
#define HVK_WIDE_ROW(MT_, CNT_)                                                       \
  {                                                                                   \
    asm volatile("s_waitcnt lgkmcnt(" #CNT_ ")" ::: "memory");                       \
    if (MT_ == 0) {                                                                   \
      af[0] = tie(ra[0]);                                                             \
      af[1] = tie(ra[1]);                                                             \
      af[2] = tie(ra[2]);                                                             \
    }                                                                                 \
    const uint4 bf = tie(rb[MT_]);                                                    \
    acc[MT_][0] = hvk_mfma16(af[0], bf, acc[MT_][0]);                                 \
    acc[MT_][1] = hvk_mfma16(af[1], bf, acc[MT_][1]);                                 \
    acc[MT_][2] = hvk_mfma16(af[2], bf, acc[MT_][2]);                                 \
  }
    HVK_WIDE_ROW(0, 12) HVK_WIDE_ROW(1, 11) HVK_WIDE_ROW(2, 10) HVK_WIDE_ROW(3, 9)
    HVK_WIDE_ROW(4, 8) HVK_WIDE_ROW(5, 7) HVK_WIDE_ROW(6, 6) HVK_WIDE_ROW(7, 5)
    HVK_WIDE_ROW(8, 4) HVK_WIDE_ROW(9, 3) HVK_WIDE_ROW(10, 2) HVK_WIDE_ROW(11, 1)
    HVK_WIDE_ROW(12, 0)
#undef HVK_WIDE_ROW
  }

  // ---- epilogue: accumulators (+ bias) -> bf16 image in LDS -> whole-row stores
  __builtin_amdgcn_s_barrier();  // every wave's ring reads are done (each waited lgkmcnt(0))
  asm volatile("" ::: "memory");
  const int c0 = WCOLS * wave + 12 * g;  // this lane's 12 columns of the tile
  float bv[12];
#pragma unroll
  for (int e = 0; e < 12; ++e) bv[e] = 0.f;
  if (bias) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(bias + n0 + c0 + 4 * q);
      bv[4 * q] = b.x; bv[4 * q + 1] = b.y; bv[4 * q + 2] = b.z; bv[4 * q + 3] = b.w;
    }
  }
  // EPI 2: the saved pre-activation h of this lane's 12 columns, two row tiles ahead
  constexpr int HD = 2;
  uint2 hq[EPI == 2 ? HD + 1 : 1][3];
  auto load_h = [&](int a) {
    if constexpr (EPI == 2) {
      int row = m0 + 16 * a + li;
      if (row >= M) row = M - 1;  // never stored
      const uint2* hp = reinterpret_cast<const uint2*>(Y2 + (size_t)row * N + n0 + c0);
#pragma unroll
      for (int q = 0; q < 3; ++q) hq[a % (HD + 1)][q] = hp[q];
    }
  };
#pragma unroll
  for (int a = 0; a < HD; ++a) load_h(a);
#pragma unroll
  for (int a = 0; a < WMT; ++a) {
    const int r = 16 * a + li;
    if (a + HD < WMT) load_h(a + HD);
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      // columns c0 + 4t .. + 3 = acc rows 4g .. 4g + 3 of column tile t (wperm)
      float v0 = acc[a][t][0] + bv[4 * t], v1 = acc[a][t][1] + bv[4 * t + 1];
      float v2 = acc[a][t][2] + bv[4 * t + 2], v3 = acc[a][t][3] + bv[4 * t + 3];
      if constexpr (EPI == 2) {  // gh = (gy W) * GELU'(h) (the fc2 input gradient, swinv2.py:60-61)
        const uint2 h2 = hq[a % (HD + 1)][t];
        const hvk_gelu::f32x2 d0 = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{hvk_lo(h2.x), hvk_hi(h2.x)});
        const hvk_gelu::f32x2 d1 = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{hvk_lo(h2.y), hvk_hi(h2.y)});
        v0 *= d0.x; v1 *= d0.y; v2 *= d1.x; v3 *= d1.y;
      }
      const uint2 pk = make_uint2(hvk_pack2(v0, v1), hvk_pack2(v2, v3));
      *reinterpret_cast<uint2*>(smem + img_off(r, 2 * (c0 + 4 * t))) = pk;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // store pass: thread i takes chunks c = i + 512 s of the image (row c / 48, chunk c % 48):
  // quads of consecutive threads hold the four 8-column chunks of one 32-column head
  const int qk_cols = 2 * (N / 3);
  uint4 v[STORE_ROUNDS];
#pragma unroll
  for (int s = 0; s < STORE_ROUNDS; ++s) {
    int c = threadIdx.x + THREADS * s;
    if (c >= WBM * CPR) c = WBM * CPR - 1;  // whole quads past the end: read a valid chunk, never stored
    const int r = c / CPR, ch = c - r * CPR;
    v[s] = *reinterpret_cast<const uint4*>(smem + img_off(r, 16 * ch));
  }
#pragma unroll
  for (int s = 0; s < STORE_ROUNDS; ++s) {
    const int c = threadIdx.x + THREADS * s;
    const int r = c / CPR, ch = c - r * CPR;
    const int row = m0 + r, col = n0 + 8 * ch;
    const bool ok = c < WBM * CPR && row < M;
    uint4 out = v[s];
    if constexpr (EPI == 4) {
      // F.normalize of the q / k head slices (swinv2.py:229) on the rounded values, q times
      // scale_h * log2e (hvk_head_normalize8's arithmetic, the lanes of a head in a quad)
      typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
      auto d2 = [](uint32_t w, float a) {
        return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, w), __builtin_bit_cast(bf16x2_t, w), a,
                                               false);
      };
      float ss = d2(out.w, d2(out.z, d2(out.y, d2(out.x, 0.f))));
      ss = quad_sum(ss);
      const float rq = __builtin_amdgcn_rsqf(fmaxf(ss, 1e-24f));
      if (col < qk_cols) {
        const float post = (qscale && col < N / 3) ? qscale[col / 32] * HVK_LOG2E : 1.f;
        const float mlt = rq * post;
        float f[8];
        hvk_unpack8(out, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] *= mlt;
        out = hvk_pack8(f);
        if (ok && (ch & 3) == 0) rn[(size_t)row * (qk_cols / 32) + col / 32] = rq;
      }
    }
    if (!ok) continue;
    hvk_u32x4* dst = reinterpret_cast<hvk_u32x4*>(Y + (size_t)row * N + col);
    if (EPI == 1 && (HVK_NT_SAVED & 1))  // h: read again only by the backward
      __builtin_nontemporal_store(__builtin_bit_cast(hvk_u32x4, out), dst);
    else
      *dst = __builtin_bit_cast(hvk_u32x4, out);
    if constexpr (EPI == 1)  // GELU of the rounded pre-activation, as the reference
      *reinterpret_cast<hvk_u32x4*>(Y2 + (size_t)row * N + col) = __builtin_bit_cast(hvk_u32x4, hvk_gelu8_bf16(out));
  }
}

template <int EPI>
int launch_wide_(const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2, int M, int N,
                 int K, hipStream_t st, float* rn, const float* qscale) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_wide_kernel<EPI>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS) != hipSuccess)
      return hvk_set_error(HVK_EHIP, "hvk_gemm_wide: %d B of LDS refused", LDS);
    attr = true;
  }
  const int mtiles = (M + WBM - 1) / WBM;
  const dim3 grid((mtiles + 7) / 8 * 8 * (N / WBN));
  const double bytes = 2.0 * ((double)M * K + (double)N * K + (double)M * N) + (EPI == 1 || EPI == 2 ? 2.0 * M * N : 0.0) +
                       (EPI == 4 ? 4.0 * M * (2.0 * N / 96.0) : 0.0);
  hvk_timer_shape("gemm_wide", EPI, WBM, M, N, K, bytes);
  HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, 2.0 * M * N * K, (gemm_wide_kernel<EPI>), grid, dim3(THREADS), LDS, st, X, W,
                     bias, Y, Y2, M, N, K, mtiles, rn, qscale);
  HVK_CHECK_LAUNCH("hvk_gemm_wide");
  return HVK_OK;
}

}  // namespace

// the wide tile where it is built: N a multiple of 384, K of 32, element offsets in 32 bits, and
// at least one full round of 208-row blocks per 8 XCDs (M >= 8 x 208); -1 otherwise
namespace hvk_wide {
bool supported(int M, int N, int K) {
  return N % WBN == 0 && K % BKW == 0 && K >= BKW && M >= 8 * WBM && (size_t)M * K < (1u << 31) &&
         (size_t)N * K < (1u << 31);
}
int launch(int epi, const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2, int M,
           int N, int K, hipStream_t st, float* rn, const float* qscale) {
  if (!supported(M, N, K)) return -1;
  switch (epi) {
    case 0: return launch_wide_<0>(X, W, bias, Y, Y2, M, N, K, st, rn, qscale);
    case 1: return launch_wide_<1>(X, W, bias, Y, Y2, M, N, K, st, rn, qscale);
    case 2: return launch_wide_<2>(X, W, bias, Y, Y2, M, N, K, st, rn, qscale);
    case 4: return launch_wide_<4>(X, W, bias, Y, Y2, M, N, K, st, rn, qscale);
    default: return -1;
  }
}
}  // namespace hvk_wide
