// Persistent row-range GEMM for the stage-2/3 SwinV2 Linears (gfx950):
//   Y[M, N] = X[M, K] W[N, K]^T (+ bias) (EPI 0) or the fc1 form h = Y + bias, GELU(h) (EPI 1)
// -- F.linear of swinv2.py:58-62, 220, 262 and the input gradients, the shapes where N is a
// multiple of 384 (qkv / proj / fc1 / fc2 and their input gradients at C = 384 and 768).
//
// Why another tiled kernel.  gemm_nt_kernel (gemm_tile.hip) runs 128 x 128 / 128 x 192 tiles,
// two workgroups per CU.  Two things bound it: (1) the L2 -> LDS stream: a CU's tile area sets
// the bytes it must stage per MFMA cycle, 4096 (1/BM + 1/BN) B/clk at full MFMA rate = 53 B/clk
// for 128 x 192, against the ~35-40 B/clk per CU that LDS-DMA sustains from L2 (DESIGN.md §3:
// 64 KB per 0.77 us k-step); (2) wave quantisation: M = 50 176 gives 784 tiles of 128 x 192 for
// 512 resident slots = 1.53 rounds, i.e. the second round runs half empty.
// Here ONE 8-wave workgroup per CU (256 workgroups, persistent) owns a balanced row range of
// n = MG-1 or MG 16-row granules (MG = 13: up to 208 rows, 12.25 on average at M = 50 176) and
// walks the 384-column N-tiles of its items: 4096 (1/208 + 1/384) = 30 B/clk, and the items are
// dealt so every workgroup gets the same number (the host picks the row-group count G with
// G * N/384 a multiple of 256).  K streams in 64-deep steps through two LDS stages of
// 48 KB (W) + MG * 2 KB (X) filled by LDS-DMA (global_load_lds_dwordx4, 1 KB per instruction,
// XOR-swizzled 16-B chunks, as gemm_nt_kernel), and the step stream runs across item
// boundaries: the next item's first two stages are in flight while an item's epilogue packs and
// stores.  Waves: 2 (token halves of the range) x 4 (96-column slices); a wave holds up to
// 7 x 6 accumulators of 16 x 16 (168 VGPRs), computes Y^T = W X^T on v_mfma_f32_16x16x32_bf16
// with the W rows of each 32-row pair permuted so a lane owns 8 consecutive output columns
// (one 16-B store).  Output stores are buffer stores over [0, M N) so rows past M drop without
// an exec branch, and every wave issues the same number of stores per item (the waits below
// count them).  The bias vector is staged in LDS once per launch.
#include "gemm_xr.h"

#include "hvk_common.h"

namespace {

typedef __attribute__((address_space(3))) void* xr_lds_ptr;
typedef __attribute__((address_space(1))) void* xr_gbl_ptr;

constexpr int XBK = 64;   // k per step
constexpr int XBN = 384;  // columns per item

template <int MG>
struct XrCfg {
  static constexpr int WBLK = XBN / 8;               // W image: 48 blocks of 8 rows x 128 B
  static constexpr int XBLK = 2 * MG;                // X image blocks
  static constexpr int BLK = WBLK + XBLK;            // 1-KB DMA instructions per stage
  static constexpr int STAGE = BLK * 1024;
  static constexpr int XOFF = WBLK * 1024;           // X image offset inside a stage
  static constexpr int BIAS = 2 * STAGE;             // bias vector (f32, <= 3072 columns)
  static constexpr int LDS = BIAS + 3072 * 4;
  static constexpr int DHI = (BLK + 7) / 8;          // DMA instructions of waves < NHI
  static constexpr int NHI = BLK % 8 ? BLK % 8 : 8;
  static constexpr int DLO = BLK / 8;
  static constexpr int GR = (MG + 1) / 2;            // granules of a wave row, at most
  static constexpr int GMIN = (MG - 1) / 2;          // ... at least (items have >= MG-1 granules)
};
static_assert(XrCfg<13>::LDS <= 160 * 1024, "LDS budget");

__device__ __forceinline__ int xr_perm_row(int p) {  // as gemm_tile.hip perm_row
  const int t = p >> 4, m = p & 15;
  return 32 * (t >> 1) + 8 * (m >> 2) + 4 * (t & 1) + (m & 3);
}
__device__ __forceinline__ uint32_t xr_lds_u32(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
template <int OFF>
__device__ __forceinline__ hvk_u32x4 xr_rd128(uint32_t a) {
  hvk_u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
// r[B .. N-1] = 16-B reads at a + 2048 B (one 16-row fragment tile apart), offsets as immediates
template <int B, int N>
__device__ __forceinline__ void xr_rd_tiles(hvk_u32x4* r, uint32_t a) {
  if constexpr (B < N) {
    r[B] = xr_rd128<2048 * B>(a);
    xr_rd_tiles<B + 1, N>(r, a);
  }
}
__device__ __forceinline__ uint4 xr_tie(hvk_u32x4 v) {
  asm volatile("" : "+v"(v));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// 16-B buffer load from inline asm: invisible to hipcc's waitcnt pass (a compiler-visible load
// makes it wait vmcnt(0) before the first use, i.e. drain every store and DMA in flight); the
// kernel counts vmcnt itself.  Descriptor {base, num_records, flags} in SGPRs; offsets past
// num_records read 0.
__device__ __forceinline__ hvk_u32x4 xr_bld16(hvk_u32x4 rs, uint32_t off) {
  hvk_u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(rs) : "memory");
  return v;
}
__device__ __forceinline__ hvk_u32x4 xr_srsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)base;
  return hvk_u32x4{(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b),
                   (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)),
                   (uint32_t)__builtin_amdgcn_readfirstlane(bytes), 0x00020000u};
}

// s_waitcnt vmcnt(N) for a runtime-selected N among the compile-time values used below
template <int N>
__device__ __forceinline__ void xr_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int EPI, int MG>
__global__ __launch_bounds__(512, 1) void gemm_xr_kernel(hvk_xr::Args p) {
  using C = XrCfg<MG>;
  constexpr int EPS = (EPI == 1 ? 2 : 1) * 3;  // stores per granule and wave
  // stores of a wave per item, at least (EPI 2 stores every slot, the unused ones out of range)
  constexpr int EMIN = (EPI == 2 ? C::GR : C::GMIN) * EPS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int li = lane & 15, g = lane >> 4;
  const int wm = wave >> 2, wn = wave & 3;
  const bool hi = wave < C::NHI;  // issues DHI DMA instructions per stage (else DLO)

  float* sbias = reinterpret_cast<float*>(smem + C::BIAS);
  if (p.bias)
    for (int i = tid; i < p.N; i += 512) sbias[i] = p.bias[i];
  __syncthreads();

  const int KT = p.K / XBK;
  const int total = p.ipw * KT;
  const int item0 = blockIdx.x * p.ipw;
  const int lr = lane >> 3, lc = lane & 7;

  // DMA of flat step s (item item0 + s / KT, k-step s % KT) into stage s & 1: block b of the
  // stage (b < 48: W image rows 8b .. 8b+7; else X image block b - 48) is issued by wave b % 8
  auto issue = [&](int s) {
    const int it = item0 + s / KT, kt = s - (s / KT) * KT;
    const int r = it / p.NT, nt = it - r * p.NT;
    const int g0 = (int)((long long)r * p.NG / p.G);
    const int k0 = kt * XBK;
    char* base = smem + (s & 1) * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::DHI; ++i) {
      const int b = wave + 8 * i;
      if (i == C::DHI - 1 && !hi) break;
      const int row = 8 * b + lr;  // image row (W rows 0..383, then X rows)
      const hvk_bf16* src;
      if (b < C::WBLK) {
        src = p.W + (size_t)(nt * XBN + xr_perm_row(row)) * p.K;
      } else {
        int xr = 16 * g0 + row - 8 * C::WBLK;
        if (xr >= p.M) xr = p.M - 1;  // rows past M: any valid row (never stored)
        src = p.X + (size_t)xr * p.K;
      }
      __builtin_amdgcn_global_load_lds((xr_gbl_ptr)(src + k0 + 8 * (lc ^ (row & 7))),
                                       (xr_lds_ptr)(base + b * 1024), 16, 0, 0);
    }
  };

  const __amdgpu_buffer_rsrc_t ry = hvk_rsrc(p.Y, (size_t)p.M * p.N * 2);
  const __amdgpu_buffer_rsrc_t ry2 = hvk_rsrc(EPI == 1 ? p.Y2 : p.Y, (size_t)p.M * p.N * 2);


  hvk_f32x4 acc[6][C::GR];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < C::GR; ++b) acc[a][b] = hvk_f32x4{0, 0, 0, 0};

  issue(0);
  if (total > 1) issue(1);

  // this item's granules of this wave row: [gb, gb + gn)
  int gn = 0, gb = 0, n0 = 0, row0 = 0;
  auto item_geom = [&](int s) {
    const int it = item0 + s / KT;
    const int r = it / p.NT, nt = it - r * p.NT;
    const int g0 = (int)((long long)r * p.NG / p.G), g1 = (int)((long long)(r + 1) * p.NG / p.G);
    const int n = g1 - g0, h0 = (n + 1) >> 1;
    gb = wm ? h0 : 0;
    gn = wm ? n - h0 : h0;
    n0 = nt * XBN;
    row0 = 16 * (g0 + gb);
  };
  item_geom(0);
  // EPI 2: the saved pre-activation h [M, N] (Y2), read in the output layout (3 x 16 B per granule)
  const hvk_u32x4 rh = xr_srsrc(EPI == 2 ? p.Y2 : p.Y, (uint32_t)((size_t)p.M * p.N * 2));

  for (int s = 0; s < total; ++s) {
    const int kt = s % KT;
    // stage s landed: younger than its DMA are DMA(s+1) and the stores of an item that ended
    // at step s-1 or s-2 (KT >= 2, so at most one)
    const bool d = s + 1 < total;
    const bool e = (s >= 1 && kt == 0) || (s >= 2 && kt == 1);
    if (hi) {
      if (d && e) xr_vmcnt<C::DHI + EMIN>();
      else if (d) xr_vmcnt<C::DHI>();
      else if (e) xr_vmcnt<EMIN>();
      else xr_vmcnt<0>();
    } else {
      if (d && e) xr_vmcnt<C::DLO + EMIN>();
      else if (d) xr_vmcnt<C::DLO>();
      else if (e) xr_vmcnt<EMIN>();
      else xr_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const uint32_t sbase = xr_lds_u32(smem) + (s & 1) * C::STAGE;
    const uint32_t aw = sbase + (96 * wn + li) * 128;
    const uint32_t ax = sbase + C::XOFF + (16 * gb + li) * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t sw = ((4 * ks + g) ^ (li & 7)) << 4;
      hvk_u32x4 ra[6], rb[C::GR];
      xr_rd_tiles<0, 6>(ra, aw + sw);
      xr_rd_tiles<0, C::GR>(rb, ax + sw);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint4 af[6], bf[C::GR];
#pragma unroll
      for (int t = 0; t < 6; ++t) af[t] = xr_tie(ra[t]);
#pragma unroll
      for (int b = 0; b < C::GR; ++b) bf[b] = xr_tie(rb[b]);
#pragma unroll
      for (int b = 0; b < C::GR; ++b)
        if (b < C::GMIN || b < gn)
#pragma unroll
          for (int t = 0; t < 6; ++t) acc[t][b] = hvk_mfma16(af[t], bf[b], acc[t][b]);
    }
    __builtin_amdgcn_s_barrier();  // every wave is done with stage s & 1
    asm volatile("" ::: "memory");
    if (s + 2 < total) issue(s + 2);

    if (EPI == 2 && kt == KT - 1) {
      // ---- epilogue, fc2's input gradient through GELU': gh = (gy w) * GELU'(h).  Straight-line
      // over every granule slot of the wave row (slots past this item's granules store at an
      // offset past the buffer: dropped), h of the next granule in flight.  Younger than h(b) when
      // it is waited for: the 3 stores of granule b-1 and the 3 loads of h(b+1); DMA(s+2), issued
      // just before h(0), lands first.
      hvk_u32x4 hq[2][3];
      auto h_load = [&](int b, hvk_u32x4 (&dst)[3]) {
        const uint32_t roff = (uint32_t)(row0 + 16 * b + li) * (uint32_t)p.N * 2u;
#pragma unroll
        for (int j = 0; j < 3; ++j) dst[j] = xr_bld16(rh, roff + (uint32_t)(n0 + 96 * wn + 32 * j + 8 * g) * 2u);
      };
      h_load(0, hq[0]);
#pragma unroll
      for (int b = 0; b < C::GR; ++b) {
        if (b + 1 < C::GR) h_load(b + 1, hq[(b + 1) & 1]);
        if (b >= 1 && b + 1 < C::GR) xr_vmcnt<6>();
        else if (b >= 1 || b + 1 < C::GR) xr_vmcnt<3>();
        else xr_vmcnt<0>();
        uint4 hv[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) hv[j] = xr_tie(hq[b & 1][j]);
        const uint32_t roff = (b < C::GMIN || b < gn) ? (uint32_t)(row0 + 16 * b + li) * (uint32_t)p.N * 2u
                                                     : HVK_OOB;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          float v[8], hf[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[2 * j][b][r];
            v[4 + r] = acc[2 * j + 1][b][r];
          }
          hvk_unpack8(hv[j], hf);
#pragma unroll
          for (int e2 = 0; e2 < 8; e2 += 2) {
            const hvk_gelu::f32x2 dd = hvk_gelu::gelu_grad2(hvk_gelu::f32x2{hf[e2], hf[e2 + 1]});
            v[e2] *= dd.x;
            v[e2 + 1] *= dd.y;
          }
          hvk_bst16(ry, roff + (uint32_t)(n0 + 96 * wn + 32 * j + 8 * g) * 2u, hvk_pack8(v));
        }
      }
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < C::GR; ++b) acc[a][b] = hvk_f32x4{0, 0, 0, 0};
      if (s + 1 < total) item_geom(s + 1);
    } else if (kt == KT - 1) {
      // ---- epilogue of this item: bias (LDS), pack, then all stores back to back
      // column pair j at a time: its 8 bias values (inline-asm LDS reads: a plain one would make
      // hipcc drain the DMA in flight first), then its stores for every granule
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        float bv[8];
        if (p.bias) {
          const uint32_t bb = xr_lds_u32(sbias) + (uint32_t)(n0 + 96 * wn + 32 * j + 8 * g) * 4u;
          const hvk_u32x4 b0 = xr_rd128<0>(bb), b1 = xr_rd128<16>(bb);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const uint4 u0 = xr_tie(b0), u1 = xr_tie(b1);
          bv[0] = __uint_as_float(u0.x); bv[1] = __uint_as_float(u0.y);
          bv[2] = __uint_as_float(u0.z); bv[3] = __uint_as_float(u0.w);
          bv[4] = __uint_as_float(u1.x); bv[5] = __uint_as_float(u1.y);
          bv[6] = __uint_as_float(u1.z); bv[7] = __uint_as_float(u1.w);
        } else {
#pragma unroll
          for (int e2 = 0; e2 < 8; ++e2) bv[e2] = 0.f;
        }
        const uint32_t coff = (uint32_t)(n0 + 96 * wn + 32 * j + 8 * g) * 2u;
#pragma unroll
        for (int b = 0; b < C::GR; ++b) {
          if (b >= C::GMIN && b >= gn) break;
          const uint32_t off = (uint32_t)(row0 + 16 * b + li) * (uint32_t)p.N * 2u + coff;
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[2 * j][b][r] + bv[r];
            v[4 + r] = acc[2 * j + 1][b][r] + bv[4 + r];
          }
          const uint4 hv = hvk_pack8(v);
          if (EPI == 1) {
            hvk_bst16_nt(ry, off, hv);  // h: read again only by the backward
            hvk_bst16(ry2, off, hvk_gelu8_bf16(hv));
          } else {
            hvk_bst16(ry, off, hv);
          }
        }
      }
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < C::GR; ++b) acc[a][b] = hvk_f32x4{0, 0, 0, 0};
      if (s + 1 < total) item_geom(s + 1);
    }
  }
}

template <int EPI, int MG>
int launch_(const hvk_xr::Args& a, hipStream_t st) {
  using C = XrCfg<MG>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_xr_kernel<EPI, MG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, 2.0 * a.M * a.N * a.K, (gemm_xr_kernel<EPI, MG>), dim3(256), dim3(512),
                     C::LDS, st, a);
  HVK_CHECK_LAUNCH("hvk_gemm_xr");
  return HVK_OK;
}

}  // namespace

namespace hvk_xr {

// Plan: G row groups of the NG = ceil(M / 16) granules, G * NT items (NT = N / 384) dealt
// 256 ways; the smallest G (largest groups) with G * NT % 256 == 0 and groups of MG-1 or MG
// granules for MG = 13 or 7.  Returns false when no plan fits (the caller keeps gemm_nt_kernel).
bool plan(int M, int N, int K, Args& a, int& mg) {
  if (M <= 0 || N % XBN || N > 3072 || K % XBK || K < 2 * XBK) return false;
  if ((long long)M * N * 2 >= (1ll << 31) || (long long)M * K >= (1ll << 31) || (long long)N * K >= (1ll << 31))
    return false;
  const int NG = (M + 15) / 16, NT = N / XBN;
  for (int G = 1; G <= NG; ++G) {
    if ((G * NT) % 256) continue;
    const int lo = NG / G, hi = (NG + G - 1) / G;
    for (int m : {13, 7}) {
      if (hi <= m && lo >= m - 1) {
        a.M = M, a.N = N, a.K = K, a.NG = NG, a.G = G, a.NT = NT, a.ipw = G * NT / 256;
        mg = m;
        return true;
      }
    }
    if (hi < 6) break;  // groups only get smaller
  }
  return false;
}

int launch(int epi, const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2, int M,
           int N, int K, hipStream_t st) {
  Args a;
  int mg = 0;
  if (!plan(M, N, K, a, mg)) return -1;
  a.X = X, a.W = W, a.bias = epi == 2 ? nullptr : bias, a.Y = Y, a.Y2 = Y2;
  if (epi == 2) return mg == 13 ? launch_<2, 13>(a, st) : launch_<2, 7>(a, st);
  if (epi == 1) return mg == 13 ? launch_<1, 13>(a, st) : launch_<1, 7>(a, st);
  return mg == 13 ? launch_<0, 13>(a, st) : launch_<0, 7>(a, st);
}

}  // namespace hvk_xr
