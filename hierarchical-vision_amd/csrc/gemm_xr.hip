// Persistent row-range GEMM for the stage-2/3 SwinV2 Linears (gfx950):
//   Y[M, N] = X[M, K] W[N, K]^T (+ bias) (EPI 0), the fc1 form h = Y + bias, GELU(h) (EPI 1), or
//   fc2's input gradient through the activation gh = (X W^T) * GELU'(h) (EPI 2)
// -- F.linear of swinv2.py:58-62, 220, 262 and the input gradients, where N is a multiple of 192.
//
// Why another tiled kernel.  gemm_nt_kernel (gemm_tile.hip) runs 128 x 128 / 128 x 192 tiles,
// two workgroups per CU, two barriers per 64-deep k-step and the next step's LDS-DMA issued one
// step ahead: its k-loop waits on the DMA it issued one step earlier, and
// M = 50 176 gives 784 tiles of 128 x 192 for 512 resident slots (1.53 rounds).
// Here ONE 8-wave workgroup per CU (256 workgroups, persistent) owns a balanced row range of
// 12 or 13 16-row granules (M = 50 176: 12.25 on average) and walks the 192-column N-tiles of
// its items; the host picks the row-group count G with G * N/192 a multiple of 256, so every
// workgroup gets the same number of items.  K streams in 64-deep steps through a THREE-stage
// LDS ring (26 KB of X rows + 24 KB of W rows per stage, filled by LDS-DMA:
// global_load_lds_dwordx4, 1 KB per instruction, 16-B chunks XOR-swizzled by row as in
// gemm_nt_kernel), with ONE barrier per step: after the barrier at the top of step s every wave
// has finished reading stage (s-1) % 3, so the DMA of step s+2 goes into it right away and has
// two steps to land.  The step stream runs across item boundaries (the next item's first stages
// are in flight during an item's epilogue).  Waves: 4 (granule quarters of the range) x 2
// (96-column halves); a wave holds up to 4 x 6 accumulators of 16 x 16 and reads both k-halves'
// fragments at once, the first half's MFMAs starting when its reads are back.  Y^T = W X^T on
// v_mfma_f32_16x16x32_bf16 with the W rows of each 32-row pair permuted so a lane owns 8
// consecutive output columns (one 16-B store).  Stores are buffer stores over [0, M N): rows
// past M drop without an exec branch; every wave issues a fixed count per item (the vmcnt
// waits count them).  Bias and EPI 2's h are loaded by inline-asm buffer loads that hipcc's
// waitcnt pass does not see (a visible load makes it wait vmcnt(0), draining the DMA ring).
// Accumulation order (k ascending, 32 per MFMA) and epilogue math equal gemm_nt_kernel's: the
// outputs are bit-identical (tests/test_gpu_linear.py).
#include "gemm_xr.h"

#include "hvk_common.h"

namespace {

typedef __attribute__((address_space(3))) void* xr_lds_ptr;
typedef __attribute__((address_space(1))) void* xr_gbl_ptr;

constexpr int XBK = 64;    // k per step
constexpr int XBN = 192;   // columns per item
constexpr int MG = 13;     // granules per item, at most (at least MG - 1)
constexpr int NSTAGE = 3;  // LDS ring depth
constexpr int WBLK = XBN / 8;                // W image: 24 blocks of 8 rows x 128 B
constexpr int XBLK = 2 * MG;                 // X image: 26 blocks
constexpr int BLK = WBLK + XBLK;             // 1-KB DMA instructions per stage (50)
constexpr int STAGE = BLK * 1024;
constexpr int XOFF = WBLK * 1024;            // X image offset inside a stage
constexpr int LDS = NSTAGE * STAGE;          // 150 KB
constexpr int DHI = (BLK + 7) / 8;           // DMA instructions of waves < NHI (7)
constexpr int NHI = BLK % 8 ? BLK % 8 : 8;   // (2)
constexpr int DLO = BLK / 8;                 // (6)
constexpr int GR = (MG + 3) / 4;             // granules of a wave row, at most (4)
constexpr int GMIN = (MG - 1) / 4;           // ... at least (3)
static_assert(LDS <= 160 * 1024, "LDS budget");

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
// 16-B buffer load from inline asm (see the header comment); descriptor {base, num_records,
// flags} in SGPRs, offsets past num_records read 0
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
template <int N>
__device__ __forceinline__ void xr_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// vmcnt(D * d + E * e) for this wave's DMA count D (DHI or DLO)
template <int E>
__device__ __forceinline__ void xr_wait_stage(bool hi, bool d, bool e) {
  if (hi) {
    if (d && e) xr_vmcnt<DHI + E>();
    else if (d) xr_vmcnt<DHI>();
    else if (e) xr_vmcnt<E>();
    else xr_vmcnt<0>();
  } else {
    if (d && e) xr_vmcnt<DLO + E>();
    else if (d) xr_vmcnt<DLO>();
    else if (e) xr_vmcnt<E>();
    else xr_vmcnt<0>();
  }
}

// IL: the next stage's DMA instructions interleaved among this step's MFMAs (one after each
// granule's six) instead of issued together right after the barrier
template <int EPI, bool IL>
__global__ __launch_bounds__(512, 1) void gemm_xr_kernel(hvk_xr::Args p) {
  // vector-memory ops a wave issues in an item's epilogue after the next stage's DMA, at least:
  // its stores (3 per granule, 6 for EPI 1; EPI 2 stores every granule slot, the unused ones out
  // of range).  (The bias loads of EPI 0 / 1 are waited for inside the epilogue.)
  constexpr int EMIN = EPI == 2 ? 3 * GR : (EPI == 1 ? 6 : 3) * GMIN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int li = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  const bool hi = wave < NHI;  // issues DHI DMA instructions per stage (else DLO)
  const int KT = p.K / XBK;
  const int total = p.ipw * KT;
  const int item0 = blockIdx.x * p.ipw;
  const int lr = lane >> 3, lc = lane & 7;

  // ---- DMA of flat step s: item item0 + s / KT, k-step s % KT, into stage s % 3.  Block b of a
  // stage (b < 24: W image rows 8b .. 8b+7; else X image block b - 24) is issued by wave b % 8.
  // The stream state (item, k-step, per-block source rows) advances incrementally
  int is_it = item0, is_kt = 0, is_buf = 0;  // the next step to issue
  const hvk_bf16* isrc[DHI];
  auto set_src = [&](int it) {
    const int r = it / p.NT, nt = it - r * p.NT;
    const int g0 = (int)(((long long)r * p.NG) / p.G);
#pragma unroll
    for (int i = 0; i < DHI; ++i) {
      const int b = wave + 8 * i;
      const int row = 8 * b + lr;
      if (b < WBLK) {
        isrc[i] = p.W + (size_t)(nt * XBN + xr_perm_row(row)) * p.K + 8 * (lc ^ (row & 7));
      } else {
        int xr = 16 * g0 + row - 8 * WBLK;
        if (xr >= p.M) xr = p.M - 1;  // rows past M: any valid row (never stored)
        isrc[i] = p.X + (size_t)xr * p.K + 8 * (lc ^ (row & 7));
      }
    }
  };
  set_src(is_it);
  auto issue_part = [&](int i) {  // DMA instruction i of the next step
    if (i == DHI - 1 && !hi) return;
    __builtin_amdgcn_global_load_lds((xr_gbl_ptr)(isrc[i] + is_kt * XBK),
                                     (xr_lds_ptr)(smem + is_buf * STAGE + (wave + 8 * i) * 1024), 16, 0, 0);
  };
  auto issue_done = [&]() {  // advance the stream state past the step just issued
    is_buf = is_buf == NSTAGE - 1 ? 0 : is_buf + 1;
    if (++is_kt == KT) {
      is_kt = 0;
      if (++is_it < item0 + p.ipw) set_src(is_it);
    }
  };

  const __amdgpu_buffer_rsrc_t ry = hvk_rsrc(p.Y, (size_t)p.M * p.N * 2);
  const __amdgpu_buffer_rsrc_t ry2 = hvk_rsrc(EPI == 1 ? p.Y2 : p.Y, (size_t)p.M * p.N * 2);
  const hvk_u32x4 rh = xr_srsrc(EPI == 2 ? p.Y2 : p.Y, (uint32_t)((size_t)p.M * p.N * 2));
  const hvk_u32x4 rbias = xr_srsrc(p.bias ? (const void*)p.bias : (const void*)p.Y, p.bias ? (uint32_t)p.N * 4u : 0u);

  hvk_f32x4 acc[6][GR];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < GR; ++b) acc[a][b] = hvk_f32x4{0, 0, 0, 0};

  // this item's granules of this wave row: [gb, gb + gn)
  int gn = 0, gb = 0, n0 = 0, row0 = 0;
  auto item_geom = [&](int it) {
    const int r = it / p.NT, nt = it - r * p.NT;
    const int g0 = (int)(((long long)r * p.NG) / p.G), g1 = (int)(((long long)(r + 1) * p.NG) / p.G);
    const int n = g1 - g0;
    const int q0 = (n * wm) >> 2, q1 = (n * (wm + 1)) >> 2;
    gb = q0;
    gn = q1 - q0;
    n0 = nt * XBN;
    row0 = 16 * (g0 + gb);
  };
  item_geom(item0);

  auto issue_next = [&]() {
#pragma unroll
    for (int i = 0; i < DHI; ++i) issue_part(i);
    issue_done();
  };
  issue_next();
  if (total > 1) issue_next();

  int kt = 0, buf = 0, it = item0;
  for (int s = 0; s < total; ++s) {
    // stage s landed: younger than its DMA are DMA(s+1) and the epilogue stores of an item that
    // ended at step s-1 or s-2 (KT >= 2: at most one)
    xr_wait_stage<EMIN>(hi, s + 1 < total, (s >= 1 && kt == 0) || (s >= 2 && kt == 1));
    __builtin_amdgcn_s_barrier();  // every wave's stage s landed; stage (s-1) % 3 is free
    asm volatile("" ::: "memory");
    const bool last = kt == KT - 1;
    // an item's bias, 3 x 8 floats per lane, loaded on its last step just before the DMA of step
    // s+2 (waited for in the epilogue: younger than it then is that DMA only)
    hvk_u32x4 bq[3][2];
    if (EPI != 2 && last && p.bias) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const uint32_t c = (uint32_t)(n0 + 96 * wn + 32 * j + 8 * g) * 4u;
        bq[j][0] = xr_bld16(rbias, c);
        bq[j][1] = xr_bld16(rbias, c + 16);
      }
    }
    const bool d2 = s + 2 < total;
    if (!IL && d2) issue_next();
    const uint32_t sbase = xr_lds_u32(smem) + buf * STAGE;
    const uint32_t aw = sbase + (96 * wn + li) * 128;
    const uint32_t ax = sbase + XOFF + (16 * gb + li) * 128;
    hvk_u32x4 ra[2][6], rx[2][GR];
    {
      const uint32_t sw0 = ((g) ^ (li & 7)) << 4, sw1 = ((4 + g) ^ (li & 7)) << 4;
      xr_rd_tiles<0, 6>(ra[0], aw + sw0);
      xr_rd_tiles<0, GR>(rx[0], ax + sw0);
      xr_rd_tiles<0, 6>(ra[1], aw + sw1);
      xr_rd_tiles<0, GR>(rx[1], ax + sw1);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(6 + GR) : "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint4 af[6], bf[GR];
#pragma unroll
      for (int t = 0; t < 6; ++t) af[t] = xr_tie(ra[ks][t]);
#pragma unroll
      for (int b = 0; b < GR; ++b) bf[b] = xr_tie(rx[ks][b]);
#pragma unroll
      for (int b = 0; b < GR; ++b) {
        if (b < GMIN || b < gn)
#pragma unroll
          for (int t = 0; t < 6; ++t) acc[t][b] = hvk_mfma16(af[t], bf[b], acc[t][b]);
        if (IL && d2 && GR * ks + b < DHI) {
          __builtin_amdgcn_sched_barrier(0);
          issue_part(GR * ks + b);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if (IL && d2) issue_done();

    if (last) {
      if constexpr (EPI == 2) {
        // ---- gh = (gy w) * GELU'(h), granule slot by slot with the next slot's h in flight;
        // younger than h(b) when it is waited for: the 3 stores of slot b-1 and the 3 loads of
        // h(b+1) (the DMA of step s+2, issued before h(0), lands first)
        hvk_u32x4 hq[2][3];
        auto h_load = [&](int b, hvk_u32x4 (&dst)[3]) {
          const uint32_t roff = (uint32_t)(row0 + 16 * b + li) * (uint32_t)p.N * 2u;
#pragma unroll
          for (int j = 0; j < 3; ++j) dst[j] = xr_bld16(rh, roff + (uint32_t)(n0 + 96 * wn + 32 * j + 8 * g) * 2u);
        };
        h_load(0, hq[0]);
#pragma unroll
        for (int b = 0; b < GR; ++b) {
          if (b + 1 < GR) h_load(b + 1, hq[(b + 1) & 1]);
          if (b >= 1 && b + 1 < GR) xr_vmcnt<6>();
          else if (b >= 1 || b + 1 < GR) xr_vmcnt<3>();
          else xr_vmcnt<0>();
          uint4 hv[3];
#pragma unroll
          for (int j = 0; j < 3; ++j) hv[j] = xr_tie(hq[b & 1][j]);
          const uint32_t roff = (b < GMIN || b < gn) ? (uint32_t)(row0 + 16 * b + li) * (uint32_t)p.N * 2u : HVK_OOB;
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
      } else {
        // ---- bias (loaded at the top of this step), pack, then the stores back to back
        float bv[3][8];
        if (p.bias) {
          xr_wait_stage<0>(hi, d2, false);
#pragma unroll
          for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint4 u = xr_tie(bq[j][h]);
              bv[j][4 * h] = __uint_as_float(u.x);
              bv[j][4 * h + 1] = __uint_as_float(u.y);
              bv[j][4 * h + 2] = __uint_as_float(u.z);
              bv[j][4 * h + 3] = __uint_as_float(u.w);
            }
        } else {
#pragma unroll
          for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int e2 = 0; e2 < 8; ++e2) bv[j][e2] = 0.f;
        }
#pragma unroll
        for (int b = 0; b < GR; ++b) {
          if (b >= GMIN && b >= gn) break;
          const uint32_t roff = (uint32_t)(row0 + 16 * b + li) * (uint32_t)p.N * 2u;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] = acc[2 * j][b][r] + bv[j][r];
              v[4 + r] = acc[2 * j + 1][b][r] + bv[j][4 + r];
            }
            const uint4 hv = hvk_pack8(v);
            const uint32_t off = roff + (uint32_t)(n0 + 96 * wn + 32 * j + 8 * g) * 2u;
            if (EPI == 1) {
              hvk_bst16_nt(ry, off, hv);  // h: read again only by the backward
              hvk_bst16(ry2, off, hvk_gelu8_bf16(hv));
            } else {
              hvk_bst16(ry, off, hv);
            }
          }
        }
      }
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < GR; ++b) acc[a][b] = hvk_f32x4{0, 0, 0, 0};
      if (s + 1 < total) item_geom(++it);
    }
    kt = last ? 0 : kt + 1;
    buf = buf == NSTAGE - 1 ? 0 : buf + 1;
  }
}

template <int EPI, bool IL>
int launch_(const hvk_xr::Args& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_xr_kernel<EPI, IL>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hvk_timer_shape("gemm_xr", EPI, IL, a.M, a.N, a.K,
                  2.0 * ((double)a.M * a.K + (double)a.N * a.K + (double)a.M * a.N * (EPI == 1 || EPI == 2 ? 2 : 1)));
  HVK_LAUNCH_TIMED_W(HVK_TIMER_GEMM, 2.0 * a.M * a.N * a.K, (gemm_xr_kernel<EPI, IL>), dim3(256), dim3(512), LDS,
                     st, a);
  HVK_CHECK_LAUNCH("hvk_gemm_xr");
  return HVK_OK;
}

}  // namespace

namespace hvk_xr {

// Plan: G row groups of the NG = ceil(M / 16) granules (12 or 13 each), G * NT items (NT =
// N / 192) dealt 256 ways, G * NT a multiple of 256.  False when no plan fits (the caller keeps
// gemm_nt_kernel).
bool plan(int M, int N, int K, Args& a, int& mg) {
  if (M <= 0 || N % XBN || K % XBK || K < 2 * XBK) return false;
  if ((long long)M * N * 2 >= (1ll << 31) || (long long)M * K >= (1ll << 31) || (long long)N * K >= (1ll << 31))
    return false;
  const int NG = (M + 15) / 16, NT = N / XBN;
  for (int G = NG / MG; G <= NG / (MG - 1); ++G) {
    if (G < 1 || (G * NT) % 256) continue;
    const int lo = NG / G, hi = (NG + G - 1) / G;
    if (hi <= MG && lo >= MG - 1) {
      a.M = M, a.N = N, a.K = K, a.NG = NG, a.G = G, a.NT = NT, a.ipw = G * NT / 256;
      mg = MG;
      return true;
    }
  }
  return false;
}

int launch(int epi, const hvk_bf16* X, const hvk_bf16* W, const float* bias, hvk_bf16* Y, hvk_bf16* Y2, int M,
           int N, int K, hipStream_t st) {
  Args a;
  int mg = 0;
  if (!plan(M, N, K, a, mg)) return -1;
  a.X = X, a.W = W, a.bias = epi == 2 ? nullptr : bias, a.Y = Y, a.Y2 = Y2;
  // option gemm_xr: 1 the DMA issued after the barrier, 2 interleaved among the MFMAs
  const bool il = hvk_opt(HVK_OPT_GEMM_XR) == 2;
  if (epi == 2) return il ? launch_<2, true>(a, st) : launch_<2, false>(a, st);
  if (epi == 1) return il ? launch_<1, true>(a, st) : launch_<1, false>(a, st);
  return il ? launch_<0, true>(a, st) : launch_<0, false>(a, st);
}

}  // namespace hvk_xr
