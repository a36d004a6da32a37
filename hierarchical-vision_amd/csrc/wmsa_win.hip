// W-MSA forward for windows <= 8 on gfx950, one workgroup per (window, head group): the
// window's q/k/v rows of the group land in LDS by ONE burst of LDS-DMA, every wave (one per
// head) computes its head's attention from LDS, writes its output back into the slab's q slots,
// and the workgroup stores the window's output as whole row segments (HG*64 contiguous bytes per
// token; at HG = nH the full C*2-byte rows, and the WIN tokens of a window row adjacent).
// Same math and results as wmsa_fwd_ring_kernel (wmsa_ring.hip), which is this kernel's
// persistent twin: the reference sequence is swinv2.py:221-261 with the roll / partition /
// reverse of swinv2.py:399-429 folded into addressing.
//
// Why a non-persistent grid: the ring kernel keeps one window of DMA in flight per workgroup and
// issues the next only after its waves hold the current window's fragments; its memory-only
// build reaches 0.65 of 8 TB/s.  Here the hardware starts a new workgroup the moment one ends,
// each with its whole window in flight at once, and the output leaves as contiguous rows from
// LDS instead of 64-B per-head pieces from registers (tools/probe/wmsa_mem.hip `win1 glds nt`:
// 0.80 memory-only, 0.74 with a stand-in for the math; profiles/round4/wmsa_fwd_mem_probe_stage0.txt).  The per-window setup the ring kernel
// amortised (bias table, head bound) overlaps the DMA: its global reads are issued first and
// waited for by count while the slab is still in flight.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "wmsa_ring.h"

#ifndef HVK_WIN_PRIO  // 1: raised wave priority while a workgroup issues its DMA and its stores
#define HVK_WIN_PRIO 0  // measured: neutral to -0.3 % (profiles/round3/wmsa_fwd_win/ab_prio.txt)
#endif
#ifndef HVK_WIN_REGSTORE  // A/B builds: 1 stores each head's output slice from registers (no LDS staging)
#define HVK_WIN_REGSTORE 0
#endif
#ifndef HVK_WIN_PROBE  // tools/ probe builds: 1 memory only (no math), 2 math only (no DMA, no stores)
#define HVK_WIN_PROBE 0
#endif

namespace {
using namespace hvk_ring;

// global_load_dword from inline asm: invisible to the compiler's waitcnt pass, so the explicit
// vmcnt wait below can leave the (later, compiler-visible) LDS-DMA in flight
__device__ __forceinline__ uint32_t gld32(const float* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ void lds_wr32(uint32_t a, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
// one LDS-DMA wave-instruction (global_load_lds_dwordx4) from inline asm: wave-uniform base
// (scalar pair) + 32-bit lane offset, M0 = the LDS destination; invisible to the compiler's
// waitcnt pass (the kernel counts vmcnt itself)
template <bool NT>
__device__ __forceinline__ void dma16_lds(const char* base, uint32_t voff, uint32_t m0) {
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  if constexpr (NT)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt"
                 :: "s"(__builtin_amdgcn_readfirstlane(m0)), "v"(voff), "s"((const void*)bs) : "memory");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :: "s"(__builtin_amdgcn_readfirstlane(m0)), "v"(voff), "s"((const void*)bs) : "memory");
}
// a * b + c on the full-rate 24-bit multiplier (a, b < 2^24): from asm, so the compiler cannot
// fold it into a quarter-rate v_mad_u64_u32 / v_mul_lo_u32
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ void lds_wr128(uint32_t a, uint4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(__builtin_bit_cast(hvk_u32x4, v)) : "memory");
}

// Slab swizzle: the 16-B chunk k (0..3) of a head's 64-B segment of token column x sits at chunk
// k ^ swz(x).  Without it the fragment reads of a wave (16 rows = token columns 0..7 of two
// window rows, 36-slot token stride) hit each 64-bank group twice and the output write-back four
// times (39 % of the stage-0 LDS cycles were bank conflicts, profiles/round4/pmc_wmsa_normed);
// with it both are conflict-free (bank model of MI355X_MICROARCH.md §LDS, every w / HG checked).
// The DMA places the chunks, every slab reader applies the same XOR.
__device__ __forceinline__ unsigned swz(unsigned x) { return (x >> 1) & 3u; }

// MM: shift-mask form, fixed at launch so no branch (and no register copies where branches
// merge) sits in the score loop: 0 unshifted block (no mask), 1 w7 / shift 3 (tile-uniform
// row band + per-lane column band: one add per element, every window), 2 any other shift
template <int WIN, int HG, bool LSE, int MM>
__global__ __launch_bounds__(64 * HG, 4) void wmsa_fwd_win_kernel(FwdArgs a) {
  using K = RingCfg<WIN, HG>;
  constexpr int NE = (K::TABF + 63) / 64;  // bias-table entries per lane
  constexpr int NKMIN = K::NINST / HG;     // fewest DMA instructions any wave issues
  static_assert(NKMIN >= 1 && NKMIN < 64, "vmcnt immediate");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  const int ng = g.nH / HG;
  // XCD-aware order: the 8 XCDs own contiguous runs of (window, group) items, so the groups of a
  // window (which split the lines of its row segments) share one L2
  const int items = g.n_windows * ng, per = (items + 7) >> 3;
  const int item = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (item >= items) return;
  const int win = (int)fdiv(item, a.fd_groups), grp = item - win * ng;
  const int b = (int)fdiv(win, a.fd_img), wrem = win - b * g.nWh * g.nWw;
  const int wh = (int)fdiv(wrem, a.fd_ww), ww = wrem - wh * g.nWw;

  if (HVK_WIN_PRIO) __builtin_amdgcn_s_setprio(2);  // get this window's loads out first
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C;
  const int h = grp * HG + wave;
  const int grp_off = grp * HG * 64;
  char* zero16 = smem + K::SLAB;
  float* btab = reinterpret_cast<float*>(smem + K::SLAB + 16);

  // 1. this head's CPB bias entries (x log2e), read before the DMA is issued: mirrored layout of
  //    wmsa_ring.hip (entry PAD + i at TABF - 1 - PAD - i), zero outside the R*R real entries
  uint32_t braw[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int e = lane + 64 * k, i = K::TABF - 1 - e - K::PAD;
    const bool ok = e < K::TABF && i >= 0 && i < K::R * K::R;
    braw[k] = gld32(a.bias + (size_t)h * K::R * K::R + (ok ? i : 0));
  }
  const uint32_t scale_raw = gld32(a.scale + h);  // counted with the bias reads

  // 2. the slab: WIN runs (window rows) of IPR 1-KB DMA instructions, lane-linear slots
  //    (wmsa_ring.hip's layout): instruction j = IPR*ty + m, slot 64m + lane of run ty holds
  //    token column tx, part, 16-B column c, all fixed by (m, lane).  pre[k % KP] = the lane's
  //    byte offset inside a token row run (bits 0-23) | tx << 24 for its k-th instruction; slots
  //    past a run's WIN*RS reload the run's first bytes (no exec masking).  Nontemporal: every
  //    byte is read once.
  {
    const unsigned RB = 6u * C, WRB = (unsigned)g.W * RB;
    unsigned pre[K::KP];
#pragma unroll
    for (int k = 0; k < K::KP; ++k) {
      const int m = (wave + HG * k) % K::IPR;
      const unsigned q = 64u * m + lane;
      // slot q = RS tx + 4HG part + c with RS = 3 (4HG): u = q / 4HG = 3 tx + part, and the byte
      // offset tx 6C + part 2C = u 2C
      const unsigned u = q / (4 * HG), c = q - mad24(u, 4u * HG, 0u), tx = u / 3;
      const unsigned cs = (c & ~3u) | ((c & 3u) ^ swz(tx));  // the global chunk this slot holds
      const unsigned v = (__umul24(u, 2u * C) + cs * 16 + grp_off) | (tx << 24);
      pre[k] = q < (unsigned)(WIN * K::RS) ? v : (unsigned)grp_off;
    }
    const char* img = reinterpret_cast<const char*>(a.qkv) + (size_t)b * g.H * WRB;
    const int y0 = wh * WIN + g.shift, x0 = ww * WIN + g.shift;
    const int ly = g.H - y0, lx = g.W - x0;  // ty >= ly (tx >= lx): the row wraps (cyclic shift)
    // per-lane offsets with this window's column wrap applied, materialised once (4 VGPRs):
    // an instruction then adds only its uniform row offset
#pragma unroll
    for (int k = 0; k < K::KP; ++k) {
      pre[k] = __umul24(pre[k], 1u) - ((lx < WIN && (int)(pre[k] >> 24) >= lx) ? WRB : 0u);
      lds_fence(pre[k]);
    }
    __builtin_assume(wave < HG);
    // the DMA from inline asm (scalar base + 32-bit lane offset, M0 = the LDS destination):
    // 1-2 VALU per instruction; the cache policy (nontemporal or not) picks one of two loops
    auto issue = [&](auto nt_t) {
#pragma unroll
      for (int k = 0; k < K::NK; ++k) {
        const int j = wave + HG * k;
        if (j < K::NINST) {
          const int ty = j / K::IPR;
          const unsigned U = ((unsigned)(y0 + ty - (ty >= ly ? g.H : 0)) * g.W + x0) * RB;  // uniform
          const unsigned off = pre[k % K::KP] + U;
#if HVK_WIN_PROBE == 2
          (void)off;
          asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(smem + j * 1024) + 16u * (threadIdx.x & 63)),
                       "v"(hvk_u32x4{0, 0, 0, 0}) : "memory");
#else
          dma16_lds<decltype(nt_t)::value>(img, off, lds_addr(smem) + (uint32_t)j * 1024u);
#endif
        }
      }
    };
    if (a.dma_nt)
      issue(std::true_type{});
    else
      issue(std::false_type{});
  }

  if (HVK_WIN_PRIO) __builtin_amdgcn_s_setprio(0);
  // 3. while the slab is in flight: the bias table shifted by the head bound M_h
  //    (= scale*log2e + max bias*log2e, wmsa_ring.hip) and the lane constants
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NKMIN) : "memory");  // the bias / scale reads only
  uint32_t sraw = scale_raw;
  lds_fence(sraw);
  const float scale_h = __uint_as_float(sraw);
  float bv[NE], mb = -INFINITY;
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    lds_fence(braw[k]);
    const int e = lane + 64 * k, i = K::TABF - 1 - e - K::PAD;
    const bool ok = e < K::TABF && i >= 0 && i < K::R * K::R;
    float x = __uint_as_float(braw[k]) * HVK_LOG2E;
    lds_fence(x);  // rounded before "- M_h", as the ring kernel's LDS round trip (no fma contraction)
    bv[k] = ok ? x : -INFINITY;
    mb = fmaxf(mb, bv[k]);
  }
  mb = hvk_group4_max(hvk_row16_max(mb));  // DPP + lane swaps: no LDS round trips
  const float Mh = __builtin_fmaf(scale_h, HVK_LOG2E, mb);
  const uint32_t tab0 = lds_addr(btab) + 4 * wave * K::TABF;
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int e = lane + 64 * k;
    if (e < K::TABF) lds_wr32(tab0 + 4 * e, bv[k] == -INFINITY ? 0.f : bv[k] - Mh);
  }
  if (lane == 0) lds_wr128(lds_addr(zero16), make_uint4(0, 0, 0, 0));
  const float sc2 = scale_h * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  int lq, lk;
  if (K::PW == 8) {
    lq = (li >> 3) * K::R + (li & 7);
    lk = (gq >> 1) * K::R + 4 * (gq & 1);
  } else {
    lq = (li >> 2) * K::R + (li & 3);
    lk = gq * K::R;
  }
  const uint32_t bta =
      lds_addr(btab) + 4 * (wave * K::TABF + K::TABF - 4 - (K::PAD + K::BASE0 + lq - lk - K::TR * (K::NT - 1) - 3) -
                            2 * K::TR * (K::NT - 1));
  static_assert(2 * K::TR * (K::NT - 1) + 3 < 256, "bias offsets exceed ds_read2_b32's field");
  uint4 ones[K::NC];
#pragma unroll
  for (int c = 0; c < K::NC; ++c) {
    uint32_t wv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * jj + e;
        const int p = 32 * c + (j < 4 ? 4 * gq + j : 16 + 4 * gq + j - 4);
        if ((p % K::PW) < WIN && (p / K::PW) < WIN) v |= 0x3F80u << (16 * e);
      }
      wv[jj] = v;
    }
    ones[c] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
  }
  // key-slot region bits (slot bit ki*4 + r): row band in bits 0-15, column band in 16-31.  Key
  // p = 16 ki + 4 gq + r sits at grid row 16/PW ki + 4 gq / PW and column (4 gq) % PW + r, so the
  // row band is one nibble per ki and the column band one nibble repeated (no per-bit selects)
  uint32_t kband;
  {
    const int lim = WIN - g.shift;
    uint32_t rowb = 0;
#pragma unroll
    for (int ki = 0; ki < K::NT; ++ki)
      rowb |= ((16 / K::PW) * ki + (4 * gq) / K::PW >= lim) ? 0xFu << (4 * ki) : 0u;
    const int cl = lim - (4 * gq) % K::PW;  // column r in band iff r >= cl
    const uint32_t nib = cl <= 0 ? 0xFu : (cl >= 4 ? 0u : (0xFu << cl) & 0xFu);
    uint32_t rep = nib;
#pragma unroll
    for (int ki = 1; ki < K::NT; ++ki) rep |= nib << (4 * ki);  // nibble per key tile, no multiply
    kband = rowb | (rep << 16);
  }

  // 4. the slab has landed (every wave's DMA + table writes): fragments into registers
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#if HVK_WIN_PROBE != 1
  const uint32_t zaddr = lds_addr(zero16);
  const int fx = li % K::PW, fy0 = li / K::PW;
  const uint32_t fb = lds_addr(smem) + (fy0 * K::RUN + fx * K::RS + wave * 4 + (gq ^ swz(fx))) * 16;
  hvk_u32x4 qr[K::NT], kr[K::NT];
  hvk_u32x2 vr[K::NC][2][2];
#pragma unroll
  for (int i = 0; i < K::NT; ++i) {
    const bool ok = fx < WIN && fy0 + (16 / K::PW) * i < WIN;
    const uint32_t aq = fb + (16 / K::PW) * i * K::RUN * 16;
    qr[i] = lds_rd128<0>(ok ? aq : zaddr);
    kr[i] = lds_rd128<0>(ok ? aq + 4 * HG * 16 : zaddr);
  }
  {
    const int pl = 4 * gq + (li >> 2);
    const int x = pl % K::PW, y0 = pl / K::PW;
    const uint32_t vb =
        lds_addr(smem) + (y0 * K::RUN + x * K::RS) * 16 + (2 * HG * 32 + wave * 32 + 8 * ((li & 3) ^ swz(x))) * 2;
#pragma unroll
    for (int c = 0; c < K::NC; ++c)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int dy = (16 / K::PW) * (2 * c + hh);
        const bool ok = x < WIN && y0 + dy < WIN;
        const uint32_t av = ok ? vb + dy * K::RUN * 16 : zaddr;
        vr[c][0][hh] = lds_rd64_tr<0>(av);
        vr[c][1][hh] = lds_rd64_tr<8>(av);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  uint4 qf[K::NT], kf[K::NT], vt[K::NC][2];
#pragma unroll
  for (int i = 0; i < K::NT; ++i) {
    lds_fence(qr[i]);
    lds_fence(kr[i]);
    qf[i] = u4(qr[i]);
    kf[i] = u4(kr[i]);
  }
#pragma unroll
  for (int c = 0; c < K::NC; ++c)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      lds_fence(vr[c][dt][0]);
      lds_fence(vr[c][dt][1]);
      vt[c][dt] = make_uint4(vr[c][dt][0][0], vr[c][dt][0][1], vr[c][dt][1][0], vr[c][dt][1][1]);
    }

  // 5. attention, one query tile at a time (the ring kernel's math); the normalised output row
  //    slice goes back into this head's q slots of the slab (read above by this wave only)
  const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
  static_assert(MM != 1 || (WIN == 7 && K::PW == 8), "the tile-uniform mask form is w7 / shift 3 only");
  const float colmask = (edge_c && (((li >> 2) ^ gq) & 1)) ? mask2 : 0.f;  // query x >= 4 vs key x >= 4
  float rn;
  if (!a.qk_normed) {  // qk_normed: q^ * scale * log2e and k^ arrive from the qkv GEMM's epilogue
#pragma unroll
    for (int i = 0; i < K::NT; ++i) {
      qf[i] = l2_normalize(qf[i], rn, sc2);
      kf[i] = l2_normalize(kf[i], rn);
    }
  }
  // the query-tile loop is instantiated twice, for windows with and without a shift mask: the
  // branch sits outside it, so nothing inside merges registers from two paths
  auto run_tiles = [&](auto edge_t) {
  constexpr bool EDGE = decltype(edge_t)::value;
#pragma unroll
  for (int qi = 0; qi < K::NT; ++qi) {
    const int pq = 16 * qi + li;
    const int tq = grid_token<WIN, K::PW>(pq);
    auto scores = [&](hvk_f32x4 (&s)[K::NT]) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      hvk_u32x2 br[K::NT][2];
      ring_bias_read_q<K::TR, K::NT>(br, bta, qi);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki) {
        lds_fence(br[ki][0]);
        lds_fence(br[ki][1]);
        const hvk_f32x4 bb = {__uint_as_float(br[ki][0][0]), __uint_as_float(br[ki][0][1]),
                              __uint_as_float(br[ki][1][0]), __uint_as_float(br[ki][1][1])};
        s[ki] = hvk_mfma16(kf[ki], qf[qi], bb);
      }
      settle_tiles(s);
      if constexpr (MM == 1 && EDGE) {
        // w7, shift 3 on the 8-wide grid: the row band of a tile pair is uniform (bands = tiles
        // {0,1} / {2,3}) and the column band of a lane's keys is fixed by gq: one add per element
        // (edge windows only)
#pragma unroll
        for (int ki = 0; ki < K::NT; ++ki) {
          const float mv = (edge_r && ((qi >= 2) != (ki >= 2))) ? mask2 : colmask;
#pragma unroll
          for (int r = 0; r < 4; ++r) s[ki][r] += mv;
        }
      } else if constexpr (MM == 2 && EDGE) {
        const int qy = pq / K::PW, qx = pq % K::PW;
        uint32_t mreg = 0;
        if (edge_r) mreg |= (kband ^ (qy >= WIN - g.shift ? 0xFFFFu : 0u)) & 0xFFFFu;
        if (edge_c) mreg |= (kband >> 16) ^ (qx >= WIN - g.shift ? 0xFFFFu : 0u);
#pragma unroll
        for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[ki][r] = fmaf((float)((mreg >> (ki * 4 + r)) & 1u), mask2, s[ki][r]);
      }
    };
    hvk_f32x4 o[2], osum;
    hvk_f32x4 s[K::NT];
    scores(s);
#pragma unroll
    for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[ki][r] = __builtin_amdgcn_exp2f(s[ki][r]);
    o[0] = o[1] = osum = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < K::NC; ++c) {
      const hvk_f32x4 a0 = s[2 * c];
      const hvk_f32x4 a1 = (2 * c + 1 < K::NT) ? s[2 * c + 1] : hvk_f32x4{0, 0, 0, 0};
      const uint4 pf = make_uint4(hvk_pack2(a0[0], a0[1]), hvk_pack2(a0[2], a0[3]),
                                  hvk_pack2(a1[0], a1[1]), hvk_pack2(a1[2], a1[3]));
      o[0] = hvk_mfma16(vt[c][0], pf, o[0]);
      o[1] = hvk_mfma16(vt[c][1], pf, o[1]);
      osum = hvk_mfma16(ones[c], pf, osum);
    }
    float lshift = 0.f;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(tq >= 0 && !(osum[0] >= 0x1p-100f)) != 0, 0)) {
      // slow path (rare, wave-uniform): the reference's softmax with the true row max
      uint32_t mreg = 0;
      if constexpr (EDGE) {
        const int qy = pq / K::PW, qx = pq % K::PW;
        if (edge_r) mreg |= (kband ^ (qy >= WIN - g.shift ? 0xFFFFu : 0u)) & 0xFFFFu;
        if (edge_c) mreg |= (kband >> 16) ^ (qx >= WIN - g.shift ? 0xFFFFu : 0u);
      }
      const uint32_t kpad = (uint32_t)(K::KPAD >> (16 * gq)) & 0xFFFFu;
      auto tile = [&](int ki) {
        const uint32_t ab = bta + 4 * K::TR * (K::NT - 1 - qi + ki);
        hvk_u32x2 b0 = lds_rd2<0, 1>(ab), b1 = lds_rd2<2, 3>(ab);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lds_fence(b0);
        lds_fence(b1);
        const hvk_f32x4 bb = {__uint_as_float(b0[0]), __uint_as_float(b0[1]), __uint_as_float(b1[0]),
                              __uint_as_float(b1[1])};
        hvk_f32x4 t = hvk_mfma16(kf[ki], qf[qi], bb);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          t[r] = fmaf((float)((mreg >> (ki * 4 + r)) & 1u), mask2, t[r]);
          t[r] = fmaf((float)((kpad >> (ki * 4 + r)) & 1u), -1e30f, t[r]);
        }
        return t;
      };
      float m = -INFINITY;
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki) {
        const hvk_f32x4 t = tile(ki);
        m = fmaxf(m, fmaxf(fmaxf(t[0], t[1]), fmaxf(t[2], t[3])));
      }
      m = fmaxf(m, __shfl_xor(m, 16));
      m = fmaxf(m, __shfl_xor(m, 32));
      lshift = m;
      o[0] = o[1] = osum = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < K::NC; ++c) {
        hvk_f32x4 a0 = tile(2 * c), a1 = {0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 4; ++r) a0[r] = __builtin_amdgcn_exp2f(a0[r] - m);
        if (2 * c + 1 < K::NT) {
          a1 = tile(2 * c + 1);
#pragma unroll
          for (int r = 0; r < 4; ++r) a1[r] = __builtin_amdgcn_exp2f(a1[r] - m);
        }
        const uint4 pf = make_uint4(hvk_pack2(a0[0], a0[1]), hvk_pack2(a0[2], a0[3]),
                                    hvk_pack2(a1[0], a1[1]), hvk_pack2(a1[2], a1[3]));
        o[0] = hvk_mfma16(vt[c][0], pf, o[0]);
        o[1] = hvk_mfma16(vt[c][1], pf, o[1]);
        osum = hvk_mfma16(ones[c], pf, osum);
      }
      hvk_settle(o[0], o[1], osum);
    }
    if (tq >= 0) {
      const float inv = __builtin_amdgcn_rcpf(osum[0]);
      const uint4 v = make_uint4(hvk_pack2(o[0][0] * inv, o[0][1] * inv), hvk_pack2(o[0][2] * inv, o[0][3] * inv),
                                 hvk_pack2(o[1][0] * inv, o[1][1] * inv), hvk_pack2(o[1][2] * inv, o[1][3] * inv));
#if HVK_WIN_REGSTORE
      *reinterpret_cast<uint4*>(a.out + (size_t)window_token_row(g, b, wh, ww, WIN, tq) * C + h * 32 + 8 * gq) = v;
#else
      lds_wr128(fb + (16 / K::PW) * qi * K::RUN * 16, v);
#endif
      if constexpr (LSE) {
        if (gq == 0)
          a.lse[(size_t)window_token_row(g, b, wh, ww, WIN, tq) * g.nH + h] = Mh + lshift + __log2f(osum[0]);
      }
    }
  }
  };
  if (MM != 0 && (edge_r || edge_c))
    run_tiles(std::true_type{});
  else
    run_tiles(std::false_type{});

#endif  // HVK_WIN_PROBE != 1
#if HVK_WIN_PROBE == 2 || HVK_WIN_REGSTORE
  return;
#endif
  // 6. the window's output row segments, HG*64 contiguous bytes per token, from the q slots
  if (HVK_WIN_PRIO) __builtin_amdgcn_s_setprio(2);  // free the LDS for the next workgroup sooner
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  {
    constexpr int SEG = 4 * HG;  // 16-B slots per token
    constexpr int NS = (K::N * SEG + 64 * HG - 1) / (64 * HG);
    static_assert(64 * HG % SEG == 0 && 64 * HG / SEG == 16, "16 tokens per store round");
    const int y0 = wh * WIN + g.shift, x0 = ww * WIN + g.shift;
    const uint32_t C2 = 2u * C;
    // window origin as a uniform byte offset; a lane adds its token's (ty W + tx) C2 + 16 c, and
    // the last window row / column (cyclic shift) subtracts H W C2 / W C2 where it wraps
    char* obase = reinterpret_cast<char*>(a.out) + (size_t)b * g.H * g.W * C * 2 + grp_off +
                  (size_t)((uint32_t)y0 * g.W + x0) * C2;
    const uint32_t rowb = (uint32_t)g.W * C2, imgb = (uint32_t)g.H * rowb;
    const int ly = g.H - y0, lx = g.W - x0;
    const bool wrap = ly < WIN || lx < WIN;  // wave-uniform
    // thread s = tid + 64 HG k holds slot c = tid % SEG of token t0 + 16k (64 HG / SEG = 16)
    const int t0 = threadIdx.x / SEG, c = threadIdx.x - t0 * SEG;
    hvk_u32x4 v[NS];
    int off[NS];  // signed: a wrapped token lies BEFORE the window origin (|off| < H W 2C < 2^31)
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int t = t0 + 16 * k, ty = t / WIN, tx = t - ty * WIN;
      // slots past the window (last round only) read a valid slab address and store nothing
      const uint32_t sl = __umul24((uint32_t)ty, (uint32_t)(K::RUN * 16)) + __umul24((uint32_t)tx, (uint32_t)(K::RS * 16));
      const unsigned cs = (c & ~3u) | ((c & 3u) ^ swz(tx));
      v[k] = lds_rd128<0>(lds_addr(smem) + (t < K::N ? sl + cs * 16 : 0u));
      uint32_t o = mad24(mad24((uint32_t)ty, (uint32_t)g.W, (uint32_t)tx), C2, c * 16u);
      if (wrap) o -= (ty >= ly ? imgb : 0u) + (tx >= lx ? rowb : 0u);
      off[k] = (int)o;  // two's complement: the wrapped offsets come out negative
      (void)HVK_BCHECK(((y0 + ty) % g.H) * g.W + (x0 + tx) % g.W, g.H * g.W);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      lds_fence(v[k]);
      if (K::N * SEG % (64 * HG) == 0 || t0 + 16 * k < K::N)
        *reinterpret_cast<uint4*>(obase + (ptrdiff_t)off[k]) = u4(v[k]);
    }
  }
}

template <int WIN, int HG, bool LSE, int MM>
int launch_win_(FwdArgs& a, hipStream_t st) {
  using K = RingCfg<WIN, HG>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_fwd_win_kernel<WIN, HG, LSE, MM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    attr = true;
  }
  const long long items = (long long)a.g.n_windows * (a.g.nH / HG);
  if (a.g.H * a.g.W >= (1 << 24))  // launch_win routes these to the ring form
    return hvk_set_error(HVK_EINVAL, "wmsa win: %d x %d image past 24-bit token offsets", a.g.H, a.g.W);
  a.fd_groups = hvk_wmsa::make_fastdiv((uint32_t)(a.g.nH / HG));
  a.fd_img = hvk_wmsa::make_fastdiv((uint32_t)(a.g.nWh * a.g.nWw));
  a.fd_ww = hvk_wmsa::make_fastdiv((uint32_t)a.g.nWw);
  // slab DMA cache policy: nontemporal only when qkv
  // exceeds the 256 MB Infinity Cache -- the qkv GEMM just wrote it, so a smaller one is read
  // from the cache (SwinV2-T stages 1-3; stage 0's 462 MB streams nontemporally): in-step
  // 0.630-0.632 of 8 TB/s vs 0.610 always nontemporal vs 0.570 never (one box,
  // profiles/round3/wmsa_fwd_win/ab_dma_policy.txt)
  a.dma_nt = (long long)a.g.B * a.g.H * a.g.W * a.g.C * 6 > (256ll << 20);
  const long long grid = (items + 7) / 8 * 8;
  if (grid > 0x7fffffffLL) return hvk_set_error(HVK_EINVAL, "wmsa win: %lld windows x groups", items);
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_FWD, (wmsa_fwd_win_kernel<WIN, HG, LSE, MM>), dim3((unsigned)grid), dim3(64 * HG),
                   K::LDS, st, a);
  HVK_CHECK_LAUNCH("wmsa_fwd_win");
  return HVK_OK;
}

template <int WIN, int HG>
int launch_win(FwdArgs& a, hipStream_t st) {
  // the win form everywhere: in-step it beats the persistent ring at every SwinV2-T stage, the
  // 1.6-round stage 3 included (19.3 vs 23.8 us; the isolated microbench, from cold caches, had
  // it the other way: profiles/round3/wmsa_fwd_win/stages_stage3_routing.txt)
  // per-image byte offsets of the output stores are 32-bit (24-bit multiplies): larger images
  // take the ring form, which addresses with 64-bit offsets
  const bool big = a.g.H * a.g.W >= (1 << 24);  // (hvk_wmsa_fwd bounds H W 6C below 2^32)
  if (big)
    return hvk_wmsa::ring_fwd(a, a.g.B, a.g.H, a.g.W, a.g.C, a.g.nH, WIN, a.g.shift, st);
  if (a.g.shift == 0) return a.lse ? launch_win_<WIN, HG, true, 0>(a, st) : launch_win_<WIN, HG, false, 0>(a, st);
  if constexpr (WIN == 7)
    if (a.g.shift == 3) return a.lse ? launch_win_<WIN, HG, true, 1>(a, st) : launch_win_<WIN, HG, false, 1>(a, st);
  return a.lse ? launch_win_<WIN, HG, true, 2>(a, st) : launch_win_<WIN, HG, false, 2>(a, st);
}

template <int WIN>
int win_win(FwdArgs& a, hipStream_t st) {
  const int nH = a.g.nH;
  // option wmsa_fwd_hg forces the heads per workgroup where it divides nH (A/B runs)
  const int hg = (int)hvk_opt(HVK_OPT_WMSA_FWD_HG);
  if (hg == 6 && nH % 6 == 0) return launch_win<WIN, 6>(a, st);
  if (hg == 4 && nH % 4 == 0) return launch_win<WIN, 4>(a, st);
  if (hg == 3 && nH % 3 == 0) return launch_win<WIN, 3>(a, st);
  if (hg == 2 && nH % 2 == 0) return launch_win<WIN, 2>(a, st);
  if (hg == 1) return launch_win<WIN, 1>(a, st);
  // 6 heads (SwinV2-T stage 1): 2 per workgroup, 58 vs 60.5 us per launch in-step (round 5 sweep,
  // profiles/round5/wmsa_fwd_hg.txt; 3 stays best at 12 and 24 heads)
  if (nH == 6) return launch_win<WIN, 2>(a, st);
  // heads per workgroup: 3 where it divides (SwinV2-T: 3 beat 2, 4, 6, 8 at every stage), else 2
  // (SwinV2-B's 4 / 8 / 16 / 32 heads: 0.614 vs 0.595 with 4, one 128-B line per head pair and
  // part, 7 workgroups per CU: profiles/round3/wmsa_fwd_win/stages_b224_hg2.txt)
  if (nH % 3 == 0) return launch_win<WIN, 3>(a, st);
  if (nH % 2 == 0) return launch_win<WIN, 2>(a, st);
  return launch_win<WIN, 1>(a, st);
}

}  // namespace

namespace hvk_wmsa {
int win_fwd(FwdArgs& a, int B, int H, int W, int C, int nH, int win, int shift, hipStream_t st) {
  int rc = make_geom(B, H, W, C, nH, win, shift, 256, a.g);
  if (rc) return rc;
  switch (win) {
    case 7: return win_win<7>(a, st);
    case 8: return win_win<8>(a, st);
    case 6: return win_win<6>(a, st);
    case 4: return win_win<4>(a, st);
    default: return hvk_set_error(HVK_EUNSUPPORTED, "wmsa win: window %d", win);
  }
}
}  // namespace hvk_wmsa
