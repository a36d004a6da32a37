// Shifted-window cosine attention for LARGE windows (12, 16, 24: SwinV2-B 384 / window-24
// configs, the stage-3 clamp to 12, swinv2.py:328-331) on gfx950.
//
// Same semantics and token layout as wmsa.hip (reference: swinv2.py:221-261 + roll/partition
// 399-412 / reverse 420-429), but a window no longer fits one wave's registers
// (N = 144 ... 576 tokens), so a WORKGROUP owns a (window, head) at a time; workgroups are
// persistent, one head each over a run of windows (XCD-aware: the heads of a window run share
// one L2):
//   forward   k^ and v of the window sit in LDS (the next window's streamed in by LDS-DMA
//             meanwhile); every wave runs its query tiles against all keys in 32-key chunks;
//   backward  phase 1 (query on the lane, k^ / v in LDS): dS, dQ, the exact delta;
//             phase 2 (key on the lane, q^ / dO in LDS): dK, dV, the CPB-table and
//             logit-scale gradients.  The forward's row constants (LSE) spare the backward
//             its row-statistics pass.
// The CPB table stays compact ((2w-1)^2 floats per head, log2e-scaled, mirrored) and enters the
// score MFMAs as their C operand: index = bq(query) - bk(key), bq = (qh+w-1)(2w-1) + qw+w-1,
// bk = kh(2w-1) + kw.
//
// LDS images are [rows][32] bf16 in "fragment-major" order: the 16-B unit (row, u) of a
// 16-row tile sits at slot 16u + (row%16 ^ 12*(u&1)), so the natural MFMA operand read
// (ds_read_b128, lane = row%16 + 16u) and the transposed read (ds_read_b64_tr_b16) are both
// bank-conflict free (checked with the LDS bank model of MI355X_MICROARCH.md).
#include "wmsa_common.h"

// forward row sums: 1 = a ones-vector MFMA over the bf16 P, 0 = f32 adds of P (fewer registers)
#ifndef HVK_FWD_ROWSUM_MFMA
#define HVK_FWD_ROWSUM_MFMA 1
#endif

#ifndef HVK_LARGE_OPS_EARLY  // 1: the backward's phase 1 reads a chunk's operands before its MFMAs
#define HVK_LARGE_OPS_EARLY 1
#endif
#ifndef HVK_LARGE_TAB_EARLY  // 1: the forward reads all its tiles' bias C operands at each chunk's start
#define HVK_LARGE_TAB_EARLY 1
#endif

namespace hvk_wmsa {
namespace {

template <int WIN>
struct LCfg {
  static constexpr int N = WIN * WIN;
  static constexpr int NT = (N + 15) / 16;     // 16-token tiles
  static constexpr int NC = (NT + 1) / 2;      // 32-token chunks (one MFMA K-step)
  static constexpr int ROWS = 32 * NC;         // padded rows of an LDS image
  static constexpr int R = 2 * WIN - 1;
  static constexpr int RR = R * R;             // CPB table entries per head
  static constexpr int IMG = ROWS * 64;        // bytes per image
  static_assert(N == 16 * NT, "strided tiles cover the window exactly");
  // mirrored CPB table: entry j = RR - 1 - (bq - bk), so the 4 consecutive keys 4g .. 4g+3 of
  // a lane (one window row: 4 | WIN) read 4 ascending floats (two ds_read2_b32) straight into
  // the MFMA C operand; padding keys (w12's last chunk) index past RR into zeros
  static constexpr int QBMIN = (WIN - 1) * R + WIN - 1;
  static constexpr int KBMAX = ((ROWS - 1) / WIN) * R + (ROWS - 1) % WIN;
  static constexpr int TABM = ((RR - QBMIN + KBMAX > RR ? RR - QBMIN + KBMAX : RR) + 4) / 4 * 4;
};

// X^T fragment (A operand) of the 32-row chunk c, head-dim half dt, from an image of X
__device__ __forceinline__ uint4 tr_frag(const char* img, int c, int dt, int li, int g) {
  const int rr = 32 * c + 4 * g + (li >> 2), c8 = 4 * dt + (li & 3);
  const uint2 lo = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(img + fm8(rr, c8)));
  const uint2 hi = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(img + fm8(rr + 16, c8)));
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// The -100 mask of a shifted block's edge window (swinv2.py:357-388, 249-254) on the 4 scores of
// a lane: its fixed token (band bits `band`: bit 0 = last row band, bit 1 = last column band,
// each kept only where the window is on that edge: erow / ecol) against 4 consecutive tokens
// of one window row (row y, columns x .. x+3).  Region bits are integer arithmetic, not lane
// masks (those pinned SGPR pairs and spilled); UNI: 4 | lim, so the 4 tokens share a region.
template <bool UNI>
__device__ __forceinline__ void edge_mask(hvk_f32x4& s, int y, int x, int band, int erow, int ecol, int lim,
                                          float mask2) {
  const int br = (int)((unsigned)(lim - 1 - y) >> 31) & erow;
  if (UNI) {
    const int bc = ((int)((unsigned)(lim - 1 - x) >> 31) & ecol) << 1;
    const float m = (br | bc) != band ? mask2 : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r] += m;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int bc = ((int)((unsigned)(lim - 1 - x - r) >> 31) & ecol) << 1;
      s[r] += (br | bc) != band ? mask2 : 0.f;
    }
  }
}

// ------------------------------------------------------------------------------ forward
// Persistent workgroups, one head each, walking a run of windows (so the head's CPB table and
// bound are set up once), K and V of the NEXT window streamed into a second LDS buffer by
// LDS-DMA while this window computes.  Per window: wait for its DMA, normalise k^ in place
// (one pass over the image), barrier, then every wave runs its QT query tiles (positions
// 16 (wave + WAVES j) + li: whole window rows apart, so their bias indices differ by a
// compile-time step) jointly over all 32-key chunks, reading each K / V fragment once for the
// QT tiles.  S' = K^ (scale log2e Q^)^T + (log2e bias - M_h) comes from one MFMA with the
// mirrored CPB table as its C operand, M_h = scale log2e + max bias the head bound of every
// logit, so P = exp2(S') needs no running max; the row sums come from a ones-vector MFMA over
// the same bf16 P that multiplies V.  A tile whose row sum fell below 2^-100 (a row far below
// the head bound, scale ~100) is recomputed with the true running max (the reference's
// softmax, swinv2.py:256).  Interior windows and unshifted blocks run a mask-free copy of the
// loop; edge windows of shifted blocks add the -100 mask (swinv2.py:249-254), per 4-key group
// when 4 | (window - shift) (a lane's 4 keys share their region), else per element.
template <int WIN>
struct FCfg {
  using K = LCfg<WIN>;
  static constexpr int WAVES = WIN == 24 ? 12 : (WIN == 16 ? 8 : 3);
  static constexpr int OCC = WIN == 24 ? 1 : (WIN == 16 ? 2 : 3);  // workgroups per CU (LDS)
  static constexpr int QT = K::NT / WAVES;                          // query tiles per wave
  static_assert(K::NT % WAVES == 0, "whole query tiles per wave");
  static constexpr int DQ = 16 * WAVES;                             // position step between them
  static_assert(DQ % WIN == 0, "a wave's query tiles are whole window rows apart");
  static constexpr int DR = (DQ / WIN) * K::R;                      // bias-index step between them
  static constexpr int BLK = K::ROWS / 16;                          // 1-KB DMA blocks per image
  static constexpr int BUF = 2 * K::IMG;                            // k^ and v of one window
  static constexpr size_t LDS = 2 * (size_t)BUF + (size_t)K::TABM * 4 + 64;
  static constexpr int MINW = (OCC * WAVES) / 4 > 0 ? (OCC * WAVES) / 4 : 1;  // waves per SIMD
  // chunks per period of whole window rows (the main loop's unroll), 0: none divides NC
  static constexpr int PER = (32 * 3) % WIN == 0 && K::NC % 3 == 0 ? 3 : (32 % WIN == 0 ? 1 : 0);
};

// LDS-DMA of 16 B per lane from base + voff into LDS m0 + 16 lane, issued from inline asm: the
// compiler's wait-count pass does not see it, so it never drains it with the vmcnt(0) it puts
// in front of LDS reads while one of its own LDS-DMAs is pending.  The kernel waits for it with
// an explicit s_waitcnt before the barrier that publishes the buffer.

template <int WIN, bool LSE>
__global__ __launch_bounds__(64 * FCfg<WIN>::WAVES, FCfg<WIN>::MINW) void wmsa_fwd_large_kernel(FwdArgs a) {
  using K = LCfg<WIN>;
  using F = FCfg<WIN>;
  constexpr int QT = F::QT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int chunk, h;
  if (!decode_item(g, blockIdx.x, chunk, h)) return;
  const int w0 = (int)((long long)chunk * g.n_windows / g.n_chunks);
  const int w1 = (int)((long long)(chunk + 1) * g.n_windows / g.n_chunks);
  if (w0 >= w1) return;
  float* mtab = reinterpret_cast<float*>(smem + 2 * F::BUF);
  float* red = mtab + K::TABM;  // [WAVES] max-bias partials
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C;
  const int per_img = g.nWh * g.nWw;
  const float sc2 = a.scale[h] * HVK_LOG2E;
  const uint32_t sbase = lds_addr(smem);
  const char* qkv = reinterpret_cast<const char*>(a.qkv);
  const unsigned RB = 6u * C;  // bytes per qkv token row
  const size_t IMGB = (size_t)g.H * g.W * RB;

  // LDS-DMA of window (b, wh, ww) into the buffer at LDS byte address buf: instruction j fills
  // 1 KB of the fm16 image (16 rows x 4 16-B columns): lane L loads row 16 blk + drow, 16-B
  // column L / 16 (the inverse of fm16).  Padding rows (w12) load the window's first token:
  // finite values that the -inf key mask / P = 0 leave without effect.
  const int drow = (lane & 15) ^ (((lane >> 4) & 1) * 12);
  const unsigned lane_col = (unsigned)(h * 64 + (lane >> 4) * 16);
  auto issue = [&](int b, int wh, int ww, uint32_t buf) {
    const char* img = qkv + (size_t)b * IMGB;
    const int y0 = wh * WIN + g.shift, x0 = ww * WIN + g.shift;
    for (int j = wave; j < 2 * F::BLK; j += F::WAVES) {
      const int part = j >= F::BLK ? 1 : 0;
      const int blk = j - part * F::BLK;
      int pos = 16 * blk + drow;
      if (K::ROWS != K::N) pos = pos < K::N ? pos : 0;
      int y = y0 + pos / WIN, x = x0 + pos % WIN;
      if (y >= g.H) y -= g.H;
      if (x >= g.W) x -= g.W;
      const unsigned voff = (unsigned)HVK_BCHECK((unsigned)(y * g.W + x) * RB + (unsigned)((1 + part) * 2 * C) + lane_col,
                                                 IMGB);
      dma16(img, voff, buf + (uint32_t)(part * K::IMG + blk * 1024));
    }
  };
  // this wave's query tiles: positions 16 (wave + WAVES j) + li (bias index step DR per tile)
  const int qp0 = 16 * wave + li, qy0 = qp0 / WIN, qx = qp0 % WIN;
  const int tq0 = K::RR - 1 - ((qy0 + WIN - 1) * K::R + qx + WIN - 1);  // mirrored entry base
  uint4 qn[QT];  // raw q of the next window (in flight under this window's math)
  auto load_q = [&](int b, int wh, int ww) {
#pragma unroll
    for (int j = 0; j < QT; ++j) {
      const int row = window_token_row(g, b, wh, ww, WIN, qp0 + F::DQ * j);
      qn[j] = hvk_ld16(a.qkv + (size_t)row * (3 * C) + h * 32 + 8 * gq);
    }
  };

  // the head's bound and mirrored table, once per workgroup (every window is head h)
  const float* bsrc = a.bias + (size_t)h * K::RR;
  float mb = -INFINITY;
  for (int e = threadIdx.x; e < K::RR; e += 64 * F::WAVES) mb = fmaxf(mb, bsrc[e]);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) mb = fmaxf(mb, __shfl_xor(mb, m));
  if (lane == 0) red[wave] = mb;
  int cb = w0 / per_img, cwh = (w0 % per_img) / g.nWw, cww = w0 % g.nWw;
  issue(cb, cwh, cww, sbase);
  load_q(cb, cwh, cww);
  __syncthreads();
  float Mh = red[0];
#pragma unroll
  for (int i = 1; i < F::WAVES; ++i) Mh = fmaxf(Mh, red[i]);
  Mh = Mh * HVK_LOG2E + sc2;
  for (int e = threadIdx.x; e < K::TABM; e += 64 * F::WAVES) {
    const int i = K::RR - 1 - e;
    mtab[e] = i >= 0 ? bsrc[i] * HVK_LOG2E - Mh : 0.f;
  }
  // A operand of the row-sum MFMA: 1.0 for real keys of chunk c in k-slot order
  // (slot 8 gq + j <-> key 32c + 4gq + j for j < 4, 32c + 16 + 4gq + j - 4 for j >= 4)
  auto ones = [&](int c) {
    uint32_t wv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * jj + e;
        const int p = 32 * c + (j < 4 ? 4 * gq + j : 16 + 4 * gq + j - 4);
        if (p < K::N) v |= 0x3F80u << (16 * e);
      }
      wv[jj] = v;
    }
    return make_uint4(wv[0], wv[1], wv[2], wv[3]);
  };
  const float mask2 = -100.f * HVK_LOG2E;
  const int lim = WIN - g.shift;
  constexpr int NST = QT * (LSE ? 2 : 1);  // global stores per window per wave (out, lse)

  for (int w = w0, cur = 0; w < w1; ++w, cur ^= 1) {
    // this window's DMA and query loads have landed (younger: the previous window's stores)
    if (w == w0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    lds_barrier();  // every wave's DMA landed; the other buffer is free (previous window done)
    char* kimg = smem + cur * F::BUF;
    char* vimg = kimg + K::IMG;
    for (int blk = wave; blk < F::BLK; blk += F::WAVES) {  // k^ in place
      const int off = fm16(16 * blk + li, gq);
      float rn;
      *reinterpret_cast<uint4*>(kimg + off) = l2_normalize_seq(lds16(kimg, off), rn);
    }
    // this window's queries (normalised, times scale log2e): the loads are complete
    uint4 qf[QT];
#pragma unroll
    for (int j = 0; j < QT; ++j) {
      hvk_u32x4 v = __builtin_bit_cast(hvk_u32x4, qn[j]);
      asm volatile("" : "+v"(v));  // a fresh value: no compiler wait on the loads below
      float rn;
      qf[j] = l2_normalize_seq(__builtin_bit_cast(uint4, v), rn, sc2);
    }
    const int b = cb, wh = cwh, ww = cww;
    if (++cww == g.nWw) {
      cww = 0;
      if (++cwh == g.nWh) {
        cwh = 0;
        ++cb;
      }
    }
    if (w + 1 < w1) {
      issue(cb, cwh, cww, sbase + (uint32_t)((cur ^ 1) * F::BUF));
      load_q(cb, cwh, cww);
    }
    lds_barrier();  // k^ normalised

    const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
    // S' of (chunk c, half t, tile j) with this lane's 4 keys kp .. kp + 3 (one window row);
    // ky / kx: their window row and first column
    const int erow = edge_r ? 1 : 0, ecol = edge_c ? 1 : 0;
    // edge_t: 0 interior / unshifted, 1 edge window with 4 | lim, 2 edge window otherwise
    auto scores = [&](auto edge_t, int c, int t, int j, const uint4& kf, int ky, int kx) {
      constexpr int EDGE = decltype(edge_t)::value;
      const float* tp = mtab + (tq0 - F::DR * j + ky * K::R + kx);
      hvk_f32x4 s = hvk_mfma16(kf, qf[j], hvk_f32x4{tp[0], tp[1], tp[2], tp[3]});
      if (EDGE) {
        const int qy = qy0 + (F::DQ / WIN) * j;
        const int band = ((int)((unsigned)(lim - 1 - qy) >> 31) & erow) |
                         (((int)((unsigned)(lim - 1 - qx) >> 31) & ecol) << 1);
        edge_mask<EDGE == 1>(s, ky, kx, band, erow, ecol, lim, mask2);
      }
      if (K::N % 32 != 0 && c == K::NC - 1) {
        const int kp = 32 * c + 16 * t + 4 * gq;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kp + r >= K::N) s[r] = -INFINITY;
      }
      return s;
    };
    const uint4 one_full = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
    const uint4 one_last = K::N % 32 != 0 ? ones(K::NC - 1) : one_full;
    hvk_f32x4 o[QT][2], ls[QT];
    // lane-constant LDS byte addresses of this window's fragments (chunk c at + 2048 c):
    // k^ rows 32c + 16t + li, 16-B column gq (fm16: 2048 c + 1024 t + kl); V^T (tr_frag) rows
    // 32c + 4gq + li/4 (+16), 8-B column li%4 (+4 dt) (2048 c + 1024 h + 512 dt + vl)
    const uint32_t kl = lds_addr(kimg) + (uint32_t)fm16(li, gq);
    const uint32_t vl = lds_addr(vimg) + (uint32_t)fm8(4 * gq + (li >> 2), li & 3);
    const uint32_t tl = lds_addr(mtab) + 4u * (uint32_t)tq0;  // + 4 (bk(key) - DR j)
    auto run = [&](auto edge_t) {
      constexpr int EDGE = decltype(edge_t)::value;
#pragma unroll
      for (int j = 0; j < QT; ++j) o[j][0] = o[j][1] = ls[j] = hvk_f32x4{0, 0, 0, 0};
      // one chunk: K / V fragments read once for the QT tiles.  kb / vb: the chunk's fragment
      // addresses, tb[t]: the bias-table address of the lane's 4 keys (tile 0); ky / kx: their
      // window row and first column (edge masks, padding)
      auto chunk = [&](int c, uint32_t kb, uint32_t vb, const uint32_t (&tb)[2], const int (&ky)[2],
                       const int (&kx)[2]) {
        const uint4 kf[2] = {lds_ld16(kb), lds_ld16(kb + 1024)};
        uint4 vt[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const uint2 lo = lds_tr8(vb + 512 * dt), hi = lds_tr8(vb + 512 * dt + 1024);
          vt[dt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
        const uint4 one = (K::N % 32 != 0 && c == K::NC - 1) ? one_last : one_full;
        (void)one;
        // TAB_EARLY: every tile's bias C operands read with the chunk's K / V fragments, so their
        // latency is not exposed in front of each tile's score MFMAs (+16 VGPRs)
        hvk_f32x4 cb[HVK_LARGE_TAB_EARLY ? QT : 1][2];
        if (HVK_LARGE_TAB_EARLY) {
#pragma unroll
          for (int j = 0; j < QT; ++j)
#pragma unroll
            for (int t = 0; t < 2; ++t) cb[j][t] = lds_ld4f(tb[t] - 4u * (uint32_t)(F::DR * j));
        }
#pragma unroll
        for (int j = 0; j < QT; ++j) {
          hvk_f32x4 st[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            st[t] = hvk_mfma16(kf[t], qf[j],
                               HVK_LARGE_TAB_EARLY ? cb[HVK_LARGE_TAB_EARLY ? j : 0][t]
                                                   : lds_ld4f(tb[t] - 4u * (uint32_t)(F::DR * j)));
            if (EDGE) {
              const int qy = qy0 + (F::DQ / WIN) * j;
              const int band = ((int)((unsigned)(lim - 1 - qy) >> 31) & erow) |
                               (((int)((unsigned)(lim - 1 - qx) >> 31) & ecol) << 1);
              edge_mask<EDGE == 1>(st[t], ky[t], kx[t], band, erow, ecol, lim, mask2);
            }
            if (K::N % 32 != 0 && c == K::NC - 1) {
              const int kp = 32 * c + 16 * t + 4 * gq;
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (kp + r >= K::N) st[t][r] = -INFINITY;
            }
          }
          float p[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[r] = __builtin_amdgcn_exp2f(st[0][r]);
            p[4 + r] = __builtin_amdgcn_exp2f(st[1][r]);
          }
          const uint4 pf = make_uint4(hvk_pack2(p[0], p[1]), hvk_pack2(p[2], p[3]),
                                      hvk_pack2(p[4], p[5]), hvk_pack2(p[6], p[7]));
#if HVK_FWD_ROWSUM_MFMA
          ls[j] = hvk_mfma16(one, pf, ls[j]);
#else
          ls[j][0] += ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
#endif
          o[j][0] = hvk_mfma16(vt[0], pf, o[j][0]);
          o[j][1] = hvk_mfma16(vt[1], pf, o[j][1]);
        }
      };
      if constexpr (F::PER > 0) {
        // PER chunks span whole window rows: the lane's key rows / columns repeat with it; the
        // addresses are laundered once per period (a few base registers, compile-time offsets)
        constexpr int RPP = 32 * F::PER / WIN;  // window rows per period
#pragma unroll 1
        for (int cg = 0; cg < K::NC / F::PER; ++cg) {
          const uint32_t kb = launder(kl + 2048u * F::PER * cg);
          const uint32_t vb = launder(vl + 2048u * F::PER * cg);
          const uint32_t tb0 = launder(tl + 4u * RPP * K::R * cg);
          const int g4 = (int)launder((uint32_t)gq);
#pragma unroll
          for (int c2 = 0; c2 < F::PER; ++c2) {
            int ky[2], kx[2];
            uint32_t tb[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              const int kq = 32 * c2 + 16 * t + 4 * g4;  // position inside the period
              ky[t] = RPP * cg + kq / WIN;
              kx[t] = kq % WIN;
              tb[t] = tb0 + 4u * (uint32_t)((kq / WIN) * K::R + kq % WIN);
            }
            chunk(F::PER * cg + c2, kb + 2048u * c2, vb + 2048u * c2, tb, ky, kx);
          }
        }
      } else {
#pragma unroll 1
        for (int c = 0; c < K::NC; ++c) {
          const int g4 = (int)launder((uint32_t)gq);
          int ky[2], kx[2];
          uint32_t tb[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int kp = 32 * c + 16 * t + 4 * g4;
            ky[t] = kp / WIN;
            kx[t] = kp - ky[t] * WIN;
            tb[t] = tl + 4u * (uint32_t)(ky[t] * K::R + kx[t]);
          }
          chunk(c, launder(kl + 2048u * c), launder(vl + 2048u * c), tb, ky, kx);
        }
      }
    };
    if (!(edge_r || edge_c))
      run(std::integral_constant<int, 0>{});
    else if ((lim & 3) == 0)
      run(std::integral_constant<int, 1>{});
    else
      run(std::integral_constant<int, 2>{});
#pragma unroll
    for (int j = 0; j < QT; ++j) {
#if HVK_FWD_ROWSUM_MFMA
      float l = ls[j][0];
#else
      float l = hvk_group4_sum(ls[j][0]);
#endif
      float lshift = 0.f;  // the slow path's row max, on top of M_h
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(l >= 0x1p-100f)) != 0, 0)) {
        // slow path (rare, wave-uniform): this tile again with the true running max
        float m = -INFINITY;
        l = 0.f;
        o[j][0] = o[j][1] = hvk_f32x4{0, 0, 0, 0};
#pragma unroll 1
        for (int c = 0; c < K::NC; ++c) {
          const uint4 kf0 = lds16(kimg, fm16(32 * c + li, gq));
          const uint4 kf1 = lds16(kimg, fm16(32 * c + 16 + li, gq));
          const uint4 vt0 = tr_frag(vimg, c, 0, li, gq), vt1 = tr_frag(vimg, c, 1, li, gq);
          const int kp0 = 32 * c + 4 * gq, kp1 = kp0 + 16;
          hvk_f32x4 s0 = scores(std::integral_constant<int, 0>{}, c, 0, j, kf0, kp0 / WIN, kp0 % WIN);
          hvk_f32x4 s1 = scores(std::integral_constant<int, 0>{}, c, 1, j, kf1, kp1 / WIN, kp1 % WIN);
          hvk_settle(s0, s1);
          if (edge_r || edge_c) {
            const int qy = qy0 + (F::DQ / WIN) * j;
            const int band = ((int)((unsigned)(lim - 1 - qy) >> 31) & erow) |
                             (((int)((unsigned)(lim - 1 - qx) >> 31) & ecol) << 1);
            edge_mask<false>(s0, kp0 / WIN, kp0 % WIN, band, erow, ecol, lim, mask2);
            edge_mask<false>(s1, kp1 / WIN, kp1 % WIN, band, erow, ecol, lim, mask2);
          }
          float mc = -INFINITY;
#pragma unroll
          for (int r = 0; r < 4; ++r) mc = fmaxf(mc, fmaxf(s0[r], s1[r]));
          mc = hvk_group4_max(mc);
          const float mn = fmaxf(m, mc);
          const float alpha = __builtin_amdgcn_exp2f(m - mn);
          m = mn;
          float p[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[r] = __builtin_amdgcn_exp2f(s0[r] - mn);
            p[4 + r] = __builtin_amdgcn_exp2f(s1[r] - mn);
          }
          l = l * alpha + ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
          o[j][0] *= alpha;
          o[j][1] *= alpha;
          const uint4 pf = make_uint4(hvk_pack2(p[0], p[1]), hvk_pack2(p[2], p[3]),
                                      hvk_pack2(p[4], p[5]), hvk_pack2(p[6], p[7]));
          o[j][0] = hvk_mfma16(vt0, pf, o[j][0]);
          o[j][1] = hvk_mfma16(vt1, pf, o[j][1]);
        }
        l = hvk_group4_sum(l);
        lshift = m;
        hvk_settle(o[j][0], o[j][1]);  // read by the store block this path branches back to
      }
      // LSE: the query's log2 row constant L2 = M_h + row max + log2(row sum) for the backward
      const size_t row = window_token_row(g, b, wh, ww, WIN, qp0 + F::DQ * j);
      if (LSE && gq == 0) a.lse[row * g.nH + h] = Mh + lshift + __log2f(l);
      const float inv = __builtin_amdgcn_rcpf(l);
      // accumulator rows: channels 4gq + r (o[0]) and 16 + 4gq + r (o[1]); one permlane swap
      // per dword gives the lane 8 consecutive channels (one 16-B store)
      const uint4 pk = hvk_pair_swap(
          make_uint2(hvk_pack2(o[j][0][0] * inv, o[j][0][1] * inv), hvk_pack2(o[j][0][2] * inv, o[j][0][3] * inv)),
          make_uint2(hvk_pack2(o[j][1][0] * inv, o[j][1][1] * inv), hvk_pack2(o[j][1][2] * inv, o[j][1][3] * inv)));
      hvk_st16(a.out + row * C + h * 32 + hvk_pair_col(gq), pk);
    }
  }
}

// ----------------------------------------------------------------------------- backward
// Persistent workgroups (8 waves: the 8 private CPB-gradient bin copies fit beside the images),
// one head each over a run of windows: the head's table and bound are set up once, the bins,
// the logit-scale and q_bias gradients accumulate over the whole run and are flushed once.
// Per window, two phases over one LDS image pair:
//   phase 1, query on the lane (k^ / v images, contiguous query tiles): S' and dP by MFMA,
//     P = exp2(S' - L2) from the forward's row constant (LSE) or from a row-statistics pass,
//     dS = P (dP - delta_O) with delta_O = dO . O, dQ = scale sum_k dS k^; with LSE the exact
//     delta = sum P dP / sum P misses delta_O by corr = rowsum(dS) / rowsum(P), which is taken
//     out of dQ (scale corr sum_k P k^) and handed to phase 2 with the exact delta;
//   phase 2, key on the lane (q^ scale log2e / dO images, strided key tiles: positions
//     kt + NT li, so a batch of bin updates never repeats a bin, tools/large_bins_check.py):
//     the EXACT dS = P (dP - delta) gives dK, dV, the CPB-table gradient (private bins, plain
//     LDS read-add-write) and the logit-scale gradient.
// The next images are loaded into registers while the current phase computes (phase 1 loads
// phase 2's q / dO rows, phase 2 the next window's k / v rows) and written to LDS between the
// phases; every tile's own global inputs are loaded one tile ahead.  Interior windows and
// unshifted blocks run mask-free copies of both loops.
#ifndef HVK_LARGE_LATE_ROWS  // 1: the next phase's image rows loaded after the current phase's loop
#define HVK_LARGE_LATE_ROWS 1   // (frees their 40 VGPRs inside the loops; their latency is exposed)
#endif
#ifndef HVK_LARGE_TR_EARLY     // 1: phase 2's transposed dV / dK fragments read before the bins
#define HVK_LARGE_TR_EARLY 1
#endif
#ifndef HVK_LARGE_PROBE  // tools/ timing probes of the backward (results wrong): 1 no CPB bins, 2 no
                         // row-constant reads, 3 phase 1 skipped, 4 phase 2 skipped
#define HVK_LARGE_PROBE 0
#endif

template <int WIN>
struct BCfg {
  using K = LCfg<WIN>;
  static constexpr int WAVES = 8;
  static constexpr int BLK = K::ROWS / 16;                    // 16-row blocks per image
  static constexpr int PB = (BLK + WAVES - 1) / WAVES;        // blocks a wave stages per image
  static constexpr int RRP = (K::RR + 3) / 4 * 4;             // bins per private copy
  static constexpr int BATCH = WIN == 24 ? 8 : (WIN == 16 ? 4 : 1);  // exact read-add-write batch
  static constexpr size_t LDS = 2 * (size_t)K::IMG + (size_t)K::TABM * 4 + (size_t)WAVES * RRP * 4 +
                                2 * (size_t)K::ROWS * 4 + 64;
};

// 8 f32 of a 16x16 accumulator pair (rows 4gq + r of tile 0 = channels 4gq + r, of tile 1 =
// channels 16 + 4gq + r) -> this lane's 8 consecutive channels from hvk_pair_col(gq)
__device__ __forceinline__ void pair_swap_f32(const hvk_f32x4& t0, const hvk_f32x4& t1, float v[8]) {
#pragma unroll
  for (int r = 0; r < 4; r += 2) {
    const uint4 s = hvk_pair_swap(make_uint2(__float_as_uint(t0[r]), __float_as_uint(t0[r + 1])),
                                  make_uint2(__float_as_uint(t1[r]), __float_as_uint(t1[r + 1])));
    // hvk_pair_swap(lo pair, hi pair) -> (lo.x', lo.y', hi.x', hi.y') in channel order 2r, 2r+1 of
    // each half: output (a0, b0, a1, b1) = channels (r, r+1) of the first four, then of the last four
    v[r] = __uint_as_float(s.x);
    v[r + 1] = __uint_as_float(s.y);
    v[4 + r] = __uint_as_float(s.z);
    v[4 + r + 1] = __uint_as_float(s.w);
  }
}

// Normalize-backward of one head row and a 16-B store: x^ = x rn, dx = (dx^ post - x^ (x^ . dx^
// post)) rn over the lane's 8 channels (x: the raw row slice at hvk_pair_col(gq), dxh: the same
// channels); the 4 lanes of the row reduce the dot product.  acc (optional): column sums.
__device__ __forceinline__ void normalize_bwd16(const uint4& xraw, float rn, const float dxh[8], float post,
                                                 hvk_bf16* dst, float* acc) {
  float x[8], dot = 0.f;
  hvk_unpack8(xraw, x);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    x[e] *= rn;
    dot = fmaf(x[e], dxh[e] * post, dot);
  }
  dot = hvk_group4_sum(dot);
  if (rn >= 1e12f) dot = 0.f;  // ||x|| <= eps: x / eps, no projection term
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] = (dxh[e] * post - x[e] * dot) * rn;
    if (acc) acc[e] += v[e];
  }
  hvk_st16(dst, hvk_pack8(v));
}

template <int WIN, bool LSE>
__global__ __launch_bounds__(64 * BCfg<WIN>::WAVES, 2) void wmsa_bwd_large_kernel(BwdArgs a) {
  using K = LCfg<WIN>;
  using F = BCfg<WIN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int chunk, h;
  if (!decode_item(g, blockIdx.x, chunk, h)) return;
  const int w0 = (int)((long long)chunk * g.n_windows / g.n_chunks);
  const int w1 = (int)((long long)(chunk + 1) * g.n_windows / g.n_chunks);
  if (w0 >= w1) return;
  char* img0 = smem;
  char* img1 = smem + K::IMG;
  float* mtab = reinterpret_cast<float*>(smem + 2 * K::IMG);  // [TABM] mirrored, - M_h
  float* bins = mtab + K::TABM;                               // [WAVES][RRP] private copies
  float* lse_s = bins + F::WAVES * F::RRP;                    // [ROWS] row constant rel. to M_h
  float* dlt_s = lse_s + K::ROWS;                             // [ROWS] exact delta
  float* red = dlt_s + K::ROWS;                               // [16]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * C;
  const int per_img = g.nWh * g.nWw;
  const float scale = a.scale[h];
  const float sc2 = scale * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  const int lim = WIN - g.shift;
  const int pcol = hvk_pair_col(gq);  // the lane's 8 output channels after the pair swap

  const float* bsrc = a.bias + (size_t)h * K::RR;
  float mb = -INFINITY;
  for (int e = threadIdx.x; e < K::RR; e += 64 * F::WAVES) mb = fmaxf(mb, bsrc[e]);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) mb = fmaxf(mb, __shfl_xor(mb, m));
  if (lane == 0) red[wave] = mb;
  for (int e = threadIdx.x; e < F::WAVES * F::RRP; e += 64 * F::WAVES) bins[e] = 0.f;
  for (int e = threadIdx.x; e < K::ROWS; e += 64 * F::WAVES) {
    lse_s[e] = INFINITY;  // padding queries (w12): P = 0 in phase 2
    dlt_s[e] = 0.f;
  }

  // image staging through registers: a wave's blocks blk = wave + WAVES j, lane (li, gq) owns row
  // 16 blk + li, 16-B column gq (written at fm16: conflict free); padding rows load the
  // window's first token (finite; masked to -inf / weighted by P = 0)
  uint4 ra[F::PB], rb[F::PB];
  auto load_rows = [&](int b, int wh, int ww, int pa, int pbp) {  // parts (0 q, 1 k, 2 v) / dO
#pragma unroll
    for (int j = 0; j < F::PB; ++j) {
      const int blk = wave + F::WAVES * j;
      if (blk < F::BLK) {
        int pos = 16 * blk + li;
        if (K::ROWS != K::N) pos = pos < K::N ? pos : 0;
        const size_t row = window_token_row(g, b, wh, ww, WIN, pos);
        ra[j] = hvk_ld16(a.qkv + row * C3 + pa * C + h * 32 + 8 * gq);
        rb[j] = pbp < 0 ? hvk_ld16(a.dout + row * C + h * 32 + 8 * gq)
                        : hvk_ld16(a.qkv + row * C3 + pbp * C + h * 32 + 8 * gq);
      }
    }
  };
  auto write_rows = [&](float post) {  // ra normalised (times post), rb raw
#pragma unroll
    for (int j = 0; j < F::PB; ++j) {
      const int blk = wave + F::WAVES * j;
      if (blk < F::BLK) {
        float rn;
        const int off = fm16(16 * blk + li, gq);
        *reinterpret_cast<uint4*>(img0 + off) = l2_normalize_seq(ra[j], rn, post);
        *reinterpret_cast<uint4*>(img1 + off) = rb[j];
      }
    }
  };

  int cb = w0 / per_img, cwh = (w0 % per_img) / g.nWw, cww = w0 % g.nWw;
  load_rows(cb, cwh, cww, 1, 2);  // k, v of the first window
  __syncthreads();
  float Mh = red[0];
#pragma unroll
  for (int i = 1; i < F::WAVES; ++i) Mh = fmaxf(Mh, red[i]);
  Mh = Mh * HVK_LOG2E + sc2;
  for (int e = threadIdx.x; e < K::TABM; e += 64 * F::WAVES) {
    const int i = K::RR - 1 - e;
    mtab[e] = i >= 0 ? bsrc[i] * HVK_LOG2E - Mh : 0.f;
  }
  write_rows(1.f);
  lds_barrier();

  const uint4 one_full = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  auto ones_c = [&](int c) {  // 1.0 for the real positions of chunk c in k-slot order
    if (K::N % 32 == 0 || c != K::NC - 1) return one_full;
    uint32_t wv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * jj + e;
        const int p = 32 * c + (j < 4 ? 4 * gq + j : 16 + 4 * gq + j - 4);
        if (p < K::N) v |= 0x3F80u << (16 * e);
      }
      wv[jj] = v;
    }
    return make_uint4(wv[0], wv[1], wv[2], wv[3]);
  };
  // run fn(c, ky[2], kx[2]) over the chunks, ky / kx the window row and first column of the
  // lane's 4 positions 32c + 16t + 4gq .. +3 (periods of whole rows where the chunks allow)
  constexpr int PER = (32 * 3) % WIN == 0 && K::NC % 3 == 0 ? 3 : (32 % WIN == 0 ? 1 : 0);
  auto for_chunks = [&](auto&& fn) {
    if constexpr (PER > 0) {
#pragma unroll 1
      for (int cg = 0; cg < K::NC / PER; ++cg) {
#pragma unroll
        for (int c2 = 0; c2 < PER; ++c2) {
          int ky[2], kx[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int kq = 32 * c2 + 16 * t + 4 * gq;
            ky[t] = (32 * PER / WIN) * cg + kq / WIN;
            kx[t] = kq % WIN;
          }
          fn(PER * cg + c2, ky, kx);
        }
      }
    } else {
#pragma unroll 1
      for (int c = 0; c < K::NC; ++c) {
        int ky[2], kx[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int kp = 32 * c + 16 * t + 4 * gq;
          ky[t] = kp / WIN;
          kx[t] = kp - ky[t] * WIN;
        }
        fn(c, ky, kx);
      }
    }
  };

  // sum dS (S' - c) over the run = sc2 sum dS cos, from phase 2's f32 dS (the same sum from
  // phase 1's q^ . dq^ goes through bf16 dS and lost 3 % of this cancelling sum at scale 100)
  float dscale = 0.f;
  float dqb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float* pb = bins + wave * F::RRP;

  for (int w = w0; w < w1; ++w) {
    const int b = cb, wh = cwh, ww = cww;
    if (++cww == g.nWw) {
      cww = 0;
      if (++cwh == g.nWh) {
        cwh = 0;
        ++cb;
      }
    }
    const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
    const bool edge = edge_r || edge_c;

    // ---------------- phase 1: query tiles qt = wave + WAVES j (positions 16 qt + li)
    struct QIn {
      uint4 q, qx, dof, o;
      float lse;
      int row;
    };
    auto load_qt = [&](int qt) {
      QIn t;
      t.row = window_token_row(g, b, wh, ww, WIN, 16 * qt + li);
      const hvk_bf16* qp = a.qkv + (size_t)t.row * C3 + h * 32;
      t.q = hvk_ld16(qp + 8 * gq);
      t.qx = hvk_ld16(qp + pcol);
      t.dof = hvk_ld16(a.dout + (size_t)t.row * C + h * 32 + 8 * gq);
      if (LSE) {
        t.o = hvk_ld16(a.out + (size_t)t.row * C + h * 32 + 8 * gq);
        t.lse = a.lse[(size_t)t.row * g.nH + h];
      } else {
        t.o = make_uint4(0, 0, 0, 0);
        t.lse = 0.f;
      }
      return t;
    };
    // the first tile's inputs before phase 2's rows: in-order wait counts then never make a
    // tile wait for the row prefetch (issued next, consumed after the phase)
    QIn cur = load_qt(wave);
    if (!HVK_LARGE_LATE_ROWS) load_rows(b, wh, ww, 0, -1);  // phase 2's q / dO rows, under phase 1
#if HVK_LARGE_PROBE == 3  // probe: phase 1 skipped (timing only)
    for (int qt = K::NT; qt < K::NT; qt += F::WAVES) {
#else
    for (int qt = wave; qt < K::NT; qt += F::WAVES) {
#endif
      QIn nxt = cur;
      if (qt + F::WAVES < K::NT) nxt = load_qt(qt + F::WAVES);
      const int pos = 16 * qt + li;
      const int qy = pos / WIN, qxp = pos - qy * WIN;
      const int tq = K::RR - 1 - ((qy + WIN - 1) * K::R + qxp + WIN - 1);
      float rnq;
      const uint4 qs = l2_normalize_seq(cur.q, rnq, sc2);
      float rowc, delta;  // row constant (rel. to M_h) and delta for dS
      // a chunk half's operands: k^ / v fragments and the lane's 4 bias entries (C operand)
      struct TOps {
        uint4 a0, a1;
        hvk_f32x4 cb;
      };
      auto tile_ops = [&](int c, int t, int ky, int kx) {
        const float* tp = mtab + (tq + ky * K::R + kx);
        return TOps{lds16(img0, fm16(32 * c + 16 * t + li, gq)), lds16(img1, fm16(32 * c + 16 * t + li, gq)),
                    hvk_f32x4{tp[0], tp[1], tp[2], tp[3]}};
      };
      auto tile_from = [&](auto edge_t, int c, int t, int ky, int kx, const TOps& o, hvk_f32x4& s, hvk_f32x4& d,
                           float d0) {
        constexpr bool EDGE = decltype(edge_t)::value;
        s = hvk_mfma16(o.a0, qs, o.cb);
        d = hvk_mfma16(o.a1, cur.dof, hvk_f32x4{-d0, -d0, -d0, -d0});
        if (EDGE) {
          const bool rmis = edge_r && ((ky >= lim) != (qy >= lim));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool cmis = edge_c && ((kx + r >= lim) != (qxp >= lim));
            s[r] += (rmis || cmis) ? mask2 : 0.f;
          }
        }
        if (K::N % 32 != 0 && c == K::NC - 1) {
          const int kp = 32 * c + 16 * t + 4 * gq;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kp + r >= K::N) s[r] = -INFINITY;
        }
      };
      // S' (masked) and dP - d0 of (chunk c, half t): d0 (the row's delta, or 0) enters the dP
      // MFMA as its C operand
      auto tile = [&](auto edge_t, int c, int t, int ky, int kx, hvk_f32x4& s, hvk_f32x4& d, float d0) {
        tile_from(edge_t, c, t, ky, kx, tile_ops(c, t, ky, kx), s, d, d0);
      };
      if (LSE) {
        rowc = cur.lse - Mh;
        float fd[8], fo[8], dl = 0.f;
        hvk_unpack8(cur.dof, fd);
        hvk_unpack8(cur.o, fo);
#pragma unroll
        for (int e = 0; e < 8; ++e) dl = fmaf(fd[e], fo[e], dl);
        delta = hvk_group4_sum(dl);
      } else {
        // row statistics against the head bound (a running max only where the sum underflows)
        float l = 0.f, dacc = 0.f;
        auto statsA = [&](auto edge_t) {
          for_chunks([&](int c, const int (&ky)[2], const int (&kx)[2]) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              hvk_f32x4 s, d;
              tile(edge_t, c, t, ky[t], kx[t], s, d, 0.f);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float p = __builtin_amdgcn_exp2f(s[r]);
                l += p;
                dacc = fmaf(p, d[r], dacc);
              }
            }
          });
        };
        if (edge) statsA(std::true_type{}); else statsA(std::false_type{});
        l = hvk_group4_sum(l);
        dacc = hvk_group4_sum(dacc);
        float m = 0.f;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(l >= 0x1p-100f)) != 0, 0)) {
          m = -INFINITY;
          l = 0.f;
          dacc = 0.f;
#pragma unroll 1
          for (int c = 0; c < K::NC; ++c) {
            hvk_f32x4 s[2], d[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              const int kp = 32 * c + 16 * t + 4 * gq;
              if (edge) tile(std::true_type{}, c, t, kp / WIN, kp % WIN, s[t], d[t], 0.f);
              else tile(std::false_type{}, c, t, kp / WIN, kp % WIN, s[t], d[t], 0.f);
            }
            hvk_settle(s[0], s[1], d[0], d[1]);
            float mc = -INFINITY;
#pragma unroll
            for (int r = 0; r < 4; ++r) mc = fmaxf(mc, fmaxf(s[0][r], s[1][r]));
            mc = hvk_group4_max(mc);
            const float mn = fmaxf(m, mc);
            const float alpha = __builtin_amdgcn_exp2f(m - mn);
            m = mn;
            float ps = 0.f, pd = 0.f;
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float p = __builtin_amdgcn_exp2f(s[t][r] - mn);
                ps += p;
                pd = fmaf(p, d[t][r], pd);
              }
            l = l * alpha + ps;
            dacc = dacc * alpha + pd;
          }
          l = hvk_group4_sum(l);
          dacc = hvk_group4_sum(dacc);
        }
        rowc = m + __log2f(l);
        delta = dacc / l;
      }
      // loop B: dS, sum_k dS k^ (and with LSE sum_k P k^, sum_k P, sum_k dS)
      hvk_f32x4 dq[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, pk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
      hvk_f32x4 pp = {0, 0, 0, 0};
      float lk = 0.f;
      auto loopB = [&](auto edge_t) {
        for_chunks([&](int c, const int (&ky)[2], const int (&kx)[2]) {
          float p[8], ds[8];
          // OPS_EARLY: both halves' operands and the transposed k^ fragments of dQ read up front,
          // one LDS wait per chunk instead of one in front of every MFMA
          TOps o[2];
          uint4 kt[2];
          if (HVK_LARGE_OPS_EARLY) {
#pragma unroll
            for (int t = 0; t < 2; ++t) o[t] = tile_ops(c, t, ky[t], kx[t]);
            kt[0] = tr_frag(img0, c, 0, li, gq);
            kt[1] = tr_frag(img0, c, 1, li, gq);
          }
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            hvk_f32x4 s, d;
            if (HVK_LARGE_OPS_EARLY) tile_from(edge_t, c, t, ky[t], kx[t], o[t], s, d, delta);  // d = dP - delta
            else tile(edge_t, c, t, ky[t], kx[t], s, d, delta);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              p[4 * t + r] = __builtin_amdgcn_exp2f(s[r] - rowc);  // padding keys: 0
              ds[4 * t + r] = p[4 * t + r] * d[r];
              if (LSE) lk += ds[4 * t + r];
            }
          }
          const uint4 dsf = make_uint4(hvk_pack2(ds[0], ds[1]), hvk_pack2(ds[2], ds[3]),
                                       hvk_pack2(ds[4], ds[5]), hvk_pack2(ds[6], ds[7]));
          const uint4 kf0 = HVK_LARGE_OPS_EARLY ? kt[0] : tr_frag(img0, c, 0, li, gq);
          const uint4 kf1 = HVK_LARGE_OPS_EARLY ? kt[1] : tr_frag(img0, c, 1, li, gq);
          dq[0] = hvk_mfma16(kf0, dsf, dq[0]);
          dq[1] = hvk_mfma16(kf1, dsf, dq[1]);
          if (LSE) {
            const uint4 pf = make_uint4(hvk_pack2(p[0], p[1]), hvk_pack2(p[2], p[3]),
                                        hvk_pack2(p[4], p[5]), hvk_pack2(p[6], p[7]));
            pk[0] = hvk_mfma16(kf0, pf, pk[0]);
            pk[1] = hvk_mfma16(kf1, pf, pk[1]);
            pp = hvk_mfma16(ones_c(c), pf, pp);
          }
        });
      };
      if (edge) loopB(std::true_type{}); else loopB(std::false_type{});
      float dlt = delta, corr = 0.f;
      if (LSE) {
        corr = hvk_group4_sum(lk) / pp[0];
        dlt = delta + corr;
      }
      if (gq == 0) {
        lse_s[pos] = rowc;
        dlt_s[pos] = -dlt;  // phase 2's dP MFMA takes -delta as its C operand
      }
      // dq^ = scale (sum_k dS k^ - corr sum_k P k^) in this lane's 8 output channels
      hvk_f32x4 e0, e1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        e0[r] = scale * fmaf(-corr, pk[0][r], dq[0][r]);
        e1[r] = scale * fmaf(-corr, pk[1][r], dq[1][r]);
      }
      float dxh[8];
      pair_swap_f32(e0, e1, dxh);
      normalize_bwd16(cur.qx, rnq, dxh, 1.f, a.dqkv + (size_t)cur.row * C3 + h * 32 + pcol, dqb);
      cur = nxt;
    }
    if (HVK_LARGE_LATE_ROWS) load_rows(b, wh, ww, 0, -1);
    lds_barrier();             // phase-1 reads done; row constants published
    write_rows(sc2);           // q^ scale log2e (exactly the forward's operand), dO
    lds_barrier();

    // ---------------- phase 2: key tiles kt = wave + WAVES j (positions kt + NT li)
    struct KIn {
      uint4 k, kx, v;
      int row;
    };
    auto load_kt = [&](int kt) {
      KIn t;
      t.row = window_token_row(g, b, wh, ww, WIN, kt + K::NT * li);
      const hvk_bf16* kp = a.qkv + (size_t)t.row * C3 + C + h * 32;
      t.k = hvk_ld16(kp + 8 * gq);
      t.kx = hvk_ld16(kp + pcol);
      t.v = hvk_ld16(kp + C + 8 * gq);
      return t;
    };
    KIn kc = load_kt(wave);
    if (!HVK_LARGE_LATE_ROWS && w + 1 < w1) load_rows(cb, cwh, cww, 1, 2);  // the next window's k / v, under phase 2
#if HVK_LARGE_PROBE == 4  // probe: phase 2 skipped (timing only)
    for (int kt = K::NT; kt < K::NT; kt += F::WAVES) {
#else
    for (int kt = wave; kt < K::NT; kt += F::WAVES) {
#endif
      KIn kn = kc;
      if (kt + F::WAVES < K::NT) kn = load_kt(kt + F::WAVES);
      const int pos = kt + K::NT * li;
      const int ky = pos / WIN, kxp = pos - ky * WIN;
      const int tk = K::RR - 1 + ky * K::R + kxp;  // mirrored entry of query bq: tk - bq
      const int bk = ky * K::R + kxp;
      float rnk;
      const uint4 kh = l2_normalize_seq(kc.k, rnk);
      hvk_f32x4 dk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, dv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
      auto loop2 = [&](auto edge_t) {
        constexpr bool EDGE = decltype(edge_t)::value;
        for_chunks([&](int c, const int (&qyy)[2], const int (&qxx)[2]) {
          float p[8], ds[8];
          // TR_EARLY: the dV / dK operands (transposed dO / q^ fragments) read up front: the compiler
          // may not move LDS reads across the bins' read-add-write below, where each read exposes
          // its whole latency in front of its MFMA
          uint4 tv[2], tkf[2];
          if (HVK_LARGE_TR_EARLY) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
              tv[dt] = tr_frag(img1, c, dt, li, gq);
              tkf[dt] = tr_frag(img0, c, dt, li, gq);
            }
          }

#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int q0 = 32 * c + 16 * t + 4 * gq;  // this lane's queries q0 .. q0 + 3
            const int bq = (qyy[t] + WIN - 1) * K::R + qxx[t] + WIN - 1;
            const float* tp = mtab + (tk - bq);  // entries tp[-r]
            const hvk_f32x4 c4 = {tp[0], tp[-1], tp[-2], tp[-3]};
#if HVK_LARGE_PROBE == 2  // probe: row constants not read (wrong values, timing only)
            const float4 l4 = make_float4(rnk, rnk, rnk, rnk), d4 = l4;
#else
            const float4 l4 = *reinterpret_cast<const float4*>(lse_s + q0);
            const float4 d4 = *reinterpret_cast<const float4*>(dlt_s + q0);  // -delta
#endif
            hvk_f32x4 s = hvk_mfma16(lds16(img0, fm16(32 * c + 16 * t + li, gq)), kh, c4);
            const hvk_f32x4 d = hvk_mfma16(lds16(img1, fm16(32 * c + 16 * t + li, gq)), kc.v,
                                           hvk_f32x4{d4.x, d4.y, d4.z, d4.w});  // dP - delta
            const float lr[4] = {l4.x, l4.y, l4.z, l4.w};
            if (EDGE) {
              const bool rmis = edge_r && ((ky >= lim) != (qyy[t] >= lim));
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const bool cmis = edge_c && ((kxp >= lim) != (qxx[t] + r >= lim));
                s[r] += (rmis || cmis) ? mask2 : 0.f;
              }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float pr = __builtin_amdgcn_exp2f(s[r] - lr[r]);  // padding query: lse +inf
              const float dsr = pr * d[r];
              p[4 * t + r] = pr;
              ds[4 * t + r] = dsr;
              dscale = fmaf(dsr, s[r] - c4[r], dscale);
            }
          }
          // CPB-table gradient: this wave's own bins, batches of BATCH elements that never share a
          // bin across the lanes (strided key tiles); the compiler fences keep one batch's reads
          // behind the previous batch's writes.  (LDS float atomics instead -- ds_add_f32, one op
          // per element -- ran the w24 backward 4.9x slower: profiles/round3/large_bins_atomic_ab.txt)
#if HVK_LARGE_PROBE == 1  // probe: no CPB-gradient bins (wrong values, timing only)
          if (false)
#endif
#pragma unroll
          for (int b0 = 0; b0 < 8; b0 += F::BATCH) {
            float v[F::BATCH];
            int bi[F::BATCH];
            asm volatile("" ::: "memory");
#pragma unroll
            for (int e = 0; e < F::BATCH; ++e) {
              const int t = (b0 + e) >> 2, r = (b0 + e) & 3;
              const int bq = (qyy[t] + WIN - 1) * K::R + qxx[t] + r + WIN - 1;
              bi[e] = bq - bk;
              const bool ok = K::N % 32 == 0 || 32 * c + 16 * t + 4 * gq + r < K::N;
              v[e] = ok ? pb[bi[e]] : 0.f;
            }
#pragma unroll
            for (int e = 0; e < F::BATCH; ++e) {
              const int t = (b0 + e) >> 2, r = (b0 + e) & 3;
              const bool ok = K::N % 32 == 0 || 32 * c + 16 * t + 4 * gq + r < K::N;
              if (ok) pb[bi[e]] = v[e] + ds[b0 + e];
            }
            asm volatile("" ::: "memory");
          }
          const uint4 pf = make_uint4(hvk_pack2(p[0], p[1]), hvk_pack2(p[2], p[3]),
                                      hvk_pack2(p[4], p[5]), hvk_pack2(p[6], p[7]));
          const uint4 dsf = make_uint4(hvk_pack2(ds[0], ds[1]), hvk_pack2(ds[2], ds[3]),
                                       hvk_pack2(ds[4], ds[5]), hvk_pack2(ds[6], ds[7]));
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            dv[dt] = hvk_mfma16(HVK_LARGE_TR_EARLY ? tv[dt] : tr_frag(img1, c, dt, li, gq), pf, dv[dt]);
            dk[dt] = hvk_mfma16(HVK_LARGE_TR_EARLY ? tkf[dt] : tr_frag(img0, c, dt, li, gq), dsf, dk[dt]);
          }
        });
      };
      if (edge) loop2(std::true_type{}); else loop2(std::false_type{});
      // dk^ = sum_q scale dS q^ = sum_q dS (q^ scale log2e) / log2e
      hvk_bf16* dst = a.dqkv + (size_t)kc.row * C3 + h * 32;
      float dxh[8];
      pair_swap_f32(dk[0], dk[1], dxh);
      normalize_bwd16(kc.kx, rnk, dxh, 1.f / HVK_LOG2E, dst + C + pcol, nullptr);
      const uint4 vk = hvk_pair_swap(make_uint2(hvk_pack2(dv[0][0], dv[0][1]), hvk_pack2(dv[0][2], dv[0][3])),
                                     make_uint2(hvk_pack2(dv[1][0], dv[1][1]), hvk_pack2(dv[1][2], dv[1][3])));
      hvk_st16(dst + 2 * C + pcol, vk);
      kc = kn;
    }
    if (HVK_LARGE_LATE_ROWS && w + 1 < w1) load_rows(cb, cwh, cww, 1, 2);
    lds_barrier();  // phase-2 reads done
    if (w + 1 < w1) {
      write_rows(1.f);  // the next window's k^, v
      lds_barrier();
    }
  }

  // this (chunk, head)'s gradients, deterministically: the waves' private bins summed in wave
  // order, the wave sums of d scale / d q_bias staged in LDS and added in wave order, all added to
  // the workgroup's own workspace slot (no float atomics; the finalize sums slots in chunk order)
  constexpr int SLOT = bwd_slot_floats(WIN);
  float* slot = a.dbias_acc + ((size_t)h * a.slot_stride + chunk) * SLOT;
  for (int e = threadIdx.x; e < K::RR; e += 64 * F::WAVES) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < F::WAVES; ++c) v += bins[c * F::RRP + e];
    slot[e] = a.slot_add ? slot[e] + v : v;
  }
  dscale = hvk_wave_sum(dscale);
  float qbv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) qbv[e] = hvk_row16_sum(dqb[e]);
  float* stg = reinterpret_cast<float*>(img0);  // free: the last window's phase-2 reads are done
  static_assert(F::WAVES <= 16, "stage layout");
  if (lane == 0) stg[wave] = dscale / sc2;
  if (li == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) stg[16 + wave * 32 + pcol + e] = qbv[e];
  }
  lds_barrier();  // LDS only: the dK / dV and slot stores stay in flight
  if (threadIdx.x < 33) {
    float v = 0.f;
    for (int w = 0; w < F::WAVES; ++w) v += threadIdx.x == 0 ? stg[w] : stg[16 + w * 32 + threadIdx.x - 1];
    slot[K::RR + threadIdx.x] = a.slot_add ? slot[K::RR + threadIdx.x] + v : v;
  }
}

// sum the (head, chunk) slots in chunk order into dtab / dscale / dq_bias, leave the workspace zero
template <int WIN>
__global__ __launch_bounds__(FIN_THREADS) void wmsa_finalize_large_kernel(BwdArgs a, float* __restrict__ dtab,
                                                                  float* __restrict__ dscale,
                                                                  float* __restrict__ dqb) {
  finalize_slots<WIN>(a, dtab, dscale, dqb, blockIdx.x, blockIdx.y);
}

template <int WIN, bool LSE>
int launch_fwd_large_(FwdArgs a, hipStream_t st) {
  using F = FCfg<WIN>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_fwd_large_kernel<WIN, LSE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)F::LDS);
    attr = true;
  }
  // persistent: OCC resident workgroups per CU, n_chunks (multiple of 8) x heads of them
  int rc = make_geom(a.g.B, a.g.H, a.g.W, a.g.C, a.g.nH, WIN, a.g.shift, 256 * F::OCC, a.g);
  if (rc) return rc;
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_FWD, (wmsa_fwd_large_kernel<WIN, LSE>), dim3(a.g.n_chunks * a.g.nH),
                   dim3(64 * F::WAVES), F::LDS, st, a);
  HVK_CHECK_LAUNCH("wmsa_fwd_large");
  return HVK_OK;
}
template <int WIN>
int launch_fwd_large(const FwdArgs& a, hipStream_t st) {
  return a.lse ? launch_fwd_large_<WIN, true>(a, st) : launch_fwd_large_<WIN, false>(a, st);
}

template <int WIN, bool LSE>
int launch_bwd_large_(BwdArgs a, hipStream_t st) {
  using F = BCfg<WIN>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_large_kernel<WIN, LSE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)F::LDS);
    attr = true;
  }
  // persistent: one resident workgroup per CU, n_chunks (multiple of 8) x heads of them
  int rc = make_geom(a.g.B, a.g.H, a.g.W, a.g.C, a.g.nH, WIN, a.g.shift, 256, a.g);
  if (rc) return rc;
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, (wmsa_bwd_large_kernel<WIN, LSE>), dim3(a.g.n_chunks * a.g.nH),
                   dim3(64 * F::WAVES), F::LDS, st, a);
  return HVK_OK;
}

template <int WIN>
int launch_bwd_large(const BwdArgs& a, float* dtab, float* dscale, float* dqb, hipStream_t st) {
  if (a.lse) launch_bwd_large_<WIN, true>(a, st);
  else launch_bwd_large_<WIN, false>(a, st);
  HVK_CHECK_LAUNCH("wmsa_bwd_large");
  hipLaunchKernelGGL(wmsa_finalize_large_kernel<WIN>, dim3(a.g.nH, finalize_blocks_y(WIN)), dim3(FIN_THREADS), 0, st, a,
                     dtab, dscale, dqb);
  HVK_CHECK_LAUNCH("wmsa_finalize_large");
  return HVK_OK;
}

}  // namespace

bool large_window(int win) { return win == 12 || win == 16 || win == 24; }

int large_fwd(const FwdArgs& a, int win, hipStream_t st) {
  switch (win) {
    case 12: return launch_fwd_large<12>(a, st);
    case 16: return launch_fwd_large<16>(a, st);
    case 24: return launch_fwd_large<24>(a, st);
    default: return hvk_set_error(HVK_EUNSUPPORTED, "wmsa: window %d not built", win);
  }
}

int large_bwd(const BwdArgs& a, int win, float* dbias_table, float* dscale, float* dq_bias,
              hipStream_t st) {
  switch (win) {
    case 12: return launch_bwd_large<12>(a, dbias_table, dscale, dq_bias, st);
    case 16: return launch_bwd_large<16>(a, dbias_table, dscale, dq_bias, st);
    case 24: return launch_bwd_large<24>(a, dbias_table, dscale, dq_bias, st);
    default: return hvk_set_error(HVK_EUNSUPPORTED, "wmsa: window %d not built", win);
  }
}

}  // namespace hvk_wmsa
