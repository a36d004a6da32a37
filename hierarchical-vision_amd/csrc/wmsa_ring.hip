// W-MSA forward for windows <= 8 on gfx950: persistent workgroups that stream window slabs
// through LDS by LDS-DMA.  Same math as the reference sequence listed in wmsa.hip
// (swinv2.py:221-261 with the roll/partition/reverse of 399-429 folded into addressing).
//
// Work unit: (window, group of HG heads); a workgroup = HG waves (one per head) walks a
// contiguous chunk of windows for one head group.  Per window:
//   1. the window's q/k/v bytes of the head group are staged into one LDS "slab"
//      [N tokens][3 parts][HG*32] bf16 (RS = 12*HG 16-B slots per token) by
//      global_load_lds_dwordx4, filled lane-linearly (slot = 64*instr + lane): every DMA
//      wave-instruction reads whole row segments (HG*64 B per token and part; at HG = nH the
//      full 6C-byte row, and the 7 tokens of a window row are adjacent in memory);
//   2. each wave copies its head's q/k fragments (ds_read_b128) and V^T fragments
//      (ds_read_b64_tr_b16) into registers, the workgroup syncs, and the NEXT window's DMA is
//      issued into the same slab, so it is in flight during this window's math and stores;
//   3. S^T = K^ (scale log2e Q^)^T + bias on MFMA with the CPB bias as the C operand,
//      gathered from a compact per-head LDS table by ds_read_b32 with compile-time offsets;
//      softmax in registers; O^T = V^T P^T on MFMA; 16-B output stores per lane.
// Tokens of a window sit in the 16-row MFMA tiles on a PW-wide grid (PW = 8; 4 for w4):
// position p = PW*y + x.  The rel-pos index of (query p, key p') is then
// TR*(qi - ki) - r + base(lane) with TR = (16/PW)(2w-1): one lane-constant VGPR plus an
// immediate offset per (qi, ki, r), no address arithmetic in the loop.  Grid positions with
// x >= w or y >= w are padding: zero fragments, zero V rows, -inf scores.
#include <stdlib.h>

#include "wmsa_ring.h"

#ifndef HVK_RING_PROBE
#define HVK_RING_PROBE 0
#endif
#ifndef HVK_RING_AUX  // slab DMA cache policy (A/B builds): 2 nontemporal, 1 only for whole-row groups, 0 never
#define HVK_RING_AUX 2
#endif
#ifndef HVK_RING_ROWMAX_CHECK  // 0: A/B probe builds without the underflow check (not exact)
#define HVK_RING_ROWMAX_CHECK 1
#endif

namespace {
using namespace hvk_ring;

template <int WIN, int HG, bool LSE>
__global__ __launch_bounds__(64 * HG, 4) void wmsa_fwd_ring_kernel(FwdArgs a) {
  using K = RingCfg<WIN, HG>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  const int ng = g.nH / HG;
  const int bid = blockIdx.x, xcd = bid & 7, loc = bid >> 3;
  const int grp = loc % ng, chunk = (loc / ng) * 8 + xcd;  // a chunk's groups share an XCD
  if (chunk >= g.n_chunks) return;
  const int w0 = (int)((long long)chunk * g.n_windows / g.n_chunks);
  const int w1 = (int)((long long)(chunk + 1) * g.n_windows / g.n_chunks);
  if (w0 >= w1) return;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C;
  const int h = grp * HG + wave;
  const int per_img = g.nWh * g.nWw;
  const char* qkv = reinterpret_cast<const char*>(a.qkv);
  const int grp_off = grp * HG * 64;  // byte offset of the group inside a q/k/v part

  char* zero16 = smem + K::SLAB;
  float* btab = reinterpret_cast<float*>(smem + K::SLAB + 16);

  // LDS-DMA of a window's slab.  Slot P = RUN*ty + 64m + lane of instruction j = IPR*ty + m
  // holds token (ty, tx), part, 16-B column c with (tx, part, c) fixed by (m, lane): each lane
  // keeps pre[k % KP] = tx*RB + part*2C + 16c + group offset (bits 0-23) | tx << 24 for its
  // k-th instruction (j = wave + HG*k) and the window adds one uniform row offset.  Slots past
  // a run's WIN*RS are never read: they load the run's first bytes again (no exec masking).
  // Offsets are 32-bit from the image base; a window's rows wrap around the image (cyclic
  // shift) only on the last window row (uniform test) / column (per lane, edge windows only).
  const unsigned RB = 6u * C, WRB = (unsigned)g.W * RB, HWRB = (unsigned)g.H * WRB;
  unsigned pre[K::KP];
#pragma unroll
  for (int k = 0; k < K::KP; ++k) {
    const int m = (wave + HG * k) % K::IPR;
    const unsigned q = 64u * m + lane;
    unsigned v = grp_off;
    if (q < (unsigned)(WIN * K::RS)) {
      const unsigned tx = q / K::RS, r = q - tx * K::RS;
      const unsigned part = r / (4 * HG), c = r - part * (4 * HG);
      v = (tx * RB + part * 2 * C + c * 16 + grp_off) | (tx << 24);
    }
    pre[k] = v;
  }
  auto issue = [&](int b, int wh, int ww) {
    const char* img = qkv + (size_t)b * HWRB;
    const int y0 = wh * WIN + g.shift, x0 = ww * WIN + g.shift;
    const int ly = g.H - y0, lx = g.W - x0;  // ty >= ly (tx >= lx): the row wraps
#pragma unroll
    for (int k = 0; k < K::NK; ++k) {
      const int j = wave + HG * k;
      if (j < K::NINST) {
        const int ty = j / K::IPR;
        const unsigned U = ((unsigned)(y0 + ty - (ty >= ly ? g.H : 0)) * g.W + x0) * RB;  // uniform
        unsigned off = __umul24(pre[k % K::KP], 1u) + U;  // v_mad_u32_u24: low 24 bits of pre
        if (lx < WIN)  // last window column: per-lane wrap of the token column
          off -= ((int)(pre[k % K::KP] >> 24) >= lx) ? WRB : 0u;
        // nontemporal: every byte is read once, and the hint keeps qkv from evicting what the
        // next kernels read (this kernel's output feeds the proj GEMM).  HVK_RING_AUX = 1 drops
        // it where several head groups share a token row: this kernel is then 2-6 % faster at
        // stages 2-3 (tools/gpu_fwdaux.sh) but the step 0.4 % slower (interleaved A/B), so 2
        if (HVK_RING_AUX == 2 || (HVK_RING_AUX == 1 && ng == 1))
          __builtin_amdgcn_global_load_lds((gbl_vptr)(img + off), (lds_vptr)(smem + j * 1024), 16, 0, 2);
        else
          __builtin_amdgcn_global_load_lds((gbl_vptr)(img + off), (lds_vptr)(smem + j * 1024), 16, 0, 0);
      }
    }
  };
  // per-workgroup setup, overlapping nothing yet: bias tables = bias*log2e - M_h, where
  // M_h = scale*log2e + max(bias)*log2e bounds every logit of head h from above.  Softmax is
  // shift invariant, so the fast path exponentiates these shifted logits without a row max.
  // That is exact unless a query's best key lies far below the head bound (q and k come from
  // different slices of qkv.weight, so max cos can be anywhere in [-1, 1]: at scale 100 a row
  // with max cos < 0.3 can underflow to a zero row sum).  Every query tile therefore checks
  // its row sums and, where any is below 2^-100, recomputes that tile with the true row max
  // (the reference's softmax, swinv2.py:256): the fast path's result is kept only when it is
  // provably accurate (every P entry is a bf16 with 8 mantissa bits at any exponent >= -126,
  // so a row sum >= 2^-100 loses nothing that matters).
  // stored mirrored (entry PAD + i at TABF - 1 - PAD - i): the 4 accumulator rows r of a
  // (query tile, key tile) pair are then 4 ASCENDING dwords, read by two ds_read2_b32 straight
  // into the MFMA C operand
  for (int e = threadIdx.x; e < HG * K::TABF; e += 64 * HG) {
    const int hl = e / K::TABF, i = K::TABF - 1 - e % K::TABF - K::PAD;
    btab[e] = (i >= 0 && i < K::R * K::R) ? a.bias[(size_t)(grp * HG + hl) * K::R * K::R + i] * HVK_LOG2E
                                          : 0.f;
  }
  if (threadIdx.x == 0) *reinterpret_cast<uint4*>(zero16) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  float Mh;  // the head bound (log2 units): L2 of a query = Mh + log2(row sum) on the fast path
  {
    float mb = -INFINITY;
    float* tb = btab + wave * K::TABF + K::TABF - K::PAD - K::R * K::R;  // mirrored real entries
    for (int i = lane; i < K::R * K::R; i += 64) mb = fmaxf(mb, tb[i]);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) mb = fmaxf(mb, __shfl_xor(mb, m));
    Mh = __builtin_fmaf(a.scale[h], HVK_LOG2E, mb);  // one rounding (wmsa_win.hip matches it)
    for (int i = lane; i < K::R * K::R; i += 64) tb[i] -= Mh;
  }
  const float sc2 = a.scale[h] * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  // lane constants: bias base index, key-slot coordinates (slot bit ki*4 + r)
  int lq, lk;
  if (K::PW == 8) {
    lq = (li >> 3) * K::R + (li & 7);
    lk = (gq >> 1) * K::R + 4 * (gq & 1);
  } else {
    lq = (li >> 2) * K::R + (li & 3);
    lk = gq * K::R;
  }
  // bias(query tile qi, key tile ki, row r) sits at dword TR*(NT - 1 - qi + ki) + r from bta:
  // non-negative immediates < 256 (the ds_read2_b32 offset fields)
  const uint32_t bta =
      lds_addr(btab) + 4 * (wave * K::TABF + K::TABF - 4 - (K::PAD + K::BASE0 + lq - lk - K::TR * (K::NT - 1) - 3) -
                            2 * K::TR * (K::NT - 1));
  static_assert(2 * K::TR * (K::NT - 1) + 3 < 256, "bias offsets exceed ds_read2_b32's field");
  // A operand of the row-sum MFMA: 1.0 for real keys of chunk c in k-slot order (B operand
  // of P^T: slot 8gq + j <-> key 32c + 4gq + j, j < 4; 32c + 16 + 4gq + j - 4, j >= 4)
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
  // key-slot region bits (slot bit ki*4 + r): row band in bits 0-15, column band in 16-31
  uint32_t kband = 0;
#pragma unroll
  for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * ki + 4 * gq + r, ky = p / K::PW, kx = p % K::PW;
      if (ky >= WIN - g.shift) kband |= 1u << (ki * 4 + r);
      if (kx >= WIN - g.shift) kband |= 1u << (16 + ki * 4 + r);
    }

  // window coordinates advance incrementally (no per-window integer divisions)
  int cb = w0 / per_img, cwh = (w0 % per_img) / g.nWw, cww = w0 % g.nWw;
  issue(cb, cwh, cww);
  const uint32_t zaddr = lds_addr(zero16);
  for (int w = w0; w < w1; ++w) {
    // this window's slab has landed: at w > w0 the NT output stores (+ NT row-constant stores
    // with LSE) of the previous window were issued after its DMA and may still be in flight
    if (w == w0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LSE ? 2 * K::NT : K::NT) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    // lane coordinates recomputed per window (kept out of the loop-invariant pool: VGPRs)
    int l16 = li, g4 = gq;
    asm volatile("" : "+v"(l16), "+v"(g4));
    hvk_u32x4 qr[K::NT], kr[K::NT];
    hvk_u32x2 vr[K::NC][2][2];
    {
      // tile i, lane li: grid (y, x) = ((16/PW) i + li/PW, li%PW): token = (16/PW) WIN i + base
      const int x = l16 % K::PW, y0 = l16 / K::PW;
      const uint32_t fb = lds_addr(smem) + (y0 * K::RUN + x * K::RS + wave * 4 + g4) * 16;
#pragma unroll
      for (int i = 0; i < K::NT; ++i) {
        const bool ok = x < WIN && y0 + (16 / K::PW) * i < WIN;
        const uint32_t aq = fb + (16 / K::PW) * i * K::RUN * 16;
        qr[i] = lds_rd128<0>(ok ? aq : zaddr);
        kr[i] = lds_rd128<0>(ok ? aq + 4 * HG * 16 : zaddr);
      }
    }
    {
      // V^T fragments: chunk c, lane (li, gq), dt: key position p = 32c + 16h + 4gq + li/4
      // (h = 0, 1 for the two 8-B halves), channels d = 8(li&3) + 4dt ..+3; the output
      // accumulator o[dt][r] of lane (q, gq) then holds d = 8gq + 4dt + r (8 consecutive
      // channels per lane: one 16-B store).  Padding keys read 16 zero bytes.
      const int pl = 4 * g4 + (l16 >> 2);  // p - 32c - 16h, in [0, 16)
      const int x = pl % K::PW, y0 = pl / K::PW;
      const uint32_t vb = lds_addr(smem) + (y0 * K::RUN + x * K::RS) * 16 +
                          (2 * HG * 32 + wave * 32 + 8 * (l16 & 3)) * 2;
#pragma unroll
      for (int c = 0; c < K::NC; ++c)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int dy = (16 / K::PW) * (2 * c + hh);
          const bool ok = x < WIN && y0 + dy < WIN;
          const uint32_t av = ok ? vb + dy * K::RUN * 16 : zaddr;
          vr[c][0][hh] = lds_rd64_tr<0>(av);
          vr[c][1][hh] = lds_rd64_tr<8>(av);  // zero16 + 8 is zero as well
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
    __builtin_amdgcn_s_barrier();  // every wave holds its fragments: the slab is free
    asm volatile("" ::: "memory");
    int nb = cb, nwh = cwh, nww = cww + 1;
    if (nww == g.nWw) {
      nww = 0;
      if (++nwh == g.nWh) {
        nwh = 0;
        ++nb;
      }
    }
#if HVK_RING_PROBE == 2  // tools/probe: math only (the first slab is reused, no DMA)
    (void)nb;
#else
    if (w + 1 < w1) issue(nb, nwh, nww);
#endif

    const int b = cb, wh = cwh, ww = cww;
    cb = nb;
    cwh = nwh;
    cww = nww;
    const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
#if HVK_RING_PROBE == 1  // tools/probe: memory only (same DMA and stores, no math)
#pragma unroll
    for (int qi = 0; qi < K::NT; ++qi) {
      const int tq = grid_token<WIN, K::PW>(16 * qi + li);
      if (tq >= 0) {
        uint4 v = qf[qi];
        v.x ^= kf[qi].x ^ vt[0][0].x;
        hvk_bf16* dst = a.out + (size_t)window_token_row(g, b, wh, ww, WIN, tq) * C + h * 32 + 8 * gq;
        ring_store(dst, v);
      }
    }
    continue;
#endif
    float rn;
    if (!a.qk_normed) {  // qk_normed: q^ * scale * log2e and k^ arrive from the qkv GEMM's epilogue
#pragma unroll
      for (int i = 0; i < K::NT; ++i) {
        qf[i] = l2_normalize(qf[i], rn, sc2);  // q^ * scale * log2e: the MFMA applies the scale
        kf[i] = l2_normalize(kf[i], rn);
      }
    }
#pragma unroll
    for (int qi = 0; qi < K::NT; ++qi) {
      const int pq = 16 * qi + li;
      const int tq = grid_token<WIN, K::PW>(pq);
      // S^T of query tile qi (shifted by the head bound) with the shift-region mask
      auto scores = [&](hvk_f32x4 (&s)[K::NT]) {
        // one query tile live at a time, its bias reads inside the iteration (VGPR budget)
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
        if (edge_r || edge_c) {  // wave-uniform: only the last window row / column is masked
          const int qy = pq / K::PW, qx = pq % K::PW;
          uint32_t mreg = 0;  // keys in another shift region than this query (swinv2.py:357-388)
          if (edge_r) mreg |= (kband ^ (qy >= WIN - g.shift ? 0xFFFFu : 0u)) & 0xFFFFu;
          if (edge_c) mreg |= (kband >> 16) ^ (qx >= WIN - g.shift ? 0xFFFFu : 0u);
#pragma unroll
          for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              s[ki][r] = fmaf((float)((mreg >> (ki * 4 + r)) & 1u), mask2, s[ki][r]);
            }
        }
      };
      // O^T = V^T P^T and the row sums of the (bf16) P over real keys
      hvk_f32x4 o[2], osum;
      auto pv = [&](const hvk_f32x4 (&s)[K::NT]) {
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
      };
      hvk_f32x4 s[K::NT];
      scores(s);
      // fast path: exp2 of the head-bound-shifted logits, no row max.  Padding keys hold
      // finite logits here; their V rows and row-sum weights are zero.
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[ki][r] = __builtin_amdgcn_exp2f(s[ki][r]);
      pv(s);
      float lshift = 0.f;  // the slow path's row max (log2 units), on top of Mh
      if (HVK_RING_ROWMAX_CHECK &&
          __builtin_expect(__builtin_amdgcn_ballot_w64(tq >= 0 && !(osum[0] >= 0x1p-100f)) != 0, 0)) {
        // slow path (rare, wave-uniform): the tile again with the true row max over real keys,
        // one 16-key tile at a time (a second 16-register score array would spill): pass 1
        // takes the max, pass 2 exponentiates against it and accumulates P V and the row sums
        uint32_t mreg = 0;
        if (edge_r || edge_c) {
          const int qy = pq / K::PW, qx = pq % K::PW;
          if (edge_r) mreg |= (kband ^ (qy >= WIN - g.shift ? 0xFFFFu : 0u)) & 0xFFFFu;
          if (edge_c) mreg |= (kband >> 16) ^ (qx >= WIN - g.shift ? 0xFFFFu : 0u);
        }
        // padding key slots of this lane (slot bit ki*4 + r) from a compile-time table indexed
        // by gq: shifts, no compares (per-slot compare masks would be hoisted into SGPRs)
        const uint32_t kpad = (uint32_t)(K::KPAD >> (16 * g4)) & 0xFFFFu;
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
            t[r] = fmaf((float)((kpad >> (ki * 4 + r)) & 1u), -1e30f, t[r]);  // padding: weight 0
          }
          return t;
        };
        float m = -INFINITY;
#pragma unroll
        for (int ki = 0; ki < K::NT; ++ki) {
          const hvk_f32x4 t = tile(ki);
          m = fmaxf(m, fmaxf(fmaxf(t[0], t[1]), fmaxf(t[2], t[3])));
        }
        m = fmaxf(m, __shfl_xor(m, 16));  // the 4 lanes (gq) holding one query's keys
        m = fmaxf(m, __shfl_xor(m, 32));
        lshift = m;
        o[0] = o[1] = osum = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
        for (int c = 0; c < K::NC; ++c) {
          hvk_f32x4 a0 = tile(2 * c), a1 = {0, 0, 0, 0};
#pragma unroll
          for (int r = 0; r < 4; ++r) a0[r] = __builtin_amdgcn_exp2f(a0[r] - m);
          if (2 * c + 1 < K::NT) {  // else the chunk's upper 16 keys do not exist: P = 0
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
        hvk_settle(o[0], o[1], osum);  // read by the store block the slow path branches back to
      }
      if (tq >= 0) {
        const float inv = __builtin_amdgcn_rcpf(osum[0]);
        const uint4 v = make_uint4(hvk_pack2(o[0][0] * inv, o[0][1] * inv),
                                   hvk_pack2(o[0][2] * inv, o[0][3] * inv),
                                   hvk_pack2(o[1][0] * inv, o[1][1] * inv),
                                   hvk_pack2(o[1][2] * inv, o[1][3] * inv));
        const int trow = window_token_row(g, b, wh, ww, WIN, tq);
        ring_store(a.out + (size_t)trow * C + h * 32 + 8 * gq, v);
        if constexpr (LSE) {  // one lane per query: L2 = log2 sum_k exp2(log2e logit)
          if (gq == 0) a.lse[(size_t)trow * g.nH + h] = Mh + lshift + __log2f(osum[0]);
        }
      }
    }
  }
}

template <int WIN, int HG, bool LSE>
int launch_ring_(FwdArgs& a, int B, int H, int W, int C, int nH, int shift, hipStream_t st) {
  using K = RingCfg<WIN, HG>;
  const int per_cu = (160 * 1024) / K::LDS;
  int rc = make_geom(B, H, W, C, nH, WIN, shift, 256 * per_cu * HG, a.g);  // capacity in groups*chunks
  if (rc) return rc;
  // make_geom sized chunks for nH "heads"; here the unit is a head GROUP
  const int ng = nH / HG;
  int chunks = 256 * per_cu / ng / 8 * 8;
  if (chunks < 8) chunks = 8;
  const int need = (a.g.n_windows + 7) / 8 * 8;
  a.g.n_chunks = chunks < need ? chunks : need;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_fwd_ring_kernel<WIN, HG, LSE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    attr = true;
  }
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_FWD, (wmsa_fwd_ring_kernel<WIN, HG, LSE>), dim3(a.g.n_chunks * ng),
                   dim3(64 * HG), K::LDS, st, a);
  HVK_CHECK_LAUNCH("wmsa_fwd_ring");
  return HVK_OK;
}

template <int WIN, int HG>
int launch_ring(FwdArgs& a, int B, int H, int W, int C, int nH, int shift, hipStream_t st) {
  return a.lse ? launch_ring_<WIN, HG, true>(a, B, H, W, C, nH, shift, st)
               : launch_ring_<WIN, HG, false>(a, B, H, W, C, nH, shift, st);
}

template <int WIN>
int ring_win(FwdArgs& a, int B, int H, int W, int C, int nH, int shift, hipStream_t st) {
  // head group: HG heads per workgroup (the group's q/k/v slices are HG*64 contiguous bytes)
  // 4 heads per workgroup from 12 heads up (stages 2-3 of SwinV2-T: 3 % faster there, where
  // each workgroup owns only a few windows), else 3
  if (nH % 4 == 0 && nH >= 12) return launch_ring<WIN, 4>(a, B, H, W, C, nH, shift, st);
  if (nH % 3 == 0) return launch_ring<WIN, 3>(a, B, H, W, C, nH, shift, st);
  if (nH % 4 == 0) return launch_ring<WIN, 4>(a, B, H, W, C, nH, shift, st);
  if (nH % 2 == 0) return launch_ring<WIN, 2>(a, B, H, W, C, nH, shift, st);
  return launch_ring<WIN, 1>(a, B, H, W, C, nH, shift, st);
}

}  // namespace

namespace hvk_wmsa {
int ring_fwd(FwdArgs& a, int B, int H, int W, int C, int nH, int win, int shift, hipStream_t st) {
  switch (win) {
    case 7: return ring_win<7>(a, B, H, W, C, nH, shift, st);
    case 8: return ring_win<8>(a, B, H, W, C, nH, shift, st);
    case 6: return ring_win<6>(a, B, H, W, C, nH, shift, st);
    case 4: return ring_win<4>(a, B, H, W, C, nH, shift, st);
    default: return hvk_set_error(HVK_EUNSUPPORTED, "wmsa ring: window %d", win);
  }
}
}  // namespace hvk_wmsa
