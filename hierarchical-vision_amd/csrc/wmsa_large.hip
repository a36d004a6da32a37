// Shifted-window cosine attention for LARGE windows (12, 16, 24: SwinV2-B 384 / window-24
// configs, the stage-3 clamp to 12, swinv2.py:328-331) on gfx950.
//
// Same semantics and token layout as wmsa.hip (reference: swinv2.py:221-261 + roll/partition
// 399-412 / reverse 420-429), but a window no longer fits one wave's registers
// (N = 144 ... 576 tokens), so one WORKGROUP owns one (window, head):
//   forward   K^ and V of the window are staged once in LDS; every wave streams its query
//             tiles against all keys in 32-key chunks with an online softmax (flash form);
//   backward  phase 1 (query on the lane, K^ / V in LDS): row max / sum / delta, then dS,
//             dQ, the CPB-bias and logit-scale gradients; phase 2 (key on the lane, Q^ / dO
//             restaged in the same LDS): dK, dV.  Nothing is saved by the forward.
// The CPB table stays compact ((2w-1)^2 floats per head, log2e-scaled) and is looked up per
// score element: index = bq(query) - bk(key), bq = (qh+w-1)(2w-1) + qw+w-1, bk = kh(2w-1)+kw.
// The bias gradient is binned with LDS float atomics and flushed once per workgroup.
//
// LDS images are [rows][32] bf16 in "fragment-major" order: the 16-B unit (row, u) of a
// 16-row tile sits at slot 16u + (row%16 ^ 12*(u&1)), so the natural MFMA operand read
// (ds_read_b128, lane = row%16 + 16u) and the transposed read (ds_read_b64_tr_b16) are both
// bank-conflict free (checked with the LDS bank model of MI355X_MICROARCH.md).
#include "wmsa_common.h"

// experiment builds (not the product): 1 no CPB-gradient accumulation, 3 no edge masks,
// 4 no phase 2, 5 no phase-1 loop B, 6 no phase-1 loop A
#ifndef HVK_LARGE_PROBE
#define HVK_LARGE_PROBE 0
#endif
#ifndef HVK_LARGE_FWAVES24  // forward waves per workgroup at w24 (9 / 12 / 16: 19.3 / 18.3 / 16.9 ms per SwinV2-B 384 step)
#define HVK_LARGE_FWAVES24 16
#endif
#ifndef HVK_LARGE_BINS
#define HVK_LARGE_BINS 1
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
  static constexpr int WAVES = WIN == 16 ? 8 : (WIN == 24 ? HVK_LARGE_FWAVES24 : 9);
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int QB = (NT % (2 * WAVES) == 0) ? 2 : 1;  // query tiles per forward pass
  static constexpr int IMG = ROWS * 64;        // bytes per image
  static_assert(NT % WAVES == 0 || QB == 1, "tile split");
  static_assert(N == 16 * NT, "strided query tiles cover the window exactly");
  // backward: BWAVES waves, each with a private copy of the CPB-gradient bins (plain LDS
  // read-add-write, no float atomics) when HVK_LARGE_BINS; 8 waves at w24 so that the 8
  // copies fit beside the two images
  static constexpr int BWAVES = HVK_LARGE_BINS ? 8 : WAVES;
  static constexpr int BTHREADS = 64 * BWAVES;
  static constexpr int RRP = (RR + 3) / 4 * 4;  // bins per copy (16-B aligned)
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

template <int WIN>
struct PosInfo {  // window-local geometry of one token position
  int b;          // bias-index base: bq for a query, bk for a key
  bool r, c;      // in the last shift band of its row / column
};
template <int WIN>
__device__ __forceinline__ PosInfo<WIN> query_info(int pos, int lim) {
  const int ph = pos / WIN, pw = pos - ph * WIN;
  return {(ph + WIN - 1) * LCfg<WIN>::R + pw + WIN - 1, ph >= lim, pw >= lim};
}
template <int WIN>
__device__ __forceinline__ PosInfo<WIN> key_info(int pos, int lim) {
  const int ph = pos / WIN, pw = pos - ph * WIN;
  return {ph * LCfg<WIN>::R + pw, ph >= lim, pw >= lim};
}
// ------------------------------------------------------------------------------ forward
// Per query tile (query on the lane), keys in 32-key chunks: S' = K^ (scale log2e Q^)^T +
// (log2e bias - M_h) with the mirrored bias table as the MFMA C operand, M_h = scale log2e +
// max bias the head bound of every logit (as the ring kernel, wmsa_ring.hip), so the fast path
// exponentiates S' directly -- no running max, no rescaling -- and checks the row sums at the
// end: a tile where any row sum fell below 2^-100 (a row far below the head bound, scale ~100)
// is recomputed with the true running max (the reference's softmax, swinv2.py:256).
template <int WIN, bool LSE>
__global__ __launch_bounds__(LCfg<WIN>::THREADS, 1) void wmsa_fwd_large_kernel(FwdArgs a) {
  using K = LCfg<WIN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int w, h;
  hvk_decode_chunk_head(blockIdx.x, g.nH, w, h);
  if (w >= g.n_windows) return;
  char* kimg = smem;
  char* vimg = smem + K::IMG;
  float* mtab = reinterpret_cast<float*>(smem + 2 * K::IMG);
  float* red = mtab + K::TABM;  // [WAVES] max-bias partials
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * C;
  const int per_img = g.nWh * g.nWw;
  const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
  const float sc2 = a.scale[h] * HVK_LOG2E;

  const float* bsrc = a.bias + (size_t)h * K::RR;
  float mb = -INFINITY;
  for (int e = threadIdx.x; e < K::RR; e += K::THREADS) mb = fmaxf(mb, bsrc[e]);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) mb = fmaxf(mb, __shfl_xor(mb, m));
  if (lane == 0) red[wave] = mb;
  // stage k^ (natural fragments) and v (head_dim permuted for 16-B output stores, as in
  // wmsa.hip: col 16dt + 4g + r <-> d = 8g + 4dt + r)
  for (int t = wave; t < 2 * K::NC; t += K::WAVES) {
    const int pos = 16 * t + li;
    uint4 kv = make_uint4(0, 0, 0, 0), vv = kv;
    if (pos < K::N) {
      const hvk_bf16* p = a.qkv + (size_t)window_token_row(g, b, wh, ww, WIN, pos) * C3 + h * 32 + 8 * gq;
      kv = hvk_ld16(p + C);
      vv = hvk_ld16(p + 2 * C);
    }
    float rn;
    kv = l2_normalize(kv, rn);  // a zero (padding) row stays zero
    *reinterpret_cast<uint4*>(kimg + fm16(pos, gq)) = kv;
    *reinterpret_cast<uint2*>(vimg + fm8(pos, gq)) = make_uint2(vv.x, vv.y);
    *reinterpret_cast<uint2*>(vimg + fm8(pos, 4 + gq)) = make_uint2(vv.z, vv.w);
  }
  __syncthreads();
  float Mh = red[0];
#pragma unroll
  for (int i = 1; i < K::WAVES; ++i) Mh = fmaxf(Mh, red[i]);
  Mh = Mh * HVK_LOG2E + sc2;
  for (int e = threadIdx.x; e < K::TABM; e += K::THREADS) {
    const int i = K::RR - 1 - e;
    mtab[e] = i >= 0 ? bsrc[i] * HVK_LOG2E - Mh : 0.f;
  }
  __syncthreads();

  const float mask2 = -100.f * HVK_LOG2E;
  const int lim = WIN - g.shift;
  const bool edge = g.shift && (wh == g.nWh - 1 || ww == g.nWw - 1);
  const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;

  for (int t0 = wave * K::QB; t0 < K::NT; t0 += K::WAVES * K::QB) {
    uint4 qf[K::QB];
    int qrow[K::QB];
    PosInfo<WIN> qi[K::QB];
    hvk_f32x4 o[K::QB][2];
    float l[K::QB];
#pragma unroll
    for (int j = 0; j < K::QB; ++j) {
      const int pos = 16 * (t0 + j) + li;
      qrow[j] = window_token_row(g, b, wh, ww, WIN, pos);
      qf[j] = hvk_ld16(a.qkv + (size_t)qrow[j] * C3 + h * 32 + 8 * gq);
      float rn;
      qf[j] = l2_normalize(qf[j], rn, sc2);  // q^ * scale * log2e
      qi[j] = query_info<WIN>(pos, lim);
    }
    // S' of (key chunk c, half t, query tile j), masked; padding keys -inf
    auto scores = [&](int c, int t, int j, const uint4& kf) {
      const int kp = 32 * c + 16 * t + 4 * gq;  // this lane's 4 keys kp .. kp + 3 (one row)
      const int ky = kp / WIN, kx = kp - ky * WIN;
      const float* tp = mtab + (K::RR - 1 - qi[j].b + ky * K::R + kx);
      hvk_f32x4 s = hvk_mfma16(kf, qf[j], hvk_f32x4{tp[0], tp[1], tp[2], tp[3]});
      hvk_settle(s);  // the unmasked path branches over the mask code to its readers
      if (edge) {  // wave-uniform: last window row / column of a shifted block only
        const bool rmis = edge_r && ((ky >= lim) != qi[j].r);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool cmis = edge_c && ((kx + r >= lim) != qi[j].c);
          s[r] += (rmis || cmis) ? mask2 : 0.f;
        }
      }
      if (K::N % 32 != 0 && c == K::NC - 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kp + r >= K::N) s[r] = -INFINITY;
      }
      return s;
    };
#pragma unroll
    for (int j = 0; j < K::QB; ++j) {
      l[j] = 0.f;
      o[j][0] = o[j][1] = hvk_f32x4{0, 0, 0, 0};
    }
#pragma unroll 3
    for (int c = 0; c < K::NC; ++c) {
      const uint4 kf0 = lds16(kimg, fm16(32 * c + li, gq));
      const uint4 kf1 = lds16(kimg, fm16(32 * c + 16 + li, gq));
      const uint4 vt0 = tr_frag(vimg, c, 0, li, gq), vt1 = tr_frag(vimg, c, 1, li, gq);
#pragma unroll
      for (int j = 0; j < K::QB; ++j) {
        hvk_f32x4 s0 = scores(c, 0, j, kf0), s1 = scores(c, 1, j, kf1);
        float p[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = __builtin_amdgcn_exp2f(s0[r]);
          p[4 + r] = __builtin_amdgcn_exp2f(s1[r]);
        }
        l[j] += ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
        const uint4 pf = make_uint4(hvk_pack2(p[0], p[1]), hvk_pack2(p[2], p[3]),
                                    hvk_pack2(p[4], p[5]), hvk_pack2(p[6], p[7]));
        o[j][0] = hvk_mfma16(vt0, pf, o[j][0]);
        o[j][1] = hvk_mfma16(vt1, pf, o[j][1]);
      }
    }
#pragma unroll
    for (int j = 0; j < K::QB; ++j) {
      l[j] = hvk_group4_sum(l[j]);
      float lshift = 0.f;  // the slow path's row max, on top of M_h
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(l[j] >= 0x1p-100f)) != 0, 0)) {
        // slow path (rare, wave-uniform): this tile again with the true running max
        float m = -INFINITY;
        l[j] = 0.f;
        o[j][0] = o[j][1] = hvk_f32x4{0, 0, 0, 0};
#pragma unroll 1
        for (int c = 0; c < K::NC; ++c) {
          const uint4 kf0 = lds16(kimg, fm16(32 * c + li, gq));
          const uint4 kf1 = lds16(kimg, fm16(32 * c + 16 + li, gq));
          const uint4 vt0 = tr_frag(vimg, c, 0, li, gq), vt1 = tr_frag(vimg, c, 1, li, gq);
          hvk_f32x4 s0 = scores(c, 0, j, kf0), s1 = scores(c, 1, j, kf1);
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
          l[j] = l[j] * alpha + ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
          o[j][0] *= alpha;
          o[j][1] *= alpha;
          const uint4 pf = make_uint4(hvk_pack2(p[0], p[1]), hvk_pack2(p[2], p[3]),
                                      hvk_pack2(p[4], p[5]), hvk_pack2(p[6], p[7]));
          o[j][0] = hvk_mfma16(vt0, pf, o[j][0]);
          o[j][1] = hvk_mfma16(vt1, pf, o[j][1]);
        }
        l[j] = hvk_group4_sum(l[j]);
        lshift = m;
        hvk_settle(o[j][0], o[j][1]);  // read by the store block this path branches back to
      }
      // LSE: the query's log2 row constant L2 = M_h + row max + log2(row sum) for the backward
      if (LSE && gq == 0) a.lse[(size_t)qrow[j] * g.nH + h] = Mh + lshift + __log2f(l[j]);
      const float inv = __builtin_amdgcn_rcpf(l[j]);
      const uint4 pk = make_uint4(hvk_pack2(o[j][0][0] * inv, o[j][0][1] * inv),
                                  hvk_pack2(o[j][0][2] * inv, o[j][0][3] * inv),
                                  hvk_pack2(o[j][1][0] * inv, o[j][1][1] * inv),
                                  hvk_pack2(o[j][1][2] * inv, o[j][1][3] * inv));
      hvk_st16(a.out + (size_t)qrow[j] * C + h * 32 + 8 * gq, pk);
    }
  }
}

// ----------------------------------------------------------------------------- backward
// Normalize-backward of a head row: x^ = x * rn; dx = (dx^ - x^ (x^ . dx^)) * rn, with the
// lane's 8 values of dx^ (times `post`) at d = 16dt + 4g + r (accumulator order).  x is
// re-read from global (L2) in that order.  Every lane must call it (group reduction inside); `x` must point at a real row; only the
// store (and the column-sum accumulation into acc, when non-null) is skipped when dst is null.

__device__ __forceinline__ void normalize_bwd_store(const hvk_bf16* x, float rn, const hvk_f32x4 dxh[2],
                                                    hvk_bf16* dst, float post, int g,
                                                    float (*acc)[4]) {
  float xh[2][4], dot = 0.f;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const uint2 v = *reinterpret_cast<const uint2*>(x + 16 * dt + 4 * g);
    xh[dt][0] = hvk_lo(v.x) * rn; xh[dt][1] = hvk_hi(v.x) * rn;
    xh[dt][2] = hvk_lo(v.y) * rn; xh[dt][3] = hvk_hi(v.y) * rn;
#pragma unroll
    for (int r = 0; r < 4; ++r) dot += xh[dt][r] * dxh[dt][r] * post;
  }
  dot = hvk_group4_sum(dot);
  if (rn >= 1e12f) dot = 0.f;  // ||x|| <= eps: x / eps, no projection term
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (dxh[dt][r] * post - xh[dt][r] * dot) * rn;
    if (dst) {
      hvk_st8(dst + 16 * dt + 4 * g, make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3])));
      if (acc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[dt][r] += v[r];
      }
    }
  }
}

template <int WIN>
constexpr size_t bwd_large_lds() {
  using K = LCfg<WIN>;
  const size_t bins = HVK_LARGE_BINS ? (size_t)K::BWAVES * K::RRP : (size_t)K::RR;
  return 2 * (size_t)K::IMG + (size_t)K::TABM * 4 + bins * 4 + 2 * (size_t)K::ROWS * 4 + 64;
}

// Logits relative to the head bound, as the forward: S' = sc2 cos + log2e bias - M_h from one
// MFMA with the mirrored CPB table as its C operand (4 ascending floats for the lane's 4
// consecutive keys in phase 1; 4 descending for its 4 consecutive queries in phase 2), plus
// the -100 mask on edge windows (wave-uniform branch).  Phase 1 loop A exponentiates S'
// directly (S' <= 0) and falls back to a running row max only for a tile whose row sum
// underflows; the row constants kept for loop B and phase 2 are relative to M_h.
template <int WIN, bool LSE>
__global__ __launch_bounds__(LCfg<WIN>::BTHREADS, 1) void wmsa_bwd_large_kernel(BwdArgs a) {
  using K = LCfg<WIN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int w, h;
  hvk_decode_chunk_head(blockIdx.x, g.nH, w, h);
  if (w >= g.n_windows) return;
  char* img0 = smem;
  char* img1 = smem + K::IMG;
  float* mtab = reinterpret_cast<float*>(smem + 2 * K::IMG);  // [TABM] mirrored, - M_h
  float* dtab = mtab + K::TABM;  // [BWAVES][RRP] private bins (HVK_LARGE_BINS) or [RR] shared
  constexpr int NBIN = HVK_LARGE_BINS ? K::BWAVES * K::RRP : K::RR;
  float* lse_s = dtab + NBIN;    // [ROWS] row constant relative to M_h (+inf: padding rows)
  float* dlt_s = lse_s + K::ROWS;  // [ROWS] delta = rowsum(P * dP)
  float* red = dlt_s + K::ROWS;  // [16] max-bias partials
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * C;
  const int per_img = g.nWh * g.nWw;
  const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
  const float scale = a.scale[h];
  const float sc2 = scale * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  const int lim = WIN - g.shift;
  const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
  const bool edge = HVK_LARGE_PROBE == 3 ? false : (edge_r || edge_c);  // probe 3: no mask (not exact)

  const float* bsrc = a.bias + (size_t)h * K::RR;
  float mb = -INFINITY;
  for (int e = threadIdx.x; e < K::RR; e += K::BTHREADS) mb = fmaxf(mb, bsrc[e]);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) mb = fmaxf(mb, __shfl_xor(mb, m));
  if (lane == 0) red[wave] = mb;
  for (int e = threadIdx.x; e < NBIN; e += K::BTHREADS) dtab[e] = 0.f;
  for (int e = threadIdx.x; e < K::ROWS; e += K::BTHREADS) {
    lse_s[e] = INFINITY;
    dlt_s[e] = 0.f;
  }
  // phase-1 images: k^ and v, natural head_dim order
  for (int t = wave; t < 2 * K::NC; t += K::BWAVES) {
    const int pos = 16 * t + li;
    uint4 kv = make_uint4(0, 0, 0, 0), vv = kv;
    if (pos < K::N) {
      const hvk_bf16* p = a.qkv + (size_t)window_token_row(g, b, wh, ww, WIN, pos) * C3 + h * 32 + 8 * gq;
      kv = hvk_ld16(p + C);
      vv = hvk_ld16(p + 2 * C);
    }
    float rn;
    kv = l2_normalize(kv, rn);
    *reinterpret_cast<uint4*>(img0 + fm16(pos, gq)) = kv;
    *reinterpret_cast<uint4*>(img1 + fm16(pos, gq)) = vv;
  }
  __syncthreads();
  float Mh = red[0];
#pragma unroll
  for (int i = 1; i < K::BWAVES; ++i) Mh = fmaxf(Mh, red[i]);
  Mh = Mh * HVK_LOG2E + sc2;
  for (int e = threadIdx.x; e < K::TABM; e += K::BTHREADS) {
    const int i = K::RR - 1 - e;
    mtab[e] = i >= 0 ? bsrc[i] * HVK_LOG2E - Mh : 0.f;
  }
  __syncthreads();

  // ---------------- phase 1: query tiles (query on the lane)
  float dscale = 0.f;
  float dqb[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int qt = wave; qt < K::NT; qt += K::BWAVES) {
    // query tile qt = positions qt + NT*li (N = 16 NT for w 12/16/24): the 16 queries of a tile
    // lie >= one window row apart, so the CPB-gradient bins of one read-add-write batch are
    // distinct across the lanes (loop B)
    const int pos = qt + K::NT * li;
    const int qrow = window_token_row(g, b, wh, ww, WIN, pos);
    const hvk_bf16* qp = a.qkv + (size_t)qrow * C3 + h * 32;
    const uint4 qraw = hvk_ld16(qp + 8 * gq);
    const uint4 dof = hvk_ld16(a.dout + (size_t)qrow * C + h * 32 + 8 * gq);
    float rnq;
    const uint4 qs = l2_normalize(qraw, rnq, sc2);
    const PosInfo<WIN> qi = query_info<WIN>(pos, lim);
    const float* tq = mtab + (K::RR - 1 - qi.b);  // + kb(key) + r

    // S' (masked; padding keys -inf) and dP - 0 of chunk c, half t; c4 = the bias C operand
    auto tile = [&](int c, int t, hvk_f32x4& s, hvk_f32x4& d, hvk_f32x4& c4) {
      const int kt = 2 * c + t, kp = 16 * kt + 4 * gq;
      const int ky = kp / WIN, kx = kp - ky * WIN;
      const float* tp = tq + ky * K::R + kx;
      c4 = hvk_f32x4{tp[0], tp[1], tp[2], tp[3]};
      s = hvk_mfma16(lds16(img0, fm16(16 * kt + li, gq)), qs, c4);
      d = hvk_mfma16(lds16(img1, fm16(16 * kt + li, gq)), dof, hvk_f32x4{0, 0, 0, 0});
      hvk_settle(s, d);  // the unmasked path branches over the mask code to their readers
      if (edge) {  // wave-uniform; selects, not branches, per element
        const bool rmis = edge_r && ((ky >= lim) != qi.r);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool cmis = edge_c && ((kx + r >= lim) != qi.c);
          s[r] += (rmis || cmis) ? mask2 : 0.f;
        }
      }
      if (K::N % 32 != 0 && c == K::NC - 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kp + r >= K::N) s[r] = -INFINITY;
      }
    };

    // LSE: the forward's row constant and delta_O = dO . O from its output; loop B then
    // measures how far its dS row sums miss zero and corrects delta, dQ and the logit-scale
    // gradient exactly (the CPB gradient keeps the small remainder)
    float lse_in = 0.f, dlt_o = 0.f;
    if (LSE) {
      lse_in = a.lse[(size_t)qrow * g.nH + h] - Mh;
      float fd[8], fo[8];
      hvk_unpack8(dof, fd);
      hvk_unpack8(hvk_ld16(a.out + (size_t)qrow * C + h * 32 + 8 * gq), fo);
#pragma unroll
      for (int e = 0; e < 8; ++e) dlt_o = fmaf(fd[e], fo[e], dlt_o);
      dlt_o = hvk_group4_sum(dlt_o);
    }
    // loop A: row sum and delta against the head bound
    float l = HVK_LARGE_PROBE == 6 ? 1.f : 0.f, dacc = 0.f, m = 0.f;
#pragma unroll 1
    for (int c = 0; c < (HVK_LARGE_PROBE == 6 || LSE ? 0 : K::NC); ++c) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        hvk_f32x4 s, d, c4;
        tile(c, t, s, d, c4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(s[r]);
          l += p;
          dacc = fmaf(p, d[r], dacc);
        }
      }
    }
    l = hvk_group4_sum(l);
    dacc = hvk_group4_sum(dacc);
    if (!LSE && __builtin_expect(__builtin_amdgcn_ballot_w64(!(l >= 0x1p-100f)) != 0, 0)) {
      // slow path (rare, wave-uniform): row max, sum and delta with a running max
      m = -INFINITY;
      l = 0.f;
      dacc = 0.f;
#pragma unroll 1
      for (int c = 0; c < K::NC; ++c) {
        hvk_f32x4 s[2], d[2], c4;
        tile(c, 0, s[0], d[0], c4);
        tile(c, 1, s[1], d[1], c4);
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
    const float lse = LSE ? lse_in : m + __log2f(l);  // relative to M_h
    const float delta = LSE ? dlt_o : dacc / l;

    // loop B: dS, dQ^, bias / scale gradients
    hvk_f32x4 dq[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, pk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    float lk = 0.f, pp = 0.f, ps = 0.f;  // LSE: row sums of dS, P and P * sc2 cos
#pragma unroll 1
    for (int c = 0; c < (HVK_LARGE_PROBE == 5 ? 0 : K::NC); ++c) {
      float ds[2][4], pl[2][4];
      int bidx[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        hvk_f32x4 s, d, c4;
        tile(c, t, s, d, c4);
        const int kp = 32 * c + 16 * t + 4 * gq, ky = kp / WIN, kx = kp - ky * WIN;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool kvalid = kp + r < K::N;
          const float p = __builtin_amdgcn_exp2f(s[r] - lse);  // padding keys: exp2(-inf) = 0
          const float dsv = p * (d[r] - delta);
          ds[t][r] = dsv;
          bidx[t][r] = qi.b - (ky * K::R + kx + r);
          if (kvalid) dscale += dsv * (s[r] - c4[r]);  // sc2 * cos (the mask only where p ~ 0)
          if (LSE) {
            pl[t][r] = p;
            lk += dsv;
            pp += p;
            if (kvalid) ps = fmaf(p, s[r] - c4[r], ps);
          }
        }
      }
      // CPB-table gradient: this wave's own bins (plain LDS read-add-write, no float atomics).
      // A batch of read-add-writes is exact when no two of its (lane, element) pairs share a
      // bin: with the strided query tiles that holds for a whole 32-key chunk at w24, for each
      // 16-key half at w16, per element at w12 (tools/large_bins_check.py); LDS operations of a
      // wave complete in order, and the compiler fences keep hipcc from merging the reads of
      // one batch ahead of another's writes (exact per lane, but it loses other lanes' updates)
      if (HVK_LARGE_PROBE >= 1) {
      } else if (HVK_LARGE_BINS) {
        float* pb = dtab + wave * K::RRP;
        constexpr int BATCH = WIN == 24 ? 8 : (WIN == 16 ? 4 : 1);
#pragma unroll
        for (int b0 = 0; b0 < 8; b0 += BATCH) {
          float v[BATCH];
          asm volatile("" ::: "memory");
#pragma unroll
          for (int e = 0; e < BATCH; ++e) {
            const int t = (b0 + e) >> 2, r = (b0 + e) & 3;
            const bool ok = 32 * c + 16 * t + 4 * gq + r < K::N;
            v[e] = ok ? pb[bidx[t][r]] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < BATCH; ++e) {
            const int t = (b0 + e) >> 2, r = (b0 + e) & 3;
            const bool ok = 32 * c + 16 * t + 4 * gq + r < K::N;
            if (ok) pb[bidx[t][r]] = v[e] + ds[t][r];
          }
          asm volatile("" ::: "memory");
        }
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (32 * c + 16 * t + 4 * gq + r < K::N)
              atomicAdd(&dtab[bidx[t][r]], ds[t][r]);  // LDS float atomic (ds_add_f32)
      }
      const uint4 bf = make_uint4(hvk_pack2(scale * ds[0][0], scale * ds[0][1]),
                                  hvk_pack2(scale * ds[0][2], scale * ds[0][3]),
                                  hvk_pack2(scale * ds[1][0], scale * ds[1][1]),
                                  hvk_pack2(scale * ds[1][2], scale * ds[1][3]));
      const uint4 kf0 = tr_frag(img0, c, 0, li, gq), kf1 = tr_frag(img0, c, 1, li, gq);
      dq[0] = hvk_mfma16(kf0, bf, dq[0]);
      dq[1] = hvk_mfma16(kf1, bf, dq[1]);
      if (LSE) {  // sum_k P k^ of this query tile, for the dQ correction
        const uint4 pf = make_uint4(hvk_pack2(pl[0][0], pl[0][1]), hvk_pack2(pl[0][2], pl[0][3]),
                                    hvk_pack2(pl[1][0], pl[1][1]), hvk_pack2(pl[1][2], pl[1][3]));
        pk[0] = hvk_mfma16(kf0, pf, pk[0]);
        pk[1] = hvk_mfma16(kf1, pf, pk[1]);
      }
    }
    float dlt = delta;
    if (LSE) {
      // dS = P (dP - delta_O) misses the exact P (dP - sum P dP / sum P) by P corr per row,
      // corr = rowsum(dS) / rowsum(P): take it out of dQ (scale corr sum_k P k^) and of the
      // logit-scale gradient, and hand phase 2 the exact delta
      const float corr = hvk_group4_sum(lk) / hvk_group4_sum(pp);
      const float psq = hvk_group4_sum(ps);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) dq[dt][r] = fmaf(-scale * corr, pk[dt][r], dq[dt][r]);
      if (gq == 0) dscale = fmaf(-corr, psq, dscale);
      dlt = delta + corr;
    }
    if (gq == 0) {
      lse_s[pos] = lse;
      dlt_s[pos] = dlt;
    }
    normalize_bwd_store(qp, rnq, dq, a.dqkv + (size_t)qrow * C3 + h * 32, 1.f, gq, dqb);
  }
  __syncthreads();

  // phase-2 images: q^ * scale * log2e (exactly the forward's operand) and dO
  for (int t = wave; t < 2 * K::NC; t += K::BWAVES) {
    const int pos = 16 * t + li;
    uint4 qv = make_uint4(0, 0, 0, 0), dv = qv;
    if (pos < K::N) {
      const int row = window_token_row(g, b, wh, ww, WIN, pos);
      qv = hvk_ld16(a.qkv + (size_t)row * C3 + h * 32 + 8 * gq);
      dv = hvk_ld16(a.dout + (size_t)row * C + h * 32 + 8 * gq);
    }
    float rn;
    qv = l2_normalize(qv, rn, sc2);
    *reinterpret_cast<uint4*>(img0 + fm16(pos, gq)) = qv;
    *reinterpret_cast<uint4*>(img1 + fm16(pos, gq)) = dv;
  }
  __syncthreads();

  // ---------------- phase 2: key tiles (key on the lane)
  for (int kt = wave; kt < (HVK_LARGE_PROBE == 4 ? 0 : K::NT); kt += K::BWAVES) {
    const int pos = 16 * kt + li;
    const int krow = window_token_row(g, b, wh, ww, WIN, pos);
    const hvk_bf16* kp = a.qkv + (size_t)krow * C3 + h * 32 + C;
    const uint4 kraw = hvk_ld16(kp + 8 * gq);
    const uint4 vf = hvk_ld16(kp + C + 8 * gq);
    float rnk;
    const uint4 kh = l2_normalize(kraw, rnk);
    const PosInfo<WIN> ki = key_info<WIN>(pos, lim);
    const float* tk = mtab + (K::RR - 1 + ki.b);  // - qb(query)
    hvk_f32x4 dk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, dv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll 1
    for (int c = 0; c < K::NC; ++c) {
      float p[2][4], ds[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int qt = 2 * c + t, q0 = 16 * qt + 4 * gq;  // this lane's queries q0 .. q0 + 3
        if (K::NT % 2 == 1 && qt >= K::NT) {  // w12's padding half chunk: no queries
#pragma unroll
          for (int r = 0; r < 4; ++r) p[t][r] = ds[t][r] = 0.f;
          continue;
        }
        const int qy = q0 / WIN, qx = q0 - qy * WIN;
        const float* tp = tk - ((qy + WIN - 1) * K::R + qx + WIN - 1);  // entries tp[-r]
        hvk_f32x4 s = hvk_mfma16(lds16(img0, fm16(16 * qt + li, gq)), kh,
                                 hvk_f32x4{tp[0], tp[-1], tp[-2], tp[-3]});
        const hvk_f32x4 d = hvk_mfma16(lds16(img1, fm16(16 * qt + li, gq)), vf, hvk_f32x4{0, 0, 0, 0});
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + q0);
        const float4 d4 = *reinterpret_cast<const float4*>(dlt_s + q0);
        const float lr[4] = {l4.x, l4.y, l4.z, l4.w}, dr[4] = {d4.x, d4.y, d4.z, d4.w};
        hvk_settle(s);
        if (edge) {  // wave-uniform; selects, not branches, per element
          const bool rmis = edge_r && (ki.r != (qy >= lim));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool cmis = edge_c && (ki.c != (qx + r >= lim));
            s[r] += (rmis || cmis) ? mask2 : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[t][r] = __builtin_amdgcn_exp2f(s[r] - lr[r]);  // padding query: lse = +inf -> 0
          ds[t][r] = p[t][r] * (d[r] - dr[r]);
        }
      }
      const uint4 pf = make_uint4(hvk_pack2(p[0][0], p[0][1]), hvk_pack2(p[0][2], p[0][3]),
                                  hvk_pack2(p[1][0], p[1][1]), hvk_pack2(p[1][2], p[1][3]));
      const uint4 dsf = make_uint4(hvk_pack2(ds[0][0], ds[0][1]), hvk_pack2(ds[0][2], ds[0][3]),
                                   hvk_pack2(ds[1][0], ds[1][1]), hvk_pack2(ds[1][2], ds[1][3]));
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        dv[dt] = hvk_mfma16(tr_frag(img1, c, dt, li, gq), pf, dv[dt]);
        dk[dt] = hvk_mfma16(tr_frag(img0, c, dt, li, gq), dsf, dk[dt]);
      }
    }
    // dk^ = sum_q scale dS q^ = sum_q dS (q^ scale log2e) / log2e
    hvk_bf16* dst = a.dqkv + (size_t)krow * C3 + h * 32;
    normalize_bwd_store(kp, rnk, dk, dst + C, 1.f / HVK_LOG2E, gq, nullptr);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
      hvk_st8(dst + 2 * C + 16 * dt + 4 * gq,
              make_uint2(hvk_pack2(dv[dt][0], dv[dt][1]), hvk_pack2(dv[dt][2], dv[dt][3])));
  }
  __syncthreads();

  float* gbias = a.dbias_acc + (size_t)h * K::RR;
  for (int e = threadIdx.x; e < K::RR; e += K::BTHREADS) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < (HVK_LARGE_BINS ? K::BWAVES : 1); ++c) v += dtab[c * K::RRP + e];
    atomicAdd(gbias + e, v);
  }
  dscale = hvk_wave_sum(dscale);
  if (lane == 0) atomicAdd(a.dscale_acc + h, dscale / sc2);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = hvk_row16_sum(dqb[dt][r]);
      if (li == 0) atomicAdd(a.dqb_acc + h * 32 + 16 * dt + 4 * gq + r, v);
    }
}

// copy the bins out, write dscale / dq_bias, leave the workspace zero
template <int WIN>
__global__ __launch_bounds__(256) void wmsa_finalize_large_kernel(BwdArgs a, float* __restrict__ dtab,
                                                                  float* __restrict__ dscale,
                                                                  float* __restrict__ dqb) {
  using K = LCfg<WIN>;
  const int h = blockIdx.x;
  float* acc = a.dbias_acc + (size_t)h * K::RR;
  for (int i = threadIdx.x; i < K::RR; i += blockDim.x) {
    dtab[(size_t)h * K::RR + i] = acc[i];
    acc[i] = 0.f;
  }
  finalize_scale_qb(a.dscale_acc, a.dqb_acc, dscale, dqb, h);
}

template <int WIN, bool LSE>
int launch_fwd_large_(const FwdArgs& a, hipStream_t st) {
  using K = LCfg<WIN>;
  const size_t lds = 2 * (size_t)K::IMG + ((size_t)K::TABM + K::WAVES) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_fwd_large_kernel<WIN, LSE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int padded = (a.g.n_windows + 7) / 8 * 8;
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_FWD, (wmsa_fwd_large_kernel<WIN, LSE>), dim3(padded * a.g.nH),
                   dim3(K::THREADS), lds, st, a);
  HVK_CHECK_LAUNCH("wmsa_fwd_large");
  return HVK_OK;
}
template <int WIN>
int launch_fwd_large(const FwdArgs& a, hipStream_t st) {
  return a.lse ? launch_fwd_large_<WIN, true>(a, st) : launch_fwd_large_<WIN, false>(a, st);
}

template <int WIN, bool LSE>
int launch_bwd_large_(const BwdArgs& a, hipStream_t st) {
  using K = LCfg<WIN>;
  const size_t lds = bwd_large_lds<WIN>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_large_kernel<WIN, LSE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int padded = (a.g.n_windows + 7) / 8 * 8;
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, (wmsa_bwd_large_kernel<WIN, LSE>), dim3(padded * a.g.nH),
                   dim3(K::BTHREADS), lds, st, a);
  return HVK_OK;
}

template <int WIN>
int launch_bwd_large(const BwdArgs& a, float* dtab, float* dscale, float* dqb, hipStream_t st) {
  if (a.lse) launch_bwd_large_<WIN, true>(a, st);
  else launch_bwd_large_<WIN, false>(a, st);
  HVK_CHECK_LAUNCH("wmsa_bwd_large");
  hipLaunchKernelGGL(wmsa_finalize_large_kernel<WIN>, dim3(a.g.nH), dim3(256), 0, st, a, dtab, dscale, dqb);
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

size_t large_acc_floats(int num_heads, int win) {
  const size_t r = 2 * (size_t)win - 1;
  return (size_t)num_heads * r * r;
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
