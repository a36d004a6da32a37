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

// experiment builds (not the product): 1 no CPB-gradient LDS atomics, 2 also no CPB gathers
#ifndef HVK_LARGE_PROBE
#define HVK_LARGE_PROBE 0
#endif
#ifndef HVK_LARGE_BINS
#define HVK_LARGE_BINS 1
#endif
#ifndef HVK_LARGE_QSTRIDE
#define HVK_LARGE_QSTRIDE 1
#endif
#define LTAB(i) (HVK_LARGE_PROBE >= 2 ? 0.f : tab[i])

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
  static constexpr int WAVES = WIN == 16 ? 8 : 9;
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
// the -100 shift-region mask of (key, query) as a select, not a branch on the (uniform) edge
// flags: a branch over the mask code left its MFMA-result reader too close (hvk_common.h hvk_settle)
template <int WIN>
__device__ __forceinline__ float mask_of(bool edge_r, bool edge_c, const PosInfo<WIN>& k,
                                         const PosInfo<WIN>& q, float mask2) {
  return ((edge_r & (k.r != q.r)) | (edge_c & (k.c != q.c))) ? mask2 : 0.f;
}

// ------------------------------------------------------------------------------ forward
template <int WIN>
__global__ __launch_bounds__(LCfg<WIN>::THREADS, 1) void wmsa_fwd_large_kernel(FwdArgs a) {
  using K = LCfg<WIN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int w, h;
  hvk_decode_chunk_head(blockIdx.x, g.nH, w, h);
  if (w >= g.n_windows) return;
  char* kimg = smem;
  char* vimg = smem + K::IMG;
  float* tab = reinterpret_cast<float*>(smem + 2 * K::IMG);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * C;
  const int per_img = g.nWh * g.nWw;
  const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;

  const float* bsrc = a.bias + (size_t)h * K::RR;
  for (int e = threadIdx.x; e < K::RR; e += K::THREADS) tab[e] = bsrc[e] * HVK_LOG2E;
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

  const float sc2 = a.scale[h] * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  const int lim = WIN - g.shift;
  const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;

  for (int t0 = wave * K::QB; t0 < K::NT; t0 += K::WAVES * K::QB) {
    uint4 qf[K::QB];
    int qrow[K::QB];
    PosInfo<WIN> qi[K::QB];
    float m[K::QB], l[K::QB];
    hvk_f32x4 o[K::QB][2];
#pragma unroll
    for (int j = 0; j < K::QB; ++j) {
      const int pos = 16 * (t0 + j) + li, posc = pos < K::N ? pos : K::N - 1;
      qrow[j] = window_token_row(g, b, wh, ww, WIN, posc);
      qf[j] = pos < K::N ? hvk_ld16(a.qkv + (size_t)qrow[j] * C3 + h * 32 + 8 * gq) : make_uint4(0, 0, 0, 0);
      float rn;
      qf[j] = l2_normalize(qf[j], rn, sc2);  // q^ * scale * log2e
      qi[j] = query_info<WIN>(posc, lim);
      m[j] = -INFINITY;
      l[j] = 0.f;
      o[j][0] = o[j][1] = hvk_f32x4{0, 0, 0, 0};
    }
#pragma unroll 1
    for (int c = 0; c < K::NC; ++c) {
      const uint4 kf0 = lds16(kimg, fm16(32 * c + li, gq));
      const uint4 kf1 = lds16(kimg, fm16(32 * c + 16 + li, gq));
      const uint4 vt0 = tr_frag(vimg, c, 0, li, gq), vt1 = tr_frag(vimg, c, 1, li, gq);
      PosInfo<WIN> ki[2][4];
      bool kpad[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = 32 * c + 16 * t + 4 * gq + r;
          kpad[t][r] = key >= K::N;
          ki[t][r] = key_info<WIN>(kpad[t][r] ? K::N - 1 : key, lim);
        }
#pragma unroll
      for (int j = 0; j < K::QB; ++j) {
        hvk_f32x4 s[2] = {hvk_mfma16(kf0, qf[j], hvk_f32x4{0, 0, 0, 0}),
                          hvk_mfma16(kf1, qf[j], hvk_f32x4{0, 0, 0, 0})};
        float mc = -INFINITY;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = s[t][r] + LTAB(qi[j].b - ki[t][r].b);
            v += mask_of(edge_r, edge_c, ki[t][r], qi[j], mask2);
            if (kpad[t][r]) v = -INFINITY;
            s[t][r] = v;
            mc = fmaxf(mc, v);
          }
        mc = hvk_group4_max(mc);
        const float mn = fmaxf(m[j], mc);
        const float alpha = __builtin_amdgcn_exp2f(m[j] - mn);
        m[j] = mn;
        float ps = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s[t][r] = __builtin_amdgcn_exp2f(s[t][r] - mn);
            ps += s[t][r];
          }
        l[j] = l[j] * alpha + ps;
        o[j][0] *= alpha;
        o[j][1] *= alpha;
        const uint4 pf = make_uint4(hvk_pack2(s[0][0], s[0][1]), hvk_pack2(s[0][2], s[0][3]),
                                    hvk_pack2(s[1][0], s[1][1]), hvk_pack2(s[1][2], s[1][3]));
        o[j][0] = hvk_mfma16(vt0, pf, o[j][0]);
        o[j][1] = hvk_mfma16(vt1, pf, o[j][1]);
      }
    }
#pragma unroll
    for (int j = 0; j < K::QB; ++j) {
      const int pos = 16 * (t0 + j) + li;
      const float inv = __builtin_amdgcn_rcpf(hvk_group4_sum(l[j]));
      if (pos < K::N) {
        const uint4 pk = make_uint4(hvk_pack2(o[j][0][0] * inv, o[j][0][1] * inv),
                                    hvk_pack2(o[j][0][2] * inv, o[j][0][3] * inv),
                                    hvk_pack2(o[j][1][0] * inv, o[j][1][1] * inv),
                                    hvk_pack2(o[j][1][2] * inv, o[j][1][3] * inv));
        hvk_st16(a.out + (size_t)qrow[j] * C + h * 32 + 8 * gq, pk);
      }
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
  return 2 * (size_t)K::IMG + (size_t)K::RRP * 4 + bins * 4 + 2 * (size_t)K::ROWS * 4;
}

template <int WIN>
__global__ __launch_bounds__(LCfg<WIN>::BTHREADS, 1) void wmsa_bwd_large_kernel(BwdArgs a) {
  using K = LCfg<WIN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int w, h;
  hvk_decode_chunk_head(blockIdx.x, g.nH, w, h);
  if (w >= g.n_windows) return;
  char* img0 = smem;
  char* img1 = smem + K::IMG;
  float* tab = reinterpret_cast<float*>(smem + 2 * K::IMG);
  float* dtab = tab + K::RRP;    // [BWAVES][RRP] private bins (HVK_LARGE_BINS) or [RR] shared
  constexpr int NBIN = HVK_LARGE_BINS ? K::BWAVES * K::RRP : K::RR;
  float* lse_s = dtab + NBIN;    // [ROWS] row log2-sum-exp2 (+inf for padding rows)
  float* dlt_s = lse_s + K::ROWS;  // [ROWS] delta = rowsum(P * dP)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * C;
  const int per_img = g.nWh * g.nWw;
  const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
  const float scale = a.scale[h];
  const float sc2 = scale * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  const int lim = WIN - g.shift;
  const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;

  const float* bsrc = a.bias + (size_t)h * K::RR;
  for (int e = threadIdx.x; e < K::RR; e += K::BTHREADS) tab[e] = bsrc[e] * HVK_LOG2E;
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

  // ---------------- phase 1: query tiles (query on the lane)
  float dscale = 0.f;
  float dqb[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int qt = wave; qt < K::NT; qt += K::BWAVES) {
    // query tile qt = positions qt + NT*li (N = 16 NT for w 12/16/24): the 16 queries of a tile
    // lie >= one window row apart, so the CPB-gradient atomics of one instruction (query li,
    // key 4g + r) never share an LDS address (consecutive queries put 4 lanes on each)
    const int pos = HVK_LARGE_QSTRIDE ? qt + K::NT * li : 16 * qt + li, posc = pos < K::N ? pos : K::N - 1;
    const bool qvalid = pos < K::N;
    const int qrow = window_token_row(g, b, wh, ww, WIN, posc);
    const hvk_bf16* qp = a.qkv + (size_t)qrow * C3 + h * 32;
    const uint4 qraw = qvalid ? hvk_ld16(qp + 8 * gq) : make_uint4(0, 0, 0, 0);
    const uint4 dof = qvalid ? hvk_ld16(a.dout + (size_t)qrow * C + h * 32 + 8 * gq) : make_uint4(0, 0, 0, 0);
    float rnq;
    const uint4 qs = l2_normalize(qraw, rnq, sc2);
    const PosInfo<WIN> qi = query_info<WIN>(posc, lim);

    // loop A: row max, sum and delta (online)
    float m = -INFINITY, l = 0.f, dacc = 0.f;
#pragma unroll 1
    for (int c = 0; c < K::NC; ++c) {
      float v[2][4], dp[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int kt = 2 * c + t;
        const hvk_f32x4 s = hvk_mfma16(lds16(img0, fm16(16 * kt + li, gq)), qs, hvk_f32x4{0, 0, 0, 0});
        const hvk_f32x4 d = hvk_mfma16(lds16(img1, fm16(16 * kt + li, gq)), dof, hvk_f32x4{0, 0, 0, 0});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = 16 * kt + 4 * gq + r;
          const PosInfo<WIN> ki = key_info<WIN>(key < K::N ? key : K::N - 1, lim);
          float x = s[r] + LTAB(qi.b - ki.b);
          x += mask_of(edge_r, edge_c, ki, qi, mask2);
          v[t][r] = key < K::N ? x : -INFINITY;
          dp[t][r] = d[r];
        }
      }
      float mc = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mc = fmaxf(mc, v[t][r]);
      mc = hvk_group4_max(mc);
      const float mn = fmaxf(m, mc);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      float ps = 0.f, pd = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(v[t][r] - mn);
          ps += p;
          pd += p * dp[t][r];
        }
      l = l * alpha + ps;
      dacc = dacc * alpha + pd;
    }
    l = hvk_group4_sum(l);
    dacc = hvk_group4_sum(dacc);
    const float lse = m + __log2f(l);
    const float delta = dacc / l;
    if (gq == 0 && qvalid) {
      lse_s[pos] = lse;
      dlt_s[pos] = delta;
    }

    // loop B: dS, dQ^, bias / scale gradients
    hvk_f32x4 dq[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll 1
    for (int c = 0; c < K::NC; ++c) {
      float ds[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int kt = 2 * c + t;
        const hvk_f32x4 s = hvk_mfma16(lds16(img0, fm16(16 * kt + li, gq)), qs, hvk_f32x4{0, 0, 0, 0});
        const hvk_f32x4 d = hvk_mfma16(lds16(img1, fm16(16 * kt + li, gq)), dof, hvk_f32x4{0, 0, 0, 0});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = 16 * kt + 4 * gq + r;
          const bool kvalid = key < K::N;
          const PosInfo<WIN> ki = key_info<WIN>(kvalid ? key : K::N - 1, lim);
          const int idx = qi.b - ki.b;
          float x = s[r] + LTAB(idx);
          x += mask_of(edge_r, edge_c, ki, qi, mask2);
          const float p = kvalid ? __builtin_amdgcn_exp2f(x - lse) : 0.f;
          const float dsv = p * (d[r] - delta);
          ds[t][r] = dsv;
          if (kvalid && qvalid) {
            if (HVK_LARGE_PROBE >= 1) {
            } else if (HVK_LARGE_BINS) {
              // this wave's own bins; the 64 lanes of one read-add-write never share a bin
              // (strided query tiles), and a wave's LDS operations complete in order.  The
              // compiler fences keep each read-add-write whole: without them hipcc merges the
              // reads of a lane's adjacent bins (r, r + 1) ahead of the writes, which is
              // exact per lane but loses the updates another lane makes in between
              float* pb = dtab + wave * K::RRP + idx;
              asm volatile("" ::: "memory");
              *pb += dsv;
              asm volatile("" ::: "memory");
            } else {
              atomicAdd(&dtab[idx], dsv);  // LDS float atomic (ds_add_f32)
            }
            dscale += dsv * s[r];        // s = sc2 * cos: divided out at the end
          }
        }
      }
      const uint4 bf = make_uint4(hvk_pack2(scale * ds[0][0], scale * ds[0][1]),
                                  hvk_pack2(scale * ds[0][2], scale * ds[0][3]),
                                  hvk_pack2(scale * ds[1][0], scale * ds[1][1]),
                                  hvk_pack2(scale * ds[1][2], scale * ds[1][3]));
      dq[0] = hvk_mfma16(tr_frag(img0, c, 0, li, gq), bf, dq[0]);
      dq[1] = hvk_mfma16(tr_frag(img0, c, 1, li, gq), bf, dq[1]);
    }
    normalize_bwd_store(qp, rnq, dq, qvalid ? a.dqkv + (size_t)qrow * C3 + h * 32 : nullptr,
                        1.f, gq, dqb);
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
  for (int kt = wave; kt < K::NT; kt += K::BWAVES) {
    const int pos = 16 * kt + li, posc = pos < K::N ? pos : K::N - 1;
    const bool kvalid = pos < K::N;
    const int krow = window_token_row(g, b, wh, ww, WIN, posc);
    const hvk_bf16* kp = a.qkv + (size_t)krow * C3 + h * 32 + C;
    const uint4 kraw = kvalid ? hvk_ld16(kp + 8 * gq) : make_uint4(0, 0, 0, 0);
    const uint4 vf = kvalid ? hvk_ld16(kp + C + 8 * gq) : make_uint4(0, 0, 0, 0);
    float rnk;
    const uint4 kh = l2_normalize(kraw, rnk);
    const PosInfo<WIN> ki = key_info<WIN>(posc, lim);
    hvk_f32x4 dk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, dv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll 1
    for (int c = 0; c < K::NC; ++c) {
      float p[2][4], ds[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int qt = 2 * c + t;
        const hvk_f32x4 s = hvk_mfma16(lds16(img0, fm16(16 * qt + li, gq)), kh, hvk_f32x4{0, 0, 0, 0});
        const hvk_f32x4 d = hvk_mfma16(lds16(img1, fm16(16 * qt + li, gq)), vf, hvk_f32x4{0, 0, 0, 0});
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + 16 * qt + 4 * gq);
        const float4 d4 = *reinterpret_cast<const float4*>(dlt_s + 16 * qt + 4 * gq);
        const float lr[4] = {l4.x, l4.y, l4.z, l4.w}, dr[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 16 * qt + 4 * gq + r;
          const PosInfo<WIN> qi = query_info<WIN>(q < K::N ? q : K::N - 1, lim);
          float x = s[r] + LTAB(qi.b - ki.b);
          x += mask_of(edge_r, edge_c, ki, qi, mask2);
          p[t][r] = __builtin_amdgcn_exp2f(x - lr[r]);  // padding query: lse = +inf -> 0
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
    normalize_bwd_store(kp, rnk, dk, kvalid ? dst + C : nullptr, 1.f / HVK_LOG2E, gq, nullptr);
    if (kvalid) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        hvk_st8(dst + 2 * C + 16 * dt + 4 * gq,
                make_uint2(hvk_pack2(dv[dt][0], dv[dt][1]), hvk_pack2(dv[dt][2], dv[dt][3])));
    }
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

template <int WIN>
int launch_fwd_large(const FwdArgs& a, hipStream_t st) {
  using K = LCfg<WIN>;
  const size_t lds = 2 * (size_t)K::IMG + (size_t)K::RR * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_fwd_large_kernel<WIN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int padded = (a.g.n_windows + 7) / 8 * 8;
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_FWD, wmsa_fwd_large_kernel<WIN>, dim3(padded * a.g.nH), dim3(K::THREADS), lds, st, a);
  HVK_CHECK_LAUNCH("wmsa_fwd_large");
  return HVK_OK;
}

template <int WIN>
int launch_bwd_large(const BwdArgs& a, float* dtab, float* dscale, float* dqb, hipStream_t st) {
  using K = LCfg<WIN>;
  const size_t lds = bwd_large_lds<WIN>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_large_kernel<WIN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int padded = (a.g.n_windows + 7) / 8 * 8;
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, wmsa_bwd_large_kernel<WIN>, dim3(padded * a.g.nH), dim3(K::BTHREADS), lds, st, a);
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
