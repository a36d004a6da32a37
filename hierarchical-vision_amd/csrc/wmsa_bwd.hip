// W-MSA backward for windows <= 8, key on the lane (gfx950).
//
// Same math as wmsa.hip's wmsa_bwd_kernel (the autograd of swinv2.py:221-261 with the roll /
// partition / reverse of 399-429 folded into addressing), reorganised so that nothing needs a
// per-row reduction and several waves share every SIMD:
//   * the forward (wmsa_ring.hip, LSE build) stores each query's row constant
//     L2 = log2 sum_k exp2(log2e * logit), and the backward computes delta = rowsum(dO o O) from
//     the attention output O (the proj layer's saved input), so P = exp2(log2e * logit - L2) and
//     dS = P (dP - delta) are elementwise;
//   * S and dP are computed with the QUERY in the accumulator rows and the KEY on the lane
//     (D = Q K^T with the bias table in C, D = dO V^T with -delta in C): their accumulators are
//     directly the B operands of dV^T += dO^T P and dK^T += Q^T dS (dO^T and Q^T by
//     ds_read_b64_tr_b16 from LDS images), so P never touches LDS; dS crosses LDS once, for
//     dQ^T += K^T dS^T;
//   * a workgroup is TWO waves sharing one (window, head): staging, the key tiles (S, dP, dV,
//     dK, the CPB-table gradient) and the query tiles of dQ are split between them, with three
//     workgroup barriers per window; per wave ~10 KB of LDS and ~150 VGPRs, so a CU holds
//     several such pairs whose barriers and memory waits cover each other.
// The CPB-table gradient accumulates per lane over the pair's windows in registers
// ([query tile][own key tile][r]) and is binned by rel-pos index in the finalize kernel.  The
// logits come out of the MFMA exactly as in the forward, S = (scale log2e q^)_bf16 . k^ +
// log2e bias (the forward's operand rounding, the bias table as the C operand), so P against
// the forward's row constant is consistent to f32 summation order; the logit-scale gradient
// accumulates sum dS S and the finalize subtracts sum_idx bias dtab.
// Token positions sit on the forward's padded grid (wmsa_ring.h, PW = 8, 4 for w4): the rel-pos
// index of (query 16qi + 4g + r, key 16kt + l) is TR (qi - kt) + r + base(lane), one lane-constant
// table pointer plus compile-time offsets into a compact per-head table.
#include "wmsa_ring.h"

#ifndef HVK_KL_MINB
#define HVK_KL_MINB 2
#endif
#ifndef HVK_KL_PROBE
#define HVK_KL_PROBE 0
#endif
#ifndef HVK_KL_SPLIT
#define HVK_KL_SPLIT 0
#endif
#ifndef HVK_KL_SB
#define HVK_KL_SB 1
#endif

namespace {
using namespace hvk_ring;

template <int WIN>
struct BCfg {
  using RC = RingCfg<WIN, 1>;
  static constexpr int PW = RC::PW, NT = RC::NT, NC = RC::NC, R = RC::R, TR = RC::TR;
  static constexpr int HALF = (NT + 1) / 2;      // key / query tiles per wave (wave 1: NT - HALF)
  // waves per workgroup: two (tiles [0, HALF) and [HALF, NT)) or, HVK_KL_SPLIT, one per tile
  static constexpr int NW = HVK_KL_SPLIT ? NT : (NT > 1 ? 2 : 1);
  template <int W>
  static constexpr int t0() { return HVK_KL_SPLIT ? W : (W == 0 ? 0 : HALF); }
  template <int W>
  static constexpr int ntl() { return HVK_KL_SPLIT ? 1 : (W == 0 ? HALF : NT - HALF); }
  static constexpr int ROWS = 32 * NC;           // token slots of the [ROWS][32] bf16 images
  static constexpr int IMG = ROWS * 64;          // bytes of one such image
  static constexpr int DSI = ROWS * ROWS * 2;    // dS image: [ROWS keys][ROWS queries] bf16
  // q^, k^, dO images, dS, -L2 and -delta per query, a dummy 128-B dS row for padding keys
  static constexpr int SHARED = 3 * IMG + DSI + 2 * ROWS * 4 + 128;
  static constexpr int LQMIN = (WIN - 1) * R + WIN - 1;
  static constexpr int LQMAX = PW == 8 ? WIN * R + 4 + WIN - 1 : (WIN + 2) * R + WIN - 1;
  static constexpr int LKMAX = PW == 8 ? R + 7 : 3 * R + 3;
  static constexpr int BMIN = LQMIN - LKMAX - TR * (NT - 1);
  static constexpr int BMAX = LQMAX - TR * (NT - 1);
  static constexpr int PAD = BMIN < 0 ? -BMIN : 0;
  static constexpr int HI = BMAX + 2 * TR * (NT - 1) + 3;  // largest index read
  static constexpr int TABF = ((PAD + (HI + 1 > R * R ? HI + 1 : R * R) + 3) / 4) * 4;
  static constexpr int TAB = NT * NT * 256;      // accumulator-order CPB-gradient floats per head
  static constexpr int LDS = SHARED + TABF * 4;
  static_assert(TAB * 4 <= SHARED, "the workgroup reduction reuses the images");
};


// dS image [ROWS keys][ROWS q] bf16, 8-B units XOR-swizzled by row (wmsa.hip pimg_off): the
// 8-B writes of a key tile and the transposed reads of dQ are bank-conflict free
template <int COLS>
__device__ __forceinline__ int ds_off(int row, int col8) {
  const int f = ((row ^ (row >> 2)) & 1) | ((row >> 2) & 2) | ((row << 1) & 4);
  return (row * COLS + (((col8 ^ f) & (COLS / 4 - 1)) << 2)) * 2;  // bytes
}

template <int WIN>
__device__ __forceinline__ bool pos_valid(int p) {
  using K = BCfg<WIN>;
  return (p % K::PW) < WIN && (p / K::PW) < WIN;
}

struct Lane {
  int li, gq, lim;
  bool edge_r, edge_c;
  float scale, sc2;
};

// Raw global inputs of this wave's token tiles of one window (issued a window ahead, so the
// loads of window w + 1 run under the key / query tiles of window w).
template <int NTL>
struct Raw {
  static constexpr int N = NTL > 0 ? NTL : 1;
  int row[N];
  uint4 q[N], k[N], v[N], d[N], o[N];
  float l2[N];
};

template <int WIN, int T0, int NTL>
__device__ __forceinline__ void load_raw(const BwdArgs& a, const Lane& L, int h, int w, Raw<NTL>& r) {
  using K = BCfg<WIN>;
  const WmsaGeom& g = a.g;
  const int C = g.C, C3 = 3 * g.C;
  const int per_img = g.nWh * g.nWw;
  const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
#pragma unroll
  for (int j = 0; j < NTL; ++j) {
    const int p = 16 * (T0 + j) + L.li;
    const int tok = grid_token<WIN, K::PW>(p);
    r.row[j] = window_token_row(g, b, wh, ww, WIN, tok >= 0 ? tok : 0);
    if (tok >= 0) {
      const hvk_bf16* src = a.qkv + (size_t)r.row[j] * C3 + h * 32 + 8 * L.gq;
      r.q[j] = hvk_ld16(src);
      r.k[j] = hvk_ld16(src + C);
      r.v[j] = hvk_ld16(src + 2 * C);
      r.d[j] = hvk_ld16(a.dout + (size_t)r.row[j] * C + h * 32 + 8 * L.gq);
      r.o[j] = hvk_ld16(a.out + (size_t)r.row[j] * C + h * 32 + 8 * L.gq);
      r.l2[j] = a.lse[(size_t)r.row[j] * g.nH + h];
    } else {
      r.q[j] = r.k[j] = r.v[j] = r.d[j] = r.o[j] = make_uint4(0, 0, 0, 0);
      r.l2[j] = 1e30f;  // padding query: P = 0
    }
  }
}

// Stage this wave's token tiles t = T0 .. T0+NTL-1 of a window from the raw loads: q^, k^, dO
// into the images, -L2 and -delta (= -dO.O) per query slot; the normalisation factors.
template <int WIN, int T0, int NTL>
__device__ __forceinline__ void stage(const Lane& L, const Raw<NTL>& r, char* qimg, char* kimg, char* dimg,
                                      float* nl2, float* ndl, float (&rnq)[NTL > 0 ? NTL : 1],
                                      float (&rnk)[NTL > 0 ? NTL : 1]) {
#pragma unroll
  for (int j = 0; j < NTL; ++j) {
    const int p = 16 * (T0 + j) + L.li;
    // q^ * scale * log2e rounded to bf16 exactly as the forward's operand: the logits (and so
    // P against the forward's row constant) are bit-consistent with the forward's
    const uint4 qh = l2_normalize(r.q[j], rnq[j], L.sc2);
    const uint4 kh = l2_normalize(r.k[j], rnk[j]);
    *reinterpret_cast<uint4*>(qimg + fm16(p, L.gq)) = qh;
    *reinterpret_cast<uint4*>(kimg + fm16(p, L.gq)) = kh;
    *reinterpret_cast<uint4*>(dimg + fm16(p, L.gq)) = r.d[j];
    float fd[8], fo[8];
    hvk_unpack8(r.d[j], fd);
    hvk_unpack8(r.o[j], fo);
    float dl = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) dl = fmaf(fd[e], fo[e], dl);
    dl = hvk_group4_sum(dl);
    if (L.gq == 0) {
      nl2[p] = -r.l2[j];
      ndl[p] = -dl;
    }
  }
}

// The wave's key tiles kt = T0 .. T0+NTL-1 against every query tile: S, dP, P, dS; dV^T and
// dK^T (stored with the normalisation backward of k); dS rows into the image; the CPB-table
// and logit-scale gradient accumulators.
template <int WIN, int T0, int NTL>
__device__ __forceinline__ void key_tiles(const BwdArgs& a, const Lane& L, int h, const float* tl,
                                          char* qimg, char* kimg, char* dimg, char* simg, char* dummy,
                                          const float* nl2, const float* ndl,
                                          const int (&row)[NTL > 0 ? NTL : 1], const float (&rnk)[NTL > 0 ? NTL : 1],
                                          const uint4 (&vf)[NTL > 0 ? NTL : 1],
                                          hvk_f32x4 (&dbias)[BCfg<WIN>::NT][NTL > 0 ? NTL : 1], float& dsc) {
  using K = BCfg<WIN>;
  const int li = L.li, gq = L.gq;
  const int C = a.g.C, C3 = 3 * a.g.C;
  const float mask2 = -100.f * HVK_LOG2E;
#pragma unroll
  for (int j = 0; j < NTL; ++j) {
    constexpr int dummy_unused = 0;
    (void)dummy_unused;
    const int kt = T0 + j;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int pk = 16 * kt + li;
    const bool kvalid = pos_valid<WIN>(pk);
    const uint4 kb = lds16(kimg, fm16(pk, gq));
    int kyb, kxb;  // the key's shift bands (row, column)
    if (K::PW == 8) {
      kyb = (2 * kt + (li >> 3)) >= L.lim;
      kxb = (li & 7) >= L.lim;
    } else {
      kyb = (4 * kt + (li >> 2)) >= L.lim;
      kxb = (li & 3) >= L.lim;
    }
    hvk_f32x4 dv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, dk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    float dsk = 0.f;
#pragma unroll
    for (int c = 0; c < K::NC; ++c) {
      // both query tiles of the chunk in flight: their S / dP MFMAs issue back to back and the
      // second pair runs under the first one's exp / dS arithmetic
      uint4 qa[2], da[2];
      float4 nl[2], nd[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int qi = 2 * c + hh < K::NT ? 2 * c + hh : 2 * c;
        qa[hh] = lds16(qimg, fm16(16 * qi + li, gq));
        da[hh] = lds16(dimg, fm16(16 * qi + li, gq));
        nl[hh] = *reinterpret_cast<const float4*>(nl2 + 16 * qi + 4 * gq);
        nd[hh] = *reinterpret_cast<const float4*>(ndl + 16 * qi + 4 * gq);
      }
      hvk_f32x4 s[2], dp[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int qi = 2 * c + hh < K::NT ? 2 * c + hh : 2 * c;
        const float* tb = tl + K::TR * (qi - kt + K::NT - 1);  // compile-time offset
        s[hh] = hvk_mfma16(qa[hh], kb, hvk_f32x4{tb[0], tb[1], tb[2], tb[3]});
        dp[hh] = hvk_mfma16(da[hh], vf[j], hvk_f32x4{nd[hh].x, nd[hh].y, nd[hh].z, nd[hh].w});
      }
      hvk_settle(s[0], dp[0], s[1], dp[1]);  // the unmasked path branches straight to their readers
      uint32_t pp[2][2], sp[2][2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int qi = 2 * c + hh;
        if (qi >= K::NT) {
          pp[hh][0] = pp[hh][1] = sp[hh][0] = sp[hh][1] = 0u;
          continue;
        }
        float arg[4] = {nl[hh].x, nl[hh].y, nl[hh].z, nl[hh].w};
        if (L.edge_r || L.edge_c) {  // wave-uniform: the last window row / column only
          int qyb, qx0;
          if (K::PW == 8) {
            qyb = (2 * qi + (gq >> 1)) >= L.lim;
            qx0 = 4 * (gq & 1);
          } else {
            qyb = (4 * qi + gq) >= L.lim;
            qx0 = 0;
          }
          const bool rmis = L.edge_r && (qyb != kyb);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool cmis = L.edge_c && ((int)((qx0 + r) >= L.lim) != kxb);
            arg[r] += (rmis || cmis) ? mask2 : 0.f;
          }
        }
        float p[4], ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = __builtin_amdgcn_exp2f(s[hh][r] + arg[r]);
          ds[r] = p[r] * dp[hh][r];
          dbias[qi][j][r] += ds[r];
          dsk = fmaf(ds[r], s[hh][r], dsk);
        }
        pp[hh][0] = hvk_pack2(p[0], p[1]);
        pp[hh][1] = hvk_pack2(p[2], p[3]);
        sp[hh][0] = hvk_pack2(ds[0], ds[1]);
        sp[hh][1] = hvk_pack2(ds[2], ds[3]);
        // dS rows (key) x 4 consecutive queries; padding keys leave their (zero) rows alone
        *reinterpret_cast<uint2*>(kvalid ? simg + ds_off<K::ROWS>(pk, 4 * qi + gq) : dummy) =
            make_uint2(sp[hh][0], sp[hh][1]);
      }
      const uint4 pf = make_uint4(pp[0][0], pp[0][1], pp[1][0], pp[1][1]);
      const uint4 sf = make_uint4(sp[0][0], sp[0][1], sp[1][0], sp[1][1]);
      // dV^T += dO^T P, dK^T += Q^T dS over this 32-query chunk (q order as the packs)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int rq = 32 * c + 4 * gq + (li >> 2), c8 = 4 * dt + (li & 3);
        const uint2 dlo = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(dimg + fm8(rq, c8)));
        const uint2 dhi = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(dimg + fm8(rq + 16, c8)));
        dv[dt] = hvk_mfma16(make_uint4(dlo.x, dlo.y, dhi.x, dhi.y), pf, dv[dt]);
        const uint2 qlo = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(qimg + fm8(rq, c8)));
        const uint2 qhi = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(qimg + fm8(rq + 16, c8)));
        dk[dt] = hvk_mfma16(make_uint4(qlo.x, qlo.y, qhi.x, qhi.y), sf, dk[dt]);
      }
    }
    dsc += kvalid ? dsk : 0.f;
    // dK (normalisation backward, scale applied here) and dV of this key tile
    float kh[2][4], dot = 0.f;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const uint2 v = *reinterpret_cast<const uint2*>(kimg + fm8(pk, 4 * dt + gq));
      kh[dt][0] = hvk_lo(v.x); kh[dt][1] = hvk_hi(v.x);
      kh[dt][2] = hvk_lo(v.y); kh[dt][3] = hvk_hi(v.y);
#pragma unroll
      for (int r = 0; r < 4; ++r) dot += kh[dt][r] * dk[dt][r];
    }
    dot = hvk_group4_sum(dot);
    if (rnk[j] >= 1e12f) dot = 0.f;  // ||k|| <= eps: x / eps, no projection term
    {
      const float f = rnk[j] * (1.f / HVK_LOG2E);  // scale dS q^ = dS (scale log2e q^) / log2e
      uint2 pk[2], pv[2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (dk[dt][r] - kh[dt][r] * dot) * f;
        pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
        pv[dt] = make_uint2(hvk_pack2(dv[dt][0], dv[dt][1]), hvk_pack2(dv[dt][2], dv[dt][3]));
      }
      const uint4 ok = hvk_pair_swap(pk[0], pk[1]), ov = hvk_pair_swap(pv[0], pv[1]);
      if (kvalid) {
        hvk_bf16* dst = a.dqkv + (size_t)row[j] * C3 + h * 32 + hvk_pair_col(gq);
        hvk_st16(dst + C, ok);
        hvk_st16(dst + 2 * C, ov);
      }
    }
  }
}

// dQ^T = K^T dS^T for the wave's query tiles over every key chunk, the normalisation backward
// of q (scale applied here), the store and the q_bias column sums.
template <int WIN, int T0, int NTL>
__device__ __forceinline__ void query_tiles(const BwdArgs& a, const Lane& L, int h, const char* qimg,
                                            const char* kimg, const char* simg,
                                            const int (&row)[NTL > 0 ? NTL : 1],
                                            const float (&rnq)[NTL > 0 ? NTL : 1], float (&dqb)[2][4]) {
  using K = BCfg<WIN>;
  const int li = L.li, gq = L.gq;
  const int C3 = 3 * a.g.C;
#pragma unroll
  for (int j = 0; j < NTL; ++j) {
    const int qi = T0 + j;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    hvk_f32x4 dq[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int cc = 0; cc < K::NC; ++cc) {
      const int rs = 32 * cc + 4 * gq + (li >> 2), c8 = 4 * qi + (li & 3);
      const uint2 slo = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(simg + ds_off<K::ROWS>(rs, c8)));
      const uint2 shi = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(simg + ds_off<K::ROWS>(rs + 16, c8)));
      const uint4 bs = make_uint4(slo.x, slo.y, shi.x, shi.y);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int k8 = 4 * dt + (li & 3);
        const uint2 lo = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(kimg + fm8(rs, k8)));
        const uint2 hi = hvk_tr_read(reinterpret_cast<const hvk_bf16*>(kimg + fm8(rs + 16, k8)));
        dq[dt] = hvk_mfma16(make_uint4(lo.x, lo.y, hi.x, hi.y), bs, dq[dt]);
      }
    }
    const int pq = 16 * qi + li;
    float qh[2][4], dot = 0.f;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const uint2 v = *reinterpret_cast<const uint2*>(qimg + fm8(pq, 4 * dt + gq));
      const float u = 1.f / L.sc2;  // the image holds q^ * scale * log2e
      qh[dt][0] = hvk_lo(v.x) * u; qh[dt][1] = hvk_hi(v.x) * u;
      qh[dt][2] = hvk_lo(v.y) * u; qh[dt][3] = hvk_hi(v.y) * u;
#pragma unroll
      for (int r = 0; r < 4; ++r) dot += qh[dt][r] * dq[dt][r];
    }
    dot = hvk_group4_sum(dot);
    if (rnq[j] >= 1e12f) dot = 0.f;
    {
      const bool ok = pos_valid<WIN>(pq);
      const float f = L.scale * rnq[j];
      uint2 pk[2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = (dq[dt][r] - qh[dt][r] * dot) * f;
          if (ok) dqb[dt][r] += v[r];
        }
        pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
      }
      const uint4 o = hvk_pair_swap(pk[0], pk[1]);
      if (ok) hvk_st16(a.dqkv + (size_t)row[j] * C3 + h * 32 + hvk_pair_col(gq), o);
    }
  }
}

// One wave's part of the pair: W = 0 owns token tiles [0, HALF), W = 1 [HALF, NT)
template <int WIN, int W>
__device__ __forceinline__ void pair_wave(const BwdArgs& a, Lane L, int h, int w0, int w1, char* smem,
                                          const float* tl) {
  using K = BCfg<WIN>;
  constexpr int T0 = K::template t0<W>();
  constexpr int NTL = K::template ntl<W>();
  constexpr int NA = NTL > 0 ? NTL : 1;
  const WmsaGeom& g = a.g;
  char* qimg = smem;
  char* kimg = smem + K::IMG;
  char* dimg = smem + 2 * K::IMG;
  char* simg = smem + 3 * K::IMG;
  float* nl2 = reinterpret_cast<float*>(smem + 3 * K::IMG + K::DSI);
  float* ndl = nl2 + K::ROWS;
  char* dummy = reinterpret_cast<char*>(ndl + K::ROWS);
  const int per_img = g.nWh * g.nWw;

  hvk_f32x4 dbias[K::NT][NA];
#pragma unroll
  for (int qi = 0; qi < K::NT; ++qi)
#pragma unroll
    for (int j = 0; j < NA; ++j) dbias[qi][j] = hvk_f32x4{0, 0, 0, 0};
  float dsc = 0.f;
  float dqb[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};

#ifdef HVK_KL_STAMP
  unsigned long long* stp = (blockIdx.x < 1024 && L.li + L.gq == 0) ? a.stamp + ((blockIdx.x * 2 + W) * 4) * 8 : nullptr;
#define KL_STAMP(ph) do { if (stp && w - w0 < 4) { stp[(w - w0) * 8 + (ph)] = __builtin_amdgcn_s_memtime(); } } while (0)
#else
#define KL_STAMP(ph) do { } while (0)
#endif
  Raw<NTL> raw;
  load_raw<WIN, T0, NTL>(a, L, h, w0, raw);
#if HVK_KL_PROBE == 1
  // memory-only probe (not the product): the same loads and 16-B stores, no math, no barriers
  for (int w = w0; w < w1; ++w) {
#pragma unroll
    for (int j = 0; j < NTL; ++j) {
      const int p = 16 * (T0 + j) + L.li;
      uint4 x = raw.q[j];
      x.x ^= raw.d[j].x ^ raw.o[j].x ^ __float_as_uint(raw.l2[j]);
      if (pos_valid<WIN>(p)) {
        hvk_bf16* dst = a.dqkv + (size_t)raw.row[j] * 3 * g.C + h * 32 + 8 * L.gq;
        hvk_st16(dst, x);
        hvk_st16(dst + g.C, raw.k[j]);
        hvk_st16(dst + 2 * g.C, raw.v[j]);
      }
    }
    load_raw<WIN, T0, NTL>(a, L, h, w + 1 < w1 ? w + 1 : w, raw);
  }
  return;
#endif
  for (int w = w0; w < w1; ++w) {
    const int rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
    L.edge_r = g.shift && wh == g.nWh - 1;
    L.edge_c = g.shift && ww == g.nWw - 1;
    int row[NA];
    float rnq[NA], rnk[NA];
    uint4 vf[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      row[j] = raw.row[j];
      vf[j] = raw.v[j];
    }
    KL_STAMP(0);
    __syncthreads();  // the previous window's readers are done with the images
    KL_STAMP(1);
    stage<WIN, T0, NTL>(L, raw, qimg, kimg, dimg, nl2, ndl, rnq, rnk);
    KL_STAMP(2);
    __syncthreads();  // images complete
    KL_STAMP(3);
    key_tiles<WIN, T0, NTL>(a, L, h, tl, qimg, kimg, dimg, simg, dummy, nl2, ndl, row, rnk, vf, dbias, dsc);
    KL_STAMP(4);
    __builtin_amdgcn_sched_barrier(0);
    // lands under the query tiles; unconditional (the last window reloads itself) so that raw
    // is dead from the stage to here
    load_raw<WIN, T0, NTL>(a, L, h, w + 1 < w1 ? w + 1 : w, raw);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // dS complete
    KL_STAMP(5);
    query_tiles<WIN, T0, NTL>(a, L, h, qimg, kimg, simg, row, rnq, dqb);
    KL_STAMP(6);
  }
#undef KL_STAMP

  // ---- workgroup reduction of the CPB / scale / q_bias gradients, one atomic per entry
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [qi][kt][lane][r] over the whole tile grid
#pragma unroll
  for (int qi = 0; qi < K::NT; ++qi)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
      *reinterpret_cast<float4*>(red + ((qi * K::NT + T0 + j) * 64 + L.li + 16 * L.gq) * 4) =
          make_float4(dbias[qi][j][0], dbias[qi][j][1], dbias[qi][j][2], dbias[qi][j][3]);
  __syncthreads();
  float* dst = a.dbias_acc + (size_t)h * K::TAB;
  for (int e = threadIdx.x; e < K::TAB; e += 64 * K::NW) atomicAdd(dst + e, red[e]);
  dsc = hvk_wave_sum(dsc);
  if (threadIdx.x == 64 * W) atomicAdd(a.dscale_acc + h, dsc);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = hvk_row16_sum(dqb[dt][r]);
      if (L.li == 0) atomicAdd(a.dqb_acc + h * 32 + 16 * dt + 4 * L.gq + r, v);
    }
}

template <int WIN>
__global__ __launch_bounds__(HVK_KL_SPLIT ? 256 : 128, HVK_KL_MINB) void wmsa_bwd_kl_kernel(BwdArgs a) {
  using K = BCfg<WIN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int chunk, h;
  if (!decode_item(g, blockIdx.x, chunk, h)) return;
  const int w0 = (int)((long long)chunk * g.n_windows / g.n_chunks);
  const int w1 = (int)((long long)(chunk + 1) * g.n_windows / g.n_chunks);
  if (w0 >= w1) return;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  Lane L;
  L.li = lane & 15;
  L.gq = lane >> 4;
  L.lim = WIN - g.shift;
  L.scale = a.scale[h];
  L.sc2 = L.scale * HVK_LOG2E;
  float* tab = reinterpret_cast<float*>(smem + K::SHARED);
  for (int e = threadIdx.x; e < K::TABF; e += 64 * K::NW) {
    const int j = e - K::PAD;
    tab[e] = (j >= 0 && j < K::R * K::R) ? a.bias[(size_t)h * K::R * K::R + j] * HVK_LOG2E : 0.f;
  }
  {  // zero the images once: rows of padding tokens are never written again
    uint4* z = reinterpret_cast<uint4*>(smem);
    for (int e = threadIdx.x; e < K::SHARED / 16; e += 64 * K::NW) z[e] = make_uint4(0, 0, 0, 0);
  }
  // lane-constant table pointer: entry TR (qi - kt + NT - 1) + r sits at tl + that offset
  int lq, lk;
  if (K::PW == 8) {
    lq = ((L.gq >> 1) + WIN - 1) * K::R + 4 * (L.gq & 1) + WIN - 1;
    lk = (L.li >> 3) * K::R + (L.li & 7);
  } else {
    lq = (L.gq + WIN - 1) * K::R + WIN - 1;
    lk = (L.li >> 2) * K::R + (L.li & 3);
  }
  const float* tl = tab + K::PAD + lq - lk - K::TR * (K::NT - 1);
  if (wave == 0)
    pair_wave<WIN, 0>(a, L, h, w0, w1, smem, tl);
  else if (K::NW > 1 && wave == 1)
    pair_wave<WIN, (K::NW > 1 ? 1 : 0)>(a, L, h, w0, w1, smem, tl);
  else if (K::NW > 2 && wave == 2)
    pair_wave<WIN, (K::NW > 2 ? 2 : 0)>(a, L, h, w0, w1, smem, tl);
  else if (K::NW > 3)
    pair_wave<WIN, (K::NW > 3 ? 3 : 0)>(a, L, h, w0, w1, smem, tl);
}

// Bin the accumulator-order partial sums ([qi][kt][lane][r]: query 16qi + 4(lane>>4) + r, key
// 16kt + (lane&15) on the padded grid) into the CPB-table gradient [nH, R*R]; dscale =
// (sum dS S / log2e - sum_idx bias[idx] dtab[idx]) / scale with S = log2e (scale cos + bias);
// dq_bias; zero the workspace for the next call.
template <int WIN>
__global__ __launch_bounds__(256) void wmsa_bwd_kl_finalize(BwdArgs a, float* __restrict__ dtab,
                                                          float* __restrict__ dscale,
                                                          float* __restrict__ dqb) {
  using K = BCfg<WIN>;
  __shared__ float bins[K::R * K::R];
  __shared__ float red[4];
  const int h = blockIdx.x;
  for (int i = threadIdx.x; i < K::R * K::R; i += blockDim.x) bins[i] = 0.f;
  __syncthreads();
  float* acc = a.dbias_acc + (size_t)h * K::TAB;
  for (int e = threadIdx.x; e < K::TAB; e += blockDim.x) {
    const int r = e & 3, lane = (e >> 2) & 63, blk = e >> 8;
    const int qi = blk / K::NT, kt = blk % K::NT;
    const int q = 16 * qi + 4 * (lane >> 4) + r, key = 16 * kt + (lane & 15);
    const int qy = q / K::PW, qx = q % K::PW, ky = key / K::PW, kx = key % K::PW;
    if (qx < WIN && qy < WIN && kx < WIN && ky < WIN)
      atomicAdd(&bins[(qy - ky + WIN - 1) * K::R + (qx - kx + WIN - 1)], acc[e]);
    acc[e] = 0.f;
  }
  __syncthreads();
  const float sc = a.scale[h];
  float part = 0.f;
  for (int i = threadIdx.x; i < K::R * K::R; i += blockDim.x) {
    dtab[(size_t)h * K::R * K::R + i] = bins[i];
    part += a.bias[(size_t)h * K::R * K::R + i] * bins[i];
  }
  part = hvk_wave_sum(part);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x < 32) {
    const int c = h * 32 + threadIdx.x;
    if (dqb) dqb[c] = a.dqb_acc[c];
    a.dqb_acc[c] = 0.f;
  }
  if (threadIdx.x == 32) {  // S = log2e (scale cos + bias): sum dS cos = (sum dS S / log2e - sum bias dtab) / scale
    dscale[h] = (a.dscale_acc[h] * (1.f / HVK_LOG2E) - (red[0] + red[1] + red[2] + red[3])) / sc;
    a.dscale_acc[h] = 0.f;
  }
}

template <int WIN>
int launch_kl(BwdArgs& a, float* dtab, float* dscale, float* dqb, hipStream_t st) {
  using K = BCfg<WIN>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_kl_kernel<WIN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    attr = true;
  }
  // resident pairs: 256 CUs x (what LDS and registers admit); (chunk, head) items dealt to the
  // XCDs in runs
  static int per_cu = 0;
  if (!per_cu) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(&wmsa_bwd_kl_kernel<WIN>),
                                                     64 * K::NW, K::LDS) != hipSuccess || nb < 1)
      nb = 1;
    per_cu = nb;
  }
  int c = 256 * per_cu / a.g.nH;
  if (c < 1) c = 1;
  a.g.n_chunks = c < a.g.n_windows ? c : a.g.n_windows;
  a.g.xcd_runs = 1;
  const int items = a.g.n_chunks * a.g.nH;
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, wmsa_bwd_kl_kernel<WIN>, dim3(8 * ((items + 7) / 8)),
                   dim3(64 * K::NW), K::LDS, st, a);
  HVK_CHECK_LAUNCH("wmsa_bwd_kl");
  hipLaunchKernelGGL(wmsa_bwd_kl_finalize<WIN>, dim3(a.g.nH), dim3(256), 0, st, a, dtab, dscale, dqb);
  HVK_CHECK_LAUNCH("wmsa_bwd_kl_finalize");
  return HVK_OK;
}

}  // namespace

namespace hvk_wmsa {
size_t kl_acc_floats(int num_heads, int win) {
  switch (win) {
    case 7: return (size_t)num_heads * BCfg<7>::TAB;
    case 8: return (size_t)num_heads * BCfg<8>::TAB;
    case 6: return (size_t)num_heads * BCfg<6>::TAB;
    case 4: return (size_t)num_heads * BCfg<4>::TAB;
    default: return 0;
  }
}

int kl_bwd(BwdArgs& a, int win, float* dtab, float* dscale, float* dqb, hipStream_t st) {
  switch (win) {
    case 7: return launch_kl<7>(a, dtab, dscale, dqb, st);
    case 8: return launch_kl<8>(a, dtab, dscale, dqb, st);
    case 6: return launch_kl<6>(a, dtab, dscale, dqb, st);
    case 4: return launch_kl<4>(a, dtab, dscale, dqb, st);
    default: return hvk_set_error(HVK_EUNSUPPORTED, "wmsa_bwd_kl: window %d", win);
  }
}
}  // namespace hvk_wmsa
