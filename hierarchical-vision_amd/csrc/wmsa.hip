// Fused (shifted-)window cosine attention for SwinV2 on gfx950.
//
// Replaces, per block, the reference's eager sequence (swinv2.py):
//   torch.roll(-s)                                  399-404
//   window_partition + view                         69-83, 407-412
//   F.normalize(q), F.normalize(k), q@k^T           229
//   * exp(clamp(logit_scale, max=ln 100))           230-231
//   + 16*sigmoid(cpb_mlp(table))[rpi]               233-247
//   + shift mask (-100 across regions)              249-254, 357-388
//   softmax, @v, transpose/reshape                  255-261
//   window_reverse + torch.roll(+s)                 86-102, 420-429
// The qkv and proj Linear layers are token-wise, so they commute with the
// shift/partition permutation: the kernels read the UN-partitioned qkv token
// tensor [B*H*W, 3C] and write the attention core output straight back to the
// UN-partitioned token rows [B*H*W, C]; the roll/partition/reverse copies of the
// reference never exist.  Windows are gathered by closed-form index math.
//
// Layout per (window, head) pair, one wave each: N = WIN^2 tokens padded to
// NT = ceil(N/16) tiles of 16; head_dim = 32 = one K-step of
// v_mfma_f32_16x16x32_bf16.  S^T = K Q^T keeps one query per lane column so
// the softmax row reduction is in-lane (16 values) + 2 permlane swaps; the S^T
// accumulators feed P*V directly as the MFMA B operand (k-order permuted
// consistently, see hvk_common.h); V^T comes from LDS through
// ds_read_b64_tr_b16.  Bias (rpi gather of the CPB table) is expanded once per
// workgroup into an LDS table laid out in accumulator order; the shift mask is
// recomputed from region bits only on edge windows.
#include <stdlib.h>

#include "wmsa_common.h"

namespace {
using namespace hvk_wmsa;

constexpr int kWaves = 4;
#ifndef HVK_BWD_PF  // 1: next window's inputs loaded under phase B (see wmsa_bwd_kernel)
#define HVK_BWD_PF 1
#endif
constexpr int kThreads = 64 * kWaves;


// balanced split of the windows over the chunks of one head
__device__ __forceinline__ void chunk_range(const WmsaGeom& g, int chunk, int& w0, int& w1) {
  w0 = (int)((long long)chunk * g.n_windows / g.n_chunks);
  w1 = (int)((long long)(chunk + 1) * g.n_windows / g.n_chunks);
}

template <int WIN>
struct WinCfg {
  static constexpr int N = WIN * WIN;
  static constexpr int NT = (N + 15) / 16;
  static constexpr int NC = (NT + 1) / 2;  // 32-key chunks (one MFMA K-step each)
  static constexpr int R = 2 * WIN - 1;
  static constexpr int TAB = NT * NT * 256;  // floats in the accumulator-order bias table
  static_assert(NT <= 4, "window larger than 8 needs the streamed-key variant");
};

// Expand 16*sigmoid(cpb) [(2w-1)^2] for one head into accumulator order:
// tab[((qi*NT + ki)*64 + lane)*4 + r] = log2e * bias(q = 16qi + (lane&15), key = 16ki + 4(lane>>4) + r)
// padded keys -> -inf (P = 0), padded queries -> 0 (never stored).
template <int WIN>
__device__ void build_bias_table(float* tab, const float* __restrict__ src) {
  using K = WinCfg<WIN>;
  static_assert(K::TAB % kThreads == 0, "table is a whole number of block strides");
#pragma unroll  // all loads of the (L2-resident) source table in flight together
  for (int k = 0; k < K::TAB / kThreads; ++k) {
    const int e = threadIdx.x + k * kThreads;
    const int r = e & 3, lane = (e >> 2) & 63, blk = e >> 8;
    const int qi = blk / K::NT, ki = blk % K::NT;
    const int q = 16 * qi + (lane & 15), key = 16 * ki + 4 * (lane >> 4) + r;
    float v;
    if (key >= K::N) {
      v = -INFINITY;
    } else if (q >= K::N) {
      v = 0.f;
    } else {
      const int idx = (q / WIN - key / WIN + WIN - 1) * K::R + (q % WIN - key % WIN + WIN - 1);
      v = src[idx] * HVK_LOG2E;
    }
    tab[e] = v;
  }
}



// Region bit of a window-local coordinate in the last window row/col (swinv2.py:359-375).
template <int WIN>
__device__ __forceinline__ uint32_t key_band_bits(int g, int shift, bool rows) {
  using K = WinCfg<WIN>;
  uint32_t bits = 0;
#pragma unroll
  for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * ki + 4 * g + r;
      const int c = rows ? key / WIN : key % WIN;
      if (key < K::N && c >= WIN - shift) bits |= 1u << (ki * 4 + r);
    }
  return bits;
}

// bit (ki*4 + r) set <=> key 16ki + 4g + r lies in a different shift region than query q
__device__ __forceinline__ uint32_t mask_bits(uint32_t krow, uint32_t kcol, int q, int lim, int win,
                                              bool edge_r, bool edge_c) {
  const uint32_t qr = (q / win) >= lim ? ~0u : 0u, qc = (q % win) >= lim ? ~0u : 0u;
  return (edge_r ? (krow ^ qr) : 0u) | (edge_c ? (kcol ^ qc) : 0u);
}

// Backward P / dS images [query][key] (ROWS bf16 per row = ROWS/4 8-B units): the 8-B unit
// col8 of `row` is stored at col8 ^ f(row), f = (r0^r2) | r3<<1 | r1<<2: the 8-B writes of a
// query tile and the transposed reads of phase B are then bank-conflict free.
template <int ROWS>
__device__ __forceinline__ int pimg_off(int row, int col8) {
  const int f = ((row ^ (row >> 2)) & 1) | ((row >> 2) & 2) | ((row << 1) & 4);
  return row * ROWS + (((col8 ^ f) & (ROWS / 4 - 1)) << 2);
}

// The forward's LDS image of V keeps head_dim columns in the order
// col 16dt + 4g + r <-> d = 8g + 4dt + r, so an MFMA that reads them as A = X^T through
// ds_read_b64_tr_b16 puts d = 8g..8g+7 of one token in lane (g, token) across its two
// accumulators (dt = 0, 1): every output row segment leaves as ONE 16-B store.  The lane
// holding d = 8g..8g+7 of a token writes the two halves to cols 4g and 16 + 4g.
// The 8-B column blocks (col8 = col/4) of a 64-B row are XOR-swizzled by (row>>1)&7: the
// 16 rows of one write group then hit 32 distinct banks, and the tr-reads' row quads too.
__device__ __forceinline__ int lds_off(int row, int col8) {
  return row * 32 + ((col8 ^ ((row >> 1) & 7)) << 2);
}
__device__ __forceinline__ void lds_write_dperm(hvk_bf16* img, int row, int g, uint4 v) {
  *reinterpret_cast<uint2*>(img + lds_off(row, g)) = make_uint2(v.x, v.y);
  *reinterpret_cast<uint2*>(img + lds_off(row, 4 + g)) = make_uint2(v.z, v.w);
}
// the two accumulator quads of a lane (d = 8g + 4dt + r) as 8 packed bf16
__device__ __forceinline__ uint4 pack_dperm(const float a[4], const float b[4]) {
  return make_uint4(hvk_pack2(a[0], a[1]), hvk_pack2(a[2], a[3]), hvk_pack2(b[0], b[1]),
                    hvk_pack2(b[2], b[3]));
}


template <int WIN>
__global__ __launch_bounds__(kThreads, 4) void wmsa_fwd_kernel(FwdArgs a) {
  using K = WinCfg<WIN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int chunk, h;
  hvk_decode_chunk_head(blockIdx.x, g.nH, chunk, h);
  if (chunk >= g.n_chunks) return;
  int w0, w1;
  chunk_range(g, chunk, w0, w1);
  if (w0 >= w1) return;

  float* btab = reinterpret_cast<float*>(smem);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  hvk_bf16* vst = reinterpret_cast<hvk_bf16*>(smem + K::TAB * 4) + wave * (32 * K::NC * 32);
  build_bias_table<WIN>(btab, a.bias + (size_t)h * K::R * K::R);
  __syncthreads();

  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * g.C;
  const float sc2 = a.scale[h] * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  const uint32_t krow = g.shift ? key_band_bits<WIN>(gq, g.shift, true) : 0u;
  const uint32_t kcol = g.shift ? key_band_bits<WIN>(gq, g.shift, false) : 0u;
  const int per_img = g.nWh * g.nWw;

  for (int w = w0 + wave; w < w1; w += kWaves) {
    const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
    const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
    int row[K::NT];
    uint4 qf[K::NT], kf[K::NT], vf[K::NT];
#pragma unroll
    for (int i = 0; i < K::NT; ++i) {
      const int t = 16 * i + li;
      row[i] = window_token_row(g, b, wh, ww, WIN, t < K::N ? t : 0);
      if (t < K::N) {
        const hvk_bf16* p = a.qkv + (size_t)row[i] * C3 + h * 32 + 8 * gq;
        qf[i] = hvk_ld16(p);
        kf[i] = hvk_ld16(p + C);
        vf[i] = hvk_ld16(p + 2 * C);
      } else {
        qf[i] = kf[i] = vf[i] = make_uint4(0, 0, 0, 0);
      }
    }
#ifdef HVK_PROBE_MEMORY_ONLY  // tools/probe: same gather/scatter, no math (memory ceiling)
#pragma unroll
    for (int i = 0; i < K::NT; ++i)
      if (16 * i + li < K::N) {
        uint4 t = qf[i];
        t.x ^= kf[i].x ^ vf[i].x; t.y ^= kf[i].y ^ vf[i].y;
        t.z ^= kf[i].z ^ vf[i].z; t.w ^= kf[i].w ^ vf[i].w;
        *reinterpret_cast<uint4*>(a.out + (size_t)row[i] * C + h * 32 + 8 * gq) = t;
      }
    continue;
#endif
#pragma unroll
    for (int i = 0; i < K::NT; ++i) lds_write_dperm(vst, 16 * i + li, gq, vf[i]);  // frees vf first
    float rn;
#pragma unroll
    for (int i = 0; i < K::NT; ++i) {
      qf[i] = l2_normalize(qf[i], rn, sc2);  // q^ * scale * log2e: the MFMA applies the scale
      kf[i] = l2_normalize(kf[i], rn);
    }
#pragma unroll
    for (int i = K::NT; i < 2 * K::NC; ++i)
      *reinterpret_cast<uint4*>(vst + (16 * i + li) * 32 + 8 * gq) = make_uint4(0, 0, 0, 0);
    asm volatile("" ::: "memory");  // same-wave LDS ops complete in order: compiler fence only
    // V^T fragments (A operand of O^T = V^T P^T), key order per chunk c, lane group g, slot j:
    // key(g, j) = 32c + (j < 4 ? 4g + j : 16 + 4g + j - 4)
    uint4 vt[K::NC][2];
#pragma unroll
    for (int c = 0; c < K::NC; ++c)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int rr = 32 * c + 4 * gq + (li >> 2), c8 = 4 * dt + (li & 3);
        const uint2 lo = hvk_tr_read(vst + lds_off(rr, c8)), hi = hvk_tr_read(vst + lds_off(rr + 16, c8));
        vt[c][dt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }

#pragma unroll
    for (int qi = 0; qi < K::NT; ++qi) {
      // keep one query tile live at a time and the bias-table reads inside the loop (VGPR budget)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // S'^T = K^ (scale log2e Q^)^T + bias: the bias tile rides in as the MFMA C operand
      hvk_f32x4 s[K::NT];
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki) {
        const float4 bb = *reinterpret_cast<const float4*>(btab + ((qi * K::NT + ki) * 64 + lane) * 4);
        s[ki] = hvk_mfma16(kf[ki], qf[qi], hvk_f32x4{bb.x, bb.y, bb.z, bb.w});
      }
      const int q = 16 * qi + li;
      if (edge_r || edge_c) {  // wave-uniform: only the last window row / column carries a mask
        const uint32_t mm = mask_bits(krow, kcol, q, WIN - g.shift, WIN, edge_r, edge_c);
#pragma unroll
        for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[ki][r] += ((mm >> (ki * 4 + r)) & 1u) ? mask2 : 0.f;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[ki][r]);
      mx = hvk_group4_max(mx);
      float sum = 0.f;
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(s[ki][r] - mx);
          s[ki][r] = p;
          sum += p;
        }
      sum = hvk_group4_sum(sum);
      hvk_f32x4 o[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int c = 0; c < K::NC; ++c) {
        const hvk_f32x4 a0 = s[2 * c];
        const hvk_f32x4 a1 = (2 * c + 1 < K::NT) ? s[2 * c + 1] : hvk_f32x4{0, 0, 0, 0};
        const uint4 pf = make_uint4(hvk_pack2(a0[0], a0[1]), hvk_pack2(a0[2], a0[3]),
                                    hvk_pack2(a1[0], a1[1]), hvk_pack2(a1[2], a1[3]));
        o[0] = hvk_mfma16(vt[c][0], pf, o[0]);
        o[1] = hvk_mfma16(vt[c][1], pf, o[1]);
      }
      if (q < K::N) {
        const float inv = __builtin_amdgcn_rcpf(sum);
        const float o0[4] = {o[0][0] * inv, o[0][1] * inv, o[0][2] * inv, o[0][3] * inv};
        const float o1[4] = {o[1][0] * inv, o[1][1] * inv, o[1][2] * inv, o[1][3] * inv};
        hvk_st16(a.out + (size_t)row[qi] * C + h * 32 + 8 * gq, pack_dperm(o0, o1));
      }
    }
  }
}


// Backward, one wave per (window, head), recomputing P from q, k (no saved
// probabilities).  Phase A (query on the lane): S^T, P^T, dP^T = V dO^T,
// dS^T = P (dP - rowsum(P dP)), dQ^ = scale dS K^ (K^T via tr-reads).
// Phase B (key on the lane): dV^T = dO^T P, dK^T = Q^T (scale dS), both with
// the P / dS images staged in LDS and read transposed.
template <int WIN>
__global__ __launch_bounds__(kThreads, 1) void wmsa_bwd_kernel(BwdArgs a) {
  using K = WinCfg<WIN>;
  constexpr int ROWS = 32 * K::NC;                 // padded token rows in LDS images
  constexpr int WAVE_LDS = ROWS * 32 * 3 + ROWS * ROWS * 2;  // q^, k^, dO [ROWS][32]; P, dS [ROWS][ROWS]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int chunk, h;
  if (!decode_item(g, blockIdx.x, chunk, h)) return;
  int w0, w1;
  chunk_range(g, chunk, w0, w1);
  if (w0 >= w1) return;

  float* btab = reinterpret_cast<float*>(smem);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  hvk_bf16* qs = reinterpret_cast<hvk_bf16*>(smem + K::TAB * 4) + wave * WAVE_LDS;
  hvk_bf16* ks = qs + ROWS * 32;
  hvk_bf16* dos = ks + ROWS * 32;
  hvk_bf16* ps = dos + ROWS * 32;
  hvk_bf16* dss = ps + ROWS * ROWS;
  build_bias_table<WIN>(btab, a.bias + (size_t)h * K::R * K::R);
  // zero the padded rows of the staged images once (never rewritten)
  for (int e = lane; e < ROWS * 32 * 3 + ROWS * ROWS * 2; e += 64) qs[e] = 0;
  __syncthreads();

  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * g.C;
  const float scale = a.scale[h];
  const float sc2 = scale * HVK_LOG2E;
  const float mask2 = -100.f * HVK_LOG2E;
  const uint32_t krow = g.shift ? key_band_bits<WIN>(gq, g.shift, true) : 0u;
  const uint32_t kcol = g.shift ? key_band_bits<WIN>(gq, g.shift, false) : 0u;
  const int per_img = g.nWh * g.nWw;

  hvk_f32x4 dbias[K::NT][K::NT];
#pragma unroll
  for (int qi = 0; qi < K::NT; ++qi)
#pragma unroll
    for (int ki = 0; ki < K::NT; ++ki) dbias[qi][ki] = hvk_f32x4{0, 0, 0, 0};
  float dscale = 0.f;
  float dqb[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};  // this lane's column sums of dq

  // q, k, v, dO of a window into registers.  HVK_BWD_PF: the next window's loads are issued
  // right after phase A, into the registers phase A was the last to read (phase B works from
  // the LDS images), so their latency hides under phase B instead of stalling the next window
  int nrow[K::NT];
  uint4 qf[K::NT], kf[K::NT], vf[K::NT], df[K::NT];
  auto load_window = [&](int w) {
    const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
#pragma unroll
    for (int i = 0; i < K::NT; ++i) {
      const int t = 16 * i + li;
      nrow[i] = window_token_row(g, b, wh, ww, WIN, t < K::N ? t : 0);
      if (t < K::N) {
        const hvk_bf16* p = a.qkv + (size_t)nrow[i] * C3 + h * 32 + 8 * gq;
        if (HVK_NT_SAVED & 32) {  // the last read of qkv and of dO
          qf[i] = hvk_ld16_nt(p);
          kf[i] = hvk_ld16_nt(p + C);
          vf[i] = hvk_ld16_nt(p + 2 * C);
          df[i] = hvk_ld16_nt(a.dout + (size_t)nrow[i] * C + h * 32 + 8 * gq);
        } else {
          qf[i] = hvk_ld16(p);
          kf[i] = hvk_ld16(p + C);
          vf[i] = hvk_ld16(p + 2 * C);
          df[i] = hvk_ld16(a.dout + (size_t)nrow[i] * C + h * 32 + 8 * gq);
        }
      } else {
        qf[i] = kf[i] = vf[i] = df[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  if (HVK_BWD_PF && w0 + wave < w1) load_window(w0 + wave);

  for (int w = w0 + wave; w < w1; w += kWaves) {
    const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
    const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
    (void)b;
    if (!HVK_BWD_PF) load_window(w);
    int row[K::NT];
#pragma unroll
    for (int i = 0; i < K::NT; ++i) row[i] = nrow[i];
    float rnq[K::NT], rnk[K::NT];
#pragma unroll
    for (int i = 0; i < K::NT; ++i) {
      qf[i] = l2_normalize(qf[i], rnq[i]);
      kf[i] = l2_normalize(kf[i], rnk[i]);
      const int o16 = fm16(16 * i + li, gq) >> 1;  // bf16 elements
      *reinterpret_cast<uint4*>(qs + o16) = qf[i];
      *reinterpret_cast<uint4*>(ks + o16) = kf[i];
      *reinterpret_cast<uint4*>(dos + o16) = df[i];
    }
    asm volatile("" ::: "memory");  // same-wave LDS ops complete in order: compiler fence only
    // K^T fragments for dQ^T = K^T dS^T (k = key, permuted order as in the forward)
    uint4 kt_frag[K::NC][2];
#pragma unroll
    for (int c = 0; c < K::NC; ++c)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int rr = 32 * c + 4 * gq + (li >> 2), c8 = 4 * dt + (li & 3);
        const uint2 lo = hvk_tr_read(ks + (fm8(rr, c8) >> 1)), hi = hvk_tr_read(ks + (fm8(rr + 16, c8) >> 1));
        kt_frag[c][dt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }

    // ---------------- phase A: one query tile at a time, query on the lane
#pragma unroll
    for (int qi = 0; qi < K::NT; ++qi) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      hvk_f32x4 s[K::NT], dp[K::NT];
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki) {
        s[ki] = hvk_mfma16(kf[ki], qf[qi], hvk_f32x4{0, 0, 0, 0});   // cos(q, k)
        dp[ki] = hvk_mfma16(vf[ki], df[qi], hvk_f32x4{0, 0, 0, 0});  // dO . V
      }
      const int q = 16 * qi + li;
      float p[K::NT][4];
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki) {
        const float4 bb = *reinterpret_cast<const float4*>(btab + ((qi * K::NT + ki) * 64 + lane) * 4);
        p[ki][0] = s[ki][0] * sc2 + bb.x;
        p[ki][1] = s[ki][1] * sc2 + bb.y;
        p[ki][2] = s[ki][2] * sc2 + bb.z;
        p[ki][3] = s[ki][3] * sc2 + bb.w;
      }
      if (edge_r || edge_c) {
        const uint32_t mm = mask_bits(krow, kcol, q, WIN - g.shift, WIN, edge_r, edge_c);
#pragma unroll
        for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
          for (int r = 0; r < 4; ++r) p[ki][r] += ((mm >> (ki * 4 + r)) & 1u) ? mask2 : 0.f;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, p[ki][r]);
      mx = hvk_group4_max(mx);
      float sum = 0.f;
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[ki][r] = __builtin_amdgcn_exp2f(p[ki][r] - mx);
          sum += p[ki][r];
        }
      sum = hvk_group4_sum(sum);
      const float inv = __builtin_amdgcn_rcpf(sum);
      float delta = 0.f;
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[ki][r] *= inv;
          delta += p[ki][r] * dp[ki][r];
        }
      delta = hvk_group4_sum(delta);
      float ds[K::NT][4];
#pragma unroll
      for (int ki = 0; ki < K::NT; ++ki) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ds[ki][r] = p[ki][r] * (dp[ki][r] - delta);
          dbias[qi][ki][r] += ds[ki][r];
          dscale += ds[ki][r] * s[ki][r];
        }
        // stage P and scale*dS as [query][key] rows for phase B
        const int off = pimg_off<ROWS>(q, 4 * ki + gq);
        *reinterpret_cast<uint2*>(ps + off) =
            make_uint2(hvk_pack2(p[ki][0], p[ki][1]), hvk_pack2(p[ki][2], p[ki][3]));
        *reinterpret_cast<uint2*>(dss + off) =
            make_uint2(hvk_pack2(scale * ds[ki][0], scale * ds[ki][1]),
                       hvk_pack2(scale * ds[ki][2], scale * ds[ki][3]));
      }
      // dQ^T = K^T (scale dS^T)
      hvk_f32x4 dq[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int c = 0; c < K::NC; ++c) {
        const bool has1 = 2 * c + 1 < K::NT;
        const uint4 bf = make_uint4(
            hvk_pack2(scale * ds[2 * c][0], scale * ds[2 * c][1]),
            hvk_pack2(scale * ds[2 * c][2], scale * ds[2 * c][3]),
            has1 ? hvk_pack2(scale * ds[2 * c + 1][0], scale * ds[2 * c + 1][1]) : 0u,
            has1 ? hvk_pack2(scale * ds[2 * c + 1][2], scale * ds[2 * c + 1][3]) : 0u);
        dq[0] = hvk_mfma16(kt_frag[c][0], bf, dq[0]);
        dq[1] = hvk_mfma16(kt_frag[c][1], bf, dq[1]);
      }
      // normalize backward: dq = (dq^ - q^ (q^ . dq^)) / max(||q||, eps)
      float qh[2][4], dot = 0.f;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint2 v = *reinterpret_cast<const uint2*>(qs + (fm8(q, 4 * dt + gq) >> 1));
        qh[dt][0] = hvk_lo(v.x); qh[dt][1] = hvk_hi(v.x);
        qh[dt][2] = hvk_lo(v.y); qh[dt][3] = hvk_hi(v.y);
#pragma unroll
        for (int r = 0; r < 4; ++r) dot += qh[dt][r] * dq[dt][r];
      }
      dot = hvk_group4_sum(dot);
      if (rnq[qi] >= 1e12f) dot = 0.f;  // ||q|| <= eps: x / eps, no projection term
      {
        uint2 pk[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = (dq[dt][r] - qh[dt][r] * dot) * rnq[qi];
            if (q < K::N) dqb[dt][r] += v[r];
          }
          pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
        }
        const uint4 o = hvk_pair_swap(pk[0], pk[1]);  // all lanes: cross-lane
        if (q < K::N) hvk_st16(a.dqkv + (size_t)row[qi] * C3 + h * 32 + hvk_pair_col(gq), o);
      }
    }
    asm volatile("" ::: "memory");  // same-wave LDS ops complete in order: compiler fence only
    if (HVK_BWD_PF && w + kWaves < w1) load_window(w + kWaves);

    // ---------------- phase B: one key tile at a time, key on the lane
    // query chunk c, slot (g, j): q(g, j) = 32c + (j < 4 ? 4g + j : 16 + 4g + j - 4)
#pragma unroll
    for (int kt = 0; kt < K::NT; ++kt) {
      hvk_f32x4 dv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, dk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int c = 0; c < K::NC; ++c) {
        const int rq = 32 * c + 4 * gq + (li >> 2);
        const int plo = pimg_off<ROWS>(rq, 4 * kt + (li & 3)), phi = pimg_off<ROWS>(rq + 16, 4 * kt + (li & 3));
        uint2 lo = hvk_tr_read(ps + plo), hi = hvk_tr_read(ps + phi);
        const uint4 pfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
        lo = hvk_tr_read(dss + plo); hi = hvk_tr_read(dss + phi);
        const uint4 dsfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int c8 = 4 * dt + (li & 3);
          const int olo = fm8(rq, c8) >> 1, ohi = fm8(rq + 16, c8) >> 1;
          lo = hvk_tr_read(dos + olo); hi = hvk_tr_read(dos + ohi);
          dv[dt] = hvk_mfma16(make_uint4(lo.x, lo.y, hi.x, hi.y), pfr, dv[dt]);
          lo = hvk_tr_read(qs + olo); hi = hvk_tr_read(qs + ohi);
          dk[dt] = hvk_mfma16(make_uint4(lo.x, lo.y, hi.x, hi.y), dsfr, dk[dt]);
        }
      }
      const int key = 16 * kt + li;
      float kh[2][4], dot = 0.f;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint2 v = *reinterpret_cast<const uint2*>(ks + (fm8(key, 4 * dt + gq) >> 1));
        kh[dt][0] = hvk_lo(v.x); kh[dt][1] = hvk_hi(v.x);
        kh[dt][2] = hvk_lo(v.y); kh[dt][3] = hvk_hi(v.y);
#pragma unroll
        for (int r = 0; r < 4; ++r) dot += kh[dt][r] * dk[dt][r];
      }
      dot = hvk_group4_sum(dot);
      if (rnk[kt] >= 1e12f) dot = 0.f;
      {
        uint2 pk[2], pv[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (dk[dt][r] - kh[dt][r] * dot) * rnk[kt];
          pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
          pv[dt] = make_uint2(hvk_pack2(dv[dt][0], dv[dt][1]), hvk_pack2(dv[dt][2], dv[dt][3]));
        }
        const uint4 ok = hvk_pair_swap(pk[0], pk[1]), ov = hvk_pair_swap(pv[0], pv[1]);
        if (key < K::N) {
          hvk_bf16* dst = a.dqkv + (size_t)row[kt] * C3 + h * 32 + hvk_pair_col(gq);
          hvk_st16(dst + C, ok);
          hvk_st16(dst + 2 * C, ov);
        }
      }
    }
    asm volatile("" ::: "memory");  // same-wave LDS ops complete in order: compiler fence only
  }

  // ---- workgroup reduction of the bias / scale gradients, then one atomic per entry
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem + K::TAB * 4) + wave * K::TAB;  // reuses staging
  static_assert(K::TAB * 4 <= WAVE_LDS * 2, "reduction buffer must fit in the wave's staging");
#pragma unroll
  for (int qi = 0; qi < K::NT; ++qi)
#pragma unroll
    for (int ki = 0; ki < K::NT; ++ki)
      *reinterpret_cast<float4*>(red + ((qi * K::NT + ki) * 64 + lane) * 4) =
          make_float4(dbias[qi][ki][0], dbias[qi][ki][1], dbias[qi][ki][2], dbias[qi][ki][3]);
  __syncthreads();
  const float* red0 = reinterpret_cast<const float*>(smem + K::TAB * 4);
  float* dst = a.dbias_acc + (size_t)h * K::TAB;
  for (int e = threadIdx.x; e < K::TAB; e += kThreads) {
    float v = 0.f;
#pragma unroll
    for (int wv = 0; wv < kWaves; ++wv) v += red0[wv * K::TAB + e];
    atomicAdd(dst + e, v);
  }
  dscale = hvk_wave_sum(dscale);
  if (lane == 0) atomicAdd(a.dscale_acc + h, dscale);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = hvk_row16_sum(dqb[dt][r]);
      if (li == 0) atomicAdd(a.dqb_acc + h * 32 + 16 * dt + 4 * gq + r, v);
    }
}

// Fold the accumulator-order partial sums into the CPB-table gradient [nH, R*R], write
// dscale / dq_bias, and leave the workspace zero for the next call.
template <int WIN>
__global__ __launch_bounds__(256) void wmsa_finalize_kernel(BwdArgs a, float* __restrict__ dtab,
                                                            float* __restrict__ dscale,
                                                            float* __restrict__ dqb) {
  using K = WinCfg<WIN>;
  __shared__ float bins[K::R * K::R];
  const int h = blockIdx.x;
  for (int i = threadIdx.x; i < K::R * K::R; i += blockDim.x) bins[i] = 0.f;
  __syncthreads();
  float* acc = a.dbias_acc + (size_t)h * K::TAB;
  for (int e = threadIdx.x; e < K::TAB; e += blockDim.x) {
    const int r = e & 3, lane = (e >> 2) & 63, blk = e >> 8;
    const int qi = blk / K::NT, ki = blk % K::NT;
    const int q = 16 * qi + (lane & 15), key = 16 * ki + 4 * (lane >> 4) + r;
    if (q < K::N && key < K::N) {
      const int idx = (q / WIN - key / WIN + WIN - 1) * K::R + (q % WIN - key % WIN + WIN - 1);
      atomicAdd(&bins[idx], acc[e]);
    }
    acc[e] = 0.f;
  }
  finalize_scale_qb(a.dscale_acc, a.dqb_acc, dscale, dqb, h);
  __syncthreads();
  for (int i = threadIdx.x; i < K::R * K::R; i += blockDim.x) dtab[(size_t)h * K::R * K::R + i] = bins[i];
}

template <int WIN>
constexpr size_t fwd_lds_bytes() {
  return WinCfg<WIN>::TAB * 4 + kWaves * (32 * WinCfg<WIN>::NC * 32) * 2;
}
template <int WIN>
constexpr size_t bwd_lds_bytes() {
  constexpr int ROWS = 32 * WinCfg<WIN>::NC;
  return WinCfg<WIN>::TAB * 4 + kWaves * (size_t)(ROWS * 32 * 3 + ROWS * ROWS * 2) * 2;
}


template <int WIN>
int launch_fwd(const FwdArgs& a, hipStream_t st) {
  const int padded = a.g.n_chunks;  // already a multiple of 8
  const size_t lds = fwd_lds_bytes<WIN>();
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_FWD, wmsa_fwd_kernel<WIN>, dim3(padded * a.g.nH), dim3(kThreads), lds, st, a);
  HVK_CHECK_LAUNCH("wmsa_fwd");
  return HVK_OK;
}

template <int WIN>
int launch_bwd(const BwdArgs& a, float* dbias_table, float* dscale, float* dqb, hipStream_t st) {
  const int items = a.g.n_chunks * a.g.nH;
  const int nblk = a.g.xcd_runs ? 8 * ((items + 7) / 8) : (a.g.n_chunks + 7) / 8 * 8 * a.g.nH;
  const size_t lds = bwd_lds_bytes<WIN>();
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_kernel<WIN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, wmsa_bwd_kernel<WIN>, dim3(nblk), dim3(kThreads), lds, st, a);
  HVK_CHECK_LAUNCH("wmsa_bwd");
  hipLaunchKernelGGL(wmsa_finalize_kernel<WIN>, dim3(a.g.nH), dim3(256), 0, st, a, dbias_table,
                     dscale, dqb);
  HVK_CHECK_LAUNCH("wmsa_finalize");
  return HVK_OK;
}

}  // namespace

extern "C" {

size_t hvk_wmsa_bwd_workspace_bytes(int num_heads, int window) {
  // [dbias accumulators][dscale nH][dq_bias 32 nH] floats
  size_t acc;
  if (hvk_wmsa::large_window(window)) {
    acc = hvk_wmsa::large_acc_floats(num_heads, window);
  } else {
    const int n = window * window, nt = (n + 15) / 16;
    acc = (size_t)num_heads * nt * nt * 256;
  }
  return (acc + (size_t)num_heads * 33) * sizeof(float);
}

int hvk_wmsa_fwd(const void* qkv, void* out, float* lse, const float* bias_table, const float* scale,
                 int B, int H, int W, int C, int num_heads, int window, int shift,
                 void* stream) {
  if (!qkv || !out || !bias_table || !scale)
    return hvk_set_error(HVK_EINVAL, "hvk_wmsa_fwd: null pointer");
  FwdArgs a;
  a.qkv = static_cast<const hvk_bf16*>(qkv);
  a.out = static_cast<hvk_bf16*>(out);
  a.bias = bias_table;
  a.scale = scale;
  a.lse = lse;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hvk_wmsa::large_window(window)) {
    int rc = make_geom(B, H, W, C, num_heads, window, shift, 256 * 4, a.g);
    if (rc) return rc;
    return hvk_wmsa::large_fwd(a, window, st);
  }
  if (window != 4 && window != 6 && window != 7 && window != 8)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_fwd: window %d not built (4,6,7,8,12,16,24)", window);
  // HVK_WMSA_FWD_V1=1: the round-1 wave-per-(window, head) kernel (A/B timing only)
  static const bool v1 = [] {
    const char* e = getenv("HVK_WMSA_FWD_V1");
    return e && atoi(e) > 0;
  }();
  if (!v1 || lse) return hvk_wmsa::ring_fwd(a, B, H, W, C, num_heads, window, shift, st);
  int rc = make_geom(B, H, W, C, num_heads, window, shift, 256 * 4, a.g);
  if (rc) return rc;
  switch (window) {
    case 7: return launch_fwd<7>(a, st);
    case 8: return launch_fwd<8>(a, st);
    case 6: return launch_fwd<6>(a, st);
    default: return launch_fwd<4>(a, st);
  }
}

int hvk_wmsa_bwd(const void* qkv, const void* dout, const void* out, const float* lse, void* dqkv,
                 float* dq_bias, const float* bias_table, const float* scale,
                 float* dbias_table, float* dscale, float* workspace, size_t workspace_bytes,
                 int B, int H, int W, int C, int num_heads, int window, int shift,
                 void* stream) {
  if (!qkv || !dout || !dqkv || !bias_table || !scale || !dbias_table || !dscale || !workspace)
    return hvk_set_error(HVK_EINVAL, "hvk_wmsa_bwd: null pointer");
  if (lse && !out) return hvk_set_error(HVK_EINVAL, "hvk_wmsa_bwd: lse given without the forward's output");
  if (workspace_bytes < hvk_wmsa_bwd_workspace_bytes(num_heads, window))
    return hvk_set_error(HVK_EINVAL, "hvk_wmsa_bwd: workspace too small");
  BwdArgs a;
  a.qkv = static_cast<const hvk_bf16*>(qkv);
  a.dout = static_cast<const hvk_bf16*>(dout);
  a.dqkv = static_cast<hvk_bf16*>(dqkv);
  a.out = static_cast<const hvk_bf16*>(out);
  a.lse = lse;
  a.bias = bias_table;
  a.scale = scale;
  const size_t ws_acc = hvk_wmsa_bwd_workspace_bytes(num_heads, window) / sizeof(float) -
                        (size_t)num_heads * 33;
  a.dbias_acc = workspace;
  a.dscale_acc = workspace + ws_acc;
  a.dqb_acc = a.dscale_acc + num_heads;
  // one resident 4-wave workgroup per CU (128 KB LDS, 1 wave/SIMD)
  int rc = make_geom(B, H, W, C, num_heads, window, shift, 256, a.g);
  if (rc) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hvk_wmsa::large_window(window))
    return hvk_wmsa::large_bwd(a, window, dbias_table, dscale, dq_bias, st);
  // windows <= 8 always recompute the row constants (exact delta = sum P dP); out / lse unused
  // fill all 256 CUs: 256 / nH chunks, not rounded down to a multiple of 8 (at 12 and 24 heads
  // the rounding left 64 CUs idle), the (chunk, head) items dealt to the XCDs in runs of at
  // most 32 (one resident workgroup per CU of each XCD)
  static const bool fill = [] {
    const char* e = getenv("HVK_WMSA_BWD_FILL");
    return !e || atoi(e) != 0;
  }();
  if (fill) {
    int c = 256 / num_heads;
    if (c < 1) c = 1;
    a.g.n_chunks = c < a.g.n_windows ? c : a.g.n_windows;
    a.g.xcd_runs = 1;
  }
  switch (window) {
    case 7: return launch_bwd<7>(a, dbias_table, dscale, dq_bias, st);
    case 8: return launch_bwd<8>(a, dbias_table, dscale, dq_bias, st);
    case 6: return launch_bwd<6>(a, dbias_table, dscale, dq_bias, st);
    case 4: return launch_bwd<4>(a, dbias_table, dscale, dq_bias, st);
    default:
      return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_bwd: window %d not built (4,6,7,8,12,16,24)", window);
  }
}

}  // extern "C"
