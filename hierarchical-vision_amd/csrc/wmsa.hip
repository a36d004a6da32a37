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
#include <string.h>

#include "wmsa_common.h"

namespace {
using namespace hvk_wmsa;

constexpr int kWaves = 4;
#ifndef HVK_BWD_PROBE  // tools/ timing probes of the w <= 8 backward (results wrong when set)
#define HVK_BWD_PROBE 0
#endif
#ifndef HVK_BWD_EARLY  // 1: the next window's own q / k / dO rows issued at the top (A/B build switch)
#define HVK_BWD_EARLY 1
#endif
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
// col8 of `row` is stored at col8 ^ pswz(row), pswz a bijection of the row's low 4 bits with
// bits 3:2 = (row >> 1) & 3 and bits 1:0 = (row >> 3 & 1, row & 1).  Under the LDS bank model
// (MI355X_MICROARCH.md §LDS): phase A's ds_write_b64 (16 lanes = the 16 rows of a query tile, one
// unit each, banks mod 32 = one 128-B row) needs 16 distinct units per tile -> a bijection; phase
// B's transposed reads (32 lanes = rows 4gq + li/4 of one 8-row block x units 4kt + li%4, banks
// mod 64 = two rows) need bits 3:2 distinct over the 4 rows of one parity.  The 3-bit form of
// round 3 left both 2-way (≈25 % of the kernel's LDS cycles, matching SQ_LDS_BANK_CONFLICT).
__device__ __forceinline__ int pswz(int row) {
  return (((row >> 1) & 3) << 2) | (((row >> 3) & 1) << 1) | (row & 1);
}

// ---------------------------------------------------------------------------------------------
// Backward, two waves per (window, head) -- a "pair" -- two pairs per 4-wave workgroup, two
// workgroups per CU: 2 waves per SIMD (<= 256 VGPRs, 72 KB LDS per workgroup), so one wave's
// MFMA / LDS / exp latency hides under the other's issue, where the one-wave-per-(window,
// head) kernel of round 2 (408 VGPRs, 1 wave per SIMD; removed in round 4) stalled on every dependency.
// Wave hf of a pair owns tiles t = hf + 2j: its query tiles in phase A and its key tiles in
// phase B.  Per window: own q, k, dO tiles + all V tiles -> registers; q^, k^, dO images of
// the own rows -> LDS; barrier; all K^ tiles back from LDS; phase A (own query tiles) writes
// the own rows of the P / scale*dS images; barrier; phase B (own key tiles) reads all rows.
// Softmax against the head bound M = sc2 + max(bias) folded into the table (no row max;
// rows whose sum underflows -- a zero query vector -- take the exact-max slow path), and
// every dS is carried as scale*dS (the dbias / dscale sums are divided by scale once).
template <int WIN>
struct PairCfg {
  using K = WinCfg<WIN>;
  static constexpr int TPW = (K::NT + 1) / 2;                 // tiles per wave
  static constexpr int ROWS = 32 * K::NC;                     // padded token rows in LDS images
  static constexpr int PAIR_LDS = ROWS * 32 * 3 + ROWS * ROWS * 2;  // bf16: q^, k^, dO; P, dS
  static constexpr size_t LDS = K::TAB * 4 + 16 + 2 * (size_t)PAIR_LDS * 2;
  static_assert(K::TAB * 4 <= PAIR_LDS * 2, "the dbias reduction reuses one pair's images");
};

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
  return v;
}

// build_bias_table with the head bound folded in: tab = bias*log2e - M for real (query, key)
// pairs, M = sc2 + max bias*log2e over the head (cos <= 1, so every logit - M <= ~0);
// padded keys -inf, padded queries 0.  Ends with a workgroup barrier.
template <int WIN>
__device__ void build_bounded_table(float* tab, float* wmax, const float* __restrict__ src, float sc2) {
  using K = WinCfg<WIN>;
  constexpr int PER = K::TAB / kThreads;
  float v[PER];
  bool real[PER];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = threadIdx.x + k * kThreads;
    const int r = e & 3, lane = (e >> 2) & 63, blk = e >> 8;
    const int qi = blk / K::NT, ki = blk % K::NT;
    const int q = 16 * qi + (lane & 15), key = 16 * ki + 4 * (lane >> 4) + r;
    real[k] = q < K::N && key < K::N;
    // every load unconditional (a padding entry reads entry 0 and discards it): behind a branch
    // each of the PER loads waited for itself, PER global-load latencies per workgroup setup
    const int si = real[k] ? (q / WIN - key / WIN + WIN - 1) * K::R + (q % WIN - key % WIN + WIN - 1) : 0;
    v[k] = src[si];
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = threadIdx.x + k * kThreads;
    const int r = e & 3, lane = (e >> 2) & 63, blk = e >> 8;
    const int ki = blk % K::NT;
    const int key = 16 * ki + 4 * (lane >> 4) + r;
    if (real[k]) {
      v[k] *= HVK_LOG2E;
      mx = fmaxf(mx, v[k]);
    } else {
      v[k] = key >= K::N ? -INFINITY : 0.f;
    }
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  const float M = sc2 + fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
#pragma unroll
  for (int k = 0; k < PER; ++k) tab[threadIdx.x + k * kThreads] = real[k] ? v[k] - M : v[k];
  __syncthreads();
}

#ifdef HVK_STAMPS
// diagnostic build (tools/bwd_stamps.py): per-phase shader-clock sums over all waves
// [0..6] window-loop phases, [7] waves, [8] setup (entry -> loop), [9] teardown (loop -> exit;
// includes draining the phase stamps' own contended atomics), [10] / [11] unused (per-XCD clocks)
__device__ unsigned long long g_bwd_stamps[12];
#define BSTAMP(k)                                             \
  do {                                                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - st_prev;                                \
    st_prev = t_;                                             \
  } while (0)
#else
#define BSTAMP(k) \
  do {            \
  } while (0)
#endif

template <int WIN, bool QNT, bool NORMED>
__global__ __launch_bounds__(kThreads, 2) void wmsa_bwd_pair_kernel(BwdArgs a) {
  using K = WinCfg<WIN>;
  using PC = PairCfg<WIN>;
  constexpr int ROWS = PC::ROWS, TPW = PC::TPW, NT = K::NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WmsaGeom& g = a.g;
  int chunk, h;
  if (!decode_item(g, blockIdx.x, chunk, h)) return;
  int w0, w1;
  chunk_range(g, chunk, w0, w1);
  if (w0 >= w1) return;
#ifdef HVK_STAMPS
  const unsigned long long st_entry = __builtin_amdgcn_s_memtime();
#endif

  // wave-uniform in SGPRs: the window index, its coordinates and edge flags stay scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int pair = wave >> 1, hf = wave & 1;
  float* btab = reinterpret_cast<float*>(smem);
  hvk_bf16* const img0 = reinterpret_cast<hvk_bf16*>(smem + K::TAB * 4 + 16);
  hvk_bf16* qs = img0 + pair * PC::PAIR_LDS;
  hvk_bf16* ks = qs + ROWS * 32;
  hvk_bf16* dos = ks + ROWS * 32;
  hvk_bf16* ps = dos + ROWS * 32;
  hvk_bf16* dss = ps + ROWS * ROWS;
  // zero the padded rows of the images once (never rewritten)
  for (int e = threadIdx.x; e < 2 * PC::PAIR_LDS; e += kThreads) img0[e] = 0;
  const float scale = a.scale[h];
  const float sc2 = scale * HVK_LOG2E;
  // uniform: kept in an SGPR (readfirstlane), not a VGPR of this 256-VGPR kernel
  const float inv_sc2 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(1.f / sc2)));
  build_bounded_table<WIN>(btab, btab + K::TAB, a.bias + (size_t)h * K::R * K::R, sc2);

  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * g.C;
  const float mask2 = -100.f * HVK_LOG2E;
  const uint32_t krow = g.shift ? key_band_bits<WIN>(gq, g.shift, true) : 0u;
  const uint32_t kcol = g.shift ? key_band_bits<WIN>(gq, g.shift, false) : 0u;
  const int per_img = g.nWh * g.nWw;
  // buffer descriptors (launch_bwd splits the batch so each tensor spans < 2^31 bytes):
  // padded tokens read zeros and drop their stores without a branch
  const size_t T = (size_t)g.B * g.H * g.W;
  const auto r_qkv = hvk_rsrc(a.qkv, T * C3 * 2), r_dout = hvk_rsrc(a.dout, T * C * 2);
  const auto r_dqkv = hvk_rsrc(a.dqkv, T * C3 * 2);
  // NORMED: q^, k^ and their 1/||x|| (a.rn) from the qkv GEMM's epilogue (a compile-time form:
  // a runtime branch around the rn loads left the compiler's wait counts conservative)
  constexpr bool normed = NORMED;
  const auto r_rn = hvk_rsrc(a.rn, normed ? T * 2 * g.nH * 4 : 0);
  // LDS byte offsets as one per-lane base + compile-time immediates (tile t of a 16-row image
  // = +1024 B; 8-B unit 4dt + u = +512 dt B): few live address registers, no spills
  const char* const qsb = reinterpret_cast<const char*>(qs);
  const char* const ksb = reinterpret_cast<const char*>(ks);
  const char* const dob = reinterpret_cast<const char*>(dos);
  const int o_row = fm16(li, gq);                       // 16-B unit gq of token row li
  const int o_r8 = fm8(li, gq);                         // 8-B unit gq of token row li
  const int o_kt = fm8(4 * gq + (li >> 2), li & 3);     // tr-read of rows 4gq + li/4, unit li&3
  // P / dS images: row q = 16qi + li, 8-B unit 4ki + gq stored at unit (4ki + gq) ^ pswz(li)
  // = 4ki ^ (gq ^ pswz(li)): byte offset (row base | unit) ^ 32 ki, the row base a multiple of
  // the row's bytes (one register; one v_xor per write)
  const int o_pw = li * ROWS * 2 + (((gq ^ pswz(li)) & (ROWS / 4 - 1)) << 3);
  // phase B transposed reads: row rq = 4gq + li/4 (+16m + 32c), unit 4kt + (li&3)
  const int rq0 = 4 * gq + (li >> 2);
  const int frq = pswz(rq0);
  const int o_trq = fm8(rq0, li & 3);

  hvk_f32x4 dbias[TPW][NT];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int ki = 0; ki < NT; ++ki) dbias[j][ki] = hvk_f32x4{0, 0, 0, 0};
  float dscale = 0.f;
  float dqb[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};

  // own q, k, dO tiles and all V tiles of a window -> registers.  HVK_BWD_EARLY: the next
  // window's own q, k, dO rows are issued at the top, right after this window's were written to
  // the LDS images (phase A reads its q / dO fragments back from there), so they land under
  // phases A and B; its V tiles, which phase A reads from registers, after phase A.
  // qkv reads (the saved activation, read once here): nontemporal when QNT, so a qkv larger
  // than the Infinity Cache does not evict dO and the dqkv this kernel writes for the next GEMMs
  auto qld = [&](uint32_t off) { return QNT ? hvk_bld16_nt(r_qkv, off) : hvk_bld16(r_qkv, off); };
  uint4 qf[TPW], kf[TPW], df[TPW], vf[NT];
  int rown[TPW];  // own token rows of the next window, -1 = padding
  // token rows of window w, recomputed per load (not hoisted into registers that would spill: a
  // spill reload would wait (vmcnt) for every store left in flight).  The lane's window-local
  // (row, column) of tile t sits in byte t of tyx (0xFF: padding), so a row is the window's
  // scalar origin + ty W + tx, less H W / W where the cyclic shift wraps it (window_token_row's
  // arithmetic without its per-tile divisions: ~20 VALU per tile before)
  uint32_t tyx = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tok = 16 * t + li;
    tyx |= (tok < K::N ? (uint32_t)((tok / WIN) | ((tok % WIN) << 4)) : 0xFFu) << (8 * t);
  }
  auto token_rows = [&](int w, int (&rt)[NT]) {
    const int b = w / per_img, rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
    const int y0 = wh * WIN + g.shift, x0 = ww * WIN + g.shift;
    const int base = (b * g.H + y0) * g.W + x0, yl = g.H - y0, xl = g.W - x0, hw = g.H * g.W;
    uint32_t e4 = tyx;
    asm volatile("" : "+v"(e4));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const uint32_t e = (e4 >> (8 * t)) & 0xFFu;
      const int ty = (int)(e & 15u), tx = (int)(e >> 4);
      int r = base + ty * g.W + tx;
      r -= ty >= yl ? hw : 0;
      r -= tx >= xl ? g.W : 0;
      rt[t] = e == 0xFFu ? -1 : (int)HVK_BCHECK(r, (long long)g.B * hw);
    }
  };
  auto load_tiles = [&](int w) {
    int rt[NT];
    token_rows(w, rt);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      rown[j] = 2 * j + 1 < NT ? (hf ? rt[2 * j + 1] : rt[2 * j]) : (hf ? -1 : rt[2 * j]);
      const uint32_t o = rown[j] < 0 ? HVK_OOB : (uint32_t)(rown[j] * C3 + h * 32 + 8 * gq) * 2;
      const uint32_t od = rown[j] < 0 ? HVK_OOB : (uint32_t)(rown[j] * C + h * 32 + 8 * gq) * 2;
      qf[j] = qld(o);
      kf[j] = qld(o + 2 * C);
      df[j] = hvk_bld16(r_dout, od);
    }
  };
  auto load_v = [&](int w) {
    int rt[NT];
    token_rows(w, rt);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      vf[t] = qld(rt[t] < 0 ? HVK_OOB : (uint32_t)(rt[t] * C3 + 2 * C + h * 32 + 8 * gq) * 2);
  };
  // every wave runs the same number of iterations (the barriers are workgroup-wide); a pair
  // without a window in the last one only joins the barriers
  const int n_iter = (w1 - w0 + 1) / 2;
  if (w0 + pair < w1) {
    load_v(w0 + pair);
    load_tiles(w0 + pair);
  }
  // phase B's dK / dV stores leave at the top of the NEXT iteration, after the waits for the
  // prefetched loads: in flight behind those loads they would be drained by the waits
  // (vmcnt counts loads and stores in issue order)
  uint4 st_k[TPW], st_v[TPW];
  uint32_t st_off[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    st_k[j] = st_v[j] = make_uint4(0, 0, 0, 0);
    st_off[j] = HVK_OOB;
  }
#ifdef HVK_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_prev = __builtin_amdgcn_s_memtime();
  const unsigned long long st_acc_setup = st_prev - st_entry;
#endif

  for (int it = 0; it < n_iter; ++it) {
    const int w = w0 + 2 * it + pair;
    const bool act = w < w1;
    const int rem = w % per_img, wh = rem / g.nWw, ww = rem % g.nWw;
    const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
    int row[TPW];
    float rnq[TPW], rnk[TPW];
    if constexpr (normed) {  // first used after phase A: issued here, ahead of the dK / dV stores below
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const uint32_t orn = rown[j] < 0 ? HVK_OOB : (uint32_t)(rown[j] * 2 * g.nH + h) * 4;
        rnq[j] = hvk_bld4f(r_rn, orn);
        rnk[j] = hvk_bld4f(r_rn, orn + 4 * g.nH);
      }
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      row[j] = rown[j];
      const int t = hf + 2 * j;
      if (act && t < NT) {
        if constexpr (!normed) {
          qf[j] = l2_normalize(qf[j], rnq[j]);
          kf[j] = l2_normalize(kf[j], rnk[j]);
        }
        const int o16 = o_row + 1024 * t;
        *reinterpret_cast<uint4*>((char*)qsb + o16) = qf[j];
        *reinterpret_cast<uint4*>((char*)ksb + o16) = kf[j];
        *reinterpret_cast<uint4*>((char*)dob + o16) = df[j];
      }
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      hvk_bst16(r_dqkv, st_off[j], st_k[j]);
      hvk_bst16(r_dqkv, st_off[j] + 2 * C, st_v[j]);
    }
    if (HVK_BWD_EARLY && w + 2 < w1) load_tiles(w + 2);  // into the registers just written to LDS
    BSTAMP(0);      // loads landed, normalised, images written
    lds_barrier();  // the pair's q^, k^, dO images complete
    BSTAMP(1);

    if (act) {
      uint4 kfa[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) kfa[t] = *reinterpret_cast<const uint4*>(ksb + o_row + 1024 * t);
      uint4 kt_frag[K::NC][2];
#pragma unroll
      for (int c = 0; c < K::NC; ++c)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const char* b = ksb + o_kt + 2048 * c + 512 * dt;
          const uint2 lo = hvk_tr_read((const hvk_bf16*)b), hi = hvk_tr_read((const hvk_bf16*)(b + 1024));
          kt_frag[c][dt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }

      // ---------------- phase A: own query tiles, query on the lane
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int qi = hf + 2 * j;
        if (qi >= NT) break;
        __builtin_amdgcn_sched_barrier(0);  // one query tile's live set at a time
        hvk_f32x4 s[NT], dp[NT];
        // the own q / dO tile: from the image when the registers already hold the next window's
        const uint4 qa = HVK_BWD_EARLY ? *reinterpret_cast<const uint4*>(qsb + o_row + 1024 * qi) : qf[j];
        const uint4 da = HVK_BWD_EARLY ? *reinterpret_cast<const uint4*>(dob + o_row + 1024 * qi) : df[j];
#pragma unroll
        for (int ki = 0; ki < NT; ++ki) {
          s[ki] = hvk_mfma16(kfa[ki], qa, hvk_f32x4{0, 0, 0, 0});  // cos(q, k)
          dp[ki] = hvk_mfma16(vf[ki], da, hvk_f32x4{0, 0, 0, 0});  // dO . V
        }
        const int q = 16 * qi + li;
        const float* tq = btab + (qi * NT * 64 + lane) * 4;
        const bool edge = edge_r || edge_c;  // wave-uniform
        const uint32_t mm = edge ? mask_bits(krow, kcol, q, WIN - g.shift, WIN, edge_r, edge_c) : 0u;
        float p[NT][4];
        float sum = 0.f, du = 0.f;
        float x[NT][4];
#pragma unroll
        for (int ki = 0; ki < NT; ++ki) {
          const float4 bb = *reinterpret_cast<const float4*>(tq + ki * 256);
          const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) x[ki][r] = NORMED ? s[ki][r] + bv[r] : fmaf(s[ki][r], sc2, bv[r]);  // NORMED: s = q^ sc2 . k^
        }
        // the -100 mask of an edge window in a branch of its own (interior windows and unshifted
        // blocks skip it): as a select per score on the uniform edge flag it cost 5 VALU each, a
        // third of the tile's VALU; mm opaque so its bit conversions stay inside the branch
        if (edge) {
          uint32_t m1 = mm;
          asm volatile("" : "+v"(m1));
#pragma unroll
          for (int ki = 0; ki < NT; ++ki)
#pragma unroll
            for (int r = 0; r < 4; ++r) x[ki][r] = fmaf((float)((m1 >> (ki * 4 + r)) & 1u), mask2, x[ki][r]);
        }
#pragma unroll
        for (int ki = 0; ki < NT; ++ki)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[ki][r] = __builtin_amdgcn_exp2f(x[ki][r]);
            sum += p[ki][r];
            du = fmaf(p[ki][r], dp[ki][r], du);
          }
        sum = hvk_group4_sum(sum);
        if (__builtin_expect(__ballot(sum < 0x1p-100f) != 0, 0)) {
          // a row whose every logit sits far below the head bound (zero query vector):
          // softmax against the row's own max
          float mx = -INFINITY;
#pragma unroll
          for (int ki = 0; ki < NT; ++ki) {
            const float4 bb = *reinterpret_cast<const float4*>(tq + ki * 256);
            const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float x = NORMED ? s[ki][r] + bv[r] : fmaf(s[ki][r], sc2, bv[r]);  // NORMED: s = q^ sc2 . k^
              if (edge) x += ((mm >> (ki * 4 + r)) & 1u) ? mask2 : 0.f;
              p[ki][r] = x;
              mx = fmaxf(mx, x);
            }
          }
          mx = hvk_group4_max(mx);
          sum = 0.f;
          du = 0.f;
#pragma unroll
          for (int ki = 0; ki < NT; ++ki)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              p[ki][r] = __builtin_amdgcn_exp2f(p[ki][r] - mx);
              sum += p[ki][r];
              du = fmaf(p[ki][r], dp[ki][r], du);
            }
          sum = hvk_group4_sum(sum);
        }
        du = hvk_group4_sum(du);
        // P = p/sum, delta = du/sum, scale*dS = p * (dp*(scale/sum) - delta*scale/sum)
        const float inv = __builtin_amdgcn_rcpf(sum);
        const float ca = inv * scale, cb = -du * inv * ca;
        uint32_t dsp[NT][2];
#pragma unroll
        for (int ki = 0; ki < NT; ++ki) {
          float ds[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ds[r] = p[ki][r] * fmaf(dp[ki][r], ca, cb);
            dbias[j][ki][r] += ds[r];
            dscale = fmaf(ds[r], s[ki][r], dscale);
          }
          dsp[ki][0] = hvk_pack2(ds[0], ds[1]);
          dsp[ki][1] = hvk_pack2(ds[2], ds[3]);
          int pw = o_pw;  // the xor per write, not four hoisted offsets held across the loop
          asm volatile("" : "+v"(pw));
          const int off = qi * 16 * ROWS * 2 + (pw ^ (32 * ki));
          *reinterpret_cast<uint2*>((char*)ps + off) =
              make_uint2(hvk_pack2(p[ki][0] * inv, p[ki][1] * inv), hvk_pack2(p[ki][2] * inv, p[ki][3] * inv));
          *reinterpret_cast<uint2*>((char*)dss + off) = make_uint2(dsp[ki][0], dsp[ki][1]);
        }
        // dQ^T = K^T (scale dS^T)
        hvk_f32x4 dq[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int c = 0; c < K::NC; ++c) {
          const bool has1 = 2 * c + 1 < NT;
          const uint4 bf = make_uint4(dsp[2 * c][0], dsp[2 * c][1], has1 ? dsp[2 * c + 1][0] : 0u,
                                      has1 ? dsp[2 * c + 1][1] : 0u);
          dq[0] = hvk_mfma16(kt_frag[c][0], bf, dq[0]);
          dq[1] = hvk_mfma16(kt_frag[c][1], bf, dq[1]);
        }
        // normalize backward: dq = (dq^ - q^ (q^ . dq^)) / max(||q||, eps)
        float qh[2][4], dot = 0.f;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const uint2 v = *reinterpret_cast<const uint2*>(qsb + o_r8 + 1024 * qi + 512 * dt);
          qh[dt][0] = hvk_lo(v.x); qh[dt][1] = hvk_hi(v.x);
          qh[dt][2] = hvk_lo(v.y); qh[dt][3] = hvk_hi(v.y);
#pragma unroll
          for (int r = 0; r < 4; ++r) dot += qh[dt][r] * dq[dt][r];
        }
        dot = hvk_group4_sum(dot);
        if constexpr (NORMED) dot *= inv_sc2 * inv_sc2;  // qh = q^ sc2: q^ (q^ . dq^) = qh (qh . dq^) / sc2^2
        if (rnq[j] >= 1e12f) dot = 0.f;  // ||q|| <= eps: x / eps, no projection term
        uint2 pk[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = (dq[dt][r] - qh[dt][r] * dot) * rnq[j];
            if (q < K::N) dqb[dt][r] += v[r];
          }
          pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
        }
        const uint4 o = hvk_pair_swap(pk[0], pk[1]);  // all lanes: cross-lane
        hvk_bst16(r_dqkv, row[j] < 0 ? HVK_OOB : (uint32_t)(row[j] * C3 + h * 32 + hvk_pair_col(gq)) * 2, o);
      }
    }
    BSTAMP(2);
    if (w + 2 < w1) {
      load_v(w + 2);  // phase A was the last reader of vf
      if (!HVK_BWD_EARLY) load_tiles(w + 2);
    }
    BSTAMP(3);
    lds_barrier();  // P / dS images complete
    BSTAMP(4);

    // ---------------- phase B: own key tiles, key on the lane
    if (act) {
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int kt = hf + 2 * j;
        if (kt >= NT) break;
        __builtin_amdgcn_sched_barrier(0);
        hvk_f32x4 dv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, dk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        // rows rq0 + 16m + 32c share f(rq0): one base, the rows as immediates
        const int o_pb = rq0 * ROWS * 2 + ((((4 * kt + (li & 3)) ^ frq) & (ROWS / 4 - 1)) << 3);
        const char* const psb = reinterpret_cast<const char*>(ps) + o_pb;
        const char* const dsb = reinterpret_cast<const char*>(dss) + o_pb;
#pragma unroll
        for (int c = 0; c < K::NC; ++c) {
          const int rlo = 32 * c * ROWS * 2, rhi = rlo + 16 * ROWS * 2;
          uint2 lo = hvk_tr_read((const hvk_bf16*)(psb + rlo)), hi = hvk_tr_read((const hvk_bf16*)(psb + rhi));
          const uint4 pfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
          lo = hvk_tr_read((const hvk_bf16*)(dsb + rlo)); hi = hvk_tr_read((const hvk_bf16*)(dsb + rhi));
          const uint4 dsfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int olo = o_trq + 2048 * c + 512 * dt, ohi = olo + 1024;
            lo = hvk_tr_read((const hvk_bf16*)(dob + olo)); hi = hvk_tr_read((const hvk_bf16*)(dob + ohi));
            dv[dt] = hvk_mfma16(make_uint4(lo.x, lo.y, hi.x, hi.y), pfr, dv[dt]);
            lo = hvk_tr_read((const hvk_bf16*)(qsb + olo)); hi = hvk_tr_read((const hvk_bf16*)(qsb + ohi));
            dk[dt] = hvk_mfma16(make_uint4(lo.x, lo.y, hi.x, hi.y), dsfr, dk[dt]);
          }
        }
        float kh[2][4], dot = 0.f;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const uint2 v = *reinterpret_cast<const uint2*>(ksb + o_r8 + 1024 * kt + 512 * dt);
          kh[dt][0] = hvk_lo(v.x); kh[dt][1] = hvk_hi(v.x);
          kh[dt][2] = hvk_lo(v.y); kh[dt][3] = hvk_hi(v.y);
#pragma unroll
          for (int r = 0; r < 4; ++r) dot += kh[dt][r] * dk[dt][r];
        }
        dot = hvk_group4_sum(dot);
        if (rnk[j] >= 1e12f) dot = 0.f;
        // NORMED: the q^ image holds q^ sc2, so dk here is sc2 dK^ (linear: the projection term
        // scales with it); one factor on the row's 1/||k||
        const float rk = NORMED ? rnk[j] * inv_sc2 : rnk[j];
        uint2 pk[2], pv[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (dk[dt][r] - kh[dt][r] * dot) * rk;
          pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
          pv[dt] = make_uint2(hvk_pack2(dv[dt][0], dv[dt][1]), hvk_pack2(dv[dt][2], dv[dt][3]));
        }
        st_k[j] = hvk_pair_swap(pk[0], pk[1]);
        st_v[j] = hvk_pair_swap(pv[0], pv[1]);
        st_off[j] = row[j] < 0 ? HVK_OOB : (uint32_t)(row[j] * C3 + C + h * 32 + hvk_pair_col(gq)) * 2;
      }
    }
    BSTAMP(5);
    lds_barrier();  // phase B reads done: the images are free for the next window
    BSTAMP(6);
  }
#ifdef HVK_STAMPS
  if (lane == 0)
    for (int k = 0; k < 7; ++k) atomicAdd(&g_bwd_stamps[k], st_acc[k]);
  if (lane == 0) atomicAdd(&g_bwd_stamps[7], 1ull);
  const unsigned long long st_loop_end = __builtin_amdgcn_s_memtime();
#endif

  // ---- the bias / scale / q_bias gradients of this (chunk, head), deterministically: the
  // accumulator-order partials (carried as scale*dS) of the two pairs staged in LDS, folded into
  // the (2w-1)^2 bins by one thread per bin in a fixed (query, key) order, the wave sums of d scale
  // and d q_bias added in wave order, and the results added to this workgroup's own workspace slot
  // (plain load + store: a later batch slice's launch adds in stream order); the finalize kernel
  // sums the slots in chunk order.  No float atomics, so two runs give the same bits.
  static_assert(kThreads == 256, "four waves: two pairs");
  constexpr int RB = K::R * K::R, SLOT = bwd_slot_floats(WIN);
  static_assert(RB <= kThreads, "one bin per thread");
  lds_barrier();  // LDS only: the last window's dQ / dK / dV stores stay in flight
  const float inv_scale = 1.f / scale;
  float* red = reinterpret_cast<float*>(img0) + pair * (PC::PAIR_LDS / 2);  // pair p's images
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int qi = hf + 2 * j;
    if (qi >= NT) break;
#pragma unroll
    for (int ki = 0; ki < NT; ++ki)
      *reinterpret_cast<float4*>(red + ((qi * NT + ki) * 64 + lane) * 4) =
          make_float4(dbias[j][ki][0], dbias[j][ki][1], dbias[j][ki][2], dbias[j][ki][3]);
  }
  lds_barrier();  // LDS only: the last window's dQ / dK / dV stores stay in flight
  const float* red0 = reinterpret_cast<const float*>(img0);
  const int tid = threadIdx.x;
#ifdef HVK_STAMPS
  const unsigned long long st_fold0 = __builtin_amdgcn_s_memtime();
#endif
  float binv = 0.f;
  if (tid < RB) {  // bin (dy, dx) = (q_y - k_y, q_x - k_x) + (w - 1)
    const int dy = tid / K::R - (WIN - 1), dx = tid % K::R - (WIN - 1);
    const int y0 = dy > 0 ? dy : 0, y1 = dy < 0 ? WIN + dy : WIN;
    const int x0 = dx > 0 ? dx : 0, x1 = dx < 0 ? WIN + dx : WIN;
    // every (q_y, q_x) of the window unrolled with a predicate (the same (q_y, q_x) order and
    // additions as a loop over the bin's own range): the reads no longer wait one by one behind
    // a divergent loop (the fold was 15-25 % of a stage-2/3 workgroup's life, HVK_STAMPS)
#pragma unroll
    for (int qy = 0; qy < WIN; ++qy)
#pragma unroll
      for (int qx = 0; qx < WIN; ++qx) {
        const bool in = qy >= y0 && qy < y1 && qx >= x0 && qx < x1;
        const int q = qy * WIN + qx, key = in ? (qy - dy) * WIN + (qx - dx) : 0;
        const int e = ((q >> 4) * NT + (key >> 4)) * 256 + ((q & 15) + 16 * ((key & 15) >> 2)) * 4 + (key & 3);
        const float t = red0[e] + red0[PC::PAIR_LDS / 2 + e];
        binv = in ? binv + t : binv;
      }
  }
#ifdef HVK_STAMPS
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long st_fold1 = __builtin_amdgcn_s_memtime();
#endif
  dscale = hvk_wave_sum(dscale);
  float qbv[2][4];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) qbv[dt][r] = hvk_row16_sum(dqb[dt][r]);
  lds_barrier();  // the bin reads are done: stage the wave sums over the partials
  float* stg = reinterpret_cast<float*>(img0);
  // NORMED: the products summed were dS (sc2 cos)
  if (lane == 0) stg[wave] = NORMED ? dscale * inv_scale * inv_sc2 : dscale * inv_scale;
  if (li == 0) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) stg[8 + wave * 32 + 16 * dt + 4 * gq + r] = qbv[dt][r];
  }
  lds_barrier();  // LDS only: the last window's dQ / dK / dV stores stay in flight
  float* slot = a.dbias_acc + ((size_t)h * a.slot_stride + chunk) * SLOT;
  for (int i = tid; i < SLOT; i += kThreads) {
    float v;
    if (i < RB) v = binv * inv_scale;
    else if (i == RB) v = (stg[0] + stg[1]) + (stg[2] + stg[3]);
    else {
      const int c = i - RB - 1;
      v = (stg[8 + c] + stg[40 + c]) + (stg[72 + c] + stg[104 + c]);
    }
    slot[i] = a.slot_add ? slot[i] + v : v;
  }
  // the last window's dK / dV leave here, after the fold: issued before it, their data registers
  // could not be reused until the stores had read them, and the fold waited for them (vmcnt;
  // 35-39 % of a stage-2/3 workgroup's teardown, HVK_STAMPS)
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    hvk_bst16(r_dqkv, st_off[j], st_k[j]);
    hvk_bst16(r_dqkv, st_off[j] + 2 * C, st_v[j]);
  }
#ifdef HVK_STAMPS
  __syncthreads();
  if (lane == 0) {
    atomicAdd(&g_bwd_stamps[8], st_acc_setup);
    atomicAdd(&g_bwd_stamps[9], __builtin_amdgcn_s_memtime() - st_loop_end);
    atomicAdd(&g_bwd_stamps[10], st_fold0 - st_loop_end);  // stores issued, partials staged
    atomicAdd(&g_bwd_stamps[11], st_fold1 - st_fold0);     // the bins fold
  }
#endif
}

// Sum the (head, chunk) slots in chunk order into the CPB-table gradient [nH, R*R], d scale and
// d q_bias, and leave the workspace zero for the next call.
template <int WIN>
__global__ __launch_bounds__(FIN_THREADS) void wmsa_finalize_kernel(BwdArgs a, float* __restrict__ dtab,
                                                            float* __restrict__ dscale,
                                                            float* __restrict__ dqb) {
  finalize_slots<WIN>(a, dtab, dscale, dqb, blockIdx.x, blockIdx.y);
}

template <int WIN>
int launch_bwd(const BwdArgs& a, float* dbias_table, float* dscale, float* dqb, hipStream_t st) {
  {
    constexpr size_t plds = PairCfg<WIN>::LDS;
    static bool pattr = false;
    if (!pattr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_pair_kernel<WIN, false, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_pair_kernel<WIN, true, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_pair_kernel<WIN, false, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_pair_kernel<WIN, true, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds);
      pattr = true;
    }
    // qkv read policy (option "wmsa_bwd_nt"): 0 default (cached), 1 always nontemporal,
    // 2 nontemporal when qkv exceeds the 256 MB Infinity Cache
    const int ntm = (int)hvk_opt(HVK_OPT_WMSA_BWD_NT);
    const bool qnt = ntm == 1 || (ntm == 2 && (size_t)a.g.B * a.g.H * a.g.W * a.g.C * 6 > ((size_t)256 << 20));
    // buffer descriptors span < 2^31 bytes: launch over batch slices when qkv is larger (option
    // "wmsa_bwd_slice_bytes" lowers the limit so the tests run several slices on small tensors)
    const size_t img_bytes = (size_t)a.g.H * a.g.W * 3 * a.g.C * 2;
    const int per = (int)((size_t)hvk_opt(HVK_OPT_WMSA_BWD_SLICE_BYTES) / img_bytes);
    if (per < 1) return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_bwd: one image's qkv exceeds 2 GiB");
    const size_t tok = (size_t)a.g.H * a.g.W;
    for (int b0 = 0; b0 < a.g.B; b0 += per) {
      BwdArgs s = a;
      s.g.B = a.g.B - b0 < per ? a.g.B - b0 : per;
      s.slot_add = b0 > 0;
      s.g.n_windows = s.g.B * a.g.nWh * a.g.nWw;
      if (s.g.n_chunks > s.g.n_windows) s.g.n_chunks = s.g.n_windows;
      s.qkv += b0 * tok * 3 * a.g.C;
      s.dout += b0 * tok * a.g.C;
      s.dqkv += b0 * tok * 3 * a.g.C;
      if (s.rn) s.rn += b0 * tok * 2 * a.g.nH;
      const int it = s.g.n_chunks * s.g.nH;
      const int nb = s.g.xcd_runs ? 8 * ((it + 7) / 8) : (s.g.n_chunks + 7) / 8 * 8 * s.g.nH;
      if (qnt && s.rn)
        HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, (wmsa_bwd_pair_kernel<WIN, true, true>), dim3(nb), dim3(kThreads), plds, st, s);
      else if (qnt)
        HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, (wmsa_bwd_pair_kernel<WIN, true, false>), dim3(nb), dim3(kThreads), plds, st, s);
      else if (s.rn)
        HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, (wmsa_bwd_pair_kernel<WIN, false, true>), dim3(nb), dim3(kThreads), plds, st, s);
      else
        HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, (wmsa_bwd_pair_kernel<WIN, false, false>), dim3(nb), dim3(kThreads), plds, st, s);
    }
  }
  HVK_CHECK_LAUNCH("wmsa_bwd");
  hipLaunchKernelGGL(wmsa_finalize_kernel<WIN>, dim3(a.g.nH, finalize_blocks_y(WIN)), dim3(FIN_THREADS), 0, st, a, dbias_table,
                     dscale, dqb);
  HVK_CHECK_LAUNCH("wmsa_finalize");
  return HVK_OK;
}

}  // namespace

extern "C" {

#ifdef HVK_STAMPS
int hvk_debug_bwd_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_stamps), 12 * sizeof(unsigned long long)) != hipSuccess)
    return HVK_EINVAL;
  const unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_stamps), z, sizeof(z)) == hipSuccess ? HVK_OK : HVK_EINVAL;
}
#endif

size_t hvk_wmsa_bwd_workspace_bytes(int num_heads, int window) {
  // [nH][slots per head][R*R bins, d scale, 32 d q_bias] floats (wmsa_common.h BwdArgs)
  if (num_heads <= 0 || window <= 0) return 0;
  return (size_t)num_heads * hvk_wmsa::bwd_slot_stride(num_heads, hvk_wmsa::large_window(window)) *
         hvk_wmsa::bwd_slot_floats(window) * sizeof(float);
}

}  // extern "C"

namespace {
int wmsa_fwd(const void* qkv, void* out, float* lse, const float* bias_table, const float* scale,
             int B, int H, int W, int C, int num_heads, int window, int shift, int normed,
             void* stream) {
  if (!qkv || !out || !bias_table || !scale)
    return hvk_set_error(HVK_EINVAL, "hvk_wmsa_fwd: null pointer");
  if (normed && hvk_wmsa::large_window(window))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_fwd_normed: windows <= 8 only (got %d)", window);
  FwdArgs a{};
  a.qk_normed = normed;
  a.qkv = static_cast<const hvk_bf16*>(qkv);
  a.out = static_cast<hvk_bf16*>(out);
  a.bias = bias_table;
  a.scale = scale;
  a.lse = lse;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // every form addresses one image's qkv rows with 32-bit byte offsets and token rows as int
  if ((long long)H * W * C * 6 >= (1ll << 32) || (long long)B * H * W >= (1ll << 31))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_fwd: %d x %d x %d x %d past 32-bit offsets", B, H, W, C);
  if (hvk_wmsa::large_window(window)) {
    int rc = make_geom(B, H, W, C, num_heads, window, shift, 256 * 4, a.g);
    if (rc) return rc;
    return hvk_wmsa::large_fwd(a, window, st);
  }
  if (window != 4 && window != 6 && window != 7 && window != 8)
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_fwd: window %d not built (4,6,7,8,12,16,24)", window);
  // option "wmsa_fwd_form" 1: the persistent slab-ring forward (A/B runs and the parity tests
  // that pin both forms to the same bits); default: one workgroup per (window, head group)
  if (hvk_opt(HVK_OPT_WMSA_FWD_FORM) == 1)
    return hvk_wmsa::ring_fwd(a, B, H, W, C, num_heads, window, shift, st);
  return hvk_wmsa::win_fwd(a, B, H, W, C, num_heads, window, shift, st);
}

int wmsa_bwd(const void* qkv, const float* rn, const void* dout, const void* out, const float* lse,
             void* dqkv, float* dq_bias, const float* bias_table, const float* scale,
             float* dbias_table, float* dscale, float* workspace, size_t workspace_bytes,
             int B, int H, int W, int C, int num_heads, int window, int shift,
             void* stream) {
  if (!qkv || !dout || !dqkv || !bias_table || !scale || !dbias_table || !dscale || !workspace)
    return hvk_set_error(HVK_EINVAL, "hvk_wmsa_bwd: null pointer");
  if (rn && hvk_wmsa::large_window(window))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_bwd_normed: windows <= 8 only (got %d)", window);
  if (lse && !out) return hvk_set_error(HVK_EINVAL, "hvk_wmsa_bwd: lse given without the forward's output");
  if (workspace_bytes < hvk_wmsa_bwd_workspace_bytes(num_heads, window))
    return hvk_set_error(HVK_EINVAL, "hvk_wmsa_bwd: workspace too small");
  // every form addresses one image's qkv rows with 32-bit byte offsets and token rows as int
  if ((long long)H * W * C * 6 >= (1ll << 32) || (long long)B * H * W >= (1ll << 31))
    return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_bwd: %d x %d x %d x %d past 32-bit offsets", B, H, W, C);
  BwdArgs a{};
  a.rn = rn;
  a.qkv = static_cast<const hvk_bf16*>(qkv);
  a.dout = static_cast<const hvk_bf16*>(dout);
  a.dqkv = static_cast<hvk_bf16*>(dqkv);
  a.out = static_cast<const hvk_bf16*>(out);
  a.lse = lse;
  a.bias = bias_table;
  a.scale = scale;
  a.dbias_acc = workspace;
  a.slot_stride = hvk_wmsa::bwd_slot_stride(num_heads, hvk_wmsa::large_window(window));
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
  {
    // HVK_BWD_SLOTS / nH chunks (two resident workgroups per CU): the workspace's slots per head,
    // so the chunk count and the workspace size come from one place
    const int c = hvk_wmsa::bwd_slot_stride(num_heads, false);
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
}  // namespace

extern "C" {

int hvk_wmsa_fwd(const void* qkv, void* out, float* lse, const float* bias_table, const float* scale,
                 int B, int H, int W, int C, int num_heads, int window, int shift, void* stream) {
  return wmsa_fwd(qkv, out, lse, bias_table, scale, B, H, W, C, num_heads, window, shift, 0, stream);
}

int hvk_wmsa_fwd_normed(const void* qkv, void* out, const float* bias_table, const float* scale,
                        int B, int H, int W, int C, int num_heads, int window, int shift, void* stream) {
  return wmsa_fwd(qkv, out, nullptr, bias_table, scale, B, H, W, C, num_heads, window, shift, 1, stream);
}

int hvk_wmsa_bwd(const void* qkv, const void* dout, const void* out, const float* lse, void* dqkv,
                 float* dq_bias, const float* bias_table, const float* scale,
                 float* dbias_table, float* dscale, float* workspace, size_t workspace_bytes,
                 int B, int H, int W, int C, int num_heads, int window, int shift, void* stream) {
  return wmsa_bwd(qkv, nullptr, dout, out, lse, dqkv, dq_bias, bias_table, scale, dbias_table, dscale,
                  workspace, workspace_bytes, B, H, W, C, num_heads, window, shift, stream);
}

int hvk_wmsa_bwd_normed(const void* qkv, const float* rn, const void* dout, void* dqkv, float* dq_bias,
                        const float* bias_table, const float* scale, float* dbias_table, float* dscale,
                        float* workspace, size_t workspace_bytes, int B, int H, int W, int C,
                        int num_heads, int window, int shift, void* stream) {
  if (!rn) return hvk_set_error(HVK_EINVAL, "hvk_wmsa_bwd_normed: null rn");
  return wmsa_bwd(qkv, rn, dout, nullptr, nullptr, dqkv, dq_bias, bias_table, scale, dbias_table, dscale,
                  workspace, workspace_bytes, B, H, W, C, num_heads, window, shift, stream);
}

}  // extern "C"
