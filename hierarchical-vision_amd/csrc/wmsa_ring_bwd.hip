// W-MSA backward for windows 6 and 7 with an even head count on gfx950: persistent workgroups
// that stream window slabs through LDS by LDS-DMA, the backward counterpart of
// wmsa_ring.hip.  Same math as wmsa_bwd_pair_kernel (wmsa.hip; reference swinv2.py:221-261
// differentiated, roll / partition / reverse folded into addressing).
//
// Work unit: (window, group of HG = 2 heads); a workgroup = 2 waves per head walks a chunk of
// windows of one head group, two workgroups per CU (2 waves per SIMD).  Per window:
//   1. the window's q/k/v (qkv rows) and dO bytes of the head group sit in one LDS slab,
//      double-buffered: the NEXT window's slab is DMA'd (global_load_lds_dwordx4, whole
//      128-B row segments of the head pair) while this one is worked on -- the memory shape
//      of tools/probe/wmsa_bwd_mem.hip "slab", not 16 rows x 64 B per load instruction;
//   2. each wave L2-normalises its own query/key tiles in place (q^, k^); barrier;
//   3. phase A (own query tiles, query on the lane): S^T, dP^T = V dO^T, P against the head
//      bound with row sums by a ones-MFMA (padding keys excluded), dS, dQ; it stores the
//      UNnormalised P image, the row constants delta/sum^2 and dO / sum in place; barrier;
//   4. phase B (own key tiles, key on the lane): dP^T recomputed from dO/sum and V, dS from P
//      and the row constants, dV^T = (dO/sum)^T P, dK^T = Q^T dS: no dS image (LDS budget).
// Tokens sit on the 8-wide grid of the forward (position p = 8y + x, x or y >= w padding):
// the forward's compact mirrored CPB table feeds the scores, and the dbias partial sums are
// kept in accumulator order over grid positions (wmsa_ring_bwd_finalize maps them to bins).
// LDS slab layout (tools/ring_bwd_layout.py: every fragment read bank-conflict free but the
// accumulator-row reads, 2 extra cycles): token slots of RSQ (qkv: 12 HG real 16-B slots)
// and RSD (dO: 4 HG) slots, window rows RUNQ / RUND slots apart.
#include <stdlib.h>

#include "wmsa_ring.h"

#ifndef HVK_RING_BWD_PROBE
#define HVK_RING_BWD_PROBE 0
#endif

namespace {
using namespace hvk_ring;

template <int WIN, int HG>
struct RBLayout;
template <>
struct RBLayout<7, 2> {
  static constexpr int RSQ = 25, RUNQ = 192, RSD = 9, RUND = 64;
};
template <>
struct RBLayout<6, 2> {
  static constexpr int RSQ = 25, RUNQ = 192, RSD = 9, RUND = 64;
};

template <int WIN, int HG>
struct RBCfg {
  using RC = RingCfg<WIN, HG>;  // grid geometry and the compact bias table
  using L = RBLayout<WIN, HG>;
  static_assert(RC::PW == 8, "8-wide grid");
  static constexpr int NT = RC::NT, NC = RC::NC, TPW = (NT + 1) / 2, R = RC::R;
  static constexpr int WAVES = 2 * HG;
  static constexpr int IPRQ = (WIN * L::RSQ + 63) / 64, IPRD = (WIN * L::RSD + 63) / 64;
  static_assert(L::RUNQ >= 64 * IPRQ && L::RUND >= 64 * IPRD, "runs hold their DMA slots");
  static_assert(L::RSQ >= 12 * HG && L::RSD >= 4 * HG, "token slots hold the head group");
  static constexpr int NQI = WIN * IPRQ, NI = NQI + WIN * IPRD;  // DMA wave-instructions per slab
  static constexpr int NK = (NI + WAVES - 1) / WAVES;             // per wave
  static constexpr int SLABQ = WIN * L::RUNQ * 16, SLAB = SLABQ + WIN * L::RUND * 16;
  static constexpr int ROWS = 32 * NC;              // padded positions of the P image
  static constexpr int PIMG = ROWS * ROWS * 2;      // bytes of one head's P image
  static constexpr int TAB = NT * NT * 256;         // accumulator-order dbias floats per head
  static constexpr int OFF_P = 2 * SLAB, OFF_D = OFF_P + HG * PIMG, OFF_T = OFF_D + HG * ROWS * 4,
                       OFF_Z = OFF_T + HG * RC::TABF * 4;
  // zero region read by padding positions: every fragment read of a padded position adds
  // the same immediates (parts, units, halves) to a zero base as a real one to its slot
  static constexpr int ZERO = 12 * HG * 16 + 64;
  static constexpr int LDS = OFF_Z + ZERO;
  static_assert(HG * TAB * 4 <= 2 * SLAB, "the dbias reduction reuses the slabs");
  static_assert(2 * LDS <= 160 * 1024, "two workgroups per CU");
};

// P image (bf16 [query][key], ROWS per row) swizzle of wmsa.hip (pimg_off): 8-B unit col8 of
// `row` at col8 ^ f(row); conflict-free 8-B row writes and transposed reads
template <int ROWS>
__device__ __forceinline__ int pimg_byte(int row, int col8) {
  const int f = ((row ^ (row >> 2)) & 1) | ((row >> 2) & 2) | ((row << 1) & 4);
  return 2 * (row * ROWS + (((col8 ^ f) & (ROWS / 4 - 1)) << 2));
}

#ifdef HVK_STAMPS
// diagnostic build (tools/bwd_stamps.py --ring): per-phase shader-clock sums over all waves
__device__ unsigned long long g_ring_bwd_stamps[8];
#define RSTAMP(k)                                               \
  do {                                                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - st_prev;                                  \
    st_prev = t_;                                               \
  } while (0)
#else
#define RSTAMP(k) \
  do {            \
  } while (0)
#endif

template <int WIN, int HG>
__global__ __launch_bounds__(128 * HG, 2) void wmsa_bwd_ring_kernel(BwdArgs a) {
  using K = RBCfg<WIN, HG>;
  using RC = typename K::RC;
  using L = typename K::L;
  constexpr int NT = K::NT, NC = K::NC, TPW = K::TPW, ROWS = K::ROWS;
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
  const int hl = wave >> 1, hf = wave & 1;
  const int h = grp * HG + hl;
  const int li = lane & 15, gq = lane >> 4;
  const int C = g.C, C3 = 3 * C;
  const int per_img = g.nWh * g.nWw;
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t zaddr = lds0 + K::OFF_Z;
  float* btab = reinterpret_cast<float*>(smem + K::OFF_T);

  // ---- LDS-DMA of a window's slab (wmsa_ring.hip's scheme): instruction j < NQI fills qkv
  // run ty = j / IPRQ, slots 64m + lane (m = j % IPRQ) = token tx, 16-B slot r; j >= NQI the
  // dO runs alike; instruction j is issued by wave j % WAVES.  A lane's offset inside the
  // window row depends only on (qkv or dO, m): pre[] = offset (bits 0-23) | tx << 24; padding
  // slots re-read the row's first bytes (never read back).
  const unsigned RBQ = 6u * C, RBD = 2u * C;
  const unsigned go = (unsigned)grp * HG * 64;  // the group's byte offset inside a part
  unsigned pre[K::IPRQ + K::IPRD];
#pragma unroll
  for (int m = 0; m < K::IPRQ + K::IPRD; ++m) {
    unsigned v = go;
    if (m < K::IPRQ) {
      const unsigned s = 64u * m + lane, tx = s / L::RSQ, r = s % L::RSQ;
      if (tx < WIN && r < 12u * HG) v = (tx * RBQ + (r / (4 * HG)) * 2u * C + (r % (4 * HG)) * 16 + go) | (tx << 24);
    } else {
      const unsigned s = 64u * (m - K::IPRQ) + lane, tx = s / L::RSD, r = s % L::RSD;
      if (tx < WIN && r < 4u * HG) v = (tx * RBD + r * 16 + go) | (tx << 24);
    }
    pre[m] = v;
  }
  const char* qkv = reinterpret_cast<const char*>(a.qkv);
  const char* dout = reinterpret_cast<const char*>(a.dout);
  auto issue = [&](int b, int wh, int ww, int buf) __attribute__((always_inline)) {
    const int y0 = wh * WIN + g.shift, x0 = ww * WIN + g.shift;
    const int ly = g.H - y0, lx = g.W - x0;  // ty >= ly (tx >= lx): the row wraps
    const uint32_t dst = lds0 + buf * K::SLAB;
    const char* imq = qkv + (size_t)b * g.H * g.W * RBQ;
    const char* imd = dout + (size_t)b * g.H * g.W * RBD;
    const unsigned row0 = (unsigned)y0 * g.W + x0, wrap = (unsigned)g.H * g.W;  // in tokens
#pragma unroll
    for (int j = 0; j < K::NI; ++j) {
      if (j % K::WAVES != wave) continue;  // wave-uniform
      const bool isq = j < K::NQI;
      const int ty = isq ? j / K::IPRQ : (j - K::NQI) / K::IPRD;
      const int m = isq ? j % K::IPRQ : K::IPRQ + (j - K::NQI) % K::IPRD;
      const unsigned rb = isq ? RBQ : RBD;
      const unsigned U = (row0 + (unsigned)ty * g.W - (ty >= ly ? wrap : 0u)) * rb;  // uniform
      unsigned off = (pre[m] & 0xFFFFFFu) + U;
      if (lx < WIN)  // last window column: per-lane wrap of the token column
        off -= ((int)(pre[m] >> 24) >= lx) ? (unsigned)g.W * rb : 0u;
      const uint32_t m0 = dst + (isq ? ty * L::RUNQ * 16 + (j % K::IPRQ) * 1024
                                     : K::SLABQ + ty * L::RUND * 16 + ((j - K::NQI) % K::IPRD) * 1024);
      dma16(isq ? imq : imd, off, m0);
    }
  };

  // ---- per-workgroup setup: mirrored compact bias tables (wmsa_ring.hip) shifted by the head
  // bound M = sc2 + max bias*log2e; zero slot; ones operands; region bits
  for (int e = threadIdx.x; e < HG * RC::TABF; e += 128 * HG) {
    const int hh = e / RC::TABF, i = RC::TABF - 1 - e % RC::TABF - RC::PAD;
    btab[e] = (i >= 0 && i < RC::R * RC::R) ? a.bias[(size_t)(grp * HG + hh) * RC::R * RC::R + i] * HVK_LOG2E : 0.f;
  }
  for (int e = threadIdx.x; e < K::ZERO / 16; e += 128 * HG)
    reinterpret_cast<uint4*>(smem + K::OFF_Z)[e] = make_uint4(0, 0, 0, 0);
  // P image rows of tiles that do not exist (NT = 3: rows 48-63) are read by phase B's
  // transposed reads: zero once, never written
  for (int e = threadIdx.x; e < HG * K::PIMG / 16; e += 128 * HG)
    reinterpret_cast<uint4*>(smem + K::OFF_P)[e] = make_uint4(0, 0, 0, 0);
  const float scale = a.scale[h];
  const float sc2 = scale * HVK_LOG2E;
  int cb = w0 / per_img, cwh = (w0 % per_img) / g.nWw, cww = w0 % g.nWw;
  issue(cb, cwh, cww, 0);
  __syncthreads();
  {
    float* tb = btab + hl * RC::TABF + RC::TABF - RC::PAD - RC::R * RC::R;  // mirrored real entries
    float mb = -INFINITY;
    for (int i = lane; i < RC::R * RC::R; i += 64) mb = fmaxf(mb, tb[i]);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) mb = fmaxf(mb, __shfl_xor(mb, m));
    const float Mh = sc2 + mb;
    if (hf == 0)
      for (int i = lane; i < RC::R * RC::R; i += 64) tb[i] -= Mh;
  }
  __syncthreads();
  const float mask2 = -100.f * HVK_LOG2E;
  int lq, lk;  // bias base index of this lane (wmsa_ring.hip)
  lq = (li >> 3) * RC::R + (li & 7);
  lk = (gq >> 1) * RC::R + 4 * (gq & 1);
  const uint32_t bta = lds0 + K::OFF_T +
                       4 * (hl * RC::TABF + RC::TABF - 4 - (RC::PAD + RC::BASE0 + lq - lk - RC::TR * (NT - 1) - 3) -
                            2 * RC::TR * (NT - 1));
  uint4 ones[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    uint32_t wv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * jj + e;
        const int p = 32 * c + (j < 4 ? 4 * gq + j : 16 + 4 * gq + j - 4);
        if ((p % 8) < WIN && (p / 8) < WIN) v |= 0x3F80u << (16 * e);
      }
      wv[jj] = v;
    }
    ones[c] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
  }
  uint32_t kband = 0;  // key-slot region bits (slot bit ki*4 + r): rows 0-15, columns 16-31
#pragma unroll
  for (int ki = 0; ki < NT; ++ki)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * ki + 4 * gq + r, ky = p / 8, kx = p % 8;
      if (ky >= WIN - g.shift) kband |= 1u << (ki * 4 + r);
      if (kx >= WIN - g.shift) kband |= 1u << (16 + ki * 4 + r);
    }

  const size_t T = (size_t)g.B * g.H * g.W;
  const auto r_dqkv = hvk_rsrc(a.dqkv, T * C3 * 2);
  const uint32_t pimg = lds0 + K::OFF_P + hl * K::PIMG;
  const uint32_t dlt = lds0 + K::OFF_D + hl * ROWS * 4;

  hvk_f32x4 dbias[TPW][NT];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int ki = 0; ki < NT; ++ki) dbias[j][ki] = hvk_f32x4{0, 0, 0, 0};
  float dscale = 0.f;
  float dqb[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  // phase B's dK / dV stores leave at the top of the next window (after its DMA wait)
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
#endif
  for (int w = w0; w < w1; ++w) {
    const int buf = (w - w0) & 1;
    // this window's slab has landed (own DMA: every op issued after it is one of the TPW dQ
    // stores of the previous window); the barrier publishes every wave's part, and every wave
    // is done with the previous window, so the other buffer and the P images are free
    if (w == w0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TPW) : "memory");
    RSTAMP(0);  // slab wait
    lds_barrier();
    RSTAMP(1);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      hvk_bst16(r_dqkv, st_off[j], st_k[j]);
      hvk_bst16(r_dqkv, st_off[j] + 2 * C, st_v[j]);
    }
    const int b = cb, wh = cwh, ww = cww;
    if (++cww == g.nWw) {
      cww = 0;
      if (++cwh == g.nWh) {
        cwh = 0;
        ++cb;
      }
    }
    if (w + 1 < w1) issue(cb, cwh, cww, buf ^ 1);
    RSTAMP(2);  // deferred stores + DMA issue
    const bool edge_r = g.shift && wh == g.nWh - 1, edge_c = g.shift && ww == g.nWw - 1;
#if HVK_RING_BWD_PROBE == 1  // tools/probe: memory only (same DMA, 3 TPW stores, no math)
    {
      (void)edge_r;
      (void)edge_c;
      const int xl = li & 7, yl = li >> 3;
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int t = hf + 2 * j;
        const bool ok = t < NT && xl < WIN && 2 * t + yl < WIN;
        const int r = ok ? window_token_row(g, b, wh, ww, WIN, (2 * t + yl) * WIN + xl) : -1;
        const uint4 v = lds_ld16(lds0 + buf * K::SLAB + 16 * lane);
        hvk_bst16(r_dqkv, r < 0 ? HVK_OOB : (uint32_t)(r * C3 + h * 32 + hvk_pair_col(gq)) * 2, v);
        st_k[j] = v;
        st_v[j] = v;
        st_off[j] = r < 0 ? HVK_OOB : (uint32_t)(r * C3 + C + h * 32 + hvk_pair_col(gq)) * 2;
      }
      lds_barrier();
      lds_barrier();
      continue;
    }
#endif

    // lane coordinates recomputed per window (out of the loop-invariant register pool)
    int l16 = li, g4 = gq;
    asm volatile("" : "+v"(l16), "+v"(g4));
    const uint32_t sq = lds0 + buf * K::SLAB;      // qkv slab of this window
    const uint32_t sd = sq + K::SLABQ;             // dO slab
    const int xl = l16 & 7, yl = l16 >> 3;
    // slot of grid position 16t + li is (2t + yl) * RUN + xl * RS; real iff xl < WIN, 2t + yl < WIN.
    // fq[t] / fd[t]: 16-B unit gq of the head's q (dO) segment, or the zero region
    auto real_t = [&](int t) __attribute__((always_inline)) { return xl < WIN && 2 * t + yl < WIN; };
    uint32_t fq[NT], fd[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      fq[t] = (real_t(t) ? sq + ((2 * t + yl) * L::RUNQ + xl * L::RSQ + 4 * hl) * 16 : zaddr) + 16 * g4;
      fd[t] = (real_t(t) ? sd + ((2 * t + yl) * L::RUND + xl * L::RSD + 4 * hl) * 16 : zaddr) + 16 * g4;
    }
    // own tiles (runtime t): the same addresses by arithmetic, not an indexed register array
    // (which the compiler lowers to scratch, and the vmcnt waits of its reloads drain the DMA)
    auto aq = [&](int t, int part) __attribute__((always_inline)) {
      return (real_t(t) ? sq + ((2 * t + yl) * L::RUNQ + xl * L::RSQ + 4 * hl) * 16 : zaddr) + 16 * g4 +
             part * 4 * HG * 16;
    };
    auto ad = [&](int t) __attribute__((always_inline)) {
      return (real_t(t) ? sd + ((2 * t + yl) * L::RUND + xl * L::RSD + 4 * hl) * 16 : zaddr) + 16 * g4;
    };

    // ---- normalise own q, k tiles in place
    float rnq[TPW], rnk[TPW];
    int row[TPW];
    uint4 qf[TPW], df[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int t = hf + 2 * j;
      row[j] = -1;
      if (t < NT) {
        const uint32_t a_q = aq(t, 0), a_k = aq(t, 1);
        qf[j] = l2_normalize(lds_ld16(a_q), rnq[j]);
        const uint4 kn = l2_normalize(lds_ld16(a_k), rnk[j]);
        df[j] = lds_ld16(ad(t));
        lds_st16(a_q, qf[j]);
        lds_st16(a_k, kn);
        const int tok = real_t(t) ? (2 * t + yl) * WIN + xl : -1;
        row[j] = tok >= 0 ? window_token_row(g, b, wh, ww, WIN, tok) : -1;
      } else {
        qf[j] = df[j] = make_uint4(0, 0, 0, 0);
        rnq[j] = rnk[j] = 0.f;
      }
    }
    RSTAMP(3);  // normalise
    lds_barrier();  // q^, k^ of every row
    RSTAMP(4);

    uint4 kfa[NT], vf[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      kfa[t] = lds_ld16(fq[t] + 4 * HG * 16);
      vf[t] = lds_ld16(fq[t] + 8 * HG * 16);
    }
    // K^T fragments (A of dQ^T = K^T dS^T): chunk c, half m: position 32c + 16m + 4gq + li/4,
    // 8-B piece (li & 3) + 4dt of the head's k segment
    const int rq0 = 4 * g4 + (l16 >> 2);  // position within a 16-row half
    const int xr = rq0 & 7, yr = rq0 >> 3;
    uint32_t trq[NC][2], trd[NC][2];  // + part offset + 32 dt
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int y = 4 * c + 2 * m + yr;
        const bool ok = xr < WIN && y < WIN;
        trq[c][m] = (ok ? sq + (y * L::RUNQ + xr * L::RSQ + 4 * hl) * 16 : zaddr) + 8 * (l16 & 3);
        trd[c][m] = (ok ? sd + (y * L::RUND + xr * L::RSD + 4 * hl) * 16 : zaddr) + 8 * (l16 & 3);
      }
    uint4 kt_frag[NC][2];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint2 lo = lds_tr8(trq[c][0] + 4 * HG * 16 + 32 * dt);
        const uint2 hi = lds_tr8(trq[c][1] + 4 * HG * 16 + 32 * dt);
        kt_frag[c][dt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }

    // ---------------- phase A: own query tiles, query on the lane
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int qi = hf + 2 * j;
      if (qi >= NT) {  // no tile (odd NT): a dropped store keeps every wave's vmcnt count at TPW
        hvk_bst16(r_dqkv, HVK_OOB, make_uint4(0, 0, 0, 0));
        break;
      }
      __builtin_amdgcn_sched_barrier(0);
      hvk_f32x4 s[NT], dp[NT];
#pragma unroll
      for (int ki = 0; ki < NT; ++ki) {
        s[ki] = hvk_mfma16(kfa[ki], qf[j], hvk_f32x4{0, 0, 0, 0});  // cos(q, k)
        dp[ki] = hvk_mfma16(vf[ki], df[j], hvk_f32x4{0, 0, 0, 0});  // dO . V
      }
      hvk_u32x2 br[NT][2];
      ring_bias_read_q<RC::TR, NT>(br, bta, qi);
      const int pq = 16 * qi + l16;
      const bool qreal = real_t(qi);
      uint32_t mreg = 0;  // keys in another shift region than this query (swinv2.py:357-388)
      if (edge_r || edge_c) {
        const int qy = pq >> 3, qx = pq & 7;
        if (edge_r) mreg |= (kband ^ (qy >= WIN - g.shift ? 0xFFFFu : 0u)) & 0xFFFFu;
        if (edge_c) mreg |= ((kband >> 16) ^ (qx >= WIN - g.shift ? 0xFFFFu : 0u)) & 0xFFFFu;
      }
      float x[NT][4];
#pragma unroll
      for (int ki = 0; ki < NT; ++ki) {
        const float bv[4] = {__uint_as_float(br[ki][0][0]), __uint_as_float(br[ki][0][1]),
                             __uint_as_float(br[ki][1][0]), __uint_as_float(br[ki][1][1])};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[ki][r] = fmaf(s[ki][r], sc2, bv[r]);
          if (edge_r || edge_c) x[ki][r] += ((mreg >> (ki * 4 + r)) & 1u) ? mask2 : 0.f;
        }
      }
      // exp2 of the head-bound-shifted logits; row sums of the bf16 P over real keys by a
      // ones-MFMA (padding keys have finite P here, zero dP and zero k^: they drop out)
      float p[NT][4];
      uint4 pf[NC];
      float du = 0.f;
      hvk_f32x4 osum = {0, 0, 0, 0};
      auto expo = [&](float shift) __attribute__((always_inline)) {
        du = 0.f;
#pragma unroll
        for (int ki = 0; ki < NT; ++ki)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[ki][r] = __builtin_amdgcn_exp2f(x[ki][r] - shift);
            du = fmaf(p[ki][r], dp[ki][r], du);
          }
        osum = hvk_f32x4{0, 0, 0, 0};
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const bool has1 = 2 * c + 1 < NT;
          pf[c] = make_uint4(hvk_pack2(p[2 * c][0], p[2 * c][1]), hvk_pack2(p[2 * c][2], p[2 * c][3]),
                             has1 ? hvk_pack2(p[2 * c + 1][0], p[2 * c + 1][1]) : 0u,
                             has1 ? hvk_pack2(p[2 * c + 1][2], p[2 * c + 1][3]) : 0u);
          osum = hvk_mfma16(ones[c], pf[c], osum);
        }
      };
      expo(0.f);
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(qreal && !(osum[0] >= 0x1p-100f)) != 0, 0)) {
        // slow path (rare, wave-uniform): a real query's every logit sits far below the head
        // bound (zero query vector, or cos far below 1 at a large scale): exponentiate against
        // the row max over real keys (the reference's softmax, swinv2.py:256)
        const uint32_t kpad = (uint32_t)(RC::KPAD >> (16 * g4)) & 0xFFFFu;
        float mx = -INFINITY;
#pragma unroll
        for (int ki = 0; ki < NT; ++ki)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if ((kpad >> (ki * 4 + r)) & 1u) x[ki][r] = -INFINITY;  // padding keys: P = 0
            mx = fmaxf(mx, x[ki][r]);
          }
        mx = hvk_group4_max(mx);
        expo(mx);
      }
      du = hvk_group4_sum(du);
      const float sum = qreal ? osum[0] : 1.f;  // padded query rows: any finite constant
      // P = p/sum; delta = du/sum; scale*dS = p * (dp*(scale/sum) - delta*scale/sum)
      const float inv = __builtin_amdgcn_rcpf(sum);
      const float ca = inv * scale, cb2 = -du * inv * ca;
      uint32_t dsp[NT][2];
#pragma unroll
      for (int ki = 0; ki < NT; ++ki) {
        float ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ds[r] = p[ki][r] * fmaf(dp[ki][r], ca, cb2);
          dbias[j][ki][r] += ds[r];
          dscale = fmaf(ds[r], s[ki][r], dscale);
        }
        dsp[ki][0] = hvk_pack2(ds[0], ds[1]);
        dsp[ki][1] = hvk_pack2(ds[2], ds[3]);
      }
      // P image rows (unnormalised p: phase B's dO rows carry the 1/sum), row constants
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        *reinterpret_cast<__attribute__((address_space(3))) hvk_u32x2*>(
            (__attribute__((address_space(3))) char*)(size_t)(pimg + pimg_byte<ROWS>(pq, 8 * c + g4))) =
            hvk_u32x2{pf[c].x, pf[c].y};
        if (2 * c + 1 < NT)
          *reinterpret_cast<__attribute__((address_space(3))) hvk_u32x2*>(
              (__attribute__((address_space(3))) char*)(size_t)(pimg + pimg_byte<ROWS>(pq, 8 * c + 4 + g4))) =
              hvk_u32x2{pf[c].z, pf[c].w};
      }
      if (g4 == 0)  // delta/sum^2 * scale: phase B's dS = p * (dP/sum * scale - this)
        *reinterpret_cast<__attribute__((address_space(3))) float*>((__attribute__((address_space(3))) char*)(size_t)(dlt + 4 * pq)) =
            du * inv * inv * scale;
      {  // dO / sum in place (own rows; zero rows of padding stay zero)
        float f[8];
        hvk_unpack8(df[j], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] *= inv;
        lds_st16(ad(qi), hvk_pack8(f));
      }
      // dQ^T = K^T (scale dS^T)
      hvk_f32x4 dq[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bool has1 = 2 * c + 1 < NT;
        const uint4 bf = make_uint4(dsp[2 * c][0], dsp[2 * c][1], has1 ? dsp[2 * c + 1][0] : 0u,
                                    has1 ? dsp[2 * c + 1][1] : 0u);
        dq[0] = hvk_mfma16(kt_frag[c][0], bf, dq[0]);
        dq[1] = hvk_mfma16(kt_frag[c][1], bf, dq[1]);
      }
      // normalize backward: dq = (dq^ - q^ (q^ . dq^)) / max(||q||, eps); q^ rows in
      // accumulator layout (8-B piece 4dt + gq of position pq)
      float qh[2][4], dot = 0.f;
      const uint32_t arow = aq(qi, 0) - 8 * g4;  // 8-B piece gq (+4 dt) of the q segment
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint2 v = lds_ld8(arow + 32 * dt);
        qh[dt][0] = hvk_lo(v.x); qh[dt][1] = hvk_hi(v.x);
        qh[dt][2] = hvk_lo(v.y); qh[dt][3] = hvk_hi(v.y);
#pragma unroll
        for (int r = 0; r < 4; ++r) dot += qh[dt][r] * dq[dt][r];
      }
      dot = hvk_group4_sum(dot);
      if (rnq[j] >= 1e12f) dot = 0.f;  // ||q|| <= eps: x / eps, no projection term
      uint2 pk[2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = (dq[dt][r] - qh[dt][r] * dot) * rnq[j];
          if (qreal) dqb[dt][r] += v[r];
        }
        pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
      }
      const uint4 o = hvk_pair_swap(pk[0], pk[1]);  // all lanes: cross-lane
      hvk_bst16(r_dqkv, row[j] < 0 ? HVK_OOB : (uint32_t)(row[j] * C3 + h * 32 + hvk_pair_col(gq)) * 2, o);
    }
    RSTAMP(5);  // phase A
    lds_barrier();  // P images, row constants, dO/sum complete
    RSTAMP(4);

    // ---------------- phase B: own key tiles, key on the lane
    uint4 dof[NT];  // (dO/sum) rows, A operand of dP^T recomputation
#pragma unroll
    for (int t = 0; t < NT; ++t) dof[t] = lds_ld16(fd[t]);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int kt = hf + 2 * j;
      if (kt >= NT) break;
      __builtin_amdgcn_sched_barrier(0);
      // dP'[q][key] = (dO/sum) . V for this key tile, all query tiles (query rows 4gq + r)
      hvk_f32x4 dpb[NT];
      const uint4 vk = lds_ld16(aq(kt, 2));
#pragma unroll
      for (int t = 0; t < NT; ++t) dpb[t] = hvk_mfma16(dof[t], vk, hvk_f32x4{0, 0, 0, 0});
      hvk_f32x4 dv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, dk[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        // P^T fragment: rows 32c + 4gq + li/4 (+16), column 16kt + li
        const int prow = 32 * c + 4 * g4 + (l16 >> 2);
        const uint32_t plo = pimg + pimg_byte<ROWS>(prow, 4 * kt + (l16 & 3));
        const uint32_t phi = pimg + pimg_byte<ROWS>(prow + 16, 4 * kt + (l16 & 3));
        const uint2 lo = lds_tr8(plo), hi = lds_tr8(phi);
        const uint4 pfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
        // scale*dS = p * (dP' * scale - delta'), rows 32c + 4gq + r and 32c + 16 + 4gq + r
        const hvk_f32x4 d0 = lds_ld4f(dlt + 4 * (32 * c + 4 * g4));
        const bool has1 = 2 * c + 1 < NT;
        const hvk_f32x4 d1 = has1 ? lds_ld4f(dlt + 4 * (32 * c + 16 + 4 * g4)) : hvk_f32x4{0, 0, 0, 0};
        const float pv[8] = {hvk_lo(pfr.x), hvk_hi(pfr.x), hvk_lo(pfr.y), hvk_hi(pfr.y),
                             hvk_lo(pfr.z), hvk_hi(pfr.z), hvk_lo(pfr.w), hvk_hi(pfr.w)};
        float ds[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ds[r] = pv[r] * fmaf(dpb[2 * c][r], scale, -d0[r]);
          ds[4 + r] = has1 ? pv[4 + r] * fmaf(dpb[2 * c + 1][r], scale, -d1[r]) : 0.f;
        }
        const uint4 dsfr = make_uint4(hvk_pack2(ds[0], ds[1]), hvk_pack2(ds[2], ds[3]), hvk_pack2(ds[4], ds[5]),
                                      hvk_pack2(ds[6], ds[7]));
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          uint2 l2 = lds_tr8(trd[c][0] + 32 * dt), h2 = lds_tr8(trd[c][1] + 32 * dt);
          dv[dt] = hvk_mfma16(make_uint4(l2.x, l2.y, h2.x, h2.y), pfr, dv[dt]);
          l2 = lds_tr8(trq[c][0] + 32 * dt);
          h2 = lds_tr8(trq[c][1] + 32 * dt);
          dk[dt] = hvk_mfma16(make_uint4(l2.x, l2.y, h2.x, h2.y), dsfr, dk[dt]);
        }
      }
      // dk normalize backward with k^ rows of position 16kt + li
      const uint32_t krow = aq(kt, 1) - 8 * g4;
      float kh[2][4], dot = 0.f;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const uint2 v = lds_ld8(krow + 32 * dt);
        kh[dt][0] = hvk_lo(v.x); kh[dt][1] = hvk_hi(v.x);
        kh[dt][2] = hvk_lo(v.y); kh[dt][3] = hvk_hi(v.y);
#pragma unroll
        for (int r = 0; r < 4; ++r) dot += kh[dt][r] * dk[dt][r];
      }
      dot = hvk_group4_sum(dot);
      if (rnk[j] >= 1e12f) dot = 0.f;
      uint2 pk[2], pv2[2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (dk[dt][r] - kh[dt][r] * dot) * rnk[j];
        pk[dt] = make_uint2(hvk_pack2(v[0], v[1]), hvk_pack2(v[2], v[3]));
        pv2[dt] = make_uint2(hvk_pack2(dv[dt][0], dv[dt][1]), hvk_pack2(dv[dt][2], dv[dt][3]));
      }
      st_k[j] = hvk_pair_swap(pk[0], pk[1]);
      st_v[j] = hvk_pair_swap(pv2[0], pv2[1]);
      st_off[j] = row[j] < 0 ? HVK_OOB : (uint32_t)(row[j] * C3 + C + h * 32 + hvk_pair_col(gq)) * 2;
    }
    RSTAMP(6);  // phase B
  }
#ifdef HVK_STAMPS
  if (lane == 0)
    for (int k = 0; k < 7; ++k) atomicAdd(&g_ring_bwd_stamps[k], st_acc[k]);
  if (lane == 0) atomicAdd(&g_ring_bwd_stamps[7], 1ull);
#endif
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    hvk_bst16(r_dqkv, st_off[j], st_k[j]);
    hvk_bst16(r_dqkv, st_off[j] + 2 * C, st_v[j]);
  }

  // ---- dbias / dscale (carried as scale*dS) and dq_bias: reduce over the workgroup, then one
  // atomic per entry.  The last window's readers are past the loop's final barrier only after
  // this one.
  __syncthreads();
  const float inv_scale = 1.f / scale;
  float* red = reinterpret_cast<float*>(smem) + hl * K::TAB;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int qi = hf + 2 * j;
    if (qi >= NT) break;
#pragma unroll
    for (int ki = 0; ki < NT; ++ki)
      *reinterpret_cast<float4*>(red + ((qi * NT + ki) * 64 + lane) * 4) =
          make_float4(dbias[j][ki][0], dbias[j][ki][1], dbias[j][ki][2], dbias[j][ki][3]);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < HG * K::TAB; e += 128 * HG) {
    const int hh = e / K::TAB;
    atomicAdd(a.dbias_acc + (size_t)(grp * HG + hh) * K::TAB + e % K::TAB,
              reinterpret_cast<const float*>(smem)[e] / a.scale[grp * HG + hh]);
  }
  dscale = hvk_wave_sum(dscale);
  if (lane == 0) atomicAdd(a.dscale_acc + h, dscale * inv_scale);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = hvk_row16_sum(dqb[dt][r]);
      if (li == 0) atomicAdd(a.dqb_acc + h * 32 + 16 * dt + 4 * gq + r, v);
    }
}

// Fold the accumulator-order partial sums over 8-wide grid positions into the CPB-table
// gradient [nH, R*R], write dscale / dq_bias, and leave the workspace zero.
template <int WIN>
__global__ __launch_bounds__(256) void wmsa_ring_bwd_finalize(BwdArgs a, float* __restrict__ dtab,
                                                             float* __restrict__ dscale,
                                                             float* __restrict__ dqb) {
  constexpr int R = 2 * WIN - 1, NT = (WIN * 8 + 15) / 16, TAB = NT * NT * 256;
  __shared__ float bins[R * R];
  const int h = blockIdx.x;
  for (int i = threadIdx.x; i < R * R; i += blockDim.x) bins[i] = 0.f;
  __syncthreads();
  float* acc = a.dbias_acc + (size_t)h * TAB;
  for (int e = threadIdx.x; e < TAB; e += blockDim.x) {
    const int r = e & 3, lane = (e >> 2) & 63, blk = e >> 8;
    const int qi = blk / NT, ki = blk % NT;
    const int pq = 16 * qi + (lane & 15), pk = 16 * ki + 4 * (lane >> 4) + r;
    const int qy = pq >> 3, qx = pq & 7, ky = pk >> 3, kx = pk & 7;
    if (qy < WIN && qx < WIN && ky < WIN && kx < WIN)
      atomicAdd(&bins[(qy - ky + WIN - 1) * R + (qx - kx + WIN - 1)], acc[e]);
    acc[e] = 0.f;
  }
  finalize_scale_qb(a.dscale_acc, a.dqb_acc, dscale, dqb, h);
  __syncthreads();
  for (int i = threadIdx.x; i < R * R; i += blockDim.x) dtab[(size_t)h * R * R + i] = bins[i];
}

template <int WIN, int HG>
int launch_ring_bwd(BwdArgs a, float* dbias_table, float* dscale, float* dq_bias, hipStream_t st) {
  using K = RBCfg<WIN, HG>;
  const int ng = a.g.nH / HG;
  int chunks = 512 / ng / 8 * 8;  // two resident workgroups per CU
  if (chunks < 8) chunks = 8;
  const int need = (a.g.n_windows + 7) / 8 * 8;
  a.g.n_chunks = chunks < need ? chunks : need;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wmsa_bwd_ring_kernel<WIN, HG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    attr = true;
  }
  // the dQ/dK/dV buffer descriptor spans < 2^31 bytes: batch slices when qkv is larger
  const size_t img = (size_t)a.g.H * a.g.W * 3 * a.g.C * 2;
  const int per = (int)(((size_t)1 << 31) / img);
  if (per < 1) return hvk_set_error(HVK_EUNSUPPORTED, "hvk_wmsa_bwd: one image's qkv exceeds 2 GiB");
  const size_t tok = (size_t)a.g.H * a.g.W;
  for (int b0 = 0; b0 < a.g.B; b0 += per) {
    BwdArgs s = a;
    s.g.B = a.g.B - b0 < per ? a.g.B - b0 : per;
    s.g.n_windows = s.g.B * a.g.nWh * a.g.nWw;
    const int nd = (s.g.n_windows + 7) / 8 * 8;
    if (s.g.n_chunks > nd) s.g.n_chunks = nd;
    s.qkv += b0 * tok * 3 * a.g.C;
    s.dout += b0 * tok * a.g.C;
    s.dqkv += b0 * tok * 3 * a.g.C;
    HVK_LAUNCH_TIMED(HVK_TIMER_WMSA_BWD, (wmsa_bwd_ring_kernel<WIN, HG>), dim3(s.g.n_chunks / 8 * 8 * ng),
                     dim3(128 * HG), K::LDS, st, s);
  }
  HVK_CHECK_LAUNCH("wmsa_bwd_ring");
  hipLaunchKernelGGL(wmsa_ring_bwd_finalize<WIN>, dim3(a.g.nH), dim3(256), 0, st, a, dbias_table, dscale, dq_bias);
  HVK_CHECK_LAUNCH("wmsa_ring_bwd_finalize");
  return HVK_OK;
}

}  // namespace

#ifdef HVK_STAMPS
extern "C" int hvk_debug_ring_bwd_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ring_bwd_stamps), 8 * sizeof(unsigned long long)) != hipSuccess)
    return HVK_EINVAL;
  const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ring_bwd_stamps), z, sizeof(z)) == hipSuccess ? HVK_OK : HVK_EINVAL;
}
#endif

namespace hvk_wmsa {
// windows 6 / 7 with an even head count; anything else: HVK_EUNSUPPORTED (the caller falls back
// to the pair kernel).  HVK_WMSA_BWD_RING=0 disables it (A/B runs).
int ring_bwd(const BwdArgs& a, int win, float* dbias_table, float* dscale, float* dq_bias, hipStream_t st) {
  static const bool on = [] {
    const char* e = getenv("HVK_WMSA_BWD_RING");
    return !e || atoi(e) != 0;
  }();
  if (!on || a.g.nH % 2) return HVK_EUNSUPPORTED;
  switch (win) {
    case 7: return launch_ring_bwd<7, 2>(a, dbias_table, dscale, dq_bias, st);
    case 6: return launch_ring_bwd<6, 2>(a, dbias_table, dscale, dq_bias, st);
    default: return HVK_EUNSUPPORTED;
  }
}
}  // namespace hvk_wmsa
