// Shared pieces of the LDS-DMA slab W-MSA forward for windows <= 8 (wmsa_ring.hip):
// slab geometry, inline-asm LDS reads, compact bias gathers.
#pragma once
#include "wmsa_common.h"

namespace hvk_ring {
using namespace hvk_wmsa;

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* gbl_vptr;

constexpr int gcd(int a, int b) { return b == 0 ? a : gcd(b, a % b); }

template <int WIN, int HG>
struct RingCfg {
  static constexpr int PW = WIN <= 4 ? 4 : 8;        // grid width of a window in the tiles
  static constexpr int N = WIN * WIN;                // real tokens
  static constexpr int NT = (WIN * PW + 15) / 16;    // 16-row tiles
  static constexpr int NC = (NT + 1) / 2;            // 32-key chunks (one MFMA K-step)
  static constexpr int R = 2 * WIN - 1;
  static constexpr int TR = (16 / PW) * R;           // index step per tile
  static constexpr int RS = 12 * HG;                 // 16-B slots per token in the slab
  // the slab is WIN runs (window rows) of IPR DMA instructions: a run holds the WIN tokens of
  // one window row (adjacent in memory), so a lane's (token column, part, 16-B column) is the
  // same for instruction m of every run, of every window
  static constexpr int IPR = (WIN * RS + 63) / 64;   // DMA wave-instructions per run
  static constexpr int RUN = IPR * 64;               // slots per run
  static constexpr int NINST = WIN * IPR;            // DMA wave-instructions per slab
  static constexpr int SLAB = NINST * 1024;
  static constexpr int NK = (NINST + HG - 1) / HG;   // DMA instructions per wave
  static constexpr int KP = IPR / gcd(HG, IPR);      // period of instruction m over a wave's k
  // compact bias table per head: R*R entries (x log2e) inside zero padding that absorbs the
  // (never used) indices of padded grid positions
  static constexpr int LQMAX = PW == 8 ? R + 7 : 3 * R + 3;
  static constexpr int LKMAX = PW == 8 ? R + 4 : 3 * R;
  static constexpr int BASE0 = (WIN - 1) * (R + 1);
  static constexpr int LO = BASE0 - LKMAX - TR * (NT - 1) - 3;   // smallest index read
  static constexpr int PAD = LO < 0 ? -LO : 0;
  static constexpr int HI = BASE0 + LQMAX + TR * (NT - 1);       // largest index read
  static constexpr int TABF = ((PAD + (HI + 1 > R * R ? HI + 1 : R * R) + 3) / 4) * 4;
  static constexpr int LDS = SLAB + 16 + HG * TABF * 4;
  // padding key slots (grid position x >= WIN or y >= WIN) of MFMA slot bit ki*4 + r for the
  // lanes with lane/16 == gq, in bits 16*gq .. 16*gq + 15
  static constexpr unsigned long long kpad_bits() {
    unsigned long long v = 0;
    for (int gq = 0; gq < 4; ++gq)
      for (int ki = 0; ki < NT; ++ki)
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * ki + 4 * gq + r;
          if (p % PW >= WIN || p / PW >= WIN) v |= 1ull << (16 * gq + ki * 4 + r);
        }
    return v;
  }
  static constexpr unsigned long long KPAD = kpad_bits();
  static_assert(NT <= 4, "window larger than 8 needs the large-window kernels");
};

// LDS reads issued from inline asm: the compiler's waitcnt pass does not see them, so it
// cannot add the conservative vmcnt(0) it inserts before LDS reads while an LDS-DMA may be
// pending (that would also wait for this workgroup's outstanding output stores).  The caller
// waits lgkmcnt(0) and then ties the results (lds_fence).
template <int OFF>
__device__ __forceinline__ hvk_u32x4 lds_rd128(uint32_t a) {
  hvk_u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ hvk_u32x2 lds_rd64_tr(uint32_t a) {
  hvk_u32x2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int O0, int O1>
__device__ __forceinline__ hvk_u32x2 lds_rd2(uint32_t a) {
  hvk_u32x2 r;
  asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(r) : "v"(a), "i"(O0), "i"(O1));
  return r;
}
template <typename T>
__device__ __forceinline__ void lds_fence(T& v) {
  asm volatile("" : "+v"(v));
}
__device__ __forceinline__ uint4 u4(hvk_u32x4 v) { return make_uint4(v[0], v[1], v[2], v[3]); }

// output row segment store: plain (default) or nontemporal (HVK_RING_NT_STORE, A/B builds)
__device__ __forceinline__ void ring_store(hvk_bf16* dst, uint4 v) {
#ifdef HVK_RING_NT_STORE
  __builtin_nontemporal_store(__builtin_bit_cast(hvk_u32x4, v), reinterpret_cast<hvk_u32x4*>(dst));
#else
  *reinterpret_cast<uint4*>(dst) = v;
#endif
}

// the 2*NT ds_read2_b32 of one query tile's bias C operands (compile-time offsets)
template <int TR, int NT, int QI, int KI = 0>
__device__ __forceinline__ void ring_bias_read(hvk_u32x2 (&br)[NT][2], uint32_t a) {
  if constexpr (KI < NT) {
    constexpr int off = TR * (NT - 1 - QI + KI);
    br[KI][0] = lds_rd2<off, off + 1>(a);
    br[KI][1] = lds_rd2<off + 2, off + 3>(a);
    ring_bias_read<TR, NT, QI, KI + 1>(br, a);
  }
}
template <int TR, int NT>
__device__ __forceinline__ void ring_bias_read_q(hvk_u32x2 (&br)[NT][2], uint32_t a, int qi) {
  if constexpr (NT > 0) if (qi == 0) ring_bias_read<TR, NT, 0>(br, a);
  if constexpr (NT > 1) if (qi == 1) ring_bias_read<TR, NT, (NT > 1 ? 1 : 0)>(br, a);
  if constexpr (NT > 2) if (qi == 2) ring_bias_read<TR, NT, (NT > 2 ? 2 : 0)>(br, a);
  if constexpr (NT > 3) if (qi == 3) ring_bias_read<TR, NT, (NT > 3 ? 3 : 0)>(br, a);
}

// hvk_settle over a query tile's NT score tiles (the unmasked-window path branches over the mask
// code straight to the exp2 that reads them; hvk_common.h)
template <int NT>
__device__ __forceinline__ void settle_tiles(hvk_f32x4 (&s)[NT]) {
  if constexpr (NT == 1) hvk_settle(s[0]);
  if constexpr (NT == 2) hvk_settle(s[0], s[1]);
  if constexpr (NT == 3) hvk_settle(s[0], s[1], s[2]);
  if constexpr (NT == 4) hvk_settle(s[0], s[1], s[2], s[3]);
}

// padded-grid position -> window token (-1 for padding)
template <int WIN, int PW>
__device__ __forceinline__ int grid_token(int p) {
  const int y = p / PW, x = p % PW;
  return (x < WIN && y < WIN) ? y * WIN + x : -1;
}

}  // namespace hvk_ring
