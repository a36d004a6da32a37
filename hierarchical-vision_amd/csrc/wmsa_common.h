// Shared pieces of the W-MSA kernels (wmsa.hip: windows <= 8, wmsa_large.hip: 12/16/24).
#pragma once
#include "hvk_common.h"
#include <type_traits>

namespace hvk_wmsa {

struct WmsaGeom {
  int B, H, W, C, nH, shift;
  int nWh, nWw, n_windows;   // windows per image row/col, total windows (B*nWh*nWw)
  int n_chunks;              // window chunks per head (multiple of 8: XCD groups)
  int xcd_runs;              // 1: (chunk, head) items dealt to the 8 XCDs in contiguous runs of
                             //    ceil(items / 8) (any n_chunks), 0: hvk_decode_chunk_head
};

// workgroup -> (chunk, head); false for the padded grid's surplus workgroups
__device__ __forceinline__ bool decode_item(const WmsaGeom& g, int bid, int& chunk, int& head) {
  if (g.xcd_runs) {
    const int items = g.n_chunks * g.nH, per = (items + 7) >> 3;
    const int item = (bid & 7) * per + (bid >> 3);
    if ((bid >> 3) >= per || item >= items) return false;
    chunk = item / g.nH;
    head = item % g.nH;
    return true;
  }
  hvk_decode_chunk_head(bid, g.nH, chunk, head);
  return chunk < g.n_chunks;
}

// token row (in the un-shifted [B*H*W] token order) of window position t
__device__ __forceinline__ int window_token_row(const WmsaGeom& g, int b, int wh, int ww, int win,
                                                int t) {
  int y = wh * win + t / win + g.shift;
  int x = ww * win + t % win + g.shift;
  if (y >= g.H) y -= g.H;
  if (x >= g.W) x -= g.W;
  return (int)HVK_BCHECK((b * g.H + y) * g.W + x, (long long)g.B * g.H * g.W);
}

// L2-normalise one 8-wide slice of a 32-wide head row spread over lanes l, l^16, l^32, l^48.
// The squared norm as a sequential f32 sum of squares (the large-window kernels: their
// whole-step test against the reference sits close to its logit-scale gradient bound, so their
// rounding stays as measured there)
__device__ __forceinline__ uint4 l2_normalize_seq(uint4 v, float& rnorm, float post = 1.f) {
  float f[8];
  hvk_unpack8(v, f);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
  ss = hvk_group4_sum(ss);
  rnorm = __builtin_amdgcn_rsqf(fmaxf(ss, 1e-24f));
  const float m = rnorm * post;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] *= m;
  return hvk_pack8(f);
}

// Windows <= 8 (forward and backward alike): the squared norm from four v_dot2_f32_bf16 on the
// packed pairs (f32 accumulation), 8 fewer VALU instructions per 8-channel slice.
__device__ __forceinline__ uint4 l2_normalize(uint4 v, float& rnorm, float post = 1.f) {
  typedef __bf16 hvk_bf16x2 __attribute__((ext_vector_type(2)));
  auto d2 = [](uint32_t w, float c) {
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(hvk_bf16x2, w), __builtin_bit_cast(hvk_bf16x2, w), c, false);
  };
  float ss = d2(v.w, d2(v.z, d2(v.y, d2(v.x, 0.f))));
  float f[8];
  hvk_unpack8(v, f);
  ss = hvk_group4_sum(ss);
  // F.normalize: x / max(||x||, eps) == x * rsqrt(max(||x||^2, eps^2))
  rnorm = __builtin_amdgcn_rsqf(fmaxf(ss, 1e-24f));
  const float m = rnorm * post;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] *= m;
  return hvk_pack8(f);
}

// LDS images [rows][32] bf16 in "fragment-major" order: the 16-B unit (row, u) of a 16-row
// tile sits at slot 16u + (row%16 ^ 12*(u&1)), so the natural MFMA operand read
// (ds_read_b128, lane = row%16 + 16u), 16-B staging writes, 8-B row reads and the
// transposed read (ds_read_b64_tr_b16) are all bank-conflict free (LDS bank model of
// MI355X_MICROARCH.md, searched exhaustively).
__device__ __forceinline__ int fm16(int row, int u) {  // byte offset of 16-B unit u of `row`
  return ((row >> 4) * 64 + 16 * u + ((row & 15) ^ ((u & 1) * 12))) << 4;
}
__device__ __forceinline__ int fm8(int row, int col8) {  // byte offset of 8-B unit col8
  return fm16(row, col8 >> 1) + ((col8 & 1) << 3);
}
// LDS byte address of a pointer into dynamic shared memory
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
// LDS access through explicit 32-bit LDS addresses (address-space-3 pointers), so a few base
// registers laundered per loop iteration plus compile-time offsets address every fragment
typedef __attribute__((address_space(3))) const char lds_cchar;
__device__ __forceinline__ lds_cchar* lds_ptr(uint32_t a) { return (lds_cchar*)(size_t)a; }
__device__ __forceinline__ uint4 lds_ld16(uint32_t a) {
  return __builtin_bit_cast(uint4, *reinterpret_cast<const __attribute__((address_space(3))) hvk_u32x4*>(lds_ptr(a)));
}
__device__ __forceinline__ hvk_f32x4 lds_ld4f(uint32_t a) {  // 4 consecutive floats (2 x ds_read2_b32)
  const __attribute__((address_space(3))) float* f = reinterpret_cast<const __attribute__((address_space(3))) float*>(lds_ptr(a));
  return hvk_f32x4{f[0], f[1], f[2], f[3]};
}
__device__ __forceinline__ uint2 lds_tr8(uint32_t a) {
  hvk_i16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) hvk_i16x4*)(lds_ptr(a)));
  return __builtin_bit_cast(uint2, r);
}
__device__ __forceinline__ uint32_t launder(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ uint2 lds_ld8(uint32_t a) {
  return __builtin_bit_cast(uint2, *reinterpret_cast<const __attribute__((address_space(3))) hvk_u32x2*>(lds_ptr(a)));
}
__device__ __forceinline__ void lds_st16(uint32_t a, uint4 v) {
  *reinterpret_cast<__attribute__((address_space(3))) hvk_u32x4*>((__attribute__((address_space(3))) char*)(size_t)a) =
      __builtin_bit_cast(hvk_u32x4, v);
}
// LDS-DMA of 16 B per lane (global_load_lds_dwordx4) from inline asm: the compiler does not see
// it, so it adds no conservative vmcnt(0) before later LDS reads; the caller waits (counted
// vmcnt) before the barrier that publishes the destination.  base and m0 are wave-uniform.
__device__ __forceinline__ void dma16(const void* base, uint32_t voff, uint32_t m0) {
  // the base and m0 are wave-uniform: make them scalar for the "s" operands
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               :: "s"(__builtin_amdgcn_readfirstlane(m0)), "v"(voff), "s"((const void*)bs) : "memory");
}

// barrier without the vmcnt(0) a __syncthreads() fence adds (prefetched global loads and
// LDS-DMA stay in flight); LDS writes before it are waited for
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ uint4 lds16(const char* img, int off) {
  return *reinterpret_cast<const uint4*>(img + off);
}

// n / d for 0 <= n < 2^31 by a multiply-high (d >= 1 fixed at launch; host-side init):
// s = ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1, q = (mulhi(n, m) + n) >> s
struct FastDiv {
  uint32_t m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FastDiv{(uint32_t)m, s};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
  return (uint32_t)(((uint64_t)__umulhi(n, f.m) + n) >> f.s);
}

struct FwdArgs {
  const hvk_bf16* qkv;       // [T, 3C]  x Wqkv^T + (q_bias, 0, 0)
  hvk_bf16* out;             // [T, C]
  const float* bias;         // [nH, R*R]   16*sigmoid(cpb)
  const float* scale;        // [nH]        exp(clamp(logit_scale))
  float* lse;                // [T, nH] or null: per query, log2 of the softmax denominator of the
                             // log2e-scaled logits (the large-window backward's row constant)
  WmsaGeom g;
  FastDiv fd_groups, fd_img, fd_ww;  // wmsa_win.hip: / (nH / HG), / (nWh nWw), / nWw
  int dma_nt;                         // wmsa_win.hip: slab DMA with the nontemporal hint
  int qk_normed;             // 1: q^ * scale * log2e and k^ arrive from the qkv GEMM's EPI 4
};

struct BwdArgs {
  const hvk_bf16* qkv;       // [T, 3C]  x Wqkv^T + (q_bias, 0, 0)
  const hvk_bf16* dout;      // [T, C]   gradient of the attention core output
  const hvk_bf16* out;       // [T, C]   the forward's output O (large windows: delta = dO . O)
  const float* lse;          // [T, nH]  the forward's row constants L2 (FwdArgs::lse), or null
  hvk_bf16* dqkv;            // [T, 3C]
  const float* bias;         // [nH, R*R]
  const float* scale;        // [nH]
  // workspace (zero on entry, re-zeroed by the finalize kernel): one slot of
  // bwd_slot_floats(win) = R*R CPB-table bins + d scale + 32 d q_bias per (head, chunk), written by
  // the workgroup that owns (chunk, head) -- its partial sums folded in a fixed order, added to the
  // slot without atomics -- and summed over chunks in chunk order by the finalize kernel, so
  // every parameter gradient is deterministic (no float atomics in any order)
  float* dbias_acc;          // [nH][slot_stride][bwd_slot_floats(win)]
  int slot_stride;           // slots per head (>= n_chunks of every launch over this workspace)
  int slot_add;              // 0: the first launch over the workspace in this call stores its slots
                             // (no load); 1: a later batch slice adds to them in stream order
  const float* rn;           // [T, 2nH] 1/max(||q||, eps), 1/max(||k||, eps) when q and k arrive
                             // normalised, q as q^ * scale * log2e (windows <= 8); null: raw q, k
  WmsaGeom g;
};

// Persistent grid: n_heads * n_chunks <= `capacity` resident workgroups (no tail round),
// n_chunks a multiple of 8 so every XCD group holds whole (chunk, all heads) sets.
inline int make_geom(int B, int H, int W, int C, int nH, int win, int shift, int capacity, WmsaGeom& g) {
  if (B <= 0 || H <= 0 || W <= 0 || nH <= 0)
    return hvk_set_error(HVK_EINVAL, "wmsa: bad shape B=%d H=%d W=%d nH=%d", B, H, W, nH);
  if (C != 32 * nH)
    return hvk_set_error(HVK_EUNSUPPORTED, "wmsa: head_dim must be 32 (C=%d, nH=%d)", C, nH);
  if (H % win || W % win)
    return hvk_set_error(HVK_EINVAL, "wmsa: H=%d W=%d not divisible by window %d", H, W, win);
  if (shift < 0 || shift >= win)
    return hvk_set_error(HVK_EINVAL, "wmsa: shift %d outside [0, %d)", shift, win);
  g.B = B; g.H = H; g.W = W; g.C = C; g.nH = nH; g.shift = shift;
  g.nWh = H / win; g.nWw = W / win;
  g.n_windows = B * g.nWh * g.nWw;
  int chunks = capacity / nH / 8 * 8;
  if (chunks < 8) chunks = 8;
  const int need = (g.n_windows + 7) / 8 * 8;  // never more chunks than windows (rounded)
  g.n_chunks = chunks < need ? chunks : need;
  g.xcd_runs = 0;
  return HVK_OK;
}

// large-window path (wmsa_large.hip): one workgroup per (window, head)
bool large_window(int win);
int large_fwd(const FwdArgs& a, int win, hipStream_t st);
// backward + finalize: dbias_table [nH, R*R], dscale [nH], dq_bias [C] (may be null)
int large_bwd(const BwdArgs& a, int win, float* dbias_table, float* dscale, float* dq_bias,
              hipStream_t st);

// windows <= 8, forward (wmsa_ring.hip): one persistent workgroup per (window chunk, head
// group), window slabs staged by LDS-DMA
int ring_fwd(FwdArgs& a, int B, int H, int W, int C, int nH, int win, int shift, hipStream_t st);
// windows <= 8, forward (wmsa_win.hip): one workgroup per (window, head group), one LDS-DMA
// burst per window, output rows stored from LDS
int win_fwd(FwdArgs& a, int B, int H, int W, int C, int nH, int win, int shift, hipStream_t st);

// backward workspace: per (head, chunk) slot, R*R bins then d scale then 32 d q_bias
__host__ __device__ constexpr int bwd_slot_floats(int win) { return (2 * win - 1) * (2 * win - 1) + 33; }
// slots per head: the most chunks a launch over nH heads uses (wmsa_bwd: 512 / nH for windows
// <= 8, make_geom's 256-workgroup plan for the large windows)
#ifndef HVK_BWD_SLOTS  // w <= 8 backward: workgroups per launch the chunk count aims at (A/B build switch)
#define HVK_BWD_SLOTS 512
#endif
// slots per head of the backward workspace = the chunk count of the w <= 8 launch (at most)
inline int bwd_slot_stride(int num_heads, bool large) {
  if (num_heads <= 0) return 1;
  if (large) {
    const int c = 256 / num_heads / 8 * 8;
    return c < 8 ? 8 : c;
  }
  const int c = HVK_BWD_SLOTS / num_heads;
  return c < 1 ? 1 : c;
}

// finalize: sum the head's slots into the CPB-table gradient [nH, R*R], d scale [nH] and d q_bias
// [C] (may be null), and leave the slots zero.  Block (h, group): FIN_ENTRIES slot entries x
// FIN_GROUPS chunk groups; thread (group g, entry e) sums the chunks c = g, g + FIN_GROUPS, ... in
// order (independent loads in flight), the groups are then added in group order through LDS -- a
// fixed order, so the result is the same bits every run.  (One block per head walking every chunk
// in turn took 17.6 us per launch at 170 chunks, 12 launches per SwinV2-T step.)
constexpr int FIN_ENTRIES = 16, FIN_GROUPS = 16, FIN_THREADS = FIN_ENTRIES * FIN_GROUPS;
__host__ __device__ constexpr int finalize_blocks_y(int win) {
  return (bwd_slot_floats(win) + FIN_ENTRIES - 1) / FIN_ENTRIES;
}
template <int WIN>
__device__ __forceinline__ void finalize_slots(const BwdArgs& a, float* dtab, float* dscale, float* dqb, int h,
                                               int grp) {
  constexpr int RR = (2 * WIN - 1) * (2 * WIN - 1), SLOT = bwd_slot_floats(WIN);
  __shared__ float part[FIN_GROUPS][FIN_ENTRIES];
  const int e = threadIdx.x % FIN_ENTRIES, g = threadIdx.x / FIN_ENTRIES;
  const int i = grp * FIN_ENTRIES + e;
  float* base = a.dbias_acc + (size_t)h * a.slot_stride * SLOT;
  float v = 0.f;
  if (i < SLOT) {
    constexpr int U = 4;
    int c = g;
    for (; c + (U - 1) * FIN_GROUPS < a.slot_stride; c += U * FIN_GROUPS) {
      float t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) t[u] = base[(size_t)(c + u * FIN_GROUPS) * SLOT + i];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v += t[u];
        base[(size_t)(c + u * FIN_GROUPS) * SLOT + i] = 0.f;
      }
    }
    for (; c < a.slot_stride; c += FIN_GROUPS) {
      v += base[(size_t)c * SLOT + i];
      base[(size_t)c * SLOT + i] = 0.f;
    }
  }
  part[g][e] = v;
  __syncthreads();
  if (g == 0 && i < SLOT) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < FIN_GROUPS; ++k) s += part[k][e];
    if (i < RR) dtab[(size_t)h * RR + i] = s;
    else if (i == RR) dscale[h] = s;
    else if (dqb) dqb[h * 32 + i - RR - 1] = s;
  }
}

// reduce v over the 16 lanes sharing lane>>4 (xor 1, 2, 4, 8)
__device__ __forceinline__ float hvk_row16_sum(float v) {
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

}  // namespace hvk_wmsa
