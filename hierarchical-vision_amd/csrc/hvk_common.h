// Shared device helpers for libhvk (gfx950 / CDNA4 only).
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>

typedef __bf16 hvk_bf16x8 __attribute__((ext_vector_type(8)));
typedef float hvk_f32x4 __attribute__((ext_vector_type(4)));
typedef short hvk_i16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short hvk_bf16;  // raw bf16 bits in memory

#define HVK_LOG2E 1.4426950408889634f
#define HVK_LDS_I16X4(p) ((__attribute__((address_space(3))) hvk_i16x4*)(p))

// ---- host-side status plumbing (defined in capi.hip) ----------------------
#ifdef __cplusplus
extern "C" {
#endif
__attribute__((visibility("hidden"))) int hvk_set_error(int code, const char* fmt, ...);
#ifdef __cplusplus
}
#endif

// ---- library options (capi.hip): a fixed table set only through hvk_set_option (include/hvk.h);
// libhvk reads no environment variable.  Each option that changes a result has a GPU test.
enum HvkOption {
  HVK_OPT_WMSA_FWD_FORM = 0,    // w <= 8 forward: 0 one workgroup per (window, head group), 1 ring
  HVK_OPT_WMSA_BWD_NT,          // w <= 8 backward qkv reads: 0 cached, 1 nontemporal, 2 nt past 256 MB
  HVK_OPT_WMSA_BWD_SLICE_BYTES, // w <= 8 backward: batch slice so one launch's qkv stays below this
  HVK_OPT_TILE_WIDE,            // tiled GEMM: -1 by shape, 0 128-column, 1 192-column tiles
  HVK_OPT_DW_TILE,              // weight gradient, 192-multiple shapes: tile variant 4..8
  HVK_OPT_WMSA_FWD_HG,          // w <= 8 forward (win form): heads per workgroup, 0 by head count, else 1 / 2 / 3 / 4 / 6
  HVK_OPT_DW_CHUNKS,            // weight gradient: workgroup target per launch (token chunks = target / output tiles)
  HVK_OPT_COUNT
};
long long hvk_opt(int id);
#ifdef __cplusplus
extern "C" {
#endif
int hvk_set_option(const char* name, long long value, long long* previous);
#ifdef __cplusplus
}
#endif

#define HVK_OK 0
#define HVK_EINVAL 1
#define HVK_EUNSUPPORTED 2
#define HVK_EHIP 3

// ---- opt-in kernel timer (capi.hip): start/stop events recorded by the dispatch packet
// itself (hipExtLaunchKernelGGL), so a duration is the kernel's execution only, like a
// rocprofv3 kernel trace (HIP events around a launch also count the dispatch gap).
#define HVK_TIMER_WMSA_FWD 0
#define HVK_TIMER_WMSA_BWD 1
#define HVK_TIMER_GEMM 2   // forward / input-gradient GEMMs (linear_kernel, gemm_nt_kernel)
#define HVK_TIMER_WGRAD 3  // weight-gradient GEMMs (dw_kernel; its slab reduction not included)
#ifdef __cplusplus
extern "C" {
#endif
// null pair: not timed; work = the launch's algorithmic flops (or bytes), summed by read
__attribute__((visibility("hidden"))) void hvk_timer_next(int kind, double work, hipEvent_t* start,
                                                     hipEvent_t* stop);
// the shape of the NEXT timed GEMM launch (kernel family, epilogue, tile variant, M N K and its
// algorithmic HBM bytes), taken by hvk_timer_next: bench.py's per-shape binding-roof table
__attribute__((visibility("hidden"))) void hvk_timer_shape(const char* family, int epi, int tile, double m,
                                                      double n, double k, double bytes);
#ifdef __cplusplus
}
#endif
#define HVK_LAUNCH_TIMED_W(kind, work, kernel, grid, block, lds, st, ...)               \
  do {                                                                                  \
    hipEvent_t e0_ = nullptr, e1_ = nullptr;                                            \
    hvk_timer_next(kind, (double)(work), &e0_, &e1_);                                   \
    if (e0_)                                                                            \
      hipExtLaunchKernelGGL(kernel, grid, block, lds, st, e0_, e1_, 0, __VA_ARGS__);     \
    else                                                                                \
      hipLaunchKernelGGL(kernel, grid, block, lds, st, __VA_ARGS__);                    \
  } while (0)
#define HVK_LAUNCH_TIMED(kind, kernel, grid, block, lds, st, ...) \
  HVK_LAUNCH_TIMED_W(kind, 0, kernel, grid, block, lds, st, __VA_ARGS__)

#define HVK_CHECK_LAUNCH(what)                                                   \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess)                                                        \
      return hvk_set_error(HVK_EHIP, "%s: %s", what, hipGetErrorString(e_));     \
  } while (0)

// ---- debug bounds checking (make bounds -> libhvk_bounds.so) ----------------
// Computed global indices are checked against their extent; a violation is reported by device
// printf and the index clamped, so the kernel completes instead of faulting the GPU.  The
// product build compiles the checks away.
#ifdef HVK_BOUNDS_CHECK
#define HVK_BCHECK(idx, n) hvk_bcheck((long long)(idx), (long long)(n), __FILE__, __LINE__)
__device__ __forceinline__ long long hvk_bcheck(long long i, long long n, const char* f, int l) {
  if (i < 0 || i >= n) {
    printf("hvk bounds: %s:%d index %lld outside [0, %lld)\n", f, l, i, n);
    return i < 0 ? 0 : n - 1;
  }
  return i;
}
#else
#define HVK_BCHECK(idx, n) (idx)
#endif

// ---- bf16 <-> f32 ----------------------------------------------------------
__device__ __forceinline__ float hvk_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hvk_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t hvk_f2bf(float f) {
  return (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)f);  // RNE, v_cvt_pk_bf16_f32
}
typedef float hvk_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 hvk_bf16x2 __attribute__((ext_vector_type(2)));
// two f32 -> packed bf16x2 (RNE) in ONE v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t hvk_pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((hvk_f32x2){lo, hi}, hvk_bf16x2));
}
__device__ __forceinline__ void hvk_unpack8(const uint4& v, float f[8]) {
  f[0] = hvk_lo(v.x); f[1] = hvk_hi(v.x); f[2] = hvk_lo(v.y); f[3] = hvk_hi(v.y);
  f[4] = hvk_lo(v.z); f[5] = hvk_hi(v.z); f[6] = hvk_lo(v.w); f[7] = hvk_hi(v.w);
}
__device__ __forceinline__ uint4 hvk_pack8(const float f[8]) {
  return make_uint4(hvk_pack2(f[0], f[1]), hvk_pack2(f[2], f[3]), hvk_pack2(f[4], f[5]),
                    hvk_pack2(f[6], f[7]));
}

// The res-post-norm `x = x0 + drop_path(norm(a))` of swinv2.py:431 / 434 (the plain norm of
// PatchEmbed, 656, with no x0) applied in a GEMM epilogue whose workgroup holds whole C-wide rows
// (gemm.hip: C = 96, linear_kernel / mlp_fwd_kernel EPI 5; gemm_tile.hip: C = 192, EPI 5)
struct LnEpi {
  const float* abias;   // [C] the Linear's bias, added in f32 inside the norm (or null)
  const float* x0;      // [M, C] f32 residual stream (null: plain norm)
  const float* gamma;   // [C]
  const float* beta;    // [C]
  const float* sscale;  // [M / rows_per_sample] DropPath factor per sample (or null)
  int rows_per_sample;
  float eps;
  float* x;             // [M, C] f32 out
  hvk_bf16* xb;         // [M, C] bf16 copy (next GEMM operand) or null
  float* mean;          // [M]
  float* rstd;          // [M]
};

// ---- PatchMerging's 2x2 gather as an operand address map (swinv2.py:484-491) ---------------
// The reduction GEMM of PatchMerging reads its [B, H/2 * W/2, 4C] operand straight from the
// token rows [B, H * W, C] (gemm_tile.hip MG 1, gemm_tn.hip MG), and its input gradient is
// written straight back to them (MG 2): merged row r = (b, i, j), 4C-column k of segment
// s = k / C (x0 .. x3 = [0::2, 0::2], [1::2, 0::2], [0::2, 1::2], [1::2, 1::2]) is source token
// (b, 2i + (s & 1), 2j + (s >> 1)), channel k - s C.  Source token of (r, s = 0):
// (b H + 2i) W + 2j = 2r + W floor(r / (W/2)); the quotient by a float reciprocal, exact while
// r < 2^21 (|error| <= r / Wo * 2^-23 < 1 / (4 Wo), the distance of (r + 1/2) / Wo to an integer
// is >= 1 / (2 Wo)); hvk_merge_*_supported bound M.  C % 8 == 0: a 16-B chunk never straddles
// two segments.
struct MergeGeo {
  int W = 0;           // source width (tokens per image row)
  int C = 0;           // source channels
  float inv_wo = 0.f;  // 1 / (W / 2)
};
__device__ __forceinline__ int hvk_merge_tok(int r, const MergeGeo& g) {
  const int q = (int)(((float)r + 0.5f) * g.inv_wo);
  return 2 * r + g.W * q;
}
// element offset of 4C-column k of a merged row from its segment-0 token row
__device__ __forceinline__ int hvk_merge_col(int k, const MergeGeo& g) {
  const int s = (k >= g.C) + (k >= 2 * g.C) + (k >= 3 * g.C);
  return ((s & 1) * g.W + (s >> 1)) * g.C + (k - s * g.C);
}

// ---- post-norm LayerNorm arithmetic, pinned op by op ---------------------------------------
// ln_fwd_kernel (layernorm.hip) and the GEMM epilogues that reproduce it bit for bit (gemm.hip,
// ln96) share these: left to the contraction pass, the SLP vectoriser turned `ss += d * d` into
// v_pk_mul_f32 + v_add_f32 in one kernel and v_pk_fma_f32 in the other (rstd 1-2 ulp apart in
// ~5 % of rows); explicit fmas round the same wherever they are vectorised.
__device__ __forceinline__ float hvk_ln_sq(float ss, float d) { return __builtin_fmaf(d, d, ss); }
__device__ __forceinline__ float hvk_ln_rstd(float ss_row, float invC, float eps) {
  return rsqrtf(__builtin_fmaf(ss_row, invC, eps));
}
// x0 + (gamma (v - mu) rstd + beta) * sc
__device__ __forceinline__ float hvk_ln_out(float x0, float v, float mu, float rs, float gm, float bt, float sc) {
  return __builtin_fmaf(__builtin_fmaf((v - mu) * rs, gm, bt), sc, x0);
}

// ---- 16-B / 8-B global access with an optional nontemporal hint ------------------------
// The nontemporal hint gains +14 % on a full-line 3:1 read:write stream on gfx950 but LOSES
// 24 % on the W-MSA access shape (64-B row segments whose line halves belong to another
// head's workgroup: the hint defeats the L2 merge), tools/probe/stream.hip.  Plain by
// default; HVK_NT builds the hinted form for A/B comparisons.
typedef unsigned int hvk_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int hvk_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 hvk_ld16(const void* p) {
#ifndef HVK_NT
  return *reinterpret_cast<const uint4*>(p);
#else
  return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const hvk_u32x4*>(p)));
#endif
}
__device__ __forceinline__ void hvk_st16(void* p, uint4 v) {
#ifndef HVK_NT
  *reinterpret_cast<uint4*>(p) = v;
#else
  __builtin_nontemporal_store(__builtin_bit_cast(hvk_u32x4, v), reinterpret_cast<hvk_u32x4*>(p));
#endif
}
// Always-nontemporal 16-B accesses for data nobody touches again soon, so it does not evict
// what the NEXT kernel reads (the 4 MB L2s and the 256 MB Infinity Cache hold a stage-2
// tensor): HVK_NT_SAVED bit 0: the fc1 pre-activation h (read again only in the backward);
// bit 1: the LayerNorm's f32 residual stream (read again only at the next LayerNorm);
// bit 2: the LayerNorm backward's f32 residual gradient (likewise); bit 3: the backward's one
// read of h in the GELU' epilogues; bit 4: the LayerNorm kernels' streamed loads; bit 5: the
// W-MSA backward's q/k/v/dO loads; bit 6: the f32 weight / bias gradients (read only by the
// optimizer at the end of the step; neutral, off).  Default 7: bits 0+1 +0.7 % per step, bit 2 +0.2 % on top,
// bit 3 neutral to -0.3 %, bit 4 -0.4 %, bit 5 -0.5 % (its kernel 185 -> 190 us): loads that
// hit the Infinity Cache lose the hit (interleaved A/B, profiles/round2/nt_saved_ab.txt)
#ifndef HVK_NT_SAVED
#define HVK_NT_SAVED 7
#endif
__device__ __forceinline__ void hvk_st16_nt(void* p, uint4 v) {
  __builtin_nontemporal_store(__builtin_bit_cast(hvk_u32x4, v), reinterpret_cast<hvk_u32x4*>(p));
}
__device__ __forceinline__ uint4 hvk_ld16_nt(const void* p) {
  return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const hvk_u32x4*>(p)));
}
// Raw buffer access over [base, base + bytes), bytes <= 2^31 (host-checked), built from
// wave-uniform inputs: a load at offset >= bytes returns 0 and a store there is dropped, so
// padded lanes take HVK_OOB instead of a branch (an exec branch around a store also makes
// the compiler's vmcnt accounting conservative: later waits then drain stores in flight).
#define HVK_OOB 0x80000000u
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hvk_rsrc(const void* base, size_t bytes) {
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)bs, 0, __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}
__device__ __forceinline__ uint4 hvk_bld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void hvk_bst16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(hvk_u32x4, v), r, off, 0, 0);
}
__device__ __forceinline__ void hvk_bst16_nt(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(hvk_u32x4, v), r, off, 0, 2);  // nt
}
__device__ __forceinline__ void hvk_bst4f(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
__device__ __forceinline__ float hvk_bld4f(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ uint4 hvk_bld16_nt(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2));
}
// pin a value as "defined here" (after an explicit s_waitcnt): the compiler then tracks no
// pending memory operation on its registers
// Whole-line row pairs for register-resident 16-row tiles (lane (li, g) holding 16 B of row li per
// 32-column slice): rows li and li ^ 8 swap one slice of a pair with a DPP row_ror:8 per dword.
// pair_rows before a store: (v0, v1) = slices (s, s+1) of row li -> a = (row li & 7, s | s+1 by
// li < 8 | li >= 8), b = the same 8 rows lower (+8): each of a, b then covers 8 rows x 128 B.
// (The mirror image for loads -- 8 x 128-B loads swapped back -- measured neutral to -2 %:
// profiles/round4/pair_stores/pair_loads_*.)
__device__ __forceinline__ uint32_t dpp_ror8(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);
}
__device__ __forceinline__ uint4 dpp_ror8(const uint4& v) {
  return make_uint4(dpp_ror8(v.x), dpp_ror8(v.y), dpp_ror8(v.z), dpp_ror8(v.w));
}
__device__ __forceinline__ void pair_rows(const uint4& v0, const uint4& v1, bool lo, uint4& a, uint4& b) {
  const uint4 r = dpp_ror8(lo ? v1 : v0);
  a = lo ? v0 : r;
  b = lo ? r : v1;
}

__device__ __forceinline__ void hvk_launder(uint4& v) {
  hvk_u32x4 t = __builtin_bit_cast(hvk_u32x4, v);
  asm volatile("" : "+v"(t));
  v = __builtin_bit_cast(uint4, t);
}
// Buffer view of the 16-row tile [r0, r0 + 16) of a row-major tensor (row_bytes per row),
// clipped at M rows: rows past M read 0 and drop their stores, with no exec branch around the
// accesses (r0 and base wave-uniform).  Offsets are lane-relative to row r0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hvk_tile_rsrc(const void* base, int r0, int M, int row_bytes) {
  int rows = M - r0;
  rows = rows < 0 ? 0 : (rows > 16 ? 16 : rows);
  return hvk_rsrc(static_cast<const char*>(base) + (size_t)(r0 < M ? r0 : 0) * row_bytes, (size_t)rows * row_bytes);
}
__device__ __forceinline__ void hvk_st8(void* p, uint2 v) {
#ifndef HVK_NT
  *reinterpret_cast<uint2*>(p) = v;
#else
  __builtin_nontemporal_store(__builtin_bit_cast(hvk_u32x2, v), reinterpret_cast<hvk_u32x2*>(p));
#endif
}

// ---- GELU, erf form (nn.GELU(), swinv2.py:60): shared by the activation kernels and the
// fused fc1 epilogue so both paths round identically
namespace hvk_gelu {
constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, below f32 erf's own noise in
// 1 + erf): one rcp + one exp2 + 6 fma instead of the library erff.  Its e^{-x^2} is the
// same exp(-u^2/2) that GELU' needs, so the backward pays for one exp2 in total.
__device__ __forceinline__ float erf_and_gauss(float x, float& e) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);  // e^{-x^2}
  return copysignf(fmaf(-p, e, 1.f), x);
}
__device__ __forceinline__ float gelu(float u) {
#ifdef HVK_PROBE_NOGELU
  return u;
#endif
  float e;
  return 0.5f * u * (1.f + erf_and_gauss(u * kInvSqrt2, e));
}
__device__ __forceinline__ float gelu_grad(float u) {
#ifdef HVK_PROBE_NOGELU
  return u;
#endif
  float e;  // e = exp(-u^2/2)
  const float er = erf_and_gauss(u * kInvSqrt2, e);
  return fmaf(u * kInvSqrt2Pi, e, 0.5f * (1.f + er));
}
// The same functions on pairs: the polynomial and products as packed f32 (v_pk_fma_f32 /
// v_pk_mul_f32), the same operations and rounding per element as the scalar forms above.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 erf_and_gauss2(f32x2 x, f32x2& e) {
  const f32x2 ax = {fabsf(x.x), fabsf(x.y)};
  const f32x2 d = ax * 0.3275911f + 1.f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = t * 1.061405429f + -1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t + -0.284496736f;
  p = p * t + 0.254829592f;
  p = p * t;
  const f32x2 q = -ax * ax * 1.4426950408889634f;
  e = f32x2{__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2 r = -p * e + 1.f;
  return f32x2{copysignf(r.x, x.x), copysignf(r.y, x.y)};
}
__device__ __forceinline__ f32x2 gelu2(f32x2 u) {
#ifdef HVK_PROBE_NOGELU
  return u;
#endif
  f32x2 e;
  return 0.5f * u * (1.f + erf_and_gauss2(u * kInvSqrt2, e));
}
__device__ __forceinline__ f32x2 gelu_grad2(f32x2 u) {
#ifdef HVK_PROBE_NOGELU
  return u;
#endif
  f32x2 e;
  const f32x2 er = erf_and_gauss2(u * kInvSqrt2, e);
  return (u * kInvSqrt2Pi) * e + 0.5f * (1.f + er);
}
}  // namespace hvk_gelu

// GELU of 8 packed bf16 pre-activations, rounded back to bf16: the fc1 epilogue's stored
// GELU(h), recomputed bit-identically where it is consumed instead of stored
__device__ __forceinline__ uint4 hvk_gelu8_bf16(uint4 h) {
  float u[8];
  hvk_unpack8(h, u);
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const hvk_gelu::f32x2 y = hvk_gelu::gelu2(hvk_gelu::f32x2{u[e], u[e + 1]});
    u[e] = y.x;
    u[e + 1] = y.y;
  }
  return hvk_pack8(u);
}

// ---- MFMA 16x16x32 bf16 -> f32 --------------------------------------------
// A lane l holds A[row l&15][k = 8(l>>4) + j], B lane l holds B[k = 8(l>>4) + j][col l&15],
// D lane l holds D[row 4(l>>4) + r][col l&15], r = 0..3.
__device__ __forceinline__ hvk_f32x4 hvk_mfma16(uint4 a, uint4 b, hvk_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hvk_bf16x8, a),
                                                 __builtin_bit_cast(hvk_bf16x8, b), c, 0, 0, 0);
}

// MFMA result hazard across a branch.  hipcc (ROCm 7.2, gfx950) pads "an MFMA wrote v -> the next
// instruction touching v" with 8 wait states inside a basic block, but NOT for a reader at a
// taken-branch target when the MFMA ends the predecessor block: an unmasked W-MSA window that
// branched over the mask code read its scores 2 states after the MFMA (wrong values, no fault).
// hvk_settle(x, ...) after such MFMAs holds this wave 8 states in an asm statement that takes the
// results as operands, so no reader can be scheduled above it (other waves issue meanwhile).
// tools/mfma_hazard_audit.py walks every path of the built ISA and must report none.
__device__ __forceinline__ void hvk_settle(hvk_f32x4& a) { asm volatile("s_nop 7" : "+v"(a)); }
__device__ __forceinline__ void hvk_settle(hvk_f32x4& a, hvk_f32x4& b) {
  asm volatile("s_nop 7" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void hvk_settle(hvk_f32x4& a, hvk_f32x4& b, hvk_f32x4& c) {
  asm volatile("s_nop 7" : "+v"(a), "+v"(b), "+v"(c));
}
__device__ __forceinline__ void hvk_settle(hvk_f32x4& a, hvk_f32x4& b, hvk_f32x4& c, hvk_f32x4& d) {
  asm volatile("s_nop 7" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, cols 4p..4p+3 of a
// 4x16 bf16 block; lane i receives column i of the 4 rows (element q = row q).
__device__ __forceinline__ uint2 hvk_tr_read(const hvk_bf16* lds) {
  hvk_i16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(HVK_LDS_I16X4(lds));
  return __builtin_bit_cast(uint2, r);
}

// Reductions over the 4 lanes l, l^16, l^32, l^48 (the 4 k-groups of a 16x16x32 MFMA
// fragment) with v_permlane16_swap / v_permlane32_swap: VALU only, no LDS round trip.
// With both operands = v, the two swap results hold v[l] and v[l ^ 16] (or ^ 32) in some
// order, so their sum / max is the pairwise reduction in every lane.
__device__ __forceinline__ float hvk_xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float hvk_xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float hvk_xor16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float hvk_xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// Two 4-channel halves of a 16x16 MFMA accumulator pair (rows 4gq..4gq+3 of tile 0 = channels
// 4gq..+3, of tile 1 = 16 + 4gq..+3; bf16-packed, lo/hi pairs) -> the 8 consecutive channels
// this lane stores with one 16-B store, at channel offset hvk_pair_col(gq): one
// v_permlane16_swap per dword exchanges tile 1 of the even rows (16 lanes) with tile 0 of the
// odd rows.  Every lane of the wave must execute it (cross-lane).
__device__ __forceinline__ uint4 hvk_pair_swap(uint2 t0, uint2 t1) {
  const auto a = __builtin_amdgcn_permlane16_swap(t0.x, t1.x, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(t0.y, t1.y, false, false);
  return make_uint4(a[0], b[0], a[1], b[1]);
}
__device__ __forceinline__ int hvk_pair_col(int gq) { return 16 * (gq & 1) + 8 * (gq >> 1); }

__device__ __forceinline__ float hvk_group4_sum(float v) { return hvk_xor32_sum(hvk_xor16_sum(v)); }
__device__ __forceinline__ float hvk_group4_max(float v) { return hvk_xor32_max(hvk_xor16_max(v)); }

// Head normalisation of the W-MSA q / k slices (F.normalize, swinv2.py:229) where the qkv rows
// are produced (the GEMM epilogues, hvk_qk_normalize): a lane holds 8 consecutive channels of one
// row and lanes l, l^16, l^32, l^48 the head's 32 channels; hv = the rounded bf16 qkv values.
// Returns the normalised bf16 values and rn = 1 / max(||x||, 1e-12) -- the arithmetic of
// wmsa_common.h's l2_normalize (dot2 sum of squares, group-4 sum, rsq), which the w <= 8
// attention kernels ran on the loaded rows before round 4.
__device__ __forceinline__ uint4 hvk_head_normalize8(uint4 v, float& rn, float post = 1.f) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  auto d2 = [](uint32_t w, float c) {
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, w), __builtin_bit_cast(bf16x2_t, w), c, false);
  };
  float ss = d2(v.w, d2(v.z, d2(v.y, d2(v.x, 0.f))));
  float f[8];
  hvk_unpack8(v, f);
  ss = hvk_group4_sum(ss);
  rn = __builtin_amdgcn_rsqf(fmaxf(ss, 1e-24f));
  const float m = rn * post;  // post: the q slices' scale * log2e (wmsa_common.h's l2_normalize)
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] *= m;
  return hvk_pack8(f);
}

// max over the 16 lanes of a row (DPP: quad swaps, half-row and row mirrors)
__device__ __forceinline__ float hvk_row16_max(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), decltype(ctrl)::value, 0xF, 0xF, false));
  };
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0xB1>{}));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x4E>{}));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x140>{}));  // row_mirror
  return v;
}

// Butterfly sum over TPR-lane groups, bit for bit `for (m = TPR / 2; m >= 1; m >>= 1) v +=
// __shfl_xor(v, m)` (the same pairings in the same order; a + b == b + a) without the LDS-pipe
// ds_bpermute per step: xor 32 / 16 by v_permlane32 / 16_swap, xor 8 by DPP row_ror:8, xor 4 by a
// quad reverse then a half-row mirror (lane i -> 7 - (i ^ 3) = i ^ 4 within 8), xor 2 / 1 by quad
// permutes.  Every lane of the wave must execute it (cross-lane).
template <int TPR>
__device__ __forceinline__ float hvk_xor_sum(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), decltype(ctrl)::value, 0xF, 0xF, false));
  };
  if constexpr (TPR >= 64) v = hvk_xor32_sum(v);
  if constexpr (TPR >= 32) v = hvk_xor16_sum(v);
  if constexpr (TPR >= 16) v += dpp(v, std::integral_constant<int, 0x128>{});  // row_ror:8
  if constexpr (TPR >= 8)
    v += dpp(dpp(v, std::integral_constant<int, 0x1B>{}), std::integral_constant<int, 0x141>{});
  if constexpr (TPR >= 4) v += dpp(v, std::integral_constant<int, 0x4E>{});  // quad_perm [2,3,0,1]
  if constexpr (TPR >= 2) v += dpp(v, std::integral_constant<int, 0xB1>{});  // quad_perm [1,0,3,2]
  return v;
}

__device__ __forceinline__ float hvk_wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// XCD-aware block id decode: logical (chunk, head) so that every head of a window chunk
// lands in the same blockIdx%8 group (same XCD L2) and is dispatched back to back.
// Grid = n_chunks_padded(multiple of 8) * n_heads.
__device__ __forceinline__ void hvk_decode_chunk_head(int bid, int n_heads, int& chunk, int& head) {
  const int xcd = bid & 7, loc = bid >> 3;
  head = loc % n_heads;
  chunk = (loc / n_heads) * 8 + xcd;
}
