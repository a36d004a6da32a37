/* libhvk -- MI355X (gfx950) kernels for the SwinV2 + taxonomy-loss training hot path of
 * samuelstevens/hierarchical-vision, behind a plain C ABI.
 *
 * Conventions (every entry point):
 *  - returns 0 on success, else HVK_EINVAL(1) / HVK_EUNSUPPORTED(2) / HVK_EHIP(3);
 *    hvk_last_error_string() gives the text (thread-local).
 *  - all pointers are device pointers owned by the caller (the PyTorch caching allocator);
 *    the library never allocates device memory.  Tensors are contiguous row-major.
 *  - `stream` is a hipStream_t; work is enqueued asynchronously, nothing synchronises.
 *  - "bf16" buffers hold raw bfloat16 bits; "f32" buffers hold float.
 *
 * The reference has no native code: each entry point replaces an eager
 * PyTorch op sequence; the citation names the reference lines it stands in for.
 */
#ifndef HVK_H_
#define HVK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* the C ABI this header describes; hvk_abi_version() returns it (bindings check it at load) */
#define HVK_ABI_VERSION 14

#define HVK_OK 0
#define HVK_EINVAL 1
#define HVK_EUNSUPPORTED 2
#define HVK_EHIP 3

int hvk_abi_version(void);
const char* hvk_last_error_string(void);

/* ---- Library options -------------------------------------------------------------------
 * libhvk reads no environment variable: the few selectable forms are a fixed table of named
 * integer options, changed only here (A/B runs and the parity tests that pin alternate forms to
 * the default one).  set returns HVK_EINVAL for an unknown name or a value outside its range and
 * stores the old value in *previous when that is not NULL.
 *   wmsa_fwd_form         0 (default) one workgroup per (window, head group), 1 persistent ring
 *   wmsa_bwd_nt           w <= 8 backward qkv reads: 0 (default) cached, 1 nontemporal, 2 nt when
 *                         qkv exceeds the 256 MB Infinity Cache
 *   wmsa_bwd_slice_bytes  w <= 8 backward: launch over batch slices whose qkv stays below this
 *                         (default 2^31, the buffer-descriptor range)
 *   tile_wide             tiled GEMM: -1 (default) tile width by shape, 0 128, 1 192 columns
 *   dw_tile               weight gradient at 192-multiple shapes: tile variant 4..8 (default 5)
 *   wmsa_fwd_hg           w <= 8 forward, win form: heads per workgroup; 0 (default) 2 at 6 heads,
 *                         else 3 where it divides the head count, else 2, else 1; 1 / 2 / 3 / 4 / 6
 *                         force it where it divides (the same results bit for bit: per-head math
 *                         unchanged)
 *   dw_chunks             weight gradient: workgroups per launch to aim for (token chunks = this /
 *                         output tiles, x2 for the 128 x 128 tiles; default 256: one per CU); the
 *                         f32 partial sums change order with it */
int hvk_set_option(const char* name, long long value, long long* previous);
int hvk_get_option(const char* name, long long* value);

/* ---- Kernel timer (measurement only; bench.py's roofline) ---------------------------
 * enable(n > 0): time the next n launches of the timed kernels (kind 0 = W-MSA forward,
 * 1 = W-MSA backward main kernel, 2 = forward / input-gradient GEMMs, 3 = weight-gradient
 * GEMMs) with start/stop events recorded by the dispatch packet itself
 * (hipExtLaunchKernelGGL): a duration is the kernel's execution, as in a rocprofv3 kernel
 * trace.  enable(0) stops timing.  read() waits for the recorded launches of `kind` since the
 * last enable and returns their summed duration (ms) and count; read_work() also the summed
 * algorithmic work of those launches (GEMMs: 2 M N K flops each; W-MSA: 0). */
int hvk_kernel_timer_enable(int max_launches);
int hvk_kernel_timer_read(int kind, double* total_ms, int* launches);
/* which kinds the timer records (bit k = kind k; default 0xF, all): bench.py times only the
 * W-MSA launches inside its timed steps and the GEMMs in extra steps after them */
int hvk_kernel_timer_kinds(int mask);
int hvk_kernel_timer_read_work(int kind, double* total_ms, int* launches, double* work);
/* the index-th timed launch since hvk_kernel_timer_enable, in launch order: its kind, duration
 * and the work the library recorded for it (bench.py's per-stage W-MSA breakdown) */
int hvk_kernel_timer_launch(int index, int* kind, double* ms, double* work);
/* the same launch's shape, for the GEMM kinds (2, 3): name = "family<epilogue,tile>" (the kernel
 * family, e.g. gemm_nt / linear / mlp_fwd / dw, its epilogue and tile variant; "" for launches
 * that recorded none), mnk[3] = M, N, K, bytes = its algorithmic HBM bytes (operands read once,
 * outputs written once: bench.py's per-shape binding roof max(flops / MFMA peak, bytes / HBM peak)).
 * ABI 10. */
int hvk_kernel_timer_launch_shape(int index, char* name, int name_cap, double* mnk, double* bytes);

/* ---- Shifted-window cosine attention core ------------------------------------------
 * Replaces swinv2.py:399-412 (roll + window_partition), 221-261 (WindowAttention core:
 * normalize, q k^T, logit scale, CPB bias gather, shift mask, softmax, @v) and 420-429
 * (window_reverse + roll back).  qkv: bf16 [B*H*W, 3C] = F.linear output of swinv2.py:220
 * in UN-partitioned token order, with bias (q_bias, 0, 0): v_bias does not enter, since
 * softmax rows sum to 1 and P (V + v_bias) = P V + v_bias, which the caller folds into
 * proj's bias (proj.bias + proj.weight v_bias).  out: bf16 [B*H*W, C] = input of proj
 * (swinv2.py:262) minus v_bias.  bias_table: f32 [num_heads, (2w-1)^2] =
 * 16*sigmoid(cpb_mlp(relative_coords_table)) (swinv2.py:233-246 before the rpi gather);
 * scale: f32 [num_heads] = exp(clamp(logit_scale, max=ln 100)) (swinv2.py:230).
 * window/shift are the clamped values of swinv2.py:328-331.  head_dim must be 32; window
 * in {4, 6, 7, 8} (one wave per (window, head)) or {12, 16, 24} (one workgroup each).
 * lse: NULL, or f32 [B*H*W, num_heads]: per query and head, L2 = log2 sum_k exp2(log2e *
 * logit), the row constant of the softmax that the backward can consume (P = exp2(log2e *
 * logit - L2)). */
int hvk_wmsa_fwd(const void* qkv, void* out, float* lse, const float* bias_table, const float* scale,
                 int B, int H, int W, int C, int num_heads, int window, int shift,
                 void* stream);
size_t hvk_wmsa_bwd_workspace_bytes(int num_heads, int window);
/* dout: bf16 [B*H*W, C] (grad of `out`); out, lse: the forward's output and row constants,
 * or both NULL (every window: the softmax row statistics are recomputed from q, k).  Given
 * them, windows 12/16/24 skip the row-statistics pass (delta from dout o out, corrected by the
 * exact dS and P row sums for dq, dk, dv and dscale); windows <= 8 ignore them and recompute
 * (exact delta = rowsum(P o dP));
 * dqkv: bf16 [B*H*W, 3C] (fully overwritten);
 * dq_bias: f32 [C] (overwritten: column sums of the q part of dqkv = d loss / d q_bias,
 * replacing the qkv bias-gradient reduction) or NULL; dbias_table: f32 [num_heads,
 * (2w-1)^2] (overwritten); dscale: f32 [num_heads] (overwritten, d loss / d scale).
 * workspace: f32, hvk_wmsa_bwd_workspace_bytes bytes, ALL ZERO on entry and left all zero
 * on return (a caller keeps one zero-filled workspace: no memset per call).  It holds one slot
 * (CPB-table bins, d scale, d q_bias) per (head, window chunk): each workgroup adds its partial
 * sums, folded in a fixed order, to its own slot and the finalize kernel sums the slots in chunk
 * order -- no float atomics, so dbias_table / dscale / dq_bias are bit-identical run to run. */
int hvk_wmsa_bwd(const void* qkv, const void* dout, const void* out, const float* lse, void* dqkv,
                 float* dq_bias, const float* bias_table, const float* scale, float* dbias_table,
                 float* dscale, float* workspace, size_t workspace_bytes, int B, int H, int W, int C,
                 int num_heads, int window, int shift, void* stream);
/* The w <= 8 pair with the q and k normalisation of swinv2.py:229 (and the forward's logit scale)
 * done upstream, by the qkv Linear's epilogue (hvk_linear_qkv_fwd / hvk_gemm_qkv_fwd) or
 * hvk_qk_normalize: qkv holds (q^ * scale * log2e, k^, v) per head, q^ = F.normalize(q),
 * k^ = F.normalize(k), rounded to bf16 once (scale = the `scale` argument, exp(clamp(logit_scale)),
 * log2e = 1/ln 2), and rn: f32 [B*H*W, 2 num_heads] = 1 / max(||q||, 1e-12) (columns 0..nH-1)
 * and 1 / max(||k||, 1e-12) (nH..2nH-1) of the un-normalised bf16 q, k.  The forward's q and k
 * operands are then exactly the ones hvk_wmsa_fwd forms from raw q, k (same results bit for
 * bit); the backward returns dqkv with respect to the UN-normalised q, k (the normalisation's
 * backward applied with rn), so the qkv Linear's backward is unchanged.  Windows 4, 6, 7, 8 only
 * (EUNSUPPORTED otherwise). */
int hvk_wmsa_fwd_normed(const void* qkv, void* out, const float* bias_table, const float* scale,
                        int B, int H, int W, int C, int num_heads, int window, int shift, void* stream);
int hvk_wmsa_bwd_normed(const void* qkv, const float* rn, const void* dout, void* dqkv, float* dq_bias,
                        const float* bias_table, const float* scale, float* dbias_table, float* dscale,
                        float* workspace, size_t workspace_bytes, int B, int H, int W, int C,
                        int num_heads, int window, int shift, void* stream);
/* In place: every 32-wide q and k head slice of qkv [T, C3 = 3C] (columns < 2C) normalised, the
 * q slices times qscale[h] * log2e (qscale: f32 [C/32] = the W-MSA `scale`, or NULL: none), and
 * rn [T, 2C/32] written, exactly as the qkv epilogues do (for a qkv produced elsewhere). */
int hvk_qk_normalize(void* qkv, float* rn, const float* qscale, int T, int C, void* stream);

/* ---- Skinny Linear (memory-bound GEMM) ------------------------------------------------
 * y[M, N] = x[M, K] w[N, K]^T (+ bias[N]), bf16 in/out, f32 accumulation: F.linear of
 * swinv2.py:58-62 (fc1/fc2), 220 (qkv), 262 (proj), 492 (PatchMerging.reduction) and
 * 652 (patch embedding as GEMM) for the (K, N) shapes hvk_linear_supported() reports
 * (the SwinV2-T stage 0-1 widths; other widths, e.g. SwinV2-B's C = 128 / 256, run on the tiled
 * hvk_gemm_fwd); with w = weight^T it is the input gradient of those layers.
 * x: bf16 [M, K]; w: bf16 [N, K]; bias: f32 [N] or NULL; y: bf16 [M, N]. */
int hvk_linear_supported(int M, int K, int N);
int hvk_linear_fwd(const void* x, const void* w, const float* bias, void* y, int M, int K, int N,
                   void* stream);
/* fc1 with its activation fused (swinv2.py:58-62): h = bf16(x w^T + bias) (kept for the
 * backward, = the reference's fc1 output) and y = GELU(h) (exact erf, bf16); replaces
 * hvk_linear_fwd + hvk_bias_gelu_fwd where hvk_linear_gelu_supported(). */
/* The qkv Linear of a w <= 8 block (swinv2.py:220 + the F.normalize of 229): y = x w^T + bias
 * (N = 3K) with the q and k head slices normalised -- q times qscale[h] * log2e when qscale (f32
 * [K/32], the block's exp(clamp(logit_scale))) is not NULL -- and rn [M, 2K/32] written (see
 * hvk_wmsa_fwd_normed); the v slice is hvk_linear_fwd's bit for bit.  Built for K = 96, 128,
 * 192, 256 (hvk_linear_qkv_supported); hvk_gemm_qkv_fwd is the tiled form (N % 96 == 0,
 * hvk_gemm_supported shapes). */
int hvk_linear_qkv_supported(int M, int K, int N);
int hvk_linear_qkv_fwd(const void* x, const void* w, const float* bias, void* y, float* rn, const float* qscale,
                       int M, int K, int N, void* stream);
int hvk_gemm_qkv_fwd(const void* x, const void* w, const float* bias, void* y, float* rn, const float* qscale,
                     int M, int K, int N, void* stream);
int hvk_linear_gelu_supported(int M, int K, int N);
int hvk_linear_gelu_fwd(const void* x, const void* w, const float* bias, void* h, void* y, int M,
                        int K, int N, void* stream);

/* fc2 input gradient through the MLP activation (swinv2.py:58-65 backward): gh =
 * bf16((gy w^T) * GELU'(h)) with gy: bf16 [M, K] (gradient of fc2's output), w: bf16 [N, K]
 * (= fc2.weight^T), h: bf16 [M, N] (fc1's pre-activation saved by hvk_linear_gelu_fwd);
 * dbias: f32 [N] or NULL, ACCUMULATED into (+= column sums of gh = the fc1 bias gradient;
 * the caller zeroes it).  Replaces the input-gradient GEMM + activation backward + bias reduction for
 * the (K, N) shapes hvk_linear_gelu_bwd_supported() reports. */
/* The whole MLP forward of the stage-0 width (swinv2.py:58-65, C = 96, hidden 384) in one
 * kernel: h = bf16(x w1^T + b1) (saved for the backward), g = GELU(h) (saved for fc2's weight
 * gradient), y = bf16(g w2^T (+ b2)); bit-identical to hvk_linear_gelu_fwd followed by
 * hvk_linear_fwd(g, w2, b2) without fc2's re-read of g.  x [M, 96], w1 [384, 96], w2 [96, 384]
 * bf16; b1 f32 [384] required, b2 f32 [96] or NULL; h, g [M, 384], y [M, 96] bf16. */
int hvk_mlp_fwd_supported(int M, int K, int N1, int N2);
int hvk_mlp_fwd(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* h,
                void* g, void* y, int M, int K, int N1, int N2, void* stream);
/* Its backward chain at the same width (the input gradients of swinv2.py:58-65): gh =
 * bf16((gy w2t^T) * GELU'(h)) and gx = bf16(gh w1t^T) in one kernel, gh also stored (fc1's
 * weight gradient reads it); bit-identical to hvk_linear_gelu_bwd + hvk_linear_fwd(gh, w1t)
 * without the second kernel's re-read of gh.  gy [M, 96], w2t = fc2.weight^T [384, 96],
 * h [M, 384], w1t = fc1.weight^T [96, 384]; gh [M, 384], gx [M, 96]. */
/* The post-norm LayerNorm + residual of swinv2.py:431 / 434 (and PatchEmbed's plain norm, 656)
 * fused into the producing GEMM's epilogue at C = 96 (SwinV2-T stage 0), replacing the Linear
 * (run without its bias) + hvk_ln_residual_fwd pair: a = bf16(x W^T) is stored (the LayerNorm
 * backward reads it) and x = x0 + s[b] (gamma (a + abias - mean) rstd + beta), xb = bf16(x), mean,
 * rstd come out of the same pass, bit-identical to hvk_ln_residual_fwd on that a (same lane layout
 * and arithmetic).  x0 NULL: plain norm; sample_scale NULL: no DropPath; xb_out NULL: not stored.
 * linear: N = 96 with K = 96 (proj) or K = 48 (the patch embedding) on the skinny kernel, and N = 192
 * with K % 64 == 0 (SwinV2-T stage 1: proj, fc2, the stage-0 -> 1 PatchMerging) on the 128 x 192 tile
 * (bit-identical to hvk_gemm_fwd + hvk_ln_residual_fwd); mlp: the hvk_mlp_fwd shape with the fc2
 * output normalised (fc2's bias passed as abias).  ABI 11. */
int hvk_linear_ln_supported(int M, int K, int N);
int hvk_linear_ln_fwd(const void* x, const void* w, int M, int K, int N, const float* abias, const float* x0,
                      const float* gamma, const float* beta, const float* sample_scale, int rows_per_sample,
                      float eps, void* a_out, float* x_out, void* xb_out, float* mean, float* rstd, void* stream);
int hvk_mlp_ln_supported(int M, int K, int N1, int N2);
int hvk_mlp_ln_fwd(const void* x, const void* w1, const float* b1, const void* w2, void* h, void* g, void* a_out,
                   int M, int K, int N1, int N2, const float* abias, const float* x0, const float* gamma,
                   const float* beta, const float* sample_scale, int rows_per_sample, float eps, float* x_out,
                   void* xb_out, float* mean, float* rstd, void* stream);
int hvk_mlp_bwd_supported(int M, int K, int N1, int N2);
int hvk_mlp_bwd(const void* gy, const void* w2t, const void* h, const void* w1t, void* gh, void* gx, int M,
                int K, int N1, int N2, void* stream);
/* fc2 forward on the saved pre-activation: y = GELU(h) w^T (+ bias), GELU recomputed per
 * loaded fragment exactly as hvk_linear_gelu_fwd stores it (swinv2.py:58-65).  Built for
 * K = 384, N = 96 (stage 0). */
int hvk_linear_gelu_in_supported(int M, int K, int N);
int hvk_linear_gelu_in_fwd(const void* h, const void* w, const float* bias, void* y, int M, int K, int N,
                           void* stream);
int hvk_linear_gelu_bwd_supported(int M, int K, int N);
int hvk_linear_gelu_bwd(const void* gy, const void* w, const void* h, void* gh, float* dbias, int M,
                        int K, int N, void* stream);

/* ---- Tiled MFMA GEMM (compute-heavier Linears) ----------------------------------------
 * y[M, N] = x[M, K] w[N, K]^T (+ bias[N]) for K % 64 == 0, N % 128 == 0 (SwinV2 stage 2-3
 * shapes: F.linear of swinv2.py:58-62, 220, 262, 492 and, with w = weight^T, their input
 * gradients).  x, w, y bf16; bias f32 or NULL.  The _gelu form is fc1 (swinv2.py:58-62):
 * h = bf16(x w^T + bias), y = GELU(h) (exact erf), bias required. */
int hvk_gemm_supported(int M, int K, int N);
int hvk_gemm_fwd(const void* x, const void* w, const float* bias, void* y, int M, int K, int N,
                 void* stream);
int hvk_gemm_gelu_fwd(const void* x, const void* w, const float* bias, void* h, void* y, int M,
                      int K, int N, void* stream);
/* fc2 input gradient through the activation on the tiled kernel (the stage-2 form of
 * hvk_linear_gelu_bwd, without the bias gradient): gh = bf16((gy w^T) * GELU'(h)), gy [M, K],
 * w [N, K] (= fc2.weight^T), h [M, N] the saved pre-activation. */
int hvk_gemm_gelu_bwd(const void* gy, const void* w, const void* h, void* gh, int M, int K, int N,
                      void* stream);

/* ---- Weight-gradient GEMM (the backward of every SwinV2 Linear) ----------------------
 * dw[N, K] = g[M, N]^T x[M, K] in f32 and, when db is not NULL, db[N] = sum_m g[m, n]
 * (F.linear backward of swinv2.py:58-62, 220, 262, 296; torch computes them as
 * grad_output^T input and grad_output.sum(0)).  g, x bf16, token-major; dw, db f32,
 * OVERWRITTEN.  M = tokens (M % 32 == 0); the (N, K) shapes hvk_weight_grad_supported()
 * reports.  ws: device scratch of at least hvk_weight_grad_workspace(M, N, K) bytes (the
 * per-chunk partial sums). */
int hvk_weight_grad_supported(int M, int N, int K);
size_t hvk_weight_grad_workspace(int M, int N, int K);
int hvk_weight_grad(const void* g, const void* x, float* dw, float* db, int M, int N, int K,
                    void* ws, size_t ws_bytes, void* stream);
/* dW = g^T (x + 1 xshift^T) = g^T x + db (x) xshift, db = sum_m g (db may be NULL: not stored):
 * the proj Linear's weight gradient when its input's constant share v_bias (swinv2.py:255-262,
 * P (V + v_bias) = P V + v_bias) was folded into the bias instead of the GEMM operand;
 * xshift f32 [K].  Same shapes as hvk_weight_grad. */
int hvk_weight_grad_shift(const void* g, const void* x, const float* xshift, float* dw, float* db, int M, int N,
                          int K, void* ws, size_t ws_bytes, void* stream);
/* The same with x = GELU(h) recomputed from the saved bf16 fc1 pre-activation h (bit-identical
 * to the stored GELU(h) of hvk_linear_gelu_fwd): fc2's weight gradient without GELU(h) kept
 * in HBM.  Built for the stage-0 fc2 shape (N = 96, K = 384). */
int hvk_weight_grad_gelu_x_supported(int M, int N, int K);
int hvk_weight_grad_gelu_x(const void* g, const void* h, float* dw, float* db, int M, int N, int K, void* ws,
                           size_t ws_bytes, void* stream);

/* ---- Classifier head (M = the batch) ---------------------------------------------------
 * The head Linear of swinv2.py:786-794 and the concatenated tiers of the multitask head
 * (hierarchy.py:19-47): M rows of pooled features, N classes (10 000 leaves for HXE), neither a
 * tile multiple.  x: bf16 [M, K]; w: bf16 [N, K]; bias: f32 [N] or NULL; y: bf16 [M, N] =
 * bf16(x w^T + bias).  K and N multiples of 8 (hvk_head_supported); the caller pads a class
 * count that is not (zero weight rows).  Backward: g = bf16 [M, N] gradient of y; gx: f32
 * [M, K] = g w (or NULL: needs the workspace of hvk_head_bwd_workspace_bytes); dw: f32 [N, K] =
 * g^T x and db: f32 [N] = column sums of g (or NULL), all overwritten. */
int hvk_head_supported(int M, int K, int N);
int hvk_head_fwd(const void* x, const void* w, const float* bias, void* y, int M, int K, int N, void* stream);
size_t hvk_head_bwd_workspace_bytes(int M, int K, int N);
int hvk_head_bwd(const void* g, const void* x, const void* w, float* gx, float* dw, float* db, int M, int K,
                 int N, float* workspace, size_t workspace_bytes, void* stream);

/* ---- bf16 weight copies for a step --------------------------------------------------
 * For k < n: dst[k] = bf16(src[k]) ([rows[k], cols[k]] row-major, f32 -> bf16 round to
 * nearest even, as weight.to(torch.bfloat16)) and, when dst_t is not NULL and dst_t[k] is
 * not NULL, dst_t[k] = its transpose [cols[k], rows[k]].  All weights in one launch per 64
 * (the per-call casts of every autocast F.linear, swinv2.py:58-62, 220, 262, 296, 492). */
int hvk_cast_weights(int n, const float* const* src, void* const* dst, void* const* dst_t,
                     const int* rows, const int* cols, void* stream);

/* ---- Fused optimizer step (DDP mean + gradient-norm clipping + DecoupledSGDW + EMA) ----
 * For the n f32 tensors p[k] (params), g[k] (grads), m[k] (momentum buffers) of numel[k]
 * elements in parameter group group[k] < ngroups <= 4: with s = grad_scale (> 0; 1/world when
 * g holds the SUM of the ranks' gradients, ddp.py) and coef = s min(1, max_norm /
 * (s ||g||_2 + 1e-6)) over ALL n gradients (max_norm <= 0: coef = s; torch clip_grad_norm_ on
 * the mean gradient), g' = coef g, m = first ? g' : momentum m + (1 - dampening) g',
 * u = nesterov ? g' + momentum m : m, p = p decay[group] - lr[group] u (composer DecoupledSGDW:
 * decay = 1 - weight_decay lr / initial_lr).  ema: NULL, or n pointers; then also
 * ema[k] = a ema[k] + (1 - a) p (the updated p; a = ema_smoothing; the EMA algorithm,
 * configs/pretrain/inat21.yaml:31-34).  hyper: NULL, or a DEVICE f32 array [8] = lr[0..3],
 * decay[0..3] read at run time instead of lr / decay (HIP-graph replays: the host refreshes it
 * before each replay).  g is not modified.  workspace: f32, hvk_sgdw_workspace_bytes(n, numel)
 * bytes. */
size_t hvk_sgdw_workspace_bytes(int n, const long long* numel);
int hvk_sgdw_step(int n, float* const* p, const float* const* g, float* const* m,
                  float* const* ema, const long long* numel, const int* group, const float* lr,
                  const float* decay, int ngroups, const float* hyper, float grad_scale,
                  float max_norm, float momentum, float dampening, int nesterov, int first,
                  float ema_smoothing, float* workspace, size_t ws_bytes, void* stream);

/* ---- W-MSA block biases (swinv2.py:218-220, 262) --------------------------------------
 * Forward: qkv_bias[3C] = (q_bias or 0, 0, 0) and eff[C] = proj_bias (or 0) + proj_w v_bias
 * (proj_w f32 [C, C]): the qkv GEMM's bias and proj's bias with v_bias folded in (softmax
 * rows sum to 1, so P (V + v_bias) = P V + v_bias).  Backward of eff w.r.t. g = d eff:
 * d_proj_bias = g (if not NULL), d_v_bias += proj_w^T g (accumulated: pass the dv_zero
 * buffer the forward zeroed), d_proj_w = g v_bias^T (written). */
int hvk_attn_bias_fwd(const float* q_bias, const float* v_bias, const float* proj_bias,
                      const float* proj_w, int C, float* qkv_bias, float* eff, float* dv_zero,
                      void* stream);
int hvk_attn_bias_bwd(const float* g, const float* v_bias, const float* proj_w, int C,
                      float* d_proj_bias, float* d_v_bias, float* d_proj_w, void* stream);

/* ---- Continuous relative-position bias table + logit scale (one block) ---------------
 * table[h, r] = 16 sigmoid(w2[h, :] . relu(w1 coords[r, :] + b1)), scale[h] =
 * exp(min(logit_scale[h], clamp_max)): swinv2.py:141-145 (cpb_mlp), 233-246 (16 sigmoid,
 * before the rpi gather) and 230 (clamp + exp).  coords: f32 [RR, 2]
 * (relative_coords_table), w1 f32 [512, 2], b1 [512], w2 [nH, 512], logit_scale [nH];
 * table f32 [nH, RR], scale [nH].  hidden must be 512, nH <= 32.  Backward: from the
 * forward table and d table / d scale, writes dw1, db1, dw2, d logit_scale (all
 * overwritten) using hvk_cpb_bwd_workspace_bytes of workspace. */
int hvk_cpb_fwd(const float* coords, const float* w1, const float* b1, const float* w2,
                const float* logit_scale, float clamp_max, int RR, int nH, int hidden,
                float* table, float* scale, void* stream);
size_t hvk_cpb_bwd_workspace_bytes(int RR, int nH);
int hvk_cpb_bwd(const float* coords, const float* w1, const float* b1, const float* w2,
                const float* logit_scale, float clamp_max, int RR, int nH, int hidden,
                const float* table, const float* dtable, const float* dscale, float* dw1,
                float* db1, float* dw2, float* dlogit, float* workspace, size_t workspace_bytes,
                void* stream);

/* One W-MSA block's small tables in one launch forward / two backward: hvk_attn_bias_fwd
 * + hvk_cpb_fwd (same arguments and results), and hvk_attn_bias_bwd + hvk_cpb_bwd (g_eff
 * NULL: the CPB part only).  Workspace: hvk_cpb_bwd_workspace_bytes(RR, nH). */
int hvk_block_bias_fwd(const float* q_bias, const float* v_bias, const float* proj_bias, const float* proj_w,
                       int C, const float* coords, const float* w1, const float* b1, const float* w2,
                       const float* logit_scale, float clamp_max, int RR, int nH, int hidden, float* qkv_bias,
                       float* eff, float* dv_zero, float* table, float* scale, void* stream);
/* d_proj_w may be NULL: the W_proj v_bias share of the proj weight gradient is then left to the
 * proj Linear's weight-gradient kernel (hvk_weight_grad_shift with xshift = v_bias). */
int hvk_block_bias_bwd(const float* g_eff, const float* v_bias, const float* proj_w, int C, float* d_proj_bias,
                       float* d_v_bias, float* d_proj_w, const float* coords, const float* w1, const float* b1,
                       const float* w2, const float* logit_scale, float clamp_max, int RR, int nH, int hidden,
                       const float* table, const float* dtable, const float* dscale, float* dw1, float* db1,
                       float* dw2, float* dlogit, float* workspace, size_t workspace_bytes, void* stream);

/* ---- Post-norm residual LayerNorm (with the producing Linear's bias folded in) -------
 * x = x0 + sample_scale[row / rows_per_sample] * LayerNorm(a + abias) (gamma, beta, eps)
 * Replaces swinv2.py:431 / 434 (shortcut + drop_path(norm(proj(x))) with proj/fc2 run
 * as GEMMs WITHOUT their bias), and with x0 == NULL the plain norms of swinv2.py:494
 * (PatchMerging), 656 (patch_embed.norm), 833 (final norm).
 * a: bf16 [rows, C]; abias: f32 [C] or NULL; x0: f32 [rows, C] or NULL; sample_scale:
 * f32 [rows/rows_per_sample] or NULL (= 1; DropPath keep-mask / keep_prob); x_out:
 * f32 [rows, C]; xb_out: bf16 copy of x_out or NULL; mean/rstd: f32 [rows] for the
 * backward.  C: multiple of 8, <= 1024. */
int hvk_ln_residual_fwd(const void* a, const float* abias, const float* x0, const float* gamma,
                        const float* beta, const float* sample_scale, int rows, int C,
                        int rows_per_sample, float eps, float* x_out, void* xb_out, float* mean,
                        float* rstd, void* stream);
/* gx: f32 [rows, C] or NULL, gxb: bf16 [rows, C] or NULL -- the two gradients of the
 * output (f32 residual stream and its bf16 copy), summed.  gx0: f32 [rows, C] or NULL
 * (gradient to the shortcut); ga: bf16 [rows, C]; dgamma/dbeta/dabias: f32 [C]
 * (overwritten; dabias = column sums of ga, may be NULL).  workspace: f32,
 * hvk_ln_bwd_workspace_bytes(C) bytes. */
size_t hvk_ln_bwd_workspace_bytes(int C);
int hvk_ln_residual_bwd(const void* a, const float* abias, const float* gamma,
                        const float* sample_scale, const float* mean, const float* rstd,
                        const float* gx, const void* gxb, int rows, int C, int rows_per_sample,
                        float* gx0, void* ga, float* dgamma, float* dbeta, float* dabias,
                        float* workspace, size_t workspace_bytes, void* stream);
/* The same with the dgamma / dbeta / dabias column sums launched on param_stream (ordered after
 * the row kernel on `stream` by an event; NULL or == stream: as above), so the parameter
 * gradients overlap the input-gradient chain.  ABI 13. */
int hvk_ln_residual_bwd_split(const void* a, const float* abias, const float* gamma, const float* sample_scale,
                              const float* mean, const float* rstd, const float* gx, const void* gxb, int rows,
                              int C, int rows_per_sample, float* gx0, void* ga, float* dgamma, float* dbeta,
                              float* dabias, float* workspace, size_t workspace_bytes, void* stream,
                              void* param_stream);

/* Final LayerNorm + token average pool (swinv2.py:833-835): y [B, C] = mean over T of
 * LN(x [B, T, C] f32) (eps, gamma, beta).  The forward keeps xsum [B, C] = sum_t xhat and
 * the row statistics mean / rstd [B*T] for the backward, and zeroes dgamma_zero / dbeta_zero
 * [C], the accumulators hvk_ln_pool_bwd adds d gamma / d beta into (float atomics).
 * hvk_ln_pool_supported(C): C a multiple of 256, C / 256 in 1..4 or 6. */
int hvk_ln_pool_supported(int C);
int hvk_ln_pool_fwd(const float* x, const float* gamma, const float* beta, int B, int T, int C, float eps,
                    float* y, float* xsum, float* mean, float* rstd, float* dgamma_zero, float* dbeta_zero,
                    void* stream);
int hvk_ln_pool_bwd(const float* x, const float* gamma, const float* mean, const float* rstd, const float* xsum,
                    const float* dy, int B, int T, int C, float* dx, float* dgamma, float* dbeta, void* stream);

/* ---- MLP activation: y = GELU(h + bias), exact erf form (swinv2.py:60-62, nn.GELU) ---
 * h: bf16 [rows, N] = fc1 GEMM output without bias; bias: f32 [N] or NULL; y: bf16.
 * Backward: gh = gy * GELU'(h + bias) (bf16) and dbias = column sums of gh (f32 [N],
 * overwritten, may be NULL; needs hvk_bias_gelu_bwd_workspace_bytes(N) of workspace). */
int hvk_bias_gelu_fwd(const void* h, const float* bias, void* y, int rows, int N, void* stream);
size_t hvk_bias_gelu_bwd_workspace_bytes(int N);
int hvk_bias_gelu_bwd(const void* h, const float* bias, const void* gy, void* gh, float* dbias,
                      float* workspace, size_t workspace_bytes, int rows, int N, void* stream);

/* ---- PatchMerging 2x2 gather (swinv2.py:484-491) -----------------------------------
 * out[b, (i, j), k*C + c] = x[b, (2i + dh_k, 2j + dw_k), c],
 * (dh, dw)_k = (0,0), (1,0), (0,1), (1,1); x: bf16 [B, H*W, C], out: bf16 [B, H*W/4, 4C].
 * scatter is the exact inverse (a permutation: every element written once). */
int hvk_patch_merge_gather(const void* x, void* out, int B, int H, int W, int C, void* stream);
/* PatchEmbed input (swinv2.py:652-660, the 4x4/s4 Conv2d as a GEMM): f32 images
 * x [B, C, H, W] -> bf16 patches [B, (H/4)(W/4), C*16] in (c, py, px) order, rounded to
 * nearest even (x.to(bfloat16) + permute + reshape in one pass).  C = 3 is built. */
int hvk_patchify_bf16(const float* x, void* out, int B, int C, int H, int W, void* stream);

/* ---- Device-side input normalisation (data.py:130-136, composer NormalizationFn) ------
 * x: the uint8 [B, C, H, W] batch of pil_image_collate (data.py:36-76); mean / std: DEVICE f32
 * [C] in the 0-255 scale (data.py:128-133).  hvk_patchify_u8_bf16 = NormalizationFn fused into
 * hvk_patchify_bf16: out[b, patch, (c, py, px)] = bf16((x - mean[c]) / std[c]) (division
 * correctly rounded, as torch's sub_ + div_ in f32, then round-to-nearest-even); C = 3,
 * H, W multiples of 4.  hvk_normalize_u8 = the transform alone: out f32 [B, C, HW] =
 * (x - mean[c]) / std[c] (HW a multiple of 4). */
int hvk_patchify_u8_bf16(const uint8_t* x, void* out, const float* mean, const float* std, int B, int C, int H,
                         int W, void* stream);
int hvk_normalize_u8(const uint8_t* x, float* out, const float* mean, const float* std, int B, int C, int HW,
                     void* stream);
int hvk_patch_merge_scatter(const void* gout, void* gx, int B, int H, int W, int C,
                            void* stream);

/* ---- PatchMerging as one strided-gather + Linear (swinv2.py:484-494), ABI 12 -------------
 * The reduction Linear (4C -> N, no bias) with the 2x2 gather above folded into its operand
 * loads, so the [B, H*W/4, 4C] tensor is never written: x bf16 [B, H*W, C] (the token rows),
 * w bf16 [N, 4C], M = B*H*W/4 merged rows.  Results are bit-identical to
 * hvk_patch_merge_gather + hvk_gemm_fwd (and + hvk_linear_ln_fwd, + hvk_gemm_fwd on the input
 * gradient + hvk_patch_merge_scatter, + hvk_weight_grad) with default options.
 *   hvk_merge_gemm_fwd:      y bf16 [M, N] = gather(x) w^T
 *   hvk_merge_linear_ln_fwd: the same with PatchMerging's norm in the epilogue (N = 192):
 *                            a = gather(x) w^T, x_out / xb_out / mean / rstd as hvk_linear_ln_fwd
 *                            with no abias, x0 or sample scale
 *   hvk_merge_gemm_dgrad:    gx bf16 [B, H*W, C] = scatter(gy wt^T), gy bf16 [M, N], wt = w^T
 *                            bf16 [4C, N] (every element of gx written once)
 *   hvk_merge_weight_grad:   dw f32 [N, 4C] = gy^T gather(x); workspace
 *                            hvk_weight_grad_workspace(M, N, 4C)
 * _supported: H, W even, C % 8 == 0, M < 2^21, and the tiled GEMM / weight-gradient plans of
 * the shape (K = 4C a multiple of 64, N of 128 or 192). */
int hvk_merge_gemm_supported(int B, int H, int W, int C, int N);
int hvk_merge_gemm_fwd(const void* x, const void* w, void* y, int B, int H, int W, int C, int N, void* stream);
int hvk_merge_linear_ln_supported(int B, int H, int W, int C, int N);
int hvk_merge_linear_ln_fwd(const void* x, const void* w, int B, int H, int W, int C, int N, const float* gamma,
                            const float* beta, float eps, void* a_out, float* x_out, void* xb_out, float* mean,
                            float* rstd, void* stream);
int hvk_merge_gemm_dgrad(const void* gy, const void* wt, void* gx, int B, int H, int W, int C, int N, void* stream);
int hvk_merge_weight_grad_supported(int B, int H, int W, int C, int N);
int hvk_merge_weight_grad(const void* gy, const void* x, float* dw, int B, int H, int W, int C, int N, void* ws,
                          size_t ws_bytes, void* stream);

/* ---- Multitask / flat cross-entropy (hierarchy.py:65-94; models.py:112) -----------
 * logits: f32 [B, ld]; head h occupies columns [head_off[h], head_off[h+1]).
 * Targets: hard int64 [B, n_heads] (targets[b*n_heads + h]) or soft f32 [B, ld] (one of
 * them non-NULL).  Forward writes row_loss f32 [n_heads, B] (per-row CE) and lse
 * f32 [n_heads, B].  Backward: dlogits = grad_out * coeff[h] / B * (softmax*sum(t) - t). */
int hvk_multitask_ce_fwd(const float* logits, int ld, int B, int n_heads, const int* head_off,
                         const int64_t* targets, const float* soft, float* row_loss,
                         float* lse, void* stream);
int hvk_multitask_ce_bwd(const float* logits, int ld, int B, int n_heads, const int* head_off,
                         const int64_t* targets, const float* soft, const float* lse,
                         const float* coeff, const float* grad_out, float* dlogits,
                         void* stream);

/* ---- Hierarchical cross-entropy (HXE) --------------------------------------------
 * Not implemented by the reference (hierarchy.py:183-185, models.py:105-106); knobs from
 * configs.py:93-96.  Leaves are visited in `perm` order (NULL = identity) in which every
 * taxonomy node owns a contiguous range: node n of tier t spans permuted positions
 * [node_start[tier_base[t] + n], node_end[tier_base[t] + n]).  targets: int64 [B, 7] tier
 * ids (tier 6 = leaf).  level_coeff f32 [8]: L_b = sum_l level_coeff[l] * LSE_l with
 * LSE_l the log-sum-exp of logits over the target's level-l node (l = 0 leaf ... 6 top
 * tier, 7 = all leaves).  Forward: row_loss f32 [B], lse f32 [B, 8].  Backward:
 * dlogits = grad_out / B * sum_l level_coeff[l] * [k in node_l] * exp(z_k - LSE_l). */
int hvk_hxe_fwd(const float* logits, int B, int L, const int* perm, const int64_t* targets,
                const int* node_start, const int* node_end, const int* tier_base,
                const float* level_coeff, float* row_loss, float* lse, void* stream);
int hvk_hxe_bwd(const float* logits, int B, int L, const int* perm, const int64_t* targets,
                const int* node_start, const int* node_end, const int* tier_base,
                const float* level_coeff, const float* lse, const float* grad_out,
                float* dlogits, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HVK_H_ */
