// Host-side argument validation of libhvk under AddressSanitizer (debug build
// with -fsanitize=address host-side).  Built by `make -C hierarchical-vision_amd/csrc asan`
// from host-only objects (--offload-host-only: no device code, so no GPU is needed): every
// call below must return before any launch -- null pointers, unsupported shapes, short
// workspaces -- and the pure host arithmetic (workspace sizes, support predicates, the error
// text) must stay inside its buffers.  Exit status 0 and no ASan report = pass.
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/hvk.h"

static int g_fail = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                        \
    }                                                                  \
  } while (0)

// a non-null address that is never dereferenced on these paths
static void* const P = reinterpret_cast<void*>(0x1000);

int main() {
  EXPECT(hvk_abi_version() == HVK_ABI_VERSION);

  // options: unknown names and out-of-range values refused, set/get round trip
  long long prev = -7, v = -7;
  EXPECT(hvk_set_option("no_such_option", 0, nullptr) == HVK_EINVAL);
  EXPECT(hvk_set_option(nullptr, 0, nullptr) == HVK_EINVAL);
  EXPECT(hvk_set_option("wmsa_fwd_form", 2, nullptr) == HVK_EINVAL);
  EXPECT(hvk_get_option("wmsa_fwd_form", nullptr) == HVK_EINVAL);
  EXPECT(hvk_set_option("wmsa_fwd_form", 1, &prev) == HVK_OK && prev == 0);
  EXPECT(hvk_get_option("wmsa_fwd_form", &v) == HVK_OK && v == 1);
  EXPECT(hvk_set_option("wmsa_fwd_form", 0, nullptr) == HVK_OK);

  // W-MSA: null pointers, head_dim != 32, window not built, indivisible maps, short workspace
  EXPECT(hvk_wmsa_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, 1, 7, 7, 96, 3, 7, 0, nullptr) == HVK_EINVAL);
  EXPECT(strstr(hvk_last_error_string(), "null") != nullptr);
  float* F = static_cast<float*>(P);
  EXPECT(hvk_wmsa_fwd(P, P, nullptr, F, F, 1, 14, 14, 100, 3, 7, 3, nullptr) == HVK_EUNSUPPORTED);
  EXPECT(hvk_wmsa_fwd(P, P, nullptr, F, F, 1, 10, 10, 96, 3, 5, 0, nullptr) == HVK_EUNSUPPORTED);
  EXPECT(hvk_wmsa_fwd(P, P, nullptr, F, F, 1, 15, 15, 96, 3, 7, 3, nullptr) == HVK_EINVAL);
  EXPECT(hvk_wmsa_fwd(P, P, nullptr, F, F, 1, 14, 14, 96, 3, 7, 7, nullptr) == HVK_EINVAL);
  // one image's qkv past 32-bit byte offsets (7168^2 tokens x 6C) -> refused, no launch, for the
  // w <= 8 forms and the large-window ones, forward and backward
  EXPECT(hvk_wmsa_fwd(P, P, nullptr, F, F, 1, 7168, 7168, 96, 3, 7, 3, nullptr) == HVK_EUNSUPPORTED);
  EXPECT(hvk_wmsa_fwd(P, P, nullptr, F, F, 1, 7176, 7176, 96, 3, 24, 12, nullptr) == HVK_EUNSUPPORTED);
  EXPECT(hvk_wmsa_bwd(P, P, nullptr, nullptr, P, nullptr, F, F, F, F, F, hvk_wmsa_bwd_workspace_bytes(3, 24),
                      1, 7176, 7176, 96, 3, 24, 12, nullptr) == HVK_EUNSUPPORTED);
  EXPECT(hvk_wmsa_bwd(P, P, nullptr, nullptr, P, nullptr, F, F, F, F, F, hvk_wmsa_bwd_workspace_bytes(3, 7),
                      1, 7168, 7168, 96, 3, 7, 3, nullptr) == HVK_EUNSUPPORTED);
  for (int w : {4, 6, 7, 8, 12, 16, 24})
    for (int nh = 1; nh <= 32; ++nh) {
      const size_t ws = hvk_wmsa_bwd_workspace_bytes(nh, w);
      EXPECT(ws > 0 && ws % 4 == 0);
      EXPECT(hvk_wmsa_bwd(P, P, nullptr, nullptr, P, nullptr, F, F, F, F, F, ws - 4, 1, 2 * w, 2 * w,
                          32 * nh, nh, w, 0, nullptr) == HVK_EINVAL);
    }
  EXPECT(hvk_wmsa_bwd(P, P, nullptr, F, P, nullptr, F, F, F, F, F, 1 << 20, 1, 24, 24, 64, 2, 12, 6,
                      nullptr) == HVK_EINVAL);  // lse without the forward's output

  // GEMM / linear predicates over a shape grid (pure host decisions)
  for (int M : {1, 16, 32, 1000, 802816})
    for (int K : {48, 96, 128, 192, 256, 384, 512, 768, 1024, 1536, 3072})
      for (int N : {96, 128, 192, 256, 288, 384, 512, 768, 1024, 1152, 1536, 3072}) {
        (void)hvk_linear_supported(M, K, N);
        (void)hvk_linear_gelu_supported(M, K, N);
        (void)hvk_linear_gelu_bwd_supported(M, K, N);
        (void)hvk_gemm_supported(M, K, N);
        (void)hvk_linear_gelu_in_supported(M, K, N);
        (void)hvk_weight_grad_gelu_x_supported(M, K, N);
        if (hvk_weight_grad_supported(M, N, K)) EXPECT(hvk_weight_grad_workspace(M, N, K) > 0);
      }
  EXPECT(hvk_linear_fwd(nullptr, nullptr, nullptr, nullptr, 16, 96, 96, nullptr) == HVK_EINVAL);
  EXPECT(hvk_gemm_fwd(nullptr, nullptr, nullptr, nullptr, 128, 384, 1152, nullptr) == HVK_EINVAL);
  EXPECT(hvk_weight_grad(nullptr, nullptr, nullptr, nullptr, 32, 96, 96, nullptr, 0, nullptr) == HVK_EINVAL);
  EXPECT(hvk_mlp_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 16, 96, 384, 96,
                     nullptr) == HVK_EINVAL);
  // no device here: the fused MLP's LDS cannot be granted, so it reports unsupported
  EXPECT(hvk_mlp_fwd_supported(16, 96, 384, 96) == 0);

  // LayerNorm / pointwise / merge / patchify
  EXPECT(hvk_ln_bwd_workspace_bytes(96) > 0);
  EXPECT(hvk_bias_gelu_fwd(P, nullptr, P, 4, 12, nullptr) == HVK_EUNSUPPORTED);
  EXPECT(hvk_patch_merge_gather(P, P, 1, 7, 7, 32, nullptr) == HVK_EINVAL);
  EXPECT(hvk_patchify_bf16(nullptr, nullptr, 1, 3, 224, 224, nullptr) == HVK_EINVAL);

  // losses
  EXPECT(hvk_hxe_fwd(nullptr, 2, 12, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                     nullptr) == HVK_EINVAL);
  EXPECT(hvk_multitask_ce_fwd(nullptr, 2, 3, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) ==
         HVK_EINVAL);

  // fused optimizer: workspace arithmetic over ragged tensor lists, then invalid calls
  std::vector<long long> numel;
  for (int i = 0; i < 300; ++i) numel.push_back(1 + (i * 7919) % 100003);
  const size_t sw = hvk_sgdw_workspace_bytes((int)numel.size(), numel.data());
  EXPECT(sw > 0);
  EXPECT(hvk_sgdw_step(0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1, nullptr,
                       1.f, 0.f, 0.9f, 0.f, 0, 1, 0.f, nullptr, 0, nullptr) == HVK_OK);  // nothing to do
  float* const* PP = reinterpret_cast<float* const*>(P);
  const float* const* CP = reinterpret_cast<const float* const*>(P);
  const int grp[1] = {0};
  const float lr[4] = {0.1f, 0, 0, 0}, dec[4] = {1, 1, 1, 1};
  EXPECT(hvk_sgdw_step(3, PP, CP, PP, nullptr, numel.data(), nullptr, lr, dec, 1, nullptr, 1.f, 0.f, 0.9f, 0.f,
                       0, 1, 0.f, F, sw, nullptr) == HVK_EINVAL);  // no group table
  EXPECT(hvk_sgdw_step(3, PP, CP, PP, nullptr, numel.data(), grp, lr, dec, 1, nullptr, 0.f, 0.f, 0.9f, 0.f,
                       0, 1, 0.f, F, sw, nullptr) == HVK_EINVAL);  // grad_scale 0
  EXPECT(hvk_sgdw_step(3, PP, CP, PP, nullptr, numel.data(), grp, lr, dec, 9, nullptr, 1.f, 0.f, 0.9f, 0.f,
                       0, 1, 0.f, F, sw, nullptr) == HVK_EINVAL);  // too many groups
  EXPECT(hvk_sgdw_step(300, PP, CP, PP, nullptr, numel.data(), grp, lr, dec, 1, nullptr, 1.f, 0.f, 0.9f, 0.f,
                       0, 1, 0.f, F, sw - 4, nullptr) == HVK_EINVAL);  // short workspace

  // timer API without launches
  double t = -1.0;
  int n = -1;
  EXPECT(hvk_kernel_timer_read(0, nullptr, &n) == HVK_EINVAL);
  EXPECT(hvk_kernel_timer_enable(0) == HVK_OK);
  EXPECT(hvk_kernel_timer_read(0, &t, &n) == HVK_OK && n == 0 && t == 0.0);

  // the error text stays inside its buffer however long the message
  EXPECT(hvk_wmsa_fwd(P, P, nullptr, F, F, 1, 14, 14, 96, 3, 9, 0, nullptr) == HVK_EUNSUPPORTED);
  EXPECT(strlen(hvk_last_error_string()) < 512);

  if (g_fail) {
    fprintf(stderr, "%d host check(s) failed\n", g_fail);
    return 1;
  }
  printf("host checks ok\n");
  return 0;
}
