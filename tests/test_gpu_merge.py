"""PatchMerging as one strided-gather + Linear (swinv2.py:484-494; hvk_merge_*, include/hvk.h):
the 2x2 gather folded into the reduction GEMM's operand loads, the input gradient scattered by the
dgrad GEMM's store and the weight gradient gathering on its DMA, against the launches they replace
(hvk_patch_merge_gather + hvk_gemm_fwd / hvk_linear_ln_fwd, hvk_gemm_fwd + hvk_patch_merge_scatter,
hvk_weight_grad on the gathered tensor): bit for bit -- the same tiles run the same k order, only
the addresses differ -- and the PatchMerging module's outputs and gradients with the option
merge_gemm on equal those with it off."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (B, H, W, C, N): the SwinV2-T merges (stage 0 -> 1, 1 -> 2, 2 -> 3), SwinV2-B's stage 0 -> 1
# (C = 128, the 128-column tiles), and ragged merged-row counts (M % 128 != 0; the weight
# gradient's plan takes M % 32 == 0)
SHAPES = [(4, 56, 56, 96, 192), (8, 28, 28, 192, 384), (32, 14, 14, 384, 768), (2, 48, 48, 128, 256),
          (5, 16, 16, 96, 192), (8, 12, 20, 192, 384)]


def _lib():
    from hvamd import _lib
    return _lib


def _same(a, b, name):
    v = torch.int16 if a.dtype == torch.bfloat16 else torch.int32
    assert torch.equal(a.view(v), b.view(v)), name


def _operands(B, H, W, C, N, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(B, H * W, C, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, 4 * C, device="cuda", generator=g) / (4 * C) ** 0.5).bfloat16()
    gy = torch.randn(B * H * W // 4, N, device="cuda", generator=g).bfloat16()
    return x, w, gy


def _gather(x, B, H, W, C):
    lib = _lib()
    xm = torch.empty(B * H * W // 4, 4 * C, device="cuda", dtype=torch.bfloat16)
    lib.call("hvk_patch_merge_gather", lib.ptr(x), lib.ptr(xm), B, H, W, C, lib.stream())
    return xm


@pytest.mark.parametrize("B,H,W,C,N", SHAPES)
def test_merge_gemm_fwd_dgrad_wgrad_bit_identical(B, H, W, C, N):
    lib = _lib()
    L = lib.load()
    assert L.hvk_merge_gemm_supported(B, H, W, C, N) and L.hvk_merge_weight_grad_supported(B, H, W, C, N)
    M = B * H * W // 4
    x, w, gy = _operands(B, H, W, C, N, B * H + C)
    xm = _gather(x, B, H, W, C)
    # forward
    y0 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    lib.call("hvk_gemm_fwd", lib.ptr(xm), lib.ptr(w), None, lib.ptr(y0), M, 4 * C, N, lib.stream())
    y1 = torch.full_like(y0, float("nan"))
    lib.call("hvk_merge_gemm_fwd", lib.ptr(x), lib.ptr(w), lib.ptr(y1), B, H, W, C, N, lib.stream())
    # input gradient: GEMM against w^T, then the scatter
    wt = w.t().contiguous()
    gxm = torch.empty(M, 4 * C, device="cuda", dtype=torch.bfloat16)
    lib.call("hvk_gemm_fwd", lib.ptr(gy), lib.ptr(wt), None, lib.ptr(gxm), M, N, 4 * C, lib.stream())
    gx0 = torch.empty_like(x)
    lib.call("hvk_patch_merge_scatter", lib.ptr(gxm), lib.ptr(gx0), B, H, W, C, lib.stream())
    gx1 = torch.full_like(x, float("nan"))
    lib.call("hvk_merge_gemm_dgrad", lib.ptr(gy), lib.ptr(wt), lib.ptr(gx1), B, H, W, C, N, lib.stream())
    # weight gradient
    nb = L.hvk_weight_grad_workspace(M, N, 4 * C)
    ws = torch.empty(nb // 4, device="cuda")
    dw0 = torch.empty(N, 4 * C, device="cuda")
    lib.call("hvk_weight_grad", lib.ptr(gy), lib.ptr(xm), lib.ptr(dw0), None, M, N, 4 * C, lib.ptr(ws), nb,
             lib.stream())
    dw1 = torch.full_like(dw0, float("nan"))
    lib.call("hvk_merge_weight_grad", lib.ptr(gy), lib.ptr(x), lib.ptr(dw1), B, H, W, C, N, lib.ptr(ws), nb,
             lib.stream())
    torch.cuda.synchronize()
    _same(y0, y1, "y")
    _same(gx0, gx1, "gx")
    _same(dw0, dw1, "dw")
    # and against torch on the permutation itself (a strided view of x)
    xr = x.view(B, H, W, C)
    xt = torch.cat([xr[:, 0::2, 0::2], xr[:, 1::2, 0::2], xr[:, 0::2, 1::2], xr[:, 1::2, 1::2]], -1)
    ref = xt.reshape(M, 4 * C).float() @ w.float().t()
    assert ((y1.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("B", [4, 3])
def test_merge_linear_ln_bit_identical(B):
    lib = _lib()
    H = W = 56
    C, N = 96, 192
    M = B * H * W // 4
    assert lib.load().hvk_merge_linear_ln_supported(B, H, W, C, N)
    x, w, _ = _operands(B, H, W, C, N, 11 + B)
    g = torch.Generator(device="cuda").manual_seed(B)
    gamma = torch.randn(N, device="cuda", generator=g)
    beta = torch.randn(N, device="cuda", generator=g)
    xm = _gather(x, B, H, W, C)
    outs = []
    for merged in (False, True):
        a = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        xo = torch.full((M, N), float("nan"), device="cuda")
        xb = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        mean = torch.full((M,), float("nan"), device="cuda")
        rstd = torch.full((M,), float("nan"), device="cuda")
        if merged:
            lib.call("hvk_merge_linear_ln_fwd", lib.ptr(x), lib.ptr(w), B, H, W, C, N, lib.ptr(gamma), lib.ptr(beta),
                     1e-5, lib.ptr(a), lib.ptr(xo), lib.ptr(xb), lib.ptr(mean), lib.ptr(rstd), lib.stream())
        else:
            lib.call("hvk_linear_ln_fwd", lib.ptr(xm), lib.ptr(w), M, 4 * C, N, None, None, lib.ptr(gamma),
                     lib.ptr(beta), None, 1, 1e-5, lib.ptr(a), lib.ptr(xo), lib.ptr(xb), lib.ptr(mean), lib.ptr(rstd),
                     lib.stream())
        outs.append((a, xo, xb, mean, rstd))
    torch.cuda.synchronize()
    for name, r, o in zip(("a", "x", "xb", "mean", "rstd"), *outs):
        _same(r, o, name)


# batches at which the materialised path runs the same tiled GEMMs (ops._tile_ok) and weight
# gradient plan (M % 32 == 0)
@pytest.mark.parametrize("H,C,B", [(56, 96, 42), (28, 192, 48), (14, 384, 192)])
@pytest.mark.parametrize("ln_tile", [True, False])
def test_patch_merging_merge_gemm_equal_materialised(H, C, B, ln_tile):
    """The module: merge_gemm on (gather folded into the GEMMs) against off (gather / scatter
    launches + the same GEMMs): outputs, input and reduction-weight gradients bit for bit, the
    norm's gradients to the run-to-run order of its column sums."""
    import hvamd.swinv2 as sw
    from hvamd import options, ops
    torch.manual_seed(H + C)
    pm = sw.PatchMerging((H, H), dim=C).cuda()
    with torch.no_grad():
        pm.norm.weight.normal_()
        pm.norm.bias.normal_()
    assert ops.merge_linear_supported(B, H, H, C, 2 * C)
    x = torch.randn(B, H * H, C, device="cuda", requires_grad=True)
    outs = []
    for on in (False, True):
        pm.zero_grad(set_to_none=True)
        x.grad = None
        with options.override(merge_gemm=on, ln_epilogue_tile=ln_tile), torch.autocast("cuda", dtype=torch.bfloat16):
            s = pm.forward_stream(sw.ResidualStream(x, x.bfloat16()))
        (s.f32.square().mean() + s.bf16.float().mean()).backward()
        outs.append((s.f32.detach(), s.bf16.detach(), x.grad.clone(),
                     {n: p.grad.clone() for n, p in pm.named_parameters()}))
    for i, name in enumerate(("x", "xb", "dx")):
        _same(outs[0][i], outs[1][i], name)
    assert set(outs[0][3]) == set(outs[1][3])
    _same(outs[0][3]["reduction.weight"], outs[1][3]["reduction.weight"], "reduction.weight")
    for n in ("norm.weight", "norm.bias"):  # the norm backward's column sums: run-to-run order
        rel = ((outs[0][3][n] - outs[1][3][n]).norm() / outs[0][3][n].norm()).item()
        assert rel < 1e-6, (n, rel)
