"""The post-norm LayerNorm + residual fused into the producing GEMM's epilogue (hvk_linear_ln_fwd:
C = 96 the stage-0 proj and the patch embedding on the skinny kernel, C = 192 the stage-1 proj / fc2
and the stage-0 -> 1 PatchMerging on the 128 x 192 tile; hvk_mlp_ln_fwd: the stage-0 fused MLP)
against the two launches they replace (the GEMM without its bias, then hvk_ln_residual_fwd with
that bias as abias): a, x, xb, mean and rstd bit for bit -- the epilogues run ln_fwd_kernel<8, 16>
/ <8, 32>'s lane layout and arithmetic -- and the block / model paths that route through them
(options.ln_epilogue) equal the unfused ones in outputs and gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from hvamd import _lib
    return _lib


def _ln_ref(a, abias, x0, gamma, beta, sscale, rps, eps):
    lib = _lib()
    M, C = a.shape
    x = torch.empty(M, C, device="cuda")
    xb = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    mean = torch.empty(M, device="cuda")
    rstd = torch.empty(M, device="cuda")
    lib.call("hvk_ln_residual_fwd", lib.ptr(a), lib.ptr(abias), lib.ptr(x0), lib.ptr(gamma), lib.ptr(beta),
             lib.ptr(sscale), M, C, rps, eps, lib.ptr(x), lib.ptr(xb), lib.ptr(mean), lib.ptr(rstd), lib.stream())
    return x, xb, mean, rstd


def _params(M, C, seed, with_x0, with_dp, rps):
    g = torch.Generator(device="cuda").manual_seed(seed)
    gamma = torch.randn(C, device="cuda", generator=g)
    beta = torch.randn(C, device="cuda", generator=g)
    abias = torch.randn(C, device="cuda", generator=g)
    x0 = torch.randn(M, C, device="cuda", generator=g) if with_x0 else None
    ss = (torch.rand(M // rps, device="cuda", generator=g) > 0.3).float() / 0.7 if with_dp else None
    return gamma, beta, abias, x0, ss


def _same(a, b, name):
    if a.dtype == torch.bfloat16:
        assert torch.equal(a.view(torch.int16), b.view(torch.int16)), name
    else:
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), name


@pytest.mark.parametrize("M,K,C", [(4099, 96, 96), (50176, 96, 96), (12544 * 2, 48, 96), (1000, 48, 96),
                                   (4099, 192, 192), (50176, 768, 192), (1000, 384, 192), (200704, 192, 192)])
@pytest.mark.parametrize("with_x0,with_dp", [(True, True), (True, False), (False, False)])
def test_linear_ln_bit_identical(M, K, C, with_x0, with_dp):
    lib = _lib()
    rps = 49 if M % 49 == 0 else 1
    assert lib.load().hvk_linear_ln_supported(M, K, C)
    g = torch.Generator(device="cuda").manual_seed(M + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(C, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    gamma, beta, abias, x0, ss = _params(M, C, M + 7, with_x0, with_dp, rps)
    a0 = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    if C == 96:  # the skinny kernel
        lib.call("hvk_linear_fwd", lib.ptr(x), lib.ptr(w), None, lib.ptr(a0), M, K, C, lib.stream())
    else:  # the 128 x 192 tile
        lib.call("hvk_gemm_fwd", lib.ptr(x), lib.ptr(w), None, lib.ptr(a0), M, K, C, lib.stream())
    ref = _ln_ref(a0, abias, x0, gamma, beta, ss, rps, 1e-5)
    a1 = torch.full_like(a0, float("nan"))
    out = [torch.full_like(ref[0], float("nan")), torch.full_like(ref[1], float("nan")),
           torch.full_like(ref[2], float("nan")), torch.full_like(ref[3], float("nan"))]
    lib.call("hvk_linear_ln_fwd", lib.ptr(x), lib.ptr(w), M, K, C, lib.ptr(abias), lib.ptr(x0), lib.ptr(gamma),
             lib.ptr(beta), lib.ptr(ss), rps, 1e-5, lib.ptr(a1), lib.ptr(out[0]), lib.ptr(out[1]), lib.ptr(out[2]),
             lib.ptr(out[3]), lib.stream())
    torch.cuda.synchronize()
    _same(a0, a1, "a")
    for name, r, o in zip(("x", "xb", "mean", "rstd"), ref, out):
        _same(r, o, name)


@pytest.mark.parametrize("M", [4099, 50176])
@pytest.mark.parametrize("with_dp", [False, True])
def test_mlp_ln_bit_identical(M, with_dp):
    lib = _lib()
    K, N1, N2, rps = 96, 384, 96, 49 if M % 49 == 0 else 1
    assert lib.load().hvk_mlp_ln_supported(M, K, N1, N2)
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w1 = (torch.randn(N1, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b1 = torch.randn(N1, device="cuda", generator=g)
    w2 = (torch.randn(N2, N1, device="cuda", generator=g) / N1 ** 0.5).bfloat16()
    gamma, beta, abias, x0, ss = _params(M, N2, M + 3, True, with_dp, rps)
    h0, g0 = (torch.empty(M, N1, device="cuda", dtype=torch.bfloat16) for _ in range(2))
    a0 = torch.empty(M, N2, device="cuda", dtype=torch.bfloat16)
    lib.call("hvk_mlp_fwd", lib.ptr(x), lib.ptr(w1), lib.ptr(b1), lib.ptr(w2), None, lib.ptr(h0), lib.ptr(g0),
             lib.ptr(a0), M, K, N1, N2, lib.stream())
    ref = _ln_ref(a0, abias, x0, gamma, beta, ss, rps, 1e-5)
    h1, g1 = (torch.full_like(h0, float("nan")) for _ in range(2))
    a1 = torch.full_like(a0, float("nan"))
    out = [torch.full_like(r, float("nan")) for r in ref]
    lib.call("hvk_mlp_ln_fwd", lib.ptr(x), lib.ptr(w1), lib.ptr(b1), lib.ptr(w2), lib.ptr(h1), lib.ptr(g1),
             lib.ptr(a1), M, K, N1, N2, lib.ptr(abias), lib.ptr(x0), lib.ptr(gamma), lib.ptr(beta), lib.ptr(ss), rps,
             1e-5, lib.ptr(out[0]), lib.ptr(out[1]), lib.ptr(out[2]), lib.ptr(out[3]), lib.stream())
    torch.cuda.synchronize()
    for name, r, o in (("h", h0, h1), ("gelu", g0, g1), ("a", a0, a1)) + tuple(zip(("x", "xb", "mean", "rstd"), ref, out)):
        _same(r, o, name)


def _run_block(blk, x, on, seed):
    from hvamd import options
    blk.zero_grad(set_to_none=True)
    blk._dp = None
    torch.manual_seed(seed)
    with options.override(ln_epilogue=on, ln_epilogue_tile=on), torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x)
    y.float().square().mean().backward()
    return y.detach(), {n: p.grad.detach().clone() for n, p in blk.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("C,heads,B", [(96, 3, 4), (192, 6, 42)])
@pytest.mark.parametrize("shift", [0, 3])
def test_block_fused_norms_equal_unfused(shift, C, heads, B):
    """A stage-0 (C = 96, 3 heads) / stage-1 (C = 192, 6 heads; B * 784 >= 32 768 tokens so the
    unfused proj / fc2 run on the same tile kernel) SwinV2 block with the norms fused into proj
    and the MLP against the unfused launches: output bit-identical, every parameter gradient
    equal (the backward runs the same kernels on the same saved tensors)."""
    import hvamd.swinv2 as sw
    from hvamd import ops
    torch.manual_seed(1)
    blk = sw.SwinTransformerBlock(C, (28, 28), heads, window_size=7, shift_size=shift).cuda().train()
    with torch.no_grad():
        for n in (blk.norm1, blk.norm2):
            n.weight.normal_()
            n.bias.normal_()
    with options_override(ln_epilogue_tile=True):
        assert ops.linear_ln_supported(B * 784, C, C) and ops.mlp_ln_supported(B * 784, C, 4 * C, C)
    x = torch.randn(B, 28 * 28, C, device="cuda")
    y0, g0 = _run_block(blk, x, False, 5)
    y1, g1 = _run_block(blk, x, True, 5)
    assert torch.equal(y0.view(torch.int32), y1.view(torch.int32))
    assert set(g0) == set(g1)
    for n in g0:
        rel = ((g0[n] - g1[n]).norm() / (g0[n].norm() + 1e-30)).item()
        assert rel < 1e-6, (n, rel)


def test_patch_embed_fused_norm_equal_unfused():
    import hvamd.swinv2 as sw
    from hvamd import options
    torch.manual_seed(2)
    pe = sw.PatchEmbed(img_size=56, embed_dim=96, norm_layer=torch.nn.LayerNorm).cuda()
    with torch.no_grad():
        pe.norm.weight.normal_()
        pe.norm.bias.normal_()
    x = torch.randn(3, 3, 56, 56, device="cuda")
    outs = []
    for on in (False, True):
        pe.zero_grad(set_to_none=True)
        with options.override(ln_epilogue=on), torch.autocast("cuda", dtype=torch.bfloat16):
            s = pe.forward_stream(x)
        s.f32.square().mean().backward()
        outs.append((s.f32.detach(), s.bf16.detach(), {n: p.grad.clone() for n, p in pe.named_parameters()}))
    assert torch.equal(outs[0][0].view(torch.int32), outs[1][0].view(torch.int32))
    assert torch.equal(outs[0][1].view(torch.int16), outs[1][1].view(torch.int16))
    for n in outs[0][2]:
        rel = ((outs[0][2][n] - outs[1][2][n]).norm() / (outs[0][2][n].norm() + 1e-30)).item()
        assert rel < 1e-6, (n, rel)


def test_patch_merging_fused_norm_equal_unfused():
    """The stage-0 -> 1 PatchMerging (2C = 192): the reduction GEMM with its norm in the tile's
    epilogue against GEMM + LayerNorm launch, bit-identical output and equal gradients."""
    import hvamd.swinv2 as sw
    from hvamd import ops
    torch.manual_seed(3)
    pm = sw.PatchMerging((56, 56), dim=96).cuda()
    with torch.no_grad():
        pm.norm.weight.normal_()
        pm.norm.bias.normal_()
    B = 42
    with options_override(ln_epilogue_tile=True):
        assert ops.linear_ln_supported(B * 784, 384, 192)
    x = torch.randn(B, 56 * 56, 96, device="cuda", requires_grad=True)
    outs = []
    for on in (False, True):
        pm.zero_grad(set_to_none=True)
        x.grad = None
        with options_override(ln_epilogue=on, ln_epilogue_tile=on, merge_gemm=False), \
                torch.autocast("cuda", dtype=torch.bfloat16):
            s = pm.forward_stream(sw.ResidualStream(x, x.bfloat16()))
        (s.f32.square().mean() + s.bf16.float().mean()).backward()
        outs.append((s.f32.detach(), s.bf16.detach(), {n: p.grad.clone() for n, p in pm.named_parameters()}))
    assert torch.equal(outs[0][0].view(torch.int32), outs[1][0].view(torch.int32))
    assert torch.equal(outs[0][1].view(torch.int16), outs[1][1].view(torch.int16))
    for n in outs[0][2]:
        rel = ((outs[0][2][n] - outs[1][2][n]).norm() / (outs[0][2][n].norm() + 1e-30)).item()
        assert rel < 1e-6, (n, rel)


def options_override(**kw):
    from hvamd import options
    return options.override(**kw)
