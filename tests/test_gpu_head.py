"""Classifier-head GEMMs (head.hip: hvk_head_fwd / hvk_head_bwd, ops.head_linear) against a
plain PyTorch fp32 reference of the same ops on the same bf16 operands: the head Linear of
swinv2.py:786-794 (10 000 HXE leaves) and the concatenated multitask tiers of
hierarchy.py:19-47.  Tolerances: the forward output is one bf16 rounding of an f32 sum (2^-8
relative); the f32 gradients differ from the reference only by summation order (1e-4)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    import hvamd._lib as lib
    return lib


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("M,K,N", [(256, 768, 10000), (37, 96, 24), (1, 1024, 16328), (130, 768, 64), (64, 32, 8)])
def test_head_kernels_match_torch(M, K, N):
    lib = _lib()
    assert lib.load().hvk_head_supported(M, K, N)
    g0 = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    x = torch.randn(M, K, device="cuda", generator=g0).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g0) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g0)
    g = torch.randn(M, N, device="cuda", generator=g0).bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    lib.call("hvk_head_fwd", lib.ptr(x), lib.ptr(w), lib.ptr(b), lib.ptr(y), M, K, N, lib.stream())
    nb = lib.load().hvk_head_bwd_workspace_bytes(M, K, N)
    ws = torch.empty(max(nb, 4) // 4, device="cuda")
    gx = torch.full((M, K), float("nan"), device="cuda")
    dw = torch.full((N, K), float("nan"), device="cuda")
    db = torch.full((N,), float("nan"), device="cuda")
    lib.call("hvk_head_bwd", lib.ptr(g), lib.ptr(x), lib.ptr(w), lib.ptr(gx), lib.ptr(dw), lib.ptr(db), M, K, N,
             lib.ptr(ws), nb, lib.stream())
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t() + b
    assert (y.float() - ref).abs().max().item() <= 2 ** -8 * ref.abs().max().item() + 1e-6
    assert _rel(y, ref) < 4e-3
    assert _rel(gx, g.float() @ w.float()) < 1e-4
    assert _rel(dw, g.float().t() @ x.float()) < 1e-4
    assert _rel(db, g.float().sum(0)) < 1e-4
    # gradients only for what is asked (NULL outputs)
    gx2 = torch.empty_like(gx)
    lib.call("hvk_head_bwd", lib.ptr(g), None, lib.ptr(w), lib.ptr(gx2), None, None, M, K, N, lib.ptr(ws), nb,
             lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(gx2, gx)


def test_head_rejects_unaligned():
    lib = _lib()
    assert not lib.load().hvk_head_supported(256, 768, 10001)
    assert not lib.load().hvk_head_supported(256, 770, 10000)


@pytest.mark.parametrize("sizes", [[10000], [4, 13, 51, 273, 1103, 4884, 9999], [1000, 24]])
@pytest.mark.parametrize("bias", [True, False])
def test_head_linear_autograd(sizes, bias):
    """ops.head_linear (one GEMM over the concatenated tiers, padded to a multiple of 8) vs one
    fp32 Linear per tier on the same bf16 operands, forward and backward."""
    import hvamd.ops as ops
    torch.manual_seed(len(sizes) + bias)
    M, K = 48, 768
    x = torch.randn(M, K, device="cuda", requires_grad=True)
    ws = [torch.nn.Parameter(torch.randn(n, K, device="cuda") / K ** 0.5) for n in sizes]
    bs = [torch.nn.Parameter(torch.randn(n, device="cuda")) if bias else None for n in sizes]
    assert ops.head_supported(x, ws)
    outs = ops.head_linear(x, ws, bs)
    gs = [torch.randn(M, n, device="cuda").bfloat16() for n in sizes]
    torch.autograd.backward(outs, gs)
    xr = x.detach().bfloat16().float().requires_grad_(True)
    wr = [w.detach().bfloat16().float().requires_grad_(True) for w in ws]
    br = [b.detach().clone().requires_grad_(True) if bias else None for b in bs]
    refs = [xr @ w.t() + (b if b is not None else 0) for w, b in zip(wr, br)]
    torch.autograd.backward(refs, [g.float() for g in gs])
    for o, r in zip(outs, refs):
        assert o.dtype == torch.bfloat16 and o.shape == r.shape
        assert _rel(o, r) < 4e-3
    assert x.grad.dtype == torch.float32 and _rel(x.grad, xr.grad) < 1e-4
    for w, r in zip(ws, wr):
        assert _rel(w.grad, r.grad) < 1e-4
    if bias:
        for b, r in zip(bs, br):
            assert _rel(b.grad, r.grad) < 1e-4
