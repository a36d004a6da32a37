"""options.wgrad_stream: parameter-gradient launches on a second HIP stream inside
ops.wgrad_stream_scope (the Trainer's backward), joined at the end of the backward.  The same
kernels run on the same operands, so the Linear weight gradients come out bit for bit and the rest
(LayerNorm column sums and the CPB chain's reductions, atomics in either mode) to their run-to-run
order; a parameter that already holds a gradient (accumulation) stays on the current stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu

EXACT = (["qkv", "weight"], ["proj", "weight"], ["fc1", "weight"], ["fc2", "weight"])


def _block(C, heads):
    import hvamd.swinv2 as sw
    torch.manual_seed(1)
    return sw.SwinTransformerBlock(C, (28, 28), heads, window_size=7, shift_size=3).cuda().train()


def _grads(blk, x, on, passes=1):
    from hvamd import options, ops
    blk.zero_grad(set_to_none=True)
    for i in range(passes):
        torch.manual_seed(5 + i)
        with options.override(wgrad_stream=on), torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(x)
            with ops.wgrad_stream_scope():
                (y.float().square().mean() * (i + 1)).backward()
    # read straight after the backward: the scope's join orders these reads after the side stream
    return {n: p.grad.detach().clone() for n, p in blk.named_parameters() if p.grad is not None}


def _compare(g0, g1):
    assert set(g0) == set(g1)
    for n in g0:
        if n.split(".")[-2:] in EXACT:
            assert torch.equal(g0[n].view(torch.int32), g1[n].view(torch.int32)), n
        rel = ((g0[n] - g1[n]).norm() / (g0[n].norm() + 1e-30)).item()
        assert rel < 1e-6, (n, rel)


@pytest.mark.parametrize("C,heads,B", [(96, 3, 4), (192, 6, 42)])
def test_block_grads_equal_with_side_stream(C, heads, B):
    blk = _block(C, heads)
    x = torch.randn(B, 28 * 28, C, device="cuda")
    _compare(_grads(blk, x, False), _grads(blk, x, True))


def test_accumulated_grads_equal_with_side_stream():
    """Two backward passes without zeroing: the second accumulates onto .grad on the current
    stream (the fork refuses a parameter that holds a gradient)."""
    blk = _block(96, 3)
    x = torch.randn(4, 28 * 28, 96, device="cuda")
    _compare(_grads(blk, x, False, passes=2), _grads(blk, x, True, passes=2))


@pytest.mark.parametrize("chunks", [64, 128, 512])
@pytest.mark.parametrize("M,N,K", [(50176, 384, 1536), (802816 // 8, 96, 384)])
def test_weight_grad_chunk_target(chunks, M, N, K):
    """libhvk option dw_chunks (workgroups per weight-gradient launch): another token-chunk count
    only reorders the f32 partial sums -- dW / db against the f64 reference."""
    from hvamd import _lib
    g = torch.Generator(device="cuda").manual_seed(M + chunks)
    gy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    ref = gy.double().t() @ x.double()
    with _lib.option("dw_chunks", chunks):
        L = _lib.load()
        nb = L.hvk_weight_grad_workspace(M, N, K)
        ws = torch.empty(nb // 4, device="cuda")
        dw = torch.empty(N, K, device="cuda")
        db = torch.empty(N, device="cuda")
        _lib.call("hvk_weight_grad", _lib.ptr(gy), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db), M, N, K, _lib.ptr(ws),
                  nb, _lib.stream())
        torch.cuda.synchronize()
    assert ((dw.double() - ref).norm() / ref.norm()).item() < 1e-6
    dbr = gy.double().sum(0)
    assert ((db.double() - dbr).norm() / dbr.norm()).item() < 1e-6
