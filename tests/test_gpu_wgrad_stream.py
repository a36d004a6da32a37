"""options.wgrad_stream: the weight-gradient GEMMs on a second HIP stream (ops.weight_grad,
joined at the end of the backward) give the gradients of the single-stream backward -- the same
kernels on the same operands, so the Linear weight gradients bit for bit, the rest (LayerNorm
column sums and the CPB chain's reductions, atomics in either mode) to their run-to-run order."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(blk, x, on):
    from hvamd import options
    blk.zero_grad(set_to_none=True)
    torch.manual_seed(5)
    with options.override(wgrad_stream=on), torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x)
        y.float().square().mean().backward()
    return {n: p.grad.detach().clone() for n, p in blk.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("C,heads,B", [(96, 3, 4), (192, 6, 42)])
def test_block_grads_equal_with_side_stream(C, heads, B):
    import hvamd.swinv2 as sw
    torch.manual_seed(1)
    blk = sw.SwinTransformerBlock(C, (28, 28), heads, window_size=7, shift_size=3).cuda().train()
    x = torch.randn(B, 28 * 28, C, device="cuda")
    g0 = _grads(blk, x, False)
    g1 = _grads(blk, x, True)
    torch.cuda.synchronize()
    assert set(g0) == set(g1)
    for n in g0:
        if n.split(".")[-2:] in (["qkv", "weight"], ["proj", "weight"], ["fc1", "weight"], ["fc2", "weight"]):
            assert torch.equal(g0[n].view(torch.int32), g1[n].view(torch.int32)), n
        rel = ((g0[n] - g1[n]).norm() / (g0[n].norm() + 1e-30)).item()
        assert rel < 1e-6, (n, rel)
