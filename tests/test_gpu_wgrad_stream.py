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


def _linear_grads(w, b, x, twice, on):
    from hvamd import ops, options
    w.grad = b.grad = None
    ops.reset_leaf_uses()
    with options.override(wgrad_stream=on), torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.linear(x, w, b)
        if twice:  # the same parameters in one graph twice: autograd sums their two gradients
            y = ops.linear(y, w, b)
        with ops.wgrad_stream_scope():
            y.float().square().mean().backward()
    return w.grad.detach().clone(), b.grad.detach().clone()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("twice", [False, True])
def test_side_stream_refuses_unsafe_leaves(dtype, twice):
    """a Linear applied twice (tied weights) and bf16 parameters (autograd casts
    the f32 gradient on the current stream) must not put their gradients on the side stream --
    the gradients equal the side-stream-off run, and the fork count does not move for them."""
    from hvamd import ops
    torch.manual_seed(3)
    w = torch.nn.Parameter((torch.randn(192, 192, device="cuda") / 14).to(dtype))
    b = torch.nn.Parameter(torch.randn(192, device="cuda").to(dtype))
    x = torch.randn(4096, 192, device="cuda")
    ref = _linear_grads(w, b, x, twice, False)
    f0 = ops.wgrad_fork_count()
    got = _linear_grads(w, b, x, twice, True)
    forked = ops.wgrad_fork_count() - f0
    torch.cuda.synchronize()
    assert forked == (1 if dtype == torch.float32 and not twice else 0), forked
    for a, r in zip(got, ref):
        assert torch.equal(a.float(), r.float())


def test_bucket_hook_takes_no_wait_path_for_side_gradients():
    """a gradient written on the side stream is recognised by storage (autograd
    stores a detached alias), so GradientBuckets' hook copies it without making the side stream
    wait on the current one; a parameter-gradient the current stream wrote is not."""
    from hvamd import ops
    blk = _block(96, 3)
    x = torch.randn(2, 28 * 28, 96, device="cuda")
    seen = {}

    def hook(name):
        def h(p):
            seen[name] = (ops.wgrad_side_pending() is not None, ops.wgrad_produced_on_side(p.grad))
        return h
    hs = [blk.mlp.fc1.weight.register_post_accumulate_grad_hook(hook("fc1")),
          blk.norm1.weight.register_post_accumulate_grad_hook(hook("norm1"))]
    ops.reset_leaf_uses()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x)
    with ops.wgrad_stream_scope():
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    assert seen["fc1"] == (True, True), seen
    assert seen["norm1"][1] is False, seen  # the LayerNorm column sums ran on the current stream


def test_ln_column_sums_on_side_stream_equal():
    """options.wgrad_stream_ln (hvk_ln_residual_bwd_split: the LayerNorm
    backward's column sums on the side stream) gives the same gradients as the single-stream
    kernel: same kernels, same partial sums (the CPB chain's atomics aside, as in _compare)."""
    from hvamd import options
    blk = _block(192, 6)
    x = torch.randn(8, 28 * 28, 192, device="cuda")
    g0 = _grads(blk, x, True)
    with options.override(wgrad_stream_ln=True):
        g1 = _grads(blk, x, True)
    _compare(g0, g1)


def test_side_stream_buffers_reused_with_host_ahead():
    """Side-stream operands are held until the join (ops.wgrad_hold), not freed with
    record_stream: with the host several steps ahead of the GPU (a spin kernel per step here;
    SwinV2-B 384's 180 ms steps against ~40 ms of enqueue in the bench), record_stream left every
    such block unavailable until the GPU caught up, so each step mapped fresh HBM (287 GB
    reserved, 470-650 ms per step).  After two warm-up steps no step may map new memory, and the
    gradients match a synchronised run."""
    from hvamd import ops
    blk = _block(96, 3)
    x = torch.randn(4, 28 * 28, 96, device="cuda")

    def step():
        blk.zero_grad(set_to_none=True)
        ops.reset_leaf_uses()
        torch.cuda._sleep(20_000_000)  # ~10 ms of GPU time: the host runs ahead
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(x)
        with ops.wgrad_stream_scope():
            y.float().square().mean().backward()
        return {n: p.grad for n, p in blk.named_parameters() if p.grad is not None}

    ref = {n: g.detach().clone() for n, g in step().items()}
    torch.cuda.synchronize()
    step()
    torch.cuda.synchronize()
    a0 = torch.cuda.memory_stats().get("num_device_alloc", 0)
    for _ in range(6):
        last = step()
    a1 = torch.cuda.memory_stats().get("num_device_alloc", 0)
    torch.cuda.synchronize()
    assert not ops._WgradStream.held  # released at the join
    assert a1 == a0, f"{a1 - a0} device allocations over 6 steps with the host ahead"
    for n, g in last.items():
        if n.split(".")[-2:] in EXACT:
            assert torch.equal(g.view(torch.int32), ref[n].view(torch.int32)), n
