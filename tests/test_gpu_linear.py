"""libhvk skinny MFMA GEMM (hvk_linear_fwd) vs an fp32 matmul of the same bf16 operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(48, 96), (96, 96), (96, 288), (96, 384), (384, 96), (288, 96), (192, 192), (192, 576),
          (192, 768), (384, 192), (384, 1536),
          # SwinV2-B stages 0-1 (C = 128, 256) and its patch embedding
          (48, 128), (128, 128), (128, 384), (128, 512), (256, 256), (256, 768), (256, 1024)]


@pytest.mark.parametrize("K,N", SHAPES)
@pytest.mark.parametrize("M", [1000, 4096])
@pytest.mark.parametrize("with_bias", [False, True])
def test_linear_matches_fp32(K, N, M, with_bias):
    from hvamd import _lib, ops
    assert _lib.load().hvk_linear_supported(M, K, N)
    g = torch.Generator(device="cuda").manual_seed(K * 1000 + N)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) if with_bias else None
    y = ops.mm_nt(x, w, b)
    ref = x.float() @ w.float().t() + (b if with_bias else 0)
    torch.cuda.synchronize()
    rel = ((y.float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel
    assert (y.float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()


def test_linear_autograd_uses_native_and_matches():
    from hvamd import ops
    torch.manual_seed(0)
    x = torch.randn(2, 784, 96, device="cuda").bfloat16().requires_grad_(True)
    w = torch.randn(288, 96, device="cuda", requires_grad=True)
    b = torch.randn(288, device="cuda", requires_grad=True)
    y = ops.linear(x, w, b)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = xr @ wr.t() + br
    yr.backward(gy.float())
    for mine, ref in [(y.float(), yr), (x.grad.float(), xr.grad), (w.grad, wr.grad), (b.grad, br.grad)]:
        rel = ((mine - ref).norm() / ref.norm()).item()
        assert rel < 1e-2, rel


@pytest.mark.parametrize("K,N", [(96, 384), (192, 768), (384, 1536), (128, 512), (256, 1024)])
def test_linear_gelu_fused_matches_fp32(K, N):
    from hvamd import _lib, ops
    M = 3000 if K < 384 else 40000
    assert _lib.load().hvk_linear_gelu_supported(M, K, N)
    gen = torch.Generator(device="cuda").manual_seed(K + N)
    x = torch.randn(M, K, device="cuda", generator=gen).bfloat16().requires_grad_(True)
    w = (torch.randn(N, K, device="cuda", generator=gen) / K ** 0.5).requires_grad_(True)
    b = torch.randn(N, device="cuda", generator=gen).requires_grad_(True)
    y = ops.linear_gelu(x, w, b)
    gy = torch.randn(M, N, device="cuda", generator=gen)
    y.backward(gy.bfloat16())
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.gelu(xr @ wr.t() + br)
    yr.backward(gy.bfloat16().float())
    torch.cuda.synchronize()
    for name, mine, ref in [("y", y.float(), yr), ("dx", x.grad.float(), xr.grad),
                            ("dw", w.grad, wr.grad), ("db", b.grad, br.grad)]:
        rel = ((mine - ref).norm() / ref.norm()).item()
        assert rel < 1e-2, (name, rel)


@pytest.mark.parametrize("with_b2", [False, True])
def test_mlp_gelu_recompute_bit_identical(monkeypatch, with_b2):
    """Stage 0 MlpFn keeps only h and recomputes GELU(h) inside fc2's forward
    (hvk_linear_gelu_in_fwd) and weight gradient (hvk_weight_grad_gelu_x): every output and
    gradient equals the stored-GELU(h) path bit for bit."""
    from hvamd import ops
    M, C = 4096, 96
    torch.manual_seed(3)
    x0 = torch.randn(M, C, device="cuda").bfloat16()
    w1 = torch.randn(4 * C, C, device="cuda") / C ** 0.5
    b1 = torch.randn(4 * C, device="cuda")
    w2 = torch.randn(C, 4 * C, device="cuda") / (4 * C) ** 0.5
    b2 = torch.randn(C, device="cuda") if with_b2 else None
    gy = torch.randn(M, C, device="cuda").bfloat16()
    res = {}
    for rec in (True, False):
        monkeypatch.setattr(ops.OPTIONS, "gelu_recompute", rec)
        assert ops._gelu_recompute(M, C, 4 * C, C) == rec
        ps = [t.clone().requires_grad_(True) if t is not None else None for t in (x0, w1, b1, w2, b2)]
        y = ops.MlpFn.apply(*ps)
        y.backward(gy)
        res[rec] = [y.detach()] + [p.grad for p in ps if p is not None]
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("C", [96, 192, 384, 768, 128, 256])
@pytest.mark.parametrize("with_b2", [False, True])
def test_mlp_fused_backward_matches_fp32(C, with_b2):
    """fc2(GELU(fc1 x)) through the fused kernels (hvk_linear_gelu_fwd / _bwd, the tiled
    hvk_gemm_gelu_fwd / _bwd at stage 2-3) vs an fp32 autograd of the same bf16 operands:
    output, dx, dW1, db1, dW2, db2."""
    from hvamd import _lib, ops
    M, N1 = {96: 3000, 192: 3000, 384: 40000, 768: 12544, 128: 40000, 256: 40000}[C], 4 * C  # stage 2: tiled at M >= 32768
    assert _lib.load().hvk_linear_gelu_bwd_supported(M, C, N1) or ops._tile_ok(M, C, N1)
    gen = torch.Generator(device="cuda").manual_seed(C)
    x = torch.randn(M, C, device="cuda", generator=gen).bfloat16().requires_grad_(True)
    w1 = (torch.randn(N1, C, device="cuda", generator=gen) / C ** 0.5).requires_grad_(True)
    b1 = torch.randn(N1, device="cuda", generator=gen).requires_grad_(True)
    w2 = (torch.randn(C, N1, device="cuda", generator=gen) / N1 ** 0.5).requires_grad_(True)
    b2 = torch.randn(C, device="cuda", generator=gen).requires_grad_(True) if with_b2 else None
    y = ops.mlp(x, w1, b1, w2, b2)
    assert y.grad_fn is not None and "MlpFn" in type(y.grad_fn).__name__
    gy = torch.randn(M, C, device="cuda", generator=gen).bfloat16()
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    w1r = w1.detach().bfloat16().float().requires_grad_(True)
    b1r = b1.detach().clone().requires_grad_(True)
    w2r = w2.detach().bfloat16().float().requires_grad_(True)
    b2r = b2.detach().clone().requires_grad_(True) if with_b2 else None
    yr = torch.nn.functional.gelu(xr @ w1r.t() + b1r) @ w2r.t()
    if with_b2:
        yr = yr + b2r
    yr.backward(gy.float())
    torch.cuda.synchronize()
    pairs = [("y", y.float(), yr), ("dx", x.grad.float(), xr.grad), ("dw1", w1.grad, w1r.grad),
             ("db1", b1.grad, b1r.grad), ("dw2", w2.grad, w2r.grad)]
    if with_b2:
        pairs.append(("db2", b2.grad, b2r.grad))
    for name, mine, ref in pairs:
        rel = ((mine - ref).norm() / ref.norm()).item()
        assert rel < 2e-2, (name, rel)


@pytest.mark.parametrize("M,K,N", [(50176, 384, 1152), (50176, 1536, 384), (12544, 768, 768),
                                   (12544, 3072, 768), (777, 1536, 2304), (300, 192, 384),
                                   (1000, 64, 128), (300, 128, 256), (20000, 768, 192),
                                   (1000, 576, 192), (777, 64, 192)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_gemm_tile_matches_fp32(M, K, N, with_bias):
    """Tiled MFMA GEMM (hvk_gemm_fwd) vs fp32 matmul of the same bf16 operands, on both tile
    widths (128 columns where 128 | N, else 192), including row counts that are not a
    multiple of the 128-row tile."""
    from hvamd import _lib
    lib = _lib.load()
    assert lib.hvk_gemm_supported(M, K, N)
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) if with_bias else None
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b) if with_bias else None, _lib.ptr(y),
              M, K, N, _lib.stream())
    ref = x.float() @ w.float().t() + (b if with_bias else 0)
    torch.cuda.synchronize()
    rel = ((y.float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("M,K,N", [(50176, 384, 1152), (12544, 768, 768), (1000, 576, 384)])
def test_gemm_tile_widths_bit_identical(M, K, N):
    """Where both tile widths divide N, the 128- and 192-column tiles (library option tile_wide)
    accumulate every output in the same k order: bit-identical outputs."""
    from hvamd import _lib
    g = torch.Generator(device="cuda").manual_seed(M * 3 + K + N)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    out = {}
    for wide in (0, 1):
        with _lib.option("tile_wide", wide):
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), M, K, N, _lib.stream())
            torch.cuda.synchronize()
        out[wide] = y
    assert torch.equal(out[0].view(torch.int16), out[1].view(torch.int16))


@pytest.mark.parametrize("N", [384, 256, 192])
def test_gemm_tile_sparse_pattern_pins_layout(N):
    """One nonzero token row and one nonzero weight row: the output must be exactly one
    nonzero element at (token, feature) -- catches permuted rows / columns."""
    from hvamd import _lib
    M, K = 3000, 128
    x = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    t, f = 2777, N - 75
    x[t] = 1
    w[f, :64] = 0.5
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), None, _lib.ptr(y), M, K, N, _lib.stream())
    ref = torch.zeros(M, N, device="cuda")
    ref[t, f] = 32
    torch.cuda.synchronize()
    assert torch.equal(y.float(), ref)


@pytest.mark.parametrize("M,K,N", [(50176, 384, 1536), (1000, 384, 1536), (1000, 512, 2048), (4096, 768, 3072)])
def test_gemm_tile_gelu_matches_fp32(M, K, N):
    """fc1 + bias + GELU on the tiled kernel (EPI 1; 128-column tiles stage h and GELU(h) as two
    LDS images, HVK_EPI1_TWO), ragged M included, against fp32 math on the same bf16 operands."""
    from hvamd import _lib
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = torch.empty_like(h)
    _lib.call("hvk_gemm_gelu_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(h), _lib.ptr(y), M, K,
              N, _lib.stream())
    href = x.float() @ w.float().t() + b
    torch.cuda.synchronize()
    assert ((h.float() - href).norm() / href.norm()).item() < 1e-2
    yref = torch.nn.functional.gelu(h.float())
    assert ((y.float() - yref).norm() / yref.norm()).item() < 1e-2


@pytest.mark.parametrize("M", [50176, 1000])
def test_gemm_tile_gelu_bwd_matches_fp32(M):
    """fc2 input gradient through GELU' on the tiled kernel (hvk_gemm_gelu_bwd): gh =
    (gy w2) * GELU'(h), against fp32 math on the same bf16 operands (ragged M included)."""
    from hvamd import _lib
    K, N = 384, 1536  # gy width (fc2 out), fc1 width
    g = torch.Generator(device="cuda").manual_seed(11)
    gy = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()  # fc2.weight^T
    h = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    gh = torch.empty_like(h)
    _lib.call("hvk_gemm_gelu_bwd", _lib.ptr(gy), _lib.ptr(w), _lib.ptr(h), _lib.ptr(gh), M, K, N,
              _lib.stream())
    hf = h.float().requires_grad_(True)
    torch.nn.functional.gelu(hf).backward(gy.float() @ w.float().t())
    ref = hf.grad
    torch.cuda.synchronize()
    assert ((gh.float() - ref).norm() / ref.norm()).item() < 1e-2
    assert (gh.float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()


@pytest.mark.parametrize("shapes", [
    [(288, 96), (96, 96), (33, 70), (1, 5), (768, 3072), (10, 1)],  # ragged: the 32 x 32 kernel
    [(288, 96), (96, 96), (768, 3072), (10000, 768), (4, 4), (68, 132), (96, 48)],  # 4 | both: 64 x 64
])
def test_cast_weights_bit_exact_and_transposed(shapes):
    """hvk_cast_weights == weight.to(bfloat16) (round to nearest even) and its transpose, for
    shapes that are not multiples of either kernel's tile, in one launch."""
    import ctypes
    from hvamd import _lib
    gen = torch.Generator(device="cuda").manual_seed(3)
    ws = [torch.randn(s, device="cuda", generator=gen) * 3 for s in shapes]
    dst = [torch.empty(s, device="cuda", dtype=torch.bfloat16) for s in shapes]
    dtt = [torch.empty(s[::-1], device="cuda", dtype=torch.bfloat16) for s in shapes]
    n = len(shapes)
    arr = ctypes.c_void_p * n
    a = [arr(*[t.data_ptr() for t in ts]) for ts in (ws, dst, dtt)]
    rows = (ctypes.c_int * n)(*[s[0] for s in shapes])
    cols = (ctypes.c_int * n)(*[s[1] for s in shapes])
    _lib.call("hvk_cast_weights", n, *[ctypes.cast(x, ctypes.c_void_p) for x in a],
              ctypes.cast(rows, ctypes.c_void_p), ctypes.cast(cols, ctypes.c_void_p), _lib.stream())
    torch.cuda.synchronize()
    for w, d, t in zip(ws, dst, dtt):
        assert torch.equal(d, w.to(torch.bfloat16))
        assert torch.equal(t, w.to(torch.bfloat16).t())


def test_cast_weights_misaligned_views():
    """Weights that are views at 4-B (not 16-B) offsets into a flat buffer, with shapes that
    would otherwise take the 16-B-load kernel: the host falls back to the unaligned kernel."""
    import ctypes
    from hvamd import _lib
    shapes = [(96, 96), (288, 96), (4, 4)]
    gen = torch.Generator(device="cuda").manual_seed(4)
    flat = torch.randn(1 + sum(r * c for r, c in shapes), device="cuda", generator=gen)
    ws, off = [], 1  # one float in: every view 4 B past a 16-B boundary
    for r, c in shapes:
        ws.append(flat[off:off + r * c].view(r, c))
        off += r * c
    assert ws[0].data_ptr() % 16 == 4
    dst = [torch.empty(s, device="cuda", dtype=torch.bfloat16) for s in shapes]
    dtt = [torch.empty(s[::-1], device="cuda", dtype=torch.bfloat16) for s in shapes]
    n = len(shapes)
    arr = ctypes.c_void_p * n
    a = [arr(*[t.data_ptr() for t in ts]) for ts in (ws, dst, dtt)]
    rows = (ctypes.c_int * n)(*[s[0] for s in shapes])
    cols = (ctypes.c_int * n)(*[s[1] for s in shapes])
    _lib.call("hvk_cast_weights", n, *[ctypes.cast(x, ctypes.c_void_p) for x in a],
              ctypes.cast(rows, ctypes.c_void_p), ctypes.cast(cols, ctypes.c_void_p), _lib.stream())
    torch.cuda.synchronize()
    for w, d, t in zip(ws, dst, dtt):
        assert torch.equal(d, w.to(torch.bfloat16))
        assert torch.equal(t, w.to(torch.bfloat16).t())


def test_prepared_weights_follow_in_place_updates():
    """The step's bf16 copies are used while the master is unchanged and bypassed after an
    in-place (optimizer-style) update until the next prepare."""
    from hvamd import ops
    torch.manual_seed(1)
    w = torch.randn(288, 96, device="cuda")
    x = torch.randn(4096, 96, device="cuda").bfloat16()
    ops.prepare_weights([w])
    wb, wt = ops._bf16_weight(w)
    assert torch.equal(wb, w.bfloat16()) and torch.equal(wt, w.bfloat16().t())
    y0 = ops.linear(x, w)
    with torch.no_grad():
        w.mul_(2.0)  # version bump: the prepared copy is stale now
    y1 = ops.linear(x, w)
    torch.cuda.synchronize()
    assert torch.allclose(y1.float(), 2 * y0.float(), rtol=2e-2, atol=1e-2)
    ops.prepare_weights([w])
    assert torch.equal(ops._bf16_weight(w)[0], w.bfloat16())


@pytest.mark.parametrize("gscale,ema", [(1.0, False), (0.5, True)])
def test_fused_sgdw_step_matches_foreach_path(gscale, ema):
    """hvk_sgdw_step (DDP mean + clip + DecoupledSGDW + EMA, one fused pass) against the
    foreach path of the same optimizer on CPU copies: two steps (first-step buffer init, then
    the momentum update), decay and no-decay groups, clipping active; with gscale the
    gradients are rank sums (ddp.py) whose 1/world mean is folded into the update, with ema
    the EMA algorithm's average (configs/pretrain/inat21.yaml:31-34) rides on the same pass."""
    from hvamd.optim import DecoupledSGDW
    torch.manual_seed(0)
    shapes = [(288, 96), (96,), (3, 1, 1), (70001,)]
    ps_gpu = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in shapes]
    ps_cpu = [torch.nn.Parameter(p.detach().cpu().clone()) for p in ps_gpu]
    em_gpu = [p.detach().clone() + 0.1 for p in ps_gpu]
    em_cpu = [e.cpu().clone() for e in em_gpu]

    def groups(ps):
        return [{"params": [ps[0], ps[2]]}, {"params": [ps[1], ps[3]], "weight_decay": 0.0}]
    og = DecoupledSGDW(groups(ps_gpu), lr=0.05, momentum=0.9, weight_decay=5e-4)
    oc = DecoupledSGDW(groups(ps_cpu), lr=0.05, momentum=0.9, weight_decay=5e-4)
    for step in range(2):
        for pg, pc in zip(ps_gpu, ps_cpu):
            g = torch.randn(pg.shape) * 3
            pg.grad, pc.grad = g.cuda(), g.clone()
        for o, ps, es in ((og, ps_gpu, em_gpu), (oc, ps_cpu, em_cpu)):
            o.pending_clip = 2.0
            o.pending_grad_scale = gscale
            if ema:
                o.pending_ema = ([(id(p), e) for p, e in zip(ps, es)], 0.8)
        assert og._fused_eligible()
        og.step()
        oc.step()
        for pg, pc in zip(ps_gpu, ps_cpu):
            assert torch.allclose(pg.detach().cpu(), pc.detach(), rtol=1e-5, atol=1e-6), step
        for eg, ec in zip(em_gpu, em_cpu):
            assert torch.allclose(eg.cpu(), ec, rtol=1e-5, atol=1e-6), step
    assert og.pending_grad_scale == 1.0 and og.pending_ema is None and og.pending_clip is None


@pytest.mark.parametrize("C", [96, 768])
def test_attn_biases_match_torch(C):
    """hvk_attn_bias_fwd/bwd: (q_bias, 0, 0) and proj.bias + W v_bias with their gradients
    against the torch ops they replace (swinv2.py:218-220, 262 folding)."""
    from hvamd import ops
    torch.manual_seed(C)
    qb = torch.randn(C, device="cuda", requires_grad=True)
    vb = torch.randn(C, device="cuda", requires_grad=True)
    pb = torch.randn(C, device="cuda", requires_grad=True)
    w = torch.randn(C, C, device="cuda", requires_grad=True)
    qkv_b, eff = ops.attn_biases(qb, vb, pb, w)
    g = torch.randn(C, device="cuda")
    eff.backward(g)
    ref_eff = pb.detach() + w.detach() @ vb.detach()
    assert torch.equal(qkv_b[:C], qb.detach()) and not qkv_b[C:].any()
    assert torch.allclose(eff, ref_eff, rtol=1e-5, atol=1e-4)
    assert torch.allclose(vb.grad, w.detach().t() @ g, rtol=1e-5, atol=1e-4)
    assert torch.equal(pb.grad, g)
    assert torch.allclose(w.grad, torch.outer(g, vb.detach()), rtol=1e-6, atol=1e-6)
    assert qb.grad is None


@pytest.mark.parametrize("M", [802816, 1000, 37])
@pytest.mark.parametrize("with_b2", [False, True])
def test_fused_mlp_forward_bit_identical(M, with_b2):
    """hvk_mlp_fwd (stage-0 MLP forward in one kernel) == hvk_linear_gelu_fwd + hvk_linear_fwd on
    the same operands, bit for bit (h, GELU(h) and y), ragged M included; and y within 1e-2 of
    fp32 math on the same bf16 operands."""
    from hvamd import _lib
    lib = _lib.load()
    K, N1, N2 = 96, 384, 96
    assert lib.hvk_mlp_fwd_supported(M, K, N1, N2)
    gen = torch.Generator(device="cuda").manual_seed(M + int(with_b2))
    x = torch.randn(M, K, device="cuda", generator=gen).bfloat16()
    w1 = (torch.randn(N1, K, device="cuda", generator=gen) / K ** 0.5).bfloat16()
    b1 = torch.randn(N1, device="cuda", generator=gen) * 0.1
    w2 = (torch.randn(N2, N1, device="cuda", generator=gen) / N1 ** 0.5).bfloat16()
    b2 = torch.randn(N2, device="cuda", generator=gen) * 0.1 if with_b2 else None
    P = _lib.ptr
    h0, g0 = (torch.empty(M, N1, device="cuda", dtype=torch.bfloat16) for _ in range(2))
    y0 = torch.empty(M, N2, device="cuda", dtype=torch.bfloat16)
    _lib.call("hvk_linear_gelu_fwd", P(x), P(w1), P(b1), P(h0), P(g0), M, K, N1, _lib.stream())
    _lib.call("hvk_linear_fwd", P(g0), P(w2), P(b2), P(y0), M, N1, N2, _lib.stream())
    h1, g1 = (torch.full((M, N1), float("nan"), device="cuda", dtype=torch.bfloat16) for _ in range(2))
    y1 = torch.full((M, N2), float("nan"), device="cuda", dtype=torch.bfloat16)
    _lib.call("hvk_mlp_fwd", P(x), P(w1), P(b1), P(w2), P(b2), P(h1), P(g1), P(y1), M, K, N1, N2, _lib.stream())
    torch.cuda.synchronize()
    for a, b in ((h0, h1), (g0, g1), (y0, y1)):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    if M <= 1000:
        ref = torch.nn.functional.gelu((x.float() @ w1.float().t() + b1).bfloat16().float()) @ w2.float().t()
        ref = ref + (b2 if with_b2 else 0)
        assert ((y1.float() - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.parametrize("M", [802816, 1000, 37])
def test_fused_mlp_input_gradients_bit_identical(M):
    """hvk_mlp_bwd (stage-0 gh = (gy w2t^T) * GELU'(h) and gx = gh w1t^T in one kernel) ==
    hvk_linear_gelu_bwd + hvk_linear_fwd on the same operands, bit for bit (gh and gx), ragged M
    included; and gx within 1e-2 of fp32 autograd on the same bf16 operands."""
    from hvamd import _lib
    lib = _lib.load()
    K, N1 = 96, 384
    assert lib.hvk_mlp_bwd_supported(M, K, N1, K)
    gen = torch.Generator(device="cuda").manual_seed(M + 5)
    gy = torch.randn(M, K, device="cuda", generator=gen).bfloat16()
    w2t = (torch.randn(N1, K, device="cuda", generator=gen) / K ** 0.5).bfloat16()
    h = torch.randn(M, N1, device="cuda", generator=gen).bfloat16()
    w1t = (torch.randn(K, N1, device="cuda", generator=gen) / N1 ** 0.5).bfloat16()
    P = _lib.ptr
    gh0 = torch.empty(M, N1, device="cuda", dtype=torch.bfloat16)
    gx0 = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    _lib.call("hvk_linear_gelu_bwd", P(gy), P(w2t), P(h), P(gh0), None, M, K, N1, _lib.stream())
    _lib.call("hvk_linear_fwd", P(gh0), P(w1t), None, P(gx0), M, N1, K, _lib.stream())
    gh1 = torch.full((M, N1), float("nan"), device="cuda", dtype=torch.bfloat16)
    gx1 = torch.full((M, K), float("nan"), device="cuda", dtype=torch.bfloat16)
    _lib.call("hvk_mlp_bwd", P(gy), P(w2t), P(h), P(w1t), P(gh1), P(gx1), M, K, N1, K, _lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(gh0.view(torch.int16), gh1.view(torch.int16))
    assert torch.equal(gx0.view(torch.int16), gx1.view(torch.int16))
    if M <= 1000:
        hf = h.float().requires_grad_(True)
        torch.nn.functional.gelu(hf).backward(gy.float() @ w2t.float().t())
        ref = hf.grad @ w1t.float().t()
        assert ((gx1.float() - ref).norm() / ref.norm()).item() < 1e-2
