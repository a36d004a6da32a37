"""libhvk weight-gradient GEMM (hvk_weight_grad): dW = g^T x and db = sum_m g against an
fp32 matmul of the same bf16 operands (the F.linear backward, swinv2.py:58-62, 220, 262)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (N, K) of every SwinV2-T Linear whose weight gradient runs on the kernel, at token counts
# that keep the fp32 reference cheap (M % 32 == 0; ragged chunk splits included)
CASES = [(288, 96, 32 * 517), (96, 96, 6272), (384, 96, 12544), (96, 384, 12544),
         (576, 192, 3136), (192, 192, 800), (768, 192, 3136), (192, 768, 3136),
         (1152, 384, 1568), (384, 384, 1568), (1536, 384, 1568), (384, 1536, 1568),
         (2304, 768, 12544), (768, 3072, 2048), (192, 384, 6272), (384, 768, 1568), (32 * 6, 192, 32),
         (96, 48, 32 * 999), (128, 48, 32 * 999), (128, 48, 32 * 4608)]


def _ref(g, x):
    return g.float().t() @ x.float(), g.float().sum(0)


@pytest.mark.parametrize("N,K,M", CASES)
@pytest.mark.parametrize("with_db", [True, False])
def test_weight_grad_matches_fp32(N, K, M, with_db):
    from hvamd import _lib
    lib = _lib.load()
    assert lib.hvk_weight_grad_supported(M, N, K)
    gen = torch.Generator(device="cuda").manual_seed(N * 7 + K * 3 + M)
    g = torch.randn(M, N, device="cuda", generator=gen).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=gen).bfloat16()
    dw = torch.full((N, K), float("nan"), device="cuda")
    db = torch.full((N,), float("nan"), device="cuda") if with_db else None
    ws = torch.empty(lib.hvk_weight_grad_workspace(M, N, K), device="cuda", dtype=torch.uint8)
    _lib.call("hvk_weight_grad", _lib.ptr(g), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db) if with_db else None,
              M, N, K, _lib.ptr(ws), ws.numel(), _lib.stream())
    rw, rb = _ref(g, x)
    torch.cuda.synchronize()
    # f32 accumulation of M products in a different order: ~sqrt(M) ulp of the partial sums
    err = (dw - rw).abs().max().item()
    assert err <= 1e-4 * M ** 0.5 * 4, err
    assert torch.isfinite(dw).all()
    if with_db:
        assert (db - rb).abs().max().item() <= 1e-4 * M ** 0.5 * 4


@pytest.mark.parametrize("tile", [4, 5, 6, 7, 8])
@pytest.mark.parametrize("N,K,M", [(1152, 384, 1568), (768, 3072, 2048), (384, 768, 1568)])
def test_weight_grad_tile_variants_match_fp32(tile, N, K, M):
    """Every selectable tile variant of the 192-multiple shapes (library option dw_tile, the
    default is 5) against the fp32 reference; variants that do not fit a shape fall back."""
    from hvamd import _lib
    lib = _lib.load()
    gen = torch.Generator(device="cuda").manual_seed(N + K + M + tile)
    g = torch.randn(M, N, device="cuda", generator=gen).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=gen).bfloat16()
    with _lib.option("dw_tile", tile):
        dw = torch.full((N, K), float("nan"), device="cuda")
        db = torch.full((N,), float("nan"), device="cuda")
        ws = torch.empty(lib.hvk_weight_grad_workspace(M, N, K), device="cuda", dtype=torch.uint8)
        _lib.call("hvk_weight_grad", _lib.ptr(g), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db), M, N, K,
                  _lib.ptr(ws), ws.numel(), _lib.stream())
        torch.cuda.synchronize()
    rw, rb = _ref(g, x)
    assert (dw - rw).abs().max().item() <= 1e-4 * M ** 0.5 * 4
    assert (db - rb).abs().max().item() <= 1e-4 * M ** 0.5 * 4


def test_weight_grad_sparse_pattern_pins_layout():
    """One nonzero token row per operand: dW must be the outer product at exactly the right
    (n, k) and db the g row -- catches transposed or permuted output layouts."""
    from hvamd import _lib
    lib = _lib.load()
    M, N, K = 3136, 576, 192
    g = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    t = 1777
    g[t] = torch.arange(N, device="cuda").bfloat16() % 7 - 3
    x[t] = torch.arange(K, device="cuda").bfloat16() % 5 + 1
    dw = torch.empty(N, K, device="cuda")
    db = torch.empty(N, device="cuda")
    ws = torch.empty(lib.hvk_weight_grad_workspace(M, N, K), device="cuda", dtype=torch.uint8)
    _lib.call("hvk_weight_grad", _lib.ptr(g), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db), M, N, K,
              _lib.ptr(ws), ws.numel(), _lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(dw, torch.outer(g[t].float(), x[t].float()))
    assert torch.equal(db, g[t].float())


def test_linear_backward_uses_weight_grad_kernel():
    from hvamd import ops
    torch.manual_seed(0)
    x = torch.randn(8, 784, 192, device="cuda").bfloat16().requires_grad_(True)
    w = torch.randn(576, 192, device="cuda", requires_grad=True)
    b = torch.randn(576, device="cuda", requires_grad=True)
    y = ops.linear(x, w, b)
    gy = torch.randn_like(y)
    y.backward(gy)
    g2 = gy.reshape(-1, 576)
    rw = g2.float().t() @ x.detach().reshape(-1, 192).float()
    assert ((w.grad - rw).norm() / rw.norm()).item() < 1e-5
    assert ((b.grad - g2.float().sum(0)).norm() / b.grad.norm()).item() < 1e-5


@pytest.mark.parametrize("N,K,M", [(96, 96, 6272), (384, 384, 1568), (768, 768, 2048), (192, 192, 800)])
@pytest.mark.parametrize("with_db", [True, False])
def test_weight_grad_shift_matches_fp32(N, K, M, with_db):
    """hvk_weight_grad_shift: dW = g^T (x + 1 xshift^T) (the proj Linear with v_bias folded into its
    bias), db = sum g, against fp32 of the same bf16 operands; bit-identical db to the plain
    kernel's."""
    from hvamd import _lib
    lib = _lib.load()
    gen = torch.Generator(device="cuda").manual_seed(N + K + M)
    g = torch.randn(M, N, device="cuda", generator=gen).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=gen).bfloat16()
    xs = torch.randn(K, device="cuda", generator=gen)
    dw = torch.full((N, K), float("nan"), device="cuda")
    db = torch.full((N,), float("nan"), device="cuda") if with_db else None
    ws = torch.empty(lib.hvk_weight_grad_workspace(M, N, K), device="cuda", dtype=torch.uint8)
    _lib.call("hvk_weight_grad_shift", _lib.ptr(g), _lib.ptr(x), _lib.ptr(xs), _lib.ptr(dw),
              _lib.ptr(db) if with_db else None, M, N, K, _lib.ptr(ws), ws.numel(), _lib.stream())
    torch.cuda.synchronize()
    rw = g.float().t() @ (x.float() + xs[None, :])
    err = (dw - rw).abs().max().item()
    assert err <= 1e-4 * M ** 0.5 * 4 * (1 + xs.abs().max().item()), err
    if with_db:
        assert (db - g.float().sum(0)).abs().max().item() <= 1e-4 * M ** 0.5 * 4
