"""The 208 x 384 whole-row GEMM tile (csrc/gemm_wide.hip, libhvk option gemm_wide) against the
128-row tile kernel it replaces on the stage-2 shapes: same k order (32-deep MFMA steps), same
bias add and rounding, same GELU / head normalisation of the rounded values -> bit-identical
outputs (and rn), nothing written past M; and within 1e-2 of an fp32 matmul."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.view(torch.int16)


def _case(M, K, N, seed, bias=True):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    return x, w, b


def _run(fn, mode, *args):
    from hvamd import _lib
    with _lib.option("gemm_wide", mode):
        _lib.call(fn, *args)
        torch.cuda.synchronize()


@pytest.mark.parametrize("M,K,N,bias", [(50176, 384, 384, False), (50176, 1536, 384, False), (50176, 1152, 384, True),
                                        (50171, 384, 768, True), (50176, 768, 384, False), (1700, 384, 384, True),
                                        (12544, 3072, 768, False)])
def test_wide_plain_bit_identical(M, K, N, bias):
    from hvamd import _lib
    assert _lib.load().hvk_gemm_supported(M, K, N)
    x, w, b = _case(M, K, N, M + K + N, bias)
    out = []
    for mode in (0, 1):
        y = torch.full((M + 8, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        _run("hvk_gemm_fwd", mode, _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), M, K, N, _lib.stream())
        out.append(y)
    assert torch.isnan(out[1][M:].float()).all()  # nothing written past M
    assert torch.equal(_bits(out[0][:M]), _bits(out[1][:M]))
    ref = x.float() @ w.float().t() + (b if bias else 0)
    rel = ((out[1][:M].float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("M,K,N", [(50176, 384, 1536), (50170, 384, 1536), (50176, 384, 768)])
def test_wide_gelu_bit_identical(M, K, N):
    """fc1 + bias + GELU (EPI 1): h and GELU(h) both bit-identical."""
    from hvamd import _lib
    x, w, b = _case(M, K, N, 7 * M + N)
    out = []
    for mode in (0, 1):
        h = torch.full((M + 8, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        y = torch.full((M + 8, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        _run("hvk_gemm_gelu_fwd", mode, _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(h), _lib.ptr(y), M, K, N,
             _lib.stream())
        out.append((h, y))
    for i in range(2):
        assert torch.isnan(out[1][i][M:].float()).all()
        assert torch.equal(_bits(out[0][i][:M]), _bits(out[1][i][:M])), i
    ref = torch.nn.functional.gelu(x.float() @ w.float().t() + b)
    rel = ((out[1][1][:M].float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("M,K,N", [(50176, 384, 1536), (50171, 384, 1536), (12544, 768, 3072)])
def test_wide_gelu_bwd_bit_identical(M, K, N):
    """fc2's input gradient through GELU' (EPI 2, hvk_gemm_gelu_bwd): gh = bf16((gy W) GELU'(h))
    with h read in the accumulator layout, bit-identical to the 128-row kernel."""
    from hvamd import _lib
    gy, w, _ = _case(M, K, N, M + 5 * N, bias=False)
    h = torch.randn(M, N, device="cuda").bfloat16()
    out = []
    for mode in (0, 1):
        gh = torch.full((M + 8, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        _run("hvk_gemm_gelu_bwd", mode, _lib.ptr(gy), _lib.ptr(w), _lib.ptr(h), _lib.ptr(gh), M, K, N, _lib.stream())
        out.append(gh)
    assert torch.isnan(out[1][M:].float()).all()
    assert torch.equal(_bits(out[0][:M]), _bits(out[1][:M]))
    hf = h.float()
    dg = 0.5 * (1 + torch.erf(hf / 2 ** 0.5)) + hf * torch.exp(-0.5 * hf * hf) / (2 * torch.pi) ** 0.5
    ref = (gy.float() @ w.float().t()) * dg
    rel = ((out[1][:M].float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("M,K,N", [(50176, 384, 1152), (49999, 384, 1152), (50176, 512, 1536)])
def test_wide_qkv_epilogue_bit_identical(M, K, N):
    """The qkv epilogue (EPI 4): q / k head slices normalised on the rounded values (the head's
    four 8-column chunks summed in a lane quad, in the 128-row kernel's order), q times the logit
    scale * log2e, rn = 1 / ||x|| per token and q / k head: all bit-identical."""
    from hvamd import _lib
    x, w, b = _case(M, K, N, M + 11 * K)
    b[N // 3:] = 0  # (q_bias, 0, 0)
    sc = torch.rand(N // 96, device="cuda") * 20 + 1
    out = []
    for mode in (0, 1):
        y = torch.full((M + 8, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        rn = torch.full((M + 8, 2 * N // 96), float("nan"), device="cuda")
        _run("hvk_gemm_qkv_fwd", mode, _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), _lib.ptr(rn), _lib.ptr(sc),
             M, K, N, _lib.stream())
        out.append((y, rn))
    assert torch.isnan(out[1][0][M:].float()).all() and torch.isnan(out[1][1][M:]).all()
    assert torch.equal(_bits(out[0][0][:M]), _bits(out[1][0][:M]))
    assert torch.equal(out[0][1][:M].view(torch.int32), out[1][1][:M].view(torch.int32))
    # against fp32: the normalised q (times scale * log2e), k and plain v slices
    ref = x.float() @ w.float().t() + b
    C = N // 3
    q, k, v = ref[:, :C], ref[:, C:2 * C], ref[:, 2 * C:]
    qn = torch.nn.functional.normalize(q.view(M, -1, 32), dim=-1) * (sc * 1.4426950408889634)[None, :, None]
    kn = torch.nn.functional.normalize(k.view(M, -1, 32), dim=-1)
    got = out[1][0][:M].float()
    for a, r in ((got[:, :C], qn.reshape(M, C)), (got[:, C:2 * C], kn.reshape(M, C)), (got[:, 2 * C:], v)):
        rel = ((a - r).norm() / r.norm()).item()
        assert rel < 1e-2, rel
