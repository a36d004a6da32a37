"""Run one GEMM shape a few times (for PMC passes): python tools/gemm_one.py dw|fwd M N K [iters]
dw: hvk_weight_grad (dW[N, K] = g[M, N]^T x[M, K]); fwd: hvk_gemm_fwd (Y[M, N] = X[M, K] W[N, K]^T)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    kind, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    from hvamd import _lib
    lib = _lib.load()
    P = _lib.ptr
    if kind == "dw":
        g = torch.randn(M, N, device="cuda").bfloat16()
        x = torch.randn(M, K, device="cuda").bfloat16()
        dw = torch.empty(N, K, device="cuda")
        ws = torch.empty(lib.hvk_weight_grad_workspace(M, N, K), device="cuda", dtype=torch.uint8)
        for _ in range(iters):
            _lib.call("hvk_weight_grad", P(g), P(x), P(dw), None, M, N, K, P(ws), ws.numel(), _lib.stream())
    else:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(iters):
            _lib.call("hvk_gemm_fwd", P(x), P(w), None, P(y), M, K, N, _lib.stream())
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
