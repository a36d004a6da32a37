"""Fused MLP kernels, skinny (hvk_linear_gelu_*) vs tiled (hvk_gemm_gelu_*), on the stage shapes
both build:  python tools/bench_mlp_tile.py [tile_wide=0|1 ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_skinny import timeit  # noqa: E402


def main():
    import ctypes
    from hvamd import _lib
    P, st = _lib.ptr, _lib.stream
    lib = _lib.load()
    for o in sys.argv[1:]:  # libhvk options NAME=VALUE (e.g. tile_wide=1)
        k, v = o.split("=")
        assert lib.hvk_set_option(k.encode(), int(v), ctypes.byref(ctypes.c_longlong())) == 0, o
    for M, C in [(200704, 192), (50176, 384), (12544, 768)]:
        N = 4 * C
        x = torch.randn(M, C, device="cuda").bfloat16()
        w1 = (torch.randn(N, C, device="cuda") / C ** 0.5).bfloat16()
        b1 = torch.randn(N, device="cuda")
        h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y = torch.empty_like(h)
        gy = torch.randn(M, C, device="cuda").bfloat16()
        w2t = (torch.randn(N, C, device="cuda") / N ** 0.5).bfloat16()
        gh = torch.empty_like(h)
        r = [f"M={M} C={C}:"]
        if lib.hvk_linear_gelu_supported(M, C, N):
            r.append("skinny fwd %.1f" % timeit(lambda: _lib.call("hvk_linear_gelu_fwd", P(x), P(w1), P(b1), P(h), P(y), M, C, N, st())))
            r.append("bwd %.1f" % timeit(lambda: _lib.call("hvk_linear_gelu_bwd", P(gy), P(w2t), P(h), P(gh), None, M, C, N, st())))
        if lib.hvk_gemm_supported(M, C, N):
            r.append("| tile fwd %.1f" % timeit(lambda: _lib.call("hvk_gemm_gelu_fwd", P(x), P(w1), P(b1), P(h), P(y), M, C, N, st())))
            r.append("bwd %.1f" % timeit(lambda: _lib.call("hvk_gemm_gelu_bwd", P(gy), P(w2t), P(h), P(gh), M, C, N, st())))
        print(" ".join(r), flush=True)
        del x, h, y, gh


if __name__ == "__main__":
    main()
