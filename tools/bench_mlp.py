"""Fused MLP kernels on the SwinV2-T bs256 stage shapes: hvk_linear_gelu_fwd (fc1 + bias + GELU,
writes h and GELU(h)) and hvk_linear_gelu_bwd (fc2 input grad x GELU'(h) + fc1 bias grad).
    python tools/bench_mlp.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_skinny import timeit  # noqa: E402

STAGES = [(802816, 96), (200704, 192), (50176, 384)]


def main():
    from hvamd import _lib
    P, st = _lib.ptr, _lib.stream
    stages = STAGES
    if len(sys.argv) > 1:  # python tools/bench_mlp.py 0  -> stage 0 only
        stages = [STAGES[int(a)] for a in sys.argv[1:]]
    for M, C in stages:
        N = 4 * C
        x = torch.randn(M, C, device="cuda").bfloat16()
        w1 = (torch.randn(N, C, device="cuda") / C ** 0.5).bfloat16()
        b1 = torch.randn(N, device="cuda")
        h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y = torch.empty_like(h)
        gy = torch.randn(M, C, device="cuda").bfloat16()
        w2t = (torch.randn(N, C, device="cuda") / N ** 0.5).bfloat16()
        gh = torch.empty_like(h)
        db = torch.zeros(N, device="cuda")
        tf = timeit(lambda: _lib.call("hvk_linear_gelu_fwd", P(x), P(w1), P(b1), P(h), P(y), M, C, N, st()))
        tb = timeit(lambda: _lib.call("hvk_linear_gelu_bwd", P(gy), P(w2t), P(h), P(gh), P(db), M, C, N, st()))
        bf = (M * C + 2 * M * N) * 2 / 5.5e12 * 1e6
        print(f"M={M} C={C}: fc1+gelu {tf:7.1f} us (hbm floor {bf:6.1f})  fc2-dx+gelu' {tb:7.1f} us "
              f"(hbm floor {bf:6.1f})", flush=True)
        del x, h, y, gh


if __name__ == "__main__":
    main()
