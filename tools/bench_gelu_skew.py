"""Does the relative placement of the two fc1 outputs (h, GELU(h)) matter?  hvk_linear_gelu_fwd
with GELU(h) written at byte offsets from a fresh allocation:  python tools/bench_gelu_skew.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_skinny import timeit  # noqa: E402


def main():
    from hvamd import _lib
    P, st = _lib.ptr, _lib.stream
    for M, C in [(802816, 96), (200704, 192)]:
        N = 4 * C
        x = torch.randn(M, C, device="cuda").bfloat16()
        w1 = (torch.randn(N, C, device="cuda") / C ** 0.5).bfloat16()
        b1 = torch.randn(N, device="cuda")
        h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        big = torch.empty(M * N + (1 << 20), device="cuda", dtype=torch.bfloat16)
        res = []
        for off in (0, 128, 1024, 4096, 65536, 1 << 19):
            y = big[off // 2: off // 2 + M * N].view(M, N)
            res.append((off, timeit(lambda: _lib.call("hvk_linear_gelu_fwd", P(x), P(w1), P(b1), P(h), P(y), M,
                                                      C, N, st()))))
        print(f"M={M} C={C}: " + "  ".join(f"+{o}B {t:.1f}us" for o, t in res), flush=True)
        gy = torch.randn(M, C, device="cuda").bfloat16()
        w2t = (torch.randn(N, C, device="cuda") / N ** 0.5).bfloat16()
        res = []
        for off in (0, 128, 1024, 4096, 65536, 1 << 19):
            gh = big[off // 2: off // 2 + M * N].view(M, N)
            res.append((off, timeit(lambda: _lib.call("hvk_linear_gelu_bwd", P(gy), P(w2t), P(h), P(gh), None, M,
                                                      C, N, st()))))
        print(f"   bwd: " + "  ".join(f"+{o}B {t:.1f}us" for o, t in res), flush=True)
        del x, h, big


if __name__ == "__main__":
    main()
