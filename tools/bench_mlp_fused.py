"""Stage-0 fused MLP kernels (hvk_mlp_fwd: fc1 + GELU + fc2; hvk_mlp_bwd: fc2 input grad x GELU'
+ fc1 input grad) at the SwinV2-T bs256 shape, one libhvk build per run (--lib), for A/B.
    python tools/bench_mlp_fused.py [--lib abl/x.so] [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from hvamd import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    P, st = _lib.ptr, _lib.stream
    M, K, N1, N2 = 802816, 96, 384, 96
    x = torch.randn(M, K, device="cuda").bfloat16()
    w1 = (torch.randn(N1, K, device="cuda") / K ** 0.5).bfloat16()
    b1 = torch.randn(N1, device="cuda")
    w2 = (torch.randn(N2, N1, device="cuda") / N1 ** 0.5).bfloat16()
    b2 = torch.randn(N2, device="cuda")
    h = torch.empty(M, N1, device="cuda", dtype=torch.bfloat16)
    gh = torch.empty_like(h)
    y = torch.empty(M, N2, device="cuda", dtype=torch.bfloat16)
    gy = torch.randn(M, N2, device="cuda").bfloat16()
    w2t = w2.t().contiguous()
    w1t = w1.t().contiguous()
    gx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    ghb = torch.empty_like(h)

    def fwd():
        _lib.call("hvk_mlp_fwd", P(x), P(w1), P(b1), P(w2), P(b2), P(h), P(gh), P(y), M, K, N1, N2, st())

    def bwd():
        _lib.call("hvk_mlp_bwd", P(gy), P(w2t), P(h), P(w1t), P(ghb), P(gx), M, N2, N1, K, st())

    for name, fn, nbytes in (("mlp_fwd", fwd, M * (K + 2 * N1 + N2) * 2), ("mlp_bwd", bwd, M * (N2 + 2 * N1 + K) * 2)):
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1000
        print(f"{name}  {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s")


if __name__ == "__main__":
    main()
