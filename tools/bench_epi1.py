"""fc1 + bias + GELU on the tiled kernel (hvk_gemm_gelu_fwd, EPI 1) at the SwinV2 stage-2/3 shapes,
for A/B of library builds.

    python tools/bench_epi1.py [--lib abl/x.so] [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("T-s2", 50176, 384, 1536), ("T-s3", 12544, 768, 3072), ("B224-s2", 50176, 512, 2048),
          ("B384-s2", 147456, 512, 2048), ("B384-s3", 36864, 1024, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    from hvamd import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    _lib.load()
    for name, M, K, N in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda")
        h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y = torch.empty_like(h)

        def run():
            _lib.call("hvk_gemm_gelu_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(h), _lib.ptr(y), M, K, N,
                      _lib.stream())
        for _ in range(3):
            run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1e3
        byts = 2 * (M * K + N * K + 2 * M * N)
        print(f"{name:8s} {M:7d} {K:5d} {N:5d} {us:8.1f} us {byts / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
