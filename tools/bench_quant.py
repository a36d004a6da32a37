"""Tile-count quantisation probe for the tiled GEMM (hvk_gemm_fwd): time per launch of one
(K, N) product against M, so the tiles-per-slot curve shows whether a shape's time follows its
work (linear in M) or its rounds of co-resident tiles (steps at multiples of the slot count).

    python tools/bench_quant.py [--k 1536 --n 384 --iters 30]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=1536)
    ap.add_argument("--n", type=int, default=384)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--ms", default="16384,24576,32768,36864,40960,45056,49152,50176,53248,57344,65536,98304")
    a = ap.parse_args()
    from hvamd import _lib
    K, N = a.k, a.n
    Ms = [int(m) for m in a.ms.split(",")]
    x = torch.randn(max(Ms), K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    y = torch.empty(max(Ms), N, device="cuda", dtype=torch.bfloat16)
    print(f"K={K} N={N}   M | tiles(128 rows) | us/launch | ns per 128-row tile | TFLOP/s | GB/s")
    for M in Ms:
        fn = lambda: _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), None, _lib.ptr(y), M, K, N, _lib.stream())
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(3):
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / a.iters)
        tiles = (M + 127) // 128
        fl = 2.0 * M * N * K
        by = 2.0 * (M * K + N * K + M * N)
        print(f"{M:7d} | {tiles:5d} | {best:8.1f} | {best * 1e3 / tiles:8.1f} | {fl / best / 1e6:7.1f} | {by / best / 1e3:7.1f}",
              flush=True)


if __name__ == "__main__":
    main()
