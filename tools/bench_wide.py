"""A/B of the 208 x 384 whole-row GEMM tile (libhvk option gemm_wide) against the 128-row tile
kernel on the SwinV2-T bs256 stage-2 (and stage-3) products, interleaved in one process, with each
shape's binding roof max(flops / 2.5 PF, algorithmic bytes / 8 TB/s).

    python tools/bench_wide.py [--iters 20 --reps 5]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name, M, K, N, epilogue (0 plain, 1 fc1 + GELU, 2 fc2 input grad through GELU', 4 qkv)
SHAPES = [("s2.qkv", 50176, 384, 1152, 4), ("s2.proj", 50176, 384, 384, 0), ("s2.fc1", 50176, 384, 1536, 1),
          ("s2.fc2.dx", 50176, 384, 1536, 2),
          ("s2.fc2", 50176, 1536, 384, 0), ("s2.proj.dx", 50176, 384, 384, 0), ("s2.qkv.dx", 50176, 1152, 384, 0),
          ("s2.fc1.dx", 50176, 1536, 384, 0), ("s1.merge", 50176, 768, 384, 0), ("s1.merge.dx", 50176, 384, 768, 0),
          ("s3.fc2", 12544, 3072, 768, 0), ("s3.qkv", 12544, 768, 2304, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    from hvamd import _lib
    lib = _lib.load()
    print(f"{'gemm':12s} {'M':>6s} {'K':>5s} {'N':>5s} epi | roof us | tile us  frac | wide us  frac | speedup")
    tot = [0.0, 0.0]
    for name, M, K, N, epi in SHAPES:
        if a.only and a.only not in name:
            continue
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y2 = torch.empty_like(y)
        rn = torch.empty(M, max(1, 2 * N // 96), device="cuda")
        sc = torch.rand(max(1, N // 96), device="cuda") + 1

        def run():
            if epi == 4:
                _lib.call("hvk_gemm_qkv_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), _lib.ptr(rn),
                          _lib.ptr(sc), M, K, N, _lib.stream())
            elif epi == 2:
                _lib.call("hvk_gemm_gelu_bwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(y2), _lib.ptr(y), M, K, N,
                          _lib.stream())
            elif epi == 1:
                _lib.call("hvk_gemm_gelu_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), _lib.ptr(y2), M, K,
                          N, _lib.stream())
            else:
                _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), None, _lib.ptr(y), M, K, N, _lib.stream())

        times = {0: [], 1: []}
        for _ in range(a.reps):
            for mode in (0, 1):
                with _lib.option("gemm_wide", mode):
                    run()
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.iters):
                        run()
                    e.record()
                    torch.cuda.synchronize()
                    times[mode].append(1000 * s.elapsed_time(e) / a.iters)
        t0, t1 = statistics.median(times[0]), statistics.median(times[1])
        byt = 2.0 * (M * K + N * K + M * N) + (2.0 * M * N if epi in (1, 2) else 0) + (8.0 * M * N / 96 if epi == 4 else 0)
        roof = max(2.0 * M * N * K / 2.5e15, byt / 8e12) * 1e6
        tot[0] += t0
        tot[1] += t1
        print(f"{name:12s} {M:6d} {K:5d} {N:5d} {epi:3d} | {roof:7.1f} | {t0:7.1f} {roof / t0:5.3f} | {t1:7.1f} "
              f"{roof / t1:5.3f} | {t0 / t1:5.2f}x", flush=True)
        del x, w, y, y2, rn
    print(f"sum: tile {tot[0]:.1f} us, wide {tot[1]:.1f} us")


if __name__ == "__main__":
    main()
