"""A/B of the tiled GEMM kernels per SwinV2 stage shape (hvk_gemm_set_pp modes, interleaved
rounds in one process): 0 = 128-row tiles at two workgroups per CU, 2 = ping-pong 256 x 256,
3 = ping-pong 128 x 384.  Prints us per launch (median over rounds) and TFLOP/s.

    python tools/bench_pp.py [--model t|b224|b384] [--rounds 5] [--iters 10]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gemm import MODELS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="t", choices=sorted(MODELS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from hvamd import _lib
    lib = _lib.load()
    shapes = []
    for s, (T, C, nb) in enumerate(MODELS[a.model]):
        if s == 0:
            continue
        for name, K, N in (("qkv", C, 3 * C), ("proj", C, C), ("fc1", C, 4 * C), ("fc2", 4 * C, C)):
            shapes.append((f"s{s}.{name}", T, K, N, "gelu" if name == "fc1" else "plain"))
            shapes.append((f"s{s}.{name}.dx", T, N, K, "gelu_bwd" if name == "fc2" else "plain"))
    tot = {0: 0.0, 1: 0.0}
    print(f"{'shape':12s} {'M':>7s} {'K':>5s} {'N':>5s} | mode0 us | pp us (mode) | TF/s 0 -> pp", flush=True)
    for name, M, K, N, epi in shapes:
        if K % 64 or not lib.hvk_gemm_supported(M, K, N):
            continue
        modes = [0] + ([2] if N % 256 == 0 else []) + ([3] if N % 384 == 0 else [])
        if len(modes) == 1:
            continue
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y2 = torch.empty_like(y)

        def run():
            if epi == "plain":
                _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), M, K, N, _lib.stream())
            elif epi == "gelu":
                _lib.call("hvk_gemm_gelu_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), _lib.ptr(y2),
                          M, K, N, _lib.stream())
            else:
                _lib.call("hvk_gemm_gelu_bwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(y2), _lib.ptr(y), M, K, N,
                          _lib.stream())
        t = {m: [] for m in modes}
        for _ in range(a.rounds):
            for m in modes:
                lib.hvk_gemm_set_pp(m)
                run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                t[m].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        med = {m: statistics.median(v) for m, v in t.items()}
        best = min((m for m in modes if m), key=lambda m: med[m])
        fl = 2.0 * M * N * K
        print(f"{name:12s} {M:7d} {K:5d} {N:5d} | {med[0]:8.1f} | {med[best]:8.1f} ({best}) "
              + " ".join(f"m{m}={med[m]:.1f}" for m in modes if m) +
              f" | {fl / med[0] / 1e6:6.0f} -> {fl / med[best] / 1e6:6.0f}", flush=True)
        tot[0] += med[0]
        tot[1] += med[best]
        del x, w, y, y2
    lib.hvk_gemm_set_pp(1)
    print(f"sum of launches: mode0 {tot[0]:.1f} us, best pp {tot[1]:.1f} us")


if __name__ == "__main__":
    main()
