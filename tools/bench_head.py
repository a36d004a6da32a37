"""Classifier-head GEMMs: libhvk's head kernels (hvk_head_fwd / hvk_head_bwd) against the
library GEMMs torch runs for the same products (hipBLASLt: F.linear forward, g @ W, g^T @ x),
bs256 x 768 features x N classes, median of interleaved rounds.

    python tools/bench_head.py [--n 10000] [--m 256] [--k 768]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--k", type=int, default=768)
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from hvamd import _lib
    lib = _lib.load()
    P, st = _lib.ptr, _lib.stream
    M, K, N = a.m, a.k, a.n
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    bb = b.bfloat16()
    g = torch.randn(M, N, device="cuda").bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gx = torch.empty(M, K, device="cuda")
    dw = torch.empty(N, K, device="cuda")
    db = torch.empty(N, device="cuda")
    nb = lib.hvk_head_bwd_workspace_bytes(M, K, N)
    ws = torch.empty(max(nb, 4) // 4, device="cuda")
    cases = {
        "hvk fwd": lambda: _lib.call("hvk_head_fwd", P(x), P(w), P(b), P(y), M, K, N, st()),
        "hvk dgrad": lambda: _lib.call("hvk_head_bwd", P(g), None, P(w), P(gx), None, None, M, K, N, P(ws), nb, st()),
        "hvk wgrad": lambda: _lib.call("hvk_head_bwd", P(g), P(x), None, None, P(dw), P(db), M, K, N, None, 0, st()),
        "torch fwd": lambda: torch.nn.functional.linear(x, w, bb),
        "torch dgrad": lambda: torch.mm(g, w, out_dtype=torch.float32),
        "torch wgrad": lambda: (torch.mm(g.t(), x, out_dtype=torch.float32), g.sum(0, dtype=torch.float32)),
    }
    times = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / a.iters * 1e3)
    for k in cases:
        t = sorted(times[k])[len(times[k]) // 2]
        print(f"{k:12s} {t:8.1f} us  {2 * M * N * K / t / 1e6:7.1f} TFLOP/s")


if __name__ == "__main__":
    main()
