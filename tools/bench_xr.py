"""A/B of the tiled GEMM kernels on the SwinV2-T bs256 stage-2/3 shapes: gemm_nt_kernel
(128 x 128 / 128 x 192 tiles, two workgroups per CU) against the persistent row-range kernel
(gemm_xr.hip, library option gemm_xr = 1), interleaved rounds in one process, outputs compared
bit for bit.

    python tools/bench_xr.py [--rounds 5] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MFMA = 2.5e15
SHAPES = [  # name, M, K, N, epi (0 plain + bias, 1 bias + GELU, 2 input gradient through GELU')
    ("s2.qkv", 50176, 384, 1152, 0), ("s2.proj", 50176, 384, 384, 0), ("s2.fc1", 50176, 384, 1536, 1),
    ("s2.fc2", 50176, 1536, 384, 0), ("s2.qkv_dx", 50176, 1152, 384, 0),
    ("s3.qkv", 12544, 768, 2304, 0), ("s3.proj", 12544, 768, 768, 0), ("s3.fc1", 12544, 768, 3072, 1),
    ("s3.fc2", 12544, 3072, 768, 0), ("s3.qkv_dx", 12544, 2304, 768, 0),
    ("s2.fc2_dx", 50176, 384, 1536, 2), ("s3.fc2_dx", 12544, 768, 3072, 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    from hvamd import _lib
    import re
    lib = _lib.load()
    P = _lib.ptr
    modes = (0, 1, 2)
    print(f"{'gemm':10s} {'M':>6s} {'K':>5s} {'N':>5s}  {'tile us':>8s} {'xr1 us':>8s} {'xr2 us':>8s}  tile/best  {'best TF/s':>9s} frac  bits")
    tot = [0.0, 0.0, 0.0]
    for name, M, K, N, epi in SHAPES:
        if a.only and not re.search(a.only, name):
            continue
        g = torch.Generator(device="cuda").manual_seed(M + K + N)
        x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda", generator=g)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y2 = torch.randn(M, N, device="cuda", generator=g).bfloat16()  # h for epi 2

        def run():
            if epi == 1:
                _lib.call("hvk_gemm_gelu_fwd", P(x), P(w), P(b), P(y), P(y2), M, K, N, _lib.stream())
            elif epi == 2:
                _lib.call("hvk_gemm_gelu_bwd", P(x), P(w), P(y2), P(y), M, K, N, _lib.stream())
            else:
                _lib.call("hvk_gemm_fwd", P(x), P(w), P(b), P(y), M, K, N, _lib.stream())

        outs, times = {}, {m: [] for m in modes}
        for r in range(a.rounds):
            for mode in modes:
                with _lib.option("gemm_xr", mode):
                    run()
                    torch.cuda.synchronize()
                    if r == 0:
                        outs[mode] = (y.clone(), y2.clone())
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.iters):
                        run()
                    e.record()
                    torch.cuda.synchronize()
                    times[mode].append(s.elapsed_time(e) / a.iters * 1e3)
        same = all(torch.equal(outs[0][0].view(torch.int16), outs[m][0].view(torch.int16)) for m in modes)
        if epi == 1:
            same = same and all(torch.equal(outs[0][1].view(torch.int16), outs[m][1].view(torch.int16)) for m in modes)
        med = [sorted(times[m])[len(times[m]) // 2] for m in modes]
        for i in range(3):
            tot[i] += med[i]
        best = min(med[1], med[2])
        tf = 2.0 * M * N * K / (best * 1e-6) / 1e12
        print(f"{name:10s} {M:6d} {K:5d} {N:5d}  {med[0]:8.1f} {med[1]:8.1f} {med[2]:8.1f}  {med[0] / best:8.3f}  {tf:9.0f} {tf * 1e12 / MFMA:.3f}  {'same' if same else 'DIFF'}")
    print(f"{'sum':29s}  {tot[0]:8.1f} {tot[1]:8.1f} {tot[2]:8.1f}")


if __name__ == "__main__":
    main()
