"""Weight-gradient GEMM (dW = g^T x, f32 out) on the SwinV2-T bs256 shapes: split-token
batched GEMM with nc chunks + sum, for several nc.   python tools/bench_dw.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (name, M, N, K): dW [N, K] = g[M, N]^T x[M, K]
    ("s0.qkv", 802816, 288, 96), ("s0.proj", 802816, 96, 96), ("s0.fc1", 802816, 384, 96),
    ("s0.fc2", 802816, 96, 384), ("s1.qkv", 200704, 576, 192), ("s1.fc1", 200704, 768, 192),
    ("s1.fc2", 200704, 192, 768), ("s2.qkv", 50176, 1152, 384), ("s2.fc1", 50176, 1536, 384),
    ("s2.fc2", 50176, 384, 1536), ("s3.fc1", 12544, 3072, 768),
    ("s1.proj", 200704, 192, 192), ("s2.proj", 50176, 384, 384), ("s3.qkv", 12544, 2304, 768),
    ("s3.fc2", 12544, 768, 3072), ("s3.proj", 12544, 768, 768), ("merge1", 200704, 192, 384),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000


def main():
    only = set(sys.argv[1:])  # e.g. python tools/bench_dw.py s2.qkv
    for name, M, N, K in SHAPES:
        if only and name not in only:
            continue
        g = torch.randn(M, N, device="cuda").bfloat16()
        x = torch.randn(M, K, device="cuda").bfloat16()
        line = [f"{name:8s} M={M:6d} N={N:4d} K={K:4d} bytes-bound {(M * (N + K) * 2) / 5e12 * 1e6:6.1f} us |"]
        for nc in ((1, 16, 64, 128) if os.environ.get("DW_ALL") else (64,)):
            if M % nc or M // nc < 64:
                continue
            kc = M // nc

            def f():
                if nc == 1:
                    return torch.mm(g.t(), x, out_dtype=torch.float32)
                return torch.bmm(g.view(nc, kc, N).transpose(1, 2), x.view(nc, kc, K),
                                 out_dtype=torch.float32).sum(dim=0)
            line.append(f"nc{nc} {timeit(f):6.1f}")
        from hvamd import ops
        if ops._lib.load().hvk_weight_grad_supported(M, N, K):
            line.append(f"| hvk {timeit(lambda: ops.weight_grad(g, x, False)):6.1f}"
                        f" +db {timeit(lambda: ops.weight_grad(g, x, True)):6.1f}")
            dw, _ = ops.weight_grad(g, x)
            ref = torch.mm(g.t(), x, out_dtype=torch.float32)
            line.append(f"err {((dw - ref).norm() / ref.norm()).item():.1e}")
        print(" ".join(line), flush=True)
        del g, x


if __name__ == "__main__":
    main()
