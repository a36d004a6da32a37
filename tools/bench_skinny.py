"""hvk_linear_fwd (weight-stationary MFMA GEMM) vs the library GEMM on given shapes.
    HVK_LINEAR_VARIANT=v python tools/bench_skinny.py M:K:N [M:K:N ...]
Prints per shape: libhvk us, library us, and the HBM / MFMA floors."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    from hvamd import _lib
    lib = _lib.load()
    v = os.environ.get("HVK_LINEAR_VARIANT", "0")
    for spec in sys.argv[1:]:
        M, K, N = map(int, spec.split(":"))
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ok = lib.hvk_linear_supported(M, K, N)
        t_h = float("nan")
        if ok:
            t_h = timeit(lambda: _lib.call("hvk_linear_fwd", _lib.ptr(x), _lib.ptr(w), None, _lib.ptr(y),
                                           M, K, N, _lib.stream()))
            ref = x.float() @ w.float().t()
            err = ((y.float() - ref).norm() / ref.norm()).item()
        else:
            err = float("nan")
        t_t = float("nan")
        if lib.hvk_gemm_supported(M, K, N):
            y2 = torch.empty_like(y)
            t_t = timeit(lambda: _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), None, _lib.ptr(y2),
                                           M, K, N, _lib.stream()))
            ref = x.float() @ w.float().t()
            err2 = ((y2.float() - ref).norm() / ref.norm()).item()
        else:
            err2 = float("nan")
        t_l = timeit(lambda: torch.nn.functional.linear(x, w))
        hbm = (M * K + M * N + N * K) * 2 / 5.5e12 * 1e6
        mf = 2 * M * K * N / 2.5e15 * 1e6
        print(f"v{v} M={M} K={K} N={N}: hvk {t_h:7.1f} us (rel err {err:.1e})  tile {t_t:7.1f} us "
              f"(rel err {err2:.1e})  lib {t_l:7.1f} us  "
              f"floors hbm {hbm:5.1f} mfma {mf:5.1f}", flush=True)


if __name__ == "__main__":
    main()
