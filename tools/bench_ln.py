"""LayerNorm kernels (hvk_ln_residual_fwd / _bwd) at the SwinV2-T bs256 stage shapes: time per
launch (dispatch-packet timer) and rate against 8 TB/s for the 12 / 14 bytes per element they
move (forward: a bf16 + x0 f32 in, x f32 + xb bf16 out; backward: a bf16, gx f32, gxb bf16 in,
gx0 f32, ga bf16 out).

    python tools/bench_ln.py [--lib abl/x.so] [--iters 20]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STAGES = [("stage0", 256 * 3136, 96), ("stage1", 256 * 784, 192), ("stage2", 256 * 196, 384), ("stage3", 256 * 49, 768)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from hvamd import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    lib = _lib.load()
    P, st = _lib.ptr, _lib.stream
    for name, T, C in STAGES:
        g = torch.Generator(device="cuda").manual_seed(C)
        av = torch.randn(T, C, device="cuda", generator=g).bfloat16()
        x0 = torch.randn(T, C, device="cuda", generator=g)
        gm, bt = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
        x, xb = torch.empty_like(x0), torch.empty_like(av)
        mean, rstd = torch.empty(T, device="cuda"), torch.empty(T, device="cuda")
        gx, gxb = torch.randn_like(x0), torch.randn(T, C, device="cuda").bfloat16()
        gx0, ga = torch.empty_like(x0), torch.empty_like(av)
        dg, db, dab = (torch.empty(C, device="cuda") for _ in range(3))
        nb = lib.hvk_ln_bwd_workspace_bytes(C)
        ws = torch.empty(nb // 4, device="cuda")

        def fwd():
            _lib.call("hvk_ln_residual_fwd", P(av), None, P(x0), P(gm), P(bt), None, T, C, T, 1e-5, P(x), P(xb),
                      P(mean), P(rstd), st())

        def bwd():
            _lib.call("hvk_ln_residual_bwd", P(av), None, P(gm), None, P(mean), P(rstd), P(gx), P(gxb), T, C, T,
                      P(gx0), P(ga), P(dg), P(db), P(dab), P(ws), nb, st())

        res = []
        for fn, nbytes in ((fwd, 12 * T * C), (bwd, 14 * T * C)):
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / a.iters * 1e3
            res.append(f"{us:7.1f} us {nbytes / us / 1e6:5.2f} TB/s {nbytes / us / 8e6:.3f}")
        print(f"{name} C={C:4d}  fwd {res[0]}  | bwd {res[1]}", flush=True)


if __name__ == "__main__":
    main()
