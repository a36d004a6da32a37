"""Microbenchmark of the W-MSA kernels on the SwinV2-T bs256 stage shapes.

    python tools/bench_wmsa.py [--iters 20]

Prints, per stage, forward and backward time per launch and algorithmic GB/s
(8*T*C forward, 16*T*C backward), on random bf16 inputs."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STAGES = [  # (name, B, H, W, C, heads, window, shift, blocks per step)
    ("stage0-s3", 256, 56, 56, 96, 3, 7, 3, 2),
    ("stage1-s3", 256, 28, 28, 192, 6, 7, 3, 2),
    ("stage2-s3", 256, 14, 14, 384, 12, 7, 3, 6),
    ("stage3", 256, 7, 7, 768, 24, 7, 0, 2),
]
# SwinV2-B 384, windows 24/24/24/12 (pretrained 12/12/12/6), bs256: BASELINE config 5
STAGES_B384 = [
    ("b384-s0-s12", 256, 96, 96, 128, 4, 24, 12, 2),
    ("b384-s1-s12", 256, 48, 48, 256, 8, 24, 12, 2),
    ("b384-s2", 256, 24, 24, 512, 16, 24, 0, 18),
    ("b384-s3", 256, 12, 12, 1024, 32, 12, 0, 2),
]


def timeit(fn, iters, kind):
    """Mean kernel duration (ms) from libhvk's dispatch-packet timer (execution only, as a
    rocprofv3 kernel trace; HIP events around the launch would add the dispatch gap)."""
    import ctypes
    from hvamd import _lib
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    _lib.call("hvk_kernel_timer_enable", 4 * iters)
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    t, n = ctypes.c_double(0.0), ctypes.c_int(0)
    _lib.call("hvk_kernel_timer_read", kind, ctypes.byref(t), ctypes.byref(n))
    _lib.call("hvk_kernel_timer_enable", 0)
    return t.value / max(n.value, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None, help="alternative libhvk build (tools/probe)")
    ap.add_argument("--stage", type=int, default=None, help="only this stage (0-3)")
    ap.add_argument("--only", choices=["fwd", "bwd"], default=None)
    ap.add_argument("--recompute", action="store_true",
                    help="large windows: backward recomputes the row statistics (no forward row constants)")
    ap.add_argument("--b384", action="store_true", help="SwinV2-B 384 w24 stage shapes (config 5)")
    ap.add_argument("--normed", action="store_true",
                    help="windows <= 8: q / k normalised upstream (hvk_wmsa_fwd_normed / _bwd_normed, the model's path)")
    args = ap.parse_args()
    from hvamd import _lib
    if args.lib:
        _lib.LIB_PATH = os.path.abspath(args.lib)
    lib = _lib.load()
    tot_f = tot_b = 0.0
    byt_f = byt_b = 0
    for si, (name, B, H, W, C, nh, win, sh, nblk) in enumerate(STAGES_B384 if args.b384 else STAGES):
        if args.stage is not None and si != args.stage:
            continue
        T = B * H * W
        qkv = torch.randn(T, 3 * C, device="cuda").bfloat16()
        out = torch.empty(T, C, device="cuda", dtype=torch.bfloat16)
        dout = torch.randn(T, C, device="cuda").bfloat16()
        dqkv = torch.empty_like(qkv)
        tab = 16 * torch.sigmoid(torch.randn(nh, (2 * win - 1) ** 2, device="cuda"))
        scale = torch.full((nh,), 10.0, device="cuda")
        dtab = torch.empty_like(tab)
        dsc = torch.empty_like(scale)
        dqb = torch.empty(C, device="cuda")
        wsb = lib.hvk_wmsa_bwd_workspace_bytes(nh, win)
        ws = torch.zeros(wsb // 4, device="cuda")  # left zero by every call
        P = _lib.ptr
        st = _lib.stream

        keep = win > 8 and not args.recompute  # as ops.WindowAttentionCore
        lse = torch.empty(T, nh, device="cuda") if keep else None
        normed = args.normed and win <= 8
        rn = torch.empty(T, 2 * nh, device="cuda")
        if normed:
            _lib.call("hvk_qk_normalize", P(qkv), P(rn), P(scale), T, C, st())

        def fwd():
            if normed:
                _lib.call("hvk_wmsa_fwd_normed", P(qkv), P(out), P(tab), P(scale), B, H, W, C, nh, win, sh, st())
            else:
                _lib.call("hvk_wmsa_fwd", P(qkv), P(out), P(lse), P(tab), P(scale), B, H, W, C, nh, win, sh, st())

        fwd()  # out / lse for the backward

        def bwd():
            if normed:
                _lib.call("hvk_wmsa_bwd_normed", P(qkv), P(rn), P(dout), P(dqkv), P(dqb), P(tab), P(scale), P(dtab),
                          P(dsc), P(ws), wsb, B, H, W, C, nh, win, sh, st())
            else:
                _lib.call("hvk_wmsa_bwd", P(qkv), P(dout), P(out) if keep else None, P(lse), P(dqkv), P(dqb),
                          P(tab), P(scale), P(dtab), P(dsc), P(ws), wsb, B, H, W, C, nh, win, sh, st())

        tf = timeit(fwd, args.iters, 0) if args.only != "bwd" else float("nan")
        tb = timeit(bwd, args.iters, 1) if args.only != "fwd" else float("nan")
        bf, bb = 8 * T * C, 16 * T * C
        tot_f += tf * nblk
        tot_b += tb * nblk
        byt_f += bf * nblk
        byt_b += bb * nblk
        print(f"{name:10s} fwd {tf * 1e3:8.1f} us {bf / tf / 1e6:7.0f} GB/s | "
              f"bwd {tb * 1e3:8.1f} us {bb / tb / 1e6:7.0f} GB/s", flush=True)
        del qkv, out, dout, dqkv
    print(f"per step: fwd {tot_f:.3f} ms ({byt_f / tot_f / 1e6:.0f} GB/s)  "
          f"bwd {tot_b:.3f} ms ({byt_b / tot_b / 1e6:.0f} GB/s)")


if __name__ == "__main__":
    main()
