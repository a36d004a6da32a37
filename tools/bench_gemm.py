"""Per-shape timing of the SwinV2-T bs256 training-step GEMMs (forward, input grad, weight
grad as hvamd.ops runs them) against their HBM and MFMA floors.

    python tools/bench_gemm.py [--iters 10]

Floors: bytes / 5.5 TB/s (measured streaming rate of this box class, tools/probe/stream.hip)
and flops / 2.5 PFLOP/s (dense bf16 MFMA)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM = 5.5e12
MFMA = 2.5e15
B = 256
STAGES = [(802816, 96, 2), (200704, 192, 2), (50176, 384, 6), (12544, 768, 2)]  # T, C, blocks
MODELS = {
    "t": STAGES,  # SwinV2-T 224 (config 3)
    "b224": [(802816, 128, 2), (200704, 256, 2), (50176, 512, 18), (12544, 1024, 2)],  # config 4
    "b384": [(2359296, 128, 2), (589824, 256, 2), (147456, 512, 18), (36864, 1024, 2)],  # config 5
}


def shapes(model="t"):
    out = []  # (name, M, K, N, count per step)
    for s, (T, C, nb) in enumerate(MODELS[model]):
        out += [(f"s{s}.qkv", T, C, 3 * C, nb), (f"s{s}.proj", T, C, C, nb),
                (f"s{s}.fc1", T, C, 4 * C, nb), (f"s{s}.fc2", T, 4 * C, C, nb)]
        if s < 3:
            out.append((f"s{s}.merge", T // 4, 4 * C, 2 * C, 1))
    out.append(("embed", MODELS[model][0][0], 48, MODELS[model][0][1], 1))
    out.append(("head", B, 768, 10000, 1))
    return out


def timeit(fn, iters):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tunable", default=None, help="enable PyTorch TunableOp, results file path")
    ap.add_argument("--only", default=None, help="regex of gemm names to run")
    ap.add_argument("--lib", default=None, help="load this libhvk build instead (tools/probe)")
    ap.add_argument("--model", default="t", choices=sorted(MODELS), help="stage shapes: t, b224, b384")
    ap.add_argument("--option", action="append", default=[], help="libhvk option NAME=VALUE (hvk_set_option)")
    a = ap.parse_args()
    if a.lib:
        from hvamd import _lib as L
        L.LIB_PATH = os.path.abspath(a.lib)
    if a.tunable:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(a.tunable)
        torch.cuda.tunable.set_max_tuning_duration(30)
    from hvamd import ops
    tot = {"fwd": 0.0, "dx": 0.0, "dw": 0.0}
    floor = {"fwd": 0.0, "dx": 0.0, "dw": 0.0}
    from hvamd import _lib
    lib = _lib.load()
    import ctypes
    for o in a.option:
        k, v = o.split("=")
        assert lib.hvk_set_option(k.encode(), int(v), ctypes.byref(ctypes.c_longlong())) == 0, o
    tot_h = 0.0
    print(f"{'gemm':10s} {'M':>7s} {'K':>5s} {'N':>6s} {'n':>2s} | {'fwd us':>8s} {'dx us':>8s} {'dw us':>8s} | floor(us) fwd/dx/dw | hvk fwd/dx us | tile fwd/dx us")
    import re
    for name, M, K, N, cnt in shapes(a.model):
        if a.only and not re.search(a.only, name):
            continue
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        tf = timeit(lambda: torch.mm(x, w.t()), a.iters)
        tx = timeit(lambda: torch.mm(dy, w), a.iters)
        tw = timeit(lambda: ops.weight_grad(dy, x), a.iters)
        wt = w.t().contiguous()
        hf = timeit(lambda: ops.mm_nt(x, w), a.iters) if ops._native_nt(M, K, N) else tf
        hx = timeit(lambda: ops.mm_nt(dy, wt), a.iters) if ops._native_nt(M, N, K) else tx
        def tile(a2, b2):  # hvk_gemm_fwd forced, wherever its tiling divides the shape
            m, k = a2.shape
            n = b2.shape[0]
            if k % 64 or (n % 128 and n % 192):
                return float("nan")
            y = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
            return timeit(lambda: _lib.call("hvk_gemm_fwd", _lib.ptr(a2), _lib.ptr(b2), None, _lib.ptr(y),
                                            m, k, n, _lib.stream()), a.iters)
        tf_t, tx_t = tile(x, w), tile(dy, wt)
        tot_h += (hf + hx + tw) * cnt
        byt = 2 * (M * K + M * N + N * K)
        fl = 2 * M * N * K
        fl_us = max(byt / HBM, fl / MFMA) * 1e6
        fw_us = max((2 * (M * K + M * N) + 4 * N * K) / HBM, fl / MFMA) * 1e6
        for k, t, f in (("fwd", tf, fl_us), ("dx", tx, fl_us), ("dw", tw, fw_us)):
            tot[k] += t * cnt
            floor[k] += f * cnt / 1e3
        print(f"{name:10s} {M:7d} {K:5d} {N:6d} {cnt:2d} | {tf * 1e3:8.1f} {tx * 1e3:8.1f} {tw * 1e3:8.1f} | "
              f"{fl_us:6.1f} {fl_us:6.1f} {fw_us:6.1f} | {hf * 1e3:7.1f} {hx * 1e3:7.1f} | {tf_t * 1e3:7.1f} {tx_t * 1e3:7.1f}",
              flush=True)
        del x, w, dy
    for k in tot:
        print(f"total {k}: {tot[k]:.3f} ms/step (floor {floor[k]:.3f})")
    print(f"all GEMMs: {sum(tot.values()):.3f} ms/step (floor {sum(floor.values()):.3f}); "
          f"with hvk fwd/dx where built: {tot_h:.3f} ms/step")


if __name__ == "__main__":
    main()
