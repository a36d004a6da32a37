"""Per-phase shader-clock split of the w7 W-MSA backward (pair kernel) from a -DHVK_STAMPS build,
on the model's path (q / k normalised upstream: hvk_wmsa_bwd_normed; --raw for hvk_wmsa_bwd):
    EXTRA=-DHVK_STAMPS tools/build_variant.sh WT stamps
    HVK_LIB_PATH=abl/stamps.so python tools/bwd_stamps.py [--stage 0] [--raw]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_wmsa import STAGES  # noqa: E402

PHASES = ["top: loads landed + image writes", "barrier 1", "K^ reads + phase A",
          "next-window V load issue", "barrier 2", "phase B", "barrier 3"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", type=int, default=0)
    ap.add_argument("--raw", action="store_true")
    a = ap.parse_args()
    from hvamd import _lib
    lib = _lib.load()
    P, st = _lib.ptr, _lib.stream
    name, B, H, W, C, nh, win, shift, _ = STAGES[a.stage]
    T = B * H * W
    qkv = torch.randn(T, 3 * C, device="cuda").bfloat16()
    dout = torch.randn(T, C, device="cuda").bfloat16()
    dqkv = torch.empty_like(qkv)
    tab = 16 * torch.sigmoid(torch.randn(nh, (2 * win - 1) ** 2, device="cuda"))
    scale = torch.full((nh,), 10.0, device="cuda")
    dtab, dsc = torch.empty_like(tab), torch.empty_like(scale)
    dqb = torch.empty(C, device="cuda")
    wsb = lib.hvk_wmsa_bwd_workspace_bytes(nh, win)
    ws = torch.zeros(wsb // 4, device="cuda")
    rn = torch.empty(T, 2 * nh, device="cuda")
    if not a.raw:
        _lib.call("hvk_qk_normalize", P(qkv), P(rn), P(scale), T, C, st())
    sl = ctypes.CDLL(os.environ["HVK_LIB_PATH"])
    buf = (ctypes.c_ulonglong * 12)()
    for it in range(3):
        torch.cuda.synchronize()
        sl.hvk_debug_bwd_stamps(buf)  # clear
        if a.raw:
            _lib.call("hvk_wmsa_bwd", P(qkv), P(dout), None, None, P(dqkv), P(dqb), P(tab), P(scale), P(dtab),
                      P(dsc), P(ws), wsb, B, H, W, C, nh, win, shift, st())
        else:
            _lib.call("hvk_wmsa_bwd_normed", P(qkv), P(rn), P(dout), P(dqkv), P(dqb), P(tab), P(scale), P(dtab),
                      P(dsc), P(ws), wsb, B, H, W, C, nh, win, shift, st())
        torch.cuda.synchronize()
        sl.hvk_debug_bwd_stamps(buf)
    tot = sum(buf[:7])
    waves = buf[7]
    print(f"{name} ({'raw' if a.raw else 'normed'}): {waves} waves, {tot / waves:.0f} cycles per wave in the window loop")
    for k, p in enumerate(PHASES):
        print(f"  {p:40s} {buf[k] / waves:10.0f} cyc/wave  {100 * buf[k] / tot:5.1f} %")
    print(f"  setup (entry -> loop)                    {buf[8] / waves:10.0f} cyc/wave")
    print(f"  teardown (loop -> exit)                  {buf[9] / waves:10.0f} cyc/wave")
    print(f"    partials staged in LDS                 {buf[10] / waves:10.0f} cyc/wave")
    print(f"    bins fold                              {buf[11] / waves:10.0f} cyc/wave")
    print(f"    wave sums, slot add, stores drained    {(buf[9] - buf[10] - buf[11]) / waves:10.0f} cyc/wave")


if __name__ == "__main__":
    main()
