"""Per-phase shader-clock split of the w7 W-MSA backward (pair kernel) from a -DHVK_STAMPS build:
    EXTRA=-DHVK_STAMPS tools/build_variant.sh WT stamps
    HVK_LIB_PATH=abl/stamps.so python tools/bwd_stamps.py [--stage 0]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_wmsa import STAGES  # noqa: E402

PHASES = ["top: loads + normalise + image writes", "barrier 1", "K^ reads + phase A",
          "next-window load issue", "barrier 2", "phase B", "barrier 3"]



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", type=int, default=0)
    a = ap.parse_args()
    from hvamd import _lib, ops
    name, B, H, W, C, nh, win, shift, _ = STAGES[a.stage]
    qkv = torch.randn(B, H * W, 3 * C, device="cuda").bfloat16().requires_grad_(True)
    tab = (16 * torch.sigmoid(torch.randn(nh, (2 * win - 1) ** 2, device="cuda"))).requires_grad_(True)
    scale = torch.full((nh,), 10.0, device="cuda", requires_grad=True)
    g = torch.randn(B, H * W, C, device="cuda").bfloat16()
    lib = ctypes.CDLL(os.environ["HVK_LIB_PATH"])
    buf = (ctypes.c_ulonglong * 12)()
    for it in range(3):
        out = ops.window_attention_core(qkv, tab, scale, H, W, nh, win, shift)
        torch.cuda.synchronize()
        lib.hvk_debug_bwd_stamps(buf)  # clear
        out.backward(g)
        torch.cuda.synchronize()
        lib.hvk_debug_bwd_stamps(buf)
    tot = sum(buf[:7])
    waves = buf[7]
    print(f"{name}: {waves} waves, {tot / waves:.0f} cycles per wave in the window loop")
    for k, p in enumerate(PHASES):
        print(f"  {p:40s} {buf[k] / waves:10.0f} cyc/wave  {100 * buf[k] / tot:5.1f} %")
    print(f"  setup (entry -> loop)                    {buf[8] / waves:10.0f} cyc/wave")
    print(f"  teardown (loop -> exit)                  {buf[9] / waves:10.0f} cyc/wave")


if __name__ == "__main__":
    main()
