"""Patch-embedding weight gradient (N = 128, K = 48, SwinV2-B) on libhvk's dW kernel against the
library path it replaced (ops.weight_grad's chunked bmm + sum), at the config-4 / config-5 token
counts.  python tools/dw_pe_ab.py"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hvamd import _lib, ops


def timed(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


lib = _lib.load()
for img in (56, 96):
    M, N, K = 256 * img * img, 128, 48
    g = torch.randn(M, N, device="cuda").bfloat16()
    x = torch.randn(M, K, device="cuda").bfloat16()
    dw = torch.empty(N, K, device="cuda")
    db = torch.empty(N, device="cuda")
    ws = torch.empty(lib.hvk_weight_grad_workspace(M, N, K), device="cuda", dtype=torch.uint8)

    def native():
        _lib.call("hvk_weight_grad", _lib.ptr(g), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db), M, N, K,
                  _lib.ptr(ws), ws.numel(), _lib.stream())

    def library():
        nc = ops._split_k_chunks(M)
        kc = M // nc
        g.sum(dim=0, dtype=torch.float32)
        torch.bmm(g.view(nc, kc, -1).transpose(1, 2), x.view(nc, kc, -1), out_dtype=torch.float32).sum(0)

    tn, tl = timed(native), timed(library)
    ref = g.float().t() @ x.float()
    native()
    torch.cuda.synchronize()
    err = ((dw - ref).abs().max() / ref.abs().max()).item()
    gb = (2.0 * M * (N + K)) / 1e9
    print(f"M={M} N={N} K={K}: libhvk {tn:.1f} us ({gb / tn * 1e6 / 1e3:.2f} TB/s), "
          f"library {tl:.1f} us, rel err {err:.2e}", flush=True)
