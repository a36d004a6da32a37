"""Per-workgroup phase timeline of the tiled GEMM from the HVK_GEMM_PROBE=4 build
(tools/probe/libhvk_gemm4.so): prologue (first tile landed), k-loop, epilogue (stores drained).
    python tools/gemm_timeline.py M K N [gelu|gelu_bwd]   (make -C tools/probe libhvk_gemm4.so first)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    M, K, N = (int(a) for a in sys.argv[1:4])
    epi = sys.argv[4] if len(sys.argv) > 4 else "plain"
    from hvamd import _lib
    _lib.LIB_PATH = os.path.abspath(os.environ.get("HVK_TL_LIB", "tools/probe/libhvk_gemm4.so"))
    lib = _lib.load()
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y2 = torch.randn(M, N, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda")
    for _ in range(5):
        if epi == "gelu":
            _lib.call("hvk_gemm_gelu_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(y), _lib.ptr(y2), M, K,
                      N, _lib.stream())
        elif epi == "gelu_bwd":
            _lib.call("hvk_gemm_gelu_bwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(y2), _lib.ptr(y), M, K, N,
                      _lib.stream())
        else:
            _lib.call("hvk_gemm_fwd", _lib.ptr(x), _lib.ptr(w), None, _lib.ptr(y), M, K, N, _lib.stream())
    torch.cuda.synchronize()
    # tile width as launch_tile picks it (HVK_TILE_WIDE unset)
    BM, BN = 128, (192 if N % 192 == 0 and (N > 384 or K >= 1536) else 128)
    mt = (M + BM - 1) // BM
    nb = (mt + 7) // 8 * 8 * (N // BN)
    buf = np.zeros(nb * 6, dtype=np.uint64)
    lib.hvk_gemm_probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert lib.hvk_gemm_probe_read(buf.ctypes.data, nb) == 0
    t = buf.reshape(nb, 6).astype(np.int64)
    ok = t[:, 0] > 0
    t = t[ok]
    us = 0.01  # 100 MHz steady counter
    t0 = t[:, 0].min()
    pro, loop, epi = (t[:, 1] - t[:, 0]) * us, (t[:, 2] - t[:, 1]) * us, (t[:, 3] - t[:, 2]) * us
    span = (t[:, 3].max() - t0) * us
    print(f"M={M} K={K} N={N}: {len(t)} workgroups, span {span:.1f} us")
    for name, v in (("prologue", pro), ("k-loop", loop), ("epilogue", epi)):
        print(f"  {name:9s} mean {v.mean():6.2f} us  p10 {np.percentile(v, 10):6.2f}  p90 {np.percentile(v, 90):6.2f}")
    life = (t[:, 3] - t[:, 0]) * us
    print(f"  lifetime  mean {life.mean():6.2f} us; sum of lifetimes / (span * slots) = "
          f"{life.sum() / (span * 512):.2f}")
    # concurrency: workgroups alive / in loop over time (1 us bins)
    bins = np.arange(0, span + 1, 1.0)
    rel0, rel1, rel2, rel3 = ((t[:, i] - t0) * us for i in range(4))
    alive = [(np.sum((rel0 <= b) & (rel3 > b))) for b in bins]
    inloop = [(np.sum((rel1 <= b) & (rel2 > b))) for b in bins]
    inepi = [(np.sum((rel2 <= b) & (rel3 > b))) for b in bins]
    inpro = [(np.sum((rel0 <= b) & (rel1 > b))) for b in bins]
    print("  t(us)  alive  prologue  loop  epilogue")
    for b, a, p, l, e in zip(bins, alive, inpro, inloop, inepi):
        print(f"  {b:5.0f}  {a:5d}  {p:8d}  {l:4d}  {e:8d}")
    # gap between a slot's consecutive workgroups: per (xcc, hw_id) sorted by start
    key = t[:, 5] * 65536 + (t[:, 4] & 0xFFFF)
    gaps = []
    for k in np.unique(key):
        r = t[key == k]
        r = r[np.argsort(r[:, 0])]
        if len(r) > 1:
            gaps += list((r[1:, 0] - r[:-1, 3]) * us)
    if gaps:
        g = np.array(gaps)
        print(f"  same-slot restart gap: mean {g.mean():.2f} us, p50 {np.median(g):.2f} (n={len(g)}; "
              "negative = overlapping workgroups on one CU/SIMD id)")


if __name__ == "__main__":
    main()
