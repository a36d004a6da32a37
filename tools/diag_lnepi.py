"""Where the fused LayerNorm epilogue (hvk_linear_ln_fwd / hvk_mlp_ln_fwd) differs from the
two-launch path: per output, the count of differing elements, the rows / columns they sit in and
the largest difference in ulps.  Diagnostic for tests/test_gpu_linear_ln.py."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_linear_ln as T  # noqa: E402


def report(tag, ref, out):
    for name, r, o in zip(("x", "xb", "mean", "rstd"), ref, out):
        iv = torch.int16 if r.dtype == torch.bfloat16 else torch.int32
        ri, oi = r.view(iv).long(), o.view(iv).long()
        bad = ri != oi
        n = int(bad.sum())
        msg = f"{tag} {name}: {n} differ"
        if n:
            idx = bad.nonzero()
            rows = idx[:, 0].unique()
            msg += f" rows[{rows.numel()}] {rows[:12].tolist()}"
            if idx.shape[1] > 1:
                msg += f" cols {idx[:, 1].unique()[:24].tolist()}"
            msg += f" max ulp {int((ri - oi).abs().max())} nan {int(torch.isnan(o.float()).sum())}"
        print(msg, flush=True)


def linear_case(M, K, with_x0, with_dp):
    lib = T._lib()
    C, rps = 96, 49 if M % 49 == 0 else 1
    g = torch.Generator(device="cuda").manual_seed(M + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(C, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    gamma, beta, abias, x0, ss = T._params(M, C, M + 7, with_x0, with_dp, rps)
    a0 = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    lib.call("hvk_linear_fwd", lib.ptr(x), lib.ptr(w), None, lib.ptr(a0), M, K, C, lib.stream())
    ref = T._ln_ref(a0, abias, x0, gamma, beta, ss, rps, 1e-5)
    a1 = torch.full_like(a0, float("nan"))
    out = [torch.full_like(r, float("nan")) for r in ref]
    lib.call("hvk_linear_ln_fwd", lib.ptr(x), lib.ptr(w), M, K, C, lib.ptr(abias), lib.ptr(x0), lib.ptr(gamma),
             lib.ptr(beta), lib.ptr(ss), rps, 1e-5, lib.ptr(a1), lib.ptr(out[0]), lib.ptr(out[1]), lib.ptr(out[2]),
             lib.ptr(out[3]), lib.stream())
    torch.cuda.synchronize()
    print(f"linear M={M} K={K} x0={with_x0} dp={with_dp} a equal {torch.equal(a0.view(torch.int16), a1.view(torch.int16))}")
    report("  ", ref, out)


def main():
    for M, K in ((4099, 96), (50176, 96), (25088, 48), (1000, 48)):
        for x0, dp in ((True, True), (True, False), (False, False)):
            linear_case(M, K, x0, dp)


if __name__ == "__main__":
    main()
