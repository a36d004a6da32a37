"""Group a `rocprofv3 --kernel-trace` trace into per-step categories.

    python tools/kernel_summary.py gpurun_out/prof/run_results.db --anchor hxe_fwd --skip 3
    python tools/kernel_summary.py gpurun_out/prof/run_kernel_trace.csv --anchor hxe_fwd --skip 3
    python tools/kernel_summary.py gpurun_out/prof/.../kernel_stats.csv --steps 15

With a rocpd .db, --anchor/--skip keep only the dispatches from the (skip+1)-th launch of
the anchor kernel (one per step) onwards, i.e. the timed steps, and the step count is the
number of anchor launches kept.
"""
import argparse
import csv
import re
import sqlite3

CATS = [  # (category, regex on the kernel name), first match wins
    ("wmsa_fwd", r"wmsa_fwd"),
    ("wmsa_bwd", r"wmsa_bwd|wmsa_dbias"),
    ("layernorm", r"ln_fwd|ln_bwd|colsum_kernel"),
    ("bias_gelu", r"bias_gelu|colsum_rows"),
    ("patch_merge", r"merge_kernel"),
    ("losses", r"multitask|hxe"),
    ("head", r"head_kernel|head_sum"),
    ("gemm(dW)", r"dw_kernel|dw_reduce"),
    ("gemm(hvk)", r"linear_kernel|gemm_nt_kernel|gemm_pp_kernel|mlp_fwd_kernel|mlp_bwd_kernel"),
    ("gemm", r"Cijk|gemm|Gemm|GEMM|mfma|MT\d+x\d+"),
    ("memset", r"[Mm]emset|fill"),
    ("reduce", r"reduce|Reduce"),
    ("optimizer", r"foreach|multi_tensor|Adam|sgd"),
    ("copy/cast", r"copy|Copy|cast|elementwise|vectorized"),
]


def category(name):
    """The CATS category of a kernel name (first match), else "other"."""
    for c, rx in CATS:
        if re.search(rx, name):
            return c
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--anchor", default=None, help="regex of a once-per-step kernel (.db only)")
    ap.add_argument("--skip", type=int, default=0, help="anchor launches to drop (warmup)")
    a = ap.parse_args()
    if a.csv.endswith(".db") or a.csv.endswith("kernel_trace.csv"):
        if a.csv.endswith(".db"):
            db = sqlite3.connect(a.csv)
            disp = db.execute("select name, start, end from kernels order by start").fetchall()
        else:
            disp = sorted((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                          for r in csv.DictReader(open(a.csv)))
            disp.sort(key=lambda d: d[1])
        if a.anchor:
            starts = [st for n, st, _ in disp if re.search(a.anchor, n)]
            t0 = starts[a.skip]
            disp = [d for d in disp if d[1] >= t0]
            a.steps = len(starts) - a.skip
            span = (disp[-1][2] - t0) / 1e6
            print(f"{a.steps} steps, {span / a.steps:.3f} ms/step wall (first kept dispatch to last end)")
        agg = {}
        for n, st, en in disp:
            t = agg.setdefault(n, [0.0, 0])
            t[0] += (en - st) / 1e6
            t[1] += 1
        rows = [{"Name": n, "ms": v[0], "Calls": v[1]} for n, v in agg.items()]
    else:
        rows = [{"Name": r["Name"], "ms": float(r["TotalDurationNs"]) / 1e6, "Calls": int(r["Calls"])}
                for r in csv.DictReader(open(a.csv))]
    cat_ms, cat_n, kern = {}, {}, []
    for r in rows:
        name = r["Name"]
        tot = r["ms"]
        n = int(r["Calls"])
        c = next((c for c, rx in CATS if re.search(rx, name)), "other")
        cat_ms[c] = cat_ms.get(c, 0) + tot
        cat_n[c] = cat_n.get(c, 0) + n
        kern.append((tot, n, c, name))
    total = sum(cat_ms.values())
    print(f"total kernel time {total / a.steps:.3f} ms/step")
    for c in sorted(cat_ms, key=cat_ms.get, reverse=True):
        print(f"  {c:12s} {cat_ms[c] / a.steps:8.3f} ms/step  {cat_n[c] / a.steps:7.1f} launches/step")
    print("top kernels:")
    for tot, n, c, name in sorted(kern, reverse=True)[: a.top]:
        print(f"  {tot / a.steps:7.3f} ms  {n / a.steps:6.1f}x  avg {tot / n * 1e3:8.1f} us  [{c}] {name[:110]}")


if __name__ == "__main__":
    main()
