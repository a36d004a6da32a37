"""Does the bucketed gradient all-reduce overlap the backward?  Reads the rocprofv3 kernel trace
of tools/ddp_trace.py and reports, per training step (anchored on the HXE forward kernel, one per
step), every RCCL kernel (name matches nccl / rccl) with its start and end relative to the end of
the step's last backward kernel (the last non-RCCL kernel before the optimizer's first sumsq /
sgdw launch), its queue and the queue of the backward's kernels.

    python tools/ddp_overlap.py TRACE_DIR_OR_CSV [--skip 1]
"""
import argparse
import csv
import glob
import os
import re


def load(path):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not cands:
            raise SystemExit(f"no *kernel_trace.csv under {path}")
        path = cands[0]
    rows = list(csv.DictReader(open(path)))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else None
    skey = "Stream_Id" if "Stream_Id" in rows[0] else None
    out = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
            r.get(qkey, "?") if qkey else "?", r.get(skey, "?") if skey else "?") for r in rows]
    out.sort(key=lambda d: d[1])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=1, help="steps to drop (warm-up)")
    a = ap.parse_args()
    disp = load(a.trace)
    rccl = re.compile(r"nccl|rccl|Nccl|Rccl", re.I)
    starts = [d[1] for d in disp if re.search(r"hxe_fwd", d[0])]
    starts.append(float("inf"))
    print(f"{len(disp)} kernels, {len(starts) - 1} steps; RCCL kernels: "
          f"{sum(1 for d in disp if rccl.search(d[0]))}")
    for si in range(a.skip, len(starts) - 1):
        step = [d for d in disp if starts[si] <= d[1] < starts[si + 1]]
        opt = [d for d in step if re.search(r"sumsq_kernel|sgdw_kernel", d[0])]
        t_opt = opt[0][1] if opt else float("inf")
        bwd = [d for d in step if not rccl.search(d[0]) and d[1] < t_opt]
        if not bwd:
            continue
        last = max(bwd, key=lambda d: d[2])
        comm = [d for d in disp if rccl.search(d[0]) and starts[si] <= d[1] < starts[si + 1]]
        qs = sorted({d[3] for d in bwd})
        print(f"step {si}: backward ends at +{(last[2] - starts[si]) / 1e3:.1f} us ({last[0][:60]}), "
              f"compute queue(s) {qs}; {len(comm)} RCCL kernels")
        for d in comm:
            rel0, rel1 = (d[1] - last[2]) / 1e3, (d[2] - last[2]) / 1e3
            tag = "OVERLAPS the backward" if rel0 < 0 else "after the backward"
            print(f"   {d[0][:70]:70s} queue {d[3]} stream {d[4]}  start {rel0:+9.1f} us  end {rel1:+9.1f} us  {tag}")


if __name__ == "__main__":
    main()
