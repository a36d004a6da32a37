"""Per-stage W-MSA kernel times of a rocprofv3 kernel trace of bench.py (SwinV2-T bs256):
    python tools/wmsa_stage_times.py kernel_trace.csv
A step launches 12 W-MSA forwards (stages 0, 0, 1, 1, 2 x 6, 3, 3) and 12 backwards (the reverse
order); the dispatches are taken in timestamp order, cut into runs of 12, and each launch gets its
stage from its position.  Prints the mean duration per stage and kernel and the algorithmic HBM
rate (8 T C bytes forward, 16 T C backward)."""
import collections
import csv
import re
import sys

STAGES = [(256 * 56 * 56, 96), (256 * 28 * 28, 192), (256 * 14 * 14, 384), (256 * 7 * 7, 768)]  # T, C
FWD_ORDER = [0, 0, 1, 1, 2, 2, 2, 2, 2, 2, 3, 3]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    for kind, per, order in (("fwd", 8, FWD_ORDER), ("bwd", 16, FWD_ORDER[::-1])):
        disp = [r for r in rows if re.search(rf"wmsa_{kind}_\w*kernel<", r["Kernel_Name"])]
        disp = disp[: len(disp) // 12 * 12]
        acc = collections.OrderedDict()
        for i, r in enumerate(disp):
            s = order[i % 12]
            name = re.search(rf"(wmsa_{kind}_\w*kernel<[^>]*>)", r["Kernel_Name"]).group(1)
            acc.setdefault((s, name), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        tot_ms = tot_b = 0.0
        for (s, name), d in sorted(acc.items()):
            us = sum(d) / len(d) / 1e3
            T, C = STAGES[s]
            b = per * T * C
            n_step = order.count(s)
            tot_ms += us * n_step / 1e3 * len(d) / (len(disp) // 12 * n_step)
            tot_b += b * len(d) / (len(disp) // 12)
            gbs = b / us / 1e3
            print(f"{kind} stage {s}  {name:32s} n={len(d):4d}  {us:8.1f} us  {gbs:6.0f} GB/s  {gbs / 8000:.3f} of 8 TB/s")
        if tot_ms:
            gbs = tot_b / tot_ms / 1e6
            print(f"{kind} per step {tot_ms:.3f} ms  {gbs:.0f} GB/s  {gbs / 8000:.3f} of 8 TB/s")


if __name__ == "__main__":
    main()
